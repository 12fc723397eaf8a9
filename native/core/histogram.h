// Lock-free log-linear latency histogram (HDR-style) for the p99 SLO.
//
// The reference reported "P99" as the running MAX of whole-millisecond
// samples (src/scheduler/scheduler.go:805-819).  This histogram records
// microsecond samples into buckets of ~1.5 % relative width from 1 us to
// ~100 s, with atomic counters so concurrent extender threads record without
// a lock, and answers any quantile.  It also renders the Prometheus bucket
// layout the reference's dashboard queries
// (kgwe_scheduling_latency_ms_bucket, le = 10..5000 ms).
#pragma once
#include <array>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <vector>

namespace kgwe {

class LatencyHistogram {
 public:
  static constexpr int kSub = 64;       // linear sub-buckets per power of two
  static constexpr int kOctaves = 28;   // 1 us .. 2^33 us; ~1.6 % bucket width
  static constexpr int kBuckets = kSub * kOctaves;

  LatencyHistogram() { reset(); }

  void reset() {
    for (auto& c : counts_) c.store(0, std::memory_order_relaxed);
    total_.store(0);
    sum_us_.store(0);
    max_us_.store(0);
  }

  void record_us(uint64_t us) {
    counts_[index(us)].fetch_add(1, std::memory_order_relaxed);
    total_.fetch_add(1, std::memory_order_relaxed);
    sum_us_.fetch_add(us, std::memory_order_relaxed);
    uint64_t m = max_us_.load(std::memory_order_relaxed);
    while (us > m && !max_us_.compare_exchange_weak(m, us)) {
    }
  }
  void record_ms(double ms) { record_us(static_cast<uint64_t>(ms < 0 ? 0 : ms * 1000.0 + 0.5)); }

  uint64_t count() const { return total_.load(); }
  double sum_ms() const { return sum_us_.load() / 1000.0; }
  double mean_ms() const {
    uint64_t n = count();
    return n ? sum_ms() / n : 0.0;
  }
  double max_ms() const { return max_us_.load() / 1000.0; }

  // q in [0, 1]; returns the upper edge of the bucket holding the q-quantile
  // (never under-reports), clamped to the observed max.
  double quantile_ms(double q) const {
    uint64_t n = count();
    if (n == 0) return 0.0;
    uint64_t rank = static_cast<uint64_t>(std::ceil(q * static_cast<double>(n)));
    if (rank < 1) rank = 1;
    uint64_t seen = 0;
    for (int i = 0; i < kBuckets; ++i) {
      seen += counts_[i].load(std::memory_order_relaxed);
      if (seen >= rank) {
        double edge = upper_us(i) / 1000.0;
        double mx = max_ms();
        return edge < mx ? edge : mx;
      }
    }
    return max_ms();
  }

  // Cumulative count of samples <= le_ms (Prometheus-style bucket).
  uint64_t cumulative_le_ms(double le_ms) const {
    uint64_t lim = static_cast<uint64_t>(le_ms * 1000.0);
    uint64_t c = 0;
    for (int i = 0; i < kBuckets; ++i) {
      if (upper_us(i) > lim) break;
      c += counts_[i].load(std::memory_order_relaxed);
    }
    return c;
  }

 private:
  static int index(uint64_t us) {
    if (us < kSub) return static_cast<int>(us);
    int msb = 63 - __builtin_clzll(us);          // >= 6
    int octave = msb - 5;                         // 1.. ; octave 0 = [0, 64)
    if (octave >= kOctaves) return kBuckets - 1;
    int sub = static_cast<int>((us >> (msb - 6)) & (kSub - 1));
    return octave * kSub + sub;
  }
  static double upper_us(int i) {
    int octave = i / kSub, sub = i % kSub;
    if (octave == 0) return sub + 1;
    int msb = octave + 5;
    double base = std::ldexp(1.0, msb);
    double width = std::ldexp(1.0, msb - 6);
    return base + (sub + 1) * width;
  }

  std::array<std::atomic<uint64_t>, kBuckets> counts_;
  std::atomic<uint64_t> total_{0};
  std::atomic<uint64_t> sum_us_{0};
  std::atomic<uint64_t> max_us_{0};
};

}  // namespace kgwe
