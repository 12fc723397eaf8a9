// Standalone timing harness for compile-time variants of native/ops/flash_attn.hip
// (no Python on the timed path).  Build one binary per variant with -D flags,
// and run them with `tools/gpu.sh fa-variants`; each run times fwd and fwd+bwd at the
// Llama-3-8B attention shape (B=2, S=4096, 32 q / 8 kv heads, d=128, causal)
// and dumps O / dQ / dK / dV checksums plus raw outputs so a variant can be
// compared bit-for-bit (or to bf16 rounding) against the baseline binary.
#include "../native/ops/flash_attn.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

static unsigned short f2b(float f) {
  unsigned int u;
  std::memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return static_cast<unsigned short>(u >> 16);
}
static float b2f(unsigned short b) {
  unsigned int u = static_cast<unsigned int>(b) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

int main(int argc, char** argv) {
  const char* tag = argc > 1 ? argv[1] : "base";
  const char* ref = argc > 2 ? argv[2] : nullptr;  // baseline dump to compare against
  // FA_B in the environment sets the batch (the training step runs B=4)
  const int B = std::getenv("FA_B") ? std::atoi(std::getenv("FA_B")) : 2, S = 4096, H = 32, HKV = 8, D = 128;
  const size_t nq = size_t(B) * S * H * D, nkv = size_t(B) * S * HKV * D;
  std::vector<unsigned short> hq(nq), hk(nkv), hv(nkv), hdo(nq);
  unsigned long long st = 12345;
  auto rnd = [&]() {
    st = st * 6364136223846793005ULL + 1442695040888963407ULL;
    return (static_cast<int>((st >> 33) & 0xffff) - 32768) / 16384.0f;
  };
  for (auto& x : hq) x = f2b(rnd());
  for (auto& x : hk) x = f2b(rnd());
  for (auto& x : hv) x = f2b(rnd());
  for (auto& x : hdo) x = f2b(rnd() * 0.1f);
  void *q, *k, *v, *o, *dout, *dq, *dk, *dv;
  float *lse, *work;
  CK(hipMalloc(&q, nq * 2)); CK(hipMalloc(&k, nkv * 2)); CK(hipMalloc(&v, nkv * 2));
  CK(hipMalloc(&o, nq * 2)); CK(hipMalloc(&dout, nq * 2)); CK(hipMalloc(&dq, nq * 2));
  CK(hipMalloc(&dk, nkv * 2)); CK(hipMalloc(&dv, nkv * 2));
  CK(hipMalloc(&lse, size_t(B) * H * S * 4));
  CK(hipMalloc(&work, kgwe_flash_attn_bwd_workspace(B, S, H, HKV, D)));
  CK(hipMemcpy(q, hq.data(), nq * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(k, hk.data(), nkv * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, hv.data(), nkv * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, hdo.data(), nq * 2, hipMemcpyHostToDevice));
  const float scale = 1.0f / std::sqrt(float(D));
  // FA_CAUSAL=0 in the environment times the full (non-causal) problem
  const int causal = std::getenv("FA_CAUSAL") ? std::atoi(std::getenv("FA_CAUSAL")) : 1;
  auto fwd = [&]() {
    if (kgwe_flash_attn_fwd(q, k, v, o, lse, B, S, H, HKV, D, scale, causal, 0)) std::exit(2);
  };
  auto bwd = [&]() {
    if (kgwe_flash_attn_bwd(q, k, v, o, lse, dout, dq, dk, dv, work, nullptr, B, S, H, HKV, D, scale, causal, 0))
      std::exit(3);
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](auto fn, int n) {
    for (int i = 0; i < 3; ++i) fn();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < n; ++i) fn();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / n;
  };
  const double fl = 4.0 * B * H * double(S) * S * D / (causal ? 2 : 1);
  const float tf = timeit(fwd, 30);
  const float tb = timeit(bwd, 20);
  fwd(); bwd();
  CK(hipDeviceSynchronize());
  std::vector<unsigned short> out(2 * nq + 2 * nkv);
  CK(hipMemcpy(out.data(), o, nq * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(out.data() + nq, dq, nq * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(out.data() + 2 * nq, dk, nkv * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(out.data() + 2 * nq + nkv, dv, nkv * 2, hipMemcpyDeviceToHost));
  double maxdiff[4] = {0, 0, 0, 0};
  bool finite = true;
  for (auto x : out) finite &= std::isfinite(b2f(x));
  if (ref) {
    std::vector<unsigned short> r(out.size());
    FILE* f = std::fopen(ref, "rb");
    if (f && std::fread(r.data(), 2, r.size(), f) == r.size()) {
      const size_t off[5] = {0, nq, 2 * nq, 2 * nq + nkv, out.size()};
      for (int t = 0; t < 4; ++t)
        for (size_t i = off[t]; i < off[t + 1]; ++i)
          maxdiff[t] = std::fmax(maxdiff[t], std::fabs(double(b2f(out[i])) - b2f(r[i])));
    }
    if (f) std::fclose(f);
  } else {
    char path[256];
    std::snprintf(path, sizeof path, "/tmp/fa_%s.bin", tag);
    FILE* f = std::fopen(path, "wb");
    if (f) { std::fwrite(out.data(), 2, out.size(), f); std::fclose(f); }
  }
  std::printf("%-10s fwd %.3f ms (%.0f TF/s)  bwd %.3f ms (%.0f TF/s)  finite=%d  maxdiff o/dq/dk/dv %.2e %.2e %.2e %.2e\n",
              tag, tf, fl / tf / 1e9, tb, 2.5 * fl / tb / 1e9, int(finite), maxdiff[0], maxdiff[1],
              maxdiff[2], maxdiff[3]);
  return 0;
}
