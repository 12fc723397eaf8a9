// Decode-time projections for a SERVING batch (8 < M <= 32 rows) on gfx950:
// weight-streaming skinny GEMMs on the matrix cores with the decode layer's
// elementwise work fused in — the M <= 8 kernels of gemv.hip, for the batch a
// shared-model server decodes (kgwe.serving: every client's rows in one step).
//
//   y[m, n] = sum_k x[m, k] W[n, k]          W: [N, K] bf16 (nn.Linear layout)
//
// At M = 32 a projection still reads each weight byte once, for 32 FLOP: an
// HBM stream, but past what v_dot2 on the vector ALU sustains, so the dot
// products go to v_mfma_f32_32x32x16_bf16 with W as the A operand (32 weight
// rows on the accumulator rows) and x as the B operand (the batch row on the
// lane).  The library's small-tile GEMMs ran these shapes at 1-2 TB/s and
// needed RMSNorm, SwiGLU and argmax as launches of their own.
//
// One workgroup = 4 waves = one block of 32 weight rows (SWIGLU: 32 gate rows
// and their 32 up rows) x one K slice of <= 2048 columns:
//   * the slice of x (all rows, residual add and RMSNorm gain applied, rows
//     >= M zero) is staged once in LDS with a 16-B row pad, so the B-operand
//     reads (ds_read_b128, batch row on the lane) are conflict-free; a
//     workgroup that loops over several row blocks stages once;
//   * each wave streams a quarter of the slice: every lane loads 16 B of ITS
//     weight row per k-step straight into the A operand (no LDS for W), eight
//     k-steps in flight and the next eight requested before the MFMAs of the
//     current ones;
//   * the four waves' accumulators meet in wave 0 through two LDS hand-offs in
//     a fixed order (deterministic sums);
//   * K split over several workgroups (K > 2048, or too few row blocks to fill
//     the chip): each publishes its fp32 partial tile with write-through
//     stores and takes a ticket; the last arriver of a row block adds the
//     partials in slice order and runs the epilogue (the hand-off of
//     decode.hip: no fence, no spin, no second launch; tickets return to 0).
// RMSNorm is applied as y = rstd[m] * sum_k (h[m, k] g[k]) W[n, k]: the gain
// goes into the staged operand, the row's rstd (sum of squares accumulated
// per slice, carried with the partials) multiplies the fp32 result.
//
// Every kernel here is graph-safe (no host sync, fixed grids, no memset).
#include <algorithm>

#include "common.h"

using namespace kgwe;

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 mfma8;

constexpr int kT = 256;          // threads per workgroup (4 waves)
constexpr int kMB = 32;          // batch rows of the MFMA tile (M is padded to it)
constexpr int kNB = 32;          // weight rows per block
constexpr int kMaxSlice = 2048;  // K columns staged per workgroup
constexpr int kU = 8;            // k-steps (16 columns each) in flight per wave
constexpr int kTile = kNB * kMB;  // fp32 values of one accumulator tile

enum Mode { kPlain = 0, kNorm = 1, kSwiglu = 2, kNormSwiglu = 3, kArgmax = 4, kNormArgmax = 5 };

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(mfma8, a), __builtin_bit_cast(mfma8, b), c,
                                                 0, 0, 0);
}

// Accumulator register r of a 32x32 tile holds row (r & 3) + 8 (r >> 2) + 4 half.
__device__ __forceinline__ int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

__device__ __forceinline__ unsigned long long argmax_key(float v, int n) {
  unsigned u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return (static_cast<unsigned long long>(u) << 32) | static_cast<unsigned>(~n);
}

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Floats of split-K workspace per (row block, slice): the tile(s) + 32 sums of squares.
__host__ __device__ constexpr int part_floats(bool swiglu) { return (swiglu ? 2 : 1) * kTile + kMB; }

template <int MODE>
__global__ __launch_bounds__(kT) void skinny_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, const bf16_t* __restrict__ g,
    bf16_t* __restrict__ h_out, float eps, const bf16_t* __restrict__ W, bf16_t* __restrict__ y,
    unsigned long long* __restrict__ best, float* __restrict__ part, unsigned* __restrict__ tickets, int M,
    int N, int K, int KS, int NB) {
  constexpr bool NORM = (MODE & kNorm) != 0;
  constexpr bool SWIGLU = (MODE & kSwiglu) != 0;
  constexpr bool ARGMAX = (MODE & kArgmax) != 0;
  constexpr int TILES = SWIGLU ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];  // [kMB][Ks + 8]
  // cross-wave hand-off: [0], [1] waves 2, 3 -> 0, 1; [2] wave 1 -> 0 (a buffer of its own: wave 0 may
  // still be reading it when waves 2, 3 write the next block's [0], [1])
  __shared__ float red[3][TILES][kTile];
  __shared__ float ssq[kMB];                                    // this slice's sum of squares per row

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Ks = K / KS, pitch = Ks + 8;
  const int ks = static_cast<int>(blockIdx.x) % KS;
  const int k0 = ks * Ks;
  const int nb0 = static_cast<int>(blockIdx.x) / KS, nb_step = static_cast<int>(gridDim.x) / KS;

  const int lq = lane & 31, hh = lane >> 5;
  const int span = Ks / 4;          // columns of this wave
  const int steps = span / 16;      // k-steps of this wave

  // Weight rows of a block and their loads.  The first two batches of a block
  // are requested before the previous block's hand-off (and, for the first
  // block, before x is staged), so their HBM latency is covered.
  const bf16_t* wg = nullptr;
  const bf16_t* wu = nullptr;
  bf16x8 wv[2][kU], uv[2][SWIGLU ? kU : 1];
  auto set_rows = [&](int nb) {
    const int n = nb * kNB + lq;
    wg = W + static_cast<size_t>(n < N ? n : N - 1) * K + k0 + w * span + 8 * hh;
    if (SWIGLU) wu = wg + static_cast<size_t>(N) * K;
  };
  auto fetch = [&](int buf, int s0) {
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (s0 + u < steps) {  // wave-uniform
        wv[buf][u] = *reinterpret_cast<const bf16x8*>(wg + 16 * (s0 + u));
        if (SWIGLU) uv[buf][u] = *reinterpret_cast<const bf16x8*>(wu + 16 * (s0 + u));
      }
  };
  if (nb0 < NB) {
    set_rows(nb0);
    fetch(0, 0);
    fetch(1, kU);
  }

  // ---- stage this slice of x ----
  // Without the fused norm the slice is a plain copy: LDS-DMA (global_load_lds, 16 B per
  // lane, no VGPR round trip), one wave instruction per KB of a row, every one of them in
  // flight at once.  Rows >= M re-read row 0: a column of the B operand only reaches its
  // own output column, which is never written.
  if (!NORM && Ks % 512 == 0) {
    const int per_row = Ks / 512;  // wave instructions per row
    for (int m = w; m < kMB; m += 4) {
      const bf16_t* xr = x + static_cast<size_t>(m < M ? m : 0) * K + k0 + 8 * lane;
      bf16_t* dst = xs + static_cast<size_t>(m) * pitch;
      for (int j = 0; j < per_row; ++j)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xr + 512 * j),
                                         (__attribute__((address_space(3))) void*)(dst + 512 * j), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    // 8 threads per batch row, 8 x 16 B in flight each
    constexpr int SU = 8;
    const int m = tid >> 3, sub = tid & 7;
    const int chunks = Ks / 8;
    const bool row = m < M;
    const bf16_t* xr = x + static_cast<size_t>(row ? m : 0) * K + k0;
    const bf16_t* rr = res ? res + static_cast<size_t>(row ? m : 0) * K + k0 : nullptr;
    const bool hw = NORM && rr && h_out && nb0 == 0;  // the new residual stream, once per slice
    float ss = 0.f;
    for (int c0 = sub; c0 < chunks; c0 += 8 * SU) {
      bf16x8 xv[SU], rv[NORM ? SU : 1], gv[NORM ? SU : 1];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int c = c0 + 8 * u;
        xv[u] = bf16x8{};
        if (row && c < chunks) {
          xv[u] = *reinterpret_cast<const bf16x8*>(xr + 8 * c);
          if (NORM) {
            rv[NORM ? u : 0] = rr ? *reinterpret_cast<const bf16x8*>(rr + 8 * c) : bf16x8{};
            gv[NORM ? u : 0] = *reinterpret_cast<const bf16x8*>(g + k0 + 8 * c);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int c = c0 + 8 * u;
        if (c >= chunks) break;
        bf16x8 v = xv[u];
        if (NORM && row) {
          if (rr) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) + bf2f(rv[NORM ? u : 0][j]));
            if (hw) *reinterpret_cast<bf16x8*>(h_out + static_cast<size_t>(m) * K + k0 + 8 * c) = v;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float f = bf2f(v[j]);
            ss += f * f;
            v[j] = f2bf(f * bf2f(gv[NORM ? u : 0][j]));
          }
        }
        *reinterpret_cast<bf16x8*>(xs + static_cast<size_t>(m) * pitch + 8 * c) = v;
      }
    }
    if (NORM) {
      ss += __shfl_xor(ss, 1, kWave);
      ss += __shfl_xor(ss, 2, kWave);
      ss += __shfl_xor(ss, 4, kWave);
      if (sub == 0) ssq[m] = ss;
    }
  }
  __syncthreads();

  const bf16_t* xw = xs + static_cast<size_t>(lq) * pitch + w * span + 8 * hh;

  for (int nb = nb0; nb < NB; nb += nb_step) {
    f32x16 acc[TILES];
#pragma unroll
    for (int t = 0; t < TILES; ++t) acc[t] = f32x16{};
    auto consume = [&](int buf, int s0) {
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (s0 + u < steps) {
          const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xw + 16 * (s0 + u));
          acc[0] = mfma(wv[buf][u], xf, acc[0]);
          if (SWIGLU) acc[TILES - 1] = mfma(uv[buf][SWIGLU ? u : 0], xf, acc[TILES - 1]);
        }
    };
    for (int s0 = 0; s0 < steps; s0 += 2 * kU) {  // batches [s0, s0 + kU) and [s0 + kU, s0 + 2 kU) are in flight
      consume(0, s0);
      fetch(0, s0 + 2 * kU);
      consume(1, s0 + kU);
      fetch(1, s0 + 3 * kU);
    }
    if (nb + nb_step < NB) {  // the next block's first batches
      set_rows(nb + nb_step);
      fetch(0, 0);
      fetch(1, kU);
    }

    // ---- the four waves' tiles meet in wave 0: (2, 3) -> (0, 1), then 1 -> 0 ----
    if (w >= 2) {
#pragma unroll
      for (int t = 0; t < TILES; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[w - 2][t][r * 64 + lane] = acc[t][r];
    }
    __syncthreads();
    if (w < 2) {
#pragma unroll
      for (int t = 0; t < TILES; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += red[w][t][r * 64 + lane];
    }
    __syncthreads();
    if (w == 1) {
#pragma unroll
      for (int t = 0; t < TILES; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[2][t][r * 64 + lane] = acc[t][r];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int t = 0; t < TILES; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += red[2][t][r * 64 + lane];

      // ---- K split over workgroups: publish, take a ticket, last arriver sums ----
      bool finish = true;
      float ss = NORM ? ssq[lq] : 0.f;
      if (KS > 1) {
        float* mine = part + (static_cast<size_t>(nb) * KS + ks) * part_floats(SWIGLU);
#pragma unroll
        for (int t = 0; t < TILES; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) st_sc1(mine + t * kTile + r * 64 + lane, acc[t][r]);
        if (NORM && hh == 0) st_sc1(mine + TILES * kTile + lq, ss);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial is out before the ticket is taken
        unsigned got = 0;
        if (lane == 0) {
          got = __hip_atomic_fetch_add(tickets + nb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // back to 0 for the next launch: every other slice of this block has arrived
          if (got == static_cast<unsigned>(KS - 1))
            __hip_atomic_store(tickets + nb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        got = __builtin_amdgcn_readfirstlane(got);
        finish = got == static_cast<unsigned>(KS - 1);
        if (finish) {  // slice order, own partial re-read with the others: the sum does not depend on who is last
#pragma unroll
          for (int t = 0; t < TILES; ++t) acc[t] = f32x16{};
          ss = 0.f;
          for (int s = 0; s < KS; ++s) {
            const float* p = part + (static_cast<size_t>(nb) * KS + s) * part_floats(SWIGLU);
#pragma unroll
            for (int t = 0; t < TILES; ++t)
#pragma unroll
              for (int r = 0; r < 16; ++r) acc[t][r] += ld_sc1(p + t * kTile + r * 64 + lane);
            if (NORM) ss += ld_sc1(p + TILES * kTile + lq);
          }
        }
      }
      if (finish) {
        // ---- epilogue: lane = batch row lq, register r = weight row acc_row(r, hh) ----
        const float rstd = NORM ? rsqrtf(ss / static_cast<float>(K) + eps) : 1.f;
        unsigned long long key = 0ull;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int nn = nb * kNB + acc_row(r, hh);
          float v = acc[0][r] * rstd;
          if (SWIGLU) v = v / (1.f + __expf(-v)) * (acc[TILES - 1][r] * rstd);
          const bf16_t o = f2bf(v);
          if (lq < M && nn < N) {
            if (y) y[static_cast<size_t>(lq) * N + nn] = o;
            if (ARGMAX) {
              const unsigned long long kk = argmax_key(bf2f(o), nn);
              key = kk > key ? kk : key;
            }
          }
        }
        if (ARGMAX) {
          const unsigned long long other = __shfl_xor(key, 32, kWave);
          key = other > key ? other : key;
          if (hh == 0 && lq < M) best[static_cast<size_t>(lq) * NB + nb] = key;
        }
      }
    }
    // Next block: red[0] / red[1] are rewritten only after this block's second barrier (their
    // readers are done), red[2] only after the next block's second barrier, which wave 0
    // reaches after the epilogue above.
  }
}

// K slices for [N, K]: the fewest slices of <= kMaxSlice columns (multiples of
// 64).  A split costs every row block a publish -> ticket -> re-read chain of
// dependent memory round trips (~4 us), more than a workgroup that streams a
// few hundred KB on its own saves by sharing them; only a projection with too
// few row blocks to occupy a quarter of the CUs is split further.
int pick_slices(int N, int K, int cus) {
  const int nb = (N + kNB - 1) / kNB;
  int best = 0;
  for (int s = 1; s <= 64; ++s) {
    if (K % (s * 64) != 0) continue;
    const int ks = K / s;
    if (ks > kMaxSlice) continue;
    if (best == 0) best = s;
    if (ks < 256) break;
    best = s;
    if (nb * s >= cus / 4) break;
  }
  return best;
}

template <int MODE>
int launch(const void* x, const void* res, const void* g, void* h_out, float eps, const void* W, void* y,
           unsigned long long* best, float* part, unsigned* tickets, int M, int N, int K, int KS, int NB,
           int grid, hipStream_t s) {
  const size_t lds = static_cast<size_t>(kMB) * (K / KS + 8) * sizeof(bf16_t);
  // Dynamic LDS above the 64 KB default needs the per-kernel opt-in (once).
  static const bool opted = hipFuncSetAttribute(reinterpret_cast<const void*>(&skinny_kernel<MODE>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                kMB * (kMaxSlice + 8) * static_cast<int>(sizeof(bf16_t))) ==
                            hipSuccess;
  if (!opted && lds > 64 * 1024) return -1;
  hipLaunchKernelGGL(skinny_kernel<MODE>, dim3(grid), dim3(kT), lds, s, static_cast<const bf16_t*>(x),
                     static_cast<const bf16_t*>(res), static_cast<const bf16_t*>(g), static_cast<bf16_t*>(h_out),
                     eps, static_cast<const bf16_t*>(W), static_cast<bf16_t*>(y), best, part, tickets, M, N, K, KS,
                     NB);
  return KGWE_CHECK_LAUNCH();
}

}  // namespace

// Largest batch the kernel takes.
KGWE_API int kgwe_decode_skinny_max_m() { return kMB; }

// Weight-row blocks of an [N, K] projection = ARGMAX partial maxima per batch row.
KGWE_API int kgwe_decode_skinny_blocks(int N) { return (N + kNB - 1) / kNB; }

// K slices the launcher uses for [N, K] on `cus` compute units (0: unsupported K).
KGWE_API int kgwe_decode_skinny_slices(int N, int K, int cus) {
  if (N <= 0 || K <= 0 || K % 64) return 0;
  return pick_slices(N, K, cus > 0 ? cus : 256);
}

// Bytes of workspace for [N, K] (SWIGLU: N = F): split-K partials, then one
// ticket per row block.  Zero it once when it is allocated; every launch
// leaves the tickets at zero.
KGWE_API int64_t kgwe_decode_skinny_workspace(int N, int K, int swiglu, int cus) {
  const int ks = kgwe_decode_skinny_slices(N, K, cus);
  if (ks <= 0) return -1;
  const int64_t nb = (N + kNB - 1) / kNB;
  return (ks > 1 ? nb * ks * part_floats(swiglu != 0) * 4 : 0) + nb * 4;
}

// x [M, K] bf16 (8 < M <= 32 also takes M <= 8), W [N, K] (SWIGLU: [2N, K]),
// y [M, N] (may be null in the ARGMAX modes 4 and 5), K % 64 == 0.  NORM modes: res [M, K]
// or null, g [K], h_out [M, K] or null (must not alias x / res).  ARGMAX:
// best [M * kgwe_decode_skinny_blocks(N)] u64, one partial maximum per row
// block, reduced by kgwe_decode_argmax_finish.  `workspace` as sized by
// kgwe_decode_skinny_workspace for the same (N, K, swiglu, cus).  `cus`: the
// compute units this process may use (grid = up to 2 workgroups per CU;
// workgroups loop over row blocks beyond that).
KGWE_API int kgwe_decode_skinny(const void* x, const void* res, const void* g, void* h_out, float eps,
                                const void* W, void* y, unsigned long long* best, void* workspace, int M, int N,
                                int K, int mode, int cus, hipStream_t s) {
  if (M <= 0 || M > kMB || N <= 0 || K <= 0 || K % 64 || !workspace) return -1;
  if ((mode & kNorm) && !g) return -1;
  if ((mode & kArgmax) && !best) return -1;
  if (cus <= 0) cus = 256;
  const int KS = pick_slices(N, K, cus);
  if (KS <= 0) return -1;
  const int NB = (N + kNB - 1) / kNB;
  const bool sw = (mode & kSwiglu) != 0;
  float* part = static_cast<float*>(workspace);
  unsigned* tickets = reinterpret_cast<unsigned*>(part + (KS > 1 ? static_cast<int64_t>(NB) * KS * part_floats(sw) : 0));
  // workgroups resident per CU by LDS (160 KB): the grid is one residency, and a
  // workgroup loops over further row blocks with its slice of x staged once
  const int lds_wg = kMB * (K / KS + 8) * 2 + 3 * (sw ? 2 : 1) * kTile * 4 + 256;
  const int per_cu = std::max(1, std::min(4, 160 * 1024 / lds_wg));
  const int blocks = std::min(NB, std::max(1, per_cu * cus / KS));
  const int grid = blocks * KS;
  switch (mode) {
    case kPlain: return launch<kPlain>(x, res, g, h_out, eps, W, y, best, part, tickets, M, N, K, KS, NB, grid, s);
    case kNorm: return launch<kNorm>(x, res, g, h_out, eps, W, y, best, part, tickets, M, N, K, KS, NB, grid, s);
    case kSwiglu: return launch<kSwiglu>(x, res, g, h_out, eps, W, y, best, part, tickets, M, N, K, KS, NB, grid, s);
    case kArgmax: return launch<kArgmax>(x, res, g, h_out, eps, W, y, best, part, tickets, M, N, K, KS, NB, grid, s);
    case kNormSwiglu:
      return launch<kNormSwiglu>(x, res, g, h_out, eps, W, y, best, part, tickets, M, N, K, KS, NB, grid, s);
    case kNormArgmax:
      return launch<kNormArgmax>(x, res, g, h_out, eps, W, y, best, part, tickets, M, N, K, KS, NB, grid, s);
    default: return -1;
  }
}
