// Decode-time projections (M <= 8 new tokens) for gfx950: weight-streaming
// skinny GEMMs with the decode layer's elementwise work fused in.
//
//   y[m, n] = sum_k x[m, k] W[n, k]          W: [N, K] bf16 (nn.Linear layout)
//
// At M = 4 a projection reads each weight byte once for 4 FLOP: it is an HBM
// stream, and hipBLASLt's tile GEMMs ran the decode step's small matrices at
// 1-4 TB/s (profiles/r02_colocate: wqkv 12.6 MB in 10.9 us).  Here one
// workgroup stages the M input rows in LDS once and every wave streams R
// weight rows (64/R lanes per row, 16 B per lane per load, UNROLL loads in
// flight) into v_dot2_f32_bf16 against the LDS copy, then reduces across its
// row's lanes with DPP-shuffles.  Modes fuse the layer around the GEMM:
//
//   NORM     x_in = bf16(x + res) (h, the new residual stream, written by
//            workgroup 0), then bf16(x_in * rstd * g) — the RMSNorm that
//            precedes wqkv / w13 / the LM head (rmsnorm.hip semantics);
//   SWIGLU   W = [gate; up] ([2F, K]); y[m, n] = silu(g) * u of rows n, F + n
//            (fp32, one rounding) — the FFN's w13 + SwiGLU in one pass;
//   ARGMAX   the logits also feed a per-row (value, index) atomicMax, so the
//            greedy token needs no separate argmax over the vocabulary.
//
// Every kernel here is graph-safe (no host sync, fixed grids).
#include <algorithm>

#include "common.h"

using namespace kgwe;

namespace {

constexpr int kMaxM = 8;
constexpr int kThreads = 256;

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;

// 8-wide bf16 dot into fp32: four v_dot2c_f32_bf16.  The pairs are cut with
// shufflevector on a __bf16 vector: extracting them through a bit-cast u32
// vector miscompiles (hipcc folded all four words into the first one).
__device__ __forceinline__ float dot8(const bf16x8& a, const bf16x8& b, float acc) {
  const bf16x8v A = __builtin_bit_cast(bf16x8v, a), Bv = __builtin_bit_cast(bf16x8v, b);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(A, A, 0, 1), __builtin_shufflevector(Bv, Bv, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(A, A, 2, 3), __builtin_shufflevector(Bv, Bv, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(A, A, 4, 5), __builtin_shufflevector(Bv, Bv, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(A, A, 6, 7), __builtin_shufflevector(Bv, Bv, 6, 7), acc, false);
  return acc;
}

// Reduce across the L lanes of one row group (L = 64 / R, groups aligned).
template <int L>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Orderable key of (value, index): larger value wins, then the SMALLER index
// (torch.argmax picks the first maximum).  Value bits: IEEE -> monotone u32.
__device__ __forceinline__ unsigned long long argmax_key(float v, int n) {
  unsigned u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return (static_cast<unsigned long long>(u) << 32) | static_cast<unsigned>(~n);
}

enum Mode { kPlain = 0, kNorm = 1, kSwiglu = 2, kNormSwiglu = 3, kNormArgmax = 5 };

// Stage x (or the normalised x) of the M rows into LDS as bf16.
template <bool NORM>
__device__ __forceinline__ void stage_x(bf16_t* xs, const bf16_t* __restrict__ x,
                                        const bf16_t* __restrict__ res, const bf16_t* __restrict__ g,
                                        bf16_t* __restrict__ h_out, float eps, int M, int K,
                                        float* red) {
  const int chunks = K / 8;
  for (int m = 0; m < M; ++m) {
    const bf16_t* xr = x + static_cast<size_t>(m) * K;
    const bf16_t* rr = res ? res + static_cast<size_t>(m) * K : nullptr;
    float ss = 0.f;
    for (int c = threadIdx.x; c < chunks; c += kThreads) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(xr + 8 * c);
      if (NORM) {
        if (rr) {
          const bf16x8 r = *reinterpret_cast<const bf16x8*>(rr + 8 * c);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) + bf2f(r[j]));
          if (h_out && blockIdx.x == 0)
            *reinterpret_cast<bf16x8*>(h_out + static_cast<size_t>(m) * K + 8 * c) = v;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += bf2f(v[j]) * bf2f(v[j]);
      }
      *reinterpret_cast<bf16x8*>(xs + static_cast<size_t>(m) * K + 8 * c) = v;
    }
    if (NORM) {
      ss = wave_sum(ss);
      if ((threadIdx.x & 63) == 0) red[m * 4 + (threadIdx.x >> 6)] = ss;
    }
  }
  __syncthreads();
  if (NORM) {
    for (int m = 0; m < M; ++m) {
      const float ss = red[m * 4] + red[m * 4 + 1] + red[m * 4 + 2] + red[m * 4 + 3];
      const float rstd = rsqrtf(ss / static_cast<float>(K) + eps);
      bf16_t* xr = xs + static_cast<size_t>(m) * K;
      for (int c = threadIdx.x; c < chunks; c += kThreads) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(xr + 8 * c);
        const bf16x8 w = *reinterpret_cast<const bf16x8*>(g + 8 * c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * rstd * bf2f(w[j]));
        *reinterpret_cast<bf16x8*>(xr + 8 * c) = v;
      }
    }
    __syncthreads();
  }
}

// One workgroup = 4 waves; wave w streams rows [row0, row0 + R) with
// L = 64 / R lanes per row.  MODE & kSwiglu: the "row" n is the pair (n, F+n).
template <int R, int M, int MODE>
__global__ __launch_bounds__(kThreads) void gemv_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, const bf16_t* __restrict__ g,
    bf16_t* __restrict__ h_out, float eps, const bf16_t* __restrict__ W, bf16_t* __restrict__ y,
    unsigned long long* __restrict__ best, int N, int K) {
  constexpr bool NORM = MODE & kNorm;
  constexpr bool SWIGLU = MODE & kSwiglu;
  constexpr bool ARGMAX = MODE == kNormArgmax;
  constexpr int L = kWave / R;
  constexpr int UNROLL = 8;  // whole 4 KB rows in flight at K = 2048
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];  // [M][K]
  __shared__ float red[kMaxM * 4];
  __shared__ unsigned long long amax[kMaxM * 4];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane / L, li = lane % L;
  // Workgroups loop over blocks of 4 R columns (grid capped at a few per
  // visible CU): the staging below is paid once per workgroup, not once per
  // block — under a CoLocate CU mask (32 CUs) an uncapped grid repeated it
  // 8x as often per CU and ran slower than hipBLASLt.
  const int nblk = (N + 4 * R - 1) / (4 * R);
  int blk = blockIdx.x;
  int n = (blk * 4 + w) * R + r;  // output column of this lane group
  bool valid = n < N;
  const bf16_t* wg = W + static_cast<size_t>(valid ? n : 0) * K;
  const bf16_t* wu = SWIGLU ? W + static_cast<size_t>(valid ? N + n : 0) * K : nullptr;
  const int stride = 8 * L;  // elements per lane-group pass
  // The first UNROLL weight chunks are requested BEFORE the input rows are
  // staged, so their HBM latency overlaps the staging (at K <= 8 * L *
  // UNROLL that is the whole row: decode projections are latency-bound).
  bf16x8 wv[UNROLL], uv[SWIGLU ? UNROLL : 1];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const bool in = valid && k0 + u * stride < K;
      wv[u] = in ? *reinterpret_cast<const bf16x8*>(wg + k0 + u * stride) : bf16x8{};
      if (SWIGLU) uv[u] = in ? *reinterpret_cast<const bf16x8*>(wu + k0 + u * stride) : bf16x8{};
    }
  };
  fetch(8 * li);
  // x is staged in LDS in every mode: read from global memory inside the dot
  // loop, each x load's vmcnt wait also drained the weight loads in flight
  // (one counter), serialising the stream.  LDS reads wait on lgkmcnt.
  stage_x<NORM>(xs, x, res, g, h_out, eps, M, K, red);
  const bf16_t* xsrc = xs;
  unsigned long long run[ARGMAX ? M : 1];
#pragma unroll
  for (int m = 0; m < (ARGMAX ? M : 1); ++m) run[m] = 0ull;

  for (; blk < nblk; blk += gridDim.x) {
    float acc[M], accu[SWIGLU ? M : 1];
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = 0.f;
    if (SWIGLU)
#pragma unroll
      for (int m = 0; m < M; ++m) accu[m] = 0.f;
    for (int k = 8 * li; k < K; k += UNROLL * stride) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (k + u * stride >= K) break;  // lane-group uniform
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xsrc + static_cast<size_t>(m) * K + k + u * stride);
          acc[m] = dot8(wv[u], xv, acc[m]);
          if (SWIGLU) accu[m] = dot8(uv[SWIGLU ? u : 0], xv, accu[m]);
        }
      }
      if (k + UNROLL * stride < K) fetch(k + UNROLL * stride);
    }
    const int n_done = n;
    const bool valid_done = valid;
    const int nb = blk + gridDim.x;  // prefetch the next block's rows now
    if (nb < nblk) {
      n = (nb * 4 + w) * R + r;
      valid = n < N;
      wg = W + static_cast<size_t>(valid ? n : 0) * K;
      if (SWIGLU) wu = W + static_cast<size_t>(valid ? N + n : 0) * K;
      fetch(8 * li);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      acc[m] = group_sum<L>(acc[m]);
      if (SWIGLU) accu[m] = group_sum<L>(accu[m]);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float v = acc[m];
      if (SWIGLU) v = v / (1.f + __expf(-v)) * accu[m];
      const bf16_t o = f2bf(v);
      if (y && valid_done && li == 0) y[static_cast<size_t>(m) * N + n_done] = o;
      if (ARGMAX && valid_done) {
        const unsigned long long key = argmax_key(bf2f(o), n_done);
        run[ARGMAX ? m : 0] = key > run[ARGMAX ? m : 0] ? key : run[ARGMAX ? m : 0];
      }
    }
  }
  if (ARGMAX) {
    // Workgroup argmax over every column it produced, ONE partial per
    // workgroup (best[m * gridDim.x + block]); argmax_finish reduces them.
    // (A global atomicMax per column serialised 500k atomics on M words.)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      unsigned long long key = run[ARGMAX ? m : 0];
#pragma unroll
      for (int off = L; off < kWave; off <<= 1) {
        const unsigned long long o = __shfl_xor(key, off, kWave);
        key = o > key ? o : key;
      }
      if (lane == 0) amax[m * 4 + w] = key;
    }
    __syncthreads();
    if (threadIdx.x < M) {
      const int m = threadIdx.x;
      unsigned long long b = amax[m * 4];
#pragma unroll
      for (int i = 1; i < 4; ++i) b = amax[m * 4 + i] > b ? amax[m * 4 + i] : b;
      best[static_cast<size_t>(m) * gridDim.x + blockIdx.x] = b;
    }
  }
}

template <int R, int M, int MODE>
int launch_one(const dim3& grid, size_t lds, const bf16_t* x, const bf16_t* res, const bf16_t* g,
               bf16_t* h_out, float eps, const bf16_t* W, bf16_t* y, unsigned long long* best, int N,
               int K, hipStream_t s) {
  // Dynamic LDS above the 64 KB default needs the per-kernel opt-in (once).
  static const bool opted = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemv_kernel<R, M, MODE>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                96 * 1024) == hipSuccess;
  if (!opted && lds > 64 * 1024) return -1;
  hipLaunchKernelGGL((gemv_kernel<R, M, MODE>), grid, dim3(kThreads), lds, s, x, res, g, h_out, eps, W, y,
                     best, N, K);
  return KGWE_CHECK_LAUNCH();
}

template <int R, int M>
int launch_m(int mode, const void* x, const void* res, const void* g, void* h_out, float eps,
             const void* W, void* y, unsigned long long* best, int N, int K, int max_wgs, hipStream_t s) {
  const int rows_per_wg = 4 * R;
  const int nblk = (N + rows_per_wg - 1) / rows_per_wg;
  const dim3 grid(max_wgs > 0 ? std::min(nblk, max_wgs) : nblk);
  const size_t lds = static_cast<size_t>(M) * K * sizeof(bf16_t);
  auto X = static_cast<const bf16_t*>(x);
  auto RS = static_cast<const bf16_t*>(res);
  auto G = static_cast<const bf16_t*>(g);
  auto H = static_cast<bf16_t*>(h_out);
  auto Wp = static_cast<const bf16_t*>(W);
  auto Y = static_cast<bf16_t*>(y);
  switch (mode) {
    case kPlain: return launch_one<R, M, kPlain>(grid, lds, X, RS, G, H, eps, Wp, Y, best, N, K, s);
    case kNorm: return launch_one<R, M, kNorm>(grid, lds, X, RS, G, H, eps, Wp, Y, best, N, K, s);
    case kSwiglu: return launch_one<R, M, kSwiglu>(grid, lds, X, RS, G, H, eps, Wp, Y, best, N, K, s);
    case kNormSwiglu: return launch_one<R, M, kNormSwiglu>(grid, lds, X, RS, G, H, eps, Wp, Y, best, N, K, s);
    case kNormArgmax: return launch_one<R, M, kNormArgmax>(grid, lds, X, RS, G, H, eps, Wp, Y, best, N, K, s);
    default: return -1;
  }
}

template <int R>
int launch_r(int M, int mode, const void* x, const void* res, const void* g, void* h_out, float eps,
             const void* W, void* y, unsigned long long* best, int N, int K, int max_wgs, hipStream_t s) {
  switch (M) {
    case 1: return launch_m<R, 1>(mode, x, res, g, h_out, eps, W, y, best, N, K, max_wgs, s);
    case 2: return launch_m<R, 2>(mode, x, res, g, h_out, eps, W, y, best, N, K, max_wgs, s);
    case 4: return launch_m<R, 4>(mode, x, res, g, h_out, eps, W, y, best, N, K, max_wgs, s);
    case 8: return launch_m<R, 8>(mode, x, res, g, h_out, eps, W, y, best, N, K, max_wgs, s);
    default: return -1;
  }
}

// One workgroup (1024 threads, 4 loads in flight each) per row m: the max of
// the workgroups' partial keys.
constexpr int kFinishThreads = 1024;
__global__ __launch_bounds__(kFinishThreads) void argmax_finish_kernel(
    const unsigned long long* __restrict__ best, long long* __restrict__ tok, int slots) {
  __shared__ unsigned long long part[kFinishThreads / kWave];
  const int m = blockIdx.x;
  const unsigned long long* row = best + static_cast<size_t>(m) * slots;
  unsigned long long b = 0ull;
  for (int i = threadIdx.x; i < slots; i += 4 * kFinishThreads) {
    unsigned long long v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = i + u * kFinishThreads;
      v[u] = j < slots ? row[j] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) b = v[u] > b ? v[u] : b;
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(b, off, kWave);
    b = o > b ? o : b;
  }
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kFinishThreads / kWave; ++i) b = part[i] > b ? part[i] : b;
    tok[m] = static_cast<long long>(~static_cast<unsigned>(b & 0xffffffffull));
  }
}

}  // namespace

// x [M, K] bf16 (M in {1, 2, 4, 8}; pad the batch), W [N, K] (SWIGLU: [2N, K]),
// y [M, N] (may be null in ARGMAX mode), K % 8 == 0.  NORM modes: res [M, K]
// or null, g [K], h_out [M, K] or null (must not alias x / res).  ARGMAX:
// best [M * kgwe_decode_argmax_slots(N, rows_per_wave)] u64: one partial
// maximum per workgroup, reduced by kgwe_decode_argmax_finish.
// rows_per_wave: 1, 2 or 4 (more rows per wave = fewer lanes per row).
// max_wgs > 0 caps the grid (workgroups then loop over column blocks).
KGWE_API int kgwe_decode_gemv(const void* x, const void* res, const void* g, void* h_out, float eps,
                              const void* W, void* y, unsigned long long* best, int M, int N, int K,
                              int mode, int rows_per_wave, int max_wgs, hipStream_t s) {
  if (K % 8 || N <= 0 || K <= 0 || M <= 0 || M > kMaxM) return -1;
  if (static_cast<size_t>(M) * K * sizeof(bf16_t) > 96 * 1024) return -1;  // LDS staging bound
  if ((mode & kNorm) && !g) return -1;
  if (mode == kNormArgmax && !best) return -1;
  switch (rows_per_wave) {
    case 1: return launch_r<1>(M, mode, x, res, g, h_out, eps, W, y, best, N, K, max_wgs, s);
    case 2: return launch_r<2>(M, mode, x, res, g, h_out, eps, W, y, best, N, K, max_wgs, s);
    case 4: return launch_r<4>(M, mode, x, res, g, h_out, eps, W, y, best, N, K, max_wgs, s);
    default: return -1;
  }
}

KGWE_API int kgwe_decode_argmax_slots(int N, int rows_per_wave, int max_wgs) {
  const int nblk = (N + 4 * rows_per_wave - 1) / (4 * rows_per_wave);  // workgroups of the ARGMAX launch
  return max_wgs > 0 ? std::min(nblk, max_wgs) : nblk;
}

KGWE_API int kgwe_decode_argmax_finish(const unsigned long long* best, long long* tok, int M, int slots,
                                       hipStream_t s) {
  if (M <= 0 || M > 64 || slots <= 0) return -1;  // one workgroup per batch row (gemv: <= 8, skinny_gemm: <= 32)
  hipLaunchKernelGGL(argmax_finish_kernel, dim3(M), dim3(kFinishThreads), 0, s, best, tok, slots);
  return KGWE_CHECK_LAUNCH();
}
