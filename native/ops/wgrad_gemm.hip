// Weight-gradient GEMM for gfx950 (MI355X): C[M, N] = A^T B with A = dY[T, M]
// and B = X[T, N], both bf16 row-major as autograd stores them, fp32
// accumulation on v_mfma_f32_32x32x16_bf16, bf16 (or fp32 split-K slab) out.
//
// Why a kernel of our own: dW = dY^T X reduces over the LEADING (token)
// dimension of both stored operands.  For the vendor GEMM that is its slowest
// layout on this chip; the usual cure, transposing one operand first, costs a
// launch and 2 x 64 MB of HBM traffic per GEMM.  Here neither operand is ever
// transposed in memory: tiles are copied HBM -> LDS as they are, rows of
// tokens, by LDS-DMA (global_load_lds, 16 B per lane, no VGPR round trip), and
// every MFMA operand is read out of LDS with the hardware-transposing
// ds_read_b64_tr_b16, which hands each lane four consecutive tokens of its
// column.  Since BOTH operands go through the same transposed read, the k
// (token) order inside a fragment only has to agree between A and B.
//
// Geometry: 256 x 256 output tile per workgroup, 64 tokens per K-tile, 8
// waves (2 x 4), each wave 128 x 64 of C = 8 accumulators of 32 x 32.  LDS per
// stage: A and B tiles as two [64 tokens][128 columns] images each (256-B
// rows = one LDS bank row), 16-B chunks XOR-swizzled by token row so the
// transposed reads of a 32-lane half touch 64 distinct banks; the swizzle is
// applied to the SOURCE address of the LDS-DMA (its LDS destination is always
// wave-linear) and to the read address.  Two stages (128 KiB): the DMA of
// K-tile t+1 is issued during the first half of K-tile t and waited for (vmcnt)
// at its end, one workgroup barrier per K-tile.  Workgroups are numbered so
// that the 32 tiles resident on one XCD form an 8 x 4 patch sharing A and B
// panels in that XCD's L2.
#include "common.h"

using namespace kgwe;

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 mfma8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kThreads = 512;
constexpr int kImage = 64 * 256;          // bytes of one [64][128] bf16 image
constexpr int kStage = 4 * kImage;        // A half 0, A half 1, B half 0, B half 1
constexpr int kLds = 2 * kStage;          // 128 KiB
constexpr int GROUP_M = 8;                // tile rows per L2 patch (8 x 4 tiles per XCD wave)

__device__ __forceinline__ u16x4 tr_read(const char* p) {
  typedef __attribute__((ext_vector_type(4))) short s4;
  const s4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(p));
  return __builtin_bit_cast(u16x4, r);
}

__device__ __forceinline__ bf16x8 cat44(u16x4 lo, u16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(mfma8, a), __builtin_bit_cast(mfma8, b), c,
                                                 0, 0, 0);
}

__device__ __forceinline__ void glds16(const bf16_t* src, char* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

// OUT_F32: write this workgroup's fp32 partial tile (split-K slab) instead of
// the bf16 result.
template <bool OUT_F32>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(const bf16_t* __restrict__ A,
                                                         const bf16_t* __restrict__ B, void* __restrict__ Cout,
                                                         int M, int N, int T, int lda, int ldb, int ldc,
                                                         int splits) {
  // One array per stage, not one array of two stages: hipcc orders a ds_read
  // after every LDS-DMA in flight (s_waitcnt vmcnt(0)) unless it can prove
  // the two do not alias, which it can for distinct LDS objects.  With one
  // array the next tile's DMA was drained before every fragment read.
  __shared__ __attribute__((aligned(1024))) char lds0[kStage];
  __shared__ __attribute__((aligned(1024))) char lds1[kStage];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // ---- tile of this workgroup (XCD-contiguous, GROUP_M-row patches) ----
  const int tiles_m = M / BM, tiles_n = N / BN;
  const int ntile = tiles_m * tiles_n;
  int id = xcd_remap(static_cast<int>(blockIdx.x), ntile * splits);
  const int split = id % splits;
  id /= splits;
  const int per_group = GROUP_M * tiles_n;
  const int grp = id / per_group;
  const int first_m = grp * GROUP_M;
  const int gsz = min(GROUP_M, tiles_m - first_m);
  const int tm = first_m + (id % per_group) % gsz;
  const int tn = (id % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  // K range of this split (in K-tiles)
  const int nt_all = T / BK;
  const int per = (nt_all + splits - 1) / splits;
  const int kt0 = split * per;
  const int nt = max(0, min(per, nt_all - kt0));

  // ---- LDS-DMA source geometry: one wave instruction = 4 token rows x 256 B ----
  const int lrow = lane >> 4, cp = lane & 15;
  const int half_ld = wave >> 2;       // which 128-column half this wave stages
  const int rg0 = (wave & 3) * 4;      // its 4 row groups: rg0 .. rg0 + 3
  int goffA[4], goffB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * (rg0 + i) + lrow;             // token row inside the K-tile
    const int ch = cp ^ ((lrow << 2) | i);            // (row & 3) = lrow, ((row >> 2) & 3) = i
    goffA[i] = row * lda + half_ld * 128 + ch * 8;
    goffB[i] = row * ldb + half_ld * 128 + ch * 8;
  }
  const bf16_t* gA = A + static_cast<size_t>(kt0) * BK * lda + m0;
  const bf16_t* gB = B + static_cast<size_t>(kt0) * BK * ldb + n0;
  const int lds_ld = half_ld * kImage + rg0 * 1024;   // wave-uniform destination inside a tile pair

  // ---- transposed-read geometry (32x32x16 operand, k = token) ----
  // lane group G = lane >> 4: k half h = G >> 1, column half rh = G & 1;
  // lane 4q + p of the group supplies row q, 8-byte piece p of the block.
  const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, h = G >> 1, rh = G & 1;
  int offp[2];
#pragma unroll
  for (int part = 0; part < 2; ++part)
    offp[part] = 256 * (8 * h + q + 4 * part) + 16 * ((2 * rh + (p >> 1)) ^ (2 * h + part)) + 8 * (p & 1);
  int aoff[4][2], boff[2][2];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int part = 0; part < 2; ++part) aoff[cb][part] = offp[part] + 64 * (cb ^ q);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int part = 0; part < 2; ++part) boff[j][part] = offp[part] + 64 * ((2 * (wn & 1) + j) ^ q);
  const int imgA = wm * kImage;                          // this wave's A image in a stage
  const int imgB = 2 * kImage + (wn >> 1) * kImage;      // and its B image

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto stage_a = [&](int stage, int t) {
    const bf16_t* a = gA + static_cast<size_t>(t) * BK * lda;
    char* d = (stage ? lds1 : lds0) + lds_ld;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(a + goffA[i], d + i * 1024);
  };
  auto stage_b = [&](int stage, int t) {
    const bf16_t* b = gB + static_cast<size_t>(t) * BK * ldb;
    char* d = (stage ? lds1 : lds0) + 2 * kImage + lds_ld;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(b + goffB[i], d + i * 1024);
  };
  auto frags = [&](const char* sa, const char* sb, int R, bf16x8 (&fa)[4], bf16x8 (&fb)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      fb[j] = cat44(tr_read(sb + 256 * R + boff[j][0]), tr_read(sb + 256 * R + boff[j][1]));
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i] = cat44(tr_read(sa + 256 * R + aoff[i][0]), tr_read(sa + 256 * R + aoff[i][1]));
  };
  auto mma = [&](const bf16x8 (&fa)[4], const bf16x8 (&fb)[2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma(fa[i], fb[j], acc[i][j]);
  };
  // One K-tile out of stage `stage`; prefetches K-tile t + 1 into the other.
  auto ktile = [&](int stage, int t) {
    const char* sa = (stage ? lds1 : lds0) + imgA;
    const char* sb = (stage ? lds1 : lds0) + imgB;
    const bool more = t + 1 < nt;
    bf16x8 fa0[4], fb0[2], fa1[4], fb1[2];
    frags(sa, sb, 0, fa0, fb0);
    if (more) stage_a(stage ^ 1, t + 1);
    frags(sa, sb, 16, fa1, fb1);
    mma(fa0, fb0);
    if (more) stage_b(stage ^ 1, t + 1);
    frags(sa, sb, 32, fa0, fb0);
    mma(fa1, fb1);
    frags(sa, sb, 48, fa1, fb1);
    mma(fa0, fb0);
    mma(fa1, fb1);
    // K-tile t + 1 has landed (all of this wave's DMAs), and after the barrier
    // everyone's; every wave is also done reading this stage, which the DMAs
    // of K-tile t + 2 overwrite.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };

  if (nt > 0) {
    stage_a(0, 0);
    stage_b(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; t += 2) {
      ktile(0, t);
      if (t + 1 < nt) ktile(1, t + 1);
    }
  }

  // ---- epilogue: C row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5), col = lane & 31 ----
  const int crow = m0 + wm * 128 + 4 * (lane >> 5);
  const int ccol = n0 + wn * 64 + (lane & 31);
  if (OUT_F32) {
    float* C = static_cast<float*>(Cout) + static_cast<size_t>(split) * M * ldc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          C[static_cast<size_t>(crow + 32 * i + (r & 3) + 8 * (r >> 2)) * ldc + ccol + 32 * j] = acc[i][j][r];
  } else {
    bf16_t* C = static_cast<bf16_t*>(Cout);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          C[static_cast<size_t>(crow + 32 * i + (r & 3) + 8 * (r >> 2)) * ldc + ccol + 32 * j] =
              f2bf(acc[i][j][r]);
  }
}

// Sum of the split-K slabs -> bf16.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slabs,
                                                           bf16_t* __restrict__ C, int64_t n, int splits) {
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  f32x4 s = *reinterpret_cast<const f32x4*>(slabs + i);
  for (int k = 1; k < splits; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(slabs + static_cast<int64_t>(k) * n + i);
    s += v;
  }
  typedef __attribute__((ext_vector_type(4))) unsigned short u4;
  u4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = f2bf(s[k]);
  *reinterpret_cast<u4*>(C + i) = o;
}

}  // namespace

// Split count the launcher will use for C[M, N] over T tokens: whole waves of
// 256 workgroups where that is cheap (every split adds an fp32 slab round trip).
KGWE_API int kgwe_wgrad_splits(int M, int N, int T) {
  if (M <= 0 || N <= 0 || T <= 0 || M % BM || N % BN || T % BK) return 0;
  const int tiles = (M / BM) * (N / BN);
  const int nt = T / BK;
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 4 && s * 8 <= nt; ++s) {
    const int wg = tiles * s;
    const int rounds = (wg + 255) / 256;
    // time ~ rounds x K-tiles per split, plus the slab write + read for s > 1
    const double cost = rounds * ((nt + s - 1) / s) + (s > 1 ? 0.02 * nt * s : 0.0);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = s;
    }
  }
  return best;
}

// Bytes of fp32 workspace kgwe_wgrad_bf16 needs for this shape (0: none).
KGWE_API int64_t kgwe_wgrad_workspace(int M, int N, int T) {
  const int s = kgwe_wgrad_splits(M, N, T);
  return s > 1 ? static_cast<int64_t>(s) * M * N * 4 : 0;
}

// C[M, N] (bf16, row stride ldc) = A[T, M]^T B[T, N]; lda / ldb row strides in
// elements.  M, N % 256 == 0, T % 64 == 0, strides % 8 == 0, 16-B aligned
// bases.  `splits` 0 = choose (kgwe_wgrad_splits); > 1 needs `workspace`.
// Returns 0, -1 for an unsupported shape, -2 for a missing workspace, else the
// HIP error of the launch.
KGWE_API int kgwe_wgrad_bf16(const void* A, const void* B, void* C, void* workspace, int M, int N, int T,
                             int lda, int ldb, int ldc, int splits, hipStream_t s) {
  if (M <= 0 || N <= 0 || T <= 0 || M % BM || N % BN || T % BK) return -1;
  if (lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -1;
  // (32-bit offsets in the kernel span one K-tile only: 64 rows x stride; the per-tile base is 64-bit.)
  if (static_cast<int64_t>(BK) * lda > 0x7fffffffLL || static_cast<int64_t>(BK) * ldb > 0x7fffffffLL) return -1;
  if (splits <= 0) splits = kgwe_wgrad_splits(M, N, T);
  if (splits < 1 || splits > 16 || splits > T / BK) return -1;
  const int tiles = (M / BM) * (N / BN);
  const bf16_t* a = static_cast<const bf16_t*>(A);
  const bf16_t* b = static_cast<const bf16_t*>(B);
  if (splits == 1) {
    hipLaunchKernelGGL(wgrad_kernel<false>, dim3(tiles), dim3(kThreads), 0, s, a, b, C, M, N, T, lda, ldb, ldc, 1);
    return KGWE_CHECK_LAUNCH();
  }
  if (!workspace) return -2;
  if (ldc != N) return -1;  // slabs are dense [splits][M][N]
  hipLaunchKernelGGL(wgrad_kernel<true>, dim3(tiles * splits), dim3(kThreads), 0, s, a, b, workspace, M, N, T, lda,
                     ldb, N, splits);
  if (int rc = KGWE_CHECK_LAUNCH()) return rc;
  const int64_t n = static_cast<int64_t>(M) * N;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(static_cast<unsigned>((n / 4 + 255) / 256)), dim3(256), 0, s,
                     static_cast<const float*>(workspace), static_cast<bf16_t*>(C), n, splits);
  return KGWE_CHECK_LAUNCH();
}
