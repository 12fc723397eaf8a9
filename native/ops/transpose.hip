// bf16 matrix transpose through LDS (gfx950), used to put the weight-gradient
// GEMMs of a linear layer into the operand layouts hipBLASLt runs fastest.
//
// Why: with token-major activations X[T, K] and output gradients dY[T, N],
// dW = dY^T X reduces over the LEADING dimension of both stored operands —
// the "tn" layout, measured at ~1.1 PF/s on MI355X for the Llama-3-8B shapes
// against ~1.35 PF/s for "tt"/"nn" and ~1.5 PF/s for "nt"
// (tools/gemm_layouts.py).  Transposing the smaller operand (a [T, 4096]
// activation: 64 MB, ~25 us at HBM rate) before the GEMM buys 0.1-0.25 ms per
// large GEMM.
//
// No LDS: every thread transposes one 8 x 8 block in registers (8 row loads
// of 16 B, 8 column vectors rebuilt with byte permutes, 8 stores of 16 B).
// A wave covers a 64 x 64 tile as 8 (rows) x 8 (column groups) threads, so
// each load instruction reads 8 rows x 128 contiguous bytes and each store
// writes 8 output rows x 128 contiguous bytes.  The LDS version gathered
// its output chunks with 8 scalar ds_read_u16 per chunk: 48.7 us for a
// [16384, 4096] operand (5.5 TB/s read + write), 41.8 us now (6.4 TB/s,
// tools/transpose_bench.py).  A workgroup = 4 waves = 4 tiles side by side.
#include "common.h"

using namespace kgwe;

namespace {

constexpr int TT = 64;  // tile edge (one wave)

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ src,
                                                             bf16_t* __restrict__ dst, int rows,
                                                             int cols, int tiles_c) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tile = blockIdx.x * 4 + w;
  const int tr = tile / tiles_c, tc = tile % tiles_c;
  const int rb = tr * TT + 8 * (lane & 7);   // this thread's 8 source rows
  const int cb = tc * TT + 8 * (lane >> 3);  // and 8 source columns
  if (tr * TT >= rows || rb >= rows || cb >= cols) return;  // rows, cols % 8 == 0: blocks are whole
  bf16x8 in[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    in[i] = *reinterpret_cast<const bf16x8*>(src + static_cast<size_t>(rb + i) * cols + cb);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = in[i][j];
    *reinterpret_cast<bf16x8*>(dst + static_cast<size_t>(cb + j) * rows + rb) = o;
  }
}

}  // namespace

// dst[cols, rows] = src[rows, cols]^T, both row-major bf16, rows % 8 == 0 and
// cols % 8 == 0 (16-B chunks), non-overlapping.
KGWE_API int kgwe_transpose_bf16(const void* src, void* dst, int64_t rows, int64_t cols,
                                 hipStream_t s) {
  if (rows <= 0 || cols <= 0 || rows % 8 || cols % 8 || rows > 0x7fffffff || cols > 0x7fffffff)
    return -1;
  const int64_t tiles_r = (rows + TT - 1) / TT, tiles_c = (cols + TT - 1) / TT;
  if (tiles_r * tiles_c > 0x7fffffff) return -1;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(static_cast<unsigned>((tiles_r * tiles_c + 3) / 4)),
                     dim3(256), 0, s, static_cast<const bf16_t*>(src), static_cast<bf16_t*>(dst),
                     static_cast<int>(rows), static_cast<int>(cols), static_cast<int>(tiles_c));
  return KGWE_CHECK_LAUNCH();
}
