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
// One workgroup = one 64 x 64 tile, 256 threads: each thread moves two 16-B
// row chunks into LDS (row stride padded by 8 bf16 so the column reads of
// the write phase spread over the banks), then writes two 16-B chunks of the
// transposed tile gathered from LDS columns.  Partial tiles are guarded.
#include "common.h"

using namespace kgwe;

namespace {

constexpr int TT = 64;        // tile edge
constexpr int LST = TT + 8;   // LDS row stride (bf16)

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ src,
                                                             bf16_t* __restrict__ dst, int rows,
                                                             int cols, int tiles_c) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[TT * LST];
  const int tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int r0 = tr * TT, c0 = tc * TT;
  // load: chunk id = threadIdx.x + 256 i -> (row = id / 8, 8-col group = id % 8)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = threadIdx.x + 256 * i;
    const int r = id >> 3, cg = (id & 7) * 8;
    bf16x8 v = bf16x8{};
    if (r0 + r < rows && c0 + cg < cols)  // cols % 8 == 0: a chunk is all-in or all-out
      v = *reinterpret_cast<const bf16x8*>(src + static_cast<size_t>(r0 + r) * cols + c0 + cg);
    *reinterpret_cast<bf16x8*>(&tile[r * LST + cg]) = v;
  }
  __syncthreads();
  // store: output row = source column c, 8 consecutive source rows per chunk
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = threadIdx.x + 256 * i;
    const int c = id >> 3, rg = (id & 7) * 8;
    if (c0 + c < cols && r0 + rg < rows) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = tile[(rg + j) * LST + c];
      *reinterpret_cast<bf16x8*>(dst + static_cast<size_t>(c0 + c) * rows + r0 + rg) = v;
    }
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
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(static_cast<unsigned>(tiles_r * tiles_c)),
                     dim3(256), 0, s, static_cast<const bf16_t*>(src), static_cast<bf16_t*>(dst),
                     static_cast<int>(rows), static_cast<int>(cols), static_cast<int>(tiles_c));
  return KGWE_CHECK_LAUNCH();
}
