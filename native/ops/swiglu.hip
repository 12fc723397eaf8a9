// SwiGLU activation forward / backward (Llama FFN: silu(x W1) * (x W3)).
//
// gate / up are read through a row stride so the kernel consumes the fused
// [T, 2F] output of the concatenated w13 projection directly (g = cols
// [0, F), u = cols [F, 2F)) without a split copy.  bf16x8 (16 B) per lane,
// grid-stride, elementwise => HBM-bound; the backward writes dg and du into
// the matching halves of one [T, 2F] gradient so the w13 backward GEMM
// consumes it in place.
#include "common.h"

using namespace kgwe;

namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ u, int64_t in_stride,
    bf16_t* __restrict__ out, int64_t T, int F) {
  const int64_t vpr = F / 8;  // vectors per row
  const int64_t n = T * vpr;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL) {
    const int64_t r = i / vpr, c = (i - r * vpr) * 8;
    const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + r * in_stride + c);
    const bf16x8 uv = *reinterpret_cast<const bf16x8*>(u + r * in_stride + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = bf2f(gv[j]);
      o[j] = f2bf(x * sigmoidf_(x) * bf2f(uv[j]));
    }
    *reinterpret_cast<bf16x8*>(out + r * static_cast<int64_t>(F) + c) = o;
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ u, int64_t in_stride,
    const bf16_t* __restrict__ dout, bf16_t* __restrict__ dg,
    bf16_t* __restrict__ du, int64_t grad_stride, int64_t T, int F) {
  const int64_t vpr = F / 8;
  const int64_t n = T * vpr;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL) {
    const int64_t r = i / vpr, c = (i - r * vpr) * 8;
    const bf16x8 gv = *reinterpret_cast<const bf16x8*>(g + r * in_stride + c);
    const bf16x8 uv = *reinterpret_cast<const bf16x8*>(u + r * in_stride + c);
    const bf16x8 dv = *reinterpret_cast<const bf16x8*>(dout + r * static_cast<int64_t>(F) + c);
    bf16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = bf2f(gv[j]), y = bf2f(uv[j]), d = bf2f(dv[j]);
      const float s = sigmoidf_(x);
      const float silu = x * s;
      og[j] = f2bf(d * y * s * (1.f + x * (1.f - s)));
      ou[j] = f2bf(d * silu);
    }
    *reinterpret_cast<bf16x8*>(dg + r * grad_stride + c) = og;
    *reinterpret_cast<bf16x8*>(du + r * grad_stride + c) = ou;
  }
}

inline int grid_for(int64_t nvec) {
  // 256 CUs x 8 WGs of 256 threads is plenty to saturate HBM; cap the grid
  // and grid-stride beyond that.
  int64_t g = (nvec + 255) / 256;
  return static_cast<int>(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

}  // namespace

KGWE_API int kgwe_swiglu_fwd(const void* g, const void* u, int64_t in_stride,
                             void* out, int64_t T, int F, hipStream_t s) {
  if (F % 8 || in_stride % 8) return -1;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(T * F / 8)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(g), static_cast<const bf16_t*>(u),
                     in_stride, static_cast<bf16_t*>(out), T, F);
  return KGWE_CHECK_LAUNCH();
}

KGWE_API int kgwe_swiglu_bwd(const void* g, const void* u, int64_t in_stride,
                             const void* dout, void* dg, void* du,
                             int64_t grad_stride, int64_t T, int F, hipStream_t s) {
  if (F % 8 || in_stride % 8 || grad_stride % 8) return -1;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(T * F / 8)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(g), static_cast<const bf16_t*>(u),
                     in_stride, static_cast<const bf16_t*>(dout),
                     static_cast<bf16_t*>(dg), static_cast<bf16_t*>(du), grad_stride,
                     T, F);
  return KGWE_CHECK_LAUNCH();
}
