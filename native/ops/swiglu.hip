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

// Row-major walk: a workgroup takes whole rows (grid-stride over rows) and
// its threads stride over the row's 16-B vectors, U vectors per thread per
// pass with all loads issued before any use.  The flat-index form (one
// vector per thread per pass, row / column by 64-bit division) kept only 2-3
// loads in flight per lane and spent VALU on the division: at T=16384,
// F=14336 forward 262 -> 251 us, backward 453 -> 439 us (tools/swiglu_ab.hip).
#ifndef SWIGLU_U
#define SWIGLU_U 4
#endif
constexpr int U = SWIGLU_U;

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ u, int64_t in_stride,
    bf16_t* __restrict__ out, int64_t T, int F) {
  const int vpr = F / 8;  // 16-B vectors per row
  for (int64_t r = blockIdx.x; r < T; r += gridDim.x) {
    const bf16_t* gr = g + r * in_stride;
    const bf16_t* ur = u + r * in_stride;
    bf16_t* orow = out + r * static_cast<int64_t>(F);
    for (int c0 = threadIdx.x; c0 < vpr; c0 += 256 * U) {
      bf16x8 gv[U], uv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int c = c0 + 256 * k;
        if (c < vpr) {
          gv[k] = *reinterpret_cast<const bf16x8*>(gr + 8 * c);
          uv[k] = *reinterpret_cast<const bf16x8*>(ur + 8 * c);
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int c = c0 + 256 * k;
        if (c >= vpr) break;
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = bf2f(gv[k][j]);
          o[j] = f2bf(x * sigmoidf_(x) * bf2f(uv[k][j]));
        }
        *reinterpret_cast<bf16x8*>(orow + 8 * c) = o;
      }
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ u, int64_t in_stride,
    const bf16_t* __restrict__ dout, bf16_t* __restrict__ dg,
    bf16_t* __restrict__ du, int64_t grad_stride, int64_t T, int F) {
  const int vpr = F / 8;
  for (int64_t r = blockIdx.x; r < T; r += gridDim.x) {
    const bf16_t* gr = g + r * in_stride;
    const bf16_t* ur = u + r * in_stride;
    const bf16_t* dr = dout + r * static_cast<int64_t>(F);
    bf16_t* dgr = dg + r * grad_stride;
    bf16_t* dur = du + r * grad_stride;
    for (int c0 = threadIdx.x; c0 < vpr; c0 += 256 * U) {
      bf16x8 gv[U], uv[U], dv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int c = c0 + 256 * k;
        if (c < vpr) {
          gv[k] = *reinterpret_cast<const bf16x8*>(gr + 8 * c);
          uv[k] = *reinterpret_cast<const bf16x8*>(ur + 8 * c);
          dv[k] = *reinterpret_cast<const bf16x8*>(dr + 8 * c);
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int c = c0 + 256 * k;
        if (c >= vpr) break;
        bf16x8 og, ou;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = bf2f(gv[k][j]), y = bf2f(uv[k][j]), d = bf2f(dv[k][j]);
          const float s = sigmoidf_(x);
          const float silu = x * s;
          og[j] = f2bf(d * y * s * (1.f + x * (1.f - s)));
          ou[j] = f2bf(d * silu);
        }
        *reinterpret_cast<bf16x8*>(dgr + 8 * c) = og;
        *reinterpret_cast<bf16x8*>(dur + 8 * c) = ou;
      }
    }
  }
}

// Backward that ALSO writes the gradient transposed: dguT [2F, T] (token
// dimension contiguous).  The w13 weight-gradient GEMM dW = dGU^T X reduces
// over tokens; with dGU^T (and X^T) at hand it runs in the library's fastest
// layout (both operands K-contiguous: 2.43 ms against 2.84 ms per layer at
// Llama-3-8B, 16,384 tokens), and producing the transposed copy here costs
// one extra write of the tile that is already in registers instead of a
// separate read-and-write pass.  One workgroup = a 64-token x 64-feature
// tile, transposed through LDS (pitch 72 elements keeps the 16-B reads
// aligned).
constexpr int kTT = 64, kPitch = 72;

__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ u, int64_t in_stride,
    const bf16_t* __restrict__ dout, bf16_t* __restrict__ dg, bf16_t* __restrict__ du, int64_t grad_stride,
    bf16_t* __restrict__ dguT, int64_t T, int F) {
  __shared__ __attribute__((aligned(16))) bf16_t sg[kTT * kPitch];
  __shared__ __attribute__((aligned(16))) bf16_t su[kTT * kPitch];
  const int tiles_c = F / kTT;
  const int64_t tile = blockIdx.x;
  const int64_t r0 = (tile / tiles_c) * kTT;
  const int c0 = static_cast<int>(tile % tiles_c) * kTT;
  bf16x8 gv[2], uv[2], dv[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int s = threadIdx.x + 256 * k, row = s >> 3, vec = s & 7;
    const int64_t r = r0 + row;
    gv[k] = *reinterpret_cast<const bf16x8*>(g + r * in_stride + c0 + 8 * vec);
    uv[k] = *reinterpret_cast<const bf16x8*>(u + r * in_stride + c0 + 8 * vec);
    dv[k] = *reinterpret_cast<const bf16x8*>(dout + r * static_cast<int64_t>(F) + c0 + 8 * vec);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int s = threadIdx.x + 256 * k, row = s >> 3, vec = s & 7;
    const int64_t r = r0 + row;
    bf16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = bf2f(gv[k][j]), y = bf2f(uv[k][j]), d = bf2f(dv[k][j]);
      const float sgm = sigmoidf_(x);
      const float silu = x * sgm;  // same operation order as swiglu_bwd_kernel: bit-identical gradients
      og[j] = f2bf(d * y * sgm * (1.f + x * (1.f - sgm)));
      ou[j] = f2bf(d * silu);
      sg[(8 * vec + j) * kPitch + row] = og[j];
      su[(8 * vec + j) * kPitch + row] = ou[j];
    }
    *reinterpret_cast<bf16x8*>(dg + r * grad_stride + c0 + 8 * vec) = og;
    *reinterpret_cast<bf16x8*>(du + r * grad_stride + c0 + 8 * vec) = ou;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int s = threadIdx.x + 256 * k, c = s >> 3, rv = s & 7;
    const bf16x8 tg = *reinterpret_cast<const bf16x8*>(&sg[c * kPitch + 8 * rv]);
    const bf16x8 tu = *reinterpret_cast<const bf16x8*>(&su[c * kPitch + 8 * rv]);
    *reinterpret_cast<bf16x8*>(dguT + static_cast<int64_t>(c0 + c) * T + r0 + 8 * rv) = tg;
    *reinterpret_cast<bf16x8*>(dguT + static_cast<int64_t>(F + c0 + c) * T + r0 + 8 * rv) = tu;
  }
}

inline int grid_for(int64_t rows) {
  // 256 CUs x 8 workgroups of 256 threads saturate HBM; rows beyond that
  // are grid-strided.
  return static_cast<int>(rows < 2048 ? (rows < 1 ? 1 : rows) : 2048);
}

}  // namespace

KGWE_API int kgwe_swiglu_fwd(const void* g, const void* u, int64_t in_stride,
                             void* out, int64_t T, int F, hipStream_t s) {
  if (F % 8 || in_stride % 8) return -1;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(T)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(g), static_cast<const bf16_t*>(u),
                     in_stride, static_cast<bf16_t*>(out), T, F);
  return KGWE_CHECK_LAUNCH();
}

KGWE_API int kgwe_swiglu_bwd(const void* g, const void* u, int64_t in_stride,
                             const void* dout, void* dg, void* du,
                             int64_t grad_stride, int64_t T, int F, hipStream_t s) {
  if (F % 8 || in_stride % 8 || grad_stride % 8) return -1;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(T)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(g), static_cast<const bf16_t*>(u),
                     in_stride, static_cast<const bf16_t*>(dout),
                     static_cast<bf16_t*>(dg), static_cast<bf16_t*>(du), grad_stride,
                     T, F);
  return KGWE_CHECK_LAUNCH();
}

// As kgwe_swiglu_bwd, and also dguT [2F, T] = the transposed [T, 2F] gradient
// (rows [0, F) = dg^T, rows [F, 2F) = du^T).  T % 64 == 0 and F % 64 == 0.
KGWE_API int kgwe_swiglu_bwd_t(const void* g, const void* u, int64_t in_stride, const void* dout, void* dg,
                               void* du, int64_t grad_stride, void* dguT, int64_t T, int F, hipStream_t s) {
  if (T <= 0 || F <= 0 || T % kTT || F % kTT || in_stride % 8 || grad_stride % 8) return -1;
  const int64_t tiles = (T / kTT) * (F / kTT);
  if (tiles > 0x7fffffffLL) return -1;
  hipLaunchKernelGGL(swiglu_bwd_t_kernel, dim3(static_cast<unsigned>(tiles)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(g), static_cast<const bf16_t*>(u), in_stride,
                     static_cast<const bf16_t*>(dout), static_cast<bf16_t*>(dg), static_cast<bf16_t*>(du),
                     grad_stride, static_cast<bf16_t*>(dguT), T, F);
  return KGWE_CHECK_LAUNCH();
}
