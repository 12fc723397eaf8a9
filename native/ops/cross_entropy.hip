// Fused softmax cross-entropy over a large vocabulary (Llama-3: V = 128256).
//
// Forward: one 256-thread workgroup per row streams the bf16 logits once
// (16 B per lane), keeps an online (max, sum-exp) pair per lane, reduces
// across the workgroup and writes loss[row] = lse - x[label] and lse[row].
// No fp32 copy of the [T, V] logits is ever materialised (PyTorch's path
// upcasts to fp32: 2x the logits bytes, twice).
// Backward: dlogits = (exp(x - lse) - onehot(label)) * (*grad_scale) with the
// mean-reduction scale read from device memory (no host sync); rows whose
// label == ignore_index get zero gradient and zero loss.
#include "common.h"

using namespace kgwe;

namespace {

__device__ __forceinline__ void merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
  m = mn;
}

__global__ __launch_bounds__(256) void ce_fwd_kernel(
    const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
    float* __restrict__ loss, float* __restrict__ lse_out, int64_t V,
    int64_t ignore_index) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  const bf16_t* x = logits + row * V;
  float m = -INFINITY, s = 0.f;
  const int64_t nv = V / 8;
  for (int64_t i = threadIdx.x; i < nv; i += 256) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    float lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) lm = fmaxf(lm, bf2f(v[j]));
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(bf2f(v[j]) - lm);
    merge(m, s, lm, ls);
  }
  for (int64_t i = nv * 8 + threadIdx.x; i < V; i += 256) merge(m, s, bf2f(x[i]), 1.f);
  // wave reduce
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(m, off, kWave), s2 = __shfl_xor(s, off, kWave);
    merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int w = 1; w < 4; ++w) merge(M, Ssum, sm[w], ss[w]);
    const float lse = M + __logf(Ssum);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    loss[row] = (lab == ignore_index || lab < 0 || lab >= V) ? 0.f : lse - bf2f(x[lab]);
  }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(
    const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
    const float* __restrict__ lse_in, const float* __restrict__ grad_scale,
    bf16_t* __restrict__ dlogits, int64_t V, int64_t ignore_index) {
  const int64_t row = blockIdx.x;
  const int64_t lab = labels[row];
  const bool ignored = (lab == ignore_index || lab < 0 || lab >= V);
  const float g = ignored ? 0.f : *grad_scale;
  const float lse = lse_in[row];
  const bf16_t* x = logits + row * V;
  bf16_t* dx = dlogits + row * V;
  const int64_t nv = V / 8;
  for (int64_t i = threadIdx.x; i < nv; i += 256) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(bf2f(v[j]) - lse);
      if (i * 8 + j == lab) p -= 1.f;
      o[j] = f2bf(p * g);
    }
    *reinterpret_cast<bf16x8*>(dx + i * 8) = o;
  }
  for (int64_t i = nv * 8 + threadIdx.x; i < V; i += 256) {
    float p = __expf(bf2f(x[i]) - lse);
    if (i == lab) p -= 1.f;
    dx[i] = f2bf(p * g);
  }
}

}  // namespace

KGWE_API int kgwe_cross_entropy_fwd(const void* logits, const int64_t* labels,
                                    float* loss, float* lse, int64_t T, int64_t V,
                                    int64_t ignore_index, hipStream_t s) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(static_cast<unsigned>(T)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(logits), labels, loss, lse, V,
                     ignore_index);
  return KGWE_CHECK_LAUNCH();
}

// dlogits may alias logits (in-place) — each element is read before written
// by the same thread.
KGWE_API int kgwe_cross_entropy_bwd(const void* logits, const int64_t* labels,
                                    const float* lse, const float* grad_scale,
                                    void* dlogits, int64_t T, int64_t V,
                                    int64_t ignore_index, hipStream_t s) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(static_cast<unsigned>(T)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(logits), labels, lse, grad_scale,
                     static_cast<bf16_t*>(dlogits), V, ignore_index);
  return KGWE_CHECK_LAUNCH();
}
