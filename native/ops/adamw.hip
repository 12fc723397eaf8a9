// Multi-tensor fused AdamW for fp32 master parameters (FSDP shards).
//
// One launch updates every parameter shard: the host builds a chunk table
// (tensor index, element offset) once, the per-tensor pointer table is a
// small device array refreshed when gradient storage moves.  Each lane
// streams 4 fp32 (16 B) of p, g, m, v per step and writes back p, m, v (and
// optionally a bf16 shadow copy of p), i.e. 28 B/param — HBM-bound, so the
// only goal is full-width coalesced access and a single launch.
//
//   m = b1 m + (1-b1) g ;  v = b2 v + (1-b2) g^2
//   p = p - lr * (m / bc1 / (sqrt(v / bc2) + eps) + wd * p)
#include "common.h"

using namespace kgwe;

struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  bf16_t* shadow;  // optional bf16 copy of p (nullptr = none)
  int64_t n;
};

struct AdamChunk {
  int tensor;
  int pad;
  int64_t start;
};

constexpr int kChunk = 256 * 4 * 16;  // elements per workgroup task (64 KiB fp32)

namespace {

__global__ __launch_bounds__(256) void adamw_kernel(
    const AdamTensor* __restrict__ tensors, const AdamChunk* __restrict__ chunks,
    int nchunks, float lr, float b1, float b2, float eps, float wd, float bc1,
    float bc2_sqrt_inv, float grad_scale) {
  for (int ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const AdamChunk ch = chunks[ci];
    const AdamTensor t = tensors[ch.tensor];
    const int64_t end = (ch.start + kChunk < t.n) ? ch.start + kChunk : t.n;
    for (int64_t i = ch.start + threadIdx.x * 4; i < end; i += 256 * 4) {
      if (i + 4 <= end && ((reinterpret_cast<uintptr_t>(t.p + i) & 15) == 0) &&
          ((reinterpret_cast<uintptr_t>(t.g + i) & 15) == 0)) {
        f32x4 p = *reinterpret_cast<const f32x4*>(t.p + i);
        const f32x4 g = *reinterpret_cast<const f32x4*>(t.g + i);
        f32x4 m = *reinterpret_cast<const f32x4*>(t.m + i);
        f32x4 v = *reinterpret_cast<const f32x4*>(t.v + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gj = g[j] * grad_scale;
          m[j] = b1 * m[j] + (1.f - b1) * gj;
          v[j] = b2 * v[j] + (1.f - b2) * gj * gj;
          const float denom = sqrtf(v[j]) * bc2_sqrt_inv + eps;
          p[j] -= lr * (m[j] / bc1 / denom + wd * p[j]);
        }
        *reinterpret_cast<f32x4*>(t.p + i) = p;
        *reinterpret_cast<f32x4*>(t.m + i) = m;
        *reinterpret_cast<f32x4*>(t.v + i) = v;
        if (t.shadow) {
#pragma unroll
          for (int j = 0; j < 4; ++j) t.shadow[i + j] = f2bf(p[j]);
        }
      } else {
        for (int64_t k = i; k < end && k < i + 4; ++k) {
          const float gj = t.g[k] * grad_scale;
          const float mk = b1 * t.m[k] + (1.f - b1) * gj;
          const float vk = b2 * t.v[k] + (1.f - b2) * gj * gj;
          t.m[k] = mk;
          t.v[k] = vk;
          const float pk = t.p[k] - lr * (mk / bc1 / (sqrtf(vk) * bc2_sqrt_inv + eps) + wd * t.p[k]);
          t.p[k] = pk;
          if (t.shadow) t.shadow[k] = f2bf(pk);
        }
      }
    }
  }
}

}  // namespace

KGWE_API int kgwe_adamw_chunk_elems() { return kChunk; }
KGWE_API int kgwe_adamw_tensor_bytes() { return sizeof(AdamTensor); }
KGWE_API int kgwe_adamw_chunk_bytes() { return sizeof(AdamChunk); }

// `step` is the 1-based step count after increment (bias corrections are
// computed here on the host side of the launch; no device sync).
KGWE_API int kgwe_adamw_step(const void* tensors, const void* chunks, int nchunks,
                             float lr, float b1, float b2, float eps, float wd,
                             int step, float grad_scale, hipStream_t s) {
  if (nchunks <= 0) return 0;
  const float bc1 = 1.f - powf(b1, static_cast<float>(step));
  const float bc2 = 1.f - powf(b2, static_cast<float>(step));
  const int grid = nchunks < 4096 ? nchunks : 4096;
  hipLaunchKernelGGL(adamw_kernel, dim3(grid), dim3(256), 0, s,
                     static_cast<const AdamTensor*>(tensors),
                     static_cast<const AdamChunk*>(chunks), nchunks, lr, b1, b2, eps,
                     wd, bc1, 1.f / sqrtf(bc2), grad_scale);
  return KGWE_CHECK_LAUNCH();
}
