// Multi-tensor fused AdamW for fp32 master parameters.
//
// Each launch updates up to 16 parameters (or optimizer-state shards) whose
// pointers travel in the kernel arguments, so a launch needs no device-side
// table and can be issued per gradient bucket from a backward hook (the
// optimizer step then overlaps the rest of backward on a side stream — see
// kgwe/parallel/zero.py).  Each lane streams 4 elements (16 B fp32 of p, m, v;
// 16 B fp32 or 8 B bf16 of g) and writes back p, m, v plus an optional bf16
// copy of p — the live bf16 model weight the next forward reads.  That copy is
// what removes the separate cast/all-gather-copy pass of a master-weight
// scheme, and reading bf16 gradients straight from autograd's output removes
// the fp32 up-cast pass.  HBM-bound (26-30 B/param), so the only goals are
// full-width coalesced access and few launches.
//
//   m = b1 m + (1-b1) g ;  v = b2 v + (1-b2) g^2
//   p = p - lr * (m / bc1 / (sqrt(v / bc2) + eps) + wd * p)
#include "common.h"

using namespace kgwe;

struct AdamTensor {
  float* p;
  const void* g;   // fp32 or bf16 (g_bf16)
  float* m;
  float* v;
  bf16_t* shadow;  // optional bf16 copy of p (nullptr = none)
  int64_t n;
  int32_t g_bf16;
  int32_t pad;
};

constexpr int kChunk = 256 * 4 * 16;  // elements per workgroup task (64 KiB fp32)

namespace {

struct AdamArgs {
  float lr, b1, b2, eps, wd, bc1, bc2_sqrt_inv, grad_scale;
};

__device__ __forceinline__ float adam_one(float& p, float& m, float& v, float g, const AdamArgs& a) {
  const float gj = g * a.grad_scale;
  m = a.b1 * m + (1.f - a.b1) * gj;
  v = a.b2 * v + (1.f - a.b2) * gj * gj;
  const float denom = sqrtf(v) * a.bc2_sqrt_inv + a.eps;
  p -= a.lr * (m / a.bc1 / denom + a.wd * p);
  return p;
}

template <bool GB>
__device__ __forceinline__ void adam_range(const AdamTensor& t, int64_t start, int64_t end,
                                           const AdamArgs& a) {
  const float* gf = static_cast<const float*>(t.g);
  const bf16_t* gb = static_cast<const bf16_t*>(t.g);
  for (int64_t i = start + threadIdx.x * 4; i < end; i += 256 * 4) {
    const bool aligned =
        ((reinterpret_cast<uintptr_t>(t.p + i) | reinterpret_cast<uintptr_t>(t.m + i) |
          reinterpret_cast<uintptr_t>(t.v + i)) & 15) == 0 &&
        (GB ? (reinterpret_cast<uintptr_t>(gb + i) & 7) == 0
            : (reinterpret_cast<uintptr_t>(gf + i) & 15) == 0) &&
        (t.shadow == nullptr || (reinterpret_cast<uintptr_t>(t.shadow + i) & 7) == 0);
    if (i + 4 <= end && aligned) {
      f32x4 p = *reinterpret_cast<const f32x4*>(t.p + i);
      f32x4 m = *reinterpret_cast<const f32x4*>(t.m + i);
      f32x4 v = *reinterpret_cast<const f32x4*>(t.v + i);
      float g[4];
      if constexpr (GB) {
        const uint2 raw = *reinterpret_cast<const uint2*>(gb + i);
        g[0] = __uint_as_float(raw.x << 16);
        g[1] = __uint_as_float(raw.x & 0xffff0000u);
        g[2] = __uint_as_float(raw.y << 16);
        g[3] = __uint_as_float(raw.y & 0xffff0000u);
      } else {
        const f32x4 gv = *reinterpret_cast<const f32x4*>(gf + i);
        g[0] = gv[0]; g[1] = gv[1]; g[2] = gv[2]; g[3] = gv[3];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adam_one(pj, mj, vj, g[j], a);
        p[j] = pj; m[j] = mj; v[j] = vj;
      }
      *reinterpret_cast<f32x4*>(t.p + i) = p;
      *reinterpret_cast<f32x4*>(t.m + i) = m;
      *reinterpret_cast<f32x4*>(t.v + i) = v;
      if (t.shadow) {
        uint2 o;
        o.x = static_cast<unsigned>(f2bf(p[0])) | (static_cast<unsigned>(f2bf(p[1])) << 16);
        o.y = static_cast<unsigned>(f2bf(p[2])) | (static_cast<unsigned>(f2bf(p[3])) << 16);
        *reinterpret_cast<uint2*>(t.shadow + i) = o;
      }
    } else {
      for (int64_t k = i; k < end && k < i + 4; ++k) {
        float pk = t.p[k], mk = t.m[k], vk = t.v[k];
        adam_one(pk, mk, vk, GB ? bf2f(gb[k]) : gf[k], a);
        t.p[k] = pk; t.m[k] = mk; t.v[k] = vk;
        if (t.shadow) t.shadow[k] = f2bf(pk);
      }
    }
  }
}

// Up to kBatch tensors per launch, passed BY VALUE in the kernel arguments
// (~0.9 KB of the 4 KB argument space): no device-side pointer/chunk tables,
// no H2D copy, nothing to cache when autograd hands out fresh gradient
// buffers every step.  Workgroup task ci belongs to the first tensor whose
// cumulative chunk count exceeds ci (linear scan over <= 16 entries).
constexpr int kBatch = 16;

struct AdamBatch {
  AdamTensor t[kBatch];
  int64_t chunk_end[kBatch];  // inclusive prefix sum of per-tensor chunk counts
  int n;
  int pad;
};

__global__ __launch_bounds__(256) void adamw_kernel(const AdamBatch b, AdamArgs a) {
  const int64_t total = b.chunk_end[b.n - 1];
  for (int64_t ci = blockIdx.x; ci < total; ci += gridDim.x) {
    int i = 0;
    while (ci >= b.chunk_end[i]) ++i;
    const int64_t first = i ? b.chunk_end[i - 1] : 0;
    const AdamTensor& t = b.t[i];
    const int64_t start = (ci - first) * kChunk;
    const int64_t end = (start + kChunk < t.n) ? start + kChunk : t.n;
    if (t.g_bf16) adam_range<true>(t, start, end, a);
    else adam_range<false>(t, start, end, a);
  }
}

}  // namespace

KGWE_API int kgwe_adamw_chunk_elems() { return kChunk; }
KGWE_API int kgwe_adamw_tensor_bytes() { return sizeof(AdamTensor); }

// `tensors`: HOST array of n AdamTensor records (device pointers inside).
// `step` is the 1-based step count after increment (bias corrections are
// computed here; no device sync).  Launches ceil(n / 16) kernels on `s`.
// `max_grid` caps the workgroups of a launch (<= 0: 4096, enough to run at
// the HBM limit).  A small cap makes the update a BACKGROUND kernel: issued
// on a side stream beside the backward GEMMs, 4096 workgroups of a
// memory-bound kernel co-reside on every CU and slow the GEMM next to them
// ~2x (tools/gemm_instep.py); a few hundred grid-striding workgroups take
// longer but leave most CUs to the GEMM.
KGWE_API int kgwe_adamw_step(const void* tensors, int n, float lr, float b1, float b2, float eps,
                             float wd, int step, float grad_scale, int max_grid, hipStream_t s) {
  const int cap = max_grid > 0 ? max_grid : 4096;
  if (n <= 0) return 0;
  AdamArgs a;
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd;
  a.bc1 = 1.f - powf(b1, static_cast<float>(step));
  a.bc2_sqrt_inv = 1.f / sqrtf(1.f - powf(b2, static_cast<float>(step)));
  a.grad_scale = grad_scale;
  const AdamTensor* ts = static_cast<const AdamTensor*>(tensors);
  for (int base = 0; base < n; base += kBatch) {
    AdamBatch b = {};
    int64_t acc = 0;
    for (int j = 0; j < kBatch && base + j < n; ++j) {
      const AdamTensor& t = ts[base + j];
      if (t.n <= 0 || t.p == nullptr || t.m == nullptr || t.v == nullptr || t.g == nullptr) return -1;
      b.t[b.n] = t;
      acc += (t.n + kChunk - 1) / kChunk;
      b.chunk_end[b.n] = acc;
      ++b.n;
    }
    const int grid = acc < cap ? static_cast<int>(acc) : cap;
    hipLaunchKernelGGL(adamw_kernel, dim3(grid), dim3(256), 0, s, b, a);
    const int rc = KGWE_CHECK_LAUNCH();
    if (rc) return rc;
  }
  return 0;
}
