// Fused QKV split + rotary position embedding (RoPE) for Llama attention.
//
// Input: the fused projection output qkv [T, (Hq + 2*Hkv) * D] (T = B*S rows).
// Forward writes q [T, Hq, D] and k [T, Hkv, D] rotated, and v [T, Hkv, D]
// copied, all contiguous — one HBM pass replaces split + 2 rotary kernels +
// contiguous copies.  Backward does the inverse rotation of dq / dk and
// scatters dq, dk, dv back into one dqkv [T, (Hq + 2*Hkv) * D] buffer that the
// QKV projection backward consumes directly.
//
// Rotation is the "rotate_half" convention: for i < D/2,
//   out[i]       = x[i] * cos[p, i] - x[i + D/2] * sin[p, i]
//   out[i + D/2] = x[i + D/2] * cos[p, i] + x[i] * sin[p, i]
// with p = row % S and fp32 cos/sin tables [S, D/2] built once on the host
// (cdna_hip_programming.md App. B: precompute trig tables, never sinf/cosf
// per element).
#include "common.h"

using namespace kgwe;

namespace {

// One thread = one 8-wide chunk of the first half of one head plus the
// matching chunk of the second half.  Heads [0, Hq) are q, [Hq, Hq+Hkv) k,
// [Hq+Hkv, Hq+2Hkv) v (copy only).
template <bool kBackward>
__global__ __launch_bounds__(256) void rope_kernel(
    const bf16_t* __restrict__ src_qkv,  // fwd: qkv input
    const bf16_t* __restrict__ src_q, const bf16_t* __restrict__ src_k,
    const bf16_t* __restrict__ src_v,  // bwd: dq, dk, dv inputs
    bf16_t* __restrict__ dst_q, bf16_t* __restrict__ dst_k,
    bf16_t* __restrict__ dst_v,    // fwd outputs
    bf16_t* __restrict__ dst_qkv,  // bwd output
    const float* __restrict__ cosT, const float* __restrict__ sinT, int64_t T,
    int S, int Hq, int Hkv, int D) {
  const int half = D / 2;
  const int cpp = half / 8;  // chunks per half-head
  const int Ht = Hq + 2 * Hkv;
  const int64_t n = T * Ht * cpp;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL) {
    const int64_t row = i / (static_cast<int64_t>(Ht) * cpp);
    const int rem = static_cast<int>(i - row * Ht * cpp);
    const int head = rem / cpp;
    const int c = (rem - head * cpp) * 8;
    const int pos = static_cast<int>(row % S);
    const int64_t qkv_off = row * static_cast<int64_t>(Ht) * D + static_cast<int64_t>(head) * D;
    // Where this head lives in the split (q/k/v) tensors.
    const bf16_t* sp;
    bf16_t* dp;
    int64_t split_off;
    bool rotate = true;
    if (head < Hq) {
      split_off = (row * Hq + head) * static_cast<int64_t>(D);
      sp = kBackward ? src_q : nullptr;
      dp = kBackward ? nullptr : dst_q;
    } else if (head < Hq + Hkv) {
      split_off = (row * Hkv + (head - Hq)) * static_cast<int64_t>(D);
      sp = kBackward ? src_k : nullptr;
      dp = kBackward ? nullptr : dst_k;
    } else {
      split_off = (row * Hkv + (head - Hq - Hkv)) * static_cast<int64_t>(D);
      sp = kBackward ? src_v : nullptr;
      dp = kBackward ? nullptr : dst_v;
      rotate = false;
    }
    const bf16_t* in = kBackward ? sp + split_off : src_qkv + qkv_off;
    bf16_t* out = kBackward ? dst_qkv + qkv_off : dp + split_off;
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(in + c);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(in + half + c);
    if (!rotate) {
      *reinterpret_cast<bf16x8*>(out + c) = a;
      *reinterpret_cast<bf16x8*>(out + half + c) = b;
      continue;
    }
    const f32x4* cp = reinterpret_cast<const f32x4*>(cosT + static_cast<int64_t>(pos) * half + c);
    const f32x4* sn = reinterpret_cast<const f32x4*>(sinT + static_cast<int64_t>(pos) * half + c);
    const f32x4 c0 = cp[0], c1 = cp[1], s0 = sn[0], s1 = sn[1];
    bf16x8 oa, ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cs = j < 4 ? c0[j & 3] : c1[j & 3];
      const float sn_ = j < 4 ? s0[j & 3] : s1[j & 3];
      const float x1 = bf2f(a[j]), x2 = bf2f(b[j]);
      if (kBackward) {  // transpose of the rotation
        oa[j] = f2bf(x1 * cs + x2 * sn_);
        ob[j] = f2bf(x2 * cs - x1 * sn_);
      } else {
        oa[j] = f2bf(x1 * cs - x2 * sn_);
        ob[j] = f2bf(x2 * cs + x1 * sn_);
      }
    }
    *reinterpret_cast<bf16x8*>(out + c) = oa;
    *reinterpret_cast<bf16x8*>(out + half + c) = ob;
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  return static_cast<int>(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

}  // namespace

KGWE_API int kgwe_rope_qkv_fwd(const void* qkv, void* q, void* k, void* v,
                               const float* cosT, const float* sinT, int64_t T,
                               int S, int Hq, int Hkv, int D, hipStream_t s) {
  if (D % 16) return -1;
  const int64_t n = T * (Hq + 2 * Hkv) * (D / 16);
  hipLaunchKernelGGL(rope_kernel<false>, dim3(grid_for(n)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(qkv), nullptr, nullptr, nullptr,
                     static_cast<bf16_t*>(q), static_cast<bf16_t*>(k),
                     static_cast<bf16_t*>(v), nullptr, cosT, sinT, T, S, Hq, Hkv, D);
  return KGWE_CHECK_LAUNCH();
}

KGWE_API int kgwe_rope_qkv_bwd(const void* dq, const void* dk, const void* dv,
                               void* dqkv, const float* cosT, const float* sinT,
                               int64_t T, int S, int Hq, int Hkv, int D,
                               hipStream_t s) {
  if (D % 16) return -1;
  const int64_t n = T * (Hq + 2 * Hkv) * (D / 16);
  hipLaunchKernelGGL(rope_kernel<true>, dim3(grid_for(n)), dim3(256), 0, s, nullptr,
                     static_cast<const bf16_t*>(dq), static_cast<const bf16_t*>(dk),
                     static_cast<const bf16_t*>(dv), nullptr, nullptr, nullptr,
                     static_cast<bf16_t*>(dqkv), cosT, sinT, T, S, Hq, Hkv, D);
  return KGWE_CHECK_LAUNCH();
}
