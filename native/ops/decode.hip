// Decode-time (one new token per sequence) kernels for the bf16 inference
// harness: fused RoPE + KV-cache append, and split-K GQA attention over the
// cache ("flash decoding"), written for 64-lane CDNA4 wavefronts.
//
// Layouts
//   qkv     [B, (Hq + 2*Hkv) * D]  fused projection output of the new token
//   pos     [B] int32              position of the new token (= tokens cached)
//   k/v cache [B, Hkv, Smax, D]    bf16, head-major so one (b, kv-head) is a
//                                  contiguous [Smax, D] slab
//   q       [B, Hq, D]; out [B, Hq, D]
//
// Decode attention is HBM-bound (every cached K/V byte is read once per
// step) and has little parallelism per sequence, so the key range of each
// (sequence, kv-head) is split into `splits` chunks that run as separate
// workgroups; the LAST of them to finish merges the partial softmax states
// in the same launch (write-through partials + one relaxed agent-scope
// ticket per (sequence, kv-head): no fence, no spin, no second kernel).  One
// workgroup serves ALL G = Hq/Hkv query heads of its kv-head (one wave per
// query head), so each K/V tile is read from HBM once and reused G times
// from LDS.  The split count depends only on the cache capacity, so a
// decode step can be captured once in a hipGraph and replayed at any length.
#include <algorithm>

#include "common.h"

using namespace kgwe;

namespace {

constexpr float kLog2e = 1.4426950408889634f;

// ---------------------------------------------------------------------------
// RoPE of q and k for the new token at pos[b] + append of k, v to the cache.
// One thread = one 8-wide chunk of the first half of one head plus the
// matching chunk of the second half ("rotate_half" convention, as rope.hip).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rope_append_kernel(
    const bf16_t* __restrict__ qkv, const int* __restrict__ pos, const float* __restrict__ cosT,
    const float* __restrict__ sinT, bf16_t* __restrict__ q_out, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, int B, int Hq, int Hkv, int D, int Smax) {
  const int half = D / 2;
  const int cpp = half / 8;
  const int Ht = Hq + 2 * Hkv;
  const int64_t n = static_cast<int64_t>(B) * Ht * cpp;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL) {
    const int b = static_cast<int>(i / (static_cast<int64_t>(Ht) * cpp));
    const int rem = static_cast<int>(i - static_cast<int64_t>(b) * Ht * cpp);
    const int head = rem / cpp;
    const int c = (rem - head * cpp) * 8;
    const int p = pos[b];
    if (p < 0 || p >= Smax) continue;  // never write outside the cache
    const bf16_t* in = qkv + static_cast<int64_t>(b) * Ht * D + static_cast<int64_t>(head) * D;
    bf16_t* out;
    bool rotate = true;
    if (head < Hq) {
      out = q_out + (static_cast<int64_t>(b) * Hq + head) * D;
    } else if (head < Hq + Hkv) {
      out = kc + ((static_cast<int64_t>(b) * Hkv + (head - Hq)) * Smax + p) * D;
    } else {
      out = vc + ((static_cast<int64_t>(b) * Hkv + (head - Hq - Hkv)) * Smax + p) * D;
      rotate = false;
    }
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(in + c);
    const bf16x8 bb = *reinterpret_cast<const bf16x8*>(in + half + c);
    if (!rotate) {
      *reinterpret_cast<bf16x8*>(out + c) = a;
      *reinterpret_cast<bf16x8*>(out + half + c) = bb;
      continue;
    }
    const f32x4* cp = reinterpret_cast<const f32x4*>(cosT + static_cast<int64_t>(p) * half + c);
    const f32x4* sp = reinterpret_cast<const f32x4*>(sinT + static_cast<int64_t>(p) * half + c);
    const f32x4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
    bf16x8 oa, ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cs = j < 4 ? c0[j & 3] : c1[j & 3];
      const float sn = j < 4 ? s0[j & 3] : s1[j & 3];
      const float x0 = bf2f(a[j]), x1 = bf2f(bb[j]);
      oa[j] = f2bf(x0 * cs - x1 * sn);
      ob[j] = f2bf(x1 * cs + x0 * sn);
    }
    *reinterpret_cast<bf16x8*>(out + c) = oa;
    *reinterpret_cast<bf16x8*>(out + half + c) = ob;
  }
}

// ---------------------------------------------------------------------------
// Split-K decode attention.  grid = (splits, Hkv, B), block = 64 * G: wave g
// owns query head kvh * G + g.  Per 64-key tile: the whole workgroup stages
// K and V in LDS (16 B vector loads, rows padded by 8 bf16 against bank
// conflicts); lane j of every wave scores key j against its head (q read
// from LDS as a broadcast); online softmax in the exp2 domain (q pre-scaled
// by softmax_scale * log2 e); then lane d accumulates sum_j p_j V[j][d].
// ---------------------------------------------------------------------------
//
// ROPE: q is the fused projection output qkv [B, (Hq + 2 Hkv) * D] of the new
// token at position p = lens[b] - 1, and this kernel also does the work of
// rope_append_kernel: RoPE of the G query heads in the prologue, and in the
// one split whose key range holds p, RoPE of the new key + the cache append
// of k and v (the staging thread of each chunk of row p computes it, stores
// it to the cache and to LDS), with the same roundings.  One launch less per
// layer.
template <int D, int G, bool ROPE>
__global__ __launch_bounds__(64 * G) void decode_attn_kernel(
    const bf16_t* __restrict__ q, bf16_t* kc, bf16_t* vc, const float* __restrict__ cosT,
    const float* __restrict__ sinT, const int* __restrict__ lens, float* part_o, float* part_ml,
    unsigned* tickets, bf16_t* __restrict__ out, int Hkv, int Smax, int splits, int chunk, float qscale) {
  constexpr int kPad = D + 8;
  constexpr int kPer = D / 64;  // output elements per lane
  __shared__ __attribute__((aligned(16))) float qs[G][D];
  __shared__ __attribute__((aligned(16))) bf16_t ks[64][kPad];
  __shared__ __attribute__((aligned(16))) bf16_t vs[64][kPad];
  __shared__ float ps[G][64];
  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int Hq = Hkv * G;
  const int h = kvh * G + wave;
  const int len = min(lens[b], Smax);
  const int start = split * chunk;
  const int end = min(len, start + chunk);
  constexpr int half = D / 2;
  const int Ht = Hq + 2 * Hkv;
  const int p = min(max(lens[b] - 1, 0), Smax - 1);  // ROPE: the new token's position
  if (ROPE) {
    const bf16_t* qrow = q + (static_cast<int64_t>(b) * Ht + h) * D;
#pragma unroll
    for (int t = 0; t < kPer; ++t) {
      const int i = lane + 64 * t, j = i < half ? i : i - half;
      const float x = bf2f(qrow[i]), y = bf2f(qrow[i < half ? i + half : i - half]);
      const float cs = cosT[static_cast<int64_t>(p) * half + j], sn = sinT[static_cast<int64_t>(p) * half + j];
      qs[wave][i] = bf2f(f2bf(i < half ? x * cs - y * sn : x * cs + y * sn)) * qscale;  // as rope_append_kernel
    }
  } else {
    const bf16_t* qrow = q + (static_cast<int64_t>(b) * Hq + h) * D;
#pragma unroll
    for (int t = 0; t < kPer; ++t) qs[wave][lane + 64 * t] = bf2f(qrow[lane + 64 * t]) * qscale;
  }
  const int64_t slab = (static_cast<int64_t>(b) * Hkv + kvh) * Smax * D;
  bf16_t* kbase = kc + slab;
  bf16_t* vbase = vc + slab;
  float m = -INFINITY, l = 0.0f;
  float acc[kPer];
#pragma unroll
  for (int t = 0; t < kPer; ++t) acc[t] = 0.0f;
  // K / V tiles of 64 keys go HBM -> registers -> LDS, and the loads of tile t + 1 are issued
  // before the math of tile t: with the loads inside the tile loop every tile exposed a full
  // memory round trip (a split of 256 keys is four of them).
  constexpr int kChunks = 64 * D / 8;
  constexpr int NCH = kChunks / (64 * G);  // 16-B chunks per thread per matrix and tile
  static_assert(kChunks % (64 * G) == 0, "tile chunks divide evenly over the workgroup");
  bf16x8 kr[NCH], vr[NCH];
  auto load_tile = [&](int t0) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = threadIdx.x + i * 64 * G;
      const int r = idx / (D / 8), c = (idx % (D / 8)) * 8;
      const int key = t0 + r;
      bf16x8 kv = {0, 0, 0, 0, 0, 0, 0, 0}, vv = {0, 0, 0, 0, 0, 0, 0, 0};
      if (ROPE && key == p && key < end) {
        // the new token: RoPE of k (a chunk lies in one half), v as is; append both
        const bf16_t* kin = q + (static_cast<int64_t>(b) * Ht + Hq + kvh) * D;
        const bf16_t* vin = q + (static_cast<int64_t>(b) * Ht + Hq + Hkv + kvh) * D;
        const int cj = c < half ? c : c - half;
        const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(kin + cj);
        const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(kin + cj + half);
        const float* cp = cosT + static_cast<int64_t>(p) * half + cj;
        const float* sp = sinT + static_cast<int64_t>(p) * half + cj;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = bf2f(x0[j]), bb = bf2f(x1[j]);
          kv[j] = f2bf(c < half ? a * cp[j] - bb * sp[j] : bb * cp[j] + a * sp[j]);
        }
        vv = *reinterpret_cast<const bf16x8*>(vin + c);
        *reinterpret_cast<bf16x8*>(kbase + static_cast<int64_t>(key) * D + c) = kv;
        *reinterpret_cast<bf16x8*>(vbase + static_cast<int64_t>(key) * D + c) = vv;
      } else if (key < end) {
        kv = *reinterpret_cast<const bf16x8*>(kbase + static_cast<int64_t>(key) * D + c);
        vv = *reinterpret_cast<const bf16x8*>(vbase + static_cast<int64_t>(key) * D + c);
      }
      kr[i] = kv;
      vr[i] = vv;
    }
  };
  if (start < end) load_tile(start);
  for (int t0 = start; t0 < end; t0 += 64) {
    __syncthreads();  // qs written / previous tile consumed
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = threadIdx.x + i * 64 * G;
      const int r = idx / (D / 8), c = (idx % (D / 8)) * 8;
      *reinterpret_cast<bf16x8*>(&ks[r][c]) = kr[i];
      *reinterpret_cast<bf16x8*>(&vs[r][c]) = vr[i];
    }
    __syncthreads();
    if (t0 + 64 < end) load_tile(t0 + 64);  // lands during this tile's math
    const int key = t0 + lane;
    float s = -INFINITY;
    if (key < end) {
      float d0 = 0.0f, d1 = 0.0f;
#pragma unroll
      for (int c = 0; c < D; c += 8) {
        const bf16x8 kv = *reinterpret_cast<const bf16x8*>(&ks[lane][c]);
        const f32x4 qa = *reinterpret_cast<const f32x4*>(&qs[wave][c]);
        const f32x4 qb = *reinterpret_cast<const f32x4*>(&qs[wave][c + 4]);
        d0 += qa[0] * bf2f(kv[0]) + qa[1] * bf2f(kv[1]) + qa[2] * bf2f(kv[2]) + qa[3] * bf2f(kv[3]);
        d1 += qb[0] * bf2f(kv[4]) + qb[1] * bf2f(kv[5]) + qb[2] * bf2f(kv[6]) + qb[3] * bf2f(kv[7]);
      }
      s = d0 + d1;
    }
    const float m_new = fmaxf(m, wave_max(s));  // finite: the tile has >= 1 valid key
    const float p = key < end ? exp2f(s - m_new) : 0.0f;
    const float alpha = exp2f(m - m_new);
    l = l * alpha + wave_sum(p);
    m = m_new;
    ps[wave][lane] = p;
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kPer; ++t) acc[t] *= alpha;
    const int nkeys = min(64, end - t0);
    for (int j = 0; j < nkeys; ++j) {
      const float pj = ps[wave][j];
#pragma unroll
      for (int t = 0; t < kPer; ++t) acc[t] += pj * bf2f(vs[j][lane + 64 * t]);
    }
  }
  const int64_t bh = static_cast<int64_t>(b) * Hq + h;
  if (splits == 1) {
    const float inv = l > 0.0f ? 1.0f / l : 0.0f;
#pragma unroll
    for (int t = 0; t < kPer; ++t) out[bh * D + lane + 64 * t] = f2bf(acc[t] * inv);
    return;
  }
  // Publish this split's state with write-through (sc1) stores: relaxed
  // agent-scope atomic stores, so another XCD's last arriver reads them
  // from memory without any L2 writeback fence (cdna_hip_programming.md
  // Guideline 16, R1).  A __threadfence() here instead cost 10x the kernel.
  const int64_t row = bh * splits + split;
#pragma unroll
  for (int t = 0; t < kPer; ++t)
    __hip_atomic_store(part_o + row * D + lane + 64 * t, acc[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane == 0) {
    __hip_atomic_store(part_ml + row * 2, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part_ml + row * 2 + 1, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
  __syncthreads();
  __shared__ unsigned last;
  if (threadIdx.x == 0) {
    unsigned* tk = tickets + static_cast<int64_t>(b) * Hkv + kvh;
    const unsigned n = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = n == static_cast<unsigned>(splits - 1);
    // The ticket returns to 0 for the next call: every other split of this
    // (b, kv head) has already added (stream order separates the calls).
    if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  // Last arriver: every split's state of each of the G heads (wave = head),
  // all loads issued together as sc1 loads (relaxed agent-scope atomic
  // loads: they bypass this CU's L1, so no acquire fence is needed — every
  // load of the handed-off bytes is one, Guideline 16); lane sp holds split
  // sp's (m, l).  Measured: 9.2 us for attention + merge, against 5.6 + 6.6
  // for the two launches and 9.8 with an acquire fence and plain loads.
  auto ld_sc1 = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const float ms = lane < splits ? ld_sc1(part_ml + (bh * splits + lane) * 2) : -INFINITY;
  const float ls = lane < splits ? ld_sc1(part_ml + (bh * splits + lane) * 2 + 1) : 0.0f;
  const float M = wave_max(ms);
  const float w = ms == -INFINITY ? 0.0f : exp2f(ms - M);  // empty split (beyond the sequence): 0
  const float L = wave_sum(w * ls);
  float o[kPer];
#pragma unroll
  for (int t = 0; t < kPer; ++t) o[t] = 0.0f;
  for (int sp0 = 0; sp0 < splits; sp0 += 16) {
    float ws[16], po[16][kPer];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int sp = min(sp0 + i, splits - 1);
      ws[i] = sp0 + i < splits ? __shfl(w, sp, 64) : 0.0f;
#pragma unroll
      for (int t = 0; t < kPer; ++t) po[i][t] = ld_sc1(part_o + (bh * splits + sp) * D + lane + 64 * t);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int t = 0; t < kPer; ++t) o[t] += ws[i] * po[i][t];
  }
  const float inv = L > 0.0f ? 1.0f / L : 0.0f;
#pragma unroll
  for (int t = 0; t < kPer; ++t) out[bh * D + lane + 64 * t] = f2bf(o[t] * inv);
}

template <int D, int G>
int launch_attn(const bf16_t* q, bf16_t* kc, bf16_t* vc, const float* cosT, const float* sinT,
                const int* lens, float* po, float* pml, unsigned* tickets, bf16_t* out, int B, int Hkv,
                int Smax, int splits, float scale, hipStream_t st) {
  const int chunk = ((Smax + splits - 1) / splits + 63) / 64 * 64;
  if (cosT != nullptr)
    hipLaunchKernelGGL((decode_attn_kernel<D, G, true>), dim3(splits, Hkv, B), dim3(64 * G), 0, st, q, kc,
                       vc, cosT, sinT, lens, po, pml, tickets, out, Hkv, Smax, splits, chunk, scale * kLog2e);
  else
    hipLaunchKernelGGL((decode_attn_kernel<D, G, false>), dim3(splits, Hkv, B), dim3(64 * G), 0, st, q, kc,
                       vc, cosT, sinT, lens, po, pml, tickets, out, Hkv, Smax, splits, chunk, scale * kLog2e);
  return KGWE_CHECK_LAUNCH();
}

}  // namespace

KGWE_API int kgwe_decode_rope_append(const void* qkv, const int* pos, const float* cos_t,
                                     const float* sin_t, void* q_out, void* kcache, void* vcache,
                                     int B, int Hq, int Hkv, int D, int Smax, hipStream_t st) {
  if (B <= 0 || Hq <= 0 || Hkv <= 0 || D % 16 != 0 || D > 256 || Smax <= 0) return -1;
  const int64_t n = static_cast<int64_t>(B) * (Hq + 2 * Hkv) * (D / 16);
  const int grid = static_cast<int>(std::min<int64_t>((n + 255) / 256, 4096));
  hipLaunchKernelGGL(rope_append_kernel, dim3(grid), dim3(256), 0, st,
                     static_cast<const bf16_t*>(qkv), pos, cos_t, sin_t, static_cast<bf16_t*>(q_out),
                     static_cast<bf16_t*>(kcache), static_cast<bf16_t*>(vcache), B, Hq, Hkv, D, Smax);
  return KGWE_CHECK_LAUNCH();
}

// Workspace 4-byte words: B * Hq * splits * (D + 2) partials, then B * Hq
// tickets (B * Hkv used).  Must be zeroed once when allocated.
KGWE_API int64_t kgwe_decode_attn_workspace(int B, int Hq, int D, int splits) {
  return static_cast<int64_t>(B) * Hq * splits * (D + 2) + static_cast<int64_t>(B) * Hq;
}

// Split count for a cache of Smax keys: enough workgroups to cover the 256
// CUs about twice, at least 64 keys per split.
KGWE_API int kgwe_decode_attn_splits(int B, int Hkv, int Smax) {
  // ~1024 workgroups up to a serving batch of 32 rows x 8 kv heads (4 splits: 22.0 us per layer
  // against 25.2 with 2 and 25.9 with 8; 640 of 1,024 positions cached); past that one split per
  // (row, kv head) is best: no partials to publish and merge (64 rows: 28.2 us with 1 split, 37.0
  // with 2; 128 rows: 44.8 against 63.4)
  const int want = B * Hkv >= 512 ? 1 : (1024 + B * Hkv - 1) / (B * Hkv);
  const int most = (Smax + 63) / 64;
  return std::max(1, std::min({want, most, 64}));  // the merge holds one split per lane
}

namespace {
int decode_attn_impl(const void* q, void* kcache, void* vcache, const float* cos_t, const float* sin_t,
                     const int* lens, float* workspace, void* out, int B, int Hq, int Hkv, int D, int Smax,
                     int splits, float scale, hipStream_t st) {
  // The merge step reads one split's partial per lane of a 64-wide wave.
  if (B <= 0 || Hkv <= 0 || Hq % Hkv != 0 || splits <= 0 || splits > 64 || Smax <= 0) return -1;
  const int G = Hq / Hkv;
  float* po = workspace;
  float* pml = workspace + static_cast<int64_t>(B) * Hq * splits * D;
  // B * Hkv tickets after the partials; zero when the workspace is created,
  // and returned to zero by every call's last arrivers.
  auto tickets = reinterpret_cast<unsigned*>(pml + static_cast<int64_t>(B) * Hq * splits * 2);
  auto qp = static_cast<const bf16_t*>(q);
  auto kp = static_cast<bf16_t*>(kcache);
  auto vp = static_cast<bf16_t*>(vcache);
  auto op = static_cast<bf16_t*>(out);
#define KGWE_DECODE_CASE(DD, GG)                                                                        \
  if (D == DD && G == GG)                                                                               \
    return launch_attn<DD, GG>(qp, kp, vp, cos_t, sin_t, lens, po, pml, tickets, op, B, Hkv, Smax, splits, \
                               scale, st);
  KGWE_DECODE_CASE(64, 1)
  KGWE_DECODE_CASE(64, 2)
  KGWE_DECODE_CASE(64, 4)
  KGWE_DECODE_CASE(64, 8)
  KGWE_DECODE_CASE(128, 1)
  KGWE_DECODE_CASE(128, 2)
  KGWE_DECODE_CASE(128, 4)
  KGWE_DECODE_CASE(128, 8)
#undef KGWE_DECODE_CASE
  return -2;  // unsupported (head_dim, group) combination
}
}  // namespace

KGWE_API int kgwe_decode_attn(const void* q, const void* kcache, const void* vcache, const int* lens,
                              float* workspace, void* out, int B, int Hq, int Hkv, int D, int Smax,
                              int splits, float scale, hipStream_t st) {
  return decode_attn_impl(q, const_cast<void*>(kcache), const_cast<void*>(vcache), nullptr, nullptr, lens,
                          workspace, out, B, Hq, Hkv, D, Smax, splits, scale, st);
}

// RoPE + cache append + attention in one launch: qkv [B, (Hq + 2 Hkv) * D] of
// the new token at position lens[b] - 1; cos/sin fp32 [>= Smax, D / 2].
KGWE_API int kgwe_decode_attn_rope(const void* qkv, const float* cos_t, const float* sin_t, void* kcache,
                                   void* vcache, const int* lens, float* workspace, void* out, int B, int Hq,
                                   int Hkv, int D, int Smax, int splits, float scale, hipStream_t st) {
  if (cos_t == nullptr || sin_t == nullptr) return -1;
  return decode_attn_impl(qkv, kcache, vcache, cos_t, sin_t, lens, workspace, out, B, Hq, Hkv, D, Smax,
                          splits, scale, st);
}
