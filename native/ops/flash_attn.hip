// Causal GQA flash attention for gfx950 (MI355X), bf16 in / fp32 accumulate,
// head_dim 128, written directly on v_mfma_f32_32x32x16_bf16.
//
// Forward (one workgroup = 4 waves = 128 query rows of one (batch, head)):
//   * each wave owns 32 query rows; Q stays in VGPRs for the whole pass
//     (8 k-steps x bf16x8 = 32 VGPRs);
//   * K/V tiles of 64 keys are staged through LDS (K row-major with a 16-B row
//     pad: conflict-free ds_read_b128; V transposed with an 8-B pad:
//     conflict-free ds_read_b64), register-prefetched one tile ahead so the
//     global loads of tile t+1 overlap the MFMAs of tile t;
//   * S^T = K Q^T is computed with the KEY on the accumulator rows and the
//     query on the lane, so every lane owns one query row: the online-softmax
//     row max / row sum are 32 in-lane ops + one cross-half exchange, and
//     the O rescale is a per-lane scalar;
//   * the P accumulator is converted pairwise to bf16 and fed straight back
//     as the B operand of O^T += V^T P (cdna_hip_programming.md §3
//     "accumulator tile as the next MFMA's operand": the permuted k order
//     is matched by the V^T reads), so P never touches LDS;
//   * workgroup ids are remapped XCD-aware so all query blocks and all query
//     heads of one (batch, kv-head) run on one XCD and share its L2 copy of
//     K/V; causal blocks are issued heaviest-first.
// Log-sum-exp is returned in the log2 domain (lse2 = max2 + log2(sum)) for
// the backward pass.
//
// Backward (FA2 split, no dQ atomics => deterministic):
//   * dkdv kernel: one workgroup = 4 waves = 128 keys of one (batch, kv-head);
//     each wave owns 32 keys, keeps K and V in VGPRs and dK^T / dV^T
//     accumulators (2 x 64 fp32) in VGPRs, and sweeps every query head of
//     its GQA group x every 32-row query tile: S (key on the lane),
//     P = exp2(S*c - lse2), dV^T += dO^T P, dP = dO V^T, dS = P (dP - delta),
//     dK^T += Q^T dS — all operands of the P/dS products come from the
//     accumulators (no LDS round trip); Q / dO tiles are staged in LDS in
//     both row and transposed images.
//   * dq kernel: one workgroup = 128 query rows of one (batch, head) (the
//     forward's geometry, query on the lane): recomputes S^T and dP^T and
//     accumulates dQ^T += K^T dS^T with K^T staged transposed in LDS.
//   * delta = rowsum(dO * O) by a small preprocess kernel.
#include "common.h"

using namespace kgwe;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 mfma8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;

constexpr int HD = 128;             // head dim
constexpr int BQ = 128;             // query rows per forward workgroup
constexpr int BKV = 64;             // keys per forward tile
constexpr int KST = HD + 8;         // K row stride in LDS (bf16): 272 B
constexpr int VST = BKV + 4;        // V^T row stride in LDS (bf16): 136 B

__device__ __forceinline__ mfma8 as_m(bf16x8 v) { return __builtin_bit_cast(mfma8, v); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_m(a), as_m(b), c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

__device__ __forceinline__ bf16x8 cat44(u16x4 lo, u16x4 hi) {
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// Accumulator register r of a 32x32 tile holds row (r&3) + 8*(r>>2) + 4*half.
__device__ __forceinline__ int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// Decode a 1-D workgroup id into (b, hkv, g, qb): XCD-aware so consecutive
// logical ids (same kv head) share an XCD; causal: heaviest query blocks first.
__device__ __forceinline__ void decode(int nQB, int G, int Hkv, bool causal, int* b, int* h,
                                       int* hkv, int* qb) {
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  int t = wg;
  int q = t % nQB;
  t /= nQB;
  const int g = t % G;
  t /= G;
  *hkv = t % Hkv;
  *b = t / Hkv;
  *h = *hkv * G + g;
  *qb = causal ? nQB - 1 - q : q;
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, float* __restrict__ lse2, int S, int Hq, int Hkv, float c,
    int causal, int nQB) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BKV * KST];
  __shared__ __attribute__((aligned(16))) bf16_t Vt[HD * VST];
  int b, h, hkv, qb;
  decode(nQB, Hq / Hkv, Hkv, causal, &b, &h, &hkv, &qb);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int q0 = qb * BQ + w * 32;
  const int qrow = q0 + lq;
  const size_t qs = static_cast<size_t>(Hq) * HD, kvs = static_cast<size_t>(Hkv) * HD;

  bf16x8 qf[8];
  {
    const bf16_t* qp = q + (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD;
#pragma unroll
    for (int t = 0; t < 8; ++t) qf[t] = qrow < S ? ld16(qp + 16 * t + 8 * hh) : bf16x8{};
  }
  f32x16 oacc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) oacc[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  const int kv_end = causal ? min(S, qb * BQ + BQ) : S;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  const bf16_t* kb = k + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  const bf16_t* vb = v + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  bf16x8 kr[4], vr[4];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + 256 * i, key = idx >> 4, ch = idx & 15;
      const int s = kt * BKV + key;
      if (s < S) {
        kr[i] = ld16(kb + static_cast<size_t>(s) * kvs + ch * 8);
        vr[i] = ld16(vb + static_cast<size_t>(s) * kvs + ch * 8);
      } else {
        kr[i] = bf16x8{};
        vr[i] = bf16x8{};
      }
    }
  };
  gload(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    __syncthreads();  // every wave is done reading the previous tile
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + 256 * i, key = idx >> 4, ch = idx & 15;
      *reinterpret_cast<bf16x8*>(&Ks[key * KST + ch * 8]) = kr[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) Vt[(ch * 8 + j) * VST + key] = vr[i][j];
    }
    __syncthreads();
    if (kt + 1 < ntiles) gload(kt + 1);  // in flight during this tile's MFMAs
    const int k0 = kt * BKV;
    if (causal && k0 > q0 + 31) continue;  // tile entirely above this wave's diagonal

    f32x16 sacc[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int t = 0; t < 8; ++t)
        sacc[st] = mfma(*reinterpret_cast<const bf16x8*>(&Ks[(st * 32 + lq) * KST + 16 * t + 8 * hh]),
                        qf[t], sacc[st]);
    float mx = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + st * 32 + acc_row(r, hh);
        float s = sacc[st][r] * c;
        if (key >= S || (causal && key > qrow)) s = -INFINITY;
        sacc[st][r] = s;
        mx = fmaxf(mx, s);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
    const float m_new = fmaxf(m, mx);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m - m_use);
    float rs = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(sacc[st][r] - m_use);
        sacc[st][r] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 32, kWave);
    l = l * alpha + rs;
    m = m_new;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[db][r] *= alpha;
    // O^T += V^T P : P (key rows, query on lane) is the B operand as is.
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int st = s >> 1, sp = s & 1;
      bf16x8 pb;
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = f2bf(sacc[st][8 * sp + j]);
      const int kl = st * 32 + 16 * sp + 4 * hh;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16_t* vrow = &Vt[(db * 32 + lq) * VST + kl];
        const bf16x8 a = cat44(*reinterpret_cast<const u16x4*>(vrow),
                               *reinterpret_cast<const u16x4*>(vrow + 8));
        oacc[db] = mfma(a, pb, oacc[db]);
      }
    }
  }
  if (qrow < S) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* op = o + (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        u16x4 v4;
#pragma unroll
        for (int j = 0; j < 4; ++j) v4[j] = f2bf(oacc[db][4 * g4 + j] * inv);
        *reinterpret_cast<u16x4*>(op + db * 32 + 8 * g4 + 4 * hh) = v4;
      }
    if (hh == 0)
      lse2[(static_cast<size_t>(b) * Hq + h) * S + qrow] = l > 0.f ? m + log2f(l) : -INFINITY;
  }
}

}  // namespace

KGWE_API int kgwe_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse2,
                                 int B, int S, int Hq, int Hkv, int D, float scale, int causal,
                                 hipStream_t s) {
  if (D != HD || Hq % Hkv != 0 || B <= 0 || S <= 0) return -1;
  const int nQB = (S + BQ - 1) / BQ;
  const long long grid = static_cast<long long>(B) * Hq * nQB;
  if (grid > 0x7fffffff) return -1;
  const float c = scale * 1.4426950408889634f;  // softmax in the exp2 domain
  hipLaunchKernelGGL(fa_fwd_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k),
                     static_cast<const bf16_t*>(v), static_cast<bf16_t*>(o), lse2, S, Hq, Hkv, c,
                     causal, nQB);
  return KGWE_CHECK_LAUNCH();
}
