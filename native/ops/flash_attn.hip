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

// ---------------------------------------------------------------------------
// backward: delta = rowsum(dO * O)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fa_bwd_pre_kernel(const bf16_t* __restrict__ o,
                                                         const bf16_t* __restrict__ dout,
                                                         float* __restrict__ delta, int B, int S,
                                                         int Hq) {
  // 16 lanes x 8 elements per (b, s, h) row of 128.
  const long long row = (static_cast<long long>(blockIdx.x) * 256 + threadIdx.x) >> 4;
  const int sub = threadIdx.x & 15;
  const long long nrows = static_cast<long long>(B) * S * Hq;
  float acc = 0.f;
  if (row < nrows) {
    const bf16x8 a = ld16(o + row * HD + sub * 8);
    const bf16x8 d = ld16(dout + row * HD + sub * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += bf2f(a[j]) * bf2f(d[j]);
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  if (row < nrows && sub == 0) {
    const long long h = row % Hq, s = (row / Hq) % S, b = row / (static_cast<long long>(Hq) * S);
    delta[(b * Hq + h) * S + s] = acc;
  }
}

constexpr int BQT = 32;        // query rows per backward step
constexpr int QST = HD + 8;    // Q / dO row-image stride (bf16)
constexpr int TST = BQT + 4;   // Q^T / dO^T image stride (bf16): 72 B rows

// dK, dV: one workgroup = 128 keys of one (b, kv head); wave = 32 keys.
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2,
    const float* __restrict__ delta, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int S,
    int Hq, int Hkv, float c, float scale, int causal, int nKB) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[BQT * QST];
  __shared__ __attribute__((aligned(16))) bf16_t Ds[BQT * QST];
  __shared__ __attribute__((aligned(16))) bf16_t Qt[HD * TST];
  __shared__ __attribute__((aligned(16))) bf16_t Dt[HD * TST];
  __shared__ float Ls[BQT], Dl[BQT];
  const int G = Hq / Hkv;
  // Decode (b, hkv, key block): XCD-aware, heaviest (earliest keys) first.
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = wg % nKB;
  const int hkv = (wg / nKB) % Hkv;
  const int b = wg / (nKB * Hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lk = lane & 31, hh = lane >> 5;
  const int key0 = kb * 128 + w * 32;
  const int key = key0 + lk;
  const size_t qs = static_cast<size_t>(Hq) * HD, kvs = static_cast<size_t>(Hkv) * HD;
  bf16x8 kf[8], vf[8];
  {
    const size_t off = (static_cast<size_t>(b) * S + key) * kvs + static_cast<size_t>(hkv) * HD;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      kf[t] = key < S ? ld16(k + off + 16 * t + 8 * hh) : bf16x8{};
      vf[t] = key < S ? ld16(v + off + 16 * t + 8 * hh) : bf16x8{};
    }
  }
  f32x16 dka[4], dva[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dka[i] = dva[i] = f32x16{};

  const int qt_begin = causal ? (kb * 128) / BQT : 0;
  const int nqt = (S + BQT - 1) / BQT;
  const int total = G * (nqt - qt_begin);
  bf16x8 qr[2], dr[2];
  float lr = 0.f, drl = 0.f;
  auto gload = [&](int it) {
    const int g = it / (nqt - qt_begin), qt = qt_begin + it % (nqt - qt_begin);
    const int h = hkv * G + g;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = threadIdx.x + 256 * i, r = idx >> 4, ch = idx & 15, s = qt * BQT + r;
      const size_t off = (static_cast<size_t>(b) * S + s) * qs + static_cast<size_t>(h) * HD + ch * 8;
      qr[i] = s < S ? ld16(q + off) : bf16x8{};
      dr[i] = s < S ? ld16(dout + off) : bf16x8{};
    }
    if (threadIdx.x < BQT) {
      const int s = qt * BQT + threadIdx.x;
      const size_t li = (static_cast<size_t>(b) * Hq + h) * S + s;
      lr = s < S ? lse2[li] : INFINITY;
      drl = s < S ? delta[li] : 0.f;
    }
  };
  if (total > 0) gload(0);
  for (int it = 0; it < total; ++it) {
    const int qt = qt_begin + it % (nqt - qt_begin);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = threadIdx.x + 256 * i, r = idx >> 4, ch = idx & 15;
      *reinterpret_cast<bf16x8*>(&Qs[r * QST + ch * 8]) = qr[i];
      *reinterpret_cast<bf16x8*>(&Ds[r * QST + ch * 8]) = dr[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Qt[(ch * 8 + j) * TST + r] = qr[i][j];
        Dt[(ch * 8 + j) * TST + r] = dr[i][j];
      }
    }
    if (threadIdx.x < BQT) {
      Ls[threadIdx.x] = lr;
      Dl[threadIdx.x] = drl;
    }
    __syncthreads();
    if (it + 1 < total) gload(it + 1);
    const int qbase = qt * BQT;
    if (causal && qbase + BQT - 1 < key0) continue;  // every query of this tile precedes our keys
    // S[q][key] = Q K^T and dP[q][key] = dO V^T (key on the lane).
    f32x16 sa = f32x16{}, pa = f32x16{};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      sa = mfma(*reinterpret_cast<const bf16x8*>(&Qs[lk * QST + 16 * t + 8 * hh]), kf[t], sa);
      pa = mfma(*reinterpret_cast<const bf16x8*>(&Ds[lk * QST + 16 * t + 8 * hh]), vf[t], pa);
    }
    // P = exp2(S c - lse2), dS = P (dP - delta); row r <-> query qbase + acc_row(r).
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = acc_row(r, hh);
      const int qrow = qbase + qi;
      float p = exp2f(sa[r] * c - Ls[qi]);
      if (key >= S || qrow >= S || (causal && key > qrow)) p = 0.f;
      sa[r] = p;
      pa[r] = p * (pa[r] - Dl[qi]);
    }
    // dV^T += dO^T P ; dK^T += Q^T dS   (P, dS as B operands, permuted q order)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 pb, sb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pb[j] = f2bf(sa[8 * s + j]);
        sb[j] = f2bf(pa[8 * s + j]);
      }
      const int ql = 16 * s + 4 * hh;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16_t* drow = &Dt[(db * 32 + lk) * TST + ql];
        const bf16_t* qrow_t = &Qt[(db * 32 + lk) * TST + ql];
        dva[db] = mfma(cat44(*reinterpret_cast<const u16x4*>(drow), *reinterpret_cast<const u16x4*>(drow + 8)),
                       pb, dva[db]);
        dka[db] = mfma(cat44(*reinterpret_cast<const u16x4*>(qrow_t),
                             *reinterpret_cast<const u16x4*>(qrow_t + 8)),
                       sb, dka[db]);
      }
    }
  }
  if (key < S) {
    const size_t off = (static_cast<size_t>(b) * S + key) * kvs + static_cast<size_t>(hkv) * HD;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        u16x4 a, bb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = f2bf(dka[db][4 * g4 + j] * scale);
          bb[j] = f2bf(dva[db][4 * g4 + j]);
        }
        *reinterpret_cast<u16x4*>(dk + off + db * 32 + 8 * g4 + 4 * hh) = a;
        *reinterpret_cast<u16x4*>(dv + off + db * 32 + 8 * g4 + 4 * hh) = bb;
      }
  }
}

// dQ: one workgroup = 128 query rows of one (b, head); wave = 32 rows (the
// forward's geometry: query on the lane).
__global__ __launch_bounds__(256, 1) void fa_bwd_dq_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2,
    const float* __restrict__ delta, bf16_t* __restrict__ dq, int S, int Hq, int Hkv, float c,
    float scale, int causal, int nQB) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BKV * KST];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[BKV * KST];
  __shared__ __attribute__((aligned(16))) bf16_t Kt[HD * VST];
  int b, h, hkv, qb;
  decode(nQB, Hq / Hkv, Hkv, causal, &b, &h, &hkv, &qb);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int q0 = qb * BQ + w * 32;
  const int qrow = q0 + lq;
  const size_t qs = static_cast<size_t>(Hq) * HD, kvs = static_cast<size_t>(Hkv) * HD;
  bf16x8 qf[8], df[8];
  {
    const size_t off = (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      qf[t] = qrow < S ? ld16(q + off + 16 * t + 8 * hh) : bf16x8{};
      df[t] = qrow < S ? ld16(dout + off + 16 * t + 8 * hh) : bf16x8{};
    }
  }
  const size_t li = (static_cast<size_t>(b) * Hq + h) * S + qrow;
  const float my_lse = qrow < S ? lse2[li] : INFINITY;
  const float my_delta = qrow < S ? delta[li] : 0.f;
  f32x16 dqa[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dqa[i] = f32x16{};
  const int kv_end = causal ? min(S, qb * BQ + BQ) : S;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  const bf16_t* kb_ = k + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  const bf16_t* vb_ = v + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  bf16x8 kr[4], vr[4];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + 256 * i, kk = idx >> 4, ch = idx & 15, s = kt * BKV + kk;
      kr[i] = s < S ? ld16(kb_ + static_cast<size_t>(s) * kvs + ch * 8) : bf16x8{};
      vr[i] = s < S ? ld16(vb_ + static_cast<size_t>(s) * kvs + ch * 8) : bf16x8{};
    }
  };
  gload(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + 256 * i, kk = idx >> 4, ch = idx & 15;
      *reinterpret_cast<bf16x8*>(&Ks[kk * KST + ch * 8]) = kr[i];
      *reinterpret_cast<bf16x8*>(&Vs[kk * KST + ch * 8]) = vr[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) Kt[(ch * 8 + j) * VST + kk] = kr[i][j];
    }
    __syncthreads();
    if (kt + 1 < ntiles) gload(kt + 1);
    const int k0 = kt * BKV;
    if (causal && k0 > q0 + 31) continue;
    f32x16 sa[2] = {f32x16{}, f32x16{}}, pa[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        sa[st] = mfma(*reinterpret_cast<const bf16x8*>(&Ks[(st * 32 + lq) * KST + 16 * t + 8 * hh]), qf[t], sa[st]);
        pa[st] = mfma(*reinterpret_cast<const bf16x8*>(&Vs[(st * 32 + lq) * KST + 16 * t + 8 * hh]), df[t], pa[st]);
      }
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = k0 + st * 32 + acc_row(r, hh);
        float p = exp2f(sa[st][r] * c - my_lse);
        if (kk >= S || qrow >= S || (causal && kk > qrow)) p = 0.f;
        pa[st][r] = p * (pa[st][r] - my_delta);  // dS^T
      }
    // dQ^T += K^T dS^T
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int st = s >> 1, sp = s & 1;
      bf16x8 sb;
#pragma unroll
      for (int j = 0; j < 8; ++j) sb[j] = f2bf(pa[st][8 * sp + j]);
      const int kl = st * 32 + 16 * sp + 4 * hh;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16_t* krow = &Kt[(db * 32 + lq) * VST + kl];
        dqa[db] = mfma(cat44(*reinterpret_cast<const u16x4*>(krow), *reinterpret_cast<const u16x4*>(krow + 8)),
                       sb, dqa[db]);
      }
    }
  }
  if (qrow < S) {
    bf16_t* p = dq + (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        u16x4 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = f2bf(dqa[db][4 * g4 + j] * scale);
        *reinterpret_cast<u16x4*>(p + db * 32 + 8 * g4 + 4 * hh) = a;
      }
  }
}

}  // namespace

KGWE_API int64_t kgwe_flash_attn_bwd_workspace(int B, int S, int Hq, int Hkv, int D) {
  return static_cast<int64_t>(B) * Hq * S * sizeof(float);  // delta
}

// lse2 from the forward (log2 units).  `work` >= workspace bytes.
KGWE_API int kgwe_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                                 const float* lse2, const void* dout, void* dq, void* dk, void* dv,
                                 float* work, void* /*reserved*/, int B, int S, int Hq, int Hkv,
                                 int D, float scale, int causal, hipStream_t s) {
  if (D != HD || Hq % Hkv != 0 || B <= 0 || S <= 0) return -1;
  const float c = scale * 1.4426950408889634f;
  const long long rows = static_cast<long long>(B) * S * Hq;
  hipLaunchKernelGGL(fa_bwd_pre_kernel, dim3(static_cast<unsigned>((rows * 16 + 255) / 256)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(o), static_cast<const bf16_t*>(dout), work, B, S, Hq);
  int rc = KGWE_CHECK_LAUNCH();
  if (rc) return rc;
  const int nKB = (S + 127) / 128;
  hipLaunchKernelGGL(fa_bwd_dkdv_kernel, dim3(static_cast<unsigned>(B * Hkv * nKB)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k),
                     static_cast<const bf16_t*>(v), static_cast<const bf16_t*>(dout), lse2, work,
                     static_cast<bf16_t*>(dk), static_cast<bf16_t*>(dv), S, Hq, Hkv, c, scale, causal, nKB);
  rc = KGWE_CHECK_LAUNCH();
  if (rc) return rc;
  const int nQB = (S + BQ - 1) / BQ;
  hipLaunchKernelGGL(fa_bwd_dq_kernel, dim3(static_cast<unsigned>(B * Hq * nQB)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k),
                     static_cast<const bf16_t*>(v), static_cast<const bf16_t*>(dout), lse2, work,
                     static_cast<bf16_t*>(dq), S, Hq, Hkv, c, scale, causal, nQB);
  return KGWE_CHECK_LAUNCH();
}

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
