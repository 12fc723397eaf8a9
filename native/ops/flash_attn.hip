// Causal GQA flash attention for gfx950 (MI355X), bf16 in / fp32 accumulate,
// head_dim 128, written directly on v_mfma_f32_32x32x16_bf16.
//
// Forward (one workgroup = 8 waves = 256 query rows of one (batch, head), one
// workgroup per CU, two waves per SIMD):
//   * each wave owns 32 query rows; Q stays in VGPRs for the whole pass
//     (8 k-steps x bf16x8 = 32 VGPRs);
//   * K/V tiles of 64 keys are double-buffered in LDS (K row-major with a
//     16-B row pad: conflict-free ds_read_b128; V row-major in an XOR-swizzled
//     image read with the gfx950 hardware transpose ds_read_b64_tr_b16, so
//     nothing is transposed on the write side); the global loads of tile t+1
//     are issued before tile t's MFMAs and stored after them, one barrier per
//     tile; O is rescaled only when some row's running max moved;
//   * S^T = K Q^T is computed with the KEY on the accumulator rows and the
//     query on the lane, so every lane owns one query row: the online-softmax
//     row max is 32 in-lane ops + one v_permlane32_swap half exchange (the
//     row sum's exchange waits for the epilogue), and the O rescale is a
//     per-lane scalar;
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
//     each wave owns 32 keys, keeps K and the dK^T / dV^T accumulators
//     (2 x 64 fp32) in VGPRs (V rows come from a per-workgroup LDS image, so
//     the kernel fits 256 VGPRs and two workgroups share a CU), and sweeps every query head of
//     its GQA group x every 32-row query tile: S (key on the lane),
//     P = exp2(S*c - lse2), dV^T += dO^T P, dP = dO V^T, dS = P (dP - delta),
//     dK^T += Q^T dS — all operands of the P/dS products come from the
//     accumulators (no LDS round trip); Q / dO tiles are double-buffered in
//     ONE swizzled image each, read by rows (ds_read_b128) for S and dP and
//     by columns (ds_read_b64_tr_b16) for dV^T and dK^T.
//   * dq kernel: one workgroup = 8 waves = 256 query rows of one (batch,
//     head) (the forward's geometry, query on the lane): recomputes S^T and
//     dP^T and accumulates dQ^T += K^T dS^T, K^T read transposed from the K
//     image.  8 waves measured ahead of 4 (two workgroups per CU): causal
//     1.097-1.110 vs 1.119-1.129 ms for the backward, full 1.861 vs 1.914.
//   * delta = rowsum(dO * O) by a small preprocess kernel.
#include "common.h"

#include <algorithm>
#include <array>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

using namespace kgwe;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 mfma8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

constexpr int HD = 128;             // head dim
#ifndef FA_DQ_DELTA
#define FA_DQ_DELTA 1
#endif
#ifndef FA_DQ_WAVES
#define FA_DQ_WAVES 8
#endif
constexpr int DQW = FA_DQ_WAVES;    // waves per dQ workgroup (32 query rows each)
constexpr int BQ = 32 * DQW;        // query rows per dQ workgroup
constexpr int DQNT = 64 * DQW;      // threads per dQ workgroup
constexpr int DQSTG = 16 / DQW;     // 16-B K (and V) chunks per thread per 64-key tile
static_assert(DQW == 4 || DQW == 8, "dQ workgroup: 4 or 8 waves");
constexpr int BKV = 64;             // keys per forward tile
constexpr int KST = HD + 8;         // K row stride in LDS (bf16): 272 B

__device__ __forceinline__ mfma8 as_m(bf16x8 v) { return __builtin_bit_cast(mfma8, v); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_m(a), as_m(b), c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// 2^x as ONE v_exp_f32.  exp2f() adds a denormal-range fixup around it
// (v_cmp + v_cndmask + v_add before, v_ldexp after: 4 extra VALU per element,
// ~30 % of the softmax VALU stream); softmax arguments are <= 0 and a result
// below 2^-126 is 0 to within bf16 anyway.  exp(-inf) is still 0.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ bf16x8 cat44(u16x4 lo, u16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);  // a register-pair concat
}

// Two floats -> one packed bf16 pair (RNE), ONE v_cvt_pk_bf16_f32.  Building
// MFMA operands element-wise from f2bf() cost a convert per element plus
// v_perm / v_or / v_mov to pack the halves (3x the VALU).
typedef __attribute__((ext_vector_type(2))) float f32x2v;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;
__device__ __forceinline__ unsigned pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){lo, hi}, bf16x2v));
}
__device__ __forceinline__ bf16x8 pk8(const u32x4& w) { return __builtin_bit_cast(bf16x8, w); }
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

// Accumulator register r of a 32x32 tile holds row (r&3) + 8*(r>>2) + 4*half.
__device__ __forceinline__ int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// Raise a wave's issue priority over its MFMA chains and drop it for the
// softmax, so each SIMD's arbiter keeps the matrix pipe fed from whichever of
// its two waves is in an MFMA phase.  Measured (tools/gpu.sh fa-variants, B=2
// S=4096 causal): backward 1.142 -> 1.128 ms, forward 0.369 -> 0.384 ms — so
// on in the dQ and dK/dV kernels, off in the forward.
#ifndef FA_MFMA_PRIO_FWD
#define FA_MFMA_PRIO_FWD 0
#endif
#ifndef FA_MFMA_PRIO_BWD
#define FA_MFMA_PRIO_BWD 1
#endif
// mode 1: MFMA chains at priority 1; mode 2: the inverse (softmax phases at
// priority 1, MFMA chains at 0); mode 3: MFMA chains at priority 3.
#define FA_PRIO_HI_(on)                                          \
  do {                                                           \
    if ((on) == 1) __builtin_amdgcn_s_setprio(1);                \
    if ((on) == 2) __builtin_amdgcn_s_setprio(0);                \
    if ((on) == 3) __builtin_amdgcn_s_setprio(3);                \
  } while (0)
#define FA_PRIO_LO_(on)                                          \
  do {                                                           \
    if ((on) == 1 || (on) == 3) __builtin_amdgcn_s_setprio(0);   \
    if ((on) == 2) __builtin_amdgcn_s_setprio(1);                \
  } while (0)

// max / sum of lane l and lane l ^ 32 in every lane: one v_permlane32_swap
// (a VALU half exchange) instead of an LDS ds_bpermute round trip.
__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Store one row of a transposed accumulator set (acc[db] register r holds
// column db*32 + acc_row(r, hh) of THIS lane's row), times `mul`, as bf16
// with 16-B stores: a lane holds 4 consecutive columns per register group,
// its partner lane (l ^ 32) the next 4, so one v_permlane32_swap per dword
// pairs them up — 8 global_store_dwordx4 per lane instead of 16 dwordx2
// (the store-issue-bound epilogue tail, cdna_hip_programming.md T21).  Every
// lane must execute it (the swaps cross lanes); `ok` guards only the stores.
__device__ __forceinline__ void store_row_t(bf16_t* row, const f32x16 (&acc)[4], float mul, int hh,
                                            bool ok) {
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const f32x16& a = acc[db];
      const int g0 = 4 * (2 * pr), g1 = 4 * (2 * pr + 1);
      const auto r0 = __builtin_amdgcn_permlane32_swap(pk_bf16(a[g0] * mul, a[g0 + 1] * mul),
                                                       pk_bf16(a[g1] * mul, a[g1 + 1] * mul), false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(pk_bf16(a[g0 + 2] * mul, a[g0 + 3] * mul),
                                                       pk_bf16(a[g1 + 2] * mul, a[g1 + 3] * mul), false, false);
      const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
      if (ok) *reinterpret_cast<u32x4*>(row + db * 32 + 16 * pr + 8 * hh) = v;
    }
}

// Decode a 1-D workgroup id into (b, hkv, g, qb): XCD-aware so consecutive
// logical ids (same kv head) share an XCD; causal: heaviest query blocks first.
//
// Causal: each XCD holds a contiguous range of whole heads, and within it the
// workgroups are dispatched heaviest query block FIRST ACROSS ALL its heads
// (all last blocks, then all second-to-last, ...): longest-processing-time
// order, so the last workgroups to start are the lightest.  Walking the
// blocks of one head after another (heavy -> light, then the next head's
// heavy block) put a 64-tile block at the end of every XCD's queue and left
// ~25 % of the wave slots idle in the tail (SQ_WAVE_CYCLES vs GRBM_GUI_ACTIVE,
// profiles/r02_attn).
__device__ __forceinline__ void decode(int nQB, int G, int Hkv, bool causal, int* b, int* h,
                                       int* hkv, int* qb) {
  const int n = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, n);
  int t, q;
  const int per_xcd = n / 8;
  if (causal && n % 8 == 0 && per_xcd % nQB == 0) {
    const int heads = per_xcd / nQB;  // heads per XCD
    const int xcd = wg / per_xcd, local = wg - xcd * per_xcd;
    q = local / heads;
    t = xcd * heads + local % heads;
  } else {
    t = wg;
    q = t % nQB;
    t /= nQB;
  }
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
// V tile image for the hardware-transposed read (ds_read_b64_tr_b16): plain
// 256-B rows [key][d] written straight from HBM with 16-B stores, 16-B chunks
// XOR-swizzled by row so the transposed reads of a 32-lane half (4 keys x 64 B)
// hit 64 distinct banks (cdna_hip_programming.md T10, layout (b)).
__device__ __forceinline__ int v_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ u16x4 tr_read(const bf16_t* lds_base, int byte_off) {
  typedef __attribute__((ext_vector_type(4))) short s4;
  const s4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(reinterpret_cast<const char*>(lds_base) + byte_off));
  return __builtin_bit_cast(u16x4, r);
}

// Deferred running max (cdna_hip_programming.md T13) with a 2^4 bound on P:
// at B=4, S=4096 causal the forward goes 0.672-0.684 -> 0.650-0.654 ms; the
// numerics cases (growing max, a x6 max jump mid-sweep) stay within one bf16
// ulp of the fp32 reference (tools/fa_fwd_err.py: max 1.56e-2 at |O| ~ 2-4).
// T = 8 had failed the max-jump case at 2 ulps.
#ifndef FA_DEFER_T
#define FA_DEFER_T 4.f
#endif
#ifndef FA_FWD_WAVES
#define FA_FWD_WAVES 8
#endif
#ifndef FA_FWD_QPW
#define FA_FWD_QPW 1
#endif
constexpr int FNW = FA_FWD_WAVES;   // waves per forward workgroup
constexpr int QPW = FA_FWD_QPW;     // 32-row query sub-blocks per wave
constexpr int FNT = 64 * FNW;       // threads per forward workgroup
constexpr int BQF = 32 * QPW * FNW; // query rows per forward workgroup
constexpr int KTILE = BKV * KST;    // bf16 elements of one K buffer
constexpr int VTILE = BKV * HD;     // bf16 elements of one V buffer
static_assert(FNW * QPW <= 8 && 16 % FNW == 0, "at most 256 query rows, 16 staging chunks split evenly");

// One workgroup = FNW waves x QPW 32-row sub-blocks of one (batch, head);
// K/V tiles of 64 keys double-buffered in LDS (67 KB): the global loads of
// tile t+1 are issued before tile t's MFMAs and written to the other buffer
// after them, so one barrier per tile separates the phases.
// Default geometry, measured with tools/fa_variants.hip (B=2, S=4096):
// 8 waves x 1 sub-block = 256 rows per workgroup, one 512-thread workgroup
// per CU (67 KB LDS, <= 256 VGPRs per wave, two waves per SIMD).  Earlier
// the 4-wave / two-workgroups-per-CU form won (641 vs 622 TF/s,
// profiles/r01_attn_counters/NOTES.md: barrier coupling of the two waves on
// a SIMD); after the VALU trims, longest-first dispatch and 16-B epilogue
// stores, the 8-wave form wins: causal 0.338-0.345 vs 0.354-0.357 ms, full
// 0.595 vs 0.631 ms (924 TF/s) — each K / V tile staged once feeds twice the
// rows.  QPW = 2 (each K / V^T fragment read feeds two MFMAs, one wave per
// SIMD) spills past 256 arch VGPRs and runs at 400-500 TF/s.
template <bool EVEN>
__global__ __launch_bounds__(FNT, (QPW == 1 && FNW <= 4) ? 2 : 1) void fa_fwd_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, float* __restrict__ lse2, int S, int Hq, int Hkv, float c,
    int causal, int nQB) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2 * KTILE];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2 * VTILE];
  int b, h, hkv, qb;
  decode(nQB, Hq / Hkv, Hkv, causal, &b, &h, &hkv, &qb);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int q0 = qb * BQF + w * 32 * QPW;  // first query row of this wave
  const size_t qs = static_cast<size_t>(Hq) * HD, kvs = static_cast<size_t>(Hkv) * HD;
  // 8 waves: the second-dispatched half loses VALU arbitration on every
  // segment; one static priority bump evens it out (MI355X_MICROARCH.md).
#ifndef FA_FWD_HALF_PRIO
#define FA_FWD_HALF_PRIO 1
#endif
  if (FA_FWD_HALF_PRIO && FNW == 8 && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256)
    __builtin_amdgcn_s_setprio(1);

  bf16x8 qf[QPW][8];
#pragma unroll
  for (int j = 0; j < QPW; ++j) {
    const int qrow = q0 + 32 * j + lq;
    const bf16_t* qp = q + (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD;
#pragma unroll
    for (int t = 0; t < 8; ++t) qf[j][t] = (EVEN || qrow < S) ? ld16(qp + 16 * t + 8 * hh) : bf16x8{};
  }
  f32x16 oacc[QPW][4];
  float m[QPW], l[QPW];
#pragma unroll
  for (int j = 0; j < QPW; ++j) {
#pragma unroll
    for (int i = 0; i < 4; ++i) oacc[j][i] = f32x16{};
    m[j] = -INFINITY;
    l[j] = 0.f;
  }

  const int kv_end = causal ? min(S, qb * BQF + BQF) : S;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  const bf16_t* kb = k + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  const bf16_t* vb = v + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  // Staging: thread t moves chunks (key, ch) = ((t + FNT i) >> 4, t & 15), i < NSTG.
  constexpr int NSTG = 16 / FNW;  // 16-B chunks per thread per tile (K and V each)
  const int skey = threadIdx.x >> 4, sch = threadIdx.x & 15;
  // K and V of the next tile are staged through registers one after the
  // other (K loaded at the top and stored after the S MFMAs, V loaded then
  // and stored after the O MFMAs) to halve the staging registers.
  bf16x8 sr[NSTG];
  // Addresses: a wave-uniform tile base plus a 32-bit per-lane offset (the
  // global_load SGPR-base form), not a 64-bit multiply per chunk and tile.
  const unsigned soff = static_cast<unsigned>(skey) * static_cast<unsigned>(kvs) + sch * 8u;
  auto gload = [&](const bf16_t* base, int kt) {
    const bf16_t* tb = base + static_cast<size_t>(kt * BKV) * kvs;
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      const int s = kt * BKV + skey + 4 * FNW * i;
      sr[i] = (EVEN || s < S) ? ld16(tb + (soff + static_cast<unsigned>(4 * FNW * i * kvs))) : bf16x8{};
    }
  };
  auto kwrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NSTG; ++i)
      *reinterpret_cast<bf16x8*>(&Ks[buf * KTILE + (skey + 4 * FNW * i) * KST + sch * 8]) = sr[i];
  };
  auto vwrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NSTG; ++i)
      *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(&Vs[buf * VTILE]) + v_off(skey + 4 * FNW * i, sch)) = sr[i];
  };
  // Transposed-read lane geometry (T10): group G = lane >> 4 reads keys
  // base + 4*(G >> 1) + qq at d chunk 4*db + 2*(G & 1) + (pp >> 1), byte 8*(pp & 1).
  const int trG = lane >> 4, trq = (lane >> 2) & 3, trp = lane & 3;
  const int tr_row = 4 * (trG >> 1) + trq;
  const int tr_ch = 2 * (trG & 1) + (trp >> 1);
  const int tr_byte = 8 * (trp & 1);
  // v_off(C + tr_row, 4 db + tr_ch) + tr_byte for a row base C that is a
  // multiple of 8: = 256 C + voff[db][(C / 8) & 1] — the swizzle's low bits
  // depend on C only through (C / 8) & 1, its high bits XOR db with trq.
  int voff[4][2];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi)
      voff[db][hi] = 256 * tr_row + tr_byte + 64 * (db ^ trq) + 16 * (tr_ch ^ (trG >> 1) ^ (2 * hi));

  gload(kb, 0);
  kwrite(0);
  gload(vb, 0);
  vwrite(0);
  // Pin the Q loads before the loop.  Left alone, hipcc sinks them past the
  // barrier to the loop entry, and the waitcnt pass — which cannot tell the
  // first iteration from the rest — then waits vmcnt(7) .. vmcnt(0) at the
  // eight S MFMAs of EVERY tile: the next tile's K prefetch is forced to land
  // inside the first half of the S chain instead of under the whole tile.
#pragma unroll
  for (int j = 0; j < QPW; ++j)
#pragma unroll
    for (int t = 0; t < 8; ++t) asm volatile("" ::"v"(qf[j][t]));
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < ntiles;
    if (more) gload(kb, kt + 1);  // lands during this tile's S MFMAs
    const int k0 = kt * BKV;
    const bool active = !causal || k0 <= q0 + 32 * QPW - 1;  // else: tile above this wave's diagonal
    f32x16 sacc[QPW][2];
    if (active) {  // else: tile entirely above this wave's diagonal
      const bf16_t* Kc = Ks + cur * KTILE;
      // S^T = K Q^T for every sub-block: each K fragment feeds QPW MFMAs.
#pragma unroll
      for (int j = 0; j < QPW; ++j) sacc[j][0] = sacc[j][1] = f32x16{};
      FA_PRIO_HI_(FA_MFMA_PRIO_FWD);
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const bf16x8 kf = ld16(&Kc[(st * 32 + lq) * KST + 16 * t + 8 * hh]);
#pragma unroll
          for (int j = 0; j < QPW; ++j) sacc[j][st] = mfma(kf, qf[j][t], sacc[j][st]);
        }
      FA_PRIO_LO_(FA_MFMA_PRIO_FWD);
    }
    // The other buffers were released by every wave at the last barrier.
    if (more) {
      kwrite(cur ^ 1);
      gload(vb, kt + 1);  // lands during this tile's softmax and O MFMAs
    }
    if (active) {
      const bf16_t* Vc = Vs + cur * VTILE;
      // Row max on the RAW scores (c > 0: max commutes with the scaling);
      // the scale is folded into the exponent's FMA below.  A sub-block
      // entirely above the diagonal is masked to -inf and contributes 0.
      const bool edge = (causal && k0 + BKV - 1 > q0) || (!EVEN && k0 + BKV > S);  // wave-uniform
      float m_use[QPW], alpha[QPW];
      bool moved = false;
#pragma unroll
      for (int j = 0; j < QPW; ++j) {
        const int qrow = q0 + 32 * j + lq;
        float mx = -INFINITY;
        if (edge) {
#pragma unroll
          for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int key = k0 + st * 32 + acc_row(r, hh);
              if ((!EVEN && key >= S) || (causal && key > qrow)) sacc[j][st][r] = -INFINITY;
              mx = fmaxf(mx, sacc[j][st][r]);
            }
        } else {
#pragma unroll
          for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[j][st][r]);
        }
        mx = xhalf_max(mx) * c;
        // FA_DEFER_T > 0: keep the running max until a tile's max exceeds it
        // by more than T (log2 units), so P stays <= 2^T and O is rescaled on
        // far fewer tiles (any of the wave's 32 rows moving triggers it).
        const float m_new = (FA_DEFER_T <= 0.f || mx > m[j] + FA_DEFER_T) ? fmaxf(m[j], mx) : m[j];
        m_use[j] = m_new == -INFINITY ? 0.f : m_new;
        moved |= m_new > m[j];
        alpha[j] = fast_exp2(m[j] - m_use[j]);
        m[j] = m_new;
      }
      // Rescale O only when some row's (deferred) max moved.
      if (__any(moved)) {
#pragma unroll
        for (int j = 0; j < QPW; ++j) {
          l[j] *= alpha[j];
#pragma unroll
          for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[j][db][r] *= alpha[j];
        }
      }
      // P = 2^(S c - m): one FMA + one v_exp per element, then bf16 pairs.
      u32x4 pb[QPW][4];
#pragma unroll
      for (int j = 0; j < QPW; ++j) {
        float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const float p0 = fast_exp2(fmaf(sacc[j][st][r], c, -m_use[j]));
            const float p1 = fast_exp2(fmaf(sacc[j][st][r + 1], c, -m_use[j]));
            rs0 += p0;
            rs1 += p1;
            pb[j][2 * st + (r >> 3)][(r & 7) >> 1] = pk_bf16(p0, p1);
          }
        const float rs = rs0 + rs1;
        l[j] += rs;  // this half-lane's 32 keys; the halves are summed once, at the end
      }
      // O^T += V^T P : P (key rows, query on lane) is the B operand as is; the
      // V^T fragment (d on the lane, the permuted key order of P on k) comes
      // from two hardware-transposed reads of the row-major V tile, at the
      // lane offsets precomputed in voff (+ a compile-time row offset); each
      // V^T fragment feeds QPW MFMAs.
      FA_PRIO_HI_(FA_MFMA_PRIO_FWD);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int st = s >> 1, sp = s & 1;
        const int rowc = 256 * (st * 32 + 16 * sp);
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const u16x4 lo = tr_read(Vc, voff[db][0] + rowc);
          const u16x4 hi = tr_read(Vc, voff[db][1] + rowc + 256 * 8);
          const bf16x8 vf = cat44(lo, hi);
#pragma unroll
          for (int j = 0; j < QPW; ++j) oacc[j][db] = mfma(vf, pk8(pb[j][s]), oacc[j][db]);
        }
      }
      FA_PRIO_LO_(FA_MFMA_PRIO_FWD);
    }
    if (more) vwrite(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < QPW; ++j) {
    const int qrow = q0 + 32 * j + lq;
    const float lt = xhalf_sum(l[j]);
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    store_row_t(o + (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD, oacc[j],
                inv, hh, EVEN || qrow < S);
    if (EVEN || qrow < S) {
      if (hh == 0)
        lse2[(static_cast<size_t>(b) * Hq + h) * S + qrow] = lt > 0.f ? m[j] + log2f(lt) : -INFINITY;
    }
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

constexpr int BQT = 32;               // query rows per backward step
// 8 waves (256 keys, one workgroup per CU) measured: full 1.930 -> 1.855 ms
// for the backward, but causal 1.131 -> 1.144 ms (coarser causal jobs): the
// training shape is causal, so 4.
#ifndef FA_DKDV_WAVES
#define FA_DKDV_WAVES 4
#endif
constexpr int KVW = FA_DKDV_WAVES;    // waves per dK/dV workgroup (32 keys each)
constexpr int KB = 32 * KVW;          // keys per dK/dV workgroup
constexpr int KVNT = 64 * KVW;        // threads per dK/dV workgroup
constexpr int QSTG = 8 / KVW;         // 16-B Q (and dO) chunks per thread per 32-row tile
static_assert(KVW == 4 || KVW == 8, "dK/dV workgroup: 4 or 8 waves");
constexpr int QTILE = BQT * HD;       // bf16 elements of one Q (or dO) image

// Backward LDS images use layout (a) of cdna_hip_programming.md T10: 8-row x
// 32-column subtiles of 512 B.  Row reads (ds_read_b128) and transposed reads
// (ds_read_b64_tr_b16) are both conflict-free as with (b), but the eight row
// reads (t = 0..7) and the sixteen transposed reads of one 32x32x16 operand
// differ only by immediate offsets from TWO base addresses each — the
// register-lean choice for kernels that sit at the 256-VGPR limit.
__device__ __forceinline__ int a_off(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// Lane-dependent parts of the layout-(a) addresses, computed once per kernel:
//   row read  (row R0 + lk, chunk 2t + hh), R0 % 8 == 0:
//       a_off = roff[t & 1] + 512 (t >> 1) + 256 R0
//   transposed read of rows base + tr_row (+8), chunks 4 db + tr_ch,
//   base % 16 == 0:  a_off + tr_byte = tro[0 or 1] + 256 base + 512 db
// so every LDS read in the inner loops is a base register + an immediate.
struct AOffs {
  int roff[2];
  int tro[2];
};

__device__ __forceinline__ AOffs make_aoffs(int lane) {
  const int lk = lane & 31, hh = lane >> 5;
  const int trG = lane >> 4, trq = (lane >> 2) & 3, trp = lane & 3;
  const int tr_row = 4 * (trG >> 1) + trq, tr_ch = 2 * (trG & 1) + (trp >> 1), tr_byte = 8 * (trp & 1);
  AOffs o;
  o.roff[0] = 2048 * (lk >> 3) + 64 * (lk & 7) + 16 * ((hh) ^ ((lk >> 2) & 3));
  o.roff[1] = 2048 * (lk >> 3) + 64 * (lk & 7) + 16 * ((2 + hh) ^ ((lk >> 2) & 3));
  o.tro[0] = 64 * tr_row + 16 * (tr_ch ^ ((tr_row >> 2) & 3)) + tr_byte;
  o.tro[1] = 2048 + 64 * tr_row + 16 * (tr_ch ^ (((8 + tr_row) >> 2) & 3)) + tr_byte;
  return o;
}

__device__ __forceinline__ bf16x8 row_rd(const bf16_t* img, const AOffs& o, int r0, int t) {
  return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(img) + o.roff[t & 1] +
                                          512 * (t >> 1) + 256 * r0);
}

__device__ __forceinline__ bf16x8 tr_rd(const bf16_t* img, const AOffs& o, int base, int db) {
  return cat44(tr_read(img, o.tro[0] + 256 * base + 512 * db),
               tr_read(img, o.tro[1] + 256 * base + 512 * db));
}

// dK, dV: one workgroup = 128 keys of one (b, kv head); wave = 32 keys.  Q and
// dO tiles (32 rows) are double-buffered in ONE layout-(b) image each: rows
// read with ds_read_b128 for S = Q K^T and dP = dO V^T, columns read with
// ds_read_b64_tr_b16 for dV^T += dO^T P and dK^T += Q^T dS — no transposed
// copy is written.  Loads of tile i+1 are issued before tile i's MFMAs and
// stored after them; one barrier per tile.
// Register budget: <= 256 per lane so two workgroups share a CU (2 waves per
// SIMD) — over it, hipcc parks the excess in AGPRs and moves it back and forth
// every iteration.  K stays in VGPRs, the WG's V tile is read from LDS.
template <bool EVEN>
__global__ __launch_bounds__(KVNT, KVW == 4 ? 2 : 1) void fa_bwd_dkdv_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2,
    const float* __restrict__ delta, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int S,
    int Hq, int Hkv, float c, float scale, int causal, int nKB, const int4* __restrict__ jobs,
    float* __restrict__ part, int B) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[2 * QTILE];
  __shared__ __attribute__((aligned(16))) bf16_t Ds[2 * QTILE];
  __shared__ __attribute__((aligned(16))) bf16_t Vw[KB * HD];  // this WG's KB keys
  __shared__ __attribute__((aligned(16))) float Ls[2 * BQT];
  __shared__ __attribute__((aligned(16))) float Dl[2 * BQT];
  const int G = Hq / Hkv;
  const int nqt = (S + BQT - 1) / BQT;
  int b, hkv, kb, it0, it1, slot;
  if (jobs) {
    // Planned job (kgwe_fa_bwd_plan): a key block, or one half of a heavy
    // causal key block's (query tile x head) sweep, in longest-first order
    // per XCD.  Half-jobs write fp32 partials that fa_bwd_dkdv_finalize sums.
    const int4 jb = jobs[blockIdx.x];
    if (jb.z >= jb.w) return;  // padding: the whole workgroup leaves before any barrier
    hkv = jb.x % Hkv;
    b = jb.x / Hkv;
    kb = jb.y & 0xffffff;
    slot = jb.y >> 24;
    it0 = jb.z;
    it1 = jb.w;
  } else {
    // Decode (b, hkv, key block): XCD-aware, heaviest (earliest keys) first.
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    kb = wg % nKB;
    hkv = (wg / nKB) % Hkv;
    b = wg / (nKB * Hkv);
    slot = 0;
    it0 = 0;
    it1 = G * (nqt - (causal ? (kb * KB) / BQT : 0));
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lk = lane & 31, hh = lane >> 5;
  const int key0 = kb * KB + w * 32;
  const int key = key0 + lk;
  const size_t qs = static_cast<size_t>(Hq) * HD, kvs = static_cast<size_t>(Hkv) * HD;
  bf16x8 kf[8];
  {
    const size_t off = (static_cast<size_t>(b) * S + key) * kvs + static_cast<size_t>(hkv) * HD;
#pragma unroll
    for (int t = 0; t < 8; ++t) kf[t] = (EVEN || key < S) ? ld16(k + off + 16 * t + 8 * hh) : bf16x8{};
    // V rows kb*128 .. +127 -> layout-(b) image (row reads only); published
    // by the barrier before the main loop.
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = (threadIdx.x >> 4) + 4 * KVW * i, ch = threadIdx.x & 15, s = kb * KB + r;
      const bf16x8 x = (EVEN || s < S) ? ld16(v + (static_cast<size_t>(b) * S + s) * kvs +
                                    static_cast<size_t>(hkv) * HD + ch * 8)
                             : bf16x8{};
      *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(Vw) + a_off(r, ch)) = x;
    }
  }
  const bf16_t* Vmine = Vw + w * 32 * HD;  // a_off: a 32-row slice is a whole number of subtiles
  f32x16 dka[4], dva[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dka[i] = dva[i] = f32x16{};

  const int total = it1 - it0;
  // Staging: thread t moves row chunks (r, ch) = ((t + KVNT i) >> 4, t & 15), i < QSTG.
  const int sr = threadIdx.x >> 4, sch = threadIdx.x & 15;
  bf16x8 qr[QSTG], dr[QSTG];
  float lr = 0.f, drl = 0.f;
  // Iteration it = (query tile nqt-1 - it/G, head g = it%G), tracked
  // incrementally (G is a runtime value: no per-iteration integer division).
  auto gload = [&](int g, int qt) {
    const int h = hkv * G + g;
#pragma unroll
    for (int i = 0; i < QSTG; ++i) {
      const int s = qt * BQT + sr + 4 * KVW * i;
      const size_t off = (static_cast<size_t>(b) * S + s) * qs + static_cast<size_t>(h) * HD + sch * 8;
      qr[i] = (EVEN || s < S) ? ld16(q + off) : bf16x8{};
      dr[i] = (EVEN || s < S) ? ld16(dout + off) : bf16x8{};
    }
    if (threadIdx.x < BQT) {
      const int s = qt * BQT + threadIdx.x;
      const size_t li = (static_cast<size_t>(b) * Hq + h) * S + s;
      lr = (EVEN || s < S) ? lse2[li] : INFINITY;
      drl = (EVEN || s < S) ? delta[li] : 0.f;
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < QSTG; ++i) {
      const int off = a_off(sr + 4 * KVW * i, sch);
      *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(Qs + buf * QTILE) + off) = qr[i];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(Ds + buf * QTILE) + off) = dr[i];
    }
    if (threadIdx.x < BQT) {
      Ls[buf * BQT + threadIdx.x] = lr;
      Dl[buf * BQT + threadIdx.x] = drl;
    }
  };
  const AOffs ao = make_aoffs(lane);
  // Iteration it = (query tile nqt-1 - it/G, head it%G), from it0.
  int qt = nqt - 1 - it0 / G, g_cur = it0 % G;
  if (total > 0) {
    gload(g_cur, qt);
    swrite(0);
  }
  // K fragments complete before the loop (see fa_fwd_kernel: otherwise the
  // loop's first MFMAs wait for the prefetch issued just above them).
#pragma unroll
  for (int t = 0; t < 8; ++t) asm volatile("" ::"v"(kf[t]));
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    // Query tiles from the LAST one down, heads innermost: every key block of
    // a (batch, kv head) — all resident on one XCD — reads the same Q / dO
    // tile at the same time (one L2 fill, not one per key block); a block
    // stops when the sweep passes its diagonal.
    const int g_nxt = g_cur + 1 == G ? 0 : g_cur + 1;
    const int qt_nxt = g_nxt == 0 ? qt - 1 : qt;
    if (it + 1 < total) gload(g_nxt, qt_nxt);
    const int qbase = qt * BQT;
    if (!causal || qbase + BQT - 1 >= key0) {  // else every query of this tile precedes our keys
      const bf16_t* Qc = Qs + cur * QTILE;
      const bf16_t* Dc = Ds + cur * QTILE;
      const float* Lc = Ls + cur * BQT;
      const float* Dlc = Dl + cur * BQT;
      // S[q][key] = Q K^T and dP[q][key] = dO V^T (key on the lane).  The dP
      // chain starts from -delta (the row constant as the initial
      // accumulator), so dS = P dP' needs no subtraction.
      f32x16 sa = f32x16{}, pa;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 del4 = *reinterpret_cast<const f32x4*>(Dlc + 8 * g4 + 4 * hh);
#pragma unroll
        for (int j = 0; j < 4; ++j) pa[4 * g4 + j] = -del4[j];
      }
      FA_PRIO_HI_(FA_MFMA_PRIO_BWD);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        sa = mfma(row_rd(Qc, ao, 0, t), kf[t], sa);
        pa = mfma(row_rd(Dc, ao, 0, t), row_rd(Vmine, ao, 0, t), pa);
      }
      FA_PRIO_LO_(FA_MFMA_PRIO_BWD);
      // P = exp2(S c - lse2), dS = P (dP - delta); row r <-> query qbase + acc_row(r).
      const bool edge = (causal && key0 + 31 > qbase) || (!EVEN && (qbase + BQT > S || key0 + 32 > S));
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        // accumulator rows 4*g4 .. +3 are queries 8*g4 + 4*hh + 0..3: one b128 read each
        const f32x4 lse4 = *reinterpret_cast<const f32x4*>(Lc + 8 * g4 + 4 * hh);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g4 + j;
          float p = fast_exp2(sa[r] * c - lse4[j]);
          if (edge) {
            const int qrow = qbase + acc_row(r, hh);
            if ((!EVEN && (key >= S || qrow >= S)) || (causal && key > qrow)) p = 0.f;
          }
          sa[r] = p;
          pa[r] = p * pa[r];
        }
      }
      // dV^T += dO^T P ; dK^T += Q^T dS   (P, dS as B operands, permuted q order)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        u32x4 pw, sw;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pw[j] = pk_bf16(sa[8 * s + 2 * j], sa[8 * s + 2 * j + 1]);
          sw[j] = pk_bf16(pa[8 * s + 2 * j], pa[8 * s + 2 * j + 1]);
        }
        const bf16x8 pb = pk8(pw), sb = pk8(sw);
        FA_PRIO_HI_(FA_MFMA_PRIO_BWD);
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          dva[db] = mfma(tr_rd(Dc, ao, 16 * s, db), pb, dva[db]);
          dka[db] = mfma(tr_rd(Qc, ao, 16 * s, db), sb, dka[db]);
        }
        FA_PRIO_LO_(FA_MFMA_PRIO_BWD);
      }
    }
    if (it + 1 < total) swrite(cur ^ 1);
    __syncthreads();
    qt = qt_nxt;
    g_cur = g_nxt;
  }
  if (slot > 0) {
    if (!(EVEN || key < S)) return;
    // fp32 partial [slot-1][dk|dv][b][hkv][key][d]
    const size_t plane = static_cast<size_t>(B) * Hkv * S * HD;
    float* pk = part + (static_cast<size_t>(slot - 1) * 2) * plane +
                ((static_cast<size_t>(b) * Hkv + hkv) * S + key) * HD;
    float* pv = pk + plane;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        f32x4 a, bb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = dka[db][4 * g4 + j];
          bb[j] = dva[db][4 * g4 + j];
        }
        *reinterpret_cast<f32x4*>(pk + db * 32 + 8 * g4 + 4 * hh) = a;
        *reinterpret_cast<f32x4*>(pv + db * 32 + 8 * g4 + 4 * hh) = bb;
      }
  } else {
    const size_t off = (static_cast<size_t>(b) * S + key) * kvs + static_cast<size_t>(hkv) * HD;
    store_row_t(dk + off, dka, scale, hh, EVEN || key < S);
    store_row_t(dv + off, dva, 1.f, hh, EVEN || key < S);
  }
}

// Sum the two fp32 halves of every split key block: dK (x scale) and dV to
// bf16.  One thread = 4 consecutive d of one key; keys [0, split_keys).
__global__ __launch_bounds__(256) void fa_bwd_dkdv_finalize(const float* __restrict__ part,
                                                            bf16_t* __restrict__ dk,
                                                            bf16_t* __restrict__ dv, int B, int S,
                                                            int Hkv, int split_keys, float scale) {
  const long long idx = static_cast<long long>(blockIdx.x) * 256 + threadIdx.x;
  const long long per_gh = static_cast<long long>(split_keys) * (HD / 4);
  if (idx >= per_gh * B * Hkv) return;
  const int gh = static_cast<int>(idx / per_gh);
  const int rem = static_cast<int>(idx % per_gh);
  const int key = rem / (HD / 4), d = 4 * (rem % (HD / 4));
  const size_t plane = static_cast<size_t>(B) * Hkv * S * HD;
  const size_t src = (static_cast<size_t>(gh) * S + key) * HD + d;
  const f32x4 k0 = *reinterpret_cast<const f32x4*>(part + src);
  const f32x4 v0 = *reinterpret_cast<const f32x4*>(part + plane + src);
  const f32x4 k1 = *reinterpret_cast<const f32x4*>(part + 2 * plane + src);
  const f32x4 v1 = *reinterpret_cast<const f32x4*>(part + 3 * plane + src);
  const int b = gh / Hkv, hkv = gh % Hkv;
  const size_t dst = ((static_cast<size_t>(b) * S + key) * Hkv + hkv) * HD + d;
  u16x4 ko, vo;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ko[j] = f2bf((k0[j] + k1[j]) * scale);
    vo[j] = f2bf(v0[j] + v1[j]);
  }
  *reinterpret_cast<u16x4*>(dk + dst) = ko;
  *reinterpret_cast<u16x4*>(dv + dst) = vo;
}

// dQ: one workgroup = 128 query rows of one (b, head); wave = 32 rows (the
// forward's geometry: query on the lane).  K and V tiles double-buffered in
// layout-(b) images: K rows for S^T = K Q^T and K columns (transposed reads)
// for dQ^T += K^T dS^T from the same image; V rows for dP^T = V dO^T.
template <bool EVEN>
__global__ __launch_bounds__(DQNT, DQW == 4 ? 2 : 1) void fa_bwd_dq_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse2, const bf16_t* __restrict__ o,
    float* __restrict__ delta, bf16_t* __restrict__ dq, int S, int Hq, int Hkv, float c,
    float scale, int causal, int nQB) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2 * VTILE];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2 * VTILE];
  int b, h, hkv, qb;
  decode(nQB, Hq / Hkv, Hkv, causal, &b, &h, &hkv, &qb);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int q0 = qb * BQ + w * 32;
  const int qrow = q0 + lq;
  const size_t qs = static_cast<size_t>(Hq) * HD, kvs = static_cast<size_t>(Hkv) * HD;
  bf16x8 qf[8], df[8];
  float dsum = 0.f;
  {
    const size_t off = (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      qf[t] = (EVEN || qrow < S) ? ld16(q + off + 16 * t + 8 * hh) : bf16x8{};
      df[t] = (EVEN || qrow < S) ? ld16(dout + off + 16 * t + 8 * hh) : bf16x8{};
    }
    if (FA_DQ_DELTA) {
      // delta = rowsum(dO * O) for this lane's row, computed here (each lane
      // pair holds the row's dO already) instead of by a separate pass; the
      // dK/dV kernel, launched after this one, reads it back.
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const bf16x8 ov = (EVEN || qrow < S) ? ld16(o + off + 16 * t + 8 * hh) : bf16x8{};
#pragma unroll
        for (int e = 0; e < 8; ++e) dsum = fmaf(bf2f(df[t][e]), bf2f(ov[e]), dsum);
      }
    }
  }
  const size_t li = (static_cast<size_t>(b) * Hq + h) * S + qrow;
  const float my_lse = (EVEN || qrow < S) ? lse2[li] : INFINITY;
  float my_delta;
  if (FA_DQ_DELTA) {
    my_delta = xhalf_sum(dsum);
    if (hh == 0 && (EVEN || qrow < S)) delta[li] = my_delta;
  } else {
    my_delta = (EVEN || qrow < S) ? delta[li] : 0.f;
  }
  f32x16 dqa[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dqa[i] = f32x16{};
  const int kv_end = causal ? min(S, qb * BQ + BQ) : S;
  const int ntiles = (kv_end + BKV - 1) / BKV;
  const bf16_t* kb_ = k + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  const bf16_t* vb_ = v + static_cast<size_t>(b) * S * kvs + static_cast<size_t>(hkv) * HD;
  // Staging: thread t moves chunks (key, ch) = ((t + DQNT i) >> 4, t & 15), i < DQSTG.
  const int skey = threadIdx.x >> 4, sch = threadIdx.x & 15;
  bf16x8 kr[DQSTG], vr[DQSTG];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < DQSTG; ++i) {
      const int s = kt * BKV + skey + 4 * DQW * i;
      kr[i] = (EVEN || s < S) ? ld16(kb_ + static_cast<size_t>(s) * kvs + sch * 8) : bf16x8{};
      vr[i] = (EVEN || s < S) ? ld16(vb_ + static_cast<size_t>(s) * kvs + sch * 8) : bf16x8{};
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < DQSTG; ++i) {
      const int off = a_off(skey + 4 * DQW * i, sch);
      *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(Ks + buf * VTILE) + off) = kr[i];
      *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(Vs + buf * VTILE) + off) = vr[i];
    }
  };
  const AOffs ao = make_aoffs(lane);
  gload(0);
  swrite(0);
  // Q / dO fragments and row constants complete before the loop (see
  // fa_fwd_kernel).
#pragma unroll
  for (int t = 0; t < 8; ++t) asm volatile("" ::"v"(qf[t]), "v"(df[t]));
  asm volatile("" ::"v"(my_lse), "v"(my_delta));
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ntiles) gload(kt + 1);
    const int k0 = kt * BKV;
    if (!causal || k0 <= q0 + 31) {
      const bf16_t* Kc = Ks + cur * VTILE;
      const bf16_t* Vc = Vs + cur * VTILE;
      const bool edge = (causal && k0 + BKV - 1 > q0) || (!EVEN && (k0 + BKV > S || q0 + 32 > S));
      // Two 32-key halves in sequence: one S^T / dP^T accumulator pair live
      // at a time keeps the kernel inside 256 VGPRs.
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        // dP^T starts from -delta (query on the lane: one constant per lane)
        f32x16 sa = f32x16{}, pa;
#pragma unroll
        for (int r = 0; r < 16; ++r) pa[r] = -my_delta;
        FA_PRIO_HI_(FA_MFMA_PRIO_BWD);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          sa = mfma(row_rd(Kc, ao, st * 32, t), qf[t], sa);
          pa = mfma(row_rd(Vc, ao, st * 32, t), df[t], pa);
        }
        FA_PRIO_LO_(FA_MFMA_PRIO_BWD);
        auto softmax = [&](auto masked) {  // unmasked copy for full tiles (see dK/dV)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float p = fast_exp2(sa[r] * c - my_lse);
            if (decltype(masked)::value) {
              const int kk = k0 + st * 32 + acc_row(r, hh);
              if ((!EVEN && (kk >= S || qrow >= S)) || (causal && kk > qrow)) p = 0.f;
            }
            pa[r] = p * pa[r];  // dS^T
          }
        };
        if (edge) softmax(std::true_type{});
        else softmax(std::false_type{});
        // dQ^T += K^T dS^T
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          u32x4 sw;
#pragma unroll
          for (int j = 0; j < 4; ++j) sw[j] = pk_bf16(pa[8 * sp + 2 * j], pa[8 * sp + 2 * j + 1]);
          const bf16x8 sb = pk8(sw);
          FA_PRIO_HI_(FA_MFMA_PRIO_BWD);
#pragma unroll
          for (int db = 0; db < 4; ++db)
            dqa[db] = mfma(tr_rd(Kc, ao, st * 32 + 16 * sp, db), sb, dqa[db]);
          FA_PRIO_LO_(FA_MFMA_PRIO_BWD);
        }
      }
    }
    if (kt + 1 < ntiles) swrite(cur ^ 1);
    __syncthreads();
  }
  store_row_t(dq + (static_cast<size_t>(b) * S + qrow) * qs + static_cast<size_t>(h) * HD, dqa, scale,
              hh, EVEN || qrow < S);
}

}  // namespace

// ---------------------------------------------------------------------------
// dK/dV job plan (host).  Causal key blocks carry very different work: block
// kb sweeps G x (nqt - 4 kb) query tiles, so at S = 4096 the first block does
// 32x the last.  One workgroup per block left ~half the CU slots idle at the
// end (fa_bwd_dkdv ran at ~22 % MFMA busy, profiles/r01_attn_counters): the
// plan splits every block heavier than the average slot load into two halves
// (fp32 partials, summed by fa_bwd_dkdv_finalize) and orders each XCD's jobs
// longest-first (LPT), with all blocks of one (batch, kv head) on one XCD so
// they share its L2 copy of Q / dO.
// ---------------------------------------------------------------------------
namespace {

struct BwdPlan {
  int4* jobs = nullptr;  // device, grid entries
  int grid = 0;
  int split_keys = 0;    // keys [0, split_keys) of every (b, hkv) are split
};

BwdPlan make_plan(int B, int S, int Hq, int Hkv, int causal, int num_cus) {
  BwdPlan p;
  constexpr int kblk = KB;  // keys per fa_bwd_dkdv_kernel workgroup
  const int G = Hq / Hkv, nqt = (S + BQT - 1) / BQT, nKB = (S + kblk - 1) / kblk;
  const int groups = B * Hkv;
  auto work = [&](int kb) { return G * (nqt - (causal ? (kb * kblk) / BQT : 0)); };
  double total = 0;
  for (int kb = 0; kb < nKB; ++kb) total += static_cast<double>(work(kb)) * groups;
  const double avg = total / ((KVW == 4 ? 2.0 : 1.0) * num_cus);  // dK/dV workgroups per CU
  struct J { int4 j; int w; };
  std::vector<std::vector<J>> per_xcd(8);
  int nsplit = 0;
  for (int kb = 0; kb < nKB; ++kb) {
    const int w = work(kb);
    const bool split = causal && w > avg && w >= 2 * G;
    if (split) nsplit = kb + 1;
    for (int gid = 0; gid < groups; ++gid) {
      auto& L = per_xcd[gid % 8];
      if (split) {
        const int h = w / 2;
        L.push_back({make_int4(gid, kb | (1 << 24), 0, h), h});
        L.push_back({make_int4(gid, kb | (2 << 24), h, w), w - h});
      } else {
        L.push_back({make_int4(gid, kb, 0, w), w});
      }
    }
  }
  size_t len = 0;
  for (auto& L : per_xcd) {
    std::stable_sort(L.begin(), L.end(), [](const J& a, const J& b) { return a.w > b.w; });
    len = std::max(len, L.size());
  }
  std::vector<int4> table(8 * len, make_int4(0, 0, 0, 0));  // padding: empty range
  for (size_t i = 0; i < table.size(); ++i) {
    const auto& L = per_xcd[i % 8];  // workgroup i is dispatched to XCD i % 8
    if (i / 8 < L.size()) table[i] = L[i / 8].j;
  }
  if (hipMalloc(&p.jobs, table.size() * sizeof(int4)) != hipSuccess) return BwdPlan{};
  if (hipMemcpy(p.jobs, table.data(), table.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(p.jobs);
    return BwdPlan{};
  }
  p.grid = static_cast<int>(table.size());
  p.split_keys = std::min(S, nsplit * kblk);
  return p;
}

// One plan per (device, shape), built on first use outside stream capture.
const BwdPlan* get_plan(int B, int S, int Hq, int Hkv, int causal, hipStream_t s) {
  static std::mutex mu;
  static std::map<std::array<int, 6>, BwdPlan> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const std::array<int, 6> key{dev, B, S, Hq, Hkv, causal};
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second.jobs ? &it->second : nullptr;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  BwdPlan p = make_plan(B, S, Hq, Hkv, causal, cus);
  auto& slot = cache[key] = p;
  return slot.jobs ? &slot : nullptr;
}

}  // namespace

KGWE_API int64_t kgwe_flash_attn_bwd_workspace(int B, int S, int Hq, int Hkv, int D) {
  // delta, then the dK/dV halves' fp32 partials [2 halves][dk|dv][B][Hkv][S][D]
  return static_cast<int64_t>(B) * Hq * S * sizeof(float) +
         static_cast<int64_t>(4) * B * Hkv * S * HD * sizeof(float);
}

// lse2 from the forward (log2 units).  `work` >= workspace bytes.
KGWE_API int kgwe_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                                 const float* lse2, const void* dout, void* dq, void* dk, void* dv,
                                 float* work, void* /*reserved*/, int B, int S, int Hq, int Hkv,
                                 int D, float scale, int causal, hipStream_t s) {
  if (D != HD || Hq % Hkv != 0 || B <= 0 || S <= 0) return -1;
  const float c = scale * 1.4426950408889634f;
  const long long rows = static_cast<long long>(B) * S * Hq;
  int rc = 0;
  if (!FA_DQ_DELTA) {
    hipLaunchKernelGGL(fa_bwd_pre_kernel, dim3(static_cast<unsigned>((rows * 16 + 255) / 256)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(o), static_cast<const bf16_t*>(dout), work, B, S, Hq);
    rc = KGWE_CHECK_LAUNCH();
    if (rc) return rc;
  }
  const int nKB = (S + KB - 1) / KB;
  const int nQB = (S + BQ - 1) / BQ;
  const bf16_t *Q = static_cast<const bf16_t*>(q), *Kp = static_cast<const bf16_t*>(k),
               *V = static_cast<const bf16_t*>(v), *DO = static_cast<const bf16_t*>(dout),
               *O = static_cast<const bf16_t*>(o);
  // dQ first: with FA_DQ_DELTA it also writes delta = rowsum(dO * O), which
  // the dK/dV kernel reads.
  if (S % 256 == 0) {
    hipLaunchKernelGGL(fa_bwd_dq_kernel<true>, dim3(static_cast<unsigned>(B * Hq * nQB)), dim3(DQNT), 0, s,
                       Q, Kp, V, DO, lse2, O, work, static_cast<bf16_t*>(dq), S, Hq, Hkv, c, scale, causal,
                       nQB);
  } else {
    hipLaunchKernelGGL(fa_bwd_dq_kernel<false>, dim3(static_cast<unsigned>(B * Hq * nQB)), dim3(DQNT), 0, s,
                       Q, Kp, V, DO, lse2, O, work, static_cast<bf16_t*>(dq), S, Hq, Hkv, c, scale, causal,
                       nQB);
  }
  rc = KGWE_CHECK_LAUNCH();
  if (rc) return rc;
  // Planned dK/dV jobs (balanced causal sweep); the analytic one-block-per-
  // workgroup grid when no plan can be built (first call inside a capture).
  const BwdPlan* plan = get_plan(B, S, Hq, Hkv, causal, s);  // null: analytic grid
  float* part = work + static_cast<size_t>(B) * Hq * S;
  const int4* jobs = plan ? plan->jobs : nullptr;
  const unsigned dkdv_grid = plan ? static_cast<unsigned>(plan->grid) : static_cast<unsigned>(B * Hkv * nKB);
  // EVEN: every tile is full (no per-row bounds checks in the inner loops).
  if (S % 256 == 0) {
    hipLaunchKernelGGL(fa_bwd_dkdv_kernel<true>, dim3(dkdv_grid), dim3(KVNT), 0,
                       s, Q, Kp, V, DO, lse2, work, static_cast<bf16_t*>(dk), static_cast<bf16_t*>(dv),
                       S, Hq, Hkv, c, scale, causal, nKB, jobs, part, B);
  } else {
    hipLaunchKernelGGL(fa_bwd_dkdv_kernel<false>, dim3(dkdv_grid), dim3(KVNT), 0,
                       s, Q, Kp, V, DO, lse2, work, static_cast<bf16_t*>(dk), static_cast<bf16_t*>(dv),
                       S, Hq, Hkv, c, scale, causal, nKB, jobs, part, B);
  }
  rc = KGWE_CHECK_LAUNCH();
  if (rc) return rc;
  if (plan && plan->split_keys > 0) {
    const long long n = static_cast<long long>(B) * Hkv * plan->split_keys * (HD / 4);
    hipLaunchKernelGGL(fa_bwd_dkdv_finalize, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s,
                       part, static_cast<bf16_t*>(dk), static_cast<bf16_t*>(dv), B, S, Hkv, plan->split_keys,
                       scale);
  }
  return KGWE_CHECK_LAUNCH();
}

KGWE_API int kgwe_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse2,
                                 int B, int S, int Hq, int Hkv, int D, float scale, int causal,
                                 hipStream_t s) {
  if (D != HD || Hq % Hkv != 0 || B <= 0 || S <= 0) return -1;
  const float c = scale * 1.4426950408889634f;  // softmax in the exp2 domain
  const int nQB = (S + BQF - 1) / BQF;
  const long long grid = static_cast<long long>(B) * Hq * nQB;
  if (grid > 0x7fffffff) return -1;
  if (S % 256 == 0)
    hipLaunchKernelGGL(fa_fwd_kernel<true>, dim3(static_cast<unsigned>(grid)), dim3(FNT), 0, s,
                       static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k),
                       static_cast<const bf16_t*>(v), static_cast<bf16_t*>(o), lse2, S, Hq, Hkv, c,
                       causal, nQB);
  else
    hipLaunchKernelGGL(fa_fwd_kernel<false>, dim3(static_cast<unsigned>(grid)), dim3(FNT), 0, s,
                       static_cast<const bf16_t*>(q), static_cast<const bf16_t*>(k),
                       static_cast<const bf16_t*>(v), static_cast<bf16_t*>(o), lse2, S, Hq, Hkv, c,
                       causal, nQB);
  return KGWE_CHECK_LAUNCH();
}
