// Fused (residual-add +) RMSNorm forward / backward for gfx950.
//
// Layout: rows of H bf16 elements, one 64-lane wave per row, 8 bf16 (16 B)
// per lane per vector, H/512 vectors cached in registers so every row is read
// from HBM exactly once per pass.  Four waves per 256-thread workgroup.
//
//   fwd:  h = x (+ res)            (written back when h_out != nullptr)
//         rstd = 1/sqrt(mean(h^2) + eps)
//         y = h * rstd * w
//   bwd:  g  = dy * w
//         dx = rstd * (g - h * rstd^2 * mean(g * h)) (+ dadd)
//         dw = sum_rows(dy * h * rstd)   — per-wave fp32 sums in LDS, reduced
//              per workgroup, then fp32 atomics into one [H] accumulator.
//
// Used by every Llama block (attention_norm / ffn_norm / final norm); fusing
// the residual add saves one full HBM round-trip of the hidden state.
#include "common.h"

using namespace kgwe;

namespace {

// Rows are cached in registers as raw bf16x8 (4 VGPRs per 8 elements) and
// widened on use: H = 4096 keeps 32 VGPRs of row data per lane.
template <int NV>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
    const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
    bf16_t* __restrict__ h_out, float* __restrict__ rstd_out, int T, int H,
    float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const size_t base = static_cast<size_t>(row) * H;
  bf16x8 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i)
    v[i] = *reinterpret_cast<const bf16x8*>(x + base + (i * kWave + lane) * 8);
  if (res) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * kWave + lane) * 8;
      bf16x8 r = *reinterpret_cast<const bf16x8*>(res + base + col);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = f2bf(bf2f(v[i][j]) + bf2f(r[j]));
      if (h_out) *reinterpret_cast<bf16x8*>(h_out + base + col) = v[i];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = bf2f(v[i][j]);
      ss += f * f;
    }
  ss = wave_sum(ss);
  const float rstd = rsqrtf(ss / static_cast<float>(H) + eps);
  if (lane == 0) rstd_out[row] = rstd;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int col = (i * kWave + lane) * 8;
    const bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + col);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[i][j]) * rstd * bf2f(wv[j]));
    *reinterpret_cast<bf16x8*>(y + base + col) = o;
  }
}

// Grid: G workgroups of 4 waves; waves stride over rows.  Each workgroup adds
// its dw contribution into the fp32 accumulator `partial[H]`.
template <int NV>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
    const bf16_t* __restrict__ w, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ dadd, bf16_t* __restrict__ dx,
    float* __restrict__ partial, int T, int H) {
  // [4][H] fp32: each wave accumulates its rows' dw contribution in its own
  // LDS row (lane-private columns, so no intra-wave sync), keeping VGPRs for
  // the two cached input rows (dy, h).
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  float* acc = lds + wid * H;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    f32x4* a = reinterpret_cast<f32x4*>(acc + (i * kWave + lane) * 8);
    a[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    a[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float invH = 1.f / static_cast<float>(H);
  for (int row = blockIdx.x * 4 + wid; row < T; row += nwaves) {
    const size_t base = static_cast<size_t>(row) * H;
    const float rstd = rstd_in[row];
    // Pass 1: dot = sum(dy*w*h) and the dw contribution.  Pass 2 re-reads the
    // row (L2-hot: 16 KB per wave just touched) instead of caching it in
    // VGPRs, which keeps the kernel at high occupancy for any H.
    float dot = 0.f;
#pragma unroll 4
    for (int i = 0; i < NV; ++i) {
      const int col = (i * kWave + lane) * 8;
      const bf16x8 d = *reinterpret_cast<const bf16x8*>(dy + base + col);
      const bf16x8 hv = *reinterpret_cast<const bf16x8*>(h + base + col);
      const bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + col);
      f32x4* a = reinterpret_cast<f32x4*>(acc + col);
      f32x4 a0 = a[0], a1 = a[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a0[j] += bf2f(d[j]) * bf2f(hv[j]) * rstd;
        a1[j] += bf2f(d[j + 4]) * bf2f(hv[j + 4]) * rstd;
      }
      a[0] = a0;
      a[1] = a1;
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += bf2f(d[j]) * bf2f(wv[j]) * bf2f(hv[j]);
    }
    dot = wave_sum(dot) * invH;
    const float c = rstd * rstd * dot;
#pragma unroll 4
    for (int i = 0; i < NV; ++i) {
      const int col = (i * kWave + lane) * 8;
      const bf16x8 d = *reinterpret_cast<const bf16x8*>(dy + base + col);
      const bf16x8 hv = *reinterpret_cast<const bf16x8*>(h + base + col);
      const bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + col);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = rstd * (bf2f(d[j]) * bf2f(wv[j]) - bf2f(hv[j]) * c);
      if (dadd) {
        float a[8];
        load8(dadd + base + col, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += a[j];
      }
      store8(dx + base + col, o);
    }
  }
  __syncthreads();
  // Reduce the 4 waves' rows in LDS, then one no-return fp32 atomic per
  // column per workgroup into dw_acc[H] (zeroed by the launcher): G x H adds
  // of 4 B = ~8 MB at the ~1.3 TB/s chip atomic rate, instead of a serial
  // column-sum pass over a [G, H] partial buffer.
  for (int c4 = threadIdx.x; c4 < H / 4; c4 += 256) {
    f32x4 s = reinterpret_cast<f32x4*>(lds)[c4];
#pragma unroll
    for (int k = 1; k < 4; ++k) s += reinterpret_cast<f32x4*>(lds + k * H)[c4];
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAdd(partial + c4 * 4 + j, s[j]);
  }
}

// dw = dw_acc cast to the parameter dtype.
__global__ __launch_bounds__(256) void dw_cast_kernel(
    const float* __restrict__ acc, int H, bf16_t* __restrict__ out_bf,
    float* __restrict__ out_f32) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= H) return;
  const float s = acc[c];
  if (out_f32) out_f32[c] = s;
  if (out_bf) out_bf[c] = f2bf(s);
}

template <int NV>
int launch_fwd(const bf16_t* x, const bf16_t* res, const bf16_t* w, bf16_t* y,
               bf16_t* h_out, float* rstd, int T, int H, float eps,
               hipStream_t s) {
  hipLaunchKernelGGL(rmsnorm_fwd_kernel<NV>, dim3((T + 3) / 4), dim3(256), 0, s,
                     x, res, w, y, h_out, rstd, T, H, eps);
  return KGWE_CHECK_LAUNCH();
}

template <int NV>
int launch_bwd(const bf16_t* dy, const bf16_t* h, const bf16_t* w,
               const float* rstd, const bf16_t* dadd, bf16_t* dx,
               float* partial, int G, int T, int H, hipStream_t s) {
  hipLaunchKernelGGL(rmsnorm_bwd_kernel<NV>, dim3(G), dim3(256),
                     4 * H * sizeof(float), s, dy, h, w, rstd, dadd, dx,
                     partial, T, H);
  return KGWE_CHECK_LAUNCH();
}

}  // namespace

// Workgroups of the backward (rows are strided over them); the caller's
// `partial` buffer only needs H floats (fp32 dw accumulator).
KGWE_API int kgwe_rmsnorm_bwd_grid(int T) {
  int g = (T + 3) / 4;
  return g < 512 ? (g < 1 ? 1 : g) : 512;
}

// Returns 0 on success, -1 for an unsupported H (must be 512 * {1,2,4,8,16}).
KGWE_API int kgwe_rmsnorm_fwd(const void* x, const void* res, const void* w,
                              void* y, void* h_out, float* rstd, int T, int H,
                              float eps, hipStream_t s) {
  auto X = static_cast<const bf16_t*>(x);
  auto R = static_cast<const bf16_t*>(res);
  auto W = static_cast<const bf16_t*>(w);
  auto Y = static_cast<bf16_t*>(y);
  auto HO = static_cast<bf16_t*>(h_out);
  switch (H) {
    case 512: return launch_fwd<1>(X, R, W, Y, HO, rstd, T, H, eps, s);
    case 1024: return launch_fwd<2>(X, R, W, Y, HO, rstd, T, H, eps, s);
    case 2048: return launch_fwd<4>(X, R, W, Y, HO, rstd, T, H, eps, s);
    case 4096: return launch_fwd<8>(X, R, W, Y, HO, rstd, T, H, eps, s);
    case 8192: return launch_fwd<16>(X, R, W, Y, HO, rstd, T, H, eps, s);
    default: return -1;
  }
}

KGWE_API int kgwe_rmsnorm_bwd(const void* dy, const void* h, const void* w,
                              const float* rstd, const void* dadd, void* dx,
                              float* partial, void* dw_bf16, float* dw_f32,
                              int T, int H, hipStream_t s) {
  const int G = kgwe_rmsnorm_bwd_grid(T);
  auto DY = static_cast<const bf16_t*>(dy);
  auto Hh = static_cast<const bf16_t*>(h);
  auto W = static_cast<const bf16_t*>(w);
  auto DA = static_cast<const bf16_t*>(dadd);
  auto DX = static_cast<bf16_t*>(dx);
  // `partial` is the fp32 dw accumulator, at least H floats.
  if (hipMemsetAsync(partial, 0, static_cast<size_t>(H) * sizeof(float), s) != hipSuccess) return -2;
  int rc;
  switch (H) {
    case 512: rc = launch_bwd<1>(DY, Hh, W, rstd, DA, DX, partial, G, T, H, s); break;
    case 1024: rc = launch_bwd<2>(DY, Hh, W, rstd, DA, DX, partial, G, T, H, s); break;
    case 2048: rc = launch_bwd<4>(DY, Hh, W, rstd, DA, DX, partial, G, T, H, s); break;
    case 4096: rc = launch_bwd<8>(DY, Hh, W, rstd, DA, DX, partial, G, T, H, s); break;
    case 8192: rc = launch_bwd<16>(DY, Hh, W, rstd, DA, DX, partial, G, T, H, s); break;
    default: return -1;
  }
  if (rc) return rc;
  hipLaunchKernelGGL(dw_cast_kernel, dim3((H + 255) / 256), dim3(256), 0, s,
                     partial, H, static_cast<bf16_t*>(dw_bf16), dw_f32);
  return KGWE_CHECK_LAUNCH();
}
