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
//         dw = sum_rows(dy * h * rstd)   — per-lane fp32 sums in registers,
//              reduced per workgroup, then fp32 atomics into one [H] accumulator.
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

// Grid: G workgroups of 4 waves; workgroups stride over rows, and the 4
// waves of a workgroup split each row's columns (wave w owns the NV/4 16-B
// vectors w, w+4, ... of every lane-slot), so a lane holds only NV/4 vectors
// of dy and of h (cached in registers: each byte is read from HBM once) and
// 2*NV fp32 dw partial sums — few enough registers for 8 waves per SIMD,
// which is what hides HBM latency in this kernel.  The row's dot product is
// combined across the 4 waves through a double-buffered LDS word per wave
// (one barrier per row).  At the end each workgroup adds its dw partial sums
// with one no-return fp32 atomic per column into partial[H] (G x H x 4 B).
template <int NV>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
    const bf16_t* __restrict__ w, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ dadd, bf16_t* __restrict__ dx,
    float* __restrict__ partial, int T, int H) {
  constexpr int NW = NV >= 4 ? NV / 4 : 1;  // vectors per lane per row
  __shared__ float dots[2][4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const bool active = NV >= 4 || wid < NV;  // H = 512 / 1024: fewer vectors than waves
  float dw[NW][8];
#pragma unroll
  for (int i = 0; i < NW; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) dw[i][j] = 0.f;
  const float invH = 1.f / static_cast<float>(H);
  int parity = 0;
  // Rows are software-pipelined: the next row's dy / h (and this row's
  // residual gradient) are issued before the row's block reduction, so their
  // latency hides behind the barrier and the output pass instead of opening
  // each row: 114 -> 108.5 us at T=16384, H=4096 (tools/rmsnorm_ab.hip).
  bf16x8 d[NW], hv[NW];
  if (active && static_cast<int>(blockIdx.x) < T) {
    const size_t base0 = static_cast<size_t>(blockIdx.x) * H;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int col = ((i * 4 + wid) * kWave + lane) * 8;
      d[i] = *reinterpret_cast<const bf16x8*>(dy + base0 + col);
      hv[i] = *reinterpret_cast<const bf16x8*>(h + base0 + col);
    }
  }
  for (int row = blockIdx.x; row < T; row += gridDim.x, parity ^= 1) {
    const size_t base = static_cast<size_t>(row) * H;
    const float rstd = rstd_in[row];
    const int nrow = row + gridDim.x;
    const size_t nbase = static_cast<size_t>(nrow) * H;
    bf16x8 dn[NW], hn[NW], av[NW];
    float dot = 0.f;
    if (active) {
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const int col = ((i * 4 + wid) * kWave + lane) * 8;
        if (dadd) av[i] = *reinterpret_cast<const bf16x8*>(dadd + base + col);
        if (nrow < T) {
          dn[i] = *reinterpret_cast<const bf16x8*>(dy + nbase + col);
          hn[i] = *reinterpret_cast<const bf16x8*>(h + nbase + col);
        }
      }
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + ((i * 4 + wid) * kWave + lane) * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) dot += bf2f(d[i][j]) * bf2f(wv[j]) * bf2f(hv[i][j]);
      }
      dot = wave_sum(dot);
    }
    if (lane == 0) dots[parity][wid] = dot;
    __syncthreads();  // the other parity slot is rewritten only after the next barrier
    dot = (dots[parity][0] + dots[parity][1] + dots[parity][2] + dots[parity][3]) * invH;
    if (!active) continue;
    const float c = rstd * rstd * dot;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const int col = ((i * 4 + wid) * kWave + lane) * 8;
      const bf16x8 wv = *reinterpret_cast<const bf16x8*>(w + col);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float df = bf2f(d[i][j]), hf = bf2f(hv[i][j]);
        dw[i][j] += df * hf * rstd;
        o[j] = rstd * (df * bf2f(wv[j]) - hf * c);
        if (dadd) o[j] += bf2f(av[i][j]);
      }
      store8(dx + base + col, o);
    }
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      d[i] = dn[i];
      hv[i] = hn[i];
    }
  }
  // Stage the workgroup's dw row in LDS, then add it with atomics whose 64
  // lanes cover 256 contiguous bytes (the full-rate atomic shape; lanes 32 B
  // apart run ~8x slower: MI355X_MICROARCH.md, global float atomics).
  extern __shared__ float red[];  // H floats
  if (active) {
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      f32x4* r = reinterpret_cast<f32x4*>(red + ((i * 4 + wid) * kWave + lane) * 8);
      r[0] = f32x4{dw[i][0], dw[i][1], dw[i][2], dw[i][3]};
      r[1] = f32x4{dw[i][4], dw[i][5], dw[i][6], dw[i][7]};
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += 256) atomicAdd(partial + c, red[c]);
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
  hipLaunchKernelGGL(rmsnorm_bwd_kernel<NV>, dim3(G), dim3(256), H * sizeof(float), s, dy, h, w,
                     rstd, dadd, dx, partial, T, H);
  return KGWE_CHECK_LAUNCH();
}

}  // namespace

// Workgroups of the backward (rows are strided over them); the caller's
// `partial` buffer only needs H floats (fp32 dw accumulator).
KGWE_API int kgwe_rmsnorm_bwd_grid(int T) {
  return T < 1024 ? (T < 1 ? 1 : T) : 1024;  // 4 workgroups (16 waves) per CU
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

namespace {
__global__ void zero_f32_kernel(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.0f;
}
}  // namespace

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
  // Cleared by a kernel, not hipMemsetAsync: memset nodes recorded into a
  // captured graph have replayed wrongly on this platform.
  hipLaunchKernelGGL(zero_f32_kernel, dim3((H + 255) / 256), dim3(256), 0, s, partial, H);
  if (KGWE_CHECK_LAUNCH()) return -2;
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
