// Shared helpers for the kgwe gfx950 (CDNA4, MI355X) kernels.
//
// Every kernel in native/ops is written for 64-lane wavefronts and 16-byte
// vector memory accesses (bf16x8 per lane).  Launchers are exported with a
// plain C ABI (extern "C") and take raw device pointers plus the caller's
// hipStream_t, so PyTorch (ctypes, torch.cuda.current_stream()) and the C++
// runtime can both drive them, and hipGraph capture works unchanged.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define KGWE_API extern "C" __attribute__((visibility("default")))

namespace kgwe {

constexpr int kWave = 64;  // CDNA wavefront width; never 32.

typedef unsigned short bf16_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(8))) unsigned short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<unsigned int>(v) << 16);
}

// Round-to-nearest-even via the hardware convert (v_cvt_pk_bf16_f32 on gfx950),
// which also keeps NaNs NaN (MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

__device__ __forceinline__ void load8(const bf16_t* p, float (&out)[8]) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = bf2f(v[i]);
}

__device__ __forceinline__ void store8(bf16_t* p, const float (&in)[8]) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = f2bf(in[i]);
  *reinterpret_cast<bf16x8*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): consecutive logical tiles land on the same
// XCD so they share its L2.  Pure performance mapping — correctness never
// depends on it.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

}  // namespace kgwe

#define KGWE_CHECK_LAUNCH() (static_cast<int>(hipGetLastError()))
