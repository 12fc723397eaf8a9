// Hardware bandwidth probes for topology discovery (gfx950 / MI355X).
//
// These replace the static per-link numbers an NVML backend would report
// (reference: src/discovery/types.go:134-146 NVLinkInfo.BandwidthGBps and
// types.go:72-73 GPUMemory.BandwidthGBps) with MEASURED numbers:
//
//   * HBM self-probe: copy / read / write streams over a buffer far larger
//     than the 256 MiB Infinity Cache, 16 B per lane, grid sized to >>256
//     CUs.  A GPU whose HBM rate falls well below the fleet median is
//     reported Degraded by the node agent.
//   * xGMI peer probe: the destination GPU pulls from a peer's HBM through
//     LDS — each wave issues 16-byte global_load_lds (LDS-DMA, no VGPR
//     round-trip) from the peer buffer into its LDS slot, then writes the
//     slot to local HBM with ds_read_b128 + global_store_dwordx4.  Pairwise
//     (one link) and all-peers-at-once (every one of the 7 links of a
//     device) modes.
//
// Plain C ABI, no torch dependency: the node agent and the C++ core can load
// this library on a box with no Python stack.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define KGWE_API extern "C" __attribute__((visibility("default")))
#define HIPOK(x)                                \
  do {                                          \
    hipError_t e_ = (x);                        \
    if (e_ != hipSuccess) return -static_cast<int>(e_) - 1000; \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

namespace {

constexpr int kThreads = 256;

// Streaming kernels: each thread keeps U 16-B vectors in flight (all U loads
// issued before the first store), a workgroup covers U * 256 consecutive
// vectors per step, and the grid strides over the buffer.  One vector per
// thread per step (U = 1) left HBM at ~5.3 TB/s of copy traffic: too few
// bytes in flight per CU to cover the miss latency.  Stores are nontemporal:
// the destination is never re-read, so it should not evict the source from
// the Infinity Cache / L2.
constexpr int kU = 4;

__global__ __launch_bounds__(kThreads) void copy_kernel(const u32x4* __restrict__ src,
                                                        u32x4* __restrict__ dst,
                                                        int64_t n) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads * kU;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads * kU + threadIdx.x;
  for (; i + (kU - 1) * kThreads < n; i += step) {
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = __builtin_nontemporal_load(src + i + u * kThreads);
#pragma unroll
    for (int u = 0; u < kU; ++u) __builtin_nontemporal_store(v[u], dst + i + u * kThreads);
  }
  for (int u = 0; u < kU; ++u)  // ragged tail of the last step
    if (i + u * kThreads < n) dst[i + u * kThreads] = src[i + u * kThreads];
}

__global__ __launch_bounds__(kThreads) void read_kernel(const u32x4* __restrict__ src,
                                                        int64_t n,
                                                        unsigned* __restrict__ sink) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads * kU;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads * kU + threadIdx.x;
  unsigned acc = 0;
  for (; i + (kU - 1) * kThreads < n; i += step) {
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = __builtin_nontemporal_load(src + i + u * kThreads);
#pragma unroll
    for (int u = 0; u < kU; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (int u = 0; u < kU; ++u)
    if (i + u * kThreads < n) {
      const u32x4 v = src[i + u * kThreads];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // practically never: defeats DCE only
}

__global__ __launch_bounds__(kThreads) void write_kernel(u32x4* __restrict__ dst,
                                                         int64_t n, unsigned val) {
  const u32x4 v = {val, val, val, val};
  const int64_t step = static_cast<int64_t>(gridDim.x) * kThreads * kU;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads * kU + threadIdx.x;
  for (; i + (kU - 1) * kThreads < n; i += step) {
#pragma unroll
    for (int u = 0; u < kU; ++u) __builtin_nontemporal_store(v, dst + i + u * kThreads);
  }
  for (int u = 0; u < kU; ++u)
    if (i + u * kThreads < n) dst[i + u * kThreads] = v;
}

// LDS-staged pull: 4 waves x 1 KiB per stage, double-buffered.  LDS-DMA
// destination is wave-uniform base + lane*16 (cdna_hip_programming.md §5
// caveat), so each wave owns a contiguous 1 KiB slot per buffer.
__global__ __launch_bounds__(kThreads) void lds_pull_kernel(const u32x4* __restrict__ src,
                                                            u32x4* __restrict__ dst,
                                                            int64_t n) {
  __shared__ u32x4 slot[2][kThreads];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  int64_t i = blockIdx.x * static_cast<int64_t>(kThreads) + threadIdx.x;
  int buf = 0;
  if (i - lane + 64 <= n) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(src + i),
        (__attribute__((address_space(3))) void*)(&slot[buf][wave * 64]), 16, 0, 0);
  }
  for (; i - lane < n; i += stride) {
    const int64_t nxt = i + stride;
    if (nxt - lane + 64 <= n) {
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src + nxt),
          (__attribute__((address_space(3))) void*)(&slot[buf ^ 1][wave * 64]), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (i - lane + 64 <= n) {
      dst[i] = slot[buf][wave * 64 + lane];
    } else if (i < n) {
      dst[i] = src[i];  // ragged tail: direct copy
    }
    buf ^= 1;
  }
}

int grid_for(int dev) {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus * 8;  // >> CU count: every CU keeps several WGs in flight
}

}  // namespace

KGWE_API int kgwe_probe_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// out[0] = copy GB/s (read+write bytes), out[1] = read GB/s, out[2] = write GB/s,
// out[3] = LDS-staged local copy GB/s (same kernel the xGMI probe uses).
KGWE_API int kgwe_probe_hbm(int dev, int64_t bytes, int iters, double* out) {
  HIPOK(hipSetDevice(dev));
  const int64_t n = bytes / 16;
  u32x4 *a = nullptr, *b = nullptr;
  unsigned* sink = nullptr;
  HIPOK(hipMalloc(&a, n * 16));
  HIPOK(hipMalloc(&b, n * 16));
  HIPOK(hipMalloc(&sink, 4));
  HIPOK(hipMemset(a, 1, n * 16));
  hipEvent_t e0, e1;
  HIPOK(hipEventCreate(&e0));
  HIPOK(hipEventCreate(&e1));
  const int grid = grid_for(dev);
  float ms = 0.f;
  for (int mode = 0; mode < 4; ++mode) {
    // warmup
    for (int w = 0; w < 2; ++w) {
      if (mode == 0) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(kThreads), 0, 0, a, b, n);
      if (mode == 1) hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(kThreads), 0, 0, a, n, sink);
      if (mode == 2) hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(kThreads), 0, 0, b, n, 7u);
      if (mode == 3) hipLaunchKernelGGL(lds_pull_kernel, dim3(grid), dim3(kThreads), 0, 0, a, b, n);
    }
    HIPOK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; ++it) {
      if (mode == 0) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(kThreads), 0, 0, a, b, n);
      if (mode == 1) hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(kThreads), 0, 0, a, n, sink);
      if (mode == 2) hipLaunchKernelGGL(write_kernel, dim3(grid), dim3(kThreads), 0, 0, b, n, 7u);
      if (mode == 3) hipLaunchKernelGGL(lds_pull_kernel, dim3(grid), dim3(kThreads), 0, 0, a, b, n);
    }
    HIPOK(hipEventRecord(e1, 0));
    HIPOK(hipEventSynchronize(e1));
    HIPOK(hipEventElapsedTime(&ms, e0, e1));
    const double moved = (mode == 0 || mode == 3 ? 2.0 : 1.0) * static_cast<double>(n * 16) * iters;
    out[mode] = moved / (ms * 1e-3) / 1e9;
  }
  // Verify the LDS-staged copy moved the right bytes (first/last vector).
  u32x4 h0, h1;
  HIPOK(hipMemcpy(&h0, b, 16, hipMemcpyDeviceToHost));
  HIPOK(hipMemcpy(&h1, b + n - 1, 16, hipMemcpyDeviceToHost));
  const int ok = (h0.x == 0x01010101u && h1.w == 0x01010101u);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(a);
  (void)hipFree(b);
  (void)hipFree(sink);
  return ok ? 0 : -2;
}

// Pull bandwidth of the link src -> dst (kernel runs on dst, reads peer HBM).
// Returns -1 if the devices cannot access each other's memory.
KGWE_API int kgwe_probe_p2p(int src, int dst, int64_t bytes, int iters, double* gbps) {
  int can = 0;
  HIPOK(hipDeviceCanAccessPeer(&can, dst, src));
  if (!can) return -1;
  HIPOK(hipSetDevice(dst));
  hipError_t pe = hipDeviceEnablePeerAccess(src, 0);
  if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) return -3;
  const int64_t n = bytes / 16;
  u32x4 *s = nullptr, *d = nullptr;
  HIPOK(hipSetDevice(src));
  HIPOK(hipMalloc(&s, n * 16));
  HIPOK(hipMemset(s, 3, n * 16));
  HIPOK(hipDeviceSynchronize());
  HIPOK(hipSetDevice(dst));
  HIPOK(hipMalloc(&d, n * 16));
  hipEvent_t e0, e1;
  HIPOK(hipEventCreate(&e0));
  HIPOK(hipEventCreate(&e1));
  const int grid = grid_for(dst);
  hipLaunchKernelGGL(lds_pull_kernel, dim3(grid), dim3(kThreads), 0, 0, s, d, n);
  HIPOK(hipEventRecord(e0, 0));
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL(lds_pull_kernel, dim3(grid), dim3(kThreads), 0, 0, s, d, n);
  HIPOK(hipEventRecord(e1, 0));
  HIPOK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPOK(hipEventElapsedTime(&ms, e0, e1));
  *gbps = static_cast<double>(n * 16) * iters / (ms * 1e-3) / 1e9;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(d);
  HIPOK(hipSetDevice(src));
  (void)hipFree(s);
  return 0;
}

// Every device pulls from every peer at once (all links busy).  matrix is
// ndev*ndev row-major: matrix[dst*ndev+src] = GB/s of that link under full
// load (diagonal = 0).  Returns the number of links measured.
namespace {

// Start gate of the all-links probe: one wave per link spins on a flag in
// pinned host memory until the host raises it, so every link's copies begin
// together however long the launches took to enqueue.  The wait is bounded
// (100 MHz wall clock): a flag that never comes costs `limit_ticks`, never a
// hung queue.  out[0] = 1 if the flag was seen, 0 if the wait timed out.
__global__ void start_gate_kernel(const int* flag, unsigned long long limit_ticks, int* out) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  int seen = 0;
  while (!(seen = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM))) {
    if (wall_clock64() - t0 > limit_ticks) break;
    __builtin_amdgcn_s_sleep(64);
  }
  if (out) *out = seen ? 1 : 0;
}

// Everything the all-links probe allocates, released on every return path.
struct AllLinks {
  static constexpr int kMax = 16;
  int ndev = 0;
  u32x4* src[kMax] = {};
  u32x4* dst[kMax][kMax] = {};
  hipStream_t stream[kMax][kMax] = {};
  hipEvent_t ev0[kMax][kMax] = {}, ev1[kMax][kMax] = {};
  int* flag = nullptr;  // pinned host memory, mapped into every device
  ~AllLinks() {
    for (int d = 0; d < ndev; ++d) {
      if (hipSetDevice(d) != hipSuccess) continue;
      (void)hipDeviceSynchronize();  // nothing of ours is still running when its buffers go
      for (int s = 0; s < ndev; ++s) {
        if (stream[d][s]) (void)hipStreamDestroy(stream[d][s]);
        if (ev0[d][s]) (void)hipEventDestroy(ev0[d][s]);
        if (ev1[d][s]) (void)hipEventDestroy(ev1[d][s]);
        if (dst[d][s]) (void)hipFree(dst[d][s]);
      }
      if (src[d]) (void)hipFree(src[d]);
    }
    if (flag) (void)hipHostFree(flag);
  }
};

}  // namespace

// Bounded-wait self test of the start gate on one device: with raise = 0 the
// flag is never set and the kernel must come back after ~limit_us on its own
// (returns 0); with raise = 1 the host raises it and the kernel must see it
// (returns 1).  Negative: a HIP error.
KGWE_API int kgwe_probe_gate_selftest(int dev, int raise, int limit_us) {
  HIPOK(hipSetDevice(dev));
  int* flag = nullptr;
  int* out = nullptr;
  if (hipHostMalloc(&flag, sizeof(int), hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return -1001;
  if (hipHostMalloc(&out, sizeof(int), hipHostMallocMapped) != hipSuccess) {
    (void)hipHostFree(flag);
    return -1001;
  }
  *flag = 0;
  *out = -1;
  hipLaunchKernelGGL(start_gate_kernel, dim3(1), dim3(64), 0, 0, flag,
                     static_cast<unsigned long long>(limit_us) * 100ull, out);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && raise) __atomic_store_n(flag, 1, __ATOMIC_RELEASE);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  const int seen = *out;
  (void)hipHostFree(flag);
  (void)hipHostFree(out);
  return e == hipSuccess ? seen : -static_cast<int>(e) - 1000;
}

// All ordered pairs at once: matrix[dst * ndev + src] = GB/s of dst pulling
// from src while every other link of the node is busy too (what a ring or
// all-to-all collective sees).  Returns the number of links measured.
KGWE_API int kgwe_probe_p2p_all(int ndev, int64_t bytes, int iters, double* matrix) {
  const int64_t n = bytes / 16;
  if (ndev > AllLinks::kMax) ndev = AllLinks::kMax;
  if (ndev < 1 || n < 1 || iters < 1) return 0;
  AllLinks r;
  r.ndev = ndev;
  int links = 0;
  HIPOK(hipHostMalloc(&r.flag, sizeof(int), hipHostMallocMapped | hipHostMallocPortable));
  *r.flag = 0;
  for (int d = 0; d < ndev; ++d) {
    HIPOK(hipSetDevice(d));
    HIPOK(hipMalloc(&r.src[d], n * 16));
    HIPOK(hipMemset(r.src[d], d + 1, n * 16));
  }
  for (int d = 0; d < ndev; ++d) {
    HIPOK(hipSetDevice(d));
    for (int s = 0; s < ndev; ++s) {
      matrix[d * ndev + s] = 0.0;
      if (s == d) continue;
      int can = 0;
      (void)hipDeviceCanAccessPeer(&can, d, s);
      if (!can) continue;
      hipError_t pe = hipDeviceEnablePeerAccess(s, 0);
      if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) continue;
      (void)hipGetLastError();
      HIPOK(hipMalloc(&r.dst[d][s], n * 16));
      HIPOK(hipStreamCreateWithFlags(&r.stream[d][s], hipStreamNonBlocking));
      HIPOK(hipEventCreate(&r.ev0[d][s]));
      HIPOK(hipEventCreate(&r.ev1[d][s]));
    }
  }
  for (int d = 0; d < ndev; ++d) {
    HIPOK(hipSetDevice(d));
    HIPOK(hipDeviceSynchronize());
  }
  // Every link: gate, timed copies.  Each link gets 1/(ndev-1) of the CUs'
  // worth of workgroups so all of a device's pulls are resident together.  The
  // gate waits at most 2 s for the host's flag (raised right after the last
  // launch below).
  const unsigned long long gate_ticks = 200000000ull;
  hipError_t launch_err = hipSuccess;
  for (int d = 0; d < ndev && launch_err == hipSuccess; ++d) {
    if ((launch_err = hipSetDevice(d)) != hipSuccess) break;
    const int grid = grid_for(d) / (ndev > 1 ? ndev - 1 : 1);
    for (int s = 0; s < ndev; ++s) {
      if (!r.stream[d][s]) continue;
      hipLaunchKernelGGL(start_gate_kernel, dim3(1), dim3(64), 0, r.stream[d][s], r.flag, gate_ticks,
                         static_cast<int*>(nullptr));
      if ((launch_err = hipEventRecord(r.ev0[d][s], r.stream[d][s])) != hipSuccess) break;
      for (int it = 0; it < iters; ++it)
        hipLaunchKernelGGL(lds_pull_kernel, dim3(grid > 0 ? grid : 1), dim3(kThreads), 0, r.stream[d][s],
                           r.src[s], r.dst[d][s], n);
      if ((launch_err = hipEventRecord(r.ev1[d][s], r.stream[d][s])) != hipSuccess) break;
      if ((launch_err = hipGetLastError()) != hipSuccess) break;
    }
  }
  // Raise the flag whatever happened above: gates already enqueued must not
  // sit out their 2 s before the cleanup's synchronize.
  __atomic_store_n(r.flag, 1, __ATOMIC_RELEASE);
  if (launch_err != hipSuccess) return -static_cast<int>(launch_err) - 1000;
  for (int d = 0; d < ndev; ++d) {
    HIPOK(hipSetDevice(d));
    for (int s = 0; s < ndev; ++s) {
      if (!r.stream[d][s]) continue;
      HIPOK(hipEventSynchronize(r.ev1[d][s]));
      float ms = 0.f;
      HIPOK(hipEventElapsedTime(&ms, r.ev0[d][s], r.ev1[d][s]));
      matrix[d * ndev + s] = static_cast<double>(n * 16) * iters / (ms * 1e-3) / 1e9;
      ++links;
    }
  }
  return links;
}
