// RCCL all-reduce bus-bandwidth sweep over the xGMI mesh (single process,
// one communicator per visible GPU via ncclCommInitAll).
//
// Reproduces the reference's only communication metric — "all-reduce
// effective bandwidth 142 -> 228 GB/s, random vs topology-aware placement"
// (docs/PRD.md:117-124, README.md:158) — on MI355X: for each message size,
// algBW = bytes / time and busBW = algBW * 2 (n - 1) / n (the ring-equivalent
// bytes each GPU moves), so results compare across GPU counts.
// librccl is dlopen'ed: the probe library still loads where RCCL is absent.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <vector>

#define KGWE_API extern "C" __attribute__((visibility("default")))

namespace {

struct Rccl {
  void* so = nullptr;
  decltype(&::ncclCommInitAll) commInitAll = nullptr;
  decltype(&::ncclCommDestroy) commDestroy = nullptr;
  decltype(&::ncclAllReduce) allReduce = nullptr;
  decltype(&::ncclGroupStart) groupStart = nullptr;
  decltype(&::ncclGroupEnd) groupEnd = nullptr;
  bool load() {
    if (so) return true;
    const char* names[] = {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"};
    for (const char* n : names)
      if ((so = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (!so) return false;
    commInitAll = reinterpret_cast<decltype(commInitAll)>(dlsym(so, "ncclCommInitAll"));
    commDestroy = reinterpret_cast<decltype(commDestroy)>(dlsym(so, "ncclCommDestroy"));
    allReduce = reinterpret_cast<decltype(allReduce)>(dlsym(so, "ncclAllReduce"));
    groupStart = reinterpret_cast<decltype(groupStart)>(dlsym(so, "ncclGroupStart"));
    groupEnd = reinterpret_cast<decltype(groupEnd)>(dlsym(so, "ncclGroupEnd"));
    return commInitAll && commDestroy && allReduce && groupStart && groupEnd;
  }
};

Rccl g_rccl;

}  // namespace

// sizes[i] in bytes (bf16 elements = bytes/2); out_busbw[i] GB/s, out_algbw[i]
// GB/s, out_us[i] microseconds per all-reduce.  Returns ndev used, < 0 on error.
KGWE_API int kgwe_rccl_allreduce_sweep(int ndev, const int64_t* sizes, int nsizes, int iters,
                                       double* out_us, double* out_algbw, double* out_busbw) {
  if (!g_rccl.load()) return -1;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail < 1) return -2;
  if (ndev <= 0 || ndev > avail) ndev = avail;
  std::vector<ncclComm_t> comms(ndev);
  std::vector<int> devs(ndev);
  for (int i = 0; i < ndev; ++i) devs[i] = i;
  if (g_rccl.commInitAll(comms.data(), ndev, devs.data()) != ncclSuccess) return -3;
  int64_t maxb = 0;
  for (int s = 0; s < nsizes; ++s) maxb = sizes[s] > maxb ? sizes[s] : maxb;
  std::vector<void*> buf(ndev, nullptr);
  std::vector<hipStream_t> st(ndev);
  std::vector<hipEvent_t> e0(ndev), e1(ndev);
  int rc = ndev;
  for (int i = 0; i < ndev; ++i) {
    if (hipSetDevice(i) != hipSuccess || hipMalloc(&buf[i], maxb) != hipSuccess ||
        hipMemset(buf[i], 0, maxb) != hipSuccess ||
        hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e0[i]) != hipSuccess || hipEventCreate(&e1[i]) != hipSuccess) {
      rc = -4;
      break;
    }
  }
  for (int s = 0; rc > 0 && s < nsizes; ++s) {
    const size_t count = static_cast<size_t>(sizes[s] / 2);  // bf16
    auto run = [&](int n) {
      for (int it = 0; it < n; ++it) {
        g_rccl.groupStart();
        for (int i = 0; i < ndev; ++i)
          g_rccl.allReduce(buf[i], buf[i], count, ncclBfloat16, ncclSum, comms[i], st[i]);
        g_rccl.groupEnd();
      }
    };
    run(2);  // warmup
    for (int i = 0; i < ndev; ++i) {
      (void)hipSetDevice(i);
      (void)hipEventRecord(e0[i], st[i]);
    }
    run(iters);
    float worst = 0.f;
    for (int i = 0; i < ndev; ++i) {
      (void)hipSetDevice(i);
      (void)hipEventRecord(e1[i], st[i]);
      (void)hipEventSynchronize(e1[i]);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0[i], e1[i]);
      worst = ms > worst ? ms : worst;
    }
    const double t = static_cast<double>(worst) * 1e-3 / iters;
    out_us[s] = t * 1e6;
    out_algbw[s] = static_cast<double>(sizes[s]) / t / 1e9;
    out_busbw[s] = ndev > 1 ? out_algbw[s] * 2.0 * (ndev - 1) / ndev : 0.0;
  }
  for (int i = 0; i < ndev; ++i) {
    (void)hipSetDevice(i);
    if (buf[i]) (void)hipFree(buf[i]);
    if (st[i]) (void)hipStreamDestroy(st[i]);
    g_rccl.commDestroy(comms[i]);
  }
  return rc;
}
