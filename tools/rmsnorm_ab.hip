// A/B timing of the RMSNorm backward: the shipped native/ops/rmsnorm.hip
// against another version of the file (-DOLD_SRC=<path>), both linked into
// one binary under different namespaces, at the Llama-3-8B step shape
// (T=16384, H=4096, with the residual-gradient add).
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "common.h"
#define KGWE_API static
namespace cur {
#include "../native/ops/rmsnorm.hip"
}
namespace old {
#include OLD_SRC
}
#define CK(x) do { if ((x) != hipSuccess) { std::printf("HIP error line %d\n", __LINE__); std::exit(1); } } while (0)
int main() {
  const int T = 16384, H = 4096;
  void *dy, *h, *w, *dadd, *dx, *dwb; float *rstd, *part;
  CK(hipMalloc(&dy, size_t(T) * H * 2)); CK(hipMalloc(&h, size_t(T) * H * 2)); CK(hipMalloc(&dadd, size_t(T) * H * 2));
  CK(hipMalloc(&dx, size_t(T) * H * 2)); CK(hipMalloc(&w, H * 2)); CK(hipMalloc(&dwb, H * 2));
  CK(hipMalloc(&rstd, T * 4)); CK(hipMalloc(&part, H * 4));
  CK(hipMemset(dy, 0x3c, size_t(T) * H * 2)); CK(hipMemset(h, 0x3c, size_t(T) * H * 2));
  CK(hipMemset(dadd, 0x3c, size_t(T) * H * 2)); CK(hipMemset(w, 0x3c, H * 2)); CK(hipMemset(rstd, 0x3c, T * 4));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto t = [&](auto fn) { for (int i = 0; i < 3; ++i) fn(); CK(hipDeviceSynchronize()); CK(hipEventRecord(a, 0));
    for (int i = 0; i < 30; ++i) fn(); CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / 30 * 1e3; };
  for (int rep = 0; rep < 3; ++rep) {
    float n = t([&] { if (cur::kgwe_rmsnorm_bwd(dy, h, w, rstd, dadd, dx, part, dwb, nullptr, T, H, 0)) std::exit(2); });
    float o = t([&] { if (old::kgwe_rmsnorm_bwd(dy, h, w, rstd, dadd, dx, part, dwb, nullptr, T, H, 0)) std::exit(3); });
    std::printf("rmsnorm bwd: new %.1f us (%.2f TB/s)  old %.1f us\n", n, 4.0 * T * H * 2 / n / 1e6, o);
  }
  return 0;
}
