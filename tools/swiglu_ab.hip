// A/B timing of the SwiGLU kernels: the shipped native/ops/swiglu.hip against
// another version of the file (-DOLD_SRC=<path>), both linked into one binary
// under different namespaces, at the Llama-3-8B step shape (T=16384, F=14336).
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "common.h"
#define KGWE_API static
namespace cur {
#include "../native/ops/swiglu.hip"
}
namespace old {
#include OLD_SRC
}
#define CK(x) do { if ((x) != hipSuccess) { std::printf("HIP error line %d\n", __LINE__); std::exit(1); } } while (0)
int main() {
  const long long T = 16384; const int F = 14336;
  void *gu, *o, *go, *dgu;
  CK(hipMalloc(&gu, T * 2 * F * 2)); CK(hipMalloc(&o, T * F * 2)); CK(hipMalloc(&go, T * F * 2));
  CK(hipMalloc(&dgu, T * 2 * F * 2));
  CK(hipMemset(gu, 0x3c, T * 2 * F * 2)); CK(hipMemset(go, 0x3c, T * F * 2));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto t = [&](auto fn) { for (int i = 0; i < 3; ++i) fn(); CK(hipDeviceSynchronize()); CK(hipEventRecord(a, 0));
    for (int i = 0; i < 30; ++i) fn(); CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / 30 * 1e3; };
  const char* g = (const char*)gu; const char* u = g + F * 2;
  for (int rep = 0; rep < 2; ++rep) {
    float f1 = t([&] { cur::kgwe_swiglu_fwd(g, u, 2 * F, o, T, F, 0); });
    float f0 = t([&] { old::kgwe_swiglu_fwd(g, u, 2 * F, o, T, F, 0); });
    float b1 = t([&] { cur::kgwe_swiglu_bwd(g, u, 2 * F, go, dgu, (char*)dgu + F * 2, 2 * F, T, F, 0); });
    float b0 = t([&] { old::kgwe_swiglu_bwd(g, u, 2 * F, go, dgu, (char*)dgu + F * 2, 2 * F, T, F, 0); });
    std::printf("swiglu fwd: new %.1f us (%.2f TB/s)  old %.1f us | bwd: new %.1f us (%.2f TB/s)  old %.1f us\n",
                f1, 3.0 * T * F * 2 / f1 / 1e6, f0, b1, 5.0 * T * F * 2 / b1 / 1e6, b0);
  }
  return 0;
}
