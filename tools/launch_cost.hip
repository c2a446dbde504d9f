// Host cost of the launch forms the executor uses (MI355X box):
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o /tmp/launch_cost && /tmp/launch_cost
// plain hipLaunchKernelGGL, hipExtLaunchKernelGGL with a stop event (the
// backward's chain launches), alternating two streams, event record / wait,
// with a 512-byte argument struct (GConvArgs-sized), queue idle and blocked.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

struct Big { char b[512]; };
__global__ void k_small(Big a, float *o) { if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[3] == 7) o[0] = 1.f; }
__global__ void k_spin(long long cyc) {
  const long long t0 = clock64();
  while (clock64() - t0 < cyc) {}
}
static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev, ev2;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
  float *o;
  CK(hipMalloc(&o, 16));
  Big a{};
  const int N = 100;
  for (int rep = 0; rep < 3; ++rep) {
    for (int blocked = 0; blocked < 2; ++blocked) {
      auto pre = [&]() {
        CK(hipDeviceSynchronize());
        if (blocked) { hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s0, (long long)200000000); }
        return 0;
      };
      double t;
      pre(); t = now_us();
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s0, a, o);
      const double plain = (now_us() - t) / N;
      pre(); t = now_us();
      for (int i = 0; i < N; ++i) hipExtLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s0, nullptr, ev, 0, a, o);
      const double ext = (now_us() - t) / N;
      pre(); t = now_us();
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, (i & 1) ? s1 : s0, a, o);
      const double alt = (now_us() - t) / N;
      pre(); t = now_us();
      for (int i = 0; i < N; ++i) { hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s0, a, o); (void)hipEventRecord(ev2, s0); }
      const double rec = (now_us() - t) / N;
      pre(); t = now_us();
      for (int i = 0; i < N; ++i) { hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s0, a, o); (void)hipStreamWaitEvent(s0, ev2, 0); }
      const double wt = (now_us() - t) / N;
      pre(); t = now_us();
      for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s1, a, o);
      const double s1us = (now_us() - t) / N;
      printf("rep %d %s: plain %.2f  ext+stopevent %.2f  alt2streams %.2f  launch+record %.2f  launch+wait %.2f  other-stream %.2f us\n",
             rep, blocked ? "blocked" : "idle   ", plain, ext, alt, rec, wt, s1us);
      CK(hipDeviceSynchronize());
    }
  }
  return 0;
}
