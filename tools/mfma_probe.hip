// Probe of the 16-block fp32 MFMA v_mfma_f32_4x4x1_16b_f32 on gfx950: the
// lane layout of its A/B operands and result, and its issue rate next to
// v_mfma_f32_16x16x4_f32.  Build and run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/bin/mfma_probe && tools/bin/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));                    \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void layout_kernel(float *out) {
  const int l = threadIdx.x;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  // pass 0: A = lane + 1, B = 1 -> D(l, r) names the A lane feeding it
  const f4 d0 = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.f, z, 0, 0, 0);
  // pass 1: A = 1, B = lane + 1 -> D(l, r) names the B lane feeding it
  const f4 d1 = __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, (float)(l + 1), z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    out[l * 4 + r] = d0[r];
    out[256 + l * 4 + r] = d1[r];
  }
}

template <int SHAPE>
__global__ void __launch_bounds__(256) rate_kernel(float *out, int iters) {
  const int l = threadIdx.x & 63;
  const float a = 1.f + 1e-3f * l, b = 1.f - 1e-3f * l;
  f4 acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = f4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (SHAPE == 0)
        acc[k] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[k], 0, 0, 0);
      else
        acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[k], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int SHAPE>
static int time_rate(float *d, const char *name, double flops_per_inst) {
  const int blocks = 256 * 8, iters = 4000;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(rate_kernel<SHAPE>, dim3(blocks), dim3(256), 0, 0, d, 100);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(rate_kernel<SHAPE>, dim3(blocks), dim3(256), 0, 0, d, iters);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double insts = (double)blocks * 4 * iters * 8;  // wave-level MFMA instructions
  printf("%-28s %8.3f ms  %7.1f TFLOP/s\n", name, ms, insts * flops_per_inst / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  float *d = nullptr;
  CHECK(hipMalloc(&d, 256 * 8 * 256 * sizeof(float)));
  hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, d);
  CHECK(hipDeviceSynchronize());
  std::vector<float> h(512);
  CHECK(hipMemcpy(h.data(), d, 512 * sizeof(float), hipMemcpyDeviceToHost));
  printf("lane: A-lane feeding D(lane, r=0..3) | B-lane feeding D(lane, r=0..3)\n");
  for (int l = 0; l < 64; ++l) {
    printf("%2d:", l);
    for (int r = 0; r < 4; ++r) printf(" %3d", (int)h[l * 4 + r] - 1);
    printf(" |");
    for (int r = 0; r < 4; ++r) printf(" %3d", (int)h[256 + l * 4 + r] - 1);
    printf("\n");
  }
  if (time_rate<0>(d, "mfma_f32_4x4x1_16b_f32", 16.0 * 4 * 4 * 2)) return 1;
  if (time_rate<1>(d, "mfma_f32_16x16x4_f32", 16.0 * 16 * 4 * 2)) return 1;
  return 0;
}
