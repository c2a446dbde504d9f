// Single-wave MFMA issue rate vs the number of independent accumulator chains
// (one / two / eight waves per SIMD).  Build and run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_rate_probe.hip -o tools/mfma_rate_probe && tools/mfma_rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int NACC, int SHAPE>
__global__ void __launch_bounds__(256) rate_kernel(float *out, int iters) {
  const int l = threadIdx.x & 63;
  const float a = 1.f + 1e-3f * l, b = 1.f - 1e-3f * l;
  f4 acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = f4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      if (SHAPE == 0) acc[k] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[k], 0, 0, 0);
      else acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[k], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NACC; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC, int SHAPE>
void run(float *d, int blocks, const char *name) {
  const int iters = 20000 / NACC * 8;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((rate_kernel<NACC, SHAPE>), dim3(blocks), dim3(256), 0, 0, d, 10);
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((rate_kernel<NACC, SHAPE>), dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double insts_per_wave = (double)iters * NACC;
  const double fl = SHAPE == 0 ? 512.0 : 2048.0;
  printf("%-10s blocks %5d nacc %2d: %8.3f ms  %7.1f TF/s  %.2f ns per MFMA per wave\n", name, blocks, NACC, ms,
         (double)blocks * 4 * insts_per_wave * fl / (ms * 1e-3) / 1e12, ms * 1e6 / insts_per_wave);
}
int main() {
  float *d; hipMalloc(&d, 256 * 8 * 256 * 4);
  for (int bl : {256, 512, 2048}) {
    run<4, 0>(d, bl, "4x4x1");
    run<8, 0>(d, bl, "4x4x1");
    run<16, 0>(d, bl, "4x4x1");
    run<4, 1>(d, bl, "16x16x4");
    run<8, 1>(d, bl, "16x16x4");
  }
  return 0;
}
