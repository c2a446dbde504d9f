// Pixel-weighted BCE-with-logits loss (hcat/loss.py:5-101, method='pixel')
// and the Adam step (torch.optim.Adam as used in tests/r_unet_test.py:24,56).
#include "common.h"
#include "timing.h"
#include <hip/hip_fp16.h>
#include <algorithm>
#include <cmath>

namespace hcu {

enum { DT_F32 = 0, DT_F16 = 1, DT_U8 = 2 };

__device__ __forceinline__ float load_as_float(const void *p, int dtype, size_t i) {
  if (dtype == DT_F16) return __half2float(reinterpret_cast<const __half *>(p)[i]);
  if (dtype == DT_U8) return (float)reinterpret_cast<const unsigned char *>(p)[i];
  return reinterpret_cast<const float *>(p)[i];
}

// (pwl + 1) evaluated in pwl's dtype (hcat/loss.py:72): for fp16 the sum is
// rounded to half before the fp32 multiply, as torch's half add does.
__device__ __forceinline__ float pixel_weight(const void *pwl, int dtype, size_t i) {
  if (!pwl) return 2.f;  // pwl=None -> ones + 1 (hcat/loss.py:46-47)
  if (dtype == DT_F16) {
    const float v = __half2float(reinterpret_cast<const __half *>(pwl)[i]);
    return __half2float(__float2half(v + 1.f));
  }
  return reinterpret_cast<const float *>(pwl)[i] + 1.f;
}

int loss_rows(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 1023) / 1024, 1024));
}

__global__ void __launch_bounds__(256)
loss_pixel_kernel(const float *pred, int PX, int PY, int PZ, const void *mask, int mdt,
                  const void *pwl, int wdt, int MX, int MY, int MZ, float *dpred,
                  float *part, int64_t n, int64_t chunk, float invN) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const int64_t beg = (int64_t)blockIdx.x * chunk;
  const int64_t end = std::min(beg + chunk, n);
  double acc = 0.0;
  for (int64_t e = beg + tid; e < end; e += 256) {
    int64_t q = e;
    const int z = (int)(q % PZ);
    q /= PZ;
    const int y = (int)(q % PY);
    q /= PY;
    const int x = (int)(q % PX);
    const int64_t bc = q / PX;
    const size_t mi = (((size_t)bc * MX + x) * MY + y) * MZ + z;
    const float xv = pred[e];
    const float m = load_as_float(mask, mdt, mi);
    const float w = pixel_weight(pwl, wdt, mi);
    // BCEWithLogits: (1 - m) * x - log_sigmoid(x)
    const float ls = fminf(xv, 0.f) - log1pf(expf(-fabsf(xv)));
    const float l = (1.f - m) * xv - ls;
    acc += (double)(l * w);
    if (dpred) {
      const float sig = 1.f / (1.f + expf(-xv));
      dpred[e] = (sig - m) * (invN * w);
    }
  }
  red[tid] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) part[blockIdx.x] = (float)red[0];
}

__global__ void __launch_bounds__(256)
loss_finalize_kernel(const float *part, int R, double n, float *loss) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int r = tid; r < R; r += 256) s += (double)part[r];
  red[tid] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  if (tid == 0) loss[0] = (float)(red[0] / n);
}

int launch_loss_pixel(const float *pred, int B, int C, int PX, int PY, int PZ,
                      const void *mask, int mask_dtype, const void *pwl, int pwl_dtype,
                      int MX, int MY, int MZ, float *loss, float *dpred, float *part,
                      int R, hipStream_t s) {
  const int64_t n = (int64_t)B * C * PX * PY * PZ;
  if (n <= 0) return fail(1, "loss: empty prediction");
  const int64_t chunk = (n + R - 1) / R;
  HCU_TIMED(s, "loss_pixel_kernel", 0.0, 0.0, HCU_LAUNCH(loss_pixel_kernel, dim3(R), dim3(256), 0, s, pred, PX, PY, PZ, mask,
                     mask_dtype, pwl, pwl_dtype, MX, MY, MZ, dpred, part, n, chunk,
                     1.f / (float)n));
  HCU_CHECK_LAUNCH();
  HCU_TIMED(s, "loss_finalize_kernel", 0.0, 0.0, HCU_LAUNCH(loss_finalize_kernel, dim3(1), dim3(256), 0, s, part, R, (double)n, loss));
  HCU_CHECK_LAUNCH();
  return 0;
}

__global__ void __launch_bounds__(256)
scale_kernel(const float *src, const float *scale, float *dst, int64_t n) {
  const float sc = scale[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256)
    dst[i] = src[i] * sc;
}

int launch_scale(const float *src, const float *scale, float *dst, int64_t n, hipStream_t s) {
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
  HCU_TIMED(s, "scale_kernel", 0.0, 0.0, HCU_LAUNCH(scale_kernel, dim3(blocks), dim3(256), 0, s, src, scale, dst, n));
  HCU_CHECK_LAUNCH();
  return 0;
}

// Adam, mirroring torch.optim.Adam's foreach arithmetic:
//   m.lerp_(g, 1-b1); v = v*b2 + (1-b2)*g*g;
//   p += -lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void __launch_bounds__(256)
adam_kernel(float *p, const float *g, float *m, float *v, int64_t n, float b1, float b2,
            float eps, float wd, float neg_step_size, float bc2_sqrt, float grad_scale) {
  const float w1 = 1.f - b1, w2 = 1.f - b2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    float gi = g[i] * grad_scale;
    float pi = p[i];
    if (wd != 0.f) gi = fmaf(wd, pi, gi);
    float mi = m[i];
    mi = mi + w1 * (gi - mi);
    float vi = v[i] * b2;
    vi = fmaf(w2, gi * gi, vi);
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = fmaf(neg_step_size, mi / denom, pi);
    m[i] = mi;
    v[i] = vi;
  }
}

int launch_adam(float *p, const float *g, float *m, float *v, int64_t n, float lr, float b1,
                float b2, float eps, float wd, int64_t step, float grad_scale, hipStream_t s) {
  if (step < 1) return fail(1, "adam: step must be >= 1");
  const double bc1 = 1.0 - std::pow((double)b1, (double)step);
  const double bc2 = 1.0 - std::pow((double)b2, (double)step);
  const float neg_step = (float)(-(double)lr / bc1);
  const float bc2s = (float)std::sqrt(bc2);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
  HCU_TIMED(s, "adam_kernel", 0.0, 0.0, HCU_LAUNCH(adam_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, n, b1, b2, eps,
                     wd, neg_step, bc2s, grad_scale));
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu
