// The reference's other loss functions (hcat/loss.py:5-178) on the device:
// cross_entropy(method='worst_z' | 'sigmoid' | 'random'), dice, L1Loss and
// MSELoss.  ('pixel', the training hot path, is the fused kernel in
// loss_adam.hip.)
//
// Every loss is a forward pass that writes fixed-size per-workgroup partial
// sums (fp64), a one-workgroup finalize that combines them in a fixed order
// into the loss and the few scalars its gradient needs (`aux`), and a
// backward pass that writes d(loss)/d(pred) already multiplied by the
// upstream gradient (a device scalar).  No float atomics: results are bitwise
// reproducible.  'random' draws its pixel indices on the host from torch's
// default generator exactly as the reference does (hcat/loss.py:87-88); the
// device counts, compacts and gathers the positive/negative pixels, and its
// gradient is count(e) * dBCE(e) with the per-pixel draw counts taken by
// integer atomics (duplicates of a pixel contribute identical terms).
#include "common.h"
#include "timing.h"
#include "hcunet.h"
#include <hip/hip_fp16.h>
#include <algorithm>
#include <cmath>

namespace hcu {

enum LossMode { LM_SIGMOID = 0, LM_WORSTZ = 1, LM_DICE = 2, LM_L1 = 3, LM_MSE = 4, LM_BCE = 5,
                LM_RANDOM = 6 };

struct LossGeom {
  const float *pred;
  int PX, PY, PZ;
  int64_t n;          // B*C*PX*PY*PZ
  const void *mask;
  int mdt;            // 0 f32, 1 f16, 2 u8
  const void *pwl;    // nullable: weight 2
  int wdt;
  int MX, MY, MZ;
};

__device__ __forceinline__ float lx_load(const void *p, int dt, size_t i) {
  if (dt == 1) return __half2float(reinterpret_cast<const __half *>(p)[i]);
  if (dt == 2) return (float)reinterpret_cast<const unsigned char *>(p)[i];
  return reinterpret_cast<const float *>(p)[i];
}
// (pwl + 1) in pwl's dtype (hcat/loss.py:72); pwl=None -> ones + 1 (:45-47)
__device__ __forceinline__ float lx_weight(const LossGeom &g, size_t mi) {
  if (!g.pwl) return 2.f;
  if (g.wdt == 1) {
    const float v = __half2float(reinterpret_cast<const __half *>(g.pwl)[mi]);
    return __half2float(__float2half(v + 1.f));
  }
  return reinterpret_cast<const float *>(g.pwl)[mi] + 1.f;
}
// pred element e -> (mask index of the top-left crop, z)
__device__ __forceinline__ size_t lx_mask_index(const LossGeom &g, int64_t e, int &z) {
  int64_t q = e;
  z = (int)(q % g.PZ);
  q /= g.PZ;
  const int y = (int)(q % g.PY);
  q /= g.PY;
  const int x = (int)(q % g.PX);
  const int64_t bc = q / g.PX;
  return (((size_t)bc * g.MX + x) * g.MY + y) * g.MZ + z;
}
// BCEWithLogits(x, m) = (1 - m) x - log_sigmoid(x)
__device__ __forceinline__ float lx_bce(float x, float m) {
  const float ls = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
  return (1.f - m) * x - ls;
}
__device__ __forceinline__ float lx_sig(float x) { return 1.f / (1.f + expf(-x)); }

__device__ void lx_block_sum2(double &a, double &b, double *red) {
  const int tid = threadIdx.x;
  __syncthreads();
  red[tid] = a;
  red[256 + tid] = b;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      red[tid] += red[tid + off];
      red[256 + tid] += red[256 + tid + off];
    }
    __syncthreads();
  }
  a = red[0];
  b = red[256];
}

// Partial sums per workgroup row r (and per z plane for worst_z: blockIdx.y).
// part[(z * R + r) * 2 + {0,1}]
__global__ void __launch_bounds__(256)
loss_ext_fwd_kernel(LossGeom g, int mode, double *part, int64_t chunk) {
  __shared__ double red[512];
  const int R = gridDim.x, r = blockIdx.x, tid = threadIdx.x;
  double s0 = 0.0, s1 = 0.0;
  if (mode == LM_WORSTZ) {
    // rows of the (b, c, x, y) space at the fixed z plane blockIdx.y
    const int zz = blockIdx.y;
    const int64_t nrows = g.n / g.PZ;
    const int64_t beg = (int64_t)r * chunk, end = min(beg + chunk, nrows);
    for (int64_t row = beg + tid; row < end; row += 256) {
      const int64_t e = row * g.PZ + zz;
      int z;
      const size_t mi = lx_mask_index(g, e, z);
      s0 += (double)(lx_bce(g.pred[e], lx_load(g.mask, g.mdt, mi)) * lx_weight(g, mi));
    }
    lx_block_sum2(s0, s1, red);
    if (tid == 0) {
      part[((size_t)zz * R + r) * 2] = s0;
      part[((size_t)zz * R + r) * 2 + 1] = 0.0;
    }
    return;
  }
  const int64_t beg = (int64_t)r * chunk, end = min(beg + chunk, g.n);
  for (int64_t e = beg + tid; e < end; e += 256) {
    int z;
    const size_t mi = lx_mask_index(g, e, z);
    const float p = g.pred[e], m = lx_load(g.mask, g.mdt, mi);
    switch (mode) {
      case LM_SIGMOID:   // pred = sigmoid(pred) (:38-40), then 'pixel' (:95-97)
        s0 += (double)(lx_bce(lx_sig(p), m) * lx_weight(g, mi));
        break;
      case LM_DICE: {    // (:123-124)
        const float s = lx_sig(p);
        s0 += (double)(s * m);
        s1 += (double)(s + m);
        break;
      }
      case LM_L1:
        s0 += (double)fabsf(p - m);
        break;
      case LM_MSE: {
        const float d = p - m;
        s0 += (double)(d * d);
        break;
      }
      default:           // LM_BCE: 'random' with no positive pixel (:84-85)
        s0 += (double)lx_bce(p, m);
        break;
    }
  }
  lx_block_sum2(s0, s1, red);
  if (tid == 0) {
    part[(size_t)r * 2] = s0;
    part[(size_t)r * 2 + 1] = s1;
  }
}

// One workgroup: fixed-order fp64 combine of the partial rows -> loss[0], aux.
//  SIGMOID/L1/MSE/BCE/RANDOM: aux[0] = 1 / N
//  DICE:   aux[0] = 2 I + 1e-10, aux[1] = U + 1e-10 (:124)
//  WORSTZ: aux[z] = scaling[rank(z)] / (X Y) / Z, zscale = linspace(1,2,Z)^2 (:76)
__global__ void __launch_bounds__(256)
loss_ext_finalize_kernel(const double *part, int R, int nz, int mode, double N, double XY,
                         const float *zscale, float *loss, float *aux) {
  __shared__ double red[512];
  __shared__ float zs[1024];
  const int tid = threadIdx.x;
  if (mode == LM_WORSTZ) {
    for (int z = 0; z < nz; ++z) {
      double a = 0.0, b = 0.0;
      for (int r = tid; r < R; r += 256) a += part[((size_t)z * R + r) * 2];
      lx_block_sum2(a, b, red);
      if (tid == 0) zs[z] = (float)a;   // loss.sum(dim=[0,1,2,3]) is an fp32 tensor
    }
    __syncthreads();
    if (tid == 0) {
      // torch.sort ascending; equal sums keep plane order
      double tot = 0.0;
      for (int z = 0; z < nz; ++z) {
        int rank = 0;
        for (int q = 0; q < nz; ++q)
          rank += (zs[q] < zs[z] || (zs[q] == zs[z] && q < z)) ? 1 : 0;
        const float term = (zs[z] * zscale[rank]) / (float)XY;
        tot += (double)term;
        aux[z] = (float)((double)zscale[rank] / XY / (double)nz);
      }
      loss[0] = (float)(tot / (double)nz);
    }
    return;
  }
  double a = 0.0, b = 0.0;
  for (int r = tid; r < R; r += 256) {
    a += part[(size_t)r * 2];
    b += part[(size_t)r * 2 + 1];
  }
  lx_block_sum2(a, b, red);
  if (tid != 0) return;
  if (mode == LM_DICE) {
    const double I2 = 2.0 * (double)(float)a + 1e-10, U = (double)(float)b + 1e-10;
    loss[0] = (float)(1.0 - I2 / U);
    aux[0] = (float)I2;
    aux[1] = (float)U;
    return;
  }
  loss[0] = (float)(a / N);
  aux[0] = (float)(1.0 / N);
}

// d(loss)/d(pred) * gout[0]
__global__ void __launch_bounds__(256)
loss_ext_bwd_kernel(LossGeom g, int mode, const float *aux, const int *cnt, const float *gout,
                    float *dpred) {
  const float go = gout ? gout[0] : 1.f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < g.n; e += (int64_t)gridDim.x * 256) {
    int z;
    const size_t mi = lx_mask_index(g, e, z);
    const float p = g.pred[e], m = lx_load(g.mask, g.mdt, mi);
    float d;
    switch (mode) {
      case LM_SIGMOID: {
        const float s = lx_sig(p);
        d = (lx_sig(s) - m) * lx_weight(g, mi) * aux[0] * (s * (1.f - s));
        break;
      }
      case LM_WORSTZ:
        d = (lx_sig(p) - m) * lx_weight(g, mi) * aux[z];
        break;
      case LM_DICE: {   // L = 1 - I2/U: dL/ds = (I2 - 2 m U) / U^2
        const float s = lx_sig(p), I2 = aux[0], U = aux[1];
        d = (I2 - 2.f * m * U) / (U * U) * (s * (1.f - s));
        break;
      }
      case LM_L1: {
        const float t = p - m;
        d = (t > 0.f ? 1.f : (t < 0.f ? -1.f : 0.f)) * aux[0];
        break;
      }
      case LM_MSE:
        d = 2.f * (p - m) * aux[0];
        break;
      case LM_RANDOM:
        d = (float)cnt[e] * ((lx_sig(p) - m) * aux[0]);
        break;
      default:   // LM_BCE
        d = (lx_sig(p) - m) * aux[0];
        break;
    }
    dpred[e] = d * go;
  }
}

// ---- 'random' (hcat/loss.py:82-93) ----
// counts[r] = (#mask==1, #mask==0) in row r's element range
__global__ void __launch_bounds__(256)
loss_random_count_kernel(LossGeom g, int64_t chunk, int *counts) {
  __shared__ double red[512];
  const int r = blockIdx.x, tid = threadIdx.x;
  const int64_t beg = (int64_t)r * chunk, end = min(beg + chunk, g.n);
  double np = 0.0, nn = 0.0;
  for (int64_t e = beg + tid; e < end; e += 256) {
    int z;
    const float m = lx_load(g.mask, g.mdt, lx_mask_index(g, e, z));
    np += m == 1.f ? 1.0 : 0.0;
    nn += m == 0.f ? 1.0 : 0.0;
  }
  lx_block_sum2(np, nn, red);
  if (tid == 0) {
    counts[r * 2] = (int)np;
    counts[r * 2 + 1] = (int)nn;
  }
}

// Element indices of the mask==1 / mask==0 pixels in flat order
// (pred[mask == 1] order), row r writing from its exclusive offsets.
__global__ void __launch_bounds__(256)
loss_random_compact_kernel(LossGeom g, int64_t chunk, const int *offsets, int *pos_list,
                           int *neg_list) {
  __shared__ int sp[256], sn[256];
  const int r = blockIdx.x, tid = threadIdx.x;
  const int64_t beg = (int64_t)r * chunk, end = min(beg + chunk, g.n);
  int op = offsets[r * 2], on = offsets[r * 2 + 1];
  for (int64_t e0 = beg; e0 < end; e0 += 256) {
    const int64_t e = e0 + tid;
    int isp = 0, isn = 0;
    if (e < end) {
      int z;
      const float m = lx_load(g.mask, g.mdt, lx_mask_index(g, e, z));
      isp = m == 1.f;
      isn = m == 0.f;
    }
    sp[tid] = isp;
    sn[tid] = isn;
    __syncthreads();
    // inclusive Hillis-Steele scan (256 entries)
    for (int off = 1; off < 256; off <<= 1) {
      const int ap = tid >= off ? sp[tid - off] : 0, an = tid >= off ? sn[tid - off] : 0;
      __syncthreads();
      sp[tid] += ap;
      sn[tid] += an;
      __syncthreads();
    }
    if (isp) pos_list[op + sp[tid] - 1] = (int)e;
    if (isn) neg_list[on + sn[tid] - 1] = (int)e;
    const int tp = sp[255], tn = sn[255];
    __syncthreads();
    op += tp;
    on += tn;
  }
}

// Gather of the 2n drawn pixels: BCE partial sums and per-pixel draw counts.
__global__ void __launch_bounds__(256)
loss_random_gather_kernel(LossGeom g, const int *pos_list, const int *neg_list,
                          const int64_t *pos_ind, const int64_t *neg_ind, int n, int *cnt,
                          double *part) {
  __shared__ double red[512];
  const int tid = threadIdx.x;
  double s = 0.0, u = 0.0;
  for (int i = blockIdx.x * 256 + tid; i < 2 * n; i += gridDim.x * 256) {
    const int e = i < n ? pos_list[pos_ind[i]] : neg_list[neg_ind[i - n]];
    int z;
    const float m = lx_load(g.mask, g.mdt, lx_mask_index(g, e, z));
    s += (double)lx_bce(g.pred[e], m);
    if (cnt) atomicAdd(cnt + e, 1);   // integer: order-independent
  }
  lx_block_sum2(s, u, red);
  if (tid == 0) {
    part[blockIdx.x * 2] = s;
    part[blockIdx.x * 2 + 1] = 0.0;
  }
}

static int lx_rows(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 1023) / 1024, 1024));
}

static int lx_geom(LossGeom &g, const float *pred, int B, int C, int PX, int PY, int PZ,
                   const void *mask, int mdt, const void *pwl, int wdt, int MX, int MY, int MZ) {
  if (!pred || !mask) return fail(HCU_ERR_INVALID, "loss: null argument");
  if (B <= 0 || C <= 0 || PX <= 0 || PY <= 0 || PZ <= 0) return fail(HCU_ERR_SHAPE, "loss: empty prediction");
  if (MX < PX || MY < PY || MZ < PZ) return fail(HCU_ERR_SHAPE, "loss: mask smaller than the prediction");
  if (mdt < 0 || mdt > 2 || wdt < 0 || wdt > 1) return fail(HCU_ERR_INVALID, "loss: unsupported dtype");
  g.pred = pred;
  g.PX = PX;
  g.PY = PY;
  g.PZ = PZ;
  g.n = (int64_t)B * C * PX * PY * PZ;
  if (g.n >= ((int64_t)1 << 31)) return fail(HCU_ERR_SHAPE, "loss: more than 2^31 elements");
  g.mask = mask;
  g.mdt = mdt;
  g.pwl = pwl;
  g.wdt = wdt;
  g.MX = MX;
  g.MY = MY;
  g.MZ = MZ;
  return 0;
}

}  // namespace hcu

using namespace hcu;

extern "C" {

size_t hcu_loss_ext_scratch_bytes(int mode, int64_t n_pred, int PZ) {
  const int64_t rows = mode == LM_WORSTZ ? lx_rows(n_pred / std::max(1, PZ)) * (int64_t)std::max(1, PZ)
                                         : lx_rows(n_pred);
  return (size_t)rows * 2 * sizeof(double) + 64;
}

int hcu_loss_ext_fwd(int mode, const float *pred, int B, int C, int PX, int PY, int PZ,
                     const void *mask, int mask_dtype, const void *pwl, int pwl_dtype, int MX,
                     int MY, int MZ, const float *zscale, float *loss, float *aux, void *scratch,
                     size_t scratch_bytes, hcu_stream_t stream) {
  LossGeom g;
  if (int e = lx_geom(g, pred, B, C, PX, PY, PZ, mask, mask_dtype, pwl, pwl_dtype, MX, MY, MZ)) return e;
  if (mode < LM_SIGMOID || mode > LM_BCE) return fail(HCU_ERR_INVALID, "loss: unknown mode");
  if (!loss || !aux || !scratch) return fail(HCU_ERR_INVALID, "loss: null argument");
  if (scratch_bytes < hcu_loss_ext_scratch_bytes(mode, g.n, PZ))
    return fail(HCU_ERR_WORKSPACE, "loss: scratch too small");
  hipStream_t s = (hipStream_t)stream;
  double *part = (double *)scratch;
  if (mode == LM_WORSTZ) {
    if (!zscale || PZ > 1024) return fail(HCU_ERR_INVALID, "loss worst_z: zscale missing or Z > 1024");
    const int64_t nrows = g.n / PZ;
    const int R = lx_rows(nrows);
    const int64_t chunk = (nrows + R - 1) / R;
    HCU_TIMED(s, "loss_ext_fwd_kernel", 0.0, 0.0,
              HCU_LAUNCH(loss_ext_fwd_kernel, dim3(R, PZ), dim3(256), 0, s, g, mode, part, chunk));
    HCU_CHECK_LAUNCH();
    HCU_TIMED(s, "loss_ext_finalize_kernel", 0.0, 0.0,
              HCU_LAUNCH(loss_ext_finalize_kernel, dim3(1), dim3(256), 0, s, part, R, PZ, mode,
                                 (double)g.n, (double)PX * PY, zscale, loss, aux));
    HCU_CHECK_LAUNCH();
    return 0;
  }
  const int R = lx_rows(g.n);
  const int64_t chunk = (g.n + R - 1) / R;
  HCU_TIMED(s, "loss_ext_fwd_kernel", 0.0, 0.0,
            HCU_LAUNCH(loss_ext_fwd_kernel, dim3(R), dim3(256), 0, s, g, mode, part, chunk));
  HCU_CHECK_LAUNCH();
  HCU_TIMED(s, "loss_ext_finalize_kernel", 0.0, 0.0,
            HCU_LAUNCH(loss_ext_finalize_kernel, dim3(1), dim3(256), 0, s, part, R, 0, mode,
                               (double)g.n, (double)PX * PY, zscale, loss, aux));
  HCU_CHECK_LAUNCH();
  return 0;
}

int hcu_loss_ext_bwd(int mode, const float *pred, int B, int C, int PX, int PY, int PZ,
                     const void *mask, int mask_dtype, const void *pwl, int pwl_dtype, int MX,
                     int MY, int MZ, const float *aux, const int *counts, const float *grad_out,
                     float *dpred, hcu_stream_t stream) {
  LossGeom g;
  if (int e = lx_geom(g, pred, B, C, PX, PY, PZ, mask, mask_dtype, pwl, pwl_dtype, MX, MY, MZ)) return e;
  if (mode < LM_SIGMOID || mode > LM_RANDOM) return fail(HCU_ERR_INVALID, "loss: unknown mode");
  if (!aux || !dpred || (mode == LM_RANDOM && !counts)) return fail(HCU_ERR_INVALID, "loss: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((g.n + 255) / 256, 4096));
  HCU_TIMED(s, "loss_ext_bwd_kernel", 0.0, 0.0,
            HCU_LAUNCH(loss_ext_bwd_kernel, dim3(blocks), dim3(256), 0, s, g, mode, aux, counts,
                               grad_out, dpred));
  HCU_CHECK_LAUNCH();
  return 0;
}

int hcu_loss_random_rows(int64_t n_pred) { return lx_rows(n_pred); }

int hcu_loss_random_count(const float *pred, int B, int C, int PX, int PY, int PZ, const void *mask,
                          int mask_dtype, int MX, int MY, int MZ, int *counts, hcu_stream_t stream) {
  LossGeom g;
  if (int e = lx_geom(g, pred, B, C, PX, PY, PZ, mask, mask_dtype, nullptr, 0, MX, MY, MZ)) return e;
  if (!counts) return fail(HCU_ERR_INVALID, "loss: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int R = lx_rows(g.n);
  const int64_t chunk = (g.n + R - 1) / R;
  HCU_TIMED(s, "loss_random_count_kernel", 0.0, 0.0,
            HCU_LAUNCH(loss_random_count_kernel, dim3(R), dim3(256), 0, s, g, chunk, counts));
  HCU_CHECK_LAUNCH();
  return 0;
}

int hcu_loss_random_fwd(const float *pred, int B, int C, int PX, int PY, int PZ, const void *mask,
                        int mask_dtype, int MX, int MY, int MZ, const int *offsets, int *pos_list,
                        int *neg_list, const int64_t *pos_ind, const int64_t *neg_ind, int n,
                        int *counts, float *loss, float *aux, void *scratch, size_t scratch_bytes,
                        hcu_stream_t stream) {
  LossGeom g;
  if (int e = lx_geom(g, pred, B, C, PX, PY, PZ, mask, mask_dtype, nullptr, 0, MX, MY, MZ)) return e;
  if (!offsets || !pos_list || !neg_list || !pos_ind || !neg_ind || !loss || !aux || !scratch || n < 1)
    return fail(HCU_ERR_INVALID, "loss random: null argument");
  const int RG = (int)std::min<int64_t>(1024, (2 * (int64_t)n + 255) / 256);
  if (scratch_bytes < (size_t)RG * 2 * sizeof(double)) return fail(HCU_ERR_WORKSPACE, "loss: scratch too small");
  hipStream_t s = (hipStream_t)stream;
  const int R = lx_rows(g.n);
  const int64_t chunk = (g.n + R - 1) / R;
  HCU_TIMED(s, "loss_random_compact_kernel", 0.0, 0.0,
            HCU_LAUNCH(loss_random_compact_kernel, dim3(R), dim3(256), 0, s, g, chunk, offsets,
                               pos_list, neg_list));
  HCU_CHECK_LAUNCH();
  double *part = (double *)scratch;
  HCU_TIMED(s, "loss_random_gather_kernel", 0.0, 0.0,
            HCU_LAUNCH(loss_random_gather_kernel, dim3(RG), dim3(256), 0, s, g, pos_list, neg_list,
                               pos_ind, neg_ind, n, counts, part));
  HCU_CHECK_LAUNCH();
  HCU_TIMED(s, "loss_ext_finalize_kernel", 0.0, 0.0,
            HCU_LAUNCH(loss_ext_finalize_kernel, dim3(1), dim3(256), 0, s, part, RG, 0,
                               (int)LM_RANDOM, 2.0 * n, 1.0, (const float *)nullptr, loss, aux));
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
