// HBM-bound kernels of the U-Net step: BatchNorm3d statistics finalisation
// (nn.BatchNorm3d train/eval semantics, hcat/unet.py:259-260,305-306),
// MaxPool3d forward/backward (hcat/unet.py:123,131), the BatchNorm+ReLU
// backward reductions, the out_conv 1x1x1 Conv3d (hcat/unet.py:120,138),
// NCXYZ <-> channels-last layout changes and the weight re-layouts feeding the
// implicit-GEMM kernels.
//
// Every reduction writes fixed-size per-workgroup partial rows that a second
// kernel sums in fp64 in a fixed order: results are bitwise reproducible run to
// run (no float atomics anywhere).
#include "common.h"
#include "timing.h"
#include <algorithm>

namespace hcu {

__device__ __forceinline__ float bnrelu(float y, float sc, float sh) {
  return fmaxf(fmaf(y, sc, sh), 0.f);
}
__device__ __forceinline__ float4 ld4(const float *p) {
  return *reinterpret_cast<const float4 *>(p);
}
__device__ __forceinline__ void st4(float *p, float4 v) {
  *reinterpret_cast<float4 *>(p) = v;
}
// Activation storage types: the fp32 path stores float, the bf16 path bf16
// (4 channels = 8 bytes); every kernel below computes in fp32 either way.
struct bf16_t {
  uint16_t v;
};
__device__ __forceinline__ float4 ld4(const bf16_t *p) {
  const uint2 u = *reinterpret_cast<const uint2 *>(p);
  return make_float4(bf_lo(u.x), bf_hi(u.x), bf_lo(u.y), bf_hi(u.y));
}
__device__ __forceinline__ void st4(bf16_t *p, float4 v) {
  *reinterpret_cast<uint2 *>(p) = make_uint2(pack_bf2(v.x, v.y), pack_bf2(v.z, v.w));
}
__device__ __forceinline__ float ld1(const float *p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t *p) { return bf2f(p->v); }
__device__ __forceinline__ float ld1(const _Float16 *p) { return (float)*p; }
__device__ __forceinline__ void st1(float *p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t *p, float v) { p->v = f2bf(v); }
#define HCU_BF_DISPATCH(bf, KERNEL, ...)                     \
  do {                                                       \
    if (bf) {                                                \
      using T = bf16_t;                                      \
      HCU_LAUNCH(KERNEL<T>, __VA_ARGS__);            \
    } else {                                                 \
      using T = float;                                       \
      HCU_LAUNCH(KERNEL<T>, __VA_ARGS__);            \
    }                                                        \
  } while (0)
__device__ __forceinline__ float comp(const float4 &v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// 16-byte channel vectors: 4 fp32 or 8 bf16 channels per thread.
template <typename T>
struct VN {
  static constexpr int N = 4;
};
template <>
struct VN<bf16_t> {
  static constexpr int N = 8;
};
__device__ __forceinline__ void ldv(const float *p, float (&f)[4]) {
  const float4 v = ld4(p);
  f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
}
__device__ __forceinline__ void ldv(const bf16_t *p, float (&f)[8]) {
  unpack8(*reinterpret_cast<const uint4 *>(p), f);
}
__device__ __forceinline__ void stv(float *p, const float (&f)[4]) {
  st4(p, make_float4(f[0], f[1], f[2], f[3]));
}
__device__ __forceinline__ void stv(bf16_t *p, const float (&f)[8]) {
  *reinterpret_cast<uint4 *>(p) = pack8(f);
}
template <int N>
__device__ __forceinline__ void ldc(const float *p, float (&f)[N]) {   // fp32 coefficients
#pragma unroll
  for (int k = 0; k < N; k += 4) {
    const float4 v = ld4(p + k);
    f[k] = v.x; f[k + 1] = v.y; f[k + 2] = v.z; f[k + 3] = v.w;
  }
}

// ---------------------------------------------------------------------------
// BatchNorm forward finalisation: one workgroup per channel.
//
// Statistics rows (StatRow, common.h) hold sums taken about a per-row pivot K
// (a value of the row's own data), so the fp32 partial sums never hold the
// large (y - 0)^2 terms whose difference E[y^2] - E[y]^2 would cancel when
// |mean| >> std (large conv biases, shifted inputs).  The rows are combined
// here in fp64, in a fixed order, by the parallel-variance identity:
//   mean = sum_r (S1_r + n_r K_r) / N
//   M2   = sum_r (S2_r - S1_r^2 / n_r) + sum_r n_r (K_r + S1_r / n_r - mean)^2
// Sum over the 256 threads: an xor butterfly of wave shuffles (IEEE addition
// is commutative, so both partners hold the same bits), then the 4 wave sums
// in a fixed order -- 2 barriers instead of a 9-barrier LDS tree.
__device__ double block_sum_f64(double v, double *red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ void __launch_bounds__(256)
bn_fwd_finalize_kernel(const float *stats, int R, int W, int C, double count,
                       const float *gamma, const float *beta, float *rm, float *rv,
                       const int64_t *nbt, float eps, float momentum, int training,
                       BNCoef coef) {
  __shared__ double red[256];
  const int c = blockIdx.x, tid = threadIdx.x;
  double m = 0.0, v = 0.0;
  if (training && c < C) {
    // a thread's first RC rows are loaded together (independent loads in
    // flight) and kept in registers for the second pass; the summation order
    // is the plain r = tid, tid + 256, ... order either way
    constexpr int RC = 8;
    float4 rows[RC];
#pragma unroll
    for (int k = 0; k < RC; ++k) {
      const int r = tid + 256 * k;
      rows[k] = r < R ? *reinterpret_cast<const float4 *>(stats + ((size_t)r * W + c) * 4)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    double t = 0.0, nn = 0.0;
#pragma unroll
    for (int k = 0; k < RC; ++k)
      if (rows[k].w > 0.f) {
        t += (double)rows[k].x + (double)rows[k].w * (double)rows[k].z;
        nn += (double)rows[k].w;
      }
    for (int r = tid + 256 * RC; r < R; r += 256) {
      const float4 row = *reinterpret_cast<const float4 *>(stats + ((size_t)r * W + c) * 4);
      if (row.w > 0.f) {
        t += (double)row.x + (double)row.w * (double)row.z;
        nn += (double)row.w;
      }
    }
    const double tot = block_sum_f64(t, red);
    const double ntot = block_sum_f64(nn, red);
    m = tot / ntot;
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < RC; ++k)
      if (rows[k].w > 0.f) {
        const double n = rows[k].w, s1 = rows[k].x;
        const double d = (double)rows[k].z + s1 / n - m;
        q += ((double)rows[k].y - s1 * s1 / n) + n * d * d;
      }
    for (int r = tid + 256 * RC; r < R; r += 256) {
      const float4 row = *reinterpret_cast<const float4 *>(stats + ((size_t)r * W + c) * 4);
      if (row.w > 0.f) {
        const double n = row.w, s1 = row.x;
        const double d = (double)row.z + s1 / n - m;
        q += ((double)row.y - s1 * s1 / n) + n * d * d;
      }
    }
    v = block_sum_f64(q, red) / ntot;
  }
  if (tid != 0) return;
  if (c >= C) {
    coef.scale[c] = coef.shift[c] = coef.mean[c] = coef.invstd[c] = 0.f;
    coef.c1[c] = coef.c0[c] = 0.f;
    return;
  }
  float mean, invstd;
  if (training) {
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    invstd = (float)(1.0 / sqrt(v + (double)eps));
    if (rm) {
      const double f = momentum >= 0.f ? (double)momentum : 1.0 / (double)(nbt[0] + 1);
      const double unb = count > 1.0 ? v * count / (count - 1.0) : v;
      rm[c] = (float)(f * m + (1.0 - f) * (double)rm[c]);
      rv[c] = (float)(f * unb + (1.0 - f) * (double)rv[c]);
    }
  } else {
    mean = rm[c];
    invstd = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
  }
  const float g = gamma ? gamma[c] : 1.f;
  const float bb = beta ? beta[c] : 0.f;
  const float sc = g * invstd;
  coef.scale[c] = sc;
  coef.shift[c] = bb - mean * sc;
  coef.mean[c] = mean;
  coef.invstd[c] = invstd;
}

int launch_bn_fwd_finalize(const float *stats, int R, int statsW, int C, int Cs,
                           double count, const float *gamma, const float *beta,
                           float *run_mean, float *run_var, int64_t *nbt,
                           float eps, float momentum, int training, BNCoef coef,
                           hipStream_t s) {
  HCU_TIMED(s, "bn_fwd_finalize_kernel", 0.0, 0.0, HCU_LAUNCH(bn_fwd_finalize_kernel, dim3(Cs), dim3(256), 0, s, stats, R,
                     statsW, C, count, gamma, beta, run_mean, run_var, nbt, eps,
                     momentum, training, coef));
  HCU_CHECK_LAUNCH();
  return 0;
}

// BatchNorm backward finalisation: per channel sum dz and sum dz*xhat.
__global__ void __launch_bounds__(256)
bn_bwd_finalize_kernel(const float *part, int R, int C, int W, double count,
                       BNCoef coef, float *dgamma, float *dbeta, int training,
                       int accumulate) {
  __shared__ double r1[256], r2[256];
  const int c = blockIdx.x, tid = threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
#pragma unroll 8
    for (int r = tid; r < R; r += 256) {
      const float2 p2 = *reinterpret_cast<const float2 *>(part + ((size_t)r * W + c) * 2);
      s1 += (double)p2.x;
      s2 += (double)p2.y;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
  }
  if ((tid & 63) == 0) {
    r1[tid >> 6] = s1;
    r2[tid >> 6] = s2;
  }
  __syncthreads();
  if (tid != 0) return;
  r1[0] = ((r1[0] + r1[1]) + r1[2]) + r1[3];
  r2[0] = ((r2[0] + r2[1]) + r2[2]) + r2[3];
  if (c >= C) {
    coef.c1[c] = coef.c0[c] = 0.f;
    return;
  }
  const double db = r1[0], dg = r2[0];
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)db : (float)db;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)dg : (float)dg;
  if (training) {
    const double sc = coef.scale[c], is = coef.invstd[c], mu = coef.mean[c];
    const double c1 = -sc * is * dg / count;
    const double c0 = -sc * db / count - c1 * mu;
    coef.c1[c] = (float)c1;
    coef.c0[c] = (float)c0;
  } else {
    coef.c1[c] = 0.f;
    coef.c0[c] = 0.f;
  }
}

int launch_bn_bwd_finalize(const float *part, int R, int C, int Cs, int W, double count,
                           BNCoef coef, float *dgamma, float *dbeta, int training,
                           int accumulate, hipStream_t s) {
  HCU_TIMED(s, "bn_bwd_finalize_kernel", 0.0, 0.0, HCU_LAUNCH(bn_bwd_finalize_kernel, dim3(Cs), dim3(256), 0, s, part, R, C,
                     W, count, coef, dgamma, dbeta, training, accumulate));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// MaxPool3d forward on relu(bn(y)), kernel == stride, floor mode.
// Index decomposition (window, channel quad) -> (b, px, py, pz, c4) with
// magic-number divisions on 32-bit indices (the launcher checks the range):
// 64-bit division is a ~100-instruction software sequence per element.
struct PoolDiv {
  FastDiv c4, pz, py, px;
};
template <typename T>
__global__ void __launch_bounds__(256)
maxpool_fwd_kernel(const T *y, const float *scale, const float *shift, T *p,
                   int B, int X, int Y, int Z, int Cs, int kx, int ky, int kz,
                   int PX, int PY, int PZ, PoolDiv dv) {
  const uint32_t n = (uint32_t)B * PX * PY * PZ * (Cs / 4);
  for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < n; idx += gridDim.x * 256) {
    int v, c4, pz, py, px, b;
    dv.c4.divmod(idx, v, c4);
    dv.pz.divmod((uint32_t)v, v, pz);
    dv.py.divmod((uint32_t)v, v, py);
    dv.px.divmod((uint32_t)v, b, px);
    const int c = c4 * 4;
    float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
    if (scale) {
      sc = ld4(scale + c);
      sh = ld4(shift + c);
    }
    float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    for (int i = 0; i < kx; ++i)
      for (int j = 0; j < ky; ++j)
        for (int k = 0; k < kz; ++k) {
          const int x = px * kx + i, yy = py * ky + j, z = pz * kz + k;
          const float4 t = ld4(y + ((((size_t)b * X + x) * Y + yy) * Z + z) * Cs + c);
          float4 a;
          if (scale) {
            a.x = bnrelu(t.x, sc.x, sh.x);
            a.y = bnrelu(t.y, sc.y, sh.y);
            a.z = bnrelu(t.z, sc.z, sh.z);
            a.w = bnrelu(t.w, sc.w, sh.w);
          } else {
            a = t;
          }
          m.x = a.x > m.x ? a.x : m.x;
          m.y = a.y > m.y ? a.y : m.y;
          m.z = a.z > m.z ? a.z : m.z;
          m.w = a.w > m.w ? a.w : m.w;
        }
    st4(p + ((((size_t)b * PX + px) * PY + py) * PZ + pz) * Cs + c, m);
  }
}

// MaxPool3d (2,2,1) on relu(bn(y)): one (window, 16-byte channel vector) per
// thread, the window's 4 vectors loaded together.
template <typename T>
__global__ void __launch_bounds__(256)
maxpool221_kernel(const T *y, const float *scale, const float *shift, T *p, int X, int Y, int Z,
                  int Cs, int PX, int PY, uint32_t n, PoolDiv dv) {
  constexpr int N = VN<T>::N;
  const uint32_t idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= n) return;
  int v, g, pz, py, px, b;
  dv.c4.divmod(idx, v, g);
  dv.pz.divmod((uint32_t)v, v, pz);
  dv.py.divmod((uint32_t)v, v, py);
  dv.px.divmod((uint32_t)v, b, px);
  const int c = g * N;
  const size_t sy = (size_t)Z * Cs, sx = (size_t)Y * sy;
  const size_t base = (((size_t)b * X + 2 * px) * Y + 2 * py) * sy + (size_t)pz * Cs + c;
  float a[4][N];
  ldv(y + base, a[0]);
  ldv(y + base + sy, a[1]);
  ldv(y + base + sx, a[2]);
  ldv(y + base + sx + sy, a[3]);
  float m[N];
  if (scale) {
    float sc[N], sh[N];
    ldc<N>(scale + c, sc);
    ldc<N>(shift + c, sh);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      m[j] = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float q = bnrelu(a[t][j], sc[j], sh[j]);
        m[j] = q > m[j] ? q : m[j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      m[j] = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t) m[j] = a[t][j] > m[j] ? a[t][j] : m[j];
    }
  }
  stv(p + ((((size_t)b * PX + px) * PY + py) * Z + pz) * Cs + c, m);
}

static int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

static PoolDiv pool_div(int Cs, int PX, int PY, int PZ) {
  PoolDiv d;
  d.c4 = FastDiv(Cs / 4);
  d.pz = FastDiv(PZ);
  d.py = FastDiv(PY);
  d.px = FastDiv(PX);
  return d;
}

int launch_maxpool_fwd(const float *y, const float *scale, const float *shift,
                       float *p, int B, int X, int Y, int Z, int Cs, int kx, int ky,
                       int kz, hipStream_t s, int bf) {
  const int PX = X / kx, PY = Y / ky, PZ = Z / kz;
  const int64_t n = (int64_t)B * PX * PY * PZ * (Cs / 4);
  if (n >= (int64_t)1 << 31) return fail(4, "max_pool3d: more than 2^31 channel quads per launch");
  if (kx == 2 && ky == 2 && kz == 1 && n > 0) {
    const int N = bf ? 8 : 4;
    if (Cs % N == 0) {
      const int64_t nv = (int64_t)B * PX * PY * PZ * (Cs / N);
      // y read, the pooled tensor written
      HCU_TIMED(s, "maxpool221_kernel", 0.0, (double)(bf ? 2 : 4) * Cs * ((double)B * X * Y * Z + (double)B * PX * PY * PZ),
                HCU_BF_DISPATCH(bf, maxpool221_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s,
                                (const T *)y, scale, shift, (T *)p, X, Y, Z, Cs, PX, PY, (uint32_t)nv,
                                pool_div(Cs * 4 / N, PX, PY, PZ)));
      HCU_CHECK_LAUNCH();
      return 0;
    }
  }
  HCU_TIMED(s, "maxpool_fwd_kernel", 0.0, 0.0,
            HCU_BF_DISPATCH(bf, maxpool_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, s,
                            (const T *)y, scale, shift, (T *)p, B, X, Y, Z, Cs, kx, ky, kz, PX,
                            PY, PZ, pool_div(Cs, PX, PY, PZ)));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Row partitioning shared by the per-channel reductions: workgroup r handles
// the element range [r*chunk, (r+1)*chunk) of the (voxel, channel-quad) space.
struct RedGeom {
  int tb;          // threads per workgroup (multiple of C4)
  int64_t chunk;   // elements per workgroup (multiple of tb)
  int64_t total;
};
__host__ __device__ inline RedGeom red_geom(int64_t nvox, int Cs, int R) {
  RedGeom g;
  const int C4 = Cs / 4;
  g.tb = C4 <= 256 ? (256 / C4) * C4 : C4;
  g.total = nvox * C4;
  int64_t per = (g.total + R - 1) / R;
  g.chunk = (per + g.tb - 1) / g.tb * g.tb;
  return g;
}
int bwd_rows(int64_t nvox, int Cs) {
  const int C4 = Cs / 4;
  const int tb = C4 <= 256 ? (256 / C4) * C4 : C4;
  const int64_t total = nvox * C4;
  int64_t r = (total + (int64_t)tb * 4 - 1) / ((int64_t)tb * 4);
  return (int)std::max<int64_t>(1, std::min<int64_t>(r, 1024));
}
int chansum_rows(int64_t nvox, int Cs) { return bwd_rows(nvox, Cs); }
int outconv_bwd_rows(int64_t nvox, int Cs) { return bwd_rows(nvox, Cs); }

// Fixed-order block reduction of NV floats per thread, grouped by c4.
template <int NV>
__device__ void block_reduce_c4(float (&v)[NV], float *lds, int tb, int C4,
                                float *out_row /* [C4][NV] */) {
  const int tid = threadIdx.x;
  if (tid < tb)
    for (int k = 0; k < NV; ++k) lds[tid * NV + k] = v[k];
  __syncthreads();
  if (tid < C4) {
    float acc[NV];
    for (int k = 0; k < NV; ++k) acc[k] = 0.f;
    for (int t = tid; t < tb; t += C4)
      for (int k = 0; k < NV; ++k) acc[k] += lds[t * NV + k];
    for (int k = 0; k < NV; ++k) out_row[tid * NV + k] = acc[k];
  }
}

// dz = dA * [z > 0] in place, partial (sum dz, sum dz*xhat) per channel.
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_reduce_dense_kernel(T *dA, const T *y, BNCoef coef, int64_t nvox,
                           int Cs, float *part, RedGeom g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int C4 = Cs / 4, tid = threadIdx.x;
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (tid < g.tb) {
    const int64_t beg = (int64_t)blockIdx.x * g.chunk;
    const int64_t end = std::min(beg + g.chunk, g.total);
    const int c = (int)((beg + tid) % C4) * 4;
    const float4 sc = ld4(coef.scale + c), sh = ld4(coef.shift + c);
    const float4 mu = ld4(coef.mean + c), is = ld4(coef.invstd + c);
    // e = vox * C4 + c / 4 with c fixed per thread: off = e * 4 exactly
    for (int64_t e = beg + tid; e < end; e += g.tb) {
      const size_t off = (size_t)e * 4;
      const float4 yy = ld4(y + off);
      float4 d = ld4(dA + off);
      d.x = fmaf(yy.x, sc.x, sh.x) > 0.f ? d.x : 0.f;
      d.y = fmaf(yy.y, sc.y, sh.y) > 0.f ? d.y : 0.f;
      d.z = fmaf(yy.z, sc.z, sh.z) > 0.f ? d.z : 0.f;
      d.w = fmaf(yy.w, sc.w, sh.w) > 0.f ? d.w : 0.f;
      st4(dA + off, d);
      v[0] += d.x;
      v[1] = fmaf(d.x, (yy.x - mu.x) * is.x, v[1]);
      v[2] += d.y;
      v[3] = fmaf(d.y, (yy.y - mu.y) * is.y, v[3]);
      v[4] += d.z;
      v[5] = fmaf(d.z, (yy.z - mu.z) * is.z, v[5]);
      v[6] += d.w;
      v[7] = fmaf(d.w, (yy.w - mu.w) * is.w, v[7]);
    }
  }
  block_reduce_c4<8>(v, lds, g.tb, C4, part + (size_t)blockIdx.x * Cs * 2);
}

int launch_bn_bwd_reduce_dense(float *dA, const float *y, BNCoef coef, int64_t nvox,
                               int Cs, float *part, int R, hipStream_t s, int bf) {
  const RedGeom g = red_geom(nvox, Cs, R);
  HCU_TIMED(s, "bn_bwd_reduce_dense_kernel", 0.0, 2.0 * nvox * Cs * (bf ? 2 : 4),
            HCU_BF_DISPATCH(bf, bn_bwd_reduce_dense_kernel, dim3(R), dim3(256),
                            (size_t)std::max(g.tb, 256) * 8 * 4, s, (T *)dA, (const T *)y, coef,
                            nvox, Cs, part, g));
  HCU_CHECK_LAUNCH();
  return 0;
}

// Max-pool backward (argmax recomputed from y, first maximum in x,y,z window
// order as torch's CPU max_pool3d) fused with the BatchNorm+ReLU reduction.
// One thread per (pool window, channel quad): the window's y values are read
// once, and dz is written for the window's voxels plus, for windows on the
// last row/column/plane, the floor-mode remainder (which gets 0), so every
// voxel of y is written exactly once and y is read from HBM once.
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_reduce_pool_kernel(const T *dP, const T *y, BNCoef coef, T *dz,
                          int B, int X, int Y, int Z, int Cs, int kx, int ky, int kz,
                          float *part, RedGeom g, PoolDiv dv) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int C4 = Cs / 4, tid = threadIdx.x;
  const int PX = X / kx, PY = Y / ky, PZ = Z / kz;
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (tid < g.tb) {
    const int64_t beg = (int64_t)blockIdx.x * g.chunk;
    const int64_t end = std::min(beg + g.chunk, g.total);
    const int c = (int)((beg + tid) % C4) * 4;
    const float4 sc = ld4(coef.scale + c), sh = ld4(coef.shift + c);
    const float4 mu = ld4(coef.mean + c), is = ld4(coef.invstd + c);
    for (int64_t e = beg + tid; e < end; e += g.tb) {
      int w, c4, wz, wy, wx, b;
      dv.c4.divmod((uint32_t)e, w, c4);
      dv.pz.divmod((uint32_t)w, w, wz);
      dv.py.divmod((uint32_t)w, w, wy);
      dv.px.divmod((uint32_t)w, b, wx);
      const int x0 = wx * kx, y0 = wy * ky, z0 = wz * kz;
      const int x1 = wx == PX - 1 ? X : x0 + kx, y1 = wy == PY - 1 ? Y : y0 + ky,
                z1 = wz == PZ - 1 ? Z : z0 + kz;
      // argmax of relu(bn(y)) over the window, first maximum wins
      float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      int4 am = make_int4(-1, -1, -1, -1);
      int idx = 0;
      for (int i = 0; i < kx; ++i)
        for (int j = 0; j < ky; ++j)
          for (int k = 0; k < kz; ++k, ++idx) {
            const float4 t = ld4(y + ((((size_t)b * X + x0 + i) * Y + y0 + j) * Z + z0 + k) * Cs + c);
            const float a0 = bnrelu(t.x, sc.x, sh.x), a1 = bnrelu(t.y, sc.y, sh.y);
            const float a2 = bnrelu(t.z, sc.z, sh.z), a3 = bnrelu(t.w, sc.w, sh.w);
            if (a0 > m.x) { m.x = a0; am.x = idx; }
            if (a1 > m.y) { m.y = a1; am.y = idx; }
            if (a2 > m.z) { m.z = a2; am.z = idx; }
            if (a3 > m.w) { m.w = a3; am.w = idx; }
          }
      const float4 gp = ld4(dP + ((((size_t)b * PX + wx) * PY + wy) * PZ + wz) * Cs + c);
      for (int x = x0; x < x1; ++x)
        for (int yy = y0; yy < y1; ++yy)
          for (int z = z0; z < z1; ++z) {
            const size_t off = ((((size_t)b * X + x) * Y + yy) * Z + z) * Cs + c;
            float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
            const bool inwin = x < x0 + kx && yy < y0 + ky && z < z0 + kz;
            if (inwin) {
              const int own = ((x - x0) * ky + (yy - y0)) * kz + (z - z0);
              const float4 yv = ld4(y + off);   // L1/L2 hit: read just above
              const float4 zv = make_float4(fmaf(yv.x, sc.x, sh.x), fmaf(yv.y, sc.y, sh.y),
                                            fmaf(yv.z, sc.z, sh.z), fmaf(yv.w, sc.w, sh.w));
              d.x = (am.x == own && zv.x > 0.f) ? gp.x : 0.f;
              d.y = (am.y == own && zv.y > 0.f) ? gp.y : 0.f;
              d.z = (am.z == own && zv.z > 0.f) ? gp.z : 0.f;
              d.w = (am.w == own && zv.w > 0.f) ? gp.w : 0.f;
              v[0] += d.x;
              v[1] = fmaf(d.x, (yv.x - mu.x) * is.x, v[1]);
              v[2] += d.y;
              v[3] = fmaf(d.y, (yv.y - mu.y) * is.y, v[3]);
              v[4] += d.z;
              v[5] = fmaf(d.z, (yv.z - mu.z) * is.z, v[5]);
              v[6] += d.w;
              v[7] = fmaf(d.w, (yv.w - mu.w) * is.w, v[7]);
            }
            st4(dz + off, d);
          }
    }
  }
  block_reduce_c4<8>(v, lds, g.tb, C4, part + (size_t)blockIdx.x * Cs * 2);
}

// The same for MaxPool3d (2,2,1) with 16-byte channel vectors (4 fp32 / 8
// bf16 channels) and two windows per iteration: the 2 x (4 + 1) vector loads
// are issued together.  Per-thread channel group fixed (tb multiple of G);
// accumulation order per channel is the generic kernel's (window order, then
// the window's taps x-major), so partial rows are reproducible.
template <int N>
struct Win221 {
  float a[4][N], gp[N];
  int wx, wy, wz, b;
  bool ok;
};
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_reduce_pool221_kernel(const T *dP, const T *y, BNCoef coef, T *dz, int X, int Y, int Z,
                             int Cs, float *part, RedGeom g, PoolDiv dv) {
  constexpr int N = VN<T>::N;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int G = Cs / N, tid = threadIdx.x;
  const int PX = X / 2, PY = Y / 2;
  const size_t sy = (size_t)Z * Cs, sx = (size_t)Y * sy;
  float v[2 * N];
#pragma unroll
  for (int k = 0; k < 2 * N; ++k) v[k] = 0.f;
  if (tid < g.tb) {
    const int64_t beg = (int64_t)blockIdx.x * g.chunk;
    const int64_t end = std::min(beg + g.chunk, g.total);
    const int c = (int)((beg + tid) % G) * N;
    float sc[N], sh[N], mu[N], is[N];
    ldc<N>(coef.scale + c, sc);
    ldc<N>(coef.shift + c, sh);
    ldc<N>(coef.mean + c, mu);
    ldc<N>(coef.invstd + c, is);
    auto load = [&](int64_t e, Win221<N> &w) {
      w.ok = e < end;
      if (!w.ok) return;
      int q, gg;
      dv.c4.divmod((uint32_t)e, q, gg);
      dv.pz.divmod((uint32_t)q, q, w.wz);
      dv.py.divmod((uint32_t)q, q, w.wy);
      dv.px.divmod((uint32_t)q, w.b, w.wx);
      const size_t base = (((size_t)w.b * X + 2 * w.wx) * Y + 2 * w.wy) * sy + (size_t)w.wz * Cs + c;
      ldv(y + base, w.a[0]);
      ldv(y + base + sy, w.a[1]);
      ldv(y + base + sx, w.a[2]);
      ldv(y + base + sx + sy, w.a[3]);
      ldv(dP + ((((size_t)w.b * PX + w.wx) * PY + w.wy) * Z + w.wz) * Cs + c, w.gp);
    };
    auto finish = [&](const Win221<N> &w) {
      if (!w.ok) return;
      float d[4][N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        float m = -INFINITY;
        int am = -1;
        float zz[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          zz[t] = fmaf(w.a[t][j], sc[j], sh[j]);
          const float q = fmaxf(zz[t], 0.f);
          if (q > m) { m = q; am = t; }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) d[t][j] = (am == t && zz[t] > 0.f) ? w.gp[j] : 0.f;
      }
      const size_t base = (((size_t)w.b * X + 2 * w.wx) * Y + 2 * w.wy) * sy + (size_t)w.wz * Cs + c;
      stv(dz + base, d[0]);
      stv(dz + base + sy, d[1]);
      stv(dz + base + sx, d[2]);
      stv(dz + base + sx + sy, d[3]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < N; ++j) {
          v[2 * j] += d[t][j];
          v[2 * j + 1] = fmaf(d[t][j], (w.a[t][j] - mu[j]) * is[j], v[2 * j + 1]);
        }
      // floor mode: the last row / column of windows also owns the dropped voxels (gradient 0)
      const bool lx = w.wx == PX - 1 && X > 2 * PX, ly = w.wy == PY - 1 && Y > 2 * PY;
      if (lx || ly) {
        float zero[N];
#pragma unroll
        for (int j = 0; j < N; ++j) zero[j] = 0.f;
        const int x1 = lx ? X : 2 * w.wx + 2, y1 = ly ? Y : 2 * w.wy + 2;
        for (int x = 2 * w.wx; x < x1; ++x)
          for (int yy = 2 * w.wy; yy < y1; ++yy)
            if (x >= 2 * w.wx + 2 || yy >= 2 * w.wy + 2)
              stv(dz + (((size_t)w.b * X + x) * Y + yy) * sy + (size_t)w.wz * Cs + c, zero);
      }
    };
    for (int64_t e = beg + tid; e < end; e += 2 * (int64_t)g.tb) {
      Win221<N> w0, w1;
      load(e, w0);
      load(e + g.tb, w1);
      finish(w0);
      finish(w1);
    }
  }
  // fixed-order reduction per channel group -> part[row][c][2]
  if (tid < g.tb)
#pragma unroll
    for (int k = 0; k < 2 * N; ++k) lds[tid * 2 * N + k] = v[k];
  __syncthreads();
  if (tid < G) {
    float acc[2 * N];
#pragma unroll
    for (int k = 0; k < 2 * N; ++k) acc[k] = 0.f;
    for (int t = tid; t < g.tb; t += G)
#pragma unroll
      for (int k = 0; k < 2 * N; ++k) acc[k] += lds[t * 2 * N + k];
    float *out = part + (size_t)blockIdx.x * Cs * 2 + (size_t)tid * 2 * N;
#pragma unroll
    for (int k = 0; k < 2 * N; ++k) out[k] = acc[k];
  }
}

int pool_bwd_rows(int B, int X, int Y, int Z, int Cs, int kx, int ky, int kz) {
  return bwd_rows((int64_t)B * (X / kx) * (Y / ky) * (Z / kz), Cs);
}

int launch_bn_bwd_reduce_pool(const float *dP, const float *y, BNCoef coef, float *dz,
                              int B, int X, int Y, int Z, int Cs, int kx, int ky,
                              int kz, float *part, int R, hipStream_t s, int bf) {
  const RedGeom g = red_geom((int64_t)B * (X / kx) * (Y / ky) * (Z / kz), Cs, R);
  if (g.total >= (int64_t)1 << 31) return fail(4, "max_pool3d backward: more than 2^31 channel quads");
  const int N = bf ? 8 : 4;
  if (kx == 2 && ky == 2 && kz == 1 && Cs % N == 0) {
    // red_geom over N-channel groups: pass Cs * 4 / N as the "quad" stride
    const RedGeom gv = red_geom((int64_t)B * (X / 2) * (Y / 2) * Z, Cs * 4 / N, R);
    // the pooled gradient and y read, dz written
    HCU_TIMED(s, "bn_bwd_reduce_pool221_kernel", 0.0,
              (double)(bf ? 2 : 4) * Cs * ((double)B * (X / 2) * (Y / 2) * Z + 2.0 * B * X * Y * Z),
              HCU_BF_DISPATCH(bf, bn_bwd_reduce_pool221_kernel, dim3(R), dim3(256),
                              (size_t)std::max(gv.tb, 256) * 2 * N * 4, s, (const T *)dP, (const T *)y,
                              coef, (T *)dz, X, Y, Z, Cs, part, gv, pool_div(Cs * 4 / N, X / 2, Y / 2, Z)));
    HCU_CHECK_LAUNCH();
    return 0;
  }
  HCU_TIMED(s, "bn_bwd_reduce_pool_kernel", 0.0, 0.0,
            HCU_BF_DISPATCH(bf, bn_bwd_reduce_pool_kernel, dim3(R), dim3(256),
                            (size_t)std::max(g.tb, 256) * 8 * 4, s, (const T *)dP, (const T *)y,
                            coef, (T *)dz, B, X, Y, Z, Cs, kx, ky, kz, part, g,
                            pool_div(Cs, X / kx, Y / ky, Z / kz)));
  HCU_CHECK_LAUNCH();
  return 0;
}

// dy = dz*scale + c1*y + c0, in place.
// The launcher makes the grid stride a multiple of C4, so each thread's channel
// quad (and its coefficients) is fixed; 4 independent quads per iteration keep
// 8 loads in flight per thread.
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_apply_kernel(T *dz, const T *y, BNCoef coef, int64_t n4, int C4) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t st = (int64_t)gridDim.x * 256;
  const int c = (int)(i0 % C4) * 4;
  const float4 sc = ld4(coef.scale + c), c1 = ld4(coef.c1 + c), c0 = ld4(coef.c0 + c);
  auto f = [&](float4 d, float4 yy) {
    d.x = fmaf(d.x, sc.x, fmaf(c1.x, yy.x, c0.x));
    d.y = fmaf(d.y, sc.y, fmaf(c1.y, yy.y, c0.y));
    d.z = fmaf(d.z, sc.z, fmaf(c1.z, yy.z, c0.z));
    d.w = fmaf(d.w, sc.w, fmaf(c1.w, yy.w, c0.w));
    return d;
  };
  int64_t i = i0;
  for (; i + 3 * st < n4; i += 4 * st) {
    float4 yy[4], d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      yy[u] = ld4(y + (i + u * st) * 4);
      d[u] = ld4(dz + (i + u * st) * 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) st4(dz + (i + u * st) * 4, f(d[u], yy[u]));
  }
  for (; i < n4; i += st) st4(dz + i * 4, f(ld4(dz + i * 4), ld4(y + i * 4)));
}

// The same with 16-byte channel vectors (8 bf16 channels per load on the bf16
// path), 4 vectors in flight per thread.
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_apply_vec_kernel(T *dz, const T *y, BNCoef coef, int64_t nv, int G) {
  constexpr int N = VN<T>::N;
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t st = (int64_t)gridDim.x * 256;
  const int c = (int)(i0 % G) * N;
  float sc[N], c1[N], c0[N];
  ldc<N>(coef.scale + c, sc);
  ldc<N>(coef.c1 + c, c1);
  ldc<N>(coef.c0 + c, c0);
  int64_t i = i0;
  for (; i + 3 * st < nv; i += 4 * st) {
    float yy[4][N], d[4][N];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ldv(y + (i + u * st) * N, yy[u]);
      ldv(dz + (i + u * st) * N, d[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int j = 0; j < N; ++j) d[u][j] = fmaf(d[u][j], sc[j], fmaf(c1[j], yy[u][j], c0[j]));
      stv(dz + (i + u * st) * N, d[u]);
    }
  }
  for (; i < nv; i += st) {
    float yy[N], d[N];
    ldv(y + i * N, yy);
    ldv(dz + i * N, d);
#pragma unroll
    for (int j = 0; j < N; ++j) d[j] = fmaf(d[j], sc[j], fmaf(c1[j], yy[j], c0[j]));
    stv(dz + i * N, d);
  }
}

int launch_bn_bwd_apply(float *dz, const float *y, BNCoef coef, int64_t nvox, int Cs,
                        hipStream_t s, int bf) {
  {
    const int N = bf ? 8 : 4;
    if (Cs % N == 0) {
      const int G = Cs / N;
      const int64_t nv = nvox * G;
      int64_t want = (nv + 1023) / 1024;   // ~4 vectors per thread
      int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, 65536));
      if (256 % G) {
        const int per = G / std::__gcd(256, G);
        grid = std::max(per, grid / per * per);
      }
      // algorithmic bytes: dz and y read, dY written
      HCU_TIMED(s, "bn_bwd_apply_vec_kernel", 0.0, 3.0 * nvox * Cs * (bf ? 2 : 4),
                HCU_BF_DISPATCH(bf, bn_bwd_apply_vec_kernel, dim3(grid), dim3(256), 0, s, (T *)dz,
                                (const T *)y, coef, nv, G));
      HCU_CHECK_LAUNCH();
      return 0;
    }
  }
  const int64_t n4 = nvox * (Cs / 4);
  const int C4 = Cs / 4;
  // grid * 256 must be a multiple of C4 (fixed channel quad per thread)
  int grid = grid_for(n4);
  if (256 % C4) {
    const int per = C4 / std::__gcd(256, C4);   // blocks per period
    grid = std::max(per, grid / per * per);
  }
  HCU_TIMED(s, "bn_bwd_apply_kernel", 0.0, 3.0 * nvox * Cs * (bf ? 2 : 4),
            HCU_BF_DISPATCH(bf, bn_bwd_apply_kernel, dim3(grid), dim3(256), 0, s,
                            (T *)dz, (const T *)y, coef, n4, Cs / 4));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// out_conv forward: pred[b][o][v] = sum_c relu(bn(y))[v][c] * w[o][c] + bias[o]
#define MAXCO 4
template <typename T>
__global__ void __launch_bounds__(256)
outconv_fwd_kernel(const T *y, BNCoef coef, const float *w, const float *bias,
                   float *pred, int B, int64_t V, int C, int Cs, int Co) {
  const int64_t n = (int64_t)B * V;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / V);
    const int64_t v = i % V;
    float acc[MAXCO];
    for (int o = 0; o < MAXCO; ++o) acc[o] = 0.f;
    const T *yr = y + (size_t)i * Cs;
    for (int c0 = 0; c0 < Cs; c0 += 4) {
      const float4 yy = ld4(yr + c0);
      const float4 sc = ld4(coef.scale + c0), sh = ld4(coef.shift + c0);
      const float a[4] = {bnrelu(yy.x, sc.x, sh.x), bnrelu(yy.y, sc.y, sh.y),
                          bnrelu(yy.z, sc.z, sh.z), bnrelu(yy.w, sc.w, sh.w)};
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        if (c < C)
          for (int o = 0; o < Co && o < MAXCO; ++o) acc[o] = fmaf(a[j], w[o * C + c], acc[o]);
      }
    }
    for (int o = 0; o < Co && o < MAXCO; ++o)
      pred[((size_t)b * Co + o) * V + v] = acc[o] + (bias ? bias[o] : 0.f);
  }
}

int launch_outconv_fwd(const float *y, BNCoef coef, const float *w, const float *bias,
                       float *pred, int B, int64_t V, int C, int Cs, int Co,
                       hipStream_t s, int bf) {
  if (Co > MAXCO) return fail(4, "out_conv: out_channels > 4 not supported");
  HCU_TIMED(s, "outconv_fwd_kernel", 0.0, 0.0,
            HCU_BF_DISPATCH(bf, outconv_fwd_kernel, dim3(grid_for((int64_t)B * V)), dim3(256), 0,
                            s, (const T *)y, coef, w, bias, pred, B, V, C, Cs, Co));
  HCU_CHECK_LAUNCH();
  return 0;
}

// out_conv backward + last BatchNorm backward reduction.
//   dA[v][c] = sum_o dpred[o][v] w[o][c];  dz = dA [z>0];
//   part_bn[r][c][2] = (sum dz, sum dz*xhat);
//   part_oc[r][o*Cs + c] = sum dpred[o] a[c];  part_oc[r][Co*Cs + o] = sum dpred[o]
template <typename T>
__global__ void __launch_bounds__(256)
outconv_bwd_kernel(const float *dpred, const T *y, BNCoef coef, const float *w,
                   T *dz, int B, int64_t V, int C, int Cs, int Co, float *part_bn,
                   float *part_oc, RedGeom g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int NV = 8 + 5 * MAXCO;
  const int C4 = Cs / 4, tid = threadIdx.x;
  float v[NV];
  for (int k = 0; k < NV; ++k) v[k] = 0.f;
  if (tid < g.tb) {
    const int64_t beg = (int64_t)blockIdx.x * g.chunk;
    const int64_t end = std::min(beg + g.chunk, g.total);
    const int c = (int)((beg + tid) % C4) * 4;
    const float4 sc = ld4(coef.scale + c), sh = ld4(coef.shift + c);
    const float4 mu = ld4(coef.mean + c), is = ld4(coef.invstd + c);
    float wv[MAXCO][4];
    for (int o = 0; o < MAXCO; ++o)
      for (int j = 0; j < 4; ++j) wv[o][j] = (o < Co && c + j < C) ? w[o * C + c + j] : 0.f;
    for (int64_t e = beg + tid; e < end; e += g.tb) {
      const int64_t vox = e / C4;
      const int b = (int)(vox / V);
      const int64_t vv = vox % V;
      const size_t off = (size_t)vox * Cs + c;
      const float4 yy = ld4(y + off);
      float dp[MAXCO];
      for (int o = 0; o < MAXCO; ++o) dp[o] = o < Co ? dpred[((size_t)b * Co + o) * V + vv] : 0.f;
      const float yv[4] = {yy.x, yy.y, yy.z, yy.w};
      const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
      const float muv[4] = {mu.x, mu.y, mu.z, mu.w}, isv[4] = {is.x, is.y, is.z, is.w};
      float dzv[4];
      for (int j = 0; j < 4; ++j) {
        const float z = fmaf(yv[j], scv[j], shv[j]);
        const float a = fmaxf(z, 0.f);
        float dA = 0.f;
        for (int o = 0; o < MAXCO; ++o) {
          dA = fmaf(dp[o], wv[o][j], dA);
          v[8 + o * 4 + j] = fmaf(dp[o], a, v[8 + o * 4 + j]);
        }
        dzv[j] = z > 0.f ? dA : 0.f;
        v[2 * j] += dzv[j];
        v[2 * j + 1] = fmaf(dzv[j], (yv[j] - muv[j]) * isv[j], v[2 * j + 1]);
      }
      if (c == 0)
        for (int o = 0; o < MAXCO; ++o) v[8 + 4 * MAXCO + o] += dp[o];
      st4(dz + off, make_float4(dzv[0], dzv[1], dzv[2], dzv[3]));
    }
  }
  // reduce per c4 group
  if (tid < g.tb)
    for (int k = 0; k < NV; ++k) lds[tid * NV + k] = v[k];
  __syncthreads();
  if (tid < C4) {
    float acc[NV];
    for (int k = 0; k < NV; ++k) acc[k] = 0.f;
    for (int t = tid; t < g.tb; t += C4)
      for (int k = 0; k < NV; ++k) acc[k] += lds[t * NV + k];
    const int c = tid * 4;
    float *pb = part_bn + (size_t)blockIdx.x * Cs * 2;
    for (int k = 0; k < 8; ++k) pb[c * 2 + k] = acc[k];
    float *po = part_oc + (size_t)blockIdx.x * (Co * Cs + Co);
    for (int o = 0; o < Co; ++o)
      for (int j = 0; j < 4; ++j) po[o * Cs + c + j] = acc[8 + o * 4 + j];
    if (tid == 0)
      for (int o = 0; o < Co; ++o) po[Co * Cs + o] = acc[8 + 4 * MAXCO + o];
  }
}

int launch_outconv_bwd(const float *dpred, const float *y, BNCoef coef, const float *w,
                       float *dz, int B, int64_t V, int C, int Cs, int Co, float *part_bn,
                       float *part_oc, int R, hipStream_t s, int bf) {
  if (Co > MAXCO) return fail(4, "out_conv: out_channels > 4 not supported");
  const RedGeom g = red_geom((int64_t)B * V, Cs, R);
  const size_t lds = (size_t)std::max(g.tb, 256) * (8 + 5 * MAXCO) * 4;
  HCU_TIMED(s, "outconv_bwd_kernel", 0.0, 0.0,
            HCU_BF_DISPATCH(bf, outconv_bwd_kernel, dim3(R), dim3(256), lds, s, dpred,
                            (const T *)y, coef, w, (T *)dz, B, V, C, Cs, Co, part_bn, part_oc,
                            g));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
chansum_kernel(const T *x, int Cs, float *part, RedGeom g) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int C4 = Cs / 4, tid = threadIdx.x;
  float v[4] = {0, 0, 0, 0};
  if (tid < g.tb) {
    const int64_t beg = (int64_t)blockIdx.x * g.chunk;
    const int64_t end = std::min(beg + g.chunk, g.total);
    for (int64_t e = beg + tid; e < end; e += g.tb) {
      const float4 t = ld4(x + e * 4);
      v[0] += t.x;
      v[1] += t.y;
      v[2] += t.z;
      v[3] += t.w;
    }
  }
  block_reduce_c4<4>(v, lds, g.tb, C4, part + (size_t)blockIdx.x * Cs);
}

int launch_chansum(const float *x, int64_t nvox, int Cs, float *part, int R, hipStream_t s,
                   int bf) {
  const RedGeom g = red_geom(nvox, Cs, R);
  HCU_TIMED(s, "chansum_kernel", 0.0, 0.0,
            HCU_BF_DISPATCH(bf, chansum_kernel, dim3(R), dim3(256),
                            (size_t)std::max(g.tb, 256) * 4 * 4, s, (const T *)x, Cs, part, g));
  HCU_CHECK_LAUNCH();
  return 0;
}

// Fixed-order fp64 sum of one column of the partial rows: one workgroup per
// output element j, 256 threads stride over the R rows, then an LDS tree.
__device__ __forceinline__ double block_sum_column(const float *part, int R, int W, int j) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int r = tid; r < R; r += 256) s += (double)part[(size_t)r * W + j];
  red[tid] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  return red[0];
}

__global__ void __launch_bounds__(256)
reduce_partials_kernel(const float *part, int R, int W, float *out, int accumulate) {
  const int j = blockIdx.x;
  const double s = block_sum_column(part, R, W, j);
  if (threadIdx.x == 0) out[j] = accumulate ? out[j] + (float)s : (float)s;
}

int launch_reduce_partials(const float *part, int R, int W, int n, float *out,
                           int accumulate, hipStream_t s) {
  HCU_TIMED(s, "reduce_partials_kernel", 0.0, 0.0, HCU_LAUNCH(reduce_partials_kernel, dim3(n), dim3(256), 0, s, part, R,
                     W, out, accumulate));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
template <typename TI, typename T>
__global__ void __launch_bounds__(256)
to_cl_kernel(const TI *x, T *xcl, int B, int C, int Cs, int64_t V, FastDiv fV, FastDiv fC4) {
  const uint32_t n = (uint32_t)(B * (Cs / 4) * V);   // < 2^31 (launcher)
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int q, v, b, c4;
    fV.divmod(i, q, v);
    fC4.divmod((uint32_t)q, b, c4);
    float r[4];
    for (int j = 0; j < 4; ++j) {
      const int c = c4 * 4 + j;
      r[j] = c < C ? ld1(x + ((size_t)b * C + c) * V + v) : 0.f;
    }
    st4(xcl + ((size_t)b * V + v) * Cs + c4 * 4, make_float4(r[0], r[1], r[2], r[3]));
  }
}

// One voxel per thread for the network input (C <= 8, Cs = 4 fp32 / 8 bf16):
// C coalesced plane loads, one 16-byte channels-last store.
template <typename TI, typename T>
__global__ void __launch_bounds__(256)
to_cl_vox_kernel(const TI *x, T *xcl, int C, int64_t V, uint32_t n, FastDiv fV) {
  constexpr int N = VN<T>::N;
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int b, v;
  fV.divmod(i, b, v);
  float r[N];
#pragma unroll
  for (int c = 0; c < N; ++c) r[c] = c < C ? ld1(x + ((size_t)b * C + c) * V + v) : 0.f;
  stv(xcl + (size_t)i * N, r);
}

// x_dtype: HCU_F32 / HCU_F16 / 3 = bf16 input volume; bf: bf16 channels-last output.
int launch_to_cl(const float *x, float *xcl, int B, int C, int Cs, int64_t V, hipStream_t s,
                 int bf, int x_dtype) {
  const int64_t n = (int64_t)B * (Cs / 4) * V;
  if (n >= (int64_t)1 << 31) return fail(4, "input volume: more than 2^31 channel quads");
  const dim3 gr(grid_for(n));
  const FastDiv fV((uint32_t)V), fC4((uint32_t)(Cs / 4));
  if (Cs == (bf ? 8 : 4) && C <= Cs && (int64_t)B * V < ((int64_t)1 << 31)) {
    const uint32_t nv = (uint32_t)(B * V);
    const dim3 g2((nv + 255) / 256);
    if (x_dtype == 1 && bf)
      HCU_TIMED(s, "to_cl_vox_kernel", 0.0, 0.0,
                HCU_LAUNCH((to_cl_vox_kernel<_Float16, bf16_t>), g2, dim3(256), 0, s,
                                   (const _Float16 *)x, (bf16_t *)xcl, C, V, nv, fV));
    else if (x_dtype == 3 && bf)
      HCU_TIMED(s, "to_cl_vox_kernel", 0.0, 0.0,
                HCU_LAUNCH((to_cl_vox_kernel<bf16_t, bf16_t>), g2, dim3(256), 0, s,
                                   (const bf16_t *)x, (bf16_t *)xcl, C, V, nv, fV));
    else if (x_dtype == 0 && bf)
      HCU_TIMED(s, "to_cl_vox_kernel", 0.0, 0.0,
                HCU_LAUNCH((to_cl_vox_kernel<float, bf16_t>), g2, dim3(256), 0, s, x,
                                   (bf16_t *)xcl, C, V, nv, fV));
    else if (x_dtype == 1)
      HCU_TIMED(s, "to_cl_vox_kernel", 0.0, 0.0,
                HCU_LAUNCH((to_cl_vox_kernel<_Float16, float>), g2, dim3(256), 0, s,
                                   (const _Float16 *)x, xcl, C, V, nv, fV));
    else if (x_dtype == 0)
      HCU_TIMED(s, "to_cl_vox_kernel", 0.0, 0.0,
                HCU_LAUNCH((to_cl_vox_kernel<float, float>), g2, dim3(256), 0, s, x, xcl, C, V,
                                   nv, fV));
    else
      return fail(4, "to_cl: unsupported input dtype");
    HCU_CHECK_LAUNCH();
    return 0;
  }
  if (launch_to_cl_tiled(x, xcl, B, C, Cs, V, s, bf, x_dtype) == 0) return 0;
  if (x_dtype == 1 && bf)
    HCU_TIMED(s, "to_cl_kernel", 0.0, 0.0,
              HCU_LAUNCH((to_cl_kernel<_Float16, bf16_t>), gr, dim3(256), 0, s,
                                 (const _Float16 *)x, (bf16_t *)xcl, B, C, Cs, V, fV, fC4));
  else if (x_dtype == 3 && bf)
    HCU_TIMED(s, "to_cl_kernel", 0.0, 0.0,
              HCU_LAUNCH((to_cl_kernel<bf16_t, bf16_t>), gr, dim3(256), 0, s,
                                 (const bf16_t *)x, (bf16_t *)xcl, B, C, Cs, V, fV, fC4));
  else if (x_dtype == 0 && bf)
    HCU_TIMED(s, "to_cl_kernel", 0.0, 0.0,
              HCU_LAUNCH((to_cl_kernel<float, bf16_t>), gr, dim3(256), 0, s, x,
                                 (bf16_t *)xcl, B, C, Cs, V, fV, fC4));
  else if (x_dtype == 1)
    HCU_TIMED(s, "to_cl_kernel", 0.0, 0.0,
              HCU_LAUNCH((to_cl_kernel<_Float16, float>), gr, dim3(256), 0, s,
                                 (const _Float16 *)x, xcl, B, C, Cs, V, fV, fC4));
  else if (x_dtype == 0)
    HCU_TIMED(s, "to_cl_kernel", 0.0, 0.0,
              HCU_LAUNCH((to_cl_kernel<float, float>), gr, dim3(256), 0, s, x, xcl, B, C,
                                 Cs, V, fV, fC4));
  else
    return fail(4, "to_cl: unsupported input dtype");
  HCU_CHECK_LAUNCH();
  return 0;
}

template <typename T>
__global__ void __launch_bounds__(256)
from_cl_kernel(const T *xcl, float *x, int B, int C, int Cs, int64_t V) {
  const int64_t n = (int64_t)B * C * V;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t v = i % V;
    const int64_t q = i / V;
    const int c = (int)(q % C);
    const int b = (int)(q / C);
    x[i] = ld1(xcl + ((size_t)b * V + v) * Cs + c);
  }
}

int launch_from_cl(const float *xcl, float *x, int B, int C, int Cs, int64_t V, hipStream_t s,
                   int bf) {
  if (launch_from_cl_tiled(xcl, nullptr, nullptr, x, B, C, Cs, V, s, bf) == 0) return 0;
  const int64_t n = (int64_t)B * C * V;
  HCU_TIMED(s, "from_cl_kernel", 0.0, 0.0,
            HCU_BF_DISPATCH(bf, from_cl_kernel, dim3(grid_for(n)), dim3(256), 0, s,
                            (const T *)xcl, x, B, C, Cs, V));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Effective (folded, block-diagonal) Conv3d weight element W_eff[o][e][t].
__device__ inline float weff(const float *w, int o, int e, int t, int Cout, int Cin_g,
                             int groups, int fold_mod, int T) {
  const int g = o / (Cout / groups);
  const int cin_total = groups * Cin_g;
  float s = 0.f;
  for (int cp = e; cp < cin_total; cp += fold_mod) {
    const int c = cp - g * Cin_g;
    if (c >= 0 && c < Cin_g) s += w[((size_t)o * Cin_g + c) * T + t];
  }
  return s;
}

__device__ __forceinline__ int64_t prep_count(const WPack &pk, int T, int ICs, int CoutW) {
  return wpack_count(pk, T, ICs, CoutW);
}
// (t, ci, co) of element i of the prepared buffer (plain or packed layout).
__device__ __forceinline__ bool prep_index(const WPack &pk, int64_t i, int T, int ICs, int CoutW,
                                           int &t, int &ci, int &co) {
  if (pk.on) return wpack_decode(pk, i, T, t, ci, co);
  co = (int)(i % CoutW);
  const int64_t q = i / CoutW;
  ci = (int)(q % ICs);
  t = (int)(q / ICs);
  return true;
}

__global__ void __launch_bounds__(256)
prep_conv_fwd_kernel(const float *w, float *wg, int Cout, int Cin_g, int groups,
                     int fold_mod, int T, int ECs, int CoutW, int E, WPack pk) {
  const int64_t n = prep_count(pk, T, ECs, CoutW);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    int t, e, co;
    float v = 0.f;
    if (prep_index(pk, i, T, ECs, CoutW, t, e, co) && co < Cout && e < E)
      v = weff(w, co, e, t, Cout, Cin_g, groups, fold_mod, T);
    wg[i] = v;
  }
}

int launch_prep_conv_fwd(const float *w, float *wg, int Cout, int Cin_g, int groups,
                         int fold_mod, int T, int ECs, int CoutW, WPack pk, hipStream_t s) {
  const int E = std::min(fold_mod, groups * Cin_g);
  const int64_t n = wpack_count(pk, T, ECs, CoutW);
  HCU_TIMED(s, "prep_conv_fwd_kernel", 0.0, 0.0, HCU_LAUNCH(prep_conv_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, w, wg, Cout,
                     Cin_g, groups, fold_mod, T, ECs, CoutW, E, pk));
  HCU_CHECK_LAUNCH();
  return 0;
}

// dgrad GEMM: rows (ci of the GEMM) = conv output channels co, cols = input channels e.
__global__ void __launch_bounds__(256)
prep_conv_dgrad_kernel(const float *w, float *wg, int Cout, int Cin_g, int groups,
                       int fold_mod, int T, int OCs, int EW, int E, WPack pk) {
  const int64_t n = prep_count(pk, T, OCs, EW);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    int tp, co, e;
    float v = 0.f;
    if (prep_index(pk, i, T, OCs, EW, tp, co, e) && co < Cout && e < E)
      v = weff(w, co, e, T - 1 - tp, Cout, Cin_g, groups, fold_mod, T);
    wg[i] = v;
  }
}

int launch_prep_conv_dgrad(const float *w, float *wg, int Cout, int Cin_g, int groups,
                           int fold_mod, int T, int OCs, int EW, int E, WPack pk, hipStream_t s) {
  const int64_t n = wpack_count(pk, T, OCs, EW);
  HCU_TIMED(s, "prep_conv_dgrad_kernel", 0.0, 0.0, HCU_LAUNCH(prep_conv_dgrad_kernel, dim3(grid_for(n)), dim3(256), 0, s, w, wg, Cout,
                     Cin_g, groups, fold_mod, T, OCs, EW, E, pk));
  HCU_CHECK_LAUNCH();
  return 0;
}

__global__ void __launch_bounds__(256)
prep_convt_fwd_kernel(const float *w, float *wg, int Cin, int Cout, int KX, int KY, int KZ,
                      int sx, int sy, int sz, int px, int py, int pz, int Jx, int Jy,
                      int Jz, int ICs, int CoutW) {
  const int Tp = Jx * Jy * Jz;
  const int64_t n = (int64_t)Tp * ICs * CoutW;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int co = (int)(i % CoutW);
    const int64_t q = i / CoutW;
    const int ci = (int)(q % ICs);
    const int t = (int)(q / ICs);
    const int tz = t % Jz, ty = (t / Jz) % Jy, tx = t / (Jz * Jy);
    const int kx = px + sx * (Jx - 1 - tx), ky = py + sy * (Jy - 1 - ty),
              kz = pz + sz * (Jz - 1 - tz);
    float v = 0.f;
    if (ci < Cin && co < Cout && kx < KX && ky < KY && kz < KZ)
      v = w[((((size_t)ci * Cout + co) * KX + kx) * KY + ky) * KZ + kz];
    wg[i] = v;
  }
}

int launch_prep_convt_fwd(const float *w, float *wg, int Cin, int Cout, int KX, int KY,
                          int KZ, int sx, int sy, int sz, int px, int py, int pz, int Jx,
                          int Jy, int Jz, int ICs, int CoutW, hipStream_t s) {
  const int64_t n = (int64_t)Jx * Jy * Jz * ICs * CoutW;
  HCU_TIMED(s, "prep_convt_fwd_kernel", 0.0, 0.0, HCU_LAUNCH(prep_convt_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, w, wg, Cin,
                     Cout, KX, KY, KZ, sx, sy, sz, px, py, pz, Jx, Jy, Jz, ICs, CoutW));
  HCU_CHECK_LAUNCH();
  return 0;
}

__global__ void __launch_bounds__(256)
prep_convt_fused_kernel(const float *w, float *wg, int Cin, int Cout, int KX, int KY, int KZ,
                        int sx, int sy, int sz, int ICs, int CoutW, WPack pk) {
  const int Jx = KX / sx, Jy = KY / sy, Jz = KZ / sz;
  const int T = Jx * Jy * Jz;
  const int nph = sx * sy * sz;
  const int64_t n = prep_count(pk, T, ICs, CoutW);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    int t, ci, nn;
    float v = 0.f;
    if (prep_index(pk, i, T, ICs, CoutW, t, ci, nn) && ci < Cin && nn < nph * Cout) {
      const int ph = nn / Cout, co = nn % Cout;
      const int qz = ph % sz, qy = (ph / sz) % sy, qx = ph / (sz * sy);
      const int tz = t % Jz, ty = (t / Jz) % Jy, tx = t / (Jz * Jy);
      const int kx = qx + sx * (Jx - 1 - tx), ky = qy + sy * (Jy - 1 - ty),
                kz = qz + sz * (Jz - 1 - tz);
      v = w[((((size_t)ci * Cout + co) * KX + kx) * KY + ky) * KZ + kz];
    }
    wg[i] = v;
  }
}

int launch_prep_convt_fused(const float *w, float *wg, int Cin, int Cout, int KX, int KY,
                            int KZ, int sx, int sy, int sz, int ICs, int CoutW, WPack pk,
                            hipStream_t s) {
  const int T = (KX / sx) * (KY / sy) * (KZ / sz);
  const int64_t n = wpack_count(pk, T, ICs, CoutW);
  HCU_TIMED(s, "prep_convt_fused_kernel", 0.0, 0.0,
            HCU_LAUNCH(prep_convt_fused_kernel, dim3(grid_for(n)), dim3(256), 0, s, w, wg,
                               Cin, Cout, KX, KY, KZ, sx, sy, sz, ICs, CoutW, pk));
  HCU_CHECK_LAUNCH();
  return 0;
}

__global__ void __launch_bounds__(256)
prep_convt_dgrad_kernel(const float *w, float *wg, int Cin, int Cout, int T, int UCs,
                        int CinW, WPack pk) {
  const int64_t n = prep_count(pk, T, UCs, CinW);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    int t, co, ci;
    float v = 0.f;
    if (prep_index(pk, i, T, UCs, CinW, t, co, ci) && ci < Cin && co < Cout)
      v = w[((size_t)ci * Cout + co) * T + t];
    wg[i] = v;
  }
}

int launch_prep_convt_dgrad(const float *w, float *wg, int Cin, int Cout, int T, int UCs,
                            int CinW, WPack pk, hipStream_t s) {
  const int64_t n = wpack_count(pk, T, UCs, CinW);
  HCU_TIMED(s, "prep_convt_dgrad_kernel", 0.0, 0.0, HCU_LAUNCH(prep_convt_dgrad_kernel, dim3(grid_for(n)), dim3(256), 0, s, w, wg, Cin,
                     Cout, T, UCs, CinW, pk));
  HCU_CHECK_LAUNCH();
  return 0;
}

// out_conv weight/bias gradient from the fused backward's partial rows
// (one workgroup per dw/db element).
__global__ void __launch_bounds__(256)
outconv_wfinalize_kernel(const float *part, int R, int Co, int C, int Cs, float *dw, float *db,
                         int accumulate) {
  const int j = blockIdx.x;
  const int W = Co * Cs + Co;
  int src;
  float *dst;
  if (j < Co * C) {
    const int o = j / C, c = j % C;
    src = o * Cs + c;
    dst = dw + j;
  } else {
    src = Co * Cs + (j - Co * C);
    dst = db + (j - Co * C);
  }
  const double s = block_sum_column(part, R, W, src);
  if (threadIdx.x == 0) *dst = accumulate ? *dst + (float)s : (float)s;
}

int launch_outconv_wfinalize(const float *part_oc, int R, int Co, int C, int Cs, float *dw,
                             float *db, int accumulate, hipStream_t s) {
  const int n = Co * C + Co;
  HCU_TIMED(s, "outconv_wfinalize_kernel", 0.0, 0.0, HCU_LAUNCH(outconv_wfinalize_kernel, dim3(n), dim3(256), 0, s, part_oc,
                     R, Co, C, Cs, dw, db, accumulate));
  HCU_CHECK_LAUNCH();
  return 0;
}

// num_batches_tracked += 1 for every BatchNorm3d of the net (train forward).
struct CountPtrs {
  int64_t *p[64];
  int n;
};
__global__ void bn_count_kernel(CountPtrs c) {
  const int i = threadIdx.x;
  if (i < c.n && c.p[i]) c.p[i][0] += 1;
}

int launch_bn_count_increment(int64_t *const *ptrs, int n, hipStream_t s) {
  if (n > 64) return fail(4, "too many BatchNorm layers");
  CountPtrs c{};
  for (int i = 0; i < n; ++i) c.p[i] = ptrs[i];
  c.n = n;
  HCU_TIMED(s, "bn_count_kernel", 0.0, 0.0, HCU_LAUNCH(bn_count_kernel, dim3(1), dim3(64), 0, s, c));
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu
