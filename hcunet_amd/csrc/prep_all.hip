// All weight re-layouts of one network step in a few launches (one workgroup
// row per job) instead of one launch per layer: the executor prepares every
// conv / convT weight once at the start of forward into the `saved`
// workspace, and forward and backward read the prepared images from there.
// Element i of a job is exactly what the per-layer prep_* kernel in
// pointwise.hip writes for that layer (same index decoding, same values).
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <cstdlib>

namespace hcu {

struct PrepBatch {
  int n;
  PrepJob j[kPrepBatch];
};
static_assert(sizeof(PrepBatch) <= 4000, "prep batch must fit the 4 KB kernel-argument limit");

__device__ __forceinline__ bool prep_index2(const WPack &pk, uint32_t i, int T, int ICs, int CoutW,
                                            int &t, int &ci, int &co) {
  if (pk.on) return wpack_decode(pk, i, T, t, ci, co);
  co = (int)(i % (uint32_t)CoutW);
  const uint32_t q = i / (uint32_t)CoutW;
  ci = (int)(q % (uint32_t)ICs);
  t = (int)(q / (uint32_t)ICs);
  return true;
}

// Effective (folded, block-diagonal) Conv3d weight element W_eff[o][e][t].
// part_cs > 0: the input is made of channel parts (ConvLayer::part_c): packed
// channel e is torch channel (e / part_cs) * part_c + e % part_cs, or padding.
__device__ __forceinline__ float weff2(const float *w, int o, int e, int t, int Cout, int Cin_g,
                                       int groups, int fold_mod, int T, int part_c = 0, int part_cs = 0) {
  if (part_cs) {
    const int r = e % part_cs;
    if (r >= part_c) return 0.f;
    e = (e / part_cs) * part_c + r;
  }
  const int g = o / (Cout / groups);
  const int cin_total = groups * Cin_g;
  float s = 0.f;
  for (int cp = e; cp < cin_total; cp += fold_mod) {
    const int c = cp - g * Cin_g;
    if (c >= 0 && c < Cin_g) s += w[((size_t)o * Cin_g + c) * T + t];
  }
  return s;
}

// Index decoding of the packed jobs: image element i -> (t, a, b), where `a`
// (the middle index) advances by one across the V = 8 (bf16) / 4 (fp32)
// consecutive elements of one packed vector (wpack_decode's j).
__device__ __forceinline__ bool prep_decode(const PrepJob &jb, uint32_t i, int &t, int &a, int &b) {
  const int *p = jb.p;
  switch (jb.kind) {
    case PREP_CONV_FWD:
    case PREP_CONV_DGRAD:
      return prep_index2(jb.pk, i, p[4], p[5], p[6], t, a, b);
    case PREP_CONVT_FUSED: {
      const int T = (p[2] / p[5]) * (p[3] / p[6]) * (p[4] / p[7]);
      return prep_index2(jb.pk, i, T, p[8], p[9], t, a, b);
    }
    default:   // PREP_CONVT_DGRAD
      return prep_index2(jb.pk, i, p[2], p[3], p[4], t, a, b);
  }
}

// Value of a decoded (t, a, b) element (0 for padding).
__device__ __forceinline__ float prep_eval(const PrepJob &jb, const float *w, int t, int a, int b) {
  const int *p = jb.p;
  switch (jb.kind) {
    case PREP_CONV_FWD:   // (t, e, co)
      return (b < p[0] && a < p[7]) ? weff2(w, b, a, t, p[0], p[1], p[2], p[3], p[4], p[8], p[9]) : 0.f;
    case PREP_CONV_DGRAD:   // (t', co, e)
      return (a < p[0] && b < p[7]) ? weff2(w, a, b, p[4] - 1 - t, p[0], p[1], p[2], p[3], p[4], p[8], p[9])
                                    : 0.f;
    case PREP_CONVT_FUSED: {   // (t, ci, nn)
      const int Cin = p[0], Cout = p[1], KX = p[2], KY = p[3], KZ = p[4];
      const int sx = p[5], sy = p[6], sz = p[7];
      const int Jx = KX / sx, Jy = KY / sy, Jz = KZ / sz;
      const int cph = p[10] > 0 ? p[10] : Cout;   // columns per phase (GConvArgs::cph)
      if (a >= Cin || b >= sx * sy * sz * cph) return 0.f;
      const int ph = b / cph, co = b % cph;
      if (co >= Cout) return 0.f;
      const int qz = ph % sz, qy = (ph / sz) % sy, qx = ph / (sz * sy);
      const int tz = t % Jz, ty = (t / Jz) % Jy, tx = t / (Jz * Jy);
      const int kx = qx + sx * (Jx - 1 - tx), ky = qy + sy * (Jy - 1 - ty), kz = qz + sz * (Jz - 1 - tz);
      return w[((((size_t)a * Cout + co) * KX + kx) * KY + ky) * KZ + kz];
    }
    default:   // PREP_CONVT_DGRAD: (t, co, ci)
      return (b < p[0] && a < p[1]) ? w[((size_t)b * p[1] + a) * p[2] + t] : 0.f;
  }
}

__device__ float prep_value(const PrepJob &jb, const float *w, uint32_t i) {
  if (jb.kind == PREP_CONVT_PHASE) {
    const int *p = jb.p;
    const int Cin = p[0], Cout = p[1], KX = p[2], KY = p[3], KZ = p[4];
    const int Jx = p[11], Jy = p[12], Jz = p[13], ICs = p[14], CoutW = p[15];
    const int co = (int)(i % (uint32_t)CoutW);
    const uint32_t q = i / (uint32_t)CoutW;
    const int ci = (int)(q % (uint32_t)ICs);
    const int t = (int)(q / (uint32_t)ICs);
    const int tz = t % Jz, ty = (t / Jz) % Jy, tx = t / (Jz * Jy);
    const int kx = p[8] + p[5] * (Jx - 1 - tx), ky = p[9] + p[6] * (Jy - 1 - ty),
              kz = p[10] + p[7] * (Jz - 1 - tz);
    if (ci < Cin && co < Cout && kx < KX && ky < KY && kz < KZ)
      return w[((((size_t)ci * Cout + co) * KX + kx) * KY + ky) * KZ + kz];
    return 0.f;
  }
  int t, a, b;
  return prep_decode(jb, i, t, a, b) ? prep_eval(jb, w, t, a, b) : 0.f;
}

// Packed images are [chunk][s][g][column][V]: consecutive vectors k walk the
// output column, whose source weights lie Cin_g*T floats apart, so a wave's
// gather touched 64 lines per element and a large layer's weights were
// re-fetched once per tap (3.6x the parameter bytes).  The vector a thread
// handles is taken column-major instead (perm): the lanes of a wave share the
// column and walk (g, s), i.e. the tap, whose source weights are adjacent.
// Same values, same image; the 16-byte stores scatter instead.
__device__ __forceinline__ uint32_t prep_perm(uint32_t u, uint32_t nv, uint32_t cw, bool on) {
  if (!on) return u;
  const uint32_t r = nv / cw;
  return (u % r) * cw + u / r;
}

__global__ void __launch_bounds__(256)
prep_all_kernel(const float *params, float *dst_base, const PrepBatch b, int perm) {
  const PrepJob &jb = b.j[blockIdx.y];
  const float *w = params + jb.src;
  float *dst = dst_base + jb.dst;
  const uint32_t n = (uint32_t)jb.n;   // < 2^31 (launch_prep_all)
  // packed images: one decode per 16-byte vector (8 bf16 / 4 fp32 elements
  // whose middle index advances by one), one 16-byte store
  if (jb.pk.on && jb.kind != PREP_CONVT_PHASE && ((uintptr_t)dst & 15) == 0) {
    const uint32_t cw = (uint32_t)(jb.pk.CoutW > 0 ? jb.pk.CoutW : 1);
    if (jb.bf16 && jb.pk.on == 3 && n % 8 == 0) {
      uint4 *d = reinterpret_cast<uint4 *>(dst);
      const bool pm = perm && (n / 8) % cw == 0;
      for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < n / 8; u += gridDim.x * 256) {
        const uint32_t k = prep_perm(u, n / 8, cw, pm);
        int t, a, b;
        const bool ok = prep_decode(jb, k * 8, t, a, b);
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ok ? prep_eval(jb, w, t, a + j, b) : 0.f;
        d[k] = make_uint4((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                          (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16),
                          (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16),
                          (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16));
      }
      return;
    }
    if (!jb.bf16 && jb.pk.on != 3 && n % 4 == 0) {
      float4 *d = reinterpret_cast<float4 *>(dst);
      const bool pm = perm && jb.pk.on == 1 && (n / 4) % cw == 0;
      for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < n / 4; u += gridDim.x * 256) {
        const uint32_t k = prep_perm(u, n / 4, cw, pm);
        int t, a, b;
        const bool ok = prep_decode(jb, k * 4, t, a, b);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = ok ? prep_eval(jb, w, t, a + j, b) : 0.f;
        d[k] = make_float4(v[0], v[1], v[2], v[3]);
      }
      return;
    }
  }
  if (jb.bf16) {
    uint16_t *d16 = reinterpret_cast<uint16_t *>(dst);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
      d16[i] = f2bf(prep_value(jb, w, i));
    return;
  }
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    dst[i] = prep_value(jb, w, i);
}

int launch_prep_all(const float *params, float *dst_base, const PrepJob *jobs, int n,
                    hipStream_t s) {
  const int perm = 1;   // the tap-fastest vector order (prep_perm; round 3: config 3 -8..-18 us)
  for (int j0 = 0; j0 < n; j0 += kPrepBatch) {
    PrepBatch b{};
    b.n = std::min(kPrepBatch, n - j0);
    int64_t most = 1;
    for (int k = 0; k < b.n; ++k) {
      b.j[k] = jobs[j0 + k];
      if (b.j[k].n >= (int64_t)1 << 31) return fail(4, "prep_all: weight image too large");
      most = std::max(most, b.j[k].n);
    }
    // enough workgroups that the largest gathered job is ~8 elements per thread
    const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((most + 2047) / 2048, 1024));
    HCU_TIMED(s, "prep_all_kernel", 0.0, 0.0,
              HCU_LAUNCH(prep_all_kernel, dim3(gx, b.n), dim3(256), 0, s, params, dst_base, b, perm));
    HCU_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace hcu
