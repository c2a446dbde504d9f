// Generic gather convolution on fp32 MFMA (v_mfma_f32_16x16x4_f32).
//
// One workgroup (4 waves) computes an output tile of TX*TY*TZ voxels x NT
// output channels.  The K dimension (taps x input channels) is walked in
// chunks of CK input channels: the input halo of the tile for those CK
// channels is staged once in LDS (BatchNorm+ReLU of the producer applied on
// the way in), the weights [T][CK][NT] next to it, and every tap then reads
// its A operand straight out of the halo (no im2col in memory).
//
// LDS image: alds[ci][voxel] (plane stride P == 16 mod 32, so the two k-lane
// groups of a ds_read_b32 hit disjoint bank halves); wlds[t][ci][NTP]
// (NTP == 16 mod 32 for the same reason).
//
// Replaces the arithmetic of nn.Conv3d / nn.ConvTranspose3d forward and their
// input gradients on the reference path (hcat/unet.py:246-257, 281-298).
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <cmath>

namespace hcu {

template <int CK, int NSUB, int MPW>
__global__ void __launch_bounds__(256) gconv_kernel(const GConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT = NSUB * 16;
  constexpr int NTP = (NSUB & 1) ? NT : NT + 16;
  constexpr int C4 = CK / 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.KX * a.KY * a.KZ;
  const int P = a.P;
  float *alds = smem;
  float *wlds = smem + CK * P;

  int tile = blockIdx.x;
  const int tzi = tile % a.ntz;
  tile /= a.ntz;
  const int tyi = tile % a.nty;
  const int txi = tile / a.nty;
  const int n0 = blockIdx.y * NT;
  const int b = blockIdx.z;
  const int ox0 = txi * a.TX, oy0 = tyi * a.TY, oz0 = tzi * a.TZ;
  const int MT = a.TX * a.TY * a.TZ;
  const int nmsub = (MT + 15) >> 4;
  const int HZ = a.HZ, HYZ = a.HY * a.HZ;
  const int HV = a.HX * HYZ;

  int vb[MPW];
#pragma unroll
  for (int j = 0; j < MPW; ++j) {
    const int i = (wave + 4 * j) * 16 + (lane & 15);
    int v = 0;
    if (i < MT) {
      int r, lz, lx, ly;
      a.fTZ.divmod(i, r, lz);
      a.fTY.divmod(r, lx, ly);
      v = lx * a.sx * HYZ + ly * a.sy * HZ + lz * a.sz;
    }
    vb[j] = v;
  }

  floatx4 acc[MPW][NSUB];
#pragma unroll
  for (int j = 0; j < MPW; ++j)
#pragma unroll
    for (int n = 0; n < NSUB; ++n) acc[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int gx0 = ox0 * a.sx - a.px, gy0 = oy0 * a.sy - a.py, gz0 = oz0 * a.sz - a.pz;
  const int kci = lane >> 4;
  const size_t in_b = (size_t)b * a.IX;

  for (int ci0 = 0; ci0 < a.ICs; ci0 += CK) {
    __syncthreads();
    // ---- stage the input halo for channels [ci0, ci0+CK)
    for (int idx = tid; idx < HV * C4; idx += 256) {
      const int c4 = idx % C4;
      const int v = idx / C4;
      int t2, hz, hx, hy;
      a.fHZ.divmod(v, t2, hz);
      a.fHY.divmod(t2, hx, hy);
      const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
      float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((unsigned)gx < (unsigned)a.IX && (unsigned)gy < (unsigned)a.IY &&
          (unsigned)gz < (unsigned)a.IZ) {
        const int c = ci0 + c4 * 4;
        val = *reinterpret_cast<const float4 *>(
            a.in + (((in_b + gx) * a.IY + gy) * a.IZ + gz) * a.ICs + c);
        if (a.in_scale) {
          const float4 sc = *reinterpret_cast<const float4 *>(a.in_scale + c);
          const float4 sh = *reinterpret_cast<const float4 *>(a.in_shift + c);
          val.x = fmaxf(fmaf(val.x, sc.x, sh.x), 0.f);
          val.y = fmaxf(fmaf(val.y, sc.y, sh.y), 0.f);
          val.z = fmaxf(fmaf(val.z, sc.z, sh.z), 0.f);
          val.w = fmaxf(fmaf(val.w, sc.w, sh.w), 0.f);
        }
      }
      float *dst = alds + (c4 * 4) * P + v;
      dst[0] = val.x;
      dst[P] = val.y;
      dst[2 * P] = val.z;
      dst[3 * P] = val.w;
    }
    // ---- stage the weights [T][CK][NT]
    constexpr int N4 = NT / 4;
    for (int idx = tid; idx < T * CK * N4; idx += 256) {
      const int n4 = idx % N4;
      const int r = idx / N4;  // t*CK + ci
      const int ci = r % CK;
      const int t = r / CK;
      const float4 w4 = *reinterpret_cast<const float4 *>(
          a.w + (size_t)(t * a.ICs + ci0 + ci) * a.CoutW + n0 + n4 * 4);
      *reinterpret_cast<float4 *>(wlds + r * NTP + n4 * 4) = w4;
    }
    __syncthreads();

    // ---- MFMA over taps x channels of this chunk
    int t = 0;
    for (int kx = 0; kx < a.KX; ++kx)
    for (int ky = 0; ky < a.KY; ++ky)
    for (int kz = 0; kz < a.KZ; ++kz, ++t) {
      const int toff = kx * a.dx * HYZ + ky * a.dy * HZ + kz * a.dz;
#pragma unroll
      for (int k4 = 0; k4 < C4; ++k4) {
        const int ci = k4 * 4 + kci;
        float bv[NSUB];
#pragma unroll
        for (int n = 0; n < NSUB; ++n)
          bv[n] = wlds[(t * CK + ci) * NTP + n * 16 + (lane & 15)];
        const float *ap = alds + ci * P + toff;
#pragma unroll
        for (int j = 0; j < MPW; ++j) {
          if (wave + 4 * j < nmsub) {
            const float av = ap[vb[j]];
#pragma unroll
            for (int n = 0; n < NSUB; ++n)
              acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[n], acc[j][n], 0, 0, 0);
          }
        }
      }
    }
  }

  // ---- epilogue: bias, store, BatchNorm partial statistics (about a pivot per
  // channel: the tile's first output voxel; StatRow in common.h)
  float s1[NSUB], s2[NSUB], pv[NSUB], cnt = 0.f;
#pragma unroll
  for (int n = 0; n < NSUB; ++n) s1[n] = s2[n] = pv[n] = 0.f;
  float bias_v[NSUB];
#pragma unroll
  for (int n = 0; n < NSUB; ++n) {
    const int co = n0 + n * 16 + (lane & 15);
    bias_v[n] = (a.bias && co < a.Cout) ? a.bias[co] : 0.f;
  }
  float *pivl = smem + 4 * NT * 3;   // [NT], past the reduction area
  if (a.stats) {
    __syncthreads();   // every wave is done with the staged operands
    if (wave == 0 && lane < 16) {
#pragma unroll
      for (int n = 0; n < NSUB; ++n) pivl[n * 16 + lane] = acc[0][n][0] + bias_v[n];
    }
    __syncthreads();
#pragma unroll
    for (int n = 0; n < NSUB; ++n) pv[n] = pivl[n * 16 + (lane & 15)];
  }
#pragma unroll
  for (int j = 0; j < MPW; ++j) {
    const int m = wave + 4 * j;
    if (m < nmsub) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = m * 16 + (lane >> 4) * 4 + r;
        if (i < MT) {
          int q, lz, lx, ly;
          a.fTZ.divmod(i, q, lz);
          a.fTY.divmod(q, lx, ly);
          const int ox = ox0 + lx, oy = oy0 + ly, oz = oz0 + lz;
          if (ox < a.OX && oy < a.OY && oz < a.OZ) {
            const size_t ob =
                ((((size_t)b * a.SX + ox * a.osx + a.ofx) * a.SY + oy * a.osy + a.ofy) * a.SZ +
                 oz * a.osz + a.ofz) * a.OCs;
#pragma unroll
            for (int n = 0; n < NSUB; ++n) {
              const int co = n0 + n * 16 + (lane & 15);
              const float val = acc[j][n][r] + bias_v[n];
              if (co < a.OCs) a.out[ob + co] = val;
              if (co < a.Cout) {
                const float d = val - pv[n];
                s1[n] += d;
                s2[n] = fmaf(d, d, s2[n]);
              }
            }
            cnt += 1.f;
          }
        }
      }
    }
  }
  if (a.stats) {
#pragma unroll
    for (int n = 0; n < NSUB; ++n) {
      s1[n] += __shfl_xor(s1[n], 16);
      s1[n] += __shfl_xor(s1[n], 32);
      s2[n] += __shfl_xor(s2[n], 16);
      s2[n] += __shfl_xor(s2[n], 32);
    }
    cnt += __shfl_xor(cnt, 16);
    cnt += __shfl_xor(cnt, 32);
    __syncthreads();
    float *red = smem;  // [4][NT][3]
    if (lane < 16) {
#pragma unroll
      for (int n = 0; n < NSUB; ++n) {
        red[(wave * NT + n * 16 + lane) * 3 + 0] = s1[n];
        red[(wave * NT + n * 16 + lane) * 3 + 1] = s2[n];
        red[(wave * NT + n * 16 + lane) * 3 + 2] = cnt;
      }
    }
    __syncthreads();
    if (tid < NT) {
      float t1 = 0.f, t2 = 0.f, tn = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        t1 += red[(w * NT + tid) * 3 + 0];
        t2 += red[(w * NT + tid) * 3 + 1];
        tn += red[(w * NT + tid) * 3 + 2];
      }
      const size_t row = (size_t)b * gridDim.x + blockIdx.x;
      *reinterpret_cast<float4 *>(a.stats + (row * a.CoutW + n0 + tid) * 4) =
          make_float4(t1, t2, pivl[tid], tn);
    }
  }
}

// ---------------------------------------------------------------------------
static int nsub_for(int Cout) {
  const int n = cdiv(Cout, 16);
  if (n >= 3) return 4;
  return n;  // 1 or 2
}

static void tile_dims(int OX, int OY, int TZ, int maxM, int &TX, int &TY) {
  int txy = std::max(1, maxM / TZ);
  TX = std::max(1, (int)std::floor(std::sqrt((double)txy)));
  TY = std::max(1, txy / TX);
  if (TX > OX) { TX = OX; TY = std::max(1, std::min(OY, txy / TX)); }
  if (TY > OY) { TY = OY; TX = std::max(1, std::min(OX, txy / TY)); }
}

int plan_gconv(GConvArgs &a, int target_blocks) {
  if (a.OX <= 0 || a.OY <= 0 || a.OZ <= 0) return fail(2, "gconv: empty output grid");
  if (a.ICs % 4 != 0 || a.OCs % 4 != 0) return fail(1, "gconv: channel strides must be multiples of 4");
  const int T = a.KX * a.KY * a.KZ;
  // widest column block first; narrower ones when the weight tile of a large
  // kernel (e.g. an 8x8x2 ConvTranspose3d input gradient) does not fit in LDS
  const int ns0 = nsub_for(a.Cout);
  const int nss[3] = {ns0, std::min(ns0, 2), 1};
  a.CK = 0;
  for (int ni = 0; ni < 3 && !a.CK; ++ni) {
    if (ni > 0 && nss[ni] == nss[ni - 1]) continue;
    a.NSUB = nss[ni];
    const int NT = a.NSUB * 16;
    const int NTP = (a.NSUB & 1) ? NT : NT + 16;
    a.CoutW = round_up(a.Cout, NT);
    const int ntz = cdiv(a.OZ, 16);
    a.TZ = cdiv(a.OZ, ntz);
    const int nchunk = a.CoutW / NT;
    const int mpws[3] = {4, 2, 1};
    for (int mi = 0; mi < 3; ++mi) {
      const int MPW = mpws[mi];
      int TX, TY;
      tile_dims(a.OX, a.OY, a.TZ, 64 * MPW, TX, TY);
      const int ntx = cdiv(a.OX, TX), nty = cdiv(a.OY, TY);
      const long blocks = (long)ntx * nty * ntz * nchunk * a.B;
      if (blocks >= target_blocks || MPW == 1) {
        a.MPW = MPW;
        a.TX = TX;
        a.TY = TY;
        a.ntx = ntx;
        a.nty = nty;
        a.ntz = ntz;
        break;
      }
    }
    a.HX = (a.TX - 1) * a.sx + (a.KX - 1) * a.dx + 1;
    a.HY = (a.TY - 1) * a.sy + (a.KY - 1) * a.dy + 1;
    a.HZ = (a.TZ - 1) * a.sz + (a.KZ - 1) * a.dz + 1;
    const int HV = a.HX * a.HY * a.HZ;
    a.P = HV + ((16 - HV % 32) + 32) % 32;
    const int cks[3] = {16, 8, 4};
    for (int ci = 0; ci < 3; ++ci) {
      const int CK = cks[ci];
      if (a.ICs % CK) continue;
      const long lds = ((long)CK * a.P + (long)T * CK * NTP) * 4;
      if (lds <= 160 * 1024 - 4096) {   // gfx950: 160 KB of LDS per workgroup
        a.CK = CK;
        a.lds_bytes = (int)lds;
        break;
      }
    }
  }
  if (!a.CK)
    return fail(4, "gconv: no tile fits in LDS (K " + std::to_string(a.KX) + "x" + std::to_string(a.KY) + "x" +
                       std::to_string(a.KZ) + ", ICs " + std::to_string(a.ICs) + ", Cout " + std::to_string(a.Cout) + ")");
  const int NT = a.NSUB * 16;
  a.fHZ = FastDiv(a.HZ);
  a.fHY = FastDiv(a.HY);
  a.fTZ = FastDiv(a.TZ);
  a.fTY = FastDiv(a.TY);
  if (a.lds_bytes < (4 * NT * 3 + NT) * 4) a.lds_bytes = (4 * NT * 3 + NT) * 4;
  return 0;
}

#define GCONV_CASE(CK_, NS_, MP_)                                                            \
  if (a.CK == CK_ && a.NSUB == NS_ && a.MPW == MP_) {                                        \
    HCU_TIMED(s, "gconv_kernel<" #CK_ "," #NS_ "," #MP_ ">", gconv_flops(a), gconv_bytes(a),  \
              HCU_LAUNCH((gconv_kernel<CK_, NS_, MP_>), grid, dim3(256), a.lds_bytes, \
                                 s, a));                                                     \
    HCU_CHECK_LAUNCH();                                                                      \
    return 0;                                                                                \
  }
#define GCONV_MP(CK_, NS_) GCONV_CASE(CK_, NS_, 1) GCONV_CASE(CK_, NS_, 2) GCONV_CASE(CK_, NS_, 4)
#define GCONV_NS(CK_) GCONV_MP(CK_, 1) GCONV_MP(CK_, 2) GCONV_MP(CK_, 4)

// Algorithmic work of one launch: useful MACs (x2) and compulsory HBM bytes
// (input + output tensors read/written once, weights once).
static double gconv_flops(const GConvArgs &a) {
  if (a.flops > 0) return a.flops;
  return 2.0 * a.B * a.OX * a.OY * a.OZ * (double)a.Cout * a.KX * a.KY * a.KZ * a.ICs;
}
static double gconv_bytes(const GConvArgs &a) {
  return 4.0 * ((double)a.B * a.IX * a.IY * a.IZ * a.ICs + (double)a.B * a.OX * a.OY * a.OZ * a.OCs +
                (double)a.KX * a.KY * a.KZ * a.ICs * a.Cout);
}

int launch_gconv(const GConvArgs &a, hipStream_t s) {
  const dim3 grid(a.ntx * a.nty * a.ntz, a.CoutW / (a.NSUB * 16), a.B);
  if (grid.y > 65535 || grid.z > 65535) return fail(4, "gconv: grid too large");
  GCONV_NS(4)
  GCONV_NS(8)
  GCONV_NS(16)
  return fail(4, "gconv: unsupported variant");
}

}  // namespace hcu
