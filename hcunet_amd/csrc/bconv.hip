// bf16 implicit-GEMM convolution on v_mfma_f32_16x16x32_bf16 (the bf16 path of
// BASELINE config 3: feature_sizes [32..512]).
//
// GEMM view as conv2.hip: M = output voxels of a TX*TY*TZ tile (TZ = the whole
// Z extent, <= 16), N = output channels (x ConvTranspose3d stride phases), K =
// (tap, input channel).  One workgroup = 4 waves; wave w owns the 16-voxel
// M-subtiles w, w+4, ... (MPW of them) and all NSUB 16-column subtiles.
//
// K ordering: one K-step is 32 K-elements = TPS taps x CK channels (TPS =
// 32/CK).  Lane group g = lane/16 supplies k = 8g..8g+7 of the MFMA: 8
// consecutive channels (group c8 = g % (CK/8)) of its voxel shifted by tap
// t = s*TPS + g/(CK/8), read with ONE ds_read_b128 from the channels-last halo
// image [hv][CKP] (bf16, CKP = CK+8 pads rows so the 16 lanes of a group hit
// distinct banks).  The B fragment of lane (g, col n) is W[t][ci0+8*c8+j][n],
// j = 0..7, stored as one 16-byte run of the packed weight image
// [chunk][s][g][n][8]: each K-step is 1 + NSUB b128 reads per NSUB MFMAs per
// 16-voxel subtile, and each MFMA is 16K FLOP.
//
// Staging: the halo of the next (tile, channel chunk) is loaded into
// registers (buffer loads whose out-of-range offsets read 0) while the current
// one is computed; BatchNorm+ReLU of the producer is applied when it is written
// to LDS (fp32 arithmetic, rounded back to bf16), positions outside the input
// are 0 after the activation.  Weights of a single-chunk block are staged once.
//
// Epilogue through LDS: the fp32 accumulator tile goes to LDS, each thread
// then owns one 8-channel group and writes 16-byte bf16 runs (+ bias), taking
// the BatchNorm statistics from the fp32 values (pivot-shifted rows, common.h),
// or, for a dgrad feeding a BatchNorm backward, the fused ReLU mask and the
// (sum dz, sum dz*xhat) rows.  With a K split the fp32 partial sums go to
// `partial` and bconv_reduce adds them in a fixed order.
//
// Replaces nn.Conv3d forward / input-gradient and nn.ConvTranspose3d forward /
// input-gradient of the reference path (hcat/unet.py:246-257, 281-298) when the
// network runs under torch.autocast(dtype=torch.bfloat16).
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace hcu {

namespace {
// Halo row stride (bf16 elements).  ds_read_b128 serves a wave in 4 lane
// groups of 16 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...); with CK = 32 the
// lanes of one group read rows r of chunk g and rows r' of chunk g+1, and a
// row of 6 x 16-byte slots (CK + 16) puts all 16 on distinct bank slots for
// consecutive rows; CK = 16 uses 3 slots, CK = 8 one (rows are contiguous).
constexpr int ckp_of(int CK) { return CK == 8 ? 8 : (CK == 16 ? 24 : CK + 16); }
}

template <int CK, int NSUB, int MPW, int NPF>
__global__ void __launch_bounds__(256) bconv_kernel(const GConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT = NSUB * 16;
  constexpr int C8 = CK / 8;           // 16-byte channel groups per chunk
  constexpr int TPS = 4 / C8;          // taps per K-step
  constexpr int CKP = ckp_of(CK);      // halo row stride (bf16 elements)
  constexpr int NTP = NT + 4;          // epilogue tile row stride (floats)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int T = a.KX * a.KY * a.KZ;
  const int S = (T + TPS - 1) / TPS;
  const int HZ = a.HZ, HYZ = a.HY * a.HZ;
  const int HV = a.HX * HYZ;
  uint16_t *alds = reinterpret_cast<uint16_t *>(smem);            // [HV][CKP]
  uint16_t *wlds = reinterpret_cast<uint16_t *>(smem + a.areg);   // [S][4][NT][8]
  int *toffs = reinterpret_cast<int *>(wlds + S * 4 * NT * 8);    // [S][4]
  int *rowpk = toffs + S * 4;                                     // [MPW*64]
  int *rowoff = rowpk + MPW * 64;                                 // [MPW*64]
  // per-block coefficients live in LDS, not registers (they are only needed in
  // short phases): epilogue [6][NT] = bias, bn scale/shift/mean/invstd, stats
  // pivot per stored column; input activation [2][ICs] = scale, shift
  float *coefL = reinterpret_cast<float *>(rowoff + MPW * 64);
  float *actL = coefL + 6 * NT;

  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int n0 = blockIdx.y * NT;
  const int MT = a.TX * a.TY * a.TZ;
  const int nmsub = (MT + 15) >> 4;
  const int nchunks = a.ICs / CK;
  const int cb = blockIdx.z * a.cps, ce = min(nchunks, cb + a.cps);
  const int nck = ce - cb;
  const bool split = a.ksplit > 1;

  int vb[MPW];
#pragma unroll
  for (int j = 0; j < MPW; ++j) {
    const int i = (wave + 4 * j) * 16 + r16;
    int v = 0;
    if (i < MT) {
      int q, lz, lx, ly;
      a.fTZ.divmod(i, q, lz);
      a.fTY.divmod(q, lx, ly);
      v = lx * a.sx * HYZ + ly * a.sy * HZ + lz * a.sz;
    }
    vb[j] = v * CKP;
  }
  for (int i = tid; i < MPW * 64; i += 256) {
    int pk = -1, ro = -1;
    if (i < MT) {
      int q, lz, lx, ly;
      a.fTZ.divmod(i, q, lz);
      a.fTY.divmod(q, lx, ly);
      pk = (lx << 20) | (ly << 10) | lz;
      ro = ((lx * a.osx * a.SY + ly * a.osy) * a.SZ + lz * a.osz) * a.OCs;
    }
    rowoff[i] = ro;
    rowpk[i] = pk;
  }
  for (int e = tid; e < S * 4; e += 256) {
    const int t = (e >> 2) * TPS + (e & 3) / C8;
    int off = 0;
    if (t < T) {
      const int kz = t % a.KZ, q = t / a.KZ, ky = q % a.KY, kx = q / a.KY;
      off = kx * a.dx * HYZ + ky * a.dy * HZ + kz * a.dz;
    }
    toffs[e] = off * CKP + ((e & 3) % C8) * 8;
  }

  {
    int ph0 = 0, c00 = n0;
    if (a.nph > 1) {
      ph0 = n0 / a.Cout;
      c00 = n0 - ph0 * a.Cout;
    }
    for (int j = tid; j < NT; j += 256) {
      const int c = c00 + j;
      coefL[j] = (!split && a.bias && c < a.Cout) ? a.bias[c] : 0.f;
      const bool bn = a.bn_y && !split && c < a.OCs;
      coefL[NT + j] = bn ? a.bn_scale[c] : 0.f;
      coefL[2 * NT + j] = bn ? a.bn_shift[c] : 0.f;
      coefL[3 * NT + j] = bn ? a.bn_mean[c] : 0.f;
      coefL[4 * NT + j] = bn ? a.bn_invstd[c] : 0.f;
      coefL[5 * NT + j] = 0.f;
    }
    if (a.in_scale)
      for (int c = tid; c < a.ICs; c += 256) {
        actL[c] = a.in_scale[c];
        actL[a.ICs + c] = a.in_shift[c];
      }
  }
  auto tile_origin = [&](int tile, int &b, int &ox0, int &oy0, int &oz0) {
    int r, tzi, tyi, txi;
    a.fNT.divmod(tile, b, r);
    a.fNTZ.divmod(r, r, tzi);
    a.fNTY.divmod(r, txi, tyi);
    ox0 = txi * a.TX;
    oy0 = tyi * a.TY;
    oz0 = tzi * a.TZ;
  };
  auto stage_w = [&](int chunk) {
    const int n16 = S * 4 * NT;
    const uint4 *src = reinterpret_cast<const uint4 *>(a.w);
    for (int idx = tid; idx < n16; idx += 256) {
      const int n = idx % NT, sg = idx / NT;
      reinterpret_cast<uint4 *>(wlds)[sg * NT + n] =
          src[((size_t)chunk * S * 4 + sg) * a.CoutW + n0 + n];
    }
  };

  // ---- halo staging: thread tid owns channel group c8 = tid % C8 of halo
  // voxels v = tid / C8 + u * (256 / C8); their halo coordinates are fixed.
  constexpr int VS = 256 / C8;
  constexpr int NPFR = NPF > 0 ? NPF : 1;
  const int c8 = tid % C8;
  int hpk[NPFR];
#pragma unroll
  for (int u = 0; u < NPFR; ++u) {
    const int v = tid / C8 + u * VS;
    hpk[u] = -1;
    if (NPF > 0 && v < HV) {
      int t2, hz, hx, hy;
      a.fHZ.divmod(v, t2, hz);
      a.fHY.divmod(t2, hx, hy);
      hpk[u] = (hx << 20) | (hy << 10) | hz;
    }
  }
  const uint32_t bX = (uint32_t)a.IY * a.IZ * a.ICs * 2, bY = (uint32_t)a.IZ * a.ICs * 2,
                 bZ = (uint32_t)a.ICs * 2;
  const int sample_bytes = a.IX * a.IY * a.IZ * a.ICs * 2;
  const bool act = a.in_scale != nullptr;
  uint4 pf[NPFR];
  uint32_t okbits = 0;
  auto fetch = [&](int tile, int chunk) {
    int b, x0, y0, z0;
    tile_origin(tile, b, x0, y0, z0);
    const int gx0 = x0 * a.sx - a.px, gy0 = y0 * a.sy - a.py, gz0 = z0 * a.sz - a.pz;
    const bool inb = gx0 >= 0 && gy0 >= 0 && gz0 >= 0 && gx0 + a.HX <= a.IX &&
                     gy0 + a.HY <= a.IY && gz0 + a.HZ <= a.IZ;
    const uint16_t *bp = reinterpret_cast<const uint16_t *>(a.in) + (size_t)b * a.IX * a.IY * a.IZ * a.ICs;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, sample_bytes, 0x00020000);
    const int base_off = gx0 * (int)bX + gy0 * (int)bY + gz0 * (int)bZ + (chunk * CK + c8 * 8) * 2;
    okbits = 0;
#pragma unroll
    for (int u = 0; u < NPFR; ++u) {
      const int hp = hpk[u];
      const int hx = hp >> 20, hy = (hp >> 10) & 1023, hz = hp & 1023;
      const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
      const bool ok = hp >= 0 && (inb || ((unsigned)gx < (unsigned)a.IX &&
                                          (unsigned)gy < (unsigned)a.IY &&
                                          (unsigned)gz < (unsigned)a.IZ));
      const int off = ok ? base_off + (int)(__umul24(hx, bX) + __umul24(hy, bY) + __umul24(hz, bZ))
                         : 0x7ffffff0;
      pf[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      okbits |= (ok ? 1u : 0u) << u;
    }
  };
  // BatchNorm+ReLU of 8 channels (fp32), 0 outside the input
  // BatchNorm+ReLU of 8 channels (fp32; coefficients from LDS), 0 outside the input
  auto activate = [&](uint4 v, bool ok, int chunk) -> uint4 {
    if (!ok) return make_uint4(0u, 0u, 0u, 0u);
    if (!act) return v;
    const int c = chunk * CK + c8 * 8;
    const float4 s0 = *reinterpret_cast<const float4 *>(actL + c);
    const float4 s1 = *reinterpret_cast<const float4 *>(actL + c + 4);
    const float4 h0 = *reinterpret_cast<const float4 *>(actL + a.ICs + c);
    const float4 h1 = *reinterpret_cast<const float4 *>(actL + a.ICs + c + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], sc[k], sh[k]), 0.f);
    return pack8(f);
  };
  // direct (non-prefetched) staging of one (tile, chunk) halo
  auto stage_direct = [&](int tile, int chunk) {
    int b, x0, y0, z0;
    tile_origin(tile, b, x0, y0, z0);
    const int gx0 = x0 * a.sx - a.px, gy0 = y0 * a.sy - a.py, gz0 = z0 * a.sz - a.pz;
    const uint16_t *bp = reinterpret_cast<const uint16_t *>(a.in) + (size_t)b * a.IX * a.IY * a.IZ * a.ICs;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, sample_bytes, 0x00020000);
    for (int base = tid / C8; base < HV; base += 4 * VS) {
      uint4 val[4];
      bool okv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = base + u * VS;
        int t2, hz, hx, hy;
        a.fHZ.divmod(v, t2, hz);
        a.fHY.divmod(t2, hx, hy);
        const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
        const bool ok = v < HV && (unsigned)gx < (unsigned)a.IX && (unsigned)gy < (unsigned)a.IY &&
                        (unsigned)gz < (unsigned)a.IZ;
        const int off = ok ? gx * (int)bX + gy * (int)bY + gz * (int)bZ + (chunk * CK + c8 * 8) * 2
                           : 0x7ffffff0;
        val[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        okv[u] = ok;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = base + u * VS;
        if (v < HV)
          *reinterpret_cast<uint4 *>(alds + v * CKP + c8 * 8) = activate(val[u], okv[u], chunk);
      }
    }
  };

  floatx4 acc[MPW][NSUB];
  auto load_frag = [&](int s, int toff, shortx8 (&bfr)[NSUB], shortx8 (&afr)[MPW]) {
    const int ss = min(s, S - 1);
#pragma unroll
    for (int n = 0; n < NSUB; ++n)
      bfr[n] = *reinterpret_cast<const shortx8 *>(wlds + ((ss * 4 + g) * NT + n * 16 + r16) * 8);
#pragma unroll
    for (int j = 0; j < MPW; ++j) afr[j] = *reinterpret_cast<const shortx8 *>(alds + vb[j] + toff);
  };
  auto toff_of = [&](int s) { return toffs[min(s, S - 1) * 4 + g]; };
  auto mfma_frag = [&](const shortx8 (&bfr)[NSUB], const shortx8 (&afr)[MPW]) {
#pragma unroll
    for (int j = 0; j < MPW; ++j)
#pragma unroll
      for (int n = 0; n < NSUB; ++n)
        acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j], bfr[n], acc[j][n], 0, 0, 0);
  };
  auto compute = [&]() {
    shortx8 b0[NSUB], a0[MPW], b1[NSUB], a1[MPW];
    int tA = toff_of(0), tB = toff_of(1);
    load_frag(0, tA, b0, a0);
    tA = toff_of(2);
    for (int s = 0; s < S; s += 2) {
      load_frag(s + 1, tB, b1, a1);
      tB = toff_of(s + 3);
      __builtin_amdgcn_sched_barrier(0);
      mfma_frag(b0, a0);
      load_frag(s + 2, tA, b0, a0);
      tA = toff_of(s + 4);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < S) mfma_frag(b1, a1);
    }
  };

  // ---- epilogue (through LDS, 8 channels = 16 bytes per store)
  const int nc8 = a.nc4;                 // 8-channel groups of the block's stored columns
  const int ec8 = tid % nc8;
  int ph = 0, co0 = n0;
  if (a.nph > 1) {
    ph = n0 / a.Cout;
    co0 = n0 - ph * a.Cout;
  }
  const int qz = ph % a.phz, qy = (ph / a.phz) % a.phy, qx = ph / (a.phz * a.phy);
  const int cst = co0 + ec8 * 8;         // first stored channel of this thread
  const bool cok = cst < a.OCs;
  const bool fwdstat = a.stats && !a.bn_y && !split;
  float st1[8], st2[8], cnt = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) st1[k] = st2[k] = 0.f;
  bool have_piv = false;
  // 8 consecutive LDS floats of coefficient array q for this thread's channels
  auto coef8 = [&](int q, float (&o)[8]) {
    const float4 c0 = *reinterpret_cast<const float4 *>(coefL + q * NT + ec8 * 8);
    const float4 c1 = *reinterpret_cast<const float4 *>(coefL + q * NT + ec8 * 8 + 4);
    o[0] = c0.x; o[1] = c0.y; o[2] = c0.z; o[3] = c0.w;
    o[4] = c1.x; o[5] = c1.y; o[6] = c1.z; o[7] = c1.w;
  };
  float *dstf = split ? a.partial + (size_t)blockIdx.z * a.slice_floats : nullptr;
  uint16_t *dsth = reinterpret_cast<uint16_t *>(a.out);
  const uint16_t *ybf = reinterpret_cast<const uint16_t *>(a.bn_y);
  auto epilogue = [&](int b, int ox0, int oy0, int oz0) {
    __syncthreads();   // every wave is done reading the halo image
#pragma unroll
    for (int j = 0; j < MPW; ++j) {
      const int m = wave + 4 * j;
      if (m < nmsub) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int n = 0; n < NSUB; ++n)
            smem[(m * 16 + g * 4 + r) * NTP + n * 16 + r16] = acc[j][n][r];
      }
    }
    __syncthreads();
    float bias8[8], piv[8];
    coef8(0, bias8);
    if (fwdstat && !have_piv) {   // pivot: the block's first output voxel (row 0)
#pragma unroll
      for (int k = 0; k < 8; ++k) piv[k] = smem[ec8 * 8 + k] + bias8[k];
      if (tid < nc8)
#pragma unroll
        for (int k = 0; k < 8; ++k) coefL[5 * NT + ec8 * 8 + k] = piv[k];
      have_piv = true;
    } else {
      coef8(5, piv);
    }
    const size_t tbase =
        ((((size_t)b * a.SX + ox0 * a.osx + a.ofx + qx) * a.SY + oy0 * a.osy + a.ofy + qy) * a.SZ +
         oz0 * a.osz + a.ofz + qz) * a.OCs + cst;
    const bool interior = ox0 + a.TX <= a.OX && oy0 + a.TY <= a.OY && oz0 + a.TZ <= a.OZ;
    const int vstep = 256 / nc8;
    for (int i = tid / nc8; i < MT; i += vstep) {
      bool ok = cok;
      if (!interior) {
        const int pk = rowpk[i];
        ok = ok && ox0 + (pk >> 20) < a.OX && oy0 + ((pk >> 10) & 1023) < a.OY &&
             oz0 + (pk & 1023) < a.OZ;
      }
      if (!ok) continue;
      const float4 v0 = *reinterpret_cast<const float4 *>(smem + i * NTP + ec8 * 8);
      const float4 v1 = *reinterpret_cast<const float4 *>(smem + i * NTP + ec8 * 8 + 4);
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      const size_t off = tbase + rowoff[i];
      if (split) {
        *reinterpret_cast<float4 *>(dstf + off) = v0;
        *reinterpret_cast<float4 *>(dstf + off + 4) = v1;
        continue;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += bias8[k];
      if (a.bn_y) {   // fused BatchNorm+ReLU backward: v = dA -> dz; (dz, dz*xhat)
        float y[8], bsc[8], bsh[8], bmu[8], bis[8];
        coef8(1, bsc);
        coef8(2, bsh);
        coef8(3, bmu);
        coef8(4, bis);
        unpack8(*reinterpret_cast<const uint4 *>(ybf + off), y);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          v[k] = fmaf(y[k], bsc[k], bsh[k]) > 0.f ? v[k] : 0.f;
          st1[k] += v[k];
          st2[k] = fmaf(v[k], (y[k] - bmu[k]) * bis[k], st2[k]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = v[k] - piv[k];
          st1[k] += d;
          st2[k] = fmaf(d, d, st2[k]);
        }
      }
      cnt += 1.f;
      *reinterpret_cast<uint4 *>(dsth + off) = pack8(v);
    }
  };

  // ---- main loop over (tile, chunk) items
  // contiguous tile range per block: consecutive tiles share halo rows, which
  // then come from this CU's L1/L2 instead of HBM
  const int tpb_ = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t_beg = blockIdx.x * tpb_, t_end = min(total, t_beg + tpb_);
  if (NPF > 0) {
    int tile = t_beg;
    if (tile < t_end) fetch(tile, cb);
    if (nck == 1) stage_w(cb);
    for (; tile < t_end; ++tile) {
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) acc[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int chunk = cb; chunk < ce; ++chunk) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < NPFR; ++u)
          if (hpk[u] >= 0)
            *reinterpret_cast<uint4 *>(alds + (tid / C8 + u * VS) * CKP + c8 * 8) =
                activate(pf[u], (okbits >> u) & 1u, chunk);
        if (nck > 1) stage_w(chunk);
        __syncthreads();
        int nt = tile, nc = chunk + 1;
        if (nc == ce) {
          nc = cb;
          nt = tile + 1;
        }
        if (nt < t_end) fetch(nt, nc);
        compute();
      }
      int b, ox0, oy0, oz0;
      tile_origin(tile, b, ox0, oy0, oz0);
      epilogue(b, ox0, oy0, oz0);
    }
  } else {
    for (int tile = t_beg; tile < t_end; ++tile) {
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) acc[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int chunk = cb; chunk < ce; ++chunk) {
        __syncthreads();
        stage_direct(tile, chunk);
        stage_w(chunk);
        __syncthreads();
        compute();
      }
      int b, ox0, oy0, oz0;
      tile_origin(tile, b, ox0, oy0, oz0);
      epilogue(b, ox0, oy0, oz0);
    }
  }

  // ---- statistics rows: fixed-order combine of the threads of a channel group
  if (!a.stats || split) return;
  float *red = smem;   // [256][3]
  for (int k = 0; k < 8; ++k) {
    __syncthreads();
    red[tid * 3 + 0] = st1[k];
    red[tid * 3 + 1] = st2[k];
    red[tid * 3 + 2] = cnt;
    __syncthreads();
    if (tid < nc8) {
      float t1 = 0.f, t2 = 0.f, tn = 0.f;
      for (int q = tid; q < 256; q += nc8) {
        t1 += red[q * 3 + 0];
        t2 += red[q * 3 + 1];
        tn += red[q * 3 + 2];
      }
      const int c = n0 + tid * 8 + k;
      const size_t row = blockIdx.x;
      if (fwdstat)
        *reinterpret_cast<float4 *>(a.stats + (row * a.CoutW + c) * 4) =
            make_float4(t1, t2, coefL[5 * NT + tid * 8 + k], tn);
      else {
        a.stats[(row * a.CoutW + c) * 2 + 0] = t1;
        a.stats[(row * a.CoutW + c) * 2 + 1] = t2;
      }
    }
  }
}

// Sum of the K-split fp32 slices in a fixed order + bias -> bf16 output, with
// the BatchNorm statistics rows (pivoted) or the fused BatchNorm-backward rows.
// Thread tid owns 8-channel group c8 = tid % C8o of voxels v0 + tid/C8o + k*(256/C8o).
__global__ void __launch_bounds__(256) bconv_reduce_kernel(const GConvArgs a, int vox_per_block) {
  __shared__ float red[256][3];
  const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
  const int C8o = a.OCs / 8;
  const int tid = threadIdx.x;
  const int c8 = tid % C8o;
  const int vstep = 256 / C8o;
  const int64_t v0 = (int64_t)blockIdx.x * vox_per_block;
  const int64_t v1 = min(v0 + vox_per_block, nvox);
  float bv[8], bsc[8], bsh[8], bmu[8], bis[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c8 * 8 + k;
    bv[k] = (a.bias && c < a.Cout) ? a.bias[c] : 0.f;
    bsc[k] = bsh[k] = bmu[k] = bis[k] = 0.f;
    if (a.bn_y) {
      bsc[k] = a.bn_scale[c];
      bsh[k] = a.bn_shift[c];
      bmu[k] = a.bn_mean[c];
      bis[k] = a.bn_invstd[c];
    }
  }
  auto vsum = [&](int64_t v, float (&s)[8]) {
    const size_t off = (size_t)v * a.OCs + c8 * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = bv[k];
    for (int q = 0; q < a.ksplit; ++q) {
      const float4 p0 = *reinterpret_cast<const float4 *>(a.partial + (size_t)q * a.slice_floats + off);
      const float4 p1 = *reinterpret_cast<const float4 *>(a.partial + (size_t)q * a.slice_floats + off + 4);
      s[0] += p0.x; s[1] += p0.y; s[2] += p0.z; s[3] += p0.w;
      s[4] += p1.x; s[5] += p1.y; s[6] += p1.z; s[7] += p1.w;
    }
  };
  const bool fwdstat = a.stats && !a.bn_y;
  float piv[8], st1[8], st2[8], cnt = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) piv[k] = st1[k] = st2[k] = 0.f;
  if (fwdstat) vsum(v0, piv);
  uint16_t *out = reinterpret_cast<uint16_t *>(a.out);
  const uint16_t *ybf = reinterpret_cast<const uint16_t *>(a.bn_y);
  for (int64_t v = v0 + tid / C8o; v < v1; v += vstep) {
    const size_t off = (size_t)v * a.OCs + c8 * 8;
    float s[8];
    vsum(v, s);
    if (a.bn_y) {
      float y[8];
      unpack8(*reinterpret_cast<const uint4 *>(ybf + off), y);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] = fmaf(y[k], bsc[k], bsh[k]) > 0.f ? s[k] : 0.f;
        st1[k] += s[k];
        st2[k] = fmaf(s[k], (y[k] - bmu[k]) * bis[k], st2[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = s[k] - piv[k];
        st1[k] += d;
        st2[k] = fmaf(d, d, st2[k]);
      }
    }
    cnt += 1.f;
    *reinterpret_cast<uint4 *>(out + off) = pack8(s);
  }
  if (!a.stats) return;
  for (int k = 0; k < 8; ++k) {
    __syncthreads();
    red[tid][0] = st1[k];
    red[tid][1] = st2[k];
    red[tid][2] = cnt;
    __syncthreads();
    if (tid < C8o) {
      float t1 = 0.f, t2 = 0.f, tn = 0.f;
      for (int q = tid; q < 256; q += C8o) {
        t1 += red[q][0];
        t2 += red[q][1];
        tn += red[q][2];
      }
      const int c = tid * 8 + k;
      if (fwdstat)
        *reinterpret_cast<float4 *>(a.stats + ((size_t)blockIdx.x * a.CoutW + c) * 4) =
            make_float4(t1, t2, piv[k], tn);
      else {
        a.stats[((size_t)blockIdx.x * a.CoutW + c) * 2 + 0] = t1;
        a.stats[((size_t)blockIdx.x * a.CoutW + c) * 2 + 1] = t2;
      }
    }
  }
}

// ---------------------------------------------------------------------------
static int env_int_b(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}

static void btile(int OX, int OY, int TZ, int maxM, int &TX, int &TY) {
  const int txy = std::max(1, maxM / TZ);
  TX = 1;
  while ((TX + 1) * (TX + 1) <= txy) ++TX;
  TY = std::max(1, txy / TX);
  if (TX > OX) { TX = OX; TY = std::max(1, std::min(OY, txy / TX)); }
  if (TY > OY) { TY = OY; TX = std::max(1, std::min(OX, txy / TY)); }
}

static long bconv_areg(const GConvArgs &a, int CK, int NT) {
  const long HV = (long)a.HX * a.HY * a.HZ;
  const long halo_f = (HV * ckp_of(CK) + 1) / 2;       // bf16 image, in floats
  const long ctile = (long)a.MPW * 64 * (NT + 4);      // fp32 epilogue tile
  return (std::max(halo_f, ctile) + 3) & ~3L;
}

static long bconv_lds(const GConvArgs &a, int CK, int NT) {
  const int T = a.KX * a.KY * a.KZ;
  const int TPS = 32 / CK;
  const int S = (T + TPS - 1) / TPS;
  return std::max(bconv_areg(a, CK, NT) + (long)S * 4 * NT * 4 + S * 4 + (long)a.MPW * 128 +
                      6L * NT + 2L * a.ICs,
                  256L * 3) * 4;
}

static int reduce_vpb(const GConvArgs &a) { return 2 * 256 / (a.OCs / 8); }

int bconv_stat_rows(const GConvArgs &a) {
  if (a.ksplit > 1) {
    const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
    const int vpb = reduce_vpb(a);
    return (int)((nvox + vpb - 1) / vpb);
  }
  return a.gridx;
}

int plan_bconv(GConvArgs &a, int target_blocks) {
  a.use_bconv = 0;
  if (a.OX <= 0 || a.OY <= 0 || a.OZ <= 0) return fail(2, "bconv: empty output grid");
  if (a.ICs % 8 || a.OCs % 8) return fail(4, "bconv: channel strides must be multiples of 8");
  if (a.nph < 1) a.nph = 1;
  if (a.phx < 1) a.phx = 1;
  if (a.phy < 1) a.phy = 1;
  if (a.phz < 1) a.phz = 1;
  const int T = a.KX * a.KY * a.KZ;
  const int Nlog = a.Cout * a.nph;
  const int nb16 = cdiv(Nlog, 16);
  const int ntz = cdiv(a.OZ, 16);
  a.TZ = cdiv(a.OZ, ntz);
  const long lds_cap = env_int_b("HCU_BCONV_LDS_KB", 80) * 1024L;
  // Candidate tilings, scored by a simple per-CU time model (cycles):
  //   per (tile, chunk): MFMA S * MPW * NSUB * 16 per wave, staging ~
  //   1200 + 40 per 16-byte element per thread (+ weights when multi-chunk);
  //   per tile: epilogue ~1500; two resident blocks hide ~40 % of a block's
  //   staging behind the other's MFMAs.
  double best = 1e300;
  GConvArgs bestA = a;
  bool found = false;
  const int mpws[3] = {4, 2, 1}, nsubs[3] = {4, 2, 1}, cks[3] = {32, 16, 8};
  for (int ni = 0; ni < 3; ++ni) {
    const int NSUB = nsubs[ni];
    if (NSUB > 1 && nb16 < NSUB && !(NSUB == 2 && nb16 >= 2)) continue;
    if (NSUB == 4 && nb16 < 4) continue;
    if (NSUB == 2 && nb16 < 2) continue;
    if (a.nph > 1 && (a.Cout % (NSUB * 16) || a.Cout % 8)) continue;
    const int NT = NSUB * 16;
    const int CoutW = round_up(Nlog, NT);
    const int nN = CoutW / NT;
    for (int mi = 0; mi < 3; ++mi) {
      const int MPW = mpws[mi];
      GConvArgs c = a;
      int TX, TY;
      btile(a.OX, a.OY, a.TZ, 64 * MPW, TX, TY);
      c.MPW = MPW;
      c.NSUB = NSUB;
      c.CoutW = CoutW;
      c.TX = TX;
      c.TY = TY;
      c.HX = (TX - 1) * a.sx + (a.KX - 1) * a.dx + 1;
      c.HY = (TY - 1) * a.sy + (a.KY - 1) * a.dy + 1;
      c.HZ = (a.TZ - 1) * a.sz + (a.KZ - 1) * a.dz + 1;
      const long tiles = (long)cdiv(a.OX, TX) * cdiv(a.OY, TY) * ntz * a.B;
      const int MT = TX * TY * a.TZ;
      for (int ki = 0; ki < 3; ++ki) {
        const int CK = cks[ki];
        if (a.ICs % CK) continue;
        const long lds = bconv_lds(c, CK, NT);
        if (lds > lds_cap) continue;
        const int occ = std::max(1, std::min(2, (int)(160 * 1024 / lds)));
        const int chunks = a.ICs / CK;
        const int TPS = 32 / CK;
        const int S = (T + TPS - 1) / TPS;
        const double helem = (double)c.HX * c.HY * c.HZ * (CK / 8) / 256.0;
        const double welem = chunks > 1 ? (double)S * 4 * NT / 256.0 : 0.0;
        const double t_mfma = (double)S * MPW * NSUB * 16.0;
        const double t_stage = 1200.0 + 40.0 * (helem + welem);
        const double hide = occ > 1 ? 0.6 : 1.0;
        const double t_tile = chunks * (t_mfma + hide * t_stage) + 1500.0 * hide;
        // blocks: tiles x N blocks (K split added below when this is too few)
        const double blocks = (double)tiles * nN;
        const double waves = std::max(1.0, blocks / (256.0 * occ));
        const double util = (double)MT / (MPW * 64.0) * std::min(1.0, (double)Nlog / CoutW);
        const double cost = waves * t_tile * occ / std::max(0.25, util) *
                            (blocks < 256.0 * occ ? 256.0 * occ / blocks * 0.5 + 0.5 : 1.0);
        if (cost < best) {
          best = cost;
          bestA = c;
          bestA.CK = CK;
          bestA.lds_bytes = (int)lds;
          found = true;
        }
      }
    }
  }
  if (!found) return fail(4, "bconv: no tile fits in LDS");
  a = bestA;
  const int NT = a.NSUB * 16;
  const int nN = a.CoutW / NT;
  a.ntx = cdiv(a.OX, a.TX);
  a.nty = cdiv(a.OY, a.TY);
  a.ntz = ntz;
  const long tiles = (long)a.ntx * a.nty * a.ntz * a.B;
  const int nchunks = a.ICs / a.CK;
  int ks = 1;
  const int ks_target = env_int_b("HCU_BCONV_KS_TARGET", 256);
  if (a.nph == 1 && 256 % (a.OCs / 8) == 0)
    while (ks < nchunks && tiles * nN * ks < ks_target) ks *= 2;
  ks = std::min(ks, nchunks);
  a.cps = cdiv(nchunks, ks);
  a.ksplit = cdiv(nchunks, a.cps);
  a.slice_floats = (size_t)a.B * a.SX * a.SY * a.SZ * a.OCs;
  const long nel = (long)a.HX * a.HY * a.HZ * (a.CK / 8);
  const long per_thread = (nel + 255) / 256;
  a.NPF = per_thread <= 4 ? 4 : per_thread <= 8 ? 8 : per_thread <= 12 ? 12 : per_thread <= 16 ? 16 : 0;
  const int occ = std::max(1, std::min(2, (int)(160 * 1024 / a.lds_bytes)));
  const long slots = (long)256 * occ;
  const long per_tile = (long)nN * a.ksplit;
  a.gridx = (int)std::min(tiles, std::max(1L, slots / per_tile));
  a.fHZ = FastDiv(a.HZ);
  a.fHY = FastDiv(a.HY);
  a.fTZ = FastDiv(a.TZ);
  a.fTY = FastDiv(a.TY);
  a.fNT = FastDiv(a.ntx * a.nty * a.ntz);
  a.fNTZ = FastDiv(a.ntz);
  a.fNTY = FastDiv(a.nty);
  a.nc4 = std::min(NT, a.OCs) / 8;   // 8-channel groups stored per block
  a.epi_lds = 1;
  a.areg = (int)bconv_areg(a, a.CK, NT);
  a.use_bconv = 1;
  a.use_conv2 = 0;
  a.use_conv8 = 0;
  if (env_int_b("HCU_CONV2_LOG", 0))
    fprintf(stderr,
            "bconv plan: B%d I%dx%dx%d ICs%d O%dx%dx%d S%dx%dx%d OCs%d Cout%d K%dx%dx%d s%d%d%d nph%d"
            " | CK%d NSUB%d MPW%d T%dx%dx%d ks%d cps%d NPF%d gridx%d lds%d\n",
            a.B, a.IX, a.IY, a.IZ, a.ICs, a.OX, a.OY, a.OZ, a.SX, a.SY, a.SZ, a.OCs, a.Cout, a.KX,
            a.KY, a.KZ, a.sx, a.sy, a.sz, a.nph, a.CK, a.NSUB, a.MPW, a.TX, a.TY, a.TZ, a.ksplit,
            a.cps, a.NPF, a.gridx, a.lds_bytes);
  (void)target_blocks;
  return 0;
}

#define BCONV_CASE(CK_, NS_, MP_, PF_)                                                         \
  if (a.CK == CK_ && a.NSUB == NS_ && a.MPW == MP_ && a.NPF == PF_) {                           \
    HCU_TIMED(s, "bconv_kernel<" #CK_ "," #NS_ "," #MP_ "," #PF_ ">", fl, by,                     \
              hipLaunchKernelGGL((bconv_kernel<CK_, NS_, MP_, PF_>), grid, dim3(256),           \
                                 a.lds_bytes, s, a));                                           \
    launched = true;                                                                            \
  }
#define BCONV_PF(CK_, NS_, MP_)                                                          \
  BCONV_CASE(CK_, NS_, MP_, 0) else BCONV_CASE(CK_, NS_, MP_, 4) else                    \
  BCONV_CASE(CK_, NS_, MP_, 8) else BCONV_CASE(CK_, NS_, MP_, 12) else                   \
  BCONV_CASE(CK_, NS_, MP_, 16)
#define BCONV_MP(CK_, NS_) BCONV_PF(CK_, NS_, 1) else BCONV_PF(CK_, NS_, 2) else BCONV_PF(CK_, NS_, 4)
#define BCONV_NS(CK_) BCONV_MP(CK_, 1) else BCONV_MP(CK_, 2) else BCONV_MP(CK_, 4)

int launch_bconv(const GConvArgs &a, hipStream_t s) {
  const dim3 grid(a.gridx, a.CoutW / (a.NSUB * 16), a.ksplit);
  if (grid.y > 65535 || grid.z > 65535) return fail(4, "bconv: grid too large");
  if (a.ksplit > 1 && !a.partial) return fail(5, "bconv: K split needs a partial workspace");
  const double fl = a.flops > 0 ? a.flops
                                : 2.0 * a.B * a.OX * a.OY * a.OZ * (double)a.Cout * a.nph * a.KX *
                                      a.KY * a.KZ * a.ICs;
  const double by = 2.0 * ((double)a.B * a.IX * a.IY * a.IZ * a.ICs +
                           (double)a.B * a.SX * a.SY * a.SZ * a.OCs);
  bool launched = false;
  BCONV_NS(8) else BCONV_NS(16) else BCONV_NS(32)
  if (!launched) return fail(4, "bconv: unsupported variant");
  HCU_CHECK_LAUNCH();
  if (a.ksplit > 1) {
    const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
    const int vpb = reduce_vpb(a);
    const int blocks = (int)((nvox + vpb - 1) / vpb);
    HCU_TIMED(s, "bconv_reduce_kernel", 0.0, (4.0 * a.ksplit + 2.0) * a.slice_floats,
              hipLaunchKernelGGL(bconv_reduce_kernel, dim3(blocks), dim3(256), 0, s, a, vpb));
    HCU_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace hcu
