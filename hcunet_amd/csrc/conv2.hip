// Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_16x16x4_f32), second
// generation: channels-last LDS images read with ds_read_b128.
//
// GEMM view: M = output voxels of a TX*TY*TZ tile, N = output channels, K =
// (tap, input channel).  One workgroup = 4 waves; wave w owns the 16-voxel
// M-subtiles w, w+4, ... (MPW of them) and all NSUB*16 output channels of the
// block.
//
// K ordering (a permutation of the reduction, so any order is exact): one
// "step" covers 16 K-elements = (taps per step TPS) x CK channels, TPS = 16/CK.
// Lane group g = lane/16 reads ONE ds_read_b128 = 4 consecutive channels
// (c4 = g % (CK/4)) of its voxel shifted by tap t = s*TPS + g/(CK/4); component
// j of that float4 feeds MFMA j.  The B fragment of lane (g, n) for MFMA j is
// W[t][ci0 + 4*c4 + j][n], stored as one float4 in LDS, so each step is
// 1 + NSUB b128 reads per (4 * NSUB) MFMAs per 16-voxel subtile.
//
// The input halo of the tile (BatchNorm+ReLU of the producer applied while
// staging, zero outside the input) is staged channels-last as [hv][CKP]; the
// block's weight slice as [s][g][NT][4].  Weights are read from the generic
// prepared layout wg[t][ICs][CoutW] (prep_conv_* / prep_convt_*).
//
// K split: blockIdx.z selects a range of channel chunks; with ksplit > 1 the
// raw partial sums go to `partial` ([ksplit][B][SX][SY][SZ][OCs]) and
// conv2_reduce adds them (fixed order), the bias and the BatchNorm partial
// statistics.
//
// Replaces the arithmetic of nn.Conv3d forward/input-gradient and
// nn.ConvTranspose3d forward/input-gradient on the reference path
// (hcat/unet.py:246-257, 281-298).
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace hcu {

template <int CK, int NSUB, int MPW, int NPF>
__global__ void __launch_bounds__(256) conv2_kernel(const GConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT = NSUB * 16;
  constexpr int C4 = CK / 4;
  constexpr int TPS = 4 / C4;          // taps per K-step
  constexpr int CKP = CK + 4;          // padded channel stride of the halo image
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int T = a.KX * a.KY * a.KZ;
  const int S = (T + TPS - 1) / TPS;
  const int HZ = a.HZ, HYZ = a.HY * a.HZ;
  const int HV = a.HX * HYZ;
  const int nel = HV * C4;             // float4 elements of one halo image
  float *alds = smem;                                  // [HV][CKP]
  float *wlds = smem + a.areg;                         // [S][4][NT][4] (areg >= HV*CKP, C tile)
  int *toffs = reinterpret_cast<int *>(wlds + S * 4 * NT * 4);  // [S][4]
  int *rowpk = toffs + S * 4;                                    // [MPW*64] (lx,ly,lz) of GEMM rows
  int *rowoff = rowpk + MPW * 64;                                // [MPW*64] store offset in the tile

  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int n0 = blockIdx.y * NT;
  const int MT = a.TX * a.TY * a.TZ;
  const int nmsub = (MT + 15) >> 4;
  const int nchunks = a.ICs / CK;
  const int cb = blockIdx.z * a.cps, ce = min(nchunks, cb + a.cps);

  // per-lane voxel offsets (halo coordinates) of the A rows: same for every tile
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
    int pk = -1;
    if (i < MT) {
      int q, lz, lx, ly;
      a.fTZ.divmod(i, q, lz);
      a.fTY.divmod(q, lx, ly);
      pk = (lx << 20) | (ly << 10) | lz;
      rowoff[i] = ((lx * a.osx * a.SY + ly * a.osy) * a.SZ + lz * a.osz) * a.OCs;
    } else {
      rowoff[i] = -1;
    }
    rowpk[i] = pk;
  }
  // tap offsets per (step, lane group); padded taps read voxel 0 (weights are 0)
  for (int e = tid; e < S * 4; e += 256) {
    const int t = (e >> 2) * TPS + (e & 3) / C4;
    int off = 0;
    if (t < T) {
      const int kz = t % a.KZ, q = t / a.KZ, ky = q % a.KY, kx = q / a.KY;
      off = kx * a.dx * HYZ + ky * a.dy * HZ + kz * a.dz;
    }
    toffs[e] = off * CKP + ((e & 3) % C4) * 4;
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
  // one halo element (float4 of 4 channels) of a tile, BN+ReLU applied; 0 outside
  auto halo_elem = [&](int idx, int b, int gx0, int gy0, int gz0, int ci0) -> float4 {
    float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
    const int c4 = idx % C4;
    const int v = idx / C4;
    int t2, hz, hx, hy;
    a.fHZ.divmod(v, t2, hz);
    a.fHY.divmod(t2, hx, hy);
    const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
    if ((unsigned)gx < (unsigned)a.IX && (unsigned)gy < (unsigned)a.IY &&
        (unsigned)gz < (unsigned)a.IZ) {
      const int c = ci0 + c4 * 4;
      val = *reinterpret_cast<const float4 *>(
          a.in + ((((size_t)b * a.IX + gx) * a.IY + gy) * a.IZ + gz) * a.ICs + c);
      if (a.in_scale) {
        const float4 sc = *reinterpret_cast<const float4 *>(a.in_scale + c);
        const float4 sh = *reinterpret_cast<const float4 *>(a.in_shift + c);
        val.x = fmaxf(fmaf(val.x, sc.x, sh.x), 0.f);
        val.y = fmaxf(fmaf(val.y, sc.y, sh.y), 0.f);
        val.z = fmaxf(fmaf(val.z, sc.z, sh.z), 0.f);
        val.w = fmaxf(fmaf(val.w, sc.w, sh.w), 0.f);
      }
    }
    return val;
  };
  auto halo_dst = [&](int idx) { return (idx / C4) * CKP + (idx % C4) * 4; };
  // weight slice of one channel chunk: contiguous float4 copies from the packed layout
  auto stage_w = [&](int chunk) {
    const int n4 = S * 4 * NT;
    const float4 *src = reinterpret_cast<const float4 *>(a.w);
    for (int idx = tid; idx < n4; idx += 256) {
      const int n = idx % NT, sg = idx / NT;
      reinterpret_cast<float4 *>(wlds)[sg * NT + n] =
          src[((size_t)chunk * S * 4 + sg) * a.CoutW + n0 + n];
    }
  };

  floatx4 acc[MPW][NSUB];
  // Subtiles past the tile (m >= nmsub) read voxel 0 and are never stored, so
  // the step body has no per-subtile branch and the MFMA chains interleave.
  // Software-pipelined over the K-steps with two register sets: the fragments
  // of step s+1 are loaded before the MFMAs of step s (a scheduling barrier
  // keeps that order), so the LDS latency hides behind 4*MPW*NSUB MFMAs.
  auto load_frag = [&](int s, int toff, floatx4 (&bfr)[NSUB], floatx4 (&afr)[MPW]) {
    const int ss = min(s, S - 1);  // past the end: re-read valid LDS, never used
#pragma unroll
    for (int n = 0; n < NSUB; ++n)
      bfr[n] = *reinterpret_cast<const floatx4 *>(wlds + ((ss * 4 + g) * NT + n * 16 + r16) * 4);
#pragma unroll
    for (int j = 0; j < MPW; ++j) afr[j] = *reinterpret_cast<const floatx4 *>(alds + vb[j] + toff);
  };
  auto toff_of = [&](int s) { return toffs[min(s, S - 1) * 4 + g]; };
  auto mfma_frag = [&](const floatx4 (&bfr)[NSUB], const floatx4 (&afr)[MPW]) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n)
          acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(afr[j][c], bfr[n][c], acc[j][n], 0, 0, 0);
  };
  auto compute = [&]() {
    floatx4 b0[NSUB], a0[MPW], b1[NSUB], a1[MPW];
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

  const bool split = a.ksplit > 1;
  float *dst = split ? a.partial + (size_t)blockIdx.z * a.slice_floats : a.out;
  // Forward statistics are taken about a block-wide pivot per channel (the
  // value of the block's first output voxel; StatRow in common.h); the fused
  // BatchNorm-backward sums (bn_y set) are plain sums.
  const bool fwdstat = a.stats && !a.bn_y && !split;
  float *pivl = reinterpret_cast<float *>(rowoff + MPW * 64);   // [NT] pivot broadcast
  float pv[NSUB], cnt = 0.f;
  bool have_piv = false;
  // per-column store offset relative to the voxel (channel + output phase), or -1
  float s1[NSUB], s2[NSUB], bias_v[NSUB];
  int coff[NSUB];
  bool cst[NSUB];
#pragma unroll
  for (int n = 0; n < NSUB; ++n) {
    s1[n] = s2[n] = pv[n] = 0.f;
    const int nn = n0 + n * 16 + r16;
    bias_v[n] = (!split && a.bias && nn < a.Cout * a.nph) ? a.bias[nn % a.Cout] : 0.f;
    int off = -1, co = nn;
    if (a.nph > 1) {
      if (nn < a.Cout * a.nph) {
        const int ph = nn / a.Cout;
        co = nn - ph * a.Cout;
        const int qz = ph % a.phz, qq = ph / a.phz, qy = qq % a.phy, qx = qq / a.phy;
        off = ((qx * a.SY + qy) * a.SZ + qz) * a.OCs + co;
      }
    } else if (nn < a.OCs) {
      off = nn;   // padded channels < OCs are stored as 0
    }
    coff[n] = off;
    cst[n] = off >= 0 && co < a.Cout;
  }
  const bool zpad = a.nph > 1 && a.OCs > a.Cout;
  auto epilogue = [&](int b, int ox0, int oy0, int oz0) {
    float *tp = dst + ((((size_t)b * a.SX + ox0 * a.osx + a.ofx) * a.SY + oy0 * a.osy + a.ofy) *
                           a.SZ + oz0 * a.osz + a.ofz) * a.OCs;
    const bool interior = ox0 + a.TX <= a.OX && oy0 + a.TY <= a.OY && oz0 + a.TZ <= a.OZ;
    if (fwdstat && !have_piv) {   // block-uniform: the first tile of this block
      if (wave == 0 && g == 0) {
#pragma unroll
        for (int n = 0; n < NSUB; ++n) pivl[n * 16 + r16] = acc[0][n][0] + bias_v[n];
      }
      lds_barrier();
#pragma unroll
      for (int n = 0; n < NSUB; ++n) pv[n] = pivl[n * 16 + r16];
      have_piv = true;
    }
#pragma unroll
    for (int j = 0; j < MPW; ++j) {
      const int m = wave + 4 * j;
      if (m < nmsub) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = m * 16 + g * 4 + r;
          const int ro = rowoff[i];
          bool ok = ro >= 0;
          if (ok && !interior) {
            const int pk = rowpk[i];
            ok = ox0 + (pk >> 20) < a.OX && oy0 + ((pk >> 10) & 1023) < a.OY &&
                 oz0 + (pk & 1023) < a.OZ;
          }
          if (ok) {
            float *vp = tp + ro;
            cnt += 1.f;
#pragma unroll
            for (int n = 0; n < NSUB; ++n) {
              if (coff[n] < 0) continue;
              float val = acc[j][n][r] + bias_v[n];
              if (a.bn_y && !split) {   // fused BatchNorm+ReLU backward (val = dA -> dz)
                const int cc = coff[n] % a.OCs;
                const float yv = a.bn_y[(vp - dst) + coff[n]];
                val = fmaf(yv, a.bn_scale[cc], a.bn_shift[cc]) > 0.f ? val : 0.f;
                vp[coff[n]] = val;
                if (cst[n]) {
                  s1[n] += val;
                  s2[n] = fmaf(val, (yv - a.bn_mean[cc]) * a.bn_invstd[cc], s2[n]);
                }
                continue;
              }
              vp[coff[n]] = val;
              if (cst[n]) {
                const float d = val - pv[n];
                s1[n] += d;
                s2[n] = fmaf(d, d, s2[n]);
              }
            }
            if (zpad) {   // ConvTranspose3d phases: zero the padded channels of U
#pragma unroll
              for (int n = 0; n < NSUB; ++n) {
                const int nn = n0 + n * 16 + r16;
                if (coff[n] >= 0 && nn % a.Cout == a.Cout - 1)
                  for (int cz = 1; cz <= a.OCs - a.Cout; ++cz) vp[coff[n] + cz] = 0.f;
              }
            }
          }
        }
      }
    }
  };

  // Epilogue through LDS: the accumulator tile is written to LDS (reusing the
  // halo image) and stored back as float4 runs of 4 channels with bias, so
  // every store instruction writes whole 16-byte channel groups.  Thread tid
  // always owns channel group c4 = tid % nc4 (256 % nc4 == 0).
  const int NTP = NT + 4;
  const int nc4 = a.nc4;
  const int ec4 = tid % max(nc4, 1);
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.epi_lds && !split && a.bias) {
    const int cc = n0 + ec4 * 4;
    bias4.x = cc + 0 < a.Cout ? a.bias[cc + 0] : 0.f;
    bias4.y = cc + 1 < a.Cout ? a.bias[cc + 1] : 0.f;
    bias4.z = cc + 2 < a.Cout ? a.bias[cc + 2] : 0.f;
    bias4.w = cc + 3 < a.Cout ? a.bias[cc + 3] : 0.f;
  }
  float4 st1 = make_float4(0.f, 0.f, 0.f, 0.f), st2 = st1, piv4 = st1;
  float4 bsc = st1, bsh = st1, bmu = st1, bis = st1;
  if (a.bn_y && a.epi_lds) {
    const int cc = n0 + ec4 * 4;
    bsc = *reinterpret_cast<const float4 *>(a.bn_scale + cc);
    bsh = *reinterpret_cast<const float4 *>(a.bn_shift + cc);
    bmu = *reinterpret_cast<const float4 *>(a.bn_mean + cc);
    bis = *reinterpret_cast<const float4 *>(a.bn_invstd + cc);
  }
  auto epilogue_lds = [&](int b, int ox0, int oy0, int oz0) {
    lds_barrier();  // every wave is done reading the halo image
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
    lds_barrier();
    float *tp = dst + ((((size_t)b * a.SX + ox0 * a.osx + a.ofx) * a.SY + oy0 * a.osy + a.ofy) *
                           a.SZ + oz0 * a.osz + a.ofz) * a.OCs + n0 + ec4 * 4;
    const bool interior = ox0 + a.TX <= a.OX && oy0 + a.TY <= a.OY && oz0 + a.TZ <= a.OZ;
    const int vstep = 256 / nc4;
    if (fwdstat && !have_piv) {   // pivot: the block's first output voxel (row 0, always valid)
      piv4 = *reinterpret_cast<const float4 *>(smem + ec4 * 4);
      piv4.x += bias4.x;
      piv4.y += bias4.y;
      piv4.z += bias4.z;
      piv4.w += bias4.w;
      have_piv = true;
    }
    for (int i = tid / nc4; i < MT; i += vstep) {
      bool ok = true;
      if (!interior) {
        const int pk = rowpk[i];
        ok = ox0 + (pk >> 20) < a.OX && oy0 + ((pk >> 10) & 1023) < a.OY && oz0 + (pk & 1023) < a.OZ;
      }
      if (ok) {
        float4 v = *reinterpret_cast<const float4 *>(smem + i * NTP + ec4 * 4);
        v.x += bias4.x;
        v.y += bias4.y;
        v.z += bias4.z;
        v.w += bias4.w;
        if (a.bn_y && !split) {   // fused BatchNorm+ReLU backward: v = dA -> dz, stats (dz, dz*xhat)
          const float4 yv = *reinterpret_cast<const float4 *>(a.bn_y + ((tp - a.out) + rowoff[i]));
          v.x = fmaf(yv.x, bsc.x, bsh.x) > 0.f ? v.x : 0.f;
          v.y = fmaf(yv.y, bsc.y, bsh.y) > 0.f ? v.y : 0.f;
          v.z = fmaf(yv.z, bsc.z, bsh.z) > 0.f ? v.z : 0.f;
          v.w = fmaf(yv.w, bsc.w, bsh.w) > 0.f ? v.w : 0.f;
          *reinterpret_cast<float4 *>(tp + rowoff[i]) = v;
          st1.x += v.x; st1.y += v.y; st1.z += v.z; st1.w += v.w;
          st2.x = fmaf(v.x, (yv.x - bmu.x) * bis.x, st2.x);
          st2.y = fmaf(v.y, (yv.y - bmu.y) * bis.y, st2.y);
          st2.z = fmaf(v.z, (yv.z - bmu.z) * bis.z, st2.z);
          st2.w = fmaf(v.w, (yv.w - bmu.w) * bis.w, st2.w);
          continue;
        }
        *reinterpret_cast<float4 *>(tp + rowoff[i]) = v;
        const float4 d = make_float4(v.x - piv4.x, v.y - piv4.y, v.z - piv4.z, v.w - piv4.w);
        st1.x += d.x; st1.y += d.y; st1.z += d.z; st1.w += d.w;
        st2.x = fmaf(d.x, d.x, st2.x);
        st2.y = fmaf(d.y, d.y, st2.y);
        st2.z = fmaf(d.z, d.z, st2.z);
        st2.w = fmaf(d.w, d.w, st2.w);
        cnt += 1.f;
      }
    }
  };
  auto finish_tile = [&](int b, int ox0, int oy0, int oz0) {
    if (a.epi_lds) epilogue_lds(b, ox0, oy0, oz0);
    else epilogue(b, ox0, oy0, oz0);
  };

  if (NPF > 0 && ce - cb == 1) {
    // ---- single channel chunk: weights staged once, next tile's halo in flight.
    // Thread tid always handles channel group c4 = tid % C4 of halo voxels
    // v = tid / C4 + u * (256 / C4); their halo coordinates are fixed per launch.
    constexpr int VS = 256 / C4;
    stage_w(cb);
    const int ci0 = cb * CK;
    const int c4 = tid % C4, c = ci0 + c4 * 4;
    float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool act = a.in_scale != nullptr;
    if (act) {
      sc = *reinterpret_cast<const float4 *>(a.in_scale + c);
      sh = *reinterpret_cast<const float4 *>(a.in_shift + c);
    }
    int hpk[NPF > 0 ? NPF : 1], goff[NPF > 0 ? NPF : 1];
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int v = tid / C4 + u * VS;
      hpk[u] = -1;
      goff[u] = 0;
      if (v < HV) {
        int t2, hz, hx, hy;
        a.fHZ.divmod(v, t2, hz);
        a.fHY.divmod(t2, hx, hy);
        hpk[u] = (hx << 20) | (hy << 10) | hz;
        goff[u] = ((hx * a.IY + hy) * a.IZ + hz) * a.ICs;
      }
    }
    const int dst0 = (tid / C4) * CKP + c4 * 4;
    float4 pf[NPF > 0 ? NPF : 1];
    auto load_tile = [&](int tile) {
      int b, x0, y0, z0;
      tile_origin(tile, b, x0, y0, z0);
      const int gx0 = x0 * a.sx - a.px, gy0 = y0 * a.sy - a.py, gz0 = z0 * a.sz - a.pz;
      const int64_t base = ((((int64_t)b * a.IX + gx0) * a.IY + gy0) * a.IZ + gz0) * a.ICs + c;
      const bool inb = gx0 >= 0 && gy0 >= 0 && gz0 >= 0 && gx0 + a.HX <= a.IX &&
                       gy0 + a.HY <= a.IY && gz0 + a.HZ <= a.IZ;
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        const int hp = hpk[u];
        if (hp >= 0) {
          const int gx = gx0 + (hp >> 20), gy = gy0 + ((hp >> 10) & 1023), gz = gz0 + (hp & 1023);
          if (inb || ((unsigned)gx < (unsigned)a.IX && (unsigned)gy < (unsigned)a.IY &&
                      (unsigned)gz < (unsigned)a.IZ)) {
            val = *reinterpret_cast<const float4 *>(a.in + base + goff[u]);
            if (act) {
              val.x = fmaxf(fmaf(val.x, sc.x, sh.x), 0.f);
              val.y = fmaxf(fmaf(val.y, sc.y, sh.y), 0.f);
              val.z = fmaxf(fmaf(val.z, sc.z, sh.z), 0.f);
              val.w = fmaxf(fmaf(val.w, sc.w, sh.w), 0.f);
            }
          }
        }
        pf[u] = val;
      }
    };
    // contiguous tile range per block (consecutive tiles share halo rows in L2)
    const int tpb_ = (total + (int)gridDim.x - 1) / (int)gridDim.x;
    const int t_end = min(total, (int)blockIdx.x * tpb_ + tpb_);
    int tile = blockIdx.x * tpb_;
    if (tile < t_end) load_tile(tile);
    for (; tile < t_end; ++tile) {
      int b, ox0, oy0, oz0;
      tile_origin(tile, b, ox0, oy0, oz0);
      lds_barrier();
#pragma unroll
      for (int u = 0; u < NPF; ++u)
        if (hpk[u] >= 0) *reinterpret_cast<float4 *>(alds + dst0 + u * VS * CKP) = pf[u];
      lds_barrier();
      if (tile + 1 < t_end) load_tile(tile + 1);
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) acc[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      compute();
      finish_tile(b, ox0, oy0, oz0);
    }
  } else {
    const int tpb_ = (total + (int)gridDim.x - 1) / (int)gridDim.x;
    const int t_end = min(total, (int)blockIdx.x * tpb_ + tpb_);
    for (int tile = blockIdx.x * tpb_; tile < t_end; ++tile) {
      int b, ox0, oy0, oz0;
      tile_origin(tile, b, ox0, oy0, oz0);
      const int gx0 = ox0 * a.sx - a.px, gy0 = oy0 * a.sy - a.py, gz0 = oz0 * a.sz - a.pz;
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) acc[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int chunk = cb; chunk < ce; ++chunk) {
        const int ci0 = chunk * CK;
        lds_barrier();
        for (int base = tid; base < nel; base += 4 * 256) {
          float4 val[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int idx = base + u * 256;
            val[u] = idx < nel ? halo_elem(idx, b, gx0, gy0, gz0, ci0) : make_float4(0.f, 0.f, 0.f, 0.f);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int idx = base + u * 256;
            if (idx < nel) *reinterpret_cast<float4 *>(alds + halo_dst(idx)) = val[u];
          }
        }
        stage_w(chunk);
        lds_barrier();
        compute();
      }
      finish_tile(b, ox0, oy0, oz0);
    }
  }

  if (a.stats && !split && a.epi_lds) {
    // fixed-order combine of the threads that share a channel group (they
    // share the pivot too, so their pivoted sums add)
    lds_barrier();
    float *red = smem;  // [256][16]: st1[4], st2[4], cnt, -, -, -, pivot[4]
    red[tid * 16 + 0] = st1.x; red[tid * 16 + 1] = st1.y; red[tid * 16 + 2] = st1.z; red[tid * 16 + 3] = st1.w;
    red[tid * 16 + 4] = st2.x; red[tid * 16 + 5] = st2.y; red[tid * 16 + 6] = st2.z; red[tid * 16 + 7] = st2.w;
    red[tid * 16 + 8] = cnt;
    red[tid * 16 + 12] = piv4.x; red[tid * 16 + 13] = piv4.y; red[tid * 16 + 14] = piv4.z; red[tid * 16 + 15] = piv4.w;
    lds_barrier();
    if (tid < nc4 * 4) {
      const int c4 = tid >> 2, comp = tid & 3;
      float t1 = 0.f, t2 = 0.f, tn = 0.f;
      for (int k = c4; k < 256; k += nc4) {
        t1 += red[k * 16 + comp];
        t2 += red[k * 16 + 4 + comp];
        tn += red[k * 16 + 8];
      }
      const size_t row = blockIdx.x;
      if (fwdstat) {
        // thread c4 (< nc4) owns channel group c4: its pivot is this channel's
        const float pk = red[c4 * 16 + 12 + comp];
        *reinterpret_cast<float4 *>(a.stats + (row * a.CoutW + n0 + tid) * 4) =
            make_float4(t1, t2, pk, tn);
      } else {
        a.stats[(row * a.CoutW + n0 + tid) * 2 + 0] = t1;
        a.stats[(row * a.CoutW + n0 + tid) * 2 + 1] = t2;
      }
    }
  } else if (a.stats && !split) {
#pragma unroll
    for (int n = 0; n < NSUB; ++n) {
      s1[n] += __shfl_xor(s1[n], 16);
      s1[n] += __shfl_xor(s1[n], 32);
      s2[n] += __shfl_xor(s2[n], 16);
      s2[n] += __shfl_xor(s2[n], 32);
    }
    cnt += __shfl_xor(cnt, 16);
    cnt += __shfl_xor(cnt, 32);
    lds_barrier();
    float *red = smem;  // [4][NT][3]
    if (lane < 16) {
#pragma unroll
      for (int n = 0; n < NSUB; ++n) {
        red[(wave * NT + n * 16 + lane) * 3 + 0] = s1[n];
        red[(wave * NT + n * 16 + lane) * 3 + 1] = s2[n];
        red[(wave * NT + n * 16 + lane) * 3 + 2] = cnt;
      }
    }
    lds_barrier();
    if (tid < NT) {
      float t1 = 0.f, t2 = 0.f, tn = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        t1 += red[(w * NT + tid) * 3 + 0];
        t2 += red[(w * NT + tid) * 3 + 1];
        tn += red[(w * NT + tid) * 3 + 2];
      }
      const size_t row = blockIdx.x;
      if (fwdstat) {
        *reinterpret_cast<float4 *>(a.stats + (row * a.CoutW + n0 + tid) * 4) =
            make_float4(t1, t2, pivl[tid], tn);
      } else {
        a.stats[(row * a.CoutW + n0 + tid) * 2 + 0] = t1;
        a.stats[(row * a.CoutW + n0 + tid) * 2 + 1] = t2;
      }
    }
  }
}

// Sum of the K-split partial slices in a fixed order, + bias, store, and the
// BatchNorm partial statistics of each block's rows (one stats row per block).
// Every element of the stored tensor [B][SX][SY][SZ][OCs] is produced by
// exactly one (voxel, channel) of the GEMM, so the slices are fully written.
// Requires 256 % (OCs/4) == 0 (plan_conv2 only splits such layers).
__global__ void __launch_bounds__(256) conv2_reduce_kernel(const GConvArgs a, int vox_per_block) {
  __shared__ float red[256][3];
  const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
  const int C4 = a.OCs / 4;
  const int tid = threadIdx.x;
  const int c4 = tid % C4;
  const int vstep = 256 / C4;
  const int64_t v0 = (int64_t)blockIdx.x * vox_per_block;
  const int64_t v1 = min(v0 + vox_per_block, nvox);
  float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.bias) {
    const int c = c4 * 4;
    bv.x = c + 0 < a.Cout ? a.bias[c + 0] : 0.f;
    bv.y = c + 1 < a.Cout ? a.bias[c + 1] : 0.f;
    bv.z = c + 2 < a.Cout ? a.bias[c + 2] : 0.f;
    bv.w = c + 3 < a.Cout ? a.bias[c + 3] : 0.f;
  }
  float st1[4] = {0.f, 0.f, 0.f, 0.f}, st2[4] = {0.f, 0.f, 0.f, 0.f};
  auto vsum = [&](int64_t v) {
    const size_t off = (size_t)v * a.OCs + c4 * 4;
    float4 s = *reinterpret_cast<const float4 *>(a.partial + off);
    for (int k = 1; k < a.ksplit; ++k) {
      const float4 p = *reinterpret_cast<const float4 *>(a.partial + (size_t)k * a.slice_floats + off);
      s.x += p.x;
      s.y += p.y;
      s.z += p.z;
      s.w += p.w;
    }
    s.x += bv.x;
    s.y += bv.y;
    s.z += bv.z;
    s.w += bv.w;
    return s;
  };
  // forward statistics about the block's first voxel (every thread of a
  // channel group computes the same pivot; StatRow in common.h)
  const bool fwdstat = a.stats && !a.bn_y;
  const float4 piv = fwdstat ? vsum(v0) : make_float4(0.f, 0.f, 0.f, 0.f);
  float cnt = 0.f;
  for (int64_t v = v0 + tid / C4; v < v1; v += vstep) {
    const size_t off = (size_t)v * a.OCs + c4 * 4;
    float4 s = vsum(v);
    if (a.bn_y) {   // fused BatchNorm+ReLU backward: s = dA -> dz, stats (dz, dz*xhat)
      const int c = c4 * 4;
      const float4 yv = *reinterpret_cast<const float4 *>(a.bn_y + off);
      const float4 sc = *reinterpret_cast<const float4 *>(a.bn_scale + c);
      const float4 sh = *reinterpret_cast<const float4 *>(a.bn_shift + c);
      const float4 mu = *reinterpret_cast<const float4 *>(a.bn_mean + c);
      const float4 is = *reinterpret_cast<const float4 *>(a.bn_invstd + c);
      s.x = fmaf(yv.x, sc.x, sh.x) > 0.f ? s.x : 0.f;
      s.y = fmaf(yv.y, sc.y, sh.y) > 0.f ? s.y : 0.f;
      s.z = fmaf(yv.z, sc.z, sh.z) > 0.f ? s.z : 0.f;
      s.w = fmaf(yv.w, sc.w, sh.w) > 0.f ? s.w : 0.f;
      *reinterpret_cast<float4 *>(a.out + off) = s;
      st1[0] += s.x; st1[1] += s.y; st1[2] += s.z; st1[3] += s.w;
      st2[0] = fmaf(s.x, (yv.x - mu.x) * is.x, st2[0]);
      st2[1] = fmaf(s.y, (yv.y - mu.y) * is.y, st2[1]);
      st2[2] = fmaf(s.z, (yv.z - mu.z) * is.z, st2[2]);
      st2[3] = fmaf(s.w, (yv.w - mu.w) * is.w, st2[3]);
      continue;
    }
    *reinterpret_cast<float4 *>(a.out + off) = s;
    const float d[4] = {s.x - piv.x, s.y - piv.y, s.z - piv.z, s.w - piv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      st1[j] += d[j];
      st2[j] = fmaf(d[j], d[j], st2[j]);
    }
    cnt += 1.f;
  }
  if (!a.stats) return;
  const float pk[4] = {piv.x, piv.y, piv.z, piv.w};
  for (int comp = 0; comp < 4; ++comp) {
    lds_barrier();
    red[tid][0] = st1[comp];
    red[tid][1] = st2[comp];
    red[tid][2] = cnt;
    lds_barrier();
    if (tid < C4) {
      float t1 = 0.f, t2 = 0.f, tn = 0.f;
      for (int k = tid; k < 256; k += C4) {
        t1 += red[k][0];
        t2 += red[k][1];
        tn += red[k][2];
      }
      const int c = tid * 4 + comp;
      if (fwdstat) {
        *reinterpret_cast<float4 *>(a.stats + ((size_t)blockIdx.x * a.CoutW + c) * 4) =
            make_float4(t1, t2, pk[comp], tn);
      } else {
        a.stats[((size_t)blockIdx.x * a.CoutW + c) * 2 + 0] = t1;
        a.stats[((size_t)blockIdx.x * a.CoutW + c) * 2 + 1] = t2;
      }
    }
  }
}

// ---------------------------------------------------------------------------
bool conv2_disabled() {
  static const bool off = [] {
    const char *e = getenv("HCU_NO_CONV2");
    return e && e[0] == '1';
  }();
  return off;
}

static void tile2(int OX, int OY, int TZ, int maxM, int &TX, int &TY) {
  const int txy = std::max(1, maxM / TZ);
  TX = 1;
  while ((TX + 1) * (TX + 1) <= txy) ++TX;
  TY = std::max(1, txy / TX);
  if (TX > OX) { TX = OX; TY = std::max(1, std::min(OY, txy / TX)); }
  if (TY > OY) { TY = OY; TX = std::max(1, std::min(OX, txy / TY)); }
}

static long conv2_areg(const GConvArgs &a, int CK, int NT) {
  const long HV = (long)a.HX * a.HY * a.HZ;
  const long ctile = (long)a.MPW * 64 * (NT + 4);   // LDS epilogue tile
  return (std::max(HV * (CK + 4), ctile) + 3) & ~3L;
}

static long conv2_lds(const GConvArgs &a, int CK, int NT) {
  const int T = a.KX * a.KY * a.KZ;
  const int TPS = 16 / CK;
  const int S = (T + TPS - 1) / TPS;
  return std::max(conv2_areg(a, CK, NT) + (long)S * 4 * NT * 4 + S * 4 + (long)a.MPW * 128 + NT,
                  256L * 16) * 4;
}

// Chooses CK / NSUB / MPW / tile / K split / prefetch depth / grid for
// conv2_kernel.  Returns 0, or a non-zero code when conv2 cannot run this
// shape (the caller then keeps gconv).
static int env_int(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}

int plan_conv2(GConvArgs &a, int target_blocks) {
  // debug: HCU_CONV2_SEL=k keeps the MPW target only for the k-th plan since
  // the variable last changed (A/B bisection of one layer's tiling)
  static int ncall = 0, last_sel = -1;
  const int sel = env_int("HCU_CONV2_SEL", -1);
  if (sel != last_sel) { ncall = 0; last_sel = sel; }
  const int call = ncall++;
  int mpw_target = env_int("HCU_CONV2_MPW_TARGET", 256);
  const int ks_target = env_int("HCU_CONV2_KS_TARGET", 256);
  if (sel >= 0 && sel != call) mpw_target = 1024;
  if (a.OX <= 0 || a.OY <= 0 || a.OZ <= 0) return fail(2, "conv2: empty output grid");
  if (a.ICs % 4 != 0 || a.OCs % 4 != 0) return fail(1, "conv2: channel strides must be multiples of 4");
  if (a.nph < 1) a.nph = 1;
  if (a.phx < 1) a.phx = 1;
  if (a.phy < 1) a.phy = 1;
  if (a.phz < 1) a.phz = 1;
  const int Nlog = a.Cout * a.nph;
  const int nb16 = cdiv(Nlog, 16);
  a.NSUB = nb16 >= 3 ? 4 : nb16;
  const int NT = a.NSUB * 16;
  a.CoutW = round_up(Nlog, NT);
  const int ntz = cdiv(a.OZ, 16);
  a.TZ = cdiv(a.OZ, ntz);
  const int nN = a.CoutW / NT;
  // MPW: largest tile that still gives enough tiles to fill the chip and whose
  // halo + epilogue images fit the LDS budget with some channel chunk CK
  const int mpws[3] = {4, 2, 1};
  bool enough = false;
  a.CK = 0;
  for (int mi = 0; mi < 3 && !(enough && a.CK); ++mi) {
    const int MPW = mpws[mi];
    int TX, TY;
    tile2(a.OX, a.OY, a.TZ, 64 * MPW, TX, TY);
    const long blocks = (long)cdiv(a.OX, TX) * cdiv(a.OY, TY) * ntz * nN * a.B;
    a.MPW = MPW;
    a.TX = TX;
    a.TY = TY;
    a.HX = (a.TX - 1) * a.sx + (a.KX - 1) * a.dx + 1;
    a.HY = (a.TY - 1) * a.sy + (a.KY - 1) * a.dy + 1;
    a.HZ = (a.TZ - 1) * a.sz + (a.KZ - 1) * a.dz + 1;
    enough = blocks >= (mpw_target ? mpw_target : target_blocks);
    a.CK = 0;
    const int cks[3] = {16, 8, 4};
    for (int i = 0; i < 3; ++i) {
      const int CK = cks[i];
      if (a.ICs % CK) continue;
      const long lds = conv2_lds(a, CK, NT);
      if (lds <= 56 * 1024) {
        a.CK = CK;
        a.lds_bytes = (int)lds;
        break;
      }
    }
  }
  a.ntx = cdiv(a.OX, a.TX);
  a.nty = cdiv(a.OY, a.TY);
  a.ntz = ntz;
  if (!a.CK) return fail(4, "conv2: no tile fits in LDS");
  if (a.lds_bytes < 4 * NT * 3 * 4) a.lds_bytes = 4 * NT * 3 * 4;
  const long tiles = (long)a.ntx * a.nty * a.ntz * a.B;
  const int nchunks = a.ICs / a.CK;
  int ks = 1;
  if (256 % (a.OCs / 4) == 0)
    while (ks < nchunks && tiles * nN * ks < (ks_target ? ks_target : target_blocks)) ks *= 2;
  ks = std::min(ks, nchunks);
  a.cps = cdiv(nchunks, ks);
  a.ksplit = cdiv(nchunks, a.cps);
  a.slice_floats = (size_t)a.B * a.SX * a.SY * a.SZ * a.OCs;
  // halo prefetch depth (float4 per thread) for single-chunk blocks
  const long nel = (long)a.HX * a.HY * a.HZ * (a.CK / 4);
  a.NPF = 0;
  if (a.cps == 1) {
    if (nel <= 4 * 256) a.NPF = 4;
    else if (nel <= 8 * 256) a.NPF = 8;
  }
  // persistent grid: up to `occ` resident blocks per CU
  const int occ = std::max(1, std::min(8, (int)(160 * 1024 / a.lds_bytes)));
  const long slots = (long)256 * occ;
  const long per_tile = (long)nN * a.ksplit;
  long gx = std::max(1L, slots / per_tile);
  a.gridx = (int)std::min(tiles, gx);
  a.fHZ = FastDiv(a.HZ);
  a.fHY = FastDiv(a.HY);
  a.fTZ = FastDiv(a.TZ);
  a.fTY = FastDiv(a.TY);
  a.fNT = FastDiv(a.ntx * a.nty * a.ntz);
  a.fNTZ = FastDiv(a.ntz);
  a.fNTY = FastDiv(a.nty);
  // LDS epilogue: plain layouts whose float4 channel groups divide 256
  a.nc4 = std::min(NT, a.OCs) / 4;
  a.epi_lds = 0;
  if (a.nph == 1 && (a.CoutW / NT == 1 || a.OCs % NT == 0) && a.nc4 > 0 && 256 % a.nc4 == 0)
    a.epi_lds = 1;
  a.areg = (int)conv2_areg(a, a.CK, NT);
  a.use_conv2 = 1;
  if (env_int("HCU_CONV2_LOG", 0))
    fprintf(stderr,
            "conv2 plan %d: B%d I%dx%dx%d ICs%d O%dx%dx%d S%dx%dx%d OCs%d Cout%d K%dx%dx%d s%d%d%d nph%d"
            " | CK%d NSUB%d MPW%d T%dx%dx%d ks%d cps%d NPF%d gridx%d epi%d\n",
            call, a.B, a.IX, a.IY, a.IZ, a.ICs, a.OX, a.OY, a.OZ, a.SX, a.SY, a.SZ, a.OCs, a.Cout,
            a.KX, a.KY, a.KZ, a.sx, a.sy, a.sz, a.nph, a.CK, a.NSUB, a.MPW, a.TX, a.TY, a.TZ,
            a.ksplit, a.cps, a.NPF, a.gridx, a.epi_lds);
  return 0;
}

size_t conv2_partial_floats(const GConvArgs &a) {
  return a.ksplit > 1 ? (size_t)a.ksplit * a.slice_floats : 0;
}

static int reduce_vox_per_block(const GConvArgs &a) { return 2 * 256 / (a.OCs / 4); }

int conv2_stat_rows(const GConvArgs &a) {
  if (a.ksplit > 1) {
    const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
    const int vpb = reduce_vox_per_block(a);
    return (int)((nvox + vpb - 1) / vpb);
  }
  return a.gridx;
}

#define CONV2_CASE(CK_, NS_, MP_, PF_)                                                         \
  if (a.CK == CK_ && a.NSUB == NS_ && a.MPW == MP_ && a.NPF == PF_) {                           \
    HCU_TIMED(s, "conv2_kernel<" #CK_ "," #NS_ "," #MP_ "," #PF_ ">", fl, by,                     \
              HCU_LAUNCH((conv2_kernel<CK_, NS_, MP_, PF_>), grid, dim3(256),           \
                                 a.lds_bytes, s, a));                                           \
    launched = true;                                                                            \
  }
#define CONV2_PF(CK_, NS_, MP_) \
  CONV2_CASE(CK_, NS_, MP_, 0) else CONV2_CASE(CK_, NS_, MP_, 4) else CONV2_CASE(CK_, NS_, MP_, 8)
#define CONV2_MP(CK_, NS_) CONV2_PF(CK_, NS_, 1) else CONV2_PF(CK_, NS_, 2) else CONV2_PF(CK_, NS_, 4)
#define CONV2_NS(CK_) CONV2_MP(CK_, 1) else CONV2_MP(CK_, 2) else CONV2_MP(CK_, 4)

int launch_conv2(const GConvArgs &a, hipStream_t s) {
  const dim3 grid(a.gridx, a.CoutW / (a.NSUB * 16), a.ksplit);
  if (grid.y > 65535 || grid.z > 65535) return fail(4, "conv2: grid too large");
  if (a.ksplit > 1 && !a.partial) return fail(5, "conv2: K split needs a partial workspace");
  const double fl = a.flops > 0 ? a.flops
                                : 2.0 * a.B * a.OX * a.OY * a.OZ * (double)a.Cout * a.nph * a.KX *
                                      a.KY * a.KZ * a.ICs;
  const double by = 4.0 * ((double)a.B * a.IX * a.IY * a.IZ * a.ICs +
                           (double)a.B * a.SX * a.SY * a.SZ * a.OCs);
  bool launched = false;
  CONV2_NS(4) else CONV2_NS(8) else CONV2_NS(16)
  if (!launched) return fail(4, "conv2: unsupported variant");
  HCU_CHECK_LAUNCH();
  if (a.ksplit > 1) {
    const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
    const int vpb = reduce_vox_per_block(a);
    const int blocks = (int)((nvox + vpb - 1) / vpb);
    HCU_TIMED(s, "conv2_reduce_kernel", 0.0, 4.0 * (double)(a.ksplit + 1) * a.slice_floats,
              HCU_LAUNCH(conv2_reduce_kernel, dim3(blocks), dim3(256), 0, s, a, vpb));
    HCU_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace hcu
