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

#ifdef HCU_BCONV_PHASES
// Per-phase cycle totals of wave 0 of every block (tools/bconv_bench only):
// [0] halo -> LDS (incl. the wait for the prefetch), [1] barrier + weights,
// [2] next-halo issue, [3] MFMA loop, [4] epilogue, [5] tiles.
__device__ unsigned long long g_bconv_phase[8];
#define PH_MARK(k)                                      \
  do {                                                  \
    const long long t__ = (long long)__builtin_readcyclecounter(); \
    ph_acc[k] += t__ - ph_t;                            \
    ph_t = t__;                                         \
  } while (0)
#else
#define PH_MARK(k) do {} while (0)
#endif

namespace {
// Halo row stride (bf16 elements).  ds_read_b128 serves a wave in 4 lane
// groups of 16 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...); with CK = 32 the
// lanes of one group read rows r of chunk g and rows r' of chunk g+1, and a
// row of 6 x 16-byte slots (CK + 16) puts all 16 on distinct bank slots for
// consecutive rows; CK = 16 uses 3 slots, CK = 8 one (rows are contiguous).
constexpr int ckp_of(int CK) { return CK == 8 ? 8 : (CK == 16 ? 24 : CK + 16); }
}

// BNB: the input-gradient epilogue fused with the BatchNorm backward (a.bn_y
// set); a template parameter so that its loads never share registers (and
// therefore waits) with the other epilogues.
template <int CK, int NSUB, int MPW, int NPF, bool BNB>
__global__ void __launch_bounds__(256) bconv_kernel(const GConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // launch constants for the tile loop, read through kuni (common.h): they are
  // live only in the phase that uses them, not for the whole kernel
  __shared__ __attribute__((aligned(16))) char sa_raw[sizeof(GConvArgs)];
  GConvArgs &sa = *reinterpret_cast<GConvArgs *>(sa_raw);
#define KA(f) kuni(sa.f)
  constexpr int NT = NSUB * 16;
  constexpr int C8 = CK / 8;           // 16-byte channel groups per chunk
  constexpr int TPS = 4 / C8;          // taps per K-step
  constexpr int CKP = ckp_of(CK);      // halo row stride (bf16 elements)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  if (tid == 0) sa = a;
  const int T = a.KX * a.KY * a.KZ;
  const int S = (T + TPS - 1) / TPS;
  const int HZ = a.HZ, HYZ = a.HY * a.HZ;
  const int HV = a.HX * HYZ;
  uint16_t *alds = reinterpret_cast<uint16_t *>(smem);            // [HV][CKP]
  uint16_t *wlds = reinterpret_cast<uint16_t *>(smem + a.areg);   // [S][4][NT][8]
  int *toffs = reinterpret_cast<int *>(wlds + S * 4 * NT * 8);    // [S][4]
  int *rowpk = toffs + S * 4;                                     // [MPW*64]
  int *rowoff = rowpk + MPW * 64;                                 // [MPW*64]
  // per-block coefficients (LDS, read in short phases): [5][NT] = bias, bn
  // scale/shift/mean/invstd per stored column; [4][NT] statistics pivots of
  // each wave; input activation [2][ICs] = scale, shift
  float *coefL = reinterpret_cast<float *>(rowoff + MPW * 64);
  float *pivL = coefL + 5 * NT;
  float *actL = pivL + 4 * NT;

  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int n0 = blockIdx.y * NT;
  const int MT = a.TX * a.TY * a.TZ;
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
  // first stored channel of the block (ConvTranspose3d phases: all NT columns
  // of a block belong to one phase, the planner requires Cout % NT == 0)
  const int co0 = a.nph > 1 ? n0 - (n0 / a.Cout) * a.Cout : n0;
  for (int j = tid; j < NT; j += 256) {
    const int c = co0 + j;
    coefL[j] = (!split && a.bias && c < a.Cout) ? a.bias[c] : 0.f;
    const bool bn = a.bn_y && !split && c < a.OCs;
    coefL[NT + j] = bn ? a.bn_scale[c] : 0.f;
    coefL[2 * NT + j] = bn ? a.bn_shift[c] : 0.f;
    coefL[3 * NT + j] = bn ? a.bn_mean[c] : 0.f;
    coefL[4 * NT + j] = bn ? a.bn_invstd[c] : 0.f;
  }
  if (a.in_scale)
    for (int c = tid; c < a.ICs; c += 256) {
      actL[c] = a.in_scale[c];
      actL[a.ICs + c] = a.in_shift[c];
    }

  auto tile_origin = [&](int tile, int &b, int &ox0, int &oy0, int &oz0) {
    int r, tzi, tyi, txi;
    sa.fNT.uni().divmod(tile, b, r);
    sa.fNTZ.uni().divmod(r, r, tzi);
    sa.fNTY.uni().divmod(r, txi, tyi);
    ox0 = txi * KA(TX);
    oy0 = tyi * KA(TY);
    oz0 = tzi * KA(TZ);
  };
  auto stage_w = [&](int chunk) {
    const int n16 = S * 4 * NT;
    const uint4 *src = reinterpret_cast<const uint4 *>(KA(w));
    const int CoutW = KA(CoutW);
    for (int idx = tid; idx < n16; idx += 256) {
      const int n = idx % NT, sg = idx / NT;
      reinterpret_cast<uint4 *>(wlds)[sg * NT + n] =
          src[((size_t)chunk * S * 4 + sg) * CoutW + blockIdx.y * NT + n];
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
  const bool act = a.in_scale != nullptr;
  uint4 pf[NPFR];
  uint32_t okbits = 0;
  // halo of (tile, chunk) -> pf (branch-free: the validity of each element is
  // a mask, invalid elements read offset 0x7ffffff0, outside the buffer -> 0)
  auto fetch = [&](int tile, int chunk) {
    int b, x0, y0, z0;
    tile_origin(tile, b, x0, y0, z0);
    const int IX = KA(IX), IY = KA(IY), IZ = KA(IZ), ICs = KA(ICs);
    const uint32_t bZ = (uint32_t)ICs * 2, bY = (uint32_t)IZ * bZ, bX = (uint32_t)IY * bY;
    const int gx0 = x0 * KA(sx) - KA(px), gy0 = y0 * KA(sy) - KA(py), gz0 = z0 * KA(sz) - KA(pz);
    const uint16_t *bp = reinterpret_cast<const uint16_t *>(KA(in)) + (size_t)b * IX * bX / 2;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, IX * (int)bX, 0x00020000);
    const int base_off = gx0 * (int)bX + gy0 * (int)bY + gz0 * (int)bZ + (chunk * CK + c8 * 8) * 2;
    okbits = 0;
#pragma unroll
    for (int u = 0; u < NPFR; ++u) {
      const int hp = hpk[u];
      const int hx = hp >> 20, hy = (hp >> 10) & 1023, hz = hp & 1023;
      const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
      const bool ok = (hp >= 0) & ((unsigned)gx < (unsigned)IX) & ((unsigned)gy < (unsigned)IY) &
                      ((unsigned)gz < (unsigned)IZ);
      const int off = ok ? base_off + (int)(__umul24(hx, bX) + __umul24(hy, bY) + __umul24(hz, bZ))
                         : 0x7ffffff0;
      pf[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      okbits |= (uint32_t)ok << u;
    }
  };
  // BatchNorm+ReLU of 8 channels: fp32 fused multiply-add (v_pk_fma_f32),
  // rounded to bf16, ReLU on the packed bf16 (v_pk_max_i16: a bf16 is negative
  // exactly when its int16 image is); 0 outside the input
  auto activate = [&](uint4 v, bool ok, int chunk) -> uint4 {
    if (!ok) return make_uint4(0u, 0u, 0u, 0u);
    if (!act) return v;
    const int c = chunk * CK + c8 * 8;
    const int ICs = KA(ICs);
    const floatx4 s0 = *reinterpret_cast<const floatx4 *>(actL + c);
    const floatx4 s1 = *reinterpret_cast<const floatx4 *>(actL + c + 4);
    const floatx4 h0 = *reinterpret_cast<const floatx4 *>(actL + ICs + c);
    const floatx4 h1 = *reinterpret_cast<const floatx4 *>(actL + ICs + c + 4);
    uint4 o;
    o.x = bn_relu_bf2(v.x, s0.xy, h0.xy);
    o.y = bn_relu_bf2(v.y, s0.zw, h0.zw);
    o.z = bn_relu_bf2(v.z, s1.xy, h1.xy);
    o.w = bn_relu_bf2(v.w, s1.zw, h1.zw);
    return o;
  };
  // direct (non-prefetched) staging of one (tile, chunk) halo
  auto stage_direct = [&](int tile, int chunk) {
    int b, x0, y0, z0;
    tile_origin(tile, b, x0, y0, z0);
    const int gx0 = x0 * a.sx - a.px, gy0 = y0 * a.sy - a.py, gz0 = z0 * a.sz - a.pz;
    const uint32_t bZ = (uint32_t)a.ICs * 2, bY = (uint32_t)a.IZ * bZ, bX = (uint32_t)a.IY * bY;
    const uint16_t *bp = reinterpret_cast<const uint16_t *>(a.in) + (size_t)b * a.IX * a.IY * a.IZ * a.ICs;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, a.IX * (int)bX, 0x00020000);
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

  // Accumulators hold the transposed tile: the MFMA is issued with the weights
  // as A and the activations as B, so acc[j][n][r] = out[voxel (wave+4j)*16 +
  // r16][column n*16 + 4g + r] and every lane owns 4 consecutive channels of
  // one voxel -> 8-byte stores straight from the accumulators, no LDS round trip.
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
        acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[n], afr[j], acc[j][n], 0, 0, 0);
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

  // ---- epilogue: straight from the accumulators.  Every lane issues exactly
  // MPW * NSUB stores (and, for the fused BatchNorm backward, as many loads)
  // per tile, invalid ones at an offset outside the buffer (dropped), so the
  // wait for the next halo can count its loads exactly.
  const bool fwdstat = a.stats && !BNB && !split;
  float st1[NSUB][4], st2[NSUB][4], cnt = 0.f;
#pragma unroll
  for (int n = 0; n < NSUB; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) st1[n][r] = st2[n][r] = 0.f;
  auto epilogue = [&](int b, int ox0, int oy0, int oz0, bool first) {
    int qx = 0, qy = 0, qz = 0;
    if (KA(nph) > 1) {
      const int ph = blockIdx.y * NT / KA(Cout), phz = KA(phz), phy = KA(phy);
      qz = ph % phz;
      qy = (ph / phz) % phy;
      qx = ph / (phz * phy);
    }
    const int OX = KA(OX), OY = KA(OY), OZ = KA(OZ), OCs = KA(OCs);
    const bool interior = ox0 + KA(TX) <= OX && oy0 + KA(TY) <= OY && oz0 + KA(TZ) <= OZ;
    const int sample = KA(SX) * KA(SY) * KA(SZ) * OCs;
    const int tb = (((ox0 * KA(osx) + KA(ofx) + qx) * KA(SY) + oy0 * KA(osy) + KA(ofy) + qy) * KA(SZ) +
                    oz0 * KA(osz) + KA(ofz) + qz) * OCs + co0;
    const size_t sb = (size_t)b * sample;
    const int es = split ? 4 : 2;
    void *obase = split ? (void *)(KA(partial) + (size_t)blockIdx.z * KA(slice_floats) + sb)
                        : (void *)(reinterpret_cast<uint16_t *>(KA(out)) + sb);
    const __amdgpu_buffer_rsrc_t ors =
        __builtin_amdgcn_make_buffer_rsrc(obase, 0, sample * es, 0x00020000);
    const uint16_t *ybf = reinterpret_cast<const uint16_t *>(KA(bn_y));
    constexpr bool bnb = BNB;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        bnb ? (void *)(ybf + sb) : obase, 0, bnb ? sample * 2 : 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < MPW; ++j) {
      const int i = (wave + 4 * j) * 16 + r16;
      const int ro = rowoff[i];
      bool vok = ro >= 0;
      if (!interior) {
        const int pk = rowpk[i];
        vok = vok & (ox0 + (pk >> 20) < OX) & (oy0 + ((pk >> 10) & 1023) < OY) &
              (oz0 + (pk & 1023) < OZ);
      }
      const int rof = tb + ro;
      u32x2 yv[NSUB];
      if (bnb)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) {
          const int col = n * 16 + g * 4;
          const bool ok = vok & (co0 + col < OCs);
          yv[n] = __builtin_bit_cast(
              u32x2, __builtin_amdgcn_raw_buffer_load_b64(yrs, ok ? (rof + col) * 2 : 0x3ffffff0, 0, 0));
        }
      if (fwdstat && first && j == 0) {
        // statistics pivot of this wave: its first voxel (+ bias), or the bias
        // when that voxel lies outside the output
        const int src = lane & 48;
        const bool pok = __shfl(vok ? 1 : 0, src) != 0;
#pragma unroll
        for (int n = 0; n < NSUB; ++n) {
          const floatx4 bias = *reinterpret_cast<const floatx4 *>(coefL + n * 16 + g * 4);
          floatx4 p;
#pragma unroll
          for (int r = 0; r < 4; ++r) p[r] = bias[r] + (pok ? __shfl(acc[0][n][r], src) : 0.f);
          if (r16 == 0) *reinterpret_cast<floatx4 *>(pivL + wave * NT + n * 16 + g * 4) = p;
        }
      }
      if (vok) cnt += 1.f;
#pragma unroll
      for (int n = 0; n < NSUB; ++n) {
        const int col = n * 16 + g * 4;
        const bool ok = vok & (co0 + col < OCs);
        const int off = ok ? rof + col : 0x1fffffff;
        floatx4 v = acc[j][n];
        if (split) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ors, off * 4, 0, 0);
          continue;
        }
        v += *reinterpret_cast<const floatx4 *>(coefL + col);
        if (bnb) {   // fused BatchNorm+ReLU backward: v = dA -> dz; (dz, dz*xhat)
          const u32x2 yw = yv[n];
          const float y[4] = {bf_lo(yw.x), bf_hi(yw.x), bf_lo(yw.y), bf_hi(yw.y)};
          const floatx4 bsc = *reinterpret_cast<const floatx4 *>(coefL + NT + col);
          const floatx4 bsh = *reinterpret_cast<const floatx4 *>(coefL + 2 * NT + col);
          const floatx4 bmu = *reinterpret_cast<const floatx4 *>(coefL + 3 * NT + col);
          const floatx4 bis = *reinterpret_cast<const floatx4 *>(coefL + 4 * NT + col);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = (ok && fmaf(y[r], bsc[r], bsh[r]) > 0.f) ? v[r] : 0.f;
            st1[n][r] += v[r];
            st2[n][r] = fmaf(v[r], (y[r] - bmu[r]) * bis[r], st2[n][r]);
          }
        } else if (fwdstat) {
          const floatx4 piv = *reinterpret_cast<const floatx4 *>(pivL + wave * NT + col);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = ok ? v[r] - piv[r] : 0.f;
            st1[n][r] += d;
            st2[n][r] = fmaf(d, d, st2[n][r]);
          }
        }
        const u32x2 pk2 = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
        __builtin_amdgcn_raw_buffer_store_b64(pk2, ors, off * 2, 0, 0);
      }
    }
  };

  // The epilogue issues MPW*NSUB stores after the next halo's loads.  So that
  // every path into a halo wait has at least as many younger stores (first
  // tile, further channel chunks), as many stores to an empty buffer (dropped)
  // follow every fetch; the compiler's vmcnt for each prefetched element then
  // does not include the epilogue's stores.
  auto dummy_epilogue = [&]() {
    const __amdgpu_buffer_rsrc_t zr = __builtin_amdgcn_make_buffer_rsrc((void *)a.in, 0, 0, 0x00020000);
    const u32x2 z = {0u, 0u};
#pragma unroll
    for (int k = 0; k < MPW * NSUB; ++k) __builtin_amdgcn_raw_buffer_store_b64(z, zr, 32 * k, 0, 0);
  };

  lds_barrier();   // sa, tables and coefficients are in LDS
  // ---- main loop over (tile, chunk) items; contiguous tile range per block:
  // consecutive tiles share halo rows, which then come from this CU's L2
  const int tpb_ = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t_beg = blockIdx.x * tpb_, t_end = min(total, t_beg + tpb_);
#ifdef HCU_BCONV_PHASES
  long long ph_acc[6] = {0, 0, 0, 0, 0, 0};
  long long ph_t = (long long)__builtin_readcyclecounter();
#endif
  bool first = true;
  if (NPF > 0) {
    int tile = t_beg;
    if (nck == 1) stage_w(cb);
    if (tile < t_end) fetch(tile, cb);
    dummy_epilogue();
    for (; tile < t_end; ++tile) {
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) acc[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int chunk = cb; chunk < ce; ++chunk) {
        lds_barrier();
#pragma unroll
        for (int u = 0; u < NPFR; ++u)   // every element is written (the waits stay exact)
          *reinterpret_cast<uint4 *>(alds + (hpk[u] >= 0 ? (tid / C8 + u * VS) * CKP + c8 * 8 : HV * CKP)) =
              activate(pf[u], (okbits >> u) & 1u, chunk);
        PH_MARK(0);
        if (nck > 1) stage_w(chunk);
        lds_barrier();
        PH_MARK(1);
        int nt = tile, nc = chunk + 1;
        if (nc == ce) {
          nc = cb;
          nt = tile + 1;
        }
        if (nt < t_end) fetch(nt, nc);
        PH_MARK(2);
        compute();
        PH_MARK(3);
        dummy_epilogue();   // unconditional: a branch here would be a path without it
      }
      int b, ox0, oy0, oz0;
      tile_origin(tile, b, ox0, oy0, oz0);
      epilogue(b, ox0, oy0, oz0, first);
      first = false;
      PH_MARK(4);
#ifdef HCU_BCONV_PHASES
      ph_acc[5] += 1;
#endif
    }
  } else {
    for (int tile = t_beg; tile < t_end; ++tile) {
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) acc[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int chunk = cb; chunk < ce; ++chunk) {
        lds_barrier();
        stage_direct(tile, chunk);
        PH_MARK(0);
        stage_w(chunk);
        lds_barrier();
        PH_MARK(1);
        compute();
        PH_MARK(3);
      }
      int b, ox0, oy0, oz0;
      tile_origin(tile, b, ox0, oy0, oz0);
      epilogue(b, ox0, oy0, oz0, first);
      first = false;
      PH_MARK(4);
#ifdef HCU_BCONV_PHASES
      ph_acc[5] += 1;
#endif
    }
  }
#ifdef HCU_BCONV_PHASES
  if (tid == 0)
    for (int k = 0; k < 6; ++k) atomicAdd(&g_bconv_phase[k], (unsigned long long)ph_acc[k]);
#endif

  // ---- statistics rows, one per (block, wave): fixed-order butterfly over the
  // 16 voxel lanes of each channel group, lane r16 == 0 writes
  if (!a.stats || split) return;
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) {
    cnt += __shfl_xor(cnt, m);
#pragma unroll
    for (int n = 0; n < NSUB; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        st1[n][r] += __shfl_xor(st1[n][r], m);
        st2[n][r] += __shfl_xor(st2[n][r], m);
      }
  }
  if (r16 != 0) return;
  const size_t row = (size_t)blockIdx.x * 4 + wave;
#pragma unroll
  for (int n = 0; n < NSUB; ++n) {
    const int col = n * 16 + g * 4;
    if (co0 + col >= a.OCs) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = n0 + col + r;
      if (fwdstat)
        *reinterpret_cast<float4 *>(a.stats + (row * a.CoutW + c) * 4) =
            make_float4(st1[n][r], st2[n][r], cnt > 0.f ? pivL[wave * NT + col + r] : 0.f, cnt);
      else
        *reinterpret_cast<float2 *>(a.stats + (row * a.CoutW + c) * 2) = make_float2(st1[n][r], st2[n][r]);
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
  const long halo_f = (HV * ckp_of(CK) + 1) / 2 + 4;   // bf16 image + a dummy 16-byte slot
  (void)NT;
  return (halo_f + 3) & ~3L;
}

static long bconv_lds(const GConvArgs &a, int CK, int NT) {
  const int T = a.KX * a.KY * a.KZ;
  const int TPS = 32 / CK;
  const int S = (T + TPS - 1) / TPS;
  return (bconv_areg(a, CK, NT) + (long)S * 4 * NT * 4 + S * 4 + (long)a.MPW * 128 + 9L * NT +
          2L * a.ICs) * 4 + (long)sizeof(GConvArgs);   // + the static copy of the arguments
}

static int reduce_vpb(const GConvArgs &a) { return 2 * 256 / (a.OCs / 8); }

int bconv_stat_rows(const GConvArgs &a) {
  if (a.ksplit > 1) {
    const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
    const int vpb = reduce_vpb(a);
    return (int)((nvox + vpb - 1) / vpb);
  }
  return a.gridx * 4;   // one row per (block, wave)
}

int plan_bconv(GConvArgs &a, int target_blocks) {
  a.use_bconv = 0;
  if (a.OX <= 0 || a.OY <= 0 || a.OZ <= 0) return fail(2, "bconv: empty output grid");
  if (a.ICs % 8 || a.OCs % 8) return fail(4, "bconv: channel strides must be multiples of 8");
  // 32-bit buffer offsets within one sample (fp32 K-split partials included)
  if ((double)a.SX * a.SY * a.SZ * a.OCs * 4 >= 2147483647.0 ||
      (double)a.IX * a.IY * a.IZ * a.ICs * 2 >= 2147483647.0)
    return fail(4, "bconv: one sample must stay below 2 GiB");
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
  // HCU_BCONV_FORCE="CK,NSUB,MPW[,NPF]" restricts the search (experiments)
  int fck = 0, fns = 0, fmp = 0, fpf = -1;
  if (const char *e = getenv("HCU_BCONV_FORCE")) sscanf(e, "%d,%d,%d,%d", &fck, &fns, &fmp, &fpf);
  for (int ni = 0; ni < 3; ++ni) {
    const int NSUB = nsubs[ni];
    if (fns && NSUB != fns) continue;
    if (NSUB > 1 && nb16 < NSUB && !(NSUB == 2 && nb16 >= 2)) continue;
    if (NSUB == 4 && nb16 < 4) continue;
    if (NSUB == 2 && nb16 < 2) continue;
    if (a.nph > 1 && (a.Cout % (NSUB * 16) || a.Cout % 8)) continue;
    const int NT = NSUB * 16;
    const int CoutW = round_up(Nlog, NT);
    const int nN = CoutW / NT;
    for (int mi = 0; mi < 3; ++mi) {
      const int MPW = mpws[mi];
      if (fmp && MPW != fmp) continue;
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
        if (a.ICs % CK || (fck && CK != fck)) continue;
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
  if (fpf >= 0 && (fpf == 0 || fpf >= per_thread)) a.NPF = fpf;
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
    if (a.bn_y)                                                                                 \
      HCU_TIMED(s, "bconv_kernel<" #CK_ "," #NS_ "," #MP_ "," #PF_ ",bnb>", fl, by,               \
                hipLaunchKernelGGL((bconv_kernel<CK_, NS_, MP_, PF_, true>), grid, dim3(256),   \
                                   a.lds_bytes - (int)sizeof(GConvArgs), s, a));                \
    else                                                                                        \
      HCU_TIMED(s, "bconv_kernel<" #CK_ "," #NS_ "," #MP_ "," #PF_ ">", fl, by,                   \
                hipLaunchKernelGGL((bconv_kernel<CK_, NS_, MP_, PF_, false>), grid, dim3(256),  \
                                   a.lds_bytes - (int)sizeof(GConvArgs), s, a));                \
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
