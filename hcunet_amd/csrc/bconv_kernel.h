// Blocked implicit-GEMM convolution on MFMA, for bf16 (v_mfma_f32_16x16x32_bf16)
// and fp32 (v_mfma_f32_16x16x4_f32) activations: the kernel template shared by
// bconv.hip (bf16 instances, the planner) and bconv_f32.hip (fp32 instances).
//
// GEMM view: M = output voxels of a TX*TY*TZ tile (TZ = the whole Z extent,
// <= 16), N = output channels (x ConvTranspose3d stride phases), K = (tap,
// input channel).  One workgroup = 4 waves; wave w owns the 16-voxel
// M-subtiles w, w+4, ... (MPW of them) and all NSUB 16-column subtiles.
//
// Element E (uint16_t = bf16 storage, or float), VEC = elements per 16 bytes
// (8 or 4).  A channel chunk is CK = CV * VEC channels (CV 16-byte groups);
// one K-step is 4 lane groups x 16 bytes: TPS = 4 / CV taps x CK channels.
// Lane group g = lane / 16 reads 16 bytes = VEC consecutive channels (group
// cv = g % CV) of its voxel shifted by tap t = s * TPS + g / CV with ONE
// ds_read_b128 from the channels-last halo image [hv][CKP]; the weight
// fragment of lane (g, column n) is the matching 16-byte run of the packed
// image [chunk][s][g][n][VEC].  Per K-step and (M-subtile, N-subtile): one
// bf16 MFMA (K = 32) or four fp32 MFMAs (K = 4 each, element c of the 16 bytes).
//
// The MFMA is issued with the weights as A and the activations as B, so the
// accumulators hold the transposed tile: acc[j][n][r] = out[voxel (wave+4j)*16
// + r16][column n*16 + 4g + r]: every lane owns 4 consecutive channels of one
// voxel and stores them straight from the accumulators (8 bytes bf16, 16 bytes
// fp32), with the bias, the BatchNorm statistics (pivot-shifted rows per
// (block, wave), common.h StatRow) or, for an input gradient feeding a
// BatchNorm backward (BNB), the fused ReLU mask and (sum dz, sum dz*xhat).
// With a K split the fp32 partial sums go to `partial` and bconv_reduce adds
// them in a fixed order.
//
// Staging: the halo of the next (tile, chunk) is loaded into registers with
// buffer loads (invalid positions read an offset past the buffer -> 0) while
// the current one is computed; BatchNorm+ReLU of the producer is applied when
// it is written to LDS (fp32 arithmetic), positions outside the input are 0.
// Barriers order LDS only (lds_barrier), launch constants come from an LDS
// copy of the arguments (kuni), and the compiler's wait for each prefetched
// element never includes the previous tile's output stores (dummy_epilogue).
//
// Replaces nn.Conv3d forward / input-gradient and nn.ConvTranspose3d forward /
// input-gradient of the reference path (hcat/unet.py:246-257, 281-298).
#pragma once
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
// per block slot (plain stores, no atomics: blocks of successive launches with
// the same index run one after another) of kPhN counters
constexpr int kPhBlocks = 8192, kPhN = 12;
extern __device__ unsigned long long g_bconv_phase[kPhBlocks * kPhN];
#define PH_MARK(k)                                                 \
  do {                                                             \
    const long long t__ = (long long)__builtin_readcyclecounter(); \
    ph_acc[k] += t__ - ph_t;                                       \
    ph_t = t__;                                                    \
  } while (0)
#else
#define PH_MARK(k) \
  do {             \
  } while (0)
#endif

// Halo row stride in bytes.  ds_read_b128 serves a wave in 4 lane groups of 16
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...); with CV = 4 the lanes of one
// group read rows r of group g and rows r' of group g+1, and a row of 6
// 16-byte slots puts all 16 on distinct bank slots for consecutive rows; CV =
// 2 uses 3 slots, CV = 1 one (rows are contiguous).
constexpr int ckp_bytes(int CV) { return CV == 1 ? 16 : (CV == 2 ? 48 : CV * 16 + 32); }

template <class E>
struct BElem;
template <>
struct BElem<uint16_t> {
  static constexpr int VEC = 8;
};
template <>
struct BElem<float> {
  static constexpr int VEC = 4;
};

// BatchNorm+ReLU of the 16 bytes v (VEC channels); s, h: VEC floats in LDS.
__device__ __forceinline__ uint4 bact16(uint16_t *, uint4 v, const float *s, const float *h) {
  // fp32 fma (v_pk_fma_f32), rounded to bf16, ReLU on the packed bf16
  const floatx4 s0 = *reinterpret_cast<const floatx4 *>(s);
  const floatx4 s1 = *reinterpret_cast<const floatx4 *>(s + 4);
  const floatx4 h0 = *reinterpret_cast<const floatx4 *>(h);
  const floatx4 h1 = *reinterpret_cast<const floatx4 *>(h + 4);
  uint4 o;
  o.x = bn_relu_bf2(v.x, s0.xy, h0.xy);
  o.y = bn_relu_bf2(v.y, s0.zw, h0.zw);
  o.z = bn_relu_bf2(v.z, s1.xy, h1.xy);
  o.w = bn_relu_bf2(v.w, s1.zw, h1.zw);
  return o;
}
__device__ __forceinline__ uint4 bact16(float *, uint4 v, const float *s, const float *h) {
  floatx4 f = __builtin_bit_cast(floatx4, v);
  f = f * *reinterpret_cast<const floatx4 *>(s) + *reinterpret_cast<const floatx4 *>(h);
  f.x = fmaxf(f.x, 0.f);
  f.y = fmaxf(f.y, 0.f);
  f.z = fmaxf(f.z, 0.f);
  f.w = fmaxf(f.w, 0.f);
  return __builtin_bit_cast(uint4, f);
}

// acc += W(16 columns x 16 bytes of K per lane group) * A(16 voxels)
__device__ __forceinline__ floatx4 bmma(uint16_t *, uint4 w, uint4 x, floatx4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(shortx8, w),
                                                 __builtin_bit_cast(shortx8, x), acc, 0, 0, 0);
}
__device__ __forceinline__ floatx4 bmma(float *, uint4 w, uint4 x, floatx4 acc) {
  const floatx4 wf = __builtin_bit_cast(floatx4, w), xf = __builtin_bit_cast(floatx4, x);
#pragma unroll
  for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[c], xf[c], acc, 0, 0, 0);
  return acc;
}

// 4 output channels of one voxel: stored value (bf16: 8 bytes, fp32: 16 bytes)
__device__ __forceinline__ void bstore4(uint16_t *, const floatx4 &v, __amdgpu_buffer_rsrc_t r, int off) {
  const u32x2 pk2 = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
  __builtin_amdgcn_raw_buffer_store_b64(pk2, r, off * 2, 0, 0);
}
__device__ __forceinline__ void bstore4(float *, const floatx4 &v, __amdgpu_buffer_rsrc_t r, int off) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off * 4, 0, 0);
}
__device__ __forceinline__ floatx4 bload4(uint16_t *, __amdgpu_buffer_rsrc_t r, int off_bytes) {
  const u32x2 w = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off_bytes, 0, 0));
  return floatx4{bf_lo(w.x), bf_hi(w.x), bf_lo(w.y), bf_hi(w.y)};
}
__device__ __forceinline__ floatx4 bload4(float *, __amdgpu_buffer_rsrc_t r, int off_bytes) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, 0));
}

// MODE 1 (BNB): the fused BatchNorm+ReLU backward epilogue.  MODE 2 (NCX,
// CV = 1, forward of the network's first layer): the input is the caller's
// NCXYZ volume (GConvArgs::in_fmt fp32 / fp16 / bf16, <= 4 channels): each
// halo element gathers its channels from the channel planes (consecutive
// lanes: consecutive z, then y -- one contiguous run of a plane per wave),
// converts them to E when the halo image is written (the rounding the
// channels-last layout pass applies), stores the channels-last copy of the
// voxels its tile owns (a.xcl), and the weights are read in their PyTorch
// layout [Cout][in_c][T] (no packed image: the first layer runs ahead of the
// weight re-layout).
template <class E, int CV, int NSUB, int MPW, int NPF, int MODE>
__global__ void __launch_bounds__(256) bconv_kernel(const GConvArgs a) {
  constexpr bool BNB = (MODE & 1) != 0;
  constexpr bool NCX = MODE == 2;
  static_assert(!NCX || (CV == 1 && NPF > 0), "NCXYZ staging: one 16-byte group, prefetched");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // launch constants for the tile loop, read through kuni (common.h): they are
  // live only in the phase that uses them, not for the whole kernel
  __shared__ __attribute__((aligned(16))) char sa_raw[sizeof(GConvArgs)];
  GConvArgs &sa = *reinterpret_cast<GConvArgs *>(sa_raw);
#define KA(f) kuni(sa.f)
  constexpr int VEC = BElem<E>::VEC;
  constexpr int ES = (int)sizeof(E);
  constexpr int NT = NSUB * 16;
  constexpr int CK = CV * VEC;         // channels per chunk
  constexpr int TPS = 4 / CV;          // taps per K-step
  constexpr int CKP = ckp_bytes(CV) / ES;   // halo row stride (elements)
  E *const tag = nullptr;              // overload selector
#ifdef HCU_BCONV_PHASES
  const long long ph_start = (long long)__builtin_readcyclecounter();
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  if (tid == 0) sa = a;
  const int T = a.KX * a.KY * a.KZ;
  const int S = (T + TPS - 1) / TPS;
  // halo image rows: (hx, hy, hz) at hx * hsx + hy * hsy + hz * hsz (the
  // planner's axis order / padding), a dummy slot at row hvp
  const int hsx = a.hsx, hsy = a.hsy, hsz = a.hsz;
  const int HV = a.HX * a.HY * a.HZ, HVP = a.hvp;
  E *alds = reinterpret_cast<E *>(smem);                          // [hvp][CKP] + a dummy slot
  E *wlds = reinterpret_cast<E *>(smem + a.areg);                 // [S][4][NT][VEC]
  int *toffs = reinterpret_cast<int *>(wlds + S * 4 * NT * VEC);  // [S][4]
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
      v = lx * a.sx * hsx + ly * a.sy * hsy + lz * a.sz * hsz;
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
    const int t = (e >> 2) * TPS + (e & 3) / CV;
    int off = 0;
    if (t < T) {
      const int kz = t % a.KZ, q = t / a.KZ, ky = q % a.KY, kx = q / a.KY;
      off = kx * a.dx * hsx + ky * a.dy * hsy + kz * a.dz * hsz;
    }
    toffs[e] = off * CKP + ((e & 3) % CV) * VEC;
  }
  // first stored channel of the block (ConvTranspose3d phases folded into N:
  // column n0 + j is channel (n0 + j) % CPH of phase (n0 + j) / CPH, CPH the
  // columns per phase: Cout, or Cout padded to the store width (GConvArgs::cph))
  const int CPH = a.cph > 0 ? a.cph : a.Cout;
  const int co0 = a.nph > 1 ? n0 - (n0 / CPH) * CPH : n0;
  // the 4 stored columns of lane group g in column subtile n: their first
  // channel (-1: past the stored channels) and the output offset of their
  // phase (CPH % 4 == 0, so the 4 share it; a block may span phases)
  int cn[NSUB], qo[NSUB];
#pragma unroll
  for (int n = 0; n < NSUB; ++n) {
    const int gcl = n0 + n * 16 + g * 4;
    if (a.nph > 1) {
      const int ph = gcl / CPH;
      const int qz = ph % a.phz, qy = (ph / a.phz) % a.phy, qx = ph / (a.phz * a.phy);
      cn[n] = ph < a.nph ? gcl - ph * CPH : -1;
      qo[n] = ((qx * a.SY + qy) * a.SZ + qz) * a.OCs;
    } else {
      cn[n] = gcl < a.OCs ? gcl : -1;
      qo[n] = 0;
    }
  }
  // (the coefficient loads follow the first halo fetch: load_coefs below)

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
    if constexpr (NCX) {   // PyTorch-layout weights: 16 bytes = channels 0..VEC-1 of tap sg, column n
      const int INC = KA(in_c), Cout = KA(Cout);
      const float *wr = KA(w);
      for (int idx = tid; idx < n16; idx += 256) {
        const int n = idx % NT, t = idx / NT, co = blockIdx.y * NT + n;
        float v[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] = (t < T && co < Cout && j < INC) ? wr[((size_t)co * INC + j) * T + t] : 0.f;
        if constexpr (ES == 2) {
          reinterpret_cast<uint4 *>(wlds)[idx] = pack8(v);
        } else {
          reinterpret_cast<uint4 *>(wlds)[idx] = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]),
                                                            __float_as_uint(v[2]), __float_as_uint(v[3]));
        }
      }
      return;
    }
    const uint4 *src = reinterpret_cast<const uint4 *>(KA(w));
    const int CoutW = KA(CoutW);
    for (int idx = tid; idx < n16; idx += 256) {
      const int n = idx % NT, sg = idx / NT;
      reinterpret_cast<uint4 *>(wlds)[sg * NT + n] =
          src[((size_t)chunk * S * 4 + sg) * CoutW + blockIdx.y * NT + n];
    }
  };

  // ---- weights of a block that walks several channel chunks per tile (the
  // deep levels: few tiles, K split over chunks inside the block): the next
  // chunk's packed weights are loaded into registers with the next halo, so
  // the per-chunk weight staging no longer waits on an L2 round trip.  Up to
  // WPR 16-byte elements per thread (NT = 16: S <= 20; NT = 32: S <= 10);
  // larger images keep the synchronous stage_w.  Only in the instances whose
  // register budget has room for the 20 extra VGPRs (NSUB <= 2, NPF <= 8):
  // measured on MI355X, the NSUB = 4 / NPF = 12 input-gradient variants lost
  // occupancy and ran 40-60 % slower with them.
  // (NSUB = 1 instances: up to 8 per thread, S <= 32 at NT = 16 -- the 125-tap
  // kernels of RDCNet at 8 channels per chunk stage their 32 KB chunk images
  // this way instead of synchronously; slots past the image are skipped, a
  // uniform branch)
#ifndef HCU_BCONV_WPR8
#define HCU_BCONV_WPR8 1
#endif
  constexpr bool WPOK = NPF > 0 && NPF <= 8 && NSUB <= 2;
  constexpr int WPR = WPOK ? ((NSUB == 1 && HCU_BCONV_WPR8) ? 8 : 5) : 1;
  const int n16w = S * 4 * NT;
  const bool wpre = WPOK && nck > 1 && n16w <= 256 * WPR;
  uint4 wpf[WPR];
  auto wfetch = [&](int chunk) {
    const int CoutW = KA(CoutW);
    const uint32_t nrec = (uint32_t)nchunks * S * 4 * CoutW * 16;
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)KA(w), 0, (int)nrec, 0x00020000);
#pragma unroll
    for (int u = 0; u < WPR; ++u) {
      if (u > 4 && u * 256 >= n16w) break;   // (uniform: the slots past the image)
      const int idx = tid + u * 256;
      const int n = idx % NT, sg = idx / NT;
      const int off = idx < n16w ? (((chunk * S * 4 + sg) * CoutW + (int)blockIdx.y * NT + n) * 16) : 0x7ffffff0;
      wpf[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
    }
  };
  auto wstore = [&]() {   // every thread writes WPR slots (past the image: the dummy slot region)
#pragma unroll
    for (int u = 0; u < WPR; ++u) {
      const int idx = tid + u * 256;
      if (idx < n16w) reinterpret_cast<uint4 *>(wlds)[idx] = wpf[u];
    }
  };

  // ---- halo staging: thread tid owns 16-byte channel group cv = tid % CV of
  // halo voxels v = tid / CV + u * (256 / CV); their halo coordinates are fixed.
  constexpr int VS = 256 / CV;
  constexpr int NPFR = NPF > 0 ? NPF : 1;
  const int cv = tid % CV;
  int hpk[NPFR];
#pragma unroll
  for (int u = 0; u < NPFR; ++u) {
    const int v = tid / CV + u * VS;
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
  // the last fetch's buffer resource and per-element byte offsets: the next
  // channel chunk of the same tile only moves every valid offset by CK
  // channels (fetch_adv) instead of re-deriving the tile origin and the
  // element addresses from the LDS copy of the arguments (~1.5 K cycles per
  // chunk in the deep levels' multi-chunk tiles)
  // (not in the fused-BatchNorm-backward instances with 12+ prefetched
  // elements: at 256 VGPRs the 12 saved offsets cost config 3's d0.c2 input
  // gradient 303 -> 340 us, and its tiles are single-chunk)
  constexpr bool ADV = !NCX && !(BNB && NPF >= 12);
  __amdgpu_buffer_rsrc_t frs = __builtin_amdgcn_make_buffer_rsrc((void *)a.in, 0, 0, 0x00020000);
  int foff[ADV ? NPFR : 1];
  // halo of (tile, chunk) -> pf (branch-free: the validity of each element is
  // a mask, invalid elements read offset 0x7ffffff0, outside the buffer -> 0)
  // NCXYZ input (NCX): element u's channels from the planes; the raw loaded
  // values (fp32 bits or a 16-bit value) in pf[u].x..w, converted when written
  auto fetch_ncx = [&](int b, int x0, int y0, int z0, int IX, int IY, int IZ, int INC, int fmt) {
    const int ESI = fmt == 1 ? 4 : 2;
    const int plane = IX * IY * IZ;
    const char *bp = reinterpret_cast<const char *>(KA(in)) + (size_t)b * INC * plane * ESI;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, INC * plane * ESI, 0x00020000);
    okbits = 0;
#pragma unroll
    for (int u = 0; u < NPFR; ++u) {
      const int hp = hpk[u];
      const int gx = x0 + (hp >> 20), gy = y0 + ((hp >> 10) & 1023), gz = z0 + (hp & 1023);
      const bool ok = (hp >= 0) & ((unsigned)gx < (unsigned)IX) & ((unsigned)gy < (unsigned)IY) &
                      ((unsigned)gz < (unsigned)IZ);
      const int vo = (gx * IY + gy) * IZ + gz;
      uint32_t r[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int off = (ok && c < INC) ? (c * plane + vo) * ESI : 0x7ffffff0;
        r[c] = fmt == 1 ? __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0)
                        : (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0);
      }
      pf[u] = make_uint4(r[0], r[1], r[2], r[3]);
      okbits |= (uint32_t)ok << u;
    }
  };
  auto fetch = [&](int tile, int chunk) {
    int b, x0, y0, z0;
    tile_origin(tile, b, x0, y0, z0);
    if constexpr (NCX) {
      fetch_ncx(b, x0 * KA(sx) - KA(px), y0 * KA(sy) - KA(py), z0 * KA(sz) - KA(pz), KA(IX), KA(IY), KA(IZ),
                KA(in_c), KA(in_fmt));
      return;
    }
    const int IX = KA(IX), IY = KA(IY), IZ = KA(IZ), ICs = KA(ICs);
    const uint32_t bZ = (uint32_t)ICs * ES, bY = (uint32_t)IZ * bZ, bX = (uint32_t)IY * bY;
    const int gx0 = x0 * KA(sx) - KA(px), gy0 = y0 * KA(sy) - KA(py), gz0 = z0 * KA(sz) - KA(pz);
    const char *bp = reinterpret_cast<const char *>(KA(in)) + (size_t)b * IX * bX;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, IX * (int)bX, 0x00020000);
    const int base_off = gx0 * (int)bX + gy0 * (int)bY + gz0 * (int)bZ + (chunk * CK + cv * VEC) * ES;
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
      if constexpr (ADV) foff[u] = off;
      pf[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      okbits |= (uint32_t)ok << u;
    }
    if constexpr (ADV) frs = rs;
  };
  auto fetch_adv = [&]() {   // the next channel chunk of the tile just fetched
    if constexpr (ADV) {
#pragma unroll
      for (int u = 0; u < NPFR; ++u) {
        foff[u] += ((okbits >> u) & 1u) ? CK * ES : 0;
        pf[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(frs, foff[u], 0, 0));
      }
    }
  };
  // The block's first halo fetch, from the kernel arguments themselves (the
  // LDS copy is not written yet): issued before the coefficient loads and the
  // weight staging, so their global round trips overlap instead of adding up
  // (a one-tile block of a deep level spent ~6 K cycles in its prologue).
  auto fetch_first = [&](int tile, int chunk) {
    int b, r, tzi, tyi, txi;
    a.fNT.divmod(tile, b, r);
    a.fNTZ.divmod(r, r, tzi);
    a.fNTY.divmod(r, txi, tyi);
    const int x0 = txi * a.TX, y0 = tyi * a.TY, z0 = tzi * a.TZ;
    if constexpr (NCX) {
      fetch_ncx(b, x0 * a.sx - a.px, y0 * a.sy - a.py, z0 * a.sz - a.pz, a.IX, a.IY, a.IZ, a.in_c, a.in_fmt);
      return;
    }
    const int IX = a.IX, IY = a.IY, IZ = a.IZ, ICs = a.ICs;
    const uint32_t bZ = (uint32_t)ICs * ES, bY = (uint32_t)IZ * bZ, bX = (uint32_t)IY * bY;
    const int gx0 = x0 * a.sx - a.px, gy0 = y0 * a.sy - a.py, gz0 = z0 * a.sz - a.pz;
    const char *bp = reinterpret_cast<const char *>(a.in) + (size_t)b * IX * bX;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, IX * (int)bX, 0x00020000);
    const int base_off = gx0 * (int)bX + gy0 * (int)bY + gz0 * (int)bZ + (chunk * CK + cv * VEC) * ES;
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
      if constexpr (ADV) foff[u] = off;
      pf[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      okbits |= (uint32_t)ok << u;
    }
    if constexpr (ADV) frs = rs;
  };
  auto load_coefs = [&]() {
    for (int j = tid; j < NT; j += 256) {
      const int c = a.nph > 1 ? (n0 + j) % CPH : n0 + j;
      coefL[j] = (!split && a.bias && c < a.Cout) ? a.bias[c] : 0.f;
      const bool bn = BNB && !split && c < a.OCs;
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
  };
  // BatchNorm+ReLU of VEC channels, 0 outside the input
  auto activate = [&](uint4 v, bool ok, int chunk) -> uint4 {
    if (!ok) return make_uint4(0u, 0u, 0u, 0u);
    const int c = chunk * CK + cv * VEC;
    if (!act) return v;
    return bact16(tag, v, actL + c, actL + KA(ICs) + c);
  };
  // direct (non-prefetched) staging of one (tile, chunk) halo
  auto stage_direct = [&](int tile, int chunk) {
    int b, x0, y0, z0;
    tile_origin(tile, b, x0, y0, z0);
    const int gx0 = x0 * a.sx - a.px, gy0 = y0 * a.sy - a.py, gz0 = z0 * a.sz - a.pz;
    const uint32_t bZ = (uint32_t)a.ICs * ES, bY = (uint32_t)a.IZ * bZ, bX = (uint32_t)a.IY * bY;
    const char *bp = reinterpret_cast<const char *>(a.in) + (size_t)b * a.IX * bX;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, a.IX * (int)bX, 0x00020000);
    for (int base = tid / CV; base < HV; base += 4 * VS) {
      uint4 val[4];
      bool okv[4];
      int hrow[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = base + u * VS;
        int t2, hz, hx, hy;
        a.fHZ.divmod(v, t2, hz);
        a.fHY.divmod(t2, hx, hy);
        const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
        const bool ok = v < HV && (unsigned)gx < (unsigned)a.IX && (unsigned)gy < (unsigned)a.IY &&
                        (unsigned)gz < (unsigned)a.IZ;
        const int off = ok ? gx * (int)bX + gy * (int)bY + gz * (int)bZ + (chunk * CK + cv * VEC) * ES
                           : 0x7ffffff0;
        val[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        okv[u] = ok;
        hrow[u] = hx * hsx + hy * hsy + hz * hsz;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = base + u * VS;
        if (v < HV)
          *reinterpret_cast<uint4 *>(alds + hrow[u] * CKP + cv * VEC) =
              activate(val[u], okv[u], chunk);
      }
    }
  };

  // NCX: pf -> E channels (0 past in_c and outside the input) into the halo
  // image, and the channels-last copy of the voxels this tile owns: its output
  // range, plus the kernel's overhang on the grid's last tile of each axis
  auto ncx_store = [&](int b, int ox0, int oy0, int oz0) {
    const int fmt = KA(in_fmt), INC = KA(in_c);
    const bool lastx = ox0 + KA(TX) >= KA(OX), lasty = oy0 + KA(TY) >= KA(OY), lastz = oz0 + KA(TZ) >= KA(OZ);
    E *const xo = reinterpret_cast<E *>(KA(xcl));
    const int IX = KA(IX), IY = KA(IY), IZ = KA(IZ), ICs = KA(ICs);
#pragma unroll
    for (int u = 0; u < NPFR; ++u) {
      const bool ok = (okbits >> u) & 1u;
      float f[VEC];
      const uint32_t r[4] = {pf[u].x, pf[u].y, pf[u].z, pf[u].w};
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float x = 0.f;
        if (j < 4) {
          x = fmt == 1 ? __uint_as_float(r[j])
                       : fmt == 2 ? (float)__builtin_bit_cast(_Float16, (uint16_t)r[j]) : __uint_as_float(r[j] << 16);
        }
        f[j] = (ok && j < INC) ? x : 0.f;
      }
      uint4 w;
      if constexpr (ES == 2) {
        w = pack8(f);
      } else {
        w = make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
      }
      const int hp = hpk[u];
      const int hx = hp >> 20, hy = (hp >> 10) & 1023, hz = hp & 1023;
      *reinterpret_cast<uint4 *>(alds + (hp >= 0 ? (hx * hsx + hy * hsy + hz * hsz) * CKP : HVP * CKP)) = w;
      if (xo && ok && (hx < KA(TX) || lastx) && (hy < KA(TY) || lasty) && (hz < KA(TZ) || lastz)) {
        const size_t vox = (((size_t)b * IX + ox0 * KA(sx) - KA(px) + hx) * IY + oy0 * KA(sy) - KA(py) + hy) * IZ +
                           oz0 * KA(sz) - KA(pz) + hz;
        *reinterpret_cast<uint4 *>(xo + vox * ICs) = w;
      }
    }
  };

  floatx4 acc[MPW][NSUB];
  // fp32 instances with a single (M, N) subtile per wave: the four 16x16x4
  // MFMAs of a K-step alternate between two accumulators (two dependency
  // chains: the 40-cycle MFMA latency no longer paces a lone chain at 4 per
  // K-step), summed once before the epilogue
  constexpr bool DUAL = ES == 4 && MPW * NSUB == 1;
  floatx4 acc2[MPW][NSUB];
  auto load_frag = [&](int s, int toff, uint4 (&bfr)[NSUB], uint4 (&afr)[MPW]) {
    const int ss = min(s, S - 1);
#pragma unroll
    for (int n = 0; n < NSUB; ++n)
      bfr[n] = *reinterpret_cast<const uint4 *>(wlds + ((ss * 4 + g) * NT + n * 16 + r16) * VEC);
#pragma unroll
    for (int j = 0; j < MPW; ++j) afr[j] = *reinterpret_cast<const uint4 *>(alds + vb[j] + toff);
  };
  auto toff_of = [&](int s) { return toffs[min(s, S - 1) * 4 + g]; };
  auto mfma_frag = [&](const uint4 (&bfr)[NSUB], const uint4 (&afr)[MPW]) {
    if constexpr (DUAL) {
      const floatx4 wf = __builtin_bit_cast(floatx4, bfr[0]), xf = __builtin_bit_cast(floatx4, afr[0]);
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[0], xf[0], acc[0][0], 0, 0, 0);
      acc2[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[1], xf[1], acc2[0][0], 0, 0, 0);
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[2], xf[2], acc[0][0], 0, 0, 0);
      acc2[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[3], xf[3], acc2[0][0], 0, 0, 0);
      return;
    }
#pragma unroll
    for (int j = 0; j < MPW; ++j)
#pragma unroll
      for (int n = 0; n < NSUB; ++n) acc[j][n] = bmma(tag, bfr[n], afr[j], acc[j][n]);
  };
  auto compute = [&]() {
    uint4 b0[NSUB], a0[MPW], b1[NSUB], a1[MPW];
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
  // MPW * NSUB stores per tile (BNB: a load before each), invalid ones at an
  // offset outside the buffer (dropped).
  const bool fwdstat = a.stats && !BNB && !split;
  float st1[NSUB][4], st2[NSUB][4], cnt = 0.f;
#pragma unroll
  for (int n = 0; n < NSUB; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) st1[n][r] = st2[n][r] = 0.f;
  // statistics pivot of each wave: set at the first valid output voxel the
  // wave stores (its value + bias), see below
  bool need_piv = true;
  auto epilogue = [&](int b, int ox0, int oy0, int oz0) {
    if constexpr (DUAL) acc[0][0] += acc2[0][0];
    const int OX = KA(OX), OY = KA(OY), OZ = KA(OZ), OCs = KA(OCs);
    const bool interior = ox0 + KA(TX) <= OX && oy0 + KA(TY) <= OY && oz0 + KA(TZ) <= OZ;
    const int sample = KA(SX) * KA(SY) * KA(SZ) * OCs;
    const int tb = (((ox0 * KA(osx) + KA(ofx)) * KA(SY) + oy0 * KA(osy) + KA(ofy)) * KA(SZ) +
                    oz0 * KA(osz) + KA(ofz)) * OCs;
    const size_t sb = (size_t)b * sample;
    const int es = split ? 4 : ES;
    void *obase = split ? (void *)(KA(partial) + (size_t)blockIdx.z * KA(slice_floats) + sb)
                        : (void *)(reinterpret_cast<E *>(KA(out)) + sb);
    const __amdgpu_buffer_rsrc_t ors =
        __builtin_amdgcn_make_buffer_rsrc(obase, 0, sample * es, 0x00020000);
    const E *ybf = BNB ? reinterpret_cast<const E *>(KA(bn_y)) : nullptr;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        BNB ? (void *)(ybf + sb) : obase, 0, BNB ? sample * ES : 0, 0x00020000);
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
      floatx4 yv[NSUB];
      if (BNB)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) {
          const bool ok = vok & (cn[n] >= 0);
          yv[n] = bload4(tag, yrs, ok ? (rof + qo[n] + cn[n]) * ES : 0x3ffffff0);
        }
      if (fwdstat && need_piv) {
        // the wave's pivot: the lowest valid voxel of this M-subtile (lanes
        // 0..15 hold the subtile's 16 voxels; every lane group has the same)
        const uint32_t m16 = (uint32_t)__ballot(vok) & 0xffffu;
        if (m16) {
          const int src = (lane & 48) | (__builtin_ctz(m16));
#pragma unroll
          for (int n = 0; n < NSUB; ++n) {
            const floatx4 bias = *reinterpret_cast<const floatx4 *>(coefL + n * 16 + g * 4);
            floatx4 p;
#pragma unroll
            for (int r = 0; r < 4; ++r) p[r] = bias[r] + __shfl(acc[j][n][r], src);
            if (r16 == 0) *reinterpret_cast<floatx4 *>(pivL + wave * NT + n * 16 + g * 4) = p;
          }
          need_piv = false;
        }
      }
      if (vok) cnt += 1.f;
#pragma unroll
      for (int n = 0; n < NSUB; ++n) {
        const int col = n * 16 + g * 4;
        const bool ok = vok & (cn[n] >= 0);
        const int off = ok ? rof + qo[n] + cn[n] : 0x1fffffff;
        floatx4 v = acc[j][n];
        if (split) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ors, off * 4, 0, 0);
          continue;
        }
        v += *reinterpret_cast<const floatx4 *>(coefL + col);
        if (BNB) {   // fused BatchNorm+ReLU backward: v = dA -> dz; (dz, dz*xhat)
          const floatx4 y = yv[n];
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
        bstore4(tag, v, ors, off);
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

  // ---- main loop over (tile, chunk) items; contiguous tile range per block:
  // consecutive tiles share halo rows, which then come from this CU's L2
  const int tpb_ = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t_beg = blockIdx.x * tpb_, t_end = min(total, t_beg + tpb_);
  if (NPF > 0 && t_beg < t_end) fetch_first(t_beg, cb);
  load_coefs();
  lds_barrier();   // sa, tables and coefficients are in LDS
#ifdef HCU_BCONV_PHASES
  long long ph_acc[6] = {0, 0, 0, 0, 0, 0};
  long long ph_t = (long long)__builtin_readcyclecounter();
  const long long ph_loop0 = ph_t;   // prologue = ph_loop0 - ph_start
#endif
  if (NPF > 0) {
    int tile = t_beg;
    if (nck == 1) stage_w(cb);
    if (tile < t_end && wpre) wfetch(cb);   // the halo of (t_beg, cb) is in flight (fetch_first)
    dummy_epilogue();
    for (; tile < t_end; ++tile) {
#pragma unroll
      for (int j = 0; j < MPW; ++j)
#pragma unroll
        for (int n = 0; n < NSUB; ++n) acc[j][n] = acc2[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
      for (int chunk = cb; chunk < ce; ++chunk) {
        lds_barrier();
        if constexpr (NCX) {
          int b, ox0, oy0, oz0;
          tile_origin(tile, b, ox0, oy0, oz0);
          ncx_store(b, ox0, oy0, oz0);
        } else {
#pragma unroll
        for (int u = 0; u < NPFR; ++u) {   // every element is written (the waits stay exact)
          const int hp = hpk[u];
          const int row = (hp >> 20) * hsx + ((hp >> 10) & 1023) * hsy + (hp & 1023) * hsz;
          *reinterpret_cast<uint4 *>(alds + (hp >= 0 ? row * CKP + cv * VEC : HVP * CKP)) =
              activate(pf[u], (okbits >> u) & 1u, chunk);
        }
        }
        PH_MARK(0);
        if (wpre)
          wstore();
        else if (nck > 1)
          stage_w(chunk);
        lds_barrier();
        PH_MARK(1);
        int nt = tile, nc = chunk + 1;
        if (nc == ce) {
          nc = cb;
          nt = tile + 1;
        }
        if (nt < t_end) {
          if (ADV && nt == tile)
            fetch_adv();
          else
            fetch(nt, nc);
          if (wpre) wfetch(nc);
        }
        PH_MARK(2);
        compute();
        PH_MARK(3);
        dummy_epilogue();   // unconditional: a branch here would be a path without it
      }
      int b, ox0, oy0, oz0;
      tile_origin(tile, b, ox0, oy0, oz0);
      epilogue(b, ox0, oy0, oz0);
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
        for (int n = 0; n < NSUB; ++n) acc[j][n] = acc2[j][n] = floatx4{0.f, 0.f, 0.f, 0.f};
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
      epilogue(b, ox0, oy0, oz0);
      PH_MARK(4);
#ifdef HCU_BCONV_PHASES
      ph_acc[5] += 1;
#endif
    }
  }
#ifdef HCU_BCONV_PHASES
  const long long ph_loop1 = (long long)__builtin_readcyclecounter();
  long long ph_post[3] = {ph_loop1, ph_loop1, ph_loop1};
  auto ph_flush = [&]() {
    if (tid != 0) return;
    const long long t_end = (long long)__builtin_readcyclecounter();
    const int slot = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) % kPhBlocks;
    unsigned long long *d = g_bconv_phase + (size_t)slot * kPhN;
    for (int k = 0; k < 6; ++k) d[k] += (unsigned long long)ph_acc[k];
    d[6] += (unsigned long long)(ph_loop0 - ph_start);   // prologue
    d[7] += (unsigned long long)(t_end - ph_start);      // lifetime
    d[8] += (unsigned long long)(ph_post[0] - ph_loop1); // post-loop: shuffles
    d[9] += (unsigned long long)(ph_post[1] - ph_post[0]);  // LDS merge (2 barriers)
    d[10] += (unsigned long long)(ph_post[2] - ph_post[1]); // row merge + store
    d[11] += (unsigned long long)(t_end - ph_post[2]);
  };
#endif

  // ---- statistics row of the block: fixed-order butterfly over the 16 voxel
  // lanes of each channel group, then the 4 waves' (S1, S2, K, n) merged in a
  // fixed order by the parallel-variance identity about the first non-empty
  // wave's pivot (fused BatchNorm backward: plain sums)
  if (!a.stats || split) {
#ifdef HCU_BCONV_PHASES
    ph_flush();
#endif
    return;
  }
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
#ifdef HCU_BCONV_PHASES
  ph_post[0] = ph_post[1] = ph_post[2] = (long long)__builtin_readcyclecounter();
#endif
  lds_barrier();   // the halo region is free: [4 waves][NT] of (S1, S2, n)
  float *mrg = smem;
  if (r16 == 0)
#pragma unroll
    for (int n = 0; n < NSUB; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float *e = mrg + ((size_t)wave * NT + n * 16 + g * 4 + r) * 3;
        e[0] = st1[n][r];
        e[1] = st2[n][r];
        e[2] = cnt;
      }
  lds_barrier();
#ifdef HCU_BCONV_PHASES
  ph_post[1] = ph_post[2] = (long long)__builtin_readcyclecounter();
#endif
  for (int col = tid; col < NT; col += 256) {
    if (co0 + col >= a.OCs) continue;
    float S1 = 0.f, S2 = 0.f, nn = 0.f, K = 0.f;
    bool have = false;
    for (int w = 0; w < 4; ++w) {
      const float *e = mrg + ((size_t)w * NT + col) * 3;
      if (!fwdstat) {
        S1 += e[0];
        S2 += e[1];
        continue;
      }
      if (e[2] <= 0.f) continue;
      const float Kw = pivL[w * NT + col];
      if (!have) {
        K = Kw;
        have = true;
      }
      const float d = Kw - K;   // shift (S1, S2) of wave w from pivot Kw to K
      S2 += e[1] + d * (2.f * e[0] + e[2] * d);
      S1 += e[0] + e[2] * d;
      nn += e[2];
    }
    const size_t c = (size_t)blockIdx.x * a.CoutW + n0 + col;
    if (fwdstat)
      *reinterpret_cast<float4 *>(a.stats + c * 4) = make_float4(S1, S2, K, nn);
    else
      *reinterpret_cast<float2 *>(a.stats + c * 2) = make_float2(S1, S2);
  }
#ifdef HCU_BCONV_PHASES
  ph_post[2] = (long long)__builtin_readcyclecounter();
#endif
#ifdef HCU_BCONV_PHASES
  ph_flush();
#endif
#undef KA
}

// Sum of the K-split fp32 slices in a fixed order + bias -> E output, with the
// BatchNorm statistics rows (pivoted) or the fused BatchNorm-backward rows.
// Thread tid owns channel group c16 = tid % G (G = OCs / GV groups of GV = 16 /
// sizeof(E) channels) of voxels v0 + tid/G + k*(256/G).
template <class E>
__global__ void __launch_bounds__(256) bconv_reduce_kernel(const GConvArgs a, int vox_per_block) {
  constexpr int GV = 16 / (int)sizeof(E);
  __shared__ float red[256][3];
  const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
  const int G = a.OCs / GV;
  const int tid = threadIdx.x;
  const int cg = tid % G;
  const int vstep = 256 / G;
  const int64_t v0 = (int64_t)blockIdx.x * vox_per_block;
  const int64_t v1 = min(v0 + vox_per_block, nvox);
  float bv[GV], bsc[GV], bsh[GV], bmu[GV], bis[GV];
#pragma unroll
  for (int k = 0; k < GV; ++k) {
    const int c = cg * GV + k;
    bv[k] = (a.bias && c < a.Cout) ? a.bias[c] : 0.f;
    bsc[k] = bsh[k] = bmu[k] = bis[k] = 0.f;
    if (a.bn_y) {
      bsc[k] = a.bn_scale[c];
      bsh[k] = a.bn_shift[c];
      bmu[k] = a.bn_mean[c];
      bis[k] = a.bn_invstd[c];
    }
  }
  auto vsum = [&](int64_t v, float (&s)[GV]) {
    const size_t off = (size_t)v * a.OCs + cg * GV;
#pragma unroll
    for (int k = 0; k < GV; ++k) s[k] = bv[k];
    for (int q = 0; q < a.ksplit; ++q) {
#pragma unroll
      for (int k4 = 0; k4 < GV; k4 += 4) {
        const float4 p = *reinterpret_cast<const float4 *>(a.partial + (size_t)q * a.slice_floats + off + k4);
        s[k4] += p.x;
        s[k4 + 1] += p.y;
        s[k4 + 2] += p.z;
        s[k4 + 3] += p.w;
      }
    }
  };
  auto load_y = [&](size_t off, float (&y)[GV]) {
    if constexpr (sizeof(E) == 2) {
      unpack8(*reinterpret_cast<const uint4 *>(reinterpret_cast<const uint16_t *>(a.bn_y) + off), y);
    } else {
      const float4 t = *reinterpret_cast<const float4 *>(a.bn_y + off);
      y[0] = t.x; y[1] = t.y; y[2] = t.z; y[3] = t.w;
    }
  };
  auto store = [&](size_t off, const float (&s)[GV]) {
    if constexpr (sizeof(E) == 2) {
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = s[k];
      *reinterpret_cast<uint4 *>(reinterpret_cast<uint16_t *>(a.out) + off) = pack8(f);
    } else {
      *reinterpret_cast<float4 *>(a.out + off) = make_float4(s[0], s[1], s[2], s[3]);
    }
  };
  const bool fwdstat = a.stats && !a.bn_y;
  float piv[GV], st1[GV], st2[GV], cnt = 0.f;
#pragma unroll
  for (int k = 0; k < GV; ++k) piv[k] = st1[k] = st2[k] = 0.f;
  if (fwdstat) vsum(v0, piv);
  for (int64_t v = v0 + tid / G; v < v1; v += vstep) {
    const size_t off = (size_t)v * a.OCs + cg * GV;
    float s[GV];
    vsum(v, s);
    if (a.bn_y) {
      float y[GV];
      load_y(off, y);
#pragma unroll
      for (int k = 0; k < GV; ++k) {
        s[k] = fmaf(y[k], bsc[k], bsh[k]) > 0.f ? s[k] : 0.f;
        st1[k] += s[k];
        st2[k] = fmaf(s[k], (y[k] - bmu[k]) * bis[k], st2[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < GV; ++k) {
        const float d = s[k] - piv[k];
        st1[k] += d;
        st2[k] = fmaf(d, d, st2[k]);
      }
    }
    cnt += 1.f;
    store(off, s);
  }
  if (!a.stats) return;
  for (int k = 0; k < GV; ++k) {
    lds_barrier();
    red[tid][0] = st1[k];
    red[tid][1] = st2[k];
    red[tid][2] = cnt;
    lds_barrier();
    if (tid < G) {
      float t1 = 0.f, t2 = 0.f, tn = 0.f;
      for (int q = tid; q < 256; q += G) {
        t1 += red[q][0];
        t2 += red[q][1];
        tn += red[q][2];
      }
      const int c = tid * GV + k;
      if (fwdstat)
        *reinterpret_cast<float4 *>(a.stats + ((size_t)blockIdx.x * a.CoutW + c) * 4) =
            make_float4(t1, t2, piv[k], tn);
      else
        *reinterpret_cast<float2 *>(a.stats + ((size_t)blockIdx.x * a.CoutW + c) * 2) = make_float2(t1, t2);
    }
  }
}

// K-split reduce geometry: voxels per reduce block
inline int bconv_reduce_vpb(const GConvArgs &a) { return 2 * 256 / (a.OCs / (16 / a.bes)); }

int launch_bconv_bf16(const GConvArgs &a, hipStream_t s);
int launch_bconv_f32(const GConvArgs &a, hipStream_t s);

// Instantiation helpers shared by the two launch files.
#define BCONV_MODE(E_, TAG_, CV_, NS_, MP_, PF_, M_, SUF_)                                         \
  case M_:                                                                                           \
    HCU_TIMED(s, "bconv_kernel<" TAG_ "," #CV_ "," #NS_ "," #MP_ "," #PF_ SUF_ ">", fl, by,          \
              HCU_LAUNCH((bconv_kernel<E_, CV_, NS_, MP_, PF_, M_>), grid, dim3(256),                \
                         a.lds_bytes - (int)sizeof(GConvArgs), s, a));                               \
    break;
#define BCONV_CASE(E_, TAG_, CV_, NS_, MP_, PF_)                                                     \
  if (a.NSUB == NS_ && a.MPW == MP_ && a.NPF == PF_) {                                               \
    switch (mode) {                                                                                  \
      BCONV_MODE(E_, TAG_, CV_, NS_, MP_, PF_, 0, "")                                                \
      BCONV_MODE(E_, TAG_, CV_, NS_, MP_, PF_, 1, ",bnb")                                            \
      BCONV_NCX(E_, TAG_, CV_, NS_, MP_, PF_)                                                        \
    }                                                                                                \
    launched = true;                                                                                 \
  }
// the NCXYZ first-layer instances (MODE 2): one channel group, prefetched halo
#define BCONV_NCX(E_, TAG_, CV_, NS_, MP_, PF_) BCONV_NCX_##CV_(E_, TAG_, NS_, MP_, PF_)
#define BCONV_NCX_2(E_, TAG_, NS_, MP_, PF_)
#define BCONV_NCX_4(E_, TAG_, NS_, MP_, PF_)
#define BCONV_NCX_1(E_, TAG_, NS_, MP_, PF_) BCONV_NCX1_PF##PF_(E_, TAG_, NS_, MP_)
#define BCONV_NCX1_PF0(E_, TAG_, NS_, MP_)
#define BCONV_NCX1_PF4(E_, TAG_, NS_, MP_) BCONV_MODE(E_, TAG_, 1, NS_, MP_, 4, 2, ",ncx")
#define BCONV_NCX1_PF8(E_, TAG_, NS_, MP_) BCONV_MODE(E_, TAG_, 1, NS_, MP_, 8, 2, ",ncx")
#define BCONV_NCX1_PF12(E_, TAG_, NS_, MP_) BCONV_MODE(E_, TAG_, 1, NS_, MP_, 12, 2, ",ncx")
#define BCONV_PF(E_, TAG_, CV_, NS_, MP_)                                               \
  BCONV_CASE(E_, TAG_, CV_, NS_, MP_, 0) else BCONV_CASE(E_, TAG_, CV_, NS_, MP_, 4) else \
  BCONV_CASE(E_, TAG_, CV_, NS_, MP_, 8) else BCONV_CASE(E_, TAG_, CV_, NS_, MP_, 12)
#define BCONV_MP(E_, TAG_, CV_, NS_)                                              \
  BCONV_PF(E_, TAG_, CV_, NS_, 1) else BCONV_PF(E_, TAG_, CV_, NS_, 2) else       \
  BCONV_PF(E_, TAG_, CV_, NS_, 4)
#define BCONV_NS(E_, TAG_, CV_)                                                          \
  BCONV_MP(E_, TAG_, CV_, 1) else BCONV_MP(E_, TAG_, CV_, 2) else BCONV_MP(E_, TAG_, CV_, 4)

// The planned variant's instances of one channel-group width CV, one
// translation unit per (element type, CV): bconv_launch_cv<E, CV>.
template <class E, int CV>
bool bconv_launch_cv(const GConvArgs &a, hipStream_t s, const dim3 &grid, double fl, double by);
template <> bool bconv_launch_cv<float, 1>(const GConvArgs &, hipStream_t, const dim3 &, double, double);
template <> bool bconv_launch_cv<float, 2>(const GConvArgs &, hipStream_t, const dim3 &, double, double);
template <> bool bconv_launch_cv<float, 4>(const GConvArgs &, hipStream_t, const dim3 &, double, double);
template <> bool bconv_launch_cv<uint16_t, 1>(const GConvArgs &, hipStream_t, const dim3 &, double, double);
template <> bool bconv_launch_cv<uint16_t, 2>(const GConvArgs &, hipStream_t, const dim3 &, double, double);
template <> bool bconv_launch_cv<uint16_t, 4>(const GConvArgs &, hipStream_t, const dim3 &, double, double);
#define BCONV_CV_BODY(E_, TAG_, CV_)                                                                 \
  const int mode = a.bn_y ? 1 : a.in_fmt ? 2 : 0;                                                    \
  bool launched = false;                                                                             \
  BCONV_NS(E_, TAG_, CV_)                                                                            \
  return launched;

// Launch of the planned variant (+ the K-split reduce) for element type E.
#define BCONV_LAUNCH_BODY(E_, TAG_)                                                                  \
  const dim3 grid(a.gridx, a.CoutW / (a.NSUB * 16), a.ksplit);                                       \
  if (a.in_fmt && (a.CK != BElem<E_>::VEC || a.NPF == 0 || a.bn_y || a.in_scale || a.ksplit > 1 ||    \
                   a.nph > 1 || a.in_c < 1 || a.in_c > 4))                                            \
    return fail(4, "bconv: NCXYZ input needs a first-layer forward (one channel group, prefetched)"); \
  if (grid.y > 65535 || grid.z > 65535) return fail(4, "bconv: grid too large");                     \
  if (a.ksplit > 1 && !a.partial) return fail(5, "bconv: K split needs a partial workspace");        \
  const double fl = a.flops > 0 ? a.flops                                                            \
                                : 2.0 * a.B * a.OX * a.OY * a.OZ * (double)a.Cout * a.nph * a.KX *   \
                                      a.KY * a.KZ * a.ICs;                                           \
  const double by = (double)sizeof(E_) * ((double)a.B * a.IX * a.IY * a.IZ * a.ICs +                 \
                                          (double)a.B * a.SX * a.SY * a.SZ * a.OCs);                 \
  const int cv = a.CK / BElem<E_>::VEC;                                                              \
  bool launched = false;                                                                             \
  if (cv == 1) launched = bconv_launch_cv<E_, 1>(a, s, grid, fl, by);                                \
  else if (cv == 2) launched = bconv_launch_cv<E_, 2>(a, s, grid, fl, by);                           \
  else if (cv == 4) launched = bconv_launch_cv<E_, 4>(a, s, grid, fl, by);                           \
  if (!launched) return fail(4, "bconv: unsupported variant");                                       \
  HCU_CHECK_LAUNCH();                                                                                \
  if (a.ksplit > 1) {                                                                                \
    const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;                                          \
    const int vpb = bconv_reduce_vpb(a);                                                             \
    const int blocks = (int)((nvox + vpb - 1) / vpb);                                                \
    HCU_TIMED(s, "bconv_reduce_kernel<" TAG_ ">", 0.0, (4.0 * a.ksplit + 2.0) * a.slice_floats,      \
              HCU_LAUNCH(bconv_reduce_kernel<E_>, dim3(blocks), dim3(256), 0, s, a, vpb));   \
    HCU_CHECK_LAUNCH();                                                                              \
  }                                                                                                  \
  return 0;

}  // namespace hcu
