// Implicit-GEMM convolution for layers with at most 8 output channels, on the
// 16-block fp32 MFMA v_mfma_f32_4x4x1_16b_f32.
//
// The 16x16x4 form pads an 8-channel N to 16, so half of its work is zeros on
// the 8-channel level of the U-Net (the 256x256 level: the largest tensors of
// the step).  Here block b of one instruction is (voxel group vg = b & 7,
// channel group cg = b >> 3): one instruction covers 32 voxels x 8 channels x
// one K element with no padding, at the same FLOP rate (tools/mfma_probe.hip:
// 122 TF/s vs 129 TF/s for 16x16x4 on an issue-bound loop).
//
// Lane layout (probed): A lane l feeds row l&3 of block l>>2, B lane l feeds
// column l&3 of block l>>2, result register r of lane l is (row r, column
// l&3) of block l>>2.  So lane l carries voxel l&31 of its 32-voxel group as
// A operand, output channel col = 4*(l>>5) + (l&3) as B operand, and holds the
// results of voxels 4*((l>>2)&7) + r of that group for channel col.
//
// K = (tap, input channel).  A K-step (tap t, channels 4q..4q+3) is one
// ds_read_b128 per lane from the halo image (4-channel planes [C4][HVP][4]:
// 16 consecutive voxels of a plane cover the 64 banks, conflict-free) and one
// ds_read_b128 of the packed weights [T][C4][8][4] (broadcast); component j
// feeds MFMA j.  A wave owns G groups (32*G voxels), so each weight read is
// shared by G groups: per K-step 1 + G b128 reads feed 4*G MFMAs.
//
// Persistent over output tiles (TX x TY x TZ voxels, TZ = the whole Z extent
// up to 16); BatchNorm+ReLU of the producer applied while staging the halo;
// bias, store and the BatchNorm partial statistics (one row per workgroup) in
// the epilogue, straight from the accumulators.  Stride-1 Conv3d forward and
// input gradient (hcat/unet.py:246-257 on the 8-channel level).
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#ifndef HCU_CONV8_EXP
#define HCU_CONV8_EXP 0   // measurement builds only: 1 no MFMA, 2 no output stores, 3 no halo loads,
                          // 4 second-half blocks start ~3 us late, 5 no next-tile fetch, 6 no LDS reads in the MFMA loop
#endif

namespace hcu {

#if HCU_CONV8_EXP == 7
// per-phase cycle totals of wave 0 of every block (measurement builds only):
// [0] halo -> LDS incl. the prefetch wait, [1] barrier, [2] next-halo issue,
// [3] MFMA loop, [4] epilogue, [5] tiles, [6] prologue, [7] lifetime
__device__ unsigned long long g_conv8_phase[8192 * 8];
#define C8_MARK(k)                                                 \
  do {                                                             \
    const long long t__ = (long long)__builtin_readcyclecounter(); \
    ph[k] += t__ - ph_t;                                           \
    ph_t = t__;                                                    \
  } while (0)
#else
#define C8_MARK(k) \
  do {             \
  } while (0)
#endif

bool conv8_disabled() {   // HCU_NO_CONV8=1 keeps the 16x16x4 kernels (A/B testing)
  static const bool off = [] {
    const char *e = getenv("HCU_NO_CONV8");
    return e && e[0] == '1';
  }();
  return off;
}

// BNB: input gradient with the fused BatchNorm backward (a.bn_y set); a
// template parameter so its loads never share registers or waits with the
// forward epilogue.  INX (C4 == 1, forward): 0 = channels-last input; 1 / 2 /
// 3 = the network input in its NCXYZ layout, fp32 / fp16 / bf16 (GConvArgs::
// in_fmt): each halo element gathers its 4 channels from the channel planes
// (consecutive lanes hold consecutive z, then y: 64 lanes read one contiguous
// run of a plane), converts them to fp32 while writing the halo image, and
// stores the channels-last copy of the voxels its tile owns (a.xcl); its
// weights are the PyTorch-layout [Cout][in_c][T] (groups 1), not the packed
// image.  Launch constants used in the tile loop are read from an
// LDS copy of the arguments (kuni, common.h), so they do not pin scalar
// registers for the whole kernel.
template <int C4, int G, int NPF, bool BNB, int INX>
__global__ void __launch_bounds__(256, 2) conv8_kernel(const GConvArgs a) {
  static_assert(INX == 0 || (C4 == 1 && !BNB), "NCXYZ input: first-layer forward only");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ __attribute__((aligned(16))) char sa_raw[sizeof(GConvArgs)];
  GConvArgs &sa = *reinterpret_cast<GConvArgs *>(sa_raw);
#define KA(f) kuni(sa.f)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if HCU_CONV8_EXP == 7
  long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long ph_start = (long long)__builtin_readcyclecounter();
  long long ph_t = ph_start;
#endif
  if (tid == 0) sa = a;
  const int T = a.KX * a.KY * a.KZ;
  const int HZ = a.HZ, HYZ = a.HY * a.HZ, HV = a.HX * HYZ, HVP = a.HVP;
  const int MT = a.TX * a.TY * a.MZ;   // M rows: z stride MZ (>= TZ; rows with lz >= TZ are idle)
  float *alds = smem;                                            // [C4][HVP][4]
  float *wlds = smem + (size_t)C4 * HVP * 4;                     // [T][C4][8][4]
  int *toffs = reinterpret_cast<int *>(wlds + T * C4 * 32);      // [T] float offsets
  int *rowoff = toffs + T;                                       // [128*G] store offsets, -1 past MT
  int *rowpk = rowoff + 128 * G;                                  // [128*G] packed (lx,ly,lz)
  float *pivl = reinterpret_cast<float *>(rowpk + 128 * G);       // [8] statistics pivot
  float *epil = pivl + 8;   // [5][8] bias, BatchNorm scale, shift, mean, invstd (epilogue)
  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;

  if constexpr (INX > 0) {
    // the first layer reads the PyTorch-layout weights [Cout][in_c][T]
    // (groups == 1) itself, so it does not wait for the packed images
    for (int i = tid; i < T * 32; i += 256) {
      const int t = i >> 5, col = (i >> 2) & 7, j = i & 3;
      wlds[i] = (col < a.Cout && j < a.in_c) ? a.w[((size_t)col * a.in_c + j) * T + t] : 0.f;
    }
  } else {
    for (int i = tid; i < T * C4 * 8; i += 256)
      reinterpret_cast<float4 *>(wlds)[i] = reinterpret_cast<const float4 *>(a.w)[i];
  }
  for (int m = tid; m < 128 * G; m += 256) {
    int q, lz, lx, ly;
    a.fTZ.divmod(m, q, lz);
    a.fTY.divmod(q, lx, ly);
    const bool valid = m < MT && lz < a.TZ;
    rowoff[m] = valid ? ((lx * a.SY + ly) * a.SZ + lz) * a.OCs : -1;
    rowpk[m] = valid ? (lx << 20) | (ly << 10) | lz : (1023 << 20);
  }
  // A rows of this lane: voxel (wave*G + g)*32 + (lane & 31) of the tile
  int vb[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int m = (wave * G + g) * 32 + (lane & 31);
    int v = 0;
    if (m < MT) {
      int q, lz, lx, ly;
      a.fTZ.divmod(m, q, lz);
      a.fTY.divmod(q, lx, ly);
      v = lx * HYZ + ly * HZ + lz;
    }
    vb[g] = v * 4;
  }
  // weight column (B operand) of this lane, and the output channels its
  // accumulators hold: with the weights as the MFMA's first operand, result
  // register r of lane l is channel 4*(l >> 5) + r of voxel l & 31 of the
  // group, so a lane stores its voxel's 4 channels as one 16-byte vector
  const int col = ((lane >> 5) << 2) | (lane & 3);
  const int wcol = col * 4;
  const int h = lane >> 5;   // channels 4h .. 4h+3
  const bool hstore = 4 * h < a.OCs;
  const int ncs = a.Cout - 4 * h;   // channel 4h + r is real when r < ncs
  if (tid < 40) {
    const int k = tid >> 3, c = tid & 7;
    const bool real = c < a.Cout;
    const float *src = k == 0 ? a.bias : k == 1 ? a.bn_scale : k == 2 ? a.bn_shift : k == 3 ? a.bn_mean : a.bn_invstd;
    epil[tid] = (real && src && (k == 0 || BNB)) ? src[c] : 0.f;
  }
  // forward statistics about a block-wide pivot per channel (the value of the
  // block's first output voxel; StatRow in common.h)
  const bool fwdstat = a.stats && !BNB;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  float cnt = 0.f;
  bool have_piv = false;
  const bool act = a.in_scale != nullptr;
  const int S = T * C4;

  // Tap offsets (floats): lane t holds tap t's (T <= 64), read with
  // v_readlane -- no LDS round trip ahead of each K-step's fragment reads.
  int toff_lane = 0;
  if (lane < T) {
    const int kz = lane % a.KZ, q = lane / a.KZ, ky = q % a.KY, kx = q / a.KY;
    toff_lane = (kx * a.dx * HYZ + ky * a.dy * HZ + kz * a.dz) * 4;
  }
  auto load = [&](int s, floatx4 &bw, floatx4 (&av)[G]) {
    const int t = s / C4, q = s - t * C4;
    bw = *reinterpret_cast<const floatx4 *>(wlds + s * 32 + wcol);
    const float *ap = alds + (size_t)q * HVP * 4 + __builtin_amdgcn_readlane(toff_lane, t);
#pragma unroll
    for (int g = 0; g < G; ++g) av[g] = *reinterpret_cast<const floatx4 *>(ap + vb[g]);
  };

  // Halo staging: thread tid always handles elements idx = tid + u*256 (channel
  // quad idx % C4 of halo voxel idx / C4); their halo coordinates are the same
  // for every tile, so they are decoded once.  The next tile's elements are
  // loaded into registers while the current tile's MFMAs run.
  int hpk[NPF];
#pragma unroll
  for (int u = 0; u < NPF; ++u) {
    const int idx = tid + u * 256;
    hpk[u] = -1;
    if (idx < HV * C4) {
      const int v = idx / C4;
      int t2, hz, hx, hy;
      a.fHZ.divmod(v, t2, hz);
      a.fHY.divmod(t2, hx, hy);
      hpk[u] = (hx << 20) | (hy << 10) | hz;
    }
  }
  const int cq = (tid % C4) * 4;   // idx % C4 == tid % C4 since 256 % C4 == 0
  const float4 sc = act ? *reinterpret_cast<const float4 *>(a.in_scale + cq)
                        : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 sh = act ? *reinterpret_cast<const float4 *>(a.in_shift + cq)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
  const float relu_lo = act ? 0.f : -INFINITY;
  // Halo loads go through a buffer descriptor of the tile's batch sample: an
  // element outside the input gets an out-of-range offset, which the hardware
  // range check turns into 0 (no branch per element); BatchNorm+ReLU is
  // applied when the element is written to LDS, selected to 0 outside.
  floatx4 pf[NPF];
  uint32_t okbits = 0;
  // NCXYZ input (INX > 0): the raw loaded values (fp32 bits, or a 16-bit
  // value in the low half), converted when the halo image is written
  auto cvt = [&](float raw) -> float {
    if constexpr (INX == 2) return (float)__builtin_bit_cast(_Float16, (uint16_t)__float_as_uint(raw));
    if constexpr (INX == 3) return __uint_as_float(__float_as_uint(raw) << 16);
    return raw;
  };
  auto tile_origin = [&](int tile, int &b, int &ox0, int &oy0, int &oz0) {
    int r, tzi, tyi, txi;
    sa.fNT.uni().divmod(tile, b, r);
    sa.fNTZ.uni().divmod(r, r, tzi);
    sa.fNTY.uni().divmod(r, txi, tyi);
    ox0 = txi * KA(TX);
    oy0 = tyi * KA(TY);
    oz0 = tzi * KA(TZ);
  };
  // branch-free: invalid elements read an offset past the buffer (-> 0)
  auto fetch = [&](int tile, bool valid) {
    int b, ox0, oy0, oz0;
    tile_origin(tile, b, ox0, oy0, oz0);
    if constexpr (INX > 0) {
      constexpr int ES = INX == 1 ? 4 : 2;
      const int IX = KA(IX), IY = KA(IY), IZ = KA(IZ), HZr = KA(HZr), INC = KA(in_c);
      const int plane = IX * IY * IZ;
      const char *bp = reinterpret_cast<const char *>(KA(in)) + (size_t)b * INC * plane * ES;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, INC * plane * ES, 0x00020000);
      const int gx0 = ox0 - KA(px), gy0 = oy0 - KA(py), gz0 = oz0 - KA(pz);
      okbits = 0;
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int hp = hpk[u];
        const int gx = gx0 + (hp >> 20), gy = gy0 + ((hp >> 10) & 1023), gz = gz0 + (hp & 1023);
        const bool ok = valid & (hp >= 0) & ((hp & 1023) < HZr) & ((unsigned)gx < (unsigned)IX) &
                        ((unsigned)gy < (unsigned)IY) & ((unsigned)gz < (unsigned)IZ);
        const int vo = (gx * IY + gy) * IZ + gz;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int off = (ok && c < INC) ? (c * plane + vo) * ES : 0x7ffffff0;
          if constexpr (INX == 1)
            pf[u][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
          else
            pf[u][c] = __uint_as_float((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0));
        }
        okbits |= (uint32_t)ok << u;
      }
      return;
    }
    const int IX = KA(IX), IY = KA(IY), IZ = KA(IZ), ICs = KA(ICs), HZr = KA(HZr);
    const uint32_t bZ = (uint32_t)ICs * 4, bY = (uint32_t)IZ * bZ, bX = (uint32_t)IY * bY;
    const int gx0 = ox0 - KA(px), gy0 = oy0 - KA(py), gz0 = oz0 - KA(pz);
    const float *bp = KA(in) + (size_t)b * IX * bX / 4;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)bp, 0, IX * (int)bX, 0x00020000);
    const int base_off = gx0 * (int)bX + gy0 * (int)bY + gz0 * (int)bZ + cq * 4;
    okbits = 0;
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int hp = hpk[u];
      const int hx = hp >> 20, hy = (hp >> 10) & 1023, hz = hp & 1023;
      const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
      const bool ok = valid & (hp >= 0) & (hz < HZr) & ((unsigned)gx < (unsigned)IX) &
                      ((unsigned)gy < (unsigned)IY) & ((unsigned)gz < (unsigned)IZ);
      const int off = ok ? base_off + (int)(__umul24(hx, bX) + __umul24(hy, bY) + __umul24(hz, bZ))
                         : 0x7ffffff0;
      if (HCU_CONV8_EXP == 3)
        pf[u] = floatx4{(float)off, 0.f, 0.f, 0.f};
      else
        pf[u] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      okbits |= (uint32_t)ok << u;
    }
  };
  // The halo image of a tile from the prefetched registers (a tile index past
  // the block's range was fetched with every element invalid: zeros)
  auto stage = [&](float *dst, int tile) {
    int b, ox0, oy0, oz0;
    tile_origin(tile, b, ox0, oy0, oz0);
    // (NCXYZ input) the input voxels this tile owns in the channels-last copy:
    // its output tile's x / y / z range, plus the kernel's overhang on the
    // grid's last tile of each axis
    const bool lastx = ox0 + KA(TX) >= KA(OX), lasty = oy0 + KA(TY) >= KA(OY), lastz = oz0 + KA(TZ) >= KA(OZ);
    float *const xclp = INX > 0 ? KA(xcl) : nullptr;
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int idx = tid + u * 256;
      floatx4 v = pf[u];
      if constexpr (INX > 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = cvt(v[c]);
        const int hp = hpk[u];
        const int hx = hp >> 20, hy = (hp >> 10) & 1023, hz = hp & 1023;
        if (xclp && ((okbits >> u) & 1u) && (hx < KA(TX) || lastx) && (hy < KA(TY) || lasty) &&
            (hz < KA(TZ) || lastz)) {
          const int IY = KA(IY), IZ = KA(IZ);
          const size_t vox = (((size_t)b * KA(IX) + ox0 - KA(px) + hx) * IY + oy0 - KA(py) + hy) * IZ + oz0 - KA(pz) + hz;
          *reinterpret_cast<floatx4 *>(xclp + vox * 4) = v;
        }
      }
      // BatchNorm+ReLU, branch-free (no input BatchNorm: scale 1, shift 0,
      // floor -inf)
      v[0] = fmaxf(fmaf(v[0], sc.x, sh.x), relu_lo);
      v[1] = fmaxf(fmaf(v[1], sc.y, sh.y), relu_lo);
      v[2] = fmaxf(fmaf(v[2], sc.z, sh.z), relu_lo);
      v[3] = fmaxf(fmaf(v[3], sc.w, sh.w), relu_lo);
      const bool ok = (okbits >> u) & 1u;
      const floatx4 z = {0.f, 0.f, 0.f, 0.f};
      // elements past the halo write the unused last slot of the last plane
      const int slot = hpk[u] >= 0 ? (idx % C4) * HVP + idx / C4 : C4 * HVP - 1;
      *reinterpret_cast<floatx4 *>(dst + (size_t)slot * 4) = ok ? v : z;
    }
  };
  lds_barrier();   // sa and the tables are in LDS
  // contiguous tile range per block (consecutive tiles share halo rows in L2)
  const int tpb_ = (total + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t_beg = blockIdx.x * tpb_, t_end = min(total, t_beg + tpb_);
  if (t_beg < t_end) fetch(t_beg, true);
  // The epilogue issues G stores after the next tile's halo loads; where the
  // path into the halo wait has no epilogue (the first tile) as many stores go
  // to an empty buffer (dropped), so the compiler's wait for each prefetched
  // element never includes output stores.
  {
    const __amdgpu_buffer_rsrc_t zr = __builtin_amdgcn_make_buffer_rsrc((void *)a.in, 0, 0, 0x00020000);
#pragma unroll
    for (int k = 0; k < G; ++k) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, zr, 256 * k, 0, 0);
  }
  C8_MARK(6);

  for (int tile = t_beg; tile < t_end; ++tile) {
    int b, ox0, oy0, oz0;
    tile_origin(tile, b, ox0, oy0, oz0);
    // output row offsets of this tile
    const int OX = KA(OX), OY = KA(OY), OZ = KA(OZ), OCs = KA(OCs), SY = KA(SY), SZ = KA(SZ);
    const int sample = KA(SX) * SY * SZ * OCs;
    const int tbase = (((ox0 * SY + oy0) * SZ + oz0) * OCs + 4 * h) * 4;
    const bool interior = ox0 + KA(TX) <= OX && oy0 + KA(TY) <= OY && oz0 + KA(TZ) <= OZ;
    int ro[G];
    const int mb = wave * G * 32 + (lane & 31);
#pragma unroll
    for (int g = 0; g < G; ++g) ro[g] = rowoff[mb + g * 32];
    if (!interior) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int pk = rowpk[mb + g * 32];
        const bool in = (ox0 + (pk >> 20) < OX) & (oy0 + ((pk >> 10) & 1023) < OY) & (oz0 + (pk & 1023) < OZ);
        ro[g] = in ? ro[g] : -1;
      }
    }
    C8_MARK(0);
    lds_barrier();   // the previous tile's MFMAs are done with the halo image
    stage(alds, tile);
    lds_barrier();
    if (HCU_CONV8_EXP != 5 && tile + 1 < t_end) fetch(tile + 1, true);
    C8_MARK(1);
    // ---- MFMA over the K-steps, next step's fragments loaded ahead
    floatx4 acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto mf = [&](int c, float w, float x, int g) {
      acc[g] = __builtin_amdgcn_mfma_f32_4x4x1f32(w, x, acc[g], 0, 0, 0);
    };
    floatx4 b0, b1, a0[G], a1[G];
    load(0, b0, a0);
    for (int s = 0; s < (HCU_CONV8_EXP == 1 ? 0 : S); s += 2) {
      if (HCU_CONV8_EXP == 6) {
        b1 = b0;
#pragma unroll
        for (int g = 0; g < G; ++g) a1[g] = a0[g];
      } else
      load(min(s + 1, S - 1), b1, a1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int g = 0; g < G; ++g)
          mf(c, b0[c], a0[g][c], g);
      if (HCU_CONV8_EXP != 6) load(min(s + 2, S - 1), b0, a0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < S) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int g = 0; g < G; ++g)
            mf(c, b1[c], a1[g][c], g);
      }
    }
    C8_MARK(3);
    // ---- epilogue: bias, store (per-sample buffer, 32-bit offsets), BatchNorm
    // partial statistics
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(KA(out) + (size_t)b * sample), 0, sample * 4, 0x00020000);
    const floatx4 bias = *reinterpret_cast<const floatx4 *>(epil + 4 * h);
    if (fwdstat && !have_piv) {   // block-uniform: the first tile of this block
      if (wave == 0 && (lane & 31) == 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) pivl[4 * h + r] = acc[0][r] + bias[r];
      lds_barrier();
      have_piv = true;
    }
    const floatx4 piv = fwdstat ? *reinterpret_cast<const floatx4 *>(pivl + 4 * h) : floatx4{0.f, 0.f, 0.f, 0.f};
    // fused BatchNorm+ReLU backward: the layer's output y of the same voxels
    // (loaded after the MFMAs: the next halo's loads, issued before them, have
    // landed by then, so waiting for y costs nothing extra)
    floatx4 yv[G];
    floatx4 bnsc, bnsh, bnmu, bnis;
    if constexpr (BNB) {
      const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(KA(bn_y) + (size_t)b * sample), 0, sample * 4, 0x00020000);
#pragma unroll
      for (int g = 0; g < G; ++g)
        yv[g] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                yrs, ro[g] >= 0 ? tbase + ro[g] * 4 : 0x7ffffff0, 0, 0));
      bnsc = *reinterpret_cast<const floatx4 *>(epil + 8 + 4 * h);
      bnsh = *reinterpret_cast<const floatx4 *>(epil + 16 + 4 * h);
      bnmu = *reinterpret_cast<const floatx4 *>(epil + 24 + 4 * h);
      bnis = *reinterpret_cast<const floatx4 *>(epil + 32 + 4 * h);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int o = ro[g];
      floatx4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[g][r] + bias[r];
        float w1 = x - piv[r], w2 = x - piv[r];
        if (BNB) {   // v = dA -> dz, stats (dz, dz*xhat)
          x = fmaf(yv[g][r], bnsc[r], bnsh[r]) > 0.f ? x : 0.f;
          w1 = x;
          w2 = (yv[g][r] - bnmu[r]) * bnis[r];
        }
        v[r] = x;
        const float w = (o >= 0 && r < ncs) ? w1 : 0.f;
        s1[r] += w;
        s2[r] = fmaf(w, w2, s2[r]);
      }
      cnt += o >= 0 ? 1.f : 0.f;
      if (HCU_CONV8_EXP != 2 || v[0] == 1234.5f)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ors,
                                               (o >= 0 && hstore) ? tbase + o * 4 : 0x7ffffff0, 0, 0);
    }
    C8_MARK(4);
#if HCU_CONV8_EXP == 7
    ph[5] += 1;
#endif
  }
#if HCU_CONV8_EXP == 7
  if (tid == 0) {
    unsigned long long *d = g_conv8_phase + (size_t)(blockIdx.x % 8192) * 8;
    for (int k = 0; k < 7; ++k) d[k] += (unsigned long long)ph[k];
    d[7] += (unsigned long long)((long long)__builtin_readcyclecounter() - ph_start);
  }
#endif
  if (!a.stats) return;
  // lanes sharing channels (the 32 voxels of a half): fixed-order butterfly
#pragma unroll
  for (int m = 1; m < 32; m <<= 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[r] += __shfl_xor(s1[r], m);
      s2[r] += __shfl_xor(s2[r], m);
    }
    cnt += __shfl_xor(cnt, m);
  }
  lds_barrier();
  float *red = smem;  // [4 waves][8 channels][3]
  if ((lane & 31) == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * h + r;
      red[(wave * 8 + c) * 3 + 0] = s1[r];
      red[(wave * 8 + c) * 3 + 1] = s2[r];
      red[(wave * 8 + c) * 3 + 2] = r < ncs ? cnt : 0.f;
    }
  lds_barrier();
  if (tid < 8) {
    float t1 = 0.f, t2 = 0.f, tn = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      t1 += red[(w * 8 + tid) * 3 + 0];
      t2 += red[(w * 8 + tid) * 3 + 1];
      tn += red[(w * 8 + tid) * 3 + 2];
    }
    if (fwdstat) {
      *reinterpret_cast<float4 *>(a.stats + ((size_t)blockIdx.x * 8 + tid) * 4) =
          make_float4(t1, t2, pivl[tid], tn);
    } else {
      a.stats[((size_t)blockIdx.x * 8 + tid) * 2 + 0] = t1;
      a.stats[((size_t)blockIdx.x * 8 + tid) * 2 + 1] = t2;
    }
  }
#undef KA
}

// ---------------------------------------------------------------------------
static long conv8_lds(const GConvArgs &a, int C4, int HVP, int G) {
  const int T = a.KX * a.KY * a.KZ;
  return ((long)C4 * HVP * 4 + (long)T * C4 * 32 + T + 2L * 128 * G + 8 + 40) * 4 +
         (long)sizeof(GConvArgs);   // + the static copy of the arguments
}

// HCU_CONV8_NPF: the prefetch limit (elements per thread) at G <= 4.  12 by
// default: config 2's d1.c1 input gradient then takes G = 2 with 12 prefetched
// elements, 63.9 us, against G = 4 with 16 at 69.6 us (round 5's limit 16;
// config 2, 5 interleaved runs each: 1.919-1.929 vs 1.925-1.941 ms/step)
static int env_npf_max() {
  const char *e = getenv("HCU_CONV8_NPF");
  const int v = e ? atoi(e) : 12;
  return v == 16 ? 16 : 12;
}

// Chooses the tile, groups per wave and grid for conv8_kernel; non-zero when
// the shape is not one conv8 handles (the caller then plans conv2 / gconv).
int plan_conv8(GConvArgs &a, int target_blocks) {
  a.use_conv8 = 0;
  if (conv8_disabled()) return 1;
  if (a.nph > 1 || a.sx != 1 || a.sy != 1 || a.sz != 1) return 1;
  if (a.osx != 1 || a.osy != 1 || a.osz != 1 || a.ofx || a.ofy || a.ofz) return 1;
  if (a.Cout > 8 || a.OCs > 8 || a.ICs % 4 || a.KX * a.KY * a.KZ > 64) return 1;
  const int C4 = a.ICs / 4;
  if (C4 != 1 && C4 != 2 && C4 != 4) return 1;
  if (a.OX <= 0 || a.OY <= 0 || a.OZ <= 0) return 2;
  const int ntz = cdiv(a.OZ, 16);
  const int TZ = cdiv(a.OZ, ntz);
  const int HZr = TZ + (a.KZ - 1) * a.dz;
  // M rows with a z stride of 16 and a halo z stride of 16: the 16 lanes of a
  // ds_read_b128 lane group then read 16 different banks (a z stride of 15
  // puts two lanes of a group on one bank).  Only when it wastes <= 1/8.
  const bool pad16 = false;  // measured slower (NPF grows); kept for reference: TZ >= 14 && HZr <= 16
  const int MZ = pad16 ? 16 : TZ, HZS = pad16 ? 16 : HZr;
  const int gs[3] = {8, 4, 2};
  bool found = false;
  for (int gi = 0; gi < 3; ++gi) {
    const int G = gs[gi];
    const int txy = std::max(1, 128 * G / MZ);
    int TX = std::max(1, (int)std::floor(std::sqrt((double)txy)));
    int TY = std::max(1, txy / TX);
    TX = std::min(TX, a.OX);
    TY = std::min(TY, a.OY);
    const int HX = TX + (a.KX - 1) * a.dx, HY = TY + (a.KY - 1) * a.dy;
    const int HV = HX * HY * HZS;
    const int HVP = round_up(HV, 16) + 8;
    const long lds = conv8_lds(a, C4, HVP, G);
    const long tiles = (long)a.B * cdiv(a.OX, TX) * cdiv(a.OY, TY) * ntz;
    // two workgroups per CU; <= 12 prefetched elements per thread at G = 8
    // (16 spills registers there); at G <= 4 the limit of env_npf_max()
    static const int npf_max = env_npf_max();
    if (lds > 80 * 1024 || HV * C4 > (G <= 4 ? npf_max : 12) * 256) continue;
    a.G8 = G;
    a.TX = TX;
    a.TY = TY;
    a.TZ = TZ;
    a.MZ = MZ;
    a.HX = HX;
    a.HY = HY;
    a.HZ = HZS;
    a.HZr = HZr;
    a.HVP = HVP;
    a.NPF = HV * C4 <= 8 * 256 ? 8 : (HV * C4 <= 12 * 256 ? 12 : 16);
    a.lds_bytes = (int)std::max(lds, 4L * 8 * 3 * 4);
    found = true;
    if (tiles >= target_blocks / 2) break;
  }
  if (!found) return 4;
  a.ntx = cdiv(a.OX, a.TX);
  a.nty = cdiv(a.OY, a.TY);
  a.ntz = ntz;
  a.CK = a.ICs;
  a.CoutW = 8;
  a.NSUB = 1;
  a.MPW = 1;
  a.ksplit = 1;
  a.cps = 1;
  a.slice_floats = 0;
  a.fHZ = FastDiv(a.HZ);
  a.fHY = FastDiv(a.HY);
  a.fTZ = FastDiv(a.MZ);   // M-row decomposition (z stride MZ)
  a.fTY = FastDiv(a.TY);
  a.fNT = FastDiv(a.ntx * a.nty * a.ntz);
  a.fNTZ = FastDiv(a.ntz);
  a.fNTY = FastDiv(a.nty);
  a.fKZ = FastDiv(a.KZ);
  a.fKY = FastDiv(a.KY);
  const long tiles = (long)a.B * a.ntx * a.nty * a.ntz;
  a.gridx = (int)std::min<long>(tiles, 512L);   // two persistent workgroups per CU
  a.use_conv8 = 1;
  a.use_conv2 = 0;
  return 0;
}

#define CONV8_CASE(C4_, G_, NPF_)                                                                \
  if (C4 == C4_ && a.G8 == G_ && a.NPF == NPF_) {                                                \
    if (a.bn_y)                                                                                  \
      HCU_TIMED(s, "conv8_kernel<" #C4_ "," #G_ "," #NPF_ ",bnb>", fl, by,                       \
                HCU_LAUNCH((conv8_kernel<C4_, G_, NPF_, true, 0>), dim3(a.gridx), dim3(256), \
                                   a.lds_bytes - (int)sizeof(GConvArgs), s, a));                 \
    else if (C4_ == 1 && a.in_fmt == 1)                                                          \
      HCU_TIMED(s, "conv8_kernel<" #C4_ "," #G_ "," #NPF_ ",ncx32>", fl, by,                     \
                HCU_LAUNCH((conv8_kernel<1, G_, NPF_, false, 1>), dim3(a.gridx), dim3(256),      \
                                   a.lds_bytes - (int)sizeof(GConvArgs), s, a));                 \
    else if (C4_ == 1 && a.in_fmt == 2)                                                          \
      HCU_TIMED(s, "conv8_kernel<" #C4_ "," #G_ "," #NPF_ ",ncx16>", fl, by,                     \
                HCU_LAUNCH((conv8_kernel<1, G_, NPF_, false, 2>), dim3(a.gridx), dim3(256),      \
                                   a.lds_bytes - (int)sizeof(GConvArgs), s, a));                 \
    else if (C4_ == 1 && a.in_fmt == 3)                                                          \
      HCU_TIMED(s, "conv8_kernel<" #C4_ "," #G_ "," #NPF_ ",ncxbf>", fl, by,                     \
                HCU_LAUNCH((conv8_kernel<1, G_, NPF_, false, 3>), dim3(a.gridx), dim3(256),      \
                                   a.lds_bytes - (int)sizeof(GConvArgs), s, a));                 \
    else                                                                                         \
      HCU_TIMED(s, "conv8_kernel<" #C4_ "," #G_ "," #NPF_ ">", fl, by,                           \
                HCU_LAUNCH((conv8_kernel<C4_, G_, NPF_, false, 0>), dim3(a.gridx), dim3(256), \
                                   a.lds_bytes - (int)sizeof(GConvArgs), s, a));                 \
    launched = true;                                                                             \
  }
#define CONV8_NPF(C4_, G_) \
  CONV8_CASE(C4_, G_, 8) else CONV8_CASE(C4_, G_, 12) else CONV8_CASE(C4_, G_, 16)

#if HCU_CONV8_EXP == 7
// the phase totals (measurement builds): sums over the blocks, then zeroed
extern "C" int hcu_debug_conv8_phases(unsigned long long *out) {
  std::vector<unsigned long long> h(8192 * 8);
  if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_conv8_phase), h.size() * 8) != hipSuccess) return 3;
  for (int k = 0; k < 8; ++k) out[k] = 0;
  for (size_t i = 0; i < h.size(); ++i) out[i % 8] += h[i];
  std::fill(h.begin(), h.end(), 0ull);
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_conv8_phase), h.data(), h.size() * 8) != hipSuccess) return 3;
  return 0;
}
#endif

int launch_conv8(const GConvArgs &a, hipStream_t s) {
  const int C4 = a.ICs / 4;
  if (a.in_fmt && (C4 != 1 || a.bn_y || a.in_scale || a.in_c < 1 || a.in_c > 4))
    return fail(4, "conv8: NCXYZ input needs a first-layer forward with <= 4 channels");
  const double fl = a.flops > 0 ? a.flops
                                : 2.0 * a.B * a.OX * a.OY * a.OZ * (double)a.Cout * a.KX * a.KY *
                                      a.KZ * a.ICs;
  const double by = 4.0 * ((double)a.B * a.IX * a.IY * a.IZ * a.ICs +
                           (double)a.B * a.SX * a.SY * a.SZ * a.OCs);
  bool launched = false;
  CONV8_NPF(1, 8) else CONV8_NPF(1, 4) else CONV8_NPF(1, 2)
  else CONV8_NPF(2, 8) else CONV8_NPF(2, 4) else CONV8_NPF(2, 2)
  else CONV8_NPF(4, 8) else CONV8_NPF(4, 4) else CONV8_NPF(4, 2)
  if (!launched) return fail(4, "conv8: unsupported variant");
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu
