// bf16 weight gradient of Conv3d / ConvTranspose3d on v_mfma_f32_16x16x32_bf16.
//
//   Conv3d (taps on the rows):  dW[(t, ci)][co] = sum_p act(A[p + off(t)][ci]) * G[p][co]
//                               (+ bias row: sum_p G[p][co])
//   ConvTranspose3d (taps on the columns): dW[ci][(t, co)] = sum_p A[p][ci] * G[p*s + t][co]
//
// The reduction runs over voxels p, so both MFMA operands need 8 consecutive
// VOXELS per lane, while activations live channels-last (8 consecutive
// channels per 16 bytes).  Instead of transposing in a staging pass, the
// channels-last tiles are staged as they come from HBM and every fragment is
// read with ds_read_b64_tr_b16: a 16-lane group reads 4 voxel rows x 16
// channel columns and each lane receives one channel of the 4 voxels.  Each
// lane supplies its own row address, so the tap shift off(t) is just a per-lane
// address offset into the A halo image (no per-tap image copies), and a row
// subtile of 16 (tap, channel) pairs may straddle two taps when a tap has fewer
// than 16 channels (first layer: 8 channel slots).
//
// Workgroup: 4 waves; the block owns a set of row subtiles (4*MSW, each wave
// MSW of them) x NSB column subtiles of dW and a strided subset of the voxel
// tiles (TX*TY*TZ voxels, TX*TY = 32 or 64 so every tile is a whole number of
// 32-voxel K-steps; voxels outside the grid are staged as zero gradient).
// Each wave keeps its own rows, so no cross-wave reduction is needed: every
// block writes one fp32 partial slab and wgrad_finalize sums the slabs in fp64
// in a fixed order (deterministic) and scatters them into the PyTorch layout.
// Replaces the weight gradients of hcat/unet.py:246-257, 294-298 under
// torch.autocast(dtype=torch.bfloat16).
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>

namespace hcu {

#ifdef HCU_BW_PHASES
// measurement builds only (tools/bw_phases.py): cycles of wave 0 of every
// block of the all-taps kernel: [0] commit (incl. the wait for the prefetched
// tile), [1] the two barriers + next-tile load issue, [2] MFMA loop, [3] tiles
__device__ unsigned long long g_bw_phase[4096 * 4];
extern "C" int hcu_debug_bw_phases(unsigned long long *out) {
  static unsigned long long h[4096 * 4];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bw_phase), sizeof h) != hipSuccess) return 3;
  for (int k = 0; k < 4; ++k) out[k] = 0;
  for (int i = 0; i < 4096 * 4; ++i) out[i % 4] += h[i];
  for (auto &x : h) x = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_bw_phase), h, sizeof h) == hipSuccess ? 0 : 3;
}
#define BW_MARK(k)                                                 \
  do {                                                             \
    const long long t__ = (long long)__builtin_readcyclecounter(); \
    bw_ph[k] += t__ - bw_t;                                        \
    bw_t = t__;                                                    \
  } while (0)
#else
#define BW_MARK(k) \
  do {             \
  } while (0)
#endif

__device__ __forceinline__ shortx4 tr_read(const uint16_t *p) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s *)(
          (__attribute__((address_space(3))) uint16_t *)(p)));
}

template <int MSW, int NS>
__global__ void __launch_bounds__(256) bwgrad_kernel(const WGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int T = a.KX * a.KY * a.KZ;
  const int CKA = a.CKA, CKG = a.CKG, RSA = a.PA2, RSG = a.PG2;
  int tapc, cic, coc;
  if (a.taps_rows) {
    tapc = blockIdx.y / a.nci;
    cic = blockIdx.y % a.nci;
    coc = blockIdx.z;
  } else {
    cic = blockIdx.y;
    tapc = blockIdx.z / a.nco;
    coc = blockIdx.z % a.nco;
  }
  const int ci0 = cic * CKA, co0 = coc * CKG;
  const int t0 = tapc * (a.taps_rows ? a.TA : a.TG);
  const bool bias_block = a.taps_rows && a.bias_row && tapc == 0 && cic == 0;
  const int HAV = a.HAV, HGV = a.HGV, PT = a.PTV;
  uint16_t *alds = reinterpret_cast<uint16_t *>(smem);          // [HAV][RSA]
  uint16_t *glds = alds + (size_t)HAV * RSA;                    // [HGV][RSG]
  int *hvA = reinterpret_cast<int *>(glds + (size_t)HGV * RSG);  // [PT] A row * RSA
  int *hvG = hvA + PT;                                           // [PT] G row * RSG
  const int HAZ = a.HAZ, HAYZ = a.HAY * a.HAZ, HGZ = a.HGZ, HGYZ = a.HGY * a.HGZ;

  for (int p = tid; p < PT; p += 256) {
    int q, lz, lx, ly;
    a.fTZ.divmod(p, q, lz);
    a.fTY.divmod(q, lx, ly);
    hvA[p] = (lx * a.asx * HAYZ + ly * a.asy * HAZ + lz * a.asz) * RSA;
    hvG[p] = (lx * a.gsx * HGYZ + ly * a.gsy * HGZ + lz * a.gsz) * RSG;
  }
  // per-lane column bases of this wave's row subtiles / the block's column
  // subtiles (tap offset folded in); rows/cols past the block's extent read a
  // valid address and are discarded at the write.
  const int rows_blk = a.taps_rows ? a.TA * CKA : CKA;
  const int cols_blk = a.taps_rows ? CKG : a.TG * CKG;
  int colA[MSW], colG[NS];
#pragma unroll
  for (int m = 0; m < MSW; ++m) {
    const int r = (wave + 4 * m) * 16 + 4 * p4;
    int off = 0;
    if (r < rows_blk) {
      if (a.taps_rows) {
        const int ta = t0 + r / CKA, c = r % CKA;
        if (ta < T) {
          const int kz = ta % a.KZ, qq = ta / a.KZ, ky = qq % a.KY, kx = qq / a.KY;
          off = (kx * a.adx * HAYZ + ky * a.ady * HAZ + kz * a.adz) * RSA + c;
        }
      } else {
        off = r;
      }
    }
    colA[m] = off;
  }
#pragma unroll
  for (int n = 0; n < NS; ++n) {
    const int c = n * 16 + 4 * p4;
    int off = 0;
    if (c < cols_blk) {
      if (a.taps_rows) {
        off = c;
      } else {
        const int tg = t0 + c / CKG, o = c % CKG;
        if (tg < T) {
          const int kz = tg % a.KZ, qq = tg / a.KZ, ky = qq % a.KY, kx = qq / a.KY;
          off = (kx * a.gdx * HGYZ + ky * a.gdy * HGZ + kz * a.gdz) * RSG + o;
        }
      }
    }
    colG[n] = off;
  }

  floatx4 acc[MSW][NS], accb[NS];
#pragma unroll
  for (int m = 0; m < MSW; ++m)
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int n = 0; n < NS; ++n) accb[n] = floatx4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = bias_block && wave == 0;
  const shortx8 ones = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};

  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int CA8 = CKA / 8, CG8 = CKG / 8;
  const bool act = a.a_scale != nullptr;
  float sc[8], sh[8];
  // activation of this thread's 8-channel A group (fixed: 256 % CA8 == 0)
  {
    const int c = ci0 + (tid % CA8) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = act ? a.a_scale[c + k] : 1.f;
      sh[k] = act ? a.a_shift[c + k] : 0.f;
    }
  }
  const uint16_t *Ab = reinterpret_cast<const uint16_t *>(a.A);
  const uint16_t *Gb = reinterpret_cast<const uint16_t *>(a.G);

  // contiguous tile range per block (consecutive tiles share halo rows in L2)
  const int KBt = (int)gridDim.x, kbi = (int)blockIdx.x;
  const int tpb_ = (total + KBt - 1) / KBt;
  const int t_end = min(total, kbi * tpb_ + tpb_);
  for (int tt = kbi * tpb_; tt < t_end; ++tt) {
    const int b = tt / ntiles;
    int tile = tt - b * ntiles;
    const int tzi = tile % a.ntz;
    tile /= a.ntz;
    const int tyi = tile % a.nty, txi = tile / a.nty;
    const int px0 = txi * a.TX, py0 = tyi * a.TY, pz0 = tzi * a.TZ;
    lds_barrier();
    {  // A halo (channels-last, activation applied, 0 outside the input)
      const int gx0 = px0 * a.asx - a.apx, gy0 = py0 * a.asy - a.apy, gz0 = pz0 * a.asz - a.apz;
      const size_t bbase = (size_t)b * a.AX * a.AY * a.AZ;
      const int c8 = tid % CA8;
      for (int v0 = tid / CA8; v0 < HAV; v0 += 4 * (256 / CA8)) {
        uint4 val[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int v = v0 + u * (256 / CA8);
          int q, hz, hx, hy;
          a.fHAZ.divmod(v, q, hz);
          a.fHAY.divmod(q, hx, hy);
          const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
          ok[u] = v < HAV && (unsigned)gx < (unsigned)a.AX && (unsigned)gy < (unsigned)a.AY &&
                  (unsigned)gz < (unsigned)a.AZ;
          val[u] = make_uint4(0u, 0u, 0u, 0u);
          if (ok[u])
            val[u] = *reinterpret_cast<const uint4 *>(
                Ab + ((bbase + ((size_t)gx * a.AY + gy) * a.AZ + gz) * a.ACs + ci0 + c8 * 8));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int v = v0 + u * (256 / CA8);
          if (v >= HAV) continue;
          uint4 w = make_uint4(0u, 0u, 0u, 0u);
          if (ok[u]) {
            if (act) {
              float f[8];
              unpack8(val[u], f);
#pragma unroll
              for (int k = 0; k < 8; ++k) f[k] = fmaxf(fmaf(f[k], sc[k], sh[k]), 0.f);
              w = pack8(f);
            } else {
              w = val[u];
            }
          }
          *reinterpret_cast<uint4 *>(alds + (size_t)v * RSA + c8 * 8) = w;
        }
      }
    }
    {  // G image (channels-last, 0 outside the gradient's grid / the output grid)
      const int gx0 = px0 * a.gsx - a.gpx, gy0 = py0 * a.gsy - a.gpy, gz0 = pz0 * a.gsz - a.gpz;
      const size_t bbase = (size_t)b * a.GX * a.GY * a.GZ;
      const int c8 = tid % CG8;
      for (int v0 = tid / CG8; v0 < HGV; v0 += 4 * (256 / CG8)) {
        uint4 val[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int v = v0 + u * (256 / CG8);
          int q, hz, hx, hy;
          a.fHGZ.divmod(v, q, hz);
          a.fHGY.divmod(q, hx, hy);
          const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
          // taps_rows: G is the output grid [PX][PY][PZ] (voxels past it are 0)
          const bool ok = v < HGV && (unsigned)gx < (unsigned)a.GX && (unsigned)gy < (unsigned)a.GY &&
                          (unsigned)gz < (unsigned)a.GZ &&
                          (!a.taps_rows || (gx < a.PX && gy < a.PY && gz < a.PZ));
          val[u] = make_uint4(0u, 0u, 0u, 0u);
          if (ok)
            val[u] = *reinterpret_cast<const uint4 *>(
                Gb + ((bbase + ((size_t)gx * a.GY + gy) * a.GZ + gz) * a.GCs + co0 + c8 * 8));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int v = v0 + u * (256 / CG8);
          if (v < HGV) *reinterpret_cast<uint4 *>(glds + (size_t)v * RSG + c8 * 8) = val[u];
        }
      }
    }
    // ConvTranspose3d: input voxels past the input grid must contribute 0; their
    // A rows are 0 (staged as outside), so nothing else is needed.
    lds_barrier();
    for (int p0 = 0; p0 < PT; p0 += 32) {
      // voxel rows of this lane's 8 K elements: rows 4g+q4 and 16+4g+q4 of
      // the 32-voxel step (the same order for both operands), so the 32 lanes
      // of each ds_read_b64_tr_b16 bank group read 8 consecutive rows
      const int pr = p0 + 4 * g + q4;
      const int ra0 = hvA[pr], ra1 = hvA[pr + 16];
      const int rg0 = hvG[pr], rg1 = hvG[pr + 16];
      shortx8 bf[NS];
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        const shortx4 lo = tr_read(glds + rg0 + colG[n]);
        const shortx4 hi = tr_read(glds + rg1 + colG[n]);
        bf[n] = shortx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int m = 0; m < MSW; ++m) {
        const shortx4 lo = tr_read(alds + ra0 + colA[m]);
        const shortx4 hi = tr_read(alds + ra1 + colA[m]);
        const shortx8 af = shortx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int n = 0; n < NS; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[n], acc[m][n], 0, 0, 0);
      }
      if (do_bias) {
#pragma unroll
        for (int n = 0; n < NS; ++n)
          accb[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bf[n], accb[n], 0, 0, 0);
      }
    }
  }

  // ---- one partial slab per block: each wave writes its own rows
  const size_t slab = (size_t)blockIdx.x * a.Mtot;
  // taps_rows slab rows (tap, real channel) and columns (real channels):
  // WGradArgs::ACr / GCr, the padding slots of the channel strides not stored
  const int ACR = a.ACr > 0 ? a.ACr : a.ACs, GCR = a.GCr > 0 ? a.GCr : a.GCs;
#pragma unroll
  for (int m = 0; m < MSW; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = (wave + 4 * m) * 16 + g * 4 + r;
      int grow = -1;
      if (lr < rows_blk) {
        if (a.taps_rows) {
          const int ta = t0 + lr / CKA, ci = ci0 + lr % CKA;
          if (ta < T && ci < ACR) grow = ta * ACR + ci;
        } else if (ci0 + lr < a.ACs) {
          grow = ci0 + lr;
        }
      }
      if (grow < 0) continue;
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        const int lc = n * 16 + (lane & 15);
        int gcol = -1;
        if (lc < cols_blk) {
          if (a.taps_rows) {
            if (co0 + lc < GCR) gcol = co0 + lc;
          } else {
            const int tg = t0 + lc / CKG, o = co0 + lc % CKG;
            if (tg < T && o < a.GCs) gcol = tg * a.GCs + o;
          }
        }
        if (gcol >= 0) a.partial[(slab + grow) * a.Ntot + gcol] = acc[m][n][r];
      }
    }
  }
  if (do_bias && g == 0) {   // row 0 of the ones-subtile holds sum_p G[p][col]
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const int lc = n * 16 + (lane & 15);
      if (lc < CKG && co0 + lc < GCR)
        a.partial[(slab + (size_t)T * ACR) * a.Ntot + co0 + lc] = accb[n][0];
    }
  }
}

// ---------------------------------------------------------------------------
// Pipelined form of bwgrad_kernel (same blocks, tiles, MFMA sequence and slab
// layout, so the same sums in the same order): each thread keeps its share of
// the NEXT tile's A halo and G image in registers -- NP 16-byte loads each,
// issued right after the current tile is committed to LDS -- so the loads are
// in flight while the current tile's MFMAs run, and a tile costs two LDS-only
// barriers.  The halo coordinates of every register slot are tile-independent
// and decoded once.
template <int MSW, int NS, int NPA, int NPG>
__global__ void __launch_bounds__(256) bwgrad_pipe_kernel(const WGradArgs a) {
  static_assert(MSW < 16 || NS == 1, "the all-taps form has one column subtile");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int T = a.KX * a.KY * a.KZ;
  const int CKA = a.CKA, CKG = a.CKG, RSA = a.PA2, RSG = a.PG2;
  int tapc, cic, coc;
  if (a.taps_rows) {
    tapc = blockIdx.y / a.nci;
    cic = blockIdx.y % a.nci;
    coc = blockIdx.z;
  } else {
    cic = blockIdx.y;
    tapc = blockIdx.z / a.nco;
    coc = blockIdx.z % a.nco;
  }
  const int ci0 = cic * CKA, co0 = coc * CKG;
  const int t0 = tapc * (a.taps_rows ? a.TA : a.TG);
  const bool bias_block = a.taps_rows && a.bias_row && tapc == 0 && cic == 0;
  const int HAV = a.HAV, HGV = a.HGV, PT = a.PTV;
  // the A image keeps HAZP >= HAZ rows per (hx, hy) column (plan_bwgrad_cka:
  // the all-taps form pads them so 8 consecutive tile voxels land on 8
  // different bank groups)
  const int HAZ = a.HAZP, HAYZ = a.HAY * a.HAZP, HGZ = a.HGZ, HGYZ = a.HGY * a.HGZ;
  uint16_t *alds = reinterpret_cast<uint16_t *>(smem);          // [HAX*HAY*HAZP][RSA]
  uint16_t *glds = alds + (size_t)a.HAX * HAYZ * RSA;           // [HGV][RSG]
  int *hvA = reinterpret_cast<int *>(glds + (size_t)HGV * RSG);  // [PT] A row * RSA
  int *hvG = hvA + PT;                                           // [PT] G row * RSG

  for (int p = tid; p < PT; p += 256) {
    int q, lz, lx, ly;
    a.fTZ.divmod(p, q, lz);
    a.fTY.divmod(q, lx, ly);
    hvA[p] = (lx * a.asx * HAYZ + ly * a.asy * HAZ + lz * a.asz) * RSA;
    hvG[p] = (lx * a.gsx * HGYZ + ly * a.gsy * HGZ + lz * a.gsz) * RSG;
  }
  const int rows_blk = a.taps_rows ? a.TA * CKA : CKA;
  const int cols_blk = a.taps_rows ? CKG : a.TG * CKG;
  int colA[MSW], colG[NS];
#pragma unroll
  for (int m = 0; m < MSW; ++m) {
    const int r = (wave + 4 * m) * 16 + 4 * p4;
    int off = 0;
    if (r < rows_blk) {
      if (a.taps_rows) {
        const int ta = t0 + r / CKA, c = r % CKA;
        if (ta < T) {
          const int kz = ta % a.KZ, qq = ta / a.KZ, ky = qq % a.KY, kx = qq / a.KY;
          off = (kx * a.adx * HAYZ + ky * a.ady * HAZ + kz * a.adz) * RSA + c;
        }
      } else {
        off = r;
      }
    }
    colA[m] = off;
  }
#pragma unroll
  for (int n = 0; n < NS; ++n) {
    const int c = n * 16 + 4 * p4;
    int off = 0;
    if (c < cols_blk) {
      if (a.taps_rows) {
        off = c;
      } else {
        const int tg = t0 + c / CKG, o = c % CKG;
        if (tg < T) {
          const int kz = tg % a.KZ, qq = tg / a.KZ, ky = qq % a.KY, kx = qq / a.KY;
          off = (kx * a.gdx * HGYZ + ky * a.gdy * HGZ + kz * a.gdz) * RSG + o;
        }
      }
    }
    colG[n] = off;
  }

  floatx4 acc[MSW][NS], accb[NS];
#pragma unroll
  for (int m = 0; m < MSW; ++m)
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int n = 0; n < NS; ++n) accb[n] = floatx4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = bias_block && wave == 0;
  const shortx8 ones = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};

  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int CA8 = CKA / 8, CG8 = CKG / 8;
  const bool act = a.a_scale != nullptr;
  const int ca = tid % CA8, cg = tid % CG8;
  const int va0 = tid / CA8, vsA = 256 / CA8, vg0 = tid / CG8, vsG = 256 / CG8;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = act ? a.a_scale[ci0 + ca * 8 + k] : 1.f;
    sh[k] = act ? a.a_shift[ci0 + ca * 8 + k] : 0.f;
  }
  // halo coordinates of each register slot: hx << 20 | hy << 10 | hz, -1 unused
  int hoA[NPA], hoG[NPG];
#pragma unroll
  for (int k = 0; k < NPA; ++k) {
    const int v = va0 + k * vsA;
    int q, hz, hx, hy;
    a.fHAZ.divmod(v, q, hz);
    a.fHAY.divmod(q, hx, hy);
    hoA[k] = v < HAV ? (hx << 20) | (hy << 10) | hz : -1;
  }
#pragma unroll
  for (int k = 0; k < NPG; ++k) {
    const int w = vg0 + k * vsG;
    int q, hz, hx, hy;
    a.fHGZ.divmod(w, q, hz);
    a.fHGY.divmod(q, hx, hy);
    hoG[k] = w < HGV ? (hx << 20) | (hy << 10) | hz : -1;
  }
  const uint16_t *Ab = reinterpret_cast<const uint16_t *>(a.A);
  const uint16_t *Gb = reinterpret_cast<const uint16_t *>(a.G);
  uint4 ra[NPA], rg[NPG];
  unsigned oka = 0;

  auto load = [&](int tt) {
    const int b = tt / ntiles;
    int tile = tt - b * ntiles;
    const int tzi = tile % a.ntz;
    tile /= a.ntz;
    const int tyi = tile % a.nty, txi = tile / a.nty;
    const int px0 = txi * a.TX, py0 = tyi * a.TY, pz0 = tzi * a.TZ;
    // buffer loads of one batch sample with 32-bit offsets: an element outside
    // the operand reads an offset past the buffer (-> 0), no branch per element
    {
      const int gx0 = px0 * a.asx - a.apx, gy0 = py0 * a.asy - a.apy, gz0 = pz0 * a.asz - a.apz;
      const int sampleA = a.AX * a.AY * a.AZ * a.ACs;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(Ab + (size_t)b * sampleA), 0, sampleA * 2, 0x00020000);
      const int cof = (ci0 + ca * 8) * 2, rowA = a.ACs * 2;
      oka = 0;
#pragma unroll
      for (int k = 0; k < NPA; ++k) {
        const int h = hoA[k];
        const int gx = gx0 + (h >> 20), gy = gy0 + ((h >> 10) & 1023), gz = gz0 + (h & 1023);
        const bool ok = h >= 0 && (unsigned)gx < (unsigned)a.AX && (unsigned)gy < (unsigned)a.AY &&
                        (unsigned)gz < (unsigned)a.AZ;
        const int off = ok ? ((gx * a.AY + gy) * a.AZ + gz) * rowA + cof : 0x7ffffff0;
        ra[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        oka |= (ok ? 1u : 0u) << k;
      }
    }
    {
      const int gx0 = px0 * a.gsx - a.gpx, gy0 = py0 * a.gsy - a.gpy, gz0 = pz0 * a.gsz - a.gpz;
      const int sampleG = a.GX * a.GY * a.GZ * a.GCs;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(Gb + (size_t)b * sampleG), 0, sampleG * 2, 0x00020000);
      const int cof = (co0 + cg * 8) * 2, rowG = a.GCs * 2;
#pragma unroll
      for (int k = 0; k < NPG; ++k) {
        const int h = hoG[k];
        const int gx = gx0 + (h >> 20), gy = gy0 + ((h >> 10) & 1023), gz = gz0 + (h & 1023);
        // taps_rows: G is the output grid [PX][PY][PZ] (voxels past it are 0)
        const bool ok = h >= 0 && (unsigned)gx < (unsigned)a.GX && (unsigned)gy < (unsigned)a.GY &&
                        (unsigned)gz < (unsigned)a.GZ &&
                        (!a.taps_rows || (gx < a.PX && gy < a.PY && gz < a.PZ));
        const int off = ok ? ((gx * a.GY + gy) * a.GZ + gz) * rowG + cof : 0x7ffffff0;
        rg[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < NPA; ++k) {
      if (hoA[k] < 0) continue;
      uint4 w = ra[k];
      if (act && ((oka >> k) & 1u)) {
        float f[8];
        unpack8(w, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
        w = pack8(f);
      }
      const int h = hoA[k];   // the halo voxel's row of the padded image
      const int row = ((h >> 20) * a.HAY + ((h >> 10) & 1023)) * HAZ + (h & 1023);
      *reinterpret_cast<uint4 *>(alds + (size_t)row * RSA + ca * 8) = w;
    }
#pragma unroll
    for (int k = 0; k < NPG; ++k) {
      if (hoG[k] < 0) continue;
      const uint4 w = rg[k];
      *reinterpret_cast<uint4 *>(glds + (size_t)(vg0 + k * vsG) * RSG + cg * 8) = w;
    }
  };

  const int KBt = (int)gridDim.x, kbi = (int)blockIdx.x;
  const int tpb_ = (total + KBt - 1) / KBt;
  const int t_beg = kbi * tpb_;
  const int t_end = min(total, t_beg + tpb_);
  if (t_beg < t_end) load(t_beg);
#ifdef HCU_BW_PHASES
  long long bw_ph[4] = {0, 0, 0, 0};
  long long bw_t = (long long)__builtin_readcyclecounter();
#endif
  for (int tt = t_beg; tt < t_end; ++tt) {
    lds_barrier();   // the previous tile's fragment reads are done
    BW_MARK(1);
    commit();
    BW_MARK(0);
    if (tt + 1 < t_end) load(tt + 1);   // in flight during this tile's MFMAs
    lds_barrier();
    BW_MARK(1);
    if constexpr (MSW >= 16) {
      // Many row subtiles per wave (the all-taps form): the A fragments run
      // through a ring of D registers, each read issued D MFMAs ahead of its
      // use and the next 32-voxel step's first fragments (and its G fragment)
      // read during the current step's last MFMAs, so the LDS latency stays
      // hidden behind the MFMA chain (the compiler's own schedule reused one
      // fragment register and waited for every read: ~3x slower).
      constexpr int D = 8;
      const int q = 4 * g + q4;
      int ra0 = hvA[q], ra1 = hvA[q + 16], rg0 = hvG[q], rg1 = hvG[q + 16];
      auto rdA = [&](int r0, int r1, int m) {
        const shortx4 lo = tr_read(alds + r0 + colA[m]);
        const shortx4 hi = tr_read(alds + r1 + colA[m]);
        return shortx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      };
      auto rdG = [&](int r0, int r1) {
        const shortx4 lo = tr_read(glds + r0 + colG[0]);
        const shortx4 hi = tr_read(glds + r1 + colG[0]);
        return shortx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      };
      shortx8 bcur = rdG(rg0, rg1), bnext = bcur;
      shortx8 fr[D];
#pragma unroll
      for (int d = 0; d < D; ++d) fr[d] = rdA(ra0, ra1, d);
      for (int p0 = 0; p0 < PT; p0 += 32) {
        // the next step's rows (the last step re-reads its own: valid addresses)
        const int pn = min(p0 + 32, PT - 32) + q;
        const int na0 = hvA[pn], na1 = hvA[pn + 16], ng0 = hvG[pn], ng1 = hvG[pn + 16];
#pragma unroll
        for (int m = 0; m < MSW; ++m) {
          acc[m][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[m % D], bcur, acc[m][0], 0, 0, 0);
          if (m + D < MSW)
            fr[m % D] = rdA(ra0, ra1, m + D);
          else
            fr[m % D] = rdA(na0, na1, m + D - MSW);
          if (m == MSW - D) bnext = rdG(ng0, ng1);
        }
        if (do_bias) accb[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bcur, accb[0], 0, 0, 0);
        bcur = bnext;
        ra0 = na0;
        ra1 = na1;
      }
      BW_MARK(2);
#ifdef HCU_BW_PHASES
      bw_ph[3] += 1;
#endif
      continue;
    }
    // Two A fragments in flight: fragment m + 1 is read while fragment m's
    // NS MFMAs run, and the next 32-voxel step's G fragments and first A
    // fragment during the step's last row subtile (the same MFMAs in the same
    // order per accumulator: bitwise the sums of the plain loop, which waited
    // for every fragment read before its MFMAs).  With an odd MSW the ring's
    // slots swap roles from one step to the next (sb), so steps run in pairs.
    // voxel rows of this lane's 8 K elements: rows 4g+q4 and 16+4g+q4 of the
    // 32-voxel step (the same order for both operands), so the 32 lanes of
    // each ds_read_b64_tr_b16 bank group read 8 consecutive rows
    const int q = 4 * g + q4;
    int ra0 = hvA[q], ra1 = hvA[q + 16];
    auto rdA = [&](int r0, int r1, int m) {
      const shortx4 lo = tr_read(alds + r0 + colA[m]);
      const shortx4 hi = tr_read(alds + r1 + colA[m]);
      return shortx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    auto rdG = [&](int r0, int r1, int n) {
      const shortx4 lo = tr_read(glds + r0 + colG[n]);
      const shortx4 hi = tr_read(glds + r1 + colG[n]);
      return shortx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    };
    shortx8 bc[NS], bn[NS], ring[2];
    {
      const int rg0 = hvG[q], rg1 = hvG[q + 16];
#pragma unroll
      for (int n = 0; n < NS; ++n) bc[n] = rdG(rg0, rg1, n);
    }
    ring[0] = rdA(ra0, ra1, 0);
    auto step = [&](auto SB, int p0) {
      constexpr int sb = decltype(SB)::value;
      const int pn = min(p0 + 32, PT - 32) + q;   // (the last step re-reads its own rows)
      const int na0 = hvA[pn], na1 = hvA[pn + 16], ng0 = hvG[pn], ng1 = hvG[pn + 16];
#pragma unroll
      for (int m = 0; m < MSW; ++m) {
        const shortx8 af = ring[(m + sb) & 1];
        if (m + 1 < MSW) {
          ring[(m + 1 + sb) & 1] = rdA(ra0, ra1, m + 1);
        } else {
          ring[(m + 1 + sb) & 1] = rdA(na0, na1, 0);
#pragma unroll
          for (int n = 0; n < NS; ++n) bn[n] = rdG(ng0, ng1, n);
        }
#pragma unroll
        for (int n = 0; n < NS; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bc[n], acc[m][n], 0, 0, 0);
      }
      if (do_bias) {
#pragma unroll
        for (int n = 0; n < NS; ++n)
          accb[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bc[n], accb[n], 0, 0, 0);
      }
#pragma unroll
      for (int n = 0; n < NS; ++n) bc[n] = bn[n];
      ra0 = na0;
      ra1 = na1;
    };
    for (int p0 = 0; p0 < PT; p0 += 64) {
      step(std::integral_constant<int, 0>{}, p0);
      if (p0 + 32 < PT) step(std::integral_constant<int, MSW & 1>{}, p0 + 32);
    }
  }

#ifdef HCU_BW_PHASES
  if (MSW >= 16 && tid == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
    unsigned long long *d = g_bw_phase + (size_t)(blockIdx.x % 4096) * 4;
    for (int k = 0; k < 4; ++k) d[k] += (unsigned long long)bw_ph[k];
  }
#endif
  const size_t slab = (size_t)blockIdx.x * a.Mtot;
  // taps_rows slab rows (tap, real channel) and columns (real channels):
  // WGradArgs::ACr / GCr, the padding slots of the channel strides not stored
  const int ACR = a.ACr > 0 ? a.ACr : a.ACs, GCR = a.GCr > 0 ? a.GCr : a.GCs;
#pragma unroll
  for (int m = 0; m < MSW; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = (wave + 4 * m) * 16 + g * 4 + r;
      int grow = -1;
      if (lr < rows_blk) {
        if (a.taps_rows) {
          const int ta = t0 + lr / CKA, ci = ci0 + lr % CKA;
          if (ta < T && ci < ACR) grow = ta * ACR + ci;
        } else if (ci0 + lr < a.ACs) {
          grow = ci0 + lr;
        }
      }
      if (grow < 0) continue;
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        const int lc = n * 16 + (lane & 15);
        int gcol = -1;
        if (lc < cols_blk) {
          if (a.taps_rows) {
            if (co0 + lc < GCR) gcol = co0 + lc;
          } else {
            const int tg = t0 + lc / CKG, o = co0 + lc % CKG;
            if (tg < T && o < a.GCs) gcol = tg * a.GCs + o;
          }
        }
        if (gcol >= 0) a.partial[(slab + grow) * a.Ntot + gcol] = acc[m][n][r];
      }
    }
  }
  if (do_bias && g == 0) {
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const int lc = n * 16 + (lane & 15);
      if (lc < CKG && co0 + lc < GCR)
        a.partial[(slab + (size_t)T * ACR) * a.Ntot + co0 + lc] = accb[n][0];
    }
  }
}

// ---------------------------------------------------------------------------
// CUs' worth of resident workgroups the bf16 weight gradient is sized for
// (HCU_BW_CUS, A/B): fewer voxel blocks write fewer fp32 slabs for the
// finalize to read, and leave the chain's kernels room on the CUs.  Config 3
// (interleaved A/B, 2 runs each): 256 -> 6.77 ms/step, 224 -> 6.63, 192 ->
// 6.65, 160 -> 6.81.
static int bw_cus() {
  static const int v = [] {
    const char *e = getenv("HCU_BW_CUS");
    const int n = e ? atoi(e) : 224;
    return n < 16 ? 16 : (n > 256 ? 256 : n);
  }();
  return v;
}

static int plan_bwgrad_cka(WGradArgs &a, int cka_cap, bool alltaps);

// HCU_BW_ALLTAPS=0: split the taps of a many-tap kernel over blocks (A/B)
static bool alltaps_enabled() {
  static const bool on = !(getenv("HCU_BW_ALLTAPS") && getenv("HCU_BW_ALLTAPS")[0] == '0');
  return on;
}

int plan_bwgrad(WGradArgs &a, int target_blocks) {
  (void)target_blocks;
  if (a.ACs % 8 || a.GCs % 8) return fail(4, "bwgrad: channel strides must be multiples of 8");
  if (a.PX <= 0 || a.PY <= 0 || a.PZ <= 0) return fail(2, "bwgrad: empty grid");
  // channel chunks: A side up to 32 channels, G side up to 64 (16-col
  // subtiles).  (16-channel A chunks measured 7.11 vs 6.63 ms per config-3
  // step; 64-channel ones fit the LDS of almost no layer.)
  if (alltaps_enabled() && plan_bwgrad_cka(a, 32, true) == 0) return 0;
  return plan_bwgrad_cka(a, 32, false);
}

// alltaps: a kernel with more (tap, channel) rows than one block's 36 row
// subtiles (RDCNet's 5x5x5 convolutions: 125 taps x 16 channel slots) keeps
// ALL of them in one block -- 32 row subtiles per wave, the column chunk one
// 16-column subtile -- so each voxel tile's A halo and G image are staged once
// for every tap instead of once per tap chunk (the split form re-stages both
// for each of its 4 tap chunks and ran at ~3-4 % of bf16 MFMA).  Fails (the
// caller then takes the split form) for any other shape.
static int plan_bwgrad_cka(WGradArgs &a, int cka_cap, bool alltaps) {
  a.use_bw = 0;
  const int T = a.KX * a.KY * a.KZ;
  // padded operands (zero padding of A, or a cropped ConvTranspose3d output
  // as G) are staged as zeros outside their grids
  a.CKA = std::min(a.ACs, cka_cap);
  // (the largest of 32 / 16 / 8 channels that divides ACs: RDCNet's mixing
  // 1x1 convolution reads 5 parts x 16 = 80 channel slots -- 5 chunks of 16,
  // not 10 of 8, each of which re-stages the G tile)
  if (a.ACs % a.CKA) a.CKA = (a.ACs % 16 == 0 && cka_cap >= 16) ? 16 : 8;
  a.CKG = std::min(a.GCs, 64);
  if (a.GCs % a.CKG) a.CKG = (a.GCs % 32 == 0) ? 32 : (a.GCs % 16 == 0 ? 16 : 8);
  const int ncol_tiles_full = a.taps_rows ? cdiv(a.CKG, 16) : 0;
  // row / column subtiles per block
  if (a.taps_rows) {
    a.NSB = ncol_tiles_full;
    const int rows_all = T * a.CKA;                    // all taps of one channel chunk
    const int sub_all = cdiv(rows_all, 16);
    int msw = cdiv(sub_all, 4);
    if (alltaps && (msw <= 9 || msw > 32 || a.NSB != 1)) return 1;
    if (alltaps) {
      a.MSW = 32;
      a.TA = T;
    } else {
      if (msw > 9) msw = 9;                            // split the taps over blocks (36 rows each)
      // (one row subtile per wave for the 1x1 kernels: 16-32 rows; three
      // per wave there left 11 of 12 MFMA subtiles of a block on padding)
      a.MSW = msw <= 1 && !getenv("HCU_BW_MSW3") ? 1 : msw <= 3 ? 3 : (msw <= 5 ? 5 : 9);
      a.TA = std::min(T, (a.MSW * 4 * 16) / a.CKA);
    }
    if (a.TA < 1) return fail(4, "bwgrad: channel chunk too large");
    a.TG = 1;
    a.ntc = cdiv(T, a.TA);
  } else {
    if (alltaps) return 1;
    // rows = input channels of one chunk (CKA / 16 subtiles), columns = (tap, co)
    a.CKA = std::min(a.ACs, 64);
    if (a.ACs % a.CKA) a.CKA = (a.ACs % 32 == 0) ? 32 : (a.ACs % 16 == 0 ? 16 : 8);
    a.MSW = 1;
    if (cdiv(a.CKA, 16) > 4 * a.MSW) return fail(4, "bwgrad: row chunk too large");
    // the G operand is a strided halo (~S^2 (TZ+1)/TZ rows per voxel): keep
    // its channel chunk small so the image fits LDS
    a.CKG = std::min(a.GCs, (a.gsx * a.gsy * a.gsz > 1) ? 16 : 32);
    if (a.GCs % a.CKG) a.CKG = (a.GCs % 16 == 0) ? 16 : 8;
    a.TG = std::max(1, std::min(T, 128 / a.CKG));      // up to 8 column subtiles
    a.NSB = cdiv(a.TG * a.CKG, 16);
    a.TA = 1;
    a.ntc = cdiv(T, a.TG);
  }
  if (a.NSB > 8) return fail(4, "bwgrad: too many column subtiles");
  a.nci = a.ACs / a.CKA;
  a.nco = a.GCs / a.CKG;
  a.mchunks = a.taps_rows ? a.ntc * a.nci : a.nci;
  a.nchunks = a.taps_rows ? a.nco : a.ntc * a.nco;
  if (!a.taps_rows || a.ACr >= a.ACs) a.ACr = 0;
  if (!a.taps_rows || a.GCr >= a.GCs) a.GCr = 0;
  const int ACR = a.ACr > 0 ? a.ACr : a.ACs, GCR = a.GCr > 0 ? a.GCr : a.GCs;
  a.Mtot = a.taps_rows ? T * ACR + (a.bias_row ? 1 : 0) : a.ACs;
  a.Ntot = a.taps_rows ? GCR : T * a.GCs;
  // voxel tile: TX*TY = 32 (or 64 when the halo fits), TZ = the whole Z (<= 16)
  // (TZ <= 8 for every layer -- half the image, two resident blocks, twice
  // the slabs -- measured 7.25 vs 6.63 ms per config-3 step)
  int ntz = cdiv(a.PZ, 16);
  a.TZ = cdiv(a.PZ, ntz);
  // LDS row strides (bf16 elements) with (CK + pad) / 16 odd for CK >= 32:
  // 8 consecutive rows' 32-byte fragments then cover the 64 banks once (CK + 8
  // put two of the 8 rows of a read on the same banks).  CK <= 16 keeps
  // CK + 8: a smaller image there lets the direct form of RDCNet's dilated
  // convolutions fit LDS, whose weight gradient then runs without the
  // sub-lattice split and 7 ms per step slower.
  // The all-taps form reads 8 consecutive voxel rows per lane group: 32-byte
  // rows (no pad) put them on the 64 banks once.
  auto pad_of = [&](int ck) { return ck <= 16 ? (alltaps && ck == 16 ? 0 : 8) : ((16 - ck % 32) % 32 + 32) % 32; };
  a.PA2 = a.CKA + pad_of(a.CKA);
  a.PG2 = a.CKG + pad_of(a.CKG);
  // (a 4 x 4 x even-TZ tile -- half the halo image, two blocks per CU on the
  // level-0/1 layers -- measured 7.60-7.66 ms per config-3 step against 6.62:
  // its larger halo share and twice the slabs cost more than the occupancy)
  const int txys[2][2] = {{8, 8}, {4, 8}};
  const int TZ0 = a.TZ;
  auto set_tile = [&](int i) {
    a.TX = txys[i][0];
    a.TY = txys[i][1];
    a.TZ = TZ0;
    a.HAX = (a.TX - 1) * a.asx + (a.taps_rows ? (a.KX - 1) * a.adx : 0) + 1;
    a.HAY = (a.TY - 1) * a.asy + (a.taps_rows ? (a.KY - 1) * a.ady : 0) + 1;
    a.HAZ = (a.TZ - 1) * a.asz + (a.taps_rows ? (a.KZ - 1) * a.adz : 0) + 1;
    a.HGX = (a.TX - 1) * a.gsx + (a.taps_rows ? 0 : (a.KX - 1) * a.gdx) + 1;
    a.HGY = (a.TY - 1) * a.gsy + (a.taps_rows ? 0 : (a.KY - 1) * a.gdy) + 1;
    a.HGZ = (a.TZ - 1) * a.gsz + (a.taps_rows ? 0 : (a.KZ - 1) * a.gdz) + 1;
    a.HAV = a.HAX * a.HAY * a.HAZ;
    a.HGV = a.HGX * a.HGY * a.HGZ;
    a.PTV = a.TX * a.TY * a.TZ;
    // (all-taps form) rows per (hx, hy) column of the A image: HAZP = TZ mod
    // 8, so the 8 consecutive tile voxels of a fragment read -- z-runs of TZ
    // rows, consecutive columns HAZP rows apart -- land on 8 different groups
    // of 8 banks (32-byte rows)
    a.HAZP = alltaps ? a.HAZ + ((a.TZ - a.HAZ) % 8 + 8) % 8 : a.HAZ;
    return ((long)a.HAX * a.HAY * a.HAZP * a.PA2 + (long)a.HGV * a.PG2) * 2 + 2L * a.PTV * 4;
  };
  // the first tile whose image fits two blocks per CU, else the smallest
  const int t0i = 0;   // (starting at the 4 x 8 tile measured equal)
  const int nti = 2;
  int pick = -1;
  long best_lds = 1L << 40;
  // (alltaps: one block per CU -- its registers allow no second one -- so
  // the largest tile that fits the CU's LDS: the smallest halo share)
  const long lds_cap = alltaps ? 156 * 1024 : 80 * 1024;
  for (int i = t0i; i < nti && pick < 0; ++i) {
    const long l = set_tile(i);
    if (l <= lds_cap) pick = i;
    else if (l < best_lds) { best_lds = l; pick = -2 - i; }
  }
  if (pick < -1) pick = -2 - pick;
  if (pick < 0) pick = t0i;
  long lds = set_tile(pick);
  // A layer whose full-Z tile leaves one block per CU and whose slab is small
  // (the level-0/1 layers: the next tile's loads are exposed, the finalize
  // reads little) takes half the Z extent per tile: two resident blocks
  // Config 3 (interleaved A/B, 2 runs): slabs <= 64 KB (d0.c2, u3.c2) 6.50 vs
  // 6.62 ms/step without; <= 160 KB 6.56; <= 640 KB 6.96.
  // (the slab size with the padding slots: the measured rule predates ACr / GCr)
  const long slab_pad = a.taps_rows ? ((long)T * a.ACs + (a.bias_row ? 1 : 0)) * a.GCs : (long)a.Mtot * a.Ntot;
  if (!alltaps && lds > 80 * 1024 && slab_pad * 4 <= 64 * 1024 && a.PZ > 8) {
    ntz = cdiv(a.PZ, 8);
    a.TZ = cdiv(a.PZ, ntz);
    const int TZh = a.TZ;
    a.HAZ = (TZh - 1) * a.asz + (a.taps_rows ? (a.KZ - 1) * a.adz : 0) + 1;
    a.HGZ = (TZh - 1) * a.gsz + (a.taps_rows ? 0 : (a.KZ - 1) * a.gdz) + 1;
    a.HAV = a.HAX * a.HAY * a.HAZ;
    a.HGV = a.HGX * a.HGY * a.HGZ;
    a.PTV = a.TX * a.TY * TZh;
    a.HAZP = a.HAZ;
    lds = ((long)a.HAV * a.PA2 + (long)a.HGV * a.PG2) * 2 + 2L * a.PTV * 4;
  }
  if (lds > 160 * 1024) return fail(4, "bwgrad: tile does not fit LDS");
  a.lds_bytes = (int)((lds + 15) & ~15L);
  a.fHAZ = FastDiv(a.HAZ);
  a.fHAY = FastDiv(a.HAY);
  a.fHGZ = FastDiv(a.HGZ);
  a.fHGY = FastDiv(a.HGY);
  a.fTZ = FastDiv(a.TZ);
  a.fTY = FastDiv(a.TY);
  a.ntx = cdiv(a.PX, a.TX);
  a.nty = cdiv(a.PY, a.TY);
  a.ntz = ntz;
  const long total = (long)a.B * a.ntx * a.nty * a.ntz;
  const long per = (long)a.mchunks * a.nchunks;
  a.occ = std::max(1, std::min(8, (int)(160 * 1024 / a.lds_bytes)));
  // register prefetch slots per thread (pipelined kernel): max over threads of
  // the 16-byte A / G loads one tile needs
  const int nA = cdiv(a.HAV, 256 / (a.CKA / 8)), nG = cdiv(a.HGV, 256 / (a.CKG / 8));
  const int np = std::max(nA, nG);
  a.NPA = a.NPG = np <= 8 ? 8 : np <= 16 ? 16 : np <= 32 ? 32 : 0;
  if (alltaps) {   // the instances of launch_bwgrad's BWT list
    a.NPA = nA <= 8 ? 8 : nA <= 12 ? 12 : nA <= 20 ? 20 : 0;
    a.NPG = nG <= 8 ? 8 : 0;
    if (!a.NPA || !a.NPG || a.CKA > 16) return 1;
  }
  // One fp32 slab per block: the pipelined kernel hides its loads behind the
  // MFMAs of the same block, so it needs at most two blocks per CU -- fewer
  // blocks, fewer slabs for the finalize to read.
  const int occ_cap = 2;   // (grids for one block per CU measured +1 %)
  const int occ_kb = a.NPA ? std::min(a.occ, occ_cap) : a.occ;
  // The network's first layer (<= 8 input channels) runs last on the branch,
  // after the chain has finished: its grid takes the whole chip (config 3,
  // interleaved A/B, 3 runs: 6.433-6.449 vs 6.455-6.461 ms/step at 224 CUs).
  const int cus = (a.ACs <= 8 || alltaps) ? 256 : bw_cus();
  long kb = std::max(1L, (long)cus * occ_kb / per);
  kb = std::min(kb, total);
  a.KB = (int)kb;
  a.use_bw = 1;
  a.v2 = 0;
  if (getenv("HCU_CONV2_LOG"))
    fprintf(stderr,
            "bwgrad plan: rows%d A%dx%dx%d ACs%d G%dx%dx%d GCs%d P%dx%dx%d K%dx%dx%d | CKA%d CKG%d "
            "TA%d TG%d MSW%d NSB%d T%dx%dx%d KB%d m%d n%d lds%d\n",
            a.taps_rows, a.AX, a.AY, a.AZ, a.ACs, a.GX, a.GY, a.GZ, a.GCs, a.PX, a.PY, a.PZ, a.KX,
            a.KY, a.KZ, a.CKA, a.CKG, a.TA, a.TG, a.MSW, a.NSB, a.TX, a.TY, a.TZ, a.KB, a.mchunks,
            a.nchunks, a.lds_bytes);
  return 0;
}

int launch_bwgrad(const WGradArgs &a, hipStream_t s) {
  const dim3 grid(a.KB, a.mchunks, a.nchunks);
  const int T = a.KX * a.KY * a.KZ;
  const double fl = a.flops > 0 ? a.flops
                                : 2.0 * a.B * a.PX * a.PY * a.PZ * (double)T * a.ACs * a.GCs;
  const double by = 2.0 * ((double)a.B * a.AX * a.AY * a.AZ * a.ACs +
                           (double)a.B * a.GX * a.GY * a.GZ * a.GCs);
  bool ok = false;
#define BWP(MS_, NS_, NP_)                                                                  \
  if (!ok && a.NPA == NP_ && a.NPG == NP_) {                                                \
    HCU_TIMED(s, "bwgrad_pipe_kernel<" #MS_ "," #NS_ "," #NP_ ">", fl, by,                    \
              HCU_LAUNCH((bwgrad_pipe_kernel<MS_, NS_, NP_, NP_>), grid, dim3(256),         \
                                 a.lds_bytes, s, a));                                       \
    ok = true;                                                                              \
  }
  // all taps of a channel chunk in one block (MSW = 32): the A halo and G tile
  // are staged once per tile for every tap (plan_bwgrad_cka)
#define BWT(NPA_, NPG_)                                                                     \
  if (!ok && a.MSW == 32 && a.NSB == 1 && a.NPA == NPA_ && a.NPG == NPG_) {                 \
    HCU_TIMED(s, "bwgrad_pipe_kernel<32,1," #NPA_ "," #NPG_ ">", fl, by,                     \
              HCU_LAUNCH((bwgrad_pipe_kernel<32, 1, NPA_, NPG_>), grid, dim3(256),          \
                         a.lds_bytes, s, a));                                               \
    ok = true;                                                                              \
  }
  BWT(8, 8) BWT(12, 8) BWT(20, 8)
#undef BWT
#define BW(MS_, NS_)                                                                        \
  if (!ok && a.MSW == MS_ && a.NSB <= NS_) {                                                \
    BWP(MS_, NS_, 8) BWP(MS_, NS_, 16) BWP(MS_, NS_, 32)                                    \
    if (!ok) {                                                                              \
      HCU_TIMED(s, "bwgrad_kernel<" #MS_ "," #NS_ ">", fl, by,                              \
                HCU_LAUNCH((bwgrad_kernel<MS_, NS_>), grid, dim3(256), a.lds_bytes, s, a)); \
    }                                                                                       \
    ok = true;                                                                              \
  }
  BW(1, 1) BW(1, 2) BW(1, 4) BW(1, 8) BW(3, 1) BW(3, 2) BW(3, 4) BW(5, 1) BW(5, 2) BW(5, 4)
  BW(9, 1) BW(9, 2) BW(9, 4)
#undef BW
#undef BWP
  if (!ok) return fail(4, "bwgrad: unsupported variant");
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu
