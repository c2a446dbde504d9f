// fp32 Conv3d weight gradient for the deep levels, taps on the rows:
//
//   dW[(t, ci)][co] = sum_p act(A[p + off(t)][ci]) * G[p][co]   (+ bias row sum_p G[p][co])
//
// on v_mfma_f32_16x16x4_f32 (hcat/unet.py:246-257's Conv3d weight gradient).
// wgrad2 splits a block's voxels over its four waves and reduces them at the
// end, so a block covers at most 64 rows; with 18 taps that is a 4-channel
// chunk, and every (tap, channel) chunk re-stages the whole gradient tile (16
// times on d3.c1 of config 2).  Here the waves split the OUTPUT instead: wave
// w owns row subtiles w*MS .. w*MS+MS-1 of the block's 64*MS rows (all taps of
// a 16/32/64-channel chunk) and every voxel of the tile, so a staged voxel
// tile feeds 64*MS rows x 16*NS columns and no cross-wave reduction is needed.
//
// LDS images are channel-major (A: [channel][halo voxel], G: [column][tile
// voxel]) with row strides = 2 (mod 32): the 16 x 4 lanes of one MFMA operand
// read (16 channels / columns) x (4 consecutive voxels) with ds_read_b32 on 32
// distinct banks per half-wave, and a tap is a per-lane voxel offset (no
// per-tap image copies, no alignment constraint).  Tiles: TX x TY x TZP
// voxels, TZ the whole (<= 16) Z extent rounded up to a multiple of 4 (the
// extra z rows read G = 0).  Every block writes one fp32 partial slab
// [Mtot][Ntot] (the wgrad2 layout); wgrad_finalize sums them in fp64 in a
// fixed order.
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace hcu {

bool wgrad3_enabled() {   // HCU_WGRAD3=0 keeps the deep layers on wgrad2 (A/B)
  static const bool on = [] {
    const char *e = getenv("HCU_WGRAD3");
    return !(e && e[0] == '0');
  }();
  return on;
}

constexpr int kW3Loads = 8;   // 16-byte staging loads in flight per thread (serial staging)

template <int MS, int NS>
__global__ void __launch_bounds__(256) wgrad3_kernel(const WGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kq = lane >> 4, r16 = lane & 15;
  const int T = a.KX * a.KY * a.KZ;
  const int CKA = a.CKA, CKG = a.CKG, RSA = a.PA2, RSG = a.PG2;
  const int tapc = blockIdx.y / a.nci, cic = blockIdx.y % a.nci, coc = blockIdx.z;
  const int ci0 = cic * CKA, co0 = coc * CKG, t0 = tapc * a.TA;
  const bool bias_block = a.bias_row && tapc == 0 && cic == 0;
  const int HAZP = a.HAZP, HAYZ = a.HAY * a.HAZP, TZP = a.TZP;
  const int HAV = a.HAX * a.HAY * HAZP, PTP = a.TX * a.TY * TZP;
  const int NK = PTP / 4;                            // K-steps of a tile (4 voxels each)
  float *alds = smem;                                // [CKA + 1][RSA]  (+ zero row)
  float *glds = alds + (size_t)(CKA + 1) * RSA;      // [CKG + 1][RSG]  (+ zero row)
  int *hvtab = reinterpret_cast<int *>(glds + (size_t)(CKG + 1) * RSG);   // [NK] halo voxel of K-step k
  float *dummy = reinterpret_cast<float *>(hvtab + NK);                   // [4][64] sink of the padding lanes
  for (int i = tid; i < RSA; i += 256) alds[(size_t)CKA * RSA + i] = 0.f;
  for (int i = tid; i < RSG; i += 256) glds[(size_t)CKG * RSG + i] = 0.f;
  for (int k = tid; k < NK; k += 256) {
    const int row = k / (TZP / 4), z0 = (k - row * (TZP / 4)) * 4;
    int lx, ly;
    a.fTY.divmod(row, lx, ly);
    hvtab[k] = lx * HAYZ + ly * HAZP + z0;
  }

  // this lane's operand bases: A row (tap, channel) of each of the wave's row
  // subtiles (tap offset in halo voxels folded in), G column of each column
  // subtile; rows / columns past the layer read the zero rows
  int aoff[MS];
#pragma unroll
  for (int m = 0; m < MS; ++m) {
    const int r = (wave * MS + m) * 16 + r16;
    const int tl = r / CKA, c = r % CKA, t = t0 + tl;
    int off = CKA * RSA;
    if (tl < a.TA && t < T && ci0 + c < a.ACs) {
      const int kz = t % a.KZ, q = t / a.KZ, ky = q % a.KY, kx = q / a.KY;
      off = c * RSA + kx * a.adx * HAYZ + ky * a.ady * HAZP + kz * a.adz;
    }
    aoff[m] = off + kq;
  }
  int goff[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) {
    const int c = n * 16 + r16;
    goff[n] = ((c < CKG && co0 + c < a.Ntot) ? c * RSG : CKG * RSG) + kq;
  }
  // ConvTranspose3d phase form (WGradArgs::nph): column c is channel c % GCout
  // of stride phase q = c / GCout, whose G is read at o*S + q.  A thread
  // always stages the same 4-column group (below), whose 4 columns share a
  // phase (GCout % 4 == 0): a block's columns may span phases.
  int gq[3] = {0, 0, 0};
  floatx4 acc[MS][NS], accb[NS];
#pragma unroll
  for (int m = 0; m < MS; ++m)
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int n = 0; n < NS; ++n) accb[n] = floatx4{0.f, 0.f, 0.f, 0.f};
  // wave-uniform (a scalar branch in the MFMA loop)
  const bool do_bias = __builtin_amdgcn_readfirstlane((int)(bias_block && wave == 0)) != 0;
  const bool act = a.a_scale != nullptr;
  // channel groups per staged voxel: powers of two (plan_wgrad3), so the
  // element -> (voxel, group) split is a shift; a thread always stages the
  // same 4-channel group (256 % CA4 == 0, 256 % CG4 == 0)
  const int lgA = __builtin_ctz(CKA / 4), lgG = __builtin_ctz(CKG / 4);
  int cg = co0 + (tid & ((1 << lgG) - 1)) * 4;
  if (a.nph > 1) {
    const int q = cg / a.GCout;
    cg -= q * a.GCout;
    gq[2] = q % a.phz;
    gq[1] = (q / a.phz) % a.phy;
    gq[0] = q / (a.phz * a.phy);
  }
  const int ca = ci0 + (tid & ((1 << lgA) - 1)) * 4;
  const int rowa = (tid & ((1 << lgA) - 1)) * 4 * RSA, rowg = (tid & ((1 << lgG) - 1)) * 4 * RSG;
  const bool cok_a = ca < a.ACs, cok_g = cg < a.GCs && co0 + (tid & ((1 << lgG) - 1)) * 4 < a.Ntot;
  float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
  if (act && cok_a) {
    sc = *reinterpret_cast<const float4 *>(a.a_scale + ca);
    sh = *reinterpret_cast<const float4 *>(a.a_shift + ca);
  }
  const int sampA = a.AX * a.AY * a.AZ * a.ACs, sampG = a.GX * a.GY * a.GZ * a.GCs;   // floats (< 2^29, plan)
  const int nA = HAV << lgA, nG = PTP << lgG;

  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int KBt = (int)gridDim.x, kbi = (int)blockIdx.x;
  const int tpb = (total + KBt - 1) / KBt;
  const int t_beg = kbi * tpb, t_end = min(total, t_beg + tpb);
  auto tile_of = [&](int tt, int &b, int &px0, int &py0, int &pz0) {
    b = tt / ntiles;
    int tile = tt - b * ntiles;
    const int tzi = tile % a.ntz;
    tile /= a.ntz;
    const int tyi = tile % a.nty, txi = tile / a.nty;
    px0 = txi * a.TX;
    py0 = tyi * a.TY;
    pz0 = tzi * a.TZ;
  };
  auto rsrc = [&](const float *base, int floats) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, floats * 4, 0x00020000);
  };
  // element idx of the A halo / G tile: byte offset in its sample (past the
  // buffer when invalid -> 0) and validity
  auto a_elem = [&](int idx, int px0, int py0, int pz0, bool &ok) {
    const int v = idx >> lgA;
    int q, hz, hx, hy;
    a.fHAZ.divmod(v, q, hz);
    a.fHAY.divmod(q, hx, hy);
    const int gx = px0 + hx - a.apx, gy = py0 + hy - a.apy, gz = pz0 + hz - a.apz;
    ok = idx < nA && cok_a && (unsigned)gx < (unsigned)a.AX && (unsigned)gy < (unsigned)a.AY &&
         (unsigned)gz < (unsigned)a.AZ;
    return ok ? (((gx * a.AY + gy) * a.AZ + gz) * a.ACs + ca) * 4 : 0x7ffffff0;
  };
  auto g_elem = [&](int idx, int px0, int py0, int pz0) {
    const int p = idx >> lgG;
    int q, lz, lx, ly;
    a.fTZ.divmod(p, q, lz);
    a.fTY.divmod(q, lx, ly);
    const int ox = px0 + lx, oy = py0 + ly, oz = pz0 + lz;
    const int gx = ox * a.gsx + gq[0], gy = oy * a.gsy + gq[1], gz = oz * a.gsz + gq[2];
    const bool ok = idx < nG && cok_g && lz < a.TZ && ox < a.PX && oy < a.PY && oz < a.PZ && gx < a.GX &&
                    gy < a.GY && gz < a.GZ;
    return ok ? (((gx * a.GY + gy) * a.GZ + gz) * a.GCs + cg) * 4 : 0x7ffffff0;
  };
  auto act4 = [&](floatx4 x, bool ok) {
    if (act) {
      x[0] = ok ? fmaxf(fmaf(x[0], sc.x, sh.x), 0.f) : 0.f;
      x[1] = ok ? fmaxf(fmaf(x[1], sc.y, sh.y), 0.f) : 0.f;
      x[2] = ok ? fmaxf(fmaf(x[2], sc.z, sh.z), 0.f) : 0.f;
      x[3] = ok ? fmaxf(fmaf(x[3], sc.w, sh.w), 0.f) : 0.f;
    }
    return x;
  };
  auto put4 = [&](float *d, int st, const floatx4 &x) {
    d[0] = x[0];
    d[st] = x[1];
    d[2 * st] = x[2];
    d[3 * st] = x[3];
  };
  for (int tt = t_beg; tt < t_end; ++tt) {
    int b, px0, py0, pz0;
    tile_of(tt, b, px0, py0, pz0);
    lds_barrier();   // the previous tile's operand reads are done
    // ---- A halo, channel-major (activation applied, 0 outside the input).
    // Branch-free: every load of a round is issued before the first LDS write
    // (an invalid element reads an offset past the buffer -> 0).
    const __amdgpu_buffer_rsrc_t rA = rsrc(a.A + (size_t)b * sampA, sampA);
    for (int base = tid; base < nA; base += kW3Loads * 256) {
      floatx4 val[kW3Loads];
      uint32_t okm = 0;
#pragma unroll
      for (int u = 0; u < kW3Loads; ++u) {
        bool ok;
        const int off = a_elem(base + u * 256, px0, py0, pz0, ok);
        val[u] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rA, off, 0, 0));
        okm |= (uint32_t)ok << u;
      }
#pragma unroll
      for (int u = 0; u < kW3Loads; ++u) {
        const int idx = base + u * 256;
        const bool in = idx < nA;
        put4(in ? alds + rowa + (idx >> lgA) : dummy + lane, in ? RSA : 64, act4(val[u], (okm >> u) & 1u));
      }
    }
    // ---- G tile, channel-major, z rows of TZP (0 past the output grid)
    const __amdgpu_buffer_rsrc_t rG = rsrc(a.G + (size_t)b * sampG, sampG);
    for (int base = tid; base < nG; base += kW3Loads * 256) {
      floatx4 val[kW3Loads];
#pragma unroll
      for (int u = 0; u < kW3Loads; ++u)
        val[u] = __builtin_bit_cast(floatx4,
                                    __builtin_amdgcn_raw_buffer_load_b128(rG, g_elem(base + u * 256, px0, py0, pz0), 0, 0));
#pragma unroll
      for (int u = 0; u < kW3Loads; ++u) {
        const int idx = base + u * 256;
        const bool in = idx < nG;
        put4(in ? glds + rowg + (idx >> lgG) : dummy + lane, in ? RSG : 64, val[u]);
      }
    }
    lds_barrier();
    // ---- MFMA over the tile's voxels, 4 per K-step (lane group kq takes
    // voxel 4k + kq of the tile, halo voxel hvtab[k] + kq); the operands of
    // step k + 1 are read while the MFMAs of step k run
    float av0[MS], bv0[NS], av1[MS], bv1[NS];
    // (hv: the K-step's halo voxel, read from hvtab two steps ahead)
    auto ld = [&](int k, int hv, float (&av)[MS], float (&bv)[NS]) {
      const int kk = min(k, NK - 1);
#pragma unroll
      for (int n = 0; n < NS; ++n) bv[n] = glds[goff[n] + 4 * kk];
#pragma unroll
      for (int m = 0; m < MS; ++m) av[m] = alds[aoff[m] + hv];
    };
    auto mf = [&](const float (&av)[MS], const float (&bv)[NS]) {
#pragma unroll
      for (int m = 0; m < MS; ++m)
#pragma unroll
        for (int n = 0; n < NS; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[n], acc[m][n], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int n = 0; n < NS; ++n) accb[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, bv[n], accb[n], 0, 0, 0);
      }
    };
    int hvA = hvtab[0], hvB = hvtab[min(1, NK - 1)];
    ld(0, hvA, av0, bv0);
    hvA = hvtab[min(2, NK - 1)];
    for (int k = 0; k < NK; k += 2) {
      ld(k + 1, hvB, av1, bv1);
      hvB = hvtab[min(k + 3, NK - 1)];
      __builtin_amdgcn_sched_barrier(0);
      mf(av0, bv0);
      ld(k + 2, hvA, av0, bv0);
      hvA = hvtab[min(k + 4, NK - 1)];
      __builtin_amdgcn_sched_barrier(0);
      if (k + 1 < NK) mf(av1, bv1);
    }
  }

  // ---- one partial slab per block: each wave writes its own rows
  const size_t slab = (size_t)blockIdx.x * a.Mtot;
#pragma unroll
  for (int m = 0; m < MS; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = (wave * MS + m) * 16 + kq * 4 + r;
      const int tl = lr / CKA, t = t0 + tl, ci = ci0 + lr % CKA;
      if (tl >= a.TA || t >= T || ci >= a.ACs) continue;
      const int grow = t * a.ACs + ci;
#pragma unroll
      for (int n = 0; n < NS; ++n) {
        const int gcol = co0 + n * 16 + r16;
        if (n * 16 + r16 < CKG && gcol < a.Ntot) a.partial[(slab + grow) * a.Ntot + gcol] = acc[m][n][r];
      }
    }
  }
  if (do_bias && kq == 0) {   // row 0 of the ones-subtile: sum_p G[p][col]
#pragma unroll
    for (int n = 0; n < NS; ++n) {
      const int gcol = co0 + n * 16 + r16;
      if (n * 16 + r16 < CKG && gcol < a.GCs)
        a.partial[(slab + (size_t)T * a.ACs) * a.Ntot + gcol] = accb[n][0];
    }
  }
}

// Row stride of a channel-major image: >= n, = 2 (mod 32) (see above).
static int cm_stride(int n) { return n + ((2 - n % 32) + 32) % 32; }

// Plans a Conv3d weight gradient (taps_rows, stride-1 unpadded operands,
// fp32) for wgrad3_kernel; 0 when it applies.  Chooses the channel chunk, the
// row subtiles per wave (3 / 5 / 9), the voxel tile and the number of voxel
// blocks by a per-CU time model: MFMA cycles of a block + its staging (~32
// bytes a cycle) + its slab write, the blocks spread over the 192 CUs the branch
// stream is sized for.
int plan_wgrad3(WGradArgs &a) {
  if (!wgrad3_enabled() || !a.taps_rows) return 1;
  const bool ph = a.nph > 1;   // ConvTranspose3d phase form: A padded, G strided by the phases
  if (a.asx != 1 || a.asy != 1 || a.asz != 1 || a.gpx || a.gpy || a.gpz) return 1;
  if (!ph && (a.apx || a.apy || a.apz || a.gsx != 1 || a.gsy != 1 || a.gsz != 1)) return 1;
  if (ph && a.bias_row) return 1;   // (its bias comes from chansum)
  // (16-channel inputs stay on wgrad2: d2.c1 of config 2 ran 65 us here
  // against 52 us there; every wider layer measured faster here)
  // (the ConvTranspose3d phase form also takes 16-channel inputs: the per-tap
  // wgrad_kernel is its alternative)
  if (a.ACs % (ph ? 16 : 32)) return 1;
  // 32-bit buffer offsets within one sample
  if ((double)a.AX * a.AY * a.AZ * a.ACs >= (double)(1 << 29) || (double)a.GX * a.GY * a.GZ * a.GCs >= (double)(1 << 29))
    return 1;
  const int T = a.KX * a.KY * a.KZ;
  const int ntz = cdiv(a.PZ, 16), TZ = cdiv(a.PZ, ntz), TZP = round_up(TZ, 4);
  const int HAZP = TZP + (a.KZ - 1) * a.adz;
  const int ncols = ph ? a.nph * a.GCout : a.GCs;
  // (phase form: a column chunk may span phases, a 4-column group may not)
  if (ncols % 32 || (ph && a.GCout % 4)) return 1;
  const int NS = ncols % 64 == 0 ? 4 : 2;
  const int CKG = NS * 16;
  const int nco = ncols / CKG;
  // Grid sized for 192 CUs: the weight-gradient branch overlaps the chain stream
  // (config 2 A/B, 3 reps: 192 -> 2.038-2.051, 176 -> 2.062-2.081, 208 -> 2.084-2.098,
  // 160 -> 2.083-2.090, side_cus() 224 -> 2.113-2.126 ms/step).
  // The small ConvTranspose3d layers (fewer than 32 output channels: u2.up /
  // u3.up of config 2, 0.2 GFLOP) on 64 CUs: their few tiles spread over 192
  // only take CUs from the chain (interleaved A/B, 3 runs: 1.998-2.002 ms per
  // config-2 step at 64, 2.014-2.020 at 32, 2.025-2.028 at 128, 2.024-2.031
  // at 192; the per-tap wgrad_kernel + chansum 2.017-2.019; a FLOP-
  // proportional grid for every wgrad3 layer measured equal).
  const int cus = ph && a.GCout < 32 ? 64 : 192;
  const int mss[3] = {9, 5, 3};
  const int ckas[3] = {64, 32, 16};
  const int txys[4][2] = {{4, 4}, {4, 2}, {2, 4}, {2, 2}};
  // (offering only the 4 x 4 tile measured 2.18 vs 2.11-2.12 ms per config-2
  // step; only 4 x 4 and 4 x 2: equal to all four)
  double best = 1e300;
  WGradArgs bestA = a;
  for (int ci = 0; ci < 3; ++ci) {
    const int CKA = ckas[ci];
    if (a.ACs % CKA) continue;
    for (int mi = 0; mi < 3; ++mi) {
      const int MS = mss[mi];
      const int rows = 64 * MS;
      const int TA = std::min(T, rows / CKA);
      if (TA < 1) continue;
      const int ntc = cdiv(T, TA), nci = a.ACs / CKA;
      const int used = TA * CKA;                   // useful rows of a block (the last tap chunk may be short)
      if (used * 3 < rows * 2 && MS > 3) continue;   // > 1/3 of the rows idle: a smaller MS fits better
      for (int ti = 0; ti < 4; ++ti) {
        const int TX = std::min(txys[ti][0], a.PX), TY = std::min(txys[ti][1], a.PY);
        const int HAX = TX + (a.KX - 1) * a.adx, HAY = TY + (a.KY - 1) * a.ady;
        const int HAV = HAX * HAY * HAZP, PTP = TX * TY * TZP;
        const int RSA = cm_stride(HAV), RSG = cm_stride(PTP);
        const long lds = ((long)(CKA + 1) * RSA + (long)(CKG + 1) * RSG + PTP / 4 + 256) * 4;
        if (lds > 150 * 1024) continue;
        // two resident blocks (LDS <= 80 KB) overlap one's staging with the
        // other's MFMAs; one block pays both
        const int occ = lds <= 80 * 1024 ? 2 : 1;
        const long tiles = (long)a.B * cdiv(a.PX, TX) * cdiv(a.PY, TY) * ntz;
        const long per = (long)ntc * nci * nco;
        const long kb = std::max(1L, std::min(tiles, (long)cus * occ / per));
        const long tpb = cdiv((int)tiles, (int)kb);
        const double mfma = (double)PTP / 4 * (MS * NS * 32.0 + 150.0);
        // staging: ~16 B a cycle per CU plus ~2500 cycles of latency per round
        // of kW3Loads loads in flight
        const double f4 = ((double)HAV * CKA + (double)PTP * CKG) / 4;
        const double stage = f4 * 16 / 16.0 + 2500.0 * std::ceil(f4 / (256.0 * kW3Loads));
        const double slab = (double)rows * CKG * 4 / 16.0;
        const long blocks = kb * per;
        const double rounds = std::ceil((double)blocks / ((double)cus * occ));
        const double tile_t = occ == 2 ? std::max(mfma, stage) * 1.15 * 2 : mfma + stage;
        const double cost = rounds * (tpb * tile_t + slab);
        // the finalize reads every slab once: ~3.3 KB a cycle chip-wide
        const double fin = (double)blocks * (used + 1) * CKG * 4 / 3300.0;
        if (cost + fin < best) {
          best = cost + fin;
          WGradArgs c = a;
          c.CKA = CKA;
          c.CKG = CKG;
          c.MS = MS;
          c.NS = NS;
          c.TA = TA;
          c.TG = 1;
          c.ntc = ntc;
          c.nci = nci;
          c.nco = nco;
          c.mchunks = ntc * nci;
          c.nchunks = nco;
          c.TX = TX;
          c.TY = TY;
          c.TZ = TZ;
          c.TZP = TZP;
          c.HAX = HAX;
          c.HAY = HAY;
          c.HAZP = HAZP;
          c.PA2 = RSA;
          c.PG2 = RSG;
          c.ntx = cdiv(a.PX, TX);
          c.nty = cdiv(a.PY, TY);
          c.ntz = ntz;
          c.KB = (int)kb;
          c.lds_bytes = (int)lds;
          c.fHAZ = FastDiv(HAZP);
          c.fHAY = FastDiv(HAY);
          c.fTY = FastDiv(TY);
          c.fTZ = FastDiv(TZP);   // G tile z rows (the staging's voxel decode)
          c.v2 = 3;
          bestA = c;
        }
      }
    }
  }
  if (bestA.v2 != 3) return 1;
  a = bestA;
  a.Mtot = T * a.ACs + (a.bias_row ? 1 : 0);
  a.Ntot = ncols;
  if (getenv("HCU_CONV2_LOG"))
    fprintf(stderr, "wgrad3 plan: A%dx%dx%d ACs%d P%dx%dx%d K%dx%dx%d nph%d | CKA%d MS%d NS%d TA%d T%dx%dx%d(%d) KB%d m%d n%d lds%d\n",
            a.AX, a.AY, a.AZ, a.ACs, a.PX, a.PY, a.PZ, a.KX, a.KY, a.KZ, a.nph, a.CKA, a.MS, a.NS, a.TA, a.TX, a.TY,
            a.TZ, a.TZP, a.KB, a.mchunks, a.nchunks, a.lds_bytes);
  return 0;
}

int launch_wgrad3(const WGradArgs &a, hipStream_t s) {
  const dim3 grid(a.KB, a.mchunks, a.nchunks);
  const int T = a.KX * a.KY * a.KZ;
  const double fl = a.flops > 0 ? a.flops : 2.0 * a.B * a.PX * a.PY * a.PZ * (double)T * a.ACs * a.GCs;
  const double by = 4.0 * ((double)a.B * a.AX * a.AY * a.AZ * a.ACs + (double)a.B * a.GX * a.GY * a.GZ * a.GCs);
  bool ok = false;
#define W3(MS_, NS_)                                                                       \
  if (!ok && a.MS == MS_ && a.NS == NS_) {                                                 \
    HCU_TIMED(s, "wgrad3_kernel<" #MS_ "," #NS_ ">", fl, by,                                \
              HCU_LAUNCH((wgrad3_kernel<MS_, NS_>), grid, dim3(256), a.lds_bytes, s, a)); \
    ok = true;                                                                             \
  }
  W3(3, 2) W3(5, 2) W3(9, 2) W3(3, 4) W3(5, 4) W3(9, 4)
#undef W3
  if (!ok) return fail(4, "wgrad3: unsupported variant");
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu
