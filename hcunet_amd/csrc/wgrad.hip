// Weight gradient of Conv3d / ConvTranspose3d on fp32 MFMA.
//
// dW is a GEMM whose reduction dimension is the voxel grid (millions of
// voxels) and whose M x N extent is tiny (taps*Cin x Cout).  Each workgroup
// owns a (row chunk, col chunk) of dW and a strided subset of the voxel tiles;
// it stages the activation halo (BatchNorm+ReLU applied on load) and the
// gradient tile in LDS, the four waves split the voxel k-steps, and the
// per-wave accumulators are summed through LDS in a fixed order and written as
// one fp32 partial slab per workgroup.  wgrad_finalize sums the slabs in fp64
// in a fixed order (bitwise reproducible, no atomics) and scatters them into
// the PyTorch weight layout, undoing the cat(U,U) weight fold
// (hcat/unet.py:310-313) and the grouped-conv block diagonal.
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <cstdlib>

namespace hcu {

bool wgrad2_disabled() {   // HCU_NO_WGRAD2=1 forces the generic kernel (A/B testing)
  static const bool off = [] {
    const char *e = getenv("HCU_NO_WGRAD2");
    return e && e[0] == '1';
  }();
  return off;
}

template <int NS, int MSMAX>
__global__ void __launch_bounds__(256) wgrad_kernel(const WGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kb = blockIdx.x;
  const int T = a.KX * a.KY * a.KZ;
  const int CKA = a.CKA, CKG = a.CKG;
  // block -> (tap chunk, channel chunks)
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
  const bool bias_block = a.bias_row && tapc == 0 && cic == 0;
  const int PA = a.PA, PG = a.PG;
  float *alds = smem;
  float *glds = smem + CKA * PA;
  const int HAZ = a.HAZ, HAYZ = a.HAY * a.HAZ, HAV = a.HAX * HAYZ;
  const int HGZ = a.HGZ, HGYZ = a.HGY * a.HGZ, HGV = a.HGX * HGYZ;
  const int MS = a.MS;

  int aoff[MSMAX];
#pragma unroll
  for (int ms = 0; ms < MSMAX; ++ms) {
    const int lr = ms * 16 + (lane & 15);
    int off = -2;
    if (a.taps_rows) {
      const int tl = lr / CKA, c = lr % CKA, ta = t0 + tl;
      if (tl < a.TA) {
        if (ta < T && ci0 + c < a.ACs) {
          const int kz = ta % a.KZ, q = ta / a.KZ, ky = q % a.KY, kx = q / a.KY;
          off = c * PA + kx * a.adx * HAYZ + ky * a.ady * HAZ + kz * a.adz;
        }
      } else if (bias_block && lr == a.TA * CKA) {
        off = -1;
      }
    } else {
      if (lr < CKA && ci0 + lr < a.ACs) off = lr * PA;
    }
    aoff[ms] = off;
  }
  int goff[NS];
#pragma unroll
  for (int ns = 0; ns < NS; ++ns) {
    const int lc = ns * 16 + (lane & 15);
    int off = -2;
    if (a.taps_rows) {
      if (lc < CKG && co0 + lc < a.GCs) off = lc * PG;
    } else {
      const int tl = lc / CKG, o = lc % CKG, tg = t0 + tl;
      if (tl < a.TG && tg < T && co0 + o < a.GCs) {
        const int kz = tg % a.KZ, q = tg / a.KZ, ky = q % a.KY, kx = q / a.KY;
        off = o * PG + kx * a.gdx * HGYZ + ky * a.gdy * HGZ + kz * a.gdz;
      }
    }
    goff[ns] = off;
  }

  floatx4 acc[MSMAX][NS];
#pragma unroll
  for (int ms = 0; ms < MSMAX; ++ms)
#pragma unroll
    for (int ns = 0; ns < NS; ++ns) acc[ms][ns] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int PT = a.TX * a.TY * a.TZ;
  const int nks = (PT + 3) >> 2;
  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int CA4 = CKA / 4, CG4 = CKG / 4;

  for (int tt = kb; tt < total; tt += a.KB) {
    const int b = tt / ntiles;
    int tile = tt % ntiles;
    const int tzi = tile % a.ntz;
    tile /= a.ntz;
    const int tyi = tile % a.nty, txi = tile / a.nty;
    const int px0 = txi * a.TX, py0 = tyi * a.TY, pz0 = tzi * a.TZ;
    lds_barrier();
    {  // stage A halo
      const int gx0 = px0 * a.asx - a.apx, gy0 = py0 * a.asy - a.apy, gz0 = pz0 * a.asz - a.apz;
      for (int idx = tid; idx < HAV * CA4; idx += 256) {
        const int c4 = idx % CA4, v = idx / CA4;
        int q, hz, hx, hy;
        a.fHAZ.divmod(v, q, hz);
        a.fHAY.divmod(q, hx, hy);
        const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
        const int c = ci0 + c4 * 4;
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)gx < (unsigned)a.AX && (unsigned)gy < (unsigned)a.AY &&
            (unsigned)gz < (unsigned)a.AZ && c < a.ACs) {
          val = *reinterpret_cast<const float4 *>(
              a.A + ((((size_t)b * a.AX + gx) * a.AY + gy) * a.AZ + gz) * a.ACs + c);
          if (a.a_scale) {
            const float4 sc = *reinterpret_cast<const float4 *>(a.a_scale + c);
            const float4 sh = *reinterpret_cast<const float4 *>(a.a_shift + c);
            val.x = fmaxf(fmaf(val.x, sc.x, sh.x), 0.f);
            val.y = fmaxf(fmaf(val.y, sc.y, sh.y), 0.f);
            val.z = fmaxf(fmaf(val.z, sc.z, sh.z), 0.f);
            val.w = fmaxf(fmaf(val.w, sc.w, sh.w), 0.f);
          }
        }
        float *dst = alds + (c4 * 4) * PA + v;
        dst[0] = val.x;
        dst[PA] = val.y;
        dst[2 * PA] = val.z;
        dst[3 * PA] = val.w;
      }
    }
    {  // stage G halo
      const int gx0 = px0 * a.gsx - a.gpx, gy0 = py0 * a.gsy - a.gpy, gz0 = pz0 * a.gsz - a.gpz;
      for (int idx = tid; idx < HGV * CG4; idx += 256) {
        const int c4 = idx % CG4, v = idx / CG4;
        int q, hz, hx, hy;
        a.fHGZ.divmod(v, q, hz);
        a.fHGY.divmod(q, hx, hy);
        const int gx = gx0 + hx, gy = gy0 + hy, gz = gz0 + hz;
        const int c = co0 + c4 * 4;
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)gx < (unsigned)a.GX && (unsigned)gy < (unsigned)a.GY &&
            (unsigned)gz < (unsigned)a.GZ && c < a.GCs) {
          val = *reinterpret_cast<const float4 *>(
              a.G + ((((size_t)b * a.GX + gx) * a.GY + gy) * a.GZ + gz) * a.GCs + c);
        }
        float *dst = glds + (c4 * 4) * PG + v;
        dst[0] = val.x;
        dst[PG] = val.y;
        dst[2 * PG] = val.z;
        dst[3 * PG] = val.w;
      }
    }
    lds_barrier();
    for (int ks = wave; ks < nks; ks += 4) {
      const int p = ks * 4 + (lane >> 4);
      const bool pv = p < PT;
      const int pp = pv ? p : 0;
      int q, lz, lx, ly;
      a.fTZ.divmod(pp, q, lz);
      a.fTY.divmod(q, lx, ly);
      const int ah = lx * a.asx * HAYZ + ly * a.asy * HAZ + lz * a.asz;
      const int gh = lx * a.gsx * HGYZ + ly * a.gsy * HGZ + lz * a.gsz;
      float bv[NS];
#pragma unroll
      for (int ns = 0; ns < NS; ++ns) bv[ns] = (pv && goff[ns] >= 0) ? glds[goff[ns] + gh] : 0.f;
#pragma unroll
      for (int ms = 0; ms < MSMAX; ++ms) {
        if (ms < MS) {
          const int o = aoff[ms];
          float av = (o >= 0) ? alds[(o >= 0 ? o : 0) + ah] : (o == -1 ? 1.f : 0.f);
          av = pv ? av : 0.f;
#pragma unroll
          for (int ns = 0; ns < NS; ++ns)
            acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[ns], acc[ms][ns], 0, 0, 0);
        }
      }
    }
  }

  // ---- cross-wave reduction in a fixed order, then one partial slab write
  lds_barrier();
  float *red = smem;  // [MS*NS][64][4]
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ms = 0; ms < MSMAX; ++ms) {
        if (ms < MS) {
#pragma unroll
          for (int ns = 0; ns < NS; ++ns) {
            float *dst = red + ((ms * NS + ns) * 64 + lane) * 4;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[r] = (w == 0) ? acc[ms][ns][r] : dst[r] + acc[ms][ns][r];
          }
        }
      }
    }
    lds_barrier();
  }
  const int nel = MS * NS * 256;
  for (int idx = tid; idx < nel; idx += 256) {
    const int r = idx & 3, ln = (idx >> 2) & 63, ti = idx >> 8;
    const int ms = ti / NS, ns = ti % NS;
    const int lr = ms * 16 + (ln >> 4) * 4 + r;
    const int lc = ns * 16 + (ln & 15);
    int grow = -1, gcol = -1;
    if (a.taps_rows) {
      const int tl = lr / CKA, ta = t0 + tl;
      if (tl < a.TA) {
        const int ci = ci0 + lr % CKA;
        if (ta < T && ci < a.ACs) grow = ta * a.ACs + ci;
      } else if (bias_block && lr == a.TA * CKA) {
        grow = T * a.ACs;
      }
      if (lc < CKG && co0 + lc < a.GCs) gcol = co0 + lc;
    } else {
      if (lr < CKA && ci0 + lr < a.ACs) grow = ci0 + lr;
      const int tl = lc / CKG, o = lc % CKG, tg = t0 + tl;
      if (tl < a.TG && tg < T && co0 + o < a.GCs) gcol = tg * a.GCs + co0 + o;
    }
    if (grow >= 0 && gcol >= 0)
      a.partial[((size_t)kb * a.Mtot + grow) * a.Ntot + gcol] = red[idx];
  }
}

// ---------------------------------------------------------------------------
// wgrad2: Conv3d weight gradient with b128 operand reads.
//   dW[(t,ci)][co] = sum_p act(A[p + off(t)][ci]) * G[p][co]   (+ bias row: sum_p G[p][co])
// K = voxels p of a TX*TY*TZP tile (TZP = TZ rounded up to 4, the extra z
// positions have G = 0).  A K-step is 16 voxels: lane group g takes the 4
// z-consecutive voxels 4g..4g+3 with ONE ds_read_b128 from a channel-major LDS
// image, component j feeding MFMA j (a permutation of the voxel sum).  To keep
// every b128 16-byte aligned the A halo is staged once per kz tap shift
// (image kz holds A[.., z + kz*dz]); rows of invalid (tap, channel) pairs read
// a zero image and the bias row reads an image of ones.
// Workgroups are persistent over tiles and each writes ONE fp32 partial slab;
// wgrad_finalize sums the slabs in a fixed order.
template <int NS, int MS>
__global__ void __launch_bounds__(256) wgrad2_kernel(const WGradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int T = a.KX * a.KY * a.KZ;
  const int CKA = a.CKA, CKG = a.CKG;
  const int tapc = blockIdx.y / a.nci, cic = blockIdx.y % a.nci, coc = blockIdx.z;
  const int ci0 = cic * CKA, co0 = coc * CKG;
  const int t0 = tapc * a.TA;
  const bool bias_block = a.bias_row && tapc == 0 && cic == 0;
  const int PA = a.PA2, PG = a.PG2;
  const int HAZP = a.HAZP, HAYZP = a.HAY * a.HAZP;
  const int nimg = a.KZ * CKA;                 // A images: [kz][c]
  float *alds = smem;                          // [nimg + 2][PA]  (+ zero, ones)
  float *glds = alds + (size_t)(nimg + 2) * PA;  // [CKG + 1][PG]   (+ zero)
  int *hvtab = reinterpret_cast<int *>(glds + (size_t)(CKG + 1) * PG);
  const int TZP = a.TZP;
  const int PT4 = a.TX * a.TY * TZP / 4;       // voxel quads of a tile
  const int nks = (PT4 + 3) / 4;               // 16-voxel K-steps (tail quads: G = 0)

  // zero everything once: padded z positions and unused rows stay finite (0)
  for (int i = tid; i < (nimg + 2) * PA + (CKG + 1) * PG; i += 256) smem[i] = 0.f;
  lds_barrier();
  for (int i = tid; i < PA; i += 256) alds[(size_t)(nimg + 1) * PA + i] = 1.f;
  for (int q = tid; q < nks * 4; q += 256) {
    const int p = q * 4;
    const int lz = p % TZP, r = p / TZP, ly = r % a.TY, lx = r / a.TY;
    hvtab[q] = q < PT4 ? lx * HAYZP + ly * HAZP + lz : 0;
  }
  // per-lane row images (A side) and column images (G side)
  int aoff[MS];
#pragma unroll
  for (int ms = 0; ms < MS; ++ms) {
    const int lr = ms * 16 + r16;
    int off = nimg * PA;  // zero image
    const int tl = lr / CKA, c = lr % CKA, ta = t0 + tl;
    if (tl < a.TA) {
      if (ta < T && ci0 + c < a.ACs) {
        const int kz = ta % a.KZ, q = ta / a.KZ, ky = q % a.KY, kx = q / a.KY;
        off = (kz * CKA + c) * PA + kx * a.adx * HAYZP + ky * a.ady * HAZP;
      }
    } else if (bias_block && lr == a.TA * CKA) {
      off = (nimg + 1) * PA;  // ones image
    }
    aoff[ms] = off;
  }
  int goff[NS];
#pragma unroll
  for (int ns = 0; ns < NS; ++ns) {
    const int lc = ns * 16 + r16;
    goff[ns] = (lc < CKG && co0 + lc < a.Ntot) ? lc * PG : CKG * PG;
  }
  // G channel base and stride phase of this block's columns (phase form: the
  // chunk lies in one phase; else phase 0, columns = channels)
  int gq[3] = {0, 0, 0}, gcb = co0;
  if (a.nph > 1) {
    const int q = co0 / a.GCout;
    gcb = co0 - q * a.GCout;
    gq[2] = q % a.phz;
    gq[1] = (q / a.phz) % a.phy;
    gq[0] = q / (a.phz * a.phy);
  }

  floatx4 acc[MS][NS];
#pragma unroll
  for (int ms = 0; ms < MS; ++ms)
#pragma unroll
    for (int ns = 0; ns < NS; ++ns) acc[ms][ns] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int ntiles = a.ntx * a.nty * a.ntz;
  const int total = a.B * ntiles;
  const int CA4 = CKA / 4, CG4 = CKG / 4;
  const int HAV = a.HAX * a.HAY * a.HAZ;        // real halo extent
  const int PTr = a.TX * a.TY * a.TZ;           // real tile extent

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
    // ---- A halo -> one channel-major image per kz shift (act applied, 0 outside)
    for (int base = tid; base < HAV * CA4; base += 4 * 256) {
      float4 val[4];
      int vv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int idx = base + u * 256;
        val[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        vv[u] = -1;
        if (idx < HAV * CA4) {
          const int c4 = idx % CA4, v = idx / CA4;
          int q, hz, hx, hy;
          a.fHAZ.divmod(v, q, hz);
          a.fHAY.divmod(q, hx, hy);
          vv[u] = (((hx << 10) | hy) << 10 | hz) * 8 + c4;  // c4 < 8
          const int gx = px0 + hx - a.apx, gy = py0 + hy - a.apy, gz = pz0 + hz - a.apz;
          const int c = ci0 + c4 * 4;
          if ((unsigned)gx < (unsigned)a.AX && (unsigned)gy < (unsigned)a.AY && (unsigned)gz < (unsigned)a.AZ &&
              c < a.ACs) {
            val[u] = *reinterpret_cast<const float4 *>(
                a.A + ((((size_t)b * a.AX + gx) * a.AY + gy) * a.AZ + gz) * a.ACs + c);
            if (a.a_scale) {
              const float4 sc = *reinterpret_cast<const float4 *>(a.a_scale + c);
              const float4 sh = *reinterpret_cast<const float4 *>(a.a_shift + c);
              val[u].x = fmaxf(fmaf(val[u].x, sc.x, sh.x), 0.f);
              val[u].y = fmaxf(fmaf(val[u].y, sc.y, sh.y), 0.f);
              val[u].z = fmaxf(fmaf(val[u].z, sc.z, sh.z), 0.f);
              val[u].w = fmaxf(fmaf(val[u].w, sc.w, sh.w), 0.f);
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (vv[u] < 0) continue;
        const int c4 = vv[u] & 7, pk = vv[u] >> 3;
        const int hz = pk & 1023, hy = (pk >> 10) & 1023, hx = pk >> 20;
        for (int kz = 0; kz < a.KZ; ++kz) {
          const int z = hz - kz * a.adz;
          if (z < 0 || z >= HAZP) continue;
          float *d = alds + (size_t)(kz * CKA + c4 * 4) * PA + hx * HAYZP + hy * HAZP + z;
          d[0] = val[u].x;
          d[PA] = val[u].y;
          d[2 * PA] = val[u].z;
          d[3 * PA] = val[u].w;
        }
      }
    }
    // ---- G tile -> channel-major [co][p] with z rows of TZP (0 outside)
    for (int base = tid; base < PTr * CG4; base += 4 * 256) {
      float4 val[4];
      int pp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int idx = base + u * 256;
        val[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        pp[u] = -1;
        if (idx < PTr * CG4) {
          const int c4 = idx % CG4, p = idx / CG4;
          int q, lz, lx, ly;
          a.fTZ.divmod(p, q, lz);
          a.fTY.divmod(q, lx, ly);
          pp[u] = ((lx * a.TY + ly) * TZP + lz) * 32 + c4;  // c4 < 32
          const int gx = px0 + lx, gy = py0 + ly, gz = pz0 + lz;
          const int c = gcb + c4 * 4;
          if (gx < a.PX && gy < a.PY && gz < a.PZ && c < a.GCs && co0 + c4 * 4 < a.Ntot) {
            const size_t go = ((((size_t)b * a.GX + gx * a.gsx + gq[0]) * a.GY + gy * a.gsy + gq[1]) * a.GZ +
                               gz * a.gsz + gq[2]) * a.GCs + c;
            val[u] = *reinterpret_cast<const float4 *>(a.G + go);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (pp[u] < 0) continue;
        const int c4 = pp[u] & 31, p = pp[u] >> 5;
        float *d = glds + (size_t)(c4 * 4) * PG + p;
        d[0] = val[u].x;
        d[PG] = val[u].y;
        d[2 * PG] = val[u].z;
        d[3 * PG] = val[u].w;
      }
    }
    lds_barrier();
    // ---- MFMA over the tile's voxels: wave w takes K-steps w, w+4, ...
    for (int ks = wave; ks < nks; ks += 4) {
      const int q = ks * 4 + g;
      const int hv = hvtab[q];
      floatx4 bv[NS], av[MS];
#pragma unroll
      for (int ns = 0; ns < NS; ++ns)
        bv[ns] = *reinterpret_cast<const floatx4 *>(glds + goff[ns] + q * 4);
#pragma unroll
      for (int ms = 0; ms < MS; ++ms)
        av[ms] = *reinterpret_cast<const floatx4 *>(alds + aoff[ms] + hv);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int ms = 0; ms < MS; ++ms)
#pragma unroll
            for (int ns = 0; ns < NS; ++ns)
              acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ms][c], bv[ns][c], acc[ms][ns], 0, 0, 0);
    }
  }

  // ---- cross-wave reduction in a fixed order, then one partial slab write
  lds_barrier();
  float *red = smem;  // [MS*NS][64][4]
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ms = 0; ms < MS; ++ms) {
        {
#pragma unroll
          for (int ns = 0; ns < NS; ++ns) {
            float *dst = red + ((ms * NS + ns) * 64 + lane) * 4;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[r] = (w == 0) ? acc[ms][ns][r] : dst[r] + acc[ms][ns][r];
          }
        }
      }
    }
    lds_barrier();
  }
  const int kb = kbi;
  const int nel = MS * NS * 256;
  for (int idx = tid; idx < nel; idx += 256) {
    const int r = idx & 3, ln = (idx >> 2) & 63, ti = idx >> 8;
    const int ms = ti / NS, ns = ti % NS;
    const int lr = ms * 16 + (ln >> 4) * 4 + r;
    const int lc = ns * 16 + (ln & 15);
    int grow = -1, gcol = -1;
    const int tl = lr / CKA, ta = t0 + tl;
    if (tl < a.TA) {
      const int ci = ci0 + lr % CKA;
      if (ta < T && ci < a.ACs) grow = ta * a.ACs + ci;
    } else if (bias_block && lr == a.TA * CKA) {
      grow = T * a.ACs;
    }
    if (lc < CKG && co0 + lc < a.Ntot) gcol = co0 + lc;
    if (grow >= 0 && gcol >= 0)
      a.partial[((size_t)kb * a.Mtot + grow) * a.Ntot + gcol] = red[idx];
  }
}

// Re-plans a Conv3d wgrad (taps_rows, stride-1 operands) for wgrad2_kernel:
// tile, padded LDS images, persistent grid.  Returns 0 when wgrad2 applies.
static int plan_wgrad2(WGradArgs &a, int target_blocks) {
  a.v2 = 0;
  // (the ConvTranspose3d phase form: A zero-padded, G strided by the phases)
  const bool ph = a.nph > 1;
  if (!a.taps_rows || a.asx != 1 || a.asy != 1 || a.asz != 1 || a.gpx || a.gpy || a.gpz ||
      (!ph && (a.gsx != 1 || a.gsy != 1 || a.gsz != 1 || a.apx || a.apy || a.apz)))
    return 1;
  if (a.CKA % 4 || a.CKA > 32 || a.CKG > 128) return 1;
  const int ntz = cdiv(a.PZ, 16);
  const int TZ = cdiv(a.PZ, ntz);
  const int TZP = round_up(TZ, 4);
  const int HAZ = TZ + (a.KZ - 1) * a.adz;
  const int HAZP = TZP;  // image z rows: the voxels p read z in [0, TZP)
  (void)HAZ;
  const int nimg = a.KZ * a.CKA;
  const int txys[5][2] = {{8, 8}, {6, 8}, {4, 8}, {4, 4}, {2, 4}};
  int best = -1;
  long lds = 0;
  for (int i = 0; i < 5; ++i) {
    const int TX = std::min(txys[i][0], a.PX), TY = std::min(txys[i][1], a.PY);
    const int HAX = TX + (a.KX - 1) * a.adx, HAY = TY + (a.KY - 1) * a.ady;
    int PA = HAX * HAY * HAZP;
    PA = round_up(PA, 64) + 4;
    const int nq = round_up(TX * TY * TZP / 4, 4);   // quads incl. the zero tail
    int PG = nq * 4;
    PG = round_up(PG, 64) + 4;
    const long bytes = ((long)(nimg + 2) * PA + (long)(a.CKG + 1) * PG + nq) * 4;
    const long red = (long)a.MS * a.NS * 256 * 4;
    const long need = std::max(bytes, red);
    if (need <= 48 * 1024 || i == 4) {
      best = i;
      lds = need;
      a.TX = TX;
      a.TY = TY;
      a.HAX = HAX;
      a.HAY = HAY;
      a.PA2 = PA;
      a.PG2 = PG;
      break;
    }
  }
  if (best < 0 || lds > 64 * 1024) return 1;
  a.TZ = TZ;
  a.TZP = TZP;
  a.HAZ = HAZ;
  a.HAZP = HAZP;
  a.lds_bytes = (int)lds;
  a.fHAZ = FastDiv(a.HAZ);
  a.fHAY = FastDiv(a.HAY);
  a.fTZ = FastDiv(a.TZ);
  a.fTY = FastDiv(a.TY);
  a.ntx = cdiv(a.PX, a.TX);
  a.nty = cdiv(a.PY, a.TY);
  a.ntz = ntz;
  const long total = (long)a.B * a.ntx * a.nty * a.ntz;
  const long per = (long)a.mchunks * a.nchunks;
  a.occ = std::max(1, std::min(8, (int)(160 * 1024 / a.lds_bytes)));
  // 192 CUs leaves room for the chain stream (config 2 A/B, 3 reps: 192 -> 2.038-2.051,
  // 160 -> 2.060-2.067, 128 -> 2.063-2.081, 224 -> 2.070-2.082 ms/step).
  long kb = std::max(1L, 192L * a.occ / per);
  kb = std::min(kb, total);
  a.KB = (int)kb;
  a.v2 = 1;
  (void)target_blocks;
  return 0;
}

int plan_wgrad(WGradArgs &a, int target_blocks) {
  const int T = a.KX * a.KY * a.KZ;
  a.ACr = a.GCr = 0;   // (bwgrad only)
  if (a.ACs % 4 || a.GCs % 4) return fail(1, "wgrad: channel strides must be multiples of 4");
  if (a.PX <= 0 || a.PY <= 0 || a.PZ <= 0) return fail(2, "wgrad: empty grid");
  const int nss[3] = {4, 2, 1};
  a.NS = 0;
  for (int i = 0; i < 3; ++i) {
    const int NS = nss[i], MSMAX = 16 / NS;
    const int rows = MSMAX * 16, cols = NS * 16;
    if (a.taps_rows) {
      if (NS > 1 && (NS / 2) * 16 >= a.GCs) continue;  // do not waste columns
      const int brow = a.bias_row ? 1 : 0;
      int cka = ((rows - brow) / T) / 4 * 4;
      int ta = T;
      if (cka < 4) {  // too many taps for one block: split the taps
        cka = 4;
        ta = (rows - brow) / 4;
      }
      cka = std::min(cka, a.ACs);
      if (a.nph > 1) cka = std::min(cka, 32);   // wgrad2's A images: at most 32 channels a block
      a.CKA = cka;
      a.TA = ta;
      a.TG = 1;
      a.CKG = std::min(a.GCs, cols);
      if (a.nph > 1) {   // column chunks inside one phase: CKG divides GCout
        int ckg = std::min(a.GCout, cols) / 4 * 4;
        while (ckg > 4 && a.GCout % ckg) ckg -= 4;
        if (ckg < 4 || a.GCout % ckg) return fail(4, "wgrad: phase columns need Cout % 4 == 0");
        a.CKG = ckg;
      }
      a.mloc = ta * cka + brow;
      a.nloc = a.CKG;
    } else {
      int ckg = (cols / T) / 4 * 4;
      int tg = T;
      if (ckg < 4) {
        ckg = 4;
        tg = cols / 4;
      }
      ckg = std::min(ckg, a.GCs);
      a.CKG = ckg;
      a.TG = tg;
      a.TA = 1;
      a.CKA = std::min(a.ACs, rows);
      a.mloc = a.CKA;
      a.nloc = tg * ckg;
    }
    a.NS = NS;
    a.MS = cdiv(a.mloc, 16);
    break;
  }
  if (!a.NS) return fail(4, "wgrad: no tile");
  a.nci = cdiv(a.ACs, a.CKA);
  const int ncols = a.nph > 1 ? a.nph * a.GCout : a.GCs;   // taps_rows columns
  a.nco = cdiv(ncols, a.CKG);
  a.ntc = a.taps_rows ? cdiv(T, a.TA) : cdiv(T, a.TG);
  a.mchunks = a.taps_rows ? a.ntc * a.nci : a.nci;
  a.nchunks = a.taps_rows ? a.nco : a.ntc * a.nco;
  a.Mtot = a.taps_rows ? T * a.ACs + (a.bias_row ? 1 : 0) : a.ACs;
  a.Ntot = a.taps_rows ? ncols : T * a.GCs;
  const int ntz = cdiv(a.PZ, 16);
  a.TZ = cdiv(a.PZ, ntz);
  int txy = std::max(1, 256 / a.TZ);
  for (;;) {
    int TX = 1;
    while ((TX + 1) * (TX + 1) <= txy) ++TX;
    int TY = std::max(1, txy / TX);
    TX = std::min(TX, a.PX);
    TY = std::min(TY, a.PY);
    a.TX = TX;
    a.TY = TY;
    a.HAX = (TX - 1) * a.asx + (a.KX - 1) * a.adx + 1;
    a.HAY = (TY - 1) * a.asy + (a.KY - 1) * a.ady + 1;
    a.HAZ = (a.TZ - 1) * a.asz + (a.KZ - 1) * a.adz + 1;
    a.HGX = (TX - 1) * a.gsx + (a.KX - 1) * a.gdx + 1;
    a.HGY = (TY - 1) * a.gsy + (a.KY - 1) * a.gdy + 1;
    a.HGZ = (a.TZ - 1) * a.gsz + (a.KZ - 1) * a.gdz + 1;
    const int HAV = a.HAX * a.HAY * a.HAZ, HGV = a.HGX * a.HGY * a.HGZ;
    a.PA = HAV + ((1 - HAV % 32) + 32) % 32;
    a.PG = HGV + ((1 - HGV % 32) + 32) % 32;
    long lds = ((long)a.CKA * a.PA + (long)a.CKG * a.PG) * 4;
    const long red = (long)a.MS * a.NS * 256 * 4;
    if (lds < red) lds = red;
    if (lds <= 65536 || txy == 1) {
      a.lds_bytes = (int)lds;
      break;
    }
    txy = std::max(1, txy / 2);
  }
  if (a.lds_bytes > 65536) return fail(4, "wgrad: tile does not fit LDS");
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
  long kb = std::max(1L, (long)target_blocks * side_cus() / 256 / per);
  kb = std::min(kb, total);
  a.KB = (int)kb;
  if (plan_wgrad3(a) == 0) return 0;   // deep layers / ConvTranspose3d phase form: the output-split form
  if (a.nph > 1) {   // the phase form runs on wgrad2 only
    if (wgrad2_disabled() || plan_wgrad2(a, target_blocks) != 0)
      return fail(4, "wgrad: no wgrad2 tile for the ConvTranspose3d phase form");
    return 0;
  }
  if (plan_wgrad8(a) != 0 && !wgrad2_disabled()) plan_wgrad2(a, target_blocks);
  return 0;
}

int launch_wgrad(const WGradArgs &a, hipStream_t s) {
  if (a.use_bw) return launch_bwgrad(a, s);
  if (a.v2 == 2) return launch_wgrad8(a, s);
  if (a.v2 == 3) return launch_wgrad3(a, s);
  const dim3 grid(a.KB, a.mchunks, a.nchunks);
  const int T = a.KX * a.KY * a.KZ;
  if (a.v2) {
    const double fl2 = a.flops > 0 ? a.flops
                                   : 2.0 * a.B * a.PX * a.PY * a.PZ * (double)T * a.ACs * a.GCs;
    const double by2 = 4.0 * ((double)a.B * a.AX * a.AY * a.AZ * a.ACs +
                              (double)a.B * a.GX * a.GY * a.GZ * a.GCs);
    bool ok = false;
#define W2(NS_, MS_)                                                                       \
  if (!ok && a.NS == NS_ && a.MS == MS_) {                                                 \
    HCU_TIMED(s, "wgrad2_kernel<" #NS_ "," #MS_ ">", fl2, by2,                              \
              HCU_LAUNCH((wgrad2_kernel<NS_, MS_>), grid, dim3(256), a.lds_bytes, s, a)); \
    ok = true;                                                                             \
  }
    W2(1, 1) W2(1, 2) W2(1, 3) W2(1, 4) W2(1, 5) W2(1, 6) W2(1, 7) W2(1, 8)
    W2(1, 9) W2(1, 10) W2(1, 11) W2(1, 12) W2(1, 13) W2(1, 14) W2(1, 15) W2(1, 16)
    W2(2, 1) W2(2, 2) W2(2, 3) W2(2, 4) W2(2, 5) W2(2, 6) W2(2, 7) W2(2, 8)
    W2(4, 1) W2(4, 2) W2(4, 3) W2(4, 4)
#undef W2
    if (!ok) return fail(4, "wgrad2: unsupported variant");
    HCU_CHECK_LAUNCH();
    return 0;
  }
  const double fl = a.flops > 0 ? a.flops
                                : 2.0 * a.B * a.PX * a.PY * a.PZ * (double)T * a.ACs * a.GCs;
  const double by = 4.0 * ((double)a.B * a.AX * a.AY * a.AZ * a.ACs +
                           (double)a.B * a.GX * a.GY * a.GZ * a.GCs +
                           (double)wgrad_partial_floats(a));
  if (a.NS == 4) {
    HCU_TIMED(s, "wgrad_kernel<4,4>", fl, by,
              HCU_LAUNCH((wgrad_kernel<4, 4>), grid, dim3(256), a.lds_bytes, s, a));
  } else if (a.NS == 2) {
    HCU_TIMED(s, "wgrad_kernel<2,8>", fl, by,
              HCU_LAUNCH((wgrad_kernel<2, 8>), grid, dim3(256), a.lds_bytes, s, a));
  } else {
    HCU_TIMED(s, "wgrad_kernel<1,16>", fl, by,
              HCU_LAUNCH((wgrad_kernel<1, 16>), grid, dim3(256), a.lds_bytes, s, a));
  }
  HCU_CHECK_LAUNCH();
  return 0;
}

// Sum of the KB partial slabs per dW element, deterministic and parallel over
// both the elements and the slabs: S threads share one element (each sums the
// slabs k = s, s+S, ... in fp64), then the S sums are combined in LDS in a
// fixed order.  The result is scattered into the PyTorch weight layout.
// S == 0 selects the tiled form (wgrad_finalize_tile) for the large layers.
__device__ __forceinline__ void wgrad_finalize_body(const WGradFinalize &f, int S, double *red);
__device__ __forceinline__ void wgrad_finalize_body4(const WGradFinalize &f, int S, double *red);
__device__ __forceinline__ void wgrad_finalize_emit(const WGradFinalize &f, int64_t idx, double s);
__device__ __forceinline__ void wgrad_finalize_tile(const WGradFinalize &f, int bx, float (*tl)[33]);
__global__ void __launch_bounds__(256) wgrad_finalize_kernel(const WGradFinalize f, int S) {
  // red[256] (S > 0), red[4][256] (S < 0: the 16-byte form) or the 32 x 33
  // float tile (S == 0)
  __shared__ double sh[1024];
  if (S == 0) wgrad_finalize_tile(f, blockIdx.x, reinterpret_cast<float (*)[33]>(sh));
  else if (S < 0) wgrad_finalize_body4(f, -S, sh);
  else wgrad_finalize_body(f, S, sh);
}
// Several layers' finalizes in one launch (grid.y = job): the backward defers
// each layer's finalize until its slabs would no longer fit the slab arena.
struct WGFBatch {
  int n;
  int S[kWgfBatch], blocks[kWgfBatch];
  WGradFinalize f[kWgfBatch];
};
static_assert(sizeof(WGFBatch) <= 4000, "finalize batch must fit the 4 KB kernel-argument limit");
__global__ void __launch_bounds__(256) wgrad_finalize_batch_kernel(const WGFBatch b) {
  __shared__ double sh[1024];
  const int j = blockIdx.y;
  if ((int)blockIdx.x >= b.blocks[j]) return;
  if (b.S[j] == 0) wgrad_finalize_tile(b.f[j], blockIdx.x, reinterpret_cast<float (*)[33]>(sh));
  else if (b.S[j] < 0) wgrad_finalize_body4(b.f[j], -b.S[j], sh);
  else wgrad_finalize_body(b.f[j], b.S[j], sh);
}

// The element-parallel sum with 16-byte slab reads: a thread owns 4
// consecutive elements (four fp64 sums, each over k = sl, sl + S, ... in
// increasing k, then the S partials combined in increasing sl -- the order of
// wgrad_finalize_body, so the results are bitwise the same), and consecutive
// threads read consecutive 16-byte groups of one slab (body's 4-byte reads
// gave a wave 256 / S elements = 32 bytes of each slab at S = 32).
__device__ __forceinline__ void wgrad_finalize_body4(const WGradFinalize &f, int S, double *red) {
  const int64_t n = (int64_t)f.Mtot * f.Ntot;
  const int TPG = 256 / S;   // threads per slab group
  const int tid = threadIdx.x, el = tid % TPG, sl = tid / TPG;
  const int64_t idx = ((int64_t)blockIdx.x * TPG + el) * 4;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (idx < n) {
    const float4 *src = reinterpret_cast<const float4 *>(f.partial + idx);
    const int64_t n4 = n / 4;
#pragma unroll 4
    for (int k = sl; k < f.KB; k += S) {
      const float4 r = src[(size_t)k * n4];
      a0 += (double)r.x;
      a1 += (double)r.y;
      a2 += (double)r.z;
      a3 += (double)r.w;
    }
  }
  red[tid] = a0;
  red[256 + tid] = a1;
  red[512 + tid] = a2;
  red[768 + tid] = a3;
  lds_barrier();
  if (sl != 0 || idx >= n) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double *rq = red + q * 256;
    double s = rq[el];
    for (int j = 1; j < S; ++j) s += rq[j * TPG + el];
    wgrad_finalize_emit(f, idx + q, s);
  }
}
__device__ __forceinline__ void wgrad_finalize_body(const WGradFinalize &f, int S, double *red) {
  const int64_t n = (int64_t)f.Mtot * f.Ntot;
  const int EPB = 256 / S;
  const int tid = threadIdx.x, el = tid % EPB, sl = tid / EPB;
  const int64_t idx = (int64_t)blockIdx.x * EPB + el;
  double acc = 0.0;
  if (idx < n && f.mode == 4) {
    // column sums from forward-statistics rows {S1, S2, K, n}: sum = S1 + n*K
    const float4 *src = reinterpret_cast<const float4 *>(f.partial) + idx;
    for (int k = sl; k < f.KB; k += S) {
      const float4 r = src[(size_t)k * n];
      acc += (double)r.x + (double)r.w * (double)r.z;
    }
  } else if (idx < n) {
    const float *src = f.partial + idx;
#pragma unroll 4
    for (int k = sl; k < f.KB; k += S) acc += (double)src[(size_t)k * n];
  }
  red[tid] = acc;
  lds_barrier();
  if (sl != 0 || idx >= n) return;
  double s = red[el];
  for (int j = 1; j < S; ++j) s += red[j * EPB + el];
  wgrad_finalize_emit(f, idx, s);
}

// The finalized element idx of the slab sum s, scattered into PyTorch's layout.
__device__ __forceinline__ void wgrad_finalize_emit(const WGradFinalize &f, int64_t idx, double s) {
  const int64_t n = (int64_t)f.Mtot * f.Ntot;
  const float v = (float)s;
  const int grow = (int)(idx / f.Ntot), gcol = (int)(idx % f.Ntot);
  if (f.mode == 3) {   // ConvTranspose3d, phase form (WGradArgs::nph)
    const int Jt = f.J[0] * f.J[1] * f.J[2];
    const int ph = gcol / f.CoutT, co = gcol % f.CoutT;
    if (grow == Jt * f.ACs) {   // bias: the phase-0 thread sums every phase's column, in order
      if (ph != 0 || !f.db) return;
      const int nph = f.Ntot / f.CoutT;
      double sb = s;
      const int64_t brow = (int64_t)grow * f.Ntot;
      for (int q = 1; q < nph; ++q) {
        const float *src = f.partial + brow + q * f.CoutT + co;
        double a2 = 0.0;
        for (int k = 0; k < f.KB; ++k) a2 += (double)src[(size_t)k * n];
        sb += a2;
      }
      const float vb = (float)sb;
      f.db[co] = f.accumulate ? f.db[co] + vb : vb;
      return;
    }
    const int j = grow / f.ACs, ci = grow % f.ACs;
    if (ci >= f.Cin) return;
    const int jz = j % f.J[2], jy = (j / f.J[2]) % f.J[1], jx = j / (f.J[2] * f.J[1]);
    const int phz = f.SS[2], phy = f.SS[1];
    const int qz = ph % phz, qy = (ph / phz) % phy, qx = ph / (phz * phy);
    const int tx = (f.J[0] - 1 - jx) * f.SS[0] + qx, ty = (f.J[1] - 1 - jy) * f.SS[1] + qy,
              tz = (f.J[2] - 1 - jz) * f.SS[2] + qz;
    const int KY = f.J[1] * f.SS[1], KZ = f.J[2] * f.SS[2];
    const int t = (tx * KY + ty) * KZ + tz;
    float *dst = f.dw + ((size_t)ci * f.CoutT + co) * f.T + t;
    *dst = f.accumulate ? *dst + v : v;
    return;
  }
  if (f.mode == 2 || f.mode == 4) {   // column sums of R rows (ConvTranspose bias)
    if (gcol < f.Cout && f.db) f.db[gcol] = f.accumulate ? f.db[gcol] + v : v;
    return;
  }
  if (f.mode == 0) {
    const int o = gcol;
    if (o >= f.Cout) return;
    if (grow == f.T * f.ACs) {
      if (f.db) f.db[o] = f.accumulate ? f.db[o] + v : v;
      return;
    }
    const int t = grow / f.ACs;
    int e = grow % f.ACs;
    if (f.part_cs) {   // channel parts: packed e -> torch channel, padding rows dropped
      const int r = e % f.part_cs;
      if (r >= f.part_c) return;
      e = (e / f.part_cs) * f.part_c + r;
    }
    const int g = o / (f.Cout / f.groups);
    const int cin_total = f.groups * f.Cin_g;
    for (int cp = e; cp < cin_total; cp += f.fold_mod) {
      const int c = cp - g * f.Cin_g;
      if (c >= 0 && c < f.Cin_g) {
        float *dst = f.dw + ((size_t)o * f.Cin_g + c) * f.T + t;
        *dst = f.accumulate ? *dst + v : v;
      }
    }
  } else {
    const int ci = grow;
    const int t = gcol / f.GCs, co = gcol % f.GCs;
    if (ci >= f.Cin || co >= f.CoutT) return;
    float *dst = f.dw + ((size_t)ci * f.CoutT + co) * f.T + t;
    *dst = f.accumulate ? *dst + v : v;
  }
}

// Tiled finalize of the Conv3d (mode 0) / ConvTranspose3d (mode 1) weights:
// a block sums the slabs of a 32 (column: o / co) x 32 (inner: c*T + t / t)
// tile of dW, reading along the GEMM column (contiguous in a slab row) and
// writing along the inner index (contiguous in PyTorch's [Cout][Cin_g][T] /
// [Cin][Cout][T] layout) through an LDS transpose -- the S == 1 path instead
// stores one 4-byte word per element with a Cin_g*T (mode 0) or T (mode 1)
// word stride.  Every destination gathers its own GEMM element (mode 0:
// e = (g*Cin_g + c) % fold_mod), summed over the slabs k = 0..KB-1 in fp64 in
// the same order as the S == 1 path, so the results are bitwise equal.
// Blocks past the tiles finalize the Conv3d bias row.
__device__ __forceinline__ void wgrad_finalize_tile(const WGradFinalize &f, int bx, float (*tl)[33]) {
  const int tid = threadIdx.x;
  const int NC = f.mode == 0 ? f.Cout : f.CoutT;
  const int NI = f.mode == 0 ? f.Cin_g * f.T : f.T;
  const int tc = (NC + 31) / 32, ti = (NI + 31) / 32;
  const int rows = f.mode == 0 ? 1 : f.Cin;
  const int64_t n = (int64_t)f.Mtot * f.Ntot;
  if (bx >= rows * tc * ti) {   // mode 0 bias row (grow = T * ACs)
    const int o = (bx - rows * tc * ti) * 256 + tid;
    if (o >= f.Cout || !f.db) return;
    const float *src = f.partial + (int64_t)f.T * f.ACs * f.Ntot + o;
    double acc = 0.0;
#pragma unroll 4
    for (int k = 0; k < f.KB; ++k) acc += (double)src[(size_t)k * n];
    const float v = (float)acc;
    f.db[o] = f.accumulate ? f.db[o] + v : v;
    return;
  }
  const int row = bx / (tc * ti), rem = bx % (tc * ti);
  const int c0 = (rem % tc) * 32, i0 = (rem / tc) * 32;
  const int cl = tid & 31, col = c0 + cl;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int il = (tid >> 5) + 8 * r, in = i0 + il;
    double acc = 0.0;
    if (col < NC && in < NI) {
      int64_t idx;
      if (f.mode == 0) {
        const int c = in / f.T, t = in % f.T;
        int e = (col / (f.Cout / f.groups) * f.Cin_g + c) % f.fold_mod;
        if (f.part_cs) e = (e / f.part_c) * f.part_cs + e % f.part_c;   // torch channel -> packed
        idx = (int64_t)(t * f.ACs + e) * f.Ntot + col;
      } else {
        idx = (int64_t)row * f.Ntot + (int64_t)in * f.GCs + col;
      }
      const float *src = f.partial + idx;
#pragma unroll 4
      for (int k = 0; k < f.KB; ++k) acc += (double)src[(size_t)k * n];
    }
    tl[il][cl] = (float)acc;
  }
  lds_barrier();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int p = tid + 256 * r, il = p & 31, cl2 = p >> 5;
    const int in = i0 + il, col2 = c0 + cl2;
    if (col2 >= NC || in >= NI) continue;
    float *dst = f.mode == 0 ? f.dw + (size_t)col2 * NI + in
                             : f.dw + ((size_t)row * f.CoutT + col2) * f.T + in;
    const float v = tl[il][cl2];
    *dst = f.accumulate ? *dst + v : v;
  }
}

// HCU_WGF_TILED: 0 keeps every finalize on the element-parallel form, 1 (the
// default) tiles the layers that need no slab parallelism, 2 tiles every
// Conv3d / ConvTranspose3d finalize (A/B and tests)
static int tiled_finalize_mode() {
  static const int m = [] {
    const char *e = getenv("HCU_WGF_TILED");
    return e && e[0] ? atoi(e) : 1;
  }();
  return m;
}

static void wgf_geometry(const WGradFinalize &f, int &S, int &blocks) {
  const int64_t n = (int64_t)f.Mtot * f.Ntot;
  S = 1;
  while (S < 64 && S * 2 <= f.KB && n * S / 256 < 1024) S *= 2;
  const int EPB = 256 / S;
  blocks = (int)((n + EPB - 1) / EPB);
  // the 16-byte form (S < 0) for the sums whose slabs it can read as float4
  // (same S, same order); HCU_WGF_VEC4=0 keeps the 4-byte form (A/B)
  static const bool v4 = !(getenv("HCU_WGF_VEC4") && getenv("HCU_WGF_VEC4")[0] == '0');
  if (v4 && S > 1 && tiled_finalize_mode() != 2 && (f.mode == 0 || f.mode == 1 || f.mode == 2) && n % 4 == 0 &&
      reinterpret_cast<uintptr_t>(f.partial) % 16 == 0) {
    blocks = (int)((n / 4 + EPB - 1) / EPB);
    S = -S;
    return;
  }
  // large layers (no slab parallelism needed): the coalescing tiled form
  const int tm = tiled_finalize_mode();
  if ((tm == 2 || (tm == 1 && S == 1)) && (f.mode == 1 || (f.mode == 0 && f.fold_mod > 0))) {
    const int NC = f.mode == 0 ? f.Cout : f.CoutT;
    const int NI = f.mode == 0 ? f.Cin_g * f.T : f.T;
    const int rows = f.mode == 0 ? 1 : f.Cin;
    S = 0;
    blocks = rows * ((NC + 31) / 32) * ((NI + 31) / 32);
    if (f.mode == 0 && f.Mtot > f.T * f.ACs) blocks += (f.Cout + 255) / 256;
  }
}

int launch_wgrad_finalize_batch(const WGradFinalize *fs, int n, hipStream_t s) {
  for (int j0 = 0; j0 < n; j0 += kWgfBatch) {
    WGFBatch b{};
    b.n = std::min(kWgfBatch, n - j0);
    int gx = 1;
    double by = 0.0;
    for (int k = 0; k < b.n; ++k) {
      b.f[k] = fs[j0 + k];
      wgf_geometry(b.f[k], b.S[k], b.blocks[k]);
      gx = std::max(gx, b.blocks[k]);
      by += 4.0 * (double)b.f[k].Mtot * b.f[k].Ntot * (b.f[k].KB + 1);
    }
    HCU_TIMED(s, "wgrad_finalize_batch_kernel", 0.0, by,
              HCU_LAUNCH(wgrad_finalize_batch_kernel, dim3(gx, b.n), dim3(256), 0, s, b));
    HCU_CHECK_LAUNCH();
  }
  return 0;
}

int launch_wgrad_finalize(const WGradFinalize &f, hipStream_t s) {
  const int64_t n = (int64_t)f.Mtot * f.Ntot;
  int S, blocks;
  wgf_geometry(f, S, blocks);
  HCU_TIMED(s, "wgrad_finalize_kernel", 0.0, 4.0 * (double)n * (f.KB + 1),
            HCU_LAUNCH(wgrad_finalize_kernel, dim3(blocks), dim3(256), 0, s, f, S));
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu
