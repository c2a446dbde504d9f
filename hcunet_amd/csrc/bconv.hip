// bf16 / fp32 blocked implicit-GEMM convolution (the kernel template is in
// bconv_kernel.h): the planner, the bf16 instances and the dispatch.  The fp32
// instances are in bconv_f32.hip (separate translation unit: compile time).
#include "bconv_kernel.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace hcu {

#ifdef HCU_BCONV_PHASES
__device__ unsigned long long g_bconv_phase[kPhBlocks * kPhN];
#endif

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

// floats of the halo image region: [HV] rows of ckp_bytes(CV) + a dummy 16-byte slot
static long bconv_areg(const GConvArgs &a, int CV) {
  const long HV = std::max((long)a.HX * a.HY * a.HZ, (long)a.hvp);
  // >= 4 waves x 64 columns x 3 floats: the statistics merge reuses the region;
  // >= 512 doubles + a flag word: the BatchNorm-backward finalize tail does too
  return std::max(1152L, ((HV * ckp_bytes(CV) + 16) / 4 + 3) & ~3L);
}

static long bconv_lds(const GConvArgs &a, int CV, int NT) {
  const int T = a.KX * a.KY * a.KZ;
  const int TPS = 4 / CV;
  const int S = (T + TPS - 1) / TPS;
  return (bconv_areg(a, CV) + (long)S * 4 * NT * 4 + S * 4 + (long)a.MPW * 128 + 9L * NT +
          3L * a.ICs) * 4 + (long)sizeof(GConvArgs);   // + the static copy of the arguments
}

int bconv_stat_rows(const GConvArgs &a) {
  if (a.ksplit > 1) {
    const int64_t nvox = (int64_t)a.B * a.SX * a.SY * a.SZ;
    const int vpb = bconv_reduce_vpb(a);
    return (int)((nvox + vpb - 1) / vpb);
  }
  return a.gridx;   // one row per block
}

static void bconv_finish(GConvArgs &a, int ntz, int VEC, int fpf, long lds_cap);
static void bconv_halo_layout(GConvArgs &a, int CV, long lds_cap);

// ---- measured planning: times a candidate on scratch buffers of its shapes
//
// Choices are kept per convolution signature as the tiling itself
// (CK, NSUB, MPW), in memory and in a persistent table (tuning/bconv_gfx950.txt
// next to libhcunet.so, or HCU_TUNE_FILE) loaded on first use, so every
// process -- every data-parallel rank -- plans the same tiling for the same
// convolution, and timing dispatches never run inside a measured step.
// Modes (hcu_tuning_set_mode / HCU_BCONV_TUNE): 0 = the cost model's first
// choice; 1 = the table, the cost model on a miss (deterministic across
// processes: what a data-parallel job uses); 2 = the table, timing on a miss
// (default).
static std::mutex g_tune_mu;
static std::map<std::string, std::string> g_tune;   // signature -> "CK,NSUB,MPW"
static bool g_tune_loaded = false;
static int g_tune_mode = -1;
static long g_tune_timed = 0;   // signatures timed by this process
// Measured planning is off while a forward-only (inference) plan is built: its
// tile-batch size follows the free device memory, so every call can bring new
// signatures, and timing those costs seconds per call.
static thread_local bool g_tune_off = false;
void bconv_tuning(bool on) { g_tune_off = !on; }

static std::string tune_file() {
  if (const char *e = getenv("HCU_TUNE_FILE")) return e;
  Dl_info info;
  if (dladdr(reinterpret_cast<void *>(&bconv_tuning), &info) && info.dli_fname) {
    std::string p = info.dli_fname;
    const size_t slash = p.rfind('/');
    return (slash == std::string::npos ? std::string(".") : p.substr(0, slash)) +
           "/tuning/bconv_gfx950.txt";
  }
  return "";
}

// Loads the persistent table once (caller holds g_tune_mu).
static void tune_load_locked() {
  if (g_tune_loaded) return;
  g_tune_loaded = true;
  if (g_tune_mode < 0) {
    const char *e = getenv("HCU_BCONV_TUNE");
    g_tune_mode = e ? std::max(0, std::min(2, atoi(e))) : 2;
  }
  const std::string path = tune_file();
  if (path.empty()) return;
  FILE *f = fopen(path.c_str(), "r");
  if (!f) return;
  char line[1024];
  while (fgets(line, sizeof line, f)) {
    if (line[0] == '#') continue;
    char *bar = strchr(line, '|');
    if (!bar) continue;
    *bar = 0;
    std::string val = bar + 1;
    while (!val.empty() && (val.back() == '\n' || val.back() == '\r' || val.back() == ' ')) val.pop_back();
    g_tune[line] = val;
  }
  fclose(f);
}

static std::string tiling_key(const GConvArgs &c) {
  return std::to_string(c.CK) + "," + std::to_string(c.NSUB) + "," + std::to_string(c.MPW);
}

static std::string bconv_signature(const GConvArgs &a) {
  const int v[] = {a.bes, a.B, a.IX, a.IY, a.IZ, a.ICs, a.OX, a.OY, a.OZ, a.SX, a.SY, a.SZ, a.OCs,
                   a.Cout, a.osx, a.osy, a.osz, a.ofx, a.ofy, a.ofz, a.KX, a.KY, a.KZ, a.sx, a.sy,
                   a.sz, a.dx, a.dy, a.dz, a.px, a.py, a.pz, a.nph, a.phx, a.phy, a.phz};
  std::string k;
  for (int x : v) k += std::to_string(x) + ",";
  return k;
}

// Microseconds per launch of the planned variant (min of 3 after a warm-up), or
// -1 when no device is usable.  The buffers hold zeros (MFMA and memory timing
// do not depend on the values); forward-shaped convolutions (no padding, or
// ConvTranspose phases) are timed with the input BatchNorm+ReLU and statistics
// rows, input gradients with the fused BatchNorm backward.
static double bconv_time(const GConvArgs &c0) {
  static char *arena = nullptr;
  static size_t arena_bytes = 0;
  static hipStream_t ts = nullptr;
  static int ndev = -1;
  if (ndev < 0) {
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    (void)hipGetLastError();
  }
  if (ndev <= 0) return -1;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(nullptr, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return -1;
  }
  GConvArgs c = c0;
  const bool fwd = (c.px == 0 && c.py == 0 && c.pz == 0) || c.nph > 1;
  const size_t es = c.bes;
  const int T = c.KX * c.KY * c.KZ;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t b_in = al((size_t)c.B * c.IX * c.IY * c.IZ * c.ICs * es);
  const size_t b_w = al((size_t)wpack_count(wpack_of(c), T, c.ICs, c.CoutW) * es);
  const size_t b_out = al((size_t)c.B * c.SX * c.SY * c.SZ * c.OCs * es);
  const size_t b_st = al((size_t)bconv_stat_rows(c) * c.CoutW * 4 * sizeof(float));
  const size_t b_part = c.ksplit > 1 ? al((size_t)c.ksplit * c.slice_floats * sizeof(float)) : 0;
  const size_t b_vec = al((size_t)std::max(std::max(c.ICs, c.OCs), c.Cout) * sizeof(float));
  const size_t need = b_in + b_w + 2 * b_out + b_st + b_part + 6 * b_vec;
  if (need > arena_bytes) {
    if (arena) (void)hipFree(arena);
    arena = nullptr;
    arena_bytes = 0;
    if (hipMalloc(&arena, need) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    arena_bytes = need;
    if (hipMemset(arena, 0, need) != hipSuccess) return -1;
  }
  if (!ts && hipStreamCreateWithFlags(&ts, hipStreamNonBlocking) != hipSuccess) return -1;
  char *p = arena;
  auto take = [&](size_t b) {
    char *r = p;
    p += b;
    return r;
  };
  c.in = reinterpret_cast<const float *>(take(b_in));
  c.w = reinterpret_cast<const float *>(take(b_w));
  c.out = reinterpret_cast<float *>(take(b_out));
  float *y = reinterpret_cast<float *>(take(b_out));
  c.stats = reinterpret_cast<float *>(take(b_st));
  c.partial = b_part ? reinterpret_cast<float *>(take(b_part)) : nullptr;
  float *v[6];
  for (float *&q : v) q = reinterpret_cast<float *>(take(b_vec));
  c.bias = v[0];
  c.in_scale = fwd ? v[1] : nullptr;
  c.in_shift = fwd ? v[2] : nullptr;
  if (!fwd && c.nph == 1) {
    c.bn_y = y;
    c.bn_scale = c.bn_shift = v[3];
    c.bn_mean = v[4];
    c.bn_invstd = v[5];
  }
  if (!fwd && !c.bn_y) c.stats = nullptr;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return -1;
  if (hipEventCreate(&e1) != hipSuccess) return -1;
  double best = -1;
  const bool was_timing = timing_on();
  for (int it = 0; it < 4 && !was_timing; ++it) {
    (void)hipEventRecord(e0, ts);
    if (launch_bconv(c, ts)) break;
    (void)hipEventRecord(e1, ts);
    if (hipEventSynchronize(e1) != hipSuccess) break;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (it > 0 && (best < 0 || ms * 1e3 < best)) best = ms * 1e3;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipGetLastError();
  return best;
}

int plan_bconv(GConvArgs &a, int target_blocks) {
  a.use_bconv = 0;
  if (a.bes == 0) a.bes = 2;
  if (a.bes != 2 && a.bes != 4) return fail(4, "bconv: element size must be 2 (bf16) or 4 (fp32)");
  const int VEC = 16 / a.bes;
  if (a.OX <= 0 || a.OY <= 0 || a.OZ <= 0) return fail(2, "bconv: empty output grid");
  if (a.ICs % VEC || a.OCs % VEC)
    return fail(4, "bconv: channel strides must be multiples of " + std::to_string(VEC));
  // 32-bit buffer offsets within one sample (fp32 K-split partials included)
  if ((double)a.SX * a.SY * a.SZ * a.OCs * 4 >= 2147483647.0 ||
      (double)a.IX * a.IY * a.IZ * a.ICs * a.bes >= 2147483647.0)
    return fail(4, "bconv: one sample must stay below 2 GiB");
  if (a.nph < 1) a.nph = 1;
  if (a.phx < 1) a.phx = 1;
  if (a.phy < 1) a.phy = 1;
  if (a.phz < 1) a.phz = 1;
  const int T = a.KX * a.KY * a.KZ;
  if (a.nph == 1 || a.cph < a.Cout) a.cph = 0;
  const int CPH = a.cph > 0 ? a.cph : a.Cout;
  if (a.cph > a.OCs) return fail(4, "bconv: padded phase columns exceed the stored channels");
  const int Nlog = CPH * a.nph;
  const int nb16 = cdiv(Nlog, 16);
  const int ntz = cdiv(a.OZ, 16);
  a.TZ = cdiv(a.OZ, ntz);
  // (96 / 160 KB measured equal on the U-Net layers: tools/gpu_bb.sh, ab8;
  // HCU_BCONV_LDS_KB for A/B)
  static const long lds_cap = 1024L * std::max(16, std::min(160, env_int_b("HCU_BCONV_LDS_KB", 80)));
  // Candidate tilings, scored by a simple per-CU time model (cycles):
  //   per (tile, chunk): MFMA S * MPW * NSUB * (16 bf16 | 128 fp32) per wave, staging ~
  //   1200 + 40 per 16-byte element per thread (+ weights when multi-chunk);
  //   per tile: epilogue ~1500; two resident blocks hide ~40 % of a block's
  //   staging behind the other's MFMAs.
  struct Cand {
    GConvArgs c;
    double cost;
    bool laid = false;
  };
  std::vector<Cand> cands;
  const int mpws[3] = {4, 2, 1}, nsubs[3] = {4, 2, 1}, cvs[3] = {4, 2, 1};
  const double mfma_cyc = a.bes == 2 ? 16.0 : 128.0;   // per K-step, subtile pair, SIMD
  // HCU_BCONV_FORCE="CK,NSUB,MPW[,NPF]" restricts the search (experiments)
  int fck = 0, fns = 0, fmp = 0, fpf = -1;
  if (const char *e = getenv("HCU_BCONV_FORCE")) sscanf(e, "%d,%d,%d,%d", &fck, &fns, &fmp, &fpf);
  for (int ni = 0; ni < 3; ++ni) {
    const int NSUB = nsubs[ni];
    if (fns && NSUB != fns) continue;
    if (NSUB > 1 && nb16 < NSUB && !(NSUB == 2 && nb16 >= 2)) continue;
    if (NSUB == 4 && nb16 < 4) continue;
    if (NSUB == 2 && nb16 < 2) continue;
    // (phases folded into N: a lane's 4 columns share a phase; bf16 stores 8
    // channels per 16 bytes of the packed weights)
    if (a.nph > 1 && (CPH % (a.bes == 2 ? 8 : 4))) continue;
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
      c.hsx = c.HY * c.HZ;
      c.hsy = c.HZ;
      c.hsz = 1;
      c.hvp = c.HX * c.HY * c.HZ;
      const long tiles = (long)cdiv(a.OX, TX) * cdiv(a.OY, TY) * ntz * a.B;
      const int MT = TX * TY * a.TZ;
      for (int ki = 0; ki < 3; ++ki) {
        const int CV = cvs[ki], CK = CV * VEC;
        if (a.ICs % CK || (fck && CK != fck)) continue;
        const long lds = bconv_lds(c, CV, NT);
        if (lds > lds_cap) continue;
        const int occ = std::max(1, std::min(2, (int)(160 * 1024 / lds)));
        const int chunks = a.ICs / CK;
        const int TPS = 4 / CV;
        const int S = (T + TPS - 1) / TPS;
        const double helem = (double)c.HX * c.HY * c.HZ * CV / 256.0;
        const double welem = chunks > 1 ? (double)S * 4 * NT / 256.0 : 0.0;
        const double t_mfma = (double)S * MPW * NSUB * mfma_cyc;
        const double t_stage = 1200.0 + 40.0 * (helem + welem);
        const double hide = occ > 1 ? 0.6 : 1.0;
        const double t_tile = chunks * (t_mfma + hide * t_stage) + 1500.0 * hide;
        // blocks: tiles x N blocks (K split added below when this is too few)
        const double blocks = (double)tiles * nN;
        const double waves = std::max(1.0, blocks / (256.0 * occ));
        const double util = (double)MT / (MPW * 64.0) * std::min(1.0, (double)Nlog / CoutW);
        const double cost = waves * t_tile * occ / std::max(0.25, util) *
                            (blocks < 256.0 * occ ? 256.0 * occ / blocks * 0.5 + 0.5 : 1.0);
        Cand cd{c, cost};
        cd.c.CK = CK;
        cd.c.lds_bytes = (int)lds;
        cands.push_back(cd);
      }
    }
  }
  if (cands.empty()) return fail(4, "bconv: no tile fits in LDS");
  std::stable_sort(cands.begin(), cands.end(),
                   [](const Cand &x, const Cand &y) { return x.cost < y.cost; });
  for (Cand &cd : cands) bconv_finish(cd.c, ntz, VEC, fpf, lds_cap);
  // halo image layout: searched only for the candidates that can be chosen
  auto lay = [&](Cand &cd) {
    if (!cd.laid) bconv_halo_layout(cd.c, cd.c.CK / VEC, lds_cap);
    cd.laid = true;
  };
  lay(cands[0]);
  a = cands[0].c;
  // Measured choice among the model's best candidates, remembered per
  // convolution signature (table above).
  const int top = std::min<int>((int)cands.size(), env_int_b("HCU_BCONV_TUNE_TOP", 6));
  if (!fck && !fns && !fmp) {
    const std::string key = bconv_signature(a);
    std::lock_guard<std::mutex> lk(g_tune_mu);
    tune_load_locked();
    auto it = g_tune_mode > 0 ? g_tune.find(key) : g_tune.end();
    bool hit = false;
    if (it != g_tune.end()) {
      for (Cand &cd : cands)
        if (tiling_key(cd.c) == it->second) {
          lay(cd);
          a = cd.c;
          hit = true;
          break;
        }
    }
    // Time on a miss -- not for very large convolutions (~10^8 output voxels:
    // seconds of timing) nor in forward-only plans (g_tune_off).
    const double out_vox = (double)a.B * a.OX * a.OY * a.OZ;
    if (!hit && g_tune_mode == 2 && top > 1 && out_vox <= 16e6 && !g_tune_off) {
      double best_us = 1e300;
      int best_i = 0;
      bool timed = false;
      for (int i = 0; i < top; ++i) {
        lay(cands[i]);
        const double us = bconv_time(cands[i].c);
        if (us <= 0) break;   // no device / allocation failed: keep the model's choice
        timed = true;
        if (us < best_us * 0.97) {   // ties keep the model's order
          best_us = us;
          best_i = i;
        }
      }
      if (timed) {
        g_tune[key] = tiling_key(cands[best_i].c);
        ++g_tune_timed;
      }
      a = cands[best_i].c;
    }
  }
  if (env_int_b("HCU_CONV2_LOG", 0))
    fprintf(stderr,
            "bconv plan (es %d): B%d I%dx%dx%d ICs%d O%dx%dx%d S%dx%dx%d OCs%d Cout%d K%dx%dx%d s%d%d%d nph%d"
            " | CK%d NSUB%d MPW%d T%dx%dx%d ks%d cps%d NPF%d gridx%d lds%d halo %d,%d,%d/%d\n",
            a.bes, a.B, a.IX, a.IY, a.IZ, a.ICs, a.OX, a.OY, a.OZ, a.SX, a.SY, a.SZ, a.OCs, a.Cout, a.KX,
            a.KY, a.KZ, a.sx, a.sy, a.sz, a.nph, a.CK, a.NSUB, a.MPW, a.TX, a.TY, a.TZ, a.ksplit,
            a.cps, a.NPF, a.gridx, a.lds_bytes, a.hsx, a.hsy, a.hsz, a.hvp);
  (void)target_blocks;
  return 0;
}

// LDS cycles of the A-fragment reads of one tile, per ds_read_b128 (4 = no
// bank conflict), for halo row strides (px, py, pz).  bf16 A fragments: lane
// (g = lane / 16, r = lane % 16) of wave w reads 16 bytes of M row
// i = (w + 4 j) * 16 + r at tap slot e = 4 s + g; a wave64 ds_read_b128 is
// served in four 16-lane groups (MI355X_MICROARCH.md, LDS table), each one
// cycle plus one per extra distinct 16-byte granule on the same 4 banks.
// Stops counting once `stop` is exceeded (the caller's best so far); sstep > 1
// samples every sstep-th 16-row subtile.
static double halo_read_cycles(const GConvArgs &a, int CV, int px, int py, int pz, double stop, int sstep) {
  static const signed char grp[4][16] = {
      {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
      {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
      {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
      {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  const int T = a.KX * a.KY * a.KZ, TPS = 4 / CV, S = (T + TPS - 1) / TPS;
  const int CKG = ckp_bytes(CV) / 16;   // granules per halo row
  const int MT = a.TX * a.TY * a.TZ, rows = a.MPW * 64;
  std::vector<int> rv(rows, 0), toff(S * 4, 0);
  for (int i = 0; i < MT && i < rows; ++i) {
    const int lz = i % a.TZ, q = i / a.TZ, ly = q % a.TY, lx = q / a.TY;
    rv[i] = (lx * a.sx * px + ly * a.sy * py + lz * a.sz * pz) * CKG;
  }
  for (int e = 0; e < S * 4; ++e) {
    const int t = (e >> 2) * TPS + (e & 3) / CV;
    int off = 0;
    if (t < T) {
      const int kz = t % a.KZ, q = t / a.KZ, ky = q % a.KY, kx = q / a.KY;
      off = kx * a.dx * px + ky * a.dy * py + kz * a.dz * pz;
    }
    toff[e] = off * CKG + (e & 3) % CV;
  }
  const int nsub = rows / 16;
  const double norm = 4.0 * S * ((nsub + sstep - 1) / sstep);
  long cyc = 0;
  for (int sub = 0; sub < nsub; sub += sstep)
    for (int s = 0; s < S; ++s) {
      for (int gi = 0; gi < 4; ++gi) {
        int addr[16], cnt[16] = {0};
        int worst = 1;
        for (int k = 0; k < 16; ++k) {
          const int l = grp[gi][k];
          const int ad = rv[sub * 16 + (l & 15)] + toff[s * 4 + ((l >> 4) & 3)];
          bool dup = false;
          for (int m = 0; m < k; ++m) dup |= addr[m] == ad;
          addr[k] = ad;
          if (!dup) worst = std::max(worst, ++cnt[ad & 15]);
        }
        cyc += worst;
      }
      if (cyc > stop * norm) return 1e30;
    }
  return cyc / norm;
}

// bf16 halo image layout: the axis order (any of the 6, z-fastest first so it
// wins ties) and row padding (0..4 rows on the two outer strides) whose
// A-fragment reads take the fewest LDS cycles, within the LDS cap.  The layout
// only moves where a halo element sits in LDS: every product and sum is the
// same (bitwise-equal results).  HCU_HALO_LAYOUT=0 keeps the dense z-fastest
// image; =2 searches the fp32 tiles too (measured neutral on configs 2/3:
// their 16x16x4 fp32 MFMA, not LDS, bounds those tiles).
static void bconv_halo_layout(GConvArgs &a, int CV, long lds_cap) {
  a.hsx = a.HY * a.HZ;
  a.hsy = a.HZ;
  a.hsz = 1;
  a.hvp = a.HX * a.HY * a.HZ;
  static const int on = env_int_b("HCU_HALO_LAYOUT", 1);
  if (!on || (a.bes != 2 && on < 2)) return;
  const int NT = a.NSUB * 16;
  const int dim[3] = {a.HX, a.HY, a.HZ};
  static const int orders[6][3] = {{2, 1, 0}, {2, 0, 1}, {1, 2, 0}, {1, 0, 2}, {0, 2, 1}, {0, 1, 2}};
  const int sstep = std::max(1, a.MPW);   // ranking on 4 of the 4 * MPW subtiles
  double best = halo_read_cycles(a, CV, a.hsx, a.hsy, a.hsz, 1e30, sstep);
  const double base = best;
  int bs[3] = {a.hsx, a.hsy, a.hsz}, bv = a.hvp;
  for (const auto &o : orders)   // o[0] fastest
    for (int p1 = 0; p1 <= 4; ++p1)
      for (int p2 = 0; p2 <= 4; ++p2) {
        int st[3];
        st[o[0]] = 1;
        st[o[1]] = dim[o[0]] + p1;
        st[o[2]] = st[o[1]] * dim[o[1]] + p2;
        const int hv = (a.HX - 1) * st[0] + (a.HY - 1) * st[1] + (a.HZ - 1) * st[2] + 1;
        GConvArgs t = a;
        t.hvp = hv;
        if (bconv_lds(t, CV, NT) > lds_cap) continue;
        const double c = halo_read_cycles(a, CV, st[0], st[1], st[2], best * 0.999, sstep);
        if (c < best * 0.999 || (c <= best * 1.0001 && hv < bv && c < base * 0.999)) {
          best = c;
          bs[0] = st[0], bs[1] = st[1], bs[2] = st[2];
          bv = hv;
        }
      }
  // kept only if all subtiles agree
  if (bv != a.hvp || bs[2] != 1) {
    const double full0 = halo_read_cycles(a, CV, a.hsx, a.hsy, a.hsz, 1e30, 1);
    const double full1 = halo_read_cycles(a, CV, bs[0], bs[1], bs[2], 1e30, 1);
    if (full1 < full0 * 0.98) {
      a.hsx = bs[0], a.hsy = bs[1], a.hsz = bs[2];
      a.hvp = bv;
    }
  }
  const int NTl = a.NSUB * 16, CVl = CV;
  a.lds_bytes = (int)bconv_lds(a, CVl, NTl);
  a.areg = (int)bconv_areg(a, CVl);
}

// Completes a candidate tiling: K split, prefetch depth, persistent grid, divisors.
static void bconv_finish(GConvArgs &a, int ntz, int VEC, int fpf, long lds_cap) {
  const int NT = a.NSUB * 16;
  const int nN = a.CoutW / NT;
  a.ntx = cdiv(a.OX, a.TX);
  a.nty = cdiv(a.OY, a.TY);
  a.ntz = ntz;
  const long tiles = (long)a.ntx * a.nty * a.ntz * a.B;
  const int nchunks = a.ICs / a.CK;
  int ks = 1;
  const int ks_target = 256;   // (512 measured +7 % on config 2)
  if (a.nph == 1 && 256 % (a.OCs / VEC) == 0)
    while (ks < nchunks && tiles * nN * ks < ks_target) ks *= 2;
  ks = std::min(ks, nchunks);
  a.cps = cdiv(nchunks, ks);
  a.ksplit = cdiv(nchunks, a.cps);
  a.slice_floats = (size_t)a.B * a.SX * a.SY * a.SZ * a.OCs;
  const int CV = a.CK / VEC;
  const long nel = (long)a.HX * a.HY * a.HZ * CV;
  const long per_thread = (nel + 255) / 256;
  a.NPF = per_thread <= 4 ? 4 : per_thread <= 8 ? 8 : per_thread <= 12 ? 12 : 0;
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
  (void)lds_cap;
  a.areg = (int)bconv_areg(a, CV);
  a.use_bconv = 1;
  a.use_conv2 = 0;
  a.use_conv8 = 0;
}

int launch_bconv_bf16(const GConvArgs &a, hipStream_t s) { BCONV_LAUNCH_BODY(uint16_t, "bf16") }

int launch_bconv(const GConvArgs &a, hipStream_t s) {
  return a.bes == 4 ? launch_bconv_f32(a, s) : launch_bconv_bf16(a, s);
}

}  // namespace hcu

extern "C" {

int hcu_tuning_set_mode(int mode) {
  if (mode < 0 || mode > 2) return hcu::fail(1, "tuning mode must be 0, 1 or 2");
  std::lock_guard<std::mutex> lk(hcu::g_tune_mu);
  hcu::tune_load_locked();
  hcu::g_tune_mode = mode;
  return 0;
}

int hcu_tuning_get_mode(void) {
  std::lock_guard<std::mutex> lk(hcu::g_tune_mu);
  hcu::tune_load_locked();
  return hcu::g_tune_mode;
}

// Entries in the table (loaded + timed by this process); *timed (nullable)
// receives the number this process timed.
int64_t hcu_tuning_entries(int64_t *timed) {
  std::lock_guard<std::mutex> lk(hcu::g_tune_mu);
  hcu::tune_load_locked();
  if (timed) *timed = hcu::g_tune_timed;
  return (int64_t)hcu::g_tune.size();
}

// Writes the whole table (sorted by signature) to `path` (null: the table the
// library loads); returns the number of entries or -1.
int64_t hcu_tuning_save(const char *path) {
  std::lock_guard<std::mutex> lk(hcu::g_tune_mu);
  hcu::tune_load_locked();
  const std::string p = path ? std::string(path) : hcu::tune_file();
  FILE *f = p.empty() ? nullptr : fopen(p.c_str(), "w");
  if (!f) return -hcu::fail(1, "cannot write tuning table " + p);
  fprintf(f, "# bconv tiling per convolution signature (bes,B,IX,IY,IZ,ICs,OX,OY,OZ,SX,SY,SZ,OCs,Cout,"
             "osx,osy,osz,ofx,ofy,ofz,KX,KY,KZ,sx,sy,sz,dx,dy,dz,px,py,pz,nph,phx,phy,phz | CK,NSUB,MPW),\n"
             "# measured on MI355X by plan-time timing (hcunet_amd/csrc/bconv.hip)\n");
  for (const auto &kv : hcu::g_tune) fprintf(f, "%s|%s\n", kv.first.c_str(), kv.second.c_str());
  fclose(f);
  return (int64_t)hcu::g_tune.size();
}

}  // extern "C"
