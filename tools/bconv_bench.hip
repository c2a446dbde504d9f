// Stand-alone timing of one bf16 convolution launch (bconv.hip) with per-phase
// cycle counts of the persistent tile loop.  Experiment tool, not part of the
// library or the tests.
//
//   tools/bconv_bench.sh            (builds tools/bconv_bench against libhcunet.so)
//   tools/bconv_bench MODE B IX IY IZ ICs Cout KX KY KZ ACT [ITERS]
//     MODE f = forward (+ BatchNorm statistics rows), d = input gradient
//     (padding K-1), db = input gradient with the fused BatchNorm backward
//     epilogue; ACT 1 = BatchNorm+ReLU applied to the input while staging.
//   HCU_BCONV_FORCE="CK,NSUB,MPW[,NPF]" pins the tiling; BCONV_ES=4 runs the
//   fp32 kernels (default 2: bf16).
#define HCU_BCONV_PHASES 1
#include "../hcunet_amd/csrc/bconv.hip"
#include "../hcunet_amd/csrc/bconv_f32.hip"
// The instances of one channel-group width only (BENCH_CV = 1, 2 or 4; the
// others report "unsupported variant"): one per-CV translation unit each.
#ifndef BENCH_CV
#define BENCH_CV 4
#endif
#define BENCH_STUB(E_, CV_)                                                                         \
  namespace hcu {                                                                                  \
  template <>                                                                                      \
  bool bconv_launch_cv<E_, CV_>(const GConvArgs &, hipStream_t, const dim3 &, double, double) {    \
    return false;                                                                                  \
  }                                                                                                \
  }
#if BENCH_CV == 1
#include "../hcunet_amd/csrc/bconv_f32_cv1.hip"
#include "../hcunet_amd/csrc/bconv_bf16_cv1.hip"
BENCH_STUB(float, 2) BENCH_STUB(float, 4) BENCH_STUB(uint16_t, 2) BENCH_STUB(uint16_t, 4)
#elif BENCH_CV == 2
#include "../hcunet_amd/csrc/bconv_f32_cv2.hip"
#include "../hcunet_amd/csrc/bconv_bf16_cv2.hip"
BENCH_STUB(float, 1) BENCH_STUB(float, 4) BENCH_STUB(uint16_t, 1) BENCH_STUB(uint16_t, 4)
#else
#include "../hcunet_amd/csrc/bconv_f32_cv4.hip"
#include "../hcunet_amd/csrc/bconv_bf16_cv4.hip"
BENCH_STUB(float, 1) BENCH_STUB(float, 2) BENCH_STUB(uint16_t, 1) BENCH_STUB(uint16_t, 2)
#endif

#include <chrono>
#include <cstring>
#include <random>
#include <vector>

namespace hcu {
// the library's error channel (unet.cpp), stand-alone here
void set_error(const std::string &msg) { fprintf(stderr, "error: %s\n", msg.c_str()); }
int fail(int code, const std::string &msg) {
  set_error(msg);
  return code;
}
}  // namespace hcu
using namespace hcu;

#define CK_HIP(x)                                                              \
  do {                                                                         \
    hipError_t e__ = (x);                                                      \
    if (e__ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e__)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static uint16_t to_bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

template <class T>
static T *dev_fill(size_t n, std::vector<T> &h) {
  T *d = nullptr;
  CK_HIP(hipMalloc(&d, std::max<size_t>(n, 1) * sizeof(T)));
  if (n) CK_HIP(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char **argv) {
  if (argc < 12) {
    fprintf(stderr, "usage: %s MODE B IX IY IZ ICs Cout KX KY KZ ACT [ITERS]\n", argv[0]);
    return 2;
  }
  const std::string mode = argv[1];
  const int B = atoi(argv[2]), IX = atoi(argv[3]), IY = atoi(argv[4]), IZ = atoi(argv[5]);
  const int ICs = atoi(argv[6]), Cout = atoi(argv[7]);
  const int K[3] = {atoi(argv[8]), atoi(argv[9]), atoi(argv[10])};
  const int act = atoi(argv[11]);
  const int iters = argc > 12 ? atoi(argv[12]) : 20;
  const bool dgrad = mode[0] == 'd';
  const bool bnbwd = mode == "db";

  GConvArgs a{};
  const char *es_env = getenv("BCONV_ES");
  a.bes = es_env ? atoi(es_env) : 2;
  const int ES = a.bes;
  a.B = B;
  a.IX = IX; a.IY = IY; a.IZ = IZ; a.ICs = ICs;
  if (dgrad) {
    a.OX = IX + K[0] - 1; a.OY = IY + K[1] - 1; a.OZ = IZ + K[2] - 1;
    a.px = K[0] - 1; a.py = K[1] - 1; a.pz = K[2] - 1;
  } else {
    a.OX = IX - K[0] + 1; a.OY = IY - K[1] + 1; a.OZ = IZ - K[2] + 1;
  }
  a.SX = a.OX; a.SY = a.OY; a.SZ = a.OZ;
  a.OCs = (Cout + 7) / 8 * 8;
  a.Cout = Cout;
  a.osx = a.osy = a.osz = 1;
  a.KX = K[0]; a.KY = K[1]; a.KZ = K[2];
  a.sx = a.sy = a.sz = 1;
  a.dx = a.dy = a.dz = 1;
  if (int e = plan_bconv(a, 0)) {
    fprintf(stderr, "plan failed %d\n", e);
    return 1;
  }
  const int T = K[0] * K[1] * K[2];
  const int TPS = (ES == 2 ? 32 : 16) / a.CK;
  const int S = (T + TPS - 1) / TPS;
  const size_t n_in = (size_t)B * IX * IY * IZ * ICs;
  const size_t n_out = (size_t)B * a.SX * a.SY * a.SZ * a.OCs;
  const size_t n_w = (size_t)(ICs / a.CK) * S * 4 * a.CoutW * (16 / ES);
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  // element images as 16-bit words (bf16, or two halves of an fp32)
  std::vector<uint16_t> hin(n_in * ES / 2), hw(n_w * ES / 2), hy(n_out * ES / 2);
  auto fill = [&](std::vector<uint16_t> &h, float sc) {
    if (ES == 2) {
      for (auto &v : h) v = to_bf(sc * U(rng));
    } else {
      for (size_t i = 0; i < h.size(); i += 2) {
        const float f = sc * U(rng);
        memcpy(&h[i], &f, 4);
      }
    }
  };
  fill(hin, 1.f);
  fill(hw, 0.05f);
  fill(hy, 1.f);
  std::vector<float> hsc(ICs, 1.1f), hsh(ICs, 0.05f), hb(Cout, 0.01f), hco(a.OCs, 0.5f);
  std::vector<uint16_t> none;
  a.in = reinterpret_cast<const float *>(dev_fill(hin.size(), hin));
  a.w = reinterpret_cast<const float *>(dev_fill(hw.size(), hw));
  uint16_t *dout = nullptr;
  CK_HIP(hipMalloc(&dout, n_out * ES));
  a.out = reinterpret_cast<float *>(dout);
  a.bias = dev_fill((size_t)Cout, hb);
  if (act) {
    a.in_scale = dev_fill((size_t)ICs, hsc);
    a.in_shift = dev_fill((size_t)ICs, hsh);
  }
  if (bnbwd) {
    a.bn_y = reinterpret_cast<const float *>(dev_fill(hy.size(), hy));
    a.bn_scale = dev_fill((size_t)a.OCs, hco);
    a.bn_shift = dev_fill((size_t)a.OCs, hco);
    a.bn_mean = dev_fill((size_t)a.OCs, hco);
    a.bn_invstd = dev_fill((size_t)a.OCs, hco);
  }
  if (!dgrad || bnbwd) {
    const size_t rows = (size_t)bconv_stat_rows(a);
    CK_HIP(hipMalloc(&a.stats, rows * a.CoutW * 4 * sizeof(float)));
  }
  if (a.ksplit > 1) CK_HIP(hipMalloc(&a.partial, (size_t)a.ksplit * a.slice_floats * sizeof(float)));

  hipStream_t s;
  CK_HIP(hipStreamCreate(&s));
  for (int i = 0; i < 3; ++i)
    if (launch_bconv(a, s)) return 1;
  CK_HIP(hipStreamSynchronize(s));
  std::vector<unsigned long long> z(kPhBlocks * kPhN, 0ull);
  CK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_bconv_phase), z.data(), z.size() * 8));
  hipEvent_t e0, e1;
  CK_HIP(hipEventCreate(&e0));
  CK_HIP(hipEventCreate(&e1));
  CK_HIP(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) launch_bconv(a, s);
  CK_HIP(hipEventRecord(e1, s));
  CK_HIP(hipEventSynchronize(e1));
  float ms = 0.f;
  CK_HIP(hipEventElapsedTime(&ms, e0, e1));
  CK_HIP(hipMemcpyFromSymbol(z.data(), HIP_SYMBOL(g_bconv_phase), z.size() * 8));
  unsigned long long ph[kPhN] = {0};
  for (int b = 0; b < kPhBlocks; ++b)
    for (int k = 0; k < kPhN; ++k) ph[k] += z[(size_t)b * kPhN + k];
  const double us = ms * 1e3 / iters;
  const double flops = 2.0 * B * a.OX * a.OY * a.OZ * (double)Cout * T * ICs;
  const double bytes = (double)ES * (n_in + n_out) + (bnbwd ? (double)ES * n_out : 0.0);
  printf("es%d %s B%d I%dx%dx%d ICs%d Cout%d K%dx%dx%d act%d | CK%d NSUB%d MPW%d T%dx%dx%d NPF%d ks%d grid%d "
         "lds%d | %.1f us  %.1f TF/s  %.0f GB/s\n",
         ES, mode.c_str(), B, IX, IY, IZ, ICs, Cout, K[0], K[1], K[2], act, a.CK, a.NSUB, a.MPW, a.TX,
         a.TY, a.TZ, a.NPF, a.ksplit, a.gridx, a.lds_bytes, us, flops / us * 1e-6,
         bytes / us * 1e-3);
  double tot = 0;
  for (int k = 0; k < 5; ++k) tot += (double)ph[k];
  const double tiles = (double)ph[5];
  if (tiles <= 0) printf("  no phase counts (raw %llu %llu %llu)\n", ph[0], ph[3], ph[5]);
  else
    printf("  per tile (wave 0, cycles): halo->lds %.0f  barrier+w %.0f  fetch %.0f  mfma %.0f  "
           "epilogue %.0f  total %.0f (tiles/launch %.0f)\n",
           ph[0] / tiles, ph[1] / tiles, ph[2] / tiles, ph[3] / tiles, ph[4] / tiles, tot / tiles,
           tiles / iters);
  const double blocks = (double)a.gridx * (a.CoutW / (a.NSUB * 16)) * a.ksplit * iters;
  printf("  per block (wave 0, cycles): prologue %.0f  lifetime %.0f  post-loop: shuffles %.0f  lds merge %.0f"
         "  rows %.0f  tail %.0f (blocks/launch %.0f)\n", ph[6] / blocks, ph[7] / blocks, ph[8] / blocks,
         ph[9] / blocks, ph[10] / blocks, ph[11] / blocks, blocks / iters);
  return 0;
}
