// Input path of the reference's data pipeline for one or more volumes, fused
// into one HBM pass: the raw confocal stack as read from the
// tif, [Z][Y][X][C] uint16 / uint8 / float64, becomes the network input
// [B][C][X][Y][Z] fp16 exactly as the reference's chain
//   to_float    hcat/transforms.py:94-116   u16 / 2^16, u8 / 2^8 (float64)
//   reshape     hcat/transforms.py:139-157  [Z,Y,X,C] -> [X,Y,Z,C]
//   normalize   hcat/transforms.py:257-283  (v + -mean_c) / std_c (float64)
//   to_tensor   hcat/transforms.py:118-137  float64 -> fp16, -> [1,C,X,Y,Z]
// computes it: the arithmetic is float64 and the fp16 rounding is torch's
// (float64 -> float32 -> fp16, each to nearest even), so the output is
// bit-identical.  The Z <-> X transpose goes through an LDS tile
// (32 x by 32 z at one y): reads are contiguous along X*C, writes along Z.
#include "common.h"
#include "timing.h"
#include "hcunet.h"
#include <algorithm>

namespace hcu {

constexpr int kIngestMaxC = 16;
struct IngestNorm {
  double mean[kIngestMaxC], std[kIngestMaxC];
  double scale;     // to_float: 2^-16 (uint16), 2^-8 (uint8), 1 (float64 / not applied)
  int on;           // normalize applied
  int transpose;    // reshape applied: [Z,Y,X,C] -> [C][X][Y][Z]; else [C][Z][Y][X]
};

// float64 -> fp16 bits, round to nearest even (overflow -> inf, NaN kept).
__device__ __forceinline__ uint16_t d2h_rne(double d) {
  const uint64_t b = (uint64_t)__double_as_longlong(d);
  const uint32_t sign = (uint32_t)(b >> 48) & 0x8000u;
  const int e = (int)((b >> 52) & 0x7ff);
  const uint64_t mant = b & 0xFFFFFFFFFFFFFull;
  if (e == 0x7ff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));
  const int ex = e - 1023;
  if (ex > 15) return (uint16_t)(sign | 0x7c00u);
  if (ex < -25) return (uint16_t)sign;   // below half the smallest subnormal
  const uint64_t m = mant | (1ull << 52);
  const int shift = ex >= -14 ? 42 : 42 + (-14 - ex);
  uint64_t q = m >> shift;
  const uint64_t rem = m & ((1ull << shift) - 1), halfw = 1ull << (shift - 1);
  if (rem > halfw || (rem == halfw && (q & 1))) ++q;
  uint32_t h;
  if (ex >= -14) h = ((uint32_t)(ex + 15) << 10) + (uint32_t)(q - 1024);   // q == 2048 carries
  else h = (uint32_t)q;                                                     // subnormal (or carry to min normal)
  return (uint16_t)(sign | h);
}

template <typename T>
__global__ void __launch_bounds__(256)
ingest_kernel(const T *src, int Z, int Y, int X, int C, int nzt, const IngestNorm nm,
              uint16_t *dst) {
  __shared__ uint16_t tile[kIngestMaxC * 32 * 33];
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * 32, y = blockIdx.y;
  const int b = blockIdx.z / nzt, z0 = (blockIdx.z % nzt) * 32;
  const int nx = min(32, X - x0), nz = min(32, Z - z0);
  // load: [zi][xi][c] contiguous along (x, c) for each z row
  const int nld = 32 * 32 * C;
  for (int i = tid; i < nld; i += 256) {
    const int c = i % C, xi = (i / C) % 32, zi = i / (C * 32);
    if (xi < nx && zi < nz) {
      const size_t off = ((((size_t)b * Z + z0 + zi) * Y + y) * X + x0 + xi) * C + c;
      double v = (double)src[off] * nm.scale;   // exact: power-of-two scale
      if (nm.on) v = (v + -nm.mean[c]) / nm.std[c];
      // torch.as_tensor(float64, dtype=half) rounds twice: float64 -> float32,
      // then float32 -> fp16 (both to nearest even); a direct float64 -> fp16
      // rounding differs where the float32 value lands on an fp16 midpoint.
      tile[(c * 32 + xi) * 33 + zi] = d2h_rne((double)(float)v);
    }
  }
  __syncthreads();
  // store: [c][x][y][z] contiguous along z
  for (int i = tid; i < nld; i += 256) {
    const int zi = i % 32, xi = (i / 32) % 32, c = i / 1024;
    if (xi < nx && zi < nz) {
      const size_t o = nm.transpose ? ((((size_t)b * C + c) * X + x0 + xi) * Y + y) * Z + z0 + zi
                                    : ((((size_t)b * C + c) * Z + z0 + zi) * Y + y) * X + x0 + xi;
      dst[o] = tile[(c * 32 + xi) * 33 + zi];
    }
  }
}

}  // namespace hcu

using namespace hcu;

extern "C" int hcu_ingest_volume(const void *src, int src_dtype, int B, int Z, int Y, int X, int C,
                                 int to_float, int reshape, const double *mean, const double *std,
                                 void *dst, hcu_stream_t stream) {
  if (!src || !dst) return fail(HCU_ERR_INVALID, "ingest: null argument");
  if (B <= 0 || Z <= 0 || Y <= 0 || X <= 0 || C <= 0) return fail(HCU_ERR_SHAPE, "ingest: empty volume");
  if (C > kIngestMaxC) return fail(HCU_ERR_UNSUPPORTED, "ingest: more than 16 channels");
  if (Y > 65535) return fail(HCU_ERR_UNSUPPORTED, "ingest: Y > 65535");
  IngestNorm nm{};
  nm.scale = !to_float ? 1.0 : (src_dtype == HCU_U16 ? 1.0 / 65536.0 : (src_dtype == HCU_U8 ? 1.0 / 256.0 : 1.0));
  nm.transpose = reshape != 0;
  nm.on = mean != nullptr;
  if (nm.on) {
    if (!std) return fail(HCU_ERR_INVALID, "ingest: mean without std");
    for (int c = 0; c < C; ++c) {
      nm.mean[c] = mean[c];
      nm.std[c] = std[c];
    }
  }
  const int nzt = cdiv(Z, 32);
  if ((int64_t)B * nzt > 65535) return fail(HCU_ERR_UNSUPPORTED, "ingest: too many volumes");
  const dim3 grid(cdiv(X, 32), Y, B * nzt);
  hipStream_t s = (hipStream_t)stream;
  uint16_t *d = (uint16_t *)dst;
  switch (src_dtype) {
    case HCU_U16:
      HCU_TIMED(s, "ingest_kernel<u16>", 0.0, 0.0,
                HCU_LAUNCH(ingest_kernel<uint16_t>, grid, dim3(256), 0, s, (const uint16_t *)src, Z, Y,
                                   X, C, nzt, nm, d));
      break;
    case HCU_U8:
      HCU_TIMED(s, "ingest_kernel<u8>", 0.0, 0.0,
                HCU_LAUNCH(ingest_kernel<uint8_t>, grid, dim3(256), 0, s, (const uint8_t *)src, Z, Y,
                                   X, C, nzt, nm, d));
      break;
    case HCU_F64:
      HCU_TIMED(s, "ingest_kernel<f64>", 0.0, 0.0,
                HCU_LAUNCH(ingest_kernel<double>, grid, dim3(256), 0, s, (const double *)src, Z, Y,
                                   X, C, nzt, nm, d));
      break;
    default:
      return fail(HCU_ERR_INVALID, "ingest: Expected image datatype of uint8 or uint16");
  }
  HCU_CHECK_LAUNCH();
  return 0;
}
