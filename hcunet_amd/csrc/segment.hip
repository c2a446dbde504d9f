// Tiled inference kernels: the device side of
// hcunet_amd/segment.py, the drop-in for hcat.segment.predict_segmentation_mask
// (hcat/segment.py:21-136) and hcat.utils.pad_image_with_reflections /
// calculate_indexes (hcat/utils.py:33-124).
//
// The reference pads the whole volume on the host with numpy reflections,
// slices one B=1 tile at a time, converts it to fp32 and copies it to the
// device, then crops, applies an in-place sigmoid (and threshold) and writes
// into a host mask.  Here the volume stays resident in HBM; one gather kernel
// builds a batch of tiles straight from the unpadded volume (the reflection is
// index arithmetic, NaN -> 0 and +-Inf -> 1 applied on the fly), and one
// scatter kernel per tile crops, applies the sigmoid/threshold and writes the
// device mask, in the reference's tile order (later tiles overwrite earlier
// ones where they overlap).
#include "common.h"
#include "timing.h"
#include "hcunet.h"

namespace hcu {

namespace {
// padded coordinate -> source index of numpy's reflection slices
// (image[pad-1::-1] | image | image[-1:-pad-1:-1]); padL = min(pad, n)
__device__ __forceinline__ int reflect_src(int p, int padL, int n) {
  if (p < padL) return padL - 1 - p;
  p -= padL;
  if (p < n) return p;
  return n - 1 - (p - n);
}

template <class TI>
__device__ __forceinline__ float load_clean(const TI *x, int64_t i, int clean) {
  const float v = (float)x[i];
  if (!clean) return v;
  if (v != v) return 0.f;               // image[np.isnan(image)] = 0
  if (__builtin_isinf(v)) return 1.f;   // image[np.isinf(image)] = 1
  return v;
}
}  // namespace

struct TileBatch {
  int n;
  int org[HCU_TILE_BATCH_MAX][3];   // tile origins in padded coordinates
};

// out[b][c][i][j][k] = clean(image[0][c][reflect(ox+i)][reflect(oy+j)][reflect(oz+k)])
template <class TI>
__global__ void __launch_bounds__(256) tile_gather_kernel(const TI *img, int C, int X, int Y, int Z,
                                                          int px, int py, int pz, int tx, int ty,
                                                          int tz, const TileBatch tb, int clean,
                                                          float *out) {
  const int64_t per = (int64_t)C * tx * ty * tz;
  const int64_t total = per * tb.n;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int b = (int)(e / per);
    int64_t r = e - (int64_t)b * per;
    const int k = (int)(r % tz);
    r /= tz;
    const int j = (int)(r % ty);
    r /= ty;
    const int i = (int)(r % tx);
    const int c = (int)(r / tx);
    const int sx = reflect_src(tb.org[b][0] + i, px, X);
    const int sy = reflect_src(tb.org[b][1] + j, py, Y);
    const int sz = reflect_src(tb.org[b][2] + k, pz, Z);
    out[e] = load_clean(img, (((int64_t)c * X + sx) * Y + sy) * Z + sz, clean);
  }
}

// mask[dst + w] = f(out[b][0][crop + (valid dim == 1 ? 0 : w)]) for w in the
// write box; f = sigmoid computed as the reference's in-place chain
// (x *= -1; exp; += 1; pow(-1)), then > thr as 0/1 when mode == 1.
template <class TM>
__global__ void __launch_bounds__(256) tile_scatter_kernel(const float *out, int OX, int OY, int OZ,
                                                           int cx, int cy, int cz, int bx, int by,
                                                           int bz, TM *mask, int MX, int MY, int MZ,
                                                           int dx, int dy, int dz, int wx, int wy,
                                                           int wz, int mode, float thr) {
  const int64_t total = (int64_t)wx * wy * wz;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int k = (int)(e % wz);
    const int64_t q = e / wz;
    const int j = (int)(q % wy);
    const int i = (int)(q / wy);
    const int sx = cx + (bx ? 0 : i), sy = cy + (by ? 0 : j), sz = cz + (bz ? 0 : k);
    float v = out[((int64_t)sx * OY + sy) * OZ + sz];
    v = __frcp_rn(1.f + expf(-v));
    const int64_t d = ((int64_t)(dx + i) * MY + (dy + j)) * MZ + (dz + k);
    if (mode == 1)
      mask[d] = (TM)(v > thr ? 1 : 0);
    else
      mask[d] = (TM)v;
  }
}

static int grid_for(int64_t n) {
  return (int)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 256 * 64);
}

}  // namespace hcu

using namespace hcu;

extern "C" int hcu_tile_gather(const void *image, int image_dtype, int C, int X, int Y, int Z,
                               const int *pad_lo, const int *origins, int n_tiles,
                               const int *tile_dims, int clean, float *out, hcu_stream_t stream) {
  if (!image || !pad_lo || !origins || !tile_dims || !out) return fail(HCU_ERR_INVALID, "null argument");
  if (n_tiles < 1 || n_tiles > HCU_TILE_BATCH_MAX)
    return fail(HCU_ERR_INVALID, "tile batch must hold 1.." + std::to_string(HCU_TILE_BATCH_MAX) + " tiles");
  if (C < 1 || X < 1 || Y < 1 || Z < 1) return fail(HCU_ERR_SHAPE, "empty image");
  const int pads[3] = {pad_lo[0], pad_lo[1], pad_lo[2]}, dims[3] = {X, Y, Z};
  for (int d = 0; d < 3; ++d) {
    if (pads[d] < 0 || pads[d] > dims[d]) return fail(HCU_ERR_SHAPE, "reflection pad must be in [0, size]");
    if (tile_dims[d] < 1) return fail(HCU_ERR_SHAPE, "empty tile");
  }
  TileBatch tb{};
  tb.n = n_tiles;
  for (int b = 0; b < n_tiles; ++b)
    for (int d = 0; d < 3; ++d) {
      const int o = origins[b * 3 + d];
      if (o < 0 || o + tile_dims[d] > dims[d] + 2 * pads[d])
        return fail(HCU_ERR_SHAPE, "tile outside the padded image");
      tb.org[b][d] = o;
    }
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = (int64_t)n_tiles * C * tile_dims[0] * tile_dims[1] * tile_dims[2];
  const int g = grid_for(n);
  const double bytes = (double)n * 4.0 * 2.0;
  if (image_dtype == HCU_F32)
    HCU_TIMED(s, "tile_gather_kernel", 0.0, bytes,
              HCU_LAUNCH((tile_gather_kernel<float>), dim3(g), dim3(256), 0, s,
                                 (const float *)image, C, X, Y, Z, pads[0], pads[1], pads[2],
                                 tile_dims[0], tile_dims[1], tile_dims[2], tb, clean, out));
  else if (image_dtype == HCU_F16)
    HCU_TIMED(s, "tile_gather_kernel", 0.0, bytes,
              HCU_LAUNCH((tile_gather_kernel<_Float16>), dim3(g), dim3(256), 0, s,
                                 (const _Float16 *)image, C, X, Y, Z, pads[0], pads[1], pads[2],
                                 tile_dims[0], tile_dims[1], tile_dims[2], tb, clean, out));
  else
    return fail(HCU_ERR_INVALID, "tile_gather: image must be float32 or float16");
  HCU_CHECK_LAUNCH();
  return HCU_OK;
}

extern "C" int hcu_tile_scatter(const float *out, const int *out_dims, const int *crop_lo,
                                const int *bcast, void *mask, int mask_dtype, const int *mask_dims,
                                const int *dst_lo, const int *write_dims, int threshold,
                                float thr, hcu_stream_t stream) {
  if (!out || !out_dims || !crop_lo || !bcast || !mask || !mask_dims || !dst_lo || !write_dims)
    return fail(HCU_ERR_INVALID, "null argument");
  for (int d = 0; d < 3; ++d) {
    if (write_dims[d] < 0 || dst_lo[d] < 0 || dst_lo[d] + write_dims[d] > mask_dims[d])
      return fail(HCU_ERR_SHAPE, "tile write outside the mask");
    const int span = bcast[d] ? 1 : write_dims[d];
    if (write_dims[d] > 0 && (crop_lo[d] < 0 || crop_lo[d] + span > out_dims[d]))
      return fail(HCU_ERR_SHAPE, "tile crop outside the network output");
  }
  const int64_t n = (int64_t)write_dims[0] * write_dims[1] * write_dims[2];
  if (n == 0) return HCU_OK;
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_for(n);
  const double bytes = (double)n * (4.0 + (mask_dtype == HCU_U8 ? 1.0 : 4.0));
  if (mask_dtype == HCU_U8)
    HCU_TIMED(s, "tile_scatter_kernel", 0.0, bytes,
              HCU_LAUNCH((tile_scatter_kernel<uint8_t>), dim3(g), dim3(256), 0, s, out,
                                 out_dims[0], out_dims[1], out_dims[2], crop_lo[0], crop_lo[1],
                                 crop_lo[2], bcast[0], bcast[1], bcast[2], (uint8_t *)mask,
                                 mask_dims[0], mask_dims[1], mask_dims[2], dst_lo[0], dst_lo[1],
                                 dst_lo[2], write_dims[0], write_dims[1], write_dims[2],
                                 threshold ? 1 : 0, thr));
  else if (mask_dtype == HCU_F32)
    HCU_TIMED(s, "tile_scatter_kernel", 0.0, bytes,
              HCU_LAUNCH((tile_scatter_kernel<float>), dim3(g), dim3(256), 0, s, out,
                                 out_dims[0], out_dims[1], out_dims[2], crop_lo[0], crop_lo[1],
                                 crop_lo[2], bcast[0], bcast[1], bcast[2], (float *)mask,
                                 mask_dims[0], mask_dims[1], mask_dims[2], dst_lo[0], dst_lo[1],
                                 dst_lo[2], write_dims[0], write_dims[1], write_dims[2],
                                 threshold ? 1 : 0, thr));
  else
    return fail(HCU_ERR_INVALID, "tile_scatter: mask must be float32 or uint8");
  HCU_CHECK_LAUNCH();
  return HCU_OK;
}
