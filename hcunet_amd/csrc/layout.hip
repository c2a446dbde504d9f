// Channels-last layout kernels of the layer-chain executor (unet.cpp,
// hcu_chain_*): the dilation sub-lattice (space-to-batch) re-layouts that let a
// large dilated Conv3d run as dilation-1 convolutions on its sub-grids
// (hcat/r_unet.py:348-353: StackedDilation's 5^3 kernels at dilation 1..5),
// the crop of a padded ConvTranspose3d output (nn.ConvTranspose3d(...,
// padding=p), hcat/r_unet.py:216-217, 319-323), and the chain output in the
// reference's NCXYZ layout with the last BatchNorm+ReLU applied.
//
// Every kernel moves 16-byte channel vectors (4 fp32 / 8 bf16 channels); the
// channel stride Cs is a multiple of that vector.
#include "common.h"
#include "timing.h"

#include <type_traits>

namespace hcu {

int layout_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 65536));
}
namespace {
// relu(v * sc + sh) on one 16-byte vector of 4 fp32 / 8 bf16 channels
__device__ __forceinline__ uint4 act16(uint4 v, const float *sc, const float *sh, int c0, bool bf) {
  if (bf) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[c0 + j], sh[c0 + j]), 0.f);
    return pack8(f);
  }
  float4 f = __builtin_bit_cast(float4, v);
  f.x = fmaxf(fmaf(f.x, sc[c0], sh[c0]), 0.f);
  f.y = fmaxf(fmaf(f.y, sc[c0 + 1], sh[c0 + 1]), 0.f);
  f.z = fmaxf(fmaf(f.z, sc[c0 + 2], sh[c0 + 2]), 0.f);
  f.w = fmaxf(fmaf(f.w, sc[c0 + 3], sh[c0 + 3]), 0.f);
  return __builtin_bit_cast(uint4, f);
}
}  // namespace

// xs[(b*N + r)][x'][y'][z'] = act(x[b][rx + Dx x'][ry + Dy y'][rz + Dz z']) (0
// outside x), r = (rx*Dy + ry)*Dz + rz, N = Dx*Dy*Dz; one 16-byte vector per
// thread.  sc == nullptr: no activation.
__global__ void __launch_bounds__(256)
s2b_kernel(const uint4 *x, const float *sc, const float *sh, uint4 *xs, int X, int Y, int Z, int NV,
           int Dx, int Dy, int Dz, int SX, int SY, int SZ, int64_t n, int bf) {
  const int per = 16 / (bf ? 2 : 4);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int64_t q = i;
    const int cv = (int)(q % NV); q /= NV;
    const int z = (int)(q % SZ); q /= SZ;
    const int y = (int)(q % SY); q /= SY;
    const int xx = (int)(q % SX); q /= SX;
    const int N = Dx * Dy * Dz;
    const int r = (int)(q % N);
    const int b = (int)(q / N);
    const int rz = r % Dz, ry = (r / Dz) % Dy, rx = r / (Dz * Dy);
    const int gx = rx + Dx * xx, gy = ry + Dy * y, gz = rz + Dz * z;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (gx < X && gy < Y && gz < Z) {
      v = x[(((int64_t)b * X + gx) * Y + gy) * (int64_t)Z * NV + (int64_t)gz * NV + cv];
      if (sc) v = act16(v, sc, sh, cv * per, bf != 0);
    }
    xs[i] = v;
  }
}

// The same two shuffles with 32-bit indices and magic-number divisions
// (FastDiv): the 64-bit forms spend six ~100-instruction software divisions
// per 16-byte vector and ran at ~3 TB/s (RDCNet: 160 launches, 2.6 ms per
// step).  Used when the vector count fits 31 bits; bitwise the same data.
struct LatticeDiv {
  FastDiv nv, sz, sy, sx, n, dz, dy, dx;
};
__global__ void __launch_bounds__(256)
s2b32_kernel(const uint4 *x, const float *sc, const float *sh, uint4 *xs, int X, int Y, int Z, int NV,
             int Dx, int Dy, int Dz, LatticeDiv dv, uint32_t n, int bf) {
  const int per = 16 / (bf ? 2 : 4);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int q, cv, z, y, xx, r, b, rz, ry, rx;
    dv.nv.divmod(i, q, cv);
    dv.sz.divmod((uint32_t)q, q, z);
    dv.sy.divmod((uint32_t)q, q, y);
    dv.sx.divmod((uint32_t)q, q, xx);
    dv.n.divmod((uint32_t)q, b, r);
    dv.dz.divmod((uint32_t)r, q, rz);
    dv.dy.divmod((uint32_t)q, rx, ry);
    const int gx = rx + Dx * xx, gy = ry + Dy * y, gz = rz + Dz * z;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (gx < X && gy < Y && gz < Z) {
      v = x[(((int64_t)b * X + gx) * Y + gy) * (int64_t)Z * NV + (int64_t)gz * NV + cv];
      if (sc) v = act16(v, sc, sh, cv * per, bf != 0);
    }
    xs[i] = v;
  }
}
// s2b with the z lattice index next to the vector index: consecutive threads
// walk one dense z row (rz fastest, then z'), so the gather reads contiguous
// rows and each lattice's z' run is written contiguously (the plain order
// reads 32 bytes every D voxels).  Thread order (cv, rz, z', y', x', rx, ry, b).
__global__ void __launch_bounds__(256)
s2b32z_kernel(const uint4 *x, const float *sc, const float *sh, uint4 *xs, int X, int Y, int Z, int NV,
              int Dx, int Dy, int Dz, int SX, int SY, int SZ, LatticeDiv dv, uint32_t n, int bf) {
  const int per = 16 / (bf ? 2 : 4);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int q, cv, rz, z, y, xx, ry, rx, b;
    dv.nv.divmod(i, q, cv);
    dv.dz.divmod((uint32_t)q, q, rz);
    dv.sz.divmod((uint32_t)q, q, z);
    dv.sy.divmod((uint32_t)q, q, y);
    dv.sx.divmod((uint32_t)q, q, xx);
    dv.dy.divmod((uint32_t)q, q, ry);
    dv.dx.divmod((uint32_t)q, b, rx);
    const int gx = rx + Dx * xx, gy = ry + Dy * y, gz = rz + Dz * z;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (gx < X && gy < Y && gz < Z) {
      v = x[(((int64_t)b * X + gx) * Y + gy) * (int64_t)Z * NV + (int64_t)gz * NV + cv];
      if (sc) v = act16(v, sc, sh, cv * per, bf != 0);
    }
    const int r = (rx * Dy + ry) * Dz + rz;
    xs[((((int64_t)b * Dx * Dy * Dz + r) * SX + xx) * SY + y) * (int64_t)SZ * NV + (int64_t)z * NV + cv] = v;
  }
}

// (dv.sz / sy / sx here divide by the output extents OZ / OY / OX and dv.dz /
// dy / dx by the lattice)
__global__ void __launch_bounds__(256)
b2s32_kernel(const uint4 *ys, uint4 *y, int NV, int Dx, int Dy, int Dz, int SX, int SY, int SZ, LatticeDiv dv,
             uint32_t n) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    int q, cv, oz, oy, ox, b, qz, rz, qy, ry, qx, rx;
    dv.nv.divmod(i, q, cv);
    dv.sz.divmod((uint32_t)q, q, oz);
    dv.sy.divmod((uint32_t)q, q, oy);
    dv.sx.divmod((uint32_t)q, b, ox);
    dv.dz.divmod((uint32_t)oz, qz, rz);
    dv.dy.divmod((uint32_t)oy, qy, ry);
    dv.dx.divmod((uint32_t)ox, qx, rx);
    const int r = (rx * Dy + ry) * Dz + rz;
    const int64_t bs = (int64_t)b * Dx * Dy * Dz + r;
    y[i] = ys[(((bs * SX + qx) * SY + qy) * SZ + qz) * NV + cv];
  }
}

// y[b][o] = ys[(b*N + r)][o'] for every output voxel o = r + D o' (< OX, OY, OZ).
__global__ void __launch_bounds__(256)
b2s_kernel(const uint4 *ys, uint4 *y, int OX, int OY, int OZ, int NV, int Dx, int Dy, int Dz,
           int SX, int SY, int SZ, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int64_t q = i;
    const int cv = (int)(q % NV); q /= NV;
    const int oz = (int)(q % OZ); q /= OZ;
    const int oy = (int)(q % OY); q /= OY;
    const int ox = (int)(q % OX);
    const int b = (int)(q / OX);
    const int r = ((ox % Dx) * Dy + oy % Dy) * Dz + oz % Dz;
    const int64_t bs = (int64_t)b * Dx * Dy * Dz + r;
    y[i] = ys[(((bs * SX + ox / Dx) * SY + oy / Dy) * SZ + oz / Dz) * NV + cv];
  }
}

// dst[b][x][y][z] = src[b][x + ox][y + oy][z + oz] (channels-last box copy).
__global__ void __launch_bounds__(256)
crop_kernel(const uint4 *src, uint4 *dst, int SX, int SY, int SZ, int DX, int DY, int DZ, int NV,
            int ox, int oy, int oz, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int64_t q = i;
    const int cv = (int)(q % NV); q /= NV;
    const int z = (int)(q % DZ); q /= DZ;
    const int y = (int)(q % DY); q /= DY;
    const int x = (int)(q % DX);
    const int b = (int)(q / DX);
    dst[i] = src[((((int64_t)b * SX + x + ox) * SY + y + oy) * SZ + z + oz) * NV + cv];
  }
}

// out[b][c][v] = act(y[b][v][c]) (NCXYZ fp32; act = relu(y*sc + sh) or identity).
template <bool BF>
__global__ void __launch_bounds__(256)
from_cl_act_kernel(const void *y, const float *sc, const float *sh, float *out, int C, int Cs, int64_t V,
                   int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t v = i % V, q = i / V;
    const int c = (int)(q % C);
    const int64_t b = q / C;
    const int64_t src = (b * V + v) * Cs + c;
    float f = BF ? bf2f(reinterpret_cast<const uint16_t *>(y)[src]) : reinterpret_cast<const float *>(y)[src];
    if (sc) f = fmaxf(fmaf(f, sc[c], sh[c]), 0.f);
    out[i] = f;
  }
}

int launch_s2b(const float *x, const float *sc, const float *sh, float *xs, int B, int X, int Y, int Z,
               int Cs, int es, const int *D, const int *S, hipStream_t s) {
  const int NV = Cs * es / 16;
  const int64_t n = (int64_t)B * D[0] * D[1] * D[2] * S[0] * S[1] * S[2] * NV;
  if (n < (int64_t)1 << 31 && !getenv("HCU_LAYOUT64")) {
    LatticeDiv dv;
    dv.nv = FastDiv(NV);
    dv.sz = FastDiv(S[2]);
    dv.sy = FastDiv(S[1]);
    dv.sx = FastDiv(S[0]);
    dv.n = FastDiv(D[0] * D[1] * D[2]);
    dv.dz = FastDiv(D[2]);
    dv.dy = FastDiv(D[1]);
    dv.dx = FastDiv(D[0]);
    // (RDCNet, 3 interleaved runs each: 27.09-27.19 -> 26.86-26.93 ms per step;
    // HCU_S2B_ZFAST=0 keeps the sub-lattice-order kernel, A/B)
    static const bool zfast = !(getenv("HCU_S2B_ZFAST") && getenv("HCU_S2B_ZFAST")[0] == '0');
    if (zfast) {
      HCU_TIMED(s, "s2b_kernel", 0.0, 16.0 * n * 2,
                HCU_LAUNCH(s2b32z_kernel, dim3(layout_grid(n)), dim3(256), 0, s, (const uint4 *)x, sc, sh,
                           (uint4 *)xs, X, Y, Z, NV, D[0], D[1], D[2], S[0], S[1], S[2], dv, (uint32_t)n,
                           es == 2));
      HCU_CHECK_LAUNCH();
      return 0;
    }
    HCU_TIMED(s, "s2b_kernel", 0.0, 16.0 * n * 2,
              HCU_LAUNCH(s2b32_kernel, dim3(layout_grid(n)), dim3(256), 0, s, (const uint4 *)x, sc, sh,
                         (uint4 *)xs, X, Y, Z, NV, D[0], D[1], D[2], dv, (uint32_t)n, es == 2));
    HCU_CHECK_LAUNCH();
    return 0;
  }
  HCU_TIMED(s, "s2b_kernel", 0.0, 16.0 * n * 2,
            HCU_LAUNCH(s2b_kernel, dim3(layout_grid(n)), dim3(256), 0, s, (const uint4 *)x, sc, sh,
                               (uint4 *)xs, X, Y, Z, NV, D[0], D[1], D[2], S[0], S[1], S[2], n, es == 2));
  HCU_CHECK_LAUNCH();
  return 0;
}

int launch_b2s(const float *ys, float *y, int B, int OX, int OY, int OZ, int Cs, int es, const int *D,
               const int *S, hipStream_t s) {
  const int NV = Cs * es / 16;
  const int64_t n = (int64_t)B * OX * OY * OZ * NV;
  if (n < (int64_t)1 << 31 && !getenv("HCU_LAYOUT64")) {
    LatticeDiv dv;
    dv.nv = FastDiv(NV);
    dv.sz = FastDiv(OZ);
    dv.sy = FastDiv(OY);
    dv.sx = FastDiv(OX);
    dv.n = FastDiv(1);
    dv.dz = FastDiv(D[2]);
    dv.dy = FastDiv(D[1]);
    dv.dx = FastDiv(D[0]);
    HCU_TIMED(s, "b2s_kernel", 0.0, 16.0 * n * 2,
              HCU_LAUNCH(b2s32_kernel, dim3(layout_grid(n)), dim3(256), 0, s, (const uint4 *)ys, (uint4 *)y, NV,
                         D[0], D[1], D[2], S[0], S[1], S[2], dv, (uint32_t)n));
    HCU_CHECK_LAUNCH();
    return 0;
  }
  HCU_TIMED(s, "b2s_kernel", 0.0, 16.0 * n * 2,
            HCU_LAUNCH(b2s_kernel, dim3(layout_grid(n)), dim3(256), 0, s, (const uint4 *)ys, (uint4 *)y,
                               OX, OY, OZ, NV, D[0], D[1], D[2], S[0], S[1], S[2], n));
  HCU_CHECK_LAUNCH();
  return 0;
}

int launch_crop_cl(const float *src, float *dst, int B, const int *sdims, const int *ddims, const int *off,
                   int Cs, int es, hipStream_t s) {
  const int NV = Cs * es / 16;
  const int64_t n = (int64_t)B * ddims[0] * ddims[1] * ddims[2] * NV;
  HCU_TIMED(s, "crop_kernel", 0.0, 16.0 * n * 2,
            HCU_LAUNCH(crop_kernel, dim3(layout_grid(n)), dim3(256), 0, s, (const uint4 *)src,
                               (uint4 *)dst, sdims[0], sdims[1], sdims[2], ddims[0], ddims[1], ddims[2], NV,
                               off[0], off[1], off[2], n));
  HCU_CHECK_LAUNCH();
  return 0;
}

// NCXYZ <-> channels-last through an LDS tile of 64 voxels x Cs channels:
// the channels-last side moves as contiguous 16-byte vectors, the NCXYZ side
// as 64 consecutive voxels of one channel (256-byte fp32 rows).  One
// workgroup per 64-voxel tile (grid.x tiles, grid.y batch).
constexpr int kTileV = 64;
template <bool BF>
__global__ void __launch_bounds__(256)
from_cl_tile_kernel(const void *y, const float *sc, const float *sh, float *out, int C, int Cs, int64_t V) {
  extern __shared__ float tl[];   // [kTileV][Cs + 1]
  const int tid = threadIdx.x;
  const int64_t v0 = (int64_t)blockIdx.x * kTileV;
  const int b = blockIdx.y;
  const int nv = (int)min((int64_t)kTileV, V - v0);
  const int es = BF ? 2 : 4, per = 16 / es, nvec = Cs / per;
  const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<const char *>(y) +
                                                     ((size_t)b * V + v0) * Cs * es);
  for (int i = tid; i < nv * nvec; i += 256) {
    const int v = i / nvec, cv = i % nvec;
    const uint4 q = src[i];
    float f[8];
    if (BF) {
      unpack8(q, f);
    } else {
      const float4 g = __builtin_bit_cast(float4, q);
      f[0] = g.x; f[1] = g.y; f[2] = g.z; f[3] = g.w;
    }
    for (int j = 0; j < per; ++j) tl[v * (Cs + 1) + cv * per + j] = f[j];
  }
  __syncthreads();
  for (int i = tid; i < C * kTileV; i += 256) {
    const int c = i / kTileV, v = i % kTileV;
    if (v >= nv) continue;
    float f = tl[v * (Cs + 1) + c];
    if (sc) f = fmaxf(fmaf(f, sc[c], sh[c]), 0.f);
    out[((size_t)b * C + c) * V + v0 + v] = f;
  }
}

// x_dtype: 0 fp32, 1 fp16, 3 bf16 input; BF: bf16 channels-last output.
template <typename TI, bool BF>
__global__ void __launch_bounds__(256)
to_cl_tile_kernel(const TI *x, void *xcl, int C, int Cs, int64_t V) {
  extern __shared__ float tl[];   // [kTileV][Cs + 1]
  const int tid = threadIdx.x;
  const int64_t v0 = (int64_t)blockIdx.x * kTileV;
  const int b = blockIdx.y;
  const int nv = (int)min((int64_t)kTileV, V - v0);
  for (int i = tid; i < Cs * kTileV; i += 256) {
    const int c = i / kTileV, v = i % kTileV;
    float f = 0.f;
    if (c < C && v < nv) {
      const TI w = x[((size_t)b * C + c) * V + v0 + v];
      if constexpr (sizeof(TI) == 2 && !std::is_same<TI, _Float16>::value)
        f = bf2f(__builtin_bit_cast(uint16_t, w));
      else
        f = (float)w;
    }
    tl[v * (Cs + 1) + c] = f;
  }
  __syncthreads();
  const int es = BF ? 2 : 4, per = 16 / es, nvec = Cs / per;
  uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<char *>(xcl) + ((size_t)b * V + v0) * Cs * es);
  for (int i = tid; i < nv * nvec; i += 256) {
    const int v = i / nvec, cv = i % nvec;
    const float *r = tl + v * (Cs + 1) + cv * per;
    if (BF) {
      float f[8];
      for (int j = 0; j < 8; ++j) f[j] = r[j];
      dst[i] = pack8(f);
    } else {
      dst[i] = __builtin_bit_cast(uint4, make_float4(r[0], r[1], r[2], r[3]));
    }
  }
}

// Tiled layout changes for channel strides up to 128 (else -1: caller falls back).
int launch_from_cl_tiled(const float *y, const float *sc, const float *sh, float *out, int B, int C, int Cs,
                         int64_t V, hipStream_t s, int bf) {
  if (Cs > 128 || B > 65535) return -1;
  const dim3 grid((unsigned)((V + kTileV - 1) / kTileV), B);
  const size_t lds = (size_t)kTileV * (Cs + 1) * sizeof(float);
  const double by = (double)B * V * (C * 4.0 + Cs * (bf ? 2.0 : 4.0));
  if (bf)
    HCU_TIMED(s, "from_cl_tile_kernel", 0.0, by,
              HCU_LAUNCH(from_cl_tile_kernel<true>, grid, dim3(256), lds, s, (const void *)y, sc, sh,
                                 out, C, Cs, V));
  else
    HCU_TIMED(s, "from_cl_tile_kernel", 0.0, by,
              HCU_LAUNCH(from_cl_tile_kernel<false>, grid, dim3(256), lds, s, (const void *)y, sc, sh,
                                 out, C, Cs, V));
  HCU_CHECK_LAUNCH();
  return 0;
}

int launch_to_cl_tiled(const float *x, float *xcl, int B, int C, int Cs, int64_t V, hipStream_t s, int bf,
                       int x_dtype) {
  if (Cs > 128 || B > 65535) return -1;
  const dim3 grid((unsigned)((V + kTileV - 1) / kTileV), B);
  const size_t lds = (size_t)kTileV * (Cs + 1) * sizeof(float);
  const double by = (double)B * V * (C * (x_dtype == 0 ? 4.0 : 2.0) + Cs * (bf ? 2.0 : 4.0));
#define TOCL(TI_, BF_)                                                                                    \
  HCU_TIMED(s, "to_cl_tile_kernel", 0.0, by,                                                             \
            HCU_LAUNCH((to_cl_tile_kernel<TI_, BF_>), grid, dim3(256), lds, s, (const TI_ *)x,     \
                               (void *)xcl, C, Cs, V))
  if (x_dtype == 0 && bf) TOCL(float, true);
  else if (x_dtype == 0) TOCL(float, false);
  else if (x_dtype == 1 && bf) TOCL(_Float16, true);
  else if (x_dtype == 1) TOCL(_Float16, false);
  else if (x_dtype == 3 && bf) TOCL(uint16_t, true);
  else return -1;
#undef TOCL
  HCU_CHECK_LAUNCH();
  return 0;
}

int launch_from_cl_act(const float *y, const float *sc, const float *sh, float *out, int B, int C, int Cs,
                       int64_t V, hipStream_t s, int bf) {
  if (launch_from_cl_tiled(y, sc, sh, out, B, C, Cs, V, s, bf) == 0) return 0;
  const int64_t n = (int64_t)B * C * V;
  if (bf)
    HCU_TIMED(s, "from_cl_act_kernel", 0.0, 6.0 * n,
              HCU_LAUNCH(from_cl_act_kernel<true>, dim3(layout_grid(n)), dim3(256), 0, s, (const void *)y,
                                 sc, sh, out, C, Cs, V, n));
  else
    HCU_TIMED(s, "from_cl_act_kernel", 0.0, 8.0 * n,
              HCU_LAUNCH(from_cl_act_kernel<false>, dim3(layout_grid(n)), dim3(256), 0, s,
                                 (const void *)y, sc, sh, out, C, Cs, V, n));
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu

// ---------------------------------------------------------------------------
// The gated recurrence of RecursiveUnet.forward (hcat/r_unet.py:150-155):
//   h = tanh(hp), z = sigmoid(zp), out = h_prev * z + (-1 * z * h)
// (h_prev == nullptr: ones, the t == 0 state, :152-153) and its gradient.
namespace hcu {
__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + expf(-v)); }

__global__ void __launch_bounds__(256)
gate_fwd_kernel(const float *hp, const float *zp, const float *hprev, float *out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float h = tanhf(hp[i]), z = sigm(zp[i]);
    const float hv = hprev ? hprev[i] : 1.f;
    out[i] = hv * z + (-1.f * z * h);
  }
}

__global__ void __launch_bounds__(256)
gate_bwd_kernel(const float *hp, const float *zp, const float *hprev, const float *dout, float *dhp,
                float *dzp, float *dhprev, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float h = tanhf(hp[i]), z = sigm(zp[i]);
    const float hv = hprev ? hprev[i] : 1.f;
    const float g = dout[i];
    if (dhprev) dhprev[i] = g * z;
    dzp[i] = g * (hv - h) * (z * (1.f - z));
    dhp[i] = -g * z * (1.f - h * h);
  }
}
}  // namespace hcu

extern "C" {
int hcu_gate_fwd(const float *hp, const float *zp, const float *hprev, float *out, int64_t n, void *stream) {
  if (!hp || !zp || !out || n < 0) return hcu::fail(1, "null argument");
  hipStream_t s = (hipStream_t)stream;
  HCU_TIMED(s, "gate_fwd_kernel", 0.0, 16.0 * n,
            HCU_LAUNCH(hcu::gate_fwd_kernel, dim3(hcu::layout_grid(n)), dim3(256), 0, s, hp, zp, hprev,
                               out, n));
  HCU_CHECK_LAUNCH();
  return 0;
}
int hcu_gate_bwd(const float *hp, const float *zp, const float *hprev, const float *dout, float *dhp,
                 float *dzp, float *dhprev, int64_t n, void *stream) {
  if (!hp || !zp || !dout || !dhp || !dzp || n < 0) return hcu::fail(1, "null argument");
  hipStream_t s = (hipStream_t)stream;
  HCU_TIMED(s, "gate_bwd_kernel", 0.0, 28.0 * n,
            HCU_LAUNCH(hcu::gate_bwd_kernel, dim3(hcu::layout_grid(n)), dim3(256), 0, s, hp, zp, hprev,
                               dout, dhp, dzp, dhprev, n));
  HCU_CHECK_LAUNCH();
  return 0;
}
}  // extern "C"

// ---------------------------------------------------------------------------
// The BatchNorm running statistics in and out of the data-parallel
// communication buffer (hcunet_amd/dist.py): n small vectors gathered into /
// scattered from one contiguous buffer in one launch (one workgroup each).
namespace hcu {
constexpr int kVecMax = 128;
struct VecList {
  float *p[kVecMax];
  int off[kVecMax + 1];
  int n, unpack;
};
__global__ void __launch_bounds__(256) vec_gather_kernel(const VecList v, float *buf) {
  const int j = blockIdx.x;
  float *p = v.p[j];
  const int o = v.off[j], len = v.off[j + 1] - o;
  for (int i = threadIdx.x; i < len; i += 256) {
    if (v.unpack) p[i] = buf[o + i];
    else buf[o + i] = p[i];
  }
}
}  // namespace hcu

extern "C" int hcu_gather_vectors(float *const *vecs, const int *lens, int n, float *buf, int unpack,
                                  void *stream) {
  if (n < 0 || n > hcu::kVecMax || (n && (!vecs || !lens || !buf)))
    return hcu::fail(1, "hcu_gather_vectors: 0..128 vectors");
  if (n == 0) return 0;
  hcu::VecList v{};
  v.off[0] = 0;
  for (int i = 0; i < n; ++i) {
    v.p[i] = vecs[i];
    v.off[i + 1] = v.off[i] + lens[i];
  }
  v.n = n;
  v.unpack = unpack != 0;
  hipStream_t s = (hipStream_t)stream;
  HCU_TIMED(s, "vec_gather_kernel", 0.0, 8.0 * v.off[n],
            HCU_LAUNCH(hcu::vec_gather_kernel, dim3(n), dim3(256), 0, s, v, buf));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Channel cat / split of channels-last tensors ([rows][C] with C the padded
// channel slots of the executor's layout): RDCNet's recurrence concatenates
// its state with the strided convolution's output and the five dilated
// branches along channels (hcat/r_unet.py:223, :362).  torch's cat copies
// each part into a strided slice of the output, and its backward hands every
// consumer a strided slice that is copied again; here both directions are
// one launch over 16-byte vectors, coalesced on the full tensor's side.
namespace hcu {
constexpr int kCatMax = 8;
struct CatList {
  uint4 *p[kCatMax];      // part bases
  int off[kCatMax + 1];   // first vector of part i in a row; off[n] = row width
  int n;
};
__global__ void __launch_bounds__(256) cl_cat_kernel(const CatList c, uint4 *full, uint32_t nvec, int split) {
  const uint32_t W = (uint32_t)c.off[c.n];
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nvec; i += gridDim.x * 256u) {
    const uint32_t row = i / W, j = i - row * W;
    // part of column j (compile-time indices into the argument block: no
    // dynamically indexed copy of it)
    uint4 *base = c.p[0];
    uint32_t o = 0, w = (uint32_t)c.off[1];
#pragma unroll
    for (int q = 1; q < kCatMax; ++q)
      if (q < c.n && j >= (uint32_t)c.off[q]) {
        base = c.p[q];
        o = (uint32_t)c.off[q];
        w = (uint32_t)(c.off[q + 1] - c.off[q]);
      }
    uint4 *pp = base + (size_t)row * w + (j - o);
    if (split) *pp = full[i];
    else full[i] = *pp;
  }
}
}  // namespace hcu

extern "C" int hcu_cl_cat(void *const *parts, const int *part_row_bytes, int nparts, void *full, int64_t rows,
                          int split, void *stream) {
  if (nparts < 1 || nparts > hcu::kCatMax || !parts || !part_row_bytes || !full || rows < 0)
    return hcu::fail(1, "hcu_cl_cat: 1..8 parts, non-null buffers");
  hcu::CatList c{};
  c.off[0] = 0;
  for (int i = 0; i < nparts; ++i) {
    if (!parts[i] || part_row_bytes[i] <= 0 || part_row_bytes[i] % 16 ||
        reinterpret_cast<uintptr_t>(parts[i]) % 16)
      return hcu::fail(1, "hcu_cl_cat: parts must be 16-byte aligned with rows of 16-byte multiples");
    c.p[i] = static_cast<uint4 *>(parts[i]);
    c.off[i + 1] = c.off[i] + part_row_bytes[i] / 16;
  }
  c.n = nparts;
  if (reinterpret_cast<uintptr_t>(full) % 16) return hcu::fail(1, "hcu_cl_cat: full tensor not 16-byte aligned");
  const double nv = (double)rows * c.off[nparts];
  if (nv >= 4294967295.0) return hcu::fail(4, "hcu_cl_cat: more than 2^32 vectors");
  if (nv == 0) return 0;
  const uint32_t nvec = (uint32_t)nv;
  hipStream_t s = (hipStream_t)stream;
  HCU_TIMED(s, split ? "cl_split_kernel" : "cl_cat_kernel", 0.0, 32.0 * nv,
            HCU_LAUNCH(hcu::cl_cat_kernel, dim3(hcu::layout_grid(nvec)), dim3(256), 0, s, c,
                       static_cast<uint4 *>(full), nvec, split));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// RDCNet's residual state under bf16 autocast (hcat/r_unet.py:223-225): the
// block output m (bf16) plus the fp32 state y promotes to fp32, and the next
// step's cat takes its bf16 cast.  Forward: out = float(m) + y and out_c =
// bf16(out) (round to nearest even, as torch's cast) in one pass.  Backward:
// g = g32 + float(gc) (either nullable: a missing one contributes nothing),
// dy = g, dm = bf16(g) -- the add's and the cast's backward together.
namespace hcu {
__global__ void __launch_bounds__(256) resid_fwd_kernel(const uint4 *m, const float4 *y, float4 *out, uint4 *outc,
                                                        uint32_t nv) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nv; i += gridDim.x * 256u) {
    float f[8];
    unpack8(m[i], f);
    const float4 y0 = y[2 * i], y1 = y[2 * i + 1];
    f[0] += y0.x; f[1] += y0.y; f[2] += y0.z; f[3] += y0.w;
    f[4] += y1.x; f[5] += y1.y; f[6] += y1.z; f[7] += y1.w;
    out[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    out[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
    outc[i] = pack8(f);
  }
}
__global__ void __launch_bounds__(256) resid_bwd_kernel(const float4 *g32, const uint4 *gc, float4 *dy, uint4 *dm,
                                                        uint32_t nv) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nv; i += gridDim.x * 256u) {
    float f[8];
    if (gc) {
      unpack8(gc[i], f);
      if (g32) {
        const float4 a = g32[2 * i], b = g32[2 * i + 1];
        f[0] = a.x + f[0]; f[1] = a.y + f[1]; f[2] = a.z + f[2]; f[3] = a.w + f[3];
        f[4] = b.x + f[4]; f[5] = b.y + f[5]; f[6] = b.z + f[6]; f[7] = b.w + f[7];
      }
    } else {
      const float4 a = g32[2 * i], b = g32[2 * i + 1];
      f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
      f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
    }
    dy[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    dy[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
    dm[i] = pack8(f);
  }
}
}  // namespace hcu

namespace {
bool al16(const void *p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }
}  // namespace

extern "C" int hcu_resid_fwd(const void *m, const float *y, float *out, void *out_c, int64_t n, void *stream) {
  if (!m || !y || !out || !out_c || n < 0 || n % 8 || !al16(m) || !al16(y) || !al16(out) || !al16(out_c))
    return hcu::fail(1, "hcu_resid_fwd: non-null 16-byte aligned buffers, n a multiple of 8");
  if ((double)n / 8 >= 4294967295.0) return hcu::fail(4, "hcu_resid_fwd: too many elements");
  if (n == 0) return 0;
  const uint32_t nv = (uint32_t)(n / 8);
  hipStream_t s = (hipStream_t)stream;
  HCU_TIMED(s, "resid_fwd_kernel", 0.0, 12.0 * n,
            HCU_LAUNCH(hcu::resid_fwd_kernel, dim3(hcu::layout_grid(nv)), dim3(256), 0, s,
                       static_cast<const uint4 *>(m), reinterpret_cast<const float4 *>(y),
                       reinterpret_cast<float4 *>(out), static_cast<uint4 *>(out_c), nv));
  HCU_CHECK_LAUNCH();
  return 0;
}

extern "C" int hcu_resid_bwd(const float *g32, const void *gc, float *dy, void *dm, int64_t n, void *stream) {
  if ((!g32 && !gc) || !dy || !dm || n < 0 || n % 8 || (g32 && !al16(g32)) || (gc && !al16(gc)) || !al16(dy) ||
      !al16(dm))
    return hcu::fail(1, "hcu_resid_bwd: a gradient, 16-byte aligned buffers, n a multiple of 8");
  if ((double)n / 8 >= 4294967295.0) return hcu::fail(4, "hcu_resid_bwd: too many elements");
  if (n == 0) return 0;
  const uint32_t nv = (uint32_t)(n / 8);
  hipStream_t s = (hipStream_t)stream;
  HCU_TIMED(s, "resid_bwd_kernel", 0.0, (g32 ? 4.0 : 0.0) * n + (gc ? 2.0 : 0.0) * n + 6.0 * n,
            HCU_LAUNCH(hcu::resid_bwd_kernel, dim3(hcu::layout_grid(nv)), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(g32), static_cast<const uint4 *>(gc),
                       reinterpret_cast<float4 *>(dy), static_cast<uint4 *>(dm), nv));
  HCU_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Sum of the gradients of a tensor that feeds several chains (RDCNet: the
// block input h feeds the five dilated branches, the strided convolution's
// output x the ten recurrence steps): autograd would add them pairwise, one
// launch and one rounding per add; here one launch sums n <= 16 of them in
// fp32 in input order and rounds once.  bf = 1: bf16 elements, else fp32;
// null inputs contribute nothing.
namespace hcu {
constexpr int kSumMax = 16;
struct SumList {
  const uint4 *p[kSumMax];
  int n;
};
template <bool BF>
__global__ void __launch_bounds__(256) sum_parts_kernel(const SumList l, uint4 *out, uint32_t nv) {
  constexpr int N = BF ? 8 : 4;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nv; i += gridDim.x * 256u) {
    float acc[N];
#pragma unroll
    for (int j = 0; j < N; ++j) acc[j] = 0.f;
    bool first = true;
#pragma unroll
    for (int q = 0; q < kSumMax; ++q) {
      if (q >= l.n || !l.p[q]) continue;
      const uint4 v = l.p[q][i];
      float f[N];
      if constexpr (BF) {
        unpack8(v, f);
      } else {
        f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
        f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
      }
#pragma unroll
      for (int j = 0; j < N; ++j) acc[j] = first ? f[j] : acc[j] + f[j];
      first = false;
    }
    if constexpr (BF) {
      out[i] = pack8(acc);
    } else {
      out[i] = make_uint4(__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]),
                          __float_as_uint(acc[3]));
    }
  }
}
}  // namespace hcu

extern "C" int hcu_sum_parts(const void *const *parts, int nparts, void *out, int64_t n, int bf, void *stream) {
  const int per = bf ? 8 : 4;
  if (nparts < 1 || nparts > hcu::kSumMax || !parts || !out || n < 0 || n % per || !al16(out))
    return hcu::fail(1, "hcu_sum_parts: 1..16 inputs, 16-byte aligned, n a multiple of the vector");
  hcu::SumList l{};
  int live = 0;
  for (int i = 0; i < nparts; ++i) {
    if (parts[i] && !al16(parts[i])) return hcu::fail(1, "hcu_sum_parts: input not 16-byte aligned");
    l.p[i] = static_cast<const uint4 *>(parts[i]);
    live += parts[i] != nullptr;
  }
  if (!live) return hcu::fail(1, "hcu_sum_parts: no input");
  l.n = nparts;
  if ((double)n / per >= 4294967295.0) return hcu::fail(4, "hcu_sum_parts: too many elements");
  if (n == 0) return 0;
  const uint32_t nv = (uint32_t)(n / per);
  hipStream_t s = (hipStream_t)stream;
  if (bf)
    HCU_TIMED(s, "sum_parts_kernel", 0.0, 2.0 * n * (live + 1),
              HCU_LAUNCH(hcu::sum_parts_kernel<true>, dim3(hcu::layout_grid(nv)), dim3(256), 0, s, l,
                         static_cast<uint4 *>(out), nv));
  else
    HCU_TIMED(s, "sum_parts_kernel", 0.0, 4.0 * n * (live + 1),
              HCU_LAUNCH(hcu::sum_parts_kernel<false>, dim3(hcu::layout_grid(nv)), dim3(256), 0, s, l,
                         static_cast<uint4 *>(out), nv));
  HCU_CHECK_LAUNCH();
  return 0;
}
