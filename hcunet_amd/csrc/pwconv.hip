// 1x1x1 Conv3d forward and input gradient on bf16 channels-last tensors
// without BatchNorm (RDCNet's mixing convolutions, hcat/r_unet.py:354-364 and
// :372-374: StackedDilation.out_conv 50 -> 10 on the cat of the five dilated
// branches, RDCBlock.conv 20 -> 10 on cat(x, y)).
//
// A 1x1 convolution is a GEMM of the voxels with a tiny weight matrix: per
// voxel 160 B (5 channel parts x 16 slots) read and 32 B written, ~2 MFMAs.
// The implicit-GEMM bconv kernel stages every (16-channel) chunk of such a
// tile through LDS behind barriers and ran at ~2 TB/s; here each wave streams
// 16-voxel groups straight from HBM into MFMA B fragments (one 16-byte load
// per lane and 32-channel K step), keeps the weights as A fragments in
// registers for the whole launch, and stores each lane's 4 consecutive output
// channels of one voxel as one 8-byte store (the accumulator holds the
// transposed tile: D[channel][voxel]).  The weights are read in the PyTorch
// layout and rounded to bf16 exactly as prep_all does, with the channel-part
// map of ConvLayer::part_c (packed slot e -> torch channel (e / part_cs) *
// part_c + e % part_cs, or padding).
//
//   forward:  out[v][o] = bias[o] + sum_e in[v][e] * W[o][torch(e)]
//   dgrad:    dx[v][e]  = sum_o dy[v][o] * W[o][torch(e)]
// fp32 accumulation in K-step order; 0 in every padding slot of the output.
#include "common.h"
#include "timing.h"
#include <algorithm>

namespace hcu {

namespace {

// torch input channel of packed slot e (-1: padding)
__device__ __forceinline__ int pw_torch_channel(int e, int Cin, int part_c, int part_cs) {
  if (part_cs > 0) {
    const int r = e % part_cs;
    return r < part_c ? (e / part_cs) * part_c + r : -1;
  }
  return e < Cin ? e : -1;
}

// KS K-steps of 32 input slots, NS output subtiles of 16, G voxel groups of 16
// per wave iteration (their loads issued together).
template <int KS, int NS, int G>
__global__ void __launch_bounds__(256) pw_kernel(const PwArgs a) {
  const int lane = threadIdx.x & 63;
  const int r16 = lane & 15, kq = lane >> 4;
  // A fragments: row = output channel / slot (ns*16 + r16), k = ks*32 + 8*kq + j
  shortx8 wa[KS][NS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int ns = 0; ns < NS; ++ns) {
      const int row = ns * 16 + r16;
      shortx8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = ks * 32 + 8 * kq + j;
        float v = 0.f;
        if (!a.dgrad) {   // row = out channel o, k = input slot e
          const int tc = k < a.ICs ? pw_torch_channel(k, a.Cin, a.part_c, a.part_cs) : -1;
          if (row < a.Cout && tc >= 0) v = a.w[(size_t)row * a.Cin + tc];
        } else {          // row = input slot e, k = out channel o
          const int tc = row < a.OCs ? pw_torch_channel(row, a.Cin, a.part_c, a.part_cs) : -1;
          if (k < a.Cout && tc >= 0) v = a.w[(size_t)k * a.Cin + tc];
        }
        f[j] = (short)f2bf(v);
      }
      wa[ks][ns] = f;
    }
  float bias[NS][4];
#pragma unroll
  for (int ns = 0; ns < NS; ++ns)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = ns * 16 + 4 * kq + i;
      bias[ns][i] = (!a.dgrad && a.bias && o < a.Cout) ? a.bias[o] : 0.f;
    }
  const long ngroups = (a.nvox + 15) / 16;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nwaves = (long)gridDim.x * 4;
  // buffer loads with offsets relative to a group's first voxel: out of range
  // (past the tensor or past the input's channel stride) reads 0
  // (num_records = the tensor's bytes: the 0x7ffffff0 sentinel lies past it)
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc((void *)a.in, 0, (int)(a.nvox * a.ICs * 2), 0x00020000);
  for (long g0 = wave * G; g0 < ngroups; g0 += nwaves * G) {
    shortx8 b[G][KS];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const long v = (g0 + gi) * 16 + r16;
      const bool vok = v < a.nvox;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int c = ks * 32 + 8 * kq;
        const bool ok = vok && c < a.ICs;
        // (64-bit voxel base folded into the resource would need a descriptor
        // per group; the tensors here stay below 2 GiB: launch_pw checks)
        const int off = ok ? (int)((v * a.ICs + c) * 2) : 0x7ffffff0;
        b[gi][ks] = __builtin_bit_cast(shortx8, __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 0));
      }
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const long v = (g0 + gi) * 16 + r16;
      floatx4 acc[NS];
#pragma unroll
      for (int ns = 0; ns < NS; ++ns) acc[ns] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int ns = 0; ns < NS; ++ns)
          acc[ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][ns], b[gi][ks], acc[ns], 0, 0, 0);
      if (v >= a.nvox) continue;
#pragma unroll
      for (int ns = 0; ns < NS; ++ns) {
        const int c0 = ns * 16 + 4 * kq;
        if (c0 >= a.OCs) continue;
        const uint2 w = make_uint2(pack_bf2(acc[ns][0] + bias[ns][0], acc[ns][1] + bias[ns][1]),
                                   pack_bf2(acc[ns][2] + bias[ns][2], acc[ns][3] + bias[ns][3]));
        *reinterpret_cast<uint2 *>(a.out + v * a.OCs + c0) = w;
      }
    }
  }
}

// Weight and bias gradient of the same 1x1x1 convolutions, on the VALU:
//   dW[e][o] = sum_v A[v][e] * G[v][o],   db[o] = sum_v G[v][o]
// (80 x 16 slots at most: 1.3 KFLOP per voxel, too little to stage for the
// MFMA's voxel-major K through transposed LDS reads).  A block takes a
// contiguous voxel range in 64-voxel chunks (the next chunk's 16-byte loads in
// registers while the current one is summed from LDS); a thread owns 8 input
// slots x 8 output channels (64 fp32 accumulators from 32 B of LDS per voxel:
// 4 bytes of LDS per accumulator update was the limit of a 8 x 4 ownership)
// for one voxel subset; the subsets are summed in a fixed order at the end
// and the block writes one slab in bwgrad's taps_rows layout (WGradArgs Mtot
// / Ntot / ACr / GCr, bias row last) for wgrad_finalize.
constexpr int kPwNV = 64;        // voxels per chunk
constexpr int kPwLoads = 4;      // 16-byte staging loads per thread and chunk (A + G)

__global__ void __launch_bounds__(256) pw_wgrad_kernel(const PwWgArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 pw_lds[];
  const int tid = threadIdx.x;
  const int E8 = a.ACs / 8, G8 = a.GCs / 8;
  const int U = E8 * G8 + G8, VS = 256 / U;   // units: (slot octet, channel octet) pairs + bias octets
  const int sub = tid / U, u = tid - sub * U;
  const bool active = sub < VS;
  const bool isb = u >= E8 * G8;
  const int e8 = isb ? 0 : u / G8, o8 = isb ? u - E8 * G8 : u % G8;
  float acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
  const long v0 = (long)blockIdx.x * a.per_block;
  const long v1 = v0 + a.per_block < a.nvox ? v0 + a.per_block : a.nvox;
  uint4 *la = pw_lds;                      // [kPwNV][E8]
  uint4 *lg = pw_lds + kPwNV * E8;         // [kPwNV][G8]
  const int nA = kPwNV * E8, nAll = kPwNV * (E8 + G8);
  uint4 rr[kPwLoads];
  auto load = [&](long c0) {
#pragma unroll
    for (int k = 0; k < kPwLoads; ++k) {
      const int i = tid + k * 256;
      uint4 w = make_uint4(0u, 0u, 0u, 0u);
      if (i < nAll) {
        const bool isA = i < nA;
        const int ii = isA ? i : i - nA, per = isA ? E8 : G8;
        const int v = ii / per, q = ii - v * per;
        if (c0 + v < v1)
          w = isA ? *reinterpret_cast<const uint4 *>(a.A + (c0 + v) * a.ACs + q * 8)
                  : *reinterpret_cast<const uint4 *>(a.G + (c0 + v) * a.GCs + q * 8);
      }
      rr[k] = w;
    }
  };
  if (v0 < v1) load(v0);
  for (long c0 = v0; c0 < v1; c0 += kPwNV) {
    __syncthreads();   // the previous chunk is consumed
#pragma unroll
    for (int k = 0; k < kPwLoads; ++k) {
      const int i = tid + k * 256;
      if (i < nAll) pw_lds[i] = rr[k];
    }
    __syncthreads();
    if (c0 + kPwNV < v1) load(c0 + kPwNV);   // lands while this chunk is summed
    const int nv = v1 - c0 < kPwNV ? (int)(v1 - c0) : kPwNV;
    if (active) {
      for (int v = sub; v < nv; v += VS) {
        float g[8];
        unpack8(lg[v * G8 + o8], g);
        if (!isb) {
          float x[8];
          unpack8(la[v * E8 + e8], x);
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(x[i], g[j], acc[i][j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[0][j] += g[j];
        }
      }
    }
  }
  // the voxel subsets' sums in a fixed order, in two halves of 32
  // accumulators (the reduction area [VS][U][32] fits the LDS of a block)
  float *red = reinterpret_cast<float *>(pw_lds);
  float *slab = a.partial + (size_t)blockIdx.x * a.Mtot * a.Ntot;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
    if (active)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) red[((size_t)sub * U + u) * 32 + i * 8 + j] = acc[4 * h + i][j];
    __syncthreads();
    for (int w = tid; w < U * 32; w += 256) {
      const int uu = w >> 5, q = w & 31, i = 4 * h + (q >> 3), j = q & 7;
      float sum = 0.f;
      for (int ss = 0; ss < VS; ++ss) sum += red[((size_t)ss * U + uu) * 32 + q];
      if (uu < E8 * G8) {
        const int e = (uu / G8) * 8 + i, o = (uu % G8) * 8 + j;
        if (e < a.ACR && o < a.GCR) slab[(size_t)e * a.Ntot + o] = sum;
      } else if (i == 0 && a.bias_row) {
        const int o = (uu - E8 * G8) * 8 + j;
        if (o < a.GCR) slab[(size_t)a.ACR * a.Ntot + o] = sum;
      }
    }
  }
}

}  // namespace

bool pw_supported(int ICs, int OCs, int Cout, bool dgrad) {
  // forward: K = ICs input slots (<= 128), N = OCs (<= 32, Cout <= OCs);
  // dgrad: K = the gradient's OCs (<= 32), N = ICs output slots (<= 96)
  if (ICs % 8 || OCs % 8 || Cout > OCs) return false;
  return dgrad ? (OCs <= 32 && ICs <= 96) : (ICs <= 128 && OCs <= 32);
}

bool pw_wgrad_supported(int ACs, int GCs) {
  if (ACs % 8 || GCs % 8 || ACs > 128 || GCs > 32) return false;
  const int U = (ACs / 8) * (GCs / 8) + GCs / 8;
  return U <= 256 && kPwNV * (ACs / 8 + GCs / 8) <= kPwLoads * 256;
}

int pw_wgrad_blocks(long nvox) {
  // one resident round: 136 VGPRs leave 3 waves per SIMD = 3 blocks per CU
  // (1024 blocks ran a second round of 256: 62 vs ~31 us), >= 4 chunks a block
  const long b = (nvox + 4 * kPwNV - 1) / (4 * kPwNV);
  return (int)std::max(1L, std::min(b, 768L));
}

int launch_pw_wgrad(const PwWgArgs &a, int blocks, hipStream_t s) {
  if (!pw_wgrad_supported(a.ACs, a.GCs)) return fail(4, "pwconv: unsupported weight-gradient channels");
  const int E8 = a.ACs / 8, G8 = a.GCs / 8;
  const int U = E8 * G8 + G8, VS = 256 / U;
  const size_t lds = std::max((size_t)kPwNV * (E8 + G8) * 16, (size_t)VS * U * 32 * 4);
  const double fl = 2.0 * a.nvox * (double)a.ACR * a.GCR;
  const double by = 2.0 * a.nvox * (double)(a.ACs + a.GCs);
  HCU_TIMED(s, "pw_wgrad_kernel", fl, by,
            HCU_LAUNCH(pw_wgrad_kernel, dim3(blocks), dim3(256), lds, s, a));
  HCU_CHECK_LAUNCH();
  return 0;
}

int launch_pw(const PwArgs &a, hipStream_t s) {
  // the kernel's input view: fwd reads in[nvox][ICs] and writes [nvox][OCs];
  // dgrad reads dy[nvox][OCs_fwd] (a.ICs = that stride) and writes [nvox][a.OCs]
  if ((double)a.nvox * std::max(a.ICs, a.OCs) * 2 >= 2147483000.0 - 64.0)
    return fail(4, "pwconv: tensor must stay below 2 GiB");
  const int KS = (a.ICs + 31) / 32, NS = (a.OCs + 15) / 16;
  const long ngroups = (a.nvox + 15) / 16;
  constexpr int G = 4;
  const long want = (ngroups + 4L * G - 1) / (4L * G);
  const int grid = (int)std::max(1L, std::min(want, 256L * 8));
  const double fl = 2.0 * a.nvox * (double)a.Cin * a.Cout;
  const double by = 2.0 * a.nvox * (double)(a.ICs + a.OCs);
  bool ok = false;
#define PW(KS_, NS_)                                                                              \
  if (!ok && KS == KS_ && NS == NS_) {                                                            \
    HCU_TIMED(s, "pw_kernel<" #KS_ "," #NS_ ">", fl, by,                                          \
              HCU_LAUNCH((pw_kernel<KS_, NS_, G>), dim3(grid), dim3(256), 0, s, a));              \
    ok = true;                                                                                    \
  }
  PW(1, 1) PW(2, 1) PW(3, 1) PW(4, 1) PW(1, 2) PW(2, 2) PW(3, 2) PW(4, 2)
  PW(1, 3) PW(1, 4) PW(1, 5) PW(1, 6)
#undef PW
  if (!ok) return fail(4, "pwconv: unsupported channel counts");
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu
