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

}  // namespace

bool pw_supported(int ICs, int OCs, int Cout, bool dgrad) {
  // forward: K = ICs input slots (<= 128), N = OCs (<= 32, Cout <= OCs);
  // dgrad: K = the gradient's OCs (<= 32), N = ICs output slots (<= 96)
  if (ICs % 8 || OCs % 8 || Cout > OCs) return false;
  return dgrad ? (OCs <= 32 && ICs <= 96) : (ICs <= 128 && OCs <= 32);
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
