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
#include "hcunet.h"
#include "common.h"
#include "timing.h"
#include <algorithm>
#include <string>

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
// PM: 0 one tensor on each side; 1 the forward's input is channel parts
// (loads); 2 the input gradient's output is channel parts (stores).
template <int KS, int NS, int G, int PM>
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
  // parts form (a.nparts > 0): the slot-strided side is the forward's input
  // (pin: loads) or the input gradient's output (pout: stores).  pin: this
  // lane's slot c of K step ks lives in part c / pcs at offset c % pcs of its
  // [nvox][pcs] rows.  (The dgrad's input is the one dy tensor.)
  constexpr bool pin = PM == 1, pout = PM == 2;
  const uint16_t *pbase[KS];
  int poff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int c = ks * 32 + 8 * kq;
    const int pi = pin ? c / a.pcs : 0;
    const uint16_t *b0 = a.inp[0];
    if constexpr (pin) {
#pragma unroll
      for (int q = 1; q < kPwMaxParts; ++q)
        if (pi == q) b0 = a.inp[q];
    }
    pbase[ks] = b0;
    poff[ks] = pin ? c - pi * a.pcs : 0;
  }
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
        if constexpr (pin) {
          // (the address stays inside part 0's first row when !ok; the value is zeroed)
          const uint16_t *ptr = ok ? pbase[ks] + v * a.pcs + poff[ks] : a.inp[0];
          const uint4 w = *reinterpret_cast<const uint4 *>(ptr);
          b[gi][ks] = __builtin_bit_cast(shortx8, ok ? w : make_uint4(0u, 0u, 0u, 0u));
          continue;
        }
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
        if constexpr (pout) {   // slot c0 of part c0 / pcs
          const int pi = c0 / a.pcs;
          uint16_t *o = a.outp[0];
#pragma unroll
          for (int q = 1; q < kPwMaxParts; ++q)
            if (pi == q) o = a.outp[q];
          *reinterpret_cast<uint2 *>(o + v * a.pcs + (c0 - pi * a.pcs)) = w;
          continue;
        }
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
constexpr int kPwNV = 64;        // voxels per chunk (128 chunks at 184 VGPRs, 2 blocks per CU: slower)
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
        if (c0 + v < v1) {
          if (isA && a.nparts > 0) {   // slot q*8 of part q*8 / pcs
            const int pi = q * 8 / a.pcs;
            const uint16_t *pa = a.Ap[0];
#pragma unroll
            for (int t = 1; t < kPwMaxParts; ++t)
              if (pi == t) pa = a.Ap[t];
            w = *reinterpret_cast<const uint4 *>(pa + (c0 + v) * a.pcs + (q * 8 - pi * a.pcs));
          } else {
            w = isA ? *reinterpret_cast<const uint4 *>(a.A + (c0 + v) * a.ACs + q * 8)
                    : *reinterpret_cast<const uint4 *>(a.G + (c0 + v) * a.GCs + q * 8);
          }
        }
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
  // (1024 blocks ran a second round of 256: 62 vs ~31 us), >= 4 chunks a
  // block.  HCU_PW_WG_BLOCKS: the cap (A/B)
  static const long cap = [] {
    const char *e = getenv("HCU_PW_WG_BLOCKS");
    return e && atoi(e) > 0 ? (long)atoi(e) : 768L;
  }();
  const long b = (nvox + 4 * kPwNV - 1) / (4 * kPwNV);
  return (int)std::max(1L, std::min(b, cap));
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
  const int PM = a.nparts > 0 ? (a.dgrad ? 2 : 1) : 0;
#define PW(KS_, NS_, PM_)                                                                         \
  if (!ok && KS == KS_ && NS == NS_ && PM == PM_) {                                               \
    HCU_TIMED(s, PM_ ? "pw_kernel<" #KS_ "," #NS_ ",parts>" : "pw_kernel<" #KS_ "," #NS_ ">", fl, by, \
              HCU_LAUNCH((pw_kernel<KS_, NS_, G, PM_>), dim3(grid), dim3(256), 0, s, a));         \
    ok = true;                                                                                    \
  }
  PW(1, 1, 0) PW(2, 1, 0) PW(3, 1, 0) PW(4, 1, 0) PW(1, 2, 0) PW(2, 2, 0) PW(3, 2, 0) PW(4, 2, 0)
  PW(1, 3, 0) PW(1, 4, 0) PW(1, 5, 0) PW(1, 6, 0)
  // the channel-parts forms (hcu_pw_conv_*): forward K <= 96 slots into <= 16
  // channels, input gradient <= 16 channels into <= 96 slots
  PW(1, 1, 1) PW(2, 1, 1) PW(3, 1, 1) PW(1, 2, 1) PW(2, 2, 1) PW(3, 2, 1) PW(1, 1, 2) PW(1, 2, 2) PW(1, 3, 2) PW(1, 4, 2) PW(1, 5, 2)
  PW(1, 6, 2)
#undef PW
  if (!ok) return fail(4, "pwconv: unsupported channel counts");
  HCU_CHECK_LAUNCH();
  return 0;
}

}  // namespace hcu

// ---------------------------------------------------------------------------
// C-ABI (include/hcunet.h): the cat + 1x1x1 convolution of RDCNet's
// recurrence on the separate channel parts (no cat, no split).
namespace {
int pw_check(const void *const *parts, int nparts, int part_c, int part_cs, int64_t nvox, int Cout,
             int out_cs, const char *who) {
  if (!parts || nparts < 1 || nparts > hcu::kPwMaxParts || part_c < 1 || part_cs % 8 || part_c > part_cs ||
      Cout < 1 || out_cs % 8 || Cout > out_cs || nvox < 0)
    return hcu::fail(1, std::string(who) + ": 1..8 parts of part_cs (a multiple of 8) slots, Cout <= out_cs");
  for (int i = 0; i < nparts && nvox > 0; ++i)   // (empty tensors may have null data)
    if (!parts[i] || reinterpret_cast<uintptr_t>(parts[i]) % 16)
      return hcu::fail(1, std::string(who) + ": parts must be non-null and 16-byte aligned");
  if (!hcu::pw_supported(nparts * part_cs, out_cs, Cout, false) ||
      !hcu::pw_supported(nparts * part_cs, out_cs, Cout, true) ||
      !hcu::pw_wgrad_supported(nparts * part_cs, out_cs))
    return hcu::fail(4, std::string(who) + ": unsupported channel counts");
  return 0;
}
}  // namespace

extern "C" int hcu_pw_conv_forward(const void *const *parts, int nparts, int part_c, int part_cs, const float *w,
                                   const float *b, void *out, int64_t nvox, int Cout, int out_cs, void *stream) {
  if (int e = pw_check(parts, nparts, part_c, part_cs, nvox, Cout, out_cs, "hcu_pw_conv_forward")) return e;
  if (nvox == 0) return 0;
  if (!w || !out) return hcu::fail(1, "hcu_pw_conv_forward: null weight or output");
  hcu::PwArgs a{};
  a.in = static_cast<const uint16_t *>(parts[0]);
  a.w = w;
  a.bias = b;
  a.out = static_cast<uint16_t *>(out);
  a.nvox = nvox;
  a.ICs = nparts * part_cs;
  a.OCs = out_cs;
  a.Cin = nparts * part_c;
  a.Cout = Cout;
  a.part_c = part_c;
  a.part_cs = part_cs;
  a.nparts = nparts;
  a.pcs = part_cs;
  for (int i = 0; i < nparts; ++i) a.inp[i] = static_cast<const uint16_t *>(parts[i]);
  return hcu::launch_pw(a, (hipStream_t)stream);
}

extern "C" size_t hcu_pw_conv_work_floats(int64_t nvox, int nparts, int part_cs, int Cout) {
  return (size_t)hcu::pw_wgrad_blocks(nvox) * ((size_t)nparts * part_cs + 1) * Cout;
}

extern "C" int hcu_pw_conv_backward(const void *const *parts, int nparts, int part_c, int part_cs, const float *w,
                                    const void *dout, int Cout, int out_cs, void *const *dparts, float *dw,
                                    float *db, int64_t nvox, float *work, size_t work_floats, int accumulate,
                                    void *stream) {
  if (int e = pw_check(parts, nparts, part_c, part_cs, nvox, Cout, out_cs, "hcu_pw_conv_backward")) return e;
  if (!w || !dw) return hcu::fail(1, "hcu_pw_conv_backward: null weight or weight gradient");
  if (nvox == 0) {   // no voxels: zero gradients (accumulate: nothing to add)
    if (!accumulate) {
      HCU_HIP(hipMemsetAsync(dw, 0, sizeof(float) * (size_t)Cout * nparts * part_c, (hipStream_t)stream));
      if (db) HCU_HIP(hipMemsetAsync(db, 0, sizeof(float) * (size_t)Cout, (hipStream_t)stream));
    }
    return 0;
  }
  if (!dout || !work) return hcu::fail(1, "hcu_pw_conv_backward: null gradient or workspace");
  if (work_floats < hcu_pw_conv_work_floats(nvox, nparts, part_cs, Cout))
    return hcu::fail(1, "hcu_pw_conv_backward: workspace too small (hcu_pw_conv_work_floats)");
  hipStream_t s = (hipStream_t)stream;
  const int ACs = nparts * part_cs, Cin = nparts * part_c;
  if (dparts) {   // input gradients, straight into the parts' layout
    hcu::PwArgs a{};
    a.in = static_cast<const uint16_t *>(dout);
    a.w = w;
    a.nvox = nvox;
    a.ICs = out_cs;
    a.OCs = ACs;
    a.Cin = Cin;
    a.Cout = Cout;
    a.part_c = part_c;
    a.part_cs = part_cs;
    a.dgrad = 1;
    a.nparts = nparts;
    a.pcs = part_cs;
    for (int i = 0; i < nparts; ++i) {
      if (!dparts[i] || reinterpret_cast<uintptr_t>(dparts[i]) % 16)
        return hcu::fail(1, "hcu_pw_conv_backward: input gradients must be non-null and 16-byte aligned");
      a.outp[i] = static_cast<uint16_t *>(dparts[i]);
    }
    a.out = a.outp[0];
    if (nvox > 0)
      if (int e = hcu::launch_pw(a, s)) return e;
  }
  // weight / bias gradient: slabs (one per block) + the fixed-order finalize
  const int KB = hcu::pw_wgrad_blocks(nvox);
  hcu::PwWgArgs g{};
  g.G = static_cast<const uint16_t *>(dout);
  g.A = static_cast<const uint16_t *>(parts[0]);
  g.partial = work;
  g.nvox = nvox;
  g.per_block = (nvox + KB - 1) / KB;
  g.ACs = ACs;
  g.GCs = out_cs;
  g.ACR = ACs;   // (slots: the finalize maps torch channels to them)
  g.GCR = Cout;
  g.Mtot = ACs + 1;
  g.Ntot = Cout;
  g.bias_row = 1;
  g.nparts = nparts;
  g.pcs = part_cs;
  for (int i = 0; i < nparts; ++i) g.Ap[i] = static_cast<const uint16_t *>(parts[i]);
  if (int e = hcu::launch_pw_wgrad(g, KB, s)) return e;
  hcu::WGradFinalize f{};
  f.partial = work;
  f.dw = dw;
  f.db = db;
  f.KB = KB;
  f.Mtot = g.Mtot;
  f.Ntot = g.Ntot;
  f.T = 1;
  f.mode = 0;
  f.Cout = Cout;
  f.Cin_g = Cin;
  f.groups = 1;
  f.fold_mod = Cin;
  f.part_c = part_c;
  f.part_cs = part_cs;
  f.ACs = ACs;
  f.accumulate = accumulate;
  return hcu::launch_wgrad_finalize(f, s);
}
