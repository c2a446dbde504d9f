// Internal declarations shared by the HIP kernels and the C++ executor.
// All activation tensors are channels-last fp32: [B][X][Y][Z][Cs], Cs = round_up(C, 4).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstddef>
#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <string>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));   // 8 bf16: one MFMA A/B fragment
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

namespace hcu {

// ---------------------------------------------------------------------------
// Every kernel launch of the library goes through HCU_LAUNCH.  While a
// chain record is armed (the backward, Ctx in unet.cpp), each kernel launched
// on the chain stream carries the chain event as its stop event, so the
// weight-gradient branch can wait on the chain's last kernel directly: no
// marker packet on the chain (measured on MI355X with HCU_FORK_DUP: each
// marker between two chain kernels costs ~3 us of GPU time).
struct ChainRec {
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  unsigned long n = 0;   // chain kernels launched while armed
};
inline ChainRec &chain_rec() {
  static thread_local ChainRec r;
  return r;
}
// Host-side cost accounting (HCU_HOST_PROF=1, diagnostics only; timing.cpp
// prints the per-call averages at exit): 0 kernel launches, 1 other HIP calls
// through HCU_HIP, 2/3 whole hcu_unet_forward / hcu_unet_backward calls.
bool host_prof_on();
double host_now_us();
void host_prof_add(int k, double us);
void host_prof_snap(double snap_us[2], long snap_n[2]);
void host_prof_call(int f, const double snap_us[2], const long snap_n[2], double total_us);
template <typename F, typename... Args>
inline void launch_ggl(F kernel, const dim3 &grid, const dim3 &block, uint32_t shmem, hipStream_t st,
                       Args... args) {
  const bool hp = host_prof_on();
  const double t0 = hp ? host_now_us() : 0.0;
  ChainRec &r = chain_rec();
  if (r.ev && st == r.s) {
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, nullptr, r.ev, 0, args...);
    ++r.n;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shmem, st, args...);
  }
  if (hp) host_prof_add(0, host_now_us() - t0);
}
#define HCU_LAUNCH(...) ::hcu::launch_ggl(__VA_ARGS__)

// ---------------------------------------------------------------------------
// bf16 storage helpers (the bf16 path keeps activations/gradients/weights in
// bf16 and does all arithmetic in fp32; conversions round to nearest even via
// v_cvt_pk_bf16_f32, which keeps NaNs NaN).
__device__ __forceinline__ float bf2f(uint32_t h16) { return __uint_as_float(h16 << 16); }
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  const floatx2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));   // v_cvt_pk_bf16_f32
}
// relu(x * s + h) of a packed bf16 pair: fp32 fma (v_pk_fma_f32), rounded to
// bf16, then the ReLU on the rounded pair with v_pk_max_i16 (a bf16 is
// negative exactly when its int16 image is; -0 becomes +0)
__device__ __forceinline__ uint32_t bn_relu_bf2(uint32_t w, floatx2 s, floatx2 h) {
  floatx2 f = {__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
  f = f * s + h;
  const shortx2 z = {0, 0};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(
                                          __builtin_bit_cast(shortx2, pack_bf2(f.x, f.y)), z));
}
__device__ __forceinline__ uint16_t f2bf(float a) {
  return __builtin_bit_cast(unsigned short, (__bf16)a);
}
// 8 bf16 (one uint4) <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4 &v, float (&f)[8]) {
  f[0] = bf_lo(v.x); f[1] = bf_hi(v.x); f[2] = bf_lo(v.y); f[3] = bf_hi(v.y);
  f[4] = bf_lo(v.z); f[5] = bf_hi(v.z); f[6] = bf_lo(v.w); f[7] = bf_hi(v.w);
}
__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]),
                    pack_bf2(f[6], f[7]));
}

inline int round_up(int a, int b) { return (a + b - 1) / b * b; }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// CUs' worth of resident workgroups the generic weight-gradient launch (the
// backward's branch stream) is sized for (wgrad3 / wgrad2 / wgrad8 fix their
// own: 192 / 192 / 256, measured per family): 256 fills the chip; fewer leave
// slots for the chain stream's kernels to start while the branch runs and
// write fewer slabs (HCU_SIDE_CUS, A/B).  Config 2, interleaved A/B (2 runs
// each): 256 -> 2.164 ms/step, 240 -> 2.226, 224 -> 2.150, 192 -> 2.267,
// 128 -> 2.217 (the grid sizes move the layers' tile partitions).
inline int side_cus() {
  static const int v = [] {
    const char *e = getenv("HCU_SIDE_CUS");
    const int n = e ? atoi(e) : 224;
    return n < 16 ? 16 : (n > 256 ? 256 : n);
  }();
  return v;
}
inline size_t align_up(size_t a, size_t b) { return (a + b - 1) / b * b; }

// Division by a runtime-constant divisor without the ~40-instruction integer
// divide: q = (umulhi(n, m) + n) >> s, exact for 0 <= n < 2^31, d >= 1.
struct FastDiv {
  uint32_t d = 1, m = 0, s = 0;
  FastDiv() = default;
  explicit FastDiv(uint32_t div) : d(div) {
    s = 0;
    while ((1ull << s) < div) ++s;
    m = (uint32_t)((((1ull << s) - div) << 32) / div + 1);
  }
  __host__ __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (uint32_t)((((uint64_t)n * m >> 32) + n) >> s);  // v_mul_hi_u32 on device
  }
  // the same divisor with its fields read through kuni (see below)
  __device__ __forceinline__ FastDiv uni() const;
  // q = n / d, r = n % d
  __host__ __device__ __forceinline__ void divmod(uint32_t n, int &q, int &r) const {
    const uint32_t qq = div(n);
    q = (int)qq;
    r = (int)(n - qq * d);
  }
};

// Uniform value re-materialised into SGPRs from an LDS copy of the launch
// arguments.  Kernels with many launch constants read them this way inside
// their tile loops: LDS loads are not hoisted across the loop's barriers, so
// the constants are live only where used instead of occupying (and spilling)
// scalar registers for the whole kernel.
template <class T>
__device__ __forceinline__ T kuni(const T &v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "kuni: 4- or 8-byte values");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
  } else {
    int2 p = __builtin_bit_cast(int2, v);
    p.x = __builtin_amdgcn_readfirstlane(p.x);
    p.y = __builtin_amdgcn_readfirstlane(p.y);
    return __builtin_bit_cast(T, p);
  }
}

__device__ __forceinline__ FastDiv FastDiv::uni() const {
  FastDiv f;
  f.d = kuni(d);
  f.m = kuni(m);
  f.s = kuni(s);
  return f;
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a fence on all
// address spaces: it waits for every outstanding global load AND store
// (vmcnt(0)) before the barrier, which drains the previous tile's output
// stores and the next tile's prefetch at every barrier of a persistent loop.
// Kernels whose barriers only publish LDS data use this instead.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Thread-local error message (hcu_last_error()).
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define HCU_HIP(expr)                                                            \
  do {                                                                           \
    const bool hp__ = ::hcu::host_prof_on();                                     \
    const double t__ = hp__ ? ::hcu::host_now_us() : 0.0;                        \
    hipError_t e__ = (expr);                                                     \
    if (hp__) ::hcu::host_prof_add(1, ::hcu::host_now_us() - t__);               \
    if (e__ != hipSuccess)                                                       \
      return ::hcu::fail(3, std::string(#expr) + ": " + hipGetErrorString(e__)); \
  } while (0)

#define HCU_CHECK_LAUNCH() HCU_HIP(hipGetLastError())

// ---------------------------------------------------------------------------
// Generic gather convolution (implicit GEMM on v_mfma_f32_16x16x4_f32):
//   out[b, o*os + of, co] = sum_{t, ci} act(in[b, o*s + t*d - p, ci]) * w[t][ci][co] (+ bias)
// act = identity or relu(x*scale[ci] + shift[ci]) (BatchNorm+ReLU of the
// producer fused on load); positions outside the input read as 0 (post-act).
// Covers Conv3d forward (s=1, p=0), Conv3d dgrad (full correlation with flipped
// taps), ConvTranspose3d dgrad (strided) and ConvTranspose3d forward (one
// launch per output phase).  Optional per-block BatchNorm partial statistics.
// ---------------------------------------------------------------------------
struct BNCoef {
  float *scale, *shift, *mean, *invstd, *c1, *c0;  // [Cs] each
};
struct GConvArgs {
  const float *in;
  const float *in_scale, *in_shift;   // [ICs] or null
  const float *w;                     // [T][ICs][CoutW]
  const float *bias;                  // [Cout] or null
  float *out;
  float *stats;                       // [B*ntiles][CoutW][2] or null
  int B, IX, IY, IZ, ICs;
  int OX, OY, OZ;                     // computed output grid
  int SX, SY, SZ, OCs, Cout, CoutW;   // stored tensor
  int osx, osy, osz, ofx, ofy, ofz;   // store mapping
  int KX, KY, KZ;
  int sx, sy, sz, dx, dy, dz, px, py, pz;
  // tiling (filled by plan_gconv)
  int TX, TY, TZ, ntx, nty, ntz;
  int HX, HY, HZ, P;
  // bconv halo image in LDS: row strides of the x / y / z halo axes and the
  // row count they span (plan-chosen axis order and padding; default
  // HY*HZ, HZ, 1 and HX*HY*HZ)
  int hsx, hsy, hsz, hvp;
  int CK, NSUB, MPW;
  int lds_bytes;
  FastDiv fHZ, fHY, fTZ, fTY;         // halo / tile index decomposition
  // conv2 (conv2.hip): output-channel phases folded into N (ConvTranspose3d
  // with kernel % stride == 0: n = phase*Cout + co, phase = (qx*phy+qy)*phz+qz
  // stored at o*os + of + q), and the K split over channel chunks.
  int nph, phx, phy, phz;
  int ksplit, cps;                    // K-split count, channel chunks per split
  size_t slice_floats;                // floats of one stored-tensor slice
  float *partial;                     // [ksplit][stored tensor] when ksplit > 1
  int use_conv2;
  int NPF, gridx;                     // conv2 halo prefetch depth, persistent grid size
  int epi_lds, nc4, areg;             // conv2 epilogue through LDS (float4 stores), float4
                                      // groups, floats of the halo / C-tile LDS region
  FastDiv fNT, fNTZ, fNTY;            // tile index decomposition
  // conv8 (conv8.hip): <= 8 output channels on the 16-block 4x4x1 MFMA
  int use_conv8, G8, HVP;             // enabled, 32-voxel groups per wave, halo plane stride
  FastDiv fKZ, fKY;                   // tap index decomposition (conv8 K loop)
  int dbg;                            // ablation bits (HCU_CONV8_DBG; 0 in production)
  int HZr, MZ;                        // conv8: loaded halo z extent, z stride of the M rows
  // The network input read in the caller's NCXYZ layout by the first layer's
  // halo staging (no separate channels-last pass): in_fmt 1 / 2 / 3 = `in` is
  // [B][in_c][IX][IY][IZ] fp32 / fp16 / bf16 (in_c <= 4 real channels, the
  // rest of the ICs channels read 0); xcl != null: the staging also stores the
  // channels-last copy [B][IX][IY][IZ][ICs] the weight gradient reads, each
  // input voxel by exactly one tile; `w` is then the PyTorch-layout weight
  // [Cout][in_c][KX*KY*KZ] (groups 1).  in_fmt 0: `in` is channels-last.
  int in_fmt, in_c;
  float *xcl;
  // dgrad epilogue fused with the BatchNorm+ReLU backward reduction of the
  // layer whose output this gradient is for (bn_y = its pre-BN y, same layout
  // as out): the stored value is dz = v * [y*scale+shift > 0] and the stats
  // rows hold (sum dz, sum dz * (y-mean)*invstd) per channel.
  const float *bn_y, *bn_scale, *bn_shift, *bn_mean, *bn_invstd;
  double flops;                       // algorithmic FLOPs (0: derive)
  // bconv (bconv.hip): the bf16 path.  in / out / bn_y / w point to bf16 data
  // (channels-last activations, packed weights); partial stays fp32.
  int use_bconv;
  int bes;   // bconv element bytes: 2 (bf16 activations) or 4 (fp32); 0 = 2
  // bconv with ConvTranspose3d phases folded into N: columns per phase (0 =
  // Cout).  Cout not a multiple of the 4 (fp32) / 8 (bf16) columns a lane's
  // store and a packed weight vector span: cph = Cout rounded up, the padded
  // columns have zero weights and zero bias (RDCNet's 5-channel output).
  int cph;
};

// Forward BatchNorm statistics rows (stats, [rows][CoutW] of float4): per
// (row, channel) {S1, S2, K, n} = sums of (y - K) and (y - K)^2 over the n
// outputs the row's workgroup produced, K a pivot value taken from those
// outputs.  bn_fwd_finalize combines the rows in fp64 (parallel-variance
// identity), so the variance never comes from E[y^2] - E[y]^2 of raw fp32 sums.
// The fused BatchNorm-backward epilogue (bn_y set) writes plain [rows][CoutW][2]
// sums (sum dz, sum dz * xhat) into the same buffer.
// Chooses the tile and kernel variant; returns 0 or an error code.
int plan_gconv(GConvArgs &a, int target_blocks);
int launch_gconv(const GConvArgs &a, hipStream_t s);
int plan_conv2(GConvArgs &a, int target_blocks);
int launch_conv2(const GConvArgs &a, hipStream_t s);
size_t conv2_partial_floats(const GConvArgs &a);
int conv2_stat_rows(const GConvArgs &a);
int plan_conv8(GConvArgs &a, int target_blocks);
int launch_conv8(const GConvArgs &a, hipStream_t s);
// Plans conv2 when it supports the shape, else the generic gconv.
bool conv2_disabled();   // HCU_NO_CONV2=1 forces the generic kernel (A/B testing)
inline int plan_conv_any(GConvArgs &a, int target_blocks) {
  GConvArgs b8 = a;
  if (plan_conv8(b8, target_blocks) == 0) {
    a = b8;
    return 0;
  }
  GConvArgs b = a;
  b.use_conv8 = 0;
  if (!conv2_disabled() && plan_conv2(b, target_blocks) == 0) {
    a = b;
    return 0;
  }
  a.use_conv2 = 0;
  a.use_conv8 = 0;
  return plan_gconv(a, target_blocks);
}
int plan_bconv(GConvArgs &a, int target_blocks);
// fp32 convolution: the blocked MFMA kernel (bconv, fp32 elements) when it
// supports the shape, else conv8 / conv2 / the generic gconv.
// HCU_NO_BCONV_F32=1 restores the older fp32 kernels (A/B testing).
inline int plan_conv_fp32(GConvArgs &a, int target_blocks) {
  static const bool off = getenv("HCU_NO_BCONV_F32") != nullptr;
  // fewer than 16 output columns: conv8's 4x4 MFMA blocks waste no MFMA rows
  if (!off && a.Cout * std::max(1, a.nph) >= 16) {
    GConvArgs b = a;
    b.bes = 4;
    if (plan_bconv(b, target_blocks) == 0) {
      a = b;
      return 0;
    }
  }
  a.cph = 0;   // (bconv only)
  return plan_conv_any(a, target_blocks);
}
int launch_bconv(const GConvArgs &a, hipStream_t s);
void bconv_tuning(bool on);   // measured planning on/off for the plans built by this thread
int bconv_stat_rows(const GConvArgs &a);
inline int launch_conv_any(const GConvArgs &a, hipStream_t s) {
  if (a.use_bconv) return launch_bconv(a, s);
  if (a.use_conv8) return launch_conv8(a, s);
  return a.use_conv2 ? launch_conv2(a, s) : launch_gconv(a, s);
}
inline int gconv_rows(const GConvArgs &a) {
  if (a.use_bconv) return bconv_stat_rows(a);
  if (a.use_conv8) return a.gridx;
  return a.use_conv2 ? conv2_stat_rows(a) : a.B * a.ntx * a.nty * a.ntz;
}
// Whether the kernel planned in `a` supports the fused BatchNorm-backward epilogue.
inline bool conv_bnbwd_fusable(const GConvArgs &a) {
  return a.use_conv8 || a.use_conv2 || a.use_bconv;
}
inline size_t conv_partial_floats(const GConvArgs &a) {
  return ((a.use_conv2 || a.use_bconv) && !a.use_conv8) ? conv2_partial_floats(a) : 0;
}

// ---------------------------------------------------------------------------
// Weight gradient (implicit GEMM, split over the reduction grid):
//   partial[kb][row][col] = sum_{p in block kb} A[p*as + t*ad - ap][ci] * G[p*gs + t*gd - gp][co]
// taps_rows=1: row=(t,ci) col=co (Conv3d);  taps_rows=0: row=ci col=(t,co) (ConvTranspose3d).
// bias_row (taps_rows only): row T*ACs is a ones-row -> sum_p G[p][co].
// ---------------------------------------------------------------------------
struct WGradArgs {
  const float *A;
  const float *a_scale, *a_shift;
  const float *G;
  float *partial;                     // [KB][Mtot][Ntot]
  int B;
  int AX, AY, AZ, ACs;
  int GX, GY, GZ, GCs;
  int PX, PY, PZ;
  int KX, KY, KZ;
  int asx, asy, asz, adx, ady, adz, apx, apy, apz;
  int gsx, gsy, gsz, gdx, gdy, gdz, gpx, gpy, gpz;
  int taps_rows, bias_row;
  int Mtot, Ntot;
  // tiling (filled by plan_wgrad)
  int TX, TY, TZ, ntx, nty, ntz;
  int HAX, HAY, HAZ, PA, HGX, HGY, HGZ, PG;
  int CKA, CKG, mloc, nloc, MS, NS;
  int TA, TG;                         // taps per block (rows / cols mode)
  int nci, nco, ntc;                  // channel chunks and tap chunks
  int mchunks, nchunks, KB;
  int lds_bytes;
  FastDiv fHAZ, fHAY, fHGZ, fHGY, fTZ, fTY;
  // wgrad2 (Conv3d, stride-1 operands): z rows padded to multiples of 4 so a
  // lane reads 4 consecutive voxels with one ds_read_b128; one A image per kz.
  int v2, TZP, HAZP, PA2, PG2, gridx, occ;
  double flops;                       // algorithmic FLOPs (0: derive)
  // bwgrad (bwgrad.hip): the bf16 path (A, G bf16 channels-last); PA2 / PG2
  // are the LDS row strides of the A halo / G images, MSW the row subtiles per
  // wave, NSB the column subtiles of a block.
  int use_bw, MSW, NSB, PTV, HAV, HGV;
  int NPA, NPG;                       // bwgrad: 16-byte A / G staging loads per thread and tile
                                      // (register prefetch of the next tile); 0 = serial kernel
  // wgrad8 (wgrad8.hip, v2 == 2): A image z-row stride (PA2 / PG2: plane
  // strides), MFMA form (0: 16x16x4, 1: 4x4x1 16-block), voxel blocks per
  // instruction and z taps on the column side (form 1)
  int ARS, w8mode, w8nbv, w8nj, w8nh;
  int w8off[128];                     // wgrad8 row (form 0) / row-quad (form 1) A image offsets
  // ConvTranspose3d with kernel % stride == 0 as the weight gradient of its
  // phase-folded forward convolution (wgrad2, taps_rows): rows (j, ci) over
  // the J = K / S taps with A zero-padded by J - 1 (apx..), columns (phase q,
  // co) with q = (qx*phy + qy)*phz + qz, G read at o*S + q (gsx = S): the
  // stride phases are extra output columns and the bias row sums dU per
  // (q, co) -- no separate chansum.  nph <= 1: plain Conv3d form.
  int nph, phx, phy, phz, GCout;
  // bwgrad, taps_rows: real input / output channels (0: ACs / GCs).  The slab
  // rows are (tap, channel < ACr) and its columns channels < GCr, so the
  // padding slots of a channels-last stride (RDCNet: 10 channels in 16) are
  // neither written nor summed; wgrad_finalize then takes ACs = ACr.
  int ACr, GCr;
};
// 1x1x1 Conv3d forward / input gradient on bf16 channels-last tensors
// without BatchNorm (pwconv.hip): RDCNet's mixing convolutions.  Weights in
// the PyTorch layout [Cout][Cin]; part_c / part_cs: ConvLayer's channel parts.
//   dgrad 0: in [nvox][ICs] -> out [nvox][OCs] (+ bias)
//   dgrad 1: in = dy [nvox][ICs = the forward's OCs] -> out = dx [nvox][OCs = the forward's ICs]
//   nparts > 0: the slot-strided side (the forward's input, the dgrad's
//   output) is nparts separate tensors [nvox][pcs] instead of one [nvox][ICs
//   | OCs] (RDCNet's channel cats, never materialised: hcu_pw_conv_*)
constexpr int kPwMaxParts = 8;
struct PwArgs {
  const uint16_t *in;
  const float *w, *bias;
  uint16_t *out;
  long nvox;
  int ICs, OCs, Cin, Cout, part_c, part_cs, dgrad;
  int nparts, pcs;
  const uint16_t *inp[kPwMaxParts];
  uint16_t *outp[kPwMaxParts];
};
bool pw_supported(int ICs, int OCs, int Cout, bool dgrad);
int launch_pw(const PwArgs &a, hipStream_t s);
// Their weight / bias gradient (pwconv.hip): A = x [nvox][ACs], G = dy
// [nvox][GCs]; one slab per block in bwgrad's taps_rows layout (T = 1): rows
// e < ACR, the bias row ACR (bias_row), columns o < GCR, Mtot x Ntot floats.
struct PwWgArgs {
  const uint16_t *A, *G;
  float *partial;
  long nvox, per_block;
  int ACs, GCs, ACR, GCR, Mtot, Ntot, bias_row;
  int nparts, pcs;                      // nparts > 0: A is nparts tensors [nvox][pcs] (Ap)
  const uint16_t *Ap[kPwMaxParts];
};
bool pw_wgrad_supported(int ACs, int GCs);
int pw_wgrad_blocks(long nvox);
int launch_pw_wgrad(const PwWgArgs &a, int blocks, hipStream_t s);
// the row stride per tap of a weight-gradient slab (WGradFinalize::ACs)
inline int wgrad_slab_acs(const WGradArgs &w) { return w.use_bw && w.ACr > 0 ? w.ACr : w.ACs; }
int plan_bwgrad(WGradArgs &a, int target_blocks);
int launch_bwgrad(const WGradArgs &a, hipStream_t s);
int plan_wgrad(WGradArgs &a, int target_blocks);
int plan_wgrad8(WGradArgs &a);
int launch_wgrad8(const WGradArgs &a, hipStream_t s);
int launch_wgrad(const WGradArgs &a, hipStream_t s);
int plan_wgrad3(WGradArgs &a);                 // wgrad3.hip (v2 == 3)
int launch_wgrad3(const WGradArgs &a, hipStream_t s);
inline size_t wgrad_partial_floats(const WGradArgs &a) {
  return (size_t)a.KB * a.Mtot * a.Ntot;
}

// Sum wgrad partials over KB and scatter into PyTorch-layout gradients.
//  mode 0 (Conv3d): dw[o][c][t] for o<Cout, c<Cin_g; effective input channel
//         e = (g(o)*Cin_g + c) % fold_mod (fold_mod = channels of U when the
//         cat(U,U) fold is active, else a large number); db[o] from bias row.
//  mode 1 (ConvTranspose3d): dw[ci][co][t].
struct WGradFinalize {
  const float *partial;
  float *dw, *db;
  int KB, Mtot, Ntot, T;
  int mode;   // 0 Conv3d (taps rows), 1 ConvTranspose3d, 2 bias column sums (db[c < Cout]),
              // 4 the same from forward-statistics rows [KB][Ntot] of {S1, S2, K, n} (S1 + n*K),
              // 3 ConvTranspose3d in the phase form (WGradArgs::nph): row (j, ci), column
              // (q, co) -> dW[ci][co][t], t = (J-1-j)*S + q per dimension; db[co] = sum_q bias row
  int Cout, Cin_g, groups, fold_mod, ACs;   // conv
  int part_c, part_cs;   // conv input made of channel parts (0: none; prep_all.hip weff2)
  int Cin, CoutT, GCs;                      // convT
  int J[3], SS[3];                          // mode 3: taps per phase, stride
  int accumulate;
};
int launch_wgrad_finalize(const WGradFinalize &f, hipStream_t s);
constexpr int kWgfBatch = 24;   // finalize jobs per launch (kernel argument < 4 KB)
int launch_wgrad_finalize_batch(const WGradFinalize *fs, int n, hipStream_t s);

// ---------------------------------------------------------------------------
// Pointwise / reduction kernels (pointwise.hip)
// ---------------------------------------------------------------------------
// Per-layer BatchNorm coefficient block, each array padded to Cs with zeros.

int launch_bn_fwd_finalize(const float *stats, int R, int statsW, int C, int Cs,
                           double count, const float *gamma, const float *beta,
                           float *run_mean, float *run_var, int64_t *nbt,
                           float eps, float momentum, int training, BNCoef coef,
                           hipStream_t s);
// part rows [R][W][2]; W = row stride in channels (>= Cs).
int launch_bn_bwd_finalize(const float *part, int R, int C, int Cs, int W, double count,
                           BNCoef coef, float *dgamma, float *dbeta, int training,
                           int accumulate, hipStream_t s);

int launch_maxpool_fwd(const float *y, const float *scale, const float *shift,
                       float *p, int B, int X, int Y, int Z, int Cs,
                       int kx, int ky, int kz, hipStream_t s, int bf = 0);

// dz = dA * [relu'(z)] in place; partials [R][Cs][2] of (sum dz, sum dz*xhat).
int bwd_rows(int64_t nvox, int Cs);
int launch_bn_bwd_reduce_dense(float *dA, const float *y, BNCoef coef,
                               int64_t nvox, int Cs, float *part, int R,
                               hipStream_t s, int bf = 0);
// dz from a max-pool gradient dP (argmax recomputed from y); R = pool_bwd_rows(...).
int pool_bwd_rows(int B, int X, int Y, int Z, int Cs, int kx, int ky, int kz);
int launch_bn_bwd_reduce_pool(const float *dP, const float *y, BNCoef coef,
                              float *dz, int B, int X, int Y, int Z, int Cs,
                              int kx, int ky, int kz, float *part, int R,
                              hipStream_t s, int bf = 0);
// dy = dz*scale + c1*y + c0 in place.
int launch_bn_bwd_apply(float *dz, const float *y, BNCoef coef, int64_t nvox,
                        int Cs, hipStream_t s, int bf = 0);

// out_conv (1x1x1 Conv3d) forward: pred[b][o][v] (NCXYZ).
int launch_outconv_fwd(const float *y, BNCoef coef, const float *w,
                       const float *bias, float *pred, int B, int64_t V, int C,
                       int Cs, int Co, hipStream_t s, int bf = 0);
// out_conv backward fused with the last BatchNorm's backward reduction.
int outconv_bwd_rows(int64_t nvox, int Cs);
int launch_outconv_bwd(const float *dpred, const float *y, BNCoef coef,
                       const float *w, float *dz, int B, int64_t V, int C,
                       int Cs, int Co, float *part_bn, float *part_oc, int R,
                       hipStream_t s, int bf = 0);

// Channel sum of a channels-last tensor: partial [R][Cs].
int chansum_rows(int64_t nvox, int Cs);
int launch_chansum(const float *x, int64_t nvox, int Cs, float *part, int R,
                   hipStream_t s, int bf = 0);
// out[j] (=|+=) sum_r part[r*W + j] for j < n, mapped: out index = j (dense).
int launch_reduce_partials(const float *part, int R, int W, int n, float *out,
                           int accumulate, hipStream_t s);

// Layout: NCXYZ <-> channels-last (padded channels written as 0).
int launch_to_cl(const float *x, float *xcl, int B, int C, int Cs, int64_t V,
                 hipStream_t s, int bf = 0, int x_dtype = 0);
int launch_from_cl(const float *xcl, float *x, int B, int C, int Cs, int64_t V,
                   hipStream_t s, int bf = 0);

// Weight preparation (PyTorch layout -> GEMM layouts).
// Plain layout: wg[t][ci][co] (t < T, ci < ICs, co < CoutW).  Packed layout
// for conv2 (on != 0): wg[chunk][s][g][co][j] with chunk = ci / CK, K-step s,
// lane group g and component j as conv2_kernel consumes them (tap t =
// s*TPS + g/(CK/4), ci = chunk*CK + 4*(g % (CK/4)) + j, TPS = 16/CK); taps
// t >= T in the last step are zero.
// on == 2: the conv8 layout wg[t][ci/4][co (8)][ci%4] (CK = ICs/4, S = T).
struct WPack {
  int on, CK, S, ICs, CoutW;
};
inline WPack wpack_of(const GConvArgs &a) {
  WPack p{};
  if (a.use_bconv && a.bes == 4) {   // fp32 bconv: the conv2 image [chunk][s][g][co][4]
    const int T = a.KX * a.KY * a.KZ, TPS = 16 / a.CK;
    p.on = 1;
    p.CK = a.CK;
    p.S = (T + TPS - 1) / TPS;
    p.ICs = a.ICs;
    p.CoutW = a.CoutW;
    return p;
  }
  if (a.use_bconv) {   // bf16 image wg[chunk][s][g][co][8] (bconv.hip), 32 K per step
    const int T = a.KX * a.KY * a.KZ, TPS = 32 / a.CK;
    p.on = 3;
    p.CK = a.CK;
    p.S = (T + TPS - 1) / TPS;
    p.ICs = a.ICs;
    p.CoutW = a.CoutW;
    return p;
  }
  if (a.use_conv8) {
    p.on = 2;
    p.CK = a.ICs / 4;
    p.S = a.KX * a.KY * a.KZ;
    p.ICs = a.ICs;
    p.CoutW = 8;
    return p;
  }
  if (!a.use_conv2) return p;
  const int T = a.KX * a.KY * a.KZ, TPS = 16 / a.CK;
  p.on = 1;
  p.CK = a.CK;
  p.S = (T + TPS - 1) / TPS;
  p.ICs = a.ICs;
  p.CoutW = a.CoutW;
  return p;
}
// Floats of the prepared weight buffer of a GEMM planned in `a`.
// Elements of a prepared weight buffer (plain [T][ICs][CoutW] when !on).
__host__ __device__ inline int64_t wpack_count(const WPack &p, int T, int ICs, int CoutW) {
  if (p.on == 3) return (int64_t)p.ICs * p.S * (32 / p.CK) * p.CoutW;
  if (p.on == 2) return (int64_t)p.S * p.CK * 32;
  if (p.on) return (int64_t)p.ICs * p.S * (16 / p.CK) * p.CoutW;
  return (int64_t)T * ICs * CoutW;
}
inline size_t wprep_floats(const GConvArgs &a) {
  const int T = a.KX * a.KY * a.KZ;
  if (a.use_bconv && a.bes == 4) return (size_t)wpack_count(wpack_of(a), T, a.ICs, a.CoutW);
  if (a.use_bconv) return (size_t)(wpack_count(wpack_of(a), T, a.ICs, a.CoutW) + 1) / 2;
  if (a.use_conv8) return (size_t)T * a.ICs * 8;
  if (!a.use_conv2) return (size_t)T * a.ICs * a.CoutW;
  const WPack p = wpack_of(a);
  return (size_t)a.ICs * p.S * (16 / p.CK) * a.CoutW;
}
// Packed index -> (t, ci, co); false for a padded tap.  I = uint32_t where the
// caller knows the image has < 2^31 elements (64-bit division is a ~100
// instruction software sequence).
template <typename I>
__device__ __forceinline__ bool wpack_decode(const WPack &p, I i, int T, int &t, int &ci,
                                             int &co) {
  if (p.on == 3) {
    const int j = (int)(i & 7);
    I q = i >> 3;
    co = (int)(q % p.CoutW);
    q /= p.CoutW;
    const int g = (int)(q & 3);
    q >>= 2;
    const int s = (int)(q % p.S);
    const int chunk = (int)(q / p.S);
    const int C8 = p.CK / 8, TPS = 4 / C8;
    t = s * TPS + g / C8;
    ci = chunk * p.CK + (g % C8) * 8 + j;
    return t < T;
  }
  if (p.on == 2) {
    const int j = (int)(i & 3);
    co = (int)((i >> 2) & 7);
    const int q = (int)(i >> 5);
    ci = (q % p.CK) * 4 + j;
    t = q / p.CK;
    return t < T;
  }
  const int j = (int)(i & 3);
  I q = i >> 2;
  co = (int)(q % p.CoutW);
  q /= p.CoutW;
  const int g = (int)(q & 3);
  q >>= 2;
  const int s = (int)(q % p.S);
  const int chunk = (int)(q / p.S);
  const int C4 = p.CK / 4, TPS = 4 / C4;
  t = s * TPS + g / C4;
  ci = chunk * p.CK + (g % C4) * 4 + j;
  return t < T;
}
// Conv3d fwd:   wg[t][e][co] (e < ECs, co < CoutW)
// Conv3d dgrad: wg[t'][co][e] (co < OCs, e < EW), t' = T-1-t
int launch_prep_conv_fwd(const float *w, float *wg, int Cout, int Cin_g, int groups,
                         int fold_mod, int T, int ECs, int CoutW, WPack pk, hipStream_t s);
int launch_prep_conv_dgrad(const float *w, float *wg, int Cout, int Cin_g,
                           int groups, int fold_mod, int T, int OCs, int EW,
                           int E, WPack pk, hipStream_t s);
// ConvTranspose3d fwd phase (px,py,pz): wg[t][ci][co], t over (Jx,Jy,Jz) taps
int launch_prep_convt_fwd(const float *w, float *wg, int Cin, int Cout, int KX,
                          int KY, int KZ, int sx, int sy, int sz, int px, int py,
                          int pz, int Jx, int Jy, int Jz, int ICs, int CoutW,
                          hipStream_t s);
// ConvTranspose3d fwd, all phases folded into N (kernel % stride == 0):
// wg[t'][ci][ph*Cout + co], t' over (Jx,Jy,Jz) taps of the padded correlation.
int launch_prep_convt_fused(const float *w, float *wg, int Cin, int Cout, int KX, int KY,
                            int KZ, int sx, int sy, int sz, int ICs, int CoutW, WPack pk,
                            hipStream_t s);
// ConvTranspose3d dgrad: wg[t][co][ci] (co < UCs, ci < CinW)
int launch_prep_convt_dgrad(const float *w, float *wg, int Cin, int Cout, int T,
                            int UCs, int CinW, WPack pk, hipStream_t s);

// Batched weight preparation: every re-layout of one network step in a few
// launches (one workgroup row per job) instead of one launch per layer.
enum PrepKind { PREP_CONV_FWD = 0, PREP_CONV_DGRAD = 1, PREP_CONVT_FUSED = 2,
                PREP_CONVT_PHASE = 3, PREP_CONVT_DGRAD = 4 };
struct PrepJob {
  int kind;
  short bf16;       // != 0: the prepared image is written as bf16 (bconv)
  short pad_;
  int64_t n;        // elements of the prepared buffer
  int64_t src;      // float offset of the PyTorch-layout weight in the parameter buffer
  int64_t dst;      // float offset of the prepared buffer in the destination workspace
  WPack pk;
  // CONV_FWD / CONV_DGRAD: Cout, Cin_g, groups, fold_mod, T, rows (ECs|OCs), cols (CoutW|EW), E
  // CONVT_FUSED: Cin, Cout, KX, KY, KZ, sx, sy, sz, ICs, CoutW, columns per phase (0: Cout)
  // CONVT_PHASE: Cin, Cout, KX, KY, KZ, sx, sy, sz, px, py, pz, Jx, Jy, Jz, ICs, CoutW
  // CONVT_DGRAD: Cin, Cout, T, UCs, CinW
  int p[16];
};
constexpr int kPrepBatch = 32;   // jobs per launch: the batch is a kernel argument (< 4 KB)
int launch_prep_all(const float *params, float *dst_base, const PrepJob *jobs, int n, hipStream_t s);

// Layer-chain layout kernels (layout.hip): dilation sub-lattices (space to
// batch) and back, crop of a padded ConvTranspose3d output, NCXYZ output with
// the last BatchNorm+ReLU applied.  es = element bytes (4 fp32, 2 bf16).
int launch_s2b(const float *x, const float *sc, const float *sh, float *xs, int B, int X, int Y, int Z,
               int Cs, int es, const int *D, const int *S, hipStream_t s);
int launch_b2s(const float *ys, float *y, int B, int OX, int OY, int OZ, int Cs, int es, const int *D,
               const int *S, hipStream_t s);
int launch_crop_cl(const float *src, float *dst, int B, const int *sdims, const int *ddims, const int *off,
                   int Cs, int es, hipStream_t s);
int launch_from_cl_act(const float *y, const float *sc, const float *sh, float *out, int B, int C, int Cs,
                       int64_t V, hipStream_t s, int bf);
// LDS-tiled NCXYZ <-> channels-last (Cs <= 128; returns -1 otherwise)
int launch_from_cl_tiled(const float *y, const float *sc, const float *sh, float *out, int B, int C, int Cs,
                         int64_t V, hipStream_t s, int bf);
int launch_to_cl_tiled(const float *x, float *xcl, int B, int C, int Cs, int64_t V, hipStream_t s, int bf,
                       int x_dtype);

// Loss / optimizer (loss_adam.hip)
int launch_loss_pixel(const float *pred, int B, int C, int PX, int PY, int PZ,
                      const void *mask, int mask_dtype, const void *pwl,
                      int pwl_dtype, int MX, int MY, int MZ, float *loss,
                      float *dpred, float *part, int R, hipStream_t s);
int loss_rows(int64_t n);
int launch_scale(const float *src, const float *scale, float *dst, int64_t n,
                 hipStream_t s);
int launch_adam(float *p, const float *g, float *m, float *v, int64_t n, float lr,
                float b1, float b2, float eps, float wd, int64_t step,
                float grad_scale, hipStream_t s);

}  // namespace hcu
