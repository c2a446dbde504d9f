// Native executor for the 3D U-Net training hot path.
//
// A plan is built once per (spec, input shape): it resolves every layer's
// shapes exactly as hcat.unet.Unet_Constructor would see them
// (hcat/unet.py:16-143), reports the errors torch would raise, picks the
// kernel tiles, and lays out two caller-owned workspaces:
//   saved   - what backward needs from forward: the channels-last input, every
//             conv's pre-BatchNorm output y (post-activation values are
//             recomputed on load as relu(y*scale+shift)), pooled maps, the
//             up-convolution outputs U and the per-BatchNorm coefficients;
//   scratch - per-call temporaries: two gradient ping-pong buffers, reduction
//             partials and the re-laid-out weights of the layer in flight.
// forward/backward then enqueue one fixed kernel sequence on the caller's
// stream (no allocation, no host sync: capturable into a hipGraph).
//
// The decoder's cat(U, U) (crop returns U itself, hcat/unet.py:311-312,
// 319-340) is folded into Up.conv1's weights: conv(cat(U,U), W) ==
// conv(U, W[:, :C] + W[:, C:]) (per group), halving that layer's work; the
// weight gradient is scattered back to both halves.
#include "common.h"
#include "timing.h"
#include "../../include/hcunet.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace hcu {
static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}
int launch_outconv_wfinalize(const float *part_oc, int R, int Co, int C, int Cs, float *dw,
                             float *db, int accumulate, hipStream_t s);
int launch_bn_count_increment(int64_t *const *ptrs, int n, hipStream_t s);
}  // namespace hcu

using namespace hcu;

namespace {

constexpr int kTargetBlocks = 1024;

// Activation tensor dims.  es = element bytes: 4 (fp32 path, channel stride a
// multiple of 4 = 16 bytes) or 2 (bf16 path, channel stride a multiple of 8).
struct Dims {
  int B = 0, X = 0, Y = 0, Z = 0, C = 0, Cs = 0, es = 4;
  // > 0: the channels are parts of part_c real channels, each padded to the
  // vector width on its own (a chain input that is the channel-wise cat of
  // channels-last chain outputs, hcu_chain_spec::in_part_channels)
  int part_c = 0;
  int64_t vox() const { return (int64_t)B * X * Y * Z; }
  // 4-byte slots the tensor occupies (buffers are carved in float units)
  size_t floats() const { return ((size_t)vox() * Cs * es + 3) / 4; }
};

Dims mkdims(int B, int X, int Y, int Z, int C, int es) {
  Dims d;
  d.B = B;
  d.X = X;
  d.Y = Y;
  d.Z = Z;
  d.C = C;
  d.es = es;
  d.Cs = round_up(C, es == 2 ? 8 : 4);
  return d;
}

struct Region {
  size_t off = 0;
  size_t take_floats(size_t n) {
    const size_t o = off;
    off = align_up(off + n * sizeof(float), 256);
    return o;
  }
};

struct BNLayer {
  int C = 0, Cs = 0;
  size_t coef_off = 0;  // saved: 6 arrays of Cs floats
  int64_t gamma = 0, beta = 0;
  int index = 0;
  double count = 0;
};

struct ConvLayer {
  std::string name;  // layer tag for per-layer timing ("d0.c1", "u3.c2", ...)
  int Cout = 0, Cin_g = 0, groups = 1, fold_mod = 0, E = 0, T = 0;
  int part_c = 0, part_cs = 0;   // input channel parts (Dims::part_c): packed e <-> torch channel
  int K[3], D[3];
  int S[3] = {1, 1, 1}, P[3] = {0, 0, 0};   // stride, zero padding (chains; the U-Net is valid)
  bool has_dgrad = true;                   // input gradient planned (stride 1)
  // Dilated convolution run on the dilation sub-lattices (space-to-batch):
  // when the dilated halo does not fit the conv kernels' LDS, the input is
  // re-laid as dx*dy*dz dense sub-grids [B*D][X'][Y'][Z'] and fwd / dgrad /
  // wgrad are planned as dilation-1 convolutions on them (padding P/D).
  bool s2b = false;
  int L3[3] = {1, 1, 1};                   // lattice (= D) of the s2b form
  bool pw = false;                         // bf16 1x1x1, no BatchNorm input: pwconv.hip (forward, dgrad)
  bool pw_wg = false;                      // ... and its weight gradient (pw_wgrad_kernel)
  Dims sub_in, sub_out;                    // sub-grid tensors (batch B*D)
  int64_t w_off = 0, b_off = 0;
  Dims in, out;
  GConvArgs fwd{}, dgrad{};
  WGradArgs wg{};
  BNLayer bn;
  size_t y_off = 0;
  size_t wf_off = 0, wd_off = 0;  // prepared fwd / dgrad weight images in `saved`
};

struct ConvTLayer {
  std::string name;
  int Cin = 0, Cout = 0, T = 0;
  int K[3], S[3];
  int64_t w_off = 0, b_off = 0;
  Dims in, out;
  std::vector<GConvArgs> phases;
  std::vector<int> pJ;  // 6 ints per phase: px,py,pz,Jx,Jy,Jz
  bool fused = false;   // kernel % stride == 0: all phases in one GEMM (N = phase x Cout)
  GConvArgs fwdf{};
  GConvArgs dgrad{};
  WGradArgs wg{};
  // the weight gradient of the phase-folded forward (WGradArgs::nph: phases
  // as extra columns; the bias from the column-sum rows of dU), fp32 U-Net
  // decoders with kernel % stride == 0 and Cout % 4 == 0
  WGradArgs wgp{};
  bool wg_phase = false;
  // layer chains, bf16, no BatchNorm+ReLU applied to the input: the weight
  // gradient as the Conv3d weight gradient of the input-gradient convolution
  // (rows (tap, co) over the strided dU halo, columns ci over x; finalize
  // mode 0 with Cout = Cin, Cin_g = Cout -- the [Cin][Cout][K] layout of a
  // ConvTranspose3d weight is a Conv3d weight's [Cout][Cin][K]): every tap in
  // one block, instead of a (tap, co)-column GEMM with one 16-row subtile
  WGradArgs wgs{};
  bool wg_swap = false;
  size_t u_off = 0;
  size_t wf_off = 0, wd_off = 0;   // prepared weights in `saved` (fused fwd, dgrad)
  std::vector<size_t> wph_off;     // per-phase fwd weights when not fused
};

BNCoef coef_at(char *saved, const BNLayer &bn) {
  float *b = reinterpret_cast<float *>(saved + bn.coef_off);
  BNCoef c;
  c.scale = b;
  c.shift = b + bn.Cs;
  c.mean = b + 2 * bn.Cs;
  c.invstd = b + 3 * bn.Cs;
  c.c1 = b + 4 * bn.Cs;
  c.c0 = b + 5 * bn.Cs;
  return c;
}

GConvArgs gconv_conv_fwd(const Dims &in, const Dims &out, const int K[3], const int D[3], int Cout) {
  GConvArgs a{};
  a.B = in.B;
  a.IX = in.X; a.IY = in.Y; a.IZ = in.Z; a.ICs = in.Cs;
  a.OX = out.X; a.OY = out.Y; a.OZ = out.Z;
  a.SX = out.X; a.SY = out.Y; a.SZ = out.Z; a.OCs = out.Cs; a.Cout = Cout;
  a.osx = a.osy = a.osz = 1;
  a.KX = K[0]; a.KY = K[1]; a.KZ = K[2];
  a.sx = a.sy = a.sz = 1;
  a.dx = D[0]; a.dy = D[1]; a.dz = D[2];
  return a;
}

GConvArgs gconv_conv_dgrad(const Dims &in, const Dims &out, const int K[3], const int D[3], int E) {
  GConvArgs a{};
  a.B = in.B;
  a.IX = out.X; a.IY = out.Y; a.IZ = out.Z; a.ICs = out.Cs;
  a.OX = in.X; a.OY = in.Y; a.OZ = in.Z;
  a.SX = in.X; a.SY = in.Y; a.SZ = in.Z; a.OCs = in.Cs; a.Cout = E;
  a.osx = a.osy = a.osz = 1;
  a.KX = K[0]; a.KY = K[1]; a.KZ = K[2];
  a.sx = a.sy = a.sz = 1;
  a.dx = D[0]; a.dy = D[1]; a.dz = D[2];
  a.px = D[0] * (K[0] - 1); a.py = D[1] * (K[1] - 1); a.pz = D[2] * (K[2] - 1);
  return a;
}

WGradArgs wgrad_conv(const Dims &in, const Dims &out, const int K[3], const int D[3]) {
  WGradArgs w{};
  w.B = in.B;
  w.AX = in.X; w.AY = in.Y; w.AZ = in.Z; w.ACs = in.Cs;
  w.GX = out.X; w.GY = out.Y; w.GZ = out.Z; w.GCs = out.Cs;
  w.PX = out.X; w.PY = out.Y; w.PZ = out.Z;
  w.KX = K[0]; w.KY = K[1]; w.KZ = K[2];
  w.asx = w.asy = w.asz = 1;
  w.adx = D[0]; w.ady = D[1]; w.adz = D[2];
  w.gsx = w.gsy = w.gsz = 1;
  w.taps_rows = 1;
  w.bias_row = 1;
  return w;
}

// bf16 Conv3d weight gradients store slab rows of real input channels and
// columns of real output channels only (WGradArgs::ACr / GCr): RDCNet's
// 10-channel tensors sit in 16-slot strides.  Inputs made of channel parts
// keep every packed slot (finalize maps torch channels to packed slots).
void compact_slab(WGradArgs &w, const ConvLayer &L, bool bf) {
  w.ACr = w.GCr = 0;
  if (!bf) return;
  if (L.part_c == 0 && L.groups == 1) w.ACr = L.E;
  w.GCr = L.Cout;
}

// An input made of channel parts (Dims::part_c): every packed channel e of
// the input stride is a GEMM row (the padding ones get zero weights), and
// e maps to torch channel (e / part_cs) * part_c + e % part_cs.
void set_parts(ConvLayer &L, const Dims &in) {
  L.part_c = in.part_c;
  L.part_cs = in.part_c ? round_up(in.part_c, in.es == 2 ? 8 : 4) : 0;
  if (in.part_c) L.E = in.Cs;
}

// A bf16 1x1x1 Conv3d (stride 1, no padding, one group, no cat fold) takes the
// streaming pointwise kernels for its forward and input gradient when its
// input carries no BatchNorm+ReLU (checked at launch) and it has none itself
// (the chain's non-BatchNorm branch).  HCU_PW=0: bconv everywhere (A/B).
void set_pw(ConvLayer &L, const Dims &in, int cin_total) {
  static const bool off = getenv("HCU_PW") && getenv("HCU_PW")[0] == '0';
  L.pw = false;
  if (off || in.es != 2 || L.groups != 1 || L.fold_mod < cin_total) return;
  for (int i = 0; i < 3; ++i)
    if (L.K[i] != 1 || L.S[i] != 1 || L.P[i] != 0) return;
  L.pw = pw_supported(in.Cs, L.out.Cs, L.Cout, false) &&
         (!L.has_dgrad || pw_supported(in.Cs, L.out.Cs, L.Cout, true));
  // (the slab layout is bwgrad's taps_rows one, planned in L.wg)
  L.pw_wg = L.wg.use_bw && L.wg.taps_rows && L.wg.ACs == in.Cs && L.wg.GCs == L.out.Cs &&
            pw_wgrad_supported(in.Cs, L.out.Cs);
}

// Conv3d with stride / zero padding (nn.Conv3d(..., stride, padding), the
// r_unet.py layers): out = floor((in + 2P - D(K-1) - 1) / S) + 1.  Forward:
// o*S + t*D - P; input gradient (stride 1): the full correlation with padding
// D(K-1) - P; weight gradient: A offset o*S + t*D - P.  A dilated kernel whose
// halo does not fit the kernels' LDS runs on the dilation sub-lattices (s2b).
int setup_conv_general(ConvLayer &L, const Dims &in, int Cout, int groups, int fold_mod,
                       int cin_total, const char *name) {
  if (groups < 1 || cin_total % groups || Cout % groups)
    return fail(HCU_ERR_INVALID, std::string(name) + ": channels must be divisible by groups");
  L.Cout = Cout;
  L.groups = groups;
  L.Cin_g = cin_total / groups;
  L.fold_mod = fold_mod;
  L.E = std::min(fold_mod, cin_total);
  set_parts(L, in);
  L.T = L.K[0] * L.K[1] * L.K[2];
  L.in = in;
  int o[3];
  const int iv[3] = {in.X, in.Y, in.Z};
  for (int i = 0; i < 3; ++i) {
    const int span = iv[i] + 2 * L.P[i] - L.D[i] * (L.K[i] - 1);
    if (span < 1)
      return fail(HCU_ERR_SHAPE, std::string(name) + ": Calculated padded input size per channel: (" +
                                     std::to_string(in.X + 2 * L.P[0]) + " x " + std::to_string(in.Y + 2 * L.P[1]) +
                                     " x " + std::to_string(in.Z + 2 * L.P[2]) +
                                     "). Kernel size can't be greater than actual input size");
    o[i] = (span - 1) / L.S[i] + 1;
  }
  L.out = mkdims(in.B, o[0], o[1], o[2], Cout, in.es);
  const bool bf = in.es == 2;
  auto plan_c = [&](GConvArgs &a) { return bf ? plan_bconv(a, kTargetBlocks) : plan_conv_fp32(a, kTargetBlocks); };
  L.has_dgrad = L.S[0] == 1 && L.S[1] == 1 && L.S[2] == 1;
  L.s2b = false;
  // direct form
  {
    GConvArgs f = gconv_conv_fwd(in, L.out, L.K, L.D, Cout);
    f.sx = L.S[0]; f.sy = L.S[1]; f.sz = L.S[2];
    f.px = L.P[0]; f.py = L.P[1]; f.pz = L.P[2];
    const int ef = plan_c(f);
    int ed = 0;
    GConvArgs dg{};
    if (L.has_dgrad) {
      dg = gconv_conv_dgrad(in, L.out, L.K, L.D, L.E);
      dg.px = L.D[0] * (L.K[0] - 1) - L.P[0];
      dg.py = L.D[1] * (L.K[1] - 1) - L.P[1];
      dg.pz = L.D[2] * (L.K[2] - 1) - L.P[2];
      if (dg.px < 0 || dg.py < 0 || dg.pz < 0)
        return fail(HCU_ERR_UNSUPPORTED, std::string(name) + ": padding larger than dilation*(kernel-1)");
      ed = plan_c(dg);
    }
    WGradArgs w = wgrad_conv(in, L.out, L.K, L.D);
    w.asx = L.S[0]; w.asy = L.S[1]; w.asz = L.S[2];
    w.apx = L.P[0]; w.apy = L.P[1]; w.apz = L.P[2];
    compact_slab(w, L, bf);
    const int ew = bf ? plan_bwgrad(w, kTargetBlocks) : plan_wgrad(w, kTargetBlocks);
    const bool dil = L.D[0] > 1 || L.D[1] > 1 || L.D[2] > 1;
    if (!ef && !ed && !ew) {
      L.fwd = f;
      L.dgrad = dg;
      L.wg = w;
    } else if (!dil || !L.has_dgrad) {
      return ef ? ef : ed ? ed : ew;
    } else {
      L.s2b = true;
    }
  }
  if (L.s2b) {
    // dilation sub-lattices: output o = r + D*o' reads input r + D*(o' + t - P/D)
    int sub_i[3], sub_o[3], Pd[3];
    const int one[3] = {1, 1, 1};
    int nlat = 1;
    for (int i = 0; i < 3; ++i) {
      if (L.P[i] % L.D[i])
        return fail(HCU_ERR_UNSUPPORTED, std::string(name) + ": dilated convolution too large for one tile "
                                                             "and padding not a multiple of the dilation");
      L.L3[i] = L.D[i];
      nlat *= L.D[i];
      Pd[i] = L.P[i] / L.D[i];
      sub_i[i] = cdiv(iv[i], L.D[i]);
      sub_o[i] = sub_i[i] + 2 * Pd[i] - (L.K[i] - 1);
      if (sub_o[i] < cdiv(o[i], L.D[i]))
        return fail(HCU_ERR_UNSUPPORTED, std::string(name) + ": sub-lattice output too small");
    }
    L.sub_in = mkdims(in.B * nlat, sub_i[0], sub_i[1], sub_i[2], in.C, in.es);
    L.sub_in.Cs = in.Cs;
    L.sub_in.part_c = in.part_c;
    L.sub_out = mkdims(in.B * nlat, sub_o[0], sub_o[1], sub_o[2], Cout, in.es);
    L.fwd = gconv_conv_fwd(L.sub_in, L.sub_out, L.K, one, Cout);
    L.fwd.px = Pd[0]; L.fwd.py = Pd[1]; L.fwd.pz = Pd[2];
    if (int e = plan_c(L.fwd)) return e;
    L.dgrad = gconv_conv_dgrad(L.sub_in, L.sub_out, L.K, one, L.E);
    L.dgrad.px = (L.K[0] - 1) - Pd[0];
    L.dgrad.py = (L.K[1] - 1) - Pd[1];
    L.dgrad.pz = (L.K[2] - 1) - Pd[2];
    if (int e = plan_c(L.dgrad)) return e;
    L.wg = wgrad_conv(L.sub_in, L.sub_out, L.K, one);
    L.wg.apx = Pd[0]; L.wg.apy = Pd[1]; L.wg.apz = Pd[2];
    compact_slab(L.wg, L, bf);
    if (int e = bf ? plan_bwgrad(L.wg, kTargetBlocks) : plan_wgrad(L.wg, kTargetBlocks)) return e;
  }
  L.bn.C = Cout;
  L.bn.Cs = L.out.Cs;
  L.bn.count = (double)L.out.vox();
  set_pw(L, in, cin_total);
  return 0;
}

int setup_conv(ConvLayer &L, const Dims &in, int Cout, int groups, int fold_mod, int cin_total,
               const int K[3], const int D[3], const char *name, const int *S = nullptr,
               const int *P = nullptr) {
  for (int i = 0; i < 3; ++i) {
    L.K[i] = K[i];
    L.D[i] = D[i];
    L.S[i] = S ? S[i] : 1;
    L.P[i] = P ? P[i] : 0;
    if (K[i] < 1 || D[i] < 1) return fail(HCU_ERR_INVALID, std::string(name) + ": bad kernel/dilation");
    if (L.S[i] < 1 || L.P[i] < 0) return fail(HCU_ERR_INVALID, std::string(name) + ": bad stride/padding");
  }
  if (S || P) return setup_conv_general(L, in, Cout, groups, fold_mod, cin_total, name);
  if (groups < 1 || cin_total % groups || Cout % groups)
    return fail(HCU_ERR_INVALID, std::string(name) + ": channels must be divisible by groups");
  L.Cout = Cout;
  L.groups = groups;
  L.Cin_g = cin_total / groups;
  L.fold_mod = fold_mod;
  L.E = std::min(fold_mod, cin_total);
  set_parts(L, in);
  L.T = K[0] * K[1] * K[2];
  L.in = in;
  const int ox = in.X - D[0] * (K[0] - 1), oy = in.Y - D[1] * (K[1] - 1), oz = in.Z - D[2] * (K[2] - 1);
  if (ox < 1 || oy < 1 || oz < 1)
    return fail(HCU_ERR_SHAPE, std::string(name) + ": Calculated padded input size per channel: (" +
                                   std::to_string(in.X) + " x " + std::to_string(in.Y) + " x " +
                                   std::to_string(in.Z) +
                                   "). Kernel size can't be greater than actual input size");
  L.out = mkdims(in.B, ox, oy, oz, Cout, in.es);
  const bool bf = in.es == 2;
  L.fwd = gconv_conv_fwd(in, L.out, K, D, Cout);
  if (int e = bf ? plan_bconv(L.fwd, kTargetBlocks) : plan_conv_fp32(L.fwd, kTargetBlocks)) return e;
  L.dgrad = gconv_conv_dgrad(in, L.out, K, D, L.E);
  if (int e = bf ? plan_bconv(L.dgrad, kTargetBlocks) : plan_conv_fp32(L.dgrad, kTargetBlocks))
    return e;
  L.wg = wgrad_conv(in, L.out, K, D);
  compact_slab(L.wg, L, bf);
  if (int e = bf ? plan_bwgrad(L.wg, kTargetBlocks) : plan_wgrad(L.wg, kTargetBlocks)) return e;
  L.bn.C = Cout;
  L.bn.Cs = L.out.Cs;
  L.bn.count = (double)L.out.vox();
  set_pw(L, in, cin_total);
  return 0;
}


int setup_convt(ConvTLayer &u, const Dims &cur, int o, const int K[3], const int S[3],
                size_t &max_wprep, size_t &max_part, size_t &max_kpart) {
  const int f = cur.C;
  u.Cin = f;
  u.Cout = o;
  u.T = K[0] * K[1] * K[2];
  for (int d = 0; d < 3; ++d) {
    u.K[d] = K[d];
    u.S[d] = S[d];
    if (K[d] < 1 || S[d] < 1) return fail(HCU_ERR_INVALID, "ConvTranspose3d: bad kernel/stride");
  }
  u.in = cur;
  const int ux = (cur.X - 1) * u.S[0] + u.K[0], uy = (cur.Y - 1) * u.S[1] + u.K[1],
            uz = (cur.Z - 1) * u.S[2] + u.K[2];
  u.out = mkdims(cur.B, ux, uy, uz, o, cur.es);
  const bool bf = cur.es == 2;
  u.phases.clear();
  u.pJ.clear();
  const int nph = u.S[0] * u.S[1] * u.S[2];
  u.fused = u.K[0] % u.S[0] == 0 && u.K[1] % u.S[1] == 0 && u.K[2] % u.S[2] == 0;
  if (bf && !u.fused)
    return fail(HCU_ERR_UNSUPPORTED,
                "ConvTranspose3d with kernel % stride != 0 is not supported on the bf16 path");
  if (u.fused) {
    const int Jx = u.K[0] / u.S[0], Jy = u.K[1] / u.S[1], Jz = u.K[2] / u.S[2];
    GConvArgs a{};
    a.B = cur.B;
    a.IX = cur.X; a.IY = cur.Y; a.IZ = cur.Z; a.ICs = cur.Cs;
    a.OX = cur.X + Jx - 1; a.OY = cur.Y + Jy - 1; a.OZ = cur.Z + Jz - 1;
    a.SX = ux; a.SY = uy; a.SZ = uz; a.OCs = u.out.Cs; a.Cout = o;
    a.osx = u.S[0]; a.osy = u.S[1]; a.osz = u.S[2];
    a.KX = Jx; a.KY = Jy; a.KZ = Jz;
    a.sx = a.sy = a.sz = 1;
    a.dx = a.dy = a.dz = 1;
    a.px = Jx - 1; a.py = Jy - 1; a.pz = Jz - 1;
    a.nph = nph; a.phx = u.S[0]; a.phy = u.S[1]; a.phz = u.S[2];
    // columns per phase padded to the 8 (bf16) / 4 (fp32) a packed vector and
    // a lane's store span (zero weights and bias; RDCNet's 5 output channels)
    const int cv = bf ? 8 : 4;
    if (o % cv) a.cph = round_up(o, cv);
    if (bf) {
      if (int e = plan_bconv(a, kTargetBlocks)) return e;
      u.fwdf = a;
      max_wprep = std::max(max_wprep, wprep_floats(a));
      max_kpart = std::max(max_kpart, conv_partial_floats(a));
    } else if (plan_conv_fp32(a, kTargetBlocks) == 0 && (a.use_bconv || a.use_conv2)) {
      u.fwdf = a;
      max_wprep = std::max(max_wprep, wprep_floats(a));
      max_kpart = std::max(max_kpart, conv_partial_floats(a));
    } else {
      u.fused = false;
    }
  }
  for (int qx = 0; qx < (bf ? 0 : u.S[0]); ++qx)
    for (int qy = 0; qy < u.S[1]; ++qy)
      for (int qz = 0; qz < u.S[2]; ++qz) {
        const int Jx = cdiv(u.K[0] - qx, u.S[0]), Jy = cdiv(u.K[1] - qy, u.S[1]),
                  Jz = cdiv(u.K[2] - qz, u.S[2]);
        if (Jx < 1 || Jy < 1 || Jz < 1)
          return fail(HCU_ERR_UNSUPPORTED, "ConvTranspose3d with kernel < stride is not supported");
        GConvArgs a{};
        a.B = cur.B;
        a.IX = cur.X; a.IY = cur.Y; a.IZ = cur.Z; a.ICs = cur.Cs;
        a.OX = cdiv(ux - qx, u.S[0]); a.OY = cdiv(uy - qy, u.S[1]); a.OZ = cdiv(uz - qz, u.S[2]);
        a.SX = ux; a.SY = uy; a.SZ = uz; a.OCs = u.out.Cs; a.Cout = o;
        a.osx = u.S[0]; a.osy = u.S[1]; a.osz = u.S[2];
        a.ofx = qx; a.ofy = qy; a.ofz = qz;
        a.KX = Jx; a.KY = Jy; a.KZ = Jz;
        a.sx = a.sy = a.sz = 1;
        a.dx = a.dy = a.dz = 1;
        a.px = Jx - 1; a.py = Jy - 1; a.pz = Jz - 1;
        if (int e = plan_gconv(a, std::max(64, kTargetBlocks / nph))) return e;
        u.phases.push_back(a);
        const int pj[6] = {qx, qy, qz, Jx, Jy, Jz};
        u.pJ.insert(u.pJ.end(), pj, pj + 6);
        max_wprep = std::max(max_wprep, (size_t)Jx * Jy * Jz * a.ICs * a.CoutW);
      }
  {  // dgrad: strided correlation of dU with W[ci][co][t]
    GConvArgs a{};
    a.B = cur.B;
    a.IX = ux; a.IY = uy; a.IZ = uz; a.ICs = u.out.Cs;
    a.OX = cur.X; a.OY = cur.Y; a.OZ = cur.Z;
    a.SX = cur.X; a.SY = cur.Y; a.SZ = cur.Z; a.OCs = cur.Cs; a.Cout = f;
    a.osx = a.osy = a.osz = 1;
    a.KX = u.K[0]; a.KY = u.K[1]; a.KZ = u.K[2];
    a.sx = u.S[0]; a.sy = u.S[1]; a.sz = u.S[2];
    a.dx = a.dy = a.dz = 1;
    if (int e = bf ? plan_bconv(a, kTargetBlocks) : plan_conv_fp32(a, kTargetBlocks)) return e;
    u.dgrad = a;
    max_wprep = std::max(max_wprep, wprep_floats(a));
    max_part = std::max(max_part, (size_t)gconv_rows(a) * a.CoutW * 2);
    max_kpart = std::max(max_kpart, conv_partial_floats(a));
  }
  {  // wgrad: rows = ci, cols = (t, co)
    WGradArgs w{};
    w.B = cur.B;
    w.AX = cur.X; w.AY = cur.Y; w.AZ = cur.Z; w.ACs = cur.Cs;
    w.GX = ux; w.GY = uy; w.GZ = uz; w.GCs = u.out.Cs;
    w.PX = cur.X; w.PY = cur.Y; w.PZ = cur.Z;
    w.KX = u.K[0]; w.KY = u.K[1]; w.KZ = u.K[2];
    w.asx = w.asy = w.asz = 1;
    w.gsx = u.S[0]; w.gsy = u.S[1]; w.gsz = u.S[2];
    w.gdx = w.gdy = w.gdz = 1;
    w.taps_rows = 0;
    w.bias_row = 0;
    if (int e = bf ? plan_bwgrad(w, kTargetBlocks) : plan_wgrad(w, kTargetBlocks)) return e;
    u.wg = w;
    max_part = std::max(max_part, wgrad_partial_floats(w));
    max_part = std::max(max_part, (size_t)chansum_rows(u.out.vox(), u.out.Cs) * u.out.Cs);
  }
  u.wg_phase = false;
  // The weight gradient of the phase-folded forward (stride phases as extra
  // output columns) on wgrad3; the other layers run the per-tap wgrad_kernel.
  // (The U-Net's bias gradient: the column sums of dU, written by the
  // folded conv1's input-gradient kernel; layer chains: chansum.)
  if (!bf && u.fused && o % 4 == 0) {
    // dW'[(j, ci)][(q, co)] = sum_o A[o + j - (J-1)][ci] * dU[o*S + q][co] over the
    // phase grid o (the forward's fused GEMM, hcat/unet.py:294-298)
    const int J[3] = {u.K[0] / u.S[0], u.K[1] / u.S[1], u.K[2] / u.S[2]};
    WGradArgs w{};
    w.B = cur.B;
    w.AX = cur.X; w.AY = cur.Y; w.AZ = cur.Z; w.ACs = cur.Cs;
    w.GX = ux; w.GY = uy; w.GZ = uz; w.GCs = u.out.Cs;
    w.PX = cur.X + J[0] - 1; w.PY = cur.Y + J[1] - 1; w.PZ = cur.Z + J[2] - 1;
    w.KX = J[0]; w.KY = J[1]; w.KZ = J[2];
    w.asx = w.asy = w.asz = 1;
    w.adx = w.ady = w.adz = 1;
    w.apx = J[0] - 1; w.apy = J[1] - 1; w.apz = J[2] - 1;
    w.gsx = u.S[0]; w.gsy = u.S[1]; w.gsz = u.S[2];
    w.gdx = w.gdy = w.gdz = 1;
    w.taps_rows = 1;
    w.bias_row = 0;
    w.nph = nph; w.phx = u.S[0]; w.phy = u.S[1]; w.phz = u.S[2]; w.GCout = o;
    if (plan_wgrad(w, kTargetBlocks) == 0 && w.v2 == 3) {
      u.wgp = w;
      u.wg_phase = true;
      max_part = std::max(max_part, wgrad_partial_floats(w));
    } else {
      set_error("");
    }
  }
  return 0;
}

}  // namespace

#define HCU_NBUF 32   // gradient slots (at most; Ctx::alloc)
#define HCU_NBUF_RING 6   // ring size when one slot per allocation does not fit
#define HCU_FORK_RING 16   // marker events of forks that cannot use the chain record

struct hcu_unet_plan {
  hcu_unet_spec spec;
  int B, X, Y, Z, L;
  int flags = 0;       // HCU_PLAN_FORWARD_ONLY: activations in two ping-pong buffers
  int es = 4;          // activation element bytes: 4 (fp32 path) or 2 (bf16 path)
  Dims xin;
  size_t xcl_off = 0;
  std::vector<ConvLayer> dc1, dc2, uc1, uc2;
  // the first convolution stages the NCXYZ input itself (conv8, or bconv
  // with one channel group; <= 4 input channels, groups 1): no channels-last
  // layout pass, and its kernel reads t->x
  bool ncx_first = false;
  std::vector<Dims> pooled;
  std::vector<size_t> pool_off;
  std::vector<ConvTLayer> up;
  int64_t oc_w = 0, oc_b = 0;
  int Co = 0;
  Dims outd;
  int64_t n_params = 0;
  int n_bn = 0;
  std::vector<PrepJob> prep_jobs;  // weight re-layouts, one batched launch per forward
  // the same split: images the forward reads / input-gradient images only the
  // backward reads (re-laid on the branch stream while the forward runs)
  std::vector<PrepJob> prep_fwd, prep_bwd;
  size_t saved_bytes = 0, scratch_bytes = 0;
  // scratch layout
  // Backward gradient buffers: a ring of HCU_NBUF activation-sized slots, so
  // a slot read by the weight-gradient branch is rewritten only several
  // layers later (see Ctx::alloc).
  size_t buf_off[HCU_NBUF] = {};
  // slots in use: one per allocation of a U-Net backward when they fit (no
  // slot is rewritten, so no reader events or waits on the gradient ring),
  // else a ring of HCU_NBUF_RING (chains, very large activations)
  int nbuf = HCU_NBUF_RING;
  bool no_reuse = false;
  size_t part_off = 0, wpart_off = 0, wprep_off = 0, kpart_off = 0;
  // per decoder level: the column-sum rows of dU (the up_conv bias gradient)
  // written by the folded conv1's input-gradient kernel
  size_t colsum_off[HCU_MAX_LEVELS] = {};
  // layer chains: the packed weight images are saved[img_lo, img_lo + img_bytes)
  size_t img_lo = 0, img_bytes = 0;
  double fwd_flops = 0.0;   // forward convolution FLOPs (graph replay only below 100 GFLOP)
  // Layer-chain plans (hcu_chain_*): a sequence of ops instead of the U-Net.
  struct ChainOp {
    int kind = 0;                  // HCU_CHAIN_CONV / POOL / CONVT
    bool bn_relu = false, fold = false;
    ConvLayer conv;
    ConvTLayer ct;
    int pk[3] = {1, 1, 1};
    Dims pooled;
    size_t pool_off = 0;
    int crop[3] = {0, 0, 0};       // ConvTranspose3d padding: crop of the full output
    Dims ufull;
    size_t xs_off = 0;             // s2b conv: the sub-lattice input (saved for the weight gradient)
  };
  std::vector<ChainOp> chain;
  bool is_chain = false;
  bool in_cl = false, out_cl = false;   // chain boundaries in the executor's layout (hcu_chain_spec)
  size_t ufull_off = 0, sub_off[3] = {};   // scratch: full ConvTranspose3d output, sub-lattice temporaries
  size_t max_sub = 0, max_ufull = 0;
  size_t wpart_floats = 0;   // weight-gradient slab arena (deferred, batched finalizes)
  size_t max_act = 0, max_part = 0, max_wprep = 0, max_kpart = 0;
  // Captured launch sequences (hipGraph) keyed by the buffers they bake in:
  // forward and backward are fixed kernel sequences, so a replay costs one
  // launch on the host instead of one per kernel.
  struct Graph {
    std::vector<uintptr_t> key;
    hipGraphExec_t exec = nullptr;
    uint64_t used = 0;
  };
  mutable std::mutex gmu;
  mutable std::vector<Graph> graphs;
  mutable hipStream_t cap_stream = nullptr;
  mutable int cap_device = -1;
  mutable uint64_t gclock = 0;
  // Weight-gradient branch of the backward: its own stream and the events
  // that order it against the data-gradient chain (created on first use).
  mutable std::mutex smu;
  mutable hipStream_t side = nullptr;
  mutable int side_device = -1;
  mutable hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_slot[HCU_NBUF] = {};
  mutable hipEvent_t ev_chain = nullptr;   // stop event of the chain's kernels (Ctx::arm_chain)
  mutable hipEvent_t ev_prep = nullptr;    // the backward's input-gradient weight images are laid out
  mutable hipEvent_t ev_fork_ring[HCU_FORK_RING] = {};   // marker forks (Ctx::fork)
  mutable unsigned fork_next = 0;
  // data-parallel overlap (hcu_unet_set_grad_events): caller-owned events the
  // backward records when the decoder's / the deep encoder levels' gradients are final
  hipEvent_t grad_ev[2] = {nullptr, nullptr};
  int grad_deep = -1;
  void destroy_side() const {
    if (side) (void)hipStreamDestroy(side);
    for (hipEvent_t *e : {&ev_fork, &ev_join, &ev_chain, &ev_prep})
      if (*e) (void)hipEventDestroy(*e);
    for (hipEvent_t &e : ev_slot)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t &e : ev_fork_ring)
      if (e) (void)hipEventDestroy(e);
    side = nullptr;
    ev_fork = ev_join = ev_chain = ev_prep = nullptr;
    for (hipEvent_t &e : ev_slot) e = nullptr;
    for (hipEvent_t &e : ev_fork_ring) e = nullptr;
  }
  ~hcu_unet_plan() {
    for (Graph &g : graphs)
      if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    destroy_side();
  }
};

namespace {

size_t prep_floats_fwd(const ConvLayer &L) { return wprep_floats(L.fwd); }
size_t prep_floats_dgrad(const ConvLayer &L) { return wprep_floats(L.dgrad); }
// Elements of a prepared weight image (bf16 images hold two per float slot).
size_t prep_elems(const GConvArgs &a) {
  if (a.use_bconv) return (size_t)wpack_count(wpack_of(a), a.KX * a.KY * a.KZ, a.ICs, a.CoutW);
  return wprep_floats(a);
}

void track_conv(hcu_unet_plan &p, const ConvLayer &L) {
  p.max_act = std::max(p.max_act, std::max(L.in.floats(), L.out.floats()));
  p.max_part = std::max(p.max_part, (size_t)gconv_rows(L.fwd) * L.fwd.CoutW * 4);  // StatRow
  p.max_part = std::max(p.max_part, wgrad_partial_floats(L.wg));
  p.max_part = std::max(p.max_part, (size_t)gconv_rows(L.dgrad) * L.dgrad.CoutW * 2);
  p.max_part = std::max(p.max_part, (size_t)bwd_rows(L.out.vox(), L.out.Cs) * L.out.Cs * 2);
  p.max_wprep = std::max(p.max_wprep, std::max(prep_floats_fwd(L), prep_floats_dgrad(L)));
  p.max_kpart = std::max(p.max_kpart, std::max(conv_partial_floats(L.fwd), conv_partial_floats(L.dgrad)));
}

int build_plan(hcu_unet_plan &p) {
  const hcu_unet_spec &s = p.spec;
  const int L = s.levels;
  if (L < 2 || L > HCU_MAX_LEVELS)
    return fail(HCU_ERR_INVALID, "The Number of Features must be at least 2");
  for (int i = 0; i + 1 < L; ++i)
    if (s.features[i] * 2 != s.features[i + 1])
      return fail(HCU_ERR_INVALID, "Feature Sizes must be multiples of two from each other");
  if (s.in_channels < 1 || s.out_channels < 1 || s.features[0] < 1)
    return fail(HCU_ERR_INVALID, "channel counts must be positive");
  if (p.B < 1 || p.X < 1 || p.Y < 1 || p.Z < 1) return fail(HCU_ERR_SHAPE, "empty input");
  for (int i = 0; i < 3; ++i)
    if (s.pool_k[i] < 1 || s.up_k[i] < 1 || s.up_s[i] < 1)
      return fail(HCU_ERR_INVALID, "bad pool/upsample kernel");
  p.L = L;
  p.dc1.resize(L);
  p.dc2.resize(L);
  p.pooled.resize(L);
  p.pool_off.resize(L);
  p.up.resize(L - 1);
  p.uc1.resize(L - 1);
  p.uc2.resize(L - 1);

  // Parameter offsets in Unet_Constructor.parameters() order (hcat/unet.py:87-123:
  // out_conv, then down_steps[i].{conv1,conv2,batch1,batch2}, then
  // up_steps[j].{conv1,conv2,up_conv,batch1,batch2}).
  int64_t off = 0;
  const int f0 = s.features[0];
  p.Co = s.out_channels;
  p.oc_w = off; off += (int64_t)p.Co * f0;
  p.oc_b = off; off += p.Co;
  const int T1 = s.k1[0] * s.k1[1] * s.k1[2], T2 = s.k2[0] * s.k2[1] * s.k2[2];
  const int Tu = s.up_k[0] * s.up_k[1] * s.up_k[2];
  int bn_index = 0;
  for (int i = 0; i < L; ++i) {
    const int cin = i == 0 ? s.in_channels : s.features[i - 1];
    const int f = s.features[i];
    if (cin % s.g1 || f % s.g1 || f % s.g2)
      return fail(HCU_ERR_INVALID, "in_channels/out_channels must be divisible by groups");
    ConvLayer &c1 = p.dc1[i], &c2 = p.dc2[i];
    c1.name = "d" + std::to_string(i) + ".c1";
    c2.name = "d" + std::to_string(i) + ".c2";
    c1.w_off = off; off += (int64_t)f * (cin / s.g1) * T1;
    c1.b_off = off; off += f;
    c2.w_off = off; off += (int64_t)f * (f / s.g2) * T2;
    c2.b_off = off; off += f;
    c1.bn.gamma = off; off += f;
    c1.bn.beta = off; off += f;
    c2.bn.gamma = off; off += f;
    c2.bn.beta = off; off += f;
    c1.bn.index = bn_index++;
    c2.bn.index = bn_index++;
  }
  for (int j = 0; j < L - 1; ++j) {
    const int f = s.features[L - 1 - j], o = s.features[L - 2 - j];
    if (f % s.g1 || o % s.g1 || o % s.g2)
      return fail(HCU_ERR_INVALID, "in_channels/out_channels must be divisible by groups");
    ConvLayer &c1 = p.uc1[j], &c2 = p.uc2[j];
    ConvTLayer &u = p.up[j];
    c1.name = "u" + std::to_string(j) + ".c1";
    c2.name = "u" + std::to_string(j) + ".c2";
    u.name = "u" + std::to_string(j) + ".up";
    c1.w_off = off; off += (int64_t)o * (f / s.g1) * T1;
    c1.b_off = off; off += o;
    c2.w_off = off; off += (int64_t)o * (o / s.g2) * T2;
    c2.b_off = off; off += o;
    u.w_off = off; off += (int64_t)f * o * Tu;
    u.b_off = off; off += o;
    c1.bn.gamma = off; off += o;
    c1.bn.beta = off; off += o;
    c2.bn.gamma = off; off += o;
    c2.bn.beta = off; off += o;
    c1.bn.index = bn_index++;
    c2.bn.index = bn_index++;
  }
  p.n_params = off;
  p.n_bn = bn_index;

  // Shapes, forward order.
  Region saved;
  // Activation tensors in forward order.  A forward-only plan keeps none of them
  // for a backward: every forward op reads only the tensor the previous op
  // wrote (the skip tensors are shape checks only, hcat/unet.py:309-315), so
  // they alternate between two buffers of the largest activation.
  const bool fwd_only = (p.flags & HCU_PLAN_FORWARD_ONLY) != 0;
  std::vector<std::pair<size_t *, size_t>> acts;
  auto act_take = [&](size_t floats, size_t &off) {
    if (fwd_only)
      acts.emplace_back(&off, floats);
    else
      off = saved.take_floats(floats);
  };
  if (s.compute_dtype != HCU_F32 && s.compute_dtype != HCU_BF16)
    return fail(HCU_ERR_INVALID, "compute_dtype must be HCU_F32 or HCU_BF16");
  p.es = s.compute_dtype == HCU_BF16 ? 2 : 4;
  p.xin = mkdims(p.B, p.X, p.Y, p.Z, s.in_channels, p.es);
  act_take(p.xin.floats(), p.xcl_off);
  p.max_act = p.xin.floats();
  Dims cur = p.xin;
  for (int i = 0; i < L; ++i) {
    const int cin = cur.C, f = s.features[i];
    if (int e = setup_conv(p.dc1[i], cur, f, s.g1, cin, cin, s.k1, s.d1, "down conv1")) return e;
    if (int e = setup_conv(p.dc2[i], p.dc1[i].out, f, s.g2, f, f, s.k2, s.d2, "down conv2")) return e;
    for (ConvLayer *c : {&p.dc1[i], &p.dc2[i]}) {
      act_take(c->out.floats(), c->y_off);
      c->bn.coef_off = saved.take_floats((size_t)6 * c->bn.Cs);
      track_conv(p, *c);
    }
    cur = p.dc2[i].out;
    if (i < L - 1) {
      const int px = cur.X / s.pool_k[0], py = cur.Y / s.pool_k[1], pz = cur.Z / s.pool_k[2];
      if (px < 1 || py < 1 || pz < 1)
        return fail(HCU_ERR_SHAPE, "max_pool3d: Output size is too small");
      p.pooled[i] = mkdims(p.B, px, py, pz, f, p.es);
      act_take(p.pooled[i].floats(), p.pool_off[i]);
      p.max_act = std::max(p.max_act, p.pooled[i].floats());
      cur = p.pooled[i];
    }
  }
  for (int j = 0; j < L - 1; ++j) {
    const int level = L - 2 - j;
    const int f = s.features[L - 1 - j], o = s.features[L - 2 - j];
    ConvTLayer &u = p.up[j];
    if (int e = setup_convt(u, cur, o, s.up_k, s.up_s, p.max_wprep, p.max_part, p.max_kpart)) return e;
    const Dims &skip = p.dc2[level].out;
    if (u.out.X > skip.X || u.out.Y > skip.Y || u.out.Z > skip.Z)
      return fail(HCU_ERR_SHAPE,
                  "Sizes of tensors must match except in dimension 1 (upsampled " +
                      std::to_string(u.out.X) + "x" + std::to_string(u.out.Y) + "x" +
                      std::to_string(u.out.Z) + " exceeds skip " + std::to_string(skip.X) + "x" +
                      std::to_string(skip.Y) + "x" + std::to_string(skip.Z) + ")");
    act_take(u.out.floats(), u.u_off);
    p.max_act = std::max(p.max_act, u.out.floats());
    // conv1 consumes cat(U, U): fold (cat channels 2*o, effective o)
    if (int e = setup_conv(p.uc1[j], u.out, o, s.g1, o, f, s.k1, s.d1, "up conv1")) return e;
    if (int e = setup_conv(p.uc2[j], p.uc1[j].out, o, s.g2, o, o, s.k2, s.d2, "up conv2")) return e;
    for (ConvLayer *c : {&p.uc1[j], &p.uc2[j]}) {
      act_take(c->out.floats(), c->y_off);
      c->bn.coef_off = saved.take_floats((size_t)6 * c->bn.Cs);
      track_conv(p, *c);
    }
    cur = p.uc2[j].out;
  }
  if (p.Co > 4) return fail(HCU_ERR_UNSUPPORTED, "out_channels > 4 is not supported yet");
  {
    // The first convolution reads the NCXYZ volume itself in fp32 plans; bf16
    // plans keep the separate channels-last pass (to_cl_vox) ahead of it: the
    // NCXYZ gather issues one 4-byte load per channel plane and element, and
    // config 3 ran 6.345-6.349 ms/step with it against 6.269-6.275 without
    // (interleaved, round 6).  HCU_NCX=0 / 1 forces either (A/B).
    static const int ncx_env = getenv("HCU_NCX") ? (getenv("HCU_NCX")[0] == '1' ? 1 : 0) : -1;
    const bool ncx_on = ncx_env >= 0 ? ncx_env == 1 : p.es == 4;
    const GConvArgs &f = p.dc1[0].fwd;
    const bool conv8_ok = f.use_conv8 && f.ICs == 4 && p.es == 4;
    const bool bconv_ok = f.use_bconv && f.CK == (p.es == 2 ? 8 : 4) && f.NPF > 0 && f.ksplit == 1 && f.nph <= 1;
    p.ncx_first = ncx_on && s.in_channels <= 4 && s.g1 == 1 && (conv8_ok || bconv_ok);
  }
  p.outd = mkdims(p.B, cur.X, cur.Y, cur.Z, p.Co, 4);
  {
    const int R = outconv_bwd_rows(cur.vox(), cur.Cs);
    p.max_part = std::max(p.max_part, (size_t)R * cur.Cs * 2 + (size_t)R * (p.Co * cur.Cs + p.Co) + 64);
  }
  // Prepared (GEMM-layout) weights of every layer: written once per forward by
  // one batched launch, read by the forward and backward GEMMs.
  p.prep_jobs.clear();
  auto add_job = [&](int kind, size_t n, int64_t src, const WPack &pk, const int *prm, int np,
                     size_t &off) {
    PrepJob j{};
    j.kind = kind;
    j.bf16 = p.es == 2;
    j.n = (int64_t)n;
    j.src = src;
    off = saved.take_floats(j.bf16 ? (n + 1) / 2 : n);
    j.dst = (int64_t)(off / sizeof(float));
    j.pk = pk;
    std::copy(prm, prm + np, j.p);
    p.prep_jobs.push_back(j);
  };
  auto conv_jobs = [&](ConvLayer &cl) {
    const int pf[8] = {cl.Cout, cl.Cin_g, cl.groups, cl.fold_mod, cl.T, cl.fwd.ICs, cl.fwd.CoutW,
                       std::min(cl.fold_mod, cl.groups * cl.Cin_g)};
    add_job(PREP_CONV_FWD, prep_elems(cl.fwd), cl.w_off, wpack_of(cl.fwd), pf, 8, cl.wf_off);
    const int pd[8] = {cl.Cout, cl.Cin_g, cl.groups, cl.fold_mod, cl.T, cl.dgrad.ICs,
                       cl.dgrad.CoutW, cl.E};
    add_job(PREP_CONV_DGRAD, prep_elems(cl.dgrad), cl.w_off, wpack_of(cl.dgrad), pd, 8,
            cl.wd_off);
  };
  for (int i = 0; i < L; ++i) {
    conv_jobs(p.dc1[i]);
    conv_jobs(p.dc2[i]);
  }
  for (int j = 0; j + 1 < L; ++j) {
    ConvTLayer &u = p.up[j];
    conv_jobs(p.uc1[j]);
    conv_jobs(p.uc2[j]);
    if (u.fused) {
      const int pf[11] = {u.Cin, u.Cout, u.K[0], u.K[1], u.K[2], u.S[0], u.S[1], u.S[2],
                          u.fwdf.ICs, u.fwdf.CoutW, u.fwdf.cph};
      add_job(PREP_CONVT_FUSED, prep_elems(u.fwdf), u.w_off, wpack_of(u.fwdf), pf, 11, u.wf_off);
    } else {
      u.wph_off.assign(u.phases.size(), 0);
      for (size_t ph = 0; ph < u.phases.size(); ++ph) {
        const int *pj = &u.pJ[ph * 6];
        const GConvArgs &a = u.phases[ph];
        const int pf[16] = {u.Cin, u.Cout, u.K[0], u.K[1], u.K[2], u.S[0], u.S[1], u.S[2],
                            pj[0], pj[1], pj[2], pj[3], pj[4], pj[5], a.ICs, a.CoutW};
        add_job(PREP_CONVT_PHASE, (size_t)pj[3] * pj[4] * pj[5] * a.ICs * a.CoutW, u.w_off,
                WPack{}, pf, 16, u.wph_off[ph]);
      }
    }
    const int pd[5] = {u.Cin, u.Cout, u.T, u.dgrad.ICs, u.dgrad.CoutW};
    add_job(PREP_CONVT_DGRAD, prep_elems(u.dgrad), u.w_off, wpack_of(u.dgrad), pd, 5, u.wd_off);
  }
  p.prep_fwd.clear();
  p.prep_bwd.clear();
  for (const PrepJob &j : p.prep_jobs)
    (j.kind == PREP_CONV_DGRAD || j.kind == PREP_CONVT_DGRAD ? p.prep_bwd : p.prep_fwd).push_back(j);
  if (fwd_only) {
    size_t mx = 1;
    for (const auto &a : acts) mx = std::max(mx, a.second);
    const size_t pp[2] = {saved.take_floats(mx), saved.take_floats(mx)};
    for (size_t k = 0; k < acts.size(); ++k) *acts[k].first = pp[k & 1];
  }
  p.saved_bytes = saved.off;
  // forward convolution FLOPs: decides graph replay vs direct launches
  p.fwd_flops = 0.0;
  for (const auto *v : {&p.dc1, &p.dc2, &p.uc1, &p.uc2})
    for (const ConvLayer &cl : *v)
      p.fwd_flops += 2.0 * cl.fwd.B * cl.fwd.OX * cl.fwd.OY * cl.fwd.OZ * (double)cl.Cout * cl.Cin_g * cl.T;

  Region scratch;
  // the gradient ring, the weight-gradient partials and the weight re-layout
  // scratch are backward-only
  {
    // a U-Net backward allocates 1 + 3 slots per decoder level + at most 3 per
    // encoder level: one slot each when that stays within 32 slots and 24 GB
    const int need = 1 + 3 * (L - 1) + 3 * L;
    p.no_reuse = !fwd_only && need <= HCU_NBUF && (double)need * p.max_act * 4.0 <= 24e9;
    p.nbuf = p.no_reuse ? need : HCU_NBUF_RING;
    for (int i = 0; i < HCU_NBUF; ++i)
      p.buf_off[i] = scratch.take_floats(fwd_only || i >= p.nbuf ? 0 : p.max_act);
  }
  p.part_off = scratch.take_floats(p.max_part);
  // the slab arena holds several layers' weight-gradient partials until their
  // finalizes run together (at least one layer's, at most 8 M floats beyond)
  p.wpart_floats = fwd_only ? 0 : std::max<size_t>(p.max_part, (size_t)8 << 20);
  p.wpart_off = scratch.take_floats(p.wpart_floats);
  p.wprep_off = scratch.take_floats(fwd_only ? 0 : p.max_wprep);
  p.kpart_off = scratch.take_floats(std::max<size_t>(p.max_kpart, 1));
  for (int j = 0; j + 1 < L; ++j)
    p.colsum_off[j] = scratch.take_floats(fwd_only ? 0 : (size_t)gconv_rows(p.uc1[j].dgrad) * p.uc1[j].dgrad.CoutW * 4);
  p.scratch_bytes = scratch.off;
  if (getenv("HCU_PLAN_LOG")) {   // weight-gradient kernels and their partial slabs (measurement)
    auto wlog = [](const std::string &n, const WGradArgs &w) {
      const char *k = w.use_bw ? "bwgrad" : w.v2 == 3 ? "wgrad3" : w.v2 == 2 ? "wgrad8" : w.v2 == 1 ? "wgrad2" : "wgrad";
      fprintf(stderr, "wgrad %-8s %-7s KB %5d M %5d N %4d slabs %7.2f MB grid %d x %d x %d\n", n.c_str(), k,
              w.KB, w.Mtot, w.Ntot, 4e-6 * w.KB * (double)w.Mtot * w.Ntot, w.KB, w.mchunks, w.nchunks);
    };
    for (const auto *v : {&p.dc1, &p.dc2, &p.uc1, &p.uc2})
      for (const ConvLayer &cl : *v) wlog(cl.name, cl.wg);
    for (const ConvTLayer &u : p.up) wlog(u.name, u.wg_phase ? u.wgp : u.wg);
  }
  return 0;
}

struct Ctx {
  const hcu_unet_plan &p;
  const hcu_unet_tensors &t;
  hipStream_t s;
  char *sv, *sc;
  const float *P;
  float *G;
  // Backward only: the weight-gradient branch runs on `ws` (== s when not
  // split).  It reads gradient slots the main chain has finished and writes
  // only its own partials (wpart) and the parameter gradients, so the one
  // hazard is the main chain reusing a slot the branch has not read yet.
  hipStream_t ws = nullptr;
  bool split = false;
  int next_slot = 0;
  unsigned slot_read = 0;   // slots whose last reader event was recorded in this enqueue
  float *fptr(char *base, size_t off) const { return reinterpret_cast<float *>(base + off); }
  // Base of the packed weight images (offsets wf_off / wd_off / wph_off): the
  // saved workspace, or a layer chain's caller-owned image buffer
  // (hcu_chain_forward_images), which then starts at plan offset img_lo.
  char *wi = nullptr;
  char *wimg() const { return wi ? wi : sv; }
  int bf() const { return p.es == 2; }   // bf16 activation storage
  float *part() const { return fptr(sc, p.part_off); }
  float *wpart() const { return fptr(sc, split ? p.wpart_off : p.part_off); }
  // Weight-gradient slab arena: each layer's partial slabs stay until its
  // finalize runs; finalizes are deferred and launched together (one batched
  // kernel on the branch stream) when the next slab would not fit, and at the
  // end of the backward.  Nothing else reads or writes the arena.
  size_t wp_off = 0;
  std::vector<WGradFinalize> pend;
  // HCU_WGF_DEFER=0: finalize each layer right after its weight gradient (A/B)
  static bool defer_wgf() {
    static const bool on = !(getenv("HCU_WGF_DEFER") && getenv("HCU_WGF_DEFER")[0] == '0');
    return on;
  }
  int pend_wgf(const WGradFinalize &f) {
    pend.push_back(f);
    return defer_wgf() ? 0 : flush_wgf();
  }
  int flush_wgf() {
    int e = 0;
    // HCU_DEBUG_NO_WGF=1 drops every weight-gradient finalize: WRONG gradients,
    // a timing probe only (what the finalizes cost a step)
    static const bool no_wgf = getenv("HCU_DEBUG_NO_WGF") && getenv("HCU_DEBUG_NO_WGF")[0] == '1';
    if (!pend.empty() && !no_wgf) e = launch_wgrad_finalize_batch(pend.data(), (int)pend.size(), wstream());
    pend.clear();
    wp_off = 0;
    return e;
  }
  // Arena space for `floats` (flushing the deferred finalizes first if needed).
  int slab(size_t floats, float *&ptr) {
    const size_t need = (floats + 63) / 64 * 64;
    if (wp_off + need > p.wpart_floats || pend.size() >= 64)
      if (int e = flush_wgf()) return e;
    ptr = fptr(sc, p.wpart_off) + wp_off;
    wp_off += need;
    return 0;
  }
  float *wprep() const { return fptr(sc, p.wprep_off); }
  float *buf(int i) const { return fptr(sc, p.buf_off[i]); }
  float *kpart() const { return fptr(sc, p.kpart_off); }
  hipStream_t wstream() const { return split ? ws : s; }
  // Fresh slot for the main chain to write; waits for the branch's last read of it.
  int alloc(int &slot) {
    slot = next_slot;
    next_slot = (next_slot + 1) % p.nbuf;
    if (split && (slot_read & (1u << slot))) HCU_HIP(hipStreamWaitEvent(s, p.ev_slot[slot], 0));
    return HCU_OK;
  }
  // Branch work issued from here on sees everything the main chain has issued.
  int fork() {
    if (!split) return HCU_OK;
    const ChainRec &r = chain_rec();
    if (r.ev == p.ev_chain && r.s == s && r.n > chain_n0) {
      // the chain's last kernel carries ev_chain as its stop event (HCU_LAUNCH)
      HCU_HIP(hipStreamWaitEvent(ws, p.ev_chain, 0));
      return HCU_OK;
    }
    // a ring of marker events: re-recording an event whose previous record the
    // GPU has not reached yet stalls the host (config 3: ~0.9 ms per step)
    hipEvent_t ev = p.ev_fork_ring[p.fork_next++ % HCU_FORK_RING];
    HCU_HIP(hipEventRecord(ev, s));
    HCU_HIP(hipStreamWaitEvent(ws, ev, 0));
    return HCU_OK;
  }
  // Arms the chain record (backward): kernels launched on s from here on
  // carry ev_chain, so forks need no marker; disarmed by the destructor.
  unsigned long chain_n0 = 0;
  bool armed = false;
  void arm_chain() {
    if (!split || !p.ev_chain) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;   // captured graphs keep their markers
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
      (void)hipGetLastError();
      return;
    }
    ChainRec &r = chain_rec();
    r.s = s;
    r.ev = p.ev_chain;
    chain_n0 = r.n;
    armed = true;
  }
  ~Ctx() {
    if (armed) chain_rec().ev = nullptr;
  }
  // The branch work issued so far is the last reader of `slot`.
  int read_done(int slot) {
    if (!split || slot < 0 || p.no_reuse) return HCU_OK;   // no_reuse: never rewritten
    HCU_HIP(hipEventRecord(p.ev_slot[slot], ws));
    slot_read |= 1u << slot;
    return HCU_OK;
  }
  int join() {
    if (!split) return HCU_OK;
    hipEvent_t ev = p.ev_fork_ring[p.fork_next++ % HCU_FORK_RING];
    HCU_HIP(hipEventRecord(ev, ws));
    HCU_HIP(hipStreamWaitEvent(s, ev, 0));
    return HCU_OK;
  }
};

void tag(const std::string &layer, const char *phase) {
  if (timing_on()) timing_set_tag((layer + "." + phase).c_str());
}

// in_fmt > 0 (the first layer, hcu_unet_plan::ncx_first): `in` is the
// caller's NCXYZ input volume, read by the conv's own halo staging, which also
// writes the channels-last copy xcl_out (when not null).
int conv_forward(const Ctx &c, const ConvLayer &L, const float *in, const float *isc,
                 const float *ish, int training, int in_fmt = 0, float *xcl_out = nullptr) {
  HCU_HIP(hipGetLastError());
  tag(L.name, "fwd");
  GConvArgs a = L.fwd;
  a.in = in;
  a.in_fmt = in_fmt;
  a.in_c = in_fmt ? L.in.C : 0;
  a.xcl = xcl_out;
  if (in_fmt) a.w = c.P + L.w_off;   // (read in the PyTorch layout by the NCXYZ staging)
  a.in_scale = isc;
  a.in_shift = ish;
  if (!in_fmt) a.w = c.fptr(c.wimg(), L.wf_off);
  a.bias = L.b_off >= 0 ? c.P + L.b_off : nullptr;
  a.out = c.fptr(c.sv, L.y_off);
  a.stats = training ? c.part() : nullptr;
  a.partial = c.kpart();
  const BNCoef coef = coef_at(c.sv, L.bn);
  if (int e = launch_conv_any(a, c.s)) return e;
  return launch_bn_fwd_finalize(c.part(), gconv_rows(L.fwd), L.fwd.CoutW, L.bn.C, L.bn.Cs,
                                L.bn.count, c.P + L.bn.gamma, c.P + L.bn.beta,
                                c.t.bn_running_mean[L.bn.index], c.t.bn_running_var[L.bn.index],
                                c.t.bn_num_batches_tracked[L.bn.index], c.p.spec.bn_eps,
                                c.p.spec.bn_momentum, training, coef, c.s);
}

// Sets up the dgrad epilogue that also performs the BatchNorm+ReLU backward
// reduction of layer `bnl` (whose output the gradient is for); false when the
// planned kernel cannot.
bool fuse_bnbwd(Ctx &c, GConvArgs &a, const ConvLayer *bnl) {
  static const bool off = getenv("HCU_NO_BNFUSE") != nullptr;   // A/B debugging
  if (off || !bnl || !conv_bnbwd_fusable(a)) return false;
  const BNCoef coef = coef_at(c.sv, bnl->bn);
  a.bn_y = c.fptr(c.sv, bnl->y_off);
  a.bn_scale = coef.scale;
  a.bn_shift = coef.shift;
  a.bn_mean = coef.mean;
  a.bn_invstd = coef.invstd;
  a.stats = c.part();
  return true;
}

// Finalize and apply of a BatchNorm backward whose reduction rows are in
// c.part(): dz -> dY of bnl in place.
int finish_bn(const Ctx &c, const ConvLayer &bnl, int R, int W, float *dz, int training, int accumulate) {
  const BNCoef coef = coef_at(c.sv, bnl.bn);
  if (int e = launch_bn_bwd_finalize(c.part(), R, bnl.bn.C, bnl.bn.Cs, W, bnl.bn.count, coef,
                                     c.G + bnl.bn.gamma, c.G + bnl.bn.beta, training, accumulate, c.s))
    return e;
  return launch_bn_bwd_apply(dz, c.fptr(c.sv, bnl.y_off), coef, bnl.out.vox(), bnl.out.Cs, c.s, c.bf());
}

int finish_bnbwd(const Ctx &c, const GConvArgs &a, const ConvLayer &bnl, float *dz, int training,
                 int accumulate) {
  return finish_bn(c, bnl, gconv_rows(a), a.CoutW, dz, training, accumulate);
}

// Weight/bias gradient and (optionally) input gradient of one Conv3d layer.
// dy holds dY of L.  With `bnl`, the input gradient leaves as dz of layer bnl
// (its BatchNorm+ReLU backward fused into the dgrad) and *bn_done is set.
// With `colsum` (and no bnl) the input gradient's kernel also writes its
// per-workgroup statistics rows there (gconv_rows x CoutW of {S1, S2, K, n}):
// the column sums of dA, finalized as the bias gradient of the layer that
// produced A (a ConvTranspose3d: no separate reduction pass over dA).
int conv_backward(Ctx &c, const ConvLayer &L, const float *A, const float *asc,
                  const float *ash, const float *dy, int dy_slot, float *dA, int accumulate,
                  const ConvLayer *bnl = nullptr, int training = 1, bool *bn_done = nullptr,
                  float *colsum = nullptr, bool wg_late = false);

// The weight-gradient half of conv_backward (forked onto the branch).
int conv_wgrad(Ctx &c, const ConvLayer &L, const float *A, const float *asc, const float *ash,
               const float *dy, int dy_slot, int accumulate) {
  tag(L.name, "wgrad");
  if (int e = c.fork()) return e;
  WGradArgs w = L.wg;
  w.A = A;
  w.a_scale = asc;
  w.a_shift = ash;
  w.G = dy;
  if (L.pw_wg && !asc) {   // 1x1x1 without a BatchNorm input: the VALU form (pwconv.hip)
    const long nvox = L.out.vox();
    w.KB = pw_wgrad_blocks(nvox);
    if (int e = c.slab(wgrad_partial_floats(w), w.partial)) return e;
    PwWgArgs pa{};
    pa.A = reinterpret_cast<const uint16_t *>(A);
    pa.G = reinterpret_cast<const uint16_t *>(dy);
    pa.partial = w.partial;
    pa.nvox = nvox;
    pa.per_block = (nvox + w.KB - 1) / w.KB;
    pa.ACs = w.ACs;
    pa.GCs = w.GCs;
    pa.ACR = w.ACr > 0 ? w.ACr : w.ACs;
    pa.GCR = w.GCr > 0 ? w.GCr : w.GCs;
    pa.Mtot = w.Mtot;
    pa.Ntot = w.Ntot;
    pa.bias_row = w.bias_row;
    if (int e = launch_pw_wgrad(pa, w.KB, c.wstream())) return e;
  } else {
    if (int e = c.slab(wgrad_partial_floats(w), w.partial)) return e;
    if (int e = launch_wgrad(w, c.wstream())) return e;
  }
  WGradFinalize f{};
  f.partial = w.partial;
  f.dw = c.G + L.w_off;
  f.db = L.b_off >= 0 ? c.G + L.b_off : nullptr;
  f.KB = w.KB;
  f.Mtot = w.Mtot;
  f.Ntot = w.Ntot;
  f.T = L.T;
  f.mode = 0;
  f.Cout = L.Cout;
  f.Cin_g = L.Cin_g;
  f.groups = L.groups;
  f.fold_mod = L.fold_mod;
  f.part_c = L.part_c;
  f.part_cs = L.part_cs;
  f.ACs = wgrad_slab_acs(w);
  f.accumulate = accumulate;
  if (int e = c.pend_wgf(f)) return e;   // finalized with the next flush (Ctx::slab / end of backward)
  return c.read_done(dy_slot);
}

// wg_late: the weight gradient is forked after the input gradient's
// convolution is enqueued (and before its BatchNorm finalize), so the
// branch's kernel does not start beside it (HCU_L0_ORDER, level 0 A/B).
int conv_backward(Ctx &c, const ConvLayer &L, const float *A, const float *asc,
                  const float *ash, const float *dy, int dy_slot, float *dA, int accumulate,
                  const ConvLayer *bnl, int training, bool *bn_done, float *colsum, bool wg_late) {
  if (!wg_late || !dA)
    if (int e = conv_wgrad(c, L, A, asc, ash, dy, dy_slot, accumulate)) return e;
  if (!dA) return 0;
  tag(L.name, "dgrad");
  if (L.pw && !bnl && !colsum) {   // (the chains' non-BatchNorm 1x1x1 convolutions)
    PwArgs w{};
    w.in = reinterpret_cast<const uint16_t *>(dy);
    w.w = c.P + L.w_off;
    w.out = reinterpret_cast<uint16_t *>(dA);
    w.nvox = L.out.vox();
    w.ICs = L.out.Cs;
    w.OCs = L.in.Cs;
    w.Cin = L.Cin_g;
    w.Cout = L.Cout;
    w.part_c = L.part_c;
    w.part_cs = L.part_cs;
    w.dgrad = 1;
    return launch_pw(w, c.s);
  }
  GConvArgs a = L.dgrad;
  a.in = dy;
  a.w = c.fptr(c.wimg(), L.wd_off);
  a.out = dA;
  a.partial = c.kpart();
  const bool fused = fuse_bnbwd(c, a, bnl);
  if (!fused && colsum) a.stats = colsum;
  if (int e = launch_conv_any(a, c.s)) return e;
  if (wg_late)
    if (int e = conv_wgrad(c, L, A, asc, ash, dy, dy_slot, accumulate)) return e;
  if (!fused) return 0;
  tag(bnl->name, "bnbwd");
  if (int e = finish_bnbwd(c, a, *bnl, dA, training, accumulate)) return e;
  if (bn_done) *bn_done = true;
  return 0;
}

// BatchNorm+ReLU backward for layer L: dbuf holds d(post-activation) on entry
// and dz (Ctx::ap(L)) or d(pre-BN y) on exit (unless pool_dP is given, in
// which case dbuf is produced from the max-pool gradient).
int bn_backward(const Ctx &c, const ConvLayer &L, float *dbuf, const float *pool_dP,
                const int *pool_k, int training, int accumulate) {
  tag(L.name, "bnbwd");
  const BNCoef coef = coef_at(c.sv, L.bn);
  const float *y = c.fptr(c.sv, L.y_off);
  const int64_t nvox = L.out.vox();
  const int R = bwd_rows(nvox, L.out.Cs);
  if (pool_dP) {
    if (int e = launch_bn_bwd_reduce_pool(pool_dP, y, coef, dbuf, L.out.B, L.out.X, L.out.Y,
                                          L.out.Z, L.out.Cs, pool_k[0], pool_k[1], pool_k[2],
                                          c.part(), R, c.s, c.bf()))
      return e;
  } else {
    if (int e = launch_bn_bwd_reduce_dense(dbuf, y, coef, nvox, L.out.Cs, c.part(), R, c.s,
                                           c.bf()))
      return e;
  }
  return finish_bn(c, L, R, L.bn.Cs, dbuf, training, accumulate);
}

}  // namespace

namespace {

// hipGraph replay of the captured sequences vs direct launches.  On MI355X /
// ROCm 7 a replayed kernel node costs ~1.5 us more on the GPU than a direct
// launch (config 3: 7.24 vs 7.10 ms per step), but a direct launch costs the
// host ~10 us: at config 2 (2.3 ms of GPU work, 1.7 ms of host enqueue) direct
// launches ran 2.31..3.34 ms per step depending on host jitter, graphs a
// steady 2.51..2.58.  So: graphs for the forward of plans under 100 GFLOP,
// direct launches otherwise; HCU_GRAPHS=0 / 1 forces either everywhere.
int graphs_forced() {
  static const int v = [] {
    const char *e = getenv("HCU_GRAPHS");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  return v;
}
// The backward (two streams joined by events) replays slower still: a graph
// of it cost 0.17 ms per config-2 step against direct launches (forward-only
// graph 2.39 ms/step vs both graphed 2.56, three interleaved A/B runs), so by
// default only a small plan's forward is replayed.
bool graphs_for(const hcu_unet_plan &p, bool backward) {
  const int f = graphs_forced();
  if (f >= 0) return f == 1;
  return !backward && p.fwd_flops < 100e9;
}

void append_bn_key(std::vector<uintptr_t> &key, const hcu_unet_plan &p, const hcu_unet_tensors *t) {
  for (int i = 0; i < p.n_bn; ++i) {
    key.push_back(t->bn_running_mean ? (uintptr_t)t->bn_running_mean[i] : 0);
    key.push_back(t->bn_running_var ? (uintptr_t)t->bn_running_var[i] : 0);
    key.push_back(t->bn_num_batches_tracked ? (uintptr_t)t->bn_num_batches_tracked[i] : 0);
  }
}

// Replays the captured launch sequence for `key`, capturing it on first use
// (on a private stream, so nothing runs during capture) and keeping the 8
// most recently used sequences.  Falls back to direct launches when graphs
// are off or per-launch timing is on.
template <class F>
int run_graphed(const hcu_unet_plan &p, std::vector<uintptr_t> key, hipStream_t s, F enqueue) {
  if (!graphs_for(p, key[0] != 0) || timing_on()) return enqueue(s);
  int dev = 0;
  HCU_HIP(hipGetDevice(&dev));
  key.push_back((uintptr_t)dev);
  std::lock_guard<std::mutex> lk(p.gmu);
  for (auto &g : p.graphs)
    if (g.key == key) {
      g.used = ++p.gclock;
      HCU_HIP(hipGraphLaunch(g.exec, s));
      return HCU_OK;
    }
  if (!p.cap_stream || p.cap_device != dev) {
    if (p.cap_stream) (void)hipStreamDestroy(p.cap_stream);
    p.cap_stream = nullptr;
    HCU_HIP(hipStreamCreateWithFlags(&p.cap_stream, hipStreamNonBlocking));
    p.cap_device = dev;
  }
  HCU_HIP(hipStreamBeginCapture(p.cap_stream, hipStreamCaptureModeThreadLocal));
  const int e = enqueue(p.cap_stream);
  hipGraph_t graph = nullptr;
  const hipError_t ce = hipStreamEndCapture(p.cap_stream, &graph);
  if (e || ce != hipSuccess) {
    if (graph) (void)hipGraphDestroy(graph);
    // A failure after the backward forked its weight-gradient branch leaves
    // the branch stream in an invalidated capture: recreate it on next use.
    p.destroy_side();
    if (e) return e;
    return fail(HCU_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
  }
  hipGraphExec_t exec = nullptr;
  const hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ie != hipSuccess)
    return fail(HCU_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
  if (p.graphs.size() >= 8) {
    auto lru = std::min_element(p.graphs.begin(), p.graphs.end(),
                                [](const auto &a, const auto &b) { return a.used < b.used; });
    (void)hipGraphExecDestroy(lru->exec);
    p.graphs.erase(lru);
  }
  p.graphs.push_back({key, exec, ++p.gclock});
  HCU_HIP(hipGraphLaunch(exec, s));
  return HCU_OK;
}

}  // namespace

extern "C" {

const char *hcu_last_error(void) { return g_err.c_str(); }
int hcu_version(void) { return 100; }

int hcu_unet_plan_create(const hcu_unet_spec *spec, int B, int X, int Y, int Z,
                         hcu_unet_plan **out) {
  return hcu_unet_plan_create_ex(spec, B, X, Y, Z, 0, out);
}

int hcu_unet_plan_create_ex(const hcu_unet_spec *spec, int B, int X, int Y, int Z, int flags,
                            hcu_unet_plan **out) {
  if (!spec || !out) return fail(HCU_ERR_INVALID, "null argument");
  if (flags & ~HCU_PLAN_FORWARD_ONLY) return fail(HCU_ERR_INVALID, "unknown plan flags");
  auto *p = new hcu_unet_plan();
  p->flags = flags;
  p->spec = *spec;
  p->B = B;
  p->X = X;
  p->Y = Y;
  p->Z = Z;
  bconv_tuning((flags & HCU_PLAN_FORWARD_ONLY) == 0);
  const int e = build_plan(*p);
  bconv_tuning(true);
  if (e) {
    delete p;
    *out = nullptr;
    return e;
  }
  *out = p;
  return HCU_OK;
}

void hcu_unet_plan_destroy(hcu_unet_plan *plan) { delete plan; }

int hcu_unet_plan_query(const hcu_unet_plan *p, int64_t *out_shape, int64_t *n_params, int *n_bn,
                        size_t *saved_bytes, size_t *scratch_bytes) {
  if (!p) return fail(HCU_ERR_INVALID, "null plan");
  if (out_shape) {
    out_shape[0] = p->B;
    out_shape[1] = p->Co;
    out_shape[2] = p->outd.X;
    out_shape[3] = p->outd.Y;
    out_shape[4] = p->outd.Z;
  }
  if (n_params) *n_params = p->n_params;
  if (n_bn) *n_bn = p->n_bn;
  if (saved_bytes) *saved_bytes = p->saved_bytes;
  if (scratch_bytes) *scratch_bytes = p->scratch_bytes;
  return HCU_OK;
}

int hcu_unet_set_grad_events(hcu_unet_plan *p, void *ev_decoder, void *ev_deep, int deep_level) {
  if (!p || p->is_chain) return fail(HCU_ERR_INVALID, "hcu_unet_set_grad_events: U-Net plan required");
  if (ev_deep && (deep_level < 1 || deep_level >= p->L))
    return fail(HCU_ERR_INVALID, "hcu_unet_set_grad_events: deep_level must be in [1, levels)");
  std::lock_guard<std::mutex> lk(p->smu);   // enqueue_backward reads them under the same lock
  p->grad_ev[0] = (hipEvent_t)ev_decoder;
  p->grad_ev[1] = (hipEvent_t)ev_deep;
  p->grad_deep = ev_deep ? deep_level : -1;
  return HCU_OK;
}

// 1 when hcu_unet_backward records the events set by hcu_unet_set_grad_events
// (a direct-launch backward), 0 when it does not (a backward replayed from a
// captured graph: the caller must then reduce after the whole backward).
int hcu_unet_grad_events_live(const hcu_unet_plan *p) {
  if (!p || p->is_chain) return 0;
  return (graphs_for(*p, true) && !timing_on()) ? 0 : 1;
}

int hcu_event_create(void **ev) {
  if (!ev) return fail(HCU_ERR_INVALID, "null argument");
  hipEvent_t e = nullptr;
  HCU_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *ev = e;
  return HCU_OK;
}

int hcu_event_destroy(void *ev) {
  if (ev) HCU_HIP(hipEventDestroy((hipEvent_t)ev));
  return HCU_OK;
}

int hcu_stream_wait_event(hcu_stream_t stream, void *ev) {
  if (!ev) return fail(HCU_ERR_INVALID, "null event");
  HCU_HIP(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0));
  return HCU_OK;
}

int hcu_unet_plan_bn_layers(const hcu_unet_plan *p, hcu_bn_layer_info *out, int max) {
  if (!p) return -fail(HCU_ERR_INVALID, "null plan");
  std::vector<const ConvLayer *> ls(p->n_bn, nullptr);
  for (const auto *v : {&p->dc1, &p->dc2, &p->uc1, &p->uc2})
    for (const ConvLayer &L : *v) ls[L.bn.index] = &L;
  for (int i = 0; i < p->n_bn && i < max && out; ++i) {
    const ConvLayer &L = *ls[i];
    hcu_bn_layer_info r{};
    r.y_offset = (int64_t)L.y_off;
    r.coef_offset = (int64_t)L.bn.coef_off;
    r.B = L.out.B;
    r.X = L.out.X;
    r.Y = L.out.Y;
    r.Z = L.out.Z;
    r.C = L.out.C;
    r.Cs = L.out.Cs;
    r.elem_bytes = L.out.es;
    out[i] = r;
  }
  return p->n_bn;
}

int ensure_side(const hcu_unet_plan &p, int dev);
bool side_enabled();

// part: 0 = the whole forward; 1 = its head (the input's channels-last
// layout, or with ncx_first the first convolution reading the NCXYZ input
// itself, and its BatchNorm finalize): the launches that read t->x, issued
// directly ahead of a replayed graph of part 2 = the rest, so a new input
// tensor every step (a data loader) does not key a new graph.
static int enqueue_forward(const hcu_unet_plan &p, const hcu_unet_tensors *t, int training,
                           hipStream_t stream, int part = 0, bool split = false) {
  Ctx c{p, *t, (hipStream_t)stream, (char *)t->saved, (char *)t->scratch, t->params, t->grads};
  c.split = split;
  c.ws = split ? p.side : c.s;
  const hcu_unet_spec &s = p.spec;
  float *xcl = c.fptr(c.sv, p.xcl_off);
  if (part != 2) {
    tag(std::string("in"), "fwd");
    if (!p.ncx_first) {
      if (int e = launch_to_cl(t->x, xcl, p.B, p.xin.C, p.xin.Cs, p.xin.vox() / p.B, c.s, c.bf(),
                               t->x_dtype))
        return e;
    } else {
      // NCXYZ input staged by the first conv; the channels-last copy only
      // where a backward will read it
      const int fmt = t->x_dtype == HCU_F16 ? 2 : t->x_dtype == HCU_BF16 ? 3 : 1;
      float *xo = (p.flags & HCU_PLAN_FORWARD_ONLY) ? nullptr : xcl;
      if (int e = conv_forward(c, p.dc1[0], t->x, nullptr, nullptr, training, fmt, xo)) return e;
    }
    if (part == 1) return HCU_OK;
  }
  tag(std::string("prep"), "fwd");
  // training forwards lay out the input-gradient weight images too; laying
  // them out on the backward's branch instead measured equal on config 3 and
  // ~10 us slower on config 2.  A split forward (hcu_unet_forward) lays out
  // level 0's forward images on the chain and every other image on the
  // branch, which the chain waits for only before level 1.
  const size_t n0 = std::min<size_t>(2, p.prep_fwd.size());   // d0.c1, d0.c2 (job order)
  hipEvent_t ev_rest = nullptr;
  if (split && training) {
    if (int e = c.fork()) return e;
    if (p.prep_fwd.size() > n0) {
      if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), p.prep_fwd.data() + n0,
                                  (int)(p.prep_fwd.size() - n0), c.ws))
        return e;
      ev_rest = p.ev_fork_ring[p.fork_next++ % HCU_FORK_RING];
      HCU_HIP(hipEventRecord(ev_rest, c.ws));
    }
    if (!p.prep_bwd.empty())
      if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), p.prep_bwd.data(),
                                  (int)p.prep_bwd.size(), c.ws))
        return e;
    if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), p.prep_fwd.data(), (int)n0, c.s))
      return e;
  } else {
    if (training && !p.prep_bwd.empty()) {
      if (int e = c.fork()) return e;
      if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), p.prep_bwd.data(),
                                  (int)p.prep_bwd.size(), c.wstream()))
        return e;
    }
    if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), p.prep_fwd.data(),
                                (int)p.prep_fwd.size(), c.s))
      return e;
  }
  const float *src = xcl;
  const float *ssc = nullptr, *ssh = nullptr;
  for (int i = 0; i < p.L; ++i) {
    const ConvLayer &c1 = p.dc1[i], &c2 = p.dc2[i];
    if (i == 1 && ev_rest) HCU_HIP(hipStreamWaitEvent(c.s, ev_rest, 0));
    if (!(i == 0 && p.ncx_first))   // (else: run in the head)
      if (int e = conv_forward(c, c1, src, ssc, ssh, training)) return e;
    const BNCoef b1 = coef_at(c.sv, c1.bn);
    if (int e = conv_forward(c, c2, c.fptr(c.sv, c1.y_off), b1.scale, b1.shift, training)) return e;
    const BNCoef b2 = coef_at(c.sv, c2.bn);
    if (i < p.L - 1) {
      float *pp = c.fptr(c.sv, p.pool_off[i]);
      tag(c2.name, "pool");
      if (int e = launch_maxpool_fwd(c.fptr(c.sv, c2.y_off), b2.scale, b2.shift, pp, p.B,
                                     c2.out.X, c2.out.Y, c2.out.Z, c2.out.Cs, s.pool_k[0],
                                     s.pool_k[1], s.pool_k[2], c.s, c.bf()))
        return e;
      src = pp;
      ssc = ssh = nullptr;
    } else {
      src = c.fptr(c.sv, c2.y_off);
      ssc = b2.scale;
      ssh = b2.shift;
    }
  }
  for (int j = 0; j < p.L - 1; ++j) {
    const ConvTLayer &u = p.up[j];
    tag(u.name, "fwd");
    float *U = c.fptr(c.sv, u.u_off);
    if (u.fused) {
      GConvArgs a = u.fwdf;
      a.in = src;
      a.in_scale = ssc;
      a.in_shift = ssh;
      a.w = c.fptr(c.wimg(), u.wf_off);
      a.bias = c.P + u.b_off;
      a.out = U;
      a.stats = nullptr;
      a.partial = c.kpart();
      if (int e = launch_conv_any(a, c.s)) return e;
    }
    for (size_t ph = 0; !u.fused && ph < u.phases.size(); ++ph) {
      GConvArgs a = u.phases[ph];
      a.in = src;
      a.in_scale = ssc;
      a.in_shift = ssh;
      a.w = c.fptr(c.wimg(), u.wph_off[ph]);
      a.bias = c.P + u.b_off;
      a.out = U;
      a.stats = nullptr;
      if (int e = launch_gconv(a, c.s)) return e;
    }
    const ConvLayer &c1 = p.uc1[j], &c2 = p.uc2[j];
    if (int e = conv_forward(c, c1, U, nullptr, nullptr, training)) return e;
    const BNCoef b1 = coef_at(c.sv, c1.bn);
    if (int e = conv_forward(c, c2, c.fptr(c.sv, c1.y_off), b1.scale, b1.shift, training)) return e;
    const BNCoef b2 = coef_at(c.sv, c2.bn);
    src = c.fptr(c.sv, c2.y_off);
    ssc = b2.scale;
    ssh = b2.shift;
  }
  const ConvLayer &last = p.L > 1 ? p.uc2[p.L - 2] : p.dc2[0];
  tag(std::string("out"), "fwd");
  if (int e = launch_outconv_fwd(src, coef_at(c.sv, last.bn), c.P + p.oc_w, c.P + p.oc_b, t->out,
                                 p.B, last.out.vox() / p.B, last.out.C, last.out.Cs, p.Co, c.s,
                                 c.bf()))
    return e;
  if (training && t->bn_num_batches_tracked)
    if (int e = launch_bn_count_increment(t->bn_num_batches_tracked, p.n_bn, c.s)) return e;
  if (int e = c.join()) return e;
  if (timing_on()) timing_set_tag("");
  return HCU_OK;
}

static int unet_forward_impl(const hcu_unet_plan *plan, const hcu_unet_tensors *t, int training,
                             hcu_stream_t stream);
int hcu_unet_forward(const hcu_unet_plan *plan, const hcu_unet_tensors *t, int training,
                     hcu_stream_t stream) {
  const double t0 = host_prof_on() ? host_now_us() : 0.0;
  double su[2];
  long sn[2];
  if (host_prof_on()) host_prof_snap(su, sn);
  const int rc = unet_forward_impl(plan, t, training, stream);
  if (host_prof_on()) {
    const double dt = host_now_us() - t0;
    host_prof_add(2, dt);
    host_prof_call(0, su, sn, dt);
  }
  return rc;
}

static int unet_forward_impl(const hcu_unet_plan *plan, const hcu_unet_tensors *t, int training,
                             hcu_stream_t stream) {
  if (!plan || !t || !t->x || !t->out || !t->params || !t->saved || !t->scratch)
    return fail(HCU_ERR_INVALID, "null argument");
  const hcu_unet_plan &p = *plan;
  if (t->x_dtype != HCU_F32 && t->x_dtype != HCU_F16 &&
      !(t->x_dtype == HCU_BF16 && p.es == 2))
    return fail(HCU_ERR_INVALID, "unsupported input dtype for this plan");
  if (training) {
    for (const auto *v : {&p.dc1, &p.dc2, &p.uc1, &p.uc2})
      for (const ConvLayer &L : *v)
        if (L.bn.count <= 1.0)
          return fail(HCU_ERR_INVALID, "Expected more than 1 value per channel when training");
  }
  // The input layout change runs ahead of the captured sequence, so a fresh
  // input tensor every step (a data loader) does not key a new graph.
  // Large parameter sets lay out their deeper weight images on the branch
  // stream while level 0 runs (Ctx in enqueue_forward).  Interleaved A/B, 3
  // runs: config 3 (11.6 M parameters) 6.418-6.434 vs 6.448-6.453 ms/step;
  // config 2 (0.7 M, ~23 us of re-layout) 2.103-2.129 vs 2.058-2.071: there
  // the branch's kernels slow level 0 more than the overlap returns.
  // (HCU_SPLIT_FWD_PARAMS: the parameter count from which the split applies;
  // tests lower it to run the split on a small network)
  static const int64_t split_min = getenv("HCU_SPLIT_FWD_PARAMS") ? atoll(getenv("HCU_SPLIT_FWD_PARAMS"))
                                                                  : (int64_t)4 << 20;
  const bool split = p.n_params >= split_min && training && side_enabled() && !timing_on() &&
                     p.prep_fwd.size() > 2;
  std::unique_lock<std::mutex> lk(p.smu, std::defer_lock);
  if (split) {
    lk.lock();
    int dev = 0;
    HCU_HIP(hipGetDevice(&dev));
    if (int e = ensure_side(p, dev)) return e;
  }
  if (graphs_for(p, false) && !timing_on()) {
    if (int e = enqueue_forward(p, t, training, (hipStream_t)stream, 1, split)) return e;
    std::vector<uintptr_t> key = {0, (uintptr_t)t->out, (uintptr_t)t->params, (uintptr_t)t->saved,
                                  (uintptr_t)t->scratch, (uintptr_t)training, (uintptr_t)split};
    append_bn_key(key, p, t);
    return run_graphed(p, key, (hipStream_t)stream,
                       [&](hipStream_t s) { return enqueue_forward(p, t, training, s, 2, split); });
  }
  return enqueue_forward(p, t, training, (hipStream_t)stream, 0, split);
}

static int enqueue_backward(const hcu_unet_plan &p, const hcu_unet_tensors *t, const float *dout,
                            float *dx, int training, int accumulate, hipStream_t stream,
                            bool split, bool record_grad_events) {
  const hcu_unet_spec &s = p.spec;
  Ctx c{p, *t, (hipStream_t)stream, (char *)t->saved, (char *)t->scratch, t->params, t->grads};
  c.split = split;
  c.ws = split ? p.side : c.s;
  c.arm_chain();
  // an eval-mode forward prepared only the forward weight images: the
  // input-gradient images are laid out here
  if (!training && !p.prep_bwd.empty())
    if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), p.prep_bwd.data(), (int)p.prep_bwd.size(),
                                c.s))
      return e;
  int cur = 0;  // slot holding the current d(pre-BN y) (or dz, Ctx::ap)
  if (int e = c.alloc(cur)) return e;

  // out_conv + last BatchNorm
  const ConvLayer &last = p.uc2[p.L - 2];
  tag(std::string("out"), "bwd");
  {
    const BNCoef coef = coef_at(c.sv, last.bn);
    const int64_t nvox = last.out.vox();
    const int R = outconv_bwd_rows(nvox, last.out.Cs);
    float *part_bn = c.part();
    float *part_oc = part_bn + (size_t)R * last.out.Cs * 2;
    if (int e = launch_outconv_bwd(dout, c.fptr(c.sv, last.y_off), coef, c.P + p.oc_w, c.buf(cur),
                                   p.B, nvox / p.B, last.out.C, last.out.Cs, p.Co, part_bn, part_oc,
                                   R, c.s, c.bf()))
      return e;
    if (int e = launch_outconv_wfinalize(part_oc, R, p.Co, last.out.C, last.out.Cs, c.G + p.oc_w,
                                         c.G + p.oc_b, accumulate, c.s))
      return e;
    if (int e = finish_bn(c, last, R, last.bn.Cs, c.buf(cur), training, accumulate)) return e;
  }
  // decoder, last to first
  for (int j = p.L - 2; j >= 0; --j) {
    const ConvLayer &c1 = p.uc1[j], &c2 = p.uc2[j];
    const ConvTLayer &u = p.up[j];
    const BNCoef b1 = coef_at(c.sv, c1.bn);
    const float *U = c.fptr(c.sv, u.u_off);
    int sb = 0, su = 0, sd = 0;
    // conv2 (+ BatchNorm/ReLU backward of conv1, fused into its dgrad when possible)
    if (int e = c.alloc(sb)) return e;
    float *A = c.buf(cur), *Bf = c.buf(sb);
    bool done1 = false;
    if (int e = conv_backward(c, c2, c.fptr(c.sv, c1.y_off), b1.scale, b1.shift, A, cur, Bf,
                              accumulate, &c1, training, &done1))
      return e;
    if (!done1)
      if (int e = bn_backward(c, c1, Bf, nullptr, nullptr, training, accumulate)) return e;
    // conv1 (folded cat): dU into a fresh slot; its input-gradient kernel also
    // writes the column-sum rows of dU, the up_conv bias gradient
    if (int e = c.alloc(su)) return e;
    float *dU = c.buf(su);
    const int cs_rows = gconv_rows(c1.dgrad), cs_w = c1.dgrad.CoutW;
    // (its own scratch region per level: written by the chain, read by the
    // deferred finalize on the branch -- never a recycled slab of the arena,
    // whose previous readers run on the branch)
    float *csr = c.fptr(c.sc, p.colsum_off[j]);
    if (int e = conv_backward(c, c1, U, nullptr, nullptr, Bf, sb, dU, accumulate, nullptr, training, nullptr, csr))
      return e;
    // up_conv: bias and weight gradients on the branch, input gradient on the chain
    const ConvLayer &prev = j == 0 ? p.dc2[p.L - 1] : p.uc2[j - 1];
    const BNCoef bp = coef_at(c.sv, prev.bn);
    tag(u.name, "wgrad");
    if (int e = c.fork()) return e;
    {
      WGradFinalize fb{};   // the bias: column sums of dU, with the batched finalizes
      fb.partial = csr;
      fb.db = c.G + u.b_off;
      fb.KB = cs_rows;
      fb.Mtot = 1;
      fb.Ntot = cs_w;
      fb.mode = 4;
      fb.Cout = u.Cout;
      fb.accumulate = accumulate;
      if (int e = c.pend_wgf(fb)) return e;
    }
    if (u.wg_phase) {   // the weight gradient in one launch (WGradArgs::nph, wgrad3)
      WGradArgs w = u.wgp;
      w.A = c.fptr(c.sv, prev.y_off);
      w.a_scale = bp.scale;
      w.a_shift = bp.shift;
      w.G = dU;
      if (int e = c.slab(wgrad_partial_floats(w), w.partial)) return e;
      if (int e = launch_wgrad(w, c.wstream())) return e;
      WGradFinalize f{};
      f.partial = w.partial;
      f.dw = c.G + u.w_off;
      f.db = nullptr;
      f.KB = w.KB;
      f.Mtot = w.Mtot;
      f.Ntot = w.Ntot;
      f.T = u.T;
      f.mode = 3;
      f.Cin = u.Cin;
      f.CoutT = u.Cout;
      f.ACs = w.ACs;
      f.GCs = w.GCs;
      for (int d = 0; d < 3; ++d) {
        f.J[d] = u.K[d] / u.S[d];
        f.SS[d] = u.S[d];
      }
      f.accumulate = accumulate;
      if (int e = c.pend_wgf(f)) return e;
    } else {
      WGradArgs w = u.wg;
      w.A = c.fptr(c.sv, prev.y_off);
      w.a_scale = bp.scale;
      w.a_shift = bp.shift;
      w.G = dU;
      if (int e = c.slab(wgrad_partial_floats(w), w.partial)) return e;
      if (int e = launch_wgrad(w, c.wstream())) return e;
      WGradFinalize f{};
      f.partial = w.partial;
      f.dw = c.G + u.w_off;
      f.db = nullptr;
      f.KB = w.KB;
      f.Mtot = w.Mtot;
      f.Ntot = w.Ntot;
      f.T = u.T;
      f.mode = 1;
      f.Cin = u.Cin;
      f.CoutT = u.Cout;
      f.GCs = w.GCs;
      f.accumulate = accumulate;
      if (int e = c.pend_wgf(f)) return e;
    }
    if (int e = c.read_done(su)) return e;
    tag(u.name, "dgrad");
    if (int e = c.alloc(sd)) return e;
    {
      float *dP = c.buf(sd);
      GConvArgs a = u.dgrad;
      a.in = dU;
      a.w = c.fptr(c.wimg(), u.wd_off);
      a.out = dP;
      a.partial = c.kpart();
      const bool fused = fuse_bnbwd(c, a, &prev);
      if (int e = launch_conv_any(a, c.s)) return e;
      if (fused) {
        tag(prev.name, "bnbwd");
        if (int e = finish_bnbwd(c, a, prev, dP, training, accumulate)) return e;
      } else if (int e = bn_backward(c, prev, dP, nullptr, nullptr, training, accumulate)) {
        return e;
      }
    }
    cur = sd;
  }
  // Data-parallel overlap: every gradient of a finished group is written by
  // the finalizes pending on the branch and by kernels the main chain issued
  // before this point; the branch flushes, joins the chain (fork) and records.
  // (not in a captured backward: a record inside stream capture is only a
  // capture dependency, a replay would never record the caller's events)
  auto grads_ready = [&](hipEvent_t ev) -> int {
    if (!ev || !record_grad_events) return 0;
    if (int e = c.flush_wgf()) return e;
    if (int e = c.fork()) return e;
    HCU_HIP(hipEventRecord(ev, c.wstream()));
    return 0;
  };
  if (int e = grads_ready(p.grad_ev[0])) return e;   // up_steps + out_conv
  // encoder, bottleneck to first
  for (int i = p.L - 1; i >= 0; --i) {
    const ConvLayer &c1 = p.dc1[i], &c2 = p.dc2[i];
    const BNCoef b1 = coef_at(c.sv, c1.bn);
    int sb = 0, sa = -1;
    if (int e = c.alloc(sb)) return e;
    float *A = c.buf(cur), *Bf = c.buf(sb);
    bool done1 = false;
    static const int l0_order = getenv("HCU_L0_ORDER") ? atoi(getenv("HCU_L0_ORDER")) : 0;
    if (int e = conv_backward(c, c2, c.fptr(c.sv, c1.y_off), b1.scale, b1.shift, A, cur, Bf,
                              accumulate, &c1, training, &done1, nullptr, i == 0 && l0_order == 1))
      return e;
    if (!done1)
      if (int e = bn_backward(c, c1, Bf, nullptr, nullptr, training, accumulate)) return e;
    const float *in = i == 0 ? c.fptr(c.sv, p.xcl_off) : c.fptr(c.sv, p.pool_off[i - 1]);
    float *dIn = nullptr;
    if (i > 0 || dx) {
      if (int e = c.alloc(sa)) return e;
      dIn = c.buf(sa);
    }
    if (int e = conv_backward(c, c1, in, nullptr, nullptr, Bf, sb, dIn, accumulate, nullptr, training))
      return e;
    if (i > 0) {
      // dIn = d(pooled): produce d(pre-BN y2_{i-1}) into a fresh slot
      int sp = 0;
      if (int e = c.alloc(sp)) return e;
      if (int e = bn_backward(c, p.dc2[i - 1], c.buf(sp), dIn, s.pool_k, training, accumulate))
        return e;
      cur = sp;
    } else if (dx) {
      if (int e = launch_from_cl(dIn, dx, p.B, p.xin.C, p.xin.Cs, p.xin.vox() / p.B, c.s, c.bf()))
        return e;
    }
    // levels >= i: both convs' weight gradients and every BatchNorm of theirs
    // (dc2[i]'s in level i+1's pooled backward, or the decoder's) are final
    if (i == p.grad_deep && i > 0)
      if (int e = grads_ready(p.grad_ev[1])) return e;
  }
  tag(std::string("wgrad"), "finalize");
  if (int e = c.fork()) return e;   // (the last weight gradient may have run half on the chain)
  if (int e = c.flush_wgf()) return e;
  if (int e = c.join()) return e;
  if (timing_on()) timing_set_tag("");
  return HCU_OK;
}

// Creates the weight-gradient branch's stream and events on `dev` (once).
int ensure_side(const hcu_unet_plan &p, int dev) {
  if (p.side && p.side_device == dev) return HCU_OK;
  p.destroy_side();
  // (stream priority of the branch, either way, measured no effect in round 3)
  HCU_HIP(hipStreamCreateWithFlags(&p.side, hipStreamNonBlocking));
  p.side_device = dev;
  for (hipEvent_t *e : {&p.ev_fork, &p.ev_join, &p.ev_chain, &p.ev_prep})
    HCU_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  for (hipEvent_t &e : p.ev_slot) HCU_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipEvent_t &e : p.ev_fork_ring) HCU_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return HCU_OK;
}

bool side_enabled() {   // HCU_SIDE=0 keeps the whole backward on one stream (A/B, debugging)
  static const bool on = [] {
    const char *e = getenv("HCU_SIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}


int hcu_unet_backward(const hcu_unet_plan *plan, const hcu_unet_tensors *t, const float *dout,
                      float *dx, int training, int accumulate, hcu_stream_t stream) {
  if (!plan || !t || !dout || !t->grads || !t->params || !t->saved || !t->scratch)
    return fail(HCU_ERR_INVALID, "null argument");
  const hcu_unet_plan &p = *plan;
  if (p.flags & HCU_PLAN_FORWARD_ONLY)
    return fail(HCU_ERR_INVALID, "backward through a forward-only plan (its activations are not kept)");
  std::vector<uintptr_t> key = {1, (uintptr_t)t->params, (uintptr_t)t->grads,
                                (uintptr_t)t->saved, (uintptr_t)t->scratch, (uintptr_t)dout,
                                (uintptr_t)dx, (uintptr_t)training, (uintptr_t)accumulate};
  // Per-launch timing attributes kernel time to layers: keep it serial.
  const bool split = side_enabled() && !timing_on();
  std::unique_lock<std::mutex> lk(p.smu, std::defer_lock);
  if (split) {
    lk.lock();   // one user of the branch stream and its events at a time
    int dev = 0;
    HCU_HIP(hipGetDevice(&dev));
    if (int e = ensure_side(p, dev)) return e;
  }
  key.push_back((uintptr_t)split);
  const bool live = graphs_for(p, true) && !timing_on() ? false : true;
  const double t0 = host_prof_on() ? host_now_us() : 0.0;
  double su[2];
  long sn[2];
  if (host_prof_on()) host_prof_snap(su, sn);
  const int rc = run_graphed(p, key, (hipStream_t)stream, [&](hipStream_t s) {
    return enqueue_backward(p, t, dout, dx, training, accumulate, s, split, live);
  });
  if (host_prof_on()) {
    const double dt = host_now_us() - t0;
    host_prof_add(3, dt);
    host_prof_call(1, su, sn, dt);
  }
  return rc;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Per-op entry points (channels-last), sharing the executor's layer setup.
// ---------------------------------------------------------------------------
namespace {

struct OpPlan {
  ConvLayer conv;
  ConvTLayer ct;
  size_t max_wprep = 0, max_part = 0, max_kpart = 0;
  size_t wprep_off = 0, part_off = 0, kpart_off = 0, scratch_bytes = 0;
};

int make_op(const hcu_conv_desc *d, OpPlan &op) {
  if (!d) return fail(HCU_ERR_INVALID, "null descriptor");
  if (d->dtype != HCU_F32 && d->dtype != HCU_BF16) return fail(HCU_ERR_INVALID, "bad dtype");
  const Dims in = mkdims(d->B, d->X, d->Y, d->Z, d->Cin, d->dtype == HCU_BF16 ? 2 : 4);
  if (!d->transposed) {
    for (int i = 0; i < 3; ++i)
      if (d->stride[i] != 1) return fail(HCU_ERR_UNSUPPORTED, "Conv3d: only stride 1 (valid) is supported");
    if (int e = setup_conv(op.conv, in, d->Cout, d->groups, d->Cin, d->Cin, d->k, d->dil, "conv3d"))
      return e;
    op.max_wprep = std::max(prep_floats_fwd(op.conv), prep_floats_dgrad(op.conv));
    op.max_part = wgrad_partial_floats(op.conv.wg);
    op.max_kpart = std::max(conv_partial_floats(op.conv.fwd), conv_partial_floats(op.conv.dgrad));
  } else {
    if (d->groups != 1) return fail(HCU_ERR_UNSUPPORTED, "ConvTranspose3d: groups must be 1");
    for (int i = 0; i < 3; ++i)
      if (d->dil[i] != 1) return fail(HCU_ERR_UNSUPPORTED, "ConvTranspose3d: dilation must be 1");
    if (int e = setup_convt(op.ct, in, d->Cout, d->k, d->stride, op.max_wprep, op.max_part,
                            op.max_kpart))
      return e;
  }
  Region r;
  op.wprep_off = r.take_floats(op.max_wprep);
  op.part_off = r.take_floats(op.max_part);
  op.kpart_off = r.take_floats(std::max<size_t>(op.max_kpart, 1));
  op.scratch_bytes = r.off;
  return 0;
}

// One weight re-layout through the batched prep kernel (the bf16 images).
int prep_one(int kind, const GConvArgs &a, const int *prm, int np, const float *w, float *dst,
             hipStream_t s) {
  PrepJob j{};
  j.kind = kind;
  j.bf16 = (a.use_bconv && a.bes != 4) ? 1 : 0;
  j.n = (int64_t)prep_elems(a);
  j.src = 0;
  j.dst = 0;
  j.pk = wpack_of(a);
  std::copy(prm, prm + np, j.p);
  return launch_prep_all(w, dst, &j, 1, s);
}

int check_scratch(const OpPlan &op, void *scratch, size_t bytes) {
  if (bytes < op.scratch_bytes || (!scratch && op.scratch_bytes))
    return fail(HCU_ERR_WORKSPACE, "scratch workspace too small: need " + std::to_string(op.scratch_bytes));
  return 0;
}

}  // namespace

extern "C" {

size_t hcu_conv_scratch_bytes(const hcu_conv_desc *d) {
  OpPlan op;
  if (make_op(d, op)) return 0;
  return op.scratch_bytes;
}

int hcu_conv_out_dims(const hcu_conv_desc *d, int *out) {
  OpPlan op;
  if (int e = make_op(d, op)) return e;
  const Dims &o = d->transposed ? op.ct.out : op.conv.out;
  out[0] = o.X;
  out[1] = o.Y;
  out[2] = o.Z;
  return HCU_OK;
}

int hcu_conv_fwd_cl(const hcu_conv_desc *d, const float *x, const float *w, const float *bias,
                    float *y, void *scratch, size_t scratch_bytes, hcu_stream_t stream) {
  OpPlan op;
  if (int e = make_op(d, op)) return e;
  if (int e = check_scratch(op, scratch, scratch_bytes)) return e;
  hipStream_t s = (hipStream_t)stream;
  float *wprep = reinterpret_cast<float *>((char *)scratch + op.wprep_off);
  float *kpart = reinterpret_cast<float *>((char *)scratch + op.kpart_off);
  if (!d->transposed) {
    const ConvLayer &L = op.conv;
    if (L.fwd.use_bconv) {
      const int pf[8] = {L.Cout, L.Cin_g, L.groups, L.fold_mod, L.T, L.fwd.ICs, L.fwd.CoutW,
                         std::min(L.fold_mod, L.groups * L.Cin_g)};
      if (int e = prep_one(PREP_CONV_FWD, L.fwd, pf, 8, w, wprep, s)) return e;
    } else if (int e = launch_prep_conv_fwd(w, wprep, L.Cout, L.Cin_g, L.groups, L.fold_mod, L.T,
                                            L.fwd.ICs, L.fwd.CoutW, wpack_of(L.fwd), s)) {
      return e;
    }
    GConvArgs a = L.fwd;
    a.in = x;
    a.w = wprep;
    a.bias = bias;
    a.out = y;
    a.partial = kpart;
    return launch_conv_any(a, s);
  }
  const ConvTLayer &u = op.ct;
  if (u.fused) {
    GConvArgs a = u.fwdf;
    if (a.use_bconv) {
      const int pf[11] = {u.Cin, u.Cout, u.K[0], u.K[1], u.K[2], u.S[0], u.S[1], u.S[2], a.ICs,
                          a.CoutW, a.cph};
      if (int e = prep_one(PREP_CONVT_FUSED, a, pf, 11, w, wprep, s)) return e;
    } else if (int e = launch_prep_convt_fused(w, wprep, u.Cin, u.Cout, u.K[0], u.K[1], u.K[2],
                                               u.S[0], u.S[1], u.S[2], a.ICs, a.CoutW,
                                               wpack_of(a), s)) {
      return e;
    }
    a.in = x;
    a.w = wprep;
    a.bias = bias;
    a.out = y;
    a.partial = kpart;
    return launch_conv_any(a, s);
  }
  for (size_t ph = 0; ph < u.phases.size(); ++ph) {
    const int *pj = &u.pJ[ph * 6];
    GConvArgs a = u.phases[ph];
    if (int e = launch_prep_convt_fwd(w, wprep, u.Cin, u.Cout, u.K[0], u.K[1], u.K[2], u.S[0],
                                      u.S[1], u.S[2], pj[0], pj[1], pj[2], pj[3], pj[4], pj[5],
                                      a.ICs, a.CoutW, s))
      return e;
    a.in = x;
    a.w = wprep;
    a.bias = bias;
    a.out = y;
    if (int e = launch_gconv(a, s)) return e;
  }
  return HCU_OK;
}

int hcu_conv_dgrad_cl(const hcu_conv_desc *d, const float *dy, const float *w, float *dx,
                      void *scratch, size_t scratch_bytes, hcu_stream_t stream) {
  OpPlan op;
  if (int e = make_op(d, op)) return e;
  if (int e = check_scratch(op, scratch, scratch_bytes)) return e;
  hipStream_t s = (hipStream_t)stream;
  float *wprep = reinterpret_cast<float *>((char *)scratch + op.wprep_off);
  float *kpart = reinterpret_cast<float *>((char *)scratch + op.kpart_off);
  GConvArgs a;
  if (!d->transposed) {
    const ConvLayer &L = op.conv;
    if (L.dgrad.use_bconv) {
      const int pd[8] = {L.Cout, L.Cin_g, L.groups, L.fold_mod, L.T, L.dgrad.ICs, L.dgrad.CoutW,
                         L.E};
      if (int e = prep_one(PREP_CONV_DGRAD, L.dgrad, pd, 8, w, wprep, s)) return e;
    } else if (int e = launch_prep_conv_dgrad(w, wprep, L.Cout, L.Cin_g, L.groups, L.fold_mod,
                                              L.T, L.dgrad.ICs, L.dgrad.CoutW, L.E,
                                              wpack_of(L.dgrad), s)) {
      return e;
    }
    a = L.dgrad;
  } else {
    const ConvTLayer &u = op.ct;
    if (u.dgrad.use_bconv) {
      const int pd[5] = {u.Cin, u.Cout, u.T, u.dgrad.ICs, u.dgrad.CoutW};
      if (int e = prep_one(PREP_CONVT_DGRAD, u.dgrad, pd, 5, w, wprep, s)) return e;
    } else if (int e = launch_prep_convt_dgrad(w, wprep, u.Cin, u.Cout, u.T, u.dgrad.ICs,
                                               u.dgrad.CoutW, wpack_of(u.dgrad), s)) {
      return e;
    }
    a = u.dgrad;
  }
  a.in = dy;
  a.w = wprep;
  a.out = dx;
  a.partial = kpart;
  return launch_conv_any(a, s);
}

int hcu_conv_wgrad_cl(const hcu_conv_desc *d, const float *x, const float *dy, float *dw,
                      float *dbias, void *scratch, size_t scratch_bytes, hcu_stream_t stream) {
  OpPlan op;
  if (int e = make_op(d, op)) return e;
  if (int e = check_scratch(op, scratch, scratch_bytes)) return e;
  hipStream_t s = (hipStream_t)stream;
  float *part = reinterpret_cast<float *>((char *)scratch + op.part_off);
  WGradFinalize f{};
  WGradArgs w;
  if (!d->transposed) {
    const ConvLayer &L = op.conv;
    w = L.wg;
    f.mode = 0;
    f.T = L.T;
    f.Cout = L.Cout;
    f.Cin_g = L.Cin_g;
    f.groups = L.groups;
    f.fold_mod = L.fold_mod;
    f.db = dbias;
  } else {
    const ConvTLayer &u = op.ct;
    w = u.wg;
    f.mode = 1;
    f.T = u.T;
    f.Cin = u.Cin;
    f.CoutT = u.Cout;
  }
  w.A = x;
  w.G = dy;
  w.partial = part;
  if (int e = launch_wgrad(w, s)) return e;
  f.partial = part;
  f.dw = dw;
  f.KB = w.KB;
  f.Mtot = w.Mtot;
  f.Ntot = w.Ntot;
  f.ACs = wgrad_slab_acs(w);
  f.GCs = w.GCs;
  if (int e = launch_wgrad_finalize(f, s)) return e;
  if (d->transposed && dbias) {
    const ConvTLayer &u = op.ct;
    const int R = chansum_rows(u.out.vox(), u.out.Cs);
    if (int e = launch_chansum(dy, u.out.vox(), u.out.Cs, part, R, s, u.out.es == 2)) return e;
    if (int e = launch_reduce_partials(part, R, u.out.Cs, u.Cout, dbias, 0, s)) return e;
  }
  return HCU_OK;
}

int hcu_maxpool_fwd_cl(int B, int C, int X, int Y, int Z, const int *k, const float *x, float *y,
                       hcu_stream_t stream) {
  if (!k || k[0] < 1 || k[1] < 1 || k[2] < 1) return fail(HCU_ERR_INVALID, "bad pool kernel");
  if (X / k[0] < 1 || Y / k[1] < 1 || Z / k[2] < 1)
    return fail(HCU_ERR_SHAPE, "max_pool3d: Output size is too small");
  return launch_maxpool_fwd(x, nullptr, nullptr, y, B, X, Y, Z, round_up(C, 4), k[0], k[1], k[2],
                            (hipStream_t)stream);
}

size_t hcu_loss_pixel_scratch_bytes(int64_t n_pred) {
  return align_up((size_t)loss_rows(n_pred) * sizeof(float), 256);
}

int hcu_loss_pixel_fwd(const float *pred, int B, int C, int PX, int PY, int PZ, const void *mask,
                       int mask_dtype, const void *pwl, int pwl_dtype, int MX, int MY, int MZ,
                       float *loss, float *dpred, void *scratch, size_t scratch_bytes,
                       hcu_stream_t stream) {
  if (!pred || !mask || !loss || !scratch) return fail(HCU_ERR_INVALID, "null argument");
  if (MX < PX || MY < PY || MZ < PZ)
    return fail(HCU_ERR_SHAPE, "mask/pwl smaller than the prediction");
  if (mask_dtype < 0 || mask_dtype > 2 || pwl_dtype < 0 || pwl_dtype > 1)
    return fail(HCU_ERR_INVALID, "unsupported mask/pwl dtype");
  const int64_t n = (int64_t)B * C * PX * PY * PZ;
  if (scratch_bytes < hcu_loss_pixel_scratch_bytes(n))
    return fail(HCU_ERR_WORKSPACE, "loss scratch too small");
  return launch_loss_pixel(pred, B, C, PX, PY, PZ, mask, mask_dtype, pwl, pwl_dtype, MX, MY, MZ,
                           loss, dpred, (float *)scratch, loss_rows(n), (hipStream_t)stream);
}

int hcu_scale_by_device_scalar(const float *src, const float *scale, float *dst, int64_t n,
                               hcu_stream_t stream) {
  return launch_scale(src, scale, dst, n, (hipStream_t)stream);
}

int hcu_adam_step(float *p, const float *g, float *m, float *v, int64_t n, float lr, float beta1,
                  float beta2, float eps, float weight_decay, int64_t step, float grad_scale,
                  hcu_stream_t stream) {
  return launch_adam(p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, step, grad_scale,
                     (hipStream_t)stream);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Layer chains (include/hcunet.h, hcu_chain_*): a sequence of Conv3d [+ BN +
// ReLU] / MaxPool3d / ConvTranspose3d [+ cat(U, U)] ops with the network
// executor's kernels and fusions: BatchNorm+ReLU applied while the consumer
// stages its operand, BatchNorm statistics in the producing conv's epilogue,
// the BatchNorm backward reduction in the consumer dgrad's epilogue or fused
// with the max-pool backward.  Single stream, direct launches.
// ---------------------------------------------------------------------------
namespace {

using ChainOp = hcu_unet_plan::ChainOp;

int build_chain(hcu_unet_plan &p, const hcu_chain_spec &cs) {
  if (cs.n_ops < 1 || cs.n_ops > HCU_CHAIN_MAX_OPS) return fail(HCU_ERR_INVALID, "chain: 1..16 ops");
  if (cs.compute_dtype != HCU_F32 && cs.compute_dtype != HCU_BF16)
    return fail(HCU_ERR_INVALID, "compute_dtype must be HCU_F32 or HCU_BF16");
  if (cs.in_channels < 1) return fail(HCU_ERR_INVALID, "chain: in_channels must be positive");
  if (p.B < 1 || p.X < 1 || p.Y < 1 || p.Z < 1) return fail(HCU_ERR_SHAPE, "empty input");
  p.is_chain = true;
  p.L = 0;
  p.es = cs.compute_dtype == HCU_BF16 ? 2 : 4;
  p.spec = hcu_unet_spec{};
  p.spec.bn_eps = cs.bn_eps;
  p.spec.bn_momentum = cs.bn_momentum;
  p.spec.compute_dtype = cs.compute_dtype;
  const bool bf = p.es == 2;
  Region saved;
  p.xin = mkdims(p.B, p.X, p.Y, p.Z, cs.in_channels, p.es);
  p.in_cl = cs.in_cl != 0;
  p.out_cl = cs.out_cl != 0;
  if (cs.in_part_channels > 0) {
    if (!p.in_cl) return fail(HCU_ERR_INVALID, "chain: in_part_channels needs in_cl");
    if (cs.in_channels % cs.in_part_channels)
      return fail(HCU_ERR_INVALID, "chain: in_channels must be a multiple of in_part_channels");
    if (cs.ops[0].kind != HCU_CHAIN_CONV || cs.ops[0].groups != 1 || cs.ops[0].cat_fold)
      return fail(HCU_ERR_UNSUPPORTED, "chain: an input of channel parts needs a first Conv3d, groups 1");
    p.xin.part_c = cs.in_part_channels;
    p.xin.Cs = (cs.in_channels / cs.in_part_channels) * round_up(cs.in_part_channels, bf ? 8 : 4);
  }
  if (p.out_cl) {
    const hcu_chain_op &l = cs.ops[cs.n_ops - 1];
    if (l.kind != HCU_CHAIN_CONV || l.bn_relu)
      return fail(HCU_ERR_UNSUPPORTED, "chain: out_cl needs a last Conv3d without BatchNorm");
  }
  // (in_cl: the caller's tensor is the first op's input, nothing is copied)
  p.xcl_off = p.in_cl ? 0 : saved.take_floats(p.xin.floats());
  p.max_act = p.xin.floats();
  p.chain.assign(cs.n_ops, ChainOp{});
  Dims cur = p.xin;
  int prev = -1;
  bool prev_bn = false;
  int bn_index = 0;
  for (int i = 0; i < cs.n_ops; ++i) {
    const hcu_chain_op &s = cs.ops[i];
    ChainOp &o = p.chain[i];
    o.kind = s.kind;
    const std::string nm = "c" + std::to_string(i);
    if (s.kind == HCU_CHAIN_CONV) {
      o.bn_relu = s.bn_relu != 0;
      o.fold = s.cat_fold != 0;
      if (o.fold && prev != HCU_CHAIN_CONVT)
        return fail(HCU_ERR_INVALID, "chain: cat_fold needs a preceding ConvTranspose3d");
      const int cin_total = o.fold ? 2 * cur.C : cur.C;
      const int fold_mod = o.fold ? cur.C : cin_total;
      ConvLayer &L = o.conv;
      L.name = nm;
      if (int e = setup_conv(L, cur, s.out_channels, s.groups, fold_mod, cin_total, s.k, s.dil, "Conv3d",
                             s.stride, s.pad))
        return e;
      if (L.s2b && o.bn_relu)
        return fail(HCU_ERR_UNSUPPORTED, "chain: BatchNorm after a sub-lattice (large dilated) Conv3d");
      L.w_off = s.w_off;
      L.b_off = s.b_off;
      if (L.s2b) {
        o.xs_off = saved.take_floats(L.sub_in.floats());
        p.max_sub = std::max({p.max_sub, L.sub_in.floats(), L.sub_out.floats()});
      }
      // (out_cl: the last conv writes the caller's tensor and, without a
      // BatchNorm, its backward never reads y: no saved buffer)
      L.y_off = p.out_cl && i + 1 == cs.n_ops ? 0 : saved.take_floats(L.out.floats());
      if (o.bn_relu) {
        L.bn.coef_off = saved.take_floats((size_t)6 * L.bn.Cs);
        L.bn.gamma = s.gamma_off;
        L.bn.beta = s.beta_off;
        L.bn.index = bn_index++;
      }
      track_conv(p, L);
      cur = L.out;
      prev_bn = o.bn_relu;
    } else if (s.kind == HCU_CHAIN_POOL) {
      if (!(prev == HCU_CHAIN_CONV && prev_bn))
        return fail(HCU_ERR_UNSUPPORTED, "chain: MaxPool3d must follow Conv3d + BatchNorm3d + ReLU");
      for (int d = 0; d < 3; ++d) {
        o.pk[d] = s.k[d];
        if (s.k[d] < 1) return fail(HCU_ERR_INVALID, "chain: bad pool kernel");
      }
      const int px = cur.X / o.pk[0], py = cur.Y / o.pk[1], pz = cur.Z / o.pk[2];
      if (px < 1 || py < 1 || pz < 1) return fail(HCU_ERR_SHAPE, "max_pool3d: Output size is too small");
      o.pooled = mkdims(p.B, px, py, pz, cur.C, p.es);
      o.pool_off = saved.take_floats(o.pooled.floats());
      p.max_act = std::max(p.max_act, o.pooled.floats());
      cur = o.pooled;
      prev_bn = false;
    } else if (s.kind == HCU_CHAIN_CONVT) {
      for (int d = 0; d < 3; ++d)
        if (s.dil[d] > 1) return fail(HCU_ERR_UNSUPPORTED, "ConvTranspose3d: dilation must be 1");
      if (s.groups > 1) return fail(HCU_ERR_UNSUPPORTED, "ConvTranspose3d: groups must be 1");
      ConvTLayer &u = o.ct;
      u.name = nm;
      if (int e = setup_convt(u, cur, s.out_channels, s.k, s.stride, p.max_wprep, p.max_part, p.max_kpart))
        return e;
      u.w_off = s.w_off;
      u.b_off = s.b_off;
      const Dims full = u.out;
      int cd[3];
      const int fd[3] = {full.X, full.Y, full.Z};
      bool crop = false;
      for (int d = 0; d < 3; ++d) {
        o.crop[d] = s.pad[d];
        if (s.pad[d] < 0) return fail(HCU_ERR_INVALID, "ConvTranspose3d: negative padding");
        cd[d] = fd[d] - 2 * s.pad[d];
        if (cd[d] < 1) return fail(HCU_ERR_SHAPE, "ConvTranspose3d: output size is too small");
        crop = crop || s.pad[d] > 0;
      }
      if (crop) {
        // forward: full output into scratch, then the crop; backward: the
        // cropped gradient read at offset pad (zero outside it)
        o.ufull = full;
        p.max_ufull = std::max(p.max_ufull, full.floats());
        u.out = mkdims(p.B, cd[0], cd[1], cd[2], s.out_channels, p.es);
        GConvArgs &a = u.dgrad;
        a.use_bconv = a.use_conv2 = a.use_conv8 = 0;   // re-planned from scratch
        a.bes = 0;
        a.IX = cd[0]; a.IY = cd[1]; a.IZ = cd[2];
        a.px = s.pad[0]; a.py = s.pad[1]; a.pz = s.pad[2];
        if (int e = bf ? plan_bconv(a, kTargetBlocks) : plan_conv_fp32(a, kTargetBlocks)) return e;
        p.max_wprep = std::max(p.max_wprep, wprep_floats(a));
        p.max_part = std::max(p.max_part, (size_t)gconv_rows(a) * a.CoutW * 2);
        p.max_kpart = std::max(p.max_kpart, conv_partial_floats(a));
        WGradArgs &w = u.wg;
        w.v2 = 0;
        w.use_bw = 0;
        w.GX = cd[0]; w.GY = cd[1]; w.GZ = cd[2];
        w.gpx = s.pad[0]; w.gpy = s.pad[1]; w.gpz = s.pad[2];
        if (int e = bf ? plan_bwgrad(w, kTargetBlocks) : plan_wgrad(w, kTargetBlocks)) return e;
        p.max_part = std::max(p.max_part, wgrad_partial_floats(w));
        p.max_part = std::max(p.max_part, (size_t)chansum_rows(u.out.vox(), u.out.Cs) * u.out.Cs);
      }
      u.wg_swap = false;
      if (bf && !prev_bn && !getenv("HCU_CONVT_NOSWAP")) {
        // dW[ci][co][k] = sum_o x[o][ci] dU[o*S + k - pad][co]
        WGradArgs v{};
        v.B = p.B;
        v.AX = u.out.X; v.AY = u.out.Y; v.AZ = u.out.Z; v.ACs = u.out.Cs;   // dU (cropped)
        v.GX = u.in.X; v.GY = u.in.Y; v.GZ = u.in.Z; v.GCs = u.in.Cs;        // x
        v.PX = u.in.X; v.PY = u.in.Y; v.PZ = u.in.Z;
        v.KX = u.K[0]; v.KY = u.K[1]; v.KZ = u.K[2];
        v.asx = u.S[0]; v.asy = u.S[1]; v.asz = u.S[2];
        v.adx = v.ady = v.adz = 1;
        v.apx = s.pad[0]; v.apy = s.pad[1]; v.apz = s.pad[2];
        v.gsx = v.gsy = v.gsz = 1;
        v.gdx = v.gdy = v.gdz = 1;
        v.taps_rows = 1;
        v.bias_row = 0;
        v.ACr = u.Cout;
        v.GCr = u.Cin;
        v.flops = 2.0 * p.B * u.in.X * u.in.Y * u.in.Z * (double)u.T * u.Cin * u.Cout;
        if (plan_bwgrad(v, kTargetBlocks) == 0) {
          u.wgs = v;
          u.wg_swap = true;
          p.max_part = std::max(p.max_part, wgrad_partial_floats(v));
        } else {
          set_error("");
        }
      }
      u.u_off = saved.take_floats(u.out.floats());
      p.max_act = std::max(p.max_act, u.out.floats());
      cur = u.out;
      prev_bn = false;
    } else {
      return fail(HCU_ERR_INVALID, "chain: unknown op kind");
    }
    prev = s.kind;
  }
  p.outd = cur;
  p.n_bn = bn_index;
  // weight re-layouts (one batched launch per forward), the last range of
  // `saved` (or the caller's image buffer: hcu_chain_forward_images)
  const size_t img0 = saved.off;
  p.prep_jobs.clear();
  auto add_job = [&](int kind, size_t n, int64_t src, const WPack &pk, const int *prm, int np, size_t &off) {
    PrepJob j{};
    j.kind = kind;
    j.bf16 = bf;
    j.n = (int64_t)n;
    j.src = src;
    off = saved.take_floats(j.bf16 ? (n + 1) / 2 : n);
    j.dst = (int64_t)(off / sizeof(float));
    j.pk = pk;
    std::copy(prm, prm + np, j.p);
    p.prep_jobs.push_back(j);
  };
  for (ChainOp &o : p.chain) {
    if (o.kind == HCU_CHAIN_CONV) {
      ConvLayer &cl = o.conv;
      const int pf[10] = {cl.Cout, cl.Cin_g, cl.groups, cl.fold_mod, cl.T, cl.fwd.ICs, cl.fwd.CoutW,
                          cl.part_c ? cl.fwd.ICs : std::min(cl.fold_mod, cl.groups * cl.Cin_g),
                          cl.part_c, cl.part_cs};
      add_job(PREP_CONV_FWD, prep_elems(cl.fwd), cl.w_off, wpack_of(cl.fwd), pf, 10, cl.wf_off);
      if (cl.has_dgrad) {
        const int pd[10] = {cl.Cout, cl.Cin_g, cl.groups, cl.fold_mod, cl.T, cl.dgrad.ICs, cl.dgrad.CoutW, cl.E,
                            cl.part_c, cl.part_cs};
        add_job(PREP_CONV_DGRAD, prep_elems(cl.dgrad), cl.w_off, wpack_of(cl.dgrad), pd, 10, cl.wd_off);
      }
    } else if (o.kind == HCU_CHAIN_CONVT) {
      ConvTLayer &u = o.ct;
      if (u.fused) {
        const int pf[11] = {u.Cin, u.Cout, u.K[0], u.K[1], u.K[2], u.S[0], u.S[1], u.S[2],
                            u.fwdf.ICs, u.fwdf.CoutW, u.fwdf.cph};
        add_job(PREP_CONVT_FUSED, prep_elems(u.fwdf), u.w_off, wpack_of(u.fwdf), pf, 11, u.wf_off);
      } else {
        u.wph_off.assign(u.phases.size(), 0);
        for (size_t ph = 0; ph < u.phases.size(); ++ph) {
          const int *pj = &u.pJ[ph * 6];
          const GConvArgs &a = u.phases[ph];
          const int pf[16] = {u.Cin, u.Cout, u.K[0], u.K[1], u.K[2], u.S[0], u.S[1], u.S[2],
                              pj[0], pj[1], pj[2], pj[3], pj[4], pj[5], a.ICs, a.CoutW};
          add_job(PREP_CONVT_PHASE, (size_t)pj[3] * pj[4] * pj[5] * a.ICs * a.CoutW, u.w_off, WPack{}, pf,
                  16, u.wph_off[ph]);
        }
      }
      const int pd[5] = {u.Cin, u.Cout, u.T, u.dgrad.ICs, u.dgrad.CoutW};
      add_job(PREP_CONVT_DGRAD, prep_elems(u.dgrad), u.w_off, wpack_of(u.dgrad), pd, 5, u.wd_off);
    }
  }
  p.prep_fwd.clear();
  p.prep_bwd.clear();
  for (const PrepJob &j : p.prep_jobs)
    (j.kind == PREP_CONV_DGRAD || j.kind == PREP_CONVT_DGRAD ? p.prep_bwd : p.prep_fwd).push_back(j);
  p.img_lo = img0;
  p.img_bytes = saved.off - img0;
  p.saved_bytes = saved.off;
  Region scratch;
  for (int i = 0; i < HCU_NBUF; ++i) p.buf_off[i] = scratch.take_floats(i < p.nbuf ? p.max_act : 0);
  p.part_off = scratch.take_floats(p.max_part);
  p.wpart_floats = std::max<size_t>(p.max_part, (size_t)1 << 20);
  p.wpart_off = scratch.take_floats(p.wpart_floats);
  p.wprep_off = scratch.take_floats(p.max_wprep);
  p.kpart_off = scratch.take_floats(std::max<size_t>(p.max_kpart, 1));
  p.ufull_off = scratch.take_floats(p.max_ufull);
  for (size_t &o : p.sub_off) o = scratch.take_floats(p.max_sub);
  p.scratch_bytes = scratch.off;
  return 0;
}

// Activation entering each op: (tensor, BatchNorm scale, shift) -- the
// producer's BatchNorm+ReLU is applied by the consumer while it loads.
struct ChainAct {
  const float *x = nullptr, *sc = nullptr, *sh = nullptr;
};

std::vector<ChainAct> chain_inputs(const hcu_unet_plan &p, char *sv, const void *x, ChainAct *out_act) {
  std::vector<ChainAct> in(p.chain.size());
  ChainAct a;
  a.x = p.in_cl ? reinterpret_cast<const float *>(x) : reinterpret_cast<const float *>(sv + p.xcl_off);
  for (size_t i = 0; i < p.chain.size(); ++i) {
    const ChainOp &o = p.chain[i];
    in[i] = a;
    if (o.kind == HCU_CHAIN_CONV) {
      a.x = reinterpret_cast<const float *>(sv + o.conv.y_off);
      if (o.bn_relu) {
        const BNCoef cf = coef_at(sv, o.conv.bn);
        a.sc = cf.scale;
        a.sh = cf.shift;
      } else {
        a.sc = a.sh = nullptr;
      }
    } else if (o.kind == HCU_CHAIN_POOL) {
      a = ChainAct{reinterpret_cast<const float *>(sv + o.pool_off), nullptr, nullptr};
    } else {
      a = ChainAct{reinterpret_cast<const float *>(sv + o.ct.u_off), nullptr, nullptr};
    }
  }
  if (out_act) *out_act = a;
  return in;
}

// images: the caller's weight-image buffer (img_bytes) or null (in `saved`);
// images_current: 1 = it holds this plan's forward images of the current
// parameters, 2 = also the input-gradient ones (no re-layout then).
int enqueue_chain_forward(const hcu_unet_plan &p, const hcu_unet_tensors *t, int training, hipStream_t s,
                          void *images = nullptr, int images_current = 0) {
  Ctx c{p, *t, s, (char *)t->saved, (char *)t->scratch, t->params, t->grads};
  if (images) c.wi = (char *)images - p.img_lo;
  const int es = p.es, bf = c.bf();
  tag(std::string("chain"), "fwd");
  if (!p.in_cl)
    if (int e = launch_to_cl(t->x, c.fptr(c.sv, p.xcl_off), p.B, p.xin.C, p.xin.Cs, p.xin.vox() / p.B, s, bf,
                             t->x_dtype))
      return e;
  const std::vector<PrepJob> &jobs = training ? p.prep_jobs : p.prep_fwd;
  if (!jobs.empty() && images_current < (training ? 2 : 1))
    if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), jobs.data(), (int)jobs.size(), s)) return e;
  ChainAct last;
  const std::vector<ChainAct> in = chain_inputs(p, c.sv, t->x, &last);
  for (size_t i = 0; i < p.chain.size(); ++i) {
    const ChainOp &o = p.chain[i];
    const ChainAct &a = in[i];
    if (o.kind == HCU_CHAIN_CONV) {
      const ConvLayer &L = o.conv;
      // (out_cl: the last conv writes the caller's tensor; no op of this chain reads it back)
      float *y = p.out_cl && i + 1 == p.chain.size() ? t->out : c.fptr(c.sv, L.y_off);
      if (L.s2b) {
        float *xs = c.fptr(c.sv, o.xs_off), *ys = c.fptr(c.sc, p.sub_off[0]);
        const int sd[3] = {L.sub_in.X, L.sub_in.Y, L.sub_in.Z}, so[3] = {L.sub_out.X, L.sub_out.Y, L.sub_out.Z};
        tag(L.name, "fwd");
        if (int e = launch_s2b(a.x, a.sc, a.sh, xs, p.B, L.in.X, L.in.Y, L.in.Z, L.in.Cs, es, L.L3, sd, s))
          return e;
        GConvArgs g = L.fwd;
        g.in = xs;
        g.in_scale = g.in_shift = nullptr;
        g.w = c.fptr(c.wimg(), L.wf_off);
        g.bias = L.b_off >= 0 ? c.P + L.b_off : nullptr;
        g.out = ys;
        g.stats = nullptr;
        g.partial = c.kpart();
        if (int e = launch_conv_any(g, s)) return e;
        if (int e = launch_b2s(ys, y, p.B, L.out.X, L.out.Y, L.out.Z, L.out.Cs, es, L.L3, so, s)) return e;
      } else if (o.bn_relu) {
        if (int e = conv_forward(c, L, a.x, a.sc, a.sh, training)) return e;
      } else if (L.pw && !a.sc) {
        tag(L.name, "fwd");
        PwArgs w{};
        w.in = reinterpret_cast<const uint16_t *>(a.x);
        w.w = c.P + L.w_off;
        w.bias = L.b_off >= 0 ? c.P + L.b_off : nullptr;
        w.out = reinterpret_cast<uint16_t *>(y);
        w.nvox = L.out.vox();
        w.ICs = L.in.Cs;
        w.OCs = L.out.Cs;
        w.Cin = L.Cin_g;
        w.Cout = L.Cout;
        w.part_c = L.part_c;
        w.part_cs = L.part_cs;
        if (int e = launch_pw(w, s)) return e;
      } else {
        tag(L.name, "fwd");
        GConvArgs g = L.fwd;
        g.in = a.x;
        g.in_scale = a.sc;
        g.in_shift = a.sh;
        g.w = c.fptr(c.wimg(), L.wf_off);
        g.bias = L.b_off >= 0 ? c.P + L.b_off : nullptr;
        g.out = y;
        g.stats = nullptr;
        g.partial = c.kpart();
        if (int e = launch_conv_any(g, s)) return e;
      }
    } else if (o.kind == HCU_CHAIN_POOL) {
      const ConvLayer &P = p.chain[i - 1].conv;
      tag(P.name, "pool");
      if (int e = launch_maxpool_fwd(a.x, a.sc, a.sh, c.fptr(c.sv, o.pool_off), p.B, P.out.X, P.out.Y,
                                     P.out.Z, P.out.Cs, o.pk[0], o.pk[1], o.pk[2], s, bf))
        return e;
    } else {
      const ConvTLayer &u = o.ct;
      tag(u.name, "fwd");
      const bool crop = o.crop[0] || o.crop[1] || o.crop[2];
      float *U = crop ? c.fptr(c.sc, p.ufull_off) : c.fptr(c.sv, u.u_off);
      const float *bias = u.b_off >= 0 ? c.P + u.b_off : nullptr;
      if (u.fused) {
        GConvArgs g = u.fwdf;
        g.in = a.x;
        g.in_scale = a.sc;
        g.in_shift = a.sh;
        g.w = c.fptr(c.wimg(), u.wf_off);
        g.bias = bias;
        g.out = U;
        g.stats = nullptr;
        g.partial = c.kpart();
        if (int e = launch_conv_any(g, s)) return e;
      }
      for (size_t ph = 0; !u.fused && ph < u.phases.size(); ++ph) {
        GConvArgs g = u.phases[ph];
        g.in = a.x;
        g.in_scale = a.sc;
        g.in_shift = a.sh;
        g.w = c.fptr(c.wimg(), u.wph_off[ph]);
        g.bias = bias;
        g.out = U;
        g.stats = nullptr;
        if (int e = launch_gconv(g, s)) return e;
      }
      if (crop) {
        const int sd[3] = {o.ufull.X, o.ufull.Y, o.ufull.Z}, dd[3] = {u.out.X, u.out.Y, u.out.Z};
        if (int e = launch_crop_cl(U, c.fptr(c.sv, u.u_off), p.B, sd, dd, o.crop, u.out.Cs, es, s)) return e;
      }
    }
  }
  tag(std::string("chain"), "out");
  if (!p.out_cl)
    if (int e = launch_from_cl_act(last.x, last.sc, last.sh, t->out, p.B, p.outd.C, p.outd.Cs,
                                   p.outd.vox() / p.B, s, bf))
      return e;
  if (training && p.n_bn && t->bn_num_batches_tracked)
    if (int e = launch_bn_count_increment(t->bn_num_batches_tracked, p.n_bn, s)) return e;
  if (timing_on()) timing_set_tag("");
  return HCU_OK;
}

int enqueue_chain_backward(const hcu_unet_plan &p, const hcu_unet_tensors *t, const float *dout, float *dx,
                           int training, int accumulate, hipStream_t s, void *images = nullptr,
                           int images_current = 0) {
  Ctx c{p, *t, s, (char *)t->saved, (char *)t->scratch, t->params, t->grads};
  if (images) c.wi = (char *)images - p.img_lo;
  const int es = p.es, bf = c.bf();
  const int n = (int)p.chain.size();
  const std::vector<ChainAct> in = chain_inputs(p, c.sv, t->x, nullptr);
  // an eval-mode forward prepared only the forward weight images
  if (!training && !p.prep_bwd.empty() && images_current < 2)
    if (int e = launch_prep_all(c.P, reinterpret_cast<float *>(c.wimg()), p.prep_bwd.data(), (int)p.prep_bwd.size(), s))
      return e;
  int cur = 0;
  if (int e = c.alloc(cur)) return e;
  tag(std::string("chain"), "bwd");
  // out_cl: dout is already in the layout (and the precision) of the gradient
  // slots, and the last op (a Conv3d without BatchNorm) only reads its output
  // gradient, so it reads the caller's tensor in place (a chain's backward
  // runs on `s` alone: every read is ordered before the caller's next use of
  // that memory on `s`).
  if (!p.out_cl)
    if (int e = launch_to_cl(dout, c.buf(cur), p.B, p.outd.C, p.outd.Cs, p.outd.vox() / p.B, s, bf, HCU_F32))
      return e;
  bool pre = false;   // buf(cur) already holds d(pre-BatchNorm y) of op i
  for (int i = n - 1; i >= 0; --i) {
    const ChainOp &o = p.chain[i];
    const ChainAct &a = in[i];
    // the output gradient of op i
    float *dY = p.out_cl && i == n - 1 ? const_cast<float *>(dout) : c.buf(cur);
    const bool need_dA = i > 0 || dx != nullptr;
    const ChainOp *pr = i > 0 ? &p.chain[i - 1] : nullptr;
    if (o.kind == HCU_CHAIN_CONV) {
      const ConvLayer &L = o.conv;
      if (o.bn_relu && !pre)
        if (int e = bn_backward(c, L, c.buf(cur), nullptr, nullptr, training, accumulate)) return e;
      int sa = -1;
      float *dA = nullptr;
      if (need_dA) {
        if (!L.has_dgrad) return fail(HCU_ERR_UNSUPPORTED, "input gradient of a strided Conv3d");
        if (i == 0 && p.in_cl) {
          dA = dx;   // the caller's gradient tensor, in the input's layout
        } else {
          if (int e = c.alloc(sa)) return e;
          dA = c.buf(sa);
        }
      }
      bool done = false;
      if (L.s2b) {
        float *dys = c.fptr(c.sc, p.sub_off[1]), *dxs = c.fptr(c.sc, p.sub_off[2]);
        const int sd[3] = {L.sub_in.X, L.sub_in.Y, L.sub_in.Z}, so[3] = {L.sub_out.X, L.sub_out.Y, L.sub_out.Z};
        tag(L.name, "wgrad");
        if (int e = launch_s2b(dY, nullptr, nullptr, dys, p.B, L.out.X, L.out.Y, L.out.Z, L.out.Cs, es,
                               L.L3, so, s))
          return e;
        if (int e = conv_backward(c, L, c.fptr(c.sv, o.xs_off), nullptr, nullptr, dys, cur,
                                  need_dA ? dxs : nullptr, accumulate))
          return e;
        if (need_dA)
          if (int e = launch_b2s(dxs, dA, p.B, L.in.X, L.in.Y, L.in.Z, L.in.Cs, es, L.L3, sd, s)) return e;
      } else {
        const ConvLayer *bnl = (pr && pr->kind == HCU_CHAIN_CONV && pr->bn_relu) ? &pr->conv : nullptr;
        if (int e = conv_backward(c, L, a.x, a.sc, a.sh, dY, cur, dA, accumulate, bnl, training, &done))
          return e;
      }
      if (!need_dA) continue;
      if (i == 0) {
        if (!p.in_cl)
          if (int e = launch_from_cl(dA, dx, p.B, p.xin.C, p.xin.Cs, p.xin.vox() / p.B, s, bf)) return e;
      } else {
        cur = sa;
        pre = done;
      }
    } else if (o.kind == HCU_CHAIN_POOL) {
      const ConvLayer &P = pr->conv;
      int sp = 0;
      if (int e = c.alloc(sp)) return e;
      if (int e = bn_backward(c, P, c.buf(sp), c.buf(cur), o.pk, training, accumulate)) return e;
      cur = sp;
      pre = true;
    } else {
      const ConvTLayer &u = o.ct;
      float *dU = c.buf(cur);
      tag(u.name, "wgrad");
      if (u.b_off >= 0) {
        const int R = chansum_rows(u.out.vox(), u.out.Cs);
        float *cs = nullptr;
        if (int e = c.slab((size_t)R * u.out.Cs, cs)) return e;
        if (int e = launch_chansum(dU, u.out.vox(), u.out.Cs, cs, R, s, bf)) return e;
        WGradFinalize fb{};
        fb.partial = cs;
        fb.db = c.G + u.b_off;
        fb.KB = R;
        fb.Mtot = 1;
        fb.Ntot = u.out.Cs;
        fb.mode = 2;
        fb.Cout = u.Cout;
        fb.accumulate = accumulate;
        if (int e = c.pend_wgf(fb)) return e;
      }
      if (u.wg_swap && !a.sc) {
        WGradArgs w = u.wgs;
        w.A = dU;
        w.a_scale = w.a_shift = nullptr;
        w.G = a.x;
        if (int e = c.slab(wgrad_partial_floats(w), w.partial)) return e;
        if (int e = launch_wgrad(w, s)) return e;
        WGradFinalize f{};
        f.partial = w.partial;
        f.dw = c.G + u.w_off;
        f.KB = w.KB;
        f.Mtot = w.Mtot;
        f.Ntot = w.Ntot;
        f.T = u.T;
        f.mode = 0;
        f.Cout = u.Cin;
        f.Cin_g = u.Cout;
        f.groups = 1;
        f.fold_mod = u.Cout;
        f.ACs = wgrad_slab_acs(w);
        f.accumulate = accumulate;
        if (int e = c.pend_wgf(f)) return e;
      } else {
        WGradArgs w = u.wg;
        w.A = a.x;
        w.a_scale = a.sc;
        w.a_shift = a.sh;
        w.G = dU;
        if (int e = c.slab(wgrad_partial_floats(w), w.partial)) return e;
        if (int e = launch_wgrad(w, s)) return e;
        WGradFinalize f{};
        f.partial = w.partial;
        f.dw = c.G + u.w_off;
        f.KB = w.KB;
        f.Mtot = w.Mtot;
        f.Ntot = w.Ntot;
        f.T = u.T;
        f.mode = 1;
        f.Cin = u.Cin;
        f.CoutT = u.Cout;
        f.GCs = w.GCs;
        f.accumulate = accumulate;
        if (int e = c.pend_wgf(f)) return e;
      }
      if (!need_dA) continue;
      tag(u.name, "dgrad");
      int sd = 0;
      float *dP = dx;   // (i == 0 with in_cl: straight into the caller's gradient tensor)
      if (!(i == 0 && p.in_cl)) {
        if (int e = c.alloc(sd)) return e;
        dP = c.buf(sd);
      }
      GConvArgs g = u.dgrad;
      g.in = dU;
      g.w = c.fptr(c.wimg(), u.wd_off);
      g.out = dP;
      g.partial = c.kpart();
      const ConvLayer *bnl = (pr && pr->kind == HCU_CHAIN_CONV && pr->bn_relu) ? &pr->conv : nullptr;
      const bool fused = fuse_bnbwd(c, g, bnl);
      if (int e = launch_conv_any(g, s)) return e;
      if (fused)
        if (int e = finish_bnbwd(c, g, *bnl, dP, training, accumulate)) return e;
      if (i == 0) {
        if (!p.in_cl)
          if (int e = launch_from_cl(dP, dx, p.B, p.xin.C, p.xin.Cs, p.xin.vox() / p.B, s, bf)) return e;
      } else {
        cur = sd;
        pre = fused;
      }
    }
  }
  tag(std::string("wgrad"), "finalize");
  if (int e = c.flush_wgf()) return e;
  if (timing_on()) timing_set_tag("");
  return HCU_OK;
}

}  // namespace

extern "C" {

int hcu_chain_plan_create(const hcu_chain_spec *spec, int B, int X, int Y, int Z, hcu_unet_plan **out) {
  if (!spec || !out) return fail(HCU_ERR_INVALID, "null argument");
  auto *p = new hcu_unet_plan();
  p->B = B;
  p->X = X;
  p->Y = Y;
  p->Z = Z;
  const int e = build_chain(*p, *spec);
  if (e) {
    delete p;
    *out = nullptr;
    return e;
  }
  *out = p;
  return HCU_OK;
}

int hcu_chain_plan_query(const hcu_unet_plan *p, int64_t *out_shape, int *n_bn, size_t *saved_bytes,
                         size_t *scratch_bytes) {
  if (!p || !p->is_chain) return fail(HCU_ERR_INVALID, "not a chain plan");
  if (out_shape) {
    out_shape[0] = p->B;
    out_shape[1] = p->outd.C;
    out_shape[2] = p->outd.X;
    out_shape[3] = p->outd.Y;
    out_shape[4] = p->outd.Z;
  }
  if (n_bn) *n_bn = p->n_bn;
  if (saved_bytes) *saved_bytes = p->saved_bytes;
  if (scratch_bytes) *scratch_bytes = p->scratch_bytes;
  return HCU_OK;
}

static int hcu_chain_forward_impl(const hcu_unet_plan *p, const hcu_unet_tensors *t, int training,
                                  hcu_stream_t stream, void *images, int images_current);

int hcu_chain_forward(const hcu_unet_plan *p, const hcu_unet_tensors *t, int training, hcu_stream_t stream) {
  if (!p || !p->is_chain) return fail(HCU_ERR_INVALID, "not a chain plan");
  return hcu_chain_forward_impl(p, t, training, stream, nullptr, 0);
}

static int hcu_chain_forward_impl(const hcu_unet_plan *p, const hcu_unet_tensors *t, int training,
                                  hcu_stream_t stream, void *images, int images_current) {
  if (!t || !t->x || !t->out || !t->params || !t->saved || !t->scratch)
    return fail(HCU_ERR_INVALID, "null argument");
  if (t->x_dtype != HCU_F32 && t->x_dtype != HCU_F16 && !(t->x_dtype == HCU_BF16 && p->es == 2))
    return fail(HCU_ERR_INVALID, "unsupported input dtype for this plan");
  if (p->in_cl && t->x_dtype != (p->es == 2 ? HCU_BF16 : HCU_F32))
    return fail(HCU_ERR_INVALID, "chain: a channels-last input must be of the compute dtype");
  if (training)
    for (const ChainOp &o : p->chain)
      if (o.kind == HCU_CHAIN_CONV && o.bn_relu && o.conv.bn.count <= 1.0)
        return fail(HCU_ERR_INVALID, "Expected more than 1 value per channel when training");
  if (p->n_bn && (!t->bn_running_mean || !t->bn_running_var))
    return fail(HCU_ERR_INVALID, "BatchNorm running statistics missing");
  return enqueue_chain_forward(*p, t, training, (hipStream_t)stream, images, images_current);
}

int hcu_chain_backward(const hcu_unet_plan *p, const hcu_unet_tensors *t, const float *dout, float *dx,
                       int training, int accumulate, hcu_stream_t stream) {
  return hcu_chain_backward_images(p, t, dout, dx, training, accumulate, stream, nullptr, 0);
}

size_t hcu_chain_weight_image_bytes(const hcu_unet_plan *p) { return p && p->is_chain ? p->img_bytes : 0; }

int hcu_chain_forward_images(const hcu_unet_plan *p, const hcu_unet_tensors *t, int training,
                             hcu_stream_t stream, void *images, int images_current) {
  if (!p || !p->is_chain) return fail(HCU_ERR_INVALID, "not a chain plan");
  if (!images) return fail(HCU_ERR_INVALID, "null weight-image buffer");
  if (images_current < 0 || images_current > 2) return fail(HCU_ERR_INVALID, "images_current must be 0, 1 or 2");
  return hcu_chain_forward_impl(p, t, training, stream, images, images_current);
}

int hcu_chain_backward_images(const hcu_unet_plan *p, const hcu_unet_tensors *t, const float *dout, float *dx,
                              int training, int accumulate, hcu_stream_t stream, void *images,
                              int images_current) {
  if (!p || !p->is_chain) return fail(HCU_ERR_INVALID, "not a chain plan");
  if (!t || !dout || !t->grads || !t->params || !t->saved || !t->scratch)
    return fail(HCU_ERR_INVALID, "null argument");
  return enqueue_chain_backward(*p, t, dout, dx, training, accumulate, (hipStream_t)stream, images, images_current);
}

}  // extern "C"
