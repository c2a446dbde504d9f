/*
 * hcunet.h -- C-ABI of the MI355X-native 3D U-Net training hot path.
 *
 * This library replaces the arithmetic behind the reference's Python operator
 * interface for ONE path: hcat.unet.Unet_Constructor forward + backward, the
 * pixel-weighted BCE loss (hcat.loss.cross_entropy, method='pixel') and the
 * Adam step that follows it in the reference training pattern -- plus the
 * callers either side of it: the tiled inference driver, the
 * input transforms and the reference's other losses.  The reference
 * binds no native code (it calls stock torch.nn ops), so each entry point below
 * names the reference symbol whose semantics it implements; the Python host
 * layer (hcunet_amd/, re-exported as hcat.unet / hcat.loss) binds these through
 * ctypes.
 *
 * Conventions
 *   - Every pointer is a device (HBM) pointer owned by the caller.  No entry
 *     point allocates device memory for tensors; scratch/saved workspaces are
 *     sized by the *_bytes / *_query functions and passed in.  One exception:
 *     creating a TRAINING plan times the best few convolution tilings on a
 *     private, grown-on-demand device arena (hipMalloc, kept for the process;
 *     HCU_BCONV_TUNE=0 disables the timing).
 *   - Work is enqueued asynchronously on `stream` (a hipStream_t, 0 = null
 *     stream).  The per-op launchers are stateless and re-entrant.
 *   - A network plan (hcu_unet_plan) is NOT read-only after creation: on first
 *     use it lazily creates, on the calling thread's current device, a private
 *     capture stream and up to 8 instantiated hipGraphs per distinct set of
 *     buffer pointers (guarded by a mutex), and for the backward a private
 *     weight-gradient stream plus fork/join/slot events.  The backward enqueues
 *     its weight-gradient branch on that private stream, ordered against the
 *     caller's stream by events (fork after the caller's prior work, join before
 *     the call returns its work to the caller's stream), so callers observe
 *     ordinary stream order.  Concurrent backwards of one plan serialise on the
 *     plan's mutex.  Call with the device of the tensors current (the Python
 *     layer does).  A failed capture destroys the branch stream; it is
 *     recreated on the next backward.
 *   - Return value: HCU_OK or an error code; no C++ exception crosses the ABI.
 *     hcu_last_error() returns a thread-local message for the last failure.
 *   - Activation tensors handled by the per-op entry points are channels-last
 *     fp32: [B][X][Y][Z][Cs] with Cs = round_up(C, 4).  The network entry points
 *     take the reference's NCXYZ ([B][C][X][Y][Z], PyTorch NCDHW) tensors.
 *   - Weight tensors are always in PyTorch layout: Conv3d [Cout][Cin/g][kx][ky][kz],
 *     ConvTranspose3d [Cin][Cout][kx][ky][kz].
 */
#ifndef HCUNET_H
#define HCUNET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *hcu_stream_t; /* hipStream_t */

enum {
  HCU_OK = 0,
  HCU_ERR_INVALID = 1,     /* bad argument (maps to ValueError / TypeError) */
  HCU_ERR_SHAPE = 2,       /* shape error   (maps to RuntimeError, as torch raises) */
  HCU_ERR_HIP = 3,         /* HIP runtime error */
  HCU_ERR_UNSUPPORTED = 4, /* configuration the reference itself rejects */
  HCU_ERR_WORKSPACE = 5    /* workspace too small */
};

enum { HCU_F32 = 0, HCU_F16 = 1, HCU_U8 = 2, HCU_BF16 = 3, HCU_U16 = 4, HCU_F64 = 5 };

const char *hcu_last_error(void);
int hcu_version(void);

/* ------------------------------------------------------------------------ */
/* Whole-network executor.                                                   */
/* Replaces: Unet_Constructor.__init__ shape logic  hcat/unet.py:16-123      */
/*           Unet_Constructor.forward               hcat/unet.py:125-143     */
/*           Down.forward / Up.forward / crop       hcat/unet.py:263-340     */
/*           and their autograd backward (torch.nn ops' derivatives).        */
/* ------------------------------------------------------------------------ */
#define HCU_MAX_LEVELS 12

typedef struct hcu_unet_spec {
  int levels;                       /* len(feature_sizes)                   */
  int in_channels, out_channels;
  int features[HCU_MAX_LEVELS];     /* feature_sizes                        */
  int k1[3], k2[3];                 /* kernel['conv1'], kernel['conv2']     */
  int d1[3], d2[3];                 /* dilation['conv1'], dilation['conv2'] */
  int g1, g2;                       /* groups['conv1'], groups['conv2']     */
  int up_k[3], up_s[3];             /* upsample_kernel, upsample_stride     */
  int pool_k[3];                    /* max_pool_kernel (kernel = stride)    */
  float bn_eps;                     /* BatchNorm3d eps (1e-5)               */
  float bn_momentum;                /* 0.1; < 0 means momentum=None         */
  int compute_dtype;                /* HCU_F32: fp32 throughout (the reference's
                                       arithmetic); HCU_BF16: bf16 activations,
                                       gradients and GEMM operands, fp32
                                       accumulation / statistics / parameters
                                       (torch.autocast(dtype=torch.bfloat16)) */
} hcu_unet_spec;

typedef struct hcu_unet_plan hcu_unet_plan;

/* Validates the spec against an input of [B, in_channels, X, Y, Z] and builds
 * the launch plan.  Fails with HCU_ERR_SHAPE where torch would raise (input
 * smaller than a kernel, pooled size 0, upsampled tensor larger than the skip
 * tensor so that torch.cat raises: hcat/unet.py:311-312). */
int hcu_unet_plan_create(const hcu_unet_spec *spec, int B, int X, int Y, int Z,
                         hcu_unet_plan **out);
void hcu_unet_plan_destroy(hcu_unet_plan *plan);

/* Plan flags.  HCU_PLAN_FORWARD_ONLY: inference (torch.no_grad) plan -- the
 * forward keeps no activation for a backward (they alternate between two
 * buffers of the largest activation), so saved_bytes is a small fraction of a
 * training plan's; hcu_unet_backward on it fails with HCU_ERR_INVALID.
 * Replaces the `with torch.no_grad(): unet(tile)` call of the reference's tiled
 * inference loop (hcat/segment.py:82-99), which keeps autograd off but still
 * runs the module's ordinary forward. */
#define HCU_PLAN_FORWARD_ONLY 1
int hcu_unet_plan_create_ex(const hcu_unet_spec *spec, int B, int X, int Y, int Z, int flags,
                            hcu_unet_plan **out);

/* out_shape[5] = output [B, out_channels, OX, OY, OZ]; n_params = number of
 * parameter scalars (flat layout = Unet_Constructor.parameters() order);
 * n_bn = number of BatchNorm3d modules; saved_bytes = forward->backward
 * workspace; scratch_bytes = per-call temporary workspace. */
int hcu_unet_plan_query(const hcu_unet_plan *plan, int64_t *out_shape,
                        int64_t *n_params, int *n_bn, size_t *saved_bytes,
                        size_t *scratch_bytes);

typedef struct hcu_unet_tensors {
  const float *x;          /* [B][Cin][X][Y][Z] of x_dtype (fp32 by default) */
  float *out;              /* [B][Cout][OX][OY][OZ] fp32                     */
  const float *params;     /* flat fp32, Unet_Constructor.parameters() order */
  float *grads;            /* flat fp32, same layout (backward only)         */
  float *const *bn_running_mean; /* n_bn pointers: down[i].batch1, batch2 ... */
  float *const *bn_running_var;  /*   then up[j].batch1, batch2 (module order) */
  int64_t *const *bn_num_batches_tracked;
  void *saved;             /* saved_bytes   */
  void *scratch;           /* scratch_bytes */
  int x_dtype;             /* HCU_F32, or with compute_dtype HCU_BF16 also
                              HCU_F16 / HCU_BF16 (16-bit volumes are read
                              directly by the channels-last staging kernel) */
} hcu_unet_tensors;

/* training != 0: BatchNorm uses batch statistics and updates running stats
 * (nn.BatchNorm3d train mode); 0: running statistics (eval mode). */
int hcu_unet_forward(const hcu_unet_plan *plan, const hcu_unet_tensors *t,
                     int training, hcu_stream_t stream);

/* dout: [B][Cout][OX][OY][OZ] gradient of the output.  Writes (accumulate=0)
 * or adds (accumulate=1) parameter gradients into t->grads; dx (nullable)
 * receives the input gradient [B][Cin][X][Y][Z].  Must follow a forward with
 * the same plan, tensors and training flag. */
int hcu_unet_backward(const hcu_unet_plan *plan, const hcu_unet_tensors *t,
                      const float *dout, float *dx, int training,
                      int accumulate, hcu_stream_t stream);

/* Introspection of the saved workspace (tests, debugging): one record per
 * BatchNorm3d in module order (down[i].batch1, batch2, ..., up[j].batch1,
 * batch2).  y_offset: byte offset in `saved` of that layer's pre-BatchNorm conv
 * output y, channels-last [B][X][Y][Z][Cs] of elem_bytes-sized elements;
 * coef_offset: byte offset of 6 fp32 arrays of Cs (scale, shift, mean, invstd,
 * c1, c0) with which the forward applied relu(y*scale + shift).  Returns the
 * number of records (written up to max). */
typedef struct hcu_bn_layer_info {
  int64_t y_offset, coef_offset;
  int B, X, Y, Z, C, Cs;
  int elem_bytes;
  int pad;
} hcu_bn_layer_info;
int hcu_unet_plan_bn_layers(const hcu_unet_plan *plan, hcu_bn_layer_info *out, int max);

/* ------------------------------------------------------------------------ */
/* Layer chains: a short sequence of Conv3d [+ BatchNorm3d + ReLU] /         */
/* MaxPool3d / ConvTranspose3d [+ cat(U, U)] ops run by the same kernels and */
/* fusions as the network executor, as one autograd node.  Replaces:         */
/*   Down.forward / Up.forward of hcat/unet.py:263-266, 309-315 called on    */
/*   their own, and the layers of hcat/r_unet.py: its Down / Up (padding,    */
/*   :249-336), f (:232-246), RDCNet's strided / 1x1 / padded ConvTranspose3d */
/*   (:207-227) and StackedDilation's dilated 5^3 convolutions (:339-364).   */
/* Input / output tensors are NCXYZ fp32 (the output with the last op's      */
/* BatchNorm + ReLU applied); parameters / gradients live in flat fp32       */
/* buffers at the per-op offsets; BatchNorm running statistics are passed    */
/* per BatchNorm op (hcu_unet_tensors' arrays, in op order).  Plans are      */
/* hcu_unet_plan objects (hcu_unet_plan_destroy frees them).                 */
/* ------------------------------------------------------------------------ */
enum { HCU_CHAIN_CONV = 0, HCU_CHAIN_POOL = 1, HCU_CHAIN_CONVT = 2 };
#define HCU_CHAIN_MAX_OPS 16
typedef struct hcu_chain_op {
  int kind;                  /* HCU_CHAIN_*                                   */
  int out_channels;          /* CONV / CONVT                                  */
  int k[3], stride[3], dil[3], pad[3];   /* CONV; CONVT: k, stride, pad (crop) */
  int groups;                /* CONV                                          */
  int bn_relu;               /* CONV: followed by BatchNorm3d + ReLU          */
  int cat_fold;              /* CONV right after a CONVT: its input is cat(U, U)
                                (hcat/unet.py:311-312; the weight has 2*C input
                                channels per group and is folded)              */
  int64_t w_off, b_off;      /* float offsets of weight / bias (b_off < 0: none) */
  int64_t gamma_off, beta_off;   /* BatchNorm weight / bias (bn_relu)         */
} hcu_chain_op;
typedef struct hcu_chain_spec {
  int n_ops;
  int in_channels;
  hcu_chain_op ops[HCU_CHAIN_MAX_OPS];
  float bn_eps, bn_momentum;     /* < 0 momentum: cumulative average (None)   */
  int compute_dtype;             /* HCU_F32 or HCU_BF16 (as hcu_unet_spec)    */
  /* Channels-last boundaries (the recurrences of hcat/r_unet.py:219-225 keep
   * their state in the executor's layout between chains instead of NCXYZ):
   * in_cl / out_cl != 0: t->x / t->out (and dx / dout) are [B][X][Y][Z][Cs]
   * tensors of the compute dtype, Cs = the channel count rounded up to 8
   * (bf16) / 4 (fp32), padding channels zero.  in_part_channels > 0 (with
   * in_cl; the first op a Conv3d): the input is the channel-wise cat of
   * in_channels / in_part_channels such tensors, each padded on its own
   * (Cs = parts * round_up(in_part_channels)), i.e. torch.cat(..., dim=-1)
   * of channels-last chain outputs.  out_cl needs a last op that is a Conv3d
   * without BatchNorm. */
  int in_cl, out_cl, in_part_channels;
} hcu_chain_spec;
/* Fails with HCU_ERR_SHAPE where torch would raise for the input shape, with
 * HCU_ERR_UNSUPPORTED for op combinations the chain does not run (a MaxPool3d
 * not fed by Conv3d + BatchNorm3d + ReLU, a strided Conv3d's input gradient). */
int hcu_chain_plan_create(const hcu_chain_spec *spec, int B, int X, int Y, int Z,
                          hcu_unet_plan **out);
int hcu_chain_plan_query(const hcu_unet_plan *plan, int64_t *out_shape, int *n_bn,
                         size_t *saved_bytes, size_t *scratch_bytes);
/* t->x, t->out: NCXYZ fp32 (or channels-last, in_cl / out_cl); t->params /
 * t->grads: flat buffers of the op offsets; training as hcu_unet_forward. */
int hcu_chain_forward(const hcu_unet_plan *plan, const hcu_unet_tensors *t, int training,
                      hcu_stream_t stream);
int hcu_chain_backward(const hcu_unet_plan *plan, const hcu_unet_tensors *t, const float *dout,
                       float *dx, int training, int accumulate, hcu_stream_t stream);
/* The same with the packed weight images (the executor's re-layout of the
 * op weights, normally rebuilt in `saved` by every forward) kept in a
 * caller-owned buffer of hcu_chain_weight_image_bytes(plan) that outlives the
 * calls: a recurrence applying one chain several times per step re-lays them
 * once.  images_current: 0 = re-lay (the parameters changed since the images
 * were written), 1 = the buffer holds the forward images of the current
 * parameters (an eval forward wrote it), 2 = forward and input-gradient
 * images (a training forward wrote it).  The backward must be given the
 * buffer its forward used; after an eval-mode forward (images_current < 2)
 * it writes the input-gradient images into that buffer, so it is not const. */
size_t hcu_chain_weight_image_bytes(const hcu_unet_plan *plan);
int hcu_chain_forward_images(const hcu_unet_plan *plan, const hcu_unet_tensors *t, int training,
                             hcu_stream_t stream, void *images, int images_current);
int hcu_chain_backward_images(const hcu_unet_plan *plan, const hcu_unet_tensors *t,
                              const float *dout, float *dx, int training, int accumulate,
                              hcu_stream_t stream, void *images, int images_current);

/* The gated recurrence of RecursiveUnet.forward (hcat/r_unet.py:150-155), n
 * fp32 elements: h = tanh(hp), z = sigmoid(zp), out = h_prev*z + (-1*z*h);
 * h_prev == NULL means ones (the t == 0 state, :152-153).  The backward writes
 * d(hp), d(zp) and (nullable) d(h_prev) from d(out). */
int hcu_gate_fwd(const float *hp, const float *zp, const float *h_prev, float *out, int64_t n,
                 hcu_stream_t stream);
int hcu_gate_bwd(const float *hp, const float *zp, const float *h_prev, const float *dout, float *dhp,
                 float *dzp, float *dh_prev, int64_t n, hcu_stream_t stream);

/* Channel cat of channels-last tensors ([rows][C], C the padded channel
 * slots): split = 0 writes full[r] = parts[0][r] ++ parts[1][r] ++ ...,
 * split = 1 the reverse (the cat's backward: one contiguous gradient per
 * part).  1..8 parts, 16-byte aligned, part_row_bytes multiples of 16.
 * Replaces torch.cat(..., dim=1) on RDCNet's recurrence (hcat/r_unet.py:223
 * cat(x, y) and :362 the StackedDilation cat) and its autograd backward. */
int hcu_cl_cat(void *const *parts, const int *part_row_bytes, int nparts, void *full, int64_t rows,
               int split, hcu_stream_t stream);

/* RDCNet's residual state under bf16 autocast (hcat/r_unet.py:223-225):
 * out = float(m) + y (fp32) and out_c = its bf16 cast, n elements (a
 * multiple of 8; m, out_c bf16).  The backward writes dy = g32 + float(gc)
 * and dm = bf16(dy); g32 or gc may be NULL (no contribution). */
int hcu_resid_fwd(const void *m, const float *y, float *out, void *out_c, int64_t n, hcu_stream_t stream);
int hcu_resid_bwd(const float *g32, const void *gc, float *dy, void *dm, int64_t n, hcu_stream_t stream);

/* The channel cat + 1x1x1 Conv3d (no BatchNorm) of RDCNet's recurrence on
 * bf16 channels-last channel parts, without the cat: hcat/r_unet.py:223
 * cat(x, y) -> RDCBlock.conv (:372-374) and :362 the cat of the dilated
 * branches -> StackedDilation.out_conv (:354-364), with their autograd
 * backward.  parts[i]: [nvox][part_cs] bf16 with part_c real channels
 * (Cin = nparts * part_c, 1..8 parts, part_cs a multiple of 8, 16-byte
 * aligned); w: the PyTorch weight [Cout][Cin] fp32, b: [Cout] or NULL; out /
 * dout: [nvox][out_cs] bf16 (out_cs = Cout rounded up to 8, padding 0).
 * Backward: dparts (NULL: no input gradients) in the parts' layout; dw / db
 * (db nullable) overwritten or, accumulate != 0, added to; work: scratch of
 * hcu_pw_conv_work_floats(...) floats.  Channel counts: nparts * part_cs <= 96
 * slots, out_cs <= 32. */
int hcu_pw_conv_forward(const void *const *parts, int nparts, int part_c, int part_cs, const float *w,
                        const float *b, void *out, int64_t nvox, int Cout, int out_cs, hcu_stream_t stream);
size_t hcu_pw_conv_work_floats(int64_t nvox, int nparts, int part_cs, int Cout);
int hcu_pw_conv_backward(const void *const *parts, int nparts, int part_c, int part_cs, const float *w,
                         const void *dout, int Cout, int out_cs, void *const *dparts, float *dw, float *db,
                         int64_t nvox, float *work, size_t work_floats, int accumulate, hcu_stream_t stream);

/* out = parts[0] + parts[1] + ... (n elements, fp32 accumulation in input
 * order, one rounding; bf = 1: bf16 tensors, else fp32; NULL parts skipped;
 * at most 16).  The gradient of a tensor read by several chains (RDCNet:
 * hcat/r_unet.py:223-225,362), which autograd would sum pairwise. */
int hcu_sum_parts(const void *const *parts, int nparts, void *out, int64_t n, int bf, hcu_stream_t stream);

/* Data-parallel overlap (hcunet_amd/dist.py): with events set, every later  */
/* hcu_unet_backward on `plan` records ev_decoder on its weight-gradient     */
/* stream once the decoder's parameter gradients (up_steps, out_conv) are    */
/* final, and ev_deep once those of encoder levels >= deep_level are, so a   */
/* caller can reduce those gradient ranges while the rest of the backward    */
/* runs (hcu_stream_wait_event on its communication stream).  Each event    */
/* costs one extra batched weight-gradient finalize launch.  NULL events:    */
/* nothing recorded (the default).  The events stay owned by the caller.     */
int hcu_unet_set_grad_events(hcu_unet_plan *plan, void *ev_decoder, void *ev_deep, int deep_level);
/* 1 when hcu_unet_backward records those events (direct launches), 0 when  */
/* its backward is replayed from a captured graph (HCU_GRAPHS=1), where a    */
/* record would only be a capture dependency: reduce after the backward.     */
int hcu_unet_grad_events_live(const hcu_unet_plan *plan);
int hcu_event_create(void **ev);          /* hipEventDisableTiming */
int hcu_event_destroy(void *ev);
int hcu_stream_wait_event(hcu_stream_t stream, void *ev);

/* Data parallel (hcunet_amd/dist.py): n <= 128 fp32 vectors (the BatchNorm
 * running statistics) gathered into (unpack = 0) or scattered from
 * (unpack = 1) one contiguous buffer in one launch, in order. */
int hcu_gather_vectors(float *const *vecs, const int *lens, int n, float *buf, int unpack,
                       hcu_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Loss.  Replaces hcat.loss.cross_entropy(pred, mask, pwl, method='pixel')  */
/* hcat/loss.py:5-101: crop mask/pwl top-left to pred (:51-53), BCE with     */
/* logits * (pwl + 1) computed in pwl's dtype (:65,71-72), mean (:101).      */
/* pwl == NULL means weight 2 everywhere (:46-47).                            */
/* ------------------------------------------------------------------------ */
size_t hcu_loss_pixel_scratch_bytes(int64_t n_pred);
/* pred [B][C][PX][PY][PZ] fp32; mask/pwl [B][C][MX][MY][MZ] of dtype
 * mask_dtype / pwl_dtype (HCU_F32, HCU_F16, HCU_U8).  loss[0] <- mean loss;
 * dpred <- d(loss)/d(pred) for an upstream gradient of 1 (nullable). */
int hcu_loss_pixel_fwd(const float *pred, int B, int C, int PX, int PY, int PZ,
                       const void *mask, int mask_dtype, const void *pwl,
                       int pwl_dtype, int MX, int MY, int MZ, float *loss,
                       float *dpred, void *scratch, size_t scratch_bytes,
                       hcu_stream_t stream);
/* dst[i] = src[i] * scale[0] (scale is a device scalar: the upstream grad). */
int hcu_scale_by_device_scalar(const float *src, const float *scale, float *dst,
                               int64_t n, hcu_stream_t stream);

/* ------------------------------------------------------------------------ */
/* The reference's other losses (hcat/loss.py:5-178), same geometry as     */
/* hcu_loss_pixel_fwd.  mode: 0 cross_entropy(method='sigmoid') (:38-40,     */
/* :95-97), 1 method='worst_z' (:74-80), 2 dice (:104-126), 3 L1Loss         */
/* (:128-152), 4 MSELoss (:154-178), 5 plain BCE mean ('random' with no      */
/* positive pixel, :84-85), 6 'random' (hcu_loss_random_fwd, :86-93).        */
/* Forward writes loss[0] and aux (the scalars the gradient needs: 1 float,  */
/* 2 for dice, PZ for worst_z); backward writes dpred = dloss/dpred *        */
/* grad_out[0].  zscale (worst_z): torch.linspace(1, 2, PZ) ** 2 (:76).      */
/* ------------------------------------------------------------------------ */
size_t hcu_loss_ext_scratch_bytes(int mode, int64_t n_pred, int PZ);
int hcu_loss_ext_fwd(int mode, const float *pred, int B, int C, int PX, int PY, int PZ,
                     const void *mask, int mask_dtype, const void *pwl, int pwl_dtype,
                     int MX, int MY, int MZ, const float *zscale, float *loss, float *aux,
                     void *scratch, size_t scratch_bytes, hcu_stream_t stream);
int hcu_loss_ext_bwd(int mode, const float *pred, int B, int C, int PX, int PY, int PZ,
                     const void *mask, int mask_dtype, const void *pwl, int pwl_dtype,
                     int MX, int MY, int MZ, const float *aux, const int *counts,
                     const float *grad_out, float *dpred, hcu_stream_t stream);
/* 'random' (hcat/loss.py:82-93): rows = hcu_loss_random_rows(n);
 * hcu_loss_random_count writes counts[rows][2] = (#mask==1, #mask==0) per row
 * of the flattened cropped mask; the caller draws pos_ind / neg_ind (int64,
 * n each) from its generator as the reference does and passes the exclusive
 * row offsets; hcu_loss_random_fwd compacts the pixel lists (pos_list /
 * neg_list: #mask==1 / #mask==0 ints), gathers the 2n drawn pixels, writes
 * the mean BCE and adds each drawn pixel's draw count into counts_px
 * (n_pred ints, zeroed by the caller) for hcu_loss_ext_bwd(mode 6). */
int hcu_loss_random_rows(int64_t n_pred);
int hcu_loss_random_count(const float *pred, int B, int C, int PX, int PY, int PZ,
                          const void *mask, int mask_dtype, int MX, int MY, int MZ,
                          int *counts, hcu_stream_t stream);
int hcu_loss_random_fwd(const float *pred, int B, int C, int PX, int PY, int PZ,
                        const void *mask, int mask_dtype, int MX, int MY, int MZ,
                        const int *offsets, int *pos_list, int *neg_list,
                        const int64_t *pos_ind, const int64_t *neg_ind, int n,
                        int *counts_px, float *loss, float *aux, void *scratch,
                        size_t scratch_bytes, hcu_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Input path.  Replaces, for B raw volumes at once, the     */
/* reference's to_float (hcat/transforms.py:94-116) -> reshape (:139-157)    */
/* -> normalize (:257-283) -> to_tensor (:118-137) chain: src [B][Z][Y][X][C] */
/* of src_dtype HCU_U16 / HCU_U8 / HCU_F64; to_float: scale by 2^-16 / 2^-8; */
/* reshape: output [B][C][X][Y][Z] (else [B][C][Z][Y][X]); mean/std (host    */
/* arrays of C doubles, nullable): (v + -mean) / std.  Arithmetic in float64, */
/* one round-to-nearest-even to fp16: bit-identical to the reference.  dst:  */
/* fp16.  Fails with HCU_ERR_INVALID for other dtypes (the reference's       */
/* TypeError, :113-114).                                                      */
/* ------------------------------------------------------------------------ */
int hcu_ingest_volume(const void *src, int src_dtype, int B, int Z, int Y, int X, int C,
                      int to_float, int reshape, const double *mean, const double *std,
                      void *dst, hcu_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Optimizer.  Replaces torch.optim.Adam.step (tests/r_unet_test.py:24,56)   */
/* for a flat parameter buffer: m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;  */
/* p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps); L2 weight decay.     */
/* ------------------------------------------------------------------------ */
int hcu_adam_step(float *p, const float *g, float *m, float *v, int64_t n,
                  float lr, float beta1, float beta2, float eps,
                  float weight_decay, int64_t step, float grad_scale,
                  hcu_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Per-op entry points (channels-last activations).  Used by the parity     */
/* tests to localise errors; the network executor calls the same kernels.    */
/* ------------------------------------------------------------------------ */
typedef struct hcu_conv_desc {
  int B, Cin, Cout;        /* logical channels                                */
  int X, Y, Z;             /* input spatial dims                              */
  int k[3], stride[3], dil[3];
  int groups;              /* Conv3d only                                     */
  int transposed;          /* 0: nn.Conv3d (valid, stride 1 only)
                              1: nn.ConvTranspose3d (pad 0, dil 1, groups 1) */
  int dtype;               /* HCU_F32: fp32 activations, Cs = round_up(C, 4);
                              HCU_BF16: bf16 activations (x, y, dy, dx),
                              Cs = round_up(C, 8); weights / dw / bias fp32 */
} hcu_conv_desc;

size_t hcu_conv_scratch_bytes(const hcu_conv_desc *d);
/* Output spatial dims of the op described by d (out[3]). */
int hcu_conv_out_dims(const hcu_conv_desc *d, int *out);
/* nn.Conv3d / nn.ConvTranspose3d forward: y = conv(x, w) + bias. */
int hcu_conv_fwd_cl(const hcu_conv_desc *d, const float *x, const float *w,
                    const float *bias, float *y, void *scratch,
                    size_t scratch_bytes, hcu_stream_t stream);
/* d(input) from d(output). */
int hcu_conv_dgrad_cl(const hcu_conv_desc *d, const float *dy, const float *w,
                      float *dx, void *scratch, size_t scratch_bytes,
                      hcu_stream_t stream);
/* d(weight), d(bias) (nullable) from input and d(output); overwrite. */
int hcu_conv_wgrad_cl(const hcu_conv_desc *d, const float *x, const float *dy,
                      float *dw, float *dbias, void *scratch,
                      size_t scratch_bytes, hcu_stream_t stream);

/* nn.MaxPool3d(kernel=stride=k, floor mode) forward, channels-last. */
int hcu_maxpool_fwd_cl(int B, int C, int X, int Y, int Z, const int *k,
                       const float *x, float *y, hcu_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Tiled inference (hcat.segment.predict_segmentation_mask, hcat/segment.py:21-136;
 * hcat.utils.pad_image_with_reflections / calculate_indexes, hcat/utils.py:33-124). */
/* ------------------------------------------------------------------------ */
#define HCU_TILE_BATCH_MAX 64
/* out[b][c][i][j][k] = image[0][c][r(o_b + (i,j,k))] for n_tiles tiles of
 * tile_dims, o_b = origins[3b..3b+2] in padded coordinates; r() is numpy's
 * reflection padding (image[pad-1::-1], image, image[-1:-pad-1:-1]) with
 * pad_lo[d] = min(pad, size) (pad_image_with_reflections, utils.py:51-71), and
 * with clean != 0 values are cleaned as segment.py:66-67 does (NaN -> 0,
 * +-Inf -> 1).
 * image: [1][C][X][Y][Z] of image_dtype (HCU_F32 or HCU_F16), device memory;
 * out: [n_tiles][C][tile_dims] fp32, the network input batch. */
int hcu_tile_gather(const void *image, int image_dtype, int C, int X, int Y, int Z,
                    const int *pad_lo, const int *origins, int n_tiles, const int *tile_dims,
                    int clean, float *out, hcu_stream_t stream);
/* mask[dst_lo + w] = f(out[crop_lo + w']) over the write box write_dims, with
 * w' = w or 0 along dimensions where bcast[d] != 0 (torch broadcasting of a
 * size-1 valid_out dimension, segment.py:121-123); out is one channel of one
 * tile's network output [out_dims]; f = the in-place sigmoid chain of
 * segment.py:110-113 (x*-1, exp, +1, pow(-1)), then 1/0 for f > thr when
 * threshold != 0 (segment.py:116-119).  mask: [mask_dims] of HCU_F32 or HCU_U8. */
int hcu_tile_scatter(const float *out, const int *out_dims, const int *crop_lo, const int *bcast,
                     void *mask, int mask_dtype, const int *mask_dims, const int *dst_lo,
                     const int *write_dims, int threshold, float thr, hcu_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Measurement: opt-in HIP-event timing of every library launch (bench.py). */
/* ------------------------------------------------------------------------ */
int hcu_timing_enable(int max_launches);
int hcu_timing_disable(void);
/* on != 0: report per network layer ("kernel@layer") instead of per symbol. */
int hcu_timing_detail(int on);
/* Prefix of this thread's launch tags in the detail records (a chain's name,
 * hcunet_amd/chain.py); empty or null: none. */
int hcu_timing_prefix(const char *prefix);
/* One line per kernel symbol: name\tcount\ttotal_ms\tflops\tbytes (totals
 * over launches; flops/bytes are algorithmic).  Returns bytes needed. */
int64_t hcu_timing_report(char *buf, int64_t len);

/* ------------------------------------------------------------------------ */
/* Convolution tiling table.  Plans pick each convolution's tiling from a    */
/* persistent table (tuning/bconv_gfx950.txt next to the library, or         */
/* $HCU_TUNE_FILE) keyed by the convolution's signature, so every process    */
/* and every data-parallel rank runs the same kernels (same summation order). */
/* mode 0: cost model only; 1: table, cost model on a miss (deterministic    */
/* across processes -- hcunet_amd.dist selects it); 2: table, the best few   */
/* candidates timed on a miss (default; $HCU_BCONV_TUNE sets the initial     */
/* mode).                                                                    */
/* ------------------------------------------------------------------------ */
int hcu_tuning_set_mode(int mode);
int hcu_tuning_get_mode(void);
/* Table entries; *timed (nullable) = entries timed by this process. */
int64_t hcu_tuning_entries(int64_t *timed);
/* Writes the table to path (NULL: the library's table file); entries or <0. */
int64_t hcu_tuning_save(const char *path);

#ifdef __cplusplus
}
#endif
#endif /* HCUNET_H */
