/*
 * jabd.h — C-ABI of libjabd.so, the MI355X (gfx950) hot path of JABD.
 *
 * Every entry point takes raw device pointers, int64 sizes and a hipStream_t
 * (passed as an opaque `void*`; 0 = the null stream).  No torch types cross
 * this boundary.  All buffers belong to the caller; scratch memory is passed
 * in as a workspace whose size is queried first.  Functions return a status
 * (JABD_OK == 0); on failure `jabd_last_error()` gives the text (thread-local).
 * Every kernel launches on the caller's stream and no function synchronises
 * the device unless its comment says so.
 *
 * The reference (/root/reference/JABD2080ti) is pure Python over PyTorch;
 * each function below cites the reference interface it replaces.  The Python
 * binding (ctypes) lives in the package's `jabd_amd/_lib.py`; see
 * INTEGRATION.md for how the reference's modules bind to it.
 */
#ifndef JABD_H_
#define JABD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* jabd_stream_t; /* hipStream_t */

enum {
  JABD_OK = 0,
  JABD_EINVAL = 1, /* bad shape / pointer / argument */
  JABD_EHIP = 2,   /* HIP runtime or launch error   */
  JABD_EWS = 3,    /* workspace too small           */
};

const char* jabd_version(void);
/* sizeof the argument structs (0: jabd_conv_args, 1: jabd_dw_args,
 * 2: jabd_expdw_args; -1 otherwise) — for bindings to check their mirrors. */
int64_t jabd_abi_struct_size(int32_t which);
/* Copies the calling thread's last error message into buf (NUL-terminated). */
int jabd_last_error(char* buf, size_t len);

/* ------------------------------------------------------------------------ *
 * A6/A10 box decoding — utils/utils_bbox.py:29-34 (decode) and :39-46
 * (decode_landm).  loc [B,A,4], landm [B,A,10], priors [A,4] (cx,cy,w,h).
 * ------------------------------------------------------------------------ */
int jabd_decode_f32(const float* loc, const float* priors, int64_t batch,
                    int64_t num_priors, float var0, float var1, float* boxes,
                    jabd_stream_t stream);
int jabd_decode_landm_f32(const float* pre, const float* priors, int64_t batch,
                          int64_t num_priors, float var0, float* landms,
                          jabd_stream_t stream);

/* ------------------------------------------------------------------------ *
 * A10 greedy NMS — torchvision.ops.nms as called at utils/utils_bbox.py:275
 * (CPU-kernel semantics: stable descending score sort, IoU = inter /
 * (area_i + area_j - inter) in fp32, suppress when IoU > iou_threshold
 * compared in double).  Batched: B independent images of up to n boxes.
 *   boxes  [B, n, 4] with row stride `box_stride` floats (>= 4) and image
 *          stride `box_bstride` floats; scores likewise with `score_stride`
 *          / `score_bstride` (scores may alias a column of boxes).
 *   n_valid   nullable device int64[B]: image b uses its first n_valid[b] rows.
 *   score_threshold: rows with score < threshold are dropped before NMS
 *          (utils/utils_bbox.py:266-267); pass -INFINITY to keep all rows.
 *   keep   device int64[B, n]: kept row indices (into the unfiltered input),
 *          in decreasing-score order; n_keep device int64[B].
 * ------------------------------------------------------------------------ */
int jabd_nms_workspace_size(int64_t batch, int64_t n, size_t* bytes);
int jabd_batched_nms_f32(const float* boxes, int64_t box_stride,
                         int64_t box_bstride, const float* scores,
                         int64_t score_stride, int64_t score_bstride,
                         const int64_t* n_valid, int64_t batch, int64_t n,
                         double iou_threshold, float score_threshold,
                         int64_t* keep, int64_t* n_keep, void* ws,
                         size_t ws_bytes, jabd_stream_t stream);

/* Measurement helper: after jabd_batched_nms_f32 with the same (batch, n,
 * ws), copy to host arrays each image's number of exact IoU tests made by
 * the grid producer (candidate pairs), its off-block suppressing pairs, and
 * its producer (0 = grid, != 0 = dense: every pair tested).  Synchronises
 * the stream; batch <= 254. */
int jabd_nms_pair_stats(const void* ws, size_t ws_bytes, int64_t batch, int64_t n,
                        int64_t* tested, int32_t* hits, int32_t* dense, jabd_stream_t stream);

/* The NMS pipeline's sort and scan (hand-written wavefront radix sort and
 * scan, radix.hip), exported so they are tested on their own.  torchvision's
 * nms sorts the scores descending, stable (utils/utils_bbox.py:275); the
 * batched pipeline sorts [image | ~score | row] keys and its grid producer's
 * cell keys with this sort, and forms its CSR offsets with this scan.
 *   jabd_sort_u64: stable sort of n uint64 keys (with int32 values when
 *     vals_in != NULL) by key bits [bit_lo, bit_lo + 8 npass), 1 <= npass <= 8,
 *     n < 2^30; keys_in is not modified.  skip_ones != 0: keys equal to ~0
 *     do not keep a lower pass from being skipped as constant (they sort last
 *     either way).  Keys/values out must not alias the inputs.
 *   jabd_scan_excl_i32: out[i] = in[0] + ... + in[i-1] (int32, exact). */
int jabd_sort_workspace_size(int64_t n, int32_t with_values, size_t* bytes);
int jabd_sort_u64(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* vals_in,
                  int32_t* vals_out, int64_t n, int32_t bit_lo, int32_t npass, int32_t skip_ones,
                  void* ws, size_t ws_bytes, jabd_stream_t stream);
int jabd_scan_workspace_size(int64_t n, size_t* bytes);
int jabd_scan_excl_i32(const int32_t* in, int32_t* out, int64_t n, void* ws, size_t ws_bytes,
                       jabd_stream_t stream);

/* ------------------------------------------------------------------------ *
 * predict.py:162-181 fused: decode + decode_landm + conf[:,1] + score filter
 * + NMS, for B images at once.  conf is the eval-mode softmax [B,A,2].
 * out [B, A, 15] receives the kept rows (x1,y1,x2,y2,score,10 landmarks) in
 * NMS order, compacted; n_keep int64[B].  Workspace: jabd_detect_workspace_size.
 * ------------------------------------------------------------------------ */
int jabd_detect_workspace_size(int64_t batch, int64_t num_priors, size_t* bytes);
int jabd_detect_f32(const float* loc, const float* conf, const float* landm,
                    const float* priors, int64_t batch, int64_t num_priors,
                    float var0, float var1, float conf_threshold,
                    double nms_threshold, float* out, int64_t* n_keep,
                    void* ws, size_t ws_bytes, jabd_stream_t stream);

/* ------------------------------------------------------------------------ *
 * A7/A8 anchor matching + encoding — nets/retinaface_training.py:93-162
 * (match/encode/encode_landm) for a whole batch in one pass.
 *   targets  [T, 15] device fp32: the B per-image target tensors concatenated
 *            (x1,y1,x2,y2, 10 landmark coords, label), `offsets` device
 *            int64[B+1] into its rows; max_gt = max rows of one image (host).
 *   priors   [A, 4] (cx,cy,w,h).
 *   loc_t [B,A,4], conf_t int64 [B,A], landm_t [B,A,10] (outputs).
 * Images with zero targets are the caller's error (the reference's `match`
 * fails on them too: max over an empty dim).
 * ------------------------------------------------------------------------ */
int jabd_match_workspace_size(int64_t batch, int64_t num_priors, size_t* bytes);
int jabd_match_encode_f32(const float* targets, const int64_t* offsets,
                          int64_t batch, int64_t max_gt, const float* priors,
                          int64_t num_priors, float threshold, float var0,
                          float var1, float* loc_t, int64_t* conf_t,
                          float* landm_t, void* ws, size_t ws_bytes,
                          jabd_stream_t stream);

/* match_iou() — nets/retinaface_training_DIOU.py:176-246 (the DIoU variant's
 * matcher): same assignment and landmark encoding as jabd_match_encode_f32,
 * but loc_t[B,A,4] holds the matched truth corners (x1,y1,x2,y2) unencoded
 * (:230 `loc = matches`).  Same arguments and workspace. */
int jabd_match_iou_f32(const float* targets, const int64_t* offsets,
                       int64_t batch, int64_t max_gt, const float* priors,
                       int64_t num_priors, float threshold, float var0,
                       float var1, float* loc_t, int64_t* conf_t,
                       float* landm_t, void* ws, size_t ws_bytes,
                       jabd_stream_t stream);

/* letterbox_image + preprocess_input — utils/utils.py:8-19,27-29 as
 * predict.py:122,143-152 chains them (§8f rank 3).  src: device float32
 * [batch, ih, iw, 3] (the np.float32 image); the image is resized to
 * nw = int(iw*s), nh = int(ih*s), s = min(w/iw, h/ih) (cv2 INTER_LINEAR float
 * path, restated) and pasted centred on an h x w canvas of `fill` (84 in the
 * reference).  nchw = 0: dst float32 [batch, h, w, 3] (letterbox_image's
 * output); nchw = 1: dst float32 [batch, 3, h, w] = canvas - mean3[c] (host
 * float[3], (104,117,123) in the reference), i.e. the network input. */
int jabd_letterbox_f32(const float* src, int64_t batch, int ih, int iw,
                       float* dst, int h, int w, float fill,
                       const float* mean3, int nchw, jabd_stream_t stream);

/* retinaface_correct_boxes (utils/utils_bbox.py:9-24, only when letterbox
 * != 0) followed (to_pixels != 0) by predict.py:195-196's rescale of the
 * normalised box and landmark columns to image pixels, in place on device rows
 * float32 [n, 15] (jabd_detect_f32's output).  Column 4 (score) untouched.
 * Every step rounds as numpy's float64 math assigned back to float32. */
int jabd_correct_boxes_f32(float* rows, int64_t n, int input_h, int input_w,
                           int image_h, int image_w, int letterbox,
                           int to_pixels, jabd_stream_t stream);

/* GPU augmentation — utils/dataloader.py:71-115 (get_random_data, image part)
 * + :62-64 (preprocess_input, CHW), §8f rank 2.  src: device uint8 RGB
 * [ih, iw, 3] (the PIL image as an array).  The host draws the reference's
 * random values (nw, nh, dx, dy, flip, hue, sat, val) in its np.random order;
 * the device resizes (PIL BICUBIC, restated), pastes at (dx, dy) on grey 128
 * of h x w, flips, applies the HSV jitter (cv2 float HSV, restated) and writes
 * dst float32 [3, h, w] = rgb*255 - (104, 117, 123).  Workspace: u8 [ih, nw, 3]. */
int jabd_augment_workspace_size(int ih, int nw, size_t* bytes);
int jabd_augment_u8(const uint8_t* src, int ih, int iw, int nw, int nh, int h,
                    int w, int dx, int dy, int flip, double hue, float sat,
                    float val, float* dst, void* ws, size_t ws_bytes,
                    jabd_stream_t stream);

/* WIDER FACE evaluation core — utils/evaluation.py:255-305 (image_eval +
 * img_pr_info) summed over images (:347-375), §8f rank 3.  Device float64:
 * pred [total_preds, 5] (x, y, w, h, normalised score) and gt [total_gts, 4]
 * (x, y, w, h) rows per image by offsets [num_images + 1]; ignore uint8 per gt
 * (1 = in the setting's keep list).  Images with no preds or no gts are
 * skipped (:364-365).  pr_curve [thresh_num, 2] (device, caller-zeroed) is
 * ACCUMULATED: += (proposals, recalled) per threshold, exact (integer sums). */
int jabd_wider_eval_workspace_size(int64_t total_preds, int64_t total_gts,
                                   size_t* bytes);
int jabd_wider_eval_f64(const double* pred, const int64_t* pred_offsets,
                        const double* gt, const uint8_t* ignore,
                        const int64_t* gt_offsets, int64_t num_images,
                        int64_t total_preds, int64_t total_gts,
                        double iou_thresh, int thresh_num, double* pr_curve,
                        void* ws, size_t ws_bytes, jabd_stream_t stream);

/* Bicubic align_corners=True resize of NHWC fp32 [batch, H, W, C] to
 * [batch, OH, OW, C] — the CSAF fusion of the bicubic FPN variant
 * (train_mobilenetV3_ecagai.py:270,279, F.interpolate(..., mode="bicubic",
 * align_corners=True)), §8f rank 4.  The backward zeroes grad_x and scatters. */
int jabd_upsample_bicubic_ac_f32(const float* x, int64_t batch, int H, int W,
                                 int C, float* y, int OH, int OW,
                                 jabd_stream_t stream);
int jabd_upsample_bicubic_ac_bwd_f32(const float* grad_y, int64_t batch, int H,
                                     int W, int C, float* grad_x, int OH, int OW,
                                     jabd_stream_t stream);

/* General-width NLM attention core (the BECA variant's NLM(40): ch = 40, PSP
 * (1,3,6,8), S = 110; train_mobilenetV3_ecagai.py:182-234, replacing its
 * torch.matmul -> F.softmax -> torch.matmul at :220-226).  q [B, P, ch]
 * (f_query of the up-sampled map, NHWC), kp / vp [B, S, ch] (f_key / f_value
 * of the PSP-pooled rows).  Forward: ctx [B, P, ch] = softmax(q kp^T) vp and
 * lse [B, P] (log-sum-exp per pixel; may be NULL for inference).  Backward
 * from dctx: dq [B, P, ch], and pmat / dsmat [B, S, P] (softmax and its
 * pre-softmax gradient, S-major) for dK = dsmat . q, dV = pmat . dctx.
 * ch a multiple of 4 in 8..64; S * ch * 8 bytes must fit in LDS (160 KiB). */
int jabd_nlm_attn_fwd_f32(const float* q, const float* kp, const float* vp, int32_t B,
                          int32_t P, int32_t S, int32_t ch, float* ctx, float* lse,
                          jabd_stream_t stream);
int jabd_nlm_attn_bwd_f32(const float* q, const float* kp, const float* vp, const float* ctx,
                          const float* lse, const float* dctx, int32_t B, int32_t P, int32_t S,
                          int32_t ch, float* dq, float* pmat, float* dsmat,
                          jabd_stream_t stream);
/* dK = dsmat . q and dV = pmat . dctx ([B, S, P] x [B, P, ch] -> [B, S, ch],
 * replacing the reference autograd's two batched matmul gradients of
 * train_mobilenetV3_ecagai.py:220,226) on the fp32 MFMA: P is cut into chunks
 * of 2048 pixels whose partial products land in ws (ws_floats >=
 * jabd_nlm_attn_dkv_ws_floats(B, P, S, ch)) and are then summed in chunk
 * order, so the result is deterministic.  ch <= 64. */
int64_t jabd_nlm_attn_dkv_ws_floats(int32_t B, int32_t P, int32_t S, int32_t ch);
int jabd_nlm_attn_dkv_f32(const float* dsmat, const float* pmat, const float* q,
                          const float* dctx, int32_t B, int32_t P, int32_t S, int32_t ch,
                          float* ws, int64_t ws_floats, float* dk, float* dv,
                          jabd_stream_t stream);
/* y = a + b (+ c if non-NULL), n floats (n % 4 == 0, 16-byte aligned): the
 * NLM residual + FPN lateral add of the bicubic variant
 * (train_mobilenetV3_ecagai.py:233, 271). */
int jabd_add3_f32(const float* a, const float* b, const float* c, int64_t n, float* y,
                  jabd_stream_t stream);

/* BECA gate — the contrast-ECA block of the bicubic variant
 * (train_mobilenetV3_ecagai.py:286-316): y = x * Hardsigmoid(conv1d_k(std_hw(x)))
 * on NHWC fp32 [batch, pixels, C]; w float[k] (k odd, no bias).  stats
 * float[4, batch*C] (mean, std, pre-activation, gate) is written by the forward
 * and read by the backward; the backward's ws is float[2, batch*C].  y may be
 * NULL: the gate alone (stats row 3) for a consumer that scales on load.
 * part / part_floats: the per-chunk reduction workspace, float
 * [jabd_beca_ws_floats(batch, pixels, C)] (NULL or too small: a slower
 * one-workgroup-per-image reduction). */
int64_t jabd_beca_ws_floats(int64_t batch, int64_t pixels, int C);
int jabd_beca_fwd_f32(const float* x, int64_t batch, int64_t pixels, int C,
                      const float* w, int k, float* y, float* stats, float* part,
                      int64_t part_floats, jabd_stream_t stream);
int jabd_beca_bwd_f32(const float* x, const float* grad_y, int64_t batch,
                      int64_t pixels, int C, const float* w, int k,
                      const float* stats, float* grad_x, float* grad_w, float* ws,
                      float* part, int64_t part_floats, jabd_stream_t stream);

/* ------------------------------------------------------------------------ *
 * A9 MultiBoxLoss — nets/retinaface_training.py:183-303.
 * Forward writes un-normalised sums and counts so data-parallel callers can
 * all-reduce the counts before normalising:
 *   sums   device float[3] = {Σ smoothL1(loc) over pos, Σ CE over pos∪neg,
 *                             Σ smoothL1(landm) over pos1}
 *   counts device int64[2] = {Σ pos, Σ pos1}
 *   sel    device uint8[B,A]: bit0 = pos (conf_t != 0), bit1 = pos1
 *          (conf_t > 0), bit2 = selected for CE (pos ∪ hard negative).
 * Backward: given the upstream gradients of the three normalised losses
 * (device float[3]) and the counts used to normalise them (device int64[2];
 * global counts under data parallelism) writes grad_loc/grad_conf/grad_landm.
 * ------------------------------------------------------------------------ */
int jabd_multibox_workspace_size(int64_t batch, int64_t num_priors, size_t* bytes);
int jabd_multibox_loss_fwd_f32(const float* loc, const float* conf,
                               const float* landm, const float* loc_t,
                               const int64_t* conf_t, const float* landm_t,
                               int64_t batch, int64_t num_priors, int neg_pos,
                               float* sums, int64_t* counts, uint8_t* sel,
                               void* ws, size_t ws_bytes, jabd_stream_t stream);
int jabd_multibox_loss_bwd_f32(const float* loc, const float* conf,
                               const float* landm, const float* loc_t,
                               const int64_t* conf_t, const float* landm_t,
                               const uint8_t* sel, int64_t batch,
                               int64_t num_priors, const float* gout,
                               const int64_t* counts,
                               float* grad_loc, float* grad_conf,
                               float* grad_landm, jabd_stream_t stream);
/* The DIoU MultiBoxLoss — nets/retinaface_training_DIOU.py:524-665: sums[0]
 * is Σ over positives of 1 - clamp(DIoU(decode(loc, prior), loc_t), -1, 1)
 * (IouLoss 'Diou', :491-522, bbox_overlaps_diou :402-442) with loc_t from
 * jabd_match_iou_f32; the CE and landmark terms, counts, sel and workspace
 * are those of jabd_multibox_loss_fwd_f32.  priors [A,4] (cx,cy,w,h). */
int jabd_multibox_diou_loss_fwd_f32(const float* loc, const float* conf,
                                    const float* landm, const float* loc_t,
                                    const int64_t* conf_t, const float* landm_t,
                                    const float* priors, float var0, float var1,
                                    int64_t batch, int64_t num_priors, int neg_pos,
                                    float* sums, int64_t* counts, uint8_t* sel,
                                    void* ws, size_t ws_bytes, jabd_stream_t stream);
int jabd_multibox_diou_loss_bwd_f32(const float* loc, const float* conf,
                                    const float* landm, const float* loc_t,
                                    const int64_t* conf_t, const float* landm_t,
                                    const float* priors, float var0, float var1,
                                    const uint8_t* sel, int64_t batch,
                                    int64_t num_priors, const float* gout,
                                    const int64_t* counts, float* grad_loc,
                                    float* grad_conf, float* grad_landm,
                                    jabd_stream_t stream);
/* loss[i] = sums[i] / max(counts[i==2 ? 1 : 0], 1)  (device, 1 thread). */
int jabd_multibox_loss_finalize_f32(const float* sums, const int64_t* counts,
                                    float* loss, jabd_stream_t stream);

/* ======================================================================== *
 * Detector forward kernels (NHWC fp32).  Layouts: an activation tensor is
 * addressed as base + b*bs + pixel*ps + c0 + c   (bs/ps in floats), so
 * channel slices (SSH concat) and the head's [B, A, k] layout are plain
 * strides.  Activation codes for `act`:
 * ======================================================================== */
enum {
  JABD_ACT_NONE = 0,
  JABD_ACT_RELU = 1,
  JABD_ACT_LEAKY = 2,    /* LeakyReLU(slope) */
  JABD_ACT_HSWISH = 3,   /* nn.Hardswish     */
  JABD_ACT_HSIGMOID = 4, /* nn.Hardsigmoid   */
  JABD_ACT_SIGMOID = 5,
};

/* A1/A4/A5 dense conv as implicit GEMM on fp32 MFMA — replaces nn.Conv2d
 * (+ folded BatchNorm2d + activation) at nets/mobilenetV3.py:101,113,126-130,
 * nets/retinaface_r.py:60-84,114-120, nets/layers.py:10-32 and torchvision
 * resnet50.  w: packed weights (see jabd_amd/packing.py): float4
 * [Kc][Ntiles][64], Kc = ceil(K/16), K = KH*KW*Cin (+ Cin2).
 *   x2/Cin2:  optional K-concatenated second source read as a strided 1x1
 *             conv (skip branch / ResNet downsample folded into the GEMM).
 *   ascale:   optional per-(image, input channel) multiplier (ECA gate).
 *   res:      optional residual added before the activation.
 *   nchw_in:  x is NCHW [B,Cin,H,W] (network input); else NHWC strided. */
typedef struct jabd_conv_args {
  const float* x; int64_t x_bs; int32_t x_ps, x_c0;
  int32_t B, H, W, Cin;
  const float* x2; int64_t x2_bs; int32_t x2_ps, Cin2;
  int32_t x2_W, x2_stride; /* x2 pixel of output (oh,ow) = (oh*x2_stride, ow*x2_stride) */
  const float* ascale; int64_t ascale_bs;
  const void* w; const float* bias;
  const float* res; int64_t res_bs; int32_t res_ps, res_c0;
  float* y; int64_t y_bs; int32_t y_ps, y_c0;
  int32_t OH, OW, Cout, Ntiles, tn, Kc;
  int32_t KH, KW, stride, pad;
  int32_t act; float slope;
  int32_t nchw_in, tconv; /* tconv: transposed conv — the data gradient of a
                             conv with this geometry: output (oh,ow) reads
                             input ((oh+pad-kh)/stride, (ow+pad-kw)/stride) */
  int32_t flags, reserved1; /* library-internal */
  int64_t M; /* filled in by the library */
  /* optional second packing for the 32x32x2-MFMA 1x1 kernel (nullable):
   * float4 [ceil(K/32)*4][ntiles32][64], each float4 holding
   * W[8*k8 + 4*(lane>>5) + e][32*nt + (lane&31)], e = 0..3; tn32 tiles per
   * workgroup (jabd_conv_pack_tn32), ntiles32 a multiple of tn32. */
  const void* w32; int32_t ntiles32, tn32;
  /* optional split output (nullable y2): output channels n >= nsplit go to
   * y2 at channel y2_c0 + n - nsplit with activation act2/slope2 (two
   * convolutions of one input fused along N, e.g. the SSH branches that read
   * the same tensor).  nsplit % 4 == 0; served by the generic kernel. */
  float* y2; int64_t y2_bs; int32_t y2_ps, y2_c0, nsplit, act2; float slope2; int32_t reserved2;
  /* optional workspace (nullable): with ws_bytes >= jabd_conv_workspace_size(args)
   * the library may split the K reduction of a k x k conv whose output grid
   * is too small to fill the device (bs1 inference of the R50 detector:
   * predict.py:253-333) over several workgroups — partial sums in ws, then a
   * fixed-order reduction (deterministic).  NULL: no split. */
  void* ws; int64_t ws_bytes;
} jabd_conv_args;
/* Workspace bytes jabd_conv2d_nhwc_f32 can use for args (0: it would not split). */
int64_t jabd_conv_workspace_size(const jabd_conv_args* args);
/* N-tiles (16 output channels each) grouped per workgroup for a Cout. */
int jabd_conv_pack_tn(int cout);
/* 32-channel N-tiles per workgroup of the 32x32x2 1x1 kernel for a Cout. */
int jabd_conv_pack_tn32(int cout);
/* Device-side weight packing: torch weight w [cout][cin][kh][kw] (transposed
 * = 1: the data-gradient form, W'[ci][co] = W[co][ci]) -> wp float4
 * [Kc][Ntiles][64] (the 16x16x4 layout above) and, if wp32 != NULL, wp32
 * float4 [K8][NT32][64] (the 32x32x2 layout); K = kh*kw*cin' rows in tap-major
 * order, zero padding outside.  One launch per weight (the training convs
 * repack after every optimizer step). */
int jabd_conv_pack_f32(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw,
                       int32_t transposed, int32_t Kc, int32_t Ntiles, float* wp, int32_t K8,
                       int32_t NT32, float* wp32, jabd_stream_t stream);
/* Batched jabd_conv_pack_f32: every conv weight an optimizer step changed,
 * repacked into its existing buffers in one launch (jabd_amd/optim.py, after
 * the fused Adam step; the reference's optimizer.step(),
 * train_mobilenetV3_ecagai.py:588).  jobs = device int64 [njobs][11] rows
 * {w, wp, wp32 (0: none), cout, cin, kh*kw, transposed, Kc, Ntiles, K8,
 * NT32}; starts = device int64 [njobs + 1]: starts[i] = the float4 outputs of
 * the jobs before i (Kc*Ntiles*64 + K8*NT32*64 each), total = starts[njobs].
 * njobs <= 1024. */
int jabd_conv_pack_multi_f32(const int64_t* jobs, const int64_t* starts, int32_t njobs,
                             int64_t total, jabd_stream_t stream);
int jabd_conv2d_nhwc_f32(const jabd_conv_args* args, jabd_stream_t stream);
/* Training forward of a 1x1 conv followed by BatchNorm (MNv3 Block_eca
 * conv1 -> bn1, nets/mobilenetV3.py:141-143 / :160-170): the streaming 1x1
 * kernel also writes the shifted batch-statistics partials of its output,
 * part [nblk][2][Cout] around shift [Cout] (the output at pixel 0), which
 * jabd_bn_stats_final_f32 turns into mean / invstd.  No gate, second
 * source or residual.  _nblk returns the partial rows the layer needs, 0 when
 * the statistics form does not serve it (the caller then runs
 * jabd_conv2d_nhwc_f32 + jabd_bn_stats_f32). */
int64_t jabd_conv1x1_bn_stats_nblk(const jabd_conv_args* args);
/* Training forward of a bias-free conv followed by BatchNorm on the 32x32
 * GEMM (the ResNet-50 bottleneck convs, nets/resnet_pytorch_r.py:122-143 —
 * the reference's Conv2d then BatchNorm2d in train mode): the GEMM epilogue
 * writes per-32-pixel-tile (mean, M2) rows into part, which a fixed-order
 * fp64 combination turns into mean / invstd and the running-statistics
 * update (momentum, unbiased variance), as jabd_bn_stats_f32 over y would.
 * _part_floats returns the floats part needs (16-byte aligned), 0 when the
 * form does not serve the layer (no bias / activation / gate / residual /
 * second source / split output / transposed form; the caller then runs
 * jabd_conv2d_nhwc_f32 + jabd_bn_stats_f32). */
/* Data gradient of a conv whose output is the dy of a training BatchNorm +
 * act (ReLU / LeakyReLU / none; the R50 bottleneck's bn1 / bn2 backward,
 * nets/resnet_pytorch_r.py:122-143): jabd_conv2d_nhwc_f32 on the 32x32 GEMM
 * whose epilogue also reads the BatchNorm's input x (pixel stride x_ps) and
 * writes per-32-pixel-tile sums of dz = dy act'(bn(x)) and dz xhat into
 * part; jabd_bn_act_bwd_rows_f32 then finishes the BatchNorm backward
 * without a reduction pass over dy and x.  _part_floats: 0 when the form does
 * not serve the conv (bias / act / gate / residual / second source / split
 * output, Cout % 32, a stride-2 transposed form). */
int64_t jabd_conv_bn_bwd_part_floats(const jabd_conv_args* args);
int jabd_conv_bn_bwd_sums_f32(const jabd_conv_args* args, const float* x, int32_t x_ps,
                              const float* mean, const float* invstd, const float* gamma,
                              const float* beta, int32_t act, float slope, float* part,
                              int64_t part_floats, jabd_stream_t stream);
/* The residual-ReLU form of the above (the R50 bottleneck's bn3 backward,
 * out = relu(bn3(x) + identity), nets/resnet_pytorch_r.py:139-143; it
 * replaces the bn3 part of jabd_bn_act_bwd_ex_f32 and its reduction pass):
 * args is a bias-free, act-free 1x1 / stride-1 data gradient (the NEXT
 * block's conv1 data gradient, whose output is this block's dout) with an
 * optional residual args->res (that block's identity-branch gradient); the
 * GEMM writes dz = (dgrad + res) * [mask > 0] — mask is the saved block
 * output `out` (pixel stride mask_ps) — and the per-32-pixel-tile sums of
 * dz and dz xhat (x: bn3's input, pixel stride x_ps) into part, sized by
 * jabd_conv_bn_bwd_part_floats of the same args without the residual.
 * jabd_bn_act_bwd_rows_f32(part, dz, x, ..., act = none) finishes bn3's
 * backward; dz itself is the identity branch's gradient. */
int jabd_conv_bn_bwd_sums_res_f32(const jabd_conv_args* args, const float* x, int32_t x_ps,
                                  const float* mask, int32_t mask_ps, const float* mean,
                                  const float* invstd, float* part, int64_t part_floats,
                                  jabd_stream_t stream);
int jabd_bn_act_bwd_rows_f32(float* part, const float* dy, const float* x, int64_t M,
                             int32_t C, const float* mean, const float* invstd,
                             const float* gamma, const float* beta, int32_t act, float slope,
                             float* dgamma, float* dbeta, float* dx, jabd_stream_t stream);
int64_t jabd_conv_bn_stats_part_floats(const jabd_conv_args* args);
int jabd_conv_bn_stats_f32(const jabd_conv_args* args, float* part, int64_t part_floats,
                           float* mean, float* invstd, float* running_mean, float* running_var,
                           float momentum, float eps, jabd_stream_t stream);
int jabd_conv1x1_bn_stats_f32(const jabd_conv_args* args, float* part, int64_t nblk,
                              float* shift, jabd_stream_t stream);

/* A1 MobileNetV3 stem — nets/mobilenetV3.py:455-457,511: conv3x3/s2/p1 3->16
 * on the NCHW input [B,3,H,W] with folded BN (w [27][16] tap-major, bias [16])
 * and activation, written NHWC [B,OH,OW,16]. */
int jabd_stem_nchw_f32(const float* x, int32_t B, int32_t H, int32_t W, const float* w,
                       const float* bias, int32_t act, float* y, jabd_stream_t stream);

/* A1 depthwise k x k conv (+ folded BN + act) — nets/mobilenetV3.py:105-108
 * and the stride-2 skip branches :126-137.  w [k*k][C] (tap-major), bias [C].
 * part (nullable): per-(image, block, channel) sums of the activated output,
 * [B][nblk][C], consumed by jabd_eca_gate_f32 (the ECA average pool). */
typedef struct jabd_dw_args {
  const float* x; int64_t x_bs; int32_t x_ps, reserved0;
  int32_t B, H, W, C;
  const float* w; const float* bias;
  float* y; int64_t y_bs; int32_t y_ps, reserved1;
  int32_t OH, OW, k, stride, pad, act;
  float slope; int32_t nblk;
  float* part;
} jabd_dw_args;
/* Number of per-image partial-sum blocks the dw kernel uses (size of part). */
int64_t jabd_dw_nblk(int64_t B, int64_t OH, int64_t OW, int64_t C);
int jabd_dwconv_nhwc_f32(const jabd_dw_args* args, jabd_stream_t stream);
/* Training form (nets/mobilenetV3.py:142, conv2 -> bn2): the depthwise conv
 * (args->part must be NULL) that also writes the BatchNorm statistics of its
 * output as shifted partial sums stats_part [jabd_dwconv_stats_nblk][2][C]
 * around shift[C] (the output at pixel (0, 0) of image 0, also written);
 * jabd_bn_stats_final_f32 turns them into mean / invstd and the running
 * statistics, replacing jabd_bn_stats_f32's pass over the output. */
int64_t jabd_dwconv_stats_nblk(int64_t B, int64_t OH, int64_t OW, int64_t C);
int jabd_dwconv_stats_f32(const jabd_dw_args* args, float* stats_part, float* shift,
                          jabd_stream_t stream);
/* jabd_dwconv_stats_f32 whose input is act(bn(x)) of the stored pre-BN tensor
 * args->x, applied on load: (x - mean) * invstd * gamma + beta, then act
 * (NONE/RELU/LEAKY/HSWISH) — MNv3 Block_eca bn1 + act feeding conv2
 * (nets/mobilenetV3.py:141-145), so the activated expansion is never
 * written; zero padding applies to the activated input. */
int jabd_dwconv_bnin_stats_f32(const jabd_dw_args* args, const float* mean, const float* invstd,
                               const float* gamma, const float* beta, int32_t act, float slope,
                               float* stats_part, float* shift, jabd_stream_t stream);

/* A1 fused block front half (eval) — nets/mobilenetV3.py:141-142: expand 1x1
 * conv (+ folded bn1, packed like jabd_conv_args.w, Kc = ceil(Cin/16)) + act
 * -> depthwise k x k (pad k/2, + folded bn2) + act, and the ECA pool partial
 * sums part [B][nblk][E] (nblk = jabd_expand_dw_nblk).  The expanded tensor
 * stays on chip.  act: NONE / RELU / HSWISH (act1 == act2 in Block_eca). */
typedef struct jabd_expdw_args {
  const float* x; int64_t x_bs; int32_t x_ps, Cin;
  int32_t B, H, W, E;
  const void* we; const float* be; int32_t Ntiles, Kc;
  const float* wd; const float* bd;
  int32_t k, stride, act, nblk;
  float* y; int64_t y_bs; int32_t y_ps, OH, OW, reserved0;
  float* part;
  /* optional (stride 2 only; sy NULL: none): the block's skip branch
   * dw3x3/s2 + folded BN on the same input tile — sw [9][Cin] tap-major, sb
   * [Cin] — written to sy [B][OH][OW][Cin] (pixel stride sy_ps, image stride
   * sy_bs) by the first expanded-channel chunk's workgroups
   * (nets/mobilenetV3.py:126-137, the K-concat source of the project GEMM). */
  const float* sw; const float* sb; float* sy; int64_t sy_bs; int32_t sy_ps, reserved1;
  /* optional (pw NULL: none; stride 2 with the skip branch, Cin <= 16): the
   * previous block's project fused in front of the expand.  x is then that
   * block's depthwise output d, and the kernel expands
   *   x' = pact( Wp (pg[b] * d) + pb + pres )      (nets/mobilenetV3.py:144-150)
   * per input-tile pixel (zero outside the image): Wp packed as `we` ([1][1][64]
   * float4, Cin -> Cin), pb [Cin], pg [B][Cin] (image stride pg_bs: the ECA
   * gate), pres the block input (the identity residual; x's strides).  x' is
   * never written: the block pair's activation between them stays on chip. */
  const void* pw; const float* pb; const float* pg; const float* pres; int32_t pg_bs, pact;
} jabd_expdw_args;
int64_t jabd_expand_dw_nblk(int32_t OH, int32_t OW, int32_t k, int32_t stride);
int jabd_expand_dw_nhwc_f32(const jabd_expdw_args* args, jabd_stream_t stream);
/* Kernel form of jabd_expand_dw_nhwc_f32: 1 = one work item per workgroup,
 * 2 = wave-specialised persistent workgroups, 3 = persistent workgroups
 * walking a fixed channel chunk's tiles (forms 1-3: the same results bit for
 * bit), 4 = chunk-pipelined persistent workgroups for Cin <= 80 (y and the
 * skip branch bit-identical to 1-3, the ECA partials summed in another fixed
 * order; geometries it does not cover run form 1), 0 = the default (1; 2
 * with JABD_EXPDW_WS=1, 3 with JABD_EXPDW2=1, 4 with JABD_EXPDW3=1).
 * Returns the previous setting.  For A/B timing and the equivalence tests. */
int jabd_expand_dw_select(int32_t form);

/* Per-(image, block, channel) sums of an NHWC tensor (ECA pooling of a tensor
 * not produced by the dw kernel: C3/C4/C5 and the FPN outputs). */
int jabd_channel_sum_f32(const float* x, int64_t x_bs, int32_t x_ps, int64_t B, int64_t HW,
                         int64_t C, int64_t nblk, float* part, jabd_stream_t stream);
/* First level of a two-level, fixed-order sum of per-block partials:
 * out[b][s][c] = sum of part[b][r][c] over rows r in [s*R, (s+1)*R),
 * R = ceil(nblk / nsplit).  Feeds jabd_eca_gate_f32 (with nblk = nsplit) when
 * a producer wrote many partial rows (one per depthwise tile). */
int jabd_partial_reduce_f32(const float* part, int64_t nblk, int64_t B, int64_t C, int64_t nsplit,
                            float* out, jabd_stream_t stream);
/* A2 ECA gate — nets/mobilenetV3.py:343-348 (gate=HSIGMOID) and
 * nets/retinaface_r.py:219-224 (gate=SIGMOID): mean = sum(part)/HW,
 * Conv1d(1,1,k,pad=(k-1)/2,no bias) over channels, gate -> scale [B][C]. */
int jabd_eca_gate_f32(const float* part, int64_t nblk, int64_t B, int64_t C, int64_t hw,
                      const float* w1d, int32_t k, int32_t gate, float* scale, float* mean_out,
                      jabd_stream_t stream);

/* A3 CSAF non-local block — nets/retinaface_r.py:85-152 + the FPN's nearest
 * up-sample and add (:192-203).  x = nearest(src [B,hs,ws,C] -> h x w).
 * nlm_pool: kpool/vpool [B][S][ch] = PSP adaptive-avg-pools (sizes[], host
 *   array) of f_key(x) / f_value(x)  (wk/wv [ch][C], bk/bv [ch]); kv_ws is
 *   scratch [B][hs*ws][2*ch].  Built for ch == 4 (the JABD NLM).
 * nlm_apply: out = lateral + (W·softmax_S(q·k)·v + bW + x), q = f_query(x),
 *   lateral/out [B,h,w,C] NHWC (may alias; lateral nullable = 0, which with
 *   hs == h, ws == w is the standalone NLM.forward); q_out/ctx_out [B,h*w,ch]
 *   (nullable) keep q and the attention context for the backward. */
int jabd_nlm_pool_f32(const float* src, int64_t src_bs, int32_t src_ps, int32_t B, int32_t hs,
                      int32_t ws, int32_t C, int32_t h, int32_t w, const float* wk,
                      const float* bk, const float* wv, const float* bv, int32_t ch,
                      const int32_t* sizes, int32_t nsizes, float* kpool, float* vpool,
                      float* kv_ws, jabd_stream_t stream);
int jabd_nlm_apply_f32(const float* src, int64_t src_bs, int32_t src_ps, int32_t B, int32_t hs,
                       int32_t ws, int32_t C, int32_t h, int32_t w, const float* wq,
                       const float* bq, const float* kpool, const float* vpool, int32_t S,
                       int32_t ch, const float* wW, const float* bW, const float* lateral,
                       float* out, float* q_out, float* ctx_out, jabd_stream_t stream);

/* A4 detection heads — nets/retinaface_r.py:17-57,335-343: the Bbox (2x4),
 * Class (2x2) and Landmark (2x10) 1x1 convs of one pyramid level, written
 * straight into loc [B,A,4] / conf [B,A,2] / landm [B,A,10] at anchor offset
 * a_off (the permute+view+cat layout); softmax over conf pairs if asked.
 * wt [32][C] rows = 8 bbox, 4 class, 20 landmark out channels; bias [32]. */
/* 3x3/stride-2/pad-1 max pool, NHWC (torchvision resnet50 stem maxpool). */
int jabd_maxpool_nhwc_f32(const float* x, int32_t B, int32_t H, int32_t W, int32_t C,
                          int32_t k, int32_t stride, int32_t pad, float* y,
                          jabd_stream_t stream);
/* A4 SSH tail + heads of one pyramid level of the 40-channel SSH (MobileNetV3
 * detectors; nets/layers.py:37-68 and the heads of nets/retinaface_r.py:
 * 17-57,335-343) in one launch: given the level's first GEMM outputs c33 =
 * relu(conv3X3) [B,H,W,>=20] (pixel stride c33_ps) and t = leaky(conv5X5_1)
 * [B,H,W,12] (10 channels + 2 zero), computes conv7X7_2 (+leaky), conv5X5_2,
 * conv7x7_3, relu(cat), the three 1x1 heads (+ the eval softmax) and stores
 * loc/conf/landm rows [B,A,4|2|10] from anchor a_off.  wb: the packed,
 * BN-folded weights, jabd_ssh_tail_weight_floats() floats: three 3x3 10->10
 * convs [n][kh*3+kw][12] + bias [10] (conv5X5_2, conv7X7_2, conv7x7_3), then
 * heads [32][40] + bias [32] (8 bbox, 4 class, 20 landmark rows). */
int64_t jabd_ssh_tail_weight_floats(void);
int jabd_ssh_tail_heads_f32(const float* c33, int64_t c33_bs, int32_t c33_ps, const float* t,
                            int64_t t_bs, int32_t B, int32_t H, int32_t W, const float* wb,
                            float leaky, int64_t A, int64_t a_off, int32_t softmax, float* loc,
                            float* conf, float* landm, jabd_stream_t stream);
int jabd_heads_f32(const float* x, int64_t x_bs, int32_t x_ps, int32_t B, int32_t HW,
                   int32_t C, const float* wt, const float* bias, int64_t A, int64_t a_off,
                   int32_t softmax, float* loc, float* conf, float* landm,
                   jabd_stream_t stream);
/* The same heads for wide levels (R50: C = 256), whose three 1x1 convs run
 * as one GEMM (jabd_conv2d_nhwc_f32, C -> 32) into y [B][HW][32] (channels as
 * wt above); this scatters y into loc / conf / landm at a_off, softmax over
 * the conf pairs if asked (the same fp32 operations as jabd_heads_f32). */
int jabd_heads_scatter_f32(const float* y, int32_t B, int64_t HW, int64_t A, int64_t a_off,
                           int32_t softmax, float* loc, float* conf, float* landm,
                           jabd_stream_t stream);

/* ======================================================================== *
 * Training-graph glue (no PyTorch kernels in a training step)
 * ======================================================================== */
/* Windowed copy: dst [d0][d1][d2] (dense) = scale * src[i0][i1][i2 + off2]
 * of src [s0][s1][s2] where that index lies inside the source dims, else
 * fill.  Pads (d >= s) or crops (d <= s) each dim, off2 starts the window
 * inside dim 2; up to JABD_WINDOW_MAX tensors per launch.  Replaces the
 * torch.cat / slice / stack glue of a training step: the zero-padding of the
 * SSH 10-channel branches (nets/layers.py:37-68 with out_channel 40:
 * conv5X5_1 / conv7X7_2 widths 10) and the crops back, column splits, the
 * loss-gradient vector. */
#define JABD_WINDOW_MAX 32
typedef struct jabd_window_copy {
  const float* src;
  float* dst;
  int32_t s0, s1, s2;
  int32_t d0, d1, d2;
  int32_t off2;
  float fill;
  float scale;
  int32_t reserved;
} jabd_window_copy;
int jabd_window_copy_multi_f32(int32_t n, const jabd_window_copy* descs, jabd_stream_t stream);
/* dst [cols][rows] = src [rows][cols]^T (depthwise weights [C][k*k] -> tap-major). */
int jabd_transpose_f32(const float* src, int32_t rows, int32_t cols, float* dst,
                       jabd_stream_t stream);
/* out[c] = sum_r part[r][c], rows in order (bias gradients from the per-block
 * channel sums of jabd_channel_sum_f32). */
int jabd_colsum_f32(const float* part, int64_t rows, int32_t C, float* out,
                    jabd_stream_t stream);
/* out[e] = in[0][e] + in[1][e] + ... (left to right), n elements, up to
 * JABD_SUM_MAX inputs: the gradient of a tensor consumed n_in times (the FPN
 * features, the SSH inputs, the head ECA weight; nets/retinaface_r.py:287-343). */
#define JABD_SUM_MAX 8
int jabd_sum_multi_f32(int32_t n_in, const float* const* in, int64_t n, float* out,
                       jabd_stream_t stream);
/* out[0] = wa * a[0] + b[0] + c[0]: the total MultiBoxLoss of a training step,
 * loss = loc_weight * loss_l + loss_c + loss_landm (train_mobilenetV3_ecagai.py:529). */
int jabd_weighted_sum3_f32(const float* a, const float* b, const float* c, float wa, float* out,
                           jabd_stream_t stream);
/* out [cout_is_rows ? K x Cout] = conv weight [Cout][Cin][KH][KW] as the
 * tap-major [(kh*KW + kw)*Cin + ci][co] matrix (the stem kernel's layout). */
int jabd_conv_w2d_f32(const float* w, int32_t cout, int32_t cin, int32_t taps, float* out,
                      jabd_stream_t stream);
/* The Bbox / Class / Landmark heads of one level (nets/retinaface_r.py:19-58:
 * 1x1 convs, 8 / 4 / 20 outputs over C channels) as one [32][Cf] matrix wt
 * and bias [32] (dir 0), or wt unpacked into the three gradients (dir 1).
 * Feature channel j sits at column j < half + q ? j : j + qp - q (SSH output
 * with its two q-channel branches padded to qp); q == qp: Cf == C. */
int jabd_heads_wpack_f32(float* wb, float* wc, float* wl, const float* bb, const float* bc,
                         const float* bl, int32_t C, int32_t half, int32_t q, int32_t qp,
                         float* wt, int32_t Cf, float* bias, int32_t dir, jabd_stream_t stream);

/* ======================================================================== *
 * A11 training (loss.backward() of train_*.py:532) — fp32 NHWC, row-major
 * [M = B*H*W rows][C], ld = row stride in floats.  BatchNorm2d in training
 * mode (batch statistics, momentum update of the running buffers).
 * ======================================================================== */
/* Partial-buffer size (blocks) of the BN reductions: part = [nblk][2][C]. */
int64_t jabd_bn_nblk(int64_t M, int32_t C);
/* mean/invstd of x over M rows (biased var); running stats updated in place
 * (running_var with the unbiased estimate) when non-null. */
/* jabd_bn_stats_f32's final step for partials written by a producer
 * (jabd_dwconv_stats_f32): shift[c] is the value they were taken around. */
int jabd_bn_stats_final_f32(const float* shift, const float* part, int64_t nblk, int64_t M,
                            int32_t C, float* mean, float* invstd, float* running_mean,
                            float* running_var, float momentum, float eps, jabd_stream_t stream);
int jabd_bn_stats_f32(const float* x, int32_t ldx, int64_t M, int32_t C, float* part,
                      float* mean, float* invstd, float* running_mean, float* running_var,
                      float momentum, float eps, jabd_stream_t stream);
/* y[:, yc0:yc0+C] = act((x - mean) * invstd * gamma + beta [+ res]) */
int jabd_bn_act_fwd_f32(const float* x, int32_t ldx, int64_t M, int32_t C, const float* mean,
                        const float* invstd, const float* gamma, const float* beta,
                        const float* res, int32_t ldr, int32_t act, float slope, float* y,
                        int32_t ldy, int32_t yc0, jabd_stream_t stream);
/* Backward of bn_act_fwd: dx [M][C] (dense), dres [M][C] (= dz, nullable),
 * dgamma/dbeta [C].  dy is read at columns dyc0.. of rows of lddy floats. */
int jabd_bn_act_bwd_f32(const float* dy, int32_t lddy, int32_t dyc0, const float* x, int32_t ldx,
                        const float* res, int32_t ldr, int64_t M, int32_t C, const float* mean,
                        const float* invstd, const float* gamma, const float* beta, int32_t act,
                        float slope, float* part, float* dgamma, float* dbeta, float* dx,
                        float* dres, jabd_stream_t stream);
/* jabd_bn_act_fwd_f32 (contiguous x / y, no residual) that also writes the
 * channel sums of y per block of rows, part[B][nblk][C] with nblk =
 * jabd_bn_sum_nblk(hw, C) (0: hw not a multiple of the block; use
 * jabd_channel_sum_f32) — the ECA pool input of a MobileNetV3 Block_eca
 * (nets/mobilenetV3.py:141-148, 343-348) without a pass over y. */
int64_t jabd_bn_sum_nblk(int64_t hw, int32_t C);
int jabd_bn_act_fwd_sum_f32(const float* x, int64_t M, int32_t C, const float* mean,
                            const float* invstd, const float* gamma, const float* beta,
                            int32_t act, float slope, float* y, int64_t hw, float* part,
                            jabd_stream_t stream);
/* The same with the incoming gradient mapped per (image, channel) first:
 * dy' = dy * dys[b][c] + dya[b][c], b = row / hw (dys NULL: no map) — the
 * backward of an ECA gate that followed this BN (jabd_eca_bwd_terms_f32). */
int jabd_bn_act_bwd_ex_f32(const float* dy, int32_t lddy, int32_t dyc0, const float* x,
                           int32_t ldx, const float* res, int32_t ldr, int64_t M, int32_t C,
                           const float* mean, const float* invstd, const float* gamma,
                           const float* beta, int32_t act, float slope, const float* dys,
                           const float* dya, int64_t hw, float* part, float* dgamma,
                           float* dbeta, float* dx, float* dres, jabd_stream_t stream);
/* Depthwise data gradient fused with the backward partials of the BatchNorm
 * that produced the depthwise input (nets/mobilenetV3.py:141-142, bn1 + act
 * -> conv2): de = dgrad(dy, w) is written to dz (bn1's output gradient), and
 * bn1's backward — dgamma, dbeta, dx = the input gradient of bn1 (x = bn1's
 * input e_pre, NHWC contiguous) — follows as jabd_bn_act_bwd_f32 would give
 * it, without its separate pass over de and x.  dz == NULL: de is never
 * stored; a second depthwise pass recomputes it and writes dx directly
 * (saves de's write and read-back for a second read of dy).  part: >=
 * jabd_dw_dgrad_bn_part_floats(B, H, W, C) floats. */
int64_t jabd_dw_dgrad_bn_part_floats(int32_t B, int32_t H, int32_t W, int32_t C);
int jabd_dw_dgrad_bn_bwd_f32(const float* dy, const float* w, int32_t B, int32_t H, int32_t W,
                             int32_t C, int32_t OH, int32_t OW, int32_t k, int32_t stride,
                             int32_t pad, const float* x, const float* mean, const float* invstd,
                             const float* gamma, const float* beta, int32_t act, float slope,
                             float* part, float* dgamma, float* dbeta, float* dz, float* dx,
                             jabd_stream_t stream);
/* n <= 4 ECA pools + gates in two launches (the head's per-level gates,
 * nets/retinaface_r.py:208-224): host arrays of n entries; tensor i is NHWC
 * with B images at x[i] (+ b * x_bs[i], pixel stride x_ps[i]), HW[i] pixels,
 * C[i] % 4 == 0 channels; part[i] is scratch of B * nblk[i] * C[i] floats;
 * w1d[i] the Conv1d weight (k[i] <= 9 taps); scale[i] [B][C[i]] receives the
 * gate (SIGMOID / HSIGMOID).  Same result as jabd_channel_sum_f32 +
 * jabd_eca_gate_f32 per tensor. */
int jabd_eca_pool_gate_multi_f32(int32_t n, int64_t B, const float* const* x, const int64_t* x_bs,
                                 const int32_t* x_ps, const int64_t* HW, const int32_t* C,
                                 const int64_t* nblk, float* const* part, const float* const* w1d,
                                 const int32_t* k, int32_t gate, float* const* scale,
                                 jabd_stream_t stream);
/* Conv weight gradient (fp32 MFMA): x/geometry as the forward jabd_conv_args
 * with `y` pointing at dY; dw in torch layout [Cout][Cin][KH][KW]; part is
 * scratch of jabd_conv_wgrad_part_floats() floats.  The data gradient is
 * jabd_conv2d_nhwc_f32 with tconv=1 and the transposed weights. */
int64_t jabd_conv_wgrad_part_floats(const jabd_conv_args* args);
int jabd_conv_wgrad_f32(const jabd_conv_args* args, float* part, float* dw, jabd_stream_t stream);
/* Depthwise gradients (nets/mobilenetV3.py:105-106): dx from dy and w
 * [k*k][C]; dw in torch layout [C][1][k][k] (part: jabd_dw_wgrad_part_floats). */
int jabd_dw_dgrad_f32(const float* dy, const float* w, int32_t B, int32_t H, int32_t W, int32_t C,
                      int32_t OH, int32_t OW, int32_t k, int32_t stride, int32_t pad, float* dx,
                      jabd_stream_t stream);
int64_t jabd_dw_wgrad_part_floats(int64_t M, int32_t C, int32_t k);
int jabd_dw_wgrad_f32(const float* x, const float* dy, int32_t B, int32_t H, int32_t W, int32_t C,
                      int32_t OH, int32_t OW, int32_t k, int32_t stride, int32_t pad, float* part,
                      float* dw, jabd_stream_t stream);
/* jabd_dw_wgrad_f32 of the BN-input depthwise conv (jabd_dwconv_bnin_stats_f32):
 * the input taps recomputed from the pre-BN tensor x_bn with the same
 * expression. */
int jabd_dw_wgrad_bnin_f32(const float* x_bn, const float* dy, int32_t B, int32_t H, int32_t W,
                           int32_t C, int32_t OH, int32_t OW, int32_t k, int32_t stride,
                           int32_t pad, const float* mean, const float* invstd, const float* gamma,
                           const float* beta, int32_t act, float slope, float* part, float* dw,
                           jabd_stream_t stream);
/* ECA backward.  The consumer saw a = x * scale[b][c]; given da:
 *   dx = da * scale + (d mean)/HW  through the gate, Conv1d and average pool,
 *   dw1d [k] the Conv1d weight gradient.  mean/scale are the forward's
 *   (jabd_eca_gate_f32 mean_out).  part [B][nblk][C], dmean_ws [B][C],
 *   dw1d_ws [B][k] are scratch. */
int jabd_eca_bwd_f32(const float* da, const float* x, int64_t B, int64_t HW, int32_t C,
                     const float* scale, const float* mean, const float* w1d, int32_t k,
                     int32_t gate, float* part, int32_t nblk, float* dmean_ws, float* dw1d_ws,
                     float* dx, float* dw1d, jabd_stream_t stream);
/* jabd_eca_bwd_f32 without the dx pass: dmean_ws [B][C] is the additive
 * term, so dx = da * scale + dmean_ws (applied by the consumer). */
int jabd_eca_bwd_terms_f32(const float* da, const float* x, int64_t B, int64_t HW, int32_t C,
                           const float* scale, const float* mean, const float* w1d, int32_t k,
                           int32_t gate, float* part, int32_t nblk, float* dmean_ws,
                           float* dw1d_ws, float* dw1d, jabd_stream_t stream);
/* ECA-gated 1x1 project conv p = conv(x * scale[b][c]) (replaces, for
 * nets/mobilenetV3.py:145-148's conv3 after eca_block :343-348, the
 * backward pair jabd_conv_wgrad_f32 with ascale + the sum(da * x) pass of
 * jabd_eca_bwd_terms_f32): args as jabd_conv_wgrad_f32 with the UNGATED x and
 * ascale NULL; w the torch weight [Cout][Cin]; outputs dw [Cout][Cin] and
 * ds[b][c] = sum_hw da * x with da the data gradient through w.  part is
 * scratch of jabd_conv_wgrad_eca_part_floats() floats (0: shape unsupported). */
int64_t jabd_conv_wgrad_eca_part_floats(const jabd_conv_args* args);
int jabd_conv_wgrad_eca_f32(const jabd_conv_args* args, const float* scale, const float* w,
                            float* part, float* dw, float* ds, jabd_stream_t stream);
/* The gate half of jabd_eca_bwd_terms_f32 given part[b][blk][c] = sum da * x. */
int jabd_eca_gate_bwd_f32(const float* part, int32_t nblk, int64_t B, int64_t HW, int32_t C,
                          const float* scale, const float* mean, const float* w1d, int32_t k,
                          int32_t gate, float* dmean_ws, float* dw1d_ws, float* dw1d,
                          jabd_stream_t stream);
/* dx = da * scale[b][c] and part[b][blk][c] = sum da * x (scale gradient). */
int jabd_scale_bwd_f32(const float* da, const float* x, int64_t B, int64_t HW, int32_t C,
                       const float* scale, float* part, int32_t nblk, float* dx,
                       jabd_stream_t stream);
/* Heads backward input: d(loc|conf|landm) rows of one level -> [B][HW][32]. */
int jabd_heads_gather_f32(const float* gloc, const float* gconf, const float* glandm, int32_t B,
                          int64_t A, int64_t a_off, int32_t HW, float* dout,
                          jabd_stream_t stream);
/* Fused Adam step over many fp32 tensors in one launch (replaces the
 * torch.optim.Adam(lr, weight_decay=5e-4) step of
 * train_mobilenetV3_ecagai.py:564 / :588 optimizer.step(); same math and
 * order as torch's single-tensor Adam, amsgrad off, maximize off).
 * rows: DEVICE array of {float* param; const float* grad; float* exp_avg;
 * float* exp_avg_sq; int64_t numel} (40 bytes each).  chunks: DEVICE array
 * filled (on the host) by jabd_adam_fill_chunks from the HOST numel array;
 * jabd_adam_num_chunks gives its length.  bias_correction1/2 = 1 - beta^step.
 * Scalars are doubles, rounded to fp32 where torch rounds its Python floats. */
int64_t jabd_adam_num_chunks(const int64_t* numel, int64_t ntensors);
int jabd_adam_fill_chunks(const int64_t* numel, int64_t ntensors, int64_t* chunks);
int jabd_adam_step_f32(const void* rows, const int64_t* chunks, int64_t nchunks, double lr,
                       double beta1, double beta2, double eps, double weight_decay,
                       double bias_correction1, double bias_correction2, jabd_stream_t stream);
/* Max-pool backward (F.max_pool2d first-max / NaN semantics), NHWC. */
int jabd_maxpool_bwd_f32(const float* x, const float* dy, int32_t B, int32_t H, int32_t W,
                         int32_t C, int32_t k, int32_t stride, int32_t pad, float* dx,
                         jabd_stream_t stream);
/* Training form (nets/resnet_pytorch_r.py:174-178 maxpool under autograd):
 * the forward also writes idx uint8 [B, OH, OW, C], each output's argmax as
 * its window position kh * k + kw (first maximum, NaN taking the place);
 * the backward gathers idx + dy (bit-identical to jabd_maxpool_bwd_f32).
 * C % 4 == 0, 16-byte aligned tensors. */
int jabd_maxpool_idx_nhwc_f32(const float* x, int32_t B, int32_t H, int32_t W, int32_t C,
                              int32_t k, int32_t stride, int32_t pad, float* y, uint8_t* idx,
                              jabd_stream_t stream);
int jabd_maxpool_bwd_idx_f32(const uint8_t* idx, const float* dy, int32_t B, int32_t H, int32_t W,
                             int32_t C, int32_t k, int32_t stride, int32_t pad, float* dx,
                             jabd_stream_t stream);
/* CSAF/NLM backward (nets/retinaface_r.py:124-152).  attn: from dOut (grad
 * of lateral + NLM(x)) -> dq [M][4], dx_up [M][C] (= dOut + Wq^T dq), and
 * dK/dV [B][S][4] (part: [B][ceil(h*w/64)][S][8] scratch).  proj: PSP
 * backward -> dkv [M][8] and dx_up += Wk^T dk + Wv^T dv.  Up-sample backward
 * gathers dx_up onto the source grid (accumulate=1 adds to dsrc). */
int jabd_nlm_bwd_attn_f32(const float* dout, int32_t B, int32_t h, int32_t w, int32_t C,
                          const float* q, const float* kpool, const float* vpool, int32_t S,
                          const float* wW, const float* wq, float* dq, float* dxup, float* part,
                          float* dk, float* dv, jabd_stream_t stream);
int jabd_nlm_bwd_proj_f32(const float* dk, const float* dv, int32_t B, int32_t S,
                          const int32_t* sizes, int32_t nsizes, int32_t h, int32_t w, int32_t C,
                          const float* wk, const float* wv, float* dkv, float* dxup,
                          jabd_stream_t stream);
int jabd_upsample_nearest_bwd_f32(const float* dxup, int32_t B, int32_t h, int32_t w, int32_t hs,
                                  int32_t ws, int32_t C, int32_t accumulate, float* dsrc,
                                  jabd_stream_t stream);
/* F.interpolate(mode='nearest', size=(h,w)) of an NHWC tensor. */
int jabd_upsample_nearest_f32(const float* src, int32_t B, int32_t hs, int32_t ws, int32_t h,
                              int32_t w, int32_t C, float* dst, jabd_stream_t stream);

/* ------------------------------------------------------------------------ *
 * Module-level ops — what the reference's individual nn.Modules compute when
 * a caller runs them one by one (nn.Sequential children, the body of a
 * torchvision IntermediateLayerGetter, a standalone eca_block / PSPModule /
 * SeModule) instead of inside the fused RetinaFace plan.
 * act / act_bwd: nn.ReLU / LeakyReLU(slope) / Hardswish / Hardsigmoid /
 *   Sigmoid (nets/mobilenetV3.py:43-56, nets/layers.py:10-34) over n dense
 *   floats (any layout); act_bwd takes the forward INPUT x.
 * bn_eval: eval-mode nn.BatchNorm2d/1d with running statistics (+ act) over
 *   x [M][C] (NHWC rows, or [B][C]); any C.
 * channel_scale: y = x * s[b][c] (eca_block / SeModule gate application,
 *   nets/mobilenetV3.py:31-32,343-348), NHWC, C % 4 == 0.
 * adaptive_pool: cat over sizes[] of nn.AdaptiveAvgPool2d((s, s)) of NHWC x
 *   -> out [B][S][C], S = sum s^2 (PSPModule, nets/retinaface_r.py:85-104);
 *   bin [floor(i*H/s), ceil((i+1)*H/s)), sum / count.  _bwd gathers dy
 *   [B][S][C] back onto every pixel (no atomics).
 * ------------------------------------------------------------------------ */
int jabd_act_f32(const float* x, int64_t n, int32_t act, float slope, float* y,
                 jabd_stream_t stream);
int jabd_act_bwd_f32(const float* x, const float* dy, int64_t n, int32_t act, float slope,
                     float* dx, jabd_stream_t stream);
int jabd_bn_eval_f32(const float* x, int64_t M, int32_t C, const float* running_mean,
                     const float* running_var, float eps, const float* gamma, const float* beta,
                     int32_t act, float slope, float* y, jabd_stream_t stream);
int jabd_channel_scale_f32(const float* x, int64_t B, int64_t HW, int32_t C, const float* scale,
                           float* y, jabd_stream_t stream);
/* cat over `sizes` of AdaptiveAvgPool2d((s, s)) of NHWC x -> out [B, S, C]
 * (PSPModule, nets/retinaface_r.py:85-104).  ws / ws_floats: row-pass
 * workspace, float[jabd_adaptive_pool_ws_floats(...)] (NULL: one-pass kernel). */
int64_t jabd_adaptive_pool_ws_floats(int32_t B, int32_t H, int32_t C, const int32_t* sizes,
                                     int32_t nsizes);
int jabd_adaptive_pool_f32(const float* x, int64_t x_bs, int32_t B, int32_t H, int32_t W,
                           int32_t C, const int32_t* sizes, int32_t nsizes, float* out,
                           float* ws, int64_t ws_floats, jabd_stream_t stream);
/* out = lateral + F.interpolate(src, size=(h, w), mode='nearest') — the
 * plain FPN's up-sample and add (nets/layers.py:106-117); NHWC, C % 4 == 0.
 * Backward: jabd_upsample_nearest_bwd_f32. */
int jabd_upsample_nearest_add_f32(const float* src, int32_t B, int32_t hs, int32_t ws, int32_t h,
                                  int32_t w, int32_t C, const float* lateral, float* out,
                                  jabd_stream_t stream);
int jabd_adaptive_pool_bwd_f32(const float* dy, int32_t B, int32_t H, int32_t W, int32_t C,
                               const int32_t* sizes, int32_t nsizes, float* dx,
                               jabd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* JABD_H_ */
