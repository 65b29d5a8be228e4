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
/* loss[i] = sums[i] / max(counts[i==2 ? 1 : 0], 1)  (device, 1 thread). */
int jabd_multibox_loss_finalize_f32(const float* sums, const int64_t* counts,
                                    float* loss, jabd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* JABD_H_ */
