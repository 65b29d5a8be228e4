// Internal entry to the batched NMS pipeline (shared with jabd_detect_f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jabd {
size_t nms_ws_bytes(int64_t batch, int64_t n);
int nms_core(const float* boxes, int64_t box_stride, int64_t box_bstride,
             const float* scores, int64_t score_stride, int64_t score_bstride,
             const int64_t* n_valid, int64_t batch, int64_t n, double iou_thr,
             float score_thr, int64_t* keep, int64_t* n_keep, void* ws,
             size_t ws_bytes, hipStream_t st);
}  // namespace jabd
