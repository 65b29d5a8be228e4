// WIDER FACE evaluation core — utils/evaluation.py:255-315 (image_eval,
// img_pr_info) summed over images as evaluation() does (:370-375), §8f rank 3.
// One workgroup per image (ragged preds/gts by offsets), float64 throughout:
//   1. per prediction, IoU against every gt (bbox_overlaps :45-63 on the xywh ->
//      corner rows of :268-271) and its first-index max/argmax (NaN wins, as
//      numpy's max/argmax), in parallel;
//   2. one lane replays the greedy recall/proposal updates (:275-286) in order,
//      writing pred_recall[h] and the running count of proposal == 1;
//   3. per threshold t (1 - (t+1)/T), the last index with score >= t picks
//      (proposals, recall) (:290-305), accumulated into pr_curve[T, 2] with
//      double atomics — every addend is an integer, so the sum is exact and
//      order-independent.
#include <math.h>

#include "common.h"

namespace jabd {

constexpr int kEvalBlock = 256;

__global__ __launch_bounds__(kEvalBlock) void wider_eval_kernel(
    const double* __restrict__ pred, const int64_t* __restrict__ poff,
    const double* __restrict__ gt, const uint8_t* __restrict__ ignore,
    const int64_t* __restrict__ goff, double iou_thresh, int thresh_num,
    double* __restrict__ maxov, int* __restrict__ maxidx, int* __restrict__ recall,
    double* __restrict__ pred_recall, double* __restrict__ prop_count,
    double* __restrict__ pr_curve) {
  const int img = blockIdx.x;
  const int64_t p0 = poff[img], np_ = poff[img + 1] - p0;
  const int64_t g0 = goff[img], ng = goff[img + 1] - g0;
  if (np_ == 0 || ng == 0) return;  // :364-365 skips the image
  // 1. overlaps row max / argmax
  for (int64_t h = threadIdx.x; h < np_; h += blockDim.x) {
    const double* p = pred + (p0 + h) * 5;
    const double ax1 = p[0], ay1 = p[1], ax2 = p[2] + p[0], ay2 = p[3] + p[1];
    const double aarea = (ax2 - ax1) * (ay2 - ay1);
    double best = -INFINITY;
    int bi = 0;
    bool nan = false;
    for (int64_t g = 0; g < ng; ++g) {
      const double* q = gt + (g0 + g) * 4;
      const double bx1 = q[0], by1 = q[1], bx2 = q[2] + q[0], by2 = q[3] + q[1];
      const double iw = fmax(fmin(ax2, bx2) - fmax(ax1, bx1), 0.0);
      const double ih = fmax(fmin(ay2, by2) - fmax(ay1, by1), 0.0);
      const double inter = iw * ih;
      const double barea = (bx2 - bx1) * (by2 - by1);
      const double v = inter / (aarea + barea - inter);
      if (v != v) {
        if (!nan) { nan = true; best = v; bi = (int)g; }
      } else if (!nan && v > best) {
        best = v;
        bi = (int)g;
      }
    }
    maxov[p0 + h] = best;
    maxidx[p0 + h] = bi;
  }
  for (int64_t g = threadIdx.x; g < ng; g += blockDim.x) recall[g0 + g] = 0;
  __syncthreads();
  // 2. the greedy replay, in prediction order
  if (threadIdx.x == 0) {
    int64_t cnt = 0, props = 0;
    for (int64_t h = 0; h < np_; ++h) {
      const double mo = maxov[p0 + h];
      const int mi = maxidx[p0 + h];
      bool prop = true;
      if (mo >= iou_thresh) {
        int& r = recall[g0 + mi];
        if (ignore[g0 + mi] == 0) {
          if (r == 1) --cnt;
          r = -1;
          prop = false;
        } else if (r == 0) {
          r = 1;
          ++cnt;
        }
      }
      props += prop ? 1 : 0;
      pred_recall[p0 + h] = (double)cnt;
      prop_count[p0 + h] = (double)props;
    }
  }
  __syncthreads();
  // 3. thresholds
  for (int t = threadIdx.x; t < thresh_num; t += blockDim.x) {
    const double thr = 1.0 - (double)(t + 1) / (double)thresh_num;
    int64_t r = -1;
    for (int64_t h = np_ - 1; h >= 0; --h)
      if (pred[(p0 + h) * 5 + 4] >= thr) { r = h; break; }
    if (r >= 0) {
      atomicAdd(&pr_curve[2 * t], prop_count[p0 + r]);
      atomicAdd(&pr_curve[2 * t + 1], pred_recall[p0 + r]);
    }
  }
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_wider_eval_workspace_size(int64_t total_preds, int64_t total_gts,
                                              size_t* bytes) {
  JABD_REQUIRE(bytes && total_preds >= 0 && total_gts >= 0, "wider_eval_ws: bad args");
  Sizer sz;
  sz.take<double>(total_preds);
  sz.take<double>(total_preds);
  sz.take<double>(total_preds);
  sz.take<int>(total_preds);
  sz.take<int>(total_gts);
  *bytes = sz.used;
  return JABD_OK;
}

extern "C" int jabd_wider_eval_f64(const double* pred, const int64_t* pred_offsets,
                                   const double* gt, const uint8_t* ignore,
                                   const int64_t* gt_offsets, int64_t num_images,
                                   int64_t total_preds, int64_t total_gts, double iou_thresh,
                                   int thresh_num, double* pr_curve, void* ws, size_t ws_bytes,
                                   jabd_stream_t stream) {
  JABD_REQUIRE(num_images >= 0 && thresh_num > 0, "wider_eval: bad size");
  JABD_REQUIRE(pr_curve, "wider_eval: null pr_curve");
  if (num_images == 0 || total_preds == 0 || total_gts == 0) return JABD_OK;
  JABD_REQUIRE(total_gts < 0x7fffffff, "wider_eval: too many gts");
  JABD_REQUIRE(pred && pred_offsets && gt && ignore && gt_offsets && ws, "wider_eval: null");
  size_t need = 0;
  jabd_wider_eval_workspace_size(total_preds, total_gts, &need);
  JABD_REQUIRE(ws_bytes >= need, "wider_eval: workspace too small");
  Carve cv(ws, ws_bytes);
  double* maxov = cv.take<double>(total_preds);
  double* prec = cv.take<double>(total_preds);
  double* pcnt = cv.take<double>(total_preds);
  int* maxidx = cv.take<int>(total_preds);
  int* recall = cv.take<int>(total_gts);
  wider_eval_kernel<<<(unsigned)num_images, kEvalBlock, 0, as_stream(stream)>>>(
      pred, pred_offsets, gt, ignore, gt_offsets, iou_thresh, thresh_num, maxov, maxidx, recall,
      prec, pcnt, pr_curve);
  return check_launch("wider_eval");
}
