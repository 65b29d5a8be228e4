/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(),
 * bench.py's cpu_baseline leg).  Never linked into or called by the product.
 *
 * Plain-C restatement of the greedy NMS that predict.py reaches through
 * utils/utils_bbox.py:275 -> torchvision.ops.nms (torchvision is a
 * third-party dependency, absent from /root/reference and from this image;
 * version unpinned by the reference's requirements.txt).  Restated from
 * torchvision's published CPU algorithm (csrc/ops/cpu/nms_kernel.cpp):
 *   areas = (x2-x1)*(y2-y1) in fp32;  order = stable descending sort of scores;
 *   for i in order: skip if suppressed; keep i; for later j not suppressed:
 *     xx1=max(x1i,x1j) yy1=max(y1i,y1j) xx2=min(x2i,x2j) yy2=min(y2i,y2j)
 *     w=max(0,xx2-xx1) h=max(0,yy2-yy1) inter=w*h
 *     ovr=inter/(areai+areaj-inter)  (fp32);  suppress j if (double)ovr > thr.
 * Compiled with -ffp-contract=off so no multiply-add is fused.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  float s;
  int64_t i;
} item_t;

/* stable descending: higher score first, NaN first, ties by lower index */
static int cmp_desc(const void* a, const void* b) {
  const item_t* x = (const item_t*)a;
  const item_t* y = (const item_t*)b;
  int xn = isnan(x->s), yn = isnan(y->s);
  if (xn != yn) return xn ? -1 : 1;
  if (!xn) {
    if (x->s > y->s) return -1;
    if (x->s < y->s) return 1;
  }
  return (x->i < y->i) ? -1 : (x->i > y->i);
}

static inline float fmax_std(float a, float b) { return (a < b) ? b : a; } /* std::max */
static inline float fmin_std(float a, float b) { return (b < a) ? b : a; } /* std::min */

/* boxes [n,4] row-major, scores [n]; writes kept indices, returns count. */
int64_t oracle_nms(const float* boxes, const float* scores, int64_t n, double thr,
                   int64_t* keep) {
  if (n <= 0) return 0;
  item_t* it = (item_t*)malloc(sizeof(item_t) * n);
  float* area = (float*)malloc(sizeof(float) * n);
  unsigned char* sup = (unsigned char*)calloc(n, 1);
  for (int64_t k = 0; k < n; ++k) {
    it[k].s = scores[k];
    it[k].i = k;
    const float* b = boxes + 4 * k;
    area[k] = (b[2] - b[0]) * (b[3] - b[1]);
  }
  qsort(it, n, sizeof(item_t), cmp_desc);
  int64_t nk = 0;
  for (int64_t a = 0; a < n; ++a) {
    int64_t i = it[a].i;
    if (sup[i]) continue;
    keep[nk++] = i;
    const float* bi = boxes + 4 * i;
    float ix1 = bi[0], iy1 = bi[1], ix2 = bi[2], iy2 = bi[3], ia = area[i];
    for (int64_t c = a + 1; c < n; ++c) {
      int64_t j = it[c].i;
      if (sup[j]) continue;
      const float* bj = boxes + 4 * j;
      float xx1 = fmax_std(ix1, bj[0]);
      float yy1 = fmax_std(iy1, bj[1]);
      float xx2 = fmin_std(ix2, bj[2]);
      float yy2 = fmin_std(iy2, bj[3]);
      float w = fmax_std(0.f, xx2 - xx1);
      float h = fmax_std(0.f, yy2 - yy1);
      float inter = w * h;
      float ovr = inter / (ia + area[j] - inter);
      if ((double)ovr > thr) sup[j] = 1;
    }
  }
  free(it);
  free(area);
  free(sup);
  return nk;
}
