// A6-A10 box work on gfx950: decode / decode_landm, the fused predict.py
// post-process, batched anchor matching + encoding, and MultiBoxLoss with
// on-device hard-negative mining.  All HBM-bound integer/fp32 elementwise
// work; compiled with -ffp-contract=off so every float op rounds like the
// reference's separate tensor ops.
#include <math.h>

#include "common.h"
#include "nms_internal.h"

namespace jabd {

// ---------------------------------------------------------------------------
// decode / decode_landm — utils/utils_bbox.py:29-46
// ---------------------------------------------------------------------------
struct Box4 {
  float x1, y1, x2, y2;
};

__device__ __forceinline__ Box4 decode_one(const float* l, const float4 p, float v0, float v1) {
  // boxes = cat(p_c + l[:2]*v0*p_wh, p_wh*exp(l[2:]*v1)); boxes[:2] -= boxes[2:]/2;
  // boxes[2:] += boxes[:2]   (each a separate fp32 op, left to right)
  float cx = p.x + (l[0] * v0) * p.z;
  float cy = p.y + (l[1] * v0) * p.w;
  float w = p.z * expf(l[2] * v1);
  float h = p.w * expf(l[3] * v1);
  Box4 b;
  b.x1 = cx - w / 2.f;
  b.y1 = cy - h / 2.f;
  b.x2 = w + b.x1;
  b.y2 = h + b.y1;
  return b;
}

__global__ void decode_kernel(const float* __restrict__ loc, const float4* __restrict__ pri,
                              int64_t A, int64_t total, float v0, float v1,
                              float* __restrict__ out) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  float l[4];
  float4 lv = reinterpret_cast<const float4*>(loc)[i];
  l[0] = lv.x; l[1] = lv.y; l[2] = lv.z; l[3] = lv.w;
  Box4 b = decode_one(l, pri[i % A], v0, v1);
  reinterpret_cast<float4*>(out)[i] = make_float4(b.x1, b.y1, b.x2, b.y2);
}

__global__ void decode_landm_kernel(const float* __restrict__ pre, const float4* __restrict__ pri,
                                    int64_t A, int64_t total, float v0, float* __restrict__ out) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  float4 p = pri[i % A];
  const float* q = pre + i * 10;
  float* o = out + i * 10;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    o[2 * k] = p.x + (q[2 * k] * v0) * p.z;
    o[2 * k + 1] = p.y + (q[2 * k + 1] * v0) * p.w;
  }
}

// predict.py:167-180: rows (x1,y1,x2,y2, conf[:,1], landmarks) per prior.
__global__ void detect_rows_kernel(const float* __restrict__ loc, const float* __restrict__ conf,
                                   const float* __restrict__ landm,
                                   const float4* __restrict__ pri, int64_t A, int64_t total,
                                   float v0, float v1, float* __restrict__ rows) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  float4 p = pri[i % A];
  float l[4];
  float4 lv = reinterpret_cast<const float4*>(loc)[i];
  l[0] = lv.x; l[1] = lv.y; l[2] = lv.z; l[3] = lv.w;
  Box4 b = decode_one(l, p, v0, v1);
  float* r = rows + i * 15;
  r[0] = b.x1; r[1] = b.y1; r[2] = b.x2; r[3] = b.y2;
  r[4] = conf[i * 2 + 1];
  const float* q = landm + i * 10;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    r[5 + 2 * k] = p.x + (q[2 * k] * v0) * p.z;
    r[6 + 2 * k] = p.y + (q[2 * k + 1] * v0) * p.w;
  }
}

__global__ void gather_rows_kernel(const float* __restrict__ rows, const int64_t* __restrict__ keep,
                                   const int64_t* __restrict__ n_keep, int64_t A,
                                   float* __restrict__ out) {
  int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int b = blockIdx.y;
  if (k >= n_keep[b]) return;
  int64_t src = keep[(int64_t)b * A + k];
  const float* r = rows + ((int64_t)b * A + src) * 15;
  float* o = out + ((int64_t)b * A + k) * 15;
#pragma unroll
  for (int c = 0; c < 15; ++c) o[c] = r[c];
}

// ---------------------------------------------------------------------------
// match / encode — nets/retinaface_training.py:8-162
// ---------------------------------------------------------------------------
__device__ __forceinline__ float nan_min(float a, float b) {  // torch.min(a, b)
  return (a != a || b != b) ? __int_as_float(0x7fc00000) : (b < a ? b : a);
}
__device__ __forceinline__ float nan_max(float a, float b) {  // torch.max(a, b)
  return (a != a || b != b) ? __int_as_float(0x7fc00000) : (a < b ? b : a);
}

// jaccard(truth, point_form(prior)) for one pair, reference op order (:20-59).
__device__ __forceinline__ float match_iou(float tx1, float ty1, float tx2, float ty2,
                                           float tarea, float px1, float py1, float px2,
                                           float py2, float parea) {
  float mx = nan_min(tx2, px2), my = nan_min(ty2, py2);
  float nx = nan_max(tx1, px1), ny = nan_max(ty1, py1);
  float iw = nan_max(mx - nx, 0.f), ih = nan_max(my - ny, 0.f);  // clamp(min=0)
  float inter = iw * ih;
  float uni = tarea + parea - inter;
  return inter / uni;
}

// torch max(): larger value wins, NaN beats numbers, ties -> lower index.
__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return v > bv || (v == bv && i < bi);
}

__device__ __forceinline__ void prior_point_form(float4 p, float& x1, float& y1, float& x2,
                                                 float& y2, float& area) {
  x1 = p.x - p.z / 2.f;
  y1 = p.y - p.w / 2.f;
  x2 = p.x + p.z / 2.f;
  y2 = p.y + p.w / 2.f;
  area = (x2 - x1) * (y2 - y1);
}

// best_prior_idx per truth (:112-114) and the forced-match scatter (:128-130):
// forced[b][a] = max j with best_prior_idx[j] == a (the last writer of the
// reference's sequential loop).
__global__ __launch_bounds__(256) void match_best_prior_kernel(
    const float* __restrict__ targets, const int64_t* __restrict__ offsets,
    const float4* __restrict__ pri, int64_t A, int* __restrict__ forced) {
  const int b = blockIdx.y;
  const int64_t j = blockIdx.x;
  const int64_t t0 = offsets[b], t1 = offsets[b + 1];
  if (j >= t1 - t0) return;
  const float* tr = targets + (t0 + j) * 15;
  const float tx1 = tr[0], ty1 = tr[1], tx2 = tr[2], ty2 = tr[3];
  const float tarea = (tx2 - tx1) * (ty2 - ty1);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int64_t a = threadIdx.x; a < A; a += blockDim.x) {
    float px1, py1, px2, py2, pa;
    prior_point_form(pri[a], px1, py1, px2, py2, pa);
    float v = match_iou(tx1, ty1, tx2, ty2, tarea, px1, py1, px2, py2, pa);
    if (better(v, (int)a, bv, bi)) { bv = v; bi = (int)a; }
  }
  for (int off = 32; off > 0; off >>= 1) {
    float ov = __shfl_xor(bv, off);
    int oi = __shfl_xor(bi, off);
    if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { sv[wave] = bv; si[wave] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
      if (better(sv[w], si[w], bv, bi)) { bv = sv[w]; bi = si[w]; }
    atomicMax(&forced[(int64_t)b * A + bi], (int)j);
  }
}

// best_truth per prior (:121-123), forced override (:127-130), threshold
// (:145), encode (:62-73) and encode_landm (:75-86).  kRaw is match_iou()
// (nets/retinaface_training_DIOU.py:176-246): the same assignment, but loc_t
// holds the matched truth box corners (:230-231 `loc = matches`).
template <bool kRaw>
__global__ __launch_bounds__(256) void match_assign_kernel(
    const float* __restrict__ targets, const int64_t* __restrict__ offsets,
    const float4* __restrict__ pri, int64_t A, const int* __restrict__ forced,
    float thr, float v0, float v1, float* __restrict__ loc_t, int64_t* __restrict__ conf_t,
    float* __restrict__ landm_t) {
  extern __shared__ float st[];  // [ngt][5]: x1,y1,x2,y2,area
  const int b = blockIdx.y;
  const int64_t t0 = offsets[b];
  const int ngt = (int)(offsets[b + 1] - t0);
  for (int j = threadIdx.x; j < ngt; j += blockDim.x) {
    const float* tr = targets + (t0 + j) * 15;
    float x1 = tr[0], y1 = tr[1], x2 = tr[2], y2 = tr[3];
    st[j * 5 + 0] = x1; st[j * 5 + 1] = y1; st[j * 5 + 2] = x2; st[j * 5 + 3] = y2;
    st[j * 5 + 4] = (x2 - x1) * (y2 - y1);
  }
  __syncthreads();
  const int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (a >= A) return;
  const float4 p = pri[a];
  float px1, py1, px2, py2, pa;
  prior_point_form(p, px1, py1, px2, py2, pa);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int j = 0; j < ngt; ++j) {
    float v = match_iou(st[j * 5], st[j * 5 + 1], st[j * 5 + 2], st[j * 5 + 3], st[j * 5 + 4],
                        px1, py1, px2, py2, pa);
    if (better(v, j, bv, bi)) { bv = v; bi = j; }
  }
  const int64_t ba = (int64_t)b * A + a;
  const int f = forced[ba];
  if (f >= 0) { bv = 2.f; bi = f; }
  const float* tr = targets + (t0 + bi) * 15;
  float label = tr[14];
  if (bv < thr) label = 0.f;
  conf_t[ba] = (int64_t)label;
  // encode: ((m_lo+m_hi)/2 - p_c) / (v0*p_wh); log((m_hi-m_lo)/p_wh) / v1
  const float sw = v0 * p.z, sh = v0 * p.w;
  if (kRaw) {
    reinterpret_cast<float4*>(loc_t)[ba] = make_float4(tr[0], tr[1], tr[2], tr[3]);
  } else {
  float gx = (tr[0] + tr[2]) / 2.f - p.x;
  float gy = (tr[1] + tr[3]) / 2.f - p.y;
  gx /= sw;
  gy /= sh;
  float gw = logf((tr[2] - tr[0]) / p.z) / v1;
  float gh = logf((tr[3] - tr[1]) / p.w) / v1;
  reinterpret_cast<float4*>(loc_t)[ba] = make_float4(gx, gy, gw, gh);
  }
  float* lm = landm_t + ba * 10;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    lm[2 * k] = (tr[4 + 2 * k] - p.x) / sw;
    lm[2 * k + 1] = (tr[5 + 2 * k] - p.y) / sh;
  }
}

// ---------------------------------------------------------------------------
// MultiBoxLoss — nets/retinaface_training.py:183-303
// ---------------------------------------------------------------------------
constexpr int kLossBlock = 256;

__device__ __forceinline__ float wave_sum(float v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int off = 32; off > 0; off >>= 1) {
    float o = __shfl_xor(v, off);
    v = (o > v || o != o) ? o : v;  // NaN propagates like torch max()
  }
  return v;
}

__device__ __forceinline__ float smooth_l1(float d) {
  float z = fabsf(d);
  return z < 1.f ? 0.5f * z * z : z - 0.5f;
}

// ---------------------------------------------------------------------------
// DIoU box term — nets/retinaface_training_DIOU.py: IouLoss 'Diou' (:491-522)
// over decode() (:319-337) and bbox_overlaps_diou (:402-442), paired rows:
//   1 - clamp(I/U - |c2-c1|^2 / |outer|^2, -1, 1)
// ---------------------------------------------------------------------------
struct DiouTerms {
  Box4 b;                                  // decoded prediction (bboxes1)
  float w1, h1, iwr, ihr, iw, ih, inter;   // iwr/ihr before clamp(min=0)
  float dcx, dcy, diag, owr, ohr, ow, oh, odiag, uni, d;
};

__device__ __forceinline__ DiouTerms diou_terms(const float4 l, const float4 p, const float4 t,
                                                float v0, float v1) {
  const float la[4] = {l.x, l.y, l.z, l.w};
  DiouTerms r;
  r.b = decode_one(la, p, v0, v1);
  const Box4 b = r.b;
  r.w1 = b.x2 - b.x1;
  r.h1 = b.y2 - b.y1;
  const float w2 = t.z - t.x, h2 = t.w - t.y;
  const float area1 = r.w1 * r.h1, area2 = w2 * h2;
  const float cx1 = (b.x2 + b.x1) / 2.f, cy1 = (b.y2 + b.y1) / 2.f;
  const float cx2 = (t.z + t.x) / 2.f, cy2 = (t.w + t.y) / 2.f;
  r.iwr = nan_min(b.x2, t.z) - nan_max(b.x1, t.x);
  r.ihr = nan_min(b.y2, t.w) - nan_max(b.y1, t.y);
  r.iw = nan_max(r.iwr, 0.f);
  r.ih = nan_max(r.ihr, 0.f);
  r.inter = r.iw * r.ih;
  r.dcx = cx2 - cx1;
  r.dcy = cy2 - cy1;
  r.diag = r.dcx * r.dcx + r.dcy * r.dcy;
  r.owr = nan_max(b.x2, t.z) - nan_min(b.x1, t.x);
  r.ohr = nan_max(b.y2, t.w) - nan_min(b.y1, t.y);
  r.ow = nan_max(r.owr, 0.f);
  r.oh = nan_max(r.ohr, 0.f);
  r.odiag = r.ow * r.ow + r.oh * r.oh;
  r.uni = area1 + area2 - r.inter;
  r.d = r.inter / r.uni - r.diag / r.odiag;
  return r;
}

__device__ __forceinline__ float diou_loss(const float4 l, const float4 p, const float4 t,
                                           float v0, float v1) {
  const float d = diou_terms(l, p, t, v0, v1).d;
  return 1.f - fminf(fmaxf(d, -1.f), 1.f);
}

// torch.minimum/maximum backward: the whole gradient to the winner, half each on a tie.
__device__ __forceinline__ float pick_lo(float a, float b) { return a < b ? 1.f : (a == b ? .5f : 0.f); }
__device__ __forceinline__ float pick_hi(float a, float b) { return a > b ? 1.f : (a == b ? .5f : 0.f); }

// d(loss)/d(loc) for one positive, scaled by s (= dL/dloss_l / N).
__device__ __forceinline__ float4 diou_grad(const float4 l, const float4 p, const float4 t,
                                            float v0, float v1, float s) {
  const DiouTerms r = diou_terms(l, p, t, v0, v1);
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!(r.d >= -1.f && r.d <= 1.f)) return g;  // clamp() passes the gradient on [-1, 1]
  const float gd = -s;
  const float U2 = r.uni * r.uni;
  const float gI = gd * (1.f / r.uni + r.inter / U2);
  const float gA1 = gd * (-r.inter / U2);
  const float gD = gd * (-1.f / r.odiag);
  const float gO = gd * (r.diag / (r.odiag * r.odiag));
  const Box4 b = r.b;
  float gx1 = 0.f, gy1 = 0.f, gx2 = 0.f, gy2 = 0.f;
  // area1 = w1*h1
  gx2 += gA1 * r.h1; gx1 -= gA1 * r.h1;
  gy2 += gA1 * r.w1; gy1 -= gA1 * r.w1;
  // inter = clamp(iw)*clamp(ih); iw = min(x2,tx2) - max(x1,tx1)
  const float giw = r.iwr >= 0.f ? gI * r.ih : 0.f;
  const float gih = r.ihr >= 0.f ? gI * r.iw : 0.f;
  gx2 += giw * pick_lo(b.x2, t.z); gx1 -= giw * pick_hi(b.x1, t.x);
  gy2 += gih * pick_lo(b.y2, t.w); gy1 -= gih * pick_hi(b.y1, t.y);
  // diag = (c2 - c1)^2, c1 = (x2 + x1)/2
  const float gcx1 = gD * -2.f * r.dcx, gcy1 = gD * -2.f * r.dcy;
  gx1 += gcx1 * .5f; gx2 += gcx1 * .5f;
  gy1 += gcy1 * .5f; gy2 += gcy1 * .5f;
  // odiag = clamp(ow)^2 + clamp(oh)^2; ow = max(x2,tx2) - min(x1,tx1)
  const float gow = r.owr >= 0.f ? gO * 2.f * r.ow : 0.f;
  const float goh = r.ohr >= 0.f ? gO * 2.f * r.oh : 0.f;
  gx2 += gow * pick_hi(b.x2, t.z); gx1 -= gow * pick_lo(b.x1, t.x);
  gy2 += goh * pick_hi(b.y2, t.w); gy1 -= goh * pick_lo(b.y1, t.y);
  // decode: x1 = cx - W/2, x2 = x1 + W; cx = px + l0*v0*pw, W = pw*exp(l2*v1)
  const float gcx = gx1 + gx2, gcy = gy1 + gy2;
  const float gW = (gx2 - gx1) * .5f, gH = (gy2 - gy1) * .5f;
  const float W = p.z * expf(l.z * v1);
  const float H = p.w * expf(l.w * v1);
  g.x = gcx * v0 * p.z;
  g.y = gcy * v0 * p.w;
  g.z = gW * W * v1;
  g.w = gH * H * v1;
  return g;
}

// Global max of conf (log_sum_exp uses x.data.max(), :86-88): block partials.
__global__ __launch_bounds__(kLossBlock) void conf_max_partial(const float* __restrict__ conf,
                                                               int64_t total,
                                                               float* __restrict__ part) {
  float m = -INFINITY;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = conf[i];
    m = (v > m || v != v) ? v : m;
  }
  m = wave_max(m);
  __shared__ float s[kLossBlock / 64];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kLossBlock / 64; ++w) m = (s[w] > m || s[w] != s[w]) ? s[w] : m;
    part[blockIdx.x] = m;
  }
}

// Per prior: box/landmark smooth-L1 partials, positive counts, and the
// hard-negative mining loss (lse(x) - x[t], positives zeroed, :256-262).
// kDiou: the box term is the DIoU loss of the decoded prediction against the
// raw matched truth (retinaface_training_DIOU.py:600-602); pri/v0/v1 unused otherwise.
template <bool kDiou>
__global__ __launch_bounds__(kLossBlock) void loss_elem_kernel(
    const float* __restrict__ loc, const float* __restrict__ conf,
    const float* __restrict__ landm, const float* __restrict__ loc_t,
    const int64_t* __restrict__ conf_t, const float* __restrict__ landm_t, int64_t A,
    const float4* __restrict__ pri, float v0, float v1,
    const float* __restrict__ gmax_part, int n_gmax_part, float* __restrict__ mining,
    uint8_t* __restrict__ sel, float* __restrict__ part_l, float* __restrict__ part_lm,
    int* __restrict__ npos_img, int* __restrict__ npos1_img) {
  __shared__ float s_gmax;
  if (threadIdx.x == 0) {
    float m = -INFINITY;
    for (int i = 0; i < n_gmax_part; ++i) {
      float v = gmax_part[i];
      m = (v > m || v != v) ? v : m;
    }
    s_gmax = m;
  }
  __syncthreads();
  const float gmax = s_gmax;
  const int b = blockIdx.y;
  const int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  float sl = 0.f, slm = 0.f;
  int p = 0, p1 = 0;
  if (a < A) {
    const int64_t i = (int64_t)b * A + a;
    const int64_t t = conf_t[i];
    const bool pos = t != 0, pos1 = t > 0;
    if (pos) {
      float4 x = reinterpret_cast<const float4*>(loc)[i];
      float4 y = reinterpret_cast<const float4*>(loc_t)[i];
      if (kDiou)
        sl = diou_loss(x, pri[a], y, v0, v1);
      else
        sl = smooth_l1(x.x - y.x) + smooth_l1(x.y - y.y) + smooth_l1(x.z - y.z) +
             smooth_l1(x.w - y.w);
    }
    if (pos1) {
      const float* x = landm + i * 10;
      const float* y = landm_t + i * 10;
#pragma unroll
      for (int k = 0; k < 10; ++k) slm += smooth_l1(x[k] - y[k]);
    }
    const float c0 = conf[i * 2], c1 = conf[i * 2 + 1];
    const float lse = logf(expf(c0 - gmax) + expf(c1 - gmax)) + gmax;
    const float mine = pos ? 0.f : lse - c0;  // target is 0 for every non-positive
    mining[i] = mine;
    sel[i] = (uint8_t)((pos ? 1 : 0) | (pos1 ? 2 : 0));
    p = pos;
    p1 = pos1;
  }
  sl = wave_sum(sl);
  slm = wave_sum(slm);
  uint64_t bp = __ballot(p), bp1 = __ballot(p1);
  __shared__ float s_l[kLossBlock / 64], s_lm[kLossBlock / 64];
  __shared__ int s_p[kLossBlock / 64], s_p1[kLossBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_l[wave] = sl; s_lm[wave] = slm;
    s_p[wave] = __popcll(bp); s_p1[wave] = __popcll(bp1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tl = 0.f, tlm = 0.f;
    int tp = 0, tp1 = 0;
    for (int w = 0; w < kLossBlock / 64; ++w) {
      tl += s_l[w]; tlm += s_lm[w]; tp += s_p[w]; tp1 += s_p1[w];
    }
    const int64_t blk = (int64_t)b * gridDim.x + blockIdx.x;
    part_l[blk] = tl;
    part_lm[blk] = tlm;
    if (tp) atomicAdd(&npos_img[b], tp);
    if (tp1) atomicAdd(&npos1_img[b], tp1);
  }
}

__device__ __forceinline__ uint32_t fkey_asc(float v) {
  uint32_t f = __float_as_uint(v);
  if (v != v) f = 0x7fc00000u;
  if (f == 0x80000000u) f = 0u;
  return (f & 0x80000000u) ? ~f : (f | 0x80000000u);
}

constexpr int kSelBlock = 1024;

// Per image: radix-select the num_neg-th largest mining loss (:270-276),
// mark pos ∪ neg (bit 2) and sum the cross-entropy of the marked rows
// (:283-293).  Ties at the threshold are taken lowest index first.
__global__ __launch_bounds__(kSelBlock) void ohem_select_kernel(
    const float* __restrict__ mining, const float* __restrict__ conf, int64_t A, int neg_pos,
    const int* __restrict__ npos_img, uint8_t* __restrict__ sel, float* __restrict__ ce_img) {
  const int b = blockIdx.x;
  const float* m = mining + (int64_t)b * A;
  __shared__ int hist[256];
  __shared__ uint32_t s_prefix;
  __shared__ int s_need;
  __shared__ int s_wave[kSelBlock / 64];
  __shared__ float s_wsum[kSelBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t npos = npos_img[b];
  int64_t num_neg = (int64_t)neg_pos * npos;
  if (num_neg > A - 1) num_neg = A - 1;

  uint32_t prefix = 0;
  int need = (int)num_neg;  // still to take among keys matching prefix
  if (num_neg > 0) {
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      const uint32_t pmask = pass == 0 ? 0u : (0xffffffffu << (32 - 8 * pass));
      for (int i = tid; i < 256; i += kSelBlock) hist[i] = 0;
      __syncthreads();
      for (int64_t i = tid; i < A; i += kSelBlock) {
        uint32_t k = fkey_asc(m[i]);
        if ((k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
      }
      __syncthreads();
      if (tid == 0) {
        int acc = 0, d = 255;
        for (; d > 0; --d) {
          if (acc + hist[d] >= need) break;
          acc += hist[d];
        }
        s_prefix = prefix | ((uint32_t)d << shift);
        s_need = need - acc;
      }
      __syncthreads();
      prefix = s_prefix;
      need = s_need;
      __syncthreads();
    }
  }
  // prefix = key of the num_neg-th largest; take every key > prefix and the
  // first `need` keys == prefix in index order.
  int taken_eq = 0;
  float ce = 0.f;
  for (int64_t base = 0; base < A; base += kSelBlock) {
    const int64_t i = base + tid;
    bool valid = i < A;
    uint32_t k = valid ? fkey_asc(m[i]) : 0u;
    bool gt = valid && num_neg > 0 && k > prefix;
    bool eq = valid && num_neg > 0 && k == prefix;
    uint64_t be = __ballot(eq);
    int rank_in_wave = __popcll(be & (((uint64_t)1 << lane) - 1));
    if (lane == 0) s_wave[wave] = __popcll(be);
    __syncthreads();
    int before = taken_eq;
    for (int w = 0; w < wave; ++w) before += s_wave[w];
    int tot = 0;
    for (int w = 0; w < kSelBlock / 64; ++w) tot += s_wave[w];
    bool take_eq = eq && (before + rank_in_wave) < need;
    if (valid) {
      const int64_t gi = (int64_t)b * A + i;
      uint8_t s = sel[gi];
      const bool pos = s & 1;
      if (pos || gt || take_eq) {
        s |= 4;
        sel[gi] = s;
        // F.cross_entropy row: -(x_t - max - log(sum exp(x - max)))
        const float c0 = conf[gi * 2], c1 = conf[gi * 2 + 1];
        const float mx = c0 < c1 ? c1 : c0;
        const float lsm = logf(expf(c0 - mx) + expf(c1 - mx));
        const float xt = pos ? c1 : c0;
        ce += -((xt - mx) - lsm);
      }
    }
    taken_eq += tot;
    __syncthreads();
  }
  ce = wave_sum(ce);
  if (lane == 0) s_wsum[wave] = ce;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int w = 0; w < kSelBlock / 64; ++w) t += s_wsum[w];
    ce_img[b] = t;
  }
}

__global__ void loss_final_kernel(const float* __restrict__ part_l,
                                  const float* __restrict__ part_lm, int64_t nparts,
                                  const float* __restrict__ ce_img, const int* __restrict__ npos,
                                  const int* __restrict__ npos1, int batch,
                                  float* __restrict__ sums, int64_t* __restrict__ counts) {
  // one wave; fixed-order partial sums -> deterministic
  const int lane = threadIdx.x;
  float sl = 0.f, slm = 0.f, sc = 0.f;
  int64_t p = 0, p1 = 0;
  for (int64_t i = lane; i < nparts; i += 64) { sl += part_l[i]; slm += part_lm[i]; }
  for (int i = lane; i < batch; i += 64) { sc += ce_img[i]; p += npos[i]; p1 += npos1[i]; }
  sl = wave_sum(sl); slm = wave_sum(slm); sc = wave_sum(sc);
  for (int off = 32; off > 0; off >>= 1) {
    p += __shfl_xor(p, off);
    p1 += __shfl_xor(p1, off);
  }
  if (lane == 0) {
    sums[0] = sl; sums[1] = sc; sums[2] = slm;
    counts[0] = p; counts[1] = p1;
  }
}

__global__ void loss_normalize_kernel(const float* __restrict__ sums,
                                      const int64_t* __restrict__ counts,
                                      float* __restrict__ loss) {
  if (threadIdx.x != 0) return;
  const float n = (float)(counts[0] > 1 ? counts[0] : 1);
  const float n1 = (float)(counts[1] > 1 ? counts[1] : 1);
  loss[0] = sums[0] / n;
  loss[1] = sums[1] / n;
  loss[2] = sums[2] / n1;
}

__device__ __forceinline__ float sl1_grad(float d) { return d < -1.f ? -1.f : (d > 1.f ? 1.f : d); }

template <bool kDiou>
__global__ void loss_bwd_kernel(const float* __restrict__ loc, const float* __restrict__ conf,
                                const float* __restrict__ landm, const float* __restrict__ loc_t,
                                const int64_t* __restrict__ conf_t,
                                const float* __restrict__ landm_t,
                                const float4* __restrict__ pri, int64_t A, float v0, float v1,
                                const uint8_t* __restrict__ sel, int64_t total,
                                const float* __restrict__ gout,
                                const int64_t* __restrict__ counts, float* __restrict__ gl,
                                float* __restrict__ gc, float* __restrict__ glm) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float n = (float)(counts[0] > 1 ? counts[0] : 1);
  const float n1 = (float)(counts[1] > 1 ? counts[1] : 1);
  const float sl = gout[0] / n, sc = gout[1] / n, slm = gout[2] / n1;
  const uint8_t s = sel[i];
  const bool pos = s & 1, pos1 = s & 2, ce = s & 4;
  if (gl) {
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (pos) {
      float4 x = reinterpret_cast<const float4*>(loc)[i];
      float4 y = reinterpret_cast<const float4*>(loc_t)[i];
      if (kDiou)
        g = diou_grad(x, pri[i % A], y, v0, v1, sl);
      else
        g = make_float4(sl1_grad(x.x - y.x) * sl, sl1_grad(x.y - y.y) * sl,
                        sl1_grad(x.z - y.z) * sl, sl1_grad(x.w - y.w) * sl);
    }
    reinterpret_cast<float4*>(gl)[i] = g;
  }
  if (glm) {
#pragma unroll
    for (int k = 0; k < 10; ++k)
      glm[i * 10 + k] = pos1 ? sl1_grad(landm[i * 10 + k] - landm_t[i * 10 + k]) * slm : 0.f;
  }
  if (gc) {
    float g0 = 0.f, g1 = 0.f;
    if (ce) {
      const float c0 = conf[i * 2], c1 = conf[i * 2 + 1];
      const float mx = c0 < c1 ? c1 : c0;
      const float e0 = expf(c0 - mx), e1 = expf(c1 - mx);
      const float z = e0 + e1;
      const float t1 = pos ? 1.f : 0.f;
      g0 = (e0 / z - (1.f - t1)) * sc;
      g1 = (e1 / z - t1) * sc;
    }
    gc[i * 2] = g0;
    gc[i * 2 + 1] = g1;
  }
}

template <typename Al>
static void carve_loss(Al& a, int64_t B, int64_t A, int64_t ngmax) {
  const int64_t nblk = cdiv(A, kLossBlock);
  a.template take<float>(ngmax);       // gmax partials
  a.template take<float>(B * A);       // mining loss
  a.template take<float>(B * nblk);    // part_l
  a.template take<float>(B * nblk);    // part_lm
  a.template take<int>(B);             // npos
  a.template take<int>(B);             // npos1
  a.template take<float>(B);           // ce per image
}

static int64_t gmax_blocks(int64_t total) {
  int64_t g = cdiv(total, kLossBlock * 8);
  return g < 1 ? 1 : (g > 1024 ? 1024 : g);
}

// ---------------------------------------------------------------------------
// letterbox_image + preprocess_input — utils/utils.py:8-19,27-29 as predict.py
// calls them (:122,143-152): a float32 HWC image is cv2.resize'd (INTER_LINEAR,
// float path) to nw x nh, pasted at ((h-nh)//2, (w-nw)//2) on a canvas filled
// with `fill`, then (NCHW mode) the channel means are subtracted and the result
// transposed to [3, h, w].  cv2's float INTER_LINEAR restated (cv2 is absent
// here, parity unpinned against it): per axis f = (float)((d + .5) * scale - .5),
// s = floor(f), f -= s; s < 0 -> (s, f) = (0, 0); s >= n-1 -> (n-1, 0); taps
// combined as S0*(1-f) + S1*f in fp32 (separate products, -ffp-contract=off),
// horizontal pass first.  An exact 2x downscale is cv2's INTER_AREA fast path:
// (S00 + S01 + S10 + S11) * 0.25f.  One thread per canvas pixel, three channels.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lin_tap(int d, double scale, int n, int& s0, int& s1, float& f) {
  float fx = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(fx);
  fx -= (float)s;
  if (s < 0) { s = 0; fx = 0.f; }
  if (s >= n - 1) { s = n - 1; fx = 0.f; }
  s0 = s;
  s1 = s + 1 < n ? s + 1 : n - 1;
  f = fx;
}

__global__ __launch_bounds__(256) void letterbox_kernel(
    const float* __restrict__ src, int ih, int iw, float* __restrict__ dst, int h, int w,
    int nw, int nh, int top, int left, double sx, double sy, int area2x, float fill, float m0,
    float m1, float m2, int nchw) {
  const int b = blockIdx.y;
  const int64_t pix = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (pix >= (int64_t)h * w) return;
  const int y = (int)(pix / w), x = (int)(pix - (int64_t)y * w);
  const float* S = src + (int64_t)b * ih * iw * 3;
  float v[3] = {fill, fill, fill};
  const int ry = y - top, rx = x - left;
  if (ry >= 0 && ry < nh && rx >= 0 && rx < nw) {
    if (area2x) {
      const float* r0 = S + ((int64_t)(2 * ry) * iw + 2 * rx) * 3;
      const float* r1 = r0 + (int64_t)iw * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = (r0[c] + r0[c + 3] + r1[c] + r1[c + 3]) * 0.25f;
    } else {
      int x0, x1, y0, y1;
      float fx, fy;
      lin_tap(rx, sx, iw, x0, x1, fx);
      lin_tap(ry, sy, ih, y0, y1, fy);
      const float ax0 = 1.f - fx, ay0 = 1.f - fy;
      const float* p00 = S + ((int64_t)y0 * iw + x0) * 3;
      const float* p01 = S + ((int64_t)y0 * iw + x1) * 3;
      const float* p10 = S + ((int64_t)y1 * iw + x0) * 3;
      const float* p11 = S + ((int64_t)y1 * iw + x1) * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float h0 = p00[c] * ax0 + p01[c] * fx;
        const float h1 = p10[c] * ax0 + p11[c] * fx;
        v[c] = h0 * ay0 + h1 * fy;
      }
    }
  }
  if (nchw) {
    float* D = dst + (int64_t)b * 3 * h * w + pix;
    const int64_t plane = (int64_t)h * w;
    D[0] = v[0] - m0;
    D[plane] = v[1] - m1;
    D[2 * plane] = v[2] - m2;
  } else {
    float* D = dst + ((int64_t)b * h * w + pix) * 3;
    D[0] = v[0]; D[1] = v[1]; D[2] = v[2];
  }
}

// retinaface_correct_boxes (utils/utils_bbox.py:9-24) then predict.py's
// rescale to image pixels (:195-196) on detection rows [n, 15]: numpy does
// both in float64 and assigns back into the float32 rows, so each step is
// (float)((double)v - off) * sc) and (float)((double)v * dim).
__global__ void correct_rows_kernel(float* __restrict__ rows, int64_t n, int letterbox,
                                    double offx, double offy, double scx, double scy,
                                    double dimx, double dimy) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n * 15) return;
  const int c = (int)(i % 15);
  if (c == 4) return;  // the score column is untouched
  const bool isx = ((c < 4 ? c : c - 5) & 1) == 0;
  float v = rows[i];
  if (letterbox) v = (float)(((double)v - (isx ? offx : offy)) * (isx ? scx : scy));
  rows[i] = (float)((double)v * (isx ? dimx : dimy));  // x * 1.0 is exact when !to_pixels
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_correct_boxes_f32(float* rows, int64_t n, int input_h, int input_w,
                                      int image_h, int image_w, int letterbox,
                                      int to_pixels, jabd_stream_t stream) {
  JABD_REQUIRE(n >= 0 && image_h > 0 && image_w > 0, "correct_boxes: bad size");
  JABD_REQUIRE(!letterbox || (input_h > 0 && input_w > 0), "correct_boxes: bad input shape");
  if (n == 0) return JABD_OK;
  JABD_REQUIRE(rows, "correct_boxes: null pointer");
  // utils_bbox.py:10-12, numpy float64 over [h, w] pairs
  double offx = 0, offy = 0, scx = 1, scy = 1;
  if (letterbox) {
    const double r = fmin((double)input_h / image_h, (double)input_w / image_w);
    const double nh = image_h * r, nw = image_w * r;
    offy = (input_h - nh) / 2. / input_h;
    offx = (input_w - nw) / 2. / input_w;
    scy = input_h / nh;
    scx = input_w / nw;
  }
  correct_rows_kernel<<<(unsigned)cdiv(n * 15, 256), 256, 0, as_stream(stream)>>>(
      rows, n, letterbox, offx, offy, scx, scy, to_pixels ? (double)image_w : 1.0,
      to_pixels ? (double)image_h : 1.0);
  return check_launch("correct_boxes");
}

extern "C" int jabd_letterbox_f32(const float* src, int64_t batch, int ih, int iw, float* dst,
                                  int h, int w, float fill, const float* mean3, int nchw,
                                  jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && ih > 0 && iw > 0 && h > 0 && w > 0, "letterbox: bad size");
  JABD_REQUIRE(!nchw || mean3, "letterbox: NCHW output needs the channel means");
  if (batch == 0) return JABD_OK;
  JABD_REQUIRE(src && dst, "letterbox: null pointer");
  // utils/utils.py:10-13: scale = min(w/iw, h/ih); nw = int(iw*scale); nh = int(ih*scale)
  const double sc = fmin((double)w / iw, (double)h / ih);
  const int nw = (int)(iw * sc), nh = (int)(ih * sc);
  JABD_REQUIRE(nw > 0 && nh > 0, "letterbox: image %dx%d collapses to %dx%d", iw, ih, nw, nh);
  const int top = (h - nh) / 2, left = (w - nw) / 2;
  // cv2.resize: inv_scale = dsize/ssize, scale = 1/inv_scale; exact 2x -> INTER_AREA
  const double sx = 1.0 / ((double)nw / iw), sy = 1.0 / ((double)nh / ih);
  const int area2x = (iw == 2 * nw && ih == 2 * nh) ? 1 : 0;
  const float m[3] = {nchw ? mean3[0] : 0.f, nchw ? mean3[1] : 0.f, nchw ? mean3[2] : 0.f};
  const int64_t npix = (int64_t)h * w;
  dim3 g((unsigned)cdiv(npix, 256), (unsigned)batch);
  letterbox_kernel<<<g, 256, 0, as_stream(stream)>>>(src, ih, iw, dst, h, w, nw, nh, top, left,
                                                      sx, sy, area2x, fill, m[0], m[1], m[2],
                                                      nchw);
  return check_launch("letterbox");
}

extern "C" int jabd_decode_f32(const float* loc, const float* priors, int64_t batch,
                               int64_t num_priors, float var0, float var1, float* boxes,
                               jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && num_priors >= 0, "decode: negative size");
  const int64_t total = batch * num_priors;
  if (total == 0) return JABD_OK;
  JABD_REQUIRE(loc && priors && boxes, "decode: null pointer");
  decode_kernel<<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      loc, reinterpret_cast<const float4*>(priors), num_priors, total, var0, var1, boxes);
  return check_launch("decode");
}

extern "C" int jabd_decode_landm_f32(const float* pre, const float* priors, int64_t batch,
                                     int64_t num_priors, float var0, float* landms,
                                     jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && num_priors >= 0, "decode_landm: negative size");
  const int64_t total = batch * num_priors;
  if (total == 0) return JABD_OK;
  JABD_REQUIRE(pre && priors && landms, "decode_landm: null pointer");
  decode_landm_kernel<<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      pre, reinterpret_cast<const float4*>(priors), num_priors, total, var0, landms);
  return check_launch("decode_landm");
}

static size_t detect_ws(int64_t B, int64_t A) {
  Sizer s;
  s.take<float>(B * A * 15);
  s.take<int64_t>(B * A);
  s.take<char>(nms_ws_bytes(B, A));
  return s.used;
}

extern "C" int jabd_detect_workspace_size(int64_t batch, int64_t num_priors, size_t* bytes) {
  JABD_REQUIRE(bytes && batch >= 0 && num_priors >= 0, "detect_workspace_size: bad args");
  *bytes = detect_ws(batch, num_priors);
  return JABD_OK;
}

extern "C" int jabd_detect_f32(const float* loc, const float* conf, const float* landm,
                               const float* priors, int64_t batch, int64_t num_priors,
                               float var0, float var1, float conf_threshold,
                               double nms_threshold, float* out, int64_t* n_keep, void* ws,
                               size_t ws_bytes, jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && num_priors >= 0, "detect: negative size");
  if (batch == 0) return JABD_OK;
  hipStream_t st = as_stream(stream);
  if (num_priors == 0) {
    const FillRange fr{n_keep, (int64_t)sizeof(int64_t) * batch, 0u};
    if (int e = fill_ranges(&fr, 1, st)) return e;
    return JABD_OK;
  }
  JABD_REQUIRE(loc && conf && landm && priors && out && n_keep, "detect: null pointer");
  JABD_REQUIRE(ws_bytes >= detect_ws(batch, num_priors), "detect: workspace too small");
  Carve cv(ws, ws_bytes);
  float* rows = cv.take<float>(batch * num_priors * 15);
  int64_t* keep = cv.take<int64_t>(batch * num_priors);
  size_t nws = nms_ws_bytes(batch, num_priors);
  void* nmsws = cv.take<char>(nws);
  const int64_t total = batch * num_priors;
  detect_rows_kernel<<<(unsigned)cdiv(total, 256), 256, 0, st>>>(
      loc, conf, landm, reinterpret_cast<const float4*>(priors), num_priors, total, var0, var1,
      rows);
  if (int e = check_launch("detect_rows")) return e;
  if (int e = nms_core(rows, 15, num_priors * 15, rows + 4, 15, num_priors * 15, nullptr, batch,
                       num_priors, nms_threshold, conf_threshold, keep, n_keep, nmsws, nws, st))
    return e;
  dim3 g((unsigned)cdiv(num_priors, 256), (unsigned)batch);
  gather_rows_kernel<<<g, 256, 0, st>>>(rows, keep, n_keep, num_priors, out);
  return check_launch("detect_gather");
}

static size_t match_ws(int64_t B, int64_t A) {
  Sizer s;
  s.take<int>(B * A);
  return s.used;
}

extern "C" int jabd_match_workspace_size(int64_t batch, int64_t num_priors, size_t* bytes) {
  JABD_REQUIRE(bytes && batch >= 0 && num_priors >= 0, "match_workspace_size: bad args");
  *bytes = match_ws(batch, num_priors);
  return JABD_OK;
}

static int match_impl(bool raw, const float* targets, const int64_t* offsets, int64_t batch,
                      int64_t max_gt, const float* priors, int64_t num_priors, float threshold,
                      float var0, float var1, float* loc_t, int64_t* conf_t, float* landm_t,
                      void* ws, size_t ws_bytes, jabd_stream_t stream) {
  JABD_REQUIRE(batch >= 0 && num_priors >= 0 && max_gt >= 0, "match: negative size");
  if (batch == 0 || num_priors == 0) return JABD_OK;
  JABD_REQUIRE(max_gt > 0, "match: an image has no targets (reference match() fails too)");
  JABD_REQUIRE(max_gt <= 3276, "match: max_gt=%lld > 3276 targets in one image", (long long)max_gt);
  JABD_REQUIRE(num_priors < 0x7fffffff, "match: too many priors");
  JABD_REQUIRE(targets && offsets && priors && loc_t && conf_t && landm_t, "match: null pointer");
  JABD_REQUIRE(ws_bytes >= match_ws(batch, num_priors), "match: workspace too small");
  hipStream_t st = as_stream(stream);
  Carve cv(ws, ws_bytes);
  int* forced = cv.take<int>(batch * num_priors);
  {
    const FillRange fr{forced, (int64_t)sizeof(int) * batch * num_priors, 0xFFFFFFFFu};  // -1
    if (int e = fill_ranges(&fr, 1, st)) return e;
  }
  const float4* pri = reinterpret_cast<const float4*>(priors);
  dim3 g1((unsigned)max_gt, (unsigned)batch);
  match_best_prior_kernel<<<g1, 256, 0, st>>>(targets, offsets, pri, num_priors, forced);
  if (int e = check_launch("match_best_prior")) return e;
  dim3 g2((unsigned)cdiv(num_priors, 256), (unsigned)batch);
  if (raw)
    match_assign_kernel<true><<<g2, 256, max_gt * 5 * sizeof(float), st>>>(
        targets, offsets, pri, num_priors, forced, threshold, var0, var1, loc_t, conf_t, landm_t);
  else
    match_assign_kernel<false><<<g2, 256, max_gt * 5 * sizeof(float), st>>>(
        targets, offsets, pri, num_priors, forced, threshold, var0, var1, loc_t, conf_t, landm_t);
  return check_launch("match_assign");
}

extern "C" int jabd_match_encode_f32(const float* targets, const int64_t* offsets,
                                     int64_t batch, int64_t max_gt, const float* priors,
                                     int64_t num_priors, float threshold, float var0,
                                     float var1, float* loc_t, int64_t* conf_t,
                                     float* landm_t, void* ws, size_t ws_bytes,
                                     jabd_stream_t stream) {
  return match_impl(false, targets, offsets, batch, max_gt, priors, num_priors, threshold, var0,
                    var1, loc_t, conf_t, landm_t, ws, ws_bytes, stream);
}

extern "C" int jabd_match_iou_f32(const float* targets, const int64_t* offsets, int64_t batch,
                                  int64_t max_gt, const float* priors, int64_t num_priors,
                                  float threshold, float var0, float var1, float* loc_t,
                                  int64_t* conf_t, float* landm_t, void* ws, size_t ws_bytes,
                                  jabd_stream_t stream) {
  return match_impl(true, targets, offsets, batch, max_gt, priors, num_priors, threshold, var0,
                    var1, loc_t, conf_t, landm_t, ws, ws_bytes, stream);
}

extern "C" int jabd_multibox_workspace_size(int64_t batch, int64_t num_priors, size_t* bytes) {
  JABD_REQUIRE(bytes && batch >= 0 && num_priors >= 0, "multibox_workspace_size: bad args");
  Sizer s;
  carve_loss(s, batch, num_priors, gmax_blocks(batch * num_priors * 2));
  *bytes = s.used;
  return JABD_OK;
}

static int loss_fwd_impl(const float* loc, const float* conf, const float* landm,
                         const float* loc_t, const int64_t* conf_t, const float* landm_t,
                         const float* priors, float v0, float v1, int64_t batch,
                         int64_t num_priors, int neg_pos, float* sums, int64_t* counts,
                         uint8_t* sel, void* ws, size_t ws_bytes, jabd_stream_t stream) {
  JABD_REQUIRE(batch > 0 && num_priors > 0, "multibox: empty batch");
  JABD_REQUIRE(num_priors < 0x7fffffff, "multibox: too many priors");
  JABD_REQUIRE(loc && conf && landm && loc_t && conf_t && landm_t && sums && counts && sel,
               "multibox: null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t B = batch, A = num_priors;
  const int64_t ng = gmax_blocks(B * A * 2);
  Sizer sz;
  carve_loss(sz, B, A, ng);
  JABD_REQUIRE(ws_bytes >= sz.used, "multibox: workspace %zu < %zu", ws_bytes, sz.used);
  Carve cv(ws, ws_bytes);
  const int64_t nblk = cdiv(A, kLossBlock);
  float* gpart = cv.take<float>(ng);
  float* mining = cv.take<float>(B * A);
  float* part_l = cv.take<float>(B * nblk);
  float* part_lm = cv.take<float>(B * nblk);
  int* npos = cv.take<int>(B);
  int* npos1 = cv.take<int>(B);
  float* ce = cv.take<float>(B);
  {
    const FillRange fr[2] = {{npos, (int64_t)sizeof(int) * B, 0u},
                             {npos1, (int64_t)sizeof(int) * B, 0u}};
    if (int e = fill_ranges(fr, 2, st)) return e;
  }
  conf_max_partial<<<(unsigned)ng, kLossBlock, 0, st>>>(conf, B * A * 2, gpart);
  if (int e = check_launch("conf_max")) return e;
  dim3 g((unsigned)nblk, (unsigned)B);
  const float4* pri = reinterpret_cast<const float4*>(priors);
  if (pri)
    loss_elem_kernel<true><<<g, kLossBlock, 0, st>>>(loc, conf, landm, loc_t, conf_t, landm_t, A,
                                                     pri, v0, v1, gpart, (int)ng, mining, sel,
                                                     part_l, part_lm, npos, npos1);
  else
    loss_elem_kernel<false><<<g, kLossBlock, 0, st>>>(loc, conf, landm, loc_t, conf_t, landm_t,
                                                      A, pri, v0, v1, gpart, (int)ng, mining,
                                                      sel, part_l, part_lm, npos, npos1);
  if (int e = check_launch("loss_elem")) return e;
  ohem_select_kernel<<<(unsigned)B, kSelBlock, 0, st>>>(mining, conf, A, neg_pos, npos, sel, ce);
  if (int e = check_launch("ohem_select")) return e;
  loss_final_kernel<<<1, 64, 0, st>>>(part_l, part_lm, B * nblk, ce, npos, npos1, (int)B, sums,
                                      counts);
  return check_launch("loss_final");
}

extern "C" int jabd_multibox_loss_fwd_f32(const float* loc, const float* conf,
                                          const float* landm, const float* loc_t,
                                          const int64_t* conf_t, const float* landm_t,
                                          int64_t batch, int64_t num_priors, int neg_pos,
                                          float* sums, int64_t* counts, uint8_t* sel, void* ws,
                                          size_t ws_bytes, jabd_stream_t stream) {
  return loss_fwd_impl(loc, conf, landm, loc_t, conf_t, landm_t, nullptr, 0.f, 0.f, batch,
                       num_priors, neg_pos, sums, counts, sel, ws, ws_bytes, stream);
}

extern "C" int jabd_multibox_diou_loss_fwd_f32(const float* loc, const float* conf,
                                               const float* landm, const float* loc_t,
                                               const int64_t* conf_t, const float* landm_t,
                                               const float* priors, float var0, float var1,
                                               int64_t batch, int64_t num_priors, int neg_pos,
                                               float* sums, int64_t* counts, uint8_t* sel,
                                               void* ws, size_t ws_bytes,
                                               jabd_stream_t stream) {
  JABD_REQUIRE(priors, "multibox_diou: null priors");
  return loss_fwd_impl(loc, conf, landm, loc_t, conf_t, landm_t, priors, var0, var1, batch,
                       num_priors, neg_pos, sums, counts, sel, ws, ws_bytes, stream);
}

extern "C" int jabd_multibox_loss_finalize_f32(const float* sums, const int64_t* counts,
                                               float* loss, jabd_stream_t stream) {
  JABD_REQUIRE(sums && counts && loss, "multibox_finalize: null pointer");
  loss_normalize_kernel<<<1, 64, 0, as_stream(stream)>>>(sums, counts, loss);
  return check_launch("loss_finalize");
}

extern "C" int jabd_multibox_loss_bwd_f32(const float* loc, const float* conf,
                                          const float* landm, const float* loc_t,
                                          const int64_t* conf_t, const float* landm_t,
                                          const uint8_t* sel, int64_t batch,
                                          int64_t num_priors, const float* gout,
                                          const int64_t* counts, float* grad_loc,
                                          float* grad_conf, float* grad_landm,
                                          jabd_stream_t stream) {
  const int64_t total = batch * num_priors;
  if (total <= 0) return JABD_OK;
  JABD_REQUIRE(sel && gout && counts, "multibox_bwd: null pointer");
  loss_bwd_kernel<false><<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      loc, conf, landm, loc_t, conf_t, landm_t, nullptr, num_priors, 0.f, 0.f, sel, total, gout,
      counts, grad_loc, grad_conf, grad_landm);
  return check_launch("multibox_bwd");
}

extern "C" int jabd_multibox_diou_loss_bwd_f32(const float* loc, const float* conf,
                                               const float* landm, const float* loc_t,
                                               const int64_t* conf_t, const float* landm_t,
                                               const float* priors, float var0, float var1,
                                               const uint8_t* sel, int64_t batch,
                                               int64_t num_priors, const float* gout,
                                               const int64_t* counts, float* grad_loc,
                                               float* grad_conf, float* grad_landm,
                                               jabd_stream_t stream) {
  const int64_t total = batch * num_priors;
  if (total <= 0) return JABD_OK;
  JABD_REQUIRE(sel && gout && counts && priors, "multibox_diou_bwd: null pointer");
  loss_bwd_kernel<true><<<(unsigned)cdiv(total, 256), 256, 0, as_stream(stream)>>>(
      loc, conf, landm, loc_t, conf_t, landm_t, reinterpret_cast<const float4*>(priors),
      num_priors, var0, var1, sel, total, gout, counts, grad_loc, grad_conf, grad_landm);
  return check_launch("multibox_diou_bwd");
}
