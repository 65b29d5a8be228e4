// A10: batched greedy NMS on gfx950, bit-exact with torchvision's CPU
// nms kernel as called by utils/utils_bbox.py:275 (non_max_suppression).
//
// Pipeline per call (B images, up to n boxes each), all on one stream:
//   1. nms_keys      one 64-bit key per row: [image:8 | ~score:32 | row:24];
//                    rows failing the score filter get image 255 (sorted last).
//   2. radix sort    radix.hip's wavefront LSD sort of the keys by bits 24-63
//                    (stable; the input is in row order per image) — gives
//                    every image's rows contiguous, in stable descending-score
//                    order (ties by lower row index, as torch's stable sort).
//   3. nms_gather    sorted boxes (float4) + areas + original row ids.
//   4. mask          which later-ranked boxes each box suppresses, as the
//                    in-block word per row + a sparse list per row.  Two
//                    producers, chosen per image on the device:
//                    grid (candidate-pruned, thr >= 0, finite boxes): only
//                    pairs of similar area in neighbouring cells are tested
//                    (grid_* kernels below);  dense (NaN boxes, thr < 0, or
//                    more candidate pairs than the workspace holds): every
//                    pair in 64x64 tiles (nms_mask).
//   5. scan          grid images: nms_scan_pull, one wave per image pulls
//                    each row block's incoming pairs against the kept bitset
//                    in LDS (lists of the next blocks in flight); dense
//                    images: nms_scan (push of per-row lists).  Both write
//                    the kept rows + count.
// Compile with -ffp-contract=off: IoU must round exactly like the CPU kernel
// (no FMA in (x2-x1)*(y2-y1) or inter/(a+b-inter)).
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "common.h"
#include "nms_internal.h"
#include "radix.h"

namespace jabd {

static constexpr int kImgBits = 8;
static constexpr int kRowBits = 24;
static constexpr int64_t kMaxRows = (int64_t(1) << kRowBits);
static constexpr int kMaxImg = 254;  // 255 marks a filtered-out row

// JABD_NMS_DENSE=1 disables the grid producer (A/B tests and measurement).
static bool nms_dense_only() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("JABD_NMS_DENSE");
    v = e && e[0] == '1' ? 1 : 0;
  }
  return v == 1;
}

// Images with at most this many candidates take the dense all-pairs mask even
// on the grid path: a few hundred clustered boxes (bs1 predict) gave the grid
// producer's per-box candidate walks 340 us of serial latency against ~10 us
// for the parallel 64x64-block mask (MNv3 640^2 predict 606 -> 767 fps);
// R50's 6.8k / 17k candidates measured equal either way.
// JABD_NMS_DENSE_MAX=<n> for A/B (0 = grid whenever possible).
// Images of at most this many rows take the dense producer without the grid
// producer's launches (its key sort, tables and pair pass are ~35 kernels of
// fixed cost: at bs1 640^2, 16.8k rows, they cost more than the all-pairs
// mask they could save).  JABD_NMS_DENSE_ROWS=<n> for A/B (0 = grid whenever
// possible).
static int64_t nms_dense_rows() {
  static const int64_t v = [] {
    const char* e = getenv("JABD_NMS_DENSE_ROWS");
    return e ? (int64_t)atoll(e) : (int64_t)20480;
  }();
  return v;
}

static int nms_dense_max() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("JABD_NMS_DENSE_MAX");
    v = e ? atoi(e) : 8192;
  }
  return v;
}

// Images per sort pass: <= 254 and the sort size must fit the sort's int32.
static int64_t images_per_pass(int64_t batch, int64_t n) {
  int64_t c = batch < kMaxImg ? batch : kMaxImg;
  if (n > 0 && c * n > (int64_t)0x7fffffff) c = (int64_t)0x7fffffff / n;
  return c < 1 ? 1 : c;
}

__device__ __forceinline__ uint32_t score_key_desc(float s) {
  uint32_t f = __float_as_uint(s);
  if (s != s) f = 0x7fc00000u;    // canonical NaN: sorts before everything
  if (f == 0x80000000u) f = 0u;   // -0.0 == +0.0 for the comparison sort
  uint32_t u = (f & 0x80000000u) ? ~f : (f | 0x80000000u);  // ascending order
  return ~u;                                                 // descending
}

__global__ __launch_bounds__(256) void nms_keys(const float* __restrict__ scores,
                                                int64_t score_stride, int64_t score_bstride,
                                                const int64_t* __restrict__ n_valid, int64_t n,
                                                int batch, float thr, int filter, int img0,
                                                uint64_t* __restrict__ keys,
                                                int* __restrict__ counts) {
  __shared__ int wg_count;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (threadIdx.x == 0) wg_count = 0;
  __syncthreads();
  bool valid = false;
  if (i < n && b < batch) {
    const float s = scores[(int64_t)(b + img0) * score_bstride + i * score_stride];
    const int64_t nv = n_valid ? n_valid[b + img0] : n;
    valid = i < nv;
    if (filter) valid = valid && (s >= thr);
    const uint64_t img = valid ? (uint64_t)b : 255u;
    keys[(int64_t)b * n + i] =
        (img << 56) | ((uint64_t)score_key_desc(s) << kRowBits) | (uint64_t)i;
  }
  // one LDS atomic per wave, one global atomic per workgroup (all the
  // workgroups of an image add into one counter)
  const uint64_t m = __ballot(valid);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(&wg_count, __popcll(m));
  __syncthreads();
  if (threadIdx.x == 0 && wg_count) atomicAdd(&counts[b], wg_count);
}

// Single-image form (bs1 predict): one workgroup walks the rows in order and
// writes only the candidates' keys, compacted in row order (wave ballot
// prefix + LDS wave totals per round), and their count — so the key sort
// (radix_sort64_devn) orders the candidates alone (400 of MNv3's 16.8k
// anchors at 640^2) and the same stable order results.
constexpr int kCompactT = 1024;
__global__ __launch_bounds__(kCompactT) void nms_keys_compact(
    const float* __restrict__ scores, int64_t score_stride, const int64_t* __restrict__ n_valid,
    int64_t n, float thr, int filter, int img0, uint64_t* __restrict__ keys,
    int* __restrict__ counts) {
  __shared__ int wtot[kCompactT / 64];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int64_t nv = n_valid ? n_valid[img0] : n;
  const float* sc = scores;
  int base = 0;
  for (int64_t i0 = 0; i0 < n; i0 += kCompactT) {
    const int64_t i = i0 + t;
    bool valid = false;
    float s = 0.f;
    if (i < n) {
      s = sc[i * score_stride];
      valid = i < nv && (!filter || s >= thr);
    }
    const uint64_t m = __ballot(valid);
    if (l == 0) wtot[w] = __popcll(m);
    __syncthreads();
    int pre = 0, all = 0;
#pragma unroll
    for (int q = 0; q < kCompactT / 64; ++q) {
      const int c = wtot[q];
      pre += q < w ? c : 0;
      all += c;
    }
    if (valid)
      keys[base + pre + __popcll(m & ((1ull << l) - 1ull))] =
          ((uint64_t)score_key_desc(s) << kRowBits) | (uint64_t)i;
    base += all;
    __syncthreads();
  }
  if (t == 0) counts[0] = base;
}

__global__ void nms_gather(const uint64_t* __restrict__ sorted, int64_t total,
                           const float* __restrict__ boxes, int64_t box_stride,
                           int64_t box_bstride, const int* __restrict__ counts,
                           int batch, int64_t n, int img0, float4* __restrict__ sbox,
                           float* __restrict__ sarea, int* __restrict__ sidx,
                           int* __restrict__ nanflag) {
  int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= total) return;
  uint64_t k = sorted[p];
  int img = (int)(k >> 56);
  if (img >= batch) return;
  int64_t start = 0;
  for (int b = 0; b < img; ++b) start += counts[b];
  int64_t r = p - start;
  int row = (int)(k & ((1u << kRowBits) - 1));
  const float* bx = boxes + (int64_t)(img + img0) * box_bstride + (int64_t)row * box_stride;
  float x1 = bx[0], y1 = bx[1], x2 = bx[2], y2 = bx[3];
  sbox[(int64_t)img * n + r] = make_float4(x1, y1, x2, y2);
  sarea[(int64_t)img * n + r] = (x2 - x1) * (y2 - y1);
  sidx[(int64_t)img * n + r] = row;
  if (x1 != x1 || y1 != y1 || x2 != x2 || y2 != y2) atomicOr(&nanflag[img], 1);
}

// Per-row sparse suppression lists.  Row i (sorted rank) of row block rb can
// suppress boxes in at most nb-rb-1 later column blocks; its non-zero 64-bit
// words are appended (any order: the scan ORs them) at
//   ent[ent_base(rb) + (i - 64 rb) * (nb - rb - 1) + slot],  slot < nzcnt[i],
// and its in-block word (column block rb, bits j > i) is diag[i].
__device__ __host__ __forceinline__ int64_t ent_base(int64_t rb, int64_t nb) {
  return 64 * (rb * (nb - 1) - rb * (rb - 1) / 2);
}

static constexpr int kColBlocksPerWave = 4;
static constexpr int kWaves = 4;
static constexpr int kColBlocksPerWG = kColBlocksPerWave * kWaves;

// IoU(i, j) > thr with torchvision's CPU rounding.  inter/union is only
// divided out when the pair is within 1e-4 of the threshold: far from it
// the comparison of inter with thr*union (fp32, margin >> 2 ulp) already
// decides the exact result.
__device__ __forceinline__ bool iou_gt(float ix1, float iy1, float ix2, float iy2,
                                       float iarea, float4 bj, float aj, double thr,
                                       float thrf, bool thr_nonneg) {
  float xx1 = (ix1 < bj.x) ? bj.x : ix1;  // std::max(ix1, x1[j])
  float yy1 = (iy1 < bj.y) ? bj.y : iy1;
  float xx2 = (bj.z < ix2) ? bj.z : ix2;  // std::min(ix2, x2[j])
  float yy2 = (bj.w < iy2) ? bj.w : iy2;
  float dw = xx2 - xx1, dh = yy2 - yy1;
  float w = (0.f < dw) ? dw : 0.f;        // std::max(0, xx2 - xx1)
  float h = (0.f < dh) ? dh : 0.f;
  float inter = w * h;
  float uni = iarea + aj - inter;
  if (thr_nonneg) {
    // inter == 0 (or NaN) gives ovr in {0, -0, NaN}: never > thr >= 0.
    if (!(inter > 0.f)) return false;
    if (uni > 1e-30f && uni < 3e38f) {
      const float tu = thrf * uni;
      if (inter < tu * 0.9999f) return false;
      if (inter > tu * 1.0001f) return true;
    }
  }
  float ovr = inter / uni;
  return (double)ovr > thr;
}

// Dense-image tiles (64 rows x kColBlocksPerWG column blocks) as a grid-
// stride loop over a fixed grid: with no dense image in the batch (the
// common case) every workgroup leaves after one look at dense[].
__global__ __launch_bounds__(256) void nms_mask(
    const float4* __restrict__ sbox, const float* __restrict__ sarea,
    const int* __restrict__ counts, int64_t n, int64_t nb, int bc, double thr,
    const int* __restrict__ nanflag, const int* __restrict__ dense, uint64_t* __restrict__ diag,
    int* __restrict__ nzcnt, int* __restrict__ ent_cb, uint64_t* __restrict__ ent_bits) {
  __shared__ int any_dense;
  if (threadIdx.x == 0) {
    int a = 0;
    for (int q = 0; q < bc; ++q) a |= dense[q];
    any_dense = a;
  }
  __syncthreads();
  if (!any_dense) return;
  __shared__ float4 cbox[kColBlocksPerWG * 64];
  __shared__ float carea[kColBlocksPerWG * 64];
  const int64_t ncbg = (nb + kColBlocksPerWG - 1) / kColBlocksPerWG;
  const int64_t ntiles = ncbg * nb * bc;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int b = (int)(tile / (ncbg * nb));
  const int64_t rb = (tile / ncbg) % nb;
  const int64_t cbg = (tile % ncbg) * kColBlocksPerWG;
  if (!dense[b]) continue;  // this image's mask came from the grid path
  const int cnt = counts[b];
  const int64_t nbv = (cnt + 63) / 64;
  if (rb >= nbv || cbg + kColBlocksPerWG <= rb || cbg >= nbv) continue;

  const float4* ib = sbox + (int64_t)b * n;
  const float* ia = sarea + (int64_t)b * n;
  for (int t = threadIdx.x; t < kColBlocksPerWG * 64; t += blockDim.x) {
    int64_t j = cbg * 64 + t;
    if (j < cnt) {
      cbox[t] = ib[j];
      carea[t] = ia[j];
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t row = rb * 64 + lane;
  const bool row_ok = row < cnt;
  float4 bi = row_ok ? ib[row] : make_float4(0.f, 0.f, 0.f, 0.f);
  float ai = row_ok ? ia[row] : 0.f;
  const bool thr_nonneg = thr >= 0.0;
  const float thrf = (float)thr;
  const float thr_hi = thrf * 1.0001f, thr_lo = thrf * 0.9999f;
  const bool fast = thr_nonneg && nanflag[b] == 0;
  const int64_t rowcap = nb - rb - 1;
  const int64_t eoff = (int64_t)b * ent_base(nb, nb) + ent_base(rb, nb) + (int64_t)lane * rowcap;
  for (int q = 0; q < kColBlocksPerWave; ++q) {
    const int64_t cb = cbg + wave * kColBlocksPerWave + q;
    if (cb < rb || cb >= nbv) continue;
    const int lbase = (wave * kColBlocksPerWave + q) * 64;
    const int64_t j0 = cb * 64;
    int jmax = (int)min((int64_t)64, (int64_t)cnt - j0);
    int jstart = (cb == rb) ? lane + 1 : 0;  // strictly after row i on the diagonal
    uint64_t bits = 0;
    if (row_ok) {
      if (fast) {
        // Branch-free: fminf/fmaxf equal std::min/max on non-NaN boxes (NaN
        // images take the exact loop below); pairs within 1e-4 of the
        // threshold (or with an out-of-range union) are resolved exactly.
        uint64_t amb = 0;
#pragma unroll 16
        for (int jj = 0; jj < 64; ++jj) {
          const float4 bj = cbox[lbase + jj];
          const float aj = carea[lbase + jj];
          const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
          const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
          const float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
          const float inter = w * h;
          const float uni = ai + aj - inter;
          const bool pos = inter > 0.f;
          const bool oku = uni > 1e-30f && uni < 3e38f;
          const bool above = inter > thr_hi * uni;
          const bool below = inter < thr_lo * uni;
          const uint64_t bit = (uint64_t)1 << jj;
          bits |= (pos && oku && above) ? bit : 0ull;
          amb |= (pos && (!oku || (!above && !below))) ? bit : 0ull;
        }
        const uint64_t vmask = (jmax >= 64 ? ~0ull : ((1ull << jmax) - 1)) &
                               ~((jstart >= 64) ? ~0ull : ((1ull << jstart) - 1));
        bits &= vmask;
        amb &= vmask;
        while (amb) {  // rare: exact division near the threshold
          const int jj = __ffsll((unsigned long long)amb) - 1;
          amb &= amb - 1;
          if (iou_gt(bi.x, bi.y, bi.z, bi.w, ai, cbox[lbase + jj], carea[lbase + jj], thr, thrf,
                     thr_nonneg))
            bits |= (uint64_t)1 << jj;
        }
      } else {
        for (int jj = jstart; jj < jmax; ++jj) {
          if (iou_gt(bi.x, bi.y, bi.z, bi.w, ai, cbox[lbase + jj], carea[lbase + jj], thr, thrf,
                     thr_nonneg))
            bits |= (uint64_t)1 << jj;
        }
      }
      if (cb == rb) {
        diag[(int64_t)b * n + row] = bits;
      } else if (bits) {
        const int slot = atomicAdd(&nzcnt[(int64_t)b * n + row], 1);
        ent_cb[eoff + slot] = (int)cb;
        ent_bits[eoff + slot] = bits;
      }
    }
  }
  __syncthreads();  // cbox is refilled by the next tile
  }
}

// ---------------------------------------------------------------------------
// Grid (candidate-pruned) mask.  For thr >= 0 a pair can only have IoU > t
// if each axis has a 1-D IoU > t (IoU <= IoU_x, IoU_y), which needs
//   * widths within a factor t (IoU_x <= w_min / w_max), heights alike, and
//   * |dcx| < (w_i + w_j)(1 - t) / (2(1 + t)) <= f * max width, dcy alike
//     (f = (1 - t)/(1 + t); 1-D overlap <= (w_i + w_j)/2 - |dcx|).
// Boxes are binned by (log w, log h) classes of width W'/kK, W' >= 1.01 *
// -ln(t), so such pairs are at most kK classes apart per axis, and per class
// into cells of s_x = 1.05 f x the largest width of width classes c-kK..c+kK
// (s_y alike), so their centres are at most one cell apart.  Each box tests
// its own class (later ranks) and the "forward" half of its neighbour classes
// in its 3x3 cell neighbourhood — every unordered pair exactly once — with
// the same exact IoU comparison as the dense path.  Candidate boxes are read
// from a copy in key order (cell runs are contiguous).  Inactive boxes (x2 <= x1,
// y2 <= y1 or infinite area) can neither suppress nor be suppressed at
// t >= 0 and are not binned.  An image falls back to the dense producer
// (dense[b] != 0) if it has NaN boxes, a cell index beyond +-2^14, or more
// off-block pairs than the workspace holds.
// Key: image 8 | width class 10 | height class 10 | cell y 18 | cell x 18.
// ---------------------------------------------------------------------------
static constexpr int kNC = 1024;          // log-extent classes per axis
static constexpr int kClassOff = 512;
static constexpr int kCellOff = 1 << 17;  // 18-bit biased cell coordinates
static constexpr int kCellLim = 1 << 14;
static constexpr int64_t kPairsPerBox = 128;  // off-block pair capacity per box
static constexpr int kWaveRec = 64 * (int)kPairsPerBox;  // pair records per key-order wave
#ifndef JABD_NMS_CAND
#define JABD_NMS_CAND 4
#endif
static constexpr int kCand = JABD_NMS_CAND;              // candidate loads in flight per lane
static constexpr int kLaneRec = 64;                      // of which each lane's own slots
static constexpr int kWaveShared = kWaveRec - 64 * kLaneRec;  // and the wave's shared tail
// Past its wave's region a pair goes to its image's overflow region (one
// global atomic per record: only a cluster's waves get there), kOvfPerBox
// records per row; an image only falls back to the dense producer past that.
// (A few hundred mutually overlapping boxes of one face put ~n_c^2 / 2 pairs
// into the handful of key-order waves that hold their cell run.)
static constexpr int64_t kOvfPerBox = 16;
// JABD_NMS_OVF_PER_BOX overrides it (read on every carve, so a test can turn
// the overflow region off between calls; the size query and the call it
// sizes must see the same value)
static int64_t nms_ovf_per_box() {
  const char* e = getenv("JABD_NMS_OVF_PER_BOX");
  return e ? std::max<int64_t>(0, atoll(e)) : kOvfPerBox;
}
static constexpr int kK = 2;                  // class sub-division (neighbour range)
static constexpr int kGridNbr = 1 + kK + kK * (2 * kK + 1);  // class pairs searched per box

__device__ __forceinline__ bool grid_active(float4 bx, float a) {
  return bx.z > bx.x && bx.w > bx.y && a < INFINITY;
}

__device__ __forceinline__ int grid_class(float e, float inv_w) {
  float c = floorf(logf(e) * inv_w);
  c = fminf(fmaxf(c, (float)-kClassOff), (float)(kNC - 1 - kClassOff));
  return (int)c + kClassOff;
}

// largest extent of classes c-kK..c+kK (ext = one axis' per-class maxima) x f
__device__ __forceinline__ float grid_cell_size(const unsigned* ext, int c, float f) {
  float e = 0.f;
#pragma unroll
  for (int d = -kK; d <= kK; ++d)
    if (c + d >= 0 && c + d < kNC) e = fmaxf(e, __uint_as_float(ext[c + d]));
  return e * f;
}

__device__ __forceinline__ uint64_t grid_key(int b, int cw, int ch, int y, int x) {
  return ((uint64_t)b << 56) | ((uint64_t)cw << 46) | ((uint64_t)ch << 36) |
         ((uint64_t)(y + kCellOff) << 18) | (uint64_t)(x + kCellOff);
}

// ext[b][0][cw] = largest width of width class cw, ext[b][1][ch] = largest
// height; ext[b][2] / ext[b][3] = the smallest width / height, stored
// complemented (~bits) so one atomicMax over a zeroed array serves both.
// The classes one image occupies are few (tens), so per-box global atomics
// would serialise on a handful of L2 addresses: each workgroup takes kExtPer
// boxes per thread into LDS extremes first and flushes the classes it
// touched with one global atomic each.
static constexpr int kExtPer = 16;
__global__ __launch_bounds__(256) void grid_ext(const float4* __restrict__ sbox,
                                                const float* __restrict__ sarea,
                                                const int* __restrict__ counts,
                                                const int* __restrict__ nanflag, int64_t n,
                                                float inv_w, unsigned* __restrict__ ext,
                                                int* __restrict__ dense, int dense_max) {
  __shared__ unsigned le[4 * kNC];
  const int t = threadIdx.x;
  const int b = blockIdx.y;
  for (int i = t; i < 4 * kNC; i += 256) le[i] = 0u;
  // NaN boxes (1), or few enough candidates that the all-pairs mask is cheaper
  // than the grid's per-box serial candidate walks (8)
  if (blockIdx.x == 0 && t == 0 && (nanflag[b] || (dense_max > 0 && counts[b] <= dense_max)))
    atomicOr(&dense[b], nanflag[b] ? 1 : 8);
  __syncthreads();
  const int cnt = counts[b];
  const int64_t base = (int64_t)blockIdx.x * 256 * kExtPer;
  for (int k = 0; k < kExtPer; ++k) {
    const int64_t r = base + (int64_t)k * 256 + t;
    if (r >= cnt) break;
    const float4 bx = sbox[(int64_t)b * n + r];
    const float a = sarea[(int64_t)b * n + r];
    if (!grid_active(bx, a)) continue;
    const float w = bx.z - bx.x, h = bx.w - bx.y;
    const int cw = grid_class(w, inv_w), ch = grid_class(h, inv_w);
    atomicMax(&le[cw], __float_as_uint(w));
    atomicMax(&le[kNC + ch], __float_as_uint(h));
    atomicMax(&le[2 * kNC + cw], ~__float_as_uint(w));
    atomicMax(&le[3 * kNC + ch], ~__float_as_uint(h));
  }
  __syncthreads();
  for (int i = t; i < 4 * kNC; i += 256)
    if (le[i]) atomicMax(&ext[(int64_t)b * 4 * kNC + i], le[i]);
}

__global__ void grid_keys(const float4* __restrict__ sbox, const float* __restrict__ sarea,
                          const int* __restrict__ counts, int64_t n, float inv_w, float fcell,
                          const unsigned* __restrict__ ext, uint64_t* __restrict__ key,
                          int* __restrict__ val, int* __restrict__ dense) {
  const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (r >= n) return;
  const int64_t o = (int64_t)b * n + r;
  uint64_t k = ~0ull;
  if (r < counts[b] && !(dense[b] & 1)) {
    const float4 bx = sbox[o];
    const float a = sarea[o];
    if (grid_active(bx, a)) {
      const int cw = grid_class(bx.z - bx.x, inv_w), ch = grid_class(bx.w - bx.y, inv_w);
      const unsigned* e = ext + (int64_t)b * 4 * kNC;
      const float sx = grid_cell_size(e, cw, fcell), sy = grid_cell_size(e + kNC, ch, fcell);
      const float fx = floorf((bx.x + bx.z) * 0.5f / sx), fy = floorf((bx.y + bx.w) * 0.5f / sy);
      if (fabsf(fx) < (float)kCellLim && fabsf(fy) < (float)kCellLim) {
        k = grid_key(b, cw, ch, (int)fy, (int)fx);
      } else {
        atomicOr(&dense[b], 2);
      }
    }
  }
  key[o] = k;
  val[o] = (int)r;
}

// candidate data in key order: gbox[q] = sbox[rank sval[q]] (areas are
// recomputed from the box where needed: nms_gather's expression)
__global__ void grid_gather(const uint64_t* __restrict__ skey, const int* __restrict__ sval,
                            int64_t total, const float4* __restrict__ sbox, int64_t n,
                            float4* __restrict__ gbox) {
  const int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (q >= total) return;
  const uint64_t k = skey[q];
  if (k == ~0ull) return;
  gbox[q] = sbox[(int64_t)(k >> 56) * n + sval[q]];
}

// Cell runs: after the sort, the boxes of one (image, classes, cell) key are
// a contiguous run [lo, hi) of the key order.  An open-addressing table maps
// each run's key to its bounds, so a box finds a neighbour cell with one or
// two 16-byte loads instead of a binary search over the image's keys.
struct CellRun {
  unsigned long long key;  // ~0: empty slot
  int lo, hi;
};
static constexpr unsigned long long kEmptyKey = ~0ull;

__device__ __forceinline__ uint32_t run_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return (uint32_t)k;
}

__global__ void grid_runs_insert(const uint64_t* __restrict__ skey, int64_t total,
                                 CellRun* __restrict__ tab, uint32_t mask, int bc,
                                 int* __restrict__ istart) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= total) return;
  const uint64_t k = skey[p];
  // istart[x] = key position of image x's first candidate (inactive keys ~0
  // sort last and count as image bc; istart[bc] = the number of active keys)
  {
    const int cur = k == kEmptyKey ? bc : (int)(k >> 56);
    const int prv = p == 0 ? -1 : (skey[p - 1] == kEmptyKey ? bc : (int)(skey[p - 1] >> 56));
    for (int x = prv + 1; x <= cur; ++x) istart[x] = (int)p;
    if (p == total - 1)
      for (int x = cur + 1; x <= bc; ++x) istart[x] = (int)total;
  }
  if (k == kEmptyKey || (p > 0 && skey[p - 1] == k)) return;  // not a run start
  tab += (k >> 56) * ((int64_t)mask + 1);  // this image's table
  uint32_t h = run_hash(k) & mask;
  for (;;) {
    const unsigned long long prev = atomicCAS(&tab[h].key, kEmptyKey, (unsigned long long)k);
    if (prev == kEmptyKey || prev == k) {
      tab[h].lo = (int)p;
      return;
    }
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ int run_find(const CellRun* __restrict__ tab, uint32_t mask, uint64_t k,
                                        int& lo) {
  uint32_t h = run_hash(k) & mask;
  for (;;) {
    const uint4 e = *reinterpret_cast<const uint4*>(&tab[h]);
    const uint64_t kk = ((uint64_t)e.y << 32) | e.x;
    if (kk == k) {
      lo = (int)e.z;
      return (int)e.w;
    }
    if (kk == kEmptyKey) return -1;
    h = (h + 1) & mask;
  }
}

__global__ void grid_runs_end(const uint64_t* __restrict__ skey, int64_t total,
                              CellRun* __restrict__ tab, uint32_t mask) {
  const int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (p >= total) return;
  const uint64_t k = skey[p];
  if (k == kEmptyKey || (p + 1 < total && skey[p + 1] == k)) return;  // not a run end
  tab += (k >> 56) * ((int64_t)mask + 1);
  uint32_t h = run_hash(k) & mask;
  while (tab[h].key != k) h = (h + 1) & mask;
  tab[h].hi = (int)(p + 1);
}

__global__ __launch_bounds__(256) void grid_pairs(
    const uint64_t* __restrict__ skey, const int* __restrict__ sval, int64_t total,
    const float4* __restrict__ gbox, int64_t n, int bc,
    float inv_w, float fcell, const unsigned* __restrict__ ext,
    const CellRun* __restrict__ tab, uint32_t tmask,
    double thr, int* __restrict__ dense, uint64_t* __restrict__ diag,
    uint64_t* __restrict__ rec, int* __restrict__ lcnt, int* __restrict__ wcnt,
    uint64_t* __restrict__ ovf, int* __restrict__ ocnt, int64_t ovcap,
    unsigned long long* __restrict__ tested) {
  // XCD-aware block order: hardware block id g runs on XCD g % 8; give each
  // XCD one contiguous eighth of the key order (= one image when the batch
  // holds 8), so an image's candidate arrays stay in one XCD's L2
  // (host: gridDim.x is a multiple of 8, so the map is a permutation)
  __shared__ int s_wcnt[4];
  const int64_t g = blockIdx.x, per = gridDim.x / 8;
  const int64_t lb = (g % 8) * per + g / 8;
  const int64_t p = lb * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // this wave's private pair region (key-order wave index p / 64): no global
  // counter, so a flush is a wave-local LDS reservation and plain stores
  const int64_t wglob = lb * 4 + wv;
  uint64_t* wrec = rec + wglob * kWaveRec;
  if (lane == 0) s_wcnt[wv] = 0;
  const uint64_t k = p < total ? skey[p] : ~0ull;
  const int b = k != ~0ull ? (int)(k >> 56) : 0;
  int nl = 0;  // records in this lane's own slots
  if (k != ~0ull && !(dense[b] & 11)) {
  const int i = sval[p];
  const float4 bi = gbox[p];
  const float ai = (bi.z - bi.x) * (bi.w - bi.y);  // nms_gather's area expression (exact)
  const int cw = (int)((k >> 46) & (kNC - 1)), ch = (int)((k >> 36) & (kNC - 1));
  const unsigned* ew = ext + (int64_t)b * 4 * kNC;
  const unsigned* eh = ew + kNC;
  const unsigned* ewn = ew + 2 * kNC;  // complemented minima
  const unsigned* ehn = ew + 3 * kNC;
  const float wi = bi.z - bi.x, hi_ = bi.w - bi.y;
  // IoU <= min(w_i, w_j) / max(w_i, w_j) (heights alike): a class whose
  // extents cannot reach a ratio above thr holds no partner (1% margin)
  const bool ratio = thr > 0.0;
  const float rlo = (float)thr * 0.99f, rhi = ratio ? 1.01f / (float)thr : 0.f;
  const float cx = (bi.x + bi.z) * 0.5f, cy = (bi.y + bi.w) * 0.5f;
  const float thrf = (float)thr;
  const uint32_t bkt0 = (uint32_t)(b * ((n + 63) >> 6));  // this image's first row block
  tab += (int64_t)b * ((int64_t)tmask + 1);  // this image's run table (resident in its XCD's L2)

  // Off-block pairs go straight to this lane's kLaneRec slots of the wave's
  // region (no reservation); a lane past them takes slots of the wave's
  // shared tail by an LDS atomic.  Records are (destination block << 32) |
  // (row << 6 | col & 63); one beyond the region sends its image to the dense
  // producer.
  uint64_t* lrec = wrec + lane;  // slot q of this lane: lrec[64 q]
  // own class, then the forward half of the neighbour classes:
  // (0, 1..kK) and (1..kK, -kK..kK)
  unsigned ntest = 0;
  bool full = false;  // the image's pair capacity is exhausted (it falls back to dense)
  for (int nbr = 0; nbr < kGridNbr && !full; ++nbr) {
    int cw2, ch2;
    if (nbr <= kK) {
      cw2 = cw;
      ch2 = ch + nbr;
    } else {
      const int q2 = nbr - kK - 1;
      cw2 = cw + 1 + q2 / (2 * kK + 1);
      ch2 = ch - kK + q2 % (2 * kK + 1);
    }
    if (cw2 >= kNC || ch2 < 0 || ch2 >= kNC || ew[cw2] == 0u || eh[ch2] == 0u) continue;
    const float wmax2 = __uint_as_float(ew[cw2]), hmax2 = __uint_as_float(eh[ch2]);
    if (ratio && (wmax2 < wi * rlo || __uint_as_float(~ewn[cw2]) > wi * rhi ||
                  hmax2 < hi_ * rlo || __uint_as_float(~ehn[ch2]) > hi_ * rhi))
      continue;
    // a partner j of this class has |dcx| < f (w_i + w_j) / 2 <= f (w_i + wmax2) / 2
    // (fcell = 1.05 f: rounding margin), and its cell is floor(cx_j / sx)
    // with the cell size sx its own key was built with (<= 3 cells per axis)
    const float sx = grid_cell_size(ew, cw2, fcell), sy = grid_cell_size(eh, ch2, fcell);
    const float rx = 0.5f * fcell * (wi + wmax2), ry = 0.5f * fcell * (hi_ + hmax2);
    const float lim = (float)(kCellLim + 1);
    const int X0 = (int)fmaxf(floorf((cx - rx) / sx), -lim), X1 = (int)fminf(floorf((cx + rx) / sx), lim);
    const int Y0 = (int)fmaxf(floorf((cy - ry) / sy), -lim), Y1 = (int)fminf(floorf((cy + ry) / sy), lim);
    for (int Y = Y0; Y <= Y1 && !full; ++Y) {
      // a row of up to three cells at once: their table probes are in flight
      // together, and their runs are walked as one candidate sequence
      for (int Xb = X0; Xb <= X1; Xb += 3) {
        uint4 e3[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const uint32_t h = run_hash(grid_key(b, cw2, ch2, Y, Xb + c)) & tmask;
          e3[c] = Xb + c <= X1 ? *reinterpret_cast<const uint4*>(&tab[h])
                               : make_uint4(~0u, ~0u, 0u, 0u);
        }
        int lo3[3], n3[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const uint64_t key = grid_key(b, cw2, ch2, Y, Xb + c);
          const uint64_t kk = ((uint64_t)e3[c].y << 32) | e3[c].x;
          lo3[c] = (int)e3[c].z;
          n3[c] = kk == key ? (int)(e3[c].w - e3[c].z) : 0;
          if (kk != key && kk != kEmptyKey) {  // first slot taken by another run: probe on
            int lo = 0;
            const int hi = run_find(tab, tmask, key, lo);
            lo3[c] = lo;
            n3[c] = hi >= 0 ? hi - lo : 0;
          }
        }
        const int qe = n3[0] + n3[1] + n3[2];
        // candidates kCand at a time: their loads are in flight together (the
        // area is recomputed from the box: nms_gather's expression, exact)
        for (int q = 0; q < qe && !full; q += kCand) {
          int jj[kCand];
          float4 bb[kCand];
#pragma unroll
          for (int u = 0; u < kCand; ++u) {
            const int t = q + u < qe ? q + u : q;
            const int qq = t < n3[0] ? lo3[0] + t
                                     : (t < n3[0] + n3[1] ? lo3[1] + (t - n3[0])
                                                          : lo3[2] + (t - n3[0] - n3[1]));
            jj[u] = sval[qq];
            bb[u] = gbox[qq];
          }
#pragma unroll
          for (int u = 0; u < kCand; ++u) {
            const int j = jj[u];
            const float aa_u = (bb[u].z - bb[u].x) * (bb[u].w - bb[u].y);
            // same class: each pair once, from the lower rank
            bool hit = q + u < qe && !(nbr == 0 && j <= i);
            ntest += hit;
#ifdef JABD_NMS_AB_NOIOU  // A/B timing build: the walk and loads alone (results wrong)
            hit = hit && __float_as_uint(bb[u].x) == 0x7fc00001u && aa_u == 1.f;
#else
            if (hit) hit = iou_gt(bi.x, bi.y, bi.z, bi.w, ai, bb[u], aa_u, thr, thrf, true);
#endif
#ifdef JABD_NMS_AB_NOSTORE  // A/B timing build: tests kept, pair output dropped
            ntest += hit ? 65536u : 0u;
            hit = false;
#endif
            if (hit) {
              const int row = i < j ? i : j, col = i < j ? j : i;
              if ((row >> 6) == (col >> 6)) {
                atomicOr((unsigned long long*)&diag[(int64_t)b * n + row],
                         (unsigned long long)1 << (col & 63));
              } else {
                const uint64_t rv = ((uint64_t)(bkt0 + (uint32_t)(col >> 6)) << 32) |
                                    (uint32_t)((row << 6) | (col & 63));
                if (nl < kLaneRec) {
                  lrec[64 * nl++] = rv;
                } else {
                  const int sl = atomicAdd(&s_wcnt[wv], 1);
                  if (sl < kWaveShared) {
                    wrec[64 * kLaneRec + sl] = rv;
                  } else {
                    const int64_t so = atomicAdd(&ocnt[b], 1);
                    if (so < ovcap) {
                      ovf[(int64_t)b * ovcap + so] = rv;
                    } else {
                      // the image goes dense: this lane's walk ends here
                      atomicOr(&dense[b], 4);
                      full = true;
                    }
                  }
                }
              }
            }
          }
        }
      }
    }
  }
  // per-lane counter slots (64 per image): a single address per image would
  // serialise ~100k L2 atomics
  if (ntest) atomicAdd(&tested[(int64_t)b * 64 + lane], (unsigned long long)ntest);
  }
  lcnt[wglob * 64 + lane] = nl;
  if (lane == 0)
    wcnt[wglob] = min(__hip_atomic_load(&s_wcnt[wv], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP),
                      kWaveShared);
}

// Pair records -> incoming lists per destination row block (a counting sort
// by block).  Image b's key-order waves [istart[b] / 64, ceil(istart[b+1] /
// 64)) are split into K chunks, one workgroup each; a wave spanning two images
// is read by both and each keeps its own records.  Count: per-chunk block
// histograms in LDS, written as hist[(b nb + block) K + chunk]; an exclusive
// scan of that table gives every (block, chunk) its CSR range; scatter: the
// chunk re-reads its records and places each at its range's start + an LDS
// counter.  Block c's incoming pairs are csr[off[(b nb + c) K], off[(b nb + c
// + 1) K]) as (row << 6) | (col & 63), in no particular order (the scan ORs
// them).  No global atomics: the old per-pair row-slot reservation cost the
// pair search a device atomic round trip per flush.
__device__ __forceinline__ void grid_chunk_waves(const int* istart, int b, int K, int k,
                                                 int64_t& wa, int64_t& wb) {
  const int64_t p0 = istart[b], p1 = istart[b + 1];
  const int64_t w0 = p0 >> 6, w1 = p1 > p0 ? (p1 + 63) >> 6 : w0;
  wa = w0 + (w1 - w0) * k / K;
  wb = w0 + (w1 - w0) * (k + 1) / K;
}

// Every record of key-order waves [wa, wb) (each lane's own slots, then the
// wave's shared tail), waves spread over the workgroup's nwv waves.
// Every record of key-order waves [wa, wb) (the lanes' own slots, interleaved
// slot-major so each slot row is one coalesced load, then the wave's shared
// tail), waves spread over the workgroup's nwv waves.
template <typename F>
__device__ __forceinline__ void grid_chunk_records(const uint64_t* __restrict__ rec,
                                                   const int* __restrict__ lcnt,
                                                   const int* __restrict__ wcnt, int64_t wa,
                                                   int64_t wb, int lane, int wv, int nwv, F&& f) {
  for (int64_t w = wa + wv; w < wb; w += nwv) {
    const uint64_t* r = rec + w * kWaveRec;
    const int ml = lcnt[w * 64 + lane];
    const int ms = wcnt[w];
    int mx = ml;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
    for (int q = 0; q < mx; q += 8) {
      uint64_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = q + u < ml ? r[(q + u) * 64 + lane] : 0ull;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (q + u < ml) f(v[u]);
    }
    const uint64_t* sr = r + 64 * kLaneRec;
    for (int q = lane; q < ms; q += 64) f(sr[q]);
  }
}

// Image b's overflow records (grid_pairs past a wave's region), split over
// its K chunks by index: count and scatter see the same partition.
template <typename F>
__device__ __forceinline__ void grid_chunk_overflow(const uint64_t* __restrict__ ovf,
                                                    const int* __restrict__ ocnt, int64_t ovcap,
                                                    int b, int K, int k, int t, int nt, F&& f) {
  const int64_t m = min((int64_t)ocnt[b], ovcap);
  const uint64_t* ob = ovf + (int64_t)b * ovcap;
  for (int64_t q = m * k / K + t; q < m * (k + 1) / K; q += nt) f(ob[q]);
}

static constexpr int kBucketT = 1024;

__global__ __launch_bounds__(kBucketT) void grid_bucket_count(
    const uint64_t* __restrict__ rec, const int* __restrict__ lcnt, const int* __restrict__ wcnt,
    const uint64_t* __restrict__ ovf, const int* __restrict__ ocnt, int64_t ovcap,
    const int* __restrict__ istart, const int* __restrict__ dense, int64_t nb, int K,
    int* __restrict__ hist, int* __restrict__ npairs) {
  extern __shared__ int h[];
  __shared__ int s_tot;
  // image fastest in the block id: with 8 images, image b's chunks all run on
  // XCD b, whose L2 holds the records grid_pairs wrote for it
  const int bc = gridDim.x / K;
  const int b = blockIdx.x % bc, k = blockIdx.x / bc, t = threadIdx.x;
  for (int64_t i = t; i < nb; i += kBucketT) h[i] = 0;
  if (t == 0) s_tot = 0;
  __syncthreads();
  int mine = 0;
  if (!dense[b]) {
    int64_t wa, wb;
    grid_chunk_waves(istart, b, K, k, wa, wb);
    const uint32_t lo = (uint32_t)(b * nb), hi = (uint32_t)(lo + nb);
    auto count = [&](uint64_t v) {
      const uint32_t bk = (uint32_t)(v >> 32);
      if (bk >= lo && bk < hi) {
        atomicAdd(&h[bk - lo], 1);
        ++mine;
      }
    };
    grid_chunk_records(rec, lcnt, wcnt, wa, wb, t & 63, t >> 6, kBucketT / 64, count);
    grid_chunk_overflow(ovf, ocnt, ovcap, b, K, k, t, kBucketT, count);
  }
  if (mine) atomicAdd(&s_tot, mine);
  __syncthreads();
  int* hb = hist + (int64_t)b * nb * K;
  for (int64_t i = t; i < nb; i += kBucketT) hb[i * K + k] = h[i];
  if (t == 0 && s_tot) atomicAdd(&npairs[b], s_tot);
}

__global__ __launch_bounds__(kBucketT) void grid_bucket_scatter(
    const uint64_t* __restrict__ rec, const int* __restrict__ lcnt, const int* __restrict__ wcnt,
    const uint64_t* __restrict__ ovf, const int* __restrict__ ocnt, int64_t ovcap,
    const int* __restrict__ istart, const int* __restrict__ dense, int64_t nb, int K,
    const int* __restrict__ off, uint32_t* __restrict__ csr) {
  extern __shared__ int h[];
  const int bc = gridDim.x / K;
  const int b = blockIdx.x % bc, k = blockIdx.x / bc, t = threadIdx.x;  // as grid_bucket_count
  if (dense[b]) return;  // workgroup-uniform
  const int* ob = off + (int64_t)b * nb * K;
  for (int64_t i = t; i < nb; i += kBucketT) h[i] = ob[i * K + k];
  __syncthreads();
  int64_t wa, wb;
  grid_chunk_waves(istart, b, K, k, wa, wb);
  const uint32_t lo = (uint32_t)(b * nb), hi = (uint32_t)(lo + nb);
  auto place = [&](uint64_t v) {
    const uint32_t bk = (uint32_t)(v >> 32);
    if (bk >= lo && bk < hi) csr[atomicAdd(&h[bk - lo], 1)] = (uint32_t)v;
  };
  grid_chunk_records(rec, lcnt, wcnt, wa, wb, t & 63, t >> 6, kBucketT / 64, place);
  grid_chunk_overflow(ovf, ocnt, ovcap, b, K, k, t, kBucketT, place);
}

// ---------------------------------------------------------------------------
// Greedy scan of a grid image as a pull over row blocks.  Block c's kept rows
// are the valid rows not removed by (a) a kept row of an earlier block with a
// pair into it — block c's incoming list, looked up in the kept bitset of the
// earlier blocks — nor (b) an earlier kept row of the same block (diag words,
// resolved in rank order).  Nothing a block reads from HBM depends on the
// scan state, so it can be staged ahead of the scan:
//   * one workgroup per image: wave 0 scans, waves 1..15 are loaders, each
//     staging every 15th row block (diag words, original row ids, incoming
//     pairs) into LDS rings and publishing it with a ready flag;
//   * the scan wave never touches HBM except for its output stores: per block
//     it waits for the flag (LDS), looks the pairs up in the kept bitset (LDS),
//     ORs the removed bits across the wave (DPP), resolves the block and
//     publishes how far it got, which frees ring space for the loaders.
// The incoming pairs of consecutive blocks are consecutive in the CSR, so
// the pair ring is indexed by CSR position modulo its size; a block whose
// list alone exceeds the ring is read by the scan wave from HBM instead.
// Every wait is bounded (kSpinMax): a broken hand-off ends the kernel with
// *err set instead of hanging the device.
// ---------------------------------------------------------------------------
static constexpr int kPullWaves = 16;     // one scan wave + loaders
#ifdef JABD_NMS_AB_SIMD0  // A/B: the scan wave alone on its SIMD (waves 4, 8, 12 idle)
static constexpr int kPullLoaders = 12;
__device__ __forceinline__ int loader_id(int wave) { return (wave & 3) ? wave - 1 - (wave >> 2) : -1; }
#else
static constexpr int kPullLoaders = 15;
__device__ __forceinline__ int loader_id(int wave) { return wave - 1; }
#endif
static constexpr int kMetaRing = 32;        // row blocks staged ahead
static constexpr int kEntRing = 16384;      // incoming pairs staged ahead (power of two)
#ifndef JABD_NMS_LAG
#define JABD_NMS_LAG 8
#endif
static constexpr int kPullLag = JABD_NMS_LAG;         // a loader resolves block c once c - kPullLag are final
static constexpr unsigned kSpinMax = 1u << 22;
static constexpr int kPullStaticLds = kEntRing * 4 + kMetaRing * 64 * 16 + kMetaRing * 24 + 16;

__device__ __forceinline__ uint32_t wave_or32(uint32_t v) {
  // inclusive OR-scan inside each 16-lane row, then across rows (gfx9 DPP)
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v |= __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ int lds_acquire(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(int* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's data writes have landed
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ uint64_t lds_acquire64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release64(uint64_t* p, uint64_t v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int prog_done(uint64_t v) { return (int)(uint32_t)v; }
__device__ __forceinline__ int prog_end(uint64_t v) { return (int)(v >> 32); }

__global__ __launch_bounds__(64 * kPullWaves) void nms_scan_pull(
    const uint64_t* __restrict__ diag, const int* __restrict__ dense,
    const int* __restrict__ boff, int K, const uint32_t* __restrict__ csr, const int* __restrict__ sidx,
    const int* __restrict__ counts, int64_t n, int img0, int64_t* __restrict__ keep,
    int64_t keep_bstride, int64_t* __restrict__ n_keep, int* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t ents[kEntRing];
  __shared__ uint64_t mdiag[kMetaRing][64];
  __shared__ int msid[kMetaRing][64];
  __shared__ uint32_t munres[kMetaRing][64];  // <= 64 unresolved pairs: the scan keeps them in registers
  __shared__ int mready[kMetaRing], me0[kMetaRing], mne[kMetaRing], mend[kMetaRing];
  __shared__ uint64_t mpre[kMetaRing];
  // scan progress, one 64-bit word: blocks done (low) | their pairs' ring end (high)
  __shared__ uint64_t s_prog;
  const int b = blockIdx.x;
  if (dense[b]) return;  // workgroup-uniform: the dense-list scan owns this image
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cnt = counts[b];
  const int nbv = (cnt + 63) >> 6;
  uint64_t* kb = reinterpret_cast<uint64_t*>(smem);  // kept bits per block
  const int64_t rb0 = (int64_t)b * n;
  if (tid < kMetaRing) mready[tid] = -1;
  if (tid == 0) {
    s_prog = 0;
  }
  __syncthreads();
  if (cnt == 0) {
    if (tid == 0) n_keep[b + img0] = 0;
    return;
  }
  const int* ob = boff + (int64_t)b * ((n + 63) >> 6) * K;  // block c's pairs: [ob[cK], ob[(c+1)K])
  const int E0 = ob[0];  // CSR position of this image's first pair

  if (wave > 0) {  // ------------------------------------------------ loaders
#ifdef JABD_NMS_TRACE
    uint64_t l_start = __builtin_readcyclecounter(), l_space = 0, l_load = 0, l_first = 0;
#endif
    const int lid = loader_id(wave);
    if (lid < 0) return;
    for (int c = lid; c < nbv; c += kPullLoaders) {
#ifdef JABD_NMS_TRACE
      const uint64_t tl0 = __builtin_readcyclecounter();
#endif
      const int slot = c % kMetaRing;
      const int e0 = ob[(int64_t)c * K];
      const int e1 = ob[(int64_t)(c + 1) * K];
      const int ne = e1 - e0;
      const bool fits = ne <= kEntRing;
      const int r = 64 * c + lane;
      const int rr = r < cnt ? r : 0;
      const uint64_t dg = r < cnt ? diag[rb0 + rr] : 0ull;
      const int sd = sidx[rb0 + rr];
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = lane + 64 * k;
        v[k] = (fits && q < ne) ? csr[e0 + q] : 0u;
      }
#ifdef JABD_NMS_TRACE
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint64_t tl1 = __builtin_readcyclecounter();
      l_load += tl1 - tl0;
#endif
      unsigned spin = 0;
      while (!(prog_done(lds_acquire64(&s_prog)) > c - kMetaRing &&
               (!fits || prog_end(lds_acquire64(&s_prog)) >= e1 - E0 - kEntRing))) {
        __builtin_amdgcn_s_sleep(2);
        if (++spin > kSpinMax) {
          if (lane == 0) atomicOr(err, 1);
          return;
        }
      }
#ifdef JABD_NMS_TRACE
      l_space += __builtin_readcyclecounter() - tl1;
#endif
      // phase A: the block's raw incoming pairs into the ring (a list larger
      // than the ring stays in HBM for the scan wave)
      if (fits) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int q = lane + 64 * k;
          if (q < ne) ents[(e0 - E0 + q) & (kEntRing - 1)] = v[k];
        }
        for (int q0 = 512; q0 < ne; q0 += 512) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int q = q0 + lane + 64 * k;
            v[k] = q < ne ? csr[e0 + q] : 0u;
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int q = q0 + lane + 64 * k;
            if (q < ne) ents[(e0 - E0 + q) & (kEntRing - 1)] = v[k];
          }
        }
      }
      // Resolution, in place over the block's ring range: pairs whose source
      // block is final (< D) are looked up in the kept bitset here; the rest
      // are compacted to the front of the range (and, the last time, also
      // into munres[] when they are at most 64).
      uint32_t plo = 0, phi = 0;
      auto resolve = [&](int nin, int D, bool last) -> int {
        int nu = 0;  // wave-uniform
        for (int q0 = 0; q0 < nin; q0 += 512) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int q = q0 + lane + 64 * k;
            v[k] = q < nin ? ents[(e0 - E0 + q) & (kEntRing - 1)] : 0u;
          }
          // every entry of this chunk is in registers before any compacted
          // write (which lands at a position <= the chunk's); the kept-word
          // lookups are all issued before the first compacted write
          uint64_t wk[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int sb = (int)(v[k] >> 12);
            wk[k] = kb[q0 + lane + 64 * k < nin && sb < D ? sb : 0];
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int q = q0 + lane + 64 * k;
            const bool ok = q < nin;
            const int sb = (int)(v[k] >> 12);  // source block
            const bool res = ok && sb < D;
            const bool hit = res && ((wk[k] >> ((v[k] >> 6) & 63)) & 1);
            const uint32_t bit = v[k] & 63;
            plo |= (hit && bit < 32) ? 1u << (bit & 31) : 0u;
            phi |= (hit && bit >= 32) ? 1u << (bit & 31) : 0u;
            const bool un = ok && !res;
            const uint64_t um = __ballot(un);
            if (un) {
              const int pos = nu + __popcll(um & ((1ull << lane) - 1));
              ents[(e0 - E0 + pos) & (kEntRing - 1)] = v[k];
              if (last && pos < 64) munres[slot][pos] = v[k];
            }
            nu += __popcll(um);
          }
        }
        return nu;
      };
      int nu = 0;
      // early: everything whose source is already final
      if (fits) nu = resolve(ne, prog_done(lds_acquire64(&s_prog)), false);
      // late, once the scan is within kPullLag blocks: the few pairs left
      // (sources in the last kPullLag blocks are left to the scan wave)
      spin = 0;
      while (prog_done(lds_acquire64(&s_prog)) < c - kPullLag) {
        __builtin_amdgcn_s_sleep(1);
        if (++spin > kSpinMax) {
          if (lane == 0) atomicOr(err, 1);
          return;
        }
      }
      if (fits) nu = resolve(nu, prog_done(lds_acquire64(&s_prog)), true);
      const uint32_t rlo = wave_or32(plo), rhi = wave_or32(phi);
      mdiag[slot][lane] = dg;
      msid[slot][lane] = sd;
      if (lane == 0) {
        me0[slot] = e0;
        mne[slot] = fits ? nu : -ne - 1;
        mpre[slot] = fits ? ((uint64_t)rhi << 32) | rlo : 0ull;
        mend[slot] = e1 - E0;
      }
      if (lane == 0) lds_release(&mready[slot], c);
#ifdef JABD_NMS_TRACE
      if (c == lid) l_first = __builtin_readcyclecounter() - l_start;
#endif
    }
#ifdef JABD_NMS_TRACE
    if (lane == 0 && b == 0)
      printf("loader %d img 0: %llu cycles, %llu loading, %llu waiting for space, first block at %llu\n", wave,
             (unsigned long long)(__builtin_readcyclecounter() - l_start),
             (unsigned long long)l_load, (unsigned long long)l_space, (unsigned long long)l_first);
#endif
    return;
  }

  // -------------------------------------------------------------- scan wave
  // Software-pipelined: block c+1's flag and staged data are read while
  // block c resolves (in registers: sources in the last kPullLag blocks come
  // from kw[]), so the wave's LDS round trips overlap its own ALU work.  The
  // flag is read first and the data after it with no wait in between: LDS
  // executes one wave's accesses in order, so data read after a flag that is
  // already set is the loader's (a flag not yet set discards the reads).
  // Publishing is likewise two in-order LDS writes (kept word, then progress).
  int64_t* kout = keep + (int64_t)(b + img0) * keep_bstride;
  int nkeep = 0;
  uint64_t kw[kPullLag];  // kept words of blocks c-1 .. c-kPullLag (wave-uniform)
#pragma unroll
  for (int x = 0; x < kPullLag; ++x) kw[x] = 0;
  struct Meta {
    int e0, ne, e_end, sd;
    uint64_t pre, dg;
    uint32_t uv;
  };
  auto read_meta = [&](int slot, Meta& m) {
    m.e0 = me0[slot];
    m.ne = mne[slot];  // unresolved pairs left by the loader (or -total - 1: read from HBM)
    m.pre = mpre[slot];
    m.e_end = mend[slot];
    m.dg = mdiag[slot][lane];
    m.sd = msid[slot][lane];
    m.uv = munres[slot][lane];
  };
  // waits (bounded) for block c's flag, then reads its data
  auto wait_meta = [&](int c, Meta& m) -> bool {
    const int slot = c % kMetaRing;
    unsigned spin = 0;
    while (lds_acquire(&mready[slot]) != c) {
      __builtin_amdgcn_s_sleep(1);
      if (++spin > kSpinMax) return false;
    }
    read_meta(slot, m);
    return true;
  };
#ifdef JABD_NMS_TRACE
  uint64_t t_start = __builtin_readcyclecounter();
  int n_late = 0;
#endif
  Meta cur;
  bool ok = wait_meta(0, cur);
  for (int c = 0; ok && c < nbv; ++c) {
    // (past the last block the reads are of an unused slot and dropped)
    Meta nxt;
    const int s1 = (c + 1) % kMetaRing;
    // flag, then an LDS-only acquire fence, then the slot's data: the
    // fence pairs with the loader's release (lds_release) when f1 == c + 1
    // and keeps the data reads after the flag read.  "workgroup-one-as"
    // orders LDS with respect to LDS only, so the AMDGPU memory model needs
    // no s_waitcnt for it (one wave's LDS operations complete in order);
    // the flag and data reads stay in flight together
    int f1 = __hip_atomic_load(&mready[s1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup-one-as");
    read_meta(s1, nxt);
    int ne = cur.ne;
    const bool fits = ne >= 0;
    if (!fits) ne = -ne - 1;
    const uint32_t uv = cur.uv;
    uint32_t mlo = 0, mhi = 0;
    uint64_t rem = cur.pre;
    if (fits && ne <= 64) {
      if (ne > 0) {
        // sources in the last kPullLag blocks: their kept words are in kw[];
        // few hits, one bit each, gathered lane by lane
        const int d = c - 1 - (int)(uv >> 12);
        uint64_t w = kw[0];
#pragma unroll
        for (int x = 1; x < kPullLag; ++x) w = d == x ? kw[x] : w;
        uint64_t hm = __ballot(lane < ne && ((w >> ((uv >> 6) & 63)) & 1));
        while (hm) {
          const int p = __ffsll((unsigned long long)hm) - 1;
          hm &= hm - 1;
          rem |= 1ull << (__builtin_amdgcn_readlane(uv, p) & 63);
        }
      }
    } else {
      if (fits) {
        for (int q0 = 0; q0 < ne; q0 += 64) {
          const int q = q0 + lane;
          const uint32_t v = q < ne ? ents[(cur.e0 - E0 + q) & (kEntRing - 1)] : 0u;
          const uint64_t w = kb[v >> 12];
          const bool hit = q < ne && ((w >> ((v >> 6) & 63)) & 1);
          const uint32_t bit = v & 63;
          mlo |= (hit && bit < 32) ? 1u << (bit & 31) : 0u;
          mhi |= (hit && bit >= 32) ? 1u << (bit & 31) : 0u;
        }
      } else {
        // a list larger than the ring: the loader left it whole; read it from
        // HBM in its own branch (a global load pending where the paths join
        // would make the compiler wait vmcnt(0) there, i.e. for this wave's
        // stores)
        for (int q0 = 0; q0 < ne; q0 += 512) {
          uint32_t v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int q = q0 + lane + 64 * k;
            v[k] = csr[cur.e0 + (q < ne ? q : 0)];
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          uint64_t w[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) w[k] = kb[v[k] >> 12];  // src block = (v >> 6) >> 6
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const bool hit = q0 + lane + 64 * k < ne && ((w[k] >> ((v[k] >> 6) & 63)) & 1);
            const uint32_t bit = v[k] & 63;
            mlo |= (hit && bit < 32) ? 1u << (bit & 31) : 0u;
            mhi |= (hit && bit >= 32) ? 1u << (bit & 31) : 0u;
          }
        }
      }
      rem |= ((uint64_t)wave_or32(mhi) << 32) | wave_or32(mlo);
    }
    const int lim = cnt - 64 * c < 64 ? cnt - 64 * c : 64;
    const uint64_t valid = lim == 64 ? ~0ull : ((1ull << lim) - 1);
    uint64_t todo = __ballot(cur.dg != 0) & valid;
    const uint32_t dlo = (uint32_t)cur.dg, dhi = (uint32_t)(cur.dg >> 32);
    while (todo) {  // rows with in-block suppressions, in rank order
      const int t = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      if (!((rem >> t) & 1)) {
        const uint32_t lo = __builtin_amdgcn_readlane(dlo, t);
        const uint32_t hi = __builtin_amdgcn_readlane(dhi, t);
        rem |= ((uint64_t)hi << 32) | lo;
      }
    }
    const uint64_t kept = valid & ~rem;
#ifndef JABD_NMS_AB_NOKOUT  // A/B timing build: kept rows not written (results wrong)
    if ((kept >> lane) & 1) kout[nkeep + __popcll(kept & ((1ull << lane) - 1))] = cur.sd;
#endif
    nkeep += __popcll(kept);
#pragma unroll
    for (int x = kPullLag - 1; x > 0; --x) kw[x] = kw[x - 1];
    kw[0] = kept;
    if (lane == 0) {
      kb[c] = kept;
      // release (LDS only, as above: no wait for this wave's kout stores):
      // a loader that acquires s_prog >= c + 1 sees kb[c]
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup-one-as");
      __hip_atomic_store(&s_prog, ((uint64_t)(uint32_t)cur.e_end << 32) | (uint32_t)(c + 1),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // the prefetched values are first touched here, so their LDS latency
    // overlaps this block's work (no early wait)
    asm volatile("" : "+v"(f1), "+v"(nxt.e0), "+v"(nxt.ne), "+v"(nxt.e_end), "+v"(nxt.sd),
                 "+v"(nxt.pre), "+v"(nxt.dg), "+v"(nxt.uv));
    f1 = __builtin_amdgcn_readfirstlane(f1);
    if (c + 1 < nbv) {
      if (f1 == c + 1) {
        cur = nxt;
        cur.e0 = __builtin_amdgcn_readfirstlane(nxt.e0);  // uniform fields back to scalars
        cur.ne = __builtin_amdgcn_readfirstlane(nxt.ne);
        cur.e_end = __builtin_amdgcn_readfirstlane(nxt.e_end);
        cur.pre = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(nxt.pre >> 32)) << 32) |
                  (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)nxt.pre);  // (int result: no sign extension)
      } else {
#ifdef JABD_NMS_TRACE
        ++n_late;
#endif
        ok = wait_meta(c + 1, cur);
      }
    }
  }
  if (!ok && lane == 0) atomicOr(err, 2);
  if (lane == 0) n_keep[b + img0] = nkeep;
#ifdef JABD_NMS_TRACE
  if (lane == 0)
    printf("nms_scan_pull img %d: %d blocks, %llu cycles, %d blocks not staged in time\n", b, nbv,
           (unsigned long long)(__builtin_readcyclecounter() - t_start), n_late);
#endif
}

// Dense-list images (NaN boxes, thr < 0, or a grid overflow: dense[b] != 0):
// one workgroup per image walks the row blocks in rank order.  Block c's
// suppressed-set word comes from LDS; wave 0 resolves the block (only rows
// with in-block suppressions need the ordered pass); then every kept row
// ORs its (column block, bits) list into the LDS bitset.  The next block's
// row data is prefetched into registers while the current one resolves.
static constexpr int kPrefetchEnt = 4;  // list entries per row prefetched (256 threads / 64 rows)

__global__ __launch_bounds__(256) void nms_scan(
    const uint64_t* __restrict__ diag, const int* __restrict__ nzcnt,
    const int* __restrict__ ent_cb, const uint64_t* __restrict__ ent_bits,
    const int* __restrict__ dense, const int* __restrict__ sidx, const int* __restrict__ counts,
    int64_t n, int64_t nb, int img0, int64_t* __restrict__ keep, int64_t keep_bstride,
    int64_t* __restrict__ n_keep) {
  extern __shared__ unsigned long long removed[];
  __shared__ uint64_t s_kept;
  __shared__ int s_nkeep;
  const int b = blockIdx.x;
  if (!dense[b]) return;  // grid images: nms_scan_pull
  const int cnt = counts[b];
  const int64_t nbv = (cnt + 63) / 64;
  const int tid = threadIdx.x, lane = tid & 63, e = tid >> 6;
  for (int64_t w = tid; w < nbv; w += blockDim.x) removed[w] = 0;
  if (tid == 0) s_nkeep = 0;
  const uint64_t* dimg = diag + (int64_t)b * n;
  const int* cimg = nzcnt + (int64_t)b * n;
  const int64_t ebase = (int64_t)b * ent_base(nb, nb);
  const int* sid = sidx + (int64_t)b * n;
  int64_t* kout = keep + (int64_t)(b + img0) * keep_bstride;

  // prefetch registers for block c: this thread's row = 64c + lane, entry e
  auto prefetch = [&](int64_t c, uint64_t& pdiag, int& pcnt, int& pcb, uint64_t& pbits) {
    const int64_t r = c * 64 + lane;
    pdiag = 0; pcnt = 0; pcb = -1; pbits = 0;
    if (c < nbv && r < cnt) {
      pcnt = cimg[r];
      if (e == 0) pdiag = dimg[r];
      if (e < pcnt) {
        const int64_t off = ebase + ent_base(c, nb) + (int64_t)lane * (nb - c - 1) + e;
        pcb = ent_cb[off];
        pbits = ent_bits[off];
      }
    }
  };
  uint64_t pdiag;
  int pcnt, pcb;
  uint64_t pbits;
  prefetch(0, pdiag, pcnt, pcb, pbits);
  __syncthreads();

  for (int64_t c = 0; c < nbv; ++c) {
    if (e == 0) {  // wave 0: resolve block c
      const int lim = (int)min((int64_t)64, (int64_t)cnt - c * 64);
      const uint64_t valid = lim == 64 ? ~0ull : ((1ull << lim) - 1);
      uint64_t rem = removed[c];
      uint64_t todo = __ballot(pdiag != 0) & valid;
      const uint32_t dlo = (uint32_t)pdiag, dhi = (uint32_t)(pdiag >> 32);
      while (todo) {  // rows with in-block suppressions, in rank order
        const int t = __ffsll((unsigned long long)todo) - 1;
        todo &= todo - 1;
        if (!((rem >> t) & 1)) {
          const uint32_t lo = __builtin_amdgcn_readlane(dlo, t);
          const uint32_t hi = __builtin_amdgcn_readlane(dhi, t);
          rem |= ((uint64_t)hi << 32) | lo;
        }
      }
      const uint64_t kept = valid & ~rem;
      const int base = s_nkeep;  // one wave: read retires before lane 0's write
      if ((kept >> lane) & 1) {
        const int pos = base + __popcll(kept & ((1ull << lane) - 1));
        kout[pos] = sid[c * 64 + lane];
      }
      if (lane == 0) {
        s_kept = kept;
        s_nkeep = base + __popcll(kept);
      }
    }
    __syncthreads();
    const uint64_t kept = s_kept;
    if ((kept >> lane) & 1) {
      if (e < pcnt) atomicOr(&removed[pcb], (unsigned long long)pbits);
      if (pcnt > kPrefetchEnt) {  // long lists: the row's 4 threads share the rest
        const int64_t off = ebase + ent_base(c, nb) + (int64_t)lane * (nb - c - 1);
        for (int q = kPrefetchEnt + e; q < pcnt; q += kPrefetchEnt)
          atomicOr(&removed[ent_cb[off + q]], (unsigned long long)ent_bits[off + q]);
      }
    }
    prefetch(c + 1, pdiag, pcnt, pcb, pbits);
    __syncthreads();
  }
  if (tid == 0) n_keep[b + img0] = s_nkeep;
}

// ---------------------------------------------------------------------------
// radix sort (keys + values) and scan workspace
static size_t sort_temp_bytes(int64_t items) {
  return std::max(radix_ws_bytes(items, true), scan_ws_bytes(items));
}

struct NmsWs {
  uint64_t *kin, *kout;
  char* tmp;
  size_t tmp_bytes;
  float4* sbox;
  float* sarea;
  int *sidx, *counts, *nanflag, *err;
  uint64_t* diag;
  int* nzcnt;
  int* ent_cb;
  uint64_t* ent_bits;
  // grid path
  unsigned* ext;
  int *dense, *npairs, *gval_in, *gval_out, *lcnt, *wcnt, *istart, *bhist, *boff, *ocnt;
  uint64_t* rec;  // per key-order wave: kWaveRec pair records
  uint64_t* ovf;  // per image: ovcap overflow pair records
  int64_t ovcap;
  uint32_t* csr;
  int kchunks;    // count-sort chunks per image
  unsigned long long* tested;  // grid candidates IoU-tested per image (measurement)
  CellRun* runs;               // cell-run hash table (power-of-two slots)
  uint32_t run_mask;
  float4* gbox;
  int64_t cap;
};

// grid_pairs workgroups (256 keys each, a multiple of 8 for the XCD map)
static int64_t grid_pair_blocks(int64_t keys) { return (cdiv(keys, 256) + 7) / 8 * 8; }
// count-sort chunks per image: about 16 key-order waves each (one per wave of
// a grid_bucket_* workgroup)
static int grid_chunks(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>(cdiv(n, 64 * 16), 1), 256); }

template <typename A>
static void carve_nms(A& a, int64_t batch, int64_t n, NmsWs* w) {
  const int64_t bc = images_per_pass(batch, n);
  const int64_t nb = cdiv(n, 64);
  const int64_t ents = bc * 64 * (nb * (nb - 1) / 2 + 1);
  const int64_t cap = kPairsPerBox * (n > 0 ? n : 1);
  const int kch = grid_chunks(n);
  const size_t tb = sort_temp_bytes(std::max(bc * n, bc * nb * kch + 1));
#define T(type, cnt, field)                        \
  do {                                             \
    auto* ptr_ = a.template take<type>(cnt);       \
    if (w) w->field = reinterpret_cast<decltype(w->field)>(ptr_); \
  } while (0)
  T(uint64_t, bc * n, kin);     // keys in (also the grid keys)
  T(uint64_t, bc * n, kout);    // keys out (also the sorted grid keys)
  T(char, tb, tmp);
  T(float4, bc * n, sbox);
  T(float, bc * n, sarea);
  T(int, bc * n, sidx);
  T(int, bc, counts);
  T(int, bc, nanflag);
  T(int, 1, err);
  T(uint64_t, bc * n, diag);
  T(int, bc * n, nzcnt);
  T(int, ents, ent_cb);
  T(uint64_t, ents, ent_bits);
  T(unsigned, bc * 4 * kNC, ext);
  T(int, bc, dense);
  T(int, bc, npairs);
  T(unsigned long long, bc * 64, tested);
  T(int, bc * n, gval_in);
  T(int, bc * n, gval_out);
  const int64_t nwaves = grid_pair_blocks(bc * n) * 4;
  T(int, nwaves * 64, lcnt);
  T(int, nwaves, wcnt);
  T(int, bc + 1, istart);
  T(int, bc * nb * kch + 1, bhist);
  T(int, bc * nb * kch + 1, boff);
  T(uint64_t, nwaves * kWaveRec, rec);
  const int64_t ovcap = nms_ovf_per_box() * (n > 0 ? n : 1);
  T(uint64_t, bc * ovcap, ovf);
  T(int, bc, ocnt);
  T(uint32_t, nwaves * kWaveRec + bc * ovcap, csr);
  T(float4, bc * n, gbox);
  // one run table per image (its own XCD's L2 holds it: 2 MiB at n = 100k),
  // power-of-two slots >= 1.25 n (load factor <= 0.8 even if every box is a run)
  int64_t slots = 1024;
  while (slots * 4 < 5 * n) slots <<= 1;
  T(CellRun, bc * slots, runs);
#undef T
  if (w) w->run_mask = (uint32_t)(slots - 1);
  if (w) {
    w->tmp_bytes = tb;
    w->cap = cap;
    w->kchunks = kch;
    w->ovcap = ovcap;
  }
}

size_t nms_ws_bytes(int64_t batch, int64_t n) {
  Sizer s;
  carve_nms(s, batch, n, (NmsWs*)nullptr);
  return s.used;
}

int nms_core(const float* boxes, int64_t box_stride, int64_t box_bstride,
             const float* scores, int64_t score_stride, int64_t score_bstride,
             const int64_t* n_valid, int64_t batch, int64_t n, double iou_thr,
             float score_thr, int64_t* keep, int64_t* n_keep, void* ws,
             size_t ws_bytes, hipStream_t st) {
  JABD_REQUIRE(n >= 0 && batch >= 0, "nms: negative size");
  JABD_REQUIRE(n < kMaxRows, "nms: n=%lld exceeds %lld rows per image", (long long)n,
               (long long)kMaxRows);
  const int64_t nb = cdiv(n, 64);
  JABD_REQUIRE(nb * 12 + 4 <= 160 * 1024, "nms: n=%lld too large for the LDS scan",
               (long long)n);
  if (batch == 0) return JABD_OK;
  if (n == 0) {
    const FillRange fr{n_keep, (int64_t)sizeof(int64_t) * batch, 0u};
    if (int e = fill_ranges(&fr, 1, st)) return e;
    return JABD_OK;
  }
  JABD_REQUIRE(ws_bytes >= nms_ws_bytes(batch, n), "nms: workspace %zu < %zu", ws_bytes,
               nms_ws_bytes(batch, n));
  const int filter = score_thr > -INFINITY ? 1 : 0;
  const int64_t per_pass = images_per_pass(batch, n);
  // log-area class width W' >= 1.01 * -ln(thr) (wider is always safe)
  // the pull scan keeps one kept word per row block in LDS next to its rings
  const bool grid = iou_thr >= 0.0 && !nms_dense_only() && n > nms_dense_rows() &&
                    nb * 8 + kPullStaticLds <= 160 * 1024;
  double wcls = iou_thr > 0.0 ? 1.01 * -std::log(iou_thr) : INFINITY;
  if (wcls < 0.2) wcls = 0.2;  // wider classes are always safe; keeps ln-range / W' < kNC
  wcls /= kK;
  const float inv_w = std::isinf(wcls) ? 0.f : (float)(1.0 / wcls);
  // cell scale f = (1 - t) / (1 + t) (>= 0.05), with a 5% rounding margin
  const double tcl = iou_thr > 0.0 ? std::min(iou_thr, 1.0) : 0.0;
  const float fcell = (float)(1.05 * std::max((1.0 - tcl) / (1.0 + tcl), 0.05));
  for (int64_t img0 = 0; img0 < batch; img0 += per_pass) {
    const int bc = (int)min(per_pass, batch - img0);
    Carve cv(ws, ws_bytes);
    NmsWs w;
    carve_nms(cv, bc, n, &w);
    if (!cv.ok()) {
      set_error("nms: workspace carve overflow");
      return JABD_EWS;
    }
    {  // every counter / table this pass starts from, one launch
      const int64_t gb = grid ? 1 : 0;  // the grid path's tables
      const FillRange fr[12] = {
          {w.counts, (int64_t)sizeof(int) * bc, 0u},
          {w.nanflag, (int64_t)sizeof(int) * bc, 0u},
          {w.err, (int64_t)sizeof(int), 0u},
          {w.nzcnt, (int64_t)sizeof(int) * bc * n, 0u},
          {w.dense, (int64_t)sizeof(int) * bc, grid ? 0u : 1u},  // 1: every image dense
          {w.npairs, gb * (int64_t)sizeof(int) * bc, 0u},
          {w.tested, gb * (int64_t)sizeof(unsigned long long) * bc * 64, 0u},
          {w.ext, gb * (int64_t)sizeof(unsigned) * bc * 4 * kNC, 0u},
          {w.runs, gb * (int64_t)sizeof(CellRun) * bc * ((int64_t)w.run_mask + 1), 0xFFFFFFFFu},
          {w.diag, gb * (int64_t)sizeof(uint64_t) * bc * n, 0u},
          {w.bhist + (int64_t)bc * nb * w.kchunks, gb * (int64_t)sizeof(int), 0u},
          {w.ocnt, gb * (int64_t)sizeof(int) * bc, 0u}};
      if (int e = fill_ranges(fr, 12, st)) return e;
    }
    dim3 g1((unsigned)cdiv(n, 256), bc);
    int sorted = -1;
    if (bc == 1 && n <= radix_small_max()) {
      // one image: the candidates' keys compacted, sorted by ~score (bits 24-55)
      nms_keys_compact<<<1, kCompactT, 0, st>>>(scores + img0 * score_bstride, score_stride,
                                                n_valid, n, score_thr, filter, (int)img0, w.kin,
                                                w.counts);
      if (int e = check_launch("nms_keys_compact")) return e;
      sorted = radix_sort64_devn(w.kin, w.kout, w.counts, n, 24, 4, w.tmp, w.tmp_bytes, st);
      if (sorted != JABD_OK) return sorted < 0 ? JABD_EINVAL : sorted;
    }
    if (sorted < 0) {
      nms_keys<<<g1, 256, 0, st>>>(scores, score_stride, score_bstride, n_valid, n, bc,
                                    score_thr, filter, (int)img0, w.kin, w.counts);
      if (int e = check_launch("nms_keys")) return e;
      // [image | ~score] (bits 24-63); rows are already in input order
      if (int e = radix_sort64(w.kin, w.kout, nullptr, nullptr, (int64_t)bc * n, 24, 5, false,
                               w.tmp, w.tmp_bytes, st))
        return e;
    }
    nms_gather<<<(unsigned)cdiv((int64_t)bc * n, 256), 256, 0, st>>>(
        w.kout, (int64_t)bc * n, boxes, box_stride, box_bstride, w.counts, bc, n, (int)img0,
        w.sbox, w.sarea, w.sidx, w.nanflag);
    if (int e = check_launch("nms_gather")) return e;
    if (grid) {
      dim3 ge((unsigned)cdiv(n, 256 * kExtPer), bc);
      grid_ext<<<ge, 256, 0, st>>>(w.sbox, w.sarea, w.counts, w.nanflag, n, inv_w, w.ext, w.dense,
                                   nms_dense_max());
      if (int e = check_launch("grid_ext")) return e;
      grid_keys<<<g1, 256, 0, st>>>(w.sbox, w.sarea, w.counts, n, inv_w, fcell, w.ext, w.kin,
                                     w.gval_in, w.dense);
      if (int e = check_launch("grid_keys")) return e;
      if (int e = radix_sort64(w.kin, w.kout, w.gval_in, w.gval_out, (int64_t)bc * n, 0, 8, true,
                               w.tmp, w.tmp_bytes, st))
        return e;
      grid_gather<<<(unsigned)cdiv((int64_t)bc * n, 256), 256, 0, st>>>(
          w.kout, w.gval_out, (int64_t)bc * n, w.sbox, n, w.gbox);
      if (int e = check_launch("grid_gather")) return e;
      const unsigned gt = (unsigned)cdiv((int64_t)bc * n, 256);
      grid_runs_insert<<<gt, 256, 0, st>>>(w.kout, (int64_t)bc * n, w.runs, w.run_mask, bc,
                                           w.istart);
      if (int e = check_launch("grid_runs_insert")) return e;
      grid_runs_end<<<gt, 256, 0, st>>>(w.kout, (int64_t)bc * n, w.runs, w.run_mask);
      if (int e = check_launch("grid_runs_end")) return e;
      grid_pairs<<<(unsigned)grid_pair_blocks((int64_t)bc * n), 256, 0, st>>>(
          w.kout, w.gval_out, (int64_t)bc * n, w.gbox, n, bc, inv_w, fcell, w.ext,
          w.runs, w.run_mask, iou_thr, w.dense, w.diag, w.rec, w.lcnt, w.wcnt, w.ovf, w.ocnt,
          w.ovcap, w.tested);
      if (int e = check_launch("grid_pairs")) return e;
      const unsigned gk = (unsigned)(w.kchunks * bc);
      const size_t hl = (size_t)nb * sizeof(int);
      grid_bucket_count<<<gk, kBucketT, hl, st>>>(w.rec, w.lcnt, w.wcnt, w.ovf, w.ocnt, w.ovcap,
                                                  w.istart, w.dense, nb, w.kchunks, w.bhist,
                                                  w.npairs);
      if (int e = check_launch("grid_bucket_count")) return e;
      if (int e = scan_excl_i32(w.bhist, w.boff, (int64_t)bc * nb * w.kchunks + 1, w.tmp,
                                w.tmp_bytes, st))
        return e;
      grid_bucket_scatter<<<gk, kBucketT, hl, st>>>(w.rec, w.lcnt, w.wcnt, w.ovf, w.ocnt, w.ovcap,
                                                    w.istart, w.dense, nb, w.kchunks, w.boff,
                                                    w.csr);
      if (int e = check_launch("grid_bucket_scatter")) return e;
    }
    nms_mask<<<2048, 256, 0, st>>>(w.sbox, w.sarea, w.counts, n, nb, bc, iou_thr, w.nanflag, w.dense,
                                 w.diag, w.nzcnt, w.ent_cb, w.ent_bits);
    if (int e = check_launch("nms_mask")) return e;
    if (nb * sizeof(uint64_t) > 64 * 1024) {
      JABD_HIP(hipFuncSetAttribute((const void*)nms_scan,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    nms_scan<<<bc, 256, nb * sizeof(uint64_t), st>>>(w.diag, w.nzcnt, w.ent_cb, w.ent_bits,
                                                      w.dense, w.sidx, w.counts, n, nb,
                                                      (int)img0, keep, n, n_keep);
    if (int e = check_launch("nms_scan")) return e;
    if (grid) {
      const size_t lds = (size_t)nb * 8;
      if (lds + kPullStaticLds > 64 * 1024) {
        JABD_HIP(hipFuncSetAttribute((const void*)nms_scan_pull,
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024 - kPullStaticLds));
      }
      nms_scan_pull<<<bc, 64 * kPullWaves, lds, st>>>(
          w.diag, w.dense, w.boff, w.kchunks, w.csr, w.sidx,
          w.counts, n, (int)img0, keep, n, n_keep, w.err);
      if (int e = check_launch("nms_scan_pull")) return e;
    }
  }
  return JABD_OK;
}

}  // namespace jabd

extern "C" int jabd_nms_workspace_size(int64_t batch, int64_t n, size_t* bytes) {
  JABD_REQUIRE(bytes && batch >= 0 && n >= 0, "nms_workspace_size: bad args");
  *bytes = jabd::nms_ws_bytes(batch, n);
  return JABD_OK;
}

extern "C" int jabd_batched_nms_f32(const float* boxes, int64_t box_stride,
                                    int64_t box_bstride, const float* scores,
                                    int64_t score_stride, int64_t score_bstride,
                                    const int64_t* n_valid, int64_t batch, int64_t n,
                                    double iou_threshold, float score_threshold,
                                    int64_t* keep, int64_t* n_keep, void* ws,
                                    size_t ws_bytes, jabd_stream_t stream) {
  JABD_REQUIRE(box_stride >= 4 && score_stride >= 1, "nms: bad row stride");
  JABD_REQUIRE((boxes && scores && keep && n_keep) || n == 0 || batch == 0,
               "nms: null pointer");
  JABD_REQUIRE(n_keep || batch == 0, "nms: null n_keep");
  return jabd::nms_core(boxes, box_stride, box_bstride, scores, score_stride, score_bstride,
                        n_valid, batch, n, iou_threshold, score_threshold, keep, n_keep, ws,
                        ws_bytes, jabd::as_stream(stream));
}

// Measurement helper (bench.py's IoU-pair count): after jabd_batched_nms_f32
// with this (batch, n, ws), copy each image's number of exact IoU tests of the
// grid producer (candidate pairs), its off-block suppressing pairs, and the
// producer (0 = grid, != 0 = dense: that image tested every pair) to the host.
// Synchronises `stream`.  Valid for batch <= 254 (one pass holds every image).
extern "C" int jabd_nms_pair_stats(const void* ws, size_t ws_bytes, int64_t batch, int64_t n,
                                   int64_t* tested, int32_t* hits, int32_t* dense,
                                   jabd_stream_t stream) {
  using namespace jabd;
  JABD_REQUIRE(ws && tested && hits && dense && batch > 0 && n > 0, "nms_pair_stats: bad args");
  JABD_REQUIRE(images_per_pass(batch, n) == batch, "nms_pair_stats: batch spans several passes");
  Carve cv(const_cast<void*>(ws), ws_bytes);
  NmsWs w;
  carve_nms(cv, batch, n, &w);
  JABD_REQUIRE(cv.ok(), "nms_pair_stats: workspace too small");
  hipStream_t st = as_stream(stream);
  std::vector<unsigned long long> slots((size_t)batch * 64);
  JABD_HIP(hipMemcpyAsync(slots.data(), w.tested, sizeof(unsigned long long) * batch * 64,
                          hipMemcpyDeviceToHost, st));
  JABD_HIP(hipMemcpyAsync(hits, w.npairs, sizeof(int32_t) * batch, hipMemcpyDeviceToHost, st));
  JABD_HIP(hipMemcpyAsync(dense, w.dense, sizeof(int32_t) * batch, hipMemcpyDeviceToHost, st));
  int err = 0;
  JABD_HIP(hipMemcpyAsync(&err, w.err, sizeof(int), hipMemcpyDeviceToHost, st));
  JABD_HIP(hipStreamSynchronize(st));
  JABD_REQUIRE(err == 0, "nms: the pull scan's staging hand-off timed out (flags %d)", err);
  for (int64_t b = 0; b < batch; ++b) {
    unsigned long long t = 0;
    for (int l = 0; l < 64; ++l) t += slots[(size_t)b * 64 + l];
    tested[b] = (int64_t)t;
  }
  return JABD_OK;
}
