// A10: batched greedy NMS on gfx950, bit-exact with torchvision's CPU
// nms kernel as called by utils/utils_bbox.py:275 (non_max_suppression).
//
// Pipeline per call (B images, up to n boxes each), all on one stream:
//   1. nms_keys      one 64-bit key per row: [image:8 | ~score:32 | row:24];
//                    rows failing the score filter get image 255 (sorted last).
//   2. radix sort    hipcub DeviceRadixSort::SortKeys (ascending) — gives
//                    every image's rows contiguous, in stable descending-score
//                    order (ties by lower row index, as torch's stable sort).
//   3. nms_gather    sorted boxes (float4) + areas + original row ids.
//   4. nms_mask      upper-triangular IoU bitmask, 64x64 tiles, one lane per
//                    row box, column boxes broadcast from LDS.
//   5. nms_scan      one workgroup per image walks the bitmask on the device
//                    (suppressed-set in LDS), writes kept rows + count.
// Compile with -ffp-contract=off: IoU must round exactly like the CPU kernel
// (no FMA in (x2-x1)*(y2-y1) or inter/(a+b-inter)).
#include <hipcub/hipcub.hpp>
#include <math.h>

#include "common.h"
#include "nms_internal.h"

namespace jabd {

static constexpr int kImgBits = 8;
static constexpr int kRowBits = 24;
static constexpr int64_t kMaxRows = (int64_t(1) << kRowBits);
static constexpr int kMaxImg = 254;  // 255 marks a filtered-out row

// Images per sort pass: <= 254 and the sort size must fit hipcub's int.
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

__global__ void nms_keys(const float* __restrict__ scores, int64_t score_stride,
                         int64_t score_bstride, const int64_t* __restrict__ n_valid,
                         int64_t n, int batch, float thr, int filter, int img0,
                         uint64_t* __restrict__ keys, int* __restrict__ counts) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int b = blockIdx.y;
  if (i >= n || b >= batch) return;
  float s = scores[(int64_t)(b + img0) * score_bstride + i * score_stride];
  int64_t nv = n_valid ? n_valid[b + img0] : n;
  bool valid = i < nv;
  if (filter) valid = valid && (s >= thr);
  uint64_t img = valid ? (uint64_t)b : 255u;
  keys[(int64_t)b * n + i] = (img << 56) | ((uint64_t)score_key_desc(s) << kRowBits) | (uint64_t)i;
  if (valid) {
    // one atomic per wave: count valid lanes with a ballot
    uint64_t m = __ballot(1);
    int lane = threadIdx.x & 63;
    int leader = __ffsll((unsigned long long)m) - 1;
    if (lane == leader) atomicAdd(&counts[b], __popcll(m));
  }
}

__global__ void nms_gather(const uint64_t* __restrict__ sorted, int64_t total,
                           const float* __restrict__ boxes, int64_t box_stride,
                           int64_t box_bstride, const int* __restrict__ counts,
                           int batch, int64_t n, int img0, float4* __restrict__ sbox,
                           float* __restrict__ sarea, int* __restrict__ sidx) {
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
}

// Offset (in u64 words) of row block rb in the per-image triangular mask.
__device__ __host__ __forceinline__ int64_t tri_base(int64_t rb, int64_t nb) {
  return 64 * (rb * nb - rb * (rb - 1) / 2);
}

static constexpr int kColBlocksPerWave = 4;
static constexpr int kWaves = 4;
static constexpr int kColBlocksPerWG = kColBlocksPerWave * kWaves;

// IoU of sorted box i (registers) against sorted box j, torchvision CPU order.
__device__ __forceinline__ bool iou_gt(float ix1, float iy1, float ix2, float iy2,
                                       float iarea, float4 bj, float aj,
                                       double thr, bool thr_nonneg) {
  float xx1 = (ix1 < bj.x) ? bj.x : ix1;  // std::max(ix1, x1[j])
  float yy1 = (iy1 < bj.y) ? bj.y : iy1;
  float xx2 = (bj.z < ix2) ? bj.z : ix2;  // std::min(ix2, x2[j])
  float yy2 = (bj.w < iy2) ? bj.w : iy2;
  float dw = xx2 - xx1, dh = yy2 - yy1;
  float w = (0.f < dw) ? dw : 0.f;        // std::max(0, xx2 - xx1)
  float h = (0.f < dh) ? dh : 0.f;
  float inter = w * h;
  // inter == 0 (or NaN) gives ovr in {0, -0, NaN}: never > a threshold >= 0.
  if (thr_nonneg && !(inter > 0.f)) return false;
  float ovr = inter / (iarea + aj - inter);
  return (double)ovr > thr;
}

__global__ __launch_bounds__(256) void nms_mask(
    const float4* __restrict__ sbox, const float* __restrict__ sarea,
    const int* __restrict__ counts, int64_t n, int64_t nb, double thr,
    uint64_t* __restrict__ mask) {
  const int b = blockIdx.z;
  const int64_t rb = blockIdx.y;
  const int64_t cbg = (int64_t)blockIdx.x * kColBlocksPerWG;
  const int cnt = counts[b];
  const int64_t nbv = (cnt + 63) / 64;
  if (rb >= nbv || cbg + kColBlocksPerWG <= rb || cbg >= nbv) return;

  __shared__ float4 cbox[kColBlocksPerWG * 64];
  __shared__ float carea[kColBlocksPerWG * 64];
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
  uint64_t* mrow = mask + (int64_t)b * tri_base(nb, nb) + tri_base(rb, nb) +
                   (int64_t)lane * (nb - rb);
  for (int q = 0; q < kColBlocksPerWave; ++q) {
    const int64_t cb = cbg + wave * kColBlocksPerWave + q;
    if (cb < rb || cb >= nbv) continue;
    const int lbase = (wave * kColBlocksPerWave + q) * 64;
    const int64_t j0 = cb * 64;
    int jmax = (int)min((int64_t)64, (int64_t)cnt - j0);
    int jstart = (cb == rb) ? lane + 1 : 0;  // strictly after row i on the diagonal
    uint64_t bits = 0;
    if (row_ok) {
      for (int jj = jstart; jj < jmax; ++jj) {
        if (iou_gt(bi.x, bi.y, bi.z, bi.w, ai, cbox[lbase + jj], carea[lbase + jj], thr,
                   thr_nonneg))
          bits |= (uint64_t)1 << jj;
      }
      mrow[cb - rb] = bits;
    }
  }
}

__global__ __launch_bounds__(256) void nms_scan(
    const uint64_t* __restrict__ mask, const int* __restrict__ sidx,
    const int* __restrict__ counts, int64_t n, int64_t nb, int img0,
    int64_t* __restrict__ keep, int64_t keep_bstride, int64_t* __restrict__ n_keep) {
  extern __shared__ uint64_t removed[];
  __shared__ uint64_t s_kept;
  __shared__ int s_nkeep;
  const int b = blockIdx.x;
  const int cnt = counts[b];
  const int64_t nbv = (cnt + 63) / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int64_t w = tid; w < nbv; w += blockDim.x) removed[w] = 0;
  if (tid == 0) s_nkeep = 0;
  __syncthreads();
  const uint64_t* mimg = mask + (int64_t)b * tri_base(nb, nb);
  const int* sid = sidx + (int64_t)b * n;
  int64_t* kout = keep + (int64_t)(b + img0) * keep_bstride;

  for (int64_t c = 0; c < nbv; ++c) {
    const uint64_t* mblk = mimg + tri_base(c, nb);  // row block c, words cb >= c
    const int64_t rowlen = nb - c;
    if (wave == 0) {
      uint64_t word = removed[c];
      const int64_t row = c * 64 + lane;
      uint64_t diag = (row < cnt) ? mblk[(int64_t)lane * rowlen] : 0;
      uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
      const int lim = (int)min((int64_t)64, (int64_t)cnt - c * 64);
      uint64_t kept = 0;
      for (int t = 0; t < lim; ++t) {
        if (!((word >> t) & 1)) {
          kept |= (uint64_t)1 << t;
          uint32_t lo = __builtin_amdgcn_readlane(dlo, t);
          uint32_t hi = __builtin_amdgcn_readlane(dhi, t);
          word |= ((uint64_t)hi << 32) | lo;
        }
      }
      // One wave: its LDS read of s_nkeep retires before lane 0's write.
      int base = s_nkeep;
      if ((kept >> lane) & 1) {
        int pos = base + __popcll(kept & (((uint64_t)1 << lane) - 1));
        kout[pos] = sid[row];
      }
      if (lane == 0) {
        s_kept = kept;
        s_nkeep = base + __popcll(kept);
      }
    }
    __syncthreads();
    const uint64_t kept = s_kept;
    if (kept) {
      for (int64_t w = c + 1 + tid; w < nbv; w += blockDim.x) {
        uint64_t acc = 0;
        uint64_t k = kept;
        while (k) {
          int t = __ffsll((unsigned long long)k) - 1;
          k &= k - 1;
          acc |= mblk[(int64_t)t * rowlen + (w - c)];
        }
        removed[w] |= acc;
      }
    }
    __syncthreads();
  }
  if (tid == 0) n_keep[b + img0] = s_nkeep;
}

// ---------------------------------------------------------------------------
static size_t sort_temp_bytes(int64_t items) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, (const uint64_t*)nullptr,
                                    (uint64_t*)nullptr, (int)items, 0, 64, (hipStream_t)0);
  return bytes;
}

template <typename A>
static void carve_nms(A& a, int64_t batch, int64_t n) {
  int64_t bc = images_per_pass(batch, n);
  int64_t nb = cdiv(n, 64);
  a.template take<uint64_t>(bc * n);       // keys in
  a.template take<uint64_t>(bc * n);       // keys out
  a.template take<char>(sort_temp_bytes(bc * n));
  a.template take<float4>(bc * n);         // sorted boxes
  a.template take<float>(bc * n);          // sorted areas
  a.template take<int>(bc * n);            // sorted row ids
  a.template take<int>(bc);                // counts
  a.template take<uint64_t>(bc * 64 * (nb * (nb + 1) / 2));  // triangular mask
}

size_t nms_ws_bytes(int64_t batch, int64_t n) {
  Sizer s;
  carve_nms(s, batch, n);
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
  JABD_REQUIRE(nb * 8 <= 160 * 1024, "nms: n=%lld too large for the LDS scan", (long long)n);
  if (batch == 0) return JABD_OK;
  if (n == 0) {
    JABD_HIP(hipMemsetAsync(n_keep, 0, sizeof(int64_t) * batch, st));
    return JABD_OK;
  }
  JABD_REQUIRE(ws_bytes >= nms_ws_bytes(batch, n), "nms: workspace %zu < %zu", ws_bytes,
               nms_ws_bytes(batch, n));
  const int filter = score_thr > -INFINITY ? 1 : 0;
  const int64_t per_pass = images_per_pass(batch, n);
  for (int64_t img0 = 0; img0 < batch; img0 += per_pass) {
    const int bc = (int)min(per_pass, batch - img0);
    Carve cv(ws, ws_bytes);
    uint64_t* kin = cv.take<uint64_t>((size_t)bc * n);
    uint64_t* kout = cv.take<uint64_t>((size_t)bc * n);
    size_t tmp_bytes = sort_temp_bytes((int64_t)bc * n);
    char* tmp = cv.take<char>(tmp_bytes);
    float4* sbox = cv.take<float4>((size_t)bc * n);
    float* sarea = cv.take<float>((size_t)bc * n);
    int* sidx = cv.take<int>((size_t)bc * n);
    int* counts = cv.take<int>(bc);
    uint64_t* mask = cv.take<uint64_t>((size_t)bc * 64 * (nb * (nb + 1) / 2));
    if (!cv.ok()) {
      set_error("nms: workspace carve overflow");
      return JABD_EWS;
    }
    JABD_HIP(hipMemsetAsync(counts, 0, sizeof(int) * bc, st));
    dim3 g1((unsigned)cdiv(n, 256), bc);
    nms_keys<<<g1, 256, 0, st>>>(scores, score_stride, score_bstride, n_valid, n, bc,
                                  score_thr, filter, (int)img0, kin, counts);
    if (int e = check_launch("nms_keys")) return e;
    JABD_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, kin, kout, (int)(bc * n), 0,
                                               64, st));
    nms_gather<<<(unsigned)cdiv((int64_t)bc * n, 256), 256, 0, st>>>(
        kout, (int64_t)bc * n, boxes, box_stride, box_bstride, counts, bc, n, (int)img0,
        sbox, sarea, sidx);
    if (int e = check_launch("nms_gather")) return e;
    dim3 g2((unsigned)cdiv(nb, kColBlocksPerWG), (unsigned)nb, (unsigned)bc);
    nms_mask<<<g2, 256, 0, st>>>(sbox, sarea, counts, n, nb, iou_thr, mask);
    if (int e = check_launch("nms_mask")) return e;
    if (nb * sizeof(uint64_t) > 64 * 1024) {
      JABD_HIP(hipFuncSetAttribute((const void*)nms_scan,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    nms_scan<<<bc, 256, nb * sizeof(uint64_t), st>>>(mask, sidx, counts, n, nb, (int)img0,
                                                      keep, n, n_keep);
    if (int e = check_launch("nms_scan")) return e;
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
