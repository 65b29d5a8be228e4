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
//                    row box, column boxes broadcast from LDS; stored sparse:
//                    the in-block word per row + a list of non-zero words.
//   5. nms_scan      one workgroup per image walks the row blocks on the
//                    device (suppressed-set bitset in LDS, next block's lists
//                    prefetched), writes kept rows + count.
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

__global__ __launch_bounds__(256) void nms_mask(
    const float4* __restrict__ sbox, const float* __restrict__ sarea,
    const int* __restrict__ counts, int64_t n, int64_t nb, double thr,
    const int* __restrict__ nanflag, uint64_t* __restrict__ diag, int* __restrict__ nzcnt,
    int* __restrict__ ent_cb, uint64_t* __restrict__ ent_bits) {
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
}

// One workgroup per image walks the row blocks in rank order.  Block c's
// suppressed-set word comes from LDS; wave 0 resolves the block (only rows
// with in-block suppressions need the ordered pass); then every kept row
// ORs its sparse list into the LDS bitset.  The next block's row data is
// prefetched into registers while the current one resolves.
static constexpr int kPrefetchEnt = 4;  // list entries per row prefetched (256 threads / 64 rows)

__global__ __launch_bounds__(256) void nms_scan(
    const uint64_t* __restrict__ diag, const int* __restrict__ nzcnt,
    const int* __restrict__ ent_cb, const uint64_t* __restrict__ ent_bits,
    const int* __restrict__ sidx, const int* __restrict__ counts, int64_t n, int64_t nb, int img0,
    int64_t* __restrict__ keep, int64_t keep_bstride, int64_t* __restrict__ n_keep) {
  extern __shared__ unsigned long long removed[];
  __shared__ uint64_t s_kept;
  __shared__ int s_nkeep;
  const int b = blockIdx.x;
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
      if (e == 0 && pcnt > kPrefetchEnt) {  // long lists: rare slow path
        const int64_t off = ebase + ent_base(c, nb) + (int64_t)lane * (nb - c - 1);
        for (int q = kPrefetchEnt; q < pcnt; ++q)
          atomicOr(&removed[ent_cb[off + q]], (unsigned long long)ent_bits[off + q]);
      }
    }
    prefetch(c + 1, pdiag, pcnt, pcb, pbits);
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
  a.template take<int>(bc);                // NaN-box flags
  a.template take<uint64_t>(bc * n);       // diag words
  a.template take<int>(bc * n);            // list lengths
  a.template take<int>(bc * 64 * (nb * (nb - 1) / 2 + 1));       // list column blocks
  a.template take<uint64_t>(bc * 64 * (nb * (nb - 1) / 2 + 1));  // list bit words
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
    int* nanflag = cv.take<int>(bc);
    uint64_t* diag = cv.take<uint64_t>((size_t)bc * n);
    int* nzcnt = cv.take<int>((size_t)bc * n);
    int* ent_cb = cv.take<int>((size_t)bc * 64 * (nb * (nb - 1) / 2 + 1));
    uint64_t* ent_bits = cv.take<uint64_t>((size_t)bc * 64 * (nb * (nb - 1) / 2 + 1));
    if (!cv.ok()) {
      set_error("nms: workspace carve overflow");
      return JABD_EWS;
    }
    JABD_HIP(hipMemsetAsync(counts, 0, sizeof(int) * bc, st));
    JABD_HIP(hipMemsetAsync(nanflag, 0, sizeof(int) * bc, st));
    JABD_HIP(hipMemsetAsync(nzcnt, 0, sizeof(int) * bc * n, st));
    dim3 g1((unsigned)cdiv(n, 256), bc);
    nms_keys<<<g1, 256, 0, st>>>(scores, score_stride, score_bstride, n_valid, n, bc,
                                  score_thr, filter, (int)img0, kin, counts);
    if (int e = check_launch("nms_keys")) return e;
    JABD_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, kin, kout, (int)(bc * n), 0,
                                               64, st));
    nms_gather<<<(unsigned)cdiv((int64_t)bc * n, 256), 256, 0, st>>>(
        kout, (int64_t)bc * n, boxes, box_stride, box_bstride, counts, bc, n, (int)img0,
        sbox, sarea, sidx, nanflag);
    if (int e = check_launch("nms_gather")) return e;
    dim3 g2((unsigned)cdiv(nb, kColBlocksPerWG), (unsigned)nb, (unsigned)bc);
    nms_mask<<<g2, 256, 0, st>>>(sbox, sarea, counts, n, nb, iou_thr, nanflag, diag, nzcnt,
                                 ent_cb, ent_bits);
    if (int e = check_launch("nms_mask")) return e;
    if (nb * sizeof(uint64_t) > 64 * 1024) {
      JABD_HIP(hipFuncSetAttribute((const void*)nms_scan,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    nms_scan<<<bc, 256, nb * sizeof(uint64_t), st>>>(diag, nzcnt, ent_cb, ent_bits, sidx, counts,
                                                      n, nb, (int)img0, keep, n, n_keep);
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
