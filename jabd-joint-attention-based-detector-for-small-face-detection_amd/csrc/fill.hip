// Workspace initialisation as one kernel launch over several ranges (32-bit
// fill words, 16-byte stores on the aligned middle of each range) instead of
// one hipMemsetAsync per buffer: the NMS / radix / loss workspaces set up to
// 12 counters and tables per call, and at bs1 each memset cost a separate
// blit launch of ~4-5 us (rocprof: 13 per detect call).  A kernel node is also
// the plainest thing a HIP graph capture can record.
#include <algorithm>

#include "common.h"

namespace jabd {

__global__ __launch_bounds__(256) void fill_ranges_kernel(const FillArgs a) {
  const FillRange r = a.r[blockIdx.y];
  const uint32_t v = r.value;
  uint32_t* p = static_cast<uint32_t*>(r.ptr);
  const int64_t n4 = r.bytes >> 2;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  // words before the first 16-byte boundary, the uint4 body, the tail words
  const int64_t head = std::min<int64_t>((int64_t)(((16 - ((uintptr_t)p & 15)) & 15) >> 2), n4);
  if (tid < head) p[tid] = v;
  const int64_t nq = (n4 - head) >> 2;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  const uint4 vv = make_uint4(v, v, v, v);
  for (int64_t i = tid; i < nq; i += nth) q[i] = vv;
  const int64_t t0 = head + 4 * nq;
  if (tid < n4 - t0) p[t0 + tid] = v;
}

int fill_ranges(const FillRange* r, int n, hipStream_t st) {
  JABD_REQUIRE(n >= 0 && n <= kFillMax, "fill_ranges: %d ranges", n);
  FillArgs a;
  int m = 0;
  int64_t most = 0;
  for (int i = 0; i < n; ++i) {
    if (r[i].bytes <= 0) continue;
    JABD_REQUIRE(r[i].ptr && r[i].bytes % 4 == 0 && ((uintptr_t)r[i].ptr & 3) == 0,
                 "fill_ranges: range %d not 4-byte granular", i);
    a.r[m++] = r[i];
    most = std::max(most, r[i].bytes);
  }
  if (m == 0) return JABD_OK;
  const int64_t blocks = std::min<int64_t>(1024, std::max<int64_t>(1, cdiv(most, 16 * 256)));
  fill_ranges_kernel<<<dim3((unsigned)blocks, (unsigned)m), 256, 0, st>>>(a);
  return check_launch("fill_ranges");
}

}  // namespace jabd
