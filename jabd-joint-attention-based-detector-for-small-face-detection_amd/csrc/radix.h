// Internal: wavefront radix sort and exclusive scan (radix.hip), used by the
// NMS pipeline (nms.hip) and exported for tests (jabd_sort_u64_f32 / jabd_scan_*).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jabd {
struct RadixWs {
  int *ghist, *plan, *cnt, *off;
  uint64_t* kalt;
  int* valt;
};
size_t radix_ws_bytes(int64_t n, bool vals);
// stable sort of n keys (and values, if vin) by bits [lo, lo + 8 npass);
// kin is not modified; skip_ones: see radix.hip
int radix_sort64(const uint64_t* kin, uint64_t* kout, const int* vin, int* vout, int64_t n,
                 int lo, int npass, bool skip_ones, void* ws, size_t ws_bytes, hipStream_t st);
// The one-workgroup form over a device-side key count: sorts the first
// min(*n_dev, n_cap) keys of kin (no values) and fills kout up to n_cap with
// ~0.  Requires n_cap <= radix_small_max(); returns -1 when the small form is
// switched off (JABD_RADIX_SMALL=0).
int radix_sort64_devn(const uint64_t* kin, uint64_t* kout, const int* n_dev, int64_t n_cap,
                      int lo, int npass, void* ws, size_t ws_bytes, hipStream_t st);
int64_t radix_small_max();
size_t scan_ws_bytes(int64_t n);
int scan_excl_i32(const int* in, int* out, int64_t n, void* ws, size_t ws_bytes, hipStream_t st);
}  // namespace jabd
