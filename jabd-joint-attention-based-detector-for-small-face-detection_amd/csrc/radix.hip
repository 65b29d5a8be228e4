// Wavefront LSD radix sort of 64-bit keys (optionally carrying int32 values)
// and an exclusive int32 scan — the NMS pipeline's sorts (utils/utils_bbox.py:
// 275 torchvision.ops.nms sorts the scores; nms.hip sorts [image | ~score |
// row] keys and the grid producer's cell keys) and its CSR offsets.
//
// Sort: 8-bit digits over bits [lo, lo + 8 npass), least significant first,
// stable (equal digits keep their input order), so the result is the stable
// sort by those bits; bits below lo keep their input order.
//   radix_hist     one pass over the keys: the histogram of every digit
//                  position at once (LDS counters, one global add per bin)
//   radix_plan     per pass: global digit bases (exclusive prefix over the
//                  256 bins), whether it runs (a pass whose keys all share one
//                  digit is skipped) and which buffers it reads and writes, so
//                  that the last pass that runs writes the output (the input
//                  is never written; if no pass runs, the last one copies)
//   per pass       radix_count  per 4096-key tile: digit counts -> cnt[d][tile]
//                  radix_scan   one workgroup per digit: tile offsets
//                               off[d][tile] = base[d] + sum of cnt[d][< tile]
//                  radix_scatter per tile: the stable rank of each key among
//                               the tile's keys of its digit, from wave ballots
//                               (8 ballots give a lane its peers of the same
//                               digit; lanes below it, the wave's earlier
//                               rounds, then the earlier waves) —
//                               dst[off[d][tile] + rank] = key (+ value).
//                  A skipped pass exits at once in all three kernels.
//                  (A one-launch pass with a decoupled look-back over the
//                  tiles' published counts measured 2x slower per pass here:
//                  the look-back is a chain of dependent cross-XCD loads.)
// Keys equal to ~0 (the grid producer's "not binned") may be excluded from
// the skip test of every pass but the last (skip_ones): such a key has digit
// 255 everywhere, and the last pass, never skipped while they exist, puts
// them after every other key; lower passes only order them among themselves.
// All counts are integers: the result is deterministic.
#include "common.h"
#include "radix.h"

namespace jabd {

constexpr int kRT = 256;                // threads per workgroup
constexpr int kRPer = 16;               // keys per thread
constexpr int kTile = kRT * kRPer;      // keys per tile
constexpr int kRWaves = kRT / 64;
constexpr int kWaveKeys = kTile / kRWaves;
constexpr int kMaxPass = 8;

__global__ __launch_bounds__(kRT) void radix_hist(const uint64_t* __restrict__ k, int64_t n, int lo,
                                                  int npass, int skip_ones,
                                                  int* __restrict__ ghist) {
  __shared__ int h[kMaxPass][256];
  const int t = threadIdx.x;
  for (int i = t; i < kMaxPass * 256; i += kRT) (&h[0][0])[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  for (int i = 0; i < kRPer; ++i) {
    const int64_t idx = base + (int64_t)i * kRT + t;
    if (idx >= n) break;
    const uint64_t key = k[idx];
    const bool ones = skip_ones && key == ~0ull;
    for (int p = ones ? npass - 1 : 0; p < npass; ++p)
      atomicAdd(&h[p][(int)((key >> (lo + 8 * p)) & 255u)], 1);
  }
  __syncthreads();
  for (int i = t; i < npass * 256; i += kRT) {
    const int v = (&h[0][0])[i];
    if (v) atomicAdd(&ghist[i], v);
  }
}

// inclusive wave scan (Hillis-Steele over the 64 lanes)
__device__ __forceinline__ int wave_incl_scan(int x) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (l >= o) x += y;
  }
  return x;
}

// exclusive block scan of one value per thread (kRT threads); returns the
// exclusive prefix, total in *tot
__device__ __forceinline__ int block_excl_scan(int x, int* tot) {
  __shared__ int ws[kRWaves];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int inc = wave_incl_scan(x);
  if (l == 63) ws[w] = inc;
  __syncthreads();
  int pre = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kRWaves; ++i) {
    const int s = ws[i];
    pre += i < w ? s : 0;
    all += s;
  }
  __syncthreads();
  *tot = all;
  return pre + inc - x;
}

// plan[p * kPlan]: [0..255] exclusive digit bases, [256] mode (0 skipped,
// 1 sorts, 2 copies), [257] source (0 input, 1 output, 2 alternate), [258]
// destination (1 output, 2 alternate).  One workgroup.
constexpr int kPlan = 260;
__global__ __launch_bounds__(kRT) void radix_plan(const int* __restrict__ ghist, int npass,
                                                  int* __restrict__ plan) {
  __shared__ int run[kMaxPass];
  const int t = threadIdx.x;
  for (int p = 0; p < npass; ++p) {
    const int v = ghist[p * 256 + t];
    int tot;
    const int ex = block_excl_scan(v, &tot);
    plan[p * kPlan + t] = ex;
    // one bin holds every key counted for this pass: nothing to reorder
    const int full = __syncthreads_or(v == tot && tot > 0);
    if (t == 0) run[p] = full ? 0 : 1;
    __syncthreads();
  }
  if (t == 0) {
    int m = 0;
    for (int p = 0; p < npass; ++p) m += run[p];
    if (m == 0) run[npass - 1] = 2;   // nothing to sort: the last pass copies
    // the passes that run alternate buffers backwards from the output
    int src = 0, left = m > 0 ? m : 1;
    for (int p = 0; p < npass; ++p) {
      plan[p * kPlan + 256] = run[p];
      if (!run[p]) continue;
      const int dst = ((left - 1) & 1) ? 2 : 1;
      plan[p * kPlan + 257] = src;
      plan[p * kPlan + 258] = dst;
      src = dst;
      --left;
    }
  }
}

__device__ __forceinline__ const uint64_t* rsel(int id, const uint64_t* a, const uint64_t* b,
                                                 const uint64_t* c) {
  return id == 0 ? a : (id == 1 ? b : c);
}

// per 4096-key tile: digit counts -> cnt[d][tile]
__global__ __launch_bounds__(kRT) void radix_count(const uint64_t* __restrict__ kin,
                                                   const uint64_t* __restrict__ kout,
                                                   const uint64_t* __restrict__ kalt, int64_t n,
                                                   int shift, const int* __restrict__ plan,
                                                   int ntiles, int* __restrict__ cnt) {
  if (plan[256] != 1) return;  // skipped or copy pass
  const uint64_t* k = rsel(plan[257], kin, kout, kalt);
  __shared__ int h[256];
  const int t = threadIdx.x;
  h[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  uint64_t v[kRPer];
#pragma unroll
  for (int i = 0; i < kRPer; ++i) {
    const int64_t idx = base + (int64_t)i * kRT + t;
    v[i] = idx < n ? k[idx] : 0ull;
  }
#pragma unroll
  for (int i = 0; i < kRPer; ++i) {
    const int64_t idx = base + (int64_t)i * kRT + t;
    if (idx < n) atomicAdd(&h[(int)((v[i] >> shift) & 255u)], 1);
  }
  __syncthreads();
  cnt[(int64_t)t * ntiles + blockIdx.x] = h[t];
}

// one workgroup per digit: off[d][tile] = base[d] + sum of cnt[d][< tile]
__global__ __launch_bounds__(kRT) void radix_scan(const int* __restrict__ cnt,
                                                  const int* __restrict__ plan, int ntiles,
                                                  int* __restrict__ off) {
  if (plan[256] != 1) return;
  const int d = blockIdx.x;
  int carry = plan[d];
  const int* c = cnt + (int64_t)d * ntiles;
  int* o = off + (int64_t)d * ntiles;
  for (int t0 = 0; t0 < ntiles; t0 += kRT) {
    const int i = t0 + threadIdx.x;
    const int x = i < ntiles ? c[i] : 0;
    int tot;
    const int ex = block_excl_scan(x, &tot);
    if (i < ntiles) o[i] = carry + ex;
    carry += tot;
  }
}

// per tile: stable rank of each key among the tile's keys of its digit (wave
// ballots), dst[off[d][tile] + rank] = key (+ value); a copy pass copies
template <bool VALS>
__global__ __launch_bounds__(kRT) void radix_scatter(
    const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout, uint64_t* __restrict__ kalt,
    const int* __restrict__ vin, int* __restrict__ vout, int* __restrict__ valt, int64_t n,
    int shift, const int* __restrict__ plan, const int* __restrict__ off, int ntiles) {
  const int mode = plan[256];
  if (mode == 0) return;
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int sid = plan[257], did = plan[258];
  const uint64_t* ks = rsel(sid, kin, kout, kalt);
  const int* vs = sid == 0 ? vin : (sid == 1 ? vout : valt);
  uint64_t* kd = did == 1 ? kout : kalt;
  int* vd = did == 1 ? vout : valt;
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)w * kWaveKeys;
  if (mode == 2) {
    for (int r = 0; r < kWaveKeys / 64; ++r) {
      const int64_t idx = base + r * 64 + l;
      if (idx < n) {
        kd[idx] = ks[idx];
        if (VALS) vd[idx] = vs[idx];
      }
    }
    return;
  }
  __shared__ int wc[kRWaves][256];   // running count per (wave, digit), then wave prefix
  __shared__ int tb[256];            // this tile's offset per digit
#pragma unroll
  for (int i = 0; i < kRWaves; ++i) wc[i][t] = 0;
  tb[t] = off[(int64_t)t * ntiles + blockIdx.x];
  __syncthreads();
  constexpr int R = kWaveKeys / 64;
  uint64_t key[R];
  int val[R], rk[R], dg[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t idx = base + r * 64 + l;
    const bool ok = idx < n;
    key[r] = ok ? ks[idx] : 0ull;
    val[r] = (VALS && ok) ? vs[idx] : 0;
  }
  const uint64_t lt = (1ull << l) - 1ull;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t idx = base + r * 64 + l;
    const bool ok = idx < n;
    const int d = (int)((key[r] >> shift) & 255u);
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t m = __ballot((d >> b) & 1);
      peers &= ((d >> b) & 1) ? m : ~m;
    }
    const int below = __popcll(peers & lt);
    const int prev = wc[w][d];           // every lane reads before the leader writes
    dg[r] = d;
    rk[r] = prev + below;
    if (ok && below == 0) wc[w][d] = prev + __popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  {
    int s = 0;
#pragma unroll
    for (int i = 0; i < kRWaves; ++i) {
      const int c = wc[i][t];
      wc[i][t] = s;
      s += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t idx = base + r * 64 + l;
    if (idx >= n) continue;
    const int64_t dst = (int64_t)tb[dg[r]] + wc[w][dg[r]] + rk[r];
    kd[dst] = key[r];
    if (VALS) vd[dst] = val[r];
  }
}

// ---------------------------------------------------------------- small sorts
// n <= kSmallMax (the bs1 predict's NMS keys: 16.8k at 640^2): the whole
// sort in one 1024-thread workgroup — every pass's histogram in one sweep,
// then per pass the tiles of 16 waves x 512 keys in order, each key's
// stable rank among its tile's keys of its digit from wave ballots (as
// radix_scatter), the tile's digit offsets from a running count in LDS.  One
// launch instead of 2 + 3 per pass: at this size every kernel of the
// multi-workgroup sort is a few microseconds of launch and drain.  The
// passes' reads see the previous pass's stores after the barrier: one
// workgroup is one CU, whose vector L1 its own stores write through.
constexpr int kST = 1024, kSWaves = kST / 64, kSR = 8;
constexpr int kSTile = kST * kSR;  // keys per tile
constexpr int kSmallMax = 4 * kSTile;

template <bool VALS>
__global__ __launch_bounds__(kST) void radix_small(const uint64_t* __restrict__ kin,
                                                   uint64_t* __restrict__ kout,
                                                   uint64_t* __restrict__ kalt,
                                                   const int* __restrict__ vin,
                                                   int* __restrict__ vout, int* __restrict__ valt,
                                                   int n, int lo, int npass, int skip_ones,
                                                   const int* __restrict__ n_dev) {
  __shared__ int hist[kMaxPass][256];
  __shared__ int wc[kSWaves][256];
  __shared__ int run[256];
  __shared__ int wsum[4];
  __shared__ int nones;
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  if (n_dev) {  // device-side count: the keys past it are ~0 in the output
    const int nd = *n_dev;
    const int nc = nd < n ? (nd > 0 ? nd : 0) : n;
    for (int i = nc + t; i < n; i += kST) kout[i] = ~0ull;
    n = nc;
  }
  for (int i = t; i < kMaxPass * 256; i += kST) (&hist[0][0])[i] = 0;
  if (t == 0) nones = 0;
  __syncthreads();
  for (int i0 = 0; i0 < n; i0 += kST) {   // wave-uniform trip count (ballots inside)
    const int i = i0 + t;
    const bool ok = i < n;
    const uint64_t key = ok ? kin[i] : 0ull;
    const bool ones = ok && skip_ones && key == ~0ull;
    if (ones) atomicAdd(&nones, 1);
    for (int p = 0; p < npass; ++p) {
      const bool cnt = ok && (!ones || p == npass - 1);
      const int d = (int)((key >> (lo + 8 * p)) & 255u);
      // a digit shared by every counted lane (the high bytes of the scores)
      // is one add instead of 64 serialised LDS atomics on one address
      const uint64_t act = __ballot(cnt);
      const int d0 = __shfl(d, act ? __ffsll((unsigned long long)act) - 1 : 0);
      if (act && __ballot(cnt && d != d0) == 0) {
        if (l == __ffsll((unsigned long long)act) - 1) atomicAdd(&hist[p][d0], __popcll(act));
      } else if (cnt) {
        atomicAdd(&hist[p][d], 1);
      }
    }
  }
  __syncthreads();
  // passes that reorder anything (one bin holding every counted key: skipped)
  unsigned runmask = 0;
  for (int p = 0; p < npass; ++p) {
    const int tot = p == npass - 1 ? n : n - nones;
    const int full = __syncthreads_or(t < 256 && tot > 0 && hist[p][t] == tot);
    if (!full) runmask |= 1u << p;
  }
  const int m = __popc(runmask);
  if (m == 0) {
    for (int i = t; i < n; i += kST) {
      kout[i] = kin[i];
      if (VALS) vout[i] = vin[i];
    }
    return;
  }
  const uint64_t lt = (1ull << l) - 1ull;
  const uint64_t* ks = kin;
  const int* vs = vin;
  int left = m;
  for (int p = 0; p < npass; ++p) {
    if (!((runmask >> p) & 1u)) continue;
    uint64_t* kd = ((left - 1) & 1) ? kalt : kout;
    int* vd = ((left - 1) & 1) ? valt : vout;
    --left;
    const int shift = lo + 8 * p;
    // digit bases: exclusive prefix of this pass's histogram (waves 0-3)
    if (t < 256) {
      const int v = hist[p][t];
      int x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (l >= o) x += y;
      }
      if (l == 63) wsum[w] = x;
      run[t] = x - v;
    }
    __syncthreads();
    if (t < 256) {
      int add = 0;
      for (int i = 0; i < w; ++i) add += wsum[i];
      run[t] += add;
    }
    for (int tile0 = 0; tile0 < n; tile0 += kSTile) {
      for (int i = t; i < kSWaves * 256; i += kST) (&wc[0][0])[i] = 0;
      __syncthreads();
      uint64_t key[kSR];
      int val[kSR], rk[kSR], dg[kSR];
      const int base = tile0 + w * (kSTile / kSWaves);
#pragma unroll
      for (int r = 0; r < kSR; ++r) {
        const int idx = base + r * 64 + l;
        const bool ok = idx < n;
        key[r] = ok ? ks[idx] : 0ull;
        val[r] = (VALS && ok) ? vs[idx] : 0;
      }
#pragma unroll
      for (int r = 0; r < kSR; ++r) {
        const bool ok = base + r * 64 + l < n;
        const int d = (int)((key[r] >> shift) & 255u);
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const uint64_t mb = __ballot((d >> b) & 1);
          peers &= ((d >> b) & 1) ? mb : ~mb;
        }
        const int below = __popcll(peers & lt);
        const int prev = wc[w][d];
        dg[r] = d;
        rk[r] = prev + below;
        if (ok && below == 0) wc[w][d] = prev + __popcll(peers);
        __builtin_amdgcn_wave_barrier();
      }
      __syncthreads();
      if (t < 256) {  // tile offsets per (wave, digit); run[] moves past the tile
        int s = run[t];
#pragma unroll
        for (int i = 0; i < kSWaves; ++i) {
          const int c = wc[i][t];
          wc[i][t] = s;
          s += c;
        }
        run[t] = s;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kSR; ++r) {
        if (base + r * 64 + l >= n) continue;
        const int dst = wc[w][dg[r]] + rk[r];
        kd[dst] = key[r];
        if (VALS) vd[dst] = val[r];
      }
      __syncthreads();
    }
    ks = kd;
    vs = vd;
  }
}

// ---------------------------------------------------------------- exclusive int32 scan
__global__ __launch_bounds__(kRT) void scan_reduce(const int* __restrict__ in, int64_t n,
                                                   int* __restrict__ bsum) {
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kRPer;
  int s = 0;
#pragma unroll
  for (int i = 0; i < kRPer; ++i)
    if (base + i < n) s += in[base + i];
  int tot;
  (void)block_excl_scan(s, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kRT) void scan_top(int* __restrict__ bsum, int nblk) {
  int carry = 0;
  for (int b0 = 0; b0 < nblk; b0 += kRT) {
    const int i = b0 + threadIdx.x;
    const int x = i < nblk ? bsum[i] : 0;
    int tot;
    const int ex = block_excl_scan(x, &tot);
    if (i < nblk) bsum[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(kRT) void scan_down(const int* __restrict__ in, int64_t n,
                                                 const int* __restrict__ bsum,
                                                 int* __restrict__ out) {
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kRPer;
  int v[kRPer];
  int s = 0;
#pragma unroll
  for (int i = 0; i < kRPer; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  int tot;
  int run = block_excl_scan(s, &tot) + bsum[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kRPer; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
}

// ---------------------------------------------------------------- host side
static int radix_ntiles(int64_t n) { return (int)cdiv(n > 0 ? n : 1, kTile); }

template <typename A>
static void carve_radix(A& a, int64_t n, bool vals, RadixWs* w) {
  const int nt = radix_ntiles(n);
  auto* gh = a.template take<int>(kMaxPass * 256);
  auto* pl = a.template take<int>(kMaxPass * kPlan);
  auto* cn = a.template take<int>((size_t)256 * nt);
  auto* of = a.template take<int>((size_t)256 * nt);
  auto* ka = a.template take<uint64_t>((size_t)n);
  auto* va = vals ? a.template take<int>((size_t)n) : nullptr;
  if (w) {
    w->ghist = gh;
    w->plan = pl;
    w->cnt = cn;
    w->off = of;
    w->kalt = ka;
    w->valt = va;
  }
}

// JABD_RADIX_SMALL=0: every size takes the multi-workgroup passes (A/B)
static bool radix_small_off() {
  static const bool off = [] {
    const char* e = getenv("JABD_RADIX_SMALL");
    return e && e[0] == '0';
  }();
  return off;
}

size_t radix_ws_bytes(int64_t n, bool vals) {
  Sizer s;
  carve_radix(s, n, vals, (RadixWs*)nullptr);
  return s.used;
}

int radix_sort64(const uint64_t* kin, uint64_t* kout, const int* vin, int* vout, int64_t n,
                 int lo, int npass, bool skip_ones, void* ws, size_t ws_bytes, hipStream_t st) {
  JABD_REQUIRE(npass >= 1 && npass <= kMaxPass && lo >= 0 && lo + 8 * npass <= 64,
               "radix_sort64: bits [%d, %d)", lo, lo + 8 * npass);
  JABD_REQUIRE(n >= 0 && n < ((int64_t)1 << 30), "radix_sort64: n = %lld", (long long)n);
  JABD_REQUIRE((vin == nullptr) == (vout == nullptr), "radix_sort64: values in and out");
  if (n == 0) return JABD_OK;
  const bool vals = vin != nullptr;
  JABD_REQUIRE(ws_bytes >= radix_ws_bytes(n, vals), "radix_sort64: workspace");
  Carve cv(ws, ws_bytes);
  RadixWs w;
  carve_radix(cv, n, vals, &w);
  if (n <= kSmallMax && !radix_small_off()) {
    if (vals)
      radix_small<true><<<1, kST, 0, st>>>(kin, kout, w.kalt, vin, vout, w.valt, (int)n, lo, npass,
                                           skip_ones ? 1 : 0, nullptr);
    else
      radix_small<false><<<1, kST, 0, st>>>(kin, kout, w.kalt, nullptr, nullptr, nullptr, (int)n,
                                            lo, npass, skip_ones ? 1 : 0, nullptr);
    return check_launch("radix_small");
  }
  const int nt = radix_ntiles(n);
  {
    const FillRange fr{w.ghist, (int64_t)sizeof(int) * kMaxPass * 256, 0u};
    if (int e = fill_ranges(&fr, 1, st)) return e;
  }
  radix_hist<<<nt, kRT, 0, st>>>(kin, n, lo, npass, skip_ones ? 1 : 0, w.ghist);
  radix_plan<<<1, kRT, 0, st>>>(w.ghist, npass, w.plan);
  if (int e = check_launch("radix_hist/plan")) return e;
  for (int p = 0; p < npass; ++p) {
    const int* pl = w.plan + p * kPlan;
    const int sh = lo + 8 * p;
    radix_count<<<nt, kRT, 0, st>>>(kin, kout, w.kalt, n, sh, pl, nt, w.cnt);
    radix_scan<<<256, kRT, 0, st>>>(w.cnt, pl, nt, w.off);
    if (vals)
      radix_scatter<true><<<nt, kRT, 0, st>>>(kin, kout, w.kalt, vin, vout, w.valt, n, sh, pl,
                                               w.off, nt);
    else
      radix_scatter<false><<<nt, kRT, 0, st>>>(kin, kout, w.kalt, nullptr, nullptr, nullptr, n,
                                                sh, pl, w.off, nt);
    if (int e = check_launch("radix pass")) return e;
  }
  return JABD_OK;
}

int64_t radix_small_max() { return radix_small_off() ? 0 : kSmallMax; }

int radix_sort64_devn(const uint64_t* kin, uint64_t* kout, const int* n_dev, int64_t n_cap,
                      int lo, int npass, void* ws, size_t ws_bytes, hipStream_t st) {
  JABD_REQUIRE(npass >= 1 && npass <= kMaxPass && lo >= 0 && lo + 8 * npass <= 64,
               "radix_sort64_devn: bits [%d, %d)", lo, lo + 8 * npass);
  JABD_REQUIRE(n_cap > 0 && n_cap <= kSmallMax && n_dev, "radix_sort64_devn: n_cap %lld",
               (long long)n_cap);
  if (radix_small_off()) return -1;
  JABD_REQUIRE(ws_bytes >= radix_ws_bytes(n_cap, false), "radix_sort64_devn: workspace");
  Carve cv(ws, ws_bytes);
  RadixWs w;
  carve_radix(cv, n_cap, false, &w);
  radix_small<false><<<1, kST, 0, st>>>(kin, kout, w.kalt, nullptr, nullptr, nullptr, (int)n_cap,
                                        lo, npass, 0, n_dev);
  return check_launch("radix_small (device count)");
}

size_t scan_ws_bytes(int64_t n) { return align_up(sizeof(int) * (size_t)cdiv(n > 0 ? n : 1, kTile)); }

int scan_excl_i32(const int* in, int* out, int64_t n, void* ws, size_t ws_bytes, hipStream_t st) {
  if (n <= 0) return JABD_OK;
  JABD_REQUIRE(ws_bytes >= scan_ws_bytes(n), "scan_excl_i32: workspace");
  const int nblk = (int)cdiv(n, kTile);
  int* bsum = static_cast<int*>(ws);
  scan_reduce<<<nblk, kRT, 0, st>>>(in, n, bsum);
  scan_top<<<1, kRT, 0, st>>>(bsum, nblk);
  scan_down<<<nblk, kRT, 0, st>>>(in, n, bsum, out);
  return check_launch("scan_excl_i32");
}

}  // namespace jabd

using namespace jabd;

extern "C" int jabd_sort_workspace_size(int64_t n, int32_t with_values, size_t* bytes) {
  JABD_REQUIRE(bytes && n >= 0, "sort_workspace_size: bad args");
  *bytes = radix_ws_bytes(n, with_values != 0);
  return JABD_OK;
}

extern "C" int jabd_sort_u64(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* vals_in,
                             int32_t* vals_out, int64_t n, int32_t bit_lo, int32_t npass,
                             int32_t skip_ones, void* ws, size_t ws_bytes, jabd_stream_t stream) {
  JABD_REQUIRE(n == 0 || (keys_in && keys_out && ws), "sort_u64: null pointer");
  JABD_REQUIRE(keys_in != keys_out && (!vals_in || vals_in != vals_out), "sort_u64: aliasing");
  return radix_sort64(keys_in, keys_out, vals_in, vals_out, n, bit_lo, npass, skip_ones != 0, ws,
                      ws_bytes, as_stream(stream));
}

extern "C" int jabd_scan_workspace_size(int64_t n, size_t* bytes) {
  JABD_REQUIRE(bytes && n >= 0, "scan_workspace_size: bad args");
  *bytes = scan_ws_bytes(n);
  return JABD_OK;
}

extern "C" int jabd_scan_excl_i32(const int32_t* in, int32_t* out, int64_t n, void* ws,
                                  size_t ws_bytes, jabd_stream_t stream) {
  JABD_REQUIRE(n == 0 || (in && out && ws), "scan_excl_i32: null pointer");
  return scan_excl_i32(in, out, n, ws, ws_bytes, as_stream(stream));
}
