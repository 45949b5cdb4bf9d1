// Outlier stage on the GPU (/root/reference/
// CommunityDetection/Graphframes.py:92-137).
//
// L1  size[l]   = |{v : L[v] = l}|                               (:100-104, :120)
//     inc[l]    = |{distinct (s,d) : L[s] = l or L[d] = l}|      (:107-118)
//     threshold rule over the community sizes, flag members of small communities
// L2  E' = distinct (s,d) with L[s] = L[d]; L' = LPA-DET(E', sub_iter)   (:121-128)
//     per community: threshold rule over its sub-label sizes     (:130-137)
//
// Threshold rule (App. B a13): groups sorted by (size desc, label asc),
// k = n // 10, thr = sorted[-k].size if k > 0 else sorted[0].size, i.e. the
// k-th smallest size (k > 0) or the largest; a group is an outlier iff size < thr.
// Per segment (community) it is computed by one radix sort of (segment << 32 | size)
// keys, after which the k-th smallest sits at segment_start + k - 1.
//
// A sub-label L'[v] is the id of a vertex of v's own community (E' never
// crosses communities), so the group (L[v], L'[v]) is identified by L'[v] alone
// and its community is L[L'[v]].
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "lpa_device.h"

namespace lpa {

int create_l2(const lpa_graph* parent, const int32_t* L, const uint8_t* marks, lpa_graph** out);
void destroy(lpa_graph* g);

namespace {

inline unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  if (b > 65536) b = 65536;
  return (unsigned)b;
}

// block-aggregated histograms: few blocks, each over a long stretch of the input
inline unsigned grid_bh(int64_t n) {
  const unsigned g = grid_for(n);
  return g < 2048u ? g : 2048u;
}
inline unsigned grid_cnt(int64_t n) {
  const unsigned g = grid_for(n);
  return g < 4096u ? g : 4096u;
}

#define GRID_STRIDE(i, n) \
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)
// uniform variant: every lane of a wave runs every trip (wave-level ballots inside);
// `act` says whether this lane holds an element
#define GRID_STRIDE_UNIFORM_BEGIN(i, act, n)                                         \
  for (int64_t i##_b = (int64_t)blockIdx.x * blockDim.x; i##_b < (n);                \
       i##_b += (int64_t)gridDim.x * blockDim.x) {                                   \
    const int64_t i = i##_b + threadIdx.x;                                           \
    const bool act = i < (n);

__global__ void k_edge_keys(const int32_t* __restrict__ s, const int32_t* __restrict__ d, int64_t m,
                            u64* __restrict__ k) {
  GRID_STRIDE(e, m) k[e] = ((u64)(u32)s[e] << 32) | (u32)d[e];
}

// first occurrence of each key of a sorted array (the distinct directed edges)
__global__ void k_mark_first(const u64* __restrict__ k, int64_t n, int32_t* __restrict__ mark) {
  GRID_STRIDE(i, n) mark[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

__global__ void k_compact_marked(const u64* __restrict__ k, const int32_t* __restrict__ mark,
                                 const int64_t* __restrict__ pos, int64_t n, u64* __restrict__ out) {
  GRID_STRIDE(i, n) if (mark[i]) out[pos[i]] = k[i];
}

// size[l] = members of community l; labels outside [0, V) are counted in *bad and
// skipped (reported after the final sync instead of a host round trip up front)
// (block-aggregated: the giant communities of a converged labelling took one device
// atomic per wave on the same counter, 7.5 ms at R-MAT-24)
__global__ __launch_bounds__(256) void k_histogram(const int32_t* __restrict__ lab, int64_t V,
                                                   int32_t* __restrict__ hist,
                                                   unsigned long long* __restrict__ bad) {
  __shared__ u32 bk[dev::kBhSlots];
  __shared__ int32_t bv[dev::kBhSlots];
  __shared__ int bsat;
  dev::BlockHist<int32_t> bh{bk, bv, &bsat};
  bh.init();
  const int lane = threadIdx.x & 63;
  GRID_STRIDE_UNIFORM_BEGIN(v, act, V)
    u32 l = act ? (u32)lab[v] : 0u;
    const bool oob = act && l >= (u32)V;
    if (oob) atomicAdd(bad, 1ull);
    bh.add1(hist, act && !oob, l, lane);
  }
  bh.flush(hist);
}

// incident distinct edges per community, over the sorted edge keys (distinct =
// first occurrences): +1 for L[s], +1 for L[d] when it differs
// (ek: the distinct directed edges); kMark (L2): also the edge's intra-community mark,
// the E' filter of the sub-graph build (the same two label reads)
template <bool kMark>
__global__ __launch_bounds__(256) void k_incident(const u64* __restrict__ ek, int64_t n,
                                                  const int32_t* __restrict__ L, int64_t nv,
                                                  int32_t* __restrict__ inc, uint8_t* __restrict__ mark) {
  __shared__ u32 bk[dev::kBhSlots];
  __shared__ int32_t bv[dev::kBhSlots];
  __shared__ int bsat;
  dev::BlockHist<int32_t> bh{bk, bv, &bsat};
  bh.init();
  const int lane = threadIdx.x & 63;
  GRID_STRIDE_UNIFORM_BEGIN(i, act, n)
    const bool a = act;
    u32 ls = 0u, ld = 0u;
    if (a) {
      const u64 k = ek[i];
      ls = (u32)L[(int32_t)(k >> 32)];
      ld = (u32)L[(int32_t)(u32)k];
    }
    const u32 V = (u32)nv;   // out-of-range labels (reported by k_histogram) are skipped
    if (kMark && a) mark[i] = ls == ld ? 1 : 0;
    bh.add1(inc, a && ls < V, ls, lane);
    bh.add1(inc, a && ld != ls && ld < V, ld, lane);
  }
  bh.flush(inc);
}

// the distinct edges in (d, s) order: keys (d << 32 | i) generated in de_keys order,
// where i ascends with s for a fixed d, so a stable sort on the d bits alone gives (d, s)
__global__ void k_t_keys(const u64* __restrict__ ek, int64_t n, u64* __restrict__ t) {
  GRID_STRIDE(i, n) t[i] = ((u64)(u32)ek[i] << 32) | (u64)i;
}
__global__ void k_t_src(const u64* __restrict__ ek, const u64* __restrict__ t, int64_t n, uint32_t* __restrict__ ts) {
  GRID_STRIDE(j, n) ts[j] = (uint32_t)(ek[(u32)t[j]] >> 32);
}
// first index of every vertex's run in keys sorted by their high 32 bits ([V + 1]):
// off[v] = lower_bound(v) by a binary search per vertex, so a long run of edgeless
// vertices costs no thread a serial fill (neighbouring vertices walk the same upper
// levels of the search, which stay cached)
__global__ void k_run_offsets(const u64* __restrict__ k, int64_t n, int64_t V, int64_t* __restrict__ off) {
  GRID_STRIDE(v, V + 1) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = lo + ((hi - lo) >> 1);
      if ((int64_t)(k[mid] >> 32) < v) lo = mid + 1;
      else hi = mid;
    }
    off[v] = lo;
  }
}

// group keys (segment << 32 | size) for every label l: size[l] > 0 -> a group of
// segment seg_of[l] (nullptr: one segment); size 0 -> the sentinel segment nseg,
// which the sort moves behind every group (no compaction, no host count)
__global__ void k_group_keys(const int32_t* __restrict__ size, const int32_t* __restrict__ seg_of,
                             int64_t V, u32 nseg, u64* __restrict__ keys) {
  GRID_STRIDE(l, V) {
    u32 sg = size[l] > 0 ? (seg_of ? (u32)seg_of[l] : 0u) : nseg;
    if (sg > nseg) sg = nseg;   // out-of-range community label (reported separately)
    keys[l] = ((u64)sg << 32) | (u32)size[l];
  }
}

// per segment: first / last index in the sorted group keys
__global__ void k_seg_bounds(const u64* __restrict__ keys, int64_t n, u32 nseg, int32_t* __restrict__ first,
                             int32_t* __restrict__ last, unsigned long long* __restrict__ ngroups) {
  GRID_STRIDE(i, n) {
    const u32 sg = (u32)(keys[i] >> 32);
    if (sg == nseg) continue;
    if (i == 0 || (u32)(keys[i - 1] >> 32) != sg) first[sg] = (int32_t)i;
    if (i == n - 1 || (u32)(keys[i + 1] >> 32) != sg) {
      last[sg] = (int32_t)i;
      if (i == n - 1 || (u32)(keys[i + 1] >> 32) == nseg) *ngroups = (unsigned long long)(i + 1);
    }
  }
}

// threshold per segment present in the keys (App. B a13: the k-th smallest size,
// k = groups / 10, or the largest when k == 0)
__global__ void k_seg_threshold(const u64* __restrict__ keys, int64_t n, u32 nseg,
                                const int32_t* __restrict__ first, const int32_t* __restrict__ last,
                                int32_t* __restrict__ thr) {
  GRID_STRIDE(i, n) {
    const u32 sg = (u32)(keys[i] >> 32);
    if (sg == nseg || first[sg] != (int32_t)i) continue;
    const int64_t cnt = (int64_t)last[sg] - first[sg] + 1;
    const int64_t k = cnt / 10;
    const int64_t at = k > 0 ? first[sg] + k - 1 : last[sg];
    thr[sg] = (int32_t)(u32)keys[at];
  }
}

// flags[v] = size(group of v) < thr(segment of v); flagged count (one atomic per wave)
__global__ __launch_bounds__(256) void k_flag(const int32_t* __restrict__ group_of,
                                              const int32_t* __restrict__ size,
                                              const int32_t* __restrict__ seg_of_v,
                                              const int32_t* __restrict__ thr, int64_t V,
                                              uint8_t* __restrict__ flags, int32_t* __restrict__ seg_flagged,
                                              unsigned long long* __restrict__ nflag) {
  const int lane = threadIdx.x & 63;
  GRID_STRIDE_UNIFORM_BEGIN(v, act, V)
    uint8_t f = 0;
    if (act) {
      const u32 gph = (u32)group_of[v];
      const u32 sg = seg_of_v ? (u32)seg_of_v[v] : 0u;
      if (gph < (u32)V && sg < (u32)V) {   // else: a bad label, reported by k_histogram
        f = size[gph] < thr[sg] ? 1 : 0;
        if (f) seg_flagged[sg] = 1;
      }
      flags[v] = f;
    }
    const u64 fm = __ballot(f != 0);
    if (lane == 0 && fm) atomicAdd(nflag, (unsigned long long)__popcll(fm));
  }
}

// one device atomic per block (per wave, 4 M same-address atomics took 3-6 ms)
__global__ __launch_bounds__(256) void k_count_nonzero(const int32_t* __restrict__ a, int64_t n,
                                                       unsigned long long* out) {
  __shared__ unsigned long long ws[4];
  unsigned long long c = 0;
  GRID_STRIDE(i, n) c += a[i] != 0;
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    c = ws[0] + ws[1] + ws[2] + ws[3];
    if (c) atomicAdd(out, c);
  }
}

__global__ void k_widen(const int32_t* __restrict__ a, int64_t n, int64_t* __restrict__ out) {
  GRID_STRIDE(i, n) out[i] = a[i];
}

struct Scratch {
  hipStream_t s;
  void* ptrs[32];
  int n = 0;
  explicit Scratch(hipStream_t st) : s(st) {}
  template <typename T>
  int get(T** p, int64_t count) {
    if (count < 1) count = 1;
    if (tmp_alloc((void**)p, sizeof(T) * count, s) != LPA_OK) {
      set_error("outlier: out of device memory (%lld x %zu B)", (long long)count, sizeof(T));
      return LPA_ENOMEM;
    }
    ptrs[n++] = *p;
    return LPA_OK;
  }
  ~Scratch() {
    for (int i = 0; i < n; ++i) tmp_free(ptrs[i], s);
  }
};

int sort_keys(u64* keys, u64* tmp, int64_t n, int bits_lo, int bits_hi, hipStream_t s) {
  int shifts[16], ns = 0;
  for (int b = 0; b < bits_lo; b += 8) shifts[ns++] = b;
  for (int b = 0; b < bits_hi; b += 8) shifts[ns++] = 32 + b;
  return radix_sort_u64(keys, tmp, n, shifts, ns, s);
}

// The handle's distinct directed edges as sorted (s << 32 | d) keys, g->de_keys[0,
// g->de_n): sort, mark first occurrences, compact.  Built by the first outlier call
// and kept with the handle: it is topology (label-independent), like the CSR, and
// its sort is most of an L1 call otherwise (20 ms of 55 at R-MAT-24).
int distinct_edges(lpa_graph* g) {
  if (g->de_n >= 0) return LPA_OK;
  hipStream_t s = g->stream;
  const int64_t m = g->m;
  if (m == 0) {
    g->de_n = 0;
    return LPA_OK;
  }
  Scratch sc(s);
  u64* keys = nullptr;
  int32_t* first = nullptr;
  int64_t* pos = nullptr;
  LPA_TRY(sc.get(&keys, 2 * m));
  LPA_TRY(sc.get(&first, m));
  LPA_TRY(sc.get(&pos, m + 1));
  hipLaunchKernelGGL(k_edge_keys, dim3(grid_for(m)), dim3(256), 0, s, g->e_src, g->e_dst, m, keys);
  LPA_HIP(hipGetLastError());
  const int b = bits_for((uint64_t)(g->V > 0 ? g->V - 1 : 0));
  LPA_TRY(sort_keys(keys, keys + m, m, b, b, s));
  hipLaunchKernelGGL(k_mark_first, dim3(grid_for(m)), dim3(256), 0, s, keys, m, first);
  LPA_HIP(hipGetLastError());
  LPA_TRY(exclusive_scan_i32_i64(first, pos, m, s));
  int64_t n = 0;
  LPA_HIP(hipMemcpyAsync(&n, pos + m, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  LPA_TRY(dev_alloc(g, (void**)&g->de_keys, sizeof(u64) * (n > 0 ? n : 1)));
  hipLaunchKernelGGL(k_compact_marked, dim3(grid_for(m)), dim3(256), 0, s, keys, first, pos, m, g->de_keys);
  LPA_HIP(hipGetLastError());
  LPA_HIP(hipStreamSynchronize(s));   // the scratch is freed on return
  g->de_n = n;
  return LPA_OK;
}

// The distinct edges in (d, s) order (de_t, de_ts) and both orders' per-vertex run
// offsets: what the L2 sub-graph build filters (build_graph_l2).  Built by the first L2
// call and kept with the handle (topology, like de_keys).
int transposed_edges(lpa_graph* g) {
  if (g->de_t) return LPA_OK;
  hipStream_t s = g->stream;
  const int64_t md = g->de_n, V = g->V;
  LPA_TRY(dev_alloc(g, (void**)&g->de_out_off, sizeof(int64_t) * (V + 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->de_in_off, sizeof(int64_t) * (V + 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->de_ts, sizeof(uint32_t) * (md > 0 ? md : 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->de_t, sizeof(u64) * (md > 0 ? md : 1)));
  if (md > 0) {
    Scratch sc(s);
    u64* tmp = nullptr;
    LPA_TRY(sc.get(&tmp, md));
    hipLaunchKernelGGL(k_t_keys, dim3(grid_for(md)), dim3(256), 0, s, g->de_keys, md, g->de_t);
    LPA_HIP(hipGetLastError());
    int shifts[8], ns = 0;
    for (int b = 0; b < bits_for((uint64_t)(V > 0 ? V - 1 : 0)); b += 8) shifts[ns++] = 32 + b;
    LPA_TRY(radix_sort_u64(g->de_t, tmp, md, shifts, ns, s));
    hipLaunchKernelGGL(k_t_src, dim3(grid_for(md)), dim3(256), 0, s, g->de_keys, g->de_t, md, g->de_ts);
    LPA_HIP(hipGetLastError());
    LPA_HIP(hipStreamSynchronize(s));   // the scratch is freed on return
  }
  hipLaunchKernelGGL(k_run_offsets, dim3(grid_for(V + 1)), dim3(256), 0, s, g->de_keys, md, V,
                     g->de_out_off);
  hipLaunchKernelGGL(k_run_offsets, dim3(grid_for(V + 1)), dim3(256), 0, s, g->de_t, md, V,
                     g->de_in_off);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// groups = labels l with size[l] > 0, segment seg_of[l] (nullptr: one segment).
// Per-segment thresholds into thr[]; the group count lands in *ngroups (device).
// No host round trip: empty labels sort behind the groups as a sentinel segment.
int segmented_threshold(lpa_graph* g, Scratch& sc, const int32_t* size, const int32_t* seg_of,
                        int64_t V, int32_t* thr, unsigned long long* ngroups) {
  hipStream_t s = g->stream;
  u64* keys = nullptr;
  int32_t *first = nullptr, *last = nullptr;
  LPA_TRY(sc.get(&keys, 2 * V));
  LPA_TRY(sc.get(&first, V + 1));
  LPA_TRY(sc.get(&last, V + 1));
  const u32 nseg = seg_of ? (u32)V : 1u;
  hipLaunchKernelGGL(k_group_keys, dim3(grid_for(V)), dim3(256), 0, s, size, seg_of, V, nseg, keys);
  LPA_HIP(hipGetLastError());
  LPA_TRY(sort_keys(keys, keys + V, V, bits_for((uint64_t)V), bits_for((uint64_t)nseg), s));
  hipLaunchKernelGGL(k_seg_bounds, dim3(grid_for(V)), dim3(256), 0, s, keys, V, nseg, first, last, ngroups);
  LPA_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_seg_threshold, dim3(grid_for(V)), dim3(256), 0, s, keys, V, nseg, first, last, thr);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// Host side of the host-array interface: copies between the caller's (pageable)
// arrays and a pinned staging area kept with the handle, split over threads (a
// single-threaded copy of ~10^8 bytes is bound by the destination's first-touch page
// faults; pageable hipMemcpy staged the same bytes through one thread).
void par_copy(void* dst, const void* src, size_t n) {
  const size_t kMin = size_t(8) << 20;
  const int T = (int)std::min<size_t>(16, n / kMin);
  if (T <= 1) {
    memcpy(dst, src, n);
    return;
  }
  // no exception crosses the C ABI: a piece whose thread cannot be started (or
  // recorded) is copied by this thread
  std::vector<std::thread> th;
  const size_t step = (n + T - 1) / T;
  try {
    th.reserve((size_t)T);
  } catch (...) {
    memcpy(dst, src, n);
    return;
  }
  for (int t = 0; t < T; ++t) {
    const size_t a = (size_t)t * step;
    if (a >= n) break;
    const size_t b = std::min(n, a + step);
    try {
      th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
    } catch (...) {
      memcpy((char*)dst + a, (const char*)src + a, b - a);
    }
  }
  for (auto& x : th) x.join();
}

int ensure_pin(lpa_graph* g, size_t bytes) {
  if (g->host_pin_bytes >= bytes) return LPA_OK;
  if (g->host_pin) (void)hipHostFree(g->host_pin);
  g->host_pin = nullptr;
  g->host_pin_bytes = 0;
  LPA_HIP(hipHostMalloc(&g->host_pin, bytes, hipHostMallocDefault));
  g->host_pin_bytes = bytes;
  return LPA_OK;
}

int bad_labels(unsigned long long n, int64_t V) {
  set_error("outlier: %llu labels outside [0, V=%lld)", n, (long long)V);
  return LPA_EINVAL;
}

// ---- partition quality (lpa_quality): modularity on the symmetrised multigraph ----
// arcs inside a community: 2 per input edge with L[s] == L[d] (a self-loop's two arcs)
__global__ __launch_bounds__(256) void k_q_intra(const int32_t* __restrict__ s, const int32_t* __restrict__ d,
                                                 int64_t m, const int32_t* __restrict__ L, int64_t V,
                                                 unsigned long long* __restrict__ acc) {
  unsigned long long c = 0;
  GRID_STRIDE(e, m) {
    const u32 a = (u32)L[s[e]], b = (u32)L[d[e]];
    c += (a == b && a < (u32)V) ? 2ull : 0ull;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(acc, c);
}
// D[l] += deg(v) for L[v] = l (out-of-range labels counted in *bad)
__global__ __launch_bounds__(256) void k_q_degsum(const int32_t* __restrict__ L, const int32_t* __restrict__ deg,
                                                  int64_t V, unsigned long long* __restrict__ D,
                                                  unsigned long long* __restrict__ bad) {
  GRID_STRIDE(v, V) {
    const u32 l = (u32)L[v];
    if (l < (u32)V) {
      if (deg[v]) atomicAdd(&D[l], (unsigned long long)deg[v]);
    } else {
      atomicAdd(bad, 1ull);
    }
  }
}
// communities (labels held by >= 1 vertex: size from k_histogram) and sum_c D_c^2
// (exact: D_c <= 2m < 2^33, sum <= (2m)^2 < 2^66 -- kept as two 64-bit halves)
__global__ __launch_bounds__(256) void k_q_sum(const int32_t* __restrict__ size, const unsigned long long* __restrict__ D,
                                               int64_t V, unsigned long long* __restrict__ acc) {
  unsigned long long n = 0, lo = 0, hi = 0;
  GRID_STRIDE(l, V) {
    n += size[l] > 0 ? 1ull : 0ull;
    const unsigned long long x = D[l];
    const unsigned long long sq_lo = x * x, sq_hi = __umul64hi(x, x);
    const unsigned long long t = lo + sq_lo;
    hi += sq_hi + (t < lo ? 1ull : 0ull);
    lo = t;
  }
  for (int off = 32; off > 0; off >>= 1) {
    n += __shfl_xor(n, off, 64);
    const unsigned long long olo = __shfl_xor(lo, off, 64), ohi = __shfl_xor(hi, off, 64);
    const unsigned long long t = lo + olo;
    hi += ohi + (t < lo ? 1ull : 0ull);
    lo = t;
  }
  if ((threadIdx.x & 63) == 0) {
    if (n) atomicAdd(&acc[0], n);
    // 128-bit accumulate: low half with carry into the high half
    const unsigned long long old = atomicAdd(&acc[1], lo);
    const unsigned long long carry = (old + lo < old) ? 1ull : 0ull;
    if (hi + carry) atomicAdd(&acc[2], hi + carry);
  }
}

}  // namespace

// Community count and Newman modularity of a labelling (dense ids) on the handle's
// symmetrised multigraph: A = 2m arcs, Q = intra / A - sum_c (D_c / A)^2 with D_c the
// degree sum of community c -- integer sums on the device, one host round trip.
int quality(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, lpa_quality_summary* out) {
  hipStream_t s = g->stream;
  const int64_t V = g->V, m = g->m;
  lpa_quality_summary q = {};
  q.arcs = 2 * m;
  if (V == 0) {
    *out = q;
    return LPA_OK;
  }
  Scratch sc(s);
  int32_t *L = nullptr, *size = nullptr;
  unsigned long long *D = nullptr, *acc = nullptr;
  LPA_TRY(sc.get(&L, V));
  LPA_TRY(sc.get(&size, V));
  LPA_TRY(sc.get(&D, V));
  LPA_TRY(sc.get(&acc, 8));
  if (labels_on_device) {
    LPA_HIP(hipMemcpyAsync(L, labels, sizeof(int32_t) * V, hipMemcpyDeviceToDevice, s));
  } else {
    LPA_TRY(ensure_pin(g, (size_t)4 * (size_t)V));
    par_copy(g->host_pin, labels, sizeof(int32_t) * V);
    LPA_HIP(hipMemcpyAsync(L, g->host_pin, sizeof(int32_t) * V, hipMemcpyHostToDevice, s));
  }
  LPA_HIP(hipMemsetAsync(size, 0, sizeof(int32_t) * V, s));
  LPA_HIP(hipMemsetAsync(D, 0, sizeof(unsigned long long) * V, s));
  LPA_HIP(hipMemsetAsync(acc, 0, sizeof(unsigned long long) * 8, s));
  hipLaunchKernelGGL(k_histogram, dim3(grid_bh(V)), dim3(256), 0, s, L, V, size, acc + 4);
  LPA_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_q_degsum, dim3(grid_bh(V)), dim3(256), 0, s, L, g->deg, V, D, acc + 5);
  LPA_HIP(hipGetLastError());
  if (m > 0) {
    hipLaunchKernelGGL(k_q_intra, dim3(grid_bh(m)), dim3(256), 0, s, g->e_src, g->e_dst, m, L, V, acc + 3);
    LPA_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(k_q_sum, dim3(grid_bh(V)), dim3(256), 0, s, size, D, V, acc);
  LPA_HIP(hipGetLastError());
  unsigned long long h[8];
  LPA_HIP(hipMemcpyAsync(h, acc, sizeof(h), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  if (h[4] || h[5]) return bad_labels(h[4] ? h[4] : h[5], V);
  q.n_communities = (int64_t)h[0];
  q.intra_arcs = (int64_t)h[3];
  const double A = (double)q.arcs;
  const double s2 = ((double)h[2] * 18446744073709551616.0 + (double)h[1]) / (A * A);
  q.degree_term = A > 0 ? s2 : 0.0;
  q.modularity = A > 0 ? (double)q.intra_arcs / A - s2 : 0.0;
  *out = q;
  return LPA_OK;
}

// Host round trips: the first call on a handle builds its distinct edge set (one);
// then none in L1 before the results are copied out, one in L2 (the size of E',
// which the second LPA's graph build needs).
int outlier(lpa_graph* g, const int32_t* labels, int32_t labels_on_device, int32_t mode,
            int32_t sub_iter, int64_t* size_hist, int64_t* incident, int32_t* sub_labels,
            uint8_t* flags, lpa_outlier_summary* summary, int32_t out_on_device) {
  if (mode != 1 && mode != 2) {
    set_error("outlier mode must be 1 (L1) or 2 (L2), got %d", mode);
    return LPA_EINVAL;
  }
  if (mode == 2 && sub_iter <= 0) {
    set_error("requirement failed: Maximum of steps must be greater than 0, but got %d", sub_iter);
    return LPA_EINVAL;
  }
  hipStream_t s = g->stream;
  const int64_t V = g->V;
  Scratch sc(s);
  lpa_outlier_summary sum = {};
  int32_t *L = nullptr, *size = nullptr, *inc = nullptr, *thr = nullptr, *segflag = nullptr;
  uint8_t* fl = nullptr;
  int64_t* wide = nullptr;
  // cnt: 0 communities, 1 flagged, 2 communities flagged, 3 bad labels, 4 groups,
  //      (distinct edges: g->de_n)
  unsigned long long* cnt = nullptr;
  LPA_TRY(sc.get(&L, V));
  LPA_TRY(sc.get(&size, V));
  LPA_TRY(sc.get(&inc, V));
  LPA_TRY(sc.get(&thr, V + 1));
  LPA_TRY(sc.get(&segflag, V));
  LPA_TRY(sc.get(&fl, V));
  LPA_TRY(sc.get(&wide, V));
  LPA_TRY(sc.get(&cnt, 8));
  if (V == 0) {
    if (summary) *summary = sum;
    return LPA_OK;
  }
  // pinned staging: [labels 4V | size 8V | incident 8V | sub-labels 4V | flags V] (host
  // labels in or host arrays out only)
  if (!labels_on_device || !out_on_device) LPA_TRY(ensure_pin(g, (size_t)25 * (size_t)V));
  char* pin = (char*)g->host_pin;
  int32_t* pin_lab = (int32_t*)pin;
  int64_t* pin_size = (int64_t*)(pin + 4 * V);
  int64_t* pin_inc = (int64_t*)(pin + 12 * V);
  int32_t* pin_sub = (int32_t*)(pin + 20 * V);
  uint8_t* pin_fl = (uint8_t*)(pin + 24 * V);
  if (labels_on_device) {
    LPA_HIP(hipMemcpyAsync(L, labels, sizeof(int32_t) * V, hipMemcpyDeviceToDevice, s));
  } else {
    par_copy(pin_lab, labels, sizeof(int32_t) * V);
    LPA_HIP(hipMemcpyAsync(L, pin_lab, sizeof(int32_t) * V, hipMemcpyHostToDevice, s));
  }
  LPA_HIP(hipMemsetAsync(size, 0, sizeof(int32_t) * V, s));
  LPA_HIP(hipMemsetAsync(inc, 0, sizeof(int32_t) * V, s));
  LPA_HIP(hipMemsetAsync(segflag, 0, sizeof(int32_t) * V, s));
  LPA_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * 8, s));

  hipLaunchKernelGGL(k_histogram, dim3(grid_bh(V)), dim3(256), 0, s, L, V, size, cnt + 3);
  LPA_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_count_nonzero, dim3(grid_cnt(V)), dim3(256), 0, s, size, V, cnt);
  LPA_HIP(hipGetLastError());

  LPA_TRY(distinct_edges(g));
  const u64* ek = g->de_keys;
  const int64_t md = g->de_n;   // distinct directed edges
  uint8_t* intra = nullptr;     // L2: the E' marks of the distinct edges
  if (mode == 2) LPA_TRY(sc.get(&intra, md));
  if (md > 0) {
    if (mode == 2)
      hipLaunchKernelGGL(k_incident<true>, dim3(grid_bh(md)), dim3(256), 0, s, ek, md, L, V, inc, intra);
    else
      hipLaunchKernelGGL(k_incident<false>, dim3(grid_bh(md)), dim3(256), 0, s, ek, md, L, V, inc,
                         (uint8_t*)nullptr);
    LPA_HIP(hipGetLastError());
  }

  if (mode == 1) {
    LPA_TRY(segmented_threshold(g, sc, size, nullptr, V, thr, cnt + 4));
    hipLaunchKernelGGL(k_flag, dim3(grid_for(V)), dim3(256), 0, s, L, size, (const int32_t*)nullptr,
                       thr, V, fl, segflag, cnt + 1);
    LPA_HIP(hipGetLastError());
    int32_t h_thr = 0;
    LPA_HIP(hipMemcpyAsync(&h_thr, thr, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    unsigned long long h_cnt[8];
    LPA_HIP(hipMemcpyAsync(h_cnt, cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    if (h_cnt[3]) return bad_labels(h_cnt[3], V);
    sum.n_groups = (int64_t)h_cnt[4];
    sum.k = sum.n_groups / 10;
    sum.threshold = h_thr;
    sum.n_flagged = (int64_t)h_cnt[1];
    sum.n_communities = (int64_t)h_cnt[0];
    sum.n_communities_flagged = sum.n_flagged > 0 ? 1 : 0;
    sum.distinct_edges = md;
  } else {
    // E' = the distinct intra-community edges: the sub-graph is built straight from the
    // handle's two sorted distinct-edge orders (build_graph_l2, no arc sort)
    int32_t *sub = nullptr, *subsize = nullptr;
    unsigned long long nbad = 0;
    LPA_HIP(hipMemcpyAsync(&nbad, cnt + 3, sizeof(nbad), hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    if (nbad) return bad_labels(nbad, V);
    LPA_TRY(sc.get(&sub, V));
    LPA_TRY(sc.get(&subsize, V));
    LPA_TRY(transposed_edges(g));
    // second LPA on the induced simple subgraph (same device, same stream)
    lpa_graph* h = nullptr;
    LPA_TRY(create_l2(g, L, intra, &h));
    // no refresh after the last superstep: only the labels are read, then h is destroyed
    int rc = run_supersteps(h, sub_iter, nullptr, false);
    if (rc == LPA_OK) rc = gather_labels(h, sub);
    if (rc == LPA_OK && hipStreamSynchronize(s) != hipSuccess) rc = LPA_EHIP;
    destroy(h);
    if (rc != LPA_OK) return rc;
    LPA_HIP(hipMemsetAsync(subsize, 0, sizeof(int32_t) * V, s));
    hipLaunchKernelGGL(k_histogram, dim3(grid_bh(V)), dim3(256), 0, s, sub, V, subsize, cnt + 3);
    LPA_HIP(hipGetLastError());
    // segment of a sub-label group = the community of the sub-label vertex: L itself
    LPA_TRY(segmented_threshold(g, sc, subsize, L, V, thr, cnt + 4));
    hipLaunchKernelGGL(k_flag, dim3(grid_for(V)), dim3(256), 0, s, sub, subsize, L, thr, V, fl,
                       segflag, cnt + 1);
    LPA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_count_nonzero, dim3(grid_cnt(V)), dim3(256), 0, s, segflag, V, cnt + 2);
    LPA_HIP(hipGetLastError());
    unsigned long long h_cnt[8];
    LPA_HIP(hipMemcpyAsync(h_cnt, cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, s));
    if (sub_labels)
      LPA_HIP(hipMemcpyAsync(out_on_device ? (void*)sub_labels : (void*)pin_sub, sub, sizeof(int32_t) * V,
                             out_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    sum.n_groups = (int64_t)h_cnt[4];
    sum.k = -1;
    sum.threshold = -1;
    sum.n_flagged = (int64_t)h_cnt[1];
    sum.n_communities = (int64_t)h_cnt[0];
    sum.n_communities_flagged = (int64_t)h_cnt[2];
    sum.distinct_edges = md;
  }

  // every output into the pinned area in stream order (`wide` is reused: each copy is
  // ordered before the next widening), one sync, then the threaded host copies
  if (out_on_device) {
    // device outputs: widened / copied in place, one sync for the stream's work
    if (size_hist) hipLaunchKernelGGL(k_widen, dim3(grid_for(V)), dim3(256), 0, s, size, V, size_hist);
    if (incident) hipLaunchKernelGGL(k_widen, dim3(grid_for(V)), dim3(256), 0, s, inc, V, incident);
    LPA_HIP(hipGetLastError());
    if (flags) LPA_HIP(hipMemcpyAsync(flags, fl, V, hipMemcpyDeviceToDevice, s));
    LPA_HIP(hipStreamSynchronize(s));
    if (summary) *summary = sum;
    return LPA_OK;
  }
  if (size_hist) {
    hipLaunchKernelGGL(k_widen, dim3(grid_for(V)), dim3(256), 0, s, size, V, wide);
    LPA_HIP(hipGetLastError());
    LPA_HIP(hipMemcpyAsync(pin_size, wide, sizeof(int64_t) * V, hipMemcpyDeviceToHost, s));
  }
  if (incident) {
    hipLaunchKernelGGL(k_widen, dim3(grid_for(V)), dim3(256), 0, s, inc, V, wide);
    LPA_HIP(hipGetLastError());
    LPA_HIP(hipMemcpyAsync(pin_inc, wide, sizeof(int64_t) * V, hipMemcpyDeviceToHost, s));
  }
  if (flags) LPA_HIP(hipMemcpyAsync(pin_fl, fl, V, hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  if (size_hist) par_copy(size_hist, pin_size, sizeof(int64_t) * V);
  if (incident) par_copy(incident, pin_inc, sizeof(int64_t) * V);
  if (mode == 2 && sub_labels) par_copy(sub_labels, pin_sub, sizeof(int32_t) * V);
  if (flags) par_copy(flags, pin_fl, V);
  if (summary) *summary = sum;
  return LPA_OK;
}

}  // namespace lpa
