// Graph construction on the GPU (replaces GraphFrames
// indexedVertices/indexedEdges/cachedTopologyGraphX and the GraphX EdgePartition
// build).
//
//   1. symmetrised degree of every vertex (each directed edge = one arc each way)
//   2. degree-ranked vertex order: sort by (degree desc, id asc) -> internal slots.
//      Rank r of P owns the vertices of degree rank k with k % P == r, at slot
//      r*slice + k/P: every rank's slice is itself degree-sorted, slices are equal
//      length (a plain allgather needs no padding) and carry ~A/P arcs each.
//      Labels keep the ORIGINAL dense ids as values, so the smallest-label
//      tie-break and the output are unaffected by the renumbering.
//   3. owned arcs emitted as 64-bit keys (row << 32 | col), LSD radix sorted
//      (rows sorted, neighbours ascending inside a row; hubs have the smallest
//      slots, so their labels sit densely in a few cache lines).
//   4. row_ptr = exclusive scan of owned degrees (int64: >2^31 arcs at scale 26).
//   5. degree bins = contiguous slot ranges (binary search on the sorted degrees),
//      hub segments, their tally staging and the combine work items.
#include "lpa_device.h"

namespace lpa {

namespace {

using dev::BlockHist;
using dev::kBhSlots;

// grid of the block-aggregated histogram kernels: few blocks, each over a long
// stretch of the input, so its LDS table absorbs the repeats before the flush
constexpr unsigned kBhGrid = 2048;
inline unsigned cap_bh(unsigned g) { return g < kBhGrid ? g : kBhGrid; }

// symmetrised degrees: a hub's counter took one device atomic per arc (same-address
// serialisation: 30 ms at R-MAT-24); block-aggregated in LDS instead
__global__ __launch_bounds__(256) void k_degree(const int32_t* __restrict__ src,
                                                const int32_t* __restrict__ dst, int64_t m, int32_t V,
                                                int32_t* __restrict__ deg, int32_t* err) {
  __shared__ u32 bk[kBhSlots];
  __shared__ int32_t bv[kBhSlots];
  __shared__ int bsat;
  BlockHist<int32_t> bh{bk, bv, &bsat};
  bh.init();
  const int lane = threadIdx.x & 63;
  for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x; e0 < m; e0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = e0 + threadIdx.x;
    u32 s = 0u, d = 0u;
    bool ok = false;
    if (e < m) {
      s = (u32)src[e];
      d = (u32)dst[e];
      ok = s < (u32)V && d < (u32)V;
      if (!ok) atomicOr(err, 1);
    }
    bh.add1(deg, ok, s, lane);
    bh.add1(deg, ok, d, lane);
  }
  bh.flush(deg);
}

// max degree: a capped grid, block-reduced, one atomic per block (a wave-level
// atomic per 64 vertices serialised ~2.6e5 same-address atomics: 3 ms at V = 16 M)
__global__ __launch_bounds__(256) void k_maxdeg(const int32_t* __restrict__ deg, int64_t V, int32_t* out) {
  __shared__ int32_t wm[4];
  int32_t mx = 0;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x)
    mx = max(mx, deg[v]);
  for (int off = 32; off > 0; off >>= 1) mx = max(mx, __shfl_xor(mx, off, 64));
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, max(max(wm[0], wm[1]), max(wm[2], wm[3])));
}

__global__ void k_vertex_keys(const int32_t* __restrict__ deg, int64_t V, int32_t maxdeg,
                              u64* __restrict__ keys) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x)
    keys[v] = ((u64)(u32)(maxdeg - deg[v]) << 32) | (u64)v;
}

// ---- locality order (g->locality): within each degree bin below the hubs, vertices
// are ordered by (smallest, second smallest) neighbour degree rank, so the
// low-degree neighbours a hub row shares with the highest-ranked hubs sit in
// contiguous slots and its label gathers (al[] rebuild) coalesce.  Hubs keep the
// (degree desc, id) order; the bins stay contiguous slot ranges.
__device__ __forceinline__ u32 degree_bin(int32_t d) {
  if (d > 1024) return 0;
  if (d == 0) return 12;
  // d in (2^(j-1), 2^j] -> bin 11 - j for j = 0..10 (1 -> g1 = 11, ..., (512, 1024] -> w16 = 1)
  const int j = d <= 1 ? 0 : 32 - __clz((u32)(d - 1));
  return (u32)(11 - j);
}

__global__ void k_rank_of(const u64* __restrict__ keys, int64_t V, int32_t* __restrict__ rank_of) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < V;
       k += (int64_t)gridDim.x * blockDim.x)
    rank_of[(u32)keys[k]] = (int32_t)k;
}

// key k of a non-hub vertex: its k-th smallest distinct neighbour rank (pass k reads
// key k-1 and takes the minimum neighbour rank above it); hubs are not reordered
__global__ void k_min_nbr(const int32_t* __restrict__ src, const int32_t* __restrict__ dst, int64_t m,
                          const int32_t* __restrict__ deg, const int32_t* __restrict__ rank_of,
                          const int32_t* __restrict__ nprev, int32_t* __restrict__ ncur) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int32_t a = src[e], b = dst[e];
    const int32_t ra = rank_of[a], rb = rank_of[b];
    if (deg[a] <= 1024 && (!nprev || rb > nprev[a])) atomicMin(&ncur[a], rb);
    if (deg[b] <= 1024 && (!nprev || ra > nprev[b])) atomicMin(&ncur[b], ra);
  }
}

// one stable radix stage of the locality order per key, last key first: stage keys
// (n_k << 32 | v) for k = K-1 .. 1, then ((bin << 28 | n_0) << 32 | v), hubs with
// (maxdeg - deg) in place of n_0 and 0 for the deeper keys.  The K + 1 stable sorts
// give (bin, n_0 | degree, n_1, ..., id).
__global__ void k_locality_keys(u64* __restrict__ keys, int64_t V, const int32_t* __restrict__ deg,
                                const int32_t* __restrict__ nk, int32_t maxdeg, int first, int last) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < V;
       k += (int64_t)gridDim.x * blockDim.x) {
    const u32 v = first ? (u32)k : (u32)keys[k];
    const int32_t d = deg[v];
    const u32 bin = degree_bin(d);
    const u32 cap = (1u << 28) - 1u;
    if (!last) {
      const u32 b2 = bin == 0 ? 0u : min((u32)nk[v], cap);
      keys[k] = ((u64)b2 << 32) | v;
    } else {
      const u32 a = bin == 0 ? (u32)(maxdeg - d) : min((u32)nk[v], cap);
      keys[k] = ((u64)((bin << 28) | a) << 32) | v;
    }
  }
}

__global__ void k_vertex_order(const u64* __restrict__ keys, int64_t V, int32_t P, int64_t S,
                               int32_t* __restrict__ new_of, int32_t* __restrict__ old_of) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < V;
       k += (int64_t)gridDim.x * blockDim.x) {
    int32_t old = (int32_t)(u32)keys[k];
    int64_t slot = (k % P) * S + k / P;
    new_of[old] = (int32_t)slot;
    old_of[slot] = old;
  }
}

__global__ void k_owned_degree(const int32_t* __restrict__ old_of_own,
                               const int32_t* __restrict__ deg, int64_t S,
                               int32_t* __restrict__ deg_own) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S;
       i += (int64_t)gridDim.x * blockDim.x) {
    int32_t o = old_of_own[i];
    deg_own[i] = o >= 0 ? deg[o] : 0;
  }
}

// P == 1: every edge gives two arcs at fixed positions (no atomics)
// rows below H (the class-blocked rows) sort their columns by (class, column): the
// class sits above the column's blo bits of the key
__global__ void k_emit_arcs_single(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                   int64_t m, const int32_t* __restrict__ new_of,
                                   u64* __restrict__ keys, int64_t H, int blo, u32 ncls) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (int64_t)gridDim.x * blockDim.x) {
    u64 s = (u32)new_of[src[e]], d = (u32)new_of[dst[e]];
    const u64 cd = (int64_t)s < H ? (u64)col_class((int32_t)d, ncls) << blo : 0ull;
    const u64 cs = (int64_t)d < H ? (u64)col_class((int32_t)s, ncls) << blo : 0ull;
    keys[2 * e] = (s << 32) | cd | d;
    keys[2 * e + 1] = (d << 32) | cs | s;
  }
}

// H = the number of rows of degree > T: with the degree-binned slot order (bins are
// contiguous, highest degrees first) they are the first H rows
__global__ void k_count_hub_rows(const int32_t* __restrict__ deg_own, int64_t S, int32_t T,
                                 int64_t* __restrict__ H) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < S; r += (int64_t)gridDim.x * blockDim.x)
    if (deg_own[r] > T && (r + 1 == S || deg_own[r + 1] <= T)) *H = r + 1;
}

// class segments of the blocked rows (index x H + h, class-major): the first position
// of row h with class >= x by binary search (the row is in (class, column) order), and
// the segment's piece count (<= 64 arcs each)
__global__ void k_class_segments(const int64_t* __restrict__ rp, const int32_t* __restrict__ col, int64_t H,
                                 u32 ncls, uint32_t* __restrict__ seg_start, int32_t* __restrict__ npieces) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)ncls * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i / H, h = i - x * H;
    const int64_t b = rp[h], e = rp[h + 1];
    auto first_ge = [&](uint32_t cls) {
      int64_t lo = b, hi = e;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (col_class(col[mid], ncls) < cls) lo = mid + 1;
        else hi = mid;
      }
      return lo;
    };
    const int64_t s0 = first_ge((uint32_t)x), s1 = x + 1 == (int64_t)ncls ? e : first_ge((uint32_t)x + 1);
    seg_start[i] = (uint32_t)s0;
    npieces[i] = (int32_t)((s1 - s0 + 63) / 64);
  }
}

__global__ void k_emit_pieces(const int64_t* __restrict__ rp, const uint32_t* __restrict__ seg_start,
                              const int64_t* __restrict__ poff, int64_t H, u32 ncls,
                              const int64_t* __restrict__ base, u64* __restrict__ pieces) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)ncls * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i / H, h = i - x * H;
    const int64_t s0 = seg_start[i];
    const int64_t s1 = x + 1 == (int64_t)ncls ? rp[h + 1] : (int64_t)seg_start[i + H];
    int64_t q = base[x] + (poff[i] - poff[x * H]);
    for (int64_t p = s0; p < s1; p += 64, ++q)
      pieces[q] = ((u64)(s1 - p < 64 ? s1 - p : 64) << 32) | (u64)p;
  }
}

// the positions [a, a0) between the last blocked row and the aligned start of the
// plain stream: pieces at the end of class 7's list
__global__ void k_tail_pieces(int64_t a, int64_t a0, int64_t q0, u64* __restrict__ pieces) {
  const int64_t n = (a0 - a + 63) / 64;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = a + 64 * j;
    pieces[q0 + j] = ((u64)(a0 - p < 64 ? a0 - p : 64) << 32) | (u64)p;
  }
}

// P > 1: keep the arcs whose row is owned; row stored slice-local.  One cursor
// atomic per wave (ballot-aggregated): a single device-wide counter saturates at
// ~88 M returning atomics/s, i.e. seconds for the ~A/P arcs of a rank.
__global__ void k_emit_arcs_owned(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                  int64_t m, const int32_t* __restrict__ new_of, int64_t lo,
                                  int64_t hi, u64* __restrict__ keys,
                                  unsigned long long* cursor) {
  const int lane = threadIdx.x & 63;
  const u64 lt = (1ull << lane) - 1ull;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = new_of[src[e]], d = new_of[dst[e]];
    const bool ks = s >= lo && s < hi, kd = d >= lo && d < hi;
    const u64 bs = __ballot(ks), bd = __ballot(kd);
    const int ns = __popcll(bs), nt = ns + __popcll(bd);
    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
    unsigned long long base = 0ull;
    if (lane == leader && nt > 0) base = atomicAdd(cursor, (unsigned long long)nt);
    base = (unsigned long long)__shfl((long long)base, leader, 64);
    if (ks) keys[base + __popcll(bs & lt)] = ((u64)(s - lo) << 32) | (u64)d;
    if (kd) keys[base + ns + __popcll(bd & lt)] = ((u64)(d - lo) << 32) | (u64)s;
  }
}

// sorted (row << 32 | col) keys -> col[] and the row of every arc position (crow[],
// read by the al[] scatter to mark the rows its writes make dirty)
__global__ void k_keys_to_col(const u64* __restrict__ keys, int64_t n, int32_t* __restrict__ col,
                              int32_t* __restrict__ crow, u32 cmask) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const u64 k = keys[j];
    col[j] = (int32_t)((u32)k & cmask);
    crow[j] = (int32_t)(k >> 32);
  }
}

// row-start bits of the arc positions (bit i of word w: position 64 w + i starts a row):
// one ballot per 64 positions; words past the arcs stay zero
__global__ void k_row_starts(const int32_t* __restrict__ crow, int64_t arcs, int64_t nwords,
                             u64* __restrict__ bits) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nwords; w += nw) {
    const int64_t i = w * 64 + lane;
    const bool st = i < arcs && (i == 0 || crow[i] != crow[i - 1]);
    const u64 m = __ballot(st);
    if (lane == 0) bits[w] = m;
  }
}

// CSC keys: (column << 32 | position), generated in position order so a stable
// sort on the column bits alone leaves positions ascending within a column
// (colcnt == nullptr: keys only -- at P = 1 the column counts are the degrees;
// otherwise block-aggregated: a hub column is one device atomic per block)
__global__ __launch_bounds__(256) void k_csc_keys(const int32_t* __restrict__ col, int64_t n,
                                                  u64* __restrict__ keys, int32_t* __restrict__ colcnt) {
  if (!colcnt) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
      keys[j] = ((u64)(u32)col[j] << 32) | (u64)j;
    return;
  }
  __shared__ u32 bk[kBhSlots];
  __shared__ int32_t bv[kBhSlots];
  __shared__ int bsat;
  BlockHist<int32_t> bh{bk, bv, &bsat};
  bh.init();
  const int lane = threadIdx.x & 63;
  for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x; j0 < n; j0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = j0 + threadIdx.x;
    u32 c = 0u;
    if (j < n) {
      c = (u32)col[j];
      keys[j] = ((u64)c << 32) | (u64)j;
    }
    bh.add1(colcnt, j < n, c, lane);
  }
  bh.flush(colcnt);
}

// scatter chunks of every column: count, then owner of each chunk
__global__ void k_col_chunks(const int32_t* __restrict__ colcnt, int64_t n, int32_t* __restrict__ nch) {
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n;
       u += (int64_t)gridDim.x * blockDim.x)
    nch[u] = (colcnt[u] + kChunkPos - 1) / kChunkPos;
}
__global__ void k_chunk_owner(const int64_t* __restrict__ cch, int64_t n, int32_t* __restrict__ cowner,
                              unsigned long long* __restrict__ scan_end) {
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n;
       u += (int64_t)gridDim.x * blockDim.x) {
    for (int64_t c = cch[u]; c < cch[u + 1]; ++c) cowner[c] = (int32_t)u;
    if (cch[u + 1] - cch[u] > 1) atomicMax(scan_end, (unsigned long long)cch[u + 1]);
  }
}

__global__ void k_keys_to_pos(const u64* __restrict__ keys, int64_t n, uint32_t* __restrict__ pos) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x)
    pos[j] = (uint32_t)keys[j];
}

// first index in the non-increasing deg_own[0, S) with deg <= t, for each threshold
__global__ void k_bin_bounds(const int32_t* __restrict__ deg_own, int64_t S,
                             const int32_t* __restrict__ thr, int nthr, int64_t* __restrict__ out) {
  int i = threadIdx.x;
  if (i >= nthr) return;
  int32_t t = thr[i];
  int64_t lo = 0, hi = S;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (deg_own[mid] > t) lo = mid + 1; else hi = mid;
  }
  out[i] = lo;
}

__global__ void k_seg_counts(const int32_t* __restrict__ deg_own, int64_t n0,
                             int32_t* __restrict__ nseg) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n0;
       v += (int64_t)gridDim.x * blockDim.x) {
    int32_t d = deg_own[v];
    nseg[v] = (d + kSegArcs - 1) / kSegArcs;
  }
}

__global__ void k_fill_segs(const int64_t* __restrict__ rp, const int32_t* __restrict__ deg_own,
                            const int64_t* __restrict__ seg_off, int64_t n0, int64_t n_hub,
                            Segment* __restrict__ segs) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n0;
       v += (int64_t)gridDim.x * blockDim.x) {
    int32_t d = deg_own[v];
    int64_t o = seg_off[v];
    int32_t ns = (d + kSegArcs - 1) / kSegArcs;
    for (int32_t j = 0; j < ns; ++j) {
      Segment sg;
      sg.begin = rp[v] + (int64_t)j * kSegArcs;
      sg.len = min(kSegArcs, d - j * kSegArcs) | (j << 10);
      sg.v = (int32_t)v;
      segs[o + j] = sg;
    }
  }
}

__global__ void k_init_labels(const int32_t* __restrict__ old_of, int64_t n, int32_t* __restrict__ a,
                              int32_t* __restrict__ b) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int32_t o = old_of[i];
    int32_t l = o >= 0 ? o : 0;
    a[i] = l;
    b[i] = l;
  }
}


// ---- the outlier stage's L2 sub-graph (build_graph_l2) ----
// intra-community marks over the parent's distinct edges in (s, d) order ...
__global__ void k_l2_mark_out(const u64* __restrict__ ek, int64_t md, const int32_t* __restrict__ L,
                              uint8_t* __restrict__ mark) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < md; i += (int64_t)gridDim.x * blockDim.x) {
    const u64 k = ek[i];
    mark[i] = L[(int32_t)(k >> 32)] == L[(int32_t)(u32)k] ? 1 : 0;
  }
}
// ... and in (d, s) order (de_t: d << 32 | index, de_ts: s)
__global__ void k_l2_mark_in(const u64* __restrict__ et, const uint32_t* __restrict__ ets, int64_t md,
                             const int32_t* __restrict__ L, uint8_t* __restrict__ mark) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < md; j += (int64_t)gridDim.x * blockDim.x)
    mark[j] = L[(int32_t)(et[j] >> 32)] == L[(int32_t)ets[j]] ? 1 : 0;
}
// degrees from segment lengths: v's intra out-edges are the marks of its run in the
// (s, d) order, its in-edges those of its run in the (d, s) order
__global__ void k_l2_degree(const int64_t* __restrict__ out_off, const int64_t* __restrict__ in_off,
                            const uint32_t* __restrict__ pos_out, const uint32_t* __restrict__ pos_in, int64_t V,
                            int32_t* __restrict__ deg, int32_t* __restrict__ dout) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V; v += (int64_t)gridDim.x * blockDim.x) {
    const int32_t o = (int32_t)(pos_out[out_off[v + 1]] - pos_out[out_off[v]]);
    const int32_t n = (int32_t)(pos_in[in_off[v + 1]] - pos_in[in_off[v]]);
    dout[v] = o;
    deg[v] = o + n;
  }
}
// (al: each arc's L0 label -- its column's dense id -- written with the arc (round 6), so
// the handle starts with al = L0[col] and init_labels runs no gather pass: 2.5 ms at C3)
// arcs of row s from its intra out-edges, in place: row s's first dout[s] positions
// (rows are the runs of the (s, d) order, so the per-row terms are cached loads; the
// column's slot is one gather from new_of, 4 B per vertex, cache-resident)
__global__ void k_l2_emit_out(const u64* __restrict__ ek, int64_t md, const uint8_t* __restrict__ mark,
                              const uint32_t* __restrict__ pos_out, const int64_t* __restrict__ out_off,
                              const int32_t* __restrict__ new_of, const int64_t* __restrict__ rp,
                              int32_t* __restrict__ col, int32_t* __restrict__ al) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < md; i += (int64_t)gridDim.x * blockDim.x) {
    if (!mark[i]) continue;
    const u64 k = ek[i];
    const int32_t sv = (int32_t)(k >> 32);
    const int64_t p = rp[new_of[sv]] + (int64_t)(pos_out[i] - pos_out[out_off[sv]]);
    col[p] = new_of[(int32_t)(u32)k];
    al[p] = (int32_t)(u32)k;   // the arc's L0 label: the column's dense id
  }
}
// arcs of row d from its intra in-edges, after its out-edges (de_t: d << 32 | index into
// the (s, d) order, de_ts: s)
__global__ void k_l2_emit_in(const u64* __restrict__ et, const uint32_t* __restrict__ ets, int64_t md,
                             const uint8_t* __restrict__ mark, const uint32_t* __restrict__ pos_in,
                             const int64_t* __restrict__ in_off, const int32_t* __restrict__ dout,
                             const int32_t* __restrict__ new_of, const int64_t* __restrict__ rp,
                             int32_t* __restrict__ col, int32_t* __restrict__ al) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < md; j += (int64_t)gridDim.x * blockDim.x) {
    if (!mark[j]) continue;
    const int32_t dv = (int32_t)(et[j] >> 32);
    const int64_t q = rp[new_of[dv]] + dout[dv] + (int64_t)(pos_in[j] - pos_in[in_off[dv]]);
    const int32_t sv = (int32_t)ets[j];
    col[q] = new_of[sv];
    al[q] = sv;
  }
}

inline unsigned grid_for(int64_t n, int threads = 256) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > 65536) b = 65536;
  return (unsigned)b;
}

}  // namespace

int init_labels(lpa_graph* g) {
  hipLaunchKernelGGL(k_init_labels, dim3(grid_for(g->vpad)), dim3(256), 0, g->stream, g->old_of,
                     g->vpad, g->lab[0], g->lab[1]);
  LPA_HIP(hipGetLastError());
  if (g->dev_err) LPA_HIP(hipMemsetAsync(g->dev_err, 0, sizeof(int32_t), g->stream));
  // L0: every row is tallied in superstep 1; no stale dirty flags
  for (int p = 0; p < 2; ++p) {
    LPA_HIP(hipMemsetAsync(g->rdirty[p], 0, g->slice, g->stream));
    LPA_HIP(hipMemsetAsync(g->udirty[p], 0, (g->n_segs + 16) / 16 * 16, g->stream));
  }
  LPA_HIP(hipMemsetD32Async((hipDeviceptr_t)g->fr_all, 1, 2, g->stream));
  LPA_HIP(hipMemsetAsync(g->fcnt, 0, sizeof(int32_t) * 32, g->stream));
  LPA_HIP(hipMemsetAsync(g->counters, 0, sizeof(unsigned long long) * 8, g->stream));
  if (g->gword) {
    LPA_HIP(hipMemsetAsync(g->gword + 2, 0, sizeof(int32_t), g->stream));  // abits stale
    LPA_HIP(hipMemsetAsync(g->gword + 9, 0, sizeof(int32_t), g->stream));  // no abits pass ran
    LPA_HIP(hipMemsetAsync(g->gword + 5, 0, sizeof(int32_t), g->stream));  // no giant-code refresh pending
  }
  g->cur = 0;
  g->since_reset = 0;
  g->force_all_next = false;
  g->prev_delta_ok = false;  // the exchange's delta chain restarts from L0
  if (g->al0) {              // al = L0[col] is al0: nothing to gather (lazy, see al0)
    g->al_pending = true;
    return LPA_OK;
  }
  if (g->al_is_l0) {         // the L2 sub-graph's build wrote al = L0[col] with the arcs
    g->al_is_l0 = false;
    return LPA_OK;
  }
  return rebuild_arc_labels(g);
}

// Degree-ranked vertex order (degree desc, id asc; optionally the locality order inside
// the bins below the hubs, which reads the kept edge list): new_of / old_of.  Needs
// g->deg and g->max_degree; P ranks take the ranks round-robin (slot (k % P) S + k / P).
int vertex_order(lpa_graph* g, int32_t V, int64_t m, bool locality) {
  hipStream_t s = g->stream;
  const int32_t P = g->nranks;
  const int64_t S = g->slice;
  LPA_TRY(dev_alloc(g, (void**)&g->new_of, sizeof(int32_t) * (V > 0 ? V : 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->old_of, sizeof(int32_t) * g->vpad));
  LPA_HIP(hipMemsetAsync(g->old_of, 0xFF, sizeof(int32_t) * g->vpad, s));
  if (V > 0) {
    u64* vk = nullptr;
    LPA_TRY(scratch_alloc(g, (void**)&vk, sizeof(u64) * 2 * V));
    hipLaunchKernelGGL(k_vertex_keys, dim3(grid_for(V)), dim3(256), 0, s, g->deg, (int64_t)V,
                       g->max_degree, vk);
    LPA_HIP(hipGetLastError());
    int shifts[16], ns = 0;
    int blo = bits_for((uint64_t)(V - 1)), bhi = bits_for((uint64_t)g->max_degree);
    for (int b = 0; b < blo; b += 8) shifts[ns++] = b;
    for (int b = 0; b < bhi; b += 8) shifts[ns++] = 32 + b;
    LPA_TRY(radix_sort_u64(vk, vk + V, V, shifts, ns, s));
    if (locality && m > 0 && V < (1 << 28)) {
      const int K = g->locality < 4 ? g->locality : 4;  // neighbour keys (LPA_LOCALITY)
      int32_t* rank_of = nullptr;
      LPA_TRY(scratch_alloc(g, (void**)&rank_of, sizeof(int32_t) * (1 + K) * (size_t)V));
      int32_t* nk[4] = {rank_of + V, rank_of + 2 * V, rank_of + 3 * V, rank_of + 4 * V};
      hipLaunchKernelGGL(k_rank_of, dim3(grid_for(V)), dim3(256), 0, s, vk, (int64_t)V, rank_of);
      LPA_HIP(hipMemsetAsync(nk[0], 0x7F, sizeof(int32_t) * K * (size_t)V, s));
      for (int k = 0; k < K; ++k)
        hipLaunchKernelGGL(k_min_nbr, dim3(grid_for(m)), dim3(256), 0, s, g->e_src, g->e_dst, m, g->deg,
                           rank_of, k ? nk[k - 1] : nullptr, nk[k]);
      LPA_HIP(hipGetLastError());
      const int hi[4] = {32, 40, 48, 56};
      for (int k = K - 1; k >= 0; --k) {
        hipLaunchKernelGGL(k_locality_keys, dim3(grid_for(V)), dim3(256), 0, s, vk, (int64_t)V, g->deg,
                           nk[k], g->max_degree, k == K - 1 ? 1 : 0, k == 0 ? 1 : 0);
        LPA_TRY(radix_sort_u64(vk, vk + V, V, hi, 4, s));
      }
      LPA_HIP(hipGetLastError());
      scratch_free(g, rank_of);
    }
    hipLaunchKernelGGL(k_vertex_order, dim3(grid_for(V)), dim3(256), 0, s, vk, (int64_t)V, P, S,
                       g->new_of, g->old_of);
    LPA_HIP(hipGetLastError());
    scratch_free(g, vk);
  }

  return LPA_OK;
}

// Everything after the CSR and its CSC position index: the arc label arrays, the degree
// bins, the hub units and combine tables, the frontier flags, the superstep-1 run
// structures and the label vectors.  Frees deg_own (the owned degrees, scratch).
int finish_build(lpa_graph* g, int32_t* deg_own, int64_t m) {
  hipStream_t s = g->stream;
  const int32_t P = g->nranks, r = g->rank;
  const int64_t S = g->slice;
  const int64_t arcs = g->arcs;
  if (!g->al) LPA_TRY(dev_alloc(g, (void**)&g->al, sizeof(int32_t) * (arcs > 0 ? arcs : 1)));
  {
    const int64_t nfl = (g->n_chunks + 16) / 16 * 16;
    LPA_TRY(dev_alloc(g, (void**)&g->chflag, nfl));
    LPA_HIP(hipMemsetAsync(g->chflag, 0, nfl, s));
    LPA_TRY(dev_alloc(g, (void**)&g->chlist, sizeof(int32_t) * g->vpad));
  }
  LPA_TRY(dev_alloc(g, (void**)&g->counters, sizeof(unsigned long long) * 8));  // 2 parities
  LPA_HIP(hipMemsetAsync(g->counters, 0, sizeof(unsigned long long) * 8, s));

  // ---- 4. degree bins (contiguous slot ranges) ----
  {
    // thresholds: bin b+1 starts at the first vertex with deg <= kBinMaxDeg[b+1];
    // the last entry finds the hubs (rows longer than one segment)
    int32_t thr_h[LPA_NBINS];
    for (int b = 1; b < LPA_NBINS; ++b) thr_h[b - 1] = kBinMaxDeg[b];
    thr_h[LPA_NBINS - 1] = kWideMaxDeg;
    int32_t* d_thr = nullptr;
    int64_t* d_bb = nullptr;
    LPA_TRY(scratch_alloc(g, (void**)&d_thr, sizeof(thr_h)));
    LPA_TRY(scratch_alloc(g, (void**)&d_bb, sizeof(int64_t) * LPA_NBINS));
    LPA_HIP(hipMemcpyAsync(d_thr, thr_h, sizeof(thr_h), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_bin_bounds, dim3(1), dim3(64), 0, s, deg_own, S, d_thr, LPA_NBINS, d_bb);
    LPA_HIP(hipGetLastError());
    int64_t bb[LPA_NBINS];
    LPA_HIP(hipMemcpyAsync(bb, d_bb, sizeof(bb), hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    scratch_free(g, d_thr);
    scratch_free(g, d_bb);
    g->bin_begin[0] = 0;
    for (int b = 1; b < LPA_NBINS; ++b) g->bin_begin[b] = bb[b - 1];
    g->bin_begin[LPA_NBINS] = S;
    g->n_hub = bb[LPA_NBINS - 1];
    int64_t rpb[LPA_NBINS + 1];
    for (int b = 0; b <= LPA_NBINS; ++b)
      LPA_HIP(hipMemcpyAsync(&rpb[b], g->rp + g->bin_begin[b], sizeof(int64_t),
                             hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    for (int b = 0; b < LPA_NBINS; ++b) g->bin_arcs[b] = rpb[b + 1] - rpb[b];
  }

  // ---- 5. hub segments + global merge tables ----
  const int64_t n0 = g->bin_begin[1];
  if (n0 > 0) {
    int32_t* nseg = nullptr;
    int64_t* seg_off = nullptr;
    LPA_TRY(scratch_alloc(g, (void**)&nseg, sizeof(int32_t) * n0));
    LPA_TRY(scratch_alloc(g, (void**)&seg_off, sizeof(int64_t) * (n0 + 1)));
    hipLaunchKernelGGL(k_seg_counts, dim3(grid_for(n0)), dim3(256), 0, s, deg_own, n0, nseg);
    LPA_HIP(hipGetLastError());
    LPA_TRY(exclusive_scan_i32_i64(nseg, seg_off, n0, s));
    LPA_HIP(hipMemcpyAsync(&g->n_segs, seg_off + n0, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    LPA_TRY(dev_alloc(g, (void**)&g->segs, sizeof(Segment) * g->n_segs));
    hipLaunchKernelGGL(k_fill_segs, dim3(grid_for(n0)), dim3(256), 0, s, g->rp, deg_own, seg_off,
                       n0, g->n_hub, g->segs);
    LPA_HIP(hipGetLastError());
    LPA_TRY(build_hub_tables(g, deg_own));
    scratch_free(g, nseg);
    LPA_TRY(dev_alloc(g, (void**)&g->ucnt, sizeof(int32_t) * (g->n_segs > 0 ? g->n_segs : 1)));
    LPA_TRY(dev_alloc(g, (void**)&g->ugc, sizeof(uint32_t) * (g->n_segs > 0 ? g->n_segs : 1)));
    LPA_TRY(dev_alloc(g, (void**)&g->umx, sizeof(uint32_t) * (g->n_segs > 0 ? g->n_segs : 1)));
    LPA_TRY(dev_alloc(g, (void**)&g->ulist2, sizeof(int32_t) * (g->n_segs > 0 ? g->n_segs : 1)));
    LPA_TRY(dev_alloc(g, (void**)&g->gdec, sizeof(int32_t) * 4));
    LPA_HIP(hipMemsetAsync(g->gdec, 0, sizeof(int32_t) * 4, s));
    LPA_TRY(dev_alloc(g, (void**)&g->glist, sizeof(int32_t) * (g->n_hub > 0 ? g->n_hub : 1)));
    g->hub_uoff = seg_off;  // the seg bin is exactly the hub rows (deg > kSegArcs)
    // first unit of the k_lpa_block rows
    LPA_HIP(hipMemcpyAsync(&g->unit_lane_begin, seg_off + g->hub_lane_begin, sizeof(int64_t),
                           hipMemcpyDeviceToHost, s));
    LPA_HIP(hipMemcpyAsync(&g->unit_block2_begin, seg_off + g->hub_block2_begin, sizeof(int64_t),
                           hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    g->device_bytes += (int64_t)sizeof(int64_t) * (n0 + 1);
  }
  scratch_free(g, deg_own);

  LPA_TRY(dev_alloc(g, (void**)&g->dev_err, sizeof(int32_t)));
  LPA_HIP(hipMemsetAsync(g->dev_err, 0, sizeof(int32_t), s));
  // frontier flags (cleared / set to "all rows" by init_labels)
  for (int p = 0; p < 2; ++p) {
    LPA_TRY(dev_alloc(g, (void**)&g->rdirty[p], S));   // S: a multiple of 64
    LPA_TRY(dev_alloc(g, (void**)&g->udirty[p], (g->n_segs + 16) / 16 * 16));
  }
  LPA_TRY(dev_alloc(g, (void**)&g->fr_all, 2 * sizeof(int32_t)));
  LPA_TRY(dev_alloc(g, (void**)&g->flist, sizeof(int32_t) * S));
  LPA_TRY(dev_alloc(g, (void**)&g->ulist, sizeof(int32_t) * (g->n_segs > 0 ? g->n_segs : 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->fcnt, sizeof(int32_t) * 32));
  // superstep-1 column-run tally (lpa_iter.hip k_first_runs): per-row maxima of rows that
  // span run tiles (zero between uses)
  if (g->cols_sorted) {
    LPA_TRY(dev_alloc(g, (void**)&g->first_best, sizeof(u64) * S));
    LPA_HIP(hipMemsetAsync(g->first_best, 0, sizeof(u64) * S, s));
    if (arcs > 0) {
      // whole run tiles of words plus the next tile's words (k_first_runs)
      const int64_t nwords = (arcs + kRunTile - 1) / kRunTile * (kRunTile / 64) + kRunTile / 64;
      LPA_TRY(dev_alloc(g, (void**)&g->rstart, sizeof(u64) * nwords));
      hipLaunchKernelGGL(k_row_starts, dim3(grid_for(nwords * 64)), dim3(256), 0, s, g->crow, arcs, nwords,
                         g->rstart);
      LPA_HIP(hipGetLastError());
    }
  }
  if (g->crow == nullptr) LPA_TRY(dev_alloc(g, (void**)&g->crow, sizeof(int32_t)));

  // ---- labels (replicated, ping-pong) ----
  LPA_TRY(dev_alloc(g, (void**)&g->gbits, sizeof(uint32_t) * ((g->vpad + 63) / 64 * 2)));
  LPA_TRY(dev_alloc(g, (void**)&g->gword, sizeof(int32_t) * 16));
  LPA_HIP(hipMemsetAsync(g->gword, 0, sizeof(int32_t) * 16, s));
  LPA_TRY(dev_alloc(g, (void**)&g->abits, sizeof(unsigned long long) * ((g->arcs + 63) / 64 + 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->lab[0], sizeof(int32_t) * g->vpad));
  LPA_TRY(dev_alloc(g, (void**)&g->lab[1], sizeof(int32_t) * g->vpad));
  LPA_TRY(init_labels(g));
  // the column-run superstep 1 can read the L0 arc labels from a kept copy (al0): a
  // reset then costs no gather pass over the arcs (2.4 ms at C3)
  if (g->cols_sorted && g->first_runs && g->arcs > 0 && !g->pooled) {
    LPA_TRY(dev_alloc(g, (void**)&g->al0, sizeof(int32_t) * g->arcs));
    LPA_HIP(hipMemcpyAsync(g->al0, g->al, sizeof(int32_t) * g->arcs, hipMemcpyDeviceToDevice, s));
  }
  // gather mode (lpa_iter.hip arc_vote): one GPU, a label vector that stays in L2 (<= 4 MB),
  // every row in the bins of <= 128 arcs (no hub / unit / block tier, no wave bin above w2)
  // and the CSC index the scatter marks the frontier with.  The tallies then read L[col[i]]
  // and no al[] refresh runs: a label-dense superstep of C2 (SBM 1 M / 20 M) spent as long
  // in the rebuild (0.18 ms, L2-request bound) as in its tallies.
#ifndef LPA_GATHER_OK
#define LPA_GATHER_OK 1   // 0: a comparison build without gather mode (tools/ab_lib)
#endif
  g->gather = LPA_GATHER_OK && P == 1 && !g->pooled && !g->no_scatter && 4 * g->vpad <= (int64_t(4) << 20) && g->n_hub == 0 &&
              g->bin_begin[BIN_W2] == g->bin_begin[BIN_SEG] && g->arcs > 0;
  // giant codes (lpa_iter.hip): the LDS hot-set rebuild's label vectors (one GPU, or the
  // rank-strided form of a partitioned job: every rank codes its own arcs against the G
  // of the replicated vector), and a superstep 2 whose hub rows take the giant decision
  // (block mode, or no hub rows)
  // (round 6: the outlier stage's pooled, rebuild-only L2 sub-graph too -- its second LPA
  // from L0 collapses like the first, and every refresh there rebuilds anyway)
  g->code_ok = g->codes_env && (P == 1 || rebuild_ranked(g)) && !g->gather && g->rebuild_hot &&
               g->vpad >= kHotMinSlots && g->arcs > 0 && (g->n_hub == 0 || g->hub_lane_begin < g->n_hub);
  if (g->code_ok) {
    // the rows of <= 64 arcs keep their labels when the label vector is small (C3: 64 MB,
    // Infinity-Cache resident): three code buckets leave 10 % of their arcs undecided, whose
    // gathers superstep 2 then pays, while their label gathers in the refresh cost little
    // more than codes (C3 superstep 2 1.96 -> 1.78 ms, superstep 1 1.69 -> 1.82); a larger
    // vector's label gathers miss (C4 superstep 1 8.0 -> 9.4 ms, C5's refresh after
    // superstep 2 +5 ms): only the rows of <= 8 arcs keep labels there.  (The vector is
    // the full replica at any P, so every rank takes the same cut.)
    g->code_lbin = 4 * g->vpad <= (int64_t(64) << 20) ? BIN_G64 : BIN_G8;
    if (g->code_lbin_env == BIN_G64 || g->code_lbin_env == BIN_G8) g->code_lbin = g->code_lbin_env;
    for (int b = 0; b < g->code_lbin; ++b) g->code_pcut += g->bin_arcs[b];
    LPA_TRY(dev_alloc(g, (void**)&g->code2, sizeof(uint32_t) * (size_t)(g->vpad / 16)));
    LPA_TRY(dev_alloc(g, (void**)&g->al2, sizeof(uint32_t) * (size_t)(((g->code_pcut + 511) / 512 * 512 + 512) / 16)));
    if (!g->h_flag) LPA_HIP(hipHostMalloc((void**)&g->h_flag, sizeof(int32_t), hipHostMallocDefault));
  }
  // pinned words every handle reads through (the code-refresh flag, the kernel-error word
  // at the end of a call); a handle that may parent an L2 sub-graph lends them to it
  if (!g->h_flag) LPA_HIP(hipHostMalloc((void**)&g->h_flag, sizeof(int32_t), hipHostMallocDefault));
  if (!g->h_err) LPA_HIP(hipHostMalloc((void**)&g->h_err, sizeof(int32_t), hipHostMallocDefault));
  LPA_HIP(hipStreamSynchronize(s));
  // the kept edge list serves the outlier stage (single-GPU handles) and lpa_quality,
  // which a distributed job runs on rank 0: the other ranks release it (at C5 over 8
  // ranks, 11 GB per rank)
  if (P > 1 && r != 0) {
    dev_free(g, g->e_src);
    dev_free(g, g->e_dst);
    g->device_bytes -= 2 * (int64_t)sizeof(int32_t) * (m > 0 ? m : 1);
    g->e_src = g->e_dst = nullptr;
  }
  return LPA_OK;
}

// The class-blocked rebuild's piece lists (lpa_iter.hip rebuild_pieces) over the first
// H rows (in (class, column) order): per class, every row's class segment in <= 64-arc
// pieces, row after row, then padding to a multiple of 8 pieces; class 7 also lists
// the positions up to blk_a0, the 512-aligned start of the plain stream.
int build_pieces(lpa_graph* g, int64_t H) {
  hipStream_t s = g->stream;
  const int C = g->blk_classes;
  int64_t aH = 0;
  LPA_HIP(hipMemcpyAsync(&aH, g->rp + H, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  uint32_t* seg = nullptr;
  int32_t* np = nullptr;
  int64_t* poff = nullptr;
  int64_t* d_base = nullptr;
  LPA_TRY(scratch_alloc(g, (void**)&seg, sizeof(uint32_t) * C * H));
  LPA_TRY(scratch_alloc(g, (void**)&np, sizeof(int32_t) * C * H));
  LPA_TRY(scratch_alloc(g, (void**)&poff, sizeof(int64_t) * (C * H + 1)));
  LPA_TRY(scratch_alloc(g, (void**)&d_base, sizeof(int64_t) * kMaxBlkClasses));
  hipLaunchKernelGGL(k_class_segments, dim3(grid_for(C * H)), dim3(256), 0, s, g->rp, g->col, H, (u32)C, seg, np);
  LPA_HIP(hipGetLastError());
  LPA_TRY(exclusive_scan_i32_i64(np, poff, C * H, s));
  int64_t cum[kMaxBlkClasses + 1];
  for (int x = 0; x <= C; ++x)
    LPA_HIP(hipMemcpyAsync(&cum[x], poff + x * H, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  int64_t a0 = (aH + 511) / 512 * 512;
  if (a0 > g->arcs) a0 = g->arcs;
  const int64_t ntail = (a0 - aH + 63) / 64;
  int64_t base[kMaxBlkClasses];
  g->blk_off[0] = 0;
  for (int x = 0; x < C; ++x) {
    base[x] = g->blk_off[x];
    const int64_t n = cum[x + 1] - cum[x] + (x == C - 1 ? ntail : 0);
    g->blk_off[x + 1] = g->blk_off[x] + (n + 7) / 8 * 8;
  }
  const int64_t npc = g->blk_off[C] > 0 ? g->blk_off[C] : 1;
  LPA_TRY(dev_alloc(g, (void**)&g->blk_pieces, sizeof(u64) * npc));
  LPA_HIP(hipMemsetAsync(g->blk_pieces, 0, sizeof(u64) * npc, s));
  LPA_HIP(hipMemcpyAsync(d_base, base, sizeof(int64_t) * C, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_emit_pieces, dim3(grid_for(C * H)), dim3(256), 0, s, g->rp, seg, poff, H, (u32)C, d_base,
                     g->blk_pieces);
  LPA_HIP(hipGetLastError());
  if (ntail > 0) {
    hipLaunchKernelGGL(k_tail_pieces, dim3(grid_for(ntail)), dim3(256), 0, s, aH, a0,
                       base[C - 1] + (cum[C] - cum[C - 1]), g->blk_pieces);
    LPA_HIP(hipGetLastError());
  }
  LPA_HIP(hipStreamSynchronize(s));
  g->blk_a0 = a0;
  scratch_free(g, d_base);
  scratch_free(g, poff);
  scratch_free(g, np);
  scratch_free(g, seg);
  return LPA_OK;
}

int build_graph(lpa_graph* g, const int32_t* src, const int32_t* dst, int64_t m, int32_t V,
                uint32_t flags) {
  hipStream_t s = g->stream;
  const int32_t P = g->nranks, r = g->rank;
  g->V = V;
  g->m = m;
  g->slice = ((int64_t)V + P - 1) / P;
  g->slice = (g->slice + 63) / 64 * 64;  // vector-aligned slices (k_diff reads int4)
  if (g->slice == 0) g->slice = 64;
  // P > 1 (a power of two): power-of-two slices, the tail of each padded with isolated
  // slots, so that the rank-strided LDS hot-set rebuild and the giant codes apply
  // (rebuild_ranked): C5 over 8 ranks has 5 M vertices per slice, which otherwise took the
  // plain labels-mode rebuild in every refresh.  The padding costs only label-vector
  // bytes (C5: 160 -> 256 MB per replica) in the vector-sized passes (diff, full exchange).
  // LPA_POW2_SLICES=0: the tight slices.
  if (P > 1 && (P & (P - 1)) == 0 && g->rebuild_hot && g->pow2_slices) {
    int64_t np2 = 64;
    while (np2 < g->slice) np2 *= 2;
    if (np2 * P <= (int64_t(1) << 30)) g->slice = np2;
  }
  g->vpad = g->slice * P;
  g->own_begin = (int64_t)r * g->slice;
  const int64_t S = g->slice;

  // ---- keep the edge list on the device (outlier stage needs it) ----
  LPA_TRY(dev_alloc(g, (void**)&g->e_src, sizeof(int32_t) * (m > 0 ? m : 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->e_dst, sizeof(int32_t) * (m > 0 ? m : 1)));
  if (m > 0) {
    hipMemcpyKind kind = (flags & LPA_INPUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    LPA_HIP(hipMemcpyAsync(g->e_src, src, sizeof(int32_t) * m, kind, s));
    LPA_HIP(hipMemcpyAsync(g->e_dst, dst, sizeof(int32_t) * m, kind, s));
  }

  // ---- 1. degrees ----
  int32_t* d_err = nullptr;
  int32_t* d_max = nullptr;
  LPA_TRY(scratch_alloc(g, (void**)&d_err, 2 * sizeof(int32_t)));
  d_max = d_err + 1;
  LPA_HIP(hipMemsetAsync(d_err, 0, 2 * sizeof(int32_t), s));
  LPA_TRY(dev_alloc(g, (void**)&g->deg, sizeof(int32_t) * (V > 0 ? V : 1)));
  LPA_HIP(hipMemsetAsync(g->deg, 0, sizeof(int32_t) * (V > 0 ? V : 1), s));
  if (m > 0) {
    hipLaunchKernelGGL(k_degree, dim3(cap_bh(grid_for(m))), dim3(256), 0, s, g->e_src, g->e_dst, m, V,
                       g->deg, d_err);
    LPA_HIP(hipGetLastError());
  }
  if (V > 0) {
    hipLaunchKernelGGL(k_maxdeg, dim3(grid_for(V) < 1024u ? grid_for(V) : 1024u), dim3(256), 0, s, g->deg,
                       (int64_t)V, d_max);
    LPA_HIP(hipGetLastError());
  }
  int32_t h_err[2] = {0, 0};
  LPA_HIP(hipMemcpyAsync(h_err, d_err, sizeof(h_err), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  scratch_free(g, d_err);
  if (h_err[0]) {
    set_error("edge endpoint outside [0, V=%d)", V);
    return LPA_EINVAL;
  }
  g->max_degree = h_err[1];

  // ---- 2. degree-ranked vertex order ----
  LPA_TRY(vertex_order(g, V, m, g->locality > 0));

  // ---- owned degrees, row_ptr ----
  int32_t* deg_own = nullptr;
  LPA_TRY(scratch_alloc(g, (void**)&deg_own, sizeof(int32_t) * S));
  hipLaunchKernelGGL(k_owned_degree, dim3(grid_for(S)), dim3(256), 0, s, g->old_of + g->own_begin,
                     g->deg, S, deg_own);
  LPA_HIP(hipGetLastError());
  LPA_TRY(dev_alloc(g, (void**)&g->rp, sizeof(int64_t) * (S + 1)));
  LPA_TRY(exclusive_scan_i32_i64(deg_own, g->rp, S, s));
  int64_t arcs = 0;
  LPA_HIP(hipMemcpyAsync(&arcs, g->rp + S, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  g->arcs = arcs;

  // ---- 3. owned arcs, sorted ----
  LPA_TRY(dev_alloc(g, (void**)&g->col, sizeof(int32_t) * (arcs > 0 ? arcs : 1)));
  if (arcs > 0) {
    u64* keys = nullptr;
    if (scratch_alloc(g, (void**)&keys, sizeof(u64) * 2 * arcs) != LPA_OK) {
      set_error("out of device memory for %lld arc keys", (long long)(2 * arcs));
      return LPA_ENOMEM;
    }
    int blo = bits_for((uint64_t)(g->vpad - 1)), bhi = bits_for((uint64_t)(S - 1));
    // class-blocked rows (P = 1 hot-set rebuild sizes; the class needs 3 key bits)
    g->cols_sorted = !g->pooled;
    int64_t H = 0;
    if (P == 1 && g->cols_sorted && g->block_deg > 0 && g->vpad >= kHotMinSlots &&
        g->vpad >= g->block_min_slots && blo + 3 <= 32) {
      int64_t* d_h = nullptr;
      LPA_TRY(scratch_alloc(g, (void**)&d_h, sizeof(int64_t)));
      LPA_HIP(hipMemsetAsync(d_h, 0, sizeof(int64_t), s));
      // a power of two: the degree bins of the locality order are (2^(j-1), 2^j]
      int32_t T = 1;
      while (2 * T <= g->block_deg && T < (1 << 30)) T *= 2;
      hipLaunchKernelGGL(k_count_hub_rows, dim3(grid_for(S)), dim3(256), 0, s, deg_own, S, T, d_h);
      LPA_HIP(hipGetLastError());
      LPA_HIP(hipMemcpyAsync(&H, d_h, sizeof(int64_t), hipMemcpyDeviceToHost, s));
      LPA_HIP(hipStreamSynchronize(s));
      scratch_free(g, d_h);
    }
    g->blk_rows = H;
    // classes: about one 4 MB L2's worth of labels each (8 per phase), at most
    // kMaxBlkClasses, and the class bits must fit above the column's in the key half
    int cb = 3;
    while ((1ll << cb) * (4ll << 20) < g->vpad * 4 && (1 << (cb + 1)) <= kMaxBlkClasses && blo + cb + 1 <= 32)
      ++cb;
    g->blk_classes = 1 << cb;
    if (P == 1) {
      hipLaunchKernelGGL(k_emit_arcs_single, dim3(grid_for(m)), dim3(256), 0, s, g->e_src,
                         g->e_dst, m, g->new_of, keys, H, blo, (u32)g->blk_classes);
    } else {
      unsigned long long* cursor = nullptr;
      LPA_TRY(scratch_alloc(g, (void**)&cursor, sizeof(unsigned long long)));
      LPA_HIP(hipMemsetAsync(cursor, 0, sizeof(unsigned long long), s));
      hipLaunchKernelGGL(k_emit_arcs_owned, dim3(grid_for(m)), dim3(256), 0, s, g->e_src,
                         g->e_dst, m, g->new_of, g->own_begin, g->own_begin + S, keys, cursor);
      scratch_free(g, cursor);
    }
    LPA_HIP(hipGetLastError());
    int shifts[16], ns = 0;
    // columns sorted inside each row (blocked rows: by class, then column): the
    // rebuild's gathers of a hub row coalesce, and superstep 1 counts runs of equal
    // columns.  No tally needs the order (a mode is order-free), so a pooled internal
    // graph (the outlier stage's 5-superstep L2 sub-graph) sorts by row only.
    if (g->cols_sorted)
      for (int b = 0; b < blo + (H > 0 ? cb : 0); b += 8) shifts[ns++] = b;
    for (int b = 0; b < bhi; b += 8) shifts[ns++] = 32 + b;
    LPA_TRY(radix_sort_u64(keys, keys + arcs, arcs, shifts, ns, s));
    LPA_TRY(dev_alloc(g, (void**)&g->crow, sizeof(int32_t) * arcs));
    hipLaunchKernelGGL(k_keys_to_col, dim3(grid_for(arcs)), dim3(256), 0, s, keys, arcs, g->col, g->crow,
                       H > 0 ? (u32)((1ull << blo) - 1ull) : ~0u);
    LPA_HIP(hipGetLastError());
    if (H > 0) LPA_TRY(build_pieces(g, H));
    // CSC position index over this rank's arcs (for the replicated-label refresh)
    if (arcs >= (int64_t)UINT32_MAX) {
      set_error("%lld arcs on one rank exceed the 32-bit position index", (long long)arcs);
      return LPA_EINVAL;
    }
    int32_t* colcnt = nullptr;
    LPA_TRY(scratch_alloc(g, (void**)&colcnt, sizeof(int32_t) * g->vpad));
    if (P == 1) {
      // one rank: column u occurs once per arc of u, i.e. deg_own[u] times
      LPA_HIP(hipMemcpyAsync(colcnt, deg_own, sizeof(int32_t) * g->vpad, hipMemcpyDeviceToDevice, s));
      hipLaunchKernelGGL(k_csc_keys, dim3(grid_for(arcs)), dim3(256), 0, s, g->col, arcs, keys, (int32_t*)nullptr);
    } else {
      LPA_HIP(hipMemsetAsync(colcnt, 0, sizeof(int32_t) * g->vpad, s));
      hipLaunchKernelGGL(k_csc_keys, dim3(cap_bh(grid_for(arcs))), dim3(256), 0, s, g->col, arcs, keys, colcnt);
    }
    LPA_HIP(hipGetLastError());
    int cs[8], ncs = 0;
    for (int b = 0; b < bits_for((uint64_t)(g->vpad - 1)); b += 8) cs[ncs++] = 32 + b;
    LPA_TRY(radix_sort_u64(keys, keys + arcs, arcs, cs, ncs, s));
    LPA_TRY(dev_alloc(g, (void**)&g->cptr, sizeof(int64_t) * (g->vpad + 1)));
    LPA_TRY(exclusive_scan_i32_i64(colcnt, g->cptr, g->vpad, s));
    LPA_TRY(dev_alloc(g, (void**)&g->cpos, sizeof(uint32_t) * arcs));
    hipLaunchKernelGGL(k_keys_to_pos, dim3(grid_for(arcs)), dim3(256), 0, s, keys, arcs, g->cpos);
    LPA_HIP(hipGetLastError());
    // static scatter chunks (colcnt is reused for the per-column chunk counts)
    hipLaunchKernelGGL(k_col_chunks, dim3(grid_for(g->vpad)), dim3(256), 0, s, colcnt, g->vpad, colcnt);
    LPA_HIP(hipGetLastError());
    LPA_TRY(dev_alloc(g, (void**)&g->cch, sizeof(int64_t) * (g->vpad + 1)));
    LPA_TRY(exclusive_scan_i32_i64(colcnt, g->cch, g->vpad, s));
    LPA_HIP(hipMemcpyAsync(&g->n_chunks, g->cch + g->vpad, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    LPA_TRY(dev_alloc(g, (void**)&g->cowner, sizeof(int32_t) * (g->n_chunks > 0 ? g->n_chunks : 1)));
    {
      // multi-chunk columns are the high-degree ones, i.e. the first slots at P = 1:
      // the scatter scans the chunk flags only up to the last such column's chunks
      unsigned long long* d_end = nullptr;
      LPA_TRY(scratch_alloc(g, (void**)&d_end, sizeof(unsigned long long)));
      LPA_HIP(hipMemsetAsync(d_end, 0, sizeof(unsigned long long), s));
      hipLaunchKernelGGL(k_chunk_owner, dim3(grid_for(g->vpad)), dim3(256), 0, s, g->cch, g->vpad,
                         g->cowner, d_end);
      LPA_HIP(hipGetLastError());
      unsigned long long h_end = 0;
      LPA_HIP(hipMemcpyAsync(&h_end, d_end, sizeof(h_end), hipMemcpyDeviceToHost, s));
      LPA_HIP(hipStreamSynchronize(s));
      scratch_free(g, d_end);
      g->n_chunk_scan = (int64_t)h_end;
    }
    scratch_free(g, colcnt);
    scratch_free(g, keys);
  } else {
    LPA_TRY(dev_alloc(g, (void**)&g->cptr, sizeof(int64_t) * (g->vpad + 1)));
    LPA_HIP(hipMemsetAsync(g->cptr, 0, sizeof(int64_t) * (g->vpad + 1), s));
    LPA_TRY(dev_alloc(g, (void**)&g->cpos, sizeof(uint32_t)));
    LPA_TRY(dev_alloc(g, (void**)&g->cch, sizeof(int64_t) * (g->vpad + 1)));
    LPA_HIP(hipMemsetAsync(g->cch, 0, sizeof(int64_t) * (g->vpad + 1), s));
    LPA_TRY(dev_alloc(g, (void**)&g->cowner, sizeof(int32_t)));
    g->n_chunks = 0;
  }
  return finish_build(g, deg_own, m);
}


// The outlier stage's L2 sub-graph (E' = the distinct (s, d) with
// L[s] == L[d], Graphframes.py:121-128) built without sorting arcs: the parent's distinct
// edges are kept in (s, d) order (de_keys) and in (d, s) order (de_t), so a row's intra
// arcs are a filter of its two runs -- marks, two exclusive scans, the degrees as
// segment-length differences (no per-vertex atomics), the degree-ranked slot order (a
// sort of V keys), then every arc written at its final position, with its CSC twin.
// Rows keep their columns in run order (cols_sorted = false: no column-run superstep).
int build_graph_l2(lpa_graph* g, const lpa_graph* parent, const int32_t* L, const uint8_t* mo_pre) {
  hipStream_t s = g->stream;
  const int32_t V = (int32_t)parent->V;
  const int64_t md = parent->de_n;
  g->V = V;
  g->slice = ((int64_t)V + 63) / 64 * 64;
  if (g->slice == 0) g->slice = 64;
  g->vpad = g->slice;
  g->own_begin = 0;
  g->cols_sorted = false;
  const int64_t S = g->slice;
  uint8_t *mo = nullptr, *mi = nullptr;
  int32_t *dout = nullptr, *d_max = nullptr;
  uint32_t *pos_out = nullptr, *pos_in = nullptr;
  if (!mo_pre) LPA_TRY(scratch_alloc(g, (void**)&mo, md > 0 ? md : 1));
  LPA_TRY(scratch_alloc(g, (void**)&mi, md > 0 ? md : 1));
  LPA_TRY(scratch_alloc(g, (void**)&pos_out, sizeof(uint32_t) * (md + 1)));
  LPA_TRY(scratch_alloc(g, (void**)&pos_in, sizeof(uint32_t) * (md + 1)));
  LPA_TRY(scratch_alloc(g, (void**)&dout, sizeof(int32_t) * (V > 0 ? V : 1)));
  LPA_TRY(scratch_alloc(g, (void**)&d_max, sizeof(int32_t)));
  LPA_TRY(dev_alloc(g, (void**)&g->deg, sizeof(int32_t) * (V > 0 ? V : 1)));
  const uint8_t* mo_c = mo_pre ? mo_pre : mo;
  if (md > 0) {
    if (!mo_pre) hipLaunchKernelGGL(k_l2_mark_out, dim3(grid_for(md)), dim3(256), 0, s, parent->de_keys, md, L, mo);
    hipLaunchKernelGGL(k_l2_mark_in, dim3(grid_for(md)), dim3(256), 0, s, parent->de_t, parent->de_ts, md, L, mi);
    LPA_HIP(hipGetLastError());
  }
  LPA_TRY(exclusive_scan_u8_u32(mo_c, pos_out, md, s));
  LPA_TRY(exclusive_scan_u8_u32(mi, pos_in, md, s));
  LPA_HIP(hipMemsetAsync(d_max, 0, sizeof(int32_t), s));
  if (V > 0) {
    hipLaunchKernelGGL(k_l2_degree, dim3(grid_for(V)), dim3(256), 0, s, parent->de_out_off, parent->de_in_off,
                       pos_out, pos_in, (int64_t)V, g->deg, dout);
    hipLaunchKernelGGL(k_maxdeg, dim3(grid_for(V) < 1024u ? grid_for(V) : 1024u), dim3(256), 0, s, g->deg,
                       (int64_t)V, d_max);
    LPA_HIP(hipGetLastError());
  }
  uint32_t m2u = 0;
  LPA_HIP(hipMemcpyAsync(&m2u, pos_out + md, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipMemcpyAsync(&g->max_degree, d_max, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  const int64_t m2 = (int64_t)m2u;
  g->m = m2;
  scratch_free(g, d_max);

  // ---- degree-ranked slots, row offsets ----
  LPA_TRY(vertex_order(g, V, m2, false));
  int32_t* deg_own = nullptr;
  LPA_TRY(scratch_alloc(g, (void**)&deg_own, sizeof(int32_t) * S));
  hipLaunchKernelGGL(k_owned_degree, dim3(grid_for(S)), dim3(256), 0, s, g->old_of, g->deg, S, deg_own);
  LPA_HIP(hipGetLastError());
  LPA_TRY(dev_alloc(g, (void**)&g->rp, sizeof(int64_t) * (S + 1)));
  LPA_TRY(exclusive_scan_i32_i64(deg_own, g->rp, S, s));
  const int64_t arcs = 2 * m2;
  g->arcs = arcs;
  if (arcs >= (int64_t)UINT32_MAX) {
    set_error("%lld arcs in the L2 sub-graph exceed the 32-bit position index", (long long)arcs);
    return LPA_EINVAL;
  }

  // ---- arcs at their final positions ----
  // No CSC position index: the sub-graph runs 5 supersteps, the first two label-dense,
  // and every refresh rebuilds al[] (no_scatter).  Its twins (cpos) would cost one random
  // read and one random write per edge into GB-sized arrays (16.8 ms at C3, more than
  // the rebuilds they save); the frontier is off with it (every refresh is a rebuild).
  g->no_scatter = true;
  // no captured superstep graphs: a handle that lives for 5 supersteps pays their capture,
  // instantiation and destruction (~8 ms of host time at C3) for ~1 ms of launches
  g->use_graphs = 0;
  LPA_TRY(dev_alloc(g, (void**)&g->col, sizeof(int32_t) * (arcs > 0 ? arcs : 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->al, sizeof(int32_t) * (arcs > 0 ? arcs : 1)));
  LPA_TRY(dev_alloc(g, (void**)&g->cptr, sizeof(int64_t) * (g->vpad + 1)));
  LPA_HIP(hipMemcpyAsync(g->cptr, g->rp, sizeof(int64_t) * (S + 1), hipMemcpyDeviceToDevice, s));
  if (md > 0) {
    hipLaunchKernelGGL(k_l2_emit_out, dim3(grid_for(md)), dim3(256), 0, s, parent->de_keys, md, mo_c, pos_out,
                       parent->de_out_off, g->new_of, g->rp, g->col, g->al);
    hipLaunchKernelGGL(k_l2_emit_in, dim3(grid_for(md)), dim3(256), 0, s, parent->de_t, parent->de_ts, md, mi,
                       pos_in, parent->de_in_off, dout, g->new_of, g->rp, g->col, g->al);
    LPA_HIP(hipGetLastError());
  }
  g->al_is_l0 = true;   // init_labels (finish_build) needs no rebuild
  if (mo) scratch_free(g, mo);
  scratch_free(g, mi);
  scratch_free(g, pos_out);
  scratch_free(g, pos_in);
  scratch_free(g, dout);
  // empty scatter-chunk tables (no column has a chunk: the diff queues nothing)
  LPA_TRY(dev_alloc(g, (void**)&g->cpos, sizeof(uint32_t)));
  LPA_TRY(dev_alloc(g, (void**)&g->cch, sizeof(int64_t) * (g->vpad + 1)));
  LPA_HIP(hipMemsetAsync(g->cch, 0, sizeof(int64_t) * (g->vpad + 1), s));
  LPA_TRY(dev_alloc(g, (void**)&g->cowner, sizeof(int32_t)));
  g->n_chunks = 0;
  g->n_chunk_scan = 0;
  return finish_build(g, deg_own, m2);
}

}  // namespace lpa
