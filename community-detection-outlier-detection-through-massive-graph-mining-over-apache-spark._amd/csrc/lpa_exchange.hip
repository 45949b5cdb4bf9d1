// Multi-GPU label exchange: after each superstep's tally every
// rank holds the new labels of its own slice; every replica must receive them.
//
//   full   ncclAllGather of the owned slices (4 V (P-1)/P bytes received per
//          rank): the label-dense supersteps right after L0, where most labels
//          change anyway.
//   delta  each rank compacts the (slot, label) pairs of its CHANGED owned
//          vertices; the per-rank counts are allgathered and read on the host,
//          then ncclAllGather moves max-count entries per rank (8 B each).
//          Converged supersteps change ~0.3 % of the vertices (R-MAT-24,
//          superstep 4+), so the exchange shrinks by ~2 orders of magnitude.
//          Chosen when the largest delta is <= slice / 4 (its bytes <= 1/2 of the
//          full slice).
//   giant  (round 4) the giant label G (k_giant_pick of the current vector, the same on
//          every rank) carries most of the new labels once LPA collapses: each rank
//          sends the bitmap (label == G) of its slice (1/32 of the slice's bytes) and
//          its CHANGED non-G labels as (slot, label) entries; a receiver writes G where
//          the bit is set, keeps its current label elsewhere, then applies the entries.
//          R-MAT (oracle, scale 22): superstep 2 1.7 B per vertex instead of 4 (full),
//          superstep 3 0.16 instead of 1.6 (delta); Chung-Lu superstep 3 0.4 instead of 4.
// Each superstep after the first allgathers one (delta, giant) count pair per rank and
// the host takes the form of fewest bytes among those that fit (delta and giant entries
// <= slice / 4 per rank).  All give the identical full label vector, so the mode never
// affects labels.
//   posted (round 5) after a delta exchange of few entries the next delta goes out at a
//          capacity fixed from the last counts (twice the largest, identical on every
//          rank) BEFORE the host reads the new counts, with its apply and the refresh's
//          change chunks queued behind it: the GPU works through the host's read instead
//          of idling.  Kernels that find a count above the capacity stand down on the
//          device and the host, reading the same counts, exchanges again in the form
//          that fits.
//
// Completing the next-label buffer Ln after a delta exchange.  Ln (the ping-pong
// partner of the current vector Lc = L_t) holds, outside the own slice, L_t if the
// previous exchange was a delta too (k_delta_finish writes every entry into both
// buffers, so they agree afterwards), else L_{t-1} and the other slices are first
// copied from Lc.  Applying the gathered E_{t+1} then gives L_{t+1}; E_{t+1} is also the
// list of changed vertices, so the al[] refresh takes its position chunks from it
// instead of diffing the whole vector.
#include <algorithm>
#include <climits>

#include "lpa_internal.h"

namespace lpa {

namespace {

// changed owned slots -> dsend[] = (local slot << 32 | new label); dcount = count.
// Block-aggregated: one global atomic per block.
__global__ __launch_bounds__(256) void k_delta_compact(const int32_t* __restrict__ Lc_own,
                                                       const int32_t* __restrict__ Ln_own,
                                                       int64_t slice, u64* __restrict__ dsend,
                                                       unsigned long long* __restrict__ dcount) {
  __shared__ int wsum[4];
  __shared__ unsigned long long base_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t i0 = (int64_t)blockIdx.x * 256; i0 < slice; i0 += (int64_t)gridDim.x * 256) {
    const int64_t i = i0 + threadIdx.x;
    int32_t nv = 0;
    bool chg = false;
    if (i < slice) {
      nv = Ln_own[i];
      chg = nv != Lc_own[i];
    }
    const u64 m = __ballot(chg);
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < w) before += wsum[k];
      tot += wsum[k];
    }
    if (threadIdx.x == 0 && tot) base_s = atomicAdd(dcount, (unsigned long long)tot);
    __syncthreads();
    if (chg) {
      const u64 pos = base_s + before + __popcll(m & ((1ull << lane) - 1ull));
      dsend[pos] = ((u64)(uint32_t)i << 32) | (u64)(uint32_t)nv;
    }
    __syncthreads();  // wsum / base_s reused by the next tile
  }
}

// this rank's changed owned slots -> dsend (slot << 32 | label), count xpair[0]; the
// changed ones whose new label is not G -> gsend, count xpair[1]; bit i of the slice's
// bitmap = (new label == G).  One streaming pass: a wave takes kCompactWords bitmap
// words (64 slots each, one coalesced 256-B load per buffer and word, all issued before
// the first compare), a ballot per word; only a wave with changes reserves its entries
// (one atomic per list).  The slice is a multiple of 64 slots.  Entry order differs
// from run to run; every consumer applies them as a set (distinct slots).
// Converged supersteps (flist given): when the tally walked its frontier lists (*fr_all
// == 0, no settle), only the listed rows can have changed -- every other owned row's
// output slot already holds its label -- so the pass walks the lists instead of the
// slice; it writes no bitmap then and marks the giant form unavailable (a giant count
// above any capacity in xpair[1]).
constexpr int kCompactWords = 8;
constexpr int kTriple = 3;   // per-rank words of the count exchange: delta, giant, posted request
constexpr unsigned long long kNoGiantForm = 1ull << 62;
struct ListBounds {
  int64_t b[LPA_NBINS + 1];
};
__global__ __launch_bounds__(256) void k_exch_compact(const int32_t* __restrict__ Lc_own,
                                                      const int32_t* __restrict__ Ln_own, int64_t slice,
                                                      const int32_t* __restrict__ gword,
                                                      u64* __restrict__ dsend, u64* __restrict__ gsend,
                                                      unsigned long long* __restrict__ xpair,
                                                      unsigned long long* __restrict__ bm_own,
                                                      const int32_t* __restrict__ flist,
                                                      const int32_t* __restrict__ fcnt,
                                                      const int32_t* __restrict__ fr_all, ListBounds lb,
                                                      long long post_req) {
  const int lane = threadIdx.x & 63;
  const u64 lt = (1ull << lane) - 1ull;
  // this rank's posted-capacity request (lpa_set_posted) rides in the count triple, so
  // every rank derives the next posted capacity from the same gathered values
  if (blockIdx.x == 0 && threadIdx.x == 0) xpair[2] = (unsigned long long)post_req;
  if (flist != nullptr && *fr_all == 0 && fcnt[kFcntSettled] == 0) {   // uniform
    if (blockIdx.x == 0 && threadIdx.x == 0) xpair[1] = kNoGiantForm;
    int64_t total = 0;
    for (int b = 0; b < BIN_ISO; ++b) total += fcnt[b];
    for (int64_t i0 = (int64_t)blockIdx.x * 256 + (threadIdx.x & ~63); i0 < total; i0 += (int64_t)gridDim.x * 256) {
      const int64_t i = i0 + lane;
      bool chg = false;
      int64_t v = 0;
      int32_t nv = 0;
      if (i < total) {
        int64_t acc = 0;
        int b = 0;
        while (i >= acc + fcnt[b]) acc += fcnt[b++];
        v = flist[lb.b[b] + (i - acc)];
        nv = Ln_own[v];
        chg = nv != Lc_own[v];
      }
      const u64 m = __ballot(chg);
      if (m == 0) continue;   // wave-uniform
      unsigned long long base = 0;
      if (lane == 0) base = atomicAdd(&xpair[0], (unsigned long long)__popcll(m));
      base = __shfl(base, 0, 64);
      if (chg) dsend[base + __popcll(m & lt)] = ((u64)(uint32_t)v << 32) | (u64)(uint32_t)nv;
    }
    return;
  }
  const int32_t G = gword[0];
  const int64_t nwords = slice >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t w0 = wave * kCompactWords; w0 < nwords; w0 += nwaves * kCompactWords) {
    int32_t nv[kCompactWords], ov[kCompactWords];
#pragma unroll
    for (int k = 0; k < kCompactWords; ++k) {
      // a word past the slice re-reads word 0 (valid address; masked below)
      const int64_t i = ((w0 + k < nwords) ? (w0 + k) : 0) * 64 + lane;
      nv[k] = Ln_own[i];
      ov[k] = Lc_own[i];
    }
    u64 m[kCompactWords], mg[kCompactWords], bmw = 0;
    int cnt = 0, gcnt = 0;
#pragma unroll
    for (int k = 0; k < kCompactWords; ++k) {
      const bool in = w0 + k < nwords;
      const bool chg = in && nv[k] != ov[k], isg = in && nv[k] == G;
      m[k] = __ballot(chg);
      mg[k] = __ballot(chg && !isg);
      const u64 mb = __ballot(isg);
      bmw = lane == k ? mb : bmw;
      cnt += __popcll(m[k]);
      gcnt += __popcll(mg[k]);
    }
    if (lane < kCompactWords && w0 + lane < nwords) bm_own[w0 + lane] = bmw;
    if (cnt == 0) continue;   // wave-uniform
    unsigned long long base = 0, gbase = 0;
    if (lane == 0) {
      base = atomicAdd(&xpair[0], (unsigned long long)cnt);
      if (gcnt) gbase = atomicAdd(&xpair[1], (unsigned long long)gcnt);
    }
    base = __shfl(base, 0, 64);
    gbase = __shfl(gbase, 0, 64);
#pragma unroll
    for (int k = 0; k < kCompactWords; ++k) {
      const u64 e = ((u64)(uint32_t)((w0 + k) * 64 + lane) << 32) | (u64)(uint32_t)nv[k];
      if ((m[k] >> lane) & 1ull) dsend[base + __popcll(m[k] & lt)] = e;
      if ((mg[k] >> lane) & 1ull) gsend[gbase + __popcll(mg[k] & lt)] = e;
      base += __popcll(m[k]);
      gbase += __popcll(mg[k]);
    }
  }
}

// Ln outside the own slice after a giant exchange: G where the sender's bit is set, the
// current label elsewhere (the changed non-G entries are applied next); one bitmap word
// per 64 slots, int4 stores
__global__ void k_giant_apply(const int4* __restrict__ Lc, int4* __restrict__ Ln,
                              const unsigned long long* __restrict__ bm, int64_t n4, int64_t own4_begin,
                              int64_t own4_end, const int32_t* __restrict__ gword) {
  const int32_t G = gword[0];
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    if (q >= own4_begin && q < own4_end) continue;
    const u32 b = (u32)(bm[q >> 4] >> ((q & 15) * 4)) & 0xFu;
    int4 v = Lc[q];
    if (b & 1u) v.x = G;
    if (b & 2u) v.y = G;
    if (b & 4u) v.z = G;
    if (b & 8u) v.w = G;
    Ln[q] = v;
  }
}

// Ln[i] = Lc[i] for every slot outside [own_begin, own_begin + slice) (int4; slices
// are multiples of 64 slots)
__global__ void k_copy_other(const int4* __restrict__ Lc, int4* __restrict__ Ln, int64_t n4,
                             int64_t own4_begin, int64_t own4_end) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
       q += (int64_t)gridDim.x * blockDim.x)
    if (q < own4_begin || q >= own4_end) Ln[q] = Lc[q];
}

// Posted form (spec != 0): the entries were gathered at a capacity fixed before the
// counts were known; if any rank's count exceeds it the kernel does nothing (the host,
// reading the same counts, then runs the exchange again in a form that fits).
// counts[r * cs]: rank r's count (cs = 2 on the gathered (delta, giant) pairs).
__device__ __forceinline__ bool posted_overflow(const unsigned long long* __restrict__ counts, int cs,
                                                int32_t P, int64_t cap) {
  bool ovf = false;
  for (int r = 0; r < P; ++r) ovf |= (int64_t)counts[(int64_t)r * cs] > cap;
  return ovf;
}

// apply gathered entries (rank r's: drecv[r * cap, r * cap + counts[r * cs])) to Ln,
// except those of rank `skip` (its slice of Ln is the tally output already): the
// giant form's changed non-G labels
__global__ void k_delta_apply(const u64* __restrict__ drecv, const unsigned long long* __restrict__ counts,
                              int cs, int64_t cap, int32_t P, int32_t skip, int64_t slice,
                              int32_t* __restrict__ Ln) {
  const int64_t tot = cap * P;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < tot;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = k / cap, j = k - r * cap;
    if (r != skip && j < (int64_t)counts[r * cs]) {
      const u64 e = drecv[k];
      Ln[r * slice + (int64_t)(e >> 32)] = (int32_t)(uint32_t)e;
    }
  }
}

// A delta exchange's whole device side in one pass over the gathered entries: every
// entry is written into BOTH label buffers -- Ln (the new vector; not for the own
// rank, whose slice is the tally output) and Lc (the current one, every rank's: the
// next superstep writes its owned rows into Lc and, frontier, a row it skips must
// already hold its label there, as k_diff's Lsync) -- so after a delta exchange the two
// buffers agree and the next delta needs no re-apply of this one; and the changes
// become flagged al[] scatter chunks + the dirty-arc count (k_diff's output, from the
// change list instead of a scan of the whole vector).
__global__ __launch_bounds__(256) void k_delta_finish(const u64* __restrict__ drecv,
                                                      const unsigned long long* __restrict__ counts, int cs,
                                                      int64_t cap, int32_t P, int64_t slice,
                                                      const int64_t* __restrict__ cptr,
                                                      const int64_t* __restrict__ cch,
                                                      uint8_t* __restrict__ chflag,
                                                      int32_t* __restrict__ chlist,
                                                      unsigned long long* __restrict__ counters,
                                                      int32_t own, int32_t* __restrict__ Lc,
                                                      int32_t* __restrict__ Ln, int spec) {
  if (spec && posted_overflow(counts, cs, P, cap)) return;
  const int lane = threadIdx.x & 63;
  const int64_t tot = cap * P;
  unsigned long long dirty = 0;
  for (int64_t k0 = (int64_t)blockIdx.x * blockDim.x; k0 < tot; k0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = k0 + threadIdx.x;
    bool one = false;
    int64_t u = 0;
    if (k < tot) {
      const int64_t r = k / cap, j = k - r * cap;
      if (j < (int64_t)counts[r * cs]) {
        const u64 e = drecv[k];
        u = r * slice + (int64_t)(e >> 32);
        const int32_t lab = (int32_t)(uint32_t)e;
        Lc[u] = lab;
        if (r != own) Ln[u] = lab;
        dirty += (unsigned long long)(cptr[u + 1] - cptr[u]);
        const int64_t nch = cch[u + 1] - cch[u];
        one = nch == 1;
        for (int64_t c = cch[u]; nch > 1 && c < cch[u + 1]; ++c) chflag[c] = 1;
      }
    }
    // one-chunk columns -> the scatter's list (one atomic per wave)
    const u64 om = __ballot(one);
    unsigned long long base = 0;
    if (lane == 0 && om) base = atomicAdd(&counters[0], (unsigned long long)__popcll(om));
    base = __shfl(base, 0, 64);
    if (one) chlist[base + __popcll(om & ((1ull << lane) - 1ull))] = (int32_t)u;
  }
  for (int off = 32; off > 0; off >>= 1) dirty += __shfl_xor(dirty, off, 64);
  if (lane == 0 && dirty) atomicAdd(&counters[1], dirty);
}

inline unsigned grid_of(int64_t n, int64_t cap) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  return (unsigned)(b < cap ? b : cap);
}

}  // namespace

int exchange_alloc(lpa_graph* g) {
  if (!exchanges(g)) return LPA_OK;
  g->dcap = g->slice / 4;
  if (g->dcap < 1) g->dcap = 1;
  const int64_t P = g->nranks;
  LPA_TRY(dev_alloc(g, (void**)&g->dsend, sizeof(u64) * g->slice));
  LPA_TRY(dev_alloc(g, (void**)&g->drecv, sizeof(u64) * g->dcap * P));
  LPA_TRY(dev_alloc(g, (void**)&g->dcount, sizeof(unsigned long long) * (1 + P)));
  LPA_TRY(dev_alloc(g, (void**)&g->gsend, sizeof(u64) * g->slice));
  LPA_TRY(dev_alloc(g, (void**)&g->gbm, sizeof(unsigned long long) * (g->slice / 64) * P));
  LPA_TRY(dev_alloc(g, (void**)&g->xpair, sizeof(unsigned long long) * kTriple * (1 + P)));
  LPA_HIP(hipHostMalloc((void**)&g->h_dcounts, sizeof(unsigned long long) * kTriple * P, hipHostMallocDefault));
  LPA_HIP(hipEventCreateWithFlags(&g->cnt_ev, hipEventDisableTiming));
  g->prev_delta_ok = false;
  return LPA_OK;
}

void exchange_free(lpa_graph* g) {
  if (g->h_dcounts) (void)hipHostFree(g->h_dcounts);
  g->h_dcounts = nullptr;
  if (g->cnt_ev) (void)hipEventDestroy(g->cnt_ev);
  g->cnt_ev = nullptr;
}

u64* exchange_recv_buf(lpa_graph* g) { return g->drecv; }
unsigned long long* exchange_recv_counts(lpa_graph* g) { return g->dcount + 1; }

// compact this rank's changed owned labels (Lc -> Ln) into dsend; count -> dcount[0]
int exchange_compact(lpa_graph* g, const int32_t* Lc, const int32_t* Ln) {
  hipStream_t s = g->stream;
  LPA_HIP(hipMemsetAsync(g->dcount, 0, sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_delta_compact, dim3(grid_of(g->slice, 4096)), dim3(256), 0, s,
                     Lc + g->own_begin, Ln + g->own_begin, g->slice, g->dsend, g->dcount);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// Ln := L_{t+1} from the gathered changes in the current receive buffer (cap entries
// per rank, counts[r * cs]) -- see the header; Lc gets them too (the buffers agree
// afterwards), and the al[] position chunks of the changes are queued (counters of
// parity `par`, the superstep's).  posted: the entries were
// gathered at the fixed capacity `cap` before the counts were read (the kernel stands
// down on the device if a count exceeds it; the host bookkeeping is then left as it was).
int exchange_finish_delta(lpa_graph* g, int32_t* Lc, int32_t* Ln, int64_t cap, int par,
                          const unsigned long long* counts, int cs, bool posted) {
  hipStream_t s = g->stream;
  const int P = g->nranks;
  const int64_t n4 = g->vpad / 4;
  if (!g->prev_delta_ok) {
    // the last exchange was not a delta: Ln outside the own slice still holds L_{t-1}
    hipLaunchKernelGGL(k_copy_other, dim3(grid_of(n4, 8192)), dim3(256), 0, s, (const int4*)Lc,
                       (int4*)Ln, n4, g->own_begin / 4, (g->own_begin + g->slice) / 4);
    LPA_HIP(hipGetLastError());
  }
  if (cap > 0) {
    hipLaunchKernelGGL(k_delta_finish, dim3(grid_of(cap * P, 4096)), dim3(256), 0, s, exchange_recv_buf(g),
                       counts, cs, cap, P, g->slice, g->cptr, g->cch, g->chflag, g->chlist,
                       g->counters + 4 * par, g->rank, Lc, Ln, posted ? 1 : 0);
    LPA_HIP(hipGetLastError());
  }
  if (!posted) g->prev_delta_ok = true;
  return LPA_OK;
}

// capacity of the next posted delta: twice the last largest count, at least kPostMin,
// power of two; none above kPostMax entries per rank (label-dense supersteps exchange
// the exact count) or beyond the delta buffers
constexpr int64_t kPostMin = 1024, kPostMax = 1 << 17;
static int64_t posted_cap(const lpa_graph* g, int64_t capd) {
  int64_t c = kPostMin;
  while (c < 2 * capd) c *= 2;
  return c <= kPostMax && c <= g->dcap ? c : 0;
}
// ... agreed over the ranks: every rank's request (its lpa_set_posted value, gathered
// with the counts: < 0 adaptive, 0 off, > 0 fixed) gives a capacity, the smallest wins.
// Computed from gathered values only, so every rank posts the same allgather size even
// when one rank alone calls lpa_set_posted, or calls it with another value
static int64_t agreed_post_cap(const lpa_graph* g, int64_t capd) {
  int64_t c = INT64_MAX;
  for (int k = 0; k < g->nranks; ++k) {
    const int64_t req = (int64_t)g->h_dcounts[kTriple * k + 2];
    c = std::min(c, req < 0 ? posted_cap(g, capd) : std::min(req, g->dcap));
  }
  return c == INT64_MAX ? 0 : c;
}

// In-library exchange of one superstep (P > 1, RCCL communicator or loopback group):
// Lown = Ln + own_begin holds the new owned labels; on return Ln holds the full new
// label vector.  *changes_listed: the refresh's position chunks were queued from the delta.
// first: the superstep right after L0 (every label changes: full, no count round trip).
int exchange_collective(lpa_graph* g, const int32_t* Lc, int32_t* Ln, bool first, bool* changes_listed) {
  hipStream_t s = g->stream;
  int32_t* Lown = Ln + g->own_begin;
  const int P = g->nranks;
  const int64_t S = g->slice, wpr = S / 64;   // bitmap words per rank
  *changes_listed = false;
  if (!first) {
    LPA_HIP(hipMemsetAsync(g->xpair, 0, 2 * sizeof(unsigned long long), s));   // [2]: the kernel
    // converged supersteps: the frontier lists of this superstep's tally (g->par)
    const bool list_mode = g->since_reset >= kDenseSupersteps + 2;
    ListBounds lbd;
    for (int b = 0; b <= LPA_NBINS; ++b) lbd.b[b] = g->bin_begin[b];
    hipLaunchKernelGGL(k_exch_compact, dim3(grid_of(S / kCompactWords, 4096)), dim3(256), 0, s, Lc + g->own_begin,
                       Lown, S,
                       g->gword, g->dsend, g->gsend, g->xpair, g->gbm + (int64_t)g->rank * wpr,
                       list_mode ? g->flist : (const int32_t*)nullptr, g->fcnt + 16 * g->par, g->fr_all + g->par, lbd,
                       (long long)g->post_fixed);
    LPA_HIP(hipGetLastError());
    LPA_TRY(coll_allgather(g, g->xpair, g->xpair + kTriple, kTriple, 8, s));
    // rank r: (delta count, giant count, posted request) at 3r, 3r + 1, 3r + 2
    const unsigned long long* pairs = g->xpair + kTriple;
    LPA_HIP(hipMemcpyAsync(g->h_dcounts, pairs, sizeof(unsigned long long) * kTriple * P, hipMemcpyDeviceToHost, s));
    LPA_HIP(hipEventRecord(g->cnt_ev, s));
    // Posted delta (converged supersteps, after a delta exchange of few entries): the
    // entries go out at a capacity fixed from the last counts and requests (the same on
    // every rank: agreed_post_cap), and their apply + the refresh's change chunks are
    // queued behind them BEFORE the host waits for the counts, so the GPU keeps working
    // through the host's read.  A count above the capacity makes the queued kernel stand
    // down; the host then sees the same counts and exchanges again below in the form that
    // fits.
    const int64_t post = g->prev_delta_ok ? g->post_cap : 0;
    if (post > 0) {
      LPA_TRY(coll_allgather(g, g->dsend, exchange_recv_buf(g), (size_t)post, 8, s));
      LPA_TRY(exchange_finish_delta(g, const_cast<int32_t*>(Lc), Ln, post, g->par, pairs, kTriple, true));
    }
    LPA_HIP(hipEventSynchronize(g->cnt_ev));
    int64_t capd = 0, capg = 0;
    for (int k = 0; k < P; ++k) {
      capd = std::max(capd, (int64_t)g->h_dcounts[kTriple * k]);
      capg = std::max(capg, (int64_t)g->h_dcounts[kTriple * k + 1]);
    }
    if (post > 0) {
      if (capd <= post) {
        g->last_exchange_delta = capd;
        g->post_cap = agreed_post_cap(g, capd);
        ++g->n_exch_delta;
        ++g->n_exch_posted;
        *changes_listed = true;
        return LPA_OK;
      }
      ++g->n_exch_post_missed;   // the queued kernel stood down
    }
    // bytes every rank receives per form (the full slice otherwise)
    const int64_t full_b = 4 * S;
    const int64_t delta_b = capd <= g->dcap ? 8 * capd : INT64_MAX;
    const int64_t giant_b = capg <= g->dcap ? 8 * wpr + 8 * capg : INT64_MAX;
    if (delta_b <= giant_b && delta_b < full_b) {
      if (capd > 0) LPA_TRY(coll_allgather(g, g->dsend, exchange_recv_buf(g), (size_t)capd, 8, s));
      g->last_exchange_delta = capd;
      g->post_cap = agreed_post_cap(g, capd);
      ++g->n_exch_delta;
      *changes_listed = true;
      return exchange_finish_delta(g, const_cast<int32_t*>(Lc), Ln, capd, g->par, pairs, kTriple);
    }
    if (giant_b < full_b) {
      // in place: rank r's bitmap words at gbm + r * wpr
      LPA_TRY(coll_allgather(g, g->gbm + (int64_t)g->rank * wpr, g->gbm, (size_t)wpr, 8, s));
      u64* ent = exchange_recv_buf(g);
      if (capg > 0) LPA_TRY(coll_allgather(g, g->gsend, ent, (size_t)capg, 8, s));
      const int64_t n4 = g->vpad / 4;
      hipLaunchKernelGGL(k_giant_apply, dim3(grid_of(n4, 8192)), dim3(256), 0, s, (const int4*)Lc, (int4*)Ln,
                         g->gbm, n4, g->own_begin / 4, (g->own_begin + S) / 4, g->gword);
      LPA_HIP(hipGetLastError());
      if (capg > 0) {
        hipLaunchKernelGGL(k_delta_apply, dim3(grid_of(capg * P, 8192)), dim3(256), 0, s, ent, pairs + 1, kTriple, capg,
                           P, g->rank, S, Ln);
        LPA_HIP(hipGetLastError());
      }
      g->last_exchange_delta = -2;
      ++g->n_exch_giant;
      g->prev_delta_ok = false;   // Ln is the full new vector; no delta chain to continue
      return LPA_OK;
    }
  }
  // full: in-place allgather of the owned slices (rank r's slice at Ln + r * slice)
  LPA_TRY(coll_allgather(g, Lown, Ln, (size_t)S, 4, s));
  g->last_exchange_delta = -1;
  ++g->n_exch_full;
  g->prev_delta_ok = false;
  return LPA_OK;
}

}  // namespace lpa
