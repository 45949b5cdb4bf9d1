// Hub combine: the mode of a row longer than one segment (deg > kSegArcs).
//
// k_lpa_units tallies each 512-arc unit of a seg-bin row (one wave) and leaves
// the unit's tally words (count << 32 | ~label) in the unit's staging slots
// (ucnt[unit] words at stage[unit begin ...)).  This file merges the units of a
// row, T_h words in all (SURVEY.md §7
// "lpa_hub_bin": block LDS hash with a global spill; here the spill is a
// bucket-partitioned staging area instead of a global hash, because random
// 64-bit global atomics run at ~20 G lanes/s on MI355X while block-aggregated
// partitioning streams).  Three regimes, chosen per hub on the device from T_h:
//
//   T <= 512            k_hub_small   one wave: words in registers, weighted
//                                     ballot peel, residual in a per-wave LDS table
//                                     (converged rows: one word per unit)
//   512 < T <= 6144     k_hub_mid     one block: LDS table of 2048 / 4096 / 8192
//                                     slots for T <= 1024 / 2048 / 6144
//   T > 6144            K = 2^ceil(log2(T / 2048)) label-hash buckets:
//                       k_hub_count   per 8-unit chunk: bucket histogram
//                       k_hub_scan    per hub: bucket offsets
//                       k_hub_scatter per chunk: words -> bucket-contiguous runs
//                       k_hub_bucket  per (hub, bucket): LDS tally -> atomicMax
//                       k_hub_final   per hub: write the label, reset
//
// Every label's votes fall in exactly one bucket, so the maximum over bucket
// maxima is the exact mode with the smallest-label tie-break; the result is
// independent of the (non-deterministic) order in which words are staged.
// In the converged supersteps every hub takes the k_hub_small path.
#include "lpa_device.h"

namespace lpa {

namespace {

using namespace dev;

constexpr int kSmallWords = 512;    // k_hub_small capacity (8 chunks x 64 lanes)
constexpr int kSmallSlots = 1024;   // its per-wave LDS table
constexpr int kChunkUnits = 8;      // units per k_hub_count / k_hub_scatter work item
constexpr int kPeelRounds = 8;
constexpr int kLaneUnits = kBlockMaxDeg / kSegArcs;  // k_hub_lanes / k_lpa_block rows: <= 8 units

__device__ __forceinline__ u32 comb_bucket(u32 label, int lg) {
  return lg == 0 ? 0u : (label * 0x85EBCA77u) >> (32 - lg);
}
__device__ __forceinline__ u32 comb_sub(u32 label, int lg) {
  return lg == 0 ? 0u : (label * 0xC2B2AE3Du) >> (32 - lg);
}
// buckets of a hub with T staged words (T > kCombDirect)
__device__ __forceinline__ int comb_lgK(int T) {
  const int lg = ceil_log2((u32)((T + kCombWords - 1) / kCombWords));
  return lg < kMaxBucketsLg ? lg : kMaxBucketsLg;
}

// Staged words of row h: unit j (j < nu = uoff[h+1] - uoff[h]) left ucnt[uoff[h] + j]
// words at stage[rp[h] + j * kSegArcs ...).
struct RowUnits {
  int64_t sbase;  // rp[h]
  int64_t u0;     // first unit
  int nu;         // units
};

__device__ __forceinline__ RowUnits row_units(const int64_t* __restrict__ rp,
                                              const int64_t* __restrict__ uoff, int64_t h) {
  RowUnits r;
  r.sbase = rp[h];
  r.u0 = uoff[h];
  r.nu = (int)(uoff[h + 1] - r.u0);
  return r;
}

// ---------------------------------------------------------------------------
// rows of <= kLaneUnits units (deg <= 4096): one LANE per row.  A converged
// row left one word per unit; the lane loads them and takes the mode of <= 8
// words in registers.  Any other row is classified here by its word count T
// (<= 8 x 512, never bucketed): T <= kSmallWords -> k_hub_small (list W), else
// the k_hub_mid tier queue_row would pick, with ONE queue atomic per wave and
// list: a row-at-a-time queue_row in k_hub_small serialised ~10^5 returning
// atomics on three counters in the label-dense supersteps (0.5 ms of waiting).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_append(bool p, int32_t* __restrict__ dst, int32_t* ctr,
                                            int32_t v, int lane) {
  const u64 m = __ballot(p);
  if (m == 0ull) return;  // uniform over the wave
  const int lead = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if (lane == lead) base = atomicAdd(ctr, __popcll(m));
  base = __builtin_amdgcn_readlane(base, lead);
  if (p) dst[base + __popcll(m & ((1ull << lane) - 1ull))] = v;
}

__global__ __launch_bounds__(256) void k_hub_lanes(int64_t h_begin, int64_t h_end,
                                                   const int64_t* __restrict__ rp,
                                                   const int64_t* __restrict__ uoff,
                                                   const int32_t* __restrict__ ucnt,
                                                   const u64* __restrict__ stage,
                                                   int32_t* __restrict__ Ln,
                                                   int32_t* __restrict__ lists, int64_t n_hub,
                                                   int32_t* __restrict__ wcount,
                                                   int32_t* __restrict__ lcnt,
                                                   const int32_t* __restrict__ flist,
                                                   const int32_t* __restrict__ fcnt0,
                                                   const int32_t* __restrict__ fr_all) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // frontier: only the listed dirty hub rows (bin 0 of k_frontier_lists; rows below
  // h_begin are k_hub_small's), else every row of [h_begin, h_end)
  const int all = *fr_all;
  const int64_t n_items = all ? h_end - h_begin : (int64_t)*fcnt0;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n_items; i0 += stride) {
    const int64_t i = i0 + threadIdx.x;
    int64_t h = 0;
    bool live = false;
    if (i < n_items) {
      h = all ? h_begin + i : (int64_t)flist[i];
      live = h >= h_begin;
    }
    bool one = false;
    int T = 0;
    if (live) {
      const int64_t b = rp[h];
      const int nu = (int)((rp[h + 1] - b + kSegArcs - 1) / kSegArcs);
      const int32_t* uc = ucnt + uoff[h];
      int c[kLaneUnits];
#pragma unroll
      for (int k = 0; k < kLaneUnits; ++k) c[k] = k < nu ? uc[k] : 1;
#pragma unroll
      for (int k = 0; k < kLaneUnits; ++k) T += k < nu ? c[k] : 0;
      one = true;
#pragma unroll
      for (int k = 0; k < kLaneUnits; ++k) one = one && c[k] == 1;
      if (one) {
        const u64* wd = stage + b;
        u64 wv[kLaneUnits];
#pragma unroll
        for (int k = 0; k < kLaneUnits; ++k) wv[k] = k < nu ? wd[(int64_t)k * kSegArcs] : 0ull;
        u64 best = 0ull;
#pragma unroll
        for (int k = 0; k < kLaneUnits; ++k) {
          u32 cs = 0u;
#pragma unroll
          for (int q = 0; q < kLaneUnits; ++q)
            if ((u32)wv[q] == (u32)wv[k]) cs += (u32)(wv[q] >> 32);
          if (wv[k] != 0ull) best = umax64(best, ((u64)cs << 32) | (u64)(u32)wv[k]);
        }
        Ln[h] = (int32_t)(~(u32)best);
      }
    }
    const bool q = live && !one;
    if (q && T > kSmallWords) wcount[h] = T;  // as queue_row
    // lists: [0] mid T <= 1024, [2n] wave path (list W), [3n] mid <= 2048, [4n] mid <= 6144
    wave_append(q && T <= kSmallWords, lists + 2 * n_hub, &lcnt[4], (int32_t)h, lane);
    wave_append(q && T > kSmallWords && T <= 1024, lists, &lcnt[0], (int32_t)h, lane);
    wave_append(q && T > 1024 && T <= 2048, lists + 3 * n_hub, &lcnt[5], (int32_t)h, lane);
    wave_append(q && T > 2048, lists + 4 * n_hub, &lcnt[6], (int32_t)h, lane);
  }
}
static_assert(kLaneUnits * kSegArcs <= kCombDirect, "lane-path rows are never bucketed");

// queue row h (T staged words) for k_hub_mid (three table sizes) or the bucket
// path.  lists: [0] mid T <= 1024, [n] bucketed, [2n] wave path, [3n] mid <= 2048,
// [4n] mid <= 6144; lcnt: 0 mid1, 1 bucketed, 2 bucket items, 3 chunk items,
// 4 wave path, 5 mid2, 6 mid3
__device__ __forceinline__ void queue_row(int64_t h, int T, int nu, int lane,
                                          int32_t* __restrict__ wcount, int32_t* __restrict__ lists,
                                          int64_t n_hub, int32_t* __restrict__ lcnt,
                                          u64* __restrict__ itemsCB, u64* __restrict__ itemsCC) {
  if (lane == 0) {
    wcount[h] = T;
    if (T <= 1024) {
      lists[atomicAdd(&lcnt[0], 1)] = (int32_t)h;
    } else if (T <= 2048) {
      lists[3 * n_hub + atomicAdd(&lcnt[5], 1)] = (int32_t)h;
    } else if (T <= kCombDirect) {
      lists[4 * n_hub + atomicAdd(&lcnt[6], 1)] = (int32_t)h;
    } else {
      lists[n_hub + atomicAdd(&lcnt[1], 1)] = (int32_t)h;
    }
  }
  if (T > kCombDirect) {
    const int K = 1 << comb_lgK(T);
    const int nch = (nu + kChunkUnits - 1) / kChunkUnits;
    int cb = 0, cc = 0;
    if (lane == 0) {
      cb = atomicAdd(&lcnt[2], K);
      cc = atomicAdd(&lcnt[3], nch);
    }
    cb = __builtin_amdgcn_readfirstlane(cb);
    cc = __builtin_amdgcn_readfirstlane(cc);
    for (int k = lane; k < K; k += 64) itemsCB[cb + k] = ((u64)h << 32) | (u64)k;
    for (int c = lane; c < nch; c += 64) itemsCC[cc + c] = ((u64)h << 32) | (u64)c;
  }
}

// Superstep 2's giant-label decision for the hub rows [0, h_end) (after
// k_lpa_units_giant): row h's G votes S_g = sum of its units' ugc, and any other
// label's row count is at most S_m = sum of its units' umx (each unit's fullest
// bucket).  On the 2-bit giant codes (gsel[5], k_lpa_units_code2) umx packs a unit's
// three bucket counts (10 bits each) and S_m = the fullest of the three row sums -- the
// row-level bucket test, not a sum of unit maxima.  S_g > S_m: G is the strict mode and
// is written.  Otherwise the row is
// tallied exactly: a unit-tallied row (h < hb2) gets wcount[h] = 0 and its units in
// ulist2 (count ndec[0]), a block-tier row (h >= hb2, <= 16 units) goes to
// glist (count ndec[2]); settled unit-tallied rows get wcount[h] = -1 (the combine's
// classify / enqueue skip them).  ndec[3] = 1 when G is not worth trying: nothing is
// decided and the exact kernels take their whole ranges (ndec[3] is their "fr_all").
// Unit-tallied rows: a wave per row; block-tier rows: a lane per row, one list atomic
// per wave.
__global__ __launch_bounds__(256) void k_hub_decide(int64_t h_end, const int64_t* __restrict__ uoff,
                                                    const uint32_t* __restrict__ ugc,
                                                    const uint32_t* __restrict__ umx,
                                                    const int32_t* __restrict__ gsel,
                                                    int32_t* __restrict__ Ln, int32_t* __restrict__ wcount,
                                                    int32_t* __restrict__ ulist2, int32_t* __restrict__ ndec,
                                                    int64_t hb2, int32_t* __restrict__ glist) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * 4;
  const int32_t G = gsel[0];
  const bool on = gsel[1] != 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) ndec[3] = on ? 0 : 1;
  if (!on) return;  // uniform: k_lpa_units_giant counted nothing
  const bool code = gsel[5] != 0;   // uniform
  const int64_t ha = hb2 < h_end ? hb2 : h_end;
  for (int64_t h = (int64_t)blockIdx.x * 4 + w; h < ha; h += stride) {
    const int64_t u0 = uoff[h];
    const int nu = (int)(uoff[h + 1] - u0);
    u64 sg = 0, sm = 0;
    if (code) {
      u64 s1 = 0, s2 = 0, s3 = 0;
      for (int j = lane; j < nu; j += 64) {
        const u32 m = umx[u0 + j];
        sg += ugc[u0 + j];
        s1 += m & 1023u;
        s2 += (m >> 10) & 1023u;
        s3 += m >> 20;
      }
      for (int off = 32; off > 0; off >>= 1) {
        sg += __shfl_xor(sg, off, 64);
        s1 += __shfl_xor(s1, off, 64);
        s2 += __shfl_xor(s2, off, 64);
        s3 += __shfl_xor(s3, off, 64);
      }
      sm = s1 > s2 ? s1 : s2;
      sm = sm > s3 ? sm : s3;
    } else {
      for (int j = lane; j < nu; j += 64) {
        sg += ugc[u0 + j];
        sm += umx[u0 + j];
      }
      for (int off = 32; off > 0; off >>= 1) {
        sg += __shfl_xor(sg, off, 64);
        sm += __shfl_xor(sm, off, 64);
      }
    }
    if (sg > sm) {
      if (lane == 0) {
        Ln[h] = G;
        wcount[h] = -1;
      }
    } else {
      int base = 0;
      if (lane == 0) {
        wcount[h] = 0;
        base = atomicAdd(&ndec[0], nu);
      }
      base = __shfl(base, 0, 64);
      for (int j = lane; j < nu; j += 64) ulist2[base + j] = (int32_t)(u0 + j);
    }
  }
  // block-tier rows: a lane per row
  for (int64_t h0 = ha + ((int64_t)blockIdx.x * 4 + w) * 64; h0 < h_end; h0 += stride * 64) {
    const int64_t h = h0 + lane;
    bool open = false;
    if (h < h_end) {
      const int64_t u0 = uoff[h];
      const int nu = (int)(uoff[h + 1] - u0);
      u32 sg = 0, sm = 0, s1 = 0, s2 = 0, s3 = 0;
      for (int j = 0; j < nu; ++j) {
        const u32 m = umx[u0 + j];
        sg += ugc[u0 + j];
        sm += m;
        s1 += m & 1023u;
        s2 += (m >> 10) & 1023u;
        s3 += m >> 20;
      }
      if (code) sm = max(s1, max(s2, s3));
      if (sg > sm) Ln[h] = G;
      else open = true;
    }
    wave_append(open, glist, &ndec[2], (int32_t)h, lane);
  }
}

// Label-dense supersteps: classify the rows of > kLaneUnits units right after the
// unit tallies, so the bucket path (count / scan / scatter / bucket, complete once
// these rows are queued: rows of <= kLaneUnits units never exceed kCombDirect words)
// can start on its own stream while k_hub_small works through the rest.  One wave
// per row sums its word count T into wcount[h] (and emits a bucketed row's work
// items); k_hub_enqueue then appends the rows to list S (<= kSmallWords units and
// words, for k_hub_small) or the tier queue_row would pick.
__global__ __launch_bounds__(256) void k_hub_classify(int64_t h_lane, int64_t n_hub,
                                                      const int64_t* __restrict__ rp,
                                                      const int64_t* __restrict__ uoff,
                                                      const int32_t* __restrict__ ucnt,
                                                      int32_t* __restrict__ wcount,
                                                      int32_t* __restrict__ lists,
                                                      int32_t* __restrict__ lcnt,
                                                      u64* __restrict__ itemsCB,
                                                      u64* __restrict__ itemsCC, int giant) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t h = (int64_t)blockIdx.x * 4 + w; h < h_lane; h += stride) {
    if (giant && wcount[h] < 0) continue;  // settled by k_hub_decide (uniform)
    const RowUnits ru = row_units(rp, uoff, h);
    const int nu = ru.nu;
    const int32_t* uc = ucnt + ru.u0;
    int T = 0;
    for (int j = lane; j < nu; j += 64) T += uc[j];
    T = (int)wave_sum_u32((u32)T);
    if (lane == 0) wcount[h] = T;
    if (T > kCombDirect) {
      // bucketed row (few per superstep): its count / bucket work items, as queue_row
      const int K = 1 << comb_lgK(T);
      const int nch = (nu + kChunkUnits - 1) / kChunkUnits;
      int cb = 0, cc = 0;
      if (lane == 0) {
        cb = atomicAdd(&lcnt[2], K);
        cc = atomicAdd(&lcnt[3], nch);
      }
      cb = __builtin_amdgcn_readfirstlane(cb);
      cc = __builtin_amdgcn_readfirstlane(cc);
      for (int k = lane; k < K; k += 64) itemsCB[cb + k] = ((u64)h << 32) | (u64)k;
      for (int c = lane; c < nch; c += 64) itemsCC[cc + c] = ((u64)h << 32) | (u64)c;
    }
  }
}

// Second half of the classification: one LANE per row of [0, h_lane), its word
// count from k_hub_classify, every list appended with one atomic per wave (a
// returning atomic per row on a shared counter serialises: 0.2 ms for ~10^4 rows
// in the label-dense supersteps).  Bucketed rows (T > kCombDirect, few) got their
// work items from k_hub_classify.
__global__ __launch_bounds__(256) void k_hub_enqueue(int64_t h_lane, int64_t n_hub,
                                                     const int64_t* __restrict__ uoff,
                                                     int32_t* __restrict__ wcount,
                                                     int32_t* __restrict__ lists,
                                                     int32_t* __restrict__ lcnt) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t h0 = (int64_t)blockIdx.x * blockDim.x; h0 < h_lane; h0 += stride) {
    const int64_t h = h0 + threadIdx.x;
    bool live = h < h_lane;
    int T = 0, nu = 0;
    if (live) {
      T = wcount[h];
      nu = (int)(uoff[h + 1] - uoff[h]);
      if (T < 0) {  // settled by k_hub_decide: not queued
        wcount[h] = 0;
        live = false;
      }
    }
    const bool sm = live && nu <= kSmallWords && T <= kSmallWords;
    const bool q = live && !sm;
    if (sm) wcount[h] = 0;  // only queued rows keep T (queue_row's contract)
    // lists: [0] mid T <= 1024, [n] bucketed, [3n] mid <= 2048, [4n] mid <= 6144, [5n] S
    wave_append(sm, lists + 5 * n_hub, &lcnt[7], (int32_t)h, lane);
    wave_append(q && T <= 1024, lists, &lcnt[0], (int32_t)h, lane);
    wave_append(q && T > 1024 && T <= 2048, lists + 3 * n_hub, &lcnt[5], (int32_t)h, lane);
    wave_append(q && T > 2048 && T <= kCombDirect, lists + 4 * n_hub, &lcnt[6], (int32_t)h, lane);
    wave_append(q && T > kCombDirect, lists + n_hub, &lcnt[1], (int32_t)h, lane);
  }
}

// weighted ballot peel over NC word chunks: rounds retire the first unretired
// label's words; lane p ends with round p's tally word in *pw, returns rounds.
template <int NC>
__device__ __forceinline__ int weighted_peel(const u64 (&wv)[NC], u64 (&act)[NC], int& nact,
                                             u64& best, u64& pw, int lane) {
  int np = 0;
  for (int p = 0; p < kPeelRounds && nact > 0; ++p) {
    u32 x = 0u;
    bool found = false;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (!found && act[c] != 0ull) {
        x = ~(u32)__builtin_amdgcn_readlane((int)(u32)wv[c], __ffsll((unsigned long long)act[c]) - 1);
        found = true;
      }
    }
    u32 cs = 0u;
    int k = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const u64 mm = __ballot(((act[c] >> lane) & 1ull) && ~(u32)wv[c] == x);
      act[c] &= ~mm;
      k += __popcll(mm);
      if ((mm >> lane) & 1ull) cs += (u32)(wv[c] >> 32);
    }
    nact -= k;
    const u64 tw = tally(wave_sum_u32(cs), x);
    best = umax64(best, tw);
    if (lane == p) pw = tw;
    np = p + 1;
    if (k < 2) break;
  }
  return np;
}

// ---------------------------------------------------------------------------
// one wave per row (grid-stride over rows [0, h_lane) and list W):
//   <= 512 units and <= 512 words      words in registers, weighted peel,
//                                      residual in the wave's LDS table
//   > 512 units, one word each         512-unit batches merged in the LDS table
//                                      (giant converged rows)
//   otherwise                          queued with T in wcount[h]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hub_small(int64_t nd, int64_t n_hub,
                                                   const int64_t* __restrict__ rp,
                                                   const int64_t* __restrict__ uoff,
                                                   const int32_t* __restrict__ ucnt,
                                                   const u64* __restrict__ stage,
                                                   int32_t* __restrict__ wcount,
                                                   int32_t* __restrict__ Ln,
                                                   int32_t* __restrict__ lists,
                                                   int32_t* __restrict__ lcnt,
                                                   u64* __restrict__ itemsCB,
                                                   u64* __restrict__ itemsCC,
                                                   const int32_t* __restrict__ flist,
                                                   const int32_t* __restrict__ fcnt0,
                                                   const int32_t* __restrict__ fr_all) {
  __shared__ u64 tab_all[4][kSmallSlots];
  // unit prefixes (< T <= kSmallWords), then the slot list (< kSmallSlots): both fit
  // 16 bits, so the block takes 36 KB of LDS and four blocks fit a CU
  __shared__ uint16_t aux_all[4][kSmallWords];
  __shared__ int lc_all[4];
  constexpr int NC = kSmallWords / 64;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u64* tab = tab_all[w];
  uint16_t* pre = aux_all[w];
  uint16_t* lst = aux_all[w];
  // rows: [0, nd) directly, then list S (pre-classified by k_hub_classify), then
  // list W (from k_hub_lanes)
  // direct rows [0, nd): with the frontier, the listed dirty hub rows below nd
  const int all = *fr_all;
  const int64_t nd_items = (all || nd == 0) ? nd : (int64_t)*fcnt0;
  const int64_t nS = lcnt[7];
  const int64_t nq = nd_items + nS + lcnt[4];
  const int64_t stride = (int64_t)gridDim.x * 4;
  if ((int64_t)blockIdx.x * 4 + w >= nq) return;  // no block-level barriers in this kernel
  for (int i = lane; i < kSmallSlots; i += 64) tab[i] = 0ull;  // only waves with rows clear
  for (int64_t q = (int64_t)blockIdx.x * 4 + w; q < nq; q += stride) {
    const int64_t h = q < nd_items ? (all ? q : (int64_t)flist[q])
                                   : (q < nd_items + nS ? (int64_t)lists[5 * n_hub + (q - nd_items)]
                                                        : (int64_t)lists[2 * n_hub + (q - nd_items - nS)]);
    if (h >= nd && q < nd_items) continue;  // a lane-path row (k_hub_lanes); uniform
    if (q < nd_items && wcount[h] < 0) {     // settled by k_hub_decide (serialized schedule)
      if (lane == 0) wcount[h] = 0;
      continue;
    }
    const RowUnits ru = row_units(rp, uoff, h);
    const int nu = ru.nu;
    const int32_t* uc = ucnt + ru.u0;
    const u64* wd = stage + ru.sbase;
    int cnt[NC];
    int T = 0;
    if (nu <= kSmallWords) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int j = c * 64 + lane;
        cnt[c] = (c * 64 < nu && j < nu) ? uc[j] : 0;
        T += cnt[c];
      }
    } else {
      for (int j = lane; j < nu; j += 64) T += uc[j];
    }
    T = (int)wave_sum_u32((u32)T);
    if (nu > kSmallWords && T == nu) {
      // giant converged row: 512-unit batches, peel groups + residual merged in LDS
      if (lane == 0) lc_all[w] = 0;
      bool ovf = false;
      u64 best = 0ull;
      for (int b0 = 0; b0 < nu; b0 += kSmallWords) {
        u64 wv[NC], act[NC];
        int nact = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int j = b0 + c * 64 + lane;
          wv[c] = j < nu ? wd[(int64_t)j * kSegArcs] : 0ull;
          act[c] = __ballot(wv[c] != 0ull);
          nact += __popcll(act[c]);
        }
        u64 pw = 0ull, pbest = 0ull;
        const int np = weighted_peel<NC>(wv, act, nact, pbest, pw, lane);
        if (lc_all[w] + np + nact > kSmallWords) {
          ovf = true;
          break;
        }
        int slot = -1;
        if (lane < np) slot = lds_insert(tab, 32 - 10, kSmallSlots - 1u, ~(u32)pw, (u32)(pw >> 32));
        list_append(lst, &lc_all[w], slot, lane);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          slot = -1;
          if ((act[c] >> lane) & 1ull)
            slot = lds_insert(tab, 32 - 10, kSmallSlots - 1u, ~(u32)wv[c], (u32)(wv[c] >> 32));
          list_append(lst, &lc_all[w], slot, lane);
        }
      }
      const int n = lc_all[w];
      for (int i = lane; i < n; i += 64) {
        const int sl = lst[i];
        best = umax64(best, tab[sl]);
        tab[sl] = 0ull;
      }
      best = wave_max_u64(best);
      if (ovf) {
        queue_row(h, T, nu, lane, wcount, lists, n_hub, lcnt, itemsCB, itemsCC);
      } else if (lane == 0) {
        Ln[h] = (int32_t)(~(u32)best);
      }
      continue;
    }
    if (nu > kSmallWords || T > kSmallWords) {
      queue_row(h, T, nu, lane, wcount, lists, n_hub, lcnt, itemsCB, itemsCC);
      continue;
    }
    u64 wv[NC];
    if (T == nu) {
      // converged rows: one word per unit, at the unit's first staging slot
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int j = c * 64 + lane;
        wv[c] = (c * 64 < nu && j < nu) ? wd[(int64_t)j * kSegArcs] : 0ull;
      }
    } else {
      // unit prefixes into LDS, then word i = unit j (largest pre[j] <= i)
      int carry = 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (c * 64 < nu) {
          int incl = cnt[c];
#pragma unroll
          for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(incl, off, 64);
            if (lane >= off) incl += o;
          }
          if (c * 64 + lane < nu) pre[c * 64 + lane] = (uint16_t)(carry + incl - cnt[c]);
          carry += __shfl(incl, 63, 64);
        }
      }
      const int steps = ceil_log2((u32)nu);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = c * 64 + lane;
        wv[c] = 0ull;
        if (c * 64 < T && i < T) {
          int lo = 0;
          for (int st = steps - 1; st >= 0; --st) {
            const int mid = lo + (1 << st);
            if (mid < nu && pre[mid] <= i) lo = mid;
          }
          wv[c] = wd[(int64_t)lo * kSegArcs + (i - pre[lo])];
        }
      }
    }
    u32 lmask = 0u;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (wv[c] != 0ull) lmask |= 1u << c;
    u64 best = 0ull, pw = 0ull;
    peel_words<NC>(wv, lmask, best, pw, lane, kPeelRounds);
    if (__ballot(lmask != 0u)) {
      int lg = ceil_log2(2u * (u32)T);
      lg = lg < 6 ? 6 : lg;
      const u32 mask = (1u << lg) - 1u;
      int slot[NC];
      insert_words<NC>(tab, 32 - lg, mask, wv, lmask, slot, nullptr);
      // the wave owns its table and list: claimed slots appended by ballot prefix
      const u64 lt = (1ull << lane) - 1ull;
      int n = 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const u64 cm = __ballot(slot[c] >= 0);
        if (slot[c] >= 0) lst[n + __popcll(cm & lt)] = (uint16_t)slot[c];
        n += __popcll(cm);
      }
      for (int i = lane; i < n; i += 64) {
        const int sl = lst[i];
        best = umax64(best, tab[sl]);
        tab[sl] = 0ull;
      }
    }
    best = wave_max_u64(best);
    if (lane == 0) Ln[h] = (int32_t)(~(u32)best);
  }
}

// Tally the words of units [j0, j1) of a row whose labels pass `keep` into the
// block's LDS table (kCombSlots slots) with kW waves.  Returns the block-uniform
// maximum.
template <int kLg, int kW, typename Keep>
__device__ u64 block_tally_units(const u64* __restrict__ wd, const int32_t* __restrict__ uc, int j0,
                                 int j1, Keep keep, u64* tab, uint16_t* lst, int* lcount, u64* redw,
                                 int32_t* err) {
  constexpr int NC = kSegArcs / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) *lcount = 0;
  __syncthreads();
  // wave w takes units j0 + w + kW i, 64 at a time: lane-per-unit for each unit's
  // first kFirst words (converged units hold one), then unit-major for longer units
  constexpr int kFirst = 4;
  for (int jb = j0 + w; jb < j1; jb += 64 * kW) {
    const int j = jb + kW * lane;
    const int nj = j < j1 ? uc[j] : 0;
    const u64* src = wd + (int64_t)j * kSegArcs;
    u64 fv[kFirst];
#pragma unroll
    for (int k = 0; k < kFirst; ++k) fv[k] = k < nj ? src[k] : 0ull;
    {
      u32 fa = 0u;
      int sl[kFirst];
#pragma unroll
      for (int k = 0; k < kFirst; ++k)
        if (fv[k] != 0ull && keep(~(u32)fv[k])) fa |= 1u << k;
      insert_words<kFirst>(tab, 32 - kLg, (1u << kLg) - 1u, fv, fa, sl, err);
      list_append_n<kFirst>(lst, lcount, sl, lane);
    }
    // longer units one at a time, the next one's words loading meanwhile
    u64 big = __ballot(nj > kFirst);
    u64 wv[NC];
    int n = 0;
    auto load_big = [&](u64 set, u64(&dst)[NC], int& cnt) {
      cnt = 0;
#pragma unroll
      for (int c = 0; c < NC; ++c) dst[c] = 0ull;
      if (set == 0ull) return;
      const int bl = __ffsll((unsigned long long)set) - 1;
      cnt = __builtin_amdgcn_readlane(nj, bl);
      const u64* us = wd + (int64_t)(jb + kW * bl) * kSegArcs;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = kFirst + c * 64 + lane;
        dst[c] = (kFirst + c * 64 < cnt && i < cnt) ? us[i] : 0ull;
      }
    };
    load_big(big, wv, n);
    while (big) {
      big &= big - 1ull;
      u64 wn[NC];
      int nn = 0;
      load_big(big, wn, nn);
      {
        u32 wa = 0u;
        int sl[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c)
          if (wv[c] != 0ull && keep(~(u32)wv[c])) wa |= 1u << c;
        insert_words<NC>(tab, 32 - kLg, (1u << kLg) - 1u, wv, wa, sl, err);
        list_append_n<NC>(lst, lcount, sl, lane);
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) wv[c] = wn[c];
      n = nn;
    }
  }
  __syncthreads();
  const int cnt = *lcount;
  u64 best = 0ull;
  for (int i = threadIdx.x; i < cnt; i += 64 * kW) {
    const int sl = lst[i];
    best = umax64(best, tab[sl]);
    tab[sl] = 0ull;
  }
  best = wave_max_u64(best);
  if (lane == 0) redw[w] = best;
  __syncthreads();
  best = redw[0];
#pragma unroll
  for (int i = 1; i < kW; ++i) best = umax64(best, redw[i]);
  __syncthreads();
  return best;
}

// Same over a compact word run wd[0, n) (a bucket after the scatter).
// No slot list: the occupied slots are found by a scan of the whole table at the
// end (a bucket pass loads it to ~1/2, so the scan reads about what a list walk
// would), which keeps the block's LDS at 64 KB + 32 B: two blocks per CU.
template <int kW, typename Keep>
__device__ u64 block_tally_run(const u64* __restrict__ wd, int n, Keep keep, u64* tab, u64* redw,
                               int32_t* err) {
  constexpr int kLg = 13;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int kT = 64 * kW;
  // words per thread per round: 24 at 4 waves (6144), 8 at 8 waves (4096: a bucket
  // pass's expected load)
  constexpr int R = kW == 4 ? kCombDirect / 256 : 8;
  for (int b0 = 0; b0 < n; b0 += R * kT) {
    u64 wv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = b0 + r * kT + threadIdx.x;
      wv[r] = i < n ? wd[i] : 0ull;
    }
    // batched inserts, 8 words per lane in flight (bounded probing: a bucket's
    // table load is not guaranteed by construction)
    static_assert(R % 8 == 0, "insert groups of 8");
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += 8) {
      if (b0 + r0 * kT >= n) break;  // uniform over the block
      u64 grp[8];
      u32 m = 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        grp[k] = wv[r0 + k];
        if (grp[k] != 0ull && keep(~(u32)grp[k])) m |= 1u << k;
      }
      int sl[8];
      insert_words<8, true>(tab, 32 - kLg, (1u << kLg) - 1u, grp, m, sl, err);
    }
  }
  __syncthreads();
  u64 best = 0ull;
  for (int i = threadIdx.x; i < kCombSlots; i += kT) {
    const u64 t = tab[i];
    if (t) {
      best = umax64(best, t);
      tab[i] = 0ull;
    }
  }
  best = wave_max_u64(best);
  if (lane == 0) redw[w] = best;
  __syncthreads();
  best = redw[0];
#pragma unroll
  for (int i = 1; i < kW; ++i) best = umax64(best, redw[i]);
  __syncthreads();
  return best;
}

// ---------------------------------------------------------------------------
// 512 < T <= kCombDirect: one block per queued row (grid-stride over the queue).
// ---------------------------------------------------------------------------
// kW waves per block: the 8K-slot tier runs two 76 KB blocks per CU, so it takes
// 8 waves each (16 resident waves per CU instead of 8 to cover LDS atomic latency)
template <int kLg, int kW>
__global__ __launch_bounds__(64 * kW) void k_hub_mid(const int32_t* __restrict__ list,
                                                 const int32_t* __restrict__ lcnt, int which,
                                                 const int64_t* __restrict__ rp,
                                                 const int64_t* __restrict__ uoff,
                                                 const int32_t* __restrict__ ucnt,
                                                 const u64* __restrict__ stage,
                                                 int32_t* __restrict__ wcount,
                                                 int32_t* __restrict__ Ln, int32_t* __restrict__ err) {
  constexpr int kSlots = 1 << kLg;
  // a row of this tier has at most T words, so at most T distinct labels (tiers:
  // T <= 1024 / 2048 / kCombDirect, queue_row): the list holds T entries, which
  // keeps the 8K-slot tier's block at 76 KB (two per CU)
  constexpr int kList = kLg == 11 ? 1024 : kLg == 12 ? 2048 : kCombDirect;
  static_assert(kList <= kSlots, "list bounded by the table");
  __shared__ u64 tab[kSlots];
  __shared__ uint16_t lst[kList];
  __shared__ int lcount;
  __shared__ u64 redw[kW];
  const int nB = lcnt[which];
  if ((int)blockIdx.x >= nB) return;
  for (int i = threadIdx.x; i < kSlots; i += 64 * kW) tab[i] = 0ull;
  for (int q = blockIdx.x; q < nB; q += gridDim.x) {
    const int64_t h = list[q];
    const RowUnits ru = row_units(rp, uoff, h);
    const u64 best = block_tally_units<kLg, kW>(stage + ru.sbase, ucnt + ru.u0, 0, ru.nu,
                                            [](u32) { return true; }, tab, lst, &lcount, redw, err);
    if (threadIdx.x == 0) {
      Ln[h] = (int32_t)(~(u32)best);
      wcount[h] = 0;
    }
  }
}

// All three mid tiers in one launch, largest rows first (queue 6, then 5, then 0),
// each row with its tier's table size inside the 8K-slot block table.
template <int kW>
__global__ __launch_bounds__(64 * kW) void k_hub_mid_all(const int32_t* __restrict__ lists, int64_t n_hub,
                                                        const int32_t* __restrict__ lcnt,
                                                        const int64_t* __restrict__ rp,
                                                        const int64_t* __restrict__ uoff,
                                                        const int32_t* __restrict__ ucnt,
                                                        const u64* __restrict__ stage,
                                                        int32_t* __restrict__ wcount,
                                                        int32_t* __restrict__ Ln, int32_t* __restrict__ err) {
  constexpr int kSlots = 1 << 13;
  __shared__ u64 tab[kSlots];
  __shared__ uint16_t lst[kCombDirect];
  __shared__ int lcount;
  __shared__ u64 redw[kW];
  const int n3 = lcnt[6], n2 = lcnt[5], n1 = lcnt[0];
  const int nB = n3 + n2 + n1;
  if ((int)blockIdx.x >= nB) return;
  for (int i = threadIdx.x; i < kSlots; i += 64 * kW) tab[i] = 0ull;
  for (int q = blockIdx.x; q < nB; q += gridDim.x) {
    int64_t h;
    u64 best;
    if (q < n3) {
      h = lists[4 * n_hub + q];
      const RowUnits ru = row_units(rp, uoff, h);
      best = block_tally_units<13, kW>(stage + ru.sbase, ucnt + ru.u0, 0, ru.nu,
                                       [](u32) { return true; }, tab, lst, &lcount, redw, err);
    } else if (q < n3 + n2) {
      h = lists[3 * n_hub + (q - n3)];
      const RowUnits ru = row_units(rp, uoff, h);
      best = block_tally_units<12, kW>(stage + ru.sbase, ucnt + ru.u0, 0, ru.nu,
                                       [](u32) { return true; }, tab, lst, &lcount, redw, err);
    } else {
      h = lists[q - n3 - n2];
      const RowUnits ru = row_units(rp, uoff, h);
      best = block_tally_units<11, kW>(stage + ru.sbase, ucnt + ru.u0, 0, ru.nu,
                                       [](u32) { return true; }, tab, lst, &lcount, redw, err);
    }
    if (threadIdx.x == 0) {
      Ln[h] = (int32_t)(~(u32)best);
      wcount[h] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// T > kCombDirect: bucket partition of the staged words, kChunkUnits units per
// count / scatter work item.
// ---------------------------------------------------------------------------
// Last-block hand-off (the converged supersteps fuse count + scan and bucket + final,
// two dependent launches fewer).  What is handed off was built only by device-scope
// atomics, which execute at the memory side, past the per-XCD L2s: so every wave
// waits for its atomics to complete (vmcnt), the block takes a ticket, and the block
// that draws the last one acquires at agent scope, reads the totals with agent-scope
// loads, does the follow-up pass and resets the tickets.
//   consumer (memory-model form): the winning ticket RMW is the one relaxed poll, then
//     ONE agent-scope acquire in the winning lane (gfx950: `s_waitcnt vmcnt(0)
//     lgkmcnt(0); buffer_inv sc1`, checked in the generated ISA of k_hub_count and
//     k_hub_bucket), an `s_waitcnt` that holds the lane until the invalidate has
//     completed, and the workgroup barrier before any wave of the block loads;
//   producer: relaxed agent-scope atomics, each wave's `s_waitcnt` for them, the block
//     barrier, then the relaxed ticket add.  A release on the ticket would lower to
//     `buffer_wbl2 sc1` (write back the XCD L2's dirty lines), and the handed-off data
//     leaves no dirty line there -- it is written only by device atomics, which execute
//     at the memory side -- so the write-back has nothing to do for it; 2048 blocks
//     issuing it cost ~90 us per launch.
//     Round 6 re-checked both forms.  ISA (hipcc -O3 -S, gfx950): an
//     agent-scope release -- a `__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent")` before
//     the ticket, or the ticket RMW itself as release / acq_rel, with or without the
//     "global" address-space qualifier -- lowers to `buffer_wbl2 sc1; s_waitcnt vmcnt(0)`
//     ahead of the atomic in every form; no release form omits the L2 write-back.  The
//     relaxed form keeps each wave's `s_waitcnt vmcnt(0)` (every wave's own atomics
//     acknowledged: for device-scope atomics that is their completion at the memory side)
//     and the workgroup barrier before thread 0's ticket.  Measured, same box, bench
//     (profiles/r06/b_release_ab/, LPA_HUB_RELEASE=1 build, tickets acq_rel): C3 666.0 ->
//     634.9 GTEPS (converged supersteps +15-28 us each: the write-backs flush the label
//     stores of the concurrent bin kernels), C5 263.4 -> 262.3.  The relaxed form stays.
// Tickets are two-level (kTicketGroups counters, one 64-B line each, then one for the
// groups): returning atomics on ONE address serialise at ~88 M/s, 2048 of them ~23 us.
// The producer side leans on gfx950 behaviour (device atomics on hipMalloc memory
// complete at the memory side once vmcnt drains), so the library is built for gfx950
// only:
#ifndef LPA_HUB_RELEASE
#define LPA_HUB_RELEASE 0
#endif
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "lpa_hub.hip: the fused last-block hand-off is validated on gfx950 only"
#endif
constexpr int kTicketGroups = 16;
constexpr int kTicketStride = 16;  // uint32 per ticket line
constexpr int kTicketWords = (kTicketGroups + 1) * kTicketStride;
__device__ __forceinline__ bool last_block(uint32_t* tk) {
  __shared__ int last;
  __builtin_amdgcn_s_waitcnt(0);  // this wave's device atomics have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    const u32 G = gridDim.x < (u32)kTicketGroups ? gridDim.x : (u32)kTicketGroups;
    const u32 gi = blockIdx.x % G;
    const u32 in_group = (gridDim.x - gi + G - 1) / G;
    uint32_t* t1 = tk + gi * kTicketStride;
    uint32_t* t2 = tk + kTicketGroups * kTicketStride;
    last = 0;
    // LPA_HUB_RELEASE (A/B build): the tickets as agent-scope acq_rel RMWs -- the C++ /
    // HSA-model form (every block's ticket a release, each winner an acquire).  gfx950
    // lowers each release to `buffer_wbl2 sc1; s_waitcnt vmcnt(0)` before the atomic
    // (hipcc -S, round 6): a write-back of this XCD's dirty L2 lines, none of which hold
    // hand-off data
#if LPA_HUB_RELEASE
    constexpr int kTicketOrder = __ATOMIC_ACQ_REL;
#else
    constexpr int kTicketOrder = __ATOMIC_RELAXED;
#endif
    if (__hip_atomic_fetch_add(t1, 1u, kTicketOrder, __HIP_MEMORY_SCOPE_AGENT) == in_group - 1) {
      __hip_atomic_store(t1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(t2, 1u, kTicketOrder, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
        __hip_atomic_store(t2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the winner alone acquires at agent scope (one block per launch, not every
        // ticket): gfx950 emits `buffer_inv sc1` -- the CU's vector L1 and this XCD's
        // L2 drop their lines, so the follow-up pass's loads cannot hit a line cached
        // before the other blocks' atomics landed; the workgroup barrier below carries
        // it to the block's other waves
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __builtin_amdgcn_s_waitcnt(0);  // the invalidate completes before the barrier releases the block
        last = 1;
      }
    }
  }
  __syncthreads();
  return last != 0;
}
__device__ __forceinline__ int32_t ld_agent(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_agent(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// gcur[k] = exclusive prefix of ghist[k] for every queued row, by the waves of one
// block (k_hub_scan, or the last block of a fused k_hub_count)
template <bool kAgent>
__device__ __forceinline__ void scan_rows(int q0, int qstep, int nC, const int32_t* __restrict__ listC,
                                          const int32_t* __restrict__ wcount, const int64_t* __restrict__ hoff,
                                          const int32_t* __restrict__ ghist, int32_t* __restrict__ gcur) {
  const int lane = threadIdx.x & 63;
  for (int q = q0; q < nC; q += qstep) {
    const int64_t h = listC[q];
    const int K = 1 << comb_lgK(wcount[h]);
    const int32_t* gh = ghist + hoff[h];
    int32_t* gc = gcur + hoff[h];
    int carry = 0;
    for (int k0 = 0; k0 < K; k0 += 64) {
      const int v = k0 + lane < K ? (kAgent ? ld_agent(gh + k0 + lane) : gh[k0 + lane]) : 0;
      int incl = v;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off, 64);
        if (lane >= off) incl += o;
      }
      if (k0 + lane < K) gc[k0 + lane] = carry + incl - v;
      carry += __shfl(incl, 63, 64);
    }
  }
}

__global__ __launch_bounds__(256) void k_hub_count(const u64* __restrict__ itemsCC,
                                                   const int32_t* __restrict__ lcnt,
                                                   const int64_t* __restrict__ rp,
                                                   const int64_t* __restrict__ uoff,
                                                   const int32_t* __restrict__ ucnt,
                                                   const u64* __restrict__ stage,
                                                   const int32_t* __restrict__ wcount,
                                                   const int64_t* __restrict__ hoff,
                                                   int32_t* __restrict__ ghist,
                                                   uint32_t* __restrict__ ticket,  // fused scan: non-null
                                                   const int32_t* __restrict__ listC,
                                                   int32_t* __restrict__ gcur) {
  __shared__ int hist[kMaxBuckets];
  constexpr int NC = kSegArcs / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lcnt[3];
  for (int it = blockIdx.x; it < n; it += gridDim.x) {
    const u64 item = itemsCC[it];
    const int64_t h = (int64_t)(item >> 32);
    const int c = (int)(u32)item;
    const RowUnits ru = row_units(rp, uoff, h);
    const int lgK = comb_lgK(wcount[h]), K = 1 << lgK;
    for (int k = threadIdx.x; k < K; k += 256) hist[k] = 0;
    __syncthreads();
    const int j1 = min(ru.nu, (c + 1) * kChunkUnits);
    for (int j = c * kChunkUnits + w; j < j1; j += 4) {
      const int nw = ucnt[ru.u0 + j];
      const u64* src = stage + ru.sbase + (int64_t)j * kSegArcs;
      u64 wv[NC];
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int i = q * 64 + lane;
        wv[q] = (q * 64 < nw && i < nw) ? src[i] : 0ull;
      }
#pragma unroll
      for (int q = 0; q < NC; ++q)
        if (wv[q] != 0ull) atomicAdd(&hist[comb_bucket(~(u32)wv[q], lgK)], 1);
    }
    __syncthreads();
    int32_t* gh = ghist + hoff[h];
    for (int k = threadIdx.x; k < K; k += 256)
      if (hist[k]) atomicAdd(&gh[k], hist[k]);
    __syncthreads();
  }
  if (ticket && last_block(ticket)) scan_rows<true>(threadIdx.x >> 6, 4, lcnt[1], listC, wcount, hoff, ghist, gcur);
}

// one wave per queued row: gcur[k] = exclusive prefix of ghist[k]
__global__ __launch_bounds__(256) void k_hub_scan(const int32_t* __restrict__ listC,
                                                  const int32_t* __restrict__ lcnt,
                                                  const int32_t* __restrict__ wcount,
                                                  const int64_t* __restrict__ hoff,
                                                  const int32_t* __restrict__ ghist,
                                                  int32_t* __restrict__ gcur) {
  scan_rows<false>(blockIdx.x * 4 + (threadIdx.x >> 6), gridDim.x * 4, lcnt[1], listC, wcount, hoff, ghist, gcur);
}

__global__ __launch_bounds__(256) void k_hub_scatter(const u64* __restrict__ itemsCC,
                                                     const int32_t* __restrict__ lcnt,
                                                     const int64_t* __restrict__ rp,
                                                     const int64_t* __restrict__ uoff,
                                                     const int32_t* __restrict__ ucnt,
                                                     const u64* __restrict__ stage,
                                                     const int32_t* __restrict__ wcount,
                                                     const int64_t* __restrict__ hoff,
                                                     int32_t* __restrict__ gcur,
                                                     u64* __restrict__ scat) {
  __shared__ int lh[kMaxBuckets];
  __shared__ int lb[kMaxBuckets];
  constexpr int NC = kSegArcs / 64;
  constexpr int kPerWave = kChunkUnits / 4;  // units per wave per item
  static_assert(kChunkUnits % 4 == 0, "units per chunk item");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lcnt[3];
  for (int it = blockIdx.x; it < n; it += gridDim.x) {
    const u64 item = itemsCC[it];
    const int64_t h = (int64_t)(item >> 32);
    const int c = (int)(u32)item;
    const RowUnits ru = row_units(rp, uoff, h);
    const int lgK = comb_lgK(wcount[h]), K = 1 << lgK;
    for (int k = threadIdx.x; k < K; k += 256) lh[k] = 0;
    __syncthreads();
    const int j1 = min(ru.nu, (c + 1) * kChunkUnits);
    u64 wv[kPerWave][NC];
    int bk[kPerWave][NC], rk[kPerWave][NC];
#pragma unroll
    for (int a = 0; a < kPerWave; ++a) {
      const int j = c * kChunkUnits + w + 4 * a;
      const int nw = j < j1 ? ucnt[ru.u0 + j] : 0;
      const u64* src = stage + ru.sbase + (int64_t)j * kSegArcs;
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int i = q * 64 + lane;
        wv[a][q] = (q * 64 < nw && i < nw) ? src[i] : 0ull;
        bk[a][q] = -1;
        rk[a][q] = 0;
      }
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        if (wv[a][q] != 0ull) {
          bk[a][q] = (int)comb_bucket(~(u32)wv[a][q], lgK);
          rk[a][q] = atomicAdd(&lh[bk[a][q]], 1);
        }
      }
    }
    __syncthreads();
    int32_t* gc = gcur + hoff[h];
    for (int k = threadIdx.x; k < K; k += 256)
      if (lh[k]) lb[k] = atomicAdd(&gc[k], lh[k]);
    __syncthreads();
    u64* out = scat + ru.sbase;
#pragma unroll
    for (int a = 0; a < kPerWave; ++a)
#pragma unroll
      for (int q = 0; q < NC; ++q)
        if (bk[a][q] >= 0) out[lb[bk[a][q]] + rk[a][q]] = wv[a][q];
    __syncthreads();
  }
}

// write the bucketed rows' labels and reset their combine state, by waves
// [q0, q0 + qstep ...) (k_hub_final, or the last block of a fused k_hub_bucket)
template <bool kAgent>
__device__ __forceinline__ void final_rows(int q0, int qstep, int nC, const int32_t* __restrict__ listC,
                                           int32_t* __restrict__ wcount, const int64_t* __restrict__ hoff,
                                           int32_t* __restrict__ ghist, u64* __restrict__ hub_best,
                                           int32_t* __restrict__ Ln) {
  const int lane = threadIdx.x & 63;
  for (int q = q0; q < nC; q += qstep) {
    const int64_t h = listC[q];
    const int K = 1 << comb_lgK(wcount[h]);
    int32_t* gh = ghist + hoff[h];
    for (int k = lane; k < K; k += 64) gh[k] = 0;
    if (lane == 0) {
      Ln[h] = (int32_t)(~(u32)(kAgent ? ld_agent(hub_best + h) : hub_best[h]));
      hub_best[h] = 0ull;
      wcount[h] = 0;
    }
  }
}

// one block per (row, bucket): after the scatter, bucket k of row h is
// scat[rp[h] + gcur[k] - ghist[k], rp[h] + gcur[k])
// kW waves per block (64.03 KB blocks: two per CU; kW = 8 gives 16 resident waves)
template <int kW>
__global__ __launch_bounds__(64 * kW) void k_hub_bucket(const u64* __restrict__ itemsCB,
                                                    const int32_t* __restrict__ lcnt,
                                                    const int64_t* __restrict__ rp,
                                                    const u64* __restrict__ scat,
                                                    const int64_t* __restrict__ hoff,
                                                    const int32_t* ghist,  // also ghist_w (fused final)
                                                    const int32_t* __restrict__ gcur,
                                                    u64* __restrict__ hub_best,
                                                    int32_t* __restrict__ err,
                                                    // fused final (non-null ticket): the last block
                                                    uint32_t* __restrict__ ticket,
                                                    const int32_t* __restrict__ listC,
                                                    int32_t* __restrict__ wcount,
                                                    int32_t* ghist_w,
                                                    int32_t* __restrict__ Ln,
                                                    int32_t* __restrict__ lcnt_next) {
  __shared__ u64 tab[kCombSlots];
  __shared__ u64 redw[kW];
  __shared__ int32_t ovf;  // a pass whose distinct labels overflowed the table
  const int n = lcnt[2];
  if ((int)blockIdx.x >= n && !ticket) return;
  if ((int)blockIdx.x < n) {  // uniform (blocks without items only take their ticket)
    for (int i = threadIdx.x; i < kCombSlots; i += 64 * kW) tab[i] = 0ull;
    if (threadIdx.x == 0) ovf = 0;
    __syncthreads();
  }
  for (int it = blockIdx.x; it < n; it += gridDim.x) {
    const u64 item = itemsCB[it];
    const int64_t h = (int64_t)(item >> 32);
    const int k = (int)(u32)item;
    const int cnt = ghist[hoff[h] + k];
    if (cnt == 0) continue;  // uniform
    const u64* wd = scat + rp[h] + (gcur[hoff[h] + k] - cnt);
    // a bucket far above its expected load is tallied in sub-bucket passes
    const int lgJ = cnt > kCombDirect ? ceil_log2((u32)((cnt + 4095) / 4096)) : 0;
    u64 best = 0ull;
    for (u32 j = 0; j < (1u << lgJ); ++j) {
      // Spill guard (the hub spill path must not lose counts): the
      // hashes spread an ordinary bucket's labels well below the table size, but a
      // pass can still meet more distinct labels than the table holds (adversarial
      // or unlucky label sets).  Such a pass is dropped and redone on half its
      // label-value range, and the range grows back after a pass fits; every label's
      // votes always fall in exactly one pass, so each count stays whole.  Ranges of
      // <= kCombSlots / 2 label values always fit, so the sweep terminates.
      u64 lo = 0, width = 1ull << 32;
      while (lo < (1ull << 32)) {
        const u64 hi = lo + width < (1ull << 32) ? lo + width : (1ull << 32);
        const u64 pass = block_tally_run<kW>(
            wd, cnt, [=](u32 lab) { return comb_sub(lab, lgJ) == j && lab >= lo && lab < hi; }, tab, redw,
            &ovf);
        if (ovf) {  // block-uniform (read after block_tally_run's closing barrier)
          __syncthreads();
          if (threadIdx.x == 0) ovf = 0;
          __syncthreads();
          width >>= 1;
          continue;
        }
        best = umax64(best, pass);
        lo = hi;
        if (width < (1ull << 32)) width <<= 1;
      }
    }
    if (threadIdx.x == 0 && best) atomicMax(&hub_best[h], best);
  }
  if (ticket && last_block(ticket)) {
    if (threadIdx.x < 8) lcnt_next[threadIdx.x] = 0;
    final_rows<true>(threadIdx.x >> 6, kW, lcnt[1], listC, wcount, hoff, ghist_w, hub_best, Ln);
  }
}

__global__ __launch_bounds__(256) void k_hub_final(const int32_t* __restrict__ listC,
                                                   const int32_t* __restrict__ lcnt,
                                                   int32_t* __restrict__ wcount,
                                                   const int64_t* __restrict__ hoff,
                                                   int32_t* __restrict__ ghist,
                                                   u64* __restrict__ hub_best,
                                                   int32_t* __restrict__ Ln,
                                                   int32_t* __restrict__ lcnt_next) {
  // the next superstep's queue counters (the other parity; no memset launch)
  if (blockIdx.x == 0 && threadIdx.x < 8) lcnt_next[threadIdx.x] = 0;
  final_rows<false>(blockIdx.x * 4 + (threadIdx.x >> 6), gridDim.x * 4, lcnt[1], listC, wcount, hoff, ghist,
                    hub_best, Ln);
}

__global__ void k_hub_bounds(const int32_t* __restrict__ deg_own, int64_t n_hub,
                             int32_t* __restrict__ nb, int32_t* __restrict__ nc) {
  for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n_hub;
       h += (int64_t)gridDim.x * blockDim.x) {
    const int d = deg_own[h];  // staged words <= arcs
    int lg = 0;
    if (d > kCombDirect) {
      lg = ceil_log2((u32)((d + kCombWords - 1) / kCombWords));
      lg = lg < kMaxBucketsLg ? lg : kMaxBucketsLg;
    }
    nb[h] = 1 << lg;
    const int nu = (d + kSegArcs - 1) / kSegArcs;
    nc[h] = (nu + kChunkUnits - 1) / kChunkUnits;
  }
}

// first index of the non-increasing deg[0, n) with deg <= t
__global__ void k_first_le(const int32_t* __restrict__ deg, int64_t n, int32_t t, int64_t* out) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (deg[mid] > t) lo = mid + 1; else hi = mid;
  }
  *out = lo;
}

inline unsigned grid_cap(int64_t want, int64_t cap) {
  if (want < 1) want = 1;
  return (unsigned)(want < cap ? want : cap);
}

}  // namespace

int build_hub_tables(lpa_graph* g, const int32_t* deg_own) {
  hipStream_t s = g->stream;
  const int64_t n = g->n_hub;
  if (n == 0) return LPA_OK;
  int64_t hub_arcs = 0;
  LPA_HIP(hipMemcpyAsync(&hub_arcs, g->rp + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  int32_t *nb = nullptr, *nc = nullptr;
  int64_t* coff = nullptr;
  LPA_TRY(scratch_alloc(g, (void**)&nb, sizeof(int32_t) * n));
  LPA_TRY(scratch_alloc(g, (void**)&nc, sizeof(int32_t) * n));
  LPA_TRY(scratch_alloc(g, (void**)&coff, sizeof(int64_t) * (n + 1)));
  hipLaunchKernelGGL(k_hub_bounds, dim3(grid_cap((n + 255) / 256, 65536)), dim3(256), 0, s, deg_own,
                     n, nb, nc);
  LPA_HIP(hipGetLastError());
  LPA_TRY(dev_alloc(g, (void**)&g->hub_hoff, sizeof(int64_t) * (n + 1)));
  LPA_TRY(exclusive_scan_i32_i64(nb, g->hub_hoff, n, s));
  LPA_TRY(exclusive_scan_i32_i64(nc, coff, n, s));
  int64_t nbk = 0, nch = 0;
  LPA_HIP(hipMemcpyAsync(&nbk, g->hub_hoff + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipMemcpyAsync(&nch, coff + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  LPA_HIP(hipStreamSynchronize(s));
  scratch_free(g, nb);
  scratch_free(g, nc);
  scratch_free(g, coff);
  if (nbk > INT32_MAX || nch > INT32_MAX || hub_arcs > ((int64_t)1 << 40)) {
    set_error("hub combine tables too large (%lld buckets, %lld chunks)", (long long)nbk,
              (long long)nch);
    return LPA_EINVAL;
  }
  g->n_hub_buckets = nbk;
  g->n_hub_chunks = nch;
  LPA_TRY(dev_alloc(g, (void**)&g->stage, sizeof(u64) * hub_arcs));
  LPA_TRY(dev_alloc(g, (void**)&g->scat, sizeof(u64) * hub_arcs));
  LPA_TRY(dev_alloc(g, (void**)&g->hub_wcount, sizeof(int32_t) * n));
  LPA_TRY(dev_alloc(g, (void**)&g->hub_best, sizeof(u64) * n));
  LPA_TRY(dev_alloc(g, (void**)&g->ghist, sizeof(int32_t) * nbk));
  LPA_TRY(dev_alloc(g, (void**)&g->gcur, sizeof(int32_t) * nbk));
  LPA_TRY(dev_alloc(g, (void**)&g->hub_lists, sizeof(int32_t) * 6 * n));
  LPA_TRY(dev_alloc(g, (void**)&g->hub_lcnt, sizeof(int32_t) * 16));
  LPA_HIP(hipMemsetAsync(g->hub_lcnt, 0, sizeof(int32_t) * 16, s));
  // the fused count / bucket kernels' two-level tickets
  LPA_TRY(dev_alloc(g, (void**)&g->hub_tickets, sizeof(uint32_t) * 2 * kTicketWords));
  LPA_HIP(hipMemsetAsync(g->hub_tickets, 0, sizeof(uint32_t) * 2 * kTicketWords, s));
  {
    // rows [hub_lane_begin, n_hub) have <= kLaneUnits units (degree-descending order)
    int64_t* d_pos = nullptr;
    LPA_TRY(scratch_alloc(g, (void**)&d_pos, sizeof(int64_t)));
    hipLaunchKernelGGL(k_first_le, dim3(1), dim3(1), 0, s, deg_own, n, kLaneUnits * kSegArcs, d_pos);
    LPA_HIP(hipGetLastError());
    LPA_HIP(hipMemcpyAsync(&g->hub_lane_begin, d_pos, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    // rows [hub_block2_begin, hub_lane_begin): the wide block tier (<= kBlockMaxDeg2)
    hipLaunchKernelGGL(k_first_le, dim3(1), dim3(1), 0, s, deg_own, n, kBlockMaxDeg2, d_pos);
    LPA_HIP(hipGetLastError());
    LPA_HIP(hipMemcpyAsync(&g->hub_block2_begin, d_pos, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    LPA_HIP(hipStreamSynchronize(s));
    scratch_free(g, d_pos);
  }
  LPA_TRY(dev_alloc(g, (void**)&g->items_cb, sizeof(u64) * nbk));
  LPA_TRY(dev_alloc(g, (void**)&g->items_cc, sizeof(u64) * nch));
  LPA_HIP(hipMemsetAsync(g->hub_wcount, 0, sizeof(int32_t) * n, s));
  LPA_HIP(hipMemsetAsync(g->hub_best, 0, sizeof(u64) * n, s));
  LPA_HIP(hipMemsetAsync(g->ghist, 0, sizeof(int32_t) * nbk, s));
  return LPA_OK;
}

// the giant-label decision of superstep 2 (before the combine, on the main stream):
// k_hub_decide over the unit-tallied rows [0, h_end), then the exact unit tally of the
// units it listed (k_lpa_units in list mode, launched by the caller's lambda)
int launch_hub_decide(lpa_graph* g, int32_t* Lown, int64_t h_end, const int32_t* gsel) {
  if (h_end <= 0) return LPA_OK;
  hipLaunchKernelGGL(k_hub_decide, dim3(grid_cap((h_end + 3) / 4, 2048)), dim3(256), 0, g->stream, h_end,
                     g->hub_uoff, g->ugc, g->umx, gsel, Lown, g->hub_wcount, g->ulist2, g->gdec,
                     block_rows_begin(g), g->glist);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

int launch_hub_combine(lpa_graph* g, int32_t* Lown, bool fork, bool join, bool giant) {
  const int64_t n = g->n_hub;
  if (n == 0) return LPA_OK;
  hipStream_t s = g->stream;
  int32_t* lists = g->hub_lists;
  int32_t* listC = g->hub_lists + n;
  // queue counters of this superstep's parity (zeroed by the previous k_hub_final)
  int32_t* lcnt = g->hub_lcnt + 8 * g->par;
  const int64_t hl = g->hub_lane_begin;
  // rows classified for the combine in the fork: in block mode only those above the
  // block tiers (their units staged nothing)
  const int64_t hc = block_mode_now(g) ? block_rows_begin(g) : hl;
  // fork (label-dense supersteps): classify the > 8-unit rows first and start the
  // bucket path on its own stream; the mid tiers follow k_hub_small on the main
  // stream.  Otherwise everything runs in order on the main stream.  In block mode the
  // fourth stream runs the wide block tier, so the bucket path follows the wave bins
  // on the second.
  const bool bm = block_mode_now(g) && !g->serial;
  hipStream_t sd = !fork ? s : bm ? g->aux_stream[0] : g->aux_stream[2];
  const unsigned ncl = grid_cap(g->n_hub_chunks, 2048);
  // fused (converged supersteps, few bucketed rows): the scan by the last block of
  // k_hub_count, the final pass by the last block of k_hub_bucket -- 5 dependent
  // launches -> 3; the label-dense supersteps, with ~10^2 bucketed rows of up to 4K
  // buckets each, keep the parallel k_hub_scan / k_hub_final
  const bool fuse = !fork;
  uint32_t* tickets = g->hub_tickets;
  int32_t* lcnt_next = g->hub_lcnt + 8 * (g->par ^ 1);
  auto bucket_path = [&]() -> int {
    // fused: grids of one resident wave of blocks (fewer tickets)
    hipLaunchKernelGGL(k_hub_count, dim3(fuse ? grid_cap(g->n_hub_chunks, 1024) : ncl), dim3(256), 0, sd,
                       g->items_cc, lcnt, g->rp,
                       g->hub_uoff, g->ucnt, g->stage, g->hub_wcount, g->hub_hoff, g->ghist,
                       fuse ? tickets : (uint32_t*)nullptr, listC, g->gcur);
    LPA_HIP(hipGetLastError());
    if (!fuse) {
      hipLaunchKernelGGL(k_hub_scan, dim3(grid_cap((n + 3) / 4, 256)), dim3(256), 0, sd, listC,
                         lcnt, g->hub_wcount, g->hub_hoff, g->ghist, g->gcur);
      LPA_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_hub_scatter, dim3(ncl), dim3(256), 0, sd, g->items_cc, lcnt, g->rp,
                       g->hub_uoff, g->ucnt, g->stage, g->hub_wcount, g->hub_hoff, g->gcur, g->scat);
    LPA_HIP(hipGetLastError());
    uint32_t* tb = fuse ? tickets + kTicketWords : (uint32_t*)nullptr;
    const unsigned nbk = grid_cap(g->n_hub_buckets, fuse ? 512 : 2048);
    hipLaunchKernelGGL(k_hub_bucket<8>, dim3(nbk), dim3(512), 0, sd,
                         g->items_cb, lcnt, g->rp, g->scat, g->hub_hoff, g->ghist, g->gcur,
                         g->hub_best, g->dev_err, tb, listC, g->hub_wcount, g->ghist, Lown, lcnt_next);
    LPA_HIP(hipGetLastError());
    if (!fuse) {
      hipLaunchKernelGGL(k_hub_final, dim3(grid_cap((n + 3) / 4, 256)), dim3(256), 0, sd, listC,
                         lcnt, g->hub_wcount, g->hub_hoff, g->ghist, g->hub_best, Lown, lcnt_next);
      LPA_HIP(hipGetLastError());
    }
    return LPA_OK;
  };
  if (fork) {
    if (hc > 0) {
      hipLaunchKernelGGL(k_hub_classify, dim3(grid_cap((hc + 3) / 4, 2048)), dim3(256), 0, s, hc, n,
                         g->rp, g->hub_uoff, g->ucnt, g->hub_wcount, lists, lcnt, g->items_cb,
                         g->items_cc, giant ? 1 : 0);
      LPA_HIP(hipGetLastError());
      hipLaunchKernelGGL(k_hub_enqueue, dim3(grid_cap((hc + 255) / 256, 2048)), dim3(256), 0, s, hc, n,
                         g->hub_uoff, g->hub_wcount, lists, lcnt);
      LPA_HIP(hipGetLastError());
    }
    LPA_HIP(hipEventRecord(g->ev_fork2, s));
    LPA_HIP(hipStreamWaitEvent(sd, g->ev_fork2, 0));
    LPA_TRY(bucket_path());
  }
  // converged supersteps with the frontier on (a few listed rows): k_hub_small takes the
  // lane-path rows too, one dependent launch fewer on the main stream's chain (same box:
  // C3 converged supersteps -4 us each, C4 -15 us; a range-mode one -- C5's superstep 5
  // -- +0.09 ms, its many small hub rows a wave each)
  const bool all_small = !fork && fused_now(g);
  const int64_t hd = all_small ? n : hc;
  if (hl < n && !block_mode_now(g) && !all_small) {  // block mode: k_lpa_block tallied these rows
    hipLaunchKernelGGL(k_hub_lanes, dim3(grid_cap((n - hl + 255) / 256, 2048)), dim3(256), 0, s, hl, n,
                       g->rp, g->hub_uoff, g->ucnt, g->stage, Lown, lists, n, g->hub_wcount, lcnt,
                       g->flist, g->fcnt + 16 * g->par, g->fr_all + g->par);
    LPA_HIP(hipGetLastError());
  }
  // direct rows [0, nd) when not forked: in block mode only those above the block tiers
  hipLaunchKernelGGL(k_hub_small, dim3(2048), dim3(256), 0, s, fork ? (int64_t)0 : hd, n, g->rp,
                     g->hub_uoff, g->ucnt, g->stage, g->hub_wcount, Lown, lists, lcnt, g->items_cb,
                     g->items_cc, g->flist, g->fcnt + 16 * g->par, g->fr_all + g->par);
  LPA_HIP(hipGetLastError());
  // one launch in the converged supersteps (few queued rows: saves two dependent
  // launches); the label-dense ones keep the per-tier launches (the 4-wave blocks of
  // the small tiers measured faster there: 5.95 vs 6.2 ms at C3 superstep 2)
  if (!fork) {
    hipLaunchKernelGGL((k_hub_mid_all<8>), dim3(grid_cap(n, 1024)), dim3(512), 0, s, lists, n, lcnt,
                       g->rp, g->hub_uoff, g->ucnt, g->stage, g->hub_wcount, Lown, g->dev_err);
    LPA_HIP(hipGetLastError());
  } else {
    hipLaunchKernelGGL((k_hub_mid<13, 8>), dim3(grid_cap(n, 512)), dim3(512), 0, s, lists + 4 * n,
                         lcnt, 6, g->rp, g->hub_uoff, g->ucnt, g->stage, g->hub_wcount, Lown,
                         g->dev_err);
    LPA_HIP(hipGetLastError());
    hipLaunchKernelGGL((k_hub_mid<12, 4>), dim3(grid_cap(n, 1024)), dim3(256), 0, s, lists + 3 * n,
                       lcnt, 5, g->rp, g->hub_uoff, g->ucnt, g->stage, g->hub_wcount, Lown,
                       g->dev_err);
    LPA_HIP(hipGetLastError());
    hipLaunchKernelGGL((k_hub_mid<11, 4>), dim3(grid_cap(n, 2048)), dim3(256), 0, s, lists, lcnt, 0,
                       g->rp, g->hub_uoff, g->ucnt, g->stage, g->hub_wcount, Lown, g->dev_err);
    LPA_HIP(hipGetLastError());
  }
  if (!fork) LPA_TRY(bucket_path());
  if (fork) {
    LPA_HIP(hipEventRecord(g->ev_join2[0], sd));
    if (join) LPA_HIP(hipStreamWaitEvent(s, g->ev_join2[0], 0));
  }
  return LPA_OK;
}

}  // namespace lpa
