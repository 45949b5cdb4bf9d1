// One LPA superstep on gfx950 (replaces GraphX
// LabelPropagation sendMessage/mergeMessage/vertexProgram driven by
// Pregel.apply -- SURVEY.md §2.2 U3/U4, §3.2).
//
// For every owned vertex v with deg(v) > 0:
//     L_next[v] = min{ l : cnt_v(l) = max_l' cnt_v(l') },  cnt_v(l) = #{arcs v->u : L_cur[u] = l}
//
// Data flow of a superstep (one handle = one rank's slice of the degree-sorted CSR):
//   0. lists    the rows (and hub units) the previous refresh marked dirty -> per-bin
//               row lists (k_frontier_lists); none after L0, a rebuild or many changes
//   1. tally    every arc's vote comes from al[i] = L_cur[col[i]], the replicated
//               neighbour label (GraphX ReplicatedVertexView: edge partitions hold
//               copies of the endpoint attributes).  al[] is STREAMED (coalesced,
//               non-temporal), so the tally has no random gathers.  With a frontier
//               only the listed rows are tallied: a row none of whose neighbours
//               changed keeps its label (exact, see lpa_internal.h).
//   2. exchange (P > 1) allgather of the owned label slices or of the changes.
//   3. refresh  the changed vertices (k_diff, or the exchange's change list) have
//               their new labels scattered into al[] through the CSC position index
//               (cptr/cpos) while they touch <= rebuild_frac of the arcs -- marking the
//               rows they dirty while <= frontier_frac -- otherwise al[] is rebuilt with
//               one gather pass al[i] = L_next[col[i]].
//   The refresh keeps the replica exact, so labels are bit-identical to the plain
//   gather formulation.
//
// A vote tally is packed into one 64-bit word  (count << 32) | ~label : the
// maximum word is the highest count and, among equal counts, the smallest label,
// so "mode with smallest-label tie-break" is a plain u64 max-reduction; an empty
// slot is 0 (label 0xFFFFFFFF never occurs; it also marks an empty lane below).
//
// Degree bins (vertices are degree-sorted, so each bin is a contiguous slot range
// and the rows a wave sees have near-equal length):
//   g1   deg == 1       thread per vertex: the neighbour's label
//   g2   deg == 2       min of the two labels (1-1 tie or equal)
//   g4 .. g64 deg <= G  G lanes per vertex, ballot "peel": each round takes the
//                       group's first unresolved label, counts its lanes with one
//                       64-bit ballot, retires them; a chunk still unresolved after
//                       3 rounds (label-dense) counts its groups in an LDS hash
//   w2..w16 deg <= 64*NC  one wave per vertex, NC chunks: cross-chunk peel in
//                       registers, the residual through a per-wave LDS hash
//   seg  deg > 1024     one wave per 512-arc unit (staged unit tally words), merged
//                       per row by the hub combine (lpa_hub.hip)
// Tables keep a touched-slot list: finishing a vertex costs O(distinct labels).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>

#include "lpa_internal.h"
#include "lpa_lane.h"

// LPA_TRACE (diagnostic build only): synchronise and log after every kernel
#ifdef LPA_TRACE
#define LPA_TRACE_POINT(name)                                        \
  do {                                                               \
    hipError_t te_ = hipStreamSynchronize(s);                        \
    fprintf(stderr, "[lpa-trace] %s done (%s)\n", name, hipGetErrorString(te_)); \
  } while (0)
#else
#define LPA_TRACE_POINT(name) \
  do {                        \
  } while (0)
#endif

namespace lpa {

namespace {

// Diagnostic ablations (separate builds only, `make diag`; never in liblpa_hip.so):
//   1 = stream the labels but skip the tally, 2 = skip the hub global merge,
//   3 = peel only (no LDS hash of the residual votes)
#ifndef LPA_DIAG
#define LPA_DIAG 0
#endif

// peel rounds of the wave / unit / block tallies in the label-dense supersteps, where a
// round rarely retires more than a few votes (measured best of 0/2/4/8 at C3)
constexpr int kDensePeel = 2;

}  // namespace

// the label-dense supersteps tally the rows [hub_lane_begin, n_hub) with k_lpa_block
// and skip their units; the superstep after them tallies every row (their units'
// staged words are stale)
bool block_mode_now(const lpa_graph* g) { return g->since_reset < kDenseSupersteps && g->hub_lane_begin < g->n_hub; }
int64_t block_rows_begin(const lpa_graph* g) { return g->hub_block2_begin; }

namespace {


constexpr int kChunks = 8;    // 64-arc chunks per wave: a wave-bin row / a quarter segment
constexpr u32 kNone = 0xFFFFFFFFu;  // empty lane
static_assert(kSegArcs == 64 * kChunks, "a unit is one batch of chunks");
static_assert(kWaveMaxDeg == 64 * kChunks, "a wave-bin row fits one batch of chunks");
static_assert(kWideMaxDeg == 2 * kWaveMaxDeg, "w16 rows: 16 chunks");

__device__ __forceinline__ u32 ld_stream(const int32_t* p) {
  return (u32)__builtin_nontemporal_load(p);
}

__device__ __forceinline__ u64 tally(u32 cnt, u32 label) {
  return ((u64)cnt << 32) | (u64)(u32)(~label);
}

__device__ __forceinline__ u64 umax64(u64 a, u64 b) { return a > b ? a : b; }

// Wave reductions over a FULL wave (every call site has all 64 lanes active):
// DPP within each 16-lane row (xor 1, xor 2, half-row mirror, row mirror: every
// lane ends with its row's result, VALU only, no LDS round trip), then the four
// row results via readlane (uniform result).
template <int kCtrl>
__device__ __forceinline__ u32 dpp_u32(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}
template <int kCtrl>
__device__ __forceinline__ u64 dpp_u64(u64 v) {
  return ((u64)dpp_u32<kCtrl>((u32)(v >> 32)) << 32) | (u64)dpp_u32<kCtrl>((u32)v);
}
__device__ __forceinline__ u64 readlane_u64(u64 v, int l) {
  return ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), l) << 32) |
         (u64)(u32)__builtin_amdgcn_readlane((int)(u32)v, l);
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
  v = umax64(v, dpp_u64<0xB1>(v));   // quad_perm [1,0,3,2]
  v = umax64(v, dpp_u64<0x4E>(v));   // quad_perm [2,3,0,1]
  v = umax64(v, dpp_u64<0x141>(v));  // row_half_mirror
  v = umax64(v, dpp_u64<0x140>(v));  // row_mirror
  return umax64(umax64(readlane_u64(v, 0), readlane_u64(v, 16)),
                umax64(readlane_u64(v, 32), readlane_u64(v, 48)));
}

__device__ __forceinline__ u32 wave_sum_u32(u32 v) {
  v += dpp_u32<0xB1>(v);
  v += dpp_u32<0x4E>(v);
  v += dpp_u32<0x141>(v);
  v += dpp_u32<0x140>(v);
  return (u32)__builtin_amdgcn_readlane((int)v, 0) + (u32)__builtin_amdgcn_readlane((int)v, 16) +
         (u32)__builtin_amdgcn_readlane((int)v, 32) + (u32)__builtin_amdgcn_readlane((int)v, 48);
}

__device__ __forceinline__ u32 wave_max_u32(u32 v) {
  v = max(v, dpp_u32<0xB1>(v));
  v = max(v, dpp_u32<0x4E>(v));
  v = max(v, dpp_u32<0x141>(v));
  v = max(v, dpp_u32<0x140>(v));
  return max(max((u32)__builtin_amdgcn_readlane((int)v, 0), (u32)__builtin_amdgcn_readlane((int)v, 16)),
             max((u32)__builtin_amdgcn_readlane((int)v, 32), (u32)__builtin_amdgcn_readlane((int)v, 48)));
}
// u64 max as two 32-bit reductions (the high words, then the low words of the lanes
// holding that high word): each DPP step is one v_max_u32 instead of two moves, a
// 64-bit compare and two selects -- fewer VALU issues, a longer dependent chain, so it
// serves only the issue-bound g64 row hash (C2 60.4 -> 61.6 GTEPS; as every kernel's
// wave max, C3's latency-bound converged supersteps lost 1.5 %)
__device__ __forceinline__ u64 wave_max_u64_split(u64 v) {
  const u32 hi = wave_max_u32((u32)(v >> 32));
  const u32 lo = wave_max_u32((u32)(v >> 32) == hi ? (u32)v : 0u);
  return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ u32 hash_slot(u32 label, int shift) {
  return (label * 0x9E3779B1u) >> shift;
}

__device__ __forceinline__ int ceil_log2(u32 x) { return x <= 1 ? 0 : 32 - __clz(x - 1); }

// Insert `cnt` votes for `label` into an LDS open-addressing table of (mask+1)
// slots.  Returns the slot index when this call claimed an empty slot, else -1.
__device__ __forceinline__ int lds_insert(u64* tab, int shift, u32 mask, u32 label, u32 cnt) {
  const u32 key = ~label;
  u32 h = hash_slot(label, shift);
  while (true) {
    u64 old = atomicCAS(&tab[h], 0ull, ((u64)cnt << 32) | key);
    if (old == 0ull) return (int)h;
    if ((u32)old == key) {
      atomicAdd(&tab[h], (u64)cnt << 32);
      return -1;
    }
    h = (h + 1u) & mask;
  }
}

// Continue a global-table insert whose first probe at slot h returned `old`;
// returns the claimed slot or -1 (merged into an existing key).
__device__ __forceinline__ int global_resolve(u64* tab, u32 mask, u64 word, u32 h, u64 old) {
  const u32 key = (u32)word;
  const u64 add = word & 0xFFFFFFFF00000000ull;
  while (true) {
    if (old == 0ull) return (int)h;
    if ((u32)old == key) {
      atomicAdd(&tab[h], add);
      return -1;
    }
    h = (h + 1u) & mask;
    old = atomicCAS(&tab[h], 0ull, word);
  }
}

// Continue an LDS insert of `word` whose probe at slot h hit another key.
__device__ __forceinline__ int lds_probe(u64* tab, u32 mask, u64 word, u32 h) {
  const u32 key = (u32)word;
  while (true) {
    h = (h + 1u) & mask;
    const u64 old = atomicCAS(&tab[h], 0ull, word);
    if (old == 0ull) return (int)h;
    if ((u32)old == key) {
      atomicAdd(&tab[h], word & 0xFFFFFFFF00000000ull);
      return -1;
    }
  }
}

// ---------------------------------------------------------------------------
// Tally of a batch of up to NC 64-arc chunks held in registers (kNone = empty
// lane; chunks >= nch, a uniform bound, are skipped).
//   peel_batch   (no LDS) the first active label of the batch and all its copies
//                are counted with one ballot per chunk and retired; repeated while
//                a round retires >= 2 lanes (a repeated label), up to kPeelMax.
//                Peel group p's tally word is left in lane p; pbest (uniform) is
//                their maximum.  A converged neighbourhood is usually resolved
//                here completely (nact == 0) and then needs no LDS at all.
//   hash_batch   the peel groups (one lane each) and every remaining lane go into
//                a wave-owned LDS open-addressing table: all first probes issued
//                back to back, then resolved; claimed slots appended to `lst`.
// ---------------------------------------------------------------------------
constexpr int kPeelMax = 8;

// The peel keeps its state per LANE in VGPRs (bit u of `mask` = this lane's label of
// chunk u is not yet tallied) and counts with VALU compares + a DPP wave sum: a
// compute unit issues one scalar instruction per cycle for all its waves but one
// vector instruction per SIMD, and per-chunk ballot/and/popcount chains made the
// steady-state tally kernels scalar-issue bound (SQ_INSTS_SALU 2.4x SQ_INSTS_VALU).
template <int NC>
struct Batch {
  u32 mask;    // per lane: chunks whose label is still untallied
  bool any;    // uniform: some lane still has an untallied label
  u64 pword;   // lane p: tally word of peel group p
  int npeel;   // uniform
  u64 pbest;   // uniform
};

template <int NC>
__device__ __forceinline__ void peel_batch(Batch<NC>& bt, const u32 (&lab)[NC], int nch, int lane,
                                           int pmax = kPeelMax, bool whole_row = false) {
  u32 mask = 0u;
#pragma unroll
  for (int u = 0; u < NC; ++u)
    if (u < nch && lab[u] != kNone) mask |= 1u << u;
  bt.pword = 0ull;
  bt.npeel = 0;
  bt.pbest = 0ull;
#pragma unroll 1
  for (int p = 0; p < pmax; ++p) {
    const u64 live = __ballot(mask != 0u);
    if (live == 0ull) break;
    // candidate: the first untallied label of the first lane that has one
    u32 cand = 0u;
#pragma unroll
    for (int u = NC - 1; u >= 0; --u)
      if ((mask >> u) & 1u) cand = lab[u];
    const u32 x = (u32)__builtin_amdgcn_readlane((int)cand, __ffsll((unsigned long long)live) - 1);
    u32 m = 0u;
#pragma unroll
    for (int u = 0; u < NC; ++u)
      if (lab[u] == x) m |= 1u << u;
    m &= mask;
    mask &= ~m;
    const u32 c = wave_sum_u32((u32)__popc(m));
    const u64 word = tally(c, x);
    if (lane == p) bt.pword = word;
    bt.pbest = umax64(bt.pbest, word);
    bt.npeel = p + 1;
    // whole_row (the batch is the entire row): decided once the best count exceeds
    // the untallied votes -- the rest is dropped, no LDS hash
    if (whole_row && (u32)(bt.pbest >> 32) > wave_sum_u32((u32)__popc(mask))) {
      mask = 0u;
      break;
    }
    if (c < 2) break;
  }
  bt.mask = mask;
  bt.any = __ballot(mask != 0u) != 0ull;
}

// kList = false: a shared (block) table scanned at the end, no touched-slot list
template <int NC, bool kList = true>
__device__ __forceinline__ void hash_batch(u64* tab, uint16_t* lst, int& cnt, int shift, u32 mask,
                                           const Batch<NC>& bt, const u32 (&lab)[NC], int nch,
                                           int lane, u64 lt) {
  int pslot = -1;
  if (lane < bt.npeel) pslot = lds_insert(tab, shift, mask, ~(u32)bt.pword, (u32)(bt.pword >> 32));
  if constexpr (kList) {
    const u64 cm = __ballot(pslot >= 0);
    if (pslot >= 0) lst[cnt + __popcll(cm & lt)] = (uint16_t)pslot;
    cnt += __popcll(cm);
  }
  // chunks in groups of up to 8 (bounded registers for the in-flight CAS results)
  constexpr int H = NC < 8 ? NC : 8;
#pragma unroll
  for (int h0 = 0; h0 < NC; h0 += H) {
    if (h0 >= nch) break;  // uniform
    u64 old[H];
    u32 hh[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      const int u = h0 + k;
      old[k] = 0ull;
      hh[k] = 0u;
      if (u < nch && ((bt.mask >> u) & 1u)) {
        hh[k] = hash_slot(lab[u], shift);
        old[k] = atomicCAS(&tab[hh[k]], 0ull, (1ull << 32) | (u64)(u32)(~lab[u]));
      }
    }
    int slot[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      const int u = h0 + k;
      slot[k] = -1;
      if (u < nch && ((bt.mask >> u) & 1u)) {
        const u64 word = (1ull << 32) | (u64)(u32)(~lab[u]);
        if (old[k] == 0ull) {
          slot[k] = (int)hh[k];
        } else if ((u32)old[k] == (u32)word) {
          atomicAdd(&tab[hh[k]], 1ull << 32);
        } else {
          slot[k] = lds_probe(tab, mask, word, hh[k]);
        }
      }
    }
    if constexpr (kList) {
#pragma unroll
      for (int k = 0; k < H; ++k) {
        if (h0 + k < nch) {
          const u64 cm = __ballot(slot[k] >= 0);
          if (slot[k] >= 0) lst[cnt + __popcll(cm & lt)] = (uint16_t)slot[k];
          cnt += __popcll(cm);
        }
      }
    }
  }
}

template <int NC>
__device__ __forceinline__ void load_labels(u32 (&lab)[NC], const int32_t* __restrict__ al,
                                            int64_t b, int64_t e, int lane) {
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int64_t i = b + u * 64 + lane;
    lab[u] = i < e ? ld_stream(al + i) : kNone;
  }
}

// ---------------------------------------------------------------------------
// The giant label of the label-dense supersteps.  One label G -- the current label of
// the top hub, L[slot 0] -- is the STRICT mode of nearly every row of more than 64
// arcs in superstep 2 (R-MAT, oracle at scale 22: G holds ~36 % of the votes of every
// degree band, a median 10-13x the next label's count).  giant_count counts G's votes
// exactly and adds every other vote to a bucket of a small label-hash histogram: a
// label's count is at most its bucket's, so G's count above every bucket decides the
// row -- no hash table, no probe chains, no table scan.  A row it cannot decide (G not
// the strict mode, or a bucket too full) takes the exact tally.
// ---------------------------------------------------------------------------
constexpr int kGiantLg = 6;   // wave histogram: 64 buckets, one per lane

// this lane's G votes among its labels; the others into hist (bucket = label hash >>
// (32 - lg)); no-return LDS adds
template <int NC>
__device__ __forceinline__ u32 giant_count(const u32 (&lab)[NC], int nch, u32 G, u32* hist, int lg) {
  u32 c = 0;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    if (u >= nch) break;  // uniform
    const u32 x = lab[u];
    if (x == G) ++c;
    else if (x != kNone) atomicAdd(&hist[hash_slot(x, 32 - lg)], 1u);
  }
  return c;
}

// one wave, one row in registers: true when G is decided (its count above every
// bucket); the histogram (kGiantLg buckets at hist) is left zeroed either way
template <int NC>
__device__ __forceinline__ bool giant_decide(const u32 (&lab)[NC], int nch, u32 G, u32* hist, int lane) {
  const u32 cg = wave_sum_u32(giant_count<NC>(lab, nch, G, hist, kGiantLg));
  __builtin_amdgcn_wave_barrier();  // no reordering across (LDS ops of a wave complete in order)
  const u32 b = hist[lane];
  hist[lane] = 0u;
  return cg > wave_max_u32(b);
}

// ---------------------------------------------------------------------------
// bins g1 / g2 / g4 / g8 / g16
// ---------------------------------------------------------------------------
// Frontier row lists (k_frontier_lists): with *fr_all == 0 a bin kernel tallies only
// the dirty rows of its bin, listed at flist[vbeg, vbeg + *fcnt); otherwise its whole
// slot range [vbeg, vend).  Index i of the bin's work -> row.
struct BinRows {
  int64_t vbeg, n;
  const int32_t* list;  // nullptr: range mode
  __device__ __forceinline__ int64_t row(int64_t i) const { return list ? (int64_t)list[vbeg + i] : vbeg + i; }
};
__device__ __forceinline__ BinRows bin_rows(int64_t vbeg, int64_t vend, const int32_t* __restrict__ flist,
                                            const int32_t* __restrict__ fcnt_b,
                                            const int32_t* __restrict__ fr_all) {
  BinRows br;
  br.vbeg = vbeg;
  if (*fr_all) {
    br.n = vend - vbeg;
    br.list = nullptr;
  } else {
    br.n = *fcnt_b;
    br.list = flist;
  }
  return br;
}

// Mode of each G-lane group's labels through a wave-owned LDS table (kRowsHashSlots u64
// slots, zero on entry and on return): group k owns slots [4G k, 4G (k + 1)) (load
// <= 1/4), every lane inserts its label -- a CAS claims an empty slot with count 1, a
// lane finding its own key adds 1 (lanes of one instruction that hit one address are
// applied one after another, each seeing the previous result) -- then reads its slot
// back: the slot holds its label's tally word.  A group max of the words gives the
// mode (every lane of a group returns it).  ~35 vector instructions per 64 labels where
// the 21-stage bitonic network it replaced (round 2: DPP / permlane exchanges) cost
// ~150, and k_lpa_rows<64> was VALU-issue bound in the label-dense supersteps (C2: 884 K
// rows of 33-64 arcs; C2 47.7 -> 55.5 GTEPS, dense supersteps 0.60 -> 0.49 ms).
constexpr int kRowsHashSlots = 256;
template <int G>
__device__ __forceinline__ u64 group_mode_hash(u32 v, int lane, u64* tab) {
  static_assert(G >= 2 && G <= 64 && (G & (G - 1)) == 0, "group width");
  constexpr int kLg = (G == 64 ? 6 : G == 32 ? 5 : G == 16 ? 4 : G == 8 ? 3 : G == 4 ? 2 : 1) + 2;
  constexpr u32 kMask = (1u << kLg) - 1u;
  u64* gt = tab + (lane & ~(G - 1)) * 4;
  u64 w = 0ull;
#if LPA_DIAG == 1
  // diagnostic (timing only, wrong modes): no table, each vote counted once
  if (v != kNone) w = (1ull << 32) | (u64)(u32)(~v);
  if (false) {
#else
  if (v != kNone) {
#endif
    const u64 word = (1ull << 32) | (u64)(u32)(~v);
    u32 h = hash_slot(v, 32 - kLg);
    while (true) {
      const u64 old = atomicCAS(&gt[h], 0ull, word);
      if (old == 0ull) break;
      if ((u32)old == (u32)word) {
        atomicAdd(&gt[h], 1ull << 32);
        break;
      }
      h = (h + 1u) & kMask;
    }
    __builtin_amdgcn_wave_barrier();
    w = gt[h];
    __builtin_amdgcn_wave_barrier();
    gt[h] = 0ull;
  }
  if constexpr (G == 64) {
    return wave_max_u64_split(w);
  } else {
#pragma unroll
    for (int off = G >> 1; off > 0; off >>= 1) {
      const u64 o = ((u64)lane::lane_xor((u32)(w >> 32), off, lane) << 32) | (u64)lane::lane_xor((u32)w, off, lane);
      w = umax64(w, o);
    }
    return w;
  }
}

#if LPA_DIAG == 2
#define LPA_GV(x) (x)
#else
#define LPA_GV(x) ((u32)Lg[(int32_t)(x)])
#endif

// peel rounds after which a chunk whose groups are still unresolved is hashed instead
constexpr int kPeelSortAfter = 3;



// lanes of the groups already decided after a peel round: a group whose best count
// so far exceeds its untallied votes cannot change its mode (no remaining label can
// reach, or tie, that count), so its lanes retire without further rounds -- a
// converged row (one dominant label plus a few strays) stops after one round instead
// of peeling the strays one by one and then hashing
template <int G>
__device__ __forceinline__ u64 decided_groups(u64 act, u64 my, u64 best, int gbase, u64 gm) {
  const u32 rem = (u32)__popcll((act >> gbase) & gm);
  return __ballot(my != 0ull && (u32)(best >> 32) > rem);
}

// A vote of arc i.  Gather mode (kG, lpa_build: one GPU, a label vector that stays in L2,
// no row above 128 arcs -- C2): src is col and the vote is L[col[i]], read from the
// current vector itself, so no al[] refresh runs at all; otherwise src is al[].
template <bool kG>
__device__ __forceinline__ u32 arc_vote(const int32_t* __restrict__ src, const int32_t* __restrict__ L, int64_t i) {
#if LPA_DIAG == 2
  // diagnostic (timing only, wrong votes): the column itself, no label gather
  if constexpr (kG) return ld_stream(src + i);
#else
  if constexpr (kG) return (u32)L[(int32_t)ld_stream(src + i)];
#endif
  else return ld_stream(src + i);
}

// the mode of each G-lane group's votes (kNone: no vote), written to Ln[v] by the group's
// first lane when live
template <int G>
__device__ __forceinline__ void group_tally(u32 lab, int32_t* __restrict__ Ln, int64_t v, bool live, int lane,
                                            u64* tab) {
  const int j = lane & (G - 1);
  if constexpr (G == 1) {
    if (live) Ln[v] = (int32_t)lab;
  } else if constexpr (G == 2) {
    const u32 o = (u32)__shfl_xor((int)lab, 1, 64);
    if (live && j == 0) Ln[v] = (int32_t)(lab < o ? lab : o);
  } else {
    const int gbase = lane & ~(G - 1);
    const u64 gm = G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull);
    u64 act = __ballot(lab != kNone);
    u64 best = 0ull;
    for (int round = 0; act; ++round) {
      if (G >= 8 && round == kPeelSortAfter) {  // uniform: a label-dense chunk
        best = group_mode_hash<G>(lab, lane, tab);
        break;
      }
      const u64 my = (act >> gbase) & gm;
      const int lead = gbase + (my ? (__ffsll((unsigned long long)my) - 1) : 0);
      const u32 x = (u32)__shfl((int)lab, lead, 64);
      const u64 mm = __ballot(((act >> lane) & 1ull) && lab == x);
      const u32 c = (u32)__popcll((mm >> gbase) & gm);
      if (my) best = umax64(best, tally(c, x));
      act &= ~mm;
      act &= ~decided_groups<G>(act, my, best, gbase, gm);
    }
    if (live && j == 0) Ln[v] = (int32_t)(~(u32)best);
  }
}

// G lanes per row (G <= 64, all 64 lanes of the wave call it: ballot peel)
template <int G, bool kG = false>
__device__ __forceinline__ void group_row(const int64_t* __restrict__ rp, const int32_t* __restrict__ al,
                                          int32_t* __restrict__ Ln, int64_t v, bool live, int lane,
                                          u64* tab = nullptr, const int32_t* __restrict__ Lg = nullptr) {
  const int j = lane & (G - 1);
  int64_t b = 0;
  int d = 0;
  if (live) {
    b = rp[v];
    d = (int)(rp[v + 1] - b);
  }
  const u32 lab = j < d ? arc_vote<kG>(al, Lg, b + j) : kNone;
  group_tally<G>(lab, Ln, v, live, lane, tab);
}

// (the bin bodies below take their block index and block count as arguments: a kernel
// of its own passes blockIdx / gridDim, k_bins_fused its share of one launch)
template <int G, bool kG = false>
__device__ __forceinline__ void group_bin(int64_t bid, int64_t nblk, const int64_t* __restrict__ rp,
                                          const int32_t* __restrict__ al, int32_t* __restrict__ Ln,
                                          int64_t vbeg, int64_t vend, const int32_t* __restrict__ flist,
                                          const int32_t* __restrict__ fcnt_b, const int32_t* __restrict__ fr_all,
                                          const int32_t* __restrict__ Lg) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const BinRows br = bin_rows(vbeg, vend, flist, fcnt_b, fr_all);
  // 64 / G rows per wave; grid-stride by waves (the grid is sized to the range: one pass)
  constexpr int64_t kRows = 64 / G;
  for (int64_t wb = (bid * 4 + w) * kRows; wb < br.n; wb += nblk * 4 * kRows) {
    const int64_t i = wb + lane / G;
    const bool live = i < br.n;
    group_row<G, kG>(rp, al, Ln, live ? br.row(i) : 0, live, lane, nullptr, Lg);
  }
}

template <int G, bool kG = false>
__global__ __launch_bounds__(256) void k_lpa_group(const int64_t* __restrict__ rp,
                                                   const int32_t* __restrict__ al,
                                                   int32_t* __restrict__ Ln, int64_t vbeg,
                                                   int64_t vend, const int32_t* __restrict__ flist,
                                                   const int32_t* __restrict__ fcnt_b,
                                                   const int32_t* __restrict__ fr_all,
                                                   const int32_t* __restrict__ Lg) {
  group_bin<G, kG>(blockIdx.x, gridDim.x, rp, al, Ln, vbeg, vend, flist, fcnt_b, fr_all, Lg);
}

// ---------------------------------------------------------------------------
// bins w2 / w4 / w8: 64 < deg <= 64 * NC, one wave per vertex, grid-stride,
// software-pipelined: the next vertex's labels stream in while the current one is
// tallied (row bounds two vertices ahead).  Per-wave LDS table of 2 * 64 * NC.
// ---------------------------------------------------------------------------
struct RowSpan {
  int64_t b, e;
};

// bounds of work item i of the bin (row br.row(i)); past the end: an empty span
__device__ __forceinline__ RowSpan row_span(const int64_t* __restrict__ rp, const BinRows& br, int64_t i) {
  RowSpan r;
  r.b = 0;
  r.e = 0;
  if (i < br.n) {
    const int64_t v = br.row(i);
    r.b = rp[v];
    r.e = rp[v + 1];
  }
  return r;
}

__device__ __forceinline__ int span_len(const RowSpan& r) { return (int)(r.e - r.b); }

// unconditional loads of a row's labels (address clamped into the row)
template <int NC>
__device__ __forceinline__ void row_load(u32 (&raw)[NC], const int32_t* __restrict__ al,
                                         const RowSpan& r, int lane) {
  const int d = span_len(r);
  if (__builtin_amdgcn_readfirstlane(d) == 0) {  // frontier-clean row: no loads
#pragma unroll
    for (int c = 0; c < NC; ++c) raw[c] = kNone;
    return;
  }
  const int last = d > 0 ? d - 1 : 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int off = c * 64 + lane;
    raw[c] = ld_stream(al + r.b + (off < last ? off : last));
  }
}

// branch-free form (k_lpa_wave's ring): an empty span (past the bin's end) loads
// al[0] and its labels are never read -- no control flow for the waitcnt pass to merge
template <int NC, bool kG = false>
__device__ __forceinline__ void row_load_nb(u32 (&raw)[NC], const int32_t* __restrict__ al,
                                            const RowSpan& r, int lane, const int32_t* __restrict__ Lg = nullptr) {
  const int d = span_len(r);
  const int last = d > 0 ? d - 1 : 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int off = c * 64 + lane;
    raw[c] = arc_vote<kG>(al, Lg, r.b + (off < last ? off : last));
  }
}

template <int NC>
__device__ __forceinline__ void row_tally(const u32 (&raw)[NC], const RowSpan& r, int64_t v,
                                          int32_t* __restrict__ Ln, u64* tab, uint16_t* lst, int lane,
                                          u64 lt, int pmax, bool giant, u32 G) {
  const int d = span_len(r);
  if (d == 0) return;
  u32 lab[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) lab[c] = c * 64 + lane < d ? raw[c] : kNone;
  int lg = ceil_log2(2u * (u32)d);
  lg = lg < 6 ? 6 : lg;
  const int nch = (d + 63) >> 6;
  // label-dense supersteps: the giant label first (the table's first 64 words, zero)
  if (giant && giant_decide<NC>(lab, nch, G, reinterpret_cast<u32*>(tab), lane)) {
    if (lane == 0) Ln[v] = (int32_t)G;
    return;
  }
  Batch<NC> bt;
  peel_batch<NC>(bt, lab, nch, lane, pmax, true);
  if (!bt.any) {
    // every vote is in a peel group (or the rest cannot win): the mode is their
    // maximum, no LDS needed
    if (lane == 0) Ln[v] = (int32_t)(~(u32)bt.pbest);
  } else {
    int cnt = 0;
    hash_batch<NC>(tab, lst, cnt, 32 - lg, (1u << lg) - 1u, bt, lab, nch, lane, lt);
    u64 best = 0ull;
    for (int i = lane; i < cnt; i += 64) {
      const int sl = lst[i];
      best = umax64(best, tab[sl]);
      tab[sl] = 0ull;
    }
    best = wave_max_u64(best);
    if (lane == 0) Ln[v] = (int32_t)(~(u32)best);
  }
}

// Row bounds of 64 work items of a wave in one load per lane: lane k holds item
// i0 + k * stride (its row, arc begin and end; empty past the bin's end).  The label
// loads of a row take its bounds by readlane, so they never wait on a bounds load
// issued after the label loads still in flight (vmcnt counts in order: a wait for the
// newest load is a wait for every older one).
struct SpanBatch {
  int64_t b, e;
  int32_t v;
};
__device__ __forceinline__ SpanBatch span_batch(const int64_t* __restrict__ rp, const BinRows& br, int64_t i0,
                                                int64_t stride, int lane) {
  SpanBatch sb;
  sb.b = sb.e = 0;
  sb.v = 0;
  const int64_t i = i0 + (int64_t)lane * stride;
  if (i < br.n) {
    const int64_t v = br.row(i);
    sb.v = (int32_t)v;
    sb.b = rp[v];
    sb.e = rp[v + 1];
  }
  return sb;
}
__device__ __forceinline__ int64_t readlane_i64(int64_t x, int l) {
  return (int64_t)(((u64)(u32)__builtin_amdgcn_readlane((int)(u32)((u64)x >> 32), l) << 32) |
                   (u64)(u32)__builtin_amdgcn_readlane((int)(u32)(u64)x, l));
}
// item q of the two batches (q < 64: cur, else nxt; uniform).  A branch, not a select:
// readlane is convergent (not speculated), so the cur side never waits for nxt's load.
__device__ __forceinline__ RowSpan span_at(const SpanBatch& cur, const SpanBatch& nxt, int q) {
  RowSpan r;
  if (q < 64) {
    r.b = readlane_i64(cur.b, q);
    r.e = readlane_i64(cur.e, q);
  } else {
    r.b = readlane_i64(nxt.b, q - 64);
    r.e = readlane_i64(nxt.e, q - 64);
  }
  return r;
}

// label register sets in the k_lpa_wave ring: labels of the next D - 1 rows in flight
// while a row is tallied
template <int NC>
constexpr int wave_ring_depth() { return NC <= 2 ? 6 : NC <= 4 ? 4 : 3; }

// bins w2 / w4 / w8 / w16 (64 < deg <= 64 * NC): one wave per row, grid-stride; D
// label register sets in an unrolled ring (labels D - 1 rows ahead), row bounds by
// 64-row batches one batch ahead (span_batch).
// (tab_all / lst_all: the block's LDS, 4 waves x 2 * 64 * NC table slots / 64 * NC
// list entries)
template <int NC, bool kG = false>
__device__ __forceinline__ void wave_bin(int64_t bid, int64_t nblk, u64* tab_all, uint16_t* lst_all,
                                         const int64_t* __restrict__ rp, const int32_t* __restrict__ al,
                                         int32_t* __restrict__ Ln, int64_t vbeg, int64_t vend,
                                         const int32_t* __restrict__ flist, const int32_t* __restrict__ fcnt_b,
                                         const int32_t* __restrict__ fr_all, int pmax,
                                         const int32_t* __restrict__ gsel, const int32_t* __restrict__ Lg) {
  constexpr int kCap = 2 * 64 * NC;
  constexpr int D = wave_ring_depth<NC>();
  static_assert(D >= 2 && D <= 64, "ring depth");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u64* tab = tab_all + w * kCap;
  uint16_t* lst = lst_all + w * 64 * NC;
  const u64 lt = (1ull << lane) - 1ull;
  const int64_t stride = nblk * 4;
  const BinRows br = bin_rows(vbeg, vend, flist, fcnt_b, fr_all);
  int64_t ib = bid * 4 + w;   // work item of the current batch's lane 0
  if (ib >= br.n) return;  // no block-level barriers in this body
  for (int k = lane; k < kCap; k += 64) tab[k] = 0ull;  // only waves with rows clear
  // gsel (label-dense supersteps): the giant-label word of the labels this superstep
  // reads (k_giant_pick: label, worth trying)
  const bool giant = gsel != nullptr && gsel[1] != 0;
  const u32 G = giant ? (u32)gsel[0] : 0u;
  SpanBatch cur = span_batch(rp, br, ib, stride, lane);
  SpanBatch nxt;  // the next batch: loaded at p == 32, half a batch before its first use
  nxt.b = nxt.e = 0;
  nxt.v = 0;
  int p = 0;  // current row: work item ib + p * stride
  u32 rl[D][NC];
#pragma unroll
  for (int k = 0; k < D - 1; ++k) row_load_nb<NC, kG>(rl[k], al, span_at(cur, nxt, k), lane, Lg);
  while (true) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      row_load_nb<NC, kG>(rl[(k + D - 1) % D], al, span_at(cur, nxt, p + D - 1), lane, Lg);
      const RowSpan s = span_at(cur, nxt, p);
      const int64_t v = (int64_t)__builtin_amdgcn_readlane(cur.v, p);
      row_tally<NC>(rl[k], s, v, Ln, tab, lst, lane, lt, pmax, giant, G);
      if (ib + (int64_t)(p + 1) * stride >= br.n) return;
      ++p;
      if (p == 32) nxt = span_batch(rp, br, ib + 64 * stride, stride, lane);
      if (p == 64) {
        p = 0;
        ib += 64 * stride;
        cur = nxt;
      }
    }
  }
}

template <int NC, bool kG = false>
__global__ __launch_bounds__(256) void k_lpa_wave(const int64_t* __restrict__ rp,
                                                  const int32_t* __restrict__ al,
                                                  int32_t* __restrict__ Ln, int64_t vbeg,
                                                  int64_t vend, const int32_t* __restrict__ flist,
                                                  const int32_t* __restrict__ fcnt_b,
                                                  const int32_t* __restrict__ fr_all, int pmax,
                                                  const int32_t* __restrict__ gsel,
                                                  const int32_t* __restrict__ Lg) {
  __shared__ u64 tab_all[4 * 2 * 64 * NC];
  __shared__ uint16_t lst_all[4 * 64 * NC];
  wave_bin<NC, kG>(blockIdx.x, gridDim.x, tab_all, lst_all, rp, al, Ln, vbeg, vend, flist, fcnt_b, fr_all, pmax,
                   gsel, Lg);
}

// ---------------------------------------------------------------------------
// Label-dense supersteps only: seg-bin rows of kSegArcs < deg <= kBlockMaxDeg (the hub
// rows [hub_lane_begin, n_hub), degree-descending), one block per row, tallied
// straight from al[].  Wave w takes the row's 512-arc batch w (ballot peel in
// registers, residual votes into the block's shared LDS table of 2^ceil(log2(2 deg))
// slots), then the block scans and clears the table.  When nearly every vote is a
// distinct label, staging a unit's words and re-tallying them in the combine costs
// about twice the direct tally; once labels settle the unit path is cheaper (a dirty
// row re-tallies only its dirty units), so the converged supersteps keep it.
// Grid-stride over the rows (frontier: over the listed bin-0 rows, those below h0
// belong to the hub combine).
// ---------------------------------------------------------------------------
template <int kLg, int kBlockWaves>
__global__ __launch_bounds__(64 * kBlockWaves) void k_lpa_block(const int64_t* __restrict__ rp,
                                                               const int32_t* __restrict__ al,
                                                               int32_t* __restrict__ Ln, int64_t h0,
                                                               int64_t h1,
                                                               const int32_t* __restrict__ flist,
                                                               const int32_t* __restrict__ fcnt0,
                                                               const int32_t* __restrict__ fr_all, int pmax,
                                                               const int32_t* __restrict__ gsel) {
  static_assert((1 << kLg) >= 2 * kBlockWaves * kSegArcs, "table load <= 1/2");
  constexpr int kSlots = 1 << kLg;
  constexpr int kT = 64 * kBlockWaves;
  constexpr int kGB = 256;   // giant-label histogram buckets of a block row
  static_assert(kT >= kGB, "one bucket per thread");
  __shared__ u64 tab[kSlots];
  __shared__ u64 redw[kBlockWaves];
  __shared__ u32 ghist[kGB];
  __shared__ u32 gcnt[2], gmax[2];   // by row parity (two barriers per decided row)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 lt = (1ull << lane) - 1ull;
  const bool all = *fr_all != 0;
  const int64_t n = all ? h1 - h0 : (int64_t)*fcnt0;
  if ((int64_t)blockIdx.x >= n) return;  // uniform
  for (int i = threadIdx.x; i < kSlots; i += kT) tab[i] = 0ull;
  if (threadIdx.x < kGB) ghist[threadIdx.x] = 0u;
  if (threadIdx.x < 2) gcnt[threadIdx.x] = gmax[threadIdx.x] = 0u;
  // gsel (label-dense supersteps): the giant-label word (k_giant_pick; giant_count)
  const bool giant = gsel != nullptr && gsel[1] != 0;
  const u32 G = giant ? (u32)gsel[0] : 0u;
  __syncthreads();
  int rpar = 0;  // parity of the rows this block has tallied
  for (int64_t q = blockIdx.x; q < n; q += gridDim.x) {
    const int64_t h = all ? h0 + q : (int64_t)flist[q];
    if (h < h0 || h >= h1) continue;  // uniform over the block
    const int64_t b = rp[h], e = rp[h + 1];
    const int d = (int)(e - b);
    int lg = ceil_log2(2u * (u32)d);
    lg = lg < 6 ? 6 : lg;
    const int64_t c0 = b + (int64_t)w * kSegArcs;
    u32 lab[kChunks];
    int nch = 0;
    if (c0 < e) {
      load_labels<kChunks>(lab, al, c0, e, lane);
      nch = (int)min<int64_t>(kChunks, (e - c0 + 63) >> 6);
    }
    if (giant) {
      // G's votes (block total) and the other votes' bucket histogram; decided when
      // G's count exceeds every bucket (uniform: read after the barrier)
      // (the counters of parity rpar: the other parity's, read by the previous row
      // before this row's first barrier, are reset before its second)
      if (c0 < e) {
        const u32 cg = wave_sum_u32(giant_count<kChunks>(lab, nch, G, ghist, 8));
        if (lane == 0 && cg) atomicAdd(&gcnt[rpar], cg);
      }
      __syncthreads();
      if (threadIdx.x < kGB) {
        const u32 m = ghist[threadIdx.x];
        ghist[threadIdx.x] = 0u;
        if (m) atomicMax(&gmax[rpar], m);
      }
      if (threadIdx.x == 0) gcnt[rpar ^ 1] = gmax[rpar ^ 1] = 0u;
      __syncthreads();
      const bool decided = gcnt[rpar] > gmax[rpar];
      rpar ^= 1;
      if (decided) {  // uniform
        if (threadIdx.x == 0) Ln[h] = (int32_t)G;
        continue;
      }
    }
    if (c0 < e) {
      Batch<kChunks> bt;
      peel_batch<kChunks>(bt, lab, nch, lane, pmax);
      int unused = 0;
      hash_batch<kChunks, false>(tab, nullptr, unused, 32 - lg, (1u << lg) - 1u, bt, lab, nch, lane, lt);
    }
    __syncthreads();
    u64 best = 0ull;
    for (int i = threadIdx.x; i < (1 << lg); i += kT) {
      const u64 t = tab[i];
      if (t) {
        best = umax64(best, t);
        tab[i] = 0ull;
      }
    }
    best = wave_max_u64(best);
    if (lane == 0) redw[w] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
      u64 m = redw[0];
#pragma unroll
      for (int k = 1; k < kBlockWaves; ++k) m = umax64(m, redw[k]);
      Ln[h] = (int32_t)(~(u32)m);
    }
  }
}

// ---------------------------------------------------------------------------
// bins g64 .. g8 (4 < deg <= 64): persistent waves over batches of RB = 512 / G
// consecutive rows (G lanes per row, 8 chunks of 64 lanes per batch).  Per batch
// a wave issues ONE row-offset load (lane r holds rp[r0 + r]) and then all 8
// label loads per lane at once; the next batch's labels and the batch after
// next's offsets stream in while the current batch is tallied (ballot peel
// within each G-lane group).  (A three-set unrolled ring, as in k_lpa_units,
// measured slower here: the per-batch tally is long enough to cover one batch.)
// ---------------------------------------------------------------------------
// label of the first active lane of this lane's G-lane group (act: the wave's
// active mask, uniform).  G >= 16: one readlane per group (scalar lane index),
// selected per lane -- VALU/SALU only; smaller groups use one ds_bpermute.
template <int G>
__device__ __forceinline__ u32 group_lead(u32 lb, u64 act, int lane, int lead) {
  if constexpr (G >= 16) {
    constexpr u64 gm = G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull);
    u32 x = 0u;
#pragma unroll
    for (int k = 0; k < 64 / G; ++k) {
      const u64 mk = (act >> (k * G)) & gm;
      const int l = k * G + (mk ? (__ffsll((unsigned long long)mk) - 1) : 0);
      const u32 xk = (u32)__builtin_amdgcn_readlane((int)lb, l);
      if (lane / G == k) x = xk;
    }
    return x;
  } else {
    return (u32)__shfl((int)lb, lead, 64);
  }
}

template <int G>
__device__ __forceinline__ void rows_rp(const int64_t* __restrict__ rp, int64_t r0, int64_t vend,
                                        int lane, int64_t& rpl, int64_t& rpe) {
  constexpr int RB = 512 / G;
  const int64_t i = r0 + lane;
  rpl = (lane < RB && i <= vend) ? rp[i] : 0;
  rpe = rp[min(r0 + RB, vend)];
}

template <int G, bool kG = false>
__device__ __forceinline__ void rows_labels(u32 (&lab)[kChunks], const int32_t* __restrict__ al,
                                            int64_t r0, int64_t vend, int64_t rpl, int64_t rpe,
                                            int lane, const int32_t* __restrict__ Lg = nullptr) {
  constexpr int RB = 512 / G;
#pragma unroll
  for (int c = 0; c < kChunks; ++c) {
    const int rl = c * (64 / G) + lane / G;
    const int j = lane & (G - 1);
    // both shuffles run on every lane (a bpermute from a lane that is masked
    // off returns garbage), then the batch end is selected
    const int64_t b = __shfl(rpl, rl, 64);
    const int64_t en = __shfl(rpl, rl + 1 < 64 ? rl + 1 : 63, 64);
    const int64_t e = rl + 1 < RB ? en : rpe;
    lab[c] = (r0 + rl < vend && j < e - b) ? arc_vote<kG>(al, Lg, b + j) : kNone;
  }
}

// branch-free forms for k_lpa_rows' ring: every lane loads, at an address clamped into
// the graph (rp[<= vend], al[< arcs]); values past the bin or the row are masked after
// the load
constexpr int kRowsRing = 3;
template <int G>
__device__ __forceinline__ void rows_rp_nb(const int64_t* __restrict__ rp, int64_t r0, int64_t vend,
                                           int lane, int64_t& rpl, int64_t& rpe) {
  constexpr int RB = 512 / G;
  const int64_t i = r0 + lane;
  rpl = rp[i < vend ? i : vend];
  rpe = rp[r0 + RB < vend ? r0 + RB : vend];
}

// (vbits bit c: chunk c's label is a vote -- one register per set, applied when the set
// is tallied, so nothing 64-bit stays live while the loads are in flight)
template <int G, bool kG = false>
__device__ __forceinline__ void rows_labels_nb(u32 (&lab)[kChunks], u32& vbits, const int32_t* __restrict__ al,
                                               int64_t r0, int64_t vend, int64_t rpl, int64_t rpe,
                                               int lane, const int32_t* __restrict__ Lg = nullptr) {
  constexpr int RB = 512 / G;
  vbits = 0u;
#pragma unroll
  for (int c = 0; c < kChunks; ++c) {
    const int rl = c * (64 / G) + lane / G;
    const int j = lane & (G - 1);
    const int64_t b = __shfl(rpl, rl, 64);
    const int64_t en = __shfl(rpl, rl + 1 < 64 ? rl + 1 : 63, 64);
    const int64_t e = rl + 1 < RB ? en : rpe;
    int64_t a = b + j < e ? b + j : e - 1;
    a = a > 0 ? a : 0;
    lab[c] = arc_vote<kG>(al, Lg, a);
    vbits |= (r0 + rl < vend && j < e - b) ? (1u << c) : 0u;
  }
  asm volatile("" : "+v"(vbits));  // computed here: not sunk to the tally (64-bit bounds would stay live)
}

constexpr int kRowsGB = 16;  // giant-label histogram buckets per row (group) of k_lpa_rows

// (htab_all / ghist_all: the block's LDS, 4 waves x kRowsHashSlots table slots /
// 64 / G * kRowsGB histogram buckets)
template <int G, bool kG = false>
__device__ __forceinline__ void rows_bin(int64_t bid, int64_t nblk, u64* htab_all, u32* ghist_all,
                                         const int64_t* __restrict__ rp, const int32_t* __restrict__ al,
                                         int32_t* __restrict__ Ln, int64_t vbeg, int64_t vend,
                                         const int32_t* __restrict__ flist, const int32_t* __restrict__ fcnt_b,
                                         const int32_t* __restrict__ fr_all, int sort_after,
                                         const int32_t* __restrict__ gsel, const int32_t* __restrict__ Lg) {
  static_assert(G >= 8 && G <= 64 && (G & (G - 1)) == 0, "lane width");
  constexpr int RB = 512 / G;  // rows per batch
  constexpr int kGB = kRowsGB;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u64* htab = htab_all + w * kRowsHashSlots;
#pragma unroll
  for (int k = 0; k < kRowsHashSlots / 64; ++k) htab[k * 64 + lane] = 0ull;
  if (!*fr_all) {
    // frontier: the listed dirty rows, G lanes each (rows are not consecutive, so
    // no batched offsets); every lane of a wave runs every trip (ballot peel)
    const BinRows br = bin_rows(vbeg, vend, flist, fcnt_b, fr_all);
    const int64_t per = 64 / G, nw = nblk * 4;
    for (int64_t i0 = (bid * 4 + w) * per; i0 < br.n; i0 += nw * per) {
      const int64_t i = i0 + lane / G;
      const bool live = i < br.n;
      group_row<G, kG>(rp, al, Ln, live ? br.row(i) : 0, live, lane, htab, Lg);
    }
    return;
  }
  const int64_t nb = (vend - vbeg + RB - 1) / RB;
  const int64_t stride = nblk * 4;
  int64_t bi = bid * 4 + w;
  if (bi >= nb) return;  // no block-level barriers in this body
  // gsel (superstep 2, rows of > 8 arcs): a chunk whose every row is decided for the
  // giant label (its exact count above each of the row's kGB label-hash buckets of
  // other votes, as giant_decide) skips the peel / hash
  const bool giant = G >= 16 && gsel != nullptr && gsel[1] != 0;
  const u32 Gl = giant ? (u32)gsel[0] : 0u;
  u32* hg = ghist_all + w * (64 / G * kGB) + (lane / G) * kGB;
  const int gj = lane & (G - 1);   // G >= kGB when giant: lane gj < kGB owns bucket gj
  if (gj < kGB) hg[gj] = 0u;
  if constexpr (G == 64 && !kG) {
    // g64 (33-64 arcs, eight rows per batch): the two-batch form -- the ring's extra
    // label set cost C2 (SBM, nearly every row here) 61.5 -> 57.6 GTEPS (same box)
    int64_t rpl0, rpe0, rpl1 = 0, rpe1 = 0;
    rows_rp<G>(rp, vbeg + bi * RB, vend, lane, rpl0, rpe0);
    if (bi + stride < nb) rows_rp<G>(rp, vbeg + (bi + stride) * RB, vend, lane, rpl1, rpe1);
    u32 lab[kChunks];
    rows_labels<G, kG>(lab, al, vbeg + bi * RB, vend, rpl0, rpe0, lane, Lg);
    const int gbase = lane & ~(G - 1);
    const u64 gm = G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull);
    while (true) {
      const int64_t bn = bi + stride;
      int64_t rpl2 = 0, rpe2 = 0;
      if (bn + stride < nb) rows_rp<G>(rp, vbeg + (bn + stride) * RB, vend, lane, rpl2, rpe2);
      u32 labn[kChunks];
      if (bn < nb) {
        rows_labels<G, kG>(labn, al, vbeg + bn * RB, vend, rpl1, rpe1, lane, Lg);
      } else {
  #pragma unroll
        for (int c = 0; c < kChunks; ++c) labn[c] = kNone;
      }
      const int64_t r0 = vbeg + bi * RB;
  #pragma unroll
      for (int c = 0; c < kChunks; ++c) {
        const u32 lb = lab[c];
        u64 act = __ballot(lb != kNone);
        u64 best = 0ull;
        if constexpr (G >= kGB) if (giant) {
          const u64 gb = __ballot(lb == Gl);
          const u32 cg = (u32)__popcll((gb >> gbase) & gm);
          if (lb != Gl && lb != kNone) atomicAdd(&hg[hash_slot(lb, 28)], 1u);
          __builtin_amdgcn_wave_barrier();  // no reordering across (LDS ops of a wave complete in order)
          u32 mx = 0u;
          if (gj < kGB) {
            mx = hg[gj];
            hg[gj] = 0u;
          }
          for (int off = G >> 1; off > 0; off >>= 1) mx = max(mx, (u32)lane::lane_xor(mx, off, lane));
          const bool dec = cg > mx;
          if (__ballot(lb != kNone && !dec) == 0ull) {  // uniform: every row decided
            best = dec ? tally(cg, Gl) : 0ull;
            act = 0ull;
          }
        }
        for (int round = 0; act; ++round) {
          // uniform: a label-dense chunk after sort_after rounds
          if (round == sort_after) {
            best = group_mode_hash<G>(lb, lane, htab);
            break;
          }
          const u64 my = (act >> gbase) & gm;
          const int lead = gbase + (my ? (__ffsll((unsigned long long)my) - 1) : 0);
          const u32 x = group_lead<G>(lb, act, lane, lead);
          const u64 mm = __ballot(((act >> lane) & 1ull) && lb == x);
          const u32 cn = (u32)__popcll((mm >> gbase) & gm);
          if (my) best = umax64(best, tally(cn, x));
          act &= ~mm;
          act &= ~decided_groups<G>(act, my, best, gbase, gm);
        }
        const int64_t row = r0 + c * (64 / G) + lane / G;
        if ((lane & (G - 1)) == 0 && row < vend && best) Ln[row] = (int32_t)(~(u32)best);
      }
      if (bn >= nb) break;
      bi = bn;
      rpl0 = rpl1;
      rpe0 = rpe1;
      rpl1 = rpl2;
      rpe1 = rpe2;
  #pragma unroll
      for (int c = 0; c < kChunks; ++c) lab[c] = labn[c];
    }

    return;
  } else {
  const int gbase = lane & ~(G - 1);
  const u64 gm = G == 64 ? ~0ull : ((1ull << (G & 63)) - 1ull);
  auto tally_batch = [&](const u32 (&lab)[kChunks], u32 vbits, int64_t r0) {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
      const u32 lb = (vbits >> c) & 1u ? lab[c] : kNone;
      u64 act = __ballot(lb != kNone);
      u64 best = 0ull;
      if constexpr (G >= kGB) if (giant) {
        const u64 gb = __ballot(lb == Gl);
        const u32 cg = (u32)__popcll((gb >> gbase) & gm);
        if (lb != Gl && lb != kNone) atomicAdd(&hg[hash_slot(lb, 28)], 1u);
        __builtin_amdgcn_wave_barrier();  // no reordering across (LDS ops of a wave complete in order)
        u32 mx = 0u;
        if (gj < kGB) {
          mx = hg[gj];
          hg[gj] = 0u;
        }
        for (int off = G >> 1; off > 0; off >>= 1) mx = max(mx, (u32)lane::lane_xor(mx, off, lane));
        const bool dec = cg > mx;
        if (__ballot(lb != kNone && !dec) == 0ull) {  // uniform: every row decided
          best = dec ? tally(cg, Gl) : 0ull;
          act = 0ull;
        }
      }
      for (int round = 0; act; ++round) {
        // uniform: a label-dense chunk after sort_after rounds
        if (round == sort_after) {
          best = group_mode_hash<G>(lb, lane, htab);
          break;
        }
        const u64 my = (act >> gbase) & gm;
        const int lead = gbase + (my ? (__ffsll((unsigned long long)my) - 1) : 0);
        const u32 x = group_lead<G>(lb, act, lane, lead);
        const u64 mm = __ballot(((act >> lane) & 1ull) && lb == x);
        const u32 cn = (u32)__popcll((mm >> gbase) & gm);
        if (my) best = umax64(best, tally(cn, x));
        act &= ~mm;
        act &= ~decided_groups<G>(act, my, best, gbase, gm);
      }
      const int64_t row = r0 + c * (64 / G) + lane / G;
      if ((lane & (G - 1)) == 0 && row < vend && best) Ln[row] = (int32_t)(~(u32)best);
    }
  };
  if constexpr (kG) {
    // gather mode (al = col): a vote is a column load and a dependent label gather, so
    // the ring runs them a step apart -- at the tally of batch i the gathers of batch
    // i + 1 (its columns arrived a step earlier) and the columns of batch i + 2 are in
    // flight, and each wait is for loads issued a full step before
    constexpr int D = kRowsRing;
    static_assert(D == 3, "slot arithmetic below");
    int64_t rpl[D], rpe[D];
    u32 cc[D][kChunks], labg[D][kChunks], vb[D];
#pragma unroll
    for (int k = 0; k < D; ++k) rows_rp_nb<G>(rp, vbeg + (bi + k * stride) * RB, vend, lane, rpl[k], rpe[k]);
    rows_labels_nb<G, false>(cc[0], vb[0], al, vbeg + bi * RB, vend, rpl[0], rpe[0], lane);
#pragma unroll
    for (int c = 0; c < kChunks; ++c) labg[0][c] = LPA_GV(cc[0][c]);
    rows_labels_nb<G, false>(cc[1], vb[1], al, vbeg + (bi + stride) * RB, vend, rpl[1], rpe[1], lane);
    while (true) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const int k1 = (k + 1) % D, k2 = (k + 2) % D;
        __builtin_amdgcn_sched_barrier(0);
        rows_rp_nb<G>(rp, vbeg + (bi + D * stride) * RB, vend, lane, rpl[k], rpe[k]);
#pragma unroll
        for (int c = 0; c < kChunks; ++c) labg[k1][c] = LPA_GV(cc[k1][c]);
        rows_labels_nb<G, false>(cc[k2], vb[k2], al, vbeg + (bi + 2 * stride) * RB, vend, rpl[k2], rpe[k2], lane);
        __builtin_amdgcn_sched_barrier(0);
        tally_batch(labg[k], vb[k], vbeg + bi * RB);
        bi += stride;
        if (bi >= nb) return;
      }
    }
  } else {
  // Ring of kRowsRing batches (batch j in slot j % kRowsRing): the offsets of batch
  // i + kRowsRing are issued before the labels of batch i + kRowsRing - 1, so the wait
  // for those labels' offsets (issued one batch earlier, ahead of the previous batch's
  // labels) leaves the previous batch's labels in flight -- two label batches load
  // while one is tallied.  Loads branch-free (rows_rp_nb / rows_labels_nb); scheduling
  // barriers keep each batch's loads from being hoisted into the tally before them.
  constexpr int D = kRowsRing;
  int64_t rpl[D], rpe[D];
  u32 lab[D][kChunks], vb[D];
#pragma unroll
  for (int k = 0; k < D; ++k) rows_rp_nb<G>(rp, vbeg + (bi + k * stride) * RB, vend, lane, rpl[k], rpe[k]);
#pragma unroll
  for (int k = 0; k < D - 1; ++k) rows_labels_nb<G, kG>(lab[k], vb[k], al, vbeg + (bi + k * stride) * RB, vend, rpl[k], rpe[k], lane, Lg);
  while (true) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      __builtin_amdgcn_sched_barrier(0);
      rows_rp_nb<G>(rp, vbeg + (bi + D * stride) * RB, vend, lane, rpl[k], rpe[k]);
      const int kl = (k + D - 1) % D;
      rows_labels_nb<G, kG>(lab[kl], vb[kl], al, vbeg + (bi + (D - 1) * stride) * RB, vend, rpl[kl], rpe[kl], lane, Lg);
      __builtin_amdgcn_sched_barrier(0);
      tally_batch(lab[k], vb[k], vbeg + bi * RB);
      bi += stride;
      if (bi >= nb) return;
    }
  }
  }
  }
}

template <int G, bool kG = false>
__global__ __launch_bounds__(256) void k_lpa_rows(const int64_t* __restrict__ rp,
                                                  const int32_t* __restrict__ al,
                                                  int32_t* __restrict__ Ln, int64_t vbeg,
                                                  int64_t vend, const int32_t* __restrict__ flist,
                                                  const int32_t* __restrict__ fcnt_b,
                                                  const int32_t* __restrict__ fr_all, int sort_after,
                                                  const int32_t* __restrict__ gsel,
                                                  const int32_t* __restrict__ Lg) {
  __shared__ u32 ghist_all[4 * (64 / G) * kRowsGB];
  __shared__ u64 htab_all[4 * kRowsHashSlots];
  rows_bin<G, kG>(blockIdx.x, gridDim.x, htab_all, ghist_all, rp, al, Ln, vbeg, vend, flist, fcnt_b, fr_all,
                  sort_after, gsel, Lg);
}

// ---------------------------------------------------------------------------
// The converged supersteps' bins in one launch per stream (round 6): blocks
// [off[k], off[k + 1]) run sub-launch k's bin body with that share as their grid --
// the same blocks, lists and ranges as the kernels of their own, minus the launch
// and drain of every kernel boundary in the stream's chain (a converged superstep's
// bins tally ~0.2 % of the rows: each of their launches was mostly fixed cost).
// kWide: 1 = the wave bins w16 / w8 / w4 (aux0), 0 = w2 and the row / group bins
// (aux1).
// ---------------------------------------------------------------------------
#ifndef LPA_FUSED_WAVES
#define LPA_FUSED_WAVES 5  // waves per SIMD the register budget is set for
#endif
constexpr int kFusedMax = 8;
struct FusedBins {
  int n;
  int bin[kFusedMax];
  int32_t off[kFusedMax + 1];
  int64_t vb[kFusedMax], ve[kFusedMax];
};

template <int kWide>
__global__ __launch_bounds__(256, LPA_FUSED_WAVES) void k_bins_fused(const FusedBins fb, const int64_t* __restrict__ rp,
                                                    const int32_t* __restrict__ al, int32_t* __restrict__ Ln,
                                                    const int32_t* __restrict__ flist,
                                                    const int32_t* __restrict__ fcnt,
                                                    const int32_t* __restrict__ fr_all, int pmax, int sort_after) {
  constexpr int kNC = kWide ? 16 : 2;  // the widest wave bin of the launch
  __shared__ u64 tab[4 * (2 * 64 * kNC > kRowsHashSlots ? 2 * 64 * kNC : kRowsHashSlots)];
  __shared__ uint16_t lst[4 * 64 * kNC];
  __shared__ u32 gh[kWide ? 1 : 4 * (64 / 8) * kRowsGB];
  int k = 0;
  while (k + 1 < fb.n && (int32_t)blockIdx.x >= fb.off[k + 1]) ++k;  // uniform
  const int64_t bid = (int64_t)blockIdx.x - fb.off[k], nblk = fb.off[k + 1] - fb.off[k];
  const int b = fb.bin[k];
  const int64_t v0 = fb.vb[k], v1 = fb.ve[k];
  const int32_t* fc = fcnt + b;
  if constexpr (kWide) {
    if (b == BIN_W16) wave_bin<16>(bid, nblk, tab, lst, rp, al, Ln, v0, v1, flist, fc, fr_all, pmax, nullptr, nullptr);
    else if (b == BIN_W8) wave_bin<8>(bid, nblk, tab, lst, rp, al, Ln, v0, v1, flist, fc, fr_all, pmax, nullptr, nullptr);
    else wave_bin<4>(bid, nblk, tab, lst, rp, al, Ln, v0, v1, flist, fc, fr_all, pmax, nullptr, nullptr);
  } else {
    switch (b) {
      case BIN_W2: wave_bin<2>(bid, nblk, tab, lst, rp, al, Ln, v0, v1, flist, fc, fr_all, pmax, nullptr, nullptr); break;
      case BIN_G64: rows_bin<64>(bid, nblk, tab, gh, rp, al, Ln, v0, v1, flist, fc, fr_all, sort_after, nullptr, nullptr); break;
      case BIN_G32: rows_bin<32>(bid, nblk, tab, gh, rp, al, Ln, v0, v1, flist, fc, fr_all, sort_after, nullptr, nullptr); break;
      case BIN_G16: rows_bin<16>(bid, nblk, tab, gh, rp, al, Ln, v0, v1, flist, fc, fr_all, sort_after, nullptr, nullptr); break;
      case BIN_G8: rows_bin<8>(bid, nblk, tab, gh, rp, al, Ln, v0, v1, flist, fc, fr_all, sort_after, nullptr, nullptr); break;
      case BIN_G4: group_bin<4>(bid, nblk, rp, al, Ln, v0, v1, flist, fc, fr_all, nullptr); break;
      case BIN_G2: group_bin<2>(bid, nblk, rp, al, Ln, v0, v1, flist, fc, fr_all, nullptr); break;
      default: group_bin<1>(bid, nblk, rp, al, Ln, v0, v1, flist, fc, fr_all, nullptr); break;
    }
  }
}

// ---------------------------------------------------------------------------
// bin seg: deg > kWaveMaxDeg.  The row is cut into 512-arc units; one wave per
// unit (grid-stride over units, unit descriptors prefetched two units ahead and
// labels one unit ahead, no block barriers, no returning atomics -- those would
// make the wave wait for its prefetched loads).  The wave tallies its unit in
// registers (peel) + its own LDS table and writes the unit's tally words to the
// unit's own staging slots stage[begin ...) plus their count ucnt[unit]; the hub
// combine (lpa_hub.hip) merges a row's units.  Unit: begin arc, row,
// len | (unit index within the row << 10).
// ---------------------------------------------------------------------------
// work item i of the units kernel -> unit id (frontier: the listed dirty units; a
// unit not listed keeps the words it staged when last tallied -- its al[] entries
// are unchanged since, so they are still exact)
struct UnitIds {
  int64_t n;
  int64_t lim;          // units >= lim are not this launch's (block-tier rows in block mode)
  const int32_t* list;  // nullptr: every unit
  __device__ __forceinline__ int64_t id(int64_t i) const { return list ? (int64_t)list[i] : i; }
};

__device__ __forceinline__ Segment load_unit(const Segment* __restrict__ units, const UnitIds& ui, int64_t i) {
  Segment d;
  d.begin = 0;
  d.len = 0;
  d.v = 0;
  if (i < ui.n) {
    const int64_t id = ui.id(i);
    if (id < ui.lim) d = units[id];  // a listed unit of a block-tier row: len 0, skipped
  }
  return d;
}

// unconditional loads (the address is clamped into the unit; lanes past the unit's
// end are masked at use time), so the compiler can count vmcnt exactly
__device__ __forceinline__ void unit_load(u32 (&raw)[kChunks], const int32_t* __restrict__ al,
                                          const Segment& d, int lane) {
  const int len = d.len & 1023;
  if (__builtin_amdgcn_readfirstlane(len) == 0) {  // frontier-clean unit: no loads
#pragma unroll
    for (int c = 0; c < kChunks; ++c) raw[c] = kNone;
    return;
  }
  const int last = len > 0 ? len - 1 : 0;
#pragma unroll
  for (int c = 0; c < kChunks; ++c) {
    const int off = c * 64 + lane;
    raw[c] = ld_stream(al + d.begin + (off < last ? off : last));
  }
}

// 64 work items' unit descriptors in one load per lane (lane k: item i0 + k * stride;
// empty past the list or for a block-tier unit), read back by readlane
struct UnitBatch {
  int64_t begin;
  int32_t len, id;
};
__device__ __forceinline__ UnitBatch unit_batch(const Segment* __restrict__ units, const UnitIds& ui, int64_t i0,
                                                int64_t stride, int lane) {
  UnitBatch b;
  b.begin = 0;
  b.len = 0;
  b.id = 0;
  const int64_t i = i0 + (int64_t)lane * stride;
  if (i < ui.n) {
    const int64_t id = ui.id(i);
    b.id = (int32_t)id;
    if (id < ui.lim) {
      const Segment d = units[id];
      b.begin = d.begin;
      b.len = d.len;
    }
  }
  return b;
}
// item q of the two batches (uniform; a branch so the cur side never waits for nxt)
__device__ __forceinline__ Segment unit_at(const UnitBatch& cur, const UnitBatch& nxt, int q) {
  Segment d;
  d.v = 0;
  if (q < 64) {
    d.begin = readlane_i64(cur.begin, q);
    d.len = __builtin_amdgcn_readlane(cur.len, q);
  } else {
    d.begin = readlane_i64(nxt.begin, q - 64);
    d.len = __builtin_amdgcn_readlane(nxt.len, q - 64);
  }
  return d;
}
constexpr int kUnitsRing = 4;

// branch-free unit_load (k_lpa_units' ring): an empty unit loads al[begin] (begin 0)
__device__ __forceinline__ void unit_load_nb(u32 (&raw)[kChunks], const int32_t* __restrict__ al,
                                             const Segment& d, int lane) {
  const int len = d.len & 1023;
  const int last = len > 0 ? len - 1 : 0;
#pragma unroll
  for (int c = 0; c < kChunks; ++c) {
    const int off = c * 64 + lane;
    raw[c] = ld_stream(al + d.begin + (off < last ? off : last));
  }
}

// tally one unit whose labels are in `raw` (loaded earlier)
__device__ __forceinline__ void unit_tally(const u32 (&raw)[kChunks], const Segment& d, int64_t u,
                                           u64* __restrict__ stage, int32_t* __restrict__ ucnt,
                                           u64* tab, uint16_t* lst, int lane, u64 lt, int pmax) {
  const int len = d.len & 1023;
  if (len == 0) return;
  u32 lab[kChunks];
#pragma unroll
  for (int c = 0; c < kChunks; ++c) lab[c] = c * 64 + lane < len ? raw[c] : kNone;
  const int nch = (len + 63) >> 6;
  // staging slots of this unit: stage[begin .. begin + words) (words <= len)
  u64* st = stage + d.begin;
  Batch<kChunks> bt;
  peel_batch<kChunks>(bt, lab, nch, lane, pmax);
  if (!bt.any) {
    // every vote is in a peel group: the unit's words are the peel groups
    if (lane < bt.npeel) st[lane] = bt.pword;
    if (lane == 0) ucnt[u] = bt.npeel;
  } else {
    int lg = ceil_log2(2u * (u32)len);
    lg = lg < 6 ? 6 : lg;
    int cnt = 0;
    hash_batch<kChunks>(tab, lst, cnt, 32 - lg, (1u << lg) - 1u, bt, lab, nch, lane, lt);
    for (int i = lane; i < cnt; i += 64) {
      const int slt = lst[i];
      st[i] = tab[slt];
      tab[slt] = 0ull;
    }
    if (lane == 0) ucnt[u] = cnt;
  }
}

__global__ __launch_bounds__(256) void k_lpa_units(const int32_t* __restrict__ al,
                                                   const Segment* __restrict__ units, int64_t nunits,
                                                   u64* __restrict__ stage,
                                                   int32_t* __restrict__ ucnt,
                                                   const int32_t* __restrict__ ulist,
                                                   const int32_t* __restrict__ fcnt_u,
                                                   const int32_t* __restrict__ fr_all, int pmax) {
  constexpr int kCap = 2 * 64 * kChunks;
  __shared__ u64 tab_all[4][kCap];
  __shared__ uint16_t lst_all[4][64 * kChunks];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u64* tab = tab_all[w];
  uint16_t* lst = lst_all[w];
  const u64 lt = (1ull << lane) - 1ull;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t u = (int64_t)blockIdx.x * 4 + w;
  if (u >= nunits) return;  // no block-level barriers in this kernel
  UnitIds ui;
  ui.n = *fr_all ? nunits : (int64_t)*fcnt_u;
  ui.lim = nunits;
  ui.list = *fr_all ? nullptr : ulist;
  if (u >= ui.n) return;
  // the wave's table is cleared only by waves with work (a frontier superstep lists
  // few units: most of the grid leaves at once)
  for (int i = lane; i < kCap; i += 64) tab[i] = 0ull;
  // unit descriptors by 64-unit batches (lane k: work item ib + k * stride), the next
  // batch loaded half a batch ahead; kUnitsRing label sets in an unrolled ring (labels
  // kUnitsRing - 1 units ahead), branch-free loads: no label load waits on a
  // descriptor load issued after other label loads (vmcnt counts in order)
  constexpr int D = kUnitsRing;
  int64_t ib = u;
  UnitBatch cur = unit_batch(units, ui, ib, stride, lane), nxt;
  nxt.begin = 0;
  nxt.len = 0;
  nxt.id = 0;
  int p = 0;
  u32 rl[D][kChunks];
#pragma unroll
  for (int k = 0; k < D - 1; ++k) unit_load_nb(rl[k], al, unit_at(cur, nxt, k), lane);
  while (true) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      unit_load_nb(rl[(k + D - 1) % D], al, unit_at(cur, nxt, p + D - 1), lane);
      const Segment d = unit_at(cur, nxt, p);
      const int64_t id = (int64_t)__builtin_amdgcn_readlane(cur.id, p);
      unit_tally(rl[k], d, id, stage, ucnt, tab, lst, lane, lt, pmax);
      if (ib + (int64_t)(p + 1) * stride >= ui.n) return;
      ++p;
      if (p == 32) nxt = unit_batch(units, ui, ib + 64 * stride, stride, lane);
      if (p == 64) {
        p = 0;
        ib += 64 * stride;
        cur = nxt;
      }
    }
  }
}

// Superstep 2, the unit-tallied hub rows (deg > kBlockMaxDeg2): each unit only counts
// the giant label's votes exactly (ugc[u]) and bounds every other label's count in the
// unit by its fullest label-hash bucket (umx[u]; giant_count, 64 buckets).  A label's
// row count is at most the sum of the units' bounds, so k_hub_decide settles a row
// whose G votes exceed that sum without staging or merging a single word; only the
// units of the rows it cannot settle are then tallied exactly (k_lpa_units, list mode).
// Block 0 also zeroes the undecided-unit list count (*ndec) for k_hub_decide.
// (k_lpa_units_code2 below: the same from the 2-bit giant codes, when the refresh took
// them -- gsel[5]; this form returns at once then.)
template <typename T>
__device__ __forceinline__ void unit_load_nb_t(u32 (&raw)[kChunks], const T* __restrict__ al, const Segment& d,
                                               int lane) {
  const int len = d.len & 1023;
  const int last = len > 0 ? len - 1 : 0;
#pragma unroll
  for (int c = 0; c < kChunks; ++c) {
    const int off = c * 64 + lane;
    if constexpr (sizeof(T) == 4) raw[c] = ld_stream(reinterpret_cast<const int32_t*>(al) + d.begin + (off < last ? off : last));
    else raw[c] = (u32)al[d.begin + (off < last ? off : last)];
  }
}
template <typename T>
__global__ __launch_bounds__(256) void k_lpa_units_giant(const T* __restrict__ al,
                                                         const Segment* __restrict__ units, int64_t nunits,
                                                         const int32_t* __restrict__ gsel,
                                                         uint32_t* __restrict__ ugc, uint32_t* __restrict__ umx,
                                                         int32_t* __restrict__ ndec) {
  __shared__ u32 hist_all[4][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) ndec[0] = ndec[2] = 0;  // unit list, block-row list
  if (gsel[5] != 0) return;  // k_lpa_units_code2's turn (uniform)
  if (gsel[1] == 0) return;  // no giant label worth trying: k_hub_decide lists every row
  u32* hist = hist_all[w];
  hist[lane] = 0u;
  const u32 G = (u32)gsel[0];
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t u = (int64_t)blockIdx.x * 4 + w;
  if (u >= nunits) return;  // no block-level barriers in this kernel
  UnitIds ui;
  ui.n = nunits;
  ui.lim = nunits;
  ui.list = nullptr;
  auto one = [&](const u32 (&raw)[kChunks], const Segment& d, int64_t id) {
    const int len = d.len & 1023;
    u32 lab[kChunks];
#pragma unroll
    for (int c = 0; c < kChunks; ++c) lab[c] = c * 64 + lane < len ? raw[c] : kNone;
    const u32 cg = wave_sum_u32(giant_count<kChunks>(lab, kChunks, G, hist, kGiantLg));
    __builtin_amdgcn_wave_barrier();  // no reordering across (LDS ops of a wave complete in order)
    const u32 b = hist[lane];
    hist[lane] = 0u;
    const u32 hm = wave_max_u32(b);
    if (lane == 0) {
      ugc[id] = cg;
      umx[id] = hm;
    }
  };
  // descriptor batches and a label ring as k_lpa_units
  constexpr int D = kUnitsRing;
  int64_t ib = u;
  UnitBatch cur = unit_batch(units, ui, ib, stride, lane), nxt;
  nxt.begin = 0;
  nxt.len = 0;
  nxt.id = 0;
  int p = 0;
  u32 rl[D][kChunks];
#pragma unroll
  for (int k = 0; k < D - 1; ++k) unit_load_nb_t<T>(rl[k], al, unit_at(cur, nxt, k), lane);
  while (true) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      unit_load_nb_t<T>(rl[(k + D - 1) % D], al, unit_at(cur, nxt, p + D - 1), lane);
      one(rl[k], unit_at(cur, nxt, p), ib + (int64_t)p * stride);
      if (ib + (int64_t)(p + 1) * stride >= nunits) return;
      ++p;
      if (p == 32) nxt = unit_batch(units, ui, ib + 64 * stride, stride, lane);
      if (p == 64) {
        p = 0;
        ib += 64 * stride;
        cur = nxt;
      }
    }
  }
}

// Superstep 4 (the settle schedule, main stream, ahead of k_lpa_units): every hub unit is
// re-tallied there so that the frontier supersteps find each unit's words staged.  A unit
// whose every arc votes G stages its one word (len, G) here without a tally: an arc votes G
// when its giant bit is set, or -- the bits kept through superstep 3's scatter are a lower
// bound, its joiners' bits clear -- when its al[] entry is G.  A lane per 64-arc chunk, eight
// units per wave; a lane reads its chunk's bit words and only the al[] entries of the clear
// bits, stopping at the first non-G vote.  The other units are listed (ulist, count
// gword[11], zeroed by k_giant_pick; a block's ids gathered in LDS first) for k_lpa_units in list mode (gword[10] = 0, its
// "fr_all").  Only with the kept bits (gword[2]: nothing writes them during superstep 4);
// otherwise gword[10] = 1 and k_lpa_units takes every unit.
constexpr int kPureIds = 8192;  // units per k_units_pure block (its LDS list)
__global__ __launch_bounds__(256) void k_units_pure(const int32_t* __restrict__ al,
                                                    const unsigned long long* __restrict__ abits, int64_t arcs,
                                                    const Segment* __restrict__ units, int64_t nunits,
                                                    int32_t* __restrict__ gword, u64* __restrict__ stage,
                                                    int32_t* __restrict__ ucnt, int32_t* __restrict__ ulist) {
  __shared__ int32_t lids[kPureIds];
  __shared__ int ln, lbase;
  const bool on = gword[2] != 0 && gword[1] != 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) gword[10] = on ? 0 : 1;
  if (!on) return;  // uniform
  const int32_t G = gword[0];
  const int lane = threadIdx.x & 63;
  const int c = lane & 7;
  const int64_t nwords = (arcs + 63) >> 6;
  // this block's units: a contiguous range of <= kPureIds (the host sizes the grid)
  const int64_t per = (nunits + gridDim.x - 1) / gridDim.x;
  const int64_t ub = (int64_t)blockIdx.x * per, ue = min(nunits, ub + per);
  if (threadIdx.x == 0) ln = 0;
  __syncthreads();
  for (int64_t u0 = ub + (threadIdx.x >> 6) * 8; u0 < ue; u0 += 32) {
    const int64_t u = u0 + (lane >> 3);
    bool ok = true;
    int64_t begin = 0;
    int len = 0;
    if (u < ue) {
      const Segment d = units[u];
      begin = d.begin;
      len = d.len & 1023;
      const int lo = c * 64, n = min(len - lo, 64);
      if (n > 0) {
        const int64_t a = begin + lo;
        const int64_t wq = a >> 6;
        const int off = (int)(a & 63);
        u64 bits = abits[wq] >> off;
        if (off && off + n > 64 && wq + 1 < nwords) bits |= abits[wq + 1] << (64 - off);
        u64 clear = ~bits & (n == 64 ? ~0ull : ((1ull << n) - 1ull));
        // the clear bits' al[] entries eight at a time, every load issued before the first
        // compare (unused slots re-read the chunk's first entry): a chunk of a hub row holds
        // several joiners, and one dependent load after another cost ~5x
        while (clear && ok) {
          int pos[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            pos[k] = clear ? __ffsll((unsigned long long)clear) - 1 : 0;
            clear &= clear - 1ull;
          }
          int32_t v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = al[a + pos[k]];
#pragma unroll
          for (int k = 0; k < 8; ++k) ok = ok && v[k] == G;  // (a padding slot's arc is the chunk's too)
        }
      }
    }
    const u64 bad = __ballot(!ok);
    const bool pure = ((bad >> (lane & ~7)) & 0xFFull) == 0ull;
    const bool head = u < ue && c == 0;
    if (head && pure) {
      stage[begin] = ((u64)(u32)len << 32) | (u64)(u32)(~(u32)G);
      ucnt[u] = 1;
    }
    if (head && !pure) lids[atomicAdd(&ln, 1)] = (int32_t)u;
  }
  // the block's impure units into the list: one global atomic per block (returning
  // atomics on one address serialise: a list atomic per wave cost C5 ~3 ms)
  __syncthreads();
  const int n = ln;
  if (n == 0) return;  // uniform
  if (threadIdx.x == 0) lbase = atomicAdd(&gword[11], n);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) ulist[lbase + i] = lids[i];
}

// ---------------------------------------------------------------------------
// refresh of the replicated neighbour labels al[]
// ---------------------------------------------------------------------------
// Scatter chunks: column u's al[] positions cpos[cptr[u] ..) are cut into chunks of
// kChunkPos, numbered statically at build time (chunks cch[u] .. cch[u+1] - 1,
// cowner[chunk] = u).  A changed column flags its chunks in the bytemap chflag[]
// (plain byte stores, no list to build); the scatter walks the bytemap.
__device__ __forceinline__ void flag_chunks(uint8_t* __restrict__ chflag, const int64_t* __restrict__ cch,
                                            int64_t u) {
  int64_t c = cch[u];
  const int64_t e = cch[u + 1];
  for (; c < e && (c & 15); ++c) chflag[c] = 1;  // hub columns: thousands of chunks,
  for (; c + 16 <= e; c += 16)                    // 16 flags per store
    *reinterpret_cast<uint4*>(chflag + c) = make_uint4(0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u);
  for (; c < e; ++c) chflag[c] = 1;
}

// changed vertices of the slot range [s0, s1): a column with one scatter chunk (the
// vast majority) is appended to chlist[] (LDS queue, one atomic per block), a longer
// one flags its chunks in chflag[]; the dirty arcs are counted (one atomic per wave);
// with Lsync != nullptr the new label is also copied into Lc (the next superstep's
// output vector: frontier, a row the next superstep skips already holds its label
// there; inside the concurrent tally the scatter does it).  int4 quads (vpad is a
// multiple of 64), kDiffQuads per block; lanes outside the range masked (the
// neighbouring slots may belong to a bin another stream is still computing).
//
// Frontier superstep (lists != nullptr and *fr_all == 0): only the rows listed for
// bins [b0, b1) were re-tallied (every other row provably kept its label, and its
// output slot already holds it), so the diff walks those lists -- grid-stride over
// their concatenation -- instead of the slot range.
struct BinBounds {
  int64_t b[LPA_NBINS + 1];
};
constexpr int kDiffQuads = 2048;
// counters[1] value that makes the refresh rebuild al[] (k_dense_decide)
constexpr unsigned long long kForcedRebuild = 1ull << 62;

// Label-dense supersteps (P = 1): the per-stream diffs only counted the changed slots.
// More than 1/10 of the slots changed: the refresh rebuilds al[] (counters[1] forced),
// so no position chunk is ever emitted; otherwise the full diff (mode 2) runs next.
// A superstep after a giant-code refresh (gword[5]) always rebuilds: its al[] entries were
// never written for the rows that superstep settled from codes.
__global__ void k_dense_decide(unsigned long long* __restrict__ counters, int64_t n_slots,
                               const int32_t* __restrict__ gword) {
  if (threadIdx.x == 0 && ((int64_t)counters[2] * 10 > n_slots || gword[5] != 0)) counters[1] = kForcedRebuild;
}
// fcnt[] slot set by the row settle of a giant superstep (k_settle_*): the bin kernels
// walk lists of the unsettled rows, but the diff scans every slot (settled rows may
// have changed label)
__global__ __launch_bounds__(256) void k_diff(const int4* __restrict__ Lc4,
                                              const int4* __restrict__ Ln4, int32_t* __restrict__ Lsync,
                                              int64_t s0, int64_t s1,
                                              const int64_t* __restrict__ cptr,
                                              const int64_t* __restrict__ cch,
                                              uint8_t* __restrict__ chflag,
                                              int32_t* __restrict__ chlist,
                                              unsigned long long* __restrict__ counters,
                                              BinBounds bb, int b0, int b1,
                                              const int32_t* __restrict__ flist,
                                              const int32_t* __restrict__ fcnt,
                                              const int32_t* __restrict__ fr_all, int mode) {
  // mode 1 (label-dense supersteps): only count the changed slots (counters[2]); mode 2:
  // the full diff unless k_dense_decide already chose the rebuild (counters[1] forced)
  if (mode == 2 && counters[1] >= kForcedRebuild) return;
  if (mode == 1) {
    unsigned long long c = 0;
    const int64_t q0 = s0 / 4 + (int64_t)blockIdx.x * kDiffQuads;
    const int64_t q1 = min((s1 + 3) / 4, q0 + kDiffQuads);
    for (int64_t q = q0 + threadIdx.x; q < q1; q += 256) {
      const int4 a = Lc4[q], b = Ln4[q];
      int chg = (a.x != b.x) | ((a.y != b.y) << 1) | ((a.z != b.z) << 2) | ((a.w != b.w) << 3);
      if (q * 4 < s0 || q * 4 + 4 > s1) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (q * 4 + k < s0 || q * 4 + k >= s1) chg &= ~(1 << k);
      }
      c += (unsigned long long)__popc(chg);
    }
    // (the counts summed per block first: one atomic per block on the counter, not one
    // per wave -- the same-address atomics of ~8 K waves queue at the counter's channel)
    __shared__ unsigned long long csum;
    if (threadIdx.x == 0) csum = 0ull;
    __syncthreads();
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&csum, c);
    __syncthreads();
    if (threadIdx.x == 0 && csum) atomicAdd(&counters[2], csum);
    return;
  }
  __shared__ int32_t q_col[kDiffQuads * 4];
  __shared__ int qn;
  __shared__ unsigned long long base_s, dsum;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
    qn = 0;
    dsum = 0ull;
  }
  __syncthreads();
  unsigned long long dirty = 0;
  auto emit = [&](int64_t u, int32_t nb) {
    if (Lsync) Lsync[u] = nb;
    dirty += (unsigned long long)(cptr[u + 1] - cptr[u]);
    const int64_t nch = cch[u + 1] - cch[u];
    if (nch == 1) q_col[atomicAdd(&qn, 1)] = (int32_t)u;
    else if (nch > 1) flag_chunks(chflag, cch, u);
  };
  if (flist != nullptr && *fr_all == 0 && fcnt[kFcntSettled] == 0) {
    // a list holds at most its bin's rows, so the grid (sized for the slot range)
    // gives each thread <= 32 entries, inside the block's queue
    int64_t total = 0;
    for (int b = b0; b < b1; ++b) total += fcnt[b];
    const int32_t* Lc = reinterpret_cast<const int32_t*>(Lc4);
    const int32_t* Ln = reinterpret_cast<const int32_t*>(Ln4);
    for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < total; v += (int64_t)gridDim.x * 256) {
      int64_t acc = 0;
      int b = b0;
      while (v >= acc + fcnt[b]) acc += fcnt[b++];
      const int64_t u = flist[bb.b[b] + (v - acc)];
      const int32_t nb = Ln[u];
      if (Lc[u] != nb) emit(u, nb);
    }
  } else {
    const int64_t q0 = s0 / 4 + (int64_t)blockIdx.x * kDiffQuads;
    const int64_t q1 = min((s1 + 3) / 4, q0 + kDiffQuads);
    for (int64_t q = q0 + threadIdx.x; q < q1; q += 256) {
      const int4 a = Lc4[q], b = Ln4[q];
      int chg = (a.x != b.x) | ((a.y != b.y) << 1) | ((a.z != b.z) << 2) | ((a.w != b.w) << 3);
      if (q * 4 < s0 || q * 4 + 4 > s1) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (q * 4 + k < s0 || q * 4 + k >= s1) chg &= ~(1 << k);
      }
      if (chg) {
        const int32_t nb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((chg >> k) & 1) emit(q * 4 + k, nb[k]);
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) dirty += __shfl_xor(dirty, off, 64);
  if (lane == 0 && dirty) atomicAdd(&dsum, dirty);
  __syncthreads();
  if (threadIdx.x == 0 && dsum) atomicAdd(&counters[1], dsum);
  const int n = qn;
  if (n == 0) return;  // uniform
  if (threadIdx.x == 0) base_s = atomicAdd(&counters[0], (unsigned long long)n);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) chlist[base_s + i] = q_col[i];
}

// Frontier lists: consume the dirty flags the previous superstep's al[] scatter left
// (rdirty / udirty of this parity) into per-bin row lists -- bin b's dirty rows at
// flist[bin_begin[b], + fcnt[b]) -- and a unit list (ulist, fcnt[kFcntUnits]); clears
// the consumed flags and zeroes the other parity's counts.  When every row is
// tallied (*fr_all) the bin kernels take their ranges and the flags are left alone
// (a stale flag only costs one redundant tally later).
#ifndef LPA_LIST_SUB
#define LPA_LIST_SUB 4
#endif
constexpr int kListSub = LPA_LIST_SUB;  // 16-byte flag groups per thread, all loaded up front
constexpr int kListTile = 256 * 16 * kListSub;  // flags per block (16 K; 8 and 2 groups measured within 3 us per superstep)
// bin of slot i from the block's bin bounds in LDS (binary search, 4 reads)
__device__ __forceinline__ int flag_bin(const int64_t* sbb, int64_t i) {
  int b = 0;
#pragma unroll
  for (int step = 8; step; step >>= 1)
    if (b + step < LPA_NBINS && sbb[b + step] <= i) b += step;
  return b;
}
// bit k set <=> byte k of the 16-byte group is non-zero
__device__ __forceinline__ u32 nz_mask16(uint4 r) {
  const u32 w[4] = {r.x, r.y, r.z, r.w};
  u32 m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    u32 t = w[q] | (w[q] >> 4);
    t |= t >> 2;
    t |= t >> 1;  // bit 8c set <=> byte c non-zero
    m |= ((t & 1u) | ((t >> 7) & 2u) | ((t >> 14) & 4u) | ((t >> 21) & 8u)) << (4 * q);
  }
  return m;
}
// bits of the 16-flag group at i0 whose slots lie in [lo, hi)
__device__ __forceinline__ u32 bin_bits(u32 m, int64_t i0, int64_t lo, int64_t hi) {
  const int64_t a = lo - i0, c = hi - i0;
  const u32 top = c >= 16 ? 0xFFFFu : (c <= 0 ? 0u : ((1u << c) - 1u));
  const u32 bot = a <= 0 ? 0u : (a >= 16 ? 0xFFFFu : ((1u << a) - 1u));
  return m & top & ~bot;
}
// The flags are sparse once the frontier is on (<= 0.5 % of the arcs dirty, in
// practice ~0.2 % of the rows) and the kernel is latency-bound: 32 K flags per
// block (few global atomics on the counter line), all loads in flight at once, and
// for a tile inside one bin a block scan instead of per-flag LDS atomics.
__global__ __launch_bounds__(256) void k_frontier_lists(uint8_t* __restrict__ rdirty, int64_t S,
                                                        uint8_t* __restrict__ udirty, int64_t nunits,
                                                        BinBounds bb, const int32_t* __restrict__ fr_all,
                                                        int32_t* __restrict__ flist,
                                                        int32_t* __restrict__ ulist,
                                                        int32_t* __restrict__ fcnt,
                                                        int32_t* __restrict__ fcnt_next,
                                                        int64_t nblk_rows) {
  __shared__ int32_t lcnt[LPA_NBINS + 1];
  __shared__ int32_t lpos[LPA_NBINS + 1];
  __shared__ int32_t gbase[LPA_NBINS + 1];
  __shared__ int64_t sbb[LPA_NBINS + 1];
  if (blockIdx.x == 0 && threadIdx.x < 16) fcnt_next[threadIdx.x] = 0;  // + kFcntSettled
  if (*fr_all) return;  // uniform
  const bool units = (int64_t)blockIdx.x >= nblk_rows;
  const int64_t n = units ? nunits : S;   // flag arrays are padded to 16 bytes
  uint8_t* flags = units ? udirty : rdirty;
  const int64_t t0 = (units ? (int64_t)blockIdx.x - nblk_rows : (int64_t)blockIdx.x) * kListTile;
  if (threadIdx.x < LPA_NBINS + 1) {
    lcnt[threadIdx.x] = 0;
    lpos[threadIdx.x] = 0;
    sbb[threadIdx.x] = bb.b[threadIdx.x];
  }
  // every group load in flight at once (coalesced 16-byte loads); set-flag masks kept
  uint4 raw[kListSub];
#pragma unroll
  for (int j = 0; j < kListSub; ++j) {
    const int64_t i0 = t0 + (int64_t)j * 4096 + (int64_t)threadIdx.x * 16;
    raw[j] = i0 < n ? *reinterpret_cast<const uint4*>(flags + i0) : make_uint4(0u, 0u, 0u, 0u);
  }
  u32 msk[kListSub];
  u32 anyw = 0;
#pragma unroll
  for (int j = 0; j < kListSub; ++j) {
    const int64_t i0 = t0 + (int64_t)j * 4096 + (int64_t)threadIdx.x * 16;
    u32 m = nz_mask16(raw[j]);
    if (i0 + 16 > n) m = bin_bits(m, i0, 0, n);
    msk[j] = m;
    anyw |= m;
  }
  if (!__syncthreads_or(anyw != 0u)) return;  // no dirty flag in the tile (uniform)
  // bins of the tile's first and last slot (independent scalar loads, no loop chain)
  int bt0 = kFcntUnits, bt1 = kFcntUnits;
  if (!units) {
    const int64_t tl = min(t0 + kListTile, n) - 1;
    bt0 = bt1 = 0;
#pragma unroll
    for (int k = 1; k < LPA_NBINS; ++k) {
      bt0 += bb.b[k] <= t0;
      bt1 += bb.b[k] <= tl;
    }
  }
  if (bt0 == bt1) {
    // the common case, a tile inside one bin: block scan of the per-thread counts,
    // one global atomic, every lane writes its rows at its offset
    int c = 0;
#pragma unroll
    for (int j = 0; j < kListSub; ++j) c += __popc(msk[j]);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(incl, d, 64);
      if (lane >= d) incl += t;
    }
    __shared__ int wtot[4];
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      before += k < w ? wtot[k] : 0;
      total += wtot[k];
    }
    if (threadIdx.x == 0) gbase[0] = atomicAdd(&fcnt[bt0], total);
    __syncthreads();
    if (!c) return;
    int32_t pos = gbase[0] + before + incl - c;
    int32_t* out = units ? ulist : flist + bb.b[bt0];
#pragma unroll
    for (int j = 0; j < kListSub; ++j) {
      const u32 m = msk[j];
      if (!m) continue;
      const int64_t i0 = t0 + (int64_t)j * 4096 + (int64_t)threadIdx.x * 16;
      for (u32 x = m; x; x &= x - 1u) out[pos++] = (int32_t)(i0 + __ffs(x) - 1);
      *reinterpret_cast<uint4*>(flags + i0) = make_uint4(0u, 0u, 0u, 0u);
    }
    return;
  }
  // a tile across a bin boundary (at most LPA_NBINS of them): per-lane bins,
  // pass 1 counts per bin, pass 2 positions
  if (anyw) {
#pragma unroll
    for (int j = 0; j < kListSub; ++j) {
      const u32 m = msk[j];
      if (!m) continue;
      const int64_t i0 = t0 + (int64_t)j * 4096 + (int64_t)threadIdx.x * 16;
      const int b0 = flag_bin(sbb, i0 + __ffs(m) - 1), b1 = flag_bin(sbb, i0 + 31 - __clz(m));
      for (int b = b0; b <= b1; ++b) {
        const int c = __popc(bin_bits(m, i0, sbb[b], sbb[b + 1]));
        if (c) atomicAdd(&lcnt[b], c);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < LPA_NBINS + 1) {
    const int c = lcnt[threadIdx.x];
    gbase[threadIdx.x] = c ? atomicAdd(&fcnt[threadIdx.x], c) : 0;
  }
  __syncthreads();
  if (!anyw) return;
#pragma unroll
  for (int j = 0; j < kListSub; ++j) {
    const u32 m = msk[j];
    if (!m) continue;
    const int64_t i0 = t0 + (int64_t)j * 4096 + (int64_t)threadIdx.x * 16;
    const int b0 = flag_bin(sbb, i0 + __ffs(m) - 1), b1 = flag_bin(sbb, i0 + 31 - __clz(m));
    for (int b = b0; b <= b1; ++b) {
      const u32 mb = bin_bits(m, i0, sbb[b], sbb[b + 1]);
      if (!mb) continue;
      int32_t pos = gbase[b] + atomicAdd(&lpos[b], __popc(mb));
      int32_t* out = flist + sbb[b];
      for (u32 x = mb; x; x &= x - 1u) out[pos++] = (int32_t)(i0 + __ffs(x) - 1);
    }
    *reinterpret_cast<uint4*>(flags + i0) = make_uint4(0u, 0u, 0u, 0u);
  }
}

// ---------------------------------------------------------------------------
// Row settle from the arc giant bits (superstep 3: the full tally right after the
// bits-mode rebuild of superstep 2).  A row's exact count of G votes is the popcount of
// its abits range (bit i = al[i] == G); a strict majority makes G the row's mode
// without reading one label.  Every row's dirty flag is WRITTEN (1: unsettled, a hub
// row's units alike, so no stale flag survives), k_settle_commit switches the
// superstep to list mode, and k_frontier_lists turns the flags into the bin lists
// (block scans, no per-row atomics).  It applies only while *fr_all (every row due),
// gword[1] (G worth trying) and gword[2] (abits match al), checked alike by every
// block before k_settle_commit changes fr_all.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool settle_on(const int32_t* fr_all, const int32_t* gword) {
  return *fr_all != 0 && gword[1] != 0 && (gword[2] != 0 || gword[9] != 0);
}

__device__ __forceinline__ unsigned long long range_mask(int64_t x, int64_t w0, int64_t w1, int64_t a, int64_t b) {
  unsigned long long m = ~0ull;
  if (x == w0) m &= ~0ull << (a & 63);
  if (x == w1) m &= ~0ull >> (63 - ((b - 1) & 63));
  return m;
}

// hub rows [0, n_hub) (> 1024 arcs): one wave per row
__global__ __launch_bounds__(256) void k_settle_big(const int64_t* __restrict__ rp,
                                                    const unsigned long long* __restrict__ abits, int64_t n_hub,
                                                    const int32_t* __restrict__ fr_all,
                                                    const int32_t* __restrict__ gword, int32_t* __restrict__ Ln,
                                                    uint8_t* __restrict__ rdirty, uint8_t* __restrict__ udirty,
                                                    const int64_t* __restrict__ uoff) {
  if (!settle_on(fr_all, gword)) return;  // uniform
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int32_t G = gword[0];
  for (int64_t v = (int64_t)blockIdx.x * 4 + w; v < n_hub; v += (int64_t)gridDim.x * 4) {
    const int64_t a = rp[v], b = rp[v + 1];
    const int64_t w0 = a >> 6, w1 = (b - 1) >> 6;
    u32 c = 0;
    for (int64_t x = w0 + lane; x <= w1; x += 64) c += (u32)__popcll(abits[x] & range_mask(x, w0, w1, a, b));
    c = wave_sum_u32(c);
    const bool settled = 2 * (int64_t)c > b - a;
    if (lane == 0) {
      if (settled) Ln[v] = G;
      rdirty[v] = settled ? 0 : 1;
    }
    const uint8_t f = settled ? 0 : 1;
    for (int64_t u = uoff[v] + lane; u < uoff[v + 1]; u += 64) udirty[u] = f;
  }
}

// rows [r0, r1) (<= 1024 arcs, not isolated): a thread per row
__global__ __launch_bounds__(256) void k_settle_rows(const int64_t* __restrict__ rp,
                                                     const unsigned long long* __restrict__ abits, int64_t r0,
                                                     int64_t r1, const int32_t* __restrict__ fr_all,
                                                     const int32_t* __restrict__ gword, int32_t* __restrict__ Ln,
                                                     uint8_t* __restrict__ rdirty) {
  if (!settle_on(fr_all, gword)) return;  // uniform
  const int32_t G = gword[0];
  for (int64_t v = r0 + (int64_t)blockIdx.x * 256 + threadIdx.x; v < r1; v += (int64_t)gridDim.x * 256) {
    const int64_t a = rp[v], b = rp[v + 1];
    const int64_t w0 = a >> 6, w1 = (b - 1) >> 6;
    u32 c = 0;
    for (int64_t x = w0; x <= w1; ++x) c += (u32)__popcll(abits[x] & range_mask(x, w0, w1, a, b));
    const bool settled = 2 * (int64_t)c > b - a;
    if (settled) Ln[v] = G;
    rdirty[v] = settled ? 0 : 1;
  }
}

// Superstep 4: the arc giant bits (bit i = al[i] == G) of the words covering positions
// [p0, arcs) -- the rows below the hubs -- from the labels the scatter of superstep 3
// left, so that k_settle_rows settles their G-majority rows by popcounts as in superstep
// 3 (after superstep 3 nearly every row's strict majority is G: R-MAT 100 % of the arcs).
// One streaming pass over 4 B/arc (the bins' giant decision cost ~2.5x that: LDS
// histogram atomics, scalar-issue bound row batches); the next batch's loads are in
// flight while a batch is packed.  Round 6: only when superstep 3's scatter did not keep
// the bits (gword[2] != 0: the bits of the bits-mode rebuild, the arcs whose column left
// G cleared by that scatter -- a lower bound of each row's G votes, which the settle's
// strict-majority test only needs).  gword[9] = 1: the bits are valid (G worth trying).
__global__ __launch_bounds__(256) void k_abits_pass(const int32_t* __restrict__ al, int64_t p0, int64_t arcs,
                                                    int32_t* __restrict__ gword,
                                                    unsigned long long* __restrict__ abits) {
  if (gword[1] == 0) return;  // uniform: no settle this superstep
  if (gword[2] != 0) return;  // uniform: the kept bits serve (no block writes gword[2] here)
  if (blockIdx.x == 0 && threadIdx.x == 0) gword[9] = 1;
  const u32 G = (u32)gword[0];
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t w1 = (arcs + 63) >> 6;
  int64_t g = (p0 >> 6) + (((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) << 3);
  const int64_t step = nw << 3;
  u32 v[8];
  auto load = [&](u32 (&x)[8], int64_t g0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = (g0 + k) * 64 + lane;
      x[k] = i < arcs ? ld_stream(al + i) : ~G;
    }
  };
  if (g < w1) load(v, g);
  for (; g < w1; g += step) {
    u32 vn[8];
    if (g + step < w1) load(vn, g + step);
    unsigned long long mine = 0ull;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned long long m = __ballot(v[k] == G);
      if (lane == k) mine = m;
    }
    if (lane < 8 && g + lane < w1) abits[g + lane] = mine;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = vn[k];
  }
}

// the settled superstep runs in list mode over the unsettled rows; the diff scans all
__global__ void k_settle_commit(int32_t* __restrict__ fr_all, const int32_t* __restrict__ gword,
                                int32_t* __restrict__ fcnt) {
  if (!settle_on(fr_all, gword)) return;
  *fr_all = 0;
  fcnt[kFcntSettled] = 1;
}

// superstep 4: the bins below the hubs walk the lists of their unsettled rows (gword[4]
// = 0, their "fr_all") when the settle ran, their ranges otherwise; the hub units and the
// combine keep fr_all = 1 (every hub row re-tallied, concurrently with the settle)
__global__ void k_settle_commit4(const int32_t* __restrict__ fr_all, int32_t* __restrict__ gword) {
  gword[4] = settle_on(fr_all, gword) ? 0 : 1;
}

// rebuild al[] when the changed vertices touch more than `thr` arcs (host-set)
__device__ __forceinline__ bool rebuild_wanted(const unsigned long long* counters, int64_t thr) {
  return (int64_t)counters[1] > thr;
}

// few changes: al[cpos[p]] = L_next[u] for the positions of each changed u.
// A chunk is (u << 32 | k): positions [cptr[u] + 256 k, ...).  A wave takes 64
// chunks, one per lane (independent loads of cptr and the label): chunks of <= 16
// positions are written by their own lane (4 stores in flight per step), longer
// ones by the whole wave (coalesced cpos).
// Frontier marks for the next superstep: the row holding arc position p (and, for a
// hub row, the 512-arc unit holding it) must be re-tallied.
struct FrontierMarks {
  const int32_t* crow;       // [arcs] row of each position
  const int64_t* rp;         // row offsets
  const int64_t* uoff;       // hub rows: first unit
  int64_t n_hub;
  uint8_t* rdirty;           // next parity
  uint8_t* udirty;           // next parity
  __device__ __forceinline__ void mark(int64_t p) const {
    const int32_t r = crow[p];
    rdirty[r] = 1;
    if (r < n_hub) udirty[uoff[r] + ((p - rp[r]) >> 9)] = 1;
  }
};
static_assert(kSegArcs == 512, "unit of a position: (p - rp[row]) >> 9");

// Wave-cooperative scatter of every lane's run: al[cpos[b + i]] = lab, i < n
// (n <= kChunkPos).  The runs are cut into 16-position pieces dealt over the wave's
// lanes (lane -> piece by a binary search over the inclusive piece prefix), so a
// wave whose lanes hold runs of 17..256 positions writes them in parallel instead of
// run after run with the whole wave.  Every lane of the wave must call it.
// clr (this lane's run): also clear the arc giant bits of its positions (a column that
// left G, superstep 3's scatter keeping the bits of the bits-mode rebuild: k_al_scatter)
__device__ __forceinline__ void scatter_runs(int64_t b, int n, int32_t lab, bool clr, const uint32_t* __restrict__ cpos,
                                             int32_t* __restrict__ al, bool all, const FrontierMarks& fm,
                                             unsigned long long* __restrict__ abits, int lane) {
  if (al == nullptr && all) return;  // gather mode without marks: nothing to write (uniform)
  const int k = (n + 15) >> 4;
  int incl = k;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  const int S = __shfl(incl, 63, 64);
  for (int r0 = 0; r0 < S; r0 += 64) {
    const int t = r0 + lane;
    int o = 0;  // the owner: first lane whose inclusive piece count exceeds t
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
      const int ic = __shfl(incl, o + st - 1, 64);
      if (ic <= t) o += st;
    }
    o = o < 64 ? o : 63;
    const int excl = __shfl(incl, o, 64) - __shfl(k, o, 64);
    const int64_t bo = __shfl(b, o, 64);
    const int no = __shfl(n, o, 64);
    const int32_t lv = __shfl(lab, o, 64);
    const bool cl = __shfl((int)clr, o, 64) != 0;
    if (t < S) {
      const int p0 = (t - excl) * 16;
      const int cnt = min(16, no - p0);
      const uint32_t* src = cpos + bo + p0;
      for (int q = 0; q < cnt; q += 4) {
        uint32_t p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = q + u < cnt ? src[q + u] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (q + u < cnt) {
            if (al) al[p[u]] = lv;   // gather mode: marks only
            if (cl) atomicAnd(&abits[p[u] >> 6], ~(1ull << (p[u] & 63u)));
            if (!all) fm.mark(p[u]);
          }
      }
    }
  }
}

// al[i] = L[col[i]] over the whole arc array by the calling grid (grid-stride): each
// thread keeps 8 gathers in flight (two int4 column quads), col / al streamed
// non-temporally
__device__ __forceinline__ void rebuild_all(const int32_t* __restrict__ col, int64_t arcs,
                                            const int32_t* __restrict__ Ln, int32_t* __restrict__ al) {
  const int64_t n4 = arcs >> 2;
  const v4i* __restrict__ c4 = reinterpret_cast<const v4i*>(col);
  v4i* __restrict__ a4 = reinterpret_cast<v4i*>(al);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; q + stride < n4; q += 2 * stride) {
    const v4i c0 = __builtin_nontemporal_load(c4 + q);
    const v4i c1 = __builtin_nontemporal_load(c4 + q + stride);
    v4i r0, r1;
    r0.x = Ln[c0.x]; r0.y = Ln[c0.y]; r0.z = Ln[c0.z]; r0.w = Ln[c0.w];
    r1.x = Ln[c1.x]; r1.y = Ln[c1.y]; r1.z = Ln[c1.z]; r1.w = Ln[c1.w];
    __builtin_nontemporal_store(r0, a4 + q);
    __builtin_nontemporal_store(r1, a4 + q + stride);
  }
  if (q < n4) {
    const v4i c0 = __builtin_nontemporal_load(c4 + q);
    v4i r0;
    r0.x = Ln[c0.x]; r0.y = Ln[c0.y]; r0.z = Ln[c0.z]; r0.w = Ln[c0.w];
    __builtin_nontemporal_store(r0, a4 + q);
  }
  if (blockIdx.x == 0 && threadIdx.x < (arcs & 3)) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    al[i] = Ln[col[i]];
  }
}

__global__ __launch_bounds__(256) void k_al_scatter(const int32_t* __restrict__ chlist,
                                                    const uint4* __restrict__ chflag16, int64_t ngroups,
                                                    const int32_t* __restrict__ cowner,
                                                    const int64_t* __restrict__ cch,
                                                    const unsigned long long* __restrict__ counters,
                                                    unsigned long long* __restrict__ counters_next,
                                                    const int64_t* __restrict__ cptr,
                                                    const uint32_t* __restrict__ cpos,
                                                    const int32_t* __restrict__ Ln,
                                                    int32_t* __restrict__ al, int64_t thr,
                                                    FrontierMarks fm, int32_t* __restrict__ fr_all_next,
                                                    int frontier, int64_t fr_thr,
                                                    int32_t* __restrict__ Lold,
                                                    const int32_t* __restrict__ col_fold, int64_t arcs,
                                                    int32_t* __restrict__ gword, int keep_bits,
                                                    const uint32_t* __restrict__ gbits,
                                                    unsigned long long* __restrict__ abits) {
  // the next superstep's counters (the other parity; no memset launch)
  if (blockIdx.x == 0 && threadIdx.x < 3) counters_next[threadIdx.x] = 0ull;
  const bool rebuild = rebuild_wanted(counters, thr);
  // al changes here (scatter, or the plain folded rebuild), so the arc giant bits go
  // stale: gword[2] = 0 -- except in superstep 3's scatter (keep_bits, host-set), right
  // after the bits-mode rebuild whose bits they are: a column that LEFT G (its gbits
  // bit, the rebuild's bitmap of the same vector and G) clears its positions' bits, one
  // atomic each (rare: R-MAT superstep 3 moves labels onto G); a column that joined G
  // leaves its bits clear.  The bits then hold a lower bound of every row's G votes, all
  // superstep 4's settle needs, and its k_abits_pass is skipped (round 6; exact upkeep
  // with an atomic per written position cost superstep 3 0.25 ms, round 3).  A wanted,
  // non-folded rebuild follows this kernel and sets gword[2] itself.
  const bool keep = keep_bits != 0 && !rebuild;
  if (blockIdx.x == 0 && threadIdx.x == 0 && (!rebuild || col_fold) && !keep) gword[2] = 0;
  const int32_t Gk = gword[0];
  auto left_g = [&](int64_t u, int32_t lab) -> bool {
    return keep && lab != Gk && ((gbits[u >> 5] >> (u & 31)) & 1u);
  };
  // The next superstep tallies every row after a rebuild, with the frontier off, or
  // when more than fr_thr arcs changed: then nearly every row has a changed neighbour
  // anyway (R-MAT superstep 3 -> 4: 1.5 % of arcs dirty, 88 % of the arcs in dirty
  // rows) and the per-position marks would cost more than they save.
  const bool all = rebuild || !frontier || (int64_t)counters[1] > fr_thr;
  if (blockIdx.x == 0 && threadIdx.x == 0) *fr_all_next = all ? 1 : 0;
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // col_fold (captured converged supersteps): a wanted rebuild is done here, the plain
  // form, instead of by a k_al_rebuild_hot launch that nearly always returns at once
  // (one dependent launch fewer per converged superstep)
  if (rebuild && col_fold) rebuild_all(col_fold, arcs, Ln, al);
  // one-chunk columns from the list: a lane each, longer rows of positions by the wave
  if (!rebuild) {
    const int64_t nl = (int64_t)counters[0];
    for (int64_t c0 = wid * 64; c0 < nl; c0 += nw * 64) {
      const int64_t c = c0 + lane;
      int64_t b = 0;
      int n = 0;
      int32_t lab = 0;
      bool clr = false;
      if (c < nl) {
        const int64_t u = chlist[c];
        b = cptr[u];
        n = (int)(cptr[u + 1] - b);  // <= kChunkPos
        lab = Ln[u];
        Lold[u] = lab;  // frontier sync (after the join)
        clr = left_g(u, lab);
      }
      scatter_runs(b, n, lab, clr, cpos, al, all, fm, abits, lane);
    }
  }
  uint4* __restrict__ flw = const_cast<uint4*>(chflag16);
  // multi-chunk columns: a wave takes 64 groups of 16 chunk flags, one group per lane,
  // and clears them.  Lane l of wave w takes group g0 + l * nw + w: the consecutive
  // chunks of one changed hub column land in different waves (wave-consecutive
  // groups would hand a column's hundreds of chunks to one wave, one after another)
  for (int64_t g0 = 0; g0 < ngroups; g0 += nw * 64) {
    const int64_t gi = g0 + (int64_t)lane * nw + wid;
    uint4 f = make_uint4(0u, 0u, 0u, 0u);
    if (gi < ngroups) f = chflag16[gi];
    const bool any = (f.x | f.y | f.z | f.w) != 0u;
    if (any) flw[gi] = make_uint4(0u, 0u, 0u, 0u);
    if (rebuild || __ballot(any) == 0ull) continue;  // the rebuild re-gathers every arc
    u32 bits = 0u;
    const u32 fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if ((fw[k >> 2] >> (8 * (k & 3))) & 0xFFu) bits |= 1u << k;
    // every lane pops its next flagged chunk per round: chunks of <= 16 positions are
    // written by their own lane, longer ones by the whole wave (coalesced cpos)
    while (__ballot(bits != 0u)) {
      int64_t b = 0;
      int n = 0;
      int32_t lab = 0;
      bool clr = false;
      if (bits) {
        const int t = __ffs(bits) - 1;
        bits &= bits - 1u;
        const int64_t cid = gi * 16 + t;
        const int64_t u = cowner[cid];
        const int64_t kk = cid - cch[u];
        b = cptr[u] + kk * kChunkPos;
        n = (int)min((int64_t)kChunkPos, cptr[u + 1] - b);
        lab = Ln[u];
        // frontier sync of a changed label into the next superstep's output vector
        // (after the join; every changed vertex with local arcs has a chunk 0)
        if (kk == 0) Lold[u] = lab;
        clr = left_g(u, lab);
      }
      scatter_runs(b, n, lab, clr, cpos, al, all, fm, abits, lane);
    }
  }
}

// After a lazy reset (al0) the first refresh that only scatters needs the L0 arc
// labels in al first: copied here unless the rebuild that follows rewrites every arc.
__global__ __launch_bounds__(256) void k_al_fill_unless_rebuild(const unsigned long long* __restrict__ counters,
                                                                int64_t thr, const v4i* __restrict__ src,
                                                                v4i* __restrict__ dst, int64_t arcs) {
  if (rebuild_wanted(counters, thr)) return;
  const int64_t n4 = arcs >> 2;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + q), dst + q);
  if (blockIdx.x == 0 && threadIdx.x < (arcs & 3)) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    reinterpret_cast<int32_t*>(dst)[i] = reinterpret_cast<const int32_t*>(src)[i];
  }
}

// many changes: al[i] = L_next[col[i]].  Random label gathers: each thread
// keeps 8 gathers in flight (two int4 column quads), streams col/al non-temporally.
template <bool kIfWanted>
__global__ __launch_bounds__(256) void k_al_rebuild(const unsigned long long* __restrict__ counters,
                                                    int64_t thr, const int32_t* __restrict__ col,
                                                    int64_t arcs,
                                                    const int32_t* __restrict__ Ln,
                                                    int32_t* __restrict__ al, int32_t* __restrict__ gword) {
  if (kIfWanted && !rebuild_wanted(counters, thr)) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) gword[2] = 0;  // no arc giant bits from this form
  rebuild_all(col, arcs, Ln, al);
}

// Giant-label bitmap of L (before a rebuild): bit u = (L[u] == G), G = L[0], the label
// of the highest-degree vertex.  Once the labels concentrate (R-MAT, after superstep
// 2: ~98.5 % of the arcs point at a column labelled G) the rebuild gathers one BIT per
// arc -- the hot slots' bits from LDS, the rest from this 1-bit-per-slot array, which
// stays in L2 (2 MB at C3 against the 64 MB label vector) -- and reads the label
// vector only for the columns whose bit is clear.  One ballot per 64 slots; lanes
// 0..7 store the wave's eight 64-bit words (64 contiguous bytes).
// The giant-label candidate of a label vector: the most frequent label among the
// kPickK highest-degree vertices (degree ranks k < kPickK; at P > 1 rank k lives at slot
// (k mod P) S + k / P), and whether it holds >= 1/5 of them (gword[1]: the tallies'
// giant step is worth trying).  On R-MAT and Chung-Lu (oracle, scale 21-22) that label
// is the degree-weighted mode of the whole vector in every superstep -- the top hub's
// own label is not (Chung-Lu superstep 2: the mode holds 43 % of the arcs' columns, the
// top hub's label 0.3 %).  One block, a 2K-slot LDS table.  The choice of G only
// affects speed: every use of it is exact for any G.
constexpr int kHotLabels = kHotRankedLabels;  // rank-strided label set (P > 1: power-of-two shares)
constexpr int kHotLabelsSingle = 40960;    // P = 1: the whole 160 KB of LDS
// bits mode: 1,310,688 slots' bits (the last LDS word counts the set bits first)
constexpr int64_t kHotBits = 32ll * (kHotLabelsSingle - 1);
constexpr int kPickK = 1024;
__global__ __launch_bounds__(1024) void k_giant_pick(const int32_t* __restrict__ L, int64_t n_real, int64_t S,
                                                     int P, int32_t* __restrict__ gword) {
  __shared__ u64 tab[2 * kPickK];
  __shared__ u64 wbest[kPickK / 64];
  const int t = threadIdx.x;
  tab[t] = 0ull;
  tab[t + kPickK] = 0ull;
  __syncthreads();
  const int64_t n = n_real < kPickK ? n_real : kPickK;
  if (t < n) lds_insert(tab, 32 - 11, 2 * kPickK - 1, (u32)L[(int64_t)(t % P) * S + t / P], 1u);
  __syncthreads();
  const u64 b = wave_max_u64(umax64(tab[t], tab[t + kPickK]));
  if ((t & 63) == 0) wbest[t >> 6] = b;
  __syncthreads();
  if (t == 0) {
    u64 m = 0ull;
#pragma unroll
    for (int k = 0; k < kPickK / 64; ++k) m = umax64(m, wbest[k]);
    const int32_t G = (int32_t)(~(u32)m);
    if (G != gword[0]) gword[2] = 0;  // the arc giant bits are relative to the old G
    gword[0] = G;
    gword[3] = 0;  // k_giant_bits counts the set bits of the hot slots here
    gword[5] = 0;  // no giant-code refresh unless k_code_mode takes it below
    gword[9] = 0;  // no k_abits_pass since this refresh
    gword[11] = 0;  // superstep 4's impure-unit list (k_units_pure)
    gword[1] = n > 0 && 5 * (int64_t)(m >> 32) >= n ? 1 : 0;
  }
}

// (abits / nzero: the class-blocked rebuild that follows ORs the arc giant bits of its
// pieces into abits[0, nzero): zeroed here, one launch ahead)
// gword[3] counts the set bits of the hot slots, slot i with (i & hmask) < hlim: the first
// kHotBits slots at P = 1 (hmask all ones), the first hlim slots of every slice of a
// rank-strided vector (hmask = slice - 1) -- the degree-ranked top set either way
template <bool kIfWanted>
__global__ __launch_bounds__(256) void k_giant_bits(const unsigned long long* __restrict__ counters, int64_t thr,
                                                    const int32_t* __restrict__ L, int64_t n,
                                                    int32_t* __restrict__ gword,
                                                    unsigned long long* __restrict__ bits,
                                                    unsigned long long* __restrict__ abits, int64_t nzero,
                                                    uint64_t hmask, int64_t hlim) {
  if (kIfWanted && !rebuild_wanted(counters, thr)) return;
  // the hot-bit count: summed per block in LDS, one global atomic per block (a returning
  // atomic per wave on the one word serialised: ~2,500 of them, ~30 us at C3)
  __shared__ u32 bcnt;
  if (threadIdx.x == 0) bcnt = 0u;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nzero; i += (int64_t)gridDim.x * blockDim.x)
    abits[i] = 0ull;
  const int32_t G = gword[0];
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t g0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 512; g0 < n; g0 += nw * 512) {
    int32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = g0 + k * 64 + lane;
      v[k] = i < n ? (int32_t)ld_stream(L + i) : ~G;
    }
    unsigned long long mine = 0ull;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned long long m = __ballot(v[k] == G);
      if (lane == k) mine = m;
    }
    if (lane < 8 && g0 + lane * 64 < n) bits[(g0 >> 6) + lane] = mine;
    // the hot slots' set bits (the rebuild's bits-mode test without an LDS fill); hlim
    // and the slice are multiples of 64, so a bit word is hot or cold as a whole
    const int64_t wi = g0 + lane * 64;
    const bool hot = lane < 8 && wi < n && (int64_t)((uint64_t)wi & hmask) < hlim;
    if (__ballot(hot)) {
      const u32 c = wave_sum_u32(hot ? (u32)__popcll(mine) : 0u);
      if (lane == 0 && c) atomicAdd(&bcnt, c);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && bcnt) atomicAdd(&gword[3], (int32_t)bcnt);
}

// al[i] = lab(col[i]) over every arc by the calling grid (one wave per 512-arc batch,
// grid-stride); bits: also the arc giant bits (abits: bit i = al[i] == G, one ballot
// per 64 arcs), which the next superstep's full tally settles rows from (k_settle_*).
template <typename Lab>
__device__ __forceinline__ void rebuild_stream(Lab lab, int32_t G, bool bits, const int32_t* __restrict__ col,
                                               int64_t arcs, int32_t* __restrict__ al,
                                               unsigned long long* __restrict__ abits) {
  // lane-consecutive arcs: one gather instruction covers 64 consecutive arcs of
  // a row, whose sorted columns often share lines (hub rows) -> fewer L2 requests.
  // Full 512-arc batches are software-pipelined: the next batch's column loads are in
  // flight while this batch's labels are looked up and stored.
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t step = nw * 512;
  const int64_t nfull = arcs & ~(int64_t)511;  // arcs of the full batches
  int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 512;
  int32_t c[8];
  if (base < nfull) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_nontemporal_load(col + base + k * 64 + lane);
  }
  for (; base < nfull; base += step) {
    int32_t cn[8], r[8];
    const int64_t nb = base + step;
    if (nb < nfull) {
#pragma unroll
      for (int k = 0; k < 8; ++k) cn[k] = __builtin_nontemporal_load(col + nb + k * 64 + lane);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = lab(c[k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(r[k], al + base + k * 64 + lane);
    if (bits) {
      unsigned long long mine = 0ull;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const unsigned long long m = __ballot(r[k] == G);
        if (lane == k) mine = m;
      }
      if (lane < 8) abits[(base >> 6) + lane] = mine;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = cn[k];
  }
  // the partial last batch (one wave)
  if (nfull < arcs && base == nfull) {
    for (int k = 0; k < 8; ++k) {
      const int64_t i = base + k * 64 + lane;
      const bool v = i < arcs;
      const int32_t x = v ? lab(col[i]) : 0;
      if (v) al[i] = x;
      const unsigned long long m = __ballot(v && x == G);
      if (bits && lane == 0 && base + k * 64 < arcs) abits[(base >> 6) + k] = m;
    }
  }
}

// The same stream in a three-stage software pipeline over 512-arc batches (P = 1 hot
// kernel): at step t the column loads of batch t + 3 are issued, batch t + 2's probe
// words fetched (p1: an LDS word, or an L2 word of gbits for a cold column), batch
// t + 1's labels resolved (p2: from the word, else a gather of L[c]) and batch t stored,
// so each wave keeps three batches' dependent loads in flight instead of one batch's
// chain (col -> bit word -> label).  Rings of 3 column sets and 2 word / label sets,
// six steps unrolled so no set is copied while its loads are in flight.
// The main loop is branch-free (every stage's batch exists, and p1 / p2 issue their
// loads unconditionally, at a clamped address where the value is not needed): the
// vector-memory counter is then tracked exactly, and waiting for batch t's labels does
// not wait for the loads of batches t + 1 .. t + 3 -- with a conditional load in the
// loop the compiler waited for every outstanding load (vmcnt(0)) at each step, which
// serialised the pipeline.  The last few batches run guarded.
//   fetch(t, c)  batch t's columns        probe(c, w)   p1 words
//   resolve(c, w, r)  p2 labels          store(t, r)    stores (+ arc giant bits)
template <typename Pre, typename F, typename Q, typename R, typename St>
__device__ __forceinline__ void pipe3(int64_t nb, Pre pre, F fetch, Q probe, R resolve, St store) {
  int32_t c0[8], c1[8], c2[8], r0[8], r1[8];
  u32 w0[8], w1[8];
  int64_t t = 0;
  if (nb <= 0) return;
  // pre(t, slot): batch t's descriptors (six slots, batch t in slot t mod 6), four
  // steps ahead of its fetch
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < nb) pre(k, k);
  fetch(0, c0, 0);
  if (nb > 1) fetch(1, c1, 1);
  if (nb > 2) fetch(2, c2, 2);
  probe(c0, w0);
  if (nb > 1) probe(c1, w1);
  resolve(c0, w0, r0);
#define LPA_PIPE_STEP(GUARD, I, CA, CB, CC, WA, WB, RA, RB) \
  if (!GUARD || t + 4 < nb) pre(t + 4, (I + 4) % 6);      \
  if (!GUARD || t + 3 < nb) fetch(t + 3, CA, (I + 3) % 6); \
  if (!GUARD || t + 2 < nb) probe(CC, WA);                 \
  if (!GUARD || t + 1 < nb) resolve(CB, WB, RB);           \
  store(t, RA, I);                                         \
  ++t;                                                     \
  if (GUARD && t >= nb) break;
#define LPA_PIPE_CYCLE(GUARD)                                 \
  LPA_PIPE_STEP(GUARD, 0, c0, c1, c2, w0, w1, r0, r1)        \
  LPA_PIPE_STEP(GUARD, 1, c1, c2, c0, w1, w0, r1, r0)        \
  LPA_PIPE_STEP(GUARD, 2, c2, c0, c1, w0, w1, r0, r1)        \
  LPA_PIPE_STEP(GUARD, 3, c0, c1, c2, w1, w0, r1, r0)        \
  LPA_PIPE_STEP(GUARD, 4, c1, c2, c0, w0, w1, r0, r1)        \
  LPA_PIPE_STEP(GUARD, 5, c2, c0, c1, w1, w0, r1, r0)
  // unguarded cycles: their last step (t + 5) issues pre(t + 9), so t + 9 < nb keeps
  // every descriptor read inside the list (a piece list has no padding past its end)
  while (t + 10 <= nb) {
    LPA_PIPE_CYCLE(false)
  }
  while (true) {
    LPA_PIPE_CYCLE(true)
  }
#undef LPA_PIPE_CYCLE
#undef LPA_PIPE_STEP
}

// arc giant bits of one 64-lane chunk at arc position st (len lanes live, lanes
// consecutive): one word, or two when st is not word-aligned (ORed: other chunks share
// the words; nzero-ed by k_giant_bits beforehand)
__device__ __forceinline__ void or_arc_bits(unsigned long long* __restrict__ abits, u32 st, unsigned long long m,
                                            int lane) {
  const u32 wd = st >> 6, off = st & 63u;
  if (m && lane == 0) atomicOr(&abits[wd], m << off);
  if (m && lane == 1 && off && (m >> (64u - off))) atomicOr(&abits[wd + 1], m >> (64u - off));
}

// the plain stream: this wave's whole 512-arc batches of [0, arcs), then the partial
// last batch (one wave)
template <typename P1, typename P2>
__device__ __forceinline__ void rebuild_pipe(P1 p1, P2 p2, int32_t G, bool bits, const int32_t* __restrict__ col,
                                             int64_t arcs, int32_t* __restrict__ al,
                                             unsigned long long* __restrict__ abits) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nbatch = arcs >> 9;
  const int64_t nb = wv < nbatch ? (nbatch - wv + nw - 1) / nw : 0;
  auto base = [&](int64_t t) { return (wv + t * nw) * 512; };
  auto pre = [](int64_t, int) {};
  auto fetch = [&](int64_t t, int32_t (&c)[8], int) {
    const int64_t b = base(t);
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_nontemporal_load(col + b + k * 64 + lane);
  };
  auto probe = [&](const int32_t (&c)[8], u32 (&w)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = p1(c[k]);
  };
  auto resolve = [&](const int32_t (&c)[8], const u32 (&w)[8], int32_t (&r)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = p2(c[k], w[k]);
  };
  auto store = [&](int64_t t, const int32_t (&r)[8], int) {
    const int64_t b = base(t);
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(r[k], al + b + k * 64 + lane);
    if (bits) {
      unsigned long long mine = 0ull;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const unsigned long long m = __ballot(r[k] == G);
        if (lane == k) mine = m;
      }
      if (lane < 8) abits[(b >> 6) + lane] = mine;
    }
  };
  pipe3(nb, pre, fetch, probe, resolve, store);
  // the partial last batch (one wave)
  const int64_t nfull = nbatch << 9;
  if (nfull < arcs && wv == nbatch % nw) {
    for (int k = 0; k < 8; ++k) {
      const int64_t i = nfull + k * 64 + lane;
      const bool v = i < arcs;
      const int32_t c = v ? col[i] : 0;
      const int32_t x = p2(c, p1(c));
      if (v) al[i] = x;
      const unsigned long long m = __ballot(v && x == G);
      if (bits && lane == 0 && nfull + k * 64 < arcs) abits[(nfull >> 6) + k] = m;
    }
  }
}

// The class-blocked part of a labels-mode rebuild (P = 1).  A labels-mode rebuild is
// bound by its L2-missing gathers (C3 superstep 1: 3.6x the algorithmic bytes); a block
// group (blocks b = x mod 8, one XCD under the observed round-robin placement, speed
// only) streams the pieces of column class x -- the class segments of the rows of degree
// > block_deg, which keep their columns in (class, column) order -- so an XCD's gathers
// touch 1/8 of the label lines and its L2 holds far more of them (C3, simulated: 0.18
// -> 0.02 missing gathers per arc).  8 pieces (<= 64 arcs, lane-consecutive) per batch
// and wave, in pipe3's pipeline; a lane past its piece carries column 0 (a hot-set LDS
// read) and stores nothing; the descriptors ride a register ring four batches ahead
// (scalar loads in the stage that used them cost a round trip per step: the pieces
// phase ran at ~7 us per batch and wave).  bits: the arc giant bits, ORed.
#ifdef LPA_BLKTIME
// diagnostic build only (csrc/Makefile blktime): per block of the last blocked rebuild,
// the wall clock at its start, after its pieces and at its end
__device__ unsigned long long g_blk_time[3 * 512];
extern "C" int lpa_diag_blk_times(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blk_time), sizeof(g_blk_time)) != hipSuccess) return -1;
  static unsigned long long zero[3 * 512];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_blk_time), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif
struct BlkInfo {
  int64_t off[kMaxBlkClasses + 1];  // class x: pieces [off[x], off[x + 1]), multiples of 8
  int64_t a0;                       // listed arcs [0, a0) (0: no blocked part)
  int phases;                       // classes / 8: group x streams x, x + 8, ...
};
template <typename P1, typename P2>
__device__ __forceinline__ void rebuild_pieces(P1 p1, P2 p2, int32_t G, bool bits, const u64* __restrict__ pieces,
                                               int64_t q0, int64_t q1, int64_t wi, int64_t nwv,
                                               const int32_t* __restrict__ col, int32_t* __restrict__ al,
                                               unsigned long long* __restrict__ abits) {
  const int lane = threadIdx.x & 63;
  auto uni = [](int64_t v) -> int64_t {
    return (int64_t)(((u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)((u64)v >> 32)) << 32) |
                     (u64)(u32)__builtin_amdgcn_readfirstlane((int)(u32)v));
  };
  const int64_t step = uni(nwv * 8), first = uni(q0 + wi * 8), last = uni(q1);
  const int64_t nb = first < last ? (last - first + step - 1) / step : 0;
  // descriptor ring: lane k < 8 of slot j holds piece k of the batch in slot j, loaded
  // four steps ahead (a vector load, so waiting for it never waits on newer loads);
  // the stages read it with readlane
  u64 dr[6];
  auto pre = [&](int64_t t, int j) {
    const int64_t qq = first + t * step;
    dr[j] = lane < 8 ? pieces[qq + lane] : 0ull;
  };
  auto desc = [&](int j, int k) -> u64 {
    return ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(dr[j] >> 32), k) << 32) |
           (u64)(u32)__builtin_amdgcn_readlane((int)(u32)dr[j], k);
  };
  auto fetch = [&](int64_t, int32_t (&c)[8], int j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u64 d = desc(j, k);
      const bool live = lane < (int)(d >> 32);
#if defined(LPA_BLK_ABL) && LPA_BLK_ABL == 3
      const int32_t x = (int32_t)(((u32)d + lane) * 2654435761u >> 8);  // ablation: no column loads
#else
      const int32_t x = __builtin_nontemporal_load(col + (u32)d + (live ? lane : 0));
#endif
      c[k] = live ? x : 0;
    }
  };
  // the probe word is read where it is used (an LDS read in the labels / hybrid modes
  // this path serves): no word ring, 16 VGPRs fewer
  auto probe = [&](const int32_t (&)[8], u32 (&)[8]) {};
  auto resolve = [&](const int32_t (&c)[8], const u32 (&)[8], int32_t (&r)[8]) {
#pragma unroll
#if defined(LPA_BLK_ABL) && LPA_BLK_ABL == 1
    for (int k = 0; k < 8; ++k) r[k] = c[k];  // ablation: no label gathers
#else
    for (int k = 0; k < 8; ++k) r[k] = p2(c[k], p1(c[k]));
#endif
  };
  auto store = [&](int64_t, const int32_t (&r)[8], int j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u64 d = desc(j, k);
      const int ln = (int)(d >> 32);
#if defined(LPA_BLK_ABL) && LPA_BLK_ABL == 2
      if (lane < ln && r[k] == -7) al[(u32)d + lane] = 0;  // ablation: no stores
#else
      if (lane < ln) __builtin_nontemporal_store(r[k], al + (u32)d + lane);
      if (bits) or_arc_bits(abits, (u32)d, __ballot(lane < ln && r[k] == G), lane);
#endif
    }
  };
  pipe3(nb, pre, fetch, probe, resolve, store);
}

// al[] rebuild with an LDS hot set (the slots of the highest-degree vertices: at P = 1
// the first slots, 30-40 % of all arc targets on R-MAT).  The rebuild is bound by the
// line traffic of its L2-missing 4-B gathers, and every gather served from LDS is one
// L2 request fewer.  One 1024-thread block per CU, 160 KB of LDS, in one of two modes
// that every block picks alike from the same data:
//   bits    (most hot slots carry the giant label G): LDS holds the giant-label bits of
//           the first 1.31 M slots, the other columns' bits come from gbits (L2); a
//           set bit is G, a clear one reads L[c].
//   labels  LDS holds the labels of the first 40,960 slots; the rest read L[c].
// kRanked (P > 1, power-of-two slices and rank count): the hottest vertices of rank
// r's slice are its first slots (degree rank k lives at slot (k mod P) S + k / P),
// so the global top set is the first H slots of every slice: slot c is hot iff
// (c mod S) < H, at LDS index (c / S) H + c mod S (H = 2^hot_lg labels or 2^hb_lg bits).
// kPieces (P = 1, a class-blocked handle: its labels-mode rebuild goes through the pieces):
// its own instantiation, so that the plain one's registers are allocated without the
// pieces' descriptor ring (one form for both spilled 16 VGPRs to scratch at the 128 of
// four waves per SIMD)
template <bool kIfWanted, bool kRanked, bool kPieces = false>
__global__ __launch_bounds__(1024) void k_al_rebuild_hot(const unsigned long long* __restrict__ counters,
                                                         int64_t thr, const int32_t* __restrict__ col,
                                                         int64_t arcs, const int32_t* __restrict__ Ln,
                                                         int32_t nhot, int32_t* __restrict__ al,
                                                         int slice_lg, int hot_lg, int hb_lg,
                                                         const uint32_t* __restrict__ gbits, int64_t nbits,
                                                         int32_t* __restrict__ gword,
                                                         unsigned long long* __restrict__ abits,
                                                         const u64* __restrict__ pieces, BlkInfo blk,
                                                         const int32_t* __restrict__ skip) {
  if (kIfWanted && !rebuild_wanted(counters, thr)) return;
  if (skip && *skip) return;  // the giant-code refresh replaces this rebuild (k_code_mode)
  __shared__ u32 hot[kHotLabelsSingle];
  u32* s_cnt = &hot[kHotLabelsSingle - 1];   // beyond the bit words; labels mode refills it
  // ---- the giant-label bits of the hot slots, and how many are set ----
  const int64_t nhb = kRanked ? ((int64_t)(nbits >> slice_lg) << hb_lg) : (nbits < kHotBits ? nbits : kHotBits);
  const int nhw = (int)((nhb + 31) >> 5);
  if (threadIdx.x == 0) *s_cnt = 0u;
  __syncthreads();
  int cnt = 0;
  for (int q = threadIdx.x; q < nhw; q += 1024) {
    int64_t gw = q;
    if constexpr (kRanked) gw = ((int64_t)(q >> (hb_lg - 5)) << (slice_lg - 5)) + (q & ((1 << (hb_lg - 5)) - 1));
    const u32 w = gbits[gw];
    hot[q] = w;
    cnt += __popc(w);
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(s_cnt, (u32)cnt);
  __syncthreads();
  const bool bits = 2 * (int64_t)*s_cnt >= nhb && nhb > 0;  // uniform: the same data in every block
  // hybrid (P = 1): G on >= 1/8 of the bit-range slots but not on half -- labels-mode
  // gathers that also write the arc giant bits (the next superstep's settle).  (Taking a
  // cold column's G from its gbits bit instead of its label measured slower: C5 186.7 ->
  // 176.4 GTEPS.)
  const bool hyb = !kRanked && !bits && 8 * (int64_t)*s_cnt >= nhb && nhb > 0;
  const int32_t G = gword[0];
  // bits / hybrid modes also write the arc giant bits (abits: bit i = al[i] == G, one
  // ballot per 64 arcs), which the next superstep's full tally settles rows from
  // (k_settle_*)
  if (blockIdx.x == 0 && threadIdx.x == 0) gword[2] = (bits || hyb) ? 1 : 0;
  if (!bits) {
    __syncthreads();
    for (int i = threadIdx.x; i < nhot; i += 1024)
      hot[i] = (u32)(kRanked ? Ln[((int64_t)(i >> hot_lg) << slice_lg) + (i & ((1 << hot_lg) - 1))] : Ln[i]);
    __syncthreads();
  }
  const u32 nh = (u32)nhot;
  const u32 smask = kRanked ? (1u << slice_lg) - 1u : 0u, hcap = 1u << hot_lg, bcap = 1u << hb_lg;
  auto lab = [&](int c) -> int32_t {
    if (bits) {
      u32 w;
      if constexpr (kRanked) {
        const u32 j = (u32)c & smask;
        w = j < bcap ? hot[((((u32)c >> slice_lg) << hb_lg) + j) >> 5] : gbits[(u32)c >> 5];
      } else {
        w = (u32)c < (u32)nhb ? hot[(u32)c >> 5] : gbits[(u32)c >> 5];
      }
      return ((w >> ((u32)c & 31u)) & 1u) ? G : Ln[c];
    }
    if constexpr (kRanked) {
      const u32 j = (u32)c & smask;
      return j < hcap ? (int32_t)hot[(((u32)c >> slice_lg) << hot_lg) + j] : Ln[c];
    } else {
      return (u32)c < nh ? (int32_t)hot[c] : Ln[c];
    }
  };
  if constexpr (kRanked) {
    rebuild_stream(lab, G, bits, col, arcs, al, abits);
  } else {
    // branch-free probes (pipe3): both sources are read -- the LDS word at a clamped
    // index, the gbits word / the label at a fixed address where it is not needed (the
    // wave's lanes then share one line)
    const u32 nhbu = (u32)nhb;
    // (the slots' labels through a buffer descriptor: launch_rebuild takes this kernel at
    // P = 1 only up to kHotMaxSlots = 2^29 slots, so every byte offset fits the voffset)
    const auto ln_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)Ln, 0, (int)(nbits * 4), 0x00020000);
    constexpr int kPast = (int)0x80000000u;  // past every record count: no request
    auto run = [&](auto p1, auto p2, bool wbits) {
      // uniform: labels / hybrid mode of a blocked handle (the bits mode through the
      // pieces measured slower, round 6: C5 superstep 3 13.4 -> 17.4 ms, C4 superstep 2
      // 8.9 -> 12.8 ms -- its lookups hit LDS / L2 anyway, the split arc ranges cost)
      if (kPieces && !bits) {
        const int grp = blockIdx.x & 7;
        const int64_t nwv = (int64_t)(gridDim.x >> 3) * (blockDim.x >> 6);
        const int64_t wi = (int64_t)(blockIdx.x >> 3) * (blockDim.x >> 6) + (threadIdx.x >> 6);
#ifdef LPA_BLKTIME
        if (threadIdx.x == 0 && blockIdx.x < 512) g_blk_time[3 * blockIdx.x] = wall_clock64();
#endif
        for (int ph = 0; ph < blk.phases; ++ph)
          rebuild_pieces(p1, p2, G, wbits, pieces, blk.off[grp + 8 * ph], blk.off[grp + 8 * ph + 1], wi, nwv,
                         col, al, abits);
#ifdef LPA_BLKTIME
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 512) atomicMax(&g_blk_time[3 * blockIdx.x + 1], wall_clock64());
#endif
        // then every block: the plain stream over the rows below block_deg
        rebuild_pipe(p1, p2, G, wbits, col + blk.a0, arcs - blk.a0, al + blk.a0, abits + blk.a0 / 64);
#ifdef LPA_BLKTIME
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 512) atomicMax(&g_blk_time[3 * blockIdx.x + 2], wall_clock64());
#endif
      } else {
        rebuild_pipe(p1, p2, G, wbits, col, arcs, al, abits);
      }
    };
    if (bits) {
      // the gbits words and the labels through buffer descriptors (base + 32-bit offset:
      // two VGPRs fewer per address under the 128 of four waves per SIMD, where the 64-bit
      // form spilled 14), and a lane that needs no word or label takes an offset past the
      // records: the range check drops its request instead of re-reading a fixed line
      const auto gb_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)gbits, 0, (int)(((nbits + 31) >> 5) * 4), 0x00020000);
      run(
          [&](int c) -> u32 {
            const bool h = (u32)c < nhbu;
            const u32 hw = hot[(h ? (u32)c : nhbu - 1u) >> 5];
            const u32 gw = __builtin_amdgcn_raw_buffer_load_b32(gb_rsrc, h ? kPast : (int)(((u32)c >> 5) << 2), 0, 0);
            return h ? hw : gw;
          },
          [&](int c, u32 w) -> int32_t {
            const bool g = (w >> ((u32)c & 31u)) & 1u;
            const int32_t x = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ln_rsrc, g ? kPast : (int)((u32)c << 2), 0, 0);
            return g ? G : x;
          },
          true);
    } else {
      run([&](int c) -> u32 { return hot[(u32)c < nh ? (u32)c : nh - 1u]; },
          [&](int c, u32 w) -> int32_t {
            const bool h = (u32)c < nh;
            const int32_t x = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ln_rsrc, h ? kPast : (int)((u32)c << 2), 0, 0);
            return h ? (int32_t)w : x;
          },
          hyb);
    }
  }
}

// al[] rebuild of a small label vector (P = 1, < kHotMinSlots slots: it stays in L2 /
// the Infinity Cache, so an LDS hot set saves no misses while every block's 160 KB fill
// costs as much as the arcs' stream at C2 scale): the same bits / labels modes, the
// bits-mode test from k_giant_bits' count of the hot slots' set bits (gword[3]).
template <bool kIfWanted>
__global__ __launch_bounds__(256) void k_al_rebuild_small(const unsigned long long* __restrict__ counters,
                                                          int64_t thr, const int32_t* __restrict__ col, int64_t arcs,
                                                          const int32_t* __restrict__ Ln, int32_t* __restrict__ al,
                                                          const uint32_t* __restrict__ gbits, int64_t nbits,
                                                          int32_t* __restrict__ gword,
                                                          unsigned long long* __restrict__ abits) {
  if (kIfWanted && !rebuild_wanted(counters, thr)) return;
  const int64_t nhb = nbits < kHotBits ? nbits : kHotBits;
  const bool bits = nhb > 0 && 2 * (int64_t)gword[3] >= nhb;  // uniform
  const int32_t G = gword[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) gword[2] = bits ? 1 : 0;
  if (!bits) {  // labels mode: the plain 16 B/lane gather stream (C2: 0.21 -> ~0.17 ms)
    rebuild_all(col, arcs, Ln, al);
    return;
  }
  auto lab = [&](int c) -> int32_t {
    if ((gbits[(u32)c >> 5] >> ((u32)c & 31u)) & 1u) return G;
    return Ln[c];
  };
  rebuild_stream(lab, G, true, col, arcs, al, abits);
}

// ---------------------------------------------------------------------------
// Giant codes (round 5): the refresh after superstep 1 without the labels-mode al[]
// rebuild.  On R-MAT the labels L1 of superstep 1 already have a giant label G (the
// label of ~97 % of the 1,024 top hubs, ~37 % of the arcs' columns) but not on half the
// hot slots, so that refresh gathered a full 4-B label per arc (C3: 2.35 ms, 3.6x its
// algorithmic bytes in L2-missing lines), and superstep 2 read them back only to
// decide nearly every row for G: a row's G votes above every bucket of a label hash of
// its other votes make G its strict mode (giant_count; oracle, R-MAT-22: 98 % of the
// arcs sit in rows so decided with 16 buckets, 100 % of the rows above 64 arcs).
// A bucket only needs a FUNCTION of the label -- and three buckets suffice (oracle,
// R-MAT-21 superstep 2: rows of 65-1024 arcs holding 99.9 % of their arcs, every hub row,
// 90 % of the 9-64-arc rows' arcs decided; 63 buckets: 100 / 100 / 99.4 %) -- so the
// refresh writes 2-bit codes, 0 = (label == G), else 1 + a hash of the label mod 3:
//   code2     per slot, 16 to a word (k_code_build): 4 MB at C3, one XCD's L2
//   al2[i]    per arc of the rows above the cut, code2[col[i]], 16 arcs to a word
//             (k_code_rebuild; the 655,360 hottest slots' codes in LDS)
//   al[i]     per arc of the rows below the cut (code_lbin: <= 64 arcs on a label vector
//             of <= 64 MB, else <= 8), their labels
// and superstep 2 decides the hub rows (k_lpa_units_code2 + k_hub_decide) and the rows of
// the other coded rows (k_code_settle) by popcounts of the code words -- no
// table, no atomics; only the rows left undecided get their al[] entries gathered
// (k_code_partial_*) and are tallied exactly, in list mode.  Exact for any G and any hash
// (a label's count is at most its bucket's); gword[5] marks the refresh taken, so the
// labels-mode rebuild is skipped and superstep 2's refresh rebuilds al[] whatever the
// change count.
// (Round 5 first shipped 8-bit codes with 64-bucket LDS histograms: C3 code rebuild 1.41
// ms, code settle 0.63 ms -- the histogram atomics and the 16 MB code array's L2 misses.)
// ---------------------------------------------------------------------------
__device__ __forceinline__ u32 giant_code2(u32 x, u32 G) {
  return x == G ? 0u : 1u + ((((x * 0x9E3779B1u) >> 24) * 3u) >> 8);
}

// the four codes' counts among the fields of w whose low bits fm selects:
// c0 | c1 << 16 (x) and c2 | c3 << 16 (y)
__device__ __forceinline__ void code2_counts(u32 w, u32 fm, u32& x, u32& y) {
  const u32 lo = w & fm, hi = (w >> 1) & fm;
  x += (u32)__popc(fm & ~(lo | hi)) | ((u32)__popc(lo & ~hi) << 16);
  y += (u32)__popc(hi & ~lo) | ((u32)__popc(lo & hi) << 16);
}
// low bits of the fields of word wi that hold arcs [b, e)
__device__ __forceinline__ u32 code2_fmask(int64_t wi, int64_t b, int64_t e) {
  const int64_t base = wi * 16;
  const int64_t l0 = b - base, h0 = e - base;
  const int lo = (int)(l0 < 0 ? 0 : l0 > 16 ? 16 : l0), hi = (int)(h0 < 0 ? 0 : h0 > 16 ? 16 : h0);
  const u32 mh = hi >= 16 ? 0xFFFFFFFFu : ((1u << (2 * hi)) - 1u);
  const u32 ml = lo >= 16 ? 0xFFFFFFFFu : ((1u << (2 * lo)) - 1u);
  return mh & ~ml & 0x55555555u;
}
// G decided from summed counts: its votes above every bucket
__device__ __forceinline__ bool code2_decided(u32 x, u32 y) {
  const u32 c0 = x & 0xFFFFu, c1 = x >> 16, c2 = y & 0xFFFFu, c3 = y >> 16;
  return c0 > max(c1, max(c2, c3));
}
__device__ __forceinline__ u32 spread16(u32 v) {
  v = (v | (v << 8)) & 0x00FF00FFu;
  v = (v | (v << 4)) & 0x0F0F0F0Fu;
  v = (v | (v << 2)) & 0x33333333u;
  return (v | (v << 1)) & 0x55555555u;
}
// the 2-bit codes r[k] of arcs b + 64 k + lane (b a multiple of 512) -> 32 words at
// al2[b / 16 ..): two ballots per chunk, lane l < 32 assembles word l (chunk l / 4)
__device__ __forceinline__ void store_code2(uint32_t* __restrict__ al2, int64_t b, const int32_t (&r)[8], int lane) {
  u64 m0 = 0, m1 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const u64 b0 = __ballot(r[k] & 1), b1 = __ballot((r[k] >> 1) & 1);
    if ((lane >> 2) == k) {
      m0 = b0;
      m1 = b1;
    }
  }
  const int sh = (lane & 3) * 16;
  const u32 w = spread16((u32)(m0 >> sh) & 0xFFFFu) | (spread16((u32)(m1 >> sh) & 0xFFFFu) << 1);
  if (lane < 32) al2[(b >> 4) + lane] = w;
}

// gword[5] = take the giant-code refresh: a rebuild is wanted, G is worth trying, and the
// bits-mode rebuild (G on >= half the hot slots) does not apply; no arc giant bits then
__global__ void k_code_mode(const unsigned long long* __restrict__ counters, int64_t thr, int64_t nhb,
                            int32_t* __restrict__ gword) {
  if (threadIdx.x != 0) return;
  const bool on = rebuild_wanted(counters, thr) && gword[1] != 0 && 2 * (int64_t)gword[3] < nhb;
  gword[5] = on ? 1 : 0;
  if (on) gword[2] = 0;
}

// code2 for every slot: 16 labels (four int4 loads) -> one word (vpad is a multiple of 64)
__global__ __launch_bounds__(256) void k_code_build(const int4* __restrict__ L4, int64_t nw,
                                                   const int32_t* __restrict__ gword, uint32_t* __restrict__ code2) {
  if (gword[5] == 0) return;
  const u32 G = (u32)gword[0];
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nw; q += (int64_t)gridDim.x * blockDim.x) {
    u32 w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int4 v = L4[4 * q + k];
      w |= (giant_code2((u32)v.x, G) | (giant_code2((u32)v.y, G) << 2) | (giant_code2((u32)v.z, G) << 4) |
            (giant_code2((u32)v.w, G) << 6))
           << (8 * k);
    }
    code2[q] = w;
  }
}

// pipe3 over this wave's whole 512-arc batches in [bat0, bat1) (grid-stride by waves)
template <typename P1, typename P2, typename St>
__device__ __forceinline__ void range_pipe(P1 p1, P2 p2, St st, const int32_t* __restrict__ col, int64_t bat0,
                                           int64_t bat1) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nb = bat0 + wv < bat1 ? (bat1 - bat0 - wv + nw - 1) / nw : 0;
  auto base = [&](int64_t t) { return (bat0 + wv + t * nw) * 512; };
  auto pre = [](int64_t, int) {};
  auto fetch = [&](int64_t t, int32_t (&c)[8], int) {
    const int64_t b = base(t);
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_nontemporal_load(col + b + k * 64 + lane);
  };
  auto probe = [&](const int32_t (&c)[8], u32 (&w)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = p1(c[k]);
  };
  auto resolve = [&](const int32_t (&c)[8], const u32 (&w)[8], int32_t (&r)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = p2(c[k], w[k]);
  };
  auto store = [&](int64_t t, const int32_t (&r)[8], int) { st(base(t), r); };
  pipe3(nb, pre, fetch, probe, resolve, store);
}

// al for [pB, arcs) (pB = code_pcut rounded down to a 512-arc batch) and al2 for [0, pA)
// (pA = code_pcut rounded up, at most the full batches): the batch across code_pcut gets
// both; the partial last batch (one wave) writes whichever applies.  One 1024-thread
// block per CU, 160 KB of LDS: the labelled rows (code_lbin) first, with the 40,960
// hottest labels in LDS, then the codes, with the 655,360 hottest slots' codes in LDS --
// the gathers are bound by their lane count, not their bytes, so the LDS share is the
// lever -- and the others from the 2-bit code array (vpad / 4 bytes: L2-resident at C3).
// kRanked (a partitioned job's rank, round 6): the hot sets are the first 2^hot_lg labels
// and the first 2^hc_lg codes of EVERY slice (degree rank k lives at slot (k mod P) S +
// k / P, so these are the global top degree ranks), at LDS index (c / S) H + c mod S as in
// k_al_rebuild_hot's ranked form; at P = 1 they are the first slots.
template <bool kRanked>
__global__ __launch_bounds__(1024) void k_code_rebuild(const int32_t* __restrict__ gword,
                                                       const int32_t* __restrict__ col, int64_t arcs,
                                                       const int32_t* __restrict__ Ln, int64_t nslots,
                                                       const uint32_t* __restrict__ code2, int64_t p64,
                                                       uint32_t* __restrict__ al2, int32_t* __restrict__ al,
                                                       int slice_lg, int hot_lg, int hc_lg) {
  if (gword[5] == 0) return;
  __shared__ u32 hot[kHotLabelsSingle];
  const u32 G = (u32)gword[0];
  const int lane = threadIdx.x & 63;
  const int64_t nfull = arcs >> 9;
  const int64_t bA = min((p64 + 511) >> 9, nfull), bB = p64 >> 9;
  const u32 smask = kRanked ? (1u << slice_lg) - 1u : 0u;
  // slot c -> its hot-set index (h: whether it has one) for a set of 2^lg per slice
  auto hot_at = [&](int c, int lg, u32 nflat, bool& h) -> u32 {
    if constexpr (kRanked) {
      const u32 j = (u32)c & smask;
      h = j < (1u << lg);
      return (((u32)c >> slice_lg) << lg) + j;
    } else {
      h = (u32)c < nflat;
      return (u32)c;
    }
  };
  // ---- the labels of the rows below the cut ----
  const u32 nh = kRanked ? (u32)((nslots >> slice_lg) << hot_lg)
                         : (u32)(nslots < kHotLabelsSingle ? nslots : kHotLabelsSingle);
  for (u32 i = threadIdx.x; i < nh; i += 1024)
    hot[i] = (u32)Ln[kRanked ? ((int64_t)(i >> hot_lg) << slice_lg) + (i & ((1u << hot_lg) - 1u)) : (int64_t)i];
  __syncthreads();
  range_pipe([&](int c) -> u32 {
               bool h;
               const u32 k = hot_at(c, hot_lg, nh, h);
               return hot[h ? k : nh - 1u];
             },
             [&](int c, u32 w) -> int32_t {
               bool h;
               (void)hot_at(c, hot_lg, nh, h);
               const int32_t x = Ln[h ? 0 : c];
               return h ? (int32_t)w : x;
             },
             [&](int64_t b, const int32_t (&r)[8]) {
#pragma unroll
               for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(r[k], al + b + k * 64 + lane);
             },
             col, bB, nfull);
  // ---- the codes of the rows above ----
  __syncthreads();
  // (a multiple of 16 either way: ranked, 2^hc_lg >= 16 codes per slice)
  const u32 nc = kRanked ? (u32)((nslots >> slice_lg) << hc_lg)
                         : (u32)(nslots < 16 * kHotLabelsSingle ? nslots : 16 * kHotLabelsSingle);
  for (u32 q = threadIdx.x; q < nc / 16; q += 1024)
    hot[q] = code2[kRanked ? ((int64_t)(q >> (hc_lg - 4)) << (slice_lg - 4)) + (q & ((1u << (hc_lg - 4)) - 1u))
                           : (int64_t)q];
  __syncthreads();
  auto cp1 = [&](int c) -> u32 {
    bool h;
    const u32 k = hot_at(c, hc_lg, nc, h);
    const u32 cc = h ? k : nc - 1u;
    return (hot[cc >> 4] >> (((u32)c & 15u) * 2u)) & 3u;   // (k = c mod 16 where hot)
  };
  auto cp2 = [&](int c, u32 w) -> int32_t {
    bool h;
    (void)hot_at(c, hc_lg, nc, h);
    const u32 x = code2[h ? 0u : ((u32)c >> 4)];
    return (int32_t)(h ? w : ((x >> (((u32)c & 15u) * 2u)) & 3u));
  };
  range_pipe(cp1, cp2, [&](int64_t b, const int32_t (&r)[8]) { store_code2(al2, b, r, lane); }, col, 0, bA);
  // the partial last batch
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t t0 = nfull << 9;
  if (t0 < arcs && wv == nfull % nw) {
    int32_t r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t i = t0 + k * 64 + lane;
      r[k] = 0;
      if (i < arcs) {
        const u32 x = (u32)Ln[col[i]];
        if (i < p64) r[k] = (int32_t)giant_code2(x, G);
        else al[i] = (int32_t)x;
      }
    }
    if (t0 < p64) store_code2(al2, t0, r, lane);   // uniform; al2 covers this batch then
  }
}

// k_lpa_units_giant on the 2-bit giant codes (the refresh took them: gsel[5]): ugc[u] = the
// unit's code-0 (G) votes, umx[u] = its three other buckets' counts (k_hub_decide sums
// each over the row and takes the fullest: the row-level bucket test), by popcounts of
// its <= 33 code words (lane l: word l).  Units in batches of 64 per wave (one descriptor
// load per lane), the words of the next three units in flight.
__global__ __launch_bounds__(256) void k_lpa_units_code2(const uint32_t* __restrict__ al2,
                                                         const Segment* __restrict__ units, int64_t nunits,
                                                         const int32_t* __restrict__ gsel,
                                                         uint32_t* __restrict__ ugc, uint32_t* __restrict__ umx,
                                                         int32_t* __restrict__ ndec) {
  constexpr int D = 4;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) ndec[0] = ndec[2] = 0;  // unit list, block-row list
  if (gsel[5] == 0) return;  // k_lpa_units_giant's turn (uniform)
  if (gsel[1] == 0) return;  // no giant label worth trying: k_hub_decide lists every row
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t base = (int64_t)blockIdx.x * 4 + w; base < nunits; base += 64 * stride) {
    const int64_t uk = base + (int64_t)lane * stride;
    int64_t bk = 0;
    int32_t lk = 0;
    if (uk < nunits) {
      const Segment sg = units[uk];
      bk = sg.begin;
      lk = sg.len & 1023;
    }
    const int64_t left = (nunits - base + stride - 1) / stride;
    const int n = (int)(left < 64 ? left : 64);
    auto ld = [&](int q) -> u32 {
      const int64_t b = readlane_i64(bk, q);
      const int64_t e = b + __builtin_amdgcn_readlane(lk, q);
      const int64_t w0 = b >> 4, wl = e > b ? (e - 1) >> 4 : w0;
      const int64_t wi = w0 + lane;
      return al2[wi <= wl ? wi : wl];
    };
    u32 r[D];
#pragma unroll
    for (int k = 0; k < D - 1; ++k) r[k] = ld(k < n ? k : n - 1);
    for (int q0 = 0; q0 < n; q0 += D) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const int q = q0 + k;
        if (q >= n) break;  // uniform
        r[(k + D - 1) % D] = ld(q + D - 1 < n ? q + D - 1 : n - 1);
        const int64_t b = readlane_i64(bk, q);
        const int64_t e = b + __builtin_amdgcn_readlane(lk, q);
        u32 x = 0, y = 0;
        code2_counts(r[k], code2_fmask((b >> 4) + lane, b, e), x, y);
        x = wave_sum_u32(x);
        y = wave_sum_u32(y);
        if (lane == 0) {   // umx: the three bucket counts (<= 512 each), 10 bits apiece
          const int64_t id = base + (int64_t)q * stride;
          ugc[id] = x & 0xFFFFu;
          umx[id] = (x >> 16) | ((y & 0xFFFFu) << 10) | ((y >> 16) << 20);
        }
      }
    }
  }
}

// The code settle of one bin (supersteps 2 and 3 after a giant-code refresh): a row is
// decided for G from its al2 codes (G's votes above each of the three buckets) -- its
// label written, its dirty flag cleared -- or flagged (rdirty = 1) for its bin's list mode.
// Bodies take their share of the bin's rows as (bx, nbx): the blocks of one merged launch
// (k_code_settle) are split over the seven bins.
//   wave bins (64 < deg <= 1024, NC chunks): one wave per row, lane l the row's l-th code
//     word (NC = 16: and word l + 64), k_lpa_wave's schedule -- row bounds by 64-row
//     batches (span_batch), the words of the next D - 1 rows in flight
//   row bins of 8 < deg <= 64: one lane per row, its <= 5 words loaded at once
//   row bins of 8 < deg <= 64 (a cut at g8): one lane per row, its <= 5 words loaded at once
// Rows below the cut keep their labels (the refresh wrote them): their tasks are empty.
template <int NC>
__device__ __forceinline__ void code_settle_wave(const int64_t* __restrict__ rp, const uint32_t* __restrict__ al2,
                                                 int64_t vbeg, int64_t vend, int32_t G, int32_t* __restrict__ Ln,
                                                 uint8_t* __restrict__ rdirty, int64_t bx, int64_t nbx) {
  constexpr int NW = NC > 8 ? 2 : 1;   // a row of <= 64 NC arcs spans <= 4 NC + 1 words
  constexpr int D = 4;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  BinRows br;
  br.vbeg = vbeg;
  br.n = vend - vbeg;
  br.list = nullptr;
  const int64_t stride = nbx * 4;
  int64_t ib = bx * 4 + w;
  if (ib >= br.n) return;
  auto load = [&](u32 (&x)[NW], const RowSpan& r) {
    const int64_t w0 = r.b >> 4, wl = r.e > r.b ? (r.e - 1) >> 4 : w0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int64_t wi = w0 + k * 64 + lane;
      x[k] = al2[wi <= wl ? wi : wl];
    }
  };
  SpanBatch cur = span_batch(rp, br, ib, stride, lane), nxt;
  nxt.b = nxt.e = 0;
  nxt.v = 0;
  int p = 0;
  u32 rl[D][NW];
#pragma unroll
  for (int k = 0; k < D - 1; ++k) load(rl[k], span_at(cur, nxt, k));
  while (true) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      load(rl[(k + D - 1) % D], span_at(cur, nxt, p + D - 1));
      const RowSpan sp = span_at(cur, nxt, p);
      const int64_t v = (int64_t)__builtin_amdgcn_readlane(cur.v, p);
      u32 x = 0, y = 0;
#pragma unroll
      for (int c = 0; c < NW; ++c) {
        const int64_t wi = (sp.b >> 4) + c * 64 + lane;
        code2_counts(rl[k][c], code2_fmask(wi, sp.b, sp.e), x, y);
      }
      x = wave_sum_u32(x);
      y = wave_sum_u32(y);
      const bool settled = code2_decided(x, y);
      if (lane == 0) {
        if (settled) Ln[v] = G;
        rdirty[v] = settled ? 0 : 1;
      }
      if (ib + (int64_t)(p + 1) * stride >= br.n) return;
      ++p;
      if (p == 32) nxt = span_batch(rp, br, ib + 64 * stride, stride, lane);
      if (p == 64) {
        p = 0;
        ib += 64 * stride;
        cur = nxt;
      }
    }
  }
}

// W words per row: 5 for the row bins (<= 64 arcs), 9 for w2 (<= 128), 17 for w4 (<= 256)
// -- a lane per row issues all its words at once, so a wave has 64 rows' loads in flight
// where a wave per row had three (the w2 / w4 rows in code_settle_wave: latency-bound)
template <int W>
__device__ __forceinline__ void code_settle_rows(const int64_t* __restrict__ rp, const uint32_t* __restrict__ al2,
                                                 int64_t vbeg, int64_t vend, int32_t G, int32_t* __restrict__ Ln,
                                                 uint8_t* __restrict__ rdirty, int64_t bx, int64_t nbx) {
  for (int64_t v = vbeg + bx * 256 + threadIdx.x; v < vend; v += nbx * 256) {
    const int64_t b = rp[v], e = rp[v + 1];
    const int64_t w0 = b >> 4, wl = e > b ? (e - 1) >> 4 : w0;
    u32 wd[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wd[k] = al2[w0 + k <= wl ? w0 + k : wl];
    u32 x = 0, y = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) code2_counts(wd[k], code2_fmask(w0 + k, b, e), x, y);
    const bool settled = code2_decided(x, y);
    if (settled) Ln[v] = G;
    rdirty[v] = settled ? 0 : 1;
  }
}

// one launch for the seven settled bins (w16 .. w2, g64 .. g16): block b belongs to the
// task t with first[t] <= b < first[t + 1]; gword[6] = 0 (the bins' "fr_all" of
// superstep 2: lists) when a giant-code refresh was taken, 1 otherwise (and nothing else
// happens then)
struct CodeTasks {
  int64_t vbeg[7], vend[7];
  int32_t first[8];
};
__global__ __launch_bounds__(256) void k_code_settle(const int64_t* __restrict__ rp, const uint32_t* __restrict__ al2,
                                                     CodeTasks ct, int32_t* __restrict__ gword,
                                                     int32_t* __restrict__ Ln, uint8_t* __restrict__ rdirty) {
  const bool on = gword[5] != 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) gword[6] = on ? 0 : 1;
  if (!on) return;  // uniform
  const int32_t G = gword[0];
  int t = 0;
  while (t < 6 && (int32_t)blockIdx.x >= ct.first[t + 1]) ++t;
  const int64_t bx = (int64_t)blockIdx.x - ct.first[t], nbx = ct.first[t + 1] - ct.first[t];
  const int64_t vb = ct.vbeg[t], ve = ct.vend[t];
  switch (t) {
    case 0: code_settle_wave<16>(rp, al2, vb, ve, G, Ln, rdirty, bx, nbx); break;
    case 1: code_settle_wave<8>(rp, al2, vb, ve, G, Ln, rdirty, bx, nbx); break;
    case 2: code_settle_rows<17>(rp, al2, vb, ve, G, Ln, rdirty, bx, nbx); break;
    case 3: code_settle_rows<9>(rp, al2, vb, ve, G, Ln, rdirty, bx, nbx); break;
    default: code_settle_rows<5>(rp, al2, vb, ve, G, Ln, rdirty, bx, nbx); break;
  }
}

// al[i] = L[col[i]] over the arcs of the rows the code settle left (the lists of bins
// [b0, b1) of this superstep): a wave per row of the wave bins, 16 lanes per row of the
// row bins (<= 64 arcs: a whole wave per row left 3/4 of its lanes idle); a row's rounds
// are issued at once (the gathers are latency-bound: C4 superstep 2 9.01 -> 8.88 ms; a lane
// per row with eight rounds measured worse -- its column loads no longer coalesce: +0.8 ms)
__global__ __launch_bounds__(256) void k_code_partial_rows(const int32_t* __restrict__ gword,
                                                           const int64_t* __restrict__ rp,
                                                           const int32_t* __restrict__ col,
                                                           const int32_t* __restrict__ L, int32_t* __restrict__ al,
                                                           const int32_t* __restrict__ flist,
                                                           const int32_t* __restrict__ fcnt, BinBounds bb, int b0,
                                                           int b1) {
  if (gword[5] == 0) return;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bm = b1 < BIN_G64 ? b1 : BIN_G64;   // [b0, bm): wave bins; [bm, b1): row bins
  int64_t n1 = 0, n2 = 0;
  for (int b = b0; b < bm; ++b) n1 += fcnt[b];
  for (int b = bm; b < b1; ++b) n2 += fcnt[b];
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t i = (int64_t)blockIdx.x * 4 + w; i < n1; i += nw) {
    int64_t acc = 0;
    int b = b0;
    while (i >= acc + fcnt[b]) acc += fcnt[b++];
    const int64_t v = flist[bb.b[b] + (i - acc)];
    const int64_t s0 = rp[v], e = rp[v + 1];
    for (int64_t p0 = s0; p0 < e; p0 += 256) {   // uniform: four 64-arc rounds at once
      int32_t c[4], x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t p = p0 + k * 64 + lane;
        c[k] = col[p < e ? p : e - 1];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = L[c[k]];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t p = p0 + k * 64 + lane;
        if (p < e) al[p] = x[k];
      }
    }
  }
  // row bins: 16 lanes per row (coalesced column loads), its <= 4 rounds issued at once
  const int gq = lane >> 4, j = lane & 15;
  for (int64_t i0 = ((int64_t)blockIdx.x * 4 + w) * 4; i0 < n2; i0 += nw * 4) {
    const int64_t i = i0 + gq;
    if (i >= n2) continue;
    int64_t acc = 0;
    int b = bm;
    while (i >= acc + fcnt[b]) acc += fcnt[b++];
    const int64_t v = flist[bb.b[b] + (i - acc)];
    const int64_t s0 = rp[v], e = rp[v + 1];   // row bins hold 1..64 arcs
    if (e == s0) continue;
    int32_t c[4], x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t p = s0 + k * 16 + j;
      c[k] = col[p < e ? p : e - 1];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = L[c[k]];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t p = s0 + k * 16 + j;
      if (p < e) al[p] = x[k];
    }
  }
}

// ... and over the hub rows left undecided: listed rows (superstep 2: k_hub_decide's
// block-tier glist, count *nr) and listed units (superstep 2: its ulist2; superstep 3:
// the frontier unit list), one wave per row or unit
__global__ __launch_bounds__(256) void k_code_partial_hub(const int32_t* __restrict__ gword,
                                                          const int64_t* __restrict__ rp,
                                                          const int32_t* __restrict__ col,
                                                          const int32_t* __restrict__ L, int32_t* __restrict__ al,
                                                          const int32_t* __restrict__ rlist,
                                                          const int32_t* __restrict__ nrp,
                                                          const int32_t* __restrict__ ulst,
                                                          const int32_t* __restrict__ nup,
                                                          const Segment* __restrict__ segs) {
  if (gword[5] == 0) return;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nr = nrp ? *nrp : 0, total = nr + *nup;
  for (int64_t i = (int64_t)blockIdx.x * 4 + w; i < total; i += (int64_t)gridDim.x * 4) {
    int64_t b, e;
    if (i < nr) {
      const int64_t v = rlist[i];
      b = rp[v];
      e = rp[v + 1];
    } else {
      const Segment sg = segs[ulst[i - nr]];
      b = sg.begin;
      e = b + (sg.len & 1023);
    }
    for (int64_t p = b + lane; p < e; p += 64) al[p] = L[col[p]];
  }
}

// Superstep 3 after a giant-code refresh (the refresh after superstep 2; Chung-Lu, where
// L1 has no giant yet but L2 has one on the hubs): every hub row from its units' G counts
// and bucket bounds (k_lpa_units_code2), as k_hub_decide -- settled: the label, no
// dirty flag on the row or its units; otherwise every unit of the row is flagged (the
// combine merges a dirty row's every unit) -- one wave per row
__global__ __launch_bounds__(256) void k_code_settle_hubs(const int64_t* __restrict__ uoff,
                                                          const uint32_t* __restrict__ ugc,
                                                          const uint32_t* __restrict__ umx, int64_t n_hub,
                                                          const int32_t* __restrict__ gword, int32_t* __restrict__ Ln,
                                                          uint8_t* __restrict__ rdirty, uint8_t* __restrict__ udirty) {
  if (gword[5] == 0) return;  // uniform
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int32_t G = gword[0];
  for (int64_t h = (int64_t)blockIdx.x * 4 + w; h < n_hub; h += (int64_t)gridDim.x * 4) {
    const int64_t u0 = uoff[h], u1 = uoff[h + 1];
    u64 sg = 0, s1 = 0, s2 = 0, s3 = 0;   // umx: three bucket counts (k_lpa_units_code2)
    for (int64_t u = u0 + lane; u < u1; u += 64) {
      const u32 m = umx[u];
      sg += ugc[u];
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
    const bool settled = sg > s1 && sg > s2 && sg > s3;
    if (lane == 0) {
      if (settled) Ln[h] = G;
      rdirty[h] = settled ? 0 : 1;
    }
    const uint8_t f = settled ? 0 : 1;
    for (int64_t u = u0 + lane; u < u1; u += 64) udirty[u] = f;
  }
}

// superstep 3: a code settle ran -> list mode for the hub and wave bins (fr_all = 0), the
// diff scans every slot (settled rows changed), the row bins keep their ranges (gword[7]
// = 1, their al[] entries were written); otherwise the row bins follow fr_all
__global__ void k_code_commit(int32_t* __restrict__ fr_all, int32_t* __restrict__ gword, int32_t* __restrict__ fcnt) {
  if (threadIdx.x != 0) return;
  gword[7] = gword[5] ? 1 : *fr_all;
  if (gword[5]) {
    *fr_all = 0;
    fcnt[kFcntSettled] = 1;
  }
}

__global__ void k_gather_dense(const int32_t* __restrict__ L, const int32_t* __restrict__ new_of,
                               int64_t V, int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < V;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = L[new_of[i]];
}

// ---------------------------------------------------------------------------
// Superstep 1 from L0 (after a reset): L0 is injective, so two votes of a row carry
// the same label exactly when they come from the same column, and a row's columns
// are sorted: its vote counts are the lengths of its runs of equal columns
// (duplicate edges, a self-loop's two arcs).  The mode -- longest run, ties to the
// smallest label -- is a segmented max over the arc stream, with no hash table.
// A wave takes kRunTile-arc tiles (16 positions per lane); a row inside the tile is
// written directly, a row crossing a tile boundary folds each piece into
// first_best[row] and k_first_final writes it.
// ---------------------------------------------------------------------------

// One step of a segmented (by row id) inclusive max scan over the wave, in DPP: the
// lane's source (row shift within 16-lane rows, or a row broadcast) is moved by VALU
// lane permutes, no LDS; lanes without a source (or outside ROWMASK) see row
// INT_MIN and combine nothing.  Rows are contiguous lanes, so an equal row id at
// the source means every lane in between is the same row.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void seg_max_step(u64& w, int32_t r) {
  const int32_t ro = __builtin_amdgcn_update_dpp((int)0x80000000, r, kCtrl, kRowMask, 0xF, false);
  const u32 lo = (u32)__builtin_amdgcn_update_dpp(0, (int)(u32)w, kCtrl, kRowMask, 0xF, false);
  const u32 hi = (u32)__builtin_amdgcn_update_dpp(0, (int)(u32)(w >> 32), kCtrl, kRowMask, 0xF, false);
  const u64 wo = ((u64)hi << 32) | lo;
  if (ro == r && wo > w) w = wo;
}

// Inclusive wave scans in DPP: row_shr 1/2/4/8 inside each 16-lane row, then the
// row broadcasts of lanes 15 and 31 (lanes without a source combine the identity).
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ int dpp_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, kCtrl, kRowMask, 0xF, false);
}
__device__ __forceinline__ int wave_incl_add(int v) {
  v += dpp_i<0x111>(0, v);
  v += dpp_i<0x112>(0, v);
  v += dpp_i<0x114>(0, v);
  v += dpp_i<0x118>(0, v);
  v += dpp_i<0x142, 0xA>(0, v);
  v += dpp_i<0x143, 0xC>(0, v);
  return v;
}
__device__ __forceinline__ int wave_incl_max(int v) {
  constexpr int kMin = (int)0x80000000;
  v = max(v, dpp_i<0x111>(kMin, v));
  v = max(v, dpp_i<0x112>(kMin, v));
  v = max(v, dpp_i<0x114>(kMin, v));
  v = max(v, dpp_i<0x118>(kMin, v));
  v = max(v, dpp_i<0x142, 0xA>(kMin, v));
  v = max(v, dpp_i<0x143, 0xC>(kMin, v));
  return v;
}

// Lane-sequential layout: lane l of a wave owns positions t0 + kP l .. t0 + kP l + kP - 1
// of its tile (kP / 4 16-B loads), walks them in registers (run lengths, the row's
// running maximum, rows that start and end inside the lane written at once), and
// only the lane-crossing parts go through cross-lane scans -- three per tile instead
// of a segmented scan per 64 arcs (the per-arc-lane form was VALU-bound: ~190
// instructions per 64 arcs, 1.34 ms at C3 against 0.27 ms of al[] stream).
//   row ids   crow[t0] + the row starts in (t0, p] (a prefix sum of the lanes' start
//             counts from the row-start bitmap; crow is read once per tile)
//   runs      a run starts at a row start or a label change; the run in progress at
//             a lane's first position started at the last run start of the lanes
//             before (a max scan), or ck positions before the tile
//   rows      a row ending inside the lane after starting in it is complete; the
//             lane's first and last segments combine with their neighbours through a
//             segmented (by row) max scan of the lanes' last segments
// Positions at or past arcs count as row starts (so the last row ends at arcs - 1) and
// hold no votes: their empty segments write nothing.
typedef int v4i_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_first_runs(const int32_t* __restrict__ al,
                                                    const int32_t* __restrict__ crow,
                                                    const u64* __restrict__ rstart, int64_t arcs,
                                                    int32_t* __restrict__ Ln, u64* __restrict__ best) {
  constexpr int kP = kRunTile / 64;  // positions per lane
  static_assert(kP % 4 == 0 && kP <= 32 && 64 % kP == 0, "whole 16-B loads, one bitmap field per lane");
  constexpr u32 kPMask = kP == 32 ? 0xFFFFFFFFu : (1u << kP) - 1u;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int64_t t0 = ((int64_t)blockIdx.x * 4 + wv) * kRunTile; t0 < arcs; t0 += nw * kRunTile) {
    const int64_t t1 = t0 + kRunTile < arcs ? t0 + kRunTile : arcs;
    const int64_t p0 = t0 + kP * lane;
    u32 a[kP];
    if (p0 + kP <= t1) {
      const v4i_t* q = reinterpret_cast<const v4i_t*>(al + p0);  // 16-B aligned: t0 % kRunTile == 0
#pragma unroll
      for (int v = 0; v < kP / 4; ++v) {
        const v4i_t x = __builtin_nontemporal_load(q + v);
        a[4 * v] = (u32)x.x; a[4 * v + 1] = (u32)x.y; a[4 * v + 2] = (u32)x.z; a[4 * v + 3] = (u32)x.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kP; ++j) a[j] = p0 + j < t1 ? (u32)al[p0 + j] : kNone;
    }
    // row-start bits of the lane's positions (bit j: p0 + j), positions >= arcs set
    u32 sb = (u32)(rstart[(t0 >> 6) + (lane * kP) / 64] >> ((lane * kP) % 64)) & kPMask;
    const int64_t dead = p0 + kP - arcs;
    if (dead > 0) sb |= dead >= kP ? kPMask : (kPMask << (kP - (int)dead)) & kPMask;
    // does position p0 + kP start a row (the next lane's bit 0; lane 63: the next tile's)
    const int tile_next = t0 + kRunTile >= arcs ? 1 : (int)(rstart[(t0 + kRunTile) >> 6] & 1ull);
    const bool ends = (dpp_i<0x130>(tile_next, (int)(sb & 1u)) & 1) != 0;  // wave_shl:1
    // carries from before the tile: row, label and (a run continuing into it) length
    const int32_t r_t0 = crow[t0];
    int32_t r_before = -1;
    u32 ca = kNone, ck = 0u;
    if (t0 > 0) {
      r_before = crow[t0 - 1];
      ca = (u32)al[t0 - 1];
      if (r_t0 == r_before && (u32)__builtin_amdgcn_readfirstlane((int)a[0]) == ca) {
        int64_t k = 1;  // a run continues into the tile (rare): its length up to t0 - 1
        while (t0 - 1 - k >= 0 && crow[t0 - 1 - k] == r_before && (u32)al[t0 - 1 - k] == ca) ++k;
        ck = (u32)k;
      }
    }
    // row of the position before the lane (lane 0: position t0's row; its start bit
    // is not a new row inside the tile)
    const u32 sbr = lane == 0 ? (sb & ~1u) : sb;
    const int nst = __popc(sbr);
    int32_t rr = r_t0 + wave_incl_add(nst) - nst;
    // run starts, and where the run in progress at the lane's first position started
    // (relative to t0; lane 0 without a start of its own: -ck)
    const u32 aprev = (u32)dpp_i<0x138>((int)ca, (int)a[kP - 1]);  // wave_shr:1
    u32 rsb = sb;
    rsb |= a[0] != aprev ? 1u : 0u;
#pragma unroll
    for (int j = 1; j < kP; ++j) rsb |= a[j] != a[j - 1] ? (1u << j) : 0u;
    const int pl = kP * lane;
    const int last_rs = rsb ? pl + 31 - __clz(rsb) : (lane == 0 ? -(int)ck : (int)0x80000000);
    int cur = dpp_i<0x138>(-(int)ck, wave_incl_max(last_rs));
    // the lane's positions in order
    u64 acc = 0ull, fw = 0ull;
    bool multi = false;  // a segment ended inside the lane: fw holds the first one
    int32_t rfirst = 0;
#pragma unroll
    for (int j = 0; j < kP; ++j) {
      if ((sbr >> j) & 1u) {
        if (j > 0) {
          if (!multi) {
            fw = acc;
            multi = true;
          } else if (acc) {
            Ln[rr] = (int32_t)(~(u32)acc);  // started and ended inside the lane
          }
        }
        ++rr;
        acc = 0ull;
      }
      if (j == 0) rfirst = rr;
      if ((rsb >> j) & 1u) cur = pl + j;
      if (a[j] != kNone) {
        const u64 w = ((u64)(u32)(pl + j - cur + 1) << 32) | (u64)(~a[j]);
        acc = w > acc ? w : acc;
      }
    }
    // segmented (by row) inclusive max of the lanes' last segments
    u64 T = acc;
    seg_max_step<0x111, 0xF>(T, rr);
    seg_max_step<0x112, 0xF>(T, rr);
    seg_max_step<0x114, 0xF>(T, rr);
    seg_max_step<0x118, 0xF>(T, rr);
    seg_max_step<0x142, 0xA>(T, rr);
    seg_max_step<0x143, 0xC>(T, rr);
    // the lane's first segment, ended inside the lane: plus the lanes before in its row
    const int32_t rprev = dpp_i<0x138>((int)0x80000000, rr);
    const u32 tlo = (u32)dpp_i<0x138>(0, (int)(u32)T), thi = (u32)dpp_i<0x138>(0, (int)(u32)(T >> 32));
    if (multi) {
      const u64 tp = ((u64)thi << 32) | tlo;
      const u64 v = rprev == rfirst && tp > fw ? tp : fw;
      if (v) {
        if (rfirst == r_before) atomicMax(&best[rfirst], v);  // started before the tile
        else Ln[rfirst] = (int32_t)(~(u32)v);
      }
    }
    // the lane's last segment: ends at the lane's end, or (lane 63) continues in the
    // next tile
    if (T && (ends || lane == 63)) {
      if (!ends || rr == r_before) atomicMax(&best[rr], T);
      else Ln[rr] = (int32_t)(~(u32)T);
    }
  }
}

// rows that cross a run tile: label from the folded maximum (reset for the next
// use); both parities' hub queue counters start from zero (superstep 1 skips the
// hub combine, whose last kernel otherwise resets the next parity's)
__global__ void k_first_final(const int64_t* __restrict__ rp, int64_t S, u64* __restrict__ best,
                              int32_t* __restrict__ Ln, int32_t* __restrict__ hub_lcnt) {
  if (hub_lcnt && blockIdx.x == 0 && threadIdx.x < 16) hub_lcnt[threadIdx.x] = 0;  // null: no hub rows
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < S;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = rp[r], e = rp[r + 1];
    if (e > b && b / kRunTile != (e - 1) / kRunTile) {
      Ln[r] = (int32_t)(~(u32)best[r]);
      best[r] = 0ull;
    }
  }
}

inline unsigned cap_grid(int64_t want, int64_t cap) {
  if (want < 1) want = 1;
  return (unsigned)(want < cap ? want : cap);
}

// tally kernels of one superstep; bev marks: 0 start, k+1 after kernel k
// (0 seg, 1 hub_final + hub_write, 2 wave, 3..7 g16..g1)
// Tally kernels of one superstep on three streams (the bins write disjoint
// label ranges and only read al[]): main = seg units -> hub combine, aux0 = the
// wave bins, aux1 = the row/group bins; they join on the main stream.  Running
// them concurrently hides the ~2-5 us launch gap of each dependent kernel and the
// tails of the small bins.  bev (nullable): events 2k / 2k+1 bracket tally kernel
// k on its own stream (0 units, 1 hub combine, 2..11 bins w8 .. g1).
int launch_diff(lpa_graph* g, hipStream_t st, const int32_t* Lc, const int32_t* Ln, int64_t s0,
                int64_t s1, bool sync, int par, int b0 = 0, int b1 = 0, int mode = 0);

// diff (P = 1, concurrent schedule): each stream diffs the slots its own bins
// produced right after them (aux0 w16..w4, aux1 w2..g1 + isolated, main the seg
// rows after the hub combine), overlapping most of the diff with the tally tail
// the per-bin dirty-row lists of this superstep (zeroes the other parity's counts)
// Gather mode (lpa_build: small label vector, no row above 128 arcs -- C2) for the first
// kGatherSteps supersteps: their tallies read L[col[i]] (arc_vote), no al[] is written
// (the scatter only marks the frontier), and the last of them rebuilds al once, for the
// later supersteps, whose cheaper tallies beat the gathers (C2, same box: label-dense
// supersteps 0.42-0.49 -> 0.34-0.37 ms gathering, converged ones 0.16-0.22 ms from al[]
// against 0.25-0.30 gathering; LPA_GATHER_STEPS=99, every superstep gathering, re-measured:
// supersteps 2-10 2.84 against 2.65 ms)
#ifndef LPA_GATHER_STEPS
#define LPA_GATHER_STEPS 6
#endif
constexpr int kGatherSteps = LPA_GATHER_STEPS;
bool gather_now(const lpa_graph* g) { return g->gather && g->since_reset < kGatherSteps; }
int launch_frontier_lists(lpa_graph* g, hipStream_t st = nullptr, const int32_t* fr = nullptr) {
  if (!st) st = g->stream;
  if (!fr) fr = g->fr_all + g->par;
  BinBounds bnd;
  for (int b = 0; b <= LPA_NBINS; ++b) bnd.b[b] = g->bin_begin[b];
  const int64_t nbr = (g->slice + kListTile - 1) / kListTile;
  const int64_t nbu = (g->n_segs + kListTile - 1) / kListTile;
  hipLaunchKernelGGL(k_frontier_lists, dim3((unsigned)(nbr + nbu)), dim3(256), 0, st, g->rdirty[g->par],
                     g->slice, g->udirty[g->par], g->n_segs, bnd, fr, g->flist, g->ulist,
                     g->fcnt + 16 * g->par, g->fcnt + 16 * (g->par ^ 1), nbr);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// label-dense superstep: its diff only counts the changed slots, and its refresh
// rebuilds al[] unless few changed (k_dense_decide).  P > 1: the count runs after the
// exchange over the whole replicated vector (launch_refresh), P = 1 per stream inside
// the tally
bool dense_refresh(const lpa_graph* g) { return g->since_reset < kDenseSupersteps; }

// superstep 1 from L0 by column runs (k_first_runs); the caller's refresh diffs
bool first_runs_now(const lpa_graph* g) {
  return g->first_runs && g->cols_sorted && g->first_best && g->rstart && g->since_reset == 0 && g->arcs > 0 &&
         !g->serial;
}

int launch_first(lpa_graph* g, int32_t* Lown) {
  hipStream_t s = g->stream;
  LPA_TRY(launch_frontier_lists(g));
  const int64_t ntiles = (g->arcs + kRunTile - 1) / kRunTile;
  // after a lazy reset the L0 arc labels are in al0 (al is rebuilt by the refresh)
  hipLaunchKernelGGL(k_first_runs, dim3(cap_grid((ntiles + 3) / 4, 8192)), dim3(256), 0, s,
                     g->al_pending ? g->al0 : g->al, g->crow, g->rstart, g->arcs, Lown, g->first_best);
  LPA_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_first_final, dim3(cap_grid((g->slice + 255) / 256, 4096)), dim3(256), 0, s, g->rp,
                     g->slice, g->first_best, Lown, g->hub_lcnt);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// the refresh after superstep 1 or 2 may take the giant codes (after superstep 1 on
// R-MAT, after superstep 2 on Chung-Lu: the first label vector whose giant carries the
// hubs without holding half the hot slots).  Round 6: on every rank of a partitioned job
// too -- the refresh follows the exchange, so it codes the replicated vector, and G (picked
// from it) is the same on every rank; each rank codes and settles its own rows
bool code_refresh_now(const lpa_graph* g) { return g->code_ok && g->since_reset <= 1; }
// ... and superstep 2 (block mode) or 3 then settles from them
bool code_tally_now(const lpa_graph* g) { return g->code_ok && g->since_reset == 1; }
bool code_tally3_now(const lpa_graph* g) { return g->code_ok && g->since_reset == 2 && g->code3; }

// the code settle of the seven settled bins in one launch (k_code_settle; it returns at
// once unless a giant-code refresh was taken): blocks split over the bins by work (a
// wave bin's row: a wave; a row bin's row: a lane and its <= 5 word loads), at most one
// row per wave (wave bins) or lane (row bins)
int launch_code_settle(lpa_graph* g, hipStream_t st, int32_t* Lown) {
  const int64_t* bb = g->bin_begin;
  const int bins[7] = {BIN_W16, BIN_W8, BIN_W4, BIN_W2, BIN_G64, BIN_G32, BIN_G16};
  const int lanes[7] = {64, 64, 16, 8, 4, 4, 4};   // work per row: a wave; a lane's W loads
  CodeTasks ct;
  int64_t work[7], tot = 0;
  for (int t = 0; t < 7; ++t) {
    ct.vbeg[t] = bb[bins[t]];
    ct.vend[t] = bins[t] < g->code_lbin ? bb[bins[t] + 1] : bb[bins[t]];   // labelled bins: no rows
    work[t] = (ct.vend[t] - ct.vbeg[t]) * lanes[t];
    tot += work[t];
  }
#ifndef LPA_CODE_SETTLE_BLOCKS
#define LPA_CODE_SETTLE_BLOCKS 4096
#endif
  const int64_t kBlocks = LPA_CODE_SETTLE_BLOCKS;   // 16 waves per CU
  ct.first[0] = 0;
  for (int t = 0; t < 7; ++t) {
    int64_t nb = tot > 0 ? (work[t] * kBlocks + tot - 1) / tot : 0;
    const int64_t rows = ct.vend[t] - ct.vbeg[t];
    const int64_t need = t < 2 ? (rows + 3) / 4 : (rows + 255) / 256;
    if (nb > need) nb = need;
    if (work[t] > 0 && nb < 1) nb = 1;
    ct.first[t + 1] = ct.first[t] + (int32_t)nb;
  }
  hipLaunchKernelGGL(k_code_settle, dim3((unsigned)(ct.first[7] > 0 ? ct.first[7] : 1)), dim3(256), 0, st, g->rp,
                     g->al2, ct, g->gword, Lown, g->rdirty[g->par]);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

int launch_tally(lpa_graph* g, int32_t* Lown, hipEvent_t* bev, const int32_t* Lc,
                 const int32_t* Ln, bool diff) {
  hipStream_t s = g->stream;
  // LPA_SERIAL=1 (profiling only): every tally kernel on the main stream, so a
  // kernel trace shows each kernel's standalone duration
  // (three streams in every superstep, the converged ones too: 2 or 1 measured slower,
  // the bin chains' overlap is worth more than the fork / join dependencies)
  // (converged supersteps with the frontier on: g->conv_streams, LPA_CONV_STREAMS --
  // their captured graphs pay a cross-queue dependency per node, ~3.5 us, where a
  // one-queue chain pays ~1.9: tools/microbench/mb_launch.hip.  With the frontier off
  // every superstep tallies every row, and the bins' overlap on three streams pays)
  const bool conv = g->since_reset >= kDenseSupersteps + 2 && g->frontier;
  const int nstr = g->serial ? 1 : conv ? g->conv_streams : 3;
  hipStream_t sb = nstr >= 2 ? g->aux_stream[0] : s;
  hipStream_t sc = nstr >= 3 ? g->aux_stream[1] : sb;
  const int64_t* bb = g->bin_begin;
  const int32_t* fr_all = g->fr_all + g->par;
  int32_t* fcnt = g->fcnt + 16 * g->par;
  // supersteps 2-4 (the label-dense ones after the column-run superstep 1): the tallies
  // try the giant label first (giant_decide); gsel = its word, picked by the previous
  // superstep's refresh from the labels this one reads
  const int32_t* gsel = (g->since_reset >= 1 && g->since_reset <= 3) ? g->gword : nullptr;
  if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv + 4], s));
  // superstep 3: rows settled from the arc giant bits of superstep 2's rebuild (each
  // kernel returns at once unless they are valid): the others' dirty flags, then the
  // lists of this superstep are built from them in list mode
  // superstep 4 (one GPU): the same settle for the rows below the hubs, from a fresh
  // abits pass, on aux0 while the main stream re-tallies every hub unit and row (range
  // mode: their staged words are current again for the frontier supersteps); the bins
  // below the hubs then walk their unsettled rows' lists (fr_bins = gword[4])
  // (P > 1: each rank settles its owned rows from its own arc giant bits; G is the same
  // on every rank, k_giant_pick reads the replicated vector)
  const bool settle4 = g->since_reset == 3 && g->abits != nullptr && !gather_now(g);  // its abits come from al
  const int32_t* fr_bins = settle4 ? g->gword + 4 : fr_all;
  if (settle4) {
    if (!g->serial) {
      LPA_HIP(hipEventRecord(g->ev_fork, s));
      LPA_HIP(hipStreamWaitEvent(sb, g->ev_fork, 0));
    }
    const int64_t p0 = g->bin_arcs[0];
    const int64_t nwd = (g->arcs + 63) / 64 - p0 / 64;
    hipLaunchKernelGGL(k_abits_pass, dim3(cap_grid((nwd + 31) / 32, 8192)), dim3(256), 0, sb, g->al, p0, g->arcs,
                       g->gword, g->abits);
    LPA_HIP(hipGetLastError());
    const int64_t r0 = g->n_hub, r1 = g->bin_begin[BIN_ISO];
    if (r1 > r0) {
      hipLaunchKernelGGL(k_settle_rows, dim3(cap_grid((r1 - r0 + 255) / 256, 8192)), dim3(256), 0, sb, g->rp,
                         g->abits, r0, r1, fr_all, g->gword, Lown, g->rdirty[g->par]);
      LPA_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_settle_commit4, dim3(1), dim3(1), 0, sb, fr_all, g->gword);
    LPA_HIP(hipGetLastError());
    LPA_TRY(launch_frontier_lists(g, sb, fr_bins));
    if (!g->serial) {
      LPA_HIP(hipEventRecord(g->ev_join2[2], sb));
      LPA_HIP(hipStreamWaitEvent(sc, g->ev_join2[2], 0));
    }
  } else {
    // superstep 3: rows settled from the arc giant bits of superstep 2's rebuild (each
    // kernel returns at once unless they are valid): the others' dirty flags, then the
    // lists of this superstep are built from them in list mode
    if (g->since_reset == 2 && g->abits && !block_mode_now(g) && !code_tally3_now(g)) {
      const int64_t r0 = g->n_hub, r1 = g->bin_begin[BIN_ISO];
      // the hub rows (main) and the rows below them (aux0) settle side by side: disjoint
      // rows, both read only abits; joined before the commit
      const bool fork_settle = sb != s && g->n_hub > 0 && r1 > r0;
      if (fork_settle) {
        LPA_HIP(hipEventRecord(g->ev_fork, s));
        LPA_HIP(hipStreamWaitEvent(sb, g->ev_fork, 0));
      }
      if (g->n_hub > 0) {
        hipLaunchKernelGGL(k_settle_big, dim3(cap_grid((g->n_hub + 3) / 4, 2048)), dim3(256), 0, s, g->rp,
                           g->abits, g->n_hub, fr_all, g->gword, Lown, g->rdirty[g->par], g->udirty[g->par],
                           g->hub_uoff);
        LPA_HIP(hipGetLastError());
      }
      if (r1 > r0) {
        hipLaunchKernelGGL(k_settle_rows, dim3(cap_grid((r1 - r0 + 255) / 256, 8192)), dim3(256), 0,
                           fork_settle ? sb : s, g->rp, g->abits, r0, r1, fr_all, g->gword, Lown,
                           g->rdirty[g->par]);
        LPA_HIP(hipGetLastError());
      }
      if (fork_settle) {
        LPA_HIP(hipEventRecord(g->ev_join2[2], sb));
        LPA_HIP(hipStreamWaitEvent(s, g->ev_join2[2], 0));
      }
      hipLaunchKernelGGL(k_settle_commit, dim3(1), dim3(1), 0, s, const_cast<int32_t*>(fr_all), g->gword, fcnt);
      LPA_HIP(hipGetLastError());
    }
    if (code_tally3_now(g)) {
      // superstep 3 after a giant-code refresh (each kernel returns at once otherwise):
      // hub rows from their units' code counts, wave-bin rows from their codes; the rest
      // listed (k_code_commit: list mode), their al[] entries gathered after the lists
      if (g->n_segs > 0) {
        hipLaunchKernelGGL(k_lpa_units_code2, dim3(cap_grid((g->n_segs + 3) / 4, 2048)), dim3(256), 0, s,
                           g->al2, g->segs, g->n_segs, g->gword, g->ugc, g->umx, g->gdec);
        LPA_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_code_settle_hubs, dim3(cap_grid((g->n_hub + 3) / 4, 2048)), dim3(256), 0, s,
                           g->hub_uoff, g->ugc, g->umx, g->n_hub, g->gword, Lown, g->rdirty[g->par],
                           g->udirty[g->par]);
        LPA_HIP(hipGetLastError());
      }
      LPA_TRY(launch_code_settle(g, s, Lown));
      hipLaunchKernelGGL(k_code_commit, dim3(1), dim3(64), 0, s, const_cast<int32_t*>(fr_all), g->gword, fcnt);
      LPA_HIP(hipGetLastError());
    }
    // frontier lists of this superstep (no-op when every row is tallied)
    LPA_TRY(launch_frontier_lists(g));
    if (code_tally3_now(g)) {
      BinBounds bnd;
      for (int b = 0; b <= LPA_NBINS; ++b) bnd.b[b] = bb[b];
      hipLaunchKernelGGL(k_code_partial_rows, dim3(2048), dim3(256), 0, s, g->gword, g->rp, g->col, Lc, g->al,
                         g->flist, fcnt, bnd, (int)BIN_W16, (int)g->code_lbin);
      LPA_HIP(hipGetLastError());
      hipLaunchKernelGGL(k_code_partial_hub, dim3(2048), dim3(256), 0, s, g->gword, g->rp, g->col, Lc, g->al,
                         (const int32_t*)nullptr, (const int32_t*)nullptr, g->ulist, fcnt + kFcntUnits, g->segs);
      LPA_HIP(hipGetLastError());
    }
  }
  // the wave bins' "fr_all": superstep 2 after a giant-code refresh walks the lists above;
  // the row bins': superstep 3's code commit keeps them in range mode (gword[7])
  const int32_t* fr_wave = code_tally_now(g) ? g->gword + 6 : fr_bins;
  // the labelled row bins of a code refresh (from code_lbin on) take their ranges (superstep
  // 3 after one: gword[7], k_code_commit); coded row bins below it follow the wave bins
  const int32_t* fr_rows = code_tally3_now(g) ? g->gword + 7 : fr_bins;
  auto fr_row = [&](int bin) { return bin < g->code_lbin ? fr_wave : fr_rows; };
  if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv + 5], s));
  if (sb != s) {
    LPA_HIP(hipEventRecord(g->ev_fork, s));
    LPA_HIP(hipStreamWaitEvent(sb, g->ev_fork, 0));
    if (sc != sb) LPA_HIP(hipStreamWaitEvent(sc, g->ev_fork, 0));
  }
  if (code_tally_now(g)) {
    // superstep 2 after a giant-code refresh (each kernel returns at once otherwise,
    // leaving the wave bins in range mode): the wave-bin rows settled from their codes,
    // the others listed, their al[] entries gathered -- on the wave bins' stream, which
    // then tallies them (w2 included), beside the hub path on main and the row bins on
    // the third stream (they read neither the flags nor those al[] entries)
    LPA_TRY(launch_code_settle(g, sb, Lown));
    LPA_TRY(launch_frontier_lists(g, sb, g->gword + 6));
    BinBounds bnd;
    for (int b = 0; b <= LPA_NBINS; ++b) bnd.b[b] = bb[b];
    hipLaunchKernelGGL(k_code_partial_rows, dim3(2048), dim3(256), 0, sb, g->gword, g->rp, g->col, Lc, g->al,
                       g->flist, fcnt, bnd, (int)BIN_W16, (int)g->code_lbin);
    LPA_HIP(hipGetLastError());
    // coded row bins (a cut below g64) on the third stream walk these lists: they wait
    if (sc != sb && g->code_lbin > BIN_G64) LPA_HIP(hipEventRecord(g->ev_join2[2], sb));
  }

  auto mark = [&](int i, hipStream_t st) -> int {
    if (bev) LPA_HIP(hipEventRecord(bev[i], st));
    return LPA_OK;
  };
  // label-dense supersteps: the rows of <= kBlockMaxDeg arcs by k_lpa_block, only
  // the longer rows' units by k_lpa_units (block_mode_now)
  const bool blk = block_mode_now(g);
  // peel rounds of the wave / unit / block tallies (LPA_DENSE_PEEL in the label-dense
  // supersteps, where a round rarely retires more than a few votes)
  const int pmax = g->since_reset < kDenseSupersteps ? kDensePeel : kPeelMax;
  // peel rounds of the row bins (range mode) before a chunk is hashed: none in the
  // label-dense supersteps (measured best of 0/1/2/3 at C3), one in supersteps 3 and 4
  // (C2's rows are still label-dense there: 0.59 -> 0.52 ms each; both are launched
  // eagerly, so no captured graph bakes the value), kPeelSortAfter after that (1 there:
  // C3's converged supersteps +10 %)
  const int sort_after = g->since_reset < kDenseSupersteps ? 0 : g->since_reset <= 3 ? 1 : kPeelSortAfter;
  // superstep 2 in block mode: every hub row by giant counts first (k_lpa_units_giant
  // over all units, k_hub_decide); only the rows it cannot settle are tallied exactly --
  // block-tier rows by k_lpa_block from glist, the longer ones by their units
  const bool giant_units = gsel != nullptr && block_mode_now(g);
  // the block tiers' rows: in giant mode the undecided ones (glist, count gdec[2]; all
  // of them when G was not worth trying: gdec[3] as "fr_all"), else the superstep's
  // rows or frontier list
  const int32_t* blist = giant_units ? g->glist : g->flist;
  const int32_t* bcnt = giant_units ? g->gdec + 2 : fcnt;
  const int32_t* ball = giant_units ? g->gdec + 3 : fr_all;
  // (the block tiers' giant step is then done: no gsel for them)
  const int32_t* bsel = giant_units ? nullptr : gsel;
  // wide tier (rows 4096 < deg <= 8192: 16 waves, a 16K-slot table, one block per CU)
  auto launch_block_wide = [&](hipStream_t st) -> int {
    const int64_t h2 = g->hub_block2_begin, hl = g->hub_lane_begin;
    if (hl > h2) {
      // (giant mode: the undecided rows only; a grid sized to few rows measured slower
      // at C5, superstep 2 48.7 -> 54.3 ms, and the same at C3)
      hipLaunchKernelGGL((k_lpa_block<14, kBlockMaxDeg2 / kSegArcs>), dim3(cap_grid(hl - h2, 1024)),
                         dim3(kBlockMaxDeg2 / kSegArcs * 64), 0, st, g->rp, g->al, Lown, h2, hl, blist, bcnt,
                         ball, pmax, bsel);
      LPA_HIP(hipGetLastError());
    }
    return LPA_OK;
  };
  // rows <= 4096 (8 waves, 8K slots, two blocks per CU)
  auto launch_block_narrow = [&](hipStream_t st) -> int {
    const int64_t nb = g->n_hub - g->hub_lane_begin;
    hipLaunchKernelGGL((k_lpa_block<13, kBlockMaxDeg / kSegArcs>), dim3(cap_grid(nb, 2048)),
                       dim3(kBlockMaxDeg / kSegArcs * 64), 0, st, g->rp, g->al, Lown, g->hub_lane_begin, g->n_hub,
                       blist, bcnt, ball, pmax, bsel);
    LPA_HIP(hipGetLastError());
    return LPA_OK;
  };
  auto launch_block = [&](hipStream_t st) -> int {
    if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv + 6], st));
    LPA_TRY(launch_block_wide(st));
    LPA_TRY(launch_block_narrow(st));
    if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv + 7], st));
    return LPA_OK;
  };
  // split (the concurrent schedule): the longest pole of a label-dense superstep is the
  // main stream's block tiers + units + hub combine, so the wide tier goes to the
  // fourth stream and the narrow tier follows the hub mid tiers on the main stream
  // (C3 293.8-295.4 -> 299.3-303.1 GTEPS over the block tiers first on the main stream)
  const bool split = blk && !g->serial;
  if (split && !giant_units) {
    LPA_HIP(hipStreamWaitEvent(g->aux_stream[2], g->ev_fork, 0));
    LPA_TRY(launch_block_wide(g->aux_stream[2]));
    LPA_HIP(hipEventRecord(g->ev_join2[1], g->aux_stream[2]));
  }
  const int64_t n_units = blk ? g->unit_block2_begin : g->n_segs;
  // the main stream's unit work (the hub path's head): enqueued before the bins in the
  // converged supersteps, after them in supersteps 2-4.  The streams share hardware queues
  // (GPU_MAX_HW_QUEUES = 4), so the enqueue order decides what waits behind what: with
  // the units last the row bins no longer queue behind the hub path in the label-dense
  // supersteps (same box: C3 superstep 2 1.87 -> 1.71 ms, C4 9.28 -> 8.89, C5 28.75 ->
  // 28.14), while the converged supersteps, whose critical path is the hub path, lost
  // 8-15 us each that way
  const bool units_last = !g->serial && g->since_reset >= 1 && g->since_reset <= 3;
  auto launch_units = [&]() -> int {
    if (giant_units && g->n_segs > 0) {
      hipLaunchKernelGGL(k_lpa_units_giant<int32_t>, dim3(cap_grid((g->n_segs + 3) / 4, 2048)), dim3(256), 0, s,
                         g->al, g->segs, g->n_segs, gsel, g->ugc, g->umx, g->gdec);
      LPA_HIP(hipGetLastError());
      if (code_tally_now(g)) {  // the form on the giant codes (one of the two returns at once)
        hipLaunchKernelGGL(k_lpa_units_code2, dim3(cap_grid((g->n_segs + 3) / 4, 2048)), dim3(256), 0, s,
                           g->al2, g->segs, g->n_segs, gsel, g->ugc, g->umx, g->gdec);
        LPA_HIP(hipGetLastError());
      }
      LPA_TRY(launch_hub_decide(g, Lown, g->n_hub, gsel));
      if (code_tally_now(g)) {  // the undecided hub rows' al[] entries (code refresh only)
        hipLaunchKernelGGL(k_code_partial_hub, dim3(2048), dim3(256), 0, s, g->gword, g->rp, g->col, Lc, g->al,
                           g->glist, g->gdec + 2, g->ulist2, g->gdec, g->segs);
        LPA_HIP(hipGetLastError());
      }
      // the wide tier's few undecided rows right here on the main stream (the fourth
      // stream shares a hardware queue with aux1, whose row bins it would delay)
      if (split) LPA_TRY(launch_block_wide(s));
    }
    // serialized profiling: the block kernel bracketed on its own (stats kernel 16),
    // ahead of the seg units' marks
    if (blk && g->serial) LPA_TRY(launch_block(s));
    LPA_TRY(mark(0, s));
    if (n_units > 0 && giant_units) {
      hipLaunchKernelGGL(k_lpa_units, dim3(cap_grid((n_units + 3) / 4, 2048)), dim3(256), 0, s,
                         g->al, g->segs, n_units, g->stage, g->ucnt, g->ulist2, g->gdec, g->gdec + 3, pmax);
      LPA_HIP(hipGetLastError());
    } else if (n_units > 0 && settle4 && g->units_pure) {
      // superstep 4: the pure-G units staged without a tally, the others listed
      const int64_t npb = std::max<int64_t>((n_units + 2047) / 2048, 32);  // units per block
      hipLaunchKernelGGL(k_units_pure, dim3((unsigned)((n_units + std::min<int64_t>(npb, kPureIds) - 1) /
                                                       std::min<int64_t>(npb, kPureIds))), dim3(256), 0, s, g->al,
                         g->abits, g->arcs, g->segs, n_units, g->gword, g->stage, g->ucnt, g->ulist2);
      LPA_HIP(hipGetLastError());
      hipLaunchKernelGGL(k_lpa_units, dim3(cap_grid((n_units + 3) / 4, 2048)), dim3(256), 0, s,
                         g->al, g->segs, n_units, g->stage, g->ucnt, g->ulist2, g->gword + 11, g->gword + 10, pmax);
      LPA_HIP(hipGetLastError());
    } else if (n_units > 0) {
      hipLaunchKernelGGL(k_lpa_units, dim3(cap_grid((n_units + 3) / 4, 2048)), dim3(256), 0, s,
                         g->al, g->segs, n_units, g->stage, g->ucnt, g->ulist, fcnt + kFcntUnits, fr_all, pmax);
      LPA_HIP(hipGetLastError());
      LPA_TRACE_POINT("seg");
    }
    LPA_TRY(mark(1, s));
    return LPA_OK;
  };
  if (!units_last) LPA_TRY(launch_units());
  // gather mode (lpa_build): the votes are Lc[col[i]] -- the kernels read col and Lc
  const bool gnow = gather_now(g);
  const int32_t* vsrc = gnow ? g->col : g->al;
#define LPA_WAVE_LAUNCH(BIN, NC, ST, FR)                                                          \
  {                                                                                           \
    const int64_t n = bb[BIN + 1] - bb[BIN];                                                  \
    LPA_TRY(mark(2 * (BIN + 1), ST));                                                         \
    if (n > 0) {                                                                              \
      if (gnow)                                                                               \
        hipLaunchKernelGGL((k_lpa_wave<NC, true>), dim3(cap_grid((n + 3) / 4, 2048)), dim3(256), 0, ST, \
                           g->rp, vsrc, Lown, bb[BIN], bb[BIN + 1], g->flist, fcnt + BIN, FR, pmax, gsel, Lc); \
      else                                                                                    \
        hipLaunchKernelGGL((k_lpa_wave<NC, false>), dim3(cap_grid((n + 3) / 4, 2048)), dim3(256), 0, ST, \
                           g->rp, vsrc, Lown, bb[BIN], bb[BIN + 1], g->flist, fcnt + BIN, FR, pmax, gsel, \
                           (const int32_t*)nullptr);                                          \
      LPA_HIP(hipGetLastError());                                                             \
    }                                                                                         \
    LPA_TRY(mark(2 * (BIN + 1) + 1, ST));                                                     \
  }
#define LPA_GROUP_LAUNCH(BIN, G, ST)                                                         \
  {                                                                                          \
    const int64_t n = bb[BIN + 1] - bb[BIN];                                                 \
    LPA_TRY(mark(2 * (BIN + 1), ST));                                                        \
    if (n > 0) {                                                                             \
      if (gnow)                                                                              \
        hipLaunchKernelGGL((k_lpa_group<G, true>), dim3((unsigned)((n * G + 255) / 256)), dim3(256), 0, \
                           ST, g->rp, vsrc, Lown, bb[BIN], bb[BIN + 1], g->flist, fcnt + BIN, fr_rows, Lc); \
      else                                                                                   \
        hipLaunchKernelGGL((k_lpa_group<G, false>), dim3((unsigned)((n * G + 255) / 256)), dim3(256), 0, \
                           ST, g->rp, vsrc, Lown, bb[BIN], bb[BIN + 1], g->flist, fcnt + BIN, fr_rows, \
                           (const int32_t*)nullptr);                                         \
      LPA_HIP(hipGetLastError());                                                            \
    }                                                                                        \
    LPA_TRY(mark(2 * (BIN + 1) + 1, ST));                                                    \
  }
#define LPA_ROWS_LAUNCH(BIN, G, FR, ST)                                                      \
  {                                                                                          \
    const int64_t n = bb[BIN + 1] - bb[BIN];                                                 \
    LPA_TRY(mark(2 * (BIN + 1), ST));                                                        \
    if (n > 0) {                                                                             \
      const int64_t nbat = (n + 512 / G - 1) / (512 / G);                                    \
      if (gnow)                                                                              \
        hipLaunchKernelGGL((k_lpa_rows<G, true>), dim3(cap_grid((nbat + 3) / 4, 2048)), dim3(256), 0, \
                           ST, g->rp, vsrc, Lown, bb[BIN], bb[BIN + 1], g->flist, fcnt + BIN, FR, \
                           sort_after, gsel, Lc);                                             \
      else                                                                                   \
        hipLaunchKernelGGL((k_lpa_rows<G, false>), dim3(cap_grid((nbat + 3) / 4, 2048)), dim3(256), 0, \
                           ST, g->rp, vsrc, Lown, bb[BIN], bb[BIN + 1], g->flist, fcnt + BIN, FR, \
                           sort_after, gsel, (const int32_t*)nullptr);                        \
      LPA_HIP(hipGetLastError());                                                            \
    }                                                                                        \
    LPA_TRY(mark(2 * (BIN + 1) + 1, ST));                                                    \
  }
  // stream balance (measured steady superstep): aux0 w16 + w8 + w4, aux1 w2 + the
  // row/group bins (round 4: superstep 2's tail bins g16 .. g1 on the main stream, ahead
  // of the hub combine, measured slower -- 2.08 -> 2.11 ms)
  hipStream_t st_tail = sc;
  // converged supersteps (captured graphs, frontier lists): each bin stream's chain as
  // one k_bins_fused launch -- the same blocks per bin as the kernels of their own
  // (group bins capped like the others: their bodies grid-stride).  Not with the
  // frontier off: every superstep is then in range mode, where the fused launch's
  // register / LDS budget (the largest bin's) costs the narrow bins occupancy
  const bool fused = fused_now(g);
  auto launch_fused = [&](int wide, hipStream_t st) -> int {
    const int b0 = wide ? BIN_W16 : BIN_W2, b1 = wide ? BIN_W2 : BIN_ISO;
    FusedBins fb{};
    int32_t tot = 0;
    for (int b = b0; b < b1; ++b) {
      const int64_t n = bb[b + 1] - bb[b];
      if (n <= 0) continue;
      int64_t want;
      if (b <= BIN_W2) {
        want = (n + 3) / 4;
      } else if (b <= BIN_G8) {
        const int64_t rb = 512 / (64 >> (b - BIN_G64));
        want = ((n + rb - 1) / rb + 3) / 4;
      } else {
        want = (n * (4 >> (b - BIN_G4)) + 255) / 256;
      }
      fb.bin[fb.n] = b;
      fb.vb[fb.n] = bb[b];
      fb.ve[fb.n] = bb[b + 1];
      fb.off[fb.n] = tot;
      tot += (int32_t)cap_grid(want, 2048);
      ++fb.n;
    }
    fb.off[fb.n] = tot;
    LPA_TRY(mark(2 * (b0 + 1), st));
    if (fb.n > 0) {
      if (wide)
        hipLaunchKernelGGL(k_bins_fused<1>, dim3((unsigned)tot), dim3(256), 0, st, fb, g->rp, g->al, Lown, g->flist,
                           fcnt, fr_bins, pmax, sort_after);
      else
        hipLaunchKernelGGL(k_bins_fused<0>, dim3((unsigned)tot), dim3(256), 0, st, fb, g->rp, g->al, Lown, g->flist,
                           fcnt, fr_bins, pmax, sort_after);
      LPA_HIP(hipGetLastError());
    }
    LPA_TRY(mark(2 * (b0 + 1) + 1, st));  // (serialized stats: the launch counts under its first bin)
    return LPA_OK;
  };
  if (fused) {
    if (g->fused_bins == 2) {  // the wave bins keep their own launches
      LPA_WAVE_LAUNCH(BIN_W16, 16, sb, fr_wave)
      LPA_WAVE_LAUNCH(BIN_W8, 8, sb, fr_wave)
      LPA_WAVE_LAUNCH(BIN_W4, 4, sb, fr_wave)
    } else {
      LPA_TRY(launch_fused(1, sb));
    }
    LPA_TRY(launch_fused(0, sc));
  } else {
  LPA_WAVE_LAUNCH(BIN_W16, 16, sb, fr_wave)
  LPA_WAVE_LAUNCH(BIN_W8, 8, sb, fr_wave)
  LPA_WAVE_LAUNCH(BIN_W4, 4, sb, fr_wave)
  LPA_WAVE_LAUNCH(BIN_W2, 2, code_tally_now(g) ? sb : sc, fr_wave)
  if (code_tally_now(g) && g->code_lbin > BIN_G64) {
    // superstep 2 after a code refresh that coded the rows of 9-64 arcs: the labelled bins
    // first (their ranges), then, behind the code settle's lists, the coded row bins
    LPA_ROWS_LAUNCH(BIN_G8, 8, fr_rows, st_tail)
    LPA_GROUP_LAUNCH(BIN_G4, 4, st_tail)
    LPA_GROUP_LAUNCH(BIN_G2, 2, st_tail)
    LPA_GROUP_LAUNCH(BIN_G1, 1, st_tail)
    if (sc != sb) LPA_HIP(hipStreamWaitEvent(sc, g->ev_join2[2], 0));
    LPA_ROWS_LAUNCH(BIN_G64, 64, fr_row(BIN_G64), sc)
    LPA_ROWS_LAUNCH(BIN_G32, 32, fr_row(BIN_G32), sc)
    LPA_ROWS_LAUNCH(BIN_G16, 16, fr_row(BIN_G16), st_tail)
  } else {
    LPA_ROWS_LAUNCH(BIN_G64, 64, fr_row(BIN_G64), sc)
    LPA_ROWS_LAUNCH(BIN_G32, 32, fr_row(BIN_G32), sc)
    LPA_ROWS_LAUNCH(BIN_G16, 16, fr_row(BIN_G16), st_tail)
    LPA_ROWS_LAUNCH(BIN_G8, 8, fr_rows, st_tail)
    LPA_GROUP_LAUNCH(BIN_G4, 4, st_tail)
    LPA_GROUP_LAUNCH(BIN_G2, 2, st_tail)
    LPA_GROUP_LAUNCH(BIN_G1, 1, st_tail)
  }
  }
#undef LPA_ROWS_LAUNCH
#undef LPA_GROUP_LAUNCH
#undef LPA_WAVE_LAUNCH
  if (units_last) LPA_TRY(launch_units());
  // hub combine after the bins are queued: its tail kernels on the aux streams
  // run after those streams' bins
  LPA_TRY(mark(2, s));
  const bool hub_fork = !g->serial && g->since_reset < kDenseSupersteps;
  LPA_TRY(launch_hub_combine(g, Lown, hub_fork, !split, giant_units));
  if (split) {
    LPA_TRY(launch_block_narrow(s));
    if (hub_fork) LPA_HIP(hipStreamWaitEvent(s, g->ev_join2[0], 0));
  }
  LPA_TRACE_POINT("hub_combine");
  // the block rows' labels are seg-bin slots: joined before the main stream's diff
  if (split && !giant_units) LPA_HIP(hipStreamWaitEvent(s, g->ev_join2[1], 0));
  LPA_TRY(mark(3, s));
  if (diff) {
    // inside the concurrent tally: no Lc sync here, the scatter refresh does it; the
    // label-dense supersteps only count the changed slots (launch_refresh decides)
    const int dm = dense_refresh(g) ? 1 : 0;
    // (the split between the two bin streams follows where w2 ran)
    const int bw = code_tally_now(g) ? BIN_G64 : BIN_W2;
    if (nstr == 1 && !g->serial) {  // one stream: one diff over every bin
      LPA_TRY(launch_diff(g, s, Lc, Ln, 0, bb[BIN_ISO], false, g->par, BIN_SEG, BIN_ISO, dm));
    } else if (nstr == 2) {  // the bins' stream: one diff over its bins
      LPA_TRY(launch_diff(g, sb, Lc, Ln, bb[BIN_W16], bb[BIN_ISO], false, g->par, BIN_W16, BIN_ISO, dm));
      LPA_TRY(launch_diff(g, s, Lc, Ln, 0, bb[BIN_W16], false, g->par, BIN_SEG, BIN_W16, dm));
    } else {
    LPA_TRY(launch_diff(g, sb, Lc, Ln, bb[BIN_W16], bb[bw], false, g->par, BIN_W16, bw, dm));
    // isolated slots (and the padding) never change: the diff stops at the isolated bin
    LPA_TRY(launch_diff(g, sc, Lc, Ln, bb[bw], bb[BIN_ISO], false, g->par, bw, BIN_ISO, dm));
    LPA_TRY(launch_diff(g, s, Lc, Ln, 0, bb[BIN_W16], false, g->par, BIN_SEG, BIN_W16, dm));
    }
  }
  if (sb != s) {
    LPA_HIP(hipEventRecord(g->ev_join[0], sb));
    LPA_HIP(hipStreamWaitEvent(s, g->ev_join[0], 0));
    if (sc != sb) {
      LPA_HIP(hipEventRecord(g->ev_join[1], sc));
      LPA_HIP(hipStreamWaitEvent(s, g->ev_join[1], 0));
    }
  }
  return LPA_OK;
}

// al[] rebuild: the LDS hot-label kernel on a single-GPU handle (hub slots are
// [0, kHotLabels) there), the plain one otherwise
constexpr int64_t kHotMaxSlots = int64_t(1) << 29;  // k_al_rebuild_hot's 32-bit label offsets (P = 1)
int launch_rebuild(lpa_graph* g, bool if_wanted, int64_t thr, const int32_t* L,
                   const unsigned long long* ctr) {
  hipStream_t s = g->stream;
  const bool code = if_wanted && code_refresh_now(g);
  // the giant label of the refreshed vector: the rebuild's bits below and the next
  // superstep's tallies (launch_tally's gsel) read it
  if (g->V > 0) {
    hipLaunchKernelGGL(k_giant_pick, dim3(1), dim3(kPickK), 0, s, L, g->V, g->slice, g->nranks, g->gword);
    LPA_HIP(hipGetLastError());
  }
  const bool ranked = rebuild_ranked(g);
  // hot slots of the bits-mode / code-mode test (k_giant_bits' count in gword[3]): the
  // first kHotBits slots at P = 1, the first kHotBits / P (whole bit words) of every slice
  // of a rank-strided vector -- the same degree-ranked top set
  const uint64_t hmask = ranked ? (uint64_t)(g->slice - 1) : ~0ull;
  const int64_t hlim = ranked ? std::min<int64_t>(g->slice, kHotBits / g->nranks / 64 * 64) : kHotBits;
  const int64_t nhot_bits = ranked ? g->nranks * hlim : std::min<int64_t>(g->vpad, kHotBits);
  if (g->rebuild_hot && g->nranks == 1 && g->vpad < kHotMinSlots) {
    const int64_t ngrp = (g->vpad + 511) / 512;
    const unsigned gb = cap_grid((ngrp + 3) / 4, 4096), gr = cap_grid((g->arcs + 2047) / 2048, 8192);
    if (if_wanted) {
      hipLaunchKernelGGL(k_giant_bits<true>, dim3(gb), dim3(256), 0, s, ctr, thr, L, g->vpad, g->gword,
                         (unsigned long long*)g->gbits, g->abits, (int64_t)0, hmask, hlim);
      hipLaunchKernelGGL(k_al_rebuild_small<true>, dim3(gr), dim3(256), 0, s, ctr, thr, g->col, g->arcs, L, g->al,
                         g->gbits, g->vpad, g->gword, g->abits);
    } else {
      hipLaunchKernelGGL(k_giant_bits<false>, dim3(gb), dim3(256), 0, s, ctr, thr, L, g->vpad, g->gword,
                         (unsigned long long*)g->gbits, g->abits, (int64_t)0, hmask, hlim);
      hipLaunchKernelGGL(k_al_rebuild_small<false>, dim3(gr), dim3(256), 0, s, ctr, thr, g->col, g->arcs, L, g->al,
                         g->gbits, g->vpad, g->gword, g->abits);
    }
  } else if (g->rebuild_hot && ((g->nranks == 1 && g->vpad <= kHotMaxSlots) || ranked)) {
    int dev_cus = 256;
    (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, g->device);
    int slice_lg = 0, hot_lg = 0, hb_lg = 0;
    int32_t nhot = (int32_t)(g->vpad < kHotLabelsSingle ? g->vpad : kHotLabelsSingle);
    if (ranked) {
      while ((int64_t(1) << slice_lg) < g->slice) ++slice_lg;
      while ((int64_t(1) << hot_lg) < kHotLabels / g->nranks) ++hot_lg;
      nhot = (int32_t)(g->nranks << hot_lg);
      // bits per slice: the largest power of two with P of them in the LDS bit budget,
      // at least one word and at most the slice
      while ((int64_t(2) << hb_lg) * g->nranks <= kHotBits && (int64_t(2) << hb_lg) <= g->slice) ++hb_lg;
      if (hb_lg < 5 || slice_lg < 5) hb_lg = 0;
    }
    // the giant-label bitmap of L first (same wanted-check: both return at once when
    // the scatter refreshes instead)
    const int64_t ngrp = (g->vpad + 511) / 512;
    // class-blocked labels-mode rebuild (P = 1): a grid of whole 8-block groups
    const bool blk = !ranked && g->blk_pieces && g->blk_a0 > 0 && dev_cus >= 8;
    if (blk) dev_cus &= ~7;
    const int64_t nzero = blk ? g->blk_a0 / 64 : 0;
    if (if_wanted)
      hipLaunchKernelGGL(k_giant_bits<true>, dim3(cap_grid((ngrp + 3) / 4, 4096)), dim3(256), 0, s, ctr, thr, L,
                         g->vpad, g->gword, (unsigned long long*)g->gbits, g->abits, nzero, hmask, hlim);
    else
      hipLaunchKernelGGL(k_giant_bits<false>, dim3(cap_grid((ngrp + 3) / 4, 4096)), dim3(256), 0, s, ctr, thr, L,
                         g->vpad, g->gword, (unsigned long long*)g->gbits, g->abits, nzero, hmask, hlim);
    LPA_HIP(hipGetLastError());
    // ranked without a usable bit share: nbits 0 keeps every block in labels mode
    const int64_t nbits = (ranked && hb_lg == 0) ? 0 : g->vpad;
    BlkInfo binfo;
    for (int x = 0; x <= kMaxBlkClasses; ++x) binfo.off[x] = g->blk_off[x];
    binfo.a0 = blk ? g->blk_a0 : 0;
    binfo.phases = g->blk_classes / 8;
#define LPA_HOT_LAUNCH(W, R, B)                                                                  \
  hipLaunchKernelGGL((k_al_rebuild_hot<W, R, B>), dim3(dev_cus), dim3(1024), 0, s, ctr, thr, g->col, \
                     g->arcs, L, nhot, g->al, slice_lg, hot_lg, hb_lg, g->gbits, nbits, g->gword, g->abits, \
                     blk ? g->blk_pieces : nullptr, binfo, code ? g->gword + 5 : nullptr)
    if (code) {
      hipLaunchKernelGGL(k_code_mode, dim3(1), dim3(64), 0, s, ctr, thr, nhot_bits, g->gword);
      LPA_HIP(hipGetLastError());
    }
    if (if_wanted) {
      if (ranked) LPA_HOT_LAUNCH(true, true, false);
      else if (blk) LPA_HOT_LAUNCH(true, false, true);
      else LPA_HOT_LAUNCH(true, false, false);
    } else {
      if (ranked) LPA_HOT_LAUNCH(false, true, false);
      else if (blk) LPA_HOT_LAUNCH(false, false, true);
      else LPA_HOT_LAUNCH(false, false, false);
    }
#undef LPA_HOT_LAUNCH
    if (code) {
      LPA_HIP(hipGetLastError());
      hipLaunchKernelGGL(k_code_build, dim3(cap_grid((g->vpad / 16 + 255) / 256, 4096)), dim3(256), 0, s,
                         (const int4*)L, g->vpad / 16, g->gword, g->code2);
      LPA_HIP(hipGetLastError());
      // ranked: 2^hc_lg codes of every slice in LDS (P << hc_lg <= 16 kHotLabelsSingle)
      int hc_lg = 4;
      while (ranked && (int64_t(g->nranks) << (hc_lg + 1)) <= 16ll * kHotLabelsSingle &&
             (int64_t(1) << (hc_lg + 1)) <= g->slice)
        ++hc_lg;
      if (ranked)
        hipLaunchKernelGGL(k_code_rebuild<true>, dim3(dev_cus), dim3(1024), 0, s, g->gword, g->col, g->arcs, L,
                           g->vpad, g->code2, g->code_pcut, g->al2, g->al, slice_lg, hot_lg, hc_lg);
      else
        hipLaunchKernelGGL(k_code_rebuild<false>, dim3(dev_cus), dim3(1024), 0, s, g->gword, g->col, g->arcs, L,
                           g->vpad, g->code2, g->code_pcut, g->al2, g->al, 0, 0, 0);
    }
  } else {
    const unsigned grid = cap_grid((g->arcs / 4 + 511) / 512, 8192);
    if (if_wanted)
      hipLaunchKernelGGL(k_al_rebuild<true>, dim3(grid), dim3(256), 0, s, ctr, thr, g->col,
                         g->arcs, L, g->al, g->gword);
    else
      hipLaunchKernelGGL(k_al_rebuild<false>, dim3(grid), dim3(256), 0, s, ctr, thr, g->col,
                         g->arcs, L, g->al, g->gword);
  }
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// changed slots in [s0, s1) -> position chunks + dirty-arc count (counters of this
// superstep's parity)
int launch_diff(lpa_graph* g, hipStream_t st, const int32_t* Lc, const int32_t* Ln, int64_t s0,
                int64_t s1, bool sync, int par, int b0, int b1, int mode) {
  if (s1 <= s0) return LPA_OK;
  const int64_t nq = (s1 + 3) / 4 - s0 / 4;
  BinBounds bnd;
  for (int b = 0; b <= LPA_NBINS; ++b) bnd.b[b] = g->bin_begin[b];
  // bins [b0, b1) given: the frontier list mode is available (the concurrent tally
  // of this superstep; its lists are those of g->par)
  const bool lists = b1 > b0;
  hipLaunchKernelGGL(k_diff, dim3((unsigned)((nq + kDiffQuads - 1) / kDiffQuads)), dim3(256), 0, st,
                     (const int4*)Lc, (const int4*)Ln, sync ? const_cast<int32_t*>(Lc) : nullptr, s0, s1,
                     g->cptr, g->cch, g->chflag, g->chlist, g->counters + 4 * par, bnd, b0, b1,
                     lists ? g->flist : nullptr, g->fcnt + 16 * g->par, g->fr_all + g->par, mode);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

// refresh al[] for L_next (after the exchange, so every rank sees all changes) of the
// superstep of parity `par`; diff_done: the tally schedule already ran the diff per
// stream (launch_tally) or the exchange listed the changes
// fold_rebuild: k_al_scatter does a wanted rebuild itself (captured converged
// supersteps: saves the rebuild launch, which is almost never wanted there)
int launch_refresh(lpa_graph* g, const int32_t* Lc, const int32_t* Ln, bool diff_done, int par,
                   hipEvent_t ev_scatter = nullptr, bool fold_rebuild = false) {
  if (g->arcs == 0) return LPA_OK;
  hipStream_t s = g->stream;
  // this superstep's counters (zeroed by the previous k_al_scatter or at build)
  unsigned long long* ctr = g->counters + 4 * par;
  // one rank: its isolated slots (and the padding) never change; P > 1: the whole
  // replicated vector (other ranks' slots change through the exchange)
  const int64_t nd = !exchanges(g) ? g->bin_begin[BIN_ISO] : g->vpad;
  // diff_done means, at P = 1, that the tally's per-stream diffs ran (count-only ones in
  // a label-dense superstep); at P > 1, that the delta exchange queued every change
  // already (nothing left to count or diff)
  if (dense_refresh(g) && !(diff_done && exchanges(g))) {
    // counted changed slots (in the tally, or here) -> rebuild, or the full diff
    if (!diff_done) LPA_TRY(launch_diff(g, s, Lc, Ln, 0, nd, false, par, 0, 0, 1));
    hipLaunchKernelGGL(k_dense_decide, dim3(1), dim3(64), 0, s, ctr, nd, g->gword);
    LPA_HIP(hipGetLastError());
    LPA_TRY(launch_diff(g, s, Lc, Ln, 0, nd, true, par, 0, 0, 2));
  } else {
    if (!diff_done) LPA_TRY(launch_diff(g, s, Lc, Ln, 0, nd, true, par));
    // P > 1, superstep 2 after a giant-code refresh, its changes exchanged as a delta
    // (the change chunks are queued): the rows it settled from codes have no al[] entries,
    // so this refresh rebuilds whatever the change count (k_dense_decide's code clause)
    if (code_tally_now(g)) {
      hipLaunchKernelGGL(k_dense_decide, dim3(1), dim3(64), 0, s, ctr, INT64_MAX, g->gword);
      LPA_HIP(hipGetLastError());
    }
  }
  LPA_TRACE_POINT("diff");
  // (a handle without the CSC position index rebuilds every time: counters[1] >= 0 > -1)
  const int64_t thr = g->no_scatter ? -1 : (int64_t)(kRebuildFrac * (double)g->arcs);
  FrontierMarks fm;
  fm.crow = g->crow;
  fm.rp = g->rp;
  fm.uoff = g->hub_uoff;
  fm.n_hub = g->n_hub;
  fm.rdirty = g->rdirty[par ^ 1];
  fm.udirty = g->udirty[par ^ 1];
  if (code_tally3_now(g)) {
    // superstep 3 after a giant-code refresh: its settled rows' al[] entries were never
    // written, so this refresh rebuilds (k_dense_decide's code clause; n_slots: no count)
    hipLaunchKernelGGL(k_dense_decide, dim3(1), dim3(64), 0, s, ctr, INT64_MAX, g->gword);
    LPA_HIP(hipGetLastError());
  }
  // gather mode (lpa_build): no al[] to keep -- the scatter only marks the rows the next
  // superstep re-tallies (and syncs the changed labels into Lc), no rebuild
  const bool gnow = gather_now(g);
  // superstep 3's refresh keeps the arc giant bits of superstep 2's bits-mode rebuild
  // (k_al_scatter; superstep 4's row settle reads them)
  const bool keep_bits = g->since_reset == 2 && g->abits != nullptr && g->gbits != nullptr && !gnow &&
                         g->keep_bits;
  if (g->al_pending && !gnow) {  // the column-run superstep after a lazy reset (al holds nothing)
    hipLaunchKernelGGL(k_al_fill_unless_rebuild, dim3(cap_grid((g->arcs / 4 + 255) / 256, 8192)), dim3(256), 0, s,
                       ctr, thr, (const v4i*)g->al0, (v4i*)g->al, g->arcs);
    LPA_HIP(hipGetLastError());
    g->al_pending = false;  // the rebuild below (or this fill + the scatter) makes al valid
  }
  hipLaunchKernelGGL(k_al_scatter, dim3(2048), dim3(256), 0, s, g->chlist, (const uint4*)g->chflag,
                     (g->n_chunk_scan + 15) / 16, g->cowner, g->cch, ctr,
                     g->counters + 4 * (par ^ 1), g->cptr,
                     g->cpos, Ln, gnow ? (int32_t*)nullptr : g->al, thr, fm, g->fr_all + (par ^ 1),
                     g->frontier, (int64_t)(kFrontierFrac * (double)g->arcs), const_cast<int32_t*>(Lc),
                     (fold_rebuild && !gnow) ? g->col : (const int32_t*)nullptr, g->arcs, g->gword,
                     keep_bits ? 1 : 0, g->gbits, g->abits);
  LPA_HIP(hipGetLastError());
  LPA_TRACE_POINT("scatter");
  if (ev_scatter) LPA_HIP(hipEventRecord(ev_scatter, s));  // profiling: scatter | rebuild
  if (gnow && g->since_reset == kGatherSteps - 1) {
    // the last gather-mode superstep: al[] for the supersteps after it, one plain rebuild
    const unsigned grid = cap_grid((g->arcs / 4 + 511) / 512, 8192);
    hipLaunchKernelGGL(k_al_rebuild<false>, dim3(grid), dim3(256), 0, s, ctr, thr, g->col, g->arcs, Ln, g->al,
                       g->gword);
    LPA_HIP(hipGetLastError());
  } else if (!fold_rebuild && !gnow) {
    LPA_TRY(launch_rebuild(g, true, thr, Ln, ctr));
  }
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

}  // namespace

// the converged supersteps' bins as one k_bins_fused launch per stream (launch_tally)
bool fused_now(const lpa_graph* g) {
  return g->fused_bins && g->frontier && g->since_reset >= kDenseSupersteps + 2 && !gather_now(g);
}

// (the caller-driven delta exchange, lpa_exchange_put_delta: the refresh of the superstep
// lpa_step just ran, which since_reset already counts -- it is seen as the in-library
// refresh of that superstep sees it: dense / code-settled supersteps, code refresh allowed)
int launch_refresh_ext(lpa_graph* g, const int32_t* Lc, const int32_t* Ln, bool diff_done, int par) {
  const bool back = g->since_reset > 0;
  if (back) --g->since_reset;
  const int rc = launch_refresh(g, Lc, Ln, diff_done, par);
  if (back) ++g->since_reset;
  return rc;
}

// Capture `body` (launches on the handle's stream and the streams it forks) into an
// executable graph.  Captures are serialised process-wide (several handles of one
// process, e.g. virtual ranks driven from threads, crashed capturing at once).
template <typename Body>
int capture_graph(lpa_graph* g, hipGraphExec_t* out, Body body) {
  static std::mutex capture_mu;
  std::lock_guard<std::mutex> lk(capture_mu);
  hipStream_t s = g->stream;
  hipGraph_t graph = nullptr;
  LPA_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  const int rc = body();
  hipError_t ec = hipStreamEndCapture(s, &graph);
  if (rc != LPA_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  LPA_HIP(ec);
  ec = hipGraphInstantiate(out, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  LPA_HIP(ec);
  return LPA_OK;
}

int run_supersteps(lpa_graph* g, int32_t n, lpa_stats* st, bool last_refresh) {
  hipStream_t s = g->stream;
  const bool timed = st != nullptr;
  const int nt = n < LPA_STATS_MAX_ITERS ? n : LPA_STATS_MAX_ITERS;
  if (timed) {
    memset(st, 0, sizeof(*st));
    for (auto& e : g->ev)
      if (!e) LPA_HIP(hipEventCreate(&e));
    for (int i = 0; i < nt * kBinEvents; ++i)
      if (!g->bin_ev[i]) LPA_HIP(hipEventCreate(&g->bin_ev[i]));
    LPA_HIP(hipEventRecord(g->ev[2 * LPA_STATS_MAX_ITERS], s));
  }
  // per timed superstep t, bin_ev[t*kBinEvents + i]: 2k / 2k+1 around tally kernel
  // k (k < kTallyKernels), then kTallyEv after the join, +1 after the exchange, +2
  // after the diff + scatter, +3 after the rebuild, +4 / +5 around the frontier lists
  bool blk_ran[LPA_STATS_MAX_ITERS] = {};  // serialized stats: k_lpa_block ran in superstep t
  bool fus_ran[LPA_STATS_MAX_ITERS] = {};  // ... the fused bins (no marks of the other bins)
  for (int32_t t = 0; t < n; ++t) {
    if (t < nt) blk_ran[t] = block_mode_now(g);
    if (t < nt) fus_ran[t] = fused_now(g);
    const int32_t* Lc = g->lab[g->cur];
    int32_t* Ln = g->lab[g->cur ^ 1];
    int32_t* Lown = Ln + g->own_begin;
    const bool tt = timed && t < nt;
    if (g->force_all_next) {  // a stream op ahead of the superstep (never captured)
      LPA_TRY(frontier_all(g, g->par));
      g->force_all_next = false;
    }
    // per-kernel events only in the serialized profiling schedule (lpa_set_serial):
    // there they give standalone kernel times; the concurrent schedule is timed per
    // superstep only, so a timed converged superstep still replays its graph
    hipEvent_t* bev = (tt && g->serial) ? &g->bin_ev[t * kBinEvents] : nullptr;
    if (tt) LPA_HIP(hipEventRecord(g->ev[2 * t], s));
    // superstep 1 from L0: column runs, no hash tallies (its diff runs in the refresh)
    const bool first = first_runs_now(g);
    // before superstep 3 on a code-capable handle: did the refresh after superstep 2 take
    // the giant codes?  One host read (~20 us of idle GPU) instead of ~10 kernels that
    // return at once in the other case (C3: ~0.1 ms of superstep 3's 0.47)
    if (g->code_ok && g->since_reset == 2) {
      LPA_HIP(hipMemcpyAsync(g->h_flag, g->gword + 5, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      LPA_HIP(hipStreamSynchronize(s));
      g->code3 = *g->h_flag != 0;
    }
    if (!first && !gather_now(g)) LPA_TRY(ensure_al(g));  // a lazy reset's al is needed by the hash tallies
    // the last gather-mode superstep's refresh rebuilds al (launched or in its graph)
    const bool gather_switch = g->gather && g->since_reset == kGatherSteps - 1;
    const bool diff_in_tally = !exchanges(g) && !g->serial && !first;
    // converged supersteps on one GPU replay a captured HIP graph of the whole
    // superstep (tally on four streams + diff + refresh; ~25 kernels and the
    // fork/join events): one launch instead of ~40 queue operations.  The graph bakes
    // the label / counter buffers, so there is one per (cur, par) state.
    // supersteps before `eager` are launched stream-ordered (their schedule differs
    // from the converged one a captured graph bakes)
    // (supersteps 3 and 4 too: the row settle is launched only in superstep 3, and
    // superstep 4 reads the giant word of the labels it tallies)
    const int eager = kDenseSupersteps + 2;
    // supersteps 2 and 3 (not 4: its settle chain on aux0 stops overlapping the hub
    // units inside a graph, 0.67 -> 0.75 ms at C3)
    const bool early_graph = g->use_graphs && !exchanges(g) && !g->serial && !first && g->since_reset >= 1 &&
                             g->since_reset <= 2;
    if (g->use_graphs && !exchanges(g) && !g->serial && g->since_reset >= eager) {
      // (gather mode's converged supersteps have their own graphs: the plain ones and the
      // switch superstep, whose refresh rebuilds al)
      const int key = gather_now(g) ? 16 + (gather_switch ? 4 : 0) + g->cur * 2 + g->par
                                    : g->cur * 2 + g->par;
      if (!g->gexec[key])
        LPA_TRY(capture_graph(g, &g->gexec[key], [&]() -> int {
          int rc = launch_tally(g, Lown, nullptr, Lc, Ln, true);
          if (rc == LPA_OK) rc = launch_refresh(g, Lc, Ln, true, g->par, nullptr, true);
          return rc;
        }));
      LPA_HIP(hipGraphLaunch(g->gexec[key], s));
      ++g->n_graph_replays;
      if (tt) LPA_HIP(hipEventRecord(g->ev[2 * t + 1], s));
      if (gather_switch) g->al_pending = false;
      g->cur ^= 1;
      g->par ^= 1;
      ++g->since_reset;
      continue;
    }
    if (g->use_graphs && exchanges(g) && !g->serial && g->since_reset >= eager) {
      // P > 1: the tally (no collective inside) replays a captured graph per
      // (cur, par); the exchange, whose delta size the host reads, and the refresh
      // follow on the stream.  A loopback group (ranks = threads of one process) runs
      // this same path: its allgather ends with a third host meeting, after which no
      // peer waits on an event of this rank's stream while it captures (lpa_comm.cpp).
      const int key = g->cur * 2 + g->par;
      if (!g->gexec[key])
        LPA_TRY(capture_graph(g, &g->gexec[key],
                              [&]() -> int { return launch_tally(g, Lown, nullptr, Lc, Ln, diff_in_tally); }));
      LPA_HIP(hipGraphLaunch(g->gexec[key], s));
      ++g->n_graph_replays;
    } else if (first) {
      LPA_TRY(launch_first(g, Lown));
    } else if (early_graph) {
      // supersteps 2 and 3 on one GPU: a captured graph per (superstep, cur, par) too --
      // each has its own fixed schedule (giant decision, row settle), and their ~40-50
      // launches become one graph launch (C2: supersteps 2-3 0.46 / 0.50 -> 0.41 / 0.45 ms)
      // (superstep 3 after a giant-code refresh has its own schedule: keys 12..15)
      const int key = code_tally3_now(g) ? 12 + g->cur * 2 + g->par
                                         : 4 + ((g->since_reset - 1) * 2 + g->cur) * 2 + g->par;
      if (!g->gexec[key])
        LPA_TRY(capture_graph(g, &g->gexec[key], [&]() -> int {
          int rc = launch_tally(g, Lown, nullptr, Lc, Ln, true);
          if (rc == LPA_OK) rc = launch_refresh(g, Lc, Ln, true, g->par);
          return rc;
        }));
      LPA_HIP(hipGraphLaunch(g->gexec[key], s));
      ++g->n_graph_replays;
    } else {
      LPA_TRY(launch_tally(g, Lown, bev, Lc, Ln, diff_in_tally));
    }
    if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv], s));
    bool changes_listed = false;
    if (exchanges(g) && has_collective(g))
      LPA_TRY(exchange_collective(g, Lc, Ln, g->since_reset == 0, &changes_listed));
    if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv + 1], s));
    // P > 1 without a communicator: the caller completes the superstep with
    // lpa_exchange_put (full vector + al[] rebuild) or lpa_exchange_put_delta
    // (changes + refresh); a refresh here would see a partial vector
    if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv + 2], s));  // stays if there is no refresh
    // (P > 1 converged supersteps: the scatter folds the rare rebuild, as the P = 1
    // graph does -- no giant pick / bits / hot-rebuild launches that return at once)
    if ((!exchanges(g) || has_collective(g)) && !early_graph && (last_refresh || t + 1 < n)) {
      LPA_TRY(launch_refresh(g, Lc, Ln, diff_in_tally || changes_listed, g->par,
                             bev ? bev[kTallyEv + 2] : nullptr,
                             exchanges(g) && g->since_reset >= eager));
      if (gather_switch) g->al_pending = false;
    }
    if (bev) LPA_HIP(hipEventRecord(bev[kTallyEv + 3], s));
    // after the last block-mode superstep the next one tallies every row and unit:
    // the block rows' units staged nothing while k_lpa_block tallied them (set at the
    // next superstep's start, after any caller-driven refresh has written fr_all)
    if (block_mode_now(g) && g->since_reset + 1 == kDenseSupersteps) g->force_all_next = true;
    // the column-run superstep staged no hub unit words: a frontier superstep after it
    // would merge every unit of a dirty hub row with stale (or never written) words of
    // its unlisted units, so the next superstep tallies every row and unit
    if (first) g->force_all_next = true;
    // a settled superstep 3 (k_settle_*) re-tallies no unit of a settled hub row: their
    // staged words are stale for a frontier superstep 4
    if (g->since_reset == 2 && g->abits) g->force_all_next = true;
    if (tt) LPA_HIP(hipEventRecord(g->ev[2 * t + 1], s));
    g->cur ^= 1;
    g->par ^= 1;
    ++g->since_reset;
  }
  if (timed) LPA_HIP(hipEventRecord(g->ev[2 * LPA_STATS_MAX_ITERS + 1], s));
  // the kernel-side error word rides the final synchronisation (a stream-ordered copy
  // into pinned memory instead of a blocking hipMemcpy after it: one round trip fewer)
  if (n > 0) {
    if (!g->h_err) LPA_HIP(hipHostMalloc((void**)&g->h_err, sizeof(int32_t), hipHostMallocDefault));
    LPA_HIP(hipMemcpyAsync(g->h_err, g->dev_err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  }
  LPA_HIP(hipStreamSynchronize(s));
  if (n > 0) {
    const int32_t err = *g->h_err;
    if (err) {
      // reported once per call: a later call on this handle starts clean
      LPA_HIP(hipMemset(g->dev_err, 0, sizeof(int32_t)));
      set_error("superstep kernel capacity overflow (flags 0x%x): a hub combine bucket exceeded "
                "its LDS table", err);
      return LPA_EOVERFLOW;
    }
  }
  if (timed) {
    st->iters = n;
    st->n_iter_ms = nt;
    for (int t = 0; t < nt; ++t) {
      LPA_HIP(hipEventElapsedTime(&st->iter_ms[t], g->ev[2 * t], g->ev[2 * t + 1]));
      if (!g->serial) continue;  // per-kernel times: serialized schedule only
      hipEvent_t* bev = &g->bin_ev[t * kBinEvents];
      float ms;
      for (int k = 0; k < kTallyKernels; ++k) {
        if (fus_ran[t] && (k > BIN_W2 + 1 || (g->fused_bins != 2 && (k == BIN_W8 + 1 || k == BIN_W4 + 1))))
          continue;  // a bin inside a fused launch (no marks of its own)
        LPA_HIP(hipEventElapsedTime(&ms, bev[2 * k], bev[2 * k + 1]));
        st->kernel_ms[k] += ms;
      }
      LPA_HIP(hipEventElapsedTime(&ms, bev[kTallyEv], bev[kTallyEv + 1]));
      st->exchange_ms += ms;
      LPA_HIP(hipEventElapsedTime(&ms, bev[kTallyEv + 1], bev[kTallyEv + 2]));
      st->kernel_ms[kTallyKernels] += ms;
      LPA_HIP(hipEventElapsedTime(&ms, bev[kTallyEv + 2], bev[kTallyEv + 3]));
      st->kernel_ms[kTallyKernels + 1] += ms;
      LPA_HIP(hipEventElapsedTime(&ms, bev[kTallyEv + 4], bev[kTallyEv + 5]));
      st->kernel_ms[kTallyKernels + 2] += ms;
      if (blk_ran[t]) {
        LPA_HIP(hipEventElapsedTime(&ms, bev[kTallyEv + 6], bev[kTallyEv + 7]));
        st->kernel_ms[kTallyKernels + 3] += ms;
      }
    }
    float tot;
    LPA_HIP(hipEventElapsedTime(&tot, g->ev[2 * LPA_STATS_MAX_ITERS], g->ev[2 * LPA_STATS_MAX_ITERS + 1]));
    st->total_ms = tot;
  }
  return LPA_OK;
}

int frontier_all(lpa_graph* g, int par) {
  LPA_HIP(hipMemsetD32Async((hipDeviceptr_t)(g->fr_all + par), 1, 1, g->stream));
  return LPA_OK;
}

int rebuild_arc_labels(lpa_graph* g) {
  if (g->arcs == 0) return LPA_OK;
  return launch_rebuild(g, false, 0, g->lab[g->cur], g->counters);
}

int refresh_after_put(lpa_graph* g) {
  if (g->arcs == 0) return LPA_OK;
  if (g->since_reset == 0) return rebuild_arc_labels(g);   // no superstep ran since L0
  // the refresh of the superstep lpa_step just ran (since_reset counted it already): an
  // unconditional rebuild (thr = -1: every rebuild_wanted test passes), the giant codes
  // allowed after superstep 1 or 2 as in the in-library schedule
  --g->since_reset;
  const int rc = launch_rebuild(g, true, -1, g->lab[g->cur], g->counters + 4 * (g->par ^ 1));
  ++g->since_reset;
  return rc;
}

int ensure_al(lpa_graph* g) {
  if (!g->al_pending) return LPA_OK;
  LPA_HIP(hipMemcpyAsync(g->al, g->al0, sizeof(int32_t) * g->arcs, hipMemcpyDeviceToDevice, g->stream));
  g->al_pending = false;
  return LPA_OK;
}

int gather_labels(lpa_graph* g, int32_t* out_dense_dev) {
  if (g->V == 0) return LPA_OK;
  int64_t blocks = (g->V + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(k_gather_dense, dim3((unsigned)blocks), dim3(256), 0, g->stream,
                     g->lab[g->cur], g->new_of, g->V, out_dense_dev);
  LPA_HIP(hipGetLastError());
  return LPA_OK;
}

}  // namespace lpa
