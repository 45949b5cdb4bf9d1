// One LPA superstep on gfx950 (replaces GraphX
// LabelPropagation sendMessage/mergeMessage/vertexProgram driven by
// Pregel.apply -- SURVEY.md §2.2 U3/U4, §3.2).
//
// For every owned vertex v with deg(v) > 0:
//     L_next[v] = min{ l : cnt_v(l) = max_l' cnt_v(l') },  cnt_v(l) = #{arcs v->u : L_cur[u] = l}
// Vertices are degree-sorted, so each bin below is one contiguous slot range and
// every wave sees rows of near-equal length (no intra-wave imbalance).
//
// A vote tally is packed into one 64-bit word  (count << 32) | ~label : the
// maximum word is the highest count and, among equal counts, the smallest label,
// so "mode with smallest-label tie-break" is a plain u64 max-reduction; an empty
// slot is 0 (label 0xFFFFFFFF never occurs).
//
//   bin g1   deg == 1       thread per vertex: the neighbour's label
//   bin g2   deg == 2       min of the two labels (1-1 tie or equal)
//   bin g4/8/16 deg <= G    G lanes per vertex, ballot "peel": each round takes the
//                           group's first unresolved label, counts its lanes with one
//                           64-bit ballot, retires them (rounds = distinct labels)
//   bin wave 16 < deg <= 512   one wave per vertex, per-wave LDS hash (64-bit CAS/add),
//                           wave-level peel pre-aggregates repeated labels so converged
//                           neighbourhoods cost one LDS atomic per 64 arcs
//   bin seg  deg > 512      one 256-thread block per <= 2048-arc segment, block LDS hash;
//                           single-segment rows finish in-block, longer rows merge their
//                           segment tallies into a per-vertex global hash (64-bit device
//                           atomics) that k_lpa_hub_final reduces
// Tables keep a touched-slot list, so finishing a vertex costs O(distinct labels),
// not O(table size).  Column indices are streamed with non-temporal loads (read
// once per superstep) so they do not evict the label vector from L2 / MALL.
#include <string.h>

#include "lpa_internal.h"

namespace lpa {

namespace {

constexpr int kPeel = 2;  // wave-level pre-aggregation rounds per 64-arc chunk
constexpr int kUnroll = 4;  // 64-arc chunks in flight per wave
static_assert(kSegArcs % (256 * kUnroll) == 0, "each wave of a segment block must own kSegArcs/4 arcs");

__device__ __forceinline__ int32_t ld_stream(const int32_t* p) {
  return __builtin_nontemporal_load(p);
}

__device__ __forceinline__ u64 tally(u32 cnt, u32 label) {
  return ((u64)cnt << 32) | (u64)(u32)(~label);
}

__device__ __forceinline__ u64 umax64(u64 a, u64 b) { return a > b ? a : b; }

__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = umax64(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ u32 hash_slot(u32 label, int shift) {
  return (label * 0x9E3779B1u) >> shift;
}

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

// Global (HBM) variant for hub vertices; claimed slots are appended to `list`.
__device__ __forceinline__ void global_insert(u64* tab, int shift, u32 mask, u64 word,
                                              int32_t* list, int32_t* count) {
  const u32 key = (u32)word;
  const u64 add = word & 0xFFFFFFFF00000000ull;
  u32 h = hash_slot(~key, shift);
  while (true) {
    u64 old = atomicCAS(&tab[h], 0ull, word);
    if (old == 0ull) {
      int p = atomicAdd(count, 1);
      list[p] = (int32_t)h;
      return;
    }
    if ((u32)old == key) {
      atomicAdd(&tab[h], add);
      return;
    }
    h = (h + 1u) & mask;
  }
}

__device__ __forceinline__ int ceil_log2(u32 x) { return x <= 1 ? 0 : 32 - __clz(x - 1); }

// ---------------------------------------------------------------------------
// Process one 64-arc chunk held in registers (lab valid where `valid`) against
// a wave-owned list: peel up to kPeel repeated labels with ballots, then insert
// the remaining lanes individually.  Claimed slots appended to `lst` (wave-local
// counter `cnt`, kept uniform).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void tally_chunk(u64* tab, uint16_t* lst, int& cnt, int shift,
                                            u32 mask, u32 lab, bool valid, int lane, u64 lt) {
  u64 act = __ballot(valid);
#pragma unroll
  for (int p = 0; p < kPeel; ++p) {
    if (act == 0ull) break;
    const int lead = __ffsll((unsigned long long)act) - 1;
    const u32 x = (u32)__builtin_amdgcn_readlane((int)lab, lead);
    const u64 mm = __ballot(lab == x) & act;
    int slot = -1;
    if (lane == lead) slot = lds_insert(tab, shift, mask, x, (u32)__popcll(mm));
    const u64 cm = __ballot(slot >= 0);
    if (slot >= 0) lst[cnt] = (uint16_t)slot;
    cnt += cm ? 1 : 0;
    act &= ~mm;
  }
  int slot = -1;
  if ((act >> lane) & 1ull) slot = lds_insert(tab, shift, mask, lab, 1u);
  const u64 cm = __ballot(slot >= 0);
  if (slot >= 0) lst[cnt + __popcll(cm & lt)] = (uint16_t)slot;
  cnt += __popcll(cm);
}

// ---------------------------------------------------------------------------
// bins g1 / g2 / g4 / g8 / g16
// ---------------------------------------------------------------------------
template <int G>
__global__ __launch_bounds__(256) void k_lpa_group(const int64_t* __restrict__ rp,
                                                   const int32_t* __restrict__ col,
                                                   const int32_t* __restrict__ Lc,
                                                   int32_t* __restrict__ Ln, int64_t vbeg,
                                                   int64_t vend) {
  const int lane = threadIdx.x & 63;
  const int64_t v = vbeg + ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const int j = threadIdx.x & (G - 1);
  const bool live = v < vend;
  int64_t b = 0;
  int d = 0;
  if (live) {
    b = rp[v];
    d = (int)(rp[v + 1] - b);
  }
  const bool ok = j < d;
  const u32 lab = ok ? (u32)Lc[ld_stream(col + b + j)] : 0u;
  if constexpr (G == 1) {
    if (live) Ln[v] = (int32_t)lab;
  } else if constexpr (G == 2) {
    const u32 o = (u32)__shfl_xor((int)lab, 1, 64);
    if (live && j == 0) Ln[v] = (int32_t)(lab < o ? lab : o);
  } else {
    const int gbase = lane & ~(G - 1);
    const u64 gm = (1ull << G) - 1ull;
    u64 act = __ballot(ok);
    u64 best = 0ull;
    while (act) {
      const u64 my = (act >> gbase) & gm;
      const int lead = gbase + (my ? (__ffsll((unsigned long long)my) - 1) : 0);
      const u32 x = (u32)__shfl((int)lab, lead, 64);
      const u64 mm = __ballot(((act >> lane) & 1ull) && lab == x);
      const u32 c = (u32)__popcll((mm >> gbase) & gm);
      if (my) best = umax64(best, tally(c, x));
      act &= ~mm;
    }
    if (live && j == 0) Ln[v] = (int32_t)(~(u32)best);
  }
}

// ---------------------------------------------------------------------------
// bin wave: 16 < deg <= kWaveMaxDeg, one wave per vertex (grid-stride)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_lpa_wave(const int64_t* __restrict__ rp,
                                                  const int32_t* __restrict__ col,
                                                  const int32_t* __restrict__ Lc,
                                                  int32_t* __restrict__ Ln, int64_t vbeg,
                                                  int64_t vend) {
  __shared__ u64 tab_all[4][kWaveCap];
  __shared__ uint16_t lst_all[4][kWaveCap];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u64* tab = tab_all[w];
  uint16_t* lst = lst_all[w];
  for (int i = lane; i < kWaveCap; i += 64) tab[i] = 0ull;
  const u64 lt = (1ull << lane) - 1ull;
  for (int64_t v = vbeg + (int64_t)blockIdx.x * 4 + w; v < vend; v += (int64_t)gridDim.x * 4) {
    const int64_t b = rp[v], e = rp[v + 1];
    const int d = (int)(e - b);
    int lg = ceil_log2(2u * (u32)d);
    lg = lg < 6 ? 6 : lg;
    const u32 mask = (1u << lg) - 1u;
    const int shift = 32 - lg;
    int cnt = 0;
    for (int64_t base = b; base < e; base += 64 * kUnroll) {
      int32_t c[kUnroll];
      u32 lab[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t i = base + u * 64 + lane;
        c[u] = i < e ? ld_stream(col + i) : -1;
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) lab[u] = c[u] >= 0 ? (u32)Lc[c[u]] : 0u;
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        tally_chunk(tab, lst, cnt, shift, mask, lab[u], c[u] >= 0, lane, lt);
    }
    u64 best = 0ull;
    for (int i = lane; i < cnt; i += 64) {
      const int s = lst[i];
      best = umax64(best, tab[s]);
      tab[s] = 0ull;
    }
    best = wave_max_u64(best);
    if (lane == 0) Ln[v] = (int32_t)(~(u32)best);
  }
}

// ---------------------------------------------------------------------------
// bin seg: deg > kWaveMaxDeg, one block per segment of <= kSegArcs arcs
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_lpa_seg(const int32_t* __restrict__ col,
                                                 const int32_t* __restrict__ Lc,
                                                 int32_t* __restrict__ Ln,
                                                 const Segment* __restrict__ segs, int64_t nseg,
                                                 u64* __restrict__ gtab, int32_t* __restrict__ glist,
                                                 int32_t* __restrict__ gcnt,
                                                 const int64_t* __restrict__ hub_off) {
  __shared__ u64 tab[kSegCap];
  __shared__ uint16_t lst_all[4][kSegArcs / 4];
  __shared__ u64 red[4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint16_t* lst = lst_all[w];
  for (int i = threadIdx.x; i < kSegCap; i += 256) tab[i] = 0ull;
  __syncthreads();
  const u64 lt = (1ull << lane) - 1ull;
  for (int64_t si = blockIdx.x; si < nseg; si += gridDim.x) {
    const Segment sg = segs[si];
    int lg = ceil_log2(2u * (u32)sg.len);
    lg = lg < 6 ? 6 : lg;
    const u32 mask = (1u << lg) - 1u;
    const int shift = 32 - lg;
    const int64_t e = sg.begin + sg.len;
    int cnt = 0;
    for (int64_t base = sg.begin + (int64_t)w * 64 * kUnroll; base < e; base += 256 * kUnroll) {
      int32_t c[kUnroll];
      u32 lab[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t i = base + u * 64 + lane;
        c[u] = i < e ? ld_stream(col + i) : -1;
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) lab[u] = c[u] >= 0 ? (u32)Lc[c[u]] : 0u;
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
        tally_chunk(tab, lst, cnt, shift, mask, lab[u], c[u] >= 0, lane, lt);
    }
    __syncthreads();  // all tallies of the segment are in `tab`
    if (sg.v >= 0) {
      u64 best = 0ull;
      for (int i = lane; i < cnt; i += 64) {
        const int s = lst[i];
        best = umax64(best, tab[s]);
        tab[s] = 0ull;
      }
      best = wave_max_u64(best);
      if (lane == 0) red[w] = best;
      __syncthreads();
      if (threadIdx.x == 0)
        Ln[sg.v] = (int32_t)(~(u32)umax64(umax64(red[0], red[1]), umax64(red[2], red[3])));
    } else {
      const int64_t h = -(int64_t)sg.v - 1;
      const int64_t off = hub_off[h];
      const u32 cap = (u32)(hub_off[h + 1] - off);
      const int gshift = 32 - ceil_log2(cap);
      for (int i = lane; i < cnt; i += 64) {
        const int s = lst[i];
        const u64 word = tab[s];
        tab[s] = 0ull;
        global_insert(gtab + off, gshift, cap - 1u, word, glist + off, gcnt + h);
      }
    }
    __syncthreads();  // table slots cleared before the next segment
  }
}

// reduce the global tallies of multi-segment (hub) vertices
__global__ __launch_bounds__(256) void k_lpa_hub_final(u64* __restrict__ gtab,
                                                       const int32_t* __restrict__ glist,
                                                       int32_t* __restrict__ gcnt,
                                                       const int64_t* __restrict__ hub_off,
                                                       int32_t* __restrict__ Ln, int64_t n_hub) {
  __shared__ u64 red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t h = blockIdx.x; h < n_hub; h += gridDim.x) {
    const int64_t off = hub_off[h];
    const int n = gcnt[h];
    u64 best = 0ull;
    for (int i = threadIdx.x; i < n; i += 256) {
      const int32_t s = glist[off + i];
      best = umax64(best, gtab[off + s]);
      gtab[off + s] = 0ull;
    }
    best = wave_max_u64(best);
    if (lane == 0) red[w] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
      Ln[h] = (int32_t)(~(u32)umax64(umax64(red[0], red[1]), umax64(red[2], red[3])));
      gcnt[h] = 0;
    }
    __syncthreads();
  }
}

__global__ void k_gather_dense(const int32_t* __restrict__ L, const int32_t* __restrict__ new_of,
                               int64_t V, int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < V;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = L[new_of[i]];
}

inline unsigned cap_grid(int64_t want, int64_t cap) {
  if (want < 1) want = 1;
  return (unsigned)(want < cap ? want : cap);
}

// launch the bin kernels of one superstep; bin events optional
int launch_superstep(lpa_graph* g, const int32_t* Lc, int32_t* Lown, hipEvent_t* bev) {
  // bev marks: 0 start, k+1 after kernel k (0 seg, 1 hub_final, 2 wave, 3..7 g16..g1)
  hipStream_t s = g->stream;
  const int64_t* bb = g->bin_begin;
  auto mark = [&](int i) -> int {
    if (bev) LPA_HIP(hipEventRecord(bev[i], s));
    return LPA_OK;
  };
  LPA_TRY(mark(0));
  if (g->n_segs > 0) {
    hipLaunchKernelGGL(k_lpa_seg, dim3(cap_grid(g->n_segs, 1024)), dim3(256), 0, s, g->col, Lc,
                       Lown, g->segs, g->n_segs, g->gtab, g->glist, g->gcnt, g->hub_off);
    LPA_HIP(hipGetLastError());
  }
  LPA_TRY(mark(1));
  if (g->n_hub > 0) {
    hipLaunchKernelGGL(k_lpa_hub_final, dim3(cap_grid(g->n_hub, 1024)), dim3(256), 0, s, g->gtab,
                       g->glist, g->gcnt, g->hub_off, Lown, g->n_hub);
    LPA_HIP(hipGetLastError());
  }
  LPA_TRY(mark(2));
  {
    const int64_t n = bb[BIN_WAVE + 1] - bb[BIN_WAVE];
    if (n > 0) {
      hipLaunchKernelGGL(k_lpa_wave, dim3(cap_grid((n + 3) / 4, 4096)), dim3(256), 0, s, g->rp,
                         g->col, Lc, Lown, bb[BIN_WAVE], bb[BIN_WAVE + 1]);
      LPA_HIP(hipGetLastError());
    }
  }
  LPA_TRY(mark(3));
#define LPA_GROUP_LAUNCH(BIN, G)                                                             \
  {                                                                                          \
    const int64_t n = bb[BIN + 1] - bb[BIN];                                                 \
    if (n > 0) {                                                                             \
      hipLaunchKernelGGL(k_lpa_group<G>, dim3((unsigned)((n * G + 255) / 256)), dim3(256), 0, \
                         s, g->rp, g->col, Lc, Lown, bb[BIN], bb[BIN + 1]);                 \
      LPA_HIP(hipGetLastError());                                                            \
    }                                                                                        \
    LPA_TRY(mark(BIN + 2));                                                                  \
  }
  LPA_GROUP_LAUNCH(BIN_G16, 16)
  LPA_GROUP_LAUNCH(BIN_G8, 8)
  LPA_GROUP_LAUNCH(BIN_G4, 4)
  LPA_GROUP_LAUNCH(BIN_G2, 2)
  LPA_GROUP_LAUNCH(BIN_G1, 1)
#undef LPA_GROUP_LAUNCH
  return LPA_OK;
}

}  // namespace

int run_supersteps(lpa_graph* g, int32_t n, lpa_stats* st) {
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
  // per timed superstep t, marks bin_ev[t*kBinEvents + i]: 0 start, k+1 after kernel k,
  // LPA_NKERNELS+1 after the exchange
  for (int32_t t = 0; t < n; ++t) {
    const int32_t* Lc = g->lab[g->cur];
    int32_t* Ln = g->lab[g->cur ^ 1];
    int32_t* Lown = Ln + g->own_begin;
    const bool tt = timed && t < nt;
    hipEvent_t* bev = tt ? &g->bin_ev[t * kBinEvents] : nullptr;
    if (tt) LPA_HIP(hipEventRecord(g->ev[2 * t], s));
    LPA_TRY(launch_superstep(g, Lc, Lown, bev));
    if (g->nranks > 1 && g->comm) {
      ncclResult_t r = ncclAllGather(Lown, Ln, (size_t)g->slice, ncclInt32, g->comm, s);
      if (r != ncclSuccess) {
        set_error("ncclAllGather: %s", ncclGetErrorString(r));
        return LPA_ERCCL;
      }
    }
    if (tt) {
      LPA_HIP(hipEventRecord(bev[LPA_NKERNELS + 1], s));
      LPA_HIP(hipEventRecord(g->ev[2 * t + 1], s));
    }
    g->cur ^= 1;
  }
  if (timed) LPA_HIP(hipEventRecord(g->ev[2 * LPA_STATS_MAX_ITERS + 1], s));
  LPA_HIP(hipStreamSynchronize(s));
  if (timed) {
    st->iters = n;
    st->n_iter_ms = nt;
    for (int t = 0; t < nt; ++t) {
      LPA_HIP(hipEventElapsedTime(&st->iter_ms[t], g->ev[2 * t], g->ev[2 * t + 1]));
      hipEvent_t* bev = &g->bin_ev[t * kBinEvents];
      float ms;
      for (int k = 0; k < LPA_NKERNELS; ++k) {
        LPA_HIP(hipEventElapsedTime(&ms, bev[k], bev[k + 1]));
        st->kernel_ms[k] += ms;
      }
      LPA_HIP(hipEventElapsedTime(&ms, bev[LPA_NKERNELS], bev[LPA_NKERNELS + 1]));
      st->exchange_ms += ms;
    }
    float tot;
    LPA_HIP(hipEventElapsedTime(&tot, g->ev[2 * LPA_STATS_MAX_ITERS], g->ev[2 * LPA_STATS_MAX_ITERS + 1]));
    st->total_ms = tot;
  }
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
