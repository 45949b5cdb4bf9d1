// Device helpers shared by the superstep kernels (lpa_iter.hip, lpa_hub.hip).
//
// A vote tally is packed into one 64-bit word  (count << 32) | ~label : the
// maximum word is the highest count and, among equal counts, the smallest label,
// so "mode with smallest-label tie-break"  is a plain u64
// max-reduction; an empty slot is 0 (label 0xFFFFFFFF never occurs).
#pragma once

#include "lpa_internal.h"

namespace lpa {
namespace dev {

constexpr u32 kNone = 0xFFFFFFFFu;  // empty lane

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

__device__ __forceinline__ u32 hash_slot(u32 label, int shift) {
  return (label * 0x9E3779B1u) >> shift;
}

__device__ __forceinline__ int ceil_log2(u32 x) { return x <= 1 ? 0 : 32 - __clz(x - 1); }

// Insert `cnt` votes for `label` into an LDS open-addressing table of (mask+1)
// slots (never full: callers size it >= 2x the distinct labels).  Returns the
// slot index when this call claimed an empty slot, else -1.
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

// Bounded variant for tables whose load is not guaranteed by construction: after
// a full sweep it raises bit 2 of *err and drops the vote.
__device__ __forceinline__ int lds_insert_bounded(u64* tab, int shift, u32 mask, u32 label, u32 cnt,
                                                  int32_t* err) {
  const u32 key = ~label;
  u32 h = hash_slot(label, shift);
  for (u32 probe = 0; probe <= mask; ++probe) {
    u64 old = atomicCAS(&tab[h], 0ull, ((u64)cnt << 32) | key);
    if (old == 0ull) return (int)h;
    if ((u32)old == key) {
      atomicAdd(&tab[h], (u64)cnt << 32);
      return -1;
    }
    h = (h + 1u) & mask;
  }
  atomicOr(err, 2);
  return -1;
}

// Continue the insert of tally word `word` (count << 32 | ~label) whose first
// probe at slot h hit another key: linear probing.  Returns the claimed slot or
// -1 (merged into an existing key).  kBounded: give up after a full sweep, raise
// bit 2 of *err and drop the votes (tables whose load is not bounded by design).
template <bool kBounded>
__device__ __forceinline__ int lds_probe_word(u64* tab, u32 mask, u64 word, u32 h, int32_t* err) {
  const u32 key = (u32)word;
  for (u32 probe = 0; !kBounded || probe < mask; ++probe) {
    h = (h + 1u) & mask;
    const u64 old = atomicCAS(&tab[h], 0ull, word);
    if (old == 0ull) return (int)h;
    if ((u32)old == key) {
      atomicAdd(&tab[h], word & 0xFFFFFFFF00000000ull);
      return -1;
    }
  }
  atomicOr(err, 2);
  return -1;
}

// Batched insert of NC chunks of tally words (this lane inserts wv[c] when bit c of
// its `lmask` is set): every first-probe CAS is issued before any is resolved, so
// NC independent LDS atomics per lane are in flight instead of one dependent chain
// per word; a key match adds the count (no return value), a collision probes on.
// slot[c] = the slot this lane claimed, or -1.
template <int NC, bool kBounded = false>
__device__ __forceinline__ void insert_words(u64* tab, int shift, u32 mask, const u64 (&wv)[NC],
                                             u32 lmask, int (&slot)[NC], int32_t* err) {
  u64 old[NC];
  u32 hh[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    old[c] = 0ull;
    hh[c] = 0u;
    if ((lmask >> c) & 1u) {
      hh[c] = hash_slot(~(u32)wv[c], shift);
      old[c] = atomicCAS(&tab[hh[c]], 0ull, wv[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    slot[c] = -1;
    if ((lmask >> c) & 1u) {
      if (old[c] == 0ull) {
        slot[c] = (int)hh[c];
      } else if ((u32)old[c] == (u32)wv[c]) {
        atomicAdd(&tab[hh[c]], wv[c] & 0xFFFFFFFF00000000ull);
      } else {
        slot[c] = lds_probe_word<kBounded>(tab, mask, wv[c], hh[c], err);
      }
    }
  }
}

// Weighted peel over NC chunks of tally words with per-lane state (bit c of
// `lmask`: word c still untallied): each round takes the first untallied label of
// the first lane holding one, sums its words' counts (VALU + DPP wave sums, no
// per-chunk scalar mask chains) and retires them; repeated while a round retires
// >= 2 words, up to `rounds`.  Round p's tally word ends in lane p's *pw; *best is
// the maximum; returns the number of rounds.
template <int NC>
__device__ __forceinline__ int peel_words(const u64 (&wv)[NC], u32& lmask, u64& best, u64& pw,
                                          int lane, int rounds) {
  int np = 0;
#pragma unroll 1
  for (int p = 0; p < rounds; ++p) {
    const u64 live = __ballot(lmask != 0u);
    if (live == 0ull) break;
    u32 cand = 0u;
#pragma unroll
    for (int c = NC - 1; c >= 0; --c)
      if ((lmask >> c) & 1u) cand = ~(u32)wv[c];
    const u32 x = (u32)__builtin_amdgcn_readlane((int)cand, __ffsll((unsigned long long)live) - 1);
    u32 m = 0u, cs = 0u;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (((lmask >> c) & 1u) && ~(u32)wv[c] == x) {
        m |= 1u << c;
        cs += (u32)(wv[c] >> 32);
      }
    }
    lmask &= ~m;
    const u32 k = wave_sum_u32((u32)__popc(m));
    const u64 tw = tally(wave_sum_u32(cs), x);
    best = umax64(best, tw);
    if (lane == p) pw = tw;
    np = p + 1;
    if (k < 2) break;
  }
  return np;
}

// Append the claimed slots of NC chunks to a block-shared LDS list with ONE
// returning LDS atomic per wave.
template <int NC>
__device__ __forceinline__ void list_append_n(uint16_t* lst, int* lcount, const int (&slot)[NC],
                                              int lane) {
  u64 cm[NC];
  int tot = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    cm[c] = __ballot(slot[c] >= 0);
    tot += __popcll(cm[c]);
  }
  if (tot == 0) return;  // uniform over the wave
  int base = 0;
  if (lane == 0) base = atomicAdd(lcount, tot);
  base = __builtin_amdgcn_readfirstlane(base);
  const u64 lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (slot[c] >= 0) lst[base + __popcll(cm[c] & lt)] = (uint16_t)slot[c];
    base += __popcll(cm[c]);
  }
}

// Wave-aggregated append of claimed slots to an LDS list (one LDS atomic per wave).
__device__ __forceinline__ void list_append(uint16_t* lst, int* lcount, int slot, int lane) {
  const u64 cm = __ballot(slot >= 0);
  if (cm == 0ull) return;
  int base = 0;
  if (lane == 0) base = atomicAdd(lcount, __popcll(cm));
  base = __builtin_amdgcn_readfirstlane(base);
  if (slot >= 0) lst[base + __popcll(cm & ((1ull << lane) - 1ull))] = (uint16_t)slot;
}

// ---------------------------------------------------------------------------
// Block-aggregated histogram: hist[key] += val over a stream of (key, val) without
// the two costs of plain device atomics here -- same-address serialisation (hub
// degrees, giant communities: every wave adding into one counter) and one
// memory-side atomic per element.  The block sums into a small LDS open-addressing
// table (kBhSlots keys, at most kBhProbes probes per key) and flushes it at the end
// with one device atomic per distinct key; a key that finds no slot goes straight
// to the device histogram.  add1 first merges the lanes of a wave that hold the same
// key (ballot rounds), so a hub repeated across a wave is one LDS atomic.
// Every lane of the block must call init / add* / flush (they contain barriers or
// wave-wide ballots); keys must differ from kBhEmpty.
// ---------------------------------------------------------------------------
constexpr int kBhLg = 12;
constexpr int kBhSlots = 1 << kBhLg;
constexpr int kBhProbes = 8;
constexpr u32 kBhEmpty = 0xFFFFFFFFu;
// Once a key has failed every probe the table is taken as saturated (random keys:
// most later keys would fail too) and later keys probe their home slot only, where
// the block's early (hub) keys mostly sit.
template <typename T>
struct BlockHist {
  u32* key;  // LDS [kBhSlots]
  T* val;    // LDS [kBhSlots]
  int* sat;  // LDS: the table has overflowed
  __device__ __forceinline__ void init() {
    for (int i = threadIdx.x; i < kBhSlots; i += blockDim.x) {
      key[i] = kBhEmpty;
      val[i] = (T)0;
    }
    if (threadIdx.x == 0) *sat = 0;
    __syncthreads();
  }
  __device__ __forceinline__ bool lds_add(u32 k, T v) {
    u32 h = (k * 0x9E3779B1u) >> (32 - kBhLg);
    const int np = *sat ? 1 : kBhProbes;
#pragma unroll 1
    for (int p = 0; p < np; ++p) {
      const u32 old = atomicCAS(&key[h], kBhEmpty, k);
      if (old == kBhEmpty || old == k) {
        atomicAdd(&val[h], v);
        return true;
      }
      h = (h + 1u) & (u32)(kBhSlots - 1);
    }
    *sat = 1;
    return false;
  }
  // weighted: lanes with act add v to hist[k]
  __device__ __forceinline__ void addw(T* __restrict__ hist, bool act, u32 k, T v) {
    if (act && !lds_add(k, v)) atomicAdd(&hist[k], v);
  }
  // count: lanes with act add 1 to hist[k] (all 64 lanes of the wave call it)
  __device__ __forceinline__ void add1(T* __restrict__ hist, bool act, u32 k, int lane) {
    bool mine = act;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const u64 pend = __ballot(mine);
      if (pend == 0ull) return;  // uniform
      const int lead = __ffsll((unsigned long long)pend) - 1;
      const u32 kk = (u32)__builtin_amdgcn_readlane((int)k, lead);
      const bool eq = mine && k == kk;
      const u64 em = __ballot(eq);
      if (lane == lead) addw(hist, true, kk, (T)__popcll(em));
      if (eq) mine = false;
    }
    addw(hist, mine, k, (T)1);
  }
  __device__ __forceinline__ void flush(T* __restrict__ hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < kBhSlots; i += blockDim.x)
      if (key[i] != kBhEmpty) atomicAdd(&hist[key[i]], val[i]);
  }
};

}  // namespace dev
}  // namespace lpa
