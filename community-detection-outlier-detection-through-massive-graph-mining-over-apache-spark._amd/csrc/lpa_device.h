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

__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = umax64(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ u32 wave_sum_u32(u32 v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += (u32)__shfl_xor((int)v, off, 64);
  return v;
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

// Wave-aggregated append of claimed slots to an LDS list (one LDS atomic per wave).
__device__ __forceinline__ void list_append(uint16_t* lst, int* lcount, int slot, int lane) {
  const u64 cm = __ballot(slot >= 0);
  if (cm == 0ull) return;
  int base = 0;
  if (lane == 0) base = atomicAdd(lcount, __popcll(cm));
  base = __builtin_amdgcn_readfirstlane(base);
  if (slot >= 0) lst[base + __popcll(cm & ((1ull << lane) - 1ull))] = (uint16_t)slot;
}

}  // namespace dev
}  // namespace lpa
