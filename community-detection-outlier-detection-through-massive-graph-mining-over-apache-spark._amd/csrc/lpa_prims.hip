// Device-wide primitives for graph construction: LSD radix sort of 64-bit
// keys and exclusive scans.  Build-time only (not on the per-superstep path);
// written for wave64 (ballot-based digit ranking, 64-bit lane masks).
#include <stdarg.h>
#include <stdio.h>

#include <mutex>

#include "lpa_internal.h"

namespace lpa {

namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;  // keys per block per radix pass

// ---------------------------------------------------------------------------
// block-level helpers (256 threads = 4 waves)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    T o = __shfl_up(v, off, 64);
    if (lane >= off) v += o;
  }
  return v;
}

// exclusive scan over the block; returns the thread's exclusive prefix and the block total
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* total) {
  __shared__ T wsum[kThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T incl = wave_incl_scan(v, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  T before = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) {
    if (i < w) before += wsum[i];
    tot += wsum[i];
  }
  __syncthreads();
  *total = tot;
  return before + incl - v;
}

// ---------------------------------------------------------------------------
// exclusive scan: reduce -> (recursive scan of partials) -> apply
// ---------------------------------------------------------------------------
template <typename Tin, typename Tout>
__global__ __launch_bounds__(kThreads) void k_scan_reduce(const Tin* __restrict__ in, int64_t n,
                                                          Tout* __restrict__ part) {
  const int64_t base = (int64_t)blockIdx.x * kTile;
  Tout s = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    int64_t idx = base + (int64_t)i * kThreads + threadIdx.x;
    if (idx < n) s += (Tout)in[idx];
  }
  Tout tot;
  block_excl_scan<Tout>(s, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(kThreads) void k_scan_apply(const Tin* __restrict__ in, int64_t n,
                                                         Tout* __restrict__ out,
                                                         const Tout* __restrict__ part_excl) {
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
  Tout v[kItems];
  Tout loc = 0;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    int64_t idx = base + j;
    v[j] = idx < n ? (Tout)in[idx] : (Tout)0;
    loc += v[j];
  }
  Tout tot;
  Tout run = block_excl_scan<Tout>(loc, &tot) + (part_excl ? part_excl[blockIdx.x] : (Tout)0);
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    int64_t idx = base + j;
    if (idx < n) out[idx] = run;
    run += v[j];
    if (idx == n - 1) out[n] = run;  // grand total
  }
}

// Byte marks -> u32 positions (the outlier stage's L2 sub-graph marks, hundreds of
// millions of bytes): the generic form's per-thread runs of 16 single-byte loads and
// 16 strided 4-B stores ran at ~1/6 of the stream rate (1.23 ms per scan at C3); here a
// thread loads its 16 bytes as one 16-B vector, and the block's 4096 positions leave
// through LDS in coalesced rows.  in / out must be 16-B aligned (allocation starts).
__device__ __forceinline__ u32 sum_bytes(uint4 x) {
  u32 t = 0;
  const u32 w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32 h = (w[k] & 0x00FF00FFu) + ((w[k] >> 8) & 0x00FF00FFu);
    t += (h & 0xFFFFu) + (h >> 16);
  }
  return t;
}
__device__ __forceinline__ uint4 load16_u8(const uint8_t* __restrict__ in, int64_t base, int64_t n) {
  if (base + 16 <= n) return *reinterpret_cast<const uint4*>(in + base);
  u32 w[4] = {0u, 0u, 0u, 0u};
  for (int j = 0; j < 16; ++j)
    if (base + j < n) w[j >> 2] |= (u32)in[base + j] << (8 * (j & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}
__global__ __launch_bounds__(kThreads) void k_scan_reduce_u8(const uint8_t* __restrict__ in, int64_t n,
                                                             u32* __restrict__ part) {
  static_assert(kItems == 16, "one 16-B vector per thread");
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
  u32 tot;
  block_excl_scan<u32>(sum_bytes(load16_u8(in, base, n)), &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}
__global__ __launch_bounds__(kThreads) void k_scan_apply_u8(const uint8_t* __restrict__ in, int64_t n,
                                                            u32* __restrict__ out, const u32* __restrict__ part_excl) {
  __shared__ u32 stage[kTile];
  const int64_t b0 = (int64_t)blockIdx.x * kTile;
  const uint4 x = load16_u8(in, b0 + (int64_t)threadIdx.x * kItems, n);
  u32 tot;
  u32 run = block_excl_scan<u32>(sum_bytes(x), &tot) + (part_excl ? part_excl[blockIdx.x] : 0u);
  const u32 w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    stage[threadIdx.x * kItems + j] = run;
    run += (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int64_t idx = b0 + (int64_t)j * kThreads + threadIdx.x;
    if (idx < n) out[idx] = stage[j * kThreads + threadIdx.x];
  }
  // grand total: the thread holding element n - 1
  const int64_t last = n - 1 - b0;
  if (last >= 0 && last < kTile && (int)(last / kItems) == (int)threadIdx.x) {
    const int j = (int)(last % kItems);
    out[n] = stage[last] + ((w[j >> 2] >> (8 * (j & 3))) & 0xFFu);
  }
}

template <typename Tin, typename Tout>
int scan_impl(const Tin* in, Tout* out, int64_t n, hipStream_t s) {
  if (n <= 0) {
    LPA_HIP(hipMemsetAsync(out, 0, sizeof(Tout), s));
    return LPA_OK;
  }
  const int64_t nblk = (n + kTile - 1) / kTile;
  if (nblk == 1) {
    hipLaunchKernelGGL((k_scan_apply<Tin, Tout>), dim3(1), dim3(kThreads), 0, s, in, n, out,
                       (const Tout*)nullptr);
    LPA_HIP(hipGetLastError());
    return LPA_OK;
  }
  Tout* part = nullptr;
  Tout* partx = nullptr;
  LPA_TRY(tmp_alloc((void**)&part, sizeof(Tout) * nblk, s));
  LPA_TRY(tmp_alloc((void**)&partx, sizeof(Tout) * (nblk + 1), s));
  hipLaunchKernelGGL((k_scan_reduce<Tin, Tout>), dim3((unsigned)nblk), dim3(kThreads), 0, s, in,
                     n, part);
  LPA_HIP(hipGetLastError());
  int rc = scan_impl<Tout, Tout>(part, partx, nblk, s);
  if (rc == LPA_OK) {
    hipLaunchKernelGGL((k_scan_apply<Tin, Tout>), dim3((unsigned)nblk), dim3(kThreads), 0, s, in,
                       n, out, (const Tout*)partx);
    LPA_HIP(hipGetLastError());
  }
  tmp_free(part, s);
  tmp_free(partx, s);
  return rc;
}

// ---------------------------------------------------------------------------
// LSD radix sort, 8-bit digits, stable.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_rs_hist(const u64* __restrict__ keys, int64_t n,
                                                      int shift, u32* __restrict__ hist,
                                                      int64_t nblk) {
  __shared__ u32 cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int lane = threadIdx.x & 63;
#pragma unroll 4
  for (int i = 0; i < kItems; ++i) {
    int64_t idx = base + (int64_t)i * kThreads + threadIdx.x;
    bool ok = idx < n;
    u32 dg = ok ? (u32)((keys[idx] >> shift) & 255u) : 0u;
    // wave-aggregate lanes with equal digits: one LDS atomic per distinct digit
    u64 peers = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      bool bit = (dg >> b) & 1u;
      u64 bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    if (ok && (peers & ((1ull << lane) - 1ull)) == 0) atomicAdd(&cnt[dg], (u32)__popcll(peers));
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nblk + blockIdx.x] = cnt[threadIdx.x];
}

// Scatter of one pass: the tile's keys are first ranked stably into LDS in digit
// order (the block's per-digit counts come from k_rs_hist), then written out in
// LDS order, so consecutive lanes write consecutive addresses of one digit's run
// (a direct per-key scatter spread every 256-key step over up to 256 runs).
__global__ __launch_bounds__(kThreads) void k_rs_scatter(const u64* __restrict__ in,
                                                         u64* __restrict__ out, int64_t n,
                                                         int shift, const u32* __restrict__ offs,
                                                         const u32* __restrict__ hist, int64_t nblk) {
  __shared__ u64 sk[kTile];
  __shared__ u32 lstart[256];  // local (in-tile) start of each digit's run
  __shared__ u32 run[256];     // next local slot of each digit
  __shared__ u32 gofs[256];    // the block's global start of each digit's run
  __shared__ u32 wsum[kThreads / 64];
  __shared__ u32 wcnt[kThreads / 64][256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  gofs[tid] = offs[(int64_t)tid * nblk + blockIdx.x];
  // exclusive prefix of the block's digit counts: wave scans, then wave totals
  const u32 c = hist[(int64_t)tid * nblk + blockIdx.x];
  u32 incl = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const u32 o = (u32)__shfl_up((int)incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) wsum[w] = incl;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) wcnt[i][tid] = 0;
  __syncthreads();
  u32 wbase = 0;
  for (int ww = 0; ww < w; ++ww) wbase += wsum[ww];
  lstart[tid] = wbase + incl - c;
  run[tid] = wbase + incl - c;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int64_t nv64 = n - base;
  const int nvalid = nv64 < kTile ? (int)nv64 : kTile;
  const u64 lt = (1ull << lane) - 1ull;
  for (int i = 0; i < kItems; ++i) {
    const int q = i * kThreads + tid;
    const bool ok = q < nvalid;
    const u64 k = ok ? in[base + q] : 0ull;
    const u32 dg = (u32)((k >> shift) & 255u);
    u64 peers = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      bool bit = (dg >> b) & 1u;
      u64 bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const u32 rank = (u32)__popcll(peers & lt);
    if (ok && rank == 0) wcnt[w][dg] = (u32)__popcll(peers);
    __syncthreads();
    if (ok) {
      u32 pos = run[dg] + rank;
      for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][dg];
      sk[pos] = k;
    }
    __syncthreads();
    u32 tot = 0;
#pragma unroll
    for (int ww = 0; ww < kThreads / 64; ++ww) {
      tot += wcnt[ww][tid];
      wcnt[ww][tid] = 0;
    }
    run[tid] += tot;
    __syncthreads();
  }
  for (int i = 0; i < kItems; ++i) {
    const int q = i * kThreads + tid;
    if (q < nvalid) {
      const u64 k = sk[q];
      const u32 dg = (u32)((k >> shift) & 255u);
      out[gofs[dg] + (u32)q - lstart[dg]] = k;
    }
  }
}

}  // namespace

// Stream-ordered scratch on the device's default memory pool, whose release threshold
// is raised once per device so that repeated calls reuse the memory (the pool is
// trimmed when a handle is destroyed): hipFree synchronised the device on every
// temporary -- 530 frees, 345 ms of host time in the C3 outlier profile.
int tmp_alloc(void** p, size_t bytes, hipStream_t s) {
  static std::once_flag once[64];
  int dev = 0;
  LPA_HIP(hipGetDevice(&dev));
  if (dev >= 0 && dev < 64)
    std::call_once(once[dev], [dev]() {
      hipMemPool_t pool = nullptr;
      if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess && pool) {
        uint64_t thr = UINT64_MAX;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
      }
    });
  hipError_t e = hipMallocAsync(p, bytes > 0 ? bytes : 1, s);
  if (e != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();
    set_error("hipMallocAsync(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
    return LPA_ENOMEM;
  }
  return LPA_OK;
}

void tmp_free(void* p, hipStream_t s) {
  if (p) (void)hipFreeAsync(p, s);
}

void tmp_trim(int device) {
  hipMemPool_t pool = nullptr;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess && pool) (void)hipMemPoolTrimTo(pool, 0);
}

int bits_for(uint64_t maxval) { return maxval == 0 ? 0 : 64 - __builtin_clzll(maxval); }

int exclusive_scan_i32_i64(const int32_t* in, int64_t* out, int64_t n, hipStream_t s) {
  return scan_impl<int32_t, int64_t>(in, out, n, s);
}

int exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s) {
  return scan_impl<int64_t, int64_t>(in, out, n, s);
}

int exclusive_scan_u8_u32(const uint8_t* in, uint32_t* out, int64_t n, hipStream_t s) {
  if (n <= 0 || ((uintptr_t)in & 15u) || ((uintptr_t)out & 15u)) return scan_impl<uint8_t, u32>(in, out, n, s);
  const int64_t nblk = (n + kTile - 1) / kTile;
  if (nblk == 1) {
    hipLaunchKernelGGL(k_scan_apply_u8, dim3(1), dim3(kThreads), 0, s, in, n, out, (const u32*)nullptr);
    LPA_HIP(hipGetLastError());
    return LPA_OK;
  }
  u32* part = nullptr;
  u32* partx = nullptr;
  LPA_TRY(tmp_alloc((void**)&part, sizeof(u32) * nblk, s));
  LPA_TRY(tmp_alloc((void**)&partx, sizeof(u32) * (nblk + 1), s));
  hipLaunchKernelGGL(k_scan_reduce_u8, dim3((unsigned)nblk), dim3(kThreads), 0, s, in, n, part);
  LPA_HIP(hipGetLastError());
  int rc = scan_impl<u32, u32>(part, partx, nblk, s);
  if (rc == LPA_OK) {
    hipLaunchKernelGGL(k_scan_apply_u8, dim3((unsigned)nblk), dim3(kThreads), 0, s, in, n, out, (const u32*)partx);
    LPA_HIP(hipGetLastError());
  }
  tmp_free(part, s);
  tmp_free(partx, s);
  return rc;
}

int radix_sort_u64(u64* keys, u64* tmp, int64_t n, const int* shifts, int nshifts,
                   hipStream_t s) {
  if (n <= 1 || nshifts == 0) return LPA_OK;
  if (n >= (int64_t)UINT32_MAX) {
    set_error("radix_sort_u64: %lld keys exceed the 32-bit offset range", (long long)n);
    return LPA_EINVAL;
  }
  const int64_t nblk = (n + kTile - 1) / kTile;
  const int64_t nh = 256 * nblk;
  u32* hist = nullptr;
  u32* offs = nullptr;
  LPA_TRY(tmp_alloc((void**)&hist, sizeof(u32) * nh, s));
  LPA_TRY(tmp_alloc((void**)&offs, sizeof(u32) * (nh + 1), s));
  u64* a = keys;
  u64* b = tmp;
  int rc = LPA_OK;
  for (int p = 0; p < nshifts && rc == LPA_OK; ++p) {
    hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)nblk), dim3(kThreads), 0, s, a, n, shifts[p],
                       hist, nblk);
    LPA_HIP(hipGetLastError());
    rc = scan_impl<u32, u32>(hist, offs, nh, s);
    if (rc != LPA_OK) break;
    hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)nblk), dim3(kThreads), 0, s, a, b, n,
                       shifts[p], offs, hist, nblk);
    LPA_HIP(hipGetLastError());
    u64* t = a;
    a = b;
    b = t;
  }
  if (rc == LPA_OK && a != keys) LPA_HIP(hipMemcpyAsync(keys, a, sizeof(u64) * n, hipMemcpyDeviceToDevice, s));
  tmp_free(hist, s);
  tmp_free(offs, s);
  return rc;
}

}  // namespace lpa
