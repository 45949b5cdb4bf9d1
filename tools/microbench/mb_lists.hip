// Microbenchmark of the frontier-list scan (k_frontier_lists) on a C3-sized flag
// array: the kernel as shipped vs pure scans, to locate its fixed cost.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
typedef uint32_t u32;
#define LPA_NBINS 13
struct BinBounds { int64_t b[LPA_NBINS + 1]; };
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int kFcntUnits = LPA_NBINS;  // fcnt[] slot of the unit count
constexpr int kListSub = 8;            // 16-byte flag groups per thread, all loaded up front
constexpr int kListTile = 256 * 16 * kListSub;  // flags per block (32 K: few global atomics per count)
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
                                                        int64_t nblk_rows, int mode = 0) {
  __shared__ int32_t lcnt[LPA_NBINS + 1];
  __shared__ int32_t lpos[LPA_NBINS + 1];
  __shared__ int32_t gbase[LPA_NBINS + 1];
  __shared__ int64_t sbb[LPA_NBINS + 1];
  if (blockIdx.x == 0 && threadIdx.x < LPA_NBINS + 1) fcnt_next[threadIdx.x] = 0;
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

__global__ void k_set(uint8_t* f, const int32_t* idx, int n) {
  int i = blockIdx.x * 256 + threadIdx.x; if (i < n) f[idx[i]] = 1;
}
__global__ __launch_bounds__(256) void k_scan_only(const uint4* f, int64_t n16, u32* out) {
  u32 acc = 0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    uint4 r = f[i]; acc |= r.x | r.y | r.z | r.w; }
  if (acc) out[0] = acc;
}
__global__ __launch_bounds__(256) void k_scan_tile(const uint4* f, int64_t n16, u32* out) {
  uint4 r[8]; const int64_t t0 = (int64_t)blockIdx.x * 2048;
  #pragma unroll
  for (int j = 0; j < 8; ++j) { int64_t i = t0 + j * 256 + threadIdx.x; r[j] = i < n16 ? f[i] : make_uint4(0,0,0,0); }
  u32 acc = 0;
  #pragma unroll
  for (int j = 0; j < 8; ++j) acc |= r[j].x | r[j].y | r[j].z | r[j].w;
  if (acc) out[0] = acc;
}
__global__ void k_empty(u32* out) { if (threadIdx.x == 1023) out[1] = 1; }
int main() {
  const int64_t S = 1 << 24, NU = 1 << 20;
  const int nset = 40000, nuset = 1000;
  uint8_t *rd, *ud; int32_t *flist, *ulist, *fcnt, *fr_all, *idx, *uidx; u32* out;
  CK(hipMalloc(&rd, S)); CK(hipMalloc(&ud, NU)); CK(hipMalloc(&flist, S * 4)); CK(hipMalloc(&ulist, NU * 4));
  CK(hipMalloc(&fcnt, 32 * 4)); CK(hipMalloc(&fr_all, 8)); CK(hipMalloc(&idx, nset * 4)); CK(hipMalloc(&uidx, nuset * 4));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(rd, 0, S)); CK(hipMemset(ud, 0, NU)); CK(hipMemset(fr_all, 0, 8)); CK(hipMemset(fcnt, 0, 128));
  std::mt19937 rng(1); std::vector<int32_t> h(nset), hu(nuset);
  for (auto& x : h) x = rng() % S; for (auto& x : hu) x = rng() % NU;
  CK(hipMemcpy(idx, h.data(), nset * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(uidx, hu.data(), nuset * 4, hipMemcpyHostToDevice));
  BinBounds bb; int64_t bounds[LPA_NBINS + 1] = {0, 20000, 60000, 150000, 400000, 900000, 1800000, 3000000, 4500000, 6000000, 7500000, 9000000, 10500000, S};
  for (int i = 0; i <= LPA_NBINS; ++i) bb.b[i] = bounds[i];
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int64_t nbr = (S + kListTile - 1) / kListTile, nbu = (NU + kListTile - 1) / kListTile;
  auto timeit = [&](const char* name, auto fn, bool reset) {
    float tot = 0; const int it = 50;
    for (int k = 0; k < it + 5; ++k) {
      if (reset) { hipLaunchKernelGGL(k_set, dim3((nset + 255) / 256), dim3(256), 0, 0, rd, idx, nset);
                   hipLaunchKernelGGL(k_set, dim3((nuset + 255) / 256), dim3(256), 0, 0, ud, uidx, nuset);
                   hipMemsetAsync(fcnt, 0, 128, 0); }
      hipEventRecord(e0, 0); fn(); hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); if (k >= 5) tot += ms;
    }
    printf("%-28s %8.2f us\n", name, tot / it * 1000);
  };
  timeit("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, out); }, false);
  timeit("lists (set+clear)", [&] { hipLaunchKernelGGL(k_frontier_lists, dim3(nbr + nbu), dim3(256), 0, 0, rd, S, ud, NU, bb, fr_all, flist, ulist, fcnt, fcnt + 16, nbr); }, true);
  timeit("lists (all clear)", [&] { hipLaunchKernelGGL(k_frontier_lists, dim3(nbr + nbu), dim3(256), 0, 0, rd, S, ud, NU, bb, fr_all, flist, ulist, fcnt, fcnt + 16, nbr); }, false);
  timeit("scan grid-stride 2048 blk", [&] { hipLaunchKernelGGL(k_scan_only, dim3(2048), dim3(256), 0, 0, (const uint4*)rd, S / 16, out); }, false);
  timeit("scan tile 8/thread", [&] { hipLaunchKernelGGL(k_scan_tile, dim3(S / 16 / 2048), dim3(256), 0, 0, (const uint4*)rd, S / 16, out); }, false);
  timeit("scan tile after set", [&] { hipLaunchKernelGGL(k_scan_tile, dim3(S / 16 / 2048), dim3(256), 0, 0, (const uint4*)rd, S / 16, out); }, true);
  for (int mode : {0}) {
    char nm[64]; snprintf(nm, 64, "lists mode %d (1=noatom 2=nolist 4=noclr)", mode);
    timeit(nm, [&] { hipLaunchKernelGGL(k_frontier_lists, dim3(nbr + nbu), dim3(256), 0, 0, rd, S, ud, NU, bb, fr_all, flist, ulist, fcnt, fcnt + 16, nbr, mode); }, true);
  }
  int32_t hc[16]; CK(hipMemcpy(hc, fcnt, 64, hipMemcpyDeviceToHost));
  long tot = 0; for (int i = 0; i < 14; ++i) tot += hc[i]; printf("listed %ld (last reset %d+%d)\n", tot, nset, nuset);
  return 0;
}
