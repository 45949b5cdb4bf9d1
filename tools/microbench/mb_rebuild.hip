// Microbenchmark of the al[] rebuild (al[i] = L[col[i]]) on a synthetic arc array
// whose column multiset follows a given degree sequence (rank-ordered, as the
// build lays vertices out): each arc's column is drawn with probability deg(v)/arcs,
// rows are the rank-ordered degree runs with sorted columns.  Variants locate the
// rebuild's bound (stream floor, plain gathers, LDS hot set, split passes).
//   mb_rebuild <deg.bin (int32 per vertex, descending)> [reps]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
typedef uint32_t u32;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}
__global__ void k_draw(const int64_t* __restrict__ cdeg, int64_t V, int64_t arcs, int32_t* __restrict__ col) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < arcs; i += (int64_t)gridDim.x * 256) {
    const int64_t t = (int64_t)(mix((uint64_t)i * 0x9E3779B97F4A7C15ull + 7) % (uint64_t)arcs);
    int64_t lo = 0, hi = V;  // first v with cdeg[v + 1] > t
    while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (cdeg[mid + 1] > t) hi = mid; else lo = mid + 1; }
    col[i] = (int32_t)lo;
  }
}
__global__ void k_init(int32_t* L, int64_t V) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < V; i += (int64_t)gridDim.x * 256) L[i] = (int32_t)(mix(i) % V);
}
__global__ void k_floor(const int32_t* __restrict__ col, int64_t arcs, int32_t* __restrict__ al) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 512; base + 512 <= arcs; base += nw * 512) {
    int32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_nontemporal_load(col + base + k * 64 + lane);
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(c[k] ^ 1, al + base + k * 64 + lane);
  }
}
template <int kHot, bool kNT>
__global__ __launch_bounds__(1024) void k_hot(const int32_t* __restrict__ col, int64_t arcs, const int32_t* __restrict__ L,
                                              int32_t* __restrict__ al, int32_t lo_col, int32_t hi_col) {
  __shared__ int32_t hot[kHot > 0 ? kHot : 1];
  for (int i = threadIdx.x; i < kHot; i += 1024) hot[i] = L[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 512; base + 512 <= arcs; base += nw * 512) {
    int32_t c[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = kNT ? __builtin_nontemporal_load(col + base + k * 64 + lane) : col[base + k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t x = c[k];
      if (x < lo_col || x >= hi_col) { r[k] = 0; continue; }   // split-pass variants
      r[k] = (kHot > 0 && x < kHot) ? hot[x] : L[x];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t x = c[k];
      if (x < lo_col || x >= hi_col) continue;
      if (kNT) __builtin_nontemporal_store(r[k], al + base + k * 64 + lane);
      else al[base + k * 64 + lane] = r[k];
    }
  }
}
template <int kHot, int kMode>
__global__ __launch_bounds__(1024) void k_hot_nt(const int32_t* __restrict__ col, int64_t arcs, const int32_t* __restrict__ L,
                                                 int32_t* __restrict__ al, int32_t cold) {
  __shared__ int32_t hot[kHot];
  for (int i = threadIdx.x; i < kHot; i += 1024) hot[i] = L[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 512; base + 512 <= arcs; base += nw * 512) {
    int32_t c[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_nontemporal_load(col + base + k * 64 + lane);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t x = c[k];
      if (x < kHot) r[k] = hot[x];
      else if (kMode == 1 ? x >= cold : true) r[k] = __builtin_nontemporal_load(L + x);
      else r[k] = L[x];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(r[k], al + base + k * 64 + lane);
  }
}
// code gathers (MB_CODES=1): labels as 16- or 8-bit codes (a denser gather footprint),
// code -> label through a small dictionary (kDict: global, L2-resident), escape code ->
// the 4-B label; LDS holds the codes of the first kHot slots (the same 160 KB)
template <typename C, int kHot, bool kDict>
__global__ __launch_bounds__(1024) void k_hot_code(const int32_t* __restrict__ col, int64_t arcs,
                                                   const C* __restrict__ code, const int32_t* __restrict__ dict,
                                                   const int32_t* __restrict__ L, int32_t* __restrict__ al) {
  __shared__ C hot[kHot];
  constexpr u32 kEsc = (u32)(C)(~(C)0);
  for (int i = threadIdx.x; i < kHot; i += 1024) hot[i] = code[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 512; base + 512 <= arcs; base += nw * 512) {
    int32_t c[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_nontemporal_load(col + base + k * 64 + lane);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t x = c[k];
      r[k] = (int32_t)(u32)(x < kHot ? hot[x] : code[x]);
    }
    if (kDict) {
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = (u32)r[k] == kEsc ? L[c[k]] : dict[r[k]];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(r[k], al + base + k * 64 + lane);
  }
}
__global__ void k_init_codes(uint16_t* c16, uint8_t* c8, int32_t* dict, int64_t V, int esc_pct16, int esc_pct8) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < V; i += (int64_t)gridDim.x * 256) {
    const uint64_t h = mix(i + 12345);
    c16[i] = (int)(h % 100) < esc_pct16 ? 0xFFFF : (uint16_t)((h >> 8) % 65535);
    c8[i] = (int)((h >> 32) % 100) < esc_pct8 ? 0xFF : (uint8_t)((h >> 40) % 255);
    if (i < 65536) dict[i] = (int32_t)(mix(i) % V);
  }
}
// XCD-split rebuild: workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8);
// XCDs 0-3 gather the arcs whose column is < T (plus the LDS hot set), XCDs 4-7 the
// rest, so each XCD's L2 caches half of the gathered label range.  Every block streams
// col over its group's share of the arcs (col is read twice in all).
__global__ __launch_bounds__(1024) void k_hot_xcd(const int32_t* __restrict__ col, int64_t arcs,
                                                  const int32_t* __restrict__ L, int32_t* __restrict__ al, int32_t T) {
  __shared__ int32_t hot[40960];
  const bool ga = (blockIdx.x & 7) < 4;
  if (ga) for (int i = threadIdx.x; i < 40960; i += 1024) hot[i] = L[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t gb = ((int64_t)(blockIdx.x >> 3) * 4 + ((blockIdx.x & 7) & 3));  // block index within its group
  const int64_t ng = (int64_t)gridDim.x / 2;
  const int64_t nw = ng * (blockDim.x >> 6);
  for (int64_t base = (gb * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 512; base + 512 <= arcs; base += nw * 512) {
    int32_t c[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = __builtin_nontemporal_load(col + base + k * 64 + lane);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t x = c[k];
      const bool mine = ga ? x < T : x >= T;
      r[k] = mine ? (ga && x < 40960 ? hot[x] : L[x]) : 0;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (ga ? c[k] < T : c[k] >= T) __builtin_nontemporal_store(r[k], al + base + k * 64 + lane);
  }
}
// cold list: al[cpos[j]] = L[ccol[j]] for the listed arcs (position-ordered or
// column-ordered lists)
__global__ __launch_bounds__(256) void k_cold_list(const uint32_t* __restrict__ cpos, const int32_t* __restrict__ ccol,
                                                   int64_t n, const int32_t* __restrict__ L, int32_t* __restrict__ al) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    uint32_t p[4]; int32_t c[4], r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { p[k] = __builtin_nontemporal_load(cpos + i + k * stride); c[k] = __builtin_nontemporal_load(ccol + i + k * stride); }
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = L[c[k]];
#pragma unroll
    for (int k = 0; k < 4; ++k) al[p[k]] = r[k];
  }
  for (; i < n; i += stride) al[cpos[i]] = L[ccol[i]];
}
struct IsCold {
  const int32_t* col; int32_t T;
  __host__ __device__ bool operator()(const uint32_t& i) const { return col[i] >= T; }
};
// columns sorted inside each row (rows = degree runs, rank order)
__global__ void k_row_bounds(const int64_t* cdeg, int64_t V, int64_t* rows_off) {}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  if (!f) { printf("no deg file\n"); return 1; }
  std::vector<int32_t> deg;
  int32_t buf[1 << 16]; size_t n;
  while ((n = fread(buf, 4, 1 << 16, f)) > 0) deg.insert(deg.end(), buf, buf + n);
  fclose(f);
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int64_t V = (int64_t)deg.size();
  std::vector<int64_t> cdeg(V + 1, 0);
  for (int64_t v = 0; v < V; ++v) cdeg[v + 1] = cdeg[v] + deg[v];
  const int64_t arcs = cdeg[V] / 512 * 512;
  printf("V %ld arcs %ld\n", (long)V, (long)arcs);
  int64_t* d_cdeg; int32_t *col, *al, *L;
  CK(hipMalloc(&d_cdeg, (V + 1) * 8)); CK(hipMalloc(&col, arcs * 4)); CK(hipMalloc(&al, arcs * 4)); CK(hipMalloc(&L, V * 4));
  CK(hipMemcpy(d_cdeg, cdeg.data(), (V + 1) * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_draw, dim3(8192), dim3(256), 0, 0, d_cdeg, V, arcs, col);
  hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, L, V);
  // sort the columns inside each row: segmented sort over the degree runs
  {
    std::vector<int64_t> off; off.reserve(V + 1);
    for (int64_t v = 0; v <= V && cdeg[v] <= arcs; ++v) off.push_back(cdeg[v]);
    if (off.back() != arcs) off.push_back(arcs);
    const int nseg = (int)off.size() - 1;
    int64_t* d_off; CK(hipMalloc(&d_off, off.size() * 8));
    CK(hipMemcpy(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice));
    // sort in slices of <= 2^30 keys (int offsets inside cub)
    size_t tmp = 0; void* dtmp = nullptr;
    int32_t* tmpk; CK(hipMalloc(&tmpk, std::min<int64_t>(arcs, 1ll << 30) * 4));
    int s0 = 0;
    while (s0 < nseg) {
      int s1 = s0;
      while (s1 < nseg && off[s1 + 1] - off[s0] <= (1ll << 30)) ++s1;
      if (s1 == s0) s1 = s0 + 1;
      const int64_t a0 = off[s0], na = off[s1] - a0;
      std::vector<int> o(s1 - s0 + 1);
      for (int s = s0; s <= s1; ++s) o[s - s0] = (int)(off[s] - a0);
      int* d_o; CK(hipMalloc(&d_o, o.size() * 4)); CK(hipMemcpy(d_o, o.data(), o.size() * 4, hipMemcpyHostToDevice));
      size_t need = 0;
      hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, need, col + a0, tmpk, (int)na, s1 - s0, d_o, d_o + 1);
      if (need > tmp) { if (dtmp) CK(hipFree(dtmp)); CK(hipMalloc(&dtmp, need)); tmp = need; }
      hipcub::DeviceSegmentedRadixSort::SortKeys(dtmp, tmp, col + a0, tmpk, (int)na, s1 - s0, d_o, d_o + 1);
      CK(hipMemcpy(col + a0, tmpk, na * 4, hipMemcpyDeviceToDevice));
      CK(hipFree(d_o));
      s0 = s1;
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(tmpk)); if (dtmp) CK(hipFree(dtmp)); CK(hipFree(d_off));
  }
  int cus = 256; (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto fn) {
    std::vector<float> t;
    for (int k = 0; k < reps + 1; ++k) {
      CK(hipEventRecord(e0, 0)); fn(); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (k) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-40s %9.3f ms  %7.1f G arcs/s\n", name, t[t.size() / 2], arcs / (t[t.size() / 2] * 1e6));
  };
  // share of arcs below some rank thresholds
  for (int64_t T : {40960ll, 1ll << 20, 1ll << 22, 1ll << 23}) if (T < V) printf("arcs with col < %ld: %.1f%%\n", (long)T, 100.0 * cdeg[T] / cdeg[V]);
  const int32_t BIG = 0x7fffffff;
  timeit("floor: stream col -> al", [&] { hipLaunchKernelGGL(k_floor, dim3(cus), dim3(1024), 0, 0, col, arcs, al); });
  // MB_BASIC=1 (PMC calibration passes): the stream floor and the shipped kernel only
  const bool basic = getenv("MB_BASIC") != nullptr;
  if (getenv("MB_XCD")) {
    timeit("hot LDS 40960 (NT) [shipped]", [&] { hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, BIG); });
    for (int32_t T : {131072, 262144, 524288, 1 << 20, 1 << 21}) {
      char nm[80];
      snprintf(nm, 80, "XCD split at %d", T);
      timeit(nm, [&] { hipLaunchKernelGGL(k_hot_xcd, dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, T); });
    }
    return 0;
  }
  if (getenv("MB_CODES")) {
    uint16_t* c16; uint8_t* c8; int32_t* dict;
    CK(hipMalloc(&c16, V * 2)); CK(hipMalloc(&c8, V)); CK(hipMalloc(&dict, 65536 * 4));
    hipLaunchKernelGGL(k_init_codes, dim3(4096), dim3(256), 0, 0, c16, c8, dict, V, 9, 32);
    CK(hipDeviceSynchronize());
    timeit("hot LDS 40960 (NT) [shipped]", [&] { hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, BIG); });
    timeit("u16 codes, LDS 81920, no dict", [&] { hipLaunchKernelGGL((k_hot_code<uint16_t, 81920, false>), dim3(cus), dim3(1024), 0, 0, col, arcs, c16, dict, L, al); });
    timeit("u16 codes, LDS 81920, dict + 9% esc", [&] { hipLaunchKernelGGL((k_hot_code<uint16_t, 81920, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, c16, dict, L, al); });
    timeit("u8 codes, LDS 163840, no dict", [&] { hipLaunchKernelGGL((k_hot_code<uint8_t, 163840, false>), dim3(cus), dim3(1024), 0, 0, col, arcs, c8, dict, L, al); });
    timeit("u8 codes, LDS 163840, dict + 32% esc", [&] { hipLaunchKernelGGL((k_hot_code<uint8_t, 163840, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, c8, dict, L, al); });
    return 0;
  }
  if (basic) {
    timeit("hot LDS 40960 (NT) [shipped]", [&] { hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, BIG); });
    return 0;
  }
  timeit("plain gathers (NT streams)", [&] { hipLaunchKernelGGL((k_hot<0, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, BIG); });
  timeit("hot LDS 40960 (NT) [shipped]", [&] { hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, BIG); });
  timeit("hot LDS 40960 (cached streams)", [&] { hipLaunchKernelGGL((k_hot<40960, false>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, BIG); });
  timeit("hot LDS, 2 blocks/CU grid", [&] { hipLaunchKernelGGL((k_hot<40960, true>), dim3(2 * cus), dim3(1024), 0, 0, col, arcs, L, al, 0, BIG); });
  timeit("hot LDS, all gathers NT", [&] { hipLaunchKernelGGL((k_hot_nt<40960, 2>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0); });
  for (int32_t T : {1 << 19, 1 << 20, 1 << 21, 1 << 22}) {
    if (T >= V) continue;
    char nm[80];
    snprintf(nm, 80, "hot LDS, NT gathers for col >= %d", T);
    timeit(nm, [&] { hipLaunchKernelGGL((k_hot_nt<40960, 1>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, T); });
  }
  for (int32_t T : {1 << 20, 1 << 22, 1 << 23}) {
    if (T >= V) continue;
    char nm[80];
    snprintf(nm, 80, "split at %d: pass A (col < T)", T);
    timeit(nm, [&] { hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, T); });
    snprintf(nm, 80, "split at %d: pass B (col >= T)", T);
    timeit(nm, [&] { hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, T, BIG); });
  }
  // hot pass + cold list: the cold arcs (col >= T) from static (position, column)
  // lists instead of a second col stream
  for (int32_t T : {1 << 20, 1 << 21, 1 << 22}) {
    if (T >= V) continue;
    uint32_t* idx; uint32_t* cp; int32_t* cc; int64_t* nsel;
    CK(hipMalloc(&idx, arcs * 4)); CK(hipMalloc(&nsel, 8));
    hipcub::CountingInputIterator<uint32_t> it(0u);
    size_t need = 0;
    IsCold pred{col, T};
    hipcub::DeviceSelect::If(nullptr, need, it, idx, nsel, (int64_t)arcs, pred);
    void* tmp; CK(hipMalloc(&tmp, need));
    hipcub::DeviceSelect::If(tmp, need, it, idx, nsel, (int64_t)arcs, pred);
    int64_t nc = 0; CK(hipMemcpy(&nc, nsel, 8, hipMemcpyDeviceToHost));
    CK(hipMalloc(&cp, nc * 4)); CK(hipMalloc(&cc, nc * 4));
    std::vector<uint32_t> hi(nc); CK(hipMemcpy(hi.data(), idx, nc * 4, hipMemcpyDeviceToHost));
    std::vector<int32_t> hc(arcs); CK(hipMemcpy(hc.data(), col, arcs * 4, hipMemcpyDeviceToHost));
    std::vector<int32_t> hcc(nc); for (int64_t j = 0; j < nc; ++j) hcc[j] = hc[hi[j]];
    CK(hipMemcpy(cp, hi.data(), nc * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(cc, hcc.data(), nc * 4, hipMemcpyHostToDevice));
    char nm[96];
    snprintf(nm, 96, "hot pass (col < %d) + cold list by position", T);
    timeit(nm, [&] {
      hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, T);
      hipLaunchKernelGGL(k_cold_list, dim3(8192), dim3(256), 0, 0, cp, cc, nc, L, al);
    });
    snprintf(nm, 96, "  cold list alone (%ld arcs, by position)", (long)nc);
    timeit(nm, [&] { hipLaunchKernelGGL(k_cold_list, dim3(8192), dim3(256), 0, 0, cp, cc, nc, L, al); });
    fflush(stdout);
    // column order (CSC of the cold arcs): sequential label reads, scattered writes
    if (nc > 300000000) { CK(hipFree(idx)); CK(hipFree(nsel)); CK(hipFree(tmp)); CK(hipFree(cp)); CK(hipFree(cc)); continue; }
    std::vector<int64_t> ord(nc); for (int64_t j = 0; j < nc; ++j) ord[j] = j;
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return hcc[a] < hcc[b]; });
    std::vector<uint32_t> p2(nc); std::vector<int32_t> c2(nc);
    for (int64_t j = 0; j < nc; ++j) { p2[j] = hi[ord[j]]; c2[j] = hcc[ord[j]]; }
    CK(hipMemcpy(cp, p2.data(), nc * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(cc, c2.data(), nc * 4, hipMemcpyHostToDevice));
    snprintf(nm, 96, "  cold list alone (by column)");
    timeit(nm, [&] { hipLaunchKernelGGL(k_cold_list, dim3(8192), dim3(256), 0, 0, cp, cc, nc, L, al); });
    CK(hipFree(idx)); CK(hipFree(nsel)); CK(hipFree(tmp)); CK(hipFree(cp)); CK(hipFree(cc));
  }
  // column windows: pass k gathers only the arcs whose column lies in
  // [k W, (k + 1) W) (the window's labels stay cache-resident while col streams past)
  for (int64_t W : {1ll << 22, 1ll << 23, 1ll << 24, 1ll << 25}) {
    if (W >= V) continue;
    char nm[80];
    snprintf(nm, 80, "windows of %ld labels (%ld passes)", (long)W, (long)((V + W - 1) / W));
    timeit(nm, [&] {
      for (int64_t lo = 0; lo < V; lo += W) {
        const int32_t hi = (int32_t)std::min<int64_t>(V, lo + W);
        if (lo == 0) hipLaunchKernelGGL((k_hot<40960, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, 0, hi);
        else hipLaunchKernelGGL((k_hot<0, true>), dim3(cus), dim3(1024), 0, 0, col, arcs, L, al, (int32_t)lo, hi);
      }
    });
  }
  return 0;
}
