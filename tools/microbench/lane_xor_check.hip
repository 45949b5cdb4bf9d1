// Checks the DPP / permlane-swap lane exchanges of lpa_lane.h (the row-bin group reductions,
// lpa_iter.hip group_mode_hash) against lane ^ j for j = 1 .. 32 and lane - 1 on one full
// wave.  Built by the csrc Makefile into build/lpa_hip/lane_xor_check; exit status 0 = all
// exchanges match (tests/test_gpu_lane_exchange.py).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "lpa_lane.h"
typedef unsigned u32;
using lpa::lane::lane_prev;
using lpa::lane::lane_xor;
__global__ void k(u32* out) {
  const int lane = threadIdx.x;
  const u32 v = 1000u + (u32)lane;
#pragma unroll
  for (int b = 0; b < 6; ++b) out[b * 64 + lane] = lane_xor(v, 1 << b, lane);
  out[6 * 64 + lane] = lane_prev(v);
}
int main() {
  u32* d;
  if (hipMalloc(&d, 7 * 64 * 4) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  u32 h[7 * 64];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int bad = 0;
  for (int b = 0; b < 6; ++b)
    for (int l = 0; l < 64; ++l)
      if (h[b * 64 + l] != 1000u + (u32)(l ^ (1 << b))) {
        if (bad++ < 10) printf("xor %d lane %d: got %u want %u\n", 1 << b, l, h[b * 64 + l] - 1000u, (u32)(l ^ (1 << b)));
      }
  for (int l = 1; l < 64; ++l)
    if (h[6 * 64 + l] != 1000u + (u32)(l - 1)) {
      if (bad++ < 20) printf("wave_shr lane %d: got %u\n", l, h[6 * 64 + l]);
    }
  printf("lane_xor_check: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
  (void)hipFree(d);
  return bad ? 1 : 0;
}
