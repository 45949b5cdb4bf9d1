// Checks the DPP / permlane-swap lane exchanges used by group_mode_sort (lpa_iter.hip)
// against lane ^ j for j = 1 .. 32 on one full wave.  Build: hipcc --offload-arch=gfx950
// -O3 lane_xor_check.hip -o lane_xor_check; exit status 0 = all exchanges match.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned u32;
template <int kCtrl>
__device__ __forceinline__ u32 dpp_u32(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}
__device__ __forceinline__ u32 lane_xor(u32 v, int j, int lane) {
  if (j == 1) return dpp_u32<0xB1>(v);
  if (j == 2) return dpp_u32<0x4E>(v);
  if (j == 4) {
    const u32 dn = dpp_u32<0x124>(v);
    const u32 up = dpp_u32<0x12C>(v);
    return (lane & 4) ? dn : up;
  }
  if (j == 8) return dpp_u32<0x128>(v);
  if (j == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? (u32)r[0] : (u32)r[1];
  }
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (lane & 32) ? (u32)r[0] : (u32)r[1];
}
__global__ void k(u32* out) {
  const int lane = threadIdx.x;
  const u32 v = 1000u + (u32)lane;
#pragma unroll
  for (int b = 0; b < 6; ++b) out[b * 64 + lane] = lane_xor(v, 1 << b, lane);
  out[6 * 64 + lane] = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
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
  hipFree(d);
  return bad ? 1 : 0;
}
