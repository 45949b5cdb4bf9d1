// Cross-lane exchanges of the row-bin group reductions (group_mode_hash, lpa_iter.hip),
// kept in a header of their own so tools/microbench/lane_xor_check.hip (run by
// tests/test_gpu_lane_exchange.py) checks the very function the kernels use.
#pragma once

#include <hip/hip_runtime.h>

namespace lpa {
namespace lane {

template <int kCtrl>
__device__ __forceinline__ unsigned dpp(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}

// v of lane ^ j for a compile-time j (every call is in a fully unrolled loop over a
// full wave) without the LDS crossbar of ds_bpermute: DPP inside a 16-lane row (j = 1, 2
// quad permutes; j = 8 one row rotation; j = 4 two rotations and a select), the gfx950
// v_permlane16/32_swap across rows (j = 16, 32: each swap leaves one copy of the
// partner row / half in one of its two results)
__device__ __forceinline__ unsigned lane_xor(unsigned v, int j, int lane) {
  if (j == 1) return dpp<0xB1>(v);  // quad_perm [1,0,3,2]
  if (j == 2) return dpp<0x4E>(v);  // quad_perm [2,3,0,1]
  if (j == 4) {
    const unsigned dn = dpp<0x124>(v);  // row_ror:4  -> lane - 4
    const unsigned up = dpp<0x12C>(v);  // row_ror:12 -> lane + 4
    return (lane & 4) ? dn : up;
  }
  if (j == 8) return dpp<0x128>(v);  // row_ror:8 -> lane ^ 8
  if (j == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? (unsigned)r[0] : (unsigned)r[1];
  }
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (lane & 32) ? (unsigned)r[0] : (unsigned)r[1];
}

// v of lane - 1 (lane 0: 0), DPP wave_shr:1
__device__ __forceinline__ unsigned lane_prev(unsigned v) { return dpp<0x138>(v); }

}  // namespace lane
}  // namespace lpa
