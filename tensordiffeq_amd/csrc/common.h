// Shared helpers for the gfx950 (CDNA4) kernels of tensordiffeq_amd.
#pragma once
#ifndef __HIPCC_RTC__  // (hipRTC, ops/fused_step.py: the HIP device API is implicit)
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define TDQ_WAVE 64

// 16x16x4 fp32 MFMA: D[16x16] += A[16x4] * B[4x16]
//   lane l supplies A[l&15][l>>4] and B[l>>4][l&15];
//   D/C: lane l, reg r holds D[4*(l>>4)+r][l&15].
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// DPP lane permutations inside a 16-lane row (pure VALU, no LDS traffic)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes that share (l >> 4); every lane of the row gets the total
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

// four 16-lane sums at once (transpose-reduce): lane i of each 16-lane row returns
//   sum over the row of v[(i >> 2) & 3]
// i.e. lanes 0-3 hold the total of v[0], 4-7 of v[1], 8-11 of v[2], 12-15 of v[3].
// 8 DPP adds + 3 selects instead of 4 x 4 DPP adds for four row16_sum calls.
__device__ __forceinline__ float row16_sum4(f32x4 v) {
  const int i = __lane_id() & 15;
  const float m0 = v[0] + dpp<0x140>(v[0]), m1 = v[1] + dpp<0x140>(v[1]);  // row_mirror: i <-> 15 - i
  const float m2 = v[2] + dpp<0x140>(v[2]), m3 = v[3] + dpp<0x140>(v[3]);
  const bool hi8 = (i & 8) != 0;
  const float k0 = hi8 ? m2 : m0, k1 = hi8 ? m3 : m1;
  const float n0 = k0 + dpp<0x141>(k0), n1 = k1 + dpp<0x141>(k1);        // row_half_mirror
  float r = (i & 4) ? n1 : n0;
  r += dpp<0x4E>(r);                                                       // xor 2
  r += dpp<0xB1>(r);                                                       // xor 1
  return r;
}

// sum over the 4 lanes l, l^16, l^32, l^48 (same point, different feature groups)
__device__ __forceinline__ float col4_sum(float v) {
#ifdef TDQ_COL4_BPERMUTE
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
#else
  // the same two butterfly steps on the CDNA4 row-swap instructions (VALU, not the LDS crossbar of
  // ds_bpermute): v_permlane16_swap pairs 16-lane rows 0-1 and 2-3, v_permlane32_swap the halves
  const int lane = __lane_id();
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v += __uint_as_float((lane & 16) ? a[0] : a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return v + __uint_as_float((lane & 32) ? b[0] : b[1]);
#endif
}

#define TDQ_CHECK_LAUNCH() \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
