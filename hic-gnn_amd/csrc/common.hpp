// Shared device helpers for the gfx950 kernels of libhicgat.so (wave64 everywhere).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hicgat.h"

namespace hicgat {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Wave index inside the block, forced into an SGPR so that everything derived from it is scalar.
__device__ __forceinline__ int wave_in_block() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
// Sum over the 32 lanes of each half wave.
__device__ __forceinline__ float half_wave_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Correctly rounded square roots.  v_sqrt_f32 and the default f64 lowering are not IEEE-exact;
// torch's CPU sqrt (and pow(x, 0.5)) is.  One Newton step brings the estimate y within 1 ulp;
// then y-1ulp is the answer iff x <= (y-1ulp)*y, y+1ulp iff x > (y+1ulp)*y (the exact products
// differ from the rounding midpoints' squares by far less than one ulp of x).
__device__ __forceinline__ float sqrt_rn_f32(float x) {
  if (!(x > 0.f) || x == INFINITY) return __builtin_sqrtf(x);
  const bool tiny = x < 0x1.0p-96f;
  const float xs = tiny ? x * 0x1.0p+32f : x;
  float y = __builtin_amdgcn_sqrtf(xs);
  y = fmaf(fmaf(-y, y, xs), 0.5f / y, y);
  const float yd = __int_as_float(__float_as_int(y) - 1), yu = __int_as_float(__float_as_int(y) + 1);
  if (fmaf(-yd, y, xs) <= 0.f) y = yd;
  else if (fmaf(-yu, y, xs) > 0.f) y = yu;
  return tiny ? y * 0x1.0p-16f : y;
}
__device__ __forceinline__ double sqrt_rn_f64(double x) {
  if (!(x > 0.0) || x == (double)INFINITY) return __builtin_sqrt(x);
  const bool tiny = x < 0x1.0p-900;
  const double xs = tiny ? x * 0x1.0p+256 : x;
  double y = (double)__builtin_amdgcn_sqrtf((float)xs);   // ~24-bit start (xs is in float range)
  if (xs > 3.0e38 || xs < 1.0e-37) y = __builtin_sqrt(xs);
  for (int it = 0; it < 3; ++it) y = fma(fma(-y, y, xs), 0.5 / y, y);   // 24 -> 48 -> >53 bits
  const double yd = __longlong_as_double(__double_as_longlong(y) - 1);
  const double yu = __longlong_as_double(__double_as_longlong(y) + 1);
  if (fma(-yd, y, xs) <= 0.0) y = yd;
  else if (fma(-yu, y, xs) > 0.0) y = yu;
  return tiny ? y * 0x1.0p-128 : y;
}

// torch.nn.functional.leaky_relu: x > 0 ? x : x * slope.
__device__ __forceinline__ float lrelu(float x, float slope) { return x > 0.f ? x : x * slope; }

__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ float4 f4_fma(float a, float4 x, float4 acc) {
  acc.x = fmaf(a, x.x, acc.x);
  acc.y = fmaf(a, x.y, acc.y);
  acc.z = fmaf(a, x.z, acc.z);
  acc.w = fmaf(a, x.w, acc.w);
  return acc;
}
// torch.relu: x <= 0 ? 0 : x (NaN passes through).
__device__ __forceinline__ float relu_t(float x) { return x <= 0.f ? 0.f : x; }
__device__ __forceinline__ float4 f4_relu(float4 a) {
  return make_float4(relu_t(a.x), relu_t(a.y), relu_t(a.z), relu_t(a.w));
}
__device__ __forceinline__ float f4_dot(float4 a, float4 b) {
  return fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
}

// "Transpose reduce": every lane holds V values; after the call lane l holds, in v[0], the sum
// over all 64 lanes of value index idx(l) where the bits of idx are taken, most significant
// first, from lane bits 5, 4, ... (V = 16: idx = (l>>5&1)*8 + (l>>4&1)*4 + (l>>3&1)*2 + (l>>2&1)).
// Cost: V-1 shuffles + 2 for the final intra-group sum (vs 6 per value for independent sums).
template <int V>
__device__ __forceinline__ void transpose_reduce(float (&v)[V], int lane) {
  static_assert(V == 16 || V == 8 || V == 4 || V == 2, "transpose_reduce: V must be 2, 4, 8 or 16");
  int mask = 32;
#pragma unroll
  for (int n = V; n > 1; n >>= 1, mask >>= 1) {
    const bool upper = (lane & mask) != 0;
#pragma unroll
    for (int q = 0; q < n / 2; ++q) {
      const float send = upper ? v[q] : v[q + n / 2];
      const float keep = upper ? v[q + n / 2] : v[q];
      v[q] = keep + __shfl_xor(send, mask);
    }
  }
  // remaining lane bits below `mask*2` are still partial: finish the sum across them
#pragma unroll
  for (int o = mask; o > 0; o >>= 1) v[0] += __shfl_xor(v[0], o);
}

// Bijective XCD-aware block remap (cdna_hip_programming.md section 5 T1): the 8 XCDs each get a
// contiguous range of logical blocks, so rows that share neighbours share an L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7, q = nblocks >> 3, r = nblocks & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

}  // namespace hicgat

#define HICGAT_CHECK_LAUNCH()                                   \
  do {                                                          \
    if (hipGetLastError() != hipSuccess) return HICGAT_ELAUNCH; \
  } while (0)
