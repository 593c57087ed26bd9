// Row-block fp32 MFMA helpers shared by the one-kernel tail (tail_fused.hip) and the xagg head
// GEMMs (gat_xagg.hip): RB (16 or 32) rows of A in LDS times a weight matrix streamed from L2, on
// v_mfma_f32_16x16x4_f32 with the k slots of one instruction taken as k = 16g + 4(l >> 4) + s, so a
// lane's four values of a 16-deep group are one float4 of A (LDS) and, for B = W^T, one float4 of a
// weight row; the weights of group g + 4 are loaded right after group g's MFMAs (a ring of 4).
// C/D: col = l & 15, row = 4(l >> 4) + r.
#pragma once
#include "common.hpp"

namespace hicgat {

constexpr int XS = 516;         // LDS row stride (floats) of the 512-wide buffers
typedef float f32x4 __attribute__((ext_vector_type(4)));

// acc[h][t] (h < RB/16 row halves, t < NT) += A[RB x K] (LDS, row stride lda) x B^T, B = the weight
// rows n0 + 16t + (l & 15) (K columns).  The weights of group g + 4 are loaded right after group g's
// MFMAs, so three groups of MFMAs cover every load (a ring of 4 float4 sets).
template <int RB, int NT, int K>
__device__ __forceinline__ void mfma_rows(const float *__restrict__ As, int lda, const float *__restrict__ W, int n0,
                                          f32x4 (&acc)[RB / 16][NT], int lane) {
  constexpr int G = K / 16, H = RB / 16;
  static_assert(G % 4 == 0, "K: a multiple of 64");
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const float *wrow = W + (size_t)(n0 + li) * K + kq;
  const float *arow = As + li * lda + kq;
  float4 b[4][NT];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int t = 0; t < NT; ++t) b[q][t] = *reinterpret_cast<const float4 *>(wrow + (size_t)16 * t * K + 16 * q);
  for (int g0 = 0; g0 < G; g0 += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = g0 + q;
      float4 a[H];
#pragma unroll
      for (int h = 0; h < H; ++h) a[h] = *reinterpret_cast<const float4 *>(arow + h * 16 * lda + 16 * g);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int h = 0; h < H; ++h) {
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].x, b[q][t].x, acc[h][t], 0, 0, 0);
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].y, b[q][t].y, acc[h][t], 0, 0, 0);
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].z, b[q][t].z, acc[h][t], 0, 0, 0);
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].w, b[q][t].w, acc[h][t], 0, 0, 0);
        }
      if (g + 4 < G) {
#pragma unroll
        for (int t = 0; t < NT; ++t) b[q][t] = *reinterpret_cast<const float4 *>(wrow + (size_t)16 * t * K + 16 * (g + 4));
      }
    }
  }
}

// acc[h][t] += A[RB x K] (LDS) x B, B[k][n] = W[k][n] (W [K][ldw] row-major: dx = dy W): lane l reads
// W[16g + 4(l >> 4) + s][n0 + 16t + (l & 15)] -- 16 consecutive floats per k across the lanes -- with
// the weights of group g + 4 loaded after group g's MFMAs (ring of 4).
template <int RB, int NT, int K>
__device__ __forceinline__ void mfma_rows_t(const float *__restrict__ As, int lda, const float *__restrict__ W, int ldw,
                                            int n0, f32x4 (&acc)[RB / 16][NT], int lane) {
  constexpr int G = K / 16, H = RB / 16;
  static_assert(G % 4 == 0, "K: a multiple of 64");
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const float *wcol = W + (size_t)kq * ldw + n0 + li;
  const float *arow = As + li * lda + kq;
  float b[4][NT][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) b[q][t][j] = wcol[(size_t)(16 * q + j) * ldw + 16 * t];
  for (int g0 = 0; g0 < G; g0 += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = g0 + q;
      float4 a[H];
#pragma unroll
      for (int h = 0; h < H; ++h) a[h] = *reinterpret_cast<const float4 *>(arow + h * 16 * lda + 16 * g);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int h = 0; h < H; ++h) {
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].x, b[q][t][0], acc[h][t], 0, 0, 0);
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].y, b[q][t][1], acc[h][t], 0, 0, 0);
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].z, b[q][t][2], acc[h][t], 0, 0, 0);
          acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[h].w, b[q][t][3], acc[h][t], 0, 0, 0);
        }
      if (g + 4 < G) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) b[q][t][j] = wcol[(size_t)(16 * (g + 4) + j) * ldw + 16 * t];
      }
    }
  }
}

}  // namespace hicgat
