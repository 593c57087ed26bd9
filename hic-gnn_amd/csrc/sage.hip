// SAGEConv of the HiC-GNN baseline model `Net`.
//
// Reference: layers.py:41-79 (SAGEConv.adjust_weights / forward / message_and_aggregate) on the
// adjacency built by utils.load_input (utils.py:29-73):
//   s_i   = sum_j w_ij                      adj_t.sum(dim=0)   (scatter_add, rows ascending)
//   n_ij  = (1 / s_i) * w_ij                matmul(diag(1/s), adj_t), fp32 product
//   agg_i = sum_j n_ij x_j                  matmul(norm_mat, x, reduce='add')
//   out   = lin_l(agg) + lin_r(x.long().float())      (the x.long() truncation quirk, :64)
// w_ij is the networkx edge weight cast to float32 (utils.py:45-52): for i != j the lower-triangle
// entry A[max, min] when it is non-zero, else A[min, max] (row-major insertion overwrites).
//
// Layout: the device CSR of the GAT path (int32, self loops inserted, sorted columns) plus one
// float32 weight per CSR entry (0 on the self loops, which the kernels skip) and inv_deg[N].
// hicgat_sage_agg writes [agg_i | trunc(x_i)] side by side into z [N, 2F] so that lin_l and lin_r
// become one GEMM against [W_l | W_r] (K = 2F).  One wave per row gathers 2 KiB x rows with the
// neighbour id and its weight broadcast through SGPRs; the transposed product (d agg -> d x) uses
// the CSR symmetry: row j's entries are the (i, j) edges, weighted by inv_deg of the neighbour.
#include "common.hpp"

namespace hicgat {

// w per CSR entry + s_i + 1/s_i; one thread per row, entries summed in ascending column order.
__global__ __launch_bounds__(256) void sage_weights_kernel(const double *__restrict__ A, int N, int64_t lda,
                                                           const int *__restrict__ rowptr,
                                                           const int *__restrict__ col, float *__restrict__ w,
                                                           float *__restrict__ inv_deg) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  float s = 0.f;
  for (int e = rowptr[i]; e < rowptr[i + 1]; ++e) {
    const int j = col[e];
    float v = 0.f;
    if (j != i) {
      const int lo = min(i, j), hi = max(i, j);
      const double a = A[(size_t)hi * lda + lo];
      v = (float)(a != 0.0 ? a : A[(size_t)lo * lda + hi]);
      s += v;
    }
    w[e] = v;
  }
  inv_deg[i] = 1.0f / s;   // IEEE division (HIP default); s == 0 only for rows without edges
}

// z[i, 0:F] = sum_e (inv[i or j] * w[e]) * x[col[e]];  if TRUNC: z[i, F:2F] = trunc(x[i]).
// Fast path F = 512 (two float4 per lane).
template <bool TRANSPOSE, bool TRUNC>
__global__ __launch_bounds__(256) void sage_agg_f512_kernel(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                            const float *__restrict__ w,
                                                            const float *__restrict__ inv_deg, int row_begin,
                                                            int row_end, const float *__restrict__ x,
                                                            float *__restrict__ z, int64_t ldz) {
  constexpr int U = 4;
  const int lane = lane_id();
  const int i = row_begin + xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_in_block();
  if (i >= row_end) return;
  const int beg = rowptr[i], end = rowptr[i + 1];
  const float own = inv_deg[i];
  const float4 *x4 = reinterpret_cast<const float4 *>(x);
  float4 acc0 = make_float4(0.f, 0.f, 0.f, 0.f), acc1 = acc0;
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    int j = i;
    float p = 0.f;
    if (e < end) {
      j = col[e];
      if (j != i) p = (TRANSPOSE ? inv_deg[j] : own) * w[e];
    }
    const int cnt = min(64, end - base);
    for (int k = 0; k < cnt; k += U) {
      float4 v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t jj = (size_t)readlane_i(j, k + u);
        v0[u] = x4[jj * 128 + lane];
        v1[u] = x4[jj * 128 + 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float pu = readlane_f(p, k + u);
        acc0 = f4_fma(pu, v0[u], acc0);
        acc1 = f4_fma(pu, v1[u], acc1);
      }
    }
  }
  float4 *z4 = reinterpret_cast<float4 *>(z + (size_t)i * ldz);
  z4[lane] = acc0;
  z4[64 + lane] = acc1;
  if (TRUNC) {
    const float4 a = x4[(size_t)i * 128 + lane], b = x4[(size_t)i * 128 + 64 + lane];
    z4[128 + lane] = make_float4(truncf(a.x), truncf(a.y), truncf(a.z), truncf(a.w));
    z4[192 + lane] = make_float4(truncf(b.x), truncf(b.y), truncf(b.z), truncf(b.w));
  }
}

// Any F: lane owns columns lane, lane + 64, ...; neighbours one at a time.
template <bool TRANSPOSE, bool TRUNC>
__global__ __launch_bounds__(256) void sage_agg_generic_kernel(const int *__restrict__ rowptr,
                                                               const int *__restrict__ col, const float *__restrict__ w,
                                                               const float *__restrict__ inv_deg, int row_begin,
                                                               int row_end, int F, const float *__restrict__ x,
                                                               float *__restrict__ z, int64_t ldz) {
  const int lane = lane_id();
  const int i = row_begin + xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_in_block();
  if (i >= row_end) return;
  const int beg = rowptr[i], end = rowptr[i + 1];
  const float own = inv_deg[i];
  for (int c0 = 0; c0 < F; c0 += 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int e = beg; e < end; ++e) {
      const int j = col[e];
      if (j == i) continue;
      const float p = (TRANSPOSE ? inv_deg[j] : own) * w[e];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c0 + q * 64 + lane;
        if (c < F) acc[q] = fmaf(p, x[(size_t)j * F + c], acc[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + q * 64 + lane;
      if (c < F) {
        z[(size_t)i * ldz + c] = acc[q];
        if (TRUNC) z[(size_t)i * ldz + F + c] = truncf(x[(size_t)i * F + c]);
      }
    }
  }
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_sage_weights(const double *A, int N, int64_t lda, const int32_t *rowptr, const int32_t *col,
                                   float *weights, float *inv_deg, hicgat_stream_t stream) {
  if (N < 0 || lda < N) return HICGAT_EINVAL;
  if (N == 0) return HICGAT_OK;
  if (!A || !rowptr || !col || !weights || !inv_deg) return HICGAT_EINVAL;
  hipLaunchKernelGGL(sage_weights_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, A, N, lda,
                     rowptr, col, weights, inv_deg);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_sage_agg(const int32_t *rowptr, const int32_t *col, const float *weights, const float *inv_deg,
                               int N, int F, int row_begin, int row_end, const float *x, int transpose,
                               int write_trunc, float *z, int64_t ldz, hicgat_stream_t stream) {
  if (N < 0 || F <= 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (ldz < (write_trunc ? 2 * (int64_t)F : (int64_t)F)) return HICGAT_EINVAL;
  if (row_begin == row_end) return HICGAT_OK;
  if (!rowptr || !col || !weights || !inv_deg || !x || !z) return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  const dim3 grid((rows + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  const bool fast = F == 512 && (ldz % 4) == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(z)) & 15) == 0;
#define HICGAT_SAGE_LAUNCH(T, R)                                                                                   \
  do {                                                                                                             \
    if (fast)                                                                                                      \
      hipLaunchKernelGGL((sage_agg_f512_kernel<T, R>), grid, block, 0, s, rowptr, col, weights, inv_deg, row_begin, \
                         row_end, x, z, ldz);                                                                      \
    else                                                                                                           \
      hipLaunchKernelGGL((sage_agg_generic_kernel<T, R>), grid, block, 0, s, rowptr, col, weights, inv_deg,        \
                         row_begin, row_end, F, x, z, ldz);                                                        \
  } while (0)
  if (transpose) {
    if (write_trunc) HICGAT_SAGE_LAUNCH(true, true);
    else HICGAT_SAGE_LAUNCH(true, false);
  } else {
    if (write_trunc) HICGAT_SAGE_LAUNCH(false, true);
    else HICGAT_SAGE_LAUNCH(false, false);
  }
#undef HICGAT_SAGE_LAUNCH
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
