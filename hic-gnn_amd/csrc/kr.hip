// Knight-Ruiz matrix balancing on gfx950: the O(N^2) parts of the
// reference's KRnorm (r_utils.R:1-93), which runs once per run between convert_to_matrix and
// load_input (HiC-GNN_main.py:76-89).  The O(N) CG bookkeeping of the algorithm stays on the host
// side of the caller (hicgat/kr.py); what touches the N x N matrix is here:
//
//   hicgat_kr_matvec: out_i = x_i * sum_j A_ij x_j p_j  (+ v_i p_i)    -- r_utils.R:24, :42, :64
//   hicgat_kr_scale:  out_ij = round6((x_i A_ij) x_j), NaN where A_ij is NaN  -- :74, :76-80, :89
//
// A is float64 row-major (the symmetric contact matrix after the zero-column removal of :3-7);
// NaN entries of A count as 0 in the products (:13-15).  HBM-bound: one pass over 8 N^2 bytes per
// call; one wave per row, lane l reads the double2 pair 2l, 2l+1 of every 128-column chunk, the
// 64 partial sums are reduced in a fixed shuffle tree (deterministic run to run).
#include "common.hpp"

namespace hicgat {

__device__ __forceinline__ double nz(double a) { return a == a ? a : 0.0; }

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <bool VEC>
__global__ __launch_bounds__(256) void kr_matvec_kernel(const double *__restrict__ A, int64_t lda, int n,
                                                        const double *__restrict__ x,
                                                        const double *__restrict__ p,
                                                        const double *__restrict__ v,
                                                        double *__restrict__ out) {
  const int lane = lane_id();
  const int i = blockIdx.x * 4 + wave_in_block();
  if (i >= n) return;
  const double *a = A + (size_t)i * lda;
  double s0 = 0.0, s1 = 0.0;
  if (VEC) {   // lda even and A 16-B aligned: double2 loads
    const double2 *a2 = reinterpret_cast<const double2 *>(a);
    const int n2 = n / 2;
    for (int q = lane; q < n2; q += 64) {
      const double2 av = a2[q];
      const int j = 2 * q;
      s0 = fma(nz(av.x), x[j] * p[j], s0);
      s1 = fma(nz(av.y), x[j + 1] * p[j + 1], s1);
    }
    if ((n & 1) && lane == 0) s0 = fma(nz(a[n - 1]), x[n - 1] * p[n - 1], s0);
  } else {
    for (int j = lane; j < n; j += 64) s0 = fma(nz(a[j]), x[j] * p[j], s0);
  }
  const double s = wave_sum_d(s0 + s1);
  if (lane == 0) out[i] = x[i] * s + (v ? v[i] * p[i] : 0.0);
}

__global__ __launch_bounds__(256) void kr_scale_kernel(const double *__restrict__ A, int64_t lda, int n,
                                                       const double *__restrict__ x, double *__restrict__ out,
                                                       int64_t ldo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)n * n) return;
  const int i = (int)(idx / n), j = (int)(idx % n);
  const double a = A[(size_t)i * lda + j];
  double r;
  if (a != a) {
    r = a;                                       // NA reintroduced (:76-80)
  } else {
    r = (x[i] * a) * x[j];                       // t(t(x * A) * x)
    r = __builtin_rint(r * 1e6) / 1e6;           // round(result, digits = 6), as write.table saves it
  }
  out[(size_t)i * ldo + j] = r;
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_kr_matvec(const double *A, int64_t lda, int n, const double *x, const double *p,
                                const double *v, double *out, hicgat_stream_t stream) {
  if (n < 0 || lda < n) return HICGAT_EINVAL;
  if (n == 0) return HICGAT_OK;
  if (!A || !x || !p || !out) return HICGAT_EINVAL;
  const bool vec = (lda % 2 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
  if (vec)
    hipLaunchKernelGGL(kr_matvec_kernel<true>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, A, lda, n,
                       x, p, v, out);
  else
    hipLaunchKernelGGL(kr_matvec_kernel<false>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, A, lda,
                       n, x, p, v, out);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_kr_scale(const double *A, int64_t lda, int n, const double *x, double *out, int64_t ldo,
                               hicgat_stream_t stream) {
  if (n < 0 || lda < n || ldo < n) return HICGAT_EINVAL;
  if (n == 0) return HICGAT_OK;
  if (!A || !x || !out) return HICGAT_EINVAL;
  const int64_t total = (int64_t)n * n;
  hipLaunchKernelGGL(kr_scale_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A,
                     lda, n, x, out, ldo);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
