// fp32 MFMA GEMM family for the MLP tail (a6 / a6') and the GAT weight gradient (a10).
//
// Reference: torch.nn.Linear forward/backward inside models.py:637-659 and the lin_l weight
// gradient of PyG GATConv, run by ATen/MKL sgemm on the CPU.  On MI355X these shapes are skinny
// (M = N_nodes = 20000 rows against 3..512 features, and the weight gradients reduce over K = 20000
// rows); a library GEMM picks tiles for square problems, so the tail gets its own kernels:
//
//   C[M,N] = op(A)[M,K] * op(B)[K,N] (+ bias[N]),  op(A) = A (row-major [M,K]) or A^T (A is [K,M]),
//                                                 op(B) = B^T (B is [N,K]) or B (B is [K,N])
//   Linear forward   Y  = X W^T + b : A = X [M,K],  B = W [N,K]           (A_KM = 0, B_KM = 0)
//   input gradient   dX = dY W      : A = dY [M,K], B = W [K,N]           (A_KM = 0, B_KM = 1)
//   weight gradient  dW = dY^T X    : A = dY [K,M], B = X [K,N], K = rows  (A_KM = 1, B_KM = 1)
//
// v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulate), 4 waves in 2x2, LDS tiles stored
// K-major (As[k][m], Bs[k][n]) so every MFMA operand read is 32 consecutive floats; the next
// K-step is prefetched into registers under the current step's MFMAs.  K can be split over
// gridDim.z: each split writes an fp32 partial slab and a second kernel adds the slabs in split
// order (deterministic, no float atomics; reduce.hip).
#include "reduce.hpp"

namespace hicgat {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GK = 16;  // K-step

template <int BM, int BN, bool A_KM, bool B_KM, bool VEC>
__global__ __launch_bounds__(256) void gemm_kernel(const float *__restrict__ A, int64_t lda,
                                                   const float *__restrict__ B, int64_t ldb,
                                                   float *__restrict__ C, int64_t ldc, int M, int N,
                                                   int K, int kchunk, const float *__restrict__ bias,
                                                   float *__restrict__ slab, int accumulate) {
  constexpr int WM = BM / 2, WN = BN / 2;        // wave tile (4 waves in 2 x 2)
  constexpr int TM = WM / 32, TN = WN / 32;      // 32x32 MFMA tiles per wave
  // staged values per thread: VEC -> float4 pieces, else scalars
  constexpr int AE = VEC ? BM * GK / 1024 : BM * GK / 256;
  constexpr int BE = VEC ? BN * GK / 1024 : BN * GK / 256;
  constexpr int W = VEC ? 4 : 1;
  __shared__ __attribute__((aligned(16))) float As[GK][BM + 4];
  __shared__ __attribute__((aligned(16))) float Bs[GK][BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);

  float ra[AE][W], rb[BE][W];
  // piece p of a tile: K-major operands walk the contiguous m (n) dim first, the others the
  // contiguous k dim first, so consecutive threads read consecutive 4 (or 16) bytes either way.
  auto load = [&](int k0) {
#pragma unroll
    for (int e = 0; e < AE; ++e) {
      const int idx = e * 256 + tid;
      int m, k;
      if (A_KM) { m = (idx % (BM / W)) * W; k = idx / (BM / W); } else { k = (idx % (GK / W)) * W; m = idx / (GK / W); }
      const int gm = m0 + m, gk = k0 + k;
      if (VEC) {
        const bool ok = A_KM ? (gm < M && gk < ke) : (gm < M && gk < ke);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) v = *reinterpret_cast<const float4 *>(A_KM ? A + (size_t)gk * lda + gm : A + (size_t)gm * lda + gk);
        ra[e][0] = v.x; ra[e][W > 1 ? 1 : 0] = v.y; ra[e][W > 2 ? 2 : 0] = v.z; ra[e][W > 3 ? 3 : 0] = v.w;
      } else {
        ra[e][0] = (gm < M && gk < ke) ? (A_KM ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk]) : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < BE; ++e) {
      const int idx = e * 256 + tid;
      int n, k;
      if (B_KM) { n = (idx % (BN / W)) * W; k = idx / (BN / W); } else { k = (idx % (GK / W)) * W; n = idx / (GK / W); }
      const int gn = n0 + n, gk = k0 + k;
      if (VEC) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gn < N && gk < ke)
          v = *reinterpret_cast<const float4 *>(B_KM ? B + (size_t)gk * ldb + gn : B + (size_t)gn * ldb + gk);
        rb[e][0] = v.x; rb[e][W > 1 ? 1 : 0] = v.y; rb[e][W > 2 ? 2 : 0] = v.z; rb[e][W > 3 ? 3 : 0] = v.w;
      } else {
        rb[e][0] = (gn < N && gk < ke) ? (B_KM ? B[(size_t)gk * ldb + gn] : B[(size_t)gn * ldb + gk]) : 0.f;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < AE; ++e) {
      const int idx = e * 256 + tid;
      if (A_KM) {
        const int m = (idx % (BM / W)) * W, k = idx / (BM / W);
        if (VEC) *reinterpret_cast<float4 *>(&As[k][m]) = make_float4(ra[e][0], ra[e][W > 1 ? 1 : 0], ra[e][W > 2 ? 2 : 0], ra[e][W > 3 ? 3 : 0]);
        else As[k][m] = ra[e][0];
      } else {
        const int k = (idx % (GK / W)) * W, m = idx / (GK / W);
#pragma unroll
        for (int c = 0; c < W; ++c) As[k + c][m] = ra[e][c];
      }
    }
#pragma unroll
    for (int e = 0; e < BE; ++e) {
      const int idx = e * 256 + tid;
      if (B_KM) {
        const int n = (idx % (BN / W)) * W, k = idx / (BN / W);
        if (VEC) *reinterpret_cast<float4 *>(&Bs[k][n]) = make_float4(rb[e][0], rb[e][W > 1 ? 1 : 0], rb[e][W > 2 ? 2 : 0], rb[e][W > 3 ? 3 : 0]);
        else Bs[k][n] = rb[e][0];
      } else {
        const int k = (idx % (GK / W)) * W, n = idx / (GK / W);
#pragma unroll
        for (int c = 0; c < W; ++c) Bs[k + c][n] = rb[e][c];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int li = lane & 31, lk = lane >> 5;
  if (kb < ke) load(kb);
  for (int k0 = kb; k0 < ke; k0 += GK) {
    __syncthreads();
    store();
    __syncthreads();
    if (k0 + GK < ke) load(k0 + GK);
#pragma unroll
    for (int kk = 0; kk < GK; kk += 2) {
      float av[TM], bv[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) av[a] = As[kk + lk][wm * WM + a * 32 + li];
#pragma unroll
      for (int b = 0; b < TN; ++b) bv[b] = Bs[kk + lk][wn * WN + b * 32 + li];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }

  // C/D map of a 32x32 f32 tile: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float *out = slab ? slab + (size_t)blockIdx.z * M * N : C;
  const int64_t ldo = slab ? N : ldc;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int gn = n0 + wn * WN + b * 32 + li;
      const float bb = (bias && !slab && gn < N) ? bias[gn] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * WM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (gm < M && gn < N) {
          float *o = out + (size_t)gm * ldo + gn;
          *o = acc[a][b][r] + bb + ((accumulate && !slab) ? *o : 0.f);
        }
      }
    }
  }
}

__global__ void colsum_zero_kernel(float *out, int N, int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n < N && !accumulate) out[n] = 0.f;
}

template <int BM, int BN, bool AK, bool BK_>
static int launch(const float *A, int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc, int M, int N,
                  int K, int splits, const float *bias, float *slab, int acc, hipStream_t s) {
  const int kchunk = ((K + splits - 1) / splits + GK - 1) / GK * GK;
  const dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
  // float4 staging needs every float4 inside its operand row and 16-B aligned rows
  const bool a_ok = AK ? (M % 4 == 0 && lda % 4 == 0) : (K % 4 == 0 && lda % 4 == 0);
  const bool b_ok = BK_ ? (N % 4 == 0 && ldb % 4 == 0) : (K % 4 == 0 && ldb % 4 == 0);
  const bool al = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0;
  if (a_ok && b_ok && al)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BK_, true>), grid, dim3(256), 0, s, A, lda, B, ldb, C, ldc, M, N,
                       K, kchunk, bias, splits > 1 ? slab : nullptr, acc);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BK_, false>), grid, dim3(256), 0, s, A, lda, B, ldb, C, ldc, M,
                       N, K, kchunk, bias, splits > 1 ? slab : nullptr, acc);
  HICGAT_CHECK_LAUNCH();
  if (splits > 1) {
    // C[m][n] = sum_z slab[z][m][n] (+ bias[n]) (+ C), splits added in order
    const ColOut o{C, ldc, N, nullptr, bias, acc};
    return colsum_wide_launch(slab, (int64_t)M * N, splits, (int64_t)M * N, o, s);
  }
  return HICGAT_OK;
}

template <bool AK, bool BK_>
static int dispatch(const float *A, int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc, int M, int N,
                    int K, int splits, const float *bias, float *slab, int acc, hipStream_t s) {
  // tall row-major problems (M = node rows): 64 x 128 tiles keep >= 2 blocks per CU in flight;
  // square-ish weight gradients (M, N = features, K = rows split): 128 x 128
  if (M >= 128 && N >= 128 && M <= 1024)
    return launch<128, 128, AK, BK_>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, acc, s);
  if (N >= 128) return launch<64, 128, AK, BK_>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, acc, s);
  return launch<64, 64, AK, BK_>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, acc, s);
}

}  // namespace hicgat

using namespace hicgat;

extern "C" size_t hicgat_gemm_workspace_bytes(int M, int N, int splits) {
  return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

extern "C" int hicgat_gemm(int a_kmajor, int b_kmajor, int M, int N, int K, const float *A, int64_t lda,
                           const float *B, int64_t ldb, const float *bias, float *C, int64_t ldc, int accumulate,
                           int splits, void *workspace, size_t workspace_bytes, hicgat_stream_t stream) {
  if (M < 0 || N < 0 || K < 0 || splits < 1) return HICGAT_EINVAL;
  if (M == 0 || N == 0) return HICGAT_OK;
  if (!A || !B || !C) return HICGAT_EINVAL;
  if (splits > 1 && (!workspace || workspace_bytes < hicgat_gemm_workspace_bytes(M, N, splits)))
    return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float *slab = static_cast<float *>(workspace);
  if (!a_kmajor && !b_kmajor) return dispatch<false, false>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, s);
  if (!a_kmajor && b_kmajor) return dispatch<false, true>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, s);
  if (a_kmajor && !b_kmajor) return dispatch<true, false>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, s);
  return dispatch<true, true>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, s);
}

extern "C" size_t hicgat_colsum_workspace_bytes(int K, int N) { return colsum_workspace_bytes(K, N); }

extern "C" int hicgat_colsum(const float *A, int64_t lda, int K, int N, float *out, int accumulate, void *workspace,
                             size_t workspace_bytes, hicgat_stream_t stream) {
  if (K < 0 || N < 0) return HICGAT_EINVAL;
  if (N == 0) return HICGAT_OK;
  if (!out || (K > 0 && !A)) return HICGAT_EINVAL;
  const size_t need = colsum_workspace_bytes(K, N);
  if (need > 0 && (!workspace || workspace_bytes < need)) return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const ColOut o{out, 0, N, nullptr, nullptr, accumulate};
  if (K == 0) {  // empty sum
    hipLaunchKernelGGL(colsum_zero_kernel, dim3((N + 255) / 256), dim3(256), 0, s, out, N, accumulate);
    HICGAT_CHECK_LAUNCH();
    return HICGAT_OK;
  }
  return colsum_launch(A, lda, K, N, o, static_cast<float *>(workspace), s);
}
