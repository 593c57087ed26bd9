// Deterministic column sums: out[n] = sum_{k < K} A[k, n], the reduction behind the bias
// gradients of every Linear (a6 / a10), the LayerNorm gamma/beta gradients and the split-K slab
// sums of the weight-gradient GEMMs.  No float atomics: the sum runs in one fixed order, so a
// training step is bitwise reproducible.
//
// Two shapes:
//  * wide (K small, N large: split-K slabs, K = splits): one thread per column, rows summed in
//    order with 8 loads in flight per thread;
//  * tall (K large, N small: 20000 node rows x <= 512 features): each 256-thread block sums a
//    64-row x 64-column chunk (4 row groups x 16 rows, all 16 loads of a thread issued before the
//    adds, groups combined in order through LDS) into a partial row; the partial rows are reduced
//    again the same way until one row is left (20000 -> 313 -> 5 -> 1).
// The last pass writes the final row through `ColOut`: element i goes to row i / cols, column
// i % cols of out0 (leading dim ld), or to out1 for row 1 when out1 is set (LayerNorm: dgamma and
// dbeta), plus bias[col], plus the old value when accumulating.
#include "reduce.hpp"

namespace hicgat {

__device__ __forceinline__ void colout_write(const ColOut &o, int64_t i, float s) {
  if (o.tail && i >= o.tail_start) {
    float *dst = o.tail + (i - o.tail_start);
    *dst = s + (o.accumulate ? *dst : 0.f);
    return;
  }
  const int64_t row = i / o.cols, col = i % o.cols;
  float *dst = (row == 1 && o.out1) ? o.out1 + col : o.out0 + row * o.ld + col;
  if (o.bias) s += o.bias[col];
  *dst = s + (o.accumulate ? *dst : 0.f);
}

__global__ __launch_bounds__(256) void colsum_wide_kernel(const float *__restrict__ A, int64_t lda, int K, int64_t N,
                                                          ColOut o) {
  for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < N; n += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= K; k += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = A[(size_t)(k + u) * lda + n];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < K; ++k) s += A[(size_t)k * lda + n];
    colout_write(o, n, s);
  }
}

// The slab sum of a split-K weight gradient (K = splits <= ~80 slabs of up to 1 MB, N = M*N + M):
// 4 consecutive columns per thread and the K slabs cut into 4 contiguous groups, one per wave of
// the block, each with all its loads issued before its in-order adds; the 4 group sums are combined
// in order through LDS.  One pass, fixed order (bitwise reproducible), ~4x the loads in flight of
// the one-column form above.  VEC: float4 loads (N % 4 == 0, lda % 4 == 0, A 16-B aligned); else
// four guarded scalar loads per row.
constexpr int kWideGroups = 4;
template <bool VEC>
__global__ __launch_bounds__(256) void colsum_wide4_kernel(const float *__restrict__ A, int64_t lda, int K,
                                                           int64_t N, ColOut o) {
  __shared__ float4 red[kWideGroups][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t n0 = 4 * ((int64_t)blockIdx.x * 64 + cl);   // first column of this thread
  const int per = (K + kWideGroups - 1) / kWideGroups;
  const int kb = g * per, ke = min(K, kb + per);
  auto ld = [&](int k) -> float4 {
    const float *a = A + (size_t)k * lda + n0;
    if (VEC) return *reinterpret_cast<const float4 *>(a);
    return make_float4(a[0], n0 + 1 < N ? a[1] : 0.f, n0 + 2 < N ? a[2] : 0.f, n0 + 3 < N ? a[3] : 0.f);
  };
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n0 < N) {
    int k = kb;
    for (; k + 8 <= ke; k += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld(k + u);
#pragma unroll
      for (int u = 0; u < 8; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; k < ke; ++k) {
      const float4 v = ld(k);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && n0 < N) {
    float4 t = red[0][cl];
#pragma unroll
    for (int h = 1; h < kWideGroups; ++h) {
      const float4 u = red[h][cl];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    colout_write(o, n0, t.x);
    if (n0 + 1 < N) colout_write(o, n0 + 1, t.y);
    if (n0 + 2 < N) colout_write(o, n0 + 2, t.z);
    if (n0 + 3 < N) colout_write(o, n0 + 3, t.w);
  }
}

constexpr int kRows = 16;               // rows per thread per pass
constexpr int kChunk = 4 * kRows;       // rows per block per pass

__global__ __launch_bounds__(256) void colsum_tall_kernel(const float *__restrict__ A, int64_t lda, int K, int N,
                                                          float *__restrict__ part, ColOut o) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + cl;
  const int k0 = blockIdx.y * kChunk + g * kRows;
  float v[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) v[r] = (n < N && k0 + r < K) ? A[(size_t)(k0 + r) * lda + n] : 0.f;
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < kRows; ++r) s += v[r];
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && n < N) {
    const float t = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
    if (gridDim.y == 1) colout_write(o, n, t);
    else part[(size_t)blockIdx.y * N + n] = t;
  }
}

size_t colsum_workspace_bytes(int64_t K, int64_t N) {
  if (K <= 64 || N > 65536) return 0;
  size_t total = 0;
  for (int64_t k = K; k > kChunk;) {
    k = (k + kChunk - 1) / kChunk;
    total += (size_t)k * N;
  }
  return total * sizeof(float);
}

int colsum_wide_launch(const float *A, int64_t lda, int64_t K, int64_t N, const ColOut &o, hipStream_t s) {
  if (N == 0) return HICGAT_OK;
  if (K >= 2 * kWideGroups) {
    const dim3 grid((unsigned)(((N + 3) / 4 + 63) / 64));
    if (N % 4 == 0 && lda % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0)
      hipLaunchKernelGGL(colsum_wide4_kernel<true>, grid, dim3(256), 0, s, A, lda, (int)K, N, o);
    else
      hipLaunchKernelGGL(colsum_wide4_kernel<false>, grid, dim3(256), 0, s, A, lda, (int)K, N, o);
    HICGAT_CHECK_LAUNCH();
    return HICGAT_OK;
  }
  const int64_t blocks = std::min<int64_t>((N + 255) / 256, 4096);
  hipLaunchKernelGGL(colsum_wide_kernel, dim3((unsigned)blocks), dim3(256), 0, s, A, lda, (int)K, N, o);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

int colsum_launch(const float *A, int64_t lda, int64_t K, int64_t N, const ColOut &o, float *ws, hipStream_t s) {
  if (N == 0) return HICGAT_OK;
  if (K <= 64 || N > 65536) return colsum_wide_launch(A, lda, K, N, o, s);
  const float *src = A;
  int64_t ld = lda, k = K;
  float *dst = ws;
  while (true) {
    const int64_t chunks = (k + kChunk - 1) / kChunk;
    hipLaunchKernelGGL(colsum_tall_kernel, dim3((unsigned)((N + 63) / 64), (unsigned)chunks), dim3(256), 0, s, src,
                       ld, (int)k, (int)N, dst, o);
    HICGAT_CHECK_LAUNCH();
    if (chunks == 1) break;
    src = dst;
    ld = N;
    k = chunks;
    dst += (size_t)chunks * N;
  }
  return HICGAT_OK;
}

}  // namespace hicgat
