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
#include <algorithm>
#include <cstdlib>

#include "reduce.hpp"

namespace hicgat {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GK = 16;  // K-step of the fp32 kernel

// min blocks per CU of the 64 x 128 fp32 kernel: 6 makes the compiler keep the accumulators in
// VGPRs (74 in all, 6 waves per SIMD instead of 4): fwd 512x512 0.104 vs 0.115 ms, dX 0.057 vs
// 0.060 (profiles/r01_kbench_gemm_tiles.txt).  The 128 x 128 kernel keeps 1: squeezed the same
// way its split-K weight gradients ran 2x slower.
constexpr int kOcc64 = 6, kOcc128 = 1;

// CS (weight gradients, A_KM only): the workgroups of the first column tile also sum their A tile
// over K, i.e. the bias gradient db[m] = sum_k dY[k][m] of the same Linear comes out of the dW
// GEMM (its per-split partials go into the slab beside the dW partials, one slab sum for both).
template <int BM, int BN, bool A_KM, bool B_KM, bool VEC, bool DB, bool CS = false>
// One BM x BN output tile (block coordinates bx, by, split bz) of the kernel below; also the body of
// the grouped weight-gradient kernel (several GEMMs in one launch).
__device__ __forceinline__ void gemm_tile(const float *__restrict__ A, int64_t lda,
                                          const float *__restrict__ B, int64_t ldb,
                                          float *__restrict__ C, int64_t ldc, int M, int N,
                                          int K, int kchunk, const float *__restrict__ bias,
                                          float *__restrict__ slab, int64_t slab_stride, int accumulate,
                                          float *__restrict__ csum, int bx, int by, int bz,
                                          float *__restrict__ crelu = nullptr, int64_t ldr = 0) {
  static_assert(!CS || A_KM, "column sums of A need the K-major (weight-gradient) layout");
  constexpr int WM = BM / 2, WN = BN / 2;        // wave tile (4 waves in 2 x 2)
  constexpr int TM = WM / 32, TN = WN / 32;      // 32x32 MFMA tiles per wave
  // staged values per thread: VEC -> float4 pieces, else scalars
  constexpr int AE = VEC ? BM * GK / 1024 : BM * GK / 256;
  constexpr int BE = VEC ? BN * GK / 1024 : BN * GK / 256;
  constexpr int W = VEC ? 4 : 1;
  // DB: double-buffered LDS, one barrier per K-step instead of two (it doubles the LDS footprint;
  // measured faster only for the input-gradient layout, profiles/r01_kbench_x3_sliced.txt)
  constexpr int NB = DB ? 2 : 1;
  __shared__ __attribute__((aligned(16))) float As[NB][GK][BM + 4];
  __shared__ __attribute__((aligned(16))) float Bs[NB][GK][BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = bx * BM, n0 = by * BN;
  const int kb = bz * kchunk, ke = min(K, kb + kchunk);

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
  auto store = [&](int sb) {
#pragma unroll
    for (int e = 0; e < AE; ++e) {
      const int idx = e * 256 + tid;
      if (A_KM) {
        const int m = (idx % (BM / W)) * W, k = idx / (BM / W);
        if (VEC) *reinterpret_cast<float4 *>(&As[sb][k][m]) = make_float4(ra[e][0], ra[e][W > 1 ? 1 : 0], ra[e][W > 2 ? 2 : 0], ra[e][W > 3 ? 3 : 0]);
        else As[sb][k][m] = ra[e][0];
      } else {
        const int k = (idx % (GK / W)) * W, m = idx / (GK / W);
#pragma unroll
        for (int c = 0; c < W; ++c) As[sb][k + c][m] = ra[e][c];
      }
    }
#pragma unroll
    for (int e = 0; e < BE; ++e) {
      const int idx = e * 256 + tid;
      if (B_KM) {
        const int n = (idx % (BN / W)) * W, k = idx / (BN / W);
        if (VEC) *reinterpret_cast<float4 *>(&Bs[sb][k][n]) = make_float4(rb[e][0], rb[e][W > 1 ? 1 : 0], rb[e][W > 2 ? 2 : 0], rb[e][W > 3 ? 3 : 0]);
        else Bs[sb][k][n] = rb[e][0];
      } else {
        const int k = (idx % (GK / W)) * W, n = idx / (GK / W);
#pragma unroll
        for (int c = 0; c < W; ++c) Bs[sb][k + c][n] = rb[e][c];
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
  auto mma = [&](int cb) {
#pragma unroll
    for (int kk = 0; kk < GK; kk += 2) {
      float av[TM], bv[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) av[a] = As[cb][kk + lk][wm * WM + a * 32 + li];
#pragma unroll
      for (int b = 0; b < TN; ++b) bv[b] = Bs[cb][kk + lk][wn * WN + b * 32 + li];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  };
  // CS: thread t < BM adds column t of every staged A tile, k in order (deterministic)
  const bool cs_on = CS && csum != nullptr && by == 0 && tid < BM;
  float cs = 0.f;
  auto colacc = [&](int cb) {
    if (cs_on) {
#pragma unroll
      for (int kk = 0; kk < GK; ++kk) cs += As[cb][kk][tid];
    }
  };
  if (kb < ke) load(kb);
  if (DB) {
    // stage k0 + GK into the other buffer while k0's MFMAs run; one barrier per K-step
    if (kb < ke) store(0);
    __syncthreads();
    int cur = 0;
    for (int k0 = kb; k0 < ke; k0 += GK) {
      const bool more = k0 + GK < ke;
      if (more) load(k0 + GK);
      mma(cur);
      colacc(cur);
      if (more) store(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  } else {
    for (int k0 = kb; k0 < ke; k0 += GK) {
      __syncthreads();
      store(0);
      __syncthreads();
      if (k0 + GK < ke) load(k0 + GK);
      mma(0);
      colacc(0);
    }
  }
  if (cs_on && m0 + tid < M) {
    if (slab) {
      csum[(size_t)bz * slab_stride + tid + m0] = cs;      // csum = this launch's slab + M*N
    } else {
      float *o = csum + m0 + tid;
      *o = cs + (accumulate ? *o : 0.f);
    }
  }

  // C/D map of a 32x32 f32 tile: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float *out = slab ? slab + (size_t)bz * slab_stride : C;
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
          const float v = acc[a][b][r] + bb + ((accumulate && !slab) ? *o : 0.f);
          *o = v;
          if (crelu && !slab) crelu[(size_t)gm * ldr + gn] = fmaxf(v, 0.f);   // relu(C) beside C (no split)
        }
      }
    }
  }
}

template <int BM, int BN, bool A_KM, bool B_KM, bool VEC, bool DB, bool CS = false>
__global__ __launch_bounds__(256, (BM == 64 && BN == 128 && VEC) ? kOcc64
                                  : (BM == 128 && BN == 128 && VEC) ? kOcc128 : 1) void gemm_kernel(const float *__restrict__ A, int64_t lda,
                                                   const float *__restrict__ B, int64_t ldb,
                                                   float *__restrict__ C, int64_t ldc, int M, int N,
                                                   int K, int kchunk, const float *__restrict__ bias,
                                                   float *__restrict__ slab, int64_t slab_stride, int accumulate,
                                                   float *__restrict__ csum) {
  gemm_tile<BM, BN, A_KM, B_KM, VEC, DB, CS>(A, lda, B, ldb, C, ldc, M, N, K, kchunk, bias, slab, slab_stride, accumulate,
                                             csum, blockIdx.x, blockIdx.y, blockIdx.z);
}

__global__ void colsum_zero_kernel(float *out, int N, int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n < N && !accumulate) out[n] = 0.f;
}

// csum (weight gradients only): also db[m] (+)= sum_k A[k][m] (the CS kernels); the slab of split z
// is then [M*N dW partials | M db partials].
template <int BM, int BN, bool AK, bool BK_>
static int launch(const float *A, int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc, int M, int N,
                  int K, int splits, const float *bias, float *slab, int acc, hipStream_t s, float *csum = nullptr) {
  const int kchunk = ((K + splits - 1) / splits + GK - 1) / GK * GK;
  const dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
  // float4 staging needs every float4 inside its operand row and 16-B aligned rows
  const bool a_ok = AK ? (M % 4 == 0 && lda % 4 == 0) : (K % 4 == 0 && lda % 4 == 0);
  const bool b_ok = BK_ ? (N % 4 == 0 && ldb % 4 == 0) : (K % 4 == 0 && ldb % 4 == 0);
  const bool al = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0;
  const bool cs = AK && csum != nullptr;
  const int64_t stride = (int64_t)M * N + (cs ? M : 0);
  float *sl = splits > 1 ? slab : nullptr;
  float *cdst = cs ? (sl ? slab + (int64_t)M * N : csum) : nullptr;
#define HICGAT_GEMM_GO(V, D, C_)                                                                            \
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AK, BK_, V, D, C_>), grid, dim3(256), 0, s, A, lda, B, ldb, C, ldc, M, N, \
                     K, kchunk, bias, sl, stride, acc, cdst)
  if (a_ok && b_ok && al) {
    constexpr bool db = !AK && BK_;   // double-buffered LDS: the dX layout (every layout measured: no gain)
    if (cs) HICGAT_GEMM_GO(true, db, AK);
    else HICGAT_GEMM_GO(true, db, false);
  } else {
    if (cs) HICGAT_GEMM_GO(false, false, AK);
    else HICGAT_GEMM_GO(false, false, false);
  }
#undef HICGAT_GEMM_GO
  HICGAT_CHECK_LAUNCH();
  if (splits > 1) {
    // C[m][n] = sum_z slab[z][m][n] (+ bias[n]) (+ C), splits added in order; db likewise
    const ColOut o{C, ldc, N, nullptr, bias, acc, cs ? csum : nullptr, (int64_t)M * N};
    return colsum_wide_launch(slab, stride, splits, stride, o, s);
  }
  return HICGAT_OK;
}

int gemm_tall_launch(bool b_kmajor, const float *A, int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc,
                     int M, int N, int K, const float *bias, int accumulate, hipStream_t s);   // gemm_tall.hip

// Problems with fewer 160x128 tiles than this go to the 64x128 kernel (2.5x the workgroups): one
// workgroup per tile with the whole K inside, the tall kernel needs ~one tile per CU -- a rank's
// 2700-row shard of a multi-GPU step is 68 tiles, a quarter of the chip (57 vs 98 us for 7x fewer
// FLOP than the 20000-row GEMM).  The single-GPU shapes (>= 250 tiles) keep the tall kernel.
static int64_t tall_min_tiles() { return 192; }

template <bool AK, bool BK_>
static int dispatch(const float *A, int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc, int M, int N,
                    int K, int splits, const float *bias, float *slab, int acc, int impl, hipStream_t s) {
  // tall node-row problems (Linear forward, input gradient): the 160x128 LDS-DMA kernel (gemm_tall.hip)
  if (!AK && splits == 1 && M >= 1024 &&
      (int64_t)((M + 159) / 160) * (N / 128) >= tall_min_tiles()) {
    const int rc = gemm_tall_launch(BK_, A, lda, B, ldb, C, ldc, M, N, K, bias, acc, s);
    if (rc != HICGAT_EUNSUPPORTED) return rc;
  }
  // tall row-major problems (M = node rows): 64 x 128 tiles keep >= 2 blocks per CU in flight;
  // square-ish weight gradients (M, N = features, K = rows split): 128 x 128
  // (128 x 128, 128 x 256 and 256 x 128 tiles for the tall problems measured slower, round 1)
  if (M >= 128 && N >= 128 && M <= 1024)
    return launch<128, 128, AK, BK_>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, acc, s);
  if (N >= 128) return launch<64, 128, AK, BK_>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, acc, s);
  return launch<64, 64, AK, BK_>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, acc, s);
}

// ---- grouped parameter gradients (hicgat_param_grads_grouped) -------------------------------------
// Launch 1: the 128 x 128 weight-gradient tiles of every job (K-major dY and X, db from the staged dY
// of the first column tile: gemm_tile's CS path) -- workgroup b finds its job by the prefix of
// workgroup counts, then (tile row, tile column, K chunk).  One K-chunk depth for all jobs, so every
// workgroup has the same MFMA work.  A job whose operands cannot be read as float4 (dense3: M = 3)
// takes the scalar-staged path of the same tile in the same launch.
constexpr int kMaxWJobs = 16, kMaxCJobs = 32, kGroupTile = 128;
constexpr int64_t WEIGHTED_LG1_ROWS = 1024;   // weighted column-sum jobs taller than this: 2 lanes per row group
// jobs of at most this many rows (the split-K slabs: 6-16 splits) take one lane per 4 columns with
// every row in that lane (lg = 8: 1024 columns per block, no LDS combine) instead of 4 row groups of
// 64 lanes (256 columns per block): a quarter of the blocks for the same bytes
#ifndef HICGAT_COLSUM_SHORT
#define HICGAT_COLSUM_SHORT 16
#endif
constexpr int64_t kColsumShortRows = HICGAT_COLSUM_SHORT;
constexpr int kWeightedLg = 1;   // log2 lanes per row group of those jobs (2: 0.425-0.427 ms, 1: 0.422-0.423 at P = 8)
// The job a block belongs to: the number of later job starts <= b, every start read at a constant
// offset of the kernel argument block (one batch of scalar loads instead of one dependent load per
// job scanned; measured even at P = 8, profiles/r04p_sim_ab.txt)
template <int KMAX>
__device__ __forceinline__ int find_job(const int (&start)[KMAX], int n, int b) {
  int q = 0;
#pragma unroll
  for (int k = 1; k < KMAX; ++k) q += (k < n && b >= start[k]) ? 1 : 0;
  return q;
}
struct WJob {
  const float *dy;
  const float *x;
  float *dw;
  float *db;
  float *slab;        // [splits][M*N + M] partials, or null (splits == 1: straight into dw / db)
  int64_t ldy, ldx, lddw;
  int M, N, K, kchunk, tm, tn, wg0, accumulate, vec;
};
struct WJobs {
  int start[kMaxWJobs];   // job k's first workgroup (= j[k].wg0), contiguous for find_job
  WJob j[kMaxWJobs];
  int n;
};
__global__ __launch_bounds__(256, kOcc128) void wgrad_grouped_kernel(const WJobs jobs) {
  const int q = find_job(jobs.start, jobs.n, (int)blockIdx.x);
  const WJob &J = jobs.j[q];
  const int local = blockIdx.x - J.wg0, per = J.tm * J.tn;
  const int bz = local / per, rem = local - bz * per, bx = rem % J.tm, by = rem / J.tm;
  const int64_t stride = (int64_t)J.M * J.N + J.M;
  float *cs = J.db ? (J.slab ? J.slab + (int64_t)J.M * J.N : J.db) : nullptr;
  if (J.vec)
    gemm_tile<kGroupTile, kGroupTile, true, true, true, false, true>(J.dy, J.ldy, J.x, J.ldx, J.dw, J.lddw, J.M, J.N,
                                                                     J.K, J.kchunk, nullptr, J.slab, stride,
                                                                     J.accumulate, cs, bx, by, bz);
  else
    gemm_tile<kGroupTile, kGroupTile, true, true, false, false, true>(J.dy, J.ldy, J.x, J.ldx, J.dw, J.lddw, J.M, J.N,
                                                                      J.K, J.kchunk, nullptr, J.slab, stride,
                                                                      J.accumulate, cs, bx, by, bz);
}

// Launch 2: column sums dst[c] (+)= sum_{r < rows} src[r * ld + c] of every job -- the slab sums of
// the split weight gradients first, then the caller's jobs.  A block takes 64 columns (VEC: 64 float4
// = 256 columns) of one job; its 4 waves sum 4 contiguous row ranges in row order (8 loads in flight
// per lane), combined in wave order through LDS: one fixed order, bitwise reproducible.
struct CJob {
  const float *src;
  float *dst;
  const float *wt;    // optional row weights (stride ldw)
  int64_t ld, rows, cols, ldw, ldd;
  int blk0, accumulate, vec, lg;   // lg: log2 of the lanes per row group (8: 1 group, 6: 4 ... 2: 64 groups)
  int segs, nchunk;   // row segments (segment s of the rows into dst + s * ldd), column chunks per segment
};
struct CJobs {
  int start[kMaxCJobs];   // job k's first block (= j[k].blk0)
  CJob j[kMaxCJobs];
  int n;
};
__device__ __forceinline__ float4 ld4(const float *p, bool vec, int64_t c, int64_t cols) {
  if (vec) return *reinterpret_cast<const float4 *>(p);
  return make_float4(p[0], c + 1 < cols ? p[1] : 0.f, c + 2 < cols ? p[2] : 0.f, c + 3 < cols ? p[3] : 0.f);
}
__global__ __launch_bounds__(256) void colsum_grouped_kernel(const CJobs jobs) {
  __shared__ float4 red[256];
  const int q = find_job(jobs.start, jobs.n, (int)blockIdx.x);
  const CJob &J = jobs.j[q];
  // a job of many rows (LayerNorm partial rows, g_src's partial rows) takes 16 or 64 row groups of
  // 16 / 4 lanes per block, a short one (split-K slabs) 4 groups of 64 lanes: the in-order chain of
  // one lane stays short either way
  const int L = 1 << J.lg, ng = 256 >> J.lg;
  const int lane = threadIdx.x & (L - 1), g = threadIdx.x >> J.lg;
  const int lb = blockIdx.x - J.blk0, seg = lb / J.nchunk;
  const int64_t c = ((int64_t)(lb - seg * J.nchunk) * L + lane) * 4;   // first of this lane's 4 columns
  const int64_t s0 = J.rows * seg / J.segs, sn = J.rows * (seg + 1) / J.segs - s0;   // the block's row segment
  const int64_t r0 = s0 + sn * g / ng, r1 = s0 + sn * (g + 1) / ng;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < J.cols) {
    const bool vec = J.vec;
    const float *p = J.src + c;
    const float *w = J.wt;
    // 8 rows per round, every load of a round issued before its adds (a short job's 3-4 rows --
    // the split-K slabs -- are one round trip, not one per row); rows added in order
    for (int64_t r = r0; r < r1; r += 8) {
      float4 v[8];
      float wv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool in = r + u < r1;
        v[u] = in ? ld4(p + (r + u) * J.ld, vec, c, J.cols) : make_float4(0.f, 0.f, 0.f, 0.f);
        wv[u] = (w && in) ? w[(r + u) * J.ldw] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (r + u >= r1) break;
        if (w) {
          s.x = fmaf(wv[u], v[u].x, s.x); s.y = fmaf(wv[u], v[u].y, s.y);
          s.z = fmaf(wv[u], v[u].z, s.z); s.w = fmaf(wv[u], v[u].w, s.w);
        } else {
          s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
        }
      }
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  // the row groups combined by a fixed pairwise tree (group g adds group g + h, h = ng/2 ... 1):
  // log2(ng) LDS rounds instead of a chain of ng - 1 dependent LDS reads (128 for the tall weighted
  // jobs); one fixed order, bitwise reproducible
  for (int h = ng >> 1; h > 0; h >>= 1) {
    if (g < h) {
      const float4 v = red[((g + h) << J.lg) + lane];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      red[threadIdx.x] = s;
    }
    __syncthreads();
  }
  if (g != 0 || c >= J.cols) return;
  float *d = J.dst + (int64_t)seg * J.ldd + c;
  const float o[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (c + e < J.cols) d[e] = o[e] + (J.accumulate ? d[e] : 0.f);
}

// The common K-chunk depth: about target_wgs workgroups over the union of the jobs' tiles, a multiple
// of the 16-deep K-step, at least 128 deep (shorter chunks spend more on the slab traffic than the
// tiles gain).  Returns per-job splits into `splits`.
static int group_kchunk(const hicgat_wgrad_job *w, int nw, int target, int *splits) {
  int64_t tk = 0;
  for (int i = 0; i < nw; ++i)
    tk += (int64_t)((w[i].M + kGroupTile - 1) / kGroupTile) * ((w[i].N + kGroupTile - 1) / kGroupTile) * w[i].K;
  int64_t kc = target > 0 ? (tk + target - 1) / target : tk;
  kc = std::max<int64_t>(128, (kc + GK - 1) / GK * GK);
  // deeper chunks until the workgroups fit the target: rounding the split count up overshoots it
  // (a P = 8 shard: 38 tiles x 7 splits = 266 one-per-CU workgroups on 256 CUs, a second round for
  // 10 of them; 6 splits: 228)
  int64_t kmax = 0;
  for (int i = 0; i < nw; ++i) kmax = std::max<int64_t>(kmax, w[i].K);
  auto wgs = [&](int64_t c) {
    int64_t t = 0;
    for (int i = 0; i < nw; ++i) {
      const int64_t tiles = (int64_t)((w[i].M + kGroupTile - 1) / kGroupTile) * ((w[i].N + kGroupTile - 1) / kGroupTile);
      t += tiles * (w[i].lddw == w[i].N ? std::max<int64_t>(1, (w[i].K + c - 1) / c) : 1);
    }
    return t;
  };
  while (target > 0 && kc < kmax && wgs(kc) > target) kc += GK;
  for (int i = 0; i < nw; ++i) {
    // a job whose dW is not one contiguous [M, N] block is not split (its slab sum writes contiguous rows)
    const bool can = w[i].lddw == w[i].N;
    splits[i] = can ? (int)std::max<int64_t>(1, (w[i].K + kc - 1) / kc) : 1;
  }
  return (int)kc;
}

// ---- grouped node-row GEMMs (hicgat_gemm_rows_grouped): C_j = A_j op(B_j) for a few jobs of one
// layout in ONE launch of 64 x 128 tiles, K split in `splits` chunks into fp32 slabs, then ONE launch
// adds the slabs in split order + bias and (optionally) writes relu of the sum to a second output --
// the two heads of the sharded step's aggregate-first GATConv (out_h = xa_h W_h^T + b_h, relu) and
// its dxa_h = dout_h W_h, which were two K-split launches + two slab sums (+ a bias/relu pass) each.
constexpr int kMaxRJobs = 8;
struct RJob {
  const float *a;
  const float *b;
  float *c;
  float *cr;          // relu(C) too (or null)
  const float *bias;
  float *slab;        // [splits][M][N]
  int64_t lda, ldb, ldc, ldr;
  int M, N, K, kchunk, tm, tn, wg0, blk0;
};
struct RJobs {
  int start[kMaxRJobs];   // job k's first GEMM workgroup (= j[k].wg0)
  int rstart[kMaxRJobs];  // job k's first reduce block (= j[k].blk0)
  RJob j[kMaxRJobs];
  int n, splits;
};
template <bool B_KM>
__global__ __launch_bounds__(256, kOcc64) void gemm_rows_grouped_kernel(const RJobs jobs) {
  const int q = find_job(jobs.start, jobs.n, (int)blockIdx.x);
  const RJob &J = jobs.j[q];
  const int local = blockIdx.x - J.wg0, per = J.tm * J.tn;
  const int bz = local / per, rem = local - bz * per, bx = rem % J.tm, by = rem / J.tm;
  // splits = 1: the tile writes C (+ bias, + relu copy) itself and no reduce launch follows
  const bool direct = jobs.splits == 1;
  gemm_tile<64, 128, false, B_KM, true, !B_KM ? false : true, false>(
      J.a, J.lda, J.b, J.ldb, J.c, J.ldc, J.M, J.N, J.K, J.kchunk, direct ? J.bias : nullptr,
      direct ? nullptr : J.slab, (int64_t)J.M * J.N, 0, nullptr, bx, by, bz, direct ? J.cr : nullptr, J.ldr);
}
__global__ __launch_bounds__(256) void rows_reduce_kernel(const RJobs jobs) {
  const int q = find_job(jobs.rstart, jobs.n, (int)blockIdx.x);
  const RJob &J = jobs.j[q];
  const int64_t e = ((int64_t)(blockIdx.x - J.blk0) * 256 + threadIdx.x) * 4;   // element (row-major M x N)
  const int64_t MN = (int64_t)J.M * J.N;
  if (e >= MN) return;
  const float4 *sl = reinterpret_cast<const float4 *>(J.slab + e);
  const int64_t st = MN / 4;
  float4 s = sl[0];
  for (int z = 1; z < jobs.splits; ++z) {
    const float4 v = sl[z * st];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const int64_t m = e / J.N, n = e % J.N;     // N % 4 == 0: the 4 elements share a row
  if (J.bias) {
    const float4 b = *reinterpret_cast<const float4 *>(J.bias + n);
    s.x += b.x; s.y += b.y; s.z += b.z; s.w += b.w;
  }
  *reinterpret_cast<float4 *>(J.c + m * J.ldc + n) = s;
  if (J.cr) *reinterpret_cast<float4 *>(J.cr + m * J.ldr + n) = f4_relu(s);
}

}  // namespace hicgat

using namespace hicgat;

extern "C" size_t hicgat_gemm_rows_grouped_workspace_bytes(const hicgat_gemm_job *jobs, int n, int splits) {
  if (n <= 0 || !jobs || splits <= 1) return 0;   // one chunk: the tiles write C directly
  size_t tot = 0;
  for (int i = 0; i < n; ++i) tot += (size_t)splits * jobs[i].M * jobs[i].N * sizeof(float);
  return tot;
}

extern "C" int hicgat_gemm_rows_grouped(const hicgat_gemm_job *jobs, int n, int b_kmajor, int splits, void *workspace,
                                        size_t workspace_bytes, hicgat_stream_t stream) {
  if (n < 0 || (n && !jobs) || splits < 1) return HICGAT_EINVAL;
  if (n > kMaxRJobs) return HICGAT_EUNSUPPORTED;
  if (n == 0) return HICGAT_OK;
  if (workspace_bytes < hicgat_gemm_rows_grouped_workspace_bytes(jobs, n, splits) || (splits > 1 && !workspace))
    return HICGAT_EINVAL;
  RJobs rj;
  rj.n = 0;
  rj.splits = splits;
  int wg = 0, blk = 0;
  float *slab = static_cast<float *>(workspace);
  for (int i = 0; i < n; ++i) {
    const hicgat_gemm_job &a = jobs[i];
    if (a.M <= 0 || a.N <= 0 || a.K <= 0 || !a.a || !a.b || !a.c) return HICGAT_EINVAL;
    // float4 staging and float4 epilogue: every row a multiple of 4 floats, 16-B aligned
    const bool ok = a.K % 4 == 0 && a.lda % 4 == 0 && a.ldb % 4 == 0 && a.N % 4 == 0 && a.ldc % 4 == 0 &&
                    (!a.c_relu || a.ldr % 4 == 0) &&
                    ((reinterpret_cast<uintptr_t>(a.a) | reinterpret_cast<uintptr_t>(a.b) | reinterpret_cast<uintptr_t>(a.c) |
                      reinterpret_cast<uintptr_t>(a.c_relu) | reinterpret_cast<uintptr_t>(a.bias)) & 15) == 0;
    if (!ok) return HICGAT_EUNSUPPORTED;
    RJob &J = rj.j[rj.n++];
    J.a = a.a;
    J.b = a.b;
    J.c = a.c;
    J.cr = a.c_relu;
    J.bias = a.bias;
    J.lda = a.lda;
    J.ldb = a.ldb;
    J.ldc = a.ldc;
    J.ldr = a.ldr;
    J.M = a.M;
    J.N = a.N;
    J.K = a.K;
    J.kchunk = ((a.K + splits - 1) / splits + GK - 1) / GK * GK;
    J.tm = (a.M + 63) / 64;
    J.tn = (a.N + 127) / 128;
    J.slab = slab;
    slab += (size_t)splits * a.M * a.N;
    J.wg0 = wg;
    rj.start[rj.n - 1] = wg;
    wg += J.tm * J.tn * splits;
    J.blk0 = blk;
    rj.rstart[rj.n - 1] = blk;
    blk += (int)(((int64_t)a.M * a.N / 4 + 255) / 256);
  }
  hipStream_t s = (hipStream_t)stream;
  if (b_kmajor)
    hipLaunchKernelGGL(gemm_rows_grouped_kernel<true>, dim3(wg), dim3(256), 0, s, rj);
  else
    hipLaunchKernelGGL(gemm_rows_grouped_kernel<false>, dim3(wg), dim3(256), 0, s, rj);
  HICGAT_CHECK_LAUNCH();
  if (splits > 1) {
    hipLaunchKernelGGL(rows_reduce_kernel, dim3(blk), dim3(256), 0, s, rj);
    HICGAT_CHECK_LAUNCH();
  }
  return HICGAT_OK;
}

extern "C" size_t hicgat_param_grads_workspace_bytes(const hicgat_wgrad_job *w, int nw, int target_wgs) {
  if (nw <= 0 || nw > kMaxWJobs || !w) return 0;
  int splits[kMaxWJobs];
  group_kchunk(w, nw, target_wgs, splits);
  size_t tot = 0;
  for (int i = 0; i < nw; ++i)
    if (splits[i] > 1) tot += (size_t)splits[i] * ((size_t)w[i].M * w[i].N + w[i].M) * sizeof(float);
  return tot;
}

extern "C" int hicgat_param_grads_grouped(const hicgat_wgrad_job *w, int nw, const hicgat_colsum_job *c, int nc,
                                          int target_wgs, void *workspace, size_t workspace_bytes,
                                          hicgat_stream_t stream) {
  if (nw < 0 || nc < 0 || (nw && !w) || (nc && !c)) return HICGAT_EINVAL;
  if (nw > kMaxWJobs) return HICGAT_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  int splits[kMaxWJobs];
  const int kc = nw ? group_kchunk(w, nw, target_wgs, splits) : 0;
  WJobs wj;
  CJobs cj;
  wj.n = 0;
  cj.n = 0;
  int wg = 0, blk = 0;
  float *slab = static_cast<float *>(workspace);
  size_t used = 0;
  auto add_col = [&](const float *src, int64_t ld, int64_t rows, int64_t cols, float *dst, int acc,
                     const float *wt = nullptr, int64_t ldw = 0, int segs = 1, int64_t ldd = 0) {
    if (cols <= 0) return HICGAT_OK;
    if (cj.n == kMaxCJobs) return HICGAT_EUNSUPPORTED;
    if (segs < 1) segs = 1;
    if (segs > 1 && (ldd < cols || rows < segs)) return HICGAT_EINVAL;
    CJob &J = cj.j[cj.n++];
    J.src = src;
    J.dst = dst;
    J.wt = wt;
    J.ld = ld;
    J.ldw = ldw;
    J.ldd = ldd;
    J.segs = segs;
    J.rows = rows;
    J.cols = cols;
    J.accumulate = acc;
    J.vec = (cols % 4 == 0 && ld % 4 == 0 && (segs == 1 || ldd % 4 == 0) &&
             ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0);
    // lanes per row group by the rows of one segment (one lane per group for the tallest jobs,
    // uncoalesced, measured slower: P = 8 rank step 0.447 vs 0.431 ms, profiles/r04m_sim_ab.txt)
    const int64_t srows = (rows + segs - 1) / segs;
    J.lg = srows <= kColsumShortRows ? 8 : srows <= 64 ? 6 : srows <= 256 ? 4
         : (wt && srows > WEIGHTED_LG1_ROWS) ? kWeightedLg : 2;
    J.blk0 = blk;
    cj.start[cj.n - 1] = blk;
    const int64_t per = 4 * ((int64_t)1 << J.lg);   // columns per block
    J.nchunk = (int)((cols + per - 1) / per);
    blk += J.nchunk * segs;
    return HICGAT_OK;
  };
  for (int i = 0; i < nw; ++i) {
    const hicgat_wgrad_job &a = w[i];
    if (a.M < 0 || a.N < 0 || a.K < 0 || a.lddw < a.N) return HICGAT_EINVAL;
    if (a.M == 0 || a.N == 0) continue;
    if (!a.dy || !a.x || !a.dw) return HICGAT_EINVAL;
    WJob &J = wj.j[wj.n++];
    J.dy = a.dy;
    J.x = a.x;
    J.dw = a.dw;
    J.db = a.db;
    J.ldy = a.ldy;
    J.ldx = a.ldx;
    J.lddw = a.lddw;
    J.M = a.M;
    J.N = a.N;
    J.K = a.K;
    J.kchunk = kc;
    J.tm = (a.M + kGroupTile - 1) / kGroupTile;
    J.tn = (a.N + kGroupTile - 1) / kGroupTile;
    J.accumulate = a.accumulate;
    J.vec = (a.M % 4 == 0 && a.ldy % 4 == 0 && a.N % 4 == 0 && a.ldx % 4 == 0 &&
             ((reinterpret_cast<uintptr_t>(a.dy) | reinterpret_cast<uintptr_t>(a.x)) & 15) == 0);
    const int sp = a.K > 0 ? splits[i] : 1;
    J.slab = nullptr;
    if (sp > 1) {
      const size_t need = (size_t)sp * ((size_t)a.M * a.N + a.M) * sizeof(float);
      if (!workspace || used + need > workspace_bytes) return HICGAT_EINVAL;
      J.slab = slab + used / sizeof(float);
      used += need;
    }
    J.wg0 = wg;
    wj.start[wj.n - 1] = wg;
    wg += J.tm * J.tn * sp;
    if (sp > 1) {
      const int64_t stride = (int64_t)a.M * a.N + a.M;
      int rc = add_col(J.slab, stride, sp, (int64_t)a.M * a.N, a.dw, a.accumulate);
      if (rc != HICGAT_OK) return rc;
      if (a.db && (rc = add_col(J.slab + (int64_t)a.M * a.N, stride, sp, a.M, a.db, a.accumulate)) != HICGAT_OK)
        return rc;
    }
  }
  for (int i = 0; i < nc; ++i) {
    if (c[i].rows < 0 || c[i].cols < 0 || (c[i].cols > 0 && !c[i].dst) || (c[i].rows > 0 && !c[i].src))
      return HICGAT_EINVAL;
    const int rc = add_col(c[i].src, c[i].ld, c[i].rows, c[i].cols, c[i].dst, c[i].accumulate, c[i].wt, c[i].ldw,
                           c[i].segs, c[i].ldd);
    if (rc != HICGAT_OK) return rc;
  }
  if (wg > 0) {
    hipLaunchKernelGGL(wgrad_grouped_kernel, dim3(wg), dim3(256), 0, s, wj);
    HICGAT_CHECK_LAUNCH();
  }
  if (blk > 0) {
    hipLaunchKernelGGL(colsum_grouped_kernel, dim3(blk), dim3(256), 0, s, cj);
    HICGAT_CHECK_LAUNCH();
  }
  return HICGAT_OK;
}

extern "C" size_t hicgat_gemm_workspace_bytes(int M, int N, int splits) {
  return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

extern "C" int hicgat_gemm(int a_kmajor, int b_kmajor, int M, int N, int K, const float *A, int64_t lda,
                           const float *B, int64_t ldb, const float *bias, float *C, int64_t ldc, int accumulate,
                           int splits, void *workspace, size_t workspace_bytes, hicgat_stream_t stream) {
  return hicgat_gemm_ex(a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, bias, C, ldc, accumulate, splits,
                        HICGAT_GEMM_AUTO, workspace, workspace_bytes, stream);
}

extern "C" int hicgat_gemm_ex(int a_kmajor, int b_kmajor, int M, int N, int K, const float *A, int64_t lda,
                              const float *B, int64_t ldb, const float *bias, float *C, int64_t ldc,
                              int accumulate, int splits, int impl, void *workspace, size_t workspace_bytes,
                              hicgat_stream_t stream) {
  if (impl == HICGAT_GEMM_X3) return HICGAT_EUNSUPPORTED;   // the bf16 x3 split was measured slower and removed
  if (impl != HICGAT_GEMM_AUTO && impl != HICGAT_GEMM_F32) return HICGAT_EINVAL;
  if (M < 0 || N < 0 || K < 0 || splits < 1) return HICGAT_EINVAL;
  if (M == 0 || N == 0) return HICGAT_OK;
  if (!A || !B || !C) return HICGAT_EINVAL;
  if (splits > 1 && (!workspace || workspace_bytes < hicgat_gemm_workspace_bytes(M, N, splits)))
    return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float *slab = static_cast<float *>(workspace);
  const int i = impl;
  if (!a_kmajor && !b_kmajor) return dispatch<false, false>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, i, s);
  if (!a_kmajor && b_kmajor) return dispatch<false, true>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, i, s);
  if (a_kmajor && !b_kmajor) return dispatch<true, false>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, i, s);
  return dispatch<true, true>(A, lda, B, ldb, C, ldc, M, N, K, splits, bias, slab, accumulate, i, s);
}

extern "C" size_t hicgat_gemm_wgrad_workspace_bytes(int M, int N, int splits) {
  return splits > 1 ? (size_t)splits * ((size_t)M * N + M) * sizeof(float) : 0;
}

extern "C" int hicgat_gemm_wgrad(int M, int N, int K, const float *dY, int64_t ldy, const float *X, int64_t ldx,
                                 float *dW, int64_t lddw, float *db, int accumulate, int splits, void *workspace,
                                 size_t workspace_bytes, hicgat_stream_t stream) {
  if (M < 0 || N < 0 || K < 0 || splits < 1 || lddw < N) return HICGAT_EINVAL;
  if (M == 0 || N == 0) return HICGAT_OK;
  if (!dY || !X || !dW) return HICGAT_EINVAL;
  if (splits > 1 && (!workspace || workspace_bytes < hicgat_gemm_wgrad_workspace_bytes(M, N, splits)))
    return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float *slab = static_cast<float *>(workspace);
  // the dispatch of hicgat_gemm_ex's fp32 path for the (K-major, K-major) layout
  if (M >= 128 && N >= 128 && M <= 1024)
    return launch<128, 128, true, true>(dY, ldy, X, ldx, dW, lddw, M, N, K, splits, nullptr, slab, accumulate, s, db);
  if (N >= 128) return launch<64, 128, true, true>(dY, ldy, X, ldx, dW, lddw, M, N, K, splits, nullptr, slab, accumulate, s, db);
  return launch<64, 64, true, true>(dY, ldy, X, ldx, dW, lddw, M, N, K, splits, nullptr, slab, accumulate, s, db);
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
