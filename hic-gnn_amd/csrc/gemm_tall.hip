// fp32 MFMA GEMM for the tall node-row problems of the MLP tail and lin_l (a2, a6): M = node rows
// (20000) against N = 128..512 output features, K = 64..512.
//
//   C[M,N] (+)= A[M,K] op(B) (+ bias[N]);  A row-major (k contiguous);
//   BKC = true : op(B) = B^T of B [N,K] (Linear forward, W [out, in]);
//   BKC = false: op(B) = B of B [K,N]   (input gradient dX = dY W).
//
// Reference: torch.nn.Linear forward / input gradient inside models.py:637-659 and PyG's lin_l
// (models.py:619), ATen/MKL sgemm on the CPU.
//
// Shape of the kernel (MI355X, v_mfma_f32_32x32x2_f32 = exact fp32 products, fp32 accumulate):
//  * 160 x 128 tiles: 20000 rows = 125 row tiles, so N = 512 gives 500 workgroups = two per CU in one
//    round (a 128-row tile leaves 2.45 rounds, i.e. a third of the chip idle in the last one);
//  * 4 waves, wave w owns all 160 rows x columns 32w..32w+31: five 32x32 accumulators (80 VGPRs);
//  * K in 16-deep stages through a 3-slot LDS ring filled by LDS-DMA (global_load_lds_dwordx4): the
//    stage s+2 copy is issued right after the barrier that opens stage s, so two stages are in
//    flight behind the MFMAs; one raw barrier per stage, counted vmcnt waits, no VGPR staging;
//  * k-contiguous operands (A, and B when BKC) sit in LDS as [row][16] with the 16-B k-groups
//    XOR-swizzled by row (group g of row r at slot g ^ ((r >> 2) & 3)), so the fragment reads are
//    conflict-free ds_read_b128: lane (i, l) of a 32x32x2 MFMA holds k-groups 2p + l of its row, and
//    the four MFMAs of a group pair take component c of both: k order (8p + c, 8p + 4 + c);
//  * a [K,N] B (BKC = false) sits as [k][128] and is read as ds_read_b32 of 32 consecutive columns;
//  * the fragment reads are inline asm: the compiler cannot tell the ring slots apart and would put
//    an s_waitcnt vmcnt(0) (both stages in flight) in front of every LDS read.  Their outputs are
//    early-clobber (=&v): a ds_read result may land before the block's last read has issued, so no
//    output may share a register with an address input.
// Results are deterministic (fixed k order); they differ from the 64x128 kernel of gemm.hip by the
// fp32 rounding of that order only.
#include "common.hpp"

namespace hicgat {

namespace {

constexpr int TBM = 160, TBN = 128, TBK = 16, TSLOTS = 3;
constexpr int TA_F = TBM * TBK;                  // floats of an A stage (10 KiB)
constexpr int TB_F = TBN * TBK;                  // floats of a B stage (8 KiB)
constexpr int TSTAGE_F = TA_F + TB_F;
constexpr size_t kTallLds = (size_t)TSLOTS * TSTAGE_F * sizeof(float);   // 54 KiB: two workgroups per CU
constexpr int TA_PIECES = TA_F * 4 / 1024;       // 1-KiB LDS-DMA pieces per A stage (10)
constexpr int TB_PIECES = TB_F * 4 / 1024;       // (8)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int kc_slot(int r, int g) { return g ^ ((r >> 2) & 3); }

template <bool BKC>
__device__ __forceinline__ void tall_issue(float *stage, const float *__restrict__ A, int64_t lda, int m0, int M,
                                           const float *__restrict__ B, int64_t ldb, int n0, int k0, int w,
                                           int lane) {
  // A: piece p = rows 16p .. 16p+15 of the tile; lane -> row 16p + lane/4, slot lane%4, which holds
  // k-group slot ^ swizzle(row)
  for (int p = w; p < TA_PIECES; p += 4) {
    const int r = 16 * p + (lane >> 2), s = lane & 3;
    const int gm = min(m0 + r, M - 1);
    const float *src = A + (size_t)gm * lda + k0 + 4 * kc_slot(r, s);
    __builtin_amdgcn_global_load_lds(src, stage + p * 256, 16, 0, 0);
  }
  float *bs = stage + TA_F;
  for (int p = w; p < TB_PIECES; p += 4) {
    const float *src;
    if (BKC) {   // [N,K]: the same swizzled [row][16] image
      const int r = 16 * p + (lane >> 2), s = lane & 3;
      src = B + (size_t)(n0 + r) * ldb + k0 + 4 * kc_slot(r, s);
    } else {     // [K,N]: k-rows 2p, 2p+1 of 128 columns
      const int t = 2 * p + (lane >> 5);
      src = B + (size_t)(k0 + t) * ldb + n0 + (lane & 31) * 4;
    }
    __builtin_amdgcn_global_load_lds(src, bs + p * 256, 16, 0, 0);
  }
}

}  // namespace

template <bool BKC>
__global__ __launch_bounds__(256, 2) void gemm_tall_kernel(const float *__restrict__ A, int64_t lda,
                                                          const float *__restrict__ B, int64_t ldb,
                                                          float *__restrict__ C, int64_t ldc, int M, int N, int K,
                                                          const float *__restrict__ bias, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, w = wave_in_block();
  const int li = lane & 31, lk = lane >> 5;
  // XCD-aware: the N/128 column tiles of one row tile run on one XCD (A read once into its L2)
  const int ntn = N / TBN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / ntn) * TBM, n0 = (tile % ntn) * TBN;
  const int S = K / TBK;
  f32x16 acc[5];
#pragma unroll
  for (int t = 0; t < 5; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  tall_issue<BKC>(lds, A, lda, m0, M, B, ldb, n0, 0, w, lane);
  if (S > 1) tall_issue<BKC>(lds + TSTAGE_F, A, lda, m0, M, B, ldb, n0, TBK, w, lane);
  const bool w_more = w < TA_PIECES - 8;   // waves 0, 1 issue 5 pieces per stage, waves 2, 3 issue 4

  // per-lane LDS byte addresses of the fragments: row 32t + li of A is at t * 2048 B from row li, and
  // its swizzle (row >> 2) & 3 = (li >> 2) & 3 does not depend on t
  const int bcol = 32 * w + li;
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const uint32_t a_row = (uint32_t)(li * TBK * 4);
  const uint32_t b_row = (uint32_t)(TA_F * 4) + (BKC ? (uint32_t)(bcol * TBK * 4) : (uint32_t)(bcol * 4));

  for (int s = 0; s < S; ++s) {
    // this wave's copy of stage s has landed (stage s+1, when there is one, may stay in flight)
    if (s + 1 < S) {
      if (w_more) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave's copy landed; every wave is past stage s-1's reads
    asm volatile("" ::: "memory");
    if (s + 2 < S)
      tall_issue<BKC>(lds + ((s + 2) % TSLOTS) * TSTAGE_F, A, lda, m0, M, B, ldb, n0, (s + 2) * TBK, w, lane);
    const uint32_t st = lds_base + (uint32_t)((s % TSLOTS) * TSTAGE_F * 4);
#pragma unroll
    for (int p = 0; p < TBK / 8; ++p) {   // k-group pairs of the stage
      const int g = 2 * p + lk;
      const uint32_t aa = st + a_row + (uint32_t)(kc_slot(li, g) * 16);
      f4v a0, a1, a2, a3, a4;
      float bk[4];
      // one asm statement for the reads and their wait, so no use can be scheduled in between
      if (BKC) {
        const uint32_t ba = st + b_row + (uint32_t)(kc_slot(bcol, g) * 16);
        f4v b;
        asm volatile(
            "ds_read_b128 %0, %6\n\tds_read_b128 %1, %6 offset:2048\n\tds_read_b128 %2, %6 offset:4096\n\t"
            "ds_read_b128 %3, %6 offset:6144\n\tds_read_b128 %4, %6 offset:8192\n\tds_read_b128 %5, %7\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(a4), "=&v"(b)
            : "v"(aa), "v"(ba)
            : "memory");
        bk[0] = b.x;
        bk[1] = b.y;
        bk[2] = b.z;
        bk[3] = b.w;
      } else {
        const uint32_t ba = st + b_row + (uint32_t)((8 * p + 4 * lk) * TBN * 4);
        asm volatile(
            "ds_read_b128 %0, %9\n\tds_read_b128 %1, %9 offset:2048\n\tds_read_b128 %2, %9 offset:4096\n\t"
            "ds_read_b128 %3, %9 offset:6144\n\tds_read_b128 %4, %9 offset:8192\n\t"
            "ds_read_b32 %5, %10\n\tds_read_b32 %6, %10 offset:512\n\tds_read_b32 %7, %10 offset:1024\n\t"
            "ds_read_b32 %8, %10 offset:1536\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(a4), "=&v"(bk[0]), "=&v"(bk[1]), "=&v"(bk[2]), "=&v"(bk[3])
            : "v"(aa), "v"(ba)
            : "memory");
      }
      const f4v a[5] = {a0, a1, a2, a3, a4};
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < 5; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t][c], bk[c], acc[t], 0, 0, 0);
    }
  }

  // C/D map of a 32x32 f32 tile: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int gn = n0 + bcol;
  const float bb = bias ? bias[gn] : 0.f;
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    float old[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) old[r] = 0.f;
    if (accumulate) {   // the tile's 16 old values in flight together (rows past M: row M-1, unused)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = min(m0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * lk, M - 1);
        old[r] = C[(size_t)gm * ldc + gn];
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int gm = m0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * lk;
      if (gm < M) C[(size_t)gm * ldc + gn] = acc[t][r] + bb + old[r];
    }
  }
}

// The tall kernel takes the problem when it fits its tiling: returns HICGAT_EUNSUPPORTED otherwise
// (the caller then uses the 64x128 kernel of gemm.hip).
int gemm_tall_launch(bool b_kmajor, const float *A, int64_t lda, const float *B, int64_t ldb, float *C, int64_t ldc,
                     int M, int N, int K, const float *bias, int accumulate, hipStream_t s) {
  const bool al = ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0;
  if (!al || M < TBM || N % TBN || K % TBK || K < TBK || lda % 4 || ldb % 4) return HICGAT_EUNSUPPORTED;
  const int64_t tiles = (int64_t)((M + TBM - 1) / TBM) * (N / TBN);
  if (tiles > 0x7fffffff) return HICGAT_EUNSUPPORTED;
  if (b_kmajor)
    hipLaunchKernelGGL(gemm_tall_kernel<false>, dim3((unsigned)tiles), dim3(256), kTallLds, s, A, lda, B, ldb, C, ldc, M,
                       N, K, bias, accumulate);
  else
    hipLaunchKernelGGL(gemm_tall_kernel<true>, dim3((unsigned)tiles), dim3(256), kTallLds, s, A, lda, B, ldb, C, ldc, M,
                       N, K, bias, accumulate);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

}  // namespace hicgat
