// fp32 MFMA weight-gradient GEMM fed by LDS-DMA: dW[M,N] (+)= dY^T X over K = node rows, split
// over K into fp32 slabs (a10: the dW of every Linear of the tail and of PyG's lin_l,
// models.py:619,637-659; ATen/MKL sgemm on the CPU).
//
//   dY [K,M] and X [K,N] row-major (both K-major operands), M and N multiples of 128.
//
// Shape (MI355X, v_mfma_f32_32x32x2_f32 = exact fp32 products, fp32 accumulate):
//  * 128 x 128 tiles, 4 waves in 2 x 2 (a wave: 64 x 64 = four 32x32 accumulators, 64 VGPRs);
//  * K in 16-deep stages through a 3-slot LDS ring (48 KiB: three workgroups per CU) filled by
//    LDS-DMA (global_load_lds_dwordx4): a stage is 16 k-rows x 128 floats of each operand = 16
//    1-KiB pieces (two k-rows each), four per wave; stage s+2 is issued right after the barrier
//    that opens stage s, so two stages are in flight behind the MFMAs -- one raw barrier and one
//    counted vmcnt per stage, no VGPR staging, no LDS stores (gemm.hip's kernel stages through
//    VGPRs with two barriers per stage and one stage of cover);
//  * the K-major image is exactly the MFMA operand layout: lane (i, l) of a 32x32x2 MFMA reads
//    k-row 2p + l, element i -- 32 consecutive floats per half wave, conflict-free ds_read_b32;
//  * the fragment reads are inline asm (as in gemm_tall.hip): the compiler cannot tell the ring
//    slots apart and would wait for every LDS-DMA in flight before each read;
//  * a split's last partial stage: rows past the split's end are loaded (clamped into the
//    matrix) and zeroed in the A fragment, so they add nothing;
//  * CS: the workgroups of the first column tile also sum their A tile over k (db = column sums
//    of dY, the Linear's bias gradient), from the same LDS image;
//  * XCD-aware: the M/128 x N/128 tiles of one K split run on one XCD, so that split's rows of dY
//    and X are read into one L2.
// Deterministic: fixed k order within a split, the slabs added in split order by reduce.hip.
#include "common.hpp"
#include "reduce.hpp"

namespace hicgat {

namespace {

constexpr int WBM = 128, WBN = 128, WBK = 16, WSLOTS = 3;
constexpr int WA_F = WBK * WBM;                  // floats of an A stage (8 KiB)
constexpr int WSTAGE_F = WA_F + WBK * WBN;       // A + B stage (16 KiB)
constexpr size_t kWgradLds = (size_t)WSLOTS * WSTAGE_F * sizeof(float);
constexpr int WPIECES = WSTAGE_F * 4 / 1024;     // 1-KiB LDS-DMA pieces per stage (16: 4 per wave)

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void wgrad_issue(float *stage, const float *__restrict__ dY, int64_t ldy, int m0,
                                            const float *__restrict__ X, int64_t ldx, int n0, int k0, int K, int w,
                                            int lane) {
  const int kl = k0 + (lane >> 5), c4 = (lane & 31) * 4;
#pragma unroll
  for (int j = 0; j < WPIECES / 4; ++j) {
    const int p = w + 4 * j;                      // pieces 0..7: A (dY), 8..15: B (X)
    const int q = p & 7;                          // k-rows 2q, 2q + 1 of the stage
    const int k = min(kl + 2 * q, K - 1);
    const float *src = p < 8 ? dY + (size_t)k * ldy + m0 + c4 : X + (size_t)k * ldx + n0 + c4;
    __builtin_amdgcn_global_load_lds(src, stage + (p < 8 ? 0 : WA_F) + q * 256, 16, 0, 0);
  }
}

// The LDS reads of one stage, 16 ds_read_b32 and their wait in one statement (so no use can be
// scheduled in between).  FRAG16: entry 2j + a = k-pair j (k-row 2j + lane/32), 32-row block a of
// this wave's 64 rows (or columns): byte offset 1024 j + 128 a.  COL16: entry r = k-row r of one
// column: byte offset 512 r.
#define HICGAT_WG_FRAG16(o, base) \
  asm volatile("ds_read_b32 %0, %16 offset:0\n\t" \
               "ds_read_b32 %1, %16 offset:128\n\t" \
               "ds_read_b32 %2, %16 offset:1024\n\t" \
               "ds_read_b32 %3, %16 offset:1152\n\t" \
               "ds_read_b32 %4, %16 offset:2048\n\t" \
               "ds_read_b32 %5, %16 offset:2176\n\t" \
               "ds_read_b32 %6, %16 offset:3072\n\t" \
               "ds_read_b32 %7, %16 offset:3200\n\t" \
               "ds_read_b32 %8, %16 offset:4096\n\t" \
               "ds_read_b32 %9, %16 offset:4224\n\t" \
               "ds_read_b32 %10, %16 offset:5120\n\t" \
               "ds_read_b32 %11, %16 offset:5248\n\t" \
               "ds_read_b32 %12, %16 offset:6144\n\t" \
               "ds_read_b32 %13, %16 offset:6272\n\t" \
               "ds_read_b32 %14, %16 offset:7168\n\t" \
               "ds_read_b32 %15, %16 offset:7296\n\t" \
               "s_waitcnt lgkmcnt(0)" \
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]), "=&v"(o[14]), "=&v"(o[15]) \
               : "v"(base) \
               : "memory")

#define HICGAT_WG_COL16(o, base) \
  asm volatile("ds_read_b32 %0, %16 offset:0\n\t" \
               "ds_read_b32 %1, %16 offset:512\n\t" \
               "ds_read_b32 %2, %16 offset:1024\n\t" \
               "ds_read_b32 %3, %16 offset:1536\n\t" \
               "ds_read_b32 %4, %16 offset:2048\n\t" \
               "ds_read_b32 %5, %16 offset:2560\n\t" \
               "ds_read_b32 %6, %16 offset:3072\n\t" \
               "ds_read_b32 %7, %16 offset:3584\n\t" \
               "ds_read_b32 %8, %16 offset:4096\n\t" \
               "ds_read_b32 %9, %16 offset:4608\n\t" \
               "ds_read_b32 %10, %16 offset:5120\n\t" \
               "ds_read_b32 %11, %16 offset:5632\n\t" \
               "ds_read_b32 %12, %16 offset:6144\n\t" \
               "ds_read_b32 %13, %16 offset:6656\n\t" \
               "ds_read_b32 %14, %16 offset:7168\n\t" \
               "ds_read_b32 %15, %16 offset:7680\n\t" \
               "s_waitcnt lgkmcnt(0)" \
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]), "=&v"(o[14]), "=&v"(o[15]) \
               : "v"(base) \
               : "memory")

}  // namespace

template <bool CS>
__global__ __launch_bounds__(256, 2) void gemm_wgrad_dma_kernel(const float *__restrict__ dY, int64_t ldy,
                                                               const float *__restrict__ X, int64_t ldx,
                                                               float *__restrict__ C, int64_t ldc, int M, int N,
                                                               int K, int kchunk, float *__restrict__ slab,
                                                               int64_t slab_stride, int accumulate,
                                                               float *__restrict__ csum) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, w = wave_in_block();
  const int li = lane & 31, lk = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int tm = M / WBM, tiles = tm * (N / WBN);
  const int id = xcd_remap(blockIdx.x, gridDim.x);          // consecutive ids: tiles of one split
  const int z = id / tiles, t = id % tiles;
  const int mt = t % tm, nt = t / tm;
  const int m0 = mt * WBM, n0 = nt * WBN;
  const int kb = z * kchunk, ke = min(K, kb + kchunk);
  const int S = ke > kb ? (ke - kb + WBK - 1) / WBK : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const bool cs_on = CS && nt == 0 && w < 2;      // threads 0..127: column threadIdx.x of the A tile
  float cs = 0.f;

  if (S > 0) wgrad_issue(lds, dY, ldy, m0, X, ldx, n0, kb, K, w, lane);
  if (S > 1) wgrad_issue(lds + WSTAGE_F, dY, ldy, m0, X, ldx, n0, kb + WBK, K, w, lane);

  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const uint32_t a_off = (uint32_t)((lk * WBM + 64 * wm + li) * 4);
  const uint32_t b_off = (uint32_t)((WA_F + lk * WBN + 64 * wn + li) * 4);
  const uint32_t c_off = (uint32_t)(threadIdx.x * 4);

  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // every wave's copy of stage s landed; every wave is past stage s-1
    asm volatile("" ::: "memory");
    if (s + 2 < S)
      wgrad_issue(lds + ((s + 2) % WSLOTS) * WSTAGE_F, dY, ldy, m0, X, ldx, n0, kb + (s + 2) * WBK, K, w, lane);
    const uint32_t st = lds_base + (uint32_t)((s % WSLOTS) * WSTAGE_F * 4);
    const int k0 = kb + s * WBK;
    const bool tail = k0 + WBK > ke;              // uniform: the split's last, partial stage
    float av[16], bv[16];
    HICGAT_WG_FRAG16(av, st + a_off);
    HICGAT_WG_FRAG16(bv, st + b_off);
    if (tail) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + 2 * j + lk >= ke) av[2 * j] = av[2 * j + 1] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[2 * j + a], bv[2 * j + b], acc[a][b], 0, 0, 0);
    if (cs_on) {
      float cv[16];
      HICGAT_WG_COL16(cv, st + c_off);
#pragma unroll
      for (int r = 0; r < 16; ++r) cs += (k0 + r < ke) ? cv[r] : 0.f;
    }
  }
  if (cs_on) {
    const int m = m0 + (int)threadIdx.x;
    if (slab) {
      csum[(size_t)z * slab_stride + m] = cs;      // csum = the slab's db part (slab + M*N)
    } else {
      float *o = csum + m;
      *o = cs + (accumulate ? *o : 0.f);
    }
  }

  // C/D map of a 32x32 f32 tile: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float *out = slab ? slab + (size_t)z * slab_stride : C;
  const int64_t ldo = slab ? N : ldc;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int gn = n0 + 64 * wn + 32 * b + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + 64 * wm + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * lk;
        float *o = out + (size_t)gm * ldo + gn;
        *o = acc[a][b][r] + ((accumulate && !slab) ? *o : 0.f);
      }
    }
}

// Takes the weight gradient when it fits the tiling (M, N multiples of 128, 16-B aligned float4
// rows); HICGAT_EUNSUPPORTED otherwise (the caller then uses gemm.hip's 128 x 128 kernel).  The
// slab layout and the slab sum are those of gemm.hip's split-K path: split z writes
// [M*N dW partials | M db partials] at slab + z * (M*N + M) (db part only with csum).
int gemm_wgrad_dma_launch(const float *dY, int64_t ldy, const float *X, int64_t ldx, float *C, int64_t ldc, int M,
                          int N, int K, int splits, float *slab, int accumulate, float *csum, hipStream_t s) {
  static const bool on = !(getenv("HICGAT_WGRAD_DMA") && atoi(getenv("HICGAT_WGRAD_DMA")) == 0);
  const bool al = ((reinterpret_cast<uintptr_t>(dY) | reinterpret_cast<uintptr_t>(X)) & 15) == 0;
  if (!on || !al || M % WBM || N % WBN || K < 1 || ldy % 4 || ldx % 4) return HICGAT_EUNSUPPORTED;
  const int kchunk = ((K + splits - 1) / splits + WBK - 1) / WBK * WBK;
  const int64_t blocks = (int64_t)(M / WBM) * (N / WBN) * splits;
  if (blocks > 0x7fffffff) return HICGAT_EUNSUPPORTED;
  const bool cs = csum != nullptr;
  const int64_t stride = (int64_t)M * N + (cs ? M : 0);
  float *sl = splits > 1 ? slab : nullptr;
  float *cdst = cs ? (sl ? slab + (int64_t)M * N : csum) : nullptr;
  if (cs)
    hipLaunchKernelGGL(gemm_wgrad_dma_kernel<true>, dim3((unsigned)blocks), dim3(256), kWgradLds, s, dY, ldy, X, ldx,
                       C, ldc, M, N, K, kchunk, sl, stride, accumulate, cdst);
  else
    hipLaunchKernelGGL(gemm_wgrad_dma_kernel<false>, dim3((unsigned)blocks), dim3(256), kWgradLds, s, dY, ldy, X,
                       ldx, C, ldc, M, N, K, kchunk, sl, stride, accumulate, cdst);
  HICGAT_CHECK_LAUNCH();
  if (splits > 1) {
    const ColOut o{C, ldc, N, nullptr, nullptr, accumulate, cs ? csum : nullptr, (int64_t)M * N};
    return colsum_wide_launch(slab, stride, splits, stride, o, s);
  }
  return HICGAT_OK;
}

}  // namespace hicgat
