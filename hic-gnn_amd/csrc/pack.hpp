// The one-kernel tail's packed weight copies (hicgat_tail_pack): layout constants, the job table
// and the per-block copy, shared by the launches the pack can ride in (tail_fused.hip: its own launch
// and the single-GPU step's first launch; gat_xagg.hip: the sharded step's first launch).
#pragma once
#include "common.hpp"

namespace hicgat {

// ---- packed weight copies (hicgat_tail_pack) ------------------------------------------------------
// Float offsets in the pack buffer: the forward (mfma_rows) layouts of W1c [512][512], W2c [256][256]
// and Wh [512][512], then their backward (mfma_rows_t) layouts.
constexpr int64_t kPackF1 = 0, kPackF2 = kPackF1 + 512 * 512, kPackFH = kPackF2 + 256 * 256,
                  kPackB1 = kPackFH + 512 * 512, kPackB2 = kPackB1 + 512 * 512, kPackBH = kPackB2 + 256 * 256,
                  kPackTotal = kPackBH + 512 * 512;
struct PackJob {
  const float *src;   // [R][C] row-major
  float *dst;
  int R, C, bwd, blk0;
};
struct PackJobs {
  PackJob j[6];
  int n;
};
// One wave per unit: the forward layout's unit is a 16-row x 32-column block of W (the two 1 KB
// chunks e = 0, 1 of super-group g), the backward layout's a 16 x 16 block (one 1 KB chunk).  The
// wave reads the block as whole 128-B / 64-B row pieces (contiguous quads of lanes), turns it
// through LDS and writes its chunks as 1 KB contiguous -- a lane-per-row read or write runs the
// vector memory path at a quarter of the rate (tools/ld_pattern_bench.hip).
// the wave's LDS writes visible to its other lanes' reads
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void pack_block(const PackJobs &jobs, int blk) {
  __shared__ float tile[4][16][36];
  int q = 0;
#pragma unroll
  for (int k = 1; k < 6; ++k) q += (k < jobs.n && blk >= jobs.j[k].blk0) ? 1 : 0;
  const PackJob &J = jobs.j[q];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int u = (blk - J.blk0) * 4 + wv;                              // this wave's unit
  float (*T)[36] = tile[wv];
  float4 *out = reinterpret_cast<float4 *>(J.dst);
  if (!J.bwd) {   // P[((b * G + g) * 2 + e) * 256 + 4L + c] = W[16b + (L & 15)][32g + 8(L >> 4) + 4e + c]
    const int G = J.C / 32;
    if (u >= (J.R / 16) * G) return;                                   // wave-uniform
    const int b = u / G, g = u % G;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int t = lane + 64 * h, r = t >> 3, c4 = t & 7;
      *reinterpret_cast<float4 *>(&T[r][4 * c4]) =
          *reinterpret_cast<const float4 *>(J.src + (size_t)(16 * b + r) * J.C + 32 * g + 4 * c4);
    }
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < 2; ++e)
      out[((size_t)u * 2 + e) * 64 + lane] = *reinterpret_cast<const float4 *>(&T[lane & 15][8 * (lane >> 4) + 4 * e]);
  } else {        // P[((g * (C / 16) + c) * 64 + L) * 4 + s] = W[16g + 4(L >> 4) + s][16c + (L & 15)]
    const int CB = J.C / 16;
    if (u >= (J.R / 16) * CB) return;
    const int g = u / CB, cb = u % CB;
    const int r = lane >> 2, c4 = lane & 3;
    *reinterpret_cast<float4 *>(&T[r][4 * c4]) =
        *reinterpret_cast<const float4 *>(J.src + (size_t)(16 * g + r) * J.C + 16 * cb + 4 * c4);
    wave_lds_sync();
    const int r0 = 4 * (lane >> 4), cc = lane & 15;
    out[(size_t)u * 64 + lane] = make_float4(T[r0][cc], T[r0 + 1][cc], T[r0 + 2][cc], T[r0 + 3][cc]);
  }
}

// the job table of one pack (blocks per weight and layout); the block count, or a HICGAT_E* code < 0
int pack_jobs(const float *W1c, const float *W2c, const float *Wh, void *pack, size_t pack_bytes, PackJobs &pj);
// the library's record of whether a pack buffer's last pack included Wh (tail_fused.hip)
void pack_note(const void *pack, bool heads);
bool pack_has_heads(const void *pack);

}  // namespace hicgat
