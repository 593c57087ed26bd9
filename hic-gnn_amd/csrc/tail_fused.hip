// The flagship's MLP tail forward (GATNetSelectiveResidualsUpdated, models.py:637-659, after the
// GATConv's relu) as ONE kernel: 16 node rows per 4-wave workgroup go through
//   block 1   Y1 = x [W_a; W_al]^T + [b_a; b_al]          (512 -> 512, fp32 MFMA)
//             z1 = relu(LN_a(Y1[:, :256])) + Y1[:, 256:]
//   block 2   Y2 = z1 [W_1; W_1al]^T + [b_1; b_1al]       (256 -> 256)
//             z2 = relu(LN_1(Y2[:, :128])) + Y2[:, 128:]
//   block 3   y3 = z2 W_2^T + b_2                          (128 -> 64)
//             z3 = relu(LN_2(y3))
//   dense3    coords = z3 W_3^T + b_3                       (64 -> 3)
// with every intermediate in LDS, instead of 10 launches (4 GEMMs, 3 LayerNorm passes, 3 split-K
// slab sums on a rank's shard) whose every output makes a round trip through HBM.  The backward
// still needs Y1, z1, Y2, z2, y3, z3 and the LN statistics (the unfused autograd functions save
// exactly these), so they are written once on the way.
//
// GEMMs: v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate).  Lane l supplies
// A[l & 15][k] and B[k][l & 15]; the four k slots of one instruction are taken as k = 16g + 4(l >> 4)
// + s for step s of the 16-deep group g, so a lane's four values of a group are ONE float4 -- a
// ds_read_b128 of the activations (LDS) and a global float4 of the weight row (L2) -- and the
// weights of group g + 4 are loaded right after group g's MFMAs.  C/D: col = l & 15, row = 4(l >> 4)
// + r.  The k order is fixed (deterministic); it differs from the tiled GEMMs' by fp32 rounding.
// LayerNorm: one wave per row, the arithmetic of ln_relu_res_fwd_kernel (layernorm.hip) on the row
// held in LDS (torch.nn.LayerNorm: biased variance, eps 1e-5 inside the square root).
#include "common.hpp"
#include "pack.hpp"

#include <algorithm>
#include <mutex>
#include <unordered_map>

extern "C" size_t hicgat_ln_relu_res_workspace_bytes(int W);   // layernorm.hip

namespace hicgat {

constexpr int XS = 516;         // LDS row stride (floats) of the 512-wide buffers
typedef float f32x4 __attribute__((ext_vector_type(4)));

// The compiler's scheduler sinks the ring's weight loads next to the MFMAs that use them (one group
// in flight: every L2 latency exposed); a scheduling barrier after each group's loads keeps them R
// groups ahead: P = 8 rank step 0.426-0.427 vs 0.431-0.432 ms, synth-2000 0.597 vs 0.604 ms without
// the barriers; R = 8: 0.442 (profiles/r04n_sim_ab.txt)
#define HICGAT_TAIL_SCHED() __builtin_amdgcn_sched_barrier(0)
constexpr int kTailRing = 4;   // weight groups in flight per wave (the prefetch ring's depth)

// acc[h][t] (h < RB/16 row halves, t < NT) += A[RB x K] (LDS, row stride lda) x B^T, B = the weight
// rows n0 + 16t + (l & 15) (K columns), in k super-groups of 32: lane l loads floats
// 32G + 8(l >> 4) .. + 7 of its row as two float4, so one load pair covers whole 128-B lines of 16
// rows (a 16-deep group per load read half lines, and the other half came back from L2 a group
// later: the forward GEMMs ran at half the backward's MFMA rate, tools/tail_stamps.py).  The MFMA's
// four k slots of step s of half e are 32G + 8(l >> 4) + 4e + s.  The weights of super-group G + R
// are loaded right after G's MFMAs (a ring of R = 2 super-groups: 64 k ahead).
//
// PK: W is the PACKED copy of the weight (hicgat_tail_pack): the two float4 of lane l for rows
// 16b .. 16b + 15 and super-group G sit at ((b * (K / 32) + G) * 2 + e) * 256 + 4l, so each load
// instruction reads 1 KB contiguous.  The row-major rows put the 64 lanes of one load on 16 rows;
// the vector memory path then serves 16 B per clock per CU where contiguous quads of lanes get
// 64 B (tools/ld_pattern_bench.hip: 16.0 vs 63.5 B/clk), and the weight stream, not the MFMAs, set
// every GEMM phase's pace (half the MFMA rate, profiles/r05rs_tail_bound.txt).  Same values in the
// same registers: bitwise the row-major form.
template <int RB, int NT, int K, bool PK = false>
__device__ __forceinline__ void mfma_rows(const float *__restrict__ As, int lda, const float *__restrict__ W, int n0,
                                          f32x4 (&acc)[RB / 16][NT], int lane) {
  constexpr int G = K / 32, H = RB / 16, R = 2;
  static_assert(K % 64 == 0 && G % R == 0, "K: a multiple of 64");
  const int li = lane & 15, kq = 8 * (lane >> 4);
  const float *wrow = W + (size_t)(n0 + li) * K + kq;
  const float *arow = As + li * lda + kq;
  // weight float4 e of super-group g for tile t (row-major or packed)
  auto wld = [&](int t, int g, int e) -> float4 {
    if constexpr (PK)
      return *reinterpret_cast<const float4 *>(W + (((size_t)(n0 / 16 + t) * G + g) * 2 + e) * 256 + 4 * lane);
    else
      return *reinterpret_cast<const float4 *>(wrow + (size_t)16 * t * K + 32 * g + 4 * e);
  };
  float4 b[R][NT][2];
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 2; ++e) b[q][t][e] = wld(t, q, e);
  // the activations of super-group g + 1 are read from LDS before g's MFMAs (two register slots)
  float4 a[2][H][2];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int e = 0; e < 2; ++e) a[0][h][e] = *reinterpret_cast<const float4 *>(arow + h * 16 * lda + 4 * e);
  HICGAT_TAIL_SCHED();   // the ring's loads stay issued here, ahead of their MFMAs
  for (int g0 = 0; g0 < G; g0 += R) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int g = g0 + q, cur = q & 1;   // R even: g and q have the same parity
      if (g + 1 < G) {
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
          for (int e = 0; e < 2; ++e)
            a[cur ^ 1][h][e] = *reinterpret_cast<const float4 *>(arow + h * 16 * lda + 32 * (g + 1) + 4 * e);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int h = 0; h < H; ++h) {
            acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h][e].x, b[q][t][e].x, acc[h][t], 0, 0, 0);
            acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h][e].y, b[q][t][e].y, acc[h][t], 0, 0, 0);
            acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h][e].z, b[q][t][e].z, acc[h][t], 0, 0, 0);
            acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h][e].w, b[q][t][e].w, acc[h][t], 0, 0, 0);
          }
      if (g + R < G) {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int e = 0; e < 2; ++e) b[q][t][e] = wld(t, g + R, e);
      }
      HICGAT_TAIL_SCHED();
    }
  }
}

// acc + bias -> LDS rows (stride lds) and the global output (rows < M, row stride ldo)
template <int RB, int NT>
__device__ __forceinline__ void store_tiles(const f32x4 (&acc)[RB / 16][NT], int n0, const float *__restrict__ bias,
                                            float *__restrict__ Ls, int lds, float *__restrict__ out, int ldo,
                                            int m0, int M, int lane) {
  const int li = lane & 15, r0 = 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = n0 + 16 * t + li;
    const float bb = bias[c];
#pragma unroll
    for (int h = 0; h < RB / 16; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * h + r0 + r;
        const float v = acc[h][t][r] + bb;
        Ls[row * lds + c] = v;
        if (m0 + row < M) out[(size_t)(m0 + row) * ldo + c] = v;
      }
  }
}

// one wave per row: z = relu((y - mean) rstd gamma + beta) (+ y[W + c] when RES), y = the row in LDS
template <int RB, int W, bool RES, int NW = 4>
__device__ __forceinline__ void ln_rows(const float *__restrict__ Ys, int lds, const float *__restrict__ gamma,
                                        const float *__restrict__ beta, float eps, float *__restrict__ Zs, int ldz,
                                        float *__restrict__ z, float2 *__restrict__ stats, int m0, int M, int wv,
                                        int lane) {
  constexpr int V = W / 64;
  for (int rr = wv; rr < RB; rr += NW) {
    const float *y = Ys + rr * lds;
    float v[V];
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = y[q * 64 + lane];
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) s += v[q];
    const float mean = wave_sum(s) / (float)W;
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const float d = v[q] - mean;
      ss = fmaf(d, d, ss);
    }
    const float rstd = 1.0f / sqrt_rn_f32(wave_sum(ss) / (float)W + eps);
    const bool live = m0 + rr < M;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int c = q * 64 + lane;
      float o = fmaxf(fmaf((v[q] - mean) * rstd, gamma[c], beta[c]), 0.f);
      if (RES) o += y[W + c];
      Zs[rr * ldz + c] = o;
      if (live) z[(size_t)(m0 + rr) * W + c] = o;
    }
    if (live && lane == 0) stats[m0 + rr] = make_float2(mean, rstd);
  }
}

// RB rows per workgroup (the launch uses 16), NW waves: every GEMM stage splits its output columns
// over the waves (a column's k order, hence its bits, do not depend on NW), the LayerNorm rows too.
// NW = 16: four waves per SIMD, so the waves' weight loads and LDS reads hide under each other's
// MFMAs (with 4, one wave per SIMD, every latency of the chain is exposed; 8: 52 vs 62 us for the
// P = 8 shard's forward; 16: rank step 0.438-0.440 vs 0.448 ms -- a rank's shard at P = 8 has 169
// workgroups for 256 CUs, one each).  The LayerNorm parameter partials are one row per wave.
constexpr int kTailWaves = 16;   // 16: 0.438 / 0.440 vs 0.448 ms per P = 8 rank step (profiles/r04k_sim_ab.txt)
// HEADS (the sharded aggregate-first GATConv, gat_xagg.hip): the tail's input rows are formed here
// from the two heads' aggregates, out^h = xa^h W_h^T + b^h (xa^h = x + h * xa_hs, row stride ldx; W_h
// = rows 256h .. of lin_l's weight Wh [512][512]), written as Y0 (pre-activation) and O = relu(Y0)
// (the tail's input, kept for the backward's weight gradients) -- the per-head GEMM launches and
// their slab sum leave the step.  Waves 0-3 take head 0's 256 columns, 4-7 head 1's.
// waves per SIMD pinned to one workgroup's (NW / 4): a shard's grid has at most one workgroup per
// CU, and without the pin the compiler schedules for the occupancy the LDS would admit (two
// workgroups, 64 VGPRs at NW = 16) and sinks every weight load next to its MFMAs -- the prefetch ring
// collapses to one group in flight
#define HICGAT_TAIL_WPE __attribute__((amdgpu_waves_per_eu(kTailWaves / 4, kTailWaves / 4)))
// PERSIST (the plain tail on grids of more than one round): one workgroup per CU walks the row tiles
// blockIdx, blockIdx + gridDim, ...; the next tile's x rows are copied into a third LDS buffer by
// LDS-DMA (global_load_lds) while this tile's LayerNorm / block 2 / block 3 run, so neither a tile's
// x load nor a workgroup's launch sits between two tiles' GEMMs.  Same arithmetic per row: bitwise
// the one-tile-per-workgroup grid.
#ifndef HICGAT_TAIL_PERSIST
#define HICGAT_TAIL_PERSIST 1
#endif
template <int RB, int NW, bool HEADS = false, bool PK = false, bool PERSIST = false>
__global__ __launch_bounds__(64 * NW) HICGAT_TAIL_WPE void tail_fwd_kernel(
    const float *__restrict__ x, int64_t ldx, int M, const float *__restrict__ W1c, const float *__restrict__ b1c,
    const float *__restrict__ g1, const float *__restrict__ be1, const float *__restrict__ W2c,
    const float *__restrict__ b2c, const float *__restrict__ g2, const float *__restrict__ be2,
    const float *__restrict__ W3, const float *__restrict__ b3, const float *__restrict__ g3,
    const float *__restrict__ be3, const float *__restrict__ W4, const float *__restrict__ b4, float eps,
    float *__restrict__ Y1, float2 *__restrict__ st1, float *__restrict__ z1, float *__restrict__ Y2,
    float2 *__restrict__ st2, float *__restrict__ z2, float *__restrict__ y3, float2 *__restrict__ st3,
    float *__restrict__ z3, float *__restrict__ coords, int64_t xa_hs = 0, const float *__restrict__ Wh = nullptr,
    const float *__restrict__ bh = nullptr, float *__restrict__ Y0 = nullptr, float *__restrict__ O = nullptr,
    int ntiles = 0) {
  extern __shared__ __attribute__((aligned(16))) float lds_tail[];
  float *As = lds_tail;              // x rows, then z1 / z2 / z3 rows
  float *Bs = lds_tail + RB * XS;    // Y1, then Y2 / y3 rows
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int H = RB / 16, NT1 = 32 / NW, NT2 = 16 / NW;   // 16-column tiles per wave: block 1 / block 2
  static_assert(NW == 4 || NW == 8 || NW == 16, "NW: 4, 8 or 16 waves");
  static_assert(!(PERSIST && HEADS), "the persistent form is the plain tail's");
  int tile = blockIdx.x;
  for (int it = 0;; ++it) {
  if constexpr (PERSIST) {
    if (tile >= ntiles) break;
    As = lds_tail + ((it & 1) ? 2 * RB * XS : 0);   // x / z rows alternate between two buffers
  }
  const int m0 = tile * RB;
  // the waves' column tiles rotated by the tile (consecutive workgroups of an XCD -- blockIdx
  // 8 apart -- start on different tiles): the CUs stream different weight rows at any moment instead
  // of all requesting the same L2 lines together.  Which wave computes a column does not change its
  // arithmetic (same k order): bitwise the unrotated kernel
  const int rot = (tile >> 3) & (NW - 1), ws = (wv + rot) & (NW - 1);
  if (!PERSIST || it == 0) {
    // x rows (HEADS: xa^0 rows -> As, xa^1 rows -> Bs) -> LDS (rows past M: zeros)
    for (int e = tid; e < (HEADS ? 2 : 1) * RB * 128; e += 64 * NW) {
      const int hd = e / (RB * 128), r = (e >> 7) % RB, c4 = e & 127;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m0 + r < M) v = reinterpret_cast<const float4 *>(x + hd * xa_hs + (size_t)(m0 + r) * ldx)[c4];
      *reinterpret_cast<float4 *>(&(hd ? Bs : As)[r * XS + 4 * c4]) = v;
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's copies of the tile's x rows landed
  }
  __syncthreads();
  if constexpr (HEADS) {
    static_assert(NW == 8 || NW == 16, "the head GEMMs take NW / 2 waves per head");
    constexpr int HW = NW / 2, NTH = 16 / HW;   // waves per head, 16-column tiles per wave
    const int hd = wv / HW, n0 = 16 * NTH * ((wv + rot) % HW);
    f32x4 acc[H][NTH];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < NTH; ++t) acc[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_rows<RB, NTH, 512, PK>(hd ? Bs : As, XS, Wh + (size_t)hd * 256 * 512, n0, acc, lane);
    __syncthreads();   // every wave is done with xa^0 / xa^1 before As takes relu(out)
    const int li = lane & 15, r0 = 4 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < NTH; ++t) {
      const int c = 256 * hd + n0 + 16 * t + li;
      const float bb = bh[c];
#pragma unroll
      for (int h = 0; h < H; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * h + r0 + r;
          const float v = acc[h][t][r] + bb, o = fmaxf(v, 0.f);
          As[row * XS + c] = o;
          if (m0 + row < M) {
            Y0[(size_t)(m0 + row) * 512 + c] = v;
            O[(size_t)(m0 + row) * 512 + c] = o;
          }
        }
    }
    __syncthreads();
  }
  // ---- block 1: 512 -> 512, wave wv: columns 16 NT1 wv .. + 16 NT1 - 1 ----
  {
    f32x4 acc[H][NT1];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < NT1; ++t) acc[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_rows<RB, NT1, 512, PK>(As, XS, W1c, 16 * NT1 * ws, acc, lane);
    store_tiles<RB, NT1>(acc, 16 * NT1 * ws, b1c, Bs, XS, Y1, 512, m0, M, lane);
  }
  if constexpr (PERSIST) {
    // the next tile's x rows into the other buffer (free: the previous tile ended at a barrier), one
    // 1 KB half row per LDS-DMA instruction; rows past M repeat row M - 1 (finite; never stored)
    const int mn = (tile + (int)gridDim.x) * RB;
    if (mn < M) {
      float *nb = lds_tail + ((it & 1) ? 0 : 2 * RB * XS);
      for (int r = wv; r < RB; r += NW)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const float *src = x + (size_t)min(mn + r, M - 1) * ldx + 256 * hf + 4 * lane;
          __builtin_amdgcn_global_load_lds(src, nb + r * XS + 256 * hf, 16, 0, 0);
        }
    }
  }
  __syncthreads();
  ln_rows<RB, 256, true, NW>(Bs, XS, g1, be1, eps, As, XS, z1, st1, m0, M, wv, lane);
  __syncthreads();
  // ---- block 2: 256 -> 256, wave wv: columns 16 NT2 wv .. ----
  {
    f32x4 acc[H][NT2];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < NT2; ++t) acc[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_rows<RB, NT2, 256, PK>(As, XS, W2c, 16 * NT2 * ws, acc, lane);
    store_tiles<RB, NT2>(acc, 16 * NT2 * ws, b2c, Bs, XS, Y2, 256, m0, M, lane);
  }
  __syncthreads();
  ln_rows<RB, 128, true, NW>(Bs, XS, g2, be2, eps, As, XS, z2, st2, m0, M, wv, lane);
  __syncthreads();
  // ---- block 3: 128 -> 64, waves 0..3: columns 16 wv .. 16 wv + 15 ----
  if (wv < 4) {
    f32x4 acc[H][1];
#pragma unroll
    for (int h = 0; h < H; ++h) acc[h][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_rows<RB, 1, 128>(As, XS, W3, 16 * ((wv + rot) & 3), acc, lane);
    store_tiles<RB, 1>(acc, 16 * ((wv + rot) & 3), b3, Bs, XS, y3, 64, m0, M, lane);
  }
  __syncthreads();
  ln_rows<RB, 64, false, NW>(Bs, XS, g3, be3, eps, As, XS, z3, st3, m0, M, wv, lane);
  __syncthreads();
  // ---- dense3: 64 -> 3, thread t < 3 RB: row t / 3, output t % 3 (fp32 fma chain over k) ----
  if (tid < RB * 3) {
    const int r = tid / 3, j = tid % 3;
    if (m0 + r < M) {
      const float *zr = As + r * XS;
      const float *w = W4 + j * 64;
      float s = 0.f;
#pragma unroll 16
      for (int k = 0; k < 64; ++k) s = fmaf(zr[k], w[k], s);
      coords[(size_t)(m0 + r) * 3 + j] = s + b4[j];
    }
  }
  if constexpr (!PERSIST) break;
  tile += gridDim.x;
  __syncthreads();   // every wave is done with this tile's LDS rows
  }
}

// ---- the tail's backward (the input-gradient chain) in one kernel ----------------------------------
// acc[h][t] += A[RB x K] (LDS) x B, B[k][n] = W[k][n] (W [K][ldw] row-major: dx = dy W): lane l reads
// W[16g + 4(l >> 4) + s][n0 + 16t + (l & 15)] -- 16 consecutive floats per k across the lanes -- with
// the weights of group g + 4 loaded after group g's MFMAs (ring of 4).
// PK: W is the packed copy (hicgat_tail_pack): lane l's four values of 16-row group g and column
// tile c (16 columns) are one float4 at ((g * (ldw / 16) + c) * 64 + l) * 4 -- 1 KB contiguous per
// load instead of four 4-B loads per lane over 4 rows; same values, bitwise the row-major form.
template <int RB, int NT, int K, bool PK = false>
__device__ __forceinline__ void mfma_rows_t(const float *__restrict__ As, int lda, const float *__restrict__ W, int ldw,
                                            int n0, f32x4 (&acc)[RB / 16][NT], int lane) {
  constexpr int G = K / 16, H = RB / 16, R = G < kTailRing ? G : kTailRing;
  static_assert(G % R == 0, "K: a multiple of 16 * ring depth");
  static_assert(R % 2 == 0, "the activation slots alternate with the group's parity");
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const float *wcol = W + (size_t)kq * ldw + n0 + li;
  const float *arow = As + li * lda + kq;
  float b[R][NT][4];
  // the four weights of lane l for 16-row group g and tile t (row-major or packed)
  auto wld = [&](float (&d)[4], int t, int g) {
    if constexpr (PK) {
      const float4 v = *reinterpret_cast<const float4 *>(W + (((size_t)g * (ldw / 16) + n0 / 16 + t) * 64 + lane) * 4);
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = wcol[(size_t)(16 * g + j) * ldw + 16 * t];
    }
  };
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int t = 0; t < NT; ++t) wld(b[q][t], t, q);
  float4 a[2][H];   // group g + 1's activations read before group g's MFMAs (as in mfma_rows)
#pragma unroll
  for (int h = 0; h < H; ++h) a[0][h] = *reinterpret_cast<const float4 *>(arow + h * 16 * lda);
  HICGAT_TAIL_SCHED();
  for (int g0 = 0; g0 < G; g0 += R) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int g = g0 + q, cur = q & 1;
      if (g + 1 < G) {
#pragma unroll
        for (int h = 0; h < H; ++h) a[cur ^ 1][h] = *reinterpret_cast<const float4 *>(arow + h * 16 * lda + 16 * (g + 1));
      }
      // k-step outer, tiles inner (as in mfma_rows)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int h = 0; h < H; ++h) acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h].x, b[q][t][0], acc[h][t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int h = 0; h < H; ++h) acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h].y, b[q][t][1], acc[h][t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int h = 0; h < H; ++h) acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h].z, b[q][t][2], acc[h][t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int h = 0; h < H; ++h) acc[h][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][h].w, b[q][t][3], acc[h][t], 0, 0, 0);
      if (g + R < G) {
#pragma unroll
        for (int t = 0; t < NT; ++t) wld(b[q][t], t, g + R);
      }
      HICGAT_TAIL_SCHED();
    }
  }
}

// acc -> LDS rows (no bias), and optionally the global output
template <int RB, int NT>
__device__ __forceinline__ void put_tiles(const f32x4 (&acc)[RB / 16][NT], int n0, float *__restrict__ Ls, int lds,
                                          float *__restrict__ out, int ldo, int m0, int M, int lane) {
  const int li = lane & 15, r0 = 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int c = n0 + 16 * t + li;
#pragma unroll
    for (int h = 0; h < RB / 16; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * h + r0 + r;
        if (Ls) Ls[row * lds + c] = acc[h][t][r];
        if (out && m0 + row < M) out[(size_t)(m0 + row) * ldo + c] = acc[h][t][r];
      }
  }
}

// LayerNorm + ReLU (+ residual) backward of rows wv, wv + 4, ... (ln_relu_res_bwd_kernel's
// arithmetic): dz from LDS (Dz, stride ldd), y / stats from global; dy (and dres = dz beside it when
// RES) into LDS (Gs, stride lds: [dy | dres]) and the global dY rows ([M][W or 2W]); the wave's
// dgamma / dbeta partials, summed over the workgroup's waves, into row ``slot`` of part ([slots][2][W],
// hicgat_ln_relu_res_bwd_params).
template <int RB, int W, bool RES, int NW = 4>
__device__ __forceinline__ void ln_bwd_rows(const float *__restrict__ Dz, int ldd, const float *__restrict__ y,
                                            int64_t ldy, const float2 *__restrict__ stats,
                                            const float *__restrict__ gamma, const float *__restrict__ beta,
                                            float *__restrict__ Gs, int lds, float *__restrict__ dY,
                                            float *__restrict__ part, int slot, float *__restrict__ red, int m0,
                                            int M, int wv, int lane) {
  constexpr int V = W / 64, LDY = RES ? 2 * W : W;
  float g_[V], b_[V], pg[V], pb[V];
#pragma unroll
  for (int q = 0; q < V; ++q) {
    g_[q] = gamma[q * 64 + lane];
    b_[q] = beta[q * 64 + lane];
    pg[q] = pb[q] = 0.f;
  }
  for (int rr = wv; rr < RB; rr += NW) {
    const int row = m0 + rr;
    const bool live = row < M;
    const float2 st = live ? stats[row] : make_float2(0.f, 0.f);
    float yh[V], dh[V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int c = q * 64 + lane;
      yh[q] = live ? (y[(size_t)row * ldy + c] - st.x) * st.y : 0.f;
      const float pre = fmaf(yh[q], g_[q], b_[q]);
      const float dzv = live ? Dz[rr * ldd + c] : 0.f;
      if (RES) {
        Gs[rr * lds + W + c] = dzv;
        if (live) dY[(size_t)row * LDY + W + c] = dzv;
      }
      const float g = pre > 0.f ? dzv : 0.f;
      pg[q] = fmaf(g, yh[q], pg[q]);
      pb[q] += g;
      dh[q] = g * g_[q];
      s1 += dh[q];
      s2 = fmaf(dh[q], yh[q], s2);
    }
    const float m1 = wave_sum(s1) / (float)W, m2 = wave_sum(s2) / (float)W;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const float v = st.y * (dh[q] - m1 - yh[q] * m2);
      Gs[rr * lds + q * 64 + lane] = v;
      if (live) dY[(size_t)row * LDY + q * 64 + lane] = v;
    }
  }
  // the NW waves' partials added in wave order through LDS (red: [NW][2W] floats), one [2W] row per
  // workgroup (slot = blockIdx.x): at 16 waves a wave holds one row, and per-wave rows would double the
  // grouped column sum's input
#pragma unroll
  for (int q = 0; q < V; ++q) {
    red[(wv * 2 + 0) * W + q * 64 + lane] = pg[q];
    red[(wv * 2 + 1) * W + q * 64 + lane] = pb[q];
  }
  __syncthreads();
  for (int c = wv * 64 + lane; c < 2 * W; c += NW * 64) {
    float v = red[c];
    for (int w = 1; w < NW; ++w) v += red[w * 2 * W + c];
    part[(size_t)slot * 2 * W + c] = v;
  }
  __syncthreads();   // red is reused by the next call
}


// HEADS: the GATConv's rows backward and its dxa GEMM after the chain (xagg_rows_bwd + the dxa
// grouped GEMM of gat_xagg.hip / gemm.hip): dx stays in LDS, dout = dx (Y0 > 0) (act) is written
// with delta^h = <dout^h, Y0^h - b^h> into row_stats[8r + 4 + h] (S3 moved to [6:8], as
// xagg_rows_bwd does), then dxa^h = dout^h W_h ([RB x 256] [256 x 512], waves 0-3 head 0, 4-7 head 1)
// into dxa [M][1024].
// ROWS (the single-GPU h-first GATConv, gat_fwd.hip's training form): the GATConv's gather-free
// rows backward (hicgat_gat_agg_bwd_rows, gat_bwd.hip) on the dx rows while they are in LDS -- dout
// = dx [y > 0] (act) or dx into dout, delta^h = <dout^h, y^h - b^h> and da_dst^h = <dout^h, out2^h>
// - delta^h S3^h into row_stats[8r + 4 .. 8r + 8), with the same arithmetic as agg_bwd_rows_kernel
// (bitwise) -- instead of writing dx for a separate pass that reads it back.  Y0 = y (the GATConv's
// relu output: the tail's input), bh = its bias, out2 = sum alpha lrelu' h; each wave's row of y /
// out2 is loaded at the kernel's start and held to the end.
template <int RB, int NW, bool HEADS = false, bool PK = false, bool ROWS = false>
__global__ __launch_bounds__(64 * NW) HICGAT_TAIL_WPE void tail_bwd_kernel(
    const float *__restrict__ dc, int M, const float *__restrict__ Y1, const float2 *__restrict__ st1,
    const float *__restrict__ Y2, const float2 *__restrict__ st2, const float *__restrict__ y3,
    const float2 *__restrict__ st3, const float *__restrict__ W4, const float *__restrict__ W3,
    const float *__restrict__ W2c, const float *__restrict__ W1c, const float *__restrict__ g1,
    const float *__restrict__ be1, const float *__restrict__ g2, const float *__restrict__ be2,
    const float *__restrict__ g3, const float *__restrict__ be3, float *__restrict__ dx, float *__restrict__ dY1,
    float *__restrict__ dY2, float *__restrict__ dy3, float *__restrict__ p1, float *__restrict__ p2,
    float *__restrict__ p3, int act = 0, const float *__restrict__ Y0 = nullptr, const float *__restrict__ Wh = nullptr,
    const float *__restrict__ bh = nullptr, float *__restrict__ dout = nullptr, float *__restrict__ row_stats = nullptr,
    float *__restrict__ dxa = nullptr, const float *__restrict__ out2 = nullptr) {
  static_assert(!(HEADS && ROWS), "one GATConv epilogue");
  static_assert(!ROWS || RB == NW, "ROWS: one row per wave");
  extern __shared__ __attribute__((aligned(16))) float lds_tail[];
  float *As = lds_tail;              // dz3, dz2, dz1 rows
  float *Bs = lds_tail + RB * XS;    // dy3, [dy2 | dres2], [dy1 | dres1] rows
  float *Rs = lds_tail + 2 * RB * XS;   // [NW][2W] LayerNorm parameter partials (W <= 256)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int slot = blockIdx.x;
  const int m0 = blockIdx.x * RB;
  constexpr int H = RB / 16;
  const int rot = (blockIdx.x >> 3) & (NW - 1), ws = (wv + rot) & (NW - 1);   // as in tail_fwd_kernel
  float4 ry0, ry1, rq0, rq1;   // ROWS: the wave's row of y and out2 (lane l: float4 l and 64 + l)
  if constexpr (ROWS) {
    const int row = m0 + wv;
    if (row < M) {
      const size_t o0 = (size_t)row * 128 + lane;
      ry0 = reinterpret_cast<const float4 *>(Y0)[o0];
      ry1 = reinterpret_cast<const float4 *>(Y0)[o0 + 64];
      rq0 = reinterpret_cast<const float4 *>(out2)[o0];
      rq1 = reinterpret_cast<const float4 *>(out2)[o0 + 64];
    }
  }
  // dense3 backward: dz3 = dc W4 ([RB x 3] [3 x 64]), fp32 fma chain over j
  for (int e = tid; e < RB * 64; e += 64 * NW) {
    const int r = e >> 6, c = e & 63;
    float s = 0.f;
    if (m0 + r < M) {
#pragma unroll
      for (int j = 0; j < 3; ++j) s = fmaf(dc[(size_t)(m0 + r) * 3 + j], W4[j * 64 + c], s);
    }
    As[r * XS + c] = s;
  }
  __syncthreads();
  ln_bwd_rows<RB, 64, false, NW>(As, XS, y3, 64, st3, g3, be3, Bs, XS, dy3, p3, slot, Rs, m0, M, wv, lane);
  __syncthreads();
  // dense2 backward: dz2 = dy3 W3 ([RB x 64] [64 x 128]), wave wv: columns 16 ND wv ..
  constexpr int WD = NW < 8 ? NW : 8, ND = 8 / WD, NT2 = 16 / NW, NT1 = 32 / NW;   // dense2: WD waves
  if (wv < WD) {
    f32x4 acc[H][ND];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < ND; ++t) acc[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int wd = (wv + rot) % WD;
    mfma_rows_t<RB, ND, 64>(Bs, XS, W3, 128, 16 * ND * wd, acc, lane);
    put_tiles<RB, ND>(acc, 16 * ND * wd, As, XS, nullptr, 0, m0, M, lane);
  }
  __syncthreads();
  ln_bwd_rows<RB, 128, true, NW>(As, XS, Y2, 256, st2, g2, be2, Bs, XS, dY2, p2, slot, Rs, m0, M, wv, lane);
  __syncthreads();
  // block 2 backward: dz1 = [dy2 | dres2] [W_1; W_1al] ([RB x 256] [256 x 256]), wave wv: columns 16 NT2 wv ..
  {
    f32x4 acc[H][NT2];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < NT2; ++t) acc[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_rows_t<RB, NT2, 256, PK>(Bs, XS, W2c, 256, 16 * NT2 * ws, acc, lane);
    put_tiles<RB, NT2>(acc, 16 * NT2 * ws, As, XS, nullptr, 0, m0, M, lane);
  }
  __syncthreads();
  ln_bwd_rows<RB, 256, true, NW>(As, XS, Y1, 512, st1, g1, be1, Bs, XS, dY1, p1, slot, Rs, m0, M, wv, lane);
  __syncthreads();
  // block 1 backward: dx = [dy1 | dres1] [W_a; W_al] ([RB x 512] [512 x 512]), wave wv: columns 16 NT1 wv ..
  {
    f32x4 acc[H][NT1];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < NT1; ++t) acc[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_rows_t<RB, NT1, 512, PK>(Bs, XS, W1c, 512, 16 * NT1 * ws, acc, lane);
    put_tiles<RB, NT1>(acc, 16 * NT1 * ws, (HEADS || ROWS) ? As : nullptr, XS, (HEADS || ROWS) ? nullptr : dx, 512,
                       m0, M, lane);
  }
  if constexpr (ROWS) {
    __syncthreads();
    const int row = m0 + wv;
    if (row < M) {   // wave-uniform; agg_bwd_rows_kernel's arithmetic on the LDS dx row
      float4 d0 = *reinterpret_cast<const float4 *>(&As[wv * XS + 4 * lane]);
      float4 d1 = *reinterpret_cast<const float4 *>(&As[wv * XS + 256 + 4 * lane]);
      const float4 b0 = reinterpret_cast<const float4 *>(bh)[lane], b1 = reinterpret_cast<const float4 *>(bh)[64 + lane];
      if (act) {
        d0 = make_float4(ry0.x <= 0.f ? 0.f : d0.x, ry0.y <= 0.f ? 0.f : d0.y, ry0.z <= 0.f ? 0.f : d0.z,
                         ry0.w <= 0.f ? 0.f : d0.w);
        d1 = make_float4(ry1.x <= 0.f ? 0.f : d1.x, ry1.y <= 0.f ? 0.f : d1.y, ry1.z <= 0.f ? 0.f : d1.z,
                         ry1.w <= 0.f ? 0.f : d1.w);
      }
      float4 *d4 = reinterpret_cast<float4 *>(dout) + (size_t)row * 128 + lane;
      d4[0] = d0;
      d4[64] = d1;
      const float4 e0 = make_float4(ry0.x - b0.x, ry0.y - b0.y, ry0.z - b0.z, ry0.w - b0.w);
      const float4 e1 = make_float4(ry1.x - b1.x, ry1.y - b1.y, ry1.z - b1.z, ry1.w - b1.w);
      float v[4] = {f4_dot(d0, e0), f4_dot(d1, e1), f4_dot(d0, rq0), f4_dot(d1, rq1)};
      transpose_reduce<4>(v, lane);
      const float dl0 = readlane_f(v[0], 0), dl1 = readlane_f(v[0], 16);
      const float q0 = readlane_f(v[0], 32), q1 = readlane_f(v[0], 48);
      if (lane == 0) {
        float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
        const float4 t = rs4[2 * (size_t)row + 1];   // (S3_0, S3_1, -, -) from the forward
        rs4[2 * (size_t)row + 1] = make_float4(dl0, dl1, fmaf(-dl0, t.x, q0), fmaf(-dl1, t.y, q1));
      }
    }
  }
  if constexpr (HEADS) {
    static_assert(NW == 8 || NW == 16, "the dxa GEMMs take NW / 2 waves per head");
    __syncthreads();
    // rows: lane l holds float4 l (head 0) and 64 + l (head 1) of the row, as xagg_rows_bwd_kernel
    for (int rr = wv; rr < RB; rr += NW) {
      const int row = m0 + rr;
      if (row >= M) {   // wave-uniform: zero rows of the A image
        *reinterpret_cast<float4 *>(&As[rr * XS + 4 * lane]) = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4 *>(&As[rr * XS + 256 + 4 * lane]) = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
      float4 d0 = *reinterpret_cast<const float4 *>(&As[rr * XS + 4 * lane]);
      float4 d1 = *reinterpret_cast<const float4 *>(&As[rr * XS + 256 + 4 * lane]);
      const float4 *y4 = reinterpret_cast<const float4 *>(Y0 + (size_t)row * 512);
      const float4 y0v = y4[lane], y1v = y4[64 + lane];
      const float4 b0 = reinterpret_cast<const float4 *>(bh)[lane], b1 = reinterpret_cast<const float4 *>(bh)[64 + lane];
      if (act) {
        d0 = make_float4(y0v.x <= 0.f ? 0.f : d0.x, y0v.y <= 0.f ? 0.f : d0.y, y0v.z <= 0.f ? 0.f : d0.z,
                         y0v.w <= 0.f ? 0.f : d0.w);
        d1 = make_float4(y1v.x <= 0.f ? 0.f : d1.x, y1v.y <= 0.f ? 0.f : d1.y, y1v.z <= 0.f ? 0.f : d1.z,
                         y1v.w <= 0.f ? 0.f : d1.w);
      }
      float4 *d4 = reinterpret_cast<float4 *>(dout + (size_t)row * 512);
      d4[lane] = d0;
      d4[64 + lane] = d1;
      *reinterpret_cast<float4 *>(&As[rr * XS + 4 * lane]) = d0;
      *reinterpret_cast<float4 *>(&As[rr * XS + 256 + 4 * lane]) = d1;
      const float4 e0 = make_float4(y0v.x - b0.x, y0v.y - b0.y, y0v.z - b0.z, y0v.w - b0.w);
      const float4 e1 = make_float4(y1v.x - b1.x, y1v.y - b1.y, y1v.z - b1.z, y1v.w - b1.w);
      float v[2] = {f4_dot(d0, e0), f4_dot(d1, e1)};
      transpose_reduce<2>(v, lane);   // lane 0: head 0, lane 32: head 1
      const float dl0 = readlane_f(v[0], 0), dl1 = readlane_f(v[0], 32);
      if (lane == 0) {
        float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
        const float4 t = rs4[2 * (size_t)row + 1];   // (S3_0, S3_1, -, -) from xagg_fwd
        rs4[2 * (size_t)row + 1] = make_float4(dl0, dl1, t.x, t.y);
      }
    }
    __syncthreads();
    constexpr int HW = NW / 2, NTX = 32 / HW;   // waves per head, 16-column tiles per wave
    const int hd = wv / HW, n0 = 16 * NTX * ((wv + rot) % HW);
    f32x4 acc[H][NTX];
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int t = 0; t < NTX; ++t) acc[h][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    mfma_rows_t<RB, NTX, 256, PK>(As + 256 * hd, XS, Wh + (size_t)hd * 256 * 512, 512, n0, acc, lane);
    put_tiles<RB, NTX>(acc, n0, nullptr, 0, dxa + 512 * hd, 1024, m0, M, lane);
  }
}

__global__ __launch_bounds__(256) void tail_pack_kernel(const PackJobs jobs) { pack_block(jobs, (int)blockIdx.x); }

// The step's first launch with the pack riding along: blocks [0, zb) are hicgat_step_begin's (zero the
// flat gradient, advance the device step count), the rest pack the tail's weights -- one launch
// fewer on the step's chain (the weights change only at the previous step's Adam).
__global__ __launch_bounds__(256) void step_pack_kernel(const PackJobs jobs, float *__restrict__ grad, int64_t n,
                                                        int64_t *__restrict__ step_ctr, int zb) {
  if ((int)blockIdx.x >= zb) {   // block-uniform
    pack_block(jobs, (int)blockIdx.x - zb);
    return;
  }
  if (step_ctr && blockIdx.x == 0 && threadIdx.x == 0) step_ctr[0] = step_ctr[0] + 1;
  const int64_t n4 = n / 4, stride = (int64_t)zb * 256;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) reinterpret_cast<float4 *>(grad)[i] = z;
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) grad[i] = 0.f;
}

}  // namespace hicgat

using namespace hicgat;

extern "C" size_t hicgat_tail_pack_bytes(void) { return (size_t)kPackTotal * sizeof(float); }

// What the last hicgat_tail_pack into each pack buffer wrote (host-side record): the head-fused
// forms read the Wh regions, which a pack made with Wh = NULL leaves unwritten -- they refuse such
// a pack (HICGAT_EINVAL) instead of reading uninitialised memory.
namespace {
std::mutex g_pack_mu;
std::unordered_map<const void *, bool> g_pack_heads;
}  // namespace
namespace hicgat {
void pack_note(const void *pack, bool heads) {
  std::lock_guard<std::mutex> lk(g_pack_mu);
  g_pack_heads[pack] = heads;
}
bool pack_has_heads(const void *pack) {
  std::lock_guard<std::mutex> lk(g_pack_mu);
  auto it = g_pack_heads.find(pack);
  return it != g_pack_heads.end() && it->second;
}

// the pack's job table (block ranges per weight and layout); returns the block count, or < 0 on error
int pack_jobs(const float *W1c, const float *W2c, const float *Wh, void *pack, size_t pack_bytes, PackJobs &pj) {
  if (!W1c || !W2c || !pack) return HICGAT_EINVAL;
  if (pack_bytes < hicgat_tail_pack_bytes()) return HICGAT_EINVAL;
  if (((uintptr_t)W1c | (uintptr_t)W2c | (uintptr_t)Wh | (uintptr_t)pack) & 15) return HICGAT_EUNSUPPORTED;
  float *pk = static_cast<float *>(pack);
  pj.n = 0;
  int blk = 0;
  auto add = [&](const float *src, int64_t off, int R, int C, int bwd) {
    PackJob &J = pj.j[pj.n++];
    J.src = src;
    J.dst = pk + off;
    J.R = R;
    J.C = C;
    J.bwd = bwd;
    J.blk0 = blk;
    const int units = bwd ? (R / 16) * (C / 16) : (R / 16) * (C / 32);   // one wave each, 4 per block
    blk += (units + 3) / 4;
  };
  add(W1c, kPackF1, 512, 512, 0);
  add(W2c, kPackF2, 256, 256, 0);
  if (Wh) add(Wh, kPackFH, 512, 512, 0);
  add(W1c, kPackB1, 512, 512, 1);
  add(W2c, kPackB2, 256, 256, 1);
  if (Wh) add(Wh, kPackBH, 512, 512, 1);
  return blk;
}
}  // namespace hicgat

extern "C" int hicgat_tail_pack(const float *W1c, const float *W2c, const float *Wh, void *pack, size_t pack_bytes,
                                hicgat_stream_t stream) {
  PackJobs pj;
  const int blk = pack_jobs(W1c, W2c, Wh, pack, pack_bytes, pj);
  if (blk < 0) return blk;
  hipLaunchKernelGGL(tail_pack_kernel, dim3(blk), dim3(256), 0, (hipStream_t)stream, pj);
  HICGAT_CHECK_LAUNCH();
  pack_note(pack, Wh != nullptr);
  return HICGAT_OK;
}

extern "C" int hicgat_step_begin_pack(float *grad, int64_t n, int64_t *step_counter, const float *W1c,
                                     const float *W2c, const float *Wh, void *pack, size_t pack_bytes,
                                     hicgat_stream_t stream) {
  if (n < 0 || (n > 0 && !grad)) return HICGAT_EINVAL;
  if (grad && (reinterpret_cast<uintptr_t>(grad) & 15)) return HICGAT_EINVAL;
  PackJobs pj;
  const int blk = pack_jobs(W1c, W2c, Wh, pack, pack_bytes, pj);
  if (blk < 0) return blk;
  const int zb = (int)std::max<int64_t>(1, std::min<int64_t>((n / 4 + 255) / 256, 1024));   // as hicgat_step_begin
  hipLaunchKernelGGL(step_pack_kernel, dim3(zb + blk), dim3(256), 0, (hipStream_t)stream, pj, grad, n, step_counter,
                     zb);
  HICGAT_CHECK_LAUNCH();
  pack_note(pack, Wh != nullptr);
  return HICGAT_OK;
}

namespace {
struct TailHeads {   // the HEADS operands of the head-fused forms (all null: the plain tail)
  const float *xa = nullptr;
  int64_t xa_hs = 0;
  const float *Wh = nullptr, *bh = nullptr;
  float *Y0 = nullptr, *O = nullptr;
};

template <bool HEADS, bool PK>
int tail_fwd_go(const float *x, int64_t ldx, int M, const float *W1c, const float *b1c, const float *g1,
                const float *be1, const float *W2c, const float *b2c, const float *g2, const float *be2, const float *W3,
                const float *b3, const float *g3, const float *be3, const float *W4, const float *b4, float eps,
                float *Y1, float *st1, float *z1, float *Y2, float *st2, float *z2, float *y3, float *st3, float *z3,
                float *coords, const float *Wh, const TailHeads &hh, hipStream_t stream) {
  // 16 rows per workgroup (66 KiB of dynamic LDS: two workgroups per CU).  A 32-row form (132 KiB,
  // one per CU, each weight fetch serving twice the rows) measured slower at N = 20000 (the one-kernel
  // tail 1.977 vs 1.913 ms per step for the per-layer kernels, profiles/r03r_ab_fused_tail.txt):
  // with one workgroup per CU every phase's latency is exposed.
  constexpr int RB = 16, NW = kTailWaves;
  const int ntiles = (M + RB - 1) / RB;
  if constexpr (!HEADS && HICGAT_TAIL_PERSIST) {
    static const int ncu = [] {
      int dev = 0, n = 0;
      return (hipGetDevice(&dev) == hipSuccess &&
              hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess) ? n : 0;
    }();
    if (ncu > 0 && ntiles > ncu) {   // more than one round of workgroups: one per CU walks the tiles
      static const bool pattr =
          hipFuncSetAttribute(reinterpret_cast<const void *>(&tail_fwd_kernel<RB, NW, false, PK, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 3 * RB * XS * (int)sizeof(float)) ==
          hipSuccess;
      if (!pattr) return HICGAT_ELAUNCH;
      hipLaunchKernelGGL((tail_fwd_kernel<RB, NW, false, PK, true>), dim3(ncu), dim3(64 * NW),
                         (size_t)3 * RB * XS * sizeof(float), stream, x, ldx, M, W1c, b1c, g1, be1, W2c, b2c, g2, be2,
                         W3, b3, g3, be3, W4, b4, eps, Y1, reinterpret_cast<float2 *>(st1), z1, Y2,
                         reinterpret_cast<float2 *>(st2), z2, y3, reinterpret_cast<float2 *>(st3), z3, coords,
                         (int64_t)0, nullptr, nullptr, nullptr, nullptr, ntiles);
      HICGAT_CHECK_LAUNCH();
      return HICGAT_OK;
    }
  }
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&tail_fwd_kernel<RB, NW, HEADS, PK>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               2 * RB * XS * (int)sizeof(float)) == hipSuccess;
  if (!attr) return HICGAT_ELAUNCH;
  hipLaunchKernelGGL((tail_fwd_kernel<RB, NW, HEADS, PK>), dim3(ntiles), dim3(64 * NW),
                     (size_t)2 * RB * XS * sizeof(float), stream, x, ldx, M, W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3,
                     b3, g3, be3, W4, b4, eps, Y1, reinterpret_cast<float2 *>(st1), z1, Y2,
                     reinterpret_cast<float2 *>(st2), z2, y3, reinterpret_cast<float2 *>(st3), z3, coords, hh.xa_hs,
                     Wh, hh.bh, hh.Y0, hh.O);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

template <bool HEADS>
int tail_fwd_launch(const float *x, int64_t ldx, int M, const float *W1c, const float *b1c, const float *g1,
                    const float *be1, const float *W2c, const float *b2c, const float *g2, const float *be2,
                    const float *W3, const float *b3, const float *g3, const float *be3, const float *W4,
                    const float *b4, float eps, float *Y1, float *st1, float *z1, float *Y2, float *st2, float *z2,
                    float *y3, float *st3, float *z3, float *coords, const TailHeads &hh, const void *pack,
                    hipStream_t stream) {
  if (M < 0 || ldx < 512 || (ldx & 3)) return HICGAT_EINVAL;
  if (M == 0) return HICGAT_OK;
  const void *ps[] = {x, W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4,
                      Y1, st1, z1, Y2, st2, z2, y3, st3, z3, coords};
  for (const void *p : ps)
    if (!p) return HICGAT_EINVAL;
  if (HEADS && (!hh.Wh || !hh.bh || !hh.Y0 || !hh.O || (hh.xa_hs & 3))) return HICGAT_EINVAL;
  // float4 rows: x, the weight rows and the LDS images need 16-B alignment
  if (((uintptr_t)x | (uintptr_t)W1c | (uintptr_t)W2c | (uintptr_t)W3 | (uintptr_t)hh.Wh | (uintptr_t)hh.Y0 |
       (uintptr_t)hh.O | (uintptr_t)pack) & 15)
    return HICGAT_EUNSUPPORTED;
  if (pack) {
    if (HEADS && !pack_has_heads(pack)) return HICGAT_EINVAL;   // packed without Wh
    const float *pk = static_cast<const float *>(pack);
    return tail_fwd_go<HEADS, true>(x, ldx, M, pk + kPackF1, b1c, g1, be1, pk + kPackF2, b2c, g2, be2, W3, b3, g3,
                                    be3, W4, b4, eps, Y1, st1, z1, Y2, st2, z2, y3, st3, z3, coords,
                                    HEADS ? pk + kPackFH : nullptr, hh, stream);
  }
  return tail_fwd_go<HEADS, false>(x, ldx, M, W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4, eps, Y1,
                                   st1, z1, Y2, st2, z2, y3, st3, z3, coords, hh.Wh, hh, stream);
}
}  // namespace

extern "C" int hicgat_tail_fwd_fused(const float *x, int64_t ldx, int M, const float *W1c, const float *b1c,
                                     const float *g1, const float *be1, const float *W2c, const float *b2c,
                                     const float *g2, const float *be2, const float *W3, const float *b3,
                                     const float *g3, const float *be3, const float *W4, const float *b4, float eps,
                                     float *Y1, float *st1, float *z1, float *Y2, float *st2, float *z2, float *y3,
                                     float *st3, float *z3, float *coords, const void *pack, hicgat_stream_t stream) {
  return tail_fwd_launch<false>(x, ldx, M, W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4, eps, Y1,
                                st1, z1, Y2, st2, z2, y3, st3, z3, coords, TailHeads{}, pack, (hipStream_t)stream);
}

extern "C" int hicgat_tail_fwd_fused_heads(const float *xa, int64_t ld_xa, int64_t xa_head_stride, const float *Wh,
                                           const float *bh, float *Y0, float *O, int M, const float *W1c,
                                           const float *b1c, const float *g1, const float *be1, const float *W2c,
                                           const float *b2c, const float *g2, const float *be2, const float *W3,
                                           const float *b3, const float *g3, const float *be3, const float *W4,
                                           const float *b4, float eps, float *Y1, float *st1, float *z1, float *Y2,
                                           float *st2, float *z2, float *y3, float *st3, float *z3, float *coords,
                                           const void *pack, hicgat_stream_t stream) {
  if (kTailWaves < 8) return HICGAT_EUNSUPPORTED;
  TailHeads hh;
  hh.xa = xa;
  hh.xa_hs = xa_head_stride;
  hh.Wh = Wh;
  hh.bh = bh;
  hh.Y0 = Y0;
  hh.O = O;
  return tail_fwd_launch<true>(xa, ld_xa, M, W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4, eps, Y1,
                               st1, z1, Y2, st2, z2, y3, st3, z3, coords, hh, pack, (hipStream_t)stream);
}

extern "C" int hicgat_tail_bwd_waves(void) { return kTailWaves; }

extern "C" size_t hicgat_tail_bwd_workspace_bytes(int M, int W) {
  return M <= 0 ? 16 : (size_t)((M + 15) / 16) * 2 * W * sizeof(float);   // one [2W] row per workgroup
}

namespace {
struct TailHeadsBwd {   // the HEADS / ROWS operands of the backward (all null: the plain tail)
  int act = 0;
  const float *Y0 = nullptr, *Wh = nullptr, *bh = nullptr, *out2 = nullptr;
  float *dout = nullptr, *row_stats = nullptr, *dxa = nullptr;
};

template <bool HEADS, bool PK, bool ROWS = false>
int tail_bwd_go(const float *dcoords, int M, const float *Y1, const float *st1, const float *Y2, const float *st2,
                const float *y3, const float *st3, const float *W4, const float *W3, const float *W2c, const float *W1c,
                const float *g1, const float *be1, const float *g2, const float *be2, const float *g3,
                const float *be3, float *dx, float *dY1, float *dY2, float *dy3, void *ws1, void *ws2, void *ws3,
                const float *Wh, const TailHeadsBwd &hh, hipStream_t stream) {
  constexpr int RB = 16, NW = kTailWaves;
  // [As | Bs] row images + the [NW][2 x 256] LayerNorm partial scratch
  constexpr int kBwdLds = (2 * RB * XS + NW * 2 * 256) * (int)sizeof(float);
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&tail_bwd_kernel<RB, NW, HEADS, PK, ROWS>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kBwdLds) == hipSuccess;
  if (!attr) return HICGAT_ELAUNCH;
  hipLaunchKernelGGL((tail_bwd_kernel<RB, NW, HEADS, PK, ROWS>), dim3((M + RB - 1) / RB), dim3(64 * NW),
                     (size_t)kBwdLds, stream, dcoords, M, Y1, reinterpret_cast<const float2 *>(st1),
                     Y2, reinterpret_cast<const float2 *>(st2), y3, reinterpret_cast<const float2 *>(st3), W4, W3, W2c,
                     W1c, g1, be1, g2, be2, g3, be3, dx, dY1, dY2, dy3, static_cast<float *>(ws1),
                     static_cast<float *>(ws2), static_cast<float *>(ws3), hh.act, hh.Y0, Wh, hh.bh, hh.dout,
                     hh.row_stats, hh.dxa, hh.out2);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

template <bool HEADS, bool ROWS = false>
int tail_bwd_launch(const float *dcoords, int M, const float *Y1, const float *st1, const float *Y2, const float *st2,
                    const float *y3, const float *st3, const float *W4, const float *W3, const float *W2c,
                    const float *W1c, const float *g1, const float *be1, const float *g2, const float *be2,
                    const float *g3, const float *be3, float *dx, float *dY1, float *dY2, float *dy3, void *ws1,
                    size_t ws1_bytes, void *ws2, size_t ws2_bytes, void *ws3, size_t ws3_bytes,
                    const TailHeadsBwd &hh, const void *pack, hipStream_t stream) {
  if (M < 0) return HICGAT_EINVAL;
  if (M == 0) return HICGAT_OK;
  const void *ps[] = {dcoords, Y1, st1, Y2, st2, y3, st3, W4, W3, W2c, W1c, g1, be1, g2, be2, g3, be3,
                      (HEADS || ROWS) ? hh.dout : dx, dY1, dY2, dy3, ws1, ws2, ws3};
  for (const void *p : ps)
    if (!p) return HICGAT_EINVAL;
  if (HEADS && (!hh.Y0 || !hh.Wh || !hh.bh || !hh.row_stats || !hh.dxa)) return HICGAT_EINVAL;
  if (ROWS && (!hh.Y0 || !hh.bh || !hh.out2 || !hh.row_stats)) return HICGAT_EINVAL;
  if ((HEADS || ROWS) &&
      (((uintptr_t)hh.Y0 | (uintptr_t)hh.bh | (uintptr_t)hh.dout | (uintptr_t)hh.row_stats | (uintptr_t)hh.out2) & 15))
    return HICGAT_EUNSUPPORTED;
  if ((uintptr_t)pack & 15) return HICGAT_EUNSUPPORTED;
  // every workgroup owns NW partial rows of each LN workspace (one per wave)
  if (ws1_bytes < hicgat_tail_bwd_workspace_bytes(M, 256) || ws2_bytes < hicgat_tail_bwd_workspace_bytes(M, 128) ||
      ws3_bytes < hicgat_tail_bwd_workspace_bytes(M, 64))
    return HICGAT_EINVAL;
  if (pack) {
    if (HEADS && !pack_has_heads(pack)) return HICGAT_EINVAL;   // packed without Wh
    const float *pk = static_cast<const float *>(pack);
    return tail_bwd_go<HEADS, true, ROWS>(dcoords, M, Y1, st1, Y2, st2, y3, st3, W4, W3, pk + kPackB2, pk + kPackB1,
                                          g1, be1, g2, be2, g3, be3, dx, dY1, dY2, dy3, ws1, ws2, ws3,
                                          HEADS ? pk + kPackBH : nullptr, hh, stream);
  }
  return tail_bwd_go<HEADS, false, ROWS>(dcoords, M, Y1, st1, Y2, st2, y3, st3, W4, W3, W2c, W1c, g1, be1, g2, be2, g3,
                                         be3, dx, dY1, dY2, dy3, ws1, ws2, ws3, hh.Wh, hh, stream);
}
}  // namespace

extern "C" int hicgat_tail_bwd_fused(const float *dcoords, int M, const float *Y1, const float *st1, const float *Y2,
                                     const float *st2, const float *y3, const float *st3, const float *W4,
                                     const float *W3, const float *W2c, const float *W1c, const float *g1,
                                     const float *be1, const float *g2, const float *be2, const float *g3,
                                     const float *be3, float *dx, float *dY1, float *dY2, float *dy3, void *ws1,
                                     size_t ws1_bytes, void *ws2, size_t ws2_bytes, void *ws3, size_t ws3_bytes,
                                     const void *pack, hicgat_stream_t stream) {
  return tail_bwd_launch<false>(dcoords, M, Y1, st1, Y2, st2, y3, st3, W4, W3, W2c, W1c, g1, be1, g2, be2, g3, be3,
                                dx, dY1, dY2, dy3, ws1, ws1_bytes, ws2, ws2_bytes, ws3, ws3_bytes, TailHeadsBwd{}, pack,
                                (hipStream_t)stream);
}

extern "C" int hicgat_tail_bwd_fused_rows(const float *dcoords, int M, const float *Y1, const float *st1,
                                          const float *Y2, const float *st2, const float *y3, const float *st3,
                                          const float *W4, const float *W3, const float *W2c, const float *W1c,
                                          const float *g1, const float *be1, const float *g2, const float *be2,
                                          const float *g3, const float *be3, float *dY1, float *dY2, float *dy3,
                                          void *ws1, size_t ws1_bytes, void *ws2, size_t ws2_bytes, void *ws3,
                                          size_t ws3_bytes, int act, const float *y, const float *out2,
                                          const float *bias, float *dout, float *row_stats, const void *pack,
                                          hicgat_stream_t stream) {
  if (kTailWaves != 16) return HICGAT_EUNSUPPORTED;   // one row per wave
  TailHeadsBwd hh;
  hh.act = act ? 1 : 0;
  hh.Y0 = y;
  hh.bh = bias;
  hh.out2 = out2;
  hh.dout = dout;
  hh.row_stats = row_stats;
  return tail_bwd_launch<false, true>(dcoords, M, Y1, st1, Y2, st2, y3, st3, W4, W3, W2c, W1c, g1, be1, g2, be2, g3,
                                      be3, nullptr, dY1, dY2, dy3, ws1, ws1_bytes, ws2, ws2_bytes, ws3, ws3_bytes, hh,
                                      pack, (hipStream_t)stream);
}

extern "C" int hicgat_tail_bwd_fused_heads(const float *dcoords, int M, const float *Y1, const float *st1,
                                           const float *Y2, const float *st2, const float *y3, const float *st3,
                                           const float *W4, const float *W3, const float *W2c, const float *W1c,
                                           const float *g1, const float *be1, const float *g2, const float *be2,
                                           const float *g3, const float *be3, float *dY1, float *dY2, float *dy3,
                                           void *ws1, size_t ws1_bytes, void *ws2, size_t ws2_bytes, void *ws3,
                                           size_t ws3_bytes, int act, const float *Y0, const float *Wh,
                                           const float *bh, float *dout, float *row_stats, float *dxa,
                                           const void *pack, hicgat_stream_t stream) {
  if (kTailWaves < 8) return HICGAT_EUNSUPPORTED;
  TailHeadsBwd hh;
  hh.act = act ? 1 : 0;
  hh.Y0 = Y0;
  hh.Wh = Wh;
  hh.bh = bh;
  hh.dout = dout;
  hh.row_stats = row_stats;
  hh.dxa = dxa;
  return tail_bwd_launch<true>(dcoords, M, Y1, st1, Y2, st2, y3, st3, W4, W3, W2c, W1c, g1, be1, g2, be2, g3, be3,
                               nullptr, dY1, dY2, dy3, ws1, ws1_bytes, ws2, ws2_bytes, ws3, ws3_bytes, hh, pack,
                               (hipStream_t)stream);
}
