// GATConv backward on gfx950 (autograd of a4+a5 in the reference: segment_csr/gather_csr/
// index_select/leaky_relu/exp backward of PyG 1.7.2), without float atomics.
//
// With out_i = sum_j alpha_ij h_j (+bias) and alpha the ptr-path softmax of
// e_ij = lrelu(a_src[j] + a_dst[i]):
//   g_ij   = <dout_i, h_j>                   (per head)
//   de_ij  = alpha_ij (g_ij - delta_i),      delta_i = sum_j alpha_ij g_ij
//   ds_ij  = de_ij * lrelu'(e_ij)
//   da_dst[i] = sum_j ds_ij,  da_src[j] = sum_i ds_ij,  dh_j = sum_i alpha_ij dout_i (+ logit terms)
// (the +1e-16 of the softmax denominator and the detached-max gradient change these by
// O(1e-16) relative; both are dropped.)
//
// Destination side, two forms with the same outputs (delta_i, da_dst_i into row_stats[i, 4:8]):
//  * agg_bwd_rows (the training path): no gather -- delta_i = <dout_i, out_i - bias> and
//    da_dst_i = <dout_i, out2_i> - delta_i S3_i from the forward's TRAIN outputs (gat_fwd.hip);
//  * agg_bwd_dst (stand-alone form, needs only h): gathers h_j and forms every g_ij; the per-edge
//    dot products are reduced 2U neighbour-heads at a time with one transpose reduce.
// Source side (row r) gathers dout_i of the rows that have r as a neighbour.  The graph is
// structurally symmetric (to_symmetric, utils.py:71), so row r's own CSR list *is* that set: the
// transpose needs no permutation array and no atomics.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"

// neighbours gathered per inner step of agg_bwd_dst (2 float4 loads per lane each).  Measured on
// MI355X at N = 20000 (tools/kbench.py): U = 8 -> 0.95 ms (118 VGPRs, 4 waves per SIMD); U = 4 ->
// 0.52; U = 2 -> 0.47.  With per-edge reductions in the loop the gather wants waves, not ILP.
constexpr int kBwdDstU = 2;
constexpr int kBwdSrcU = 4;   // neighbours per inner step of the (reduction-free) source pass

namespace hicgat {

// After transpose_reduce<2U> over values [head*U + k], lane l owns head l>>5 and slot k; the
// 64/(2U) lanes of a group hold the same sum and the first of them is the "owner".
template <int U> struct Owner {
  static constexpr int kShift = U == 8 ? 2 : U == 4 ? 3 : U == 2 ? 4 : 5;
  __device__ static int slot(int lane) { return (lane >> kShift) & (U - 1); }
  __device__ static bool owner(int lane) { return (lane & ((1 << kShift) - 1)) == 0; }
};

__global__ __launch_bounds__(256) void agg_bwd_dst_h2c256_kernel(
    const int *__restrict__ rowptr, const int *__restrict__ col, int row_begin, int row_end,
    const float *__restrict__ h, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    const float *__restrict__ dout, float ns, float *__restrict__ row_stats) {
  constexpr int U = kBwdDstU;
  const int lane = lane_id();
  const int i = row_begin + xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_in_block();
  if (i >= row_end) return;
  const int beg = rowptr[i], end = rowptr[i + 1];
  const float4 *h4 = reinterpret_cast<const float4 *>(h);
  const float4 *g4 = reinterpret_cast<const float4 *>(dout);
  const float4 d0 = g4[(size_t)i * 128 + lane], d1 = g4[(size_t)i * 128 + 64 + lane];
  const int hh = lane >> 5, kk = Owner<U>::slot(lane);
  const bool owner = Owner<U>::owner(lane);
  const float2 ad = *reinterpret_cast<const float2 *>(a_dst + 2 * (size_t)i);
  const float4 ms = reinterpret_cast<const float4 *>(row_stats)[2 * (size_t)i];  // max0 max1 sum0 sum1
  const float2 *as2 = reinterpret_cast<const float2 *>(a_src);
  float S1 = 0.f, S2 = 0.f, S3 = 0.f;
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    int j = i;
    // per-edge softmax weight and leaky-relu slope of this chunk, one edge per lane (the only
    // scattered loads of the row), later broadcast to the lane that owns each reduced dot product
    float al0 = 0.f, al1 = 0.f, alp0 = 0.f, alp1 = 0.f;
    if (e < end) {
      j = col[e];
      const float2 s = as2[j];
      const float e0 = s.x + ad.x, e1 = s.y + ad.y;
      al0 = expf(lrelu(e0, ns) - ms.x) / (ms.z + 1e-16f);
      al1 = expf(lrelu(e1, ns) - ms.y) / (ms.w + 1e-16f);
      alp0 = al0 * (e0 > 0.f ? 1.f : ns);
      alp1 = al1 * (e1 > 0.f ? 1.f : ns);
    }
    const int cnt = min(64, end - base);
    for (int k = 0; k < cnt; k += U) {
      float4 v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t jj = (size_t)readlane_i(j, k + u);
        v0[u] = h4[jj * 128 + lane];
        v1[u] = h4[jj * 128 + 64 + lane];
      }
      float v[2 * U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = f4_dot(d0, v0[u]);
        v[U + u] = f4_dot(d1, v1[u]);
      }
      transpose_reduce<2 * U>(v, lane);
      const int src = k + kk;
      const float a0 = __shfl(al0, src), a1 = __shfl(al1, src);
      const float p0 = __shfl(alp0, src), p1 = __shfl(alp1, src);
      const float al = hh ? a1 : a0, alp = hh ? p1 : p0;
      if (owner && src < cnt) {
        S1 = fmaf(al, v[0], S1);
        S2 = fmaf(alp, v[0], S2);
        S3 += alp;
      }
    }
  }
  S1 = half_wave_sum(S1);
  S2 = half_wave_sum(S2);
  S3 = half_wave_sum(S3);
  const float dl0 = readlane_f(S1, 0), dl1 = readlane_f(S1, 32);
  const float dd0 = readlane_f(S2 - S1 * S3, 0), dd1 = readlane_f(S2 - S1 * S3, 32);
  if (lane == 0) reinterpret_cast<float4 *>(row_stats)[2 * (size_t)i + 1] = make_float4(dl0, dl1, dd0, dd1);
}

// Source side, algebraically regrouped so that no per-edge dot product (and no cross-lane
// reduction) sits inside the gather loop:
//   da_src[r] = sum_i alpha_ir s_ir (<dout_i, h_r> - delta_i)
//             = <sum_i alpha_ir s_ir dout_i, h_r> - sum_i alpha_ir s_ir delta_i      (s = lrelu')
// so the loop only accumulates two vectors (sum alpha dout_i, sum alpha s dout_i) and a scalar.
// SPLIT (the tiled form, gat_tiles.hip): rowptr/col are the sparse remainder of the row's edges;
// dh gets the raw sum (no logit terms) and da_src the remainder's share of da_src; the matrix-core
// pass over the dense tiles adds the rest and finishes both.
template <bool SPLIT = false>
__device__ __forceinline__ void agg_bwd_src_row(
    int r, const int *__restrict__ rowptr, const int *__restrict__ col,
    const float *__restrict__ h, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    const float *__restrict__ row_stats, int64_t ldr, const float *__restrict__ dout, int64_t ldq,
    const float *__restrict__ att_s, const float *__restrict__ att_d, float ns,
    float *__restrict__ dh, float *__restrict__ da_src);

// One workgroup per 4 rows (a persistent grid of 2-3 workgroups per CU, leaving slots to the side
// stream's GEMMs, measured the same step or slower and was removed).
// REMAP: the XCD-aware block order (each XCD a contiguous row range: the rows of a banded Hi-C
// neighbourhood share that XCD's L2).  Off (plain round-robin over the XCDs) for the multi-GPU "slab"
// pass, whose heavy rows -- the rank's own diagonal block -- are contiguous: under the remap they
// would all land on one XCD.
template <bool SPLIT = false, bool REMAP = true>
__global__ __launch_bounds__(256) void agg_bwd_src_h2c256_kernel(
    const int *__restrict__ rowptr, const int *__restrict__ col, int row_begin, int row_end,
    const float *__restrict__ h, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    const float *__restrict__ row_stats, int64_t ldr, const float *__restrict__ dout, int64_t ldq,
    const float *__restrict__ att_s, const float *__restrict__ att_d, float ns,
    float *__restrict__ dh, float *__restrict__ da_src) {
  const int r = row_begin + (REMAP ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x) * 4 + wave_in_block();
  if (r < row_end)
    agg_bwd_src_row<SPLIT>(r, rowptr, col, h, a_src, a_dst, row_stats, ldr, dout, ldq, att_s, att_d, ns, dh, da_src);
}

template <bool SPLIT>
__device__ __forceinline__ void agg_bwd_src_row(
    int r, const int *__restrict__ rowptr, const int *__restrict__ col,
    const float *__restrict__ h, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    const float *__restrict__ row_stats, int64_t ldr, const float *__restrict__ dout, int64_t ldq,
    const float *__restrict__ att_s, const float *__restrict__ att_d, float ns,
    float *__restrict__ dh, float *__restrict__ da_src) {
  // ldq: dout row stride in float4, ldr: row_stats row stride in floats (both multiples of 4, so
  // a multi-GPU caller can all-gather [dout | row stats] rows as one packed buffer)
  constexpr int U = kBwdSrcU;
  const int lane = lane_id();
  const int beg = rowptr[r], end = rowptr[r + 1];
  const float4 *h4 = reinterpret_cast<const float4 *>(h);
  const float4 *g4 = reinterpret_cast<const float4 *>(dout);
  const float2 asr = *reinterpret_cast<const float2 *>(a_src + 2 * (size_t)r);
  const float2 *ad2 = reinterpret_cast<const float2 *>(a_dst);
  const float4 *rs4 = reinterpret_cast<const float4 *>(row_stats);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc0 = z4, acc1 = z4, c0 = z4, c1 = z4;
  float sb0 = 0.f, sb1 = 0.f;
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    int inb = r;
    float al0 = 0.f, al1 = 0.f, A0 = 0.f, A1 = 0.f;
    if (e < end) {
      inb = col[e];
      const float2 ad = ad2[inb];
      const float4 ms = rs4[(size_t)inb * (ldr / 4)];                         // max0 max1 sum0 sum1
      const float2 dl = *reinterpret_cast<const float2 *>(row_stats + ldr * inb + 4);       // delta
      const float e0 = asr.x + ad.x, e1 = asr.y + ad.y;
      al0 = expf(lrelu(e0, ns) - ms.x) / (ms.z + 1e-16f);
      al1 = expf(lrelu(e1, ns) - ms.y) / (ms.w + 1e-16f);
      A0 = al0 * (e0 > 0.f ? 1.f : ns);
      A1 = al1 * (e1 > 0.f ? 1.f : ns);
      sb0 = fmaf(A0, dl.x, sb0);
      sb1 = fmaf(A1, dl.y, sb1);
    }
    const int cnt = min(64, end - base);
    for (int k = 0; k < cnt; k += U) {
      float4 g0[U], g1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t ii = (size_t)readlane_i(inb, k + u);
        g0[u] = g4[ii * ldq + lane];
        g1[u] = g4[ii * ldq + 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc0 = f4_fma(readlane_f(al0, k + u), g0[u], acc0);
        acc1 = f4_fma(readlane_f(al1, k + u), g1[u], acc1);
        c0 = f4_fma(readlane_f(A0, k + u), g0[u], c0);
        c1 = f4_fma(readlane_f(A1, k + u), g1[u], c1);
      }
    }
  }
  const float4 hr0 = h4[(size_t)r * 128 + lane], hr1 = h4[(size_t)r * 128 + 64 + lane];
  float v[4] = {f4_dot(c0, hr0), f4_dot(c1, hr1), sb0, sb1};
  transpose_reduce<4>(v, lane);   // lane 0: v0, 16: v1, 32: v2, 48: v3 (summed over the wave)
  const float ds0 = readlane_f(v[0], 0) - readlane_f(v[0], 32);
  const float ds1 = readlane_f(v[0], 16) - readlane_f(v[0], 48);
  float4 *o4 = reinterpret_cast<float4 *>(dh);
  if (SPLIT) {
    o4[(size_t)r * 128 + lane] = acc0;
    o4[(size_t)r * 128 + 64 + lane] = acc1;
    if (lane == 0) *reinterpret_cast<float2 *>(da_src + 2 * (size_t)r) = make_float2(ds0, ds1);
    return;
  }
  const float2 dd = *reinterpret_cast<const float2 *>(row_stats + ldr * r + 6);
  const float4 *s4 = reinterpret_cast<const float4 *>(att_s);
  const float4 *t4 = reinterpret_cast<const float4 *>(att_d);
  const float4 as0 = s4[lane], as1 = s4[64 + lane], at0 = t4[lane], at1 = t4[64 + lane];
  acc0 = f4_fma(ds0, as0, acc0);
  acc0 = f4_fma(dd.x, at0, acc0);
  acc1 = f4_fma(ds1, as1, acc1);
  acc1 = f4_fma(dd.y, at1, acc1);
  o4[(size_t)r * 128 + lane] = acc0;
  o4[(size_t)r * 128 + 64 + lane] = acc1;
  if (lane == 0) {
    da_src[2 * (size_t)r] = ds0;
    da_src[2 * (size_t)r + 1] = ds1;
  }
}

// Destination side without a gather (the forward's TRAIN outputs, gat_fwd.hip):
//   dout_i = g_i * [y_i > 0] (ACT = 1: the relu after the GATConv, torch's threshold_backward on
//   its output) or g_i (ACT = 0);  delta_i = <dout_i, y_i - bias> (y = out where the mask is on);
//   da_dst_i = <dout_i, out2_i> - delta_i * S3_i.   One wave per row, 8 KB streamed per row.
template <int ACT>
__global__ __launch_bounds__(256) void agg_bwd_rows_kernel(int row_begin, int row_end,
                                                           const float *__restrict__ g,
                                                           const float *__restrict__ y,
                                                           const float *__restrict__ bias,
                                                           const float *__restrict__ out2,
                                                           float *__restrict__ dout, int64_t ldq,
                                                           float *__restrict__ row_stats) {
  const int lane = lane_id();
  const int i = row_begin + blockIdx.x * 4 + wave_in_block();
  if (i >= row_end) return;
  const size_t o0 = (size_t)i * 128 + lane, o1 = o0 + 64;
  const float4 *g4 = reinterpret_cast<const float4 *>(g);
  const float4 *y4 = reinterpret_cast<const float4 *>(y);
  const float4 *q4 = reinterpret_cast<const float4 *>(out2);
  const float4 *b4 = reinterpret_cast<const float4 *>(bias);
  float4 d0 = g4[o0], d1 = g4[o1];
  const float4 y0 = y4[o0], y1 = y4[o1], q0 = q4[o0], q1 = q4[o1];
  const float4 b0 = b4[lane], b1 = b4[64 + lane];
  if (ACT == 1) {
    d0 = make_float4(y0.x <= 0.f ? 0.f : d0.x, y0.y <= 0.f ? 0.f : d0.y, y0.z <= 0.f ? 0.f : d0.z,
                     y0.w <= 0.f ? 0.f : d0.w);
    d1 = make_float4(y1.x <= 0.f ? 0.f : d1.x, y1.y <= 0.f ? 0.f : d1.y, y1.z <= 0.f ? 0.f : d1.z,
                     y1.w <= 0.f ? 0.f : d1.w);
    float4 *d4 = reinterpret_cast<float4 *>(dout) + (size_t)i * ldq + lane;   // ldq: row stride, float4
    d4[0] = d0;
    d4[64] = d1;
  }
  const float4 e0 = make_float4(y0.x - b0.x, y0.y - b0.y, y0.z - b0.z, y0.w - b0.w);
  const float4 e1 = make_float4(y1.x - b1.x, y1.y - b1.y, y1.z - b1.z, y1.w - b1.w);
  float v[4] = {f4_dot(d0, e0), f4_dot(d1, e1), f4_dot(d0, q0), f4_dot(d1, q1)};
  transpose_reduce<4>(v, lane);
  const float dl0 = readlane_f(v[0], 0), dl1 = readlane_f(v[0], 16);
  const float p0 = readlane_f(v[0], 32), p1 = readlane_f(v[0], 48);
  if (lane == 0) {
    float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
    const float4 t = rs4[2 * (size_t)i + 1];   // (S3_0, S3_1, -, -) from the forward
    rs4[2 * (size_t)i + 1] = make_float4(dl0, dl1, fmaf(-dl0, t.x, p0), fmaf(-dl1, t.y, p1));
  }
}

// ---- GATConv parameter gradients: deterministic two-stage column reductions over N rows. ------
// Three parts: datt_src (sum_n da_src[n,h] h[n,:]), datt_dst (sum_n da_dst[n,h] h[n,:]) and dbias
// (sum_n dout[n,:]); any subset may be asked for (PARTS bit 0 / 1 / 2), so datt_dst and dbias --
// known after the gather-free row pass -- can be summed beside the source-side gather and only
// datt_src is left behind it.  Each part's sum runs in the same order whatever subset is asked for
// (bitwise the all-parts call).
// stage 1: block b sums rows [b*R, (b+1)*R) into part[b][P][D] (the P asked-for parts in order);
// stage 2: one thread per output column sums the partials in block order.
// row blocks of stage 1 (128 left half the CUs idle; 1024 measured slower: stage 2 sums twice the partials)
constexpr int kParamBlocks = 512;

template <int PARTS>
__global__ __launch_bounds__(256) void param_grad_stage1(const float *__restrict__ h,
                                                         const float *__restrict__ dout,
                                                         const float *__restrict__ da_src,
                                                         const float *__restrict__ row_stats, int N,
                                                         int H, int C, int rows_per_block,
                                                         float *__restrict__ part) {
  constexpr bool kS = PARTS & 1, kT = PARTS & 2, kB = PARTS & 4;
  constexpr int P = (int)kS + (int)kT + (int)kB;
  const int D = H * C, Q = D / 4;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(N, r0 + rows_per_block);
  const float4 *h4 = reinterpret_cast<const float4 *>(h);
  const float4 *g4 = reinterpret_cast<const float4 *>(dout);
  float4 *p4 = reinterpret_cast<float4 *>(part + (size_t)blockIdx.x * P * D);
  for (int q = threadIdx.x; q < Q; q += blockDim.x) {
    const int hd = (4 * q) / C;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), t = s, b = s;
#pragma unroll 4   // several rows' loads in flight per thread (one wave per SIMD at this grid size)
    for (int n = r0; n < r1; ++n) {
      if (kS || kT) {
        const float4 hv = h4[(size_t)n * Q + q];
        if (kS) s = f4_fma(da_src[(size_t)n * H + hd], hv, s);
        if (kT) t = f4_fma(row_stats[(size_t)n * 4 * H + 3 * H + hd], hv, t);
      }
      if (kB) {
        const float4 gv = g4[(size_t)n * Q + q];
        b.x += gv.x; b.y += gv.y; b.z += gv.z; b.w += gv.w;
      }
    }
    int o = 0;
    if (kS) p4[(o++) * Q + q] = s;
    if (kT) p4[(o++) * Q + q] = t;
    if (kB) p4[o * Q + q] = b;
  }
}

// block = 16 output columns x 16 groups (256 threads); group g adds partials b = g, g+16, ...;
// the groups are combined in order through LDS (fixed order: bitwise reproducible).  The partial
// range is cut 16 ways to keep each thread's chain of dependent loads short (32 partials at
// nblk = 512); 256-thread blocks (P*D/16 of them) find room on CUs that the side stream's GEMMs
// occupy, where 1024-thread blocks waited (25-43 us in the step instead of a few).
constexpr int kPG2Groups = 16, kPG2Cols = 16;
struct PGOut {
  float *o[3];
};
__global__ __launch_bounds__(256) void param_grad_stage2(const float *__restrict__ part, int nblk, int P, int D,
                                                         PGOut out, int accumulate) {
  __shared__ float red[kPG2Groups][kPG2Cols];
  const int cl = threadIdx.x % kPG2Cols, grp = threadIdx.x / kPG2Cols;
  const int c = blockIdx.x * kPG2Cols + cl;
  float s = 0.f;
  if (c < P * D) {
    // all of this thread's partials (<= kParamBlocks / 16 = 32) in flight together, then added in order
    constexpr int kMax = (kParamBlocks + kPG2Groups - 1) / kPG2Groups;
    float v[kMax];
#pragma unroll
    for (int i = 0; i < kMax; ++i) {
      const int b = grp + i * kPG2Groups;
      v[i] = b < nblk ? part[(size_t)b * P * D + c] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kMax; ++i) s += v[i];
  }
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && c < P * D) {
    float t = red[0][cl];
#pragma unroll
    for (int g = 1; g < kPG2Groups; ++g) t += red[g][cl];
    float *o = out.o[c / D] + c % D;
    *o = t + (accumulate ? *o : 0.f);
  }
}

// Unused dynamic LDS per workgroup of the whole-graph source pass (hicgat_gat_agg_bwd_src): 5
// workgroups per CU (the 160 KiB / 32 KiB) instead of the 7 its 68 VGPRs allow -- fewer rows in
// flight per CU (L2 misses), and the side stream's dW kernels wait for the pass instead of sharing
// its CUs: single-GPU step -8 us alone, -20 us with the forward gather's cap (gat_fwd.hip; 3 per CU:
// even, 6 per CU: even), profiles/r05at_gather_occupancy_ab.txt
constexpr size_t kSrcOccLds = 32768;

// Grid of the source pass: one workgroup per 4 rows.  (A persistent grid of 2-3 workgroups per CU,
// leaving slots to the side stream's GEMMs, measured the same step or slower)
#define HICGAT_SRC_LAUNCH(SPLIT_, rows_, ...)                                                              \
  hipLaunchKernelGGL((agg_bwd_src_h2c256_kernel<SPLIT_>), dim3(((rows_) + 3) / 4), dim3(256), 0,           \
                     __VA_ARGS__)

// The gather half of hicgat_gat_agg_bwd_src_tiled (gat_tiles.hip): the sparse remainder's shares.
int agg_bwd_src_split_launch(const int *rowptr_s, const int *col_s, int row_begin, int row_end, const float *h,
                             const float *a_src, const float *a_dst, const float *row_stats, int64_t ldr,
                             const float *dout, int64_t ldq4, float ns, float *dh, float *da_src, hipStream_t s) {
  HICGAT_SRC_LAUNCH(true, row_end - row_begin, s, rowptr_s,
                     col_s, row_begin, row_end, h, a_src, a_dst, row_stats, ldr, dout, ldq4, nullptr, nullptr, ns, dh,
                     da_src);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_gat_agg_bwd_dst(const int32_t *rowptr, const int32_t *col, int N, int H,
                                      int C, int row_begin, int row_end, const float *h,
                                      const float *a_src, const float *a_dst, const float *dout,
                                      float neg_slope, float *row_stats, hicgat_stream_t stream) {
  if (N < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !h || !a_src || !a_dst || !dout || !row_stats) return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  hipLaunchKernelGGL(agg_bwd_dst_h2c256_kernel, dim3((rows + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, rowptr, col, row_begin, row_end, h, a_src, a_dst, dout,
                     neg_slope, row_stats);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_gat_agg_bwd_src_ld(const int32_t *rowptr, const int32_t *col, int N, int H,
                                         int C, int row_begin, int row_end, const float *h,
                                         const float *a_src, const float *a_dst,
                                         const float *row_stats, int64_t ld_stats, const float *dout,
                                         int64_t ld_dout, const float *att_src, const float *att_dst,
                                         float neg_slope, float *dh, float *da_src,
                                         hicgat_stream_t stream) {
  if (N < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (ld_stats < 4 * H || ld_stats % 4 || ld_dout < H * C || ld_dout % 4) return HICGAT_EINVAL;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !h || !a_src || !a_dst || !row_stats || !dout || !att_src || !att_dst ||
      !dh || !da_src)
    return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  hipLaunchKernelGGL((agg_bwd_src_h2c256_kernel<false>), dim3((rows + 3) / 4), dim3(256), kSrcOccLds,
                     (hipStream_t)stream, rowptr, col, row_begin, row_end, h, a_src, a_dst,
                     row_stats, ld_stats, dout, ld_dout / 4, att_src, att_dst, neg_slope, dh, da_src);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_gat_agg_bwd_src_ex(const int32_t *rowptr, const int32_t *col, int N, int H,
                                         int C, int row_begin, int row_end, const float *h,
                                         const float *a_src, const float *a_dst,
                                         const float *row_stats, int64_t ld_stats, const float *dout,
                                         int64_t ld_dout, const float *att_src, const float *att_dst,
                                         float neg_slope, float *dh, float *da_src, int flags,
                                         hicgat_stream_t stream) {
  if (!(flags & HICGAT_SRC_ROUND_ROBIN))
    return hicgat_gat_agg_bwd_src_ld(rowptr, col, N, H, C, row_begin, row_end, h, a_src, a_dst, row_stats, ld_stats,
                                     dout, ld_dout, att_src, att_dst, neg_slope, dh, da_src, stream);
  if (flags & ~HICGAT_SRC_ROUND_ROBIN) return HICGAT_EINVAL;
  if (N < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (ld_stats < 4 * H || ld_stats % 4 || ld_dout < H * C || ld_dout % 4) return HICGAT_EINVAL;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !h || !a_src || !a_dst || !row_stats || !dout || !att_src || !att_dst ||
      !dh || !da_src)
    return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  hipLaunchKernelGGL((agg_bwd_src_h2c256_kernel<false, false>), dim3((rows + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, rowptr, col, row_begin, row_end, h, a_src, a_dst, row_stats, ld_stats, dout,
                     ld_dout / 4, att_src, att_dst, neg_slope, dh, da_src);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_gat_agg_bwd_src(const int32_t *rowptr, const int32_t *col, int N, int H,
                                      int C, int row_begin, int row_end, const float *h,
                                      const float *a_src, const float *a_dst,
                                      const float *row_stats, const float *dout,
                                      const float *att_src, const float *att_dst,
                                      float neg_slope, float *dh, float *da_src,
                                      hicgat_stream_t stream) {
  return hicgat_gat_agg_bwd_src_ld(rowptr, col, N, H, C, row_begin, row_end, h, a_src, a_dst,
                                   row_stats, 4 * (int64_t)H, dout, (int64_t)H * C, att_src, att_dst,
                                   neg_slope, dh, da_src, stream);
}

extern "C" int hicgat_gat_agg_bwd_rows(int N, int H, int C, int row_begin, int row_end, int act,
                                       const float *g, const float *y, const float *bias,
                                       const float *out2, float *dout, int64_t ld_dout,
                                       float *row_stats, hicgat_stream_t stream) {
  if (N < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (act && (ld_dout < (int64_t)H * C || ld_dout % 4)) return HICGAT_EINVAL;
  if (act != 0 && act != 1) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!g || !y || !bias || !out2 || !row_stats || (act && !dout)) return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  if (act)
    hipLaunchKernelGGL(agg_bwd_rows_kernel<1>, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       row_begin, row_end, g, y, bias, out2, dout, ld_dout / 4, row_stats);
  else
    hipLaunchKernelGGL(agg_bwd_rows_kernel<0>, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       row_begin, row_end, g, y, bias, out2, dout, (int64_t)0, row_stats);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" size_t hicgat_gat_param_grad_workspace_bytes(int N, int D) {
  (void)N;
  return (size_t)kParamBlocks * 3 * (size_t)(D > 0 ? D : 0) * sizeof(float);
}

extern "C" int hicgat_gat_param_grad(const float *h, const float *dout, const float *da_src,
                                     const float *row_stats, int N, int H, int C, float *datt_src,
                                     float *datt_dst, float *dbias, int accumulate, void *workspace,
                                     size_t workspace_bytes, hicgat_stream_t stream) {
  if (N < 0 || H <= 0 || C <= 0 || (C % 4) != 0) return HICGAT_EINVAL;
  const int D = H * C;
  const int parts = (datt_src ? 1 : 0) | (datt_dst ? 2 : 0) | (dbias ? 4 : 0);
  if (!parts || !workspace) return HICGAT_EINVAL;
  if (((parts & 3) && !h) || ((parts & 1) && !da_src) || ((parts & 2) && !row_stats) || ((parts & 4) && !dout))
    return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_gat_param_grad_workspace_bytes(N, D)) return HICGAT_EINVAL;
  const int rpb = N > 0 ? (N + kParamBlocks - 1) / kParamBlocks : 1;
  const int nblk = N > 0 ? (N + rpb - 1) / rpb : 0;
  float *part = static_cast<float *>(workspace);
  PGOut out{};
  int P = 0;
  if (datt_src) out.o[P++] = datt_src;
  if (datt_dst) out.o[P++] = datt_dst;
  if (dbias) out.o[P++] = dbias;
  hipStream_t s = (hipStream_t)stream;
  if (nblk > 0) {
#define HICGAT_PG1(PARTS_)                                                                                      \
  case PARTS_:                                                                                                  \
    hipLaunchKernelGGL(param_grad_stage1<PARTS_>, dim3(nblk), dim3(128), 0, s, h, dout, da_src, row_stats, N, H, \
                       C, rpb, part);                                                                           \
    break;
    switch (parts) {
      HICGAT_PG1(1) HICGAT_PG1(2) HICGAT_PG1(3) HICGAT_PG1(4) HICGAT_PG1(5) HICGAT_PG1(6) HICGAT_PG1(7)
    }
#undef HICGAT_PG1
    HICGAT_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(param_grad_stage2, dim3((P * D + kPG2Cols - 1) / kPG2Cols), dim3(kPG2Cols * kPG2Groups), 0, s,
                     part, nblk, P, D, out, accumulate);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
