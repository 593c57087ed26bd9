// Row-block GAT aggregation (a4+a5 and the source half of its backward) for gfx950.
//
// Reference: the same PyG 1.7.2 GATConv arithmetic as gat_fwd.hip / gat_bwd.hip (models.py:634-662):
//   out_i = sum_j alpha_ij h_j,  alpha_ij = softmax_j(leaky_relu(a_src[j] + a_dst[i]))
// and its source-side backward  dh_r = sum_i alpha_ir dout_i + ... (include/hicgat.h).
//
// Why a second form.  The row-per-wave kernels gather one 2 KiB neighbour row per edge; on the
// Hi-C graphs most edges lie near the diagonal (every |i-j| <= ~10 is a contact, the rest decays
// as 1/|i-j|), so consecutive destination rows share most of their near neighbours.  Here one
// workgroup owns R = 16 consecutive rows and walks the UNION of their neighbour lists ("runs":
// one source j plus a 16-bit mask of the block rows that have the edge (i, j)), loading each
// source row once and applying it to every masked row from registers.  At N = 20000 (1 %) that
// is 2.2 M row loads instead of 4.0 M (1.8x fewer bytes from L2 into the CUs, the measured
// ceiling of the row-per-wave form).
//
// Per step the edge weights are formed once, in CSR order, by a row pass (the softmax max / sum
// of gat_fwd.hip's passes 1-2, then alpha) and scattered into block order through the static
// permutation `pos` (graph.py BlockCSR).  A record is alpha as fp32 with the SIGN BIT carrying
// the leaky-relu branch: set when e <= 0, i.e. lrelu'(e) = negative_slope (alpha >= 0, so the
// bit is free); the gather reads w1 = |rec| and w2 = w1 * lrelu'(e) from it.
//
// Layout (R = 16): runs int64 = j | (mask << 32), sorted by (block, j); run_ptr [nblk + 1];
// within a block the records follow the runs, and inside a run the set mask bits in ascending
// row order; block b's records occupy the CSR positions of its own rows,
// [rowptr[row_begin + 16 b], rowptr[row_begin + 16 b + 16]).  Block b covers the rows
// row_begin + 16 b ... (a launch's row range is the block structure's row range).
//
// Workgroup = 4 waves; wave q owns columns [128 q, 128 q + 128) (head q / 2), lane l columns
// 128 q + 2 l, +1, so each run costs every wave one coalesced 512 B row segment, and the 16
// rows' accumulators (x2 for the second weight) live in 64 VGPRs per lane.
#include "common.hpp"

#ifndef HICGAT_BLK_U
#define HICGAT_BLK_U 8   // runs whose source rows are in flight per wave
#endif

namespace hicgat {

constexpr int kBlkRows = 16;

__device__ __forceinline__ float rec_pack(float a, float e) {
  return e > 0.f ? a : __int_as_float(__float_as_int(a) | (int)0x80000000);
}
__device__ __forceinline__ float2 f2_fma(float a, float2 x, float2 acc) {
  acc.x = fmaf(a, x.x, acc.x);
  acc.y = fmaf(a, x.y, acc.y);
  return acc;
}

// ---- forward row pass: softmax statistics (bit-identical to agg_fwd_h2c256_kernel's row_stats)
// and the records of every edge of the row, written at their block-order position.
template <bool TRAIN>
__global__ __launch_bounds__(256) void blk_fwd_rows_kernel(
    const int *__restrict__ rowptr, const int *__restrict__ col, const int *__restrict__ pos,
    int row_begin, int row_end, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    float ns, float2 *__restrict__ rec, float *__restrict__ row_stats) {
  const int lane = lane_id();
  const int i = row_begin + blockIdx.x * 4 + wave_in_block();
  if (i >= row_end) return;
  const int e0g = rowptr[row_begin];
  const int beg = rowptr[i], end = rowptr[i + 1];
  const float2 ad = *reinterpret_cast<const float2 *>(a_dst + 2 * (size_t)i);
  const float2 *as2 = reinterpret_cast<const float2 *>(a_src);
  float m0 = -INFINITY, m1 = -INFINITY;
  for (int e = beg + lane; e < end; e += 64) {
    const float2 s = as2[col[e]];
    m0 = fmaxf(m0, lrelu(s.x + ad.x, ns));
    m1 = fmaxf(m1, lrelu(s.y + ad.y, ns));
  }
  m0 = wave_max(m0);
  m1 = wave_max(m1);
  float s0 = 0.f, s1 = 0.f;
  for (int e = beg + lane; e < end; e += 64) {
    const float2 s = as2[col[e]];
    s0 += expf(lrelu(s.x + ad.x, ns) - m0);
    s1 += expf(lrelu(s.y + ad.y, ns) - m1);
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  const float den0 = s0 + 1e-16f, den1 = s1 + 1e-16f;
  float t0 = 0.f, t1 = 0.f;
  for (int e = beg + lane; e < end; e += 64) {
    const float2 s = as2[col[e]];
    const float x0 = s.x + ad.x, x1 = s.y + ad.y;
    const float p0 = expf(lrelu(x0, ns) - m0) / den0;
    const float p1 = expf(lrelu(x1, ns) - m1) / den1;
    if (TRAIN) {
      t0 += p0 * (x0 > 0.f ? 1.f : ns);
      t1 += p1 * (x1 > 0.f ? 1.f : ns);
    }
    rec[e0g + pos[e - e0g]] = make_float2(rec_pack(p0, x0), rec_pack(p1, x1));
  }
  float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
  if (TRAIN) {
    t0 = wave_sum(t0);
    t1 = wave_sum(t1);
    if (lane == 0) rs4[2 * (size_t)i + 1] = make_float4(t0, t1, 0.f, 0.f);
  }
  if (lane == 0) rs4[2 * (size_t)i] = make_float4(m0, m1, s0, s1);
}

// ---- backward row pass over SOURCE rows r: alpha_ir (the forward weight of edge (i, r); the
// graph is symmetric, so row r's list holds every such i), sb[r] = sum_i alpha_ir lrelu'(e_ir)
// delta_i, and the records.  Same per-edge arithmetic as agg_bwd_src_h2c256_kernel.
__global__ __launch_bounds__(256) void blk_bwd_rows_kernel(
    const int *__restrict__ rowptr, const int *__restrict__ col, const int *__restrict__ pos,
    int row_begin, int row_end, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    const float *__restrict__ row_stats, int64_t ldr, float ns, float2 *__restrict__ rec,
    float2 *__restrict__ sb) {
  const int lane = lane_id();
  const int r = row_begin + blockIdx.x * 4 + wave_in_block();
  if (r >= row_end) return;
  const int e0g = rowptr[row_begin];
  const int beg = rowptr[r], end = rowptr[r + 1];
  const float2 asr = *reinterpret_cast<const float2 *>(a_src + 2 * (size_t)r);
  const float2 *ad2 = reinterpret_cast<const float2 *>(a_dst);
  float sb0 = 0.f, sb1 = 0.f;
  for (int e = beg + lane; e < end; e += 64) {
    const int inb = col[e];
    const float2 ad = ad2[inb];
    const float4 ms = *reinterpret_cast<const float4 *>(row_stats + ldr * inb);   // max0 max1 sum0 sum1
    const float2 dl = *reinterpret_cast<const float2 *>(row_stats + ldr * inb + 4);  // delta
    const float x0 = asr.x + ad.x, x1 = asr.y + ad.y;
    const float al0 = expf(lrelu(x0, ns) - ms.x) / (ms.z + 1e-16f);
    const float al1 = expf(lrelu(x1, ns) - ms.y) / (ms.w + 1e-16f);
    sb0 = fmaf(al0 * (x0 > 0.f ? 1.f : ns), dl.x, sb0);
    sb1 = fmaf(al1 * (x1 > 0.f ? 1.f : ns), dl.y, sb1);
    rec[e0g + pos[e - e0g]] = make_float2(rec_pack(al0, x0), rec_pack(al1, x1));
  }
  sb0 = wave_sum(sb0);
  sb1 = wave_sum(sb1);
  if (lane == 0) sb[r] = make_float2(sb0, sb1);
}

// ---- the gather: MODE 0 forward with out2 (training), 1 forward only, 2 source-side backward.
// X = h (forward) or dout (backward), row stride ldx2 in float2.
template <int MODE, int ACT>
__global__ __launch_bounds__(256) void blk_gather_kernel(
    const int *__restrict__ rowptr, const long long *__restrict__ runs,
    const int *__restrict__ run_ptr, int row_begin, int row_end, const float *__restrict__ rec,
    const float2 *__restrict__ X, int64_t ldx2, float ns,
    const float2 *__restrict__ bias, float2 *__restrict__ out, float2 *__restrict__ out2,
    const float2 *__restrict__ h, const float2 *__restrict__ sb, const float *__restrict__ row_stats,
    int64_t ldr, const float2 *__restrict__ att_s, const float2 *__restrict__ att_d,
    float2 *__restrict__ dh, float *__restrict__ da_src) {
  constexpr int U = HICGAT_BLK_U;
  constexpr bool TWO = MODE != 1;
  const int lane = lane_id();
  const int q = wave_in_block();      // column quarter
  const int head = q >> 1;
  const int cofs = q * 64 + lane;     // float2 column of this lane
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = row_begin + b * kBlkRows;
  const int nr = min(kBlkRows, row_end - r0);
  int k = rowptr[r0];
  const int kend = rowptr[r0 + nr];
  const int u_beg = run_ptr[b], u_end = run_ptr[b + 1];

  float2 acc[kBlkRows], acc2[kBlkRows];
#pragma unroll
  for (int r = 0; r < kBlkRows; ++r) {
    acc[r] = make_float2(0.f, 0.f);
    acc2[r] = make_float2(0.f, 0.f);
  }
  // record window: lane l holds this head's weight of record kc + l; the next window is in flight
  int kc = k;
  float rw = (kc + lane < kend) ? rec[2 * (size_t)(kc + lane) + head] : 0.f;
  float rn = (kc + 64 + lane < kend) ? rec[2 * (size_t)(kc + 64 + lane) + head] : 0.f;

  for (int ub = u_beg; ub < u_end; ub += 64) {
    const long long w = (ub + lane < u_end) ? runs[ub + lane] : 0ll;   // padding: j = 0, mask 0
    const int jv = (int)(w & 0xffffffffll), mv = (int)(w >> 32);
    const int cnt = min(64, u_end - ub);
    for (int t = 0; t < cnt; t += U) {
      float2 v[U];
#pragma unroll
      for (int uu = 0; uu < U; ++uu) {
        const size_t jj = (size_t)readlane_i(jv, t + uu);
        v[uu] = X[jj * ldx2 + cofs];
      }
#pragma unroll
      for (int uu = 0; uu < U; ++uu) {
        const int m = readlane_i(mv, t + uu);
#pragma unroll
        for (int r = 0; r < kBlkRows; ++r) {
          if (m & (1 << r)) {
            if (k - kc >= 64) {
              kc += 64;
              rw = rn;
              rn = (kc + 64 + lane < kend) ? rec[2 * (size_t)(kc + 64 + lane) + head] : 0.f;
            }
            const float x = readlane_f(rw, k - kc);
            ++k;
            const float w1 = fabsf(x);
            acc[r] = f2_fma(w1, v[uu], acc[r]);
            if (TWO) {
              const float w2 = __float_as_int(x) < 0 ? w1 * ns : w1;
              acc2[r] = f2_fma(w2, v[uu], acc2[r]);
            }
          }
        }
      }
    }
  }

  if (MODE != 2) {
    const float2 bb = bias[cofs];
#pragma unroll
    for (int r = 0; r < kBlkRows; ++r) {
      if (r < nr) {
        const size_t i = (size_t)(r0 + r);
        float2 o = make_float2(acc[r].x + bb.x, acc[r].y + bb.y);
        if (ACT == 1) o = make_float2(relu_t(o.x), relu_t(o.y));
        out[i * 256 + cofs] = o;
        if (MODE == 0) out2[i * 256 + cofs] = acc2[r];
      }
    }
  } else {
    // ds_r = <acc2_r, h_r> over the head's 256 columns (two waves) - sb_r
    __shared__ float part[4][kBlkRows];
    float d[kBlkRows];
#pragma unroll
    for (int r = 0; r < kBlkRows; ++r) {
      const float2 hv = r < nr ? h[(size_t)(r0 + r) * 256 + cofs] : make_float2(0.f, 0.f);
      d[r] = fmaf(acc2[r].x, hv.x, acc2[r].y * hv.y);
    }
    transpose_reduce<16>(d, lane);
    if ((lane & 3) == 0) {
      const int idx = ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
      part[q][idx] = d[0];
    }
    __syncthreads();
    const float2 as = att_s[cofs], at = att_d[cofs];
#pragma unroll
    for (int r = 0; r < kBlkRows; ++r) {
      if (r < nr) {
        const size_t i = (size_t)(r0 + r);
        const float2 sbi = sb[i];
        const float ds = part[2 * head][r] + part[2 * head + 1][r] - (head ? sbi.y : sbi.x);
        const float dd = row_stats[ldr * i + 6 + head];
        float2 o = f2_fma(ds, as, acc[r]);
        o = f2_fma(dd, at, o);
        dh[i * 256 + cofs] = o;
        if ((q & 1) == 0 && lane == 0) da_src[2 * i + head] = ds;
      }
    }
  }
}

}  // namespace hicgat

using namespace hicgat;

extern "C" size_t hicgat_gat_blk_workspace_bytes(int N, int nnz) {
  if (N < 0 || nnz < 0) return 0;
  return (size_t)nnz * 8 + (size_t)N * 8 + 256;
}

extern "C" int hicgat_gat_blk_fwd(const int32_t *rowptr, const int32_t *col, const int32_t *pos,
                                  const int64_t *runs, const int32_t *run_ptr, int N, int nnz, int H,
                                  int C, int row_begin, int row_end, const float *h,
                                  const float *a_src, const float *a_dst, const float *bias,
                                  float neg_slope, int act, float *out, float *out2,
                                  float *row_stats, void *workspace, size_t workspace_bytes,
                                  hicgat_stream_t stream) {
  if (N < 0 || nnz < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (act != 0 && act != 1) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !pos || !runs || !run_ptr || !h || !a_src || !a_dst || !bias || !out ||
      !row_stats || !workspace)
    return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_gat_blk_workspace_bytes(N, nnz)) return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  const int nblk = (rows + kBlkRows - 1) / kBlkRows;
  hipStream_t s = (hipStream_t)stream;
  float2 *rec = reinterpret_cast<float2 *>(workspace);
  if (out2)
    hipLaunchKernelGGL((blk_fwd_rows_kernel<true>), dim3((rows + 3) / 4), dim3(256), 0, s, rowptr, col,
                       pos, row_begin, row_end, a_src, a_dst, neg_slope, rec, row_stats);
  else
    hipLaunchKernelGGL((blk_fwd_rows_kernel<false>), dim3((rows + 3) / 4), dim3(256), 0, s, rowptr,
                       col, pos, row_begin, row_end, a_src, a_dst, neg_slope, rec, row_stats);
  HICGAT_CHECK_LAUNCH();
  const float2 *X = reinterpret_cast<const float2 *>(h);
  const float2 *b2 = reinterpret_cast<const float2 *>(bias);
  float2 *o2 = reinterpret_cast<float2 *>(out), *q2 = reinterpret_cast<float2 *>(out2);
  const float *rf = reinterpret_cast<const float *>(rec);
#define HICGAT_BLK_FWD(MO, AC)                                                                      \
  hipLaunchKernelGGL((blk_gather_kernel<MO, AC>), dim3(nblk), dim3(256), 0, s, rowptr,                \
                     reinterpret_cast<const long long *>(runs), run_ptr, row_begin, row_end, rf, X,  \
                     (int64_t)256, neg_slope, b2, o2, q2, nullptr, nullptr, nullptr, (int64_t)0,     \
                     nullptr, nullptr, nullptr, nullptr)
  if (out2) {
    if (act) HICGAT_BLK_FWD(0, 1);
    else HICGAT_BLK_FWD(0, 0);
  } else {
    if (act) HICGAT_BLK_FWD(1, 1);
    else HICGAT_BLK_FWD(1, 0);
  }
#undef HICGAT_BLK_FWD
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_gat_blk_bwd_src(const int32_t *rowptr, const int32_t *col, const int32_t *pos,
                                      const int64_t *runs, const int32_t *run_ptr, int N, int nnz,
                                      int H, int C, int row_begin, int row_end, const float *h,
                                      const float *a_src, const float *a_dst,
                                      const float *row_stats, int64_t ld_stats, const float *dout,
                                      int64_t ld_dout, const float *att_src, const float *att_dst,
                                      float neg_slope, float *dh, float *da_src, void *workspace,
                                      size_t workspace_bytes, hicgat_stream_t stream) {
  if (N < 0 || nnz < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (ld_stats < 8 || (ld_stats % 4) != 0 || ld_dout < 512 || (ld_dout % 4) != 0) return HICGAT_EINVAL;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !pos || !runs || !run_ptr || !h || !a_src || !a_dst || !row_stats ||
      !dout || !att_src || !att_dst || !dh || !da_src || !workspace)
    return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_gat_blk_workspace_bytes(N, nnz)) return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  const int nblk = (rows + kBlkRows - 1) / kBlkRows;
  hipStream_t s = (hipStream_t)stream;
  float2 *rec = reinterpret_cast<float2 *>(workspace);
  // sb after the records, 256-byte aligned
  const size_t sb_off = (((size_t)nnz * 8 + 255) / 256) * 256;
  float2 *sb = reinterpret_cast<float2 *>(reinterpret_cast<char *>(workspace) + sb_off);
  hipLaunchKernelGGL(blk_bwd_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, rowptr, col, pos,
                     row_begin, row_end, a_src, a_dst, row_stats, ld_stats, neg_slope, rec, sb);
  HICGAT_CHECK_LAUNCH();
  hipLaunchKernelGGL((blk_gather_kernel<2, 0>), dim3(nblk), dim3(256), 0, s, rowptr,
                     reinterpret_cast<const long long *>(runs), run_ptr, row_begin, row_end,
                     reinterpret_cast<const float *>(rec), reinterpret_cast<const float2 *>(dout),
                     ld_dout / 2, neg_slope, nullptr, nullptr, nullptr,
                     reinterpret_cast<const float2 *>(h), sb, row_stats, ld_stats,
                     reinterpret_cast<const float2 *>(att_src),
                     reinterpret_cast<const float2 *>(att_dst), reinterpret_cast<float2 *>(dh),
                     da_src);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
