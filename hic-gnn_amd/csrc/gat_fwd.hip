// GATConv forward on gfx950: attention logits (a2) and the fused edge-softmax + aggregation (a4+a5).
//
// Reference: PyG 1.7.2 GATConv.forward / propagate / message + torch_geometric.utils.softmax
// (ptr path) + torch_scatter segment_csr(sum), as called from models.py:634-662.  Those ops
// materialise an [nnz, H, C] message tensor; here one wave owns one destination row and never
// writes anything per edge.
//
// Layout: h [N, D] fp32 row-major (D = H*C = 512 -> one 2 KiB row), a_src/a_dst [N, H],
// CSR int32 (rowptr [N+1], col [nnz]) with the self loops already inserted, row_stats [N, 4H]
// = (max[H], sum[H], delta[H], da_dst[H]) per row.  A launch covers rows [row_begin, row_end)
// (a rank's destination shard); every per-row array is indexed by the global row id.
#include "common.hpp"

constexpr int kFwdU = 8;   // neighbours gathered per inner step

namespace hicgat {

// ---- a2: a_src[n,h] = <h[n,h,:], att_src[h,:]>, a_dst likewise (one wave per row). -------------
__global__ __launch_bounds__(256) void att_logits_kernel(const float *__restrict__ h,
                                                         const float *__restrict__ att_s,
                                                         const float *__restrict__ att_d, int N,
                                                         int H, int C, float *__restrict__ a_src,
                                                         float *__restrict__ a_dst) {
  const int lane = lane_id();
  const int n = blockIdx.x * 4 + wave_in_block();
  if (n >= N) return;
  const int D = H * C;
  const float4 *h4 = reinterpret_cast<const float4 *>(h + (size_t)n * D);
  const float4 *s4 = reinterpret_cast<const float4 *>(att_s);
  const float4 *d4 = reinterpret_cast<const float4 *>(att_d);
  // C % 4 == 0: a float4 never straddles two heads.  Heads are visited one after the other.
  for (int hh = 0; hh < H; ++hh) {
    float ps = 0.f, pd = 0.f;
    for (int q = lane; q < C / 4; q += 64) {
      const int idx = hh * (C / 4) + q;
      const float4 v = h4[idx];
      ps += f4_dot(v, s4[idx]);
      pd += f4_dot(v, d4[idx]);
    }
    ps = wave_sum(ps);
    pd = wave_sum(pd);
    if (lane == 0) {
      a_src[(size_t)n * H + hh] = ps;
      a_dst[(size_t)n * H + hh] = pd;
    }
  }
}

// ---- a4+a5 fast path: H = 2, C = 256 (D = 512, the GATConv(512, 256, heads=2) of models.py:619).
// Lane l holds float4 #l of head 0 (cols 4l..4l+3) and float4 #l of head 1 (cols 256+4l..).
// Pass 1/2 stream only col[] and a_src[] (row max, row sum); pass 3 gathers h[j] rows with the
// neighbour index and both alphas broadcast from lane k through SGPRs (v_readlane), so each
// gather is one scalar base + per-lane offset global_load_dwordx4, 8 neighbours in flight.
//
// TRAIN also accumulates, from the same gathered rows (FMAs only, no extra loads),
//   out2[i] = sum_j alpha_ij lrelu'(e_ij) h_j    and    S3[i] = sum_j alpha_ij lrelu'(e_ij)
// (S3 into row_stats[i, 4:6]).  With those the destination half of the backward needs no gather:
//   delta_i = sum_j alpha_ij <dout_i, h_j> = <dout_i, out_i - bias>,
//   da_dst_i = sum_j alpha_ij lrelu'(e_ij) (<dout_i, h_j> - delta_i) = <dout_i, out2_i> - delta_i S3_i
// (agg_bwd_rows_kernel, gat_bwd.hip).  ACT = 1 applies the relu that follows the GATConv in
// GATNetSelectiveResidualsUpdated (models.py:637) in the epilogue: out = relu(acc + bias).
//
// SPLIT (the tiled form, gat_tiles.hip): the softmax statistics still come from the whole row
// (rowptr/col), but only the edges of the sparse remainder (rowptr_s/col_s) are gathered, and the
// raw sums (no bias, no activation) go to out/out2 with S3 of those edges; the matrix-core pass over
// the row's dense 32x32 tiles adds the rest and applies the epilogue.
template <bool TRAIN, int ACT, bool SPLIT = false>
__global__ __launch_bounds__(256, 1) void agg_fwd_h2c256_kernel(
    const int *__restrict__ rowptr, const int *__restrict__ col, int row_begin, int row_end,
    const float *__restrict__ h, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    const float *__restrict__ bias, float ns, float *__restrict__ out, float *__restrict__ out2,
    float *__restrict__ row_stats, const int *__restrict__ rowptr_s = nullptr,
    const int *__restrict__ col_s = nullptr) {
  constexpr int U = kFwdU;  // neighbours in flight per lane
  const int lane = lane_id();
  const int i = row_begin + xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_in_block();
  if (i >= row_end) return;
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

  const float4 *h4 = reinterpret_cast<const float4 *>(h);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc0 = z4, acc1 = z4, acs0 = z4, acs1 = z4;
  float t0 = 0.f, t1 = 0.f;
  const int gbeg = SPLIT ? rowptr_s[i] : beg, gend = SPLIT ? rowptr_s[i + 1] : end;
  const int *__restrict__ gcol = SPLIT ? col_s : col;
  for (int base = gbeg; base < gend; base += 64) {
    const int e = base + lane;
    int j = i;  // padded slots gather the (valid) own row with weight 0
    float p0 = 0.f, p1 = 0.f, q0 = 0.f, q1 = 0.f;
    if (e < gend) {
      j = gcol[e];
      const float2 s = as2[j];
      const float e0 = s.x + ad.x, e1 = s.y + ad.y;
      p0 = expf(lrelu(e0, ns) - m0) / den0;
      p1 = expf(lrelu(e1, ns) - m1) / den1;
      if (TRAIN) {
        q0 = p0 * (e0 > 0.f ? 1.f : ns);
        q1 = p1 * (e1 > 0.f ? 1.f : ns);
        t0 += q0;
        t1 += q1;
      }
    }
    const int cnt = min(64, gend - base);
    for (int k = 0; k < cnt; k += U) {
      float4 v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t jj = (size_t)readlane_i(j, k + u);
        v0[u] = h4[jj * 128 + lane];
        v1[u] = h4[jj * 128 + 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc0 = f4_fma(readlane_f(p0, k + u), v0[u], acc0);
        acc1 = f4_fma(readlane_f(p1, k + u), v1[u], acc1);
        if (TRAIN) {
          acs0 = f4_fma(readlane_f(q0, k + u), v0[u], acs0);
          acs1 = f4_fma(readlane_f(q1, k + u), v1[u], acs1);
        }
      }
    }
  }
  const float4 *b4 = reinterpret_cast<const float4 *>(bias);
  float4 *o4 = reinterpret_cast<float4 *>(out);
  float4 b0 = SPLIT ? z4 : b4[lane], b1 = SPLIT ? z4 : b4[64 + lane];
  acc0.x += b0.x; acc0.y += b0.y; acc0.z += b0.z; acc0.w += b0.w;
  acc1.x += b1.x; acc1.y += b1.y; acc1.z += b1.z; acc1.w += b1.w;
  if (ACT == 1 && !SPLIT) {
    acc0 = f4_relu(acc0);
    acc1 = f4_relu(acc1);
  }
  o4[(size_t)i * 128 + lane] = acc0;
  o4[(size_t)i * 128 + 64 + lane] = acc1;
  float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
  if (TRAIN) {
    float4 *q4 = reinterpret_cast<float4 *>(out2);
    q4[(size_t)i * 128 + lane] = acs0;
    q4[(size_t)i * 128 + 64 + lane] = acs1;
    t0 = wave_sum(t0);
    t1 = wave_sum(t1);
    if (lane == 0) rs4[2 * (size_t)i + 1] = make_float4(t0, t1, 0.f, 0.f);
  }
  if (lane == 0) rs4[2 * (size_t)i] = make_float4(m0, m1, s0, s1);
}

// The gather half of hicgat_gat_agg_fwd_tiled (gat_tiles.hip): raw sums over the sparse remainder.
int agg_fwd_split_launch(const int *rowptr, const int *col, const int *rowptr_s, const int *col_s, int row_begin,
                         int row_end, const float *h, const float *a_src, const float *a_dst, float ns, float *out,
                         float *out2, float *row_stats, hipStream_t s) {
  const dim3 grid((row_end - row_begin + 3) / 4), block(256);
  if (out2)
    hipLaunchKernelGGL((agg_fwd_h2c256_kernel<true, 0, true>), grid, block, 0, s, rowptr, col, row_begin, row_end,
                       h, a_src, a_dst, nullptr, ns, out, out2, row_stats, rowptr_s, col_s);
  else
    hipLaunchKernelGGL((agg_fwd_h2c256_kernel<false, 0, true>), grid, block, 0, s, rowptr, col, row_begin, row_end,
                       h, a_src, a_dst, nullptr, ns, out, out2, row_stats, rowptr_s, col_s);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_gat_att_logits(const float *h, const float *att_src, const float *att_dst,
                                     int N, int H, int C, float *a_src, float *a_dst,
                                     hicgat_stream_t stream) {
  if (N < 0 || H <= 0 || C <= 0 || (C % 4) != 0) return HICGAT_EINVAL;
  if (N == 0) return HICGAT_OK;
  if (!h || !att_src || !att_dst || !a_src || !a_dst) return HICGAT_EINVAL;
  hipLaunchKernelGGL(att_logits_kernel, dim3((N + 3) / 4), dim3(256), 0, (hipStream_t)stream, h,
                     att_src, att_dst, N, H, C, a_src, a_dst);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

// Unused dynamic LDS per workgroup of the gather launch below: 3 workgroups per CU (160 KiB / 52 KiB)
// instead of the 4 its 98 VGPRs allow -- fewer rows in flight per CU, fewer L2 misses: the
// single-GPU step 1.798-1.803 vs 1.820-1.821 ms together with the source pass's cap (gat_bwd.hip;
// 2 per CU: +30 us), profiles/r05at_gather_occupancy_ab.txt
constexpr size_t kAggFwdOccLds = 53248;

extern "C" int hicgat_gat_agg_fwd_act(const int32_t *rowptr, const int32_t *col, int N, int nnz,
                                      int H, int C, int row_begin, int row_end, const float *h,
                                      const float *a_src, const float *a_dst, const float *bias,
                                      float neg_slope, int act, float *out, float *out2,
                                      float *row_stats, hicgat_stream_t stream) {
  if (N < 0 || nnz < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (act != 0 && act != 1) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !h || !a_src || !a_dst || !bias || !out || !row_stats) return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  const dim3 grid((rows + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
#define HICGAT_FWD_LAUNCH(TR, AC)                                                                  \
  hipLaunchKernelGGL((agg_fwd_h2c256_kernel<TR, AC>), grid, block, kAggFwdOccLds, s, rowptr, col, row_begin, \
                     row_end, h, a_src, a_dst, bias, neg_slope, out, out2, row_stats)
  if (out2) {
    if (act) HICGAT_FWD_LAUNCH(true, 1);
    else HICGAT_FWD_LAUNCH(true, 0);
  } else {
    if (act) HICGAT_FWD_LAUNCH(false, 1);
    else HICGAT_FWD_LAUNCH(false, 0);
  }
#undef HICGAT_FWD_LAUNCH
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_gat_agg_fwd(const int32_t *rowptr, const int32_t *col, int N, int nnz, int H,
                                  int C, int row_begin, int row_end, const float *h,
                                  const float *a_src, const float *a_dst, const float *bias,
                                  float neg_slope, float *out, float *row_stats,
                                  hicgat_stream_t stream) {
  return hicgat_gat_agg_fwd_act(rowptr, col, N, nnz, H, C, row_begin, row_end, h, a_src, a_dst, bias,
                                neg_slope, 0, out, nullptr, row_stats, stream);
}
