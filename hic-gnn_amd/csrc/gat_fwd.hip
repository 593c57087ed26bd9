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

#ifndef HICGAT_FWD_U
#define HICGAT_FWD_U 8   // neighbours gathered per inner step
#endif

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
__global__ __launch_bounds__(256) void agg_fwd_h2c256_kernel(
    const int *__restrict__ rowptr, const int *__restrict__ col, int row_begin, int row_end,
    const float *__restrict__ h, const float *__restrict__ a_src, const float *__restrict__ a_dst,
    const float *__restrict__ bias, float ns, float *__restrict__ out,
    float *__restrict__ row_stats) {
  constexpr int U = HICGAT_FWD_U;  // neighbours in flight per lane
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
  float4 acc0 = make_float4(0.f, 0.f, 0.f, 0.f), acc1 = acc0;
  for (int base = beg; base < end; base += 64) {
    const int e = base + lane;
    int j = i;  // padded slots gather the (valid) own row with weight 0
    float p0 = 0.f, p1 = 0.f;
    if (e < end) {
      j = col[e];
      const float2 s = as2[j];
      p0 = expf(lrelu(s.x + ad.x, ns) - m0) / den0;
      p1 = expf(lrelu(s.y + ad.y, ns) - m1) / den1;
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
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc0 = f4_fma(readlane_f(p0, k + u), v0[u], acc0);
        acc1 = f4_fma(readlane_f(p1, k + u), v1[u], acc1);
      }
    }
  }
  const float4 *b4 = reinterpret_cast<const float4 *>(bias);
  float4 *o4 = reinterpret_cast<float4 *>(out);
  float4 b0 = b4[lane], b1 = b4[64 + lane];
  acc0.x += b0.x; acc0.y += b0.y; acc0.z += b0.z; acc0.w += b0.w;
  acc1.x += b1.x; acc1.y += b1.y; acc1.z += b1.z; acc1.w += b1.w;
  o4[(size_t)i * 128 + lane] = acc0;
  o4[(size_t)i * 128 + 64 + lane] = acc1;
  if (lane == 0) reinterpret_cast<float4 *>(row_stats)[2 * (size_t)i] = make_float4(m0, m1, s0, s1);
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

extern "C" int hicgat_gat_agg_fwd(const int32_t *rowptr, const int32_t *col, int N, int nnz, int H,
                                  int C, int row_begin, int row_end, const float *h,
                                  const float *a_src, const float *a_dst, const float *bias,
                                  float neg_slope, float *out, float *row_stats,
                                  hicgat_stream_t stream) {
  if (N < 0 || nnz < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !h || !a_src || !a_dst || !bias || !out || !row_stats) return HICGAT_EINVAL;
  const int rows = row_end - row_begin;
  hipLaunchKernelGGL(agg_fwd_h2c256_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     rowptr, col, row_begin, row_end, h, a_src, a_dst, bias, neg_slope, out, row_stats);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
