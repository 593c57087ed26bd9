// Column-sliced GAT aggregation (a4+a5) and its source-side backward, for the 8 XCDs of gfx950.
//
// Reference: the same math as gat_fwd.hip / gat_bwd.hip (PyG 1.7.2 GATConv propagate + ptr-path
// softmax + segment_csr(sum), models.py:634-662, and their autograd).  Why a second form: the
// row-per-wave kernels gather whole 2 KiB rows, so every XCD touches all of h (41 MB at
// N = 20000) and its 4 MB L2 misses about a third of the lines (PMC:
// profiles/r01_pmc_l2_hit_synth20000.txt) -- the gathers are served by the Infinity Cache.  Here
// the D = 512 columns are cut into NS = 512/SW strips; block b runs on XCD b & 7 (the hardware's
// round-robin workgroup dispatch) and works on strip (b & 7) + 8*pass, so one XCD's L2 only holds
// an SW-column strip of the gathered matrix (N*SW*4 B = 2.56 MB at SW = 32).
//
// The softmax weights are computed once per edge into per-head edge records
// rec[head][e] = {neighbour, alpha} (8 B).  alpha >= 0, so its sign bit is free and carries the
// leaky-relu branch [e <= 0]: alpha*lrelu'(e) needs no logits.  The strip kernels stage 64 records
// per wave in LDS; each group of L = SW/4 lanes gathers one neighbour's SW columns (one float4 per
// lane), G = 64/L neighbours per load instruction, and the G partial sums of a column are
// combined by a butterfly at the end of the row (fixed order: deterministic, no atomics).
#include "common.hpp"

namespace hicgat {

__device__ __forceinline__ int2 edge_rec(int j, float alpha, float e) {
  return make_int2(j, (int)(__float_as_uint(alpha) | (e > 0.f ? 0u : 0x80000000u)));
}

// Destination rows: row max / sum (and S3 = sum alpha lrelu' for TRAIN) exactly as
// agg_fwd_h2c256_kernel, plus the edge records.  One wave per row.
template <bool TRAIN>
__global__ __launch_bounds__(256) void agg_edge_rec_kernel(const int *__restrict__ rowptr,
                                                           const int *__restrict__ col, int row_begin,
                                                           int row_end, int nnz,
                                                           const float *__restrict__ a_src,
                                                           const float *__restrict__ a_dst, float ns,
                                                           int2 *__restrict__ rec,
                                                           float *__restrict__ row_stats) {
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
  float t0 = 0.f, t1 = 0.f;
  for (int e = beg + lane; e < end; e += 64) {
    const int j = col[e];
    const float2 s = as2[j];
    const float e0 = s.x + ad.x, e1 = s.y + ad.y;
    const float p0 = expf(lrelu(e0, ns) - m0) / den0;
    const float p1 = expf(lrelu(e1, ns) - m1) / den1;
    rec[e] = edge_rec(j, p0, e0);
    rec[(size_t)nnz + e] = edge_rec(j, p1, e1);
    if (TRAIN) {
      t0 += p0 * (e0 > 0.f ? 1.f : ns);
      t1 += p1 * (e1 > 0.f ? 1.f : ns);
    }
  }
  float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
  if (TRAIN) {
    t0 = wave_sum(t0);
    t1 = wave_sum(t1);
    if (lane == 0) rs4[2 * (size_t)i + 1] = make_float4(t0, t1, 0.f, 0.f);
  }
  if (lane == 0) rs4[2 * (size_t)i] = make_float4(m0, m1, s0, s1);
}

// Source rows r (the graph is symmetric: r's CSR list is every i that has r as a neighbour):
// records {i, alpha_ir} (alpha from row i's max / sum, ldr = row_stats row stride in floats) and
// sb[r,h] = sum_i alpha_ir lrelu'_ir delta_i, parked in da_src[r] until agg_src_finalize_kernel.
__global__ __launch_bounds__(256) void agg_src_rec_kernel(const int *__restrict__ rowptr,
                                                          const int *__restrict__ col, int row_begin,
                                                          int row_end, int nnz,
                                                          const float *__restrict__ a_src,
                                                          const float *__restrict__ a_dst,
                                                          const float *__restrict__ row_stats, int64_t ldr,
                                                          float ns, int2 *__restrict__ rec,
                                                          float *__restrict__ da_src) {
  const int lane = lane_id();
  const int r = row_begin + xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_in_block();
  if (r >= row_end) return;
  const int beg = rowptr[r], end = rowptr[r + 1];
  const float2 asr = *reinterpret_cast<const float2 *>(a_src + 2 * (size_t)r);
  const float2 *ad2 = reinterpret_cast<const float2 *>(a_dst);
  float sb0 = 0.f, sb1 = 0.f;
  for (int e = beg + lane; e < end; e += 64) {
    const int inb = col[e];
    const float2 ad = ad2[inb];
    const float *rs = row_stats + (size_t)ldr * inb;
    const float4 ms = *reinterpret_cast<const float4 *>(rs);       // max0 max1 sum0 sum1
    const float2 dl = *reinterpret_cast<const float2 *>(rs + 4);   // delta0 delta1
    const float e0 = asr.x + ad.x, e1 = asr.y + ad.y;
    const float al0 = expf(lrelu(e0, ns) - ms.x) / (ms.z + 1e-16f);
    const float al1 = expf(lrelu(e1, ns) - ms.y) / (ms.w + 1e-16f);
    sb0 = fmaf(al0 * (e0 > 0.f ? 1.f : ns), dl.x, sb0);
    sb1 = fmaf(al1 * (e1 > 0.f ? 1.f : ns), dl.y, sb1);
    rec[e] = edge_rec(inb, al0, e0);
    rec[(size_t)nnz + e] = edge_rec(inb, al1, e1);
  }
  sb0 = wave_sum(sb0);
  sb1 = wave_sum(sb1);
  if (lane == 0) *reinterpret_cast<float2 *>(da_src + 2 * (size_t)r) = make_float2(sb0, sb1);
}

// NU load instructions (NU*G neighbours) from the staged records st[k ..]: the lane of neighbour
// group `sub` gathers float4 m4[nb * ld4] (m4 already offset to the lane's column) of neighbour
// k + u*G + sub and accumulates alpha * v into acc and alpha*lrelu' * v into acs (TRAIN).
template <int NU, int G, bool TRAIN>
__device__ __forceinline__ void strip_step(const long long *st, int k, int sub, const float4 *m4, int64_t ld4,
                                           float ns, float4 &acc, float4 &acs) {
  float4 v[NU];
  float a[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const long long t = st[k + u * G + sub];
    a[u] = __int_as_float((int)(t >> 32));
    v[u] = m4[(size_t)(uint32_t)t * ld4];
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const float p = fabsf(a[u]);
    acc = f4_fma(p, v[u], acc);
    if (TRAIN) acs = f4_fma(__float_as_int(a[u]) < 0 ? p * ns : p, v[u], acs);
  }
}

__device__ __forceinline__ float4 f4_xor_sum(float4 a, int o) {
  a.x += __shfl_xor(a.x, o);
  a.y += __shfl_xor(a.y, o);
  a.z += __shfl_xor(a.z, o);
  a.w += __shfl_xor(a.w, o);
  return a;
}

#ifndef HICGAT_STRIP_RPW
#define HICGAT_STRIP_RPW 4   // consecutive rows one strip wave walks (amortises the per-row latencies)
#endif
constexpr int kRPW = HICGAT_STRIP_RPW;

// Block -> (strip, 4 waves x kRPW consecutive rows): XCD x = b & 7 walks strips x, x + 8, ... one
// pass after the other.
struct Strip {
  int slice, row0;
  __device__ Strip(int row_begin, int row_blocks) {
    const int q = blockIdx.x >> 3;
    slice = (blockIdx.x & 7) + 8 * (q / row_blocks);
    row0 = row_begin + ((q % row_blocks) * 4 + wave_in_block()) * kRPW;
  }
};

// The gather loop shared by the forward and the backward strip kernels: rows row0 .. row0+kRPW-1
// (< row_end) of one head's records, 64 records per LDS chunk; the NEXT chunk's records (possibly
// the next row's) are loaded while the current chunk is gathered, so a record round trip is paid
// once per wave, not once per chunk.  Padded slots gather the (valid) own row with weight +0.
// finish(i, acc, acs) runs when row i is complete.
template <int G, bool TRAIN, typename Finish>
__device__ __forceinline__ void strip_wave(const int *__restrict__ rowptr, const long long *__restrict__ rh,
                                           int row0, int row_end, long long *st, int lane, int sub,
                                           const float4 *m4, int64_t ld4, float ns, Finish finish) {
  const int rlast = min(row_end, row0 + kRPW);
  int i = row0, end = rowptr[i + 1], base = rowptr[i];
  long long pre = base + lane < end ? __builtin_nontemporal_load(rh + base + lane) : (long long)(uint32_t)i;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc = z4, acs = z4;
  while (true) {
    st[lane] = pre;
    __builtin_amdgcn_wave_barrier();
    const int cnt = min(64, end - base);
    // the next chunk: the rest of this row, else the next row of the wave
    int ni = i, nbase = base + 64, nend = end;
    const bool row_done = nbase >= end;
    if (row_done) {
      ni = i + 1;
      if (ni < rlast) {
        nbase = rowptr[ni];
        nend = rowptr[ni + 1];
      }
    }
    if (ni < rlast) pre = nbase + lane < nend ? __builtin_nontemporal_load(rh + nbase + lane) : (long long)(uint32_t)ni;
    int k = 0;
    while (k < cnt) {   // the widest step the remaining records fill at least half of
      const int r = cnt - k;
      if (r > 4 * G) {
        strip_step<8, G, TRAIN>(st, k, sub, m4, ld4, ns, acc, acs);
        k += 8 * G;
      } else if (r > 2 * G) {
        strip_step<4, G, TRAIN>(st, k, sub, m4, ld4, ns, acc, acs);
        k += 4 * G;
      } else if (r > G) {
        strip_step<2, G, TRAIN>(st, k, sub, m4, ld4, ns, acc, acs);
        k += 2 * G;
      } else {
        strip_step<1, G, TRAIN>(st, k, sub, m4, ld4, ns, acc, acs);
        k += G;
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (row_done) {
      finish(i, acc, acs);
      acc = z4;
      acs = z4;
      if (ni >= rlast) break;
    }
    i = ni;
    base = nbase;
    end = nend;
  }
}

template <int SW, bool TRAIN, int ACT>
__global__ __launch_bounds__(256) void agg_fwd_strip_kernel(const int *__restrict__ rowptr, int row_begin,
                                                            int row_end, int nnz, int row_blocks,
                                                            const int2 *__restrict__ rec,
                                                            const float *__restrict__ h,
                                                            const float *__restrict__ bias, float ns,
                                                            float *__restrict__ out, float *__restrict__ out2) {
  constexpr int L = SW / 4, G = 64 / L;
  __shared__ long long stage[4][64];
  const Strip s(row_begin, row_blocks);
  if (s.row0 >= row_end) return;
  const int lane = lane_id(), sub = lane / L, c4 = s.slice * L + lane % L;
  const long long *rh = reinterpret_cast<const long long *>(rec) + (size_t)((s.slice * SW) >> 8) * nnz;
  const float4 b = reinterpret_cast<const float4 *>(bias)[c4];
  strip_wave<G, TRAIN>(rowptr, rh, s.row0, row_end, stage[wave_in_block()], lane, sub,
                       reinterpret_cast<const float4 *>(h) + c4, 128, ns, [&](int i, float4 acc, float4 acs) {
#pragma unroll
    for (int o = L; o < 64; o <<= 1) {
      acc = f4_xor_sum(acc, o);
      if (TRAIN) acs = f4_xor_sum(acs, o);
    }
    if (sub == 0) {
      acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
      if (ACT == 1) acc = f4_relu(acc);
      reinterpret_cast<float4 *>(out)[(size_t)i * 128 + c4] = acc;
      if (TRAIN) reinterpret_cast<float4 *>(out2)[(size_t)i * 128 + c4] = acs;
    }
  });
}

// dh[r, strip] = sum_i alpha_ir dout_i[strip] and part[r][strip] = <sum_i alpha_ir lrelu'_ir dout_i, h_r>
// over the strip's columns (ld4: dout row stride in float4).
template <int SW>
__global__ __launch_bounds__(256) void agg_bwd_src_strip_kernel(const int *__restrict__ rowptr, int row_begin,
                                                                int row_end, int nnz, int row_blocks,
                                                                const int2 *__restrict__ rec,
                                                                const float *__restrict__ h,
                                                                const float *__restrict__ dout, int64_t ld4,
                                                                float ns, float *__restrict__ dh,
                                                                float *__restrict__ part) {
  constexpr int L = SW / 4, G = 64 / L, NS = 512 / SW;
  __shared__ long long stage[4][64];
  const Strip s(row_begin, row_blocks);
  if (s.row0 >= row_end) return;
  const int lane = lane_id(), sub = lane / L, c4 = s.slice * L + lane % L;
  const long long *rh = reinterpret_cast<const long long *>(rec) + (size_t)((s.slice * SW) >> 8) * nnz;
  const int slice = s.slice;
  strip_wave<G, true>(rowptr, rh, s.row0, row_end, stage[wave_in_block()], lane, sub,
                      reinterpret_cast<const float4 *>(dout) + c4, ld4, ns, [&](int r, float4 acc, float4 cc) {
    const float d = wave_sum(f4_dot(cc, reinterpret_cast<const float4 *>(h)[(size_t)r * 128 + c4]));
#pragma unroll
    for (int o = L; o < 64; o <<= 1) acc = f4_xor_sum(acc, o);
    if (sub == 0) reinterpret_cast<float4 *>(dh)[(size_t)r * 128 + c4] = acc;
    if (lane == 0) part[(size_t)r * NS + slice] = d;
  });
}

// da_src[r,h] = (sum of head h's strip shares) - sb[r,h];  dh_r += da_src (x) att_src + da_dst (x) att_dst.
template <int NS>
__global__ __launch_bounds__(256) void agg_src_finalize_kernel(int row_begin, int row_end,
                                                               const float *__restrict__ part,
                                                               const float *__restrict__ row_stats, int64_t ldr,
                                                               const float *__restrict__ att_s,
                                                               const float *__restrict__ att_d,
                                                               float *__restrict__ dh, float *__restrict__ da_src) {
  const int lane = lane_id();
  const int r = row_begin + blockIdx.x * 4 + wave_in_block();
  if (r >= row_end) return;
  const float *pr = part + (size_t)r * NS;
  float ds0 = 0.f, ds1 = 0.f;
#pragma unroll
  for (int k = 0; k < NS / 2; ++k) {
    ds0 += pr[k];
    ds1 += pr[NS / 2 + k];
  }
  const float2 sb = *reinterpret_cast<const float2 *>(da_src + 2 * (size_t)r);
  ds0 -= sb.x;
  ds1 -= sb.y;
  const float2 dd = *reinterpret_cast<const float2 *>(row_stats + (size_t)ldr * r + 6);
  const float4 *s4 = reinterpret_cast<const float4 *>(att_s);
  const float4 *t4 = reinterpret_cast<const float4 *>(att_d);
  float4 *o4 = reinterpret_cast<float4 *>(dh) + (size_t)r * 128;
  float4 a0 = o4[lane], a1 = o4[64 + lane];
  a0 = f4_fma(ds0, s4[lane], a0);
  a0 = f4_fma(dd.x, t4[lane], a0);
  a1 = f4_fma(ds1, s4[64 + lane], a1);
  a1 = f4_fma(dd.y, t4[64 + lane], a1);
  o4[lane] = a0;
  o4[64 + lane] = a1;
  if (lane == 0) *reinterpret_cast<float2 *>(da_src + 2 * (size_t)r) = make_float2(ds0, ds1);
}

static size_t rec_bytes(int nnz, int H) {
  return ((size_t)(nnz > 0 ? nnz : 0) * (size_t)(H > 0 ? H : 0) * sizeof(int2) + 255) & ~(size_t)255;
}

}  // namespace hicgat

using namespace hicgat;

extern "C" size_t hicgat_gat_sliced_workspace_bytes(int N, int nnz, int H, int slice_width) {
  const int ns = slice_width > 0 ? 512 / slice_width : 0;
  return rec_bytes(nnz, H) + (size_t)(N > 0 ? N : 0) * ns * sizeof(float);
}

extern "C" int hicgat_gat_agg_fwd_sliced(const int32_t *rowptr, const int32_t *col, int N, int nnz, int H,
                                         int C, int row_begin, int row_end, const float *h,
                                         const float *a_src, const float *a_dst, const float *bias,
                                         float neg_slope, int act, int slice_width, float *out, float *out2,
                                         float *row_stats, void *workspace, size_t workspace_bytes,
                                         hicgat_stream_t stream) {
  if (N < 0 || nnz < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (act != 0 && act != 1) return HICGAT_EINVAL;
  if (slice_width != 32 && slice_width != 64) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !h || !a_src || !a_dst || !bias || !out || !row_stats || !workspace)
    return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_gat_sliced_workspace_bytes(N, nnz, H, slice_width)) return HICGAT_EINVAL;
  const int rb = (row_end - row_begin + 3) / 4;
  const int sb = (row_end - row_begin + 4 * kRPW - 1) / (4 * kRPW);   // strip row blocks
  hipStream_t s = (hipStream_t)stream;
  int2 *rec = static_cast<int2 *>(workspace);
  if (out2)
    hipLaunchKernelGGL(agg_edge_rec_kernel<true>, dim3(rb), dim3(256), 0, s, rowptr, col, row_begin, row_end,
                       nnz, a_src, a_dst, neg_slope, rec, row_stats);
  else
    hipLaunchKernelGGL(agg_edge_rec_kernel<false>, dim3(rb), dim3(256), 0, s, rowptr, col, row_begin, row_end,
                       nnz, a_src, a_dst, neg_slope, rec, row_stats);
  HICGAT_CHECK_LAUNCH();
  const dim3 grid((512 / slice_width) * sb), block(256);
#define HICGAT_STRIP(SW, TR, AC)                                                                     \
  hipLaunchKernelGGL((agg_fwd_strip_kernel<SW, TR, AC>), grid, block, 0, s, rowptr, row_begin, row_end, \
                     nnz, sb, rec, h, bias, neg_slope, out, out2)
#define HICGAT_STRIP_W(SW)                   \
  do {                                       \
    if (out2) {                              \
      if (act) HICGAT_STRIP(SW, true, 1);    \
      else HICGAT_STRIP(SW, true, 0);        \
    } else {                                 \
      if (act) HICGAT_STRIP(SW, false, 1);   \
      else HICGAT_STRIP(SW, false, 0);       \
    }                                        \
  } while (0)
  if (slice_width == 32) HICGAT_STRIP_W(32);
  else HICGAT_STRIP_W(64);
#undef HICGAT_STRIP_W
#undef HICGAT_STRIP
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_gat_agg_bwd_src_sliced(const int32_t *rowptr, const int32_t *col, int N, int nnz, int H,
                                             int C, int row_begin, int row_end, const float *h,
                                             const float *a_src, const float *a_dst, const float *row_stats,
                                             int64_t ld_stats, const float *dout, int64_t ld_dout,
                                             const float *att_src, const float *att_dst, float neg_slope,
                                             int slice_width, float *dh, float *da_src, void *workspace,
                                             size_t workspace_bytes, hicgat_stream_t stream) {
  if (N < 0 || nnz < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (slice_width != 32 && slice_width != 64) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (ld_stats < 4 * H || ld_stats % 4 || ld_dout < H * C || ld_dout % 4) return HICGAT_EINVAL;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !h || !a_src || !a_dst || !row_stats || !dout || !att_src || !att_dst || !dh ||
      !da_src || !workspace)
    return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_gat_sliced_workspace_bytes(N, nnz, H, slice_width)) return HICGAT_EINVAL;
  const int rb = (row_end - row_begin + 3) / 4;
  const int sb = (row_end - row_begin + 4 * kRPW - 1) / (4 * kRPW);   // strip row blocks
  hipStream_t s = (hipStream_t)stream;
  int2 *rec = static_cast<int2 *>(workspace);
  float *part = reinterpret_cast<float *>(static_cast<char *>(workspace) + rec_bytes(nnz, H));
  hipLaunchKernelGGL(agg_src_rec_kernel, dim3(rb), dim3(256), 0, s, rowptr, col, row_begin, row_end, nnz, a_src,
                     a_dst, row_stats, ld_stats, neg_slope, rec, da_src);
  HICGAT_CHECK_LAUNCH();
  const dim3 grid((512 / slice_width) * sb), block(256);
  if (slice_width == 32) {
    hipLaunchKernelGGL(agg_bwd_src_strip_kernel<32>, grid, block, 0, s, rowptr, row_begin, row_end, nnz, sb, rec,
                       h, dout, ld_dout / 4, neg_slope, dh, part);
    HICGAT_CHECK_LAUNCH();
    hipLaunchKernelGGL(agg_src_finalize_kernel<16>, dim3(rb), block, 0, s, row_begin, row_end, part, row_stats,
                       ld_stats, att_src, att_dst, dh, da_src);
  } else {
    hipLaunchKernelGGL(agg_bwd_src_strip_kernel<64>, grid, block, 0, s, rowptr, row_begin, row_end, nnz, sb, rec,
                       h, dout, ld_dout / 4, neg_slope, dh, part);
    HICGAT_CHECK_LAUNCH();
    hipLaunchKernelGGL(agg_src_finalize_kernel<8>, dim3(rb), block, 0, s, row_begin, row_end, part, row_stats,
                       ld_stats, att_src, att_dst, dh, da_src);
  }
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
