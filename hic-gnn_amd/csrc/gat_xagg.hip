// GATConv (H = 2, C = 256, F = 512) in AGGREGATE-FIRST order, for the multi-GPU "xagg" step form
// (hicgat.dist).  The reference computes h = x W^T for every node and aggregates h (PyG 1.7.2
// GATConv.forward / propagate, models.py:619); by linearity the same layer is
//   out_i^h = W_h (sum_j alpha_ij^h x_j) + b^h = W_h xa_i^h + b^h,
//   a_src_j^h = <att_src^h, W_h x_j> = <W_h^T att_src^h, x_j>        (a_dst likewise),
// so a rank that owns destination rows i needs no h of any other row: it aggregates the (constant,
// replicated) input rows x_j, and every GEMM runs on its own rows only.  The backward follows the
// same algebra (d alpha_ij = <dout_i^h, W_h x_j> = <dxa_i^h, x_j> with dxa_i^h = dout_i^h W_h):
//   dW_h   = sum_i dout_i^h xa_i^h^T + att_src^h g_src^h^T + att_dst^h g_dst^h^T,
//   g_src^h = sum_j da_src_j^h x_j,   g_dst^h = sum_i da_dst_i^h x_i,
//   datt_src^h = W_h g_src^h,  datt_dst^h = W_h g_dst^h,
// every term a sum over the rank's rows (or its edges) -- partial sums the gradient all-reduce adds.
// Same values as the h-first order up to fp32 reassociation (tests/test_dist_gloo.py,
// tests/test_gpu_dist.py).
//
// Kernels (wave64, no atomics; the two gather passes one row per 4-wave block, the others one wave per row):
//   xagg_vec_kernel     v = [W_0^T att_src^0, W_1^T att_src^1, W_0^T att_dst^0, W_1^T att_dst^1] [4, 512]
//   xagg_logits_kernel  a_src / a_dst [N, 2] = x . v (every row: the rank's neighbours are anywhere)
//   xagg_fwd_kernel     own rows: softmax stats, then ONE gather pass over x_j accumulating
//                       xa^h = sum alpha x_j and xa2^h = sum alpha lrelu' x_j for both heads
//                       (S3 into row_stats as the h-first training form does, gat_fwd.hip)
//   xagg_bias_relu      y0 += bias, o = relu(y0)      (after the [xa; xa2] W_h^T GEMMs)
//   xagg_edge_kernel    own rows: per edge ds_ij^h = alpha lrelu' (<dxa_i^h, x_j> - delta_i^h)
//                       written in the rank's CSR order
//   xagg_rows_bwd       own rows: dout = g relu'(y0), delta^h = <dout^h, y0^h - b^h> (no gather)
//   xagg_slab_sum       every row j: da_src_j = sum of ds over the rank's edges (i, j), read
//                       through the column slab (the transpose, by a precomputed permutation),
//                       and g_src^h = sum_j da_src_j^h x_j in the same pass (+ xagg_colred)
//   xagg_param_finish   dW += att (x) g terms, datt_src / datt_dst = W_h g
#include "common.hpp"
#include "pack.hpp"

constexpr int kXaggU = 4;    // neighbours gathered per inner step (4 x 2 float4 in flight per lane)
constexpr int kXaggGL = 8;   // edge pass (slab form): lanes per edge (16 float4 of x_j per lane in flight)

namespace hicgat {

// ---- v [4][512]: block b = (which, 64-column group); thread (q, k) sums the 64 weights c in
// [64q, 64q + 64) of column k, the four quarters added in order (32 blocks: the 8-block form with a
// 256-long chain per thread took 14 us, one launch on every step's critical path) -------------------
__global__ __launch_bounds__(256) void xagg_vec_kernel(const float *__restrict__ W, const float *__restrict__ att_s,
                                                       const float *__restrict__ att_d, float *__restrict__ v,
                                                       float *__restrict__ zero_buf, int64_t zero_n,
                                                       int64_t *__restrict__ step_ctr, const PackJobs pj) {
  __shared__ float red[4][64];
  // the optimizer's device step count advances here, at the step's first launch (Adam reads it at
  // the step's end: hicgat_adam_step_table_ex with counted = 1, no increment launch of its own)
  if (step_ctr && blockIdx.x == 0 && threadIdx.x == 0) step_ctr[0] = step_ctr[0] + 1;
  if (zero_buf) {   // the step's flat gradient buffer (zero_grad) rides along: float4 stores, then the tail
    const int64_t n4 = zero_n / 4, stride = (int64_t)gridDim.x * 256;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) reinterpret_cast<float4 *>(zero_buf)[i] = z;
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < zero_n; i += stride) zero_buf[i] = 0.f;
  }
  // blocks 32.. (hicgat_xagg_logits_zero_pack): the one-kernel tail's packed weights of this step
  // (pack.hpp; hicgat_tail_pack's launch folded into the step's first one)
  if (blockIdx.x >= 32) {
    pack_block(pj, blockIdx.x - 32);
    return;
  }
  const int which = blockIdx.x >> 3;                 // 0, 1: att_src heads 0, 1; 2, 3: att_dst heads 0, 1
  const int kl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int k = (blockIdx.x & 7) * 64 + kl;
  const int hd = which & 1;
  const float *att = (which < 2 ? att_s : att_d) + hd * 256 + q * 64;
  const float *w = W + ((size_t)hd * 256 + q * 64) * 512 + k;
  float s = 0.f;
#pragma unroll 8
  for (int c = 0; c < 64; ++c) s = fmaf(att[c], w[(size_t)c * 512], s);
  red[q][kl] = s;
  __syncthreads();
  if (q == 0) v[which * 512 + k] = ((red[0][kl] + red[1][kl]) + red[2][kl]) + red[3][kl];
}

// ---- a_src / a_dst for every row: lane l holds float4 #l and #64+l of x_n and of each v --------
__global__ __launch_bounds__(256) void xagg_logits_kernel(const float *__restrict__ x, const float *__restrict__ v,
                                                          int N, float *__restrict__ a_src, float *__restrict__ a_dst) {
  const int lane = lane_id();
  const int n = blockIdx.x * 4 + wave_in_block();
  if (n >= N) return;
  const float4 *x4 = reinterpret_cast<const float4 *>(x) + (size_t)n * 128;
  const float4 *v4 = reinterpret_cast<const float4 *>(v);
  const float4 xa = x4[lane], xb = x4[64 + lane];
  float r[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) r[w] = f4_dot(xa, v4[w * 128 + lane]) + f4_dot(xb, v4[w * 128 + 64 + lane]);
  transpose_reduce<4>(r, lane);   // lane 0: r0, 16: r1, 32: r2, 48: r3
  const float s0 = readlane_f(r[0], 0), s1 = readlane_f(r[0], 16);
  const float d0 = readlane_f(r[0], 32), d1 = readlane_f(r[0], 48);
  if (lane == 0) {
    *reinterpret_cast<float2 *>(a_src + 2 * (size_t)n) = make_float2(s0, s1);
    *reinterpret_cast<float2 *>(a_dst + 2 * (size_t)n) = make_float2(d0, d1);
  }
}

// ---- own rows: softmax statistics + one gather pass over x_j ---------------------------------
// X4 [2 heads][2 kinds][rows][512]: kind 0 = xa (sum alpha x_j), kind 1 = xa2 (sum alpha lrelu' x_j);
// row i of the launch range is local row i - row_begin.  row_stats (global rows): (max, sum) and S3.
// One row per 4-wave block: wave w takes the row's 64-edge chunks w, w + 4, ... in every pass (max,
// sum, gather); the partial sums meet in LDS and are added in wave order (deterministic).  A rank's
// shard at P = 8 is ~2700 rows: one wave per row left ~2.6 waves per SIMD, each walking ~190 edges
// serially (66 us, profiles/r03g_simprof_xagg_P8_rank0_timeline.txt).
__global__ __launch_bounds__(256) void xagg_fwd_kernel(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                       int row_begin, int row_end, const float *__restrict__ x,
                                                       const float *__restrict__ a_src,
                                                       const float *__restrict__ a_dst, float ns,
                                                       float *__restrict__ X4, float *__restrict__ row_stats) {
  constexpr int U = kXaggU;
  __shared__ float4 part[3][8][64];      // waves 1..3: acc[hd][kd][half] per lane
  __shared__ float red[4][4];            // per wave: (m0, m1) then (s0, s1), then (t0, t1)
  const int lane = lane_id(), wv = wave_in_block();
  const int i = row_begin + xcd_remap(blockIdx.x, gridDim.x);
  if (i >= row_end) return;              // uniform over the block
  const int rows = row_end - row_begin, r = i - row_begin;
  const int beg = rowptr[i], end = rowptr[i + 1];
  const float2 ad = *reinterpret_cast<const float2 *>(a_dst + 2 * (size_t)i);
  const float2 *as2 = reinterpret_cast<const float2 *>(a_src);
  float m0 = -INFINITY, m1 = -INFINITY;
  for (int e = beg + 64 * wv + lane; e < end; e += 256) {
    const float2 s = as2[col[e]];
    m0 = fmaxf(m0, lrelu(s.x + ad.x, ns));
    m1 = fmaxf(m1, lrelu(s.y + ad.y, ns));
  }
  m0 = wave_max(m0);
  m1 = wave_max(m1);
  if (lane == 0) { red[wv][0] = m0; red[wv][1] = m1; }
  __syncthreads();
  m0 = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]));
  m1 = fmaxf(fmaxf(red[0][1], red[1][1]), fmaxf(red[2][1], red[3][1]));
  float s0 = 0.f, s1 = 0.f;
  for (int e = beg + 64 * wv + lane; e < end; e += 256) {
    const float2 s = as2[col[e]];
    s0 += expf(lrelu(s.x + ad.x, ns) - m0);
    s1 += expf(lrelu(s.y + ad.y, ns) - m1);
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if (lane == 0) { red[wv][2] = s0; red[wv][3] = s1; }
  __syncthreads();
  s0 = ((red[0][2] + red[1][2]) + red[2][2]) + red[3][2];
  s1 = ((red[0][3] + red[1][3]) + red[2][3]) + red[3][3];
  const float den0 = s0 + 1e-16f, den1 = s1 + 1e-16f;
  const float4 *x4 = reinterpret_cast<const float4 *>(x);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // [head][kind][half]: head h, kind 0 (alpha) / 1 (alpha lrelu'), columns 4l.. (half 0) / 256+4l.. (1)
  float4 acc[2][2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b][0] = acc[a][b][1] = z4;
  float t0 = 0.f, t1 = 0.f;
  for (int base = beg + 64 * wv; base < end; base += 256) {
    const int e = base + lane;
    int j = i;
    float p0 = 0.f, p1 = 0.f, q0 = 0.f, q1 = 0.f;
    if (e < end) {
      j = col[e];
      const float2 s = as2[j];
      const float e0 = s.x + ad.x, e1 = s.y + ad.y;
      p0 = expf(lrelu(e0, ns) - m0) / den0;
      p1 = expf(lrelu(e1, ns) - m1) / den1;
      q0 = p0 * (e0 > 0.f ? 1.f : ns);
      q1 = p1 * (e1 > 0.f ? 1.f : ns);
      t0 += q0;
      t1 += q1;
    }
    const int cnt = min(64, end - base);
    for (int k = 0; k < cnt; k += U) {
      float4 va[U], vb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t jj = (size_t)readlane_i(j, k + u);   // k + u < 64: U divides 64
        va[u] = x4[jj * 128 + lane];
        vb[u] = x4[jj * 128 + 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {   // slots past the row's end hold weight 0 (the padded lanes)
        const float w00 = readlane_f(p0, k + u), w01 = readlane_f(q0, k + u);
        const float w10 = readlane_f(p1, k + u), w11 = readlane_f(q1, k + u);
        acc[0][0][0] = f4_fma(w00, va[u], acc[0][0][0]);
        acc[0][0][1] = f4_fma(w00, vb[u], acc[0][0][1]);
        acc[0][1][0] = f4_fma(w01, va[u], acc[0][1][0]);
        acc[0][1][1] = f4_fma(w01, vb[u], acc[0][1][1]);
        acc[1][0][0] = f4_fma(w10, va[u], acc[1][0][0]);
        acc[1][0][1] = f4_fma(w10, vb[u], acc[1][0][1]);
        acc[1][1][0] = f4_fma(w11, va[u], acc[1][1][0]);
        acc[1][1][1] = f4_fma(w11, vb[u], acc[1][1][1]);
      }
    }
  }
  t0 = wave_sum(t0);
  t1 = wave_sum(t1);
  if (wv > 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) part[wv - 1][q][lane] = acc[q >> 2][(q >> 1) & 1][q & 1];
    if (lane == 0) { red[wv][0] = t0; red[wv][1] = t1; }
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 v = part[w][q][lane];
      float4 &a = acc[q >> 2][(q >> 1) & 1][q & 1];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  t0 = ((t0 + red[1][0]) + red[2][0]) + red[3][0];
  t1 = ((t1 + red[1][1]) + red[2][1]) + red[3][1];
  float4 *o4 = reinterpret_cast<float4 *>(X4);
#pragma unroll
  for (int hd = 0; hd < 2; ++hd)
#pragma unroll
    for (int kd = 0; kd < 2; ++kd) {
      float4 *dst = o4 + (((size_t)(hd * 2 + kd) * rows + r) * 128);
      dst[lane] = acc[hd][kd][0];
      dst[64 + lane] = acc[hd][kd][1];
    }
  float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
  if (lane == 0) {
    rs4[2 * (size_t)i] = make_float4(m0, m1, s0, s1);
    rs4[2 * (size_t)i + 1] = make_float4(t0, t1, 0.f, 0.f);
  }
}

// ---- y0 += bias; o = relu(y0) (torch.relu: x <= 0 -> 0) over [rows, 512] -----------------------
__global__ __launch_bounds__(256) void xagg_bias_relu_kernel(float *__restrict__ y0, const float *__restrict__ bias,
                                                             float *__restrict__ o, int64_t n4) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n4) return;
  float4 v = reinterpret_cast<float4 *>(y0)[t];
  const float4 b = reinterpret_cast<const float4 *>(bias)[t & 127];
  v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  reinterpret_cast<float4 *>(y0)[t] = v;
  reinterpret_cast<float4 *>(o)[t] = f4_relu(v);
}

// ---- own rows: dout = g [y0 > 0] (relu backward, ACT) or g; delta^h = <dout^h, y0^h - bias^h>; the
// forward's S3 moves to row_stats[6:8] (the edge pass forms da_dst there from it) ------------------
template <int ACT>
__global__ __launch_bounds__(256) void xagg_rows_bwd_kernel(int rows, const float *__restrict__ g,
                                                            const float *__restrict__ y0,
                                                            const float *__restrict__ bias, float *__restrict__ dout,
                                                            float *__restrict__ row_stats) {
  const int lane = lane_id();
  const int r = blockIdx.x * 4 + wave_in_block();
  if (r >= rows) return;
  const size_t o0 = (size_t)r * 128 + lane, o1 = o0 + 64;
  const float4 *g4 = reinterpret_cast<const float4 *>(g);
  const float4 *y4 = reinterpret_cast<const float4 *>(y0);
  const float4 *b4 = reinterpret_cast<const float4 *>(bias);
  float4 d0 = g4[o0], d1 = g4[o1];
  const float4 y0v = y4[o0], y1v = y4[o1], b0 = b4[lane], b1 = b4[64 + lane];
  if (ACT) {
    d0 = make_float4(y0v.x <= 0.f ? 0.f : d0.x, y0v.y <= 0.f ? 0.f : d0.y, y0v.z <= 0.f ? 0.f : d0.z,
                     y0v.w <= 0.f ? 0.f : d0.w);
    d1 = make_float4(y1v.x <= 0.f ? 0.f : d1.x, y1v.y <= 0.f ? 0.f : d1.y, y1v.z <= 0.f ? 0.f : d1.z,
                     y1v.w <= 0.f ? 0.f : d1.w);
  }
  float4 *d4 = reinterpret_cast<float4 *>(dout);
  d4[o0] = d0;
  d4[o1] = d1;
  const float4 e0 = make_float4(y0v.x - b0.x, y0v.y - b0.y, y0v.z - b0.z, y0v.w - b0.w);
  const float4 e1 = make_float4(y1v.x - b1.x, y1v.y - b1.y, y1v.z - b1.z, y1v.w - b1.w);
  float v[2] = {f4_dot(d0, e0), f4_dot(d1, e1)};
  transpose_reduce<2>(v, lane);   // lane 0: head 0, lane 32: head 1
  const float dl0 = readlane_f(v[0], 0), dl1 = readlane_f(v[0], 32);
  if (lane == 0) {
    float4 *rs4 = reinterpret_cast<float4 *>(row_stats);
    const float4 t = rs4[2 * (size_t)r + 1];   // (S3_0, S3_1, -, -) from xagg_fwd
    rs4[2 * (size_t)r + 1] = make_float4(dl0, dl1, t.x, t.y);
  }
}

// ---- own rows: per-edge softmax-gradient terms (the destination pass of the aggregate-first form) --
// dxa [rows][1024] (local rows): head h at columns 512h..; row_stats (global) holds delta at [4:6]
// (xagg_rows_bwd).  ds [nnz_own][2] in the rank's CSR order (rowptr[row_begin] = 0).
// xa2 != NULL (X4's kind-1 planes, local rows; the caller's forward skipped out2): the row's
// da_dst^h = <dxa_i^h, xa2_i^h> - delta_i^h S3_i^h is formed here too, with S3 read from
// row_stats[6:8] (xagg_rows_bwd put it there) and da_dst written over it.
// One row per 4-wave block, the row's dxa (4 KiB) in LDS.  A wave takes 64/GL edges at a time, one
// per GL-lane group: lane t of a group reads float4s t, t + GL, ... of its neighbour's x_j (each load
// instruction is 64/GL row segments of 16 GL bytes, 128/GL loads of a lane in flight) against the LDS
// dxa (the same address in every group: a broadcast), and the two head dots are summed over the GL
// lanes (log2 GL xor-shuffle steps), no 64-lane transposed reduction per 4 edges as in the former
// one-wave-per-row form.  Measured at P = 8 beside the side lanes' dW GEMMs: 111 us (wave per row),
// 100 (GL = 8, dxa kept in 128 VGPRs: 238, 2 waves per SIMD), 112 (GL = 16, 130 VGPRs) -- against
// 64 us for the forward's gather of the same rows alone (profiles/r03h_/r03i_/r03k_simprof_xagg_P8_
// rank0_timeline.txt).  dxa re-read from LDS every pass (100 VGPRs, 4 waves per SIMD): rank 0's
// whole step at P = 2 1.372 ms with GL = 8 against 1.42-1.43 (GL = 16) and 1.448 (GL = 16, dxa in
// VGPRs); even at P = 8 (profiles/r03p_sim_ab_edge.txt).
__global__ __launch_bounds__(256) void xagg_edge_kernel(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                        int row_begin, int row_end, const float *__restrict__ x,
                                                        const float *__restrict__ a_src,
                                                        const float *__restrict__ a_dst,
                                                        float *__restrict__ row_stats,
                                                        const float *__restrict__ dxa, float ns,
                                                        float *__restrict__ ds, const float *__restrict__ xa2) {
  __shared__ float4 dl4[256];          // dxa row: head 0 float4s 0..127, head 1 128..255
  const int lane = lane_id(), wv = wave_in_block();
  const int i = row_begin + xcd_remap(blockIdx.x, gridDim.x);
  if (i >= row_end) return;            // uniform over the block
  const int r = i - row_begin;
  dl4[threadIdx.x] = reinterpret_cast<const float4 *>(dxa)[(size_t)r * 256 + threadIdx.x];
  __syncthreads();
  const int beg = rowptr[i], end = rowptr[i + 1];
  const float4 *x4 = reinterpret_cast<const float4 *>(x);
  const float2 ad = *reinterpret_cast<const float2 *>(a_dst + 2 * (size_t)i);
  const float4 ms = reinterpret_cast<const float4 *>(row_stats)[2 * (size_t)i];       // max0 max1 sum0 sum1
  const float2 dl = *reinterpret_cast<const float2 *>(row_stats + 8 * (size_t)i + 4);  // delta0 delta1
  const float2 *as2 = reinterpret_cast<const float2 *>(a_src);
  constexpr int GL = kXaggGL, NG = 64 / GL, NC = 128 / GL;   // lanes per edge, edges per wave, float4s per lane
  const int g = lane / GL, t = lane % GL;
  for (int e0 = beg + NG * wv; e0 < end; e0 += 4 * NG) {   // wave wv: edges e0 .. e0 + NG - 1 of every 4 NG
    asm volatile("" ::: "memory");   // re-read dxa from LDS each pass: no 64-128 VGPR copy, more waves
    const int e = e0 + g;
    const bool live = e < end;
    const int j = live ? col[e] : i;
    const float4 *xr = x4 + (size_t)j * 128 + t;
    float4 xv[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) xv[c] = xr[GL * c];
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      s0 += f4_dot(xv[c], dl4[t + GL * c]);
      s1 += f4_dot(xv[c], dl4[128 + t + GL * c]);
    }
#pragma unroll
    for (int o = 1; o < GL; o <<= 1) {
      s0 += __shfl_xor(s0, o);
      s1 += __shfl_xor(s1, o);
    }
    if (live && t == 0) {
      const float2 sv = as2[j];
      const float ea = sv.x + ad.x, eb = sv.y + ad.y;
      const float al0 = expf(lrelu(ea, ns) - ms.x) / (ms.z + 1e-16f);
      const float al1 = expf(lrelu(eb, ns) - ms.y) / (ms.w + 1e-16f);
      const float alp0 = al0 * (ea > 0.f ? 1.f : ns), alp1 = al1 * (eb > 0.f ? 1.f : ns);
      reinterpret_cast<float2 *>(ds)[e] = make_float2(alp0 * (s0 - dl.x), alp1 * (s1 - dl.y));
    }
  }
  if (xa2 && wv == 0) {
    const int rows = row_end - row_begin;
    const float4 *q0 = reinterpret_cast<const float4 *>(xa2) + (size_t)r * 128;                     // head 0
    const float4 *q1 = reinterpret_cast<const float4 *>(xa2) + ((size_t)2 * rows + r) * 128;         // head 1
    float v[2] = {f4_dot(dl4[lane], q0[lane]) + f4_dot(dl4[64 + lane], q0[64 + lane]),
                  f4_dot(dl4[128 + lane], q1[lane]) + f4_dot(dl4[192 + lane], q1[64 + lane])};
    transpose_reduce<2>(v, lane);
    const float p0 = readlane_f(v[0], 0), p1 = readlane_f(v[0], 32);
    if (lane == 0) {
      const float2 s3 = *reinterpret_cast<const float2 *>(row_stats + 8 * (size_t)i + 6);
      *reinterpret_cast<float2 *>(row_stats + 8 * (size_t)i + 6) = make_float2(fmaf(-dl.x, s3.x, p0), fmaf(-dl.y, s3.y, p1));
    }
  }
}

// ---- own rows, the edge pass with the source-side sum folded in (no slab pass) ----------------------
// The source side enters the parameters only through g_src^h = sum_j da_src_j^h x_j, and
// da_src_j = sum over the rank's edges (i, j) of ds_ij, so g_src^h = sum_i sum_j ds_ij^h x_j: the
// edge pass that forms ds_ij has x_j in registers and adds ds_ij^h x_j into the block's running sum
// -- no per-edge ds array, no transposed (slab) structure, no second gather.
// Workgroup b (XCD-aware map) takes own rows [b R / G, (b+1) R / G) in order (G = rows / RPB: a
// persistent grid of 512 workgroups -- 2 per CU, 2 waves per SIMD -- left the gathers latency-bound);
// per row its dxa (4 KiB) goes to LDS; 16-lane groups take the row's edges g, g + 16, ... (lane t of a
// group holds float4 t, t + 16, ..., t + 112 of x_j); the two head dots are summed over the group by
// DPP (sum16), then y^h += ds^h x_j per lane (64 accumulators).  At the end the 16 group sums are
// added in fixed order (xor 16, xor 32 within a wave, then the 4 waves in order through LDS) into the
// block's partial row gpart[b][0:1024] (head 0 | head 1); their column sum (a grouped column-sum job,
// hicgat_param_grads_grouped) is g_src.  With xa2 the row's da_dst is formed as in xagg_edge_kernel.
template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float v) {   // every lane of a 16-lane DPP row: the row's sum
  v += dpp_row<0x128>(v);   // row_ror:8
  v += dpp_row<0x124>(v);   // row_ror:4
  v += dpp_row<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_row<0xB1>(v);    // quad_perm [1,0,3,2]
  return v;
}
// v of lane k of this lane's 16-lane DPP row (DPP row_share, gfx90a+: one VALU op); k is uniform
template <int K>
__device__ __forceinline__ int row_share_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xF, 0xF, false);
}
template <int K>
__device__ __forceinline__ float row_share_f(float v) {
  return __int_as_float(row_share_i<K>(__float_as_int(v)));
}
// (j, q0, q1) of edges k .. k + U - 1 of the group's chunk (k a multiple of U, < 16; a slot past the
// row's end has q = 0 and j = the row itself, so it adds nothing)
constexpr int EU = 2;   // edges per group per step of the edge pass (neighbour rows in flight)
template <int U>
__device__ __forceinline__ void row_share_n(int k, int j, float q0, float q1, int (&jj)[U], float (&qq0)[U],
                                            float (&qq1)[U]) {
  switch (k) {
#define HICGAT_RS1(K, u)                                                        \
  jj[u] = row_share_i<((K) + (u)) & 15>(j);                                     \
  qq0[u] = row_share_f<((K) + (u)) & 15>(q0);                                   \
  qq1[u] = row_share_f<((K) + (u)) & 15>(q1);
#define HICGAT_RSN(K)                                                           \
  case K:                                                                       \
    HICGAT_RS1(K, 0)                                                            \
    if constexpr (U > 1) { HICGAT_RS1(K, 1) }                                   \
    if constexpr (U > 2) { HICGAT_RS1(K, 2) HICGAT_RS1(K, 3) }                  \
    break;
    HICGAT_RSN(0) HICGAT_RSN(1) HICGAT_RSN(2) HICGAT_RSN(3) HICGAT_RSN(4) HICGAT_RSN(5) HICGAT_RSN(6)
    HICGAT_RSN(7) HICGAT_RSN(8) HICGAT_RSN(9) HICGAT_RSN(10) HICGAT_RSN(11) HICGAT_RSN(12) HICGAT_RSN(13)
    HICGAT_RSN(14)
    default: HICGAT_RSN(15)
#undef HICGAT_RSN
#undef HICGAT_RS1
  }
}
constexpr int kEdgeRPB = 2;   // own rows per workgroup of the edge pass (= partial rows of g_src: rows / RPB)
__host__ __device__ inline int edge_acc_blocks(int rows) { return rows <= 0 ? 1 : (rows + kEdgeRPB - 1) / kEdgeRPB; }
__global__ __launch_bounds__(256) void xagg_edge_acc_kernel(const int *__restrict__ rowptr,
                                                            const int *__restrict__ col, int row_begin,
                                                            int row_end, const float *__restrict__ x,
                                                            const float *__restrict__ a_src,
                                                            const float *__restrict__ a_dst,
                                                            float *__restrict__ row_stats,
                                                            const float *__restrict__ dxa, float ns,
                                                            const float *__restrict__ xa2,
                                                            float *__restrict__ gpart) {
  __shared__ float4 dl4[256];          // dxa row: head 0 float4s 0..127, head 1 128..255
  __shared__ float4 wred[3][256];      // waves 1..3: their group sums (float4 q of head h at [h*128 + q])
  const int lane = lane_id(), wv = wave_in_block();
  const int g = wv * 4 + (lane >> 4), t = lane & 15;   // 16 groups per block
  const int rows = row_end - row_begin, G = gridDim.x;
  const int b = xcd_remap(blockIdx.x, G);
  const int rb = (int)((int64_t)rows * b / G), re = (int)((int64_t)rows * (b + 1) / G);
  const float4 *x4 = reinterpret_cast<const float4 *>(x);
  const float2 *as2 = reinterpret_cast<const float2 *>(a_src);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 y0[8], y1[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) y0[c] = y1[c] = z4;
  for (int r = rb; r < re; ++r) {
    const int i = row_begin + r;
    __syncthreads();                                   // the previous row's dl4 readers are done
    dl4[threadIdx.x] = reinterpret_cast<const float4 *>(dxa)[(size_t)r * 256 + threadIdx.x];
    __syncthreads();
    const int beg = rowptr[i], end = rowptr[i + 1];
    const float2 ad = *reinterpret_cast<const float2 *>(a_dst + 2 * (size_t)i);
    const float4 ms = reinterpret_cast<const float4 *>(row_stats)[2 * (size_t)i];       // max0 max1 sum0 sum1
    const float2 dl = *reinterpret_cast<const float2 *>(row_stats + 8 * (size_t)i + 4);  // delta0 delta1
    const float den0 = ms.z + 1e-16f, den1 = ms.w + 1e-16f;
    // the row's edges in chunks of 256: group g takes edges beg + 256 c + g + 16 k (k < 16); lane t
    // of the group first computes, for ITS edge k = t, the neighbour j and the two softmax-gradient
    // weights q = alpha lrelu' (one col / a_src load per lane, all in flight together), then the group
    // walks k with j, q broadcast from lane k of its DPP row (row_share: one VALU op), two edges per
    // step so two neighbour rows are in flight; ds = q (<dxa, x_j> - delta).
    for (int cb = beg; cb < end; cb += 256) {
      const int et = cb + g + 16 * t;
      const bool lv = et < end;
      const int jt = lv ? col[et] : i;
      float q0t = 0.f, q1t = 0.f;
      if (lv) {
        const float2 sv = as2[jt];
        const float ea = sv.x + ad.x, eb = sv.y + ad.y;
        q0t = expf(lrelu(ea, ns) - ms.x) / den0 * (ea > 0.f ? 1.f : ns);
        q1t = expf(lrelu(eb, ns) - ms.y) / den1 * (eb > 0.f ? 1.f : ns);
      }
      // edges of this chunk for the wave's first group (the most of its four): a wave-uniform bound
      const int kmax = min(16, (end - cb - 4 * wv + 15) / 16);
#pragma unroll 1
      for (int k = 0; k < kmax; k += EU) {
        asm volatile("" ::: "memory");   // dxa re-read from LDS every step: no 128-VGPR copy, more waves
        int jj[EU];
        float qq0[EU], qq1[EU];
        row_share_n<EU>(k, jt, q0t, q1t, jj, qq0, qq1);
        float4 v[EU][8];
#pragma unroll
        for (int u = 0; u < EU; ++u) {
          const float4 *xr = x4 + (size_t)jj[u] * 128 + t;
#pragma unroll
          for (int c = 0; c < 8; ++c) v[u][c] = xr[16 * c];
        }
        float s0[EU], s1[EU];
#pragma unroll
        for (int u = 0; u < EU; ++u) s0[u] = s1[u] = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float4 d0 = dl4[t + 16 * c], d1 = dl4[128 + t + 16 * c];
#pragma unroll
          for (int u = 0; u < EU; ++u) {
            s0[u] += f4_dot(v[u][c], d0);
            s1[u] += f4_dot(v[u][c], d1);
          }
        }
#pragma unroll
        for (int u = 0; u < EU; ++u) {
          const float ds0 = qq0[u] * (row_sum16(s0[u]) - dl.x), ds1 = qq1[u] * (row_sum16(s1[u]) - dl.y);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            y0[c] = f4_fma(ds0, v[u][c], y0[c]);
            y1[c] = f4_fma(ds1, v[u][c], y1[c]);
          }
        }
      }
    }
    if (xa2 && wv == 0) {
      const float4 *q0 = reinterpret_cast<const float4 *>(xa2) + (size_t)r * 128;                     // head 0
      const float4 *q1 = reinterpret_cast<const float4 *>(xa2) + ((size_t)2 * rows + r) * 128;         // head 1
      float v[2] = {f4_dot(dl4[lane], q0[lane]) + f4_dot(dl4[64 + lane], q0[64 + lane]),
                    f4_dot(dl4[128 + lane], q1[lane]) + f4_dot(dl4[192 + lane], q1[64 + lane])};
      transpose_reduce<2>(v, lane);
      const float p0 = readlane_f(v[0], 0), p1 = readlane_f(v[0], 32);
      if (lane == 0) {
        const float2 s3 = *reinterpret_cast<const float2 *>(row_stats + 8 * (size_t)i + 6);
        *reinterpret_cast<float2 *>(row_stats + 8 * (size_t)i + 6) = make_float2(fmaf(-dl.x, s3.x, p0), fmaf(-dl.y, s3.y, p1));
      }
    }
  }
  // the 4 groups of a wave (its 4 DPP rows), lanes t of rows 0..3: (0 + 1) + (2 + 3)
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float *a = reinterpret_cast<float *>(&y0[c]), *bq = reinterpret_cast<float *>(&y1[c]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] += __shfl_xor(a[k], 16);
      a[k] += __shfl_xor(a[k], 32);
      bq[k] += __shfl_xor(bq[k], 16);
      bq[k] += __shfl_xor(bq[k], 32);
    }
  }
  __syncthreads();
  if (wv > 0 && lane < 16) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      wred[wv - 1][t + 16 * c] = y0[c];
      wred[wv - 1][128 + t + 16 * c] = y1[c];
    }
  }
  __syncthreads();
  if (wv == 0 && lane < 16) {
    float4 *o = reinterpret_cast<float4 *>(gpart) + (size_t)blockIdx.x * 256;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float4 a = y0[c], bq = y1[c];
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        const float4 u = wred[w][t + 16 * c], v = wred[w][128 + t + 16 * c];
        a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
        bq.x += v.x; bq.y += v.y; bq.z += v.z; bq.w += v.w;
      }
      o[t + 16 * c] = a;
      o[128 + t + 16 * c] = bq;
    }
  }
}

// ---- every row j: da_src_j = sum over the slab entries (j, i) of ds at the rank's edge (i, j), and
// g_src^h += da_src_j^h x_j: persistent waves, each taking 4 rows at a time (rows 4w .. 4w + 3, then
// + 4W): 16-lane group q sums row 4w + q's entries (float2, 4 xor-shuffle steps), then the four x_j
// rows (8 columns per lane) go into the wave's two 512-column partial rows in row order; part
// [W][2][512] is summed in wave order by xagg_colred_kernel (no atomics).  Four rows per pass
// overlap their rowptr -> perm -> ds load chains (one row per pass: ~20 rows x 3 dependent loads per
// wave, 31-46 us at P = 8, profiles/r03h_simprof_xagg_P8_rank0_timeline.txt). ------------------------------------
constexpr int kSlabWaves = 1024;   // partial rows of g_src (256 workgroups x 4 waves)
__global__ __launch_bounds__(256) void xagg_slab_sum_kernel(const int *__restrict__ rowptr_s,
                                                            const int *__restrict__ perm, int N,
                                                            const float *__restrict__ ds,
                                                            const float *__restrict__ x,
                                                            float *__restrict__ da_src, float *__restrict__ part) {
  const int lane = lane_id();
  const int w = blockIdx.x * 4 + wave_in_block(), W = gridDim.x * 4;
  const int q = lane >> 4, t = lane & 15;
  const float2 *ds2 = reinterpret_cast<const float2 *>(ds);
  const float4 *x4 = reinterpret_cast<const float4 *>(x);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 g00 = z4, g01 = z4, g10 = z4, g11 = z4;   // head 0 / 1, columns 4l.. / 256+4l..
  for (int j0 = 4 * w; j0 < N; j0 += 4 * W) {
    const int j = j0 + q;
    float a = 0.f, b = 0.f;
    if (j < N) {
      const int k1 = rowptr_s[j + 1];
      for (int k = rowptr_s[j] + t; k < k1; k += 16) {
        const float2 v = ds2[perm[k]];
        a += v.x;
        b += v.y;
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      a += __shfl_xor(a, o);
      b += __shfl_xor(b, o);
    }
    if (t == 0 && j < N) reinterpret_cast<float2 *>(da_src)[j] = make_float2(a, b);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int jj = j0 + u;
      if (jj >= N) break;
      const float au = __shfl(a, 16 * u), bu = __shfl(b, 16 * u);
      const float4 xa = x4[(size_t)jj * 128 + lane], xb = x4[(size_t)jj * 128 + 64 + lane];
      g00 = f4_fma(au, xa, g00);
      g01 = f4_fma(au, xb, g01);
      g10 = f4_fma(bu, xa, g10);
      g11 = f4_fma(bu, xb, g11);
    }
  }
  float4 *p4 = reinterpret_cast<float4 *>(part) + (size_t)w * 256;
  p4[lane] = g00;
  p4[64 + lane] = g01;
  p4[128 + lane] = g10;
  p4[192 + lane] = g11;
}

// out[c] = sum_w part[w][c] over the kSlabWaves partial rows, c < 1024: block = 16 columns x 16
// groups, group q adds w = q, q + 16, ... with its loads in flight, groups combined in order.
__global__ __launch_bounds__(256) void xagg_colred_kernel(const float *__restrict__ part, int nw, float *__restrict__ out) {
  __shared__ float red[16][16];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  constexpr int kMax = kSlabWaves / 16;
  float v[kMax];
#pragma unroll
  for (int t = 0; t < kMax; ++t) {
    const int w = grp + 16 * t;
    v[t] = w < nw ? part[(size_t)w * 1024 + c] : 0.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int t = 0; t < kMax; ++t) acc += v[t];
  red[grp][cl] = acc;
  __syncthreads();
  if (grp == 0) {
    float tsum = red[0][cl];
#pragma unroll
    for (int q = 1; q < 16; ++q) tsum += red[q][cl];
    out[c] = tsum;
  }
}

// ---- dW[w, :] += att_src[w] g_src[h, :] + att_dst[w] g_dst[h, :]; datt[w] += <W[w, :], g[h, :]> -----
// one block per row w = 256 h + c of W (512 rows), 256 threads over its 512 columns
// g in `segs` segments (seg_stride floats apart), added in segment order
__global__ __launch_bounds__(256) void xagg_param_finish_kernel(const float *__restrict__ W,
                                                                const float *__restrict__ att_s,
                                                                const float *__restrict__ att_d,
                                                                const float *__restrict__ g_src,
                                                                const float *__restrict__ g_dst,
                                                                float *__restrict__ dW, float *__restrict__ datt_s,
                                                                float *__restrict__ datt_d, int segs,
                                                                int64_t seg_stride) {
  __shared__ float red[2][4];
  const int w = blockIdx.x, hd = w >> 8, t = threadIdx.x;
  const float as = att_s[w], adv = att_d[w];
  float ps = 0.f, pd = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = q * 256 + t;
    float gs = g_src[hd * 512 + k], gd = g_dst[hd * 512 + k];
    for (int sg = 1; sg < segs; ++sg) {
      gs += g_src[sg * seg_stride + hd * 512 + k];
      gd += g_dst[sg * seg_stride + hd * 512 + k];
    }
    const float wk = W[(size_t)w * 512 + k];
    dW[(size_t)w * 512 + k] += fmaf(as, gs, adv * gd);
    ps = fmaf(wk, gs, ps);
    pd = fmaf(wk, gd, pd);
  }
  ps = wave_sum(ps);
  pd = wave_sum(pd);
  if (lane_id() == 0) {
    red[0][t >> 6] = ps;
    red[1][t >> 6] = pd;
  }
  __syncthreads();
  if (t == 0) {
    datt_s[w] += ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    datt_d[w] += ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  }
}

}  // namespace hicgat

using namespace hicgat;

extern "C" size_t hicgat_xagg_vec_bytes(void) { return 4 * 512 * sizeof(float); }

extern "C" int hicgat_xagg_logits_zero_pack(const float *x, const float *W, const float *att_src,
                                            const float *att_dst, int N, int F, int H, int C, float *vec,
                                            float *a_src, float *a_dst, float *zero_buf, int64_t zero_n,
                                            int64_t *step_counter, const float *W1c, const float *W2c, void *pack,
                                            size_t pack_bytes, hicgat_stream_t stream) {
  if (N < 0 || zero_n < 0) return HICGAT_EINVAL;
  if (F != 512 || H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (!W || !att_src || !att_dst || !vec || (zero_n > 0 && !zero_buf)) return HICGAT_EINVAL;
  if (zero_buf && (reinterpret_cast<uintptr_t>(zero_buf) & 15)) return HICGAT_EINVAL;
  PackJobs pj{};
  int nb = 0;
  if (pack) {   // the heads form's pack: Wh is lin_l's weight W itself
    nb = pack_jobs(W1c, W2c, W, pack, pack_bytes, pj);
    if (nb < 0) return nb;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(xagg_vec_kernel, dim3(32 + nb), dim3(256), 0, s, W, att_src, att_dst, vec,
                     zero_n > 0 ? zero_buf : nullptr, zero_n, step_counter, pj);
  HICGAT_CHECK_LAUNCH();
  if (pack) pack_note(pack, true);
  if (N == 0) return HICGAT_OK;
  if (!x || !a_src || !a_dst) return HICGAT_EINVAL;
  hipLaunchKernelGGL(xagg_logits_kernel, dim3((N + 3) / 4), dim3(256), 0, s, x, vec, N, a_src, a_dst);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_xagg_logits_zero(const float *x, const float *W, const float *att_src, const float *att_dst,
                                       int N, int F, int H, int C, float *vec, float *a_src, float *a_dst,
                                       float *zero_buf, int64_t zero_n, int64_t *step_counter,
                                       hicgat_stream_t stream) {
  return hicgat_xagg_logits_zero_pack(x, W, att_src, att_dst, N, F, H, C, vec, a_src, a_dst, zero_buf, zero_n,
                                      step_counter, nullptr, nullptr, nullptr, 0, stream);
}

extern "C" int hicgat_xagg_logits(const float *x, const float *W, const float *att_src, const float *att_dst, int N,
                                  int F, int H, int C, float *vec, float *a_src, float *a_dst,
                                  hicgat_stream_t stream) {
  return hicgat_xagg_logits_zero(x, W, att_src, att_dst, N, F, H, C, vec, a_src, a_dst, nullptr, 0, nullptr, stream);
}

extern "C" int hicgat_xagg_fwd(const int32_t *rowptr, const int32_t *col, int N, int F, int H, int C, int row_begin,
                               int row_end, const float *x, const float *a_src, const float *a_dst, float neg_slope,
                               float *X4, float *row_stats, hicgat_stream_t stream) {
  if (N < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (F != 512 || H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !x || !a_src || !a_dst || !X4 || !row_stats) return HICGAT_EINVAL;
  hipLaunchKernelGGL(xagg_fwd_kernel, dim3(row_end - row_begin), dim3(256), 0, (hipStream_t)stream, rowptr,
                     col, row_begin, row_end, x, a_src, a_dst, neg_slope, X4, row_stats);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_xagg_bias_relu(float *y0, const float *bias, float *o, int rows, int D,
                                     hicgat_stream_t stream) {
  if (rows < 0 || D != 512) return D != 512 ? HICGAT_EUNSUPPORTED : HICGAT_EINVAL;
  if (rows == 0) return HICGAT_OK;
  if (!y0 || !bias || !o) return HICGAT_EINVAL;
  const int64_t n4 = (int64_t)rows * D / 4;
  hipLaunchKernelGGL(xagg_bias_relu_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, y0,
                     bias, o, n4);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_xagg_rows_bwd(int rows, int D, int act, const float *g, const float *y0, const float *bias,
                                    float *dout, float *row_stats, hicgat_stream_t stream) {
  if (rows < 0 || (act != 0 && act != 1)) return HICGAT_EINVAL;
  if (D != 512) return HICGAT_EUNSUPPORTED;
  if (rows == 0) return HICGAT_OK;
  if (!g || !y0 || !bias || !dout || !row_stats) return HICGAT_EINVAL;
  if (act)
    hipLaunchKernelGGL(xagg_rows_bwd_kernel<1>, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, rows, g, y0,
                       bias, dout, row_stats);
  else
    hipLaunchKernelGGL(xagg_rows_bwd_kernel<0>, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, rows, g, y0,
                       bias, dout, row_stats);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_xagg_edge(const int32_t *rowptr, const int32_t *col, int N, int F, int H, int C, int row_begin,
                                int row_end, const float *x, const float *a_src, const float *a_dst, float *row_stats,
                                const float *dxa, const float *xa2, float neg_slope, float *ds,
                                hicgat_stream_t stream) {
  if (N < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (F != 512 || H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  if (!rowptr || !col || !x || !a_src || !a_dst || !row_stats || !dxa || !ds) return HICGAT_EINVAL;
  hipLaunchKernelGGL(xagg_edge_kernel, dim3(row_end - row_begin), dim3(256), 0, (hipStream_t)stream, rowptr,
                     col, row_begin, row_end, x, a_src, a_dst, row_stats, dxa, neg_slope, ds, xa2);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_xagg_edge_acc_blocks(int rows) { return edge_acc_blocks(rows); }

extern "C" int hicgat_xagg_edge_acc(const int32_t *rowptr, const int32_t *col, int N, int F, int H, int C,
                                    int row_begin, int row_end, const float *x, const float *a_src,
                                    const float *a_dst, float *row_stats, const float *dxa, const float *xa2,
                                    float neg_slope, float *gpart, hicgat_stream_t stream) {
  if (N < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (F != 512 || H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (!rowptr || !col || !x || !a_src || !a_dst || !row_stats || !dxa || !gpart) return HICGAT_EINVAL;
  // rows == 0 still writes the (zero) partial rows: the column sum that follows reads all of them
  hipLaunchKernelGGL(xagg_edge_acc_kernel, dim3(edge_acc_blocks(row_end - row_begin)), dim3(256), 0,
                     (hipStream_t)stream, rowptr, col,
                     row_begin, row_end, x, a_src, a_dst, row_stats, dxa, neg_slope, xa2, gpart);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" size_t hicgat_xagg_slab_workspace_bytes(void) { return (size_t)kSlabWaves * 1024 * sizeof(float); }

extern "C" int hicgat_xagg_slab_sum(const int32_t *rowptr_s, const int32_t *perm, int N, const float *ds,
                                    const float *x, float *da_src, float *g_src, void *workspace,
                                    size_t workspace_bytes, hicgat_stream_t stream) {
  if (N < 0) return HICGAT_EINVAL;
  if (!rowptr_s || !perm || !ds || !x || !da_src || !g_src || !workspace) return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_xagg_slab_workspace_bytes()) return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float *part = static_cast<float *>(workspace);
  hipLaunchKernelGGL(xagg_slab_sum_kernel, dim3(kSlabWaves / 4), dim3(256), 0, s, rowptr_s, perm, N, ds, x, da_src,
                     part);
  HICGAT_CHECK_LAUNCH();
  hipLaunchKernelGGL(xagg_colred_kernel, dim3(1024 / 16), dim3(256), 0, s, part, kSlabWaves, g_src);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_xagg_param_finish(const float *W, const float *att_src, const float *att_dst, const float *g_src,
                                        const float *g_dst, int F, int H, int C, float *dW, float *datt_src,
                                        float *datt_dst, hicgat_stream_t stream) {
  if (F != 512 || H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (!W || !att_src || !att_dst || !g_src || !g_dst || !dW || !datt_src || !datt_dst) return HICGAT_EINVAL;
  hipLaunchKernelGGL(xagg_param_finish_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, W, att_src, att_dst,
                     g_src, g_dst, dW, datt_src, datt_dst, 1, (int64_t)0);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_xagg_param_finish_seg(const float *W, const float *att_src, const float *att_dst,
                                            const float *g_src, const float *g_dst, int segs, int64_t seg_stride,
                                            int F, int H, int C, float *dW, float *datt_src, float *datt_dst,
                                            hicgat_stream_t stream) {
  if (F != 512 || H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (!W || !att_src || !att_dst || !g_src || !g_dst || !dW || !datt_src || !datt_dst) return HICGAT_EINVAL;
  if (segs < 1 || (segs > 1 && seg_stride < 1024)) return HICGAT_EINVAL;
  hipLaunchKernelGGL(xagg_param_finish_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, W, att_src, att_dst,
                     g_src, g_dst, dW, datt_src, datt_dst, segs, seg_stride);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
