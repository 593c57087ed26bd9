// GATConv aggregation (a4+a5) and its source-side backward with the dense part of the contact graph
// on the matrix cores.
//
// Reference: the same ops as gat_fwd.hip / gat_bwd.hip (PyG 1.7.2 GATConv.propagate + softmax + the
// autograd of models.py:634-662).  A Hi-C contact graph is dense near the diagonal (every locus
// touches its genomic neighbours; synth-20000 keeps the first ~12 diagonals whole and |i-j|^-1 of the
// rest): 52 % of its 4.0 M edges lie in the 8.7 k 32x32 tiles holding >= 64 edges.  The gather form
// reads a whole 2 KiB neighbour row per edge from L2 and sits at the L2->CU gather ceiling
// (DESIGN.md section 3); inside a dense tile the same 32 neighbour rows serve 32 destination rows,
// so those edges become a dense 32x32 x 32x512 product per tile, A = the tile's softmax weights
// (0 off the edge set), on v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulation).
//
// Split of one aggregation (rows [row_begin, row_end) in blocks of 32, block b = rows row_begin+32b..):
//   * tiles: tptr [nrb+1] / tcol [ntiles] (32-column block index) / tmask [ntiles*32] (bit c of word
//     32t+i: edge (row 32b+i, column 32 tcol[t] + c)) -- the row blocks' dense tiles;
//   * rowptr_s / col_s: the CSR of every other edge (the sparse remainder, CSR order kept).
// Forward: the gather kernel (SPLIT form, gat_fwd.hip) computes each row's softmax statistics over
// ALL its edges, gathers only the remainder and writes raw sums; band_fwd_kernel adds the tiles'
// products and applies bias / relu.  Backward source pass: the gather kernel (SPLIT, gat_bwd.hip)
// writes the remainder's raw dh and da_src shares; band_bwd_kernel adds the tiles' products and
// finishes dh (logit terms) and da_src.  The graph is symmetric (to_symmetric, utils.py:71), so the
// tiles of a row block are also the tiles of the transposed product the backward needs.
//
// Wave w of a 4-wave workgroup owns columns [128w, 128w+128) of head w/2 for the block's 32 rows.
// B operand = neighbour rows read straight from L2: lane (n = lane&31, k = lane>>5) loads the float4
// at columns 128w + 4n .. 4n+3 of neighbour k of a k-pair, and component t feeds the MFMA of output
// chunk t -- so chunk t's column n is feature 128w + 4n + t and the epilogue stores float4s.
#include "common.hpp"

namespace hicgat {

typedef float f32x16 __attribute__((ext_vector_type(16)));

int agg_fwd_split_launch(const int *rowptr, const int *col, const int *rowptr_s, const int *col_s, int row_begin,
                         int row_end, const float *h, const float *a_src, const float *a_dst, float ns, float *out,
                         float *out2, float *row_stats, hipStream_t s);   // gat_fwd.hip
int agg_bwd_src_split_launch(const int *rowptr_s, const int *col_s, int row_begin, int row_end, const float *h,
                             const float *a_src, const float *a_dst, const float *row_stats, int64_t ldr,
                             const float *dout, int64_t ldq4, float ns, float *dh, float *da_src,
                             hipStream_t s);   // gat_bwd.hip

__device__ __forceinline__ float f4_c(const float4 &v, int t) { return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w; }

// row of accumulator element r (C/D layout of a 32x32 f32 tile: col = lane & 31)
__device__ __forceinline__ int acc_row(int r, int lk) { return (r & 3) + 8 * (r >> 2) + 4 * lk; }

constexpr int KB = 8;    // k-pairs of neighbour rows loaded per batch (two batches per 32-column tile)
constexpr int KBB = 4;   // the same for the backward (four more per-column constants live)
static_assert(16 % KB == 0 && 16 % KBB == 0, "KB / KBB must divide 16");

constexpr int kBandOcc = 2;   // min workgroups per CU (accumulators + one tile of B operands fit 2 waves/SIMD)

// ---- forward: out_i += sum over the block's dense tiles of alpha_ij h_j (and out2 with alpha lrelu'),
// then the epilogue (bias, relu) for every row of the block.  out/out2 hold the gather kernel's raw
// sums on entry; row_stats holds (max, sum) over the whole row and S3 of the remainder.
template <bool TRAIN, int ACT>
__global__ __launch_bounds__(256, kBandOcc) void band_fwd_kernel(
    const int *__restrict__ tptr, const int *__restrict__ tcol, const uint32_t *__restrict__ tmask, int row_begin,
    int row_end, int ncols, const float *__restrict__ h, const float *__restrict__ a_src,
    const float *__restrict__ a_dst, const float *__restrict__ bias, float ns, float *__restrict__ out,
    float *__restrict__ out2, float *__restrict__ row_stats, int splits, float *__restrict__ ws) {
  const int lane = lane_id(), w = wave_in_block();
  const int sp = blockIdx.y;   // tile split: this workgroup takes tiles tb + sp, tb + sp + splits, ...
  const int li = lane & 31, lk = lane >> 5;
  const int rb = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = row_begin + rb * 32;
  const int hd = w >> 1, q0 = 32 * w;   // head; first float4 column of this wave
  const float4 *h4 = reinterpret_cast<const float4 *>(h);

  // A-operand row constants: row r0 + li
  const int ri = r0 + li;
  const bool rvalid = ri < row_end;
  float adst = 0.f, m = 0.f, den = 1.f;
  if (rvalid) {
    adst = a_dst[2 * (size_t)ri + hd];
    const float4 st = reinterpret_cast<const float4 *>(row_stats)[2 * (size_t)ri];
    m = hd ? st.y : st.x;
    den = (hd ? st.w : st.z) + 1e-16f;
  }

  f32x16 acc[4], acs[4];
  float4 *o4 = reinterpret_cast<float4 *>(out);
  float4 *p4 = reinterpret_cast<float4 *>(out2);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = r0 + acc_row(r, lk);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f), u = v;
    if (splits == 1 && row < row_end) {   // split form: the epilogue kernel adds the gather's sums
      v = o4[(size_t)row * 128 + q0 + li];
      if (TRAIN) u = p4[(size_t)row * 128 + q0 + li];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t][r] = f4_c(v, t);
      acs[t][r] = f4_c(u, t);
    }
  }

  float s3 = 0.f;
  const int tb = tptr[rb], te = tptr[rb + 1];
  for (int tt = tb + sp; tt < te; tt += splits) {
    const int cbase = 32 * tcol[tt];
    const uint32_t mk = tmask[(size_t)tt * 32 + li];
    const int cj = cbase + li;
    const float asj = cj < ncols ? a_src[2 * (size_t)cj + hd] : 0.f;
#pragma unroll
    for (int half = 0; half < 16 / KB; ++half) {
    float4 hb[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int j = min(cbase + 2 * (half * KB + u) + lk, ncols - 1);   // past the last row: weight 0, any valid row
      hb[u] = h4[(size_t)j * 128 + q0 + li];
    }
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int kp = half * KB + u;
      const int kc = 2 * kp + lk;
      const float as = __shfl(asj, kc);
      const float e = as + adst;
      const bool on = rvalid && ((mk >> kc) & 1u);
      const float p = on ? expf(lrelu(e, ns) - m) / den : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(p, f4_c(hb[u], t), acc[t], 0, 0, 0);
      if (TRAIN) {
        const float q = p * (e > 0.f ? 1.f : ns);
        s3 += q;
#pragma unroll
        for (int t = 0; t < 4; ++t) acs[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(q, f4_c(hb[u], t), acs[t], 0, 0, 0);
      }
    }
    }
  }

  if (splits > 1) {   // raw partial sums of this split -> workspace (band_fwd_epilogue adds them)
    const int64_t R = row_end - row_begin;
    float4 *wa = reinterpret_cast<float4 *>(ws) + ((int64_t)sp * R - row_begin) * 128;
    float4 *wq = reinterpret_cast<float4 *>(ws) + ((int64_t)(splits + sp) * R - row_begin) * 128;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = r0 + acc_row(r, lk);
      if (row < row_end) {
        wa[(size_t)row * 128 + q0 + li] = make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
        if (TRAIN) wq[(size_t)row * 128 + q0 + li] = make_float4(acs[0][r], acs[1][r], acs[2][r], acs[3][r]);
      }
    }
    if (TRAIN) {
      s3 += __shfl_xor(s3, 32);
      float *w3 = ws + (size_t)2 * splits * R * 512 + ((int64_t)sp * R - row_begin) * 2;
      if ((w & 1) == 0 && lk == 0 && rvalid) w3[2 * (size_t)ri + hd] = s3;
    }
    return;
  }
  const float4 b = reinterpret_cast<const float4 *>(bias)[q0 + li];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = r0 + acc_row(r, lk);
    if (row < row_end) {
      float4 v = make_float4(acc[0][r] + b.x, acc[1][r] + b.y, acc[2][r] + b.z, acc[3][r] + b.w);
      if (ACT == 1) v = f4_relu(v);
      o4[(size_t)row * 128 + q0 + li] = v;
      if (TRAIN) p4[(size_t)row * 128 + q0 + li] = make_float4(acs[0][r], acs[1][r], acs[2][r], acs[3][r]);
    }
  }
  if (TRAIN) {
    // S3 of the tiles' edges: lanes li and li + 32 saw the two halves of row li's k-pairs
    s3 += __shfl_xor(s3, 32);
    if ((w & 1) == 0 && lk == 0 && rvalid) row_stats[8 * (size_t)ri + 4 + hd] += s3;
  }
}

// ---- backward, source side: for source row r of the block,
//   dh_r     += sum over the tiles of alpha_ir dout_i,   c_r = sum alpha_ir s_ir dout_i,
//   sb_r      = sum alpha_ir s_ir delta_i   (the same tiles, VALU),
//   da_src_r  = (remainder share on entry) + <c_r, h_r> - sb_r,
//   dh_r     += da_src_r att_src + da_dst_r att_dst.
// alpha_ir is the softmax weight of edge (i -> r) in destination row i's softmax, so the per-column
// constants (a_dst_i, max_i, sum_i, delta_i) come from row_stats rows of the tile's columns.
__global__ __launch_bounds__(256, kBandOcc) void band_bwd_kernel(
    const int *__restrict__ tptr, const int *__restrict__ tcol, const uint32_t *__restrict__ tmask, int row_begin,
    int row_end, int ncols, const float *__restrict__ h, const float *__restrict__ a_src,
    const float *__restrict__ a_dst, const float *__restrict__ row_stats, int64_t ldr, const float *__restrict__ dout,
    int64_t ldq, const float *__restrict__ att_s, const float *__restrict__ att_d, float ns, float *__restrict__ dh,
    float *__restrict__ da_src, int splits, float *__restrict__ ws) {
  __shared__ float red[4][32];
  const int lane = lane_id(), w = wave_in_block();
  const int sp = blockIdx.y;
  const int li = lane & 31, lk = lane >> 5;
  const int rb = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = row_begin + rb * 32;
  const int hd = w >> 1, q0 = 32 * w;
  const float4 *g4 = reinterpret_cast<const float4 *>(dout);

  const int ri = r0 + li;
  const bool rvalid = ri < row_end;
  const float asr = rvalid ? a_src[2 * (size_t)ri + hd] : 0.f;

  f32x16 acc[4], cc[4];
  float4 *o4 = reinterpret_cast<float4 *>(dh);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = r0 + acc_row(r, lk);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (splits == 1 && row < row_end) v = o4[(size_t)row * 128 + q0 + li];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t][r] = f4_c(v, t);
      cc[t][r] = 0.f;
    }
  }

  float sb = 0.f;
  const int tb = tptr[rb], te = tptr[rb + 1];
  for (int tt = tb + sp; tt < te; tt += splits) {
    const int cbase = 32 * tcol[tt];
    const uint32_t mk = tmask[(size_t)tt * 32 + li];
    // constants of destination row (column) cbase + li
    const int ci = min(cbase + li, ncols - 1);
    const float adi = a_dst[2 * (size_t)ci + hd];
    const float mi = row_stats[ldr * ci + hd];
    const float dni = row_stats[ldr * ci + 2 + hd] + 1e-16f;
    const float dli = row_stats[ldr * ci + 4 + hd];
#pragma unroll
    for (int half = 0; half < 16 / KBB; ++half) {
    float4 gb[KBB];
#pragma unroll
    for (int u = 0; u < KBB; ++u) {
      const int i = min(cbase + 2 * (half * KBB + u) + lk, ncols - 1);
      gb[u] = g4[(size_t)i * ldq + q0 + li];
    }
#pragma unroll
    for (int u = 0; u < KBB; ++u) {
      const int kp = half * KBB + u;
      const int kc = 2 * kp + lk;
      const float ad = __shfl(adi, kc), mx = __shfl(mi, kc), dn = __shfl(dni, kc), dl = __shfl(dli, kc);
      const float e = asr + ad;
      const bool on = rvalid && ((mk >> kc) & 1u);
      const float p = on ? expf(lrelu(e, ns) - mx) / dn : 0.f;
      const float q = p * (e > 0.f ? 1.f : ns);
      sb = fmaf(q, dl, sb);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(p, f4_c(gb[u], t), acc[t], 0, 0, 0);
        cc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(q, f4_c(gb[u], t), cc[t], 0, 0, 0);
      }
    }
    }
  }

  // <c_r, h_r> over this wave's 128 columns: per accumulator row, a float4 dot, then a sum over the
  // 32 lanes of the half wave (the 32 column quads)
  const float4 *h4 = reinterpret_cast<const float4 *>(h);
  float part[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = r0 + acc_row(r, lk);
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < row_end) hv = h4[(size_t)row * 128 + q0 + li];
    part[r] = fmaf(cc[0][r], hv.x, fmaf(cc[1][r], hv.y, fmaf(cc[2][r], hv.z, cc[3][r] * hv.w)));
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) part[r] = half_wave_sum(part[r]);
  if (li == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][acc_row(r, lk)] = part[r];
  }
  // sb of row li: the two half waves saw the two halves of its k-pairs
  sb += __shfl_xor(sb, 32);
  __syncthreads();
  if (splits > 1) {   // raw partials of this split -> workspace (band_bwd_epilogue finishes dh, da_src)
    const int64_t R = row_end - row_begin;
    float4 *wa = reinterpret_cast<float4 *>(ws) + ((int64_t)sp * R - row_begin) * 128;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = r0 + acc_row(r, lk);
      if (row < row_end) wa[(size_t)row * 128 + q0 + li] = make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
    }
    float *wc = ws + (size_t)splits * R * 512 + ((int64_t)sp * R - row_begin) * 2;
    if ((w & 1) == 0 && lk == 0 && rvalid) wc[2 * (size_t)ri + hd] = (red[2 * hd][li] + red[2 * hd + 1][li]) - sb;
    return;
  }
  // da_src of row li of this head: remainder share + both waves' dot shares - sb
  float ds_row = 0.f;
  if (rvalid) ds_row = (da_src[2 * (size_t)ri + hd] + (red[2 * hd][li] + red[2 * hd + 1][li])) - sb;
  __syncthreads();   // every wave has read its share of da_src before one of them overwrites it
  if ((w & 1) == 0 && lk == 0 && rvalid) da_src[2 * (size_t)ri + hd] = ds_row;

  const float4 as4 = reinterpret_cast<const float4 *>(att_s)[q0 + li];
  const float4 at4 = reinterpret_cast<const float4 *>(att_d)[q0 + li];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int mrow = acc_row(r, lk), row = r0 + mrow;
    const float ds = __shfl(ds_row, mrow);
    if (row < row_end) {
      const float dd = row_stats[ldr * row + 6 + hd];
      float4 v = make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
      v = f4_fma(ds, as4, v);
      v.x = fmaf(dd, at4.x, v.x);
      v.y = fmaf(dd, at4.y, v.y);
      v.z = fmaf(dd, at4.z, v.z);
      v.w = fmaf(dd, at4.w, v.w);
      o4[(size_t)row * 128 + q0 + li] = v;
    }
  }
}

// ---- split form (splits > 1: a row block's tiles spread over `splits` workgroups, so a graph with
// few row blocks -- a dense 2000-node contact map has 63 -- still fills the chip): the tile kernels
// leave raw partials in the workspace and these one-wave-per-row passes add them to the gather's
// sums in split order and apply the epilogue (bitwise reproducible).
template <bool TRAIN, int ACT>
__global__ __launch_bounds__(256) void band_fwd_epilogue(int row_begin, int row_end, int splits,
                                                         const float *__restrict__ ws, const float *__restrict__ bias,
                                                         float *__restrict__ out, float *__restrict__ out2,
                                                         float *__restrict__ row_stats) {
  const int lane = lane_id();
  const int i = row_begin + blockIdx.x * 4 + wave_in_block();
  if (i >= row_end) return;
  const int64_t R = row_end - row_begin, lr = i - row_begin;
  const float4 *w4 = reinterpret_cast<const float4 *>(ws);
  float4 *o4 = reinterpret_cast<float4 *>(out) + (size_t)i * 128;
  float4 a0 = o4[lane], a1 = o4[64 + lane];
  for (int s = 0; s < splits; ++s) {
    const float4 *p = w4 + ((int64_t)s * R + lr) * 128;
    const float4 u0 = p[lane], u1 = p[64 + lane];
    a0.x += u0.x; a0.y += u0.y; a0.z += u0.z; a0.w += u0.w;
    a1.x += u1.x; a1.y += u1.y; a1.z += u1.z; a1.w += u1.w;
  }
  const float4 b0 = reinterpret_cast<const float4 *>(bias)[lane], b1 = reinterpret_cast<const float4 *>(bias)[64 + lane];
  a0 = make_float4(a0.x + b0.x, a0.y + b0.y, a0.z + b0.z, a0.w + b0.w);
  a1 = make_float4(a1.x + b1.x, a1.y + b1.y, a1.z + b1.z, a1.w + b1.w);
  if (ACT == 1) {
    a0 = f4_relu(a0);
    a1 = f4_relu(a1);
  }
  o4[lane] = a0;
  o4[64 + lane] = a1;
  if (TRAIN) {
    float4 *q4 = reinterpret_cast<float4 *>(out2) + (size_t)i * 128;
    float4 c0 = q4[lane], c1 = q4[64 + lane];
    for (int s = 0; s < splits; ++s) {
      const float4 *p = w4 + ((int64_t)(splits + s) * R + lr) * 128;
      const float4 u0 = p[lane], u1 = p[64 + lane];
      c0.x += u0.x; c0.y += u0.y; c0.z += u0.z; c0.w += u0.w;
      c1.x += u1.x; c1.y += u1.y; c1.z += u1.z; c1.w += u1.w;
    }
    q4[lane] = c0;
    q4[64 + lane] = c1;
    if (lane < 2) {
      const float *w3 = ws + (size_t)2 * splits * R * 512;
      float t = row_stats[8 * (size_t)i + 4 + lane];
      for (int s = 0; s < splits; ++s) t += w3[((int64_t)s * R + lr) * 2 + lane];
      row_stats[8 * (size_t)i + 4 + lane] = t;
    }
  }
}

__global__ __launch_bounds__(256) void band_bwd_epilogue(int row_begin, int row_end, int splits,
                                                         const float *__restrict__ ws,
                                                         const float *__restrict__ row_stats, int64_t ldr,
                                                         const float *__restrict__ att_s,
                                                         const float *__restrict__ att_d, float *__restrict__ dh,
                                                         float *__restrict__ da_src) {
  const int lane = lane_id();
  const int r = row_begin + blockIdx.x * 4 + wave_in_block();
  if (r >= row_end) return;
  const int64_t R = row_end - row_begin, lr = r - row_begin;
  const float *wc = ws + (size_t)splits * R * 512;
  float ds0 = da_src[2 * (size_t)r], ds1 = da_src[2 * (size_t)r + 1];
  for (int s = 0; s < splits; ++s) {
    ds0 += wc[((int64_t)s * R + lr) * 2];
    ds1 += wc[((int64_t)s * R + lr) * 2 + 1];
  }
  const float4 *w4 = reinterpret_cast<const float4 *>(ws);
  float4 *o4 = reinterpret_cast<float4 *>(dh) + (size_t)r * 128;
  float4 a0 = o4[lane], a1 = o4[64 + lane];
  for (int s = 0; s < splits; ++s) {
    const float4 *p = w4 + ((int64_t)s * R + lr) * 128;
    const float4 u0 = p[lane], u1 = p[64 + lane];
    a0.x += u0.x; a0.y += u0.y; a0.z += u0.z; a0.w += u0.w;
    a1.x += u1.x; a1.y += u1.y; a1.z += u1.z; a1.w += u1.w;
  }
  const float2 dd = *reinterpret_cast<const float2 *>(row_stats + ldr * r + 6);
  const float4 *s4 = reinterpret_cast<const float4 *>(att_s);
  const float4 *t4 = reinterpret_cast<const float4 *>(att_d);
  a0 = f4_fma(ds0, s4[lane], a0);
  a0 = f4_fma(dd.x, t4[lane], a0);
  a1 = f4_fma(ds1, s4[64 + lane], a1);
  a1 = f4_fma(dd.y, t4[64 + lane], a1);
  o4[lane] = a0;
  o4[64 + lane] = a1;
  if (lane == 0) *reinterpret_cast<float2 *>(da_src + 2 * (size_t)r) = make_float2(ds0, ds1);
}

}  // namespace hicgat

using namespace hicgat;

static bool tiles_args_ok(const int32_t *tptr, const int32_t *tcol, const uint32_t *tmask, int ntiles) {
  return tptr && (ntiles == 0 || (tcol && tmask));
}

extern "C" size_t hicgat_gat_tiled_workspace_bytes(int rows, int splits) {
  if (rows <= 0 || splits <= 1) return 0;
  return (size_t)splits * rows * (2 * 512 + 2) * sizeof(float);
}

static int tiled_ws_ok(int rows, int splits, const void *workspace, size_t workspace_bytes) {
  if (splits < 1 || splits > 64) return 0;
  const size_t need = hicgat_gat_tiled_workspace_bytes(rows, splits);
  return need == 0 || (workspace && workspace_bytes >= need && (reinterpret_cast<uintptr_t>(workspace) & 15) == 0);
}

extern "C" int hicgat_gat_agg_fwd_tiled(const int32_t *rowptr, const int32_t *col, const int32_t *rowptr_s,
                                        const int32_t *col_s, const int32_t *tptr, const int32_t *tcol,
                                        const uint32_t *tmask, int ntiles, int N, int H, int C, int row_begin,
                                        int row_end, const float *h, const float *a_src, const float *a_dst,
                                        const float *bias, float neg_slope, int act, float *out, float *out2,
                                        float *row_stats, int splits, void *workspace, size_t workspace_bytes,
                                        hicgat_stream_t stream) {
  if (N < 0 || ntiles < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (act != 0 && act != 1) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (row_end == row_begin) return HICGAT_OK;
  const int rows = row_end - row_begin;
  if (!rowptr || !col || !rowptr_s || !col_s || !tiles_args_ok(tptr, tcol, tmask, ntiles) || !h || !a_src ||
      !a_dst || !bias || !out || !row_stats || !tiled_ws_ok(rows, splits, workspace, workspace_bytes))
    return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int rc = agg_fwd_split_launch(rowptr, col, rowptr_s, col_s, row_begin, row_end, h, a_src, a_dst, neg_slope, out,
                                out2, row_stats, s);
  if (rc != HICGAT_OK) return rc;
  const dim3 grid((rows + 31) / 32, splits), block(256), egrid((rows + 3) / 4);
  float *ws = static_cast<float *>(workspace);
#define HICGAT_BAND_FWD(TR, AC)                                                                                   \
  do {                                                                                                           \
    hipLaunchKernelGGL((band_fwd_kernel<TR, AC>), grid, block, 0, s, tptr, tcol, tmask, row_begin, row_end, N, h, \
                       a_src, a_dst, bias, neg_slope, out, out2, row_stats, splits, ws);                          \
    if (splits > 1)                                                                                               \
      hipLaunchKernelGGL((band_fwd_epilogue<TR, AC>), egrid, block, 0, s, row_begin, row_end, splits, ws, bias,   \
                         out, out2, row_stats);                                                                   \
  } while (0)
  if (out2) {
    if (act) HICGAT_BAND_FWD(true, 1);
    else HICGAT_BAND_FWD(true, 0);
  } else {
    if (act) HICGAT_BAND_FWD(false, 1);
    else HICGAT_BAND_FWD(false, 0);
  }
#undef HICGAT_BAND_FWD
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_gat_agg_bwd_src_tiled(const int32_t *rowptr_s, const int32_t *col_s, const int32_t *tptr,
                                            const int32_t *tcol, const uint32_t *tmask, int ntiles, int N, int H,
                                            int C, int row_begin, int row_end, const float *h, const float *a_src,
                                            const float *a_dst, const float *row_stats, int64_t ld_stats,
                                            const float *dout, int64_t ld_dout, const float *att_src,
                                            const float *att_dst, float neg_slope, float *dh, float *da_src,
                                            int splits, void *workspace, size_t workspace_bytes,
                                            hicgat_stream_t stream) {
  if (N < 0 || ntiles < 0 || row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  if (H != 2 || C != 256) return HICGAT_EUNSUPPORTED;
  if (ld_stats < 4 * H || ld_stats % 4 || ld_dout < H * C || ld_dout % 4) return HICGAT_EINVAL;
  if (row_end == row_begin) return HICGAT_OK;
  const int rows = row_end - row_begin;
  if (!rowptr_s || !col_s || !tiles_args_ok(tptr, tcol, tmask, ntiles) || !h || !a_src || !a_dst || !row_stats ||
      !dout || !att_src || !att_dst || !dh || !da_src || !tiled_ws_ok(rows, splits, workspace, workspace_bytes))
    return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int rc = agg_bwd_src_split_launch(rowptr_s, col_s, row_begin, row_end, h, a_src, a_dst, row_stats, ld_stats, dout,
                                    ld_dout / 4, neg_slope, dh, da_src, s);
  if (rc != HICGAT_OK) return rc;
  float *ws = static_cast<float *>(workspace);
  hipLaunchKernelGGL(band_bwd_kernel, dim3((rows + 31) / 32, splits), dim3(256), 0, s, tptr, tcol, tmask, row_begin,
                     row_end, N, h, a_src, a_dst, row_stats, ld_stats, dout, ld_dout / 4, att_src, att_dst, neg_slope,
                     dh, da_src, splits, ws);
  if (splits > 1)
    hipLaunchKernelGGL(band_bwd_epilogue, dim3((rows + 3) / 4), dim3(256), 0, s, row_begin, row_end, splits, ws,
                       row_stats, ld_stats, att_src, att_dst, dh, da_src);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
