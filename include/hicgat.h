/*
 * hicgat.h -- C ABI of libhicgat.so, the MI355X (gfx950) kernels of the GAT-HiC per-epoch step.
 *
 * The reference (beyzoskaya/HiC-GNN, /root/reference) is pure Python: its "native boundary" is the
 * set of third-party torch custom ops that PyG 1.7.2's GATConv, torch.cdist and torch.optim.Adam
 * call.  Each entry point below replaces one group of those ops; the
 * comment on each names the reference call site it stands in for.
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (PyTorch's caching allocator); nothing
 *     is allocated inside; scratch ("workspace") is passed in and sized by the *_workspace_bytes()
 *     query;
 *   - work is enqueued on `stream` (a hipStream_t passed as void*; NULL = the legacy default
 *     stream) and is stream-ordered; no call synchronises the host, so every call can be captured
 *     into a hipGraph;
 *   - return 0 on success or a negative HICGAT_E* code (hicgat_strerror() names it);
 *   - stateless and re-entrant; one process drives one GPU;
 *   - index arrays are int32 (nnz < 2^31), converted once from the reference's int64 when the
 *     adjacency is built; every matrix is row-major with the stated leading dimension.
 */
#ifndef HICGAT_H
#define HICGAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *hicgat_stream_t;

/* loss_kind of the fused distance / loss entry points */
enum { HICGAT_LOSS_MSE = 0, HICGAT_LOSS_COMBINED = 1, HICGAT_LOSS_CONTRASTIVE = 2 };

enum {
  HICGAT_OK = 0,
  HICGAT_EINVAL = -1,   /* bad size / null pointer / misaligned buffer */
  HICGAT_ELAUNCH = -2,  /* hipGetLastError() reported a launch failure */
  HICGAT_EUNSUPPORTED = -3
};

int hicgat_version(void);
const char *hicgat_strerror(int code);

/* ---- a13/a3: graph build -------------------------------------------------------------------
 * Reference: utils.load_input (utils.py:29-73; networkx edges + SparseTensor(...).to_symmetric())
 * followed by torch_sparse.set_diag inside PyG 1.7.2 GATConv.forward.  From a dense row-major
 * N x N contact matrix A (float64, leading dim lda), builds the symmetric CSR of
 * (A[i,j] != 0 || A[j,i] != 0) for i != j, with one self loop (i,i) inserted per row at its sorted
 * position.  Two calls: first with col == NULL to get rowptr (row_counts scratch of N+1 ints is
 * rowptr itself), then with col to fill the columns.  Bit-exact with the reference pattern. */
int hicgat_csr_from_dense(const double *A, int N, int64_t lda, int32_t *rowptr, int32_t *col,
                          void *workspace, size_t workspace_bytes, hicgat_stream_t stream);
size_t hicgat_csr_workspace_bytes(int N);

/* ---- a12: utils.cont2dist (utils.py:75-80) on the device ------------------------------------
 * dist = (1/y)^factor, diagonal 0, +inf -> max finite, NaN -> 0, divided by the max; float64 in,
 * float32 (or float64) out with leading dimension ldo. workspace: hicgat_cont2dist_workspace_bytes */
int hicgat_cont2dist(const double *y, int N, int64_t ldy, double factor, float *out32, double *out64,
                     int64_t ldo, void *workspace, size_t workspace_bytes, hicgat_stream_t stream);
size_t hicgat_cont2dist_workspace_bytes(int N);

/* ---- a2: GATConv lin_l + attention logits (PyG 1.7.2 GATConv.forward) ----------------------
 * h [N, H*C] = x [N, F] * W^T (W [H*C, F], lin_l.weight, no bias; lin_r is lin_l) and
 * a_src[n,h] = <h[n,h,:], att_l[h,:]>, a_dst[n,h] = <h[n,h,:], att_r[h,:]>.
 * hicgat_gat_linear_att computes both (fp32 MFMA GEMM with the logits fused in its epilogue);
 * hicgat_gat_att_logits computes only the logits from an existing h. */
int hicgat_gat_linear_att(const float *x, const float *W, const float *att_src, const float *att_dst,
                          int N, int F, int H, int C, float *h, float *a_src, float *a_dst,
                          hicgat_stream_t stream);
int hicgat_gat_att_logits(const float *h, const float *att_src, const float *att_dst, int N, int H,
                          int C, float *a_src, float *a_dst, hicgat_stream_t stream);

/* ---- a4+a5: edge softmax + neighbour aggregation (PyG 1.7.2 GATConv.propagate) --------------
 * CSR rows are destinations i, columns sources j, self loops already present (set_diag).
 *   e_ij = leaky_relu(a_src[j] + a_dst[i], neg_slope)
 *   alpha_ij = exp(e_ij - max_i) / (sum_i + 1e-16)        (torch_geometric.utils.softmax, ptr path)
 *   out[i] = sum_j alpha_ij * h[j] + bias                  (segment_csr sum; concat=True)
 * Only rows [row_begin, row_end) are computed (a rank's destination shard; 0..N on one GPU);
 * every per-row array is indexed by the GLOBAL row id: h, a_src, a_dst [N, .] (the neighbour
 * rows of the shard must be present), out [N, H*C] (rows of the range written),
 * row_stats [N, 4H] = (max[H], sum[H], delta[H], da_dst[H]) -- max/sum written here, delta/da_dst
 * by hicgat_gat_agg_bwd_dst.  Supported: H == 2, C == 256 (the GATConv(512, 256, heads=2) of
 * models.py:619); other shapes return HICGAT_EUNSUPPORTED. */
int hicgat_gat_agg_fwd(const int32_t *rowptr, const int32_t *col, int N, int nnz, int H, int C,
                       int row_begin, int row_end, const float *h, const float *a_src,
                       const float *a_dst, const float *bias, float neg_slope, float *out,
                       float *row_stats, hicgat_stream_t stream);
/* Training form of the same aggregation.  act = 1 writes out = relu(sum + bias) (the relu that
 * follows the GATConv at models.py:637), act = 0 the plain sum + bias.  out2 != NULL (training)
 * also writes, from the same gathered rows, out2 [N, H*C] = sum_j alpha_ij lrelu'(e_ij) h_j and
 * S3[i,h] = sum_j alpha_ij lrelu'(e_ij) into row_stats[i, 2H..3H) -- the inputs that let
 * hicgat_gat_agg_bwd_rows form the destination half of the backward without a gather. */
int hicgat_gat_agg_fwd_act(const int32_t *rowptr, const int32_t *col, int N, int nnz, int H, int C,
                           int row_begin, int row_end, const float *h, const float *a_src,
                           const float *a_dst, const float *bias, float neg_slope, int act,
                           float *out, float *out2, float *row_stats, hicgat_stream_t stream);

/* ---- a10 (part): backward of a4+a5 ----------------------------------------------------------
 * Pass 1 (destination side, rows of the range):  g_ij = <dout[i,h,:], h[j,h,:]>,
 *   delta[i,h] = sum_j alpha_ij g_ij,  da_dst[i,h] = sum_j alpha_ij lrelu'(e_ij) (g_ij - delta[i,h])
 *   -> row_stats[i, 2H..4H).
 * Pass 2 (source side, rows r of the range; the graph is symmetric so N(r) lists every i that
 *   has r as a neighbour; needs dout, row_stats of all those i):
 *   dh[r] = sum_i alpha_ir dout[i] + da_src[r] (x) att_l + da_dst[r] (x) att_r,
 *   da_src[r,h] = sum_i alpha_ir lrelu'(e_ir) (g_ir - delta[i,h]).
 * Requires a structurally symmetric CSR (utils.py:71 to_symmetric guarantees it). */
int hicgat_gat_agg_bwd_dst(const int32_t *rowptr, const int32_t *col, int N, int H, int C,
                           int row_begin, int row_end, const float *h, const float *a_src,
                           const float *a_dst, const float *dout, float neg_slope,
                           float *row_stats, hicgat_stream_t stream);
/* Pass 1 without a gather, after hicgat_gat_agg_fwd_act(..., out2, ...) (same row_stats):
 *   dout = g * [y > 0] (act = 1, written to dout with row stride ld_dout floats; torch's relu
 *   backward on the output y) or g
 *   (act = 0, dout unused); delta = <dout, y - bias>; da_dst = <dout, out2> - delta * S3,
 * per row of the range and head -> row_stats[i, 2H..4H) exactly as hicgat_gat_agg_bwd_dst. */
int hicgat_gat_agg_bwd_rows(int N, int H, int C, int row_begin, int row_end, int act, const float *g,
                            const float *y, const float *bias, const float *out2, float *dout,
                            int64_t ld_dout, float *row_stats, hicgat_stream_t stream);
int hicgat_gat_agg_bwd_src(const int32_t *rowptr, const int32_t *col, int N, int H, int C,
                           int row_begin, int row_end, const float *h, const float *a_src,
                           const float *a_dst, const float *row_stats, const float *dout,
                           const float *att_src, const float *att_dst, float neg_slope, float *dh,
                           float *da_src, hicgat_stream_t stream);
/* The same with strided rows: dout row i at dout + i*ld_dout, row_stats row i at
 * row_stats + i*ld_stats (floats, multiples of 4) -- e.g. one all-gathered [dout | row stats]
 * buffer per row (hicgat.dist). */
int hicgat_gat_agg_bwd_src_ld(const int32_t *rowptr, const int32_t *col, int N, int H, int C,
                              int row_begin, int row_end, const float *h, const float *a_src,
                              const float *a_dst, const float *row_stats, int64_t ld_stats,
                              const float *dout, int64_t ld_dout, const float *att_src,
                              const float *att_dst, float neg_slope, float *dh, float *da_src,
                              hicgat_stream_t stream);
/* The same with launch flags: HICGAT_SRC_ROUND_ROBIN spreads consecutive row blocks over the XCDs
 * instead of giving each XCD a contiguous row range (the multi-GPU "slab" pass, hicgat.dist, whose
 * heavy rows are one contiguous block); flags 0 = hicgat_gat_agg_bwd_src_ld. */
enum { HICGAT_SRC_ROUND_ROBIN = 1 };
int hicgat_gat_agg_bwd_src_ex(const int32_t *rowptr, const int32_t *col, int N, int H, int C, int row_begin,
                              int row_end, const float *h, const float *a_src, const float *a_dst,
                              const float *row_stats, int64_t ld_stats, const float *dout, int64_t ld_dout,
                              const float *att_src, const float *att_dst, float neg_slope, float *dh, float *da_src,
                              int flags, hicgat_stream_t stream);
/* ---- GATConv in aggregate-first order (gat_xagg.hip; the multi-GPU "xagg" step of hicgat.dist) ----
 * Reference: the same PyG 1.7.2 GATConv (models.py:619) -- out_i^h = W_h (sum_j alpha_ij^h x_j) +
 * b^h and a_src_j^h = <W_h^T att_src^h, x_j> are the h-first expressions regrouped, so a rank that
 * owns destination rows needs no other rank's h and runs every GEMM on its own rows.  F = 512,
 * H = 2, C = 256 only.  Row ranges [row_begin, row_end) are the rank's rows of a CSR in global
 * numbering whose rowptr[row_begin] = 0 (hicgat.dist.ShardPlan.own_csr); per-row outputs marked
 * "local" are indexed i - row_begin, row_stats by the global row.
 *   hicgat_xagg_logits: vec [4][512] = W_h^T att_src^h (h = 0, 1), W_h^T att_dst^h; a_src / a_dst
 *     [N][2] = x . vec for all N rows (workspace vec: hicgat_xagg_vec_bytes()).
 *   hicgat_xagg_fwd: softmax statistics (row_stats [N][8]: max, sum at [0:4], S3 at [4:6]) and
 *     X4 [2 heads][2 kinds][rows][512] (local): kind 0 xa = sum alpha x_j, kind 1 xa2 = sum alpha
 *     lrelu'(e) x_j.  The caller then forms [out; out2] per head = [xa; xa2] W_h^T (hicgat_gemm_ex).
 *   hicgat_xagg_bias_relu: y0 += bias, o = relu(y0) over [rows][512].
 *   hicgat_xagg_rows_bwd: own rows (local row_stats view): dout = g [y0 > 0] (act 1) or g,
 *     delta^h = <dout^h, y0^h - bias^h> into row_stats[4:6]; the forward's S3 moves to [6:8].
 *   hicgat_xagg_edge: ds [nnz_own][2] (the rank's CSR order) = alpha lrelu'(e) (<dxa_i^h, x_j> -
 *     delta_i^h), dxa [rows][1024] (local; head h at columns 512h = dout_i^h W_h), delta from
 *     row_stats[i][4:6]; with xa2 (X4's kind-1 planes: X4 + rows*512) also da_dst^h =
 *     <dxa_i^h, xa2_i^h> - delta_i^h S3_i^h into row_stats[i][6:8] (S3 read from there).
 *   hicgat_xagg_slab_sum: da_src [N][2], da_src_j = sum over the slab entries k of row j
 *     (rowptr_s, N + 1) of ds[perm[k]] (perm: the rank's CSR index of the transposed edge), and
 *     g_src [2][512] = sum_j da_src_j^h x_j (x: all N rows), fixed-order partial sums
 *     (workspace hicgat_xagg_slab_workspace_bytes()).
 *   hicgat_xagg_param_finish: dW[256h + c][:] += att_src^h[c] g_src[h][:] + att_dst^h[c] g_dst[h][:],
 *     datt_src^h[c] += <W[256h + c][:], g_src[h][:]>, datt_dst likewise (g [2][512]: sum_j da_j^h x_j). */
size_t hicgat_xagg_vec_bytes(void);
int hicgat_xagg_logits(const float *x, const float *W, const float *att_src, const float *att_dst, int N, int F,
                       int H, int C, float *vec, float *a_src, float *a_dst, hicgat_stream_t stream);
/* hicgat_xagg_logits that also zeroes zero_buf[0, zero_n) (a step's flat gradient buffer: the
 * optimizer's zero_grad, HiC-GNN_main.py:124) in its first launch -- one launch fewer per step --
 * and, with step_counter (NULL: none), advances the optimizer's device step count there (the step's
 * Adam then calls hicgat_adam_step_table_ex with counted = 1). */
int hicgat_xagg_logits_zero(const float *x, const float *W, const float *att_src, const float *att_dst, int N,
                            int F, int H, int C, float *vec, float *a_src, float *a_dst, float *zero_buf,
                            int64_t zero_n, int64_t *step_counter, hicgat_stream_t stream);
/* hicgat_xagg_logits_zero that, with pack (NULL: none), also writes the head-fused tail's packed
 * weights of W1c, W2c and Wh = W (hicgat_tail_pack's layout and pack_bytes rule) in the same launch:
 * the sharded step's tail kernels then read them without a pack launch of their own. */
int hicgat_xagg_logits_zero_pack(const float *x, const float *W, const float *att_src, const float *att_dst, int N,
                                 int F, int H, int C, float *vec, float *a_src, float *a_dst, float *zero_buf,
                                 int64_t zero_n, int64_t *step_counter, const float *W1c, const float *W2c, void *pack,
                                 size_t pack_bytes, hicgat_stream_t stream);
int hicgat_xagg_fwd(const int32_t *rowptr, const int32_t *col, int N, int F, int H, int C, int row_begin,
                    int row_end, const float *x, const float *a_src, const float *a_dst, float neg_slope, float *X4,
                    float *row_stats, hicgat_stream_t stream);
int hicgat_xagg_bias_relu(float *y0, const float *bias, float *o, int rows, int D, hicgat_stream_t stream);
int hicgat_xagg_rows_bwd(int rows, int D, int act, const float *g, const float *y0, const float *bias, float *dout,
                         float *row_stats, hicgat_stream_t stream);
int hicgat_xagg_edge(const int32_t *rowptr, const int32_t *col, int N, int F, int H, int C, int row_begin,
                     int row_end, const float *x, const float *a_src, const float *a_dst, float *row_stats,
                     const float *dxa, const float *xa2, float neg_slope, float *ds, hicgat_stream_t stream);
/* The edge pass with the source side folded in (replaces hicgat_xagg_edge + hicgat_xagg_slab_sum in
 * the sharded step): g_src^h = sum_j da_src_j^h x_j = sum over the own rows' edges (i, j) of
 * ds_ij^h x_j, formed in the pass that computes ds_ij; written as hicgat_xagg_edge_acc_blocks(rows)
 * partial rows gpart [blocks][1024] (head 0 | head 1) whose column sums are g_src (e.g. a
 * hicgat_param_grads_grouped column-sum job); with xa2, da_dst into row_stats[6:8] as hicgat_xagg_edge.
 * Deterministic (fixed row-to-block map and summation order). */
int hicgat_xagg_edge_acc(const int32_t *rowptr, const int32_t *col, int N, int F, int H, int C, int row_begin,
                         int row_end, const float *x, const float *a_src, const float *a_dst, float *row_stats,
                         const float *dxa, const float *xa2, float neg_slope, float *gpart, hicgat_stream_t stream);
int hicgat_xagg_edge_acc_blocks(int rows);
size_t hicgat_xagg_slab_workspace_bytes(void);
int hicgat_xagg_slab_sum(const int32_t *rowptr_s, const int32_t *perm, int N, const float *ds, const float *x,
                         float *da_src, float *g_src, void *workspace, size_t workspace_bytes,
                         hicgat_stream_t stream);
int hicgat_xagg_param_finish(const float *W, const float *att_src, const float *att_dst, const float *g_src,
                             const float *g_dst, int F, int H, int C, float *dW, float *datt_src, float *datt_dst,
                             hicgat_stream_t stream);
/* The same with g in `segs` segments (the segmented column sums of hicgat_param_grads_grouped):
 * g_src = sum over s of g_src + s * seg_stride (floats), g_dst likewise, added in segment order. */
int hicgat_xagg_param_finish_seg(const float *W, const float *att_src, const float *att_dst, const float *g_src,
                                 const float *g_dst, int segs, int64_t seg_stride, int F, int H, int C, float *dW,
                                 float *datt_src, float *datt_dst, hicgat_stream_t stream);

/* ---- a4+a5 and the source pass with the dense tiles on the matrix cores (gat_tiles.hip) -------
 * The same results as hicgat_gat_agg_fwd_act / hicgat_gat_agg_bwd_src_ld (fp32; the tiles' sums are
 * added in another order), with the edge set split in two:
 *   tiles: rows [row_begin, row_end) in blocks of 32 (block b = rows row_begin + 32b ..);
 *     tptr [nrb + 1] (nrb = ceil((row_end - row_begin) / 32)) indexes tcol [ntiles] (a 32-column
 *     block: columns 32*tcol[t] ..) and tmask [ntiles * 32] (bit c of word 32t + i: the edge
 *     (row_begin + 32b + i, 32*tcol[t] + c) exists); tiles of a block in any order, each edge in at
 *     most one tile;
 *   rowptr_s / col_s: the CSR (N + 1 row pointers, rows of the range) of every OTHER edge.
 * rowptr / col (the whole rows) give the softmax statistics.  The tiles' products run as dense
 * 32 x 32 x 32 x 512 blocks on v_mfma_f32_32x32x2_f32 (weights 0 off the edge set).  Built from the
 * CSR by hicgat.graph.build_tiles (a 32x32 tile is dense when it holds >= min_edges edges). */
int hicgat_gat_agg_fwd_tiled(const int32_t *rowptr, const int32_t *col, const int32_t *rowptr_s,
                             const int32_t *col_s, const int32_t *tptr, const int32_t *tcol,
                             const uint32_t *tmask, int ntiles, int N, int H, int C, int row_begin,
                             int row_end, const float *h, const float *a_src, const float *a_dst,
                             const float *bias, float neg_slope, int act, float *out, float *out2,
                             float *row_stats, int splits, void *workspace, size_t workspace_bytes,
                             hicgat_stream_t stream);
int hicgat_gat_agg_bwd_src_tiled(const int32_t *rowptr_s, const int32_t *col_s, const int32_t *tptr,
                                 const int32_t *tcol, const uint32_t *tmask, int ntiles, int N, int H,
                                 int C, int row_begin, int row_end, const float *h, const float *a_src,
                                 const float *a_dst, const float *row_stats, int64_t ld_stats,
                                 const float *dout, int64_t ld_dout, const float *att_src,
                                 const float *att_dst, float neg_slope, float *dh, float *da_src,
                                 int splits, void *workspace, size_t workspace_bytes,
                                 hicgat_stream_t stream);
/* splits (1..64): the tiles of a row block are spread over `splits` workgroups (a graph with few
 * row blocks, e.g. a dense 2000-node map: 63); splits > 1 needs a 16-B aligned workspace of
 * hicgat_gat_tiled_workspace_bytes(row_end - row_begin, splits) bytes for the partial sums, which
 * one more pass adds in split order. */
size_t hicgat_gat_tiled_workspace_bytes(int rows, int splits);
/* Column reductions for the GATConv parameter gradients over N rows (pass pointers offset to a
 * shard's first row for a partial sum; deterministic, two-stage):
 *   datt_src[h,c] = sum_n da_src[n,h] h[n,h,c];  datt_dst likewise with row_stats' da_dst;
 *   dbias[c] = sum_n dout[n,c].  workspace: hicgat_gat_param_grad_workspace_bytes(N, H*C).
 * Any of datt_src / datt_dst / dbias may be NULL (that part is skipped, and the inputs only it
 * reads may be NULL too): datt_dst and dbias need no source-pass output, so they can be summed
 * beside that pass; each part is bitwise the same whichever subset is asked for. */
int hicgat_gat_param_grad(const float *h, const float *dout, const float *da_src,
                          const float *row_stats, int N, int H, int C, float *datt_src,
                          float *datt_dst, float *dbias, int accumulate, void *workspace,
                          size_t workspace_bytes, hicgat_stream_t stream);
size_t hicgat_gat_param_grad_workspace_bytes(int N, int D);

/* ---- a7: torch.cdist(c, c, p=2) (models.py:661) and its backward -----------------------------
 * D[i,j] = ||c_i - c_j||_2 (exact formula; the diagonal is exactly 0), ld = leading dim of D.
 * Backward: dc_i = sum_j (G_ij + G_ji) (c_i - c_j) / D_ij over D_ij != 0 (torch's
 * _euclidean_dist_backward masks res == 0).  workspace: hicgat_pairdist_workspace_bytes(N, HICGAT_PD_SQUARE). */
int hicgat_pairdist_fwd(const float *coords, int N, float *D, int64_t ldd, hicgat_stream_t stream);
int hicgat_pairdist_bwd(const float *coords, const float *G, int N, int64_t ldg, float *dcoords,
                        void *workspace, size_t workspace_bytes, hicgat_stream_t stream);

/* ---- a7+a8+a9 fused: distance + MSE + Pearson moments + d(MSE)/dcoords, D never stored ------
 * Reference: out = cdist(coords) (models.py:661); MSELoss()(out, truth) (HiC-GNN_main.py:127);
 * pearsonr / alpha / total (HiC_GAT_generalize_directly.py:210-225).  T is the SYMMETRIC truth
 * (leading dim ldt); only upper-triangle tiles [tile_begin, tile_end) of the 128x128 tiling are
 * read (pass 0, -1 for all).  Outputs:
 *   stats[12] (float64): 0 sum_{i<j}(d-t)^2, 1 sum d, 2 sum d^2, 3 sum dt, 4 sum t, 5 sum t^2,
 *     6 sum_i T_ii^2 (moments 0..6 over the tile range; a multi-GPU caller all-reduces them and
 *     calls hicgat_pairdist_finalize), 7 mse = (2*[0] + [6])/N^2, 8 pearson r over i<j,
 *     9 alpha = min(1, 0.1 + 1/(mse + 1e-6)), 10 total = mse + alpha*(1 - r), 11 reserved;
 *   loss_kind 0 (the MSE of HiC-GNN_main.py) forms moments 0 and 6 only: 1..5 are 0, r (8) is NaN
 *     and 9..10 are not meaningful; loss_kind 1 (combined loss) forms all of them;
 *   loss_kind 2 (HICGAT_LOSS_CONTRASTIVE, train_and_test_same_res_GAT_node2vec.py:107-134:
 *     0.1 * mean_{i<j} |T_ij - D_ij|) forms moment 0 = sum_{i<j} |d - t| only (6 = 0: no diagonal
 *     term); finalized: 7 = mean |d - t| (fp64), 8 = NaN, 9 = 0.1, 10 = total = 0.1 * [7];
 *   loss[1] (float32): mse (loss_kind 0), total (loss_kind 1) or fp32(total) (loss_kind 2);
 *   dcoords [N,3] = d(loss)/dcoords restricted to the tile range (sum over ranks = full gradient):
 *     d(mse) (loss_kind 0, 1: the Pearson term carries no gradient in the reference) or
 *     float32(0.1 / M) * sum_j sign(d_ij - t_ij) (c_i - c_j) / d_ij, sign(0) = 0 (loss_kind 2).
 * workspace: hicgat_pairdist_workspace_bytes(N, HICGAT_PD_TRI). */
int hicgat_pairdist_mse_fused(const float *coords, const float *T, int N, int64_t ldt,
                              int64_t tile_begin, int64_t tile_end, int loss_kind, double *stats,
                              float *loss, float *dcoords, void *workspace, size_t workspace_bytes,
                              hicgat_stream_t stream);
/* The same over a BAND of the truth (a rank's share, hicgat.dist): T holds rows
 * [t_row0, t_row0 + t_rows) and columns [t_col0, t_col0 + ldt) of the N x N truth, element (i, j) at
 * T[(i - t_row0) * ldt + (j - t_col0)].  The band must cover every pair of the tile range: rows of
 * its tile-rows I0..I1 and columns from I0*128 on (else HICGAT_EINVAL). */
int hicgat_pairdist_mse_fused_band(const float *coords, const float *T, int N, int64_t ldt,
                                   int64_t t_row0, int64_t t_rows, int64_t t_col0, int64_t tile_begin,
                                   int64_t tile_end, int loss_kind, double *stats, float *loss,
                                   float *dcoords, void *workspace, size_t workspace_bytes,
                                   hicgat_stream_t stream);
int hicgat_pairdist_finalize(int N, int loss_kind, double *stats, float *loss, hicgat_stream_t stream);
/* hicgat_pairdist_finalize + dcoords[r][c] = (float)dc64[r][c] for rows [row_begin, row_end) of the
 * (all-reduced) fp64 coordinate gradient [N][3], in one launch (a rank's rows for its tail backward). */
int hicgat_pairdist_finalize_rows(int N, int loss_kind, double *stats, float *loss, const double *dc64, int row_begin,
                                  int row_end, float *dcoords, hicgat_stream_t stream);
/* The same; with cbuf (the padded all-gather coordinates [P*R][3]) also cglob[i] = cbuf[gidx[i]]
 * (i < N: the coordinates in global row order, hicgat.dist's step() output) in the same launch. */
int hicgat_pairdist_finalize_rows_ex(int N, int loss_kind, double *stats, float *loss, const double *dc64,
                                     int row_begin, int row_end, float *dcoords, const float *cbuf,
                                     const int32_t *gidx, float *cglob, hicgat_stream_t stream);
/* Tile count and workspace of the two tilings, mode HICGAT_PD_TRI (the fused loss: upper-triangle
 * 128x128 tiles, nb(nb+1)/2) or HICGAT_PD_SQUARE (hicgat_pairdist_bwd: nb*nb), nb = ceil(N/128). */
enum { HICGAT_PD_SQUARE = 0, HICGAT_PD_TRI = 1 };
int64_t hicgat_pairdist_num_tiles(int N, int mode);
size_t hicgat_pairdist_workspace_bytes(int N, int mode);
/* The same fused loss (all tiles, stats / loss / dcoords as above) for a truth given in BACKGROUND
 * form: T[i][j] = background for i != j except at the support -- a symmetric CSR (rowptr [N+1],
 * sorted col, val = T there, no diagonal entries) -- and T[i][i] = diag[i].  cont2dist's target
 * (utils.py:75-80) is of this form with background 1 (zero contacts: inf -> max -> 1) and the
 * support = the contacts, so the O(N^2) pass reads no truth at all: it takes every pair at the
 * background value and a pass over the support adds the difference (same sums up to fp32 /
 * fp64 reassociation).  Build the form with hicgat_truth_support.
 * workspace: hicgat_pairdist_support_workspace_bytes(N). */
int hicgat_pairdist_mse_fused_support(const float *coords, int N, float background, const int32_t *rowptr,
                                      const int32_t *col, const float *val, const float *diag, int loss_kind,
                                      double *stats, float *loss, float *dcoords, void *workspace,
                                      size_t workspace_bytes, hicgat_stream_t stream);
size_t hicgat_pairdist_support_workspace_bytes(int N);
/* The background-form loss over a SHARE of the pairs (a rank of hicgat.dist): the bulk over the
 * upper-triangle tiles [tile_begin, tile_end) and the support rows [support_row_begin,
 * support_row_end) (their entries j != i and their diagonal).  stats[0..6] and dcoords [N,3] are
 * that share's partial sums (the sum over shares that cover every tile and every row once is the
 * whole loss: a caller all-reduces stats[0..6] + dcoords and calls hicgat_pairdist_finalize);
 * 0, -1, 0, N is hicgat_pairdist_mse_fused_support.  dcoords64 (instead of dcoords): the same
 * fp32 gradient values widened to fp64, e.g. right behind stats[12] in one fp64 buffer that the
 * caller all-reduces as a whole; with dcoords64 and at most 4096 tiles + support blocks in the share,
 * stats[7..11] and loss are not written (the caller's finalize after the all-reduce sets them).
 * Same workspace. */
int hicgat_pairdist_mse_fused_support_range(const float *coords, int N, float background, const int32_t *rowptr,
                                            const int32_t *col, const float *val, const float *diag,
                                            int64_t tile_begin, int64_t tile_end, int support_row_begin,
                                            int support_row_end, int loss_kind, double *stats, float *loss,
                                            float *dcoords, double *dcoords64, void *workspace,
                                            size_t workspace_bytes, hicgat_stream_t stream);
/* The same with cmap (NULL = as above): cmap [N] maps global row g to its row in ``coords`` (the
 * sharded step's padded [P*R, 3] all-gather buffer, so no reorder launch before the loss). */
int hicgat_pairdist_mse_fused_support_range_ex(const float *coords, const int32_t *cmap, int N, float background,
                                               const int32_t *rowptr, const int32_t *col, const float *val,
                                               const float *diag, int64_t tile_begin, int64_t tile_end,
                                               int support_row_begin, int support_row_end, int loss_kind,
                                               double *stats, float *loss, float *dcoords, double *dcoords64,
                                               void *workspace, size_t workspace_bytes, hicgat_stream_t stream);
/* The background form of a symmetric N x N fp32 truth T (leading dim ldt): the sorted CSR of the
 * off-diagonal entries != background, their values, and the diagonal.  Two calls, as
 * hicgat_csr_from_dense: col == NULL fills rowptr (the counts, scanned); then col / val / diag. */
int hicgat_truth_support(const float *T, int N, int64_t ldt, float background, int32_t *rowptr, int32_t *col,
                         float *val, float *diag, hicgat_stream_t stream);

/* ---- a6 / a10: fp32 MFMA GEMM for torch.nn.Linear forward/backward (models.py:637-659) -------
 *   C[M,N] (+)= op(A) op(B) (+ bias[N]);  op(A) = A [M,K] (lda = row stride) or, with a_kmajor,
 *   A^T of A [K,M];  op(B) = B^T of B [N,K] or, with b_kmajor, B [K,N].
 *   Linear forward Y = X W^T + b (0,0); input grad dX = dY W (0,1); weight grad dW = dY^T X (1,1).
 * accumulate != 0 adds into C (a parameter's .grad).  splits > 1 splits K over workgroups into fp32
 * slabs (workspace: hicgat_gemm_workspace_bytes) added in split order: deterministic. */
int hicgat_gemm(int a_kmajor, int b_kmajor, int M, int N, int K, const float *A, int64_t lda,
                const float *B, int64_t ldb, const float *bias, float *C, int64_t ldc, int accumulate,
                int splits, void *workspace, size_t workspace_bytes, hicgat_stream_t stream);
size_t hicgat_gemm_workspace_bytes(int M, int N, int splits);
/* The same GEMM with the matrix-core arithmetic named explicitly: HICGAT_GEMM_F32 (= AUTO, the
 * only one): v_mfma_f32_32x32x2_f32, fp32 products, fp32 accumulate.  HICGAT_GEMM_X3 (a three-way
 * bf16 operand split on the bf16 matrix cores, round 1-3) measured slower per step and was removed:
 * HICGAT_EUNSUPPORTED. */
enum { HICGAT_GEMM_AUTO = 0, HICGAT_GEMM_F32 = 1, HICGAT_GEMM_X3 = 2 };
int hicgat_gemm_ex(int a_kmajor, int b_kmajor, int M, int N, int K, const float *A, int64_t lda,
                   const float *B, int64_t ldb, const float *bias, float *C, int64_t ldc, int accumulate,
                   int splits, int impl, void *workspace, size_t workspace_bytes, hicgat_stream_t stream);
/* Weight AND bias gradient of a Linear in one GEMM (replaces the dW GEMM + bias column sum of the
 * Linear backward, torch.nn.Linear via ATen addmm_backward / sum(0), models.py:637-659):
 *   dW[M,N] (+)= dY^T X  (dY [K,M] and X [K,N] row-major, K = node rows),
 *   db[M]   (+)= sum_k dY[k][m]  (db may be NULL)
 * the workgroups of the first column tile sum their staged dY tile over K; with splits > 1 the
 * per-split db partials sit in the slab beside the dW partials and ONE slab sum (split order,
 * deterministic) writes both.  fp32 MFMA (HICGAT_GEMM_F32 arithmetic).  Workspace:
 * hicgat_gemm_wgrad_workspace_bytes(M, N, splits). */
int hicgat_gemm_wgrad(int M, int N, int K, const float *dY, int64_t ldy, const float *X, int64_t ldx, float *dW,
                      int64_t lddw, float *db, int accumulate, int splits, void *workspace, size_t workspace_bytes,
                      hicgat_stream_t stream);
size_t hicgat_gemm_wgrad_workspace_bytes(int M, int N, int splits);
/* ---- grouped parameter gradients (one training step's dW / db / LayerNorm sums in two launches) ----
 * Replaces the per-Linear autograd weight-gradient calls (the ATen mm of dY^T X and the bias sum
 * behind every torch.nn.Linear.backward in models.py:637-659, and GATConv lin_l's) when a
 * step issues all of them at one point (the sharded step, hicgat.dist): the W weight-gradient
 * jobs dW (+)= dY^T X, db (+)= column sums of dY (db may be NULL; dY [K, M] ld ldy, X [K, N] ld
 * ldx, dW [M, N] ld lddw) run as ONE launch of 128 x 128 fp32-MFMA tiles over the union of their
 * tiles, K split into chunks of one common depth (about target_wgs workgroups in all), partials in
 * fp32 slabs; then ONE launch adds, in fixed order, every job's slabs into dW / db AND the C extra
 * column-sum jobs dst[c] (+)= sum_{r < rows} (wt ? wt[r * ldw] : 1) src[r * ld + c] (LayerNorm
 * dgamma/dbeta partial rows, bias sums, the rows of a few-row weight gradient).  Deterministic (no atomics); at most 16 weight-gradient and 32 column-sum jobs
 * (HICGAT_EUNSUPPORTED beyond).  Workspace: hicgat_param_grads_workspace_bytes(same jobs). */
typedef struct hicgat_wgrad_job {
  const float *dy;
  int64_t ldy;
  const float *x;
  int64_t ldx;
  float *dw;
  int64_t lddw;
  float *db;
  int M, N, K, accumulate;
} hicgat_wgrad_job;
typedef struct hicgat_colsum_job {
  const float *src;
  int64_t ld;
  int64_t rows;
  int64_t cols;
  float *dst;
  int accumulate;
  const float *wt;    /* NULL, or row weights: dst[c] (+)= sum_r wt[r * ldw] src[r * ld + c] (a dW row of a */
  int64_t ldw;        /* weight gradient with a handful of output rows, e.g. dense3's 3 x 64) */
  int segs;           /* <= 1: one sum into dst; else the rows in `segs` contiguous segments, segment s */
  int64_t ldd;        /* (rows [rows s / segs, rows (s + 1) / segs)) into dst + s * ldd: a tall job's sum
                       * spread over segs x more blocks, the segments added by the consumer */
} hicgat_colsum_job;
size_t hicgat_param_grads_workspace_bytes(const hicgat_wgrad_job *wjobs, int nw, int target_wgs);
int hicgat_param_grads_grouped(const hicgat_wgrad_job *wjobs, int nw, const hicgat_colsum_job *cjobs, int nc,
                               int target_wgs, void *workspace, size_t workspace_bytes, hicgat_stream_t stream);
/* Grouped node-row GEMMs of one layout: C_j = A_j op(B_j) (+ bias_j), A_j [M, K] row-major (ld lda),
 * op(B) = B^T (B [N, K], b_kmajor = 0: a Linear / head forward) or B (B [K, N], b_kmajor = 1: an
 * input gradient), c_relu (NULL or ld ldr): relu of the result too.  ONE launch of 64 x 128 fp32-MFMA
 * tiles over every job's tiles, K split in `splits` chunks into fp32 slabs; ONE launch adds the slabs
 * in split order (+ bias, relu copy).  splits = 1: the tiles write C (+ bias, relu copy) themselves,
 * no second launch, no workspace (NULL allowed).  Replaces the per-head GEMM calls (ATen mm of GATConv lin_l,
 * by linearity per head: hicgat.dist's aggregate-first form).  K, N, every ld a multiple of 4, every
 * pointer 16-B aligned (else HICGAT_EUNSUPPORTED); at most 8 jobs.
 * Workspace: hicgat_gemm_rows_grouped_workspace_bytes(same jobs, splits). */
typedef struct hicgat_gemm_job {
  const float *a;
  int64_t lda;
  const float *b;
  int64_t ldb;
  float *c;
  int64_t ldc;
  float *c_relu;
  int64_t ldr;
  const float *bias;
  int M, N, K;
} hicgat_gemm_job;
size_t hicgat_gemm_rows_grouped_workspace_bytes(const hicgat_gemm_job *jobs, int n, int splits);
int hicgat_gemm_rows_grouped(const hicgat_gemm_job *jobs, int n, int b_kmajor, int splits, void *workspace,
                             size_t workspace_bytes, hicgat_stream_t stream);
/* out[n] = sum_k A[k][n] over K rows (a Linear bias gradient), deterministic two-stage. */
int hicgat_colsum(const float *A, int64_t lda, int K, int N, float *out, int accumulate, void *workspace,
                  size_t workspace_bytes, hicgat_stream_t stream);
size_t hicgat_colsum_workspace_bytes(int K, int N);

/* ---- a6: LayerNorm + ReLU (+ residual) of the flagship tail (models.py:641-655) --------------
 * z = relu(LayerNorm(y) * gamma + beta) + res (res may be NULL), W in {64, 128, 256}, eps as in
 * torch.nn.LayerNorm (biased variance); row_stats [M, 2] = (mean, rstd) saved for the backward.
 * Backward: dy (ld lddy), dgamma/dbeta (accumulate != 0 adds into them); dres = dz: the caller's
 * dz, or (dres != NULL) also written to dres (ld lddres), e.g. beside dy in one packed [dy | dres]
 * row for the fused dual-Linear backward.  workspace: hicgat_ln_relu_res_workspace_bytes(W). */
int hicgat_ln_relu_res_fwd(const float *y, int64_t ldy, int M, int W, const float *gamma, const float *beta,
                           float eps, const float *res, int64_t ldr, float *z, float *row_stats,
                           hicgat_stream_t stream);
int hicgat_ln_relu_res_bwd(const float *dz, const float *y, int64_t ldy, int M, int W, const float *row_stats,
                           const float *gamma, const float *beta, float *dy, int64_t lddy, float *dres,
                           int64_t lddres, float *dgamma, float *dbeta, int accumulate, void *workspace,
                           size_t workspace_bytes, hicgat_stream_t stream);
size_t hicgat_ln_relu_res_workspace_bytes(int W);
/* dgamma = dbeta = NULL in hicgat_ln_relu_res_bwd: only dy (and dres) are written and the per-wave
 * partials stay in the workspace; this call then reduces them into dgamma / dbeta (fixed order, the
 * same bits as the one-call form) -- on another stream after an event, so the parameter
 * reduction leaves the backward's critical path. */
int hicgat_ln_relu_res_bwd_params(int W, float *dgamma, float *dbeta, int accumulate, void *workspace,
                                  size_t workspace_bytes, hicgat_stream_t stream);

/* ---- The flagship's MLP tail forward in one launch (tail_fused.hip; replaces the dual-Linear GEMMs,
 * ln_relu_res passes and Linear GEMMs of models.py:637-659 for GATNetSelectiveResidualsUpdated) ----
 * x [M][512] (ld ldx, 16-B aligned rows): the GATConv output after its relu.  W1c [512][512] = [W_densea;
 * W_align_densea], b1c [512]; g1/be1 [256] = norm_a; W2c [256][256] = [W_dense1; W_align_dense1], b2c
 * [256]; g2/be2 [128] = norm1; W3 [64][128] / b3 = dense2; g3/be3 [64] = norm2; W4 [3][64] / b4 = dense3.
 * Writes what the backward reads: Y1 [M][512] (block-1 GEMM + bias), st1 [M][2] (mean, rstd), z1
 * [M][256], Y2 [M][256], st2, z2 [M][128], y3 [M][64], st3, z3 [M][64], and coords [M][3].
 * 16 rows per workgroup, fp32 MFMA (16x16x4), LayerNorm eps inside the square root. */
int hicgat_tail_fwd_fused(const float *x, int64_t ldx, int M, const float *W1c, const float *b1c, const float *g1,
                          const float *be1, const float *W2c, const float *b2c, const float *g2, const float *be2,
                          const float *W3, const float *b3, const float *g3, const float *be3, const float *W4,
                          const float *b4, float eps, float *Y1, float *st1, float *z1, float *Y2, float *st2,
                          float *z2, float *y3, float *st3, float *z3, float *coords, const void *pack,
                          hicgat_stream_t stream);
/* pack: NULL, or the packed weight copies hicgat_tail_pack made from THESE W1c / W2c (and, for the head
 * forms, Wh): the kernels then read W1c, W2c and Wh from it (1 KB contiguous per wave load instead of
 * 16 rows x 64 B: the vector memory path serves the row-major rows at 16 B per clock per CU, a quarter
 * of the contiguous rate, and that set the pace of the kernels' GEMM phases); results bitwise the
 * row-major form.  W3 / W4 are always read row-major.  hicgat_tail_pack_bytes(): the buffer's size.
 * Not a reference interface: the copies are a layout of the same parameters.  The library records,
 * per pack buffer, whether its last hicgat_tail_pack included Wh: the head-fused forms
 * (hicgat_tail_{fwd,bwd}_fused_heads) return HICGAT_EINVAL for a pack made with Wh = NULL. */
size_t hicgat_tail_pack_bytes(void);
int hicgat_tail_pack(const float *W1c, const float *W2c, const float *Wh, void *pack, size_t pack_bytes,
                     hicgat_stream_t stream);
/* The same tail's backward input-gradient chain in one launch: from dcoords [M][3] and the forward's
 * Y1, st1, Y2, st2, y3, st3 (hicgat_tail_fwd_fused), with W4 = dense3.weight [3][64], W3 = dense2.weight
 * [64][128], W2c = [W_dense1; W_align_dense1] [256][256], W1c = [W_densea; W_align_densea] [512][512],
 * g1/be1 = norm_a, g2/be2 = norm1, g3/be3 = norm2: writes dx [M][512] (the gradient of the tail's
 * input), dY1 [M][512] = [dy | dres] of block 1, dY2 [M][256] of block 2, dy3 [M][64] (dense2's output
 * gradient) -- the inputs of the weight-gradient GEMMs -- and each LayerNorm's dgamma/dbeta partials
 * into ws1 / ws2 / ws3: rows
 * [0, ceil(M/16)) of a [.][2W] = [dgamma | dbeta] matrix, one per 16-row workgroup (its waves'
 * partials added in wave order; the rows' column sums, e.g. hicgat_colsum, are dgamma / dbeta); each
 * workspace at least hicgat_tail_bwd_workspace_bytes(M, W) for W = 256 / 128 / 64.
 * hicgat_tail_bwd_waves(): the waves per workgroup of both tail kernels. */
int hicgat_tail_bwd_waves(void);
size_t hicgat_tail_bwd_workspace_bytes(int M, int W);
int hicgat_tail_bwd_fused(const float *dcoords, int M, const float *Y1, const float *st1, const float *Y2,
                          const float *st2, const float *y3, const float *st3, const float *W4, const float *W3,
                          const float *W2c, const float *W1c, const float *g1, const float *be1, const float *g2,
                          const float *be2, const float *g3, const float *be3, float *dx, float *dY1, float *dY2,
                          float *dy3, void *ws1, size_t ws1_bytes, void *ws2, size_t ws2_bytes, void *ws3,
                          size_t ws3_bytes, const void *pack, hicgat_stream_t stream);
/* The head-fused forms for the sharded aggregate-first GATConv (hicgat.dist "xagg"; the GATConv of
 * models.py:619 by linearity per head, then the tail): the forward forms the tail's input rows
 * itself, Y0[:, 256h:256h+256] = xa^h W_h^T + b^h (xa^h = xa + h * xa_head_stride, [M][ld_xa]; W_h =
 * rows 256h.. of lin_l's weight Wh [512][512]; bh [512]) and O = relu(Y0) (both [M][512], written),
 * replacing the per-head GEMM launches and their slab sum; then the tail as hicgat_tail_fwd_fused.
 * The backward runs the chain of hicgat_tail_bwd_fused and, instead of writing dx, the GATConv's rows
 * backward and its input-gradient GEMM: dout = dx * (Y0 > 0) (act = 1; act = 0: dout = dx) into
 * dout [M][512], delta^h = <dout^h, Y0^h - b^h> into row_stats[8r + 4 + h] (its [4:6] S3 values move
 * to [6:8], as hicgat_xagg_rows_bwd does), dxa [M][1024] = [dout^0 W_0 | dout^1 W_1].  Both need
 * hicgat_tail_bwd_waves() == 8 (else HICGAT_EUNSUPPORTED). */
int hicgat_tail_fwd_fused_heads(const float *xa, int64_t ld_xa, int64_t xa_head_stride, const float *Wh,
                                const float *bh, float *Y0, float *O, int M, const float *W1c, const float *b1c,
                                const float *g1, const float *be1, const float *W2c, const float *b2c, const float *g2,
                                const float *be2, const float *W3, const float *b3, const float *g3, const float *be3,
                                const float *W4, const float *b4, float eps, float *Y1, float *st1, float *z1,
                                float *Y2, float *st2, float *z2, float *y3, float *st3, float *z3, float *coords,
                                const void *pack, hicgat_stream_t stream);
int hicgat_tail_bwd_fused_heads(const float *dcoords, int M, const float *Y1, const float *st1, const float *Y2,
                                const float *st2, const float *y3, const float *st3, const float *W4, const float *W3,
                                const float *W2c, const float *W1c, const float *g1, const float *be1, const float *g2,
                                const float *be2, const float *g3, const float *be3, float *dY1, float *dY2,
                                float *dy3, void *ws1, size_t ws1_bytes, void *ws2, size_t ws2_bytes, void *ws3,
                                size_t ws3_bytes, int act, const float *Y0, const float *Wh, const float *bh,
                                float *dout, float *row_stats, float *dxa, const void *pack, hicgat_stream_t stream);
/* The plain tail's backward with the single-GPU GATConv's gather-free rows pass in its epilogue
 * (hicgat_gat_agg_bwd_rows on the dx rows while they are in LDS, same arithmetic, bitwise): no dx is
 * written; dout [M][512] = dx [y > 0] (act != 0) or dx, and row_stats[8i + 4 .. 8i + 8) = (delta,
 * da_dst) from the forward's S3 there, for y = the GATConv's relu output (the tail's input rows),
 * out2 and bias of hicgat_gat_agg_fwd_act.  One row per wave: HICGAT_EUNSUPPORTED unless the kernels
 * run 16 waves (hicgat_tail_bwd_waves). */
int hicgat_tail_bwd_fused_rows(const float *dcoords, int M, const float *Y1, const float *st1, const float *Y2,
                               const float *st2, const float *y3, const float *st3, const float *W4, const float *W3,
                               const float *W2c, const float *W1c, const float *g1, const float *be1, const float *g2,
                               const float *be2, const float *g3, const float *be3, float *dY1, float *dY2,
                               float *dy3, void *ws1, size_t ws1_bytes, void *ws2, size_t ws2_bytes, void *ws3,
                               size_t ws3_bytes, int act, const float *y, const float *out2, const float *bias,
                               float *dout, float *row_stats, const void *pack, hicgat_stream_t stream);

/* ---- f1: SAGEConv of the baseline model Net (layers.py:41-79, models.py:14-55) ----------------
 * hicgat_sage_weights: the float32 edge weight w of every entry of the (set_diag'd) device CSR --
 * the networkx weight utils.load_input assigns (utils.py:37-52): A[max(i,j), min(i,j)] when
 * non-zero, else A[min, max]; 0 on the self loops -- and inv_deg[i] = 1 / sum_j w_ij, the
 * SAGEConv.adjust_weights normaliser (layers.py:41-53; sum in ascending column order).
 * hicgat_sage_agg: z[i, 0:F] = sum_{j != i} (inv_deg[i] * w_ij) x[j]  (matmul(norm_mat, x), :74-77)
 * over rows [row_begin, row_end); transpose != 0 weights by inv_deg[j] instead (the adjoint,
 * d agg -> d x); write_trunc != 0 also writes z[i, F:2F] = trunc(x[i]) (x.long().float(), :64). */
int hicgat_sage_weights(const double *A, int N, int64_t lda, const int32_t *rowptr, const int32_t *col,
                        float *weights, float *inv_deg, hicgat_stream_t stream);
int hicgat_sage_agg(const int32_t *rowptr, const int32_t *col, const float *weights, const float *inv_deg,
                    int N, int F, int row_begin, int row_end, const float *x, int transpose, int write_trunc,
                    float *z, int64_t ldz, hicgat_stream_t stream);

/* ---- f2: Knight-Ruiz normalisation (r_utils.R:1-93 KRnorm, run by normalize.R from
 * HiC-GNN_main.py:85) -- the O(N^2) parts; the O(N) CG bookkeeping is the caller's (hicgat/kr.py).
 * A: float64 row-major n x n (leading dim lda), NaN entries count as 0.
 *   hicgat_kr_matvec: out_i = x_i * sum_j A_ij x_j p_j (+ v_i p_i if v != NULL)   (r_utils.R:24,42,64)
 *   hicgat_kr_scale:  out_ij = rint(((x_i A_ij) x_j) * 1e6) / 1e6, NaN kept        (r_utils.R:74-89) */
int hicgat_kr_matvec(const double *A, int64_t lda, int n, const double *x, const double *p, const double *v,
                     double *out, hicgat_stream_t stream);
int hicgat_kr_scale(const double *A, int64_t lda, int n, const double *x, double *out, int64_t ldo,
                    hicgat_stream_t stream);

/* ---- f4: node2vec embeddings (HiC_GAT_generalize_directly.py:150-155: node2vec 0.4 + gensim 4
 * Word2Vec, restated; see csrc/node2vec.hip).
 * hicgat_n2v_walks: nwalks biased walks of walk_length nodes from starts[w] over the weighted CSR
 *   (rows sorted, cum_weights[k] = inclusive per-row cumulative edge weight); second-order factors
 *   1/p (back to the previous node), 1 (a neighbour of it), 1/q (otherwise), by rejection sampling
 *   with a counter-based RNG (deterministic for a seed); a walk that reaches a node without
 *   neighbours ends and is padded with -1.  walks [nwalks, walk_length] int32.
 * hicgat_n2v_sgns_epoch: one skip-gram negative-sampling epoch over the walks (window, negative,
 *   learning rate decaying linearly from alpha0 to alpha1 over `epochs`), gensim's downsampling
 *   (keep_prob[v]) and unigram^0.75 negative table (cum_table[V], cumulative), syn0 / syn1 [V, D]
 *   fp32 (D a multiple of 64, <= 1024; negative <= 7), updated Hogwild-style by at most max_waves walks in flight
 *   (one wave per walk; a small vocabulary wants few, the reference trains with one worker). */
int hicgat_n2v_walks(const int32_t *rowptr, const int32_t *col, const float *cum_weights, int N,
                     const int32_t *starts, int nwalks, int walk_length, float p, float q, uint64_t seed,
                     int32_t *walks, hicgat_stream_t stream);
int hicgat_n2v_sgns_epoch(const int32_t *walks, int nwalks, int walk_length, const float *keep_prob,
                          const uint32_t *cum_table, int V, int D, int window, int negative, float alpha0,
                          float alpha1, int epoch, int epochs, uint64_t seed, int max_waves, float *syn0,
                          float *syn1, hicgat_stream_t stream);

/* ---- a10 (part): torch.optim.Adam step (HiC-GNN_main.py:118,130) over one flat fp32 buffer ----
 * Same arithmetic as torch's single-tensor CPU Adam (lerp / addcmul / addcdiv, no weight decay):
 *   m = fma(1-b1, g-m, m); v = fma((1-b2)*g, g, b2*v);
 *   p += (-lr/(1-b1^t) * m) / (sqrt(v)/sqrt(1-b2^t) + eps). */
int hicgat_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                     double lr, double beta1, double beta2, double eps, int64_t step,
                     hicgat_stream_t stream);
/* Graph-replayable form: the step count lives on the device (*step_counter = steps done so far,
 * incremented by the call), the per-step constants come from table[step] = (-lr/(1-b1^t),
 * sqrt(1-b2^t)) for t = step+1, computed on the host exactly like hicgat_adam_step does. */
int hicgat_adam_step_table(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                           int64_t n, double beta1, double beta2, double eps, const float *table,
                           int64_t table_len, int64_t *step_counter, hicgat_stream_t stream);
/* The same; counted = 1: this step's increment of *step_counter already happened in an earlier
 * launch of the step (hicgat_xagg_logits_zero), so the table row is *step_counter - 1 and no
 * increment follows (one launch fewer); counted = 0 is hicgat_adam_step_table. */
int hicgat_adam_step_table_ex(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                              int64_t n, double beta1, double beta2, double eps, const float *table,
                              int64_t table_len, int64_t *step_counter, int counted, hicgat_stream_t stream);
/* A step's first launch: grad[0, n) = 0 (zero_grad, HiC-GNN_main.py:124) and, with step_counter
 * (NULL: none), *step_counter += 1 (the step's Adam then uses counted = 1).  grad 16-B aligned. */
int hicgat_step_begin(float *grad, int64_t n, int64_t *step_counter, hicgat_stream_t stream);
/* hicgat_step_begin and hicgat_tail_pack(W1c, W2c, Wh, pack) in ONE launch (the step's first: the
 * weights change only at the previous step's Adam), so the one-kernel tail's packed copies cost no
 * launch of their own on the step's chain.  Same arguments and checks as the two. */
int hicgat_step_begin_pack(float *grad, int64_t n, int64_t *step_counter, const float *W1c, const float *W2c,
                           const float *Wh, void *pack, size_t pack_bytes, hicgat_stream_t stream);

/* ---- measurement infrastructure (no reference counterpart) ----------------------------------
 * An emulated collective for the simulated P-rank step (bench.py --simulate-world,
 * hicgat.dist.SimComm): `workgroups` x `threads` threads resident on the device for `us`
 * microseconds of wall time, enqueued where the RCCL call would be, so the captured rank step
 * shows the modeled collective's duration, its overlap with the kernels on other streams and the
 * CU slots it holds.  Not used by the training path. */
int hicgat_sim_collective(float us, int workgroups, int threads, hicgat_stream_t stream);

/* ---- streams and stamps (host plumbing; no reference counterpart) ----------------------------
 * A non-blocking HIP stream at `priority` (hipStreamCreateWithPriority), made ONCE per device and
 * name by hicgat.streams and kept for the process: every side / comm / warm-up stream of the step
 * is one of these, never a stream from torch's round-robin pool (which aliases after 32 requests),
 * so two lanes of one step are always two streams.  *out receives the stream. */
int hicgat_stream_create(int priority, hicgat_stream_t *out);
/* out[slot] = the device's steady wall clock (100 MHz counter) when this one-wave launch runs on
 * `stream`: enqueued at fork / join points of a captured step it records, per replay, when each
 * branch started and ended (tests/test_gpu_overlap.py).  out 8-B aligned, slot >= 0. */
int hicgat_wall_stamp(unsigned long long *out, int slot, hicgat_stream_t stream);
#ifdef __cplusplus
}
#endif
#endif /* HICGAT_H */
