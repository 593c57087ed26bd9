// All-pairs 3-D distance, MSE + Pearson moments and their gradient on gfx950 (a7, a8, a9).
//
// Reference: out = torch.cdist(c, c, p=2) (models.py:661) -> MSELoss()(out, truth)
// (HiC-GNN_main.py:127), scipy pearsonr of the triu pairs (HiC_GAT_generalize_directly.py:220), and
// the contrastive loss 0.1 * mean_{i<j} |T_ij - D_ij| (train_and_test_same_res_GAT_node2vec.py:107-134).
// The reference materialises D [N, N] (and its grad) in HBM; the fused kernel here streams the
// truth matrix once, only its upper-triangle 128x128 tiles, and never stores D.
//
// Tile kernel: one 256-thread block per 128x128 tile; thread (ty, tx) in a 16x16 grid owns rows
// {4ty..4ty+3, 64+4ty..} x cols {4tx..4tx+3, 64+4tx..}, so every T row segment is two coalesced
// 256 B float4 sweeps.  Per pair it forms d, r = d - t, the moments and w = r/d, and accumulates
// w*(c_i - c_j) into row partials (reduced over the 16 tx lanes) and column partials (reduced over
// ty through LDS).  Partials go to a [tile][2][128] float4 slab and a second kernel adds, per row,
// the slabs of every tile touching it in a fixed order: bitwise reproducible, no float atomics.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "common.hpp"

namespace hicgat {

constexpr int BT = 128;
enum { MODE_SYM = 0, MODE_FULL = 1 };
// loss kinds (include/hicgat.h): the KIND template parameter below
enum { KIND_MSE = HICGAT_LOSS_MSE, KIND_COMBINED = HICGAT_LOSS_COMBINED, KIND_CONTRASTIVE = HICGAT_LOSS_CONTRASTIVE };

// d|r|/dr = sign(r) with sign(0) = 0 (torch.abs's backward, sgn), times inv = 1/d
__device__ __forceinline__ float sgn_inv(float r, float inv) { return r == 0.f ? 0.f : copysignf(inv, r); }

__host__ __device__ inline int pd_nb(int N) { return (N + BT - 1) / BT; }
__host__ __device__ inline int64_t tri_start(int64_t I, int64_t nb) { return I * nb - I * (I - 1) / 2; }

__device__ inline void tri_decode(int64_t t, int nb, int &I, int &J) {
  const double b = 2.0 * nb + 1.0;
  int64_t Ii = (int64_t)floor((b - sqrt(b * b - 8.0 * (double)t)) * 0.5);
  if (Ii < 0) Ii = 0;
  if (Ii > nb - 1) Ii = nb - 1;
  while (Ii > 0 && tri_start(Ii, nb) > t) --Ii;
  while (Ii + 1 < nb && tri_start(Ii + 1, nb) <= t) ++Ii;
  // block-uniform: into SGPRs, so every branch on I / J (interior vs edge tiles) is a scalar
  // branch, not an if-converted (both paths) VALU select
  I = __builtin_amdgcn_readfirstlane((int)Ii);
  J = __builtin_amdgcn_readfirstlane((int)(Ii + (t - tri_start(Ii, nb))));
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 16 lanes of a DPP row (the 16 tx lanes sharing ty): row rotations by 8 and 4, then
// quad permutes (xor 2, xor 1); VALU-only, every lane ends with the row sum.
__device__ __forceinline__ float sum16(float v) {
  v += dpp<0x128>(v);   // row_ror:8
  v += dpp<0x124>(v);   // row_ror:4
  v += dpp<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp<0xB1>(v);    // quad_perm [1,0,3,2]
  return v;
}


// v + the values of lanes l^16, l^32 and l^48 (ds_bpermute shuffles; a v_permlane16/32_swap form
// measured slower: the loss chain 0.162 vs 0.157 ms, profiles/r04h_kbench_pairdist.txt)
__device__ __forceinline__ float sum_rows4(float v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  const int2 p = *reinterpret_cast<int2 *>(&v);
  int2 q;
  q.x = __shfl_xor(p.x, m);
  q.y = __shfl_xor(p.y, m);
  return *reinterpret_cast<double *>(&q);
}

// Row partials of the background form: each thread's 8-column partial of every row it touches goes
// to LDS (stride kRowPad float4: 16 lanes of a row-sum read hit distinct banks) and threads 128..255
// add the 16 per row in tx order at the end, while 0..127 add the column partials -- instead of
// three 16-lane DPP sums per row inside the pair loop (~20 % of its VALU issue).
constexpr int kRowPad = 17;

// Per-thread accumulators of one tile: the moments and the column partials of its 8 columns.
struct TileAcc {
  float L = 0.f, sd = 0.f, sdd = 0.f, sdt = 0.f, st = 0.f, stt = 0.f, dg = 0.f;
  float ax[8], ay[8], az[8];
};

// The 8 rows x 8 columns of one thread.  MASK: the diagonal and the edge tiles (row / column
// bounds, i < j on the diagonal, the diagonal moment); interior tiles take MASK = false and do
// no per-pair selection at all.  d2 == 0 (coincident points) gives inv = 1e30, d = 0 and a finite
// w times dx = dy = dz = 0, i.e. no gradient -- torch's _euclidean_dist_backward masks it too.
template <int MODE, bool VEC, int KIND, bool MASK, int K0, int K1, bool BG = false, bool RLDS = false>
__device__ __forceinline__ void tile_rows(const float *__restrict__ T, int64_t ldt, int64_t row0, int64_t col0,
                                          int N, int I, int J, float bg,
                                          const float *tile, const float (*sc)[BT][3], int tx, int ty,
                                          const float *cx, const float *cy, const float *cz, const int *gj,
                                          float4 *__restrict__ prow, TileAcc &A, float4 *rowpart) {
  constexpr bool PEARSON = KIND == KIND_COMBINED, ABSL = KIND == KIND_CONTRASTIVE;
#pragma unroll 1
  for (int k = K0; k < K1; ++k) {
    const int lr = ty * 4 + (k & 3) + (k >> 2) * 64;
    const int gi = I * BT + lr;
    const float rx = sc[0][lr][0], ry = sc[0][lr][1], rz = sc[0][lr][2];
    float tv[8];
    if (BG) {   // background form: every pair at the background value, the support added later
#pragma unroll
      for (int q = 0; q < 8; ++q) tv[q] = bg;
    } else if (VEC) {  // from the LDS image of the tile (conflict-free ds_read_b128: 16 lanes = one row)
      const float4 a = *reinterpret_cast<const float4 *>(&tile[lr * BT + tx * 4]);
      const float4 b = *reinterpret_cast<const float4 *>(&tile[lr * BT + 64 + tx * 4]);
      tv[0] = a.x; tv[1] = a.y; tv[2] = a.z; tv[3] = a.w;
      tv[4] = b.x; tv[5] = b.y; tv[6] = b.z; tv[7] = b.w;
    } else if (gi < N) {
      const float *trow = T + (size_t)(gi - row0) * ldt + (size_t)((int64_t)J * BT - col0);
#pragma unroll
      for (int q = 0; q < 8; ++q) tv[q] = gj[q] < N ? trow[tx * 4 + (q & 3) + (q >> 2) * 64] : 0.f;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) tv[q] = 0.f;
    }
    float px = 0.f, py = 0.f, pz = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float dx = rx - cx[q], dy = ry - cy[q], dz = rz - cz[q];
      const float d2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
      // one v_rsq for both d and 1/d (1-2 ulp; the reference's own mm-formula cdist is far
      // coarser)
      const float inv = fminf(__builtin_amdgcn_rsqf(d2), 1e30f);
      const float d = d2 * inv;
      const float tt = tv[q];
      float w;
      if (MODE == MODE_SYM) {
        const float r = d - tt;
        if (MASK) {
          bool valid = gi < N && gj[q] < N;
          // (D_ii - T_ii)^2 = T_ii^2 (MSE over all N^2 entries; the contrastive loss is over i < j only)
          if (!BG && !ABSL && valid && gi == gj[q]) A.dg = fmaf(tt, tt, A.dg);
          valid = valid && (I != J || gi < gj[q]);
          if (valid) {
            A.L = ABSL ? A.L + fabsf(r) : fmaf(r, r, A.L);
            if (PEARSON) {
              A.sd += d;
              A.sdd = fmaf(d, d, A.sdd);
              A.sdt = fmaf(d, tt, A.sdt);
              A.st += tt;
              A.stt = fmaf(tt, tt, A.stt);
            }
          }
          w = valid ? (ABSL ? sgn_inv(r, inv) : r * inv) : 0.f;
        } else {
          A.L = ABSL ? A.L + fabsf(r) : fmaf(r, r, A.L);
          if (PEARSON) {
            A.sd += d;
            A.sdd = fmaf(d, d, A.sdd);
            A.sdt = fmaf(d, tt, A.sdt);
            A.st += tt;
            A.stt = fmaf(tt, tt, A.stt);
          }
          w = ABSL ? sgn_inv(r, inv) : r * inv;
        }
      } else {
        w = tt * inv;
        if (MASK) w = (gi < N && gj[q] < N && gi != gj[q]) ? w : 0.f;
      }
      px = fmaf(w, dx, px);
      py = fmaf(w, dy, py);
      pz = fmaf(w, dz, pz);
      A.ax[q] = fmaf(-w, dx, A.ax[q]);
      A.ay[q] = fmaf(-w, dy, A.ay[q]);
      A.az[q] = fmaf(-w, dz, A.az[q]);
    }
    if constexpr (RLDS) {   // the thread's 8-column partial of row lr; the 16 of a row are added at the end
      rowpart[lr * kRowPad + tx] = make_float4(px, py, pz, 0.f);
    } else {
      px = sum16(px);
      py = sum16(py);
      pz = sum16(pz);
      if (tx == 0) prow[lr] = make_float4(px, py, pz, 0.f);
    }
  }
}

// Interior tiles of the training loss (MODE_SYM, T from the LDS image, no masks) in packed fp32:
// the thread's 8 columns as 4 float2 pairs, so the subtractions, multiplies and FMAs issue as
// v_pk_{add,mul,fma}_f32 (two pairs per instruction); v_rsq stays scalar.
typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND, int K0, int K1, bool BG = false, bool RLDS = false>
__device__ __forceinline__ void tile_rows_pk(const float *tile, float bg, const float (*sc)[BT][3], int tx, int ty,
                                             const float *cx, const float *cy, const float *cz,
                                             float4 *__restrict__ prow, TileAcc &A, float4 *rowpart) {
  constexpr bool PEARSON = KIND == KIND_COMBINED, ABSL = KIND == KIND_CONTRASTIVE;
  f2 cx2[4], cy2[4], cz2[4], ax2[4], ay2[4], az2[4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    cx2[h] = f2{cx[2 * h], cx[2 * h + 1]};
    cy2[h] = f2{cy[2 * h], cy[2 * h + 1]};
    cz2[h] = f2{cz[2 * h], cz[2 * h + 1]};
    ax2[h] = f2{A.ax[2 * h], A.ax[2 * h + 1]};
    ay2[h] = f2{A.ay[2 * h], A.ay[2 * h + 1]};
    az2[h] = f2{A.az[2 * h], A.az[2 * h + 1]};
  }
  const f2 z2 = f2{0.f, 0.f};
  f2 L2 = z2, sd2 = z2, sdd2 = z2, sdt2 = z2, st2 = z2, stt2 = z2;
#pragma unroll 2   // rows per iteration (the next row's LDS reads in flight)
  for (int k = K0; k < K1; ++k) {
    const int lr = ty * 4 + (k & 3) + (k >> 2) * 64;
    const f2 rx = f2{sc[0][lr][0], sc[0][lr][0]}, ry = f2{sc[0][lr][1], sc[0][lr][1]},
             rz = f2{sc[0][lr][2], sc[0][lr][2]};
    f2 tv[4];
    if constexpr (BG) {
#pragma unroll
      for (int h = 0; h < 4; ++h) tv[h] = f2{bg, bg};
    } else {
      const float4 a = *reinterpret_cast<const float4 *>(&tile[lr * BT + tx * 4]);
      const float4 b = *reinterpret_cast<const float4 *>(&tile[lr * BT + 64 + tx * 4]);
      tv[0] = f2{a.x, a.y};
      tv[1] = f2{a.z, a.w};
      tv[2] = f2{b.x, b.y};
      tv[3] = f2{b.z, b.w};
    }
    f2 px = z2, py = z2, pz = z2;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const f2 dx = rx - cx2[h], dy = ry - cy2[h], dz = rz - cz2[h];
      // d2 + 2^-100 (below one ulp of any d2 that is not ~0): coincident points give a finite
      // inv = 2^50, d = 2^-50 and w * (dx, dy, dz) = 0 -- the clamp of the generic path for free
      const f2 d2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy,
                                              __builtin_elementwise_fma(dz, dz, f2{0x1.0p-100f, 0x1.0p-100f})));
      const f2 inv = f2{__builtin_amdgcn_rsqf(d2.x), __builtin_amdgcn_rsqf(d2.y)};
      const f2 d = d2 * inv;
      const f2 r = d - tv[h];
      if constexpr (ABSL) L2 += __builtin_elementwise_abs(r);
      else L2 = __builtin_elementwise_fma(r, r, L2);
      if (PEARSON) {
        sd2 += d;
        sdd2 = __builtin_elementwise_fma(d, d, sdd2);
        if constexpr (!BG) {   // background form: t = bg at every pair, these three follow below
          sdt2 = __builtin_elementwise_fma(d, tv[h], sdt2);
          st2 += tv[h];
          stt2 = __builtin_elementwise_fma(tv[h], tv[h], stt2);
        }
      }
      const f2 w = ABSL ? f2{sgn_inv(r.x, inv.x), sgn_inv(r.y, inv.y)} : r * inv;
      px = __builtin_elementwise_fma(w, dx, px);
      py = __builtin_elementwise_fma(w, dy, py);
      pz = __builtin_elementwise_fma(w, dz, pz);
      ax2[h] = __builtin_elementwise_fma(-w, dx, ax2[h]);
      ay2[h] = __builtin_elementwise_fma(-w, dy, ay2[h]);
      az2[h] = __builtin_elementwise_fma(-w, dz, az2[h]);
    }
    if constexpr (RLDS) {
      rowpart[lr * kRowPad + tx] = make_float4(px.x + px.y, py.x + py.y, pz.x + pz.y, 0.f);
    } else {
      const float sx = sum16(px.x + px.y), sy = sum16(py.x + py.y), sz = sum16(pz.x + pz.y);
      if (tx == 0) prow[lr] = make_float4(sx, sy, sz, 0.f);
    }
  }
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    A.ax[2 * h] = ax2[h].x;
    A.ax[2 * h + 1] = ax2[h].y;
    A.ay[2 * h] = ay2[h].x;
    A.ay[2 * h + 1] = ay2[h].y;
    A.az[2 * h] = az2[h].x;
    A.az[2 * h + 1] = az2[h].y;
  }
  const float L = L2.x + L2.y;
  A.L += L;
  if (PEARSON) {
    const float sd = sd2.x + sd2.y;
    A.sd += sd;
    A.sdd += sdd2.x + sdd2.y;   // summed directly in every form: sum (d - bg)^2 + bg (2 sum d - n bg)
                                // cancels when d << bg (collapsed coordinates early in training)
    if constexpr (BG) {
      // t = bg at all 8 (K1 - K0) pairs: sum d t = bg sum d, sum t and sum t^2 by count (three packed
      // ops per two pairs out of the loop)
      constexpr float npair = 8.f * (K1 - K0);
      A.sdt = fmaf(bg, sd, A.sdt);
      A.st = fmaf(npair, bg, A.st);
      A.stt = fmaf(npair * bg, bg, A.stt);
    } else {
      A.sdt += sdt2.x + sdt2.y;
      A.st += st2.x + st2.y;
      A.stt += stt2.x + stt2.y;
    }
  }
}


// MODE_SYM: T = symmetric truth, tiles I <= J, pairs i < j, w = (d - t)/d (scale 4/N^2 later).
// MODE_FULL: T = upstream grad G of D, all tiles, pairs i != j, w = g/d.
// KIND: KIND_MSE: sum (d - t)^2; KIND_COMBINED: also the d / t moments of the Pearson term;
// KIND_CONTRASTIVE: sum |d - t| and w = sgn(d - t) / d.
// BG: the background form (T = bg at every pair; no T read, no diagonal term -- the support pass,
// pairdist_support_kernel, adds the entries that differ and the diagonal).
template <int KIND>
__device__ void support_block(const float *__restrict__ coords, float bg, int row_begin, int row_end,
                              const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col,
                              const float *__restrict__ val, const float *__restrict__ diag, float4 *__restrict__ corr,
                              double *__restrict__ mom, const int *__restrict__ cmap, int blk,
                              const float4 *__restrict__ cpad = nullptr);

// The support pass riding in the background-form tile launch (SUP): blocks [ntiles, ntiles +
// blocks) of the grid run pairdist_support_kernel's work for support block (blockIdx.x - ntiles).
struct SupportArgs {
  const int32_t *rowptr = nullptr, *col = nullptr;
  const float *val = nullptr, *diag = nullptr;
  float4 *corr = nullptr;
  double *mom = nullptr;
  int row_begin = 0, row_end = 0;
  int64_t ntiles = 0;
};

template <int MODE, bool VEC, int KIND, bool BG = false, bool SUP = false>
__global__ __launch_bounds__(256, 1) void pairdist_tile_kernel(const float *__restrict__ coords,
                                                            const float *__restrict__ T, int N,
                                                            int64_t ldt, int64_t row0, int64_t col0,
                                                            int nb, int64_t t0,
                                                            float4 *__restrict__ part,
                                                            double *__restrict__ mom, float bg,
                                                            const int *__restrict__ cmap = nullptr,
                                                            const SupportArgs sup = SupportArgs{},
                                                            float4 *__restrict__ cpad = nullptr) {
  static_assert(!BG || (MODE == MODE_SYM && !VEC), "the background form is the training loss without a T image");
  static_assert(!SUP || BG, "the support pass rides only in the background form's launch");
  if (SUP && (int64_t)blockIdx.x >= sup.ntiles) {   // block-uniform
    support_block<KIND>(coords, bg, sup.row_begin, sup.row_end, sup.rowptr, sup.col, sup.val, sup.diag, sup.corr,
                           sup.mom, cmap, (int)(blockIdx.x - sup.ntiles));
    return;
  }
  // one dynamic LDS array: [T tile 128x128 fp32 (VEC only)] -- 64 KiB, 16-B aligned
  extern __shared__ __attribute__((aligned(16))) float tile[];
  __shared__ float sc[2][BT][3];
  __shared__ float4 colred[4][BT];
  __shared__ double mred[4][7];
  constexpr bool RL = BG;
  __shared__ float4 rowpart_s[RL ? BT * kRowPad : 1];
  float4 *rowpart = RL ? rowpart_s : nullptr;
  const int64_t t = t0 + blockIdx.x;
  int I, J;
  if (MODE == MODE_SYM) {
    tri_decode(t, nb, I, J);
  } else {
    I = (int)(t / nb);
    J = (int)(t % nb);
  }
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4, lane = tid & 63, wv = tid >> 6;
  for (int k = tid; k < 2 * BT; k += 256) {
    const int which = k / BT, li = k % BT;
    const int g = (which ? J : I) * BT + li;
    float x = 0.f, y = 0.f, z = 0.f;
    if (g < N) {
      const size_t gc = cmap ? (size_t)cmap[g] : (size_t)g;   // cmap: global row -> coords row (sharded step)
      x = coords[3 * gc];
      y = coords[3 * gc + 1];
      z = coords[3 * gc + 2];
    }
    sc[which][li][0] = x;
    sc[which][li][1] = y;
    sc[which][li][2] = z;
    // the diagonal tile of row block I writes its rows' float4 copy for the support pass that follows
    if (cpad && I == J && which == 0 && g < N) cpad[g] = make_float4(x, y, z, 0.f);
  }
  if (VEC) {
    // LDS-DMA of the T tile (global_load_lds_dwordx4: each wave instruction moves 1 KiB = two 512-B
    // tile rows, wave-uniform LDS base + lane*16), each wave only the 32 rows its threads read:
    // rows 16w .. 16w+15 (k = 0..3 of tile_rows) first, then 64+16w .. 64+16w+15 (k = 4..7), so the
    // first half is computed while the second is in flight.  Rows past N are clamped to a valid row
    // (their values are masked); columns past N lie inside the padded leading dimension.  T may be
    // a band of the truth (rows from row0, columns from col0: a rank's share, hicgat.dist).
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r0 = (q < 8 ? 0 : 64) + wv * 16 + (q & 7) * 2;
      const int gi = min(I * BT + r0 + (lane >> 5), N - 1);
      const float *src = T + (size_t)(gi - row0) * ldt + (size_t)((int64_t)J * BT - col0) + (lane & 31) * 4;
      __builtin_amdgcn_global_load_lds(src, &tile[r0 * BT], 16, 0, 0);
    }
  }
  // sc[] (written above with ds_write) to all waves: LDS drain + raw barrier -- __syncthreads()
  // would also drain vmcnt and so wait for the whole tile
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  float cx[8], cy[8], cz[8];
  int gj[8];
  TileAcc A;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int lc = tx * 4 + (q & 3) + (q >> 2) * 64;
    gj[q] = J * BT + lc;
    cx[q] = sc[1][lc][0];
    cy[q] = sc[1][lc][1];
    cz[q] = sc[1][lc][2];
    A.ax[q] = A.ay[q] = A.az[q] = 0.f;
  }
  float4 *prow = part + (size_t)t * 2 * BT;
  const bool interior = I != J && (I + 1) * BT <= N && (J + 1) * BT <= N;   // block-uniform
  if (VEC) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");    // this wave's first 16 rows landed
  constexpr bool PK = (VEC || BG) && MODE == MODE_SYM;   // packed interior path (tile_rows_pk)
  if (interior) {
    if constexpr (PK) tile_rows_pk<KIND, 0, 4, BG, RL>(tile, bg, sc, tx, ty, cx, cy, cz, prow, A, rowpart);
    else tile_rows<MODE, VEC, KIND, false, 0, 4>(T, ldt, row0, col0, N, I, J, bg, tile, sc, tx, ty, cx, cy, cz, gj, prow, A, rowpart);
  } else {
    tile_rows<MODE, VEC, KIND, true, 0, 4, BG, RL>(T, ldt, row0, col0, N, I, J, bg, tile, sc, tx, ty, cx, cy, cz, gj, prow, A, rowpart);
  }
  if (VEC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // and the second 16
  if (interior) {
    if constexpr (PK) tile_rows_pk<KIND, 4, 8, BG, RL>(tile, bg, sc, tx, ty, cx, cy, cz, prow, A, rowpart);
    else tile_rows<MODE, VEC, KIND, false, 4, 8>(T, ldt, row0, col0, N, I, J, bg, tile, sc, tx, ty, cx, cy, cz, gj, prow, A, rowpart);
  } else {
    tile_rows<MODE, VEC, KIND, true, 4, 8, BG, RL>(T, ldt, row0, col0, N, I, J, bg, tile, sc, tx, ty, cx, cy, cz, gj, prow, A, rowpart);
  }

  // column partials: reduce over the 4 ty of this wave (lanes l, l^16, l^32, l^48), then waves
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    A.ax[q] = sum_rows4(A.ax[q]);
    A.ay[q] = sum_rows4(A.ay[q]);
    A.az[q] = sum_rows4(A.az[q]);
  }
  if (lane < 16) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      colred[wv][tx * 4 + (q & 3) + (q >> 2) * 64] = make_float4(A.ax[q], A.ay[q], A.az[q], 0.f);
  }
  if (MODE == MODE_SYM) {
    constexpr bool PEARSON = KIND == KIND_COMBINED;
    double m[7] = {A.L, A.sd, A.sdd, A.sdt, A.st, A.stt, A.dg};
#pragma unroll
    for (int c = 0; c < 7; ++c) {
      if (!PEARSON && c >= 1 && c <= 5) continue;
      for (int o = 32; o > 0; o >>= 1) m[c] += shfl_xor_d(m[c], o);
    }
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < 7; ++c) mred[wv][c] = m[c];
    }
  }
  __syncthreads();
  if (tid < BT) {
    float4 s = colred[0][tid];
#pragma unroll
    for (int w2 = 1; w2 < 4; ++w2) {
      const float4 o = colred[w2][tid];
      s.x += o.x;
      s.y += o.y;
      s.z += o.z;
    }
    prow[BT + tid] = s;
  } else if (RL) {
    const int lr = tid - BT;
    float4 s = rowpart[lr * kRowPad];
#pragma unroll
    for (int q = 1; q < 16; ++q) {
      const float4 o = rowpart[lr * kRowPad + q];
      s.x += o.x;
      s.y += o.y;
      s.z += o.z;
    }
    prow[lr] = make_float4(s.x, s.y, s.z, 0.f);
  }
  if (MODE == MODE_SYM && tid < 7) {
    mom[(size_t)t * 8 + tid] = ((mred[0][tid] + mred[1][tid]) + mred[2][tid]) + mred[3][tid];
  }
}

// dcoords[i] = scale * (sum of the row partials of tiles (R, *) + column partials of (*, R));
// ncol = column slabs per tile (1 here; the slab layout is [row partials | ncol column partials]).
// Block = 64 rows x 4 groups; group g adds the tiles J = g, g+4, ... of its row, then the 4 group
// sums are combined in group order (fixed order: bitwise reproducible).
constexpr int kRedGroups = 16;   // J-groups per row in pairdist_reduce (1024-thread blocks)

__device__ void moments_partial_block(const double *__restrict__ mom, int64_t t0, int64_t t1, int blk, int nblk,
                                      double *__restrict__ part);

// mom != NULL: the blocks from row_blocks on (gridDim.x - row_blocks of them) sum runs of the moment
// records [m0, m1) (tiles, then the support pass's blocks) into mpart instead (moments_partial_block);
// blocks [0, row_blocks) reduce the coordinate partials, plus the support pass's per-row term corr
// (background form) last.
__global__ __launch_bounds__(1024) void pairdist_reduce_kernel(const float4 *__restrict__ part, int ncol,
                                                               int N, int nb, int mode, int64_t t0,
                                                               int64_t t1, float scale,
                                                               float *__restrict__ dcoords,
                                                               const double *__restrict__ mom, int64_t m0, int64_t m1,
                                                               int row_blocks, double *__restrict__ mpart,
                                                               const float4 *__restrict__ corr, int corr_r0,
                                                               int corr_r1, double *__restrict__ dc64) {
  if (mom && (int)blockIdx.x >= row_blocks) {
    moments_partial_block(mom, m0, m1, (int)blockIdx.x - row_blocks, (int)gridDim.x - row_blocks, mpart);
    return;
  }
  __shared__ float4 red[kRedGroups][64];
  const int lr64 = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int gi = blockIdx.x * 64 + lr64;
  float sx = 0.f, sy = 0.f, sz = 0.f;
  if (gi < N) {
    const int R = gi / BT, lr = gi % BT;
#pragma unroll 2
    for (int J = grp; J < nb; J += kRedGroups) {
      int64_t trow, tcol;
      if (mode == MODE_SYM) {
        trow = J >= R ? tri_start(R, nb) + (J - R) : -1;
        tcol = J <= R ? tri_start(J, nb) + (R - J) : -1;
      } else {
        trow = (int64_t)R * nb + J;
        tcol = (int64_t)J * nb + R;
      }
      // slab of tile t: [row partials | ncol column-partial rows], (1 + ncol) x BT float4
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, c = a;
      const size_t st = (size_t)(1 + ncol) * BT;
      if (trow >= t0 && trow < t1) a = part[(size_t)trow * st + lr];
      if (tcol >= t0 && tcol < t1) {
        b = part[(size_t)tcol * st + BT + lr];
        if (ncol == 2) c = part[(size_t)tcol * st + 2 * BT + lr];
      }
      sx += a.x; sy += a.y; sz += a.z;
      sx += b.x; sy += b.y; sz += b.z;
      sx += c.x; sy += c.y; sz += c.z;
    }
  }
  red[grp][lr64] = make_float4(sx, sy, sz, 0.f);
  __syncthreads();
  if (grp == 0 && gi < N) {
    float4 s0 = red[0][lr64];
#pragma unroll
    for (int g = 1; g < kRedGroups; ++g) {
      const float4 o = red[g][lr64];
      s0.x += o.x; s0.y += o.y; s0.z += o.z;
    }
    if (corr && gi >= corr_r0 && gi < corr_r1) {
      const float4 o = corr[gi];
      s0.x += o.x; s0.y += o.y; s0.z += o.z;
    }
    const float gx = s0.x * scale, gy = s0.y * scale, gz = s0.z * scale;
    if (dc64) {   // the fp32 values, widened: straight into a caller's fp64 all-reduce buffer
      dc64[3 * (size_t)gi] = gx;
      dc64[3 * (size_t)gi + 1] = gy;
      dc64[3 * (size_t)gi + 2] = gz;
    } else {
      dcoords[3 * (size_t)gi] = gx;
      dcoords[3 * (size_t)gi + 1] = gy;
      dcoords[3 * (size_t)gi + 2] = gz;
    }
  }
}

// stats[7..10] and loss from the (all-reduced) moments stats[0..6]: mse, pearson r, alpha, total;
// contrastive: stats[7] = mean_{i<j} |T - D| (fp64, as the reference's float64 truth makes it),
// stats[8] = NaN, stats[9] = 0.1, stats[10] = total = 0.1 * stats[7].
__device__ void finalize_stats(int N, int loss_kind, double *__restrict__ stats, float *__restrict__ loss) {
  if (loss_kind == KIND_CONTRASTIVE) {
    const double M = 0.5 * (double)N * (double)(N - 1);
    const double mae = M > 0.0 ? stats[0] / M : 0.0;
    const double total = 0.1 * mae;
    stats[7] = mae;
    stats[8] = NAN;
    stats[9] = 0.1;
    stats[10] = total;
    stats[11] = 0.0;
    if (loss) loss[0] = (float)total;
    return;
  }
  const double n2 = (double)N * (double)N;
  const double mse = (2.0 * stats[0] + stats[6]) / n2;
  const double M = 0.5 * (double)N * (double)(N - 1);
  const double sd = stats[1], sdd = stats[2], sdt = stats[3], st = stats[4], stt = stats[5];
  const double cov = sdt - sd * st / M, vd = sdd - sd * sd / M, vt = stt - st * st / M;
  const double r = (vd > 0.0 && vt > 0.0) ? cov / sqrt(vd * vt) : NAN;
  // HiC_GAT_generalize_directly.py:223-225: alpha from mse_loss.item() (the fp32 value), then
  // total_loss = mse_loss + alpha*(1-r) evaluated as an fp32 tensor + scalar add.
  const float msef = (float)mse;
  const double alpha = fmin(1.0, 0.1 + 1.0 / ((double)msef + 1e-6));
  const float totalf = msef + (float)(alpha * (1.0 - r));
  stats[7] = mse;
  stats[8] = r;
  stats[9] = alpha;
  stats[10] = (double)totalf;
  stats[11] = 0.0;
  if (loss) loss[0] = loss_kind == 1 ? totalf : msef;
}

__global__ __launch_bounds__(64) void finalize_kernel(int N, int loss_kind, double *__restrict__ stats,
                                                      float *__restrict__ loss) {
  if (threadIdx.x == 0) finalize_stats(N, loss_kind, stats, loss);
}

// Tile moments over [t0,t1) in two fixed-order stages (deterministic): kMomBlocks extra blocks of
// pairdist_reduce_kernel each sum a contiguous tile run (256 threads, each a strided subset with
// its loads in flight, then a fixed tree) into part[b][0..6]; moments_finalize_kernel adds the
// kMomBlocks partials in block order into stats[0..6] and finalizes.  A rank's share whose partial
// moments are all-reduced before the finalize (the sharded step) with at most kOneBlockMoments
// records: ONE such block writes stats[0..6] itself (no moments_finalize launch).
constexpr int kMomBlocks = 64;
constexpr int64_t kOneBlockMoments = 4096;

__device__ void moments_partial_block(const double *__restrict__ mom, int64_t t0, int64_t t1, int blk, int nblk,
                                      double *__restrict__ part) {
  __shared__ double mred[7][256];
  const int tid = threadIdx.x;
  const int64_t per = (t1 - t0 + nblk - 1) / nblk;
  const int64_t b0 = t0 + (int64_t)blk * per, b1 = min(t1, b0 + per);
  double s[7] = {0, 0, 0, 0, 0, 0, 0};
  if (tid < 256) {
    for (int64_t t = b0 + tid; t < b1; t += 256) {
#pragma unroll
      for (int c = 0; c < 7; ++c) s[c] += mom[(size_t)t * 8 + c];
    }
#pragma unroll
    for (int c = 0; c < 7; ++c) mred[c][tid] = s[c];
  }
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
#pragma unroll
      for (int c = 0; c < 7; ++c) mred[c][tid] += mred[c][tid + o];
    }
    __syncthreads();
  }
  if (tid < 7) part[blk * 8 + tid] = mred[tid][0];
}

__global__ __launch_bounds__(64) void moments_finalize_kernel(const double *__restrict__ part, int N, int loss_kind,
                                                              double *__restrict__ stats, float *__restrict__ loss) {
  if (threadIdx.x < 7) {
    double s = 0.0;
    for (int b = 0; b < kMomBlocks; ++b) s += part[b * 8 + threadIdx.x];
    stats[threadIdx.x] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) finalize_stats(N, loss_kind, stats, loss);
}

// Support pass of the background form: T = bg except at the sorted CSR support (symmetric, no
// diagonal) and the diagonal.  One wave per row i, lanes over its support entries j:
//   gradient  corr[i] = sum_j ((d - t) - (d - bg)) / d * (c_i - c_j) = sum_j (bg - t) / d * (c_i - c_j)
//             (every j: the bulk tiles gave row i the bg term of each pair, as row or column partial);
//   moments   over j > i only (each pair once, in fp64), the support's change of the bulk's terms:
//             L += (d - t)^2 - (d - bg)^2, sdt += d (t - bg), st += t - bg, stt += t^2 - bg^2; and the
//             diagonal's (0 - T_ii)^2 into the dg moment.
// Contrastive (KIND_CONTRASTIVE): corr[i] = sum_j (sgn(d - t) - sgn(d - bg)) / d * (c_i - c_j), and
// L += |d - t| - |d - bg| over j > i; no diagonal term (the loss is over i < j only).
// d is formed exactly as in the bulk's interior path.  Per-block moment records (fixed order).
template <int KIND>
__device__ void support_block(const float *__restrict__ coords, float bg, int row_begin, int row_end,
                                              const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col,
                                              const float *__restrict__ val, const float *__restrict__ diag,
                                              float4 *__restrict__ corr, double *__restrict__ mom,
                                              const int *__restrict__ cmap, int blk, const float4 *__restrict__ cpad) {
  constexpr bool PEARSON = KIND == KIND_COMBINED, ABSL = KIND == KIND_CONTRASTIVE;
  __shared__ double mred[4][7];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = row_begin + blk * 4 + wv;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  double L = 0.0, sdt = 0.0, st = 0.0, stt = 0.0, dg = 0.0;   // the support's moment changes in fp64
  if (i < row_end) {   // wave-uniform
    const size_t ic = cmap ? (size_t)cmap[i] : (size_t)i;
    const float xi = coords[3 * ic], yi = coords[3 * ic + 1], zi = coords[3 * ic + 2];
    const int e1 = rowptr[i + 1];
    // four of the lane's entries per round, every index and coordinate load of the round issued before
    // its arithmetic (one wave per row: the col -> coordinate load chain was the pass's latency)
    constexpr int SU = 4;
    for (int e0 = rowptr[i] + lane; e0 < e1; e0 += 64 * SU) {
      int jj[SU];
      float tt[SU], cx[SU], cy[SU], cz[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int e = e0 + 64 * u;
        jj[u] = e < e1 ? col[e] : i;
        tt[u] = e < e1 ? val[e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const size_t jc = cmap ? (size_t)cmap[jj[u]] : (size_t)jj[u];
        // cpad: the coordinates as float4 rows (one 16-B load per lane instead of three 4-B loads)
        if (cpad) {
          const float4 c = cpad[jc];
          cx[u] = c.x; cy[u] = c.y; cz[u] = c.z;
        } else {
          cx[u] = coords[3 * jc]; cy[u] = coords[3 * jc + 1]; cz[u] = coords[3 * jc + 2];
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        if (e0 + 64 * u >= e1) break;
        const int j = jj[u];
        const float t = tt[u];
        const float dx = xi - cx[u], dy = yi - cy[u], dz = zi - cz[u];
        const float d2 = fmaf(dx, dx, fmaf(dy, dy, fmaf(dz, dz, 0x1.0p-100f)));
        const float inv = __builtin_amdgcn_rsqf(d2);
        const float d = d2 * inv;
        const float w = ABSL ? sgn_inv(d - t, inv) - sgn_inv(d - bg, inv) : (bg - t) * inv;
        gx = fmaf(w, dx, gx);
        gy = fmaf(w, dy, gy);
        gz = fmaf(w, dz, gz);
        if (j > i) {
          const double dd = d, td = t, bd = bg;
          const double r = dd - td, rb = dd - bd;
          L += ABSL ? fabs(r) - fabs(rb) : r * r - rb * rb;
          if (PEARSON) {
            sdt += dd * (td - bd);
            st += td - bd;
            stt += td * td - bd * bd;
          }
        }
      }
    }
    if (lane == 0 && !ABSL) {
      const float ti = diag[i];
      dg = (double)ti * (double)ti;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    gx += __shfl_xor(gx, o);
    gy += __shfl_xor(gy, o);
    gz += __shfl_xor(gz, o);
  }
  if (i < row_end && lane == 0) corr[i] = make_float4(gx, gy, gz, 0.f);
  double m[7] = {L, 0.0, 0.0, sdt, st, stt, dg};
#pragma unroll
  for (int c = 0; c < 7; ++c) {
    if (c == 1 || c == 2 || (!PEARSON && c >= 3 && c <= 5)) continue;
    for (int o = 32; o > 0; o >>= 1) m[c] += shfl_xor_d(m[c], o);
  }
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 7; ++c) mred[wv][c] = m[c];
  }
  __syncthreads();
  if (threadIdx.x < 7)
    mom[(size_t)blk * 8 + threadIdx.x] =
        ((mred[0][threadIdx.x] + mred[1][threadIdx.x]) + mred[2][threadIdx.x]) + mred[3][threadIdx.x];
}

template <int KIND>
__global__ __launch_bounds__(256) void pairdist_support_kernel(const float *__restrict__ coords, int N, float bg,
                                                               int row_begin, int row_end,
                                                               const int32_t *__restrict__ rowptr,
                                                               const int32_t *__restrict__ col,
                                                               const float *__restrict__ val,
                                                               const float *__restrict__ diag,
                                                               float4 *__restrict__ corr, double *__restrict__ mom,
                                                               const int *__restrict__ cmap,
                                                               const float4 *__restrict__ cpad = nullptr) {
  support_block<KIND>(coords, bg, row_begin, row_end, rowptr, col, val, diag, corr, mom, cmap, blockIdx.x, cpad);
}

// D[i, j] = ||c_i - c_j||: one thread per element.
__global__ __launch_bounds__(256) void pairdist_fwd_kernel(const float *__restrict__ coords, int N,
                                                           float *__restrict__ D, int64_t ldd) {
  __shared__ float ci[3];
  const int i = blockIdx.y;
  if (threadIdx.x < 3) ci[threadIdx.x] = coords[3 * (size_t)i + threadIdx.x];
  __syncthreads();
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  const float dx = ci[0] - coords[3 * (size_t)j], dy = ci[1] - coords[3 * (size_t)j + 1],
              dz = ci[2] - coords[3 * (size_t)j + 2];
  D[(size_t)i * ldd + j] = i == j ? 0.f : sqrtf(fmaf(dx, dx, fmaf(dy, dy, dz * dz)));
}

}  // namespace hicgat

using namespace hicgat;

constexpr size_t kTileLds = (size_t)BT * BT * sizeof(float);  // LDS image of one T tile

// mode: HICGAT_PD_TRI (1) = the upper-triangle tiling of the fused loss, HICGAT_PD_SQUARE (0) =
// the square tiling of the backward -- one convention for both queries (include/hicgat.h).
extern "C" int64_t hicgat_pairdist_num_tiles(int N, int mode) {
  if (N <= 0) return 0;
  const int64_t nb = pd_nb(N);
  return mode == HICGAT_PD_TRI ? nb * (nb + 1) / 2 : nb * nb;
}

// per tile: a (1 + ncol) x 128 float4 partial slab and ncol x 8 fp64 moments (ncol = 1: one column
// slab per tile)
static int pd_ncol(int) { return 1; }

// the per-pair gradient factor the reduction applies: MSE over N^2 entries of the symmetric D
// (each pair twice, d(d - t)^2 = 2 (d - t)): 4 / N^2; contrastive: 0.1 / M, M = N (N - 1) / 2 pairs --
// float32(0.1 / M), the value the reference's autograd hands to cdist's backward
static float loss_scale(int N, int loss_kind) {
  if (loss_kind == KIND_CONTRASTIVE) return N > 1 ? (float)(0.1 / (0.5 * (double)N * (double)(N - 1))) : 0.f;
  return (float)(4.0 / ((double)N * (double)N));
}

extern "C" size_t hicgat_pairdist_workspace_bytes(int N, int mode) {
  const int64_t tiles = hicgat_pairdist_num_tiles(N, mode);
  const int nc = pd_ncol(mode);
  return (size_t)tiles * ((1 + nc) * BT * sizeof(float4) + nc * 8 * sizeof(double)) + kMomBlocks * 8 * sizeof(double) +
         256;
}

// Host twin of tri_decode (exact integer search): tile-row of upper-triangle tile t.
static int tri_row_host(int64_t t, int nb) {
  int lo = 0, hi = nb - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (tri_start(mid, nb) <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

static void carve(void *ws, int64_t tiles, int ncol, float4 **part, double **mom) {
  char *p = static_cast<char *>(ws);
  *part = reinterpret_cast<float4 *>(p);
  *mom = reinterpret_cast<double *>(p + (size_t)tiles * (1 + ncol) * BT * sizeof(float4));
}

extern "C" int hicgat_pairdist_fwd(const float *coords, int N, float *D, int64_t ldd,
                                   hicgat_stream_t stream) {
  if (N < 0 || ldd < N) return HICGAT_EINVAL;
  if (N == 0) return HICGAT_OK;
  if (!coords || !D) return HICGAT_EINVAL;
  hipLaunchKernelGGL(pairdist_fwd_kernel, dim3((N + 255) / 256, N), dim3(256), 0,
                     (hipStream_t)stream, coords, N, D, ldd);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_pairdist_bwd(const float *coords, const float *G, int N, int64_t ldg,
                                   float *dcoords, void *workspace, size_t workspace_bytes,
                                   hicgat_stream_t stream) {
  if (N < 0 || ldg < N) return HICGAT_EINVAL;
  if (N == 0) return HICGAT_OK;
  if (!coords || !G || !dcoords || !workspace) return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_pairdist_workspace_bytes(N, HICGAT_PD_SQUARE)) return HICGAT_EINVAL;
  const int nb = pd_nb(N);
  const int64_t tiles = (int64_t)nb * nb;
  float4 *part;
  double *mom;
  carve(workspace, tiles, 1, &part, &mom);
  const bool vec = (ldg % 4 == 0) && ((reinterpret_cast<uintptr_t>(G) & 15) == 0) &&
                   ldg >= (int64_t)nb * BT;
  if (vec)
    hipLaunchKernelGGL((pairdist_tile_kernel<MODE_FULL, true, KIND_MSE>), dim3(tiles), dim3(256), kTileLds,
                       (hipStream_t)stream, coords, G, N, ldg, (int64_t)0, (int64_t)0, nb, (int64_t)0, part, mom, 0.f);
  else
    hipLaunchKernelGGL((pairdist_tile_kernel<MODE_FULL, false, KIND_MSE>), dim3(tiles), dim3(256), 0,
                       (hipStream_t)stream, coords, G, N, ldg, (int64_t)0, (int64_t)0, nb, (int64_t)0, part, mom, 0.f);
  HICGAT_CHECK_LAUNCH();
  hipLaunchKernelGGL(pairdist_reduce_kernel, dim3((N + 63) / 64), dim3(1024), 0,
                     (hipStream_t)stream, part, 1, N, nb, (int)MODE_FULL, (int64_t)0, tiles, 1.0f,
                     dcoords, nullptr, (int64_t)0, (int64_t)0, 0, nullptr, nullptr, 0, 0, nullptr);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_pairdist_mse_fused_band(const float *coords, const float *T, int N, int64_t ldt,
                                              int64_t t_row0, int64_t t_rows, int64_t t_col0,
                                              int64_t tile_begin, int64_t tile_end, int loss_kind,
                                              double *stats, float *loss, float *dcoords, void *workspace,
                                              size_t workspace_bytes, hicgat_stream_t stream) {
  if (N < 0 || loss_kind < KIND_MSE || loss_kind > KIND_CONTRASTIVE) return HICGAT_EINVAL;
  if (N == 0) return HICGAT_OK;
  if (!coords || !T || !stats || !workspace) return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_pairdist_workspace_bytes(N, HICGAT_PD_TRI)) return HICGAT_EINVAL;
  const int nb = pd_nb(N);
  const int64_t tiles = (int64_t)nb * (nb + 1) / 2;
  if (tile_end < 0 || tile_end > tiles) tile_end = tiles;
  if (tile_begin < 0) tile_begin = 0;
  if (tile_begin > tile_end) return HICGAT_EINVAL;
  const int64_t nt = tile_end - tile_begin;
  if (nt > 0) {
    // the band must hold every row / column the tile range reads: rows of tile-rows I0..I1 and
    // columns from I0's diagonal tile on (tiles (I, J) have J >= I >= I0)
    const int64_t I0 = tri_row_host(tile_begin, nb), I1 = tri_row_host(tile_end - 1, nb);
    const int64_t need_r1 = std::min<int64_t>(N, (I1 + 1) * BT);
    if (t_row0 < 0 || t_col0 < 0 || t_row0 > I0 * BT || t_col0 > I0 * BT || t_row0 + t_rows < need_r1 ||
        ldt < (int64_t)N - t_col0)
      return HICGAT_EINVAL;
  }
  float4 *part;
  double *mom;
  carve(workspace, tiles, 1, &part, &mom);
  const bool vec = (ldt % 4 == 0) && (t_col0 % 4 == 0) && ((reinterpret_cast<uintptr_t>(T) & 15) == 0) &&
                   ldt >= (int64_t)nb * BT - t_col0;
  if (nt > 0) {
    // the Pearson moments only for the combined loss; MSE needs sum (d - t)^2 only
#define HICGAT_PD_SYM(V, KD)                                                                          \
  hipLaunchKernelGGL((pairdist_tile_kernel<MODE_SYM, V, KD>), dim3(nt), dim3(256), V ? kTileLds : 0, \
                     (hipStream_t)stream, coords, T, N, ldt, t_row0, t_col0, nb, tile_begin, part, mom, 0.f)
#define HICGAT_PD_KINDS(V)                                                  \
  if (loss_kind == KIND_COMBINED) HICGAT_PD_SYM(V, KIND_COMBINED);          \
  else if (loss_kind == KIND_CONTRASTIVE) HICGAT_PD_SYM(V, KIND_CONTRASTIVE); \
  else HICGAT_PD_SYM(V, KIND_MSE)
    if (vec) {
      HICGAT_PD_KINDS(true);
    } else {
      HICGAT_PD_KINDS(false);
    }
#undef HICGAT_PD_KINDS
#undef HICGAT_PD_SYM
    HICGAT_CHECK_LAUNCH();
  }
  // row / column partials -> dcoords (when wanted) and, in the same launch, kMomBlocks blocks of
  // tile-moment partials; then one small launch: partials -> stats[0..6] -> mse / r / alpha / total
  const float scale = loss_scale(N, loss_kind);
  const int row_blocks = dcoords ? (N + 63) / 64 : 0;
  double *mpart = mom + (size_t)tiles * 8;
  hipLaunchKernelGGL(pairdist_reduce_kernel, dim3(row_blocks + kMomBlocks), dim3(1024), 0, (hipStream_t)stream, part,
                     1, N, nb, (int)MODE_SYM, tile_begin, tile_end, scale, dcoords, mom, tile_begin, tile_end,
                     row_blocks, mpart, nullptr, 0, 0, nullptr);
  HICGAT_CHECK_LAUNCH();
  hipLaunchKernelGGL(moments_finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, mpart, N, loss_kind, stats,
                     loss);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_pairdist_mse_fused(const float *coords, const float *T, int N, int64_t ldt,
                                         int64_t tile_begin, int64_t tile_end, int loss_kind,
                                         double *stats, float *loss, float *dcoords,
                                         void *workspace, size_t workspace_bytes,
                                         hicgat_stream_t stream) {
  if (ldt < N) return HICGAT_EINVAL;
  return hicgat_pairdist_mse_fused_band(coords, T, N, ldt, 0, N, 0, tile_begin, tile_end, loss_kind, stats, loss,
                                        dcoords, workspace, workspace_bytes, stream);
}

extern "C" int hicgat_pairdist_finalize(int N, int loss_kind, double *stats, float *loss,
                                        hicgat_stream_t stream) {
  if (N <= 0 || !stats || loss_kind < KIND_MSE || loss_kind > KIND_CONTRASTIVE) return HICGAT_EINVAL;
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, N, loss_kind,
                     stats, loss);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

// finalize + a rank's rows of the all-reduced fp64 dcoords narrowed to fp32 (one launch after the
// multi-GPU loss all-reduce instead of two); with cbuf, also the coordinates in global row order,
// cglob[i] = cbuf[gidx[i]] (the padded all-gather layout reordered: step()'s return value, no launch
// of its own)
__global__ __launch_bounds__(256) void finalize_rows_kernel(int N, int loss_kind, double *__restrict__ stats,
                                                            float *__restrict__ loss, const double *__restrict__ dc64,
                                                            int64_t n3, float *__restrict__ dcoords,
                                                            const float *__restrict__ cbuf,
                                                            const int32_t *__restrict__ gidx, float *__restrict__ cglob) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t == 0) finalize_stats(N, loss_kind, stats, loss);
  if (t < n3) dcoords[t] = (float)dc64[t];
  if (cbuf && t < 3 * (int64_t)N) {
    const int64_t i = t / 3;
    cglob[t] = cbuf[3 * (int64_t)gidx[i] + (t - 3 * i)];
  }
}

extern "C" int hicgat_pairdist_finalize_rows_ex(int N, int loss_kind, double *stats, float *loss, const double *dc64,
                                                int row_begin, int row_end, float *dcoords, const float *cbuf,
                                                const int32_t *gidx, float *cglob, hicgat_stream_t stream) {
  if (N <= 0 || !stats || loss_kind < KIND_MSE || loss_kind > KIND_CONTRASTIVE) return HICGAT_EINVAL;
  if (row_begin < 0 || row_end > N || row_begin > row_end) return HICGAT_EINVAL;
  const int64_t n3 = 3 * (int64_t)(row_end - row_begin);
  if (n3 > 0 && (!dc64 || !dcoords)) return HICGAT_EINVAL;
  if (cbuf && (!gidx || !cglob)) return HICGAT_EINVAL;
  const int64_t off = 3 * (int64_t)row_begin;
  const int64_t work = std::max<int64_t>(std::max<int64_t>(n3, cbuf ? 3 * (int64_t)N : 0), 1);
  hipLaunchKernelGGL(finalize_rows_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream, N,
                     loss_kind, stats, loss, n3 ? dc64 + off : nullptr, n3, n3 ? dcoords + off : nullptr, cbuf, gidx,
                     cglob);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_pairdist_finalize_rows(int N, int loss_kind, double *stats, float *loss, const double *dc64,
                                             int row_begin, int row_end, float *dcoords, hicgat_stream_t stream) {
  return hicgat_pairdist_finalize_rows_ex(N, loss_kind, stats, loss, dc64, row_begin, row_end, dcoords, nullptr,
                                          nullptr, nullptr, stream);
}

// ---- background form: T = bg except at a sorted symmetric CSR support + the diagonal -----------
static int64_t pd_support_blocks(int N) { return (N + 3) / 4; }

extern "C" size_t hicgat_pairdist_support_workspace_bytes(int N) {
  if (N <= 0) return 256;
  const int64_t tiles = hicgat_pairdist_num_tiles(N, HICGAT_PD_TRI);
  return (size_t)tiles * 2 * BT * sizeof(float4) + (size_t)(tiles + pd_support_blocks(N)) * 8 * sizeof(double) +
         kMomBlocks * 8 * sizeof(double) + 2 * (size_t)N * sizeof(float4) + 256;   // corr + the float4 coords
}

extern "C" int hicgat_pairdist_mse_fused_support_range_ex(const float *coords, const int32_t *cmap, int N,
                                                          float background, const int32_t *rowptr, const int32_t *col,
                                                          const float *val, const float *diag, int64_t tile_begin,
                                                          int64_t tile_end, int support_row_begin, int support_row_end,
                                                          int loss_kind, double *stats, float *loss, float *dcoords,
                                                          double *dcoords64, void *workspace,
                                                          size_t workspace_bytes, hicgat_stream_t stream) {
  if (N < 0 || loss_kind < KIND_MSE || loss_kind > KIND_CONTRASTIVE) return HICGAT_EINVAL;
  if (N == 0) return HICGAT_OK;
  if (!coords || !rowptr || !col || !val || !diag || !stats || !workspace) return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_pairdist_support_workspace_bytes(N)) return HICGAT_EINVAL;
  const int nb = pd_nb(N);
  const int64_t tiles = (int64_t)nb * (nb + 1) / 2;
  if (tile_end < 0 || tile_end > tiles) tile_end = tiles;
  if (tile_begin < 0) tile_begin = 0;
  if (tile_begin > tile_end) return HICGAT_EINVAL;
  if (support_row_end < 0 || support_row_end > N) support_row_end = N;
  if (support_row_begin < 0) support_row_begin = 0;
  if (support_row_begin > support_row_end) return HICGAT_EINVAL;
  const int64_t nt = tile_end - tile_begin;
  const int64_t sblocks = (support_row_end - support_row_begin + 3) / 4;
  char *p = static_cast<char *>(workspace);
  float4 *part = reinterpret_cast<float4 *>(p);
  // moment records: tiles [tile_begin, tile_end) at their tile index, the support blocks right
  // after tile_end (so [tile_begin, tile_end + sblocks) is one contiguous run; the workspace holds
  // tiles + pd_support_blocks(N) records, and tile_end + sblocks never exceeds that)
  double *mom = reinterpret_cast<double *>(p + (size_t)tiles * 2 * BT * sizeof(float4));
  double *mpart = mom + (size_t)(tiles + pd_support_blocks(N)) * 8;
  float4 *corr = reinterpret_cast<float4 *>(mpart + kMomBlocks * 8);
  hipStream_t s = (hipStream_t)stream;
  // bulk: every pair i < j of the tile range at the background value (no T read); support: the
  // entries of rows [support_row_begin, support_row_end) that differ, and those rows' diagonal
  // a rank's share (dcoords64: the sharded step): the support blocks ride in the tile launch (one
  // launch fewer on the critical path; at N = 20000 on one GPU the support pass needs the occupancy
  // of its own launch: 1.881 / 1.884 vs 1.875 / 1.877 ms per step, profiles/r04u_ab_single_gpu.txt)
  const bool ride = dcoords64 && nt > 0 && sblocks > 0;
  SupportArgs sa;
  if (ride) {
    sa.rowptr = rowptr;
    sa.col = col;
    sa.val = val;
    sa.diag = diag;
    sa.corr = corr;
    sa.mom = mom + (size_t)tile_end * 8;
    sa.row_begin = support_row_begin;
    sa.row_end = support_row_end;
    sa.ntiles = nt;
  }
  // the whole triangle in one launch before a separate support launch (one GPU): the diagonal tiles
  // write the float4 copy of the coordinates the support pass gathers (19 -> 8 us at N = 20000)
  float4 *cpad = (!ride && !cmap && tile_begin == 0 && tile_end == tiles && sblocks > 0) ? corr + N : nullptr;
  const auto tiles_for = [&](auto kind_c) {
    constexpr int KD = decltype(kind_c)::value;
    if (ride)
      hipLaunchKernelGGL((pairdist_tile_kernel<MODE_SYM, false, KD, true, true>), dim3(nt + sblocks), dim3(256), 0, s,
                         coords, nullptr, N, (int64_t)0, (int64_t)0, (int64_t)0, nb, tile_begin, part, mom, background,
                         cmap, sa);
    else if (nt > 0)
      hipLaunchKernelGGL((pairdist_tile_kernel<MODE_SYM, false, KD, true>), dim3(nt), dim3(256), 0, s, coords,
                         nullptr, N, (int64_t)0, (int64_t)0, (int64_t)0, nb, tile_begin, part, mom, background, cmap,
                         SupportArgs{}, cpad);
    if (sblocks > 0 && !ride)
      hipLaunchKernelGGL(pairdist_support_kernel<KD>, dim3(sblocks), dim3(256), 0, s, coords, N, background,
                         support_row_begin, support_row_end, rowptr, col, val, diag, corr, mom + (size_t)tile_end * 8,
                         cmap, cpad);
  };
  if (loss_kind == KIND_COMBINED) tiles_for(std::integral_constant<int, KIND_COMBINED>{});
  else if (loss_kind == KIND_CONTRASTIVE) tiles_for(std::integral_constant<int, KIND_CONTRASTIVE>{});
  else tiles_for(std::integral_constant<int, KIND_MSE>{});
  HICGAT_CHECK_LAUNCH();
  const float scale = loss_scale(N, loss_kind);
  const int row_blocks = (dcoords || dcoords64) ? (N + 63) / 64 : 0;
  // dcoords64: the caller all-reduces [stats | dcoords64] and finalizes (hicgat_pairdist_finalize_rows),
  // so a small share's moments go straight into stats[0..6] (stats[7..11] and loss are left alone)
  const bool one = dcoords64 && nt + sblocks <= kOneBlockMoments;
  hipLaunchKernelGGL(pairdist_reduce_kernel, dim3(row_blocks + (one ? 1 : kMomBlocks)), dim3(1024), 0, s, part, 1,
                     N, nb, (int)MODE_SYM, tile_begin, tile_end, scale, dcoords, mom, tile_begin, tile_end + sblocks,
                     row_blocks, one ? stats : mpart, corr, support_row_begin, support_row_end, dcoords64);
  HICGAT_CHECK_LAUNCH();
  if (!one) {
    hipLaunchKernelGGL(moments_finalize_kernel, dim3(1), dim3(64), 0, s, mpart, N, loss_kind, stats, loss);
    HICGAT_CHECK_LAUNCH();
  }
  return HICGAT_OK;
}

extern "C" int hicgat_pairdist_mse_fused_support_range(const float *coords, int N, float background,
                                                       const int32_t *rowptr, const int32_t *col, const float *val,
                                                       const float *diag, int64_t tile_begin, int64_t tile_end,
                                                       int support_row_begin, int support_row_end, int loss_kind,
                                                       double *stats, float *loss, float *dcoords, double *dcoords64,
                                                       void *workspace, size_t workspace_bytes,
                                                       hicgat_stream_t stream) {
  return hicgat_pairdist_mse_fused_support_range_ex(coords, nullptr, N, background, rowptr, col, val, diag, tile_begin,
                                                    tile_end, support_row_begin, support_row_end, loss_kind, stats,
                                                    loss, dcoords, dcoords64, workspace, workspace_bytes, stream);
}

extern "C" int hicgat_pairdist_mse_fused_support(const float *coords, int N, float background,
                                                 const int32_t *rowptr, const int32_t *col, const float *val,
                                                 const float *diag, int loss_kind, double *stats, float *loss,
                                                 float *dcoords, void *workspace, size_t workspace_bytes,
                                                 hicgat_stream_t stream) {
  return hicgat_pairdist_mse_fused_support_range(coords, N, background, rowptr, col, val, diag, 0, -1, 0, N,
                                                 loss_kind, stats, loss, dcoords, nullptr, workspace, workspace_bytes,
                                                 stream);
}
