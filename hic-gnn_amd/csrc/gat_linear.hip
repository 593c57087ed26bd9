// GATConv lin_l (a2) on the gfx950 fp32 matrix cores, attention logits fused in the epilogue.
//
// Reference: PyG 1.7.2 GATConv.forward: x_l = lin_l(x).view(-1, H, C); alpha_l = (x_l*att_l).sum(-1)
// (and alpha_r with att_r), called from models.py:635.  h = x W^T is the only GEMM on the GAT
// path; fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32 (exact fp32 products, one rounding
// per fma, the same numerics class as the CPU sgemm of the reference).
//
// Tile: 64 rows x 256 columns (one whole head when C == 256) x BK = 16 per K-step, 4 waves, each
// wave a 64x64 output = 2x2 MFMA 32x32 tiles.  A and B are staged K-major in LDS (As[k][m],
// Bs[k][n]) so every MFMA operand read is 32 consecutive floats (conflict-free ds_read_b32); the
// next K-step's global loads are issued into registers before the current step's MFMAs.  The
// epilogue writes h and, when the column tile is one head, reduces h*att over its 256 columns
// (lane shuffles inside each 32-column MFMA tile, LDS across waves) into a_src / a_dst.
#include "common.hpp"

namespace hicgat {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GBM = 64, GBN = 256, GBK = 16;
constexpr int APAD = GBM + 4, BPAD = GBN + 4;

__global__ __launch_bounds__(256, 1) void linear_att_kernel(const float *__restrict__ x,
                                                         const float *__restrict__ W, int M, int K,
                                                         int Nc, int C, const float *__restrict__ att_s,
                                                         const float *__restrict__ att_d,
                                                         float *__restrict__ h, float *__restrict__ a_src,
                                                         float *__restrict__ a_dst, int H,
                                                         int fuse_logits) {
  __shared__ float As[GBK][APAD];
  __shared__ float Bs[GBK][BPAD];
  __shared__ float red[2][4][GBM];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int m0 = blockIdx.x * GBM, n0 = blockIdx.y * GBN;

  // global -> register staging map: A tile 64 x 16 = 256 float4 (1 per thread),
  // B tile 256 x 16 = 1024 float4 (4 per thread)
  const int arow = tid >> 2, akq = (tid & 3) * 4;
  float4 ra, rb[4];
  auto load_tile = [&](int k0) {
    const int gr = m0 + arow;
    ra = gr < M ? *reinterpret_cast<const float4 *>(x + (size_t)gr * K + k0 + akq)
                : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int bn = (tid >> 2) + 64 * u;
      rb[u] = *reinterpret_cast<const float4 *>(W + (size_t)(n0 + bn) * K + k0 + akq);
    }
  };
  auto store_tile = [&]() {
    As[akq + 0][arow] = ra.x;
    As[akq + 1][arow] = ra.y;
    As[akq + 2][arow] = ra.z;
    As[akq + 3][arow] = ra.w;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int bn = (tid >> 2) + 64 * u;
      Bs[akq + 0][bn] = rb[u].x;
      Bs[akq + 1][bn] = rb[u].y;
      Bs[akq + 2][bn] = rb[u].z;
      Bs[akq + 3][bn] = rb[u].w;
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int li = lane & 31, lk = lane >> 5;
  load_tile(0);
  for (int k0 = 0; k0 < K; k0 += GBK) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (k0 + GBK < K) load_tile(k0 + GBK);
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      const float a0 = As[kk + lk][li], a1 = As[kk + lk][32 + li];
      const float b0 = Bs[kk + lk][wv * 64 + li], b1 = Bs[kk + lk][wv * 64 + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }

  // epilogue: C/D map of the 32x32 f32 tiles: col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float ps[2][16], pd[2][16];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 16; ++r) ps[mi][r] = pd[mi][r] = 0.f;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int gc = n0 + wv * 64 + ni * 32 + li;
      const float ws = fuse_logits ? att_s[gc] : 0.f, wd = fuse_logits ? att_d[gc] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gr = m0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        const float v = acc[mi][ni][r];
        if (gr < M) h[(size_t)gr * Nc + gc] = v;
        ps[mi][r] = fmaf(v, ws, ps[mi][r]);
        pd[mi][r] = fmaf(v, wd, pd[mi][r]);
      }
    }
  }
  if (!fuse_logits) return;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float s = ps[mi][r], d = pd[mi][r];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        d += __shfl_xor(d, o);
      }
      if (li == 0) {
        const int lr = mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        red[0][wv][lr] = s;
        red[1][wv][lr] = d;
      }
    }
  }
  __syncthreads();
  if (tid < 2 * GBM) {
    const int which = tid / GBM, lr = tid % GBM, gr = m0 + lr;
    const float v = ((red[which][0][lr] + red[which][1][lr]) + red[which][2][lr]) + red[which][3][lr];
    const int head = n0 / C;
    if (gr < M) (which ? a_dst : a_src)[(size_t)gr * H + head] = v;
  }
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_gat_linear_att(const float *x, const float *W, const float *att_src,
                                     const float *att_dst, int N, int F, int H, int C, float *h,
                                     float *a_src, float *a_dst, hicgat_stream_t stream) {
  if (N < 0 || F <= 0 || H <= 0 || C <= 0) return HICGAT_EINVAL;
  const int D = H * C;
  if ((F % GBK) != 0 || (D % GBN) != 0) return HICGAT_EUNSUPPORTED;
  if (N == 0) return HICGAT_OK;
  if (!x || !W || !att_src || !att_dst || !h || !a_src || !a_dst) return HICGAT_EINVAL;
  const uintptr_t mis = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(W);
  if (mis & 15) return HICGAT_EINVAL;
  const int fuse = (C == GBN) ? 1 : 0;
  hipLaunchKernelGGL(linear_att_kernel, dim3((N + GBM - 1) / GBM, D / GBN), dim3(256), 0,
                     (hipStream_t)stream, x, W, N, F, D, C, att_src, att_dst, h, a_src, a_dst, H,
                     fuse);
  HICGAT_CHECK_LAUNCH();
  if (!fuse) return hicgat_gat_att_logits(h, att_src, att_dst, N, H, C, a_src, a_dst, stream);
  return HICGAT_OK;
}
