// Fused LayerNorm + ReLU (+ residual add) of the GATNetSelectiveResidualsUpdated tail (a6).
//
// Reference: models.py:641-655, e.g. `x = self.norm_a(self.densea(x)); x = F.relu(x);
// x = x + x_initial` -- three torch ops (and three more in the backward) per block; here one
// wave per row does all of it in one pass over the row:
//   forward : z = relu((y - mean) * rstd * gamma + beta) + res,   rstd = 1/sqrt(var + eps)
//             (biased variance, torch.nn.LayerNorm semantics), saves (mean, rstd) per row;
//   backward: g = dz * [pre > 0];  dgamma += g * yhat;  dbeta += g;  dyhat = g * gamma;
//             dy = rstd * (dyhat - mean(dyhat) - yhat * mean(dyhat * yhat));  dres = dz (optionally
//             written beside dy, so a packed [dy | dres] feeds one dual-Linear backward GEMM).
// dgamma/dbeta: per-wave register partials over a grid-stride row loop, then the fixed-order
// column reduction of reduce.hip over the waves (deterministic).  Width W in {64, 128, 256} (W/64 values per lane).
#include "reduce.hpp"

namespace hicgat {

constexpr int kLnWaves = 4096;  // waves of the backward grid (partials: kLnWaves x 2 x W; 4 blocks per CU)

template <int W>
__global__ __launch_bounds__(256) void ln_relu_res_fwd_kernel(const float *__restrict__ y, int64_t ldy, int M,
                                                              const float *__restrict__ gamma,
                                                              const float *__restrict__ beta, float eps,
                                                              const float *__restrict__ res, int64_t ldr,
                                                              float *__restrict__ z, float2 *__restrict__ stats) {
  constexpr int V = W / 64;
  const int lane = lane_id();
  const int row = blockIdx.x * 4 + wave_in_block();
  if (row >= M) return;
  float v[V];
#pragma unroll
  for (int q = 0; q < V; ++q) v[q] = y[(size_t)row * ldy + q * 64 + lane];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < V; ++q) s += v[q];
  const float mean = wave_sum(s) / (float)W;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const float d = v[q] - mean;
    ss = fmaf(d, d, ss);
  }
  const float rstd = 1.0f / sqrt_rn_f32(wave_sum(ss) / (float)W + eps);
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const int c = q * 64 + lane;
    float o = fmaxf(fmaf((v[q] - mean) * rstd, gamma[c], beta[c]), 0.f);
    if (res) o += res[(size_t)row * ldr + c];
    z[(size_t)row * W + c] = o;
  }
  if (lane == 0) stats[row] = make_float2(mean, rstd);
}

template <int W>
__global__ __launch_bounds__(256) void ln_relu_res_bwd_kernel(const float *__restrict__ dz, const float *__restrict__ y,
                                                              int64_t ldy, int M, const float2 *__restrict__ stats,
                                                              const float *__restrict__ gamma,
                                                              const float *__restrict__ beta,
                                                              float *__restrict__ dy, int64_t lddy,
                                                              float *__restrict__ dres, int64_t lddres,
                                                              float *__restrict__ part) {
  constexpr int V = W / 64;
  const int lane = lane_id();
  const int gw = blockIdx.x * 4 + wave_in_block();
  const int nw = gridDim.x * 4;
  float g_[V], b_[V], pg[V], pb[V];
#pragma unroll
  for (int q = 0; q < V; ++q) {
    g_[q] = gamma[q * 64 + lane];
    b_[q] = beta[q * 64 + lane];
    pg[q] = pb[q] = 0.f;
  }
  for (int row = gw; row < M; row += nw) {
    const float2 st = stats[row];
    float yh[V], dh[V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int c = q * 64 + lane;
      yh[q] = (y[(size_t)row * ldy + c] - st.x) * st.y;
      const float pre = fmaf(yh[q], g_[q], b_[q]);
      const float dzv = dz[(size_t)row * W + c];
      if (dres) dres[(size_t)row * lddres + c] = dzv;   // d(residual) = dz, written beside dy
      const float g = pre > 0.f ? dzv : 0.f;
      pg[q] = fmaf(g, yh[q], pg[q]);
      pb[q] += g;
      dh[q] = g * g_[q];
      s1 += dh[q];
      s2 = fmaf(dh[q], yh[q], s2);
    }
    const float m1 = wave_sum(s1) / (float)W, m2 = wave_sum(s2) / (float)W;
#pragma unroll
    for (int q = 0; q < V; ++q) dy[(size_t)row * lddy + q * 64 + lane] = st.y * (dh[q] - m1 - yh[q] * m2);
  }
#pragma unroll
  for (int q = 0; q < V; ++q) {
    part[((size_t)gw * 2 + 0) * W + q * 64 + lane] = pg[q];
    part[((size_t)gw * 2 + 1) * W + q * 64 + lane] = pb[q];
  }
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_ln_relu_res_fwd(const float *y, int64_t ldy, int M, int W, const float *gamma,
                                      const float *beta, float eps, const float *res, int64_t ldr, float *z,
                                      float *row_stats, hicgat_stream_t stream) {
  if (M < 0 || (W != 64 && W != 128 && W != 256)) return M < 0 ? HICGAT_EINVAL : HICGAT_EUNSUPPORTED;
  if (M == 0) return HICGAT_OK;
  if (!y || !gamma || !beta || !z || !row_stats) return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((M + 3) / 4);
  float2 *st = reinterpret_cast<float2 *>(row_stats);
  if (W == 64)
    hipLaunchKernelGGL(ln_relu_res_fwd_kernel<64>, grid, dim3(256), 0, s, y, ldy, M, gamma, beta, eps, res, ldr, z, st);
  else if (W == 128)
    hipLaunchKernelGGL(ln_relu_res_fwd_kernel<128>, grid, dim3(256), 0, s, y, ldy, M, gamma, beta, eps, res, ldr, z, st);
  else
    hipLaunchKernelGGL(ln_relu_res_fwd_kernel<256>, grid, dim3(256), 0, s, y, ldy, M, gamma, beta, eps, res, ldr, z, st);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" size_t hicgat_ln_relu_res_workspace_bytes(int W) {
  return (size_t)kLnWaves * 2 * W * sizeof(float) + colsum_workspace_bytes(kLnWaves, 2 * W);
}

extern "C" int hicgat_ln_relu_res_bwd_params(int W, float *dgamma, float *dbeta, int accumulate,
                                             void *workspace, size_t workspace_bytes,
                                             hicgat_stream_t stream);

extern "C" int hicgat_ln_relu_res_bwd(const float *dz, const float *y, int64_t ldy, int M, int W,
                                      const float *row_stats, const float *gamma, const float *beta, float *dy,
                                      int64_t lddy, float *dres, int64_t lddres, float *dgamma, float *dbeta,
                                      int accumulate, void *workspace, size_t workspace_bytes,
                                      hicgat_stream_t stream) {
  if (M < 0 || (W != 64 && W != 128 && W != 256)) return M < 0 ? HICGAT_EINVAL : HICGAT_EUNSUPPORTED;
  if (!dz || !y || !row_stats || !gamma || !beta || !dy || !workspace) return HICGAT_EINVAL;
  if ((dgamma == nullptr) != (dbeta == nullptr)) return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_ln_relu_res_workspace_bytes(W)) return HICGAT_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float *part = static_cast<float *>(workspace);
  const float2 *st = reinterpret_cast<const float2 *>(row_stats);
  const dim3 grid(kLnWaves / 4);
  if (W == 64)
    hipLaunchKernelGGL(ln_relu_res_bwd_kernel<64>, grid, dim3(256), 0, s, dz, y, ldy, M, st, gamma, beta, dy, lddy, dres, lddres, part);
  else if (W == 128)
    hipLaunchKernelGGL(ln_relu_res_bwd_kernel<128>, grid, dim3(256), 0, s, dz, y, ldy, M, st, gamma, beta, dy, lddy, dres, lddres, part);
  else
    hipLaunchKernelGGL(ln_relu_res_bwd_kernel<256>, grid, dim3(256), 0, s, dz, y, ldy, M, st, gamma, beta, dy, lddy, dres, lddres, part);
  HICGAT_CHECK_LAUNCH();
  if (!dgamma) return HICGAT_OK;   // partials stay in the workspace for hicgat_ln_relu_res_bwd_params
  return hicgat_ln_relu_res_bwd_params(W, dgamma, dbeta, accumulate, workspace, workspace_bytes, stream);
}

// dgamma / dbeta = column sums of the per-wave partials [kLnWaves, 2W] (fixed order) that a
// hicgat_ln_relu_res_bwd call left in `workspace` -- e.g. on another stream, after an event.
extern "C" int hicgat_ln_relu_res_bwd_params(int W, float *dgamma, float *dbeta, int accumulate,
                                             void *workspace, size_t workspace_bytes,
                                             hicgat_stream_t stream) {
  if (W != 64 && W != 128 && W != 256) return HICGAT_EUNSUPPORTED;
  if (!dgamma || !dbeta || !workspace) return HICGAT_EINVAL;
  if (workspace_bytes < hicgat_ln_relu_res_workspace_bytes(W)) return HICGAT_EINVAL;
  float *part = static_cast<float *>(workspace);
  const ColOut o{dgamma, 0, W, dbeta, nullptr, accumulate};
  return colsum_launch(part, 2 * W, kLnWaves, 2 * W, o, part + (size_t)kLnWaves * 2 * W,
                       (hipStream_t)stream);
}
