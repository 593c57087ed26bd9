// torch.optim.Adam step (HiC-GNN_main.py:118,130) over ONE flat fp32 parameter buffer (a10).
//
// Every model parameter is a view into one flat buffer (and every .grad a view into another), so
// one launch updates all of them and a multi-GPU run all-reduces one contiguous gradient buffer.
// The arithmetic is torch's single-tensor CPU Adam, operation for operation (checked bit-exact
// against torch on the CPU in tests/test_oracle_golden.py::test_adam_restatement_matches_torch):
//   exp_avg.lerp_(g, 1-b1)                    -> m = fma(1-b1, g - m, m)
//   exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)  -> v = fma((1-b2)*g, g, v*b2)
//   denom = sqrt(v) / sqrt(1 - b2^t) + eps;  p.addcdiv_(m, denom, -lr/(1 - b1^t)) -> p + (s*m)/denom
#include "common.hpp"

namespace hicgat {

struct AdamConsts {
  float w1, b2, c2, bc2s, eps, neg_step;
};

__device__ __forceinline__ void adam_one(float &p, float g, float &m, float &v, const AdamConsts &k) {
  m = fmaf(k.w1, g - m, m);
  v = fmaf(k.c2 * g, g, v * k.b2);
  const float denom = sqrt_rn_f32(v) / k.bc2s + k.eps;
  p = p + __fdiv_rn(k.neg_step * m, denom);
}

__global__ __launch_bounds__(256) void adam_kernel(float *__restrict__ p, const float *__restrict__ g,
                                                   float *__restrict__ m, float *__restrict__ v,
                                                   int64_t n, AdamConsts k,
                                                   const float2 *__restrict__ table,
                                                   const int64_t *__restrict__ step_ctr, int64_t table_len,
                                                   int counted) {
  if (table) {  // graph-replayable form: per-step constants from the host-computed table
    int64_t s = *step_ctr - counted;   // counted: this step's increment already happened (step start)
    if (s < 0) s = 0;
    if (s >= table_len) s = table_len - 1;
    k.neg_step = table[s].x;
    k.bc2s = table[s].y;
  }
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4 *p4 = reinterpret_cast<float4 *>(p);
  float4 *m4 = reinterpret_cast<float4 *>(m);
  float4 *v4 = reinterpret_cast<float4 *>(v);
  const float4 *g4 = reinterpret_cast<const float4 *>(g);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = p4[i], mm = m4[i], vv = v4[i];
    const float4 gg = g4[i];
    adam_one(pp.x, gg.x, mm.x, vv.x, k);
    adam_one(pp.y, gg.y, mm.y, vv.y, k);
    adam_one(pp.z, gg.z, mm.z, vv.z, k);
    adam_one(pp.w, gg.w, mm.w, vv.w, k);
    p4[i] = pp;
    m4[i] = mm;
    v4[i] = vv;
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_one(pp, g[i], mm, vv, k);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

__global__ void step_increment_kernel(int64_t *step_ctr) { *step_ctr += 1; }

// zero_grad + the device step count's advance in one launch (the step's first; its Adam then runs
// with counted = 1)
__global__ __launch_bounds__(256) void step_begin_kernel(float *__restrict__ grad, int64_t n,
                                                         int64_t *__restrict__ step_ctr) {
  if (step_ctr && blockIdx.x == 0 && threadIdx.x == 0) step_ctr[0] = step_ctr[0] + 1;
  const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * 256;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) reinterpret_cast<float4 *>(grad)[i] = z;
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) grad[i] = 0.f;
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                                int64_t n, double lr, double beta1, double beta2, double eps,
                                int64_t step, hicgat_stream_t stream) {
  if (n < 0 || step < 1) return HICGAT_EINVAL;
  if (n == 0) return HICGAT_OK;
  if (!param || !grad || !exp_avg || !exp_avg_sq) return HICGAT_EINVAL;
  const uintptr_t mis = reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                        reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq);
  if (mis & 15) return HICGAT_EINVAL;
  AdamConsts k;
  k.w1 = (float)(1.0 - beta1);
  k.b2 = (float)beta2;
  k.c2 = (float)(1.0 - beta2);
  k.bc2s = (float)std::pow(1.0 - std::pow(beta2, (double)step), 0.5);  // Python (1-b2**t)**0.5
  k.eps = (float)eps;
  k.neg_step = (float)(-(lr / (1.0 - std::pow(beta1, (double)step))));
  const int64_t work = (n + 3) / 4;
  const int blocks = (int)std::min<int64_t>((work + 255) / 256, 4096);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, param, grad,
                     exp_avg, exp_avg_sq, n, k, nullptr, nullptr, (int64_t)0, 0);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_adam_step_table_ex(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                                         int64_t n, double beta1, double beta2, double eps, const float *table,
                                         int64_t table_len, int64_t *step_counter, int counted,
                                         hicgat_stream_t stream) {
  if (n < 0 || table_len < 1 || (counted != 0 && counted != 1)) return HICGAT_EINVAL;
  if (!param || !grad || !exp_avg || !exp_avg_sq || !table || !step_counter) return HICGAT_EINVAL;
  const uintptr_t mis = reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                        reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq);
  if ((mis & 15) || (reinterpret_cast<uintptr_t>(table) & 7)) return HICGAT_EINVAL;
  AdamConsts k;
  k.w1 = (float)(1.0 - beta1);
  k.b2 = (float)beta2;
  k.c2 = (float)(1.0 - beta2);
  k.eps = (float)eps;
  k.bc2s = 1.f;
  k.neg_step = 0.f;
  if (n > 0) {
    const int64_t work = (n + 3) / 4;
    const int blocks = (int)std::min<int64_t>((work + 255) / 256, 4096);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, param, grad, exp_avg,
                       exp_avg_sq, n, k, reinterpret_cast<const float2 *>(table), step_counter, table_len, counted);
    HICGAT_CHECK_LAUNCH();
  }
  if (!counted) {
    hipLaunchKernelGGL(step_increment_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step_counter);
    HICGAT_CHECK_LAUNCH();
  }
  return HICGAT_OK;
}

extern "C" int hicgat_adam_step_table(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                                      int64_t n, double beta1, double beta2, double eps, const float *table,
                                      int64_t table_len, int64_t *step_counter, hicgat_stream_t stream) {
  return hicgat_adam_step_table_ex(param, grad, exp_avg, exp_avg_sq, n, beta1, beta2, eps, table, table_len,
                                   step_counter, 0, stream);
}

extern "C" int hicgat_step_begin(float *grad, int64_t n, int64_t *step_counter, hicgat_stream_t stream) {
  if (n < 0 || (n > 0 && !grad)) return HICGAT_EINVAL;
  if (grad && (reinterpret_cast<uintptr_t>(grad) & 15)) return HICGAT_EINVAL;
  if (n == 0 && !step_counter) return HICGAT_OK;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n / 4 + 255) / 256, 1024));
  hipLaunchKernelGGL(step_begin_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, grad, n, step_counter);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
