// Per-CU load rate of the one-kernel tail's weight-stream address pattern against a contiguous one
// (diagnostic, not part of the library).  A workgroup of 16 waves streams a [512 x 512] fp32 matrix
// once per pass, 4 passes, each wave reading its 32 rows, in one of two lane -> address maps:
//   rows : lane (li = lane & 15, j = lane >> 4) loads row n0 + li, k 8j + 4e .. +3  (the tail's map:
//          16 rows per instruction, 64 B of each)
//   flat : lane loads the 16 B at 16 * lane of a contiguous 1 KB block (a pre-permuted copy)
// Also the store side (st_kernel): a wave writing 1 KB per instruction as dwordx4 (contiguous), as
// dwords of 16 consecutive columns in 4 rows (the tail's MFMA C-tile stores: lane & 15 = column,
// 4 (lane >> 4) + r = row), and as dwords of 64 consecutive floats (a LayerNorm row).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ld_pattern_bench.hip -o tools/ld_pattern_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(1024) void ld_kernel(const float *__restrict__ W, float *__restrict__ sink, long long *cyc) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, j = lane >> 4;
  constexpr int K = 512;
  const int n0 = 32 * ((wv + blockIdx.x) & 15);   // wave's 32 rows (rotated by workgroup)
  float acc = 0.f;
  __syncthreads();
  const long long t0 = clock64();
  for (int pass = 0; pass < 4; ++pass) {
#pragma unroll 2
    for (int g = 0; g < K / 32; ++g) {
      float4 v[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float *p;
          if (MODE == 0)
            p = W + (size_t)(n0 + 16 * t + li) * K + 32 * g + 8 * j + 4 * e;
          else   // the same 16 KB per (wave, g) as 4 contiguous 1 KB blocks
            p = W + (((size_t)(n0 / 16 + t) * (K / 32) + g) * 2 + e) * 256 + 4 * lane;
          v[t][e] = *reinterpret_cast<const float4 *>(p);
        }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 2; ++e) acc += (v[t][e].x + v[t][e].y) + (v[t][e].z + v[t][e].w);
    }
  }
  __syncthreads();
  const long long t1 = clock64();
  if (acc == -1.5e-38f) sink[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
__global__ __launch_bounds__(1024) void st_kernel(float *__restrict__ O, long long *cyc) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // each wave writes 64 KB per pass into its own region: 16 rows x 1024 floats (row stride 1024)
  float *base = O + ((size_t)blockIdx.x * 16 + wv) * 16 * 1024;
  float4 *b4 = reinterpret_cast<float4 *>(O) + ((size_t)blockIdx.x * 16 + wv) * 4096;
  __syncthreads();
  const long long t0 = clock64();
  for (int pass = 0; pass < 4; ++pass) {
    const float v = (float)(pass + lane);
    if (MODE == 0) {          // dwordx4, 1 KB contiguous per instruction
#pragma unroll 4
      for (int i = 0; i < 64; ++i)
        b4[(size_t)i * 64 + lane] = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
    } else if (MODE == 1) {   // dword, C-tile map: row 4 (lane >> 4) + r, 16 columns per row
#pragma unroll 4
      for (int i = 0; i < 256; ++i) {
        const int t = i & 63, r = i >> 6;   // 64 column tiles x 4 rows
        base[(size_t)(4 * (lane >> 4) + r) * 1024 + 16 * t + (lane & 15)] = v;
      }
    } else {                  // dword, 64 consecutive floats per instruction
#pragma unroll 4
      for (int i = 0; i < 256; ++i) base[(size_t)i * 64 + lane] = v;
    }
  }
  __syncthreads();
  const long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int K = 512, N = 512;
  float *W, *sink;
  long long *cyc;
  hipMalloc(&W, (size_t)N * K * 4);
  hipMemset(W, 0, (size_t)N * K * 4);
  hipMalloc(&sink, 4096);
  hipMalloc(&cyc, 4096 * 8);
  for (int blocks : {1, 8, 169, 256}) {
    for (int mode = 0; mode < 2; ++mode) {
      for (int rep = 0; rep < 3; ++rep) {
        if (mode == 0) hipLaunchKernelGGL(ld_kernel<0>, dim3(blocks), dim3(1024), 0, 0, W, sink, cyc);
        else hipLaunchKernelGGL(ld_kernel<1>, dim3(blocks), dim3(1024), 0, 0, W, sink, cyc);
      }
      hipDeviceSynchronize();
      std::vector<long long> c(blocks);
      hipMemcpy(c.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
      double s = 0;
      for (auto x : c) s += (double)x;
      s /= blocks;
      const double bytes = 4.0 * N * K * 4;   // 4 passes of the matrix per workgroup
      printf("blocks %3d  %-4s  %9.0f cycles per workgroup  %6.1f B/clk per CU\n", blocks, mode ? "flat" : "rows", s,
             bytes / s);
    }
  }
  float *O;
  hipMalloc(&O, (size_t)256 * 16 * 16 * 1024 * 4);
  const char *names[3] = {"st-x4", "st-tile", "st-row"};
  for (int blocks : {1, 169}) {
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 3; ++rep) {
        if (mode == 0) hipLaunchKernelGGL(st_kernel<0>, dim3(blocks), dim3(1024), 0, 0, O, cyc);
        else if (mode == 1) hipLaunchKernelGGL(st_kernel<1>, dim3(blocks), dim3(1024), 0, 0, O, cyc);
        else hipLaunchKernelGGL(st_kernel<2>, dim3(blocks), dim3(1024), 0, 0, O, cyc);
      }
      hipDeviceSynchronize();
      std::vector<long long> c(blocks);
      hipMemcpy(c.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
      double sum = 0;
      for (auto x : c) sum += (double)x;
      sum /= blocks;
      const double bytes = 4.0 * 16 * 64 * 1024;   // 4 passes x 16 waves x 64 KB
      printf("blocks %3d  %-7s %9.0f cycles per workgroup  %6.1f B/clk per CU\n", blocks, names[mode], sum, bytes / sum);
    }
  }
  return 0;
}
