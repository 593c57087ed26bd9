// Deterministic column sums shared by the GEMM (bias gradients, split-K slabs) and LayerNorm
// (gamma/beta gradients) entry points; see reduce.hip.
#pragma once
#include "common.hpp"

namespace hicgat {

struct ColOut {
  float *out0;          // row r of the result -> out0 + r * ld
  int64_t ld;
  int64_t cols;         // elements per result row
  float *out1;          // if set, row 1 goes here instead (LayerNorm dbeta)
  const float *bias;    // added per column (split-K GEMM epilogue), may be null
  int accumulate;       // add the previous value of the destination
  float *tail;          // if set, elements from tail_start on go to tail[i - tail_start] (GEMM: db)
  int64_t tail_start;
};

// Sum rows [0, K) of A [K, N] (leading dim lda) into the ColOut target.  ws: colsum_workspace_bytes.
int colsum_launch(const float *A, int64_t lda, int64_t K, int64_t N, const ColOut &o, float *ws, hipStream_t s);
size_t colsum_workspace_bytes(int64_t K, int64_t N);
// One pass, one thread per column (any K; no workspace): the split-K slab sum.
int colsum_wide_launch(const float *A, int64_t lda, int64_t K, int64_t N, const ColOut &o, hipStream_t s);

}  // namespace hicgat
