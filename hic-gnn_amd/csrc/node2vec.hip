// node2vec embeddings on gfx950: biased second-order random walks
// and skip-gram with negative sampling.
//
// Reference: `Node2Vec(G, dimensions=512, walk_length=150, num_walks=50, p=1.75, q=0.4, workers=1,
// seed=42).fit(window=25, min_count=1, batch_words=4)` at HiC_GAT_generalize_directly.py:150-155
// (node2vec 0.4.x over networkx, then gensim 4 Word2Vec with sg=1, negative=5, sample=1e-3,
// alpha 0.025 -> 0.0001, 5 epochs).  Neither package is installed; the algorithms are
// restated from their published code:
//   walk step from cur (previous node prev): neighbour d of cur with weight w(cur, d) x
//     1/p if d == prev, 1 if d is adjacent to prev, 1/q otherwise (the first step: w(cur, d) alone);
//   skip-gram: for every kept centre word and every context word in a reduced window, the context's
//     input vector predicts the centre word (label 1) and `negative` unigram^0.75 samples (label 0);
//     g = (label - sigmoid(f)) * alpha, |f| >= 6 skipped (gensim's MAX_EXP rule).
// MI355X form: one thread per walk, sampling the second-order distribution by rejection (first-order
// candidate from the row's cumulative weights by binary search, accepted with probability
// factor / max factor; the adjacency test is a binary search in prev's sorted CSR row), with a
// counter-based RNG (splitmix64 of (seed, walk, step, attempt)), so walks are deterministic.  SGNS:
// one wave per walk, the walk's kept words compacted into LDS with a ballot, each dot product a
// 64-lane reduction over D/64 values per lane, vectors updated Hogwild-style across waves (as gensim's
// multi-worker mode does; the reference's workers=1 is sequential).
#include "common.hpp"

namespace hicgat {

__device__ __forceinline__ uint64_t splitmix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rng4(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
  return splitmix(seed ^ splitmix(a ^ splitmix(b ^ splitmix(c))));
}
__device__ __forceinline__ float u24(uint64_t r) { return (float)(r >> 40) * 0x1p-24f; }   // [0, 1)

// row r of the CSR contains column c (rows sorted ascending)
__device__ __forceinline__ bool has_col(const int *__restrict__ rowptr, const int *__restrict__ col, int r, int c) {
  int lo = rowptr[r], hi = rowptr[r + 1];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const int v = col[mid];
    if (v == c) return true;
    if (v < c) lo = mid + 1;
    else hi = mid;
  }
  return false;
}

constexpr int kMaxAttempts = 4096;   // rejection cap: every walk step terminates

__global__ __launch_bounds__(256) void n2v_walks_kernel(const int *__restrict__ rowptr, const int *__restrict__ col,
                                                        const float *__restrict__ cumw,
                                                        const int *__restrict__ starts, int nwalks, int L,
                                                        float inv_p, float inv_q, float fmax, uint64_t seed,
                                                        int *__restrict__ walks) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwalks) return;
  int *out = walks + (size_t)w * L;
  int cur = starts[w], prev = -1, len = 1;
  out[0] = cur;
  for (; len < L; ++len) {
    const int b = rowptr[cur], e = rowptr[cur + 1];
    if (b == e) break;                                   // no neighbours: the walk ends (node2vec)
    const float tot = cumw[e - 1];
    int nxt = col[b];
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
      const uint64_t r = rng4(seed, (uint64_t)w, (uint64_t)len, (uint64_t)attempt);
      const float u = u24(r) * tot;
      int lo = b, hi = e - 1;                            // first k with cumw[k] > u
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cumw[mid] > u) hi = mid;
        else lo = mid + 1;
      }
      nxt = col[lo];
      if (prev < 0) break;                               // first step: first-order weights only
      const float f = nxt == prev ? inv_p : (has_col(rowptr, col, prev, nxt) ? 1.f : inv_q);
      if ((float)(r & 0xFFFFFFull) * 0x1p-24f * fmax < f) break;
    }
    prev = cur;
    cur = nxt;
    out[len] = cur;
  }
  for (; len < L; ++len) out[len] = -1;                  // a shorter walk is padded with -1
}

// one wave per walk; D = 64 * VPL.  keep[v]: gensim's downsampling keep probability; cum[V]: the
// unigram^0.75 cumulative table (cum[V-1] = its total).
template <int VPL>
__global__ __launch_bounds__(256) void n2v_sgns_kernel(const int *__restrict__ walks, int nwalks, int L,
                                                       const float *__restrict__ keep,
                                                       const uint32_t *__restrict__ cum, int V, int window,
                                                       int negative, float alpha0, float alpha1, int epoch,
                                                       int epochs, uint64_t seed, float *syn0, float *syn1) {
  constexpr int D = 64 * VPL;
  __shared__ int sent[4][1024];
  const int lane = lane_id(), wv = wave_in_block();
  // grid-stride over walks: the caller bounds the waves in flight (Hogwild contention on a small
  // vocabulary loses updates; the reference trains with one worker)
  for (int w = blockIdx.x * 4 + wv; w < nwalks; w += gridDim.x * 4) {
  const float prog = ((float)epoch * nwalks + w) / ((float)epochs * nwalks);
  const float alpha = alpha0 - (alpha0 - alpha1) * prog;
  int *s = sent[wv];
  int n = 0;
  for (int base = 0; base < L; base += 64) {
    const int pos = base + lane;
    const int tok = pos < L ? walks[(size_t)w * L + pos] : -1;
    const bool kept = tok >= 0 && u24(rng4(seed, 0x5A3Full + epoch, (uint64_t)w, (uint64_t)pos)) < keep[tok];
    const uint64_t m = __ballot(kept);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (kept) s[n + before] = tok;
    n += __popcll(m);
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t total = cum[V - 1];
  for (int i = 0; i < n; ++i) {
    const int word = s[i];
    const int red = (int)(rng4(seed, 0x77ull + epoch, (uint64_t)w, (uint64_t)i) % (uint64_t)window);
    const int j0 = max(0, i - window + red), j1 = min(n, i + window + 1 - red);
    for (int j = j0; j < j1; ++j) {
      if (j == i) continue;
      float *in = syn0 + (size_t)s[j] * D;
      float l1[VPL], work[VPL];
#pragma unroll
      for (int q = 0; q < VPL; ++q) {
        l1[q] = in[q * 64 + lane];
        work[q] = 0.f;
      }
      // the positive and the `negative` sampled targets: rows loaded together, the 8 dot products
      // reduced in one transpose reduce, then the updates applied in gensim's order (a target drawn
      // twice in one pair reads its row once -- within Hogwild's own reordering)
      int tg[8];
      float lab[8], s1[8][VPL], f[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        tg[d] = -1;
        lab[d] = d == 0 ? 1.f : 0.f;
        if (d > negative) continue;
        int target = word;
        if (d > 0) {
          const uint32_t x = (uint32_t)(rng4(seed, 0x9Dull + epoch, ((uint64_t)w << 20) | (uint64_t)i,
                                             ((uint64_t)j << 8) | (uint64_t)d) % total);
          int lo = 0, hi = V - 1;                        // first k with cum[k] >= x (gensim's bisect_left)
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cum[mid] >= x) hi = mid;
            else lo = mid + 1;
          }
          target = lo;
          if (target == word) continue;
        }
        tg[d] = target;
      }
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        f[d] = 0.f;
        const float *row = syn1 + (size_t)(tg[d] < 0 ? 0 : tg[d]) * D;
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          s1[d][q] = tg[d] < 0 ? 0.f : row[q * 64 + lane];
          f[d] = fmaf(l1[q], s1[d][q], f[d]);
        }
      }
      transpose_reduce<8>(f, lane);                      // lane l: the sum of dot idx(l) in f[0]
      float dots[8];
#pragma unroll
      for (int d = 0; d < 8; ++d) dots[d] = readlane_f(f[0], ((d >> 2) & 1) << 5 | ((d >> 1) & 1) << 4 | (d & 1) << 3);
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        if (tg[d] < 0 || dots[d] <= -6.f || dots[d] >= 6.f) continue;
        const float g = (lab[d] - 1.f / (1.f + expf(-dots[d]))) * alpha;
        float *out = syn1 + (size_t)tg[d] * D;
#pragma unroll
        for (int q = 0; q < VPL; ++q) {
          work[q] = fmaf(g, s1[d][q], work[q]);
          out[q * 64 + lane] = fmaf(g, l1[q], s1[d][q]);
        }
      }
#pragma unroll
      for (int q = 0; q < VPL; ++q) in[q * 64 + lane] = l1[q] + work[q];
    }
  }
  __builtin_amdgcn_wave_barrier();   // the next walk reuses s[]
  }
}

}  // namespace hicgat

using namespace hicgat;

extern "C" int hicgat_n2v_walks(const int32_t *rowptr, const int32_t *col, const float *cum_weights, int N,
                                const int32_t *starts, int nwalks, int walk_length, float p, float q,
                                uint64_t seed, int32_t *walks, hicgat_stream_t stream) {
  if (N < 0 || nwalks < 0 || walk_length < 1 || !(p > 0.f) || !(q > 0.f)) return HICGAT_EINVAL;
  if (nwalks == 0) return HICGAT_OK;
  if (!rowptr || !col || !cum_weights || !starts || !walks) return HICGAT_EINVAL;
  const float inv_p = 1.f / p, inv_q = 1.f / q;
  const float fmax = fmaxf(1.f, fmaxf(inv_p, inv_q));
  hipLaunchKernelGGL(n2v_walks_kernel, dim3((nwalks + 255) / 256), dim3(256), 0, (hipStream_t)stream, rowptr, col,
                     cum_weights, starts, nwalks, walk_length, inv_p, inv_q, fmax, seed, walks);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

extern "C" int hicgat_n2v_sgns_epoch(const int32_t *walks, int nwalks, int walk_length, const float *keep_prob,
                                     const uint32_t *cum_table, int V, int D, int window, int negative,
                                     float alpha0, float alpha1, int epoch, int epochs, uint64_t seed,
                                     int max_waves, float *syn0, float *syn1, hicgat_stream_t stream) {
  if (max_waves < 1) return HICGAT_EINVAL;
  if (nwalks < 0 || walk_length < 1 || walk_length > 1024 || V < 1 || window < 1 || negative < 0 || negative > 7 ||
      epochs < 1 ||
      epoch < 0 || epoch >= epochs)
    return HICGAT_EINVAL;
  if (D % 64 || D < 64 || D > 1024) return HICGAT_EUNSUPPORTED;
  if (nwalks == 0) return HICGAT_OK;
  if (!walks || !keep_prob || !cum_table || !syn0 || !syn1) return HICGAT_EINVAL;
  const dim3 grid((min(nwalks, max_waves) + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
#define HICGAT_SGNS(VPL)                                                                                       \
  hipLaunchKernelGGL(n2v_sgns_kernel<VPL>, grid, block, 0, s, walks, nwalks, walk_length, keep_prob, cum_table, V, \
                     window, negative, alpha0, alpha1, epoch, epochs, seed, syn0, syn1)
  switch (D / 64) {
    case 1: HICGAT_SGNS(1); break;
    case 2: HICGAT_SGNS(2); break;
    case 4: HICGAT_SGNS(4); break;
    case 8: HICGAT_SGNS(8); break;
    case 16: HICGAT_SGNS(16); break;
    default: return HICGAT_EUNSUPPORTED;
  }
#undef HICGAT_SGNS
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
