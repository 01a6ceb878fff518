// Device-side finish of a score matrix and the rank step of the evaluation.
//
// acoss_ds_finish — what the reference does after the pair loop, on the host, element by element:
//   symmetrise         Ds += Ds.T              (acoss/algorithms/algorithm_template.py:188-191;
//                                               numpy buffers the overlapping operand, so this is
//                                               out[i,j] = D[i,j] + D[j,i] on the ORIGINAL values,
//                                               one float32 add)
//   Serra09 normalise  Ds[i,j] /= sqrt(n_j)     (rqa_serra09.py:71-83: float32 element / float64
//                                               scalar in float64, stored back as float32)
//   Chen normalise     Ds[i,j] = sqrt(n_j) / Ds[i,j]   (latefusion_chen.py:75-85, same dtypes)
// One block owns the tile pair (bi, bj), (bj, bi) with bi <= bj: it reads both 64 x 64 tiles into
// LDS, forms both outputs from the original values and writes both, so the kernel may run in place
// (out == D) with no cross-block hazard. Traffic: 4 B read + 4 B written per element (HBM bound).
//
// acoss_eval_ranks — the O(N^2) part of getEvalStatistics (algorithm_template.py:206-291): the
// 1-based rank of every other clique member in its query's row, in the order of
// np.argsort(-D', 1, kind="stable") where D' is D permuted to the reference's clique order (pos[k]
// = position of song k in it) with the diagonal set to -inf (:234). That order sorts -D ascending
// (NaN last), ties by position, so the rank of member j is 1 + #{k : key_k before key_j}. One block
// per query reads its row once per chunk of 16 members and counts; no sort is materialised.
#include "common.hpp"

namespace acoss {
namespace {

constexpr int kTile = 64;

// D and out may be the same matrix (every caller finishes in place), so neither is __restrict__:
// each block loads both of its tiles into LDS before its barrier and stores after it.
__global__ __launch_bounds__(256) void k_ds_finish(const float* D, int32_t n, int64_t ld,
                                                   const double* __restrict__ norm, int32_t symmetric, int32_t mode,
                                                   float* out) {
  __shared__ float A[kTile][kTile + 1];
  __shared__ float B[kTile][kTile + 1];
  // linear block index -> (bi, bj) with bi <= bj over the upper triangle of tiles
  const int nt = (n + kTile - 1) / kTile;
  int64_t lin = blockIdx.x;
  int bi = 0;
  while (lin >= nt - bi) {
    lin -= nt - bi;
    ++bi;
  }
  const int bj = bi + (int)lin;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 columns x 4 rows per pass
  const int ri = bi * kTile, rj = bj * kTile;
  for (int r = ty; r < kTile; r += 4) {
    const int gi = ri + r, gj = rj + tx;
    A[r][tx] = (gi < n && gj < n) ? D[(int64_t)gi * ld + gj] : 0.0f;
    const int hi = rj + r, hj = ri + tx;
    B[r][tx] = (hi < n && hj < n) ? D[(int64_t)hi * ld + hj] : 0.0f;
  }
  __syncthreads();
  auto fin = [&](float v, int col) -> float {
    if (mode == 1) return (float)((double)v / norm[col]);
    if (mode == 2) return (float)(norm[col] / (double)v);
    return v;
  };
  for (int r = ty; r < kTile; r += 4) {
    const int gi = ri + r, gj = rj + tx;
    if (gi < n && gj < n) {
      float v = A[r][tx];
      if (symmetric) v = v + B[tx][r];
      out[(int64_t)gi * ld + gj] = fin(v, gj);
    }
    if (bi != bj) {
      const int hi = rj + r, hj = ri + tx;
      if (hi < n && hj < n) {
        float v = B[r][tx];
        if (symmetric) v = v + A[tx][r];
        out[(int64_t)hi * ld + hj] = fin(v, hj);
      }
    }
  }
}

constexpr int kMemChunk = 16;

// before(k, j): does element k precede element j in the stable ascending order of -D'?
__device__ __forceinline__ bool before(float dk, int pk, float dj, int pj) {
  const bool nk = dk != dk, nj = dj != dj;
  if (nj) return !nk || pk < pj;  // NaN keys sort last, stably among themselves
  if (nk) return false;
  return dk > dj || (dk == dj && pk < pj);  // -dk < -dj  <=>  dk > dj
}

__global__ __launch_bounds__(256) void k_eval_ranks(const float* __restrict__ D, int32_t n, int64_t ld,
                                                    const int32_t* __restrict__ pos,
                                                    const int32_t* __restrict__ q_song,
                                                    const int64_t* __restrict__ m_off,
                                                    const int32_t* __restrict__ members, int32_t* __restrict__ ranks) {
  __shared__ int red[kMemChunk][4];
  const int q = blockIdx.x;
  const int i = q_song[q];
  const float* row = D + (int64_t)i * ld;
  const int64_t m0 = m_off[q], m1 = m_off[q + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t c0 = m0; c0 < m1; c0 += kMemChunk) {
    const int cnt = (int)((m1 - c0) < kMemChunk ? (m1 - c0) : kMemChunk);
    float dj[kMemChunk];
    int pj[kMemChunk], acc[kMemChunk];
#pragma unroll
    for (int t = 0; t < kMemChunk; ++t) {
      const int j = t < cnt ? members[c0 + t] : i;
      dj[t] = (j == i) ? -INFINITY : row[j];
      pj[t] = pos[j];
      acc[t] = 0;
    }
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const float dk = (k == i) ? -INFINITY : row[k];
      const int pk = pos[k];
#pragma unroll
      for (int t = 0; t < kMemChunk; ++t) acc[t] += before(dk, pk, dj[t], pj[t]) ? 1 : 0;
    }
#pragma unroll
    for (int t = 0; t < kMemChunk; ++t) {
      const int s = wave_sum(acc[t]);
      if (lane == 0) red[t][wv] = s;
    }
    __syncthreads();
    if (threadIdx.x < cnt) {
      const int t = threadIdx.x;
      ranks[c0 + t] = 1 + red[t][0] + red[t][1] + red[t][2] + red[t][3];
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace acoss

using namespace acoss;

extern "C" int acoss_ds_finish(const float* D, int32_t n, int64_t ld, const double* norm, int32_t symmetric,
                               int32_t mode, float* out, void* hip_stream) {
  clear_error();
  if (n < 0 || ld < n || mode < 0 || mode > 2 || (mode != 0 && !norm) || (n > 0 && (!D || !out))) {
    set_error("acoss_ds_finish: bad arguments (n=%d ld=%lld mode=%d)", n, (long long)ld, mode);
    return ACOSS_E_ARG;
  }
  if (n == 0) return ACOSS_OK;
  const int64_t nt = (n + kTile - 1) / kTile;
  const int64_t blocks = nt * (nt + 1) / 2;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  hipLaunchKernelGGL(k_ds_finish, dim3((unsigned)blocks), dim3(256), 0, s, D, n, ld, norm, symmetric, mode, out);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

extern "C" int acoss_eval_ranks(const float* D, int32_t n, int64_t ld, const int32_t* pos, const int32_t* q_song,
                                const int64_t* m_off, const int32_t* members, int32_t n_queries, int32_t* ranks_out,
                                void* hip_stream) {
  clear_error();
  if (n < 0 || ld < n || n_queries < 0 || (n_queries > 0 && (!D || !pos || !q_song || !m_off || !ranks_out))) {
    set_error("acoss_eval_ranks: bad arguments");
    return ACOSS_E_ARG;
  }
  if (n_queries == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  hipLaunchKernelGGL(k_eval_ranks, dim3(n_queries), dim3(256), 0, s, D, n, ld, pos, q_song, m_off, members,
                     ranks_out);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}
