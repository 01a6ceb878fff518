// simple.hip — SiMPle similarity (acoss/algorithms/simple_silva.py) for a batch of ordered pairs.
//
// Per pair (query a, reference b), both (12 x n) float64 dim-major blocks:
//   Simple.oti (:45-54):  p = sum over time of each chroma bin; v[k] = <p_a, roll(p_b, k)>;
//                         k* = argsort(v)[-1] (ties: the last index, numpy's small-array sort is
//                         stable); the reference is rolled by k* on the chroma axis.
//   Simple.simple_sim (:68-118): MP[i] = min_j (|b_j|^2 + |a_i|^2) - 2 QT[i][j] over length-L
//                         subsequences, score = median(MP). The reference builds QT with FFT
//                         convolutions plus the STOMP update; here QT[i][j] = sum_t G[i+t][j+t]
//                         with G the 12-term dot product of single frames (same value, different
//                         rounding: parity is a tolerance, 1e-9 relative in the tests).
//
// One 256-thread block per pair. Thread t walks diagonals j - i = off of the (P x Q) profile
// matrix: the last L G values live in a shift register, every completed window gives one
// distance, folded into the row minimum with ds_min_u64 on order-preserving keys. The median
// is an exact rank count over the P row minima in LDS.
#include "common.hpp"

namespace acoss {

namespace {

constexpr int kMaxL = 16;
constexpr int kMaxLen = 4096;  // LDS: 3 x 8 B x kMaxLen (window norms of a, b; row minima)

__device__ __forceinline__ unsigned long long dkey(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_inv(unsigned long long k) {
  const unsigned long long u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __builtin_bit_cast(double, u);
}

// per-track chroma profile (sum over time, sequential) and per-frame squared norms
__global__ void k_simple_track(const double* __restrict__ feats, const int64_t* __restrict__ off,
                               const int32_t* __restrict__ len, int n_tracks, double* __restrict__ prof,
                               double* __restrict__ fnorm, int64_t ldf) {
  const int tr = blockIdx.x;
  if (tr >= n_tracks) return;
  const double* S = feats + off[tr];
  const int n = len[tr];
  const int t = threadIdx.x;
  if (t < 12) {
    double acc = 0.0;
    for (int x = 0; x < n; ++x) acc = acc + S[(size_t)t * n + x];
    prof[tr * 12 + t] = acc;
  }
  for (int x = t; x < n; x += blockDim.x) {
    double acc = 0.0;
    for (int d = 0; d < 12; ++d) {
      const double v = S[(size_t)d * n + x];
      acc = acc + v * v;
    }
    fnorm[(size_t)tr * ldf + x] = acc;
  }
}

__global__ __launch_bounds__(256) void k_simple_pair(const double* __restrict__ feats, const int64_t* __restrict__ off,
                                                     const int32_t* __restrict__ len, const int32_t* __restrict__ pairs,
                                                     const double* __restrict__ prof, const double* __restrict__ fnorm,
                                                     int64_t ldf, int L, int apply_oti, double* __restrict__ score,
                                                     int32_t* __restrict__ oti_out) {
  __shared__ double sa[kMaxLen];
  __shared__ double sb[kMaxLen];
  __shared__ unsigned long long mpk[kMaxLen];
  __shared__ int s_k;
  __shared__ double s_med[2];
  const int p = blockIdx.x;
  const int t = threadIdx.x;
  const int ta = pairs[2 * p], tb = pairs[2 * p + 1];
  const int na = len[ta], nb = len[tb];
  const double* A = feats + off[ta];
  const double* B = feats + off[tb];
  const int P = na - L + 1, Q = nb - L + 1;
  if (t == 0) {
    // Simple.oti: v[k] = dot(p_a, roll(p_b, k)); argsort(v)[-1] -> last index of the maximum
    const double* pa = prof + ta * 12;
    const double* pb = prof + tb * 12;
    int best = 0;
    double bv = 0.0;
    for (int k = 0; k < 12; ++k) {
      double acc = 0.0;
      for (int c = 0; c < 12; ++c) acc = acc + pa[c] * pb[(c - k + 12) % 12];
      if (k == 0 || acc >= bv) {
        bv = acc;
        best = k;
      }
    }
    s_k = apply_oti ? best : 0;
    if (oti_out) oti_out[p] = best;
  }
  if (P <= 0 || Q <= 0) {
    if (t == 0) score[p] = __builtin_nan("");
    return;
  }
  // query window norms: sequential sums of L frame norms
  const double* fa = fnorm + (size_t)ta * ldf;
  for (int i = t; i < P; i += 256) {
    double acc = 0.0;
    for (int u = 0; u < L; ++u) acc = acc + fa[i + u];
    sa[i] = acc;
    mpk[i] = ~0ull;
  }
  __syncthreads();
  const int k = s_k;
  int rowB[12];  // rolled reference: Brot[c] = B[(c - k) mod 12]
#pragma unroll
  for (int c = 0; c < 12; ++c) rowB[c] = ((c - k + 12) % 12) * nb;
  // reference window norms in the rolled bin order (the oracle sums Brot's bins 0..11)
  for (int j = t; j < Q; j += 256) {
    double acc = 0.0;
    for (int u = 0; u < L; ++u) {
      double f = 0.0;
#pragma unroll
      for (int c = 0; c < 12; ++c) {
        const double v = B[rowB[c] + j + u];
        f = f + v * v;
      }
      acc = acc + f;
    }
    sb[j] = acc;
  }
  __syncthreads();
  for (int dg = t; dg < P + Q - 1; dg += 256) {
    const int o = dg - (P - 1);  // j - i
    const int r0 = o < 0 ? -o : 0;
    const int r1 = min(P - 1, Q - 1 - o);  // last row on this diagonal
    double buf[kMaxL];
#pragma unroll
    for (int u = 0; u < kMaxL; ++u) buf[u] = 0.0;
    for (int x = r0; x <= r1 + L - 1; ++x) {
      const int y = x + o;
      double g = 0.0;
#pragma unroll
      for (int c = 0; c < 12; ++c) g = g + A[(size_t)c * na + x] * B[rowB[c] + y];
#pragma unroll
      for (int u = 0; u < kMaxL - 1; ++u) buf[u] = buf[u + 1];
      buf[kMaxL - 1] = g;
      const int r = x - L + 1;
      if (r >= r0) {
        double qt = 0.0;
#pragma unroll
        for (int u = 0; u < kMaxL; ++u)
          if (u >= kMaxL - L) qt = qt + buf[u];
        const double dist = (sb[r + o] + sa[r]) - 2.0 * qt;
        atomicMin(&mpk[r], dkey(dist));
      }
    }
  }
  __syncthreads();
  // median: the order statistics P/2 (and P/2 - 1 for even P) by exact rank counting
  const int k_hi = P / 2, k_lo = (P % 2) ? P / 2 : P / 2 - 1;
  for (int e = t; e < P; e += 256) {
    const unsigned long long me = mpk[e];
    int less = 0, eq = 0;
    for (int f = 0; f < P; ++f) {
      const unsigned long long v = mpk[f];
      less += v < me;
      eq += v == me;
    }
    // the first holder (lowest index) of a tied value writes
    int first = 1;
    for (int f = 0; f < e; ++f) first &= mpk[f] != me;
    if (first) {
      if (less <= k_hi && k_hi < less + eq) s_med[1] = dkey_inv(me);
      if (less <= k_lo && k_lo < less + eq) s_med[0] = dkey_inv(me);
    }
  }
  __syncthreads();
  if (t == 0) score[p] = (P % 2) ? s_med[1] : 0.5 * (s_med[0] + s_med[1]);
}

}  // namespace
}  // namespace acoss

using namespace acoss;

extern "C" int acoss_simple_mp(const double* feats, const int64_t* track_off, const int32_t* track_len,
                               int32_t n_tracks, int32_t max_len, const int32_t* pairs, int64_t n_pairs, int32_t sslen,
                               int32_t apply_oti, double* score_out, int32_t* oti_out, void* hip_stream) {
  clear_error();
  if (n_tracks < 0 || n_pairs < 0 || (n_pairs > 0 && (!feats || !track_off || !track_len || !pairs || !score_out))) {
    set_error("acoss_simple_mp: bad arguments");
    return ACOSS_E_ARG;
  }
  if (sslen < 1 || sslen > kMaxL) {
    set_error("acoss_simple_mp: sslen=%d outside [1, %d]", sslen, kMaxL);
    return ACOSS_E_ARG;
  }
  if (max_len > kMaxLen) {
    set_error("acoss_simple_mp: max_len=%d exceeds %d SiMPle frames", max_len, kMaxLen);
    return ACOSS_E_SHAPE;
  }
  if (n_pairs == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  prof_begin(PH_SIMPLE, s);
  const int64_t ldf = (int64_t)align_up((size_t)max(max_len, 1), 64);
  const size_t bytes = align_up((size_t)n_tracks * 12 * 8, 256) + (size_t)n_tracks * ldf * 8;
  char* ws = static_cast<char*>(workspace(8, bytes));
  if (!ws) return ACOSS_E_HIP;
  double* prof = reinterpret_cast<double*>(ws);
  double* fnorm = reinterpret_cast<double*>(ws + align_up((size_t)n_tracks * 12 * 8, 256));
  hipLaunchKernelGGL(k_simple_track, dim3(n_tracks), dim3(256), 0, s, feats, track_off, track_len, n_tracks, prof,
                     fnorm, ldf);
  ACOSS_LAUNCH_CHECK();
  for (int64_t p0 = 0; p0 < n_pairs; p0 += 1 << 20) {
    const int64_t np = std::min<int64_t>(n_pairs - p0, 1 << 20);
    hipLaunchKernelGGL(k_simple_pair, dim3((unsigned)np), dim3(256), 0, s, feats, track_off, track_len, pairs + 2 * p0,
                       prof, fnorm, ldf, sslen, apply_oti, score_out + p0, oti_out ? oti_out + p0 : nullptr);
    ACOSS_LAUNCH_CHECK();
  }
  prof_end(PH_SIMPLE, s);
  return ACOSS_OK;
}
