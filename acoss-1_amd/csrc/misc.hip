// misc.hip — the acoss-side pairwise helpers used by EarlyFusionTraile (and exposed on their
// own through the C-ABI):
//   get_oti              acoss/algorithms/utils/cross_recurrence.py:75-103
//   get_csm / get_csm_cosine / get_ssm / get_csm_blocked_oti     cross_recurrence.py:10-134
//   csm_to_binary        cross_recurrence.py:136-161
//   getWCSM              acoss/algorithms/utils/similarity_fusion.py:38-54
//   smith_waterman_constrained   acoss/algorithms/utils/alignment_tools.py:7-46
#include <cstdlib>

#include "common.hpp"

namespace acoss {

namespace {

// ---------------------------------------------------------------------------------------
// get_oti: argmax_i sum(roll(C1, i) * C2), first max wins (np.argmax).
// ---------------------------------------------------------------------------------------
__global__ void k_get_oti(const float* __restrict__ C1, const float* __restrict__ C2, int n, int32_t* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  float a[12], b[12];
#pragma unroll
  for (int c = 0; c < 12; ++c) {
    a[c] = C1[k * 12 + c];
    b[c] = C2[k * 12 + c];
  }
  int best = 0;
  float bv = 0.0f;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    float s = 0.0f;  // np.sum of the 12 products (sequential; numpy pairwise == sequential below 8+)
#pragma unroll
    for (int c = 0; c < 12; ++c) s = s + a[(c - i + 12) % 12] * b[c];
    if (i == 0 || s > bv) {
      bv = s;
      best = i;
    }
  }
  out[k] = best;
}

// ---------------------------------------------------------------------------------------
// CSM: C = Xr . Yn^T on MFMA (v_mfma_f32_32x32x2_f32, exact f32), 64x64 tile per block of 4
// waves, K staged through LDS in chunks of 32; fused epilogue per kind:
//   0 euclid: sqrt(max(0, (|x|^2 + |y|^2) - 2 C))          (get_csm, :46-48)
//   1 cosine: 1 - C   on rows pre-normalised               (get_csm_cosine, :67-73)
//   2 ssm:    euclid of X with itself, diagonal forced 0    (get_ssm, :24-28)
// Xr = X with every 12-bin block rolled by `roll` (get_csm_blocked_oti, :131-133).
// ---------------------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kT = 64, kKC = 32;

__global__ void k_row_prep(const float* __restrict__ X, int M, int d, int roll, int normalise, float* __restrict__ Xo,
                           float* __restrict__ sq) {
  // one wave per row: rolled (and optionally L2-normalised) copy + squared norm
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* x = X + (size_t)row * d;
  float s = 0.0f;
  for (int c = lane; c < d; c += 64) s += x[c] * x[c];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float nrm = sqrtf(s);
  const float inv_den = (normalise && nrm != 0.0f) ? nrm : 1.0f;  // XNorm[XNorm == 0] = 1
  float s2 = 0.0f;
  for (int c = lane; c < d; c += 64) {
    int src = c;
    if (roll > 0) {  // np.roll over the chroma axis of each 12-bin block
      const int blk = c / 12, cc = c - blk * 12;
      src = blk * 12 + (cc - roll + 12) % 12;
    }
    const float v = normalise ? x[src] / inv_den : x[src];
    Xo[(size_t)row * d + c] = v;
    s2 += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o);
  if (lane == 0) sq[row] = s2;
}

template <int KIND>
__global__ __launch_bounds__(256) void k_csm(const float* __restrict__ X, const float* __restrict__ Y, int M, int N,
                                             int d, const float* __restrict__ xsq, const float* __restrict__ ysq,
                                             float* __restrict__ out) {
  __shared__ float Xs[kT][kKC + 1];
  __shared__ float Ys[kT][kKC + 1];
  const int bi = blockIdx.y * kT, bj = blockIdx.x * kT;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  f32x16 acc = {};
  for (int k0 = 0; k0 < d; k0 += kKC) {
    __syncthreads();
    for (int e = t; e < kT * kKC; e += 256) {
      const int r = e / kKC, c = e - r * kKC;
      const int k = k0 + c;
      Xs[r][c] = (bi + r < M && k < d) ? X[(size_t)(bi + r) * d + k] : 0.0f;
      Ys[r][c] = (bj + r < N && k < d) ? Y[(size_t)(bj + r) * d + k] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kKC; kk += 2) {
      const float a = Xs[32 * wr + (lane & 31)][kk + (lane >> 5)];
      const float b = Ys[32 * wc + (lane & 31)][kk + (lane >> 5)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
  }
  const int col = bj + 32 * wc + (lane & 31);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = bi + 32 * wr + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    if (row < M && col < N) {
      float v;
      if (KIND == 1) {
        v = 1.0f - acc[reg];
      } else {
        float c2 = (xsq[row] + ysq[col]) - 2.0f * acc[reg];
        if (c2 < 0.0f) c2 = 0.0f;
        if (KIND == 2 && row == col) c2 = 0.0f;
        v = sqrtf(c2);
      }
      out[(size_t)row * N + col] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// csm_to_binary: the nn smallest of every row -> 1 (ties: lowest column first).
// One wave per row; order-preserving u32 keys of the floats; lane l holds columns
// [l*KPL, (l+1)*KPL) in registers (KPL*64 >= N) or reads the row in passes.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __builtin_bit_cast(unsigned, f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(256) void k_binarize_rows(const float* __restrict__ D, int M, int N, int nn,
                                                       uint8_t* __restrict__ B) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* x = D + (size_t)row * N;
  uint8_t* o = B + (size_t)row * N;
  if (nn <= 0) {
    for (int c = lane; c < N; c += 64) o[c] = 1;
    return;
  }
  const int per = (N + 63) / 64;  // columns per lane (chunked)
  const int c0 = lane * per, c1 = min(N, c0 + per);
  // kth = smallest key with count(key <= kth) >= nn
  unsigned a = 0, b = 0xffffffffu;
  while (a < b) {
    const unsigned mid = a + ((b - a) >> 1);
    int c = 0;
    for (int k = c0; k < c1; ++k) c += fkey(x[k]) <= mid;
    if (wave_sum(c) >= nn)
      b = mid;
    else
      a = mid + 1;
  }
  const unsigned kth = a;
  int less = 0, eq = 0;
  for (int k = c0; k < c1; ++k) {
    const unsigned kk = fkey(x[k]);
    less += kk < kth;
    eq += kk == kth;
  }
  const int less_all = wave_sum(less);
  const int take_eq = nn - less_all;  // equal keys taken in column order
  const int eq_before = wave_incl_scan(eq) - eq;
  int seen = eq_before;
  for (int k = c0; k < c1; ++k) {
    const unsigned kk = fkey(x[k]);
    uint8_t v = kk < kth;
    if (kk == kth) {
      v = seen < take_eq;
      ++seen;
    }
    o[k] = v;
  }
}

// ---------------------------------------------------------------------------------------
// getWCSM: Eps = (mean of k2 smallest per row + mean of k1 smallest per column + CSM) / 3,
// W = exp(-CSM^2 / (2 (mu Eps)^2)).
// ---------------------------------------------------------------------------------------
template <bool COLS>
__global__ __launch_bounds__(256) void k_kmean(const float* __restrict__ C, int M, int N, int k, float* __restrict__ out) {
  // mean of the k smallest values of a row (COLS=false) or column, canonical order (kmean_canon)
  const int line = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nl = COLS ? N : M, len = COLS ? M : N;
  if (line >= nl) return;
  auto at = [&](int e) { return COLS ? C[(size_t)e * N + line] : C[(size_t)line * N + e]; };
  const float m = kmean_canon(at, len, k, lane);
  if (lane == 0) out[line] = m;
}

__global__ void k_wcsm_apply(const float* __restrict__ C, int M, int N, const float* __restrict__ r,
                             const float* __restrict__ c, float mu, float* __restrict__ W) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)M * N) return;
  const int i = (int)(e / N), j = (int)(e - (size_t)i * N);
  const float v = C[e];
  const float eps = ((r[i] + c[j]) + v) / 3.0f;
  const float me = mu * eps;
  W[e] = canon_expf(-(v * v) / (2.0f * (me * me)));
}

// ---------------------------------------------------------------------------------------
// smith_waterman_constrained in float64, one wave per matrix. The binary matrix arrives as a
// bit plane: word W[g][c] (u16) holds rows 16g..16g+15 of column c. Lane l owns R rows of a
// 64R-row band and sweeps the columns skewed by one per lane, reading one word per column
// (prefetched four columns ahead); boundary rows (2 of S, 3 of B) pass down with __shfl_up;
// bands chain through global memory.
//   S[i][j] = max((S[i-1][j-1] + m) + d(B[i-2][j-2]), (S[i-2][j-1] + m) + d(B[i-3][j-2]),
//                 (S[i-1][j-2] + m) + d(B[i-2][j-3]), 0),  i, j >= 3,
//   m = B[i-1][j-1] ? 1 : -1,  d(v) = v > 0 ? 0 : -0.7   (alignment_tools.py:7-46)
// R = 8 when the batch's matrices have <= 512 rows (56 of 64 lanes busy at 446 rows), else 16.
// ---------------------------------------------------------------------------------------
struct SwAbove {
  double sa, sb;  // S rows R-2, R-1 of the lane above
  unsigned b;     // B bits rows R-3, R-2, R-1 (bits 0..2)
};

template <int R>
__global__ __launch_bounds__(64) void k_swb(const uint16_t* __restrict__ W, int64_t wstride, int ldw,
                                            const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                            double4* __restrict__ bnd, int64_t bnd_stride, double* __restrict__ out) {
  static_assert(R == 8 || R == 16, "rows per lane");
  constexpr unsigned kMask = (1u << R) - 1;
  const int mid = blockIdx.x;
  const int lane = threadIdx.x;
  const int M = rows[mid], N = cols[mid];
  if (M < 4 || N < 4) {
    if (lane == 0) out[mid] = 0.0;
    return;
  }
  const uint16_t* Wm = W + (size_t)mid * wstride;
  const int nbands = (M + 64 * R - 1) / (64 * R);
  double best = 0.0;
  for (int band = 0; band < nbands; ++band) {
    const int row0 = band * 64 * R + lane * R;
    const bool rows_ok = row0 < M;
    const uint16_t* wr = Wm + (size_t)(row0 >> 4) * ldw;
    const int sh = row0 & 15;
    auto word = [&](int c) -> unsigned {
      return (rows_ok && c >= 0 && c < N) ? (((unsigned)wr[c] >> sh) & kMask) : 0u;
    };
    double4* bout = bnd + (size_t)mid * bnd_stride + (size_t)band * N;
    const double4* bin = bnd + (size_t)mid * bnd_stride + (size_t)(band - 1) * N;
    const int lanes = min(64, (M - band * 64 * R + R - 1) / R);  // lanes holding rows of this band
    double s1[R], s2[R];                                         // columns c-1, c-2
#pragma unroll
    for (int r = 0; r < R; ++r) s1[r] = s2[r] = 0.0;
    unsigned w1 = 0, w2 = 0, w3 = 0;  // B bits of my rows at c-1, c-2, c-3
    SwAbove h1{0, 0, 0}, h2{0, 0, 0}, h3{0, 0, 0};
    double pa = 0.0, pb = 0.0;
    unsigned pbits = 0;
    unsigned q0 = word(-lane), q1 = word(1 - lane), q2 = word(2 - lane), q3 = word(3 - lane);
    const int S_end = N + lanes - 1;
    for (int s = 0; s < S_end; ++s) {
      const int c = s - lane;
      const unsigned w0 = q0;
      q0 = q1;
      q1 = q2;
      q2 = q3;
      q3 = word(c + 4);
      SwAbove h0;
      h0.sa = __shfl_up(pa, 1);
      h0.sb = __shfl_up(pb, 1);
      h0.b = (unsigned)__shfl_up((int)pbits, 1);
      if (lane == 0) {
        if (band > 0 && c >= 0 && c < N) {
          const double4 v = bin[c];
          h0.sa = v.x;
          h0.sb = v.y;
          h0.b = (unsigned)v.z;
        } else {
          h0.sa = h0.sb = 0.0;
          h0.b = 0;
        }
      }
      // extended bit words: bit r+3 <-> my row r; bits 0..2 <-> rows -3..-1
      const uint32_t e1 = (w1 << 3) | h1.b;
      const uint32_t e2 = (w2 << 3) | h2.b;
      const uint32_t e3 = (w3 << 3) | h3.b;
      const bool cok = c >= 3 && c < N;
      double s0[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double A = r >= 1 ? s1[r - 1] : h1.sb;                     // S[i-1][c-1]
        const double Bv = r >= 2 ? s1[r - 2] : (r == 1 ? h1.sb : h1.sa);  // S[i-2][c-1]
        const double Cv = r >= 1 ? s2[r - 1] : h2.sb;                    // S[i-1][c-2]
        const double mv = ((e1 >> (r + 2)) & 1) ? 1.0 : -1.0;            // B[i-1][c-1]
        const double d1 = ((e2 >> (r + 1)) & 1) ? 0.0 : -0.7;            // B[i-2][c-2]
        const double d2 = ((e2 >> r) & 1) ? 0.0 : -0.7;                  // B[i-3][c-2]
        const double d3 = ((e3 >> (r + 1)) & 1) ? 0.0 : -0.7;            // B[i-2][c-3]
        const double x1 = (A + mv) + d1;
        const double x2 = (Bv + mv) + d2;
        const double x3 = (Cv + mv) + d3;
        double v = x1;
        v = x2 > v ? x2 : v;
        v = x3 > v ? x3 : v;
        v = 0.0 > v ? 0.0 : v;
        const int i = row0 + r;
        v = (cok && i >= 3 && i < M) ? v : 0.0;
        best = v > best ? v : best;
        s0[r] = v;
      }
      pa = s0[R - 2];
      pb = s0[R - 1];
      pbits = (w0 >> (R - 3)) & 7u;
      if (lane == 63 && band + 1 < nbands && c >= 0 && c < N) bout[c] = make_double4(pa, pb, (double)pbits, 0.0);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        s2[r] = s1[r];
        s1[r] = s0[r];
      }
      w3 = w2;
      w2 = w1;
      w1 = w0;
      h3 = h2;
      h2 = h1;
      h1 = h0;
    }
    __threadfence_block();
    __syncthreads();
  }
  best = wave_max(best);
  if (lane == 0) out[mid] = best;
}

// Small matrices (at most 64 LP rows, LP <= 32: EarlyFusion's beat-block CSMs, M ~ 14..47): a
// group of LP lanes per matrix (lane ll of a group owns rows 8 ll .. 8 ll + 7, one band), G = 64 /
// LP matrices per wave instead of one matrix per wave with most lanes idle. The same cell
// recurrence in the same order as k_swb<8>, so the same scores bit for bit.
__global__ __launch_bounds__(64) void k_swb_grp(const uint16_t* __restrict__ W, int64_t wstride, int ldw,
                                                const int32_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                                int n, int LP, double* __restrict__ out) {
  constexpr int R = 8;
  constexpr unsigned kMask = (1u << R) - 1;
  __shared__ double s_best[64];
  const int lane = threadIdx.x;
  const int G = 64 / LP;
  const int g = lane / LP, ll = lane - g * LP;
  const int mid = blockIdx.x * G + g;
  const bool in_group = g < G && mid < n;
  const int M = in_group ? rows[mid] : 0, N = in_group ? cols[mid] : 0;
  const bool live = in_group && M >= 4 && N >= 4;
  const int row0 = ll * R;
  const bool rows_ok = live && row0 < M;
  const uint16_t* wr = W + (size_t)(in_group ? mid : 0) * wstride + (size_t)(row0 >> 4) * ldw;
  const int sh = row0 & 15;
  auto word = [&](int c) -> unsigned {
    return (rows_ok && c >= 0 && c < N) ? (((unsigned)wr[c] >> sh) & kMask) : 0u;
  };
  double s1[R], s2[R];
#pragma unroll
  for (int r = 0; r < R; ++r) s1[r] = s2[r] = 0.0;
  unsigned w1 = 0, w2 = 0, w3 = 0;
  SwAbove h1{0, 0, 0}, h2{0, 0, 0}, h3{0, 0, 0};
  double pa = 0.0, pb = 0.0, best = 0.0;
  unsigned pbits = 0;
  unsigned q0 = word(-ll), q1 = word(1 - ll), q2 = word(2 - ll), q3 = word(3 - ll);
  // steps until every group of the wave is done (wave-uniform bound)
  const int S_end = (int)wave_max_u32(live ? (unsigned)(N + LP - 1) : 0u);
  for (int s = 0; s < S_end; ++s) {
    const int c = s - ll;
    const unsigned w0 = q0;
    q0 = q1;
    q1 = q2;
    q2 = q3;
    q3 = word(c + 4);
    SwAbove h0;
    h0.sa = __shfl_up(pa, 1);
    h0.sb = __shfl_up(pb, 1);
    h0.b = (unsigned)__shfl_up((int)pbits, 1);
    if (ll == 0) {  // the group's first rows: nothing above
      h0.sa = h0.sb = 0.0;
      h0.b = 0;
    }
    const uint32_t e1 = (w1 << 3) | h1.b;
    const uint32_t e2 = (w2 << 3) | h2.b;
    const uint32_t e3 = (w3 << 3) | h3.b;
    const bool cok = c >= 3 && c < N;
    double s0[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double A = r >= 1 ? s1[r - 1] : h1.sb;
      const double Bv = r >= 2 ? s1[r - 2] : (r == 1 ? h1.sb : h1.sa);
      const double Cv = r >= 1 ? s2[r - 1] : h2.sb;
      const double mv = ((e1 >> (r + 2)) & 1) ? 1.0 : -1.0;
      const double d1 = ((e2 >> (r + 1)) & 1) ? 0.0 : -0.7;
      const double d2 = ((e2 >> r) & 1) ? 0.0 : -0.7;
      const double d3 = ((e3 >> (r + 1)) & 1) ? 0.0 : -0.7;
      const double x1 = (A + mv) + d1;
      const double x2 = (Bv + mv) + d2;
      const double x3 = (Cv + mv) + d3;
      double v = x1;
      v = x2 > v ? x2 : v;
      v = x3 > v ? x3 : v;
      v = 0.0 > v ? 0.0 : v;
      const int i = row0 + r;
      v = (cok && i >= 3 && i < M) ? v : 0.0;
      best = v > best ? v : best;
      s0[r] = v;
    }
    pa = s0[R - 2];
    pb = s0[R - 1];
    pbits = (w0 >> (R - 3)) & 7u;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      s2[r] = s1[r];
      s1[r] = s0[r];
    }
    w3 = w2;
    w2 = w1;
    w1 = w0;
    h3 = h2;
    h2 = h1;
    h1 = h0;
  }
  // per-group maximum through LDS (groups need not be a power of two wide)
  s_best[lane] = best;
  __syncthreads();
  if (in_group && ll == 0) {
    double m = 0.0;
    for (int k = 0; k < LP; ++k) m = s_best[lane + k] > m ? s_best[lane + k] : m;
    out[mid] = live ? m : 0.0;
  }
}

// Byte matrices (acoss_sw_constrained's layout) -> bit planes; flags elements other than 0/1.
__global__ void k_sw_pack(const uint8_t* __restrict__ mats, const int64_t* __restrict__ off,
                          const int32_t* __restrict__ rows, const int32_t* __restrict__ cols, uint16_t* __restrict__ W,
                          int64_t wstride, int ldw, int* __restrict__ err) {
  const int mid = blockIdx.x, g = blockIdx.y;
  const int c = blockIdx.z * blockDim.x + threadIdx.x;
  const int M = rows[mid], N = cols[mid];
  if (c >= N || 16 * g >= M) return;
  const uint8_t* B = mats + off[mid];
  unsigned w = 0;
  bool bad = false;
  for (int r = 0; r < 16; ++r) {
    const int i = 16 * g + r;
    if (i < M) {
      const uint8_t v = B[(size_t)i * N + c];
      bad |= v > 1;
      w |= (unsigned)(v != 0) << r;
    }
  }
  W[(size_t)mid * wstride + (size_t)g * ldw + c] = (uint16_t)w;
  if (bad) atomicOr(err, 1);
}

int sw_rows_per_lane(int max_rows) { return max_rows <= 512 ? 8 : 16; }

}  // namespace

size_t sw_bnd_bytes(int max_rows, int max_cols) {
  const int R = sw_rows_per_lane(max_rows);
  const int nbands = (max_rows + 64 * R - 1) / (64 * R);
  return nbands > 1 ? 32 * (size_t)nbands * align_up((size_t)max_cols, 8) : 32;
}

// Batched constrained Smith-Waterman over bit planes (also used by earlyfusion.hip): matrix
// mid's words start at W + mid * wstride, row stride ldw words; bnd: sw_bnd_bytes per matrix.
int launch_swb_batch(const uint16_t* W, int64_t wstride, int ldw, const int32_t* rows, const int32_t* cols, int n,
                     int max_rows, int max_cols, void* bnd, double* out, hipStream_t s) {
  const int64_t bstride = (int64_t)(sw_bnd_bytes(max_rows, max_cols) / 32);
  const int LP = (max_rows + 7) / 8;  // lanes per matrix at 8 rows per lane
  if (LP <= 32) {  // two or more matrices per wave (Da-TACOS EarlyFusion: +18 % over one per wave)
    const int G = 64 / LP;
    hipLaunchKernelGGL(k_swb_grp, dim3((unsigned)((n + G - 1) / G)), dim3(64), 0, s, W, wstride, ldw, rows, cols, n, LP,
                       out);
  } else if (sw_rows_per_lane(max_rows) == 8)
    hipLaunchKernelGGL(k_swb<8>, dim3(n), dim3(64), 0, s, W, wstride, ldw, rows, cols, static_cast<double4*>(bnd),
                       bstride, out);
  else
    hipLaunchKernelGGL(k_swb<16>, dim3(n), dim3(64), 0, s, W, wstride, ldw, rows, cols, static_cast<double4*>(bnd),
                       bstride, out);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

}  // namespace acoss

using namespace acoss;

extern "C" int acoss_get_oti(const float* C1, const float* C2, int32_t n, int32_t* out, void* hip_stream) {
  clear_error();
  if (n < 0 || (n > 0 && (!C1 || !C2 || !out))) {
    set_error("acoss_get_oti: bad arguments");
    return ACOSS_E_ARG;
  }
  if (n == 0) return ACOSS_OK;
  hipLaunchKernelGGL(k_get_oti, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(hip_stream), C1, C2, n,
                     out);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

extern "C" int acoss_csm(const float* X, int32_t M, const float* Y, int32_t N, int32_t d, int32_t kind,
                         int32_t oti_shift, float* out, void* hip_stream) {
  clear_error();
  if (M < 0 || N < 0 || d <= 0 || kind < 0 || kind > 2 || !X || !out || (kind != 2 && !Y)) {
    set_error("acoss_csm: bad arguments");
    return ACOSS_E_ARG;
  }
  if (oti_shift > 0 && d % 12 != 0) {
    set_error("acoss_csm: oti_shift needs d to be a multiple of 12");
    return ACOSS_E_ARG;
  }
  if (kind == 2) {
    Y = X;
    N = M;
  }
  if (M == 0 || N == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  prof_begin(PH_CSM, s);
  const size_t bytes = align_up((size_t)M * d * 4, 256) * 2 + align_up((size_t)(M + N) * 4, 256);
  char* ws = static_cast<char*>(workspace(4, bytes));
  if (!ws) return ACOSS_E_HIP;
  float* Xp = reinterpret_cast<float*>(ws);
  float* Yp = reinterpret_cast<float*>(ws + align_up((size_t)M * d * 4, 256));
  float* sq = reinterpret_cast<float*>(ws + 2 * align_up((size_t)M * d * 4, 256));
  const int roll = oti_shift > 0 ? oti_shift % 12 : 0;
  const int norm = kind == 1;
  // workspace slot 4 holds the prepared X; Y gets its own slot (may be larger than X)
  float* Yw = reinterpret_cast<float*>(workspace(5, align_up((size_t)N * d * 4, 256) + align_up((size_t)N * 4, 256)));
  if (!Yw) return ACOSS_E_HIP;
  float* ysq = Yw + align_up((size_t)N * d, 64);
  (void)Yp;
  hipLaunchKernelGGL(k_row_prep, dim3((M + 3) / 4), dim3(256), 0, s, X, M, d, roll, norm, Xp, sq);
  ACOSS_LAUNCH_CHECK();
  if (kind == 2) {
    hipLaunchKernelGGL(k_row_prep, dim3((N + 3) / 4), dim3(256), 0, s, X, N, d, 0, 0, Yw, ysq);
  } else {
    hipLaunchKernelGGL(k_row_prep, dim3((N + 3) / 4), dim3(256), 0, s, Y, N, d, 0, norm, Yw, ysq);
  }
  ACOSS_LAUNCH_CHECK();
  const dim3 grid((N + kT - 1) / kT, (M + kT - 1) / kT);
  if (kind == 0)
    hipLaunchKernelGGL(k_csm<0>, grid, dim3(256), 0, s, Xp, Yw, M, N, d, sq, ysq, out);
  else if (kind == 1)
    hipLaunchKernelGGL(k_csm<1>, grid, dim3(256), 0, s, Xp, Yw, M, N, d, sq, ysq, out);
  else
    hipLaunchKernelGGL(k_csm<2>, grid, dim3(256), 0, s, Xp, Yw, M, N, d, sq, ysq, out);
  ACOSS_LAUNCH_CHECK();
  prof_end(PH_CSM, s);
  return ACOSS_OK;
}

extern "C" int acoss_binarize_rows(const float* D, int32_t M, int32_t N, int32_t nneighbs, uint8_t* B,
                                   void* hip_stream) {
  clear_error();
  if (M < 0 || N < 0 || (M > 0 && N > 0 && (!D || !B)) || nneighbs > N) {
    set_error("acoss_binarize_rows: bad arguments (nneighbs=%d, N=%d)", nneighbs, N);
    return ACOSS_E_ARG;
  }
  if (M == 0 || N == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  prof_begin(PH_BIN, s);
  hipLaunchKernelGGL(k_binarize_rows, dim3((M + 3) / 4), dim3(256), 0, s, D, M, N, nneighbs, B);
  ACOSS_LAUNCH_CHECK();
  prof_end(PH_BIN, s);
  return ACOSS_OK;
}

extern "C" int acoss_wcsm(const float* CSM, int32_t M, int32_t N, int32_t k1, int32_t k2, float mu, float* W,
                          void* hip_stream) {
  clear_error();
  if (M <= 0 || N <= 0 || !CSM || !W || k1 <= 0 || k2 <= 0 || k1 > M || k2 > N) {
    set_error("acoss_wcsm: bad arguments");
    return ACOSS_E_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  prof_begin(PH_WCSM, s);
  float* ws = static_cast<float*>(workspace(6, ((size_t)M + N) * 4 + 256));
  if (!ws) return ACOSS_E_HIP;
  float* rmean = ws;
  float* cmean = ws + M;
  hipLaunchKernelGGL(k_kmean<false>, dim3((M + 3) / 4), dim3(256), 0, s, CSM, M, N, k2, rmean);
  ACOSS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_kmean<true>, dim3((N + 3) / 4), dim3(256), 0, s, CSM, M, N, k1, cmean);
  ACOSS_LAUNCH_CHECK();
  const size_t tot = (size_t)M * N;
  hipLaunchKernelGGL(k_wcsm_apply, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, CSM, M, N, rmean, cmean, mu,
                     W);
  ACOSS_LAUNCH_CHECK();
  prof_end(PH_WCSM, s);
  return ACOSS_OK;
}

__global__ void k_neg_exp(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) out[e] = canon_expf(-x[e]);
}

extern "C" int acoss_neg_exp(const float* x, int64_t n, float* out, void* hip_stream) {
  clear_error();
  if (n < 0 || (n > 0 && (!x || !out))) {
    set_error("acoss_neg_exp: bad arguments");
    return ACOSS_E_ARG;
  }
  if (n == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  hipLaunchKernelGGL(k_neg_exp, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n, out);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

extern "C" int acoss_sw_constrained(const uint8_t* mats, const int64_t* off, const int32_t* rows, const int32_t* cols,
                                    int32_t n_mats, int32_t max_rows, int32_t max_cols, double* score_out,
                                    void* hip_stream) {
  clear_error();
  if (n_mats < 0 || (n_mats > 0 && (!mats || !off || !rows || !cols || !score_out)) || max_rows < 0 || max_cols < 0) {
    set_error("acoss_sw_constrained: bad arguments");
    return ACOSS_E_ARG;
  }
  if (n_mats == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  prof_begin(PH_SW, s);
  const int G = (max_rows + 15) / 16;
  const int ldw = (int)align_up((size_t)max_cols, 4);
  const int64_t wstride = (int64_t)G * ldw;
  const size_t bb = sw_bnd_bytes(max_rows, max_cols);
  char* ws = static_cast<char*>(workspace(7, 256 + bb * n_mats + align_up((size_t)wstride * 2 * n_mats, 256)));
  if (!ws) return ACOSS_E_HIP;
  int* d_err = reinterpret_cast<int*>(ws);
  void* bnd = ws + 256;
  uint16_t* W = reinterpret_cast<uint16_t*>(ws + 256 + bb * n_mats);
  ACOSS_HIP_CHECK(hipMemsetAsync(d_err, 0, 4, s));
  if (G > 0 && max_cols > 0) {
    hipLaunchKernelGGL(k_sw_pack, dim3(n_mats, G, (max_cols + 255) / 256), dim3(256), 0, s, mats, off, rows, cols, W,
                       wstride, ldw, d_err);
    ACOSS_LAUNCH_CHECK();
  }
  int rc = launch_swb_batch(W, wstride, ldw, rows, cols, n_mats, max_rows, max_cols, bnd, score_out, s);
  if (rc) return rc;
  prof_end(PH_SW, s);
  int h_err = 0;
  ACOSS_HIP_CHECK(hipMemcpyAsync(&h_err, d_err, 4, hipMemcpyDeviceToHost, s));
  ACOSS_HIP_CHECK(hipStreamSynchronize(s));
  if (h_err) {
    set_error("smith_waterman_constrained: Non-binary elements found in input");
    return ACOSS_E_NONBINARY;
  }
  return ACOSS_OK;
}
