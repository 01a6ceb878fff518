// ef_oracle.cpp — CPU restatement of EarlyFusion's per-feature scores in a canonical order.
//
// TEST INFRASTRUCTURE ONLY (parity checker; built into oracle/_build/liboracle.so with
// crp_oracle.cpp). The product path (acoss-1_amd/) never links or calls it.
//
// What it restates: the four scores of EarlyFusion.similarity
// (/root/reference/acoss/algorithms/earlyfusion_traile.py:165-183):
//   mfccs   = smith_waterman_constrained(csm_to_binary(get_csm(mfccs_a, mfccs_b), kappa))
//   ssms    = smith_waterman_constrained(csm_to_binary(get_csm(ssms_a, ssms_b), kappa))
//   chromas = smith_waterman_constrained(csm_to_binary(get_csm_blocked_oti(chromas_a, chromas_b,
//                                          med_a, med_b, get_csm_cosine), kappa))
//   early   = smith_waterman_constrained(csm_to_binary(exp(-(((0 + W_m) + W_s) + W_c)), kappa)),
//             W_f = getWCSM(CSM_f, K, K) (acoss/algorithms/utils/similarity_fusion.py:38-54)
// with get_csm / get_csm_cosine / get_oti / get_csm_blocked_oti from
// acoss/algorithms/utils/cross_recurrence.py:30-134, csm_to_binary :136-161 and
// smith_waterman_constrained from alignment_tools.py:25-46 (or_sw_constrained).
//
// The reference computes the CSMs with numpy BLAS products, whose float32 summation order is
// unspecified (and differs between BLAS builds). This restatement fixes ONE order, the one the
// HIP kernels (earlyfusion.hip) follow, so the two can be compared with ==; np_oracle's
// BLAS-order composition (golden-pinned get_csm / get_csm_cosine) checks it within float32
// tolerance (tests/test_ef_oracle.py). Canonical arithmetic, float32 unless noted:
//   row norm   s_l = sum_{c = l mod 64} (x[c] * x[c]) sequential per l < 64 (product rounded,
//              then added), then a xor butterfly over l: s_l = s_l + s_{l ^ o}, o = 32 .. 1;
//              the value of l = 0 (all lanes agree: every add is commutative)
//   cosine     xn = x / (sqrt(s) != 0 ? sqrt(s) : 1)                    (cross_recurrence.py:67-70)
//   oti        s_i = sum_c (a[(c - i) mod 12] * b[c]) sequential adds; first maximum (np.argmax)
//   roll       query block g: X1[12 g + c] = xn[12 g + (c - oti) mod 12]       (np.roll, :124-131)
//   dot        fmaf chain over k ascending from +0 (the MFMA f32 chain)
//   euclid     d2 = (s_a + s_b) - 2 dot; D = sqrt(max(d2, 0))               (:47-51)
//   cosine CSM D = 1 - dot                                                   (:71-73)
//   binarize   nn = kappa < 1 ? rint(kappa * N) : (int)kappa (np.round: half to even); the nn
//              smallest of each row by (value, column): ties go to the lowest column (the
//              reference's argpartition leaves the choice unspecified)
//   k-means    getWCSM's mean of the K smallest of a row / column: the K smallest values (NaN never
//              taken, +inf when fewer than K are not NaN) added one at a time in ASCENDING order to
//              +0, then / K (np.mean of np.partition's output sums in an unspecified order)
//   getWCSM    Eps = ((rmean_i + cmean_j) + CSM) / 3; W = exp(-(CSM * CSM) / (2 ((mu Eps) (mu Eps))))
//   exp        canon_expf: one fixed sequence of correctly rounded double operations (below; the
//              HIP kernels' copy is acoss-1_amd/csrc/common.hpp canon_expf), so no libm / ocml
//              last-ulp differences enter; < 1e-15 relative before the rounding to float
// Build: oracle/Makefile (g++ -O3 -march=x86-64-v3 -ffp-contract=off -fopenmp).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

extern "C" double or_sw_constrained(const uint8_t* B, int M, int N);

namespace {

float row_sq(const float* x, int d) {
  float s[64];
  for (int l = 0; l < 64; ++l) {
    float a = 0.0f;
    for (int c = l; c < d; c += 64) {
      const float p = x[c] * x[c];
      a = a + p;
    }
    s[l] = a;
  }
  for (int o = 32; o > 0; o >>= 1) {
    float t[64];
    for (int l = 0; l < 64; ++l) t[l] = s[l] + s[l ^ o];
    std::memcpy(s, t, sizeof s);
  }
  return s[0];
}

int ef_oti(const float* a, const float* b) {
  int best = 0;
  float bv = 0.0f;
  for (int i = 0; i < 12; ++i) {
    float s = 0.0f;
    for (int c = 0; c < 12; ++c) {
      const float p = a[(c - i + 12) % 12] * b[c];
      s = s + p;
    }
    if (i == 0 || s > bv) {
      bv = s;
      best = i;
    }
  }
  return best;
}

float canon_expf(float xf) {
  const double x = (double)xf;
  if (x != x) return xf;
  if (x < -104.0) return 0.0f;
  if (x > 89.0) return INFINITY;
  const double k = std::nearbyint(x * 0x1.71547652b82fep+0);
  double r = std::fma(-k, 0x1.62e42fefa39efp-1, x);
  r = std::fma(-k, 0x1.abc9e3b39803fp-56, r);
  static const double c[14] = {0x1p+0, 0x1p+0, 0x1p-1, 0x1.5555555555555p-3, 0x1.5555555555555p-5,
                               0x1.1111111111111p-7, 0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-13,
                               0x1.a01a01a01a01ap-16, 0x1.71de3a556c734p-19, 0x1.27e4fb7789f5cp-22,
                               0x1.ae64567f544e4p-26, 0x1.1eed8eff8d898p-29, 0x1.6124613a86d09p-33};  // 1/n!
  double p = c[13];
  for (int n = 12; n >= 0; --n) p = std::fma(p, r, c[n]);
  uint64_t bits = (uint64_t)((int64_t)k + 1023) << 52;
  double sc;
  std::memcpy(&sc, &bits, 8);
  return (float)(p * sc);
}

inline uint32_t fkey(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

void binarize(const float* D, int M, int N, double kappa, uint8_t* B) {
  if (kappa == 0.0) {
    std::fill(B, B + (size_t)M * N, 1);
    return;
  }
  int nn = kappa < 1.0 ? (int)std::nearbyint(kappa * (double)N) : (int)kappa;
  nn = std::min(nn, N);
  std::fill(B, B + (size_t)M * N, 0);
  if (nn <= 0) return;
  std::vector<uint64_t> k(N);
  for (int i = 0; i < M; ++i) {
    for (int j = 0; j < N; ++j) k[j] = ((uint64_t)fkey(D[(size_t)i * N + j]) << 32) | (uint32_t)j;
    std::nth_element(k.begin(), k.begin() + (nn - 1), k.end());
    const uint64_t kth = k[nn - 1];
    for (int j = 0; j < N; ++j)
      if ((((uint64_t)fkey(D[(size_t)i * N + j]) << 32) | (uint32_t)j) <= kth) B[(size_t)i * N + j] = 1;
  }
}

// Mean of the k smallest of n values at x[0], x[stride], ... (canonical ascending order).
float kmean(const float* x, int n, int64_t stride, int k, std::vector<float>& buf) {
  buf.clear();
  for (int e = 0; e < n; ++e) {
    const float v = x[(int64_t)e * stride];
    if (v == v) buf.push_back(v);
  }
  const int take = std::min<int>(k, (int)buf.size());
  std::partial_sort(buf.begin(), buf.begin() + take, buf.end());
  float s = 0.0f;
  for (int t = 0; t < take; ++t) s = s + buf[t];
  if (take < k) s = s + INFINITY;
  return s / (float)k;
}

// getWCSM(D, k1, k2, mu) (similarity_fusion.py:38-54): k2 smallest per row, k1 per column.
void wcsm(const float* D, int M, int N, int k1, int k2, float mu, float* W) {
  std::vector<float> rm(M), cm(N), buf;
  for (int i = 0; i < M; ++i) rm[i] = kmean(D + (size_t)i * N, N, 1, k2, buf);
  for (int j = 0; j < N; ++j) cm[j] = kmean(D + j, M, N, k1, buf);
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      const float v = D[(size_t)i * N + j];
      const float eps = ((rm[i] + cm[j]) + v) / 3.0f;
      const float me = mu * eps;
      const float num = -(v * v);
      const float den = 2.0f * (me * me);
      W[(size_t)i * N + j] = canon_expf(num / den);
    }
}

// Euclidean (kind 0) or OTI-rolled cosine (kind 1) CSM of X (M x d) against Y (N x d).
void csm(const float* X, int M, const float* Y, int N, int d, int kind, int oti, float* D) {
  std::vector<float> xs(M), ys(N);
  std::vector<float> Xn, Yn;
  const float* A = X;
  const float* Bm = Y;
  if (kind == 0) {
    for (int i = 0; i < M; ++i) xs[i] = row_sq(X + (size_t)i * d, d);
    for (int j = 0; j < N; ++j) ys[j] = row_sq(Y + (size_t)j * d, d);
  } else {
    Xn.resize((size_t)M * d);
    Yn.resize((size_t)N * d);
    auto norm_rows = [&](const float* S, int n, std::vector<float>& O, bool roll) {
      std::vector<float> tmp(d);
      for (int i = 0; i < n; ++i) {
        const float* x = S + (size_t)i * d;
        const float r = std::sqrt(row_sq(x, d));
        const float den = r != 0.0f ? r : 1.0f;
        for (int c = 0; c < d; ++c) tmp[c] = x[c] / den;
        float* o = &O[(size_t)i * d];
        if (roll) {
          for (int g = 0; g < d / 12; ++g)
            for (int c = 0; c < 12; ++c) o[12 * g + c] = tmp[12 * g + (c - oti + 12) % 12];
        } else {
          std::memcpy(o, tmp.data(), sizeof(float) * d);
        }
      }
    };
    norm_rows(X, M, Xn, oti != 0);
    norm_rows(Y, N, Yn, false);
    A = Xn.data();
    Bm = Yn.data();
  }
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      const float* a = A + (size_t)i * d;
      const float* b = Bm + (size_t)j * d;
      float acc = 0.0f;
      for (int c = 0; c < d; ++c) acc = std::fma(a[c], b[c], acc);
      float v;
      if (kind == 0) {
        float c2 = (xs[i] + ys[j]) - 2.0f * acc;
        if (c2 < 0.0f) c2 = 0.0f;
        v = std::sqrt(c2);
      } else {
        v = 1.0f - acc;
      }
      D[(size_t)i * N + j] = v;
    }
}

}  // namespace

extern "C" {

// One feature's CSM for the canonical-order checks: kind 0 euclid, 1 cosine with the OTI of
// med_a / med_b (nullptr: no roll).
void or_ef_csm(const float* X, int M, const float* Y, int N, int d, int kind, const float* med_a,
               const float* med_b, float* D) {
  const int oti = (kind == 1 && med_a && med_b) ? ef_oti(med_a, med_b) : 0;
  csm(X, M, Y, N, d, kind, oti, D);
}

int or_ef_oti(const float* med_a, const float* med_b) { return ef_oti(med_a, med_b); }

void or_ef_binarize(const float* D, int M, int N, double kappa, uint8_t* B) { binarize(D, M, N, kappa, B); }

void or_ef_wcsm(const float* D, int M, int N, int k1, int k2, float mu, float* W) { wcsm(D, M, N, k1, k2, mu, W); }

float or_canon_expf(float x) { return canon_expf(x); }

// The four scores (mfccs, ssms, chromas, early) of every pair into scores[4 p + f]. Banks of packed
// block rows (block offsets off[t], counts nb[t]); med: (T, 12) chroma medians; K, mu: getWCSM's.
int or_ef_batch(const float* mf, int d_m, const float* ss, int d_s, const float* ch, int d_c, const float* med,
                const int64_t* off, const int32_t* nb, const int32_t* pairs, int64_t n_pairs, double kappa, int K,
                float mu, double* scores, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t p = 0; p < n_pairs; ++p) {
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int M = nb[a], N = nb[b];
    std::vector<float> D((size_t)M * N), W((size_t)M * N), S((size_t)M * N, 0.0f);
    std::vector<uint8_t> B((size_t)M * N);
    const float* banks[3] = {mf, ss, ch};
    const int dims[3] = {d_m, d_s, d_c};
    for (int f = 0; f < 3; ++f) {
      const int d = dims[f];
      const int oti = f == 2 ? ef_oti(med + 12 * a, med + 12 * b) : 0;
      csm(banks[f] + off[a] * d, M, banks[f] + off[b] * d, N, d, f == 2 ? 1 : 0, oti, D.data());
      binarize(D.data(), M, N, kappa, B.data());
      scores[4 * p + f] = or_sw_constrained(B.data(), M, N);
      wcsm(D.data(), M, N, K, K, mu, W.data());
      for (size_t e = 0; e < S.size(); ++e) S[e] = S[e] + W[e];  // WCSM_sum += W (:179-181)
    }
    for (size_t e = 0; e < S.size(); ++e) S[e] = canon_expf(-S[e]);  // np.exp(-WCSM_sum) (:182)
    binarize(S.data(), M, N, kappa, B.data());
    scores[4 * p + 3] = or_sw_constrained(B.data(), M, N);
  }
  return 0;
}

}  // extern "C"
