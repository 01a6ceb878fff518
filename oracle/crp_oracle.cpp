// crp_oracle.cpp — CPU restatement of the acoss all-pairs hot path.
//
// TEST INFRASTRUCTURE ONLY. This file is the parity checker and the timed CPU baseline
// (bench.py's `cpu_baseline` leg). Only tests/, __graft_entry__.smoke() and bench.py may
// load the library built from it (oracle/_build/liboracle.so). The product path
// (acoss-1_amd/) never links or calls it.
//
// What it restates
// ----------------
// * essentia ChromaCrossSimilarity(frameStackSize=m, frameStackStride=tau,
//   binarizePercentile=kappa, oti=True) as called at
//   /root/reference/acoss/algorithms/rqa_serra09.py:60-66 and latefusion_chen.py:63-69.
// * essentia CoverSongSimilarity(alignmentType='serra09'|'chen17', distanceType='symmetric')
//   as called at rqa_serra09.py:64,67 and latefusion_chen.py:67-71.
//   essentia is a third-party dependency that is NOT in /root/reference (setup.py:53
//   `extra-deps: essentia`, install.sh:32, version unpinned). Its published algorithm
//   (Serra et al. 2009 NJP 11:093017, Serra/Gomez/Herrera 2008 OTI, Chen et al. 2017,
//   essentia 2.1-beta6 docs) is restated below. PARITY WITH ESSENTIA IS UNPINNED: the
//   reference's own tests hold no vector for it (test/basetest.py is an import smoke test);
//   the conventions chosen are frozen by the known-answer tests test_kat_* in
//   tests/test_oracle_golden.py.
// * acoss smith_waterman_constrained (alignment_tools.py:7-46), bit-exact float64.
// * acoss Simple.simple_sim (simple_silva.py:68-118), float64 (direct sums instead of the
//   reference's FFT + STOMP updates; agrees to ~1e-12, pinned by tests/golden).
//
// Canonical arithmetic (the HIP kernels reproduce every rounding step of it bit for bit)
// -------------------------------------------------------------------------------------
//   profile    p[c] = (sum_t X[t][c]) / n, sequential f32 adds; then p[c] / max_c p[c]
//   oti        score[k] = fmaf-chain_c p_q[c]*p_r[(c-k) mod 12]; argmax, first max wins
//   frame norm nx[a] = fmaf-chain_c X[a][c]^2                (own, unrotated bin order)
//   stacked    NX[s] = sum_{t<m} nx[(s+t)*tau], sequential f32 adds
//   gram       G[a][b] = fmaf-chain_c X[a][c]*Y[b][(c-k) mod 12]  (reference Y rotated by k)
//   dot        dot[i][j] = sum_{t<m} G[(i+t)tau][(j+t)tau], sequential f32 adds
//   distance   d2 = (NX[i] - 2*dot) + NY[j];  D = d2 > 0 ? sqrtf(d2) : 0
//   threshold  q = (float)(n-1)*kappa; lo = floor(q), hi = ceil(q)
//              thr = lo==hi ? s[lo] : s[lo]*(hi-q) + s[hi]*(q-lo)   (s = sorted row/col)
//   mask       C[i][j] = (D <= thr_row[i]) && (D <= thr_col[j])
//   Qmax/dmax  essentia recurrences in f32 (values are multiples of 0.5: exact)
//
// Build: oracle/Makefile (g++ -O3 -march=x86-64-v3 -ffp-contract=off -fopenmp).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

extern "C" {

int or_stacked_len(int n, int m, int tau) {
  // essentia stackChromaFrames: for (i = 0; i < n - m*tau; i += tau)
  const int inc = m * tau;
  if (n <= inc || tau <= 0) return 0;
  return (n - inc + tau - 1) / tau;
}

void or_track_profile(const float* X, int n, float* prof) {
  float s[12];
  for (int c = 0; c < 12; ++c) s[c] = 0.0f;
  for (int t = 0; t < n; ++t)
    for (int c = 0; c < 12; ++c) s[c] = s[c] + X[(size_t)t * 12 + c];
  const float fn = (float)n;
  for (int c = 0; c < 12; ++c) s[c] = s[c] / fn;
  float mx = s[0];
  for (int c = 1; c < 12; ++c)
    if (s[c] > mx) mx = s[c];
  for (int c = 0; c < 12; ++c) prof[c] = mx > 0.0f ? s[c] / mx : 0.0f;
}

int or_oti(const float* pq, const float* pr) {
  int best = 0;
  float bestv = 0.0f;
  for (int k = 0; k < 12; ++k) {
    float acc = 0.0f;
    for (int c = 0; c < 12; ++c) acc = fmaf(pq[c], pr[(c - k + 12) % 12], acc);
    if (k == 0 || acc > bestv) {
      bestv = acc;
      best = k;
    }
  }
  return best;
}

void or_frame_norms(const float* X, int n, float* nx) {
  for (int a = 0; a < n; ++a) {
    float acc = 0.0f;
    for (int c = 0; c < 12; ++c) acc = fmaf(X[(size_t)a * 12 + c], X[(size_t)a * 12 + c], acc);
    nx[a] = acc;
  }
}

void or_stacked_norms(const float* nx, int n, int m, int tau, float* NX) {
  const int S = or_stacked_len(n, m, tau);
  for (int s = 0; s < S; ++s) {
    float acc = 0.0f;
    for (int t = 0; t < m; ++t) acc = acc + nx[(size_t)(s + t) * tau];
    NX[s] = acc;
  }
}

// D (Mp x Np, row-major). Y is rotated by k (np.roll semantics on the chroma axis).
// Loops run across j so the compiler vectorises them; every element keeps the canonical
// sequential order (c for the Gram fma chain, t for the window sum).
void or_crp_dist(const float* X, int M, const float* Y, int N, int k, int m, int tau, float* D) {
  const int Mp = or_stacked_len(M, m, tau), Np = or_stacked_len(N, m, tau);
  if (Mp <= 0 || Np <= 0) return;
  std::vector<float> nx(M), ny(N), NX(Mp), NY(Np);
  or_frame_norms(X, M, nx.data());
  or_frame_norms(Y, N, ny.data());
  or_stacked_norms(nx.data(), M, m, tau, NX.data());
  or_stacked_norms(ny.data(), N, m, tau, NY.data());
  // G only at the (a, b) used: frames a*tau, b*tau of the stacked-frame grid.
  const int Ma = (Mp - 1 + m), Nb = (Np - 1 + m);
  std::vector<float> YT((size_t)12 * Nb), G((size_t)Ma * Nb), acc(Np);
  for (int jb = 0; jb < Nb; ++jb)
    for (int c = 0; c < 12; ++c) YT[(size_t)c * Nb + jb] = Y[(size_t)jb * tau * 12 + ((c - k + 12) % 12)];
  for (int ia = 0; ia < Ma; ++ia) {
    const float* x = X + (size_t)ia * tau * 12;
    float* g = G.data() + (size_t)ia * Nb;
    for (int jb = 0; jb < Nb; ++jb) g[jb] = 0.0f;
    for (int c = 0; c < 12; ++c) {
      const float xc = x[c];
      const float* yc = YT.data() + (size_t)c * Nb;
      for (int jb = 0; jb < Nb; ++jb) g[jb] = __builtin_fmaf(xc, yc[jb], g[jb]);
    }
  }
  for (int i = 0; i < Mp; ++i) {
    for (int j = 0; j < Np; ++j) acc[j] = 0.0f;
    for (int t = 0; t < m; ++t) {
      const float* g = G.data() + (size_t)(i + t) * Nb + t;
      for (int j = 0; j < Np; ++j) acc[j] = acc[j] + g[j];
    }
    float* d = D + (size_t)i * Np;
    const float nxi = NX[i];
    for (int j = 0; j < Np; ++j) {
      const float d2 = (nxi - 2.0f * acc[j]) + NY[j];
      d[j] = d2 > 0.0f ? sqrtf(d2) : 0.0f;
    }
  }
}

// essentia percentile (essentiamath.h), restated; s is the sorted line.
float or_percentile_sorted(const float* s, int n, float kappa) {
  const float q = (float)(n - 1) * kappa;
  const float lo = floorf(q), hi = ceilf(q);
  if (lo == hi) return s[(int)lo];
  const float a = s[(int)lo] * (hi - q);
  const float b = s[(int)hi] * (q - lo);
  return a + b;
}

// The same value without sorting the whole line: only the order statistics at floor(q) and
// ceil(q) enter the interpolation, so nth_element + the minimum above it give them exactly.
// literal = 1: essentia's d0 + d1 form with no integer-q case (an integer q gives 0).
static float pct_select(float* v, int n, float kappa, int literal) {
  const float q = (float)(n - 1) * kappa;
  const float lo = floorf(q), hi = ceilf(q);
  const int ilo = (int)lo, ihi = (int)hi;
  std::nth_element(v, v + ilo, v + n);
  const float slo = v[ilo];
  const float shi = (ihi == ilo) ? slo : *std::min_element(v + ilo + 1, v + n);
  if (lo == hi && !literal) return slo;
  const float a = slo * (hi - q);
  const float b = shi * (q - lo);
  return a + b;
}

static void crp_thresholds_impl(const float* D, int Mp, int Np, float kappa, int literal, float* thr_r,
                                float* thr_c) {
  std::vector<float> v(std::max(Mp, Np));
  for (int i = 0; i < Mp; ++i) {
    std::copy(D + (size_t)i * Np, D + (size_t)(i + 1) * Np, v.begin());
    thr_r[i] = pct_select(v.data(), Np, kappa, literal);
  }
  for (int j = 0; j < Np; ++j) {
    for (int i = 0; i < Mp; ++i) v[i] = D[(size_t)i * Np + j];
    thr_c[j] = pct_select(v.data(), Mp, kappa, literal);
  }
}

void or_crp_thresholds(const float* D, int Mp, int Np, float kappa, float* thr_r, float* thr_c) {
  crp_thresholds_impl(D, Mp, Np, kappa, 0, thr_r, thr_c);
}

void or_crp_mask(const float* D, int Mp, int Np, const float* thr_r, const float* thr_c, uint8_t* C) {
  for (int i = 0; i < Mp; ++i)
    for (int j = 0; j < Np; ++j) {
      const float d = D[(size_t)i * Np + j];
      C[(size_t)i * Np + j] = (uint8_t)((d <= thr_r[i]) && (d <= thr_c[j]));
    }
}

// essentia CoverSongSimilarity, alignmentType 'serra09' (which=0) or 'chen17' (which=1),
// distanceType 'symmetric' -> max of the score matrix. Loops start at 2; rows/cols 0,1 = 0.
float or_align(const uint8_t* C, int M, int N, float g_open, float g_ext, int which) {
  if (M <= 0 || N <= 0) return 0.0f;
  std::vector<float> q0(N, 0.0f), q1(N, 0.0f), q2(N, 0.0f);  // rows i, i-1, i-2
  float best = 0.0f;
  auto g = [&](uint8_t c) { return c ? g_open : g_ext; };
  for (int i = 2; i < M; ++i) {
    std::fill(q0.begin(), q0.end(), 0.0f);
    const uint8_t* c0 = C + (size_t)i * N;
    const uint8_t* c1 = C + (size_t)(i - 1) * N;
    const uint8_t* c2 = C + (size_t)(i - 2) * N;
    for (int j = 2; j < N; ++j) {
      float a = q1[j - 1], b = q2[j - 1], c = q1[j - 2];
      if (which == 1) {
        b = b + (float)c1[j];
        c = c + (float)c0[j - 1];
      }
      float v;
      if (c0[j]) {
        v = std::max(std::max(a, b), c) + 1.0f;
      } else {
        const float x = a - g(c1[j - 1]);
        const float y = b - g(c2[j - 1]);
        const float z = c - g(c1[j - 2]);
        v = std::max(std::max(0.0f, x), std::max(y, z));
      }
      q0[j] = v;
      if (v > best) best = v;
    }
    std::swap(q2, q1);
    std::swap(q1, q0);
  }
  return best;
}

// One pair of the Serra09/Chen path. X: query (M x 12), Y: reference (N x 12).
// mask_out (Mp x Np) and thr outputs optional (may be NULL). Returns 0 or -1 (too short).
int or_crp_pair(const float* X, int M, const float* Y, int N, int m, int tau, float kappa, int use_oti,
                float g_open, float g_ext, float* qmax, float* dmax, int* oti_out, uint8_t* mask_out,
                float* thr_r_out, float* thr_c_out) {
  const int Mp = or_stacked_len(M, m, tau), Np = or_stacked_len(N, m, tau);
  if (Mp <= 0 || Np <= 0) return -1;
  int k = 0;
  if (use_oti) {
    float pq[12], pr[12];
    or_track_profile(X, M, pq);
    or_track_profile(Y, N, pr);
    k = or_oti(pq, pr);
  }
  if (oti_out) *oti_out = k;
  std::vector<float> D((size_t)Mp * Np), tr(Mp), tc(Np);
  std::vector<uint8_t> C((size_t)Mp * Np);
  or_crp_dist(X, M, Y, N, k, m, tau, D.data());
  or_crp_thresholds(D.data(), Mp, Np, kappa, tr.data(), tc.data());
  or_crp_mask(D.data(), Mp, Np, tr.data(), tc.data(), C.data());
  if (mask_out) std::memcpy(mask_out, C.data(), C.size());
  if (thr_r_out) std::memcpy(thr_r_out, tr.data(), Mp * sizeof(float));
  if (thr_c_out) std::memcpy(thr_c_out, tc.data(), Np * sizeof(float));
  if (qmax) *qmax = or_align(C.data(), Mp, Np, g_open, g_ext, 0);
  if (dmax) *dmax = or_align(C.data(), Mp, Np, g_open, g_ext, 1);
  return 0;
}

// Batch driver over (query, reference) index pairs into a packed feature block
// (sum of n_t x 12 float32, row offsets off[t]). Uses `nthreads` OpenMP threads.
int or_crp_batch(const float* feats, const int64_t* off, const int32_t* len, const int32_t* pairs, int64_t n_pairs,
                 int m, int tau, float kappa, int use_oti, float g_open, float g_ext, float* qmax, float* dmax,
                 int32_t* oti, int nthreads) {
  int err = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
  for (int64_t p = 0; p < n_pairs; ++p) {
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    int k = 0;
    float qv = 0.0f, dv = 0.0f;
    const int rc = or_crp_pair(feats + off[a] * 12, len[a], feats + off[b] * 12, len[b], m, tau, kappa, use_oti,
                               g_open, g_ext, &qv, dmax ? &dv : nullptr, &k, nullptr, nullptr, nullptr);
    if (rc) err |= 1;
    if (qmax) qmax[p] = qv;
    if (dmax) dmax[p] = dv;
    if (oti) oti[p] = k;
  }
  return err ? -1 : 0;
}

// ------------------------------------------------------------------------------------------
// essentia-order restatement (comparison mode; NOT what the HIP kernels reproduce).
//
// essentia ChromaCrossSimilarity::compute [ext, essentia 2.1-beta6-dev, unpinned] as its
// published source reads, restated literally rather than in the canonical decomposed order:
//   globalAverageChroma = sumFrames (sequential f32 adds per bin) [mean variant: / nframes],
//                         then normalize() (each bin / max bin)
//   optimalTranspositionIndex: for i = 0..noti(12): rotate the reference profile right by
//                         one (std::rotate, i > 0), dotProduct(query, reference); argmax
//                         (first maximum)
//   rotateChroma(reference, oti): every frame rotated right by oti (np.roll)
//   stackChromaFrames(m, tau): row s = frames s*tau .. s*tau + (m-1)*tau concatenated (m*12-d)
//   pairwiseDistance: item = dotProduct(a,a) - 2*dotProduct(a,b) + dotProduct(b,b);
//                     D = sqrt(item) (a negative item gives NaN: counted, see n_neg)
//   dotProduct = std::inner_product over the m*12 products. The accumulator is the open
//     question; `acc` selects it:
//       0  float accumulator, product rounded to float, then a separate add (init (T)0.0,
//          no contraction: a generic x86-64 build has no FMA)
//       1  double accumulator (init 0.0): float product, widened, added in double, the sum
//          rounded to float on return
//       2  float accumulator with the multiply-add contracted into fmaf (an -march=native
//          build with FMA and GCC's default -ffp-contract=fast)
//   percentile(line, 9.5): sort, k = (n-1)*0.095f, d0 + d1 interpolation; pct_literal = 1
//     drops the integer-k special case of the canonical restatement (d0 + d1 = 0 there)
//   binarize: C = (D <= thr_row) * (D <= thr_col); strict = 1 uses < (the other Heaviside)
// Nothing but tests/golden/make_essentia_bound.py and tests/ call this.
// ------------------------------------------------------------------------------------------
static inline float ess_dot(const float* a, const float* b, int n, int acc) {
  if (acc == 1) {
    double s = 0.0;
    for (int e = 0; e < n; ++e) {
      const float p = a[e] * b[e];
      s = s + (double)p;
    }
    return (float)s;
  }
  float s = 0.0f;
  if (acc == 2) {
    for (int e = 0; e < n; ++e) s = __builtin_fmaf(a[e], b[e], s);
  } else {
    for (int e = 0; e < n; ++e) {
      const float p = a[e] * b[e];
      s = s + p;
    }
  }
  return s;
}

void or_ess_profile(const float* X, int n, int mean, float* prof) {
  float s[12];
  for (int c = 0; c < 12; ++c) s[c] = 0.0f;
  for (int c = 0; c < 12; ++c)
    for (int t = 0; t < n; ++t) s[c] = s[c] + X[(size_t)t * 12 + c];
  if (mean)
    for (int c = 0; c < 12; ++c) s[c] = s[c] / (float)n;
  float mx = s[0];
  for (int c = 1; c < 12; ++c)
    if (s[c] > mx) mx = s[c];
  for (int c = 0; c < 12; ++c) prof[c] = mx != 0.0f ? s[c] / mx : s[c];
}

int or_ess_oti(const float* pq, const float* pr, int acc) {
  float r[12];
  for (int c = 0; c < 12; ++c) r[c] = pr[c];
  int best = 0;
  float bestv = 0.0f;
  for (int i = 0; i <= 12; ++i) {
    if (i > 0) {  // std::rotate(begin, end - 1, end): right by one
      const float last = r[11];
      for (int c = 11; c > 0; --c) r[c] = r[c - 1];
      r[0] = last;
    }
    const float v = ess_dot(pq, r, 12, acc);
    if (i == 0 || v > bestv) {
      bestv = v;
      best = i;
    }
  }
  return best % 12;
}

// Literal pairwiseDistance over stacked vectors. Vectorised across j; each element keeps
// the sequential inner_product order over e = t*12 + c. Returns the count of negative items.
int64_t or_ess_dist(const float* X, int M, const float* Y, int N, int k, int m, int tau, int acc, float* D) {
  const int Mp = or_stacked_len(M, m, tau), Np = or_stacked_len(N, m, tau);
  if (Mp <= 0 || Np <= 0) return 0;
  const int E = m * 12;
  std::vector<float> XS((size_t)Mp * E), YST((size_t)E * Np), a(Mp), cc(Np), ys(E);
  for (int s = 0; s < Mp; ++s)
    for (int t = 0; t < m; ++t)
      for (int c = 0; c < 12; ++c) XS[(size_t)s * E + t * 12 + c] = X[(size_t)(s * tau + t * tau) * 12 + c];
  for (int s = 0; s < Np; ++s) {
    for (int t = 0; t < m; ++t)
      for (int c = 0; c < 12; ++c) ys[t * 12 + c] = Y[(size_t)(s * tau + t * tau) * 12 + ((c - k + 12) % 12)];
    for (int e = 0; e < E; ++e) YST[(size_t)e * Np + s] = ys[e];
    cc[s] = ess_dot(ys.data(), ys.data(), E, acc);
  }
  for (int s = 0; s < Mp; ++s) a[s] = ess_dot(&XS[(size_t)s * E], &XS[(size_t)s * E], E, acc);
  int64_t neg = 0;
  std::vector<float> bf(Np);
  std::vector<double> bd(acc == 1 ? Np : 0);
  for (int i = 0; i < Mp; ++i) {
    const float* x = &XS[(size_t)i * E];
    if (acc == 1) {
      for (int j = 0; j < Np; ++j) bd[j] = 0.0;
      for (int e = 0; e < E; ++e) {
        const float xe = x[e];
        const float* y = &YST[(size_t)e * Np];
        for (int j = 0; j < Np; ++j) {
          const float p = xe * y[j];
          bd[j] = bd[j] + (double)p;
        }
      }
      for (int j = 0; j < Np; ++j) bf[j] = (float)bd[j];
    } else {
      for (int j = 0; j < Np; ++j) bf[j] = 0.0f;
      for (int e = 0; e < E; ++e) {
        const float xe = x[e];
        const float* y = &YST[(size_t)e * Np];
        if (acc == 2) {
          for (int j = 0; j < Np; ++j) bf[j] = __builtin_fmaf(xe, y[j], bf[j]);
        } else {
          for (int j = 0; j < Np; ++j) {
            const float p = xe * y[j];
            bf[j] = bf[j] + p;
          }
        }
      }
    }
    float* d = D + (size_t)i * Np;
    for (int j = 0; j < Np; ++j) {
      const float item = (a[i] - 2.0f * bf[j]) + cc[j];
      if (item < 0.0f) ++neg;
      d[j] = sqrtf(item);
    }
  }
  return neg;
}

// One pair in both modes. Per-pair outputs (index p):
//   st[8*p + 0..7] = cells, mask bits that differ, cells whose D differs, negative items,
//                    essentia cells equal to a threshold (where strict vs <= matters),
//                    rows + columns whose threshold differs, CRP ones canonical, CRP ones essentia
//   qc/qe = canonical / essentia Qmax; oc/oe = the two OTI indices.
int or_ess_compare_batch(const float* feats, const int64_t* off, const int32_t* len, const int32_t* pairs,
                         int64_t n_pairs, int m, int tau, float kappa, int acc, int prof_mean, int strict,
                         int pct_literal, float g_open, float g_ext, int64_t* st, float* qc, float* qe,
                         int32_t* oc, int32_t* oe, int nthreads) {
  int err = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
  for (int64_t p = 0; p < n_pairs; ++p) {
    const int ia = pairs[2 * p], ib = pairs[2 * p + 1];
    const float* X = feats + off[ia] * 12;
    const float* Y = feats + off[ib] * 12;
    const int M = len[ia], N = len[ib];
    const int Mp = or_stacked_len(M, m, tau), Np = or_stacked_len(N, m, tau);
    int64_t* s = st + 8 * p;
    for (int u = 0; u < 8; ++u) s[u] = 0;
    if (Mp <= 0 || Np <= 0) {
      err |= 1;
      continue;
    }
    float pq[12], pr[12];
    or_track_profile(X, M, pq);
    or_track_profile(Y, N, pr);
    const int kc = or_oti(pq, pr);
    or_ess_profile(X, M, prof_mean, pq);
    or_ess_profile(Y, N, prof_mean, pr);
    const int ke = or_ess_oti(pq, pr, acc);
    oc[p] = kc;
    oe[p] = ke;
    const size_t cells = (size_t)Mp * Np;
    std::vector<float> Dc(cells), De(cells), trc(Mp), tcc(Np), tre(Mp), tce(Np);
    std::vector<uint8_t> Cc(cells), Ce(cells);
    or_crp_dist(X, M, Y, N, kc, m, tau, Dc.data());
    const int64_t neg = or_ess_dist(X, M, Y, N, ke, m, tau, acc, De.data());
    crp_thresholds_impl(Dc.data(), Mp, Np, kappa, 0, trc.data(), tcc.data());
    crp_thresholds_impl(De.data(), Mp, Np, kappa, pct_literal, tre.data(), tce.data());
    or_crp_mask(Dc.data(), Mp, Np, trc.data(), tcc.data(), Cc.data());
    int64_t flips = 0, ddiff = 0, eq = 0, onc = 0, one = 0;
    for (int i = 0; i < Mp; ++i)
      for (int j = 0; j < Np; ++j) {
        const size_t t = (size_t)i * Np + j;
        const float d = De[t];
        const bool r = strict ? (d < tre[i]) : (d <= tre[i]);
        const bool c = strict ? (d < tce[j]) : (d <= tce[j]);
        Ce[t] = (uint8_t)(r && c);
        eq += (d == tre[i]) || (d == tce[j]);
        flips += Ce[t] != Cc[t];
        ddiff += De[t] != Dc[t];
        onc += Cc[t];
        one += Ce[t];
      }
    int64_t thr_diff = 0;
    for (int i = 0; i < Mp; ++i) thr_diff += trc[i] != tre[i];
    for (int j = 0; j < Np; ++j) thr_diff += tcc[j] != tce[j];
    s[0] = (int64_t)cells;
    s[1] = flips;
    s[2] = ddiff;
    s[3] = neg;
    s[4] = eq;
    s[5] = thr_diff;
    s[6] = onc;
    s[7] = one;
    qc[p] = or_align(Cc.data(), Mp, Np, g_open, g_ext, 0);
    qe[p] = or_align(Ce.data(), Mp, Np, g_open, g_ext, 0);
  }
  return err ? -1 : 0;
}

// acoss smith_waterman_constrained (alignment_tools.py:25-46), float64, same evaluation
// order as the Python: d = (S + match) + delta, S = max([d1, d2, d3, 0.0]).
// Returns -1.0 on a non-binary element (the reference raises IOError, :22-23).
double or_sw_constrained(const uint8_t* B, int M, int N) {
  double best = 0.0;
  if (M < 4 || N < 4) return best;
  for (size_t t = 0; t < (size_t)M * N; ++t)
    if (B[t] > 1) return -1.0;
  std::vector<double> S((size_t)M * N, 0.0);
  auto at = [&](int i, int j) { return B[(size_t)i * N + j]; };
  for (int i = 3; i < M; ++i)
    for (int j = 3; j < N; ++j) {
      const double mv = at(i - 1, j - 1) ? 1.0 : -1.0;
      const double d1 = (S[(size_t)(i - 1) * N + (j - 1)] + mv) + (at(i - 2, j - 2) > 0 ? 0.0 : -0.7);
      const double d2 = (S[(size_t)(i - 2) * N + (j - 1)] + mv) + (at(i - 3, j - 2) > 0 ? 0.0 : -0.7);
      const double d3 = (S[(size_t)(i - 1) * N + (j - 2)] + mv) + (at(i - 2, j - 3) > 0 ? 0.0 : -0.7);
      double v = d1;
      if (d2 > v) v = d2;
      if (d3 > v) v = d3;
      if (0.0 > v) v = 0.0;
      S[(size_t)i * N + j] = v;
      if (v > best) best = v;
    }
  return best;
}

// acoss Simple.simple_sim (simple_silva.py:68-118): median over i of
// min_j ||A[:, i:i+L] - Brot[:, j:j+L]||^2 computed as sa + sb - 2 QT (float64), where Brot is
// the reference rolled by k on the chroma axis (Simple.oti, :45-54). Canonical order (shared
// with simple.hip): the frame dot <A[:, x], Brot[:, y]> runs over the reference's OWN bins
// j = 0..11 paired with the query's bin (j + k) mod 12 -- the product for j = 0, then an fma
// chain; frame norms likewise over bins 0..11 (a roll does not change them); window sums are
// sequential adds.
double or_simple_sim(const double* A, int na, const double* B, int nb, int k, int L) {
  const int P = na - L + 1, Q = nb - L + 1;
  if (P <= 0 || Q <= 0) return NAN;
  k = ((k % 12) + 12) % 12;
  std::vector<double> ga((size_t)na * nb);
  for (int x = 0; x < na; ++x)
    for (int y = 0; y < nb; ++y) {
      double acc = A[(size_t)(k % 12) * na + x] * B[y];
      for (int d = 1; d < 12; ++d) acc = std::fma(A[(size_t)((d + k) % 12) * na + x], B[(size_t)d * nb + y], acc);
      ga[(size_t)x * nb + y] = acc;
    }
  std::vector<double> na2(na), nb2(nb), sa(P), sb(Q), mp(P);
  for (int x = 0; x < na; ++x) {
    double acc = A[x] * A[x];
    for (int d = 1; d < 12; ++d) acc = std::fma(A[(size_t)d * na + x], A[(size_t)d * na + x], acc);
    na2[x] = acc;
  }
  for (int y = 0; y < nb; ++y) {
    double acc = B[y] * B[y];
    for (int d = 1; d < 12; ++d) acc = std::fma(B[(size_t)d * nb + y], B[(size_t)d * nb + y], acc);
    nb2[y] = acc;
  }
  for (int i = 0; i < P; ++i) {
    double acc = 0.0;
    for (int t = 0; t < L; ++t) acc += na2[i + t];
    sa[i] = acc;
  }
  for (int j = 0; j < Q; ++j) {
    double acc = 0.0;
    for (int t = 0; t < L; ++t) acc += nb2[j + t];
    sb[j] = acc;
  }
  for (int i = 0; i < P; ++i) {
    double mn = INFINITY;
    for (int j = 0; j < Q; ++j) {
      double qt = 0.0;
      for (int t = 0; t < L; ++t) qt += ga[(size_t)(i + t) * nb + (j + t)];
      const double dist = (sb[j] + sa[i]) - 2.0 * qt;
      if (dist < mn) mn = dist;
    }
    mp[i] = mn;
  }
  std::sort(mp.begin(), mp.end());
  return (P % 2) ? mp[P / 2] : 0.5 * (mp[P / 2 - 1] + mp[P / 2]);
}

// Simple.oti (acoss/algorithms/simple_silva.py:45-54): profiles are per-bin sums over time
// (sequential), v[k] = <p_a, roll(p_b, k)> (sequential), k* = argsort(v)[-1]: numpy's
// small-array sort is stable, so among equal maxima the last index wins.
int or_simple_oti(const double* A, int na, const double* B, int nb) {
  double pa[12], pb[12];
  for (int c = 0; c < 12; ++c) {
    double x = 0.0, y = 0.0;
    for (int t = 0; t < na; ++t) x += A[(size_t)c * na + t];
    for (int t = 0; t < nb; ++t) y += B[(size_t)c * nb + t];
    pa[c] = x;
    pb[c] = y;
  }
  int best = 0;
  double bv = 0.0;
  for (int k = 0; k < 12; ++k) {
    double acc = 0.0;
    for (int c = 0; c < 12; ++c) acc += pa[c] * pb[(c - k + 12) % 12];
    if (k == 0 || acc >= bv) {
      bv = acc;
      best = k;
    }
  }
  return best;
}

// SiMPle over a batch of ordered pairs of packed (12 x n_t) float64 blocks (element offsets),
// with the Simple.oti roll: the CPU baseline of bench.py's SiMPle line. OpenMP over pairs.
int or_simple_batch(const double* feats, const int64_t* off, const int32_t* len, const int32_t* pairs,
                    int64_t n_pairs, int L, double* score, int32_t* oti, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t p = 0; p < n_pairs; ++p) {
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    const int k = or_simple_oti(feats + off[a], len[a], feats + off[b], len[b]);
    if (oti) oti[p] = k;
    score[p] = or_simple_sim(feats + off[a], len[a], feats + off[b], len[b], k, L);
  }
  return 0;
}

}  // extern "C"
