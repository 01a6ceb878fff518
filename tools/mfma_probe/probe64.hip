// Probe: does v_mfma_f64_16x16x4_f64 accumulate exactly as the sequential fma chain in k order?
// (the SiMPle frame dot's canonical order is the bin-0 product, then an f64
// fma chain over bins 1..11 -- simple.hip / oracle or_simple_sim.) Compared bit for bit with CPU
// emulations: the sequential fma chain, the exact 4-term sum rounded once, and a pairwise order.
//   hipcc --offload-arch=gfx950 -O2 -o probe64 tools/mfma_probe/probe64.hip && ./probe64
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
typedef double f64x4 __attribute__((ext_vector_type(4)));

// one 16x16 tile per wave, K = 4 per MFMA, NK steps. Operand layout (as the f32 16x16x4):
// lane l holds A[t][i = l % 16][k = l / 16] and B[t][k = l / 16][j = l % 16]. Output: 4 doubles per
// lane, acc[r] = D[i = l / 16 + 4 r][j = l % 16] (found by layout64.hip: unique integer products).
__global__ void k16(const double* A, const double* B, const double* C, double* D, int NK, int layout) {
  const int l = threadIdx.x;
  f64x4 acc;
  for (int r = 0; r < 4; ++r) {
    const int i = (l / 16) + 4 * r, j = l % 16;  // measured (tools/mfma_probe/layout64.hip)
    acc[r] = C[i * 16 + j];
  }
  for (int t = 0; t < NK; ++t) {
    const double a = A[t * 64 + (l % 16) * 4 + (l / 16)];
    const double b = B[t * 64 + (l / 16) * 16 + (l % 16)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) {
    const int i = (l / 16) + 4 * r, j = l % 16;  // measured (tools/mfma_probe/layout64.hip)
    D[i * 16 + j] = acc[r];
  }
}

static double rnd(std::mt19937_64& g, int mode) {
  std::uniform_real_distribution<double> u(0.0, 1.0);
  double x = u(g);
  if (mode == 1) x = std::ldexp(x, (int)(g() % 80) - 40);
  if (mode == 2 && g() % 3 == 0) x = -x;
  if (mode == 3 && g() % 8 == 0) x = 0.0;
  if (mode == 4) x = std::ldexp(x, -(int)(g() % 40) - 500);  // products near / below DBL_MIN
  if (mode == 5 && g() % 2) x = std::ldexp(x, -1030);         // denormal inputs
  if (mode == 6) x = std::ldexp(x, (int)(g() % 8) - 4) * ((g() & 1) ? 1.0 : -1.0);  // cancellation
  if (mode == 7) x = (double)(g() % 9) - 4.0;  // small integers: every order exact (checks the layout)
  return x;
}

// exact sum of c + sum a_k b_k rounded once (long double has 64 mantissa bits: not exact in general,
// so this is only reported; the chain comparison is the decisive one)
int main() {
  const int NK = 3, TILES = 4000;  // K = 12: one SiMPle frame dot per output
  std::mt19937_64 g(20250101);
  double *dA, *dB, *dC, *dD;
  hipMalloc(&dA, NK * 64 * 8);
  hipMalloc(&dB, NK * 64 * 8);
  hipMalloc(&dC, 256 * 8);
  hipMalloc(&dD, 256 * 8);
  double A[NK * 64], B[NK * 64], C[256], D[256];
  for (int layout = 0; layout < 1; ++layout) {
    long tot = 0, m_chain = 0, m_chain0 = 0, m_pair = 0, m_fused = 0, m_rev = 0, tot_int = 0, m_int = 0;
    for (int tile = 0; tile < TILES; ++tile) {
      const int mode = tile % 8;
      for (int e = 0; e < NK * 64; ++e) {
        A[e] = rnd(g, mode);
        B[e] = rnd(g, mode);
      }
      const bool zeroc = tile % 2 == 0;  // SiMPle starts every dot from +0
      for (int e = 0; e < 256; ++e) C[e] = zeroc ? 0.0 : rnd(g, mode);
      hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice);
      hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
      hipMemcpy(dC, C, sizeof C, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, NK, layout);
      hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double chain = C[i * 16 + j], pair = C[i * 16 + j], fused = C[i * 16 + j], rev = C[i * 16 + j];
          for (int t = 0; t < NK; ++t) {
            // one rounding per MFMA: c + sum of the 4 exact products, rounded once (__float128: 113 bits)
            __float128 e = (__float128)fused;
            for (int k = 0; k < 4; ++k) e += (__float128)A[t * 64 + i * 4 + k] * (__float128)B[t * 64 + k * 16 + j];
            fused = (double)e;
            for (int k = 3; k >= 0; --k) rev = std::fma(A[t * 64 + i * 4 + k], B[t * 64 + k * 16 + j], rev);
            double s0 = 0.0;
            for (int k = 0; k < 4; ++k) chain = std::fma(A[t * 64 + i * 4 + k], B[t * 64 + k * 16 + j], chain);
            // pairwise: (a0b0 + a1b1) + (a2b2 + a3b3), then + c
            const double p0 = A[t * 64 + i * 4 + 0] * B[t * 64 + 0 * 16 + j] + A[t * 64 + i * 4 + 1] * B[t * 64 + 1 * 16 + j];
            const double p1 = A[t * 64 + i * 4 + 2] * B[t * 64 + 2 * 16 + j] + A[t * 64 + i * 4 + 3] * B[t * 64 + 3 * 16 + j];
            pair = pair + (p0 + p1);
            (void)s0;
          }
          // the canonical SiMPle order when c = 0: the first product rounded, then fma
          double chain0 = 0.0;
          bool first = true;
          for (int t = 0; t < NK; ++t)
            for (int k = 0; k < 4; ++k) {
              const double a = A[t * 64 + i * 4 + k], b = B[t * 64 + k * 16 + j];
              chain0 = first && zeroc ? a * b : std::fma(a, b, first ? C[i * 16 + j] : chain0);
              first = false;
            }
          const double d = D[i * 16 + j];
          ++tot;
          m_chain += memcmp(&d, &chain, 8) == 0;
          m_chain0 += memcmp(&d, &chain0, 8) == 0;
          m_pair += memcmp(&d, &pair, 8) == 0;
          m_fused += memcmp(&d, &fused, 8) == 0;
          m_rev += memcmp(&d, &rev, 8) == 0;
          if (mode == 7) {
            ++tot_int;
            m_int += memcmp(&d, &chain, 8) == 0;
          }
        }
    }
    printf("layout %d: %ld outputs; == sequential fma chain: %ld; == canonical (product, then fma): %ld; "
           "== pairwise sums: %ld; == one rounding per MFMA: %ld; == reversed fma chain: %ld; small integers %ld of %ld\n",
           layout, tot, m_chain, m_chain0, m_pair, m_fused, m_rev, m_int, tot_int);
  }
  return 0;
}
