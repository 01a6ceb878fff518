// Probe: the rounding of v_mfma_f32_32x32x2f32 / v_mfma_f32_16x16x4f32 accumulation steps,
// compared bit for bit with CPU emulations (sequential fmaf chains, exact sum + one rounding).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <random>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// one 32x32 tile per wave, K = 2 per MFMA, NK steps: A[t][i][k], B[t][k][j] for t < NK
__global__ void k32(const float* A, const float* B, const float* C, float* D, int NK) {
  const int l = threadIdx.x;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) {
    const int i = (r / 4) * 8 + (l / 32) * 4 + (r % 4), j = l % 32;
    acc[r] = C[i * 32 + j];
  }
  for (int t = 0; t < NK; ++t) {
    const float a = A[t * 64 + (l % 32) * 2 + (l / 32)];   // A[t][i=l%32][k=l/32]
    const float b = B[t * 64 + (l / 32) * 32 + (l % 32)];  // B[t][k=l/32][j=l%32]
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) {
    const int i = (r / 4) * 8 + (l / 32) * 4 + (r % 4), j = l % 32;
    D[i * 32 + j] = acc[r];
  }
}
// 16x16 tile, K = 4 per MFMA: lane l holds A[i=l%16][k=l/16], B[k=l/16][j=l%16]; D: 4 per lane, i = 4*(l/16)+r, j = l%16
__global__ void k16(const float* A, const float* B, const float* C, float* D, int NK) {
  const int l = threadIdx.x;
  f32x4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C[(4 * (l / 16) + r) * 16 + (l % 16)];
  for (int t = 0; t < NK; ++t) {
    const float a = A[t * 64 + (l % 16) * 4 + (l / 16)];
    const float b = B[t * 64 + (l / 16) * 16 + (l % 16)];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + (l % 16)] = acc[r];
}

static float rnd(std::mt19937& g, int mode) {
  std::uniform_real_distribution<float> u(0.f, 1.f);
  float x = u(g);
  if (mode == 1) x = std::ldexp(x, (int)(g() % 40) - 20);
  if (mode == 2 && g() % 3 == 0) x = -x;
  if (mode == 3 && g() % 8 == 0) x = 0.f;
  if (mode == 4) x = std::ldexp(x, -(int)(g() % 20) - 55);  // products near / below FLT_MIN
  if (mode == 5 && g() % 2) x = std::ldexp(x, -130);       // denormal inputs
  return x;
}

int main() {
  const int NK = 6, TILES = 6000;
  std::mt19937 g(12345);
  long tot = 0, m_chain = 0, m_rchain = 0, m_exact = 0, m_pair = 0;
  long t16 = 0, m16_chain = 0, m16_exact = 0, m16_pairs = 0;
  float *dA, *dB, *dC, *dD;
  hipMalloc(&dA, NK * 64 * 4); hipMalloc(&dB, NK * 64 * 4); hipMalloc(&dC, 1024 * 4); hipMalloc(&dD, 1024 * 4);
  float A[NK * 64], B[NK * 64], C[1024], D[1024];
  for (int tile = 0; tile < TILES; ++tile) {
    const int mode = (tile / 2) % 6;
    for (int e = 0; e < NK * 64; ++e) { A[e] = rnd(g, mode); B[e] = rnd(g, mode); }
    for (int e = 0; e < 1024; ++e) C[e] = (tile % 2) ? 0.f : rnd(g, mode);
    hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, sizeof C, hipMemcpyHostToDevice);
    if (tile % 2 == 0) {
      hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, NK);
      hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
      for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
        float c1 = C[i * 32 + j], c2 = c1, c3 = c1, c4 = c1;
        for (int t = 0; t < NK; ++t) {
          const float a0 = A[t * 64 + i * 2], a1 = A[t * 64 + i * 2 + 1];
          const float b0 = B[t * 64 + j], b1 = B[t * 64 + 32 + j];
          c1 = fmaf(a1, b1, fmaf(a0, b0, c1));
          c2 = fmaf(a0, b0, fmaf(a1, b1, c2));
          c3 = (float)((__float128)c3 + (__float128)a0 * b0 + (__float128)a1 * b1);
          c4 = c4 + (float)((double)a0 * b0 + (double)a1 * b1);
        }
        const float d = D[i * 32 + j];
        ++tot; m_chain += !memcmp(&d, &c1, 4); m_rchain += !memcmp(&d, &c2, 4); m_exact += !memcmp(&d, &c3, 4);
        m_pair += !memcmp(&d, &c4, 4);
      }
    } else {
      hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, NK);
      hipMemcpy(D, dD, 256 * 4, hipMemcpyDeviceToHost);
      for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
        float c1 = C[i * 16 + j], c3 = c1, c4 = c1;
        for (int t = 0; t < NK; ++t) {
          __float128 s = c3;
          float cc = c1;
          double pp = 0;
          for (int k = 0; k < 4; ++k) {
            const float a = A[t * 64 + i * 4 + k], b = B[t * 64 + k * 16 + j];
            cc = fmaf(a, b, cc); s += (__float128)a * b; pp += (double)a * b;
          }
          c1 = cc; c3 = (float)s; c4 = c4 + (float)pp;
        }
        const float d = D[i * 16 + j];
        ++t16; m16_chain += !memcmp(&d, &c1, 4); m16_exact += !memcmp(&d, &c3, 4); m16_pairs += !memcmp(&d, &c4, 4);
      }
    }
  }
  printf("32x32x2: n=%ld  fma_chain(k0,k1)=%ld  fma_chain(k1,k0)=%ld  exact_sum_one_round=%ld  c+round(p0+p1)=%ld\n", tot,
         m_chain, m_rchain, m_exact, m_pair);
  printf("16x16x4: n=%ld  fma_chain=%ld  exact_sum_one_round=%ld  c+round(sum p)=%ld\n", t16, m16_chain, m16_exact, m16_pairs);
  return 0;
}
