#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* Draw) {
  const int l = threadIdx.x;
  f64x4 acc = {0, 0, 0, 0};
  const double a = A[(l % 16) * 4 + (l / 16)];
  const double b = B[(l / 16) * 16 + (l % 16)];
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) Draw[l * 4 + r] = acc[r];
}
int main() {
  std::mt19937 g(7);
  double A[64], B[64], D[256];
  for (int e = 0; e < 64; ++e) { A[e] = (double)(g() % 1000); B[e] = (double)(g() % 1000); }
  double *dA, *dB, *dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048);
  hipMemcpy(dA, A, 512, hipMemcpyHostToDevice); hipMemcpy(dB, B, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(D, dD, 2048, hipMemcpyDeviceToHost);
  int found = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      int hits = 0, hi = -1, hj = -1;
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double s = 0;
          for (int k = 0; k < 4; ++k) s += A[i * 4 + k] * B[k * 16 + j];
          if (s == D[l * 4 + r]) { ++hits; hi = i; hj = j; }
        }
      if (l < 20 || l % 16 == 0) printf("lane %d r %d -> %d hits, i %d j %d\n", l, r, hits, hi, hj);
      found += hits == 1;
    }
  printf("unique matches %d of 256\n", found);
  return 0;
}
