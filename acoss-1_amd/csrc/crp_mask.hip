// crp_mask.hip — the cross-recurrence plot (mutual-neighbour mask) of a batch of pairs,
// written as one 32-bit word per (32-row strip, column): the layout the DP kernel reads.
//
// Replaces the final binarisation of essentia ChromaCrossSimilarity (rqa_serra09.py:60-66):
// C[i][j] = H(thr_row[i] - D[i][j]) * H(thr_col[j] - D[i][j]), evaluated in the squared
// domain (key <= T) which is exactly equivalent (common.hpp sq_threshold).
//
// Fast path for frameStackSize m = 9. One 256-thread block per (32-row strip, pair) sweeps
// the reference in parallelogram panels; thread t walks one diagonal: at step k the 12-term
// fmaf chain of the query frame (wave-uniform, scalar loads) with the rolled reference frame
// (LDS, 3 ds_read_b128), the last 9 chain values kept in registers give the stacked distance
// of cell (k-8, j0+t+k-8). A set bit is OR-ed into a rolling LDS word buffer; complete
// columns are streamed out after each panel. Same rounding sequence as oracle/crp_oracle.cpp.
#include "crp_internal.hpp"

namespace acoss {

namespace {

constexpr int kR = 32;                     // rows per strip = bits per word
constexpr int kW = 256;                    // diagonals per panel
constexpr int kMS = 9;
constexpr int kYRows = kW + kR + kMS - 2;  // 295 reference frames per panel
constexpr int kCols = kW + kR - 1;         // 287 columns touched per panel

__device__ __forceinline__ void load_query(const float* base_ptr, int f, float (&x)[12]) {
  const float* base = base_ptr + (size_t)f * 12;
  asm volatile("" : "+s"(base));  // keep the scalar load in the loop (no hoisting of 40 rows)
  const cfloat4* p = (const cfloat4*)base;
  const f32x4 a = p[0], b = p[1], c = p[2];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w;
}

__global__ __launch_bounds__(256) void k_crp_mask9(CrpBatch B, const float* __restrict__ Trow,
                                                   const float* __restrict__ Tcol, int64_t thr_stride,
                                                   uint32_t* __restrict__ maskT, int64_t mask_stride, int ld) {
  __shared__ __attribute__((aligned(16))) float Ys[kYRows * 12];
  __shared__ float Tc[kCols + 1];
  __shared__ float Ns[kCols + 1];
  __shared__ uint32_t wb[kCols + 1];
  const int p = blockIdx.y;
  const int2 dm = B.dims[p];
  const int Mp = dm.x, Np = dm.y;
  const int strip = blockIdx.x;
  const int i0 = strip * kR;
  if (i0 >= Mp || Np <= 0) return;
  const int t = threadIdx.x;
  const int ta = B.pairs[2 * p], tb = B.pairs[2 * p + 1];
  const float* X = B.feats + B.off[ta] * 12;
  const float* Yr = B.yrot + (size_t)p * B.yrot_stride;
  const int nq = B.len[ta], nr = B.len[tb], tau = B.tau;
  const float* NXq = B.NX + (size_t)ta * B.ldn;
  const float* NXr = B.NX + (size_t)tb * B.ldn;
  const float* Tr = Trow + (size_t)p * thr_stride;
  const float* Tcp = Tcol + (size_t)p * thr_stride;
  const int rows = min(kR, Mp - i0);
  // per-row constants (wave-uniform): query stacked norm and squared-domain row threshold;
  // rows past the end get T = -1 (never set)
  float nq_r[kR], tr_r[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int i = min(i0 + r, Mp - 1);
    nq_r[r] = *(const __attribute__((address_space(4))) float*)(NXq + i);
    tr_r[r] = (r < rows) ? *(const __attribute__((address_space(4))) float*)(Tr + i) : -1.0f;
  }
  uint32_t* out = maskT + (size_t)p * mask_stride + (size_t)strip * ld;
  for (int e = t; e < kCols + 1; e += kW) wb[e] = 0u;
  for (int j0 = -(kR - 1); j0 < Np; j0 += kW) {
    __syncthreads();
    for (int e = t; e < kYRows * 3; e += kW) {
      const int b = e / 3, piece = e - b * 3;
      const int jr = j0 + b;
      const int f = jr * tau;
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
      if (jr >= 0 && f < nr) v = reinterpret_cast<const f32x4*>(Yr + (size_t)f * 12)[piece];
      reinterpret_cast<f32x4*>(Ys)[e] = v;
    }
    for (int b = t; b < kCols; b += kW) {
      const int jr = j0 + b;
      const bool ok = jr >= 0 && jr < Np;
      Tc[b] = ok ? Tcp[jr] : -1.0f;
      Ns[b] = ok ? NXr[jr] : 0.0f;
    }
    __syncthreads();
    float gw[kMS];
    float xb[2][12];
    f32x4 yb[2][3];
    load_query(X, min(i0 * tau, nq - 1), xb[0]);
    {
      const f32x4* yp = reinterpret_cast<const f32x4*>(Ys + t * 12);
      yb[0][0] = yp[0];
      yb[0][1] = yp[1];
      yb[0][2] = yp[2];
    }
#pragma unroll
    for (int kk = 0; kk < kR + kMS - 1; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if (kk + 1 < kR + kMS - 1) {
        load_query(X, min((i0 + kk + 1) * tau, nq - 1), xb[nxt]);
        const f32x4* yp = reinterpret_cast<const f32x4*>(Ys + (t + kk + 1) * 12);
        yb[nxt][0] = yp[0];
        yb[nxt][1] = yp[1];
        yb[nxt][2] = yp[2];
      }
      const float* x = xb[cur];
      const f32x4 ya = yb[cur][0], yb1 = yb[cur][1], yc = yb[cur][2];
      float g = 0.0f;
      g = __builtin_fmaf(x[0], ya.x, g);
      g = __builtin_fmaf(x[1], ya.y, g);
      g = __builtin_fmaf(x[2], ya.z, g);
      g = __builtin_fmaf(x[3], ya.w, g);
      g = __builtin_fmaf(x[4], yb1.x, g);
      g = __builtin_fmaf(x[5], yb1.y, g);
      g = __builtin_fmaf(x[6], yb1.z, g);
      g = __builtin_fmaf(x[7], yb1.w, g);
      g = __builtin_fmaf(x[8], yc.x, g);
      g = __builtin_fmaf(x[9], yc.y, g);
      g = __builtin_fmaf(x[10], yc.z, g);
      g = __builtin_fmaf(x[11], yc.w, g);
      gw[kk % kMS] = g;
      if (kk >= kMS - 1) {
        const int r = kk - (kMS - 1);
        float dot = 0.0f;
#pragma unroll
        for (int u = 0; u < kMS; ++u) dot = dot + gw[(r + u) % kMS];
        const float d2 = (nq_r[r] - 2.0f * dot) + Ns[t + r];  // (N_query - 2 dot) + N_reference
        const float key = d2 > 0.0f ? d2 : 0.0f;
        const bool bit = (key <= tr_r[r]) & (key <= Tc[t + r]);
        if (bit) atomicOr(&wb[t + r], 1u << r);
      }
    }
    __syncthreads();
    // columns [j0, j0 + 256) are complete: stream them out; keep the 31-column tail
    const int jj = j0 + t;
    const uint32_t w = wb[t];
    const uint32_t tail = (t < kR - 1) ? wb[kW + t] : 0u;
    __syncthreads();
    if (jj >= 0 && jj < Np) out[jj] = w;
    wb[t] = tail;
    if (t < kR) wb[kW + t] = 0u;
  }
}

}  // namespace

int launch_mask9(const CrpBatch& B, int nb, int L, const float* Trow, const float* Tcol, int64_t thr_stride,
                 uint32_t* maskT, int64_t mask_stride, int ld, hipStream_t s) {
  if (B.m != kMS) return 1;
  hipLaunchKernelGGL(k_crp_mask9, dim3((L + kR - 1) / kR, nb), dim3(kW), 0, s, B, Trow, Tcol, thr_stride, maskT,
                     mask_stride, ld);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

}  // namespace acoss
