// crp_split.hip — Serra09/Chen CRP in three kernels around ONE distance sweep (m = 9).
//
// Replaces, per pair, the body of essentia ChromaCrossSimilarity (rqa_serra09.py:60-66,
// latefusion_chen.py:63-69): stacked distances, percentile(row/column, 9.5) and the mutual
// binary mask, bit-identical to oracle/crp_oracle.cpp.
//
//  k_sweep9      one 256-thread block per (32-row strip, pair): diagonal walk (G in
//                registers, query frames by scalar loads, rolled reference frames in LDS);
//                the high 16 bits of every squared-distance key go to HBM twice: row-major
//                K16r[i][j] and column-major K16c[j][i] (through a rolling LDS tile).
//  k_sel_rows9   one wave per CRP row: 32 keys per lane in registers, the 16-bit prefixes of
//                the two order statistics by binary search with ballot counts (v_cmp +
//                s_bcnt1: no cross-lane reduction), the cells sharing a prefix recomputed
//                exactly (one per lane), rank inside the group -> percentile -> squared-domain
//                threshold T_row.
//  k_sel_cols9   one wave per CRP column: the same select gives T_col; lane l then holds rows
//                32l..32l+31 of the column, i.e. exactly one 32-bit CRP word, so the mask is
//                emitted here (key <= T_row && key <= T_col, decided on the 16-bit prefix;
//                cells whose prefix ties a threshold prefix are recomputed exactly).
#include <cstdlib>

#include "crp_internal.hpp"

namespace acoss {

namespace {

constexpr int kMS = 9;

struct PairView {
  const float* X;   // query frames
  const float* Yr;  // OTI-rolled reference frames
  int nq, nr, tau;
  const float* NXq;
  const float* NXr;
  int Mp, Np;
};

__device__ __forceinline__ PairView pair_view(const CrpBatch& B, int p) {
  PairView v;
  const int ta = B.pairs[2 * p], tb = B.pairs[2 * p + 1];
  v.X = B.feats + B.off[ta] * 12;
  v.Yr = B.yrot + (size_t)p * B.yrot_stride;
  v.nq = B.len[ta];
  v.nr = B.len[tb];
  v.tau = B.tau;
  v.NXq = B.NX + (size_t)ta * B.ldn;
  v.NXr = B.NX + (size_t)tb * B.ldn;
  const int2 dm = B.dims[p];
  v.Mp = dm.x;
  v.Np = dm.y;
  return v;
}

// ---------------------------------------------------------------------------------------
// k_sweep9
// ---------------------------------------------------------------------------------------
constexpr int kSR = 32;                       // rows per strip
constexpr int kSW = 256;                      // diagonals per panel
constexpr int kSYRows = kSW + kSR + kMS - 2;  // 295 reference frames per panel
constexpr int kSCols = kSW + kSR;             // 288 columns touched (+1 pad)

__device__ __forceinline__ void load_query(const float* base_ptr, int f, float (&x)[12]) {
  const float* base = base_ptr + (size_t)f * 12;
  asm volatile("" : "+s"(base));  // keep each row's scalar load inside the loop
  const cfloat4* p = (const cfloat4*)base;
  const f32x4 a = p[0], b = p[1], c = p[2];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w;
}

// Key planes of one pair: high / low 16 bits, row-major (line = CRP row) and column-major.
struct KeyPlanes {
  uint16_t* hr;
  uint16_t* lr;
  uint16_t* hc;
  uint16_t* lc;
};

__global__ __launch_bounds__(256) void k_sweep9(CrpBatch B, KeyPlanes K, int ldr, int ldc, int64_t kstride) {
  __shared__ __attribute__((aligned(16))) float Ys[kSYRows * 12];
  __shared__ float Ns[kSCols];
  __shared__ __attribute__((aligned(16))) uint32_t tile[kSR][kSCols + 4];  // rolling full-key tile
  const int p = blockIdx.y;
  const PairView V = pair_view(B, p);
  const int strip = blockIdx.x, i0 = strip * kSR;
  if (i0 >= V.Mp || V.Np <= 0) return;
  const int t = threadIdx.x;
  const int rows = min(kSR, V.Mp - i0);
  float nq_r[kSR];
#pragma unroll
  for (int r = 0; r < kSR; ++r) nq_r[r] = *(const __attribute__((address_space(4))) float*)(V.NXq + min(i0 + r, V.Mp - 1));
  uint16_t* Hr = K.hr + (size_t)p * kstride;
  uint16_t* Lr = K.lr + (size_t)p * kstride;
  uint16_t* Hc = K.hc + (size_t)p * kstride;
  uint16_t* Lc = K.lc + (size_t)p * kstride;
  for (int j0 = -(kSR - 1); j0 < V.Np; j0 += kSW) {
    __syncthreads();
    for (int e = t; e < kSYRows * 3; e += kSW) {
      const int b = e / 3, piece = e - b * 3;
      const int jr = j0 + b;
      const int f = jr * V.tau;
      f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
      if (jr >= 0 && f < V.nr) v = reinterpret_cast<const f32x4*>(V.Yr + (size_t)f * 12)[piece];
      reinterpret_cast<f32x4*>(Ys)[e] = v;
    }
    for (int b = t; b < kSCols; b += kSW) {
      const int jr = j0 + b;
      Ns[b] = (jr >= 0 && jr < V.Np) ? V.NXr[jr] : 0.0f;
    }
    __syncthreads();
    float gw[kMS];
    float xb[2][12];
    f32x4 yb[2][3];
    load_query(V.X, min(i0 * V.tau, V.nq - 1), xb[0]);
    {
      const f32x4* yp = reinterpret_cast<const f32x4*>(Ys + t * 12);
      yb[0][0] = yp[0];
      yb[0][1] = yp[1];
      yb[0][2] = yp[2];
    }
#pragma unroll
    for (int kk = 0; kk < kSR + kMS - 1; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if (kk + 1 < kSR + kMS - 1) {
        load_query(V.X, min((i0 + kk + 1) * V.tau, V.nq - 1), xb[nxt]);
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
        const float d2 = (nq_r[r] - 2.0f * dot) + Ns[t + r];
        const float key = d2 > 0.0f ? d2 : 0.0f;
        tile[r][t + r] = __builtin_bit_cast(unsigned, key);
      }
    }
    __syncthreads();
    // columns [j0, j0 + 256) complete: row-major (coalesced along j) and column-major (32
    // consecutive rows = 64 B per column and plane) stores
    const int jj = j0 + t;
    if (jj >= 0 && jj < V.Np) {
      for (int r = 0; r < rows; ++r) {
        const unsigned k = tile[r][t];
        Hr[(size_t)(i0 + r) * ldr + jj] = (uint16_t)(k >> 16);
        Lr[(size_t)(i0 + r) * ldr + jj] = (uint16_t)(k & 0xffffu);
      }
      unsigned col[kSR];
#pragma unroll
      for (int r = 0; r < kSR; ++r) col[r] = tile[r][t];
      uint4* dh = reinterpret_cast<uint4*>(Hc + (size_t)jj * ldc + i0);
      uint4* dl = reinterpret_cast<uint4*>(Lc + (size_t)jj * ldc + i0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint4 h, l;
        h.x = (col[8 * q] >> 16) | (col[8 * q + 1] & 0xffff0000u);
        h.y = (col[8 * q + 2] >> 16) | (col[8 * q + 3] & 0xffff0000u);
        h.z = (col[8 * q + 4] >> 16) | (col[8 * q + 5] & 0xffff0000u);
        h.w = (col[8 * q + 6] >> 16) | (col[8 * q + 7] & 0xffff0000u);
        l.x = (col[8 * q] & 0xffffu) | (col[8 * q + 1] << 16);
        l.y = (col[8 * q + 2] & 0xffffu) | (col[8 * q + 3] << 16);
        l.z = (col[8 * q + 4] & 0xffffu) | (col[8 * q + 5] << 16);
        l.w = (col[8 * q + 6] & 0xffffu) | (col[8 * q + 7] << 16);
        dh[q] = h;
        dl[q] = l;
      }
    }
    __syncthreads();
    // roll the 31-column tail to the front
    if (t < kSR - 1)
      for (int r = 0; r < kSR; ++r) tile[r][t] = tile[r][kSW + t];
  }
}

// ---------------------------------------------------------------------------------------
// Per-wave select on one line (CRP row or column) of 16-bit key prefixes.
// Lane l holds keys [l*KPL, (l+1)*KPL) (0xffffffff = no element).
// ---------------------------------------------------------------------------------------
template <int KPL>
struct Line {
  unsigned v[KPL];
  __device__ __forceinline__ void load(const uint16_t* src, int n) {
    const int lane = threadIdx.x & 63;
    const int base = lane * KPL;
    if (base + KPL <= n) {
#pragma unroll
      for (int q = 0; q < KPL / 8; ++q) {
        const uint4 w = reinterpret_cast<const uint4*>(src + base)[q];
        v[8 * q + 0] = w.x & 0xffffu;
        v[8 * q + 1] = w.x >> 16;
        v[8 * q + 2] = w.y & 0xffffu;
        v[8 * q + 3] = w.y >> 16;
        v[8 * q + 4] = w.z & 0xffffu;
        v[8 * q + 5] = w.z >> 16;
        v[8 * q + 6] = w.w & 0xffffu;
        v[8 * q + 7] = w.w >> 16;
      }
    } else {
#pragma unroll
      for (int q = 0; q < KPL; ++q) v[q] = (base + q < n) ? (unsigned)src[base + q] : 0xffffffffu;
    }
  }
  // #keys <= x (x <= 0xffff): ballot per slot, popcount on the scalar unit
  __device__ __forceinline__ int count_le(unsigned x) const {
    int c = 0;
#pragma unroll
    for (int q = 0; q < KPL; ++q) c += __popcll(__ballot(v[q] <= x));
    return c;
  }
  __device__ __forceinline__ void min_max(unsigned* mn, unsigned* mx) const {
    unsigned a = 0xffffu, b = 0u;
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const bool ok = v[q] != 0xffffffffu;
      a = ok ? min(a, v[q]) : a;
      b = ok ? max(b, v[q]) : b;
    }
    *mn = wave_min_u32(a);
    *mx = wave_max_u32(b);
  }
  __device__ __forceinline__ unsigned min_greater(unsigned x) const {
    unsigned a = 0xffffffffu;
#pragma unroll
    for (int q = 0; q < KPL; ++q) a = (v[q] > x) ? min(a, v[q]) : a;
    return wave_min_u32(a);
  }
};

// Smallest prefix P with count(keys <= P) > rho.
template <int KPL>
__device__ __forceinline__ unsigned prefix_of_rank(const Line<KPL>& L, int rho, unsigned a, unsigned b) {
  while (a < b) {
    const unsigned mid = (a + b) >> 1;
    if (L.count_le(mid) > rho)
      b = mid;
    else
      a = mid + 1;
  }
  return a;
}

// Exact key (32 bits) of rank rho among the g keys of the line whose prefix is P; the low
// halves come from the line's low plane `lo`. list = 64 ints of LDS owned by the wave.
template <int KPL>
__device__ unsigned exact_rank(const Line<KPL>& L, unsigned P, int rho, int g, const uint16_t* lo, int* list) {
  const int lane = threadIdx.x & 63;
  if (g <= 64) {
    int base = 0;
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const bool m = L.v[q] == P;
      const unsigned long long bal = __ballot(m);
      if (m)
        list[base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] =
            lane * KPL + q;
      base += __popcll(bal);
    }
    __builtin_amdgcn_wave_barrier();
    const bool act = lane < g;
    const unsigned key = act ? ((P << 16) | (unsigned)lo[list[lane]]) : 0xffffffffu;
    __builtin_amdgcn_wave_barrier();
    int cl = 0, ce = 0;
    for (int k = 0; k < g; ++k) {
      const unsigned o = (unsigned)lane_bcast((int)key, k);
      cl += o < key;
      ce += o == key;
    }
    const int src = __builtin_ctzll(__ballot(act && cl <= rho && rho < cl + ce));
    return (unsigned)lane_bcast((int)key, src);
  }
  // large groups (long silences): low halves of the whole line into registers, then a
  // binary search over the low 16 bits counting group members only
  unsigned lw[KPL];
  const int base = lane * KPL;
#pragma unroll
  for (int q = 0; q < KPL; ++q) lw[q] = (L.v[q] == P) ? (unsigned)lo[base + q] : 0x10000u;
  unsigned a = 0, b = 0xffffu;
  while (a < b) {
    const unsigned mid = (a + b) >> 1;
    int c = 0;
#pragma unroll
    for (int q = 0; q < KPL; ++q) c += __popcll(__ballot(lw[q] <= mid));
    if (c > rho)
      b = mid;
    else
      a = mid + 1;
  }
  return (P << 16) | a;
}

// Threshold (distance units) and squared-domain threshold of a line of n keys.
template <int KPL>
__device__ void line_threshold(const Line<KPL>& L, int n, float kappa, const uint16_t* lo_plane, int* list,
                               float* thr, float* T) {
  const float q = (float)(n - 1) * kappa;
  const float lo_f = floorf(q), hi_f = ceilf(q);
  const int lo = (int)lo_f, hi = (int)hi_f;
  unsigned kmin, kmax;
  L.min_max(&kmin, &kmax);
  const unsigned Pl = prefix_of_rank(L, lo, kmin, kmax);
  const int le = L.count_le(Pl);
  const int less = Pl > kmin ? L.count_le(Pl - 1) : 0;
  const unsigned vlo = exact_rank(L, Pl, lo - less, le - less, lo_plane, list);
  unsigned vhi = vlo;
  if (hi != lo) {
    if (hi < le) {
      vhi = exact_rank(L, Pl, hi - less, le - less, lo_plane, list);
    } else {
      const unsigned Ph = L.min_greater(Pl);
      vhi = exact_rank(L, Ph, 0, L.count_le(Ph) - le, lo_plane, list);
    }
  }
  const float slo = sqrt_rn(__builtin_bit_cast(float, vlo));
  float th;
  if (lo_f == hi_f) {
    th = slo;
  } else {
    const float shi = sqrt_rn(__builtin_bit_cast(float, vhi));
    const float aa = slo * (hi_f - q);
    const float bb = shi * (q - lo_f);
    th = aa + bb;
  }
  *thr = th;
  *T = sq_threshold(th);
}

// ---------------------------------------------------------------------------------------
// k_sel_rows9<KPL>: one wave per CRP row.
// ---------------------------------------------------------------------------------------
template <int KPL>
__global__ __launch_bounds__(256) void k_sel_rows9(CrpBatch B, KeyPlanes K, int ldr, int64_t kstride, float kappa,
                                                   float* __restrict__ thr, float* __restrict__ Tq,
                                                   int64_t thr_stride) {
  __shared__ int lists[4][64];
  const int p = blockIdx.y;
  const PairView V = pair_view(B, p);
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= V.Mp) return;
  int* list = lists[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  Line<KPL> L;
  const size_t line = (size_t)p * kstride + (size_t)i * ldr;
  L.load(K.hr + line, V.Np);
  float th, T;
  line_threshold(L, V.Np, kappa, K.lr + line, list, &th, &T);
  if (lane == 0) {
    thr[(size_t)p * thr_stride + i] = th;
    Tq[(size_t)p * thr_stride + i] = T;
  }
}

// ---------------------------------------------------------------------------------------
// k_sel_cols9<KPL>: one wave per CRP column; also emits the CRP words of the column.
// Requires KPL == 32 for the word emission (lane l <-> rows 32l..32l+31).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sel_cols9(CrpBatch B, KeyPlanes K, int ldc, int64_t kstride, float kappa,
                                                   const float* __restrict__ Trow,
                                                   float* __restrict__ thr, float* __restrict__ Tq,
                                                   int64_t thr_stride, uint32_t* __restrict__ maskT,
                                                   int64_t mask_stride, int ld) {
  constexpr int KPL = 32;
  __shared__ int lists[4][64];
  const int p = blockIdx.y;
  const PairView V = pair_view(B, p);
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= V.Np) return;
  int* list = lists[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  Line<KPL> L;
  const size_t line = (size_t)p * kstride + (size_t)j * ldc;
  L.load(K.hc + line, V.Mp);
  const uint16_t* lo_plane = K.lc + line;
  float th, Tc;
  line_threshold(L, V.Mp, kappa, lo_plane, list, &th, &Tc);
  if (lane == 0) {
    thr[(size_t)p * thr_stride + j] = th;
    Tq[(size_t)p * thr_stride + j] = Tc;
  }
  // CRP word of strip `lane` (rows 32*lane .. +31) at column j
  const int i0 = lane * KPL;
  if (i0 >= V.Mp) return;
  const unsigned Tc_bits = __builtin_bit_cast(unsigned, Tc);
  const unsigned Tc16 = Tc_bits >> 16;
  const float* tr = Trow + (size_t)p * thr_stride + i0;
  uint32_t word = 0, amb = 0;
#pragma unroll
  for (int q = 0; q < KPL; ++q) {
    const unsigned k = L.v[q];
    if (k == 0xffffffffu) continue;
    const unsigned Tr_bits = __builtin_bit_cast(unsigned, tr[q]);
    const unsigned Tr16 = Tr_bits >> 16;
    const bool surely = (k < Tr16) && (k < Tc16);
    const bool maybe = (k <= Tr16) && (k <= Tc16);
    word |= (uint32_t)surely << q;
    amb |= (uint32_t)(maybe && !surely) << q;
  }
  while (amb) {  // prefix ties a threshold prefix: decide on the exact key
    const int q = __builtin_ctz(amb);
    amb &= amb - 1;
    const unsigned key = (L.v[q] << 16) | (unsigned)lo_plane[i0 + q];
    const unsigned Tr_bits = __builtin_bit_cast(unsigned, tr[q]);
    word |= (uint32_t)((key <= Tr_bits) && (key <= Tc_bits)) << q;
  }
  maskT[(size_t)p * mask_stride + (size_t)lane * ld + j] = word;
}

}  // namespace

// Three-kernel CRP (m = 9, lines up to 2048 keys). Returns 1 if not applicable.
int launch_crp_split(const CrpBatch& B, int nb, int L, float kappa, uint16_t* kplanes, int ldk, int64_t kstride,
                     float* thr_r, float* T_r, float* thr_c, float* T_c, int64_t thr_stride, uint32_t* maskT,
                     int64_t mask_stride, int ld, hipStream_t s) {
  if (B.m != kMS || L > 2048) return 1;
  const size_t plane = (size_t)nb * kstride;
  const KeyPlanes K{kplanes, kplanes + plane, kplanes + 2 * plane, kplanes + 3 * plane};
  prof_begin(PH_SWEEP, s);
  hipLaunchKernelGGL(k_sweep9, dim3((L + kSR - 1) / kSR, nb), dim3(kSW), 0, s, B, K, ldk, ldk, kstride);
  ACOSS_LAUNCH_CHECK();
  prof_end(PH_SWEEP, s);
  prof_begin(PH_SEL_ROWS, s);
  hipLaunchKernelGGL(k_sel_rows9<32>, dim3((L + 3) / 4, nb), dim3(256), 0, s, B, K, ldk, kstride, kappa, thr_r, T_r,
                     thr_stride);
  ACOSS_LAUNCH_CHECK();
  prof_end(PH_SEL_ROWS, s);
  prof_begin(PH_SEL_COLS, s);
  hipLaunchKernelGGL(k_sel_cols9, dim3((L + 3) / 4, nb), dim3(256), 0, s, B, K, ldk, kstride, kappa, T_r, thr_c,
                     T_c, thr_stride, maskT, mask_stride, ld);
  ACOSS_LAUNCH_CHECK();
  prof_end(PH_SEL_COLS, s);
  return ACOSS_OK;
}

}  // namespace acoss
