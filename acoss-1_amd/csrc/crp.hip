// crp.hip — Serra09 / LateFusionChen hot path on gfx950:
//   OTI key shift -> stacked-frame Euclidean distances -> per-row / per-column percentile
//   thresholds -> mutual-neighbour CRP mask -> Qmax (serra09) / dmax (chen17) wavefront DP.
//
// Replaces, per pair, essentia ChromaCrossSimilarity + CoverSongSimilarity as called at
// acoss/algorithms/rqa_serra09.py:55-69 and acoss/algorithms/latefusion_chen.py:58-73.
// Arithmetic follows the canonical rounding sequence documented in oracle/crp_oracle.cpp
// step for step (fmaf chains, sequential adds, correctly rounded sqrt), so the OTI index,
// the thresholds and the CRP mask are bit-identical to the CPU restatement.
//
// Design: nothing of size M'xN' ever touches HBM.
//  * k_crp_select<TRANS>: one 256-thread block per (pair, stripe of R own frames). It
//    sweeps the other song in 256-column panels: the 12-d Gram of (R+m-1) x (256+m-1)
//    frames is computed into LDS (fmaf chains), the m-tap diagonal window gives the squared
//    stacked distance of R x 256 cells, which stay in an LDS stripe. A block-wide 3-pass
//    radix select (11/10/10 bits of the float key) then gives the two order statistics of
//    each row (column for TRANS) and the interpolated percentile threshold. The mask is
//    later evaluated in the squared domain (sq_threshold), so no per-cell sqrt is needed.
//  * k_crp_panel: recomputes the distances of a 32-row x 256-column panel and writes the
//    CRP as one 32-bit word per (32-row strip, column): the layout the DP consumes.
//  * k_crp_dp: one wave per pair. Lane l owns 32 rows of a 2048-row band and sweeps the
//    columns skewed by one column per lane (anti-diagonal wavefront); the two boundary rows
//    pass down one lane per step with __shfl_up; bands chain through a small HBM buffer.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "crp_internal.hpp"

namespace acoss {

constexpr int kPanelW = 256;  // columns per panel = threads per block

// --------------------------------------------------------------------------------------
// Per-track preparation (O(sum n)): OTI profile and stacked squared norms.
// --------------------------------------------------------------------------------------
__device__ inline float frame_norm(const float* __restrict__ x) {
  float acc = 0.0f;
#pragma unroll
  for (int c = 0; c < 12; ++c) acc = __builtin_fmaf(x[c], x[c], acc);
  return acc;
}

// 64 threads = 4 tracks x 16 lanes (lanes 12..15 idle). prof[t*12+c].
__global__ void k_track_profile(const float* __restrict__ feats, const int64_t* __restrict__ off,
                                const int32_t* __restrict__ len, int n_tracks, float* __restrict__ prof) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 4);
  const int c = threadIdx.x & 15;
  float s = 0.0f;
  if (t < n_tracks && c < 12) {
    const int n = len[t];
    const float* x = feats + off[t] * 12 + c;
    for (int a = 0; a < n; ++a) s = s + x[(size_t)a * 12];
    s = n > 0 ? s / (float)n : 0.0f;
  }
  float mx = (c < 12) ? s : -INFINITY;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 16));
  if (t < n_tracks && c < 12) prof[t * 12 + c] = mx > 0.0f ? s / mx : 0.0f;
}

// NX[t*ldn + s] = sum_{u<m} |frame (s+u)*tau|^2 (sequential), s < stacked_len.
__global__ void k_track_norms(const float* __restrict__ feats, const int64_t* __restrict__ off,
                              const int32_t* __restrict__ len, int m, int tau, int ldn, float* __restrict__ NX) {
  const int t = blockIdx.x;
  const int s = blockIdx.y * blockDim.x + threadIdx.x;
  const int S = stacked_len(len[t], m, tau);
  if (s >= S) return;
  const float* x = feats + off[t] * 12;
  float acc = 0.0f;
  for (int u = 0; u < m; ++u) acc = acc + frame_norm(x + (size_t)(s + u) * tau * 12);
  NX[(size_t)t * ldn + s] = acc;
}

// X2[t][f] = frames f and f + 1 of track t interleaved bin by bin (24 floats; frame n is 0):
// the operand pairs of the split sweep's packed-FP32 Gram (crp_split.hip).
__global__ void k_track_pairs(const float* __restrict__ feats, const int64_t* __restrict__ off,
                              const int32_t* __restrict__ len, int ldn, float* __restrict__ X2) {
  const int t = blockIdx.x;
  const int f = blockIdx.y * blockDim.x + threadIdx.x;
  const int n = len[t];
  if (f >= n) return;
  const float* x = feats + (off[t] + f) * 12;
  float4* o = reinterpret_cast<float4*>(X2 + ((size_t)t * ldn + f) * 24);
  const bool nx = f + 1 < n;
#pragma unroll
  for (int c = 0; c < 6; ++c)
    o[c] = make_float4(x[2 * c], nx ? x[12 + 2 * c] : 0.0f, x[2 * c + 1], nx ? x[12 + 2 * c + 1] : 0.0f);
}

// Per pair: OTI index (essentia optimalTranspositionIndex restated) and stacked dims.
__global__ void k_pair_oti(const float* __restrict__ prof, const int32_t* __restrict__ len,
                           const int32_t* __restrict__ pairs, int64_t n_pairs, int use_oti, int m, int tau,
                           int32_t* __restrict__ oti, int2* __restrict__ dims) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const int a = pairs[2 * p], b = pairs[2 * p + 1];
  int best = 0;
  if (use_oti) {
    float pq[12], pr[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      pq[c] = prof[a * 12 + c];
      pr[c] = prof[b * 12 + c];
    }
    float bestv = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      float acc = 0.0f;
#pragma unroll
      for (int c = 0; c < 12; ++c) acc = __builtin_fmaf(pq[c], pr[(c - k + 12) % 12], acc);
      if (k == 0 || acc > bestv) {
        bestv = acc;
        best = k;
      }
    }
  }
  oti[p] = best;
  dims[p] = make_int2(stacked_len(len[a], m, tau), stacked_len(len[b], m, tau));
}

// yrot[p][f][c] = reference[f][(c - oti[p]) mod 12]  (np.roll of every reference frame).
__global__ void k_rotate_ref(const float* __restrict__ feats, const int64_t* __restrict__ off,
                             const int32_t* __restrict__ len, const int32_t* __restrict__ pairs,
                             const int32_t* __restrict__ oti, float* __restrict__ yrot, int64_t stride) {
  const int p = blockIdx.y;
  const int b = pairs[2 * p + 1];
  const int n = len[b], k = oti[p];
  const float* src = feats + off[b] * 12;
  float* dst = yrot + (size_t)p * stride;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n * 12; e += gridDim.x * blockDim.x) {
    const int f = e / 12, c = e - f * 12;
    dst[e] = src[(size_t)f * 12 + (c - k + 12) % 12];
  }
}

// --------------------------------------------------------------------------------------
// Panel machinery: rows = R "own" stacked frames starting at i0, columns = 256 "inner"
// stacked frames starting at j0. LDS: Xs[GR][12], Ys[GW][13], Gs[GR][GW],
// GR = R+m-1, GW = 256+m-1. Own = query unless TRANS (then own = reference).
// --------------------------------------------------------------------------------------
struct PanelArgs {
  const float* own;    // frames of the own track (n_own x 12)
  const float* inner;  // frames of the inner track
  int k_own, k_inner;  // chroma roll applied to own / inner frames (one of them is 0)
  int n_own, n_inner;  // frame counts
  int m, tau;
};

// Stage own frames (once per block): Xs[a][c] = own[(i0+a)*tau][(c-k) mod 12].
__device__ inline void stage_own(const PanelArgs& A, int i0, int GR, float* Xs) {
  for (int e = threadIdx.x; e < GR * 12; e += blockDim.x) {
    const int a = e / 12, c = e - a * 12;
    const int f = (i0 + a) * A.tau;
    Xs[e] = f < A.n_own ? A.own[(size_t)f * 12 + ((c - A.k_own + 12) % 12)] : 0.0f;
  }
}

// Stage inner frames of panel j0 and build the Gram Gs[a][b] = fmaf-chain_c Xs[a][c]*Ys[b][c].
__device__ inline void panel_gram(const PanelArgs& A, int j0, int GR, int GW, const float* Xs, float* Ys,
                                  float* Gs) {
  for (int e = threadIdx.x; e < GW * 12; e += blockDim.x) {
    const int b = e / 12, c = e - b * 12;
    const int f = (j0 + b) * A.tau;
    Ys[b * 13 + c] = f < A.n_inner ? A.inner[(size_t)f * 12 + ((c - A.k_inner + 12) % 12)] : 0.0f;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < GW; b += blockDim.x) {
    float y[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) y[c] = Ys[b * 13 + c];
    for (int a = 0; a < GR; ++a) {
      const float4* xr = reinterpret_cast<const float4*>(Xs + a * 12);
      const float4 x0 = xr[0], x1 = xr[1], x2 = xr[2];
      float acc = 0.0f;
      acc = __builtin_fmaf(x0.x, y[0], acc);
      acc = __builtin_fmaf(x0.y, y[1], acc);
      acc = __builtin_fmaf(x0.z, y[2], acc);
      acc = __builtin_fmaf(x0.w, y[3], acc);
      acc = __builtin_fmaf(x1.x, y[4], acc);
      acc = __builtin_fmaf(x1.y, y[5], acc);
      acc = __builtin_fmaf(x1.z, y[6], acc);
      acc = __builtin_fmaf(x1.w, y[7], acc);
      acc = __builtin_fmaf(x2.x, y[8], acc);
      acc = __builtin_fmaf(x2.y, y[9], acc);
      acc = __builtin_fmaf(x2.z, y[10], acc);
      acc = __builtin_fmaf(x2.w, y[11], acc);
      Gs[a * GW + b] = acc;
    }
  }
  __syncthreads();
}

// Squared stacked distance key of cell (row r of the panel, column t): max(d2, +0).
template <bool TRANS>
__device__ inline float cell_key(const float* Gs, int GW, int m, int r, int t, float n_own, float n_inner) {
  float dot = 0.0f;
  for (int u = 0; u < m; ++u) dot = dot + Gs[(r + u) * GW + t + u];
  // canonical: (N_query - 2*dot) + N_reference
  const float d2 = TRANS ? (n_inner - 2.0f * dot) + n_own : (n_own - 2.0f * dot) + n_inner;
  return d2 > 0.0f ? d2 : 0.0f;
}

__host__ __device__ inline size_t panel_lds_floats(int R, int m) {
  const int GR = R + m - 1, GW = kPanelW + m - 1;
  return align_up((size_t)GR * 12, 4) + align_up((size_t)GW * 13, 4) + (size_t)GR * GW;
}

// --------------------------------------------------------------------------------------
// Block-wide radix select on non-negative float keys held in LDS.
// --------------------------------------------------------------------------------------
struct SelScratch {
  int* hist;  // >= 2048 ints
  int* sh;    // >= 16 ints
};

// Exclusive scan of one int per thread over a 256-thread block; returns the total in *tot.
__device__ inline int block_excl_scan256(int v, int* sh, int* tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int inc = wave_incl_scan(v);
  if (lane == 63) sh[8 + w] = inc;
  __syncthreads();
  int before = 0, all = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int wq = sh[8 + q];
    before += (q < w) ? wq : 0;
    all += wq;
  }
  *tot = all;
  return before + inc - v;
}

// Key of rank k (0-based) among keys[0..n); *eq = multiplicity of that key, *less = #keys below.
__device__ inline unsigned block_select_rank(const unsigned* keys, int n, int k, SelScratch S, int* eq, int* less) {
  unsigned prefix = 0;
  const int k0 = k;
  int eqc = 0;
#pragma unroll 1
  for (int pass = 0; pass < 3; ++pass) {
    const int shift = pass == 0 ? 20 : (pass == 1 ? 10 : 0);
    const int bits = pass == 0 ? 11 : 10;
    const int nb = 1 << bits;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) S.hist[i] = 0;
    __syncthreads();
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      const unsigned key = keys[e];
      if ((key >> (shift + bits)) == prefix) atomicAdd(&S.hist[(key >> shift) & (nb - 1)], 1);
    }
    __syncthreads();
    const int per = nb / 256;  // 8 or 4 bins per thread
    const int base = threadIdx.x * per;
    int part = 0;
    for (int i = 0; i < per; ++i) part += S.hist[base + i];
    int tot;
    const int before = block_excl_scan256(part, S.sh, &tot);
    if (k >= before && k < before + part) {
      int acc = before;
      for (int i = 0; i < per; ++i) {
        const int h = S.hist[base + i];
        if (k < acc + h) {
          S.sh[0] = base + i;
          S.sh[1] = k - acc;
          S.sh[2] = h;
          break;
        }
        acc += h;
      }
    }
    __syncthreads();
    prefix = (prefix << bits) | (unsigned)S.sh[0];
    k = S.sh[1];
    eqc = S.sh[2];
    __syncthreads();
  }
  *eq = eqc;
  *less = k0 - k;
  return prefix;
}

// Smallest key strictly greater than v (0xffffffff if none).
__device__ inline unsigned block_min_greater(const unsigned* keys, int n, unsigned v, int* sh) {
  unsigned mn = 0xffffffffu;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const unsigned key = keys[e];
    if (key > v && key < mn) mn = key;
  }
  mn = wave_min_u32(mn);
  if ((threadIdx.x & 63) == 0) sh[4 + (threadIdx.x >> 6)] = (int)mn;
  __syncthreads();
  unsigned r = 0xffffffffu;
  for (int q = 0; q < 4; ++q) r = min(r, (unsigned)sh[4 + q]);
  __syncthreads();
  return r;
}

// essentia percentile of the n keys (squared distances) in D units + the squared-domain
// threshold. Written by thread 0.
__device__ inline void block_percentile(const unsigned* keys, int n, float kappa, SelScratch S, float* thr_out,
                                        float* T_out) {
  const float q = (float)(n - 1) * kappa;
  const float lo_f = floorf(q), hi_f = ceilf(q);
  const int lo = (int)lo_f, hi = (int)hi_f;
  int eq, less;
  const unsigned vlo = block_select_rank(keys, n, lo, S, &eq, &less);
  unsigned vhi = vlo;
  if (hi != lo && less + eq <= hi) vhi = block_min_greater(keys, n, vlo, S.sh);
  if (threadIdx.x == 0) {
    const float slo = sqrt_rn(__builtin_bit_cast(float, vlo));
    float thr;
    if (lo_f == hi_f) {
      thr = slo;
    } else {
      const float shi = sqrt_rn(__builtin_bit_cast(float, vhi));
      const float a = slo * (hi_f - q);
      const float b = shi * (q - lo_f);
      thr = a + b;
    }
    *thr_out = thr;
    *T_out = sq_threshold(thr);
  }
  __syncthreads();
}

// --------------------------------------------------------------------------------------
// k_crp_select<TRANS>: per (stripe of R own frames, pair) -> thresholds of those rows
// (TRANS=false: rows of the CRP / query frames) or columns (TRANS=true: reference frames).
// Dynamic LDS: Dst[R][ld] keys | panel buffers. Hist aliases the Ys|Gs panel region.
// --------------------------------------------------------------------------------------

template <bool TRANS>
__global__ __launch_bounds__(256) void k_crp_select(CrpBatch B, int R, int ld, float kappa, float* __restrict__ thr,
                                                    float* __restrict__ Tq, int64_t thr_stride) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int p = blockIdx.y;
  const int2 dm = B.dims[p];
  const int n_own_s = TRANS ? dm.y : dm.x, n_in_s = TRANS ? dm.x : dm.y;
  const int i0 = blockIdx.x * R;
  if (i0 >= n_own_s || n_in_s <= 0) return;
  const int ta = B.pairs[2 * p], tb = B.pairs[2 * p + 1];
  const int t_own = TRANS ? tb : ta, t_in = TRANS ? ta : tb;
  const int k = B.oti[p];
  PanelArgs A;
  A.own = B.feats + B.off[t_own] * 12;
  A.inner = B.feats + B.off[t_in] * 12;
  A.k_own = TRANS ? k : 0;
  A.k_inner = TRANS ? 0 : k;
  A.n_own = B.len[t_own];
  A.n_inner = B.len[t_in];
  A.m = B.m;
  A.tau = B.tau;
  const int m = B.m, GR = R + m - 1, GW = kPanelW + m - 1;
  float* Dst = smem;
  float* Xs = Dst + (size_t)R * ld;
  float* Ys = Xs + align_up((size_t)GR * 12, 4);
  float* Gs = Ys + align_up((size_t)GW * 13, 4);
  const float* NXown = B.NX + (size_t)t_own * B.ldn;
  const float* NXin = B.NX + (size_t)t_in * B.ldn;
  const int rows = min(R, n_own_s - i0);
  float nown[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) nown[r] = (r < rows) ? NXown[i0 + r] : 0.0f;

  stage_own(A, i0, GR, Xs);
  for (int j0 = 0; j0 < n_in_s; j0 += kPanelW) {
    panel_gram(A, j0, GR, GW, Xs, Ys, Gs);
    const int t = threadIdx.x, j = j0 + t;
    if (j < n_in_s) {
      const float nin = NXin[j];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r < rows) Dst[(size_t)r * ld + j] = cell_key<TRANS>(Gs, GW, m, r, t, nown[r], nin);
    }
    __syncthreads();
  }
  SelScratch S;
  S.hist = reinterpret_cast<int*>(Ys);
  S.sh = S.hist + 2048;
  for (int r = 0; r < rows; ++r) {
    block_percentile(reinterpret_cast<const unsigned*>(Dst + (size_t)r * ld), n_in_s, kappa, S,
                     thr + (size_t)p * thr_stride + i0 + r, Tq + (size_t)p * thr_stride + i0 + r);
  }
}

__host__ inline size_t select_lds_bytes(int R, int m, int ld) {
  return ((size_t)R * ld + panel_lds_floats(R, m)) * sizeof(float);
}

// --------------------------------------------------------------------------------------
// k_crp_panel<MODE>: 32 query rows (one strip) x 256 reference columns.
// MODE 0: CRP bits -> maskT[p][strip][j] (bit r = row 32*strip + r). MODE 1: dist (sqrt).
// --------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void k_crp_panel(CrpBatch B, const float* __restrict__ Trow,
                                                   const float* __restrict__ Tcol, int64_t thr_stride,
                                                   uint32_t* __restrict__ maskT, int64_t mask_stride, int ld,
                                                   float* __restrict__ dist) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int R = 32;
  const int p = blockIdx.z;
  const int2 dm = B.dims[p];
  const int strip = blockIdx.y;
  const int i0 = strip * R, j0 = blockIdx.x * kPanelW;
  if (i0 >= dm.x || j0 >= dm.y) return;
  const int ta = B.pairs[2 * p], tb = B.pairs[2 * p + 1];
  PanelArgs A;
  A.own = B.feats + B.off[ta] * 12;
  A.inner = B.feats + B.off[tb] * 12;
  A.k_own = 0;
  A.k_inner = B.oti[p];
  A.n_own = B.len[ta];
  A.n_inner = B.len[tb];
  A.m = B.m;
  A.tau = B.tau;
  const int m = B.m, GR = R + m - 1, GW = kPanelW + m - 1;
  float* Xs = smem;
  float* Ys = Xs + align_up((size_t)GR * 12, 4);
  float* Gs = Ys + align_up((size_t)GW * 13, 4);
  const float* NXq = B.NX + (size_t)ta * B.ldn;
  const float* NXr = B.NX + (size_t)tb * B.ldn;
  stage_own(A, i0, GR, Xs);
  panel_gram(A, j0, GR, GW, Xs, Ys, Gs);
  const int t = threadIdx.x, j = j0 + t;
  if (j >= dm.y) return;
  const int rows = min(R, dm.x - i0);
  const float nin = NXr[j];
  if (MODE == 0) {
    const float tc = Tcol[(size_t)p * thr_stride + j];
    const float* tr = Trow + (size_t)p * thr_stride + i0;
    uint32_t bits = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r < rows) {
        const float key = cell_key<false>(Gs, GW, m, r, t, NXq[i0 + r], nin);
        bits |= (uint32_t)((key <= tr[r]) & (key <= tc)) << r;
      }
    }
    maskT[(size_t)p * mask_stride + (size_t)strip * ld + j] = bits;
  } else {
#pragma unroll 4
    for (int r = 0; r < rows; ++r) {
      const float key = cell_key<false>(Gs, GW, m, r, t, NXq[i0 + r], nin);
      dist[(size_t)(i0 + r) * dm.y + j] = sqrt_rn(key);
    }
  }
}

// --------------------------------------------------------------------------------------
// k_crp_dp<ALIGN, EQG, R>: essentia CoverSongSimilarity(serra09 | chen17, 'symmetric').
// One wave per pair; lane l owns R rows, band*64R + Rl .. +R-1 (R = 32, 16 or 8 by the batch's
// longest CRP, so short tracks keep every lane busy); column c = s - l at step s.
// --------------------------------------------------------------------------------------
struct DpAbove {  // what lane l-1 (or the band above) hands down for one column
  float q30, q31;  // its last two rows (R-2, R-1)
  uint32_t b;      // bit0 = C[row R-2], bit1 = C[row R-1]
};

// FAST (serra09 with gamma_open == gamma_ext = K/2 >= 0, the reference's setting): every score is
// an exact multiple of 1/2, so "hit ? mx + 1 : max(mx - go, 0)" is max(fma(hit, 1 + go, mx - go), 0)
// exactly, and the validity masks move out of the row loop: the kernel zeroes the CRP words of
// columns < 2 and rows outside [2, Mp) at the fetch. Cells there then hold 0 (top-left: all their
// predecessors are 0) or at most max(0, best - go) (bottom/right: no hit, and they never feed a
// valid cell), so neither the valid scores nor their maximum change.
// v_cvt_f32_ubyteB: byte B of v as a float (the compiler emits only the byte-0 form plus shifts).
template <int B>
__device__ __forceinline__ float cvt_f32_ubyte(uint32_t v) {
  float f;
  if constexpr (B == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(v));
  else if constexpr (B == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f) : "v"(v));
  else if constexpr (B == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f) : "v"(v));
  else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f) : "v"(v));
  return f;
}

// b is a constant after the row loops unroll, so the switch folds away
__device__ __forceinline__ float cvt_f32_ubyte_n(uint32_t v, int b) {
  switch (b) {
    case 0: return cvt_f32_ubyte<0>(v);
    case 1: return cvt_f32_ubyte<1>(v);
    case 2: return cvt_f32_ubyte<2>(v);
    default: return cvt_f32_ubyte<3>(v);
  }
}

template <int ALIGN, bool EQG, int R, bool FAST = false>
struct DpLane {
  float go, ge;
  int Np, lane, c_off;  // column of this lane at step s: s - lane
  uint32_t rowvalid;    // bit r: 2 <= global row < Mp
  uint32_t w1, w2;      // CRP words of columns c-1, c-2 (bit r = row r)
  DpAbove h1, h2;       // from above for columns c-1, c-2
  float best;

  __device__ __forceinline__ float gam(uint32_t bit) const { return EQG ? go : (bit ? go : ge); }

  // qn: new column c; q1: column c-1; q2: column c-2. w0: CRP word of column c;
  // h0: from above for column c. Returns the values to hand to the lane below.
  __device__ __forceinline__ DpAbove step(float (&qn)[R], const float (&q1)[R], const float (&q2)[R],
                                          uint32_t w0, const DpAbove& h0, int c) {
    const bool colvalid = (c >= 2) && (c < Np);
    const uint32_t vmask = colvalid ? rowvalid : 0u;
    // extended words: bit r+2 <-> row r; bits 0,1 <-> rows -2,-1 (from above)
    const uint64_t e0 = ((uint64_t)w0 << 2) | h0.b;
    const uint64_t e1 = ((uint64_t)w1 << 2) | h1.b;
    const uint64_t e2 = ((uint64_t)w2 << 2) | h2.b;
    if constexpr (FAST) {
      // two rows per v_pk_add_f32 / v_pk_fma_f32; the hit bits as bytes (rows k, k+8, k+16, k+24
      // of one masked word), one v_cvt_f32_ubyteN each
      typedef float dp_f32x2 __attribute__((ext_vector_type(2)));
      const dp_f32x2 g1 = {1.0f + go, 1.0f + go};
      const dp_f32x2 ngo = {-go, -go};
      uint32_t bm[R < 8 ? R : 8];
#pragma unroll
      for (int k = 0; k < (R < 8 ? R : 8); ++k) bm[k] = (w0 >> k) & 0x01010101u;
#pragma unroll
      for (int r = 0; r < R; r += 2) {
        float mxs[2], hb[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int rr = r + e;
          const float Qa = rr >= 1 ? q1[rr - 1] : h1.q31;
          const float Qb = rr >= 2 ? q1[rr - 2] : (rr == 1 ? h1.q31 : h1.q30);
          const float Qc = rr >= 1 ? q2[rr - 1] : h2.q31;
          mxs[e] = fmaxf(fmaxf(Qa, Qb), Qc);
          hb[e] = cvt_f32_ubyte_n(bm[rr & 7], rr >> 3);
        }
        const dp_f32x2 mx = {mxs[0], mxs[1]};
        const dp_f32x2 hv = {hb[0], hb[1]};
        const dp_f32x2 t = __builtin_elementwise_fma(hv, g1, mx + ngo);
        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(best) : "v"(best), "v"(t.x), "v"(t.y));
        qn[r] = fmaxf(t.x, 0.0f);
        qn[r + 1] = fmaxf(t.y, 0.0f);
      }
    } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float Qa = r >= 1 ? q1[r - 1] : h1.q31;                            // Q[r-1][c-1]
      float Qb = r >= 2 ? q1[r - 2] : (r == 1 ? h1.q31 : h1.q30);              // Q[r-2][c-1]
      float Qc = r >= 1 ? q2[r - 1] : h2.q31;                                  // Q[r-1][c-2]
      if (ALIGN == 1) {
        Qb = Qb + (float)((e0 >> (r + 1)) & 1u);  // + C[r-1][c]
        Qc = Qc + (float)((e1 >> (r + 2)) & 1u);  // + C[r][c-1]
      }
      const bool hit = (e0 >> (r + 2)) & 1u;
      float v;
      if (EQG) {
        const float mx = fmaxf(fmaxf(Qa, Qb), Qc);
        v = hit ? mx + 1.0f : fmaxf(mx - go, 0.0f);
      } else {
        const float x = Qa - gam((e1 >> (r + 1)) & 1u);  // gamma(C[r-1][c-1])
        const float y = Qb - gam((e1 >> r) & 1u);        // gamma(C[r-2][c-1])
        const float z = Qc - gam((e2 >> (r + 1)) & 1u);  // gamma(C[r-1][c-2])
        const float miss = fmaxf(fmaxf(0.0f, x), fmaxf(y, z));
        v = hit ? fmaxf(fmaxf(Qa, Qb), Qc) + 1.0f : miss;
      }
      v = ((vmask >> r) & 1u) ? v : 0.0f;
      best = fmaxf(best, v);
      qn[r] = v;
    }
    }
    DpAbove out;
    out.q30 = qn[R - 2];
    out.q31 = qn[R - 1];
    out.b = (w0 >> (R - 2)) & 3u;
    h2 = h1;
    h1 = h0;
    w2 = w1;
    w1 = w0;
    return out;
  }
};

template <int ALIGN, bool EQG, int R, bool FAST>
__device__ __forceinline__ void crp_dp_body(const uint32_t* __restrict__ maskT, int64_t mask_stride, int ld,
                                               const int2* __restrict__ dims, float go, float ge,
                                               float4* __restrict__ bnd, int64_t bnd_stride,
                                               float* __restrict__ out) {
  const int p = blockIdx.x;
  const int lane = threadIdx.x;
  const int2 dm = dims[p];
  const int Mp = dm.x, Np = dm.y;
  float best = 0.0f;
  constexpr int kBand = 64 * R;
  const int nbands = (Mp + kBand - 1) / kBand;
  for (int band = 0; band < nbands; ++band) {
    const int row0 = band * kBand + lane * R;
    const uint32_t* mrow = maskT + (size_t)p * mask_stride + (size_t)(row0 >> 5) * ld;
    const int sh = row0 & 31;  // this lane's R rows inside its 32-row strip word
    float4* bout = bnd + (size_t)p * bnd_stride + (size_t)band * ld;
    const float4* bin = bnd + (size_t)p * bnd_stride + (size_t)(band - 1) * ld;
    DpLane<ALIGN, EQG, R, FAST> L;
    L.go = go;
    L.ge = ge;
    L.Np = Np;
    L.lane = lane;
    uint32_t rv = 0;
    for (int r = 0; r < R; ++r) rv |= (uint32_t)((row0 + r >= 2) && (row0 + r < Mp)) << r;
    L.rowvalid = rv;
    L.w1 = L.w2 = 0;
    L.h1 = L.h2 = DpAbove{0.0f, 0.0f, 0u};
    L.best = 0.0f;
    float qa[R], qb[R], qc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) qa[r] = qb[r] = qc[r] = 0.0f;
    DpAbove pub{0.0f, 0.0f, 0u};
    const int S_end = Np + 63;
    const bool lane_active = row0 < Mp;
    auto fetch = [&](int c) -> uint32_t {
      if (!(lane_active && c >= (FAST ? 2 : 0) && c < Np)) return 0u;
      const uint32_t w = mrow[c];
      const uint32_t wr = R == 32 ? w : (w >> sh) & ((1u << (R & 31)) - 1u);
      return FAST ? (wr & rv) : wr;
    };
    auto recv = [&](const DpAbove& mine, int c) -> DpAbove {
      DpAbove h;
      h.q30 = __shfl_up(mine.q30, 1);
      h.q31 = __shfl_up(mine.q31, 1);
      h.b = (uint32_t)__shfl_up((int)mine.b, 1);
      if (lane == 0) {
        if (band > 0 && c >= 0 && c < Np) {
          const float4 v = bin[c];
          h = DpAbove{v.x, v.y, (uint32_t)v.z};
        } else {
          h = DpAbove{0.0f, 0.0f, 0u};
        }
      }
      return h;
    };
    auto publish = [&](const DpAbove& o, int c) {
      if (lane == 63 && band + 1 < nbands && c >= 0 && c < Np) bout[c] = make_float4(o.q30, o.q31, (float)o.b, 0.0f);
    };
    uint32_t wnext = fetch(-lane);
    for (int s = 0; s < S_end; s += 3) {
      {
        const int c = s - lane;
        const uint32_t w0 = wnext;
        wnext = fetch(c + 1);
        const DpAbove h0 = recv(pub, c);
        pub = L.step(qa, qb, qc, w0, h0, c);
        publish(pub, c);
      }
      if (s + 1 < S_end) {
        const int c = s + 1 - lane;
        const uint32_t w0 = wnext;
        wnext = fetch(c + 1);
        const DpAbove h0 = recv(pub, c);
        pub = L.step(qc, qa, qb, w0, h0, c);
        publish(pub, c);
      }
      if (s + 2 < S_end) {
        const int c = s + 2 - lane;
        const uint32_t w0 = wnext;
        wnext = fetch(c + 1);
        const DpAbove h0 = recv(pub, c);
        pub = L.step(qb, qc, qa, w0, h0, c);
        publish(pub, c);
      }
    }
    best = fmaxf(best, L.best);
    __threadfence_block();
    __syncthreads();
  }
  best = wave_max(best);
  if (lane == 0) out[p] = best;
}

template <int ALIGN, bool EQG, int R>
__global__ __launch_bounds__(64) void k_crp_dp(const uint32_t* __restrict__ maskT, int64_t mask_stride, int ld,
                                               const int2* __restrict__ dims, float go, float ge,
                                               float4* __restrict__ bnd, int64_t bnd_stride,
                                               float* __restrict__ out) {
  crp_dp_body<ALIGN, EQG, R, false>(maskT, mask_stride, ld, dims, go, ge, bnd, bnd_stride, out);
}

// No occupancy hint: the FAST body compiles to about 200 VGPRs (2 waves per SIMD), which measured
// faster than forcing it into 128 (4 waves per SIMD): 14.2 vs 14.8 ms per covers80 step.
template <int R>
__global__ __launch_bounds__(64) void k_crp_dp_fast(
    const uint32_t* __restrict__ maskT, int64_t mask_stride, int ld, const int2* __restrict__ dims, float go, float ge,
    float4* __restrict__ bnd, int64_t bnd_stride, float* __restrict__ out) {
  crp_dp_body<0, true, R, true>(maskT, mask_stride, ld, dims, go, ge, bnd, bnd_stride, out);
}

// --------------------------------------------------------------------------------------
// k_crp_dp_grp: the FAST DP (serra09, gamma_open == gamma_ext = K/2) with SEVERAL pairs per
// wave for CRPs of at most 2048 rows: a group of LP = ceil(L / 32) lanes per pair (lane ll owns
// rows 32 ll .. 32 ll + 31, one band), G = 64 / LP groups per wave. A one-pair wave walks
// N' + 63 steps however short the pair; a group walks N' + LP - 1, and every lane keeps 32 rows
// per step, so short tracks (Da-TACOS lengths: L ~ 500) no longer leave most lanes idle or pay
// the per-step shuffles for 8 rows. Same recurrence, same DpLane step: bit-identical scores.
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_crp_dp_grp(const uint32_t* __restrict__ maskT, int64_t mask_stride, int ld,
                                                   const int2* __restrict__ dims, int nb, int LP, float go,
                                                   float* __restrict__ out) {
  constexpr int R = 32;
  __shared__ float s_best[64];
  const int lane = threadIdx.x;
  const int G = 64 / LP;
  const int g = lane / LP, ll = lane - g * LP;
  const int p = blockIdx.x * G + g;
  const bool in_group = g < G && p < nb;
  const int2 dm = in_group ? dims[p] : make_int2(0, 0);
  const int Mp = dm.x, Np = dm.y;
  const int row0 = ll * R;
  const uint32_t* mrow = maskT + (size_t)(in_group ? p : 0) * mask_stride + (size_t)ll * ld;
  DpLane<0, true, R, true> L;
  L.go = go;
  L.ge = go;
  L.Np = Np;
  L.lane = ll;
  uint32_t rv = 0;
  for (int r = 0; r < R; ++r) rv |= (uint32_t)((row0 + r >= 2) && (row0 + r < Mp)) << r;
  L.rowvalid = rv;
  L.w1 = L.w2 = 0;
  L.h1 = L.h2 = DpAbove{0.0f, 0.0f, 0u};
  L.best = 0.0f;
  float qa[R], qb[R], qc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) qa[r] = qb[r] = qc[r] = 0.0f;
  DpAbove pub{0.0f, 0.0f, 0u};
  // steps until every group of the wave is done (wave-uniform bound)
  const int S_end = (int)wave_max_u32(in_group ? (unsigned)(Np + LP - 1) : 0u);
  const bool lane_active = in_group && row0 < Mp;
  auto fetch = [&](int c) -> uint32_t {
    if (!(lane_active && c >= 2 && c < Np)) return 0u;
    return mrow[c] & rv;
  };
  auto recv = [&](const DpAbove& mine) -> DpAbove {
    DpAbove h;
    h.q30 = __shfl_up(mine.q30, 1);
    h.q31 = __shfl_up(mine.q31, 1);
    h.b = (uint32_t)__shfl_up((int)mine.b, 1);
    if (ll == 0) h = DpAbove{0.0f, 0.0f, 0u};  // the group's first rows: nothing above
    return h;
  };
  uint32_t wnext = fetch(-ll);
  for (int s = 0; s < S_end; s += 3) {
    {
      const int c = s - ll;
      const uint32_t w0 = wnext;
      wnext = fetch(c + 1);
      pub = L.step(qa, qb, qc, w0, recv(pub), c);
    }
    if (s + 1 < S_end) {
      const int c = s + 1 - ll;
      const uint32_t w0 = wnext;
      wnext = fetch(c + 1);
      pub = L.step(qc, qa, qb, w0, recv(pub), c);
    }
    if (s + 2 < S_end) {
      const int c = s + 2 - ll;
      const uint32_t w0 = wnext;
      wnext = fetch(c + 1);
      pub = L.step(qb, qc, qa, w0, recv(pub), c);
    }
  }
  // per-group maximum through LDS (groups need not be a power of two wide)
  s_best[lane] = L.best;
  __syncthreads();
  if (in_group && ll == 0) {
    float b = 0.0f;
    for (int k = 0; k < LP; ++k) b = fmaxf(b, s_best[lane + k]);
    out[p] = b;
  }
}

// --------------------------------------------------------------------------------------
// k_crp_dp_pk<ALIGN>: k_crp_dp<ALIGN, true, 32> in packed 16-bit integers. With
// gamma_open == gamma_ext = K/2 (K a small integer, 1 for the reference's 0.5), every score is
// a multiple of 1/2, so 2Q is an exact integer below 4 L: lane l keeps rows (h, h + 16) of a
// column in one u32 (row h low, row h + 16 high) and takes two rows per v_pk_max_u16 /
// v_pk_add_u16 / saturating v_pk_sub_u16 (max(x - K, 0) in one instruction). The predecessor
// rows of pair h are pair h - 1 / h - 2 of the previous columns; pairs 0 and 1 splice in the
// rows handed down by the lane above (v_perm). Bit-identical to the f32 kernel: both compute
// the same exact multiples of 1/2 (the f32 values never round).
// --------------------------------------------------------------------------------------
typedef unsigned short dp_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk16(dp_u16x2 v) { return __builtin_bit_cast(unsigned, v); }
__device__ __forceinline__ dp_u16x2 up16(unsigned v) { return __builtin_bit_cast(dp_u16x2, v); }
__device__ __forceinline__ unsigned pk_max16(unsigned a, unsigned b) { return pk16(__builtin_elementwise_max(up16(a), up16(b))); }
__device__ __forceinline__ unsigned pk_add16(unsigned a, unsigned b) { return pk16(up16(a) + up16(b)); }
__device__ __forceinline__ unsigned pk_sub16(unsigned a, unsigned b) { return pk16(up16(a) - up16(b)); }
__device__ __forceinline__ unsigned pk_subsat16(unsigned a, unsigned b) {
  return pk16(__builtin_elementwise_sub_sat(up16(a), up16(b)));
}

struct DpAbovePk {  // what lane l-1 (or the band above) hands down for one column
  unsigned hq;      // its rows 30 (low half) and 31 (high half), x2 units
  uint32_t b;       // bit0 = C[row 30], bit1 = C[row 31]
};

template <int ALIGN>
struct DpLanePk {
  unsigned K;          // gamma in x2 units, both halves
  int Np;
  uint32_t rz0, rz1;   // AND masks of pairs 0 / 1: rows 0 and 1 of the first band are 0
  uint32_t w1, w2;     // CRP words of columns c-1, c-2
  DpAbovePk h1, h2;    // from above for columns c-1, c-2
  unsigned best;

  __device__ __forceinline__ DpAbovePk step(unsigned (&pn)[16], const unsigned (&p1)[16], const unsigned (&p2)[16],
                                            uint32_t w0, const DpAbovePk& h0, int c) {
    const bool colok = (c >= 2) && (c < Np);
    // rows (-1, 15) and (-2, 14) of column c-1, (-1, 15) of column c-2
    const unsigned a0 = __builtin_amdgcn_perm(p1[15], h1.hq, 0x05040302u);
    const unsigned b0 = __builtin_amdgcn_perm(p1[14], h1.hq, 0x05040100u);
    const unsigned c0 = __builtin_amdgcn_perm(p2[15], h2.hq, 0x05040302u);
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      const unsigned A = h >= 1 ? p1[h - 1] : a0;                  // Q[r-1][c-1]
      unsigned B = h >= 2 ? p1[h - 2] : (h == 1 ? a0 : b0);        // Q[r-2][c-1]
      unsigned Cq = h >= 1 ? p2[h - 1] : c0;                       // Q[r-1][c-2]
      if (ALIGN == 1) {
        const unsigned cb = h >= 1 ? (w0 >> (h - 1)) & 0x10001u : ((h0.b >> 1) & 1u) | (((w0 >> 15) & 1u) << 16);
        B = pk_add16(B, cb << 1);                                  // + C[r-1][c]
        Cq = pk_add16(Cq, ((w1 >> h) & 0x10001u) << 1);            // + C[r][c-1]
      }
      const unsigned mx = pk_max16(pk_max16(A, B), Cq);
      const unsigned m = pk_sub16(0u, (w0 >> h) & 0x10001u);      // 0xffff where C[r][c] = 1
      unsigned v = (m & pk_add16(mx, 0x00020002u)) | (~m & pk_subsat16(mx, K));
      if (h == 0) v &= rz0;
      if (h == 1) v &= rz1;
      v = colok ? v : 0u;
      best = pk_max16(best, v);
      pn[h] = v;
    }
    DpAbovePk out;
    out.hq = __builtin_amdgcn_perm(pn[15], pn[14], 0x07060302u);
    out.b = (w0 >> 30) & 3u;
    h2 = h1;
    h1 = h0;
    w2 = w1;
    w1 = w0;
    return out;
  }
};

template <int ALIGN>
__global__ __launch_bounds__(64) void k_crp_dp_pk(const uint32_t* __restrict__ maskT, int64_t mask_stride, int ld,
                                                  const int2* __restrict__ dims, unsigned K,
                                                  float4* __restrict__ bnd, int64_t bnd_stride,
                                                  float* __restrict__ out) {
  const int p = blockIdx.x;
  const int lane = threadIdx.x;
  const int2 dm = dims[p];
  const int Mp = dm.x, Np = dm.y;
  unsigned best = 0u;
  constexpr int kBand = 64 * 32;
  const int nbands = (Mp + kBand - 1) / kBand;
  for (int band = 0; band < nbands; ++band) {
    const int row0 = band * kBand + lane * 32;
    const uint32_t* mrow = maskT + (size_t)p * mask_stride + (size_t)(row0 >> 5) * ld;
    float4* bout = bnd + (size_t)p * bnd_stride + (size_t)band * ld;
    const float4* bin = bnd + (size_t)p * bnd_stride + (size_t)(band - 1) * ld;
    DpLanePk<ALIGN> L;
    L.K = K * 0x10001u;
    L.Np = Np;
    L.rz0 = row0 == 0 ? 0xffff0000u : 0xffffffffu;
    L.rz1 = L.rz0;
    L.w1 = L.w2 = 0;
    L.h1 = L.h2 = DpAbovePk{0u, 0u};
    L.best = 0u;
    unsigned qa[16], qb[16], qc[16];
#pragma unroll
    for (int h = 0; h < 16; ++h) qa[h] = qb[h] = qc[h] = 0u;
    DpAbovePk pub{0u, 0u};
    const int S_end = Np + 63;
    const bool lane_active = row0 < Mp;
    auto fetch = [&](int c) -> uint32_t { return (lane_active && c >= 0 && c < Np) ? mrow[c] : 0u; };
    auto recv = [&](const DpAbovePk& mine, int c) -> DpAbovePk {
      DpAbovePk h;
      h.hq = (unsigned)__shfl_up((int)mine.hq, 1);
      h.b = (uint32_t)__shfl_up((int)mine.b, 1);
      if (lane == 0) {
        if (band > 0 && c >= 0 && c < Np) {
          const float4 v = bin[c];
          h = DpAbovePk{__builtin_bit_cast(unsigned, v.x), __builtin_bit_cast(unsigned, v.y)};
        } else {
          h = DpAbovePk{0u, 0u};
        }
      }
      return h;
    };
    auto publish = [&](const DpAbovePk& o, int c) {
      if (lane == 63 && band + 1 < nbands && c >= 0 && c < Np)
        bout[c] = make_float4(__builtin_bit_cast(float, o.hq), __builtin_bit_cast(float, o.b), 0.0f, 0.0f);
    };
    uint32_t wnext = fetch(-lane);
    for (int s = 0; s < S_end; s += 3) {
      {
        const int c = s - lane;
        const uint32_t w0 = wnext;
        wnext = fetch(c + 1);
        const DpAbovePk h0 = recv(pub, c);
        pub = L.step(qa, qb, qc, w0, h0, c);
        publish(pub, c);
      }
      if (s + 1 < S_end) {
        const int c = s + 1 - lane;
        const uint32_t w0 = wnext;
        wnext = fetch(c + 1);
        const DpAbovePk h0 = recv(pub, c);
        pub = L.step(qc, qa, qb, w0, h0, c);
        publish(pub, c);
      }
      if (s + 2 < S_end) {
        const int c = s + 2 - lane;
        const uint32_t w0 = wnext;
        wnext = fetch(c + 1);
        const DpAbovePk h0 = recv(pub, c);
        pub = L.step(qb, qc, qa, w0, h0, c);
        publish(pub, c);
      }
    }
    best = pk_max16(best, L.best);
    __threadfence_block();
    __syncthreads();
  }
  const unsigned b2 = max(best & 0xffffu, best >> 16);
  const float r = wave_max(0.5f * (float)b2);
  if (lane == 0) out[p] = r;
}

// Dense (M x N) uint8 CRP <-> strip words maskT[i/32][j] (bit i%32).
__global__ void k_unpack_mask(const uint32_t* __restrict__ maskT, int ld, int M, int N, uint8_t* __restrict__ C) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (j >= N || i >= M) return;
  C[(size_t)i * N + j] = (uint8_t)((maskT[(size_t)(i >> 5) * ld + j] >> (i & 31)) & 1u);
}

__global__ void k_pack_mask(const uint8_t* __restrict__ C, int M, int N, int ld, uint32_t* __restrict__ maskT,
                            int* __restrict__ err) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int strip = blockIdx.y;
  if (j >= N) return;
  uint32_t w = 0;
  int bad = 0;
  for (int r = 0; r < 32; ++r) {
    const int i = strip * 32 + r;
    if (i < M) {
      const uint8_t v = C[(size_t)i * N + j];
      bad |= v > 1;
      w |= (uint32_t)(v & 1) << r;
    }
  }
  maskT[(size_t)strip * ld + j] = w;
  if (bad) atomicOr(err, 1);
}

// --------------------------------------------------------------------------------------
// Host orchestration
// --------------------------------------------------------------------------------------
namespace {

int check_params(const acoss_crp_params* P) {
  if (!P) {
    set_error("params is NULL");
    return ACOSS_E_ARG;
  }
  if (P->m < 1 || P->m > 64 || P->tau < 1 || !(P->kappa >= 0.0f && P->kappa <= 1.0f)) {
    set_error("unsupported params m=%d tau=%d kappa=%g", P->m, P->tau, (double)P->kappa);
    return ACOSS_E_ARG;
  }
  return ACOSS_OK;
}

// Largest R (<=16) whose select block fits: prefer two blocks per CU.
int pick_R(int m, int ld) {
  const size_t lds_max = 160 * 1024;
  for (int R = 16; R >= 1; --R)
    if (2 * select_lds_bytes(R, m, ld) <= lds_max) return R;
  for (int R = 16; R >= 1; --R)
    if (select_lds_bytes(R, m, ld) <= lds_max) return R;
  return 0;
}

template <typename K>
int set_lds(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    ACOSS_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  return ACOSS_OK;
}

struct Stage {
  int R = 0;
  size_t sel_lds = 0, pan_lds = 0;
};

int prepare_stage(int m, int ld, Stage* st) {
  st->R = pick_R(m, ld);
  if (st->R <= 0) {
    set_error("track too long for the LDS stripe (stacked length %d)", ld);
    return ACOSS_E_SHAPE;
  }
  st->sel_lds = select_lds_bytes(st->R, m, ld);
  st->pan_lds = panel_lds_floats(32, m) * sizeof(float);
  int rc;
  if ((rc = set_lds(k_crp_select<false>, st->sel_lds))) return rc;
  if ((rc = set_lds(k_crp_select<true>, st->sel_lds))) return rc;
  if ((rc = set_lds(k_crp_panel<0>, st->pan_lds))) return rc;
  if ((rc = set_lds(k_crp_panel<1>, st->pan_lds))) return rc;
  return ACOSS_OK;
}

template <int ALIGN, int R>
void launch_dp_r(bool eqg, int nb, const uint32_t* maskT, int64_t mstride, int ld, const int2* dims, float go,
                 float ge, float4* bnd, int64_t bstride, float* out, hipStream_t s, int L = 0) {
  const float k2 = 2.0f * go;
  static const bool no_fast = getenv("ACOSS_DP_NOFAST") != nullptr;
  static const bool no_grp = getenv("ACOSS_DP_NOGROUP") != nullptr;
  const int LP = (L + 31) / 32;  // lanes per pair at 32 rows per lane
  if (ALIGN == 0 && eqg && !no_fast && !no_grp && k2 >= 0.0f && k2 <= 1024.0f && k2 == floorf(k2) && L > 0 &&
      LP <= 21) {  // three or more pairs per wave (two per wave measured slower at L ~ 1000)
    const int G = 64 / LP;
    hipLaunchKernelGGL(k_crp_dp_grp, dim3((unsigned)((nb + G - 1) / G)), dim3(64), 0, s, maskT, mstride, ld, dims, nb,
                       LP, go, out);
  } else if (ALIGN == 0 && eqg && !no_fast && k2 >= 0.0f && k2 <= 1024.0f && k2 == floorf(k2))
    hipLaunchKernelGGL((k_crp_dp_fast<R>), dim3(nb), dim3(64), 0, s, maskT, mstride, ld, dims, go, ge,
                       bnd, bstride, out);
  else if (eqg)
    hipLaunchKernelGGL((k_crp_dp<ALIGN, true, R>), dim3(nb), dim3(64), 0, s, maskT, mstride, ld, dims, go, ge, bnd,
                       bstride, out);
  else
    hipLaunchKernelGGL((k_crp_dp<ALIGN, false, R>), dim3(nb), dim3(64), 0, s, maskT, mstride, ld, dims, go, ge, bnd,
                       bstride, out);
}

// The packed 16-bit DP (k_crp_dp_pk) is exact when gamma_open == gamma_ext is a multiple of 1/2
// and every doubled score fits 16 bits: scores grow by at most 2 per column (chen17), so 2Q < 4L.
inline bool dp_packed_ok(bool eqg, int L, float go) {
  static const bool off = getenv("ACOSS_DP_F32") != nullptr;
  const float k2 = 2.0f * go;
  return !off && eqg && L <= 16000 && k2 >= 0.0f && k2 <= 1024.0f && k2 == floorf(k2);
}

// Rows per lane from the batch's longest CRP (L rows): every choice below 2048 rows is one band,
// so the band-boundary buffer (ceil(L / 2048) bands) always suffices.
template <int ALIGN>
void launch_dp(bool eqg, int nb, int L, const uint32_t* maskT, int64_t mstride, int ld, const int2* dims, float go,
               float ge, float4* bnd, int64_t bstride, float* out, hipStream_t s) {
  if (L <= 512)
    launch_dp_r<ALIGN, 8>(eqg, nb, maskT, mstride, ld, dims, go, ge, bnd, bstride, out, s, L);
  else if (L <= 1024)
    launch_dp_r<ALIGN, 16>(eqg, nb, maskT, mstride, ld, dims, go, ge, bnd, bstride, out, s, L);
  else if (ALIGN == 1 && dp_packed_ok(eqg, L, go))
    hipLaunchKernelGGL(k_crp_dp_pk<ALIGN>, dim3(nb), dim3(64), 0, s, maskT, mstride, ld, dims, (unsigned)(2.0f * go), bnd,
                       bstride, out);
  else
    launch_dp_r<ALIGN, 32>(eqg, nb, maskT, mstride, ld, dims, go, ge, bnd, bstride, out, s);
}

// Thresholds of one side: fast m=9 path (crp_select.hip) unless ACOSS_SELECT_GENERIC is set
// or the shape is outside it; otherwise the generic LDS-Gram kernel above.
int run_select(bool trans, const Stage& st, const CrpBatch& B, int nb, int L, int ld, float kappa, float* thr, float* T,
               int64_t thr_stride, hipStream_t s) {
  static const bool generic = getenv("ACOSS_SELECT_GENERIC") != nullptr;
  if (!generic) {
    const int rc = launch_select16(trans, B, nb, L, kappa, thr, T, thr_stride, s);
    if (rc != 1) return rc;
  }
  if (trans)
    hipLaunchKernelGGL(k_crp_select<true>, dim3((L + st.R - 1) / st.R, nb), dim3(256), st.sel_lds, s, B, st.R, ld,
                       kappa, thr, T, thr_stride);
  else
    hipLaunchKernelGGL(k_crp_select<false>, dim3((L + st.R - 1) / st.R, nb), dim3(256), st.sel_lds, s, B, st.R, ld,
                       kappa, thr, T, thr_stride);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

// CRP words: fast m=9 kernel (crp_mask.hip) unless ACOSS_MASK_GENERIC is set.
int run_mask(const Stage& st, const CrpBatch& B, int nb, int L, int nstrips, const float* Tr, const float* Tc,
             int64_t thr_stride, uint32_t* maskT, int64_t mask_stride, int ld, hipStream_t s) {
  static const bool generic = getenv("ACOSS_MASK_GENERIC") != nullptr;
  if (!generic) {
    const int rc = launch_mask9(B, nb, L, Tr, Tc, thr_stride, maskT, mask_stride, ld, s);
    if (rc != 1) return rc;
  }
  hipLaunchKernelGGL(k_crp_panel<0>, dim3((L + kPanelW - 1) / kPanelW, nstrips, nb), dim3(256), st.pan_lds, s, B,
                     Tr, Tc, thr_stride, maskT, mask_stride, ld, (float*)nullptr);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

// Per-track prep into workspace slot 0: prof (n_tracks x 12) | NX (n_tracks x ldn) | and, when
// X2 is requested, the interleaved frame pairs (n_tracks x ldn x 24).
int run_prep(const float* feats, const int64_t* off, const int32_t* len, int n_tracks, int max_len, int m, int tau,
             hipStream_t s, float** prof, float** NX, int* ldn, float** X2 = nullptr) {
  // 32 spare frames per track: the systolic sweep's last (partial) strip reads query frames up
  // to 31 past the track's end (values unused: those rows are never stored)
  *ldn = (int)align_up((size_t)max_len + 32, 64);
  const size_t base = align_up((size_t)n_tracks * 12 + (size_t)n_tracks * (*ldn), 64);
  const size_t bytes = (base + (X2 ? (size_t)n_tracks * (*ldn) * 24 : 0)) * sizeof(float);
  float* ws = static_cast<float*>(workspace(0, bytes));
  if (!ws) return ACOSS_E_HIP;
  *prof = ws;
  *NX = ws + (size_t)n_tracks * 12;
  if (X2) {
    *X2 = ws + base;
    if (max_len > 0) {
      hipLaunchKernelGGL(k_track_pairs, dim3(n_tracks, (max_len + 255) / 256), dim3(256), 0, s, feats, off, len, *ldn,
                         *X2);
      ACOSS_LAUNCH_CHECK();
    }
  }
  hipLaunchKernelGGL(k_track_profile, dim3((n_tracks + 3) / 4), dim3(64), 0, s, feats, off, len, n_tracks, *prof);
  ACOSS_LAUNCH_CHECK();
  if (max_len > 0) {
    hipLaunchKernelGGL(k_track_norms, dim3(n_tracks, (max_len + 255) / 256), dim3(256), 0, s, feats, off, len, m,
                       tau, *ldn, *NX);
    ACOSS_LAUNCH_CHECK();
  }
  return ACOSS_OK;
}

}  // namespace

}  // namespace acoss

using namespace acoss;

extern "C" int acoss_crp_align(const float* feats, const int64_t* track_off, const int32_t* track_len,
                               int32_t n_tracks, int32_t max_len, const int32_t* pairs, int64_t n_pairs,
                               const acoss_crp_params* params, float* qmax_out, float* dmax_out, int32_t* oti_out,
                               void* hip_stream) {
  clear_error();
  int rc = check_params(params);
  if (rc) return rc;
  if (n_pairs < 0 || n_tracks < 0 || max_len < 0) {
    set_error("negative size");
    return ACOSS_E_ARG;
  }
  if (n_pairs == 0) return ACOSS_OK;
  if (!feats || !track_off || !track_len || !pairs) {
    set_error("NULL input pointer");
    return ACOSS_E_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  const int m = params->m, tau = params->tau;
  const int L = stacked_len(max_len, m, tau);
  if (L <= 0) {
    set_error("max_len %d too short for m=%d tau=%d", max_len, m, tau);
    return ACOSS_E_SHAPE;
  }
  const int ld = (int)align_up((size_t)L, 8);  // x16 B = 128 B: band rows never share a cache line
  Stage st;
  if ((rc = prepare_stage(m, ld, &st))) return rc;
  float *prof, *NX;
  int ldn;
  prof_begin(PH_PREP, s);
  float* X2 = nullptr;
  if ((rc = run_prep(feats, track_off, track_len, n_tracks, max_len, m, tau, s, &prof, &NX, &ldn, &X2))) return rc;
  prof_end(PH_PREP, s);

  // per-pair slot: oti, dims, thr/T rows+cols, maskT, band boundary
  const int nstrips = (L + 31) / 32;
  const int nbands = (L + 2047) / 2048;
  const int64_t thr_stride = ld;
  const int64_t mask_stride = (int64_t)nstrips * ld;
  const int64_t bnd_stride = (int64_t)nbands * ld;
  const int64_t yrot_stride = (int64_t)align_up((size_t)max_len * 12, 64);
  // split path (one sweep + two line-select kernels, crp_split.hip) needs 16-bit key planes
  static const char* path_env = getenv("ACOSS_CRP_PATH");
  const bool split = m == 9 && tau == 1 && L <= 4096 && !(path_env && strcmp(path_env, "fused") == 0);
  // row pitch: the selects' 32-element runs end at align32(L); one pad column beyond them takes
  // the sweep's branchless out-of-range stores
  const int ldk = (int)align_up(align_up((size_t)L, 32) + 1, 64);
  const int64_t kstride = split ? (int64_t)align_up((size_t)L, 32) * ldk : 0;  // whole 32-row strips
  // Two-level batching: a DP batch of nb_alloc pairs keeps its CRP words (0.5 MB per pair at
  // 2000 frames) so the one-wave-per-pair DP launch is wide enough; the CRP itself runs in
  // sub-batches whose 16-bit key planes (split path, 16 MB per pair) stay near the 256 MB
  // Infinity Cache.
  const size_t slot = 4 + 8 + 4 * (size_t)thr_stride * 4 + 4 * (size_t)mask_stride + 16 * (size_t)bnd_stride +
                      4 * (size_t)yrot_stride;
  size_t budget = (size_t)16 << 30;  // DP batch scratch: ~25k pairs at 2000 frames in one DP launch
  if (const char* e = getenv("ACOSS_WS_BYTES")) budget = strtoull(e, nullptr, 10);
  int64_t nbmax = (int64_t)(budget / slot);
  if (const char* e = getenv("ACOSS_BATCH_PAIRS")) nbmax = atoll(e);
  if (nbmax < 1) nbmax = 1;
  if (nbmax > 65535) nbmax = 65535;
  const int64_t nb_alloc = n_pairs < nbmax ? n_pairs : nbmax;
  int64_t sub = nb_alloc;
  // split sub-batch scratch per pair: 16-bit prefixes row-major and strip-major (2 + 2 B per
  // cell) and the row-threshold words RT
  const size_t sub_pair = 4 * (size_t)kstride + 4 * (size_t)mask_stride;
  if (split) {
    size_t kbudget = (size_t)1 << 30;  // ~42 pairs at 2000 frames (x2 buffers): fills 256 CUs per launch
    if (const char* e = getenv("ACOSS_KEY_BYTES")) kbudget = strtoull(e, nullptr, 10);
    sub = (int64_t)(kbudget / sub_pair);
    if (sub < 1) sub = 1;
    if (sub > nb_alloc) sub = nb_alloc;
  }
  // split sub-batches alternate between the caller's stream and a side stream, each with its
  // own key-plane buffer, so one sub-batch's selects overlap the next one's sweep
  // read per call: bench.py takes its per-kernel profile with ACOSS_SPLIT_STREAMS=1, so the
  // kernel durations of that call add up to its wall time
  const int nbuf = [] {
    const char* e = getenv("ACOSS_SPLIT_STREAMS");
    const int v = e ? atoi(e) : 2;
    return v < 1 ? 1 : (v > 3 ? 3 : v);
  }();
  const int nkb = nbuf;
  char* ws = static_cast<char*>(workspace(1, slot * nb_alloc + (split ? nkb * sub_pair * sub : 0) + 8192));
  if (!ws) return ACOSS_E_HIP;
  size_t o = 0;
  auto carve = [&](size_t bytes) {
    char* r = ws + o;
    o = align_up(o + bytes, 256);
    return r;
  };
  int32_t* w_oti = reinterpret_cast<int32_t*>(carve(4 * nb_alloc));
  int2* w_dims = reinterpret_cast<int2*>(carve(8 * nb_alloc));
  float* w_thr_r = reinterpret_cast<float*>(carve(4 * thr_stride * nb_alloc));
  float* w_T_r = reinterpret_cast<float*>(carve(4 * thr_stride * nb_alloc));
  float* w_thr_c = reinterpret_cast<float*>(carve(4 * thr_stride * nb_alloc));
  float* w_T_c = reinterpret_cast<float*>(carve(4 * thr_stride * nb_alloc));
  uint32_t* w_mask = reinterpret_cast<uint32_t*>(carve(4 * mask_stride * nb_alloc));
  float4* w_bnd = reinterpret_cast<float4*>(carve(16 * bnd_stride * nb_alloc));
  float* w_yrot = reinterpret_cast<float*>(carve(4 * yrot_stride * nb_alloc));
  void* w_kpl[3] = {nullptr, nullptr, nullptr};
  uint32_t* w_rt[3] = {nullptr, nullptr, nullptr};
  for (int b = 0; split && b < nkb; ++b) {
    w_kpl[b] = static_cast<void*>(carve(4 * (size_t)kstride * sub));
    w_rt[b] = reinterpret_cast<uint32_t*>(carve(4 * (size_t)mask_stride * sub));
  }
  hipStream_t ss[3] = {s, s, s};
  for (int b = 1; split && b < nbuf; ++b) {
    ss[b] = side_stream(b - 1);
    if (!ss[b]) {
      set_error("could not create the side stream");
      return ACOSS_E_HIP;
    }
  }

  const bool eqg = params->gamma_open == params->gamma_ext;
  for (int64_t base = 0; base < n_pairs; base += nb_alloc) {
    const int nb = (int)((n_pairs - base) < nb_alloc ? (n_pairs - base) : nb_alloc);
    const int32_t* pb = pairs + 2 * base;
    prof_begin(PH_OTI, s);
    hipLaunchKernelGGL(k_pair_oti, dim3((nb + 255) / 256), dim3(256), 0, s, prof, track_len, pb, (int64_t)nb,
                       params->oti, m, tau, w_oti, w_dims);
    ACOSS_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_rotate_ref, dim3(16, nb), dim3(256), 0, s, feats, track_off, track_len, pb, w_oti, w_yrot,
                       yrot_stride);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_OTI, s);
    if (split) {
      const int nsb = (int)((nb + sub - 1) / sub);     // sub-batches of this batch
      const int nst = nbuf < nsb ? nbuf : nsb;         // streams they rotate over
      if (nst > 1) {  // the side streams start after this batch's OTI / roll on the caller's stream
        hipEvent_t e0 = sync_event(0);
        ACOSS_HIP_CHECK(hipEventRecord(e0, s));
        for (int q = 1; q < nst; ++q) ACOSS_HIP_CHECK(hipStreamWaitEvent(ss[q], e0, 0));
      }
      int k = 0;
      for (int s0 = 0; s0 < nb; s0 += (int)sub, ++k) {
        const int ns = (nb - s0) < sub ? (nb - s0) : (int)sub;
        const int b = k % nst;
        CrpBatch Bs{feats, X2, track_off, track_len, NX, ldn, pb + 2 * s0, w_oti + s0, w_dims + s0, m, tau,
                    w_yrot + (size_t)s0 * yrot_stride, yrot_stride};
        if ((rc = launch_crp_split(Bs, ns, L, params->kappa, w_kpl[b], ldk, kstride, w_rt[b],
                                   w_thr_r + (size_t)s0 * thr_stride, w_T_r + (size_t)s0 * thr_stride,
                                   w_thr_c + (size_t)s0 * thr_stride, w_T_c + (size_t)s0 * thr_stride, thr_stride,
                                   w_mask + (size_t)s0 * mask_stride, mask_stride, ld, ss[b])))
          return rc;
      }
      for (int q = 1; q < nst; ++q) {  // the DP (caller's stream) needs every sub-batch of every stream
        hipEvent_t e1 = sync_event(q);
        ACOSS_HIP_CHECK(hipEventRecord(e1, ss[q]));
        ACOSS_HIP_CHECK(hipStreamWaitEvent(s, e1, 0));
      }
    } else {
      CrpBatch B{feats, X2, track_off, track_len, NX, ldn, pb, w_oti, w_dims, m, tau, w_yrot, yrot_stride};
      prof_begin(PH_SEL_ROWS, s);
      if ((rc = run_select(false, st, B, nb, L, ld, params->kappa, w_thr_r, w_T_r, thr_stride, s))) return rc;
      prof_end(PH_SEL_ROWS, s);
      prof_begin(PH_SEL_COLS, s);
      if ((rc = run_select(true, st, B, nb, L, ld, params->kappa, w_thr_c, w_T_c, thr_stride, s))) return rc;
      prof_end(PH_SEL_COLS, s);
      prof_begin(PH_MASK, s);
      if ((rc = run_mask(st, B, nb, L, nstrips, w_T_r, w_T_c, thr_stride, w_mask, mask_stride, ld, s))) return rc;
      prof_end(PH_MASK, s);
    }
    if (qmax_out) {
      prof_begin(PH_DP_QMAX, s);
      launch_dp<0>(eqg, nb, L, w_mask, mask_stride, ld, w_dims, params->gamma_open, params->gamma_ext, w_bnd,
                   bnd_stride, qmax_out + base, s);
      ACOSS_LAUNCH_CHECK();
      prof_end(PH_DP_QMAX, s);
    }
    if (dmax_out) {
      prof_begin(PH_DP_DMAX, s);
      launch_dp<1>(eqg, nb, L, w_mask, mask_stride, ld, w_dims, params->gamma_open, params->gamma_ext, w_bnd,
                   bnd_stride, dmax_out + base, s);
      ACOSS_LAUNCH_CHECK();
      prof_end(PH_DP_DMAX, s);
    }
    if (oti_out) ACOSS_HIP_CHECK(hipMemcpyAsync(oti_out + base, w_oti, 4 * nb, hipMemcpyDeviceToDevice, s));
  }
  return ACOSS_OK;
}

extern "C" int acoss_crp_pair(const float* X, int32_t M, const float* Y, int32_t N, const acoss_crp_params* params,
                              float* dist, float* thr_row, float* thr_col, uint8_t* crp, int32_t* oti,
                              void* hip_stream) {
  clear_error();
  int rc = check_params(params);
  if (rc) return rc;
  const int m = params->m, tau = params->tau;
  const int Mp = stacked_len(M, m, tau), Np = stacked_len(N, m, tau);
  if (Mp <= 0 || Np <= 0) {
    set_error("track too short: M=%d N=%d m=%d tau=%d", M, N, m, tau);
    return ACOSS_E_SHAPE;
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  const int L = Mp > Np ? Mp : Np;
  const int ld = (int)align_up((size_t)L, 8);  // x16 B = 128 B: band rows never share a cache line
  Stage st;
  if ((rc = prepare_stage(m, ld, &st))) return rc;
  // packed features + tables in workspace slot 2
  const int nstrips = (Mp + 31) / 32;
  const size_t fbytes = align_up((size_t)(M + N) * 12 * 4, 256);
  const size_t ybytes = align_up((size_t)N * 12 * 4, 256);
  const size_t bytes = fbytes + 256 * 4 + 4 * 4 * (size_t)ld + 4 * (size_t)nstrips * ld + ybytes;
  char* ws = static_cast<char*>(workspace(2, bytes));
  if (!ws) return ACOSS_E_HIP;
  float* f = reinterpret_cast<float*>(ws);
  char* tab = ws + fbytes;
  int64_t* d_off = reinterpret_cast<int64_t*>(tab);
  int32_t* d_len = reinterpret_cast<int32_t*>(tab + 64);
  int32_t* d_pairs = reinterpret_cast<int32_t*>(tab + 128);
  int32_t* d_oti = reinterpret_cast<int32_t*>(tab + 192);
  int2* d_dims = reinterpret_cast<int2*>(tab + 256);
  float* thr_r = reinterpret_cast<float*>(tab + 1024);
  float* T_r = thr_r + ld;
  float* thr_c = T_r + ld;
  float* T_c = thr_c + ld;
  uint32_t* maskT = reinterpret_cast<uint32_t*>(T_c + ld);
  float* yrot = reinterpret_cast<float*>(reinterpret_cast<char*>(maskT) + 4 * (size_t)nstrips * ld);
  yrot = reinterpret_cast<float*>(align_up(reinterpret_cast<uintptr_t>(yrot), 256));
  const int64_t h_off[2] = {0, M};
  const int32_t h_len[2] = {M, N};
  const int32_t h_pairs[2] = {0, 1};
  ACOSS_HIP_CHECK(hipMemcpyAsync(f, X, (size_t)M * 12 * 4, hipMemcpyDeviceToDevice, s));
  ACOSS_HIP_CHECK(hipMemcpyAsync(f + (size_t)M * 12, Y, (size_t)N * 12 * 4, hipMemcpyDeviceToDevice, s));
  ACOSS_HIP_CHECK(hipStreamSynchronize(s));
  ACOSS_HIP_CHECK(hipMemcpy(d_off, h_off, sizeof(h_off), hipMemcpyHostToDevice));
  ACOSS_HIP_CHECK(hipMemcpy(d_len, h_len, sizeof(h_len), hipMemcpyHostToDevice));
  ACOSS_HIP_CHECK(hipMemcpy(d_pairs, h_pairs, sizeof(h_pairs), hipMemcpyHostToDevice));
  float *prof, *NX;
  int ldn;
  if ((rc = run_prep(f, d_off, d_len, 2, M > N ? M : N, m, tau, s, &prof, &NX, &ldn))) return rc;
  hipLaunchKernelGGL(k_pair_oti, dim3(1), dim3(64), 0, s, prof, d_len, d_pairs, (int64_t)1, params->oti, m, tau,
                     d_oti, d_dims);
  ACOSS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_rotate_ref, dim3(16, 1), dim3(256), 0, s, f, d_off, d_len, d_pairs, d_oti, yrot, (int64_t)0);
  ACOSS_LAUNCH_CHECK();
  CrpBatch B{f, nullptr, d_off, d_len, NX, ldn, d_pairs, d_oti, d_dims, m, tau, yrot, 0};
  if ((rc = run_select(false, st, B, 1, L, ld, params->kappa, thr_r, T_r, (int64_t)ld, s))) return rc;
  if ((rc = run_select(true, st, B, 1, L, ld, params->kappa, thr_c, T_c, (int64_t)ld, s))) return rc;
  if (dist) {
    hipLaunchKernelGGL(k_crp_panel<1>, dim3((Np + kPanelW - 1) / kPanelW, nstrips, 1), dim3(256), st.pan_lds, s, B,
                       T_r, T_c, (int64_t)ld, maskT, (int64_t)0, ld, dist);
    ACOSS_LAUNCH_CHECK();
  }
  if (crp) {
    if ((rc = run_mask(st, B, 1, L, nstrips, T_r, T_c, (int64_t)ld, maskT, (int64_t)0, ld, s))) return rc;
    hipLaunchKernelGGL(k_unpack_mask, dim3((Np + 255) / 256, Mp), dim3(256), 0, s, maskT, ld, Mp, Np, crp);
    ACOSS_LAUNCH_CHECK();
  }
  if (thr_row) ACOSS_HIP_CHECK(hipMemcpyAsync(thr_row, thr_r, 4 * (size_t)Mp, hipMemcpyDeviceToDevice, s));
  if (thr_col) ACOSS_HIP_CHECK(hipMemcpyAsync(thr_col, thr_c, 4 * (size_t)Np, hipMemcpyDeviceToDevice, s));
  if (oti) ACOSS_HIP_CHECK(hipMemcpyAsync(oti, d_oti, 4, hipMemcpyDeviceToDevice, s));
  ACOSS_HIP_CHECK(hipStreamSynchronize(s));
  return ACOSS_OK;
}

extern "C" int acoss_align_crp(const uint8_t* crp, int32_t M, int32_t N, int32_t align, float gamma_open,
                               float gamma_ext, float* score_out, void* hip_stream) {
  clear_error();
  if (M < 0 || N < 0 || (align != 0 && align != 1) || !score_out) {
    set_error("bad arguments to acoss_align_crp");
    return ACOSS_E_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  if (M == 0 || N == 0) {
    const float z = 0.0f;
    ACOSS_HIP_CHECK(hipMemcpyAsync(score_out, &z, 4, hipMemcpyHostToDevice, s));
    ACOSS_HIP_CHECK(hipStreamSynchronize(s));
    return ACOSS_OK;
  }
  const int ld = (int)align_up((size_t)N, 8);
  const int nstrips = (M + 31) / 32, nbands = (M + 2047) / 2048;
  const size_t bytes = 256 + 4 * (size_t)nstrips * ld + 16 * (size_t)nbands * ld;
  char* ws = static_cast<char*>(workspace(3, bytes));
  if (!ws) return ACOSS_E_HIP;
  int* d_err = reinterpret_cast<int*>(ws);
  int2* d_dims = reinterpret_cast<int2*>(ws + 64);
  uint32_t* maskT = reinterpret_cast<uint32_t*>(ws + 256);
  float4* bnd = reinterpret_cast<float4*>(ws + 256 + 4 * (size_t)nstrips * ld);
  const int h_hdr[4] = {0, 0, M, N};  // err, pad, dims
  ACOSS_HIP_CHECK(hipMemcpy(d_err, h_hdr, 8, hipMemcpyHostToDevice));
  ACOSS_HIP_CHECK(hipMemcpy(d_dims, h_hdr + 2, 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_pack_mask, dim3((N + 255) / 256, nstrips), dim3(256), 0, s, crp, M, N, ld, maskT, d_err);
  ACOSS_LAUNCH_CHECK();
  const bool eqg = gamma_open == gamma_ext;
  if (align == 0)
    launch_dp<0>(eqg, 1, M, maskT, 0, ld, d_dims, gamma_open, gamma_ext, bnd, 0, score_out, s);
  else
    launch_dp<1>(eqg, 1, M, maskT, 0, ld, d_dims, gamma_open, gamma_ext, bnd, 0, score_out, s);
  ACOSS_LAUNCH_CHECK();
  int h_err = 0;
  ACOSS_HIP_CHECK(hipMemcpyAsync(&h_err, d_err, 4, hipMemcpyDeviceToHost, s));
  ACOSS_HIP_CHECK(hipStreamSynchronize(s));
  if (h_err) {
    set_error("CoverSongSimilarity: non-binary elements found in the input similarity matrix");
    return ACOSS_E_NONBINARY;
  }
  return ACOSS_OK;
}
