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
//                         rounding: parity with the reference is a tolerance, 1e-9 relative in the
//                         tests; with the oracle's canonical order it is bit-exact).
//
// Canonical rounding (oracle/crp_oracle.cpp or_simple_sim): the frame dot <a, roll(b, k)> runs
// over the reference's own bins j = 0..11 paired with the query's bin (j + k) mod 12 (the
// product for j = 0, then an fma chain); frame norms likewise over bins 0..11;
// window sums are sequential adds t = 0..L-1; dist = (sb[j] + sa[i]) - 2 qt.
//
// Fast path (L = 10, the reference's SSLEN; k_simple_diag<K>, K = 5 by default): one 256-thread
// block per pair (2 or 4 pairs per block for short tracks).
// A wave owns 64·K consecutive diagonals o = j - i of the (P x Q) profile matrix, K adjacent
// ones per lane, and walks down the rows: at step x every lane forms G(x, x + o) for its K
// diagonals. The query frame x is wave-uniform (scalar loads); the K reference frames of a lane
// are consecutive columns, so each step needs ONE new frame per lane (one aligned 128-B record)
// and rotates the others (the ring index is static after unrolling by lcm(10, K)). With SH (the
// default for tracks of >= 512 frames, K = 4) that frame is the one lane l + 1 drops this step:
// a DPP wave_shl:1 hands it over and only lane 63's frame, a wave-uniform column, is loaded. Each diagonal keeps its 10 open window
// partials in registers (slot = start step mod 10), so every G is formed once and added into the
// windows in the canonical order. All cells completed at step x lie in row x - 9: one DPP wave
// minimum per step, one LDS atomic per row per wave. Per track: a frame-major query copy with
// the 12 bins stored twice (the OTI pairing is the scalar load at bin offset k) and a reference
// copy of 128-B records (12 bins + 4 pad). The median is a bitonic sort of the row minima in LDS.
#include "common.hpp"

namespace acoss {

namespace {

constexpr int kMaxL = 16;
constexpr int kMaxLen = 4096;  // frames per track (LDS: row minima + reference window norms)
constexpr int kFastL = 10;     // simple_silva.py SSLEN
constexpr int kExt = 24;       // doubles per frame in the query copy (bins 0..11 twice)
constexpr int kRec = 16;       // doubles per frame in the reference copy (bins 0..11 + pad: 128 B)

__device__ __forceinline__ unsigned long long dkey(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_inv(unsigned long long k) {
  const unsigned long long u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __builtin_bit_cast(double, u);
}

// Simple.oti: v[k] = dot(p_a, roll(p_b, k)); argsort(v)[-1] -> last index of the maximum
__device__ int simple_oti_index(const double* pa, const double* pb) {
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
  return best;
}

// Per-track scratch is packed by the tracks' own lengths and only for the tracks the call's pairs
// name: k_simple_mark flags them, k_simple_scan gives each flagged track its frame offset toff[t]
// (lengths rounded up to 8 frames) and the total, which sizes the workspace.
__global__ void k_simple_mark(const int32_t* __restrict__ pairs, int64_t n_pairs, int32_t* __restrict__ used) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n_pairs) {
    used[pairs[2 * p]] = 1;
    used[pairs[2 * p + 1]] = 1;
  }
}

// The MFMA kernel reads the window norms from a padded copy (k_simple_track's wpad): every flagged
// track's norms at woff[t] = toff[t] + kWPad (rank + 1), with kWPad +inf entries before the first
// track and after every track, so its reads past either end of a track need neither a clamped index
// nor a mask (they fall in [-136, Q + 157] around the track; an out-of-range column's +inf is
// exactly the masked value).
constexpr int kWPad = 256;

__global__ __launch_bounds__(1024) void k_simple_scan(const int32_t* __restrict__ len, const int32_t* __restrict__ used,
                                                      int n_tracks, int64_t* __restrict__ toff,
                                                      int64_t* __restrict__ woff, int64_t* __restrict__ total) {
  __shared__ int64_t wsum[16], wcnt[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int per = (n_tracks + 1023) / 1024;
  const int a = min(n_tracks, t * per), b = min(n_tracks, a + per);
  int64_t mine = 0, mcnt = 0;
  for (int u = a; u < b; ++u) {
    mine += used[u] ? (int64_t)align_up((size_t)len[u], 8) : 0;
    mcnt += used[u] ? 1 : 0;
  }
  // inclusive scans of the per-thread sums: within the wave, then across the 16 waves
  int64_t x = mine, c = mcnt;
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t y = __shfl_up(x, d, 64), z = __shfl_up(c, d, 64);
    if (lane >= d) {
      x += y;
      c += z;
    }
  }
  if (lane == 63) {
    wsum[w] = x;
    wcnt[w] = c;
  }
  __syncthreads();
  int64_t before = 0, cbefore = 0;
  for (int v = 0; v < w; ++v) {
    before += wsum[v];
    cbefore += wcnt[v];
  }
  int64_t run = before + x - mine, rank = cbefore + c - mcnt;  // exclusive prefixes of this thread
  for (int u = a; u < b; ++u) {
    toff[u] = used[u] ? run : -1;
    woff[u] = used[u] ? run + kWPad * (rank + 1) : -1;
    run += used[u] ? (int64_t)align_up((size_t)len[u], 8) : 0;
    rank += used[u] ? 1 : 0;
  }
  if (t == 1023) {
    total[0] = run;
    total[1] = rank;
  }
}

__global__ void k_fill_f64(double* __restrict__ x, int64_t n, double v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) x[i] = v;
}

// per flagged track: chroma profile (sum over time, sequential), per-frame squared norms (fma
// chain), the L-window norms of the unrolled track, and (fast path) the frame-major doubled
// query copy ext[x][0..23] and the 128-B reference records rec[x][0..15]
__global__ void k_simple_track(const double* __restrict__ feats, const int64_t* __restrict__ off,
                               const int32_t* __restrict__ len, int n_tracks, int L, double* __restrict__ prof,
                               double* __restrict__ fnorm, double* __restrict__ wnorm, double* __restrict__ ext,
                               double* __restrict__ rec, const int64_t* __restrict__ toff, int copies,
                               double* __restrict__ wpad, const int64_t* __restrict__ woff) {
  const int tr = blockIdx.x;
  if (tr >= n_tracks || toff[tr] < 0) return;
  const double* S = feats + off[tr];
  const int n = len[tr];
  const int t = threadIdx.x;
  const int64_t o = toff[tr];
  if (t < 12) {
    double acc = 0.0;
    for (int x = 0; x < n; ++x) acc = acc + S[(size_t)t * n + x];
    prof[tr * 12 + t] = acc;
  }
  double* E = ext + (size_t)o * kExt;
  double* R = rec + (size_t)o * kRec;
  for (int x = t; x < n; x += blockDim.x) {
    double acc = 0.0;
    for (int d = 0; d < 12; ++d) {
      const double v = S[(size_t)d * n + x];
      acc = d == 0 ? v * v : fma(v, v, acc);
      if (copies) {
        E[(size_t)x * kExt + d] = v;
        E[(size_t)x * kExt + 12 + d] = v;
        R[(size_t)x * kRec + d] = v;
      }
    }
    if (copies)
      for (int d = 12; d < kRec; ++d) R[(size_t)x * kRec + d] = 0.0;
    fnorm[o + x] = acc;
  }
  __syncthreads();
  for (int i = t; i + L <= n; i += blockDim.x) {
    double acc = 0.0;
    for (int u = 0; u < L; ++u) acc = acc + fnorm[o + i + u];
    wnorm[o + i] = acc;
    if (wpad) wpad[woff[tr] + i] = acc;
  }
}

// Generic sslen (1..16): one thread per diagonal, L-deep shift register of G.
__global__ __launch_bounds__(256) void k_simple_pair(const double* __restrict__ feats, const int64_t* __restrict__ off,
                                                     const int32_t* __restrict__ len, const int32_t* __restrict__ pairs,
                                                     const double* __restrict__ prof, const double* __restrict__ wnorm,
                                                     const int64_t* __restrict__ toff, int L, int apply_oti,
                                                     double* __restrict__ score,
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
    const int best = simple_oti_index(prof + ta * 12, prof + tb * 12);
    s_k = apply_oti ? best : 0;
    if (oti_out) oti_out[p] = best;
  }
  if (P <= 0 || Q <= 0) {
    if (t == 0) score[p] = __builtin_nan("");
    return;
  }
  for (int i = t; i < P; i += 256) {
    sa[i] = wnorm[toff[ta] + i];
    mpk[i] = ~0ull;
  }
  __syncthreads();
  const int k = s_k;
  int rowA[12];  // reference bin j pairs with query bin (j + k) mod 12
#pragma unroll
  for (int c = 0; c < 12; ++c) rowA[c] = ((c + k) % 12) * na;
  for (int j = t; j < Q; j += 256) sb[j] = wnorm[toff[tb] + j];  // a roll keeps the norms
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
      double g = A[rowA[0] + x] * B[y];
#pragma unroll
      for (int c = 1; c < 12; ++c) g = fma(A[rowA[c] + x], B[(size_t)c * nb + y], g);
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

// ---- fast path: L = 10, K adjacent diagonals per lane ----

typedef __attribute__((address_space(4))) double CDouble;  // scalar (s_load) path for uniform loads

// v_min_f64 without fmin's NaN canonicalisation (IEEE minNum: a NaN operand yields the other)
__device__ __forceinline__ double vmin_f64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Wave minimum of a double (DPP row_shr 1/2/4/8, row_bcast 15/31; total in lane 63).
__device__ __forceinline__ double wave_min_f64(double v) {
  const unsigned IHI = 0x7ff00000u;  // +inf: lo 0, hi 0x7ff00000
#define ACOSS_MIN_STAGE(CTRL, RM)                                                                     \
  {                                                                                                 \
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);                         \
    const unsigned lo = dpp_u32<CTRL, RM>(0u, (unsigned)u);                                         \
    const unsigned hi = dpp_u32<CTRL, RM>(IHI, (unsigned)(u >> 32));                                \
    v = vmin_f64(v, __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo));               \
  }
  ACOSS_MIN_STAGE(0x111, 0xf)
  ACOSS_MIN_STAGE(0x112, 0xf)
  ACOSS_MIN_STAGE(0x114, 0xf)
  ACOSS_MIN_STAGE(0x118, 0xf)
  ACOSS_MIN_STAGE(0x142, 0xa)
  ACOSS_MIN_STAGE(0x143, 0xc)
#undef ACOSS_MIN_STAGE
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

constexpr int gcd_c(int a, int b) { return b == 0 ? a : gcd_c(b, a % b); }

// Row minima of one unrolled chunk of U steps through LDS (RED = 1): every step stores the lane
// minima m (one row per step) to the wave's rbuf[step][lane]; after the chunk, S = 64 / U lanes
// per row each fold a 16-B aligned segment of that row and ds_min the key (at most S-way).
constexpr int kRbufStride = 72;  // doubles per rbuf row: 64 lanes + pad (+inf) for the segments

// Lane l gets lane l + 1's double; lane 63 keeps `old` (DPP wave_shl:1, bound_ctrl off).
__device__ __forceinline__ double dpp_shl1_f64(double old, double v) {
  const unsigned long long o = __builtin_bit_cast(unsigned long long, old);
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = dpp_u32<0x130, 0xf>((unsigned)o, (unsigned)u);
  const unsigned hi = dpp_u32<0x130, 0xf>((unsigned)(o >> 32), (unsigned)(u >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// SH = 1: a lane's new reference frame is the frame lane l + 1 drops this step (DPP), so the
// wave reads ONE frame per step (lane 63's, a wave-uniform address loaded a step ahead).
template <int K, int RED, int SH = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_simple_diag(const double* __restrict__ ext, const double* __restrict__ rec, const int32_t* __restrict__ len,
                                                     const int32_t* __restrict__ pairs, const double* __restrict__ prof,
                                                     const double* __restrict__ wnorm,
                                                     const int64_t* __restrict__ toff, int n2max,
                                                     int sboff, int slotsz, int rboff, int ppb, int64_t n_pairs,
                                                     int apply_oti, double* __restrict__ score,
                                                     int32_t* __restrict__ oti_out) {
  constexpr int L = kFastL;
  constexpr int U = L * K / gcd_c(L, K);  // unroll: window slots (mod L) and frame ring (mod K) static
  extern __shared__ unsigned long long smem[];
  __shared__ int s_k[4];
  // ppb pairs per block (short tracks: a pair has fewer than 4 diagonal groups); WPP waves each
  const int t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);  // wave: SGPR
  const int WPP = 4 / ppb, slot = wave / WPP, lw = wave % WPP;
  const int nthr = 64 * WPP, tl = t - slot * nthr;
  unsigned long long* mpk = smem + (size_t)slot * slotsz;                // n2max row-minimum keys
  double* sb = reinterpret_cast<double*>(mpk + sboff);                  // reference window norms (rolled)
  const int64_t p = (int64_t)blockIdx.x * ppb + slot;
  const bool active = p < n_pairs;
  const int ta = active ? pairs[2 * p] : 0, tb = active ? pairs[2 * p + 1] : 0;
  const int na = len[ta], nb = len[tb];
  const int P = na - L + 1, Q = nb - L + 1;
  const bool live = active && P > 0 && Q > 0;
  if (active && tl == 0) {
    const int best = simple_oti_index(prof + ta * 12, prof + tb * 12);
    s_k[slot] = apply_oti ? best : 0;
    if (oti_out) oti_out[p] = best;
    if (!live) score[p] = __builtin_nan("");
  }
  __syncthreads();
  const int kq = live ? __builtin_amdgcn_readfirstlane(s_k[slot]) : 0;  // query bin offset of the OTI pairing
  const int64_t oa = live ? toff[ta] : 0, ob = live ? toff[tb] : 0;
  const double* Ea = ext + (size_t)oa * kExt + kq;
  const double* Eb = rec + (size_t)ob * kRec;
  const double* Wa = wnorm + oa;
  // the reference's window norms (a roll keeps them) into LDS
  for (int j = tl; live && j < Q; j += nthr) sb[j] = wnorm[ob + j];
  __syncthreads();
  const int n2 = n2max;
  for (int i = tl; i < n2; i += nthr) mpk[i] = ~0ull;
  constexpr int RS = 64 / U;                  // lanes per row in the chunk reduction
  constexpr int RSEG = ((64 + RS - 1) / RS + 1) / 2 * 2;  // segment length (even: b128 reads)
  static_assert(RS * RSEG <= kRbufStride, "rbuf pad");
  double* rbuf = reinterpret_cast<double*>(smem + rboff) + wave * (U * kRbufStride);
  if (RED) {
    for (int i = lane; i < U * kRbufStride; i += 64) rbuf[i] = __builtin_inf();
  }
  __syncthreads();

  constexpr int DW = 64 * K;  // diagonals per wave group
  const int ND = P + Q - 1;
  const int NG = live ? (ND + DW - 1) / DW : 0;
  const double kInf = __builtin_inf();
  for (int g = lw; g < NG; g += WPP) {
    const int ob = -(P - 1) + g * DW;  // diagonal of lane 0, k = 0
    const int x_lo = max(0, -(ob + DW - 1));
    const int x_hi = min(P - 1, Q - 1 - ob) + L - 1;
    const int xs = x_lo - x_lo % U;
    const int yl = ob + K * lane;  // column of diagonal k at step x: x + yl + k
    double F[K][12];
    double SB[K];
    double part[K][L];
    auto load_frame = [&](int slot, int y) {
      const int yc = min(max(y, 0), nb - 1);
      const double* src = Eb + (size_t)yc * kRec;
#pragma unroll
      for (int c = 0; c < 12; ++c) F[slot][c] = src[c];
      const int cc = y - (L - 1);  // the cell column this frame closes
      SB[slot] = (cc >= 0 && cc < Q) ? sb[cc] : kInf;
    };
#pragma unroll
    for (int k = 0; k < K - 1; ++k) load_frame(k, xs + yl + k);
    double PF[12], PFsb = 0.0;  // SH: lane 63's next frame (wave-uniform column)
    auto load_pf = [&](int y) {
      const int yc = min(max(y, 0), nb - 1);
      const double* src = Eb + (size_t)yc * kRec;
#pragma unroll
      for (int c = 0; c < 12; ++c) PF[c] = src[c];
      const int cc = y - (L - 1);
      PFsb = (cc >= 0 && cc < Q) ? sb[cc] : kInf;
    };
    if (SH) {
      load_frame(K - 1, xs - 1 + yl);  // what lane l - 1 takes over at the first step
      load_pf(xs + ob + 64 * K - 1);
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int s = 0; s < L; ++s) part[k][s] = 0.0;
    for (int x0 = xs; x0 <= x_hi; x0 += U) {
#pragma unroll
      for (int ph = 0; ph < U; ++ph) {
        const int x = x0 + ph;
        if (SH) {
          const int sl = (ph + K - 1) % K;
#pragma unroll
          for (int c = 0; c < 12; ++c) F[sl][c] = dpp_shl1_f64(PF[c], F[sl][c]);
          SB[sl] = dpp_shl1_f64(PFsb, SB[sl]);
          load_pf(x + 1 + ob + 64 * K - 1);
        } else {
          load_frame((ph + K - 1) % K, x + yl + K - 1);
        }
        // wave-uniform query frame and window norm: scalar loads (constant address space)
        const CDouble* Arow = (const CDouble*)(Ea + (size_t)min(x, na - 1) * kExt);
        double a[12];
#pragma unroll
        for (int c = 0; c < 12; ++c) a[c] = Arow[c];
        const int r = x - (L - 1);
        const bool emit = r >= 0 && r < P;
        const double sar = *(const CDouble*)(Wa + min(max(r, 0), P - 1));
        double m = kInf;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int slot = (ph + k) % K;
          double gv = a[0] * F[slot][0];
#pragma unroll
          for (int c = 1; c < 12; ++c) gv = fma(a[c], F[slot][c], gv);
          const int s0 = ph % L;
          part[k][s0] = gv;
#pragma unroll
          for (int j = 1; j < L; ++j) {
            const int s = (ph - j + L) % L;
            part[k][s] = part[k][s] + gv;
          }
          const double qt = part[k][(ph + 1) % L];
          m = vmin_f64(m, fma(-2.0, qt, SB[slot] + sar));
        }
        if (RED) {
          rbuf[ph * kRbufStride + lane] = m;
        } else if (emit) {
          const double wm = wave_min_f64(m);
          if (lane == 0 && wm < kInf) atomicMin(&mpk[r], dkey(wm));
        }
      }
      if (RED) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int ph = lane / RS, seg = lane % RS;
        const int r = x0 + ph - (L - 1);
        if (ph < U && r >= 0 && r < P) {
          const double* src = rbuf + ph * kRbufStride + seg * RSEG;
          double v = src[0];
#pragma unroll 1
          for (int i = 1; i < RSEG; i += 1) v = vmin_f64(v, src[i]);
          if (v < kInf) atomicMin(&mpk[r], dkey(v));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
  __syncthreads();
  // bitonic sort of the n2 keys (pads are ~0 and sort last)
  for (int kk = 2; kk <= n2; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = tl; i < n2; i += nthr) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = mpk[i], b = mpk[ixj];
          const bool up = (i & kk) == 0;
          if ((a > b) == up) {
            mpk[i] = b;
            mpk[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  if (live && tl == 0)
    score[p] = (P % 2) ? dkey_inv(mpk[P / 2]) : 0.5 * (dkey_inv(mpk[P / 2 - 1]) + dkey_inv(mpk[P / 2]));
}

// ---- MFMA path: L = 10; the frame dots on v_mfma_f64_16x16x4_f64, the windows on the VALU ----
// A wave owns DW = 64 * KM consecutive diagonals (KM adjacent ones per lane) and walks the rows in
// blocks of 16 steps. Per block the 16 x (DW + 16) parallelogram of frame dots G(x, y) it needs is
// computed as DW / 16 + 1 tiles of 16 x 16 by three chained MFMAs each (K = 12 bins in chunks of 4:
// measured equal to the sequential fma chain, profiles/r05/mfma_probe; the chain starts from -0,
// so a zero first product keeps its sign exactly as the canonical first product does) and staged
// in LDS by (step, diagonal); then each step adds its lane's KM dots into the open windows (a shift
// register per diagonal: W[a] = the a most recent dots, so the completed window W[9] + g is the
// sequential sum in canonical order). The MFMA tiles of block b + 1 are issued between block b's
// steps (G is free once those steps' dots are read), and the 16 steps' lane minima are reduced
// over the wave in registers (permlane32 / permlane16 swaps, then DPP: each 4-lane quad ends with
// one step's row minimum) and merged into the pair's row-minimum keys by one global atomic per row.
// What this removes from the VALU: the 12 fma of every dot and the per-step frame hand-over (the
// K = 4 kernel's 26 DPP moves), about half of its instructions per cell. Measured steps:
// profiles/r06/simple_mfma/README.txt.

// f64 lane exchanges for the step-minimum reduce-scatter of k_simple_mfma (two 32-bit halves each)
__device__ __forceinline__ void swap32_f64(double& x, double& y) {  // x' = [x_lo, y_lo], y' = [x_hi, y_hi]
  const unsigned long long ux = __builtin_bit_cast(unsigned long long, x), uy = __builtin_bit_cast(unsigned long long, y);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ux, (unsigned)uy, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ux >> 32), (unsigned)(uy >> 32), false, false);
  x = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi[0] << 32) | (unsigned)lo[0]);
  y = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi[1] << 32) | (unsigned)lo[1]);
}
__device__ __forceinline__ void swap16_f64(double& x, double& y) {  // x' = rows [x0 y0 x2 y2], y' = [x1 y1 x3 y3]
  const unsigned long long ux = __builtin_bit_cast(unsigned long long, x), uy = __builtin_bit_cast(unsigned long long, y);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ux, (unsigned)uy, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ux >> 32), (unsigned)(uy >> 32), false, false);
  x = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi[0] << 32) | (unsigned)lo[0]);
  y = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi[1] << 32) | (unsigned)lo[1]);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {  // every lane reads its DPP source (full masks)
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = dpp_u32<CTRL>(0u, (unsigned)u), hi = dpp_u32<CTRL>(0u, (unsigned)(u >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// Pair (x, y) across lanes l and l ^ D (D = 8 or 4, within 16-lane rows): lanes with bit D clear keep
// min(x, x from l ^ D), the others min(y, y from l ^ D).
template <int D>
__device__ __forceinline__ double xpair_min(double x, double y, int lane) {
  const bool hi = (lane & D) != 0;
  const double send = hi ? x : y, keep = hi ? y : x;
  double recv;
  if constexpr (D == 8) {
    recv = dpp_f64<0x128>(send);  // row_ror:8 = lane ^ 8 within the row
  } else {
    const double from_up = dpp_f64<0x12C>(send);   // row_ror:12: lane l reads l + 4
    const double from_down = dpp_f64<0x124>(send); // row_ror:4: lane l reads l - 4
    recv = hi ? from_down : from_up;
  }
  return vmin_f64(keep, recv);
}
constexpr int kKM = 2;                   // diagonals per lane
constexpr int kDW = 64 * kKM;            // diagonals per wave
constexpr int kGT = kDW / 16 + 1;        // 16 x 16 tiles per 16-step block
constexpr int kGS = kDW + 17;            // LDS row stride in doubles: (kGS - 1) * 2 = 32 mod 64 banks
typedef double f64x4m __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_simple_mfma(
    const double* __restrict__ ext, const double* __restrict__ rec, const int32_t* __restrict__ len,
    const int32_t* __restrict__ pairs, const double* __restrict__ prof, const double* __restrict__ wpad,
    const int64_t* __restrict__ woff, const int64_t* __restrict__ toff, int n2max, int64_t n_pairs, int apply_oti,
    unsigned long long* __restrict__ mpk_g, double* __restrict__ score, int32_t* __restrict__ oti_out) {
  constexpr int L = kFastL;
  extern __shared__ double gsm[];  // 4 waves x 16 x kGS doubles; reused for the final sort
  __shared__ int s_k;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t p = blockIdx.x;
  if (p >= n_pairs) return;  // whole block
  const int ta = pairs[2 * p], tb = pairs[2 * p + 1];
  const int na = len[ta], nb = len[tb];
  const int P = na - L + 1, Q = nb - L + 1;
  const bool live = P > 0 && Q > 0;
  unsigned long long* mpk = mpk_g + (size_t)blockIdx.x * n2max;  // this launch's pair slot
  if (t == 0) {
    const int best = simple_oti_index(prof + ta * 12, prof + tb * 12);
    s_k = apply_oti ? best : 0;
    if (oti_out) oti_out[p] = best;
    if (!live) score[p] = __builtin_nan("");
  }
  for (int i = t; i < n2max; i += 256) mpk[i] = ~0ull;
  __threadfence();
  __syncthreads();
  if (!live) return;  // whole block (uniform)
  const int kq = __builtin_amdgcn_readfirstlane(s_k);
  const int64_t oa = toff[ta], ob0 = toff[tb];
  const double* Ea = ext + (size_t)oa * kExt + kq;  // query bin (j + kq) mod 12 at offset j
  const double* Rb = rec + (size_t)ob0 * kRec;
  const double* Wa = wpad + woff[ta];  // padded with +inf on both sides (kWPad)
  const double* Wb = wpad + woff[tb];
  double* G = gsm + (size_t)wave * 16 * kGS;
  const int ND = P + Q - 1;
  const int NG = (ND + kDW - 1) / kDW;
  const double kInf = __builtin_inf();
  const int li = lane & 15, lk = lane >> 4;  // MFMA operand row / k index
  for (int g = wave; g < NG; g += 4) {
    const int ob = -(P - 1) + g * kDW;  // diagonal of lane 0, k = 0
    const int x_lo = max(0, -(ob + kDW - 1));
    const int x_hi = min(P - 1, Q - 1 - ob) + L - 1;
    const int yl = ob + kKM * lane;     // column of diagonal k at step x: x + yl + k
    double W[kKM][L];                    // W[k][a]: sum of the a most recent dots (a = 1..9)
#pragma unroll
    for (int k = 0; k < kKM; ++k)
#pragma unroll
      for (int a = 0; a < L; ++a) W[k][a] = 0.0;
    // MFMA operands of a 16-step block: the query rows (A) and every tile's reference columns (B).
    // Block b + 1's are loaded while block b's steps run (software pipelined: their latency hides
    // behind the VALU work of 16 steps).
    // Block b + 1's tile t covers block b's tile t + 1 columns (both advance by 16), so a block
    // shifts the B operands down one tile and loads only its last tile: 3 loads of 64 lanes per
    // block instead of 27 (the per-tile loads of 16 records each kept the L1 busy).
    double a0, a1, a2, bv[kGT][3];
    auto load_a = [&](int xb) {
      const double* ar = Ea + (size_t)min(xb + li, na - 1) * kExt + lk;
      a0 = ar[0];
      a1 = ar[4];
      a2 = ar[8];
    };
    auto load_b = [&](int xb, int tt) {
      const int col = min(max(xb + ob + 16 * tt + li, 0), nb - 1);
      const double* br = Rb + (size_t)col * kRec + lk;
      bv[tt][0] = br[0];
      bv[tt][1] = br[4];
      bv[tt][2] = br[8];
    };
    load_a(x_lo);
#pragma unroll
    for (int tt = 0; tt < kGT; ++tt) load_b(x_lo, tt);
    // Producer / consumer overlapped: block b's steps issue block b + 1's MFMA tiles (tile t at step
    // kP0 + t, its four results stored to G one step later; G is free once the steps' dots are
    // read), and the step minima are reduced in registers (a permlane32 / permlane16 /
    // DPP reduce-scatter folded into the steps), so G holds nothing else. Operands: a / bv hold
    // block b + 1's (a from an, loaded a block ahead); after tile 8 the B tiles shift down one
    // and the last tile of block b + 2 is loaded.
    auto store_tile = [&](const f64x4m& acc, int tt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int s = lk + 4 * r;
        const int d = 16 * tt + li - s;
        if (tt == 0 || tt == kGT - 1)
          G[s * kGS + ((d >= 0 && d < kDW) ? d : kDW)] = acc[r];
        else
          G[(kGS - 1) * s + li + 16 * tt] = acc[r];
      }
    };
    // block 0's dots, then block 1's operands
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the previous group's reads of G are done
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int tt = 0; tt < kGT; ++tt) {
      f64x4m acc = {-0.0, -0.0, -0.0, -0.0};
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bv[tt][0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bv[tt][1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, bv[tt][2], acc, 0, 0, 0);
      store_tile(acc, tt);
    }
    load_a(x_lo + 16);
#pragma unroll
    for (int tt = 0; tt < kGT - 1; ++tt)
#pragma unroll
      for (int c = 0; c < 3; ++c) bv[tt][c] = bv[tt + 1][c];
    load_b(x_lo + 16, kGT - 1);
    // the block's reference window norms (+inf past the track's ends, from the padded copy). Register
    // q is reloaded with the next block's column once step q has used it (16 steps ahead of its use)
    double sbv[16 + kKM - 1];
#pragma unroll
    for (int q = 0; q < 16 + kKM - 1; ++q) sbv[q] = Wb[x_lo - (L - 1) + yl + q];
    double san = Wa[x_lo + (lane & 15) - (L - 1)];
    for (int x0 = x_lo; x0 <= x_hi; x0 += 16) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // this block's dots are in G
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int send = min(16, x_hi - x0 + 1);
      const int i0 = x0 - (L - 1) + yl;
      const double sa_l = san;
      san = Wa[x0 + 16 + (lane & 15) - (L - 1)];
      // the dots of steps 0..7 now, of steps 8..15 at step kP0 (before the first store into G:
      // LDS ops of one wave run in order), so only half of them are live through the first steps
      constexpr int kP0 = 16 - kGT - 1;  // step of block b + 1's tile 0 (its last tile stored at step 15)
      double gall[16][kKM];
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int k = 0; k < kKM; ++k) gall[s][k] = G[s * kGS + kKM * lane + k];
      f64x4m acc[kGT];
      double mv[16], ra[8], rb[4], rc[2];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (s == kP0) {
#pragma unroll
          for (int s2 = 8; s2 < 16; ++s2)
#pragma unroll
            for (int k = 0; k < kKM; ++k) gall[s2][k] = G[s2 * kGS + kKM * lane + k];
        }
        const int tt = s - kP0;  // block b + 1's tile tt at step kP0 + tt
        if (tt >= 0 && tt < kGT) {
          acc[tt] = f64x4m{-0.0, -0.0, -0.0, -0.0};
          acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bv[tt][0], acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bv[tt][1], acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, bv[tt][2], acc[tt], 0, 0, 0);
        }
        if (tt == kGT - 1) {  // every tile issued: block b + 2's operands (B shifted, fresh A and last tile)
          load_a(x0 + 32);
#pragma unroll
          for (int tt = 0; tt < kGT - 1; ++tt)
#pragma unroll
            for (int c = 0; c < 3; ++c) bv[tt][c] = bv[tt + 1][c];
          load_b(x0 + 32, kGT - 1);
        }
        const double sar = __builtin_bit_cast(double,
            ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(unsigned long long, sa_l) >> 32), s) << 32) |
            (unsigned)__builtin_amdgcn_readlane((int)(unsigned)__builtin_bit_cast(unsigned long long, sa_l), s));
        double m = kInf;
#pragma unroll
        for (int k = 0; k < kKM; ++k) {
          const double qt = W[k][L - 1] + gall[s][k];
          m = vmin_f64(m, fma(-2.0, qt, sbv[s + k] + sar));
        }
#pragma unroll
        for (int k = 0; k < kKM; ++k) {
#pragma unroll
          for (int a = L - 1; a >= 2; --a) W[k][a] = W[k][a - 1] + gall[s][k];
          W[k][1] = gall[s][k];
        }
        sbv[s] = Wb[i0 + 16 + s];  // the next block's column s
        if (s == 15) sbv[16] = Wb[i0 + 32];
        // reduce-scatter of the 16 step minima over the 64 lanes, as the steps complete
        mv[s] = m;
        if (s & 1) {  // lanes l, l ^ 32: lanes < 32 keep step s - 1, the others step s
          double x = mv[s - 1], y = mv[s];
          swap32_f64(x, y);
          ra[s >> 1] = vmin_f64(x, y);
        }
        if ((s & 3) == 3) {  // lanes l, l ^ 16
          double x = ra[(s >> 1) - 1], y = ra[s >> 1];
          swap16_f64(x, y);
          rb[s >> 2] = vmin_f64(x, y);
        }
        if ((s & 7) == 7) rc[s >> 3] = xpair_min<8>(rb[(s >> 2) - 1], rb[s >> 2], lane);  // lanes l, l ^ 8
        if (tt >= 1 && tt <= kGT) store_tile(acc[tt - 1], tt - 1);  // a step after its MFMAs (their latency)
        __builtin_amdgcn_sched_barrier(0);    // one step per scheduling region: no tile's MFMAs hoisted
      }
      double v = xpair_min<4>(rc[0], rc[1], lane);  // lanes l, l ^ 4
      v = vmin_f64(v, dpp_f64<0x4E>(v));               // quad_perm [2,3,0,1]: l ^ 2
      v = vmin_f64(v, dpp_f64<0xB1>(v));               // quad_perm [1,0,3,2]: l ^ 1
      // lane l now holds the minimum of step 8 b2 + 4 b3 + 2 b4 + b5 (bi = bit i of l)
      const int step = 8 * ((lane >> 2) & 1) + 4 * ((lane >> 3) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 5) & 1);
      const int r = x0 + step - (L - 1);
      if ((lane & 3) == 0 && step < send && r >= 0 && r < P && v < kInf) atomicMin(&mpk[r], dkey(v));
    }
  }
  __threadfence();
  __syncthreads();  // every wave's atomics complete
  // the row-minimum keys into LDS, then the bitonic sort and the median as k_simple_diag
  unsigned long long* sk = reinterpret_cast<unsigned long long*>(gsm);
  for (int i = t; i < n2max; i += 256) sk[i] = __hip_atomic_load(&mpk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  for (int kk = 2; kk <= n2max; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = t; i < n2max; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = sk[i], b = sk[ixj];
          const bool up = (i & kk) == 0;
          if ((a > b) == up) {
            sk[i] = b;
            sk[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  if (t == 0) score[p] = (P % 2) ? dkey_inv(sk[P / 2]) : 0.5 * (dkey_inv(sk[P / 2 - 1]) + dkey_inv(sk[P / 2]));
}

int pow2_at_least(int v) {
  int p = 2;
  while (p < v) p <<= 1;
  return p;
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
  // kernel choice first: the per-track query / reference copies exist only for the fast path
  const char* kenv = getenv("ACOSS_SIMPLE_K");
  // K = 4 with DPP frame passing for long tracks (2000 frames: 133.5k pairs/s vs 101.3k for K = 5
  // loading every frame), K = 5 for short ones (200 frames: 5.27M vs 5.11M); an override other
  // than 2, 4 or 5 is ignored
  int kdiag = max_len >= 512 ? 4 : 5;
  if (kenv) {
    const int v = atoi(kenv);
    if (v == 2 || v == 4 || v == 5) kdiag = v;
  }
  const bool fast = sslen == kFastL;
  const char* senv = getenv("ACOSS_SIMPLE_SH");
  const int sh = senv ? atoi(senv) : 1;
  // per-track tables (workspace slot 8): prof | toff | used | total; slot 13: fnorm, wnorm and, on
  // the fast path, ext and rec, each packed by toff (the call's tracks only, at their own lengths:
  // 336 B per frame on the fast path, 16 B otherwise)
  const size_t prof_bytes = align_up((size_t)n_tracks * 12 * 8, 256);
  const size_t toff_bytes = align_up((size_t)n_tracks * 8, 256);
  const size_t used_bytes = align_up((size_t)n_tracks * 4, 256);
  // the MFMA kernel (frame dots on v_mfma_f64_16x16x4_f64), bit-identical to the VALU kernels: the
  // default for tracks of >= 256 frames (the VALU kernels pack several short pairs per block:
  // 200 frames 6.8M vs 5.5M pairs/s; profiles/r06/simple_mfma/); ACOSS_SIMPLE_MFMA=0 / 1 forces either
  const char* menv = getenv("ACOSS_SIMPLE_MFMA");
  const bool mfma = fast && (menv ? menv[0] == '1' : max_len >= 256);
  const size_t head = prof_bytes + 2 * toff_bytes + used_bytes + 256;
  char* hd = static_cast<char*>(workspace(8, head));
  if (!hd) return ACOSS_E_HIP;
  double* prof = reinterpret_cast<double*>(hd);
  int64_t* toff = reinterpret_cast<int64_t*>(hd + prof_bytes);
  int64_t* woff = reinterpret_cast<int64_t*>(hd + prof_bytes + toff_bytes);
  int32_t* used = reinterpret_cast<int32_t*>(hd + prof_bytes + 2 * toff_bytes);
  int64_t* d_total = reinterpret_cast<int64_t*>(hd + prof_bytes + 2 * toff_bytes + used_bytes);
  ACOSS_HIP_CHECK(hipMemsetAsync(used, 0, used_bytes, s));
  hipLaunchKernelGGL(k_simple_mark, dim3((unsigned)((n_pairs + 255) / 256)), dim3(256), 0, s, pairs, n_pairs, used);
  ACOSS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_simple_scan, dim3(1), dim3(1024), 0, s, track_len, used, n_tracks, toff, woff, d_total);
  ACOSS_LAUNCH_CHECK();
  int64_t tot[2] = {0, 0};  // frames, flagged tracks
  ACOSS_HIP_CHECK(hipMemcpyAsync(tot, d_total, 16, hipMemcpyDeviceToHost, s));
  ACOSS_HIP_CHECK(hipStreamSynchronize(s));
  const int64_t frames = tot[0];
  const size_t vec_bytes = align_up((size_t)std::max<int64_t>(frames, 8) * 8, 256);
  const int64_t wpad_n = mfma ? frames + (int64_t)kWPad * (tot[1] + 1) : 0;
  const size_t wpad_bytes = align_up((size_t)wpad_n * 8, 256);
  const size_t bytes = 2 * vec_bytes + (fast ? vec_bytes * (kExt + kRec) : 0) + wpad_bytes;
  char* ws = static_cast<char*>(workspace(13, bytes));
  if (!ws) return ACOSS_E_HIP;
  double* fnorm = reinterpret_cast<double*>(ws);
  double* wnorm = reinterpret_cast<double*>(ws + vec_bytes);
  double* ext = reinterpret_cast<double*>(ws + 2 * vec_bytes);
  double* rec = reinterpret_cast<double*>(ws + 2 * vec_bytes + vec_bytes * kExt);
  double* wpad = mfma ? reinterpret_cast<double*>(ws + 2 * vec_bytes + (fast ? vec_bytes * (kExt + kRec) : 0)) : nullptr;
  if (mfma) {
    hipLaunchKernelGGL(k_fill_f64, dim3((unsigned)std::min<int64_t>((wpad_n + 255) / 256, 4096)), dim3(256), 0, s, wpad,
                       wpad_n, __builtin_inf());
    ACOSS_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_simple_track, dim3(n_tracks), dim3(256), 0, s, feats, track_off, track_len, n_tracks, sslen,
                     prof, fnorm, wnorm, ext, rec, toff, fast ? 1 : 0, wpad, woff);
  ACOSS_LAUNCH_CHECK();
  const int n2max = pow2_at_least(max(max_len - kFastL + 1, 2));
  const int sboff = n2max;
  const int slotsz = sboff + (int)align_up((size_t)max_len, 2);
  const int U = kdiag == 4 ? 20 : 10;  // lcm(10, K)
  // pairs per block: a block's 4 waves stay busy when a pair has fewer than 4 diagonal groups
  const int ngmax = (2 * max(max_len - kFastL + 1, 1) - 1 + 64 * kdiag - 1) / (64 * kdiag);
  // a pair with at most 2 groups goes to ONE wave (it walks both: no wave of the block idles
  // while its partner finishes the longer group; 200 frames: 6.02M vs 4.95M pairs/s with 2 waves)
  // pairs of up to 8 groups (tracks up to ~1,030 frames, Da-TACOS lengths) two per block, two
  // waves each (500 frames: +6-9 %; 2,000 frames: -14 %, one pair per block stays there;
  // profiles/r05/simple_k/)
  const char* penv = getenv("ACOSS_SIMPLE_PPB");
  int ppb = penv ? atoi(penv) : (ngmax <= 2 ? 4 : (ngmax <= 8 ? 2 : 1));
  if (ppb != 1 && ppb != 2 && ppb != 4) ppb = 1;
  while (ppb > 1 && (size_t)ppb * (n2max + align_up((size_t)max_len, 2)) * 8 > 96 * 1024) ppb /= 2;
  // row minima through LDS chunks for packed short pairs, per-step DPP minima for long ones
  // (measured: 200 frames 5.85M vs 5.58M pairs/s, 2000 frames 48.0k vs 51.0k); the K = 5 and the
  // frame-passing kernels always take the DPP minima, so they reserve no reduction buffer
  const char* renv = getenv("ACOSS_SIMPLE_RED");
  const bool red_kernel = !(kdiag == 5 || (kdiag == 4 && sh));
  const int red = red_kernel ? (renv ? atoi(renv) : (ppb > 1 ? 1 : 0)) : 0;
  const int rboff = ppb * slotsz;
  const size_t lds = ((size_t)rboff + (red ? (size_t)4 * U * kRbufStride : 0)) * 8;
  if (mfma) {
    // one block per pair; the pair's row-minimum keys in a global slot of its own (n2max keys),
    // so a launch takes at most 256 MB of them
    const int64_t per = std::max<int64_t>(1, ((int64_t)256 << 20) / ((int64_t)n2max * 8));
    const size_t mlds = (size_t)4 * 16 * kGS * 8;
    unsigned long long* mpk_g =
        static_cast<unsigned long long*>(workspace(16, (size_t)std::min<int64_t>(per, n_pairs) * n2max * 8));
    if (!mpk_g) return ACOSS_E_HIP;
    ACOSS_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_simple_mfma),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlds));
    for (int64_t p0 = 0; p0 < n_pairs; p0 += per) {
      const int64_t np = std::min<int64_t>(n_pairs - p0, per);
      hipLaunchKernelGGL(k_simple_mfma, dim3((unsigned)np), dim3(256), mlds, s, ext, rec, track_len, pairs + 2 * p0,
                         prof, wpad, woff, toff, n2max, np, apply_oti, mpk_g, score_out + p0,
                         oti_out ? oti_out + p0 : nullptr);
      ACOSS_LAUNCH_CHECK();
    }
    prof_end(PH_SIMPLE, s);
    return ACOSS_OK;
  }
  for (int64_t p0 = 0; p0 < n_pairs; p0 += (int64_t)ppb << 20) {
    const int64_t np = std::min<int64_t>(n_pairs - p0, (int64_t)ppb << 20);
    const int32_t* pp = pairs + 2 * p0;
    double* so = score_out + p0;
    int32_t* oo = oti_out ? oti_out + p0 : nullptr;
    if (fast) {
      auto kern = (kdiag == 4 && sh) ? k_simple_diag<4, 0, 1>
                  : kdiag == 5 ? k_simple_diag<5, 0>
                  : kdiag == 4 ? (red ? k_simple_diag<4, 1> : k_simple_diag<4, 0>)
                               : (red ? k_simple_diag<2, 1> : k_simple_diag<2, 0>);
      if (lds > 64 * 1024)
        ACOSS_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(kern, dim3((unsigned)((np + ppb - 1) / ppb)), dim3(256), lds, s, ext, rec, track_len, pp, prof,
                         wnorm, toff, n2max, sboff, slotsz, rboff, ppb, np, apply_oti, so, oo);
    } else {
      hipLaunchKernelGGL(k_simple_pair, dim3((unsigned)np), dim3(256), 0, s, feats, track_off, track_len, pp, prof,
                         wnorm, toff, sslen, apply_oti, so, oo);
    }
    ACOSS_LAUNCH_CHECK();
  }
  prof_end(PH_SIMPLE, s);
  return ACOSS_OK;
}
