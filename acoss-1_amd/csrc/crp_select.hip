// crp_select.hip — per-row / per-column percentile thresholds of the CRP (fast path, m = 9).
//
// Replaces, inside essentia ChromaCrossSimilarity (called at acoss/algorithms/
// rqa_serra09.py:60-66), the all-pairs stacked distance + percentile(row / column, 9.5) steps.
// Bit-identical to the canonical arithmetic of oracle/crp_oracle.cpp.
//
// One 256-thread block owns a stripe of R = 16 "own" stacked frames (rows of the CRP for the
// query pass, columns for the TRANS pass) and sweeps the other song in parallelogram panels:
//  * thread t walks ONE diagonal (row r, column j0+t+r): at step k it computes the 12-term
//    fmaf chain G[k][j0+t+k] from the own frame (wave-uniform -> scalar loads, SGPR operands)
//    and the inner frame staged in LDS (3 ds_read_b128, conflict-free), keeps the last 9 G
//    values in registers and emits the 9-tap window sum of cell r = k-8 — no Gram matrix in
//    LDS, no per-cell LDS round trip;
//  * each cell's squared distance key (f32 bits, >= 0) is stored as its HIGH 16 BITS in an
//    LDS stripe (R x N' x 2 B = 62 KB at N' = 1991), which keeps two blocks per CU;
//  * after the sweep every wave selects its rows independently (no block barriers): a
//    512-bin histogram of (key16 - min) gives the exact 16-bit prefix of the two order
//    statistics; the few cells sharing that prefix are recomputed exactly (108 fmaf) and
//    ranked among themselves. The percentile is interpolated in distance units and turned
//    into a squared-domain threshold (sq_threshold) for the mask kernel.
#include <cstdlib>

#include "crp_internal.hpp"

namespace acoss {

namespace {

constexpr int kR = 16;                           // stripe rows per block
constexpr int kW = 256;                          // diagonals (= threads) per panel
constexpr int kMS = 9;                           // frameStackSize of the fast path
constexpr int kYRows = kW + kR + kMS - 2;        // 279 inner frames staged per panel
constexpr int kNRows = kW + kR;                  // 272 inner norms staged per panel

struct SelCtx {
  const float* own;    // own frames (query, or the OTI-rolled reference in the TRANS pass)
  const float* inner;  // inner frames (rolled reference, or the query in the TRANS pass)
  int n_own_f, n_in_f; // frame counts
  int tau;
  const float* Nown;   // stacked norms of own / inner track
  const float* Nin;
  int i0, rows, n_in_s;
  int ld16;
};

// own frame (i0 + kk): wave-uniform address through the constant address space -> s_load.
__device__ __forceinline__ void load_own(const SelCtx& C, int srow, float (&x)[12]) {
  int f = srow * C.tau;
  f = f < C.n_own_f ? f : C.n_own_f - 1;  // rows past the end only feed invalid cells
  const float* base = C.own + (size_t)f * 12;
  asm volatile("" : "+s"(base));  // keep the load in the loop: 24 rows x 12 SGPRs do not fit
  const cfloat4* p = (const cfloat4*)base;
  const f32x4 a = p[0], b = p[1], c = p[2];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w;
}

// Same load for a caller whose row index is not provably uniform to the compiler (a
// non-inlined function): the address is made uniform with readfirstlane.
__device__ __forceinline__ void load_own_rfl(const SelCtx& C, int srow, float (&x)[12]) {
  int f = srow * C.tau;
  f = f < C.n_own_f ? f : C.n_own_f - 1;
  const uintptr_t a = reinterpret_cast<uintptr_t>(C.own + (size_t)f * 12);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const cfloat4* p = (const cfloat4*)(((uintptr_t)hi << 32) | lo);
  const f32x4 u = p[0], v = p[1], w = p[2];
  x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
  x[4] = v.x; x[5] = v.y; x[6] = v.z; x[7] = v.w;
  x[8] = w.x; x[9] = w.y; x[10] = w.z; x[11] = w.w;
}

template <bool TRANS>
__device__ __forceinline__ float make_key(float nown, float nin, float dot) {
  const float d2 = TRANS ? (nin - 2.0f * dot) + nown : (nown - 2.0f * dot) + nin;
  return d2 > 0.0f ? d2 : 0.0f;
}

// Exact key of cell (own stacked row i, inner stacked column j): same op sequence as the
// panel sweep (used only for the few candidates of the select). Own frames: wave-uniform
// scalar loads; inner frames: 27 float4 loads issued up front.
template <bool TRANS>
__device__ __noinline__ unsigned full_key(const SelCtx& C, int i, int j, bool active) {
  f32x4 y[kMS * 3];
  if (active) {
#pragma unroll
    for (int u = 0; u < kMS; ++u) {
      const f32x4* yp = reinterpret_cast<const f32x4*>(C.inner + (size_t)((j + u) * C.tau) * 12);
      y[3 * u] = yp[0];
      y[3 * u + 1] = yp[1];
      y[3 * u + 2] = yp[2];
    }
  }
  float dot = 0.0f;
#pragma unroll
  for (int u = 0; u < kMS; ++u) {
    float x[12];
    load_own_rfl(C, i + u, x);
    const f32x4 a = y[3 * u], b = y[3 * u + 1], c = y[3 * u + 2];
    float g = 0.0f;
    g = __builtin_fmaf(x[0], a.x, g);
    g = __builtin_fmaf(x[1], a.y, g);
    g = __builtin_fmaf(x[2], a.z, g);
    g = __builtin_fmaf(x[3], a.w, g);
    g = __builtin_fmaf(x[4], b.x, g);
    g = __builtin_fmaf(x[5], b.y, g);
    g = __builtin_fmaf(x[6], b.z, g);
    g = __builtin_fmaf(x[7], b.w, g);
    g = __builtin_fmaf(x[8], c.x, g);
    g = __builtin_fmaf(x[9], c.y, g);
    g = __builtin_fmaf(x[10], c.z, g);
    g = __builtin_fmaf(x[11], c.w, g);
    dot = dot + g;
  }
  if (!active) return 0xffffffffu;
  return __builtin_bit_cast(unsigned, make_key<TRANS>(C.Nown[i], C.Nin[j], dot));
}

// Fast variant for the common small candidate groups: own frames of the stripe staged in
// LDS (Xown[a] = own stacked row i0 + a), inner frames loaded all at once; inlined.
template <bool TRANS>
__device__ __forceinline__ unsigned full_key_fast(const SelCtx& C, const float* Xown, int i, int j, bool active) {
  f32x4 y[kMS * 3];
#pragma unroll
  for (int u = 0; u < kMS; ++u) {
    const f32x4* yp = reinterpret_cast<const f32x4*>(C.inner + (size_t)((active ? j + u : 0) * C.tau) * 12);
    y[3 * u] = yp[0];
    y[3 * u + 1] = yp[1];
    y[3 * u + 2] = yp[2];
  }
  float dot = 0.0f;
#pragma unroll
  for (int u = 0; u < kMS; ++u) {
    const f32x4* xp = reinterpret_cast<const f32x4*>(Xown + (i - C.i0 + u) * 12);
    const f32x4 xa = xp[0], xb = xp[1], xc = xp[2];
    const f32x4 a = y[3 * u], b = y[3 * u + 1], c = y[3 * u + 2];
    float g = 0.0f;
    g = __builtin_fmaf(xa.x, a.x, g);
    g = __builtin_fmaf(xa.y, a.y, g);
    g = __builtin_fmaf(xa.z, a.z, g);
    g = __builtin_fmaf(xa.w, a.w, g);
    g = __builtin_fmaf(xb.x, b.x, g);
    g = __builtin_fmaf(xb.y, b.y, g);
    g = __builtin_fmaf(xb.z, b.z, g);
    g = __builtin_fmaf(xb.w, b.w, g);
    g = __builtin_fmaf(xc.x, c.x, g);
    g = __builtin_fmaf(xc.y, c.y, g);
    g = __builtin_fmaf(xc.z, c.z, g);
    g = __builtin_fmaf(xc.w, c.w, g);
    dot = dot + g;
  }
  if (!active) return 0xffffffffu;
  return __builtin_bit_cast(unsigned, make_key<TRANS>(C.Nown[i], C.Nin[j], dot));
}

// ---- per-wave helpers ----

// ---- per-row select on 16-bit key prefixes held in registers ----
// Keys of one row as seen by one lane: lane l holds elements l + 64q (0xffffffff = none).
template <int KPL>
struct RowKeys {
  unsigned v[KPL];
  __device__ __forceinline__ void load(const uint16_t* row, int n) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const int e = lane + 64 * q;
      v[q] = e < n ? (unsigned)row[e] : 0xffffffffu;
    }
  }
  __device__ __forceinline__ int count_le(unsigned x) const {  // #keys <= x (x <= 0xffff)
    int c = 0;
#pragma unroll
    for (int q = 0; q < KPL; ++q) c += v[q] <= x;
    return wave_sum(c);
  }
  __device__ __forceinline__ void min_max(unsigned* mn, unsigned* mx) const {
    unsigned a = 0xffffu, b = 0u;
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      if (v[q] != 0xffffffffu) {
        a = min(a, v[q]);
        b = max(b, v[q]);
      }
    }
    *mn = wave_min_u32(a);
    *mx = wave_max_u32(b);
  }
  __device__ __forceinline__ unsigned min_greater(unsigned x) const {
    unsigned a = 0xffffffffu;
#pragma unroll
    for (int q = 0; q < KPL; ++q)
      if (v[q] > x) a = min(a, v[q]);
    return wave_min_u32(a);
  }
  // write the (row, column) of every key == P to list (wave-cooperative, ballot + mbcnt)
  __device__ __forceinline__ void collect(unsigned P, int r, int* list) const {
    const int lane = threadIdx.x & 63;
    int base = 0;
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const bool m = v[q] == P;
      const unsigned long long bal = __ballot(m);
      if (m)
        list[base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] =
            (r << 16) | (lane + 64 * q);
      base += __popcll(bal);
    }
  }
};

// Smallest prefix P with count(keys <= P) > rho (binary search over [kmin, kmax]).
template <int KPL>
__device__ __forceinline__ unsigned prefix_of_rank(const RowKeys<KPL>& K, int rho, unsigned kmin, unsigned kmax) {
  unsigned a = kmin, b = kmax;
  while (a < b) {
    const unsigned mid = (a + b) >> 1;
    if (K.count_le(mid) > rho)
      b = mid;
    else
      a = mid + 1;
  }
  return a;
}

// Slow exact path for one group (very large prefix groups, e.g. long silences, or a full
// candidate list): MSB-first search on the low 16 bits, recomputing member keys each step.
template <bool TRANS>
__device__ unsigned exact_slow(const SelCtx& C, const uint16_t* row, int n, int srow, unsigned P, int rho) {
  const int lane = threadIdx.x & 63;
  unsigned res = 0;
  for (int b = 15; b >= 0; --b) {
    const unsigned cand = res | (1u << b);
    int cnt = 0;
    for (int e0 = 0; e0 < n; e0 += 64) {
      const int e = e0 + lane;
      const bool m = e < n && row[e] == (uint16_t)P;
      if (__ballot(m)) {
        const unsigned k = full_key<TRANS>(C, srow, m ? e : 0, m);
        cnt += m && (k & 0xffffu) < cand;
      }
    }
    cnt = wave_sum(cnt);
    if (cnt <= rho) res = cand;
  }
  return (P << 16) | res;
}

// Per-row bookkeeping between the phases (LDS).
struct RowSel {
  unsigned P[2];     // prefixes of the lo / hi order statistic
  int rho[2];        // rank inside its prefix group
  int off[2], g[2];  // candidate list slice (g == -1: slow path for that group, -2: whole row)
};

constexpr int kCand = 1024;  // block-wide candidate list capacity

template <bool TRANS>
__device__ __forceinline__ void select_body(const SelCtx& C, uint16_t* K16, float* Ys, float* Ns, float kappa, float* thr_out,
                            float* T_out) {
  const int t = threadIdx.x;
  // own stacked norms of the stripe: wave-uniform, loaded once (SGPRs)
  float nown[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
    const int i = min(C.i0 + r, C.i0 + C.rows - 1);
    nown[r] = *(const __attribute__((address_space(4))) float*)(C.Nown + i);
  }
  // ---- sweep: parallelogram panels of 256 diagonals ----
  for (int j0 = -(kR - 1); j0 < C.n_in_s; j0 += kW) {
    __syncthreads();
    for (int e = t; e < kYRows * 3; e += kW) {  // stage inner frames (float4 pieces)
      const int b = e / 3, piece = e - b * 3;
      const int jr = j0 + b;
      const int f = jr * C.tau;
      float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (jr >= 0 && f < C.n_in_f) v = reinterpret_cast<const float4*>(C.inner + (size_t)f * 12)[piece];
      reinterpret_cast<float4*>(Ys)[e] = v;
    }
    for (int b = t; b < kNRows; b += kW) {
      const int jr = j0 + b;
      Ns[b] = (jr >= 0 && jr < C.n_in_s) ? C.Nin[jr] : 0.0f;
    }
    __syncthreads();
    float gw[kMS];
    float xb[2][12];
    f32x4 yb[2][3];
    load_own(C, C.i0, xb[0]);
    {
      const f32x4* yp = reinterpret_cast<const f32x4*>(Ys + t * 12);
      yb[0][0] = yp[0];
      yb[0][1] = yp[1];
      yb[0][2] = yp[2];
    }
#pragma unroll
    for (int kk = 0; kk < kR + kMS - 1; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if (kk + 1 < kR + kMS - 1) {  // software pipeline: next step's frames in flight
        load_own(C, C.i0 + kk + 1, xb[nxt]);
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
        const int jj = j0 + t + r;
        const float key = make_key<TRANS>(nown[r], Ns[t + r], dot);  // all lanes; store predicated
        if (r < C.rows && jj >= 0 && jj < C.n_in_s)
          K16[r * C.ld16 + jj] = (uint16_t)(__builtin_bit_cast(unsigned, key) >> 16);
      }
    }
  }
  __syncthreads();
  // ---- selects ----
  // LDS scratch (aliases the panel buffers): own frames | candidate list | row records | counter
  float* Xown = Ys;
  int* cand = reinterpret_cast<int*>(Ys) + (kR + kMS - 1) * 12;
  RowSel* rs = reinterpret_cast<RowSel*>(cand + kCand);
  int* ncand = reinterpret_cast<int*>(rs + kR);
  for (int e = t; e < (kR + kMS - 1) * 12; e += kW) {
    const int a = e / 12, c = e - a * 12;
    int f = (C.i0 + a) * C.tau;
    f = f < C.n_own_f ? f : C.n_own_f - 1;
    Xown[e] = C.own[(size_t)f * 12 + c];
  }
  if (t == 0) *ncand = 0;
  __syncthreads();
  const int lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform (SGPR)
  const int n = C.n_in_s;
  const float q = (float)(n - 1) * kappa;
  const float lo_f = floorf(q), hi_f = ceilf(q);
  const int lo = (int)lo_f, hi = (int)hi_f;
  const bool regs = n <= 64 * 32;
  const int nrows = C.rows;
  // phase A (per wave): 16-bit prefixes of both order statistics; candidates collected
  for (int r = w; r < nrows; r += 4) {
    const uint16_t* row = K16 + r * C.ld16;
    RowSel sel;
    if (regs) {
      RowKeys<32> K;
      K.load(row, n);
      unsigned kmin, kmax;
      K.min_max(&kmin, &kmax);
      const unsigned Pl = prefix_of_rank(K, lo, kmin, kmax);
      const int le = K.count_le(Pl);
      const int less = Pl > 0 ? K.count_le(Pl - 1) : 0;
      sel.P[0] = Pl;
      sel.rho[0] = lo - less;
      sel.g[0] = le - less;
      if (hi < le) {  // hi shares the prefix group of lo
        sel.P[1] = Pl;
        sel.rho[1] = hi - less;
        sel.g[1] = sel.g[0];
      } else {  // hi = smallest key of the next group
        const unsigned Ph = K.min_greater(Pl);
        sel.P[1] = Ph;
        sel.rho[1] = 0;
        sel.g[1] = K.count_le(Ph) - le;
      }
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && sel.P[1] == sel.P[0]) {
          sel.off[1] = sel.off[0];
          sel.g[1] = sel.g[0];
          continue;
        }
        int off = -1;
        if (sel.g[h] <= 64 && lane == 0) off = atomicAdd(ncand, sel.g[h]);
        off = lane_bcast(off, 0);
        if (off >= 0 && off + sel.g[h] <= kCand) {
          K.collect(sel.P[h], r, cand + off);
          sel.off[h] = off;
        } else {
          sel.off[h] = -1;
          sel.g[h] = -1;  // slow path for this group
        }
      }
    } else {
      sel.g[0] = sel.g[1] = -2;  // long rows: fully slow path in phase C
    }
    if (lane == 0) rs[r] = sel;
  }
  __syncthreads();
  // phase B (block): exact keys of every collected candidate, one per thread, in one round
  const int nc = min(*ncand, kCand);
  for (int e = t; e < nc; e += kW) {
    const int pk = cand[e];
    const int r = pk >> 16, j = pk & 0xffff;
    cand[e] = (int)full_key_fast<TRANS>(C, Xown, C.i0 + r, j, true);
  }
  __syncthreads();
  // phase C (per wave): rank inside the groups, interpolate, squared-domain threshold
  for (int r = w; r < nrows; r += 4) {
    const int srow = __builtin_amdgcn_readfirstlane(C.i0 + r);
    const RowSel sel = rs[r];
    const uint16_t* row = K16 + r * C.ld16;
    unsigned v[2];
    if (sel.g[0] == -2) {  // long row: count-based search straight from LDS (slow, rare)
      for (int h = 0; h < 2; ++h) {
        const int rho = h == 0 ? lo : hi;
        unsigned a = 0, b = 0xffffu;
        while (a < b) {
          const unsigned mid = (a + b) >> 1;
          int c = 0;
          for (int e = lane; e < n; e += 64) c += row[e] <= mid;
          if (wave_sum(c) > rho)
            b = mid;
          else
            a = mid + 1;
        }
        int less = 0;
        for (int e = lane; e < n; e += 64) less += row[e] < a;
        less = wave_sum(less);
        v[h] = exact_slow<TRANS>(C, row, n, srow, a, rho - less);
      }
    } else {
      for (int h = 0; h < 2; ++h) {
        if (sel.g[h] < 0) {
          v[h] = exact_slow<TRANS>(C, row, n, srow, sel.P[h], sel.rho[h]);
          continue;
        }
        const int g = sel.g[h];
        const unsigned key = lane < g ? (unsigned)cand[sel.off[h] + lane] : 0xffffffffu;
        int cl = 0, ce = 0;
        for (int qq = 0; qq < g; ++qq) {
          const unsigned o = (unsigned)lane_bcast((int)key, qq);
          cl += o < key;
          ce += o == key;
        }
        const int src = __builtin_ctzll(__ballot(lane < g && cl <= sel.rho[h] && sel.rho[h] < cl + ce));
        v[h] = (unsigned)lane_bcast((int)key, src);
      }
    }
    if (lane == 0) {
      const float slo = sqrt_rn(__builtin_bit_cast(float, v[0]));
      float thr;
      if (lo_f == hi_f) {
        thr = slo;
      } else {
        const float shi = sqrt_rn(__builtin_bit_cast(float, v[1]));
        const float aa = slo * (hi_f - q);
        const float bb = shi * (q - lo_f);
        thr = aa + bb;
      }
      thr_out[srow] = thr;
      T_out[srow] = sq_threshold(thr);
    }
  }
}

template <bool TRANS>
__global__ __launch_bounds__(256, 2) void k_crp_select16(CrpBatch B, int ld16, float kappa, float* __restrict__ thr,
                                                         float* __restrict__ Tq, int64_t thr_stride) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem8[];
  const int p = blockIdx.y;
  const int2 dm = B.dims[p];
  const int n_own_s = TRANS ? dm.y : dm.x, n_in_s = TRANS ? dm.x : dm.y;
  const int i0 = blockIdx.x * kR;
  if (i0 >= n_own_s || n_in_s <= 0) return;
  const int ta = B.pairs[2 * p], tb = B.pairs[2 * p + 1];
  const int t_own = TRANS ? tb : ta, t_in = TRANS ? ta : tb;
  SelCtx C;
  const float* X = B.feats + B.off[ta] * 12;
  const float* Yr = B.yrot + (size_t)p * B.yrot_stride;
  C.own = TRANS ? Yr : X;
  C.inner = TRANS ? X : Yr;
  C.n_own_f = B.len[t_own];
  C.n_in_f = B.len[t_in];
  C.tau = B.tau;
  C.Nown = B.NX + (size_t)t_own * B.ldn;
  C.Nin = B.NX + (size_t)t_in * B.ldn;
  C.i0 = i0;
  C.rows = min(kR, n_own_s - i0);
  C.n_in_s = n_in_s;
  C.ld16 = ld16;
  uint16_t* K16 = reinterpret_cast<uint16_t*>(smem8);
  float* Ys = reinterpret_cast<float*>(smem8 + align_up((size_t)kR * ld16 * 2, 16));
  float* Ns = Ys + kYRows * 12;
  select_body<TRANS>(C, K16, Ys, Ns, kappa, thr + (size_t)p * thr_stride, Tq + (size_t)p * thr_stride);
}

size_t select16_lds(int ld16) {
  const size_t scratch = (size_t)(kR + kMS - 1) * 12 * 4 + (size_t)kCand * 4 + sizeof(RowSel) * kR + 16;
  const size_t panel = (size_t)kYRows * 12 * 4 + (size_t)kNRows * 4;
  return align_up((size_t)kR * ld16 * 2, 16) + (panel > scratch ? panel : scratch);
}

}  // namespace

int launch_select16(bool trans, const CrpBatch& B, int nb, int L, float kappa, float* thr, float* T,
                    int64_t thr_stride, hipStream_t s) {
  if (B.m != kMS) return 1;
  const int ld16 = (int)align_up((size_t)L, 8);
  const size_t lds = select16_lds(ld16);
  if (lds > 160 * 1024) return 1;
  const void* fn = trans ? reinterpret_cast<const void*>(k_crp_select16<true>)
                         : reinterpret_cast<const void*>(k_crp_select16<false>);
  if (lds > 64 * 1024) ACOSS_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const dim3 grid((L + kR - 1) / kR, nb);
  if (trans)
    hipLaunchKernelGGL(k_crp_select16<true>, grid, dim3(256), lds, s, B, ld16, kappa, thr, T, thr_stride);
  else
    hipLaunchKernelGGL(k_crp_select16<false>, grid, dim3(256), lds, s, B, ld16, kappa, thr, T, thr_stride);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

}  // namespace acoss
