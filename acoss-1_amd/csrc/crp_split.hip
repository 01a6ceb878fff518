// crp_split.hip — Serra09/Chen CRP in three kernels around ONE distance sweep (m = 9).
//
// Replaces, per pair, the body of essentia ChromaCrossSimilarity (rqa_serra09.py:60-66,
// latefusion_chen.py:63-69): stacked distances, percentile(row/column, 9.5) and the mutual
// binary mask, bit-identical to oracle/crp_oracle.cpp.
//
//  k_sweep9      one 256-thread block per (32-row strip, pair): diagonal walk (G in
//                registers, query frames by scalar loads, rolled reference frames in LDS);
//                every squared-distance key goes to HBM as the FULL 32-bit key row-major
//                F[i][j] and as its HIGH 16 bits strip-major Hc[i/32][j][i%32] (64 B per
//                column and strip, a block's columns contiguous; through a rolling LDS tile).
//  k_sel_rows9   one 512-thread block per (32-row strip, pair), one wave per CRP row: 32 full
//                keys per lane in registers, the 16-bit prefixes of the two order statistics
//                by binary search with ballot counts (v_cmp + s_bcnt1), the tied group ranked
//                on the exact keys -> percentile -> squared-domain threshold T_row; then the
//                row's "key <= T_row" bits, transposed in LDS into the 32-bit strip words RT.
//  k_sel_cols9   one wave per CRP column on the 16-bit prefixes: the same select gives T_col,
//                the tied group's exact keys come from F (one gather round); lane l then
//                holds rows 32l..32l+31 of the column, i.e. exactly one 32-bit CRP word:
//                (key <= T_col bits) & RT[strip l][j].
#include <cstdlib>
#include <cstring>

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
constexpr int kSCols = kSW + kSR;             // 288 columns touched

__device__ __forceinline__ void load_query(const float* base_ptr, int f, float (&x)[12]) {
  const float* base = base_ptr + (size_t)f * 12;
  asm volatile("" : "+s"(base));  // keep each row's scalar load inside the loop
  const cfloat4* p = (const cfloat4*)base;
  const f32x4 a = p[0], b = p[1], c = p[2];
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w;
}

// Key planes of one pair: full keys row-major (line = CRP row), high 16 bits column-major.
struct KeyPlanes {
  uint32_t* fr;
  uint16_t* hc;
};

constexpr int kTP = 34;  // tile pitch in halfwords: 17 words, odd -> lane stride hits distinct banks

// FAST: tau == 1, a full 32-row strip and all 40 query frames inside the track, so the query
// frames and row norms sit at compile-time offsets from one base (s_load immediates) and no
// per-row clamp or bound is needed; otherwise the clamped general path.
template <bool FAST>
__device__ __forceinline__ void sweep_body(const PairView& V, int p, int strip, const KeyPlanes& K, int ldr, int ldc,
                                           int64_t kstride, float* Ys, float* Ns, uint16_t* tileT) {
  const int i0 = strip * kSR;
  const int t = threadIdx.x;
  const int rows = FAST ? kSR : min(kSR, V.Mp - i0);
  const float* Xi0 = V.X + (size_t)i0 * 12;
  const float* Nq0 = V.NXq + i0;
  auto nqr = [&](int r) {  // row norm: a scalar load at a compile-time offset
    const float* base = Nq0;
    asm volatile("" : "+s"(base));
    return *(const __attribute__((address_space(4))) float*)(FAST ? base + r : V.NXq + min(i0 + r, V.Mp - 1));
  };
  uint32_t* Fr = K.fr + (size_t)p * kstride + (size_t)i0 * ldr;
  uint16_t* Hc = K.hc + (size_t)p * kstride;
  auto query = [&](int kk, float (&x)[12]) {
    if (FAST) {
      const float* base = Xi0;
      asm volatile("" : "+s"(base));  // keep each row's scalar load in the loop
      const cfloat4* q = (const cfloat4*)(base + kk * 12);
      const f32x4 a = q[0], b = q[1], c = q[2];
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
      x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      x[8] = c.x; x[9] = c.y; x[10] = c.z; x[11] = c.w;
    } else {
      load_query(V.X, min((i0 + kk) * V.tau, V.nq - 1), x);
    }
  };
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
    query(0, xb[0]);
    uint32_t* frow = Fr;
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
        query(kk + 1, xb[nxt]);
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
        const float d2 = (nqr(r) - 2.0f * dot) + Ns[t + r];
        const unsigned key = __builtin_bit_cast(unsigned, d2 > 0.0f ? d2 : 0.0f);
        // full key row-major straight from registers: the 64 lanes write 64 consecutive columns
        const int col = j0 + t + r;
        // out-of-range columns (< 0 or >= Np) land in the pad column ldr - 1 (never read):
        // branchless, no per-row lane masks to keep live
        if (FAST || r < rows) frow[min((unsigned)col, (unsigned)(ldr - 1))] = key;
        frow += ldr;  // next row: one scalar add instead of 32 hoisted row pointers
        asm volatile("" : "+s"(frow));
        tileT[(t + r) * kTP + r] = (uint16_t)(key >> 16);
      }
    }
    __syncthreads();
    // columns [j0, j0 + 256) complete: column-major prefixes, 32 rows = 64 B per column
    const int jj = j0 + t;
    if (jj >= 0 && jj < V.Np) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(tileT + t * kTP);
      uint4* dh = reinterpret_cast<uint4*>(Hc + ((size_t)strip * ldc + jj) * kSR);  // [strip][column][32 rows]
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint4 h;
        h.x = src[4 * q];
        h.y = src[4 * q + 1];
        h.z = src[4 * q + 2];
        h.w = src[4 * q + 3];
        dh[q] = h;
      }
    }
    __syncthreads();
    // roll the 31-column tail to the front
    for (int e = t; e < (kSR - 1) * (kTP / 2); e += kSW) {
      const int c = e / (kTP / 2), w = e - c * (kTP / 2);
      reinterpret_cast<uint32_t*>(tileT)[c * (kTP / 2) + w] = reinterpret_cast<const uint32_t*>(tileT)[(kSW + c) * (kTP / 2) + w];
    }
  }
}

__global__ __launch_bounds__(256) void k_sweep9(CrpBatch B, KeyPlanes K, int ldr, int ldc, int64_t kstride) {
  __shared__ __attribute__((aligned(16))) float Ys[kSYRows * 12];
  __shared__ float Ns[kSCols];
  __shared__ __attribute__((aligned(16))) uint16_t tileT[kSCols * kTP];  // [column][row] 16-bit prefixes
  const int p = blockIdx.y;
  const PairView V = pair_view(B, p);
  const int strip = blockIdx.x, i0 = strip * kSR;
  if (i0 >= V.Mp || V.Np <= 0) return;
  if (V.tau == 1 && i0 + kSR <= V.Mp && i0 + kSR + kMS - 1 <= V.nq)
    sweep_body<true>(V, p, strip, K, ldr, ldc, kstride, Ys, Ns, tileT);
  else
    sweep_body<false>(V, p, strip, K, ldr, ldc, kstride, Ys, Ns, tileT);
}

// ---------------------------------------------------------------------------------------
// Per-wave select on one line (CRP row or column) of 16-bit key prefixes.
// Lane l holds elements [l*KPL, (l+1)*KPL) as KPL/2 packed words: element 2h in bits 0..15,
// 2h+1 in bits 16..31. Real prefixes are <= 0x7f80 (keys are >= +0, the sign bit is 0), so
// 0x7fff marks "no element" and every field keeps a free guard bit for SWAR arithmetic.
// ---------------------------------------------------------------------------------------
constexpr unsigned kNone = 0x7fffu;

__device__ __forceinline__ unsigned pk_min_u16(unsigned a, unsigned b) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ unsigned pk_max_u16(unsigned a, unsigned b) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ unsigned pk_add_u16(unsigned a, unsigned b) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}

template <int KPL>
struct Line {
  unsigned pv[KPL / 2];
  __device__ __forceinline__ unsigned pfx(int q) const { return (q & 1) ? (pv[q >> 1] >> 16) : (pv[q >> 1] & 0xffffu); }
  // lane l's KPL elements start at col0 + l * lane_stride (strip-major column plane): the
  // loaded words already are the packed pairs
  __device__ __forceinline__ void load_lanes(const uint16_t* col0, size_t lane_stride, int n) {
    const int lane = threadIdx.x & 63;
    const int base = lane * KPL;
    const uint16_t* src = col0 + (size_t)lane * lane_stride;
    if (base + KPL <= n) {
#pragma unroll
      for (int q = 0; q < KPL / 8; ++q) {
        const uint4 w = reinterpret_cast<const uint4*>(src)[q];
        pv[4 * q + 0] = w.x;
        pv[4 * q + 1] = w.y;
        pv[4 * q + 2] = w.z;
        pv[4 * q + 3] = w.w;
      }
    } else {
#pragma unroll
      for (int h = 0; h < KPL / 2; ++h) {
        const unsigned a = (base + 2 * h < n) ? (unsigned)src[2 * h] : kNone;
        const unsigned b = (base + 2 * h + 1 < n) ? (unsigned)src[2 * h + 1] : kNone;
        pv[h] = a | (b << 16);
      }
    }
  }
  // from full keys (0xffffffff = none): high halves of two keys in one v_perm, clamped to kNone
  __device__ __forceinline__ void from_full(const unsigned* f) {
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) pv[h] = pk_min_u16(__builtin_amdgcn_perm(f[2 * h + 1], f[2 * h], 0x07060302u), 0x7fff7fffu);
  }
  // #elements <= x (x <= 0x7fff): per field (x + 0x8000) - a keeps bit 15 iff a <= x, with no
  // borrow across fields; popcount on VALU, one DPP wave sum (no SGPR per compare, no SALU).
  __device__ __forceinline__ int count_le(unsigned x) const {
    const unsigned X2 = (x + 0x8000u) * 0x10001u;
    unsigned c = 0;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) c = __builtin_popcount((X2 - pv[h]) & 0x80008000u) + c;
    return wave_sum((int)c);
  }
  // min over elements (kNone is above every real prefix) and max over real elements
  // (kNone + 1 wraps to 0x8000, masked to 0: below every real prefix + 1)
  __device__ __forceinline__ void min_max(unsigned* mn, unsigned* mx) const {
    unsigned a = 0xffffffffu, b = 0u;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) {
      a = pk_min_u16(a, pv[h]);
      b = pk_max_u16(b, pk_add_u16(pv[h], 0x00010001u) & 0x7fff7fffu);
    }
    a = min(a & 0xffffu, a >> 16);
    b = max(b & 0xffffu, b >> 16);
    *mn = wave_min_u32(a);
    const unsigned m = wave_max_u32(b);
    *mx = m ? m - 1 : 0u;
  }
  __device__ __forceinline__ unsigned min_greater(unsigned x) const {
    unsigned a = 0xffffffffu;
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
      const unsigned k = pfx(q);
      a = (k > x && k != kNone) ? min(a, k) : a;
    }
    return wave_min_u32(a);
  }
};

// A line of FULL keys (CRP row from F): f = exact keys, packed prefixes for the search.
template <int KPL>
struct LineFull : Line<KPL> {
  unsigned f[KPL];
  __device__ __forceinline__ void load_full(const uint32_t* src, int n) {
    const int lane = threadIdx.x & 63;
    const int base = lane * KPL;
    if (base + KPL <= n) {
#pragma unroll
      for (int q = 0; q < KPL / 4; ++q) {
        const uint4 w = reinterpret_cast<const uint4*>(src + base)[q];
        f[4 * q + 0] = w.x;
        f[4 * q + 1] = w.y;
        f[4 * q + 2] = w.z;
        f[4 * q + 3] = w.w;
      }
    } else {
      // opaque per-lane count: keeps the 32 tail predicates from being hoisted out of the
      // caller's row loop into (spilled) SGPR masks
      int nv = n - base;
      asm volatile("" : "+v"(nv));
#pragma unroll
      for (int q = 0; q < KPL; ++q) f[q] = (q < nv) ? src[base + q] : 0xffffffffu;
    }
    this->from_full(f);
  }
};

// Smallest prefix P with count(keys <= P) > rho, bisecting [a, b]; also returns
// le = count(<= P) and less = count(< P) (carried through the search: no extra counts).
// hint (wave-uniform, or kNoHint): the previous line's answer. Adjacent stacked rows/columns
// share 8 of their 9 frames, so the answer is usually a few prefixes away: gallop out from
// the hint to a bracket, then bisect inside it.
constexpr unsigned kNoHint = 0xffffffffu;

template <int KPL>
__device__ __forceinline__ unsigned prefix_of_rank(const Line<KPL>& L, int rho, unsigned a, unsigned b, int n,
                                                   unsigned hint, int* le_out, int* less_out) {
  int c_b = n;    // count(<= b): every element is <= kmax
  int c_am1 = 0;  // count(<= a - 1): none is below kmin
  // one count per iteration, probe chosen by the mode (a single count_le site keeps the
  // unrolled SWAR body once): 0 hint, 1 gallop down, 2 gallop up, 3 bisect
  int mode = (hint != kNoHint) ? 0 : 3;
  unsigned step = 1;
  while (a < b) {
    unsigned t;
    if (mode == 0)
      t = hint < a ? a : (hint > b ? b : hint);
    else if (mode == 1)
      t = (b - a > step) ? b - step : a;
    else if (mode == 2)
      t = (b - a > step) ? a + step - 1 : (a + b) >> 1;
    else
      t = (a + b) >> 1;
    const int c = L.count_le(t);
    const bool greater = c > rho;
    if (greater) {
      b = t;
      c_b = c;
    } else {
      a = t + 1;
      c_am1 = c;
    }
    if (mode == 0)
      mode = greater ? 1 : 2;
    else if (mode == 1)
      mode = greater ? (step <<= 1, 1) : 3;
    else if (mode == 2)
      mode = greater ? 3 : (step <<= 1, 2);
  }
  *le_out = c_b;
  *less_out = c_am1;
  return a;
}

// Scratch of one wave in LDS: element list and 64 bit-words.
struct WaveLds {
  int list[64];
  uint32_t words[64];
};

// Exact keys of a prefix group (the line elements whose 16-bit prefix is P), computed in ONE
// batched round: lane k < g recomputes element list[k]. Valid when g <= 64.
struct Group {
  unsigned P;
  int g;
  int elem;      // this lane's element (lane < g)
  unsigned key;  // its exact key (0xffffffff for lane >= g)
};

template <int KPL, class KF>
__device__ Group group_keys(const Line<KPL>& L, unsigned P, int g, const KF& keyf, WaveLds& W) {
  const int lane = threadIdx.x & 63;
  int base = 0;
#pragma unroll
  for (int q = 0; q < KPL; ++q) {
    const bool m = L.pfx(q) == P;
    const unsigned long long bal = __ballot(m);
    if (m)
      W.list[base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] =
          lane * KPL + q;
    base += __popcll(bal);
  }
  __builtin_amdgcn_wave_barrier();
  Group G;
  G.P = P;
  G.g = g;
  G.elem = lane < g ? W.list[lane] : 0;
  __builtin_amdgcn_wave_barrier();
  G.key = lane < g ? keyf(G.elem) : 0xffffffffu;
  return G;
}

// Same group from a line that holds its exact keys in registers (no recompute).
template <int KPL>
__device__ Group group_keys_full(const LineFull<KPL>& L, unsigned P, int g, WaveLds& W) {
  const int lane = threadIdx.x & 63;
  int base = 0;
#pragma unroll
  for (int q = 0; q < KPL; ++q) {
    const bool m = L.pfx(q) == P;
    const unsigned long long bal = __ballot(m);
    if (m)
      W.list[base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] =
          (int)L.f[q];
    base += __popcll(bal);
  }
  __builtin_amdgcn_wave_barrier();
  Group G;
  G.P = P;
  G.g = g;
  G.elem = 0;
  G.key = lane < g ? (unsigned)W.list[lane] : 0xffffffffu;
  __builtin_amdgcn_wave_barrier();
  return G;
}

// Key of rank rho (0-based) inside a batched group.
__device__ __forceinline__ unsigned group_rank(const Group& G, int rho) {
  const int lane = threadIdx.x & 63;
  int cl = 0, ce = 0;
  for (int k = 0; k < G.g; ++k) {
    const unsigned o = (unsigned)lane_bcast((int)G.key, k);
    cl += o < G.key;
    ce += o == G.key;
  }
  const bool act = lane < G.g;
  const int src = __builtin_ctzll(__ballot(act && cl <= rho && rho < cl + ce));
  return (unsigned)lane_bcast((int)G.key, src);
}

// Large groups (g > 64, long silences): recompute the group's low halves lane by lane, then
// binary-search the low 16 bits counting group members only.
template <int KPL, class KF>
__device__ unsigned big_group_rank(const Line<KPL>& L, unsigned P, int rho, const KF& keyf) {
  const int base = (threadIdx.x & 63) * KPL;
  unsigned lw[KPL];
#pragma unroll
  for (int q = 0; q < KPL; ++q) lw[q] = 0x10000u;
  for (int q = 0; q < KPL; ++q)
    if (L.pfx(q) == P) lw[q] = keyf(base + q) & 0xffffu;
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

template <int KPL, class KF>
__device__ unsigned rank_in_prefix(const Line<KPL>& L, unsigned P, int rho, int g, const KF& keyf, WaveLds& W,
                                   Group* cache) {
  if (g <= 64) {
    if (cache->g < 0 || cache->P != P) *cache = group_keys(L, P, g, keyf, W);
    return group_rank(*cache, rho);
  }
  return big_group_rank(L, P, rho, keyf);
}

// Threshold (distance units) and squared-domain threshold of a line of n keys; leaves the
// exact keys of the last batched group in *cache for le_bits.
template <int KPL, class KF>
__device__ void line_threshold(const Line<KPL>& L, int n, float kappa, const KF& keyf, WaveLds& W, Group* c_lo,
                               Group* c_hi, float* thr, float* T, unsigned* hint) {
  const float q = (float)(n - 1) * kappa;
  const float lo_f = floorf(q), hi_f = ceilf(q);
  const int lo = (int)lo_f, hi = (int)hi_f;
  unsigned kmin, kmax;
  L.min_max(&kmin, &kmax);
  int le, less;
  const unsigned Pl = prefix_of_rank(L, lo, kmin, kmax, n, *hint, &le, &less);
  *hint = Pl;
  const unsigned vlo = rank_in_prefix(L, Pl, lo - less, le - less, keyf, W, c_lo);
  unsigned vhi = vlo;
  if (hi != lo) {
    if (hi < le) {
      vhi = rank_in_prefix(L, Pl, hi - less, le - less, keyf, W, c_lo);
    } else {
      const unsigned Ph = L.min_greater(Pl);
      vhi = rank_in_prefix(L, Ph, 0, L.count_le(Ph) - le, keyf, W, c_hi);
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

// Row variant of line_threshold: the line holds its exact keys, groups rank from registers;
// groups above 64 members binary-search the low halves held in registers.
template <int KPL>
__device__ unsigned row_rank(const LineFull<KPL>& L, unsigned P, int rho, int g, WaveLds& W) {
  if (g <= 64) return group_rank(group_keys_full(L, P, g, W), rho);
  unsigned a = 0, b = 0xffffu;
  while (a < b) {
    const unsigned mid = (a + b) >> 1;
    int c = 0;
#pragma unroll
    for (int q = 0; q < KPL; ++q) c += __popcll(__ballot(L.pfx(q) == P && (L.f[q] & 0xffffu) <= mid));
    if (c > rho)
      b = mid;
    else
      a = mid + 1;
  }
  return (P << 16) | a;
}

template <int KPL>
__device__ void row_threshold(const LineFull<KPL>& L, int n, float kappa, WaveLds& W, float* thr, float* T,
                              unsigned* hint) {
  const float q = (float)(n - 1) * kappa;
  const float lo_f = floorf(q), hi_f = ceilf(q);
  const int lo = (int)lo_f, hi = (int)hi_f;
  unsigned kmin, kmax;
  L.min_max(&kmin, &kmax);
  int le, less;
  const unsigned Pl = prefix_of_rank(L, lo, kmin, kmax, n, *hint, &le, &less);
  *hint = Pl;
  const unsigned vlo = row_rank(L, Pl, lo - less, le - less, W);
  unsigned vhi = vlo;
  if (hi != lo) {
    if (hi < le) {
      vhi = row_rank(L, Pl, hi - less, le - less, W);
    } else {
      const unsigned Ph = L.min_greater(Pl);
      vhi = row_rank(L, Ph, 0, L.count_le(Ph) - le, W);
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

// Bits of "key <= T" for the KPL elements of this lane (element e = lane*KPL + q). Decided on
// the prefix; the elements whose prefix equals T's are decided on exact keys from a batched
// group (reused from the threshold search when it has that prefix).
template <int KPL, class KF>
__device__ uint32_t le_bits(const Line<KPL>& L, unsigned Tbits, const KF& keyf, WaveLds& W, const Group& c_lo,
                            const Group& c_hi) {
  const unsigned T16 = Tbits >> 16;
  const int lane = threadIdx.x & 63;
  uint32_t word = 0;
  int amb = 0;
#pragma unroll
  for (int q = 0; q < KPL; ++q) {
    const unsigned k = L.pfx(q);  // kNone is never <= T16 (T16 <= 0x7f80)
    word |= (uint32_t)(k < T16) << q;
    amb += k == T16;
  }
  const int g = wave_sum(amb);
  if (g == 0) return word;
  if (g <= 64) {
    Group G;
    if (c_lo.g >= 0 && c_lo.P == T16)
      G = c_lo;
    else if (c_hi.g >= 0 && c_hi.P == T16)
      G = c_hi;
    else
      G = group_keys(L, T16, g, keyf, W);
    W.words[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    if (lane < G.g && G.key <= Tbits) atomicOr(&W.words[G.elem / KPL], 1u << (G.elem % KPL));
    __builtin_amdgcn_wave_barrier();
    return word | W.words[lane];
  }
  const int base = lane * KPL;
  for (int q = 0; q < KPL; ++q)
    if (L.pfx(q) == T16) word |= (uint32_t)(keyf(base + q) <= Tbits) << q;
  return word;
}

// ---------------------------------------------------------------------------------------
// k_sel_rows9: one 512-thread block per (32-row strip, pair); wave w takes rows w, w+8, ...
// Emits T_row and the strip's row-threshold words RT[strip][j] (bit r: key(i0+r, j) <= T_row).
// ---------------------------------------------------------------------------------------
constexpr int kRowWaves = 8;

// Row select of one (32-row strip, pair) by NW waves: wave w takes rows w, w+NW, ...
template <int NW>
__device__ __forceinline__ void rows_body(const PairView& V, int p, int strip, const KeyPlanes& K, int ldr,
                                          int64_t kstride, float kappa, float* __restrict__ thr,
                                          float* __restrict__ Tq, int64_t thr_stride, uint32_t* __restrict__ RT,
                                          int64_t rt_stride, int ld, WaveLds* wl, uint32_t (*rowbits)[64]) {
  constexpr int KPL = 32;
  const int i0 = strip * kSR;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  WaveLds& W = wl[w];
  constexpr int RPW = kSR / NW;  // consecutive rows per wave: each search starts from its neighbour's
  unsigned hint = kNoHint;
#pragma unroll 1
  for (int r = w * RPW; r < (w + 1) * RPW; ++r) {
    const int i = i0 + r;
    uint32_t word = 0;
    if (i < V.Mp) {
      LineFull<KPL> L;
      L.load_full(K.fr + (size_t)p * kstride + (size_t)i * ldr, V.Np);
      float th, T;
      row_threshold(L, V.Np, kappa, W, &th, &T, &hint);
      if (lane == 0) {
        thr[(size_t)p * thr_stride + i] = th;
        Tq[(size_t)p * thr_stride + i] = T;
      }
      const unsigned Tb = __builtin_bit_cast(unsigned, T);
#pragma unroll
      for (int q = 0; q < KPL; ++q) word |= (uint32_t)(L.f[q] <= Tb) << q;  // 0xffffffff never <= T
    }
    rowbits[r][lane] = word;
  }
  __syncthreads();
  // transpose: word of column j = bit (j & 31) of rowbits[r][j >> 5], r = 0..31
  uint32_t* out = RT + (size_t)p * rt_stride + (size_t)strip * ld;
  for (int j = threadIdx.x; j < V.Np; j += NW * 64) {
    const int l = j >> 5, q = j & 31;
    uint32_t word = 0;
#pragma unroll
    for (int r = 0; r < kSR; ++r) word |= ((rowbits[r][l] >> q) & 1u) << r;
    out[j] = word;
  }
}

__global__ __launch_bounds__(512, 4) void k_sel_rows9(CrpBatch B, KeyPlanes K, int ldr, int64_t kstride, float kappa,
                                                   float* __restrict__ thr, float* __restrict__ Tq,
                                                   int64_t thr_stride, uint32_t* __restrict__ RT,
                                                   int64_t rt_stride, int ld) {
  __shared__ WaveLds wl[kRowWaves];
  __shared__ uint32_t rowbits[kSR][64];
  const int p = blockIdx.y;
  const PairView V = pair_view(B, p);
  const int strip = blockIdx.x;
  if (strip * kSR >= V.Mp) return;
  rows_body<kRowWaves>(V, p, strip, K, ldr, kstride, kappa, thr, Tq, thr_stride, RT, rt_stride, ld, wl, rowbits);
}

// Sweep and row select fused: the block selects the 32 rows it has just swept, reading its
// full keys back while they are cache-resident (no second pass over F from HBM, one launch
// fewer). LDS of the two phases is one union.
constexpr int kSweepLds = (kSYRows * 12 + kSCols) * 4 + kSCols * kTP * 2;
constexpr int kRowsLds = 4 * (int)sizeof(WaveLds) + kSR * 64 * 4;
constexpr int kFusedLds = kSweepLds > kRowsLds ? kSweepLds : kRowsLds;

__global__ __launch_bounds__(256, 4) void k_sweep_rows9(CrpBatch B, KeyPlanes K, int ldr, int ldc, int64_t kstride,
                                                     float kappa, float* __restrict__ thr, float* __restrict__ Tq,
                                                     int64_t thr_stride, uint32_t* __restrict__ RT, int64_t rt_stride,
                                                     int ld) {
  __shared__ __attribute__((aligned(16))) char smem[kFusedLds];
  float* Ys = reinterpret_cast<float*>(smem);
  float* Ns = Ys + kSYRows * 12;
  uint16_t* tileT = reinterpret_cast<uint16_t*>(Ns + kSCols);
  const int p = blockIdx.y;
  const PairView V = pair_view(B, p);
  const int strip = blockIdx.x, i0 = strip * kSR;
  if (i0 >= V.Mp || V.Np <= 0) return;
  if (V.tau == 1 && i0 + kSR <= V.Mp && i0 + kSR + kMS - 1 <= V.nq)
    sweep_body<true>(V, p, strip, K, ldr, ldc, kstride, Ys, Ns, tileT);
  else
    sweep_body<false>(V, p, strip, K, ldr, ldc, kstride, Ys, Ns, tileT);
  __syncthreads();  // the strip's F rows are complete (block-scope visibility of the global stores)
  rows_body<4>(V, p, strip, K, ldr, kstride, kappa, thr, Tq, thr_stride, RT, rt_stride, ld,
               reinterpret_cast<WaveLds*>(smem), reinterpret_cast<uint32_t(*)[64]>(smem + 4 * sizeof(WaveLds)));
}

// ---------------------------------------------------------------------------------------
// k_sel_cols9: one wave per CRP column; emits T_col and the column's CRP words.
// Lane l <-> rows 32l..32l+31 (KPL == 32).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sel_cols9(CrpBatch B, KeyPlanes K, int ldc, int64_t kstride, float kappa,
                                                   const uint32_t* __restrict__ RT, float* __restrict__ thr,
                                                   float* __restrict__ Tq, int64_t thr_stride,
                                                   uint32_t* __restrict__ maskT, int64_t mask_stride, int ld) {
  constexpr int KPL = 32;
  __shared__ WaveLds wl[4];
  // neighbouring columns share the lines of RT and of the F gathers: keep them on one XCD
  const int lb = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int p = lb / gridDim.x;
  const PairView V = pair_view(B, p);
  const int j = (lb - p * gridDim.x) * 4 + (threadIdx.x >> 6);
  if (j >= V.Np) return;
  WaveLds& W = wl[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  Line<KPL> L;
  L.load_lanes(K.hc + (size_t)p * kstride + (size_t)j * kSR, (size_t)ldc * kSR, V.Mp);
  const uint32_t* Fcol = K.fr + (size_t)p * kstride + j;
  auto keyf = [&](int e) { return Fcol[(size_t)e * ldc]; };
  float th, Tc;
  Group c_lo, c_hi;
  c_lo.g = c_hi.g = -1;
  unsigned hint = kNoHint;
  line_threshold(L, V.Mp, kappa, keyf, W, &c_lo, &c_hi, &th, &Tc, &hint);
  if (lane == 0) {
    thr[(size_t)p * thr_stride + j] = th;
    Tq[(size_t)p * thr_stride + j] = Tc;
  }
  const size_t w = (size_t)p * mask_stride + (size_t)lane * ld + j;
  const uint32_t bits = le_bits(L, __builtin_bit_cast(unsigned, Tc), keyf, W, c_lo, c_hi);
  if (lane * KPL >= V.Mp) return;
  maskT[w] = bits & RT[w];
}

}  // namespace

// Three-kernel CRP (m = 9, lines up to 2048 keys). Returns 1 if not applicable.
// kplanes: nb * kstride uint32 full keys, then nb * kstride uint16 prefixes; RT: nb * mask_stride
// words (same layout as maskT).
int launch_crp_split(const CrpBatch& B, int nb, int L, float kappa, void* kplanes, int ldk, int64_t kstride,
                     uint32_t* RT, float* thr_r, float* T_r, float* thr_c, float* T_c, int64_t thr_stride,
                     uint32_t* maskT, int64_t mask_stride, int ld, hipStream_t s) {
  if (B.m != kMS || L > 2048) return 1;
  const size_t plane = (size_t)nb * kstride;
  const KeyPlanes K{static_cast<uint32_t*>(kplanes), reinterpret_cast<uint16_t*>(static_cast<uint32_t*>(kplanes) + plane)};
  const int nstrips = (L + kSR - 1) / kSR;
  static const bool fused = [] {
    const char* e = getenv("ACOSS_FUSE_ROWS");
    return !(e && strcmp(e, "0") == 0);
  }();
  if (fused) {
    prof_begin(PH_SWEEP, s);
    hipLaunchKernelGGL(k_sweep_rows9, dim3(nstrips, nb), dim3(256), 0, s, B, K, ldk, ldk, kstride, kappa, thr_r, T_r,
                       thr_stride, RT, mask_stride, ld);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_SWEEP, s);
  } else {
    prof_begin(PH_SWEEP, s);
    hipLaunchKernelGGL(k_sweep9, dim3(nstrips, nb), dim3(kSW), 0, s, B, K, ldk, ldk, kstride);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_SWEEP, s);
    prof_begin(PH_SEL_ROWS, s);
    hipLaunchKernelGGL(k_sel_rows9, dim3(nstrips, nb), dim3(512), 0, s, B, K, ldk, kstride, kappa, thr_r, T_r,
                       thr_stride, RT, mask_stride, ld);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_SEL_ROWS, s);
  }
  prof_begin(PH_SEL_COLS, s);
  hipLaunchKernelGGL(k_sel_cols9, dim3((L + 3) / 4, nb), dim3(256), 0, s, B, K, ldk, kstride, kappa, RT, thr_c, T_c,
                     thr_stride, maskT, mask_stride, ld);
  ACOSS_LAUNCH_CHECK();
  prof_end(PH_SEL_COLS, s);
  return ACOSS_OK;
}

}  // namespace acoss
