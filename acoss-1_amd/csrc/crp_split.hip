// crp_split.hip — Serra09/Chen CRP (m = 9, tau = 1) in two kernels around ONE distance sweep.
//
// Replaces, per pair, the body of essentia ChromaCrossSimilarity (rqa_serra09.py:60-66,
// latefusion_chen.py:63-69): stacked distances, percentile(row/column, 9.5) and the mutual
// binary mask, bit-identical to oracle/crp_oracle.cpp.
//
//  k_sweep_rows9  one 256-thread block per (32-row strip, pair). Systolic walk (no LDS): lane =
//                 reference column, query frames as SGPR pairs, 9-term diagonal windows carried
//                 one lane per step by DPP; every squared-distance key leaves as its HIGH 16
//                 bits only, twice: row-major Hr[i][j] and strip-major Hc[i/32][j][32 rows in
//                 split word order]. Then the fused row select: one wave per CRP row on Hr, the
//                 16-bit prefixes of the two order statistics by a hinted SWAR-count search (7-bit
//                 window codes around the hint), the tied prefix group's exact keys RECOMPUTED
//                 (cell_key, one batched round, ~20-30 cells) and ranked -> percentile ->
//                 squared-domain threshold T_row; then the row's "key <= T_row" bits, transposed
//                 in LDS into the strip words RT.
//  k_sel_cols9    one wave per CRP column on Hc: the same select gives T_col; lane l then holds
//                 rows 32l..32l+31 of the column, i.e. exactly one 32-bit CRP word:
//                 (key <= T_col bits) & RT[strip l][j].
// The round-1 LDS diagonal walk and the MFMA Gram sweep (bit-exact, slower)
// were retired in round 2.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "crp_internal.hpp"

// v_writelane_b32 through the LLVM intrinsic (hipcc has no builtin for it), so the compiler's
// hazard recognizer inserts the wait state between the ballot's SGPR write and the writelane
// (the inline-asm form of round 3 lacked it and produced wrong words)
__device__ int acoss_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace acoss {

namespace {

constexpr int kMS = 9;

// 16-bit prefix of "no element": above every real prefix (finite keys >= +0 have prefixes <= 0x7f80)
constexpr unsigned kNone = 0x7fffu;


struct PairView {
  const float* X;   // query frames
  const float* X2;  // query frame pairs (f, f + 1) interleaved bin by bin (24 floats per f)
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
  v.X2 = B.feats2 ? B.feats2 + (size_t)ta * B.ldn * 24 : nullptr;
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
// Key planes of one pair: high 16 bits of every key, row-major (line = CRP row) and
// strip-major (line = CRP column).
struct KeyPlanes {
  uint16_t* hr;
  uint16_t* hc;
};

// Exact key of cell (i, j), recomputed in the sweep's canonical order: 12-term fmaf chain per
// frame pair (cell_gram), sequential 9-term sum, d2 = (NX_i - 2 dot) + NY_j clamped at +0
// (cell_finish). Valid cells only (i < M', j < N'): every frame is inside its track.
__device__ __forceinline__ float gram12(const f32x4& x0, const f32x4& x1, const f32x4& x2, const f32x4& y0,
                                        const f32x4& y1, const f32x4& y2) {
  float g = 0.0f;
  g = __builtin_fmaf(x0.x, y0.x, g);
  g = __builtin_fmaf(x0.y, y0.y, g);
  g = __builtin_fmaf(x0.z, y0.z, g);
  g = __builtin_fmaf(x0.w, y0.w, g);
  g = __builtin_fmaf(x1.x, y1.x, g);
  g = __builtin_fmaf(x1.y, y1.y, g);
  g = __builtin_fmaf(x1.z, y1.z, g);
  g = __builtin_fmaf(x1.w, y1.w, g);
  g = __builtin_fmaf(x2.x, y2.x, g);
  g = __builtin_fmaf(x2.y, y2.y, g);
  g = __builtin_fmaf(x2.z, y2.z, g);
  g = __builtin_fmaf(x2.w, y2.w, g);
  return g;
}

__device__ __forceinline__ float cell_gram(const PairView& V, int fq, int fr) {
  const f32x4* x = reinterpret_cast<const f32x4*>(V.X + (size_t)fq * 12);
  const f32x4* y = reinterpret_cast<const f32x4*>(V.Yr + (size_t)fr * 12);
  const f32x4 x0 = x[0], x1 = x[1], x2 = x[2], y0 = y[0], y1 = y[1], y2 = y[2];
  return gram12(x0, x1, x2, y0, y1, y2);
}

__device__ __forceinline__ unsigned cell_finish(const PairView& V, int i, int j, float dot) {
  const float d2 = (V.NXq[i] - 2.0f * dot) + V.NXr[j];
  return __builtin_bit_cast(unsigned, d2 > 0.0f ? d2 : 0.0f);
}

__device__ __forceinline__ unsigned cell_key(const PairView& V, int i, int j) {
  float dot = cell_gram(V, i * V.tau, j * V.tau);  // as the sweep: G_0, then + G_1 ... + G_8
#pragma unroll 1
  for (int u = 1; u < kMS; ++u) dot = dot + cell_gram(V, (i + u) * V.tau, (j + u) * V.tau);
  return cell_finish(V, i, j, dot);
}

// The cells of one CRP line: element e of row i is (i, e), of column j is (e, j). Holds the
// pair's pointers by value (a reference to the kernel's PairView would put it on the stack).
template <bool ROW>
struct LineCells {
  static constexpr bool kRow = ROW;
  PairView V;
  int fix;
  __device__ __forceinline__ int qi(int e) const { return ROW ? fix : e; }
  __device__ __forceinline__ int rj(int e) const { return ROW ? e : fix; }
  __device__ __forceinline__ unsigned operator()(int e) const { return cell_key(V, qi(e), rj(e)); }
};

typedef float f32x2 __attribute__((ext_vector_type(2)));
// Global-address-space u16 pointer: a pointer pinned to SGPRs by an empty asm loses its address
// space, and generic (flat) stores count in lgkmcnt too, so every s_waitcnt for the LDS reads
// would also wait for the previous rows' stores to be acknowledged.
typedef __attribute__((address_space(1))) uint16_t gu16;
// Store at a 32-bit byte offset from an SGPR base: global_store_short v_off, v, s[base] (saddr
// form; a u16 element index would need a 64-bit address per store).
__device__ __forceinline__ void st_u16(gu16* base, unsigned idx, unsigned v) {
  typedef __attribute__((address_space(1))) char gchar;
  *(gu16*)((gchar*)base + idx * 2u) = (uint16_t)v;
}

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// ---------------------------------------------------------------------------------------
// Systolic sweep (FAST strips: tau == 1, a full 32-row strip, all 40 query frames in the track).
// Lane l of a wave holds reference frame jb + l (12 VGPRs) for a whole column block; the
// strip's 40 query frames arrive as SGPR pairs (scalar loads of the interleaved frame pairs),
// and one packed-FP32 fmaf chain per step pair gives the lane's Gram terms G(i0 + kk, jb + l),
// G(i0 + kk + 1, jb + l) in the canonical order. The 9-term window of cell (r, c) starts on
// lane c - jb at step r and moves one lane per step (v_add_f32 with a DPP wave_shr:1 operand),
// collecting G(r + u, c + u) in the canonical sequential order; it completes on lane
// c - jb + 8 at step r + 8. Lanes 0..7 finish windows that began left of the block and are
// dropped: kSysCols = 56 valid columns per 64 lanes. No LDS and no barriers: each lane owns
// its output column's 32 rows, so the strip-major prefixes leave straight from registers (split
// word order) and a step's row-major prefixes are 56 consecutive columns.
// ---------------------------------------------------------------------------------------
constexpr int kSysCols = 56;
constexpr int kThreads = 256;  // sweep block: 4 waves

__device__ __forceinline__ float dpp_shr1(float v) {  // lane l <- lane l - 1 (lane 0 <- 0)
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}

// PARTIAL: the last strip of a pair (fewer than 32 rows in the track); the full strips keep a
// branch-free emit.
template <bool PARTIAL>
__device__ __forceinline__ void sweep_body_sys(const PairView& V, int p, int strip, const KeyPlanes& K, int ldr,
                                               int ldc, int64_t kstride, uint16_t* Hr) {
  constexpr int kSteps = kSR + kMS - 1;  // 40
  const int i0 = strip * kSR;
  const int rows = PARTIAL ? min(kSR, V.Mp - i0) : kSR;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint16_t* Hc = K.hc + (size_t)p * kstride;
  const float* X2b = V.X2 + (size_t)i0 * 24;
  const float* Nq0 = V.NXq + i0;
  auto nqr = [&](int r) {  // row norm: a scalar load at a compile-time offset
    const float* base = Nq0;
    asm volatile("" : "+s"(base));
    return *(const __attribute__((address_space(4))) float*)(base + r);
  };
  auto xpair = [&](int kk, f32x2 (&x)[12]) {  // (X_{i0+kk}[b], X_{i0+kk+1}[b]), scalar loads
    const float* base = X2b;
    asm volatile("" : "+s"(base));
    const cfloat4* q = (const cfloat4*)(base + kk * 24);
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const f32x4 v = q[c];
      x[2 * c] = f32x2{v.x, v.y};
      x[2 * c + 1] = f32x2{v.z, v.w};
    }
  };
  auto load_y = [&](int jb, f32x4 (&y)[3]) {
    const int f = min(jb + lane, V.nr - 1);  // frames past the track: only dropped cells use them
    const f32x4* src = reinterpret_cast<const f32x4*>(V.Yr + (size_t)f * 12);
    y[0] = src[0];
    y[1] = src[1];
    y[2] = src[2];
  };
  const int nblk = (V.Np + kSysCols - 1) / kSysCols;
  f32x4 ynext[3];
  if (w < nblk) load_y(w * kSysCols, ynext);
#pragma unroll 1
  for (int cb = w; cb < nblk; cb += 4) {
    const int jb = cb * kSysCols;
    float y[12];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      y[4 * q] = ynext[q].x;
      y[4 * q + 1] = ynext[q].y;
      y[4 * q + 2] = ynext[q].z;
      y[4 * q + 3] = ynext[q].w;
    }
    if (cb + 4 < nblk) load_y(jb + 4 * kSysCols, ynext);
    // this lane's output column; dropped lanes and columns past N' store to the pad column
    const int col = jb + lane - (kMS - 1);
    const bool valid = lane >= kMS - 1 && col < V.Np;
    const unsigned hcol = valid ? (unsigned)col : (unsigned)(ldr - 1);
    const float ny = valid ? V.NXr[col] : 0.0f;
    gu16* hrow = (gu16*)Hr;
    float A[kMS];  // A[u]: window of row kk - u after u + 1 terms
    unsigned kh[16];    // rows 0..15: full keys until their split partner (row + 16) is done
    unsigned hw[16];    // split-order words: rows (h, h + 16)
    f32x2 xb[12];
    xpair(0, xb);
#pragma unroll
    for (int kk = 0; kk < kSteps; kk += 2) {
      f32x2 g2 = pk_fma(xb[0], f32x2{y[0], y[0]}, f32x2{0.0f, 0.0f});
#pragma unroll
      for (int b = 1; b < 12; ++b) g2 = pk_fma(xb[b], f32x2{y[b], y[b]}, g2);
      if (kk + 2 < kSteps) xpair(kk + 2, xb);
      float dots[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = kk + h;
        const float g = h ? g2.y : g2.x;
#pragma unroll
        for (int u = kMS - 1; u >= 1; --u) {
          const int r = k - u;
          if (r >= 0 && r < kSR) A[u] = dpp_shr1(A[u - 1]) + g;
        }
        if (k < kSR) A[0] = g;
        dots[h] = A[kMS - 1];
      }
      const int r = kk - (kMS - 1);  // rows r, r + 1 complete on this step pair
      if (r >= 0) {
        const f32x2 nq = f32x2{nqr(r), nqr(r + 1)};
        const f32x2 d2 = pk_fma(f32x2{-2.0f, -2.0f}, f32x2{dots[0], dots[1]}, nq) + f32x2{ny, ny};
        unsigned k0 = __builtin_bit_cast(unsigned, d2.x > 0.0f ? d2.x : 0.0f);
        unsigned k1 = __builtin_bit_cast(unsigned, d2.y > 0.0f ? d2.y : 0.0f);
        if (!PARTIAL || r + 1 < rows) {  // wave-uniform; rows past M' are never stored
          st_u16(hrow, hcol, k0 >> 16);
          st_u16(hrow, (unsigned)ldr + hcol, k1 >> 16);
        } else {
          if (r < rows) st_u16(hrow, hcol, k0 >> 16);
          if (r >= rows) k0 = kNone << 16;  // and read as "no element" in the column plane
          k1 = kNone << 16;
        }
        hrow += 2 * ldr;
        asm volatile("" : "+s"(hrow));
        if (r < 16) {
          kh[r] = k0;
          kh[r + 1] = k1;
        } else {
          hw[r - 16] = __builtin_amdgcn_perm(k0, kh[r - 16], 0x07060302u);
          hw[r - 15] = __builtin_amdgcn_perm(k1, kh[r - 15], 0x07060302u);
        }
      }
    }
    // strip-major stores in 64-byte runs: a 4 x 4 transpose of the 16-byte pieces inside each lane
    // quad (two DPP butterfly stages per piece word), then store k: lane b + m (b = lane & ~3)
    // writes piece m of lane b + k's column, so a quad writes one column's 64 bytes contiguously
    // (each lane writing its own column's four pieces at a 64-byte stride: ACOSS_HC_LANE_STORES,
    // 1.5 % slower at 2,000 frames, profiles/r04/ab_hcquad2000.txt)
    {
      const int m = lane & 3, b = lane & ~3;
      const bool o1 = (m & 1) != 0, o2 = (m & 2) != 0;
      uint32_t T[4][4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t x0 = hw[d], x1 = hw[4 + d], x2 = hw[8 + d], x3 = hw[12 + d];
        // every DPP on all lanes (left to itself the compiler sinks them under the selects' exec
        // masks, where the partner lane is off and reads as 0)
        uint32_t p0 = dpp_u32<0xB1>(x0, x0), p1 = dpp_u32<0xB1>(x1, x1), p2 = dpp_u32<0xB1>(x2, x2),
                 p3 = dpp_u32<0xB1>(x3, x3);
        asm volatile("" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
        const uint32_t y0 = o1 ? p1 : x0, y1 = o1 ? x1 : p0, y2 = o1 ? p3 : x2, y3 = o1 ? x3 : p2;
        uint32_t q0 = dpp_u32<0x4E>(y0, y0), q1 = dpp_u32<0x4E>(y1, y1), q2 = dpp_u32<0x4E>(y2, y2),
                 q3 = dpp_u32<0x4E>(y3, y3);
        asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3));
        T[0][d] = o2 ? q2 : y0;
        T[1][d] = o2 ? q3 : y1;
        T[2][d] = o2 ? y2 : q0;
        T[3][d] = o2 ? y3 : q1;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = jb + b + k - (kMS - 1);
        if (b + k >= kMS - 1 && c < V.Np)
          reinterpret_cast<uint4*>(Hc + ((size_t)strip * ldc + c) * kSR)[m] = make_uint4(T[k][0], T[k][1], T[k][2], T[k][3]);
      }
    }
  }
  // kNone over [N', align32(N')) of every row: the row select's last 32-element run then needs
  // no tail mask. After the barrier, so it lands after the walk's stores (which went to valid
  // columns or the pad column only).
  __syncthreads();
  const int padw = (int)((V.Np + 31) & ~31) - V.Np;
  for (int e = threadIdx.x; e < kSR * 32; e += kThreads) {
    const int r = e >> 5, c = e & 31;
    if (c < padw && r < rows) Hr[(size_t)r * ldr + V.Np + c] = (uint16_t)kNone;
  }
}

// ---------------------------------------------------------------------------------------
// Per-wave select on one line (CRP row or column) of 16-bit key prefixes.
// Lane l holds elements [l*KPL, (l+1)*KPL) as KPL/2 packed words: element 2h in bits 0..15,
// 2h+1 in bits 16..31. Real prefixes are <= 0x7f80 (keys are >= +0, the sign bit is 0), so
// 0x7fff marks "no element" and every field keeps a free guard bit for SWAR arithmetic.
// ---------------------------------------------------------------------------------------

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

// Bits h and h + 16 of the result take the per-field flags (bits 15 and 31) of SWAR word h.
__device__ __forceinline__ uint32_t gather_flags(uint32_t acc, uint32_t s, int h) {
  return ((s >> (15 - h)) & (0x00010001u << h)) | acc;
}

// Lane l holds its KPL = 32 elements (element q = line element 32 l + q) as 16 packed words in
// SPLIT order: word h = element h (bits 0..15) and element h + 16 (bits 16..31). In this order
// the flag bits of a SWAR compare on word h (bits 15 and 31) become mask bits h and h + 16 with
// one shift and one and-or, so an element mask costs 3 VALU per word.
__device__ __forceinline__ unsigned pk_subsat_u16(unsigned a, unsigned b) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}

// Smallest prefix > x (x < kNone) among a lane's packed words, or 0xffffffff: per field
// (k - x - 1) mod 2^16 (one wrapping packed add) puts every real k > x at k - x - 1 <= 0x7f80 - x - 1,
// kNone at 0x7fff - x - 1 and every k <= x at >= 0x10000 - x - 1, so a packed minimum and one
// compare find it (2 VALU per word; the per-element compare/select form took ~7 per element).
template <int NW>
__device__ __forceinline__ unsigned swar_min_greater(const unsigned (&pv)[NW], unsigned x) {
  const unsigned X = ((0x10000u - x - 1u) & 0xffffu) * 0x10001u;
  unsigned a = 0xffffffffu;
#pragma unroll
  for (int h = 0; h < NW; ++h) a = pk_min_u16(a, pk_add_u16(pv[h], X));
  const unsigned d = min(a & 0xffffu, a >> 16);
  return d < kNone - x - 1u ? d + x + 1u : 0xffffffffu;
}

// Bits h, h + 8, h + 16, h + 24 of the result take the flags (bits 7, 15, 23, 31) of word h.
__device__ __forceinline__ uint32_t gather_flags8(uint32_t acc, uint32_t s, int h) {
  return ((s >> (7 - h)) & (0x01010101u << h)) | acc;
}

// Unconditional histogram adds: an element outside the bins goes to this lane's own sink word
// (the 64 words after the 128 bins, WaveLds::sink; a lane-private address, no bank conflict), so
// every element issues the same ds_add instead of a compare, an exec-mask save / restore and a
// masked add. Used by the window-code histogram (hist_rank_w8); the 16-bit-prefix histograms keep
// the masked add (hist_add below), where the sink measured 6 % slower at 500 frames.
typedef __attribute__((address_space(3))) unsigned lds_u32;
// 32-bit LDS addresses of a wave's histogram: the bins' base as an SGPR (bin address = c * 4 +
// base in one v_lshl_add) and this lane's sink word
struct HistAddr {
  unsigned hb, sk;
  __device__ __forceinline__ explicit HistAddr(unsigned* hist) {
    hb = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(size_t)(lds_u32*)hist);
    sk = hb + 512u + 4u * (threadIdx.x & 63);
  }
};
__device__ __forceinline__ void hist_add(unsigned* hist, const HistAddr& A, unsigned c, bool in) {
  if (in) __hip_atomic_fetch_add(hist + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// The rank search of hist_rank on a line's 7-bit window codes (w8: four codes per word; window
// base8 = hint - 63, code c <-> prefix base8 + c exactly for c in 1..126, and for c = 0 too when
// base8 = 0; code 0 otherwise means "at or below base8", 127 "at or above base8 + 127"): every
// code below 127 is counted into its LDS bin straight from its byte (bin 0 then holds the
// elements at or below base8), and one wave scan of the bins places rank rho. False when the
// answer is not an exact code (above the window, or in bin 0 of a window above 0).
template <int NW>
__device__ __forceinline__ bool hist_rank_w8(const unsigned (&w8)[NW], unsigned base8, int rho, unsigned* hist,
                                             unsigned* P, int* le, int* less) {
  const int lane = threadIdx.x & 63;
  reinterpret_cast<uint2*>(hist)[lane] = make_uint2(0u, 0u);
  __builtin_amdgcn_wave_barrier();
  const unsigned cmin = base8 == 0u ? 0u : 1u;  // code 0 is exact only when base8 == 0
  // every code below 127 into its bin, code 0 included (the elements at or below base8, exact
  // only when base8 == 0: a rank landing in bin 0 otherwise returns false below), so no separate
  // count of the elements under the window; code 127 to this lane's sink; no exec masking.
  // The sink select is done on a whole word at once (SWAR): byte k of wp = code + 1 (1..128, no
  // carry between bytes); the bytes at 128 (code 127) get lane + 1 more, to 129 + lane; then bin
  // index b - 1 for every byte b, so the sink of lane l is index 128 + l (A.sk). Per code one byte
  // extract and one address, per word six ops (a per-code compare, hazard nop and select measured
  // 0.8 % slower end to end).
  const HistAddr A(hist);
  const unsigned lane1 = (unsigned)(lane + 1) * 0x01010101u;  // lane + 1 (<= 64) in every byte
  const unsigned hbm = A.hb - 4u;
#pragma unroll
  for (int h = 0; h < NW; ++h) {
    const unsigned wp = w8[h] + 0x01010101u;
    const unsigned H = wp & 0x80808080u;
    const unsigned S = wp + ((H - (H >> 7)) & lane1);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned a = hbm + 4u * ((S >> (8 * k)) & 0xffu);
      __hip_atomic_fetch_add((lds_u32*)(size_t)a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  }
  __builtin_amdgcn_wave_barrier();
  const uint2 hv = reinterpret_cast<const uint2*>(hist)[lane];
  const int sl = (int)(hv.x + hv.y);
  const int S = wave_incl_scan(sl);
  const int tot = __builtin_amdgcn_readlane(S, 63);
  const int r = rho;
  if (r < 0 || r >= tot) return false;
  const int E = S - sl;
  const int src = __builtin_ctzll(__ballot(E <= r && r < S));
  const int Es = __builtin_amdgcn_readlane(E, src);
  const int h0 = __builtin_amdgcn_readlane((int)hv.x, src), h1 = __builtin_amdgcn_readlane((int)hv.y, src);
  const bool second = r >= Es + h0;
  if (cmin && src == 0 && !second) return false;  // bin 0 of a window above 0: not an exact prefix
  *P = base8 + 2u * (unsigned)src + (second ? 1u : 0u);
  *less = Es + (second ? h0 : 0);
  *le = *less + (second ? h1 : h0);
  return true;
}

template <int KPL>
struct Line {
  static_assert(KPL == 32, "split word order assumes 32 elements per lane");
  unsigned pv[KPL / 2];
  // Optional 7-bit window around a hint: w8 holds min(max(prefix - base8, 0), 127) for the
  // lane's 32 elements, four per word (word h = elements h, h + 8, h + 16, h + 24). For
  // thresholds in [base8, base8 + 126] it answers count / member / le queries exactly at half
  // the VALU of the 16-bit words (codes 0 and 127 are the saturated "below" and "above" classes).
  unsigned w8[KPL / 4];
  unsigned base8;
  bool win;
  __device__ __forceinline__ void build_window(unsigned center) {
    base8 = center > 63u ? center - 63u : 0u;
    win = true;
    const unsigned B2 = base8 * 0x10001u;
    unsigned c[KPL / 2];
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) c[h] = pk_min_u16(pk_subsat_u16(pv[h], B2), 0x007f007fu);
#pragma unroll
    for (int h = 0; h < KPL / 4; ++h) w8[h] = __builtin_amdgcn_perm(c[h + 8], c[h], 0x06020400u);
  }
  __device__ __forceinline__ bool in_win(unsigned x) const { return win && x >= base8 && x <= base8 + 126u; }
  // element of mask bit b: lane * KPL + b (ebase() opaque, so element indices are not hoisted
  // out of callers' loops)
  __device__ __forceinline__ int ebase() const {
    int e = (threadIdx.x & 63) * KPL;
    asm volatile("" : "+v"(e));
    return e;
  }
  __device__ __forceinline__ int elem(int eb, int b) const { return eb + b; }
  static __device__ __forceinline__ int lane_of(int e) { return e / KPL; }
  static __device__ __forceinline__ int bit_of(int e) { return e % KPL; }
  // sample for sample_hint: element KPL * lane (kNone past the line)
  __device__ __forceinline__ unsigned sample() const { return pv[0] & 0xffffu; }
  __device__ __forceinline__ unsigned pfx(int q) const { return q < 16 ? (pv[q] & 0xffffu) : (pv[q - 16] >> 16); }
  // Lane l's KPL elements start at col0 + l * lane_stride. STORED_SPLIT: the plane holds every
  // run in split order already (the strip-major column plane, written so by the sweep);
  // otherwise (row-major plane, natural order) the loaded pairs are repacked, one v_perm per word.
  template <bool STORED_SPLIT>
  __device__ __forceinline__ void load_lanes(const uint16_t* col0, size_t lane_stride, int n) {
    const int lane = threadIdx.x & 63;
    const int base = lane * KPL;
    // every lane loads a whole run: the lane holding the end of the line reads its run in full
    // (runs lie inside the plane: the row pitch and the strips are whole runs) and masks the
    // tail; lanes past the line re-read lane 0's run and mask all of it. No per-element
    // conditional loads: hipcc branches around each and waits vmcnt(0) after each (16-32
    // serial L2 round trips per line)
    // (lanes past the line reading a constant run of kNone instead of the fill below: -1 % at
    // 2,000 frames, profiles/r04/ab_q2000.txt)
    const uint16_t* src = col0 + (base < n ? (size_t)lane * lane_stride : (size_t)0);
    win = false;
    base8 = 0u;
    unsigned w[KPL / 2];
#pragma unroll
    for (int q = 0; q < KPL / 8; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(src)[q];
      w[4 * q + 0] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
    if (STORED_SPLIT) {
#pragma unroll
      for (int h = 0; h < KPL / 2; ++h) pv[h] = w[h];
    } else {
#pragma unroll
      for (int h = 0; h < KPL / 2; ++h)  // (element h, element h + 16) from natural pairs
        pv[h] = __builtin_amdgcn_perm(w[8 + (h >> 1)], w[h >> 1], (h & 1) ? 0x07060302u : 0x05040100u);
    }
    // the planes hold kNone past the line's end inside the last run (the sweep stores it), so
    // only lanes wholly past the line need filling
    if (base >= n) {
#pragma unroll
      for (int h = 0; h < KPL / 2; ++h) pv[h] = kNone * 0x10001u;
    }
  }
  // #elements <= x (x <= 0x7fff): per field (x + 0x8000) - a keeps bit 15 iff a <= x, with no
  // borrow across fields; popcount on VALU, one DPP wave sum (no SGPR per compare, no SALU).
  // branch-free pieces (window codes / 16-bit words) for Line2, which picks by in_win once for
  // both halves (the branching forms below are kept for the long lines' own codegen)
  __device__ __forceinline__ unsigned cnt8(unsigned x) const {
    const unsigned X4 = (x - base8 + 0x80u) * 0x01010101u;
    unsigned c = 0;
#pragma unroll
    for (int h = 0; h < KPL / 4; ++h) c = __builtin_popcount((X4 - w8[h]) & 0x80808080u) + c;
    return c;
  }
  __device__ __forceinline__ unsigned cnt16(unsigned x) const {
    const unsigned X2 = (x + 0x8000u) * 0x10001u;
    unsigned c = 0;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) c = __builtin_popcount((X2 - pv[h]) & 0x80008000u) + c;
    return c;
  }
  __device__ __forceinline__ int count_le(unsigned x) const {
    if (in_win(x)) {  // wave-uniform
      const unsigned X4 = (x - base8 + 0x80u) * 0x01010101u;
      unsigned c = 0;
#pragma unroll
      for (int h = 0; h < KPL / 4; ++h) c = __builtin_popcount((X4 - w8[h]) & 0x80808080u) + c;
      return wave_sum((int)c);
    }
    const unsigned X2 = (x + 0x8000u) * 0x10001u;
    unsigned c = 0;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) c = __builtin_popcount((X2 - pv[h]) & 0x80008000u) + c;
    return wave_sum((int)c);
  }
  // Bit q set iff element q's prefix == P (P <= kCodeMax). Per field, (a ^ P) + 0x7fff keeps bit
  // 15 iff a != P; fields are <= 0x7fff, so nothing carries across.
  __device__ __forceinline__ bool eq_in_win(unsigned P) const {
    return in_win(P) && (P > base8 || base8 == 0u);  // code 0 is exact only when base8 == 0
  }
  __device__ __forceinline__ uint32_t eq8(unsigned P) const {
    const unsigned PP = (P - base8) * 0x01010101u;
    uint32_t ne8 = 0;
#pragma unroll
    for (int h = 0; h < KPL / 4; ++h) ne8 = gather_flags8(ne8, (w8[h] ^ PP) + 0x7f7f7f7fu, h);
    return ~ne8;
  }
  __device__ __forceinline__ uint32_t eq16(unsigned P) const {
    const unsigned PP = P * 0x10001u;
    uint32_t ne = 0;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) ne = gather_flags(ne, (pv[h] ^ PP) + 0x7fff7fffu, h);
    return ~ne;
  }
  __device__ __forceinline__ uint32_t eq_mask(unsigned P) const {
    if (in_win(P) && (P > base8 || base8 == 0u)) {  // code 0 is exact only when base8 == 0
      const unsigned PP = (P - base8) * 0x01010101u;
      uint32_t ne8 = 0;
#pragma unroll
      for (int h = 0; h < KPL / 4; ++h) ne8 = gather_flags8(ne8, (w8[h] ^ PP) + 0x7f7f7f7fu, h);
      return ~ne8;
    }
    const unsigned PP = P * 0x10001u;
    uint32_t ne = 0;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) ne = gather_flags(ne, (pv[h] ^ PP) + 0x7fff7fffu, h);
    return ~ne;
  }
  // Bit q set iff element q's prefix <= x (x <= 0x7fff; kNone is never <= a real x).
  __device__ __forceinline__ uint32_t le8(unsigned x) const {
    const unsigned X4 = (x - base8 + 0x80u) * 0x01010101u;
    uint32_t le8 = 0;
#pragma unroll
    for (int h = 0; h < KPL / 4; ++h) le8 = gather_flags8(le8, X4 - w8[h], h);
    return le8;
  }
  __device__ __forceinline__ uint32_t le16(unsigned x) const {
    const unsigned X2 = (x + 0x8000u) * 0x10001u;
    uint32_t le = 0;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) le = gather_flags(le, X2 - pv[h], h);
    return le;
  }
  __device__ __forceinline__ uint32_t le_mask(unsigned x) const {
    if (in_win(x)) {
      const unsigned X4 = (x - base8 + 0x80u) * 0x01010101u;
      uint32_t le8 = 0;
#pragma unroll
      for (int h = 0; h < KPL / 4; ++h) le8 = gather_flags8(le8, X4 - w8[h], h);
      return le8;
    }
    const unsigned X2 = (x + 0x8000u) * 0x10001u;
    uint32_t le = 0;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) le = gather_flags(le, X2 - pv[h], h);
    return le;
  }
  // min over elements (kNone is above every real prefix) and max over real elements
  // (kNone + 1 wraps to 0x8000, masked to 0: below every real prefix + 1); lane shares first
  __device__ __forceinline__ void min_max_lane(unsigned* a_io, unsigned* b_io) const {
    unsigned a = *a_io, b = *b_io;
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) {
      a = pk_min_u16(a, pv[h]);
      b = pk_max_u16(b, pk_add_u16(pv[h], 0x00010001u) & 0x7fff7fffu);
    }
    *a_io = a;
    *b_io = b;
  }
  __device__ __forceinline__ void min_max(unsigned* mn, unsigned* mx) const {
    unsigned a = 0xffffffffu, b = 0u;
    min_max_lane(&a, &b);
    a = min(a & 0xffffu, a >> 16);
    b = max(b & 0xffffu, b >> 16);
    *mn = wave_min_u32(a);
    const unsigned m = wave_max_u32(b);
    *mx = m ? m - 1 : 0u;
  }
  __device__ __forceinline__ unsigned min_greater_lane(unsigned x) const { return swar_min_greater(pv, x); }
  __device__ __forceinline__ unsigned min_greater(unsigned x) const { return wave_min_u32(min_greater_lane(x)); }
  static constexpr int kHalves = 1;
  // LineS::hist_rank for the 32 elements per lane of a long line
  static constexpr bool kHist = true;
  __device__ __forceinline__ bool hist_rank(unsigned hint, int rho, unsigned* hist, unsigned* P, int* le,
                                            int* less, unsigned* hbase) const {
    if (win) {  // the window codes around the same hint (built before every hinted search)
      *hbase = base8;
      return hist_rank_w8(w8, base8, rho, hist, P, le, less);
    }
    const int lane = threadIdx.x & 63;
    const unsigned base = hint > 64u ? hint - 64u : 0u;
    *hbase = base;
    reinterpret_cast<uint2*>(hist)[lane] = make_uint2(0u, 0u);
    __builtin_amdgcn_wave_barrier();
    const HistAddr HA(hist);
    unsigned below = 0;
    if (base > 0u) {
      const unsigned X2 = (base - 1u + 0x8000u) * 0x10001u;
#pragma unroll
      for (int h = 0; h < KPL / 2; ++h) below = __builtin_popcount((X2 - pv[h]) & 0x80008000u) + below;
    }
#pragma unroll
    for (int h = 0; h < KPL / 2; ++h) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const unsigned c = (half ? (pv[h] >> 16) : (pv[h] & 0xffffu)) - base;
        hist_add(hist, HA, c, c < 128u);
      }
    }
    const int below_tot = wave_sum((int)below);
    __builtin_amdgcn_wave_barrier();
    const uint2 hv = reinterpret_cast<const uint2*>(hist)[lane];
    const int sl = (int)(hv.x + hv.y);
    const int S = wave_incl_scan(sl);
    const int tot = __builtin_amdgcn_readlane(S, 63);
    const int r = rho - below_tot;
    if (r < 0 || r >= tot) return false;
    const int E = S - sl;
    const int src = __builtin_ctzll(__ballot(E <= r && r < S));
    const int Es = __builtin_amdgcn_readlane(E, src);
    const int h0 = __builtin_amdgcn_readlane((int)hv.x, src), h1 = __builtin_amdgcn_readlane((int)hv.y, src);
    const bool second = r >= Es + h0;
    *P = base + 2u * (unsigned)src + (second ? 1u : 0u);
    *less = below_tot + Es + (second ? h0 : 0);
    *le = *less + (second ? h1 : h0);
    return true;
  }
};

// Short lines (up to 64 KQ elements): lane l holds elements l + 64 q, q < KQ,
// so a wave-wide ballot of one mask bit is two consecutive 32-element words of the line (the
// CRP's row and strip words) and every load is coalesced across the wave. KQ/2 packed words:
// word h = element q = h (bits 0..15) and q = h + KQ/2 (bits 16..31); mask bit h <-> q = h and
// bit h + 16 <-> q = h + KQ/2, the same flag gather as the long lines' split order. KQ = 16
// adds the long lines' 7-bit window codes (4 words: word h = elements q = h + 4k, k = 0..3, one
// per byte; its flag gather puts q = h + 4k on bit h + 8k, which wmask moves to the 16-bit
// layout's bits); KQ = 8 searches its 4 words directly.
template <int KQ>
struct LineS {
  static_assert(KQ == 8 || KQ == 16, "short lines: 8 or 16 elements per lane");
  static constexpr bool kWin = KQ == 16;
  unsigned pv[KQ / 2];
  unsigned w8[kWin ? KQ / 4 : 1];
  unsigned base8;
  bool win;
  static constexpr uint32_t kWinLo = ((1u << (KQ / 4)) - 1u) * 0x10001u;
  static __device__ __forceinline__ uint32_t wmask(uint32_t m) {
    return (m & kWinLo) | ((m >> (8 - KQ / 4)) & (kWinLo << (KQ / 4)));
  }
  __device__ __forceinline__ void build_window(unsigned center) {
    static_assert(kWin, "window codes: 16 codes per lane only");
    base8 = center > 63u ? center - 63u : 0u;
    win = true;
    const unsigned B2 = base8 * 0x10001u;
    unsigned c[KQ / 2];
#pragma unroll
    for (int h = 0; h < KQ / 2; ++h) c[h] = pk_min_u16(pk_subsat_u16(pv[h], B2), 0x007f007fu);
#pragma unroll
    for (int h = 0; h < KQ / 4; ++h) w8[h] = __builtin_amdgcn_perm(c[h + KQ / 4], c[h], 0x06020400u);
  }
  __device__ __forceinline__ bool in_win(unsigned x) const { return win && x >= base8 && x <= base8 + 126u; }
  static __device__ __forceinline__ int q_of_bit(int b) { return b < 16 ? b : b - 16 + KQ / 2; }
  static __device__ __forceinline__ int bit_of_q(int q) { return q < KQ / 2 ? q : q - KQ / 2 + 16; }
  __device__ __forceinline__ int ebase() const {
    int e = threadIdx.x & 63;
    asm volatile("" : "+v"(e));
    return e;
  }
  __device__ __forceinline__ int elem(int eb, int b) const { return eb + 64 * q_of_bit(b); }
  static __device__ __forceinline__ int lane_of(int e) { return e & 63; }
  static __device__ __forceinline__ int bit_of(int e) { return bit_of_q(e >> 6); }
  __device__ __forceinline__ unsigned pfx(int q) const {
    return q < KQ / 2 ? (pv[q] & 0xffffu) : (pv[q - KQ / 2] >> 16);
  }
  // sample for sample_hint: element l + 64 (l mod KQ), spread over the line
  __device__ __forceinline__ unsigned sample() const {
    // a mux tree on the lane bits (an index compare chain becomes a scratch-array lookup)
    const int lane = threadIdx.x & 63;
    unsigned t[KQ / 2];
#pragma unroll
    for (int k = 0; k < KQ / 2; ++k) t[k] = pv[k];
#pragma unroll
    for (int bit = 1, n = KQ / 2; n > 1; bit <<= 1, n >>= 1) {
      const bool sel = (lane & bit) != 0;
#pragma unroll
      for (int k = 0; k < n / 2; ++k) t[k] = sel ? t[2 * k + 1] : t[2 * k];
    }
    return (lane & (KQ / 2)) ? (t[0] >> 16) : (t[0] & 0xffffu);
  }
  // the n codes of a line; addr(e): where element e's code is. Every lane loads (elements past
  // the line re-read element n - 1 and are replaced by kNone): no per-element branches.
  template <class AT>
  __device__ __forceinline__ void load(AT addr, int n) {
    const int lane = threadIdx.x & 63;
    if constexpr (kWin) {
      win = false;
      base8 = 0u;
    }
    unsigned v[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) v[q] = *addr(min(lane + 64 * q, n - 1));
#pragma unroll
    for (int q = 0; q < KQ; ++q) v[q] = lane + 64 * q < n ? v[q] : kNone;
#pragma unroll
    for (int h = 0; h < KQ / 2; ++h) pv[h] = v[h] | (v[h + KQ / 2] << 16);
  }
  __device__ __forceinline__ int count_le(unsigned x) const {
    if constexpr (kWin) {
      if (in_win(x)) {  // wave-uniform
        const unsigned X4 = (x - base8 + 0x80u) * 0x01010101u;
        unsigned c = 0;
#pragma unroll
        for (int h = 0; h < KQ / 4; ++h) c = __builtin_popcount((X4 - w8[h]) & 0x80808080u) + c;
        return wave_sum((int)c);
      }
    }
    const unsigned X2 = (x + 0x8000u) * 0x10001u;
    unsigned c = 0;
#pragma unroll
    for (int h = 0; h < KQ / 2; ++h) c = __builtin_popcount((X2 - pv[h]) & 0x80008000u) + c;
    return wave_sum((int)c);
  }
  __device__ __forceinline__ uint32_t eq_mask(unsigned P) const {
    if constexpr (kWin) {
      if (in_win(P) && (P > base8 || base8 == 0u)) {  // code 0 is exact only when base8 == 0
        const unsigned PP = (P - base8) * 0x01010101u;
        uint32_t ne8 = 0;
#pragma unroll
        for (int h = 0; h < KQ / 4; ++h) ne8 = gather_flags8(ne8, (w8[h] ^ PP) + 0x7f7f7f7fu, h);
        return wmask(~ne8);
      }
    }
    const unsigned PP = P * 0x10001u;
    uint32_t ne = 0;
#pragma unroll
    for (int h = 0; h < KQ / 2; ++h) ne = gather_flags(ne, (pv[h] ^ PP) + 0x7fff7fffu, h);
    return ~ne & kMaskAll;
  }
  __device__ __forceinline__ uint32_t le_mask(unsigned x) const {
    if constexpr (kWin) {
      if (in_win(x)) {
        const unsigned X4 = (x - base8 + 0x80u) * 0x01010101u;
        uint32_t le8 = 0;
#pragma unroll
        for (int h = 0; h < KQ / 4; ++h) le8 = gather_flags8(le8, X4 - w8[h], h);
        return wmask(le8);
      }
    }
    const unsigned X2 = (x + 0x8000u) * 0x10001u;
    uint32_t le = 0;
#pragma unroll
    for (int h = 0; h < KQ / 2; ++h) le = gather_flags(le, X2 - pv[h], h);
    return le;
  }
  static constexpr uint32_t kMaskAll = ((1u << (KQ / 2)) - 1u) * 0x10001u;
  static constexpr int kHalves = 1;
  __device__ __forceinline__ void min_max(unsigned* mn, unsigned* mx) const {
    unsigned a = 0xffffffffu, b = 0u;
#pragma unroll
    for (int h = 0; h < KQ / 2; ++h) {
      a = pk_min_u16(a, pv[h]);
      b = pk_max_u16(b, pk_add_u16(pv[h], 0x00010001u) & 0x7fff7fffu);
    }
    a = min(a & 0xffffu, a >> 16);
    b = max(b & 0xffffu, b >> 16);
    *mn = wave_min_u32(a);
    const unsigned m = wave_max_u32(b);
    *mx = m ? m - 1 : 0u;
  }
  __device__ __forceinline__ unsigned min_greater(unsigned x) const { return wave_min_u32(swar_min_greater(pv, x)); }
  // Prefix of rank rho (0-based: the least P with count(<= P) > rho) from ONE pass over the line:
  // every element inside the 128-prefix window [base, base + 128) around the hint (the previous
  // line's answer; adjacent lines share 8 of their 9 stacked frames, so the answer lies inside
  // the window for about 99 % of the lines) is counted into its LDS bin, the elements below the
  // window by one SWAR count; one wave scan of the bins then places rank rho. Two wave reductions
  // instead of the search's ~5 dependent count passes. Returns false, deciding nothing, when the
  // answer lies outside the window. le / less: count(<= P) / count(< P), as prefix_of_rank.
  static constexpr bool kHist = true;
  __device__ __forceinline__ bool hist_rank(unsigned hint, int rho, unsigned* hist, unsigned* P, int* le,
                                            int* less, unsigned* hbase) const {
    if constexpr (kWin) {
      if (win) {
        *hbase = base8;
        return hist_rank_w8(w8, base8, rho, hist, P, le, less);
      }
    }
    const int lane = threadIdx.x & 63;
    const unsigned base = hint > 64u ? hint - 64u : 0u;
    *hbase = base;
    reinterpret_cast<uint2*>(hist)[lane] = make_uint2(0u, 0u);
    __builtin_amdgcn_wave_barrier();
    const HistAddr HA(hist);
    // elements below the window (kNone never is): #(prefix <= base - 1), SWAR as count_le
    unsigned below = 0;
    if (base > 0u) {
      const unsigned X2 = (base - 1u + 0x8000u) * 0x10001u;
#pragma unroll
      for (int h = 0; h < KQ / 2; ++h) below = __builtin_popcount((X2 - pv[h]) & 0x80008000u) + below;
    }
#pragma unroll
    for (int h = 0; h < KQ / 2; ++h) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const unsigned p = half ? (pv[h] >> 16) : (pv[h] & 0xffffu);
        // (wraps for p < base; kNone, 0x7fff, is never inside: base <= 0x7f80 - 64)
        const unsigned c = p - base;
        hist_add(hist, HA, c, c < 128u);
      }
    }
    const int below_tot = wave_sum((int)below);
    __builtin_amdgcn_wave_barrier();
    const uint2 hv = reinterpret_cast<const uint2*>(hist)[lane];
    const int sl = (int)(hv.x + hv.y);
    const int S = wave_incl_scan(sl);
    const int tot = __builtin_amdgcn_readlane(S, 63);
    const int r = rho - below_tot;
    if (r < 0 || r >= tot) return false;  // wave-uniform: the answer is outside the window
    const int E = S - sl;
    const int src = __builtin_ctzll(__ballot(E <= r && r < S));
    const int Es = __builtin_amdgcn_readlane(E, src);
    const int h0 = __builtin_amdgcn_readlane((int)hv.x, src), h1 = __builtin_amdgcn_readlane((int)hv.y, src);
    const bool second = r >= Es + h0;
    *P = base + 2u * (unsigned)src + (second ? 1u : 0u);
    *less = below_tot + Es + (second ? h0 : 0);
    *le = *less + (second ? h1 : h0);
    return true;
  }
};

// Lane t's 32-bit line word t (elements 32 t .. 32 t + 31) from a short line's per-lane mask:
// word 2q + half is the low / high half of the ballot of bit q. Lanes past 2 KQ get 0.
template <int KQ>
__device__ __forceinline__ uint32_t lane_words(uint32_t mask) {
  // each ballot half is wave-uniform (an SGPR): one v_writelane_b32 places it on its lane
  uint32_t out = 0;
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const unsigned long long bal = __ballot((mask >> LineS<KQ>::bit_of_q(q)) & 1u);
    out = (uint32_t)acoss_writelane((int)(uint32_t)bal, 2 * q, (int)out);
    out = (uint32_t)acoss_writelane((int)(uint32_t)(bal >> 32), 2 * q + 1, (int)out);
  }
  return out;
}

// Lines of 2049..4096 codes: two long-line halves held by one wave, elements [0, 2048) in A
// and [2048, n) in B (lane l: elements 32 l.. and 2048 + 32 l..). One wave sum per count; masks
// are 64-bit (A in bits 0..31, B in 32..63); the le words of B live in W.words[64 + lane].
struct Line2 {
  Line<32> A, B;
  static constexpr int kHalves = 2;
  static constexpr bool kHist = false;
  __device__ __forceinline__ int ebase() const { return A.ebase(); }
  __device__ __forceinline__ int elem(int eb, int b) const { return b < 32 ? eb + b : 2048 + eb + (b - 32); }
  static __device__ __forceinline__ int lane_of(int e) { return e < 2048 ? (e >> 5) : 64 + ((e - 2048) >> 5); }
  static __device__ __forceinline__ int bit_of(int e) { return e & 31; }
  // sample: even lanes from A (element 32 l), odd lanes from B (element 2048 + 32 l)
  __device__ __forceinline__ unsigned sample() const {
    const unsigned a = A.sample(), b = B.sample();  // (selecting the half object would keep both in scratch)
    return (threadIdx.x & 1) ? b : a;
  }
  __device__ __forceinline__ void build_window(unsigned c) {
    A.build_window(c);
    B.build_window(c);
  }
  // (both halves share the window, so one wave-uniform branch serves both: branching per half
  // lets the compiler merge the two halves' paths into pointer phis, which keeps the line in scratch)
  __device__ __forceinline__ int count_le(unsigned x) const {
    if (A.in_win(x)) return wave_sum((int)(A.cnt8(x) + B.cnt8(x)));
    return wave_sum((int)(A.cnt16(x) + B.cnt16(x)));
  }
  __device__ __forceinline__ uint64_t eq_mask(unsigned P) const {
    if (A.eq_in_win(P)) return (uint64_t)A.eq8(P) | ((uint64_t)B.eq8(P) << 32);
    return (uint64_t)A.eq16(P) | ((uint64_t)B.eq16(P) << 32);
  }
  __device__ __forceinline__ uint64_t le_mask(unsigned x) const {
    if (A.in_win(x)) return (uint64_t)A.le8(x) | ((uint64_t)B.le8(x) << 32);
    return (uint64_t)A.le16(x) | ((uint64_t)B.le16(x) << 32);
  }
  __device__ __forceinline__ void min_max(unsigned* mn, unsigned* mx) const {
    unsigned a = 0xffffffffu, b = 0u;
    A.min_max_lane(&a, &b);
    B.min_max_lane(&a, &b);
    a = min(a & 0xffffu, a >> 16);
    b = max(b & 0xffffu, b >> 16);
    *mn = wave_min_u32(a);
    const unsigned m = wave_max_u32(b);
    *mx = m ? m - 1 : 0u;
  }
  __device__ __forceinline__ unsigned min_greater(unsigned x) const {
    return wave_min_u32(min(A.min_greater_lane(x), B.min_greater_lane(x)));
  }
};

__device__ __forceinline__ int popc(uint32_t m) { return __builtin_popcount(m); }
__device__ __forceinline__ int popc(uint64_t m) { return __builtin_popcountll(m); }
__device__ __forceinline__ int ctz(uint32_t m) { return __builtin_ctz(m); }
__device__ __forceinline__ int ctz(uint64_t m) { return __builtin_ctzll(m); }

// Smallest prefix P with count(keys <= P) > rho, bisecting [a, b]; also returns
// le = count(<= P) and less = count(< P) (carried through the search: no extra counts).
// hint (wave-uniform, or kNoHint): the previous line's answer. Adjacent stacked rows/columns
// share 8 of their 9 frames, so the answer is usually a few prefixes away: gallop out from
// the hint to a bracket, then bisect inside it.
constexpr unsigned kNoHint = 0xffffffffu;

template <class LT>
__device__ __forceinline__ unsigned prefix_of_rank(const LT& L, int rho, unsigned a, unsigned b, int n,
                                                   unsigned hint, int* le_out, int* less_out, int* passes) {
  int c_b = n;    // count(<= b): every element is <= kmax
  int c_am1 = 0;  // count(<= a - 1): none is below kmin
  // one count per iteration, probe chosen by the mode (a single count_le site keeps the
  // unrolled SWAR body once): 0 hint, 1 gallop down, 2 gallop up, 3 bisect
  int mode = (hint != kNoHint) ? 0 : 3;
  unsigned step = 1;
  // The same search with its control kept in integer arithmetic on wave-uniform values (the
  // compare result as a 0/1 int from the sign of rho - c, the mode transitions and step doublings
  // as 2-bit / 1-bit table lookups): no per-pass branches and no bool round trip through a VGPR.
  // mode' = T[2 mode + g] (2 bits each): (0,0)->2 (0,1)->1 (1,0)->3 (1,1)->1 (2,0)->2 (2,1)->3 (3,*)->3
  constexpr unsigned kNext = (2u << 0) | (1u << 2) | (3u << 4) | (1u << 6) | (2u << 8) | (3u << 10) | (3u << 12) |
                             (3u << 14);
  constexpr unsigned kDouble = (1u << 3) | (1u << 4);  // gallop continues: (1, greater), (2, not greater)
  while (a < b) {
    const unsigned w = b - a, mid = (a + b) >> 1;
    const unsigned th = hint < a ? a : (hint > b ? b : hint);
    const unsigned tdown = w > step ? b - step : a;
    const unsigned tup = w > step ? a + step - 1 : mid;
    const unsigned t = mode == 0 ? th : (mode == 1 ? tdown : (mode == 2 ? tup : mid));
    const int c = L.count_le(t);
    ++*passes;
    const unsigned g = (unsigned)(rho - c) >> 31;  // 1 iff c > rho
    b = g ? t : b;
    c_b = g ? c : c_b;
    a = g ? a : t + 1;
    c_am1 = g ? c_am1 : c;
    const unsigned idx = 2u * (unsigned)mode + g;
    step <<= (kDouble >> idx) & 1u;
    mode = (int)((kNext >> (2u * idx)) & 3u);
  }
  *le_out = c_b;
  *less_out = c_am1;
  return a;
}

// Search state carried from one line to the next of a wave's run: the previous line's answer
// prefix and the local density (elements per prefix unit) seen around it.
struct Hint {
  unsigned P;  // kNoHint: none
  float dens;
};

// First guess for a line without a neighbour's answer: the order statistic of the same
// quantile in a systematic sample of the line, one element per lane (line elements 32 l), off
// by about ten prefix units; it replaces the [min, max] bisection (about nine counts) by a
// window search from the guess. Found by ONE pass of the samples into the wave's 128-bin LDS
// histogram (bins 2^s prefix units wide over the samples' [min, max], s the least shift that
// fits the range in 128 bins) and one wave scan: the middle of the bin holding the k-th smallest
// sample (within 2^(s-1) units of it). A bisection over the samples with one ballot per step
// (~10 dependent ballot rounds) measured 0.7 % slower end to end.
template <class LT>
__device__ __forceinline__ unsigned sample_hint(const LT& L, int n, float kappa, unsigned* hist) {
  const int lane = threadIdx.x & 63;
  const unsigned v = L.sample();  // kNone on lanes whose sample is past the line
  const bool ok = v != kNone;
  const int ns = __popcll(__ballot(ok));
  // (a guess only: the hardware reciprocal instead of an IEEE division sequence)
  // clamped into [0, ns - 1] so that some lane's bin holds rank k (a kappa >= 1 through the C ABI,
  // or the approximate reciprocal, could otherwise leave the ballot empty)
  const int k = min(max((int)((float)(n - 1) * kappa * (float)ns * __builtin_amdgcn_rcpf((float)n)), 0), ns - 1);
  const unsigned lo = wave_min_u32(v), hi = wave_max_u32(ok ? v : 0u);
  if (lo >= hi) return lo > 0x7f80u ? 0x7f80u : lo;
  const unsigned range = hi - lo;
  const int sh = range < 128u ? 0 : 25 - __builtin_clz(range);  // (range >> sh) <= 127
  reinterpret_cast<uint2*>(hist)[lane] = make_uint2(0u, 0u);
  __builtin_amdgcn_wave_barrier();
  if (ok) __hip_atomic_fetch_add(hist + ((v - lo) >> sh), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  __builtin_amdgcn_wave_barrier();
  const uint2 hv = reinterpret_cast<const uint2*>(hist)[lane];
  const int sl = (int)(hv.x + hv.y);
  const int S = wave_incl_scan(sl);
  const int E = S - sl;
  const int src = __builtin_ctzll(__ballot(E <= k && k < S));
  const int Es = __builtin_amdgcn_readlane(E, src);
  const int h0 = __builtin_amdgcn_readlane((int)hv.x, src);
  const unsigned bin = 2u * (unsigned)src + (k >= Es + h0 ? 1u : 0u);
  __builtin_amdgcn_wave_barrier();
  const unsigned P = lo + (bin << sh) + ((1u << sh) >> 1);
  return P > 0x7f80u ? 0x7f80u : P;
}

// The least prefix above P that has elements, and their count, from the bins hist_rank left in
// LDS (window [base, base + 128)); false when no bin above P inside the window has any.
__device__ __forceinline__ bool hist_next(const unsigned* hist, unsigned base, unsigned P, unsigned* Pn, int* cnt) {
  const int lane = threadIdx.x & 63;
  const uint2 hv = reinterpret_cast<const uint2*>(hist)[lane];
  const unsigned b0 = base + 2u * (unsigned)lane;
  const bool n0 = hv.x != 0u && b0 > P, n1 = hv.y != 0u && b0 + 1u > P;
  const unsigned long long m = __ballot(n0 || n1);
  if (!m) return false;
  const int src = __builtin_ctzll(m);
  const unsigned x = (unsigned)__builtin_amdgcn_readlane((int)hv.x, src);
  const unsigned y = (unsigned)__builtin_amdgcn_readlane((int)hv.y, src);
  const unsigned c0 = base + 2u * (unsigned)src;
  const bool first = x != 0u && c0 > P;
  *Pn = first ? c0 : c0 + 1u;
  *cnt = (int)(first ? x : y);
  return true;
}

// Scratch of one wave in LDS: element list and 64 bit-words.
struct alignas(16) WaveLds {
  int list[64];
  uint32_t words[128];  // le words (64 per line half)
  uint32_t hist[128];   // the lines' prefix histogram (hist_rank)
  uint32_t sink[64];    // per-lane targets of the elements outside the histogram (hist_add)
  float gv[64 * kMS];  // Gram terms of a group's cells, [member][frame]
};

// Exact keys of a prefix group (the line elements whose 16-bit prefix is P), computed in ONE
// batched round: lane k < g recomputes element list[k]. Valid when g <= 64.
struct Group {
  unsigned P;
  int g;
  int elem;      // this lane's element (lanes off .. off + g - 1)
  unsigned key;  // its exact key (0xffffffff on lanes without a member)
  int off;       // first lane of the group's members (0, or g1 for the second group of group_keys2)
  __device__ __forceinline__ bool mine(int lane) const { return (unsigned)(lane - off) < (unsigned)g; }
};

template <class LT, class KF>
__device__ __forceinline__ Group group_keys(const LT& L, unsigned P, int g, const KF& keyf, WaveLds& W) {
  const int lane = threadIdx.x & 63;
  const int ebase = L.ebase();
  // member list: per-lane SWAR member mask, one wave scan for the lane's first slot, then each
  // lane writes its own members (usually 0-2 per lane; no per-element ballot)
  auto m = L.eq_mask(P);
  const int cnt = popc(m);
  int idx = wave_incl_scan(cnt) - cnt;
  while (m) {
    W.list[idx++] = L.elem(ebase, ctz(m));
    m &= m - 1;
  }
  __builtin_amdgcn_wave_barrier();
  // this lane's member (lanes >= g take member 0: a valid cell) and its two stacked norms,
  // requested before the Gram rounds so that their latency overlaps them
  const int e_me = W.list[lane < g ? lane : 0];
  const float nq_me = keyf.V.NXq[keyf.qi(e_me)], nr_me = keyf.V.NXr[keyf.rj(e_me)];
  // the 9 g Gram terms, one per lane and round (about 2 rounds for a typical group of 8-9)
  for (int t = lane; t < kMS * g; t += 64) {
    const int k = t / kMS, u = t - k * kMS;
    const int e = W.list[k];
    W.gv[t] = cell_gram(keyf.V, (keyf.qi(e) + u) * keyf.V.tau, (keyf.rj(e) + u) * keyf.V.tau);
  }
  __builtin_amdgcn_wave_barrier();
  Group G;
  G.P = P;
  G.g = g;
  G.off = 0;
  G.elem = lane < g ? e_me : 0;
  G.key = 0xffffffffu;
  if (lane < g) {
    float dot = W.gv[lane * kMS];
#pragma unroll
    for (int u = 1; u < kMS; ++u) dot = dot + W.gv[lane * kMS + u];
    const float d2 = (nq_me - 2.0f * dot) + nr_me;  // cell_finish with the preloaded norms
    G.key = __builtin_bit_cast(unsigned, d2 > 0.0f ? d2 : 0.0f);
  }
  __builtin_amdgcn_wave_barrier();
  return G;
}

// The exact keys of TWO prefix groups in one batched pass (the lower order statistic's group P1
// and, when the upper one is the least key of the next non-empty prefix P2, that group): one
// packed scan for both member lists, then the same rounds over 9 (g1 + g2) Gram terms. Members
// of P1 on lanes [0, g1), of P2 on lanes [g1, g1 + g2); g1 + g2 <= 64. One recompute round trip
// instead of two for the ~28 % of lines whose two order statistics straddle a prefix boundary.
template <class LT, class KF>
__device__ __forceinline__ void group_keys2(const LT& L, unsigned P1, int g1, unsigned P2, int g2, const KF& keyf,
                                            WaveLds& W, Group* G1, Group* G2) {
  const int lane = threadIdx.x & 63;
  const int ebase = L.ebase();
  auto m1 = L.eq_mask(P1);
  auto m2 = L.eq_mask(P2);
  const int c1 = popc(m1), c2 = popc(m2);
  const int packed = c1 | (c2 << 16);  // per-lane counts <= 64: one scan for both lists
  const int sc = wave_incl_scan(packed) - packed;
  int i1 = sc & 0xffff, i2 = g1 + (sc >> 16);
  while (m1) {
    W.list[i1++] = L.elem(ebase, ctz(m1));
    m1 &= m1 - 1;
  }
  while (m2) {
    W.list[i2++] = L.elem(ebase, ctz(m2));
    m2 &= m2 - 1;
  }
  __builtin_amdgcn_wave_barrier();
  const int g = g1 + g2;
  const int e_me = W.list[lane < g ? lane : 0];
  const float nq_me = keyf.V.NXq[keyf.qi(e_me)], nr_me = keyf.V.NXr[keyf.rj(e_me)];
  for (int t = lane; t < kMS * g; t += 64) {
    const int k = t / kMS, u = t - k * kMS;
    const int e = W.list[k];
    W.gv[t] = cell_gram(keyf.V, (keyf.qi(e) + u) * keyf.V.tau, (keyf.rj(e) + u) * keyf.V.tau);
  }
  __builtin_amdgcn_wave_barrier();
  unsigned key = 0xffffffffu;
  if (lane < g) {
    float dot = W.gv[lane * kMS];
#pragma unroll
    for (int u = 1; u < kMS; ++u) dot = dot + W.gv[lane * kMS + u];
    const float d2 = (nq_me - 2.0f * dot) + nr_me;
    key = __builtin_bit_cast(unsigned, d2 > 0.0f ? d2 : 0.0f);
  }
  __builtin_amdgcn_wave_barrier();
  const int elem = lane < g ? e_me : 0;
  *G1 = Group{P1, g1, elem, lane < g1 ? key : 0xffffffffu, 0};
  *G2 = Group{P2, g2, elem, (lane >= g1 && lane < g) ? key : 0xffffffffu, g1};
}

// Least key of a batched group (its rank 0), one wave minimum.
__device__ __forceinline__ unsigned group_min(const Group& G) {
  return wave_min_u32(G.mine(threadIdx.x & 63) ? G.key : 0xffffffffu);
}

// Key of rank rho (0-based) inside a batched group whose members start at lane 0 (off == 0).
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

// Keys of ranks rho and rho + 1 inside a batched group (rho + 1 < g), one counting loop.
__device__ __forceinline__ void group_rank2(const Group& G, int rho, unsigned* v0, unsigned* v1) {
  const int lane = threadIdx.x & 63;
  int cl = 0, ce = 0;
  for (int k = 0; k < G.g; ++k) {
    const unsigned o = (unsigned)lane_bcast((int)G.key, k);
    cl += o < G.key;
    ce += o == G.key;
  }
  const bool act = lane < G.g;
  const int s0 = __builtin_ctzll(__ballot(act && cl <= rho && rho < cl + ce));
  const int s1 = __builtin_ctzll(__ballot(act && cl <= rho + 1 && rho + 1 < cl + ce));
  *v0 = (unsigned)lane_bcast((int)G.key, s0);
  *v1 = (unsigned)lane_bcast((int)G.key, s1);
}

// Members of prefix group P in rounds of 64: round r lists members [64r, 64r + 64) (line order)
// in W.list and runs fn(element) on lane k < (members in the round). Per-lane member masks and
// one wave scan give each lane its members' positions; no per-element register arrays.
template <class LT, class F>
__device__ __forceinline__ void group_rounds(const LT& L, unsigned P, int g, WaveLds& W, F fn) {
  const int lane = threadIdx.x & 63;
  auto m = L.eq_mask(P);
  const int cnt = popc(m);
  int idx = wave_incl_scan(cnt) - cnt;
  const int ebase = L.ebase();
  for (int r0 = 0; r0 < g; r0 += 64) {
    while (m && idx < r0 + 64) {
      const int q = ctz(m);
      m &= m - 1;
      W.list[idx - r0] = L.elem(ebase, q);
      ++idx;
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < min(64, g - r0)) fn(W.list[lane]);
    __builtin_amdgcn_wave_barrier();
  }
}

// Bin of rank rho in a 256-bin LDS histogram (lane l owns bins 4l..4l+3); rho becomes the rank
// inside that bin.
__device__ __forceinline__ unsigned hist_bin_of_rank(const unsigned* hist, int* rho) {
  const int lane = threadIdx.x & 63;
  const unsigned c0 = hist[4 * lane], c1 = hist[4 * lane + 1], c2 = hist[4 * lane + 2], c3 = hist[4 * lane + 3];
  const int tot = (int)(c0 + c1 + c2 + c3);
  const int ex = wave_incl_scan(tot) - tot;
  const int r = *rho;
  int bin = -1, below = ex;
  if (r >= ex && r < ex + tot) {
    if (r < below + (int)c0) {
      bin = 0;
    } else if (r < below + (int)(c0 + c1)) {
      bin = 1;
      below += c0;
    } else if (r < below + (int)(c0 + c1 + c2)) {
      bin = 2;
      below += c0 + c1;
    } else {
      bin = 3;
      below += c0 + c1 + c2;
    }
  }
  const int src = __builtin_ctzll(__ballot(bin >= 0));
  *rho = r - lane_bcast(below, src);
  return (unsigned)(4 * src + lane_bcast(bin, src));
}

// Key of rank rho in a large prefix group (g > 64; long silences): two passes of recomputed
// member keys into 8-bit LDS histograms of the low half (bits 15..8, then 7..0).
template <class LT, class KF>
__device__ __forceinline__ unsigned big_group_rank(const LT& L, unsigned P, int rho, int g, const KF& keyf, WaveLds& W) {
  const int lane = threadIdx.x & 63;
  unsigned* hist = reinterpret_cast<unsigned*>(W.gv);  // 256 bins
  unsigned hi8 = 0, lo8 = 0;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    for (int b = lane; b < 256; b += 64) hist[b] = 0u;
    __builtin_amdgcn_wave_barrier();
    group_rounds(L, P, g, W, [&](int e) {
      const unsigned k = keyf(e);
      if (pass == 0)
        atomicAdd(&hist[(k >> 8) & 0xffu], 1u);
      else if (((k >> 8) & 0xffu) == hi8)
        atomicAdd(&hist[k & 0xffu], 1u);
    });
    __builtin_amdgcn_wave_barrier();
    const unsigned bin = hist_bin_of_rank(hist, &rho);
    __builtin_amdgcn_wave_barrier();
    if (pass == 0)
      hi8 = bin;
    else
      lo8 = bin;
  }
  return (P << 16) | (hi8 << 8) | lo8;
}

template <class LT, class KF>
__device__ __forceinline__ unsigned rank_in_prefix(const LT& L, unsigned P, int rho, int g, const KF& keyf, WaveLds& W,
                                   Group* cache) {
  if (g <= 64) {
    if (cache->g < 0 || cache->P != P) *cache = group_keys(L, P, g, keyf, W);
    return group_rank(*cache, rho);
  }
  return big_group_rank(L, P, rho, g, keyf, W);
}

// The search half of a line's threshold: the rank targets lo / hi of the percentile, the prefix
// Pl of rank lo with count(<= Pl) = le and count(< Pl) = less, and, when the two order statistics
// straddle a prefix boundary and the histogram holds it, the next group (Ph2, gh2).
struct Plan {
  unsigned Pl, hbase, Ph2;
  int le, less, gh2, lo, hi;
  float q, lo_f, hi_f;
  bool found, next_ok, both;  // next_ok: (Ph2, gh2) = the next group, read from the histogram
};

template <class LT, class KF>
__device__ __forceinline__ Plan line_plan(const LT& L, int n, float kappa, WaveLds& W, Hint* hint) {
  Plan pl;
  pl.q = (float)(n - 1) * kappa;
  pl.lo_f = floorf(pl.q);
  pl.hi_f = ceilf(pl.q);
  pl.lo = (int)pl.lo_f;
  pl.hi = (int)pl.hi_f;
  const int lo = pl.lo, hi = pl.hi;
  unsigned kmin = 0, kmax = 0x7f80u;  // every real prefix (finite non-negative float) is <= 0x7f80
  const bool hinted = hint->P != kNoHint;
  if (!hinted) L.min_max(&kmin, &kmax);
  int le = 0, less = 0;
  int passes = 0;
  unsigned Pl = 0u, hbase = 0u;
  bool found = false;
  if constexpr (LT::kHist) {
    if (hinted) found = L.hist_rank(hint->P, lo, W.hist, &Pl, &le, &less, &hbase);
  }
  if (!found) Pl = prefix_of_rank(L, lo, kmin, kmax, n, hint->P, &le, &less, &passes);
  hint->P = Pl;
  // density around the answer: the group at Pl, smoothed over the run
  hint->dens = hinted ? 0.5f * hint->dens + 0.5f * (float)(le - less) : (float)(le - less);
  pl.Pl = Pl;
  pl.hbase = hbase;
  pl.le = le;
  pl.less = less;
  pl.found = found;
  pl.Ph2 = 0u;
  pl.gh2 = 0;
  // the upper statistic is the least key above Pl: its group from the histogram's bins, read now
  // (the bins belong to this line only until the next line's search)
  pl.next_ok = hi != lo && hi >= le && found && hist_next(W.hist, hbase, Pl, &pl.Ph2, &pl.gh2);
  pl.both = pl.next_ok && le - less <= 64 && (le - less) + pl.gh2 <= 64;
  return pl;
}

// The exact values vlo / vhi of the two order statistics from a plan: the groups' keys recomputed
// (cached in *c_lo / *c_hi for le_bits).
template <class LT, class KF>
__device__ __forceinline__ void line_groups(const LT& L, const Plan& pl, const KF& keyf, WaveLds& W, Group* c_lo,
                                            Group* c_hi, unsigned* vlo_o, unsigned* vhi_o) {
  const unsigned Pl = pl.Pl;
  const int le = pl.le, less = pl.less, lo = pl.lo, hi = pl.hi;
  unsigned vlo, vhi;
  if (pl.both) {
    group_keys2(L, Pl, le - less, pl.Ph2, pl.gh2, keyf, W, c_lo, c_hi);
    vlo = group_rank(*c_lo, lo - less);
    vhi = group_min(*c_hi);
  } else if (hi != lo && hi < le && le - less <= 64) {
    *c_lo = group_keys(L, Pl, le - less, keyf, W);
    group_rank2(*c_lo, lo - less, &vlo, &vhi);
  } else {
    vlo = rank_in_prefix(L, Pl, lo - less, le - less, keyf, W, c_lo);
    vhi = vlo;
  }
  if (!pl.both && hi != lo && !(hi < le && le - less <= 64)) {
    if (hi < le) {
      vhi = rank_in_prefix(L, Pl, hi - less, le - less, keyf, W, c_lo);
    } else {
      unsigned Ph;
      int gh;
      // the next group from the histogram's bins when the search used one, else two counts
      if (pl.next_ok) {
        Ph = pl.Ph2;
        gh = pl.gh2;
      } else {
        Ph = L.min_greater(Pl);
        gh = L.count_le(Ph) - le;
      }
      vhi = rank_in_prefix(L, Ph, 0, gh, keyf, W, c_hi);
    }
  }
  *vlo_o = vlo;
  *vhi_o = vhi;
}

// Percentile threshold (linear interpolation in the sqrt domain) and its squared-domain form.
__device__ __forceinline__ void plan_threshold(const Plan& pl, unsigned vlo, unsigned vhi, float* thr, float* T) {
  const float slo = sqrt_rn(__builtin_bit_cast(float, vlo));
  float th;
  if (pl.lo_f == pl.hi_f) {
    th = slo;
  } else {
    const float shi = sqrt_rn(__builtin_bit_cast(float, vhi));
    const float aa = slo * (pl.hi_f - pl.q);
    const float bb = shi * (pl.q - pl.lo_f);
    th = aa + bb;
  }
  *thr = th;
  *T = sq_threshold(th);
}

// Threshold (distance units) and squared-domain threshold of a line of n keys; leaves the
// exact keys of the last batched group in *cache for le_bits.
template <class LT, class KF>
__device__ __forceinline__ void line_threshold(const LT& L, int n, float kappa, const KF& keyf, WaveLds& W, Group* c_lo,
                               Group* c_hi, float* thr, float* T, Hint* hint) {
  const Plan pl = line_plan<LT, KF>(L, n, kappa, W, hint);
  unsigned vlo, vhi;
  line_groups(L, pl, keyf, W, c_lo, c_hi, &vlo, &vhi);
  plan_threshold(pl, vlo, vhi, thr, T);
}

// Bits of "key <= T" for this lane's elements (in the line type's bit order): every
// element whose prefix is <= T's prefix, minus the members of T's prefix group whose exact key
// exceeds T. The group's exact keys come from the threshold search (the group at the answer's
// prefix, cached), so normally no member mask or recompute is needed here.
template <class LT, class KF>
__device__ __forceinline__ auto le_bits(const LT& L, unsigned Tbits, const KF& keyf, WaveLds& W, const Group& c_lo,
                            const Group& c_hi) {
  const unsigned T16 = Tbits >> 16;
  const int lane = threadIdx.x & 63;
  const auto word = L.le_mask(T16);  // kNone is never <= T16 <= 0x7f80
  // (selected by value: a pointer to either cached group would put both on the stack)
  const bool lo_hit = c_lo.g >= 0 && c_lo.P == T16, hi_hit = c_hi.g >= 0 && c_hi.P == T16;
  W.words[lane] = 0xffffffffu;
  if (LT::kHalves == 2) W.words[64 + lane] = 0xffffffffu;
  __builtin_amdgcn_wave_barrier();
  if (lo_hit || hi_hit) {
    const bool cmine = lo_hit ? c_lo.mine(lane) : c_hi.mine(lane);
    const unsigned ckey = lo_hit ? c_lo.key : c_hi.key;
    const int celem = lo_hit ? c_lo.elem : c_hi.elem;
    if (cmine && ckey > Tbits) atomicAnd(&W.words[LT::lane_of(celem)], ~(1u << LT::bit_of(celem)));
  } else {
    const int g = wave_sum(popc(L.eq_mask(T16)));
    if (g == 0) return word;
    if (g <= 64) {
      const Group G = group_keys(L, T16, g, keyf, W);
      if (lane < G.g && G.key > Tbits) atomicAnd(&W.words[LT::lane_of(G.elem)], ~(1u << LT::bit_of(G.elem)));
    } else {  // large group: member keys in rounds of 64
      group_rounds(L, T16, g, W, [&](int e) {
        if (keyf(e) > Tbits) atomicAnd(&W.words[LT::lane_of(e)], ~(1u << LT::bit_of(e)));
      });
    }
  }
  __builtin_amdgcn_wave_barrier();
  if constexpr (LT::kHalves == 2)
    return word & (((uint64_t)W.words[64 + lane] << 32) | W.words[lane]);
  else
    return word & W.words[lane];
}

// ---------------------------------------------------------------------------------------
// k_sel_rows9: one 512-thread block per (32-row strip, pair); wave w takes rows w, w+8, ...
// Emits T_row and the strip's row-threshold words RT[strip][j] (bit r: key(i0+r, j) <= T_row).
// ---------------------------------------------------------------------------------------
// LDS of the fused row select: one WaveLds per wave and the strip's row bits
constexpr int kRowsLds = 4 * (int)sizeof(WaveLds) + kSR * 64 * 4;
// launches with lines past 2048 codes: row bits of 128 words per row
constexpr int kRowsLds2 = 4 * (int)sizeof(WaveLds) + kSR * 128 * 4;

// In-register transpose of a 32 x 32 bit matrix: a[r] bit q -> a[q] bit r (stage J swaps the
// off-diagonal J x J sub-blocks).
template <int J>
__device__ __forceinline__ void transpose_stage(uint32_t (&a)[32]) {
  constexpr uint32_t m = J == 16 ? 0x0000ffffu : J == 8 ? 0x00ff00ffu : J == 4 ? 0x0f0f0f0fu : J == 2 ? 0x33333333u
                                                                                                      : 0x55555555u;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k & J) continue;
    const uint32_t t = ((a[k] >> J) ^ a[k + J]) & m;
    a[k + J] ^= t;
    a[k] ^= t << J;
  }
}

__device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
  transpose_stage<16>(a);
  transpose_stage<8>(a);
  transpose_stage<4>(a);
  transpose_stage<2>(a);
  transpose_stage<1>(a);
}

// Row select of one (32-row strip, pair) by NW waves: wave w takes rows w, w+NW, ...
// Line type of a select: KQ = 0 -> the long-line layout (Line<32>), else LineS<KQ>.
template <int KQ>
struct LineOf {
  using T = LineS<KQ>;
};
template <>
struct LineOf<0> {
  using T = Line<32>;
};
template <>
struct LineOf<2> {
  using T = Line2;
};

template <int NW, int KQ, int RB>
__device__ __forceinline__ void rows_body(const PairView& V, int p, int strip, const uint16_t* Hr, int ldr,
                                          float kappa, float* __restrict__ thr,
                                          float* __restrict__ Tq, int64_t thr_stride, uint32_t* __restrict__ RT,
                                          int64_t rt_stride, int ld, WaveLds* wl, uint32_t (*rowbits)[RB]) {
  using LT = typename LineOf<KQ>::T;
  const int i0 = strip * kSR;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // w: wave-uniform (SGPR)
  WaveLds& W = wl[w];
  constexpr int RPW = kSR / NW;  // consecutive rows per wave: each search starts from its neighbour's
  Hint hint{kNoHint, 1.0f};
  // the next row's line is loaded while this one is searched (its latency hidden)
  auto load_row = [&](LT& Ld, int i) {
    int64_t rowoff = (int64_t)(i - i0) * ldr;
    asm volatile("" : "+s"(rowoff));  // per-row address: nothing per lane hoisted out of the loop
    if constexpr (KQ == 0) {
      Ld.template load_lanes<false>(Hr + rowoff, 32, V.Np);
    } else if constexpr (KQ == 2) {
      Ld.A.template load_lanes<false>(Hr + rowoff, 32, V.Np);
      Ld.B.template load_lanes<false>(Hr + rowoff + 2048, 32, V.Np - 2048);
    } else {
      const uint16_t* row = Hr + rowoff;
      Ld.load([&](int e) { return row + (unsigned)e; }, V.Np);
    }
  };
  // Line2 loads each line when it starts (no prefetch: 48 VGPRs, the 4th wave per SIMD)
  constexpr bool kPF = KQ != 2;
  // one row's select on its loaded line L; prefetch() requests the wave's next line once this
  // one's window is built
  auto row = [&](LT& L, int r, auto&& prefetch) {
    const int i = i0 + r;
    uint64_t word = 0;  // (Line2: the second half's word in bits 32..63)
    if (i < V.Mp) {
      if (hint.P == kNoHint) hint.P = sample_hint(L, V.Np, kappa, W.hist);
      if constexpr (KQ != 8) {
        if (hint.P != kNoHint) L.build_window(hint.P);
      }
      prefetch();
      const LineCells<true> keyf{V, i};
      float th, T;
      Group c_lo, c_hi;
      c_lo.g = c_hi.g = -1;
      line_threshold(L, V.Np, kappa, keyf, W, &c_lo, &c_hi, &th, &T, &hint);
      if (lane == 0) {
        thr[(size_t)p * thr_stride + i] = th;
        Tq[(size_t)p * thr_stride + i] = T;
      }
      word = le_bits(L, __builtin_bit_cast(unsigned, T), keyf, W, c_lo, c_hi);
      if constexpr (KQ == 8 || KQ == 16) word = lane_words<KQ>((uint32_t)word);  // lane t: columns 32t .. 32t + 31
    }
    rowbits[r][lane] = (uint32_t)word;
    if constexpr (KQ == 2) rowbits[r][64 + lane] = (uint32_t)(word >> 32);
  };
  // (unrolled by two for long lines, each line in its own registers instead of the copy of the
  // prefetched line: neutral, profiles/r04/ab_unroll2000.txt)
  const int r1 = (w + 1) * RPW;
  {
    LT Lnext;
    if (kPF && i0 + w * RPW < V.Mp) load_row(Lnext, i0 + w * RPW);
#pragma unroll 1
    for (int r = w * RPW; r < r1; ++r) {
      LT L;
      if (i0 + r < V.Mp) {
        if constexpr (kPF)
          L = Lnext;
        else
          load_row(L, i0 + r);
      }
      row(L, r, [&] {
        if (kPF && r + 1 < r1 && i0 + r + 1 < V.Mp) load_row(Lnext, i0 + r + 1);
      });
    }
  }
  __syncthreads();
  // transpose: word of column j = bit (j & 31) of rowbits[r][j >> 5], r = 0..31. Thread b takes
  // the 32 x 32 bit block of columns 32b..32b+31 and transposes it in registers (five
  // masked-swap stages, about half an op per bit).
  uint32_t* out = RT + (size_t)p * rt_stride + (size_t)strip * ld;
  for (int b = threadIdx.x; 32 * b < V.Np; b += NW * 64) {
    uint32_t a[32];
#pragma unroll
    for (int r = 0; r < 32; ++r) a[r] = rowbits[r][b];
    transpose32(a);
    uint32_t* o = out + 32 * b;
    if (32 * b + 32 <= ld) {  // whole block inside the row pitch (ld is a multiple of 32 when Np > 32b)
#pragma unroll
      for (int q = 0; q < 32; q += 4) *reinterpret_cast<uint4*>(o + q) = make_uint4(a[q], a[q + 1], a[q + 2], a[q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 32; ++q)
        if (32 * b + q < V.Np) o[q] = a[q];
    }
  }
}


// Sweep and row select fused: the block selects the 32 rows it has just swept, reading its
// full keys back while they are cache-resident (no second pass over F from HBM, one launch
// fewer). LDS of the two phases is one union.
// KQ = 8: every line of the launch is short; KQ = 0: each pair picks its row line type (rows of
// at most short_n codes take LineS<8>; short_n = 0 disables); KQ = 16: as 0 with LineS<16> for
// the rest (every line <= 1024 codes); KQ = 2: as 0, and rows past 2048 codes take Line2.
constexpr int kSweepWPE = 4;  // sweep blocks per CU (waves per SIMD)
// Arguments of one sweep + row-select launch (k_sweep_rows9) and of one column-select launch
// (k_sel_cols9).
struct SweepArgs {
  CrpBatch B;
  KeyPlanes K;
  int ldr, ldc;
  int64_t kstride;
  float kappa;
  float* thr;
  float* Tq;
  int64_t thr_stride;
  uint32_t* RT;
  int64_t rt_stride;
  int ld, short_n;
};
struct ColsArgs {
  CrpBatch B;
  KeyPlanes K;
  int ldc;
  int64_t kstride;
  float kappa;
  const uint32_t* RT;
  float* thr;
  float* Tq;
  int64_t thr_stride;
  uint32_t* maskT;
  int64_t mask_stride;
  int ld, short_n;
};
template <int KQ>
constexpr int kSweepLds = KQ == 2 ? kRowsLds2 : kRowsLds;

// One (32-row strip, pair) block of the sweep and its fused row select; smem: kSweepLds<KQ> bytes.
template <int KQ>
__device__ __forceinline__ void sweep_rows_block(const SweepArgs& A, int strip, int p, char* smem) {
  constexpr int RB = KQ == 2 ? 128 : 64;  // row-bit words per row
  const CrpBatch& B = A.B;
  const KeyPlanes& K = A.K;
  const int ldr = A.ldr, ldc = A.ldc, ld = A.ld, short_n = A.short_n;
  const int64_t kstride = A.kstride, thr_stride = A.thr_stride, rt_stride = A.rt_stride;
  const float kappa = A.kappa;
  float* thr = A.thr;
  float* Tq = A.Tq;
  uint32_t* RT = A.RT;
  const PairView V = pair_view(B, p);
  const int i0 = strip * kSR;
  if (i0 >= V.Mp || V.Np <= 0) return;
  uint16_t* Hr = K.hr + (size_t)p * kstride + (size_t)i0 * ldr;
  if (i0 + kSR <= V.Mp)
    sweep_body_sys<false>(V, p, strip, K, ldr, ldc, kstride, Hr);
  else
    sweep_body_sys<true>(V, p, strip, K, ldr, ldc, kstride, Hr);
  __syncthreads();  // the strip's F rows are complete (block-scope visibility of the global stores)
  WaveLds* wl = reinterpret_cast<WaveLds*>(smem);
  uint32_t(*rowbits)[RB] = reinterpret_cast<uint32_t(*)[RB]>(smem + 4 * sizeof(WaveLds));
  // lines of <= short_n codes take LineS<8> in every launch type but KQ = 8 (all short); KQ = 16
  // launches (every line <= 1024 codes) take LineS<16> for the rest (a third select type in a
  // KQ = 0 launch costs more than it saves)
  if (KQ == 8 || V.Np <= short_n)
    rows_body<4, 8, RB>(V, p, strip, Hr, ldr, kappa, thr, Tq, thr_stride, RT, rt_stride, ld, wl, rowbits);
  else if (KQ == 16)
    rows_body<4, 16, RB>(V, p, strip, Hr, ldr, kappa, thr, Tq, thr_stride, RT, rt_stride, ld, wl, rowbits);
  else if (KQ == 2 && V.Np > 2048)
    rows_body<4, 2, RB>(V, p, strip, Hr, ldr, kappa, thr, Tq, thr_stride, RT, rt_stride, ld, wl, rowbits);
  else
    rows_body<4, 0, RB>(V, p, strip, Hr, ldr, kappa, thr, Tq, thr_stride, RT, rt_stride, ld, wl, rowbits);
}

template <int KQ>
__global__ __launch_bounds__(kThreads, kSweepWPE) void k_sweep_rows9(SweepArgs A) {
  __shared__ __attribute__((aligned(16))) char smem[kSweepLds<KQ>];
  sweep_rows_block<KQ>(A, blockIdx.x, blockIdx.y, smem);
}

// ---------------------------------------------------------------------------------------
// k_sel_cols9: one wave per run of kCPW consecutive CRP columns; emits T_col and the columns'
// CRP words. Lane l <-> rows 32l..32l+31 (KPL == 32). Neighbouring columns share 8 of their 9
// stacked frames, so each column's search starts from the previous column's answer (the first
// column of a run bisects from its min/max).
// ---------------------------------------------------------------------------------------
constexpr int kCPWLong = 2;  // columns per wave, long lines (1: -1.5 %, 4: -3.5 %, round 5)
// short lines: a run start (sample guess, longer search) is a larger share of a cheap line
constexpr int kCPWShort = 4;
template <int KQ>
constexpr int kCPW = (KQ == 8 || KQ == 16) ? kCPWShort : kCPWLong;
constexpr int kColsWPE = 4;  // column-select waves per SIMD
template <int KQ>
constexpr int kColsPerBlock = 4 * kCPW<KQ>;

// Columns [j0, jend) of pair p with line type LineOf<KQ>.
template <int KQ>
__device__ __forceinline__ void cols_body(const PairView& V, int p, int j0, int jend, const KeyPlanes& K, int ldc,
                                          int64_t kstride, float kappa, const uint32_t* __restrict__ RT,
                                          float* __restrict__ thr, float* __restrict__ Tq, int64_t thr_stride,
                                          uint32_t* __restrict__ maskT, int64_t mask_stride, int ld, WaveLds& W) {
  constexpr int KPL = 32;  // rows per CRP word (= per lane for long lines)
  using LT = typename LineOf<KQ>::T;
  const int lane = threadIdx.x & 63;
  Hint hint{kNoHint, 1.0f};
  // the next column's line is loaded while this one is searched (its HBM latency hidden)
  auto load_col = [&](LT& Ld, int j) {
    int64_t coloff = (int64_t)p * kstride + (int64_t)j * kSR;
    asm volatile("" : "+s"(coloff));  // per-column address: nothing per lane hoisted out of the loop
    if constexpr (KQ == 0) {
      Ld.template load_lanes<true>(K.hc + coloff, (size_t)ldc * kSR, V.Mp);
    } else if constexpr (KQ == 2) {  // rows 2048.. start at strip 64
      Ld.A.template load_lanes<true>(K.hc + coloff, (size_t)ldc * kSR, V.Mp);
      Ld.B.template load_lanes<true>(K.hc + coloff + (size_t)64 * ldc * kSR, (size_t)ldc * kSR, V.Mp - 2048);
    } else {  // row e: strip e / 32, split-order slot of row e % 32 in the strip's 32-row chunk
      const uint16_t* col = K.hc + coloff;
      Ld.load([&](int e) { return col + (unsigned)((e >> 5) * ldc * kSR + (e & 15) * 2 + ((e >> 4) & 1)); }, V.Mp);
    }
  };
  // one column's select on its loaded line L
  auto column = [&](LT& L, int j) {
    if (hint.P == kNoHint) hint.P = sample_hint(L, V.Mp, kappa, W.hist);
    if constexpr (KQ != 8) {
      if (hint.P != kNoHint) L.build_window(hint.P);
    }
    // this column's row-threshold word, requested now and used after the select
    const size_t w = (size_t)p * mask_stride + (size_t)(lane * KPL < V.Mp ? lane : 0) * ld + j;
    const uint32_t rt = RT[w];
    // Line2: the second half's strip 64 + lane
    const size_t w2 = (size_t)p * mask_stride + (size_t)(2048 + lane * KPL < V.Mp ? 64 + lane : 0) * ld + j;
    const uint32_t rt2 = KQ == 2 ? RT[w2] : 0u;
    const LineCells<false> keyf{V, j};
    float th, Tc;
    Group c_lo, c_hi;
    c_lo.g = c_hi.g = -1;
    line_threshold(L, V.Mp, kappa, keyf, W, &c_lo, &c_hi, &th, &Tc, &hint);
    if (lane == 0) {
      thr[(size_t)p * thr_stride + j] = th;
      Tq[(size_t)p * thr_stride + j] = Tc;
    }
    uint64_t bits = le_bits(L, __builtin_bit_cast(unsigned, Tc), keyf, W, c_lo, c_hi);
    if constexpr (KQ == 8 || KQ == 16) bits = lane_words<KQ>((uint32_t)bits);  // lane s: rows 32s .. 32s + 31
    if (lane * KPL < V.Mp) maskT[w] = (uint32_t)bits & rt;
    if (KQ == 2 && 2048 + lane * KPL < V.Mp) maskT[w2] = (uint32_t)(bits >> 32) & rt2;
  };
  constexpr bool kPF = KQ != 2;  // as the rows
  // (both columns of a long-line pair in their own registers, fully unrolled, instead of the
  // copy of the prefetched line: -4.5 % at 2,000 frames, profiles/r04/ab_unroll2000.txt)
  {
    LT Lnext;
    if (kPF && j0 < jend) load_col(Lnext, j0);
#pragma unroll 1
    for (int j = j0; j < jend; ++j) {
      LT L;
      if constexpr (kPF)
        L = Lnext;
      else
        load_col(L, j);
      if (kPF && j + 1 < jend) load_col(Lnext, j + 1);
      column(L, j);
    }
  }
}


// KQ = 8: every line of the launch is short (runs of kCPW<8> columns); KQ = 0: runs of kCPW<0>,
// each pair picking its column line type (columns of at most short_n codes take LineS<8>);
// KQ = 16: as 0 with LineS<16> for the rest; KQ = 2: as 0, and columns past 2048 codes take Line2.
// One column-select block: linear index lin of nblk = ncb * nb blocks (ncb column blocks per
// pair), lin % 8 being the XCD the block runs on.
template <int KQ>
__device__ __forceinline__ void cols_block(const ColsArgs& A, int lin, int ncb, int nblk, WaveLds* wl) {
  const CrpBatch& B = A.B;
  const KeyPlanes& K = A.K;
  const int ldc = A.ldc, ld = A.ld, short_n = A.short_n;
  const int64_t kstride = A.kstride, thr_stride = A.thr_stride, mask_stride = A.mask_stride;
  const float kappa = A.kappa;
  const uint32_t* RT = A.RT;
  float* thr = A.thr;
  float* Tq = A.Tq;
  uint32_t* maskT = A.maskT;
  // neighbouring columns share the lines of RT and the recomputed cells' frames: keep them on one XCD
  const int lb = xcd_remap(lin, nblk);
  const int p = lb / ncb;
  const PairView V = pair_view(B, p);
  const int j0 = (lb - p * ncb) * kColsPerBlock<KQ> + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * kCPW<KQ>;
  const int jend = min(j0 + kCPW<KQ>, V.Np);
  WaveLds& W = wl[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];  // an SGPR base for the LDS addresses
  if (KQ == 8 || V.Mp <= short_n)
    cols_body<8>(V, p, j0, jend, K, ldc, kstride, kappa, RT, thr, Tq, thr_stride, maskT, mask_stride, ld, W);
  else if (KQ == 16)
    cols_body<16>(V, p, j0, jend, K, ldc, kstride, kappa, RT, thr, Tq, thr_stride, maskT, mask_stride, ld, W);
  else if (KQ == 2 && V.Mp > 2048)
    cols_body<2>(V, p, j0, jend, K, ldc, kstride, kappa, RT, thr, Tq, thr_stride, maskT, mask_stride, ld, W);
  else
    cols_body<0>(V, p, j0, jend, K, ldc, kstride, kappa, RT, thr, Tq, thr_stride, maskT, mask_stride, ld, W);
}

template <int KQ>
__global__ __launch_bounds__(256, kColsWPE) void k_sel_cols9(ColsArgs A) {
  __shared__ WaveLds wl[4];
  cols_block<KQ>(A, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x, gridDim.x * gridDim.y, wl);
}

}  // namespace

// Two-kernel CRP (m = 9, tau = 1, lines up to 4096 keys). Returns 1 if not applicable.
// kplanes: nb * kstride uint16 row-major prefixes, then nb * kstride uint16 strip-major ones;
// RT: nb * mask_stride
// words (same layout as maskT).
// Line type of the selects of a launch (by the batch's longest stacked line L): 8 / 16 short lines,
// 2 some line past 2048 codes, 0 the long-line layout.
static int split_kq(int L, int* short_n) {
  static const bool no_short = getenv("ACOSS_NO_SHORT") != nullptr;
  *short_n = no_short ? 0 : 512;
  return L > 2048 ? 2 : (no_short ? 0 : (L <= 512 ? 8 : (L <= 1024 ? 16 : 0)));
}

static SweepArgs sweep_args(const CrpBatch& B, void* kplanes, int ldk, int64_t kstride, int nb,
                            float kappa, float* thr_r, float* T_r, int64_t thr_stride, uint32_t* RT,
                            int64_t mask_stride, int ld, int short_n) {
  const size_t plane = (size_t)nb * kstride;
  const KeyPlanes K{static_cast<uint16_t*>(kplanes), static_cast<uint16_t*>(kplanes) + plane};
  return SweepArgs{B, K, ldk, ldk, kstride, kappa, thr_r, T_r, thr_stride, RT, mask_stride, ld, short_n};
}

static ColsArgs cols_args(const CrpBatch& B, void* kplanes, int ldk, int64_t kstride, int nb, float kappa,
                          const uint32_t* RT, float* thr_c, float* T_c, int64_t thr_stride, uint32_t* maskT,
                          int64_t mask_stride, int ld, int short_n) {
  const size_t plane = (size_t)nb * kstride;
  const KeyPlanes K{static_cast<uint16_t*>(kplanes), static_cast<uint16_t*>(kplanes) + plane};
  return ColsArgs{B, K, ldk, kstride, kappa, RT, thr_c, T_c, thr_stride, maskT, mask_stride, ld, short_n};
}

// Two-kernel CRP (m = 9, tau = 1, lines up to 4096 keys). Returns 1 if not applicable.
// kplanes: nb * kstride uint16 row-major prefixes, then nb * kstride uint16 strip-major ones;
// RT: nb * mask_stride words (same layout as maskT).
int launch_crp_split(const CrpBatch& B, int nb, int L, float kappa, void* kplanes, int ldk,
                     int64_t kstride,
                     uint32_t* RT, float* thr_r, float* T_r, float* thr_c, float* T_c, int64_t thr_stride,
                     uint32_t* maskT, int64_t mask_stride, int ld, hipStream_t s) {
  if (B.m != kMS || B.tau != 1 || L > 4096) return 1;
  const int nstrips = (L + kSR - 1) / kSR;
  int short_n;
  const int kq = split_kq(L, &short_n);
  const SweepArgs SA = sweep_args(B, kplanes, ldk, kstride, nb, kappa, thr_r, T_r, thr_stride, RT, mask_stride,
                                  ld, short_n);
  const ColsArgs CA = cols_args(B, kplanes, ldk, kstride, nb, kappa, RT, thr_c, T_c, thr_stride, maskT, mask_stride,
                                ld, short_n);
  auto launch = [&](auto kqc) -> int {
    constexpr int KQ = decltype(kqc)::value;
    prof_begin(PH_SWEEP, s);
    hipLaunchKernelGGL(k_sweep_rows9<KQ>, dim3(nstrips, nb), dim3(kThreads), 0, s, SA);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_SWEEP, s);
    prof_begin(PH_SEL_COLS, s);
    hipLaunchKernelGGL(k_sel_cols9<KQ>, dim3((L + kColsPerBlock<KQ> - 1) / kColsPerBlock<KQ>, nb), dim3(256), 0, s, CA);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_SEL_COLS, s);
    return ACOSS_OK;
  };
  if (kq == 8) return launch(std::integral_constant<int, 8>{});
  if (kq == 16) return launch(std::integral_constant<int, 16>{});
  if (kq == 2) return launch(std::integral_constant<int, 2>{});
  return launch(std::integral_constant<int, 0>{});
}

}  // namespace acoss

