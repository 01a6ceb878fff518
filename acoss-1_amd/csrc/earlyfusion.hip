// earlyfusion.hip — EarlyFusion.similarity (acoss/algorithms/earlyfusion_traile.py:157-198) for a
// batch of pairs: one launch per stage for a whole chunk of pairs instead of ~15 launches per pair.
//
// Per pair (a, b) with beat-synchronous block features (M = n_blocks[a] rows, N = n_blocks[b]):
//   CSM_m = get_csm(mfccs_a, mfccs_b)              euclid, d = 1000   (:173)
//   CSM_s = get_csm(ssms_a, ssms_b)                euclid, d = 1225   (:175)
//   CSM_c = get_csm_blocked_oti(chromas_a, chromas_b, med_a, med_b, get_csm_cosine)  d = 480 (:178)
//   scores[mfccs|ssms|chromas] = SW(csm_to_binary(CSM_x, kappa))                      (:174-181)
//   W = ((0 + getWCSM(CSM_m)) + getWCSM(CSM_s)) + getWCSM(CSM_c); E = exp(-W)          (:184-188)
//   scores[early] = SW(csm_to_binary(E, kappa))                                        (:189)
// Stages (workspace chunk of P pairs, every per-pair matrix padded to ld x ld):
//   k_ef_rows     per block row: squared norm (euclid) / L2-normalised copy (cosine; zero -> 1)
//   k_ef_oti      per pair: get_oti(med_a, med_b), first maximum
//   k_ef_csm<K>   64x64 MFMA f32 tiles x pairs (blockIdx.z); the OTI roll of the query's 12-bin
//                 blocks is applied in the tile loader
//   k_ef_binarize wave per (row, pair, matrix): the round(kappa * N) smallest -> 1, ties lowest
//                 column; 16 rows per block packed into u16 bit words (the SW input)
//   k_ef_kmin*    thread per (row|column, pair, matrix): mean of the K smallest (K <= 16;
//                 k_ef_kmean, a wave-per-line select, beyond that)
//   k_ef_wsum     elementwise: E = exp(-(((0 + W_m) + W_s) + W_c)) in float32, exp = canon_expf
//   SW            launch_swb_batch (misc.hip) over the 4P bit planes
// Tolerance vs the reference: the GEMMs' summation order (BLAS vs MFMA), the k-smallest means'
// order (ascending here, np.partition's unspecified there) and exp (canon_expf vs numpy's); every
// other step is the reference's float32 arithmetic. Against the canonical CPU oracle
// (oracle/ef_oracle.cpp) all four scores are bit-identical.
#include <cmath>
#include <cstdlib>

#include "common.hpp"

namespace acoss {

int launch_swb_batch(const uint16_t* W, int64_t wstride, int ldw, const int32_t* rows, const int32_t* cols, int n,
                     int max_rows, int max_cols, void* bnd, double* out, hipStream_t s);
size_t sw_bnd_bytes(int max_rows, int max_cols);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kT = 64, kKC = 32;
constexpr int kBinRegs = 16;  // row keys per lane kept in registers by k_ef_binarize (N <= 1024)
constexpr int kKmax = 16;     // largest K of the streaming k-smallest means

__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __builtin_bit_cast(unsigned, f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void k_ef_rows(const float* __restrict__ X, int64_t nrows, int d, int normalise, float* __restrict__ Xo,
                          float* __restrict__ sq) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const float* x = X + row * d;
  float s = 0.0f;
  for (int c = lane; c < d; c += 64) s += x[c] * x[c];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (!normalise) {
    if (lane == 0) sq[row] = s;
    return;
  }
  const float nrm = sqrtf(s);
  const float den = nrm != 0.0f ? nrm : 1.0f;  // XNorm[XNorm == 0] = 1 (cross_recurrence.py:67-70)
  for (int c = lane; c < d; c += 64) Xo[row * d + c] = x[c] / den;
}

__global__ void k_ef_oti(const float* __restrict__ med, const int32_t* __restrict__ pairs, int P,
                         int* __restrict__ oti) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const float* a = med + pairs[2 * p] * 12;
  const float* b = med + pairs[2 * p + 1] * 12;
  int best = 0;
  float bv = 0.0f;
  for (int i = 0; i < 12; ++i) {
    float s = 0.0f;
    for (int c = 0; c < 12; ++c) s = s + a[(c - i + 12) % 12] * b[c];
    if (i == 0 || s > bv) {
      bv = s;
      best = i;
    }
  }
  oti[p] = best;
}

struct EfPairs {
  const int32_t* pairs;
  const int64_t* off;  // block offsets per track
  const int32_t* nb;   // blocks per track
};

__device__ __forceinline__ void pair_dims(const EfPairs& E, int p, int* a, int* b, int* M, int* N) {
  *a = E.pairs[2 * p];
  *b = E.pairs[2 * p + 1];
  *M = E.nb[*a];
  *N = E.nb[*b];
}

template <int KIND>  // 0 euclid, 1 cosine (pre-normalised rows, query blocks rolled by oti)
__global__ __launch_bounds__(256) void k_ef_csm(const float* __restrict__ bank, int d, const float* __restrict__ sq,
                                                EfPairs E, const int* __restrict__ oti, int ld,
                                                float* __restrict__ out) {
  // two LDS buffers: the next K chunk is loaded into registers while the MFMAs read this one,
  // then stored to the other buffer; one barrier per chunk
  __shared__ float Xs[2][kT][kKC + 1];
  __shared__ float Ys[2][kT][kKC + 1];
  // 1-D grid of tiles x tiles x pairs, XCD-aware: the tiles of one pair run on one XCD, so its
  // row and column panels are read into that XCD's L2 once and reused by the pair's other tiles
  const int tiles = (ld + kT - 1) / kT;
  const int lg = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int p = lg / (tiles * tiles), tix = lg - p * tiles * tiles;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  const int bi = (tix / tiles) * kT, bj = (tix % tiles) * kT;
  if (bi >= M || bj >= N) return;
  const float* X = bank + E.off[a] * d;
  const float* Y = bank + E.off[b] * d;
  const int roll = KIND == 1 ? oti[p] : 0;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  // loader: per load i, lane t reads row t / 32 + 8 i, k = k0 + t % 32 (32 lanes = one 128-B run)
  constexpr int kPer = kT * kKC / 256;
  const int lc = t % kKC, lr0 = t / kKC;
  float xr[kPer], yr[kPer];
  auto gload = [&](int k0) {
    const int k = k0 + lc;
    int kx = k;
    if (KIND == 1 && roll) {  // X1 = np.roll(X blocks, oti, axis=2): X1[k] = X[blk*12 + (cc - oti) mod 12]
      const int blk = k / 12, cc = k - blk * 12;
      kx = blk * 12 + (cc - roll + 12) % 12;
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int r = lr0 + (256 / kKC) * i;
      xr[i] = (bi + r < M && k < d) ? X[(size_t)(bi + r) * d + kx] : 0.0f;
      yr[i] = (bj + r < N && k < d) ? Y[(size_t)(bj + r) * d + k] : 0.0f;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      Xs[buf][lr0 + (256 / kKC) * i][lc] = xr[i];
      Ys[buf][lr0 + (256 / kKC) * i][lc] = yr[i];
    }
  };
  f32x16 acc = {};
  gload(0);
  sstore(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < d; k0 += kKC) {
    const bool more = k0 + kKC < d;
    if (more) gload(k0 + kKC);
#pragma unroll
    for (int kk = 0; kk < kKC; kk += 2) {
      const float xa = Xs[buf][32 * wr + (lane & 31)][kk + (lane >> 5)];
      const float yb = Ys[buf][32 * wc + (lane & 31)][kk + (lane >> 5)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa, yb, acc, 0, 0, 0);
    }
    if (more) sstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  float* o = out + (size_t)p * ld * ld;
  const int col = bj + 32 * wc + (lane & 31);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = bi + 32 * wr + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    if (row < M && col < N) {
      float v;
      if (KIND == 1) {
        v = 1.0f - acc[reg];
      } else {
        float c2 = (sq[E.off[a] + row] + sq[E.off[b] + col]) - 2.0f * acc[reg];
        if (c2 < 0.0f) c2 = 0.0f;
        v = sqrtf(c2);
      }
      o[(size_t)row * ld + col] = v;
    }
  }
}

typedef float f32x4e __attribute__((ext_vector_type(4)));

// Row-padded copy of a feature bank (nrows x d -> nrows x ldp, zeros in [d, ldp)) so that
// k_ef_csm_w's 16-byte row loads are aligned for any d (the SSM blocks have d = 1225). The zero
// columns add exact +0 terms at the end of every fmaf chain, so the CSM is unchanged bit for bit.
__global__ void k_ef_pad_rows(const float* __restrict__ X, int64_t nrows, int d, int ldp, float* __restrict__ Xp) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  for (int c = threadIdx.x & 63; c < ldp; c += 64) Xp[row * ldp + c] = c < d ? X[row * d + c] : 0.0f;
}

// Euclidean CSM tiles with no LDS and no barriers: one WAVE per 64 x 64 output tile (2 x 2
// accumulators of 32x32x2 f32 MFMAs), operands loaded straight into registers. Per block of KB
// k-values, lane l (r = l % 32, h = l / 32) reads KB / 2 contiguous floats of each of its four
// operand rows (k0 + h KB / 2 ..., 16-byte loads: the two halves cover KB floats of the row),
// and one v_permlane32_swap per register pair turns that into the MFMA layout (step s: half h
// holds k0 + 2 s + h), so every output is the same ascending-k fmaf chain as k_ef_csm:
// bit-identical. The loads run DEPTH - 1 blocks ahead of the multiplies (a ring of register
// blocks; the last blocks' look-ahead loads are clamped to a valid block and never used).
// Needs d % 4 == 0 (16-byte aligned rows; acoss_earlyfusion pads the SSM bank).
#ifndef ACOSS_EF_KB
#define ACOSS_EF_KB 16
#endif
#ifndef ACOSS_EF_DEPTH
#define ACOSS_EF_DEPTH 3
#endif
#ifndef ACOSS_EF_WPE
#define ACOSS_EF_WPE 2
#endif
// KIND = 1: the cosine chroma CSM of get_csm_blocked_oti (pre-normalised rows, 1 - dot): blocks
// of KB = 24 k-values, so each half-wave holds one whole 12-bin chroma block of a row and the
// query rows' OTI roll (X1[12 g + c] = X[12 g + (c - oti) mod 12], wave-uniform per pair) is a
// register rotation; needs d % 24 == 0.
// TILE = 64: 2 x 2 accumulators per wave; TILE = 32: one (the beat-block CSMs of short tracks,
// M, N ~ 14..47 at Da-TACOS lengths, where a 64 x 64 tile is mostly padding).
template <int KIND, int TILE = 64>
__global__ __launch_bounds__(256, ACOSS_EF_WPE) void k_ef_csm_w(const float* __restrict__ bank, int d,
                                                                const float* __restrict__ sq, EfPairs E,
                                                                const int* __restrict__ oti, int ld,
                                                                int n_tiles, float* __restrict__ out) {
  constexpr int KB = KIND == 1 ? 24 : ACOSS_EF_KB, DEPTH = ACOSS_EF_DEPTH, NQ = KB / 8;  // NQ 16-byte loads per row
  constexpr int NA = TILE / 32;  // 32 x 32 accumulators per tile side
  constexpr int NO = 2 * NA;     // operand rows per lane: NA query rows, then NA reference rows
  const int tiles = (ld + TILE - 1) / TILE;
  const int lb = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int tile = lb * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (tile >= n_tiles) return;
  const int p = tile / (tiles * tiles), tix = tile - p * tiles * tiles;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  const int bi = (tix / tiles) * TILE, bj = (tix % tiles) * TILE;
  if (bi >= M || bj >= N) return;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  // this lane's operand rows (clamped into the track: rows past M / N are never stored)
  const float* rows[NO];
#pragma unroll
  for (int o = 0; o < NA; ++o) {
    rows[o] = bank + (E.off[a] + min(bi + 32 * o + r, M - 1)) * (int64_t)d + (KB / 2) * h;
    rows[NA + o] = bank + (E.off[b] + min(bj + 32 * o + r, N - 1)) * (int64_t)d + (KB / 2) * h;
  }
  const int nfull = d / KB;
  f32x4e ring[DEPTH][NO][NQ];
  auto load = [&](f32x4e (&v)[NO][NQ], int blk) {  // a whole block (clamped to the last whole one)
    const int k0 = min(blk, nfull - 1) * KB;
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[o][q] = *reinterpret_cast<const f32x4e*>(rows[o] + k0 + 4 * q);
  };
  f32x16 acc[NA][NA] = {};
  const int roll = KIND == 1 ? __builtin_amdgcn_readfirstlane(oti[p]) : 0;
  // operands of steps s and s + KB / 4 come from registers 2 s and 2 s + 1 of every operand row
  auto mul = [&](const f32x4e (&vin)[NO][NQ]) {
    f32x4e v[NO][NQ];
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[o][q] = vin[o][q];
    if constexpr (KIND == 1) {  // rotate the query rows' 12-bin block by the pair's OTI
      if (roll) {
#pragma unroll
        for (int o = 0; o < NA; ++o) {
          float e[12], t[12];
#pragma unroll
          for (int c = 0; c < 12; ++c) e[c] = vin[o][c >> 2][c & 3];
#pragma unroll
          for (int R = 1; R < 12; ++R)
            if (roll == R) {
#pragma unroll
              for (int c = 0; c < 12; ++c) t[c] = e[(c - R + 12) % 12];
            }
#pragma unroll
          for (int c = 0; c < 12; ++c) v[o][c >> 2][c & 3] = t[c];
        }
      }
    }
    float op[NO][KB / 2];
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int s2 = 0; s2 < KB / 4; ++s2) {
        const float lo = v[o][s2 >> 1][(s2 & 1) * 2], hi = v[o][s2 >> 1][(s2 & 1) * 2 + 1];
        const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, lo),
                                                         __builtin_bit_cast(unsigned, hi), false, false);
        op[o][s2] = __builtin_bit_cast(float, (unsigned)sw[0]);
        op[o][s2 + KB / 4] = __builtin_bit_cast(float, (unsigned)sw[1]);
      }
#pragma unroll
    for (int st = 0; st < KB / 2; ++st)
#pragma unroll
      for (int ti = 0; ti < NA; ++ti)
#pragma unroll
        for (int tj = 0; tj < NA; ++tj)
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x2f32(op[ti][st], op[NA + tj][st], acc[ti][tj], 0, 0, 0);
  };
  if (nfull > 0) {
#pragma unroll
    for (int i = 0; i < DEPTH - 1; ++i) load(ring[i], i);
#pragma unroll 1
    for (int kb = 0; kb < nfull; kb += DEPTH) {
#pragma unroll
      for (int j = 0; j < DEPTH; ++j) {
        load(ring[(j + DEPTH - 1) % DEPTH], kb + j + DEPTH - 1);
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the multiplies they overlap
        if (kb + j < nfull) mul(ring[j]);
      }
    }
  }
  if (d % KB) {  // the partial tail block: zeros past d
    const int k0 = nfull * KB;
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        ring[0][o][q] = k0 + (KB / 2) * h + 4 * q < d ? *reinterpret_cast<const f32x4e*>(rows[o] + k0 + 4 * q)
                                                       : f32x4e{0.0f, 0.0f, 0.0f, 0.0f};
    mul(ring[0]);
  }
  float* ob = out + (size_t)p * ld * ld;
#pragma unroll
  for (int ti = 0; ti < NA; ++ti)
#pragma unroll
    for (int tj = 0; tj < NA; ++tj) {
      const int col = bj + 32 * tj + r;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = bi + 32 * ti + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (row < M && col < N) {
          if constexpr (KIND == 1) {
            ob[(size_t)row * ld + col] = 1.0f - acc[ti][tj][reg];
          } else {
            float c2 = (sq[E.off[a] + row] + sq[E.off[b] + col]) - 2.0f * acc[ti][tj][reg];
            if (c2 < 0.0f) c2 = 0.0f;
            ob[(size_t)row * ld + col] = sqrtf(c2);
          }
        }
      }
    }
}

// Short tracks (every track <= 64 blocks: the 32 x 32 tiles of k_ef_csm_w<KIND, 32>), PP pairs per
// wave. The pairs of a call come in (reference band, query) order, so runs of consecutive pairs
// share their query track: a wave takes PP consecutive pairs and, when they share it, loads the
// query rows once for all PP tiles (1 + PP row loads per block instead of 2 PP) and keeps PP
// independent accumulators in flight. Otherwise (a run boundary) it takes the pairs one at a time.
// Each output is the same ascending-k fmaf chain as k_ef_csm_w: bit-identical. Used for the cosine
// chroma CSM (-12 %); the euclid CSMs did not gain (profiles/r06/ef_short_w4/README.txt). Work unit:
// (group of PP pairs, tile row ti, tile column tj).
// pairs per wave of the cosine chroma CSM of short tracks. The euclid CSMs (d = 1000, 1228) keep one
// pair per wave: 2 or 4 pairs sharing the query rows, and a deeper load ring, left them within
// +-5 % (profiles/r06/ef_short_w4/README.txt); the cosine one (d = 480, 24-k blocks) is 12 % faster
// with 2 (4: 40 % slower, registers)
constexpr int kEfPPc = 2;

template <int KIND, int PP>
__device__ __forceinline__ void ef_csm_w4_tiles(const float* __restrict__ bank, int d, const float* __restrict__ sq,
                                                const EfPairs& E, const int* __restrict__ oti, int ld, int pbase,
                                                int npp, int ti, int tj, float* __restrict__ out) {
  constexpr int KB = KIND == 1 ? 24 : ACOSS_EF_KB, DEPTH = ACOSS_EF_DEPTH, NQ = KB / 8;
  constexpr int NO = 1 + PP;  // operand rows per lane: the query row, then one reference row per pair
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int a = E.pairs[2 * pbase], M = E.nb[a];
  const int bi = ti * 32, bj = tj * 32;
  int bq[PP], Nq[PP];
  const float* rows[NO];
  rows[0] = bank + (E.off[a] + min(bi + r, M - 1)) * (int64_t)d + (KB / 2) * h;
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    const int qq = min(q, npp - 1);  // pairs past the group's end repeat its last one (never stored)
    bq[q] = E.pairs[2 * (pbase + qq) + 1];
    Nq[q] = E.nb[bq[q]];
    rows[1 + q] = bank + (E.off[bq[q]] + min(bj + r, Nq[q] - 1)) * (int64_t)d + (KB / 2) * h;
  }
  const int nfull = d / KB;
  f32x4e ring[DEPTH][NO][NQ];
  auto load = [&](f32x4e (&v)[NO][NQ], int blk) {
    const int k0 = min(blk, nfull - 1) * KB;
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[o][q] = *reinterpret_cast<const f32x4e*>(rows[o] + k0 + 4 * q);
  };
  f32x16 acc[PP] = {};
  int roll[PP];
#pragma unroll
  for (int q = 0; q < PP; ++q) roll[q] = KIND == 1 ? __builtin_amdgcn_readfirstlane(oti[pbase + min(q, npp - 1)]) : 0;
  auto mul = [&](const f32x4e (&vin)[NO][NQ]) {
    float op[NO][KB / 2];
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int s2 = 0; s2 < KB / 4; ++s2) {
        const float lo = vin[o][s2 >> 1][(s2 & 1) * 2], hi = vin[o][s2 >> 1][(s2 & 1) * 2 + 1];
        const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, lo),
                                                         __builtin_bit_cast(unsigned, hi), false, false);
        op[o][s2] = __builtin_bit_cast(float, (unsigned)sw[0]);
        op[o][s2 + KB / 4] = __builtin_bit_cast(float, (unsigned)sw[1]);
      }
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      float oq[KB / 2];  // the query operand, rolled by pair q's OTI (cosine)
#pragma unroll
      for (int st = 0; st < KB / 2; ++st) oq[st] = op[0][st];
      if constexpr (KIND == 1) {
        if (roll[q]) {  // the query row's 12-bin block rotated, as k_ef_csm_w<1> does before the swap
          float e[12], t[12];
#pragma unroll
          for (int c = 0; c < 12; ++c) e[c] = vin[0][c >> 2][c & 3];
#pragma unroll
          for (int R = 1; R < 12; ++R)
            if (roll[q] == R) {
#pragma unroll
              for (int c = 0; c < 12; ++c) t[c] = e[(c - R + 12) % 12];
            }
#pragma unroll
          for (int s2 = 0; s2 < KB / 4; ++s2) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, t[2 * s2]),
                                                             __builtin_bit_cast(unsigned, t[2 * s2 + 1]), false, false);
            oq[s2] = __builtin_bit_cast(float, (unsigned)sw[0]);
            oq[s2 + KB / 4] = __builtin_bit_cast(float, (unsigned)sw[1]);
          }
        }
      }
#pragma unroll
      for (int st = 0; st < KB / 2; ++st) acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(oq[st], op[1 + q][st], acc[q], 0, 0, 0);
    }
  };
  if (nfull > 0) {
#pragma unroll
    for (int i = 0; i < DEPTH - 1; ++i) load(ring[i], i);
#pragma unroll 1
    for (int kb = 0; kb < nfull; kb += DEPTH) {
#pragma unroll
      for (int j = 0; j < DEPTH; ++j) {
        load(ring[(j + DEPTH - 1) % DEPTH], kb + j + DEPTH - 1);
        __builtin_amdgcn_sched_barrier(0);
        if (kb + j < nfull) mul(ring[j]);
      }
    }
  }
  if (d % KB) {
    const int k0 = nfull * KB;
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        ring[0][o][q] = k0 + (KB / 2) * h + 4 * q < d ? *reinterpret_cast<const f32x4e*>(rows[o] + k0 + 4 * q)
                                                       : f32x4e{0.0f, 0.0f, 0.0f, 0.0f};
    mul(ring[0]);
  }
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    if (q >= npp) break;
    float* ob = out + (size_t)(pbase + q) * ld * ld;
    const int col = bj + r;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = bi + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (row < M && col < Nq[q]) {
        if constexpr (KIND == 1) {
          ob[(size_t)row * ld + col] = 1.0f - acc[q][reg];
        } else {
          float c2 = (sq[E.off[a] + row] + sq[E.off[bq[q]] + col]) - 2.0f * acc[q][reg];
          if (c2 < 0.0f) c2 = 0.0f;
          ob[(size_t)row * ld + col] = sqrtf(c2);
        }
      }
    }
  }
}

template <int KIND, int PP>
__global__ __launch_bounds__(256, ACOSS_EF_WPE) void k_ef_csm_w4(const float* __restrict__ bank, int d,
                                                                 const float* __restrict__ sq, EfPairs E,
                                                                 const int* __restrict__ oti, int ld, int n_pairs,
                                                                 int n_units, float* __restrict__ out) {
  const int tiles = (ld + 31) / 32;
  const int lb = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int unit = lb * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= n_units) return;
  const int g = unit / (tiles * tiles), tix = unit - g * tiles * tiles;
  const int ti = tix / tiles, tj = tix - ti * tiles;
  const int p0 = g * PP, npp = min(PP, n_pairs - p0);
  bool same = true;  // wave-uniform: every pair of the group has the group's query track
  for (int q = 1; q < npp; ++q) same = same && E.pairs[2 * (p0 + q)] == E.pairs[2 * p0];
  // a pair's tile (ti, tj) exists when both tracks reach it; ragged tracks (14..47 blocks at
  // Da-TACOS lengths) leave many groups where only some pairs reach tile column tj
  int nv = 0;
  for (int q = 0; q < npp; ++q)
    nv += (ti * 32 < E.nb[E.pairs[2 * (p0 + q)]] && tj * 32 < E.nb[E.pairs[2 * (p0 + q) + 1]]) ? 1 : 0;
  if (same && nv == npp) {
    ef_csm_w4_tiles<KIND, PP>(bank, d, sq, E, oti, ld, p0, npp, ti, tj, out);
    return;
  }
  for (int q = 0; q < npp; ++q)  // a run boundary or a partial group: one pair at a time
    if (ti * 32 < E.nb[E.pairs[2 * (p0 + q)]] && tj * 32 < E.nb[E.pairs[2 * (p0 + q) + 1]])
      ef_csm_w4_tiles<KIND, 1>(bank, d, sq, E, oti, ld, p0 + q, 1, ti, tj, out);
}

// Euclidean CSMs of short tracks (<= 128 blocks) with the reference columns PACKED: the pairs of a
// call come in (reference band, query) order, so consecutive pairs share their query track; the
// columns of a run of such pairs (all blocks of every reference track, concatenated) fill
// 32 NB-wide tiles with no per-pair padding. A tile per pair wastes the part of the tile past the
// track's block count (14..47 blocks at Da-TACOS lengths: 2.3x the useful MFMA work over rows and
// columns with 32 x 32 tiles); packing leaves only the rows' padding (1.5x). Lane r of a tile
// holds NB packed columns, each with its own reference track, block and output pair, so the same
// 32x32x2 MFMA chains as k_ef_csm_w<0, .> compute every output (bit-identical: the same operands in
// the same ascending-k fmaf order). Work unit: (group of kEfPack consecutive pairs, row tile ti,
// packed column tile tc). Within a group the maximal runs of one query track are packed
// separately; tc counts the runs' tiles in order (at most kEfPack * ceil(ld / 32 NB) of them, so
// that is the grid's column-tile count).
// Groups of 64 pairs (one per lane in the walk below): with runs of 32 pairs per query, kernel time
// per 1M Da-TACOS-shape pairs 209 / 148 / 94 / 87 / 85 ms for groups of 4 / 8 / 16 / 32 / 64, against
// 119 ms for a 32 x 32 tile per pair (profiles/r06/ef_pack/README.txt)
#ifndef ACOSS_EF_PACKN
#define ACOSS_EF_PACKN 64
#endif
constexpr int kEfPack = ACOSS_EF_PACKN;
static_assert(kEfPack <= 64, "one pair per lane");

template <int NB>  // packed columns per wave tile: 32 * NB (NB accumulators sharing the query rows)
__global__ __launch_bounds__(256, 4) void k_ef_csm_pack(const float* __restrict__ bank, int d,
                                                                   const float* __restrict__ sq, EfPairs E, int ld,
                                                                   int n_pairs, int n_units, float* __restrict__ out) {
  constexpr int KB = ACOSS_EF_KB, DEPTH = ACOSS_EF_DEPTH, NQ = KB / 8, TW = 32 * NB, NO = 1 + NB;
  const int wt = (ld + 31) / 32;                // row tiles per track
  const int ct = kEfPack * ((ld + TW - 1) / TW);  // column-tile slots per group
  const int lb = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int unit = lb * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= n_units) return;
  const int g = unit / (wt * ct), u = unit - g * wt * ct;
  const int p0 = g * kEfPack, npp = min(kEfPack, n_pairs - p0);
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  // the group's pairs, one per lane (lanes < npp), in two rounds of loads; the walk below reads
  // them with readlane (a chain of dependent scalar loads here cost more than the tile's MFMAs)
  int ga = 0, gb = 0;
  if (lane < npp) {
    ga = E.pairs[2 * (p0 + lane)];
    gb = E.pairs[2 * (p0 + lane) + 1];
  }
  int gm = 0, gn = 0;
  int64_t goa = 0, gob = 0;
  if (lane < npp) {
    gm = E.nb[ga];
    gn = E.nb[gb];
    goa = E.off[ga];
    gob = E.off[gb];
  }
  auto rl64 = [](int64_t v, int l) {
    return ((int64_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  };
  // Walk the group's SUPER-RUNS: a run of L pairs with one query track, extended by the following
  // runs of L pairs whose reference tracks are the same, in the same order (the next queries of a
  // reference band). A super-run of R queries packs its R queries' blocks into the rows and its L
  // references' blocks into the columns: (query k, reference t) is pair s + k L + t. Its tiles
  // are ceil(sum M / 32) x ceil(sum N / TW); u counts the super-runs' tiles in order (at most the
  // per-pair tile count, so the grid's wt * ct slots per group hold them).
  int s0 = 0, L = 0, R = 0, sumM = 0, sumN = 0, tb = 0, nct = 1;
  bool found = false;
  while (s0 < npp) {
    const int a = __builtin_amdgcn_readlane(ga, s0);
    int e = s0 + 1;
    while (e < npp && __builtin_amdgcn_readlane(ga, e) == a) ++e;
    L = e - s0;
    sumN = 0;
    for (int t = s0; t < e; ++t) sumN += __builtin_amdgcn_readlane(gn, t);
    sumM = __builtin_amdgcn_readlane(gm, s0);
    R = 1;
    int f = e;
    while (f + L <= npp) {  // absorb the next run if it is L pairs with the same references
      const int a2 = __builtin_amdgcn_readlane(ga, f);
      bool same = f + L == npp || __builtin_amdgcn_readlane(ga, f + L) != a2;
      for (int t = 0; t < L && same; ++t)
        same = __builtin_amdgcn_readlane(ga, f + t) == a2 &&
               __builtin_amdgcn_readlane(gb, f + t) == __builtin_amdgcn_readlane(gb, s0 + t);
      if (!same) break;
      sumM += __builtin_amdgcn_readlane(gm, f);
      ++R;
      f += L;
    }
    nct = (sumN + TW - 1) / TW;
    const int nt = (sumM + 31) / 32 * nct;
    if (u < tb + nt) {
      found = true;
      break;
    }
    tb += nt;
    s0 = f;
  }
  if (!found) return;
  const int rt = (u - tb) / nct, tc = (u - tb) - rt * nct;
  // packed row gr -> (query k of the super-run, block within it); rows past sum M clamp to the last.
  // Every lane runs every iteration and selects (no per-lane exit from a loop over readlane
  // values: a value a lane keeps from an earlier iteration than its neighbours is divergent,
  // which the compiler must not mistake for the uniform loop counter)
  auto locate_row = [&](int gr, int* k, int* row, int64_t* offa) {
    int pre = 0, kk_ = R - 1, row_ = 0;
    int64_t off_ = 0;
    bool done = false;
    for (int kk = 0; kk < R; ++kk) {
      const int m = __builtin_amdgcn_readlane(gm, s0 + kk * L);
      const int64_t o = rl64(goa, s0 + kk * L);
      const bool hit = !done && (gr < pre + m || kk == R - 1);
      kk_ = hit ? kk : kk_;
      row_ = hit ? min(gr - pre, m - 1) : row_;
      off_ = hit ? o : off_;
      done = done || hit;
      pre += m;
    }
    *k = kk_;
    *row = row_;
    *offa = off_;
  };
  const float* rows[NO];
  {
    int k, row;
    int64_t offa;
    locate_row(rt * 32 + r, &k, &row, &offa);
    rows[0] = bank + (offa + row) * (int64_t)d + (KB / 2) * h;
  }
  // this lane's packed columns (one per accumulator): reference t of the super-run, block c
  int ct_[NB], cc[NB];
  int64_t cob[NB];
  bool cvalid[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int gc = tc * TW + 32 * j + r;
    cvalid[j] = gc < sumN;
    int t = L - 1, pre = 0, cpre = 0, N = 1;
    int64_t offb = 0;
    bool done = false;
    for (int k = 0; k < L; ++k) {  // the last reference takes every column past the others
      const int n = __builtin_amdgcn_readlane(gn, s0 + k);
      const int64_t o = rl64(gob, s0 + k);
      const bool hit = !done && (gc < pre + n || k == L - 1);
      t = hit ? k : t;
      N = hit ? n : N;
      cpre = hit ? pre : cpre;
      offb = hit ? o : offb;
      done = done || hit;
      pre += n;
    }
    ct_[j] = t;
    cc[j] = min(gc - cpre, N - 1);  // clamped for the padding lanes (never stored)
    cob[j] = offb;
    rows[1 + j] = bank + (offb + cc[j]) * (int64_t)d + (KB / 2) * h;
  }
  const int nfull = d / KB;
  f32x4e ring[DEPTH][NO][NQ];
  auto load = [&](f32x4e (&v)[NO][NQ], int blk) {
    const int k0 = min(blk, nfull - 1) * KB;
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) v[o][qq] = *reinterpret_cast<const f32x4e*>(rows[o] + k0 + 4 * qq);
  };
  f32x16 acc[NB] = {};
  auto mul = [&](const f32x4e (&vin)[NO][NQ]) {
    float op[NO][KB / 2];
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int s2 = 0; s2 < KB / 4; ++s2) {
        const float lo = vin[o][s2 >> 1][(s2 & 1) * 2], hi = vin[o][s2 >> 1][(s2 & 1) * 2 + 1];
        const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, lo),
                                                         __builtin_bit_cast(unsigned, hi), false, false);
        op[o][s2] = __builtin_bit_cast(float, (unsigned)sw[0]);
        op[o][s2 + KB / 4] = __builtin_bit_cast(float, (unsigned)sw[1]);
      }
#pragma unroll
    for (int st = 0; st < KB / 2; ++st)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(op[0][st], op[1 + j][st], acc[j], 0, 0, 0);
  };
  if (nfull > 0) {
#pragma unroll
    for (int i = 0; i < DEPTH - 1; ++i) load(ring[i], i);
#pragma unroll 1
    for (int kb = 0; kb < nfull; kb += DEPTH) {
#pragma unroll
      for (int j = 0; j < DEPTH; ++j) {
        load(ring[(j + DEPTH - 1) % DEPTH], kb + j + DEPTH - 1);
        __builtin_amdgcn_sched_barrier(0);
        if (kb + j < nfull) mul(ring[j]);
      }
    }
  }
  if (d % KB) {
    const int k0 = nfull * KB;
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq)
        ring[0][o][qq] = k0 + (KB / 2) * h + 4 * qq < d ? *reinterpret_cast<const f32x4e*>(rows[o] + k0 + 4 * qq)
                                                         : f32x4e{0.0f, 0.0f, 0.0f, 0.0f};
    mul(ring[0]);
  }
  float sqc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) sqc[j] = sq[cob[j] + cc[j]];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int gr = rt * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
    if (gr >= sumM) continue;
    int k, row;
    int64_t offa;
    locate_row(gr, &k, &row, &offa);
    const float sqr = sq[offa + row];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (!cvalid[j]) continue;
      float c2 = (sqr + sqc[j]) - 2.0f * acc[j][reg];
      if (c2 < 0.0f) c2 = 0.0f;
      out[(size_t)(p0 + s0 + k * L + ct_[j]) * ld * ld + (size_t)row * ld + cc[j]] = sqrtf(c2);
    }
  }
}

// The nn smallest of every row -> 1, ties lowest column (csm_to_binary). A block of 16 waves
// takes 16 rows (one wave per row) and writes them as one row of u16 bit words (bit r = row
// 16g + r) in LDS, then to the pair's bit plane for SW. blockIdx.z = CSM plane, written to
// bit plane z + plane0 of the pair (plane stride = wplane words, 4 planes per pair).
// The nn-th smallest (1-based) of the wave's keys kr (KB per lane) within [lo, hi], by radix
// select: from the highest bit where lo and hi differ, 8-bit digits, each digit from one LDS
// histogram of the candidates (keys matching the digits so far) and one wave scan of its 256
// bins; about 4 passes instead of the ~26 count passes of a bisection over [lo, hi]. Every key
// issues one unconditional ds_add: candidates to their digit's bin, the rest to a lane-private
// sink word (hist: 256 bins + 64 sink words, this wave's own). Same answer as the bisection:
// the least key v with #(keys <= v) >= nn.
template <int KB>
__device__ __forceinline__ unsigned radix_kth(const unsigned (&kr)[KB], unsigned lo, unsigned hi, int nn, int lane,
                                              unsigned* hist) {
  if (lo >= hi) return lo;
  typedef __attribute__((address_space(3))) unsigned lds_u32;
  const unsigned hb = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(size_t)(lds_u32*)hist);
  const unsigned sk = hb + 1024u + 4u * (unsigned)lane;
  int sh = 32 - __builtin_clz(lo ^ hi);  // bits [0, sh) differ inside [lo, hi]
  unsigned prefix = sh >= 32 ? 0u : (lo >> sh) << sh;
  int rank = nn - 1;
  while (sh > 0) {  // wave-uniform
    const int dsh = sh > 8 ? sh - 8 : 0;
    reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
    const unsigned P = sh >= 32 ? 0u : prefix >> sh;
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const unsigned k = kr[q];
      const bool cand = sh >= 32 || (k >> sh) == P;
      const unsigned d = (k >> dsh) & 0xffu;
      const unsigned a = cand ? hb + 4u * d : sk;
      __hip_atomic_fetch_add((lds_u32*)(size_t)a, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    __builtin_amdgcn_wave_barrier();
    const uint4 hv = reinterpret_cast<const uint4*>(hist)[lane];  // bins 4 lane .. 4 lane + 3
    const int sl = (int)(hv.x + hv.y + hv.z + hv.w);
    const int S = wave_incl_scan(sl);
    const int E = S - sl;
    const int src = __builtin_ctzll(__ballot(E <= rank && rank < S));
    int r = rank - __builtin_amdgcn_readlane(E, src);
    const int h0 = __builtin_amdgcn_readlane((int)hv.x, src), h1 = __builtin_amdgcn_readlane((int)hv.y, src),
              h2 = __builtin_amdgcn_readlane((int)hv.z, src);
    unsigned b = 0;
    if (r >= h0) {
      r -= h0;
      b = 1;
      if (r >= h1) {
        r -= h1;
        b = 2;
        if (r >= h2) {
          r -= h2;
          b = 3;
        }
      }
    }
    prefix |= (4u * (unsigned)src + b) << dsh;
    rank = r;
    sh = dsh;
    __builtin_amdgcn_wave_barrier();
  }
  return prefix;
}

template <int KB>  // keys per lane held in registers (rows of up to 64 * KB columns)
__device__ __forceinline__ void ef_binarize_row(const float* __restrict__ x, int N, double kappa, int lane,
                                                unsigned* bits, unsigned bit, unsigned* hist) {
  if (kappa == 0.0) {
    for (int c = lane; c < N; c += 64) atomicOr(&bits[c], bit);
    return;
  }
  // np.round: half to even. The host wrapper rejects nn >= N as the reference's argpartition does;
  // the clamp keeps the radix select's rank inside the row if the ABI is called directly
  const int nn = min(kappa < 1.0 ? (int)rint(kappa * (double)N) : (int)kappa, N);
  if (nn <= 0) return;
  const int per = (N + 63) / 64;
  const int c0 = lane * per, c1 = min(N, c0 + per);
  unsigned lo = 0, hi = 0xffffffffu;
  unsigned kr[KB];
  const bool inreg = per <= KB;
  if (inreg) {  // the row's keys in registers: one pass over memory
#pragma unroll
    for (int q = 0; q < KB; ++q) kr[q] = (q < per && c0 + q < c1) ? fkey(x[c0 + q]) : 0xffffffffu;
    unsigned mn = 0xffffffffu, mx = 0u;  // bound the search by the row's range
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      mn = min(mn, kr[q]);
      if (q < per && c0 + q < c1) mx = max(mx, kr[q]);
    }
    lo = wave_min_u32(mn);
    hi = wave_max_u32(mx);
    lo = radix_kth(kr, lo, hi, nn, lane, hist);
  } else {
    while (lo < hi) {
      const unsigned mid = lo + ((hi - lo) >> 1);
      int c = 0;
      for (int k = c0; k < c1; ++k) c += fkey(x[k]) <= mid;
      if (wave_sum(c) >= nn)
        hi = mid;
      else
        lo = mid + 1;
    }
  }
  const unsigned kth = lo;
  int less = 0, eq = 0;
  if (inreg) {  // the keys are still in registers: no second and third read of the row
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      less += kr[q] < kth;
      eq += kr[q] == kth;
    }
    const int take_eq = nn - wave_sum(less);
    int seen = wave_incl_scan(eq) - eq;
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      bool v = kr[q] < kth;
      if (kr[q] == kth && q < per && c0 + q < c1) {
        v = seen < take_eq;
        ++seen;
      }
      if (v) atomicOr(&bits[c0 + q], bit);
    }
    return;
  }
  for (int k = c0; k < c1; ++k) {
    const unsigned kk = fkey(x[k]);
    less += kk < kth;
    eq += kk == kth;
  }
  const int take_eq = nn - wave_sum(less);
  int seen = wave_incl_scan(eq) - eq;
  for (int k = c0; k < c1; ++k) {
    const unsigned kk = fkey(x[k]);
    bool v = kk < kth;
    if (kk == kth) {
      v = seen < take_eq;
      ++seen;
    }
    if (v) atomicOr(&bits[k], bit);
  }
}

// Rows of at most 64 columns (one key per lane) with a small nn (Da-TACOS beat blocks: N ~ 14..47,
// nn = round(kappa N) ~ 1..5): nn rounds of (wave minimum of the remaining keys, the lowest lane
// holding it leaves and sets its bit). Each round takes the least remaining key and, among equal
// keys, the lowest column, so the nn lanes taken are exactly csm_to_binary's nn smallest with ties
// to the lowest column -- the radix select's answer at a fraction of its passes.
__device__ __forceinline__ void ef_binarize_row_knock(const float* __restrict__ x, int N, int nn, int lane,
                                                      unsigned* bits, unsigned bit) {
  unsigned k = lane < N ? fkey(x[lane]) : 0xffffffffu;
  bool alive = lane < N;
  for (int t = 0; t < nn; ++t) {  // wave-uniform
    const unsigned m = wave_min_u32(alive ? k : 0xffffffffu);
    const int src = __builtin_ctzll(__ballot(alive && k == m));
    if (lane == src) {
      alive = false;
      atomicOr(&bits[lane], bit);
    }
  }
}
constexpr int kKnockMax = 16;  // largest nn taken by ef_binarize_row_knock

__global__ __launch_bounds__(1024) void k_ef_binarize(const float* __restrict__ C, int64_t mat_stride, int ld,
                                                      EfPairs E, double kappa, uint16_t* __restrict__ Wb,
                                                      int64_t wplane, int plane0) {
  extern __shared__ unsigned bits[];
  __shared__ __attribute__((aligned(16))) unsigned s_hist[16][256 + 64];  // radix_kth, one per wave
  const int p = blockIdx.y, m = blockIdx.z, g = blockIdx.x;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  if (16 * g >= M) return;  // whole block: no barrier skipped by part of it
  for (int c = threadIdx.x; c < N; c += 1024) bits[c] = 0;
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = 16 * g + w;
  if (row < M) {
    const float* xr = C + m * mat_stride + (size_t)p * ld * ld + (size_t)row * ld;
    const int nn = min(kappa < 1.0 ? (int)rint(kappa * (double)N) : (int)kappa, N);  // as ef_binarize_row
    if (N <= 64 && kappa != 0.0 && nn <= kKnockMax) {
      if (nn > 0) ef_binarize_row_knock(xr, N, nn, lane, bits, 1u << w);
    } else if (N <= 64 * 8)  // EarlyFusion's ~450-block tracks: 8 key registers halve the count passes
      ef_binarize_row<8>(xr, N, kappa, lane, bits, 1u << w, s_hist[w]);
    else
      ef_binarize_row<kBinRegs>(xr, N, kappa, lane, bits, 1u << w, s_hist[w]);
  }
  __syncthreads();
  uint16_t* o = Wb + ((size_t)p * 4 + plane0 + m) * wplane + (size_t)g * ld;
  for (int c = threadIdx.x; c < N; c += 1024) o[c] = (uint16_t)bits[c];
}

// k_ef_binarize for batches whose tracks all have at most 64 blocks and a small nn (Da-TACOS beat
// blocks, kappa = 0.1: nn = 1..6): ONE WAVE per (pair, matrix), lane r = row r. The lane loads its
// row's keys into registers (16-byte loads), then nn rounds each take the row's least key not yet
// taken (strict <, columns ascending: the lowest column among equal keys, as csm_to_binary's tie
// rule here); a ballot per column then gives lane c its column's 64-bit row mask, which
// it writes as the u16 words of the SW bit plane. No LDS, no barrier, no cross-lane reduction per
// round (k_ef_binarize_small spent 4 waves, two block barriers and a 6-stage wave minimum per round
// and row). Same selected set as every other binarize kernel.
__global__ __launch_bounds__(256) void k_ef_binarize_lanes(const float* __restrict__ C, int64_t mat_stride, int ld,
                                                           EfPairs E, double kappa, uint16_t* __restrict__ Wb,
                                                           int64_t wplane, int plane0, int nplanes, int n_units) {
  const int unit = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= n_units) return;
  const int p = unit / nplanes, m = unit - p * nplanes;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  const int lane = threadIdx.x & 63;
  const int nn = min(kappa < 1.0 ? (int)rint(kappa * (double)N) : (int)kappa, N);  // as ef_binarize_row
  unsigned long long sel = 0ull;  // this lane's row: its selected columns
  if (kappa == 0.0) {
    sel = N >= 64 ? ~0ull : ((1ull << N) - 1ull);
  } else if (nn > 0) {
    const float* xr = C + m * mat_stride + (size_t)p * ld * ld + (size_t)min(lane, M - 1) * ld;
    unsigned key[64];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (4 * q < N) {  // wave-uniform; ld is a multiple of 4, so the 16-byte load stays in the row
        const f32x4e v = *reinterpret_cast<const f32x4e*>(xr + 4 * q);
#pragma unroll
        for (int u = 0; u < 4; ++u) key[4 * q + u] = 4 * q + u < N ? fkey(v[u]) : 0xffffffffu;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) key[4 * q + u] = 0xffffffffu;
      }
    }
#pragma unroll 1
    for (int t = 0; t < nn; ++t) {  // wave-uniform; nn <= N, so an untaken column always exists
      unsigned bk = 0xffffffffu;
      int bc = -1;
#pragma unroll
      for (int c = 0; c < 64; ++c) {
        if (c < N) {  // wave-uniform
          const bool better = !((sel >> c) & 1ull) && (bc < 0 || key[c] < bk);
          bk = better ? key[c] : bk;
          bc = better ? c : bc;
        }
      }
      sel |= 1ull << bc;
    }
  }
  const unsigned long long rows = M >= 64 ? ~0ull : ((1ull << M) - 1ull);
  unsigned long long colbits = 0ull;
#pragma unroll
  for (int c = 0; c < 64; ++c) {
    if (c < N) {
      const unsigned long long bcol = __ballot((sel >> c) & 1ull) & rows;
      colbits = lane == c ? bcol : colbits;
    }
  }
  const int ng = (M + 15) / 16;
  uint16_t* o = Wb + ((size_t)p * 4 + plane0 + m) * wplane;
  if (lane < N)
    for (int g = 0; g < ng; ++g) o[(size_t)g * ld + lane] = (uint16_t)(colbits >> (16 * g));
}

// k_ef_binarize for batches whose tracks all have at most 64 blocks (Da-TACOS beat blocks): ONE
// 256-thread block per (pair, matrix) instead of a 1024-thread block per 16 rows; wave w takes
// rows w, w + 4, ... with the same per-row selects as k_ef_binarize, into LDS words of 16 rows.
__global__ __launch_bounds__(256) void k_ef_binarize_small(const float* __restrict__ C, int64_t mat_stride, int ld,
                                                           EfPairs E, double kappa, uint16_t* __restrict__ Wb,
                                                           int64_t wplane, int plane0) {
  __shared__ unsigned bits[4][64];
  __shared__ __attribute__((aligned(16))) unsigned s_hist[4][256 + 64];  // radix_kth, one per wave
  const int p = blockIdx.x, m = blockIdx.y;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  for (int e = threadIdx.x; e < 4 * 64; e += 256) bits[e >> 6][e & 63] = 0u;
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nn = min(kappa < 1.0 ? (int)rint(kappa * (double)N) : (int)kappa, N);  // as ef_binarize_row
  for (int row = w; row < M; row += 4) {
    const float* xr = C + m * mat_stride + (size_t)p * ld * ld + (size_t)row * ld;
    unsigned* brow = bits[row >> 4];
    const unsigned bit = 1u << (row & 15);
    if (kappa != 0.0 && nn <= kKnockMax) {
      if (nn > 0) ef_binarize_row_knock(xr, N, nn, lane, brow, bit);
    } else {
      ef_binarize_row<8>(xr, N, kappa, lane, brow, bit, s_hist[w]);
    }
  }
  __syncthreads();
  const int ng = (M + 15) / 16;
  uint16_t* o = Wb + ((size_t)p * 4 + plane0 + m) * wplane;
  for (int e = threadIdx.x; e < ng * 64; e += 256) {
    const int g = e >> 6, c = e & 63;
    if (c < N) o[(size_t)g * ld + c] = (uint16_t)bits[g][c];
  }
}

// Mean of the k smallest of each row (COLS = false) or column (K > kKmax); blockIdx.z = matrix;
// canonical order (kmean_canon, common.hpp), as k_ef_kmin.
template <bool COLS>
__global__ __launch_bounds__(256) void k_ef_kmean(const float* __restrict__ C, int64_t mat_stride, int ld, EfPairs E,
                                                  int k, float* __restrict__ out, int64_t omat_stride) {
  const int p = blockIdx.y, m = blockIdx.z;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  const int line = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int nl = COLS ? N : M, len = COLS ? M : N;
  if (line >= nl) return;
  const float* base = C + m * mat_stride + (size_t)p * ld * ld;
  auto at = [&](int e) { return COLS ? base[(size_t)e * ld + line] : base[(size_t)line * ld + e]; };
  const float mean = kmean_canon(at, len, k, lane);
  if (lane == 0) out[m * omat_stride + (size_t)p * ld + line] = mean;
}

// Mean of the k smallest of each row / column, one THREAD per line streaming it once: the k
// smallest so far stay sorted in registers (one compare rejects most elements, a bubble of
// min/max inserts the rest). Columns: lanes read consecutive columns (coalesced); rows: each
// lane walks its own row (cache lines reused along the walk). Sum in ascending order (the
// reference's np.mean over np.partition output has unspecified order; this ascending order is the
// canonical one the oracle and kmean_canon share).
template <bool COLS, int KMAX, int KC = 0>  // KC > 0: k fixed at compile time (k = KC = KMAX)
__global__ __launch_bounds__(256) void k_ef_kmin(const float* __restrict__ C, int64_t mat_stride, int ld, EfPairs E,
                                                 int k_rt, float* __restrict__ out, int64_t omat_stride, int ppb,
                                                 int n_pairs) {
  const int k = KC ? KC : k_rt;
  // ppb pairs per block (short tracks: 4 pairs x 64 lines per 256-thread block, ld <= 64)
  const int lpb = 256 / ppb;
  const int p = blockIdx.y * ppb + (int)threadIdx.x / lpb, m = blockIdx.z;
  if (p >= n_pairs) return;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  const int line = blockIdx.x * lpb + (int)threadIdx.x % lpb;
  const int nl = COLS ? N : M, len = COLS ? M : N;
  if (line >= nl) return;
  const float* base = C + m * mat_stride + (size_t)p * ld * ld + (COLS ? (size_t)line : (size_t)line * ld);
  const size_t step = COLS ? (size_t)ld : 1;
  float top[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) top[q] = INFINITY;
  for (int e = 0; e < len; ++e) {
    float v = base[e * step];
    float kth = top[0];
#pragma unroll
    for (int q = 1; q < KMAX; ++q) kth = (q == k - 1) ? top[q] : kth;
    if (v < kth) {
#pragma unroll
      for (int q = 0; q < KMAX; ++q) {
        if (q < k) {
          const float lo = fminf(top[q], v), hi = fmaxf(top[q], v);
          top[q] = lo;
          v = hi;
        }
      }
    }
  }
  float sum = 0.0f;
#pragma unroll
  for (int q = 0; q < KMAX; ++q)
    if (q < k) sum += top[q];
  out[m * omat_stride + (size_t)p * ld + line] = sum / (float)k;
}

// Row variant of k_ef_kmin: a wave takes 64 rows and stages 64 x 64 tiles through LDS with
// coalesced row-segment loads; lane r then walks row r of the tile (same insertion order as
// k_ef_kmin<false>: columns ascending).
template <int KMAX, int KC = 0>
__global__ __launch_bounds__(64) void k_ef_kmin_rows(const float* __restrict__ C, int64_t mat_stride, int ld,
                                                     EfPairs E, int k_rt, float* __restrict__ out,
                                                     int64_t omat_stride) {
  const int k = KC ? KC : k_rt;
#ifndef ACOSS_EF_KMIN_TW
#define ACOSS_EF_KMIN_TW 16
#endif
  // 16-column tiles: 4.3 KB of LDS per one-wave block, so LDS no longer caps the resident waves
  // (the 64-column tile, 16.6 KB, allowed 9 per CU: EarlyFusion 58.0k -> 61.8k pairs/s); each
  // load instruction takes 64 / TW rows x TW columns
  constexpr int TW = ACOSS_EF_KMIN_TW;
  __shared__ float t[64][TW + 1];
  const int p = blockIdx.y, m = blockIdx.z;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  const int row0 = blockIdx.x * 64;
  if (row0 >= M) return;
  const int lane = threadIdx.x;
  const float* base = C + m * mat_stride + (size_t)p * ld * ld;
  const int nr = min(64, M - row0);
  float top[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) top[q] = INFINITY;
  for (int c0 = 0; c0 < N; c0 += TW) {
    const int nc = min(TW, N - c0);
    __syncthreads();
    constexpr int RPI = 64 / TW;  // rows per load instruction
    const int lc = lane % TW, lr = lane / TW;
    for (int rr = lr; rr < nr; rr += RPI) t[rr][lc] = lc < nc ? base[(size_t)(row0 + rr) * ld + c0 + lc] : 0.0f;
    __syncthreads();
    for (int e = 0; e < nc; ++e) {
      float v = t[lane][e];
      float kth = top[0];
#pragma unroll
      for (int q = 1; q < KMAX; ++q) kth = (q == k - 1) ? top[q] : kth;
      if (v < kth) {
#pragma unroll
        for (int q = 0; q < KMAX; ++q) {
          if (q < k) {
            const float lo = fminf(top[q], v), hi = fmaxf(top[q], v);
            top[q] = lo;
            v = hi;
          }
        }
      }
    }
  }
  if (lane >= nr) return;
  float sum = 0.0f;
#pragma unroll
  for (int q = 0; q < KMAX; ++q)
    if (q < k) sum += top[q];
  out[m * omat_stride + (size_t)p * ld + row0 + lane] = sum / (float)k;
}

// E = exp(-(((0 + W_0) + W_1) + W_2)), W_s = getWCSM(C_s); written over C_0 (elementwise, in place).
__global__ void k_ef_wsum(float* __restrict__ C, int64_t mat_stride, int ld, EfPairs E, const float* __restrict__ rmean,
                          const float* __restrict__ cmean, int64_t mean_stride, float mu) {
  const int p = blockIdx.y;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;  // M N <= ld^2 < 2^31: 32-bit division
  if (e >= (unsigned)(M * N)) return;
  const int i = (int)(e / (unsigned)N), j = (int)(e - (unsigned)i * (unsigned)N);
  const size_t idx = (size_t)p * ld * ld + (size_t)i * ld + j;
  float wsum = 0.0f;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const float v = C[m * mat_stride + idx];
    const float eps = ((rmean[m * mean_stride + (size_t)p * ld + i] + cmean[m * mean_stride + (size_t)p * ld + j]) + v) / 3.0f;
    const float me = mu * eps;
    wsum = wsum + canon_expf(-(v * v) / (2.0f * (me * me)));
  }
  C[idx] = canon_expf(-wsum);
}

// SW metadata of the 4 matrices of each pair (matrix p*4 + s = bit plane s of pair p).
__global__ void k_ef_swmeta(EfPairs E, int P, int32_t* rows, int32_t* cols) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  int a, b, M, N;
  pair_dims(E, p, &a, &b, &M, &N);
  for (int s = 0; s < 4; ++s) {
    rows[p * 4 + s] = M;
    cols[p * 4 + s] = N;
  }
}

}  // namespace
}  // namespace acoss

using namespace acoss;

extern "C" int acoss_earlyfusion(const float* mfcc, const float* ssm, const float* chroma, const float* chroma_med,
                                 const int64_t* block_off, const int32_t* n_blocks, int32_t n_tracks,
                                 int32_t max_blocks, int32_t d_mfcc, int32_t d_ssm, int32_t d_chroma,
                                 const int32_t* pairs, int64_t n_pairs, double kappa, int32_t K, float mu,
                                 double* scores_out, void* hip_stream) {
  clear_error();
  if (n_tracks <= 0 || n_pairs < 0 || max_blocks <= 0 || d_mfcc <= 0 || d_ssm <= 0 || d_chroma <= 0 ||
      d_chroma % 12 != 0 || K <= 0 || K >= max_blocks + 1 || kappa < 0.0 ||
      (n_pairs > 0 && (!mfcc || !ssm || !chroma || !chroma_med || !block_off || !n_blocks || !pairs || !scores_out))) {
    set_error("acoss_earlyfusion: bad arguments");
    return ACOSS_E_ARG;
  }
  if (n_pairs == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  const int ld = (int)align_up((size_t)max_blocks, 4);
  if (ld > 16384) {  // k_ef_binarize keeps one u32 per column in LDS
    set_error("acoss_earlyfusion: more than 16384 blocks in a track");
    return ACOSS_E_ARG;
  }
  // per-track scratch: squared norms of the MFCC and SSM blocks, normalised chroma blocks; the
  // caller's block_off / n_blocks give the total row count through the last track
  int64_t h_off = 0;
  int32_t h_nb = 0;
  ACOSS_HIP_CHECK(hipMemcpy(&h_off, block_off + (n_tracks - 1), 8, hipMemcpyDeviceToHost));
  ACOSS_HIP_CHECK(hipMemcpy(&h_nb, n_blocks + (n_tracks - 1), 4, hipMemcpyDeviceToHost));
  const int64_t nrows = h_off + h_nb;
  const size_t tr_bytes = align_up((size_t)nrows * 4, 256) * 2 + align_up((size_t)nrows * d_chroma * 4, 256);
  char* tws = static_cast<char*>(workspace(10, tr_bytes));
  if (!tws) return ACOSS_E_HIP;
  float* sq_m = reinterpret_cast<float*>(tws);
  float* sq_s = reinterpret_cast<float*>(tws + align_up((size_t)nrows * 4, 256));
  float* chn = reinterpret_cast<float*>(tws + 2 * align_up((size_t)nrows * 4, 256));
  prof_begin(PH_CSM, s);
  const unsigned rb = (unsigned)((nrows + 3) / 4);
  hipLaunchKernelGGL(k_ef_rows, dim3(rb), dim3(256), 0, s, mfcc, nrows, d_mfcc, 0, nullptr, sq_m);
  ACOSS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_ef_rows, dim3(rb), dim3(256), 0, s, ssm, nrows, d_ssm, 0, nullptr, sq_s);
  ACOSS_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_ef_rows, dim3(rb), dim3(256), 0, s, chroma, nrows, d_chroma, 1, chn, nullptr);
  ACOSS_LAUNCH_CHECK();
  static const bool wave_tiles = getenv("ACOSS_EF_LDS_CSM") == nullptr;
  const float* ssm_p = nullptr;  // SSM bank with rows padded to a multiple of 4 (k_ef_csm_w)
  if (wave_tiles && d_ssm % 4 != 0) {
    const int ldp = (int)align_up((size_t)d_ssm, 4);
    float* pb = static_cast<float*>(workspace(15, (size_t)nrows * ldp * 4));
    if (!pb) return ACOSS_E_HIP;
    hipLaunchKernelGGL(k_ef_pad_rows, dim3(rb), dim3(256), 0, s, ssm, nrows, d_ssm, ldp, pb);
    ACOSS_LAUNCH_CHECK();
    ssm_p = pb;
  }
  prof_end(PH_CSM, s);

  // chunk of pairs: 3 CSMs (E overwrites the first), 4 binary matrices, 6 mean vectors, SW scratch
  const size_t mat = (size_t)ld * ld;
  const size_t sw_b = sw_bnd_bytes(ld, ld);
  const int64_t wplane = (int64_t)((ld + 15) / 16) * ld;  // u16 words of one bit plane
  const size_t per_pair = 3 * mat * 4 + 4 * (size_t)wplane * 2 + 6 * (size_t)ld * 4 + 4 * sw_b + 4 * (4 + 4) + 4;
  size_t budget = (size_t)4 << 30;
  if (const char* e = getenv("ACOSS_EF_BYTES")) budget = strtoull(e, nullptr, 10);
  // chunks alternate between two streams with a scratch set each, so one chunk's MFMA CSMs overlap
  // the previous chunk's VALU/latency-bound binarize, k-smallest means and SW (one stream while
  // phases are profiled, or with ACOSS_EF_STREAMS=1)
  const char* st_env = getenv("ACOSS_EF_STREAMS");
  const int nset = (profiling() || (st_env && st_env[0] == '1')) ? 1 : 2;
  int64_t chunk = (int64_t)(budget / nset / per_pair);
  if (chunk < 1) chunk = 1;
  if (chunk > 65535) chunk = 65535;
  // sub-batches start at multiples of the packing group (k_ef_csm_pack), so the caller's runs of
  // one query stay aligned with the groups
  if (chunk > kEfPack) chunk -= chunk % kEfPack;
  if (chunk > n_pairs) chunk = n_pairs;
  char* ws = static_cast<char*>(workspace(11, nset * (per_pair * chunk + 16 * 256)));
  if (!ws) return ACOSS_E_HIP;
  size_t o = 0;
  auto carve = [&](size_t bytes) {
    char* r = ws + o;
    o = align_up(o + bytes, 256);
    return r;
  };
  struct EfSet {
    float* C;
    uint16_t* Wb;
    float *rmean, *cmean;
    void* bnd;
    int32_t *m_rows, *m_cols;
    int* oti;
  } sets[2];
  for (int q = 0; q < nset; ++q) {
    sets[q].C = reinterpret_cast<float*>(carve(3 * mat * 4 * chunk));
    sets[q].Wb = reinterpret_cast<uint16_t*>(carve(4 * (size_t)wplane * 2 * chunk));
    sets[q].rmean = reinterpret_cast<float*>(carve(3 * (size_t)ld * 4 * chunk));
    sets[q].cmean = reinterpret_cast<float*>(carve(3 * (size_t)ld * 4 * chunk));
    sets[q].bnd = carve(4 * sw_b * chunk);
    sets[q].m_rows = reinterpret_cast<int32_t*>(carve(4 * 4 * chunk));
    sets[q].m_cols = reinterpret_cast<int32_t*>(carve(4 * 4 * chunk));
    sets[q].oti = reinterpret_cast<int*>(carve(4 * chunk));
  }
  hipStream_t ss[2] = {s, s};
  if (nset == 2) {
    ss[1] = side_stream(0);
    if (!ss[1]) {
      set_error("could not create the side stream");
      return ACOSS_E_HIP;
    }
    hipEvent_t e0 = sync_event(0);  // the side stream starts after the per-track prep above
    ACOSS_HIP_CHECK(hipEventRecord(e0, s));
    ACOSS_HIP_CHECK(hipStreamWaitEvent(ss[1], e0, 0));
  }
  const size_t bin_lds = (size_t)ld * 4;
  const int64_t mstride = (int64_t)mat * chunk;       // between the 3 CSM planes
  const int64_t meanstride = (int64_t)ld * chunk;     // between the 3 mean vectors
  const int tiles = (ld + kT - 1) / kT;  // LDS kernel tiles
  // wave-tile CSMs: 32 x 32 tiles when every track has at most 64 blocks (Da-TACOS beat blocks:
  // 14..47, a 64 x 64 tile there is mostly padding; profiles/r05/ef_short), 64 x 64 otherwise
  const int wtile = ld <= 64 ? 32 : 64;
  const int wtiles = (ld + wtile - 1) / wtile;
  auto kw_euclid = wtile == 32 ? k_ef_csm_w<0, 32> : k_ef_csm_w<0, 64>;
  // one binarize block per (pair, matrix) when every track has at most 64 blocks (15,000 Da-TACOS-
  // shape songs: 4.04M -> 4.38M pairs/s, profiles/r05/ef_short/efbin15k_*.log)
  const bool small_bin = ld <= 64;
  // ... and one wave per (pair, matrix) with a row per lane when every row's nn is small (the nn
  // rounds cost nn passes over the row's registers); ACOSS_EF_LANEBIN=0 keeps k_ef_binarize_small
  const int nn_max = kappa < 1.0 ? (int)rint(kappa * 64.0) : (int)kappa;
  static const bool lanebin_env = !(getenv("ACOSS_EF_LANEBIN") && getenv("ACOSS_EF_LANEBIN")[0] == '0');
  const bool lane_bin = small_bin && lanebin_env && nn_max <= 8;
  // column k-smallest means: 4 pairs per 256-thread block when every track has at most 64 blocks
  const int kmin_ppb = ld <= 64 ? 4 : 1;
  const unsigned kmin_gx = ld <= 64 ? 1u : (unsigned)((ld + 255) / 256);
  auto kw_cosine = wtile == 32 ? k_ef_csm_w<1, 32> : k_ef_csm_w<1, 64>;
  // short tracks: the cosine CSM with several consecutive pairs per wave sharing their query rows
  // (k_ef_csm_w4); ACOSS_EF_W4=0 keeps one pair per wave
  static const bool w4 = !(getenv("ACOSS_EF_W4") && getenv("ACOSS_EF_W4")[0] == '0');
  // ... and the euclid CSMs with the reference columns of a query's run packed (k_ef_csm_pack):
  // 32 x 64 tiles (pack_nb = 2) for every track up to 128 blocks; ACOSS_EF_PACK=1 takes 32 x 32
  // tiles, 0 a tile per pair (Da-TACOS shapes, profiles/r06/ef_pack/README.txt: 14..47 blocks
  // 4.85M -> 5.72M pairs/s, 30..80 blocks 1.12M -> 1.62M; 32 x 32 tiles 5.68M / 1.59M)
  static const char* pack_env = getenv("ACOSS_EF_PACK");
  const int pack_nb = ld > 128 || (pack_env && pack_env[0] == '0') ? 0 : pack_env && pack_env[0] == '1' ? 1 : 2;
  int ci = 0;
  for (int64_t p0 = 0; p0 < n_pairs; p0 += chunk, ++ci) {
    const int P = (int)((n_pairs - p0) < chunk ? (n_pairs - p0) : chunk);
    const EfPairs E{pairs + 2 * p0, block_off, n_blocks};
    hipStream_t st = ss[ci & 1];
    float* C = sets[ci & (nset - 1)].C;
    uint16_t* Wb = sets[ci & (nset - 1)].Wb;
    float* rmean = sets[ci & (nset - 1)].rmean;
    float* cmean = sets[ci & (nset - 1)].cmean;
    void* bnd = sets[ci & (nset - 1)].bnd;
    int32_t* m_rows = sets[ci & (nset - 1)].m_rows;
    int32_t* m_cols = sets[ci & (nset - 1)].m_cols;
    int* oti = sets[ci & (nset - 1)].oti;
    prof_begin(PH_CSM, st);
    hipLaunchKernelGGL(k_ef_oti, dim3((P + 255) / 256), dim3(256), 0, st, chroma_med, pairs + 2 * p0, P, oti);
    ACOSS_LAUNCH_CHECK();
    {
      const int n_tiles = tiles * tiles * P, n_wtiles = wtiles * wtiles * P;
      auto euclid = [&](const float* bank, int d, const float* sq, float* dst) -> int {
        if (wave_tiles && d % 4 != 0 && bank == ssm && ssm_p) {
          bank = ssm_p;  // the row-padded copy made above
          d = (int)align_up((size_t)d, 4);
        }
        if (wave_tiles && d % 4 == 0 && pack_nb) {
          const int tw = 32 * pack_nb;
          const int units = (P + kEfPack - 1) / kEfPack * ((ld + 31) / 32) * (kEfPack * ((ld + tw - 1) / tw));
          hipLaunchKernelGGL(pack_nb == 1 ? k_ef_csm_pack<1> : k_ef_csm_pack<2>, dim3((unsigned)((units + 3) / 4)),
                             dim3(256), 0, st, bank, d, sq, E, ld, P, units, dst);
        } else if (wave_tiles && d % 4 == 0)
          hipLaunchKernelGGL(kw_euclid, dim3((unsigned)((n_wtiles + 3) / 4)), dim3(256), 0, st, bank, d, sq, E, oti, ld,
                             n_wtiles, dst);
        else
          hipLaunchKernelGGL(k_ef_csm<0>, dim3((unsigned)n_tiles), dim3(256), 0, st, bank, d, sq, E, oti, ld, dst);
        ACOSS_LAUNCH_CHECK();
        return ACOSS_OK;
      };
      if (euclid(mfcc, d_mfcc, sq_m, C) != ACOSS_OK || euclid(ssm, d_ssm, sq_s, C + mstride) != ACOSS_OK)
        return ACOSS_E_HIP;
    }
    if (wave_tiles && d_chroma % 24 == 0 && w4 && wtile == 32) {
      const int units = (P + kEfPPc - 1) / kEfPPc * wtiles * wtiles;
      hipLaunchKernelGGL((k_ef_csm_w4<1, kEfPPc>), dim3((unsigned)((units + 3) / 4)), dim3(256), 0, st, chn, d_chroma,
                         nullptr, E, oti, ld, P, units, C + 2 * mstride);
    } else if (wave_tiles && d_chroma % 24 == 0)
      hipLaunchKernelGGL(kw_cosine, dim3((unsigned)((wtiles * wtiles * P + 3) / 4)), dim3(256), 0, st, chn, d_chroma, nullptr, E,
                         oti, ld, wtiles * wtiles * P, C + 2 * mstride);
    else
      hipLaunchKernelGGL(k_ef_csm<1>, dim3((unsigned)(tiles * tiles * P)), dim3(256), 0, st, chn, d_chroma, nullptr, E,
                         oti, ld, C + 2 * mstride);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_CSM, st);
    prof_begin(PH_BIN, st);
    if (lane_bin)
      hipLaunchKernelGGL(k_ef_binarize_lanes, dim3((unsigned)((3 * P + 3) / 4)), dim3(256), 0, st, C, mstride, ld, E,
                         kappa, Wb, wplane, 0, 3, 3 * P);
    else if (small_bin)
      hipLaunchKernelGGL(k_ef_binarize_small, dim3(P, 3), dim3(256), 0, st, C, mstride, ld, E, kappa, Wb, wplane, 0);
    else
      hipLaunchKernelGGL(k_ef_binarize, dim3((ld + 15) / 16, P, 3), dim3(1024), bin_lds, st, C, mstride, ld, E, kappa,
                         Wb, wplane, 0);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_BIN, st);
    prof_begin(PH_WCSM, st);
    if (K == 10) {  // EarlyFusion's K: the k-th smallest is a fixed register, no per-element select
      hipLaunchKernelGGL((k_ef_kmin_rows<10, 10>), dim3((ld + 63) / 64, P, 3), dim3(64), 0, st, C, mstride, ld, E,
                         (int)K, rmean, meanstride);
      ACOSS_LAUNCH_CHECK();
      hipLaunchKernelGGL((k_ef_kmin<true, 10, 10>), dim3(kmin_gx, (P + kmin_ppb - 1) / kmin_ppb, 3), dim3(256), 0, st,
                         C, mstride, ld, E, (int)K, cmean, meanstride, kmin_ppb, P);
      ACOSS_LAUNCH_CHECK();
    } else if (K <= kKmax) {
      hipLaunchKernelGGL((k_ef_kmin_rows<kKmax>), dim3((ld + 63) / 64, P, 3), dim3(64), 0, st, C, mstride, ld, E,
                         (int)K, rmean, meanstride);
      ACOSS_LAUNCH_CHECK();
      hipLaunchKernelGGL((k_ef_kmin<true, kKmax>), dim3(kmin_gx, (P + kmin_ppb - 1) / kmin_ppb, 3), dim3(256), 0, st,
                         C, mstride, ld, E, (int)K, cmean, meanstride, kmin_ppb, P);
      ACOSS_LAUNCH_CHECK();
    } else {
      hipLaunchKernelGGL(k_ef_kmean<false>, dim3((ld + 3) / 4, P, 3), dim3(256), 0, st, C, mstride, ld, E, (int)K,
                         rmean, meanstride);
      ACOSS_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_ef_kmean<true>, dim3((ld + 3) / 4, P, 3), dim3(256), 0, st, C, mstride, ld, E, (int)K,
                         cmean, meanstride);
      ACOSS_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_ef_wsum, dim3((unsigned)((mat + 255) / 256), P), dim3(256), 0, st, C, mstride, ld, E, rmean,
                       cmean, meanstride, mu);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_WCSM, st);
    prof_begin(PH_BIN, st);
    if (lane_bin)
      hipLaunchKernelGGL(k_ef_binarize_lanes, dim3((unsigned)((P + 3) / 4)), dim3(256), 0, st, C, mstride, ld, E, kappa,
                         Wb, wplane, 3, 1, P);
    else if (small_bin)
      hipLaunchKernelGGL(k_ef_binarize_small, dim3(P, 1), dim3(256), 0, st, C, mstride, ld, E, kappa, Wb, wplane, 3);
    else
      hipLaunchKernelGGL(k_ef_binarize, dim3((ld + 15) / 16, P, 1), dim3(1024), bin_lds, st, C, mstride, ld, E, kappa,
                         Wb, wplane, 3);
    ACOSS_LAUNCH_CHECK();
    prof_end(PH_BIN, st);
    prof_begin(PH_SW, st);
    hipLaunchKernelGGL(k_ef_swmeta, dim3((P + 255) / 256), dim3(256), 0, st, E, P, m_rows, m_cols);
    ACOSS_LAUNCH_CHECK();
    int rc = launch_swb_batch(Wb, wplane, ld, m_rows, m_cols, 4 * P, ld, ld, bnd, scores_out + 4 * p0, st);
    if (rc) return rc;
    prof_end(PH_SW, st);
  }
  if (nset == 2) {  // the caller's stream waits for the side stream's chunks
    hipEvent_t e1 = sync_event(1);
    ACOSS_HIP_CHECK(hipEventRecord(e1, ss[1]));
    ACOSS_HIP_CHECK(hipStreamWaitEvent(s, e1, 0));
  }
  return ACOSS_OK;
}
