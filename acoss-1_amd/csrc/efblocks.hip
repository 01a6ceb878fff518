// EarlyFusion beat-synchronous block features on the device.
//
// Replaces EarlyFusion.load_features' per-track loops (acoss/algorithms/earlyfusion_traile.py:67-154)
// and its resize_block (:214-247), which the reference runs in Python with
// skimage.transform.resize(x, (frames_per_block, d), anti_aliasing=True, mode='constant') per beat
// block (about 0.6 s per 20,000-frame track on one core; Da-TACOS has 15,000 tracks). skimage's
// published algorithm, restated in float64 as the reference computes it:
//   factor = n_in / R; sigma = max(0, (factor - 1) / 2); Gaussian pre-filter along frames
//   (scipy gaussian_filter: radius int(4 sigma + 0.5), weights exp(-x^2 / (2 sigma^2)) / sum,
//   zero padding), then linear interpolation at input coordinate (k + 0.5) factor - 0.5 with zeros
//   outside the block (ndimage.zoom, grid_mode=True, mode 'grid-constant').
// Per block b of a track (onsets o[]):
//   mfccs[b]   = z-normalised resize of mfcc[o[b] : o[b + blocksize - 1]] to R = mfccs_per_block rows
//                (column means removed, each row divided by its L2 norm, zero norms -> 1), flattened
//   ssms[b]    = get_ssm(that block)[I < J] (cross_recurrence.py:10-28): for a = 0..R-1, b' < a,
//                sqrt(max(0, (|x_a|^2 + |x_b'|^2) - 2 x_a.x_b')), row-major over (a, b')
//   chromas[b] = resize of chroma[o[b] : o[b + blocksize]] to chromas_per_block rows, flattened
// and chroma_med = np.median(chroma, axis=0) per track (k_track_median: the two middle order
// statistics by a bitwise search on order-preserving keys, their float32 mean for even n).
// One 256-thread block per beat block; everything in float64 in LDS, stored as float32.
#include "common.hpp"

namespace acoss {
namespace {

constexpr int kEfMaxR = 64;    // rows per block feature (reference: 50 and 40)
constexpr int kEfMaxD = 32;    // MFCC coefficients (reference: 20)
constexpr int kEfMaxRad = 512; // Gaussian taps kept in LDS (sigma < 128: blocks of < 12,800 frames at R = 50)

// Gaussian tap t (|t| <= rad) of a radius above kEfMaxRad, formed on the fly exactly as the LDS
// table would hold it: exp(-x^2 / (2 sigma^2)) divided by the sequential sum of all taps.
__device__ __forceinline__ double ef_tap(int t, double s2, double wsum) {
  const double x = (double)t;
  return exp(-0.5 / s2 * (x * x)) / wsum;
}

// filtered value of column c at frame i of the block (zero outside [0, n_in)); taps from the LDS
// table w when rad <= kEfMaxRad, else on the fly (s2 = sigma^2, wsum = the taps' sum)
__device__ __forceinline__ double ef_filtered(const float* X, int64_t ld, int n_in, int c, int i, const double* w,
                                              int rad, double s2, double wsum) {
  if (i < 0 || i >= n_in) return 0.0;
  if (rad == 0) return (double)X[(int64_t)i * ld + c];
  double acc = 0.0;
  const int t0 = max(-rad, -i), t1 = min(rad, n_in - 1 - i);
  if (rad <= kEfMaxRad) {
    for (int t = t0; t <= t1; ++t) acc = fma(w[t + rad], (double)X[(int64_t)(i + t) * ld + c], acc);
  } else {
    for (int t = t0; t <= t1; ++t) acc = fma(ef_tap(t, s2, wsum), (double)X[(int64_t)(i + t) * ld + c], acc);
  }
  return acc;
}

// skimage-style resize of X (n_in x D rows, row stride ld) to R x D into out (LDS, stride D)
__device__ void ef_resize(const float* X, int64_t ld, int n_in, int R, int D, double* out, double* w, int* s_rad) {
  const double factor = (double)n_in / (double)R;
  const double sigma = fmax(0.0, (factor - 1.0) / 2.0);
  if (threadIdx.x == 0) *s_rad = sigma > 0.0 ? (int)(4.0 * sigma + 0.5) : 0;
  __syncthreads();
  const int rad = *s_rad;
  const double s2 = sigma * sigma;
  double wsum = 0.0;
  if (rad > kEfMaxRad) {  // very long beat blocks: the taps' sum here, the taps in ef_filtered
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int t = -rad; t <= rad; ++t) s += exp(-0.5 / s2 * ((double)t * (double)t));
      w[0] = s;
    }
    __syncthreads();
    wsum = w[0];
  } else if (rad > 0) {
    for (int t = threadIdx.x; t <= 2 * rad; t += blockDim.x) {
      const double x = (double)(t - rad);
      w[t] = exp(-0.5 / s2 * (x * x));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int t = 0; t <= 2 * rad; ++t) s += w[t];
      w[2 * rad + 1] = s;
    }
    __syncthreads();
    const double s = w[2 * rad + 1];
    for (int t = threadIdx.x; t <= 2 * rad; t += blockDim.x) w[t] = w[t] / s;
    __syncthreads();
  }
  for (int e = threadIdx.x; e < R * D; e += blockDim.x) {
    const int k = e / D, c = e - k * D;
    const double cc = ((double)k + 0.5) * factor - 0.5;
    const double fl = floor(cc);
    const int i0 = (int)fl;
    const double f = cc - fl;
    const double v0 = ef_filtered(X, ld, n_in, c, i0, w, rad, s2, wsum);
    const double v1 = ef_filtered(X, ld, n_in, c, i0 + 1, w, rad, s2, wsum);
    double v = (1.0 - f) * v0 + f * v1;
    if (!(v == v) || v == INFINITY || v == -INFINITY) v = 0.0;  // ret[isinf|isnan] = 0 (:244-245)
    out[e] = v;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_ef_blocks(const float* __restrict__ mfcc, const float* __restrict__ chroma,
                                                   const int64_t* __restrict__ frame_off,
                                                   const int32_t* __restrict__ n_frames,
                                                   const int64_t* __restrict__ mfcc_off,
                                                   const int32_t* __restrict__ mfcc_frames,
                                                   const int64_t* __restrict__ onsets,
                                                   const int64_t* __restrict__ onset_off,
                                                   const int64_t* __restrict__ block_off, int n_tracks, int bs,
                                                   int Rm, int Rc, int Dm, float* __restrict__ out_mfcc,
                                                   float* __restrict__ out_ssm, float* __restrict__ out_chroma) {
  __shared__ double xs[kEfMaxR * kEfMaxD];
  __shared__ double w[2 * kEfMaxRad + 2];
  __shared__ double sq[kEfMaxR];
  __shared__ double red[kEfMaxD];
  __shared__ int s_rad;
  const int64_t gb = blockIdx.x;
  // track of this global block: last t with block_off[t] <= gb
  int lo = 0, hi = n_tracks - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (block_off[mid] <= gb) lo = mid;
    else hi = mid - 1;
  }
  const int tr = lo;
  const int b = (int)(gb - block_off[tr]);
  const int64_t* on = onsets + onset_off[tr];
  const int64_t f0 = frame_off[tr], m0 = mfcc_off[tr];
  // ---- MFCC block: resize, z-normalise. The span is mfcc[o[b] : o[b + bs - 1]] clamped to the
  // MFCC's own frame count, as Python slicing clamps (the extractor's mfcc_htk has fewer frames
  // than the chroma, features.py:884); the host checked that every clamped span is non-empty.
  {
    const int nm = mfcc_frames[tr];
    const int i1 = (int)on[b], i2 = min((int)on[b + bs - 1], nm);
    ef_resize(mfcc + (m0 + i1) * Dm, Dm, i2 - i1, Rm, Dm, xs, w, &s_rad);
    if (threadIdx.x < Dm) {  // column means (sequential over the rows)
      double s = 0.0;
      for (int k = 0; k < Rm; ++k) s += xs[k * Dm + threadIdx.x];
      red[threadIdx.x] = s / (double)Rm;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < Rm * Dm; e += blockDim.x) xs[e] -= red[e % Dm];
    __syncthreads();
    if (threadIdx.x < Rm) {
      double s = 0.0;
      for (int c = 0; c < Dm; ++c) s += xs[threadIdx.x * Dm + c] * xs[threadIdx.x * Dm + c];
      const double nrm = sqrt(s);
      sq[threadIdx.x] = nrm == 0.0 ? 1.0 : nrm;
    }
    __syncthreads();
    float* om = out_mfcc + gb * (int64_t)(Rm * Dm);
    for (int e = threadIdx.x; e < Rm * Dm; e += blockDim.x) {
      const double v = xs[e] / sq[e / Dm];
      xs[e] = v;
      om[e] = (float)v;
    }
    __syncthreads();
    if (threadIdx.x < Rm) {
      double s = 0.0;
      for (int c = 0; c < Dm; ++c) s += xs[threadIdx.x * Dm + c] * xs[threadIdx.x * Dm + c];
      sq[threadIdx.x] = s;
    }
    __syncthreads();
    const int npair = Rm * (Rm - 1) / 2;
    float* os = out_ssm + gb * (int64_t)npair;
    for (int e = threadIdx.x; e < npair; e += blockDim.x) {
      // e -> (a, b') with b' < a, row-major over a: e = a (a - 1) / 2 + b'
      int a = (int)((1.0 + sqrt(1.0 + 8.0 * (double)e)) * 0.5);
      while (a * (a - 1) / 2 > e) --a;
      while ((a + 1) * a / 2 <= e) ++a;
      const int bb = e - a * (a - 1) / 2;
      double dot = 0.0;
      for (int c = 0; c < Dm; ++c) dot += xs[a * Dm + c] * xs[bb * Dm + c];
      double d2 = (sq[a] + sq[bb]) - 2.0 * dot;
      if (d2 < 0.0) d2 = 0.0;
      os[e] = (float)sqrt(d2);
    }
    __syncthreads();
  }
  // ---- chroma block: resize (span clamped to the chroma's frame count, likewise)
  {
    const int i1 = (int)on[b], i2 = min((int)on[b + bs], (int)n_frames[tr]);
    ef_resize(chroma + (f0 + i1) * 12, 12, i2 - i1, Rc, 12, xs, w, &s_rad);
    float* oc = out_chroma + gb * (int64_t)(Rc * 12);
    for (int e = threadIdx.x; e < Rc * 12; e += blockDim.x) oc[e] = (float)xs[e];
  }
}

__device__ __forceinline__ unsigned f2key(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  return (u >> 31) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
  const unsigned u = (k >> 31) ? (k & 0x7fffffffu) : ~k;
  return __builtin_bit_cast(float, u);
}

// k-th smallest (0-based) of column c of a track's (n x 12) chroma: the least key K with
// #(keys <= K) > k, bit by bit from the top (32 block-wide counts).
__device__ float ef_kth(const float* X, int n, int c, int k, int* cnt) {
  unsigned res = 0;
  for (int bit = 31; bit >= 0; --bit) {
    const unsigned cand = res | ((1u << bit) - 1u);  // every key with the bits fixed so far and 0 here
    int my = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) my += f2key(X[(int64_t)i * 12 + c]) <= cand;
    my = wave_sum(my);
    if ((threadIdx.x & 63) == 0) atomicAdd(cnt, my);
    __syncthreads();
    const int total = *cnt;
    __syncthreads();
    if (threadIdx.x == 0) *cnt = 0;
    __syncthreads();
    if (total <= k) res |= 1u << bit;  // the k-th key has this bit set
  }
  return key2f(res);
}

__global__ __launch_bounds__(256) void k_track_median(const float* __restrict__ chroma,
                                                      const int64_t* __restrict__ frame_off,
                                                      const int32_t* __restrict__ n_frames, float* __restrict__ med) {
  __shared__ int cnt;
  const int tr = blockIdx.x, c = blockIdx.y;
  const int n = n_frames[tr];
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  const float* X = chroma + frame_off[tr] * 12;
  float m;
  if (n % 2) {
    m = ef_kth(X, n, c, n / 2, &cnt);
  } else {
    const float a = ef_kth(X, n, c, n / 2 - 1, &cnt);
    const float b = ef_kth(X, n, c, n / 2, &cnt);
    m = (a + b) / 2.0f;  // np.mean of the two middle float32 values
  }
  if (threadIdx.x == 0) med[tr * 12 + c] = m;
}

}  // namespace
}  // namespace acoss

using namespace acoss;

extern "C" int acoss_ef_block_features(const float* mfcc, const float* chroma, const int64_t* frame_off,
                                       const int32_t* n_frames, const int64_t* mfcc_off,
                                       const int32_t* mfcc_frames, const int64_t* onsets, const int64_t* onset_off,
                                       const int64_t* block_off, int32_t n_tracks, int64_t total_blocks,
                                       int32_t blocksize, int32_t mfccs_per_block, int32_t chromas_per_block,
                                       int32_t d_mfcc, float* out_mfcc, float* out_ssm, float* out_chroma,
                                       float* out_med, void* hip_stream) {
  clear_error();
  if (n_tracks < 0 || total_blocks < 0 || blocksize < 1 || mfccs_per_block < 2 || mfccs_per_block > kEfMaxR ||
      chromas_per_block < 1 || chromas_per_block > kEfMaxR || d_mfcc < 1 || d_mfcc > kEfMaxD) {
    set_error("acoss_ef_block_features: bad sizes (rows per block 2..%d, d_mfcc 1..%d)", kEfMaxR, kEfMaxD);
    return ACOSS_E_ARG;
  }
  if (n_tracks == 0) return ACOSS_OK;
  if (!chroma || !frame_off || !n_frames || !out_med || (total_blocks > 0 && (!mfcc || !mfcc_off || !mfcc_frames || !onsets || !onset_off ||
      !block_off || !out_mfcc || !out_ssm || !out_chroma))) {
    set_error("acoss_ef_block_features: NULL pointer");
    return ACOSS_E_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  if (total_blocks > 0) {
    hipLaunchKernelGGL(k_ef_blocks, dim3((unsigned)total_blocks), dim3(256), 0, s, mfcc, chroma, frame_off, n_frames,
                       mfcc_off, mfcc_frames, onsets, onset_off, block_off, n_tracks, blocksize, mfccs_per_block, chromas_per_block, d_mfcc,
                       out_mfcc, out_ssm, out_chroma);
    ACOSS_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_track_median, dim3(n_tracks, 12), dim3(256), 0, s, chroma, frame_off, n_frames, out_med);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}
