// features.hip — per-track feature preparation on the device.
//
//   A13 median downsample (Serra09.load_features / ChenFusion.load_features,
//       acoss/algorithms/rqa_serra09.py:44-53, latefusion_chen.py:46-56):
//       librosa.util.sync(chroma.T, arange(0, n, f), aggregate=np.median) -> segments
//       [0, f), [f, 2f), ..., [kf, n); per bin the median (mean of the two middle values,
//       computed in float32 like np.median on float32, for even counts).
//   A12 SiMPle features (Simple.load_features + smooth, simple_silva.py:34-43,56-66):
//       window means over [i*skip, i*skip + win) (float32 accumulation and division, as np.mean
//       on the float32 chroma), then a zero-filled 'same' convolution along time with the
//       normalised symmetric Hann window (host-supplied weights), then per-column L2
//       normalisation (librosa.util.normalize: columns with norm < tiny are left as is).
#include "common.hpp"

namespace acoss {

namespace {

constexpr int kMaxFac = 64;
constexpr int kMaxSmooth = 16;

struct SmoothWin {
  double w[kMaxSmooth];
  int len;
};

// thread per (segment, bin): insertion sort of <= 64 values in registers/scratch
__global__ void k_median_downsample(const float* __restrict__ feats, const int64_t* __restrict__ off,
                                    const int32_t* __restrict__ len, int n_tracks, int fac, float* __restrict__ out,
                                    const int64_t* __restrict__ out_off) {
  const int tr = blockIdx.y;
  if (tr >= n_tracks) return;
  const int n = len[tr];
  const int nseg = (n + fac - 1) / fac;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nseg * 12) return;
  const int seg = e / 12, c = e - seg * 12;
  const float* X = feats + off[tr] * 12;
  const int a = seg * fac, b = min(n, a + fac), cnt = b - a;
  float v[kMaxFac];
  for (int t = 0; t < cnt; ++t) {
    const float x = X[(size_t)(a + t) * 12 + c];
    int k = t;
    while (k > 0 && v[k - 1] > x) {
      v[k] = v[k - 1];
      --k;
    }
    v[k] = x;
  }
  float med;
  if (cnt & 1)
    med = v[cnt / 2];
  else
    med = (v[cnt / 2 - 1] + v[cnt / 2]) / 2.0f;
  out[(out_off[tr] + seg) * 12 + c] = med;
}

// block per track: window means -> LDS-free two passes through global scratch (out itself)
__global__ void k_simple_features(const float* __restrict__ feats, const int64_t* __restrict__ off,
                                  const int32_t* __restrict__ len, int n_tracks, int win, int skip, SmoothWin sw,
                                  double* __restrict__ means, double* __restrict__ out,
                                  const int64_t* __restrict__ out_off) {
  const int tr = blockIdx.x;
  if (tr >= n_tracks) return;
  const int n = len[tr];
  const int T = n / skip;
  if (T <= 0) return;
  const float* X = feats + off[tr] * 12;
  double* Mn = means + out_off[tr];
  double* O = out + out_off[tr];
  // pass 1: means[c][i] (dim-major 12 x T)
  for (int e = threadIdx.x; e < 12 * T; e += blockDim.x) {
    const int c = e / T, i = e - c * T;
    const int a = i * skip, b = min(n, a + win);
    float acc = 0.0f;
    for (int t = a; t < b; ++t) acc = acc + X[(size_t)t * 12 + c];
    Mn[e] = (double)(acc / (float)(b - a));
  }
  __syncthreads();
  // pass 2: 'same' convolution along time, offset (len - 1) / 2, zero fill
  const int s0 = (sw.len - 1) / 2;
  for (int e = threadIdx.x; e < 12 * T; e += blockDim.x) {
    const int c = e / T, i = e - c * T;
    double acc = 0.0;
    for (int k = 0; k < sw.len; ++k) {
      const int src = i + s0 - k;
      if (src >= 0 && src < T) acc = acc + Mn[c * T + src] * sw.w[k];
    }
    O[e] = acc;
  }
  __syncthreads();
  // pass 3: L2-normalise every column
  for (int i = threadIdx.x; i < T; i += blockDim.x) {
    double s = 0.0;
    for (int c = 0; c < 12; ++c) s = s + O[c * T + i] * O[c * T + i];
    double nrm = sqrt(s);
    if (nrm < 2.2250738585072014e-308) nrm = 1.0;
    for (int c = 0; c < 12; ++c) O[c * T + i] = O[c * T + i] / nrm;
  }
}

}  // namespace
}  // namespace acoss

using namespace acoss;

extern "C" int acoss_median_downsample(const float* feats, const int64_t* track_off, const int32_t* track_len,
                                       int32_t n_tracks, int32_t max_len, int32_t factor, float* out,
                                       const int64_t* out_off, void* hip_stream) {
  clear_error();
  if (n_tracks < 0 || factor < 1 || factor > kMaxFac ||
      (n_tracks > 0 && (!feats || !track_off || !track_len || !out || !out_off))) {
    set_error("acoss_median_downsample: bad arguments (factor must be in [1, %d])", kMaxFac);
    return ACOSS_E_ARG;
  }
  if (n_tracks == 0 || max_len <= 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  const int nseg = (max_len + factor - 1) / factor;
  hipLaunchKernelGGL(k_median_downsample, dim3((nseg * 12 + 255) / 256, n_tracks), dim3(256), 0, s, feats, track_off,
                     track_len, n_tracks, factor, out, out_off);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}

extern "C" int acoss_simple_features(const float* feats, const int64_t* track_off, const int32_t* track_len,
                                     int32_t n_tracks, int32_t win, int32_t skip, const double* smooth,
                                     int32_t smooth_len, double* out, const int64_t* out_off, int64_t out_elems,
                                     void* hip_stream) {
  clear_error();
  if (n_tracks < 0 || win < 1 || skip < 1 || smooth_len < 1 || smooth_len > kMaxSmooth || !smooth || out_elems < 0 ||
      (n_tracks > 0 && (!feats || !track_off || !track_len || !out || !out_off))) {
    set_error("acoss_simple_features: bad arguments");
    return ACOSS_E_ARG;
  }
  if (n_tracks == 0 || out_elems == 0) return ACOSS_OK;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  SmoothWin sw{};
  sw.len = smooth_len;
  for (int k = 0; k < smooth_len; ++k) sw.w[k] = smooth[k];  // host array
  double* means = static_cast<double*>(workspace(9, (size_t)out_elems * 8));
  if (!means) return ACOSS_E_HIP;
  hipLaunchKernelGGL(k_simple_features, dim3(n_tracks), dim3(256), 0, s, feats, track_off, track_len, n_tracks, win,
                     skip, sw, means, out, out_off);
  ACOSS_LAUNCH_CHECK();
  return ACOSS_OK;
}
