// crp_internal.hpp — types shared by the Serra09/Chen kernels (crp.hip, crp_select.hip).
#pragma once
#include "common.hpp"

namespace acoss {

// One batch of pairs of the Serra09/Chen path, all device pointers.
struct CrpBatch {
  const float* feats;    // packed (sum n, 12) chroma
  const float* feats2;   // per track (ldn frames): frames f, f+1 interleaved (24 floats); split path only
  const int64_t* off;    // track row offsets
  const int32_t* len;    // track frame counts
  const float* NX;       // stacked squared norms, track t at NX[t*ldn]
  int ldn;
  const int32_t* pairs;  // (P, 2) query, reference (already offset to the batch)
  const int32_t* oti;    // per pair OTI shift of the reference
  const int2* dims;      // per pair (M', N')
  int m, tau;
  const float* yrot;     // per pair: reference frames rolled by the pair's OTI (max_len x 12)
  int64_t yrot_stride;   // floats between consecutive pairs in yrot
};

// Constant-address-space view of read-only global data: wave-uniform loads through it
// become scalar (s_load) loads whose values live in SGPRs.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const f32x4 cfloat4;

// Fast threshold kernels (crp_select.hip). Returns ACOSS_OK, an error code, or 1 when the
// shape is not covered by the fast path (caller falls back to k_crp_select).
// Fast CRP mask kernel (crp_mask.hip); 1 = not covered (caller falls back to k_crp_panel<0>).
int launch_mask9(const CrpBatch& B, int nb, int L, const float* Trow, const float* Tcol, int64_t thr_stride,
                 uint32_t* maskT, int64_t mask_stride, int ld, hipStream_t s);

// Two-kernel CRP around one sweep (crp_split.hip); 1 = not covered.
// kplanes: 2 planes of nb*kstride uint16 (16-bit key prefixes, row-major and strip-major).
int launch_crp_split(const CrpBatch& B, int nb, int L, float kappa, void* kplanes, int ldk,
                     int64_t kstride,
                     uint32_t* RT, float* thr_r, float* T_r, float* thr_c, float* T_c, int64_t thr_stride,
                     uint32_t* maskT, int64_t mask_stride, int ld, hipStream_t s);

int launch_select16(bool trans, const CrpBatch& B, int nb, int L, float kappa, float* thr, float* T,
                    int64_t thr_stride, hipStream_t s);

}  // namespace acoss
