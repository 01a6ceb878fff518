// pending.cpp — C-ABI entry points whose kernels are not built yet (fail loudly).
#include "common.hpp"

#define PENDING(name)                                                       \
  do {                                                                      \
    acoss::set_error("%s: not implemented in this build", name);            \
    return ACOSS_E_ARG;                                                     \
  } while (0)

extern "C" {
int acoss_sw_constrained(const uint8_t*, const int64_t*, const int32_t*, const int32_t*, int32_t, int32_t, int32_t,
                         double*, void*) { PENDING("acoss_sw_constrained"); }
int acoss_csm(const float*, int32_t, const float*, int32_t, int32_t, int32_t, int32_t, float*, void*) {
  PENDING("acoss_csm");
}
int acoss_get_oti(const float*, const float*, int32_t, int32_t*, void*) { PENDING("acoss_get_oti"); }
int acoss_binarize_rows(const float*, int32_t, int32_t, int32_t, uint8_t*, void*) { PENDING("acoss_binarize_rows"); }
int acoss_wcsm(const float*, int32_t, int32_t, int32_t, int32_t, float, float*, void*) { PENDING("acoss_wcsm"); }
int acoss_simple_mp(const double*, const int64_t*, const int32_t*, int32_t, int32_t, const int32_t*, int64_t, int32_t,
                    double*, int32_t*, void*) { PENDING("acoss_simple_mp"); }
}
