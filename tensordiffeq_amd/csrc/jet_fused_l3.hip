// Instantiations of the persistent point-tile jet kernels (jet_fused.h) for LM = 3 MFMA hidden
// layers at 128-feature padded width (WT = 8), every (S, NSO) with S <= 4, both modes.
#include "jet_fused.h"

#ifdef TDQ_PHASE_TIMING
extern "C" int tdq_fz_set_timing_buffer(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(tdq_ts), &p, sizeof(p));
}
#endif

int fz_dispatch_w8_l3(int mode, int S, int nso, const FzArgs& a) {
  switch ((S * 16 + nso) * 2 + mode) {
#define FZ_CASE(S_, N_) \
  case (S_ * 16 + N_) * 2 + 0: return launch_fused<8, S_, N_, 3, 0>(a); \
  case (S_ * 16 + N_) * 2 + 1: return launch_fused<8, S_, N_, 3, 1>(a);
    FZ_CASE(1, 0)
    FZ_CASE(2, 0)
    FZ_CASE(3, 0)
    FZ_CASE(3, 1)
    FZ_CASE(4, 0)
    FZ_CASE(4, 1)
#undef FZ_CASE
    default: return (int)hipErrorInvalidValue;
  }
}
