// bf16x3 jet kernel instantiations for 128-feature-padded hidden layers (WT = 8).
// Generated case list: every (S, NSO) with S <= 4, NSO <= S - 2 (or S = 1).
#include "jet_bf3.h"

#ifdef TDQ_PHASE_TIMING
extern "C" int tdq_set_timing_buffer(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(tdq_ts), &p, sizeof(p));
}
#endif

int bf3_fwd_w8(int S, int nso, const Bf3Args& a) {
  switch (S * 16 + nso) {
    case 16: return launch_fwd_bf3<8, 1, 0>(a);
    case 32: return launch_fwd_bf3<8, 2, 0>(a);
    case 48: return launch_fwd_bf3<8, 3, 0>(a);
    case 49: return launch_fwd_bf3<8, 3, 1>(a);
    case 64: return launch_fwd_bf3<8, 4, 0>(a);
    case 65: return launch_fwd_bf3<8, 4, 1>(a);
    case 66: return launch_fwd_bf3<8, 4, 2>(a);
    default: return (int)hipErrorInvalidValue;
  }
}

int bf3_bwd_w8(int S, int nso, const Bf3Args& a) {
  switch (S * 16 + nso) {
    case 16: return launch_bwd_bf3<8, 1, 0>(a);
    case 32: return launch_bwd_bf3<8, 2, 0>(a);
    case 48: return launch_bwd_bf3<8, 3, 0>(a);
    case 49: return launch_bwd_bf3<8, 3, 1>(a);
    case 64: return launch_bwd_bf3<8, 4, 0>(a);
    case 65: return launch_bwd_bf3<8, 4, 1>(a);
    case 66: return launch_bwd_bf3<8, 4, 2>(a);
    default: return (int)hipErrorInvalidValue;
  }
}
