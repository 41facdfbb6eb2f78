// bf16x3 jet kernel instantiations for 32-feature-padded hidden layers (WT = 2).
// Generated case list: every (S, NSO) with S <= 8, NSO <= S - 2 (or S = 1).
#include "jet_bf3.h"

int bf3_fwd_w2(int S, int nso, const Bf3Args& a) {
  switch (S * 16 + nso) {
    case 16: return launch_fwd_bf3<2, 1, 0>(a);
    case 32: return launch_fwd_bf3<2, 2, 0>(a);
    case 48: return launch_fwd_bf3<2, 3, 0>(a);
    case 49: return launch_fwd_bf3<2, 3, 1>(a);
    case 64: return launch_fwd_bf3<2, 4, 0>(a);
    case 65: return launch_fwd_bf3<2, 4, 1>(a);
    case 66: return launch_fwd_bf3<2, 4, 2>(a);
    case 80: return launch_fwd_bf3<2, 5, 0>(a);
    case 81: return launch_fwd_bf3<2, 5, 1>(a);
    case 82: return launch_fwd_bf3<2, 5, 2>(a);
    case 83: return launch_fwd_bf3<2, 5, 3>(a);
    case 96: return launch_fwd_bf3<2, 6, 0>(a);
    case 97: return launch_fwd_bf3<2, 6, 1>(a);
    case 98: return launch_fwd_bf3<2, 6, 2>(a);
    case 99: return launch_fwd_bf3<2, 6, 3>(a);
    case 100: return launch_fwd_bf3<2, 6, 4>(a);
    case 112: return launch_fwd_bf3<2, 7, 0>(a);
    case 113: return launch_fwd_bf3<2, 7, 1>(a);
    case 114: return launch_fwd_bf3<2, 7, 2>(a);
    case 115: return launch_fwd_bf3<2, 7, 3>(a);
    case 116: return launch_fwd_bf3<2, 7, 4>(a);
    case 117: return launch_fwd_bf3<2, 7, 5>(a);
    case 128: return launch_fwd_bf3<2, 8, 0>(a);
    case 129: return launch_fwd_bf3<2, 8, 1>(a);
    case 130: return launch_fwd_bf3<2, 8, 2>(a);
    case 131: return launch_fwd_bf3<2, 8, 3>(a);
    case 132: return launch_fwd_bf3<2, 8, 4>(a);
    case 133: return launch_fwd_bf3<2, 8, 5>(a);
    case 134: return launch_fwd_bf3<2, 8, 6>(a);
    default: return (int)hipErrorInvalidValue;
  }
}

int bf3_bwd_w2(int S, int nso, const Bf3Args& a) {
  switch (S * 16 + nso) {
    case 16: return launch_bwd_bf3<2, 1, 0>(a);
    case 32: return launch_bwd_bf3<2, 2, 0>(a);
    case 48: return launch_bwd_bf3<2, 3, 0>(a);
    case 49: return launch_bwd_bf3<2, 3, 1>(a);
    case 64: return launch_bwd_bf3<2, 4, 0>(a);
    case 65: return launch_bwd_bf3<2, 4, 1>(a);
    case 66: return launch_bwd_bf3<2, 4, 2>(a);
    case 80: return launch_bwd_bf3<2, 5, 0>(a);
    case 81: return launch_bwd_bf3<2, 5, 1>(a);
    case 82: return launch_bwd_bf3<2, 5, 2>(a);
    case 83: return launch_bwd_bf3<2, 5, 3>(a);
    case 96: return launch_bwd_bf3<2, 6, 0>(a);
    case 97: return launch_bwd_bf3<2, 6, 1>(a);
    case 98: return launch_bwd_bf3<2, 6, 2>(a);
    case 99: return launch_bwd_bf3<2, 6, 3>(a);
    case 100: return launch_bwd_bf3<2, 6, 4>(a);
    case 112: return launch_bwd_bf3<2, 7, 0>(a);
    case 113: return launch_bwd_bf3<2, 7, 1>(a);
    case 114: return launch_bwd_bf3<2, 7, 2>(a);
    case 115: return launch_bwd_bf3<2, 7, 3>(a);
    case 116: return launch_bwd_bf3<2, 7, 4>(a);
    case 117: return launch_bwd_bf3<2, 7, 5>(a);
    case 128: return launch_bwd_bf3<2, 8, 0>(a);
    case 129: return launch_bwd_bf3<2, 8, 1>(a);
    case 130: return launch_bwd_bf3<2, 8, 2>(a);
    case 131: return launch_bwd_bf3<2, 8, 3>(a);
    case 132: return launch_bwd_bf3<2, 8, 4>(a);
    case 133: return launch_bwd_bf3<2, 8, 5>(a);
    case 134: return launch_bwd_bf3<2, 8, 6>(a);
    default: return (int)hipErrorInvalidValue;
  }
}
