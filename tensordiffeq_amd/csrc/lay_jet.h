// The tanh jet of one hidden layer and its adjoint, per (point, feature), shared by the layer-wise
// engine's standalone epilogue pass (jet_layered.hip) and the GEMM epilogues of its hand-written
// MFMA kernels (lay_gemm.hip).  Streams follow the JetPlan order (value, first-order,
// second-order; ops/jet_hip.py stream_spec):
//
//   forward:   h = tanh(z + b), s1 = 1 - h^2, h_a = s1 z_a, h_ab = s1 (z_ab - 2 h z_a z_b)
//   adjoint:   zb_ab = s1 hb_ab
//              zb_a  = s1 hb_a - 2 h sum_{(a,b)} h_b hb_ab      (both slots of a pair)
//              zb    = s1 hb - 2 h sum_{s>0} h_s hb_s - 2 sum_{(a,b)} h_a h_b hb_ab
// (from the post-activations only - no tanh recompute).  Reference behaviour: the nested
// tf.gradients of the PDE residual.
#pragma once
#include "jet_common.h"

struct LSpec {
  int stype[TDQ_MAXS];
  int ia[TDQ_MAXS], ib[TDQ_MAXS];  // second-order streams: their two first-order factor streams
  int coord[TDQ_MAXS];             // first-order streams: the input coordinate
};

// host: JetPlan spec (3 ints per stream) -> LSpec; false when malformed
static inline bool lspec_parse(const int* spec, int S, LSpec& sp) {
  if (S < 1 || S > TDQ_MAXS) return false;
  for (int s = 0; s < TDQ_MAXS; ++s) {
    const int ty = s < S ? spec[3 * s] : 0;
    sp.stype[s] = ty;
    sp.ia[s] = ty == 2 ? spec[3 * s + 1] : 0;
    sp.ib[s] = ty == 2 ? spec[3 * s + 2] : 0;
    sp.coord[s] = ty == 1 ? spec[3 * s + 1] : 0;
    if (s < S && (ty < 0 || ty > 2 || (s == 0) != (ty == 0))) return false;
    if (ty == 2 && (sp.ia[s] <= 0 || sp.ia[s] >= S || sp.ib[s] <= 0 || sp.ib[s] >= S ||
                    spec[3 * sp.ia[s]] != 1 || spec[3 * sp.ib[s]] != 1))
      return false;
  }
  return true;
}

template <int S, int V>
__device__ __forceinline__ void lay_jet_fwd(const float (&z)[S][V], const float (&b)[V], const LSpec& sp,
                                            float (&o)[S][V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const float h = tanhf(z[0][v] + b[v]);
    const float s1 = 1.f - h * h;
    o[0][v] = h;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      if (sp.stype[s] == 1) {
        o[s][v] = s1 * z[s][v];
      } else {
        float za = 0.f, zb = 0.f;
#pragma unroll
        for (int q = 1; q < S; ++q) {  // register-indexed select of the two first-order factors
          za = (q == sp.ia[s]) ? z[q][v] : za;
          zb = (q == sp.ib[s]) ? z[q][v] : zb;
        }
        o[s][v] = s1 * (z[s][v] - 2.f * h * za * zb);
      }
    }
  }
}

template <int S, int V>
__device__ __forceinline__ void lay_jet_bwd(const float (&h)[S][V], const float (&hb)[S][V], const LSpec& sp,
                                            float (&zb)[S][V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const float h0 = h[0][v], s1 = 1.f - h0 * h0;
    float acc0 = s1 * hb[0][v];
#pragma unroll
    for (int s = 1; s < S; ++s) {
      acc0 -= 2.f * h0 * h[s][v] * hb[s][v];
      zb[s][v] = s1 * hb[s][v];
    }
#pragma unroll
    for (int s = 1; s < S; ++s) {
      if (sp.stype[s] != 2) continue;
      float ha = 0.f, hbb = 0.f;
#pragma unroll
      for (int q = 1; q < S; ++q) {
        ha = (q == sp.ia[s]) ? h[q][v] : ha;
        hbb = (q == sp.ib[s]) ? h[q][v] : hbb;
      }
      const float w = hb[s][v];
      acc0 -= 2.f * ha * hbb * w;
#pragma unroll
      for (int q = 1; q < S; ++q) {  // both factor slots (a diagonal pair (a, a) adds twice)
        if (q == sp.ia[s]) zb[q][v] -= 2.f * h0 * hbb * w;
        if (q == sp.ib[s]) zb[q][v] -= 2.f * h0 * ha * w;
      }
    }
    zb[0][v] = acc0;
  }
}
