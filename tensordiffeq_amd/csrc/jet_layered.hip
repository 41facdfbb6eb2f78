// Layer-wise jet engine epilogues (hidden widths beyond the fused kernels' register envelope).
//
// The fused jet kernels (jet_bf3.h) keep every stream of a 16-point tile in registers through the
// whole layer stack, which caps the hidden width at 128 (16 x 8 feature tiles).  The reference's
// neural_net takes any layer list (tensordiffeq/networks.py:10-20), so wider networks run
// layer by layer: the stacked-stream GEMMs [S*N, W_in] x [W_in, W_out] are plain library GEMMs
// (hipBLASLt through torch.mm), and everything between them - bias, tanh jet (value, first- and
// second-order streams, Faa di Bruno) and its adjoint - is fused into one memory-bound pass per
// layer here.  Streams are planes [S][N][W] (stream-major, contiguous), spec = JetPlan order
// (value, first-order, second-order; jet_hip.stream_spec).
//
//   forward  (in place Z -> H):  h = tanh(z + b), s1 = 1 - h^2, h_a = s1 z_a,
//                                h_ab = s1 (z_ab - 2 h z_a z_b)
//   backward (in place HB -> ZB, from the saved post-activations only):
//                                zb_ab = s1 hb_ab
//                                zb_a  = s1 hb_a - 2 h sum_{(a,b)} h_b hb_ab   (both slots of a pair)
//                                zb    = s1 hb - 2 h sum_{s>0} h_s hb_s - 2 sum_{(a,b)} h_a h_b hb_ab
// Reference behaviour: the nested tf.gradients of the PDE residual.
#include "common.h"
#include "jet_common.h"

struct LSpec {
  int stype[TDQ_MAXS];
  int ia[TDQ_MAXS], ib[TDQ_MAXS];
};

// bf16 GEMM operands of an output, written by the same pass (nullptr: none): hi = rne(x), lo =
// rne(x - hi) for the bf16x3 family (ops/jet_layered.py _Op)
template <int V>
__device__ __forceinline__ void store_split(__bf16* __restrict__ hi, __bf16* __restrict__ lo, long long off,
                                            const float (&x)[V]) {
  if (hi == nullptr) return;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const __bf16 h = (__bf16)x[v];
    hi[off + v] = h;
    if (lo != nullptr) lo[off + v] = (__bf16)(x[v] - (float)h);
  }
}

template <int S, int V>
__global__ void __launch_bounds__(256) layered_fwd_kernel(float* __restrict__ Z, const float* __restrict__ bias,
                                                          long long NW, int W, LSpec sp, __bf16* __restrict__ bh,
                                                          __bf16* __restrict__ bl) {
  const long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * V;
  if (e >= NW) return;
  float z[S][V];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (V == 4) {
      const float4 q = *reinterpret_cast<const float4*>(Z + (long long)s * NW + e);
      z[s][0] = q.x; z[s][1] = q.y; z[s][2] = q.z; z[s][3] = q.w;
    } else {
      z[s][0] = Z[(long long)s * NW + e];
    }
  }
  float o[S][V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const float h = tanhf(z[0][v] + bias[(int)((e + v) % W)]);
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
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (V == 4)
      *reinterpret_cast<float4*>(Z + (long long)s * NW + e) = make_float4(o[s][0], o[s][1], o[s][2], o[s][3]);
    else
      Z[(long long)s * NW + e] = o[s][0];
    store_split<V>(bh, bl, (long long)s * NW + e, o[s]);
  }
}

template <int S, int V>
__global__ void __launch_bounds__(256) layered_bwd_kernel(float* __restrict__ HB, const float* __restrict__ H,
                                                          long long NW, LSpec sp, __bf16* __restrict__ bh,
                                                          __bf16* __restrict__ bl) {
  const long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * V;
  if (e >= NW) return;
  float h[S][V], hb[S][V];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (V == 4) {
      const float4 a = *reinterpret_cast<const float4*>(H + (long long)s * NW + e);
      const float4 b = *reinterpret_cast<const float4*>(HB + (long long)s * NW + e);
      h[s][0] = a.x; h[s][1] = a.y; h[s][2] = a.z; h[s][3] = a.w;
      hb[s][0] = b.x; hb[s][1] = b.y; hb[s][2] = b.z; hb[s][3] = b.w;
    } else {
      h[s][0] = H[(long long)s * NW + e];
      hb[s][0] = HB[(long long)s * NW + e];
    }
  }
  float zb[S][V];
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
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (V == 4)
      *reinterpret_cast<float4*>(HB + (long long)s * NW + e) = make_float4(zb[s][0], zb[s][1], zb[s][2], zb[s][3]);
    else
      HB[(long long)s * NW + e] = zb[s][0];
    store_split<V>(bh, bl, (long long)s * NW + e, zb[s]);
  }
}

template <int S>
static int launch_layered(int fwd, float* A, const float* B, const float* bias, long long NW, int W, const LSpec& sp,
                          __bf16* bh, __bf16* bl, hipStream_t st) {
  const bool vec = (NW % 4) == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0 &&
                   (B == nullptr || (reinterpret_cast<uintptr_t>(B) & 15) == 0);
  const int V = vec ? 4 : 1;
  const long long threads = (NW + V - 1) / V;
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (fwd) {
    if (vec) hipLaunchKernelGGL((layered_fwd_kernel<S, 4>), grid, dim3(256), 0, st, A, bias, NW, W, sp, bh, bl);
    else hipLaunchKernelGGL((layered_fwd_kernel<S, 1>), grid, dim3(256), 0, st, A, bias, NW, W, sp, bh, bl);
  } else {
    if (vec) hipLaunchKernelGGL((layered_bwd_kernel<S, 4>), grid, dim3(256), 0, st, A, B, NW, sp, bh, bl);
    else hipLaunchKernelGGL((layered_bwd_kernel<S, 1>), grid, dim3(256), 0, st, A, B, NW, sp, bh, bl);
  }
  TDQ_CHECK_LAUNCH();
  return 0;
}

static inline __bf16* H16(void* p) { return reinterpret_cast<__bf16*>(p); }

extern "C" {

// fwd = 1: A = Z [S][N][W] -> H in place (bias [W] on the value stream).
// fwd = 0: A = HB [S][N][W] -> ZB in place, B = H (saved post-activations of the same layer).
// bh / bl (nullable, [S][N][W] bf16): the output's bf16 GEMM operand (hi) and its residual (lo).
int tdq_layered_epi(int fwd, float* A, const float* B, const float* bias, long long N, int W, int S, const int* spec,
                    void* bh, void* bl, void* stream) {
  if (N <= 0) return 0;
  if (S < 1 || S > TDQ_MAXS || W < 1 || A == nullptr || (fwd && bias == nullptr) || (!fwd && B == nullptr))
    return (int)hipErrorInvalidValue;
  LSpec sp;
  for (int s = 0; s < TDQ_MAXS; ++s) {
    const int ty = s < S ? spec[3 * s] : 0;
    sp.stype[s] = ty;
    sp.ia[s] = ty == 2 ? spec[3 * s + 1] : 0;
    sp.ib[s] = ty == 2 ? spec[3 * s + 2] : 0;
    if (s < S && (ty < 0 || ty > 2 || (s == 0) != (ty == 0))) return (int)hipErrorInvalidValue;
    if (ty == 2 && (sp.ia[s] <= 0 || sp.ia[s] >= S || sp.ib[s] <= 0 || sp.ib[s] >= S ||
                    spec[3 * sp.ia[s]] != 1 || spec[3 * sp.ib[s]] != 1))
      return (int)hipErrorInvalidValue;
  }
  const long long NW = N * (long long)W;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (S) {
    case 1: return launch_layered<1>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    case 2: return launch_layered<2>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    case 3: return launch_layered<3>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    case 4: return launch_layered<4>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    case 5: return launch_layered<5>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    case 6: return launch_layered<6>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    case 7: return launch_layered<7>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    case 8: return launch_layered<8>(fwd, A, B, bias, NW, W, sp, H16(bh), H16(bl), st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // extern "C"
