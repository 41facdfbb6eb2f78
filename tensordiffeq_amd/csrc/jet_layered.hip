// Layer-wise jet engine epilogues (hidden widths beyond the fused kernels' register envelope).
//
// The fused jet kernels (jet_bf3.h) keep every stream of a 16-point tile in registers through the
// whole layer stack, which caps the hidden width at 128 (16 x 8 feature tiles).  The reference's
// neural_net takes any layer list (tensordiffeq/networks.py:10-20), so wider networks run
// layer by layer: the stacked-stream GEMMs [S*N, W_in] x [W_in, W_out] are the hand-written MFMA
// GEMMs of lay_gemm.hip (or the library GEMMs, TDQ_LAY_GEMM=0), and the bias + tanh jet (value,
// first- and second-order streams, Faa di Bruno) and its adjoint (lay_jet.h) run either in those
// GEMMs' epilogues (hidden layers, bf16 families) or as the memory-bound pass here (the input
// layer, the output layer's adjoint, fp32, the library path).  Streams are planes [S][N][W]
// (stream-major, contiguous), spec = JetPlan order (jet_hip.stream_spec).
//
//   forward  (in place Z -> H), backward (in place HB -> ZB from the saved post-activations: fp32
//   H, or - when the forward pass kept only the bf16 GEMM operands - H = hi + lo of two bf16 planes)
// Reference behaviour: the nested tf.gradients of the PDE residual.
#include "jet_bf3.h"  // (vector types)
#include "lay_jet.h"

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
  float z[S][V], b[V];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (V == 4) {
      const float4 q = *reinterpret_cast<const float4*>(Z + (long long)s * NW + e);
      z[s][0] = q.x; z[s][1] = q.y; z[s][2] = q.z; z[s][3] = q.w;
    } else {
      z[s][0] = Z[(long long)s * NW + e];
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) b[v] = bias[(int)((e + v) % W)];
  float o[S][V];
  lay_jet_fwd<S, V>(z, b, sp, o);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (V == 4)
      *reinterpret_cast<float4*>(Z + (long long)s * NW + e) = make_float4(o[s][0], o[s][1], o[s][2], o[s][3]);
    else
      Z[(long long)s * NW + e] = o[s][0];
    store_split<V>(bh, bl, (long long)s * NW + e, o[s]);
  }
}

// H: fp32 planes, or (Hh, Hl) bf16 planes with H = hi + lo (HP)
template <int S, int V, bool HP>
__global__ void __launch_bounds__(256) layered_bwd_kernel(float* __restrict__ HB, const float* __restrict__ H,
                                                          const __bf16* __restrict__ Hh, const __bf16* __restrict__ Hl,
                                                          long long NW, LSpec sp, __bf16* __restrict__ bh,
                                                          __bf16* __restrict__ bl) {
  const long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * V;
  if (e >= NW) return;
  float h[S][V], hb[S][V];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const long long o = (long long)s * NW + e;
    if constexpr (V == 4) {
      const float4 b = *reinterpret_cast<const float4*>(HB + o);
      hb[s][0] = b.x; hb[s][1] = b.y; hb[s][2] = b.z; hb[s][3] = b.w;
      if constexpr (HP) {
        const bf16x4 a = *reinterpret_cast<const bf16x4*>(Hh + o), c = *reinterpret_cast<const bf16x4*>(Hl + o);
#pragma unroll
        for (int v = 0; v < 4; ++v) h[s][v] = (float)a[v] + (float)c[v];
      } else {
        const float4 a = *reinterpret_cast<const float4*>(H + o);
        h[s][0] = a.x; h[s][1] = a.y; h[s][2] = a.z; h[s][3] = a.w;
      }
    } else {
      h[s][0] = HP ? (float)Hh[o] + (float)Hl[o] : H[o];
      hb[s][0] = HB[o];
    }
  }
  float zb[S][V];
  lay_jet_bwd<S, V>(h, hb, sp, zb);
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
static int launch_layered(int fwd, float* A, const float* B, const __bf16* Hh, const __bf16* Hl, const float* bias,
                          long long NW, int W, const LSpec& sp, __bf16* bh, __bf16* bl, hipStream_t st) {
  const bool vec = (NW % 4) == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0 &&
                   (B == nullptr || (reinterpret_cast<uintptr_t>(B) & 15) == 0) &&
                   (Hh == nullptr || ((reinterpret_cast<uintptr_t>(Hh) | reinterpret_cast<uintptr_t>(Hl)) & 7) == 0);
  const int V = vec ? 4 : 1;
  const long long threads = (NW + V - 1) / V;
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (fwd) {
    if (vec) hipLaunchKernelGGL((layered_fwd_kernel<S, 4>), grid, dim3(256), 0, st, A, bias, NW, W, sp, bh, bl);
    else hipLaunchKernelGGL((layered_fwd_kernel<S, 1>), grid, dim3(256), 0, st, A, bias, NW, W, sp, bh, bl);
  } else if (Hh != nullptr) {
    if (vec)
      hipLaunchKernelGGL((layered_bwd_kernel<S, 4, true>), grid, dim3(256), 0, st, A, B, Hh, Hl, NW, sp, bh, bl);
    else
      hipLaunchKernelGGL((layered_bwd_kernel<S, 1, true>), grid, dim3(256), 0, st, A, B, Hh, Hl, NW, sp, bh, bl);
  } else {
    if (vec)
      hipLaunchKernelGGL((layered_bwd_kernel<S, 4, false>), grid, dim3(256), 0, st, A, B, Hh, Hl, NW, sp, bh, bl);
    else
      hipLaunchKernelGGL((layered_bwd_kernel<S, 1, false>), grid, dim3(256), 0, st, A, B, Hh, Hl, NW, sp, bh, bl);
  }
  TDQ_CHECK_LAUNCH();
  return 0;
}

static inline __bf16* H16(void* p) { return reinterpret_cast<__bf16*>(p); }
static inline const __bf16* H16c(const void* p) { return reinterpret_cast<const __bf16*>(p); }

extern "C" {

// fwd = 1: A = Z [S][N][W] -> H in place (bias [W] on the value stream).
// fwd = 0: A = HB [S][N][W] -> ZB in place from the same layer's post-activations: B = H (fp32), or
//          B = nullptr and hh / hl the bf16 planes with H = hi + lo.
// bh / bl (nullable, [S][N][W] bf16): the output's bf16 GEMM operand (hi) and its residual (lo).
int tdq_layered_epi(int fwd, float* A, const float* B, const float* bias, long long N, int W, int S, const int* spec,
                    void* bh, void* bl, const void* hh, const void* hl, void* stream) {
  if (N <= 0) return 0;
  const bool hp = !fwd && B == nullptr;
  if (S < 1 || S > TDQ_MAXS || W < 1 || A == nullptr || (fwd && bias == nullptr) ||
      (hp && (hh == nullptr || hl == nullptr)))
    return (int)hipErrorInvalidValue;
  LSpec sp;
  if (!lspec_parse(spec, S, sp)) return (int)hipErrorInvalidValue;
  const long long NW = N * (long long)W;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const __bf16 *Hh = hp ? H16c(hh) : nullptr, *Hl = hp ? H16c(hl) : nullptr;
  switch (S) {
#define TDQ_LAY_CASE(s_) \
  case s_: return launch_layered<s_>(fwd, A, B, Hh, Hl, bias, NW, W, sp, H16(bh), H16(bl), st);
    TDQ_LAY_CASE(1) TDQ_LAY_CASE(2) TDQ_LAY_CASE(3) TDQ_LAY_CASE(4)
    TDQ_LAY_CASE(5) TDQ_LAY_CASE(6) TDQ_LAY_CASE(7) TDQ_LAY_CASE(8)
#undef TDQ_LAY_CASE
    default: return (int)hipErrorInvalidValue;
  }
}

}  // extern "C"
