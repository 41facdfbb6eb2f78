// Jet backward with the forward RECOMPUTED on chip ("bwdr"), precision bf16, for gfx950.
//
// Why: the saved-activation stream is the largest data stream of the split-bf16 step - the forward
// writes every hidden layer's post-activation jets (223 MB at 50k points, AC-SA) and the backward
// reads them back (268 MB), at 2-4 TB/s that is most of the step (profiles/r3_roofline_bf16.txt).
// Here the forward kernel only writes the jets J the loss needs (a few hundred KB), and this
// backward re-runs the forward for its own 64 points - the same MFMA sequence and tanh-jet code, so
// the same bits - keeping every hidden layer's post-activations IN REGISTERS (one wave per SIMD: 512
// VGPR + AGPR slots; value stream fp32, derivative streams bf16 exactly as the forward saves them;
// layer 0 rebuilt from x in fp32), then runs the backward of jet_bwd_bf3_kernel from those registers:
// output layer, then per hidden layer the dK images (points onto the MFMA k index through LDS,
// ds_read_b64_tr_b16) and hb = K zb fused with the tanh-jet adjoint.  Cost: the forward's MFMAs once
// more (~1/3 of the step's) against ~490 MB of HBM traffic.
//
// The layer count is a template parameter (LH hidden layers), so every layer's storage is static:
//   * the last hidden layer is never stored - its forward epilogue runs the output-layer backward
//     (hb = Ko ub, dKo, tanh-jet adjoint) tile by tile where the activations are produced;
//   * hidden layer LH-2 stays in registers (80 VGPRs at width 128 and 4 streams);
//   * layer 0 keeps its value stream (32 VGPRs), its derivative streams are rebuilt from it;
//   * layers 1 .. LH-3 go through the saved-activation buffer as before (one wave per SIMD has
//     512 registers; a second full layer spilled in the first build) - at the AC net (4 hidden
//     layers) one of the three stored layers, a third of the old traffic.
// Workgroup = 4 waves x 16 points (one wave per SIMD), gradient slab rows per 64 points (reduced by
// the same fused step tail).
// Reference behaviour: SURVEY.md §2.2 K2-K8 (the nested tf.gradients of models.py:update_loss).
#pragma once
#include "jet_bf3.h"

template <int I>
struct IntC {
  static constexpr int value = I;
};
// f(IntC<I>), I = A .. B - 1 ascending (DESC: descending), at compile time
template <int A, int B, bool DESC = false, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (A < B) {
    if constexpr (DESC) {
      f(IntC<B - 1>{});
      static_for<A, B - 1, DESC>(f);
    } else {
      f(IntC<A>{});
      static_for<A + 1, B, DESC>(f);
    }
  }
}

__device__ __forceinline__ u32x2 bf4_pack(const f32x4 v) {
  return __builtin_bit_cast(u32x2, __builtin_convertvector(v, bf16x4));
}
__device__ __forceinline__ f32x4 bf4_unpack(const u32x2 u) {
  return f32x4{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
               __uint_as_float(u[1] & 0xffff0000u)};
}

// one hidden layer's post-activation streams of this lane's (point, feature rows): the value stream
// fp32 (s1 = 1 - h^2 of a saturated unit needs it), derivative streams bf16 (as the forward's saves)
template <int S, int WT>
struct HLayer {
  f32x4 v[WT];
  u32x2 d[S > 1 ? S - 1 : 1][WT];
  __device__ __forceinline__ f32x4 get(int s, int t) const { return s == 0 ? v[t] : bf4_unpack(d[s - 1][t]); }
};

// hidden layer i of the recomputed forward: fwd_hidden<LO = false> with the epilogue writing the
// layer's registers instead of the saved-activation buffer
template <int WT, int S, int NSO, bool LAST, bool REG>
__device__ __forceinline__ void fwdr_hidden(bf16x8 (&ah)[S][WT / 2], const Tl& Wi, const float* __restrict__ bi,
                                            HLayer<S, WT>& H, const Tl& Hg, bf16x4* stage, const JetSpec& sp, int l,
                                            int g) {
  constexpr int KB = WT / 2, NSTEP = WT * KB, D = NSTEP < 4 ? NSTEP : 4;
  bf16x8 wh[D], wl[D];
#pragma unroll
  for (int k = 0; k < D; ++k) img_frag<false>(Wi, k, wh[k], wl[k]);
  f32x4 accA[S], accB[S], biasA = zero4(), biasB = zero4();
#pragma unroll
  for (int s = 0; s < S; ++s) accA[s] = accB[s] = zero4();
#pragma unroll
  for (int o = 0; o <= WT; ++o) {
    f32x4(&accC)[S] = (o & 1) ? accB : accA;
    f32x4(&accP)[S] = (o & 1) ? accA : accB;
    f32x4& biasC = (o & 1) ? biasB : biasA;
    const f32x4& biasP = (o & 1) ? biasA : biasB;
    if (o < WT) {
      biasC = *reinterpret_cast<const f32x4*>(bi + 16 * o + 4 * g);
#pragma unroll
      for (int s = 0; s < S; ++s) accC[s] = zero4();
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int st = o * KB + kb;
        const bf16x8 Ah = wh[st % D];
        if (st + D < NSTEP) img_frag<false>(Wi, st + D, wh[st % D], wl[st % D]);
#pragma unroll
        for (int s = 0; s < S; ++s) accC[s] = mfma_bf(Ah, ah[s][kb], accC[s]);
      }
    }
    if (o > 0) {
      const int t = o - 1;
      f32x4 z[S], h[S];
#pragma unroll
      for (int s = 0; s < S; ++s) z[s] = accP[s];
      z[0] += biasP;
      tanh_jet_f<S, NSO>(sp, z, h);
      if constexpr (REG) {
        H.v[t] = h[0];
#pragma unroll
        for (int s = 1; s < S; ++s) H.d[s - 1][t] = bf4_pack(h[s]);
      } else {  // the register budget holds one full layer: the others go through the saved-activation buffer
#pragma unroll
        for (int s = 0; s < S; ++s) hs_store<WT, false>(Hg, s, t, h[s]);
      }
      if (!LAST) {
#pragma unroll
        for (int s = 0; s < S; ++s) stage[((s * KB + (t >> 1)) * 64 + l) * 2 + (t & 1)] = cvt_hi4(h[s]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (!LAST) {  // wave-private LDS stage: program order suffices
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) ah[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[((s * KB + kb) * 64 + l) * 2]);
  }
}

// the LAST hidden layer of the recomputed forward fused with the output-layer backward: its
// post-activations are consumed tile by tile where they are produced (hb = Ko ub, dKo partials,
// the tanh-jet adjoint -> zb_{LH-1} bias partials and B fragments), so they are never kept
template <int WT, int S, int NSO>
__device__ __forceinline__ void fwdr_last(const bf16x8 (&ah)[S][WT / 2], const Tl& Wi, const float* __restrict__ bi,
                                          const float* __restrict__ Ko, const float (&ub)[S][TDQ_MAXO],
                                          bf16x8 (&zh)[S][WT / 2], float* accKo, float* accBslot, const JetSpec& sp,
                                          const NetDims& d, int w, int l, int p, int g) {
  constexpr int KB = WT / 2, NSTEP = WT * KB, D = NSTEP < 4 ? NSTEP : 4, W = 16 * WT;
  bf16x8 wh[D], wl[D];
#pragma unroll
  for (int k = 0; k < D; ++k) img_frag<false>(Wi, k, wh[k], wl[k]);
  f32x4 accA[S], accB[S], biasA = zero4(), biasB = zero4();
#pragma unroll
  for (int s = 0; s < S; ++s) accA[s] = accB[s] = zero4();
  bf16x4 ph[S];
#pragma unroll
  for (int o = 0; o <= WT; ++o) {
    f32x4(&accC)[S] = (o & 1) ? accB : accA;
    f32x4(&accP)[S] = (o & 1) ? accA : accB;
    f32x4& biasC = (o & 1) ? biasB : biasA;
    const f32x4& biasP = (o & 1) ? biasA : biasB;
    if (o < WT) {
      biasC = *reinterpret_cast<const f32x4*>(bi + 16 * o + 4 * g);
#pragma unroll
      for (int s = 0; s < S; ++s) accC[s] = zero4();
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int st = o * KB + kb;
        const bf16x8 Ah = wh[st % D];
        if (st + D < NSTEP) img_frag<false>(Wi, st + D, wh[st % D], wl[st % D]);
#pragma unroll
        for (int s = 0; s < S; ++s) accC[s] = mfma_bf(Ah, ah[s][kb], accC[s]);
      }
    }
    if (o > 0) {
      const int t = o - 1;
      f32x4 z[S], h[S];
#pragma unroll
      for (int s = 0; s < S; ++s) z[s] = accP[s];
      z[0] += biasP;
      tanh_jet_f<S, NSO>(sp, z, h);
      // the saved forward keeps derivative streams as bf16: the same rounding here
#pragma unroll
      for (int s = 1; s < S; ++s) h[s] = bf4_unpack(bf4_pack(h[s]));
      f32x4 hbt[S];
#pragma unroll
      for (int s = 0; s < S; ++s) hbt[s] = zero4();
      f32x4 kq[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) kq[c] = *reinterpret_cast<const f32x4*>(Ko + (16 * t + 4 * g + c) * 4);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int q = 0; q < TDQ_MAXO; ++q)
#pragma unroll
          for (int s = 0; s < S; ++s) hbt[s][c] = fmaf(kq[c][q], ub[s][q], hbt[s][c]);
#pragma unroll
      for (int q = 0; q < TDQ_MAXO; ++q) {
        if (q >= d.d_out) break;
        f32x4 part;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float a = 0.f;
#pragma unroll
          for (int s = 0; s < S; ++s) a = fmaf(ub[s][q], h[s][c], a);
          part[c] = a;
        }
        const float r = row16_sum4(part);
        if ((p & 3) == 0) accKo[w * W * TDQ_MAXO + (16 * t + 4 * g + (p >> 2)) * TDQ_MAXO + q] = r;
      }
      f32x4 zb[S];
      tanh_jet_b<S, NSO>(sp, h, hbt, zb);
      {
        const float r = row16_sum4(zb[0]);
        if ((p & 3) == 0) accBslot[w * W + 16 * t + 4 * g + (p >> 2)] = r;
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const bf16x4 hi = cvt_hi4(zb[s]);
        if (t & 1)
          zh[s][t >> 1] = cat8(ph[s], hi);
        else
          ph[s] = hi;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// (d) of hidden layer i from registers: hb_{i-1} = K_i zb_i on MFMA, the epilogue of output tile o-1
// (tanh-jet adjoint with h_{i-1}, bias partials, stage - or, i = 1, the first-layer partials) in the
// scheduling region of tile o's MFMAs (bwd_hidden_d with the saved tiles read from `hp`)
template <int WT, int S, int NSO, bool TO_FIRST, typename HG>
__device__ __forceinline__ void bwdr_hidden_d(const bf16x8 (&zh)[S][WT / 2], const Tl& Ki, const HG& hp,
                                              bf16x4* stage, float* accBslot, float* accK0,
                                              const float* __restrict__ xrow, const JetSpec& sp, const NetDims& d,
                                              int w, int l, int p, int g) {
  constexpr int KB = WT / 2, NSTEP = WT * KB, D = NSTEP < 4 ? NSTEP : 4;
  bf16x8 wh[D], wl[D];
#pragma unroll
  for (int k = 0; k < D; ++k) img_frag<false>(Ki, k, wh[k], wl[k]);
  f32x4 accA[S], accB[S];
#pragma unroll
  for (int s = 0; s < S; ++s) accA[s] = accB[s] = zero4();
#pragma unroll
  for (int o = 0; o <= WT; ++o) {
    f32x4(&accC)[S] = (o & 1) ? accB : accA;
    f32x4(&accP)[S] = (o & 1) ? accA : accB;
    if (o < WT) {
#pragma unroll
      for (int s = 0; s < S; ++s) accC[s] = zero4();
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int st = o * KB + kb;
        const bf16x8 Ah = wh[st % D];
        if (st + D < NSTEP) img_frag<false>(Ki, st + D, wh[st % D], wl[st % D]);
#pragma unroll
        for (int s = 0; s < S; ++s) accC[s] = mfma_bf(Ah, zh[s][kb], accC[s]);
      }
    }
    if (o > 0) {
      const int t = o - 1;
      f32x4 h[S], zb[S];
#pragma unroll
      for (int s = 0; s < S; ++s) h[s] = hp(s, t);
      tanh_jet_b<S, NSO>(sp, h, accP, zb);
      if constexpr (TO_FIRST)
        first_layer_partials<WT, S, NSO>(sp, zb, xrow, d, t, w, p, g, accBslot, accK0);
      else
        zb_to_stage<WT, S, false>(zb, d, t, w, l, p, g, accBslot, stage);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__host__ __device__ constexpr int bwdr_union_floats(int WT, int S) {
  // union of: forward stage (4 waves x S * WT * 128 floats) = zb stage, and the two dK image
  // buffers (h, zb for 64 points, row stride 144 bf16)
  return ((4 * S * WT * 128 > 2 * 2 * 64 * 144 / 2 ? 4 * S * WT * 128 : 2 * 2 * 64 * 144 / 2) + 3) / 4 * 4;
}
__host__ __device__ constexpr int bwdr_lds_floats(int WT, int S) {
  // + bias partials [3][4 waves][W], output-layer partials [4][W * MAXO] + [4][MAXO] and
  // first-layer partials [4][MAXD * W] - outside the union: waves reach the fused output phase
  // while others still read their forward stage
  return bwdr_union_floats(WT, S) + 3 * 4 * 16 * WT + 4 * 16 * WT * TDQ_MAXO + 4 * TDQ_MAXO + 4 * TDQ_MAXD * 16 * WT;
}

template <int WT, int S, int NSO, int LH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
jet_bwdr_kernel(const float* __restrict__ X, const float* __restrict__ aux, const bf16x8* __restrict__ Fimg,
                const bf16x8* __restrict__ Kimg, const float* __restrict__ dJ, const float* __restrict__ Hs_,
                float* __restrict__ slab, int N, int Ptot, NetDims d, JetSpec sp, int rev, int wg0) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int W = 16 * WT, KB = WT / 2, NSTEP = WT * KB;
  constexpr int NWV = 4, PTS = 64;
  constexpr int RS = 144, IMG = PTS * RS;
  constexpr int NR = WT / (NWV / 2), NC = WT / 2;
  constexpr int IH = 0, IZ = IMG;  // bf16 offsets inside one image buffer (h, zb)
  constexpr int IBUF = 2 * IMG;    // one buffer, in bf16
  static_assert(LH >= 2, "the recompute backward needs two hidden layers or more");
  constexpr int U = bwdr_union_floats(WT, S);
  __bf16* img = reinterpret_cast<__bf16*>(lds);
  float* accB = lds + U;                  // [3: layer parity 0/1, layer 0][NWV][W]
  float* accKo = accB + 3 * NWV * W;      // [NWV][W * TDQ_MAXO]
  float* accBo = accKo + NWV * W * TDQ_MAXO;  // [NWV][TDQ_MAXO]
  float* accK0 = accBo + NWV * TDQ_MAXO;  // [NWV][TDQ_MAXD * W]

  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwl = gridDim.x, wg = wg0 + (rev ? nwl - 1 - (int)blockIdx.x : (int)blockIdx.x);
  const int n = wg * PTS + w * 16 + p;
  const bool valid = n < N;
  const int nc = valid ? n : N - 1;
  const float vmask = valid ? 1.f : 0.f;
  __bf16* gs = reinterpret_cast<__bf16*>(slab) + (size_t)wg * Ptot;  // bf16 slab rows (slab_half(false))
  bf16x4* stage = reinterpret_cast<bf16x4*>(lds) + (size_t)w * (S * KB * 64 * 2);
  const int tr_row = 8 * g + ((l & 15) >> 2);
  const int swz = (g & 1) << 6;
  const int tr_col1 = 4 * ((l & 3) ^ ((2 * g) & 3));
  const int tr_col2 = 4 * ((l & 3) ^ ((2 * g + 1) & 3));
  auto dw_row = [](int wv, int r) { return NR * (wv >> 1) + r; };
  auto dw_col = [](int wv, int c) { return NC * (wv & 1) + c; };
  const float* xrow = X + (size_t)nc * d.d_in;
  float* Hs = const_cast<float*>(Hs_);
  const int nwgf = (N + 63) / 64;  // the saved-activation layout of the forward's 64-point workgroups

  // ---- forward, recomputed: layer 0 (its value stream kept; derivative streams rebuilt from it,
  //      h0_stream), hidden layers 1 .. LH-2 kept in registers, layer LH-1 fused with the
  //      output-layer backward -------------------------------------------------------------------
  float x[TDQ_MAXD];
#pragma unroll
  for (int j = 0; j < TDQ_MAXD; ++j) x[j] = j < d.d_in ? xrow[j] : 0.f;
  float ub[S][TDQ_MAXO];
#pragma unroll
  for (int q = 0; q < TDQ_MAXO; ++q)
#pragma unroll
    for (int s = 0; s < S; ++s) ub[s][q] = q < d.d_out ? vmask * dJ[((size_t)s * N + nc) * d.d_out + q] : 0.f;
  f32x4 h0v[WT];
  HLayer<S, WT> H[LH];
  bf16x8 zh[S][KB];
  {
    bf16x8 ah[S][KB];
    bf16x4 ph[S];
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      f32x4 h[S];
      h0_jet<WT, S, NSO>(sp, aux, d, x, t, g, h);
      h0v[t] = h[0];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const bf16x4 hi = cvt_hi4(h[s]);
        if (t & 1)
          ah[s][t >> 1] = cat8(ph[s], hi);
        else
          ph[s] = hi;
      }
    }
    static_for<1, LH - 1>([&](auto I) {
      constexpr int i = decltype(I)::value;
      fwdr_hidden<WT, S, NSO, false, i == LH - 2>(ah, tl_make(Fimg + (size_t)(i - 1) * NSTEP * 128, l),
                                                  aux + aux_bh(d, W) + (i - 1) * W, H[i],
                                                  hs_region<WT, false>(Hs, i, nwgf, wg, S, w, l), stage, sp, l, g);
    });
    fwdr_last<WT, S, NSO>(ah, tl_make(Fimg + (size_t)(LH - 2) * NSTEP * 128, l), aux + aux_bh(d, W) + (LH - 2) * W,
                          aux + aux_ko(d, W), ub, zh, accKo, accB + ((LH - 1) & 1) * NWV * W, sp, d, w, l, p, g);
  }
#pragma unroll
  for (int q = 0; q < TDQ_MAXO; ++q) {
    if (q >= d.d_out) break;
    const float v = row16_sum(ub[0][q]);
    if (l == 0) accBo[w * TDQ_MAXO + q] = v;
  }

  // the saved streams of hidden layer i as a callable (s, t) -> f32x4 (layer 0: rebuilt from its
  // value stream)
  auto hl = [&](auto I) {
    constexpr int i = decltype(I)::value;
    if constexpr (i == 0)
      return [&](int s, int t) { return h0_stream<WT, S, NSO>(sp, aux, h0v[t], t, g, s); };
    else if constexpr (i == LH - 2)
      return [&](int s, int t) { return H[i].get(s, t); };
    else
      return [&, Hg = hs_region<WT, false>(Hs, i, nwgf, wg, S, w, l)](int s, int t) { return hs_load<WT, false>(Hg, s, t); };
  };

  __syncthreads();
  if (w == 2) {
    const int ko = off_layer(d, LH);
    for (int e = l; e < hw(d, LH - 1) * d.d_out; e += 64) {
      const int f = e / d.d_out, q = e - f * d.d_out;
      const int k = f * TDQ_MAXO + q, st = W * TDQ_MAXO;
      float a = accKo[k];
#pragma unroll
      for (int v = 1; v < NWV; ++v) a += accKo[v * st + k];
      slab_put(gs + ko + e, a);
    }
    if (l < d.d_out) {
      float a = accBo[l];
#pragma unroll
      for (int v = 1; v < NWV; ++v) a += accBo[v * TDQ_MAXO + l];
      slab_put(gs + ko + hw(d, LH - 1) * d.d_out + l, a);
    }
  }

  // ---- hidden layers i = LH-1 .. 1: zh holds zb_i ---------------------------------------------
  static_for<1, LH, true>([&](auto I) {
    constexpr int i = decltype(I)::value;
    const auto hp = hl(IntC<i - 1>{});
    f32x4 dw[NR][NC];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) dw[r][c] = zero4();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      // previous users of the region done: the zb stage / forward stage (s = 0); with two image
      // buffers the barrier after this stream's writes orders them after the MFMAs of s - 1
      if (s == 0) __syncthreads();
      __bf16* const im = img + (s & 1) * IBUF;
      if (s == 0 && w == 0) {  // bias of layer i: partials of all waves landed before this barrier
        const float* accBi = accB + (i & 1) * NWV * W;
        const int bo = off_layer(d, i) + hw(d, i - 1) * hw(d, i);
        for (int f = l; f < hw(d, i); f += 64) {
          float a = accBi[f];
#pragma unroll
          for (int v = 1; v < NWV; ++v) a += accBi[v * W + f];
          slab_put(gs + bo + f, a);
        }
      }
      {
        const int row = 16 * w + p;
        const int rsw = ((row >> 3) & 1) << 6;
        const int wch = g ^ ((row >> 2) & 3);
#pragma unroll
        for (int t = 0; t < WT; ++t) {
          const int off = row * RS + ((16 * t + 4 * wch) ^ rsw);
          *reinterpret_cast<bf16x4*>(im + IH + off) = cvt_hi4(hp(s, t));
          *reinterpret_cast<bf16x4*>(im + IZ + off) = half8(zh[s][t >> 1], t & 1);
        }
      }
      __syncthreads();
      const int ra1 = tr_row * RS + ((16 * dw_row(w, 0) + tr_col1) ^ swz);
      const int ra2 = (tr_row + 4) * RS + ((16 * dw_row(w, 0) + tr_col2) ^ swz);
      const int ca1 = tr_row * RS + ((16 * dw_col(w, 0) + tr_col1) ^ swz);
      const int ca2 = (tr_row + 4) * RS + ((16 * dw_col(w, 0) + tr_col2) ^ swz);
#pragma unroll
      for (int kb = 0; kb < PTS / 32; ++kb) {
        bf16x8 Ah[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int off = ra1 + 32 * kb * RS + 16 * r;
          const int of2 = ra2 + 32 * kb * RS + 16 * r;
          Ah[r] = cat8(tr_read(im + IH + off), tr_read(im + IH + of2));
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int off = ca1 + 32 * kb * RS + 16 * c;
          const int of2 = ca2 + 32 * kb * RS + 16 * c;
          const bf16x8 Bh = cat8(tr_read(im + IZ + off), tr_read(im + IZ + of2));
#pragma unroll
          for (int r = 0; r < NR; ++r) dw[r][c] = mfma_bf(Ah[r], Bh, dw[r][c]);
        }
      }
    }
    {
      int in0 = 16 * dw_row(w, 0) + 4 * g, out0 = 16 * dw_col(w, 0) + p;
      asm volatile("" : "+v"(in0), "+v"(out0));
      __bf16* gk = gs + off_layer(d, i);
      if (d.uniform && d.width == W) {
        const Tl G = tl_make(gk, 0);
        const int voff = (in0 * W + out0) * 2;
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int c2 = 0; c2 < NC; ++c2)
#pragma unroll
            for (int c = 0; c < 4; ++c)
              __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (__bf16)dw[r][c2][c]), G.r, voff,
                                                    ((16 * r + c) * W + 16 * c2) * 2, 0);
      } else {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int c2 = 0; c2 < NC; ++c2)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const int in = in0 + 16 * r + c, out = out0 + 16 * c2;
              if (in < hw(d, i - 1) && out < hw(d, i)) slab_put(gk + in * hw(d, i) + out, dw[r][c2][c]);
            }
      }
    }
    __syncthreads();  // images consumed: the region becomes the zb fragment stage
    const Tl Ki = tl_make(Kimg + (size_t)(i - 1) * NSTEP * 128, l);
    if constexpr (i >= 2) {
      bwdr_hidden_d<WT, S, NSO, false>(zh, Ki, hp, stage, accB + ((i - 1) & 1) * NWV * W, accK0, xrow, sp, d, w, l,
                                       p, g);
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) zh[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[((s * KB + kb) * 64 + l) * 2]);
    } else {
      bwdr_hidden_d<WT, S, NSO, true>(zh, Ki, hp, stage, accB + 2 * NWV * W, accK0, xrow, sp, d, w, l, p, g);
    }
  });

  // ---- first-layer slabs (partials of all waves are in LDS) -----------------------------------
  __syncthreads();
  if (w == 0) {
    const float* accB0 = accB + 2 * NWV * W;
    const int bo = d.d_in * hw(d, 0);
    for (int f = l; f < hw(d, 0); f += 64) {
      float a = accB0[f];
#pragma unroll
      for (int v = 1; v < NWV; ++v) a += accB0[v * W + f];
      slab_put(gs + bo + f, a);
    }
  } else if (w == 1) {
    for (int e = l; e < d.d_in * hw(d, 0); e += 64) {
      const int j = e / hw(d, 0), f = e - j * hw(d, 0);
      const int k = j * W + f;
      float a = accK0[k];
#pragma unroll
      for (int v = 1; v < NWV; ++v) a += accK0[v * TDQ_MAXD * W + k];
      slab_put(gs + e, a);
    }
  }
}

// bwdr_dispatch (jet_bf3.h): a.img = the backward A image, a.fimg = the forward A image; -1 when
// the geometry has no instantiation

template <int WT, int S, int NSO, int LH>
int launch_bwdr(const Bf3Args& a) {
  constexpr int PTS = 64;
  const int hi = a.p_hi < 0 ? a.N : a.p_hi, wg0 = a.p_lo / PTS;
  const int nwg = (hi + PTS - 1) / PTS - wg0;
  const size_t lds = (size_t)bwdr_lds_floats(WT, S) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&jet_bwdr_kernel<WT, S, NSO, LH>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((jet_bwdr_kernel<WT, S, NSO, LH>), dim3(nwg), dim3(256), lds, a.st, a.X, a.aux, a.fimg, a.img, a.dJ,
                     a.Hs, a.slab, a.N, a.Ptot, a.d, a.sp, bwd_reverse_order(), wg0);
  TDQ_CHECK_LAUNCH();
  return 0;
}
