// Fused Taylor-jet tanh-MLP forward / backward for gfx950 (MI355X, CDNA4).
//
// What it computes (reference: the nested tf.gradients graphs of the PDE residual,
// SURVEY.md §2.2 K2-K8): for every point x and every derivative stream s of a plan
//   stream types   0: value u      1: d/dx_a u      2: d2/dx_a dx_b u   (order <= 2)
// the network output jet J[s][n][q], and in the backward the parameter gradient
//   dL/dtheta = sum_n sum_s (dL/dJ[s][n]) . dJ[s][n]/dtheta.
//
// Layout / mapping (MFMA v_mfma_f32_16x16x4_f32, exact fp32):
//   * one workgroup = 4 waves = 64 points; one wave = 16 points (one MFMA column tile).
//   * "feature-major": activations of every stream live in VGPRs as f32x4 act[s][t]; lane l
//     holds point (l & 15) and features 16t + 4(l>>4) + {0..3}.  That is exactly the C/D
//     layout of the MFMA AND the B-operand layout of the next layer's GEMM (k = l>>4 ranges
//     over 4 features per MFMA), so no cross-lane movement is needed between layers; a layer's
//     outputs are parked in a wave-private LDS image while its inputs are still being consumed
//     (only one activation set occupies VGPRs: the arch-VGPR budget is 256).
//   * the A operand (weights) comes from zero-padded W x W images in global memory (64 KiB per
//     layer, L2 resident): one 16-B load per lane feeds 4 MFMAs x S streams.
//   * tanh jet (Faa di Bruno, order 2): h = tanh z, s1 = 1 - h^2, s2 = -2 h s1,
//       h_a = s1 z_a,  h_ab = s1 z_ab + s2 z_a z_b
//   * the forward saves every hidden pre-activation stream ("register image": 1 KiB of
//     16-B-per-lane stores per (layer, stream, wave, feature tile)) for the backward.
//   * backward: recompute tanh, s1, s2, s3 from the saved z, chain the stream adjoints
//       zb_ab = s1 hb_ab ; zb_a = s1 hb_a + sum s2 z_b hb_ab ; zb = s1 hb + s2 sb1 + s3 sb2
//     (sb1 = sum z_c hb_c, sb2 = sum z_a z_b hb_ab), propagate hb_prev = K zb on MFMA, and form
//     dK = sum_points sum_streams h_prev zb^T on MFMA after an LDS transpose (points move from
//     the lane index to the k index).  Each workgroup writes one partial-gradient slab; a
//     deterministic two-pass reduction folds the slabs into the flat gradient (Keras order).
#include "jet_common.h"


template <int S, int WT>
__device__ __forceinline__ f32x4 pick(const f32x4 (&v)[S][WT], const float (&sel)[TDQ_MAXS], int t) {
  f32x4 r = zero4();
#pragma unroll
  for (int q = 1; q < S; ++q) r += sel[q] * v[q][t];
  return r;
}

// forward tanh jet on feature tile t: z -> h  (in place allowed: writes h after reading z)
template <int S, int WT>
__device__ __forceinline__ void tanh_jet_fwd(const JetSpec sp, const f32x4 (&z)[S][WT], int t,
                                             f32x4 (&h)[S][WT], int to) {
  f32x4 za2[S], zb2[S];
#pragma unroll
  for (int s = 1; s < S; ++s) {
    if (sp.stype[s] == 2) {
      za2[s] = pick<S, WT>(z, sp.selA[s], t);
      zb2[s] = pick<S, WT>(z, sp.selB[s], t);
    } else {
      za2[s] = zero4();
      zb2[s] = zero4();
    }
  }
  f32x4 zz[S];
#pragma unroll
  for (int s = 0; s < S; ++s) zz[s] = z[s][t];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float hv = tanhf(zz[0][c]);
    const float s1 = 1.f - hv * hv;
    const float s2 = -2.f * hv * s1;
    h[0][to][c] = hv;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      float v = s1 * zz[s][c];
      if (sp.stype[s] == 2) v = fmaf(s2 * za2[s][c], zb2[s][c], v);
      h[s][to][c] = v;
    }
  }
}


// ------------------------------------------------------------------------------------------
// weight images: zero-padded W x W copies of the hidden kernels, read directly by the MFMA
// A-operand loads (L2 resident: 64 KiB per layer at width 128).
//   transposed = 1: [out][in]  (forward:  z = K^T h)
//   transposed = 0: [in][out]  (backward: hb = K zb)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) pad_weights_kernel(const float* __restrict__ P, float* __restrict__ img,
                                                          NetDims d, int W, int transposed) {
  const int64_t total = (int64_t)(d.n_hidden - 1) * W * W;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int i = (int)(e / ((int64_t)W * W)) + 1;
    const int rem = (int)(e - (int64_t)(i - 1) * W * W);
    const int r = rem / W, c = rem - (rem / W) * W;
    const int in = transposed ? c : r, out = transposed ? r : c;
    img[e] = (in < d.width && out < d.width) ? P[off_layer(d, i) + in * d.width + out] : 0.f;
  }
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
template <int WT, int S>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
jet_fwd_kernel(const float* __restrict__ X, const float* __restrict__ P, const float* __restrict__ Wt,
               float* __restrict__ J, float* __restrict__ Zs, int N, NetDims d, JetSpec sp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int W = 16 * WT;
  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR addressing
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int n = wg * 64 + w * 16 + p;
  const bool valid = n < N;
  float* stage = lds + (size_t)w * (S * WT * 256);  // this wave's private activation image

  float x[TDQ_MAXD];
#pragma unroll
  for (int j = 0; j < TDQ_MAXD; ++j) x[j] = (j < d.d_in && valid) ? X[(size_t)n * d.d_in + j] : 0.f;

  f32x4 act[S][WT];
  // ---- layer 0 (input -> width): VALU; derivative streams are columns of K0 ---------------
  {
    const float* K0 = P;
    const float* b0 = P + d.d_in * d.width;
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      f32x4 zt[S][1], ht[S][1];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * t + 4 * g + c;
        const bool fv = f < d.width;
        float z0 = fv ? b0[f] : 0.f;
#pragma unroll
        for (int j = 0; j < TDQ_MAXD; ++j)
          if (j < d.d_in) z0 = fmaf(x[j], fv ? K0[j * d.width + f] : 0.f, z0);
        zt[0][0][c] = z0;
#pragma unroll
        for (int s = 1; s < S; ++s)
          zt[s][0][c] = (sp.stype[s] == 1 && fv) ? K0[sp.var[s] * d.width + f] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < S; ++s)
        *reinterpret_cast<f32x4*>(Zs + zs_index(0, nwg, wg, S, s, w, WT, t, l)) = zt[s][0];
      tanh_jet_fwd<S, 1>(sp, zt, 0, ht, 0);
#pragma unroll
      for (int s = 0; s < S; ++s) act[s][t] = ht[s][0];
    }
  }

  // ---- hidden layers (width -> width) on MFMA; A = padded K^T image from global (L2) ------
  //      weight fragments are prefetched one (o, t) step ahead (4 VGPRs in flight); the
  //      sched_barrier fences stop the compiler from hoisting every fragment load.
  for (int i = 1; i < d.n_hidden; ++i) {
    const float* Wi = Wt + (size_t)(i - 1) * W * W + (unsigned)(p * W + 4 * g);
    const float* b = P + off_layer(d, i) + d.width * d.width;
    f32x4 a_cur = *reinterpret_cast<const f32x4*>(Wi);
#pragma unroll
    for (int o = 0; o < WT; ++o) {
      f32x4 acc[S];
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] = zero4();
#pragma unroll
      for (int t = 0; t < WT; ++t) {
        const int nt = (t + 1 < WT) ? t + 1 : 0, no = (t + 1 < WT) ? o : o + 1;
        f32x4 a_nxt = a_cur;
        if (no < WT) a_nxt = *reinterpret_cast<const f32x4*>(Wi + (size_t)16 * no * W + 16 * nt);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int s = 0; s < S; ++s) acc[s] = mfma16x16x4(a_cur[r], act[s][t][r], acc[s]);
        a_cur = a_nxt;
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * o + 4 * g + c;
        acc[0][c] += (f < d.width) ? b[f] : 0.f;
      }
      f32x4 zt[S][1], ht[S][1];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        zt[s][0] = acc[s];
        *reinterpret_cast<f32x4*>(Zs + zs_index(i, nwg, wg, S, s, w, WT, o, l)) = acc[s];
      }
      tanh_jet_fwd<S, 1>(sp, zt, 0, ht, 0);
#pragma unroll
      for (int s = 0; s < S; ++s)
        *reinterpret_cast<f32x4*>(&stage[((s * WT + o) * 64 + l) * 4]) = ht[s][0];
    }
    // this wave's image -> registers (wave-private LDS region: program order suffices)
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int t = 0; t < WT; ++t) act[s][t] = *reinterpret_cast<const f32x4*>(&stage[((s * WT + t) * 64 + l) * 4]);
  }

  // ---- output layer (width -> d_out): VALU dot + cross-lane sum over feature groups ------
  {
    const float* Ko = P + off_layer(d, d.n_hidden);
    const float* bo = Ko + d.width * d.d_out;
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q) {
      if (q >= d.d_out) break;
      float kq[WT][4];
#pragma unroll
      for (int t = 0; t < WT; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 16 * t + 4 * g + c;
          kq[t][c] = f < d.width ? Ko[f * d.d_out + q] : 0.f;
        }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        float v = 0.f;
#pragma unroll
        for (int t = 0; t < WT; ++t)
#pragma unroll
          for (int c = 0; c < 4; ++c) v = fmaf(act[s][t][c], kq[t][c], v);
        v = col4_sum(v);
        if (s == 0) v += bo[q];
        if (g == 0 && valid) J[((size_t)s * N + n) * d.d_out + q] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void tanh_jet_bwd(const JetSpec sp, const f32x4 (&z)[S], const f32x4 (&hb)[S],
                                             f32x4 (&zb)[S]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float hv = tanhf(z[0][c]);
    const float s1 = 1.f - hv * hv;
    const float s2 = -2.f * hv * s1;
    const float s3 = -2.f * s1 * s1 - 2.f * hv * s2;
    float sb1 = 0.f, sb2 = 0.f;
    float zbv[S];
    zbv[0] = s1 * hb[0][c];
#pragma unroll
    for (int s = 1; s < S; ++s) {
      zbv[s] = s1 * hb[s][c];
      sb1 = fmaf(z[s][c], hb[s][c], sb1);
    }
#pragma unroll
    for (int s = 1; s < S; ++s) {
      if (sp.stype[s] == 2) {
        float za = 0.f, zbb = 0.f;
#pragma unroll
        for (int q = 1; q < S; ++q) {
          za = fmaf(sp.selA[s][q], z[q][c], za);
          zbb = fmaf(sp.selB[s][q], z[q][c], zbb);
        }
        const float hbs = hb[s][c];
        sb2 = fmaf(za * zbb, hbs, sb2);
        const float ga = s2 * zbb * hbs, gb = s2 * za * hbs;
#pragma unroll
        for (int q = 1; q < S; ++q) zbv[q] = fmaf(sp.selA[s][q], ga, fmaf(sp.selB[s][q], gb, zbv[q]));
      }
    }
    zbv[0] = fmaf(s2, sb1, fmaf(s3, sb2, zbv[0]));
#pragma unroll
    for (int s = 0; s < S; ++s) zb[s][c] = zbv[s];
  }
}

// saved pre-activation streams needed to rebuild h stream `s` of a layer on one feature tile
struct HLoad {
  f32x4 z0, zs, za, zb;
};

template <int S>
__device__ __forceinline__ void h_load(HLoad& L, const JetSpec sp, const float* __restrict__ Zs, int layer,
                                       int nwg, int wg, int s, int w, int WT, int t, int lane) {
  L.z0 = *reinterpret_cast<const f32x4*>(Zs + zs_index(layer, nwg, wg, S, 0, w, WT, t, lane));
  L.zs = L.za = L.zb = zero4();
  if (s > 0) L.zs = *reinterpret_cast<const f32x4*>(Zs + zs_index(layer, nwg, wg, S, s, w, WT, t, lane));
  if (sp.stype[s] == 2) {
    L.za = *reinterpret_cast<const f32x4*>(Zs + zs_index(layer, nwg, wg, S, sp.ia[s], w, WT, t, lane));
    L.zb = *reinterpret_cast<const f32x4*>(Zs + zs_index(layer, nwg, wg, S, sp.ib[s], w, WT, t, lane));
  }
}

__device__ __forceinline__ f32x4 h_compute(const HLoad& L, const JetSpec sp, int s) {
  f32x4 out;
  const bool second = sp.stype[s] == 2;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float hv = tanhf(L.z0[c]);
    const float s1 = 1.f - hv * hv;
    const float s2 = -2.f * hv * s1;
    const float v = second ? fmaf(s2 * L.za[c], L.zb[c], s1 * L.zs[c]) : s1 * L.zs[c];
    out[c] = s == 0 ? hv : v;
  }
  return out;
}

template <int S, int WT>
__device__ __forceinline__ void z_load(f32x4 (&z)[S], const float* __restrict__ Zs, int layer, int nwg, int wg,
                                       int w, int t, int lane) {
#pragma unroll
  for (int s = 0; s < S; ++s) z[s] = *reinterpret_cast<const f32x4*>(Zs + zs_index(layer, nwg, wg, S, s, w, WT, t, lane));
}

template <int WT, int S>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
jet_bwd_kernel(const float* __restrict__ X, const float* __restrict__ P, const float* __restrict__ Kp,
               const float* __restrict__ dJ, const float* __restrict__ Zs, float* __restrict__ slab, int N,
               int Ptot, NetDims d, JetSpec sp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int W = 16 * WT;
  constexpr int HS = W + 16;
  // dK tile ownership: WT >= 4 -> wave w owns tile rows {w, w+4, ..} x all columns;
  // WT = 2 -> one tile (w>>1, w&1) per wave; WT = 1 -> wave 0 owns the single tile.
  constexpr int NR = WT >= 4 ? WT / 4 : 1;
  constexpr int NC = WT >= 4 ? WT : 1;
  constexpr int NQ = NR * NC;
  constexpr int U1 = 2 * 64 * HS;             // transpose images
  constexpr int U2 = 4 * S * WT * 256;        // per-wave hb staging
  constexpr int U = U1 > U2 ? U1 : U2;
  float* ldsH = lds;
  float* ldsZ = lds + 64 * HS;
  // small-gradient partials, one slot per wave (summed in fixed wave order: bitwise deterministic)
  float* accK0 = lds + U;                     // [4][TDQ_MAXD * W]
  float* accB = accK0 + 4 * TDQ_MAXD * W;     // [2 (layer parity)][4][W]
  float* accKo = accB + 8 * W;                // [4][W * TDQ_MAXO]
  float* accBo = accKo + 4 * W * TDQ_MAXO;    // [4][TDQ_MAXO]

  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR addressing
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int n = wg * 64 + w * 16 + p;
  const bool valid = n < N;
  const int Lh = d.n_hidden;
  float* gs = slab + (size_t)wg * Ptot;
  float* hstage = lds + (size_t)w * (S * WT * 256);
  const bool DW_ACTIVE = WT > 1 || w == 0;
  auto dw_row = [](int wv, int r) { return WT >= 4 ? wv + 4 * r : (WT == 2 ? (wv >> 1) : 0); };
  auto dw_col = [](int wv, int c) { return WT >= 4 ? c : (WT == 2 ? (wv & 1) : 0); };

  __syncthreads();  // accumulators zeroed

  // ---- output layer: hb = Ko ub ; dKo += h_last ub ; dbo += ub_value ----------------------
  //      hb (the adjoint entering the top tanh layer) is parked in this wave's LDS staging
  //      image; every layer reads it tile by tile, so only zb occupies VGPRs across a layer.
  {
    const float* Ko = P + off_layer(d, Lh);
    f32x4 zc[S], zn[S];
    z_load<S, WT>(zc, Zs, Lh - 1, nwg, wg, w, 0, l);
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      if (t + 1 < WT) z_load<S, WT>(zn, Zs, Lh - 1, nwg, wg, w, t + 1, l);
      f32x4 zl[S][1], hl[S][1];
#pragma unroll
      for (int s = 0; s < S; ++s) zl[s][0] = zc[s];
      tanh_jet_fwd<S, 1>(sp, zl, 0, hl, 0);
      f32x4 hbt[S];
#pragma unroll
      for (int s = 0; s < S; ++s) hbt[s] = zero4();
      for (int q = 0; q < d.d_out; ++q) {
        float ubq[S];
#pragma unroll
        for (int s = 0; s < S; ++s) ubq[s] = valid ? dJ[((size_t)s * N + n) * d.d_out + q] : 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 16 * t + 4 * g + c;
          const bool fv = f < d.width;
          const float kq = fv ? Ko[f * d.d_out + q] : 0.f;
          float part = 0.f;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            hbt[s][c] = fmaf(kq, ubq[s], hbt[s][c]);
            part = fmaf(hl[s][0][c], ubq[s], part);
          }
          part = row16_sum(part);
          if (p == 0 && fv) accKo[w * W * TDQ_MAXO + f * TDQ_MAXO + q] = part;
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) *reinterpret_cast<f32x4*>(&hstage[((s * WT + t) * 64 + l) * 4]) = hbt[s];
      if (t + 1 < WT) {
#pragma unroll
        for (int s = 0; s < S; ++s) zc[s] = zn[s];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int q = 0; q < d.d_out; ++q) {
      const float v = row16_sum(valid ? dJ[(size_t)n * d.d_out + q] : 0.f);
      if (l == 0) accBo[w * TDQ_MAXO + q] = v;
    }
  }

  // ---- hidden layers i = Lh-1 .. 1 (the first layer is peeled below so that hb is
  //      redefined on every back edge - otherwise its old value stays live through the body)
  for (int i = Lh - 1; i >= 1; --i) {
    // (a) stream adjoints of the pre-activation (zb replaces hb)
    f32x4 zb[S][WT];
    {
      f32x4 zc[S], zn[S];
      z_load<S, WT>(zc, Zs, i, nwg, wg, w, 0, l);
#pragma unroll
      for (int t = 0; t < WT; ++t) {
        if (t + 1 < WT) z_load<S, WT>(zn, Zs, i, nwg, wg, w, t + 1, l);
        f32x4 hh[S], oo[S];
#pragma unroll
        for (int s = 0; s < S; ++s) hh[s] = *reinterpret_cast<const f32x4*>(&hstage[((s * WT + t) * 64 + l) * 4]);
        tanh_jet_bwd<S>(sp, zc, hh, oo);
#pragma unroll
        for (int s = 0; s < S; ++s) zb[s][t] = oo[s];
        if (t + 1 < WT) {
#pragma unroll
          for (int s = 0; s < S; ++s) zc[s] = zn[s];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // (b) bias gradient partials (value stream only)
    float* accBi = accB + (i & 1) * 4 * W;
#pragma unroll
    for (int t = 0; t < WT; ++t)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * t + 4 * g + c;
        const float v = row16_sum(zb[0][t][c]);
        if (p == 0 && f < d.width) accBi[w * W + f] = v;
      }

    // (c) dK_i = sum_points sum_streams h_{i-1} zb^T : per stream, both operands go through an
    //     LDS image [point][feature] so that points move to the MFMA k index.
    f32x4 dw[NQ];
#pragma unroll
    for (int qi = 0; qi < NQ; ++qi) dw[qi] = zero4();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      __syncthreads();
      {
        HLoad cur, nxt;
        h_load<S>(cur, sp, Zs, i - 1, nwg, wg, s, w, WT, 0, l);
#pragma unroll
        for (int t = 0; t < WT; ++t) {
          if (t + 1 < WT) h_load<S>(nxt, sp, Zs, i - 1, nwg, wg, s, w, WT, t + 1, l);
          *reinterpret_cast<f32x4*>(&ldsH[(16 * w + p) * HS + 16 * t + 4 * g]) = h_compute(cur, sp, s);
          *reinterpret_cast<f32x4*>(&ldsZ[(16 * w + p) * HS + 16 * t + 4 * g]) = zb[s][t];
          if (t + 1 < WT) cur = nxt;
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __syncthreads();
      if (DW_ACTIVE) {
        float fa[NR], fb[NC];
#pragma unroll
        for (int r = 0; r < NR; ++r) fa[r] = ldsH[g * HS + 16 * dw_row(w, r) + p];
#pragma unroll
        for (int c = 0; c < NC; ++c) fb[c] = ldsZ[g * HS + 16 * dw_col(w, c) + p];
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
          float na[NR], nb[NC];
          if (ks + 1 < 16) {
#pragma unroll
            for (int r = 0; r < NR; ++r) na[r] = ldsH[(4 * (ks + 1) + g) * HS + 16 * dw_row(w, r) + p];
#pragma unroll
            for (int c = 0; c < NC; ++c) nb[c] = ldsZ[(4 * (ks + 1) + g) * HS + 16 * dw_col(w, c) + p];
          }
#pragma unroll
          for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int c = 0; c < NC; ++c) dw[r * NC + c] = mfma16x16x4(fa[r], fb[c], dw[r * NC + c]);
          if (ks + 1 < 16) {
#pragma unroll
            for (int r = 0; r < NR; ++r) fa[r] = na[r];
#pragma unroll
            for (int c = 0; c < NC; ++c) fb[c] = nb[c];
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __syncthreads();  // transpose images consumed: the region is reused as hb staging below
    if (DW_ACTIVE) {
      const int ko = off_layer(d, i);
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c2 = 0; c2 < NC; ++c2) {
          const int out = 16 * dw_col(w, c2) + p;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int in = 16 * dw_row(w, r) + 4 * g + c;
            if (in < d.width && out < d.width) gs[ko + in * d.width + out] = dw[r * NC + c2][c];
          }
        }
    }
    // (d) hb_{i-1} = K_i zb  (MFMA; A = padded [in][out] image from global, B = zb registers)
    {
      const float* Ki = Kp + (size_t)(i - 1) * W * W + (unsigned)(p * W + 4 * g);
      f32x4 a_cur = *reinterpret_cast<const f32x4*>(Ki);
#pragma unroll
      for (int o = 0; o < WT; ++o) {
        f32x4 acc[S];
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s] = zero4();
#pragma unroll
        for (int t = 0; t < WT; ++t) {
          const int nt = (t + 1 < WT) ? t + 1 : 0, no = (t + 1 < WT) ? o : o + 1;
          f32x4 a_nxt = a_cur;
          if (no < WT) a_nxt = *reinterpret_cast<const f32x4*>(Ki + (size_t)16 * no * W + 16 * nt);
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int s = 0; s < S; ++s) acc[s] = mfma16x16x4(a_cur[r], zb[s][t][r], acc[s]);
          a_cur = a_nxt;
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int s = 0; s < S; ++s)
          *reinterpret_cast<f32x4*>(&hstage[((s * WT + o) * 64 + l) * 4]) = acc[s];
      }
    }
    __syncthreads();  // bias (and first-layer) partials of all waves are in LDS
    if (w == 0) {
      const int bo = (i == 0) ? d.d_in * d.width : off_layer(d, i) + d.width * d.width;
      for (int f = l; f < d.width; f += 64)
        gs[bo + f] = ((accBi[f] + accBi[W + f]) + accBi[2 * W + f]) + accBi[3 * W + f];
    }
  }
  {
    const int i = 0;
    // (a) stream adjoints of the pre-activation (zb replaces hb)
    f32x4 zb[S][WT];
    {
      f32x4 zc[S], zn[S];
      z_load<S, WT>(zc, Zs, i, nwg, wg, w, 0, l);
#pragma unroll
      for (int t = 0; t < WT; ++t) {
        if (t + 1 < WT) z_load<S, WT>(zn, Zs, i, nwg, wg, w, t + 1, l);
        f32x4 hh[S], oo[S];
#pragma unroll
        for (int s = 0; s < S; ++s) hh[s] = *reinterpret_cast<const f32x4*>(&hstage[((s * WT + t) * 64 + l) * 4]);
        tanh_jet_bwd<S>(sp, zc, hh, oo);
#pragma unroll
        for (int s = 0; s < S; ++s) zb[s][t] = oo[s];
        if (t + 1 < WT) {
#pragma unroll
          for (int s = 0; s < S; ++s) zc[s] = zn[s];
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // (b) bias gradient partials (value stream only)
    float* accBi = accB + (i & 1) * 4 * W;
#pragma unroll
    for (int t = 0; t < WT; ++t)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * t + 4 * g + c;
        const float v = row16_sum(zb[0][t][c]);
        if (p == 0 && f < d.width) accBi[w * W + f] = v;
      }

    // (e) first layer: dK0[j][f] = sum_p x_j zb_value + sum_{first-order streams on var j} zb_s
    for (int j = 0; j < d.d_in; ++j) {
      const float xj = valid ? X[(size_t)n * d.d_in + j] : 0.f;
#pragma unroll
      for (int t = 0; t < WT; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 16 * t + 4 * g + c;
          float v = xj * zb[0][t][c];
#pragma unroll
          for (int s = 1; s < S; ++s)
            if (sp.stype[s] == 1 && sp.var[s] == j) v += zb[s][t][c];
          v = row16_sum(v);
          if (p == 0 && f < d.width) accK0[w * TDQ_MAXD * W + j * W + f] = v;
        }
    }
    __syncthreads();  // bias (and first-layer) partials of all waves are in LDS
    if (w == 0) {
      const int bo = (i == 0) ? d.d_in * d.width : off_layer(d, i) + d.width * d.width;
      for (int f = l; f < d.width; f += 64)
        gs[bo + f] = ((accBi[f] + accBi[W + f]) + accBi[2 * W + f]) + accBi[3 * W + f];
    }
  }
  // ---- remaining small accumulators --------------------------------------------------------
  if (w == 1) {
    for (int e = l; e < d.d_in * d.width; e += 64) {
      const int j = e / d.width, f = e - j * d.width;
      const int k = j * W + f;
      gs[e] = ((accK0[k] + accK0[TDQ_MAXD * W + k]) + accK0[2 * TDQ_MAXD * W + k]) + accK0[3 * TDQ_MAXD * W + k];
    }
  } else if (w == 2) {
    const int ko = off_layer(d, Lh);
    for (int e = l; e < d.width * d.d_out; e += 64) {
      const int f = e / d.d_out, q = e - f * d.d_out;
      const int k = f * TDQ_MAXO + q, st = W * TDQ_MAXO;
      gs[ko + e] = ((accKo[k] + accKo[st + k]) + accKo[2 * st + k]) + accKo[3 * st + k];
    }
    if (l < d.d_out)
      gs[ko + d.width * d.d_out + l] = ((accBo[l] + accBo[TDQ_MAXO + l]) + accBo[2 * TDQ_MAXO + l]) + accBo[3 * TDQ_MAXO + l];
  }
}

// deterministic slab reduction (fixed summation order): pass 1 sums chunks of workgroups, one
// float4 column per thread with four independent 16-byte loads in flight; pass 2 sums the chunks
template <bool H>
__global__ void __launch_bounds__(256) slab_reduce1(const float* __restrict__ slab, float* __restrict__ part,
                                                    int nwg, int Pst, int chunks) {
  const int q = blockIdx.x * 256 + threadIdx.x;  // float4 column
  if (4 * q >= Pst) return;
  slab_reduce1_body<H>(slab, part, nwg, Pst, chunks, q, blockIdx.y);
}

__global__ void __launch_bounds__(256) slab_reduce2(const float* __restrict__ part, float* __restrict__ grad, int P,
                                                    int Pst, int chunks) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (4 * q >= P) return;
  const f32x4 a = slab_reduce2_sum(part, Pst, chunks, q);
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (4 * q + e < P) grad[4 * q + e] = a[e];
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
namespace {


size_t fwd_lds_bytes(int WT, int S) { return (size_t)4 * S * WT * 256 * sizeof(float); }

size_t bwd_lds_bytes(int WT, int S) {
  const int W = 16 * WT;
  const size_t u1 = 2 * 64 * (size_t)(W + 16), u2 = (size_t)4 * S * WT * 256;
  const size_t floats = (u1 > u2 ? u1 : u2) + 4 * TDQ_MAXD * W + 8 * W + 4 * W * TDQ_MAXO + 4 * TDQ_MAXO;
  return floats * sizeof(float);
}


template <int WT, int S>
int launch_fwd(const float* X, const float* P, const float* Wt, float* J, float* Zs, int N, NetDims d,
               JetSpec sp, hipStream_t st) {
  const int nwg = (N + 63) / 64;
  const size_t lds = fwd_lds_bytes(WT, S);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&jet_fwd_kernel<WT, S>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((jet_fwd_kernel<WT, S>), dim3(nwg), dim3(256), lds, st, X, P, Wt, J, Zs, N, d, sp);
  TDQ_CHECK_LAUNCH();
  return 0;
}

template <int WT, int S>
int launch_bwd(const float* X, const float* P, const float* Kp, const float* dJ, const float* Zs, float* slab,
               int N, int Ptot, NetDims d, JetSpec sp, hipStream_t st) {
  const int nwg = (N + 63) / 64;
  const size_t lds = bwd_lds_bytes(WT, S);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&jet_bwd_kernel<WT, S>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((jet_bwd_kernel<WT, S>), dim3(nwg), dim3(256), lds, st, X, P, Kp, dJ, Zs, slab, N,
                     Ptot, d, sp);
  TDQ_CHECK_LAUNCH();
  return 0;
}

#define TDQ_DISPATCH_S(WT_, FN, ...)                                        \
  switch (S) {                                                              \
    case 1: return FN<WT_, 1>(__VA_ARGS__);                                 \
    case 2: return FN<WT_, 2>(__VA_ARGS__);                                 \
    case 3: return FN<WT_, 3>(__VA_ARGS__);                                 \
    case 4: return FN<WT_, 4>(__VA_ARGS__);                                 \
    default: break;                                                         \
  }                                                                         \
  if (WT_ * 8 <= 32) switch (S) {                                           \
      case 5: return FN<(WT_ <= 4 ? WT_ : 4), 5>(__VA_ARGS__);              \
      case 6: return FN<(WT_ <= 4 ? WT_ : 4), 6>(__VA_ARGS__);              \
      case 7: return FN<(WT_ <= 4 ? WT_ : 4), 7>(__VA_ARGS__);              \
      case 8: return FN<(WT_ <= 4 ? WT_ : 4), 8>(__VA_ARGS__);              \
      default: break;                                                       \
    }                                                                       \
  return (int)hipErrorInvalidValue;

#ifdef TDQ_SINGLE_CONFIG  // resource-usage experiments: instantiate one (WT, S) only
#define TDQ_DISPATCH(FN, ...) return FN<TDQ_SINGLE_WT, TDQ_SINGLE_S>(__VA_ARGS__);
#else
#define TDQ_DISPATCH(FN, ...)                      \
  switch (WT) {                                    \
    case 1: { TDQ_DISPATCH_S(1, FN, __VA_ARGS__) } \
    case 2: { TDQ_DISPATCH_S(2, FN, __VA_ARGS__) } \
    case 4: { TDQ_DISPATCH_S(4, FN, __VA_ARGS__) } \
    case 8: { TDQ_DISPATCH_S(8, FN, __VA_ARGS__) } \
    default: return (int)hipErrorInvalidValue;    \
  }
#endif

int launch_pad(const float* P, float* img, NetDims d, int W, int transposed, hipStream_t st) {
  const int64_t total = (int64_t)(d.n_hidden - 1) * W * W;
  if (total <= 0) return 0;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(pad_weights_kernel, dim3((unsigned)blocks), dim3(256), 0, st, P, img, d, W, transposed);
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" {

// Zs (saved pre-activations) + padded weight image, in floats
int64_t tdq_jet_scratch_floats(int N, int width, int n_hidden, int S, int unused) {
  (void)unused;
  const int WT = width_tiles(width);
  if (WT < 0) return -1;
  const int64_t nwg = (N + 63) / 64;
  const int64_t W = 16 * WT;
  return (int64_t)n_hidden * nwg * S * 4 * WT * 256 + (int64_t)(n_hidden > 1 ? n_hidden - 1 : 0) * W * W;
}

// per-workgroup gradient slabs + reduction partials + padded weight image, in floats
int64_t tdq_jet_slab_floats(int N, int d_in, int width, int d_out, int n_hidden) {
  const int WT = width_tiles(width);
  if (WT < 0) return -1;
  const int nwg = (N + 63) / 64;
  const int64_t P = slab_stride(param_count(d_in, width, d_out, n_hidden));
  const int64_t chunks = slab_chunks(nwg);
  const int64_t W = 16 * WT;
  return (int64_t)nwg * P + chunks * P + (int64_t)(n_hidden > 1 ? n_hidden - 1 : 0) * W * W;
}

int tdq_jet_fwd(const float* X, const float* P, float* J, float* scratch, int N, int d_in, int width,
                int d_out, int n_hidden, int S, const int* spec, void* stream) {
  if (N <= 0) return 0;
  const int WT = width_tiles(width);
  JetSpec sp;
  if (WT < 0 || S * WT > 32 || d_in > TDQ_MAXD || d_out > TDQ_MAXO || n_hidden < 1 || !make_spec(S, spec, sp))
    return (int)hipErrorInvalidValue;
  NetDims d = uniform_dims(d_in, width, d_out, n_hidden);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nwg = (N + 63) / 64;
  float* Zs = scratch;
  float* Wt = scratch + (int64_t)n_hidden * nwg * S * 4 * WT * 256;
  int rc = launch_pad(P, Wt, d, 16 * WT, 1, st);
  if (rc) return rc;
  TDQ_DISPATCH(launch_fwd, X, P, Wt, J, Zs, N, d, sp, st)
}

int tdq_jet_bwd(const float* X, const float* P, const float* dJ, const float* Zs, float* work, float* grad,
                int N, int d_in, int width, int d_out, int n_hidden, int S, const int* spec, void* stream) {
  if (N <= 0) return 0;
  const int WT = width_tiles(width);
  JetSpec sp;
  if (WT < 0 || S * WT > 32 || d_in > TDQ_MAXD || d_out > TDQ_MAXO || n_hidden < 1 || !make_spec(S, spec, sp))
    return (int)hipErrorInvalidValue;
  NetDims d = uniform_dims(d_in, width, d_out, n_hidden);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nwg = (N + 63) / 64;
  const int Ptot = param_count(d_in, width, d_out, n_hidden);
  const int Pst = slab_stride(Ptot);
  const int chunks = slab_chunks(nwg);
  float* slab = work;
  float* part = work + (size_t)nwg * Pst;
  float* Kp = part + (size_t)chunks * Pst;
  int rc = launch_pad(P, Kp, d, 16 * WT, 0, st);
  if (rc) return rc;
  {
    auto run = [&]() -> int { TDQ_DISPATCH(launch_bwd, X, P, Kp, dJ, Zs, slab, N, Pst, d, sp, st) };
    rc = run();
  }
  if (rc) return rc;
  return tdq_slab_reduce(work, grad, nwg, Ptot, chunks, stream);
}

int tdq_slab_reduce(float* work, float* grad, int nwg, int P, int chunks, void* stream) {
  return tdq_slab_reduce_h(work, grad, nwg, P, chunks, 0, stream);
}

int tdq_slab_reduce_h(float* work, float* grad, int nwg, int P, int chunks, int half, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int Pst = slab_stride(P);
  const int nq = Pst / 4;
  float* slab = work;
  float* part = work + (size_t)nwg * Pst;
  dim3 g1((nq + 255) / 256, chunks);
  if (half)
    hipLaunchKernelGGL(slab_reduce1<true>, g1, dim3(256), 0, st, slab, part, nwg, Pst, chunks);
  else
    hipLaunchKernelGGL(slab_reduce1<false>, g1, dim3(256), 0, st, slab, part, nwg, Pst, chunks);
  TDQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(slab_reduce2, dim3((nq + 255) / 256), dim3(256), 0, st, part, grad, P, Pst, chunks);
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
