// Split-bf16 ("bf16x3") Taylor-jet tanh-MLP forward / backward for gfx950 (MI355X, CDNA4).
//
// Same contract as jet_mlp.hip (stream jets J[s][n][q] of a tanh MLP and the flat parameter
// gradient of <dJ, J>), re-tiled for the bf16 matrix cores: on gfx950 the exact-fp32 MFMA runs
// at the fp32 VECTOR rate (64 FLOP/clk/SIMD) while v_mfma_f32_16x16x32_bf16 runs 16x faster.
// Every GEMM operand is split x = hi + lo (two bf16, |x - hi - lo| <= 2^-17 |x|) and a product
// is formed as ah*bh + ah*bl + al*bh with fp32 accumulation: 3 bf16 MFMAs per fp32-equivalent
// product (5.3x the fp32-MFMA rate) at ~2^-16 relative error per product (the dropped al*bl
// term), i.e. ~19 significant bits instead of bf16's 8.
//
// Layout (16x16x32 MFMA: lane l = (p = l&15, g = l>>4); A[p][8g+j], B[8g+j][p], D[4g+r][p]):
//   * one workgroup = 4 waves x 16 points, one point per lane column, features in registers;
//   * k-block kb of a layer covers features 32kb..32kb+31 in the PERMUTED order
//       k = 8g + j  <->  feature 32kb + (j < 4 ? 4g + j : 16 + 4g + j - 4)
//     so the fp32 accumulator tiles 2kb and 2kb+1 (lane holds rows 4g..4g+3 of each) ARE the
//     B fragment of k-block kb after a hi/lo split - no lane movement between layers;
//   * weights are pre-split into hi/lo A-fragment images in that permuted k order
//     (pack_bf3_kernel: 16 B per lane per (layer, out tile, k-block)), streamed from L2 with a
//     4-step register prefetch ring;
//   * the forward saves the POST-activation streams h (fp32).  The backward needs no tanh
//     recompute: with s1 = 1 - h^2 and s2 z_a = -2 h h_a the adjoint of the tanh jet is
//       zb_ab = s1 hb_ab
//       zb_a  = s1 hb_a - 2 h sum_{(a,b)} h_b hb_ab          (one-hot over the pair factors)
//       zb    = s1 hb - 2 h sum_{s>0} h_s hb_s - 2 sum_{(a,b)} h_a h_b hb_ab
//   * dK = sum_points sum_streams h_prev zb^T reduces over POINTS: both operands go through
//     [point][feature] bf16 LDS images read back transposed with ds_read_b64_tr_b16, so points
//     land on the MFMA k index (8 consecutive points per lane).
// Reference behaviour: the nested tf.gradients of the PDE residual (SURVEY.md §2.2 K2-K8,
// tensordiffeq/models.py:update_loss / utils.py:get_tf_model); see jet_mlp.hip for the fp32 twin.
#include "jet_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// c += a * b  with a ~ ah + al, b ~ bh + bl  (al*bl dropped)
__device__ __forceinline__ f32x4 mfma3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 c) {
  c = mfma_bf(al, bh, c);
  c = mfma_bf(ah, bl, c);
  return mfma_bf(ah, bh, c);
}

__device__ __forceinline__ void split4(const f32x4 v, bf16x4& hi, bf16x4& lo) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const __bf16 h = (__bf16)v[c];
    hi[c] = h;
    lo[c] = (__bf16)(v[c] - (float)h);
  }
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x4 half8(bf16x8 v, int hi_half) {
  return hi_half ? __builtin_shufflevector(v, v, 4, 5, 6, 7) : __builtin_shufflevector(v, v, 0, 1, 2, 3);
}

// transposed LDS read (T10): lane 4q+c of each 16-lane group addresses row q, columns 4c..4c+3
// of a 4 x 16 block; lane i of the group receives column i, rows 0..3.
__device__ __forceinline__ bf16x4 tr_read(const __bf16* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// tanh(z) and s1 = 1 - tanh(z)^2 without cancellation: e = exp(-2|z|),
//   tanh|z| = (1 - e) / (1 + e)  (odd Taylor polynomial below 1/8),  s1 = 4 e / (1 + e)^2
__device__ __forceinline__ void tanh_s1(float z, float& h, float& s1) {
  const float az = fabsf(z);
  const float e = __builtin_amdgcn_exp2f(-2.8853900817779268f * az);
  const float r = __builtin_amdgcn_rcpf(1.f + e);
  const float z2 = az * az;
  const float poly = az * fmaf(z2, fmaf(z2, fmaf(z2, -0.053968254f, 0.13333334f), -0.33333334f), 1.f);
  const float t = az < 0.125f ? poly : (1.f - e) * r;
  h = __builtin_copysignf(t, z);
  s1 = 4.f * e * (r * r);
}

template <int S>
__device__ __forceinline__ f32x4 pick1(const f32x4 (&v)[S], const float (&sel)[TDQ_MAXS]) {
  f32x4 r = zero4();
#pragma unroll
  for (int q = 1; q < S; ++q) r += sel[q] * v[q];
  return r;
}

// forward tanh jet of one feature tile: z -> h
template <int S>
__device__ __forceinline__ void tanh_jet_f(const JetSpec& sp, const f32x4 (&z)[S], f32x4 (&h)[S]) {
  f32x4 za[S], zb[S];
#pragma unroll
  for (int s = 1; s < S; ++s) {
    za[s] = sp.stype[s] == 2 ? pick1<S>(z, sp.selA[s]) : zero4();
    zb[s] = sp.stype[s] == 2 ? pick1<S>(z, sp.selB[s]) : zero4();
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float hv, s1;
    tanh_s1(z[0][c], hv, s1);
    const float s2 = -2.f * hv * s1;
    h[0][c] = hv;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      float v = s1 * z[s][c];
      if (sp.stype[s] == 2) v = fmaf(s2 * za[s][c], zb[s][c], v);
      h[s][c] = v;
    }
  }
}

// backward tanh jet of one feature tile from the saved post-activations h: hb -> zb
template <int S>
__device__ __forceinline__ void tanh_jet_b(const JetSpec& sp, const f32x4 (&h)[S], const f32x4 (&hb)[S],
                                           f32x4 (&zb)[S]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float hv = h[0][c];
    const float s1 = fmaf(-hv, hv, 1.f);
    const float m2h = -2.f * hv;
    float zbv[S];
    float sb1 = 0.f, sb2 = 0.f;
    zbv[0] = s1 * hb[0][c];
#pragma unroll
    for (int s = 1; s < S; ++s) {
      zbv[s] = s1 * hb[s][c];
      sb1 = fmaf(h[s][c], hb[s][c], sb1);
    }
#pragma unroll
    for (int s = 1; s < S; ++s) {
      if (sp.stype[s] == 2) {
        float ha = 0.f, hq = 0.f;
#pragma unroll
        for (int q = 1; q < S; ++q) {
          ha = fmaf(sp.selA[s][q], h[q][c], ha);
          hq = fmaf(sp.selB[s][q], h[q][c], hq);
        }
        const float hbs = hb[s][c];
        sb2 = fmaf(ha * hq, hbs, sb2);
        const float ga = m2h * hq * hbs, gb = m2h * ha * hbs;
#pragma unroll
        for (int q = 1; q < S; ++q) zbv[q] = fmaf(sp.selA[s][q], ga, fmaf(sp.selB[s][q], gb, zbv[q]));
      }
    }
    zbv[0] = fmaf(m2h, sb1, fmaf(-2.f, sb2, zbv[0]));
#pragma unroll
    for (int s = 0; s < S; ++s) zb[s][c] = zbv[s];
  }
}

// ------------------------------------------------------------------------------------------
// A-operand images: img[layer-1][o][kb][hl][lane] = 8 bf16 (hl 0 = hi, 1 = lo)
//   element j of lane (p, g): row 16o + p, k = 8g + j -> feature 32kb + (j<4 ? 4g+j : 16+4g+j-4)
//   transposed = 1 (forward):  A[row = out][k = in]  ;  0 (backward): A[row = in][k = out]
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) pack_bf3_kernel(const float* __restrict__ P, bf16x8* __restrict__ img,
                                                       NetDims d, int WT, int transposed) {
  const int KB = WT / 2;
  const int total = (d.n_hidden - 1) * WT * KB * 64;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int lane = e & 63, frag = e >> 6;
    const int kb = frag % KB, o = (frag / KB) % WT, layer = frag / (KB * WT) + 1;
    const int p = lane & 15, g = lane >> 4, row = 16 * o + p;
    const float* K = P + off_layer(d, layer);
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kf = 32 * kb + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4);
      const int in = transposed ? kf : row, out = transposed ? row : kf;
      const float v = (in < d.width && out < d.width) ? K[in * d.width + out] : 0.f;
      const __bf16 h = (__bf16)v;
      hi[j] = h;
      lo[j] = (__bf16)(v - (float)h);
    }
    img[(size_t)(frag * 2) * 64 + lane] = hi;
    img[(size_t)(frag * 2 + 1) * 64 + lane] = lo;
  }
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
template <int WT, int S>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
jet_fwd_bf3_kernel(const float* __restrict__ X, const float* __restrict__ P, const bf16x8* __restrict__ Wimg,
                   float* __restrict__ J, float* __restrict__ Hs, int N, NetDims d, JetSpec sp) {
  constexpr int KB = WT / 2;
  constexpr int NSTEP = WT * KB;
  constexpr int D = NSTEP < 4 ? NSTEP : 4;  // weight-fragment prefetch ring (steps)
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int n = wg * 64 + w * 16 + p;
  const bool valid = n < N;
  const int Lh = d.n_hidden;
  // wave-private staging image of the next layer's B fragments: [s][kb][hl][lane][2 halves]
  bf16x4* stage = reinterpret_cast<bf16x4*>(lds_raw) + (size_t)w * (S * KB * 2 * 64 * 2);
  const float* Ko = P + off_layer(d, Lh);

  float x[TDQ_MAXD];
#pragma unroll
  for (int j = 0; j < TDQ_MAXD; ++j) x[j] = (j < d.d_in && valid) ? X[(size_t)n * d.d_in + j] : 0.f;

  bf16x8 ah[S][KB], al[S][KB];
  float* hlast = reinterpret_cast<float*>(stage);  // last layer: fp32 h image [s][t][lane][4]

  // ---- layer 0 (input -> width) on VALU: derivative streams are columns of K0 -------------
  {
    const float* K0 = P;
    const float* b0 = P + d.d_in * d.width;
    const bool last = Lh == 1;
    bf16x4 ph[S], pl[S];
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      f32x4 z[S], h[S];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * t + 4 * g + c;
        const bool fv = f < d.width;
        float z0 = fv ? b0[f] : 0.f;
#pragma unroll
        for (int j = 0; j < TDQ_MAXD; ++j)
          if (j < d.d_in) z0 = fmaf(x[j], fv ? K0[j * d.width + f] : 0.f, z0);
        z[0][c] = z0;
#pragma unroll
        for (int s = 1; s < S; ++s) z[s][c] = (sp.stype[s] == 1 && fv) ? K0[sp.var[s] * d.width + f] : 0.f;
      }
      tanh_jet_f<S>(sp, z, h);
#pragma unroll
      for (int s = 0; s < S; ++s) *reinterpret_cast<f32x4*>(Hs + zs_index(0, nwg, wg, S, s, w, WT, t, l)) = h[s];
      if (last) {
#pragma unroll
        for (int s = 0; s < S; ++s) *reinterpret_cast<f32x4*>(&hlast[((s * WT + t) * 64 + l) * 4]) = h[s];
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          bf16x4 hi, lo;
          split4(h[s], hi, lo);
          if (t & 1) {
            ah[s][t >> 1] = cat8(ph[s], hi);
            al[s][t >> 1] = cat8(pl[s], lo);
          } else {
            ph[s] = hi;
            pl[s] = lo;
          }
        }
      }
    }
  }

  // ---- hidden layers on bf16x3 MFMA --------------------------------------------------------
  for (int i = 1; i < Lh; ++i) {
    const bf16x8* Wi = Wimg + (size_t)(i - 1) * NSTEP * 128 + l;
    const float* b = P + off_layer(d, i) + d.width * d.width;
    const bool last = i == Lh - 1;
    bf16x8 wh[D], wl[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      wh[k] = Wi[k * 128];
      wl[k] = Wi[k * 128 + 64];
    }
#pragma unroll
    for (int o = 0; o < WT; ++o) {
      f32x4 acc[S];
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] = zero4();
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int st = o * KB + kb;
        const bf16x8 Ah = wh[st % D], Al = wl[st % D];
        if (st + D < NSTEP) {
          wh[st % D] = Wi[(st + D) * 128];
          wl[st % D] = Wi[(st + D) * 128 + 64];
        }
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s] = mfma3(Ah, Al, ah[s][kb], al[s][kb], acc[s]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * o + 4 * g + c;
        acc[0][c] += (f < d.width) ? b[f] : 0.f;
      }
      f32x4 h[S];
      tanh_jet_f<S>(sp, acc, h);
#pragma unroll
      for (int s = 0; s < S; ++s) *reinterpret_cast<f32x4*>(Hs + zs_index(i, nwg, wg, S, s, w, WT, o, l)) = h[s];
      if (last) {
#pragma unroll
        for (int s = 0; s < S; ++s) *reinterpret_cast<f32x4*>(&hlast[((s * WT + o) * 64 + l) * 4]) = h[s];
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          bf16x4 hi, lo;
          split4(h[s], hi, lo);
          stage[(((s * KB + (o >> 1)) * 2 + 0) * 64 + l) * 2 + (o & 1)] = hi;
          stage[(((s * KB + (o >> 1)) * 2 + 1) * 64 + l) * 2 + (o & 1)] = lo;
        }
      }
    }
    if (!last) {  // wave-private region: program order suffices
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          ah[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[(((s * KB + kb) * 2 + 0) * 64 + l) * 2]);
          al[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[(((s * KB + kb) * 2 + 1) * 64 + l) * 2]);
        }
    }
  }

  // ---- output layer (width -> d_out): VALU dot over the staged fp32 h + cross-lane sum ----
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
      for (int t = 0; t < WT; ++t) {
        const f32x4 h = *reinterpret_cast<const f32x4*>(&hlast[((s * WT + t) * 64 + l) * 4]);
#pragma unroll
        for (int c = 0; c < 4; ++c) v = fmaf(h[c], kq[t][c], v);
      }
      v = col4_sum(v);
      if (s == 0) v += bo[q];
      if (g == 0 && valid) J[((size_t)s * N + n) * d.d_out + q] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
template <int S, int WT>
__device__ __forceinline__ void h_tile(f32x4 (&h)[S], const float* __restrict__ Hs, int layer, int nwg, int wg,
                                       int w, int t, int lane) {
#pragma unroll
  for (int s = 0; s < S; ++s) h[s] = *reinterpret_cast<const f32x4*>(Hs + zs_index(layer, nwg, wg, S, s, w, WT, t, lane));
}

template <int WT, int S>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
jet_bwd_bf3_kernel(const float* __restrict__ X, const float* __restrict__ P, const bf16x8* __restrict__ Kimg,
                   const float* __restrict__ dJ, const float* __restrict__ Hs, float* __restrict__ slab, int N,
                   int Ptot, NetDims d, JetSpec sp) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int W = 16 * WT;
  constexpr int KB = WT / 2;
  constexpr int NSTEP = WT * KB;
  constexpr int D = NSTEP < 4 ? NSTEP : 4;
  // [point][feature] bf16 images (h hi/lo, zb hi/lo).  Row stride 144 bf16 = 72 words (= 8 mod 64)
  // and the 64-column XOR on bit 3 of the row put the 8 rows of a transposed read's 32-lane half
  // (4 rows x 2 groups 8 rows apart, 8 words each) on 8 disjoint bank windows: conflict-free.
  constexpr int RS = 144;
  constexpr int IMG = 64 * RS;
  // dK tile ownership: WT >= 4 -> wave w owns tile rows {w, w+4, ..} x all columns;
  // WT = 2 -> one tile (w>>1, w&1) per wave
  constexpr int NR = WT >= 4 ? WT / 4 : 1;
  constexpr int NC = WT >= 4 ? WT : 1;
  constexpr int U1 = (4 * IMG) / 2;           // images, in floats
  constexpr int U2 = 4 * S * WT * 256;        // per-wave hb staging (fp32)
  constexpr int U = ((U1 > U2 ? U1 : U2) + 3) / 4 * 4;
  __bf16* img = reinterpret_cast<__bf16*>(lds);
  float* accK0 = lds + U;                     // [4][TDQ_MAXD * W]
  float* accB = accK0 + 4 * TDQ_MAXD * W;     // [2 (layer parity)][4][W]
  float* accKo = accB + 8 * W;                // [4][W * TDQ_MAXO]
  float* accBo = accKo + 4 * W * TDQ_MAXO;    // [4][TDQ_MAXO]

  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = blockIdx.x, nwg = gridDim.x;
  const int n = wg * 64 + w * 16 + p;
  const bool valid = n < N;
  const int Lh = d.n_hidden;
  float* gs = slab + (size_t)wg * Ptot;
  float* hstage = lds + (size_t)w * (S * WT * 256);
  auto dw_row = [](int wv, int r) { return WT >= 4 ? wv + 4 * r : (wv >> 1); };
  auto dw_col = [](int wv, int c) { return WT >= 4 ? c : (wv & 1); };
  // transposed-read lane address inside a 4 x 16 block: row (l & 15) >> 2, column 4 (l & 3)
  const int tr_row = 8 * g + ((l & 15) >> 2), tr_col = 4 * (l & 3);
  const int swz = (g & 1) << 6;  // bit 3 of every row this lane's transposed reads touch

  // ---- output layer: hb = Ko ub ; dKo += h_last ub ; dbo += ub_value ----------------------
  {
    float ub[S][TDQ_MAXO];
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q)
#pragma unroll
      for (int s = 0; s < S; ++s) ub[s][q] = (q < d.d_out && valid) ? dJ[((size_t)s * N + n) * d.d_out + q] : 0.f;
    const float* Ko = P + off_layer(d, Lh);
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      f32x4 h[S];
      h_tile<S, WT>(h, Hs, Lh - 1, nwg, wg, w, t, l);
      f32x4 hbt[S];
#pragma unroll
      for (int s = 0; s < S; ++s) hbt[s] = zero4();
#pragma unroll
      for (int q = 0; q < TDQ_MAXO; ++q) {
        if (q >= d.d_out) break;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 16 * t + 4 * g + c;
          const bool fv = f < d.width;
          const float kq = fv ? Ko[f * d.d_out + q] : 0.f;
          float part = 0.f;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            hbt[s][c] = fmaf(kq, ub[s][q], hbt[s][c]);
            part = fmaf(h[s][c], ub[s][q], part);
          }
          part = row16_sum(part);
          if (p == 0 && fv) accKo[w * W * TDQ_MAXO + f * TDQ_MAXO + q] = part;
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) *reinterpret_cast<f32x4*>(&hstage[((s * WT + t) * 64 + l) * 4]) = hbt[s];
    }
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q) {
      if (q >= d.d_out) break;
      const float v = row16_sum(ub[0][q]);
      if (l == 0) accBo[w * TDQ_MAXO + q] = v;
    }
  }

  // ---- hidden layers i = Lh-1 .. 1 ---------------------------------------------------------
  for (int i = Lh - 1; i >= 1; --i) {
    // (a) stream adjoints of the pre-activation, split into B fragments; (b) bias partials
    bf16x8 zh[S][KB], zl[S][KB];
    float* accBi = accB + (i & 1) * 4 * W;
    {
      bf16x4 ph[S], pl[S];
#pragma unroll
      for (int t = 0; t < WT; ++t) {
        f32x4 h[S], hb[S], zb[S];
        h_tile<S, WT>(h, Hs, i, nwg, wg, w, t, l);
#pragma unroll
        for (int s = 0; s < S; ++s) hb[s] = *reinterpret_cast<const f32x4*>(&hstage[((s * WT + t) * 64 + l) * 4]);
        tanh_jet_b<S>(sp, h, hb, zb);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 16 * t + 4 * g + c;
          const float v = row16_sum(zb[0][c]);
          if (p == 0 && f < d.width) accBi[w * W + f] = v;
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
          bf16x4 hi, lo;
          split4(zb[s], hi, lo);
          if (t & 1) {
            zh[s][t >> 1] = cat8(ph[s], hi);
            zl[s][t >> 1] = cat8(pl[s], lo);
          } else {
            ph[s] = hi;
            pl[s] = lo;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // (c) dK_i = sum_points sum_streams h_{i-1} zb^T on bf16x3 MFMA, points on the k index
    f32x4 dw[NR][NC];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) dw[r][c] = zero4();
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
      __syncthreads();  // previous readers of the region (hb staging / last stream's images) done
      {
        const int row = 16 * w + p;
#pragma unroll
        for (int t = 0; t < WT; ++t) {
          const f32x4 hp = *reinterpret_cast<const f32x4*>(Hs + zs_index(i - 1, nwg, wg, S, s, w, WT, t, l));
          bf16x4 hi, lo;
          split4(hp, hi, lo);
          const int off = row * RS + ((16 * t + 4 * g) ^ (((row >> 3) & 1) << 6));
          *reinterpret_cast<bf16x4*>(img + off) = hi;
          *reinterpret_cast<bf16x4*>(img + IMG + off) = lo;
          bf16x8 zhs = zh[0][0], zls = zl[0][0];
#pragma unroll
          for (int q = 0; q < S; ++q)
            if (q == s) {
              zhs = zh[q][t >> 1];
              zls = zl[q][t >> 1];
            }
          *reinterpret_cast<bf16x4*>(img + 2 * IMG + off) = half8(zhs, t & 1);
          *reinterpret_cast<bf16x4*>(img + 3 * IMG + off) = half8(zls, t & 1);
        }
      }
      __syncthreads();
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {  // 64 points = 2 k-blocks of 32
        bf16x8 Ah[NR], Al[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int off = (32 * kb + tr_row) * RS + ((16 * dw_row(w, r) + tr_col) ^ swz);
          Ah[r] = cat8(tr_read(img + off), tr_read(img + off + 4 * RS));
          Al[r] = cat8(tr_read(img + IMG + off), tr_read(img + IMG + off + 4 * RS));
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int off = (32 * kb + tr_row) * RS + ((16 * dw_col(w, c) + tr_col) ^ swz);
          const bf16x8 Bh = cat8(tr_read(img + 2 * IMG + off), tr_read(img + 2 * IMG + off + 4 * RS));
          const bf16x8 Bl = cat8(tr_read(img + 3 * IMG + off), tr_read(img + 3 * IMG + off + 4 * RS));
#pragma unroll
          for (int r = 0; r < NR; ++r) dw[r][c] = mfma3(Ah[r], Al[r], Bh, Bl, dw[r][c]);
        }
      }
    }
    {
      const int ko = off_layer(d, i);
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c2 = 0; c2 < NC; ++c2) {
          const int out = 16 * dw_col(w, c2) + p;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int in = 16 * dw_row(w, r) + 4 * g + c;
            if (in < d.width && out < d.width) gs[ko + in * d.width + out] = dw[r][c2][c];
          }
        }
    }
    __syncthreads();  // images consumed: the region becomes hb staging again

    // (d) hb_{i-1} = K_i zb on bf16x3 MFMA (A = [in][out] image, B = zb fragments)
    {
      const bf16x8* Ki = Kimg + (size_t)(i - 1) * NSTEP * 128 + l;
      bf16x8 wh[D], wl[D];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        wh[k] = Ki[k * 128];
        wl[k] = Ki[k * 128 + 64];
      }
#pragma unroll
      for (int o = 0; o < WT; ++o) {
        f32x4 acc[S];
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s] = zero4();
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          const int st = o * KB + kb;
          const bf16x8 Ah = wh[st % D], Al = wl[st % D];
          if (st + D < NSTEP) {
            wh[st % D] = Ki[(st + D) * 128];
            wl[st % D] = Ki[(st + D) * 128 + 64];
          }
#pragma unroll
          for (int s = 0; s < S; ++s) acc[s] = mfma3(Ah, Al, zh[s][kb], zl[s][kb], acc[s]);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int s = 0; s < S; ++s) *reinterpret_cast<f32x4*>(&hstage[((s * WT + o) * 64 + l) * 4]) = acc[s];
      }
    }
    __syncthreads();  // bias partials of all waves are in LDS
    if (w == 0) {
      const int bo = off_layer(d, i) + d.width * d.width;
      for (int f = l; f < d.width; f += 64)
        gs[bo + f] = ((accBi[f] + accBi[W + f]) + accBi[2 * W + f]) + accBi[3 * W + f];
    }
  }

  // ---- first layer (i = 0): bias + dK0[j][f] = sum_p x_j zb + sum_{first-order on var j} zb_s
  {
    float* accBi = accB;
    f32x4 zb0[S][WT];
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      f32x4 h[S], hb[S], zb[S];
      h_tile<S, WT>(h, Hs, 0, nwg, wg, w, t, l);
#pragma unroll
      for (int s = 0; s < S; ++s) hb[s] = *reinterpret_cast<const f32x4*>(&hstage[((s * WT + t) * 64 + l) * 4]);
      tanh_jet_b<S>(sp, h, hb, zb);
#pragma unroll
      for (int s = 0; s < S; ++s) zb0[s][t] = zb[s];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * t + 4 * g + c;
        const float v = row16_sum(zb[0][c]);
        if (p == 0 && f < d.width) accBi[w * W + f] = v;
      }
    }
    for (int j = 0; j < d.d_in; ++j) {
      const float xj = valid ? X[(size_t)n * d.d_in + j] : 0.f;
#pragma unroll
      for (int t = 0; t < WT; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 16 * t + 4 * g + c;
          float v = xj * zb0[0][t][c];
#pragma unroll
          for (int s = 1; s < S; ++s)
            if (sp.stype[s] == 1 && sp.var[s] == j) v += zb0[s][t][c];
          v = row16_sum(v);
          if (p == 0 && f < d.width) accK0[w * TDQ_MAXD * W + j * W + f] = v;
        }
    }
    __syncthreads();
    if (w == 0) {
      const int bo = d.d_in * d.width;
      for (int f = l; f < d.width; f += 64)
        gs[bo + f] = ((accBi[f] + accBi[W + f]) + accBi[2 * W + f]) + accBi[3 * W + f];
    } else if (w == 1) {
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
        gs[ko + d.width * d.d_out + l] =
            ((accBo[l] + accBo[TDQ_MAXO + l]) + accBo[2 * TDQ_MAXO + l]) + accBo[3 * TDQ_MAXO + l];
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
namespace {

size_t fwd_bf3_lds(int WT, int S) { return (size_t)4 * S * WT * 1024; }

size_t bwd_bf3_lds(int WT, int S) {
  const int W = 16 * WT;
  const size_t u1 = (size_t)(4 * 64 * 144) / 2, u2 = (size_t)4 * S * WT * 256;
  const size_t u = ((u1 > u2 ? u1 : u2) + 3) / 4 * 4;
  return (u + 4 * TDQ_MAXD * W + 8 * W + 4 * W * TDQ_MAXO + 4 * TDQ_MAXO) * sizeof(float);
}

int64_t img_floats(int WT, int n_hidden) {  // hi/lo A images, in floats
  return (int64_t)(n_hidden > 1 ? n_hidden - 1 : 0) * WT * (WT / 2) * 128 * 4;
}

template <int WT, int S>
int launch_fwd_bf3(const float* X, const float* P, const bf16x8* Wimg, float* J, float* Hs, int N, NetDims d,
                   JetSpec sp, hipStream_t st) {
  const int nwg = (N + 63) / 64;
  const size_t lds = fwd_bf3_lds(WT, S);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&jet_fwd_bf3_kernel<WT, S>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((jet_fwd_bf3_kernel<WT, S>), dim3(nwg), dim3(256), lds, st, X, P, Wimg, J, Hs, N, d, sp);
  TDQ_CHECK_LAUNCH();
  return 0;
}

template <int WT, int S>
int launch_bwd_bf3(const float* X, const float* P, const bf16x8* Kimg, const float* dJ, const float* Hs,
                   float* slab, int N, int Ptot, NetDims d, JetSpec sp, hipStream_t st) {
  const int nwg = (N + 63) / 64;
  const size_t lds = bwd_bf3_lds(WT, S);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&jet_bwd_bf3_kernel<WT, S>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((jet_bwd_bf3_kernel<WT, S>), dim3(nwg), dim3(256), lds, st, X, P, Kimg, dJ, Hs, slab, N,
                     Ptot, d, sp);
  TDQ_CHECK_LAUNCH();
  return 0;
}

#define TDQ_BF3_DISPATCH_S(WT_, FN, ...)                                    \
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

#ifdef TDQ_SINGLE_CONFIG
#define TDQ_BF3_DISPATCH(FN, ...) return FN<TDQ_SINGLE_WT, TDQ_SINGLE_S>(__VA_ARGS__);
#else
#define TDQ_BF3_DISPATCH(FN, ...)                      \
  switch (WT) {                                        \
    case 2: { TDQ_BF3_DISPATCH_S(2, FN, __VA_ARGS__) } \
    case 4: { TDQ_BF3_DISPATCH_S(4, FN, __VA_ARGS__) } \
    case 8: { TDQ_BF3_DISPATCH_S(8, FN, __VA_ARGS__) } \
    default: return (int)hipErrorInvalidValue;        \
  }
#endif

int launch_pack(const float* P, bf16x8* img, NetDims d, int WT, int transposed, hipStream_t st) {
  const int total = (d.n_hidden - 1) * WT * (WT / 2) * 64;
  if (total <= 0) return 0;
  int blocks = (total + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(pack_bf3_kernel, dim3(blocks), dim3(256), 0, st, P, img, d, WT, transposed);
  TDQ_CHECK_LAUNCH();
  return 0;
}

bool bf3_ok(int WT, int S, int d_in, int d_out, int n_hidden) {
  return (WT == 2 || WT == 4 || WT == 8) && S * WT <= 32 && d_in <= TDQ_MAXD && d_out <= TDQ_MAXO && n_hidden >= 1;
}

}  // namespace

extern "C" {

// saved post-activations Hs + forward A image, in floats (-1: configuration unsupported)
int64_t tdq_jet_bf3_scratch_floats(int N, int width, int n_hidden, int S) {
  const int WT = width_tiles(width);
  if (WT < 2) return -1;
  const int64_t nwg = (N + 63) / 64;
  return (int64_t)n_hidden * nwg * S * 4 * WT * 256 + img_floats(WT, n_hidden);
}

// per-workgroup gradient slabs + reduction partials + backward A image, in floats
int64_t tdq_jet_bf3_slab_floats(int N, int d_in, int width, int d_out, int n_hidden) {
  const int WT = width_tiles(width);
  if (WT < 2) return -1;
  const int64_t nwg = (N + 63) / 64;
  const int64_t P = param_count(d_in, width, d_out, n_hidden);
  const int64_t chunks = nwg < 32 ? nwg : 32;
  return (nwg * P + chunks * P + 3) / 4 * 4 + img_floats(WT, n_hidden);
}

int tdq_jet_fwd_bf3(const float* X, const float* P, float* J, float* scratch, int N, int d_in, int width,
                    int d_out, int n_hidden, int S, const int* spec, void* stream) {
  if (N <= 0) return 0;
  const int WT = width_tiles(width);
  JetSpec sp;
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || !make_spec(S, spec, sp)) return (int)hipErrorInvalidValue;
  NetDims d{d_in, width, d_out, n_hidden};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nwg = (N + 63) / 64;
  float* Hs = scratch;
  bf16x8* Wimg = reinterpret_cast<bf16x8*>(scratch + (int64_t)n_hidden * nwg * S * 4 * WT * 256);
  int rc = launch_pack(P, Wimg, d, WT, 1, st);
  if (rc) return rc;
  TDQ_BF3_DISPATCH(launch_fwd_bf3, X, P, Wimg, J, Hs, N, d, sp, st)
}

int tdq_jet_bwd_bf3(const float* X, const float* P, const float* dJ, const float* Hs, float* work, float* grad,
                    int N, int d_in, int width, int d_out, int n_hidden, int S, const int* spec, void* stream) {
  if (N <= 0) return 0;
  const int WT = width_tiles(width);
  JetSpec sp;
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || !make_spec(S, spec, sp)) return (int)hipErrorInvalidValue;
  NetDims d{d_in, width, d_out, n_hidden};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nwg = (N + 63) / 64;
  const int Ptot = param_count(d_in, width, d_out, n_hidden);
  const int chunks = nwg < 32 ? nwg : 32;
  float* slab = work;
  float* part = work + (size_t)nwg * Ptot;
  bf16x8* Kimg = reinterpret_cast<bf16x8*>(work + ((size_t)nwg * Ptot + (size_t)chunks * Ptot + 3) / 4 * 4);
  int rc = launch_pack(P, Kimg, d, WT, 0, st);
  if (rc) return rc;
  {
    auto run = [&]() -> int { TDQ_BF3_DISPATCH(launch_bwd_bf3, X, P, Kimg, dJ, Hs, slab, N, Ptot, d, sp, st) };
    rc = run();
  }
  if (rc) return rc;
  return tdq_slab_reduce(work, grad, nwg, Ptot, chunks, stream);
}

}  // extern "C"
