// Split-bf16 ("bf16x3") Taylor-jet tanh-MLP forward / backward kernels for gfx950 (MI355X, CDNA4).
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
//     4-step register prefetch ring; biases / first and last layer come from a zero-padded
//     fp32 "aux" image so that no load in a kernel needs a bounds guard (no exec branches);
//   * streams are in JetPlan's canonical order - value, S1 first-order, NSO second-order - and
//     NSO is a template parameter: the jet epilogues are branch-free straight-line code, the
//     two first-order factors of a second-order stream are picked by uniform-index selects;
//   * forward: the epilogue of output tile o-1 (bias, tanh jet, save, hi/lo split, stage) is
//     issued in the same scheduling region as the MFMAs of tile o (double-buffered
//     accumulators), so VALU work fills the MFMA shadow; it saves the POST-activation streams
//     h (fp32).  The backward needs no tanh recompute: with s1 = 1 - h^2 and s2 z_a = -2 h h_a
//       zb_ab = s1 hb_ab
//       zb_a  = s1 hb_a - 2 h sum_{(a,b)} h_b hb_ab
//       zb    = s1 hb - 2 h sum_{s>0} h_s hb_s - 2 sum_{(a,b)} h_a h_b hb_ab
//   * dK = sum_points sum_streams h_prev zb^T reduces over POINTS: both operands go through
//     [point][feature] bf16 LDS images read back transposed with ds_read_b64_tr_b16, so points
//     land on the MFMA k index (8 consecutive points per lane); the next stream's h_prev tiles
//     are in flight from HBM while the current stream's MFMAs run.
// Reference behaviour: the nested tf.gradients of the PDE residual (SURVEY.md §2.2 K2-K8,
// tensordiffeq/models.py:update_loss / utils.py:get_tf_model); jet_mlp.hip is the fp32 twin.
#pragma once
#include "jet_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// Optional per-phase timestamps (build with -DTDQ_PHASE_TIMING, tools/phase_timing.py): lane 0
// of every wave stores s_memtime at numbered points into tdq_ts[(wg * 4 + wave) * 64 + k].
#ifdef TDQ_PHASE_TIMING
#ifdef __HIPCC_RTC__
extern "C" {
__device__ unsigned long long* tdq_ts;  // run-time compiled kernels: set through hipModuleGetGlobal
}
#else
static __device__ unsigned long long* tdq_ts;  // per translation unit (no -fgpu-rdc)
#endif
#define TDQ_TS(k)                                                                                 \
  do {                                                                                            \
    if ((threadIdx.x & 63) == 0)                                                                  \
      tdq_ts[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define TDQ_TS(k) \
  do {            \
  } while (0)
#endif

// aux image (fp32, zero padded to W = 16 WT features; TDQ_MAXO output columns):
//   K0 [d_in][W] | b0 [W] | b_1..b_{Lh-1} [Lh-1][W] | Ko [W][4] | bo [4]
__host__ __device__ inline int aux_b0(const NetDims& d, int W) { return d.d_in * W; }
__host__ __device__ inline int aux_bh(const NetDims& d, int W) { return (d.d_in + 1) * W; }
__host__ __device__ inline int aux_ko(const NetDims& d, int W) { return (d.d_in + d.n_hidden) * W; }
__host__ __device__ inline int aux_bo(const NetDims& d, int W) { return (d.d_in + d.n_hidden + 4) * W; }
__host__ __device__ inline int aux_floats(const NetDims& d, int W) { return (d.d_in + d.n_hidden + 4) * W + 4; }

__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// c += a * b  with a ~ ah + al, b ~ bh + bl  (al*bl dropped)
__device__ __forceinline__ f32x4 mfma3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 c) {
  c = mfma_bf(al, bh, c);
  c = mfma_bf(ah, bl, c);
  return mfma_bf(ah, bh, c);
}

// weight x activation products.  LO (precision "bf16x3"): both operands split hi + lo, 3 MFMAs
// per product.  !LO (precision "bf16"): weights and activations rounded to bf16 once, 1 MFMA: the
// kernels then run a consistently bf16-rounded network (fp32 master weights, fp32 accumulation and
// tanh jets), with half the activation fragments / staging / images - which is what lets two
// workgroups share a CU.
template <bool LO>
__device__ __forceinline__ f32x4 mfma_w(bf16x8 ah, bf16x8 al, const bf16x8& bh, const bf16x8& bl, f32x4 c) {
  if constexpr (LO) {
    c = mfma_bf(al, bh, c);
    c = mfma_bf(ah, bl, c);
  }
  return mfma_bf(ah, bh, c);
}
// dK products: both operands are activations (saved h, adjoint zb)
template <bool LO>
__device__ __forceinline__ f32x4 mfma_aa(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                         f32x4 c) {
  if constexpr (LO) return mfma3(ah, al, bh, bl, c);
  return mfma_bf(ah, bh, c);
}

// "Wide" plans: streams x width tiles > 32 (e.g. a 2-D Laplacian at width 128: 5 streams; the 3-D
// mixed-derivative periodic model of the reference's examples/testing.py: 7 streams).  Their
// activation fragments (S * WT / 2 bf16x8 per lane, twice that under LO) plus two accumulator sets
// do not fit the 256 VGPRs of two waves per SIMD, so wide kernels run ONE wave per SIMD with the
// whole 512-entry VGPR + AGPR file (MFMA A/B operands may live in AGPRs on gfx950), and the
// backward keeps 4-wave workgroups.  Under LO (bf16x3) the wave-private fragment stage (S * WT * 512
// bytes per wave: 224 KiB per workgroup at S = 7) no longer fits the 160 KiB LDS, so it moves to a
// wave-private region of global scratch (L2-resident: every wave writes its own lines and reads
// them back after an s_waitcnt), leaving the LDS to the backward's dK images.
__host__ __device__ constexpr bool bf3_wide(int WT, int S) { return S * WT > 32; }
__host__ __device__ constexpr int bf3_wpe(int WT, int S, bool lo) { return (lo || bf3_wide(WT, S) || WT > 8) ? 1 : 2; }
__host__ __device__ constexpr bool bf3_gstage(int WT, int S, bool lo) { return lo && bf3_wide(WT, S); }
// bf16x4 entries of one wave's fragment stage ([s][kb][hl][lane][2 halves])
// backward [point][feature] image row stride, bf16: 144 (72 words = 8 mod 64) up to 128 features,
// 16 WT + 16 beyond (WT = 16: 272 = 136 words, again 8 mod 64, so the same conflict-free pattern)
__host__ __device__ constexpr int bf3_img_rs(int WT) { return WT > 8 ? 16 * WT + 16 : 144; }
__host__ __device__ constexpr int stage_wave_elems(int WT, int S, bool lo) { return S * (WT / 2) * (lo ? 2 : 1) * 128; }

// the wave's own stage writes have landed before it reads them back (global stage only; an LDS
// stage is ordered by program order)
template <bool G>
__device__ __forceinline__ void stage_fence() {
  if constexpr (G) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// hi = rne_bf16(x), lo = rne_bf16(x - hi), two values per v_cvt_pk_bf16_f32
__device__ __forceinline__ void split4(const f32x4 v, bf16x4& hi, bf16x4& lo) {
  u32x2 H, L;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const f32x2 x = {v[2 * k], v[2 * k + 1]};
    const unsigned hb = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2));
    // scalar subtracts: packed f32 VALU (v_pk_add_f32) next to MFMAs costs extra issue cycles
    const float r0 = v[2 * k] - __builtin_bit_cast(float, hb << 16);
    const float r1 = v[2 * k + 1] - __builtin_bit_cast(float, hb & 0xffff0000u);
    const f32x2 rl = {r0, r1};
    H[k] = hb;
    L[k] = __builtin_bit_cast(unsigned, __builtin_convertvector(rl, bf16x2));
  }
  hi = __builtin_bit_cast(bf16x4, H);
  lo = __builtin_bit_cast(bf16x4, L);
}

// hi only (precision "bf16")
__device__ __forceinline__ bf16x4 cvt_hi4(const f32x4 v) {
  return __builtin_convertvector(v, bf16x4);
}

// split (LO) or round (!LO) one 4-element accumulator row
template <bool LO>
__device__ __forceinline__ void split_or_round(const f32x4 v, bf16x4& hi, bf16x4& lo) {
  if constexpr (LO)
    split4(v, hi, lo);
  else
    hi = cvt_hi4(v);
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

// first-order stream `idx` (uniform, 1..S1) of a per-stream array.  Up to two candidates: a
// select; more: the one-hot FMA over `sel` (LLVM turns a longer select chain over a register
// array back into an indexed scratch load).
template <int S, int S1, typename T>
__device__ __forceinline__ T sel_first(const T (&v)[S], int idx, const float (&sel)[TDQ_MAXS]) {
  if constexpr (S1 <= 2) {
    T r = v[1];
    if constexpr (S1 == 2) r = (idx == 2) ? v[2] : r;
    return r;
  } else {
    T r = sel[1] * v[1];
#pragma unroll
    for (int q = 2; q <= S1; ++q) r += sel[q] * v[q];
    return r;
  }
}

// Packed-fp32 (v_pk_mul / v_pk_fma / v_pk_add_f32) variant of the forward tanh jet: the two
// halves of each f32x4 accumulator tile are already even-aligned register pairs, so the jet
// arithmetic runs on pairs (exp / rcp / compares stay per element).  -DTDQ_PK_TANH=0: scalar.
#ifndef TDQ_PK_TANH
#define TDQ_PK_TANH 1
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void tanh_s1_x2(f32x2 z, f32x2& h, f32x2& s1) {
  const f32x2 az = {fabsf(z.x), fabsf(z.y)};
  const f32x2 a = az * -2.8853900817779268f;
  const f32x2 e = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  const f32x2 ep = e + 1.f;
  const f32x2 r = {__builtin_amdgcn_rcpf(ep.x), __builtin_amdgcn_rcpf(ep.y)};
  const f32x2 z2 = az * az;
  const f32x2 poly = az * (z2 * (z2 * (z2 * -0.053968254f + 0.13333334f) + -0.33333334f) + 1.f);
  const f32x2 big = (1.f - e) * r;
  const f32x2 t = {az.x < 0.125f ? poly.x : big.x, az.y < 0.125f ? poly.y : big.y};
  h = f32x2{__builtin_copysignf(t.x, z.x), __builtin_copysignf(t.y, z.y)};
  s1 = (e * 4.f) * (r * r);
}

// forward tanh jet of one feature tile: z -> h
template <int S, int NSO>
__device__ __forceinline__ void tanh_jet_f(const JetSpec& sp, const f32x4 (&z)[S], f32x4 (&h)[S]) {
#if TDQ_PK_TANH
  constexpr int S1p = S - 1 - NSO, SOp = 1 + S1p;
  f32x4 zap[S], zbp[S];
#pragma unroll
  for (int s = SOp; s < S; ++s) {
    zap[s] = sel_first<S, S1p>(z, sp.ia[s], sp.selA[s]);
    zbp[s] = sel_first<S, S1p>(z, sp.ib[s], sp.selB[s]);
  }
#pragma unroll
  for (int cp = 0; cp < 2; ++cp) {
    f32x2 hv, s1;
    tanh_s1_x2(f32x2{z[0][2 * cp], z[0][2 * cp + 1]}, hv, s1);
    const f32x2 s2 = (hv * -2.f) * s1;
    h[0][2 * cp] = hv.x;
    h[0][2 * cp + 1] = hv.y;
#pragma unroll
    for (int s = 1; s < SOp; ++s) {
      const f32x2 r = s1 * f32x2{z[s][2 * cp], z[s][2 * cp + 1]};
      h[s][2 * cp] = r.x;
      h[s][2 * cp + 1] = r.y;
    }
#pragma unroll
    for (int s = SOp; s < S; ++s) {
      const f32x2 r = (s2 * f32x2{zap[s][2 * cp], zap[s][2 * cp + 1]}) * f32x2{zbp[s][2 * cp], zbp[s][2 * cp + 1]} +
                      s1 * f32x2{z[s][2 * cp], z[s][2 * cp + 1]};
      h[s][2 * cp] = r.x;
      h[s][2 * cp + 1] = r.y;
    }
  }
  return;
#endif
  constexpr int S1 = S - 1 - NSO, SO = 1 + S1;
  f32x4 za[S], zb[S];
#pragma unroll
  for (int s = SO; s < S; ++s) {
    za[s] = sel_first<S, S1>(z, sp.ia[s], sp.selA[s]);
    zb[s] = sel_first<S, S1>(z, sp.ib[s], sp.selB[s]);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float hv, s1;
    tanh_s1(z[0][c], hv, s1);
    const float s2 = -2.f * hv * s1;
    h[0][c] = hv;
#pragma unroll
    for (int s = 1; s < SO; ++s) h[s][c] = s1 * z[s][c];
#pragma unroll
    for (int s = SO; s < S; ++s) h[s][c] = fmaf(s2 * za[s][c], zb[s][c], s1 * z[s][c]);
  }
}

// backward tanh jet of one feature tile from the saved post-activations h: hb -> zb
template <int S, int NSO>
__device__ __forceinline__ void tanh_jet_b(const JetSpec& sp, const f32x4 (&h)[S], const f32x4 (&hb)[S],
                                           f32x4 (&zb)[S]) {
  constexpr int S1 = S - 1 - NSO, SO = 1 + S1;
#if TDQ_PK_TANH
#pragma unroll
  for (int cp = 0; cp < 2; ++cp) {
    f32x2 hc[S], hbc[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      hc[s] = f32x2{h[s][2 * cp], h[s][2 * cp + 1]};
      hbc[s] = f32x2{hb[s][2 * cp], hb[s][2 * cp + 1]};
    }
    const f32x2 hv = hc[0];
    const f32x2 s1 = 1.f - hv * hv;
    const f32x2 m2h = hv * -2.f;
    f32x2 zbv[S];
    f32x2 sb1 = {0.f, 0.f}, sb2 = {0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S; ++s) zbv[s] = s1 * hbc[s];
#pragma unroll
    for (int s = 1; s < S; ++s) sb1 = hc[s] * hbc[s] + sb1;
#pragma unroll
    for (int s = SO; s < S; ++s) {
      const f32x2 ha = sel_first<S, S1>(hc, sp.ia[s], sp.selA[s]), hq = sel_first<S, S1>(hc, sp.ib[s], sp.selB[s]);
      const f32x2 hbs = hbc[s];
      sb2 = (ha * hq) * hbs + sb2;
      const f32x2 ga = (m2h * hq) * hbs, gb = (m2h * ha) * hbs;
      // one-hot FMAs (uniform 0 / 1 weights): two packed FMAs per first-order stream, where the
      // compiler if-converts the equivalent uniform branches into adds + per-element selects
#pragma unroll
      for (int q = 1; q < SO; ++q) zbv[q] = sp.selA[s][q] * ga + (sp.selB[s][q] * gb + zbv[q]);
    }
    zbv[0] = m2h * sb1 + (sb2 * -2.f + zbv[0]);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      zb[s][2 * cp] = zbv[s].x;
      zb[s][2 * cp + 1] = zbv[s].y;
    }
  }
  return;
#endif
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float hc[S];
#pragma unroll
    for (int s = 0; s < S; ++s) hc[s] = h[s][c];
    const float hv = hc[0];
    const float s1 = fmaf(-hv, hv, 1.f);
    const float m2h = -2.f * hv;
    float zbv[S];
    float sb1 = 0.f, sb2 = 0.f;
#pragma unroll
    for (int s = 0; s < S; ++s) zbv[s] = s1 * hb[s][c];
#pragma unroll
    for (int s = 1; s < S; ++s) sb1 = fmaf(hc[s], hb[s][c], sb1);
#pragma unroll
    for (int s = SO; s < S; ++s) {
      const float ha = sel_first<S, S1>(hc, sp.ia[s], sp.selA[s]), hq = sel_first<S, S1>(hc, sp.ib[s], sp.selB[s]);
      const float hbs = hb[s][c];
      sb2 = fmaf(ha * hq, hbs, sb2);
      const float ga = m2h * hq * hbs, gb = m2h * ha * hbs;
      if constexpr (S1 <= 2) {
#pragma unroll
        for (int q = 1; q < SO; ++q) {
          zbv[q] += (sp.ia[s] == q) ? ga : 0.f;
          zbv[q] += (sp.ib[s] == q) ? gb : 0.f;
        }
      } else {
#pragma unroll
        for (int q = 1; q < SO; ++q) zbv[q] = fmaf(sp.selA[s][q], ga, fmaf(sp.selB[s][q], gb, zbv[q]));
      }
    }
    zbv[0] = fmaf(m2h, sb1, fmaf(-2.f, sb2, zbv[0]));
#pragma unroll
    for (int s = 0; s < S; ++s) zb[s][c] = zbv[s];
  }
}

// Hs (saved post-activations, fp32): [layer][wg][s][wave][tile][lane][4]
__device__ __forceinline__ size_t hs_base(int layer, int nwg, int wg, int S, int w, int WT, int lane) {
  return ((((size_t)layer * nwg + wg) * S * 4 + w) * WT) * 256 + (unsigned)(lane * 4);
}
__device__ __forceinline__ int hs_off(int s, int t, int WT) { return (s * 4 * WT + t) * 256; }

// Saved activations move with non-temporal stores (forward) and loads (backward): they are written
// once, read after the whole forward + loss, and each read is too far from the next use of the
// line for the caches to help, so allocating them only evicts the weight images and partials that
// are reused.  A/B on MI355X (AC-SA step): plain 0.532 ms, nt stores 0.520, + nt loads 0.502;
// keeping the first of the two backward reads of a hidden layer cached (the tanh-adjoint pass reads
// the same lines right after) 0.494 vs 0.500; nt gradient-slab stores are slower (0.545 vs 0.520:
// the reduction re-reads them at once).  -DTDQ_TEMPORAL_STORES / -DTDQ_TEMPORAL_LOADS /
// -DTDQ_NT_C_LOADS / -DTDQ_NT_SLAB build the other variants (profiles/r1_v9_nontemporal_ab.txt).
// Saved-activation regions and weight images are addressed through buffer resources: the lane
// offset (lane * 16 bytes) is ONE VGPR shared by every access and the tile's uniform byte offset
// goes to soffset / the immediate field.  Per-lane 64-bit pointers plus tile offsets beyond the
// global instructions' 4 KiB immediate range cost a VGPR pair per distinct tile.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
struct Tl {
  __amdgpu_buffer_rsrc_t r;
  int v;
};
__device__ __forceinline__ Tl tl_make(const void* uniform_base, int lane) {
  return Tl{__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uniform_base), 0, 0x7fffffff, 0x00020000), lane * 16};
}
// Round 3 (profiles/r3_f_ab.txt): precision bf16 is faster with default-policy stores (0.2155-0.2175
// vs 0.2235-0.2243 ms per AC-SA step; a pure 217 MB store stream: 38 us default vs 60 us nt,
// tools/microbench/store_bw.hip), bf16x3 stays faster with nt stores (0.451-0.455 vs 0.480-0.481).
// -DTDQ_TEMPORAL_STORES: default policy for both; -DTDQ_NT_STORES: nt for both.
#if defined(TDQ_TEMPORAL_STORES)
#define TDQ_POL_ST_LO(LO) 0
#elif defined(TDQ_NT_STORES)
#define TDQ_POL_ST_LO(LO) 2
#else
#define TDQ_POL_ST_LO(LO) ((LO) ? 2 : 0)
#endif
#ifdef TDQ_TEMPORAL_LOADS
#define TDQ_POL_LD 0
#else
#define TDQ_POL_LD 2  // nt
#endif
// Precision "bf16" (!LO) saves the derivative streams (s >= 1) as bf16: the next layer's GEMM already
// consumed them rounded to bf16, so the dK images are unchanged, and the tanh-jet adjoint sees the
// same 2^-9 relative rounding the forward applied.  The value stream h stays fp32: s1 = 1 - h^2
// of a saturated unit loses every digit to a 16-bit h (fp16 ulp at |h| ~ 1 is 2^-11).  Storing it
// as fp16 (-DTDQ_HS_VALUE_FP16: every tile 8 B per lane) was 2.5 % faster per step, but the AC-SA
// reference schedule (Adam bf16 + L-BFGS bf16x3) ended at L2 4.3/2.8/4.9/3.7/3.6e-2 over seeds
// 0-4 against 3.3/2.6/3.4/4.8/2.9e-2 with the fp32 value stream (profiles/r2_v7_accuracy_seeds.txt).
// -DTDQ_BF16_HS_FP32 keeps every stream fp32 (A/B).
#ifdef TDQ_BF16_HS_FP32
#define TDQ_HS_HALF(LO) false
#else
#define TDQ_HS_HALF(LO) (!(LO))
#endif
#ifdef TDQ_HS_VALUE_FP16
#define TDQ_HS_V16 1
#else
#define TDQ_HS_V16 0
#endif
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
template <int WT, bool LO>
__host__ __device__ constexpr int hs_wave_floats(int S) {
  return TDQ_HS_HALF(LO) ? WT * ((TDQ_HS_V16 ? 128 : 256) + (S - 1) * 128) : S * WT * 256;
}
// byte offset of tile (s, t) inside a wave's half-precision region (lane stride 8 B, or 16 B for
// an fp32 value stream)
template <int WT>
__device__ __forceinline__ int hs_half_off(int s, int t) {
  return TDQ_HS_V16 ? (s * WT + t) * 512 : (s == 0 ? t * 1024 : WT * 1024 + ((s - 1) * WT + t) * 512);
}
// wave w's region of saved layer `layer` (uniform base; the lane offset lives in Tl::v)
template <int WT, bool LO>
__device__ __forceinline__ Tl hs_region(const float* Hs, int layer, int nwg, int wg, int S, int w, int lane) {
  if constexpr (TDQ_HS_HALF(LO))
    return tl_make(Hs + (((size_t)layer * nwg + wg) * 4 + w) * hs_wave_floats<WT, LO>(S), lane);
  else
    return tl_make(Hs + hs_base(layer, nwg, wg, S, w, WT, 0), lane);
}
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
template <int WT, bool LO>
__device__ __forceinline__ void hs_store(const Tl& T, int s, int t, const f32x4& v) {
  if constexpr (TDQ_HS_HALF(LO)) {
    if (s == 0 && !TDQ_HS_V16) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), T.r, T.v, hs_half_off<WT>(0, t),
                                             TDQ_POL_ST_LO(LO));
      return;
    }
    const u32x2v u = s == 0 ? __builtin_bit_cast(u32x2v, __builtin_convertvector(v, f16x4))
                            : __builtin_bit_cast(u32x2v, __builtin_convertvector(v, bf16x4));
    __builtin_amdgcn_raw_buffer_store_b64(u, T.r, T.v >> 1, hs_half_off<WT>(s, t), TDQ_POL_ST_LO(LO));
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), T.r, T.v, hs_off(s, t, WT) * 4, TDQ_POL_ST_LO(LO));
  }
}
template <int WT, bool LO, int POL>
__device__ __forceinline__ f32x4 hs_load_p(const Tl& T, int s, int t) {
  if constexpr (TDQ_HS_HALF(LO)) {
    if (s == 0 && !TDQ_HS_V16)
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(T.r, T.v, hs_half_off<WT>(0, t), POL));
    const u32x2v u = __builtin_amdgcn_raw_buffer_load_b64(T.r, T.v >> 1, hs_half_off<WT>(s, t), POL);
    if (s == 0) return __builtin_convertvector(__builtin_bit_cast(f16x4, u), f32x4);
    // bf16 -> fp32: the bf16 bits are the high half of the fp32 word
    return f32x4{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
                 __uint_as_float(u[1] & 0xffff0000u)};
  } else {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(T.r, T.v, hs_off(s, t, WT) * 4, POL));
  }
}
template <int WT, bool LO>
__device__ __forceinline__ f32x4 hs_load(const Tl& T, int s, int t) {
  return hs_load_p<WT, LO, TDQ_POL_LD>(T, s, t);
}
// the dK pass's read of h_{i-1} (the same lines are read again by the tanh-adjoint pass): cached
template <int WT, bool LO>
__device__ __forceinline__ f32x4 hs_load_c(const Tl& T, int s, int t) {
#ifdef TDQ_NT_C_LOADS
  return hs_load<WT, LO>(T, s, t);
#else
  return hs_load_p<WT, LO, 0>(T, s, t);
#endif
}
// hi / lo A fragment of step `st` of a layer's weight image (lo 64 lanes = 1 KiB later; hi only
// under !LO)
template <bool LO>
__device__ __forceinline__ void img_frag(const Tl& I, int st, bf16x8& hi, bf16x8& lo) {
  hi = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(I.r, I.v, st * 2048, 0));
  if constexpr (LO) lo = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(I.r, I.v, st * 2048 + 1024, 0));
}

__device__ __forceinline__ void slab_store(float* p, float v) {
#ifdef TDQ_NT_SLAB
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// Precision "bf16" (!LO) writes its per-workgroup gradient slabs as bf16 (RNE): half the slab
// bytes written by the backward and re-read by the reduction.  Each entry is a 128-point partial
// sum; the reduction adds the rows in fp32, so the rounding adds ~2^-9 relative error per partial,
// below the bf16 GEMM operands' own (kernel gradient error vs fp64: profiles/r2_v12_*).
// -DTDQ_SLAB_BF16=0 keeps fp32 slabs (A/B); bf16x3 always uses fp32.
#ifndef TDQ_SLAB_BF16
#define TDQ_SLAB_BF16 1
#endif
__host__ __device__ constexpr bool slab_half(bool lo) { return TDQ_SLAB_BF16 && !lo; }
template <bool H> struct SlabType { using T = float; };
template <> struct SlabType<true> { using T = __bf16; };
__device__ __forceinline__ void slab_put(float* p, float v) { slab_store(p, v); }
__device__ __forceinline__ void slab_put(__bf16* p, float v) { *p = (__bf16)v; }

// Weight images written element by element (the inverse of the pack kernels of jet_bf3.hip): the
// Adam tail (tail_adam_kernel) and the L-BFGS direction kernel (lbfgs.hip) scatter every updated
// parameter straight into the next evaluation's images, so no pack launch is needed.
struct TailImg {
  __bf16* fimg;  // forward A image (nullptr: no image update)
  __bf16* bimg;  // backward A image
  float* aux;
  NetDims d;
  int WT;
};

// element (row, kf) of hidden layer `layer`'s A image -> bf16 hi / lo (inverse of pack_frag)
__device__ __forceinline__ void img_put(__bf16* __restrict__ img, int layer, int row, int kf, int WT, __bf16 hi,
                                        __bf16 lo) {
  const int KB = WT / 2;
  const int o = row >> 4, p = row & 15, kb = kf >> 5, rr = kf & 31;
  const int g = (rr & 15) >> 2, j = (rr & 3) + (rr >= 16 ? 4 : 0);
  const int lane = p + 16 * g;
  const size_t frag = ((size_t)(layer - 1) * WT + o) * KB + kb;
  img[((frag * 2) * 64 + lane) * 8 + j] = hi;
  img[((frag * 2 + 1) * 64 + lane) * 8 + j] = lo;
}

// flat (Keras-order) parameter e with new value v -> its slot in the images (inverse of pack_all)
__device__ __forceinline__ void scatter_param(float v, int e, const TailImg& ti) {
  const NetDims& d = ti.d;
  const int W = 16 * ti.WT, w = hw(d, 0);
  const int n0 = d.d_in * w;
  if (e < n0) {
    const int j = e / w;
    ti.aux[j * W + (e - j * w)] = v;
    return;
  }
  if (e < n0 + w) {
    ti.aux[aux_b0(d, W) + (e - n0)] = v;
    return;
  }
  if (e < off_layer(d, d.n_hidden)) {  // hidden layer i >= 1: kernel [w_{i-1}][w_i], bias [w_i]
    int i = 1;
    while (i + 1 < d.n_hidden && e >= off_layer(d, i + 1)) ++i;
    const int q = e - off_layer(d, i), wi = hw(d, i - 1), wo = hw(d, i);
    if (q < wi * wo) {
      const int in = q / wo, out = q - in * wo;
      const __bf16 hi = (__bf16)v, lo = (__bf16)(v - (float)hi);
      img_put(ti.fimg, i, out, in, ti.WT, hi, lo);  // forward: A[row = out][k = in]
      img_put(ti.bimg, i, in, out, ti.WT, hi, lo);  // backward: A[row = in][k = out]
    } else {
      ti.aux[aux_bh(d, W) + (i - 1) * W + (q - wi * wo)] = v;
    }
    return;
  }
  const int r2 = e - off_layer(d, d.n_hidden), wl = hw(d, d.n_hidden - 1);
  if (r2 < wl * d.d_out) {
    const int f = r2 / d.d_out;
    ti.aux[aux_ko(d, W) + f * 4 + (r2 - f * d.d_out)] = v;
  } else {
    ti.aux[aux_bo(d, W) + (r2 - wl * d.d_out)] = v;
  }
}

// layer 0 (input -> width, VALU; derivative streams are rows of K0): the post-activation streams of
// feature tile t (forward).
template <int WT, int S, int NSO>
__device__ __forceinline__ void h0_jet(const JetSpec& sp, const float* __restrict__ aux, const NetDims& d,
                                       const float* __restrict__ x, int t, int g, f32x4 (&h)[S]) {
  constexpr int S1 = S - 1 - NSO, SO = 1 + S1, W = 16 * WT;
  const int f0 = 16 * t + 4 * g;
  f32x4 z[S];
  z[0] = *reinterpret_cast<const f32x4*>(aux + aux_b0(d, W) + f0);
#pragma unroll
  for (int j = 0; j < TDQ_MAXD; ++j)
    if (j < d.d_in) z[0] += x[j] * *reinterpret_cast<const f32x4*>(aux + j * W + f0);
#pragma unroll
  for (int s = 1; s < SO; ++s) z[s] = *reinterpret_cast<const f32x4*>(aux + sp.var[s] * W + f0);
#pragma unroll
  for (int s = SO; s < S; ++s) z[s] = zero4();
  tanh_jet_f<S, NSO>(sp, z, h);
}

// Layer 0's derivative streams are functions of its value stream alone (z_a = a row of K0,
// z_ab = 0): h_a = s1 K0[a], h_ab = -2 h s1 K0[a] K0[b], s1 = 1 - h^2.  With h0r set the forward
// saves only the value stream of layer 0 and the backward rebuilds stream s here - 3/4 less
// layer-0 saved-activation traffic (the step is bound by that traffic) for ~2 VALU ops per value.
template <int WT, int S, int NSO>
__device__ __forceinline__ f32x4 h0_stream(const JetSpec& sp, const float* __restrict__ aux, const f32x4& h, int t,
                                           int g, int s) {
  constexpr int S1 = S - 1 - NSO, SO = 1 + S1, W = 16 * WT;
  if (s == 0) return h;
  const int f0 = 16 * t + 4 * g;
  f32x4 r;
  if (s < SO) {
    const f32x4 k = *reinterpret_cast<const f32x4*>(aux + sp.var[s] * W + f0);
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = fmaf(-h[c], h[c], 1.f) * k[c];
  } else {
    const f32x4 ka = *reinterpret_cast<const f32x4*>(aux + sp.var[sp.ia[s]] * W + f0);
    const f32x4 kb = *reinterpret_cast<const f32x4*>(aux + sp.var[sp.ib[s]] * W + f0);
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = (-2.f * h[c]) * fmaf(-h[c], h[c], 1.f) * (ka[c] * kb[c]);
  }
  return r;
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// output layer (width -> d_out, VALU) of one feature tile of the last hidden layer, straight from
// the epilogue registers: per-lane partial dots, summed across the 4 row groups at the end
template <int S>
__device__ __forceinline__ void out_dot(const f32x4 (&h)[S], const float* __restrict__ Ko, int t, int g,
                                        float (&v)[S][TDQ_MAXO]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x4 kq = *reinterpret_cast<const f32x4*>(Ko + (16 * t + 4 * g + c) * 4);
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int q = 0; q < TDQ_MAXO; ++q) v[s][q] = fmaf(h[s][c], kq[q], v[s][q]);
  }
}

template <int WT, int S, int NSO, bool LO, bool LAST>
__device__ __forceinline__ void fwd_hidden(bf16x8 (&ah)[S][WT / 2], bf16x8 (&al)[S][WT / 2], const Tl& Wi,
                                           const float* __restrict__ bi, const Tl& Hl, bf16x4* stage,
                                           const float* __restrict__ Ko, float (&vout)[S][TDQ_MAXO],
                                           const JetSpec& sp, int l, int g) {
  constexpr int KB = WT / 2, NSTEP = WT * KB, D = NSTEP < 4 ? NSTEP : 4, HL = LO ? 2 : 1;
  bf16x8 wh[D], wl[D];
#pragma unroll
  for (int k = 0; k < D; ++k) img_frag<LO>(Wi, k, wh[k], wl[k]);
  f32x4 accA[S], accB[S], biasA = zero4(), biasB = zero4();
#pragma unroll
  for (int s = 0; s < S; ++s) accA[s] = accB[s] = zero4();
#pragma unroll
  for (int o = 0; o <= WT; ++o) {
    f32x4(&accC)[S] = (o & 1) ? accB : accA;
    f32x4(&accP)[S] = (o & 1) ? accA : accB;
    f32x4& biasC = (o & 1) ? biasB : biasA;
    const f32x4& biasP = (o & 1) ? biasA : biasB;
    if (o < WT) {  // MFMAs of output tile o
      biasC = *reinterpret_cast<const f32x4*>(bi + 16 * o + 4 * g);
#pragma unroll
      for (int s = 0; s < S; ++s) accC[s] = zero4();
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int st = o * KB + kb;
        const bf16x8 Ah = wh[st % D], Al = wl[st % D];
        if (st + D < NSTEP) img_frag<LO>(Wi, st + D, wh[st % D], wl[st % D]);
#pragma unroll
        for (int s = 0; s < S; ++s) accC[s] = mfma_w<LO>(Ah, Al, ah[s][kb], al[s][kb], accC[s]);
      }
    }
    if (o > 0) {  // epilogue of tile o-1 in the same scheduling region
      const int t = o - 1;
      f32x4 z[S], h[S];
#pragma unroll
      for (int s = 0; s < S; ++s) z[s] = accP[s];
      z[0] += biasP;
      tanh_jet_f<S, NSO>(sp, z, h);
#pragma unroll
      for (int s = 0; s < S; ++s) hs_store<WT, LO>(Hl, s, t, h[s]);
      if (LAST) {
        out_dot<S>(h, Ko, t, g, vout);
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          bf16x4 hi, lo;
          split_or_round<LO>(h[s], hi, lo);
          stage[(((s * KB + (t >> 1)) * HL + 0) * 64 + l) * 2 + (t & 1)] = hi;
          if constexpr (LO) stage[(((s * KB + (t >> 1)) * HL + 1) * 64 + l) * 2 + (t & 1)] = lo;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (!LAST) {  // wave-private region: program order suffices (LDS) / a vmcnt wait (global stage)
    stage_fence<bf3_gstage(WT, S, LO)>();
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        ah[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[(((s * KB + kb) * HL + 0) * 64 + l) * 2]);
        if constexpr (LO) al[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[(((s * KB + kb) * HL + 1) * 64 + l) * 2]);
      }
  }
}

template <int WT, int S, int NSO, bool LO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(bf3_wpe(WT, S, LO), bf3_wpe(WT, S, LO))))
jet_fwd_bf3_kernel(const float* __restrict__ X, const float* __restrict__ aux, const bf16x8* __restrict__ Wimg,
                   float* __restrict__ J, float* __restrict__ Hs, int N, NetDims d, JetSpec sp, int h0r,
                   bf16x4* __restrict__ gstage, int wg0) {
  constexpr int KB = WT / 2, NSTEP = WT * KB, W = 16 * WT;
  constexpr int S1 = S - 1 - NSO, SO = 1 + S1;
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // wg0: first workgroup of this launch (a point range of the whole set, see Bf3Args::p_lo); the
  // saved-activation layout and J always index the whole set
  const int wg = wg0 + (int)blockIdx.x, nwg = (N + 63) / 64;
  const int n = wg * 64 + w * 16 + p;
  const bool valid = n < N;
  const int nc = valid ? n : N - 1;  // clamped: every load is in bounds, no exec branches
  const int Lh = d.n_hidden;
  // wave-private staging image of the next layer's B fragments: [s][kb][hl][lane][2 halves]
  constexpr int HL = LO ? 2 : 1;
  bf16x4* stage = bf3_gstage(WT, S, LO)
                      ? gstage + (size_t)(wg * 4 + w) * stage_wave_elems(WT, S, LO)
                      : reinterpret_cast<bf16x4*>(lds_raw) + (size_t)w * (S * KB * HL * 64 * 2);
  const float* Ko = aux + aux_ko(d, W);

  TDQ_TS(0);
  float x[TDQ_MAXD];
#pragma unroll
  for (int j = 0; j < TDQ_MAXD; ++j) x[j] = j < d.d_in ? X[(size_t)nc * d.d_in + j] : 0.f;

  bf16x8 ah[S][KB], al[S][KB];
  float v[S][TDQ_MAXO];  // output-layer partial dots (last hidden layer's epilogue)
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q) v[s][q] = 0.f;

  // ---- layer 0 (input -> width) on VALU ---------------------------------------------------
  {
    const Tl H0 = hs_region<WT, LO>(Hs, 0, nwg, wg, S, w, l);
    const bool save_all = !h0r || Lh == 1;  // else the backward rebuilds streams >= 1 (h0_stream)
    const bool save0 = true;  // (Lh = 1: the backward's output phase reads the saved layer 0)
    bf16x4 ph[S], pl[S];
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      f32x4 h[S];
      h0_jet<WT, S, NSO>(sp, aux, d, x, t, g, h);
      if (save0) {
        hs_store<WT, LO>(H0, 0, t, h[0]);
        if (save_all) {
#pragma unroll
          for (int s = 1; s < S; ++s) hs_store<WT, LO>(H0, s, t, h[s]);
        }
      }
      if (Lh == 1) {
        out_dot<S>(h, Ko, t, g, v);
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          bf16x4 hi, lo;
          split_or_round<LO>(h[s], hi, lo);
          if (t & 1) {
            ah[s][t >> 1] = cat8(ph[s], hi);
            if constexpr (LO) al[s][t >> 1] = cat8(pl[s], lo);
          } else {
            ph[s] = hi;
            if constexpr (LO) pl[s] = lo;
          }
        }
      }
    }
  }

  TDQ_TS(1);
  // ---- hidden layers on bf16x3 MFMA --------------------------------------------------------
  for (int i = 1; i < Lh - 1; ++i) {
    fwd_hidden<WT, S, NSO, LO, false>(ah, al, tl_make(Wimg + (size_t)(i - 1) * NSTEP * 128, l),
                                      aux + aux_bh(d, W) + (i - 1) * W, hs_region<WT, LO>(Hs, i, nwg, wg, S, w, l), stage,
                                      Ko, v, sp, l, g);
    TDQ_TS(1 + i);
  }
  if (Lh >= 2) {
    const int i = Lh - 1;
    fwd_hidden<WT, S, NSO, LO, true>(ah, al, tl_make(Wimg + (size_t)(i - 1) * NSTEP * 128, l),
                                     aux + aux_bh(d, W) + (i - 1) * W, hs_region<WT, LO>(Hs, i, nwg, wg, S, w, l), stage,
                                     Ko, v, sp, l, g);
    TDQ_TS(1 + i);
  }

  // ---- output layer (width -> d_out): cross-lane sum of the epilogue partial dots ---------
  const f32x4 bo = *reinterpret_cast<const f32x4*>(aux + aux_bo(d, W));
#pragma unroll
  for (int q = 0; q < TDQ_MAXO; ++q) {
    if (q >= d.d_out) break;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float r = col4_sum(v[s][q]);
      if (s == 0) r += bo[q];
      if (g == 0 && valid) J[((size_t)s * N + n) * d.d_out + q] = r;
    }
  }
  TDQ_TS(15);
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
template <int S, int WT, bool LO>
__device__ __forceinline__ void h_tile(f32x4 (&h)[S], const Tl& Hl, int t) {
#pragma unroll
  for (int s = 0; s < S; ++s) h[s] = hs_load<WT, LO>(Hl, s, t);
}

// first-layer partials from zb_0 (fp32) of one feature tile: bias b0 and dK0[j][f] (one LDS slot
// per wave, summed in fixed wave order later)
template <int WT, int S, int NSO>
__device__ __forceinline__ void first_layer_partials(const JetSpec& sp, const f32x4 (&zb)[S],
                                                     const float* __restrict__ xrow, const NetDims& d, int t,
                                                     int w, int p, int g, float* accB0, float* accK0) {
  constexpr int S1 = S - 1 - NSO, SO = 1 + S1, W = 16 * WT;
  const int fo = 16 * t + 4 * g + (p >> 2);  // feature this lane stores after row16_sum4
  {
    const float r = row16_sum4(zb[0]);
    if ((p & 3) == 0) accB0[w * W + fo] = r;
  }
  for (int j = 0; j < d.d_in; ++j) {
    const float xj = xrow[j];
    f32x4 v;  // scalar per component: packed f32 VALU beside MFMAs costs issue cycles
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float a = xj * zb[0][c];
#pragma unroll
      for (int s = 1; s < SO; ++s) a += (sp.var[s] == j) ? zb[s][c] : 0.f;
      v[c] = a;
    }
    const float r = row16_sum4(v);
    if ((p & 3) == 0) accK0[w * TDQ_MAXD * W + j * W + fo] = r;
  }
}

// zb of one feature tile -> bias partial of its layer + hi/lo halves into the wave's fragment
// stage ([s][kb][hl][lane][2 halves] bf16x4, the forward's staging layout)
template <int WT, int S, bool LO>
__device__ __forceinline__ void zb_to_stage(const f32x4 (&zb)[S], const NetDims& d, int t, int w, int l, int p,
                                            int g, float* accBslot, bf16x4* stage) {
  constexpr int KB = WT / 2, W = 16 * WT, HL = LO ? 2 : 1;
  {
    const float r = row16_sum4(zb[0]);
    if ((p & 3) == 0) accBslot[w * W + 16 * t + 4 * g + (p >> 2)] = r;
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    bf16x4 hi, lo;
    split_or_round<LO>(zb[s], hi, lo);
    stage[(((s * KB + (t >> 1)) * HL + 0) * 64 + l) * 2 + (t & 1)] = hi;
    if constexpr (LO) stage[(((s * KB + (t >> 1)) * HL + 1) * 64 + l) * 2 + (t & 1)] = lo;
  }
}

// (d) of hidden layer i: hb_{i-1} = K_i zb_i on bf16x3 MFMA; the epilogue of output tile o-1
// (tanh-jet adjoint with the saved h_{i-1}, bias partials, split + stage - or, when i = 1, the
// first-layer partials) runs in the scheduling region of tile o's MFMAs.
template <int WT, int S, int NSO, bool LO, bool TO_FIRST>
__device__ __forceinline__ void bwd_hidden_d(const bf16x8 (&zh)[S][WT / 2], const bf16x8 (&zl)[S][WT / 2],
                                             const Tl& Ki, const Tl& Hp,
                                             bf16x4* stage, float* accBslot, float* accK0,
                                             const float* __restrict__ xrow, const JetSpec& sp, const NetDims& d,
                                             const float* __restrict__ aux, bool h0r, int w, int l, int p, int g) {
  constexpr int KB = WT / 2, NSTEP = WT * KB, D = NSTEP < 4 ? NSTEP : 4;
  bf16x8 wh[D], wl[D];
#pragma unroll
  for (int k = 0; k < D; ++k) img_frag<LO>(Ki, k, wh[k], wl[k]);
  // TO_FIRST && h0r: only layer 0's value stream is saved; the others are rebuilt (h0_stream)
  const bool rec = TO_FIRST && h0r;
  f32x4 hr[2][S];
  if (rec) {
    hr[0][0] = hs_load<WT, LO>(Hp, 0, 0);
    if (WT > 1) hr[1][0] = hs_load<WT, LO>(Hp, 0, 1);
  } else {
    h_tile<S, WT, LO>(hr[0], Hp, 0);
    if (WT > 1) h_tile<S, WT, LO>(hr[1], Hp, 1);
  }
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
        const bf16x8 Ah = wh[st % D], Al = wl[st % D];
        if (st + D < NSTEP) img_frag<LO>(Ki, st + D, wh[st % D], wl[st % D]);
#pragma unroll
        for (int s = 0; s < S; ++s) accC[s] = mfma_w<LO>(Ah, Al, zh[s][kb], zl[s][kb], accC[s]);
      }
    }
    if (o > 0) {
      const int t = o - 1;
      f32x4 h[S], zb[S];
      if (rec) {
        h[0] = hr[t & 1][0];
        if (t + 2 < WT) hr[t & 1][0] = hs_load<WT, LO>(Hp, 0, t + 2);
#pragma unroll
        for (int s = 1; s < S; ++s) h[s] = h0_stream<WT, S, NSO>(sp, aux, h[0], t, g, s);
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) h[s] = hr[t & 1][s];
        if (t + 2 < WT) h_tile<S, WT, LO>(hr[t & 1], Hp, t + 2);
      }
      tanh_jet_b<S, NSO>(sp, h, accP, zb);
      if (TO_FIRST)
        first_layer_partials<WT, S, NSO>(sp, zb, xrow, d, t, w, p, g, accBslot, accK0);
      else
        zb_to_stage<WT, S, LO>(zb, d, t, w, l, p, g, accBslot, stage);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Waves per backward workgroup.  bf16 (!LO) at WT >= 4: 8 waves = 128 points, one workgroup per
// CU (2 waves per SIMD, like two 4-wave workgroups): half the per-workgroup gradient slab rows
// (written here, re-read by tdq_slab_reduce) and half the dK accumulators per wave (each wave owns
// 8 of the 64 16x16 dK tiles instead of 16).  bf16x3 keeps 4 waves: its 32 KiB per-wave fragment
// stage leaves no LDS for 8.  -DTDQ_BWD_WIDE=0 builds the 4-wave bf16 kernel (A/B).
#ifndef TDQ_BWD_WIDE
#define TDQ_BWD_WIDE 1
#endif
// WT = 16: dK column tiles per pass (of a wave's 8): 4 (two passes) 0.945 ms vs 2 (four passes) 1.035 ms per
// width-256 AC step (profiles/r4v_w256_ncp_ab.jsonl); -DTDQ_W16_NCP for A/B runs
#ifndef TDQ_W16_NCP
#define TDQ_W16_NCP 4
#endif
// (wide plans: 4 waves - an 8-wave workgroup puts two waves on each SIMD, 256 registers each)
__host__ __device__ constexpr int bwd_waves(int WT, bool lo, int S) {
  return (TDQ_BWD_WIDE && !lo && WT >= 4 && WT <= 8 && !bf3_wide(WT, S)) ? 8 : 4;
}

template <int WT, int S, int NSO, bool LO>
__global__ void __launch_bounds__(64 * bwd_waves(WT, LO, S))
__attribute__((amdgpu_waves_per_eu(bf3_wpe(WT, S, LO), bf3_wpe(WT, S, LO))))
jet_bwd_bf3_kernel(const float* __restrict__ X, const float* __restrict__ aux, const bf16x8* __restrict__ Kimg,
                   const float* __restrict__ dJ, const float* __restrict__ Hs, float* __restrict__ slab, int N,
                   int Ptot, NetDims d, JetSpec sp, int rev, int h0r, bf16x4* __restrict__ gstage,
                   int wg0) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int W = 16 * WT;
  constexpr int KB = WT / 2;
  // [point][feature] bf16 images (h hi/lo, zb hi/lo).  Row stride 144 bf16 = 72 words (= 8 mod 64)
  // and the 64-column XOR on bit 3 of the row put the 8 rows of a transposed read's 32-lane half
  // (4 rows x 2 groups 8 rows apart, 8 words each) on 8 disjoint bank windows: conflict-free.
  // Inside each 16-column block the 4-column chunks are XOR-permuted by bits 2-3 of the row
  // (chunk' = chunk ^ ((row >> 2) & 3)): a ds_write_b64 lane group (16 rows, one chunk, banks
  // mod 32) then covers 32 distinct banks instead of 8 (4-way conflicts on every image store), and
  // a transposed read still fetches each row's same 8-word window, each lane at its chunk's new
  // place.
#ifdef TDQ_NO_CHUNK_SWIZZLE
  constexpr int CHUNK_SWZ = 0;
#else
  constexpr int CHUNK_SWZ = 1;
#endif
  constexpr int NWV = bwd_waves(WT, LO, S), PTS = 16 * NWV;  // waves / points per workgroup
  constexpr bool GST = bf3_gstage(WT, S, LO);                 // zb stage in global scratch
  constexpr int RS = bf3_img_rs(WT);
  constexpr int IMG = PTS * RS;
  // dK tile ownership: the WT x WT output tiles split into (NWV/2) x 2 blocks, wave w owns block
  // (w >> 1, w & 1): NR x NC tiles from NR A and NC B fragments per k-block (4 waves: quadrants;
  // a 2 x 8 strip per wave would need 2 + 8 fragment loads for the same 16 tiles at WT = 8)
  constexpr int NR = WT / (NWV / 2);
  constexpr int NC = WT / 2;
  // WT = 16: the 8 x 8 tiles of a wave's block take 256 accumulator registers - done in PC column
  // passes of NCP tiles (the images are rebuilt per pass; a pass's MFMAs read 8 + NCP fragments)
  constexpr int NCP = NC > 4 ? TDQ_W16_NCP : NC, PC = NC / NCP;
  // row tiles past the fourth start a second transposed-read base (the immediate offsets 16 r of
  // one base must stay below the swizzled column bit 6)
  constexpr int RB = NR > 4 ? 2 : 1, NRB = NR / RB;
  // images: h hi, (h lo,) zb hi, (zb lo) - the lo images only under LO
  constexpr int HL = LO ? 2 : 1;
  constexpr int IH = 0, IHL = IMG, IZ = HL * IMG, IZL = 3 * IMG;
  // bf16 (!LO): two image buffers, stream s writes buffer s & 1, so one barrier per stream
  // separates "images of s written" from "MFMAs of s - 1 done" (bf16x3: one buffer, two barriers;
  // its LDS holds no second set)
  constexpr bool DBUF = !LO;
  constexpr int IBUF = 2 * HL * IMG;          // one buffer's images, in bf16
  constexpr int U1 = (DBUF ? 2 : 1) * IBUF / 2;  // images, in floats
  constexpr int U2 = GST ? 0 : NWV * S * WT * HL * 128;  // per-wave zb fragment stages (bf16 hi(/lo))
  constexpr int U = ((U1 > U2 ? U1 : U2) + 3) / 4 * 4;
  static_assert(NWV * (W * TDQ_MAXO + TDQ_MAXO + TDQ_MAXD * W) <= U, "partials must fit the union");
  __bf16* img = reinterpret_cast<__bf16*>(lds);
  float* accB = lds + U;                      // [3: layer parity 0/1, layer 0][NWV][W]
  // output- and first-layer partials alias the image / stage union: they live while neither does
  // (Ko is reduced right after the output phase, K0 after the last image read)
  float* accKo = lds;                         // [NWV][W * TDQ_MAXO]
  float* accK0 = accKo + NWV * W * TDQ_MAXO + NWV * TDQ_MAXO;  // [NWV][TDQ_MAXD * W]
  float* accBo = accKo + NWV * W * TDQ_MAXO;  // [NWV][TDQ_MAXO]

  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // rev: tiles in reverse dispatch order - the forward wrote the highest tiles last, so theirs are
  // the saved activations still resident in the 256 MiB Infinity Cache when the backward starts
  // (wg0: first workgroup of a point-range launch; slabs and saved activations index the whole set)
  const int nwl = gridDim.x, wg = wg0 + (rev ? nwl - 1 - (int)blockIdx.x : (int)blockIdx.x);
  const int n = wg * PTS + w * 16 + p;
  // saved activations are laid out by the forward's 64-point workgroups: this wave's region is
  // forward workgroup wg_f, wave w_f (clamped: the padding half of a last 128-point workgroup
  // reads a real region - finite values, multiplied by zero adjoints)
  const int nwg_f = (N + 63) / 64;
  const int wg_f = min(wg * (NWV / 4) + (w >> 2), nwg_f - 1), w_f = w & 3;
  const bool valid = n < N;
  const int nc = valid ? n : N - 1;
  const float vmask = valid ? 1.f : 0.f;  // zero adjoints for padding points: zb = 0 downstream
  const int Lh = d.n_hidden;
  constexpr bool SH = slab_half(LO);
  using ST = typename SlabType<SH>::T;
  ST* gs = reinterpret_cast<ST*>(slab) + (size_t)wg * Ptot;
  bf16x4* stage = GST ? gstage + (size_t)(wg * NWV + w) * stage_wave_elems(WT, S, LO)
                      : reinterpret_cast<bf16x4*>(lds) + (size_t)w * (S * KB * HL * 64 * 2);
  auto dw_row = [](int wv, int r) { return NR * (wv >> 1) + r; };
  auto dw_col = [](int wv, int c) { return NC * (wv & 1) + c; };
  // transposed-read lane address inside a 4 x 16 block: row (l & 15) >> 2, column 4 (l & 3)
  const int tr_row = 8 * g + ((l & 15) >> 2), tr_col = 4 * (l & 3);
  const int swz = (g & 1) << 6;  // bit 3 of every row this lane's transposed reads touch
  // the chunk swizzle of the rows this lane reads: rows 8g + q (first read) and 8g + 4 + q
  // (second read), q < 4, so (row >> 2) & 3 = 2g & 3 and (2g + 1) & 3
  const int tr_col1 = CHUNK_SWZ ? 4 * ((l & 3) ^ ((2 * g) & 3)) : tr_col;
  const int tr_col2 = CHUNK_SWZ ? 4 * ((l & 3) ^ ((2 * g + 1) & 3)) : tr_col;
  const float* xrow = X + (size_t)nc * d.d_in;  // padding points: zb = 0, x is irrelevant
  TDQ_TS(0);

  bf16x8 zh[S][KB], zl[S][KB];

  // ---- output layer: hb = Ko ub ; dKo += h_last ub ; dbo += ub ; then the top tanh layer's
  //      adjoint zb_{Lh-1} tile by tile (bias partials + B fragments, or first-layer partials)
  {
    const float* Ko = aux + aux_ko(d, W);
    const Tl Hl = hs_region<WT, LO>(Hs, Lh - 1, nwg_f, wg_f, S, w_f, l);
    float* accBslot = Lh >= 2 ? accB + ((Lh - 1) & 1) * NWV * W : accB + 2 * NWV * W;
    float ub[S][TDQ_MAXO];
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q)
#pragma unroll
      for (int s = 0; s < S; ++s) ub[s][q] = q < d.d_out ? vmask * dJ[((size_t)s * N + nc) * d.d_out + q] : 0.f;
    constexpr int DH = WT < 3 ? WT : 3;  // H tiles in flight
    f32x4 hr[DH][S];
#pragma unroll
    for (int k = 0; k < DH; ++k) h_tile<S, WT, LO>(hr[k], Hl, k);
    bf16x4 ph[S], pl[S];
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      f32x4 h[S];
#pragma unroll
      for (int s = 0; s < S; ++s) h[s] = hr[t % DH][s];
      if (t + DH < WT) h_tile<S, WT, LO>(hr[t % DH], Hl, t + DH);
      // hb = Ko ub over the zero-padded 4 output columns: no branches
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
      // dKo[f][q] partials: sum over points of sum_s h_s ub_s
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
      if (Lh >= 2) {
        {
          const float r = row16_sum4(zb[0]);
          if ((p & 3) == 0) accBslot[w * W + 16 * t + 4 * g + (p >> 2)] = r;
        }
#pragma unroll
        for (int s = 0; s < S; ++s) {
          bf16x4 hi, lo;
          split_or_round<LO>(zb[s], hi, lo);
          if (t & 1) {
            zh[s][t >> 1] = cat8(ph[s], hi);
            if constexpr (LO) zl[s][t >> 1] = cat8(pl[s], lo);
          } else {
            ph[s] = hi;
            if constexpr (LO) pl[s] = lo;
          }
        }
      } else {
        first_layer_partials<WT, S, NSO>(sp, zb, xrow, d, t, w, p, g, accBslot, accK0);
      }
    }
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q) {
      if (q >= d.d_out) break;
      const float v = row16_sum(ub[0][q]);
      if (l == 0) accBo[w * TDQ_MAXO + q] = v;
    }
  }
  // output-layer slab now: its partials alias the images (the first dK pass starts with a barrier)
  __syncthreads();
  if (w == 2) {
    const int ko = off_layer(d, Lh);
    for (int e = l; e < hw(d, Lh - 1) * d.d_out; e += 64) {
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
      slab_put(gs + ko + hw(d, Lh - 1) * d.d_out + l, a);
    }
  }
  TDQ_TS(1);

  // ---- hidden layers i = Lh-1 .. 1: zh/zl hold zb_i --------------------------------------
  for (int i = Lh - 1; i >= 1; --i) {
    const int tsb = 2 + 8 * (Lh - 1 - i);
    const Tl Hp = hs_region<WT, LO>(Hs, i - 1, nwg_f, wg_f, S, w_f, l);
    // layer 0 under h0r: hp keeps the value stream, stream s is rebuilt from it (h0_stream)
    const bool rec0 = h0r && i == 1;
    // h_{i-1} tiles of stream 0 for the dK images
    f32x4 hp[WT];
#pragma unroll
    for (int t = 0; t < WT; ++t) hp[t] = hs_load_c<WT, LO>(Hp, 0, t);
    TDQ_TS(tsb);

#pragma unroll
    for (int pc = 0; pc < PC; ++pc) {
    if (pc > 0) {  // next column pass: the images are rebuilt from stream 0
#pragma unroll
      for (int t = 0; t < WT; ++t) hp[t] = hs_load_c<WT, LO>(Hp, 0, t);
    }
    // (c) dK_i = sum_points sum_streams h_{i-1} zb^T on bf16x3 MFMA, points on the k index
    f32x4 dw[NR][NCP];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NCP; ++c) dw[r][c] = zero4();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      // previous users of the region done: the zb stage (s = 0) / the last stream's images (one
      // buffer only; with two, the barrier after this stream's image writes already orders them
      // after the MFMAs of s - 1, the last readers of the buffer written here)
      if (s == 0 || !DBUF) __syncthreads();
      __bf16* const im = img + (DBUF ? (s & 1) * IBUF : 0);
      if (s == 0 && w == 0 && pc == 0) {  // bias of layer i: partials of all waves landed before this barrier
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
        const int wch = CHUNK_SWZ ? (g ^ ((row >> 2) & 3)) : g;  // swizzled 4-column chunk
#pragma unroll
        for (int t = 0; t < WT; ++t) {
          bf16x4 hi, lo;
          split_or_round<LO>(rec0 ? h0_stream<WT, S, NSO>(sp, aux, hp[t], t, g, s) : hp[t], hi, lo);
          const int off = row * RS + ((16 * t + 4 * wch) ^ rsw);
          *reinterpret_cast<bf16x4*>(im + IH + off) = hi;
          *reinterpret_cast<bf16x4*>(im + IZ + off) = half8(zh[s][t >> 1], t & 1);
          if constexpr (LO) {
            *reinterpret_cast<bf16x4*>(im + IHL + off) = lo;
            *reinterpret_cast<bf16x4*>(im + IZL + off) = half8(zl[s][t >> 1], t & 1);
          }
        }
      }
      if (s + 1 < S && !rec0) {  // next stream's h_{i-1} tiles fly while this stream's MFMAs run
#pragma unroll
        for (int t = 0; t < WT; ++t) hp[t] = hs_load_c<WT, LO>(Hp, s + 1, t);
      }
      __syncthreads();
      if (s == 0 && pc == 0) TDQ_TS(tsb + 1);
      // transposed-read bases of this wave's first row / column tile: the other tiles (+16 r / c
      // columns) and the second k-block (+32 rows) are immediate offsets of these addresses (adding
      // 16 r never crosses the swizzled bit 6: the bases' low six bits + 16 (NRB - 1) < 64)
      int ra1[RB], ra2[RB];
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        ra1[rb] = tr_row * RS + ((16 * (dw_row(w, 0) + NRB * rb) + tr_col1) ^ swz);
        ra2[rb] = (tr_row + 4) * RS + ((16 * (dw_row(w, 0) + NRB * rb) + tr_col2) ^ swz);
      }
      const int ca1 = tr_row * RS + ((16 * (dw_col(w, 0) + NCP * pc) + tr_col1) ^ swz);
      const int ca2 = (tr_row + 4) * RS + ((16 * (dw_col(w, 0) + NCP * pc) + tr_col2) ^ swz);
#pragma unroll
      for (int kb = 0; kb < PTS / 32; ++kb) {  // k-blocks of 32 points
        bf16x8 Ah[NR], Al[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int off = ra1[r / NRB] + 32 * kb * RS + 16 * (r % NRB);
          const int of2 = ra2[r / NRB] + 32 * kb * RS + 16 * (r % NRB);
          Ah[r] = cat8(tr_read(im + IH + off), tr_read(im + IH + of2));
          if constexpr (LO) Al[r] = cat8(tr_read(im + IHL + off), tr_read(im + IHL + of2));
        }
#pragma unroll
        for (int c = 0; c < NCP; ++c) {
          const int off = ca1 + 32 * kb * RS + 16 * c;
          const int of2 = ca2 + 32 * kb * RS + 16 * c;
          const bf16x8 Bh = cat8(tr_read(im + IZ + off), tr_read(im + IZ + of2));
          bf16x8 Bl;
          if constexpr (LO) Bl = cat8(tr_read(im + IZL + off), tr_read(im + IZL + of2));
#pragma unroll
          for (int r = 0; r < NR; ++r) dw[r][c] = mfma_aa<LO>(Ah[r], Al[r], Bh, Bl, dw[r][c]);
        }
      }
    }
    {
      // dK_i rows / columns this wave owns.  Unpadded width: one lane offset + uniform (r, c2, c)
      // offsets through a buffer resource (no per-store address VGPRs, no exec branches);
      // padded width: guarded stores.
      int in0 = 16 * dw_row(w, 0) + 4 * g, out0 = 16 * (dw_col(w, 0) + NCP * pc) + p;
      // opaque per iteration: otherwise LICM hoists the padded path's 64 guarded store addresses
      // (and their exec masks) out of the layer loop, where they stay live and spill
      asm volatile("" : "+v"(in0), "+v"(out0));
      ST* gk = gs + off_layer(d, i);
      if (d.uniform && d.width == W) {
        const Tl G = tl_make(gk, 0);
        constexpr int EB = (int)sizeof(ST);  // slab entry bytes
        const int voff = (in0 * W + out0) * EB;
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int c2 = 0; c2 < NCP; ++c2)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float v = dw[r][c2][c];
              if constexpr (SH)
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (__bf16)v), G.r, voff,
                                                      ((16 * r + c) * W + 16 * c2) * EB, 0);
              else
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), G.r, voff, ((16 * r + c) * W + 16 * c2) * 4, 0);
            }
      } else {
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int c2 = 0; c2 < NCP; ++c2)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const int in = in0 + 16 * r + c, out = out0 + 16 * c2;
              if (in < hw(d, i - 1) && out < hw(d, i)) slab_put(gk + in * hw(d, i) + out, dw[r][c2][c]);
            }
      }
    }
    }  // column passes
    TDQ_TS(tsb + 2);
    __syncthreads();  // images consumed: the region becomes the zb fragment stage
    TDQ_TS(tsb + 3);

    // (d) hb_{i-1} = K_i zb_i, fused with the adjoint of tanh layer i-1
    const Tl Ki = tl_make(Kimg + (size_t)(i - 1) * (WT * KB) * 128, l);
    if (i >= 2) {
      bwd_hidden_d<WT, S, NSO, LO, false>(zh, zl, Ki, Hp, stage, accB + ((i - 1) & 1) * NWV * W, accK0, xrow, sp, d, aux,
                                      h0r != 0, w, l, p, g);
      stage_fence<GST>();
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {  // wave-private stage: program order suffices
          zh[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[(((s * KB + kb) * HL + 0) * 64 + l) * 2]);
          if constexpr (LO) zl[s][kb] = *reinterpret_cast<const bf16x8*>(&stage[(((s * KB + kb) * HL + 1) * 64 + l) * 2]);
        }
    } else {
      bwd_hidden_d<WT, S, NSO, LO, true>(zh, zl, Ki, Hp, stage, accB + 2 * NWV * W, accK0, xrow, sp, d, aux, h0r != 0, w, l,
                                     p, g);
    }
    TDQ_TS(tsb + 4);
  }

  // ---- first-layer / output-layer slabs (partials of all waves are in LDS) ----------------
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
  TDQ_TS(63);
}

// ------------------------------------------------------------------------------------------
// host-side launch templates (instantiated per width class in jet_bf3_w{2,4,8}.hip)
// ------------------------------------------------------------------------------------------
#ifndef __HIPCC_RTC__
inline size_t fwd_bf3_lds(int WT, int S, bool lo) {
  return bf3_gstage(WT, S, lo) ? 0 : (size_t)2 * S * WT * 1024 * (lo ? 2 : 1);
}

// backward tile order: reverse (default) or dispatch order (TDQ_BWD_ORDER=forward, for A/B runs)
inline int bwd_reverse_order() {
  static const int rev = [] {
    const char* e = getenv("TDQ_BWD_ORDER");
    return (e != nullptr && e[0] == 'f') ? 0 : 1;
  }();
  return rev;
}

// layer-0 activations recomputed in the backward (default) or saved by the forward
// (TDQ_H0_RECOMPUTE=0, for A/B runs).  Read once per process: forward and backward always agree.
inline int h0_recompute() {
  static const int on = [] {
    const char* e = getenv("TDQ_H0_RECOMPUTE");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  return on;
}

inline size_t bwd_bf3_lds(int WT, int S, bool lo) {
  const int W = 16 * WT, hl = lo ? 2 : 1, nwv = bwd_waves(WT, lo, S);
  const size_t u1 = (size_t)(lo ? 1 : 2) * (2 * hl * 16 * nwv * bf3_img_rs(WT)) / 2,
               u2 = bf3_gstage(WT, S, lo) ? 0 : (size_t)nwv * S * WT * hl * 128;
  const size_t u = ((u1 > u2 ? u1 : u2) + 3) / 4 * 4;
  return (u + 3 * nwv * W) * sizeof(float);
}

struct Bf3Args {
  const float* X;
  const float* aux;
  const bf16x8* img;
  const float* dJ;   // bwd
  float* J;          // fwd
  float* Hs;
  float* slab;       // bwd
  int N, Ptot;
  NetDims d;
  JetSpec sp;
  hipStream_t st;
  int lo;            // 1: bf16x3 (operands hi + lo), 0: bf16 (operands rounded to bf16)
  bf16x4* gstage;    // wide bf16x3 plans: global fragment stage (bf3_gstage), else unused
  // point range [p_lo, p_hi) of this launch (p_lo a multiple of 128, p_hi one too or = N): the
  // kernels index J / dJ, the saved activations and the slabs of the whole set N, so launches
  // over disjoint ranges may run concurrently (separate streams) into the same buffers
  int p_lo = 0, p_hi = -1;
};

template <int WT, int S, int NSO, bool LO>
int launch_fwd_bf3_lo(const Bf3Args& a) {
  const int hi = a.p_hi < 0 ? a.N : a.p_hi, wg0 = a.p_lo / 64;
  const int nwg = (hi + 63) / 64 - wg0;
  const size_t lds = fwd_bf3_lds(WT, S, LO);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&jet_fwd_bf3_kernel<WT, S, NSO, LO>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((jet_fwd_bf3_kernel<WT, S, NSO, LO>), dim3(nwg), dim3(256), lds, a.st, a.X, a.aux, a.img, a.J,
                     a.Hs, a.N, a.d, a.sp, h0_recompute(), a.gstage, wg0);
  TDQ_CHECK_LAUNCH();
  return 0;
}

template <int WT, int S, int NSO>
int launch_fwd_bf3(const Bf3Args& a) {
  if constexpr (WT > 8) {  // widths 129..256: bf16 only (bf16x3 keeps the layer-wise engine)
    return a.lo ? (int)hipErrorInvalidValue : launch_fwd_bf3_lo<WT, S, NSO, false>(a);
  } else {
    return a.lo ? launch_fwd_bf3_lo<WT, S, NSO, true>(a) : launch_fwd_bf3_lo<WT, S, NSO, false>(a);
  }
}

template <int WT, int S, int NSO, bool LO>
int launch_bwd_bf3_lo(const Bf3Args& a) {
  constexpr int NWV = bwd_waves(WT, LO, S);
  const int hi = a.p_hi < 0 ? a.N : a.p_hi, wg0 = a.p_lo / (16 * NWV);
  const int nwg = (hi + 16 * NWV - 1) / (16 * NWV) - wg0;
  const size_t lds = bwd_bf3_lds(WT, S, LO);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&jet_bwd_bf3_kernel<WT, S, NSO, LO>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((jet_bwd_bf3_kernel<WT, S, NSO, LO>), dim3(nwg), dim3(64 * NWV), lds, a.st, a.X, a.aux, a.img, a.dJ,
                     a.Hs, a.slab, a.N, a.Ptot, a.d, a.sp, bwd_reverse_order(), h0_recompute(), a.gstage, wg0);
  TDQ_CHECK_LAUNCH();
  return 0;
}

template <int WT, int S, int NSO>
int launch_bwd_bf3(const Bf3Args& a) {
  if constexpr (WT > 8) {
    return a.lo ? (int)hipErrorInvalidValue : launch_bwd_bf3_lo<WT, S, NSO, false>(a);
  } else {
    return a.lo ? launch_bwd_bf3_lo<WT, S, NSO, true>(a) : launch_bwd_bf3_lo<WT, S, NSO, false>(a);
  }
}

// per-width-class entry points (jet_bf3_w{2,4,8}.hip); return hipErrorInvalidValue when
// (S, NSO) has no instantiation
int bf3_fwd_w2(int S, int nso, const Bf3Args& a);
int bf3_fwd_w4(int S, int nso, const Bf3Args& a);
int bf3_fwd_w8(int S, int nso, const Bf3Args& a);
int bf3_fwd_w16(int S, int nso, const Bf3Args& a);
int bf3_bwd_w2(int S, int nso, const Bf3Args& a);
int bf3_bwd_w4(int S, int nso, const Bf3Args& a);
int bf3_bwd_w8(int S, int nso, const Bf3Args& a);
int bf3_bwd_w16(int S, int nso, const Bf3Args& a);
#endif  // __HIPCC_RTC__
