// One-launch training step for precision "bf16" (gfx950 / MI355X): a persistent point-tile kernel
// that runs, per 32-point tile, the Taylor-jet forward of the network with every activation kept on
// chip (LDS images + registers), the per-point loss of the traced loss program (generated C++,
// compiled with hipRTC: ops/fused_step.py) and its reverse sweep, and the recompute-free backward -
// with the weight gradient dK of every hidden layer accumulated in MFMA accumulator registers
// across all of a workgroup's tiles.
//
// Why (profiles/r3_roofline_bf16.txt): the saved-activation design streams
// 4.35 KB per point out of the forward and back into the backward (223 + 268 MB per 50k-point
// step) at 2-4 TB/s, with the backward at 12 % MFMA busy and two wave rounds per launch.  Here:
//   * one workgroup (8 waves, two per SIMD) per CU, a static contiguous share of 32-point tiles per
//     workgroup (deterministic summation order);
//   * per tile, the forward writes each layer's post-activation streams into [point][feature]
//     bf16 LDS images - the B operand of the next layer's GEMM (two ds_read_b64 per fragment in
//     the permuted k order of the weight images) and, read transposed (ds_read_b64_tr_b16), the
//     A operand of the backward's dK = sum_points sum_streams h_{l-1} zb_l^T;
//   * the value stream keeps a bf16 "lo" image beside its hi image (hi + lo ~ 2^-17 relative) for
//     the tanh-jet adjoint's s1 = 1 - h^2;
//   * the reverse sweep writes each zb_l in place of h_l once every wave's dK_{l+1} has read
//     h_l; layer 0 (input -> width, VALU) is rebuilt from x instead of being kept;
//   * dK_l (l = 1..LM) lives in accumulators for the whole launch; vector-parameter partials
//     (biases, first / output layer) accumulate in LDS; one bf16 gradient-slab row and one loss-
//     partial row per workgroup at the end, reduced by the fused step tail (jet_bf3.hip).
// No activation or jet traffic through HBM: the kernel reads x, the loss inputs and the
// (L2-resident) weight images.
// Removed after measurement (tools/patches/fused_step_experiments_REMOVED.patch, A/B notes there):
// the MODE 0 / 1 forward-only and backward-only persistent launches (TDQ_FUSED=1), the dynamic
// tile queue (TDQ_FS_DYNAMIC), the loss inputs prefetched a tile ahead (TDQ_FS_PREFETCH), the
// cheap tanh in the hidden layers (FZ_CHEAP_TANH) and the weight-lo "bf16w" objective (WLO).
// The L-BFGS objective in bf16x3 runs the 16-point-tile kernel of jet_fused3.h.
// Reference behaviour: the nested tf.gradients of the PDE residual and its tape.gradient
// (tensordiffeq/models.py:116-225, fit.py:125-147).
#pragma once
#include "jet_bf3.h"

// Phase stamps (-DTDQ_PHASE_TIMING build, tools/fused_step_timing.py): the phases of tile
// t0 + FZ_TS_TILE of every workgroup (0: the first, cold tile; 1: a steady-state one) and the whole
// tile loop, per wave
#ifndef FZ_TS_TILE
#define FZ_TS_TILE 0
#endif
#define FZ_TS(k) \
  do {                \
    if (t == t0 + FZ_TS_TILE) TDQ_TS(k); \
  } while (0)

#define FZ_PT 32  // points per tile (two 16-point MFMA column tiles; waves 0-3 / 4-7)
#define FZ_WAVES 8

__host__ __device__ constexpr int fz_nslot(int LM) { return LM < 2 ? 2 : LM; }
// bf16 elements of the image area: every slot holds S stream images plus the value stream's lo image
__host__ __device__ constexpr int fz_img_elems(int WT, int S, int LM) {
  return (S + 1) * fz_nslot(LM) * FZ_PT * bf3_img_rs(WT);
}
// float area after the images: aux copy | xs | ubs | per-column-tile partials (biases of layers
// 0..LM, K0, Ko), bo | output-layer partial dots
__host__ __device__ inline int fz_aux_floats(const NetDims& d, int W) { return (aux_floats(d, W) + 3) / 4 * 4; }
__host__ __device__ inline int fz_fl_floats(const NetDims& d, int WT, int S, int LM) {
  const int W = 16 * WT;
  const int common = fz_aux_floats(d, W) + FZ_PT * TDQ_MAXD + S * FZ_PT * 4;
  const int part = 2 * ((LM + 1) * W + d.d_in * W + 4 * W) + 4;
  const int outp = 4 * S * FZ_PT;
  return common + part + outp + FZ_PT;  // + the loss's prefetched per-point input
}
__host__ __device__ inline int fz_lds_bytes(const NetDims& d, int WT, int S, int LM) {
  return fz_img_elems(WT, S, LM) * 2 + fz_fl_floats(d, WT, S, LM) * 4;
}

// Layer 0 (input -> width, VALU) of feature tile t at one point x (LDS row) - computed twice per
// tile in the bf16 step (forward, the h_0 image rebuild for dK_1 that the layer-0 adjoint then reads;
// three times in the bf16x3 objective, whose adjoint recomputes it), always by this function, so
// every pass sees the same h_0.  Its derivative streams are rows of K0: h_a = s1 K0[a],
// h_ab = s2 K0[a] K0[b] (z_ab = 0).
// CHEAP (the bf16 step): tanh z = 1 - 2 r, s1 = 4 e r^2 with e = exp(2 min(z, 15)), r = 1 / (1 + e)
// (exp, rcp and ~6 FMA-class ops; s1 from e, not 1 - h^2, which cancels for saturated units).  On
// the AC-SA reference schedule seeds 0-5 ended at L2 2.41 / 2.29 / 1.86 / 2.03 / 2.59 / 2.44e-2
// with it (median 2.35e-2, the separate-launch step's) and 1.45 / 2.63 / 3.17 / 3.02 / 3.43 /
// 2.57e-2 with tanh_s1 (profiles/r5acc2_l2_six_seeds.jsonl).  In the hidden layers the cheap form
// cost accuracy (L2 median 2.99e-2, profiles/r5acc_accuracy_ab.jsonl): they use tanh_jet_f.
// !CHEAP (the bf16x3 objective, jet_fused3.h): tanh_s1, the saved-activation kernels' tanh.
template <int WT, int S, int NSO, bool CHEAP = true, int DIN = 0>
__device__ __forceinline__ void fz_h0(const JetSpec& sp, const float* aux, const NetDims& d, const float* xrow, int t,
                                      int g, f32x4 (&h)[S]) {
  constexpr int S1 = S - 1 - NSO, SO = 1 + S1, W = 16 * WT;
  const int f0 = 16 * t + 4 * g;
  f32x4 z = *reinterpret_cast<const f32x4*>(aux + (DIN > 0 ? DIN * W : aux_b0(d, W)) + f0);
  if constexpr (DIN > 0) {  // compile-time input width (the generated fused-step kernels)
    // scalar FMAs, not f32x4 arithmetic: the vector form compiles to v_pk_fma_f32 whose result
    // the next-but-one VALU reads; in the layer-0 adjoint (right after the dK_1 MFMA burst) that
    // read returned stale lanes 48-63 of component 0 on some runs - b0 / K0 gradients of every
    // 12th-of-16 feature differed run to run (profiles/r6s_bf16_nondeterminism.md).  Scalar form:
    // bitwise reproducible, same step time.
    float x[DIN];
#pragma unroll
    for (int j = 0; j < DIN; ++j) x[j] = xrow[j];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float a = z[c];
#pragma unroll
      for (int j = 0; j < DIN; ++j) a = fmaf(x[j], aux[j * W + f0 + c], a);
      z[c] = a;
    }
  } else {
    for (int j = 0; j < d.d_in; ++j) z += xrow[j] * *reinterpret_cast<const f32x4*>(aux + j * W + f0);
  }
  f32x4 ka[S];
  ka[0] = zero4();
#pragma unroll
  for (int s = 1; s < SO; ++s) ka[s] = *reinterpret_cast<const f32x4*>(aux + sp.var[s] * W + f0);
#pragma unroll
  for (int s = SO; s < S; ++s) ka[s] = zero4();
  f32x4 kp[S];
#pragma unroll
  for (int s = SO; s < S; ++s) kp[s] = sel_first<S, S1>(ka, sp.ia[s], sp.selA[s]) * sel_first<S, S1>(ka, sp.ib[s], sp.selB[s]);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float hv, s1;
    if constexpr (CHEAP) {
      const float e = __builtin_amdgcn_exp2f(fminf(z[c], 15.f) * 2.8853900817779268f);
      const float r = __builtin_amdgcn_rcpf(1.f + e);
      hv = fmaf(-2.f, r, 1.f);
      s1 = (4.f * e) * (r * r);
    } else {
      tanh_s1(z[c], hv, s1);
    }
    const float s2 = -2.f * hv * s1;
    h[0][c] = hv;
#pragma unroll
    for (int s = 1; s < SO; ++s) h[s][c] = s1 * ka[s][c];
#pragma unroll
    for (int s = SO; s < S; ++s) h[s][c] = s2 * kp[s][c];
  }
}

// Image addressing.  Element (row, feature 16 t + 4 g + e) of a [point][feature] image with row
// stride RS lives at row * RS + ((16 t + 4 ch) ^ rsw) + e, ch = g ^ ((row >> 2) & 3) (4-column chunk
// swizzle), rsw = 64 * bit 3 of row (64-column half swap) - the backward images' conflict-free
// layout (jet_bf3.h).  For row = 16 q + p, (16 t + 4 ch) ^ rsw = 16 t + 4 ch + (bit 2 of t ? -rsw : rsw),
// so every access is one of two per-lane bases plus an offset that is uniform (t) or immediate
// (q, k-block, stream): no per-access address registers (the XOR form pinned one per access).
struct FzLane {
  int lo, r2;  // lane base for feature tiles with bit 2 of t clear; minus r2 (= 2 rsw) when set
};
template <int RS>
__device__ __forceinline__ FzLane fz_lane(int p, int g) {
  const int ch = g ^ ((p >> 2) & 3), rsw = (p & 8) << 3;
  return FzLane{p * RS + 4 * ch + rsw, 2 * rsw};
}
template <int RS>
__device__ __forceinline__ int fz_at(const FzLane& L, int q, int t) {
  // (arithmetic, not a select between two members: that became an indexed scratch load)
  return L.lo - ((t >> 2) & 1) * L.r2 + 16 * q * RS + 16 * t;
}
template <int RS>
__device__ __forceinline__ void fz_put(__bf16* im, const FzLane& L, int q, int t, bf16x4 v) {
  *reinterpret_cast<bf16x4*>(im + fz_at<RS>(L, q, t)) = v;
}
template <int RS>
__device__ __forceinline__ bf16x4 fz_get(const __bf16* im, const FzLane& L, int q, int t) {
  return *reinterpret_cast<const bf16x4*>(im + fz_at<RS>(L, q, t));
}
// B fragment of k-block kb (features in the weight images' permuted k order) for column tile q
template <int RS>
__device__ __forceinline__ bf16x8 fz_bfrag(const __bf16* im, const FzLane& L, int q, int kb) {
  return cat8(fz_get<RS>(im, L, q, 2 * kb), fz_get<RS>(im, L, q, 2 * kb + 1));
}
__device__ __forceinline__ f32x4 fz_bf4(bf16x4 v) {
  const u32x2 u = __builtin_bit_cast(u32x2, v);
  return f32x4{__uint_as_float(u[0] << 16), __uint_as_float(u[0] & 0xffff0000u), __uint_as_float(u[1] << 16),
               __uint_as_float(u[1] & 0xffff0000u)};
}

// acc[oo][s] = sum_kb A(o0 + oo, kb) B(kb, s) for the 16 points of column tile q: A from a weight
// image in global memory (hi only, one k-block ahead), B from the LDS image `im` (S stream images of
// FZ_PT rows; the SIMD's other wave covers the LDS latency).
template <int WT, int S, int OPW>
__device__ __forceinline__ void fz_gemm(f32x4 (&acc)[OPW][S], const bf16x8* __restrict__ wimg, int layer, int o0,
                                        const __bf16* im, int q, const FzLane& L, int l) {
  constexpr int KB = WT / 2, RS = bf3_img_rs(WT), SIMG = FZ_PT * RS, NSTEP = WT * KB;
  const Tl Wi = tl_make(wimg + (size_t)(layer - 1) * NSTEP * 128, l);
  bf16x8 a[2][OPW], alo[2][OPW];
#pragma unroll
  for (int oo = 0; oo < OPW; ++oo) img_frag<false>(Wi, (o0 + oo) * KB, a[0][oo], alo[0][oo]);
#pragma unroll
  for (int oo = 0; oo < OPW; ++oo)
#pragma unroll
    for (int s = 0; s < S; ++s) acc[oo][s] = zero4();
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + 1 < KB) {
#pragma unroll
      for (int oo = 0; oo < OPW; ++oo)
        img_frag<false>(Wi, (o0 + oo) * KB + kb + 1, a[(kb + 1) & 1][oo], alo[(kb + 1) & 1][oo]);
    }
    bf16x8 b[S];
#pragma unroll
    for (int s = 0; s < S; ++s) b[s] = fz_bfrag<RS>(im + s * SIMG, L, q, kb);
#pragma unroll
    for (int oo = 0; oo < OPW; ++oo)
#pragma unroll
      for (int s = 0; s < S; ++s) acc[oo][s] = mfma_bf(a[kb & 1][oo], b[s], acc[oo][s]);
    // (a scheduling barrier per k-block: without it the step took 0.152 vs 0.146 ms, gpurun_out r6n)
    __builtin_amdgcn_sched_barrier(0);
  }
}

// dK[r][c] += sum over the tile's points and streams of H^T Z (transposed LDS reads; the wave's
// NR x NC block of 16 x 16 output tiles at row tiles r0.., column tiles c0..).  The k index of
// each MFMA runs over 32 image rows: 32 points of one stream here (SIMG = FZ_PT * RS); the
// 16-point-tile kernel of jet_fused3.h passes two streams' 16-row images as one 32-row image.
template <int WT, int S, int NR, int NC, bool SB = true, int SIMG = FZ_PT * bf3_img_rs(WT)>
__device__ __forceinline__ void fz_dk(f32x4 (&dk)[NR][NC], const __bf16* H, const __bf16* Z, int r0, int c0, int l) {
  constexpr int RS = bf3_img_rs(WT);
  const int g = l >> 4;
  const int tr_row = 8 * g + ((l & 15) >> 2);
  const int swz = (g & 1) << 6;
  const int tr_col1 = 4 * ((l & 3) ^ ((2 * g) & 3)), tr_col2 = 4 * ((l & 3) ^ ((2 * g + 1) & 3));
  // (16 (r0 + r) + tr_col) ^ swz = ((16 r0) ^ swz) + 16 r + tr_col as long as no carry crosses
  // bit 6: blocks of 4 tiles start on multiples of 64 columns, blocks of 2 on multiples of 32 (and
  // 16 r + tr_col <= 28) - one base per read, immediates after
  static_assert((NR == 4 || NR <= 2) && (NC == 4 || NC <= 2), "fz_dk: tile blocks of 1, 2 or 4");
  const int a1 = tr_row * RS + tr_col1 + ((16 * r0) ^ swz), a2 = (tr_row + 4) * RS + tr_col2 + ((16 * r0) ^ swz);
  const int z1 = tr_row * RS + tr_col1 + ((16 * c0) ^ swz), z2 = (tr_row + 4) * RS + tr_col2 + ((16 * c0) ^ swz);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    bf16x8 A[NR], B[NC];
#pragma unroll
    for (int r = 0; r < NR; ++r) A[r] = cat8(tr_read(H + s * SIMG + a1 + 16 * r), tr_read(H + s * SIMG + a2 + 16 * r));
#pragma unroll
    for (int c = 0; c < NC; ++c) B[c] = cat8(tr_read(Z + s * SIMG + z1 + 16 * c), tr_read(Z + s * SIMG + z2 + 16 * c));
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) dk[r][c] = mfma_bf(A[r], B[c], dk[r][c]);
    if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
  }
}

// The fused loss's pointer table (csrc/loss_fused.hip LFPtrs, ops/loss_fused.py): value arrays,
// per-point SA weights and their gradients, scalar parameters
struct FzLossPtrs {
  const float* val[16];
  const float* lam[8];
  float* dlam[8];
  const float* scal[8];
};

struct FzParams {
  const float* X;
  const float* aux;
  const bf16x8* fimg;   // forward A image ([out][in] k order)
  const bf16x8* bimg;   // backward A image ([in][out])
  float* slab;          // gradient-slab rows srow + blockIdx.x
  int N, Pst, ntiles;
  int p_lo;             // the tiles cover points [p_lo, N)
  int srow;
  NetDims d;
  JetSpec sp;
  // the loss program's pointer table (the generated loss maps a point to its group)
  const FzLossPtrs* lptrs;
  float* lpart;         // loss / scalar-gradient partials, row prow + blockIdx.x, nacc floats each
  int prow, nacc;
};

// J of stream s at tile point k from the NW waves' partial output dots jv[(w * S + s) * PT + k]
// (summed in wave order, + the output bias on the value stream) - read by the generated loss
template <int S, int PT, int NW>
__device__ __forceinline__ float fz_jsum(const float* jv, int s, int k, float bo) {
  float a = jv[s * PT + k];
#pragma unroll
  for (int w = 1; w < NW; ++w) a += jv[(w * S + s) * PT + k];
  return s == 0 ? a + bo : a;
}

// The generated loss (ops/fused_step.py gen_loss) has this interface:
//   NACC: loss / scalar-gradient sums per point-thread;
//   eval<S, PT, NW>(jv, xs, t, n, N, ptrs, ubs, acc, pv, bo) on the tile's point-thread t (point n
//   of the fused point set): J of the tile's point k, stream s = fz_jsum(jv, s, k, bo), coordinates at
//   xs[k * TDQ_MAXD + j]; writes dJ of the points it owns to ubs[(s * PT + k) * 4] (zero for points
//   outside every loss group) and adds loss / scalar-gradient sums to acc;
//   pre(n, N, ptrs): the first per-point global input of point n's group (an SA weight or a data
//   value), which the kernel loads one tile ahead (with the coordinates) and passes in as pv - the
//   loss phase then waits for no global load on the common groups.
// Eight waves (two per SIMD, so one wave's tanh-jet VALU work runs beside the other's MFMAs):
// wave w computes column tile q = w >> 2 (16 points) of feature tiles 2 (w & 3).. (OPW of them) in
// every GEMM / epilogue, and owns an NR x NC block of each hidden layer's dK tiles.
template <int WT, int S, int NSO, int LM, class LossF>
__device__ __forceinline__ void fz_body(const FzParams& P, char* lds_raw) {
  const float* __restrict__ X = P.X;
  const float* __restrict__ aux_g = P.aux;
  const int N = P.N, Pst = P.Pst, ntiles = P.ntiles;
  const NetDims& d = P.d;
  // the stream spec and input width as compile-time constants of the generated loss struct
  // (ops/fused_step.py spec_source): the one-hot stream selects and first-layer loops fold away
  constexpr JetSpec sp = LossF::SPEC;
  constexpr int DIN = LossF::DIN;
  // compile-time aux-image / LDS offsets (d_in = DIN, n_hidden = LM + 1): LDS accesses then take
  // immediate offsets instead of runtime address arithmetic
  constexpr int W_ = 16 * WT;
  constexpr int A_B0 = DIN * W_, A_BH = (DIN + 1) * W_, A_KO = (DIN + LM + 1) * W_, A_BO = (DIN + LM + 5) * W_;
  constexpr int NAUX = (A_BO + 4 + 3) / 4 * 4;           // fz_aux_floats
  constexpr int W = 16 * WT, OPW = WT / 4, RS = bf3_img_rs(WT), SIMG = FZ_PT * RS;
  constexpr int NR = WT / 4, NC = WT / 2;  // dK tiles per wave: row block (w >> 1), column block (w & 1)
  constexpr int ZS = 0;                    // slot of h_LM / zb_LM (h_0's slot once layer 1 has read it)
  static_assert(OPW >= 1 && OPW * 4 == WT, "fused step: WT = 4 or 8");
  static_assert(LM >= 2, "fused step keeps h_LM in h_0's slot");
  __bf16* img = reinterpret_cast<__bf16*>(lds_raw);
  auto slot = [&](int k) { return img + k * (S + 1) * SIMG; };
  float* fl = reinterpret_cast<float*>(img + fz_img_elems(WT, S, LM));
  constexpr int naux = NAUX;
  float* aux = fl;                            // the aux image (biases, K0, Ko, bo), copied once
  float* xs = aux + naux;                     // [FZ_PT][TDQ_MAXD]
  float* ubs = xs + FZ_PT * TDQ_MAXD;         // [S][FZ_PT][4] dJ of the tile
  float* part = ubs + S * FZ_PT * 4;          // [2 column tiles][...] partials
  constexpr int pq = (LM + 1) * W + DIN * W + 4 * W;  // partial floats per column tile
  float* outp = part + 2 * pq + 4;            // [4][S][FZ_PT] output-layer dots
  float* lpre = outp + 4 * S * FZ_PT;         // [FZ_PT] the loss's prefetched first input

  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = w >> 2, wo = w & 3;
  const int G = gridDim.x, gi = blockIdx.x;
  const int t0 = (int)((long long)ntiles * gi / G), t1 = (int)((long long)ntiles * (gi + 1) / G);
  const int r0 = NR * (w >> 1), c0 = NC * (w & 1);  // dK block of this wave
  const int o0 = wo * OPW;                          // feature tiles of this wave (GEMM outputs)
  const int row = 16 * q + p;                       // this lane's point in the tile
  const FzLane L = fz_lane<RS>(p, g);
  float* accB = part + q * pq;                      // [LM + 1][W]  bias partials (layer 0..LM)
  float* accK0 = accB + (LM + 1) * W;               // [d_in][W]
  float* accKo = accK0 + d.d_in * W;                // [W][4]
  // Loop-invariant weight loads must not be hoisted out of the tile loop (they would pin ~100
  // VGPRs for the whole launch): the image pointers go through an opaque copy at every tile.
  const bf16x8* Wimg = P.fimg;
  const bf16x8* Kimg = P.bimg;

  // this thread's element of a tile's x (one: FZ_PT * TDQ_MAXD <= 512), fetched one tile ahead so
  // the global latency hides behind the current tile
  static_assert(FZ_PT * TDQ_MAXD + FZ_PT <= 64 * FZ_WAVES, "one element per thread");
  float xpre = 0.f;
  auto fetch = [&](int tt) {
    const int pb = P.p_lo + tt * FZ_PT;
    if (tid < FZ_PT * TDQ_MAXD) {
      const int pt = tid / TDQ_MAXD, j = tid - pt * TDQ_MAXD;
      const int n = min(pb + pt, N - 1);
      xpre = j < DIN ? X[(size_t)n * DIN + j] : 0.f;
    } else if (tid < FZ_PT * TDQ_MAXD + FZ_PT) {  // the loss's first per-point input (GenLoss::pre)
      xpre = LossF::pre(pb + tid - FZ_PT * TDQ_MAXD, N, *P.lptrs);
    }
  };
  if (t0 < t1) fetch(t0);  // first, so its latency overlaps the set-up below
  // warm this XCD's L2 with the weight images before the first tile's GEMMs: the workgroups of an
  // XCD (blocks gi, gi + 8, ... when the dispatcher deals them round-robin) each touch a slice (the
  // first tile's GEMMs ran 500-800 cycles slower each without: step 0.1429 -> 0.1400 ms,
  // profiles/r6x_weight_prefetch_ab.txt)
  bf16x8 wpf[2];
  {
    constexpr int NI16 = LM * WT * (WT / 2) * 128 * 4 * 4 / 16;  // 16-byte granules per image
    const int xw = gi >> 3, nx = (G + 7) >> 3;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = (xw + k * nx) * 64 * FZ_WAVES + tid;
      wpf[k] = e < 2 * NI16 ? (e < NI16 ? P.fimg[e] : P.bimg[e - NI16]) : bf16x8{};
    }
  }
  for (int e = tid; e < naux; e += 64 * FZ_WAVES) aux[e] = e < aux_floats(d, W) ? aux_g[e] : 0.f;
  asm volatile("" ::"v"(wpf[0]), "v"(wpf[1]));
  f32x4 dk[LM][NR][NC];
  float lacc[LossF::NACC];  // this point-thread's loss / scalar-gradient sums (all tiles)
  float bo_acc = 0.f;       // this point-thread's output-bias gradient (its points' value-stream dJ)
#pragma unroll
  for (int k = 0; k < LossF::NACC; ++k) lacc[k] = 0.f;
#pragma unroll
  for (int i = 0; i < LM; ++i)
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) dk[i][r][c] = zero4();
  for (int e = tid; e < 2 * pq + 4; e += 64 * FZ_WAVES) part[e] = 0.f;
  const float* Ko = aux + A_KO;

  // layer 0 (input -> width, VALU) of feature tile o0 + oo at this lane's point
  auto layer0 = [&](int oo, f32x4(&h)[S]) { fz_h0<WT, S, NSO, true, DIN>(sp, aux, d, xs + row * TDQ_MAXD, o0 + oo, g, h); };


  int t = t0;
  TDQ_TS(0);
  while (t < t1) {
    const int pb = P.p_lo + t * FZ_PT;
    asm volatile("" : "+s"(Wimg), "+s"(Kimg));
    __syncthreads();  // the previous tile's readers of xs / ubs / images are done (and aux / part set)
    if (tid < FZ_PT * TDQ_MAXD) xs[tid] = xpre;
    else if (tid < FZ_PT * TDQ_MAXD + FZ_PT) lpre[tid - FZ_PT * TDQ_MAXD] = xpre;
    if (t + 1 < t1) fetch(t + 1);
    __syncthreads();
    FZ_TS(1);

    // ---- layer 0 -> slot 0 ----------------------------------------------------------------
#pragma unroll
    for (int oo = 0; oo < OPW; ++oo) {
      f32x4 h[S];
      layer0(oo, h);
#pragma unroll
      for (int s = 0; s < S; ++s) fz_put<RS>(slot(0) + s * SIMG, L, q, o0 + oo, cvt_hi4(h[s]));
    }
    __syncthreads();
    FZ_TS(2);

    // ---- hidden layers 1..LM on MFMA ------------------------------------------------------
#pragma unroll
    for (int ly = 1; ly <= LM; ++ly) {
      const float* bi = aux + A_BH + (ly - 1) * W;
      f32x4 acc[OPW][S];
      fz_gemm<WT, S, OPW>(acc, Wimg, ly, o0, slot(ly - 1), q, L, l);
      FZ_TS(1 + 2 * ly);
      f32x4 hq[OPW][S];  // top layer: the streams for the output dots
#pragma unroll
      for (int oo = 0; oo < OPW; ++oo) {
        const int to = o0 + oo;
        f32x4 z[S], h[S];
#pragma unroll
        for (int s = 0; s < S; ++s) z[s] = acc[oo][s];
        z[0] += *reinterpret_cast<const f32x4*>(bi + 16 * to + 4 * g);
        tanh_jet_f<S, NSO>(sp, z, h);
        // h_l into slot l; h_LM waits in h_0's slot (hi / lo value) for the loss
        __bf16* im = slot(ly < LM ? ly : ZS);
        bf16x4 hi, lo;
        split4(h[0], hi, lo);
        fz_put<RS>(im, L, q, to, hi);
        fz_put<RS>(im + S * SIMG, L, q, to, lo);
#pragma unroll
        for (int s = 1; s < S; ++s) fz_put<RS>(im + s * SIMG, L, q, to, cvt_hi4(h[s]));
        if (ly == LM) {
#pragma unroll
          for (int s = 0; s < S; ++s) hq[oo][s] = h[s];
        }
      }
      if (ly == LM) {  // output-layer partial dots of this wave's features -> LDS
#pragma unroll
        for (int s = 0; s < S; ++s) {
          float a = 0.f;
#pragma unroll
          for (int oo = 0; oo < OPW; ++oo)
#pragma unroll
            for (int c = 0; c < 4; ++c) a = fmaf(hq[oo][s][c], Ko[(16 * (o0 + oo) + 4 * g + c) * 4], a);
          const float r = col4_sum(a);
          if (g == 0) outp[(wo * S + s) * FZ_PT + row] = r;
        }
      }
      __syncthreads();
      FZ_TS(2 + 2 * ly);
    }

    // ---- the per-point loss (generated code: every loss group of the program - residual, SA
    // weighting, boundary terms with the two points of a periodic pair side by side - and its
    // reverse sweep) -> dJ of the tile's points into ubs -----------------------------------
    // (J = the four wo-waves' partial dots, summed inside the loss: one phase and one barrier
    // fewer, 0.1383 -> 0.1376 ms, profiles/r6ag_jsum_ab.txt)
    int tl = tid;
    asm volatile("" : "+v"(tl));
    if (tl < FZ_PT) LossF::template eval<S, FZ_PT, 4>(outp, xs, tl, pb + tl, N, *P.lptrs, ubs, lacc, lpre[tl], aux[A_BO]);
    __syncthreads();
    FZ_TS(9);
    // dbo: each point-thread adds its point's value-stream dJ (one LDS read; a 32-step loop on
    // four lanes of wave 0 used to hold that wave - and the next barrier - for ~1-2k cycles)
    tl = tid;
    asm volatile("" : "+v"(tl));
    if (tl < FZ_PT) bo_acc += ubs[tl * 4];
    // ---- reverse through the output layer: hb = Ko ub, dKo, the top tanh layer's adjoint ----
#pragma unroll
    for (int oo = 0; oo < OPW; ++oo) {
      const int to = o0 + oo;
      __bf16* im = slot(ZS);
      f32x4 h[S], hb[S], zb[S];
      h[0] = fz_bf4(fz_get<RS>(im, L, q, to)) + fz_bf4(fz_get<RS>(im + S * SIMG, L, q, to));
#pragma unroll
      for (int s = 1; s < S; ++s) h[s] = fz_bf4(fz_get<RS>(im + s * SIMG, L, q, to));
      f32x4 kq, pp = zero4();
#pragma unroll
      for (int c = 0; c < 4; ++c) kq[c] = Ko[(16 * to + 4 * g + c) * 4];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const float ub = ubs[(s * FZ_PT + row) * 4];
        hb[s] = kq * ub;
        pp += h[s] * ub;
      }
      {
        const float r = row16_sum4(pp);
        if ((p & 3) == 0) accKo[(16 * to + 4 * g + (p >> 2)) * 4] += r;
      }
      tanh_jet_b<S, NSO>(sp, h, hb, zb);
      const float r = row16_sum4(zb[0]);
      if ((p & 3) == 0) accB[LM * W + 16 * to + 4 * g + (p >> 2)] += r;
#pragma unroll
      for (int s = 0; s < S; ++s) fz_put<RS>(im + s * SIMG, L, q, to, cvt_hi4(zb[s]));
    }
    __syncthreads();
    // ---- hidden layers LM..1: dK_l, hb_{l-1} = K_l zb_l, adjoint of tanh layer l-1 --------
#pragma unroll
    for (int ly = LM; ly >= 1; --ly) {
      const __bf16* Z = slot(ly == LM ? ZS : ly);
      __bf16* H = slot(ly - 1);
      const int tb = 10 + 5 * (LM - ly);
      f32x4 acc[OPW][S];
      fz_gemm<WT, S, OPW>(acc, Kimg, ly, o0, Z, q, L, l);
      FZ_TS(tb);
      // the tanh-jet adjoint (VALU) and dK_ly (MFMA: every wave reads all of H and Z) in one
      // scheduling region; zb_{ly-1} goes in place of h_{ly-1} after the barrier
      bf16x4 zbh[OPW][S];
      float rb[OPW];
      if (ly >= 2) {
#pragma unroll
        for (int oo = 0; oo < OPW; ++oo) {
          const int to = o0 + oo;
          f32x4 h[S], zb[S];
          h[0] = fz_bf4(fz_get<RS>(H, L, q, to)) + fz_bf4(fz_get<RS>(H + S * SIMG, L, q, to));
#pragma unroll
          for (int s = 1; s < S; ++s) h[s] = fz_bf4(fz_get<RS>(H + s * SIMG, L, q, to));
          tanh_jet_b<S, NSO>(sp, h, acc[oo], zb);
          rb[oo] = row16_sum4(zb[0]);
#pragma unroll
          for (int s = 0; s < S; ++s) zbh[oo][s] = cvt_hi4(zb[s]);
        }
      }
      fz_dk<WT, S, NR, NC, false>(dk[ly - 1], H, Z, r0, c0, l);
      FZ_TS(tb + 1);
      if (ly >= 2) {
        __syncthreads();  // every wave's dK reads of H are done
        FZ_TS(tb + 2);
#pragma unroll
        for (int oo = 0; oo < OPW; ++oo) {
          const int to = o0 + oo;
          if ((p & 3) == 0) accB[(ly - 1) * W + 16 * to + 4 * g + (p >> 2)] += rb[oo];
#pragma unroll
          for (int s = 0; s < S; ++s) fz_put<RS>(H + s * SIMG, L, q, to, zbh[oo][s]);
        }
      } else {
        // layer 0: zb_0 from h_0 (the slot-0 image the ly = 2 step rebuilt) -> first-layer
        // partials (K0, b0)
#pragma unroll
        for (int oo = 0; oo < OPW; ++oo) {
          const int to = o0 + oo;
          f32x4 h[S], zb[S];
          h[0] = fz_bf4(fz_get<RS>(H, L, q, to)) + fz_bf4(fz_get<RS>(H + S * SIMG, L, q, to));
#pragma unroll
          for (int s = 1; s < S; ++s) h[s] = fz_bf4(fz_get<RS>(H + s * SIMG, L, q, to));
          tanh_jet_b<S, NSO>(sp, h, acc[oo], zb);
          const int fo = 16 * to + 4 * g + (p >> 2);
          {
            const float r = row16_sum4(zb[0]);
            if ((p & 3) == 0) accB[fo] += r;
          }
#pragma unroll
          for (int j = 0; j < DIN; ++j) {
            const float xj = xs[row * TDQ_MAXD + j];
            f32x4 vv;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              float a = xj * zb[0][c];
              constexpr int SO = S - NSO;
#pragma unroll
              for (int s = 1; s < SO; ++s) a += (sp.var[s] == j) ? zb[s][c] : 0.f;
              vv[c] = a;
            }
            const float r = row16_sum4(vv);
            if ((p & 3) == 0) accK0[j * W + fo] += r;
          }
        }
      }
      FZ_TS(tb + 3);
      if (ly == 2) {  // rebuild h_0 into slot 0 (zb_LM there is consumed)
        if (LM == 2) __syncthreads();  // (LM = 2: it was this step's Z)
#pragma unroll
        for (int oo = 0; oo < OPW; ++oo) {
          f32x4 h[S];
          layer0(oo, h);
          // with the value stream's lo plane, as the hidden layers' images: the layer-0 adjoint
          // (ly = 1) reads h_0 back from here instead of recomputing layer 0 a third time (step
          // 0.1425 vs 0.1452 ms, L2 median 2.23e-2 vs 2.16e-2 - seed noise; fp64 gradient 2.8e-3
          // either way: profiles/r6w_l0_image_ab.txt)
          bf16x4 hi, lo;
          split4(h[0], hi, lo);
          fz_put<RS>(slot(0), L, q, o0 + oo, hi);
          fz_put<RS>(slot(0) + S * SIMG, L, q, o0 + oo, lo);
#pragma unroll
          for (int s = 1; s < S; ++s) fz_put<RS>(slot(0) + s * SIMG, L, q, o0 + oo, cvt_hi4(h[s]));
        }
      }
      if (ly >= 2) __syncthreads();
      FZ_TS(tb + 4);
    }
    ++t;
  }
  TDQ_TS(62);

  // ---- this workgroup's gradient-slab row (bf16) ---------------------------------------------
  __bf16* gs = reinterpret_cast<__bf16*>(P.slab) + (size_t)(P.srow + gi) * Pst;
#pragma unroll
  for (int ly = 1; ly <= LM; ++ly) {
    const int voff = ((16 * r0 + 4 * g) * W + 16 * c0 + p) * 2;
    const Tl Gt = tl_make(gs + off_layer(d, ly), 0);
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (__bf16)dk[ly - 1][r][c][e]),
                                                Gt.r, voff, ((16 * r + e) * W + 16 * c) * 2, 0);
  }
  __syncthreads();  // LDS partials complete
  const float* pA = part;
  const float* pB = part + pq;
  for (int f = tid; f < W; f += 64 * FZ_WAVES) {
    gs[d.d_in * W + f] = (__bf16)(pA[f] + pB[f]);  // b0
    for (int ly = 1; ly <= LM; ++ly)
      gs[off_layer(d, ly) + W * W + f] = (__bf16)(pA[ly * W + f] + pB[ly * W + f]);
    for (int j = 0; j < d.d_in; ++j) {
      const int k = (LM + 1) * W + j * W + f;
      gs[j * W + f] = (__bf16)(pA[k] + pB[k]);
    }
    for (int qo = 0; qo < d.d_out; ++qo) {
      const int k = (LM + 1 + d.d_in) * W + f * 4 + qo;
      gs[off_layer(d, LM + 1) + f * d.d_out + qo] = (__bf16)(pA[k] + pB[k]);
    }
  }
  // the output bias (d_out = 1) and the loss partials: the point-threads (wave 0, lanes < FZ_PT) summed
  if (w == 0) {
    const float bo = col4_sum(row16_sum(bo_acc));
    if (l == 0) gs[off_layer(d, LM + 1) + W] = (__bf16)bo;
#pragma unroll
    for (int k = 0; k < LossF::NACC; ++k) {
      const float v = col4_sum(row16_sum(lacc[k]));
      if (l == 0 && k < P.nacc) P.lpart[(size_t)(P.prow + gi) * P.nacc + k] = v;
    }
  }
  TDQ_TS(63);
}

#ifndef __HIPCC_RTC__
// jet_fused.hip
int fz_cus();
extern "C" int tdq_jet_fused_lds(int d_in, const int* widths, int d_out, int n_hidden, int S, int lo);
#endif  // __HIPCC_RTC__
