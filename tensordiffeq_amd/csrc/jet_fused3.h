// One-launch L-BFGS objective for precision "bf16x3" (gfx950 / MI355X): forward -> per-point loss
// -> recompute-free backward of every point in ONE persistent launch, like the bf16 step of
// jet_fused.h, but with every GEMM operand split into bf16 hi + lo (three MFMAs per product,
// ~2^-16 relative error: the accuracy the L-BFGS curvature pairs need - all-bf16 L-BFGS stalls at
// AC-SA L2 6-7e-2, weight-lo-only "bf16w" diverged, profiles/r5wlo2_bf16w_lbfgs.json).
//
// Layout: the lo planes of every activation stream double the LDS images, so
// a tile is 16 points (one MFMA column tile) instead of 32:
//   * slot k = [SP hi images][SP lo images] of 16 rows x RS bf16 (SP = S rounded up to even; a
//     padding stream's images stay zero) + an fp32 image of the value stream, whose s1 = 1 - h^2
//     in the tanh-jet adjoint must not see the hi + lo rounding (a saturated unit's s1 ~ 1e-5
//     would lose most digits) - the saved-activation kernels keep that stream fp32 too;
//   * 8 waves (two per SIMD), wave w owns feature tile w of every GEMM / epilogue (16 x 16
//     outputs per stream, 12 MFMAs per k-block) and the same 2 x 4 block of dK tiles as the bf16
//     step;
//   * dK = sum over points and streams of h_{l-1} zb_l^T takes two streams per MFMA: two
//     streams' 16-row images are adjacent, so they read as ONE 32-row image (k = 16 points x 2
//     streams) with the bf16 step's transposed-read addressing (fz_dk) - the row swizzle depends
//     on row bits 2-3 only, so rows 16-31 of the pair match rows 0-15 of the next image;
//   * fp32 gradient-slab rows (the bf16x3 backward's), loss partials as in the bf16 step.
// Tiles per 50k-point step: 3,183 over ~245 workgroups (13 rounds).  The weight images (hi + lo)
// are re-read from L2 per tile: 4 KB per point per GEMM.
// Reference: the L-BFGS objective loss + flat gradient of tensordiffeq/models.py:283-295 (the
// lua-port loop of optimizers.py:107-308 calls it once per iteration).
#pragma once
#include "jet_fused.h"

#define FZ3_PT 16  // points per tile (one 16-point MFMA column tile)

__host__ __device__ constexpr int fz3_sp(int S) { return (S + 1) / 2 * 2; }
__host__ __device__ constexpr int fz3_vrs() { return 132; }  // fp32 value image row stride (floats)
// bytes of one slot: 2 SP bf16 images + the fp32 value image
__host__ __device__ constexpr int fz3_slot_bytes(int WT, int S) {
  return 2 * fz3_sp(S) * FZ3_PT * bf3_img_rs(WT) * 2 + FZ3_PT * fz3_vrs() * 4;
}
// float area after the slots: aux copy | xs | ubs | partials (biases of layers 0..LM, K0, Ko), bo |
// output-layer partial dots [8 waves][S][FZ3_PT]
__host__ __device__ inline int fz3_fl_floats(const NetDims& d, int WT, int S, int LM) {
  const int W = 16 * WT;
  return fz_aux_floats(d, W) + FZ3_PT * TDQ_MAXD + S * FZ3_PT * 4 + ((LM + 1) * W + d.d_in * W + 4 * W) + 4 +
         FZ_WAVES * S * FZ3_PT + FZ3_PT;  // + the loss's prefetched per-point input
}
__host__ __device__ inline int fz3_lds_bytes(const NetDims& d, int WT, int S, int LM) {
  return fz_nslot(LM) * fz3_slot_bytes(WT, S) + fz3_fl_floats(d, WT, S, LM) * 4;
}

// A fragments (hi + lo, every k-block) of one GEMM's weight-image rows, all issued at the GEMM's
// start (one L2 latency per GEMM).  Issuing them one phase ahead (right after the previous GEMM's
// MFMAs, so the latency hides behind the epilogue / loss) measured SLOWER: 430 vs 324 us per
// objective evaluation - the 32 extra live VGPRs spilled (28 vs 12, gpurun_out r6e)
template <int WT>
struct Fz3W {
  bf16x8 h[WT / 2], l[WT / 2];
};
template <int WT>
__device__ __forceinline__ void fz3_load_w(Fz3W<WT>& w, const bf16x8* __restrict__ wimg, int layer, int o, int l) {
  constexpr int KB = WT / 2, NSTEP = WT * KB;
  const Tl Wi = tl_make(wimg + (size_t)(layer - 1) * NSTEP * 128, l);
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) img_frag<true>(Wi, o * KB + kb, w.h[kb], w.l[kb]);
}

// acc[s] = sum_kb A(o, kb) B(kb, s), both split: A from the preloaded weight fragments, B from the
// slot's hi / lo images; three MFMAs per product (lo terms first, as mfma3)
template <int WT, int S>
__device__ __forceinline__ void fz3_gemm(f32x4 (&acc)[S], const Fz3W<WT>& w, const __bf16* im, const FzLane& L) {
  constexpr int KB = WT / 2, RS = bf3_img_rs(WT), SIMG = FZ3_PT * RS, SP = fz3_sp(S);
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = zero4();
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    bf16x8 bh[S], bl[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      bh[s] = fz_bfrag<RS>(im + s * SIMG, L, 0, kb);
      bl[s] = fz_bfrag<RS>(im + (SP + s) * SIMG, L, 0, kb);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) acc[s] = mfma3(w.h[kb], w.l[kb], bh[s], bl[s], acc[s]);
    // (a scheduling barrier per k-block: without it the step took 0.152 vs 0.146 ms, gpurun_out r6n)
    __builtin_amdgcn_sched_barrier(0);
  }
}

// dK[r][c] += H^T Z over the tile's 16 points and S streams, two streams per MFMA (a pair's two
// 16-row images read as one 32-row image), hi / lo split on both sides
template <int WT, int S, int NR, int NC>
__device__ __forceinline__ void fz3_dk(f32x4 (&dk)[NR][NC], const __bf16* H, const __bf16* Z, int r0, int c0, int l) {
  constexpr int RS = bf3_img_rs(WT), SIMG = FZ3_PT * RS, SP = fz3_sp(S);
  const int g = l >> 4;
  const int tr_row = 8 * g + ((l & 15) >> 2);
  const int swz = (g & 1) << 6;
  const int tr_col1 = 4 * ((l & 3) ^ ((2 * g) & 3)), tr_col2 = 4 * ((l & 3) ^ ((2 * g + 1) & 3));
  const int a1 = tr_row * RS + tr_col1 + ((16 * r0) ^ swz), a2 = (tr_row + 4) * RS + tr_col2 + ((16 * r0) ^ swz);
  const int z1 = tr_row * RS + tr_col1 + ((16 * c0) ^ swz), z2 = (tr_row + 4) * RS + tr_col2 + ((16 * c0) ^ swz);
#pragma unroll
  for (int pr = 0; pr < SP / 2; ++pr) {
    const __bf16* Hh = H + 2 * pr * SIMG;
    const __bf16* Hl = H + (SP + 2 * pr) * SIMG;
    const __bf16* Zh = Z + 2 * pr * SIMG;
    const __bf16* Zl = Z + (SP + 2 * pr) * SIMG;
    bf16x8 Ah[NR], Al[NR], Bh[NC], Bl[NC];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      Ah[r] = cat8(tr_read(Hh + a1 + 16 * r), tr_read(Hh + a2 + 16 * r));
      Al[r] = cat8(tr_read(Hl + a1 + 16 * r), tr_read(Hl + a2 + 16 * r));
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      Bh[c] = cat8(tr_read(Zh + z1 + 16 * c), tr_read(Zh + z2 + 16 * c));
      Bl[c] = cat8(tr_read(Zl + z1 + 16 * c), tr_read(Zl + z2 + 16 * c));
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) dk[r][c] = mfma3(Ah[r], Al[r], Bh[c], Bl[c], dk[r][c]);
  }
}

// the fp32 value image: element (point p, feature f) at p * fz3_vrs() + f (row stride 132 floats:
// the 16 rows of a lane group's f32x4 reads land on distinct banks)
__device__ __forceinline__ float* fz3_vimg(__bf16* slot, int WT, int S) {
  return reinterpret_cast<float*>(slot + 2 * fz3_sp(S) * FZ3_PT * bf3_img_rs(WT));
}

// the post-activation streams of one feature tile -> a slot: hi + lo of every stream, the value
// stream also in fp32
template <int WT, int S>
__device__ __forceinline__ void fz3_put_h(__bf16* slot, const FzLane& L, int t, const f32x4 (&h)[S], float* vrow) {
  constexpr int RS = bf3_img_rs(WT), SIMG = FZ3_PT * RS, SP = fz3_sp(S);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    bf16x4 hi, lo;
    split4(h[s], hi, lo);
    fz_put<RS>(slot + s * SIMG, L, 0, t, hi);
    fz_put<RS>(slot + (SP + s) * SIMG, L, 0, t, lo);
  }
  *reinterpret_cast<f32x4*>(vrow) = h[0];
}
// the streams of one feature tile from a slot (value stream from the fp32 image)
template <int WT, int S>
__device__ __forceinline__ void fz3_get_h(const __bf16* slot, const FzLane& L, int t, f32x4 (&h)[S], const float* vrow) {
  constexpr int RS = bf3_img_rs(WT), SIMG = FZ3_PT * RS, SP = fz3_sp(S);
  h[0] = *reinterpret_cast<const f32x4*>(vrow);
#pragma unroll
  for (int s = 1; s < S; ++s)
    h[s] = fz_bf4(fz_get<RS>(slot + s * SIMG, L, 0, t)) + fz_bf4(fz_get<RS>(slot + (SP + s) * SIMG, L, 0, t));
}

template <int WT, int S, int NSO, int LM, class LossF>
__device__ __forceinline__ void fz3_body(const FzParams& P, char* lds_raw) {
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
  constexpr int W = 16 * WT, RS = bf3_img_rs(WT), SIMG = FZ3_PT * RS, SP = fz3_sp(S), VRS = fz3_vrs();
  constexpr int NR = WT / 4, NC = WT / 2;  // dK tiles per wave: row block (w >> 1), column block (w & 1)
  constexpr int SLOT = fz3_slot_bytes(WT, S), PT = FZ3_PT;
  static_assert(WT == 8, "bf16x3 fused step: width 128");
  static_assert(LM >= 2, "bf16x3 fused step keeps h_LM in h_0's slot");
  static_assert(SLOT % 16 == 0, "slot alignment");
  auto slot = [&](int k) { return reinterpret_cast<__bf16*>(lds_raw + k * SLOT); };
  float* fl = reinterpret_cast<float*>(lds_raw + fz_nslot(LM) * SLOT);
  constexpr int naux = NAUX;
  float* aux = fl;                            // the aux image (biases, K0, Ko, bo), copied once
  float* xs = aux + naux;                     // [PT][TDQ_MAXD]
  float* ubs = xs + PT * TDQ_MAXD;            // [S][PT][4] dJ of the tile
  float* part = ubs + S * PT * 4;             // partials
  constexpr int pq = (LM + 1) * W + DIN * W + 4 * W;
  float* outp = part + pq + 4;                // [8 waves][S][PT] output-layer dots
  float* lpre = outp + FZ_WAVES * S * PT;     // [PT] the loss's prefetched first input

  const int tid = threadIdx.x, l = tid & 63, p = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, gi = blockIdx.x;
  const int t0 = (int)((long long)ntiles * gi / G), t1 = (int)((long long)ntiles * (gi + 1) / G);
  const int r0 = NR * (w >> 1), c0 = NC * (w & 1);  // dK block of this wave
  const int o = w;                                  // feature tile of this wave (GEMM outputs)
  const FzLane L = fz_lane<RS>(p, g);
  const int voff = p * VRS + 16 * o + 4 * g;        // this lane's f32x4 in a value image
  float* accB = part;                               // [LM + 1][W]  bias partials (layer 0..LM)
  float* accK0 = accB + (LM + 1) * W;               // [d_in][W]
  float* accKo = accK0 + d.d_in * W;                // [W][4]
  const bf16x8* Wimg = P.fimg;
  const bf16x8* Kimg = P.bimg;

  float xpre = 0.f;
  auto fetch = [&](int tt) {
    const int pb = P.p_lo + tt * PT;
    if (tid < PT * TDQ_MAXD) {
      const int pt = tid / TDQ_MAXD, j = tid - pt * TDQ_MAXD;
      const int n = min(pb + pt, N - 1);
      xpre = j < DIN ? X[(size_t)n * DIN + j] : 0.f;
    } else if (tid < PT * TDQ_MAXD + PT) {  // the loss's first per-point input (GenLoss::pre)
      xpre = LossF::pre(pb + tid - PT * TDQ_MAXD, N, *P.lptrs);
    }
  };
  if (t0 < t1) fetch(t0);  // first, so its latency overlaps the set-up below
  // this XCD's L2 warmed with the weight images (hi and lo) before the first tile (as fz_body)
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
  for (int e = tid; e < pq + 4; e += 64 * FZ_WAVES) part[e] = 0.f;
  if constexpr (SP != S) {  // the padding stream's images (hi, lo) of every slot stay zero
    for (int k = 0; k < fz_nslot(LM); ++k)
      for (int e = tid; e < SIMG; e += 64 * FZ_WAVES) {
        slot(k)[S * SIMG + e] = (__bf16)0.f;
        slot(k)[(SP + S) * SIMG + e] = (__bf16)0.f;
      }
  }
  f32x4 dk[LM][NR][NC];
  float lacc[LossF::NACC];
  float bo_acc = 0.f;  // this point-thread's output-bias gradient (its points' value-stream dJ)
#pragma unroll
  for (int k = 0; k < LossF::NACC; ++k) lacc[k] = 0.f;
#pragma unroll
  for (int i = 0; i < LM; ++i)
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c) dk[i][r][c] = zero4();
  const float* Ko = aux + A_KO;

  // layer 0 (input -> width, VALU; the accurate tanh) of this wave's feature tile at this lane's point
  auto layer0 = [&](f32x4(&h)[S]) { fz_h0<WT, S, NSO, false, DIN>(sp, aux, d, xs + p * TDQ_MAXD, o, g, h); };

  static_assert(PT * TDQ_MAXD <= 64 * FZ_WAVES, "one element per thread");

  int t = t0;
  Fz3W<WT> wf;  // a GEMM's weight fragments
  TDQ_TS(0);
  while (t < t1) {
    const int pb = P.p_lo + t * PT;
    asm volatile("" : "+s"(Wimg), "+s"(Kimg));
    __syncthreads();  // the previous tile's readers of xs / ubs / images are done (and aux / part set)
    if (tid < PT * TDQ_MAXD) xs[tid] = xpre;
    else if (tid < PT * TDQ_MAXD + PT) lpre[tid - PT * TDQ_MAXD] = xpre;
    if (t + 1 < t1) fetch(t + 1);
    __syncthreads();
    FZ_TS(1);

    // ---- layer 0 -> slot 0 ----------------------------------------------------------------
    {
      f32x4 h[S];
      layer0(h);
      fz3_put_h<WT, S>(slot(0), L, o, h, fz3_vimg(slot(0), WT, S) + voff);
    }
    __syncthreads();
    FZ_TS(2);

    // ---- hidden layers 1..LM on MFMA ------------------------------------------------------
#pragma unroll
    for (int ly = 1; ly <= LM; ++ly) {
      const float* bi = aux + A_BH + (ly - 1) * W;
      f32x4 z[S], h[S];
      fz3_load_w<WT>(wf, Wimg, ly, o, l);
      fz3_gemm<WT, S>(z, wf, slot(ly - 1), L);
      FZ_TS(1 + 2 * ly);
      z[0] += *reinterpret_cast<const f32x4*>(bi + 16 * o + 4 * g);
      tanh_jet_f<S, NSO>(sp, z, h);
      // h_l into slot l; h_LM waits in h_0's slot for the loss and the top adjoint
      __bf16* im = slot(ly < LM ? ly : 0);
      fz3_put_h<WT, S>(im, L, o, h, fz3_vimg(im, WT, S) + voff);
      if (ly == LM) {  // output-layer partial dots of this wave's features -> LDS
#pragma unroll
        for (int s = 0; s < S; ++s) {
          float a = 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) a = fmaf(h[s][c], Ko[(16 * o + 4 * g + c) * 4], a);
          const float r = col4_sum(a);
          if (g == 0) outp[(w * S + s) * PT + p] = r;
        }
      }
      __syncthreads();
      FZ_TS(2 + 2 * ly);
    }

    // ---- J of the tile's points: the wave-ordered sums of the partial dots (here, over 64
    // threads: eight partials per J read inside the 16-thread loss measured 1 % slower,
    // profiles/r6ag_jsum_ab.txt) -------------------------------------------------------------
    int tl = tid;
    asm volatile("" : "+v"(tl));
    if (tl < S * PT) {
      const int s = tl / PT, pt = tl - s * PT;
      float a = outp[s * PT + pt];
#pragma unroll
      for (int ww = 1; ww < FZ_WAVES; ++ww) a += outp[(ww * S + s) * PT + pt];
      outp[s * PT + pt] = s == 0 ? a + aux[A_BO] : a;
    }
    __syncthreads();
    // ---- the per-point loss (generated) and its reverse sweep -> dJ into ubs ---------------
    tl = tid;
    asm volatile("" : "+v"(tl));
    if (tl < PT) LossF::template eval<S, PT, 1>(outp, xs, tl, pb + tl, N, *P.lptrs, ubs, lacc, lpre[tl], 0.f);
    __syncthreads();
    FZ_TS(9);
    tl = tid;
    asm volatile("" : "+v"(tl));
    if (tl < PT) bo_acc += ubs[tl * 4];  // dbo: this point's value-stream dJ
    // ---- reverse through the output layer: hb = Ko ub, dKo, the top tanh layer's adjoint ----
    {
      __bf16* im = slot(0);
      f32x4 h[S], hb[S], zb[S];
      fz3_get_h<WT, S>(im, L, o, h, fz3_vimg(im, WT, S) + voff);
      f32x4 kq, pp = zero4();
#pragma unroll
      for (int c = 0; c < 4; ++c) kq[c] = Ko[(16 * o + 4 * g + c) * 4];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const float ub = ubs[(s * PT + p) * 4];
        hb[s] = kq * ub;
        pp += h[s] * ub;
      }
      {
        const float r = row16_sum4(pp);
        if ((p & 3) == 0) accKo[(16 * o + 4 * g + (p >> 2)) * 4] += r;
      }
      tanh_jet_b<S, NSO>(sp, h, hb, zb);
      const float r = row16_sum4(zb[0]);
      if ((p & 3) == 0) accB[LM * W + 16 * o + 4 * g + (p >> 2)] += r;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        bf16x4 hi, lo;
        split4(zb[s], hi, lo);
        fz_put<RS>(im + s * SIMG, L, 0, o, hi);
        fz_put<RS>(im + (SP + s) * SIMG, L, 0, o, lo);
      }
    }
    __syncthreads();
    // ---- hidden layers LM..1: dK_l, hb_{l-1} = K_l zb_l, adjoint of tanh layer l-1 --------
#pragma unroll
    for (int ly = LM; ly >= 1; --ly) {
      const __bf16* Z = slot(ly == LM ? 0 : ly);
      __bf16* H = slot(ly - 1);
      const int tb = 10 + 5 * (LM - ly);
      f32x4 acc[S];
      fz3_load_w<WT>(wf, Kimg, ly, o, l);
      fz3_gemm<WT, S>(acc, wf, Z, L);
      FZ_TS(tb);
      bf16x4 zbh[S], zbl[S];
      float rb = 0.f;
      if (ly >= 2) {
        f32x4 h[S], zb[S];
        fz3_get_h<WT, S>(H, L, o, h, fz3_vimg(H, WT, S) + voff);
        tanh_jet_b<S, NSO>(sp, h, acc, zb);
        rb = row16_sum4(zb[0]);
#pragma unroll
        for (int s = 0; s < S; ++s) split4(zb[s], zbh[s], zbl[s]);
      }
      fz3_dk<WT, S, NR, NC>(dk[ly - 1], H, Z, r0, c0, l);
      FZ_TS(tb + 1);
      if (ly >= 2) {
        __syncthreads();  // every wave's dK reads of H are done
        FZ_TS(tb + 2);
        if ((p & 3) == 0) accB[(ly - 1) * W + 16 * o + 4 * g + (p >> 2)] += rb;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          fz_put<RS>(H + s * SIMG, L, 0, o, zbh[s]);
          fz_put<RS>(H + (SP + s) * SIMG, L, 0, o, zbl[s]);
        }
      } else {
        // layer 0: zb_0 from h_0 as the ly = 2 step rebuilt it into slot 0 (value stream fp32,
        // the others hi + lo) -> first-layer partials (K0, b0); not a third layer-0 evaluation
        f32x4 h[S], zb[S];
        fz3_get_h<WT, S>(H, L, o, h, fz3_vimg(H, WT, S) + voff);
        tanh_jet_b<S, NSO>(sp, h, acc, zb);
        const int fo = 16 * o + 4 * g + (p >> 2);
        {
          const float r = row16_sum4(zb[0]);
          if ((p & 3) == 0) accB[fo] += r;
        }
#pragma unroll
        for (int j = 0; j < DIN; ++j) {
          const float xj = xs[p * TDQ_MAXD + j];
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
      FZ_TS(tb + 3);
      if (ly == 2) {  // rebuild h_0 into slot 0 (zb_LM there is consumed)
        if (LM == 2) __syncthreads();  // (LM = 2: it was this step's Z)
        f32x4 h[S];
        layer0(h);
        fz3_put_h<WT, S>(slot(0), L, o, h, fz3_vimg(slot(0), WT, S) + voff);
      }
      if (ly >= 2) __syncthreads();
      FZ_TS(tb + 4);
    }
    ++t;
  }
  TDQ_TS(62);

  // ---- this workgroup's gradient-slab row (fp32) ---------------------------------------------
  float* gs = P.slab + (size_t)(P.srow + gi) * Pst;
#pragma unroll
  for (int ly = 1; ly <= LM; ++ly) {
    float* row = gs + off_layer(d, ly) + (16 * r0 + 4 * g) * W + 16 * c0 + p;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) row[(16 * r + e) * W + 16 * c] = dk[ly - 1][r][c][e];
  }
  __syncthreads();  // LDS partials complete
  for (int f = tid; f < W; f += 64 * FZ_WAVES) {
    gs[d.d_in * W + f] = part[f];  // b0
    for (int ly = 1; ly <= LM; ++ly) gs[off_layer(d, ly) + W * W + f] = part[ly * W + f];
    for (int j = 0; j < d.d_in; ++j) gs[j * W + f] = part[(LM + 1) * W + j * W + f];
    gs[off_layer(d, LM + 1) + f] = part[(LM + 1 + d.d_in) * W + f * 4];
  }
  // the output bias and the loss partials: the point-threads (wave 0, lanes < PT) summed
  if (w == 0) {
    const float bo = col4_sum(row16_sum(bo_acc));
    if (l == 0) gs[off_layer(d, LM + 1) + W] = bo;
#pragma unroll
    for (int k = 0; k < LossF::NACC; ++k) {
      const float v = col4_sum(row16_sum(lacc[k]));
      if (l == 0 && k < P.nacc) P.lpart[(size_t)(P.prow + gi) * P.nacc + k] = v;
    }
  }
  TDQ_TS(63);
}
