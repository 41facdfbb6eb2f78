// Host ABI + weight-image packing for the split-bf16 (bf16x3) jet kernels (kernels: jet_bf3.h,
// instantiations: jet_bf3_w{2,4,8,16}.hip), and the fused step tail of a captured Adam step.
//
// Step tail (tdq_step_tail_bf3): the single-GPU Adam step used to end in seven small launches
// (weight-image pack, loss reduction, two slab-reduction passes, bookkeeping, Adam) of ~4.7 us
// each on MI355X, mostly launch/drain floor.  Two launches now do that work:
//   tail_reduce1: slab pass 1 (columns x chunks) + ONE extra workgroup that reduces the loss
//                 partials (per-term losses, scalar-lambda gradients) and runs the scalar
//                 bookkeeping (history row, best loss + "improved" flag, step counters, epoch) -
//                 nothing else in that launch reads those scalars, so no grid sync is needed;
//   tail_adam:    slab pass 2 fused element-wise into the Adam update of theta (the reduced
//                 gradient is also written out), the Adam ascent of the SA weights, the best-
//                 weights snapshot, and the next step's weight images: every updated weight is
//                 scattered straight into its forward / backward A-image (bf16 hi + lo) or aux
//                 slot, so the next forward runs without a pack launch.
#include "jet_fused3.h"
#include "optim_common.h"

// A-operand images: img[layer-1][o][kb][hl][lane] = 8 bf16 (hl 0 = hi, 1 = lo)
//   element j of lane (p, g): row 16o + p, k = 8g + j -> feature 32kb + (j<4 ? 4g+j : 16+4g+j-4)
//   transposed = 1 (forward):  A[row = out][k = in]  ;  0 (backward): A[row = in][k = out]
__device__ __forceinline__ void pack_frag(const float* __restrict__ P, bf16x8* __restrict__ img, const NetDims& d,
                                          int WT, int transposed, int e) {
  const int KB = WT / 2;
  {
    const int lane = e & 63, frag = e >> 6;
    const int kb = frag % KB, o = (frag / KB) % WT, layer = frag / (KB * WT) + 1;
    const int p = lane & 15, g = lane >> 4, row = 16 * o + p;
    const float* K = P + off_layer(d, layer);
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kf = 32 * kb + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4);
      const int in = transposed ? kf : row, out = transposed ? row : kf;
      const int win = hw(d, layer - 1), wout = hw(d, layer);
      const float v = (in < win && out < wout) ? K[in * wout + out] : 0.f;
      const __bf16 h = (__bf16)v;
      hi[j] = h;
      lo[j] = (__bf16)(v - (float)h);
    }
    img[(size_t)(frag * 2) * 64 + lane] = hi;
    img[(size_t)(frag * 2 + 1) * 64 + lane] = lo;
  }
}

// zero-padded fp32 aux image (layout: jet_bf3.h aux_*)
__device__ __forceinline__ void pack_aux(const float* __restrict__ P, float* __restrict__ aux, const NetDims& d,
                                         int W, int e) {
  {
    float v = 0.f;
    const int w0 = hw(d, 0), wl = hw(d, d.n_hidden - 1);
    if (e < aux_b0(d, W)) {  // K0 [d_in][W]
      const int j = e / W, f = e - j * W;
      if (f < w0) v = P[j * w0 + f];
    } else if (e < aux_bh(d, W)) {  // b0
      const int f = e - aux_b0(d, W);
      if (f < w0) v = P[d.d_in * w0 + f];
    } else if (e < aux_ko(d, W)) {  // hidden biases
      const int r = e - aux_bh(d, W), i = r / W + 1, f = r - (i - 1) * W;
      if (f < hw(d, i)) v = P[off_layer(d, i) + hw(d, i - 1) * hw(d, i) + f];
    } else if (e < aux_bo(d, W)) {  // Ko [W][4]
      const int r = e - aux_ko(d, W), f = r >> 2, q = r & 3;
      if (f < wl && q < d.d_out) v = P[off_layer(d, d.n_hidden) + f * d.d_out + q];
    } else {  // bo [4]
      const int q = e - aux_bo(d, W);
      if (q < d.d_out) v = P[off_layer(d, d.n_hidden) + wl * d.d_out + q];
    }
    aux[e] = v;
  }
}

// one launch per step: forward A image ([out][in]), backward A image ([in][out]) and aux image
__global__ void __launch_bounds__(256) pack_all_kernel(const float* __restrict__ P, bf16x8* __restrict__ fimg,
                                                       bf16x8* __restrict__ bimg, float* __restrict__ aux, NetDims d,
                                                       int WT) {
  const int nf = (d.n_hidden - 1) * WT * (WT / 2) * 64;
  const int total = 2 * nf + aux_floats(d, 16 * WT);
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    if (e < nf)
      pack_frag(P, fimg, d, WT, 1, e);
    else if (e < 2 * nf)
      pack_frag(P, bimg, d, WT, 0, e - nf);
    else
      pack_aux(P, aux, d, 16 * WT, e - 2 * nf);
  }
}

// ---- fused step tail ------------------------------------------------------------------------
struct TailBook {
  const float* lpart;  // loss-kernel block partials [n_lblocks][n_terms + n_scal]
  int n_lblocks, n_terms, n_scal;
  float* losses;
  float* total;
  float* dscal;
  float* hist;
  int64_t hist_rows;
  int64_t* epoch;
  float* best_loss;
  int64_t* best_epoch;
  int* improved;
  Counters cnt;
};

// chunks [c0, c0 + gridDim.y) of the first pass; blocks x >= nqb (at most one, and only with
// gridDim.x > nqb) run the loss reduction + bookkeeping
__global__ void __launch_bounds__(256) tail_reduce1_kernel(const float* __restrict__ slab, float* __restrict__ part,
                                                           int nwg, int Pst, int chunks, int nqb, int half, int c0,
                                                           TailBook tb) {
  if ((int)blockIdx.x < nqb) {
    const int q = blockIdx.x * 256 + threadIdx.x, c = c0 + (int)blockIdx.y;
    if (half) {  // bf16 slabs: 8 columns per thread, 16-byte loads (nqb counts 8-column groups)
      if (8 * q < Pst) slab_reduce1_body8(slab, part, nwg, Pst, chunks, q, c);
    } else if (4 * q < Pst) {
      slab_reduce1_body<false>(slab, part, nwg, Pst, chunks, q, c);
    }
    return;
  }
  if (blockIdx.y != 0) return;
  // loss partials -> per-term losses / scalar gradients (the loss_reduce_kernel order), then the
  // bookkeeping on the summed terms
  __shared__ float sh[256];
  const int ns = tb.n_terms + tb.n_scal;
  for (int slot = 0; slot < ns; ++slot) {
    float s = 0.f;
    for (int b = threadIdx.x; b < tb.n_lblocks; b += 256) s += tb.lpart[(size_t)b * ns + slot];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
      if ((int)threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (slot < tb.n_terms) tb.losses[slot] = sh[0];
      else tb.dscal[slot - tb.n_terms] = sh[0];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && tb.hist == nullptr && tb.total != nullptr) {  // loss + gradient only (L-BFGS)
    float s = 0.f;
    for (int t = 0; t < tb.n_terms; ++t) s += tb.losses[t];
    *tb.total = s;
  }
  if (threadIdx.x == 0 && tb.hist != nullptr)  // DP: the bookkeeping waits for the all-reduce
    step_book_body(tb.total, tb.losses, tb.n_terms, 1, tb.hist, tb.hist_rows, tb.epoch, tb.best_loss, tb.best_epoch,
                   tb.improved, tb.cnt);
}

// gx (optional): a second gradient added element-wise (the high-order points' part, jet_hi.hip)
__global__ void __launch_bounds__(256) slab_reduce2_bf3(const float* __restrict__ part, float* __restrict__ grad, int P,
                                                        int Pst, int chunks, const float* __restrict__ gx) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (4 * q >= P) return;
  const f32x4 a = slab_reduce2_sum(part, Pst, chunks, q);
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (4 * q + e < P) grad[4 * q + e] = gx != nullptr ? a[e] + gx[4 * q + e] : a[e];
}

// Adam over every group, one ELEMENT per thread (args.start in elements; float4 slots per thread
// measured ~2 us slower per step, profiles/r2_v10_ab_tail_elem.jsonl); group 0 = theta, whose
// gradient is the second slab pass of its column (the f32x4 pass's summation order, so the
// result is bit-identical) plus gx[e] when given (the high-order points' gradient, jet_hi.hip),
// written to args.grp[0].g as well
__global__ void __launch_bounds__(256) tail_adam_kernel(AdamArgs args, const float* __restrict__ part, int Pst,
                                                        int chunks, const int* __restrict__ improved,
                                                        float* __restrict__ snap, TailImg ti,
                                                        const float* __restrict__ gx) {
  const bool do_snap = snap != nullptr && *improved != 0;
  const int64_t total = args.start[args.ngroups];
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int gi = adam_group_of(args, idx);
    const AdamGroup gr = args.grp[gi];
    const int64_t e = idx - args.start[gi];
    const bool th = gi == 0;
    float g;
    if (th && part != nullptr) {
      float a0 = 0.f, a1 = 0.f;
      int c = 0;
      for (; c + 7 < chunks; c += 8) {  // (slab_reduce2_sum's order, eight loads in flight)
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = part[(size_t)(c + k) * Pst + e];
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          a0 += v[k];
          a1 += v[k + 1];
        }
      }
      for (; c + 1 < chunks; c += 2) {
        a0 += part[(size_t)c * Pst + e];
        a1 += part[(size_t)(c + 1) * Pst + e];
      }
      if (c < chunks) a0 += part[(size_t)c * Pst + e];
      g = a0 + a1;
      if (gx != nullptr) g += gx[e];
      const_cast<float*>(gr.g)[e] = g;
    } else {
      g = gr.g[e];
    }
    float p = gr.p[e], m = gr.m[e], v = gr.v[e];
    if (do_snap && th) snap[e] = p;
    adam_elem(p, gr.sign * g, m, v, gr.b1, gr.b2, gr.eps, adam_lr_t(gr));
    gr.p[e] = p;
    gr.m[e] = m;
    gr.v[e] = v;
    if (th && ti.fimg != nullptr) scatter_param(p, (int)e, ti);
  }
}

namespace {

int64_t img_floats(int WT, int n_hidden) {  // hi/lo A images, in floats
  return (int64_t)(n_hidden > 1 ? n_hidden - 1 : 0) * WT * (WT / 2) * 128 * 4;
}

int64_t aux_alloc(int d_in, int n_hidden, int W) { return ((int64_t)(d_in + n_hidden + 4) * W + 4 + 3) / 4 * 4; }

int64_t stage_floats(int N, int WT, int S, int lo) {  // the wide bf16x3 plans' global fragment stage
  const int64_t nwg = (N + 63) / 64;
  return bf3_gstage(WT, S, lo != 0) ? nwg * 4 * stage_wave_elems(WT, S, true) * 2 : 0;
}

// gradient-slab rows of a backward over N points
int bf3_rows(int N, const NetDims& d, int WT, int S, int lo) {
  const int pts_b = 16 * bwd_waves(WT, lo != 0, S);
  return (N + pts_b - 1) / pts_b;
}

int launch_pack(const float* P, bf16x8* fimg, bf16x8* bimg, float* aux, NetDims d, int WT, hipStream_t st) {
  const int total = 2 * (d.n_hidden - 1) * WT * (WT / 2) * 64 + aux_floats(d, 16 * WT);
  int blocks = (total + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(pack_all_kernel, dim3(blocks), dim3(256), 0, st, P, fimg, bimg, aux, d, WT);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// S <= 8 streams at every width class (S * WT <= 32: the 2-waves-per-SIMD kernels; beyond: the
// "wide" one-wave-per-SIMD kernels of jet_bf3.h)
bool bf3_ok(int WT, int S, int d_in, int d_out, int n_hidden) {
  // WT = 16 (widths 129..256, bf16 only): S <= 4 keeps the per-wave stream registers of the wide
  // WT = 8, S = 8 kernels
  return (WT == 2 || WT == 4 || WT == 8 || (WT == 16 && S <= 4)) && S >= 1 && S <= TDQ_MAXS &&
         d_in <= TDQ_MAXD && d_out <= TDQ_MAXO && n_hidden >= 1;
}

int dispatch(bool fwd, int WT, int S, int nso, const Bf3Args& a) {
  switch (WT) {
    case 2: return fwd ? bf3_fwd_w2(S, nso, a) : bf3_bwd_w2(S, nso, a);
    case 4: return fwd ? bf3_fwd_w4(S, nso, a) : bf3_bwd_w4(S, nso, a);
    case 8: return fwd ? bf3_fwd_w8(S, nso, a) : bf3_bwd_w8(S, nso, a);
    case 16: return fwd ? bf3_fwd_w16(S, nso, a) : bf3_bwd_w16(S, nso, a);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

extern "C" {

// scratch = forward A image | backward A image | aux image | (wide bf16x3 plans) the global
// fragment stage | saved post-activations Hs - floats; -1: unsupported.  The forward
// packs all three images in one launch; the backward reuses them.
int64_t tdq_jet_bf3_scratch_floats(int N, int d_in, const int* widths, int n_hidden, int S, int lo) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, 1, n_hidden)) return -1;
  const int WT = width_tiles(d.width);
  if (WT < 2) return -1;
  const int64_t nwg = (N + 63) / 64;
  const int64_t hs = (int64_t)n_hidden * nwg * S * 4 * WT * 256;
  return hs + 2 * img_floats(WT, n_hidden) + aux_alloc(d_in, n_hidden, 16 * WT) + stage_floats(N, WT, S, lo);
}

// per-workgroup gradient slabs + reduction partials, in floats (rows: the saved-activation
// backward's 64-point workgroups or the fused step's workgroups, whichever is more)
int64_t tdq_jet_bf3_slab_floats(int N, int d_in, const int* widths, int d_out, int n_hidden) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return -1;
  const int WT = width_tiles(d.width);
  if (WT < 2) return -1;
  int nwg = (N + 63) / 64;
  // the fused step's rows: at most one workgroup per CU, at most one per 16-point tile
  const int fz = (N + 15) / 16 < fz_cus() ? (N + 15) / 16 : fz_cus();
  if (fz > nwg) nwg = fz;
  const int64_t P = slab_stride(param_count(d));
  return ((int64_t)nwg + slab_chunks(nwg)) * P;
}

// floats of `rows` gradient-slab rows + their reduction partials (the fused step's rows)
int64_t tdq_slab_floats_rows(int rows, int d_in, const int* widths, int d_out, int n_hidden) {
  NetDims d;
  if (rows < 1 || !make_dims(d, d_in, widths, 0, d_out, n_hidden)) return -1;
  return ((int64_t)rows + slab_chunks(rows)) * slab_stride(param_count(d));
}

// image pointers inside the forward's scratch (at its start)
static inline void scratch_images(float* scratch, int n_hidden, int WT, float** img, float** bimg, float** aux) {
  *img = scratch;
  *bimg = *img + img_floats(WT, n_hidden);
  *aux = *bimg + img_floats(WT, n_hidden);
}

// the global fragment stage of a wide bf16x3 plan (after the aux image), else nullptr
static inline bf16x4* scratch_stage(float* scratch, int N, int d_in, int n_hidden, int S, int WT, int lo) {
  if (!bf3_gstage(WT, S, lo != 0)) return nullptr;
  float *img, *bimg, *aux;
  scratch_images(scratch, n_hidden, WT, &img, &bimg, &aux);
  return reinterpret_cast<bf16x4*>(aux + aux_alloc(d_in, n_hidden, 16 * WT));
}

// the saved post-activations (after the stage)
static inline float* scratch_hs(float* scratch, int N, int d_in, int n_hidden, int S, int WT, int lo) {
  return scratch + 2 * img_floats(WT, n_hidden) + aux_alloc(d_in, n_hidden, 16 * WT) + stage_floats(N, WT, S, lo);
}

// lo: 1 = "bf16x3" (activations split hi + lo), 0 = "bf16" (activations rounded to bf16).
// pack = 0: the weight images in scratch are already current (written by the previous step's
// tail_adam), so the forward skips its pack launch.
// forward over the point range [p_lo, p_hi) of the N-point set (p_lo a multiple of 128, p_hi one
// too or = N); pack = 1 packs the weight images first
int tdq_jet_fwd_bf3_range(const float* X, const float* P, float* J, float* scratch, int N, int p_lo, int p_hi,
                          int d_in, const int* widths, int d_out, int n_hidden, int S, const int* spec, int lo, int pack,
                          void* stream) {
  if (N <= 0) return 0;
  if (p_lo < 0 || p_lo % 128 != 0 || p_hi > N || p_hi <= p_lo || (p_hi != N && p_hi % 128 != 0))
    return (int)hipErrorInvalidValue;
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  JetSpec sp;
  // geometry first: spec holds 3 S ints, parse it only for a valid S (tools/asan/host_check.cpp)
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int nso = spec_nso(S, spec);
  if (nso < 0 || !make_spec(S, spec, sp)) return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* Hs = scratch_hs(scratch, N, d_in, n_hidden, S, WT, lo);
  float *img, *bimg, *aux;
  scratch_images(scratch, n_hidden, WT, &img, &bimg, &aux);
  if (pack) {
    int rc = launch_pack(P, reinterpret_cast<bf16x8*>(img), reinterpret_cast<bf16x8*>(bimg), aux, d, WT, st);
    if (rc) return rc;
  }
  Bf3Args a{X, aux, reinterpret_cast<const bf16x8*>(img), nullptr, J, Hs, nullptr, N, 0, d, sp, st, lo,
            scratch_stage(scratch, N, d_in, n_hidden, S, WT, lo), p_lo, p_hi};
  return dispatch(true, WT, S, nso, a);
}

int tdq_jet_fwd_bf3_ex(const float* X, const float* P, float* J, float* scratch, int N, int d_in, const int* widths,
                       int d_out, int n_hidden, int S, const int* spec, int lo, int pack, void* stream) {
  return tdq_jet_fwd_bf3_range(X, P, J, scratch, N, 0, N, d_in, widths, d_out, n_hidden, S, spec, lo, pack, stream);
}

int tdq_jet_fwd_bf3(const float* X, const float* P, float* J, float* scratch, int N, int d_in, const int* widths,
                    int d_out, int n_hidden, int S, const int* spec, int lo, void* stream) {
  return tdq_jet_fwd_bf3_ex(X, P, J, scratch, N, d_in, widths, d_out, n_hidden, S, spec, lo, 1, stream);
}

// the weight images of a forward scratch, packed from P (one launch)
int tdq_jet_bf3_pack(const float* P, float* scratch, int N, int d_in, const int* widths, int d_out, int n_hidden, int S,
                     void* stream) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  float *img, *bimg, *aux;
  scratch_images(scratch, n_hidden, WT, &img, &bimg, &aux);
  return launch_pack(P, reinterpret_cast<bf16x8*>(img), reinterpret_cast<bf16x8*>(bimg), aux, d, WT,
                     reinterpret_cast<hipStream_t>(stream));
}

// backward over the point range [p_lo, p_hi) (see tdq_jet_fwd_bf3_range): the slabs of the
// range's workgroups only; tdq_step_tail_bf3 / tdq_dp_tail_a_bf3 reduce all of them
int tdq_jet_bwd_bf3_range(const float* X, const float* dJ, const float* Hs, float* work, int N, int p_lo, int p_hi,
                          int d_in, const int* widths, int d_out, int n_hidden, int S, const int* spec, int lo,
                          void* stream) {
  if (N <= 0) return 0;
  if (p_lo < 0 || p_lo % 128 != 0 || p_hi > N || p_hi <= p_lo || (p_hi != N && p_hi % 128 != 0))
    return (int)hipErrorInvalidValue;
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  JetSpec sp;
  // geometry first: spec holds 3 S ints, parse it only for a valid S (tools/asan/host_check.cpp)
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int nso = spec_nso(S, spec);
  if (nso < 0 || !make_spec(S, spec, sp)) return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int Ptot = param_count(d);
  // images packed by the forward at the start of its scratch (see tdq_jet_bf3_scratch_floats)
  float* scr = const_cast<float*>(Hs);
  float *img, *bimg, *aux;
  scratch_images(scr, n_hidden, WT, &img, &bimg, &aux);
  // slab rows use the 16-byte aligned stride that tdq_slab_reduce's float4 passes assume
  Bf3Args a{X, aux, reinterpret_cast<const bf16x8*>(bimg), dJ, nullptr, scratch_hs(scr, N, d_in, n_hidden, S, WT, lo),
            work, N, slab_stride(Ptot), d, sp, st, lo, scratch_stage(scr, N, d_in, n_hidden, S, WT, lo), p_lo, p_hi};
  return dispatch(false, WT, S, nso, a);
}

// reduce = 0: only the backward kernel (gradient slabs in work); tdq_step_tail_bf3 reduces them
int tdq_jet_bwd_bf3_ex(const float* X, const float* P, const float* dJ, const float* Hs, float* work, float* grad,
                       int N, int d_in, const int* widths, int d_out, int n_hidden, int S, const int* spec, int lo, int reduce,
                       void* stream) {
  if (N <= 0) return 0;
  (void)P;
  int rc = tdq_jet_bwd_bf3_range(X, dJ, Hs, work, N, 0, N, d_in, widths, d_out, n_hidden, S, spec, lo, stream);
  if (rc || !reduce) return rc;
  NetDims d;
  make_dims(d, d_in, widths, 0, d_out, n_hidden);
  const int WT = width_tiles(d.width);
  const int nwg_b = bf3_rows(N, d, WT, S, lo);  // slab rows
  const int Ptot = param_count(d);
  return tdq_slab_reduce_h(work, grad, nwg_b, Ptot, slab_chunks(nwg_b), (int)slab_half(lo != 0), stream);
}

int tdq_jet_bwd_bf3(const float* X, const float* P, const float* dJ, const float* Hs, float* work, float* grad,
                    int N, int d_in, const int* widths, int d_out, int n_hidden, int S, const int* spec, int lo,
                    void* stream) {
  return tdq_jet_bwd_bf3_ex(X, P, dJ, Hs, work, grad, N, d_in, widths, d_out, n_hidden, S, spec, lo, 1, stream);
}

// The end of a single-process Adam step in two launches (see the file comment).  work: the
// backward's gradient slabs (tdq_jet_bwd_bf3_ex with reduce = 0); grad: receives the reduced theta
// gradient; scratch: the forward's scratch whose images are rewritten for the next step (nullptr:
// leave them).  groups[0] must be theta (n == parameter count); its g pointer is replaced by grad.
int tdq_step_tail_bf3(float* work, float* grad, float* scratch, int N, int d_in, const int* widths, int d_out, int n_hidden,
                      int S, int lo, const float* lpart, int n_lblocks, int n_terms, int n_scal, float* losses,
                      float* total, float* dscal, float* hist, int64_t hist_rows, int64_t* epoch, float* best_loss,
                      int64_t* best_epoch, int* improved, double* const* counters, int ncnt, const void* groups,
                      int ngroups, float* snap, int c_first, const float* gx, int rows, void* stream) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || ncnt < 0 || ncnt > TDQ_MAX_COUNTERS || n_lblocks < 0 ||
      n_terms < 0 || n_scal < 0)
    return (int)hipErrorInvalidValue;
  AdamArgs args;
  if (!adam_args_fill(args, reinterpret_cast<const AdamGroup*>(groups), ngroups, true))
    return (int)hipErrorInvalidValue;
  const int Ptot = param_count(d);
  if (args.grp[0].n != Ptot) return (int)hipErrorInvalidValue;
  args.grp[0].g = grad;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nwg_b = rows > 0 ? rows : bf3_rows(N, d, WT, S, lo);  // rows: the fused step's (ops/fused_step.py)
  const int Pst = slab_stride(Ptot), chunks = slab_chunks(nwg_b);
  if (c_first < 0 || c_first >= chunks) return (int)hipErrorInvalidValue;
  float* part = work + (size_t)nwg_b * Pst;
  TailBook tb;
  tb.lpart = lpart;
  tb.n_lblocks = n_lblocks;
  tb.n_terms = n_terms;
  tb.n_scal = n_scal;
  tb.losses = losses;
  tb.total = total;
  tb.dscal = dscal;
  tb.hist = hist;
  tb.hist_rows = hist_rows;
  tb.epoch = epoch;
  tb.best_loss = best_loss;
  tb.best_epoch = best_epoch;
  tb.improved = improved;
  tb.cnt.n = ncnt;
  for (int i = 0; i < TDQ_MAX_COUNTERS; ++i) tb.cnt.c[i] = i < ncnt ? counters[i] : nullptr;
  const int half = (int)slab_half(lo != 0);
  const int nqb = (Pst / (half ? 8 : 4) + 255) / 256;
  // chunks [0, c_first) were pre-reduced (tdq_slab_prereduce_bf3) while the other range ran
  hipLaunchKernelGGL(tail_reduce1_kernel, dim3(nqb + 1, chunks - c_first), dim3(256), 0, st, work, part, nwg_b, Pst,
                     chunks, nqb, half, c_first, tb);
  TDQ_CHECK_LAUNCH();
  TailImg ti{nullptr, nullptr, nullptr, d, WT};
  if (scratch != nullptr) {
    float *img, *bimg, *aux;
    scratch_images(scratch, n_hidden, WT, &img, &bimg, &aux);
    ti.fimg = reinterpret_cast<__bf16*>(img);
    ti.bimg = reinterpret_cast<__bf16*>(bimg);
    ti.aux = aux;
  }
  const int64_t tot = args.start[ngroups];
  int64_t blocks = (tot + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(tail_adam_kernel, dim3((unsigned)blocks), dim3(256), 0, st, args, part, Pst, chunks, improved,
                     snap, ti, gx);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// Data-parallel step, first half (before the all-reduce): slab pass 1 + the loss reduction in one
// launch (no bookkeeping: it needs the all-reduced terms), then slab pass 2 into grad (+ gx, the
// high-order points' gradient, when given).  total (optional): also the summed loss - the L-BFGS
// objective writes [grad | loss] in place this way.
int tdq_dp_tail_a_bf3(float* work, float* grad, int N, int d_in, const int* widths, int d_out, int n_hidden, int S, int lo,
                      const float* lpart, int n_lblocks, int n_terms, int n_scal, float* losses, float* dscal,
                      float* total, int c_first, const float* gx, int rows, int half_ovr, void* stream) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || N < 1 || n_lblocks < 0 || n_terms < 0 || n_scal < 0)
    return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int Ptot = param_count(d);
  const int nwg_b = rows > 0 ? rows : bf3_rows(N, d, WT, S, lo);
  const int Pst = slab_stride(Ptot), chunks = slab_chunks(nwg_b);
  if (c_first < 0 || c_first >= chunks) return (int)hipErrorInvalidValue;
  float* part = work + (size_t)nwg_b * Pst;
  TailBook tb{};
  tb.lpart = lpart;
  tb.n_lblocks = n_lblocks;
  tb.n_terms = n_terms;
  tb.n_scal = n_scal;
  tb.losses = losses;
  tb.dscal = dscal;
  tb.total = total;
  const int half = half_ovr >= 0 ? (half_ovr != 0) : (int)slab_half(lo != 0);
  const int nqb = (Pst / (half ? 8 : 4) + 255) / 256, nq2 = (Pst / 4 + 255) / 256;
  hipLaunchKernelGGL(tail_reduce1_kernel, dim3(nqb + 1, chunks - c_first), dim3(256), 0, st, work, part, nwg_b, Pst,
                     chunks, nqb, half, c_first, tb);
  TDQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(slab_reduce2_bf3, dim3(nq2), dim3(256), 0, st, part, grad, Ptot, Pst, chunks, gx);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// Geometry of the backward's gradient slabs: out = [points per backward workgroup, slab rows (nwg),
// first-pass chunks, 0].  fit.point_ranges places a range cut on a chunk boundary (slab_chunk_lo).
int tdq_bf3_slab_geometry(int N, int d_in, const int* widths, int d_out, int n_hidden, int S, int lo, int* out) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || N < 1) return (int)hipErrorInvalidValue;
  const int pts_b = 16 * bwd_waves(WT, lo != 0, S), nwg_b = bf3_rows(N, d, WT, S, lo),
            chunks = slab_chunks(nwg_b);
  out[0] = pts_b;
  out[1] = nwg_b;
  out[2] = chunks;
  out[3] = 0;
  return 0;
}

// First-pass chunks [c0, c1) of the slab reduction alone (no bookkeeping): launched on the first
// point range's stream right after its backward, so those rows are reduced while the second range's
// backward still runs; tdq_step_tail_bf3(c_first = c1) reduces the rest.  Same kernel and partial
// rows as the full pass: bit-identical.
int tdq_slab_prereduce_bf3(float* work, int N, int d_in, const int* widths, int d_out, int n_hidden, int S, int lo,
                           int c0, int c1, void* stream) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || N < 1) return (int)hipErrorInvalidValue;
  const int Ptot = param_count(d);
  const int nwg_b = bf3_rows(N, d, WT, S, lo);
  const int Pst = slab_stride(Ptot), chunks = slab_chunks(nwg_b);
  if (c0 < 0 || c1 > chunks || c1 <= c0) return (int)hipErrorInvalidValue;
  float* part = work + (size_t)nwg_b * Pst;
  const int half = (int)slab_half(lo != 0);
  const int nqb = (Pst / (half ? 8 : 4) + 255) / 256;
  TailBook tb{};
  hipLaunchKernelGGL(tail_reduce1_kernel, dim3(nqb, c1 - c0), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     work, part, nwg_b, Pst, chunks, nqb, half, c0, tb);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// Data-parallel step, second half (after the all-reduce and tdq_step_book): Adam over every group
// with theta's gradient read from groups[0].g (the all-reduced bucket), the best-weights snapshot
// and the next step's weight images written into the forward scratch.
int tdq_dp_tail_b_bf3(float* scratch, int N, int d_in, const int* widths, int d_out, int n_hidden, int S,
                      const void* groups, int ngroups, const int* improved, float* snap, void* stream) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  AdamArgs args;
  if (!adam_args_fill(args, reinterpret_cast<const AdamGroup*>(groups), ngroups, true))
    return (int)hipErrorInvalidValue;
  if (args.grp[0].n != param_count(d)) return (int)hipErrorInvalidValue;
  TailImg ti{nullptr, nullptr, nullptr, d, WT};
  if (scratch != nullptr) {
    float *img, *bimg, *aux;
    scratch_images(scratch, n_hidden, WT, &img, &bimg, &aux);
    ti.fimg = reinterpret_cast<__bf16*>(img);
    ti.bimg = reinterpret_cast<__bf16*>(bimg);
    ti.aux = aux;
  }
  const int64_t tot = args.start[ngroups];
  int64_t blocks = (tot + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(tail_adam_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     args, nullptr, 0, 0, improved, snap, ti, nullptr);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// One launch of a run-time compiled fused training step (ops/fused_step.py; lo = 0: the bf16 step of
// csrc/jet_fused.h, 32-point tiles; lo = 1: the bf16x3 objective of csrc/jet_fused3.h, 16-point
// tiles): forward -> loss -> backward over the points [p_lo, N), G workgroups, gradient-slab rows
// srow.., loss-partial rows prow.. (nacc floats each)
int tdq_fused_step_launch(void* func, const float* X, float* scratch, float* work, int N, int d_in, const int* widths,
                          int d_out, int n_hidden, int S, const int* spec, int p_lo, int srow, int G, const void* lptrs,
                          float* lpart, int prow, int nacc, int lo, void* stream) {
  if (func == nullptr || N <= 0 || p_lo < 0 || p_lo >= N || G < 1 || srow < 0 || prow < 0 || nacc < 1 || lo < 0 ||
      lo > 1)
    return (int)hipErrorInvalidValue;
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return (int)hipErrorInvalidValue;
  const int WT = width_tiles(d.width);
  // the kernels' geometry (also what the LDS size was computed for): width 128, 2-3 MFMA layers
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || tdq_jet_fused_lds(d_in, widths, d_out, n_hidden, S, lo) < 0)
    return (int)hipErrorInvalidValue;
  const int PT = lo ? FZ3_PT : FZ_PT;
  // at most one workgroup per tile: every workgroup owns at least one tile
  if (G > (N - p_lo + PT - 1) / PT) return (int)hipErrorInvalidValue;
  JetSpec sp;
  if (spec_nso(S, spec) < 0 || !make_spec(S, spec, sp)) return (int)hipErrorInvalidValue;
  float *img, *bimg, *aux;
  scratch_images(scratch, n_hidden, WT, &img, &bimg, &aux);
  FzParams P{};
  P.X = X;
  P.aux = aux;
  P.fimg = reinterpret_cast<const bf16x8*>(img);
  P.bimg = reinterpret_cast<const bf16x8*>(bimg);
  P.slab = work;
  P.N = N;
  P.Pst = slab_stride(param_count(d));
  P.ntiles = (N - p_lo + PT - 1) / PT;
  P.p_lo = p_lo;
  P.srow = srow;
  P.d = d;
  P.sp = sp;
  P.lptrs = reinterpret_cast<const FzLossPtrs*>(lptrs);
  P.lpart = lpart;
  P.prow = prow;
  P.nacc = nacc;
  void* args[] = {(void*)&P};
  return (int)hipModuleLaunchKernel((hipFunction_t)func, (unsigned)G, 1, 1, 64 * FZ_WAVES, 1, 1, 0,
                                    reinterpret_cast<hipStream_t>(stream), args, nullptr);
}

int tdq_fused_params_size() { return (int)sizeof(FzParams); }

// The weight-image target of a forward scratch (TailImg: forward / backward A images + aux image)
// for kernels that scatter updated parameters into it (lbfgs.hip lbfgs_dir_step_kernel); returns
// the struct's size, or -1 (unsupported network / buffer too small).
int tdq_img_target(float* scratch, int d_in, const int* widths, int d_out, int n_hidden, void* out, int out_bytes) {
  NetDims d;
  if (scratch == nullptr || out == nullptr || !make_dims(d, d_in, widths, 0, d_out, n_hidden)) return -1;
  const int WT = width_tiles(d.width);
  if (WT < 2 || out_bytes < (int)sizeof(TailImg)) return -1;
  float *img, *bimg, *aux;
  scratch_images(scratch, n_hidden, WT, &img, &bimg, &aux);
  TailImg ti{reinterpret_cast<__bf16*>(img), reinterpret_cast<__bf16*>(bimg), aux, d, WT};
  *reinterpret_cast<TailImg*>(out) = ti;
  return (int)sizeof(TailImg);
}

}  // extern "C"
