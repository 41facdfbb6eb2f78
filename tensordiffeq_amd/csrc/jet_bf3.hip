// Host ABI + weight-image packing for the split-bf16 (bf16x3) jet kernels (kernels: jet_bf3.h,
// instantiations: jet_bf3_w{2,4,8}.hip).
#include "jet_bf3.h"

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
      const float v = (in < d.width && out < d.width) ? K[in * d.width + out] : 0.f;
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
    if (e < aux_b0(d, W)) {  // K0 [d_in][W]
      const int j = e / W, f = e - j * W;
      if (f < d.width) v = P[j * d.width + f];
    } else if (e < aux_bh(d, W)) {  // b0
      const int f = e - aux_b0(d, W);
      if (f < d.width) v = P[d.d_in * d.width + f];
    } else if (e < aux_ko(d, W)) {  // hidden biases
      const int r = e - aux_bh(d, W), i = r / W + 1, f = r - (i - 1) * W;
      if (f < d.width) v = P[off_layer(d, i) + d.width * d.width + f];
    } else if (e < aux_bo(d, W)) {  // Ko [W][4]
      const int r = e - aux_ko(d, W), f = r >> 2, q = r & 3;
      if (f < d.width && q < d.d_out) v = P[off_layer(d, d.n_hidden) + f * d.d_out + q];
    } else {  // bo [4]
      const int q = e - aux_bo(d, W);
      if (q < d.d_out) v = P[off_layer(d, d.n_hidden) + d.width * d.d_out + q];
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

namespace {

int64_t img_floats(int WT, int n_hidden) {  // hi/lo A images, in floats
  return (int64_t)(n_hidden > 1 ? n_hidden - 1 : 0) * WT * (WT / 2) * 128 * 4;
}

int64_t aux_alloc(int d_in, int n_hidden, int W) { return ((int64_t)(d_in + n_hidden + 4) * W + 4 + 3) / 4 * 4; }

int launch_pack(const float* P, bf16x8* fimg, bf16x8* bimg, float* aux, NetDims d, int WT, hipStream_t st) {
  const int total = 2 * (d.n_hidden - 1) * WT * (WT / 2) * 64 + aux_floats(d, 16 * WT);
  int blocks = (total + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(pack_all_kernel, dim3(blocks), dim3(256), 0, st, P, fimg, bimg, aux, d, WT);
  TDQ_CHECK_LAUNCH();
  return 0;
}

bool bf3_ok(int WT, int S, int d_in, int d_out, int n_hidden) {
  return (WT == 2 || WT == 4 || WT == 8) && S * WT <= 32 && d_in <= TDQ_MAXD && d_out <= TDQ_MAXO && n_hidden >= 1;
}

int dispatch(bool fwd, int WT, int S, int nso, const Bf3Args& a) {
  switch (WT) {
    case 2: return fwd ? bf3_fwd_w2(S, nso, a) : bf3_bwd_w2(S, nso, a);
    case 4: return fwd ? bf3_fwd_w4(S, nso, a) : bf3_bwd_w4(S, nso, a);
    case 8: return fwd ? bf3_fwd_w8(S, nso, a) : bf3_bwd_w8(S, nso, a);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

extern "C" {

// scratch = saved post-activations Hs | forward A image | backward A image | aux image (floats;
// -1: unsupported).  The forward packs all three images in one launch; the backward reuses them.
int64_t tdq_jet_bf3_scratch_floats(int N, int d_in, int width, int n_hidden, int S) {
  const int WT = width_tiles(width);
  if (WT < 2) return -1;
  const int64_t nwg = (N + 63) / 64;
  return (int64_t)n_hidden * nwg * S * 4 * WT * 256 + 2 * img_floats(WT, n_hidden) + aux_alloc(d_in, n_hidden, 16 * WT);
}

// per-workgroup gradient slabs + reduction partials, in floats
int64_t tdq_jet_bf3_slab_floats(int N, int d_in, int width, int d_out, int n_hidden) {
  const int WT = width_tiles(width);
  if (WT < 2) return -1;
  const int nwg = (N + 63) / 64;
  const int64_t P = slab_stride(param_count(d_in, width, d_out, n_hidden));
  return ((int64_t)nwg + slab_chunks(nwg)) * P;
}

// lo: 1 = "bf16x3" (activations split hi + lo), 0 = "bf16" (activations rounded to bf16)
int tdq_jet_fwd_bf3(const float* X, const float* P, float* J, float* scratch, int N, int d_in, int width,
                    int d_out, int n_hidden, int S, const int* spec, int lo, void* stream) {
  if (N <= 0) return 0;
  const int WT = width_tiles(width);
  JetSpec sp;
  const int nso = spec_nso(S, spec);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || nso < 0 || !make_spec(S, spec, sp)) return (int)hipErrorInvalidValue;
  NetDims d{d_in, width, d_out, n_hidden};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nwg = (N + 63) / 64;
  float* Hs = scratch;
  float* img = scratch + (int64_t)n_hidden * nwg * S * 4 * WT * 256;
  float* bimg = img + img_floats(WT, n_hidden);
  float* aux = bimg + img_floats(WT, n_hidden);
  int rc = launch_pack(P, reinterpret_cast<bf16x8*>(img), reinterpret_cast<bf16x8*>(bimg), aux, d, WT, st);
  if (rc) return rc;
  Bf3Args a{X, aux, reinterpret_cast<const bf16x8*>(img), nullptr, J, Hs, nullptr, N, 0, d, sp, st, lo};
  return dispatch(true, WT, S, nso, a);
}

int tdq_jet_bwd_bf3(const float* X, const float* P, const float* dJ, const float* Hs, float* work, float* grad,
                    int N, int d_in, int width, int d_out, int n_hidden, int S, const int* spec, int lo,
                    void* stream) {
  if (N <= 0) return 0;
  const int WT = width_tiles(width);
  JetSpec sp;
  const int nso = spec_nso(S, spec);
  if (!bf3_ok(WT, S, d_in, d_out, n_hidden) || nso < 0 || !make_spec(S, spec, sp)) return (int)hipErrorInvalidValue;
  NetDims d{d_in, width, d_out, n_hidden};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nwg = (N + 63) / 64;                               // forward (saved-activation) geometry
  const int pts_b = 16 * bwd_waves(WT, lo != 0), nwg_b = (N + pts_b - 1) / pts_b;  // slab rows
  const int Ptot = param_count(d_in, width, d_out, n_hidden);
  const int chunks = slab_chunks(nwg_b);
  float* slab = work;
  // images packed by the forward into its scratch, right after Hs (see tdq_jet_bf3_scratch_floats)
  const float* img = Hs + (int64_t)n_hidden * nwg * S * 4 * WT * 256 + img_floats(WT, n_hidden);
  const float* aux = img + img_floats(WT, n_hidden);
  (void)P;
  // slab rows use the 16-byte aligned stride that tdq_slab_reduce's float4 passes assume
  Bf3Args a{X, aux, reinterpret_cast<const bf16x8*>(img), dJ, nullptr, const_cast<float*>(Hs), slab, N,
            slab_stride(Ptot), d, sp, st, lo};
  int rc = dispatch(false, WT, S, nso, a);
  if (rc) return rc;
  return tdq_slab_reduce(work, grad, nwg_b, Ptot, chunks, stream);
}

}  // extern "C"
