// Definitions shared by the fp32 (jet_mlp.hip) and split-bf16 (jet_bf3.hip) jet kernels.
#pragma once
#include "common.h"

#define TDQ_MAXS 8
#define TDQ_MAXD 8
#define TDQ_MAXO 4

// Stream plan.  Second-order streams pick their two first-order factors with one-hot FLOAT
// weights (selA/selB) instead of an integer index: an index-driven select over a register
// array is turned back into a scratch-memory lookup by LLVM, an FMA chain is not.
struct JetSpec {
  int stype[TDQ_MAXS];             // 0 value, 1 first order, 2 second order
  int var[TDQ_MAXS];               // type 1: input variable index
  float selA[TDQ_MAXS][TDQ_MAXS];  // type 2: one-hot over streams of first-order factor a
  float selB[TDQ_MAXS][TDQ_MAXS];  // type 2: one-hot over streams of first-order factor b
  int ia[TDQ_MAXS], ib[TDQ_MAXS];  // type 2: the same factors as stream indices (memory addressing only)
};

#define TDQ_MAXL 16  // hidden layers

// Network geometry.  Hidden layers may have different widths (the reference's neural_net takes
// any layer list, tensordiffeq/networks.py:10-20): the kernels pad every hidden layer to the
// widest one's W = 16 WT features (zero weights and biases -> the padded units are exactly 0 in
// every jet stream and never reach a gradient slab); `lw` / `lo` map the flat Keras-order buffer.
struct NetDims {
  int d_in, width, d_out, n_hidden;  // width: the WIDEST hidden layer
  int lw[TDQ_MAXL];                  // hidden layer widths
  int lo[TDQ_MAXL + 1];              // flat offset of dense layer i (0: input -> hidden 0; n_hidden: output)
  int uniform;                       // every hidden layer is `width` wide
};

// start of dense layer i (>= 1) in the flat Keras-order buffer
__host__ __device__ __forceinline__ int off_layer(const NetDims& d, int i) { return d.lo[i]; }
// width of hidden layer i (its kernel is [lw[i-1]][lw[i]] for i >= 1)
__host__ __device__ __forceinline__ int hw(const NetDims& d, int i) { return d.lw[i]; }

// widths: n_hidden hidden widths (nullptr: all `width`); false on an unsupported geometry
static inline bool make_dims(NetDims& d, int d_in, const int* widths, int width, int d_out, int n_hidden) {
  if (n_hidden < 1 || n_hidden > TDQ_MAXL || d_in < 1 || d_out < 1) return false;
  d.d_in = d_in;
  d.d_out = d_out;
  d.n_hidden = n_hidden;
  int mx = 0, off = 0, prev = d_in;
  for (int i = 0; i < TDQ_MAXL; ++i) d.lw[i] = 0;
  for (int i = 0; i < n_hidden; ++i) {
    const int w = widths ? widths[i] : width;
    if (w < 1) return false;
    d.lw[i] = w;
    d.lo[i] = off;
    off += prev * w + w;
    prev = w;
    mx = w > mx ? w : mx;
  }
  d.lo[n_hidden] = off;
  for (int i = n_hidden + 1; i <= TDQ_MAXL; ++i) d.lo[i] = off;
  d.width = mx;
  d.uniform = 1;
  for (int i = 0; i < n_hidden; ++i) d.uniform &= d.lw[i] == mx;
  return true;
}

static inline int param_count(const NetDims& d) { return d.lo[d.n_hidden] + d.lw[d.n_hidden - 1] * d.d_out + d.d_out; }

__device__ __forceinline__ size_t zs_index(int layer, int nwg, int wg, int S, int s, int w, int WT,
                                           int t, int lane) {
  // (wave-uniform tile base) + (32-bit lane offset): lets hipcc use SGPR-base addressing
  return ((((((size_t)layer * nwg + wg) * S + s) * 4 + w) * WT + t) * 256) + (unsigned)(lane * 4);
}

// ---- host helpers ----
static inline int width_tiles(int width) {
  int wt = (width + 15) / 16;
  if (wt <= 1) return 1;
  if (wt <= 2) return 2;
  if (wt <= 4) return 4;
  if (wt <= 8) return 8;
  if (wt <= 16) return 16;  // split-bf16 kernels only (bf3_ok)
  return -1;
}

static inline int param_count(int d_in, int width, int d_out, int n_hidden) {
  return d_in * width + width + (n_hidden - 1) * (width * width + width) + width * d_out + d_out;
}

// NetDims of an equal-width network (the exact-fp32 family, jet_mlp.hip)
static inline NetDims uniform_dims(int d_in, int width, int d_out, int n_hidden) {
  NetDims d;
  make_dims(d, d_in, nullptr, width, d_out, n_hidden);
  return d;
}

// spec: 3 ints per stream (type, a, b): type 1 -> a = input variable; type 2 -> a, b = stream
// indices of the two first-order factors.
static inline bool make_spec(int S, const int* spec, JetSpec& sp) {
  if (S < 1 || S > TDQ_MAXS) return false;
  for (int s = 0; s < TDQ_MAXS; ++s) {
    const int ty = s < S ? spec[3 * s] : 0, a = s < S ? spec[3 * s + 1] : 0, b = s < S ? spec[3 * s + 2] : 0;
    sp.stype[s] = ty;
    sp.var[s] = ty == 1 ? a : 0;
    sp.ia[s] = ty == 2 ? a : 0;
    sp.ib[s] = ty == 2 ? b : 0;
    for (int q = 0; q < TDQ_MAXS; ++q) {
      sp.selA[s][q] = (ty == 2 && q == a) ? 1.f : 0.f;
      sp.selB[s][q] = (ty == 2 && q == b) ? 1.f : 0.f;
    }
    if (ty == 2 && (a <= 0 || a >= S || b <= 0 || b >= S || spec[3 * a] != 1 || spec[3 * b] != 1)) return false;
    if (ty == 1 && a < 0) return false;
  }
  return true;
}

// number of second-order streams when the plan is in canonical order (value, first-order
// streams, second-order streams - JetPlan always emits this order); -1 otherwise
static inline int spec_nso(int S, const int* spec) {
  int nso = 0, prev = 0;
  for (int s = 0; s < S; ++s) {
    const int ty = spec[3 * s];
    if (ty < prev || (s == 0) != (ty == 0)) return -1;
    prev = ty;
    nso += ty == 2;
  }
  if (nso > 0 && S - 1 - nso < 1) return -1;
  return nso;
}

// per-workgroup gradient slab row stride: parameter count rounded up to 8 entries, so every slab
// row is 16-byte aligned for the float4 reduction of fp32 slabs and for the 16-byte (8 x bf16)
// loads of the bf16 slab reduction (slab_reduce1_body8)
static inline int slab_stride(int P) { return (P + 7) & ~7; }

// workgroup-chunk count of the first reduction pass (-DTDQ_SLAB_CHUNKS for A/B runs): 8 up to 2047
// rows (the 50k-point steps: tuned, their summation order and range cuts depend on it); beyond, one
// chunk per 256 rows up to 256 chunks - with 8 chunks a 2M-point step summed ~2000 rows per thread
// (0.42 of 3.7 ms per Poisson step, profiles/r4pois_*)
#ifndef TDQ_SLAB_CHUNKS
#define TDQ_SLAB_CHUNKS 8
#endif
static inline int slab_chunks(int nwg) {
  if (nwg < 2048) return nwg < TDQ_SLAB_CHUNKS ? nwg : TDQ_SLAB_CHUNKS;
  const int c = nwg / 256;
  return c < TDQ_SLAB_CHUNKS ? TDQ_SLAB_CHUNKS : (c > 256 ? 256 : c);
}
// chunk c of the first pass covers slab rows [floor(nwg c / chunks), floor(nwg (c + 1) / chunks)); a
// point-range cut placed on one of these row boundaries splits the reduction into chunks of the first
// range (pre-reduced while the second range's backward runs) and of the second (fit.point_ranges,
// tdq_slab_prereduce_bf3) without changing any summation order
__host__ __device__ inline int slab_chunk_lo(int nwg, int chunks, int c) {
  return (int)(((long long)nwg * c) / chunks);
}

// four consecutive slab entries (float4 column q of row `row`) as fp32; H: the slab holds bf16
template <bool H>
__device__ __forceinline__ f32x4 slab_ld4(const void* __restrict__ slab, size_t row, int Pst, int q) {
  if constexpr (H) {
    const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const unsigned short*>(slab) + row * Pst + 4 * q);
    return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                 __uint_as_float(u.y & 0xffff0000u)};
  } else {
    return reinterpret_cast<const f32x4*>(slab)[row * (size_t)(Pst >> 2) + q];
  }
}

// first reduction pass, float4 column q of chunk c: part[c][q] = sum of slab rows of the chunk
// (fp32 partials; H: bf16 slab rows)
template <bool H = false>
__device__ __forceinline__ void slab_reduce1_body(const void* __restrict__ slab, float* __restrict__ part, int nwg,
                                                  int Pst, int chunks, int q, int c) {
  const int lo = slab_chunk_lo(nwg, chunks, c), hi = slab_chunk_lo(nwg, chunks, c + 1);
  const size_t row = (size_t)(Pst >> 2);
  f32x4 a0 = zero4(), a1 = zero4(), a2 = zero4(), a3 = zero4();
  int wgi = lo;
  for (; wgi + 3 < hi; wgi += 4) {
    a0 += slab_ld4<H>(slab, wgi, Pst, q);
    a1 += slab_ld4<H>(slab, wgi + 1, Pst, q);
    a2 += slab_ld4<H>(slab, wgi + 2, Pst, q);
    a3 += slab_ld4<H>(slab, wgi + 3, Pst, q);
  }
  for (; wgi < hi; ++wgi) a0 += slab_ld4<H>(slab, wgi, Pst, q);
  reinterpret_cast<f32x4*>(part)[(size_t)c * row + q] = (a0 + a1) + (a2 + a3);
}

// the same first pass over bf16 slab rows with 16-byte loads: 8 columns (float4 columns 2 q8 and
// 2 q8 + 1) per thread, 8 rows in flight.  Every column is summed in slab_reduce1_body's order
// (rows round-robin into four accumulators, the remainder into the first, then (a0 + a1) + (a2 + a3)),
// so the partials are bit-identical; 8-byte loads ran at 0.54-0.70x the 16-byte rate (guide).
__device__ __forceinline__ void bf8_add(f32x4& lo, f32x4& hi, const uint4 u) {
  lo += f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
              __uint_as_float(u.y & 0xffff0000u)};
  hi += f32x4{__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u), __uint_as_float(u.w << 16),
              __uint_as_float(u.w & 0xffff0000u)};
}
__device__ __forceinline__ void slab_reduce1_body8(const void* __restrict__ slab, float* __restrict__ part, int nwg,
                                                   int Pst, int chunks, int q8, int c) {
  const int lo = slab_chunk_lo(nwg, chunks, c), hi = slab_chunk_lo(nwg, chunks, c + 1);
  const uint4* s8 = reinterpret_cast<const uint4*>(slab) + q8;  // row stride Pst / 8 uint4
  const size_t rs = (size_t)(Pst >> 3);
  f32x4 a0 = zero4(), a1 = zero4(), a2 = zero4(), a3 = zero4();
  f32x4 b0 = zero4(), b1 = zero4(), b2 = zero4(), b3 = zero4();
  int w = lo;
  for (; w + 7 < hi; w += 8) {
    uint4 u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = s8[(size_t)(w + k) * rs];
    bf8_add(a0, b0, u[0]);
    bf8_add(a1, b1, u[1]);
    bf8_add(a2, b2, u[2]);
    bf8_add(a3, b3, u[3]);
    bf8_add(a0, b0, u[4]);
    bf8_add(a1, b1, u[5]);
    bf8_add(a2, b2, u[6]);
    bf8_add(a3, b3, u[7]);
  }
  for (; w + 3 < hi; w += 4) {
    const uint4 u0 = s8[(size_t)w * rs], u1 = s8[(size_t)(w + 1) * rs], u2 = s8[(size_t)(w + 2) * rs],
                u3 = s8[(size_t)(w + 3) * rs];
    bf8_add(a0, b0, u0);
    bf8_add(a1, b1, u1);
    bf8_add(a2, b2, u2);
    bf8_add(a3, b3, u3);
  }
  for (; w < hi; ++w) bf8_add(a0, b0, s8[(size_t)w * rs]);
  f32x4* p4 = reinterpret_cast<f32x4*>(part) + (size_t)c * (size_t)(Pst >> 2) + 2 * q8;
  p4[0] = (a0 + a1) + (a2 + a3);
  p4[1] = (b0 + b1) + (b2 + b3);
}

// second pass: the gradient of float4 column q (fixed summation order: deterministic; chunk pairs
// alternate between two accumulators, eight partials loaded before they are added)
__device__ __forceinline__ f32x4 slab_reduce2_sum(const float* __restrict__ part, int Pst, int chunks, int q) {
  const f32x4* p4 = reinterpret_cast<const f32x4*>(part) + q;
  const size_t row = (size_t)(Pst >> 2);
  f32x4 a0 = zero4(), a1 = zero4();
  int c = 0;
  for (; c + 7 < chunks; c += 8) {
    f32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p4[(size_t)(c + k) * row];
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
      a0 += v[k];
      a1 += v[k + 1];
    }
  }
  for (; c + 1 < chunks; c += 2) {
    a0 += p4[(size_t)c * row];
    a1 += p4[(size_t)(c + 1) * row];
  }
  if (c < chunks) a0 += p4[(size_t)c * row];
  return a0 + a1;
}

// slabs [nwg][slab_stride(P)] at work, partials [chunks][slab_stride(P)] right after -> grad[P]
extern "C" int tdq_slab_reduce(float* work, float* grad, int nwg, int P, int chunks, void* stream);
// the same for bf16 slab rows when half != 0 (partials stay fp32, right after nwg fp32-sized rows)
extern "C" int tdq_slab_reduce_h(float* work, float* grad, int nwg, int P, int chunks, int half, void* stream);
