// Fused loss: interpret the traced per-point loss program (tensordiffeq_amd/fusion.py) for every
// collocation / boundary point in ONE launch, forward + reverse mode.
//
// One thread = one instance (a point of a segment group; a periodic group reads the upper and
// lower face point with the same index).  The program is straight-line SSA bytecode shared by
// the whole group, so decoding is wave-uniform (scalar loads, no divergence); each thread's
// value and adjoint registers live in LDS ([reg][thread], conflict-free).  Per instance:
//   forward   v[r] = op(v[a], v[b])                         (STREAM/COORD/VAL/LAM/SCAL loads)
//   losses    loss[term] += c * w * f^2 for every output (f, w, term, c)
//   seeds     adj[f] += 2 c w f ; adj[w] += c f^2
//   reverse   adjoints through every op; STREAM -> dJ[stream][point], LAM -> dlam[k][i],
//             SCAL -> block-reduced gradient of a scalar parameter
//   zeros     dJ of every (point, stream) the program does not read is written as 0, so dJ
//             needs no separate memset.
// Block partials (losses, scalar grads) are reduced by a second kernel in fixed order
// (bitwise deterministic), which also writes the total loss.
#include "common.h"

#define LF_BLOCK 128
#define LF_MAX_GROUPS 32
#define LF_MAX_SLOTS 2
#define LF_MAX_VAL 16
#define LF_MAX_LAM 8
#define LF_MAX_SCAL 8
#define LF_MAX_TERMS 32

enum {
  OP_STREAM = 1, OP_COORD = 2, OP_VAL = 3, OP_CONST = 4, OP_LAM = 5, OP_SCAL = 6,
  OP_ADD = 10, OP_SUB = 11, OP_MUL = 12, OP_DIV = 13, OP_NEG = 14, OP_POWI = 15, OP_POWF = 16,
  OP_SIN = 17, OP_COS = 18, OP_EXP = 19, OP_TANH = 20, OP_LOG = 21, OP_SQRT = 22, OP_SQUARE = 23
};

struct LFGroup {
  int code_off, n_code, const_off, n_regs;
  int n, block_off, out_off, n_out;
  int n_slots, seg_off[LF_MAX_SLOTS];
  unsigned loaded[LF_MAX_SLOTS];  // bit s set: stream s of that slot is read by the program
  // instances start `phase` threads into the group's first block: single-segment groups put their
  // block boundaries on absolute point indices that are multiples of LF_BLOCK, so point-range
  // launches of the jet kernels (multiples of 128) cut the loss blocks cleanly
  int phase;
};

struct LFOut {
  int f, w, term;
  float c;
};

// static per-program pointer table (device buffer, written once when the program is built;
// lambda / scalar / value / dlam buffers are persistent tensors, so it never changes)
struct LFPtrs {
  const float* val[LF_MAX_VAL];
  const float* lam[LF_MAX_LAM];
  float* dlam[LF_MAX_LAM];
  const float* scal[LF_MAX_SCAL];
};

struct LFMeta {
  int n_groups, n_terms, n_scal, S, d_in, N;
};

__device__ __forceinline__ float block_sum(float v, float* red) {
  // 128 threads = 2 waves: DPP row sums, then 8 row partials through LDS
  v = row16_sum(v);
  const int t = threadIdx.x;
  __syncthreads();
  if ((t & 15) == 0) red[t >> 4] = v;
  __syncthreads();
  float s = 0.f;
  if (t == 0) {
#pragma unroll
    for (int k = 0; k < LF_BLOCK / 16; ++k) s += red[k];
  }
  return s;  // valid in thread 0
}

__global__ void __launch_bounds__(LF_BLOCK) loss_fused_kernel(const int4* __restrict__ code,
                                                              const float* __restrict__ consts,
                                                              const LFOut* __restrict__ outs,
                                                              const LFGroup* __restrict__ groups, LFMeta meta,
                                                              const LFPtrs* __restrict__ ptrp, const float* __restrict__ J,
                                                              const float* __restrict__ X, float* __restrict__ dJ,
                                                              float* __restrict__ partials, int blk0) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ float red[LF_BLOCK / 16];
  __shared__ float acc[LF_MAX_TERMS + LF_MAX_SCAL];
  const int tid = threadIdx.x;
  const int blk = blk0 + (int)blockIdx.x;  // blk0: first block of a range launch
  int gi = 0;
  for (int q = 1; q < meta.n_groups; ++q)
    if (blk >= groups[q].block_off) gi = q;
  const LFGroup G = groups[gi];
  const LFPtrs& ptr = *ptrp;
  // slot lookups by select (a runtime-indexed member array would be placed in scratch)
  const int so0 = G.seg_off[0], so1 = G.seg_off[1];
  auto seg_off = [&](int slot) { return slot == 0 ? so0 : so1; };
  const int i = (blk - G.block_off) * LF_BLOCK + tid - G.phase;
  const bool active = i >= 0 && i < G.n;
  const int ii = active ? i : 0;
  float* V = lds;                               // [n_regs][LF_BLOCK]
  float* A = lds + G.n_regs * LF_BLOCK;         // [n_regs][LF_BLOCK]
  const int NP = meta.N;
  const int nslot_acc = meta.n_terms + meta.n_scal;
  if (tid < nslot_acc) acc[tid] = 0.f;

  // ---- forward ------------------------------------------------------------------------------
  for (int pc = 0; pc < G.n_code; ++pc) {
    const int4 in = code[G.code_off + pc];
    float v;
    switch (in.x) {
      case OP_STREAM: v = J[(size_t)in.w * NP + seg_off(in.z) + ii]; break;
      case OP_COORD: v = X[(size_t)(seg_off(in.z) + ii) * meta.d_in + in.w]; break;
      case OP_VAL: v = ptr.val[in.z][ii]; break;
      case OP_CONST: v = consts[G.const_off + in.z]; break;
      case OP_LAM: v = ptr.lam[in.z][ii]; break;
      case OP_SCAL: v = *ptr.scal[in.z]; break;
      case OP_ADD: v = V[in.z * LF_BLOCK + tid] + V[in.w * LF_BLOCK + tid]; break;
      case OP_SUB: v = V[in.z * LF_BLOCK + tid] - V[in.w * LF_BLOCK + tid]; break;
      case OP_MUL: v = V[in.z * LF_BLOCK + tid] * V[in.w * LF_BLOCK + tid]; break;
      case OP_DIV: v = V[in.z * LF_BLOCK + tid] / V[in.w * LF_BLOCK + tid]; break;
      case OP_NEG: v = -V[in.z * LF_BLOCK + tid]; break;
      case OP_POWI: {
        const float x = V[in.z * LF_BLOCK + tid];
        v = 1.f;
        for (int k = 0; k < in.w; ++k) v *= x;
        break;
      }
      case OP_POWF: v = powf(V[in.z * LF_BLOCK + tid], consts[G.const_off + in.w]); break;
      case OP_SIN: v = sinf(V[in.z * LF_BLOCK + tid]); break;
      case OP_COS: v = cosf(V[in.z * LF_BLOCK + tid]); break;
      case OP_EXP: v = expf(V[in.z * LF_BLOCK + tid]); break;
      case OP_TANH: v = tanhf(V[in.z * LF_BLOCK + tid]); break;
      case OP_LOG: v = logf(V[in.z * LF_BLOCK + tid]); break;
      case OP_SQRT: v = sqrtf(V[in.z * LF_BLOCK + tid]); break;
      case OP_SQUARE: { const float x = V[in.z * LF_BLOCK + tid]; v = x * x; break; }
      default: v = 0.f; break;
    }
    V[in.y * LF_BLOCK + tid] = v;
    A[in.y * LF_BLOCK + tid] = 0.f;
  }

  // ---- losses and seeds ----------------------------------------------------------------------
  for (int o = 0; o < G.n_out; ++o) {
    const LFOut out = outs[G.out_off + o];
    const float f = V[out.f * LF_BLOCK + tid], w = V[out.w * LF_BLOCK + tid];
    const float contrib = active ? out.c * w * f * f : 0.f;
    const float s = block_sum(contrib, red);
    if (tid == 0) acc[out.term] += s;
    if (active) {
      A[out.f * LF_BLOCK + tid] += 2.f * out.c * w * f;
      A[out.w * LF_BLOCK + tid] += out.c * f * f;
    }
  }

  // ---- reverse sweep -------------------------------------------------------------------------
  for (int pc = G.n_code - 1; pc >= 0; --pc) {
    const int4 in = code[G.code_off + pc];
    const float g = A[in.y * LF_BLOCK + tid];
    switch (in.x) {
      case OP_STREAM:
        if (active) dJ[(size_t)in.w * NP + seg_off(in.z) + i] = g;
        break;
      case OP_LAM:
        if (active) ptr.dlam[in.z][i] = g;
        break;
      case OP_SCAL: {
        const float s = block_sum(active ? g : 0.f, red);
        if (tid == 0) acc[meta.n_terms + in.z] += s;
        break;
      }
      case OP_ADD:
        A[in.z * LF_BLOCK + tid] += g;
        A[in.w * LF_BLOCK + tid] += g;
        break;
      case OP_SUB:
        A[in.z * LF_BLOCK + tid] += g;
        A[in.w * LF_BLOCK + tid] -= g;
        break;
      case OP_MUL: {
        const float a = V[in.z * LF_BLOCK + tid], b = V[in.w * LF_BLOCK + tid];
        A[in.z * LF_BLOCK + tid] += g * b;
        A[in.w * LF_BLOCK + tid] += g * a;
        break;
      }
      case OP_DIV: {
        const float a = V[in.z * LF_BLOCK + tid], b = V[in.w * LF_BLOCK + tid];
        A[in.z * LF_BLOCK + tid] += g / b;
        A[in.w * LF_BLOCK + tid] -= g * a / (b * b);
        break;
      }
      case OP_NEG: A[in.z * LF_BLOCK + tid] -= g; break;
      case OP_POWI: {
        const float x = V[in.z * LF_BLOCK + tid];
        float p = 1.f;
        for (int k = 0; k + 1 < in.w; ++k) p *= x;
        A[in.z * LF_BLOCK + tid] += g * (float)in.w * (in.w > 0 ? p : 0.f);
        break;
      }
      case OP_POWF: {
        const float x = V[in.z * LF_BLOCK + tid], e = consts[G.const_off + in.w];
        A[in.z * LF_BLOCK + tid] += g * e * powf(x, e - 1.f);
        break;
      }
      case OP_SIN: A[in.z * LF_BLOCK + tid] += g * cosf(V[in.z * LF_BLOCK + tid]); break;
      case OP_COS: A[in.z * LF_BLOCK + tid] -= g * sinf(V[in.z * LF_BLOCK + tid]); break;
      case OP_EXP: A[in.z * LF_BLOCK + tid] += g * V[in.y * LF_BLOCK + tid]; break;
      case OP_TANH: {
        const float t = V[in.y * LF_BLOCK + tid];
        A[in.z * LF_BLOCK + tid] += g * (1.f - t * t);
        break;
      }
      case OP_LOG: A[in.z * LF_BLOCK + tid] += g / V[in.z * LF_BLOCK + tid]; break;
      case OP_SQRT: A[in.z * LF_BLOCK + tid] += g * 0.5f / V[in.y * LF_BLOCK + tid]; break;
      case OP_SQUARE: A[in.z * LF_BLOCK + tid] += 2.f * g * V[in.z * LF_BLOCK + tid]; break;
      default: break;
    }
  }

  // ---- zero the dJ entries this program does not produce --------------------------------------
  if (active) {
    for (int sl = 0; sl < G.n_slots; ++sl) {
      const unsigned ld = sl == 0 ? G.loaded[0] : G.loaded[1];
      for (int s = 0; s < meta.S; ++s)
        if (!((ld >> s) & 1u)) dJ[(size_t)s * NP + seg_off(sl) + i] = 0.f;
    }
  }

  __syncthreads();
  if (tid < nslot_acc) partials[(size_t)blk * nslot_acc + tid] = acc[tid];
}

// losses[t] = sum_b partials[b][t] (fixed order); total = sum_t losses[t]; dscal[k] likewise
__global__ void __launch_bounds__(256) loss_reduce_kernel(const float* __restrict__ partials, int n_blocks,
                                                          int n_terms, int n_scal, float* __restrict__ losses,
                                                          float* __restrict__ total, float* __restrict__ dscal) {
  __shared__ float sh[256];
  const int slot = blockIdx.x;
  const int ns = n_terms + n_scal;
  float s = 0.f;
  for (int b = threadIdx.x; b < n_blocks; b += 256) s += partials[(size_t)b * ns + slot];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) sh[threadIdx.x] += sh[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (slot < n_terms) losses[slot] = sh[0];
    else dscal[slot - n_terms] = sh[0];
  }
}

__global__ void loss_total_kernel(const float* __restrict__ losses, int n_terms, float* __restrict__ total) {
  float s = 0.f;
  for (int t = 0; t < n_terms; ++t) s += losses[t];
  *total = s;
}

// partials -> per-term losses and scalar gradients (+ the total when with_total)
static int loss_reduce(const float* partials, int n_blocks, int n_terms, int n_scal, float* losses, float* total,
                    float* dscal, int with_total, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int ns = n_terms + n_scal;
  if (ns > 0) {
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(ns), dim3(256), 0, st, partials, n_blocks, n_terms, n_scal, losses,
                       total, dscal);
    TDQ_CHECK_LAUNCH();
  }
  if (with_total) {  // the Adam step's bookkeeping kernel (tdq_step_book) sums the terms itself
    hipLaunchKernelGGL(loss_total_kernel, dim3(1), dim3(1), 0, st, losses, n_terms, total);
    TDQ_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" {

// code: int4 per instruction; outs / groups / ptrs: device buffers of LFOut / LFGroup / LFPtrs
// do_reduce = 0: only the loss kernel (dJ, dlam, block partials); the fused step tail
// (tdq_step_tail_bf3 / tdq_dp_tail_a_bf3) reduces the partials itself
// blocks [blk0, blk0 + nblk) only (a range launch: dJ / dlam / partials of those blocks); the
// reduction is left to the fused step tail
int tdq_loss_fused_range(const int* code, const float* consts, const void* outs, const void* groups,
                         const void* ptrs, int n_groups, int n_terms, int n_scal, int S, int d_in, int N,
                         const float* J, const float* X, float* dJ, float* partials, int n_blocks, int blk0, int nblk,
                         int max_regs, void* stream) {
  LFMeta meta{n_groups, n_terms, n_scal, S, d_in, N};
  if (meta.n_groups < 1 || meta.n_groups > LF_MAX_GROUPS || meta.n_terms > LF_MAX_TERMS ||
      meta.n_scal > LF_MAX_SCAL || blk0 < 0 || nblk < 1 || blk0 + nblk > n_blocks)
    return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t lds = (size_t)2 * max_regs * LF_BLOCK * sizeof(float);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&loss_fused_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 120 * LF_BLOCK * (int)sizeof(float));
    attr = true;
  }
  hipLaunchKernelGGL(loss_fused_kernel, dim3(nblk), dim3(LF_BLOCK), lds, st,
                     reinterpret_cast<const int4*>(code), consts, reinterpret_cast<const LFOut*>(outs),
                     reinterpret_cast<const LFGroup*>(groups), meta, reinterpret_cast<const LFPtrs*>(ptrs), J, X,
                     dJ, partials, blk0);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// code: int4 per instruction; outs / groups / ptrs: device buffers of LFOut / LFGroup / LFPtrs
// do_reduce = 0: only the loss kernel (dJ, dlam, block partials); the fused step tail
// (tdq_step_tail_bf3 / tdq_dp_tail_a_bf3) reduces the partials itself
int tdq_loss_fused(const int* code, const float* consts, const void* outs, const void* groups,
                   const void* ptrs, int n_groups, int n_terms, int n_scal, int S, int d_in, int N,
                   const float* J, const float* X, float* dJ, float* partials, int n_blocks, int max_regs,
                   float* losses, float* total, float* dscal, int with_total, int do_reduce, void* stream) {
  int rc = tdq_loss_fused_range(code, consts, outs, groups, ptrs, n_groups, n_terms, n_scal, S, d_in, N, J, X, dJ,
                                partials, n_blocks, 0, n_blocks, max_regs, stream);
  if (rc || !do_reduce) return rc;
  return loss_reduce(partials, n_blocks, n_terms, n_scal, losses, total, dscal, with_total, stream);
}

// the per-term / scalar-gradient reduction alone (after a specialized loss kernel, ops/loss_jit.py)
int tdq_loss_reduce_partials(const float* partials, int n_blocks, int n_terms, int n_scal, float* losses,
                             float* total, float* dscal, int with_total, void* stream) {
  if (n_blocks < 1 || n_terms < 0 || n_terms > LF_MAX_TERMS || n_scal < 0 || n_scal > LF_MAX_SCAL)
    return (int)hipErrorInvalidValue;
  return loss_reduce(partials, n_blocks, n_terms, n_scal, losses, total, dscal, with_total, stream);
}

int tdq_loss_meta_sizes(int* out) {
  out[0] = (int)sizeof(LFMeta);
  out[1] = (int)sizeof(LFPtrs);
  out[2] = (int)sizeof(LFOut);
  out[3] = (int)sizeof(LFGroup);
  return 0;
}

}  // extern "C"
