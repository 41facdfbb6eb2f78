// Small fixed-order kernels of the layer-wise engine (ops/jet_layered.py) that used to be torch
// ops between the hand-written GEMMs (`at::native::reduce_kernel` and the bf16
// copy kernels were ~7 % of the W512 bf16 step, profiles/r5lay10_kstats_bf16_w512.txt):
//
//   tdq_colsum      out[m] = sum_r src[r][m] (+ bias) - TN-GEMM chunk partials, J's 64-column
//                   partials, per-tile bias partials, column sums over all points; one pass when the
//                   row count is small, else row chunks -> partial rows -> a second pass.  Every
//                   element is summed in an order fixed by (R, M) alone: deterministic.
//   tdq_lay_bplanes the B operand of an NN GEMM (B^T [Nout, K]) from fp32 weights: transpose (the
//                   forward reads K^T) + bf16 hi (+ lo = x - hi) planes in one pass
//   tdq_lay_l0grad  the input layer's gradient from its summed partials: dK0 = X^T zb rows plus the
//                   first-order streams' sums, b0 = the value stream's sum
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "jet_common.h"

namespace {

constexpr int CS_THREADS = 256;

// one block: CB columns x RL row lanes (CB * RL = 256); rows [r0, r1) of columns [m0, m0 + CB);
// thread (rl, c) sums rows r0 + rl, r0 + rl + RL, ... (four accumulators round-robin), then the RL
// lane sums are added in lane order.  out_mode 0: work[blockIdx.y][m] (a partial row); 1: the final
// value to dst[(m / W) * sj + (m % W) * sf] (+ bias[m % bdim] for m < nbias)
__global__ void __launch_bounds__(CS_THREADS) colsum_kernel(const float* __restrict__ src, int64_t lds, int R,
                                                            int64_t M, int CB, int rows_per_chunk,
                                                            float* __restrict__ work, float* __restrict__ dst,
                                                            int64_t W, int64_t sj, int64_t sf,
                                                            const float* __restrict__ bias, int64_t nbias, int bdim,
                                                            int out_mode) {
  __shared__ float red[CS_THREADS];
  const int RL = CS_THREADS / CB;
  const int c = threadIdx.x % CB, rl = threadIdx.x / CB;
  const int64_t m = (int64_t)blockIdx.x * CB + c;
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = r0 + rows_per_chunk < R ? r0 + rows_per_chunk : R;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (m < M) {
    const float* p = src + m;
    int r = r0 + rl;
    for (; r + 3 * RL < r1; r += 4 * RL) {
      a0 += p[(int64_t)r * lds];
      a1 += p[(int64_t)(r + RL) * lds];
      a2 += p[(int64_t)(r + 2 * RL) * lds];
      a3 += p[(int64_t)(r + 3 * RL) * lds];
    }
    for (; r < r1; r += RL) a0 += p[(int64_t)r * lds];
  }
  red[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (rl != 0 || m >= M) return;
  float s = red[c];
  for (int k = 1; k < RL; ++k) s += red[k * CB + c];
  if (out_mode == 0) {
    work[(int64_t)blockIdx.y * M + m] = s;
  } else {
    if (m < nbias) s += bias[m % bdim];
    dst[(m / W) * sj + (m % W) * sf] = s;
  }
}

// dst[c][r] (transpose) or dst[r][c] of src [rows][cols] as bf16 hi and (optional) lo = x - hi
__global__ void __launch_bounds__(256) bplanes_kernel(const float* __restrict__ src, int rows, int cols, int transpose,
                                                      __bf16* __restrict__ h, __bf16* __restrict__ l) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    // i indexes the destination; its source element
    int64_t si;
    if (transpose) {
      const int64_t dr = i / rows, dc = i - dr * rows;  // dst [cols][rows]
      si = dc * cols + dr;
    } else {
      si = i;
    }
    const float x = src[si];
    const __bf16 hv = (__bf16)x;
    h[i] = hv;
    if (l != nullptr) l[i] = (__bf16)(x - (float)hv);
  }
}

// tot [S + d_in][W0] (stream sums, then X^T zb rows) -> dK0 [d_in][W0], b0 [W0]
struct L0Spec {
  int S, d_in, var[TDQ_MAXS], first[TDQ_MAXS];
};
__global__ void __launch_bounds__(256) l0grad_kernel(const float* __restrict__ tot, int W0, L0Spec sp,
                                                     float* __restrict__ dK0, float* __restrict__ b0) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= W0) return;
  for (int j = 0; j < sp.d_in; ++j) {
    float v = tot[(int64_t)(sp.S + j) * W0 + f];
    for (int s = 1; s < sp.S; ++s)
      if (sp.first[s] && sp.var[s] == j) v += tot[(int64_t)s * W0 + f];
    dK0[(int64_t)j * W0 + f] = v;
  }
  b0[f] = tot[f];
}

}  // namespace

extern "C" {

// Column sums of src [R][M] (row stride lds) into dst (element m at (m / W) * sj + (m % W) * sf),
// bias[m % bdim] added to the first nbias elements.  work: >= tdq_colsum_work(R, M) floats (may
// be null when that is 0).
int64_t tdq_colsum_work(int R, int64_t M);
int tdq_colsum(const float* src, int64_t lds, int R, int64_t M, float* dst, int64_t W, int64_t sj, int64_t sf,
               const float* bias, int64_t nbias, int bdim, float* work, void* stream);

}  // extern "C"

namespace {

struct ColsumPlan {
  int CB, RL, nrc, rows_per_chunk;
  int64_t gx;
};

ColsumPlan colsum_plan(int R, int64_t M) {
  ColsumPlan p;
  p.CB = 64;
  while (p.CB > 1 && p.CB / 2 >= M) p.CB /= 2;
  p.RL = CS_THREADS / p.CB;
  p.gx = (M + p.CB - 1) / p.CB;
  // row chunks: enough blocks to spread the read over the chip (~512), at least 4 rows per lane
  int64_t want = (512 + p.gx - 1) / p.gx;
  const int64_t maxc = ((int64_t)R + 4 * p.RL - 1) / (4 * p.RL);
  if (want > maxc) want = maxc;
  if (want < 1) want = 1;
  if (want > 4096) want = 4096;
  p.rows_per_chunk = (int)((R + want - 1) / want);
  p.nrc = (R + p.rows_per_chunk - 1) / p.rows_per_chunk;
  return p;
}

}  // namespace

extern "C" {

int64_t tdq_colsum_work(int R, int64_t M) {
  if (R < 1 || M < 1) return 0;
  const ColsumPlan p = colsum_plan(R, M);
  return p.nrc > 1 ? (int64_t)p.nrc * M : 0;
}

int tdq_colsum(const float* src, int64_t lds, int R, int64_t M, float* dst, int64_t W, int64_t sj, int64_t sf,
               const float* bias, int64_t nbias, int bdim, float* work, void* stream) {
  if (R < 1 || M < 1 || lds < M || W < 1 || dst == nullptr || src == nullptr) return (int)hipErrorInvalidValue;
  if (nbias > 0 && (bias == nullptr || bdim < 1)) return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const ColsumPlan p = colsum_plan(R, M);
  if (p.nrc > 1) {
    if (work == nullptr) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)p.gx, (unsigned)p.nrc), dim3(CS_THREADS), 0, st, src, lds, R, M,
                       p.CB, p.rows_per_chunk, work, dst, W, sj, sf, bias, nbias, bdim, 0);
    TDQ_CHECK_LAUNCH();
    // second pass: one chunk of all p.nrc partial rows per column block
    const ColsumPlan q = colsum_plan(p.nrc, M);
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)q.gx, 1), dim3(CS_THREADS), 0, st, work, M, p.nrc, M, q.CB, p.nrc,
                       nullptr, dst, W, sj, sf, bias, nbias, bdim, 1);
  } else {
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)p.gx, 1), dim3(CS_THREADS), 0, st, src, lds, R, M, p.CB, R,
                       nullptr, dst, W, sj, sf, bias, nbias, bdim, 1);
  }
  TDQ_CHECK_LAUNCH();
  return 0;
}

int tdq_lay_bplanes(const float* src, int rows, int cols, int transpose, void* h, void* l, void* stream) {
  if (src == nullptr || h == nullptr || rows < 1 || cols < 1) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)rows * cols;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(bplanes_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), src,
                     rows, cols, transpose, reinterpret_cast<__bf16*>(h), reinterpret_cast<__bf16*>(l));
  TDQ_CHECK_LAUNCH();
  return 0;
}

// spec: 3 S ints (type, a, b) per stream (type 1: first-order stream in variable a)
int tdq_lay_l0grad(const float* tot, int S, int d_in, const int* spec, int W0, float* dK0, float* b0, void* stream) {
  if (tot == nullptr || S < 1 || S > TDQ_MAXS || d_in < 1 || W0 < 1 || spec == nullptr) return (int)hipErrorInvalidValue;
  L0Spec sp;
  sp.S = S;
  sp.d_in = d_in;
  for (int s = 0; s < TDQ_MAXS; ++s) {
    sp.first[s] = s < S && s > 0 && spec[3 * s] == 1;
    sp.var[s] = s < S ? spec[3 * s + 1] : 0;
    if (sp.first[s] && (sp.var[s] < 0 || sp.var[s] >= d_in)) return (int)hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(l0grad_kernel, dim3((unsigned)((W0 + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), tot, W0, sp, dK0, b0);
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
