// Hand-written MFMA GEMMs of the layer-wise jet engine (ops/jet_layered.py), for hidden widths
// beyond the fused kernels' register envelope (> 256, or 129..256 in fp32 / bf16x3 / S > 4).
//
// Every weight multiplication of a layer is one of two shapes over the stacked streams
// [S*N, W] (stream-major planes, jet_layered.hip):
//   NN  C[M][N] = A[M][K] B           forward Z = H K, backward HB = ZB K^T
//       A row-major (the activations / adjoints), B given as B^T [N][K] (the weights, W x W)
//   TN  C[Ma][Nb] = sum_r A[r][:]^T B[r][:]   the weight gradient dK = H^T ZB, a long reduction
//       over r = S*N rows: split into row chunks (grid z), fixed-order chunk partials summed by the
//       caller (deterministic)
// Precisions (the fused kernels' families): P = 0 bf16 (operands rounded once, 1 MFMA), 1 bf16x3
// (hi + lo operands, lo*lo dropped, 3 MFMAs), 2 fp32 (v_mfma_f32_16x16x4_f32 on fp32 operands);
// fp32 accumulation throughout.
//
// gfx950 MFMA lane layouts (16 x 16 output tiles; lane l = 16 g + p):
//   bf16 16x16x32: A frag = A[p][8g .. 8g + 7], B frag = B[8g .. 8g + 7][p], D[4g + r][p]
//   fp32 16x16x4:  one element each; the k order is permuted so a lane's 8 fp32 k-values are
//                  contiguous too (MFMA kk of the block takes k = 8g + kk for lane group g)
// bf16 families (the throughput path): 128 x 128 workgroup tiles, 4 waves in 2 x 2 of 64 x 64, k-steps
// of 32 through LDS - NN double-buffered with 16-byte fragment reads, TN row-major staging read
// back with ds_read_b64_tr_b16.  fp32: 64 x 128 (NN, fragments straight from global memory) and
// 64 x 64 (TN, LDS-transposed) tiles on v_mfma_f32_16x16x4_f32.
// The layer jet (lay_jet.h) runs in the GEMM epilogues (lay_nnj_kernel) and in two elementwise end-layer
// kernels (lay_in_fwd_kernel: X K0 + jet; lay_out_bwd_kernel: dJ Ko^T + adjoint jet), so no fp32
// activation / adjoint plane of a hidden layer ever goes through HBM.  Measured on MI355X (AC
// [2, W x 4, 1], 50k points, one Adam step, profiles/r5lay4_*): bf16 width 512 2.59 ms and bf16x3
// width 256 1.79 ms per step, vs 4.75 / 5.69 ms on the library GEMMs (hipBLASLt) + standalone pass.
// Reference: tensordiffeq/networks.py:10-20 (any layer list), the reference's tape GEMMs.
#include "jet_bf3.h"
#include "lay_jet.h"

namespace {

template <int P>
struct Op;  // operand element type
template <>
struct Op<0> {
  using T = __bf16;
};
template <>
struct Op<1> {
  using T = __bf16;
};
template <>
struct Op<2> {
  using T = float;
};

// 8 consecutive k-values of row `row` (zero outside [0, nrows) x [0, K)); vec: 16 / 32-byte loads
template <class T>
__device__ __forceinline__ void ld8(const T* __restrict__ base, long long ld, int row, int nrows, int k, int K, bool vec,
                                    T (&v)[8]) {
  if (row < nrows) {
    const T* p = base + (long long)row * ld + k;
    if (vec && k + 8 <= K) {
      if constexpr (sizeof(T) == 2) {
        const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = x[j];
      } else {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = x0[j];
          v[4 + j] = x1[j];
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (k + j < K) ? p[j] : (T)0.f;
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (T)0.f;
}

__device__ __forceinline__ bf16x8 pack8(const __bf16 (&v)[8]) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = v[j];
  return r;
}

// acc += a * b for one 16 x 16 x 32 block (per precision)
template <int P, class T>
__device__ __forceinline__ f32x4 mma32(const T (&ah)[8], const T (&al)[8], const T (&bh)[8], const T (&bl)[8],
                                       f32x4 acc) {
  if constexpr (P == 2) {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ah[kk], bh[kk], acc, 0, 0, 0);
    return acc;
  } else {
    const bf16x8 a = pack8(ah), b = pack8(bh);
    if constexpr (P == 1) {
      acc = mfma_bf(pack8(al), b, acc);
      acc = mfma_bf(a, pack8(bl), acc);
    }
    return mfma_bf(a, b, acc);
  }
}

template <int P>
__global__ void __launch_bounds__(256) lay_nn_kernel(const typename Op<P>::T* __restrict__ Ah,
                                                     const typename Op<P>::T* __restrict__ Al, long long lda,
                                                     const typename Op<P>::T* __restrict__ Bh,
                                                     const typename Op<P>::T* __restrict__ Bl, long long ldb,
                                                     float* __restrict__ C, long long ldc, int M, int N, int K,
                                                     int vec) {
  using T = typename Op<P>::T;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, p = l & 15, g = l >> 4;
  const int rbase = blockIdx.y * 64 + 16 * w, n0 = blockIdx.x * 128;
  const int row = rbase + p;
  f32x4 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool v = vec != 0;
  for (int k0 = 0; k0 < K; k0 += 32) {
    const int k = k0 + 8 * g;
    T ah[8], al[8];
    ld8(Ah, lda, row, M, k, K, v, ah);
    if constexpr (P == 1) ld8(Al, lda, row, M, k, K, v, al);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int col = n0 + 16 * c + p;
      if (n0 + 16 * c >= N) break;  // (uniform)
      T bh[8], bl[8];
      ld8(Bh, ldb, col, N, k, K, v, bh);
      if constexpr (P == 1) ld8(Bl, ldb, col, N, k, K, v, bl);
      acc[c] = mma32<P>(ah, al, bh, bl, acc[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int col = n0 + 16 * c + p;
    if (col >= N) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ro = rbase + 4 * g + r;
      if (ro < M) C[(long long)ro * ldc + col] = acc[c][r];
    }
  }
}

// TN: C[z][i][j] = sum over rows r of chunk z of A[r][i] B[r][j]
constexpr int TN_PAD = 40;  // LDS row (32 k-values + 8): 16-byte aligned fragments, fewer conflicts
template <int P>
__global__ void __launch_bounds__(256) lay_tn_kernel(const typename Op<P>::T* __restrict__ Ah,
                                                     const typename Op<P>::T* __restrict__ Al, long long lda,
                                                     const typename Op<P>::T* __restrict__ Bh,
                                                     const typename Op<P>::T* __restrict__ Bl, long long ldb,
                                                     float* __restrict__ Cp, int L, int Ma, int Nb, int rows_per_chunk,
                                                     int vec) {
  using T = typename Op<P>::T;
  constexpr int NB = P == 1 ? 2 : 1;  // hi (+ lo) planes
  __shared__ __attribute__((aligned(16))) T sA[NB][64][TN_PAD];
  __shared__ __attribute__((aligned(16))) T sB[NB][64][TN_PAD];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, p = l & 15, g = l >> 4;
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const int r_lo = blockIdx.z * rows_per_chunk, r_hi = min(L, r_lo + rows_per_chunk);
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool v = vec != 0;
  // staging: thread t -> row rr = t >> 3 of the 32-row step, columns 8 (t & 7) .. + 7 of the tile
  const int rr = tid >> 3, cb = 8 * (tid & 7);
  for (int r0 = r_lo; r0 < r_hi; r0 += 32) {
    const int r = r0 + rr;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      T va[8], vb[8];
      // a row of A / B is contiguous in the feature index: 8 features of row r
      ld8(b ? Al : Ah, lda, r, r_hi, i0 + cb, Ma, v, va);
      ld8(b ? Bl : Bh, ldb, r, r_hi, j0 + cb, Nb, v, vb);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sA[b][cb + e][rr] = va[e];
        sB[b][cb + e][rr] = vb[e];
      }
    }
    __syncthreads();
    T ah[8], al[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) ah[j] = sA[0][16 * w + p][8 * g + j];
    if constexpr (P == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) al[j] = sA[1][16 * w + p][8 * g + j];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      T bh[8], bl[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bh[j] = sB[0][16 * c + p][8 * g + j];
      if constexpr (P == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bl[j] = sB[1][16 * c + p][8 * g + j];
      }
      acc[c] = mma32<P>(ah, al, bh, bl, acc[c]);
    }
    __syncthreads();
  }
  float* out = Cp + (long long)blockIdx.z * Ma * Nb;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int j = j0 + 16 * c + p;
    if (j >= Nb) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 16 * w + 4 * g + r;
      if (i < Ma) out[(long long)i * Nb + j] = acc[c][r];
    }
  }
}

// X^T Z partials, C[z][j][f] = sum over rows n of chunk z of X[n][j] Z[n][f], for D <= TDQ_MAXD
// columns of exact fp32 X (no GEMM shape): the input layer's dK0 = X^T ZB0 (Z fp32) and the output
// layer's dKo^T = dJ^T H (X = dJ, Z = the saved post-activations as hi + lo bf16 planes, ZP).  4
// features per thread (16 / 2 x 8-byte Z loads), short row chunks so that many waves are in flight
// (the kernel is latency-bound); blockDim.x threads cover 4 blockDim.x features.
template <int D, bool ZP>
__global__ void __launch_bounds__(256) lay_xtz_kernel(const float* __restrict__ X, const float* __restrict__ Z,
                                                      const __bf16* __restrict__ Zh, const __bf16* __restrict__ Zl,
                                                      int N, int W, float* __restrict__ Cp, int rows_per_chunk) {
  const int f = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (f >= W) return;
  const int n_lo = blockIdx.y * rows_per_chunk, n_hi = min(N, n_lo + rows_per_chunk);
  const bool v4 = (W % 4 == 0);
  f32x4 a[D];
#pragma unroll
  for (int j = 0; j < D; ++j) a[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int n = n_lo; n < n_hi; ++n) {
    const long long o = (long long)n * W + f;
    f32x4 z;
    if (v4) {
      if constexpr (ZP) {
        const bf16x4 h = *reinterpret_cast<const bf16x4*>(Zh + o), l = *reinterpret_cast<const bf16x4*>(Zl + o);
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = (float)h[e] + (float)l[e];
      } else {
        z = *reinterpret_cast<const f32x4*>(Z + o);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        z[e] = f + e < W ? (ZP ? (float)Zh[o + e] + (float)Zl[o + e] : Z[o + e]) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < D; ++j) a[j] += X[(long long)n * D + j] * z;
  }
  float* out = Cp + (long long)blockIdx.y * D * W;
#pragma unroll
  for (int j = 0; j < D; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (f + e < W) out[(long long)j * W + f + e] = a[j][e];
}

// ---- bf16 families: 128 x 128 workgroup tiles staged through LDS --------------------------------
// 4 waves in 2 x 2, each a 64 x 64 block (4 x 4 MFMA tiles): per 32-deep k-substep a wave reads 4 A
// and 4 B fragments from LDS for 16 MFMAs (x3 in bf16x3).  Two buffers: the next k-step's global
// loads are in flight while the current one is multiplied.

// 8 bf16 at element offset off + k of a row (zero when !ok or past K)
__device__ __forceinline__ bf16x8 ldr8(const __bf16* __restrict__ base, long long off, bool ok, int k, int K,
                                       bool vec) {
  bf16x8 r;
  if (ok) {
    const __bf16* p = base + off + k;
    if (vec && k + 8 <= K) return *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (k + j < K) ? p[j] : (__bf16)0.f;
    return r;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)0.f;
  return r;
}

typedef float f32x8 __attribute__((ext_vector_type(8)));

// 8 fp32 at element offset off + k of a row (zero when !ok or past K)
__device__ __forceinline__ f32x8 ldr8(const float* __restrict__ base, long long off, bool ok, int k, int K, bool vec) {
  f32x8 r;
  if (ok) {
    const float* p = base + off + k;
    if (vec && k + 8 <= K) {
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        r[j] = x0[j];
        r[4 + j] = x1[j];
      }
      return r;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (k + j < K) ? p[j] : 0.f;
    return r;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = 0.f;
  return r;
}

template <class T>
struct Vec8;
template <>
struct Vec8<__bf16> {
  using V = bf16x8;
};
template <>
struct Vec8<float> {
  using V = f32x8;
};

// 8 bf16 of (row, k..k+7) of a row-major [nrows][ld] matrix, zero outside
__device__ __forceinline__ bf16x8 ldg8(const __bf16* __restrict__ base, long long ld, int row, int nrows, int k, int K,
                                       bool vec) {
  return ldr8(base, (long long)row * ld, row < nrows, k, K, vec);
}

// Staged k-depth BK (template): 32 in general (bf16: 40 KB of staging, so with the half-tile
// epilogue 3-4 workgroups fit a CU), 64 where the LDS holds two workgroups per CU anyway.
template <int P, int BK>
constexpr int nn_lk() {  // LDS row stride (elements): 40 / 72 bf16, 36 fp32 - conflict-free fragment reads
  return BK + (P == 2 ? 4 : 8);
}
template <int BK>
constexpr int nn_rows_per_thread() {  // rows of the 128-row tiles one thread stages (8 k-values each)
  return 128 * (BK / 8) / 256;
}
template <int P, int BK>
constexpr int nn_stage_bytes() {  // {A, B} x 2 buffers x planes x 128 rows x LK elements
  return 2 * 2 * (P == 1 ? 2 : 1) * 128 * nn_lk<P, BK>() * (P == 2 ? 4 : 2);
}

// the A and B rows a thread stages (element offsets of row starts, validity): row c is tile row
// tid / (BK / 8) + c * 256 / (BK / 8)
struct NnRows {
  long long a[4], b[4];
  bool va[4], vb[4];
};
template <int BK>
__device__ __forceinline__ int nn_row(int c) {
  constexpr int CPR = BK / 8;
  return (int)threadIdx.x / CPR + c * (256 / CPR);
}

// The main loop of a 128 x 128 tile: acc[i][j] = the wave's (i, j) 16 x 16 block of A B over K.
// bf16 families: one v_mfma_f32_16x16x32_bf16 per block and 32-deep substep (x3 in bf16x3); fp32:
// eight v_mfma_f32_16x16x4_f32 on the same 8-value fragments (MFMA kk takes k = 8 g + kk of lane
// group g in both operands, so the permuted order sums the same products).
template <int P, int BK>
__device__ __forceinline__ void nn_loop(typename Op<P>::T* smem, const typename Op<P>::T* __restrict__ Ah,
                                        const typename Op<P>::T* __restrict__ Al,
                                        const typename Op<P>::T* __restrict__ Bh,
                                        const typename Op<P>::T* __restrict__ Bl, const NnRows& R, int K, bool v,
                                        f32x4 (&acc)[4][4]) {
  using V = typename Vec8<typename Op<P>::T>::V;
  constexpr int NB = P == 1 ? 2 : 1;
  constexpr int LK = nn_lk<P, BK>(), NR = nn_rows_per_thread<BK>(), CPR = BK / 8;
  constexpr int SZ = 128 * LK;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, p = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int sk = (tid % CPR) * 8;
  auto sA = [&](int buf, int b) { return smem + (buf * NB + b) * SZ; };
  auto sB = [&](int buf, int b) { return smem + (2 * NB + buf * NB + b) * SZ; };
  V ra[NR][NB], rb[NR][NB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < NR; ++c) {
        ra[c][b] = ldr8(b ? Al : Ah, R.a[c], R.va[c], k0 + sk, K, v);
        rb[c][b] = ldr8(b ? Bl : Bh, R.b[c], R.vb[c], k0 + sk, K, v);
      }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < NR; ++c) {
        const int r = nn_row<BK>(c);
        *reinterpret_cast<V*>(sA(buf, b) + r * LK + sk) = ra[c][b];
        *reinterpret_cast<V*>(sB(buf, b) + r * LK + sk) = rb[c][b];
      }
  };
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  gload(0);
  sstore(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) gload(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      V a[4][NB], b[4][NB];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          a[i][q] = *reinterpret_cast<const V*>(sA(buf, q) + (wm * 64 + 16 * i + p) * LK + kk + 8 * g);
          b[i][q] = *reinterpret_cast<const V*>(sB(buf, q) + (wn * 64 + 16 * i + p) * LK + kk + 8 * g);
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (P == 2) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][0][e], b[j][0][e], acc[i][j], 0, 0, 0);
          } else {
            if constexpr (P == 1) {
              acc[i][j] = mfma_bf(a[i][1], b[j][0], acc[i][j]);
              acc[i][j] = mfma_bf(a[i][0], b[j][1], acc[i][j]);
            }
            acc[i][j] = mfma_bf(a[i][0], b[j][0], acc[i][j]);
          }
        }
    }
    if (more) {
      sstore(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
}

// XCD-aware tile order: workgroup L runs on XCD L % 8, so the tiles of one XCD are made logically
// consecutive (consecutive tiles share an A row block - it is read once into that XCD's L2)
__device__ __forceinline__ int xcd_tile(int L, int total) {
  const int q = total / 8;
  return L < 8 * q ? (L % 8) * q + L / 8 : L;
}

template <int P>
__global__ void __launch_bounds__(256) lay_nn2_kernel(const __bf16* __restrict__ Ah, const __bf16* __restrict__ Al,
                                                      long long lda, const __bf16* __restrict__ Bh,
                                                      const __bf16* __restrict__ Bl, long long ldb,
                                                      float* __restrict__ C, long long ldc, int M, int N, int K,
                                                      int vec) {
  constexpr int BK = 32;
  __shared__ __attribute__((aligned(16))) __bf16 smem[nn_stage_bytes<P, BK>() / 2];  // (bf16 families only)
  const int gx = (N + 127) / 128;
  const int T = xcd_tile(blockIdx.x, gridDim.x);
  const int m0 = (T / gx) * 128, n0 = (T % gx) * 128;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, p = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  NnRows R;
#pragma unroll
  for (int c = 0; c < nn_rows_per_thread<BK>(); ++c) {
    const int r = nn_row<BK>(c);
    R.a[c] = (long long)(m0 + r) * lda;
    R.b[c] = (long long)(n0 + r) * ldb;
    R.va[c] = m0 + r < M;
    R.vb[c] = n0 + r < N;
  }
  f32x4 acc[4][4];
  nn_loop<P, BK>(smem, Ah, Al, Bh, Bl, R, K, vec != 0, acc);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + 16 * j + p;
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ro = m0 + wm * 64 + 16 * i + 4 * g + r;
        if (ro < M) C[(long long)ro * ldc + col] = acc[i][j][r];
      }
    }
}

// ---- the layer jet on (point, feature) tiles: GEMM epilogues and the elementwise end layers ------
// Tiles are PT = 128 / S points x 128 features; thread t owns feature quad 4 (t & 31) of points
// t >> 5, + 8, ... for all S streams.  Modes:
//   EPI_FWD   Z -> H = jet(Z + b), written as the next GEMMs' bf16 operands hi = rne(H) and
//             lo = rne(H - hi) (hi + lo is also the saved post-activation of the adjoint)
//   EPI_BWD   HB + saved H (hi + lo) -> ZB = adjoint jet, written as bf16 hi (+ lo for bf16x3), and
//             per-tile column sums of ZB's value stream (the bias gradient's partials)
//   EPI_BWD0  the input layer's adjoint: no ZB leaves the kernel, only per-tile partials of every
//             quantity the input layer's gradient needs - column sums of all S streams (bias; the
//             first-order streams' dK0 rows) and X^T zb (dK0 = X^T ZB0 over the d_in <= 8 exact
//             fp32 coordinates)
// Partials: part[tile_y][q][Nout], q < 1 (EPI_BWD) or S + d_in (EPI_BWD0), summed by the caller.
enum { EPI_FWD = 0, EPI_BWD = 1, EPI_BWD0 = 2, EPI_FWDJ = 3 };  // FWDJ: EPI_FWD + the output layer's J dots

struct EpiArgs {
  int Npts, Nout, d_in;
  const float* bias;         // EPI_FWD: [Nout]
  const __bf16 *Hh, *Hl;     // EPI_BWD*: the layer's saved post-activations [S * Npts][Nout]
  __bf16 *Oh, *Ol;           // EPI_FWD / EPI_BWD outputs [S * Npts][Nout] (Ol nullable in EPI_BWD)
  const float* H32;          // fp32 engine (F32): the saved post-activations, one fp32 plane
  float* O32;                // fp32 engine: the output plane
  // EPI_FWD of the last hidden layer (nullable): the output layer's J = H Ko fused in - per
  // 64-column group partial dots jpart[col / 64][s][n][q] (the caller sums the groups, adds bo)
  const float* Ko;           // [Nout][d_out]
  float* jpart;
  int d_out;
  float* part;               // EPI_BWD* partials (nullable in EPI_BWD)
  const float* X;            // EPI_BWD0: [Npts][d_in]
  LSpec sp;
};

// src(s, t) -> the f32x4 input (Z or HB) of stream s, tile point t, this thread's feature quad.
// red: LDS scratch of 4 x (S + TDQ_MAXD) x 128 floats (may alias the source tile: a barrier
// precedes its first write).  Every thread of the block must call this.  F32: the fp32 engine -
// activations / adjoints are single fp32 planes (H32 / O32) instead of bf16 hi / lo pairs.
// CW: feature columns per call (128, or 64 when a GEMM tile's epilogue runs in two column halves
// to halve its LDS tile); CW / 4 threads cover a row, 1024 / CW rows per pass.
template <int S, int MODE_, bool F32, int CW = 128, class Src>
__device__ __forceinline__ void lay_epilogue(const EpiArgs& e, int ty, int n0, Src src, float* red) {
  constexpr bool JDOT = MODE_ == EPI_FWDJ;
  constexpr int MODE = JDOT ? (int)EPI_FWD : MODE_;
  constexpr int PT = 128 / S;
  constexpr int NS = MODE == EPI_BWD0 ? S : 1;
  constexpr int NX = MODE == EPI_BWD0 ? TDQ_MAXD : 1;
  constexpr int QL = CW / 4, RP = 256 / QL;  // threads per row, rows per pass
  const int tid = threadIdx.x, pt0 = ty * PT;
  const int f4 = (tid % QL) * 4, col = n0 + f4;
  const bool cok = col < e.Nout;  // (Nout % 4 == 0: a quad is all in or all out)
  float bb[4] = {0.f, 0.f, 0.f, 0.f}, ps[NS][4], px[NX][4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
#pragma unroll
    for (int q = 0; q < NS; ++q) ps[q][v] = 0.f;
#pragma unroll
    for (int q = 0; q < NX; ++q) px[q][v] = 0.f;
  }
  if (MODE == EPI_FWD && cok) {
#pragma unroll
    for (int v = 0; v < 4; ++v) bb[v] = e.bias[col + v];
  }
  float ko[JDOT ? TDQ_MAXO : 1][4];
#pragma unroll
  for (int q = 0; q < (JDOT ? TDQ_MAXO : 1); ++q)
#pragma unroll
    for (int v = 0; v < 4; ++v) ko[q][v] = (JDOT && cok && q < e.d_out) ? e.Ko[(long long)(col + v) * e.d_out + q] : 0.f;
  auto point = [&](int t) {
    const int n = pt0 + t;
    const bool ok = cok && n < e.Npts;
    float y[S][4];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int v = 0; v < 4; ++v) y[s][v] = 0.f;
    if (ok) {
    float x[S][4];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const f32x4 q = src(s, t);
#pragma unroll
      for (int v = 0; v < 4; ++v) x[s][v] = q[v];
    }
    if constexpr (MODE == EPI_FWD) {
      lay_jet_fwd<S, 4>(x, bb, e.sp, y);
    } else {
      float h[S][4];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const long long o = ((long long)s * e.Npts + n) * e.Nout + col;
        if constexpr (F32) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(e.H32 + o);
#pragma unroll
          for (int v = 0; v < 4; ++v) h[s][v] = q[v];
        } else {
          const bf16x4 hh = *reinterpret_cast<const bf16x4*>(e.Hh + o), hl = *reinterpret_cast<const bf16x4*>(e.Hl + o);
#pragma unroll
          for (int v = 0; v < 4; ++v) h[s][v] = (float)hh[v] + (float)hl[v];
        }
      }
      lay_jet_bwd<S, 4>(h, x, e.sp, y);
#pragma unroll
      for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int v = 0; v < 4; ++v) ps[q][v] += y[q][v];
      if constexpr (MODE == EPI_BWD0) {
#pragma unroll
        for (int j = 0; j < TDQ_MAXD; ++j) {
          if (j < e.d_in) {
            const float xv = e.X[(long long)n * e.d_in + j];
#pragma unroll
            for (int v = 0; v < 4; ++v) px[j][v] += xv * y[0][v];
          }
        }
      }
    }
    if constexpr (MODE != EPI_BWD0) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const long long o = ((long long)s * e.Npts + n) * e.Nout + col;
        if constexpr (F32) {
          *reinterpret_cast<f32x4*>(e.O32 + o) = f32x4{y[s][0], y[s][1], y[s][2], y[s][3]};
        } else {
          bf16x4 hv, lv;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            hv[v] = (__bf16)y[s][v];
            lv[v] = (__bf16)(y[s][v] - (float)hv[v]);
          }
          *reinterpret_cast<bf16x4*>(e.Oh + o) = hv;
          if (e.Ol != nullptr) *reinterpret_cast<bf16x4*>(e.Ol + o) = lv;
        }
      }
    }
    }  // ok
    if constexpr (JDOT) {
      {  // J partials of this row's 64-column group: a 16-lane reduction (whole groups share t)
#pragma unroll
        for (int q = 0; q < TDQ_MAXO; ++q) {
          if (q >= e.d_out) break;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            float a = y[s][0] * ko[q][0] + y[s][1] * ko[q][1] + y[s][2] * ko[q][2] + y[s][3] * ko[q][3];
#pragma unroll
            for (int m = 1; m < 16; m <<= 1) a += __shfl_xor(a, m, 64);
            if ((tid & 15) == 0 && n < e.Npts && col < e.Nout)
              e.jpart[(((long long)(col >> 6) * S + s) * e.Npts + n) * e.d_out + q] = a;
          }
        }
      }
    }
  };
  if constexpr (MODE == EPI_BWD0) {  // (rolled: the partial accumulators already hold 4 (S + 8) registers)
#pragma unroll 1
    for (int t = tid / QL; t < PT; t += RP) point(t);
  } else {
    for (int t = tid / QL; t < PT; t += RP) point(t);
  }
  if constexpr (MODE != EPI_FWD) {
    if (e.part == nullptr) return;  // (uniform)
    const int NP = MODE == EPI_BWD ? 1 : S + e.d_in;
    // the lanes of a wave with the same features (lane % QL) combined, then the 4 waves via LDS
    const int w = tid >> 6;
    __syncthreads();  // red may alias the source tile
#pragma unroll
    for (int q = 0; q < NS + (MODE == EPI_BWD0 ? TDQ_MAXD : 0); ++q) {
      if (q >= NP) break;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float a = q < NS ? ps[q < NS ? q : 0][v] : px[q >= NS ? q - NS : 0][v];
#pragma unroll
        for (int m = QL; m < 64; m <<= 1) a += __shfl_xor(a, m, 64);
        if ((tid & 63) < QL) red[(w * NP + q) * CW + f4 + v] = a;
      }
    }
    __syncthreads();
    for (int i = tid; i < NP * CW; i += 256) {
      const int q = i / CW, c = i % CW;
      if (n0 + c >= e.Nout) continue;
      const float a = red[q * CW + c] + red[(NP + q) * CW + c] + red[(2 * NP + q) * CW + c] +
                      red[(3 * NP + q) * CW + c];
      e.part[((long long)ty * NP + q) * e.Nout + n0 + c] = a;
    }
  }
}

// NN GEMM + layer jet: the 128 tile rows are S streams x PT points (row s PT + t = stream s of point
// pt0 + t, global row s Npts + pt0 + t of the stream-major planes), so one tile holds every stream of
// its points; the accumulators go through LDS (a 128 x 132 fp32 tile) into lay_epilogue.
// LDS row strides of the fp32 C tile (whole: 132, half: 68): the 4 row groups of a store land 16
// banks apart

struct NnjArgs {
  const void *Ah, *Al, *Bh, *Bl;  // A planes [S * Npts][K]; B^T [Nout][K] (bf16, or fp32 when P == 2)
  int K, vec;
  EpiArgs e;
};

template <int P, int S, int MODE>
__global__ void __launch_bounds__(256) lay_nnj_kernel(NnjArgs a) {
  constexpr int PT = 128 / S;
  // k-depth of a staged step: 32, except the bf16 input-layer adjoint (whole C tile, 2 workgroups
  // per CU either way: 64-deep steps halve its barriers, 286 vs 328 us at W512)
  constexpr int BK = (P == 0 && MODE == EPI_BWD0) ? 64 : 32;
  constexpr int STG = nn_stage_bytes<P, BK>();
  // bf16 forward / hidden adjoint: the C tile through LDS in two 64-column halves (40 KB of LDS in
  // all, so 3-4 workgroups per CU instead of 2: forward 238 vs 278 us at W512); the other modes and
  // precisions keep the whole tile (two halves measured slower there: profiles/r5lay7_*)
  constexpr bool HALF = P == 0 && MODE != EPI_BWD0;  // (EPI_FWDJ included)
  constexpr int CW = HALF ? 64 : 128, CS = CW + 4;
  constexpr int EPI = 128 * CS * 4;
  static_assert(4 * (TDQ_MAXS + TDQ_MAXD) * CW * 4 <= EPI, "partials scratch fits the C tile");
  using E = typename Op<P>::T;
  __shared__ __attribute__((aligned(16))) E smem[(STG > EPI ? STG : EPI) / sizeof(E)];
  const int gx = (a.e.Nout + 127) / 128;
  const int T = xcd_tile(blockIdx.x, gridDim.x);
  const int ty = T / gx, n0 = (T % gx) * 128, pt0 = ty * PT;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, p = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  NnRows R;
#pragma unroll
  for (int c = 0; c < nn_rows_per_thread<BK>(); ++c) {
    const int r = nn_row<BK>(c), rs = r / PT, rt = r % PT;
    R.va[c] = rs < S && pt0 + rt < a.e.Npts;
    R.a[c] = ((long long)rs * a.e.Npts + pt0 + rt) * a.K;
    R.b[c] = (long long)(n0 + r) * a.K;
    R.vb[c] = n0 + r < a.e.Nout;
  }
  f32x4 acc[4][4];
  nn_loop<P, BK>(smem, (const E*)a.Ah, (const E*)a.Al, (const E*)a.Bh, (const E*)a.Bl, R, a.K, a.vec != 0, acc);
  float* sC = reinterpret_cast<float*>(smem);
  const int f4 = (tid % (CW / 4)) * 4;
#pragma unroll
  for (int hh = 0; hh < (HALF ? 2 : 1); ++hh) {
    __syncthreads();  // staging buffers (first pass) / the previous half's readers are done
    if (!HALF || wn == hh) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sC[(wm * 64 + 16 * i + 4 * g + r) * CS + (HALF ? 0 : wn * 64) + 16 * j + p] = acc[i][j][r];
    }
    __syncthreads();
    lay_epilogue<S, MODE, P == 2, CW>(a.e, ty, n0 + 64 * hh, [&](int s, int t) {
      return *reinterpret_cast<const f32x4*>(&sC[(s * PT + t) * CS + f4]);
    }, sC);
  }
}

// The input layer forward without a GEMM: Z = X K0 (d_in <= 8 exact fp32 columns), the first-order
// streams' Z = the K0 row of their coordinate, second-order streams 0 - straight into the jet.
template <int S, bool F32>
__global__ void __launch_bounds__(256) lay_in_fwd_kernel(EpiArgs e, const float* __restrict__ X,
                                                         const float* __restrict__ K0) {
  __shared__ float red[4];  // (EPI_FWD: no partials)
  const int gx = (e.Nout + 127) / 128;
  const int ty = blockIdx.x / gx, n0 = (blockIdx.x % gx) * 128, pt0 = ty * (128 / S);
  const int col = n0 + (threadIdx.x & 31) * 4;
  const bool cok = col < e.Nout;
  float k[TDQ_MAXD][4];
#pragma unroll
  for (int j = 0; j < TDQ_MAXD; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v) k[j][v] = (cok && j < e.d_in) ? K0[(long long)j * e.Nout + col + v] : 0.f;
  lay_epilogue<S, EPI_FWD, F32>(e, ty, n0, [&](int s, int t) {
    f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
    if (s == 0) {
      const int n = pt0 + t;
#pragma unroll
      for (int j = 0; j < TDQ_MAXD; ++j)
        if (j < e.d_in) {
          const float xv = X[(long long)n * e.d_in + j];
#pragma unroll
          for (int v = 0; v < 4; ++v) z[v] += xv * k[j][v];
        }
    } else if (e.sp.stype[s] == 1) {  // d/dx_c of X K0 = row c of K0 (register-indexed select)
#pragma unroll
      for (int j = 0; j < TDQ_MAXD; ++j)
        if (j == e.sp.coord[s]) {
#pragma unroll
          for (int v = 0; v < 4; ++v) z[v] = k[j][v];
        }
    }
    return z;
  }, red);
}

// The last hidden layer's adjoint without materializing HB = dJ Ko^T (the output layer, d_out <= 4
// columns): hb computed per (point, feature quad) from dJ and the thread's Ko rows.  MODE EPI_BWD,
// or EPI_BWD0 when the last hidden layer is the input layer.
template <int S, int MODE, bool F32>
__global__ void __launch_bounds__(256) lay_out_bwd_kernel(EpiArgs e, const float* __restrict__ dJ,
                                                          const float* __restrict__ Ko, int d_out) {
  __shared__ __attribute__((aligned(16))) float red[4 * (TDQ_MAXS + TDQ_MAXD) * 128];
  const int gx = (e.Nout + 127) / 128;
  const int ty = blockIdx.x / gx, n0 = (blockIdx.x % gx) * 128, pt0 = ty * (128 / S);
  const int col = n0 + (threadIdx.x & 31) * 4;
  const bool cok = col < e.Nout;
  float ko[TDQ_MAXO][4];
#pragma unroll
  for (int q = 0; q < TDQ_MAXO; ++q)
#pragma unroll
    for (int v = 0; v < 4; ++v) ko[q][v] = (cok && q < d_out) ? Ko[(long long)(col + v) * d_out + q] : 0.f;
  lay_epilogue<S, MODE, F32>(e, ty, n0, [&](int s, int t) {
    const float* dj = dJ + ((long long)s * e.Npts + pt0 + t) * d_out;
    f32x4 hb = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q)
      if (q < d_out) {
        const float d = dj[q];
#pragma unroll
        for (int v = 0; v < 4; ++v) hb[v] += d * ko[q][v];
      }
    return hb;
  }, red);
}


// TN, bf16 families: 128 x 128 output tiles.  The 32-row k-step of A [rows][Ma] and B [rows][Nb]
// is staged row-major ([row][feature], 16-byte stores, rows of 144 elements = 72 banks) and the
// fragments are read with ds_read_b64_tr_b16 (cdna_hip_programming.md T10): a 16-lane group reads
// rows 8g + q, columns 4p .. 4p + 3 (lane 4q + p) and lane i receives feature column i of those 4
// k-rows - two reads (rows 8g.., 8g + 4..) give the 8 k-values of a 16x16x32 fragment.
constexpr int TS = 144;
template <int P>
__global__ void __launch_bounds__(256) lay_tn2_kernel(const __bf16* __restrict__ Ah, const __bf16* __restrict__ Al,
                                                      long long lda, const __bf16* __restrict__ Bh,
                                                      const __bf16* __restrict__ Bl, long long ldb,
                                                      float* __restrict__ Cp, int L, int Ma, int Nb,
                                                      int rows_per_chunk, int vec) {
  constexpr int NB = P == 1 ? 2 : 1;
  constexpr int RK = P == 1 ? 32 : 64;  // rows per staged step (bf16x3: two planes, 32)
  constexpr int NRS = RK / 16;          // rows one thread stages per step
  __shared__ __attribute__((aligned(16))) __bf16 sA[2][NB][RK * TS];
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][NB][RK * TS];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  // XCD-aware order (xcd_tile): the tiles of one row chunk run on one XCD, so its A / B rows are read
  // from HBM once into that XCD's L2 (round-robin placement read them ~3x)
  const int gx = (Nb + 127) / 128, gy = (Ma + 127) / 128;
  const int T = xcd_tile(blockIdx.x, gridDim.x);
  const int bz = T / (gx * gy), i0 = ((T / gx) % gy) * 128, j0 = (T % gx) * 128;
  const int r_lo = bz * rows_per_chunk, r_hi = min(L, r_lo + rows_per_chunk);
  const bool v = vec != 0;
  // staging: thread t stages feature chunk (t & 15) of rows (t >> 4) + 16 c of an RK-row step
  const int rr = tid >> 4, fc = (tid & 15) * 8;
  // transposed-read address of this lane: row 8g + q, column 4p (+ the tile's first column)
  const int trq = (l & 15) >> 2, trp = l & 3;
  const int ta = (8 * g + trq) * TS + 4 * trp, tb = ta + 4 * TS;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // double-buffered: the next step's global loads are in flight during this step's MFMAs
  bf16x8 ra[NRS][NB], rb[NRS][NB];
  auto gload = [&](int r0) {
#pragma unroll
    for (int q = 0; q < NB; ++q)
#pragma unroll
      for (int c = 0; c < NRS; ++c) {
        ra[c][q] = ldg8(q ? Al : Ah, lda, r0 + rr + 16 * c, r_hi, i0 + fc, Ma, v);
        rb[c][q] = ldg8(q ? Bl : Bh, ldb, r0 + rr + 16 * c, r_hi, j0 + fc, Nb, v);
      }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NB; ++q)
#pragma unroll
      for (int c = 0; c < NRS; ++c) {
        *reinterpret_cast<bf16x8*>(&sA[buf][q][(rr + 16 * c) * TS + fc]) = ra[c][q];
        *reinterpret_cast<bf16x8*>(&sB[buf][q][(rr + 16 * c) * TS + fc]) = rb[c][q];
      }
  };
  if (r_lo < r_hi) {
    gload(r_lo);
    sstore(0);
  }
  __syncthreads();
  int buf = 0;
  for (int r0 = r_lo; r0 < r_hi; r0 += RK) {
    const bool more = r0 + RK < r_hi;
    if (more) gload(r0 + RK);
#pragma unroll
    for (int kk = 0; kk < RK; kk += 32) {
      bf16x8 a[4][NB], b[4][NB];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int ca = kk * TS + wm * 64 + 16 * i, cb = kk * TS + wn * 64 + 16 * i;
          a[i][q] = cat8(tr_read(&sA[buf][q][ta + ca]), tr_read(&sA[buf][q][tb + ca]));
          b[i][q] = cat8(tr_read(&sB[buf][q][ta + cb]), tr_read(&sB[buf][q][tb + cb]));
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (P == 1) {
            acc[i][j] = mfma_bf(a[i][1], b[j][0], acc[i][j]);
            acc[i][j] = mfma_bf(a[i][0], b[j][1], acc[i][j]);
          }
          acc[i][j] = mfma_bf(a[i][0], b[j][0], acc[i][j]);
        }
    }
    if (more) {
      sstore(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  const int p = l & 15;
  float* out = Cp + (long long)bz * Ma * Nb;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = j0 + wn * 64 + 16 * j + p;
      if (jj >= Nb) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = i0 + wm * 64 + 16 * i + 4 * g + r;
        if (ii < Ma) out[(long long)ii * Nb + jj] = acc[i][j][r];
      }
    }
}

template <class T>
bool aligned16(const void* p, long long ld) {
  return ((reinterpret_cast<uintptr_t>(p) & 15) == 0) && (ld % (16 / (long long)sizeof(T))) == 0;
}

}  // namespace

extern "C" {

// prec: 0 bf16, 1 bf16x3, 2 fp32 (Ah / Bh then fp32).  Al / Bl: the lo planes (bf16x3 only).
int tdq_lay_nn(int prec, const void* Ah, const void* Al, long long lda, const void* Bh, const void* Bl, long long ldb,
               float* C, long long ldc, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || prec < 0 || prec > 2 || (prec == 1 && (Al == nullptr || Bl == nullptr)))
    return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((N + 127) / 128, (M + 63) / 64);
  if (grid.y > 65535u) return (int)hipErrorInvalidValue;
  if (prec < 2) {  // the LDS-tiled kernels
    const int vec = aligned16<__bf16>(Ah, lda) && aligned16<__bf16>(Bh, ldb) &&
                    (prec == 0 || (aligned16<__bf16>(Al, lda) && aligned16<__bf16>(Bl, ldb)));
    const long long tiles = (long long)((N + 127) / 128) * ((M + 127) / 128);
    if (tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    const dim3 g2((unsigned)tiles);
    if (prec == 0)
      hipLaunchKernelGGL(lay_nn2_kernel<0>, g2, dim3(256), 0, st, (const __bf16*)Ah, (const __bf16*)Al, lda,
                         (const __bf16*)Bh, (const __bf16*)Bl, ldb, C, ldc, M, N, K, vec);
    else
      hipLaunchKernelGGL(lay_nn2_kernel<1>, g2, dim3(256), 0, st, (const __bf16*)Ah, (const __bf16*)Al, lda,
                         (const __bf16*)Bh, (const __bf16*)Bl, ldb, C, ldc, M, N, K, vec);
    TDQ_CHECK_LAUNCH();
    return 0;
  }
  {  // fp32: the direct-load kernel with fp32 MFMA
    const int vec = aligned16<float>(Ah, lda) && aligned16<float>(Bh, ldb);
    hipLaunchKernelGGL(lay_nn_kernel<2>, grid, dim3(256), 0, st, (const float*)Ah, (const float*)nullptr, lda,
                       (const float*)Bh, (const float*)nullptr, ldb, C, ldc, M, N, K, vec);
  }
  TDQ_CHECK_LAUNCH();
  return 0;
}

// Cp: nchunks x Ma x Nb fp32 partials (rows_per_chunk a multiple of 32); the caller sums dim 0
int tdq_lay_tn(int prec, const void* Ah, const void* Al, long long lda, const void* Bh, const void* Bl, long long ldb,
               float* Cp, int L, int Ma, int Nb, int rows_per_chunk, void* stream) {
  if (L <= 0 || Ma <= 0 || Nb <= 0 || rows_per_chunk <= 0 || rows_per_chunk % 32 != 0 || prec < 0 || prec > 2 ||
      (prec == 1 && (Al == nullptr || Bl == nullptr)))
    return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nch = (L + rows_per_chunk - 1) / rows_per_chunk;
  dim3 grid((Nb + 63) / 64, (Ma + 63) / 64, nch);
  if (grid.z > 65535u) return (int)hipErrorInvalidValue;
  if (prec < 2) {  // the 128 x 128 LDS-tiled kernels
    const int vec = aligned16<__bf16>(Ah, lda) && aligned16<__bf16>(Bh, ldb) &&
                    (prec == 0 || (aligned16<__bf16>(Al, lda) && aligned16<__bf16>(Bl, ldb)));
    const long long tiles = (long long)((Nb + 127) / 128) * ((Ma + 127) / 128) * nch;
    if (tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
    const dim3 g2((unsigned)tiles);
    if (prec == 0)
      hipLaunchKernelGGL(lay_tn2_kernel<0>, g2, dim3(256), 0, st, (const __bf16*)Ah, (const __bf16*)Al, lda,
                         (const __bf16*)Bh, (const __bf16*)Bl, ldb, Cp, L, Ma, Nb, rows_per_chunk, vec);
    else
      hipLaunchKernelGGL(lay_tn2_kernel<1>, g2, dim3(256), 0, st, (const __bf16*)Ah, (const __bf16*)Al, lda,
                         (const __bf16*)Bh, (const __bf16*)Bl, ldb, Cp, L, Ma, Nb, rows_per_chunk, vec);
    TDQ_CHECK_LAUNCH();
    return 0;
  }
  {  // fp32: LDS-transposed staging with fp32 MFMA
    const int vec = aligned16<float>(Ah, lda) && aligned16<float>(Bh, ldb);
    hipLaunchKernelGGL(lay_tn_kernel<2>, grid, dim3(256), 0, st, (const float*)Ah, (const float*)nullptr, lda,
                       (const float*)Bh, (const float*)nullptr, ldb, Cp, L, Ma, Nb, rows_per_chunk, vec);
  }
  TDQ_CHECK_LAUNCH();
  return 0;
}

// Cp: nchunks x d_in x W partials of X^T Z (X [N][d_in] fp32; Z [N][W] fp32, or - Z == nullptr - the
// bf16 planes Zh + Zl); the caller sums dim 0
int tdq_lay_xtz2(const float* X, int d_in, const float* Z, const void* Zh, const void* Zl, int N, int W, float* Cp,
                 int rows_per_chunk, void* stream) {
  if (N <= 0 || W <= 0 || d_in < 1 || d_in > TDQ_MAXD || rows_per_chunk <= 0 ||
      (Z == nullptr && (Zh == nullptr || Zl == nullptr)))
    return (int)hipErrorInvalidValue;
  const int nch = (N + rows_per_chunk - 1) / rows_per_chunk;
  const int quads = (W + 3) / 4;
  const int bs = quads >= 256 ? 256 : ((quads + 63) / 64) * 64;
  const dim3 grid((quads + bs - 1) / bs, nch);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const __bf16 *h = (const __bf16*)Zh, *l = (const __bf16*)Zl;
  switch (d_in) {
#define TDQ_XTZ(d_)                                                                                          \
  case d_:                                                                                                   \
    if (Z != nullptr)                                                                                        \
      hipLaunchKernelGGL((lay_xtz_kernel<d_, false>), grid, dim3(bs), 0, st, X, Z, h, l, N, W, Cp, rows_per_chunk); \
    else                                                                                                     \
      hipLaunchKernelGGL((lay_xtz_kernel<d_, true>), grid, dim3(bs), 0, st, X, Z, h, l, N, W, Cp, rows_per_chunk);  \
    break;
    TDQ_XTZ(1) TDQ_XTZ(2) TDQ_XTZ(3) TDQ_XTZ(4) TDQ_XTZ(5) TDQ_XTZ(6) TDQ_XTZ(7) TDQ_XTZ(8)
#undef TDQ_XTZ
  }
  TDQ_CHECK_LAUNCH();
  return 0;
}

int tdq_lay_xtz(const float* X, int d_in, const float* Z, int N, int W, float* Cp, int rows_per_chunk, void* stream) {
  if (Z == nullptr) return (int)hipErrorInvalidValue;
  return tdq_lay_xtz2(X, d_in, Z, nullptr, nullptr, N, W, Cp, rows_per_chunk, stream);
}

// Host side of the layer-jet kernels: EpiArgs from the common arguments; false when invalid.
// f32: the fp32 engine - Hh is the fp32 H plane and Oh the fp32 output plane (Hl / Ol unused).
static bool epi_args(EpiArgs& e, int S, const int* spec, int Npts, int Nout, int d_in, bool f32, const void* Hh,
                     const void* Hl, void* Oh, void* Ol) {
  if (Npts <= 0 || Nout <= 0 || Nout % 4 != 0 || d_in < 0 || d_in > TDQ_MAXD) return false;
  if (!lspec_parse(spec, S, e.sp)) return false;
  for (int s = 0; s < S; ++s)
    if (e.sp.stype[s] == 1 && (spec[3 * s + 1] < 0 || spec[3 * s + 1] >= TDQ_MAXD)) return false;
  const uintptr_t al = f32 ? 15 : 7;  // 16-byte fp32 / 8-byte bf16 quads
  if (((reinterpret_cast<uintptr_t>(Hh) | reinterpret_cast<uintptr_t>(Oh)) & al) != 0 ||
      (!f32 && ((reinterpret_cast<uintptr_t>(Hl) | reinterpret_cast<uintptr_t>(Ol)) & 7) != 0))
    return false;
  e.Npts = Npts;
  e.Nout = Nout;
  e.d_in = d_in;
  e.bias = nullptr;
  e.part = nullptr;
  e.X = nullptr;
  e.Hh = f32 ? nullptr : (const __bf16*)Hh;
  e.Hl = f32 ? nullptr : (const __bf16*)Hl;
  e.Oh = f32 ? nullptr : (__bf16*)Oh;
  e.Ol = f32 ? nullptr : (__bf16*)Ol;
  e.H32 = f32 ? (const float*)Hh : nullptr;
  e.O32 = f32 ? (float*)Oh : nullptr;
  e.Ko = nullptr;
  e.jpart = nullptr;
  e.d_out = 0;
  return true;
}

static long long epi_tiles(int S, int Npts, int Nout) {
  return (long long)((Nout + 127) / 128) * ((Npts + 128 / S - 1) / (128 / S));
}

// prec 0 bf16 / 1 bf16x3 / 2 fp32; mode: EPI_FWD (bias, Oh, Ol), EPI_BWD (Hh, Hl, Oh, Ol nullable,
// part nullable [tiles_y][1][Nout]), EPI_BWD0 (Hh, Hl, part [tiles_y][S + d_in][Nout], X [Npts][d_in]);
// tiles_y = ceil(Npts / (128 / S)).  fp32: A / B fp32, Hh / Oh single fp32 planes, Hl / Ol unused.
// EPI_FWD with jpart: the output layer's J partials (Ko [Nout][d_out], d_out <= 4; jpart
// [ceil(Nout / 64)][S][Npts][d_out]).
// Planes are contiguous: A [S * Npts][K], B^T [Nout][K], H / outputs [S * Npts][Nout].
int tdq_lay_nnj(int prec, int mode, int S, const int* spec, const void* Ah, const void* Al, const void* Bh,
                const void* Bl, int Npts, int K, int Nout, const float* bias, const void* Hh, const void* Hl, void* Oh,
                void* Ol, float* part, const float* X, int d_in, const float* Ko, float* jpart, int d_out,
                void* stream) {
  NnjArgs a;
  const bool f32 = prec == 2;
  if (prec < 0 || prec > 2 || mode < 0 || mode > 2 || K <= 0 || Ah == nullptr || Bh == nullptr ||
      (prec == 1 && (Al == nullptr || Bl == nullptr)) ||
      !epi_args(a.e, S, spec, Npts, Nout, mode == EPI_BWD0 ? d_in : 0, f32, Hh, Hl, Oh, Ol))
    return (int)hipErrorInvalidValue;
  if (mode == EPI_FWD ? (bias == nullptr || Oh == nullptr || (!f32 && Ol == nullptr))
                      : (Hh == nullptr || (!f32 && Hl == nullptr) ||
                         (mode == EPI_BWD ? Oh == nullptr : (part == nullptr || X == nullptr || d_in < 1))))
    return (int)hipErrorInvalidValue;
  a.e.bias = bias;
  a.e.part = part;
  a.e.X = X;
  if (jpart != nullptr && (mode != EPI_FWD || Ko == nullptr || d_out < 1 || d_out > TDQ_MAXO))
    return (int)hipErrorInvalidValue;
  const int kmode = (mode == EPI_FWD && jpart != nullptr) ? (int)EPI_FWDJ : mode;
  a.e.Ko = Ko;
  a.e.jpart = jpart;
  a.e.d_out = d_out;
  a.Ah = Ah; a.Al = Al; a.Bh = Bh; a.Bl = Bl;
  a.K = K;
  a.vec = f32 ? (aligned16<float>(Ah, K) && aligned16<float>(Bh, K))
              : (aligned16<__bf16>(Ah, K) && aligned16<__bf16>(Bh, K) &&
                 (prec == 0 || (aligned16<__bf16>(Al, K) && aligned16<__bf16>(Bl, K))));
  const long long tiles = epi_tiles(S, Npts, Nout);
  if (tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)tiles);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define TDQ_NNJ_M(P_, S_, M_) hipLaunchKernelGGL((lay_nnj_kernel<P_, S_, M_>), grid, dim3(256), 0, st, a)
#define TDQ_NNJ(P_, S_)                                    \
  case S_:                                                 \
    if (kmode == EPI_FWD) TDQ_NNJ_M(P_, S_, EPI_FWD);      \
    else if (kmode == EPI_FWDJ) TDQ_NNJ_M(P_, S_, EPI_FWDJ); \
    else if (kmode == EPI_BWD) TDQ_NNJ_M(P_, S_, EPI_BWD); \
    else TDQ_NNJ_M(P_, S_, EPI_BWD0);                      \
    break;
#define TDQ_NNJ_P(P_)                                                                                         \
  switch (S) {                                                                                                \
    TDQ_NNJ(P_, 1) TDQ_NNJ(P_, 2) TDQ_NNJ(P_, 3) TDQ_NNJ(P_, 4) TDQ_NNJ(P_, 5) TDQ_NNJ(P_, 6) TDQ_NNJ(P_, 7) \
    TDQ_NNJ(P_, 8)                                                                                            \
    default: return (int)hipErrorInvalidValue;                                                                \
  }
  if (prec == 0) {
    TDQ_NNJ_P(0)
  } else if (prec == 1) {
    TDQ_NNJ_P(1)
  } else {
    TDQ_NNJ_P(2)
  }
#undef TDQ_NNJ_P
#undef TDQ_NNJ
#undef TDQ_NNJ_M
  TDQ_CHECK_LAUNCH();
  return 0;
}

// The input layer forward (lay_in_fwd_kernel): X [Npts][d_in] fp32, K0 [d_in][Nout], bias [Nout] ->
// the layer's post-activations as hi / lo bf16 planes [S * Npts][Nout] (f32: one fp32 plane Oh).
int tdq_lay_in_fwd(int f32, int S, const int* spec, const float* X, int d_in, const float* K0, const float* bias,
                   int Npts, int Nout, void* Oh, void* Ol, void* stream) {
  EpiArgs e;
  if (!epi_args(e, S, spec, Npts, Nout, d_in, f32 != 0, nullptr, nullptr, Oh, Ol) || d_in < 1 || X == nullptr ||
      K0 == nullptr || bias == nullptr || Oh == nullptr || (!f32 && Ol == nullptr))
    return (int)hipErrorInvalidValue;
  for (int s = 0; s < S; ++s)
    if (e.sp.stype[s] == 1 && e.sp.coord[s] >= d_in) return (int)hipErrorInvalidValue;
  e.bias = bias;
  const long long tiles = epi_tiles(S, Npts, Nout);
  if (tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)tiles);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (S) {
#define TDQ_INF(S_)                                                                                   \
  case S_:                                                                                            \
    if (f32) hipLaunchKernelGGL((lay_in_fwd_kernel<S_, true>), grid, dim3(256), 0, st, e, X, K0);   \
    else hipLaunchKernelGGL((lay_in_fwd_kernel<S_, false>), grid, dim3(256), 0, st, e, X, K0);      \
    break;
    TDQ_INF(1) TDQ_INF(2) TDQ_INF(3) TDQ_INF(4) TDQ_INF(5) TDQ_INF(6) TDQ_INF(7) TDQ_INF(8)
#undef TDQ_INF
    default: return (int)hipErrorInvalidValue;
  }
  TDQ_CHECK_LAUNCH();
  return 0;
}

// The last hidden layer's adjoint from the output layer (lay_out_bwd_kernel): dJ [S * Npts][d_out]
// fp32, Ko [Nout][d_out]; mode EPI_BWD / EPI_BWD0 with the outputs of tdq_lay_nnj (f32: fp32 planes).
int tdq_lay_out_bwd(int f32, int mode, int S, const int* spec, const float* dJ, int d_out, const float* Ko,
                    const void* Hh, const void* Hl, int Npts, int Nout, void* Oh, void* Ol, float* part, const float* X,
                    int d_in, void* stream) {
  EpiArgs e;
  if ((mode != EPI_BWD && mode != EPI_BWD0) ||
      !epi_args(e, S, spec, Npts, Nout, mode == EPI_BWD0 ? d_in : 0, f32 != 0, Hh, Hl, Oh, Ol) || d_out < 1 ||
      d_out > TDQ_MAXO || dJ == nullptr || Ko == nullptr || Hh == nullptr || (!f32 && Hl == nullptr) ||
      (mode == EPI_BWD ? Oh == nullptr : (part == nullptr || X == nullptr || d_in < 1)))
    return (int)hipErrorInvalidValue;
  e.part = part;
  e.X = X;
  const long long tiles = epi_tiles(S, Npts, Nout);
  if (tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)tiles);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define TDQ_OB_L(S_, M_, F_) \
  hipLaunchKernelGGL((lay_out_bwd_kernel<S_, M_, F_>), grid, dim3(256), 0, st, e, dJ, Ko, d_out)
#define TDQ_OB(S_)                                         \
  case S_:                                                 \
    if (mode == EPI_BWD) {                                 \
      if (f32) TDQ_OB_L(S_, EPI_BWD, true);                \
      else TDQ_OB_L(S_, EPI_BWD, false);                   \
    } else {                                               \
      if (f32) TDQ_OB_L(S_, EPI_BWD0, true);               \
      else TDQ_OB_L(S_, EPI_BWD0, false);                  \
    }                                                      \
    break;
  switch (S) {
    TDQ_OB(1) TDQ_OB(2) TDQ_OB(3) TDQ_OB(4) TDQ_OB(5) TDQ_OB(6) TDQ_OB(7) TDQ_OB(8)
    default: return (int)hipErrorInvalidValue;
  }
#undef TDQ_OB
#undef TDQ_OB_L
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
