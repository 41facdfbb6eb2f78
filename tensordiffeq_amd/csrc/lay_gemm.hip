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
// Measured on MI355X (AC [2,W x4,1], 50k points, Adam step, gpurun_out/r5lay): bf16x3 width 256
// 4.95 ms vs 5.82 ms on the library GEMMs (hipBLASLt); bf16 width 512 5.56 vs 4.81 ms.
// Reference: tensordiffeq/networks.py:10-20 (any layer list), the reference's tape GEMMs.
#include "jet_bf3.h"

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

// dK0 partial: C[z][j][f] = sum over rows n of chunk z of X[n][j] Z[n][f] (the input layer: d_in <=
// TDQ_MAXD columns of exact fp32 coordinates, no GEMM shape): 4 features per thread (16-byte Z
// loads), rows unrolled by 4 so several loads are in flight
__global__ void __launch_bounds__(256) lay_xtz_kernel(const float* __restrict__ X, int d_in,
                                                      const float* __restrict__ Z, int N, int W,
                                                      float* __restrict__ Cp, int rows_per_chunk) {
  const int f = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (f >= W) return;
  const int n_lo = blockIdx.y * rows_per_chunk, n_hi = min(N, n_lo + rows_per_chunk);
  const bool v4 = (W % 4 == 0);
  f32x4 a[TDQ_MAXD];
#pragma unroll
  for (int j = 0; j < TDQ_MAXD; ++j) a[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto zrow = [&](int n) {
    if (v4) return *reinterpret_cast<const f32x4*>(Z + (long long)n * W + f);
    f32x4 z;
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = f + e < W ? Z[(long long)n * W + f + e] : 0.f;
    return z;
  };
  int n = n_lo;
  for (; n + 3 < n_hi; n += 4) {
    f32x4 z[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) z[u] = zrow(n + u);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < TDQ_MAXD; ++j)
        if (j < d_in) a[j] += X[(long long)(n + u) * d_in + j] * z[u];
  }
  for (; n < n_hi; ++n) {
    const f32x4 z = zrow(n);
#pragma unroll
    for (int j = 0; j < TDQ_MAXD; ++j)
      if (j < d_in) a[j] += X[(long long)n * d_in + j] * z;
  }
  float* out = Cp + (long long)blockIdx.y * d_in * W;
  for (int j = 0; j < d_in; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (f + e < W) out[(long long)j * W + f + e] = a[j][e];
}

// ---- bf16 families: 128 x 128 workgroup tiles staged through LDS --------------------------------
// 4 waves in 2 x 2, each a 64 x 64 block (4 x 4 MFMA tiles): per 32-deep k-step a wave reads 4 A and
// 4 B fragments from LDS for 16 MFMAs (x3 in bf16x3).  LDS rows of 32 k-values padded to 40 (80 B):
// the 16 rows of a fragment read land on distinct banks.  Two buffers: the next k-step's global
// loads are in flight while the current one is multiplied.
constexpr int LS = 40;

// 8 bf16 of (row, k..k+7) of a row-major [nrows][ld] matrix, zero outside
__device__ __forceinline__ bf16x8 ldg8(const __bf16* __restrict__ base, long long ld, int row, int nrows, int k, int K,
                                       bool vec) {
  __bf16 v[8];
  ld8(base, ld, row, nrows, k, K, vec, v);
  return pack8(v);
}

template <int P>
__global__ void __launch_bounds__(256) lay_nn2_kernel(const __bf16* __restrict__ Ah, const __bf16* __restrict__ Al,
                                                      long long lda, const __bf16* __restrict__ Bh,
                                                      const __bf16* __restrict__ Bl, long long ldb,
                                                      float* __restrict__ C, long long ldc, int M, int N, int K,
                                                      int vec) {
  constexpr int NB = P == 1 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 sA[2][NB][128 * LS];
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][NB][128 * LS];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, p = l & 15, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * 128, n0 = blockIdx.x * 128;
  const bool v = vec != 0;
  // staging: chunks t and t + 256 of the 512 8-element chunks of a 128 x 32 tile
  const int sr0 = tid >> 2, sk = (tid & 3) * 8, sr1 = sr0 + 64;
  bf16x8 ra[2][NB], rb[2][NB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const __bf16* A = b ? Al : Ah;
      const __bf16* B = b ? Bl : Bh;
      ra[0][b] = ldg8(A, lda, m0 + sr0, M, k0 + sk, K, v);
      ra[1][b] = ldg8(A, lda, m0 + sr1, M, k0 + sk, K, v);
      rb[0][b] = ldg8(B, ldb, n0 + sr0, N, k0 + sk, K, v);
      rb[1][b] = ldg8(B, ldb, n0 + sr1, N, k0 + sk, K, v);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      *reinterpret_cast<bf16x8*>(&sA[buf][b][sr0 * LS + sk]) = ra[0][b];
      *reinterpret_cast<bf16x8*>(&sA[buf][b][sr1 * LS + sk]) = ra[1][b];
      *reinterpret_cast<bf16x8*>(&sB[buf][b][sr0 * LS + sk]) = rb[0][b];
      *reinterpret_cast<bf16x8*>(&sB[buf][b][sr1 * LS + sk]) = rb[1][b];
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  gload(0);
  sstore(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += 32) {
    const bool more = k0 + 32 < K;
    if (more) gload(k0 + 32);
    bf16x8 a[4][NB], b[4][NB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        a[i][q] = *reinterpret_cast<const bf16x8*>(&sA[buf][q][(wm * 64 + 16 * i + p) * LS + 8 * g]);
        b[i][q] = *reinterpret_cast<const bf16x8*>(&sB[buf][q][(wn * 64 + 16 * i + p) * LS + 8 * g]);
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
    if (more) {
      sstore(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
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
  __shared__ __attribute__((aligned(16))) __bf16 sA[NB][32 * TS];
  __shared__ __attribute__((aligned(16))) __bf16 sB[NB][32 * TS];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int i0 = blockIdx.y * 128, j0 = blockIdx.x * 128;
  const int r_lo = blockIdx.z * rows_per_chunk, r_hi = min(L, r_lo + rows_per_chunk);
  const bool v = vec != 0;
  // staging: chunks t, t + 256 of the 512 8-feature chunks of a 32-row x 128-feature tile
  const int rr0 = tid >> 4, rr1 = rr0 + 16, fc = (tid & 15) * 8;
  // transposed-read address of this lane: row 8g + q, column 4p (+ the tile's first column)
  const int trq = (l & 15) >> 2, trp = l & 3;
  const int ta = (8 * g + trq) * TS + 4 * trp, tb = ta + 4 * TS;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int r0 = r_lo; r0 < r_hi; r0 += 32) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const bf16x8 a0 = ldg8(q ? Al : Ah, lda, r0 + rr0, r_hi, i0 + fc, Ma, v);
      const bf16x8 a1 = ldg8(q ? Al : Ah, lda, r0 + rr1, r_hi, i0 + fc, Ma, v);
      const bf16x8 b0 = ldg8(q ? Bl : Bh, ldb, r0 + rr0, r_hi, j0 + fc, Nb, v);
      const bf16x8 b1 = ldg8(q ? Bl : Bh, ldb, r0 + rr1, r_hi, j0 + fc, Nb, v);
      *reinterpret_cast<bf16x8*>(&sA[q][rr0 * TS + fc]) = a0;
      *reinterpret_cast<bf16x8*>(&sA[q][rr1 * TS + fc]) = a1;
      *reinterpret_cast<bf16x8*>(&sB[q][rr0 * TS + fc]) = b0;
      *reinterpret_cast<bf16x8*>(&sB[q][rr1 * TS + fc]) = b1;
    }
    __syncthreads();
    bf16x8 a[4][NB], b[4][NB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int ca = wm * 64 + 16 * i, cb = wn * 64 + 16 * i;
        a[i][q] = cat8(tr_read(&sA[q][ta + ca]), tr_read(&sA[q][tb + ca]));
        b[i][q] = cat8(tr_read(&sB[q][ta + cb]), tr_read(&sB[q][tb + cb]));
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
    __syncthreads();
  }
  const int p = l & 15;
  float* out = Cp + (long long)blockIdx.z * Ma * Nb;
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
    dim3 g2((N + 127) / 128, (M + 127) / 128);
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
    dim3 g2((Nb + 127) / 128, (Ma + 127) / 128, nch);
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

// Cp: nchunks x d_in x W partials of X^T Z (X [N][d_in], Z [N][W], fp32); the caller sums dim 0
int tdq_lay_xtz(const float* X, int d_in, const float* Z, int N, int W, float* Cp, int rows_per_chunk, void* stream) {
  if (N <= 0 || W <= 0 || d_in < 1 || d_in > TDQ_MAXD || rows_per_chunk <= 0) return (int)hipErrorInvalidValue;
  const int nch = (N + rows_per_chunk - 1) / rows_per_chunk;
  hipLaunchKernelGGL(lay_xtz_kernel, dim3((W + 1023) / 1024, nch), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     X, d_in, Z, N, W, Cp, rows_per_chunk);
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
