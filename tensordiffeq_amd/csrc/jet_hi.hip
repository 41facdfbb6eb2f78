// High-order Taylor jets (any multi-index up to order 4) of a tanh MLP on SMALL point sets: fp32
// elementwise work, split-bf16 (bf16x3) MFMA layer GEMMs, fp32 MFMA weight gradients.
//
// Why a separate kernel: the fused jet kernels (jet_bf3.h) carry value, first- and second-order
// streams only, with the post-activation identities of the order-2 tanh jet.  The reference's
// AC-baseline / AC-dist-new periodic BCs (examples/AC-baseline.py:23-29, AC-dist-new.py:23-29)
// also ask for u_xxx and u_xxxx - on the 2 x 201 boundary points only.  Those points stay in the
// main point set (the fused kernels compute their order <= 2 streams with everything else); this
// kernel pair computes the EXTRA streams (order 3 / 4) for them and the parameter gradient of the
// adjoints of those extra streams, so the step keeps the fused loss, the fused tail and the K-step
// graphs ("Taylor-jet order <= 4 along one axis").
//
// Math (jet.py is the torch reference): every stream s = multi-index mi of input variables;
// linear layers map every stream with the same weights (bias on the value stream only); tanh maps
//   h_mi = sum over set partitions P of mi:  tanh^(|P|)(z) * prod_{B in P} z_B     (Faa di Bruno)
// with tanh^(k) = s1 * q_k(h), s1 = 1 - h^2 (computed as 4e / (1 + e)^2, e = exp(-2|z|)):
//   q1 = 1, q2 = -2h, q3 = 6h^2 - 2, q4 = h (16 - 24h^2), q5 = 16 - 120h^2 + 120h^4.
// The host passes the partition table (term = tanh order k, coefficient, up to 4 factor streams);
// the backward differentiates each term by product rule, and through tanh^(k)(z) with
// d/dz tanh^(k) = tanh^(k+1).  The forward saves every hidden layer's PRE-activation streams z
// and post-activation streams h (fp32, [layer][point x stream][feature]); order >= 3 adjoints need
// z itself, the weight gradients need h.
//
// Kernels (a few hundred points: latency, not bandwidth, is the budget):
//   * forward: workgroup = 512 threads = 4 points, thread (f, g) owns feature f of point g; one
//     layer's weights and the points' activations in LDS, the layer GEMM on bf16x3 MFMA tiles
//     (hi_mma: rows point x stream, wave w = 16 output columns); the next layer's weights load
//     into registers during this layer's GEMM (zero padding applied at the LDS store, so nothing
//     waits for them before it).
//   * adjoint chain (same layout): zb_i = tanh-jet adjoint of hb_i, hb_{i-1} = W_i zb_i -> B.
//   * weight gradients: dK_i = H_{i-1}^T B_i as 32 x 32 tiles over point splits (one slab row per
//     split); the vector parameters (biases, K0, Ko, bo) summed per workgroup by the chain itself
//     (one vslab row per workgroup); a fixed-order sum of the rows gives the gradient
//     (deterministic), which the fused step tail adds to theta's.
// Loads are unconditional from clamped addresses (a conditional load is a branch with a wait
// behind it).  The stream count is a template parameter, and the common plan - the
// univariate chain u, u_v, u_vv, u_vvv(, u_vvvv) of the reference's periodic BCs - has its tanh jet
// and adjoint as straight-line code; other plans interpret the partition table.
// History (AC-baseline, 402 points, order 4; profiles/): interpreted 256-thread first build
// 0.31 + 0.40 ms per step; this layout 26 + 57 us isolated (profiles/r4g_kernel_stats_hi_isolated.txt);
// MFMA layer GEMMs: chain -16 %, forward -7 % of workgroup cycles (profiles/r4x_hi_phase_stamps_mfma.txt);
// A rows split once at the store instead of per wave: forward 35.0 -> 30.4k, chain 38.8 -> 33.2k cycles,
// bit-identical (profiles/r4asplit_*; the AC-baseline step does not move: 0.221-0.224 vs 0.220-0.222 ms).
#include "jet_common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define HI_MAXS 8
#define HI_MAXT 48
#define HI_MAXB 4
#define HI_W 128
#define HI_TG 4                      // 128-thread groups per workgroup (one feature per thread)
#define HI_PT 1                      // points per thread
#define HI_NP (HI_TG * HI_PT)        // points per workgroup
#define HI_THREADS (HI_W * HI_TG)
#define HI_WS (HI_W + 4)             // LDS row strides (float4 rows, conflict-free)
#define HI_AS (HI_W + 4)
#define HI_KS 8                      // point splits of the weight-gradient pass (slab rows)

struct HiSpec {
  int S;
  int order[HI_MAXS];
  int var[HI_MAXS];    // order-1 streams: input variable
  int out[HI_MAXS];    // J / dJ row of the stream (-1: neither written nor seeded)
  int t0[HI_MAXS], nt[HI_MAXS];
  int tk[HI_MAXT];     // tanh derivative order of the term
  float tc[HI_MAXT];   // coefficient
  int tnb[HI_MAXT];    // factor count
  int tb[HI_MAXT][HI_MAXB];  // factor streams
  int chain;           // 1: streams are the univariate chain (), (v), (v,v), ... of one variable
};

// tanh and its derivatives 1..5 at z: sg[0] = h, sg[k] = tanh^(k)(z)
__device__ __forceinline__ void hi_sigmas(float z, float (&sg)[6]) {
  const float az = fabsf(z);
  const float e = __expf(-2.f * az);
  const float r = 1.f / (1.f + e);
  const float z2 = az * az;
  const float poly = az * fmaf(z2, fmaf(z2, fmaf(z2, -0.053968254f, 0.13333334f), -0.33333334f), 1.f);
  const float t = az < 0.125f ? poly : (1.f - e) * r;
  const float h = copysignf(t, z);
  const float s1 = 4.f * e * (r * r);
  const float h2 = h * h;
  sg[0] = h;
  sg[1] = s1;
  sg[2] = -2.f * h * s1;
  sg[3] = s1 * fmaf(6.f, h2, -2.f);
  sg[4] = s1 * h * fmaf(-24.f, h2, 16.f);
  sg[5] = s1 * fmaf(h2, fmaf(120.f, h2, -120.f), 16.f);
}

// univariate chain z_k = d^k z / dv^k (k < S): Faa di Bruno written out, order <= 4
template <int S>
__device__ __forceinline__ void chain_f(const float (&z)[S], float (&h)[S]) {
  float sg[6];
  hi_sigmas(z[0], sg);
  h[0] = sg[0];
  if constexpr (S > 1) h[1] = sg[1] * z[1];
  if constexpr (S > 2) h[2] = fmaf(sg[1], z[2], sg[2] * z[1] * z[1]);
  if constexpr (S > 3) h[3] = sg[1] * z[3] + 3.f * sg[2] * z[1] * z[2] + sg[3] * z[1] * z[1] * z[1];
  if constexpr (S > 4)
    h[4] = sg[1] * z[4] + sg[2] * (4.f * z[1] * z[3] + 3.f * z[2] * z[2]) + 6.f * sg[3] * z[1] * z[1] * z[2] +
           sg[4] * z[1] * z[1] * z[1] * z[1];
}
template <int S>
__device__ __forceinline__ void chain_b(const float (&z)[S], const float (&hb)[S], float (&zb)[S]) {
  float sg[6];
  hi_sigmas(z[0], sg);
  zb[0] = sg[1] * hb[0];
  if constexpr (S > 1) {
    zb[0] += sg[2] * z[1] * hb[1];
    zb[1] = sg[1] * hb[1];
  }
  if constexpr (S > 2) {
    zb[0] += (sg[2] * z[2] + sg[3] * z[1] * z[1]) * hb[2];
    zb[1] += 2.f * sg[2] * z[1] * hb[2];
    zb[2] = sg[1] * hb[2];
  }
  if constexpr (S > 3) {
    zb[0] += (sg[2] * z[3] + 3.f * sg[3] * z[1] * z[2] + sg[4] * z[1] * z[1] * z[1]) * hb[3];
    zb[1] += (3.f * sg[2] * z[2] + 3.f * sg[3] * z[1] * z[1]) * hb[3];
    zb[2] += 3.f * sg[2] * z[1] * hb[3];
    zb[3] = sg[1] * hb[3];
  }
  if constexpr (S > 4) {
    zb[0] += (sg[2] * z[4] + sg[3] * (4.f * z[1] * z[3] + 3.f * z[2] * z[2]) + 6.f * sg[4] * z[1] * z[1] * z[2] +
              sg[5] * z[1] * z[1] * z[1] * z[1]) * hb[4];
    zb[1] += (4.f * sg[2] * z[3] + 12.f * sg[3] * z[1] * z[2] + 4.f * sg[4] * z[1] * z[1] * z[1]) * hb[4];
    zb[2] += (6.f * sg[2] * z[2] + 6.f * sg[3] * z[1] * z[1]) * hb[4];
    zb[3] += 4.f * sg[2] * z[1] * hb[4];
    zb[4] = sg[1] * hb[4];
  }
}

// generic plans: the partition table, read with wave-uniform indices from the kernel arguments
template <int S>
__device__ __forceinline__ float zsel(const float (&z)[S], int idx) {
  float r = z[0];
#pragma unroll
  for (int q = 1; q < S; ++q) r = idx == q ? z[q] : r;
  return r;
}
template <int S>
__device__ __forceinline__ void table_f(const HiSpec& sp, const float (&z)[S], float (&h)[S]) {
  float sg[6];
  hi_sigmas(z[0], sg);
  h[0] = sg[0];
#pragma unroll
  for (int s = 1; s < S; ++s) {
    float a = 0.f;
    for (int t = sp.t0[s]; t < sp.t0[s] + sp.nt[s]; ++t) {
      const int k = sp.tk[t];
      float v = sp.tc[t] * (k == 1 ? sg[1] : k == 2 ? sg[2] : k == 3 ? sg[3] : sg[4]);
      for (int b = 0; b < sp.tnb[t]; ++b) v *= zsel(z, sp.tb[t][b]);
      a += v;
    }
    h[s] = a;
  }
}
template <int S>
__device__ __forceinline__ void table_b(const HiSpec& sp, const float (&z)[S], const float (&hb)[S], float (&zb)[S]) {
  float sg[6];
  hi_sigmas(z[0], sg);
#pragma unroll
  for (int s = 0; s < S; ++s) zb[s] = 0.f;
  zb[0] = hb[0] * sg[1];
#pragma unroll
  for (int s = 1; s < S; ++s) {
    const float g = hb[s];
    for (int t = sp.t0[s]; t < sp.t0[s] + sp.nt[s]; ++t) {
      const int k = sp.tk[t], nb = sp.tnb[t];
      const float base = sp.tc[t] * g;
      float fac[HI_MAXB];
      int ib[HI_MAXB];
      float prod = 1.f;
#pragma unroll
      for (int b = 0; b < HI_MAXB; ++b) {
        ib[b] = b < nb ? sp.tb[t][b] : 0;
        fac[b] = b < nb ? zsel(z, ib[b]) : 1.f;
        prod *= fac[b];
      }
      const float sk = k == 1 ? sg[1] : k == 2 ? sg[2] : k == 3 ? sg[3] : sg[4];
      const float sk1 = k == 1 ? sg[2] : k == 2 ? sg[3] : k == 3 ? sg[4] : sg[5];
      zb[0] += base * sk1 * prod;  // d tanh^(k)(z0) / dz0 = tanh^(k+1)
#pragma unroll
      for (int b = 0; b < HI_MAXB; ++b) {
        if (b >= nb) continue;
        float others = 1.f;
#pragma unroll
        for (int c = 0; c < HI_MAXB; ++c)
          if (c != b) others *= fac[c];
        const float v = base * sk * others;
#pragma unroll
        for (int q = 0; q < S; ++q) zb[q] += ib[b] == q ? v : 0.f;
      }
    }
  }
}

template <int S, bool CH>
__device__ __forceinline__ void hi_tanh_f(const HiSpec& sp, const float (&z)[S], float (&h)[S]) {
  if constexpr (CH)
    chain_f<S>(z, h);
  else
    table_f<S>(sp, z, h);
}
template <int S, bool CH>
__device__ __forceinline__ void hi_tanh_b(const HiSpec& sp, const float (&z)[S], const float (&hb)[S], float (&zb)[S]) {
  if constexpr (CH)
    chain_b<S>(z, hb, zb);
  else
    table_b<S>(sp, z, hb, zb);
}

// LDS of the forward / adjoint-chain kernels (floats, dynamic, sized per launch):
//   W [HI_W][HI_WS]          one layer's weights (row stride 132: the 8-float MFMA fragment rows
//                            of 16 lanes land on distinct banks)
//   A 2 x [HI_NP][S][HI_AB]  the workgroup's activations / adjoints as MFMA A rows, split once into
//                            bf16 hi and lo at the store (every wave reads the same rows)
//   R [HI_MR][HI_AS]         GEMM product (rows point * S + stream; both 16-row MFMA tiles)
//   V [HI_TG][nvs][HI_W]     (chain) vector-parameter partials (nvs slots, hi_nvs)
constexpr int HI_MR = 32;  // GEMM rows: HI_NP points x at most HI_MAXS streams
// bf16 row stride of the split A rows: 272 B = 68 words, so the 16 rows of a ds_read_b128 pass
// (one 8-element column group) start 4 banks apart - conflict-free
constexpr int HI_AB = 136;
static_assert(HI_NP * HI_MAXS <= HI_MR, "two 16-row MFMA tiles cover the workgroup's rows");
struct HiLds {
  float* W;
  float* A;
  float* R;
  float* V;
  int S;
  __device__ float& w(int k, int f) const { return W[k * HI_WS + f]; }
  __device__ __bf16* ah() const { return reinterpret_cast<__bf16*>(A); }
  __device__ __bf16* al() const { return reinterpret_cast<__bf16*>(A) + HI_NP * S * HI_AB; }
};
__host__ __device__ inline size_t hi_lds_floats(int S, int nvs) {
  return (size_t)HI_W * HI_WS + (size_t)HI_NP * S * HI_AB + (size_t)HI_MR * HI_AS + (size_t)HI_TG * nvs * HI_W;
}
__device__ inline HiLds hi_lds_map(float* base, int S) {
  HiLds L;
  L.S = S;
  L.W = base;
  L.A = L.W + HI_W * HI_WS;
  L.R = L.A + HI_NP * S * HI_AB;  // (two bf16 arrays = HI_AB floats per row)
  L.V = L.R + HI_MR * HI_AS;
  return L;
}

// Diagnostic build only (tools/hi_stamps.cpp, -DHI_STAMPS): s_memtime at phase boundaries of
// workgroup 0, printed at the end; compiled out otherwise.
#ifdef HI_STAMPS
#define HI_TS_DECL long long hi_ts[24]; int hi_nts = 0;
#define HI_TS() \
  if (hi_nts < 24) hi_ts[hi_nts++] = __builtin_amdgcn_s_memtime();
#define HI_TS_PRINT(name)                                                       \
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {                 \
    printf("%s", name);                                                         \
    for (int q = 1; q < hi_nts; ++q) printf(" %lld", hi_ts[q] - hi_ts[q - 1]); \
    printf(" | total %lld\n", hi_ts[hi_nts - 1] - hi_ts[0]);                   \
  }
#else
#define HI_TS_DECL
#define HI_TS()
#define HI_TS_PRINT(name)
#endif

// Loads in these kernels are unconditional, from clamped (valid) addresses, and masked after the
// fact: a `cond ? load : 0` compiles to a branch around the load with a wait behind it, which
// serialises a whole batch of loads into one memory latency each.
__device__ __forceinline__ float ldm(const float* p, bool keep) {
  const float v = *p;
  return keep ? v : 0.f;
}

// W (in x out) of dense layer `layer`, zero-padded to HI_W x HI_W, as float4 pieces in registers:
// piece u of thread t = row (t + HI_THREADS u) >> 5, columns 4 ((t + HI_THREADS u) & 31) + [0, 4).  All loads of a
// layer are issued back to back (one memory latency per layer, not one per element) and overlap
// the previous layer's GEMM; hi_put_w writes them to LDS after that GEMM's barrier.
constexpr int HI_WQ = HI_W * HI_W / 4 / HI_THREADS;
struct HiWRegs {
  f32x4 q[HI_WQ];
};
__device__ __forceinline__ void hi_get_w(HiWRegs& r, const float* __restrict__ P, const NetDims& d, int layer) {
  const float* K = P + off_layer(d, layer);
  const int win = hw(d, layer - 1), wout = hw(d, layer);
  // one uniform branch around each whole batch (a branch per piece makes the compiler wait for
  // every load at the join); clamped addresses, the zero padding is hi_put_w's (a select here would
  // wait for the loads before the GEMM they are meant to overlap)
  if (((off_layer(d, layer) | wout) & 3) == 0) {
#pragma unroll
    for (int u = 0; u < HI_WQ; ++u) {
      const int e = threadIdx.x + HI_THREADS * u, k = e >> 5, c = (e & 31) * 4;
      const int kc = k < win ? k : win - 1, cc = c < wout ? c : wout - 4;
      r.q[u] = *reinterpret_cast<const f32x4*>(K + kc * wout + cc);
    }
  } else {
#pragma unroll
    for (int u = 0; u < HI_WQ; ++u) {
      const int e = threadIdx.x + HI_THREADS * u, k = e >> 5, c = (e & 31) * 4;
      const int kc = k < win ? k : win - 1;
#pragma unroll
      for (int x = 0; x < 4; ++x) r.q[u][x] = K[kc * wout + (c + x < wout ? c + x : wout - 1)];
    }
  }
}
__device__ __forceinline__ void hi_put_w(const HiLds& L, const HiWRegs& r, const NetDims& d, int layer) {
  const int win = hw(d, layer - 1), wout = hw(d, layer);
#pragma unroll
  for (int u = 0; u < HI_WQ; ++u) {
    const int e = threadIdx.x + HI_THREADS * u, k = e >> 5, c = (e & 31) * 4;
    f32x4 v;
#pragma unroll
    for (int x = 0; x < 4; ++x) v[x] = (k < win && c + x < wout) ? r.q[u][x] : 0.f;
    *reinterpret_cast<f32x4*>(&L.w(k, c)) = v;
  }
}

// activation-sized scratch: [layer][n * S + s][HI_W] (Z: pre-activations, H: post-activations,
// B: adjoints of the pre-activations)
__device__ __forceinline__ size_t hi_row(int layer, int n, int s, int S, int N) {
  return (((size_t)layer * N + n) * S + s) * HI_W;
}

// Layer GEMMs on bf16x3 MFMA (v_mfma_f32_16x16x32_bf16; fp32 operands split into bf16 hi + lo,
// products hi*hi + hi*lo + lo*hi, fp32 accumulation - the split-bf16 family of the fused kernels,
// ~1e-5 relative).  Rows m = point * S + stream (at most 32: two 16-row tiles, rows >= 4 S zero);
// wave w owns the 16 output columns [16 w, 16 w + 16).  Lane l: A[row l & 15][k = 8 (l >> 4) + j],
// B[k][col l & 15], C[4 (l >> 4) + r][l & 15].  The product lands in R as [m][HI_AS].
typedef __bf16 hbf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void hi_split(const float (&x)[8], hbf16x8& h, hbf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 hx = (__bf16)x[j];
    h[j] = hx;
    lo[j] = (__bf16)(x[j] - (float)hx);
  }
}
__device__ __forceinline__ f32x4 hi_mma3(const hbf16x8& ah, const hbf16x8& al, const hbf16x8& bh, const hbf16x8& bl,
                                         f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
}
// element (m, k) of the A rows, split into bf16 hi + lo (hi_split's rounding)
__device__ __forceinline__ void hi_put_a(const HiLds& L, int m, int k, float x) {
  const __bf16 hx = (__bf16)x;
  L.ah()[m * HI_AB + k] = hx;
  L.al()[m * HI_AB + k] = (__bf16)(x - (float)hx);
}
// A fragment (row m, columns k0 .. k0 + 7) of the workgroup, hi and lo; rows past 4 S read as zero
__device__ __forceinline__ void hi_arow(const HiLds& L, int m, int k0, int S, hbf16x8& h, hbf16x8& lo) {
  const bool in = m < HI_NP * S;
  const int o = (in ? m : 0) * HI_AB + k0;
  const hbf16x8 u = *reinterpret_cast<const hbf16x8*>(L.ah() + o), v = *reinterpret_cast<const hbf16x8*>(L.al() + o);
  const hbf16x8 z = {};
  h = in ? u : z;
  lo = in ? v : z;
}
// TRANS = false (forward): out[m][c] = sum_k A[m][k] W[k][c]; true (adjoint chain): out[m][c] =
// sum_o A[m][o] W[c][o]
template <bool TRANS>
__device__ __forceinline__ void hi_mma(const HiLds& L, int S, int kin) {
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63, p = l & 15, g = l >> 4, col = 16 * wv + p;
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
  const int nk = (kin + 31) >> 5;
  for (int kk = 0; kk < nk; ++kk) {
    const int k0 = 32 * kk + 8 * g;
    float w[8];
    hbf16x8 a0h, a0l, a1h, a1l, wh, wl;
    hi_arow(L, p, k0, S, a0h, a0l);
    hi_arow(L, 16 + p, k0, S, a1h, a1l);
    if constexpr (TRANS) {
      const float* r = &L.w(col, k0);
      const f32x4 u = *reinterpret_cast<const f32x4*>(r), v = *reinterpret_cast<const f32x4*>(r + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w[j] = u[j];
        w[4 + j] = v[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = L.w(k0 + j, col);
    }
    hi_split(w, wh, wl);
    c0 = hi_mma3(a0h, a0l, wh, wl, c0);
    c1 = hi_mma3(a1h, a1l, wh, wl, c1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    L.R[(4 * g + r) * HI_AS + col] = c0[r];
    L.R[(16 + 4 * g + r) * HI_AS + col] = c1[r];
  }
}

// thread t: point p = t >> 7 and feature f = t & 127 in the elementwise phases; in the GEMM, feature
// quad f4 = (t >> 2) & 31 and k-quarter ks = t & 3 (so f = 4 f4 + ks)
template <int S, bool CH>
__global__ void __launch_bounds__(HI_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) jet_hi_fwd_kernel(const float* __restrict__ X, int N,
                                                                const float* __restrict__ P, NetDims d, HiSpec sp,
                                                                float* __restrict__ J, int ldJ, int j0,
                                                                float* __restrict__ Zb, float* __restrict__ Hb) {
  extern __shared__ __attribute__((aligned(16))) float hi_lds[];
  const HiLds L = hi_lds_map(hi_lds, S);
  HI_TS_DECL
  HI_TS()
  const int t = threadIdx.x, f = t & (HI_W - 1), pg = t >> 7;
  const int Lh = d.n_hidden;
  const int m0 = blockIdx.x * HI_NP + pg;
  const bool ok = m0 < N;
  const int n = ok ? m0 : N - 1;
  HiWRegs wr;
  if (Lh > 1) hi_get_w(wr, P, d, 1);
  float z[S], hl[S];  // hl: the last hidden layer's h (output layer products)
  {  // layer 0: z = x K0 + b0 (value), K0[var] (first order), 0 (higher)
    const int w0 = hw(d, 0);
    const int fc = f < w0 ? f : w0 - 1;
    float xv[TDQ_MAXD], kv[TDQ_MAXD];
#pragma unroll
    for (int v = 0; v < TDQ_MAXD; ++v) {
      const int vc = v < d.d_in ? v : d.d_in - 1;
      kv[v] = P[vc * w0 + fc];
      xv[v] = X[(size_t)n * d.d_in + vc];
    }
    float a = P[d.d_in * w0 + fc];
    __builtin_amdgcn_sched_barrier(0);  // all loads in flight first
#pragma unroll
    for (int v = 0; v < TDQ_MAXD; ++v) {
      kv[v] = (v < d.d_in && f < w0) ? kv[v] : 0.f;
      xv[v] = v < d.d_in ? xv[v] : 0.f;
    }
    a = f < w0 ? a : 0.f;
#pragma unroll
    for (int v = 0; v < TDQ_MAXD; ++v) a = fmaf(xv[v], kv[v], a);
    z[0] = a;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      float k1 = 0.f;
#pragma unroll
      for (int v = 0; v < TDQ_MAXD; ++v) k1 = sp.var[s] == v ? kv[v] : k1;
      z[s] = sp.order[s] == 1 ? k1 : 0.f;
    }
  }
  if (Lh > 1) hi_put_w(L, wr, d, 1);
  HI_TS()
  for (int i = 0; i < Lh; ++i) {
    const int wi = hw(d, i);
    if (i >= 1) {  // z_i = h_{i-1} W_i (+ b_i); W_{i+1} loads in flight meanwhile
      if (i + 1 < Lh) hi_get_w(wr, P, d, i + 1);
      float b = P[off_layer(d, i) + hw(d, i - 1) * wi + (f < wi ? f : wi - 1)];  // masked after the GEMM
      hi_mma<false>(L, S, hw(d, i - 1));
      HI_TS()
      __syncthreads();  // z in R; every GEMM read of A / W done
      b = f < wi ? b : 0.f;
#pragma unroll
      for (int s = 0; s < S; ++s) z[s] = L.R[(pg * S + s) * HI_AS + f] + (s == 0 ? b : 0.f);
      if (i + 1 < Lh) hi_put_w(L, wr, d, i + 1);
      HI_TS()
    }
    {
      float h[S];
      if (f < wi) {
        hi_tanh_f<S, CH>(sp, z, h);
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) h[s] = 0.f;
      }
      if (ok) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          Zb[hi_row(i, n, s, S, N) + f] = z[s];
          Hb[hi_row(i, n, s, S, N) + f] = h[s];
        }
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        hi_put_a(L, pg * S + s, f, h[s]);
        hl[s] = h[s];
      }
    }
    HI_TS()
    __syncthreads();  // A (and W) of the next GEMM written; R read
    HI_TS()
  }
  // ---- output layer: u_s[q] = sum_f h_s[f] Ko[f][q] (+ bo[q] on the value stream): per-feature
  // products into LDS (the free weight area), then one thread per (point, stream, q) sums them
  const int wl = hw(d, Lh - 1), dout = d.d_out;
  const float* Ko = P + off_layer(d, Lh);
  float* part = L.W;  // [p][s][q][HI_W]
  {
    float ko[TDQ_MAXO];
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q)
      ko[q] = ldm(Ko + (f < wl ? f : wl - 1) * dout + (q < dout ? q : dout - 1), q < dout && f < wl);
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int q = 0; q < TDQ_MAXO; ++q)
        if (q < dout) part[((pg * S + s) * TDQ_MAXO + q) * HI_W + f] = hl[s] * ko[q];
  }
  __syncthreads();
  for (int c = t; c < HI_NP * S * dout; c += blockDim.x) {
    const int q = c % dout, s = (c / dout) % S, pp = c / (dout * S);
    const int m = blockIdx.x * HI_NP + pp;
    if (m >= N || sp.out[s] < 0) continue;
    const f32x4* r = reinterpret_cast<const f32x4*>(part + ((pp * S + s) * TDQ_MAXO + q) * HI_W);
    f32x4 a4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int k = 0; k < HI_W / 4; ++k) a4 += r[k];
    float a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    if (s == 0) a += Ko[wl * dout + q];
    J[((size_t)sp.out[s] * ldJ + j0 + m) * dout + q] = a;
  }
  HI_TS()
  HI_TS_PRINT("fwd")
}

// Per-workgroup partials of the vector parameters (hidden biases, K0, Ko, bo), written by the
// adjoint chain (one row per workgroup, compact layout below) and summed by jet_hi_reduce_kernel:
//   [i * HI_W + f]                       bias of hidden layer i
//   [(Lh + v) * HI_W + f]                K0[v][f]
//   [(Lh + d_in) * HI_W + f * MAXO + q]   Ko[f][q]
//   [(Lh + d_in) * HI_W + HI_W * MAXO + q] bo[q]
__host__ __device__ inline int hi_vrow(const NetDims& d) {
  return (((d.n_hidden + d.d_in) * HI_W + HI_W * TDQ_MAXO + TDQ_MAXO) + 3) & ~3;
}
// V slots: 0 bias; 1 .. d_in K0 (layer 0); from hi_vko: d_out Ko then d_out bo (last layer) - with
// two or more hidden layers the first and the last layer share slots 1.. (never both live)
__host__ __device__ inline int hi_vko(const NetDims& d) { return d.n_hidden == 1 ? 1 + d.d_in : 1; }
__host__ __device__ inline int hi_nvs(const NetDims& d) {
  return d.n_hidden == 1 ? 1 + d.d_in + 2 * d.d_out : 1 + (d.d_in > 2 * d.d_out ? d.d_in : 2 * d.d_out);
}

// fixed-order sum over the point groups of layer i's vector partials (slots: hi_nvs) -> the
// workgroup's vslab row; thread (f, group g) takes slots g, g + HI_TG, ...
__device__ __forceinline__ void hi_vsum(const HiLds& L, float* __restrict__ vrow, const NetDims& d, int i, int g,
                                        int f) {
  const int Lh = d.n_hidden, din = d.d_in, dout = d.d_out, nvs = hi_nvs(d), vko = hi_vko(d);
  for (int sl = g; sl < nvs; sl += HI_TG) {
    const bool k0 = i == 0 && sl >= 1 && sl <= din;
    const bool ko = i == Lh - 1 && sl >= vko && sl < vko + dout;
    const bool bo = i == Lh - 1 && sl >= vko + dout && sl < vko + 2 * dout;
    if (!(sl == 0 || k0 || ko || (bo && f == 0))) continue;
    float a = L.V[sl * HI_W + f];
#pragma unroll
    for (int gg = 1; gg < HI_TG; ++gg) a += L.V[(gg * nvs + sl) * HI_W + f];
    if (sl == 0)
      vrow[i * HI_W + f] = a;
    else if (k0)
      vrow[(Lh + sl - 1) * HI_W + f] = a;
    else if (ko)
      vrow[(Lh + din) * HI_W + f * TDQ_MAXO + (sl - vko)] = a;
    else
      vrow[(Lh + din) * HI_W + HI_W * TDQ_MAXO + (sl - vko - dout)] = a;
  }
}

// adjoint chain: hb of the last hidden layer from dJ, then zb_i = tanh-jet adjoint, hb_{i-1} = W_i zb_i;
// zb_i -> Bb (the hidden-to-hidden kernels' gradients are jet_hi_wgrad_kernel's); the vector
// parameters' gradients are summed over the workgroup's points here -> vslab row blockIdx.x.
// Thread t: point p = t >> 7, feature f = t & 127; the GEMM is hi_mma's (wave w: columns 16 w ..).
template <int S, bool CH>
__global__ void __launch_bounds__(HI_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) jet_hi_chain_kernel(int N, const float* __restrict__ P, NetDims d,
                                                                  HiSpec sp, const float* __restrict__ X,
                                                                  const float* __restrict__ dJ, int ldJ,
                                                                  int j0, const float* __restrict__ Zb,
                                                                  float* __restrict__ Bb, float* __restrict__ vslab) {
  extern __shared__ __attribute__((aligned(16))) float hi_lds[];
  const HiLds L = hi_lds_map(hi_lds, S);
  HI_TS_DECL
  HI_TS()
  const int t = threadIdx.x, pg = t >> 7, f = t & (HI_W - 1);
  const int Lh = d.n_hidden, dout = d.d_out, din = d.d_in, nvs = hi_nvs(d);
  const int m0 = blockIdx.x * HI_NP + pg;
  const bool ok = m0 < N;
  const int n = ok ? m0 : N - 1;
  HiWRegs wr;
  if (Lh > 1) hi_get_w(wr, P, d, Lh - 1);
  const int wl = hw(d, Lh - 1);
  const float* Ko = P + off_layer(d, Lh);
  float* vrow = vslab + (size_t)blockIdx.x * hi_vrow(d);
  float hb[S], z[S];
  float vo[TDQ_MAXO], vbo[TDQ_MAXO];  // Ko / bo partials of this thread's point
  float xv[TDQ_MAXD];
  {
    float ko[TDQ_MAXO];
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q)
      ko[q] = ldm(Ko + (f < wl ? f : wl - 1) * dout + (q < dout ? q : dout - 1), q < dout && f < wl);
    float u[S][TDQ_MAXO];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int orow = sp.out[s] >= 0 ? sp.out[s] : 0;
#pragma unroll
      for (int q = 0; q < TDQ_MAXO; ++q) u[s][q] = dJ[((size_t)orow * ldJ + j0 + n) * dout + (q < dout ? q : 0)];
      z[s] = Zb[hi_row(Lh - 1, n, s, S, N) + f];
    }
    // the input point (K0 partials of the last step; loaded here: a load inside the loop's exit
    // branch makes the waitcnt pass wait for it on every iteration's GEMM)
#pragma unroll
    for (int v = 0; v < TDQ_MAXD; ++v) xv[v] = X[(size_t)n * din + (v < din ? v : din - 1)];
    // every load above in flight before the first use (the scheduler otherwise interleaves each load
    // with its use: one memory latency per load); masks applied after
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int q = 0; q < TDQ_MAXO; ++q) u[s][q] = (sp.out[s] >= 0 && ok && q < dout) ? u[s][q] : 0.f;
      z[s] = f < wl ? z[s] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < TDQ_MAXO; ++q) a = fmaf(ko[q], u[s][q], a);
      hb[s] = a;
    }
    // Ko[f][q] = sum over points and seeded streams of h_s[f] dJ_s[q]; bo[q] = sum of dJ_value[q]
    float h[S];
    hi_tanh_f<S, CH>(sp, z, h);
#pragma unroll
    for (int q = 0; q < TDQ_MAXO; ++q) {
      float a = 0.f;
#pragma unroll
      for (int s = 0; s < S; ++s) a = fmaf(f < wl ? h[s] : 0.f, u[s][q], a);
      vo[q] = a;
      vbo[q] = u[0][q];
    }
  }
  HI_TS()
  for (int i = Lh - 1; i >= 0; --i) {
    const int wi = hw(d, i);
    {
      float zb[S];
      if (f < wi) {
        hi_tanh_b<S, CH>(sp, z, hb, zb);
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) zb[s] = 0.f;
      }
      if (ok) {
#pragma unroll
        for (int s = 0; s < S; ++s) Bb[hi_row(i, n, s, S, N) + f] = zb[s];
      }
#pragma unroll
      for (int s = 0; s < S; ++s) hi_put_a(L, pg * S + s, f, zb[s]);
      // vector-parameter partials of this point (padding points: zero adjoints already)
      float* V = L.V + pg * nvs * HI_W;
      V[f] = ok ? zb[0] : 0.f;
      if (i == 0) {
#pragma unroll
        for (int v = 0; v < TDQ_MAXD; ++v) {
          float g = xv[v] * zb[0];
#pragma unroll
          for (int s = 1; s < S; ++s) g += (sp.order[s] == 1 && sp.var[s] == v) ? zb[s] : 0.f;
          if (v < din) V[(1 + v) * HI_W + f] = ok ? g : 0.f;
        }
      }
      if (i == Lh - 1) {
        const int vko = hi_vko(d);
#pragma unroll
        for (int q = 0; q < TDQ_MAXO; ++q) {
          if (q >= dout) break;
          V[(vko + q) * HI_W + f] = vo[q];
          V[(vko + dout + q) * HI_W + f] = vbo[q];
        }
      }
    }
    HI_TS()
    if (i == 0) {
      __syncthreads();
      hi_vsum(L, vrow, d, i, pg, f);
      HI_TS()
      break;
    }
    // hb_{i-1}[k] = sum_o zb_i[o] W_i[k][o]; the next pre-activations load meanwhile
    hi_put_w(L, wr, d, i);
    __syncthreads();
    HI_TS()
    hi_vsum(L, vrow, d, i, pg, f);
    if (i >= 2) hi_get_w(wr, P, d, i - 1);
    const int wp = hw(d, i - 1);
#pragma unroll
    for (int s = 0; s < S; ++s) z[s] = Zb[hi_row(i - 1, n, s, S, N) + f];  // used (masked) after the GEMM
    __builtin_amdgcn_sched_barrier(0);
    hi_mma<true>(L, S, wi);
    HI_TS()
    __syncthreads();  // hb in R; GEMM reads of A / W done
    {
#pragma unroll
      for (int s = 0; s < S; ++s) hb[s] = L.R[(pg * S + s) * HI_AS + f];
      if (f >= wp) {
#pragma unroll
        for (int s = 0; s < S; ++s) hb[s] = z[s] = 0.f;
      }
    }
    __syncthreads();  // R, A, V reused by the next layer
    HI_TS()
  }
  HI_TS_PRINT("chain")
}

// Weight gradients over the point range of split blockIdx.y (one slab row per split, reduced in
// a fixed order afterwards): dK_i = H_{i-1}^T B_i of the hidden-to-hidden layers on 32 x 32 tiles.
// Rows (point x stream) are staged HI_RB at a time through LDS with all loads of a batch in flight
// at once (a split of the AC-baseline set is one batch: one memory latency per workgroup).
#define HI_TILE 32
#define HI_RB 256
__global__ void __launch_bounds__(256) jet_hi_wgrad_kernel(int N, int S, NetDims d, const float* __restrict__ Hb,
                                                           const float* __restrict__ Bb, float* __restrict__ slab,
                                                           int Pst) {
  __shared__ __attribute__((aligned(16))) float Hc[HI_RB][HI_TILE];
  __shared__ __attribute__((aligned(16))) float Gc[HI_RB][HI_TILE];
  const int t = threadIdx.x;
  const int ks = gridDim.y, y = blockIdx.y;
  const int n0 = (int)((long long)N * y / ks), n1 = (int)((long long)N * (y + 1) / ks);
  float* row = slab + (size_t)y * Pst;
  constexpr int TPL = (HI_W / HI_TILE) * (HI_W / HI_TILE);
  const int i = 1 + (int)blockIdx.x / TPL, tile = (int)blockIdx.x % TPL;
  const int kt = tile / (HI_W / HI_TILE), ft = tile % (HI_W / HI_TILE);
  const int win = hw(d, i - 1), wout = hw(d, i);
  if (kt * HI_TILE >= win || ft * HI_TILE >= wout) return;  // uniform: the whole workgroup leaves
  HI_TS_DECL
  HI_TS()
  const int wv = t >> 6, l = t & 63;
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
  const int r0 = n0 * S, r1 = n1 * S;
  const float* Hl = Hb + hi_row(i - 1, 0, 0, S, N) + kt * HI_TILE;
  const float* Bl = Bb + hi_row(i, 0, 0, S, N) + ft * HI_TILE;
  constexpr int NQ = HI_RB * HI_TILE / 4 / 256;  // float4 pieces per thread per operand
  for (int r = r0; r < r1; r += HI_RB) {
    f32x4 hv[NQ], gv[NQ];
#pragma unroll
    for (int u = 0; u < NQ; ++u) {  // every load of the batch first (clamped rows, masked after)
      const int e = t + 256 * u, rr = e >> 3, c = (e & 7) * 4;
      const int rc = r + rr < r1 ? r + rr : r1 - 1;
      hv[u] = *reinterpret_cast<const f32x4*>(Hl + (size_t)rc * HI_W + c);
      gv[u] = *reinterpret_cast<const f32x4*>(Bl + (size_t)rc * HI_W + c);
    }
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int e = t + 256 * u, rr = e >> 3, c = (e & 7) * 4;
      const bool in = r + rr < r1;
      *reinterpret_cast<f32x4*>(&Hc[rr][c]) = in ? hv[u] : f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(&Gc[rr][c]) = in ? gv[u] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
    HI_TS()
    // fp32 MFMA 32x32x2: wave w takes the row pairs 2 (w + 4 m); lane l supplies A[k = l & 31][row
    // l >> 5] = H[row][k] and B[row l >> 5][f = l & 31] = G[row][f] - one conflict-free LDS read each
    const int nb = min(HI_RB, r1 - r);
    for (int rb = 2 * wv; rb < nb; rb += 8) {
      const int rr = min(rb + (l >> 5), HI_RB - 1);  // rows past nb are zero-filled
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Hc[rr][l & 31], Gc[rr][l & 31], acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // the four waves' partials -> fixed-order sum (the staging area is free now); lane l, register q
  // of the 32x32 accumulator holds D[8 (q >> 2) + 4 (l >> 5) + (q & 3)][l & 31]
  float* red = &Hc[0][0];  // [wave][32][32]
#pragma unroll
  for (int q = 0; q < 16; ++q)
    red[(wv * HI_TILE + 8 * (q >> 2) + 4 * (l >> 5) + (q & 3)) * HI_TILE + (l & 31)] = acc[q];
  __syncthreads();
  float* dk = row + off_layer(d, i);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int o = t + 256 * q, kk = o / HI_TILE, ff = o % HI_TILE;
    const float v = (red[(0 * HI_TILE + kk) * HI_TILE + ff] + red[(1 * HI_TILE + kk) * HI_TILE + ff]) +
                    (red[(2 * HI_TILE + kk) * HI_TILE + ff] + red[(3 * HI_TILE + kk) * HI_TILE + ff]);
    const int k = kt * HI_TILE + kk, f = ft * HI_TILE + ff;
    if (k < win && f < wout) dk[k * wout + f] = v;
  }
  HI_TS()
  HI_TS_PRINT("wgrad")
}

// gradient of the hidden-to-hidden kernels: fixed-order sums over the ks split rows of the tile slab
__device__ __forceinline__ void hi_tile_reduce(int bx, const float* __restrict__ slab, int ks, int Pst, const NetDims& d,
                                               float* __restrict__ grad) {
  const int Lh = d.n_hidden;
  const int e = off_layer(d, 1) + bx * 256 + threadIdx.x;
  if (e >= off_layer(d, Lh)) return;
  int layer = 1;
  while (layer + 1 < Lh && e >= off_layer(d, layer + 1)) ++layer;
  const int r = e - off_layer(d, layer);
  if (r >= hw(d, layer - 1) * hw(d, layer)) return;  // bias: the vector reduction's
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int q = 0;
  for (; q + 3 < ks; q += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += slab[(size_t)(q + u) * Pst + e];
  for (; q < ks; ++q) a[0] += slab[(size_t)q * Pst + e];
  grad[e] = (a[0] + a[1]) + (a[2] + a[3]);
}

// gradient of the vector parameters (hidden biases, K0, Ko, bo): one wave per vslab column; lane l
// sums the workgroup rows l, l + 64, ... in order, then a fixed butterfly across the wave
// (deterministic, and ~nwg / 64 dependent loads per lane instead of nwg)
__device__ __forceinline__ void hi_vec_reduce(int bx, const float* __restrict__ vslab, int nwg, int Vst, const NetDims& d,
                                              float* __restrict__ grad) {
  const int Lh = d.n_hidden, din = d.d_in, dout = d.d_out, wl = hw(d, Lh - 1);
  const int vi = bx * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  int e = -1;  // parameter index of vslab column vi (-1: padding column)
  if (vi < Lh * HI_W) {
    const int i = vi / HI_W, f = vi % HI_W;
    if (f < hw(d, i)) e = off_layer(d, i) + (i == 0 ? din : hw(d, i - 1)) * hw(d, i) + f;
  } else if (vi < (Lh + din) * HI_W) {
    const int v = vi / HI_W - Lh, f = vi % HI_W;
    if (f < hw(d, 0)) e = v * hw(d, 0) + f;
  } else if (vi < (Lh + din) * HI_W + HI_W * TDQ_MAXO) {
    const int r = vi - (Lh + din) * HI_W, f = r / TDQ_MAXO, q = r % TDQ_MAXO;
    if (f < wl && q < dout) e = off_layer(d, Lh) + f * dout + q;
  } else {
    const int q = vi - (Lh + din) * HI_W - HI_W * TDQ_MAXO;
    if (q < dout) e = off_layer(d, Lh) + wl * dout + q;
  }
  if (e < 0) return;  // wave-uniform
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int r = l, u = 0;
  for (; r < nwg; r += 64, u = (u + 1) & 3) a[u] += vslab[(size_t)r * Vst + vi];
  float v = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  if (l == 0) grad[e] = v;
}

// both reductions in one launch: blocks [0, ntb) the tile slab, the rest the vector slab
__global__ void __launch_bounds__(256) jet_hi_reduce_kernel(const float* __restrict__ slab, int ks, int Pst,
                                                            const float* __restrict__ vslab, int nwg, int Vst, int ntb,
                                                            NetDims d, float* __restrict__ grad) {
  if ((int)blockIdx.x < ntb)
    hi_tile_reduce(blockIdx.x, slab, ks, Pst, d, grad);
  else
    hi_vec_reduce(blockIdx.x - ntb, vslab, nwg, Vst, d, grad);
}

namespace {

// spec_i: [S, order[S], var[S], out[S], n_terms, (stream, k, nb, b0, b1, b2, b3) x n_terms]
// (terms grouped by stream in stream order); spec_c: coefficients per term
bool hi_spec(HiSpec& sp, const int* si, const float* sc) {
  const int S = si[0];
  if (S < 1 || S > HI_MAXS) return false;
  sp.S = S;
  for (int s = 0; s < HI_MAXS; ++s) {
    sp.order[s] = s < S ? si[1 + s] : 0;
    sp.var[s] = s < S ? si[1 + S + s] : 0;
    sp.out[s] = s < S ? si[1 + 2 * S + s] : -1;
    sp.t0[s] = 0;
    sp.nt[s] = 0;
    if (s < S && (sp.order[s] < 0 || sp.order[s] > 4)) return false;
  }
  if (sp.order[0] != 0) return false;
  const int nt = si[1 + 3 * S];
  if (nt < 0 || nt > HI_MAXT) return false;
  const int* tt = si + 2 + 3 * S;
  int prev = 0;
  for (int k = 0; k < nt; ++k) {
    const int s = tt[7 * k], tk = tt[7 * k + 1], nb = tt[7 * k + 2];
    if (s < 1 || s >= S || s < prev || tk < 1 || tk > 4 || nb < 1 || nb > HI_MAXB) return false;
    if (s != prev) sp.t0[s] = k;
    prev = s;
    sp.nt[s] += 1;
    sp.tk[k] = tk;
    sp.tc[k] = sc[k];
    sp.tnb[k] = nb;
    for (int b = 0; b < HI_MAXB; ++b) {
      const int v = b < nb ? tt[7 * k + 3 + b] : 0;
      if (v < 0 || v >= S || (b < nb && v == 0)) return false;
      sp.tb[k][b] = v;
    }
  }
  // the univariate chain (), (v), (v, v), ...: stream k of order k, one variable, in order
  sp.chain = S >= 2 && S <= 5;
  for (int s = 1; s < S; ++s) sp.chain = sp.chain && sp.order[s] == s;
  if (sp.chain) {
    // every stream's factors are lower streams of the same chain: check via the order-1 variable
    for (int k = 0; k < nt; ++k)
      for (int b = 0; b < tt[7 * k + 2]; ++b) sp.chain = sp.chain && sp.order[tt[7 * k + 3 + b]] >= 1;
  }
  return true;
}

bool hi_dims(NetDims& d, int d_in, const int* widths, int d_out, int n_hidden) {
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return false;
  return d.width <= HI_W && d_in <= TDQ_MAXD && d_out <= TDQ_MAXO;
}

constexpr size_t HI_LDS_MAX = 160 * 1024;
template <typename K>
void hi_attr(K* kern) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)HI_LDS_MAX);
}
bool hi_lds_fits(int S, const NetDims& d) { return hi_lds_floats(S, hi_nvs(d)) * sizeof(float) <= HI_LDS_MAX; }

int hi_splits(int N) { return std::min(HI_KS, std::max(1, (N + 63) / 64)); }

template <int S, bool CH>
int hi_launch_fwd(const float* X, int N, const float* P, const NetDims& d, const HiSpec& sp, float* J, int ldJ, int j0,
                  float* Zb, float* Hb, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    hi_attr(&jet_hi_fwd_kernel<S, CH>);
    attr = true;
  }
  hipLaunchKernelGGL((jet_hi_fwd_kernel<S, CH>), dim3((N + HI_NP - 1) / HI_NP), dim3(HI_THREADS),
                     hi_lds_floats(S, 0) * sizeof(float), st,
                     X, N, P, d, sp, J, ldJ, j0, Zb, Hb);
  TDQ_CHECK_LAUNCH();
  return 0;
}

template <int S, bool CH>
int hi_launch_chain(int N, const float* P, const NetDims& d, const HiSpec& sp, const float* X, const float* dJ,
                    int ldJ, int j0, const float* Zb, float* Bb, float* vslab, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    hi_attr(&jet_hi_chain_kernel<S, CH>);
    attr = true;
  }
  hipLaunchKernelGGL((jet_hi_chain_kernel<S, CH>), dim3((N + HI_NP - 1) / HI_NP), dim3(HI_THREADS),
                     hi_lds_floats(S, hi_nvs(d)) * sizeof(float), st, N, P, d, sp, X, dJ, ldJ, j0, Zb, Bb, vslab);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// (S, chain) -> instantiation
#define HI_CASES(X)                                                                                           \
  X(2, true) X(3, true) X(4, true) X(5, true) X(2, false) X(3, false) X(4, false) X(5, false) X(6, false) \
      X(7, false) X(8, false)

int hi_fwd(const float* X, int N, const float* P, const NetDims& d, const HiSpec& sp, float* J, int ldJ, int j0,
           float* Zb, float* Hb, hipStream_t st) {
  const bool ch = sp.chain != 0;
#define HI_F(SS, CC) \
  if (sp.S == SS && ch == CC) return hi_launch_fwd<SS, CC>(X, N, P, d, sp, J, ldJ, j0, Zb, Hb, st);
  HI_CASES(HI_F)
#undef HI_F
  return (int)hipErrorInvalidValue;
}

int hi_chain(int N, const float* P, const NetDims& d, const HiSpec& sp, const float* X, const float* dJ, int ldJ,
             int j0, const float* Zb, float* Bb, float* vslab, hipStream_t st) {
  const bool ch = sp.chain != 0;
#define HI_B(SS, CC) \
  if (sp.S == SS && ch == CC) return hi_launch_chain<SS, CC>(N, P, d, sp, X, dJ, ldJ, j0, Zb, Bb, vslab, st);
  HI_CASES(HI_B)
#undef HI_B
  return (int)hipErrorInvalidValue;
}

int hi_wgrad(int N, const NetDims& d, const HiSpec& sp, const float* Hb, const float* Bb, float* work, int Pst,
             int ks, hipStream_t st) {
  const int n_tiles = (d.n_hidden - 1) * (HI_W / HI_TILE) * (HI_W / HI_TILE);
  if (n_tiles > 0) {
    hipLaunchKernelGGL(jet_hi_wgrad_kernel, dim3(n_tiles, ks), dim3(256), 0, st, N, sp.S, d, Hb, Bb, work, Pst);
    TDQ_CHECK_LAUNCH();
  }
  return 0;
}

// one activation-sized scratch buffer (Z, H or B), in floats
size_t hi_act_floats(int N, int n_hidden) { return (size_t)n_hidden * N * HI_MAXS * HI_W; }

}  // namespace

extern "C" {

// Z | H | B: pre-activations, post-activations and pre-activation adjoints of every hidden layer
int64_t tdq_jet_hi_scratch_floats(int N, int n_hidden) { return 3 * (int64_t)hi_act_floats(N, n_hidden); }

// tile slab (split rows) + the chain's vector slab (workgroup rows), in floats
int64_t tdq_jet_hi_work_floats(int N, int d_in, const int* widths, int d_out, int n_hidden) {
  NetDims d;
  if (!hi_dims(d, d_in, widths, d_out, n_hidden)) return -1;
  const int nwg = (N + HI_NP - 1) / HI_NP;
  return (int64_t)hi_splits(N) * slab_stride(param_count(d)) + (int64_t)nwg * hi_vrow(d);
}

// forward over N points X[N][d_in]: stream s with out[s] >= 0 -> J[(out[s] * ldJ + j0 + n) * d_out + q];
// hidden-layer activations -> Z (tdq_jet_hi_scratch_floats)
int tdq_jet_hi_fwd(const float* X, int N, const float* P, int d_in, const int* widths, int d_out, int n_hidden,
                   const int* spec_i, const float* spec_c, float* J, int ldJ, int j0, float* Z, void* stream) {
  if (N <= 0) return 0;
  NetDims d;
  HiSpec sp;
  if (!hi_dims(d, d_in, widths, d_out, n_hidden) || !hi_spec(sp, spec_i, spec_c) || !hi_lds_fits(sp.S, d))
    return (int)hipErrorInvalidValue;
  const size_t A = hi_act_floats(N, n_hidden);
  return hi_fwd(X, N, P, d, sp, J, ldJ, j0, Z, Z + A, reinterpret_cast<hipStream_t>(stream));
}

// backward: the adjoints dJ of the streams with out[s] >= 0 -> the flat parameter gradient `grad`
// (adjoint chain per point group, then the weight gradients over point splits into slab rows in
// `work`, reduced in a fixed order: deterministic)
// part: 0 = all, 1 = the adjoint chain only, 2 = the weight-gradient tiles + reduction only (after a
// part-1 call on the same buffers; the two halves may run on different streams, fit.run_ranges)
int tdq_jet_hi_bwd_part(const float* X, int N, const float* P, int d_in, const int* widths, int d_out, int n_hidden,
                        const int* spec_i, const float* spec_c, const float* dJ, int ldJ, int j0, float* Z,
                        float* work, float* grad, int part, void* stream) {
  NetDims d;
  HiSpec sp;
  if (!hi_dims(d, d_in, widths, d_out, n_hidden) || !hi_spec(sp, spec_i, spec_c) || !hi_lds_fits(sp.S, d))
    return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int Ptot = param_count(d), Pst = slab_stride(Ptot);
  if (N <= 0) return (int)hipMemsetAsync(grad, 0, sizeof(float) * Ptot, st);
  const size_t A = hi_act_floats(N, n_hidden);
  const int ks = hi_splits(N), nwg = (N + HI_NP - 1) / HI_NP;
  float* vslab = work + (size_t)ks * Pst;
  if (part != 2) {
    const int rc = hi_chain(N, P, d, sp, X, dJ, ldJ, j0, Z, Z + 2 * A, vslab, st);
    if (rc || part == 1) return rc;
  }
  const int rc = hi_wgrad(N, d, sp, Z + A, Z + 2 * A, work, Pst, ks, st);
  if (rc) return rc;
  const int ntile = off_layer(d, n_hidden) - off_layer(d, 1);
  const int ntb = (ntile + 255) / 256;
  const int ncol = (n_hidden + d_in) * HI_W + HI_W * TDQ_MAXO + TDQ_MAXO;
  hipLaunchKernelGGL(jet_hi_reduce_kernel, dim3(ntb + (ncol + 3) / 4), dim3(256), 0, st, work, ks, Pst, vslab, nwg,
                     hi_vrow(d), ntb, d, grad);
  TDQ_CHECK_LAUNCH();
  return 0;
}

int tdq_jet_hi_bwd(const float* X, int N, const float* P, int d_in, const int* widths, int d_out, int n_hidden,
                   const int* spec_i, const float* spec_c, const float* dJ, int ldJ, int j0, float* Z,
                   float* work, float* grad, void* stream) {
  return tdq_jet_hi_bwd_part(X, N, P, d_in, widths, d_out, n_hidden, spec_i, spec_c, dJ, ldJ, j0, Z, work, grad, 0,
                             stream);
}

// whether the kernels' LDS takes S streams with this input / output width and depth (1) or not (0)
int tdq_jet_hi_lds_ok(int S, int d_in, int d_out, int n_hidden) {
  NetDims d;
  d.d_in = d_in;
  d.d_out = d_out;
  d.n_hidden = n_hidden;
  return S >= 1 && S <= HI_MAXS && d_in <= TDQ_MAXD && d_out <= TDQ_MAXO && hi_lds_fits(S, d) ? 1 : 0;
}

int tdq_jet_hi_limits(int* out) {
  out[0] = HI_MAXS;
  out[1] = HI_MAXT;
  out[2] = HI_W;
  out[3] = HI_NP;
  return 0;
}

}  // extern "C"
