// Device-resident L-BFGS for gfx950.
//
// The reference runs the lua-port L-BFGS on the host (tensordiffeq/optimizers.py:107-308): a
// two-loop recursion of ~200 tiny TF ops over <= 50 history pairs, several device->host syncs and
// a numpy weight round-trip per iteration.  Here one iteration is five small kernels that live in
// the same HIP graph as the loss/gradient evaluation, and the host reads nothing until it polls
// the "active" flag every few dozen iterations:
//
//   lbfgs_dots   grid (chunks, slot groups of LB_G): every dot product the iteration needs in ONE
//                pass over the history ring - per slot i: s_i.g, y_i.g, s_i.y, y_i.y, s.y_i - and for
//                the new pair s.y, y.y, s.g, y.g plus |g|_1 (s = t d, y = g - g_old formed on the
//                fly); fp64 partial sums per chunk;
//   lbfgs_logic  one workgroup: reduces the partials in fixed order, runs the post-evaluation tests
//                (NaN, best iterate, maxIter / maxEval, tolFun / tolX / |f - f_old|), the curvature
//                test y.s > 1e-10 with ring push (H0 = y.s / y.y), keeps S^T Y and Y^T Y current by
//                one new row + column per push, and turns the compact representation of Byrd,
//                Nocedal & Schnabel (1994) into per-slot coefficients with two k x k triangular
//                solves (one wave, one lane per history pair, rows in registers);
//   lbfgs_dir    64-element tiles, the history sum split over the block's 4 waves: stores the
//                pushed pair into the ring, d = cG g + sum_i (cS_i s_i + cY_i y_i), g_old = g,
//                best-weights snapshot, partials of g.d and |d|_1;
//   lbfgs_step   one workgroup: descent test g.d > -tolX, step t = min(1, 1/|g|_1) on the first
//                iteration else the fixed learning rate (0.8, reference fit.py:67), f_old = f;
//   lbfgs_axpy   x += t d (launched in front of the next evaluation).
//
// All scalar state is fp64 in one small device array (layout LB_* below, mirrored by
// tensordiffeq_amd/optimizers/lbfgs_device.py).  Once a stopping test fires every kernel is a
// no-op, so graph replays past convergence change nothing.
#include "common.h"
#include "jet_bf3.h"

#define LB_MAXM 64
#define LB_NF 5

enum {
  LB_ACTIVE = 0,  // 1 while iterating
  LB_NITER,       // reference nIter
  LB_FEVAL,       // reference currentFuncEval (the initial evaluation included)
  LB_K,           // valid history pairs
  LB_HEAD,        // ring slot of the oldest pair
  LB_PUSHED,      // the current iteration pushed a pair ...
  LB_SLOT,        // ... into this slot
  LB_BEST,        // snapshot x into best_x in the next lbfgs_dir
  LB_F,           // loss at the current x
  LB_FOLD,        // loss before the last step
  LB_MINLOSS,     // best loss so far
  LB_BESTEP,      // epoch of the best loss (-1 = initial point)
  LB_HDIAG,       // H0 scale y.s / y.y
  LB_T,           // step length of the current direction
  LB_DT1,         // |d|_1 * t
  LB_G1,          // |g|_1 at the current x
  LB_REASON,      // why the run stopped (0 = running)
  LB_GTD,         // g.d of the current direction
  LB_NST = 24
};

enum { LB_R_RUN = 0, LB_R_TOLFUN0 = 1, LB_R_NAN = 2, LB_R_MAXITER = 3, LB_R_TOL = 4, LB_R_GTD = 5 };

struct LbCfg {
  int p;            // parameters
  int m;            // history size (<= LB_MAXM)
  int max_iter;
  int nchunks;      // lbfgs_dots chunks
  int nblk;         // lbfgs_dir blocks
  int fhist_len;    // length of the loss history buffer (0: none)
  double max_eval;  // 1.25 max_iter (reference optimizers.py:113)
  double lr;        // fixed step (0.8)
  double tol_fun;
  double tol_x;
  int legacy_stop;  // 1: the reference's effective function-change test |f| < tolX (tf.abs(f, f_old),
                    //    optimizers.py:273 - the second argument is the op name); 0: |f - f_old| < tolX
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 256-thread block sum of NV doubles; the result is valid in thread 0
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* red) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NV; ++q) v[q] = wave_sum(v[q]);
  if (l == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) red[w * NV + q] = v[q];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = ((red[q] + red[NV + q]) + red[2 * NV + q]) + red[3 * NV + q];
}

// partial loads of the fused kernels' last-arriving block: relaxed agent-scope atomics = sc1 loads
// that bypass this CU's L1 (the producers stored with sc1, MI355X_MICROARCH.md hand-off table)
template <bool SC1>
__device__ __forceinline__ double part_ld(const double* p) {
  if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}
template <bool SC1>
__device__ __forceinline__ void part_st(double* p, double v) {
  if constexpr (SC1)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

__device__ __forceinline__ bool slot_valid(int i, int head, int k, int m) { return ((i - head + m) % m) < k; }

// lane `q` (wave-uniform) of a double, through two v_readlane_b32
__device__ __forceinline__ double readlane_d(double v, int q) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, q), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), q);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// d_j = cG g_j + sum_q (cS_q s_qj + cY_q y_qj) over the k history pairs (chronological q): the
// four waves of a direction block share one 64-element tile, wave w sums the pairs of quarter w
// (at most LB_MAXM / 4, every load of it in flight together), and wave 0 adds the quarters in
// fixed order.  Shared by both update paths (same summation order, so the same bits).
__device__ __forceinline__ double dir_quarter(const float* __restrict__ S, const float* __restrict__ Y,
                                              const double* __restrict__ coef, int j, int p, int k, int head, int m,
                                              int pushed, int slot, float tf, float g, float dj, float oj, int w) {
  const int q0 = (w * k) >> 2, q1 = ((w + 1) * k) >> 2;
  double acc[2] = {0.0, 0.0};
  // branch-free so every load of the quarter is in flight together: past the quarter's end the
  // first pair is re-read and masked out; the pushed slot's row is read (this block has not
  // overwritten it yet) and replaced by the new pair
  constexpr int NQ = LB_MAXM / 4;
  int ir[NQ];
  float sl[NQ], yl[NQ];
#pragma unroll
  for (int t = 0; t < NQ; ++t) {
    int i = head + (q0 + t < q1 ? q0 + t : q0);
    if (i >= m) i -= m;
    ir[t] = i;
    // uniform row bases (scalar registers) + the lane's 32-bit element offset
    sl[t] = (S + (size_t)i * p)[j];
    yl[t] = (Y + (size_t)i * p)[j];
  }
  const float s = tf * dj, y = g - oj;  // the new pair (after the loads: nothing waits on them)
#pragma unroll
  for (int t = 0; t < NQ; ++t) {
    const int i = ir[t];
    const bool nw = pushed && i == slot;
    const double si = nw ? (double)s : (double)sl[t];
    const double yi = nw ? (double)y : (double)yl[t];
    const double v = coef[i] * si + coef[m + i] * yi;
    acc[t & 1] += (q0 + t < q1) ? v : 0.0;
  }
  return acc[0] + acc[1];
}

// ---------------------------------------------------------------------------------------------
// the partial sums of one (chunk, slot group) block of the dots grid -> part (thread 0 stores
// them).  A block covers LB_G history slots (the new pair is slot m); a thread takes LB_R
// elements per round and issues every load of the round (g, d, g_old and the 2 LB_G history
// values of each element) before the first use, so a round costs one memory latency.  Each
// slot's sum runs over its elements in a fixed order shared by both update paths.
#define LB_G 1
#define LB_R 8
template <bool SC1>
__device__ __forceinline__ void lbfgs_dots_body(const float* __restrict__ fg, const float* __restrict__ g_old,
                                                const float* __restrict__ d, const float* __restrict__ S,
                                                const float* __restrict__ Y, const double* __restrict__ st,
                                                double* __restrict__ part, const LbCfg& c, double* red) {
  const int i0 = blockIdx.y * LB_G, ch = blockIdx.x;
  const int lo = (int)(((long long)c.p * ch) / c.nchunks), hi = (int)(((long long)c.p * (ch + 1)) / c.nchunks);
  const float tf = (float)st[LB_T];
  const int k = (int)st[LB_K], head = (int)st[LB_HEAD];
  const bool active = st[LB_ACTIVE] != 0.0;
  bool run[LB_G];
  const float* Si[LB_G];
  const float* Yi[LB_G];
#pragma unroll
  for (int u = 0; u < LB_G; ++u) {
    const int i = i0 + u;
    run[u] = active && i < c.m && slot_valid(i, head, k, c.m);
    Si[u] = S + (size_t)(run[u] ? i : 0) * c.p;  // row 0 for idle slots: the loads stay unconditional
    Yi[u] = Y + (size_t)(run[u] ? i : 0) * c.p;
  }
  const bool newp = active && i0 <= c.m && c.m < i0 + LB_G;  // this group holds the new pair
  double a[LB_G][LB_NF];
#pragma unroll
  for (int u = 0; u < LB_G; ++u)
#pragma unroll
    for (int q = 0; q < LB_NF; ++q) a[u][q] = 0.0;
  for (int j0 = lo + (int)threadIdx.x; j0 < hi; j0 += 256 * LB_R) {
    float gv[LB_R], dv[LB_R], ov[LB_R], sv[LB_G][LB_R], yv[LB_G][LB_R];
#pragma unroll
    for (int r = 0; r < LB_R; ++r) {
      const int j = min(j0 + 256 * r, hi - 1);  // clamped: past the chunk's end masked below
      gv[r] = fg[j];
      dv[r] = d[j];
      ov[r] = g_old[j];
#pragma unroll
      for (int u = 0; u < LB_G; ++u) {
        sv[u][r] = Si[u][j];
        yv[u][r] = Yi[u][j];
      }
    }
#pragma unroll
    for (int r = 0; r < LB_R; ++r) {
      if (j0 + 256 * r >= hi) break;
      const float g = gv[r];
      const float s = tf * dv[r], y = g - ov[r];
#pragma unroll
      for (int u = 0; u < LB_G; ++u) {
        if (i0 + u == c.m) {
          if (newp) {
            a[u][0] += (double)s * y;
            a[u][1] += (double)y * y;
            a[u][2] += (double)s * g;
            a[u][3] += (double)y * g;
            a[u][4] += fabs((double)g);
          }
        } else if (run[u]) {
          const double si = sv[u][r], yi = yv[u][r];
          a[u][0] += si * g;
          a[u][1] += yi * g;
          a[u][2] += si * y;
          a[u][3] += yi * y;
          a[u][4] += (double)s * yi;
        }
      }
    }
  }
  double* flat = &a[0][0];
  block_sum<LB_G * LB_NF>(*reinterpret_cast<double(*)[LB_G * LB_NF]>(flat), red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int u = 0; u < LB_G; ++u) {
      const int i = i0 + u;
      if (i > c.m) break;
      double* o = part + ((size_t)ch * (c.m + 1) + i) * LB_NF;
#pragma unroll
      for (int q = 0; q < LB_NF; ++q) part_st<SC1>(&o[q], a[u][q]);
    }
  }
}

__global__ void __launch_bounds__(256) lbfgs_dots_kernel(const float* __restrict__ fg, const float* __restrict__ g_old,
                                                         const float* __restrict__ d, const float* __restrict__ S,
                                                         const float* __restrict__ Y, const double* __restrict__ st,
                                                         double* __restrict__ part, LbCfg c) {
  __shared__ double red[4 * LB_G * LB_NF];
  lbfgs_dots_body<false>(fg, g_old, d, S, Y, st, part, c, red);
}

// ---------------------------------------------------------------------------------------------
// S^T Y and Y^T Y live in global memory by PHYSICAL ring slot (m x m each).  The logic copies both
// into LDS while it reduces the dot partials (every load of a thread issued before the first
// store), patches the pushed slot's row and column in both copies, and solves from LDS.
//
// dynamic LDS (doubles): dots[(m+1)*5] | SYl[m*m] | YYl[m*m]
__host__ __device__ inline size_t lbfgs_logic_lds(int m) { return ((size_t)(m + 1) * LB_NF + 2 * (size_t)m * m) * 8; }

template <bool SC1>
__device__ __forceinline__ void lbfgs_logic_body(const float* __restrict__ fg, const double* __restrict__ part,
                                                 double* __restrict__ st, double* __restrict__ SY,
                                                 double* __restrict__ YY, double* __restrict__ coef,
                                                 float* __restrict__ fhist, const LbCfg& c, double* lb_lds) {
  const int tid = threadIdx.x, m = c.m, mm = m * m;
  double* dots = lb_lds;
  double* SYl = dots + (m + 1) * LB_NF;
  double* YYl = SYl + mm;
  // 1. copy S^T Y / Y^T Y into LDS and reduce the chunk partials (fixed order: deterministic)
  {
    constexpr int NE = (LB_MAXM * LB_MAXM + 255) / 256;
    double sv[NE], yv[NE];
#pragma unroll
    for (int r = 0; r < NE; ++r) {
      const int e = min(tid + 256 * r, mm - 1);
      sv[r] = SY[e];
      yv[r] = YY[e];
    }
    for (int v = tid; v < (m + 1) * LB_NF; v += 256) {
      double a0 = 0.0, a1 = 0.0;
      int ch = 0;
      for (; ch + 15 < c.nchunks; ch += 16) {  // sixteen loads in flight
        double q[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) q[u] = part_ld<SC1>(&part[(size_t)(ch + u) * (m + 1) * LB_NF + v]);
#pragma unroll
        for (int u = 0; u < 16; u += 2) {
          a0 += q[u];
          a1 += q[u + 1];
        }
      }
      if (ch + 7 < c.nchunks) {
        double q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = part_ld<SC1>(&part[(size_t)(ch + u) * (m + 1) * LB_NF + v]);
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
          a0 += q[u];
          a1 += q[u + 1];
        }
        ch += 8;
      }
      for (; ch + 1 < c.nchunks; ch += 2) {
        a0 += part_ld<SC1>(&part[(size_t)ch * (m + 1) * LB_NF + v]);
        a1 += part_ld<SC1>(&part[(size_t)(ch + 1) * (m + 1) * LB_NF + v]);
      }
      if (ch < c.nchunks) a0 += part_ld<SC1>(&part[(size_t)ch * (m + 1) * LB_NF + v]);
      dots[v] = a0 + a1;
    }
#pragma unroll
    for (int r = 0; r < NE; ++r) {
      const int e = tid + 256 * r;
      if (e < mm) {
        SYl[e] = sv[r];
        YYl[e] = yv[r];
      }
    }
  }
  __syncthreads();
  // everything below runs on wave 0: the scalar logic is evaluated by every lane (uniform values,
  // lane 0 stores), the pair coefficients with one lane per history pair - no further barriers
  // (LDS accesses of one wave complete in program order; the wavefront fences below only keep
  // the compiler from reordering them)
  if (tid >= 64) return;
  const int lane = tid;
  const bool L0 = lane == 0;
  // 2. post-evaluation tests of the previous step (reference optimizers.py:241-296, with the
  //    B9 fixes of eager_lbfgs), then the curvature test and ring push (optimizers.py:168-185)
  const double* sc = dots + m * LB_NF;  // s.y, y.y, s.g, y.g, |g|_1
  const double f = (double)fg[c.p];
  int n_iter = (int)st[LB_NITER];
  const double fe0 = st[LB_FEVAL], dt1 = st[LB_DT1], fold = st[LB_FOLD], hd_old = st[LB_HDIAG];
  double minloss = st[LB_MINLOSS];
  int k = (int)st[LB_K], head = (int)st[LB_HEAD];
  int best = 0, done = 0, reason = LB_R_RUN;
  if (L0) st[LB_G1] = sc[4];
  if (n_iter == 0) {
    if (L0 && fhist != nullptr && c.fhist_len > 0) fhist[0] = (float)f;
    if (isfinite(f)) {
      best = 1;
      minloss = f;
      if (L0) st[LB_BESTEP] = -1.0;
    }
    if (sc[4] <= c.tol_fun) {
      done = 1;
      reason = LB_R_TOLFUN0;
    }
  } else {
    const double fe = fe0 + 1.0;
    if (L0) st[LB_FEVAL] = fe;
    if (L0 && fhist != nullptr && n_iter < c.fhist_len) fhist[n_iter] = (float)f;
    if (isnan(f)) {
      done = 1;
      reason = LB_R_NAN;
    } else {
      if (f < minloss) {
        best = 1;
        minloss = f;
        if (L0) st[LB_BESTEP] = (double)(n_iter - 1);
      }
      if (n_iter >= c.max_iter || fe >= c.max_eval) {
        done = 1;
        reason = LB_R_MAXITER;
      } else if (sc[4] <= c.tol_fun || dt1 <= c.tol_x || (c.legacy_stop ? fabs(f) : fabs(f - fold)) < c.tol_x) {
        done = 1;
        reason = LB_R_TOL;
      }
    }
  }
  if (L0) {
    st[LB_F] = f;
    st[LB_MINLOSS] = minloss;
    st[LB_BEST] = (double)best;
  }
  int pushed = 0, slot = -1;
  double hd = hd_old;
  const double ys = sc[0], yy = sc[1];
  if (done) {
    if (L0) {
      st[LB_ACTIVE] = 0.0;
      st[LB_REASON] = (double)reason;
      st[LB_PUSHED] = 0.0;
      st[LB_SLOT] = -1.0;
    }
    return;
  }
  n_iter += 1;
  if (n_iter > 1 && ys > 1e-10) {
    if (k == m) {
      slot = head;
      head = (head + 1) % m;
    } else {
      slot = (head + k) % m;
      k += 1;
    }
    hd = ys / yy;
    pushed = 1;
  }
  if (L0) {
    st[LB_NITER] = (double)n_iter;
    st[LB_K] = (double)k;
    st[LB_HEAD] = (double)head;
    st[LB_HDIAG] = hd;
    st[LB_PUSHED] = (double)pushed;
    st[LB_SLOT] = (double)slot;
  }
  const double gam = n_iter == 1 ? 1.0 : hd;
  // 3. the pushed slot's row / column of S^T Y and Y^T Y, in memory (later iterations) and LDS
  if (pushed && lane < m && slot_valid(lane, head, k, m)) {
    const int j = lane;
    const double* dj = dots + j * LB_NF;
    const double snj = j == slot ? ys : dj[4], sjn = j == slot ? ys : dj[2], yj = j == slot ? yy : dj[3];
    SY[slot * m + j] = snj;  // s_new . y_j
    SY[j * m + slot] = sjn;  // s_j . y_new
    YY[j * m + slot] = yj;
    YY[slot * m + j] = yj;
    SYl[slot * m + j] = snj;
    SYl[j * m + slot] = sjn;
    YYl[j * m + slot] = yj;
    YYl[slot * m + j] = yj;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (n_iter == 1 || k == 0) {  // d = -H0 g (first iteration: H0 = I)
    for (int v = lane; v < 2 * m; v += 64) coef[v] = 0.0;
    if (L0) coef[2 * m] = -gam;
    return;
  }
  // 4. compact product (lane j = chronological pair j, physical slot ij):
  //    R u = S^T g ; rhs = D u + gam Y^T Y u - gam Y^T g ; R^T p1 = rhs ;
  //    H g = gam g + S p1 - gam Y u   ->   d = -H g
  //    R = upper triangle of S^T Y in chronological order.  Each substitution step broadcasts its
  //    pivot with v_readlane (uniform q) and multiplies by the pivot's reciprocal, computed for
  //    every lane up front; the LDS operands of a step do not depend on the chain, so the
  //    8-step unrolled groups keep them ahead of it.
  const int j = lane;
  const bool jv = j < k;
  int ij = head + j;
  if (ij >= m) ij -= m;
  ij = jv ? ij : 0;
  const double rjj = SYl[ij * m + ij];
  const double rdj = jv ? 1.0 / rjj : 0.0;
  const bool nwj = pushed && ij == slot;
  double r = jv ? (nwj ? dots[m * LB_NF + 2] : dots[ij * LB_NF + 0]) : 0.0;  // s_j . g
  double u = 0.0;
  // back substitution: q = k-1 .. 0 ; R[j][q] = SYl[ij][iq]
  int iq = head + k - 1;
  if (iq >= m) iq -= m;
#pragma unroll 8
  for (int q = k - 1; q >= 0; --q) {
    const double rq = SYl[ij * m + iq];
    const double uq = readlane_d(r, q) * readlane_d(rdj, q);
    if (j == q) u = uq;
    if (j < q) r -= rq * uq;
    iq = iq == 0 ? m - 1 : iq - 1;
  }
  // rhs = R[j][j] u_j + gam (Y^T Y u)_j - gam y_j.g
  double yu = 0.0;
  iq = head;
#pragma unroll 8
  for (int q = 0; q < k; ++q) {
    yu += YYl[iq * m + ij] * readlane_d(u, q);
    iq = iq + 1 == m ? 0 : iq + 1;
  }
  const double bj = jv ? (nwj ? dots[m * LB_NF + 3] : dots[ij * LB_NF + 1]) : 0.0;  // y_j . g
  double rr = jv ? rjj * u + gam * yu - gam * bj : 0.0;
  // forward substitution with R^T: R[q][j] = SYl[iq][ij]
  double p1 = 0.0;
  iq = head;
#pragma unroll 8
  for (int q = 0; q < k; ++q) {
    const double cq = SYl[iq * m + ij];
    const double pq = readlane_d(rr, q) * readlane_d(rdj, q);
    if (j == q) p1 = pq;
    if (j > q && jv) rr -= cq * pq;
    iq = iq + 1 == m ? 0 : iq + 1;
  }
  // 5. per PHYSICAL slot
  if (jv) {
    coef[ij] = -p1;
    coef[m + ij] = gam * u;
  }
  for (int v = lane; v < m; v += 64)
    if (((v - head + m) % m) >= k) coef[v] = coef[m + v] = 0.0;
  if (L0) coef[2 * m] = -gam;
}

__global__ void __launch_bounds__(256) lbfgs_logic_kernel(const float* __restrict__ fg, const double* __restrict__ part,
                                                          double* __restrict__ st, double* __restrict__ SY,
                                                          double* __restrict__ YY, double* __restrict__ coef,
                                                          float* __restrict__ fhist, LbCfg c) {
  extern __shared__ __attribute__((aligned(16))) double lb_lds[];
  if (st[LB_ACTIVE] == 0.0) {
    if (threadIdx.x == 0) st[LB_BEST] = 0.0;
    return;
  }
  lbfgs_logic_body<false>(fg, part, st, SY, YY, coef, fhist, c, lb_lds);
}

// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) lbfgs_dir_kernel(const float* __restrict__ x, const float* __restrict__ fg,
                                                        float* __restrict__ g_old, float* __restrict__ d,
                                                        float* __restrict__ S, float* __restrict__ Y,
                                                        float* __restrict__ best_x, const double* __restrict__ st,
                                                        const double* __restrict__ coef, double* __restrict__ part2,
                                                        LbCfg c) {
  __shared__ double red[8];
  __shared__ double qs[4][64];
  const bool best = st[LB_BEST] != 0.0, active = st[LB_ACTIVE] != 0.0;
  const int n_iter = (int)st[LB_NITER], pushed = (int)st[LB_PUSHED], slot = (int)st[LB_SLOT];
  const int k = (int)st[LB_K], head = (int)st[LB_HEAD], m = c.m;
  const float tf = (float)st[LB_T];
  const double cG = coef[2 * m];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // w: wave-uniform
  double acc[2] = {0.0, 0.0};
  for (int jb = blockIdx.x * 64; jb < c.p; jb += gridDim.x * 64) {
    const int j = jb + l;
    const bool in = j < c.p;
    const int jc = in ? j : c.p - 1;  // unconditional loads: all in flight before the first use
    const float g = fg[jc], dj = d[jc], oj = g_old[jc], xj = x[jc];
    // branch-free (k = 0 before the first push: every pair masked; rows stay in range)
    const double qv = dir_quarter(S, Y, coef, jc, c.p, k, head, m, pushed, slot, tf, g, dj, oj, w);
    qs[w][l] = (active && n_iter > 1) ? qv : 0.0;
    const float s = tf * dj, y = g - oj;
    __syncthreads();
    if (w == 0 && in) {
      if (best) best_x[j] = xj;
      if (active) {
        double dn = cG * g;
        if (n_iter > 1) {
          if (pushed) {
            S[(size_t)slot * c.p + j] = s;
            Y[(size_t)slot * c.p + j] = y;
          }
          dn += (qs[0][l] + qs[1][l]) + (qs[2][l] + qs[3][l]);
        }
        const float df = (float)dn;
        g_old[j] = g;
        d[j] = df;
        acc[0] += (double)g * df;
        acc[1] += fabs((double)df);
      }
    }
    __syncthreads();  // qs is rewritten by the next tile
  }
  block_sum<2>(acc, red);
  if (threadIdx.x == 0) {
    part2[2 * blockIdx.x] = acc[0];
    part2[2 * blockIdx.x + 1] = acc[1];
  }
}

// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) lbfgs_step_kernel(const double* __restrict__ part2, double* __restrict__ st,
                                                         LbCfg c) {
  __shared__ double red[8];
  if (st[LB_ACTIVE] == 0.0) return;
  double acc[2] = {0.0, 0.0};
  for (int b = threadIdx.x; b < c.nblk; b += 256) {
    acc[0] += part2[2 * b];
    acc[1] += part2[2 * b + 1];
  }
  block_sum<2>(acc, red);
  if (threadIdx.x == 0) {
    const double gtd = acc[0];
    st[LB_GTD] = gtd;
    if (gtd > -c.tol_x) {  // cannot make progress along d (reference optimizers.py:224)
      st[LB_ACTIVE] = 0.0;
      st[LB_REASON] = (double)LB_R_GTD;
      return;
    }
    const double t = ((int)st[LB_NITER] == 1) ? fmin(1.0, 1.0 / st[LB_G1]) : c.lr;
    st[LB_T] = t;
    st[LB_DT1] = acc[1] * t;
    st[LB_FOLD] = st[LB_F];
  }
}

__global__ void __launch_bounds__(256) lbfgs_axpy_kernel(float* __restrict__ x, const float* __restrict__ d,
                                                         const double* __restrict__ st, int p) {
  if (st[LB_ACTIVE] == 0.0) return;
  const float tf = (float)st[LB_T];
  for (int j = blockIdx.x * 256 + threadIdx.x; j < p; j += gridDim.x * 256) x[j] = fmaf(tf, d[j], x[j]);
}

// ---------------------------------------------------------------------------------------------
// Fused update: TWO launches per iteration instead of dots -> logic -> dir -> step -> axpy.
//   lbfgs_dots_logic  the dots grid; every block stores its partials write-through (sc1), waits
//                     for them, and draws a ticket (agent-scope atomic add); the block that draws
//                     the last ticket runs the logic on the partials (sc1 loads) and re-arms the
//                     ticket.  (Hand-off protocol: MI355X_MICROARCH.md, inter-workgroup table row 1.)
//   lbfgs_dir_step    the direction pass, plus the step taken speculatively: t of the NEXT step
//                     is known before g.d is (min(1, 1/|g|_1) on the first iteration, else the
//                     fixed lr), so every element does x += t d right after computing d (old x
//                     kept in x_prev); the last-ticket block reduces g.d / |d|_1 and runs the
//                     descent test - in the rare stop case it restores x from x_prev, so the
//                     trajectory is bit-identical to the five-launch path.  With a weight-image
//                     target (the split-bf16 objective's scratch) every new x element is also
//                     scattered into the next evaluation's bf16 hi / lo A images and fp32 aux
//                     image, so the objective runs without its pack launch.
// The order of every reduction is the five-launch path's: same values, bit for bit.
__global__ void __launch_bounds__(256) lbfgs_dots_logic_kernel(const float* __restrict__ fg,
                                                               const float* __restrict__ g_old,
                                                               const float* __restrict__ d, const float* __restrict__ S,
                                                               const float* __restrict__ Y, double* __restrict__ st,
                                                               double* __restrict__ part, double* __restrict__ SY,
                                                               double* __restrict__ YY, double* __restrict__ coef,
                                                               float* __restrict__ fhist, int* __restrict__ ticket,
                                                               LbCfg c) {
  extern __shared__ __attribute__((aligned(16))) double lb_lds[];
  __shared__ double red[4 * LB_G * LB_NF];
  __shared__ int last;
  if (st[LB_ACTIVE] == 0.0) {  // every block sees the same value: only the last block changes it
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) st[LB_BEST] = 0.0;
    return;
  }
  lbfgs_dots_body<true>(fg, g_old, d, S, Y, st, part, c, red);
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's sc1 partial stores have landed
    const int nb = (int)(gridDim.x * gridDim.y);
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == nb - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lbfgs_logic_body<true>(fg, part, st, SY, YY, coef, fhist, c, lb_lds);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) lbfgs_dir_step_kernel(float* __restrict__ x, const float* __restrict__ fg,
                                                             float* __restrict__ g_old, float* __restrict__ d,
                                                             float* __restrict__ S, float* __restrict__ Y,
                                                             float* __restrict__ best_x, float* __restrict__ x_prev,
                                                             double* __restrict__ st, const double* __restrict__ coef,
                                                             double* __restrict__ part2, int* __restrict__ ticket,
                                                             LbCfg c, TailImg ti) {
  __shared__ double red[8];
  __shared__ double qs[4][64];
  __shared__ int last, stop;
  const bool best = st[LB_BEST] != 0.0, active = st[LB_ACTIVE] != 0.0;
  const int n_iter = (int)st[LB_NITER], pushed = (int)st[LB_PUSHED], slot = (int)st[LB_SLOT];
  const int k = (int)st[LB_K], head = (int)st[LB_HEAD], m = c.m;
  const float tf = (float)st[LB_T];
  // the next step's length (the five-launch lbfgs_step_kernel's formula)
  const double tnext = (n_iter == 1) ? fmin(1.0, 1.0 / st[LB_G1]) : c.lr;
  const float tn = (float)tnext;
  const double cG = coef[2 * m];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // w: wave-uniform
  double acc[2] = {0.0, 0.0};
  for (int jb = blockIdx.x * 64; jb < c.p; jb += gridDim.x * 64) {
    const int j = jb + l;
    const bool in = j < c.p;
    const int jc = in ? j : c.p - 1;  // unconditional loads: all in flight before the first use
    const float g = fg[jc], dj = d[jc], oj = g_old[jc], xj = x[jc];
    // branch-free (k = 0 before the first push: every pair masked; rows stay in range)
    const double qv = dir_quarter(S, Y, coef, jc, c.p, k, head, m, pushed, slot, tf, g, dj, oj, w);
    qs[w][l] = (active && n_iter > 1) ? qv : 0.0;
    const float s = tf * dj, y = g - oj;
    __syncthreads();
    if (w == 0 && in) {
      if (best) best_x[j] = xj;
      if (active) {
        double dn = cG * g;
        if (n_iter > 1) {
          if (pushed) {
            S[(size_t)slot * c.p + j] = s;
            Y[(size_t)slot * c.p + j] = y;
          }
          dn += (qs[0][l] + qs[1][l]) + (qs[2][l] + qs[3][l]);
        }
        const float df = (float)dn;
        g_old[j] = g;
        d[j] = df;
        // speculative step, undone below if the descent test fails.  Both x stores are
        // write-through (sc1): a plain store would leave a dirty line in this XCD's L2 whose
        // write-back at kernel end could land after the last block's restore of the same element.
        __hip_atomic_store(&x_prev[j], xj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float xn = fmaf(tn, df, xj);
        __hip_atomic_store(&x[j], xn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ti.fimg != nullptr) scatter_param(xn, j, ti);  // the next evaluation's weight images
        acc[0] += (double)g * df;
        acc[1] += fabs((double)df);
      }
    }
    __syncthreads();  // qs is rewritten by the next tile
  }
  if (!active) return;  // uniform: no ticket, nothing to reduce
  block_sum<2>(acc, red);
  if (threadIdx.x == 0) {
    part_st<true>(&part2[2 * blockIdx.x], acc[0]);
    part_st<true>(&part2[2 * blockIdx.x + 1], acc[1]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  double a2[2] = {0.0, 0.0};
  for (int b = threadIdx.x; b < c.nblk; b += 256) {
    a2[0] += part_ld<true>(&part2[2 * b]);
    a2[1] += part_ld<true>(&part2[2 * b + 1]);
  }
  __syncthreads();  // red is reused
  block_sum<2>(a2, red);
  if (threadIdx.x == 0) {
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double gtd = a2[0];
    st[LB_GTD] = gtd;
    stop = gtd > -c.tol_x;
    if (stop) {  // cannot make progress along d (reference optimizers.py:224)
      st[LB_ACTIVE] = 0.0;
      st[LB_REASON] = (double)LB_R_GTD;
    } else {
      st[LB_T] = tnext;
      st[LB_DT1] = a2[1] * tnext;
      st[LB_FOLD] = st[LB_F];
    }
  }
  __syncthreads();
  if (stop) {  // undo the speculative step: x stays where the reference leaves it
    // every block stored x_prev / x write-through and drained them before its ticket (vmcnt(0)
    // above): sc1 loads see them, sc1 stores overwrite the speculative x in memory
    for (int j = threadIdx.x; j < c.p; j += 256) {
      const float xo = __hip_atomic_load(&x_prev[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&x[j], xo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ti.fimg != nullptr) scatter_param(xo, j, ti);  // (the images' lines: one block, kernel end)
    }
  }
}

// ---------------------------------------------------------------------------------------------
extern "C" {

int tdq_lbfgs_nst() { return LB_NST; }

// After an evaluation at x (fg = [g | f]): dots -> logic -> dir -> step.
//   part: nchunks * (m + 1) * 5 doubles, part2: 2 * nblk doubles, SY / YY: m * m doubles,
//   coef: 2 m + 1 doubles, S / Y: m * p floats, fhist: fhist_len floats (or null).
int tdq_lbfgs_update(const float* x, const float* fg, float* g_old, float* d, float* S, float* Y, float* best_x,
                     double* st, double* SY, double* YY, double* coef, double* part, double* part2, float* fhist,
                     int p, int m, int max_iter, int nchunks, int nblk, int fhist_len, double max_eval, double lr,
                     double tol_fun, double tol_x, int legacy_stop, void* stream) {
  if (p <= 0 || m < 1 || m > LB_MAXM || nchunks < 1 || nblk < 1) return (int)hipErrorInvalidValue;
  LbCfg c{p, m, max_iter, nchunks, nblk, fhist_len, max_eval, lr, tol_fun, tol_x, legacy_stop};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t lds = lbfgs_logic_lds(m);
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lbfgs_logic_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lbfgs_logic_lds(LB_MAXM));
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(lbfgs_dots_kernel, dim3(nchunks, (m + LB_G) / LB_G), dim3(256), 0, s, fg, g_old, d, S, Y, st, part, c);
  TDQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(lbfgs_logic_kernel, dim3(1), dim3(256), lds, s, fg, part, st, SY, YY, coef, fhist, c);
  TDQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(lbfgs_dir_kernel, dim3(nblk), dim3(256), 0, s, x, fg, g_old, d, S, Y, best_x, st, coef, part2,
                     c);
  TDQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(lbfgs_step_kernel, dim3(1), dim3(256), 0, s, part2, st, c);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// The same update in two launches (lbfgs_dots_logic + lbfgs_dir_step, see above); it also takes
// the step (no tdq_lbfgs_axpy).  ticket: 2 ints, zero on the first call (re-armed by the kernels);
// x_prev: p floats; img (nullable): a TailImg (tdq_img_target) whose images the step also writes.
int tdq_lbfgs_update_fused(float* x, const float* fg, float* g_old, float* d, float* S, float* Y, float* best_x,
                           float* x_prev, double* st, double* SY, double* YY, double* coef, double* part, double* part2,
                           float* fhist, int* ticket, int p, int m, int max_iter, int nchunks, int nblk, int fhist_len,
                           double max_eval, double lr, double tol_fun, double tol_x, int legacy_stop, const void* img,
                           void* stream) {
  if (p <= 0 || m < 1 || m > LB_MAXM || nchunks < 1 || nblk < 1) return (int)hipErrorInvalidValue;
  TailImg ti{};
  if (img != nullptr) {
    ti = *reinterpret_cast<const TailImg*>(img);
    if (param_count(ti.d) != p) return (int)hipErrorInvalidValue;  // images of another network
  }
  LbCfg c{p, m, max_iter, nchunks, nblk, fhist_len, max_eval, lr, tol_fun, tol_x, legacy_stop};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t lds = lbfgs_logic_lds(m);
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lbfgs_dots_logic_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lbfgs_logic_lds(LB_MAXM));
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(lbfgs_dots_logic_kernel, dim3(nchunks, (m + LB_G) / LB_G), dim3(256), lds, s, fg, g_old, d, S, Y, st, part, SY,
                     YY, coef, fhist, ticket, c);
  TDQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(lbfgs_dir_step_kernel, dim3(nblk), dim3(256), 0, s, x, fg, g_old, d, S, Y, best_x, x_prev, st,
                     coef, part2, ticket + 1, c, ti);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// x += t d (a no-op once the run has stopped)
int tdq_lbfgs_axpy(float* x, const float* d, const double* st, int p, int nblk, void* stream) {
  if (p <= 0 || nblk < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(lbfgs_axpy_kernel, dim3(nblk), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), x, d, st, p);
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
