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
#include <cstdlib>

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
  LB_TS0 = 18,    // 18..23: phase stamps (LbCfg::ts): kernel start (block 0), then sums of
                  // the shader clock cycles over the logic, its step 1, steps 2-3, step 4-5 (100 MHz
                  // ticks), and the count
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
  int ts;           // TDQ_LBFGS_TS=1 (fused path): phase stamps of the dots + logic kernel summed into
                    //    st[LB_TS0 ..] (tools/prof_lbfgs.py --ts)
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

// "Am I the last block?" for the fused kernels' hand-off, as a two-level tree of arrival counters:
// block b adds on counter b % LB_TG (one 128-B line each), the block completing a group adds on the
// top counter, and the block completing the top runs the tail; every completed counter is re-armed
// by the block that completed it.  One counter for the whole grid serialises every block's atomic
// at one address: 7.7 us at 663 blocks, 9.0 us at 783, against ~1.3 us for this tree with 32
// groups (tools/microbench/ticket_cost.hip, profiles/r6bg_ticket_cost.txt).  Thread 0 only, after
// its partial stores have drained; the counters: LB_TCNT ints.
#define LB_TG 32
#define LB_TCNT (32 * (LB_TG + 1))
__device__ __forceinline__ bool last_block(int* cnt, int b, int n) {
  const int g = b % LB_TG, ng = n < LB_TG ? n : LB_TG;
  const int gs = n / LB_TG + (g < n % LB_TG ? 1 : 0);
  if (__hip_atomic_fetch_add(&cnt[32 * g], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gs - 1) return false;
  __hip_atomic_store(&cnt[32 * g], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__hip_atomic_fetch_add(&cnt[32 * LB_TG], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ng - 1) return false;
  __hip_atomic_store(&cnt[32 * LB_TG], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

__device__ __forceinline__ bool slot_valid(int i, int head, int k, int m) { return ((i - head + m) % m) < k; }

// d_j = cG g_j + sum_q (cS_q s_qj + cY_q y_qj) over the k history pairs (chronological q): the
// four waves of a direction block share one 64-element tile, wave w sums the pairs of quarter w
// (at most LB_MAXM / 4, every load of it in flight together), and wave 0 adds the quarters in
// fixed order.  Shared by both update paths (same summation order, so the same bits).
__device__ __forceinline__ double dir_quarter(const float* __restrict__ S, const float* __restrict__ Y,
                                              const double* coef, int j, int p, int k, int head, int m,
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
// R^{-1} (R = the upper triangle of S^T Y in chronological order, as below) is kept current by one
// new column per push: dropping the oldest pair leaves the inverse of the remaining block as the
// lower-right block of the old inverse, and bordering R with the new column c (c_i = s_i.y_new)
// and diagonal d = s_new.y_new gives the new column -R^{-1} c / d and the diagonal 1 / d.  The two
// triangular solves of the compact product become matrix-vector products, whose steps do not
// depend on each other (a substitution step waits on the previous one: 7.5 us of the update at
// k = 50 on one wave, profiles/r6bk_lbfgs_solve_stamps.txt).  R^{-1} shares the YY buffer with
// Y^T Y: for physical slots a, b with a older than b, Y^T Y's entry sits at [a][b] and R^{-1}'s at
// [b][a]; the diagonal is Y^T Y's (R^{-1}'s is 1 / R[a][a]).  So the LDS image stays at two
// matrices (a third one cost the fused dots part its occupancy, profiles/r6bp_lbfgs_rinv_packed.txt).
//
// dynamic LDS (doubles): dots[(m+1)*5] | SYl[m*m] | YRl[m*m] | vecl[64] | red[256]
__host__ __device__ inline size_t lbfgs_logic_lds(int m) {
  return ((size_t)(m + 1) * LB_NF + 2 * (size_t)m * m + 64 + 256) * 8;
}

template <bool SC1>
__device__ __forceinline__ void lbfgs_logic_body(const float* __restrict__ fg, const double* __restrict__ part,
                                                 double* __restrict__ st, double* __restrict__ SY,
                                                 double* __restrict__ YY, double* __restrict__ coef,
                                                 float* __restrict__ fhist, const LbCfg& c, double* lb_lds) {
  const int tid = threadIdx.x, m = c.m, mm = m * m;
  double* dots = lb_lds;
  double* SYl = dots + (m + 1) * LB_NF;
  double* YYl = SYl + mm;  // Y^T Y and R^{-1} (lbfgs_logic_lds)
  double* vecl = YYl + mm;
  double* red = vecl + 64;
  const unsigned long long ts1 = c.ts ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const unsigned long long mt1 = c.ts ? __builtin_amdgcn_s_memtime() : 0ull;  // shader clock cycles
  // the scalar state, loaded first: its latency overlaps step 1's
  const double f = (double)fg[c.p];
  int n_iter = (int)st[LB_NITER];
  const double fe0 = st[LB_FEVAL], dt1 = st[LB_DT1], fold = st[LB_FOLD], hd_old = st[LB_HDIAG];
  double minloss = st[LB_MINLOSS];
  int k = (int)st[LB_K], head = (int)st[LB_HEAD];
  // 1. copy S^T Y / Y^T Y + R^{-1} into LDS and reduce the chunk partials (fixed order: deterministic)
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
      // sixteen loads in flight per round (one round up to 16 chunks); even chunks into a0, odd
      // into a1, each in increasing order (the summation order of every earlier version)
      for (int ch = 0; ch < c.nchunks; ch += 16) {
        double q[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          q[u] = part_ld<SC1>(&part[(size_t)min(ch + u, c.nchunks - 1) * (m + 1) * LB_NF + v]);
#pragma unroll
        for (int u = 0; u < 16; u += 2) {
          if (ch + u < c.nchunks) a0 += q[u];
          if (ch + u + 1 < c.nchunks) a1 += q[u + 1];
        }
      }
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
  // the scalar logic below is evaluated by every thread (uniform values, thread 0 stores, every
  // early return uniform); per-pair values with one lane of each wave per history pair (lane j =
  // chronological pair j), wave 0 storing them; the matrix-vector products split their sums over
  // the four waves
  const unsigned long long ts2 = c.ts ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int lane = tid & 63, w = tid >> 6;
  const bool L0 = tid == 0, W0 = w == 0;
  // 2. post-evaluation tests of the previous step (reference optimizers.py:241-296, with the
  //    B9 fixes of eager_lbfgs), then the curvature test and ring push (optimizers.py:168-185)
  const double* sc = dots + m * LB_NF;  // s.y, y.y, s.g, y.g, |g|_1
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
  if (W0 && pushed && lane < m && slot_valid(lane, head, k, m)) {
    const int j = lane;
    const double* dj = dots + j * LB_NF;
    const double snj = j == slot ? ys : dj[4], sjn = j == slot ? ys : dj[2], yj = j == slot ? yy : dj[3];
    SY[slot * m + j] = snj;  // s_new . y_j
    SY[j * m + slot] = sjn;  // s_j . y_new
    YY[j * m + slot] = yj;  // j older than the new pair ([slot][j] holds R^{-1}[j][new], step 4)
    SYl[slot * m + j] = snj;
    SYl[j * m + slot] = sjn;
    YYl[j * m + slot] = yj;
  }
  if (n_iter == 1 || k == 0) {  // d = -H0 g (first iteration: H0 = I)
    if (W0)
      for (int v = lane; v < 2 * m; v += 64) coef[v] = 0.0;
    if (L0) coef[2 * m] = -gam;
    return;
  }
  __syncthreads();  // the patched rows / columns
  const unsigned long long ts3 = c.ts ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // 4. compact product (lane j = chronological pair j, physical slot ij):
  //    R u = S^T g ; rhs = D u + gam Y^T Y u - gam Y^T g ; R^T p1 = rhs ;
  //    H g = gam g + S p1 - gam Y u   ->   d = -H g
  //    R = upper triangle of S^T Y in chronological order, R^{-1} kept current (RIl, see
  //    lbfgs_logic_lds): u = R^{-1} S^T g and p1 = R^{-T} rhs are matrix-vector products.
  const int j = lane;
  const bool jv = j < k;
  int ij = head + j;
  if (ij >= m) ij -= m;
  ij = jv ? ij : 0;
  const double rjj = SYl[ij * m + ij];
  const bool nwj = pushed && ij == slot;
  const double rdj = jv ? 1.0 / rjj : 0.0;  // R^{-1}[j][j]
  // sum over q in [qa, qb) of A(j, q) * vec[q], vec[q] = `val` of lane q; A by the pairs' order:
  //   sel 0: R^{-1}[j][q], q >= j   (at [iq][ij], q > j)
  //   sel 1: R^{-1}[q][j], q <= j   (at [ij][iq], q < j)
  //   sel 2: Y^T Y[j][q]            (at [iq][ij] for q < j, [ij][iq] for q > j, the diagonal)
  // Wave w sums its quarter of [0, k) - operands of four pairs loaded ahead of their products,
  // the vector read as an LDS broadcast - and every wave adds the four partials in fixed order.
  auto mv = [&](int sel, double val, int qa, int qb) {
    if (W0) vecl[lane] = val;
    __syncthreads();
    const int q0 = (w * k) >> 2, q1 = ((w + 1) * k) >> 2;
    int iq = head + q0;
    if (iq >= m) iq -= m;
    double a0 = 0.0, a1 = 0.0;
    for (int q = q0; q < q1; q += 4) {
      double av[4], bv[4];
      int ip = iq;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int qq = q + t < q1 ? q + t : q, pq = q + t < q1 ? ip : iq;
        const bool below = sel == 0 || (sel == 2 && qq < j);  // [iq][ij] rather than [ij][iq]
        av[t] = YYl[below ? pq * m + ij : ij * m + pq];
        bv[t] = vecl[qq];
        ip = ip + 1 == m ? 0 : ip + 1;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int qq = q + t;
        const double a = (sel != 2 && qq == j) ? rdj : av[t];
        const double v = (qq < q1 && qq >= qa && qq < qb) ? a * bv[t] : 0.0;
        if (t & 1) a1 += v;
        else a0 += v;
      }
      iq = ip;
    }
    red[tid] = a0 + a1;
    __syncthreads();
    const double r = ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
    __syncthreads();  // red and vecl are rewritten by the next product
    return r;
  };
  if (pushed) {  // the new pair's column of R^{-1} (chronological k-1; c_q = SYl[q][slot] = s_q.y_new)
    const double cq = (jv && j < k - 1) ? SYl[ij * m + slot] : 0.0;
    const double v = mv(0, cq, j, k - 1);
    if (W0 && j < k - 1) {  // R^{-1}[j][new] at [slot][ij]; the diagonal 1 / ys is 1 / rjj
      const double ri = -v / ys;
      YYl[slot * m + ij] = ri;
      YY[slot * m + ij] = ri;
    }
    __syncthreads();
  }
  const double r0 = jv ? (nwj ? dots[m * LB_NF + 2] : dots[ij * LB_NF + 0]) : 0.0;  // s_j . g
  // u = R^{-1} r0: u_j = sum_{q >= j} RI[j][q] r0_q
  const double u = mv(0, r0, j, k);
  // rhs = R[j][j] u_j + gam (Y^T Y u)_j - gam y_j.g
  const double yu = mv(2, jv ? u : 0.0, 0, k);
  const double bj = jv ? (nwj ? dots[m * LB_NF + 3] : dots[ij * LB_NF + 1]) : 0.0;  // y_j . g
  const double rr = jv ? rjj * u + gam * yu - gam * bj : 0.0;
  // p1 = R^{-T} rr: p1_j = sum_{q <= j} RI[q][j] rr_q
  const double p1 = mv(1, rr, 0, j + 1);
  // 5. per PHYSICAL slot
  if (!W0) return;
  if (jv) {
    coef[ij] = -p1;
    coef[m + ij] = gam * u;
  }
  for (int v = lane; v < m; v += 64)
    if (((v - head + m) % m) >= k) coef[v] = coef[m + v] = 0.0;
  if (L0) coef[2 * m] = -gam;
  if (SC1 && c.ts && L0) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const unsigned long long ts4 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long mt4 = __builtin_amdgcn_s_memtime();
    st[LB_TS0 + 1] += (double)(mt4 - mt1);  // shader clock cycles over [ts1, ts4]
    st[LB_TS0 + 2] += (double)(ts2 - ts1);
    st[LB_TS0 + 3] += (double)(ts3 - ts2);
    st[LB_TS0 + 4] += (double)(ts4 - ts3);
    st[LB_TS0 + 5] += 1.0;
  }
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
  // the pair coefficients staged in LDS: read as uniform scalar loads they were fetched one at a
  // time (each result spilled before the next load could issue: ~11 us of a 15.5 us launch)
  __shared__ double cf[2 * LB_MAXM + 1];
  if ((int)threadIdx.x <= 2 * c.m) cf[threadIdx.x] = coef[threadIdx.x];
  __syncthreads();
  const bool best = st[LB_BEST] != 0.0, active = st[LB_ACTIVE] != 0.0;
  const int n_iter = (int)st[LB_NITER], pushed = (int)st[LB_PUSHED], slot = (int)st[LB_SLOT];
  const int k = (int)st[LB_K], head = (int)st[LB_HEAD], m = c.m;
  const float tf = (float)st[LB_T];
  const double cG = cf[2 * m];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // w: wave-uniform
  double acc[2] = {0.0, 0.0};
  for (int jb = blockIdx.x * 64; jb < c.p; jb += gridDim.x * 64) {
    const int j = jb + l;
    const bool in = j < c.p;
    const int jc = in ? j : c.p - 1;  // unconditional loads: all in flight before the first use
    const float g = fg[jc], dj = d[jc], oj = g_old[jc], xj = x[jc];
    // branch-free (k = 0 before the first push: every pair masked; rows stay in range)
    const double qv = dir_quarter(S, Y, cf, jc, c.p, k, head, m, pushed, slot, tf, g, dj, oj, w);
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
//                     for them, and arrives on the counter tree (last_block); the block that
//                     arrives last runs the logic on the partials (sc1 loads).  (Hand-off protocol:
//                     MI355X_MICROARCH.md, inter-workgroup table row 1.)
//   lbfgs_dir_step    the direction pass, plus the step taken speculatively: t of the NEXT step
//                     is known before g.d is (min(1, 1/|g|_1) on the first iteration, else the
//                     fixed lr), so every element does x += t d right after computing d (old x
//                     kept in x_prev); the last-arriving block reduces g.d / |d|_1 and runs the
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
  if (c.ts && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    __hip_atomic_store(&st[LB_TS0], (double)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  lbfgs_dots_body<true>(fg, g_old, d, S, Y, st, part, c, red);
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's sc1 partial stores have landed
    last = last_block(ticket, (int)(blockIdx.y * gridDim.x + blockIdx.x), (int)(gridDim.x * gridDim.y));
  }
  __syncthreads();
  if (!last) return;
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
  // the pair coefficients staged in LDS: read as uniform scalar loads they were fetched one at a
  // time (each result spilled before the next load could issue: ~11 us of a 15.5 us launch)
  __shared__ double cf[2 * LB_MAXM + 1];
  if ((int)threadIdx.x <= 2 * c.m) cf[threadIdx.x] = coef[threadIdx.x];
  __syncthreads();
  __shared__ int last, stop;
  const bool best = st[LB_BEST] != 0.0, active = st[LB_ACTIVE] != 0.0;
  const int n_iter = (int)st[LB_NITER], pushed = (int)st[LB_PUSHED], slot = (int)st[LB_SLOT];
  const int k = (int)st[LB_K], head = (int)st[LB_HEAD], m = c.m;
  const float tf = (float)st[LB_T];
  // the next step's length (the five-launch lbfgs_step_kernel's formula)
  const double tnext = (n_iter == 1) ? fmin(1.0, 1.0 / st[LB_G1]) : c.lr;
  const float tn = (float)tnext;
  const double cG = cf[2 * m];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;  // w: wave-uniform
  double acc[2] = {0.0, 0.0};
  for (int jb = blockIdx.x * 64; jb < c.p; jb += gridDim.x * 64) {
    const int j = jb + l;
    const bool in = j < c.p;
    const int jc = in ? j : c.p - 1;  // unconditional loads: all in flight before the first use
    const float g = fg[jc], dj = d[jc], oj = g_old[jc], xj = x[jc];
    // branch-free (k = 0 before the first push: every pair masked; rows stay in range)
    const double qv = dir_quarter(S, Y, cf, jc, c.p, k, head, m, pushed, slot, tf, g, dj, oj, w);
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
    last = last_block(ticket, (int)blockIdx.x, (int)gridDim.x);
  }
  __syncthreads();
  if (!last) return;
  double a2[2] = {0.0, 0.0};
  // blocks b = tid, tid + 256, ... in increasing order; the coherent (atomic) loads of four of them
  // issued together - one after the other they cost a memory latency each
  for (int b0 = threadIdx.x; b0 < c.nblk; b0 += 1024) {
    double v0[4], v1[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int b = min(b0 + 256 * t, c.nblk - 1);
      v0[t] = part_ld<true>(&part2[2 * b]);
      v1[t] = part_ld<true>(&part2[2 * b + 1]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (b0 + 256 * t < c.nblk) {
        a2[0] += v0[t];
        a2[1] += v1[t];
      }
  }
  __syncthreads();  // red is reused
  block_sum<2>(a2, red);
  if (threadIdx.x == 0) {
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
int tdq_lbfgs_ticket_ints() { return LB_TCNT; }

// After an evaluation at x (fg = [g | f]): dots -> logic -> dir -> step.
//   part: nchunks * (m + 1) * 5 doubles, part2: 2 * nblk doubles, SY / YY: m * m doubles (YY holds
//   Y^T Y and R^{-1}, lbfgs_logic_lds),
//   coef: 2 m + 1 doubles, S / Y: m * p floats, fhist: fhist_len floats (or null).
int tdq_lbfgs_update(const float* x, const float* fg, float* g_old, float* d, float* S, float* Y, float* best_x,
                     double* st, double* SY, double* YY, double* coef, double* part, double* part2, float* fhist,
                     int p, int m, int max_iter, int nchunks, int nblk, int fhist_len, double max_eval, double lr,
                     double tol_fun, double tol_x, int legacy_stop, void* stream) {
  if (p <= 0 || m < 1 || m > LB_MAXM || nchunks < 1 || nblk < 1) return (int)hipErrorInvalidValue;
  LbCfg c{p, m, max_iter, nchunks, nblk, fhist_len, max_eval, lr, tol_fun, tol_x, legacy_stop, 0};
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
// the step (no tdq_lbfgs_axpy).  ticket: 2 tdq_lbfgs_ticket_ints() ints, zero on the first call
// (re-armed by the kernels);
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
  LbCfg c{p, m, max_iter, nchunks, nblk, fhist_len, max_eval, lr, tol_fun, tol_x, legacy_stop, 0};
  {
    const char* e = getenv("TDQ_LBFGS_TS");
    c.ts = e != nullptr && e[0] == '1';
  }
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
                     coef, part2, ticket + LB_TCNT, c, ti);
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
