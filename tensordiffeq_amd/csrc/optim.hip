// Fused optimizer-side kernels for gfx950.
//
// tdq_adam_multi: one launch updates up to 16 tensors with the Keras/TF ResourceApplyAdam
//   formula (reference models.py:49-50 -> TF 2.4 Adam):
//     m <- b1 m + (1-b1) g ; v <- b2 v + (1-b2) g^2 ;
//     p <- p - lr sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)
//   with g multiplied by the group's sign (-1 = gradient ascent for self-adaptive weights,
//   reference fit.py:136-141).  The step counter t is read from device memory, so the launch
//   is replayable inside a captured HIP graph.  float4 vector path + scalar tail per group.
// tdq_best_track: snapshot the flat parameters when the step's loss improves (two tiny
//   kernels: copy-if-improved, then the scalar update, so no block races on best_loss).
// tdq_step_book: ONE single-thread kernel per step for all scalar bookkeeping - history row
//   [loss, terms...] at the device epoch, best-loss / best-epoch update and the "improved" flag,
//   every Adam step counter += 1, epoch += 1.  The Adam kernel then snapshots theta into the
//   best-weights buffer (before its update) when the flag is set, so best tracking costs no
//   extra launch.
#include "optim_common.h"

__global__ void __launch_bounds__(256) adam_multi_kernel(AdamArgs args, const int* __restrict__ improved,
                                                          float* __restrict__ snap) {
  const bool do_snap = snap != nullptr && *improved != 0;  // group 0 only
  const int64_t total = args.start[args.ngroups];
  for (int64_t slot = (int64_t)blockIdx.x * 256 + threadIdx.x; slot < total;
       slot += (int64_t)gridDim.x * 256) {
    const int gi = adam_group_of(args, slot);
    const AdamGroup gr = args.grp[gi];
    const int64_t e0 = (slot - args.start[gi]) * 4;
    const float sg = gr.sign, b1 = gr.b1, b2 = gr.b2, eps = gr.eps;
    const float lr_t = adam_lr_t(gr);
    const bool aligned = ((((uintptr_t)gr.p) | ((uintptr_t)gr.g) | ((uintptr_t)gr.m) | ((uintptr_t)gr.v)) & 15) == 0;
    if (aligned && e0 + 4 <= gr.n) {
      f32x4 p = *reinterpret_cast<const f32x4*>(gr.p + e0);
      if (do_snap && gi == 0) *reinterpret_cast<f32x4*>(snap + e0) = p;
      const f32x4 g = *reinterpret_cast<const f32x4*>(gr.g + e0);
      f32x4 m = *reinterpret_cast<const f32x4*>(gr.m + e0);
      f32x4 v = *reinterpret_cast<const f32x4*>(gr.v + e0);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float pc = p[c], mc = m[c], vc = v[c];
        adam_elem(pc, sg * g[c], mc, vc, b1, b2, eps, lr_t);
        p[c] = pc; m[c] = mc; v[c] = vc;
      }
      *reinterpret_cast<f32x4*>(gr.p + e0) = p;
      *reinterpret_cast<f32x4*>(gr.m + e0) = m;
      *reinterpret_cast<f32x4*>(gr.v + e0) = v;
    } else {
      for (int c = 0; c < 4; ++c) {
        const int64_t e = e0 + c;
        if (e < gr.n) {
          if (do_snap && gi == 0) snap[e] = gr.p[e];
          adam_elem(gr.p[e], sg * gr.g[e], gr.m[e], gr.v[e], b1, b2, eps, lr_t);
        }
      }
    }
  }
}

__global__ void __launch_bounds__(256) best_copy_kernel(const float* __restrict__ loss,
                                                         const float* __restrict__ best_loss,
                                                         const float* __restrict__ flat,
                                                         float* __restrict__ best_flat, int64_t n) {
  const float lv = *loss;
  if (!(lv < *best_loss)) return;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    best_flat[i] = flat[i];
}

__global__ void best_scalar_kernel(const float* __restrict__ loss, float* __restrict__ best_loss,
                                   int64_t* __restrict__ best_epoch, const int64_t* __restrict__ epoch) {
  const float lv = *loss;
  if (lv < *best_loss) {
    *best_loss = lv;
    *best_epoch = *epoch;
  }
}

__global__ void step_book_kernel(float* __restrict__ loss, const float* __restrict__ terms, int n_terms, int sum_terms,
                                 float* __restrict__ hist, int64_t hist_rows, int64_t* __restrict__ epoch,
                                 float* __restrict__ best_loss, int64_t* __restrict__ best_epoch,
                                 int* __restrict__ improved, Counters cnt) {
  step_book_body(loss, terms, n_terms, sum_terms, hist, hist_rows, epoch, best_loss, best_epoch, improved, cnt);
}

extern "C" {

int tdq_abi_version() { return 27; }

int tdq_step_book(float* loss, const float* terms, int n_terms, int sum_terms, float* hist, int64_t hist_rows,
                  int64_t* epoch, float* best_loss, int64_t* best_epoch, int* improved, double* const* counters,
                  int ncnt, void* stream) {
  if (ncnt < 0 || ncnt > TDQ_MAX_COUNTERS) return (int)hipErrorInvalidValue;
  Counters c;
  c.n = ncnt;
  for (int i = 0; i < TDQ_MAX_COUNTERS; ++i) c.c[i] = i < ncnt ? counters[i] : nullptr;
  hipLaunchKernelGGL(step_book_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), loss, terms,
                     n_terms, sum_terms, hist, hist_rows, epoch, best_loss, best_epoch, improved, c);
  TDQ_CHECK_LAUNCH();
  return 0;
}

// groups carry their own lr / b1 / b2 / eps / step-counter pointer.  improved / snap: optional
// (nullptr) best-weights snapshot of group 0 before its update
int tdq_adam_multi(const void* groups, int ngroups, const int* improved, float* snap, void* stream) {
  AdamArgs args;
  if (!adam_args_fill(args, reinterpret_cast<const AdamGroup*>(groups), ngroups)) return (int)hipErrorInvalidValue;
  const int64_t total = args.start[ngroups];
  if (total == 0) return 0;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), args, improved, snap);
  TDQ_CHECK_LAUNCH();
  return 0;
}

int tdq_best_track(const float* loss, float* best_loss, const float* flat, float* best_flat,
                   int64_t* best_epoch, const int64_t* epoch, int64_t n, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(best_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, st, loss, best_loss, flat,
                     best_flat, n);
  TDQ_CHECK_LAUNCH();
  hipLaunchKernelGGL(best_scalar_kernel, dim3(1), dim3(1), 0, st, loss, best_loss, best_epoch, epoch);
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
