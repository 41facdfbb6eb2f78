// Optimizer-side pieces shared by optim.hip (stand-alone Adam / bookkeeping launches) and the
// fused step tail of the split-bf16 jet kernels (jet_bf3.hip): the multi-tensor Keras-Adam
// argument block, the per-element update and the per-step scalar bookkeeping.
#pragma once
#include "common.h"

#define TDQ_MAX_GROUPS 16
#define TDQ_MAX_COUNTERS 8

// one tensor of the update with its optimizer's hyper-parameters and device step counter, so the
// network (descent) and self-adaptive-weight (ascent) optimizers share one launch
struct AdamGroup {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  float sign;
  float lr, b1, b2, eps;
  float pad;
  const double* t;
};

struct AdamArgs {
  AdamGroup grp[TDQ_MAX_GROUPS];
  int64_t start[TDQ_MAX_GROUPS + 1];  // prefix sums of float4 "slots" per group
  int ngroups;
};

struct Counters {
  double* c[TDQ_MAX_COUNTERS];
  int n;
};

// Keras / TF ResourceApplyAdam (reference models.py:49-50): epsilon-hat form
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1, float b2,
                                          float eps, float lr_t) {
  m = fmaf(1.f - b1, g, b1 * m);
  v = fmaf(1.f - b2, g * g, b2 * v);
  p = p - lr_t * m / (sqrtf(v) + eps);
}

// bias-corrected step size from the group's device step counter (already incremented)
__device__ __forceinline__ float adam_lr_t(const AdamGroup& gr) {
  const double t = *gr.t;
  return (float)((double)gr.lr * sqrt(1.0 - pow((double)gr.b2, t)) / (1.0 - pow((double)gr.b1, t)));
}

__device__ __forceinline__ int adam_group_of(const AdamArgs& args, int64_t slot) {
  int gi = 0;
#pragma unroll
  for (int q = 1; q < TDQ_MAX_GROUPS; ++q)
    if (q < args.ngroups && slot >= args.start[q]) gi = q;
  return gi;
}

// host: fill the argument block (prefix sums of float4 slots, or of elements with per_elem);
// false on a bad group count
static inline bool adam_args_fill(AdamArgs& args, const AdamGroup* src, int ngroups, bool per_elem = false) {
  if (ngroups <= 0 || ngroups > TDQ_MAX_GROUPS) return false;
  args.ngroups = ngroups;
  args.start[0] = 0;
  for (int i = 0; i < TDQ_MAX_GROUPS; ++i) {
    if (i < ngroups) {
      args.grp[i] = src[i];
      args.start[i + 1] = args.start[i] + (per_elem ? src[i].n : (src[i].n + 3) / 4);
    } else {
      args.grp[i] = AdamGroup{nullptr, nullptr, nullptr, nullptr, 0, 1.f, 0.f, 0.f, 0.f, 0.f, 0.f, nullptr};
      args.start[i + 1] = args.start[i];
    }
  }
  return true;
}

// Per-step scalar bookkeeping (one thread): optional total = sum of the terms (fused loss, in
// term order), history row [loss, terms...] at the device epoch, best loss / epoch and the
// "improved" flag (NaN never improves), every Adam step counter += 1, epoch += 1.
__device__ __forceinline__ void step_book_body(float* __restrict__ loss, const float* __restrict__ terms,
                                               int n_terms, int sum_terms, float* __restrict__ hist,
                                               int64_t hist_rows, int64_t* __restrict__ epoch,
                                               float* __restrict__ best_loss, int64_t* __restrict__ best_epoch,
                                               int* __restrict__ improved, const Counters& cnt) {
  float lv = *loss;
  if (sum_terms) {
    lv = 0.f;
    for (int t = 0; t < n_terms; ++t) lv += terms[t];
    *loss = lv;
  }
  const int64_t ep = *epoch;
  if (ep >= 0 && ep < hist_rows) {
    float* row = hist + ep * (1 + n_terms);
    row[0] = lv;
    for (int t = 0; t < n_terms; ++t) row[1 + t] = terms[t];
  }
  const int imp = lv < *best_loss;
  if (imp) {
    *best_loss = lv;
    *best_epoch = ep;
  }
  *improved = imp;
  for (int i = 0; i < cnt.n; ++i) *cnt.c[i] += 1.0;
  *epoch = ep + 1;
}
