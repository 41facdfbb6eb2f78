// Host-side sanitizer driver (SURVEY.md §5 "race detection / sanitizers"; GPU ASan and xnack+
// are not available on the MI355X pool, so the host half of the native library is checked on the
// CPU).  Built by tools/asan_host_check.py with every HIP source compiled host-only
// (--offload-host-only) and -Xarch_host -fsanitize=address,undefined; no kernel is launched: the
// driver exercises the host code paths - geometry / plan validation of every entry point (they
// must reject bad arguments BEFORE any launch), scratch / slab sizing over a sweep of geometries,
// stream-spec parsing, the Adam group packing - so out-of-bounds host accesses, overflows in the
// size arithmetic and undefined behaviour surface here.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "jet_bf3.h"
#include "optim_common.h"

// stubs for the kernel instantiation tables (jet_bf3_w*.hip, not part of this build): only
// reached when an entry point accepted its arguments - which no call below does
#define TDQ_STUB(name) \
  int name(int, int, const Bf3Args&) { return (int)hipErrorNotSupported; }
TDQ_STUB(bf3_fwd_w2)
TDQ_STUB(bf3_fwd_w4)
TDQ_STUB(bf3_fwd_w8)
TDQ_STUB(bf3_bwd_w2)
TDQ_STUB(bf3_bwd_w4)
TDQ_STUB(bf3_bwd_w8)

extern "C" {
int64_t tdq_jet_bf3_scratch_floats(int N, int d_in, const int* widths, int n_hidden, int S, int lo);
int64_t tdq_jet_bf3_slab_floats(int N, int d_in, const int* widths, int d_out, int n_hidden);
int64_t tdq_jet_scratch_floats(int N, int width, int n_hidden, int S, int unused);
int64_t tdq_jet_slab_floats(int N, int d_in, int width, int d_out, int n_hidden);
int tdq_jet_fwd_bf3(const float* X, const float* P, float* J, float* scratch, int N, int d_in, const int* widths, int d_out,
                    int n_hidden, int S, const int* spec, int lo, void* stream);
int tdq_jet_bwd_bf3(const float* X, const float* P, const float* dJ, const float* Hs, float* work, float* grad, int N,
                    int d_in, const int* widths, int d_out, int n_hidden, int S, const int* spec, int lo, void* stream);
int tdq_dp_tail_a_bf3(float* work, float* grad, int N, int d_in, const int* widths, int d_out, int n_hidden, int S, int lo,
                      const float* lpart, int n_lblocks, int n_terms, int n_scal, float* losses, float* dscal,
                      float* total, int c_first, const float* gx, int rows, int half_ovr, void* stream);
int tdq_lbfgs_update_fused(float* x, const float* fg, float* g_old, float* d, float* S, float* Y, float* best_x,
                           float* x_prev, double* st, double* SY, double* YY, double* coef, double* part, double* part2,
                           float* fhist, int* ticket, int p, int m, int max_iter, int nchunks, int nblk, int fhist_len,
                           double max_eval, double lr, double tol_fun, double tol_x, int legacy_stop, void* stream);
int tdq_loss_meta_sizes(int* out);
int tdq_abi_version();
}

static int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      ++fails;                                                      \
    }                                                               \
  } while (0)

int main() {
  CHECK(tdq_abi_version() > 0);
  // scratch / slab sizing: positive, monotone in N, no overflow up to 10M points
  for (int width : {16, 20, 32, 50, 64, 100, 128})
    for (int S = 1; S <= 8; ++S)
      for (int lo = 0; lo < 2; ++lo) {
        int64_t prev = 0;
        const int ws[4] = {width, width, width / 2 + 1, width};  // unequal hidden widths too
        for (int N : {1, 63, 64, 65, 1000, 50000, 10000000}) {
          const int64_t a = tdq_jet_bf3_scratch_floats(N, 3, ws, 4, S, lo);
          if (width <= 16) {
            CHECK(a == -1);
            continue;
          }
          CHECK(a > 0 && a >= prev);
          prev = a;
          CHECK(tdq_jet_bf3_slab_floats(N, 3, ws, 1, 4) > 0);
        }
        CHECK(tdq_jet_scratch_floats(1000, width, 3, S, 0) > 0);
        CHECK(tdq_jet_slab_floats(1000, 2, width, 1, 3) > 0);
      }
  // stream specs: canonical order, second-order factors must be first-order streams
  int spec_ok[] = {0, 0, 0, 1, 0, 0, 1, 1, 0, 2, 1, 2};  // u, u_x, u_t, u_xt
  JetSpec sp;
  CHECK(make_spec(4, spec_ok, sp) && spec_nso(4, spec_ok) == 1);
  int spec_bad[] = {0, 0, 0, 2, 1, 1, 1, 0, 0};  // second order before its factor
  CHECK(spec_nso(3, spec_bad) == -1);
  int spec_bad2[] = {0, 0, 0, 2, 0, 7};  // factor index out of range
  CHECK(!make_spec(2, spec_bad2, sp));
  CHECK(!make_spec(9, spec_ok, sp) && !make_spec(0, spec_ok, sp));
  // entry points reject bad geometry before launching anything (dummy device pointers)
  std::vector<float> dummy(64);
  float* f = dummy.data();
  const int w128[4] = {128, 128, 128, 128}, w300[4] = {300, 300, 300, 300};
  CHECK(tdq_jet_bf3_scratch_floats(100, 2, w128, 17, 4, 0) == -1);  // more than TDQ_MAXL layers
  CHECK(tdq_jet_fwd_bf3(f, f, f, f, 100, 2, w128, 1, 4, 9, spec_ok, 0, nullptr) != 0);   // S = 9
  CHECK(tdq_jet_fwd_bf3(f, f, f, f, 100, 2, w300, 1, 4, 4, spec_ok, 0, nullptr) != 0);   // width 300
  CHECK(tdq_jet_fwd_bf3(f, f, f, f, 100, 9, w128, 1, 4, 4, spec_ok, 0, nullptr) != 0);   // d_in 9
  CHECK(tdq_jet_fwd_bf3(f, f, f, f, 100, 2, w128, 5, 4, 4, spec_ok, 0, nullptr) != 0);   // d_out 5
  CHECK(tdq_jet_fwd_bf3(f, f, f, f, 100, 2, w128, 1, 4, 3, spec_bad, 0, nullptr) != 0);  // bad spec
  CHECK(tdq_jet_fwd_bf3(f, f, f, f, 0, 2, w128, 1, 4, 4, spec_ok, 0, nullptr) == 0);     // N = 0: no-op
  CHECK(tdq_jet_bwd_bf3(f, f, f, f, f, f, 100, 2, w128, 1, 0, 4, spec_ok, 1, nullptr) != 0);  // no hidden layer
  CHECK(tdq_dp_tail_a_bf3(f, f, 100, 2, w128, 1, 4, 9, 0, f, 1, 1, 0, f, f, f, 0, nullptr, 0, -1, nullptr) != 0);
  CHECK(tdq_dp_tail_a_bf3(f, f, 0, 2, w128, 1, 4, 4, 0, f, 1, 1, 0, f, f, f, 0, nullptr, 0, -1, nullptr) != 0);
  double* dd = reinterpret_cast<double*>(f);
  int tk[2] = {0, 0};
  CHECK(tdq_lbfgs_update_fused(f, f, f, f, f, f, f, f, dd, dd, dd, dd, dd, dd, f, tk, 100, 65, 10, 1, 1, 0, 12.5,
                               0.8, 1e-12, 1e-12, 1, nullptr) != 0);  // history > 64
  int sizes[8] = {0};
  CHECK(tdq_loss_meta_sizes(sizes) == 0 && sizes[0] > 0);
  // Adam group packing: prefix sums of float4 slots, limits
  std::vector<AdamGroup> g(TDQ_MAX_GROUPS + 1);
  double t = 1.0;
  for (size_t i = 0; i < g.size(); ++i) g[i] = AdamGroup{f, f, f, f, (int64_t)(i * 7 + 1), 1.f, 1e-3f, .9f, .999f,
                                                        1e-7f, 0.f, &t};
  AdamArgs args;
  CHECK(adam_args_fill(args, g.data(), TDQ_MAX_GROUPS, false));
  CHECK(args.start[TDQ_MAX_GROUPS] > args.start[0]);
  CHECK(!adam_args_fill(args, g.data(), TDQ_MAX_GROUPS + 1, false));
  CHECK(!adam_args_fill(args, g.data(), 0, false));
  std::printf("host check: %d failure(s)\n", fails);
  return fails ? 1 : 0;
}
