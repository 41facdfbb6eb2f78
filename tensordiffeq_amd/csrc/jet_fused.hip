// Host side of the persistent point-tile jet kernels (jet_fused.h): eligibility, geometry and the
// launches behind the split-bf16 entry points of jet_bf3.hip (tdq_jet_fwd_bf3_range /
// tdq_jet_bwd_bf3_range route here when fz_active), plus direct entry points for tests.
#include <cstdlib>

#include "jet_fused.h"

int fz_dispatch_w8_l1(int mode, int S, int nso, const FzArgs& a);
int fz_dispatch_w8_l2(int mode, int S, int nso, const FzArgs& a);
int fz_dispatch_w8_l3(int mode, int S, int nso, const FzArgs& a);

// TDQ_FUSED=1 selects the persistent kernels, 0 the saved-activation kernels (default while the
// persistent ones are being tuned); read once per process, so the forward, the backward, the
// scratch / slab sizes and the step tails always agree
#ifndef FZ_DEFAULT
#define FZ_DEFAULT 0
#endif
static int g_fz_override = -1;  // tdq_jet_fused_override (tests): 0 / 1, -1 = the environment
static int fz_env() {
  static const int on = [] {
    const char* e = getenv("TDQ_FUSED");
    return e == nullptr ? FZ_DEFAULT : (e[0] == '0' ? 0 : 1);
  }();
  return g_fz_override >= 0 ? g_fz_override : on;
}

bool fz_active(const NetDims& d, int WT, int S, int lo) {
  if (!fz_env() || lo != 0 || WT != 8 || S < 1 || S > 4) return false;
  const int LM = d.n_hidden - 1;
  if (LM < 1 || LM > 3 || !d.uniform || d.width != 16 * WT || d.d_in > TDQ_MAXD || d.d_out > TDQ_MAXO) return false;
  return fz_lds_bytes(d, WT, S, LM, 0) <= 160 * 1024 && fz_lds_bytes(d, WT, S, LM, 1) <= 160 * 1024;
}

static int fz_cus() {
  static const int n = [] {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cu < 1)
      cu = 256;
    return cu;
  }();
  return n;
}

// workgroups (= gradient-slab rows) of a launch over N points: one per CU, at most one per tile
int fz_rows(int N) {
  const int ntiles = (N + FZ_PT - 1) / FZ_PT;
  const int c = fz_cus();
  return ntiles < c ? (ntiles < 1 ? 1 : ntiles) : c;
}

int fz_launch(int mode, const float* X, const float* aux, const bf16x8* fimg, const bf16x8* bimg, const float* dJ,
              float* J, float* slab, int N, int Pst, const NetDims& d, const JetSpec& sp, int S, int nso,
              hipStream_t st) {
  FzArgs a{X, aux, fimg, bimg, dJ, J, slab, N, Pst, fz_rows(N), (N + FZ_PT - 1) / FZ_PT, d, sp, st};
  switch (d.n_hidden - 1) {
    case 1: return fz_dispatch_w8_l1(mode, S, nso, a);
    case 2: return fz_dispatch_w8_l2(mode, S, nso, a);
    case 3: return fz_dispatch_w8_l3(mode, S, nso, a);
    default: return (int)hipErrorInvalidValue;
  }
}

extern "C" {

// 1 when the persistent kernels serve this configuration (fit.point_ranges: no point ranges then)
int tdq_jet_fused_active(int d_in, const int* widths, int d_out, int n_hidden, int S, int lo) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden)) return 0;
  return fz_active(d, width_tiles(d.width), S, lo) ? 1 : 0;
}

int tdq_jet_fused_rows(int N) { return fz_rows(N); }

// LDS bytes of a persistent-kernel workgroup (mode 0 / 1 / 2 of jet_fused.h), -1 if the network is
// not one the kernels take (the run-time compiled fused step declares it statically)
int tdq_jet_fused_lds(int d_in, const int* widths, int d_out, int n_hidden, int S, int mode) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden) || mode < 0 || mode > 2) return -1;
  const int WT = width_tiles(d.width), LM = d.n_hidden - 1;
  if (WT != 8 || S < 1 || S > 4 || LM < 1 || LM > 3 || (mode == 2 && LM < 2) || !d.uniform || d.width != 16 * WT)
    return -1;
  return (int)fz_lds_bytes(d, WT, S, LM, mode);
}

// compute units of the current device (the persistent kernels' workgroup count)
int tdq_device_cus() { return fz_cus(); }

// tests only: force the persistent kernels off (0) / on (1) or back to TDQ_FUSED (-1).  Scratch and
// slab sizes follow the switch, so buffers must be allocated after it (a new model / forward).
int tdq_jet_fused_override(int v) {
  g_fz_override = v < 0 ? -1 : (v ? 1 : 0);
  return 0;
}

}  // extern "C"
