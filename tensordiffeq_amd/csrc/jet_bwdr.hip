// Instantiations of the recompute backward (jet_bwdr.h) and its host-side selection.
//
// Selected per geometry when TDQ_BWD_RECOMPUTE is not "0" and the precision is bf16: the forward
// then writes only the jets (no saved activations) and the backward recomputes them on chip.
// Geometries without an instantiation (and bf16x3, whose split operands do not fit the register
// budget) keep the saved-activation pair of jet_bf3.h.
#include "jet_bwdr.h"

#define BWDR_KEY(WT, S, NSO, LH) ((((WT) * 16 + (S)) * 8 + (NSO)) * 32 + (LH))

// (WT, S, hidden layers) geometries with EVERY feasible second-order count instantiated: the slab
// geometry (and so the fused tail) is decided from (WT, S, layers) alone
int bwdr_dispatch(int WT, int S, int nso, int n_hidden, const Bf3Args& a) {
  switch (BWDR_KEY(WT, S, nso, n_hidden)) {
    case BWDR_KEY(8, 4, 0, 4): return launch_bwdr<8, 4, 0, 4>(a);
    case BWDR_KEY(8, 4, 1, 4): return launch_bwdr<8, 4, 1, 4>(a);  // AC-SA / AC-baseline [2,128x4,1]
    default: return -1;
  }
}

static bool bwdr_instantiated(int WT, int S, int n_hidden) {
  switch (BWDR_KEY(WT, S, 0, n_hidden)) {
    case BWDR_KEY(8, 4, 0, 4): return true;
    default: return false;
  }
}

// TDQ_BWD_RECOMPUTE, read once per process (forward, backward, slab geometry and the fused tail
// must agree); tdq_bwdr_set overrides it between steps (tests compare both paths in one process)
static int g_bwdr = -1;
static int bwdr_enabled() {
  if (g_bwdr < 0) {
    const char* e = getenv("TDQ_BWD_RECOMPUTE");
    g_bwdr = (e != nullptr && e[0] == '1') ? 1 : 0;  // opt-in until measured (TDQ_BWD_RECOMPUTE=1)
  }
  return g_bwdr;
}

bool bwdr_active(int WT, int S, int n_hidden, int lo) {
  return bwdr_enabled() && lo == 0 && bwdr_instantiated(WT, S, n_hidden);
}

extern "C" int tdq_bwdr_enabled() { return bwdr_enabled(); }
extern "C" int tdq_bwdr_set(int on) {
  g_bwdr = on ? 1 : 0;
  return 0;
}
// the recompute backward serves this geometry at this precision (lo: 1 = bf16x3)
extern "C" int tdq_bwdr_active(int d_in, const int* widths, int n_hidden, int S, int lo) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, 1, n_hidden)) return 0;
  return bwdr_active(width_tiles(d.width), S, n_hidden, lo) ? 1 : 0;
}
