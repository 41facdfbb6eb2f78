// Host side of the one-launch training step (jet_fused.h; the kernel itself is generated per loss
// program and compiled with hipRTC, ops/fused_step.py): its LDS size, and the device's CU count
// that sizes its grid.
#include "jet_fused.h"
#include "jet_fused3.h"

int fz_cus() {
  static const int n = [] {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cu < 1)
      cu = 256;
    return cu;
  }();
  return n;
}

extern "C" {

// LDS bytes of a fused-step workgroup, -1 if the network is not one the kernel takes (width 128,
// 2-3 MFMA hidden layers, S <= 4).  lo = 0: the bf16 step (jet_fused.h, 32-point tiles); lo = 1:
// the bf16x3 objective (jet_fused3.h, 16-point tiles).
int tdq_jet_fused_lds(int d_in, const int* widths, int d_out, int n_hidden, int S, int lo) {
  NetDims d;
  if (!make_dims(d, d_in, widths, 0, d_out, n_hidden) || lo < 0 || lo > 1) return -1;
  const int WT = width_tiles(d.width), LM = d.n_hidden - 1;
  if (WT != 8 || S < 1 || S > 4 || LM < 2 || LM > 3 || !d.uniform || d.width != 16 * WT || d.d_out != 1) return -1;
  return lo ? (int)fz3_lds_bytes(d, WT, S, LM) : (int)fz_lds_bytes(d, WT, S, LM);
}

// compute units of the current device (the fused step's workgroup count)
int tdq_device_cus() { return fz_cus(); }

}  // extern "C"
