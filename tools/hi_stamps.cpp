// Diagnostic: phase timestamps of the high-order jet kernels (csrc/jet_hi.hip built with
// -DHI_STAMPS into this one program; workgroup 0 prints s_memtime deltas).  AC-baseline shape:
// 402 points, [2, 128 x 4, 1], univariate chain of order 4.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DHI_STAMPS -I tensordiffeq_amd/csrc \
//         tools/hi_stamps.cpp -o tools/hi_stamps
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../tensordiffeq_amd/csrc/jet_hi.hip"

int main() {
  const int N = 402, d_in = 2, d_out = 1, L = 4;
  const int widths[L] = {128, 128, 128, 128};
  const int P = d_in * 128 + 128 + 3 * (128 * 128 + 128) + 128 + 1;
  std::vector<float> hX(N * d_in), hP(P);
  srand(1);
  for (auto& v : hX) v = 2.f * rand() / RAND_MAX - 1.f;
  for (auto& v : hP) v = 0.2f * (2.f * rand() / RAND_MAX - 1.f);
  // streams (), (0), (0,0), (0,0,0), (0,0,0,0); the two highest written / seeded (rows 0, 1)
  std::vector<int> si = {5, 0, 1, 2, 3, 4, 0, 0, 0, 0, 0, -1, -1, -1, 0, 1, 0};
  std::vector<float> sc;
  float *X, *Pd, *J, *Z, *work, *grad;
  const int64_t nz = tdq_jet_hi_scratch_floats(N, L), nw = tdq_jet_hi_work_floats(N, d_in, widths, d_out, L);
  hipMalloc(&X, sizeof(float) * hX.size());
  hipMalloc(&Pd, sizeof(float) * P);
  hipMalloc(&J, sizeof(float) * 2 * N);
  hipMalloc(&Z, sizeof(float) * nz);
  hipMalloc(&work, sizeof(float) * nw);
  hipMalloc(&grad, sizeof(float) * P);
  hipMemcpy(X, hX.data(), sizeof(float) * hX.size(), hipMemcpyHostToDevice);
  hipMemcpy(Pd, hP.data(), sizeof(float) * P, hipMemcpyHostToDevice);
  hipMemset(J, 0, sizeof(float) * 2 * N);
  for (int it = 0; it < 3; ++it) {
    int rc = tdq_jet_hi_fwd(X, N, Pd, d_in, widths, d_out, L, si.data(), sc.data(), J, N, 0, Z, nullptr);
    if (rc) { printf("fwd rc %d\n", rc); return 1; }
    rc = tdq_jet_hi_bwd(X, N, Pd, d_in, widths, d_out, L, si.data(), sc.data(), J, N, 0, Z, work, grad, nullptr);
    if (rc) { printf("bwd rc %d\n", rc); return 1; }
    hipDeviceSynchronize();
  }
  printf("ok\n");
  return 0;
}
