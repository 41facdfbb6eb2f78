// Write-bandwidth probe for the jet forward's saved-activation stream (tools/gpu_runs/r3_d.sh).
// The forward kernel writes 217 MB per AC-SA step (rocprofv3 WRITE_SIZE, profiles/r3_pmc_bf16.txt)
// in 57 us; this measures what a pure store stream of the same size and shape reaches: 782
// workgroups x 256 threads, each wave writing its own contiguous region with 16-B (value stream)
// or 8-B (bf16 derivative streams) per lane buffer stores, default or non-temporal policy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <int BYTES, int POL>
__global__ void __launch_bounds__(256) store_kernel(char* out, size_t per_wave, int reps) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* base = out + ((size_t)blockIdx.x * 4 + w) * per_wave;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  const int n = (int)(per_wave / (64 * BYTES));
  float acc = (float)l;
  for (int i = 0; i < n; ++i) {
    acc = acc * 1.0001f + 1.f;  // a little VALU per store, like an epilogue
    if constexpr (BYTES == 16) {
      u32x4 v = {__float_as_uint(acc), (unsigned)i, (unsigned)l, 7u};
      __builtin_amdgcn_raw_buffer_store_b128(v, r, l * 16, i * 1024, POL);
    } else {
      u32x2 v = {__float_as_uint(acc), (unsigned)i};
      __builtin_amdgcn_raw_buffer_store_b64(v, r, l * 8, i * 512, POL);
    }
  }
}

template <int BYTES, int POL>
float run(char* buf, size_t total, int nwg) {
  const size_t per_wave = total / ((size_t)nwg * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((store_kernel<BYTES, POL>), dim3(nwg), dim3(256), 0, 0, buf, per_wave, 1);
  hipEventRecord(a);
  const int iters = 20;
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((store_kernel<BYTES, POL>), dim3(nwg), dim3(256), 0, 0, buf, per_wave, 1);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / iters;
}

int main() {
  const size_t total = 217ull << 20;  // the forward's saved-activation bytes per step
  char* buf = nullptr;
  if (hipMalloc(&buf, total + (1 << 20)) != hipSuccess) return 1;
  const int nwgs[] = {782, 1564, 256};
  for (int nwg : nwgs) {
    const float t16 = run<16, 0>(buf, total, nwg), t16n = run<16, 2>(buf, total, nwg);
    const float t8 = run<8, 0>(buf, total, nwg), t8n = run<8, 2>(buf, total, nwg);
    std::printf("{\"wgs\": %d, \"MB\": %.0f, \"us_b128\": %.1f, \"us_b128_nt\": %.1f, \"us_b64\": %.1f, "
                "\"us_b64_nt\": %.1f, \"TBps_b128_nt\": %.2f}\n", nwg, total / 1048576.0, t16, t16n, t8, t8n,
                total / (t16n * 1e-6) / 1e12);
  }
  hipFree(buf);
  return 0;
}
