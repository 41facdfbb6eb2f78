// Cost of the "last block runs the tail" hand-off (lbfgs.hip lbfgs_dots_logic / lbfgs_dir_step)
// as a function of the grid size: N workgroups x 256 threads that
//   empty    return at once (the launch + drain floor);
//   part     store 5 fp64 partials write-through (agent scope) and drain them;
//   ticket   part + one agent-scope atomic add on ONE word (the last block re-arms it);
//   tree     part + an atomic add on one of G words (one 128-B line each); the last block of a
//            group adds on the top word; the last of those re-arms everything.
// Each variant is captured 200 times into a HIP graph and replayed; us per launch reported.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void __launch_bounds__(256) k_empty(double*, int*, int) {}

__device__ __forceinline__ void store_part(double* part) {
  if (threadIdx.x == 0)
    for (int q = 0; q < 5; ++q)
      __hip_atomic_store(&part[blockIdx.x * 5 + q], (double)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(256) k_part(double* part, int*, int) {
  store_part(part);
  if (threadIdx.x == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void __launch_bounds__(256) k_ticket(double* part, int* ticket, int) {
  __shared__ int last;
  store_part(part);
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// groups of blocks b with b % G == g; counters 32 ints (128 B) apart; top at index 32 G
__global__ void __launch_bounds__(256) k_tree(double* part, int* cnt, int G) {
  __shared__ int last;
  store_part(part);
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int g = blockIdx.x % G, n = (int)gridDim.x;
    const int gs = n / G + (g < n % G ? 1 : 0);
    int l = 0;
    const int t = __hip_atomic_fetch_add(&cnt[32 * g], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gs - 1) {
      __hip_atomic_store(&cnt[32 * g], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int ng = n < G ? n : G;
      const int t2 = __hip_atomic_fetch_add(&cnt[32 * G], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t2 == ng - 1) {
        __hip_atomic_store(&cnt[32 * G], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        l = 1;
      }
    }
    last = l;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) part[0] = 1.0;
}

typedef void (*KFn)(double*, int*, int);

static int run(const char* name, KFn fn, int n, int G, double* part, int* cnt, hipStream_t s) {
  hipGraph_t g;
  hipGraphExec_t ge;
  const int reps = 200;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(fn, dim3(n), dim3(256), 0, s, part, cnt, G);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int it = 0; it < 6; ++it) {
    CHK(hipEventRecord(a, s));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (it > 0 && ms < best) best = ms;
  }
  printf("%-7s N=%5d G=%3d  %7.2f us/launch\n", name, n, G, best * 1000.f / reps);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return 0;
}

int main() {
  double* part;
  int* cnt;
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  CHK(hipMalloc(&part, 4096 * 5 * sizeof(double)));
  CHK(hipMalloc(&cnt, 32 * 65 * sizeof(int)));
  CHK(hipMemset(cnt, 0, 32 * 65 * sizeof(int)));
  const int ns[] = {13, 64, 169, 256, 512, 663, 783, 1024, 2048};
  for (int n : ns) {
    if (run("empty", k_empty, n, 1, part, cnt, s)) return 1;
    if (run("part", k_part, n, 1, part, cnt, s)) return 1;
    if (run("ticket", k_ticket, n, 1, part, cnt, s)) return 1;
    for (int G : {8, 16, 32, 64})
      if (G < n && run("tree", k_tree, n, G, part, cnt, s)) return 1;
  }
  CHK(hipStreamSynchronize(s));
  int h[32 * 65];
  CHK(hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 32 * 65; ++i) bad += h[i] != 0;
  printf("counters re-armed: %s\n", bad ? "NO" : "yes");
  return 0;
}
