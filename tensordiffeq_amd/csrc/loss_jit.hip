// Host side of the specialized fused-loss kernels (tensordiffeq_amd/ops/loss_jit.py).
//
// The fused loss interpreter (loss_fused.hip) decodes one bytecode instruction per step with its
// SSA registers in LDS: per point a chain of scalar code loads, a switch and two LDS round trips per
// op.  On the AC-SA step that is 11-16 us per launch on MI355X, and each point range's launch sits
// between its forward and its backward on the critical path.  A loss program is fixed once
// compile() has traced it, so ops/loss_jit.py emits it as straight-line HIP C++ (registers become
// VGPR locals, constants literals, the group table compile-time branches) and this file compiles
// it at run time with hipRTC for the device's gfx950 target, loads the code object and launches it
// with the interpreter's grid and block mapping - every block, output and summation order is the
// interpreter's, so the two agree bit for bit (tests/test_loss_jit_gpu.py).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

extern "C" {

// Compile `src` for `arch` (e.g. "gfx950") with the options `opts` (space-separated; nullptr: the
// fused-loss kernels' set below).  On success *code (malloc'ed, free with tdq_rtc_free) holds the
// code object of *size bytes.  log: the compiler log (truncated to log_len); returns 0 or a nonzero
// hipRTC / HIP error code.
int tdq_rtc_compile_ex(const char* src, const char* name, const char* arch, const char* opts, void** code,
                       long long* size, char* log, int log_len) {
  *code = nullptr;
  *size = 0;
  if (log_len > 0) log[0] = 0;
  hiprtcProgram prog;
  hiprtcResult r = hiprtcCreateProgram(&prog, src, name, 0, nullptr, nullptr);
  if (r != HIPRTC_SUCCESS) return 1000 + (int)r;
  char archopt[64];
  snprintf(archopt, sizeof(archopt), "--offload-arch=%s", arch);
  // default: statement-level FMA contraction only (a*b + c inside one statement, as in the
  // interpreter's statements, never across the SSA temporaries it keeps in LDS) and fp32 division /
  // sqrt correctly rounded, as hipcc compiles the interpreter
  const char* dflt = "-O3 -std=c++17 -ffp-contract=on -fhip-fp32-correctly-rounded-divide-sqrt";
  char buf[512];
  snprintf(buf, sizeof(buf), "%s", opts != nullptr ? opts : dflt);
  const char* ov[24];
  int no = 0;
  ov[no++] = archopt;
  for (char* t = strtok(buf, " "); t != nullptr && no < 24; t = strtok(nullptr, " ")) ov[no++] = t;
  r = hiprtcCompileProgram(prog, no, ov);
  size_t lsz = 0;
  if (hiprtcGetProgramLogSize(prog, &lsz) == HIPRTC_SUCCESS && lsz > 1 && log_len > 1) {
    char* lb = (char*)malloc(lsz);
    if (lb != nullptr && hiprtcGetProgramLog(prog, lb) == HIPRTC_SUCCESS) {
      strncpy(log, lb, (size_t)log_len - 1);
      log[log_len - 1] = 0;
    }
    free(lb);
  }
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return 1000 + (int)r;
  }
  size_t csz = 0;
  r = hiprtcGetCodeSize(prog, &csz);
  if (r != HIPRTC_SUCCESS || csz == 0) {
    hiprtcDestroyProgram(&prog);
    return 1000 + (int)r;
  }
  void* out = malloc(csz);
  if (out == nullptr) {
    hiprtcDestroyProgram(&prog);
    return (int)hipErrorOutOfMemory;
  }
  r = hiprtcGetCode(prog, (char*)out);
  hiprtcDestroyProgram(&prog);
  if (r != HIPRTC_SUCCESS) {
    free(out);
    return 1000 + (int)r;
  }
  *code = out;
  *size = (long long)csz;
  return 0;
}

int tdq_rtc_compile(const char* src, const char* name, const char* arch, void** code, long long* size, char* log,
                    int log_len) {
  return tdq_rtc_compile_ex(src, name, arch, nullptr, code, size, log, log_len);
}

void tdq_rtc_free(void* p) { free(p); }

// Load a code object and look up `name`: *module / *func for tdq_rtc_unload / the launchers.
int tdq_rtc_load(const void* code, const char* name, void** module, void** func) {
  hipModule_t m;
  hipError_t e = hipModuleLoadData(&m, code);
  if (e != hipSuccess) return (int)e;
  hipFunction_t f;
  e = hipModuleGetFunction(&f, m, name);
  if (e != hipSuccess) {
    hipModuleUnload(m);
    return (int)e;
  }
  *module = (void*)m;
  *func = (void*)f;
  return 0;
}

// write a pointer into a run-time compiled module's extern "C" __device__ pointer variable
int tdq_rtc_set_global_ptr(void* module, const char* name, void* value) {
  hipDeviceptr_t p = nullptr;
  size_t bytes = 0;
  hipError_t e = hipModuleGetGlobal(&p, &bytes, (hipModule_t)module, name);
  if (e != hipSuccess) return (int)e;
  if (bytes != sizeof(void*)) return (int)hipErrorInvalidValue;
  return (int)hipMemcpyHtoD(p, &value, sizeof(void*));
}

int tdq_rtc_unload(void* module) { return (int)hipModuleUnload((hipModule_t)module); }

// One launch of a specialized loss kernel over blocks [blk0, blk0 + nblk) (128 threads each, the
// interpreter's block mapping); signature of the generated kernel:
//   (const float* J, const float* X, float* dJ, float* partials, const LFPtrs* ptrs, int blk0)
int tdq_loss_jit_range(void* func, const float* J, const float* X, float* dJ, float* partials, const void* ptrs,
                       int blk0, int nblk, void* stream) {
  if (func == nullptr || nblk < 1 || blk0 < 0) return (int)hipErrorInvalidValue;
  void* args[] = {(void*)&J, (void*)&X, (void*)&dJ, (void*)&partials, (void*)&ptrs, (void*)&blk0};
  return (int)hipModuleLaunchKernel((hipFunction_t)func, (unsigned)nblk, 1, 1, 128, 1, 1, 0,
                                    reinterpret_cast<hipStream_t>(stream), args, nullptr);
}

}  // extern "C"
