// One-shot peer-memory all-reduce (SUM, fp32) for data parallelism inside one node.
//
// The per-step DP message of a PINN is small (the AC-SA bucket [grad theta | SA grads | loss terms]
// is ~196 KiB) and the step is short (~0.2 ms), so the collective is latency-bound: a ring
// all-reduce pays 2 (world - 1) link hops of latency.  MI355X nodes connect every GPU pair by its
// own xGMI link, so here every rank PUSHES its bucket straight into a receive slot of every peer
// (world - 1 concurrent point-to-point writes, one link each), raises one flag per (source rank,
// chunk) in the peer's memory, waits for the flags of its own chunks and sums the world copies in
// rank order - one kernel, one hop, and bitwise the same result on every rank (same operands, same
// order).  The kernel is a plain launch on the caller's stream, so it is captured inside the
// step's HIP graph like every other kernel of the step.
//
// Memory (one allocation per rank, exported with hipIpcGetMemHandle, opened by every peer):
//   recv  float    [2 parities][TDQ_PEER_MAXW source ranks][cap]
//   flags unsigned [TDQ_PEER_MAXW source ranks][max_blocks]
// allocated uncached (hipDeviceMallocUncached) so that writes arriving over the fabric are never
// hidden behind a stale line of the receiver's L2; the release / acquire fences are system scope.
// Block b of a call owns floats [b*1024, b*1024+1024).  Every block keeps its own call counter
// seq[b] (local memory, touched only by block b): flags carry seq, the receive slot is picked by
// seq's parity.  A rank reuses a slot parity two calls later only after every peer has signalled
// the call in between, which each peer does only after finishing its reads of that slot - no
// second barrier is needed.  Waits are bounded (TDQ_PEER timeout, s_memrealtime at 100 MHz): a
// peer that never arrives sets err[0] and the kernel drains instead of hanging the GPU.
//
// Reference behaviour: the NCCL all-reduce that MirroredStrategy issues inside apply_gradients
// (tensordiffeq/fit.py:150-224); design: SURVEY.md §5 / §7.2 step 8 (one-shot xGMI all-reduce).
#include "common.h"
#include <string.h>

#define TDQ_PEER_MAXW 8
#define TDQ_PEER_CHUNK 1024  // floats per block: 256 threads x float4

struct PeerPtrs {
  float* recv[TDQ_PEER_MAXW];      // rank q's receive region, mapped into this process
  unsigned* flag[TDQ_PEER_MAXW];   // rank q's flag region, mapped into this process
};

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 load_chunk(const float* p, int i0, int n) {
  if (i0 + 4 <= n) return *reinterpret_cast<const f4*>(p + i0);
  f4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (i0 + c < n) v[c] = p[i0 + c];
  return v;
}

__device__ __forceinline__ void store_chunk(float* p, int i0, int n, f4 v) {
  if (i0 + 4 <= n) {
    *reinterpret_cast<f4*>(p + i0) = v;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (i0 + c < n) p[i0 + c] = v[c];
  }
}

__global__ void __launch_bounds__(256) peer_allreduce_kernel(float* __restrict__ buf, int n, int rank, int world,
                                                               long long cap, int max_blocks, PeerPtrs pp,
                                                               unsigned* __restrict__ seqs, int* __restrict__ err,
                                                               long long timeout_ticks) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int i0 = b * TDQ_PEER_CHUNK + 4 * tid;
  const unsigned seq = seqs[b] + 1u;
  const int par = (int)(seq & 1u);
  const f4 mine = load_chunk(buf, i0, n);
  // push this rank's chunk into slot [par][rank] of every peer (one xGMI link per peer)
  for (int q = 0; q < world; ++q) {
    if (q == rank) continue;
    store_chunk(pp.recv[q] + ((long long)par * TDQ_PEER_MAXW + rank) * cap, i0, n, mine);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's pushes acknowledged
  __syncthreads();
  if (tid < world && tid != rank) {
    // lane q signals peer q: system-scope release (wave-uniform fence, one per block)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(pp.flag[tid] + (long long)rank * max_blocks + b, seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    // then waits for peer q's chunk b in this rank's memory
    unsigned* f = pp.flag[rank] + (long long)tid * max_blocks + b;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout_ticks) {
        err[0] = 1;  // vector store; the host reads it (PeerComm.check)
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // sum the world copies in rank order: identical operands and order on every rank
  const float* slot = pp.recv[rank] + (long long)par * TDQ_PEER_MAXW * cap;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < world; ++r) acc += (r == rank) ? mine : load_chunk(slot + (long long)r * cap, i0, n);
  store_chunk(buf, i0, n, acc);
  if (tid == 0) seqs[b] = seq;
}

extern "C" {

int tdq_peer_maxw() { return TDQ_PEER_MAXW; }
int tdq_peer_chunk() { return TDQ_PEER_CHUNK; }

// Allocate `bytes` of device memory for a peer region.  kind: 0 uncached, 1 fine-grained,
// 2 plain hipMalloc.  Zero-filled.
int tdq_peer_alloc(long long bytes, int kind, void** out) {
  *out = nullptr;
  hipError_t e;
  if (kind == 0)
    e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached);
  else if (kind == 1)
    e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocFinegrained);
  else
    e = hipMalloc(out, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*out, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}

int tdq_peer_free(void* p) { return (int)hipFree(p); }

// 64-byte IPC handle of an allocation (out: 64 bytes)
int tdq_peer_ipc_handle(void* p, void* out) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) == 64, "hipIpcMemHandle_t is 64 bytes");
  memcpy(out, &h, sizeof(h));
  return 0;
}

int tdq_peer_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

int tdq_peer_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

// buf (n floats, in place) += every peer's buf.  recv / flag: arrays of `world` pointers (this
// rank's own entries are its local pointers).  seqs: max_blocks counters, err: 1 int (local).
int tdq_peer_allreduce(float* buf, int n, int rank, int world, long long cap, int max_blocks, void* const* recv,
                       void* const* flag, unsigned* seqs, int* err, long long timeout_ticks, void* stream) {
  if (n <= 0) return 0;
  if (world < 1 || world > TDQ_PEER_MAXW || rank < 0 || rank >= world || (long long)n > cap)
    return (int)hipErrorInvalidValue;
  const int nb = (n + TDQ_PEER_CHUNK - 1) / TDQ_PEER_CHUNK;
  if (nb > max_blocks || (cap % 4) != 0 || (reinterpret_cast<uintptr_t>(buf) & 15) != 0)
    return (int)hipErrorInvalidValue;
  PeerPtrs pp;
  for (int q = 0; q < TDQ_PEER_MAXW; ++q) {
    pp.recv[q] = q < world ? reinterpret_cast<float*>(recv[q]) : nullptr;
    pp.flag[q] = q < world ? reinterpret_cast<unsigned*>(flag[q]) : nullptr;
    if (q < world && (pp.recv[q] == nullptr || pp.flag[q] == nullptr)) return (int)hipErrorInvalidValue;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(peer_allreduce_kernel, dim3(nb), dim3(256), 0, st, buf, n, rank, world, cap, max_blocks, pp,
                     seqs, err, timeout_ticks);
  TDQ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
