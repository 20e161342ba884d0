// One-shot peer-memory all-reduce over xGMI for the data-parallel GBDT stage histograms (SURVEY.md
// §5.8 R1: "IPC-mapped peer buffers let each GPU read/write its peers' histograms directly over
// all 7 links"; the reference's GBC, train_ensemble_public.py:45, has no distributed path).
//
// Every rank owns one uncached device buffer, IPC-shared with every other rank of the node:
//     recv [W ranks][3 slots][cap] int64   — rank r's contribution to slot k lands in recv[r][k]
//     flag [3 slots][W ranks][nchunk] u32  — epoch of the last contribution of rank r, chunk c
// xgmi_allreduce_i64 (grid = chunks of the payload, 256 threads each): a block
//   1. writes its chunk of the local slot into recv[me][k] of EVERY rank (remote 8-byte stores
//      over the peer links, one chunk per block, all blocks in flight at once),
//   2. drains its stores (system-scope release) and stores its epoch into flag[k][me][c] of every
//      rank (one lane per destination),
//   3. polls its own flag[k][r][c] for r = 0..W−1 (one lane per source, relaxed system-scope loads,
//      s_sleep between polls, bounded by an s_memrealtime deadline — the fixed 100 MHz clock, not
//      the DVFS-scaled shader clock — that sets *err),
//   4. after a system-scope acquire sums recv[r][k][chunk] over r and writes the total back into
//      the local slot.
// int64 sums are exact, so the result is bit-identical to RCCL's all-reduce and to one process.
// Slots rotate with the stage index (period 3, like the stage kernel's comm slots): a rank can be
// at most one stage ahead of another in writing, so a slot is never overwritten while still read.
// Epochs are the global stage sequence number (strictly increasing per process, equal on all
// ranks), so flags never need resetting.  No RCCL call is made per stage.
#include <cstring>

#include "common.h"

namespace hfens {

constexpr int kXgThreads = 256;
constexpr long long kXgChunk = 2048;   // int64 per block (16 KiB; mirrored in parallel/xgmi.py)
constexpr int kXgMaxRanks = 16;

typedef __attribute__((address_space(1))) unsigned xg_gu32_t;

__device__ __forceinline__ unsigned xg_load_sys(const unsigned* p) {
  return __hip_atomic_load((xg_gu32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void xg_store_sys(unsigned* p, unsigned v) {
  __hip_atomic_store((xg_gu32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// T = long long (exact sums) or double (sum / max / min folded in RANK order 0 … W−1: every rank
// computes the same bits, deterministic for a fixed world; the row-sharded interior point's
// reductions, svc_lowrank._Red).  OP: 0 sum, 1 max, 2 min.
template <typename T, int OP>
__device__ __forceinline__ T xg_fold(T a, T b) {
  if constexpr (OP == 0) return a + b;
  else if constexpr (OP == 1) return a > b ? a : b;
  else return a < b ? a : b;
}

template <typename T, int OP>
__global__ __launch_bounds__(kXgThreads) void xgmi_allreduce_kernel(T* __restrict__ local,
                                                                    long long count,
                                                                    long long* const* __restrict__ peers,
                                                                    int W, int me, int k, long long cap,
                                                                    int nchunk, unsigned epoch_base,
                                                                    int t_host, const int* __restrict__ t_dev,
                                                                    unsigned* __restrict__ err,
                                                                    long long spin_ticks) {
  static_assert(sizeof(T) == 8, "8-byte elements (the receive slots are int64-sized)");
  const int c = blockIdx.x, tid = threadIdx.x;
  const long long beg = (long long)c * kXgChunk;
  const long long end = min(count, beg + kXgChunk);
  // epoch = stage sequence number: the graph-replayed loop reads the stage from device memory
  // (already ticked past this stage), the eager loop passes it
  const unsigned epoch = epoch_base + (unsigned)(t_dev != nullptr ? *t_dev : t_host + 1);
  const size_t recv_slot = (size_t)k * cap;
  auto flags_of = [&](long long* base) {
    return reinterpret_cast<unsigned*>(base + (size_t)W * 3 * cap);
  };
  // 1. push this chunk to every rank (the comm slots of the stage kernel are 8-byte aligned only:
  //    8-byte stores, 512 B per wave instruction; the chunk's values are loaded once)
  constexpr int kPer = (int)(kXgChunk / kXgThreads);
  T v[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const long long i = beg + tid + (long long)q * kXgThreads;
    v[q] = i < end ? local[i] : T(0);
  }
  for (int p = 0; p < W; ++p) {
    T* dst = reinterpret_cast<T*>(peers[p] + (size_t)me * 3 * cap + recv_slot);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const long long i = beg + tid + (long long)q * kXgThreads;
      if (i < end) dst[i] = v[q];
    }
  }
  // 2. every storing wave drains its stores, system-scope release, then one lane per rank flags it
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (tid < W) xg_store_sys(flags_of(peers[tid]) + ((size_t)k * W + me) * nchunk + c, epoch);
  // 3. wait for every rank's chunk c (one lane per source rank)
  __shared__ int s_fail;
  if (tid == 0) s_fail = 0;
  __syncthreads();
  if (tid < W) {
    const unsigned* f = flags_of(peers[me]) + ((size_t)k * W + tid) * nchunk + c;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (xg_load_sys(f) != epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > spin_ticks) {
        atomicOr(err, 1u);
        s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (s_fail) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  // 4. the fold over the ranks, in rank order, back into the local slot (int64 sums: exact)
  const T* recv = reinterpret_cast<const T*>(peers[me] + recv_slot);
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const long long i = beg + tid + (long long)q * kXgThreads;
    if (i < end) {
      T s = recv[i];
      for (int r = 1; r < W; ++r) s = xg_fold<T, OP>(s, recv[(size_t)r * 3 * cap + i]);
      local[i] = s;
    }
  }
}

// ---- host side ------------------------------------------------------------------------------
// out[0] = device pointer of a zeroed allocation of `bytes` bytes (IPC-shareable): uncached
// (every access bypasses the caches: the only form the peer path uses across GPUs) or, uncached =
// 0, plain device memory (tests only)
void xgmi_alloc(long long bytes, int uncached, uintptr_t out) {
  void* p = nullptr;
  if (uncached) HFENS_CHECK(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached));
  else HFENS_CHECK(hipMalloc(&p, (size_t)bytes));
  HFENS_CHECK(hipMemset(p, 0, (size_t)bytes));
  HFENS_CHECK(hipDeviceSynchronize());
  *reinterpret_cast<uintptr_t*>(out) = reinterpret_cast<uintptr_t>(p);
}

void xgmi_free(uintptr_t p) { HFENS_CHECK(hipFree(reinterpret_cast<void*>(p))); }

// out: host buffer of sizeof(hipIpcMemHandle_t) (64) bytes
void xgmi_ipc_handle(uintptr_t p, uintptr_t out) {
  hipIpcMemHandle_t h;
  HFENS_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(p)));
  std::memcpy(reinterpret_cast<void*>(out), &h, sizeof(h));
}

void xgmi_ipc_open(uintptr_t handle, uintptr_t out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, reinterpret_cast<const void*>(handle), sizeof(h));
  void* p = nullptr;
  HFENS_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  *reinterpret_cast<uintptr_t*>(out) = reinterpret_cast<uintptr_t>(p);
}

void xgmi_ipc_close(uintptr_t p) { HFENS_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(p))); }

// All-reduce of `count` 8-byte elements at `local` (dtype 0: int64, 1: f64; op 0 sum, 1 max, 2 min —
// int64 supports sum only) over the W ranks whose buffers `peers` (device array of W base pointers,
// this rank's own at index me) points to; slot k rotates with the call sequence (period 3).
void xgmi_allreduce(uintptr_t local, long long count, int dtype, int op, uintptr_t peers, int W, int me, int k,
                    long long cap, long long epoch_base, int t_host, uintptr_t t_dev, uintptr_t err, double timeout_s,
                    uintptr_t stream) {
  HFENS_REQUIRE(W >= 1 && W <= kXgMaxRanks && me >= 0 && me < W, "xgmi_allreduce: 1 <= W <= 16, 0 <= me < W");
  HFENS_REQUIRE(k >= 0 && k < 3 && count >= 0 && count <= cap, "xgmi_allreduce: slot 0..2, count <= cap");
  HFENS_REQUIRE((local & 7) == 0, "xgmi_allreduce: the local buffer must be 8-byte aligned");
  HFENS_REQUIRE((dtype == 0 && op == 0) || (dtype == 1 && op >= 0 && op <= 2),
                "xgmi_allreduce: int64 sum, or f64 sum / max / min");
  if (count == 0) return;
  const int nchunk = (int)((cap + kXgChunk - 1) / kXgChunk);
  const int grid = (int)((count + kXgChunk - 1) / kXgChunk);
  const long long ticks = (long long)(timeout_s * 1.0e8);   // s_memrealtime: fixed 100 MHz
  auto go = [&](auto kern, auto* loc) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kXgThreads), 0, as_stream(stream), loc, count,
                       reinterpret_cast<long long* const*>(peers), W, me, k, cap, nchunk, (unsigned)epoch_base, t_host,
                       reinterpret_cast<const int*>(t_dev), reinterpret_cast<unsigned*>(err), ticks);
  };
  if (dtype == 0) go(xgmi_allreduce_kernel<long long, 0>, reinterpret_cast<long long*>(local));
  else if (op == 0) go(xgmi_allreduce_kernel<double, 0>, reinterpret_cast<double*>(local));
  else if (op == 1) go(xgmi_allreduce_kernel<double, 1>, reinterpret_cast<double*>(local));
  else go(xgmi_allreduce_kernel<double, 2>, reinterpret_cast<double*>(local));
  launch_check();
}

void xgmi_allreduce_i64(uintptr_t local, long long count, uintptr_t peers, int W, int me, int k, long long cap,
                        long long epoch_base, int t_host, uintptr_t t_dev, uintptr_t err, double timeout_s,
                        uintptr_t stream) {
  xgmi_allreduce(local, count, 0, 0, peers, W, me, k, cap, epoch_base, t_host, t_dev, err, timeout_s, stream);
}

}  // namespace hfens
