// Device → pinned-host read-backs written by a kernel on the producer's own stream
// (hfens/utils/hostread.py).
//
// The stacking fit's tail reads a few words back after each of its last kernels (the SMO's early
// read, the Platt pairs, the meta model's error word and guards).  An async D2H copy of a few bytes
// goes through a copy engine that first has to see the compute queue's kernel finish; here the
// words go out as system-scope stores from a one-workgroup kernel queued right behind the producer
// on the same queue, straight into the host's pinned buffer, which the host polls for its sentinel
// (utils/hostread.landed).  Elements are stored whole (4- or 8-byte atomic stores), so a polled
// element is either the sentinel or its final value — never half of an 8-byte value.
#include "common.h"

namespace hfens {

constexpr int kHsThreads = 256;

typedef __attribute__((address_space(1))) unsigned hs_gu32_t;
typedef __attribute__((address_space(1))) unsigned long long hs_gu64_t;

template <typename T>
__global__ __launch_bounds__(kHsThreads) void host_store_kernel(const T* __restrict__ src, T* dst, long long n) {
  for (long long i = (long long)blockIdx.x * kHsThreads + threadIdx.x; i < n; i += (long long)gridDim.x * kHsThreads) {
    const T v = src[i];
    if constexpr (sizeof(T) == 8)
      __hip_atomic_store((hs_gu64_t*)(dst + i), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store((hs_gu32_t*)(dst + i), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// src: device buffer; dst_host: pinned host buffer (hipHostMalloc'd — torch's pinned allocator),
// mapped into the device's address space via hipHostGetDevicePointer; n elements of elem_bytes.
void host_store(uintptr_t src, uintptr_t dst_host, long long n, int elem_bytes, uintptr_t stream) {
  HFENS_REQUIRE(elem_bytes == 4 || elem_bytes == 8, "host_store: 4- or 8-byte elements");
  HFENS_REQUIRE(n >= 0, "host_store: n >= 0");
  if (n == 0) return;
  void* dptr = nullptr;
  HFENS_CHECK(hipHostGetDevicePointer(&dptr, reinterpret_cast<void*>(dst_host), 0));
  const int grid = (int)std::min<long long>((n + kHsThreads - 1) / kHsThreads, 64);
  if (elem_bytes == 8)
    hipLaunchKernelGGL(host_store_kernel<unsigned long long>, dim3(grid), dim3(kHsThreads), 0, as_stream(stream),
                       reinterpret_cast<const unsigned long long*>(src), reinterpret_cast<unsigned long long*>(dptr), n);
  else
    hipLaunchKernelGGL(host_store_kernel<unsigned>, dim3(grid), dim3(kHsThreads), 0, as_stream(stream),
                       reinterpret_cast<const unsigned*>(src), reinterpret_cast<unsigned*>(dptr), n);
  launch_check();
}

}  // namespace hfens
