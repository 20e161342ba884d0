// Shared helpers for the hfens gfx950 (CDNA4) kernels.
// Wave = 64 lanes everywhere; no CUDA shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace hfens {

constexpr int kWave = 64;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define HFENS_CHECK(expr)                                                                  \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                 \
  } while (0)

#define HFENS_REQUIRE(cond, msg)                                   \
  do {                                                            \
    if (!(cond)) throw std::invalid_argument(std::string(msg));   \
  } while (0)

inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

inline void launch_check() { HFENS_CHECK(hipGetLastError()); }

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// ---- wave reductions (64 lanes) ---------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// max of (value, index) with lowest-index tie-break
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, kWave);
    int oi = __shfl_xor(i, o, kWave);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}
__device__ __forceinline__ void wave_argmin(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, kWave);
    int oi = __shfl_xor(i, o, kWave);
    if (ov < v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

// Broadcast lane `l` (wave-uniform) of a value: v_readlane_b32 into an SGPR — far cheaper than
// a ds_bpermute shuffle when every lane wants the same source lane.
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float readlane_f32(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Wave-wide u32 max on DPP + CDNA4 half-swaps (no LDS round trips): quad_perm xor 1 / xor 2,
// row_half_mirror (8), row_mirror (16), v_permlane16_swap (32), v_permlane32_swap (64).
// Every lane receives the result.
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
  v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = max((unsigned)r[0], (unsigned)r[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return max((unsigned)q[0], (unsigned)q[1]);
}

// order-preserving f32 ↔ u32 (larger float ⇒ larger key; finite floats map to ≥ 0x00800000)
__device__ __forceinline__ unsigned f32_okey(float x) {
  const unsigned u = __float_as_uint(x);
  return u ^ ((u >> 31) ? 0xFFFFFFFFu : 0x80000000u);
}
__device__ __forceinline__ float f32_from_okey(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}

// order-preserving f64 ↔ u64
__device__ __forceinline__ unsigned long long f64_okey(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  return u ^ ((u >> 63) ? ~0ull : 0x8000000000000000ull);
}
__device__ __forceinline__ double f64_from_okey(unsigned long long k) {
  return __longlong_as_double((long long)((k >> 63) ? (k ^ 0x8000000000000000ull) : ~k));
}

// exact wave max of doubles: order-preserving u64 key, max of the high words, then of the low
// words among the lanes holding that high word
__device__ __forceinline__ double wave_max_f64_exact(double x) {
  unsigned long long u = (unsigned long long)__double_as_longlong(x);
  u ^= (u >> 63) ? ~0ull : 0x8000000000000000ull;
  const unsigned hi = (unsigned)(u >> 32), lo = (unsigned)u;
  const unsigned mh = wave_max_u32(hi);
  const unsigned ml = wave_max_u32(hi == mh ? lo : 0u);
  unsigned long long k = ((unsigned long long)mh << 32) | ml;
  k = (k >> 63) ? (k ^ 0x8000000000000000ull) : ~k;
  return __longlong_as_double((long long)k);
}

__device__ __forceinline__ float fast_exp(float x) {  // e^x via v_exp_f32 (2^x)
  return __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
}

// XCD-aware bijective block remap (8 XCDs; blocks b and b+8 share an XCD under
// round-robin dispatch).  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int nx = 8;
  if (nblk < nx) return bid;
  int q = nblk / nx, r = nblk % nx, x = bid % nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / nx;
}

}  // namespace hfens
