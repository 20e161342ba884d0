// Batched inference of stump ensembles on binned inputs (SURVEY.md §2.3 K12 tree_apply, BASELINE
// config 5 "deep ensemble": 1000 trees × 5 seeds).
//
// Every split of a histogram-trained tree sits on a bin boundary, so for depth-1 trees the whole
// ensemble of model b folds EXACTLY into one table per feature:
//     raw_b(x) = init_b + Σ_f T_b[f][bin_f(x)],   T_b[f][k] = lr·Σ_{stumps t on f} v_t(k ≤ blo_t)
// — 1000 stumps become F (≤ 64) LDS lookups per row, independent of the tree count.  The table of
// one model (F × 256 f32 ≤ 64 KB) is staged in LDS per workgroup; rows arrive feature-major as the
// binner emits them ([F][n] u8), four consecutive rows per lane via one 32-bit load per feature.
#include "common.h"

namespace hfens {

__global__ __launch_bounds__(256) void binned_stump_raw_kernel(const unsigned char* __restrict__ bins, long long n,
                                                               int F, const float* __restrict__ tables,
                                                               const double* __restrict__ init,
                                                               float* __restrict__ out) {
  extern __shared__ float tab[];   // [F][256]
  const int b = blockIdx.y;
  const float* tb = tables + (size_t)b * F * 256;
  for (int i = threadIdx.x; i < F * 256; i += blockDim.x) tab[i] = tb[i];
  __syncthreads();
  const float base = (float)init[b];
  const long long n4 = (n + 3) / 4;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (long long)gridDim.x * blockDim.x) {
    const long long i0 = 4 * q;
    float r0 = base, r1 = base, r2 = base, r3 = base;
    if (i0 + 3 < n && (n & 3) == 0) {
      for (int f = 0; f < F; ++f) {
        const unsigned v = *reinterpret_cast<const unsigned*>(bins + (size_t)f * n + i0);
        const float* tf = tab + f * 256;
        r0 += tf[v & 0xFF];
        r1 += tf[(v >> 8) & 0xFF];
        r2 += tf[(v >> 16) & 0xFF];
        r3 += tf[v >> 24];
      }
    } else {
      for (int f = 0; f < F; ++f) {
        const unsigned char* col = bins + (size_t)f * n;
        const float* tf = tab + f * 256;
        r0 += tf[col[i0]];
        if (i0 + 1 < n) r1 += tf[col[i0 + 1]];
        if (i0 + 2 < n) r2 += tf[col[i0 + 2]];
        if (i0 + 3 < n) r3 += tf[col[i0 + 3]];
      }
    }
    float* o = out + (size_t)b * n + i0;
    o[0] = r0;
    if (i0 + 1 < n) o[1] = r1;
    if (i0 + 2 < n) o[2] = r2;
    if (i0 + 3 < n) o[3] = r3;
  }
}

void binned_stump_raw(uintptr_t bins, long long n, int F, uintptr_t tables, int B, uintptr_t init, uintptr_t out,
                      uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "binned_stump_raw: 1 <= F <= 64");
  if (n == 0 || B == 0) return;
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const long long n4 = (n + 3) / 4;
  long long gx = (n4 + 255) / 256;
  const long long cap = (8LL * ncu + B - 1) / B;   // ≈ 8 workgroups per CU over all models
  if (gx > cap) gx = cap;
  hipLaunchKernelGGL(binned_stump_raw_kernel, dim3((unsigned)gx, B), dim3(256), (size_t)F * 256 * 4,
                     as_stream(stream), (const unsigned char*)bins, n, F, (const float*)tables,
                     (const double*)init, (float*)out);
  launch_check();
}

// ------------------------------------------------------------------------------------------
// K7 quantize_bins: rows [n][F] (f64 or f32, row-major as the pipeline holds them) → feature-major
// u8 bins [F][ldb] against the per-feature +inf-padded edge table (bin = first edge ≥ float32(x),
// clamped to the feature's bin count — torch.searchsorted's left rule).  The edge table sits in
// LDS; each thread bins one row over all features (binary search, ≤ 8 probes), and the stores of
// one feature by consecutive threads are consecutive bytes.
template <typename T>
__global__ __launch_bounds__(256) void quantize_bins_kernel(const T* __restrict__ X, long long n, int F,
                                                            const float* __restrict__ edges, int K,
                                                            const int* __restrict__ nbins,
                                                            unsigned char* __restrict__ out, long long ldb) {
  extern __shared__ float qe[];   // [F][K]
  __shared__ int qnb[128];
  for (int i = threadIdx.x; i < F * K; i += blockDim.x) qe[i] = edges[i];
  for (int i = threadIdx.x; i < F; i += blockDim.x) qnb[i] = nbins[i];
  __syncthreads();
  for (long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long long)gridDim.x * blockDim.x) {
    const T* xr = X + (size_t)r * F;
    for (int f = 0; f < F; ++f) {
      const float x = (float)xr[f];
      const float* e = qe + f * K;
      int lo = 0, hi = K;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (e[mid] < x) lo = mid + 1;
        else hi = mid;
      }
      const int b = lo < qnb[f] - 1 ? lo : qnb[f] - 1;
      out[(size_t)f * ldb + r] = (unsigned char)b;
    }
  }
}

void quantize_bins(uintptr_t X, int f64, long long n, int F, uintptr_t edges, int K, uintptr_t nbins, uintptr_t out,
                   long long ldb, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 128 && K >= 1 && K <= 256, "quantize_bins: F <= 128 features, K <= 256 edges");
  HFENS_REQUIRE(ldb >= n, "quantize_bins: ldb < n");
  if (n == 0) return;
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  long long g = (n + 255) / 256;
  if (g > 8LL * ncu) g = 8LL * ncu;
  const size_t lds = (size_t)F * K * sizeof(float);
  if (f64)
    hipLaunchKernelGGL(quantize_bins_kernel<double>, dim3((unsigned)g), dim3(256), lds, as_stream(stream),
                       (const double*)X, n, F, (const float*)edges, K, (const int*)nbins, (unsigned char*)out, ldb);
  else
    hipLaunchKernelGGL(quantize_bins_kernel<float>, dim3((unsigned)g), dim3(256), lds, as_stream(stream),
                       (const float*)X, n, F, (const float*)edges, K, (const int*)nbins, (unsigned char*)out, ldb);
  launch_check();
}

}  // namespace hfens
