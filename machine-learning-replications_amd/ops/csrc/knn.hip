// nan-euclidean 1-NN donor search for KNN imputation (reference
// KNNImputer(n_neighbors=1), train_ensemble_public.py:37-40; distance semantics of sklearn
// nan_euclidean_distances: d² = F/|common| · Σ_{common present} (x−y)²).
//
// One thread owns one receiver row (values in LDS, its ≤ 8 missing-column slots and their running
// (distance, donor) minima in registers).  Donor rows stream through LDS in tiles of 256 rows and
// are read by every thread simultaneously (LDS broadcast).  Per (receiver, donor) pair the
// distance is the direct difference form Σ(x_r − x_d)² over zero-filled rows (no ‖x‖²+‖y‖²−2x·y
// cancellation, so exact ties stay exact) minus the cross-missing corrections, which only loop
// over the set bits of the two 64-bit missing masks.  Tie-break: lowest donor index.
#include "common.h"

namespace hfens {

constexpr int kKnnTile = 256;
constexpr int kKnnSlots = 8;

__global__ __launch_bounds__(256) void knn_donor_kernel(
    const float* __restrict__ R, const unsigned long long* __restrict__ rmask, int nr,
    const float* __restrict__ D, const unsigned long long* __restrict__ dmask, int nd, int F,
    const int* __restrict__ slot_col /*[nr][kKnnSlots] column or −1*/, int* __restrict__ best_idx,
    float* __restrict__ best_dist) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int ld = F | 1;
  float* rs = sm;                                  // [256][ld]  receiver rows
  float* ds = sm + 256 * ld;                       // [256][ld]  donor tile
  unsigned long long* dm = (unsigned long long*)(ds + 256 * ld + ((256 * ld) & 1));  // [256]
  const int r = blockIdx.x * 256 + threadIdx.x;
  for (int e = threadIdx.x; e < 256 * F; e += 256) {
    const int rr = e / F, c = e % F;
    const int gr = blockIdx.x * 256 + rr;
    rs[rr * ld + c] = gr < nr ? R[(size_t)gr * F + c] : 0.f;
  }
  const bool active = r < nr;
  const unsigned long long mr = active ? rmask[r] : 0ull;
  int col[kKnnSlots];
  float bd[kKnnSlots];
  int bi[kKnnSlots];
  int nslot = 0;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k) {
    col[k] = active ? slot_col[(size_t)r * kKnnSlots + k] : -1;
    bd[k] = INFINITY;
    bi[k] = -1;
    if (col[k] >= 0) nslot = k + 1;
  }
  const float* xr = rs + threadIdx.x * ld;
  for (int d0 = 0; d0 < nd; d0 += kKnnTile) {
    __syncthreads();
    const int nt = min(kKnnTile, nd - d0);
    for (int e = threadIdx.x; e < nt * F; e += 256) {
      const int rr = e / F, c = e % F;
      ds[rr * ld + c] = D[(size_t)(d0 + rr) * F + c];
    }
    if (threadIdx.x < nt) dm[threadIdx.x] = dmask[d0 + threadIdx.x];
    __syncthreads();
    if (nslot == 0) continue;
    for (int t = 0; t < nt; ++t) {
      const float* xd = ds + t * ld;
      const unsigned long long md = dm[t];
      // does this donor have any of the receiver's missing columns?  (cheap early-out)
      bool useful = false;
#pragma unroll
      for (int k = 0; k < kKnnSlots; ++k)
        if (col[k] >= 0 && !((md >> col[k]) & 1ull)) useful = true;
      if (!useful) continue;
      float s = 0.f;
      for (int f = 0; f < F; ++f) {
        const float df = xr[f] - xd[f];
        s = fmaf(df, df, s);
      }
      // remove terms where exactly one side is missing (the other side's x² was added)
      unsigned long long only_r = mr & ~md, only_d = md & ~mr;
      while (only_r) {
        const int f = __builtin_ctzll(only_r);
        only_r &= only_r - 1;
        s -= xd[f] * xd[f];
      }
      while (only_d) {
        const int f = __builtin_ctzll(only_d);
        only_d &= only_d - 1;
        s -= xr[f] * xr[f];
      }
      const int present = F - __builtin_popcountll(mr | md);
      if (present <= 0) continue;  // undefined distance (sklearn: NaN, ignored)
      const float dist = fmaxf(s, 0.f) * ((float)F / (float)present);
      const int di = d0 + t;
#pragma unroll
      for (int k = 0; k < kKnnSlots; ++k) {
        if (col[k] >= 0 && !((md >> col[k]) & 1ull) && dist < bd[k]) { bd[k] = dist; bi[k] = di; }
      }
    }
  }
  if (active) {
#pragma unroll
    for (int k = 0; k < kKnnSlots; ++k) {
      best_idx[(size_t)r * kKnnSlots + k] = bi[k];
      best_dist[(size_t)r * kKnnSlots + k] = bd[k];
    }
  }
}

void knn_donors(uintptr_t R, uintptr_t rmask, int nr, uintptr_t D, uintptr_t dmask, int nd, int F,
                uintptr_t slot_col, uintptr_t best_idx, uintptr_t best_dist, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "knn_donors: 1 <= F <= 64 (64-bit missing masks)");
  if (nr == 0) return;
  const int ld = F | 1;
  const size_t lds = (size_t)2 * 256 * ld * sizeof(float) + 16 + 256 * sizeof(unsigned long long);
  HFENS_REQUIRE(lds <= 160 * 1024, "knn_donors: LDS budget");
  hipLaunchKernelGGL(knn_donor_kernel, dim3((nr + 255) / 256), dim3(256), lds, as_stream(stream),
                     (const float*)R, (const unsigned long long*)rmask, nr, (const float*)D,
                     (const unsigned long long*)dmask, nd, F, (const int*)slot_col, (int*)best_idx,
                     (float*)best_dist);
  launch_check();
}

}  // namespace hfens
