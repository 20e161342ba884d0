// nan-euclidean 1-NN donor search for KNN imputation (reference
// KNNImputer(n_neighbors=1), train_ensemble_public.py:37-40; distance semantics of sklearn
// nan_euclidean_distances: d² = F/|common| · Σ_{common present} (x−y)²).
//
// grid = (receiver blocks of 256) × (donor splits).  One thread owns one receiver row (values in
// registers, statically indexed up to FMAX features) and up to 8 missing-column slots.  Each
// workgroup streams its donor range through LDS in 256-row tiles (row stride padded to 4 floats
// so every lane reads the same 16-byte vector: broadcast ds_read_b128).  Per (receiver, donor) the
// distance is the direct difference form Σ(x_r − x_d)² over the features present in both rows
// (masked by the two 64-bit missing masks; no ‖x‖²+‖y‖²−2x·y and no add-then-subtract
// corrections, so exact ties stay exact).  Results merge across donor splits with a
// 64-bit atomicMin on (float bits of d², donor index): smallest distance, then lowest donor index
// — deterministic regardless of split count or arrival order.
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace hfens {

constexpr int kKnnTile = 256;
constexpr int kKnnSlots = 8;

// Merge of one donor split's per-slot results: the best as (f32 distance bits, donor) by 64-bit
// atomicMin, and alt = the smallest distance of any OTHER donor (the f64 refine's ambiguity test):
// the loser of every best exchange (this split's key, or the key it displaced) and this split's own
// runner-up go to alt — every non-winning split best ends there exactly once, whatever the order.
__device__ __forceinline__ void knn_merge_slots(unsigned long long* best, unsigned* alt, int r,
                                                const float (&bd)[kKnnSlots], const float (&b2)[kKnnSlots],
                                                const int (&bi)[kKnnSlots]) {
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k) {
    if (bi[k] < 0) continue;
    const size_t e = (size_t)r * kKnnSlots + k;
    const unsigned long long key =
        ((unsigned long long)__float_as_uint(bd[k]) << 32) | (unsigned long long)(unsigned)bi[k];
    const unsigned long long old = atomicMin(&best[e], key);
    const unsigned long long loser = old < key ? key : old;
    if (loser != ~0ull) atomicMin(&alt[e], (unsigned)(loser >> 32));
    if (b2[k] < INFINITY) atomicMin(&alt[e], __float_as_uint(b2[k]));
  }
}

template <int FMAX>
__global__ __launch_bounds__(256) void knn_donor_kernel(
    const float* __restrict__ R, const unsigned long long* __restrict__ rmask, int nr,
    const float* __restrict__ D, const unsigned long long* __restrict__ dmask, int nd, int F,
    int per_split, const int* __restrict__ slot_col /*[nr][kKnnSlots] column or −1*/,
    unsigned long long* __restrict__ best /*[nr][kKnnSlots] packed (dist bits, idx)*/,
    unsigned* __restrict__ alt /*[nr][kKnnSlots] f32 bits of the runner-up distance*/,
    const int* __restrict__ cnt /*device plan: [nr, nslot] or null*/, int s0) {
  if (cnt != nullptr) {   // planned on the device (knn_plan_dev): receiver count and slot groups there
    if (s0 >= cnt[1]) return;
    nr = cnt[0];
  }
  constexpr int LD = (FMAX + 3) / 4 * 4;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* ds = sm;                                                        // [256][LD] donor tile
  unsigned long long* dm = (unsigned long long*)(ds + kKnnTile * LD);    // [256]
  const int r = blockIdx.x * 256 + threadIdx.x;
  const bool active = r < nr;
  const int d_begin = blockIdx.y * per_split;
  const int d_end = min(nd, d_begin + per_split);
  float xr[LD];
#pragma unroll
  for (int f = 0; f < LD; ++f) xr[f] = (active && f < F) ? R[(size_t)r * F + f] : 0.f;
  const unsigned long long mr = active ? rmask[r] : 0ull;
  int col[kKnnSlots];
  float bd[kKnnSlots], b2[kKnnSlots];   // best and runner-up distance per slot
  int bi[kKnnSlots];
  bool any = false;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k) {
    col[k] = active ? slot_col[(size_t)r * kKnnSlots + k] : -1;
    bd[k] = INFINITY;
    b2[k] = INFINITY;
    bi[k] = -1;
    any |= col[k] >= 0;
  }
  unsigned long long need = 0ull;  // bitmask of this receiver's slot columns
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k)
    if (col[k] >= 0) need |= 1ull << col[k];
  // largest current best over the active slots: a donor at distance ≥ it can improve no slot
  // (the slot test is strict), so the 8-slot update is skipped for it — once the bests settle,
  // almost every donor (exact: skipping changes no comparison)
  float bmax = INFINITY;
  for (int d0 = d_begin; d0 < d_end; d0 += kKnnTile) {
    __syncthreads();
    const int nt = min(kKnnTile, d_end - d0);
    for (int e = threadIdx.x; e < nt * LD; e += 256) {
      const int rr = e / LD, c = e % LD;
      ds[e] = c < F ? D[(size_t)(d0 + rr) * F + c] : 0.f;
    }
    if (threadIdx.x < nt) dm[threadIdx.x] = dmask[d0 + threadIdx.x];
    __syncthreads();
    if (!any) continue;
    for (int t = 0; t < nt; ++t) {
      const unsigned long long md = dm[t];
      if ((need & ~md) == 0ull) continue;  // donor lacks every column this receiver needs
      const float4* xd4 = reinterpret_cast<const float4*>(ds + t * LD);
      // Σ over the features present in BOTH rows, as masked direct differences: no
      // add-then-subtract cross-missing corrections, so rows whose common values agree get
      // bit-identical distances (exact ties stay ties, as in the f64 reference)
      const unsigned long long both = ~(mr | md);
      const unsigned blo = (unsigned)both, bhi = (unsigned)(both >> 32);
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int q = 0; q < LD / 4; ++q) {
        if (4 * q < F) {
          const float4 v = xd4[q];
          const unsigned bq = ((4 * q < 32 ? blo >> (4 * q) : bhi >> (4 * q - 32))) & 0xFu;
          const float a = (bq & 1u) ? xr[4 * q] - v.x : 0.f;
          const float b = (bq & 2u) ? xr[4 * q + 1] - v.y : 0.f;
          const float c = (bq & 4u) ? xr[4 * q + 2] - v.z : 0.f;
          const float d = (bq & 8u) ? xr[4 * q + 3] - v.w : 0.f;
          s0 = fmaf(a, a, s0);
          s1 = fmaf(b, b, s1);
          s0 = fmaf(c, c, s0);
          s1 = fmaf(d, d, s1);
        }
      }
      const float s = s0 + s1;
      const int present = F - __builtin_popcountll(mr | md);
      if (present <= 0) continue;  // undefined distance (sklearn: NaN, ignored)
      const float dist = fmaxf(s, 0.f) * ((float)F / (float)present);
      if (!(dist < bmax)) continue;
      const int di = d0 + t;
      float m = 0.f;
#pragma unroll
      for (int k = 0; k < kKnnSlots; ++k) {
        // strict best (ties: the lower donor index, met first) and the runner-up (a tie with the
        // best lands there): a donor at or past every slot's runner-up changes nothing
        if (col[k] >= 0 && !((md >> col[k]) & 1ull) && dist < b2[k]) {
          const bool nb = dist < bd[k];
          b2[k] = nb ? bd[k] : dist;
          bi[k] = nb ? di : bi[k];
          bd[k] = nb ? dist : bd[k];
        }
        if (col[k] >= 0) m = fmaxf(m, b2[k]);
      }
      bmax = m;
    }
  }
  if (active) knn_merge_slots(best, alt, r, bd, b2, bi);
}

// The same search with a packed-FMA fast pass in front of the exact distance.
// Receiver and donor rows are zero-filled at missing cells (as staged above); with m_r the
// receiver's 0/1 present mask, the fast pass accumulates Σ_f fma(−m_r, x_d, x_r)² over all
// features with v_pk_fma_f32 (two features per instruction, the same even/odd accumulator split):
//   * a COMPLETE donor (md = 0): every term is the exact kernel's term bit for bit (x_r − x_d with
//     one rounding when both are present, +0 when the receiver is missing), so the sum IS the exact
//     distance;
//   * a donor with missing cells: the terms of its missing features that the receiver has
//     contribute x_r² instead of 0.  corr = Σ of those x_r² (a uniform loop over the donor's few
//     missing features) gives a lower bound lb = (fast − corr) − 2⁻¹⁶·(fast + corr) of the exact
//     sum (≤ ~100 roundings of ≤ 2⁻²⁴ each); a donor whose bound cannot beat the receiver's current
//     worst slot is skipped — exactly, since the slot test is strict — and only the others run
//     the exact masked direct-difference pass of knn_donor_kernel.
// The exact pass decides every update, so the donors equal knn_donor_kernel's bit for bit (tested).
// XS (LD ≤ 40): the receiver rows also sit in LDS, column-major per thread, for the correction's
// uniform-index reads; the donor tile is then kKnnFastTile rows so two workgroups still fit per CU.
constexpr int kKnnFastTile = 224;
template <int FMAX>
constexpr bool knn_fast_xs() { return (FMAX + 3) / 4 * 4 <= 40; }
template <int FMAX>
constexpr int knn_fast_tile() { return knn_fast_xs<FMAX>() ? kKnnFastTile : kKnnTile; }

template <int FMAX>
constexpr size_t knn_fast_lds() {
  constexpr int LD = (FMAX + 3) / 4 * 4;
  return (size_t)knn_fast_tile<FMAX>() * LD * sizeof(float) + knn_fast_tile<FMAX>() * sizeof(unsigned long long) +
         (knn_fast_xs<FMAX>() ? (size_t)LD * 256 * sizeof(float) : 0);
}
template <int FMAX>
constexpr size_t knn_fast_lds_sm() {   // SM: only the receiver-value table
  return knn_fast_xs<FMAX>() ? (size_t)((FMAX + 3) / 4 * 4) * 256 * sizeof(float) : 0;
}

// SM (F == LD): the donor rows are read straight from global memory at wave-uniform addresses —
// scalar loads into SGPRs, the VALU reading them as operands — instead of broadcast LDS reads of a
// staged tile.  A broadcast ds_read_b128 still moves 1 KB per wave through the CU's LDS port, so
// with 8 waves per CU the staged kernel was bound by LDS bandwidth (≈ 20 b128 reads per donor pair).
template <int FMAX, bool SM>
__global__ __launch_bounds__(256) void knn_donor_fast_kernel(
    const float* __restrict__ R, const unsigned long long* __restrict__ rmask, int nr,
    const float* __restrict__ D, const unsigned long long* __restrict__ dmask, int nd, int F,
    int per_split, const int* __restrict__ slot_col, unsigned long long* __restrict__ best,
    unsigned* __restrict__ alt, const int* __restrict__ cnt, int s0) {
  if (cnt != nullptr) {
    if (s0 >= cnt[1]) return;
    nr = cnt[0];
  }
  constexpr int LD = (FMAX + 3) / 4 * 4;
  constexpr bool XS = knn_fast_xs<FMAX>();
  constexpr int TILE = knn_fast_tile<FMAX>();
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* ds = sm;                                                           // !SM: [TILE][LD]
  unsigned long long* dm = (unsigned long long*)(ds + (SM ? 0 : TILE * LD));  // !SM: [TILE]
  float* xs = SM ? sm : reinterpret_cast<float*>(dm + TILE);   // XS: [LD][256] receiver values
  const int r = blockIdx.x * 256 + threadIdx.x;
  const bool active = r < nr;
  const int d_begin = blockIdx.y * per_split;
  const int d_end = min(nd, d_begin + per_split);
  const unsigned long long mr = active ? rmask[r] : 0ull;
  // receiver values and −(present) as feature pairs (the only copy of the row: 2 waves → 3 per SIMD)
  f32x2v xr2[LD / 2], nm2[LD / 2];
#pragma unroll
  for (int h = 0; h < LD / 2; ++h) {
    xr2[h] = f32x2v{(active && 2 * h < F) ? R[(size_t)r * F + 2 * h] : 0.f,
                    (active && 2 * h + 1 < F) ? R[(size_t)r * F + 2 * h + 1] : 0.f};
    const float m0 = (2 * h < F && !((mr >> (2 * h)) & 1ull)) ? -1.f : -0.f;
    const float m1 = (2 * h + 1 < F && !((mr >> (2 * h + 1)) & 1ull)) ? -1.f : -0.f;
    nm2[h] = f32x2v{m0, m1};
    if constexpr (XS) {
      xs[(2 * h) * 256 + threadIdx.x] = xr2[h][0];
      xs[(2 * h + 1) * 256 + threadIdx.x] = xr2[h][1];
    }
  }
  int col[kKnnSlots];
  float bd[kKnnSlots], b2[kKnnSlots];   // best and runner-up distance per slot
  int bi[kKnnSlots];
  bool any = false;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k) {
    col[k] = active ? slot_col[(size_t)r * kKnnSlots + k] : -1;
    bd[k] = INFINITY;
    b2[k] = INFINITY;
    bi[k] = -1;
    any |= col[k] >= 0;
  }
  unsigned long long need = 0ull;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k)
    if (col[k] >= 0) need |= 1ull << col[k];
  float bmax = INFINITY;
  // F / present for every present count, the same IEEE division as the exact kernel, looked up
  // instead of recomputed per donor (a full-precision f32 divide is ~10 VALU instructions)
  __shared__ float s_scale[65];
  if (threadIdx.x <= 64) s_scale[threadIdx.x] = threadIdx.x > 0 ? (float)F / (float)threadIdx.x : 0.f;
  for (int d0 = d_begin; d0 < d_end; d0 += TILE) {
    const int nt = min(TILE, d_end - d0);
    if constexpr (SM) {
      __syncthreads();   // (s_scale / xs written before the first tile)
    } else {
    __syncthreads();
    if (XS && F == LD) {   // (XS widths only: at LD ≥ 48 the copy's registers cost occupancy)
      // the tile is one contiguous run of D: float4 copies, all of a thread's loads in flight
      // before its first LDS write (a scalar loop waited out one global round trip per element)
      const float4* src = reinterpret_cast<const float4*>(D + (size_t)d0 * F);
      float4* dst = reinterpret_cast<float4*>(ds);
      const int n4 = nt * LD / 4;
      constexpr int U = XS ? (TILE * LD / 4 + 255) / 256 : 0, UC = 4;   // rounds of UC loads
#pragma unroll
      for (int u0 = 0; u0 < U; u0 += UC) {
        float4 v[UC];
#pragma unroll
        for (int u = 0; u < UC; ++u) {
          const int e = threadIdx.x + 256 * (u0 + u);
          v[u] = (u0 + u < U && e < n4) ? src[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < UC; ++u) {
          const int e = threadIdx.x + 256 * (u0 + u);
          if (u0 + u < U && e < n4) dst[e] = v[u];
        }
      }
    } else {
      for (int e = threadIdx.x; e < nt * LD; e += 256) {
        const int rr = e / LD, c = e % LD;
        ds[e] = c < F ? D[(size_t)(d0 + rr) * F + c] : 0.f;
      }
    }
    if (threadIdx.x < nt) dm[threadIdx.x] = dmask[d0 + threadIdx.x];
    __syncthreads();
    }
    if (!any) continue;
    // donors two at a time: their fast sums are independent fma chains (each 2 × ≤ 32 dependent
    // steps: the accumulation order must stay the exact kernel's), interleaved to hide the latency;
    // the bookkeeping then runs donor t before donor t + 1, exactly as one at a time
    auto donor = [&](int t, float sf) {
      const unsigned long long md = SM ? dmask[d0 + t] : dm[t];
      if ((need & ~md) == 0ull) return;
      const int present = F - __builtin_popcountll(mr | md);
      if (present <= 0) return;
      const float scale = s_scale[present];
      const bool exact = md == 0ull;
      if (!exact) {
        // the receiver-present features the donor lacks added x_r² each: a uniform loop (the
        // donor's missing cells, usually one), register index from a scalar
        // XS: each cell's x_r from this thread's column of the LDS copy of the receiver rows (one
        // conflict-free read); otherwise an LD-way register select
        float corr = 0.f;
        unsigned long long mm = md & ~mr & ((F >= 64) ? ~0ull : ((1ull << F) - 1ull));
        while (mm) {
          const int f = __builtin_ctzll(mm);
          mm &= mm - 1ull;
          float xv = 0.f;
          if constexpr (XS) {
            xv = xs[f * 256 + threadIdx.x];
          } else {
#pragma unroll
            for (int g = 0; g < LD; ++g) xv = g == f ? xr2[g >> 1][g & 1] : xv;
          }
          corr = fmaf(xv, xv, corr);
        }
        // ≤ 32 fma roundings per accumulator in either pass, ≤ 64 in corr, one subtraction: ≤ ~100
        // units of 2^-24 of (fast + corr); 2^-16 = 256 units
        const float lb = (sf - corr) - 1.52587890625e-05f * (sf + corr);
        // a donor whose lower bound (scaled, rounded down a further 2^-20) reaches the worst
        // active slot can improve no slot: skipped, exactly as the exact pass would skip it
        if (!(fmaxf(lb, 0.f) * scale * 0.99999905f < bmax)) return;
      } else if (!(fmaxf(sf, 0.f) * scale < bmax)) {
        return;
      }
      float s = sf;
      if (!exact) {
        // ---- exact pass (knn_donor_kernel's masked direct differences, same order and roundings)
        const float4* xd4 = SM ? reinterpret_cast<const float4*>(D + (size_t)(d0 + t) * LD)
                               : reinterpret_cast<const float4*>(ds + t * LD);
        const unsigned long long both = ~(mr | md);
        const unsigned blo = (unsigned)both, bhi = (unsigned)(both >> 32);
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int q = 0; q < LD / 4; ++q) {   // (features ≥ F: 0 − 0 on both sides, adds 0)
          const float4 v = xd4[q];
          const unsigned bq = ((4 * q < 32 ? blo >> (4 * q) : bhi >> (4 * q - 32))) & 0xFu;
          const float a = (bq & 1u) ? xr2[2 * q][0] - v.x : 0.f;
          const float b = (bq & 2u) ? xr2[2 * q][1] - v.y : 0.f;
          const float c = (bq & 4u) ? xr2[2 * q + 1][0] - v.z : 0.f;
          const float d = (bq & 8u) ? xr2[2 * q + 1][1] - v.w : 0.f;
          s0 = fmaf(a, a, s0);
          s1 = fmaf(b, b, s1);
          s0 = fmaf(c, c, s0);
          s1 = fmaf(d, d, s1);
        }
        s = s0 + s1;
      }
      const float dist = fmaxf(s, 0.f) * scale;
      if (!(dist < bmax)) return;
      const int di = d0 + t;
      float m = 0.f;
#pragma unroll
      for (int k = 0; k < kKnnSlots; ++k) {
        // strict best (ties: the lower donor index, met first) and the runner-up (a tie with the
        // best lands there): a donor at or past every slot's runner-up changes nothing
        if (col[k] >= 0 && !((md >> col[k]) & 1ull) && dist < b2[k]) {
          const bool nb = dist < bd[k];
          b2[k] = nb ? bd[k] : dist;
          bi[k] = nb ? di : bi[k];
          bd[k] = nb ? dist : bd[k];
        }
        if (col[k] >= 0) m = fmaxf(m, b2[k]);
      }
      bmax = m;
    };
    for (int t = 0; t < nt; t += 2) {
      const int t1 = t + 1 < nt ? t + 1 : t;
      const float4* xa = SM ? reinterpret_cast<const float4*>(D + (size_t)(d0 + t) * LD)
                            : reinterpret_cast<const float4*>(ds + t * LD);
      const float4* xb = SM ? reinterpret_cast<const float4*>(D + (size_t)(d0 + t1) * LD)
                            : reinterpret_cast<const float4*>(ds + t1 * LD);
      // ---- fast pass: packed fma over feature pairs, even features into .x, odd into .y — every
      // quad, F or not (features ≥ F are zero on both sides: fma(0, 0, acc) = acc; a runtime
      // `4q < F` guard would put a branch and an LDS wait between the quads' reads)
      f32x2v accA = f32x2v{0.f, 0.f}, accB = f32x2v{0.f, 0.f};
#pragma unroll
      for (int q = 0; q < LD / 4; ++q) {
        const float4 va = xa[q], vb = xb[q];
        const f32x2v a0 = __builtin_elementwise_fma(nm2[2 * q], f32x2v{va.x, va.y}, xr2[2 * q]);
        const f32x2v a1 = __builtin_elementwise_fma(nm2[2 * q + 1], f32x2v{va.z, va.w}, xr2[2 * q + 1]);
        const f32x2v b0 = __builtin_elementwise_fma(nm2[2 * q], f32x2v{vb.x, vb.y}, xr2[2 * q]);
        const f32x2v b1 = __builtin_elementwise_fma(nm2[2 * q + 1], f32x2v{vb.z, vb.w}, xr2[2 * q + 1]);
        accA = __builtin_elementwise_fma(a0, a0, accA);
        accB = __builtin_elementwise_fma(b0, b0, accB);
        accA = __builtin_elementwise_fma(a1, a1, accA);
        accB = __builtin_elementwise_fma(b1, b1, accB);
      }
      donor(t, accA.x + accA.y);
      if (t1 != t) donor(t1, accB.x + accB.y);
    }
  }
  if (active) knn_merge_slots(best, alt, r, bd, b2, bi);
}

// cnt (optional, device [nr, nslot] of knn_plan_dev): nr is then the capacity (grid, buffers) and the
// kernels take the receiver count from the device; slot group s0 ≥ nslot exits at once.
void knn_donors(uintptr_t R, uintptr_t rmask, int nr, uintptr_t D, uintptr_t dmask, int nd, int F,
                uintptr_t slot_col, uintptr_t best, uintptr_t alt, uintptr_t cnt, int s0, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "knn_donors: 1 <= F <= 64 (64-bit missing masks)");
  if (nr == 0 || nd == 0) return;
  hipStream_t st = as_stream(stream);
  HFENS_CHECK(hipMemsetAsync((void*)best, 0xFF, (size_t)nr * kKnnSlots * sizeof(unsigned long long), st));
  HFENS_CHECK(hipMemsetAsync((void*)alt, 0xFF, (size_t)nr * kKnnSlots * sizeof(unsigned), st));
  const int rb = (nr + 255) / 256;
  // enough splits for ≥ 2048 workgroups, and donor ranges of ≤ 16k rows per workgroup: a
  // workgroup then runs for milliseconds, not the whole search, so kernels of other streams (the
  // LassoCV path beside the held-out imputation at 10⁶ rows) get CUs as workgroups retire instead
  // of waiting for the donor search to drain.  The (distance, index) atomicMin merge makes the
  // result independent of the split count.
  int splits = 2048 / rb;
  const int by_range = (nd + 16383) / 16384;
  if (splits < by_range) splits = by_range;
  const int max_splits = (nd + kKnnTile - 1) / kKnnTile;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  const char* kenv = std::getenv("HFENS_KNN_KERNEL");
  const bool direct = kenv && kenv[0] == 'd';   // "direct": the exact pass for every donor
  const bool lds_tiles = kenv && kenv[0] == 'l';  // "lds": the fast pass on staged LDS tiles
  auto go = [&](auto fm) {
    constexpr int FM = decltype(fm)::value;
    constexpr int LD = (FM + 3) / 4 * 4;
    const int tile = direct ? kKnnTile : knn_fast_tile<FM>();
    int per = (nd + splits - 1) / splits;
    per = (per + tile - 1) / tile * tile;
    const int nsp = (nd + per - 1) / per;
    const size_t lds = direct ? (size_t)kKnnTile * LD * sizeof(float) + kKnnTile * sizeof(unsigned long long)
                              : knn_fast_lds<FM>();
    if (direct)
      hipLaunchKernelGGL(knn_donor_kernel<FM>, dim3(rb, nsp), dim3(256), lds, st, (const float*)R,
                         (const unsigned long long*)rmask, nr, (const float*)D,
                         (const unsigned long long*)dmask, nd, F, per, (const int*)slot_col,
                         (unsigned long long*)best, (unsigned*)alt, (const int*)cnt, s0);
    else if (F == LD && !lds_tiles && (D & 15) == 0)
      hipLaunchKernelGGL((knn_donor_fast_kernel<FM, true>), dim3(rb, nsp), dim3(256), knn_fast_lds_sm<FM>(), st,
                         (const float*)R, (const unsigned long long*)rmask, nr, (const float*)D,
                         (const unsigned long long*)dmask, nd, F, per, (const int*)slot_col,
                         (unsigned long long*)best, (unsigned*)alt, (const int*)cnt, s0);
    else
      hipLaunchKernelGGL((knn_donor_fast_kernel<FM, false>), dim3(rb, nsp), dim3(256), lds, st, (const float*)R,
                         (const unsigned long long*)rmask, nr, (const float*)D,
                         (const unsigned long long*)dmask, nd, F, per, (const int*)slot_col,
                         (unsigned long long*)best, (unsigned*)alt, (const int*)cnt, s0);
    launch_check();
  };
  if (F <= 16) go(std::integral_constant<int, 16>{});
  else if (F <= 32) go(std::integral_constant<int, 32>{});
  else if (F <= 40) go(std::integral_constant<int, 40>{});
  else if (F <= 48) go(std::integral_constant<int, 48>{});
  else go(std::integral_constant<int, 64>{});
}


// ---- the donor filter on the bf16 matrix cores (SURVEY K1's Gram form) ----------
// The packed-FMA fast pass above costs ~2 VALU instructions per feature and pair.  Here the whole
// masked filter distance of 32 donors × 32 receivers is one GEMM on v_mfma_f32_32x32x16_bf16.
// With x̃, ỹ the rows zero-filled at missing cells, the squared distance over the features present
// in BOTH rows is
//     ‖x̃‖² + ‖ỹ‖² − 2 x̃·ỹ − Σ_f [d misses f] x̃_f² − Σ_f [r misses f] ỹ_f²,
// and all three sums are inner products along K: items (ỹ hi, −2x̃ hi), (ỹ hi, −2x̃ lo),
// (ỹ lo, −2x̃ hi), ([d misses f], −x̃² hi), ([d misses f], −x̃² lo), (ỹ² hi, −[r misses f]),
// (ỹ² lo, −[r misses f]) — 7F items, each f32 value cut into two bf16 pieces (hi = truncation,
// lo = truncation of the rest; the indicators are exact).  The dropped lo×lo pieces and the f32
// accumulation stay below 2⁻¹³·(‖x̃‖² + ‖ỹ‖²); a donor whose estimate minus 2⁻¹¹·(‖x̃‖² + ‖ỹ‖²),
// scaled by F/common and rounded down, reaches the lane's worst slot cannot improve any slot and is
// skipped (a scale-free test first: five VALU instructions per pair); every other donor is queued
// per lane and runs knn_donor_kernel's exact masked direct-difference pass in batches compacted over
// the wave's 64 lanes, and that pass alone decides the slots.  The exact
// pass sees every donor the packed-FMA kernel's exact pass would (the skip is sound), so the per-slot
// best and runner-up are the same bits (tests/test_prep_gpu.py::test_knn_mfma_filter_same_slots).
// Lane ℓ and ℓ + 32 share a receiver (column ℓ mod 32 of the tile) and take alternating donor quads
// of each 32-donor tile, each with its own slots — merged like donor splits (knn_merge_slots:
// order-independent).  8 waves share each staged donor tile (256 receivers per workgroup), the
// receivers' rows live in LDS (registers go to the 18 operand blocks), and the next tile's loads
// are issued before this tile's product.
template <int FM>
struct KnnMf {
  static constexpr int NB = (7 * FM + 15) / 16;    // MFMA k-blocks of the items
  static constexpr int LP = NB * 16;
  static constexpr int LPS = LP + 8;               // LDS row stride (u16): rows 16 B apart in the banks
  static constexpr int TILE = 32;
  static constexpr int WAVES = FM >= 48 ? 4 : 8;   // (LDS: 160 KB per workgroup)
  static constexpr int A4 = TILE * LP / 8;         // uint4 of a tile's items
  static constexpr int Y4 = TILE * FM / 4;         // float4 of a tile's rows
};
typedef __bf16 knn_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int knn_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned knn_bf_hi(float v) { return __float_as_uint(v) >> 16; }
__device__ __forceinline__ unsigned knn_bf_lo(float v) {
  const float r = v - __uint_as_float(__float_as_uint(v) & 0xFFFF0000u);
  return __float_as_uint(r) >> 16;
}

// donor side: items [nd][LP] (bf16 bits, kinds: 0/1 ỹ hi, 2 ỹ lo, 3/4 [d misses f], 5 ỹ² hi, 6 ỹ² lo),
// rows [nd][FM] zero-filled
// f32 (FM-strided: float4 staging), ‖ỹ‖² [nd]
template <int FM>
__global__ __launch_bounds__(256) void knn_mfma_prep_kernel(const float* __restrict__ D,
                                                            const unsigned long long* __restrict__ dmask,
                                                            int nd, int F, unsigned short* __restrict__ items,
                                                            float* __restrict__ rowsFM, float* __restrict__ ny) {
  using K = KnnMf<FM>;
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= nd) return;
  const unsigned long long md = dmask[d];
  unsigned short* it = items + (size_t)d * K::LP;
  float nsum = 0.f;
  for (int f = 0; f < FM; ++f) {
    const float y = (f < F && !((md >> f) & 1ull)) ? D[(size_t)d * F + f] : 0.f;
    rowsFM[(size_t)d * FM + f] = y;
    nsum = fmaf(y, y, nsum);
  }
  for (int q = 0; q < K::LP; ++q) {
    const int kind = q / FM, f = q - kind * FM;
    const bool miss = f >= F || ((md >> f) & 1ull);
    const float y = miss ? 0.f : D[(size_t)d * F + f];
    unsigned w = 0u;
    if (kind <= 1) w = knn_bf_hi(y);
    else if (kind == 2) w = knn_bf_lo(y);
    else if (kind <= 4) w = (f < F && miss) ? 0x3F80u : 0u;
    else if (kind == 5) w = knn_bf_hi(y * y);
    else if (kind == 6) w = knn_bf_lo(y * y);
    it[q] = (unsigned short)w;
  }
  ny[d] = nsum;
}

// MODE 1 (knn_refine's window listing, the role of knn_cand_kernel<·, 0>): the receivers are
// rlist[0 … counts[0]), each slot k has a fixed window thr[k] (≥ 0: listed), and every (slot, donor)
// with exact f32 distance ≤ thr[k] is appended to pairs (pcount[0]; overflow → pcount[1]) — the same
// pairs knn_cand_kernel lists (the matrix-core bound only skips donors above every window)
template <int FM, int MODE = 0>
__global__ __launch_bounds__(512) void knn_donor_mfma_kernel(
    const float* __restrict__ R, const unsigned long long* __restrict__ rmask, int nr,
    const float* __restrict__ rowsFM, const unsigned long long* __restrict__ dmask, int nd, int F,
    int per_split, const int* __restrict__ slot_col, unsigned long long* __restrict__ best,
    unsigned* __restrict__ alt, const int* __restrict__ cnt, int s0,
    const unsigned short* __restrict__ items, const float* __restrict__ ny_all,
    const int* __restrict__ rlist = nullptr, const float* __restrict__ thr = nullptr,
    int* __restrict__ pairs = nullptr, long long cap = 0, int* __restrict__ pcount = nullptr) {
  using K = KnnMf<FM>;
  if constexpr (MODE == 1) {
    nr = cnt[0];
    if ((int)blockIdx.x * (32 * K::WAVES) >= nr) return;
  } else if (cnt != nullptr) {
    if (s0 >= cnt[1]) return;
    nr = cnt[0];
  }
  constexpr int LD = FM;   // (FM is a multiple of 8)
  constexpr int NT = 64 * K::WAVES;
  __shared__ __attribute__((aligned(16))) unsigned short tA[K::TILE * K::LPS];
  __shared__ __attribute__((aligned(16))) float tY[K::TILE * LD];
  __shared__ unsigned long long tM[K::TILE];
  __shared__ knn_u32x4 tR[K::TILE];   // a donor's mask and ‖ỹ‖² in one 16-byte read
  __shared__ __attribute__((aligned(16))) float tNy[K::TILE];
  __shared__ float s_scale[65];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r32 = lane & 31, hh = lane >> 5;
  const int li = blockIdx.x * (32 * K::WAVES) + wave * 32 + r32;
  const bool active = li < nr;
  const int r = MODE == 1 ? (active ? rlist[li] : 0) : li;
  const int d_begin = blockIdx.y * per_split;
  const int d_end = min(nd, d_begin + per_split);
  const unsigned long long mr = active ? rmask[r] : 0ull;
  // the receivers' zero-filled rows stay in LDS (the operand build and the exact pass read them)
  __shared__ __attribute__((aligned(16))) float xs[32 * K::WAVES][LD + 4];
  __shared__ unsigned long long smr[32 * K::WAVES];
  constexpr int kQc = 16;   // ≥ 16: a tile adds at most 16 candidates per lane after a flush
  __shared__ unsigned short clist[K::WAVES][64 * kQc];   // a wave's queued (lane, entry) candidates
  __shared__ int q_idx[K::WAVES][64][kQc];               // each lane's queued donors
  __shared__ float q_dist[K::WAVES][64][kQc];            // their exact distances
  float* xrow = xs[wave * 32 + r32];
  if (hh == 0) smr[wave * 32 + r32] = mr;
  float nx = 0.f;
  for (int f = hh; f < LD; f += 2) {
    const float v = (active && f < F && !((mr >> f) & 1ull)) ? R[(size_t)r * F + f] : 0.f;
    xrow[f] = v;
  }
  __syncthreads();
#pragma unroll 8
  for (int f = 0; f < LD; ++f) nx = fmaf(xrow[f], xrow[f], nx);
  // receiver operands: item q = 16m + 8hh + e of the lane's half (kinds: 0 −2x̃ hi, 1 −2x̃ lo, 2 −2x̃ hi,
  // 3 −x̃² hi, 4 −x̃² lo, 5/6 −[r misses f])
  knn_bf16x8 bq[K::NB];
#pragma unroll
  for (int m = 0; m < K::NB; ++m) {
    unsigned w[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      unsigned v2[2];
#pragma unroll
      for (int dd = 0; dd < 2; ++dd) {
        const int q = 16 * m + 8 * hh + 2 * e2 + dd;
        const int kind = q / FM, f = q - kind * FM;
        const float xv = kind < 7 ? xrow[f] : 0.f;
        const float v = kind <= 2 ? -2.f * xv : -(xv * xv);
        const bool rm = f < F && ((mr >> f) & 1ull);
        unsigned ww = 0u;
        if (kind == 0 || kind == 2 || kind == 3) ww = knn_bf_hi(v);
        else if (kind == 1 || kind == 4) ww = knn_bf_lo(v);
        else if (kind <= 6) ww = rm ? 0xBF80u : 0u;
        v2[dd] = ww;
      }
      w[e2] = v2[0] | (v2[1] << 16);
    }
    bq[m] = __builtin_bit_cast(knn_bf16x8, (knn_u32x4){w[0], w[1], w[2], w[3]});
  }
  int col[kKnnSlots];
  float bd[kKnnSlots], b2[kKnnSlots];   // MODE 1: b2 holds the slot's window
  int bi[kKnnSlots];
  bool any = false;
  float tmax = -1.f;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k) {
    const size_t e = (size_t)r * kKnnSlots + k;
    bd[k] = INFINITY;
    b2[k] = INFINITY;
    bi[k] = -1;
    if constexpr (MODE == 1) {
      const float t = active ? thr[e] : -1.f;
      col[k] = t >= 0.f ? slot_col[e] : -1;
      b2[k] = t;
      if (col[k] >= 0) tmax = fmaxf(tmax, t);
    } else {
      col[k] = active ? slot_col[e] : -1;
    }
    any |= col[k] >= 0;
  }
  unsigned long long need = 0ull;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k)
    if (col[k] >= 0) need |= 1ull << col[k];
  // MODE 1: the windows are fixed; ×(1 + 2⁻²⁰) so the strict tests below keep a pair at the window
  float bmax = MODE == 1 ? (tmax >= 0.f ? tmax * 1.00000095f : -1.f) : INFINITY;
  if (tid <= 64) s_scale[tid] = tid > 0 ? (float)F / (float)tid : 0.f;
  const float fF = (float)F * 0.99999905f;
  const bool wave_any = __ballot(any) != 0ull;
  // prefetch of a tile into registers (issued one tile ahead)
  constexpr int PA = (K::A4 + NT - 1) / NT, PY = (K::Y4 + NT - 1) / NT;
  knn_u32x4 pa[PA];
  float4 py[PY];
  unsigned long long pm = ~0ull;
  float pn = 0.f;
  auto fetch = [&](int d0) {
    const int nt = min(K::TILE, d_end - d0);
    const knn_u32x4* srcA = reinterpret_cast<const knn_u32x4*>(items + (size_t)d0 * K::LP);
    const float4* srcY = reinterpret_cast<const float4*>(rowsFM + (size_t)d0 * LD);
#pragma unroll
    for (int u = 0; u < PA; ++u) {
      const int e = tid + u * NT;
      pa[u] = (e < nt * K::LP / 8) ? srcA[e] : (knn_u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < PY; ++u) {
      const int e = tid + u * NT;
      py[u] = (e < nt * LD / 4) ? srcY[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (tid < K::TILE) {
      pm = tid < nt ? dmask[d0 + tid] : ~0ull;
      pn = tid < nt ? ny_all[d0 + tid] : 0.f;
    }
  };
  // candidate queue of each lane (donor indices, increasing) and the batched exact pass: the wave's
  // queued candidates are compacted over its 64 lanes (one lane per candidate, donor rows from global
  // memory), then every lane folds its own in donor order — a wave pays the exact pass's latency
  // once per kQc-entry batch instead of once per tile that holds any candidate
  int qlen = 0;
  auto flush = [&]() {
    const int mine = qlen;
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int total = __shfl(incl, 63, 64);
    if (total == 0) return;
    for (int e = 0, pos = incl - mine; e < mine; ++e, ++pos) clist[wave][pos] = (unsigned short)((lane << 5) | e);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int c = lane; c < total; c += 64) {
      const int code = clist[wave][c];
      const int owner = code >> 5, e = code & 31;
      const int di = q_idx[wave][owner][e];
      const unsigned long long md = dmask[di];
      const unsigned long long mro = smr[wave * 32 + (owner & 31)];
      const int present = F - __builtin_popcountll(mro | md);
      // knn_donor_kernel's masked direct differences, same order and roundings
      const float4* xd4 = reinterpret_cast<const float4*>(rowsFM + (size_t)di * LD);
      const float4* xr4 = reinterpret_cast<const float4*>(xs[wave * 32 + (owner & 31)]);
      const unsigned long long both = ~(mro | md);
      const unsigned blo = (unsigned)both, bhi = (unsigned)(both >> 32);
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int q = 0; q < LD / 4; ++q) {
        const float4 v = xd4[q];
        const float4 u = xr4[q];
        const unsigned bqm = ((4 * q < 32 ? blo >> (4 * q) : bhi >> (4 * q - 32))) & 0xFu;
        const float a = (bqm & 1u) ? u.x - v.x : 0.f;
        const float b = (bqm & 2u) ? u.y - v.y : 0.f;
        const float cc = (bqm & 4u) ? u.z - v.z : 0.f;
        const float d = (bqm & 8u) ? u.w - v.w : 0.f;
        sa = fmaf(a, a, sa);
        sb = fmaf(b, b, sb);
        sa = fmaf(cc, cc, sa);
        sb = fmaf(d, d, sb);
      }
      q_dist[wave][owner][e] = fmaxf(sa + sb, 0.f) * s_scale[present];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int e = 0; e < mine; ++e) {
      const float dist = q_dist[wave][lane][e];
      if constexpr (MODE == 1) {
        const int di = q_idx[wave][lane][e];
        const unsigned long long md = dmask[di];
#pragma unroll
        for (int k = 0; k < kKnnSlots; ++k) {
          if (col[k] >= 0 && !((md >> col[k]) & 1ull) && dist <= b2[k]) {
            const int p = atomicAdd(&pcount[0], 1);
            if (p < cap) {
              pairs[2 * (size_t)p] = (int)((size_t)r * kKnnSlots + k);
              pairs[2 * (size_t)p + 1] = di;
            } else {
              pcount[1] = 1;
            }
          }
        }
        continue;
      }
      if (!(dist < bmax)) continue;
      const int di = q_idx[wave][lane][e];
      const unsigned long long md = dmask[di];
      float mx = 0.f;
#pragma unroll
      for (int k = 0; k < kKnnSlots; ++k) {
        if (col[k] >= 0 && !((md >> col[k]) & 1ull) && dist < b2[k]) {
          const bool nb = dist < bd[k];
          b2[k] = nb ? bd[k] : dist;
          bi[k] = nb ? di : bi[k];
          bd[k] = nb ? dist : bd[k];
        }
        if (col[k] >= 0) mx = fmaxf(mx, b2[k]);
      }
      bmax = mx;
    }
    qlen = 0;
    __builtin_amdgcn_wave_barrier();
  };
  if (d_begin < d_end) fetch(d_begin);
  for (int d0 = d_begin; d0 < d_end; d0 += K::TILE) {
    const int nt = min(K::TILE, d_end - d0);
    __syncthreads();   // the previous tile is consumed
#pragma unroll
    for (int u = 0; u < PA; ++u) {
      const int e = tid + u * NT;
      if (e < K::A4) reinterpret_cast<knn_u32x4*>(tA)[(e / (K::LP / 8)) * (K::LPS / 8) + e % (K::LP / 8)] = pa[u];
    }
#pragma unroll
    for (int u = 0; u < PY; ++u) {
      const int e = tid + u * NT;
      if (e < K::Y4) reinterpret_cast<float4*>(tY)[e] = py[u];
    }
    if (tid < K::TILE) {
      tM[tid] = pm;
      tR[tid] = (knn_u32x4){(unsigned)pm, (unsigned)(pm >> 32), __float_as_uint(pn), 0u};
      tNy[tid] = pn;
    }
    __syncthreads();
    if (d0 + K::TILE < d_end) fetch(d0 + K::TILE);   // the next tile's loads fly under this one
    if (!wave_any) continue;
    f32x16 acc = {0.f};
#pragma unroll
    for (int m = 0; m < K::NB; ++m) {
      const knn_u32x4 raw = *reinterpret_cast<const knn_u32x4*>(&tA[r32 * K::LPS + 16 * m + 8 * hh]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(knn_bf16x8, raw), bq[m], acc, 0, 0, 0);
    }
    // (a) the bound: which of the lane's 16 donors can still improve a slot (bmax of the tile start:
    //     a stale bmax only lets more donors through, and those change nothing below)
    unsigned cand = 0u;
    if (any) {
      // first a cheap test without the F/common scale (≥ 1): max(est − bound, 0) ≥ bmax already
      // skips, and it holds for almost every pair once the slots have filled
      const float bq1 = bmax * 1.0000038f;                   // (1 + 2^-18): covers the roundings
      const float nxk = nx * 0.99951171875f;                  // (1 − 2^-11) ‖x̃‖²
      unsigned pre = 0u;
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // accumulators 4g..4g+3 are donors 8g + 4hh + 0..3
        const float4 ny4 = *reinterpret_cast<const float4*>(&tNy[8 * g + 4 * hh]);
        pre |= (unsigned)(fmaf(ny4.x, 0.99951171875f, nxk) + acc[4 * g] < bq1) << (4 * g);
        pre |= (unsigned)(fmaf(ny4.y, 0.99951171875f, nxk) + acc[4 * g + 1] < bq1) << (4 * g + 1);
        pre |= (unsigned)(fmaf(ny4.z, 0.99951171875f, nxk) + acc[4 * g + 2] < bq1) << (4 * g + 2);
        pre |= (unsigned)(fmaf(ny4.w, 0.99951171875f, nxk) + acc[4 * g + 3] < bq1) << (4 * g + 3);
      }
      // then the full test: lb·(1 + ε) < bmax ⇔ max(est − bound, 0)·F·c < bmax·common (no
      // division); rows ≥ nt carry an all-ones mask (no common feature)
      while (pre) {
        const int j = __builtin_ctz(pre);
        pre &= pre - 1u;
        const int row = (j & 3) + 8 * (j >> 2) + 4 * hh;
        const knn_u32x4 rw = *reinterpret_cast<const knn_u32x4*>(&tR[row]);
        const unsigned long long md = (unsigned long long)rw.x | ((unsigned long long)rw.y << 32);
        const float ynorm = __uint_as_float(rw.z);
        const int present = F - __builtin_popcountll(mr | md);
        float aj = 0.f;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) aj = jj == j ? acc[jj] : aj;
        const float lhs = fmaxf((nx + ynorm) + aj - 4.8828125e-04f * (nx + ynorm), 0.f) * fF;
        const bool ok = ((need & ~md) != 0ull) & (present > 0) & (lhs < bmax * (float)present);
        cand |= (unsigned)ok << j;
      }
    }
    // (b) queue the lane's candidates (donor order); the exact passes run batched over the wave
    if (__ballot(cand != 0u) == 0ull) continue;
    if (__ballot(qlen + __builtin_popcount(cand) > kQc) != 0ull) flush();
    while (cand) {
      const int j = __builtin_ctz(cand);
      cand &= cand - 1u;
      q_idx[wave][lane][qlen++] = d0 + (j & 3) + 8 * (j >> 2) + 4 * hh;
    }
  }
  flush();
  if constexpr (MODE == 0)
    if (active) knn_merge_slots(best, alt, r, bd, b2, bi);
}

// 32-bit words per donor of the prep buffer (bf16 items, then the FM-strided zero-filled f32 row) → *out
static int knn_mf_fm(int F) { return F <= 16 ? 16 : F <= 24 ? 24 : F <= 32 ? 32 : F <= 40 ? 40 : 48; }
void knn_mfma_item_words(int F, uintptr_t out) {
  const int FM = knn_mf_fm(F);
  *reinterpret_cast<long long*>(out) = (long long)(((7 * FM + 15) / 16) * 16 / 2 + FM);
}

void knn_mfma_prep(uintptr_t D, uintptr_t dmask, int nd, int F, uintptr_t items, uintptr_t ny, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 48, "knn_mfma_prep: 1 <= F <= 48");
  if (nd == 0) return;
  auto go = [&](auto fm) {
    constexpr int FM = decltype(fm)::value;
    using K = KnnMf<FM>;
    unsigned short* it = (unsigned short*)items;
    float* rows = reinterpret_cast<float*>(it + (size_t)nd * K::LP);
    hipLaunchKernelGGL(knn_mfma_prep_kernel<FM>, dim3((nd + 255) / 256), dim3(256), 0, as_stream(stream),
                       (const float*)D, (const unsigned long long*)dmask, nd, F, it, rows, (float*)ny);
  };
  const int FM = knn_mf_fm(F);
  if (FM == 16) go(std::integral_constant<int, 16>{});
  else if (FM == 24) go(std::integral_constant<int, 24>{});
  else if (FM == 32) go(std::integral_constant<int, 32>{});
  else if (FM == 40) go(std::integral_constant<int, 40>{});
  else go(std::integral_constant<int, 48>{});
  launch_check();
}

// knn_donors with the matrix-core filter; `items` / `ny` from knn_mfma_prep of the same donors
void knn_donors_mfma(uintptr_t R, uintptr_t rmask, int nr, uintptr_t D, uintptr_t dmask, int nd, int F,
                     uintptr_t slot_col, uintptr_t best, uintptr_t alt, uintptr_t cnt, int s0, uintptr_t items,
                     uintptr_t ny, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 48, "knn_donors_mfma: 1 <= F <= 48");
  (void)D;
  if (nr == 0 || nd == 0) return;
  hipStream_t st = as_stream(stream);
  HFENS_CHECK(hipMemsetAsync((void*)best, 0xFF, (size_t)nr * kKnnSlots * sizeof(unsigned long long), st));
  HFENS_CHECK(hipMemsetAsync((void*)alt, 0xFF, (size_t)nr * kKnnSlots * sizeof(unsigned), st));
  const int rpb = knn_mf_fm(F) >= 48 ? 128 : 256;   // receivers per workgroup (32 per wave)
  const int rb = (nr + rpb - 1) / rpb;
  // ≈ kWgs workgroups, ≥ kMinPer donors each: fewer, longer splits (each restarts the slots' filling
  // phase) beat a fuller grid down to 8k rows (scans: profiles/r5_runs/knn_mfma_grid.log, knn_mfma_small.log)
  static const int kWgs = getenv("HFENS_KNN_MFMA_WGS") ? atoi(getenv("HFENS_KNN_MFMA_WGS")) : 256;
  static const int kMinPer = getenv("HFENS_KNN_MFMA_MINPER") ? atoi(getenv("HFENS_KNN_MFMA_MINPER")) : 256;
  // no cap on a split's donor range: each split restarts the slots' filling phase (every donor a
  // candidate until the slots hold two), which at 1M rows cost more than the grid's width gained
  // (1M-row imputation 0.81 s at ≤ 16,384 donors per split, 0.71 at 32,768, 0.58 unsplit:
  // profiles/r5_runs/knn_split_range.log)
  static const int kRange = getenv("HFENS_KNN_MFMA_RANGE") ? atoi(getenv("HFENS_KNN_MFMA_RANGE")) : (1 << 30);
  int splits = kWgs / rb;
  const int by_range = (nd + kRange - 1) / kRange;
  if (splits < by_range) splits = by_range;
  const int max_splits = (nd + kMinPer - 1) / kMinPer;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int per = (nd + splits - 1) / splits;
  per = (per + 31) / 32 * 32;
  const int nsp = (nd + per - 1) / per;
  auto go = [&](auto fm) {
    constexpr int FM = decltype(fm)::value;
    using K = KnnMf<FM>;
    const unsigned short* it = (const unsigned short*)items;
    const float* rows = reinterpret_cast<const float*>(it + (size_t)nd * K::LP);
    static_assert(32 * K::WAVES == (FM >= 48 ? 128 : 256), "receivers per workgroup");
    hipLaunchKernelGGL(knn_donor_mfma_kernel<FM>, dim3(rb, nsp), dim3(64 * K::WAVES), 0, st, (const float*)R,
                       (const unsigned long long*)rmask, nr, rows, (const unsigned long long*)dmask, nd, F, per,
                       (const int*)slot_col, (unsigned long long*)best, (unsigned*)alt, (const int*)cnt, s0, it,
                       (const float*)ny);
  };
  const int FM = knn_mf_fm(F);
  if (FM == 16) go(std::integral_constant<int, 16>{});
  else if (FM == 24) go(std::integral_constant<int, 24>{});
  else if (FM == 32) go(std::integral_constant<int, 32>{});
  else if (FM == 40) go(std::integral_constant<int, 40>{});
  else go(std::integral_constant<int, 48>{});
  launch_check();
}

// ---- f64-exact donors: the f32 search above picks the same donor as the f64
// direct-difference mirror (models/imputer.py _impute_host: Σ over common features in feature
// order of fl((x−y)·(x−y)) in f64, × F / |common|, lowest index on ties) except where another
// donor's distance is within the f32 error of the best.  Those slots are found from the runner-up
// distance (alt) and re-decided in f64 over the donors whose f32 distance can reach the best:
//   knn_ambig : per (receiver, slot): ambiguous ⇔ alt ≤ d1 + W(d1), W a bound of the f32 distance
//               error (both distances, ×8 margin; a relative term and one in sqrt(d) scaled by the
//               per-column largest centred magnitudes, for near-duplicate rows); compacts the
//               ambiguous receivers, records each ambiguous slot's f32 threshold d1 + W;
//   knn_cand  : the f32 direct-difference scan again, over the ambiguous receivers only (grid
//               sized for every receiver, blocks past the device count exit at once), listing every
//               (slot, donor) pair inside the slot's window;
//   knn_eval  : the pairs in parallel (one thread each — a slot can have thousands of exact-tie
//               donors, far too many for its scanning thread): the f64 distance, compared with the
//               f32 winner's own (knn_ambig): at it, atomicMin of the index (exact ties: the lowest
//               index, as the mirror's argmin); below it, atomicMin of the new f64 minimum
//               (order-preserving u64 bits); then, for the slots where that happened (rare), the
//               lowest index at the new minimum.  A list overflow falls back to evaluating in the
//               scanning threads;
//   knn_commit: the slot's donor ← that index.
// Cost ≈ one f32 scan of the ambiguous receivers plus one f64 distance per window pair;
// the result does not depend on atomic arrival order.

__device__ __forceinline__ double knn_dist64(const double* __restrict__ x, unsigned long long mr,
                                             const double* __restrict__ y, unsigned long long md, int F);

__global__ __launch_bounds__(256) void knn_ambig_kernel(const unsigned long long* __restrict__ best,
                                                        const unsigned* __restrict__ alt,
                                                        const int* __restrict__ slot_col, int nr, int F,
                                                        const float* __restrict__ Mx, float* __restrict__ thr,
                                                        unsigned long long* __restrict__ dmin,
                                                        int* __restrict__ didx, int* __restrict__ rlist,
                                                        int* __restrict__ counts,
                                                        const double* __restrict__ R64,
                                                        const unsigned long long* __restrict__ rmask,
                                                        const double* __restrict__ D64,
                                                        const unsigned long long* __restrict__ dmask,
                                                        unsigned long long* __restrict__ dwin,
                                                        const int* __restrict__ cnt, int s0) {
  if (cnt != nullptr) {
    if (s0 >= cnt[1]) return;
    nr = cnt[0];
  }
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nr) return;
  const float mn = Mx[0], Ff = (float)F;   // ‖m‖: norm over columns of the largest centred magnitude
  bool any = false;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k) {
    const size_t e = (size_t)r * kKnnSlots + k;
    float t = -1.f;
    const unsigned long long b = best[e];
    if (slot_col[e] >= 0 && b != ~0ull) {
      const float d1 = __uint_as_float((unsigned)(b >> 32));
      // error of a scaled f32 distance d = (F/p)·Σ δ_f² with δ_f the difference of two f32-rounded
      // centred values: each δ_f is off by ≤ u(|x_f−c_f| + |y_f−c_f| + |δ_f|), u = 2^-24, so
      //   |Δd| ≤ 8u·‖m‖·sqrt(F·d) + (F+2)u·d + 4F²u²‖m‖²      (Cauchy–Schwarz, F/p ≤ F)
      // with m_f the largest centred magnitude of column f; ×2 for the two distances compared and
      // ×8 margin
      const float W = 0x1p-20f * (8.f * mn * sqrtf(Ff * d1) + (Ff + 2.f) * d1) + 0x1p-42f * Ff * Ff * mn * mn;
      const unsigned a = alt[e];
      if (a != 0xFFFFFFFFu && __uint_as_float(a) <= d1 + W) {
        t = d1 + W;
        any = true;
      }
    }
    thr[e] = t;
    // the f32 winner's own f64 distance: pass 0 looks for donors strictly below it (rare) and, at it,
    // for a lower index; only slots where something strictly below exists need pass 1
    unsigned long long w64 = ~0ull;
    int wi = 0x7fffffff;
    if (t >= 0.f) {
      wi = (int)(unsigned)(b & 0xFFFFFFFFull);
      w64 = (unsigned long long)__double_as_longlong(
          knn_dist64(R64 + (size_t)r * F, rmask[r], D64 + (size_t)wi * F, dmask[wi], F));
    }
    dwin[e] = w64;
    dmin[e] = w64;
    didx[e] = wi;
  }
  if (any) rlist[atomicAdd(&counts[0], 1)] = r;
}

// f64 distance of the mirror: common features in order, fl((x−y)·(x−y)) summed, × F / |common|
#pragma clang fp contract(off)
__device__ __forceinline__ double knn_dist64(const double* __restrict__ x, unsigned long long mr,
                                             const double* __restrict__ y, unsigned long long md, int F) {
  double s = 0.0;
  int present = 0;
  for (int f = 0; f < F; ++f) {
    if (((mr | md) >> f) & 1ull) continue;
    const double t = x[f] - y[f];
    s = s + t * t;
    ++present;
  }
  return present > 0 ? (s * (double)F) / (double)present : INFINITY;
}
#pragma clang fp contract(on)

// MODE 0: list every (slot, donor) inside a window into pairs (cap entries; counts[1] = pairs,
// counts[2] = overflow) for the parallel f64 evaluation below.  MODE 1 / 2: the serial fallback
// used only after an overflow (counts[2] ≠ 0) — pass 0 / pass 1 evaluated in the scanning thread.
template <int FMAX, int MODE>
__global__ __launch_bounds__(256) void knn_cand_kernel(
    const float* __restrict__ R, const unsigned long long* __restrict__ rmask, const int* __restrict__ rlist,
    const int* __restrict__ counts, const float* __restrict__ D, const unsigned long long* __restrict__ dmask,
    int nd, int F, int per_split, const int* __restrict__ slot_col, const float* __restrict__ thr,
    const double* __restrict__ R64, const double* __restrict__ D64, unsigned long long* __restrict__ dmin,
    int* __restrict__ didx, const unsigned long long* __restrict__ dwin, int* __restrict__ didx2,
    int* __restrict__ pairs, long long cap, int* __restrict__ pcount) {
  constexpr int LD = (FMAX + 3) / 4 * 4;
  if (MODE != 0 && pcount[1] == 0) return;   // (fallback only after an overflow)
  const int nrl = counts[0];
  if ((int)blockIdx.x * 256 >= nrl) return;   // (grid sized for every receiver)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* ds = sm;
  unsigned long long* dm = (unsigned long long*)(ds + kKnnTile * LD);
  const int li = blockIdx.x * 256 + threadIdx.x;
  const bool active = li < nrl;
  const int r = active ? rlist[li] : 0;
  const int d_begin = blockIdx.y * per_split;
  const int d_end = min(nd, d_begin + per_split);
  float xr[LD];
#pragma unroll
  for (int f = 0; f < LD; ++f) xr[f] = (active && f < F) ? R[(size_t)r * F + f] : 0.f;
  const unsigned long long mr = active ? rmask[r] : 0ull;
  int col[kKnnSlots];
  float th[kKnnSlots];
  unsigned long long need = 0ull;
  float tmax = -1.f;
#pragma unroll
  for (int k = 0; k < kKnnSlots; ++k) {
    const size_t e = (size_t)r * kKnnSlots + k;
    th[k] = active ? thr[e] : -1.f;
    col[k] = (active && th[k] >= 0.f) ? slot_col[e] : -1;
    if (col[k] >= 0) need |= 1ull << col[k];
    tmax = fmaxf(tmax, col[k] >= 0 ? th[k] : -1.f);
  }
  const double* x64 = R64 + (size_t)r * F;
  for (int d0 = d_begin; d0 < d_end; d0 += kKnnTile) {
    __syncthreads();
    const int nt = min(kKnnTile, d_end - d0);
    for (int e = threadIdx.x; e < nt * LD; e += 256) {
      const int rr = e / LD, c = e % LD;
      ds[e] = c < F ? D[(size_t)(d0 + rr) * F + c] : 0.f;
    }
    if (threadIdx.x < nt) dm[threadIdx.x] = dmask[d0 + threadIdx.x];
    __syncthreads();
    if (need == 0ull) continue;
    for (int t = 0; t < nt; ++t) {
      const unsigned long long md = dm[t];
      if ((need & ~md) == 0ull) continue;
      const float4* xd4 = reinterpret_cast<const float4*>(ds + t * LD);
      const unsigned long long both = ~(mr | md);
      const unsigned blo = (unsigned)both, bhi = (unsigned)(both >> 32);
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int q = 0; q < LD / 4; ++q) {
        if (4 * q < F) {
          const float4 v = xd4[q];
          const unsigned bq = ((4 * q < 32 ? blo >> (4 * q) : bhi >> (4 * q - 32))) & 0xFu;
          const float a = (bq & 1u) ? xr[4 * q] - v.x : 0.f;
          const float b = (bq & 2u) ? xr[4 * q + 1] - v.y : 0.f;
          const float c = (bq & 4u) ? xr[4 * q + 2] - v.z : 0.f;
          const float d = (bq & 8u) ? xr[4 * q + 3] - v.w : 0.f;
          s0 = fmaf(a, a, s0);
          s1 = fmaf(b, b, s1);
          s0 = fmaf(c, c, s0);
          s1 = fmaf(d, d, s1);
        }
      }
      const int present = F - __builtin_popcountll(mr | md);
      if (present <= 0) continue;
      const float dist = fmaxf(s0 + s1, 0.f) * ((float)F / (float)present);
      if (!(dist <= tmax)) continue;
      const int di = d0 + t;
      double d64 = -1.0;
#pragma unroll
      for (int k = 0; k < kKnnSlots; ++k) {
        if (col[k] >= 0 && !((md >> col[k]) & 1ull) && dist <= th[k]) {
          const size_t e = (size_t)r * kKnnSlots + k;
          if constexpr (MODE == 0) {
            const int p = atomicAdd(&pcount[0], 1);
            if (p < cap) {
              pairs[2 * (size_t)p] = (int)e;
              pairs[2 * (size_t)p + 1] = di;
            } else {
              pcount[1] = 1;
            }
          } else {
            if (d64 < 0.0) d64 = knn_dist64(x64, mr, D64 + (size_t)di * F, md, F);
            const unsigned long long key = (unsigned long long)__double_as_longlong(d64);   // d64 ≥ 0
            if constexpr (MODE == 1) {
              if (key < dwin[e]) atomicMin(&dmin[e], key);
              else if (key == dwin[e]) atomicMin(&didx[e], di);
            } else if (key == dmin[e]) {
              atomicMin(&didx2[e], di);
            }
          }
        }
      }
    }
  }
}

// the listed (slot, donor) pairs in parallel, one per thread: STAGE 0 — the f64 distance (kept),
// below the f32 winner's → atomicMin of the minimum, at it → of the index; STAGE 1 — at a smaller
// minimum (slots flagged by knn_pass1_list), the lowest index there
template <int STAGE>
__global__ __launch_bounds__(256) void knn_eval_kernel(const int* __restrict__ pairs, const int* __restrict__ pcount,
                                                       long long cap, const int* __restrict__ slot_col,
                                                       const double* __restrict__ R64,
                                                       const unsigned long long* __restrict__ rmask,
                                                       const double* __restrict__ D64,
                                                       const unsigned long long* __restrict__ dmask, int F,
                                                       unsigned long long* __restrict__ keys,
                                                       unsigned long long* __restrict__ dmin,
                                                       const unsigned long long* __restrict__ dwin,
                                                       int* __restrict__ didx, const float* __restrict__ thr2,
                                                       int* __restrict__ didx2) {
  const long long np = min((long long)pcount[0], cap);
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < np; p += (long long)gridDim.x * 256) {
    const size_t e = (size_t)pairs[2 * p];
    const int di = pairs[2 * p + 1];
    if constexpr (STAGE == 0) {
      const int r = (int)(e / kKnnSlots);
      const double d64 = knn_dist64(R64 + (size_t)r * F, rmask[r], D64 + (size_t)di * F, dmask[di], F);
      const unsigned long long key = (unsigned long long)__double_as_longlong(d64);
      keys[p] = key;
      if (key < dwin[e]) atomicMin(&dmin[e], key);
      else if (key == dwin[e]) atomicMin(&didx[e], di);
    } else {
      if (thr2[e] >= 0.f && keys[p] == dmin[e]) atomicMin(&didx2[e], di);
    }
  }
}

__global__ __launch_bounds__(256) void knn_pass1_list_kernel(const int* __restrict__ rlist, const int* __restrict__ counts,
                                                             const float* __restrict__ thr,
                                                             const unsigned long long* __restrict__ dmin,
                                                             const unsigned long long* __restrict__ dwin,
                                                             float* __restrict__ thr2, int* __restrict__ didx2,
                                                             int* __restrict__ rlist2, int* __restrict__ counts2) {
  const int nrl = counts[0];
  for (int w = blockIdx.x * 256 + threadIdx.x; w < nrl; w += gridDim.x * 256) {
    const int r = rlist[w];
    bool any = false;
#pragma unroll
    for (int k = 0; k < kKnnSlots; ++k) {
      const size_t e = (size_t)r * kKnnSlots + k;
      const bool need = thr[e] >= 0.f && dmin[e] < dwin[e];
      thr2[e] = need ? thr[e] : -1.f;
      didx2[e] = 0x7fffffff;
      any |= need;
    }
    if (any) rlist2[atomicAdd(&counts2[0], 1)] = r;
  }
}

__global__ __launch_bounds__(256) void knn_commit_kernel(const int* __restrict__ rlist, const int* __restrict__ counts,
                                                         const float* __restrict__ thr, const float* __restrict__ thr2,
                                                         const int* __restrict__ didx, const int* __restrict__ didx2,
                                                         unsigned long long* __restrict__ best) {
  const int nrl = counts[0];
  for (int w = blockIdx.x * 256 + threadIdx.x; w < nrl * kKnnSlots; w += gridDim.x * 256) {
    const size_t e = (size_t)rlist[w / kKnnSlots] * kKnnSlots + w % kKnnSlots;
    if (thr[e] < 0.f) continue;
    const int d = thr2[e] >= 0.f ? didx2[e] : didx[e];
    if (d != 0x7fffffff) best[e] = (best[e] & 0xFFFFFFFF00000000ull) | (unsigned long long)(unsigned)d;
  }
}

// work: 8-byte aligned scratch of knn_refine_work_words(nr) int32 words
// items / ny: knn_mfma_prep of the donors (0: none) — the window listing then runs on the matrix-core
// filter (knn_donor_mfma_kernel<·, 1>) instead of knn_cand_kernel's packed-FMA scan
static int knn_mf_fm(int F);
template <int FM>
static void knn_cand_mfma(const float* R, const unsigned long long* rmask, int nr, const unsigned long long* dmask,
                          int nd, int F, const int* slot_col, const int* rlist, const int* counts, const float* thr,
                          int* pairs, long long cap, int* pcount, const unsigned short* items, const float* ny,
                          hipStream_t st) {
  using K = KnnMf<FM>;
  const int rpb = 32 * K::WAVES;
  const int rb = (nr + rpb - 1) / rpb;
  int splits = (nd + 16383) / 16384;
  if (splits < 64) splits = 64;
  const int max_splits = (nd + 255) / 256;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int per = (nd + splits - 1) / splits;
  per = (per + 31) / 32 * 32;
  const int nsp = (nd + per - 1) / per;
  const float* rows = reinterpret_cast<const float*>(items + (size_t)nd * K::LP);
  hipLaunchKernelGGL((knn_donor_mfma_kernel<FM, 1>), dim3(rb, nsp), dim3(64 * K::WAVES), 0, st, R, rmask, nr, rows,
                     dmask, nd, F, per, slot_col, (unsigned long long*)nullptr, (unsigned*)nullptr, counts, 0, items,
                     ny, rlist, thr, pairs, cap, pcount);
}

void knn_refine(uintptr_t R, uintptr_t rmask, int nr, uintptr_t D, uintptr_t dmask, int nd, int F,
                uintptr_t slot_col, uintptr_t best, uintptr_t alt, uintptr_t R64, uintptr_t D64, uintptr_t Mx,
                uintptr_t work, long long cap, uintptr_t cnt, int s0, uintptr_t items, uintptr_t ny,
                uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "knn_refine: 1 <= F <= 64");
  HFENS_REQUIRE((work & 7) == 0 && cap >= 1, "knn_refine: work must be 8-byte aligned, cap >= 1");
  if (nr == 0 || nd == 0) return;
  hipStream_t st = as_stream(stream);
  // work (8-byte aligned): keys u64 [cap] | dmin | dwin u64 [nr·8] | didx | didx2 i32 [nr·8] |
  // thr | thr2 f32 [nr·8] | pairs i32 [2·cap] | rlist | rlist2 i32 [nr] | counts | counts2 | pcount i32 [4]
  const size_t ns = (size_t)nr * kKnnSlots;
  unsigned long long* keys = (unsigned long long*)work;
  unsigned long long* dmin = keys + cap;
  unsigned long long* dwin = dmin + ns;
  int* didx = (int*)(dwin + ns);
  int* didx2 = didx + ns;
  float* thr = (float*)(didx2 + ns);
  float* thr2 = thr + ns;
  int* pairs = (int*)(thr2 + ns);
  int* rlist = pairs + 2 * cap;
  int* rlist2 = rlist + nr;
  int* counts = rlist2 + nr;
  int* counts2 = counts + 4;
  int* pcount = counts2 + 4;
  HFENS_CHECK(hipMemsetAsync(counts, 0, 12 * sizeof(int), st));
  const int rb = (nr + 255) / 256;
  hipLaunchKernelGGL(knn_ambig_kernel, dim3(rb), dim3(256), 0, st, (const unsigned long long*)best,
                     (const unsigned*)alt, (const int*)slot_col, nr, F, (const float*)Mx, thr, dmin, didx, rlist,
                     counts, (const double*)R64, (const unsigned long long*)rmask, (const double*)D64,
                     (const unsigned long long*)dmask, dwin, (const int*)cnt, s0);
  launch_check();
  // donor splits as in knn_donors (≥ 2048 workgroups, ≤ 16k donors each); blocks past the device
  // receiver count exit at once
  int splits = 2048 / rb;
  const int by_range = (nd + 16383) / 16384;
  if (splits < by_range) splits = by_range;
  const int max_splits = (nd + kKnnTile - 1) / kKnnTile;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int eg = (int)((cap + 255) / 256);
  if (eg > 2048) eg = 2048;
  auto go = [&](auto fm) {
    constexpr int FM = decltype(fm)::value;
    constexpr int LD = (FM + 3) / 4 * 4;
    int per = (nd + splits - 1) / splits;
    per = (per + kKnnTile - 1) / kKnnTile * kKnnTile;
    const int nsp = (nd + per - 1) / per;
    const size_t lds = (size_t)kKnnTile * LD * sizeof(float) + kKnnTile * sizeof(unsigned long long);
    auto cand = [&](auto mode, const int* rl, const int* cn, const float* th) {
      constexpr int MD = decltype(mode)::value;
      hipLaunchKernelGGL((knn_cand_kernel<FM, MD>), dim3(rb, nsp), dim3(256), lds, st, (const float*)R,
                         (const unsigned long long*)rmask, rl, cn, (const float*)D, (const unsigned long long*)dmask,
                         nd, F, per, (const int*)slot_col, th, (const double*)R64, (const double*)D64, dmin, didx,
                         (const unsigned long long*)dwin, didx2, pairs, cap, pcount);
    };
    if (items != 0 && F <= 48) {                                          // list the window pairs
      const int fm = knn_mf_fm(F);
      auto mf = [&](auto k) {
        knn_cand_mfma<decltype(k)::value>((const float*)R, (const unsigned long long*)rmask, nr,
                                          (const unsigned long long*)dmask, nd, F, (const int*)slot_col, rlist,
                                          counts, thr, pairs, cap, pcount, (const unsigned short*)items,
                                          (const float*)ny, st);
      };
      if (fm == 16) mf(std::integral_constant<int, 16>{});
      else if (fm == 24) mf(std::integral_constant<int, 24>{});
      else if (fm == 32) mf(std::integral_constant<int, 32>{});
      else if (fm == 40) mf(std::integral_constant<int, 40>{});
      else mf(std::integral_constant<int, 48>{});
      launch_check();
    } else {
      cand(std::integral_constant<int, 0>{}, rlist, counts, thr);
    }
    hipLaunchKernelGGL(knn_eval_kernel<0>, dim3(eg), dim3(256), 0, st, (const int*)pairs, (const int*)pcount, cap,
                       (const int*)slot_col, (const double*)R64, (const unsigned long long*)rmask, (const double*)D64,
                       (const unsigned long long*)dmask, F, keys, dmin, (const unsigned long long*)dwin, didx,
                       (const float*)thr2, didx2);
    cand(std::integral_constant<int, 1>{}, rlist, counts, thr);          // (overflow only)
    int g1 = rb < 1024 ? rb : 1024;
    hipLaunchKernelGGL(knn_pass1_list_kernel, dim3(g1), dim3(256), 0, st, rlist, counts, thr, dmin,
                       (const unsigned long long*)dwin, thr2, didx2, rlist2, counts2);
    hipLaunchKernelGGL(knn_eval_kernel<1>, dim3(eg), dim3(256), 0, st, (const int*)pairs, (const int*)pcount, cap,
                       (const int*)slot_col, (const double*)R64, (const unsigned long long*)rmask, (const double*)D64,
                       (const unsigned long long*)dmask, F, keys, dmin, (const unsigned long long*)dwin, didx,
                       (const float*)thr2, didx2);
    cand(std::integral_constant<int, 2>{}, rlist2, counts2, thr2);       // (overflow only)
    launch_check();
  };
  if (F <= 16) go(std::integral_constant<int, 16>{});
  else if (F <= 32) go(std::integral_constant<int, 32>{});
  else if (F <= 40) go(std::integral_constant<int, 40>{});
  else if (F <= 48) go(std::integral_constant<int, 48>{});
  else go(std::integral_constant<int, 64>{});
  int grid = (nr * kKnnSlots + 255) / 256;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(knn_commit_kernel, dim3(grid), dim3(256), 0, st, rlist, counts, thr, thr2, didx, didx2,
                     (unsigned long long*)best);
  launch_check();
}

// ---- device planning of an imputation (no host read of the missing-value pattern) ----------------
// knn_plan_dev: rows of X [n][F] (f64, NaN = missing) with a missing feature, in row order (a
// per-256-row-block count, one scan block, then the writes): rows [n] i64, rbits [n] u64,
// slot [G][n][8] i32 (group g: the row's missing columns 8g … 8g+7 in column order, −1 padded),
// R32 [n][F] f32 (x − centre, 0 where missing), R64 [n][F] f64 (x, 0 where missing),
// colmax [F] f32 bits (max |R32| per column, atomicMax on the non-negative float bits),
// cnt [4] i32 = {nr, nslot (max missing per row rounded up to 8), nc, 0}.  Work: bcnt [nb] i32.
__global__ __launch_bounds__(256) void knn_plan_count_kernel(const double* __restrict__ X, long long n, int F,
                                                             int* __restrict__ bcnt, int* __restrict__ cnt) {
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  int m = 0;
  if (r < n)
    for (int f = 0; f < F; ++f) m += isnan(X[r * F + f]) ? 1 : 0;
  const unsigned long long b = __ballot(m > 0);
  int mx = m;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, kWave));
  __shared__ int wc[4], wm[4], wn[4];
  int nc = m;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nc += __shfl_xor(nc, o, kWave);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { wc[wave] = __popcll(b); wm[wave] = mx; wn[wave] = nc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    bcnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
    atomicMax(&cnt[1], max(max(wm[0], wm[1]), max(wm[2], wm[3])));
    atomicAdd(&cnt[2], wn[0] + wn[1] + wn[2] + wn[3]);
  }
}

// one workgroup: exclusive scan of the block counts in place, nr, nslot rounded up to 8
__global__ __launch_bounds__(1024) void knn_plan_scan_kernel(int* __restrict__ bcnt, int nb, int* __restrict__ cnt) {
  __shared__ int part[1024];
  const int per = (nb + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  int s = 0;
  for (int i = 0; i < per; ++i) s += (b0 + i < nb) ? bcnt[b0 + i] : 0;
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = part[threadIdx.x] - s;   // exclusive
  for (int i = 0; i < per; ++i) {
    if (b0 + i < nb) {
      const int c = bcnt[b0 + i];
      bcnt[b0 + i] = run;
      run += c;
    }
  }
  if (threadIdx.x == 1023) {
    cnt[0] = part[1023];
    cnt[1] = (cnt[1] + kKnnSlots - 1) / kKnnSlots * kKnnSlots;
  }
}

__global__ __launch_bounds__(256) void knn_plan_fill_kernel(const double* __restrict__ X, long long n, int F,
                                                            const double* __restrict__ centre,
                                                            const int* __restrict__ boff, int G,
                                                            long long* __restrict__ rows,
                                                            unsigned long long* __restrict__ rbits,
                                                            int* __restrict__ slot, float* __restrict__ R32,
                                                            double* __restrict__ R64, unsigned* __restrict__ colmax) {
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  unsigned long long bits = 0ull;
  if (r < n)
    for (int f = 0; f < F; ++f) bits |= (isnan(X[r * F + f]) ? 1ull : 0ull) << f;
  const unsigned long long b = __ballot(bits != 0ull);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ int wc[4];
  if (lane == 0) wc[wave] = __popcll(b);
  __syncthreads();
  if (bits == 0ull) return;
  int k = boff[blockIdx.x] + __popcll(b & ((1ull << lane) - 1ull));
  for (int w = 0; w < wave; ++w) k += wc[w];
  rows[k] = r;
  rbits[k] = bits;
  int s = 0;
  for (int f = 0; f < F; ++f) {
    const double x = X[r * F + f];
    const bool miss = (bits >> f) & 1ull;
    const float z = miss ? 0.f : (float)(x - centre[f]);
    R32[(size_t)k * F + f] = z;
    R64[(size_t)k * F + f] = miss ? 0.0 : x;
    if (!miss) atomicMax(&colmax[f], __float_as_uint(fabsf(z)));
    if (miss) {
      slot[((size_t)(s / kKnnSlots) * n + k) * kKnnSlots + s % kKnnSlots] = f;
      ++s;
    }
  }
  for (; s < G * kKnnSlots; ++s) slot[((size_t)(s / kKnnSlots) * n + k) * kKnnSlots + s % kKnnSlots] = -1;
}

// Mx[0] = ‖max(dmax, colmax)‖₂ (f64 sum of squares in column order, then f32): the refine's
// error-window scale (knn_ambig)
__global__ void knn_plan_mx_kernel(const float* __restrict__ dmax, const unsigned* __restrict__ colmax, int F,
                                   float* __restrict__ Mx) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int f = 0; f < F; ++f) {
    const double v = (double)fmaxf(dmax[f], __uint_as_float(colmax[f]));
    s += v * v;
  }
  Mx[0] = (float)sqrt(s);
}

void knn_plan_dev(uintptr_t X, long long n, int F, uintptr_t centre, uintptr_t dmax, uintptr_t rows, uintptr_t rbits,
                  uintptr_t slot, int G, uintptr_t R32, uintptr_t R64, uintptr_t colmax, uintptr_t Mx, uintptr_t cnt,
                  uintptr_t bcnt, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64 && G * kKnnSlots >= F && n >= 1, "knn_plan_dev: 1 <= F <= 64, G·8 >= F");
  hipStream_t st = as_stream(stream);
  const long long nb = (n + 255) / 256;
  HFENS_REQUIRE(nb <= (1LL << 30), "knn_plan_dev: too many rows");
  HFENS_CHECK(hipMemsetAsync((void*)cnt, 0, 4 * sizeof(int), st));
  HFENS_CHECK(hipMemsetAsync((void*)colmax, 0, (size_t)F * sizeof(unsigned), st));
  hipLaunchKernelGGL(knn_plan_count_kernel, dim3((unsigned)nb), dim3(256), 0, st, (const double*)X, n, F,
                     (int*)bcnt, (int*)cnt);
  hipLaunchKernelGGL(knn_plan_scan_kernel, dim3(1), dim3(1024), 0, st, (int*)bcnt, (int)nb, (int*)cnt);
  hipLaunchKernelGGL(knn_plan_fill_kernel, dim3((unsigned)nb), dim3(256), 0, st, (const double*)X, n, F,
                     (const double*)centre, (const int*)bcnt, G, (long long*)rows, (unsigned long long*)rbits,
                     (int*)slot, (float*)R32, (double*)R64, (unsigned*)colmax);
  hipLaunchKernelGGL(knn_plan_mx_kernel, dim3(1), dim3(64), 0, st, (const float*)dmax, (const unsigned*)colmax, F,
                     (float*)Mx);
  launch_check();
}

// X[rows[k], c] ← the donor's value (fitX [nd][F], NaN-free where the donor has c) or the column
// mean when no donor has a defined distance; best [G][n][8] packed (d² bits, donor), all-ones = none
__global__ __launch_bounds__(256) void knn_apply_kernel(double* __restrict__ X, long long n, int F,
                                                        const long long* __restrict__ rows,
                                                        const int* __restrict__ slot,
                                                        const unsigned long long* __restrict__ best,
                                                        const double* __restrict__ fitX,
                                                        const double* __restrict__ colmean,
                                                        const int* __restrict__ cnt) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k >= cnt[0]) return;
  const long long r = rows[k];
  const int G = cnt[1] / kKnnSlots;
  for (int g = 0; g < G; ++g) {
    for (int j = 0; j < kKnnSlots; ++j) {
      const size_t e = ((size_t)g * n + k) * kKnnSlots + j;
      const int c = slot[e];
      if (c < 0) continue;
      const unsigned long long b = best[e];
      const long long d = b == ~0ull ? -1 : (long long)(b & 0xFFFFFFFFull);
      X[r * F + c] = d >= 0 ? fitX[d * F + c] : colmean[c];
    }
  }
}

void knn_apply(uintptr_t X, long long n, int F, uintptr_t rows, uintptr_t slot, uintptr_t best, uintptr_t fitX,
               uintptr_t colmean, uintptr_t cnt, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64 && n >= 1, "knn_apply: bad shape");
  hipLaunchKernelGGL(knn_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), (double*)X,
                     n, F, (const long long*)rows, (const int*)slot, (const unsigned long long*)best,
                     (const double*)fitX, (const double*)colmean, (const int*)cnt);
  launch_check();
}

}  // namespace hfens
