// Tall-skinny f64 products of the interior-point SVC (models/svc_lowrank.py) over the Nyström
// map Φ [n][r] (n up to ~10⁶ rows, r ≤ 512 landmarks, row-major f64):
//
//  wsyrk_f64 : S = Φᵀ diag(d) Φ (r × r, symmetric).  Only the upper 128×128 tiles are computed
//              (10 of 16 for r = 512: 0.62 of the GEMM's flops) on v_mfma_f64_16x16x4_f64, with no
//              materialised diag(d)·Φ (the library path wrote and re-read a 4 GB scaled copy per
//              iteration).  grid = (upper tiles, row groups): every workgroup accumulates one tile
//              over its row group (split-K), staging 16-row slabs of the tile's two column blocks
//              through LDS (double-buffered, d applied while staging); per-group partial tiles are
//              summed in group order by wsyrk_reduce (deterministic) and mirrored to both triangles.
//  phi_gemv  : Y = Φ·W for W [r][k], k ≤ 4: one wave per row block, lanes own 8 consecutive
//              columns (one pass over Φ at HBM rate; the library ran these as N = 1–2 GEMMs).
//
// f64 MFMA 16x16x4 operand maps (gfx950): A[i = l&15][k = l>>4], B[k = l>>4][j = l&15];
// C/D col = l&15, row = (l>>4) + 4·reg (the f64 exception to the common C map).
#include <type_traits>

#include "common.h"

namespace hfens {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kSyT = 128;          // output tile
constexpr int kSyKC = 16;          // rows per LDS slab
constexpr int kSyLd = kSyT + 16;   // padded LDS row (f64): stride ≡ 32 banks, fragment reads split over bank halves
constexpr int kSyThreads = 256;    // 4 waves, 2×2 of 64×64

__global__ __launch_bounds__(kSyThreads) void wsyrk_f64_kernel(const double* __restrict__ Phi, const double* __restrict__ d,
                                                                long long n, int r, int nt, int T, int G,
                                                                long long rows_per_group, double* __restrict__ part) {
  __shared__ double As[2][kSyKC][kSyLd];
  __shared__ double Bs[2][kSyKC][kSyLd];
  // XCD-aware block map: workgroups are dispatched round-robin over the 8 XCDs, so block b runs
  // on XCD b & 7.  All T tiles of one row group go to the same XCD (consecutive q there), so the
  // group's rows are fetched from HBM once per group and re-read by its other tiles from that
  // XCD's L2 (a tile-fastest map spreads them over all 8 L2s).
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int gi = xcd + 8 * (q / T), tile = q % T;
  if (gi >= G) return;
  // upper tile index → (I, J), I ≤ J
  int t = tile, I = 0;
  while (t >= nt - I) { t -= nt - I; ++I; }
  const int J = I + t;
  const int c0a = I * kSyT, c0b = J * kSyT;
  const long long g = gi;
  const long long r0 = g * rows_per_group, r1 = min(n, r0 + rows_per_group);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
  f64x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
  // staging: 16 rows × 128 cols per operand = 2048 f64 = 8 per thread per operand; the next slab
  // is loaded into registers before this slab's MFMAs and written to LDS after them, so its
  // global-load latency hides under the matrix work
  // loads are branch-free (indices clamped into range, validity and the weight applied at the
  // LDS store), so all 24 of them issue back to back and ONE wait covers them
  double va[8], vb[8], vd[8];
  long long lrow0 = r0;
  auto load = [&](long long row0) {
    lrow0 = row0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + q * kSyThreads;
      const int rr = e >> 7, cc = e & 127;
      const long long row = min(row0 + rr, r1 - 1);
      const double* pr = Phi + row * r;
      va[q] = pr[min(c0a + cc, r - 1)];
      vb[q] = pr[min(c0b + cc, r - 1)];
      vd[q] = d[row];
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + q * kSyThreads;
      const int rr = e >> 7, cc = e & 127;
      const bool ok = lrow0 + rr < r1;
      As[buf][rr][cc] = (ok && c0a + cc < r) ? va[q] : 0.0;
      Bs[buf][rr][cc] = (ok && c0b + cc < r) ? vd[q] * vb[q] : 0.0;
    }
  };
  int buf = 0;
  if (r0 < r1) {
    load(r0);
    store(0);
  }
  __syncthreads();
  for (long long row0 = r0; row0 < r1; row0 += kSyKC) {
    const bool more = row0 + kSyKC < r1;
    if (more) load(row0 + kSyKC);
#pragma unroll
    for (int ks = 0; ks < kSyKC / 4; ++ks) {
      const int kr = 4 * ks + (lane >> 4);
      double a[4], b[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[q] = As[buf][kr][wr + 16 * q + (lane & 15)];
        b[q] = Bs[buf][kr][wc + 16 * q + (lane & 15)];
      }
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[p], b[q], acc[p][q], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // partial tile [128][128] of this (group, tile)
  double* out = part + ((size_t)g * T + tile) * kSyT * kSyT;
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = wr + 16 * p + (lane >> 4) + 4 * reg;
        const int col = wc + 16 * q + (lane & 15);
        out[row * kSyT + col] = acc[p][q][reg];
      }
}

// S[i][j] = S[j][i] = Σ_g part[g][tile(i, j)]  (group order: deterministic)
__global__ __launch_bounds__(256) void wsyrk_reduce_kernel(const double* __restrict__ part, int G, int T, int nt, int r,
                                                           double* __restrict__ S) {
  int t = blockIdx.x, I = 0;
  while (t >= nt - I) { t -= nt - I; ++I; }
  const int J = I + t;
  for (int e = blockIdx.y * 256 + threadIdx.x; e < kSyT * kSyT; e += gridDim.y * 256) {
    const int row = e >> 7, col = e & 127;
    const int i = I * kSyT + row, j = J * kSyT + col;
    if (i >= r || j >= r) continue;
    if (I == J && j < i) continue;   // diagonal tile: the upper half covers it
    double s = 0.0;
    for (int g = 0; g < G; ++g) s += part[((size_t)g * T + blockIdx.x) * kSyT * kSyT + e];
    S[(size_t)i * r + j] = s;
    S[(size_t)j * r + i] = s;
  }
}

// row groups of the split-K (models/svc_lowrank.py sizes the partial buffer with the same rule)
static int wsyrk_groups(long long n, int T) {
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  long long G = (2LL * ncu + T - 1) / T;                       // ≈ 2 workgroups per CU
  const long long max_g = (n + 4 * kSyKC - 1) / (4 * kSyKC);    // ≥ 4 slabs per group
  if (G > max_g) G = max_g;
  return (int)(G < 1 ? 1 : G);
}

void wsyrk_f64(uintptr_t Phi, uintptr_t d, long long n, int r, uintptr_t part, long long part_len, uintptr_t S,
               uintptr_t stream) {
  HFENS_REQUIRE(n >= 1 && r >= 1 && r <= 2048, "wsyrk_f64: n >= 1, 1 <= r <= 2048");
  const int nt = (r + kSyT - 1) / kSyT, T = nt * (nt + 1) / 2;
  const int G = wsyrk_groups(n, T);
  HFENS_REQUIRE(part_len >= (long long)G * T * kSyT * kSyT, "wsyrk_f64: partial buffer too small");
  long long per = (n + G - 1) / G;
  per = (per + kSyKC - 1) / kSyKC * kSyKC;
  hipStream_t st = as_stream(stream);
  const long long blocks = 8LL * ((G + 7) / 8) * T;
  hipLaunchKernelGGL(wsyrk_f64_kernel, dim3((unsigned)blocks), dim3(kSyThreads), 0, st, (const double*)Phi,
                     (const double*)d, n, r, nt, T, G, per, (double*)part);
  launch_check();
  hipLaunchKernelGGL(wsyrk_reduce_kernel, dim3(T, 16), dim3(256), 0, st, (const double*)part, G, T, nt, r,
                     (double*)S);
  launch_check();
}

// Y[i][q] = Σ_c Φ[i][c]·W[c][q], q < k ≤ 4.  Waves stride over rows (one 4 KB row per wave step:
// lane l owns columns 8l … 8l+7, r ≤ 512, with its W slice in registers); wave-sum per (row, q).
constexpr int kGvMaxK = 4;

template <int K>
__global__ __launch_bounds__(256) void phi_gemv_kernel(const double* __restrict__ Phi, const double* __restrict__ W,
                                                       long long n, int r, double* __restrict__ Y) {
  const int lane = threadIdx.x & 63;
  const long long wave = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const long long waves = (long long)gridDim.x * 4;
  double w[8][K];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const int c = 8 * lane + e;
      w[e][q] = c < r ? W[(size_t)c * K + q] : 0.0;
    }
  for (long long i = wave; i < n; i += waves) {
    const double* pr = Phi + i * r;
    double x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 8 * lane + e;
      x[e] = c < r ? pr[c] : 0.0;
    }
    double s[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
      double v = 0.0;
#pragma unroll
      for (int e = 0; e < 8; ++e) v = fma(x[e], w[e][q], v);
      s[q] = wave_sum(v);
    }
    if (lane < K) {
      double o = s[0];
#pragma unroll
      for (int q = 1; q < K; ++q)
        if (lane == q) o = s[q];
      Y[i * K + lane] = o;
    }
  }
}

void phi_gemv(uintptr_t Phi, uintptr_t W, long long n, int r, int k, uintptr_t Y, uintptr_t stream) {
  HFENS_REQUIRE(n >= 1 && r >= 1 && r <= 512 && k >= 1 && k <= kGvMaxK, "phi_gemv: r <= 512, 1 <= k <= 4");
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  long long blocks = (long long)ncu * 8;
  const long long need = (n + 3) / 4;
  if (blocks > need) blocks = need;
  hipStream_t st = as_stream(stream);
  auto go = [&](auto kk) {
    constexpr int K = decltype(kk)::value;
    hipLaunchKernelGGL(phi_gemv_kernel<K>, dim3((unsigned)blocks), dim3(256), 0, st, (const double*)Phi,
                       (const double*)W, n, r, (double*)Y);
    launch_check();
  };
  if (k == 1) go(std::integral_constant<int, 1>{});
  else if (k == 2) go(std::integral_constant<int, 2>{});
  else if (k == 3) go(std::integral_constant<int, 3>{});
  else go(std::integral_constant<int, 4>{});
}

}  // namespace hfens
