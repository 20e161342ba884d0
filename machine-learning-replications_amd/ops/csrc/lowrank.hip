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
#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

// ---- wsyrk_f32: the same product on the f32-input MFMA -------------------------
// Φ is exactly f32 (svc_lowrank rounds the Nyström map once), so the left operand A = Φ is exact;
// the right operand B = d ⊙ Φ is formed in f64 while staging and rounded to f32 (2⁻²⁴ relative per
// element).  v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation, 2× the f64 MFMA rate)
// accumulates kWfFlush rows at a time; those partial sums are then added into f64 registers, so the
// f32 rounding never spans more than 256 rows and the split-K partials and their reduction are f64
// (the same deterministic wsyrk_reduce as the f64 kernel).  Tile 128×128 per workgroup (4 waves,
// 2×2 of 64×64, each 2×2 MFMA blocks); a wave whose 64-column (or 64-row) half lies entirely past r
// skips its MFMAs, so the padding of r = 428 costs (448/428)², not (512/428)².
constexpr int kWfKC = 32;                 // rows per LDS slab
constexpr int kWfLd = kSyT + 4;           // padded LDS row (f32)
constexpr int kWfFlush = 256;             // rows per f32 accumulation before the f64 fold

__global__ __launch_bounds__(kSyThreads) void wsyrk_f32_kernel(const float* __restrict__ Phi, const double* __restrict__ d,
                                                                long long n, int r, int nt, int T, int G,
                                                                long long rows_per_group, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float As[2][kWfKC][kWfLd];
  __shared__ __attribute__((aligned(16))) float Bs[2][kWfKC][kWfLd];
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;   // (XCD-aware map: see wsyrk_f64_kernel)
  const int gi = xcd + 8 * (q / T), tile = q % T;
  if (gi >= G) return;
  int t = tile, I = 0;
  while (t >= nt - I) { t -= nt - I; ++I; }
  const int J = I + t;
  const int c0a = I * kSyT, c0b = J * kSyT;
  const long long r0 = (long long)gi * rows_per_group, r1 = min(n, r0 + rows_per_group);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
  const bool active = c0a + wr < r && c0b + wc < r;   // wave-uniform
  f32x16 acc[2][2];
  double accd[2][2][16];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      acc[a][b] = f32x16{0.f};
#pragma unroll
      for (int e = 0; e < 16; ++e) accd[a][b][e] = 0.0;
    }
  // staging: 32 rows × 128 columns per operand = 1024 float4, 4 per thread per operand; the next
  // slab's loads are issued before this slab's MFMAs and stored to LDS after them
  f32x4 va[4], vb[4];
  double vd[4];
  long long lrow0 = r0;
  auto load = [&](long long row0) {
    lrow0 = row0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * kSyThreads;
      const int rr = e >> 5, c4 = (e & 31) * 4;
      const long long row = min(row0 + rr, r1 - 1);
      const float* pr = Phi + row * r;
      va[u] = *reinterpret_cast<const f32x4*>(pr + min(c0a + c4, r - 4));
      vb[u] = *reinterpret_cast<const f32x4*>(pr + min(c0b + c4, r - 4));
      vd[u] = d[row];
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * kSyThreads;
      const int rr = e >> 5, c4 = (e & 31) * 4;
      const bool ok = lrow0 + rr < r1;
      const bool oka = ok && c0a + c4 < r, okb = ok && c0b + c4 < r;
      f32x4 a, b;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] = oka ? va[u][k] : 0.f;
        b[k] = okb ? (float)(vd[u] * (double)vb[u][k]) : 0.f;
      }
      *reinterpret_cast<f32x4*>(&As[buf][rr][c4]) = a;
      *reinterpret_cast<f32x4*>(&Bs[buf][rr][c4]) = b;
    }
  };
  int buf = 0;
  if (r0 < r1) {
    load(r0);
    store(0);
  }
  __syncthreads();
  int since = 0;
  for (long long row0 = r0; row0 < r1; row0 += kWfKC) {
    const bool more = row0 + kWfKC < r1;
    if (more) load(row0 + kWfKC);
    if (active) {
#pragma unroll
      for (int ks = 0; ks < kWfKC / 2; ++ks) {
        const int kr = 2 * ks + (lane >> 5);
        float a[2], b[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          a[p] = As[buf][kr][wr + 32 * p + (lane & 31)];
          b[p] = Bs[buf][kr][wc + 32 * p + (lane & 31)];
        }
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) acc[p][qq] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[p], b[qq], acc[p][qq], 0, 0, 0);
      }
      since += kWfKC;
      if (since >= kWfFlush || !more) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) {
#pragma unroll
            for (int e = 0; e < 16; ++e) accd[p][qq][e] += (double)acc[p][qq][e];
            acc[p][qq] = f32x16{0.f};
          }
        since = 0;
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // partial tile [128][128] of this (group, tile): the f32x16 C map, row = 8(e>>2) + 4(lane>>5) + (e&3)
  double* out = part + ((size_t)gi * T + tile) * kSyT * kSyT;
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int qq = 0; qq < 2; ++qq)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wr + 32 * p + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
        const int col = wc + 32 * qq + (lane & 31);
        out[row * kSyT + col] = active ? accd[p][qq][e] : 0.0;
      }
}

// ---- wsyrk_f64x: the f64 product read from the exact f32 copy of Φ -------------
// 64 × 64 output tiles (upper triangle only: 28 tiles for r = 428, padding (448/428)² instead of
// the 128-tile kernels' 40 blocks of 64²), 4 waves of 32 × 32 (2 × 2 f64 MFMA 16x16x4 blocks; the
// wave below the diagonal of a diagonal tile skips, the reduction reads only j ≥ i there), 32-row
// slabs staged through LDS with the next slab's loads in flight under this slab's MFMAs.  Φ is read as
// f32 (exact; half the bytes) and widened while staging; d ⊙ Φ is formed in f64; every product and
// sum is f64 — only the summation order differs from the library path.  Row groups (split-K) are
// XCD-aware as in wsyrk_f64_kernel; partial tiles are summed in group order (deterministic).
constexpr int kXT = 64;
constexpr int kXKC = 32;
constexpr int kXLd = kXT + 16;  // padded LDS row (f64): rows 32 banks apart, each half-wave read conflict-free

__global__ __launch_bounds__(kSyThreads, 2) void wsyrk_f64x_kernel(const float* __restrict__ Phi,
                                                                    const double* __restrict__ d, long long n, int r,
                                                                    int nt, int T, int G, long long rows_per_group,
                                                                    double* __restrict__ part) {
  __shared__ double As[kXKC][kXLd];
  __shared__ double Bs[kXKC][kXLd];
  const int xcd = blockIdx.x & 7, q = blockIdx.x >> 3;
  const int gi = xcd + 8 * (q / T), tile = q % T;
  if (gi >= G) return;
  int t = tile, I = 0;
  while (t >= nt - I) { t -= nt - I; ++I; }
  const int J = I + t;
  const int c0a = I * kXT, c0b = J * kXT;
  const long long r0 = (long long)gi * rows_per_group, r1 = min(n, r0 + rows_per_group);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const bool active = c0a + wr < r && c0b + wc < r && !(I == J && wr > wc);   // wave-uniform
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
  // staging: 32 rows × 64 columns per operand = 512 float4, 2 per thread per operand
  f32x4 va[2], vb[2];
  double vd[2];
  long long lrow0 = r0;
  auto load = [&](long long row0) {
    lrow0 = row0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * kSyThreads;
      const int rr = e >> 4, c4 = (e & 15) * 4;
      const long long row = min(row0 + rr, r1 - 1);
      const float* pr = Phi + row * r;
      va[u] = *reinterpret_cast<const f32x4*>(pr + min(c0a + c4, r - 4));
      vb[u] = *reinterpret_cast<const f32x4*>(pr + min(c0b + c4, r - 4));
      vd[u] = d[row];
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + u * kSyThreads;
      const int rr = e >> 4, c4 = (e & 15) * 4;
      const bool ok = lrow0 + rr < r1;
      const bool oka = ok && c0a + c4 < r, okb = ok && c0b + c4 < r;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        As[rr][c4 + k] = oka ? (double)va[u][k] : 0.0;
        Bs[rr][c4 + k] = okb ? vd[u] * (double)vb[u][k] : 0.0;
      }
    }
  };
  if (r0 < r1) load(r0);
  for (long long row0 = r0; row0 < r1; row0 += kXKC) {
    __syncthreads();   // the previous slab's operand reads are done
    store();
    __syncthreads();
    if (row0 + kXKC < r1) load(row0 + kXKC);   // the next slab's loads fly under this slab's MFMAs
    if (active) {
#pragma unroll
      for (int ks = 0; ks < kXKC / 4; ++ks) {
        const int kr = 4 * ks + (lane >> 4);
        double a[2], b[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          a[p] = As[kr][wr + 16 * p + (lane & 15)];
          b[p] = Bs[kr][wc + 16 * p + (lane & 15)];
        }
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) acc[p][qq] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[p], b[qq], acc[p][qq], 0, 0, 0);
      }
    }
  }
  double* out = part + ((size_t)gi * T + tile) * kXT * kXT;
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int qq = 0; qq < 2; ++qq)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = wr + 16 * p + (lane >> 4) + 4 * reg;
        const int col = wc + 16 * qq + (lane & 15);
        out[row * kXT + col] = active ? acc[p][qq][reg] : 0.0;
      }
}

__global__ __launch_bounds__(256) void wsyrk_x_reduce_kernel(const double* __restrict__ part, int G, int T, int nt,
                                                             int r, double* __restrict__ S) {
  int t = blockIdx.x, I = 0;
  while (t >= nt - I) { t -= nt - I; ++I; }
  const int J = I + t;
  for (int e = blockIdx.y * 256 + threadIdx.x; e < kXT * kXT; e += gridDim.y * 256) {
    const int row = e / kXT, col = e % kXT;
    const int i = I * kXT + row, j = J * kXT + col;
    if (i >= r || j >= r) continue;
    if (I == J && j < i) continue;
    double s = 0.0;
    for (int g = 0; g < G; ++g) s += part[((size_t)g * T + blockIdx.x) * kXT * kXT + e];
    S[(size_t)i * r + j] = s;
    S[(size_t)j * r + i] = s;
  }
}

// row groups of the split-K (the partial buffer is sized from wsyrk_part_len below)
static int wsyrk_groups(long long n, int T) {
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  long long G = (2LL * ncu + T - 1) / T;                       // ≈ 2 workgroups per CU
  const long long max_g = (n + 4 * kSyKC - 1) / (4 * kSyKC);    // ≥ 4 slabs per group
  if (G > max_g) G = max_g;
  return (int)(G < 1 ? 1 : G);
}

// partial-buffer lengths (f64 elements) of wsyrk_f64 / phit_f32: the Python side sizes its
// workspaces from these, never from a copy of the rules
void wsyrk_part_len(long long n, int r, uintptr_t out) {
  const int nt = (r + kSyT - 1) / kSyT, T = nt * (nt + 1) / 2;
  long long len = (long long)wsyrk_groups(n, T) * T * kSyT * kSyT;
  // the 64-tile kernel's partials (wsyrk_f64x): ≤ its workgroup budget + one group of tiles
  const int ntx = (r + 63) / 64, Tx = ntx * (ntx + 1) / 2;
  const int wgs = getenv("HFENS_WSYRKX_WGS") ? atoi(getenv("HFENS_WSYRKX_WGS")) : 2048;
  const long long lx = (long long)((wgs + Tx - 1) / Tx) * Tx * 64 * 64;
  *reinterpret_cast<long long*>(out) = len > lx ? len : lx;
}

// launch shape of the skinny passes: rows in flight per thread / wave, and the grid (sweep knobs
// of scripts/probes/skinny_probe.py: HFENS_PHIT_CFG / HFENS_GEMV_CFG = "rows,grid")
struct SkinnyCfg { int rows, grid; };
static SkinnyCfg skinny_cfg(const char* env, int rows, int grid) {
  SkinnyCfg c{rows, grid};
  if (const char* e = std::getenv(env)) {
    int a = 0, b = 0;
    if (std::sscanf(e, "%d,%d", &a, &b) == 2) { c.rows = a; c.grid = b; }
  }
  return c;
}

template <int K, int R>
__global__ void phit_flat_kernel(const float* __restrict__, const double* __restrict__, long long, int, long long,
                                 double* __restrict__);

// phit launch: the flat kernel (HFENS_PHIT_CFG "R,0", the default: R rows in flight per thread,
// the grid exactly the resident workgroups) or the row-slab kernel ("R,w": w workgroups per CU).
// The partial buffer is sized from phit_groups through phit_part_len, so both sides agree.
static int phit_flat_rows() {
  const SkinnyCfg c = skinny_cfg("HFENS_PHIT_CFG", 4, 0);
  return c.grid == 0 ? (c.rows == 8 ? 8 : (c.rows == 2 ? 2 : 4)) : 0;
}

template <int K, int R>
static long long phit_flat_groups(long long n, int r, int ncu) {
  int per_cu = 1;
  HFENS_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, phit_flat_kernel<K, R>, 256, 0));
  const long long need = std::max(1LL, ((long long)n * (r / 4) + 256LL * 4 * R - 1) / (256LL * 4 * R));
  return std::min((long long)ncu * std::max(1, per_cu), need);
}

static long long phit_groups(long long n, int r, int k) {
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int R = phit_flat_rows();
  if (R > 0 && r % 4 == 0) {
    auto byk = [&](auto rr) -> long long {
      constexpr int RR = decltype(rr)::value;
      if (k == 1) return phit_flat_groups<1, RR>(n, r, ncu);
      if (k == 2) return phit_flat_groups<2, RR>(n, r, ncu);
      if (k == 3) return phit_flat_groups<3, RR>(n, r, ncu);
      return phit_flat_groups<4, RR>(n, r, ncu);
    };
    if (R == 8) return byk(std::integral_constant<int, 8>{});
    if (R == 2) return byk(std::integral_constant<int, 2>{});
    return byk(std::integral_constant<int, 4>{});
  }
  if (n < 1024 * 64) return (n + 63) / 64;
  const int wpc = skinny_cfg("HFENS_PHIT_CFG", 4, 0).grid;
  return (long long)ncu * std::min(16, std::max(1, wpc));
}

void phit_part_len(long long n, int r, int k, uintptr_t out) {
  *reinterpret_cast<long long*>(out) = phit_groups(n, r, k) * r * k;
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

// S = Φᵀ diag(d) Φ from the f32 copy of Φ (wsyrk_f32_kernel); the same partial layout, row
// groups and reduction as wsyrk_f64 (part_len from wsyrk_part_len).
void wsyrk_f32(uintptr_t Phi, uintptr_t d, long long n, int r, uintptr_t part, long long part_len, uintptr_t S,
               uintptr_t stream) {
  HFENS_REQUIRE(n >= 1 && r >= 4 && r <= 2048 && r % 4 == 0, "wsyrk_f32: n >= 1, 4 <= r <= 2048, r % 4 == 0");
  HFENS_REQUIRE((Phi & 15) == 0, "wsyrk_f32: Φ must be 16-byte aligned");
  const int nt = (r + kSyT - 1) / kSyT, T = nt * (nt + 1) / 2;
  const int G = wsyrk_groups(n, T);
  HFENS_REQUIRE(part_len >= (long long)G * T * kSyT * kSyT, "wsyrk_f32: partial buffer too small");
  long long per = (n + G - 1) / G;
  per = (per + kWfKC - 1) / kWfKC * kWfKC;
  hipStream_t st = as_stream(stream);
  const long long blocks = 8LL * ((G + 7) / 8) * T;
  hipLaunchKernelGGL(wsyrk_f32_kernel, dim3((unsigned)blocks), dim3(kSyThreads), 0, st, (const float*)Phi,
                     (const double*)d, n, r, nt, T, G, per, (double*)part);
  launch_check();
  hipLaunchKernelGGL(wsyrk_reduce_kernel, dim3(T, 16), dim3(256), 0, st, (const double*)part, G, T, nt, r,
                     (double*)S);
  launch_check();
}

// S = Φᵀ diag(d) Φ in f64 from the exact f32 copy of Φ (wsyrk_f64x_kernel); the same partial layout,
// row groups and reduction as wsyrk_f64 (part_len from wsyrk_part_len).
void wsyrk_f64x(uintptr_t Phi, uintptr_t d, long long n, int r, uintptr_t part, long long part_len, uintptr_t S,
                uintptr_t stream) {
  HFENS_REQUIRE(n >= 1 && r >= 4 && r <= 2048 && r % 4 == 0, "wsyrk_f64x: n >= 1, 4 <= r <= 2048, r % 4 == 0");
  HFENS_REQUIRE((Phi & 15) == 0, "wsyrk_f64x: Φ must be 16-byte aligned");
  const int nt = (r + kXT - 1) / kXT, T = nt * (nt + 1) / 2;
  static const int kWgs = getenv("HFENS_WSYRKX_WGS") ? atoi(getenv("HFENS_WSYRKX_WGS")) : 2048;
  long long G = (kWgs + T - 1) / T;
  const long long max_g = (n + 4 * kXKC - 1) / (4 * kXKC);
  if (G > max_g) G = max_g;
  if (G < 1) G = 1;
  HFENS_REQUIRE(part_len >= G * T * kXT * kXT, "wsyrk_f64x: partial buffer too small");
  long long per = (n + G - 1) / G;
  per = (per + kXKC - 1) / kXKC * kXKC;
  hipStream_t st = as_stream(stream);
  const long long blocks = 8LL * ((G + 7) / 8) * T;
  hipLaunchKernelGGL(wsyrk_f64x_kernel, dim3((unsigned)blocks), dim3(kSyThreads), 0, st, (const float*)Phi,
                     (const double*)d, n, r, nt, T, (int)G, per, (double*)part);
  launch_check();
  hipLaunchKernelGGL(wsyrk_x_reduce_kernel, dim3(T, 4), dim3(256), 0, st, (const double*)part, (int)G, T, nt, r,
                     (double*)S);
  launch_check();
}

// Y[i][q] = Σ_c Φ[i][c]·W[c][q], q < k ≤ 4.  Waves stride over rows (one 4 KB row per wave step:
// lane l owns columns 8l … 8l+7, r ≤ 512, with its W slice in registers); wave-sum per (row, q).
constexpr int kGvMaxK = 4;

// CONTIG: lane l owns columns 4l … 4l+3 and 256 + 4l … (each float4 load instruction reads one
// contiguous 1 KB run of the row) instead of 8l … 8l+7 (two half-used runs)
template <int K, typename TP, int kGvRows, bool CONTIG = false>
__global__ __launch_bounds__(256) void phi_gemv_kernel(const TP* __restrict__ Phi, const double* __restrict__ W,
                                                       long long n, int r, double* __restrict__ Y) {
  const int lane = threadIdx.x & 63;
  const long long wave = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const long long waves = (long long)gridDim.x * 4;
  const bool vec4 = (r & 3) == 0 && (reinterpret_cast<uintptr_t>(Phi) & 15) == 0;
  double w[8][K];
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const int c = CONTIG ? 4 * lane + 256 * (e >> 2) + (e & 3) : 8 * lane + e;
      w[e][q] = c < r ? W[(size_t)c * K + q] : 0.0;
    }
  // kGvRows rows per wave step: their loads are issued together (the pass is bound by bytes in
  // flight per wave, not by arithmetic)
  for (long long i0 = wave * kGvRows; i0 < n; i0 += waves * kGvRows) {
    double x[kGvRows][8];
#pragma unroll
    for (int u = 0; u < kGvRows; ++u) {
      const long long i = i0 + u;
      const TP* pr = Phi + (i < n ? i : 0) * r;
      if constexpr (sizeof(TP) == 4) {
        if (vec4) {   // two 16-byte loads per lane (8 columns): the pass is load-instruction bound
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int c = CONTIG ? 4 * lane + 256 * h : 8 * lane + 4 * h;
            const float4 v = (i < n && c < r) ? *reinterpret_cast<const float4*>(pr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            x[u][4 * h] = v.x; x[u][4 * h + 1] = v.y; x[u][4 * h + 2] = v.z; x[u][4 * h + 3] = v.w;
          }
          continue;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = CONTIG ? 4 * lane + 256 * (e >> 2) + (e & 3) : 8 * lane + e;
        x[u][e] = (i < n && c < r) ? (double)pr[c] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < kGvRows; ++u) {
      const long long i = i0 + u;
      double s[K];
#pragma unroll
      for (int q = 0; q < K; ++q) {
        double v = 0.0;
#pragma unroll
        for (int e = 0; e < 8; ++e) v = fma(x[u][e], w[e][q], v);
        s[q] = wave_sum(v);
      }
      if (lane < K && i < n) {
        double o = s[0];
#pragma unroll
        for (int q = 1; q < K; ++q)
          if (lane == q) o = s[q];
        Y[i * K + lane] = o;
      }
    }
  }
}

static void phi_gemv_any(const void* Phi, bool f32, uintptr_t W, long long n, int r, int k, uintptr_t Y,
                         uintptr_t stream) {
  HFENS_REQUIRE(n >= 1 && r >= 1 && r <= 512 && k >= 1 && k <= kGvMaxK, "phi_gemv: r <= 512, 1 <= k <= 4");
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const SkinnyCfg cfg = skinny_cfg("HFENS_GEMV_CFG", 2, 3);   // 2 rows per wave, contiguous, resident grid
  hipStream_t st = as_stream(stream);
  auto launch = [&](auto kern, int rows) {
    long long blocks = (long long)ncu * 8;
    if (cfg.grid == 1 || cfg.grid == 3) {   // exactly the resident workgroups: no second, partial round of waves
      int per_cu = 1;
      HFENS_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0));
      blocks = (long long)ncu * std::max(1, per_cu);
    }
    const long long need = (n + 4 * rows - 1) / (4 * rows);
    if (blocks > need) blocks = need;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, (const float*)Phi, (const double*)W, n, r,
                       (double*)Y);
    launch_check();
  };
  auto go = [&](auto kk) {
    constexpr int K = decltype(kk)::value;
    if (!f32) {
      long long blocks = (long long)ncu * 8;
      const long long need = (n + 15) / 16;
      if (blocks > need) blocks = need;
      hipLaunchKernelGGL((phi_gemv_kernel<K, double, 4>), dim3((unsigned)blocks), dim3(256), 0, st, (const double*)Phi,
                         (const double*)W, n, r, (double*)Y);
      launch_check();
      return;
    }
    if (cfg.grid == 3) {   // contiguous lane → column map, resident grid
      if (cfg.rows == 4) launch(phi_gemv_kernel<K, float, 4, true>, 4);
      else launch(phi_gemv_kernel<K, float, 2, true>, 2);
      return;
    }
    if (cfg.rows == 8) launch(phi_gemv_kernel<K, float, 8>, 8);
    else if (cfg.rows == 2) launch(phi_gemv_kernel<K, float, 2>, 2);
    else launch(phi_gemv_kernel<K, float, 4>, 4);
  };
  if (k == 1) go(std::integral_constant<int, 1>{});
  else if (k == 2) go(std::integral_constant<int, 2>{});
  else if (k == 3) go(std::integral_constant<int, 3>{});
  else go(std::integral_constant<int, 4>{});
}

void phi_gemv(uintptr_t Phi, uintptr_t W, long long n, int r, int k, uintptr_t Y, uintptr_t stream) {
  phi_gemv_any((const void*)Phi, false, W, n, r, k, Y, stream);
}

// Φ stored as f32 (the IPM's skinny passes are HBM-bound: half the bytes), f64 arithmetic.
void phi_gemv_f32(uintptr_t Phi, uintptr_t W, long long n, int r, int k, uintptr_t Y, uintptr_t stream) {
  phi_gemv_any((const void*)Phi, true, W, n, r, k, Y, stream);
}

// out[c][q] = Σ_i Φ[i][c]·V[i][q] (Φᵀ V, V [n][k], k ≤ 4) with Φ in f32, f64 arithmetic: workgroup g
// sums its row slab (thread t owns columns t and t + 256; 4 rows in flight; V rows are uniform loads)
// into a partial [r][k] slot, and a second launch adds the G slots in slot order (deterministic).
template <int K, int kPtRows>
__global__ __launch_bounds__(256) void phit_f32_kernel(const float* __restrict__ Phi, const double* __restrict__ V,
                                                       long long n, int r, long long per, double* __restrict__ part) {
  // thread t: columns 4·(t % 128) … +3 (one 16-byte load per row), row stream t / 128 (rows of the
  // slab alternate between the two halves of the workgroup: waves 0–1 and 2–3, so each wave's V
  // reads are uniform); kPtRows rows in flight per thread
  const int t = threadIdx.x, cb = t & 127, rs = t >> 7;
  const int c = 4 * cb;
  const bool act = c < r;
  const long long i0 = (long long)blockIdx.x * per, i1 = i0 + per < n ? i0 + per : n;
  double acc[4][K];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int q = 0; q < K; ++q) acc[e][q] = 0.0;
  long long i = i0 + rs;
  for (; i + 2 * (kPtRows - 1) < i1; i += 2 * kPtRows) {
    float4 x[kPtRows];
    double v[kPtRows][K];
#pragma unroll
    for (int u = 0; u < kPtRows; ++u) {
      x[u] = act ? *reinterpret_cast<const float4*>(Phi + (i + 2 * u) * r + c) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < K; ++q) v[u][q] = V[(i + 2 * u) * K + q];
    }
#pragma unroll
    for (int u = 0; u < kPtRows; ++u)
#pragma unroll
      for (int q = 0; q < K; ++q) {
        acc[0][q] = fma((double)x[u].x, v[u][q], acc[0][q]);
        acc[1][q] = fma((double)x[u].y, v[u][q], acc[1][q]);
        acc[2][q] = fma((double)x[u].z, v[u][q], acc[2][q]);
        acc[3][q] = fma((double)x[u].w, v[u][q], acc[3][q]);
      }
  }
  for (; i < i1; i += 2) {
    const float4 x = act ? *reinterpret_cast<const float4*>(Phi + i * r + c) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const double vq = V[i * K + q];
      acc[0][q] = fma((double)x.x, vq, acc[0][q]);
      acc[1][q] = fma((double)x.y, vq, acc[1][q]);
      acc[2][q] = fma((double)x.z, vq, acc[2][q]);
      acc[3][q] = fma((double)x.w, vq, acc[3][q]);
    }
  }
  // row stream 1 hands its sums to stream 0 through LDS (fixed order: deterministic)
  __shared__ double sh[128][4 * kGvMaxK];
  if (rs == 1)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int q = 0; q < K; ++q) sh[cb][e * K + q] = acc[e][q];
  __syncthreads();
  if (rs == 0 && act) {
    double* slot = part + (size_t)blockIdx.x * r * K;
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int q = 0; q < K; ++q)
        if (c + e < r) slot[(size_t)(c + e) * K + q] = acc[e][q] + sh[cb][e * K + q];
  }
}

// Φᵀ V over Φ as one flat stream of float4s (r % 4 == 0): grid thread g takes elements g, g + S,
// g + 2S, … with S a multiple of r/4, so its column group (g mod r/4) never changes and its rows
// advance by S/(r/4); every lane of every load is active and a wave's load is 1 KB contiguous.
// A workgroup's threads of one column group meet in LDS in thread order (deterministic), one
// partial [r][k] slot per workgroup as in phit_f32_kernel.
template <int K, int R>
__global__ __launch_bounds__(256) void phit_flat_kernel(const float* __restrict__ Phi, const double* __restrict__ V,
                                                        long long n, int r4, long long S, double* __restrict__ part) {
  const int t = threadIdx.x;
  const long long g = (long long)blockIdx.x * 256 + t;
  const long long Sq = S / r4;
  double acc[4][K];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int q = 0; q < K; ++q) acc[e][q] = 0.0;
  if (g < S) {
    const float4* P4 = reinterpret_cast<const float4*>(Phi);
    const long long c4 = g % r4;
    long long i = g / r4;
    for (; i + (R - 1) * Sq < n; i += R * Sq) {
      float4 x[R];
      double v[R][K];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const long long iu = i + u * Sq;
        x[u] = P4[iu * r4 + c4];
#pragma unroll
        for (int q = 0; q < K; ++q) v[u][q] = V[iu * K + q];
      }
#pragma unroll
      for (int u = 0; u < R; ++u)
#pragma unroll
        for (int q = 0; q < K; ++q) {
          acc[0][q] = fma((double)x[u].x, v[u][q], acc[0][q]);
          acc[1][q] = fma((double)x[u].y, v[u][q], acc[1][q]);
          acc[2][q] = fma((double)x[u].z, v[u][q], acc[2][q]);
          acc[3][q] = fma((double)x[u].w, v[u][q], acc[3][q]);
        }
    }
    for (; i < n; i += Sq) {
      const float4 x = P4[i * r4 + c4];
#pragma unroll
      for (int q = 0; q < K; ++q) {
        const double vq = V[i * K + q];
        acc[0][q] = fma((double)x.x, vq, acc[0][q]);
        acc[1][q] = fma((double)x.y, vq, acc[1][q]);
        acc[2][q] = fma((double)x.z, vq, acc[2][q]);
        acc[3][q] = fma((double)x.w, vq, acc[3][q]);
      }
    }
  }
  __shared__ double sh[256][4 * K];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int q = 0; q < K; ++q) sh[t][e * K + q] = acc[e][q];
  __syncthreads();
  if (t < r4) {
    const long long g0 = (long long)blockIdx.x * 256;
    const int cg = (int)((g0 + t) % r4);
    double* slot = part + (size_t)blockIdx.x * 4 * r4 * K;
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int q = 0; q < K; ++q) {
        double sum = 0.0;
        for (int tt = t; tt < 256; tt += r4) sum += sh[tt][e * K + q];
        slot[(size_t)(4 * cg + e) * K + q] = sum;
      }
  }
}

// one wave per output element: lanes take every 64th partial, then a wave sum (fixed order:
// deterministic)
__global__ __launch_bounds__(256) void phit_reduce_kernel(const double* __restrict__ part, int G, long long m,
                                                          double* __restrict__ out) {
  const long long e = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (e >= m) return;
  double s = 0.0;
  for (int g = lane; g < G; g += 64) s += part[(size_t)g * m + e];
  s = wave_sum(s);
  if (lane == 0) out[e] = s;
}

void phit_f32(uintptr_t Phi, uintptr_t V, long long n, int r, int k, uintptr_t part, long long part_len, uintptr_t out,
              uintptr_t stream) {
  HFENS_REQUIRE(n >= 1 && r >= 1 && r <= 512 && r % 4 == 0 && k >= 1 && k <= kGvMaxK && (Phi & 15) == 0,
                "phit_f32: r <= 512, r % 4 == 0, 16-byte aligned Φ, 1 <= k <= 4");
  const long long G = phit_groups(n, r, k);
  HFENS_REQUIRE(part_len >= G * r * k, "phit_f32: partial buffer too small (size it with phit_part_len)");
  const long long per = (n + G - 1) / G;
  hipStream_t st = as_stream(stream);
  const int R = phit_flat_rows();
  const int rows = skinny_cfg("HFENS_PHIT_CFG", 4, 0).rows;
  const int r4 = r / 4;
  const long long S = G * 256 - (G * 256) % r4;   // a multiple of r/4: each thread keeps its column group
  auto go = [&](auto kk) {
    constexpr int K = decltype(kk)::value;
    if (R == 8)
      hipLaunchKernelGGL((phit_flat_kernel<K, 8>), dim3((unsigned)G), dim3(256), 0, st, (const float*)Phi,
                         (const double*)V, n, r4, S, (double*)part);
    else if (R == 2)
      hipLaunchKernelGGL((phit_flat_kernel<K, 2>), dim3((unsigned)G), dim3(256), 0, st, (const float*)Phi,
                         (const double*)V, n, r4, S, (double*)part);
    else if (R == 4)
      hipLaunchKernelGGL((phit_flat_kernel<K, 4>), dim3((unsigned)G), dim3(256), 0, st, (const float*)Phi,
                         (const double*)V, n, r4, S, (double*)part);
    else if (rows == 8)
      hipLaunchKernelGGL((phit_f32_kernel<K, 8>), dim3((unsigned)G), dim3(256), 0, st, (const float*)Phi,
                         (const double*)V, n, r, per, (double*)part);
    else
      hipLaunchKernelGGL((phit_f32_kernel<K, 4>), dim3((unsigned)G), dim3(256), 0, st, (const float*)Phi,
                         (const double*)V, n, r, per, (double*)part);
    launch_check();
  };
  if (k == 1) go(std::integral_constant<int, 1>{});
  else if (k == 2) go(std::integral_constant<int, 2>{});
  else if (k == 3) go(std::integral_constant<int, 3>{});
  else go(std::integral_constant<int, 4>{});
  const long long m = (long long)r * k;
  hipLaunchKernelGGL(phit_reduce_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, st, (const double*)part,
                     (int)G, m, (double*)out);
  launch_check();
}

// out[0 … n) = *src: a device scalar (an interior-point step length, a 0-dim torch tensor) as a dense
// vector without a host read — torch's own broadcast of a 0-dim device tensor over 10⁶ f64 ran at
// 63–193 µs per op against ≈ 5 µs for this write.
__global__ __launch_bounds__(256) void fill_dev_kernel(double* __restrict__ out, long long n, const double* __restrict__ src) {
  const double v = *src;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) out[i] = v;
}

void fill_dev(uintptr_t out, long long n, uintptr_t src, uintptr_t stream) {
  HFENS_REQUIRE(n >= 1, "fill_dev: n >= 1");
  long long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(fill_dev_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), (double*)out, n,
                     (const double*)src);
  launch_check();
}

// ---- the interior point's step-length bound in ONE pass (models/svc_lowrank.py step_len):
// min over the 4 (v, dv) pairs and all rows of −v_i / dv_i where dv_i < 0 (the pair's dv scaled by
// sign[k] = ±1: the slack pair uses −Δα), capped at 1.  The same IEEE quotient as the torch
// expression it replaces (and min is exact), so the step lengths are bit-identical; ~45 small torch
// launches per call become two.  Ratios are ≥ 0, so their f64 bit patterns order as unsigned ints:
// the block minima merge with a 64-bit atomicMin into *out (pre-set to 1.0).
__global__ __launch_bounds__(256) void ipm_max_step_kernel(const double* __restrict__ v0, const double* __restrict__ d0,
                                                           const double* __restrict__ v1, const double* __restrict__ d1,
                                                           const double* __restrict__ v2, const double* __restrict__ d2,
                                                           const double* __restrict__ v3, const double* __restrict__ d3,
                                                           double s0, double s1, double s2, double s3, long long n,
                                                           unsigned long long* __restrict__ out) {
  double m = 1.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double a0 = s0 * d0[i], a1 = s1 * d1[i], a2 = s2 * d2[i], a3 = s3 * d3[i];
    if (a0 < 0.0) m = fmin(m, -v0[i] / a0);
    if (a1 < 0.0) m = fmin(m, -v1[i] / a1);
    if (a2 < 0.0) m = fmin(m, -v2[i] / a2);
    if (a3 < 0.0) m = fmin(m, -v3[i] / a3);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o, 64));
  __shared__ double wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmin(fmin(wm[0], wm[1]), fmin(wm[2], wm[3]));
    atomicMin(out, (unsigned long long)__double_as_longlong(m));
  }
}

void ipm_max_step(uintptr_t v0, uintptr_t d0, uintptr_t v1, uintptr_t d1, uintptr_t v2, uintptr_t d2, uintptr_t v3,
                  uintptr_t d3, double s0, double s1, double s2, double s3, long long n, uintptr_t out,
                  uintptr_t stream) {
  if (n <= 0) return;
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  long long blocks = (n + 255) / 256;
  if (blocks > 4LL * ncu) blocks = 4LL * ncu;
  hipLaunchKernelGGL(ipm_max_step_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), (const double*)v0,
                     (const double*)d0, (const double*)v1, (const double*)d1, (const double*)v2, (const double*)d2,
                     (const double*)v3, (const double*)d3, s0, s1, s2, s3, n, (unsigned long long*)out);
  launch_check();
}

// ---- the interior point's per-row direction algebra, fused (models/svc_lowrank.py ipm_svc_dual):
// each kernel is the elementwise tail of one step in ONE pass over the rows, the same IEEE
// operations in the same order as the torch expressions it replaces (contraction off), so the
// iterates are bit-identical; ~50 small launches per iteration become 5.  Device scalars are read
// on the device (no host round trip).  Mh / My may be strided columns of a [l, k] solve result.
__global__ __launch_bounds__(256) void ipm_dirs_kernel(const double* __restrict__ Mh, int smh, const double* __restrict__ My,
                                                       int smy, const double* __restrict__ dbp,
                                                       const double* __restrict__ rnu, const double* __restrict__ rmu,
                                                       const double* __restrict__ nu, const double* __restrict__ mu,
                                                       const double* __restrict__ a, const double* __restrict__ s,
                                                       long long n, double* __restrict__ da, double* __restrict__ dnu,
                                                       double* __restrict__ dmu) {
#pragma clang fp contract(off)
  const double db = *dbp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double d = Mh[i * smh] - db * My[i * smy];
    da[i] = d;
    dnu[i] = (-rnu[i] - nu[i] * d) / a[i];
    dmu[i] = (-rmu[i] + mu[i] * d) / s[i];
  }
}

// iteration prologue: s = c − α and the dual residual rd = ((y·(Φw) − 1) + b·y − ν) + μ
// (P: the column Φw, stride sp; b a device scalar)
__global__ __launch_bounds__(256) void ipm_resid_kernel(const double* __restrict__ c, const double* __restrict__ a,
                                                        const double* __restrict__ y, const double* __restrict__ P, int sp,
                                                        const double* __restrict__ bp, const double* __restrict__ nu,
                                                        const double* __restrict__ mu, long long n, double* __restrict__ s,
                                                        double* __restrict__ rd) {
#pragma clang fp contract(off)
  const double b = *bp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    s[i] = c[i] - a[i];
    const double g = y[i] * P[i * sp] - 1.0;
    rd[i] = ((g + b * y[i]) - nu[i]) + mu[i];
  }
}

// predictor set-up: D⁻¹ = 1 / (ν/α + μ/s) (and its two-column copy), rν = α·ν, rμ = s·μ and the
// right-hand sides [h, y] with h = ((−rd) − rν/α) + rμ/s
__global__ __launch_bounds__(256) void ipm_pred_kernel(const double* __restrict__ a, const double* __restrict__ s,
                                                       const double* __restrict__ nu, const double* __restrict__ mu,
                                                       const double* __restrict__ rd, const double* __restrict__ y,
                                                       long long n, double* __restrict__ Dinv, double* __restrict__ Dinv2,
                                                       double* __restrict__ rnu, double* __restrict__ rmu,
                                                       double* __restrict__ H2) {
#pragma clang fp contract(off)
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double D = nu[i] / a[i] + mu[i] / s[i];
    const double di = 1.0 / D;
    Dinv[i] = di;
    Dinv2[2 * i] = di;
    Dinv2[2 * i + 1] = di;
    const double rn = a[i] * nu[i], rm = s[i] * mu[i];
    rnu[i] = rn;
    rmu[i] = rm;
    H2[2 * i] = (-rd[i] - rn / a[i]) + rm / s[i];
    H2[2 * i + 1] = y[i];
  }
}

// corrector right-hand side: rν = (α·ν + Δα·Δν) − τ, rμ = (s·μ − Δα·Δμ) − τ, h = ((−rd) − rν/α) + rμ/s
__global__ __launch_bounds__(256) void ipm_corr_kernel(const double* __restrict__ a, const double* __restrict__ s,
                                                       const double* __restrict__ nu, const double* __restrict__ mu,
                                                       const double* __restrict__ da, const double* __restrict__ dnu,
                                                       const double* __restrict__ dmu, const double* __restrict__ rd,
                                                       const double* __restrict__ taup, long long n,
                                                       double* __restrict__ rnu, double* __restrict__ rmu,
                                                       double* __restrict__ h) {
#pragma clang fp contract(off)
  const double tau = *taup;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double rn = (a[i] * nu[i] + da[i] * dnu[i]) - tau;
    const double rm = (s[i] * mu[i] - da[i] * dmu[i]) - tau;
    rnu[i] = rn;
    rmu[i] = rm;
    h[i] = (-rd[i] - rn / a[i]) + rm / s[i];
  }
}

// the Woodbury solve's row passes around Φᵀ / Φ: du = D⁻¹ ∘ U, V = y ∘ du (k columns, row-major),
// and afterwards out = du − D⁻¹ ∘ (y ∘ P)
__global__ __launch_bounds__(256) void ipm_minv_pre_kernel(const double* __restrict__ Dinv, const double* __restrict__ y,
                                                           const double* __restrict__ U, int k, long long n,
                                                           double* __restrict__ du, double* __restrict__ V) {
#pragma clang fp contract(off)
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n * k; e += (long long)gridDim.x * 256) {
    const long long i = e / k;
    const double d = Dinv[i] * U[e];
    du[e] = d;
    V[e] = y[i] * d;
  }
}

__global__ __launch_bounds__(256) void ipm_minv_post_kernel(const double* __restrict__ Dinv, const double* __restrict__ y,
                                                            const double* __restrict__ du, const double* __restrict__ P,
                                                            int k, long long n, double* __restrict__ out) {
#pragma clang fp contract(off)
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n * k; e += (long long)gridDim.x * 256) {
    const long long i = e / k;
    out[e] = du[e] - Dinv[i] * (y[i] * P[e]);
  }
}

// the step: α + t·Δα, ν + t·Δν, μ + t·Δμ (t a device scalar)
__global__ __launch_bounds__(256) void ipm_update_kernel(const double* __restrict__ a, const double* __restrict__ nu,
                                                         const double* __restrict__ mu, const double* __restrict__ da,
                                                         const double* __restrict__ dnu, const double* __restrict__ dmu,
                                                         const double* __restrict__ tp, long long n,
                                                         double* __restrict__ a2, double* __restrict__ nu2,
                                                         double* __restrict__ mu2) {
#pragma clang fp contract(off)
  const double t = *tp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    a2[i] = a[i] + t * da[i];
    nu2[i] = nu[i] + t * dnu[i];
    mu2[i] = mu[i] + t * dmu[i];
  }
}

// Gondzio corrector target: the trial point's complementarity products pushed into [0.1τ, 10τ]
__global__ __launch_bounds__(256) void ipm_gondzio_rhs_kernel(const double* __restrict__ a, const double* __restrict__ s,
                                                              const double* __restrict__ nu, const double* __restrict__ mu,
                                                              const double* __restrict__ da, const double* __restrict__ dnu,
                                                              const double* __restrict__ dmu, const double* __restrict__ alphap,
                                                              const double* __restrict__ taup, long long n,
                                                              double* __restrict__ ta, double* __restrict__ ts,
                                                              double* __restrict__ rhs) {
#pragma clang fp contract(off)
  const double at = fmin(1.5 * *alphap + 0.1, 1.0);
  const double tau = *taup;
  const double lo = 0.1 * tau, hi = 10.0 * tau;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double va = (a[i] + at * da[i]) * (nu[i] + at * dnu[i]);
    const double vs = (s[i] - at * da[i]) * (mu[i] + at * dmu[i]);
    const double tca = fmax(fmin(fmax(va, lo), hi) - va, -hi);
    const double tcs = fmax(fmin(fmax(vs, lo), hi) - vs, -hi);
    ta[i] = tca;
    ts[i] = tcs;
    rhs[i] = tca / a[i] - tcs / s[i];
  }
}

// Gondzio corrector applied to the direction: the corrected (Δα, Δν, Δμ)
__global__ __launch_bounds__(256) void ipm_gondzio_apply_kernel(const double* __restrict__ Mh, int smh,
                                                                const double* __restrict__ My, int smy,
                                                                const double* __restrict__ dbcp,
                                                                const double* __restrict__ da, const double* __restrict__ dnu,
                                                                const double* __restrict__ dmu, const double* __restrict__ ta,
                                                                const double* __restrict__ ts, const double* __restrict__ nu,
                                                                const double* __restrict__ mu, const double* __restrict__ a,
                                                                const double* __restrict__ s, long long n,
                                                                double* __restrict__ nda, double* __restrict__ ndnu,
                                                                double* __restrict__ ndmu) {
#pragma clang fp contract(off)
  const double dbc = *dbcp;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double dac = Mh[i * smh] - dbc * My[i * smy];
    nda[i] = da[i] + dac;
    ndnu[i] = dnu[i] + (ta[i] - nu[i] * dac) / a[i];
    ndmu[i] = dmu[i] + (ts[i] + mu[i] * dac) / s[i];
  }
}

// keep the corrected direction where *ok (a device bool as 0/1 byte), in place
__global__ __launch_bounds__(256) void ipm_select3_kernel(const bool* __restrict__ okp, const double* __restrict__ x0,
                                                          const double* __restrict__ x1, const double* __restrict__ x2,
                                                          long long n, double* __restrict__ y0, double* __restrict__ y1,
                                                          double* __restrict__ y2) {
  if (!*okp) return;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    y0[i] = x0[i];
    y1[i] = x1[i];
    y2[i] = x2[i];
  }
}

static unsigned ipm_blocks(long long n) {
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  long long b = (n + 255) / 256;
  if (b > 8LL * ncu) b = 8LL * ncu;
  return (unsigned)(b < 1 ? 1 : b);
}

static int ipm_grid(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

void ipm_resid(uintptr_t c, uintptr_t a, uintptr_t y, uintptr_t P, int sp, uintptr_t b, uintptr_t nu, uintptr_t mu,
               long long n, uintptr_t s, uintptr_t rd, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_resid_kernel, dim3(ipm_grid(n)), dim3(256), 0, as_stream(stream), (const double*)c,
                     (const double*)a, (const double*)y, (const double*)P, sp, (const double*)b, (const double*)nu,
                     (const double*)mu, n, (double*)s, (double*)rd);
  launch_check();
}

void ipm_pred(uintptr_t a, uintptr_t s, uintptr_t nu, uintptr_t mu, uintptr_t rd, uintptr_t y, long long n,
              uintptr_t Dinv, uintptr_t Dinv2, uintptr_t rnu, uintptr_t rmu, uintptr_t H2, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_pred_kernel, dim3(ipm_grid(n)), dim3(256), 0, as_stream(stream), (const double*)a,
                     (const double*)s, (const double*)nu, (const double*)mu, (const double*)rd, (const double*)y, n,
                     (double*)Dinv, (double*)Dinv2, (double*)rnu, (double*)rmu, (double*)H2);
  launch_check();
}

void ipm_corr(uintptr_t a, uintptr_t s, uintptr_t nu, uintptr_t mu, uintptr_t da, uintptr_t dnu, uintptr_t dmu,
              uintptr_t rd, uintptr_t tau, long long n, uintptr_t rnu, uintptr_t rmu, uintptr_t h, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_corr_kernel, dim3(ipm_grid(n)), dim3(256), 0, as_stream(stream), (const double*)a,
                     (const double*)s, (const double*)nu, (const double*)mu, (const double*)da, (const double*)dnu,
                     (const double*)dmu, (const double*)rd, (const double*)tau, n, (double*)rnu, (double*)rmu,
                     (double*)h);
  launch_check();
}

void ipm_minv_pre(uintptr_t Dinv, uintptr_t y, uintptr_t U, int k, long long n, uintptr_t du, uintptr_t V,
                  uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_minv_pre_kernel, dim3(ipm_grid(n * k)), dim3(256), 0, as_stream(stream), (const double*)Dinv,
                     (const double*)y, (const double*)U, k, n, (double*)du, (double*)V);
  launch_check();
}

void ipm_minv_post(uintptr_t Dinv, uintptr_t y, uintptr_t du, uintptr_t P, int k, long long n, uintptr_t out,
                   uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_minv_post_kernel, dim3(ipm_grid(n * k)), dim3(256), 0, as_stream(stream), (const double*)Dinv,
                     (const double*)y, (const double*)du, (const double*)P, k, n, (double*)out);
  launch_check();
}

void ipm_update(uintptr_t a, uintptr_t nu, uintptr_t mu, uintptr_t da, uintptr_t dnu, uintptr_t dmu, uintptr_t t,
                long long n, uintptr_t a2, uintptr_t nu2, uintptr_t mu2, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_update_kernel, dim3(ipm_grid(n)), dim3(256), 0, as_stream(stream), (const double*)a,
                     (const double*)nu, (const double*)mu, (const double*)da, (const double*)dnu, (const double*)dmu,
                     (const double*)t, n, (double*)a2, (double*)nu2, (double*)mu2);
  launch_check();
}

void ipm_dirs(uintptr_t Mh, int smh, uintptr_t My, int smy, uintptr_t db, uintptr_t rnu, uintptr_t rmu, uintptr_t nu,
              uintptr_t mu, uintptr_t a, uintptr_t s, long long n, uintptr_t da, uintptr_t dnu, uintptr_t dmu,
              uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_dirs_kernel, dim3(ipm_blocks(n)), dim3(256), 0, as_stream(stream), (const double*)Mh, smh,
                     (const double*)My, smy, (const double*)db, (const double*)rnu, (const double*)rmu,
                     (const double*)nu, (const double*)mu, (const double*)a, (const double*)s, n, (double*)da,
                     (double*)dnu, (double*)dmu);
  launch_check();
}

void ipm_gondzio_rhs(uintptr_t a, uintptr_t s, uintptr_t nu, uintptr_t mu, uintptr_t da, uintptr_t dnu, uintptr_t dmu,
                     uintptr_t alpha, uintptr_t tau, long long n, uintptr_t ta, uintptr_t ts, uintptr_t rhs,
                     uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_gondzio_rhs_kernel, dim3(ipm_blocks(n)), dim3(256), 0, as_stream(stream), (const double*)a,
                     (const double*)s, (const double*)nu, (const double*)mu, (const double*)da, (const double*)dnu,
                     (const double*)dmu, (const double*)alpha, (const double*)tau, n, (double*)ta, (double*)ts,
                     (double*)rhs);
  launch_check();
}

void ipm_gondzio_apply(uintptr_t Mh, int smh, uintptr_t My, int smy, uintptr_t dbc, uintptr_t da, uintptr_t dnu,
                       uintptr_t dmu, uintptr_t ta, uintptr_t ts, uintptr_t nu, uintptr_t mu, uintptr_t a, uintptr_t s,
                       long long n, uintptr_t nda, uintptr_t ndnu, uintptr_t ndmu, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_gondzio_apply_kernel, dim3(ipm_blocks(n)), dim3(256), 0, as_stream(stream), (const double*)Mh,
                     smh, (const double*)My, smy, (const double*)dbc, (const double*)da, (const double*)dnu,
                     (const double*)dmu, (const double*)ta, (const double*)ts, (const double*)nu, (const double*)mu,
                     (const double*)a, (const double*)s, n, (double*)nda, (double*)ndnu, (double*)ndmu);
  launch_check();
}

void ipm_select3(uintptr_t ok, uintptr_t x0, uintptr_t x1, uintptr_t x2, long long n, uintptr_t y0, uintptr_t y1,
                 uintptr_t y2, uintptr_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(ipm_select3_kernel, dim3(ipm_blocks(n)), dim3(256), 0, as_stream(stream), (const bool*)ok,
                     (const double*)x0, (const double*)x1, (const double*)x2, n, (double*)y0, (double*)y1, (double*)y2);
  launch_check();
}

// ---- diag(d)·Φ for the weighted Gram, from the exact f32 copy of Φ (half the bytes of the f64 read;
// the product is the same f64 multiply of the same values as torch's broadcast P * d).
__global__ __launch_bounds__(256) void scale_rows_f32_kernel(const float* __restrict__ P, const double* __restrict__ d,
                                                             long long n, int r, double* __restrict__ out) {
  const int r4 = r >> 2;   // r % 4 == 0 (checked)
  const long long tot = n * r4;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < tot; e += (long long)gridDim.x * 256) {
    const long long i = e / r4;
    const int c = (int)(e - i * r4) * 4;
    const float4 p = *reinterpret_cast<const float4*>(P + i * r + c);
    const double di = d[i];
    double2* o = reinterpret_cast<double2*>(out + i * r + c);
    o[0] = double2{(double)p.x * di, (double)p.y * di};
    o[1] = double2{(double)p.z * di, (double)p.w * di};
  }
}

void scale_rows_f32(uintptr_t P, uintptr_t d, long long n, int r, uintptr_t out, uintptr_t stream) {
  HFENS_REQUIRE(r % 4 == 0 && r >= 4, "scale_rows_f32: r must be a positive multiple of 4");
  if (n <= 0) return;
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  long long blocks = (n * (r / 4) + 255) / 256;
  if (blocks > 16LL * ncu) blocks = 16LL * ncu;
  hipLaunchKernelGGL(scale_rows_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), (const float*)P,
                     (const double*)d, n, r, (double*)out);
  launch_check();
}

}  // namespace hfens
