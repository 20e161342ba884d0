// Small dense SPD factor / solve for the interior-point SVC (models/svc_lowrank.py): the r × r
// Woodbury system S = I + Φᵀ D⁻¹ Φ (r ≤ 1024 landmarks) is factored every IPM iteration.
//
// Library potrf/potrs stalled the solve: the profile of one 1M-row solve (profiles/
// r2_ipm_native.md) shows 5–14 ms GPU-idle gaps before rocSOLVER/rocBLAS kernels (their workspace
// handling) and a blocking read of potrf's `info` every iteration.  Here:
//
//  chol_spd  : ONE workgroup (1024 threads), r ≤ 1024.  Symmetric equilibration sc = diag(S)^-½,
//              then a right-looking blocked Cholesky of sc·S·sc (+ jit·I) into L (row-major, lower
//              triangle): NB-column diagonal blocks (NB = 32, 16 above r = 512) factored in LDS by
//              all threads, the panel below solved one row per thread into a transposed LDS copy,
//              the trailing lower triangle updated from it on v_mfma_f64_16x16x4_f64 (16×16 blocks
//              over the 16 waves; f64 MFMA maps A[l&15][l>>4], B[l>>4][l&15], C row (l>>4)+4·reg).  A non-positive or non-finite pivot
//              restarts the factorisation from S with jit = 1e-14, 1e-12, … 1 — on the device,
//              so the host never reads `info`.  out_info[0] = retries used (−1 = still failed).
//  chol_solve: x = sc ∘ (L Lᵀ)⁻¹ (sc ∘ b) for k ≤ 4 right-hand sides, one workgroup: blocked
//              forward / backward substitution, 64-row diagonal blocks solved by wave 0 (readlane
//              chain), the off-diagonal updates by all threads.
#include <type_traits>

#include "common.h"

namespace hfens {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kChThreads = 1024;
constexpr int kChWaves = kChThreads / 64;
constexpr int kChNB = 64;   // solve block (wave 0 substitution chains)
constexpr int kChMaxK = 4;
constexpr int kChTU = 4;    // trailing-update blocks per load round (chol_spd)

__device__ __forceinline__ double ch_readlane(double v, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, lane);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

size_t chol_spd_lds(int r, int NB) { return ((size_t)NB * (NB + 1) + (size_t)NB * r + NB) * sizeof(double); }

// LDS: Dg [NB][NB+1] the diagonal block; PT [NB][r] the panel, TRANSPOSED (lanes of a wave read
// consecutive rows: conflict-free), dgl [NB] the block's pivots.
template <int NB>
__global__ __launch_bounds__(kChThreads) void chol_spd_kernel(const double* __restrict__ S, int r,
                                                              double* __restrict__ L, double* __restrict__ sc,
                                                              int* __restrict__ out_info,
                                                              const int* __restrict__ skip_if_ok = nullptr) {
  // (the multi-workgroup factorisation ran first and succeeded: nothing to do)
  if (skip_if_ok != nullptr && skip_if_ok[0] == 0) return;
  extern __shared__ __attribute__((aligned(16))) double chsm[];
  double* Dg = chsm;
  double* PT = Dg + NB * (NB + 1);
  double* dgl = PT + (size_t)NB * r;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < r; i += kChThreads) {
    const double d = S[(size_t)i * r + i];
    sc[i] = d > 0.0 ? 1.0 / sqrt(d) : 1.0;
  }
  __syncthreads();
  double jit = 0.0;
  int tries = 0;
  for (;;) {
    // L ← lower triangle of sc·S·sc + jit·I (upper triangle zeroed: potrf's output convention)
    for (size_t e = tid; e < (size_t)r * r; e += kChThreads) {
      const int i = (int)(e / r), j = (int)(e % r);
      L[e] = j <= i ? S[e] * sc[i] * sc[j] + (i == j ? jit : 0.0) : 0.0;
    }
    __syncthreads();
    bool bad = false;
    for (int k0 = 0; k0 < r && !bad; k0 += NB) {
      const int nb = min(NB, r - k0), m0 = k0 + nb, m = r - m0;
      for (int e = tid; e < nb * nb; e += kChThreads) {
        const int a = e / nb, b = e % nb;
        Dg[a * (NB + 1) + b] = b <= a ? L[(size_t)(k0 + a) * r + k0 + b] : 0.0;
      }
      __syncthreads();
      // ---- diagonal block, right-looking, all threads (the pivot test is uniform)
      for (int j = 0; j < nb; ++j) {
        const double pj = Dg[j * (NB + 1) + j];
        if (!(pj > 0.0) || !isfinite(pj)) { bad = true; break; }
        const double dj = sqrt(pj);
        for (int a = j + 1 + tid; a < nb; a += kChThreads) Dg[a * (NB + 1) + j] /= dj;
        if (tid == 0) dgl[j] = dj;
        __syncthreads();
        for (int a = j + 1 + wave; a < nb; a += kChWaves)
          for (int b = j + 1 + lane; b <= a; b += 64)
            Dg[a * (NB + 1) + b] -= Dg[a * (NB + 1) + j] * Dg[b * (NB + 1) + j];
        __syncthreads();
      }
      if (bad) break;
      for (int j = tid; j < nb; j += kChThreads) Dg[j * (NB + 1) + j] = dgl[j];
      __syncthreads();
      for (int e = tid; e < nb * nb; e += kChThreads) {
        const int a = e / nb, b = e % nb;
        if (b <= a) L[(size_t)(k0 + a) * r + k0 + b] = Dg[a * (NB + 1) + b];
      }
      // ---- panel: row m0+t ← A[m0+t][k0:k0+nb] · L_blockᵀ⁻¹ (one row per thread)
      for (int t = tid; t < m; t += kChThreads) {
        double x[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) x[b] = b < nb ? L[(size_t)(m0 + t) * r + k0 + b] : 0.0;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          if (b < nb) {
            double v = x[b];
#pragma unroll
            for (int p = 0; p < b; ++p) v -= x[p] * Dg[b * (NB + 1) + p];
            x[b] = v / Dg[b * (NB + 1) + b];
          }
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
          if (b < nb) {
            L[(size_t)(m0 + t) * r + k0 + b] = x[b];
            PT[(size_t)b * r + t] = x[b];
          }
      }
      __syncthreads();
      // ---- trailing lower triangle: A[m0+i][m0+j] −= Σ_b P[i][b]·P[j][b] (j ≤ i) on the f64 matrix
      //      cores: 16×16 output blocks (bj ≤ bi) round-robin over the 16 waves, NB/4 MFMAs each with
      //      both operands read from the transposed panel (rows past m are zero-padded)
      const int m16 = (m + 15) & ~15;
      for (int e = m + tid; e < m16; e += kChThreads)
        for (int b = 0; b < NB; ++b) PT[(size_t)b * r + e] = 0.0;
      __syncthreads();
      const int nbk = m16 / 16;
      const int nblocks = nbk * (nbk + 1) / 2;
      // kChTU blocks per round: their L tiles are loaded before any of them is written back (a
      // store into L between a block's load and the next one's would serialise one L2 round trip
      // per block), then the MFMAs, then the stores — the same L − acc per element as before
      for (int blk0 = wave; blk0 < nblocks; blk0 += kChWaves * kChTU) {
        double old[kChTU][4];
        int bis[kChTU], bjs[kChTU];
#pragma unroll
        for (int c = 0; c < kChTU; ++c) {
          const int blk = blk0 + c * kChWaves;
          int bi = 0, rem = blk;
          while (rem > bi) { rem -= bi + 1; ++bi; }
          bis[c] = blk < nblocks ? bi : -1;
          bjs[c] = rem;                                    // 0 ≤ bj ≤ bi
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int i = 16 * bi + (lane >> 4) + 4 * reg, j = 16 * rem + (lane & 15);
            old[c][reg] = (blk < nblocks && i < m && j <= i) ? L[(size_t)(m0 + i) * r + m0 + j] : 0.0;
          }
        }
#pragma unroll
        for (int c = 0; c < kChTU; ++c) {
          const int bi = bis[c], bj = bjs[c];
          if (bi < 0) continue;
          f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ks = 0; ks < NB / 4; ++ks) {
            const int kb = 4 * ks + (lane >> 4);
            const double a = PT[(size_t)kb * r + 16 * bi + (lane & 15)];
            const double b = PT[(size_t)kb * r + 16 * bj + (lane & 15)];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
          }
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int i = 16 * bi + (lane >> 4) + 4 * reg, j = 16 * bj + (lane & 15);
            if (i < m && j <= i) L[(size_t)(m0 + i) * r + m0 + j] = old[c][reg] - acc[reg];
          }
        }
      }
      __syncthreads();
    }
    if (!bad) break;
    ++tries;
    // 1e-14 … 1e-6 are numerical repairs; beyond that the step is a damped (regularised) Newton
    // step, which the interior-point iteration tolerates — only a non-finite S ends the ladder
    jit = jit == 0.0 ? 1e-14 : jit * 100.0;
    if (jit > 1.0) {
      if (tid == 0) out_info[0] = -1;
      return;
    }
    __syncthreads();
  }
  if (tid == 0) out_info[0] = tries;
}

// ---- chol_spd_mw: the same blocked factorisation spread over the GPU -------
// chol_spd_kernel runs every phase inside ONE workgroup (≈ 1.2 ms at r = 512, the largest single item
// of the interior point after the Gram and the skinny passes).  Here each NB-column step is three
// launches — the NB × NB diagonal block (one workgroup, the same loops), the panel rows (one thread
// per row over ⌈m/256⌉ workgroups, the transposed panel PT in global memory instead of LDS), the
// trailing lower triangle (one wave per 16 × 16 block on v_mfma_f64_16x16x4_f64 over ⌈blocks/8⌉
// workgroups) — with every element computed by the same operations in the same order as the
// one-workgroup kernel, so L is bit-identical to it.  Only the unjittered attempt runs here: a
// failed pivot sets work[0] and the remaining launches exit at once; chol_spd_kernel then runs with
// skip_if_ok = work and does its full jitter ladder from S.
template <int NB>
__global__ __launch_bounds__(256) void chol_mw_init_kernel(const double* __restrict__ S, int r,
                                                           double* __restrict__ L, double* __restrict__ sc,
                                                           int* __restrict__ work) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e == 0) work[0] = 0;
  if (e >= (size_t)r * r) return;
  const int i = (int)(e / r), j = (int)(e % r);
  const double di = S[(size_t)i * r + i], dj = S[(size_t)j * r + j];
  const double si = di > 0.0 ? 1.0 / sqrt(di) : 1.0, sj = dj > 0.0 ? 1.0 / sqrt(dj) : 1.0;
  if (j == 0) sc[i] = si;
  L[e] = j <= i ? S[e] * si * sj + (i == j ? 0.0 : 0.0) : 0.0;
}

template <int NB>
__global__ __launch_bounds__(kChThreads) void chol_mw_diag_kernel(double* __restrict__ L, int r, int k0,
                                                                  int* __restrict__ work) {
  if (work[0] != 0) return;
  __shared__ double Dg[NB * (NB + 1)];
  __shared__ double dgl[NB];
  __shared__ int s_bad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = min(NB, r - k0);
  if (tid == 0) s_bad = 0;
  for (int e = tid; e < nb * nb; e += kChThreads) {
    const int a = e / nb, b = e % nb;
    Dg[a * (NB + 1) + b] = b <= a ? L[(size_t)(k0 + a) * r + k0 + b] : 0.0;
  }
  __syncthreads();
  for (int j = 0; j < nb; ++j) {
    const double pj = Dg[j * (NB + 1) + j];
    if (!(pj > 0.0) || !isfinite(pj)) {
      if (tid == 0) work[0] = 1;
      return;
    }
    const double dj = sqrt(pj);
    for (int a = j + 1 + tid; a < nb; a += kChThreads) Dg[a * (NB + 1) + j] /= dj;
    if (tid == 0) dgl[j] = dj;
    __syncthreads();
    for (int a = j + 1 + wave; a < nb; a += kChWaves)
      for (int b = j + 1 + lane; b <= a; b += 64)
        Dg[a * (NB + 1) + b] -= Dg[a * (NB + 1) + j] * Dg[b * (NB + 1) + j];
    __syncthreads();
  }
  for (int j = tid; j < nb; j += kChThreads) Dg[j * (NB + 1) + j] = dgl[j];
  __syncthreads();
  for (int e = tid; e < nb * nb; e += kChThreads) {
    const int a = e / nb, b = e % nb;
    if (b <= a) L[(size_t)(k0 + a) * r + k0 + b] = Dg[a * (NB + 1) + b];
  }
}

template <int NB>
__global__ __launch_bounds__(256) void chol_mw_panel_kernel(double* __restrict__ L, int r, int k0,
                                                            double* __restrict__ PT, const int* __restrict__ work) {
  if (work[0] != 0) return;
  __shared__ double Dg[NB * (NB + 1)];
  const int nb = min(NB, r - k0), m0 = k0 + nb, m = r - m0;
  for (int e = threadIdx.x; e < nb * nb; e += 256) {
    const int a = e / nb, b = e % nb;
    Dg[a * (NB + 1) + b] = b <= a ? L[(size_t)(k0 + a) * r + k0 + b] : 0.0;
  }
  __syncthreads();
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int m16 = (m + 15) & ~15;
  if (t >= m && t < m16) {
#pragma unroll
    for (int b = 0; b < NB; ++b) PT[(size_t)b * r + t] = 0.0;
  }
  if (t >= m) return;
  double x[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) x[b] = b < nb ? L[(size_t)(m0 + t) * r + k0 + b] : 0.0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b < nb) {
      double v = x[b];
#pragma unroll
      for (int p = 0; p < b; ++p) v -= x[p] * Dg[b * (NB + 1) + p];
      x[b] = v / Dg[b * (NB + 1) + b];
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b)
    if (b < nb) {
      L[(size_t)(m0 + t) * r + k0 + b] = x[b];
      PT[(size_t)b * r + t] = x[b];
    }
}

template <int NB>
__global__ __launch_bounds__(256) void chol_mw_trail_kernel(double* __restrict__ L, int r, int k0,
                                                            const double* __restrict__ PT,
                                                            const int* __restrict__ work) {
  if (work[0] != 0) return;
  const int nb = min(NB, r - k0), m0 = k0 + nb, m = r - m0;
  const int m16 = (m + 15) & ~15;
  const int nbk = m16 / 16;
  const int nblocks = nbk * (nbk + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per 16 × 16 block
  if (blk >= nblocks) return;
  int bi = 0, rem = blk;
  while (rem > bi) { rem -= bi + 1; ++bi; }
  const int bj = rem;
  double old[4];
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int i = 16 * bi + (lane >> 4) + 4 * reg, j = 16 * bj + (lane & 15);
    old[reg] = (i < m && j <= i) ? L[(size_t)(m0 + i) * r + m0 + j] : 0.0;
  }
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < NB / 4; ++ks) {
    const int kb = 4 * ks + (lane >> 4);
    const double a = PT[(size_t)kb * r + 16 * bi + (lane & 15)];
    const double b = PT[(size_t)kb * r + 16 * bj + (lane & 15)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int i = 16 * bi + (lane >> 4) + 4 * reg, j = 16 * bj + (lane & 15);
    if (i < m && j <= i) L[(size_t)(m0 + i) * r + m0 + j] = old[reg] - acc[reg];
  }
}

// x ← sc ∘ (L Lᵀ)⁻¹ (sc ∘ B): B [r][k] row-major (k ≤ 4), overwritten with the solution.  Per
// 64-row block: wave 0 runs the substitution chain on the block's diagonal block of L (staged in
// LDS; the pivots inverted in parallel first, the chain then multiplies) while waves 1… stage the
// NEXT diagonal block (double-buffered), so the staging round trip overlaps the chain; then every
// thread loads its row's 64-column slice of L in one round (512 threads: the 64 values fit in
// registers; the 1024-thread version needed four rounds of 16) and updates its right-hand sides.
// The arithmetic and its order are unchanged.  K = right-hand sides (compile time: the per-lane
// vectors stay in registers).
constexpr int kCsThreads = 512;

template <int K>
__global__ __launch_bounds__(kCsThreads) void chol_solve_kernel(const double* __restrict__ L, const double* __restrict__ sc,
                                                                int r, double* __restrict__ B) {
  __shared__ double Db[2][kChNB][kChNB + 1];
  __shared__ double Xb[kChNB][kChMaxK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nblk = (r + kChNB - 1) / kChNB;
  auto stage = [&](int buf, int k0, int t0, int nt) {   // Db[buf] ← diagonal block at k0
    const int nb = min(kChNB, r - k0);
    for (int e = t0; e < nb * nb; e += nt) {
      const int a = e / nb, c = e % nb;
      Db[buf][a][c] = c <= a ? L[(size_t)(k0 + a) * r + k0 + c] : 0.0;
    }
  };
  for (int e = tid; e < r * K; e += kCsThreads) B[e] *= sc[e / K];
  stage(0, 0, tid, kCsThreads);
  __syncthreads();
  // forward: L y = b
  for (int kb = 0; kb < nblk; ++kb) {
    const int k0 = kb * kChNB, nb = min(kChNB, r - k0), cur = kb & 1;
    if (wave != 0 && kb + 1 < nblk) stage(cur ^ 1, k0 + kChNB, tid - 64, kCsThreads - 64);
    if (wave == 0) {
      double y[K];
#pragma unroll
      for (int q = 0; q < K; ++q) y[q] = lane < nb ? B[(size_t)(k0 + lane) * K + q] : 0.0;
      const double dinv = lane < nb ? 1.0 / Db[cur][lane][lane] : 0.0;
      for (int j = 0; j < nb; ++j) {
        const double dj = ch_readlane(dinv, j);
        const double lij = (lane > j && lane < nb) ? Db[cur][lane][j] : 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) {
          if (lane == j) y[q] *= dj;
          const double yj = ch_readlane(y[q], j);
          if (lane > j) y[q] -= lij * yj;
        }
      }
      if (lane < nb)
#pragma unroll
        for (int q = 0; q < K; ++q) {
          B[(size_t)(k0 + lane) * K + q] = y[q];
          Xb[lane][q] = y[q];
        }
    }
    __syncthreads();
    for (int i = k0 + nb + tid; i < r; i += kCsThreads) {
      double l[kChNB];   // the row's whole slice in one round of loads
      const double* li = L + (size_t)i * r + k0;
#pragma unroll
      for (int u = 0; u < kChNB; ++u) l[u] = u < nb ? li[u] : 0.0;
      double acc[K];
#pragma unroll
      for (int q = 0; q < K; ++q) acc[q] = 0.0;
      // 16 columns at a time: the scheduler would otherwise hoist all 64·K LDS reads of Xb next to
      // the 64 loaded L values (spills)
#pragma unroll
      for (int b0 = 0; b0 < kChNB; b0 += 16) {
#pragma unroll
        for (int u = b0; u < b0 + 16; ++u)
#pragma unroll
          for (int q = 0; q < K; ++q) acc[q] = fma(l[u], u < nb ? Xb[u][q] : 0.0, acc[q]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int q = 0; q < K; ++q) B[(size_t)i * K + q] -= acc[q];
    }
    __syncthreads();
  }
  // backward: Lᵀ x = y (blocks from the bottom); the last forward block is staged in Db[(nblk-1)&1]
  for (int bi = nblk - 1; bi >= 0; --bi) {
    const int k0 = bi * kChNB, nb = min(kChNB, r - k0), cur = (nblk - 1 - bi + (nblk - 1)) & 1;
    const double* Lb = L + (size_t)k0 * r;
    if (wave != 0 && bi > 0) stage(cur ^ 1, k0 - kChNB, tid - 64, kCsThreads - 64);
    if (wave == 0) {
      double x[K];
#pragma unroll
      for (int q = 0; q < K; ++q) x[q] = lane < nb ? B[(size_t)(k0 + lane) * K + q] : 0.0;
      const double dinv = lane < nb ? 1.0 / Db[cur][lane][lane] : 0.0;
      for (int j = nb - 1; j >= 0; --j) {
        const double dj = ch_readlane(dinv, j);
        // Lᵀ[lane][j] = L[j][lane] for lane < j
        const double lji = lane < j ? Db[cur][j][lane] : 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) {
          if (lane == j) x[q] *= dj;
          const double xj = ch_readlane(x[q], j);
          if (lane < j) x[q] -= lji * xj;
        }
      }
      if (lane < nb)
#pragma unroll
        for (int q = 0; q < K; ++q) {
          B[(size_t)(k0 + lane) * K + q] = x[q];
          Xb[lane][q] = x[q];
        }
    }
    __syncthreads();
    // rows above the block: b_i −= Σ_{j in block} L[j][i]·x_j (lanes read consecutive i: coalesced)
    for (int i = tid; i < k0; i += kCsThreads) {
      double l[kChNB];
#pragma unroll
      for (int u = 0; u < kChNB; ++u) l[u] = u < nb ? Lb[(unsigned)(u * r + i)] : 0.0;
      double acc[K];
#pragma unroll
      for (int q = 0; q < K; ++q) acc[q] = 0.0;
      // 16 columns at a time: the scheduler would otherwise hoist all 64·K LDS reads of Xb next to
      // the 64 loaded L values (spills)
#pragma unroll
      for (int b0 = 0; b0 < kChNB; b0 += 16) {
#pragma unroll
        for (int u = b0; u < b0 + 16; ++u)
#pragma unroll
          for (int q = 0; q < K; ++q) acc[q] = fma(l[u], u < nb ? Xb[u][q] : 0.0, acc[q]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int q = 0; q < K; ++q) B[(size_t)i * K + q] -= acc[q];
    }
    __syncthreads();
  }
  for (int e = tid; e < r * K; e += kCsThreads) B[e] *= sc[e / K];
}

void chol_spd(uintptr_t S, int r, uintptr_t L, uintptr_t sc, uintptr_t info, uintptr_t stream) {
  HFENS_REQUIRE(r >= 1 && r <= 1024, "chol_spd: 1 <= r <= 1024");
  if (r <= 512) {
    hipLaunchKernelGGL(chol_spd_kernel<32>, dim3(1), dim3(kChThreads), chol_spd_lds(r, 32), as_stream(stream),
                       (const double*)S, r, (double*)L, (double*)sc, (int*)info);
  } else {
    hipLaunchKernelGGL(chol_spd_kernel<16>, dim3(1), dim3(kChThreads), chol_spd_lds(r, 16), as_stream(stream),
                       (const double*)S, r, (double*)L, (double*)sc, (int*)info);
  }
  launch_check();
}

__global__ void chol_mw_info_kernel(const int* __restrict__ work, int* __restrict__ info) {
  if (threadIdx.x == 0 && work[0] == 0) info[0] = 0;
}

// work: int32 [≥ 2] scratch (failure flag), PT: f64 [32 · r] scratch (the transposed panel)
void chol_spd_mw(uintptr_t S, int r, uintptr_t L, uintptr_t sc, uintptr_t info, uintptr_t work, uintptr_t PT,
                 uintptr_t stream) {
  HFENS_REQUIRE(r >= 1 && r <= 512, "chol_spd_mw: 1 <= r <= 512");
  constexpr int NB = 32;
  hipStream_t st = as_stream(stream);
  double* Lp = (double*)L;
  int* wk = (int*)work;
  const size_t rr = (size_t)r * r;
  hipLaunchKernelGGL(chol_mw_init_kernel<NB>, dim3((unsigned)((rr + 255) / 256)), dim3(256), 0, st, (const double*)S, r,
                     Lp, (double*)sc, wk);
  for (int k0 = 0; k0 < r; k0 += NB) {
    hipLaunchKernelGGL(chol_mw_diag_kernel<NB>, dim3(1), dim3(kChThreads), 0, st, Lp, r, k0, wk);
    const int m = r - min(NB, r - k0) - k0;
    if (m <= 0) break;
    hipLaunchKernelGGL(chol_mw_panel_kernel<NB>, dim3((m + 15 + 255) / 256), dim3(256), 0, st, Lp, r, k0,
                       (double*)PT, (const int*)wk);
    const int nbk = ((m + 15) & ~15) / 16;
    const int nblocks = nbk * (nbk + 1) / 2;
    hipLaunchKernelGGL(chol_mw_trail_kernel<NB>, dim3((nblocks + 3) / 4), dim3(256), 0, st, Lp, r, k0,
                       (const double*)PT, (const int*)wk);
  }
  launch_check();
  // the one-workgroup kernel with its jitter ladder, only if the plain attempt failed; else info = 0
  hipLaunchKernelGGL(chol_spd_kernel<32>, dim3(1), dim3(kChThreads), chol_spd_lds(r, 32), st, (const double*)S, r, Lp,
                     (double*)sc, (int*)info, (const int*)wk);
  hipLaunchKernelGGL(chol_mw_info_kernel, dim3(1), dim3(64), 0, st, (const int*)wk, (int*)info);
  launch_check();
}

void chol_solve(uintptr_t L, uintptr_t sc, int r, int k, uintptr_t B, uintptr_t stream) {
  HFENS_REQUIRE(r >= 1 && r <= 1024 && k >= 1 && k <= kChMaxK, "chol_solve: 1 <= r <= 1024, 1 <= k <= 4");
  auto go = [&](auto kk) {
    constexpr int K = decltype(kk)::value;
    hipLaunchKernelGGL(chol_solve_kernel<K>, dim3(1), dim3(kCsThreads), 0, as_stream(stream), (const double*)L,
                       (const double*)sc, r, (double*)B);
    launch_check();
  };
  if (k == 1) go(std::integral_constant<int, 1>{});
  else if (k == 2) go(std::integral_constant<int, 2>{});
  else if (k == 3) go(std::integral_constant<int, 3>{});
  else go(std::integral_constant<int, 4>{});
}

}  // namespace hfens
