// Working-set decomposition SMO for batches of C-SVC duals (the reference
// fits libsvm through sklearn SVC, train_ensemble_public.py:43-48).
//
// libsvm's SMO (svm.hip: smo_kernel) moves ONE pair per iteration and every iteration is a chain of
// two block reductions and two dependent Gram-row reads: on a 10k-point problem that is ~9 µs of
// latency per pair and ~7k pairs.  This solver keeps libsvm's dual, WSS3 pair rule inside the
// working set and libsvm's global stopping rule (m(α) − M(α) < eps, evaluated in f64 over ALL
// points), but restructures the work for the MI355X:
//
//   ws_select_solve (one 1024-thread workgroup per problem)
//     1. global gap m − M (f64), convergence test;
//     2. working set B = the q/2 most violating points of I_up and of I_low (two-level 11-bit
//        radix histograms in LDS + index-ordered tie compaction: deterministic);
//     3. K_BB (q×q) from the rows' features into LDS;
//     4. inner SMO on B by one wave — libsvm's WSS3 pair rule and clipping on the local gradient,
//        K rows from LDS, α/G in registers, wave-level reductions only (no barriers, no HBM);
//     5. publishes the changed coefficients y_i·Δα_i and their feature rows (MFMA layout).
//   ws_gupdate (grid = row tiles × problems)
//     G_t += y_t Σ_{i∈B} y_i Δα_i K(x_t, x_i) for every t: an RBF "GEMM + exp + GEMV" on the
//     f32-input MFMA (rows of the problem = B operand, changed working-set rows = A operand),
//     i.e. the kernel matrix is recomputed instead of stored — O(n·F) memory instead of O(n²).
//
// Results satisfy the same KKT tolerance as libsvm but follow a different pair sequence, so α
// agrees with libsvm to O(eps) rather than bit-for-bit (the exact-sequence solver stays in
// svm.hip for small problems and for parity tests).
#include "common.h"

namespace hfens {

struct WsProb {
  long long zoff;   // first row of this problem in zcat ([rows][F] f32)
  long long aoff;   // offset of α / G / ‖z‖² (per point)
  int l;            // points
  int npos;         // [0, npos) have y = +1
  double Cp, Cn;    // box constraints for y = +1 / −1
  float ngl2e;      // −γ·log2(e)
  int pad;
};

struct WsState {
  int done;
  int outer;        // outer (working-set) iterations
  long long inner;  // pair updates
  double gap;       // last global m − M
  int nc;           // changed working-set entries published for ws_gupdate (0 ⇒ nothing to do)
  int nws;
  long long cyc_select, cyc_build, cyc_inner;   // s_memtime phase totals (diagnostics)
  long long cyc_p0, cyc_p1, cyc_p2;             // selection sub-phases: gap pass, level-1, level-2
};

constexpr int kWsQ = 128;          // working-set size (q/2 from each side)
constexpr int kWsHalf = kWsQ / 2;
constexpr int kWsThreads = 1024;
constexpr int kWsWaves = kWsThreads / 64;
constexpr double kWsTau = 1e-12;
constexpr double kWsInf = 1.0e300;

// order-preserving f32 → u32 (larger float ⇒ larger key; every finite float maps to ≥ 0x00800000,
// so 0 can mean "not a member")
__device__ __forceinline__ unsigned ws_key(double v) {
  const unsigned u = __float_as_uint((float)v);
  return u ^ ((u >> 31) ? 0xFFFFFFFFu : 0x80000000u);
}

__device__ __forceinline__ double block_max_f64(double v, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_max_f64_exact(v);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double r = sh[0];
  for (int w = 1; w < kWsWaves; ++w) r = fmax(r, sh[w]);
  return r;
}

__device__ __forceinline__ double block_sum_f64(double v, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double r = 0.0;
  for (int w = 0; w < kWsWaves; ++w) r += sh[w];
  return r;
}

// exclusive scan over the 1024 threads in thread order; *total = block sum
__device__ __forceinline__ int block_excl_scan(int v, int* sh, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += u;
  }
  __syncthreads();
  if (lane == 63) sh[wave] = incl;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < kWsWaves; ++w) {
    const int s = sh[w];
    base += w < wave ? s : 0;
    tot += s;
  }
  *total = tot;
  return base + incl - v;
}

// Find, over a 2048-bin histogram scanned from the top bin down, the bin holding the k-th
// member: returns the bin and the count strictly above it (both lists packed 16|16 bits).
__device__ __forceinline__ void ws_find_bin(const int* hist, int k_up, int k_low, int* sh_scan,
                                            int* out /*[4]: bin_up, above_up, bin_low, above_low*/) {
  const int tid = threadIdx.x;
  const int hb = 2047 - 2 * tid, lb = 2046 - 2 * tid;
  const int hu = hist[hb], lu = hist[lb], hl = hist[2048 + hb], ll = hist[2048 + lb];
  int tot;
  const int ex = block_excl_scan((hu + lu) | ((hl + ll) << 16), sh_scan, &tot);
  const int eu = ex & 0xFFFF, el = ex >> 16;
  if (k_up > 0 && eu < k_up && eu + hu + lu >= k_up) {
    if (eu + hu >= k_up) { out[0] = hb; out[1] = eu; }
    else { out[0] = lb; out[1] = eu + hu; }
  }
  if (k_low > 0 && el < k_low && el + hl + ll >= k_low) {
    if (el + hl >= k_low) { out[2] = hb; out[3] = el; }
    else { out[2] = lb; out[3] = el + hl; }
  }
}

// libsvm's two-variable update (Solver::Solve, "update alpha[i] and alpha[j]").
__device__ __forceinline__ void ws_pair_update(double& ai, double& aj, int yi, int yj, double Ci, double Cj,
                                               double Gi, double Gj, double Kij) {
#pragma clang fp contract(off)
  const double Qij = (double)(yi * yj) * Kij;
  if (yi != yj) {
    double quad = 2.0 + 2.0 * Qij;
    if (quad <= 0) quad = kWsTau;
    const double delta = (-Gi - Gj) / quad;
    const double diff = ai - aj;
    ai += delta;
    aj += delta;
    if (diff > 0) {
      if (aj < 0) { aj = 0; ai = diff; }
    } else {
      if (ai < 0) { ai = 0; aj = -diff; }
    }
    if (diff > Ci - Cj) {
      if (ai > Ci) { ai = Ci; aj = Ci - diff; }
    } else {
      if (aj > Cj) { aj = Cj; ai = Cj + diff; }
    }
  } else {
    double quad = 2.0 - 2.0 * Qij;
    if (quad <= 0) quad = kWsTau;
    const double delta = (Gi - Gj) / quad;
    const double sum = ai + aj;
    ai -= delta;
    aj += delta;
    if (sum > Ci) {
      if (ai > Ci) { ai = Ci; aj = sum - Ci; }
    } else {
      if (aj < 0) { aj = 0; ai = sum; }
    }
    if (sum > Cj) {
      if (aj > Cj) { aj = Cj; ai = sum - Cj; }
    } else {
      if (ai < 0) { ai = 0; aj = sum; }
    }
  }
}

// Wave-level helpers for the selector: lanes below this one, and an exclusive prefix over the
// 16 waves of per-wave totals (one barrier).
__device__ __forceinline__ unsigned long long lanes_below() {
  return (1ull << (threadIdx.x & 63)) - 1ull;
}
__device__ __forceinline__ int wave_base(int wave_total, int* sh, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = wave_total;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWsWaves; ++w) {
    const int v = sh[w];
    base += w < wave ? v : 0;
    tot += v;
  }
  *total = tot;
  return base;
}

// LDS histogram add: when every active lane of the wave hits one bin (massive ties, e.g. all
// G = −1 at the start) one lane adds the popcount instead of 64 serialized atomics.
__device__ __forceinline__ void hist_add(int* hist, bool on, int bin) {
  const unsigned long long act = __ballot(on);
  if (!act) return;
  const int first = __builtin_amdgcn_readlane(bin, __builtin_ctzll(act));
  const unsigned long long same = __ballot(on && bin == first);
  if (same == act) {
    if ((threadIdx.x & 63) == __builtin_ctzll(act)) atomicAdd(&hist[first], __popcll(act));
  } else if (on) {
    atomicAdd(&hist[bin], 1);
  }
}

// Selection keys are produced where the gradient is produced: the kernel that writes G_t (init,
// then every gradient update) also writes t's order-preserving up/low keys and folds the exact
// f64 maxima (global gap) into the problem's atomics, so the per-problem selector only reads u32
// keys (one coalesced pass) instead of re-deriving them from α and G.
struct WsAux {
  unsigned* keys;              // [2][n]: I_up keys (−yG), then I_low keys (yG); 0 = not a member
  long long n;                 // total points over all problems (offset of the low keys)
  unsigned long long* gkey;    // [P][2] order-preserving keys of max(−yG, I_up), max(yG, I_low)
};

// One point per thread (valid ⇔ t < l); wave-level only (every lane of the wave must call it).
__device__ __forceinline__ void ws_publish_keys(const WsProb& P, int b, int t, bool valid, double a, double g,
                                                const WsAux& X) {
  double su = -kWsInf, sl = -kWsInf;
  if (valid) {
    unsigned ku = 0u, kl = 0u;
    const bool pos = t < P.npos;
    const double C = pos ? P.Cp : P.Cn;
    const double yg = pos ? g : -g;
    if (pos ? a < C : a > 0) { su = -yg; ku = ws_key(su); }
    if (pos ? a > 0 : a < C) { sl = yg; kl = ws_key(sl); }
    X.keys[P.aoff + t] = ku;
    X.keys[X.n + P.aoff + t] = kl;
  }
  su = wave_max_f64_exact(su);
  sl = wave_max_f64_exact(sl);
  if ((threadIdx.x & 63) == 0) {
    if (su > -kWsInf) atomicMax(&X.gkey[2 * b], f64_okey(su));
    if (sl > -kWsInf) atomicMax(&X.gkey[2 * b + 1], f64_okey(sl));
  }
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ws_init_kernel(const WsProb* __restrict__ probs, const float* __restrict__ zcat,
                                                      int F, float* __restrict__ zn, double* __restrict__ alpha,
                                                      double* __restrict__ G, WsState* __restrict__ states,
                                                      WsAux X) {
  const int b = blockIdx.y;
  const WsProb P = probs[b];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x * blockDim.x >= P.l) return;   // whole workgroup past the end
  if (blockIdx.x == 0 && threadIdx.x == 0) states[b] = WsState{0, 0, 0, 0.0, 0, 0, 0, 0, 0, 0, 0, 0};
  const bool valid = t < P.l;
  if (valid) {
    const float* z = zcat + (P.zoff + t) * F;
    float s = 0.f;
    for (int k = 0; k < F; ++k) s = fmaf(z[k], z[k], s);
    zn[P.aoff + t] = s;
    alpha[P.aoff + t] = 0.0;
    G[P.aoff + t] = -1.0;
  }
  ws_publish_keys(P, b, t, valid, 0.0, -1.0, X);
}

// M = points per lane.  Wave w owns the contiguous chunk [w·64M, (w+1)·64M) and lane L its points
// w·64M + m·64 + L: loads are coalesced and index order = (wave, m, lane), so ballots give
// index-ordered ranks.
template <int M>
__global__ __launch_bounds__(kWsThreads) void ws_select_solve_kernel(
    const WsProb* __restrict__ probs, WsState* __restrict__ states, const float* __restrict__ zcat, int F,
    const float* __restrict__ zn_all, double* __restrict__ alpha_all, const double* __restrict__ G_all,
    float* __restrict__ wsz, float* __restrict__ wsn, float* __restrict__ wdc, int Fp, double eps,
    int max_outer, int max_inner, double inner_frac, WsAux X) {
  const int b = blockIdx.x;
  WsState* S = states + b;
  if (S->done) return;
  const WsProb P = probs[b];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l = P.l;
  const int ldz = F | 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char ws_lds[];
  int* hist = reinterpret_cast<int*>(ws_lds);                          // [2][2048]
  float* KB = reinterpret_cast<float*>(hist + 4096);                   // [q][q+1]
  float* zB = KB + kWsQ * (kWsQ + 1);                                  // [q][F|1]
  float* znB = zB + kWsQ * ldz;                                        // [q]
  int* widx = reinterpret_cast<int*>(znB + kWsQ);                      // [q]
  __shared__ int shi[kWsWaves];
  __shared__ int binfo[8];
  const int t0 = wave * 64 * M + lane;

  const double* Gp = G_all + P.aoff;
  double* ap = alpha_all + P.aoff;
  const long long c0 = __builtin_amdgcn_s_memtime();
  // ---- global gap from the maxima published by the gradient kernel
  const unsigned long long gku = X.gkey[2 * b], gkl = X.gkey[2 * b + 1];
  const double Gmax = gku ? f64_from_okey(gku) : -kWsInf;
  const double Gmax2 = gkl ? f64_from_okey(gkl) : -kWsInf;
  const double gap = Gmax + Gmax2;
  // keys of this lane's points (coalesced: t = wave·64M + m·64 + lane) + member counts
  unsigned ku[M], kl[M];
  int nu = 0, nl = 0;
  // all loads issued before any use (one memory latency, not M of them)
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int t = t0 + 64 * m;
    ku[m] = t < l ? __builtin_nontemporal_load(X.keys + P.aoff + t) : 0u;
    kl[m] = t < l ? __builtin_nontemporal_load(X.keys + X.n + P.aoff + t) : 0u;
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    nu += __popcll(__ballot(ku[m] != 0u));
    nl += __popcll(__ballot(kl[m] != 0u));
  }
  for (int i = tid; i < 4096; i += kWsThreads) hist[i] = 0;
  if (tid < 8) binfo[tid] = 0;
  int n_up;
  wave_base(nu | (nl << 16), shi, &n_up);
  const int n_low = n_up >> 16;
  n_up &= 0xFFFF;
  if (!(gap >= eps) || S->outer >= max_outer || n_up == 0 || n_low == 0) {
    if (tid == 0) { S->done = 1; S->gap = gap; S->nc = 0; }
    return;
  }
  if (tid == 0) { X.gkey[2 * b] = 0ull; X.gkey[2 * b + 1] = 0ull; }   // consumed (all read it above)
  // ---- level-1 histograms (top 11 key bits)
#pragma unroll
  for (int m = 0; m < M; ++m) {
    hist_add(hist, ku[m] != 0u, (int)(ku[m] >> 21));
    hist_add(hist, kl[m] != 0u, 2048 + (int)(kl[m] >> 21));
  }
  __syncthreads();
  const int k_up = min(kWsHalf, n_up), k_low = min(kWsHalf, n_low);
  const long long c0a = __builtin_amdgcn_s_memtime();
  ws_find_bin(hist, k_up, k_low, shi, binfo);
  __syncthreads();
  const long long c0b = __builtin_amdgcn_s_memtime();
  const unsigned bu1 = binfo[0], bl1 = binfo[2];
  const int au1 = binfo[1], al1 = binfo[3];
  for (int i = tid; i < 4096; i += kWsThreads) hist[i] = 0;
  __syncthreads();
#pragma unroll
  for (int m = 0; m < M; ++m) {
    hist_add(hist, ku[m] != 0u && (ku[m] >> 21) == bu1, (int)((ku[m] >> 10) & 2047));
    hist_add(hist, kl[m] != 0u && (kl[m] >> 21) == bl1, 2048 + (int)((kl[m] >> 10) & 2047));
  }
  __syncthreads();
  ws_find_bin(hist, k_up - au1, k_low - al1, shi, binfo + 4);
  __syncthreads();
  const long long c0c = __builtin_amdgcn_s_memtime();
  const unsigned Tu = (bu1 << 11) | (unsigned)binfo[4], Tl = (bl1 << 11) | (unsigned)binfo[6];
  const int need_u = k_up - au1 - binfo[5], need_l = k_low - al1 - binfo[7];
  // ---- pass 3: index-ordered compaction (up list, then low list without the up picks)
  unsigned selm = 0u;
  int base = 0;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const unsigned T = side ? Tl : Tu;
    const int need = side ? need_l : need_u;
    // ranks of the boundary-prefix ties, in index order
    int wt = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const unsigned k = side ? kl[m] : ku[m];
      wt += __popcll(__ballot(k && (k >> 10) == T && !((selm >> m) & 1u)));
    }
    int ttot;
    int trank = wave_base(wt, shi, &ttot);
    unsigned pick = 0u;
    int ws_cnt = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const unsigned k = side ? kl[m] : ku[m];
      const bool cand = k && !((selm >> m) & 1u);
      const bool tie = cand && (k >> 10) == T;
      const unsigned long long tb = __ballot(tie);
      const bool take = cand && ((k >> 10) > T || (tie && trank + __popcll(tb & lanes_below()) < need));
      trank += __popcll(tb);
      if (take) pick |= 1u << m;
      ws_cnt += __popcll(__ballot(take));
    }
    int stot;
    int pos = base + wave_base(ws_cnt, shi, &stot);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const bool take = (pick >> m) & 1u;
      const unsigned long long tb = __ballot(take);
      if (take) widx[pos + __popcll(tb & lanes_below())] = t0 + 64 * m;
      pos += __popcll(tb);
    }
    selm |= pick;
    base += stot;
  }
  __syncthreads();
  const int nws = base;
  const long long c1 = __builtin_amdgcn_s_memtime();
  // ---- gather features of B and build K_BB in LDS (f32-input MFMA, one 32×32 tile per wave)
  for (int e = tid; e < nws * F; e += kWsThreads) {
    const int w = e / F, c = e - w * F;
    zB[w * ldz + c] = zcat[(P.zoff + widx[w]) * F + c];
  }
  for (int w = tid; w < nws; w += kWsThreads) znB[w] = zn_all[P.aoff + widx[w]];
  __syncthreads();
  {
    const int r32 = lane & 31, hi = lane >> 5;
    const int tr = wave >> 2, tc = wave & 3;   // 4 × 4 tiles of the 128 × 128 block
    if (tr * 32 < nws && tc * 32 < nws) {
      f32x16 acc = {0.f};
      const int ra = tr * 32 + r32, cb = tc * 32 + r32;
      for (int k0 = 0; k0 < F; k0 += 2) {
        const int k = k0 + hi;
        const float av = (k < F && ra < nws) ? zB[ra * ldz + k] : 0.f;
        const float bv = (k < F && cb < nws) ? zB[cb * ldz + k] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
      }
      // acc reg q ↔ row tr·32 + (q&3) + 8(q>>2) + 4·hi, column tc·32 + r32
      const int c = tc * 32 + r32;
      const float znc = c < nws ? znB[c] : 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int r = tr * 32 + (q & 3) + 8 * (q >> 2) + 4 * hi;
        if (r < nws && c < nws) {
          const float d2 = fmaxf(znB[r] + znc - 2.f * acc[q], 0.f);
          KB[r * (kWsQ + 1) + c] = r == c ? 1.f : __builtin_amdgcn_exp2f(P.ngl2e * d2);
        }
      }
    }
  }
  __syncthreads();
  if (tid >= 64) return;
  const long long c2 = __builtin_amdgcn_s_memtime();
  // ---- inner SMO on B: one wave, lane owns slots w = lane and lane + 64, local α/G in f32.
  // Pair selection uses u32 keys (order-preserving f32 with the slot in the low 7 bits) reduced
  // on DPP/permlane; libsvm's clipped two-variable step in f32.  The global state stays f64: the
  // published change is α_new − α_old with exact bound values (0 or C) kept exact.
  float a[2], g[2], Cw[2], ys[2];
  double a0[2];
  int tw[2];
  bool val[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int w = lane + 64 * s;
    val[s] = w < nws;
    tw[s] = val[s] ? widx[w] : 0;
    const bool pos = tw[s] < P.npos;
    ys[s] = pos ? 1.f : -1.f;
    a0[s] = val[s] ? ap[tw[s]] : 0.0;
    a[s] = (float)a0[s];
    g[s] = val[s] ? (float)Gp[tw[s]] : 0.f;
    Cw[s] = (float)(pos ? P.Cp : P.Cn);
  }
  float tol_in = -1.f;
  const float epsf = (float)eps;
  int it = 0;
  for (; it < max_inner; ++it) {
    // step 1: i = argmax_{I_up ∩ B} −y·G
    unsigned k1 = 0u;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool up = val[s] && (ys[s] > 0.f ? a[s] < Cw[s] : a[s] > 0.f);
      if (up) k1 = max(k1, (f32_okey(-ys[s] * g[s]) & ~0x7Fu) | (unsigned)(lane + 64 * s));
    }
    k1 = wave_max_u32(k1);
    if (k1 == 0u) break;
    const int i = (int)(k1 & 0x7Fu);
    const float Gi = readlane_f32(i < 64 ? g[0] : g[1], i & 63);
    const float yi = readlane_f32(i < 64 ? ys[0] : ys[1], i & 63);
    const float GmaxB = -yi * Gi;
    // step 2: j = argmax over I_low ∩ B of (GmaxB + yG)² / quad; K row i cached for the update
    float Ki[2];
    unsigned k2 = 0u, k3 = 0u;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Ki[s] = KB[i * (kWsQ + 1) + lane + 64 * s];
      const bool low = val[s] && (ys[s] > 0.f ? a[s] > 0.f : a[s] < Cw[s]);
      if (!low) continue;
      const float yG = ys[s] * g[s];
      k3 = max(k3, f32_okey(yG));
      const float gd = GmaxB + yG;
      if (gd > 0.f) {
        float quad = 2.f - 2.f * Ki[s];
        if (quad <= 0.f) quad = 1e-12f;
        k2 = max(k2, (f32_okey(gd * gd * __builtin_amdgcn_rcpf(quad)) & ~0x7Fu) | (unsigned)(lane + 64 * s));
      }
    }
    k2 = wave_max_u32(k2);
    k3 = wave_max_u32(k3);
    const float lgap = GmaxB + f32_from_okey(k3);
    if (tol_in < 0.f) tol_in = fmaxf(epsf, (float)inner_frac * lgap);
    if (lgap < tol_in || k2 == 0u) break;
    const int j = (int)(k2 & 0x7Fu);
    const float ai_old = readlane_f32(i < 64 ? a[0] : a[1], i & 63);
    const float aj_old = readlane_f32(j < 64 ? a[0] : a[1], j & 63);
    const float Gj = readlane_f32(j < 64 ? g[0] : g[1], j & 63);
    const float yj = readlane_f32(j < 64 ? ys[0] : ys[1], j & 63);
    const float Ci = readlane_f32(i < 64 ? Cw[0] : Cw[1], i & 63);
    const float Cj = readlane_f32(j < 64 ? Cw[0] : Cw[1], j & 63);
    const float Kij = KB[i * (kWsQ + 1) + j];
    float ai = ai_old, aj = aj_old;
    if (yi != yj) {
      float quad = 2.f + 2.f * (yi * yj) * Kij;
      if (quad <= 0.f) quad = 1e-12f;
      const float delta = (-Gi - Gj) * __builtin_amdgcn_rcpf(quad);
      const float diff = ai - aj;
      ai += delta;
      aj += delta;
      if (diff > 0.f) { if (aj < 0.f) { aj = 0.f; ai = diff; } }
      else { if (ai < 0.f) { ai = 0.f; aj = -diff; } }
      if (diff > Ci - Cj) { if (ai > Ci) { ai = Ci; aj = Ci - diff; } }
      else { if (aj > Cj) { aj = Cj; ai = Cj + diff; } }
    } else {
      float quad = 2.f - 2.f * (yi * yj) * Kij;
      if (quad <= 0.f) quad = 1e-12f;
      const float delta = (Gi - Gj) * __builtin_amdgcn_rcpf(quad);
      const float sum = ai + aj;
      ai -= delta;
      aj += delta;
      if (sum > Ci) { if (ai > Ci) { ai = Ci; aj = sum - Ci; } }
      else { if (aj < 0.f) { aj = 0.f; ai = sum; } }
      if (sum > Cj) { if (aj > Cj) { aj = Cj; ai = sum - Cj; } }
      else { if (ai < 0.f) { ai = 0.f; aj = sum; } }
    }
    const float ci = yi * (ai - ai_old), cj = yj * (aj - aj_old);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int w = lane + 64 * s;
      if (w == i) a[s] = ai;
      if (w == j) a[s] = aj;
      const float Kj = KB[j * (kWsQ + 1) + w];
      g[s] += ys[s] * fmaf(Ki[s], ci, Kj * cj);
    }
  }
  // ---- publish: α of B, changed entries (slot order) for the global gradient update
  int nc = 0;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    double anew = a0[s];
    if (val[s] && a[s] != (float)a0[s]) {
      const double C = ys[s] > 0.f ? P.Cp : P.Cn;
      anew = a[s] <= 0.f ? 0.0 : (a[s] >= Cw[s] ? C : a0[s] + ((double)a[s] - (double)(float)a0[s]));
    }
    const bool ch = val[s] && anew != a0[s];
    const unsigned long long mask = __ballot(ch);
    const int pos = nc + __popcll(mask & ((1ull << lane) - 1ull));
    if (ch) {
      const int w = lane + 64 * s;
      ap[tw[s]] = anew;
      for (int k = 0; k < Fp; ++k) wsz[((size_t)b * Fp + k) * kWsQ + pos] = k < F ? zB[w * ldz + k] : 0.f;
      wsn[(size_t)b * kWsQ + pos] = P.ngl2e * znB[w];
      wdc[(size_t)b * kWsQ + pos] = (float)((double)ys[s] * (anew - a0[s]));
    }
    nc += __popcll(mask);
  }
  const int ncp = (nc + 31) & ~31;
  for (int pos = nc + lane; pos < ncp; pos += 64) {
    for (int k = 0; k < Fp; ++k) wsz[((size_t)b * Fp + k) * kWsQ + pos] = 0.f;
    wsn[(size_t)b * kWsQ + pos] = 0.f;
    wdc[(size_t)b * kWsQ + pos] = 0.f;
  }
  const long long c3 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    S->cyc_select += c1 - c0;
    S->cyc_p0 += c0a - c0;
    S->cyc_p1 += c0b - c0a;
    S->cyc_p2 += c0c - c0b;
    S->cyc_build += c2 - c1;
    S->cyc_inner += c3 - c2;
    // no pair moved: the f32 selection keys hid an f64 violation below eps-resolution — done
    if (it == 0 || nc == 0) S->done = 1;
    S->nc = nc;
    S->nws = nws;
    S->outer += 1;
    S->inner += it;
    S->gap = gap;
  }
}

// G_t += y_t · Σ_c dc_c · exp2(γ'‖x_t − x_c‖²) for every point t of every active problem, then t's
// selection keys for the next working set.
template <int KS>
__global__ __launch_bounds__(256) void ws_gupdate_kernel(const WsProb* __restrict__ probs,
                                                         const WsState* __restrict__ states,
                                                         const float* __restrict__ zcat, int F,
                                                         const float* __restrict__ zn_all,
                                                         const double* __restrict__ alpha_all,
                                                         double* __restrict__ G_all,
                                                         const float* __restrict__ wsz,
                                                         const float* __restrict__ wsn,
                                                         const float* __restrict__ wdc, int Fp, WsAux X) {
  const int b = blockIdx.y;
  const int nc = states[b].nc;
  if (nc == 0) return;
  const WsProb P = probs[b];
  const int row_blk = blockIdx.x * 256;
  if (row_blk >= P.l) return;
  const int ncp = (nc + 31) & ~31;
  __shared__ __attribute__((aligned(16))) float sv_l[2 * KS * kWsQ];
  __shared__ __attribute__((aligned(16))) float sn_l[kWsQ];
  __shared__ __attribute__((aligned(16))) float cf_l[kWsQ];
  for (int i = threadIdx.x; i < 2 * KS * ncp; i += blockDim.x) {
    const int k = i / ncp, c = i - k * ncp;
    sv_l[k * kWsQ + c] = k < Fp ? wsz[((size_t)b * Fp + k) * kWsQ + c] : 0.f;
  }
  for (int c = threadIdx.x; c < ncp; c += blockDim.x) {
    sn_l[c] = wsn[(size_t)b * kWsQ + c];
    cf_l[c] = wdc[(size_t)b * kWsQ + c];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r32 = lane & 31, hi = lane >> 5;
  const int r0 = row_blk + wave * 64;
  const int row = r0 + lane;
  const bool valid = row < P.l;
  if (r0 >= P.l) return;   // wave-uniform
  // issue this lane's G/α loads first: their latency hides under the MFMA work
  const double gold = valid ? G_all[P.aoff + row] : 0.0;
  const double a = valid ? alpha_all[P.aoff + row] : 0.0;
  double gnew = 0.0;
  const int ra = r0 + r32, rb = r0 + 32 + r32;
  float za[KS], zb[KS];
  const float* zA = zcat + (P.zoff + ra) * F;
  const float* zBp = zcat + (P.zoff + rb) * F;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 2 * s + hi;
    za[s] = (k < F && ra < P.l) ? zA[k] : 0.f;
    zb[s] = (k < F && rb < P.l) ? zBp[k] : 0.f;
  }
  const float zsa = ra < P.l ? P.ngl2e * zn_all[P.aoff + ra] : 0.f;
  const float zsb = rb < P.l ? P.ngl2e * zn_all[P.aoff + rb] : 0.f;
  const float k2 = -2.f * P.ngl2e;
  float pa = 0.f, pb = 0.f;
  for (int t = 0; t < ncp; t += 32) {
    f32x16 A = {0.f}, B = {0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float sv = sv_l[(2 * s + hi) * kWsQ + t + r32];
      A = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, za[s], A, 0, 0, 0);
      B = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, zb[s], B, 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = t + 8 * g + 4 * hi;
      const f32x4 snv = *reinterpret_cast<const f32x4*>(&sn_l[c0]);
      const f32x4 cfv = *reinterpret_cast<const f32x4*>(&cf_l[c0]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pa = fmaf(cfv[q], __builtin_amdgcn_exp2f(fminf(fmaf(k2, A[4 * g + q], snv[q] + zsa), 0.f)), pa);
        pb = fmaf(cfv[q], __builtin_amdgcn_exp2f(fminf(fmaf(k2, B[4 * g + q], snv[q] + zsb), 0.f)), pb);
      }
    }
  }
  pa += __shfl_xor(pa, 32, kWave);
  pb += __shfl_xor(pb, 32, kWave);
  if (valid) {
    const double upd = (double)(lane < 32 ? pa : pb);
    gnew = gold + (row < P.npos ? upd : -upd);
    G_all[P.aoff + row] = gnew;
  }
  ws_publish_keys(P, b, row, valid, a, gnew, X);
}

// libsvm calculate_rho over the final gradient.
__global__ __launch_bounds__(kWsThreads) void ws_finalize_kernel(const WsProb* __restrict__ probs,
                                                                 const WsState* __restrict__ states,
                                                                 const double* __restrict__ alpha_all,
                                                                 const double* __restrict__ G_all,
                                                                 double* __restrict__ rho, int* __restrict__ iters,
                                                                 long long* __restrict__ inner,
                                                                 double* __restrict__ gap) {
  const WsProb P = probs[blockIdx.x];
  __shared__ double shd[kWsWaves];
  double ub = kWsInf, lb = -kWsInf, sum_free = 0.0, nfree = 0.0;
  for (int t = threadIdx.x; t < P.l; t += kWsThreads) {
    const bool pos = t < P.npos;
    const double a = alpha_all[P.aoff + t], g = G_all[P.aoff + t];
    const double C = pos ? P.Cp : P.Cn;
    const double yG = pos ? g : -g;
    if (a >= C) {
      if (!pos) ub = fmin(ub, yG); else lb = fmax(lb, yG);
    } else if (a <= 0) {
      if (pos) ub = fmin(ub, yG); else lb = fmax(lb, yG);
    } else {
      nfree += 1.0;
      sum_free += yG;
    }
  }
  const double UB = -block_max_f64(-ub, shd);
  const double LB = block_max_f64(lb, shd);
  const double SF = block_sum_f64(sum_free, shd);
  const double NF = block_sum_f64(nfree, shd);
  if (threadIdx.x == 0) {
    rho[blockIdx.x] = NF > 0 ? SF / NF : (UB + LB) / 2;
    iters[blockIdx.x] = states[blockIdx.x].outer;
    inner[blockIdx.x] = states[blockIdx.x].inner;
    gap[blockIdx.x] = states[blockIdx.x].gap;
  }
}

// ------------------------------------------------------------------------------------------
static size_t ws_lds_bytes(int F) {
  return (size_t)4096 * 4 + (size_t)kWsQ * (kWsQ + 1) * 4 + (size_t)kWsQ * (F | 1) * 4 + kWsQ * 4 + kWsQ * 4;
}

static int ws_ks(int F) {
  const int ks = (F + 1) / 2;
  return ks <= 4 ? 4 : ks <= 9 ? 9 : ks <= 12 ? 12 : ks <= 16 ? 16 : 32;
}

static WsAux ws_aux(uintptr_t keys, long long n, uintptr_t hist, uintptr_t gkey) {
  (void)hist;
  return WsAux{(unsigned*)keys, n, (unsigned long long*)gkey};
}

void ws_init(uintptr_t probs, int P, int max_l, uintptr_t zcat, int F, uintptr_t zn, uintptr_t alpha,
             uintptr_t G, uintptr_t states, uintptr_t keys, long long n, uintptr_t hist, uintptr_t gkey,
             uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "ws_init: 1 <= F <= 64");
  if (P == 0 || max_l == 0) return;
  hipLaunchKernelGGL(ws_init_kernel, dim3((max_l + 255) / 256, P), dim3(256), 0, as_stream(stream),
                     (const WsProb*)probs, (const float*)zcat, F, (float*)zn, (double*)alpha, (double*)G,
                     (WsState*)states, ws_aux(keys, n, hist, gkey));
  launch_check();
}

// n_iter outer iterations (select+solve, then the gradient update) enqueued back to back.
void ws_steps(uintptr_t probs, int P, int max_l, uintptr_t zcat, int F, uintptr_t zn, uintptr_t alpha,
              uintptr_t G, uintptr_t states, uintptr_t wsz, uintptr_t wsn, uintptr_t wdc, uintptr_t keys,
              long long n, uintptr_t hist, uintptr_t gkey, double eps, int max_outer, int max_inner,
              double inner_frac, int n_iter, uintptr_t stream) {
  const WsAux X = ws_aux(keys, n, hist, gkey);
  HFENS_REQUIRE(F >= 1 && F <= 64, "ws_steps: 1 <= F <= 64");
  // (< 32768: the packed 16|16-bit member counts of the radix selector)
  HFENS_REQUIRE(max_l < 32 * kWsThreads, "ws_steps: problems of 32768+ points need the multi-workgroup selector");
  if (P == 0 || max_l == 0) return;
  hipStream_t st = as_stream(stream);
  const int KS = ws_ks(F);
  const int Fp = 2 * KS;
  const size_t lds = ws_lds_bytes(F);
  auto pp = (const WsProb*)probs;
  auto sp = (WsState*)states;
  auto zp = (const float*)zcat;
  auto np_ = (const float*)zn;
  auto ap = (double*)alpha;
  auto gp = (double*)G;
  auto wz = (float*)wsz;
  auto wn = (float*)wsn;
  auto wd = (float*)wdc;
  for (int it = 0; it < n_iter; ++it) {
#define WS_SEL(MM)                                                                                      \
  if (max_l <= MM * kWsThreads) {                                                                       \
    hipLaunchKernelGGL(ws_select_solve_kernel<MM>, dim3(P), dim3(kWsThreads), lds, st, pp, sp, zp, F,  \
                       np_, ap, gp, wz, wn, wd, Fp, eps, max_outer, max_inner, inner_frac, X);          \
  } else
    WS_SEL(1) WS_SEL(2) WS_SEL(4) WS_SEL(8) WS_SEL(16) WS_SEL(32) {}
#undef WS_SEL
    launch_check();
    const dim3 grid((max_l + 255) / 256, P);
#define WS_UPD(K)                                                                                    \
  case K:                                                                                           \
    hipLaunchKernelGGL(ws_gupdate_kernel<K>, grid, dim3(256), 0, st, pp, sp, zp, F, np_, ap, gp, wz, \
                       wn, wd, Fp, X);                                                              \
    break;
    switch (KS) { WS_UPD(4) WS_UPD(9) WS_UPD(12) WS_UPD(16) WS_UPD(32) }
#undef WS_UPD
    launch_check();
  }
}

void ws_finalize(uintptr_t probs, int P, uintptr_t states, uintptr_t alpha, uintptr_t G, uintptr_t rho,
                 uintptr_t iters, uintptr_t inner, uintptr_t gap, uintptr_t stream) {
  if (P == 0) return;
  hipLaunchKernelGGL(ws_finalize_kernel, dim3(P), dim3(kWsThreads), 0, as_stream(stream), (const WsProb*)probs,
                     (const WsState*)states, (const double*)alpha, (const double*)G, (double*)rho, (int*)iters,
                     (long long*)inner, (double*)gap);
  launch_check();
}

}  // namespace hfens
