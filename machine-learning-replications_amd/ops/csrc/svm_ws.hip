// Working-set decomposition SMO for batches of C-SVC duals (the reference
// fits libsvm through sklearn SVC, train_ensemble_public.py:43-48, 61).
//
// libsvm's SMO moves ONE pair per iteration, and every iteration is a chain of two global
// reductions and two dependent kernel-row reads.  Spread over CUs (svm_coop.hip) each reduction is
// a cross-workgroup hand-off, so a pair costs ~7.7 µs and the bench's 10k-point problem (~7.6k
// pairs) ~56 ms.  This solver keeps libsvm's dual, its WSS3 pair rule INSIDE a large working set
// and libsvm's global stopping rule (m(α) − M(α) < eps over ALL points, f64), and moves the
// sequential part into one CU:
//
//   ws_select_solve (one 1024-thread workgroup per problem)
//     1. global gap m − M (f64) from the maxima the gradient kernel published; convergence test;
//     2. working set B (q = 1024, or 512 for F > 24): the q/4 most violating points of I_up and
//        of I_low (two-level 11-bit radix histograms in LDS, index-ordered tie compaction:
//        deterministic), plus the previous round's new picks that were not picked again
//        (ThunderSVM-style half reuse: on the bench's 10k problem 35 outer rounds instead of
//        ~280 without reuse, scripts/ws_sim.py);
//     3. the features of B into LDS; every thread owns ONE slot of B, its features in registers;
//     4. inner SMO on B: libsvm's WSS3 pair rule and clipping on the local gradient; each kernel
//        row K(x_i, ·) is recomputed in registers (F fmas + one exp2 per slot, the same f32
//        expression as the gradient kernel's MFMA, bit for bit), so a pair is two block
//        reductions (DPP/permlane wave max + one barrier each) and no memory traffic beyond LDS;
//     5. publishes the changed coefficients y_i·Δα_i and their feature rows (MFMA layout).
//   ws_gupdate (grid = row tiles × problems)
//     G_t += y_t Σ_{c changed} y_c Δα_c K(x_t, x_c) for every t: an RBF "GEMM + exp + GEMV" on the
//     f32-input MFMA in 256-coefficient chunks — the kernel matrix is recomputed, never stored:
//     O(n·F) memory instead of the exact solver's O(n²) Gram.
//
// Results meet libsvm's KKT tolerance but follow a different pair sequence, so α agrees with
// libsvm to O(eps), not bit for bit (the exact-sequence solvers stay in svm.hip / svm_coop.hip for
// small problems and parity tests).  Deterministic: no order-dependent atomics.
#include <type_traits>

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
  int nws;          // size of the last working set
  int nprev;        // new picks of the last round (kept in wsprev for the next working set)
  int pad;
  long long cyc_select, cyc_build, cyc_inner;   // s_memtime phase totals (diagnostics)
  long long cyc_p0, cyc_p1, cyc_p2;             // selection sub-phases: gap pass, level-1, level-2
};
static_assert(sizeof(WsState) == 88, "WsState layout is mirrored in models/smo.py");

constexpr int kWsThreads = 1024;
constexpr int kWsWaves = kWsThreads / 64;
constexpr int kWsChunk = 256;      // changed coefficients staged per LDS pass of ws_gupdate
constexpr double kWsTau = 1e-12;
constexpr double kWsInf = 1.0e300;

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
// G = −1 at the start) one lane adds the popcount instead of 64 serialized atomics.  (Folding up to
// three clusters per instruction was measured slower: 23 → 35 µs per selection, r4d.)
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

__device__ __forceinline__ unsigned ws_key(double v) { return f32_okey((float)v); }

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
  if (blockIdx.x == 0 && threadIdx.x == 0) states[b] = WsState{0, 0, 0, 0.0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
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

// ---- ws_select: the next working set (one 1024-thread workgroup per problem) -------------------
// LDS (dynamic region only, every block a multiple of 16 bytes): scan scratch (16 ints), bin info
// (8), histograms [2][2048] int, membership bitmap [1024] u32 (points picked this round), widx [Q].
constexpr size_t ws_sel_lds_bytes(int Q) { return 32 * 4 + 4096 * 4 + 1024 * 4 + (size_t)Q * 4; }

// M = points per lane.  Wave w owns the contiguous chunk [w·64M, (w+1)·64M) and lane L its points
// w·64M + m·64 + L: loads are coalesced and index order = (wave, m, lane), so ballots give
// index-ordered ranks.
//
// ws_pick_lists: the k_up largest non-zero I_up keys, then the k_low largest I_low keys among the
// positions not picked for I_up (two-level 11-bit radix histograms in LDS, ties taken in position
// order: deterministic).  emit(i, p) is called for every pick (i = output slot, new picks of the up
// list first, each list in position order); returns the pick count.  Every thread calls it.
template <int M, typename Emit>
__device__ __forceinline__ int ws_pick_lists(const unsigned (&ku)[M], const unsigned (&kl)[M], int t0, int k_up,
                                             int k_low, int* shi, int* binfo, int* hist, Emit emit) {
  const int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += kWsThreads) hist[i] = 0;
  if (tid < 8) binfo[tid] = 0;
  __syncthreads();
  // ---- level-1 histograms (top 11 key bits)
#pragma unroll
  for (int m = 0; m < M; ++m) {
    hist_add(hist, ku[m] != 0u, (int)(ku[m] >> 21));
    hist_add(hist, kl[m] != 0u, 2048 + (int)(kl[m] >> 21));
  }
  __syncthreads();
  ws_find_bin(hist, k_up, k_low, shi, binfo);
  __syncthreads();
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
  const unsigned Tu = (bu1 << 11) | (unsigned)binfo[4], Tl = (bl1 << 11) | (unsigned)binfo[6];
  const int need_u = k_up - au1 - binfo[5], need_l = k_low - al1 - binfo[7];
  // ---- position-ordered compaction (up list, then low list without the up picks)
  unsigned selm = 0u;
  int base = 0;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const unsigned T = side ? Tl : Tu;
    const int need = side ? need_l : need_u;
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
      if (take) emit(pos + __popcll(tb & lanes_below()), t0 + 64 * m);
      pos += __popcll(tb);
    }
    selm |= pick;
    base += stot;
  }
  return base;
}

// Candidate lists for problems too large for one workgroup's selector (ws_cand_kernel): per block
// of kWsCandBlk points the union of its top-(Q/4) I_up and top-(Q/4) I_low points, as (index, up key,
// low key) in ncand = blocks · kWsCandPer slots per problem (unused slots: key 0).  The global top
// of each list is the top of the union of the blocks' tops, so the selector then only reads the
// candidates.
struct WsCand {
  int* idx;          // [P][ncand] point index (−1: empty)
  unsigned* ku;      // [P][ncand]
  unsigned* kl;      // [P][ncand]
  int ncand;         // 0: the selector reads every point's keys
};
constexpr int kWsCandM = 8;
constexpr int kWsCandBlk = kWsCandM * kWsThreads;   // 8192 points per candidate block

// The selection body, shared by ws_select_kernel and the fused K-cached round (ws_kc_round_kernel):
// every thread of the 1024-thread workgroup calls it; returns the working-set size (B in widx[0, nws),
// LDS, visible to every thread on return) or −1 when problem b is done.  LDS: shi [16], binfo [16],
// hist [2][2048], bm [1024] (both dead on return), widx [Q].  kCand: the keys come from the
// candidate lists C (positions → point indices) instead of every point.
template <int M, int Q, bool kWriteIdx, bool kCand = false>
__device__ __forceinline__ int ws_select_body(const WsProb& P, int b, WsState* S, int* __restrict__ wsidx,
                                              int* __restrict__ wsprev, double eps, int max_outer, const WsAux& X,
                                              int* shi, int* binfo, int* hist, unsigned* bm, int* widx,
                                              const WsCand& C = WsCand{nullptr, nullptr, nullptr, 0}) {
  const int nprev = S->nprev;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int L = kCand ? C.ncand : P.l;
  const int t0 = wave * 64 * M + lane;
  const long long c0 = __builtin_amdgcn_s_memtime();
  // ---- global gap from the maxima published by the gradient kernel
  const unsigned long long gku = X.gkey[2 * b], gkl = X.gkey[2 * b + 1];
  const double Gmax = gku ? f64_from_okey(gku) : -kWsInf;
  const double Gmax2 = gkl ? f64_from_okey(gkl) : -kWsInf;
  const double gap = Gmax + Gmax2;
  // keys of this lane's points (candidates) + member counts; all loads issued before any use
  unsigned ku[M], kl[M];
  int nu = 0, nl = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int t = t0 + 64 * m;
    if (kCand) {
      ku[m] = t < L ? C.ku[(size_t)b * C.ncand + t] : 0u;
      kl[m] = t < L ? C.kl[(size_t)b * C.ncand + t] : 0u;
    } else {
      ku[m] = t < L ? __builtin_nontemporal_load(X.keys + P.aoff + t) : 0u;
      kl[m] = t < L ? __builtin_nontemporal_load(X.keys + X.n + P.aoff + t) : 0u;
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    nu += __popcll(__ballot(ku[m] != 0u));
    nl += __popcll(__ballot(kl[m] != 0u));
  }
  if (!kCand)
    for (int i = tid; i < 1024; i += kWsThreads) bm[i] = 0;
  int n_up;
  wave_base(nu | (nl << 16), shi, &n_up);
  const int n_low = n_up >> 16;
  n_up &= 0xFFFF;
  if (!(gap >= eps) || S->outer >= max_outer || n_up == 0 || n_low == 0) {
    if (tid == 0) { S->done = 1; S->gap = gap; S->nc = 0; S->nws = 0; }
    return -1;
  }
  if (tid == 0) { X.gkey[2 * b] = 0ull; X.gkey[2 * b + 1] = 0ull; }   // consumed (all read it above)
  const int k_up = min(Q / 4, n_up), k_low = min(Q / 4, n_low);
  const long long c0a = __builtin_amdgcn_s_memtime();
  const int nnew = ws_pick_lists<M>(ku, kl, t0, k_up, k_low, shi, binfo, hist, [&](int i, int p) {
    if (kCand) {
      widx[i] = C.idx[(size_t)b * C.ncand + p];
    } else {
      widx[i] = p;
      atomicOr(&bm[p >> 5], 1u << (p & 31));
    }
  });
  const long long c0b = __builtin_amdgcn_s_memtime();
  const long long c0c = c0b;
  __syncthreads();
  // ---- the previous round's new picks that were not picked again (in their old order)
  const int pv = tid < nprev ? wsprev[(size_t)b * (Q / 2) + tid] : -1;
  bool again = false;
  if (pv >= 0) {
    if (kCand) {
      for (int w = 0; w < nnew; ++w) again |= widx[w] == pv;
    } else {
      again = (bm[pv >> 5] >> (pv & 31)) & 1u;
    }
  }
  const bool keep = pv >= 0 && !again;
  const unsigned long long kb = __ballot(keep);
  int ktot;
  const int kpos = nnew + wave_base(__popcll(kb), shi, &ktot) + __popcll(kb & lanes_below());
  if (keep) widx[kpos] = pv;
  __syncthreads();   // every old entry was read before the new picks overwrite the list
  const int nws = nnew + ktot;
  for (int w = tid; w < nnew; w += kWsThreads) wsprev[(size_t)b * (Q / 2) + w] = widx[w];
  if (kWriteIdx)
    for (int w = tid; w < nws; w += kWsThreads) wsidx[(size_t)b * Q + w] = widx[w];
  const long long c1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) {
    S->cyc_select += c1 - c0;
    S->cyc_p0 += c0a - c0;
    S->cyc_p1 += c0b - c0a;
    S->cyc_p2 += c0c - c0b;
    S->nws = nws;
    S->nprev = nnew;
    S->gap = gap;
  }
  return nws;
}

// Stage 1 of the selection for large problems: grid = (blocks of kWsCandBlk points, P).  Each block
// writes the union of its top-(Q/4) I_up and I_low points to its kWsCandPer(Q) candidate slots.
template <int Q>
__global__ __launch_bounds__(kWsThreads) void ws_cand_kernel(const WsProb* __restrict__ probs,
                                                             const WsState* __restrict__ states, WsAux X, WsCand C) {
  constexpr int M = kWsCandM;
  constexpr int per = Q / 2;   // candidate slots per block
  const int b = blockIdx.y, blk = blockIdx.x;
  if (states[b].done) return;
  const WsProb P = probs[b];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int beg = blk * kWsCandBlk;
  int* out_idx = C.idx + (size_t)b * C.ncand + (size_t)blk * per;
  unsigned* out_ku = C.ku + (size_t)b * C.ncand + (size_t)blk * per;
  unsigned* out_kl = C.kl + (size_t)b * C.ncand + (size_t)blk * per;
  __shared__ int shi[16], binfo[16];
  __shared__ int hist[4096];
  __shared__ int pick[per];
  const int t0 = wave * 64 * M + lane;
  unsigned ku[M], kl[M];
  int nu = 0, nl = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int t = beg + t0 + 64 * m;
    ku[m] = t < P.l ? __builtin_nontemporal_load(X.keys + P.aoff + t) : 0u;
    kl[m] = t < P.l ? __builtin_nontemporal_load(X.keys + X.n + P.aoff + t) : 0u;
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    nu += __popcll(__ballot(ku[m] != 0u));
    nl += __popcll(__ballot(kl[m] != 0u));
  }
  int n_up;
  wave_base(nu | (nl << 16), shi, &n_up);
  const int n_low = n_up >> 16;
  n_up &= 0xFFFF;
  const int np = (n_up == 0 && n_low == 0) ? 0
                 : ws_pick_lists<M>(ku, kl, t0, min(Q / 4, n_up), min(Q / 4, n_low), shi, binfo, hist,
                                    [&](int i, int p) { pick[i] = beg + p; });
  __syncthreads();
  if (tid < per) {
    const int t = tid < np ? pick[tid] : -1;
    out_idx[tid] = t;
    out_ku[tid] = t >= 0 ? X.keys[P.aoff + t] : 0u;
    out_kl[tid] = t >= 0 ? X.keys[X.n + P.aoff + t] : 0u;
  }
}

template <int M, int Q>
__global__ __launch_bounds__(kWsThreads) void ws_select_kernel(
    const WsProb* __restrict__ probs, WsState* __restrict__ states, int* __restrict__ wsidx,
    int* __restrict__ wsprev, double eps, int max_outer, WsAux X) {
  const int b = blockIdx.x;
  WsState* S = states + b;
  if (S->done) return;
  const WsProb P = probs[b];
  extern __shared__ __attribute__((aligned(16))) unsigned char ws_lds[];
  int* shi = reinterpret_cast<int*>(ws_lds);                     // [16]
  int* binfo = shi + 16;                                         // [8] (+8 pad)
  int* hist = shi + 32;                                          // [2][2048]
  unsigned* bm = reinterpret_cast<unsigned*>(hist + 4096);       // [1024]
  int* widx = reinterpret_cast<int*>(bm + 1024);                 // [Q]
  ws_select_body<M, Q, true>(P, b, S, wsidx, wsprev, eps, max_outer, X, shi, binfo, hist, bm, widx);
}

// ---- ws_solve: the inner SMO on B (one TH-thread workgroup per problem) ------------------------
// TH/64 waves, SL = Q/TH slots per thread (slot s = tid + TH·m), each slot's features in
// registers.  LDS: reduction slots (4 keys × 2 parities × 4 waves), z_B [Q][FP] f32, γ'‖z‖² [Q],
// widx [Q], and per-slot mirrors of g, α and K(x_i,·), 2 parities each (a slot is read by every
// thread after the barrier that follows its write, and rewritten only two barriers later).
constexpr size_t ws_solve_lds_bytes(int Q, int FP) {
  return 64 * 4 + (size_t)Q * FP * 4 + (size_t)Q * 4 * 2 + (size_t)6 * Q * 4;
}

template <int FP, int Q, int TH>
__global__ __launch_bounds__(TH) void ws_solve_kernel(
    const WsProb* __restrict__ probs, WsState* __restrict__ states, const float* __restrict__ zcat, int F,
    const float* __restrict__ zn_all, double* __restrict__ alpha_all, const double* __restrict__ G_all,
    const int* __restrict__ wsidx, float* __restrict__ wsz, float* __restrict__ wsn, float* __restrict__ wdc,
    int Fp2, double eps, int max_inner, double inner_frac, long long* __restrict__ prof) {
  static_assert(Q % TH == 0 && (Q & (Q - 1)) == 0 && TH % 64 == 0 && TH <= 512, "whole slots per thread");
  static_assert(FP % 4 == 0, "z rows are read as float4");
  constexpr int SL = Q / TH;
  static_assert(SL % 2 == 0, "slots go in pairs (packed f32 fma)");
  constexpr int NW = TH / 64;        // waves
  constexpr unsigned kIdx = Q - 1;   // slot bits packed under the selection keys
  const int b = blockIdx.x;
  WsState* S = states + b;
  if (S->done) return;
  const WsProb P = probs[b];
  const int nws = S->nws;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  extern __shared__ __attribute__((aligned(16))) unsigned char ws_lds[];
  unsigned* red = reinterpret_cast<unsigned*>(ws_lds);            // [4 keys][2 parities][NW ≤ 8 waves]
  float* zB = reinterpret_cast<float*>(ws_lds + 64 * 4);       // [Q][FP]
  float* snB = zB + (size_t)Q * FP;                                 // [Q]
  int* widx = reinterpret_cast<int*>(snB + Q);                      // [Q]
  float* gl = reinterpret_cast<float*>(widx + Q);                   // [2][Q]
  float* al = gl + 2 * Q;                                           // [2][Q]
  float* kil = al + 2 * Q;                                          // [2][Q]
  const double* Gp = G_all + P.aoff;
  double* ap = alpha_all + P.aoff;
  const long long c1 = __builtin_amdgcn_s_memtime();
  // features of B: thread s loads the rows of its own slots (all loads in flight at once) into
  // LDS, zero-padded to FP (the padded terms of the dot are exact no-ops)
  {
    int wi[SL];
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int s = tid + TH * m;
      wi[m] = s < nws ? wsidx[(size_t)b * Q + s] : -1;
    }
    float zv[SL][FP];
    float znv[SL];
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const float* zrow = zcat + (P.zoff + (wi[m] < 0 ? 0 : wi[m])) * F;
#pragma unroll
      for (int k = 0; k < FP; ++k) zv[m][k] = (wi[m] >= 0 && k < F) ? zrow[k] : 0.f;
      znv[m] = wi[m] >= 0 ? zn_all[P.aoff + wi[m]] : 0.f;
    }
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int s = tid + TH * m;
      widx[s] = wi[m] < 0 ? 0 : wi[m];
      snB[s] = P.ngl2e * znv[m];
#pragma unroll
      for (int k = 0; k < FP; k += 4)
        *reinterpret_cast<f32x4*>(&zB[s * FP + k]) = f32x4{zv[m][k], zv[m][k + 1], zv[m][k + 2], zv[m][k + 3]};
    }
  }
  __syncthreads();
  const long long c2 = __builtin_amdgcn_s_memtime();
  const long long r2 = __builtin_amdgcn_s_memrealtime();   // (100 MHz: the inner phase's clock, diagnostics)
  bool valid[SL], pos[SL];
  int tt[SL];
  // yg = y·G (the solver's natural variable: keys −yG / yG, gd = GmaxB + yG, and the update
  // yG += K_i c_i + K_j c_j with y² = 1 — bit for bit y·(G + y·Δ) since ×(±1) is exact); the
  // I_up / I_low tests as y·α < tu and −y·α < tl with per-slot bounds (−∞ for empty slots)
  float y[SL], Cw[SL], a[SL], yg[SL], sn[SL], tu[SL], tl[SL];
  double a0[SL];
  f32x2 zp[SL / 2][FP];   // features of slots (2h, 2h+1) side by side: one v_pk_fma_f32 per k
#pragma unroll
  for (int m = 0; m < SL; ++m) {
    const int s = tid + TH * m;
    valid[m] = s < nws;
    tt[m] = valid[m] ? widx[s] : 0;
    pos[m] = tt[m] < P.npos;
    y[m] = pos[m] ? 1.f : -1.f;
    Cw[m] = (float)(pos[m] ? P.Cp : P.Cn);
    tu[m] = valid[m] ? (pos[m] ? Cw[m] : 0.f) : -INFINITY;
    tl[m] = valid[m] ? (pos[m] ? 0.f : Cw[m]) : -INFINITY;
    a0[m] = valid[m] ? ap[tt[m]] : 0.0;
    a[m] = (float)a0[m];
    yg[m] = valid[m] ? y[m] * (float)Gp[tt[m]] : 0.f;
    sn[m] = valid[m] ? snB[s] : 0.f;
#pragma unroll
    for (int k = 0; k < FP; k += 4) {
      const f32x4 v = valid[m] ? *reinterpret_cast<const f32x4*>(&zB[s * FP + k]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) zp[m / 2][k + q][m & 1] = v[q];
    }
  }
  const float k2c = -2.f * P.ngl2e;
  const float Cpf = (float)P.Cp, Cnf = (float)P.Cn;
  // K(x_r, x_s) for every slot s of this thread: the gradient kernel's expression (MFMA = k-ordered
  // fma chain from 0), so the inner solver and ws_gupdate see the same f32 kernel values
  // (packed: each lane of the pair is the same k-ordered fma chain, bit for bit)
  auto krow = [&](int r, float (&out)[SL]) {
    f32x2 d[SL / 2];
#pragma unroll
    for (int h = 0; h < SL / 2; ++h) d[h] = f32x2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < FP; k += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(&zB[r * FP + k]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int h = 0; h < SL / 2; ++h) d[h] = __builtin_elementwise_fma(f32x2{v[q], v[q]}, zp[h][k + q], d[h]);
      }
    }
    const float snr = snB[r];
#pragma unroll
    for (int m = 0; m < SL; ++m)
      out[m] = __builtin_amdgcn_exp2f(fminf(fmaf(k2c, d[m / 2][m & 1], snr + sn[m]), 0.f));
  };
  auto red4 = [&](const unsigned* r) {   // max over the NW waves' slots (uint4 reads)
    unsigned x = 0u;
#pragma unroll
    for (int w = 0; w < NW; w += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(r + w);
      x = max(max(x, max(v.x, v.y)), max(v.z, v.w));
    }
    return x;
  };
  float tol_in = -1.f;
  const float epsf = (float)eps;
  // optional in-kernel phase stamps (HFENS_PROFILE_WS=1): keys, barrier 1, row i, barrier 2,
  // pair update, row j + gradient — s_memtime waits for outstanding LDS reads, so this perturbs
  // (compiled in only with -DHFENS_WS_STAMPS: even an untaken stamp costs scalar work per pair)
#ifdef HFENS_WS_STAMPS
  const bool pf = prof != nullptr;
  long long ph[6] = {0, 0, 0, 0, 0, 0};
  long long tp = pf ? __builtin_amdgcn_s_memtime() : 0;
#define WS_STAMP(k)                                         \
  if (pf) {                                                 \
    const long long tn = __builtin_amdgcn_s_memtime();      \
    ph[k] += tn - tp;                                       \
    tp = tn;                                                \
  }
#else
  const bool pf = false;
  long long ph[6] = {0, 0, 0, 0, 0, 0};
#define WS_STAMP(k)
#endif
  int it = 0;
  // one pair; false = stop.  Unrolled by parity (compile-time mirror / reduction-slot offsets)
  auto pair = [&](auto parc) -> bool {
    constexpr int par = decltype(parc)::value;
    float* glp = gl + par * Q;
    float* alp = al + par * Q;
    float* kip = kil + par * Q;
    unsigned* r1 = red + (0 * 2 + par) * NW;   // step-1 keys (slot in the low bits)
    unsigned* r3 = red + (1 * 2 + par) * NW;   // I_low maxima (local gap)
    unsigned* r2 = red + (2 * 2 + par) * NW;   // step-2 keys
    unsigned* r4 = red + (3 * 2 + par) * NW;   // I_up maxima, unmasked (local gap)
    // Branch-free per-slot work (masks, not conditionals: hipcc turns `valid && …` into exec-mask
    // branches, measured at ~40 % of a pair).  Slots ≥ nws write their own unused mirror entries
    // and compute on zero features; their keys are masked to 0.
    unsigned k1 = 0u, k3 = 0u, k4 = 0u;
    bool low[SL];
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const unsigned s = (unsigned)(tid + TH * m);
      glp[s] = yg[m];
      alp[s] = a[m];
      const float ya = y[m] * a[m];
      const bool up = ya < tu[m];
      low[m] = -ya < tl[m];
      // step 1: i = argmax_{I_up ∩ B} −y·G.  The slot rides in the key's low bits (a ~1e-4
      // relative tie window for the pick); the stopping test uses the unmasked maxima.
      const unsigned um = 0u - (unsigned)up, lm = 0u - (unsigned)low[m];
      const unsigned kv = f32_okey(-yg[m]) & um;
      k4 = max(k4, kv);
      k1 = max(k1, ((kv & ~kIdx) | s) & um);
      k3 = max(k3, f32_okey(yg[m]) & lm);
    }
    k1 = wave_max_u32(k1);
    k3 = wave_max_u32(k3);
    k4 = wave_max_u32(k4);
    if (lane == 0) { r1[wave] = k1; r3[wave] = k3; r4[wave] = k4; }
    WS_STAMP(0)
    __syncthreads();
    const unsigned K1 = __builtin_amdgcn_readfirstlane(red4(r1));
    const unsigned K3 = __builtin_amdgcn_readfirstlane(red4(r3));
    const unsigned K4 = __builtin_amdgcn_readfirstlane(red4(r4));
    if (K1 == 0u || K3 == 0u) return false;
    const int i = (int)(K1 & kIdx);
    const float ygi = glp[i];
    const bool ipos = widx[i] < P.npos;
    const float yi = ipos ? 1.f : -1.f;
    const float Gi = yi * ygi;
    const float GmaxB = -ygi;
    const float lgap = f32_from_okey(K4) + f32_from_okey(K3);
    // (0.9999: the f32 local gap of a problem whose f64 gap is still ≥ eps always takes a pair)
    if (tol_in < 0.f) tol_in = fmaxf(0.9999f * epsf, (float)inner_frac * lgap);
    if (lgap < tol_in) return false;
    // step 2: j = argmax over I_low ∩ B of (GmaxB + yG)² / (2 − 2 K_it)
    WS_STAMP(1)
    float Ki[SL];
    krow(i, Ki);
    unsigned k2 = 0u;
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const unsigned s = (unsigned)(tid + TH * m);
      kip[s] = Ki[m];
      const float gd = GmaxB + yg[m];
      const float q0 = 2.f - 2.f * Ki[m];
      const float quad = q0 <= 0.f ? 1e-12f : q0;
      const unsigned ok = 0u - (unsigned)(low[m] & (gd > 0.f));
      k2 = max(k2, ((f32_okey(gd * gd * __builtin_amdgcn_rcpf(quad)) & ~kIdx) | s) & ok);
    }
    k2 = wave_max_u32(k2);
    if (lane == 0) r2[wave] = k2;
    WS_STAMP(2)
    __syncthreads();
    const unsigned K2 = __builtin_amdgcn_readfirstlane(red4(r2));
    if (K2 == 0u) return false;
    const int j = (int)(K2 & kIdx);
    const float ai_old = alp[i], aj_old = alp[j];
    const float Kij = kip[j];
    const bool jpos = widx[j] < P.npos;
    const float yj = jpos ? 1.f : -1.f;
    const float Gj = yj * glp[j];
    const float Ci = ipos ? Cpf : Cnf, Cj = jpos ? Cpf : Cnf;
    WS_STAMP(3)
    // libsvm's two-variable step and clipping, both label cases evaluated, then selected
    // (Q_ii + Q_jj ∓ 2 Q_ij = 2 − 2 K_ij either way)
    const float q0 = 2.f - 2.f * Kij;
    const float rq = __builtin_amdgcn_rcpf(q0 <= 0.f ? 1e-12f : q0);
    float ao, bo, as, bs;
    {  // y_i ≠ y_j
      const float delta = (-Gi - Gj) * rq;
      const float diff = ai_old - aj_old;
      ao = ai_old + delta;
      bo = aj_old + delta;
      const bool c1 = (diff > 0.f) & (bo < 0.f), c2 = !(diff > 0.f) & (ao < 0.f);
      ao = c1 ? diff : (c2 ? 0.f : ao);
      bo = c1 ? 0.f : (c2 ? -diff : bo);
      const bool c3 = (diff > Ci - Cj) & (ao > Ci), c4 = !(diff > Ci - Cj) & (bo > Cj);
      ao = c3 ? Ci : (c4 ? Cj + diff : ao);
      bo = c3 ? Ci - diff : (c4 ? Cj : bo);
    }
    {  // y_i = y_j
      const float delta = (Gi - Gj) * rq;
      const float sum = ai_old + aj_old;
      as = ai_old - delta;
      bs = aj_old + delta;
      const bool c1 = (sum > Ci) & (as > Ci), c2 = !(sum > Ci) & (bs < 0.f);
      as = c1 ? Ci : (c2 ? sum : as);
      bs = c1 ? sum - Ci : (c2 ? 0.f : bs);
      const bool c3 = (sum > Cj) & (bs > Cj), c4 = !(sum > Cj) & (as < 0.f);
      as = c3 ? sum - Cj : (c4 ? 0.f : as);
      bs = c3 ? Cj : (c4 ? sum : bs);
    }
    const bool opp = ipos != jpos;
    const float ai = opp ? ao : as, aj = opp ? bo : bs;
    const float ci = yi * (ai - ai_old), cj = yj * (aj - aj_old);
    WS_STAMP(4)
    float Kj[SL];
    krow(j, Kj);
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int s = tid + TH * m;
      a[m] = s == i ? ai : (s == j ? aj : a[m]);
      yg[m] += fmaf(Ki[m], ci, Kj[m] * cj);
    }
    WS_STAMP(5)
    ++it;
    return true;
  };
  while (it < max_inner && pair(std::integral_constant<int, 0>{}) && it < max_inner &&
         pair(std::integral_constant<int, 1>{})) {
  }
#undef WS_STAMP
  if (pf && tid == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) prof[(size_t)b * 6 + k] += ph[k];
  }
  // ---- publish: α of B, changed entries (slot order) for the global gradient update
  int nc = 0;
#pragma unroll
  for (int m = 0; m < SL; ++m) {
    const int s = tid + TH * m;
    double anew = a0[m];
    if (valid[m] && a[m] != (float)a0[m]) {
      const double C = pos[m] ? P.Cp : P.Cn;
      anew = a[m] <= 0.f ? 0.0 : (a[m] >= Cw[m] ? C : a0[m] + ((double)a[m] - (double)(float)a0[m]));
    }
    const bool ch = valid[m] && anew != a0[m];
    const unsigned long long cm = __ballot(ch);
    // exclusive prefix over the 4 waves for this m (one barrier pair), then this lane's rank
    __syncthreads();
    if (lane == 0) red[wave] = (unsigned)__popcll(cm);
    __syncthreads();
    int wb = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int v = (int)red[w];
      wb += w < wave ? v : 0;
      tot += v;
    }
    const int cpos = nc + wb + __popcll(cm & lanes_below());
    if (ch) {
      ap[tt[m]] = anew;
      for (int k = 0; k < Fp2; ++k) wsz[((size_t)b * Fp2 + k) * Q + cpos] = k < F ? zB[s * FP + k] : 0.f;
      wsn[(size_t)b * Q + cpos] = sn[m];
      wdc[(size_t)b * Q + cpos] = (float)((double)y[m] * (anew - a0[m]));
    }
    nc += tot;
  }
  const int ncp = (nc + 31) & ~31;
  for (int p = nc + tid; p < ncp; p += TH) {
    for (int k = 0; k < Fp2; ++k) wsz[((size_t)b * Fp2 + k) * Q + p] = 0.f;
    wsn[(size_t)b * Q + p] = 0.f;
    wdc[(size_t)b * Q + p] = 0.f;
  }
  const long long c3 = __builtin_amdgcn_s_memtime();
  const long long r3 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    S->cyc_build += c2 - c1;
    S->cyc_inner += c3 - c2;
    S->cyc_p2 += r3 - r2;   // (the selector's third sub-phase slot is unused: real-time ticks of the inner phase)
    // no pair moved: the f32 selection keys hid an f64 violation below eps-resolution — done
    if (it == 0 || nc == 0) S->done = 1;
    S->nc = nc;
    S->outer += 1;
    S->inner += it;
  }
}

// v[m] for a wave-uniform m, branch-free: the masks are scalar values (the compiler turned the
// ternary form into scalar branches, a fetch bubble each inside the pair loops)
__device__ __forceinline__ unsigned sel4u(const unsigned (&v)[4], int m) {
  const unsigned m0 = 0u - (unsigned)(m == 0), m1 = 0u - (unsigned)(m == 1);
  const unsigned m2 = 0u - (unsigned)(m == 2), m3 = 0u - (unsigned)(m == 3);
  return (v[0] & m0) | (v[1] & m1) | (v[2] & m2) | (v[3] & m3);
}

// ---- ws_kc_round: one whole round with the working set's kernel matrix cached in LDS -------------
// The q = 1024 solver above pays ≈ 4.3k cycles per pair: four waves, two barriers and two dependent
// LDS round trips per pair, and an F-term RBF row recomputed per pick (profiles/r3_headline.md).
// On the bench's problems the pair count barely depends on q (10k points: 8.5k pairs at q = 1024,
// 10.5k at q = 256; scripts/probes/ws_qsim.py), only the round count does (41 → 193).  So this
// variant shrinks the working set to q = 256, whose kernel matrix fits the CU's LDS as an f32 upper
// triangle (256·257/2 words = 128.5 KB), and makes the pair loop ONE wave:
//   1. selection (ws_select_body, all 16 waves; no separate launch, B stays in LDS);
//   2. z_B gathered into LDS ([2·KS][QP] f32, the MFMA operand layout), then K_BB on the f32-input
//      MFMA (36 upper 32×32 tiles over 16 waves) with ws_gupdate's exact expression, so the inner
//      solver and the gradient kernel see the same f32 kernel values bit for bit;
//   3. wave 0 alone runs libsvm's WSS3 pairs: 4 slots per lane in registers, the i / j picks are DPP
//      wave maxima (no barrier, no LDS round trip), a kernel row is 4 LDS reads, no exp;
//   4. wave 0 publishes α of B and the changed coefficients (slot order) for ws_gupdate.
// Same dual, same pair rule, same global f64 stopping rule as ws_solve_kernel.
constexpr int kKcQ = 256;
constexpr int kKcQP = kKcQ + 1;                       // zbuf row stride (conflict-free gather stores)
constexpr int kKcTri = kKcQ * (kKcQ + 1) / 2;         // f32 words of the upper triangle
constexpr size_t kc_zbuf_bytes(int KS) {
  return (size_t)2 * KS * kKcQP * 4 > (4096 + 1024) * 4 ? (size_t)2 * KS * kKcQP * 4 : (4096 + 1024) * 4;
}
// LDS: shi [16] + binfo [16] | widx [Q] | snB [Q] | zbuf (aliases the selector's hist + bm) | tri
constexpr size_t kc_lds_bytes(int KS) { return 128 + 2 * kKcQ * 4 + (kc_zbuf_bytes(KS) + 15) / 16 * 16 + (size_t)kKcTri * 4; }
static_assert(kc_lds_bytes(12) <= 163840, "the K-cached round must fit the CU's 160 KiB of LDS");

__device__ __forceinline__ int kc_rowstart(int r) { return r * kKcQ - ((r * (r - 1)) >> 1); }

__device__ __forceinline__ float sel4(const float (&v)[4], int m) {
  const unsigned u[4] = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  return __uint_as_float(sel4u(u, m));
}
__device__ __forceinline__ int sel4(const int (&v)[4], int m) {
  const unsigned u[4] = {(unsigned)v[0], (unsigned)v[1], (unsigned)v[2], (unsigned)v[3]};
  return (int)sel4u(u, m);
}
__device__ __forceinline__ float rdlane_f(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

// kStamp: in-kernel s_memtime phase totals of the pair loop into prof[b][5] (diagnostic instance,
// HFENS_PROFILE_WS=1; the stamps wait for outstanding LDS reads, so they perturb what they measure)
template <int M, int KS, bool kCand, bool kStamp = false>
__global__ __launch_bounds__(kWsThreads) void ws_kc_round_kernel(
    const WsProb* __restrict__ probs, WsState* __restrict__ states, const float* __restrict__ zcat, int F,
    const float* __restrict__ zn_all, double* __restrict__ alpha_all, const double* __restrict__ G_all,
    int* __restrict__ wsprev, float* __restrict__ wsz, float* __restrict__ wsn, float* __restrict__ wdc,
    int Fp2, double eps, int max_outer, int max_inner, double inner_frac, WsAux X, WsCand C,
    long long* __restrict__ prof = nullptr) {
  constexpr int Q = kKcQ;
  constexpr int SL = Q / 64;            // slots per lane of the solving wave (slot s = 64·m + lane)
  constexpr unsigned kIdx = Q - 1;      // slot bits packed under the selection keys
  static_assert(SL == 4, "sel4 assumes four slots per lane");
  const int b = blockIdx.x;
  WsState* S = states + b;
  if (S->done) return;
  const WsProb P = probs[b];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  extern __shared__ __attribute__((aligned(16))) unsigned char ws_lds[];
  int* shi = reinterpret_cast<int*>(ws_lds);
  int* binfo = shi + 16;
  int* widx = shi + 32;                                                  // [Q]
  float* snB = reinterpret_cast<float*>(widx + Q);                       // [Q]
  float* zbuf = snB + Q;                                                 // [2·KS][QP]
  int* hist = reinterpret_cast<int*>(zbuf);                              // (selector only) [2][2048]
  unsigned* bm = reinterpret_cast<unsigned*>(hist + 4096);               // (selector only) [1024]
  float* tri = zbuf + (kc_zbuf_bytes(KS) + 15) / 16 * 4;                 // [Q(Q+1)/2]
  const int nws = ws_select_body<M, Q, false, kCand>(P, b, S, nullptr, wsprev, eps, max_outer, X, shi, binfo,
                                                     hist, bm, widx, C);
  if (nws < 0) return;
  const long long c1 = __builtin_amdgcn_s_memtime();
  // ---- z_B and γ'‖z‖² into LDS (zero rows past nws / features past F: exact no-ops in the dots)
  for (int e = tid; e < 2 * KS * Q; e += kWsThreads) {
    const int k = e / Q, s = e - k * Q;
    zbuf[k * kKcQP + s] = (s < nws && k < F) ? zcat[(P.zoff + widx[s]) * F + k] : 0.f;
  }
  if (tid < Q) snB[tid] = tid < nws ? P.ngl2e * zn_all[P.aoff + widx[tid]] : 0.f;
  __syncthreads();
  // ---- K_BB upper triangle: tile (ta ≤ tb) of 32×32, ws_gupdate's MFMA chain and epilogue
  {
    const int r32 = lane & 31, hi = lane >> 5;
    const float k2 = -2.f * P.ngl2e;
    for (int t = wave; t < 36; t += kWsWaves) {
      int ta = 0, rem = t;
      while (rem >= 8 - ta) { rem -= 8 - ta; ++ta; }
      const int tb = ta + rem;
      f32x16 A = {0.f};
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        const float* zr = zbuf + (2 * q + hi) * kKcQP;
        A = __builtin_amdgcn_mfma_f32_32x32x2f32(zr[ta * 32 + r32], zr[tb * 32 + r32], A, 0, 0, 0);
      }
      const int col = tb * 32 + r32;
      const float snc = snB[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = ta * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
        const float kv = __builtin_amdgcn_exp2f(fminf(fmaf(k2, A[r], snB[row] + snc), 0.f));
        if (row <= col) tri[kc_rowstart(row) + col - row] = kv;
      }
    }
  }
  __syncthreads();
  const long long c2 = __builtin_amdgcn_s_memtime();
  if (wave != 0) return;
  // ---- the pair loop: wave 0 alone
  const double* Gp = G_all + P.aoff;
  double* ap = alpha_all + P.aoff;
  bool valid[SL], pos[SL];
  int tt[SL], rb[SL];
  // yg = y·G and the y·α < tu / −y·α < tl membership tests: see ws_solve_kernel
  float y[SL], Cw[SL], a[SL], yg[SL], tu[SL], tl[SL];
  double a0[SL];
#pragma unroll
  for (int m = 0; m < SL; ++m) {
    const int s = 64 * m + lane;
    valid[m] = s < nws;
    tt[m] = valid[m] ? widx[s] : 0;
    pos[m] = tt[m] < P.npos;
    y[m] = pos[m] ? 1.f : -1.f;
    Cw[m] = (float)(pos[m] ? P.Cp : P.Cn);
    tu[m] = valid[m] ? (pos[m] ? Cw[m] : 0.f) : -INFINITY;
    tl[m] = valid[m] ? (pos[m] ? 0.f : Cw[m]) : -INFINITY;
    a0[m] = valid[m] ? ap[tt[m]] : 0.0;
    a[m] = (float)a0[m];
    yg[m] = valid[m] ? y[m] * (float)Gp[tt[m]] : 0.f;
    rb[m] = kc_rowstart(s) - s;   // K(r, s) for r > s lives at rowstart(s) + r − s
  }
  // K(r, ·) for this lane's slots (r wave-uniform): upper-triangle address of (min, max)
  auto krow = [&](int r, float (&out)[SL]) {
    const int ra = kc_rowstart(r) - r;
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int s = 64 * m + lane;
      out[m] = tri[s >= r ? ra + s : rb[m] + r];
    }
  };
  const float Cpf = (float)P.Cp, Cnf = (float)P.Cn;
  const float epsf = (float)eps;
  float tol_in = -1.f;
  int it = 0;
  long long ph[5] = {0, 0, 0, 0, 0};
  long long tp = kStamp ? (long long)__builtin_amdgcn_s_memtime() : 0;
  auto stamp = [&](int k) {
    if constexpr (kStamp) {
      const long long tn = __builtin_amdgcn_s_memtime();
      ph[k] += tn - tp;
      tp = tn;
    }
  };
  while (it < max_inner) {
    // step 1: i = argmax_{I_up ∩ B} −y·G (slot in the key's low bits); I_low maximum for the gap
    unsigned k1 = 0u, k3 = 0u;
    bool low[SL];
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const unsigned s = (unsigned)(64 * m + lane);
      const float ya = y[m] * a[m];
      const bool up = ya < tu[m];
      low[m] = -ya < tl[m];
      const unsigned um = 0u - (unsigned)up, lm = 0u - (unsigned)low[m];
      k1 = max(k1, ((f32_okey(-yg[m]) & ~kIdx) | s) & um);
      k3 = max(k3, f32_okey(yg[m]) & lm);
    }
    const unsigned K1 = __builtin_amdgcn_readfirstlane(wave_max_u32(k1));
    const unsigned K3 = __builtin_amdgcn_readfirstlane(wave_max_u32(k3));
    stamp(0);
    if (K1 == 0u || K3 == 0u) break;
    const int i = (int)(K1 & kIdx), mi = i >> 6, li = i & 63;
    const float ygi = rdlane_f(sel4(yg, mi), li);
    const float ai_old = rdlane_f(sel4(a, mi), li);
    const bool ipos = __builtin_amdgcn_readlane(sel4(tt, mi), li) < P.npos;
    const float yi = ipos ? 1.f : -1.f;
    const float Gi = yi * ygi;
    const float GmaxB = -ygi;
    const float lgap = GmaxB + f32_from_okey(K3);
    if (tol_in < 0.f) tol_in = fmaxf(0.9999f * epsf, (float)inner_frac * lgap);
    if (lgap < tol_in) break;
    // step 2: j = argmax over I_low ∩ B of (GmaxB + yG)² / (2 − 2 K_it)
    float Ki[SL];
    krow(i, Ki);
    stamp(1);
    unsigned k2 = 0u;
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const unsigned s = (unsigned)(64 * m + lane);
      const float gd = GmaxB + yg[m];
      const float q0 = 2.f - 2.f * Ki[m];
      const float quad = q0 <= 0.f ? 1e-12f : q0;
      const unsigned ok = 0u - (unsigned)(low[m] & (gd > 0.f));
      k2 = max(k2, ((f32_okey(gd * gd * __builtin_amdgcn_rcpf(quad)) & ~kIdx) | s) & ok);
    }
    const unsigned K2 = __builtin_amdgcn_readfirstlane(wave_max_u32(k2));
    stamp(2);
    if (K2 == 0u) break;
    const int j = (int)(K2 & kIdx), mj = j >> 6, lj = j & 63;
    float Kj[SL];
    krow(j, Kj);   // issued before the scalar step below: its LDS latency hides under it
    const float ygj = rdlane_f(sel4(yg, mj), lj);
    const float aj_old = rdlane_f(sel4(a, mj), lj);
    const float Kij = rdlane_f(sel4(Ki, mj), lj);
    const bool jpos = __builtin_amdgcn_readlane(sel4(tt, mj), lj) < P.npos;
    const float yj = jpos ? 1.f : -1.f;
    const float Gj = yj * ygj;
    const float Ci = ipos ? Cpf : Cnf, Cj = jpos ? Cpf : Cnf;
    // libsvm's two-variable step and clipping (ws_solve_kernel's branch-free form)
    const float q0 = 2.f - 2.f * Kij;
    const float rq = __builtin_amdgcn_rcpf(q0 <= 0.f ? 1e-12f : q0);
    float ao, bo, as, bs;
    {  // y_i ≠ y_j
      const float delta = (-Gi - Gj) * rq;
      const float diff = ai_old - aj_old;
      ao = ai_old + delta;
      bo = aj_old + delta;
      const bool c1 = (diff > 0.f) & (bo < 0.f), c2 = !(diff > 0.f) & (ao < 0.f);
      ao = c1 ? diff : (c2 ? 0.f : ao);
      bo = c1 ? 0.f : (c2 ? -diff : bo);
      const bool c3 = (diff > Ci - Cj) & (ao > Ci), c4 = !(diff > Ci - Cj) & (bo > Cj);
      ao = c3 ? Ci : (c4 ? Cj + diff : ao);
      bo = c3 ? Ci - diff : (c4 ? Cj : bo);
    }
    {  // y_i = y_j
      const float delta = (Gi - Gj) * rq;
      const float sum = ai_old + aj_old;
      as = ai_old - delta;
      bs = aj_old + delta;
      const bool c1 = (sum > Ci) & (as > Ci), c2 = !(sum > Ci) & (bs < 0.f);
      as = c1 ? Ci : (c2 ? sum : as);
      bs = c1 ? sum - Ci : (c2 ? 0.f : bs);
      const bool c3 = (sum > Cj) & (bs > Cj), c4 = !(sum > Cj) & (as < 0.f);
      as = c3 ? sum - Cj : (c4 ? 0.f : as);
      bs = c3 ? Cj : (c4 ? sum : bs);
    }
    const bool opp = ipos != jpos;
    const float ai = opp ? ao : as, aj = opp ? bo : bs;
    const float ci = yi * (ai - ai_old), cj = yj * (aj - aj_old);
    stamp(3);
#pragma unroll
    for (int m = 0; m < SL; ++m) {
      const int s = 64 * m + lane;
      a[m] = s == i ? ai : (s == j ? aj : a[m]);
      yg[m] += fmaf(Ki[m], ci, Kj[m] * cj);
    }
    stamp(4);
    ++it;
  }
  if constexpr (kStamp) {
    if (lane == 0)
      for (int k = 0; k < 5; ++k) prof[(size_t)b * 6 + k] += ph[k];
  }
  // ---- publish: α of B, changed entries (slot order) for the global gradient update
  int nc = 0;
#pragma unroll
  for (int m = 0; m < SL; ++m) {
    const int s = 64 * m + lane;
    double anew = a0[m];
    if (valid[m] && a[m] != (float)a0[m]) {
      const double C = pos[m] ? P.Cp : P.Cn;
      anew = a[m] <= 0.f ? 0.0 : (a[m] >= Cw[m] ? C : a0[m] + ((double)a[m] - (double)(float)a0[m]));
    }
    const bool ch = valid[m] && anew != a0[m];
    const unsigned long long cm = __ballot(ch);
    const int cpos = nc + __popcll(cm & lanes_below());
    if (ch) {
      ap[tt[m]] = anew;
      for (int k = 0; k < Fp2; ++k) wsz[((size_t)b * Fp2 + k) * Q + cpos] = zbuf[k * kKcQP + s];
      wsn[(size_t)b * Q + cpos] = snB[s];
      wdc[(size_t)b * Q + cpos] = (float)((double)y[m] * (anew - a0[m]));
    }
    nc += __popcll(cm);
  }
  const int ncp = (nc + 31) & ~31;
  for (int p = nc + lane; p < ncp; p += 64) {
    for (int k = 0; k < Fp2; ++k) wsz[((size_t)b * Fp2 + k) * Q + p] = 0.f;
    wsn[(size_t)b * Q + p] = 0.f;
    wdc[(size_t)b * Q + p] = 0.f;
  }
  const long long c3 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    S->cyc_build += c2 - c1;
    S->cyc_inner += c3 - c2;
    if (it == 0 || nc == 0) S->done = 1;
    S->nc = nc;
    S->outer += 1;
    S->inner += it;
  }
}

// G_t += y_t · Σ_c dc_c · exp2(γ'‖x_t − x_c‖²) for every point t of every active problem, then t's
// selection keys for the next working set.  The changed coefficients are staged through LDS in
// chunks of kWsChunk; every wave takes part in every barrier (waves past the end compute nothing).
template <int KS>
__global__ __launch_bounds__(256) void ws_gupdate_kernel(const WsProb* __restrict__ probs,
                                                         const WsState* __restrict__ states,
                                                         const float* __restrict__ zcat, int F,
                                                         const float* __restrict__ zn_all,
                                                         const double* __restrict__ alpha_all,
                                                         double* __restrict__ G_all,
                                                         const float* __restrict__ wsz,
                                                         const float* __restrict__ wsn,
                                                         const float* __restrict__ wdc, int Fp2, int Q, WsAux X) {
  const int b = blockIdx.y;
  const int nc = states[b].nc;
  if (nc == 0) return;
  const WsProb P = probs[b];
  const int row_blk = blockIdx.x * 256;
  if (row_blk >= P.l) return;
  const int ncp = (nc + 31) & ~31;
  __shared__ __attribute__((aligned(16))) float sv_l[2 * KS * kWsChunk];
  __shared__ __attribute__((aligned(16))) float sn_l[kWsChunk];
  __shared__ __attribute__((aligned(16))) float cf_l[kWsChunk];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r32 = lane & 31, hi = lane >> 5;
  const int r0 = row_blk + wave * 64;
  const int row = r0 + lane;
  const bool valid = row < P.l;
  const bool live = r0 < P.l;   // wave-uniform
  // this lane's G/α loads first: their latency hides under the MFMA work
  const double gold = valid ? G_all[P.aoff + row] : 0.0;
  const double a = valid ? alpha_all[P.aoff + row] : 0.0;
  const int ra = r0 + r32, rb = r0 + 32 + r32;
  float za[KS], zb[KS];
  const float* zA = zcat + (P.zoff + ra) * F;
  const float* zBp = zcat + (P.zoff + rb) * F;
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const int k = 2 * q + hi;
    za[q] = (k < F && ra < P.l) ? zA[k] : 0.f;
    zb[q] = (k < F && rb < P.l) ? zBp[k] : 0.f;
  }
  const float zsa = ra < P.l ? P.ngl2e * zn_all[P.aoff + ra] : 0.f;
  const float zsb = rb < P.l ? P.ngl2e * zn_all[P.aoff + rb] : 0.f;
  const float k2 = -2.f * P.ngl2e;
  float pa = 0.f, pb = 0.f;
  for (int c0 = 0; c0 < ncp; c0 += kWsChunk) {
    const int cn = min(kWsChunk, ncp - c0);
    __syncthreads();   // the previous chunk is consumed
    for (int i = threadIdx.x; i < 2 * KS * cn; i += blockDim.x) {
      const int k = i / cn, c = i - k * cn;
      sv_l[k * kWsChunk + c] = k < Fp2 ? wsz[((size_t)b * Fp2 + k) * Q + c0 + c] : 0.f;
    }
    for (int c = threadIdx.x; c < cn; c += blockDim.x) {
      sn_l[c] = wsn[(size_t)b * Q + c0 + c];
      cf_l[c] = wdc[(size_t)b * Q + c0 + c];
    }
    __syncthreads();
    if (!live) continue;
    for (int t = 0; t < cn; t += 32) {
      f32x16 A = {0.f}, B = {0.f};
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        const float sv = sv_l[(2 * q + hi) * kWsChunk + t + r32];
        A = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, za[q], A, 0, 0, 0);
        B = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, zb[q], B, 0, 0, 0);
      }
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int cc = t + 8 * gq + 4 * hi;
        const f32x4 snv = *reinterpret_cast<const f32x4*>(&sn_l[cc]);
        const f32x4 cfv = *reinterpret_cast<const f32x4*>(&cf_l[cc]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pa = fmaf(cfv[q], __builtin_amdgcn_exp2f(fminf(fmaf(k2, A[4 * gq + q], snv[q] + zsa), 0.f)), pa);
          pb = fmaf(cfv[q], __builtin_amdgcn_exp2f(fminf(fmaf(k2, B[4 * gq + q], snv[q] + zsb), 0.f)), pb);
        }
      }
    }
  }
  if (!live) return;
  pa += __shfl_xor(pa, 32, kWave);
  pb += __shfl_xor(pb, 32, kWave);
  double gnew = 0.0;
  if (valid) {
    const double upd = (double)(lane < 32 ? pa : pb);
    gnew = gold + (row < P.npos ? upd : -upd);
    G_all[P.aoff + row] = gnew;
  }
  ws_publish_keys(P, b, row, valid, a, gnew, X);
}

// Warm start (cascade seed, models/smo.py _cascade_seed): α = aseed (a feasible point: the
// concatenated solutions of disjoint sub-problems with the same C) and G_t = −1 + y_t Σ_c y_c α_c K_tc
// over the nonzero α_c, then t's selection keys.  Every workgroup walks the problem's points in
// chunks of kWsChunk, compacts the nonzero coefficients into LDS (ballot + per-wave prefix) and
// runs ws_gupdate's MFMA + exp2 tile on them; each chunk's f32 partial joins an f64 accumulator
// (≤ 256 terms per f32 sum, as in a gradient update round).  gkey must be zero on entry.
template <int KS>
__global__ __launch_bounds__(256) void ws_seed_kernel(const WsProb* __restrict__ probs,
                                                      const float* __restrict__ zcat, int F,
                                                      const float* __restrict__ zn_all,
                                                      const double* __restrict__ aseed,
                                                      double* __restrict__ alpha_all,
                                                      double* __restrict__ G_all, WsAux X,
                                                      double* __restrict__ part, int max_l, int cols_per_split) {
  const int b = blockIdx.y;
  const WsProb P = probs[b];
  const int row_blk = blockIdx.x * 256;
  if (row_blk >= P.l) return;
  // split-K over the columns (gridDim.z > 1): this workgroup's column range, partial sums to part
  const int c_begin = blockIdx.z * cols_per_split;
  const int c_end = min(P.l, c_begin + cols_per_split);
  if (gridDim.z > 1 && c_begin >= P.l) {
    const int row = row_blk + threadIdx.x;
    if (row < P.l) part[((size_t)blockIdx.z * gridDim.y + b) * max_l + row] = 0.0;
    return;
  }
  __shared__ __attribute__((aligned(16))) float sv_l[2 * KS * kWsChunk];
  __shared__ __attribute__((aligned(16))) float sn_l[kWsChunk];
  __shared__ __attribute__((aligned(16))) float cf_l[kWsChunk];
  __shared__ int wcnt[4];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hi = lane >> 5;
  const int r0 = row_blk + wave * 64;
  const int row = r0 + lane;
  const bool valid = row < P.l;
  const bool live = r0 < P.l;   // wave-uniform
  const double a = valid ? aseed[P.aoff + row] : 0.0;
  const int ra = r0 + r32, rb = r0 + 32 + r32;
  float za[KS], zb[KS];
  const float* zA = zcat + (P.zoff + ra) * F;
  const float* zBp = zcat + (P.zoff + rb) * F;
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const int k = 2 * q + hi;
    za[q] = (k < F && ra < P.l) ? zA[k] : 0.f;
    zb[q] = (k < F && rb < P.l) ? zBp[k] : 0.f;
  }
  const float zsa = ra < P.l ? P.ngl2e * zn_all[P.aoff + ra] : 0.f;
  const float zsb = rb < P.l ? P.ngl2e * zn_all[P.aoff + rb] : 0.f;
  const float k2 = -2.f * P.ngl2e;
  double da = 0.0, db = 0.0;
  for (int c0 = c_begin; c0 < c_end; c0 += kWsChunk) {
    const int c = c0 + tid;
    const double ac = c < c_end ? aseed[P.aoff + c] : 0.0;
    const bool nz = ac > 0.0;
    const unsigned long long m = __ballot(nz);
    __syncthreads();   // the previous chunk is consumed
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int base = 0, cnt = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int v = wcnt[w];
      base += w < wave ? v : 0;
      cnt += v;
    }
    if (cnt == 0) continue;   // block-uniform
    const int ncp = (cnt + 31) & ~31;
    if (nz) {
      const int pos = base + __popcll(m & lanes_below());
      const float* zc = zcat + (P.zoff + c) * F;
#pragma unroll
      for (int k = 0; k < 2 * KS; ++k) sv_l[k * kWsChunk + pos] = k < F ? zc[k] : 0.f;
      sn_l[pos] = P.ngl2e * zn_all[P.aoff + c];
      cf_l[pos] = (float)(c < P.npos ? ac : -ac);
    }
    for (int p = cnt + tid; p < ncp; p += 256) {
#pragma unroll
      for (int k = 0; k < 2 * KS; ++k) sv_l[k * kWsChunk + p] = 0.f;
      sn_l[p] = 0.f;
      cf_l[p] = 0.f;
    }
    __syncthreads();
    if (!live) continue;
    float pa = 0.f, pb = 0.f;
    for (int t = 0; t < ncp; t += 32) {
      f32x16 A = {0.f}, B = {0.f};
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        const float sv = sv_l[(2 * q + hi) * kWsChunk + t + r32];
        A = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, za[q], A, 0, 0, 0);
        B = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, zb[q], B, 0, 0, 0);
      }
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int cc = t + 8 * gq + 4 * hi;
        const f32x4 snv = *reinterpret_cast<const f32x4*>(&sn_l[cc]);
        const f32x4 cfv = *reinterpret_cast<const f32x4*>(&cf_l[cc]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pa = fmaf(cfv[q], __builtin_amdgcn_exp2f(fminf(fmaf(k2, A[4 * gq + q], snv[q] + zsa), 0.f)), pa);
          pb = fmaf(cfv[q], __builtin_amdgcn_exp2f(fminf(fmaf(k2, B[4 * gq + q], snv[q] + zsb), 0.f)), pb);
        }
      }
    }
    da += (double)pa;
    db += (double)pb;
  }
  if (!live) return;
  da += __shfl_xor(da, 32, kWave);
  db += __shfl_xor(db, 32, kWave);
  if (gridDim.z > 1) {
    if (valid) part[((size_t)blockIdx.z * gridDim.y + b) * max_l + row] = lane < 32 ? da : db;
    return;
  }
  double g = -1.0;
  if (valid) {
    const double upd = lane < 32 ? da : db;
    g = -1.0 + (row < P.npos ? upd : -upd);
    alpha_all[P.aoff + row] = a;
    G_all[P.aoff + row] = g;
  }
  ws_publish_keys(P, b, row, valid, a, g, X);
}

// the split-K seed's partial sums in split order (deterministic), then α, G and the keys
__global__ __launch_bounds__(256) void ws_seed_fin_kernel(const WsProb* __restrict__ probs,
                                                          const double* __restrict__ aseed,
                                                          double* __restrict__ alpha_all, double* __restrict__ G_all,
                                                          WsAux X, const double* __restrict__ part, int max_l, int S) {
  const int b = blockIdx.y;
  const WsProb P = probs[b];
  if ((int)blockIdx.x * 256 >= P.l) return;
  const int row = blockIdx.x * 256 + threadIdx.x;
  const bool valid = row < P.l;
  double g = -1.0, a = 0.0;
  if (valid) {
    double upd = 0.0;
    for (int s = 0; s < S; ++s) upd += part[((size_t)s * gridDim.y + b) * max_l + row];
    a = aseed[P.aoff + row];
    g = -1.0 + (row < P.npos ? upd : -upd);
    alpha_all[P.aoff + row] = a;
    G_all[P.aoff + row] = g;
  }
  ws_publish_keys(P, b, row, valid, a, g, X);
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
static int ws_ks(int F) {
  const int ks = (F + 1) / 2;
  return ks <= 4 ? 4 : ks <= 9 ? 9 : ks <= 12 ? 12 : 24;
}

// Working-set size for F features: 1024 slots while z_B fits (F ≤ 24), else 512 (F ≤ 48).
static int ws_q(int F) { return F <= 24 ? 1024 : 512; }

static WsAux ws_aux(uintptr_t keys, long long n, uintptr_t gkey) {
  return WsAux{(unsigned*)keys, n, (unsigned long long*)gkey};
}

void ws_init(uintptr_t probs, int P, int max_l, uintptr_t zcat, int F, uintptr_t zn, uintptr_t alpha,
             uintptr_t G, uintptr_t states, uintptr_t keys, long long n, uintptr_t hist, uintptr_t gkey,
             uintptr_t stream) {
  (void)hist;
  HFENS_REQUIRE(F >= 1 && F <= 48, "ws_init: 1 <= F <= 48");
  if (P == 0 || max_l == 0) return;
  hipLaunchKernelGGL(ws_init_kernel, dim3((max_l + 255) / 256, P), dim3(256), 0, as_stream(stream),
                     (const WsProb*)probs, (const float*)zcat, F, (float*)zn, (double*)alpha, (double*)G,
                     (WsState*)states, ws_aux(keys, n, gkey));
  launch_check();
}

// After ws_init: α ← aseed (per point, the problems' layout) and G, keys from it (ws_seed_kernel).
void ws_seed(uintptr_t probs, int P, int max_l, uintptr_t zcat, int F, uintptr_t zn, uintptr_t aseed,
             uintptr_t alpha, uintptr_t G, uintptr_t keys, long long n, uintptr_t gkey, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 48, "ws_seed: 1 <= F <= 48");
  if (P == 0 || max_l == 0) return;
  hipStream_t st = as_stream(stream);
  // ws_init folded the α = 0 maxima into gkey: the seeded point's replace them
  HFENS_CHECK(hipMemsetAsync(reinterpret_cast<void*>(gkey), 0, sizeof(unsigned long long) * 2 * (size_t)P, st));
  const int rb = (max_l + 255) / 256;
  const WsAux X = ws_aux(keys, n, gkey);
  // split-K over the columns when the row blocks alone leave the chip idle (the stacking fit's
  // 10k-point final problem: 40 workgroups; its seed sat on the critical path for ≈ 0.3 ms):
  // ≈ 2048 workgroups, whole 256-column chunks per split, partials summed in split order
  const int nchunk = (max_l + kWsChunk - 1) / kWsChunk;
  int S = (2048 + rb * P - 1) / (rb * P);
  if (S > nchunk) S = nchunk;
  if (S < 1) S = 1;
  const int cps = (nchunk + S - 1) / S * kWsChunk;
  S = (max_l + cps - 1) / cps;
  double* part = nullptr;
  if (S > 1) HFENS_CHECK(hipMallocAsync(reinterpret_cast<void**>(&part), sizeof(double) * (size_t)S * P * max_l, st));
  const dim3 grid(rb, P, S);
#define WS_SEED(K)                                                                                   \
  case K:                                                                                           \
    hipLaunchKernelGGL(ws_seed_kernel<K>, grid, dim3(256), 0, st, (const WsProb*)probs, (const float*)zcat, F, \
                       (const float*)zn, (const double*)aseed, (double*)alpha, (double*)G, X, part, max_l, cps); \
    break;
  switch (ws_ks(F)) { WS_SEED(4) WS_SEED(9) WS_SEED(12) WS_SEED(24) }
#undef WS_SEED
  launch_check();
  if (S > 1) {
    hipLaunchKernelGGL(ws_seed_fin_kernel, dim3(rb, P), dim3(256), 0, st, (const WsProb*)probs, (const double*)aseed,
                       (double*)alpha, (double*)G, X, (const double*)part, max_l, S);
    launch_check();
    HFENS_CHECK(hipFreeAsync(part, st));
  }
}

// n_iter outer iterations (select+solve, then the gradient update) enqueued back to back; finished
// problems return at once.  wsz/wsn/wdc hold [P][2·KS][q] / [P][q] / [P][q]; wsprev [P][q/2];
// wsidx [P][q].
void ws_steps(uintptr_t probs, int P, int max_l, uintptr_t zcat, int F, uintptr_t zn, uintptr_t alpha,
              uintptr_t G, uintptr_t states, uintptr_t wsz, uintptr_t wsn, uintptr_t wdc, uintptr_t wsprev,
              uintptr_t wsidx, uintptr_t keys, long long n, uintptr_t gkey, double eps, int max_outer, int max_inner,
              double inner_frac, int n_iter, uintptr_t prof, int inner_threads, int q, uintptr_t stream) {
  const WsAux X = ws_aux(keys, n, gkey);
  HFENS_REQUIRE(F >= 1 && F <= 48, "ws_steps: 1 <= F <= 48");
  // (< 32768: the packed 16|16-bit member counts of the radix selector)
  HFENS_REQUIRE(max_l < 32 * kWsThreads, "ws_steps: problems of 32768+ points need the multi-workgroup selector");
  if (P == 0 || max_l == 0) return;
  hipStream_t st = as_stream(stream);
  const int KS = ws_ks(F);
  const int Fp2 = 2 * KS;
  // q: 0 = the default for F; 512 for F ≤ 24 is the smaller working set (half the per-pair slots)
  const int Q = q == 0 ? ws_q(F) : q;
  HFENS_REQUIRE(Q == 512 || (Q == 1024 && F <= 24), "ws_steps: q is 512, or 1024 for F <= 24");
  const int FP = F <= 24 ? (F + 3) / 4 * 4 : (F + 7) / 8 * 8;
  auto pp = (const WsProb*)probs;
  auto sp = (WsState*)states;
  auto zp = (const float*)zcat;
  auto np_ = (const float*)zn;
  auto ap = (double*)alpha;
  auto gp = (double*)G;
  auto wz = (float*)wsz;
  auto wn = (float*)wsn;
  auto wd = (float*)wdc;
  auto wp = (int*)wsprev;
  const int M = max_l <= 4 * kWsThreads ? 4 : max_l <= 16 * kWsThreads ? 16 : 32;
  int* wi = (int*)wsidx;
  const int TH = inner_threads == 512 ? 512 : 256;
  for (int it = 0; it < n_iter; ++it) {
#define WS_SEL(MM, QQ)                                                                                  \
  if (M == MM && Q == QQ) {                                                                             \
    hipLaunchKernelGGL((ws_select_kernel<MM, QQ>), dim3(P), dim3(kWsThreads), ws_sel_lds_bytes(QQ), st,  \
                       pp, sp, wi, wp, eps, max_outer, X);                                              \
  } else
    WS_SEL(4, 1024) WS_SEL(16, 1024) WS_SEL(32, 1024) WS_SEL(4, 512) WS_SEL(16, 512) WS_SEL(32, 512) {}
#undef WS_SEL
    launch_check();
#define WS_SOL_TH(FF, QQ, TT)                                                                           \
  hipLaunchKernelGGL((ws_solve_kernel<FF, QQ, TT>), dim3(P), dim3(TT), ws_solve_lds_bytes(QQ, FF), st, pp, sp, \
                     zp, F, np_, ap, gp, wi, wz, wn, wd, Fp2, eps, max_inner, inner_frac, (long long*)prof)
#define WS_SOL(FF)                                                                                      \
  if (FP == FF && Q == 1024) {                                                                          \
    if (TH == 512) WS_SOL_TH(FF, 1024, 512);                                                            \
    else WS_SOL_TH(FF, 1024, 256);                                                                      \
  } else
#define WS_SOL512(FF)                                                                                   \
  if (FP == FF && Q == 512) {                                                                           \
    WS_SOL_TH(FF, 512, 256);                                                                            \
  } else
    WS_SOL(4) WS_SOL(8) WS_SOL(12) WS_SOL(16) WS_SOL(20) WS_SOL(24)
    WS_SOL512(4) WS_SOL512(8) WS_SOL512(12) WS_SOL512(16) WS_SOL512(20) WS_SOL512(24)
    WS_SOL512(32) WS_SOL512(40) WS_SOL512(48) {
      HFENS_REQUIRE(false, "ws_steps: no solve instance for this F");
    }
#undef WS_SOL512
#undef WS_SOL_TH
#undef WS_SOL
    launch_check();
    const dim3 grid((max_l + 255) / 256, P);
#define WS_UPD(K)                                                                                    \
  case K:                                                                                           \
    hipLaunchKernelGGL(ws_gupdate_kernel<K>, grid, dim3(256), 0, st, pp, sp, zp, F, np_, ap, gp, wz, \
                       wn, wd, Fp2, Q, X);                                                          \
    break;
    switch (KS) { WS_UPD(4) WS_UPD(9) WS_UPD(12) WS_UPD(24) }
#undef WS_UPD
    launch_check();
  }
}

// n_iter K-cached rounds (ws_kc_round + ws_gupdate) enqueued back to back; q = kKcQ, F ≤ 24.
// wsz/wsn/wdc hold [P][2·KS][256] / [P][256] / [P][256]; wsprev [P][128].
// Selection mode: problems of ≤ kWsDirectMax points are selected from every point's keys by the
// round kernel itself; larger ones first get per-block candidate lists (ws_cand_kernel, one more
// launch per round) and the round kernel selects among those.  cand: [3][P][ncand] u32 workspace,
// ncand = ws_kc_ncand(max_l) (0 below the threshold).
constexpr int kWsDirectMax = 16 * kWsThreads;
long long ws_kc_ncand(long long max_l) {
  return max_l <= kWsDirectMax ? 0 : (max_l + kWsCandBlk - 1) / kWsCandBlk * (kKcQ / 2);
}

void ws_kc_cand_len(long long max_l, uintptr_t out) { *reinterpret_cast<long long*>(out) = ws_kc_ncand(max_l); }

void ws_steps_kc(uintptr_t probs, int P, int max_l, uintptr_t zcat, int F, uintptr_t zn, uintptr_t alpha,
                 uintptr_t G, uintptr_t states, uintptr_t wsz, uintptr_t wsn, uintptr_t wdc, uintptr_t wsprev,
                 uintptr_t keys, long long n, uintptr_t gkey, uintptr_t cand, double eps, int max_outer,
                 int max_inner, double inner_frac, int n_iter, uintptr_t prof, uintptr_t stream) {
  const WsAux X = ws_aux(keys, n, gkey);
  HFENS_REQUIRE(F >= 1 && F <= 24, "ws_steps_kc: 1 <= F <= 24");
  const long long ncand = ws_kc_ncand(max_l);
  HFENS_REQUIRE(ncand <= 32LL * kWsThreads, "ws_steps_kc: at most 2^21 points per problem");
  HFENS_REQUIRE(ncand == 0 || cand != 0, "ws_steps_kc: the candidate workspace is missing");
  if (P == 0 || max_l == 0) return;
  hipStream_t st = as_stream(stream);
  const int KS = ws_ks(F);
  const int Fp2 = 2 * KS;
  const long long L = ncand ? ncand : max_l;   // keys the round kernel's selector reads per problem
  const int M = L <= 4 * kWsThreads ? 4 : L <= 16 * kWsThreads ? 16 : 32;
  WsCand C{nullptr, nullptr, nullptr, (int)ncand};
  if (ncand) {
    C.idx = reinterpret_cast<int*>(cand);
    C.ku = reinterpret_cast<unsigned*>(cand) + (size_t)P * ncand;
    C.kl = reinterpret_cast<unsigned*>(cand) + 2 * (size_t)P * ncand;
  }
  const dim3 cgrid((max_l + kWsCandBlk - 1) / kWsCandBlk, P);
  auto pp = (const WsProb*)probs;
  auto sp = (WsState*)states;
  auto zp = (const float*)zcat;
  auto np_ = (const float*)zn;
  auto ap = (double*)alpha;
  auto gp = (double*)G;
  auto wz = (float*)wsz;
  auto wn = (float*)wsn;
  auto wd = (float*)wdc;
  auto wp = (int*)wsprev;
  const dim3 grid((max_l + 255) / 256, P);
  for (int it = 0; it < n_iter; ++it) {
    if (ncand) {
      hipLaunchKernelGGL((ws_cand_kernel<kKcQ>), cgrid, dim3(kWsThreads), 0, st, pp, sp, X, C);
      launch_check();
    }
    if (prof && M == 16 && KS == 9 && ncand == 0) {   // diagnostic instance (the bench's shape)
      hipLaunchKernelGGL((ws_kc_round_kernel<16, 9, false, true>), dim3(P), dim3(kWsThreads), kc_lds_bytes(9), st,
                         pp, sp, zp, F, np_, ap, gp, wp, wz, wn, wd, Fp2, eps, max_outer, max_inner, inner_frac, X, C,
                         (long long*)prof);
    } else
#define KC_ROUND(MM, KK, CC)                                                                                     \
  if (M == MM && KS == KK && (ncand != 0) == CC) {                                                               \
    hipLaunchKernelGGL((ws_kc_round_kernel<MM, KK, CC>), dim3(P), dim3(kWsThreads), kc_lds_bytes(KK), st, pp, sp, \
                       zp, F, np_, ap, gp, wp, wz, wn, wd, Fp2, eps, max_outer, max_inner, inner_frac, X, C);    \
  } else
    KC_ROUND(4, 4, false) KC_ROUND(4, 9, false) KC_ROUND(4, 12, false) KC_ROUND(16, 4, false)
    KC_ROUND(16, 9, false) KC_ROUND(16, 12, false)
    KC_ROUND(4, 9, true) KC_ROUND(16, 9, true) KC_ROUND(32, 9, true) KC_ROUND(4, 4, true) KC_ROUND(16, 4, true)
    KC_ROUND(32, 4, true) KC_ROUND(4, 12, true) KC_ROUND(16, 12, true) KC_ROUND(32, 12, true) {
      HFENS_REQUIRE(false, "ws_steps_kc: no round instance for this F / size");
    }
#undef KC_ROUND
    launch_check();
#define WS_UPD(K)                                                                                    \
  case K:                                                                                           \
    hipLaunchKernelGGL(ws_gupdate_kernel<K>, grid, dim3(256), 0, st, pp, sp, zp, F, np_, ap, gp, wz, \
                       wn, wd, Fp2, kKcQ, X);                                                       \
    break;
    switch (KS) { WS_UPD(4) WS_UPD(9) WS_UPD(12) }
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
