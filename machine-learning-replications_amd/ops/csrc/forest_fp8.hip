// Tree-ensemble inference as an fp8 leaf-value GEMV on the CDNA4 matrix cores (BASELINE config 5:
// "deep ensemble (1000 trees × 5 seeds), fp8 leaf values on CDNA4 MFMA").
//
// For binned rows the prediction of S models is a product
//     raw[n × S] = Onehot[n × K] · V[K × S],   K = T · 2^d leaf slots (tree t, leaf v at t·2^d + v)
// where Onehot has exactly one 1 per tree and row (the leaf the row reaches) and V holds the
// learning-rate-scaled leaf values.  Here V is stored in OCP fp8 e4m3 as a TWO-TERM split
// (hi = fp8(σ_s·v), lo = fp8(σ_s·v − hi), σ_s a power of two per model placing the largest
// value near the top of the e4m3 range), so the 16 B-columns carry [hi_0..hi_{S−1} | lo_0..lo_{S−1}]
// and the split costs nothing: the MFMA's N = 16 is there anyway.  Products 1·fp8 are exact and
// accumulate in f32; the end result is ≈ 2^-8-relative per leaf value (fp8 alone: 2^-4).
//
// One wave computes 16 rows × all K with gfx950's block-scaled v_mfma_scale_f32_16x16x128_f8f6f4
// (e4m3 operands, unit E8M0 scales): per 128-slot K step, lane ℓ builds its A fragment — row ℓ mod
// 16, slots 32⌊ℓ/16⌋ … +31 (32 bytes) — by walking the (≤ 16 for stumps) trees those slots belong
// to on the row's bins (LDS), and reads its B fragment (32 bytes, pre-swizzled on the host into the
// same lane / byte → slot order) from LDS.  A and B use one (lane group, byte) → k assignment, so
// the product sums every slot once whatever the hardware's internal k order.  4× fewer MFMAs than
// the gfx940-era 16x16x32 fp8 form; the tree walks that build the one-hot dominate either way.  Workgroups are persistent over
// 64-row tiles, so V, the tree table and the fragment layout are staged in LDS once per workgroup.
#include "common.h"

namespace hfens {

typedef float f8x4_acc __attribute__((ext_vector_type(4)));
typedef int f8x8i __attribute__((ext_vector_type(8)));

struct F8Job {
  const unsigned char* bins;          // [F][ldb] u8 feature-major bins
  long long ldb, n;
  int F, T, d, Q, S;                  // features, trees, depth, K steps (K_pad / 128), models
  const unsigned short* nodes;        // [T][2^d − 1] internal heap nodes: (blo << 8) | feat, feat 255 = leaf
  const unsigned long long* bfrag;    // [Q][64][4] B fragments (32 × fp8 per lane, MFMA lane order)
  const float* inv_scale;             // [S]
  const double* init;                 // [S]
  float* out;                         // [S][n]
};

constexpr int kF8Waves = 4;
constexpr int kF8MaxF = 128;
constexpr unsigned kF8One = 0x38u;    // e4m3: 1.0

// DEPTH = tree depth: the 32 slots a lane owns per K step hold NT = 32 / 2^DEPTH whole trees, walked
// level-synchronously (all NT node reads, then all NT bin reads, per level) so their LDS latencies
// overlap instead of chaining tree after tree.
template <int DEPTH>
__global__ __launch_bounds__(kF8Waves * 64) void forest_fp8_kernel(F8Job J, int stage_b, int stage_nodes) {
  constexpr int LT = 1 << DEPTH, NT = 32 / LT, NIT = LT - 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char f8_lds[];
  const int NI = (1 << J.d) - 1;
  unsigned long long* sb = reinterpret_cast<unsigned long long*>(f8_lds);                 // [Q][64][4]
  unsigned short* sn = reinterpret_cast<unsigned short*>(f8_lds + (stage_b ? (size_t)J.Q * 64 * 32 : 0));
  unsigned char* rb = f8_lds + (stage_b ? (size_t)J.Q * 64 * 32 : 0) +
                      (stage_nodes ? (((size_t)J.T * NI * 2 + 15) & ~(size_t)15) : 0);    // [waves][16][F]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (stage_b)
    for (int i = tid; i < J.Q * 64 * 4; i += blockDim.x) sb[i] = J.bfrag[i];
  if (stage_nodes)
    for (int i = tid; i < J.T * NI; i += blockDim.x) sn[i] = J.nodes[i];
  __syncthreads();
  const unsigned long long* Bf = stage_b ? sb : J.bfrag;
  const unsigned short* Nd = stage_nodes ? sn : J.nodes;
  unsigned char* myb = rb + (size_t)wave * 16 * J.F;
  const int r = lane & 15, kb = lane >> 4;
  const long long tiles = (J.n + 15) / 16;
  for (long long tile = (long long)blockIdx.x * kF8Waves + wave; tile < tiles; tile += (long long)gridDim.x * kF8Waves) {
    const long long row0 = tile * 16;
    // this tile's 16 rows × F bins into the wave's LDS slab (rows past n read bin 0)
    for (int i = lane; i < 16 * J.F; i += 64) {
      const int rr = i & 15, f = i >> 4;
      myb[rr * J.F + f] = row0 + rr < J.n ? J.bins[(size_t)f * J.ldb + row0 + rr] : 0;
    }
    // the slab is read by other lanes of this wave only: drain its LDS stores (no workgroup
    // barrier — the waves of a workgroup run different numbers of tiles)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned char* rowb = myb + r * J.F;
    f8x4_acc acc = {0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < J.Q; ++q) {
      const int k0 = 128 * q + 32 * kb;
      unsigned w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      const int t0 = k0 >> DEPTH;          // the lane's first tree (k0 is a multiple of 32 ≥ LT)
      int h[NT];
#pragma unroll
      for (int i = 0; i < NT; ++i) h[i] = 0;
#pragma unroll
      for (int lev = 0; lev < DEPTH; ++lev) {
        unsigned nd[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) nd[i] = t0 + i < J.T ? Nd[(size_t)(t0 + i) * NIT + h[i]] : 0xFFu;
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          const unsigned f = nd[i] & 0xFFu;
          const int right = (f != 0xFFu) && (rowb[f < (unsigned)J.F ? f : 0u] > (nd[i] >> 8));
          h[i] = 2 * h[i] + 1 + right;
        }
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        if (t0 + i >= J.T) continue;
        const int leaf = h[i] - (LT - 1);            // slot i·LT + leaf of the lane's 32
        if constexpr (LT <= 4) {
          const int dw = (i * LT) >> 2;              // the tree's slots lie in one dword
          w[dw] |= kF8One << (8 * (((i * LT) & 3) + leaf));
        } else {
#pragma unroll
          for (int c = 0; c < LT / 4; ++c)
            w[(i * LT >> 2) + c] |= (leaf >> 2) == c ? kF8One << (8 * (leaf & 3)) : 0u;
        }
      }
      const f8x8i a = {(int)w[0], (int)w[1], (int)w[2], (int)w[3], (int)w[4], (int)w[5], (int)w[6], (int)w[7]};
      const unsigned long long* bq = Bf + ((size_t)q * 64 + lane) * 4;
      const f8x8i b = {(int)(unsigned)bq[0], (int)(unsigned)(bq[0] >> 32), (int)(unsigned)bq[1],
                       (int)(unsigned)(bq[1] >> 32), (int)(unsigned)bq[2], (int)(unsigned)(bq[2] >> 32),
                       (int)(unsigned)bq[3], (int)(unsigned)(bq[3] >> 32)};
      // fmt 0/0 = e4m3 A and B; scales 127 = 2^0 (E8M0) for both
      acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 127, 0, 127);
    }
    // C: lane ℓ holds rows 4⌊ℓ/16⌋ + i (i < 4) of column ℓ mod 16; model s = hi column s + lo column S + s
    const int col = lane & 15;
    float part[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) part[i] = __shfl(acc[i], (lane & 48) | ((col + J.S) & 15), 64);
    if (col < J.S) {
      const float is = J.inv_scale[col];
      const float base = (float)J.init[col];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long row = row0 + 4 * kb + i;
        if (row < J.n) J.out[(size_t)col * J.n + row] = base + (acc[i] + part[i]) * is;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slab reads done before the next tile's stores
  }
}

void forest_fp8(uintptr_t bins, long long ldb, long long n, int F, int T, int d, uintptr_t nodes, uintptr_t bfrag,
                int Q, int S, uintptr_t inv_scale, uintptr_t init, uintptr_t out, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= kF8MaxF, "forest_fp8: 1 <= F <= 128");
  HFENS_REQUIRE(d >= 1 && d <= 5 && T >= 1, "forest_fp8: depth 1..5");
  HFENS_REQUIRE(S >= 1 && 2 * S <= 16, "forest_fp8: 1..8 models per launch (hi/lo columns of one 16-wide tile)");
  HFENS_REQUIRE((long long)Q * 128 >= (long long)T << d, "forest_fp8: K steps do not cover the leaf slots");
  if (n == 0) return;
  const size_t bsz = (size_t)Q * 64 * 32;
  const size_t nsz = (((size_t)T * ((1 << d) - 1) * 2) + 15) & ~(size_t)15;
  const size_t rsz = (size_t)kF8Waves * 16 * F;
  int stage_b = 1, stage_n = 1;
  size_t lds = bsz + nsz + rsz;
  if (lds > 150 * 1024) { stage_b = 0; lds = nsz + rsz; }   // B fragments from L2 instead
  if (lds > 150 * 1024) { stage_n = 0; lds = rsz; }
  int dev = 0, ncu = 256;
  HFENS_CHECK(hipGetDevice(&dev));
  HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const long long tiles = (n + 15) / 16;
  long long g = (tiles + kF8Waves - 1) / kF8Waves;
  const long long cap = 4LL * ncu;                       // persistent: ≈ 4 workgroups per CU
  if (g > cap) g = cap;
  F8Job J{(const unsigned char*)bins, ldb, n, F, T, d, Q, S, (const unsigned short*)nodes,
          (const unsigned long long*)bfrag, (const float*)inv_scale, (const double*)init, (float*)out};
  switch (d) {
#define F8_CASE(D)                                                                                            \
  case D:                                                                                                    \
    hipLaunchKernelGGL(forest_fp8_kernel<D>, dim3((unsigned)g), dim3(kF8Waves * 64), lds, as_stream(stream), J, \
                       stage_b, stage_n);                                                                    \
    break;
    F8_CASE(1) F8_CASE(2) F8_CASE(3) F8_CASE(4) F8_CASE(5)
#undef F8_CASE
  }
  launch_check();
}

}  // namespace hfens
