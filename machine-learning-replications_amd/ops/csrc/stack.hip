// Fused inference of the whole HF stack (SURVEY.md §2.3 K11 stack_infer; reference
// predict_hf.py:36 → StackingClassifier.predict_proba, semantics SURVEY.md Appendix B):
//
//   z      = (x − mean)·(1/scale)                                  (StandardScaler)
//   dec    = Σ_i c_i·exp(−γ‖sv_i − z‖²) + b_svc                    (RBF SVC, f32-input MFMA)
//   p_svc  = libsvm Platt sigmoid + iterative 2-class coupling      (f64)
//   p_gbc  = σ(init + lr·Σ_t value_t[leaf_t(x)])                    (tree walk, trees in LDS)
//   p_lg   = σ(w·x + b)                                             (L1-LR on raw inputs)
//   P      = σ(w_m·[p_svc, p_gbc, p_lg] + b_m)                      (meta LR)
//
// One wave owns 64 rows: two 32-row MFMA tiles (data rows are the B operand/columns, SVs the A
// operand, so Σ over SVs = register sum + one cross-half shuffle), then every lane finishes one
// row's scalar tail.  Each input row is read from HBM exactly once — prefetched into registers
// one tile ahead, then parked in a per-wave LDS tile that the MFMA operands, the tree walk and
// the LR dot all read — and one f32 probability is written.  For the shipped model that is
// 72 B/row against ~15 kFLOP of MFMA work + 434 exp2/row, i.e. MFMA/transcendental-bound, not
// HBM-bound.  All support vectors (+‖sv‖², coefs) and the tree tables are staged in LDS once per
// workgroup (streamed in chunks when they exceed LDS); the grid is persistent (occupancy-sized).
#include "common.h"

#include <cstdlib>

namespace hfens {

struct StackModel {
  int F;
  int mp;           // padded SV count (multiple of 32) — all SVs staged in LDS at once
  int T, K;         // trees × nodes per tree
  float ngl2e;      // −γ·log2(e)
  float svc_b;      // libsvm intercept (−rho)
  double probA, probB;
  float gb_init, gb_lr;
  float lr_b;
  float meta_w0, meta_w1, meta_w2, meta_b;
  const float* mean;       // [F]
  const float* inv_scale;  // [F]
  const float* svt;        // [F'][mp] k-major
  const float* sn;         // [mp]
  const float* coef;       // [mp]
  const int4* nodes;       // [T*K] {feature, left, right, bits(thr32)}
  const float* values;     // [T*K]
  const float* lr_w;       // [F]
  const int* st_off;       // [F+1] stump-table offsets (nullptr ⇒ generic tree walk)
  const float2* st_pairs;  // [P] {thr32, lr·(v_right − v_left)}
  float st_base;           // init + lr·Σ v_left
};

__device__ __forceinline__ double couple_p1(double dec, double A, double B) {
  const double fApB = dec * A + B;
  double r01 = fApB >= 0 ? exp(-fApB) / (1.0 + exp(-fApB)) : 1.0 / (1.0 + exp(fApB));
  r01 = fmin(fmax(r01, 1e-7), 1 - 1e-7);
  const double r10 = 1.0 - r01;
  const double q00 = r10 * r10, q11 = r01 * r01, q01 = -r10 * r01;
  double p0 = 0.5, p1 = 0.5;
  for (int it = 0; it < 100; ++it) {
    double qp0 = q00 * p0 + q01 * p1;
    double qp1 = q01 * p0 + q11 * p1;
    double pqp = p0 * qp0 + p1 * qp1;
    if (fmax(fabs(qp0 - pqp), fabs(qp1 - pqp)) < 0.0025) break;
    double d = (-qp0 + pqp) / q00;
    p0 += d;
    pqp = (pqp + d * (d * q00 + 2 * qp0)) / (1 + d) / (1 + d);
    qp0 = (qp0 + d * q00) / (1 + d);
    qp1 = (qp1 + d * q01) / (1 + d);
    p0 /= (1 + d);
    p1 /= (1 + d);
    d = (-qp1 + pqp) / q11;
    p1 += d;
    p0 /= (1 + d);
    p1 /= (1 + d);
  }
  return p1;
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + __expf(-v)); }

// X3: the sv·z products on the bf16 matrix cores, exactly split.  Every f32 operand v is cut into
// three bf16 pieces v = v0 + v1 + v2 (truncation: 8 + 8 + 8 significant bits, no rounding), and
// sv·z = Σ_f Σ_{i+j ≤ 2} sv_f,i · z_f,j (the 6 largest piece products; the dropped ones are
// ≤ 3·2⁻²⁴ of |sv_f||z_f|, f32-level).  The 6·2KS (product, feature) items are packed along K in two
// lane-half lists — half 0: (0,0), (0,1), (1,0); half 1: (0,2), (1,1), (2,0) as (sv piece, z
// piece) — so one v_mfma_f32_32x32x16_bf16 takes 16 items: ⌈3KS/4⌉ MFMAs per 32 × 32 tile against
// KS of v_mfma_f32_32x32x2f32 (7 vs 9 for the 17-feature model, at 16× the rate per instruction).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <int KS>
constexpr int x3_blocks() { return (3 * 2 * KS + 7) / 8; }   // MFMA k-blocks of 8 items per half

__device__ __forceinline__ void x3_split(float v, unsigned (&b)[3]) {   // bf16 bits of the 3 pieces
  const unsigned u0 = __float_as_uint(v) & 0xFFFF0000u;
  const float r1 = v - __uint_as_float(u0);
  const unsigned u1 = __float_as_uint(r1) & 0xFFFF0000u;
  const float r2 = r1 - __uint_as_float(u1);
  b[0] = u0 >> 16;
  b[1] = u1 >> 16;
  b[2] = __float_as_uint(r2) >> 16;   // r2 has ≤ 8 significant bits: exact in bf16
}

// piece of the SV (js) and of the row (iz) for item-list position p (0..2) of lane half h
__host__ __device__ constexpr int x3_sv_piece(int h, int p) { return h ? 2 - p : (p == 1 ? 1 : 0); }
__host__ __device__ constexpr int x3_z_piece(int h, int p) { return h ? p : (p == 2 ? 1 : 0); }

// KS = MFMA k-steps (2 features each); the row tile holds 64·F ≤ 64·2KS values, so each lane
// prefetches at most 2KS of them.
template <int KS, int W, typename TX, bool X3 = false>
__global__ __launch_bounds__(64 * W) void stack_infer_kernel(const TX* __restrict__ X,
                                                                       long long n, StackModel M,
                                                                       int CH, int nodes_in_lds,
                                                                       float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int F = M.F, mp = M.mp;
  const int ldx = F | 1;
  const int nch = (mp + CH - 1) / CH;
  constexpr int NB3 = x3_blocks<KS>();
  float* sv_l = lds;                              // [2KS][CH] f32, or X3: [NB3][CH][16] bf16
  unsigned short* sv3 = reinterpret_cast<unsigned short*>(lds);
  float* sn_l = sv_l + (X3 ? NB3 * CH * 8 : 2 * KS * CH);   // [CH]
  float* cf_l = sn_l + CH;                        // [CH]
  float* mu_l = cf_l + CH;                        // [2KS] mean, then [2KS] 1/scale
  float* is_l = mu_l + 2 * KS;
  float* xs = is_l + 2 * KS;                      // [waves][64][ldx]
  const int xs_n = W * 64 * ldx;
  int4* nd_l = reinterpret_cast<int4*>(xs + ((xs_n + 3) & ~3));
  float* nv_l = reinterpret_cast<float*>(nd_l + (nodes_in_lds ? M.T * M.K : 0));
  auto stage = [&](int c) {  // SV chunk c → LDS (block-wide; caller synchronises)
    const int c0 = c * CH, cl = min(CH, mp - c0);
    if constexpr (X3) {
      // item (m, j, 8h + e): list position q = 8m + e of half h → (piece, feature) of SV j
      for (int i = threadIdx.x; i < NB3 * CH * 16; i += blockDim.x) {
        const int m = i / (CH * 16), rem = i - m * CH * 16, j = rem >> 4, he = rem & 15;
        const int h = he >> 3, q = 8 * m + (he & 7);
        unsigned v = 0;
        if (j < cl && q < 3 * 2 * KS) {
          const int pl = q / (2 * KS), f = q - pl * (2 * KS);
          if (f < F) {
            unsigned b[3];
            x3_split(M.svt[(size_t)f * mp + c0 + j], b);
            const int js = x3_sv_piece(h, pl);
            v = js == 0 ? b[0] : (js == 1 ? b[1] : b[2]);
          }
        }
        sv3[i] = (unsigned short)v;
      }
      for (int i = threadIdx.x; i < 2 * CH; i += blockDim.x) {
        const int k = i / CH, j = i - k * CH;
        sn_l[i] = j < cl ? (k == 0 ? M.ngl2e * M.sn[c0 + j] : M.coef[c0 + j]) : 0.f;
      }
      return;
    }
    for (int i = threadIdx.x; i < (2 * KS + 2) * CH; i += blockDim.x) {
      const int k = i / CH, j = i - k * CH;
      float v = 0.f;
      if (j < cl) {
        if (k < 2 * KS) v = k < F ? M.svt[(size_t)k * mp + c0 + j] : 0.f;
        else if (k == 2 * KS) v = M.ngl2e * M.sn[c0 + j];
        else v = M.coef[c0 + j];
      }
      lds[i] = v;
    }
  };
  stage(0);
  for (int i = threadIdx.x; i < 2 * KS; i += blockDim.x) {
    mu_l[i] = i < F ? M.mean[i] : 0.f;
    is_l[i] = i < F ? M.inv_scale[i] : 0.f;
  }
  if (nodes_in_lds) {
    for (int i = threadIdx.x; i < M.T * M.K; i += blockDim.x) {
      nd_l[i] = M.nodes[i];
      nv_l[i] = M.values[i];
    }
  }
  __syncthreads();
  const int4* nodes = nodes_in_lds ? nd_l : M.nodes;
  const float* nvals = nodes_in_lds ? nv_l : M.values;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r32 = lane & 31, hi = lane >> 5;
  float* xw = xs + wave * 64 * ldx;
  const long long ntile = (n + 63) / 64;
  const long long stride = (long long)gridDim.x * W;
  const long long nel = n * F;

  // register prefetch of one 64-row tile: element e = lane + 64·i of the tile's flat block
  float pre[2 * KS];
  auto fetch = [&](long long tile) {
    const long long base = tile * 64 * F;
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      const long long g = base + lane + 64 * i;
      pre[i] = (i < F && tile < ntile && g < nel) ? (float)X[g] : 0.f;
    }
  };
  // block-uniform tile loop (all waves take part in the chunk barriers when nch > 1)
  for (long long base = (long long)blockIdx.x * W; base < ntile; base += stride) {
    const long long tile = base + wave;
    const bool valid = tile < ntile;
    const long long row0 = tile * 64;
    if (base == (long long)blockIdx.x * W) fetch(tile);
    // park the prefetched tile in LDS (flat index e ↔ row e/F, col e%F), fetch the next one
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      if (i < F) {
        const int e = lane + 64 * i;
        const int r = e / F;
        xw[r * ldx + (e - r * F)] = pre[i];
      }
    }
    fetch(tile + stride);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float za[KS], zb[KS];
    float zna = 0.f, znb = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 2 * s + hi;
      float a = 0.f, b = 0.f;
      if (k < F) {
        const float mu = mu_l[k], is = is_l[k];
        a = (xw[r32 * ldx + k] - mu) * is;
        b = (xw[(32 + r32) * ldx + k] - mu) * is;
      }
      za[s] = a;
      zb[s] = b;
      zna = fmaf(a, a, zna);
      znb = fmaf(b, b, znb);
    }
    zna += __shfl_xor(zna, 32, kWave);
    znb += __shfl_xor(znb, 32, kWave);
    // X3: this lane's row pieces for its lane half's item list (rows r32 and 32 + r32)
    bf16x8_t z3a[X3 ? NB3 : 1], z3b[X3 ? NB3 : 1];
    if constexpr (X3) {
      unsigned pa3[2 * KS][3], pb3[2 * KS][3];
#pragma unroll
      for (int f = 0; f < 2 * KS; ++f) {
        float a = 0.f, b = 0.f;
        if (f < F) {
          const float mu = mu_l[f], is = is_l[f];
          a = (xw[r32 * ldx + f] - mu) * is;
          b = (xw[(32 + r32) * ldx + f] - mu) * is;
        }
        x3_split(a, pa3[f]);
        x3_split(b, pb3[f]);
      }
#pragma unroll
      for (int m = 0; m < NB3; ++m) {
        unsigned wa[4], wb[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          unsigned lo_a = 0, hi_a = 0, lo_b = 0, hi_b = 0;
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const int q = 8 * m + 2 * e2 + d;
            unsigned va = 0, vb = 0;
            if (q < 3 * 2 * KS) {
              const int pl = q / (2 * KS), f = q - pl * (2 * KS);
              const int i0 = x3_z_piece(0, pl), i1 = x3_z_piece(1, pl);
              va = hi ? pa3[f][i1] : pa3[f][i0];
              vb = hi ? pb3[f][i1] : pb3[f][i0];
            }
            if (d == 0) { lo_a = va; lo_b = vb; } else { hi_a = va; hi_b = vb; }
          }
          wa[e2] = lo_a | (hi_a << 16);
          wb[e2] = lo_b | (hi_b << 16);
        }
        z3a[m] = __builtin_bit_cast(bf16x8_t, (u32x4_t){wa[0], wa[1], wa[2], wa[3]});
        z3b[m] = __builtin_bit_cast(bf16x8_t, (u32x4_t){wb[0], wb[1], wb[2], wb[3]});
      }
    }
    // exponent of exp(−γ‖sv−z‖²) in base 2: (γ'·‖sv‖²) + (γ'·‖z‖²) + (−2γ')·(sv·z), γ' = −γ·log2 e;
    // ‖sv‖² is staged pre-scaled.  No clamp at 0: a rounding-negative distance only turns
    // exp2 into 1+ε, exactly like the double-precision kernel evaluation it mirrors.
    const float zsa = M.ngl2e * zna, zsb = M.ngl2e * znb, k2 = -2.f * M.ngl2e;
    float pa = 0.f, pb = 0.f;
    auto mma = [&](int t, f32x16& A, f32x16& B) {
      A = f32x16{0.f};
      B = f32x16{0.f};
      if constexpr (X3) {
#pragma unroll
        for (int m = 0; m < NB3; ++m) {
          const u32x4_t raw = *reinterpret_cast<const u32x4_t*>(&sv3[((size_t)m * CH + t + r32) * 16 + 8 * hi]);
          const bf16x8_t sv = __builtin_bit_cast(bf16x8_t, raw);
          A = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sv, z3a[m], A, 0, 0, 0);
          B = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sv, z3b[m], B, 0, 0, 0);
        }
        return;
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float sv = sv_l[(2 * s + hi) * CH + t + r32];
        A = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, za[s], A, 0, 0, 0);
        B = __builtin_amdgcn_mfma_f32_32x32x2f32(sv, zb[s], B, 0, 0, 0);
      }
    };
    // accumulator reg r ↔ SV t + (r&3) + 8(r>>2) + 4·hi ; column (lane&31) ↔ data row
    auto epi = [&](int t, const f32x16& A, const f32x16& B) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int b0 = t + 8 * g + 4 * hi;
        const f32x4 snv = *reinterpret_cast<const f32x4*>(&sn_l[b0]);
        const f32x4 cfv = *reinterpret_cast<const f32x4*>(&cf_l[b0]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pa = fmaf(cfv[q], __builtin_amdgcn_exp2f(fmaf(k2, A[4 * g + q], snv[q] + zsa)), pa);
          pb = fmaf(cfv[q], __builtin_amdgcn_exp2f(fmaf(k2, B[4 * g + q], snv[q] + zsb)), pb);
        }
      }
    };
    for (int c = 0; c < nch; ++c) {
      if (nch > 1) {  // block-uniform: restage chunk c (chunk 0 is resident on entry)
        if (c > 0 || base != (long long)blockIdx.x * W) {
          __syncthreads();
          stage(c);
          __syncthreads();
        }
      }
      const int cl = min(CH, mp - c * CH);
      // (a software-pipelined variant — MFMAs of tile t+32 issued before the epilogue of t —
      // measured 9 % slower: +49 VGPRs cost a wave/SIMD of occupancy)
      for (int t = 0; t < cl; t += 32) {
        f32x16 A, B;
        mma(t, A, B);
        epi(t, A, B);
      }
    }
    pa += __shfl_xor(pa, 32, kWave);
    pb += __shfl_xor(pb, 32, kWave);
    if (valid) {
      // ---- scalar tail: lane ↔ row row0 + lane
      const float dec = (lane < 32 ? pa : pb) + M.svc_b;
      const double p_svc = couple_p1((double)dec, M.probA, M.probB);
      const float* xr = xw + lane * ldx;
      float p_gbc, lin = M.lr_b;
      if (M.st_off != nullptr) {
        // folded stumps: one LDS read per feature feeds both the LR dot and the stump pairs;
        // the tables are wave-uniform (scalar loads)
        float raw = M.st_base;
        for (int k = 0; k < F; ++k) {
          const float xv = xr[k];
          lin = fmaf(xv, M.lr_w[k], lin);
          const int j1 = M.st_off[k + 1];
          for (int j = M.st_off[k]; j < j1; ++j) {
            const float2 pr = M.st_pairs[j];
            raw += xv > pr.x ? pr.y : 0.f;
          }
        }
        p_gbc = sigmoidf_(raw);
      } else {
        float raw = 0.f;
        for (int tr = 0; tr < M.T; ++tr) {
          const int4* tn = nodes + tr * M.K;
          int node = 0;
          int4 ndv = tn[0];
          while (ndv.x >= 0) {
            node = (xr[ndv.x] <= __int_as_float(ndv.w)) ? ndv.y : ndv.z;
            ndv = tn[node];
          }
          raw += nvals[tr * M.K + node];
        }
        p_gbc = sigmoidf_(M.gb_init + M.gb_lr * raw);
        for (int k = 0; k < F; ++k) lin = fmaf(xr[k], M.lr_w[k], lin);
      }
      const float p_lg = sigmoidf_(lin);
      const float m = M.meta_b + M.meta_w0 * (float)p_svc + M.meta_w1 * p_gbc + M.meta_w2 * p_lg;
      if (row0 + lane < n) out[row0 + lane] = sigmoidf_(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // xw is rewritten by the next tile
  }
}

// floats of LDS per staged SV: f32 k-major features, or X3's bf16 item blocks; + ‖sv‖², coef
static int stack_sv_floats(int ks, bool x3) { return x3 ? ((3 * 2 * ks + 7) / 8) * 8 + 2 : 2 * ks + 2; }

static size_t stack_lds_bytes(int W, int F, int CH, int ks, size_t node_bytes, bool x3 = false) {
  size_t xs = (size_t)W * 64 * (F | 1);
  xs = (xs + 3) & ~(size_t)3;
  return ((size_t)stack_sv_floats(ks, x3) * CH + 4 * ks + xs) * 4 + node_bytes;
}

constexpr size_t kStackLdsCap = 160 * 1024;

// SV chunk (multiple of 32): all SVs resident when they fit, else the largest chunk that does.
static int stack_chunk(int W, int F, int mp, int ks, size_t node_bytes, bool x3 = false) {
  const size_t fixed = stack_lds_bytes(W, F, 0, ks, node_bytes, x3);
  if (fixed >= kStackLdsCap) return 0;
  long long ch = (long long)((kStackLdsCap - fixed) / ((size_t)stack_sv_floats(ks, x3) * 4)) / 32 * 32;
  if (ch > mp) ch = mp;
  return (int)ch;
}

static int stack_ks(int F) {
  const int ks = (F + 1) / 2;
  return ks <= 4 ? 4 : ks <= 9 ? 9 : ks <= 12 ? 12 : ks <= 16 ? 16 : 32;
}

struct StackPlan {
  int CH = 0, in_lds = 0, blocks_per_cu = 0;
  size_t lds = 0;
};

// LDS plan for W waves/workgroup: SVs resident if at all possible (trees only when they fit too);
// occupancy from the runtime for the kernel's real register count.
template <int KS, int W, typename TX, bool X3 = false>
static StackPlan stack_plan(const StackModel& M) {
  StackPlan p;
  const size_t node_bytes = M.st_off ? 0 : (size_t)M.T * M.K * 20;
  bool in_lds = node_bytes > 0 && node_bytes <= 24 * 1024;
  int CH = stack_chunk(W, M.F, M.mp, KS, in_lds ? node_bytes : 0, X3);
  if (in_lds && CH < M.mp) {
    const int ch2 = stack_chunk(W, M.F, M.mp, KS, 0, X3);
    if (ch2 > CH) { in_lds = false; CH = ch2; }
  }
  if (CH < 32) return p;
  p.CH = CH;
  p.in_lds = in_lds;
  p.lds = stack_lds_bytes(W, M.F, CH, KS, in_lds ? node_bytes : 0, X3);
  HFENS_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&p.blocks_per_cu, stack_infer_kernel<KS, W, TX, X3>,
                                                           64 * W, p.lds));
  return p;
}

template <int KS, int W, typename TX, bool X3 = false>
static void stack_go(const TX* X, long long n, const StackModel& M, const StackPlan& p, int grid,
                     float* out, hipStream_t st) {
  if (grid <= 0) {
    int dev = 0, ncu = 256;
    HFENS_CHECK(hipGetDevice(&dev));
    HFENS_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const long long tiles = (n + 63) / 64;
    const long long need = (tiles + W - 1) / W;
    const long long cap = (long long)(p.blocks_per_cu > 0 ? p.blocks_per_cu : 1) * ncu;
    grid = (int)(need < cap ? need : cap);
  }
  hipLaunchKernelGGL((stack_infer_kernel<KS, W, TX, X3>), dim3(grid), dim3(64 * W), p.lds, st, X, n, M, p.CH,
                     p.in_lds, out);
  launch_check();
}

static int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// Pick the workgroup size that keeps the most waves resident per CU: one workgroup shares one
// LDS copy of the SVs, so wider workgroups trade LDS for occupancy.  Only shapes that compile
// without VGPR spills are candidates (KS ≤ 9: 8 or 12 waves; 12 waves fit 152 VGPRs at 3
// waves/SIMD — measured 4.9 G rows/s vs 4.7 for 8); HFENS_STACK_WAVES=8|12|16 forces a shape.
template <int KS, typename TX>
static void stack_pick(const TX* X, long long n, const StackModel& M, int grid, float* out,
                       hipStream_t st) {
  static const int forced = env_int("HFENS_STACK_WAVES", 0);
  constexpr bool narrow = KS <= 9;
  if constexpr (narrow) {
    // X3 (bf16x3 products on the bf16 matrix cores) when every SV stays resident in LDS;
    // HFENS_STACK_X3=0 keeps the f32 MFMA path
    if (env_int("HFENS_STACK_X3", 1) != 0) {
      const int xw = forced == 12 || forced == 8 ? forced : env_int("HFENS_STACK_X3_WAVES", 8);
      if (xw == 12) {
        const StackPlan q = stack_plan<KS, 12, TX, true>(M);
        if (q.CH >= M.mp && q.blocks_per_cu > 0) return stack_go<KS, 12, TX, true>(X, n, M, q, grid, out, st);
      } else {
        const StackPlan q = stack_plan<KS, 8, TX, true>(M);
        if (q.CH >= M.mp && q.blocks_per_cu > 0) return stack_go<KS, 8, TX, true>(X, n, M, q, grid, out, st);
      }
    }
  }
  const StackPlan p8 = stack_plan<KS, 8, TX>(M);
  StackPlan p12, p16;
  if constexpr (narrow) {
    p12 = stack_plan<KS, 12, TX>(M);
    p16 = stack_plan<KS, 16, TX>(M);
  }
  // fewer SV chunks first (restaging costs L2 traffic + barriers), then more resident waves
  auto score = [&](const StackPlan& p, int w) {
    return p.CH ? (long long)(p.CH >= M.mp) * 1000 + w * p.blocks_per_cu : -1LL;
  };
  const long long s8 = score(p8, 8), s12 = narrow ? score(p12, 12) : -1;
  if constexpr (narrow) {
    if (forced == 16 && p16.CH) return stack_go<KS, 16, TX>(X, n, M, p16, grid, out, st);
    if (forced == 12 && p12.CH) return stack_go<KS, 12, TX>(X, n, M, p12, grid, out, st);
  }
  HFENS_REQUIRE(s8 > 0 || s12 > 0, "stack_infer: feature tile does not fit LDS");
  if constexpr (narrow) {
    if (forced != 8 && s12 > s8) return stack_go<KS, 12, TX>(X, n, M, p12, grid, out, st);
  }
  stack_go<KS, 8, TX>(X, n, M, p8, grid, out, st);
}

template <typename TX>
static void stack_launch(const TX* X, long long n, const StackModel& M, int grid, float* out,
                         hipStream_t st) {
  switch (stack_ks(M.F)) {
    case 4: stack_pick<4, TX>(X, n, M, grid, out, st); break;
    case 9: stack_pick<9, TX>(X, n, M, grid, out, st); break;
    case 12: stack_pick<12, TX>(X, n, M, grid, out, st); break;
    case 16: stack_pick<16, TX>(X, n, M, grid, out, st); break;
    default: stack_pick<32, TX>(X, n, M, grid, out, st); break;
  }
}

// Largest SV chunk over the workgroup shapes (== mp ⇔ every SV stays resident in LDS).
long long stack_infer_lds(int F, int mp, int nodes_total) {
  (void)nodes_total;
  return stack_chunk(8, F, mp, stack_ks(F), 0);
}

void stack_infer(uintptr_t X, int x_f64, long long n, int F, int mp, int T, int K, double ngl2e,
                 double svc_b, double probA, double probB, double gb_init, double gb_lr, double lr_b,
                 double mw0, double mw1, double mw2, double mb, uintptr_t mean, uintptr_t inv_scale,
                 uintptr_t svt, uintptr_t sn, uintptr_t coef, uintptr_t nodes, uintptr_t values,
                 uintptr_t lr_w, uintptr_t st_off, uintptr_t st_pairs, double st_base, uintptr_t out,
                 int grid, uintptr_t stream) {
  HFENS_REQUIRE(F >= 1 && F <= 64, "stack_infer: 1 <= F <= 64");
  HFENS_REQUIRE(mp % 32 == 0 && mp > 0, "stack_infer: padded SV count must be a positive multiple of 32");
  HFENS_REQUIRE(T >= 0 && K >= 1, "stack_infer: bad tree table shape");
  if (n == 0) return;
  StackModel M{F, mp, T, K, (float)ngl2e, (float)svc_b, probA, probB, (float)gb_init, (float)gb_lr,
               (float)lr_b, (float)mw0, (float)mw1, (float)mw2, (float)mb, (const float*)mean,
               (const float*)inv_scale, (const float*)svt, (const float*)sn, (const float*)coef,
               (const int4*)nodes, (const float*)values, (const float*)lr_w, (const int*)st_off,
               (const float2*)st_pairs, (float)st_base};
  hipStream_t st = as_stream(stream);
  if (x_f64) stack_launch((const double*)X, n, M, grid, (float*)out, st);
  else stack_launch((const float*)X, n, M, grid, (float*)out, st);
}

}  // namespace hfens
