// Inference kernels for the HF stack.
//
//  * rbf_decision  : dec_j = Σ_i coef_i·exp(-γ‖sv_i − z_j‖²) + b.  ‖sv−z‖² = ‖sv‖²+‖z‖²−2 sv·z with
//                    the dot products on the f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32
//                    fma chains, no TF32-like rounding).  The support vectors are the MFMA A operand
//                    (rows = SVs in the accumulator registers), the data rows the B operand
//                    (columns = lanes), so the Σ over SVs is a register sum + one cross-half
//                    shuffle and each lane ends owning one output row (coalesced store).
//                    SVs (+ norms, coefs) stream through LDS in ≤96 KiB chunks (one chunk ⇒
//                    staged once per workgroup).
//  * svc_proba1    : libsvm Platt sigmoid + iterative 2-class pairwise coupling, in fp64.
//  * forest_raw    : generic tree-ensemble walk (thresholds pre-rounded down to f32 so that
//                    `x32 <= thr32` ≡ sklearn's `float(x32) <= thr64`).
#include "common.h"

namespace hfens {

// ------------------------------------------------------------------------------------------
// RBF decision (MFMA)
// SVt : [F'][mp] (k-major, F' >= F rows), sn/coef : [mp], zero padded (coef 0 ⇒ no contribution).
// SVs stream through LDS in chunks of CH (multiple of 32); with one chunk they are staged once
// per workgroup and stay resident across the grid-stride row loop.
template <int KS>
__global__ __launch_bounds__(256) void rbf_decision_kernel(
    const float* __restrict__ Z, int n, int F, const float* __restrict__ SVt,
    const float* __restrict__ sn, const float* __restrict__ coef, int mp, int CH, float ngl2e,
    float intercept, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* sv_l = lds;                   // [2KS][CH]
  float* sn_l = lds + 2 * KS * CH;     // [CH]
  float* cf_l = sn_l + CH;             // [CH]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r32 = lane & 31;
  const int hi = lane >> 5;
  const int ntile = (n + 31) >> 5;
  const int wpb = blockDim.x >> 6;
  const int nch = (mp + CH - 1) / CH;
  int staged = -1;
  for (int base = blockIdx.x * wpb; base < ntile; base += gridDim.x * wpb) {
    const int tile = base + wave;
    const bool valid = tile < ntile;
    const int row = tile * 32 + r32;
    float z[KS];
    float znp = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 2 * s + hi;
      z[s] = (valid && row < n && k < F) ? Z[(size_t)row * F + k] : 0.f;
      znp = fmaf(z[s], z[s], znp);
    }
    const float zn = znp + __shfl_xor(znp, 32, kWave);
    float part = 0.f;
    for (int c = 0; c < nch; ++c) {
      const int c0 = c * CH;
      const int cl = min(CH, mp - c0);
      if (staged != c) {  // block-uniform
        __syncthreads();
        for (int i = threadIdx.x; i < (2 * KS + 2) * cl; i += blockDim.x) {
          const int k = i / cl, j = i % cl;
          float v;
          if (k < 2 * KS) v = k < F ? SVt[(size_t)k * mp + c0 + j] : 0.f;
          else if (k == 2 * KS) v = sn[c0 + j];
          else v = coef[c0 + j];
          (k < 2 * KS ? sv_l[k * CH + j] : (k == 2 * KS ? sn_l[j] : cf_l[j])) = v;
        }
        __syncthreads();
        staged = c;
      }
      if (!valid) continue;
      for (int t = 0; t < cl; t += 32) {
        f32x16 acc = {0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const float a = sv_l[(2 * s + hi) * CH + t + r32];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, z[s], acc, 0, 0, 0);
        }
        // accumulator reg r ↔ SV t + (r&3) + 8*(r>>2) + 4*hi ; column (lane&31) ↔ data row
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int b0 = t + 8 * g + 4 * hi;
          const f32x4 snv = *reinterpret_cast<const f32x4*>(&sn_l[b0]);
          const f32x4 cfv = *reinterpret_cast<const f32x4*>(&cf_l[b0]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float d2 = fmaf(-2.f, acc[4 * g + q], snv[q] + zn);
            d2 = fmaxf(d2, 0.f);
            part = fmaf(cfv[q], __builtin_amdgcn_exp2f(ngl2e * d2), part);
          }
        }
      }
    }
    part += __shfl_xor(part, 32, kWave);
    if (valid && hi == 0 && row < n) out[row] = part + intercept;
    if (nch > 1) staged = -1;  // next row tile restarts at chunk 0
  }
}

template <int KS>
static void launch_rbf(const float* Z, int n, int F, const float* SVt, const float* sn,
                       const float* coef, int mp, float gamma, float b, float* out, hipStream_t st) {
  // chunk so that one chunk image stays ≤ 96 KiB of LDS
  int CH = (96 * 1024 / (int)((2 * KS + 2) * sizeof(float))) / 32 * 32;
  if (CH > mp) CH = mp;
  const size_t lds = (size_t)(2 * KS + 2) * CH * sizeof(float);
  const int ntile = (n + 31) / 32;
  int grid = (ntile + 3) / 4;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(rbf_decision_kernel<KS>, dim3(grid), dim3(256), lds, st, Z, n, F, SVt, sn,
                     coef, mp, CH, -gamma * 1.4426950408889634f, b, out);
  launch_check();
}

void rbf_decision(uintptr_t Z, int n, int F, uintptr_t SVt, uintptr_t sn, uintptr_t coef, int mp,
                  double gamma, double b, uintptr_t out, uintptr_t stream) {
  HFENS_REQUIRE(mp % 32 == 0 && mp > 0, "rbf_decision: padded SV count must be a positive multiple of 32");
  HFENS_REQUIRE(F >= 1 && F <= 64, "rbf_decision: 1 <= F <= 64");
  const int ks = (F + 1) / 2;
  auto Zp = reinterpret_cast<const float*>(Z);
  auto Sp = reinterpret_cast<const float*>(SVt);
  auto np_ = reinterpret_cast<const float*>(sn);
  auto cp = reinterpret_cast<const float*>(coef);
  auto op = reinterpret_cast<float*>(out);
  hipStream_t st = as_stream(stream);
  if (n == 0) return;
#define RBF_CASE(K) \
  if (ks <= K) return launch_rbf<K>(Zp, n, F, Sp, np_, cp, mp, (float)gamma, (float)b, op, st);
  RBF_CASE(2) RBF_CASE(4) RBF_CASE(8) RBF_CASE(12) RBF_CASE(16) RBF_CASE(24) RBF_CASE(32)
#undef RBF_CASE
}

// ------------------------------------------------------------------------------------------
// Platt + coupling
__device__ __forceinline__ double platt_couple_p1(double dec, double A, double B) {
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
    double err = fmax(fabs(qp0 - pqp), fabs(qp1 - pqp));
    if (err < 0.0025) break;
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

__global__ void svc_proba1_kernel(const float* __restrict__ dec, float* __restrict__ out, int n,
                                  double A, double B) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = (float)platt_couple_p1((double)dec[i], A, B);
}

void svc_proba1(uintptr_t dec, uintptr_t out, int n, double A, double B, uintptr_t stream) {
  if (n == 0) return;
  int grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(svc_proba1_kernel, dim3(grid), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float*>(dec), reinterpret_cast<float*>(out), n, A, B);
  launch_check();
}

// Out-of-fold P(class 1) of several SVC models straight from their decision sums, on the device:
// row i (model k = model[i]) gets meta[rows[i]·ld + col] = proba(f32(dec[i] − rho[k]); A_k, B_k) with
// (A_k, B_k) = AB[2k], AB[2k+1] as the Platt kernel left them — the stacking trainer's OOF column
// without reading the fitted models back to the host (predict_proba's precision: f32 decision,
// f64 sigmoid + coupling, f32 result).
__global__ void svc_oof_kernel(const double* __restrict__ dec, const int* __restrict__ model,
                               const double* __restrict__ rho, const double* __restrict__ AB,
                               const long long* __restrict__ rows, double* __restrict__ meta, int ld, int col,
                               int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int k = model[i];
    const float d = (float)(dec[i] - rho[k]);
    meta[rows[i] * ld + col] = (double)(float)platt_couple_p1((double)d, AB[2 * k], AB[2 * k + 1]);
  }
}

void svc_oof(uintptr_t dec, uintptr_t model, uintptr_t rho, uintptr_t AB, uintptr_t rows, uintptr_t meta, int ld,
             int col, int n, uintptr_t stream) {
  if (n == 0) return;
  int grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(svc_oof_kernel, dim3(grid), dim3(256), 0, as_stream(stream), reinterpret_cast<const double*>(dec),
                     reinterpret_cast<const int*>(model), reinterpret_cast<const double*>(rho),
                     reinterpret_cast<const double*>(AB), reinterpret_cast<const long long*>(rows),
                     reinterpret_cast<double*>(meta), ld, col, n);
  launch_check();
}

// ------------------------------------------------------------------------------------------
// Generic forest walk.  nodes: int4 {feature, left, right, float_as_int(thr32)} [T*K];
// values float [T*K] (unshrunk leaf values).  One thread per row; the row tile lives in LDS
// (row stride F|1 to avoid power-of-two bank conflicts).
__global__ __launch_bounds__(256) void forest_raw_kernel(const float* __restrict__ X, int n, int F,
                                                         const int4* __restrict__ nodes,
                                                         const float* __restrict__ values, int T,
                                                         int K, float init, float lr,
                                                         float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float xs[];
  const int ld = F | 1;
  const int row0 = blockIdx.x * blockDim.x;
  for (int i = threadIdx.x; i < blockDim.x * F; i += blockDim.x) {
    const int r = i / F, c = i % F;
    xs[r * ld + c] = (row0 + r < n) ? X[(size_t)(row0 + r) * F + c] : 0.f;
  }
  __syncthreads();
  const int r = threadIdx.x;
  const float* xr = xs + r * ld;
  float acc = 0.f;
  for (int t = 0; t < T; ++t) {
    const int4* tn = nodes + (size_t)t * K;
    int node = 0;
    int4 nd = tn[0];
    while (nd.x >= 0) {
      node = (xr[nd.x] <= __int_as_float(nd.w)) ? nd.y : nd.z;
      nd = tn[node];
    }
    acc += values[(size_t)t * K + node];
  }
  if (row0 + r < n) out[row0 + r] = init + lr * acc;
}

void forest_raw(uintptr_t X, int n, int F, uintptr_t nodes, uintptr_t values, int T, int K,
                double init, double lr, uintptr_t out, uintptr_t stream) {
  if (n == 0) return;
  const int block = 256;
  const size_t lds = (size_t)block * (F | 1) * sizeof(float);
  HFENS_REQUIRE(lds <= 160 * 1024, "forest_raw: feature count too large for the LDS row tile");
  hipLaunchKernelGGL(forest_raw_kernel, dim3((n + block - 1) / block), dim3(block), lds,
                     as_stream(stream), reinterpret_cast<const float*>(X), n, F,
                     reinterpret_cast<const int4*>(nodes), reinterpret_cast<const float*>(values),
                     T, K, (float)init, (float)lr, reinterpret_cast<float*>(out));
  launch_check();
}

}  // namespace hfens
