// Shared device/host helpers for the Shift-GCN gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shiftgcn.h"

// Diagnostic builds (timing probes whose results are wrong; `make diag` only): any of
// these macros marks the library, and sgcn_abi_version() then carries SGCN_ABI_DIAG_FLAG.
#if defined(SGCN_PW_DIAG) || defined(SGCN_PW_STAMPS) || defined(SGCN_DIAG_X1B_BOUND) || \
    defined(SGCN_DIAG_F2_BOUND) || defined(SGCN_DIAG_F1B_BOUND) || \
    defined(SGCN_DIAG_F1B_REAL) || defined(SGCN_DIAG_DW64_SKIP)
#define SGCN_DIAG_BUILD 1
#else
#define SGCN_DIAG_BUILD 0
#endif

// Wave priority of the critical path's kernels (s_setprio): every kernel except the
// weight-gradient family (pw_dw*, slab_reduce) and the optimizer-only finalizes, which run
// on the side stream, co-resident with them on the same SIMDs. The fp32 MFMA shares the VALU
// issue, so without it a latency-bound critical-path kernel (e.g. a BatchNorm finalize)
// co-resident with MFMA-saturated weight-gradient waves crawled (profiles/r04_prio/). 0 = off.
#ifndef SGCN_CRIT_PRIO_LEVEL
#define SGCN_CRIT_PRIO_LEVEL 2
#endif
#define SGCN_CRIT_PRIO()                                                   \
  do {                                                                     \
    if (SGCN_CRIT_PRIO_LEVEL) __builtin_amdgcn_s_setprio(SGCN_CRIT_PRIO_LEVEL); \
  } while (0)

#define SGCN_LAUNCH_CHECK()                                   \
  do {                                                        \
    hipError_t e__ = hipGetLastError();                       \
    if (e__ != hipSuccess) return (int)e__;                   \
  } while (0)

#define SGCN_REQUIRE(cond)                                    \
  do {                                                        \
    if (!(cond)) return SGCN_EINVAL;                          \
  } while (0)

namespace sgcn {

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Block-wide sum of one float; result valid in every thread. `red` needs
// blockDim.x/64 floats of LDS. Deterministic (fixed tree).
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// Two floats at once (one barrier pair).
__device__ __forceinline__ void block_sum2(float& a, float& b, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  __syncthreads();
  if (lane == 0) { red[2 * wid] = a; red[2 * wid + 1] = b; }
  __syncthreads();
  float sa = 0.f, sb = 0.f;
  for (int i = 0; i < nw; ++i) { sa += red[2 * i]; sb += red[2 * i + 1]; }
  a = sa;
  b = sb;
}

// The stride-1 temporal shift of an H x W plane evaluated at one output position (h, w),
// from the plane's four taps around (h + y1, w + x1) (shift_cuda_kernel.cu:49-73): tap
// outside the plane = 0, `x1 = floorf(x), dx = x - x1`, the blend left to right with no
// contraction — the same operations in the same order as tshift.hip's forward kernels,
// so the value is bit-identical to the element sgcn_tshift_fwd stores. Used by the
// kernels that read a shift output which is never written (the training unit tail).
struct ShiftGeom {
  int x1, y1;
  float dx, dy;
};
__device__ __forceinline__ ShiftGeom shift_geom(float x, float y) {
#pragma clang fp contract(off)
  ShiftGeom g;
  g.x1 = (int)floorf(x);
  g.y1 = (int)floorf(y);
  g.dx = x - (float)g.x1;
  g.dy = y - (float)g.y1;
  return g;
}
__device__ __forceinline__ float shifted_at(const float* __restrict__ p, const ShiftGeom& g,
                                            int h, int w, int H, int W) {
#pragma clang fp contract(off)
  const int r = h + g.y1, c = w + g.x1;
  const bool r0 = (unsigned)r < (unsigned)H, r1 = (unsigned)(r + 1) < (unsigned)H;
  const bool c0 = (unsigned)c < (unsigned)W, c1 = (unsigned)(c + 1) < (unsigned)W;
  const int rr0 = min(max(r, 0), H - 1) * W, rr1 = min(max(r + 1, 0), H - 1) * W;
  const int cc0 = min(max(c, 0), W - 1), cc1 = min(max(c + 1, 0), W - 1);
  float q11 = p[rr0 + cc0], q21 = p[rr0 + cc1], q12 = p[rr1 + cc0], q22 = p[rr1 + cc1];
  q11 = (r0 && c0) ? q11 : 0.f;
  q21 = (r0 && c1) ? q21 : 0.f;
  q12 = (r1 && c0) ? q12 : 0.f;
  q22 = (r1 && c1) ? q22 : 0.f;
  const float omdx = 1.f - g.dx, omdy = 1.f - g.dy;
  return q11 * omdx * omdy + q21 * g.dx * omdy + q12 * omdx * g.dy + q22 * g.dx * g.dy;
}

// Four floats at once (one barrier pair); `red` needs 4*blockDim.x/64 floats.
__device__ __forceinline__ void block_sum4(float& a, float& b, float& c, float& d, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  d = wave_sum(d);
  __syncthreads();
  if (lane == 0) {
    red[4 * wid] = a;
    red[4 * wid + 1] = b;
    red[4 * wid + 2] = c;
    red[4 * wid + 3] = d;
  }
  __syncthreads();
  float sa = 0.f, sb = 0.f, sc = 0.f, sd = 0.f;
  for (int i = 0; i < nw; ++i) {
    sa += red[4 * i];
    sb += red[4 * i + 1];
    sc += red[4 * i + 2];
    sd += red[4 * i + 3];
  }
  a = sa;
  b = sb;
  c = sc;
  d = sd;
}

// buffer descriptor over [base, base + bytes): 32-bit per-lane voffset + wave-uniform
// soffset, hardware range check (out-of-range loads return 0, stores are dropped)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
// the same with a cache-policy operand (bit 1 = nt, bit 4 = sc1; 0 = default)
template <int AUX>
__device__ __forceinline__ float bload_pol(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, float v, unsigned voff,
                                       unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, 0);
}

// Chan et al. merge of (n, mean, M2) partial statistics, in double.
struct Moments {
  double n, mean, m2;
};
__host__ __device__ inline Moments merge(Moments a, Moments b) {
  if (a.n == 0) return b;
  if (b.n == 0) return a;
  const double n = a.n + b.n, d = b.mean - a.mean;
  return {n, a.mean + d * (b.n / n), a.m2 + b.m2 + d * d * (a.n * b.n / n)};
}

// Training-mode BatchNorm coefficients from the batch sums of per-plane {mean, M2}
// partials (all B partials over n_part elements each): smean = sum mean_b, sm2 = sum M2_b,
// smean2 = sum mean_b^2, in double (bn_finalize_kernel).
struct BnCoef {
  float mean, invstd, scale, shift;
  double unbiased;
};
__device__ __forceinline__ BnCoef bn_train_coef(double smean, double sm2, double smean2, int B,
                                                int n_part, float eps, float g, float bb) {
  const double nb = (double)B, np_ = (double)n_part, n = nb * np_;
  const double mean_d = smean / nb;
  const double m2 = sm2 + np_ * (smean2 - smean * smean / nb);
  const double var = n > 0 ? fmax(m2, 0.0) / n : 0.0;
  BnCoef r;
  r.mean = (float)mean_d;
  r.invstd = (float)(1.0 / sqrt(var + (double)eps));
  r.scale = g * r.invstd;
  r.shift = bb - r.mean * r.scale;
  r.unbiased = n > 1 ? fmax(m2, 0.0) / (n - 1.0) : var;
  return r;
}
__device__ __forceinline__ void bn_running_update(float* rm, float* rv, int rf, float momentum,
                                                  const BnCoef& c) {
  rm[rf] = (1.f - momentum) * rm[rf] + momentum * c.mean;
  rv[rf] = (1.f - momentum) * rv[rf] + momentum * (float)c.unbiased;
}

// Training BatchNorm backward coefficients (dx = k1*g + k2*x + k3) from the batch sums
// sg = sum g, sgx = sum g*xhat (bn_bwd_finalize_kernel's math).
__device__ __forceinline__ float3 bn_bwd_coef(double sg, double sgx, float g, float is,
                                              float mean, double n_total, int batch_stats) {
  const float k1 = g * is;
  // running-statistics (eval) BatchNorm is a fixed affine map: dx = k1 * g
  const float k2 = batch_stats ? (float)(-(double)k1 * (double)is * (sgx / n_total)) : 0.f;
  const float k3 = batch_stats ? (float)(-(double)k1 * (sg / n_total) - (double)k2 * (double)mean)
                               : 0.f;
  return make_float3(k1, k2, k3);
}

}  // namespace sgcn
