// Shared device/host helpers for the Shift-GCN gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shiftgcn.h"

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

}  // namespace sgcn
