// Does an f32-MFMA-only wave overlap with a VALU-only wave on the same SIMD (gfx950)?
// 512-thread workgroups, one per CU: waves 0-3 (one per SIMD) run a v_mfma_f32_32x32x2_f32
// chain, waves 4-7 (the other wave on each SIMD) run independent v_fma_f32 work.
// Modes: 0 = MFMA waves only (VALU waves exit), 1 = VALU waves only, 2 = both.
// Tuning harness (not part of the product library).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/mfma_overlap.hip -o tools/bench/mfma_overlap
#include <hip/hip_runtime.h>

#include <cstdio>

using f32x16 = __attribute__((ext_vector_type(16))) float;

__global__ __launch_bounds__(512) void k(float* out, int mode, int iters, int vpm) {
  const int wid = threadIdx.x >> 6;
  const bool mfma_wave = wid < 4;
  float x = threadIdx.x * 0.001f, y = 1.0001f;
  if (mfma_wave) {
    if (mode == 1) return;
    f32x16 a0 = {}, a1 = {}, a2 = {}, a3 = {};
    for (int it = 0; it < iters; ++it) {
      a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a3, 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += a0[i] + a1[i] + a2[i] + a3[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  } else {
    if (mode == 0) return;
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = x + i;
    // vpm v_fma per "MFMA slot": 4 slots per iteration, like the MFMA waves' 4 MFMAs
    for (int it = 0; it < iters; ++it) {
      for (int v = 0; v < 4 * vpm; ++v) {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = __builtin_fmaf(f[i], y, x);
        v += 7;
      }
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += f[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
  }
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4 * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  for (int vpm : {8, 16, 32}) {
    for (int mode = 0; mode < 3; ++mode) {
      k<<<256, 512>>>(out, mode, iters, vpm);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      k<<<256, 512>>>(out, mode, iters, vpm);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double mfma_tf = 256.0 * 4 * iters * 4 * 64 * 4096 / 64 / (ms * 1e-3) / 1e12;
      printf("vpm=%2d mode=%s %8.3f ms  (MFMA-only rate would be %.1f TF/s)\n", vpm,
             mode == 0 ? "mfma-only" : mode == 1 ? "valu-only" : "both     ", ms, mfma_tf);
    }
  }
  return 0;
}
