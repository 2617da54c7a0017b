// How much independent VALU work hides under v_mfma_f32_32x32x2_f32 on gfx950?
// One wave per SIMD (or two), a chain of MFMAs on 4 accumulators, with N independent
// v_fma_f32 / v_add_u32 between MFMA pairs. Reports cycles per MFMA (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>

using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int NV>
__global__ __launch_bounds__(256) void k(float* out, long long* cyc, int iters) {
  f32x16 a0 = {}, a1 = {}, a2 = {}, a3 = {};
  float x = threadIdx.x * 0.001f, y = 1.0001f;
  float f[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = x + i;
  int u = threadIdx.x;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
#pragma unroll
    for (int v = 0; v < NV; ++v) f[v & 7] = __builtin_fmaf(f[v & 7], y, x);
    __builtin_amdgcn_sched_barrier(0);
    a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a1, 0, 0, 0);
#pragma unroll
    for (int v = 0; v < NV; ++v) f[(v + 3) & 7] = __builtin_fmaf(f[(v + 3) & 7], y, x);
    __builtin_amdgcn_sched_barrier(0);
    a2 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a2, 0, 0, 0);
#pragma unroll
    for (int v = 0; v < NV; ++v) f[(v + 5) & 7] = __builtin_fmaf(f[(v + 5) & 7], y, x);
    __builtin_amdgcn_sched_barrier(0);
    a3 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a3, 0, 0, 0);
#pragma unroll
    for (int v = 0; v < NV; ++v) f[(v + 1) & 7] = __builtin_fmaf(f[(v + 1) & 7], y, x);
    __builtin_amdgcn_sched_barrier(0);
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += a0[i] + a1[i] + a2[i] + a3[i];
  for (int i = 0; i < 8; ++i) s += f[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NV>
void run(int wpsimd, float* out, long long* cyc) {
  const int iters = 2000;
  // 256 CUs x wpsimd waves per SIMD: block = 256 threads (4 waves, one per SIMD)
  dim3 grid(256 * wpsimd);
  k<NV><<<grid, 256>>>(out, cyc, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  k<NV><<<grid, 256>>>(out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double mf = 4.0 * iters * grid.x * 4;   // MFMAs (4 waves per block)
  printf("waves/SIMD=%d VALU per MFMA=%2d: %.1f cyc/MFMA (wave view), %.1f TF/s\n", wpsimd, NV,
         (double)c / (4.0 * iters), mf * 4096 / (ms * 1e-3) / 1e12);
}

int main() {
  float* out; long long* cyc;
  hipMalloc(&out, 256 * 8 * 256 * 4); hipMalloc(&cyc, 256 * 8 * 8);
  for (int w : {1, 2}) {
    run<0>(w, out, cyc); run<2>(w, out, cyc); run<4>(w, out, cyc); run<8>(w, out, cyc);
    run<12>(w, out, cyc); run<16>(w, out, cyc); run<24>(w, out, cyc);
  }
  return 0;
}
