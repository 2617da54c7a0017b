// Streaming-pass microbenchmark (tuning harness; not part of the product library).
//
// (1) Infinity-Cache reuse between dependent streaming passes: a producer pass writes Y
//     (reads X); a consumer pass then reads Y (+ W) and writes Z. The consumer walks its
//     blocks either in the producer's order or REVERSED (the last-written lines first,
//     while they may still sit in the 256 MiB die-level cache). Sizes = the Shift-GCN
//     activation tensors (245.8 MB at NTU bs=64) and fractions of it.
// (2) FETCH_SIZE / WRITE_SIZE calibration: known-byte copies with 4-byte and 16-byte lanes
//     (`./l3order calib <bytes-per-lane>` runs ONE copy kind, for a rocprofv3 --pmc pass).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/l3order.hip -o tools/bench/l3order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int NT = 256;
constexpr int V4 = 4;   // float4 per thread per block

__global__ __launch_bounds__(NT) void produce(const float4* __restrict__ x, float4* __restrict__ y,
                                              long n4) {
  const long base = (long)blockIdx.x * NT * V4;
  float4 v[V4];
#pragma unroll
  for (int k = 0; k < V4; ++k) {
    const long i = base + k * NT + threadIdx.x;
    v[k] = i < n4 ? x[i] : float4{0, 0, 0, 0};
  }
#pragma unroll
  for (int k = 0; k < V4; ++k) {
    const long i = base + k * NT + threadIdx.x;
    if (i < n4) y[i] = float4{v[k].x * 1.0001f, v[k].y * 1.0001f, v[k].z * 1.0001f, v[k].w * 1.0001f};
  }
}

template <bool REV>
__global__ __launch_bounds__(NT) void consume(const float4* __restrict__ y, const float4* __restrict__ w,
                                              float4* __restrict__ z, long n4) {
  const long b = REV ? (long)(gridDim.x - 1 - blockIdx.x) : (long)blockIdx.x;
  const long base = b * NT * V4;
  float4 a[V4], c[V4];
#pragma unroll
  for (int k = 0; k < V4; ++k) {
    const long i = base + k * NT + threadIdx.x;
    a[k] = i < n4 ? y[i] : float4{0, 0, 0, 0};
    c[k] = i < n4 ? w[i] : float4{0, 0, 0, 0};
  }
#pragma unroll
  for (int k = 0; k < V4; ++k) {
    const long i = base + k * NT + threadIdx.x;
    if (i < n4) z[i] = float4{a[k].x + c[k].x, a[k].y + c[k].y, a[k].z + c[k].z, a[k].w + c[k].w};
  }
}

template <bool REV>
__global__ __launch_bounds__(NT) void consume1(const float4* __restrict__ y, float4* __restrict__ z,
                                               long n4) {
  const long b = REV ? (long)(gridDim.x - 1 - blockIdx.x) : (long)blockIdx.x;
  const long base = b * NT * V4;
  float4 a[V4];
#pragma unroll
  for (int k = 0; k < V4; ++k) {
    const long i = base + k * NT + threadIdx.x;
    a[k] = i < n4 ? y[i] : float4{0, 0, 0, 0};
  }
#pragma unroll
  for (int k = 0; k < V4; ++k) {
    const long i = base + k * NT + threadIdx.x;
    if (i < n4) z[i] = float4{a[k].x + 1.f, a[k].y, a[k].z, a[k].w};
  }
}

// known-byte copies: 4-byte lanes (dword) and 16-byte lanes
__global__ __launch_bounds__(NT) void copy1(const float* __restrict__ x, float* __restrict__ y, long n) {
  const long base = (long)blockIdx.x * NT * 16;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const long i = base + k * NT + threadIdx.x;
    if (i < n) y[i] = x[i] + 1.f;
  }
}
__global__ __launch_bounds__(NT) void copy4(const float4* __restrict__ x, float4* __restrict__ y, long n4) {
  const long base = (long)blockIdx.x * NT * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long i = base + k * NT + threadIdx.x;
    if (i < n4) { float4 v = x[i]; v.x += 1.f; y[i] = v; }
  }
}

int main(int argc, char** argv) {
  const long NMAX = 61440000L;   // floats in one NTU bs=64 activation tensor (245.76 MB)
  float *x, *y, *w, *z;
  CK(hipMalloc(&x, NMAX * 4));
  CK(hipMalloc(&y, NMAX * 4));
  CK(hipMalloc(&w, NMAX * 4));
  CK(hipMalloc(&z, NMAX * 4));
  CK(hipMemset(x, 0, NMAX * 4));
  CK(hipMemset(w, 0, NMAX * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  if (argc > 2 && strcmp(argv[1], "calib") == 0) {
    const int lane = atoi(argv[2]);
    for (int r = 0; r < 3; ++r) {
      if (lane == 4) copy1<<<(NMAX + NT * 16 - 1) / (NT * 16), NT, 0, st>>>(x, y, NMAX);
      else copy4<<<(NMAX / 4 + NT * 4 - 1) / (NT * 4), NT, 0, st>>>((const float4*)x, (float4*)y, NMAX / 4);
    }
    CK(hipStreamSynchronize(st));
    printf("calib lane=%d bytes read %ld written %ld per launch\n", lane, NMAX * 4, NMAX * 4);
    return 0;
  }
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
  const long sizes[] = {NMAX, NMAX / 2, NMAX / 4, NMAX / 8};
  for (long n : sizes) {
    const long n4 = n / 4;
    const int grid = (int)((n4 + NT * V4 - 1) / (NT * V4));
    for (int mode = 0; mode < 4; ++mode) {
      float tp = 0, tc = 0;
      const int reps = 10;
      for (int r = 0; r < reps + 2; ++r) {
        // flush: a big unrelated write between iterations
        produce<<<(int)((NMAX / 4 + NT * V4 - 1) / (NT * V4)), NT, 0, st>>>((const float4*)w, (float4*)z, NMAX / 4);
        CK(hipEventRecord(e0, st));
        produce<<<grid, NT, 0, st>>>((const float4*)x, (float4*)y, n4);
        CK(hipEventRecord(e1, st));
        if (mode == 0) consume<false><<<grid, NT, 0, st>>>((const float4*)y, (const float4*)w, (float4*)z, n4);
        if (mode == 1) consume<true><<<grid, NT, 0, st>>>((const float4*)y, (const float4*)w, (float4*)z, n4);
        if (mode == 2) consume1<false><<<grid, NT, 0, st>>>((const float4*)y, (float4*)z, n4);
        if (mode == 3) consume1<true><<<grid, NT, 0, st>>>((const float4*)y, (float4*)z, n4);
        CK(hipEventRecord(e2, st));
        CK(hipEventSynchronize(e2));
        float a, b;
        CK(hipEventElapsedTime(&a, e0, e1));
        CK(hipEventElapsedTime(&b, e1, e2));
        if (r >= 2) { tp += a; tc += b; }
      }
      tp /= reps; tc /= reps;
      const double cb = (mode < 2 ? 3.0 : 2.0) * n * 4;
      printf("n=%9ld (%6.1f MB) %-22s producer %7.1f us (%5.2f TB/s)  consumer %7.1f us (%5.2f TB/s)\n",
             n, n * 4 / 1e6,
             mode == 0 ? "read Y+W fwd" : mode == 1 ? "read Y+W REVERSED" : mode == 2 ? "read Y fwd" : "read Y REVERSED",
             tp * 1e3, 2.0 * n * 4 / (tp * 1e-3) / 1e12, tc * 1e3, cb / (tc * 1e-3) / 1e12);
    }
  }
  CK(hipGetLastError());
  return 0;
}
