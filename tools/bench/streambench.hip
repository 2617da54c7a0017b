// Streaming-primitive microbenchmark (tuning harness; not part of the product library): the
// rate at which one 122.9 MB operand (64 rows x 960k positions, fp32) can be read and a
// same-sized result written, per access primitive, to size the HBM-bound K = M = 64
// contraction's memory side (profiles/r05_dma/). Every kernel is a persistent grid of
// 512-thread workgroups walking 128/256-position tiles; the copy result is checked.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/streambench.hip -o tools/bench/streambench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 rsrc4(const void* p, unsigned bytes) {
  const unsigned long long a = (unsigned long long)p;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(size_t)(__attribute__((address_space(3))) const float*)p;
}
template <int W>
__device__ __forceinline__ void dma(i32x4 r, unsigned lds, unsigned voff, unsigned soff) {
  unsigned keep;
  if (W == 4)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(r), "s"(soff), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                 "buffer_load_dword %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(r), "s"(soff), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(N) : "memory");
}

// rows R = 64 of P positions, row stride P (one plane per row, the layout of one sample's
// channels stacked: enough for the access-pattern question)
struct Args { const float* x; float* y; int P; int ntiles; int N; };
// byte offset of position p's column: N = 0 -> rows of P positions (row stride P); else the
// model's (sample, channel, t, v) planes: sample stride 64 N, row (channel) stride N
__device__ __forceinline__ unsigned colb(const Args& a, int p) {
  if (a.N == 0) return (unsigned)p * 4u;
  const int b = p / a.N;
  return (unsigned)((b * 64 * a.N + (p - b * a.N)) * 4);
}
__device__ __forceinline__ unsigned rowb(const Args& a, int r) {
  return (unsigned)(r * (a.N ? a.N : a.P) * 4);
}

// (1) register loads, 16-row stages double-buffered in registers, plain stores (the
// product's memory pattern without the MFMA): each lane one column, W floats per access
template <int W, int BN, int POL = 0>
__global__ __launch_bounds__(512) void reg_copy(Args a) {
  const int tid = threadIdx.x;
  constexpr int LPR = BN / W;            // lanes per row
  constexpr int RPI = 512 / LPR;         // rows per pass
  const auto xr = mk(a.x, (unsigned)((size_t)a.P * 64 * 4));
  const auto yr = mk(a.y, (unsigned)((size_t)a.P * 64 * 4));
  const int c = (tid % LPR) * W, r0 = tid / LPR;
  for (int t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const unsigned col = colb(a, t * BN + c);
    if (W == 4) {
      f32x4 v[64 / RPI];
#pragma unroll
      for (int i = 0; i < 64 / RPI; ++i)
        v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, col, rowb(a, r0 + i * RPI), 0));
#pragma unroll
      for (int i = 0; i < 64 / RPI; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v[i]) , yr, col, rowb(a, r0 + i * RPI), POL);
    } else {
      float v[64 / RPI];
#pragma unroll
      for (int i = 0; i < 64 / RPI; ++i)
        v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, col, rowb(a, r0 + i * RPI), 0));
#pragma unroll
      for (int i = 0; i < 64 / RPI; ++i)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i]), yr, col, rowb(a, r0 + i * RPI), POL);
    }
  }
}

// (2) LDS-DMA ring: 16-row stages of BN positions into an R-slot ring (R-1 stages ahead),
// each stage read back from LDS and stored (dword stores, whole rows) — the ring kernel's
// memory side. W = 1: buffer_load_dword lds; W = 4: buffer_load_dwordx4 lds.
template <int W, int BN, int R>
__global__ __launch_bounds__(512) void dma_copy(Args a) {
  constexpr int SLOT = 16 * BN;
  constexpr int IPR = BN / (64 * W);                 // DMA instructions per row
  constexpr int IPS = 16 * IPR;                      // per stage
  constexpr int BPER = IPS / 8;                      // per wave per stage
  static_assert(BPER >= 1 && IPS % 8 == 0, "shape");
  constexpr int SPW = 16 * BN / 64 / 8;              // dword stores per wave per stage
  static_assert(BPER * (R - 2) + SPW * (R - 1) <= 63, "vmcnt");
  __shared__ float ring[R * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const i32x4 xr = rsrc4(a.x, (unsigned)((size_t)a.P * 64 * 4));
  const auto yr = mk(a.y, (unsigned)((size_t)a.P * 64 * 4));
  const unsigned r0 = lds_addr(ring);
  int nt = 0;
  for (int t = blockIdx.x; t < a.ntiles; t += gridDim.x) ++nt;
  const int nst = 4 * nt;
  auto issue = [&](int g) {
    const int t = blockIdx.x + (g >> 2) * gridDim.x, st = g & 3;
    const unsigned sl = r0 + (unsigned)((g % R) * SLOT * 4);
#pragma unroll
    for (int i = 0; i < BPER; ++i) {
      const int idx = wid + 8 * i, rs = idx / IPR, part = idx % IPR;
      const unsigned voff = g < nst ? colb(a, t * BN + part * 64 * W + lane * W) : 0xfffffff0u;
      dma<W>(xr, sl + (unsigned)((rs * BN + part * 64 * W) * 4), voff, rowb(a, st * 16 + rs));
    }
  };
  for (int g = 0; g < R - 1; ++g) issue(g);
  for (int g = 0; g < nst; ++g) {
    // younger: R-2 stages of DMA and the stores of the last R-1 iterations (fewer at the start)
    if (g >= R - 1) vm_barrier<BPER * (R - 2) + SPW * (R - 1)>();
    else {
      // the first iterations: fewer stores are younger; wait for everything (start-up only)
      vm_barrier<0>();
    }
    issue(g + R - 1);
    const int t = blockIdx.x + (g >> 2) * gridDim.x, st = g & 3;
    const float* S = ring + (g % R) * SLOT;
#pragma unroll
    for (int i = 0; i < SPW; ++i) {
      const int e = (wid + 8 * i) * 64 + lane;   // element of the 16 x BN stage
      const int rs = e / BN, c = e % BN;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(S[e]), yr, colb(a, t * BN + c),
                                            rowb(a, st * 16 + rs), 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// (0) reference: flat float4 grid-stride copy of the whole buffer
__global__ __launch_bounds__(512) void flat_copy(const f32x4* __restrict__ x, f32x4* __restrict__ y, size_t n4) {
  for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 512) y[i] = x[i];
}

// (3) read-only references (the weight gradient's memory side): flat float4 reads, and
// 64-row tiles of BN positions (dword per lane), each summed into one value per thread
__global__ __launch_bounds__(512) void flat_read(const f32x4* __restrict__ x, float* y, size_t n4) {
  f32x4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 512) acc += x[i];
  const float v = acc.x + acc.y + acc.z + acc.w;
  if (v == 1.2345f) y[0] = v;
}
template <int BN>
__global__ __launch_bounds__(512) void tile_read(Args a) {
  const int tid = threadIdx.x;
  constexpr int RPI = 512 / BN;
  const auto xr = mk(a.x, (unsigned)((size_t)a.P * 64 * 4));
  const int c = tid % BN, r0 = tid / BN;
  float acc = 0.f;
  for (int t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const unsigned col = colb(a, t * BN + c);
    float v[64 / RPI];
#pragma unroll
    for (int i = 0; i < 64 / RPI; ++i)
      v[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, col, rowb(a, r0 + i * RPI), 0));
#pragma unroll
    for (int i = 0; i < 64 / RPI; ++i) acc += v[i];
  }
  if (acc == 1.2345f) a.y[0] = acc;
}

// (4) flat copies with more in flight: U float4 per thread per iteration (all loads, then
// all stores), optionally non-temporal stores
template <int U, bool NT>
__global__ __launch_bounds__(512) void flat_copy_u(const f32x4* __restrict__ x, f32x4* __restrict__ y, size_t n4) {
  const size_t stride = (size_t)gridDim.x * 512 * U;
  for (size_t i0 = blockIdx.x * 512ull * U + threadIdx.x; i0 < n4; i0 += stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i0 + u * 512 < n4 ? x[i0 + u * 512] : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * 512 < n4) {
        if (NT) __builtin_nontemporal_store(v[u], &y[i0 + u * 512]);
        else y[i0 + u * 512] = v[u];
      }
  }
}
// (5) write-only stream (float4)
__global__ __launch_bounds__(512) void flat_fill(f32x4* __restrict__ y, size_t n4) {
  for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 512)
    y[i] = f32x4{1.f, 2.f, 3.f, 4.f};
}

template <typename F>
float timeit(F&& launch, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1000.f / reps;
}

int main() {
  const int P = 960000;
  const size_t n = (size_t)64 * P;
  float *x, *y;
  CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4));
  std::vector<float> h(n), g(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)(i % 1013);
  CK(hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice));
  const double by = 2.0 * n * 4;
  auto report = [&](const char* nm, float us) {
    CK(hipMemcpy(g.data(), y, n * 4, hipMemcpyDeviceToHost));
    const bool ok = memcmp(g.data(), h.data(), n * 4) == 0;
    printf("%-34s %8.1f us  %6.2f TB/s  %s\n", nm, us, by / us / 1e6, ok ? "ok" : "WRONG");
  };
  for (int rep = 0; rep < 2; ++rep) {
    const int NL = rep & 1 ? 7500 : 0;
    printf("layout: %s\n", NL ? "model planes (b, c, t, v), N = 7500" : "rows of 960k positions");
#define RUN(NM, K, BN, G)                                                                    \
  do {                                                                                       \
    CK(hipMemset(y, 0, n * 4));                                                              \
    Args a{x, y, P, P / (BN), NL};                                                               \
    float us = timeit([&]() { K<<<(G), 512>>>(a); }, 20);                                    \
    report(NM, us);                                                                          \
  } while (0)
    if (rep == 0) {
      CK(hipMemset(y, 0, n * 4));
      float us = timeit([&]() { flat_copy<<<2048, 512>>>((const f32x4*)x, (f32x4*)y, n / 4); }, 20);
      report("flat float4 copy g2048", us);
      us = timeit([&]() { flat_read<<<2048, 512>>>((const f32x4*)x, y, n / 4); }, 20);
      printf("%-34s %8.1f us  %6.2f TB/s  (read only)\n", "flat float4 read g2048", us, n * 4.0 / us / 1e6);
      us = timeit([&]() { flat_fill<<<2048, 512>>>((f32x4*)y, n / 4); }, 20);
      printf("%-34s %8.1f us  %6.2f TB/s  (write only)\n", "flat float4 fill g2048", us, n * 4.0 / us / 1e6);
      for (int gsz : {1024, 2048, 4096, 8192}) {
        char nm[64];
        CK(hipMemset(y, 0, n * 4));
        us = timeit([&]() { flat_copy_u<4, false><<<gsz, 512>>>((const f32x4*)x, (f32x4*)y, n / 4); }, 20);
        snprintf(nm, 64, "flat copy x4 g%d", gsz);
        report(nm, us);
        CK(hipMemset(y, 0, n * 4));
        us = timeit([&]() { flat_copy_u<4, true><<<gsz, 512>>>((const f32x4*)x, (f32x4*)y, n / 4); }, 20);
        snprintf(nm, 64, "flat copy x4 nt g%d", gsz);
        report(nm, us);
        CK(hipMemset(y, 0, n * 4));
        us = timeit([&]() { flat_copy_u<1, false><<<gsz, 512>>>((const f32x4*)x, (f32x4*)y, n / 4); }, 20);
        snprintf(nm, 64, "flat copy x1 g%d", gsz);
        report(nm, us);
      }
    }
    {
      Args a{x, y, P, P / 256, NL};
      float us = timeit([&]() { tile_read<256><<<2048, 512>>>(a); }, 20);
      printf("%-34s %8.1f us  %6.2f TB/s  (read only)\n", "tile read dword BN256 g2048", us, n * 4.0 / us / 1e6);
      us = timeit([&]() { tile_read<256><<<1024, 512>>>(a); }, 20);
      printf("%-34s %8.1f us  %6.2f TB/s  (read only)\n", "tile read dword BN256 g1024", us, n * 4.0 / us / 1e6);
    }
    RUN("reg dword BN256 g1024", (reg_copy<1, 256>), 256, 1024);
    RUN("reg dword nt BN256 g1024", (reg_copy<1, 256, 2>), 256, 1024);
    RUN("reg dword nt BN256 g2048", (reg_copy<1, 256, 2>), 256, 2048);
    RUN("reg dwordx4 nt BN256 g2048", (reg_copy<4, 256, 2>), 256, 2048);
    RUN("reg dword BN256 g2048", (reg_copy<1, 256>), 256, 2048);
    RUN("reg dwordx4 BN256 g1024", (reg_copy<4, 256>), 256, 1024);
    RUN("reg dwordx4 BN256 g2048", (reg_copy<4, 256>), 256, 2048);
    RUN("dma dword BN128 R8 g512", (dma_copy<1, 128, 8>), 128, 512);
    RUN("dma dword BN128 R4 g1024", (dma_copy<1, 128, 4>), 128, 1024);
    RUN("dma dwordx4 BN256 R4 g512", (dma_copy<4, 256, 4>), 256, 512);
    RUN("dma dwordx4 BN256 R6 g256", (dma_copy<4, 256, 6>), 256, 256);
  }
  printf("done\n");
  return 0;
}
