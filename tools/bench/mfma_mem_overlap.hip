// Does a v_mfma_f32_32x32x2_f32 wave overlap with a memory-streaming wave on the same SIMD
// (gfx950)? 512-thread workgroups, one per CU: waves 0-3 (one per SIMD) run four independent
// MFMA chains, waves 4-7 stream HBM with no VALU work: LDS-DMA reads (buffer_load ... lds),
// register reads (buffer_load, values folded once at the end), or stores of a constant.
// Modes: 0 = MFMA waves only, 1 = memory waves only, 2 = both. Tuning harness (not part of
// the product library); profiles/r05_dwr/.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/mfma_mem_overlap.hip -o tools/bench/mfma_mem_overlap
#include <hip/hip_runtime.h>

#include <cstdio>

using f32x16 = __attribute__((ext_vector_type(16))) float;
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 rsrc4(const void* p, unsigned bytes) {
  const unsigned long long a = (unsigned long long)p;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

// kind: 0 = LDS-DMA reads, 1 = register reads, 2 = stores
__global__ __launch_bounds__(512) void k(const float* src, float* dst, float* out, int mode,
                                         int kind, int iters, unsigned per_wave_bytes) {
  __shared__ float lds[4 * 16 * 64];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid < 4) {
    if (mode == 1) return;
    const float x = threadIdx.x * 0.001f, y = 1.0001f;
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
    return;
  }
  if (mode == 0) return;
  // this wave's contiguous byte range of the buffer, 256 B per wave-instruction
  const unsigned base = (unsigned)((blockIdx.x * 4 + (wid - 4))) * per_wave_bytes;
  const unsigned n = per_wave_bytes / 256;
  if (kind == 0) {
    const i32x4 r = rsrc4(src, 0xffffffffu);
    const unsigned l0 = (unsigned)(size_t)(__attribute__((address_space(3))) float*)lds +
                        (unsigned)((wid - 4) * 16 * 64 * 4);
    for (unsigned i = 0; i < n; i += 16) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                     "buffer_load_dword %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"((unsigned)lane * 4u), "s"(r), "s"(base + (i + u) * 256u),
                       "s"(l0 + (unsigned)(u * 256))
                     : "memory");
      }
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (kind == 1) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, -1, 0x00020000);
    unsigned acc = 0;
    for (unsigned i = 0; i < n; i += 16) {
      unsigned v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        v[u] = __builtin_amdgcn_raw_buffer_load_b32(r, (unsigned)lane * 4u, base + (i + u) * 256u, 0);
#pragma unroll
      for (int u = 0; u < 16; ++u) acc ^= v[u];   // one VALU per 256-B load
    }
    if (acc == 0x12345678u) out[0] = 1.f;
  } else if (kind == 5) {
    // register reads, 16 B per lane (buffer_load_dwordx4): a quarter of kind 1's instructions
    // for the same bytes
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, -1, 0x00020000);
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    u4 acc = {0, 0, 0, 0};
    for (unsigned i = 0; i < n; i += 16) {
      u4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)lane * 16u, base + (i + 4 * u) * 256u, 0));
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= v[u];
    }
    if (acc.x == 0x12345678u) out[0] = 1.f;
  } else if (kind == 3 || kind == 4) {   // per 16-step: 16 (b32) / 4 (b128) instructions
    // LDS -> VGPR reads (ds_read_b32 / ds_read_b128), as many instructions as kind 1's loads
    // x 4 (b32) or x 1 (b128); values kept live by an empty asm (no VALU)
    float* L = lds + (wid - 4) * 16 * 64;
    for (unsigned i = 0; i < n; i += 16) {
      if (kind == 3) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = L[(u * 64 + lane + i) & 1023];
        asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]),
                     "v"(v[6]), "v"(v[7]), "v"(v[8]), "v"(v[9]), "v"(v[10]), "v"(v[11]),
                     "v"(v[12]), "v"(v[13]), "v"(v[14]), "v"(v[15]));
      } else {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4* L4 = reinterpret_cast<const f4*>(L);
        f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = L4[(u * 64 + lane + i) & 255];
        asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
      }
    }
  } else {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, -1, 0x00020000);
    const unsigned v = (unsigned)lane;
    for (unsigned i = 0; i < n; i += 16) {
#pragma unroll
      for (int u = 0; u < 16; ++u)
        __builtin_amdgcn_raw_buffer_store_b32(v, r, (unsigned)lane * 4u, base + (i + u) * 256u, 0);
    }
  }
}

int main() {
  const unsigned per_wave = 1u << 20;   // 1 MiB per memory wave: 1 GiB per launch
  float *src, *dst, *out;
  hipMalloc(&src, (size_t)256 * 4 * per_wave);
  hipMalloc(&dst, (size_t)256 * 4 * per_wave);
  hipMalloc(&out, 256 * 512 * 4);
  hipMemset(src, 0, (size_t)256 * 4 * per_wave);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* kn[] = {"LDS-DMA reads", "register reads", "stores", "ds_read_b32", "ds_read_b128",
                      "reg reads x4"};
  for (int rep = 0; rep < 2; ++rep)
    for (int kind : {1, 5})
      for (int iters : {1500, 3000})
        for (int mode = 0; mode < 3; ++mode) {
          if (mode == 1 && iters != 1500) continue;
          k<<<256, 512>>>(src, dst, out, mode, kind, iters, per_wave);
          hipDeviceSynchronize();
          hipEventRecord(e0);
          k<<<256, 512>>>(src, dst, out, mode, kind, iters, per_wave);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms;
          hipEventElapsedTime(&ms, e0, e1);
          printf("%-15s iters %5d %-10s %8.1f us  (memory %.2f TB/s if alone)\n", kn[kind], iters,
                 mode == 0 ? "mfma-only" : mode == 1 ? "mem-only" : "both", ms * 1e3,
                 256.0 * 4 * per_wave / (ms * 1e-3) / 1e12);
        }
  return 0;
}
