// Experiment (tuning harness; not part of the product library): the read-only weight gradient
// of the 64-wide layers, dW[m][c] = sum_p G(m, p) X(c, p) (+ dbias[m] = sum_p G(m, p)), with
// its operands streamed through an R-slot LDS ring by LDS-DMA (64-position chunks, R-1 in
// flight per workgroup, persistent workgroups over contiguous chunk ranges), against the
// product's register-staged pw_dw_kernel<64, 64>. The ring form sums in another order, so the
// comparison is relative (both against an fp64 reference on the host).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/dwdma.hip -o tools/bench/dwdma
#include "../../shift-gcn_amd/csrc/pwconv.hip"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace sgcn;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(size_t)(__attribute__((address_space(3))) const float*)p;
}
__device__ __forceinline__ void dma(i32x4 r, unsigned lds, unsigned voff, unsigned soff) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
               "buffer_load_dword %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(soff), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(N) : "memory");
}

// 8 waves: wave w owns the 32 x 32 output block ((w >> 1) & 1, w & 1) over the chunk half
// w >> 2 (positions 32 h .. 32 h + 31 of each 64-position chunk); the halves are added at the
// end (fixed order) and the workgroup's partial goes to slab[blockIdx] (S = gridDim.x).
// ACC2: two accumulators per wave (even / odd k pairs) for two independent MFMA chains
template <int R, bool BIAS, bool ACC2 = false>
__global__ __launch_bounds__(512) void pw_dw_ring_kernel(DwArgs p) {
  constexpr int CK_ = 64, PITCH = 65, ROWS = 128;   // G rows 0-63, X rows 64-127
  constexpr int SLOT = ROWS * PITCH;
  constexpr int DPW = ROWS / 8;                       // DMA per wave per chunk (16)
  static_assert(DPW * (R - 2) <= 63 && R >= 2, "ring");
  __shared__ float ring[R * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bm = (wid >> 1) & 1, bn = wid & 1, hk = wid >> 2;
  const int kl = lane >> 5, cl = lane & 31;
  const int V = p.V, T = p.T, N = T * V, P = p.B * N, M = p.M, Nc = p.Nc;
  const int nch = (P + CK_ - 1) / CK_;
  const int r = xcd_tile<SGCN_DW_XCD>(blockIdx.x, gridDim.x);
  const int q0 = (int)((long long)nch * r / gridDim.x), q1 = (int)((long long)nch * (r + 1) / gridDim.x);
  const int nq = q1 - q0;
  const i32x4 gr = rsrc4(p.g.ptr, p.g_bytes), xr = rsrc4(p.x.ptr, p.x_bytes);
  const unsigned r0 = lds_addr(ring);
  const unsigned gcs4 = (unsigned)(p.g.cstride * 4), xcs4 = (unsigned)(p.x.cstride * 4);
  // the lane's position in the chunk being fetched, advanced by 64 per chunk
  int pp = q0 * CK_ + lane;
  int b = pp / N, n = pp - (pp / N) * N;
  auto issue = [&](int g) {   // chunk q0 + g into slot g % R (past the range: zeros)
    unsigned go = p.g_bytes, xo = p.x_bytes;
    if (g < nq && pp < P) {
      const int t = n / V, v = n - (n / V) * V;
      go = (unsigned)(((long long)b * p.g.bstride + (long long)t * p.g.tstride * V + v) * 4);
      xo = (unsigned)(((long long)b * p.x.bstride + (long long)t * p.x.tstride * V + v) * 4);
    }
    const unsigned sl = r0 + (unsigned)((g % R) * SLOT * 4);
    // rows wid + 8 i: i < 8 are G rows, the rest X rows (offsets advanced, not unrolled: the
    // 16 precomputed row offsets would not fit the SGPRs)
    unsigned lds = sl + (unsigned)(wid * PITCH * 4), so = (unsigned)wid * gcs4;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
      dma(gr, lds, wid + 8 * i < M ? go : p.g_bytes, so);
      lds += 8 * PITCH * 4;
      so += 8 * gcs4;
    }
    so = (unsigned)wid * xcs4;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
      dma(xr, lds, wid + 8 * i < Nc ? xo : p.x_bytes, so);
      lds += 8 * PITCH * 4;
      so += 8 * xcs4;
    }
    pp += CK_;
    n += CK_;
    while (n >= N) { n -= N; ++b; }
  };
  f32x16 acc = f32x16{}, acc1 = f32x16{};
  float bsum = 0.f;   // BIAS: row tid >> 3 of G, positions 8 (tid & 7) .. + 7 of each chunk
#pragma unroll 1
  for (int g = 0; g < R - 1; ++g) issue(g);
#pragma unroll 1
  for (int g = 0; g < nq; ++g) {
    vm_barrier<DPW * (R - 2)>();
    issue(g + R - 1);
    const float* S = ring + (g % R) * SLOT;
    const float* Aw = S + (bm * 32 + cl) * PITCH + hk * 32 + kl;
    const float* Bw = S + (64 + bn * 32 + cl) * PITCH + hk * 32 + kl;
    float af[2], bf[2];
    af[0] = Aw[0];
    bf[0] = Bw[0];
#pragma unroll
    for (int kk = 0; kk < 32; kk += 2) {
      const int c2 = (kk >> 1) & 1;
      if (kk + 2 < 32) {
        af[c2 ^ 1] = Aw[kk + 2];
        bf[c2 ^ 1] = Bw[kk + 2];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (ACC2 && c2) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c2], bf[c2], acc1, 0, 0, 0);
      else acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c2], bf[c2], acc, 0, 0, 0);
    }
    if (BIAS) {
      const float* gb = S + (tid >> 3) * PITCH + 8 * (tid & 7);
#pragma unroll
      for (int e = 0; e < 8; ++e) bsum += gb[e];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (ACC2) acc += acc1;
  // fixed-order combine of the two chunk halves through LDS (slot 0)
  float* E = ring;
  if (hk == 1) {
#pragma unroll
    for (int i = 0; i < 16; ++i) E[((wid & 3) * 16 + i) * 64 + lane] = acc[i];
  }
  __syncthreads();
  float* slab = p.slab + (size_t)blockIdx.x * M * Nc;
  if (hk == 0) {
    const int c = bn * 32 + cl;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[i] + E[((wid & 3) * 16 + i) * 64 + lane];
      const int m = bm * 32 + (i & 3) + 8 * (i >> 2) + 4 * kl;
      if (m < M && c < Nc) slab[(size_t)m * Nc + c] = v;
    }
  }
  if (BIAS) {
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) bsum += __shfl_xor(bsum, o, 64);
    const int m = tid >> 3;
    if ((tid & 7) == 0 && m < M) p.bslab[(size_t)blockIdx.x * M + m] = bsum;
  }
}

template <int R, bool BIAS, bool ACC2 = false>
int launch_ring(DwArgs a, float* ws, int S, hipStream_t st) {
  a.slab = ws;
  a.bslab = BIAS ? ws + (size_t)S * a.M * a.Nc : nullptr;
  pw_dw_ring_kernel<R, BIAS, ACC2><<<S, 512, 0, st>>>(a);
  return S;
}

template <typename F>
float timeit(F&& launch, hipStream_t st, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1000.f / reps;
}

struct Shape { const char* name; int B, M, Nc, T, V; };

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 2;
  Shape shapes[] = {
    {"l2 tcn dW 64x64 T300", 128, 64, 64, 300, 25},
    {"mp tcn dW 64x64 T300", 64, 64, 64, 300, 33},
    {"ragged 50x37 T37 V7 B5", 5, 50, 37, 37, 7},
    {"ragged 64x64 T3 V5 B3", 3, 64, 64, 3, 5},
  };
  hipStream_t st; CK(hipStreamCreate(&st));
  const size_t maxe = (size_t)128 * 64 * 300 * 25;
  float *g, *x, *ws, *dw1, *dw2, *db1, *db2;
  CK(hipMalloc(&g, maxe * 4)); CK(hipMalloc(&x, maxe * 4)); CK(hipMalloc(&ws, 64 << 20));
  CK(hipMalloc(&dw1, 64 * 64 * 4)); CK(hipMalloc(&dw2, 64 * 64 * 4));
  CK(hipMalloc(&db1, 64 * 4)); CK(hipMalloc(&db2, 64 * 4));
  std::vector<float> h(maxe);
  for (size_t i = 0; i < maxe; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(g, h.data(), maxe * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(x, h.data() + 13, maxe * 4, hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  for (auto& s : shapes) {
    const int N = s.T * s.V;
    const double P = (double)s.B * N;
    const double fl = 2.0 * P * s.M * s.Nc, by = 4.0 * P * (s.M + s.Nc);
    const size_t wsb = sgcn_pw_dw_ws_bytes(s.B, s.M, s.Nc, s.T, s.V);
    auto prod = [&]() {
      if (sgcn_pw_dw(g, (long long)s.M * N, N, 1, 0, x, (long long)s.Nc * N, N, 1, 0, nullptr, dw1,
                     0, 0, db1, 0, ws, wsb, s.B, s.M, s.Nc, s.T, s.V, st)) {
        printf("sgcn_pw_dw failed\n");
        exit(1);
      }
    };
    DwArgs a{};
    a.g = {g, (long long)s.M * N, N, 1, 0};
    a.x = {x, (long long)s.Nc * N, N, 1, 0};
    a.M = s.M; a.Nc = s.Nc; a.T = s.T; a.V = s.V; a.B = s.B;
    a.g_bytes = plane_bytes(a.g.bstride, a.g.cstride, 1, s.B, s.M, s.T, s.V);
    a.x_bytes = plane_bytes(a.x.bstride, a.x.cstride, 1, s.B, s.Nc, s.T, s.V);
    // fp64 reference on the host for the small shapes, else the product as reference
    std::vector<double> ref(s.M * s.Nc, 0.0), rb(s.M, 0.0);
    const bool small = P < 100000;
    if (small) {
      std::vector<float> hg((size_t)s.B * s.M * N), hx((size_t)s.B * s.Nc * N);
      CK(hipMemcpy(hg.data(), g, hg.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hx.data(), x, hx.size() * 4, hipMemcpyDeviceToHost));
      for (int bb = 0; bb < s.B; ++bb)
        for (int m = 0; m < s.M; ++m)
          for (int nn = 0; nn < N; ++nn) {
            const double gv = hg[((size_t)bb * s.M + m) * N + nn];
            rb[m] += gv;
            for (int c = 0; c < s.Nc; ++c) ref[m * s.Nc + c] += gv * hx[((size_t)bb * s.Nc + c) * N + nn];
          }
    }
    auto err = [&](float* dw, float* db) {
      std::vector<float> o(s.M * s.Nc), ob(s.M);
      CK(hipMemcpy(o.data(), dw, o.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(ob.data(), db, ob.size() * 4, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (int i = 0; i < s.M * s.Nc; ++i) { md = fmax(md, fabs(o[i] - ref[i])); mx = fmax(mx, fabs(ref[i])); }
      for (int i = 0; i < s.M; ++i) { md = fmax(md, fabs(ob[i] - rb[i])); mx = fmax(mx, fabs(rb[i])); }
      return md / mx;
    };
    const int reps = s.B > 16 ? 30 : 5;
    for (int rr = 0; rr < rounds; ++rr) {
      float us = timeit(prod, st, reps);
      if (!small) {
        std::vector<float> o(s.M * s.Nc), ob(s.M);
        CK(hipMemcpy(o.data(), dw1, o.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ob.data(), db1, ob.size() * 4, hipMemcpyDeviceToHost));
        for (int i = 0; i < s.M * s.Nc; ++i) ref[i] = o[i];
        for (int i = 0; i < s.M; ++i) rb[i] = ob[i];
      }
      printf("%-26s %-22s %8.1f us  %6.1f TF/s  %6.2f TB/s  err %.2e\n", s.name, "product", us,
             fl / us / 1e6, by / us / 1e6, small ? err(dw1, db1) : 0.0);
#define RING(RR, G, NM) RING2(RR, G, false, NM)
#define RING2(RR, G, A2, NM)                                                                       \
  do {                                                                                        \
    const int S = (G) * cus;                                                                  \
    float u = timeit([&]() {                                                                  \
      launch_ring<RR, true, A2>(a, ws, S, st);                                                    \
      launch_slab_reduce(ws, ws + (size_t)S * s.M * s.Nc, S, s.M, s.Nc, dw2, 0, 0, db2, 0, st); \
    }, st, reps);                                                                             \
    printf("%-26s %-22s %8.1f us  %6.1f TF/s  %6.2f TB/s  err %.2e\n", s.name, NM, u,        \
           fl / u / 1e6, by / u / 1e6, err(dw2, db2));                                        \
  } while (0)
      RING(2, 2, "ring R2 2/CU");
      RING2(2, 2, true, "ring R2 2/CU acc2");
      RING(3, 1, "ring R3 1/CU");
      RING2(3, 1, true, "ring R3 1/CU acc2");
      RING2(4, 1, true, "ring R4 1/CU acc2");
    }
  }
  printf("done\n");
  return 0;
}
