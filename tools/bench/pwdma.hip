// Experiment (tuning harness; not part of the product library): the HBM-bound K, M <= 64
// forward contraction with its WHOLE operand tile fetched by LDS-DMA (buffer_load ... lds)
// at the start of the tile — every stage's X loads in flight at once, no VGPR staging —
// against the product's register-staged pwg_fwd_kernel. Bit-exact comparison with the
// product output (same MFMA, same k order).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/pwdma.hip -o tools/bench/pwdma
#include "../../shift-gcn_amd/csrc/pwconv.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace sgcn;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));

// a buffer descriptor in SGPRs for inline asm (same fields as make_rsrc)
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
// one wave-instruction of LDS-DMA: lane l's dword (voff + soff, 0 past the range) to LDS byte
// lds + 4 l. Inline asm, so the compiler adds no vmcnt(0) of its own before LDS reads (it
// cannot tell which LDS a DMA writes); completion is counted by hand (vm_barrier).
__device__ __forceinline__ void dma(i32x4 r, unsigned lds, unsigned voff, unsigned soff) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
               "buffer_load_dword %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(soff), "s"(lds) : "memory");
}
// this wave's DMA but the last N landed, then the workgroup barrier
template <int N>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(N) : "memory");
}

// BN positions x 64 rows per tile, 4 waves (2 x 2), A (<= 64 x 64) and the whole K <= 64 x
// BN operand tile in LDS, fetched by DMA: A first, then the B rows stage by stage (16 rows
// a stage); the MFMAs of stage s start once stage s has landed (counted vmcnt + barrier).
// WAITS = false: one vmcnt(0) + barrier for everything (the simple form).
template <int BN, bool AMC, bool WAITS>
__global__ __launch_bounds__(256) void pwd_kernel(FwdArgs p) {
  constexpr int BM = 64, KM = 64, WN = 2;
  constexpr int NJ = BN / WN / 32;
  constexpr int CH = BN / 64;          // 64-column chunks of a B row
  constexpr int AP = AMC ? 64 : 65;    // LDS A: AMC [k][m] (pitch 64), else [m][k] (pitch 65)
  constexpr int BPER = 4 * CH;         // B DMA per wave per 16-row stage
  static_assert(CH == 1 || CH == 2 || CH == 4, "chunks");
  __shared__ float As[KM * 65];
  __shared__ float Bs[KM * BN];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int V = p.V, N = p.T * V, K = p.K, M = p.M;
  const int P = p.B * N;
  const int p0 = xcd_tile<SGCN_PW_XCD>(blockIdx.x, gridDim.x) * BN;
  const i32x4 xr = rsrc4(p.x.ptr, p.x_bytes);
  const i32x4 ar = rsrc4(p.A, p.a_bytes);
  const unsigned as0 = lds_addr(As), bs0 = lds_addr(Bs);
  const auto yr = make_rsrc(p.y.ptr, p.y_bytes);
  // this wave's B chunk (fixed: (w + 4 i) mod CH = w mod CH) and the lane's column in it
  const int ch = wid % CH;
  unsigned xcol = p.x_bytes;
  {
    const int pc = p0 + ch * 64 + lane;
    if (pc < P) {
      const int b = fdiv(pc, p.divN_m, p.divN_s), n = pc - b * N;
      const int t = fdiv(n, p.divV_m, p.divV_s), v = n - t * V;
      xcol = ((unsigned)b * (unsigned)p.x.bstride + (unsigned)t * (unsigned)(p.x.tstride * V) +
              (unsigned)v) * 4u;
    }
  }
  const unsigned xcs4 = (unsigned)(p.x.cstride * 4);
  // ---- A: 64 rows (AMC: k rows of M; else m rows of K), 16 per wave, lane = column ----
  {
    const int ncol = AMC ? M : K, nrow = AMC ? K : M;
    const unsigned acol = lane < ncol ? (unsigned)lane * 4u : p.a_bytes;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = wid + 4 * i;
      dma(ar, as0 + (unsigned)(r * AP * 4), r < nrow ? acol : p.a_bytes, (unsigned)(r * p.lda * 4));
    }
  }
  // ---- B: the whole K x BN tile, stage by stage ----
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < BPER; ++i) {
      const int row = s * 16 + (wid + 4 * i) / CH;
      dma(xr, bs0 + (unsigned)((row * BN + ch * 64) * 4), row < K ? xcol : p.x_bytes,
          (unsigned)row * xcs4);
    }
  f32x16 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x16{};
  const int kl = lane >> 5, cl = lane & 31;
  const int nstage = (K + 15) / 16;
  auto stage = [&](int s) {
    const float* Aw = AMC ? As + (s * 16 + kl) * AP + wm * 32 + cl
                          : As + (wm * 32 + cl) * AP + s * 16 + kl;
    const float* Bw = Bs + (s * 16 + kl) * BN + wn * (BN / 2) + cl;
    float af[2], bf[2][NJ];
    af[0] = Aw[0];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[0][j] = Bw[j * 32];
#pragma unroll
    for (int kk = 0; kk < 16; kk += 2) {
      const int c2 = (kk >> 1) & 1;
      if (kk + 2 < 16) {
        af[c2 ^ 1] = AMC ? Aw[(kk + 2) * AP] : Aw[kk + 2];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bf[c2 ^ 1][j] = Bw[(kk + 2) * BN + j * 32];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c2], bf[c2][j], acc[j], 0, 0, 0);
    }
  };
  if (WAITS) {
    vm_barrier<3 * BPER>();
    stage(0);
    if (nstage > 1) {
      vm_barrier<2 * BPER>();
      stage(1);
    }
    if (nstage > 2) {
      vm_barrier<BPER>();
      stage(2);
    }
    vm_barrier<0>();
    if (nstage > 3) stage(3);
  } else {
    vm_barrier<0>();
    for (int s = 0; s < nstage; ++s) stage(s);
  }
  __syncthreads();
  // ---- epilogue: the 64 x BN tile staged in Bs, then whole rows stored ----
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
      Bs[row * BN + wn * (BN / 2) + j * 32 + cl] = acc[j][r];
    }
  __syncthreads();
  unsigned ycol[CH];
#pragma unroll
  for (int q = 0; q < CH; ++q) {
    const int pc = p0 + q * 64 + lane;
    ycol[q] = p.y_bytes;
    if (pc < P) {
      const int b = fdiv(pc, p.divN_m, p.divN_s), n = pc - b * N;
      const int t = fdiv(n, p.divV_m, p.divV_s), v = n - t * V;
      ycol[q] = ((unsigned)b * (unsigned)p.y.bstride + (unsigned)t * (unsigned)(p.y.tstride * V) +
                 (unsigned)v) * 4u;
    }
  }
  const unsigned ycs4 = (unsigned)(p.y.cstride * 4);
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int row = wid + 4 * k;
    if (row >= M) break;
    const float bv = p.bias ? p.bias[row] : 0.f;
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      float val = Bs[row * BN + q * 64 + lane] + bv;
      if (p.relu) val = fmaxf(val, 0.f);
      bstore(yr, val, ycol[q], (unsigned)row * ycs4);
    }
  }
}

template <int BN, bool AMC, bool WAITS>
void launch_pwd(const FwdArgs& a, hipStream_t st) {
  const int P = a.B * a.T * a.V;
  pwd_kernel<BN, AMC, WAITS><<<(P + BN - 1) / BN, 256, 0, st>>>(a);
}

struct Shape { const char* name; int B, M, K, T, V; int amc; };

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

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  Shape shapes[] = {
    {"l2 tcn 64x64 T300", 128, 64, 64, 300, 25, 0},
    {"l2 tcn dX 64x64 T300", 128, 64, 64, 300, 25, 1},
    {"l1 tcn 64x64 T300 K48", 128, 64, 48, 300, 25, 0},
    {"ragged 64x40 T37 V7 B5", 5, 40, 37, 37, 7, 0},
    {"ragged 50x64 T37 V7 B5 mc", 5, 50, 64, 37, 7, 1},
  };
  hipStream_t st; CK(hipStreamCreate(&st));
  const size_t maxe = (size_t)128 * 64 * 300 * 25;
  float *x, *y1, *y2, *w;
  CK(hipMalloc(&x, maxe * 4)); CK(hipMalloc(&y1, maxe * 4)); CK(hipMalloc(&y2, maxe * 4));
  CK(hipMalloc(&w, 64 * 64 * 4));
  std::vector<float> h(maxe);
  for (size_t i = 0; i < maxe; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(x, h.data(), maxe * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data() + 11, 64 * 64 * 4, hipMemcpyHostToDevice));
  std::vector<float> g1(maxe), g2(maxe);
  for (auto& s : shapes) {
    const int N = s.T * s.V;
    const double P = (double)s.B * N;
    const double by = 4.0 * P * (s.M + s.K);
    const size_t ny = (size_t)s.B * s.M * N;
    auto prod = [&]() {
      if (sgcn_pw_fwd(w, s.amc, nullptr, x, (long long)s.K * N, N, 1, 0, nullptr, y1,
                      (long long)s.M * N, N, 1, 0, 0, 0, s.B, s.M, s.K, s.T, s.V, st)) {
        printf("sgcn_pw_fwd failed\n");
        exit(1);
      }
    };
    FwdArgs a{};
    a.A = w; a.lda = s.amc ? s.M : s.K; a.a_mcontig = s.amc; a.bias = nullptr;
    a.x = {x, (long long)s.K * N, N, 1, 0};
    a.y = {y2, (long long)s.M * N, N, 1, 0};
    a.M = s.M; a.K = s.K; a.T = s.T; a.V = s.V; a.B = s.B;
    fwd_divisors(a);
    a.x_bytes = plane_bytes(a.x.bstride, a.x.cstride, 1, s.B, s.K, s.T, s.V);
    a.y_bytes = plane_bytes(a.y.bstride, a.y.cstride, 1, s.B, s.M, s.T, s.V);
    a.a_bytes = (unsigned)(s.M * s.K * 4);
    auto check = [&](const char* nm, float us) {
      CK(hipMemcpy(g1.data(), y1, ny * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(g2.data(), y2, ny * 4, hipMemcpyDeviceToHost));
      const bool ok = memcmp(g1.data(), g2.data(), ny * 4) == 0;
      printf("%-28s %-22s %8.1f us  %6.2f TB/s  %s\n", s.name, nm, us, by / us / 1e6,
             ok ? "bit-exact" : "MISMATCH");
    };
    const int reps = s.B > 16 ? 50 : 5;
    for (int r = 0; r < rounds; ++r) {
      CK(hipMemset(y2, 0xff, ny * 4));
      float us = timeit(prod, st, reps);
      printf("%-28s %-22s %8.1f us  %6.2f TB/s\n", s.name, "product", us, by / us / 1e6);
#define V_(BN, W, NM)                                                                       \
  do {                                                                                      \
    CK(hipMemset(y2, 0xff, ny * 4));                                                        \
    float u = s.amc ? timeit([&]() { launch_pwd<BN, true, W>(a, st); }, st, reps)           \
                    : timeit([&]() { launch_pwd<BN, false, W>(a, st); }, st, reps);         \
    check(NM, u);                                                                           \
  } while (0)
      V_(128, true, "dma 128 staged");
      V_(128, false, "dma 128 one-wait");
      V_(64, true, "dma 64 staged");
      V_(256, true, "dma 256 staged");
    }
  }
  printf("done\n");
  return 0;
}
