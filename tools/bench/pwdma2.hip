// Experiment (tuning harness; not part of the product library): the MFMA-bound forward
// contraction tile (256 x 128, 8 waves, BK = 16 double-buffered LDS stages) with BOTH operands
// staged by LDS-DMA (buffer_load ... lds from inline asm) instead of global -> VGPR -> LDS.
// Why (profiles/r05_dwr/mfma_mem_overlap.txt, mfma_lds_overlap.txt): on gfx950 a wave's
// VGPR-returning loads (global or LDS) do not overlap another wave's v_mfma_f32_32x32x2_f32
// on the same SIMD (both = the sum of the two alone), while LDS-DMA reads and stores do.
// Same MFMA sequence as the product (bit-exact expected for K % 16 == 0).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/pwdma2.hip -o tools/bench/pwdma2
#include "../../shift-gcn_amd/csrc/pwconv.hip"
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
__device__ __forceinline__ void vm0_barrier() {
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int BM, int BN, int WM, int WN, bool AMC, bool ADMA>
__global__ __launch_bounds__(64 * WM * WN) void pwd2_kernel(FwdArgs p) {
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int BK = 16;
  constexpr int MI = BM / WM / 32, NJ = BN / WN / 32;
  constexpr int AP = BM + 1, BP = BN + 1;
  constexpr int ASZ = 2 * BK * AP, BSZ = 2 * BK * BP;
  constexpr int BQ = BN / 64, AQ = BM / 64;          // 64-lane DMA pieces per row
  constexpr int B_DMA = BK * BQ / NW, A_DMA = BK * AQ / NW;   // per wave per stage
  static_assert(B_DMA >= 1 && A_DMA >= 1 && (BK * BQ) % NW == 0 && (BK * AQ) % NW == 0, "tile");
  __shared__ float smem[ASZ + BSZ];
  __shared__ float bias_s[BM];
  float* As = smem;
  float* Bs = smem + ASZ;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int V = p.V, N = p.T * V, K = p.K, M = p.M;
  const int P = p.B * N;
  const int p0 = xcd_tile<SGCN_PW_XCD>(blockIdx.x, gridDim.x) * BN;
  const int m0 = blockIdx.y * BM;
  const i32x4 xr = rsrc4(p.x.ptr, p.x_bytes), ar = rsrc4(p.A, p.a_bytes);
  const auto yr = make_rsrc(p.y.ptr, p.y_bytes);
  const unsigned as0 = lds_addr(As), bs0 = lds_addr(Bs);
  for (int i = tid; i < BM; i += NT) bias_s[i] = (p.bias && m0 + i < M) ? p.bias[m0 + i] : 0.f;
  // per lane: the operand / output column of each 64-column piece of the tile
  unsigned xcol[BQ], ycol[BQ];
#pragma unroll
  for (int q = 0; q < BQ; ++q) {
    const int pc = p0 + q * 64 + lane;
    xcol[q] = p.x_bytes;
    ycol[q] = p.y_bytes;
    if (pc < P) {
      const int b = fdiv(pc, p.divN_m, p.divN_s), n = pc - b * N;
      const int t = fdiv(n, p.divV_m, p.divV_s), v = n - t * V;
      xcol[q] = ((unsigned)b * (unsigned)p.x.bstride + (unsigned)t * (unsigned)(p.x.tstride * V) + (unsigned)v) * 4u;
      ycol[q] = ((unsigned)b * (unsigned)p.y.bstride + (unsigned)t * (unsigned)(p.y.tstride * V) + (unsigned)v) * 4u;
    }
  }
  // per lane: the weight element of each 64-row piece (AMC: W^T[k][m], else W[m][k])
  unsigned acol[AQ];
#pragma unroll
  for (int q = 0; q < AQ; ++q) {
    const int m = m0 + q * 64 + lane;
    acol[q] = m < M ? (unsigned)((AMC ? m : m * p.lda) * 4) : p.a_bytes;
  }
  const unsigned xcs4 = (unsigned)(p.x.cstride * 4);
  // a wave's DMA always take the same 64-column / 64-row piece (NW is a multiple of BQ, AQ)
  static_assert(NW % BQ == 0 && NW % AQ == 0, "pieces");
  unsigned xq = xcol[0], aq = acol[0];
#pragma unroll
  for (int q = 1; q < BQ; ++q) xq = wid % BQ == q ? xcol[q] : xq;
#pragma unroll
  for (int q = 1; q < AQ; ++q) aq = wid % AQ == q ? acol[q] : aq;
  // stage k0 into buffer buf: B rows k0..k0+15 (64 columns per DMA), A rows k (64 m per DMA)
  // A through registers (!ADMA): the product's thread map (AMC: m = tid % BM; else k-contiguous)
  constexpr int A_PER = BM * BK / NT;
  const int lda = p.lda;
  const int am = AMC ? tid % BM : tid / BK, ak = AMC ? tid / BM : tid % BK;
  const unsigned avoff = AMC ? (m0 + am < M ? (unsigned)((ak * lda + m0 + am) * 4) : p.a_bytes)
                             : (unsigned)(((m0 + am) * lda + ak) * 4);
  const unsigned astep = AMC ? (unsigned)((NT / BM) * lda * 4) : (unsigned)((NT / BK) * lda * 4);
  const auto arr = make_rsrc(p.A, p.a_bytes);
  float ra[ADMA ? 1 : A_PER];
  auto load_a = [&](int k0) {
    if (ADMA) return;
    const unsigned ak0 = AMC ? (unsigned)(k0 * lda * 4) : (unsigned)(k0 * 4);
#pragma unroll
    for (int i = 0; i < A_PER; ++i)
      ra[i] = bload(arr, AMC ? avoff : (k0 + ak < K ? avoff : p.a_bytes), ak0 + (unsigned)i * astep);
  };
  auto store_a = [&](int buf) {
    if (ADMA) return;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int m = AMC ? am : am + i * (NT / BK);
      const int k = AMC ? ak + i * (NT / BM) : ak;
      As[buf * BK * AP + k * AP + m] = ra[i];
    }
  };
  auto issue = [&](int k0, int buf) {
#pragma unroll
    for (int i = 0; i < B_DMA; ++i) {
      const int idx = wid + NW * i, k = idx / BQ, q = idx % BQ;   // uniform
      const bool ok = k0 + k < K;
      dma(xr, bs0 + (unsigned)((buf * BK * BP + k * BP + q * 64) * 4), ok ? xq : p.x_bytes,
          (unsigned)(k0 + k) * xcs4);
    }
#pragma unroll
    for (int i = 0; i < (ADMA ? A_DMA : 0); ++i) {
      const int idx = wid + NW * i, k = idx / AQ, q = idx % AQ;
      const bool ok = k0 + k < K;
      dma(ar, as0 + (unsigned)((buf * BK * AP + k * AP + q * 64) * 4), ok ? aq : p.a_bytes,
          (unsigned)((AMC ? (k0 + k) * p.lda : (k0 + k)) * 4));
    }
  };
  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};
  const int kl = lane >> 5, cl = lane & 31;
  const int nstage = (K + BK - 1) / BK;
  issue(0, 0);
  load_a(0);
  store_a(0);
  vm0_barrier();
  for (int s = 0; s < nstage; ++s) {
    const int cur = s & 1;
    if (s + 1 < nstage) {
      issue((s + 1) * BK, cur ^ 1);
      load_a((s + 1) * BK);
    }
    const float* __restrict__ Aw = As + cur * BK * AP + kl * AP + wm * (BM / WM) + cl;
    const float* __restrict__ Bw = Bs + cur * BK * BP + kl * BP + wn * (BN / WN) + cl;
    float af[2][MI], bf[2][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) af[0][i] = Aw[i * 32];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[0][j] = Bw[j * 32];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int c2 = (kk >> 1) & 1;
      if (kk + 2 < BK) {
#pragma unroll
        for (int i = 0; i < MI; ++i) af[c2 ^ 1][i] = Aw[(kk + 2) * AP + i * 32];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bf[c2 ^ 1][j] = Bw[(kk + 2) * BP + j * 32];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c2][i], bf[c2][j], acc[i][j], 0, 0, 0);
    }
    if (s + 1 < nstage) store_a(cur ^ 1);
    vm0_barrier();   // stage s+1 landed (this wave's DMA) and every wave done with stage s
  }
  // epilogue (the product's LDS-staged whole-row stores, no rotation / accumulate)
  const unsigned ycs4 = (unsigned)(p.y.cstride * 4);
  constexpr int RB = WM * 16, RPW = RB / NW;
  static_assert(RB * BN <= ASZ + BSZ && RB % NW == 0, "epilogue staging");
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const int r = 8 * h + rr;
          const int lr = wm * 16 + (r & 3) + 8 * ((r >> 2) & 1) + 4 * kl;
          smem[lr * BN + wn * (BN / WN) + j * 32 + cl] = acc[i][j][r];
        }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int lr = wid + k * NW;
        const int trow = (lr >> 4) * (BM / WM) + i * 32 + 16 * h + (lr & 15);
        if (m0 + trow >= M) break;
        const float bv = bias_s[trow];
        const unsigned soff = (unsigned)(m0 + trow) * ycs4;
#pragma unroll
        for (int q = 0; q < BQ; ++q) {
          float val = smem[lr * BN + lane + 64 * q] + bv;
          if (p.relu) val = fmaxf(val, 0.f);
          bstore(yr, val, ycol[q], soff);
        }
      }
      __syncthreads();
    }
}

template <int BM, int BN, int WM, int WN, bool ADMA = true>
void launch_pwd2(const FwdArgs& a, hipStream_t st) {
  const long long P = (long long)a.B * a.T * a.V;
  dim3 grid((unsigned)((P + BN - 1) / BN), (a.M + BM - 1) / BM);
  if (a.a_mcontig) pwd2_kernel<BM, BN, WM, WN, true, ADMA><<<grid, 64 * WM * WN, 0, st>>>(a);
  else pwd2_kernel<BM, BN, WM, WN, false, ADMA><<<grid, 64 * WM * WN, 0, st>>>(a);
}

// ---- pwd3: DMA staging into a k-interleaved, chunk-swizzled LDS image read by ds_read_b128 --
// Row r of a stage image (r = m for A, r = position n for B) holds the stage's 16 k values as
// four 16-byte chunks; logical chunk c = 2 kl + kq holds k = 2 (4 kq + u) + kl, u = 0..3, i.e.
// the MFMA operand of lane (r, kl) for the four k-steps 4 kq .. 4 kq + 3; it is stored at
// physical chunk c ^ ((r >> 2) & 3) (conflict-free b128 reads). One DMA instruction fills four
// rows (64 dwords): lane l -> row 4 idx + l / 16, physical slot l % 16. So per four k-steps a
// wave issues MI + NJ ds_read_b128 for 4 MI NJ MFMAs (instead of 4 (MI + NJ) ds_read_b32).
template <int BM, int BN, int WM, int WN, bool AMC>
__global__ __launch_bounds__(64 * WM * WN) void pwd3_kernel(FwdArgs p) {
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int BK = 16;
  constexpr int MI = BM / WM / 32, NJ = BN / WN / 32;
  constexpr int ASZ = BM * BK, BSZ = BN * BK;            // one stage image
  constexpr int A_DMA = BM / 4 / NW, B_DMA = BN / 4 / NW;   // per wave per stage
  static_assert(A_DMA >= 1 && B_DMA >= 1 && (BM / 4) % NW == 0 && (BN / 4) % NW == 0, "tile");
  __shared__ float smem[2 * (ASZ + BSZ)];
  __shared__ float bias_s[BM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int V = p.V, N = p.T * V, K = p.K, M = p.M;
  const int P = p.B * N;
  const int p0 = xcd_tile<SGCN_PW_XCD>(blockIdx.x, gridDim.x) * BN;
  const int m0 = blockIdx.y * BM;
  const i32x4 xr = rsrc4(p.x.ptr, p.x_bytes), ar = rsrc4(p.A, p.a_bytes);
  const auto yr = make_rsrc(p.y.ptr, p.y_bytes);
  const unsigned sm0 = lds_addr(smem);
  for (int i = tid; i < BM; i += NT) bias_s[i] = (p.bias && m0 + i < M) ? p.bias[m0 + i] : 0.f;
  const unsigned xcs4 = (unsigned)(p.x.cstride * 4);
  const int lda = p.lda;
  // this lane's logical k within a stage for a DMA instruction whose rows r have (r>>2)&3 = sw
  auto klane = [&](int sw) {
    const int c = ((lane & 15) >> 2) ^ sw, u = lane & 3;
    return 2 * (4 * (c & 1) + u) + (c >> 1);
  };
  // per-instruction lane offsets (fixed for the tile; the stage adds a uniform soffset)
  unsigned boff[B_DMA], aoff[A_DMA];
  int bk[B_DMA], ak[A_DMA];
#pragma unroll
  for (int i = 0; i < B_DMA; ++i) {
    const int idx = wid + NW * i, n = 4 * idx + (lane >> 4), k = klane(idx & 3);
    const int pc = p0 + n;
    bk[i] = k;
    boff[i] = p.x_bytes;
    if (pc < P) {
      const int b = fdiv(pc, p.divN_m, p.divN_s), nn = pc - b * N;
      const int t = fdiv(nn, p.divV_m, p.divV_s), v = nn - t * V;
      boff[i] = ((unsigned)b * (unsigned)p.x.bstride + (unsigned)t * (unsigned)(p.x.tstride * V) +
                 (unsigned)v) * 4u + (unsigned)k * xcs4;
    }
  }
#pragma unroll
  for (int i = 0; i < A_DMA; ++i) {
    const int idx = wid + NW * i, m = m0 + 4 * idx + (lane >> 4), k = klane(idx & 3);
    ak[i] = k;
    aoff[i] = m < M ? (unsigned)((AMC ? k * lda + m : m * lda + k) * 4) : p.a_bytes;
  }
  auto issue = [&](int k0, int buf) {
    const bool full = k0 + BK <= K;
    const unsigned bbase = sm0 + (unsigned)(buf * (ASZ + BSZ) * 4);
#pragma unroll
    for (int i = 0; i < A_DMA; ++i) {
      const int idx = wid + NW * i;
      const unsigned vo = full || k0 + ak[i] < K ? aoff[i] : p.a_bytes;
      dma(ar, bbase + (unsigned)(idx * 64 * 4), vo, (unsigned)((AMC ? k0 * lda : k0) * 4));
    }
#pragma unroll
    for (int i = 0; i < B_DMA; ++i) {
      const int idx = wid + NW * i;
      const unsigned vo = full || k0 + bk[i] < K ? boff[i] : p.x_bytes;
      dma(xr, bbase + (unsigned)((ASZ + idx * 64) * 4), vo, (unsigned)k0 * xcs4);
    }
  };
  // fragment read offsets (floats within a stage image) for kq = 0, 1
  const int kl = lane >> 5, cl = lane & 31;
  int aro[2][MI], bro[2][NJ];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int r = wm * (BM / WM) + i * 32 + cl;
      aro[q][i] = r * 16 + (((2 * kl + q) ^ ((r >> 2) & 3)) * 4);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = wn * (BN / WN) + j * 32 + cl;
      bro[q][j] = ASZ + r * 16 + (((2 * kl + q) ^ ((r >> 2) & 3)) * 4);
    }
  }
  typedef float f4 __attribute__((ext_vector_type(4)));
  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};
  const int nstage = (K + BK - 1) / BK;
  issue(0, 0);
  vm0_barrier();
  for (int s = 0; s < nstage; ++s) {
    const int cur = s & 1;
    if (s + 1 < nstage) issue((s + 1) * BK, cur ^ 1);
    const float* img = smem + cur * (ASZ + BSZ);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      f4 af[MI], bf[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const f4*>(img + aro[q][i]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[j] = *reinterpret_cast<const f4*>(img + bro[q][j]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][u], bf[j][u], acc[i][j], 0, 0, 0);
    }
    vm0_barrier();
  }
  const unsigned ycs4 = (unsigned)(p.y.cstride * 4);
  constexpr int RB = WM * 16, RPW = RB / NW, BQ = BN / 64;
  static_assert(RB * BN <= 2 * (ASZ + BSZ) && RB % NW == 0 && BN % 64 == 0, "epilogue staging");
  unsigned ycol[BQ];
#pragma unroll
  for (int q = 0; q < BQ; ++q) {
    const int pc = p0 + q * 64 + lane;
    ycol[q] = p.y_bytes;
    if (pc < P) {
      const int b = fdiv(pc, p.divN_m, p.divN_s), n = pc - b * N;
      const int t = fdiv(n, p.divV_m, p.divV_s), v = n - t * V;
      ycol[q] = ((unsigned)b * (unsigned)p.y.bstride + (unsigned)t * (unsigned)(p.y.tstride * V) + (unsigned)v) * 4u;
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const int r = 8 * h + rr;
          const int lr = wm * 16 + (r & 3) + 8 * ((r >> 2) & 1) + 4 * kl;
          smem[lr * BN + wn * (BN / WN) + j * 32 + cl] = acc[i][j][r];
        }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < RPW; ++k) {
        const int lr = wid + k * NW;
        const int trow = (lr >> 4) * (BM / WM) + i * 32 + 16 * h + (lr & 15);
        if (m0 + trow >= M) break;
        const float bv = bias_s[trow];
        const unsigned soff = (unsigned)(m0 + trow) * ycs4;
#pragma unroll
        for (int q = 0; q < BQ; ++q) {
          float val = smem[lr * BN + lane + 64 * q] + bv;
          if (p.relu) val = fmaxf(val, 0.f);
          bstore(yr, val, ycol[q], soff);
        }
      }
      __syncthreads();
    }
}

template <int BM, int BN, int WM, int WN>
void launch_pwd3(const FwdArgs& a, hipStream_t st) {
  const long long P = (long long)a.B * a.T * a.V;
  dim3 grid((unsigned)((P + BN - 1) / BN), (a.M + BM - 1) / BM);
  if (a.a_mcontig) pwd3_kernel<BM, BN, WM, WN, true><<<grid, 64 * WM * WN, 0, st>>>(a);
  else pwd3_kernel<BM, BN, WM, WN, false><<<grid, 64 * WM * WN, 0, st>>>(a);
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
  const int rounds = argc > 1 ? atoi(argv[1]) : 2;
  Shape shapes[] = {
    {"l9 tcn 256 T75", 128, 256, 256, 75, 25, 0},
    {"l9 tcn dX 256 T75", 128, 256, 256, 75, 25, 1},
    {"l8 tcn-in 256x128 T150", 128, 256, 128, 150, 25, 0},
    {"l6 tcn 128 T150", 128, 128, 128, 150, 25, 0},
    {"l5 tcn 128 T300", 128, 128, 128, 300, 25, 0},
    {"ragged 200x72 T37 V7 B5", 5, 200, 72, 37, 7, 0},
    {"ragged 130x40 T37 V7 B5 mc", 5, 130, 40, 37, 7, 1},
  };
  hipStream_t st; CK(hipStreamCreate(&st));
  const size_t maxe = (size_t)128 * 256 * 150 * 25;
  float *x, *y1, *y2, *w, *bias;
  CK(hipMalloc(&x, maxe * 4)); CK(hipMalloc(&y1, maxe * 4)); CK(hipMalloc(&y2, maxe * 4));
  CK(hipMalloc(&w, 256 * 256 * 4)); CK(hipMalloc(&bias, 256 * 4));
  std::vector<float> h(maxe);
  for (size_t i = 0; i < maxe; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(x, h.data(), maxe * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data() + 11, 256 * 256 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h.data() + 5, 256 * 4, hipMemcpyHostToDevice));
  std::vector<float> g1(maxe), g2(maxe);
  for (auto& s : shapes) {
    const int N = s.T * s.V;
    const double P = (double)s.B * N;
    const double fl = 2.0 * P * s.M * s.K;
    const size_t ny = (size_t)s.B * s.M * N;
    auto prod = [&]() {
      if (sgcn_pw_fwd(w, s.amc, bias, x, (long long)s.K * N, N, 1, 0, nullptr, y1,
                      (long long)s.M * N, N, 1, 0, 1, 0, s.B, s.M, s.K, s.T, s.V, st)) {
        printf("sgcn_pw_fwd failed\n");
        exit(1);
      }
    };
    FwdArgs a{};
    a.A = w; a.lda = s.amc ? s.M : s.K; a.a_mcontig = s.amc; a.bias = bias; a.relu = 1;
    a.x = {x, (long long)s.K * N, N, 1, 0};
    a.y = {y2, (long long)s.M * N, N, 1, 0};
    a.M = s.M; a.K = s.K; a.T = s.T; a.V = s.V; a.B = s.B;
    fwd_divisors(a);
    a.x_bytes = plane_bytes(a.x.bstride, a.x.cstride, 1, s.B, s.K, s.T, s.V);
    a.y_bytes = plane_bytes(a.y.bstride, a.y.cstride, 1, s.B, s.M, s.T, s.V);
    a.a_bytes = (unsigned)(s.M * s.K * 4);
    const int reps = s.B > 16 ? 20 : 5;
    for (int r = 0; r < rounds; ++r) {
      float us = timeit(prod, st, reps);
      printf("%-28s %-18s %8.1f us  %6.1f TF/s\n", s.name, "product", us, fl / us / 1e6);
      auto run = [&](const char* nm, auto L) {
        CK(hipMemset(y2, 0xff, ny * 4));
        const float u = timeit(L, st, reps);
        CK(hipMemcpy(g1.data(), y1, ny * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(g2.data(), y2, ny * 4, hipMemcpyDeviceToHost));
        printf("%-28s %-18s %8.1f us  %6.1f TF/s  %s\n", s.name, nm, u, fl / u / 1e6,
               memcmp(g1.data(), g2.data(), ny * 4) == 0 ? "bit-exact" : "MISMATCH");
      };
      if (s.M > 128) {
        run("b128 256x128", [&]() { launch_pwd3<256, 128, 4, 2>(a, st); });
        run("b128 128x128 x2", [&]() { launch_pwd3<128, 128, 4, 2>(a, st); });
      } else {
        run("b128 128x128", [&]() { launch_pwd3<128, 128, 4, 2>(a, st); });
        run("b128 128x256 w2x4", [&]() { launch_pwd3<128, 256, 2, 4>(a, st); });
      }
    }
  }
  printf("done\n");
  return 0;
}
