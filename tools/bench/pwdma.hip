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
// DIAG (timing only, results wrong): 1 = no MFMA, 2 = no Y stores, 4 = no B DMA
template <int BN, bool AMC, bool WAITS, int DIAG = 0>
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
      if (!(DIAG & 4)) dma(xr, bs0 + (unsigned)((row * BN + ch * 64) * 4), row < K ? xcol : p.x_bytes,
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
        if (!(DIAG & 1))
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[c2], bf[c2][j], acc[j], 0, 0, 0);
    }
  };
  if (WAITS) {
    vm_barrier<(DIAG & 4) ? 0 : 3 * BPER>();
    stage(0);
    if (nstage > 1) {
      vm_barrier<(DIAG & 4) ? 0 : 2 * BPER>();
      stage(1);
    }
    if (nstage > 2) {
      vm_barrier<(DIAG & 4) ? 0 : BPER>();
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
      if (!(DIAG & 2)) bstore(yr, val, ycol[q], (unsigned)row * ycs4);
      else if (val == 12345.f) bstore(yr, val, ycol[q], (unsigned)row * ycs4);
    }
  }
}

template <int BN, bool AMC, bool WAITS, int DIAG = 0>
void launch_pwd(const FwdArgs& a, hipStream_t st) {
  const int P = a.B * a.T * a.V;
  pwd_kernel<BN, AMC, WAITS, DIAG><<<(P + BN - 1) / BN, 256, 0, st>>>(a);
}

// ---- persistent form: A in registers (loaded once per workgroup), two B buffers in LDS;
// tile j+1's DMA is in flight while tile j computes and stores. NW waves (2 x NW/2), BN
// positions x 64 rows per tile; the DMA counts per wave keep every counted wait <= 63.
template <int BASE, int SPW, int BT>
__device__ __forceinline__ void vm_wait_code(int code) {
  // code bit 0: the previous tile's stores are younger; bit 1: the next tile's DMA is
  switch (code) {
    case 0: vm_barrier<BASE>(); break;
    case 1: vm_barrier<BASE + SPW>(); break;
    case 2: vm_barrier<BASE + BT>(); break;
    default: vm_barrier<BASE + SPW + BT>(); break;
  }
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int BN, int NW, bool AMC, int DIAG = 0>
__global__ __launch_bounds__(64 * NW) void pwp_kernel(FwdArgs p, int ntiles) {
  constexpr int CH = BN / 64;
  constexpr int WN = NW / 2;
  constexpr int NJ = BN / WN / 32;
  constexpr int BPER = 16 * CH / NW;   // DMA per wave per 16-row stage
  constexpr int BT = 4 * BPER;         // DMA per wave per tile
  constexpr int RPW = 64 / NW;         // stored rows per wave
  constexpr int SPW = RPW * CH;        // stores per wave per tile
  static_assert(NJ >= 1 && BPER >= 1 && NW % CH == 0, "tile");
  static_assert(3 * BPER + SPW + BT <= 63, "vmcnt range");
  __shared__ float Bs[2 * 64 * BN];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int kl = lane >> 5, cl = lane & 31;
  const int V = p.V, N = p.T * V, K = p.K, M = p.M;
  const int P = p.B * N;
  // XCD-contiguous tile ranges (workgroup b on XCD b mod 8): adjacent tiles share an L2
  const int GX = gridDim.x >> 3, xc = blockIdx.x & 7, wi = blockIdx.x >> 3;
  const int lo = (int)((long long)ntiles * xc / 8), hi = (int)((long long)ntiles * (xc + 1) / 8);
  int t = lo + wi;
  if (t >= hi) return;
  const i32x4 xr = rsrc4(p.x.ptr, p.x_bytes);
  const auto ar = make_rsrc(p.A, p.a_bytes);
  const auto yr = make_rsrc(p.y.ptr, p.y_bytes);
  const unsigned bs0 = lds_addr(Bs);
  const unsigned xcs4 = (unsigned)(p.x.cstride * 4), ycs4 = (unsigned)(p.y.cstride * 4);
  // A fragments of this wave's 32 rows for all 64 k (rows / columns past M / K: 0)
  float a[32];
  {
    const int m = wm * 32 + cl;
#pragma unroll
    for (int kp = 0; kp < 32; ++kp) {
      const int k = 2 * kp + kl;
      const bool ok = k < K && m < M;
      a[kp] = bload(ar, ok ? (unsigned)((AMC ? k * p.lda + m : m * p.lda + k) * 4) : p.a_bytes, 0);
    }
  }
  float bias[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int row = wid + NW * i;
    bias[i] = (p.bias && row < M) ? p.bias[row] : 0.f;
  }
  // the compiler waits for these loads here, before any (uncounted) DMA is issued
  asm volatile("" ::"v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
               "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]),
               "v"(a[12]), "v"(a[13]), "v"(a[14]), "v"(a[15]));
  asm volatile("" ::"v"(a[16]), "v"(a[17]), "v"(a[18]), "v"(a[19]), "v"(a[20]), "v"(a[21]),
               "v"(a[22]), "v"(a[23]), "v"(a[24]), "v"(a[25]), "v"(a[26]), "v"(a[27]),
               "v"(a[28]), "v"(a[29]), "v"(a[30]), "v"(a[31]));
#pragma unroll
  for (int i = 0; i < RPW; ++i) asm volatile("" ::"v"(bias[i]));
  const int ch = wid % CH;
  auto col_off = [&](int pc, long long bstride, int tstride, unsigned oob) {
    if (pc >= P) return oob;
    const int b = fdiv(pc, p.divN_m, p.divN_s), n = pc - b * N;
    const int tq = fdiv(n, p.divV_m, p.divV_s), v = n - tq * V;
    return ((unsigned)b * (unsigned)bstride + (unsigned)tq * (unsigned)(tstride * V) + (unsigned)v) * 4u;
  };
  auto issue = [&](int tt, int buf) {
    const unsigned xcol = col_off(tt * BN + ch * 64 + lane, p.x.bstride, p.x.tstride, p.x_bytes);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < BPER; ++i) {
        const int row = s * 16 + (wid + NW * i) / CH;
        if (!(DIAG & 4))
          dma(xr, bs0 + (unsigned)(((buf * 64 + row) * BN + ch * 64) * 4),
              row < K ? xcol : p.x_bytes, (unsigned)row * xcs4);
      }
  };
  issue(t, 0);
  if (t + GX < hi) issue(t + GX, 1);
  for (int j = 0; t < hi; ++j, t += GX) {
    const int buf = j & 1;
    const int code = (j > 0 ? 1 : 0) | (t + GX < hi ? 2 : 0);
    const float* B = Bs + buf * 64 * BN;
    f32x16 acc[NJ];
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) acc[jj] = f32x16{};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (DIAG & 4) lds_barrier();
      else if (s == 0) vm_wait_code<3 * BPER, SPW, BT>(code);
      else if (s == 1) vm_wait_code<2 * BPER, SPW, BT>(code);
      else if (s == 2) vm_wait_code<BPER, SPW, BT>(code);
      else vm_wait_code<0, SPW, BT>(code);
      if (s * 16 >= K) continue;
      const float* Bw = B + (s * 16 + kl) * BN + wn * (BN / WN) + cl;
      float bf[2][NJ];
#pragma unroll
      for (int jj = 0; jj < NJ; ++jj) bf[0][jj] = Bw[jj * 32];
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        const int c2 = (kk >> 1) & 1;
        if (kk + 2 < 16) {
#pragma unroll
          for (int jj = 0; jj < NJ; ++jj) bf[c2 ^ 1][jj] = Bw[(kk + 2) * BN + jj * 32];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj)
          if (!(DIAG & 1))
            acc[jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s * 8 + kk / 2], bf[c2][jj], acc[jj],
                                                           0, 0, 0);
      }
    }
    lds_barrier();   // every wave done reading this buffer's operand rows
    float* Bo = Bs + buf * 64 * BN;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        Bo[row * BN + wn * (BN / WN) + jj * 32 + cl] = acc[jj][r];
      }
    lds_barrier();
    unsigned ycol[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) ycol[q] = col_off(t * BN + q * 64 + lane, p.y.bstride, p.y.tstride, p.y_bytes);
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int row = wid + NW * i;
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        float val = Bo[row * BN + q * 64 + lane] + bias[i];
        if (p.relu) val = fmaxf(val, 0.f);
        // rows past M: an offset past the range (dropped), so every wave issues SPW stores
        const unsigned vo = row < M ? ycol[q] : p.y_bytes;
        if (!(DIAG & 2)) bstore(yr, val, vo, (unsigned)row * ycs4);
        else if (val == 12345.f) bstore(yr, val, vo, (unsigned)row * ycs4);
      }
    }
    lds_barrier();   // the staged rows read before the buffer takes tile j+2's operand
    if (t + 2 * GX < hi) issue(t + 2 * GX, buf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BN, int NW, bool AMC, int DIAG = 0>
void launch_pwp(const FwdArgs& a, hipStream_t st, int wgs_per_cu) {
  const int P = a.B * a.T * a.V;
  const int ntiles = (P + BN - 1) / BN;
  int g = 256 * wgs_per_cu;
  if (g > ntiles) g = (ntiles + 7) / 8 * 8;
  pwp_kernel<BN, NW, AMC, DIAG><<<g, 64 * NW, 0, st>>>(a, ntiles);
}

// ---- ring form: one continuous stream of 16-row operand stages through an R-slot LDS ring
// (stage g+R-1's DMA issued when stage g starts, across tile boundaries), persistent
// workgroups, A in registers, 8 waves (2 x 4) on 128-position tiles. EPI: true = stores from
// an LDS-staged copy of the tile (whole rows), false = straight from the accumulators.
template <int BASE, int STEP>
__device__ __forceinline__ void vm_wait_ys(int ys) {
  if (ys == 0) vm_barrier<BASE>();
  else if (ys == 1) vm_barrier<BASE + STEP>();
  else vm_barrier<BASE + 2 * STEP>();
}

template <int R, bool EPI, bool AMC, int DIAG = 0>
__global__ __launch_bounds__(512) void pwr_kernel(FwdArgs p, int ntiles) {
  constexpr int BN = 128, NW = 8, WN = 4, CH = 2;
  constexpr int BPER = 16 * CH / NW;   // DMA per wave per stage (4)
  constexpr int SLOT = 16 * BN;        // floats per ring slot
  constexpr int SPW = EPI ? (64 / NW) * CH : 16;   // stores per wave per tile
  static_assert(BPER * (R - 2) + 2 * SPW <= 63, "vmcnt range");
  static_assert(R >= 3 && R <= 9, "ring");
  __shared__ float ring[R * SLOT];
  __shared__ float E[EPI ? 64 * BN : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int kl = lane >> 5, cl = lane & 31;
  const int V = p.V, N = p.T * V, K = p.K, M = p.M;
  const int P = p.B * N;
  const int GX = gridDim.x >> 3, xc = blockIdx.x & 7, wi = blockIdx.x >> 3;
  const int lo = (int)((long long)ntiles * xc / 8), hi = (int)((long long)ntiles * (xc + 1) / 8);
  const int t0 = lo + wi;
  if (t0 >= hi) return;
  const int ntl = (hi - t0 + GX - 1) / GX;   // tiles of this workgroup
  const int nst = 4 * ntl;                  // stages of this workgroup
  const i32x4 xr = rsrc4(p.x.ptr, p.x_bytes);
  const auto ar = make_rsrc(p.A, p.a_bytes);
  const auto yr = make_rsrc(p.y.ptr, p.y_bytes);
  const unsigned r0 = lds_addr(ring);
  const unsigned xcs4 = (unsigned)(p.x.cstride * 4), ycs4 = (unsigned)(p.y.cstride * 4);
  float a[32];
  {
    const int m = wm * 32 + cl;
#pragma unroll
    for (int kp = 0; kp < 32; ++kp) {
      const int k = 2 * kp + kl;
      const bool ok = k < K && m < M;
      a[kp] = bload(ar, ok ? (unsigned)((AMC ? k * p.lda + m : m * p.lda + k) * 4) : p.a_bytes, 0);
    }
  }
  // bias of the rows this lane stores
  constexpr int NB = EPI ? 64 / NW : 16;
  float bias[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = EPI ? wid + NW * i : wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * kl;
    bias[i] = (p.bias && row < M) ? p.bias[row] : 0.f;
  }
  asm volatile("" ::"v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
               "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]),
               "v"(a[12]), "v"(a[13]), "v"(a[14]), "v"(a[15]));
  asm volatile("" ::"v"(a[16]), "v"(a[17]), "v"(a[18]), "v"(a[19]), "v"(a[20]), "v"(a[21]),
               "v"(a[22]), "v"(a[23]), "v"(a[24]), "v"(a[25]), "v"(a[26]), "v"(a[27]),
               "v"(a[28]), "v"(a[29]), "v"(a[30]), "v"(a[31]));
#pragma unroll
  for (int i = 0; i < NB; ++i) asm volatile("" ::"v"(bias[i]));
  const int ch = wid % CH;
  auto col_off = [&](int pc, long long bstride, int tstride, unsigned oob) {
    if (pc >= P) return oob;
    const int b = fdiv(pc, p.divN_m, p.divN_s), n = pc - b * N;
    const int tq = fdiv(n, p.divV_m, p.divV_s), v = n - tq * V;
    return ((unsigned)b * (unsigned)bstride + (unsigned)tq * (unsigned)(tstride * V) + (unsigned)v) * 4u;
  };
  // the lane's operand column of the tile being fetched (recomputed at each tile change)
  int fetch_tile = -1;
  unsigned xcol = p.x_bytes;
  // stage gg of this workgroup into ring slot gg % R (past the last stage: zeros, so every
  // iteration issues the same number of DMA and the counted waits stay exact)
  auto issue = [&](int gg) {
    const int tl = gg >> 2, st = gg & 3;
    if (tl != fetch_tile) {
      fetch_tile = tl;
      xcol = gg < nst ? col_off((t0 + tl * GX) * BN + ch * 64 + lane, p.x.bstride, p.x.tstride,
                                p.x_bytes)
                      : p.x_bytes;
    }
    const unsigned sl = r0 + (unsigned)((gg % R) * SLOT * 4);
#pragma unroll
    for (int i = 0; i < BPER; ++i) {
      const int rs = (wid + NW * i) / CH, row = st * 16 + rs;
      if (!(DIAG & 4))
        dma(xr, sl + (unsigned)((rs * BN + ch * 64) * 4), row < K ? xcol : p.x_bytes,
            (unsigned)row * xcs4);
    }
  };
#pragma unroll 1
  for (int gg = 0; gg < R - 1; ++gg) issue(gg);
  f32x16 acc = f32x16{};
#pragma unroll 1
  for (int g = 0; g < nst; ++g) {
    const int st = g & 3;
    // stores younger than stage g's DMA: the epilogues of iterations max(0, g-R+1) .. g-1
    int ys = 0;
    for (int i = g - 1; i >= 0 && i >= g - R + 1; --i) ys += (i & 3) == 3;
    if (DIAG & 4) lds_barrier();
    else vm_wait_ys<BPER * (R - 2), SPW>(ys);
    issue(g + R - 1);
    if (st * 16 < K) {
      const float* Bw = ring + (g % R) * SLOT + kl * BN + wn * 32 + cl;
      float bf[2];
      bf[0] = Bw[0];
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        const int c2 = (kk >> 1) & 1;
        if (kk + 2 < 16) bf[c2 ^ 1] = Bw[(kk + 2) * BN];
        __builtin_amdgcn_sched_barrier(0);
        float av;
        switch (st) {   // a[] indexed by a compile-time constant
          case 0: av = a[kk / 2]; break;
          case 1: av = a[8 + kk / 2]; break;
          case 2: av = a[16 + kk / 2]; break;
          default: av = a[24 + kk / 2]; break;
        }
        if (!(DIAG & 1)) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bf[c2], acc, 0, 0, 0);
      }
    }
    if (st == 3) {
      const int t = t0 + (g >> 2) * GX;
      if constexpr (EPI) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
          E[row * BN + wn * 32 + cl] = acc[r];
        }
        lds_barrier();
        unsigned ycol[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) ycol[q] = col_off(t * BN + q * 64 + lane, p.y.bstride, p.y.tstride, p.y_bytes);
#pragma unroll
        for (int i = 0; i < 64 / NW; ++i) {
          const int row = wid + NW * i;
#pragma unroll
          for (int q = 0; q < CH; ++q) {
            float val = E[row * BN + q * 64 + lane] + bias[i];
            if (p.relu) val = fmaxf(val, 0.f);
            const unsigned vo = row < M ? ycol[q] : p.y_bytes;
            if (!(DIAG & 2)) bstore(yr, val, vo, (unsigned)row * ycs4);
          }
        }
      } else {
        const unsigned ycol = col_off(t * BN + wn * 32 + cl, p.y.bstride, p.y.tstride, p.y_bytes);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rb = wm * 32 + (r & 3) + 8 * (r >> 2);   // uniform part of the row
          const int row = rb + 4 * kl;
          float val = acc[r] + bias[r];
          if (p.relu) val = fmaxf(val, 0.f);
          const unsigned vo = row < M ? ycol + (unsigned)(4 * kl) * ycs4 : p.y_bytes;
          if (!(DIAG & 2)) bstore(yr, val, vo, (unsigned)rb * ycs4);
        }
      }
      acc = f32x16{};
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int R, bool EPI, bool AMC, int DIAG = 0>
void launch_pwr(const FwdArgs& a, hipStream_t st, int wgs_per_cu) {
  const int P = a.B * a.T * a.V;
  const int ntiles = (P + 127) / 128;
  int g = 256 * wgs_per_cu;
  if (g > ntiles) g = (ntiles + 7) / 8 * 8;
  pwr_kernel<R, EPI, AMC, DIAG><<<g, 512, 0, st>>>(a, ntiles);
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
  const bool diag = argc > 2 && argv[2][0] == 'd';
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
      if (diag) {
        if (s.amc || s.B < 16 || s.K != 64) continue;
#define D_(F, NM)                                                                           \
  do {                                                                                      \
    float u = timeit([&]() { launch_pwd<128, false, true, F>(a, st); }, st, reps);          \
    printf("%-28s %-22s %8.1f us  %6.2f TB/s\n", s.name, NM, u, by / u / 1e6);               \
  } while (0)
        D_(0, "dma 128 staged");
#define Q_(F, NM)                                                                           \
  do {                                                                                      \
    float u = timeit([&]() { launch_pwp<128, 8, false, F>(a, st, 2); }, st, reps);           \
    printf("%-28s %-22s %8.1f us  %6.2f TB/s\n", s.name, NM, u, by / u / 1e6);               \
  } while (0)
#define W_(F, NM)                                                                           \
  do {                                                                                      \
    float u = timeit([&]() { launch_pwr<8, false, false, F>(a, st, 2); }, st, reps);         \
    printf("%-28s %-22s %8.1f us  %6.2f TB/s\n", s.name, NM, u, by / u / 1e6);               \
  } while (0)
        W_(0, "ring8 direct g2");
        W_(1, "  no MFMA");
        W_(2, "  no Y stores");
        W_(4, "  no X loads");
        W_(3, "  no MFMA, no stores");
        W_(6, "  only MFMA");
        continue;
      }
#define P_(BN, NW, G, NM)                                                                   \
  do {                                                                                      \
    CK(hipMemset(y2, 0xff, ny * 4));                                                        \
    float u = s.amc ? timeit([&]() { launch_pwp<BN, NW, true>(a, st, G); }, st, reps)       \
                    : timeit([&]() { launch_pwp<BN, NW, false>(a, st, G); }, st, reps);     \
    check(NM, u);                                                                           \
  } while (0)
#define R_(RR, EP, G, NM)                                                                   \
  do {                                                                                      \
    CK(hipMemset(y2, 0xff, ny * 4));                                                        \
    float u = s.amc ? timeit([&]() { launch_pwr<RR, EP, true>(a, st, G); }, st, reps)       \
                    : timeit([&]() { launch_pwr<RR, EP, false>(a, st, G); }, st, reps);     \
    check(NM, u);                                                                           \
  } while (0)
      R_(8, false, 2, "ring8 direct g2");
      R_(8, false, 1, "ring8 direct g1");
      R_(8, true, 1, "ring8 staged g1");
      R_(6, true, 2, "ring6 staged g2");
      R_(4, false, 4, "ring4 direct g4");
      P_(128, 8, 2, "persist 128 w8 g2");
      V_(128, true, "dma 128 staged");

    }
  }
  printf("done\n");
  return 0;
}
