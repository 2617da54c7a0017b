// Pointwise (1x1) channel contractions of the Shift-GCN hot path on fp32 MFMA (gfx950).
//
// Every "trailing pointwise conv" of the reference is one C_in x C_out contraction over
// P = N·M·T·V positions of the (N·M, C, T, V) layout:
//   Shift_gcn : einsum('nwc,cd->nwd') between the two joint-shift gathers
//               (model/shift_gcn.py:125-136), + Linear_bias
//   Shift_tcn : temporal_linear Conv2d(C, C, 1) (shift_gcn.py:62,69)
//   down / residual tcn(k=1, stride s) Conv2d (shift_gcn.py:84, 35-36)
// The joint-shift gathers (index_select with shift_in / shift_out, shift_gcn.py:108-118,
// 127, 136) and the feature mask are NOT separate passes here: shift_in + mask are
// applied while staging the B operand (a per-channel rotation inside each V-row), and
// shift_out is applied in the epilogue's store addresses (rotation by the output
// channel). No permute to (n·t, v·c) is ever materialised.
//
// Kernels
//  * pw_fwd_kernel : Y[b][m][pos_out(n,m)] (+)= act(sum_k A[m][k] * Bop(b,k,n) + bias[m])
//      used for the forward (A = weights) and for dX (A = weights^T).
//      Tile BM x 128 positions x BK, 4 waves (2x2), v_mfma_f32_32x32x2_f32 (exact f32,
//      one rounding per product == an fmaf chain), LDS-staged operands with register
//      prefetch of the next K stage, M-tiles fastest in the grid so the blocks sharing an
//      X tile run back to back (Infinity-Cache hits for the second M-tile).
//  * pw_dw_kernel  : split-K dW[m][n] = sum_{b,p} G(b,m,p) * X(b,n,p) over all positions,
//      deterministic fp32 partial slabs [split][M][N] + row sums (bias grad), reduced in
//      fixed order by slab_reduce_kernel (optionally transposed, for Linear_weight's
//      (C_in, C_out) layout).
#include "common.hpp"

namespace sgcn {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kThreads = 256;
constexpr int kMaskMaxV = 64;      // joints per row supported by the dW LDS mask table
constexpr int kMaskFwdMax = 8448;  // V*K floats of the forward LDS mask table (33 x 256)

// A position-mapped plane operand: element (b, ch, n) with n = t*V + v (logical
// position) lives at ptr[b*bstride + ch*cstride + (t*tstride)*V + rot(v, ch)], where
// rot(v, ch) = (v + rsign*ch) mod V.
struct Plane {
  const float* ptr;
  long long bstride;
  long long cstride;
  int tstride;
  int rsign;
};

struct OutPlane {
  float* ptr;
  long long bstride;
  long long cstride;
  int tstride;
  int rsign;
};

struct FwdArgs {
  const float* A;   // weights
  int lda;
  int a_mcontig;    // A[m][k] = a_mcontig ? A[k*lda+m] : A[m*lda+k]
  const float* bias;
  Plane x;
  const float* mask;  // optional mask[v*K + k] multiplied into B (Shift_gcn feature mask)
  OutPlane y;
  int M, K, T, V;
};

__device__ __forceinline__ int pmod(int a, int V) {
  int r = a % V;
  return r < 0 ? r + V : r;
}

// keep v where ok, exact +0 elsewhere: a bit-AND the compiler cannot turn back into a
// branch around the (always in-bounds) load
__device__ __forceinline__ float keep(float v, bool ok) {
  return __uint_as_float(__float_as_uint(v) & (ok ? 0xffffffffu : 0u));
}

// rotation step (d*rsign) mod V in [0, V)
__device__ __forceinline__ int rot_step(int d, int rsign, int V) { return pmod(d * rsign, V); }

// ------------------------------------------------------------------------------------
// forward / dX
// ------------------------------------------------------------------------------------
template <int BM, int BK, int WM, bool MASK, bool RELU, bool ACCUM, bool AMC>
__global__ __launch_bounds__(64 * WM * 2) void pw_fwd_kernel(FwdArgs p) {
  constexpr int NT = 64 * WM * 2;      // waves: WM along M x 2 along N
  constexpr int BN = 128;
  constexpr int MI = BM / WM / 32;     // 32-row sub-tiles per wave
  constexpr int NJ = BN / 2 / 32;      // 32-col sub-tiles per wave
  constexpr int AP = BM + 1, BP = BN + 1;
  constexpr int A_PER = BM * BK / NT;
  constexpr int B_PER = BN * BK / NT;
  constexpr int KSTEP_B = NT / BN;     // k rows between a thread's B elements
  static_assert(MI >= 1, "wave tile too small");
  static_assert(A_PER >= 1 && B_PER >= 1, "tile too small");
  __shared__ float As[BK * AP];
  __shared__ float Bs[BK * BP];
  __shared__ short rot_out[BM];
  __shared__ float bias_s[BM];
  extern __shared__ float mask_s[];   // [v][k] feature mask table (dynamic: V*K floats)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN, b = blockIdx.z;
  const int V = p.V, N = p.T * V, K = p.K, M = p.M;

  // row-constant epilogue data staged once (no runtime-conditional load in the epilogue)
  for (int i = tid; i < BM; i += NT) {
    rot_out[i] = (short)pmod(p.y.rsign * (m0 + i), V);
    bias_s[i] = (p.bias && m0 + i < M) ? p.bias[m0 + i] : 0.f;
  }
  if (MASK)
    for (int i = tid; i < V * K; i += NT) mask_s[i] = p.mask[i];
  __syncthreads();   // rot_out / bias_s / mask_s are read before the main loop's barrier

  // B staging: thread owns column n and rows kb0 + KSTEP_B*i. 32-bit offsets from the
  // sample's base; the shift_in rotation (v + rsign*k) mod V advances incrementally.
  const int nb = tid % BN, kb0 = tid / BN;
  const int n = n0 + nb;
  const bool nvalid = n < N;
  const int ncl = min(n, N - 1);
  const int tt = ncl / V;
  const int vv = ncl - tt * V;
  const float* __restrict__ xb =
      p.x.ptr + (long long)b * p.x.bstride + (long long)tt * p.x.tstride * V;
  const int xcs = (int)p.x.cstride;
  const int bstep = rot_step(KSTEP_B, p.x.rsign, V);
  // A staging
  constexpr int A_MSTEP = NT / BK;   // (k-contig) rows per step
  constexpr int A_KSTEP = NT / BM;   // (m-contig) k per step
  const int am = AMC ? tid % BM : tid / BK;
  const int ak = AMC ? tid / BM : tid % BK;
  const float* __restrict__ A = p.A;
  const int lda = p.lda;

  // Raw loads only (always in bounds); validity is applied at the LDS store, after the
  // MFMAs of the current stage, so no instruction consumes a prefetched value early
  // (consuming it right away made hipcc drain vmcnt(0) after every load).
  float ra[A_PER], rb[B_PER];
  auto load_stage = [&](int k0) {
    int cv = pmod(vv + p.x.rsign * (k0 + kb0), V);
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int kc = min(k0 + kb0 + i * KSTEP_B, K - 1);
      rb[i] = xb[kc * xcs + cv];
      cv += bstep;
      cv = cv >= V ? cv - V : cv;
    }
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int m = AMC ? am : am + i * A_MSTEP;
      const int k = AMC ? ak + i * A_KSTEP : ak;
      const int gmc = min(m0 + m, M - 1), gkc = min(k0 + k, K - 1);
      ra[i] = AMC ? A[gkc * lda + gmc] : A[gmc * lda + gkc];
    }
  };
  auto store_stage = [&](int kst) {
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int k = kst + kb0 + i * KSTEP_B;
      float v = keep(rb[i], nvalid && k < K);
      if (MASK) v *= mask_s[vv * K + min(k, K - 1)];
      Bs[(kb0 + i * KSTEP_B) * BP + nb] = v;
    }
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int m = AMC ? am : am + i * A_MSTEP;
      const int k = AMC ? ak + i * A_KSTEP : ak;
      As[k * AP + m] = keep(ra[i], m0 + m < M && kst + k < K);
    }
  };

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};

  const int kl = lane >> 5, cl = lane & 31;
  load_stage(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    store_stage(k0);
    __syncthreads();
    if (k0 + BK < K) load_stage(k0 + BK);
    // fragments double-buffered in registers: the LDS reads of k-step kk+2 are in
    // flight while the MFMAs of k-step kk issue (no lgkmcnt(0) stall per k-step)
    float af[2][MI], bf[2][NJ];
    const float* __restrict__ Aw = As + kl * AP + wm * (BM / WM) + cl;
    const float* __restrict__ Bw = Bs + kl * BP + wn * (BN / 2) + cl;
#pragma unroll
    for (int i = 0; i < MI; ++i) af[0][i] = Aw[i * 32];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[0][j] = Bw[j * 32];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int cur = (kk >> 1) & 1;
      if (kk + 2 < BK) {
#pragma unroll
        for (int i = 0; i < MI; ++i) af[cur ^ 1][i] = Aw[(kk + 2) * AP + i * 32];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bf[cur ^ 1][j] = Bw[(kk + 2) * BP + j * 32];
      }
      // keep the prefetch reads above this k-step's MFMAs (the scheduler otherwise sinks
      // them below to reuse registers, exposing LDS latency every k-step)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[cur][i], bf[cur][j], acc[i][j],
                                                           0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // Row-constant data (bias, output rotation) per register; stores are predicated, never
  // branched around a load (ACCUM loads everything first).
  float* __restrict__ yb = p.y.ptr + (long long)b * p.y.bstride;
  const int ycs = (int)p.y.cstride;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = n0 + wn * (BN / 2) + j * 32 + cl;
    const bool cok = col < N;
    const int colc = min(col, N - 1);
    const int t = colc / V, v = colc - t * V;
    const int rowoff = t * p.y.tstride * V;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      int off[16];
      float prev[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const int mc = min(m0 + row, M - 1);
        int vo = v + rot_out[row];
        vo = vo >= V ? vo - V : vo;
        off[r] = mc * ycs + rowoff + vo;
        if (ACCUM) prev[r] = yb[off[r]];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const int m = m0 + row;
        float val = acc[i][j][r] + bias_s[row];
        if (RELU) val = fmaxf(val, 0.f);
        if (ACCUM) val += prev[r];
        if (cok && m < M) yb[off[r]] = val;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// dW (split-K over all positions)
// ------------------------------------------------------------------------------------
struct DwArgs {
  Plane g;            // A operand rows m: G(b, m, n)
  Plane x;            // B operand rows n: X(b, c, n)
  const float* mask;  // optional mask[v*Nc + c] on X
  float* slab;        // [S][M][Nc]
  float* bslab;       // optional [S][M] row sums of G
  int M, Nc, T, V, B;
  int chunks_per_split;
};

template <int BM, int BN, int WM, int WN, bool MASK>
__global__ __launch_bounds__(64 * WM * WN) void pw_dw_kernel(DwArgs p) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BK = 32;
  constexpr int MI = BM / WM / 32, NJ = BN / WN / 32;
  constexpr int AP = BM + 1, BP = BN + 1;
  constexpr int RSTEP = NT / BK;             // rows per load step
  constexpr int A_PER = BM / RSTEP, B_PER = BN / RSTEP;
  static_assert(MI >= 1 && NJ >= 1 && A_PER >= 1 && B_PER >= 1, "bad tile");
  __shared__ float As[BK * AP];
  __shared__ float Bs[BK * BP];
  extern __shared__ float mask_s[];   // [v][c - c0] (dynamic: V*BN floats)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntiles = (p.Nc + BN - 1) / BN;
  const int m0 = (blockIdx.x / ntiles) * BM, c0 = (blockIdx.x % ntiles) * BN;
  const int split = blockIdx.y;
  const int V = p.V, N = p.T * V;
  const int nchunk = (N + BK - 1) / BK;
  const int q_begin = split * p.chunks_per_split;
  const int q_end = min(q_begin + p.chunks_per_split, p.B * nchunk);
  const bool want_bias = p.bslab != nullptr && (blockIdx.x % ntiles) == 0;

  if (MASK) {
    for (int i = tid; i < V * BN; i += NT) {
      const int v = i / BN, c = c0 + (i - v * BN);
      mask_s[i] = c < p.Nc ? p.mask[v * p.Nc + c] : 0.f;
    }
    __syncthreads();
  }

  const int kq = tid % BK, r0 = tid / BK;
  // rotation of row r0 + RSTEP*i is (base + i*step) mod V, advanced incrementally
  const int g_rot0 = pmod(p.g.rsign * (m0 + r0), V), g_step = rot_step(RSTEP, p.g.rsign, V);
  const int x_rot0 = pmod(p.x.rsign * (c0 + r0), V), x_step = rot_step(RSTEP, p.x.rsign, V);
  const int gcs = (int)p.g.cstride, xcs = (int)p.x.cstride;
  float ra[A_PER], rb[B_PER], rsum[A_PER];
  int vcur = 0;
  bool ncur = false;
#pragma unroll
  for (int i = 0; i < A_PER; ++i) rsum[i] = 0.f;

  auto load_stage = [&](int q) {
    const int b = q / nchunk;
    const int n = (q - b * nchunk) * BK + kq;
    const bool nvalid = n < N;
    const int ncl = min(n, N - 1);
    const int t = ncl / V;
    const int v = ncl - t * V;
    vcur = v;
    ncur = nvalid;
    const float* __restrict__ gb =
        p.g.ptr + (long long)b * p.g.bstride + (long long)t * p.g.tstride * V;
    const float* __restrict__ xb =
        p.x.ptr + (long long)b * p.x.bstride + (long long)t * p.x.tstride * V;
    int cg = v + g_rot0;
    cg = cg >= V ? cg - V : cg;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int mc = min(m0 + r0 + i * RSTEP, p.M - 1);
      ra[i] = gb[mc * gcs + cg];
      cg += g_step;
      cg = cg >= V ? cg - V : cg;
    }
    int cx = v + x_rot0;
    cx = cx >= V ? cx - V : cx;
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int ccl = min(c0 + r0 + i * RSTEP, p.Nc - 1);
      rb[i] = xb[ccl * xcs + cx];
      cx += x_step;
      cx = cx >= V ? cx - V : cx;
    }
  };

  f32x16 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};

  const int kl = lane >> 5, cl = lane & 31;
  if (q_begin < q_end) load_stage(q_begin);
  for (int q = q_begin; q < q_end; ++q) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const float gv = keep(ra[i], ncur && m0 + r0 + i * RSTEP < p.M);
      As[kq * AP + r0 + i * RSTEP] = gv;
      rsum[i] += gv;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      float xv = keep(rb[i], ncur && c0 + r0 + i * RSTEP < p.Nc);
      if (MASK) xv *= mask_s[vcur * BN + r0 + i * RSTEP];
      Bs[kq * BP + r0 + i * RSTEP] = xv;
    }
    __syncthreads();
    if (q + 1 < q_end) load_stage(q + 1);
    float af[2][MI], bf[2][NJ];
    const float* __restrict__ Aw = As + kl * AP + wm * (BM / WM) + cl;
    const float* __restrict__ Bw = Bs + kl * BP + wn * (BN / WN) + cl;
#pragma unroll
    for (int i = 0; i < MI; ++i) af[0][i] = Aw[i * 32];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bf[0][j] = Bw[j * 32];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int cur = (kk >> 1) & 1;
      if (kk + 2 < BK) {
#pragma unroll
        for (int i = 0; i < MI; ++i) af[cur ^ 1][i] = Aw[(kk + 2) * AP + i * 32];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bf[cur ^ 1][j] = Bw[(kk + 2) * BP + j * 32];
      }
      // keep the prefetch reads above this k-step's MFMAs (the scheduler otherwise sinks
      // them below to reuse registers, exposing LDS latency every k-step)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[cur][i], bf[cur][j], acc[i][j],
                                                           0, 0, 0);
    }
    __syncthreads();
  }

  float* slab = p.slab + (size_t)split * p.M * p.Nc;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = c0 + wn * (BN / WN) + j * 32 + cl;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (m < p.M && c < p.Nc) slab[(size_t)m * p.Nc + c] = acc[i][j][r];
      }
  }
  if (want_bias) {
    // rows r0 + i*RSTEP are shared by the BK (= 32) lanes with equal tid/BK
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      float s = rsum[i];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const int m = m0 + r0 + i * RSTEP;
      if (kq == 0 && m < p.M) p.bslab[(size_t)split * p.M + m] = s;
    }
  }
}

// out[i] (+)= sum_s slab[s*n + i], i < n, in a FIXED order (deterministic): 64 outputs
// per block, 4 split-groups of 64 threads each summing every 4th split with 8 loads in
// flight, then the 4 group sums added in order. transpose: i = m*Nc + c -> out[c*M + m].
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab,
                                                          int S, int n, int M, int Nc,
                                                          float* __restrict__ out,
                                                          int transpose, int accum) {
  __shared__ float red[4][64];
  const int il = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + il;
  const int ic = min(i, n - 1);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = q;
  for (; s + 28 < S; s += 32) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += slab[(size_t)(s + 4 * k) * n + ic];
  }
  for (; s < S; s += 4) acc[0] += slab[(size_t)s * n + ic];
  red[q][il] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (q == 0 && i < n) {
    const float tot = (red[0][il] + red[1][il]) + (red[2][il] + red[3][il]);
    int dst = i;
    if (transpose) {
      const int m = i / Nc, c = i - m * Nc;
      dst = c * M + m;
    }
    out[dst] = accum ? out[dst] + tot : tot;
  }
}

// ------------------------------------------------------------------------------------
// launch helpers
// ------------------------------------------------------------------------------------
template <int BM, int BK, bool AMC>
void launch_fwd_bm(const FwdArgs& a, int B, bool mask, bool relu, bool accum, hipStream_t st) {
  constexpr int WM = BM / 32;   // one 32-row sub-tile per wave along M
  dim3 grid((a.M + BM - 1) / BM, (a.T * a.V + 127) / 128, B);
  const size_t dyn = mask ? (size_t)a.V * a.K * sizeof(float) : 0;
#define SGCN_PWF(MS, RL, AC) \
  pw_fwd_kernel<BM, BK, WM, MS, RL, AC, AMC><<<grid, 64 * WM * 2, dyn, st>>>(a)
  if (mask) {
    if (relu) { if (accum) SGCN_PWF(true, true, true); else SGCN_PWF(true, true, false); }
    else { if (accum) SGCN_PWF(true, false, true); else SGCN_PWF(true, false, false); }
  } else {
    if (relu) { if (accum) SGCN_PWF(false, true, true); else SGCN_PWF(false, true, false); }
    else { if (accum) SGCN_PWF(false, false, true); else SGCN_PWF(false, false, false); }
  }
#undef SGCN_PWF
}

int dw_splits(int M, int Nc, int B, int N, int tiles) {
  // ~512 workgroups (2 per CU at this kernel's register budget); slab <= 16 MiB
  const int total = B * ((N + 31) / 32);
  int S = (512 + tiles - 1) / tiles;
  const long long cap = (16LL << 20) / (4LL * M * Nc);
  if (S > cap) S = (int)cap;
  if (S > total) S = total;
  return S < 1 ? 1 : S;
}

int dw_tile(int X) { return X > 64 ? 128 : 64; }

}  // namespace
}  // namespace sgcn

using namespace sgcn;

extern "C" {

int sgcn_pw_fwd(const float* w, int w_mcontig, const float* bias, const float* x,
                long long x_bstride, long long x_cstride, int x_tstride, int x_rsign,
                const float* mask, float* y, long long y_bstride, long long y_cstride,
                int y_tstride, int y_rsign, int relu, int accumulate, int B, int M, int K,
                int T, int V, void* stream) {
  SGCN_REQUIRE(B >= 0 && M > 0 && K > 0 && K <= 256 && T >= 0 && V > 0 && V < 32768);
  SGCN_REQUIRE(x_tstride >= 1 && y_tstride >= 1);
  SGCN_REQUIRE(x_rsign >= -1 && x_rsign <= 1 && y_rsign >= -1 && y_rsign <= 1);
  SGCN_REQUIRE(x_cstride * (long long)K < (1LL << 31) && y_cstride * (long long)M < (1LL << 31));
  SGCN_REQUIRE(!mask || V * K <= kMaskFwdMax);
  if (B == 0 || T == 0) return 0;
  SGCN_REQUIRE(w && x && y);
  FwdArgs a;
  a.A = w;
  a.lda = w_mcontig ? M : K;
  a.a_mcontig = w_mcontig;
  a.bias = bias;
  a.x = {x, x_bstride, x_cstride, x_tstride, x_rsign};
  a.mask = mask;
  a.y = {y, y_bstride, y_cstride, y_tstride, y_rsign};
  a.M = M;
  a.K = K;
  a.T = T;
  a.V = V;
  hipStream_t st = (hipStream_t)stream;
  const bool mk = mask != nullptr, rl = relu != 0, ac = accumulate != 0;
#define SGCN_FWD_BM(BM_, BK_)                                                       \
  (w_mcontig ? launch_fwd_bm<BM_, BK_, true>(a, B, mk, rl, ac, st)                  \
             : launch_fwd_bm<BM_, BK_, false>(a, B, mk, rl, ac, st))
  if (K <= 4) {
    if (M <= 64) SGCN_FWD_BM(64, 4); else SGCN_FWD_BM(128, 4);
  } else {
    if (M <= 64) SGCN_FWD_BM(64, 32); else SGCN_FWD_BM(128, 32);
  }
#undef SGCN_FWD_BM
  SGCN_LAUNCH_CHECK();
  return 0;
}

size_t sgcn_pw_dw_ws_bytes(int B, int M, int Nc, int T, int V) {
  const int tiles = ((M + dw_tile(M) - 1) / dw_tile(M)) * ((Nc + dw_tile(Nc) - 1) / dw_tile(Nc));
  const int S = dw_splits(M, Nc, B, T * V, tiles);
  return (size_t)S * ((size_t)M * Nc + M) * sizeof(float);
}

int sgcn_pw_dw(const float* g, long long g_bstride, long long g_cstride, int g_tstride,
               int g_rsign, const float* x, long long x_bstride, long long x_cstride,
               int x_tstride, int x_rsign, const float* mask, float* dw, int dw_transpose,
               int dw_accumulate, float* dbias, int dbias_accumulate, void* ws,
               size_t ws_bytes, int B, int M, int Nc, int T, int V, void* stream) {
  SGCN_REQUIRE(B > 0 && M > 0 && Nc > 0 && T > 0 && V > 0 && V < 32768);
  SGCN_REQUIRE(g && x && dw && ws && g_tstride >= 1 && x_tstride >= 1);
  SGCN_REQUIRE(!mask || V <= kMaskMaxV);
  SGCN_REQUIRE(ws_bytes >= sgcn_pw_dw_ws_bytes(B, M, Nc, T, V));
  SGCN_REQUIRE(g_cstride * (long long)M < (1LL << 31) && x_cstride * (long long)Nc < (1LL << 31));
  const int bm = dw_tile(M), bn = dw_tile(Nc);
  const int tiles = ((M + bm - 1) / bm) * ((Nc + bn - 1) / bn);
  const int N = T * V;
  const int S = dw_splits(M, Nc, B, N, tiles);
  const int total = B * ((N + 31) / 32);
  DwArgs a;
  a.g = {g, g_bstride, g_cstride, g_tstride, g_rsign};
  a.x = {x, x_bstride, x_cstride, x_tstride, x_rsign};
  a.mask = mask;
  a.slab = (float*)ws;
  a.bslab = dbias ? (float*)ws + (size_t)S * M * Nc : nullptr;
  a.M = M;
  a.Nc = Nc;
  a.T = T;
  a.V = V;
  a.B = B;
  a.chunks_per_split = (total + S - 1) / S;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(tiles, S);
#define SGCN_DW(BM_, BN_)                                                                    \
  (mask ? pw_dw_kernel<BM_, BN_, BM_ / 32, 2, true>                                           \
              <<<grid, 64 * (BM_ / 32) * 2, (size_t)V * BN_ * sizeof(float), st>>>(a)       \
        : pw_dw_kernel<BM_, BN_, BM_ / 32, 2, false><<<grid, 64 * (BM_ / 32) * 2, 0, st>>>(a))
  if (bm == 128 && bn == 128) SGCN_DW(128, 128);
  else if (bm == 128) SGCN_DW(128, 64);
  else if (bn == 128) SGCN_DW(64, 128);
  else SGCN_DW(64, 64);
#undef SGCN_DW
  SGCN_LAUNCH_CHECK();
  const int MN = M * Nc;
  slab_reduce_kernel<<<(MN + 63) / 64, 256, 0, st>>>(a.slab, S, MN, M, Nc, dw, dw_transpose,
                                                    dw_accumulate);
  SGCN_LAUNCH_CHECK();
  if (dbias) {
    slab_reduce_kernel<<<(M + 63) / 64, 256, 0, st>>>(a.bslab, S, M, M, 1, dbias, 0,
                                                     dbias_accumulate);
    SGCN_LAUNCH_CHECK();
  }
  return 0;
}

}  // extern "C"
