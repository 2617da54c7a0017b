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

// ------------------------------------------------------------------------------------
// forward / dX
// ------------------------------------------------------------------------------------
template <int BM, int BK, bool MASK, bool RELU, bool ACCUM>
__global__ __launch_bounds__(kThreads) void pw_fwd_kernel(FwdArgs p) {
  constexpr int BN = 128;
  constexpr int MI = BM / 64;          // 32-row sub-tiles per wave (waves are 2 x 2)
  constexpr int NJ = BN / 64;          // 32-col sub-tiles per wave
  constexpr int AP = BM + 1, BP = BN + 1;
  constexpr int A_PER = BM * BK / kThreads;
  constexpr int B_PER = BN * BK / kThreads;
  static_assert(A_PER >= 1 && B_PER >= 1, "tile too small");
  __shared__ float As[BK * AP];
  __shared__ float Bs[BK * BP];
  __shared__ short rot_in[256];
  __shared__ short rot_out[BM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN, b = blockIdx.z;
  const int V = p.V, N = p.T * V, K = p.K, M = p.M;

  for (int i = tid; i < K; i += kThreads) rot_in[i] = (short)pmod(p.x.rsign * i, V);
  for (int i = tid; i < BM; i += kThreads) rot_out[i] = (short)pmod(p.y.rsign * (m0 + i), V);
  __syncthreads();

  // B staging: thread owns one column n and rows kb0 + i*(kThreads/BN)
  const int nb = tid % BN, kb0 = tid / BN;
  const int n = n0 + nb;
  const bool nvalid = n < N;
  const int ncl = min(n, N - 1);           // clamped: loads stay in bounds, value masked
  const int tt = ncl / V;
  const int vv = ncl - tt * V;
  const float* xb = p.x.ptr + (long long)b * p.x.bstride + (long long)tt * p.x.tstride * V;
  // A staging
  const int am = p.a_mcontig ? tid % BM : tid / BK;
  const int ak = p.a_mcontig ? tid / BM : tid % BK;
  constexpr int A_MSTEP = kThreads / BK;   // (k-contig) rows per step
  constexpr int A_KSTEP = kThreads / BM;   // (m-contig) k per step

  float ra[A_PER], rb[B_PER];
  auto load_stage = [&](int k0) {
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int k = k0 + kb0 + i * (kThreads / BN);
      const int kc = min(k, K - 1);
      int c = vv + rot_in[kc];
      c = c >= V ? c - V : c;
      float v = xb[(long long)kc * p.x.cstride + c];
      if (MASK) v *= p.mask[vv * K + kc];
      rb[i] = (nvalid && k < K) ? v : 0.f;
    }
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int m, k;
      if (p.a_mcontig) { m = am; k = ak + i * A_KSTEP; }
      else { m = am + i * A_MSTEP; k = ak; }
      const int gm = m0 + m, gk = k0 + k;
      const int gmc = min(gm, M - 1), gkc = min(gk, K - 1);
      const float v = p.a_mcontig ? p.A[(long long)gkc * p.lda + gmc]
                                  : p.A[(long long)gmc * p.lda + gkc];
      ra[i] = (gm < M && gk < K) ? v : 0.f;
    }
  };
  auto store_stage = [&]() {
#pragma unroll
    for (int i = 0; i < B_PER; ++i) Bs[(kb0 + i * (kThreads / BN)) * BP + nb] = rb[i];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int m, k;
      if (p.a_mcontig) { m = am; k = ak + i * A_KSTEP; }
      else { m = am + i * A_MSTEP; k = ak; }
      As[k * AP + m] = ra[i];
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
    store_stage();
    __syncthreads();
    if (k0 + BK < K) load_stage(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float af[MI], bf[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = As[(kk + kl) * AP + wm * (BM / 2) + i * 32 + cl];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[j] = Bs[(kk + kl) * BP + wn * (BN / 2) + j * 32 + cl];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* yb = p.y.ptr + (long long)b * p.y.bstride;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = n0 + wn * (BN / 2) + j * 32 + cl;
    if (col >= N) continue;
    const int t = col / V, v = col - t * V;
    float* yt = yb + (long long)t * p.y.tstride * V;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const int m = m0 + row;
        if (m >= M) continue;
        float val = acc[i][j][r];
        if (p.bias) val += p.bias[m];
        if (RELU) val = fmaxf(val, 0.f);
        int vo = v + rot_out[row];
        vo = vo >= V ? vo - V : vo;
        float* dst = yt + (long long)m * p.y.cstride + vo;
        if (ACCUM) *dst += val; else *dst = val;
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

template <int BM, int BN, bool MASK>
__global__ __launch_bounds__(kThreads) void pw_dw_kernel(DwArgs p) {
  constexpr int BK = 32;
  constexpr int MI = BM / 64, NJ = BN / 64;
  constexpr int AP = BM + 1, BP = BN + 1;
  constexpr int RSTEP = kThreads / BK;       // rows per load step (8)
  constexpr int A_PER = BM / RSTEP, B_PER = BN / RSTEP;
  __shared__ float As[BK * AP];
  __shared__ float Bs[BK * BP];
  __shared__ short rot_g[BM];
  __shared__ short rot_x[BN];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntiles = (p.Nc + BN - 1) / BN;
  const int m0 = (blockIdx.x / ntiles) * BM, c0 = (blockIdx.x % ntiles) * BN;
  const int split = blockIdx.y;
  const int V = p.V, N = p.T * V;
  const int nchunk = (N + BK - 1) / BK;
  const int q_begin = split * p.chunks_per_split;
  const int q_end = min(q_begin + p.chunks_per_split, p.B * nchunk);
  const bool want_bias = p.bslab != nullptr && (blockIdx.x % ntiles) == 0;

  for (int i = tid; i < BM; i += kThreads) rot_g[i] = (short)pmod(p.g.rsign * (m0 + i), V);
  for (int i = tid; i < BN; i += kThreads) rot_x[i] = (short)pmod(p.x.rsign * (c0 + i), V);
  __syncthreads();

  const int kq = tid % BK, r0 = tid / BK;
  float ra[A_PER], rb[B_PER], rsum[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) rsum[i] = 0.f;

  auto load_stage = [&](int q) {
    const int b = q / nchunk;
    const int n = (q - b * nchunk) * BK + kq;
    const bool nvalid = n < N;
    const int ncl = min(n, N - 1);
    const int t = ncl / V;
    const int v = ncl - t * V;
    const float* gb = p.g.ptr + (long long)b * p.g.bstride + (long long)t * p.g.tstride * V;
    const float* xb = p.x.ptr + (long long)b * p.x.bstride + (long long)t * p.x.tstride * V;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int row = r0 + i * RSTEP, m = m0 + row;
      const int mc = min(m, p.M - 1);
      int c = v + rot_g[row];
      c = c >= V ? c - V : c;
      const float val = gb[(long long)mc * p.g.cstride + c];
      ra[i] = (nvalid && m < p.M) ? val : 0.f;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int row = r0 + i * RSTEP, c = c0 + row;
      const int ccl = min(c, p.Nc - 1);
      int cc = v + rot_x[row];
      cc = cc >= V ? cc - V : cc;
      float val = xb[(long long)ccl * p.x.cstride + cc];
      if (MASK) val *= p.mask[v * p.Nc + ccl];
      rb[i] = (nvalid && c < p.Nc) ? val : 0.f;
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
      As[kq * AP + r0 + i * RSTEP] = ra[i];
      rsum[i] += ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) Bs[kq * BP + r0 + i * RSTEP] = rb[i];
    __syncthreads();
    if (q + 1 < q_end) load_stage(q + 1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float af[MI], bf[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = As[(kk + kl) * AP + wm * (BM / 2) + i * 32 + cl];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[j] = Bs[(kk + kl) * BP + wn * (BN / 2) + j * 32 + cl];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  float* slab = p.slab + (size_t)split * p.M * p.Nc;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = c0 + wn * (BN / 2) + j * 32 + cl;
    if (c >= p.Nc) continue;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (m < p.M) slab[(size_t)m * p.Nc + c] = acc[i][j][r];
      }
  }
  if (want_bias) {
    // rows r0 + i*RSTEP are shared by the 32 lanes with equal tid/BK (one half-wave)
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
template <int BM, int BK>
void launch_fwd_bm(const FwdArgs& a, int B, bool mask, bool relu, bool accum, hipStream_t st) {
  dim3 grid((a.M + BM - 1) / BM, (a.T * a.V + 127) / 128, B);
#define SGCN_PWF(MS, RL, AC) pw_fwd_kernel<BM, BK, MS, RL, AC><<<grid, kThreads, 0, st>>>(a)
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
  if (K <= 4) {
    if (M <= 64) launch_fwd_bm<64, 4>(a, B, mk, rl, ac, st);
    else launch_fwd_bm<128, 4>(a, B, mk, rl, ac, st);
  } else {
    if (M <= 64) launch_fwd_bm<64, 32>(a, B, mk, rl, ac, st);
    else launch_fwd_bm<128, 32>(a, B, mk, rl, ac, st);
  }
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
  SGCN_REQUIRE(ws_bytes >= sgcn_pw_dw_ws_bytes(B, M, Nc, T, V));
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
#define SGCN_DW(BM_, BN_)                                                       \
  (mask ? pw_dw_kernel<BM_, BN_, true><<<grid, kThreads, 0, st>>>(a)           \
        : pw_dw_kernel<BM_, BN_, false><<<grid, kThreads, 0, st>>>(a))
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
