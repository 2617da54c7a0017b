// Model head and tail of the training step (shift_gcn.py:193-216), native:
//   input side : permute (N, C, T, V, M) -> planes (N*M, C, T, V) fused with data_bn =
//                BatchNorm1d(M*V*C) over (n, t), feature f = m*V*C + v*C + c (:194-198);
//   output side: global average pool  x.view(N, M, C, -1).mean(3).mean(1)  (:211-214).
//
// data_bn statistics reuse the BatchNorm finalize kernels of bn.hip: sgcn_head_moments
// writes per-(n, feature) {mean, M2} partials over t in the reference feature order
// (perm_V = 0), sgcn_bn_finalize merges them over n; the backward partials
// {sum g, sum g*xhat} feed sgcn_bn_bwd_finalize the same way.
//
// Data sizes (NTU, bs=64): the clip is 11.5 MB, the pooled tensor 245 MB — every kernel
// here is a single HBM pass (bytes per element listed at each kernel).
#include "common.hpp"

namespace sgcn {
namespace {

constexpr int kHT = 256;
constexpr int kHU = 8;   // rows in flight per thread

// Column j of the (n, c) slab enumerates (m, v) as j = m*V + v; the clip element of
// column j at frame t is x[((n*C + c)*T + t)*V*M + v*M + m], the plane element
// y[((n*M + m)*C + c)*T*V + t*V + v] (consecutive j -> consecutive plane addresses).
__device__ __forceinline__ int clip_col(int j, int V, int M) {
  const int m = j / V, v = j - m * V;
  return v * M + m;
}

// part[n][f] = {mean, M2} over t of clip column (m, v) of channel c (shifted sums, as
// bn.hip moments_kernel). Grid N*C; bytes: 4 per clip element.
__global__ __launch_bounds__(kHT) void head_moments_kernel(const float* __restrict__ x,
                                                           float2* __restrict__ part, int C,
                                                           int T, int V, int M) {
  SGCN_CRIT_PRIO();
  __shared__ float s1[kHT], s2[kHT];
  const int nc = blockIdx.x, n = nc / C, c = nc - n * C;
  const int J = V * M, F = J * C;
  const float* __restrict__ xs = x + (size_t)nc * T * J;
  const int i = threadIdx.x;
  const int Jc = min(J, kHT), G = kHT / Jc;
  const int jl = i % Jc, r = i / Jc;
  for (int jb = 0; jb < J; jb += Jc) {
    const int j = jb + jl;
    const bool act = r < G && j < J;
    const int col = act ? clip_col(j, V, M) : 0;
    const float k0 = xs[col];
    float a = 0.f, q = 0.f;
    if (act) {
      for (int t0 = r; t0 < T; t0 += G * kHU) {
        float xv[kHU];
#pragma unroll
        for (int u = 0; u < kHU; ++u) xv[u] = xs[(size_t)min(t0 + u * G, T - 1) * J + col];
#pragma unroll
        for (int u = 0; u < kHU; ++u) {
          const float d = (t0 + u * G < T) ? xv[u] - k0 : 0.f;
          a += d;
          q += d * d;
        }
      }
    }
    s1[i] = a;
    s2[i] = q;
    __syncthreads();
    if (i < Jc && jb + i < J) {
      float ta = 0.f, tq = 0.f;
      for (int g = 0; g < G; ++g) { ta += s1[g * Jc + i]; tq += s2[g * Jc + i]; }
      const int jj = jb + i, m = jj / V, v = jj - m * V;
      const float nT = (float)T;
      part[(size_t)n * F + (m * V + v) * C + c] = make_float2(k0 + ta / nT, tq - ta * ta / nT);
    }
    __syncthreads();
  }
}

// y[(n*M + m), c, t, v] = x[n, c, t, v, m] * scale[f] + shift[f]. One thread per plane
// element (coalesced stores, the loads of neighbouring threads share cache lines).
// Bytes: 8 per element.
__global__ __launch_bounds__(kHT) void head_apply_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         float* __restrict__ y, long long total,
                                                         int C, int T, int V, int M) {
  SGCN_CRIT_PRIO();
  const long long i = (long long)blockIdx.x * kHT + threadIdx.x;
  if (i >= total) return;
  long long r = i;
  const int v = (int)(r % V); r /= V;
  const int t = (int)(r % T); r /= T;
  const int c = (int)(r % C); r /= C;
  const int m = (int)(r % M);
  const long long n = r / M;
  const int f = (m * V + v) * C + c;
  const float xv = x[(((n * C + c) * T + t) * V + v) * M + m];
  y[i] = xv * scale[f] + shift[f];
}

// Backward partials of data_bn: part[n][f] = {sum_t g, sum_t g*(x - mean[f])*invstd[f]},
// g the plane-layout output gradient. Grid N*C; bytes: 8 per element.
__global__ __launch_bounds__(kHT) void head_bwd_reduce_kernel(
    const float* __restrict__ g, const float* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ invstd, float2* __restrict__ part, int C, int T, int V, int M) {
  SGCN_CRIT_PRIO();
  __shared__ float s1[kHT], s2[kHT];
  const int nc = blockIdx.x, n = nc / C, c = nc - n * C;
  const int J = V * M, F = J * C;
  const float* __restrict__ xs = x + (size_t)nc * T * J;
  const size_t TV = (size_t)T * V;
  const int i = threadIdx.x;
  const int Jc = min(J, kHT), G = kHT / Jc;
  const int jl = i % Jc, r = i / Jc;
  for (int jb = 0; jb < J; jb += Jc) {
    const int j = jb + jl;
    const bool act = r < G && j < J;
    const int jc = act ? j : 0;
    const int m = jc / V, v = jc - m * V;
    const int col = v * M + m, f = (m * V + v) * C + c;
    const float* __restrict__ gp = g + (((size_t)n * M + m) * C + c) * TV + v;
    const float mu = mean[f], is = invstd[f];
    float a = 0.f, b = 0.f;
    if (act) {
      for (int t0 = r; t0 < T; t0 += G * kHU) {
        float gv[kHU], xv[kHU];
#pragma unroll
        for (int u = 0; u < kHU; ++u) {
          const int t = min(t0 + u * G, T - 1);
          gv[u] = gp[(size_t)t * V];
          xv[u] = xs[(size_t)t * J + col];
        }
#pragma unroll
        for (int u = 0; u < kHU; ++u) {
          const float gg = (t0 + u * G < T) ? gv[u] : 0.f;
          a += gg;
          b += gg * ((xv[u] - mu) * is);
        }
      }
    }
    s1[i] = a;
    s2[i] = b;
    __syncthreads();
    if (i < Jc && jb + i < J) {
      float ta = 0.f, tb = 0.f;
      for (int k = 0; k < G; ++k) { ta += s1[k * Jc + i]; tb += s2[k * Jc + i]; }
      const int jj = jb + i, mm = jj / V, vv = jj - mm * V;
      part[(size_t)n * F + (mm * V + vv) * C + c] = make_float2(ta, tb);
    }
    __syncthreads();
  }
}

// dx[n, c, t, v, m] = k1[f]*g + k2[f]*x + k3[f] (coef [3][F] from sgcn_bn_bwd_finalize),
// one thread per clip element (coalesced clip loads/stores). Bytes: 12 per element.
__global__ __launch_bounds__(kHT) void head_bwd_apply_kernel(
    const float* __restrict__ g, const float* __restrict__ x, const float* __restrict__ coef,
    float* __restrict__ dx, long long total, int C, int T, int V, int M) {
  SGCN_CRIT_PRIO();
  const long long i = (long long)blockIdx.x * kHT + threadIdx.x;
  if (i >= total) return;
  long long r = i;
  const int m = (int)(r % M); r /= M;
  const int v = (int)(r % V); r /= V;
  const int t = (int)(r % T); r /= T;
  const int c = (int)(r % C);
  const long long n = r / C;
  const int F = M * V * C, f = (m * V + v) * C + c;
  const float gv = g[(((n * M + m) * C + c) * T + t) * V + v];
  dx[i] = coef[f] * gv + coef[F + f] * x[i] + coef[2 * F + f];
}

// out[n][c] = (sum_m (sum_p x[n*M + m][c][p]) / P) / M  — x.view(N, M, C, P).mean(3).mean(1)
// with the two divisions in the reference's order. Grid N*C; bytes: 4 per element.
__global__ __launch_bounds__(kHT) void pool_kernel(const float* __restrict__ x,
                                                   float* __restrict__ out, int C, int M,
                                                   long long P) {
  SGCN_CRIT_PRIO();
  __shared__ float red[2 * kHT / 64];
  const int nc = blockIdx.x, n = nc / C, c = nc - n * C;
  float acc = 0.f;
  for (int m = 0; m < M; ++m) {
    const float* __restrict__ xp = x + (((size_t)n * M + m) * C + c) * P;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (long long p0 = threadIdx.x; p0 < P; p0 += 4 * kHT) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long p = p0 + u * kHT;
        s[u] += p < P ? xp[p] : 0.f;
      }
    }
    float tot = (s[0] + s[1]) + (s[2] + s[3]);
    tot = block_sum(tot, red);
    acc += tot * (1.f / (float)P);      // torch's mean: sum times the fp32 reciprocal
  }
  if (threadIdx.x == 0) out[nc] = acc * (1.f / (float)M);
}

// dx[n*M + m][c][p] = dout[n][c] / M / P (mean(1) then mean(3) backward, same order and
// rounding as autograd). Four consecutive elements per thread, one 16-byte store (the
// tensor base is 16-byte aligned; rows of P elements may start mid-vector, so each lane
// of the vector finds its own row). Bytes: 4 per element (the dout read is cached).
__global__ __launch_bounds__(kHT) void pool_bwd_kernel(const float* __restrict__ dout,
                                                       float* __restrict__ dx, long long total,
                                                       int C, int M, long long P) {
  SGCN_CRIT_PRIO();
  const long long i0 = ((long long)blockIdx.x * kHT + threadIdx.x) * 4;
  if (i0 >= total) return;
  const float rm = 1.f / (float)M, rp = 1.f / (float)P;
  float v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long row = (i0 + u) / P;        // (n*M + m)*C + c
    const int c = (int)(row % C);
    const long long n = row / C / M;
    // autograd's mean backward divides by a CPU scalar, which the device kernel turns into
    // a multiply by the fp32 reciprocal: (dout * (1/M)) * (1/P)
    v[u] = i0 + u < total ? (dout[n * C + c] * rm) * rp : 0.f;
  }
  if (i0 + 4 <= total) {
    *reinterpret_cast<float4*>(dx + i0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    for (int u = 0; u < 4 && i0 + u < total; ++u) dx[i0 + u] = v[u];
  }
}

unsigned grid1(long long total) { return (unsigned)((total + kHT - 1) / kHT); }

}  // namespace
}  // namespace sgcn

using namespace sgcn;

extern "C" {

size_t sgcn_head_ws_bytes(int N, int C, int V, int M) {
  return (size_t)(N > 0 ? N : 0) * C * V * M * sizeof(float2);
}

int sgcn_head_moments(const float* x, float* part, int N, int C, int T, int V, int M,
                      void* stream) {
  SGCN_REQUIRE(N >= 0 && C > 0 && T > 0 && V > 0 && M > 0);
  if (N == 0) return 0;
  SGCN_REQUIRE(x && part);
  SGCN_REQUIRE((long long)N * C < (1ll << 31) && (long long)T * V * M < (1ll << 31));
  head_moments_kernel<<<N * C, kHT, 0, (hipStream_t)stream>>>(x, (float2*)part, C, T, V, M);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_head_apply(const float* x, const float* scale, const float* shift, float* y, int N,
                    int C, int T, int V, int M, void* stream) {
  SGCN_REQUIRE(N >= 0 && C > 0 && T > 0 && V > 0 && M > 0);
  const long long total = (long long)N * M * C * T * V;
  if (total == 0) return 0;
  SGCN_REQUIRE(x && scale && shift && y);
  SGCN_REQUIRE(total < (1ll << 40));
  head_apply_kernel<<<grid1(total), kHT, 0, (hipStream_t)stream>>>(x, scale, shift, y, total,
                                                                    C, T, V, M);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_head_bwd_reduce(const float* g, const float* x, const float* mean, const float* invstd,
                         float* part, int N, int C, int T, int V, int M, void* stream) {
  SGCN_REQUIRE(N >= 0 && C > 0 && T > 0 && V > 0 && M > 0);
  if (N == 0) return 0;
  SGCN_REQUIRE(g && x && mean && invstd && part);
  SGCN_REQUIRE((long long)N * C < (1ll << 31) && (long long)T * V * M < (1ll << 31));
  head_bwd_reduce_kernel<<<N * C, kHT, 0, (hipStream_t)stream>>>(g, x, mean, invstd,
                                                                 (float2*)part, C, T, V, M);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_head_bwd_apply(const float* g, const float* x, const float* coef, float* dx, int N,
                        int C, int T, int V, int M, void* stream) {
  SGCN_REQUIRE(N >= 0 && C > 0 && T > 0 && V > 0 && M > 0);
  const long long total = (long long)N * M * C * T * V;
  if (total == 0) return 0;
  SGCN_REQUIRE(g && x && coef && dx);
  SGCN_REQUIRE(total < (1ll << 40));
  head_bwd_apply_kernel<<<grid1(total), kHT, 0, (hipStream_t)stream>>>(g, x, coef, dx, total, C,
                                                                        T, V, M);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_pool(const float* x, float* out, int N, int M, int C, long long P, void* stream) {
  SGCN_REQUIRE(N >= 0 && M > 0 && C > 0 && P > 0);
  if (N == 0) return 0;
  SGCN_REQUIRE(x && out);
  SGCN_REQUIRE((long long)N * C < (1ll << 31));
  pool_kernel<<<N * C, kHT, 0, (hipStream_t)stream>>>(x, out, C, M, P);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_pool_bwd(const float* dout, float* dx, int N, int M, int C, long long P,
                  void* stream) {
  SGCN_REQUIRE(N >= 0 && M > 0 && C > 0 && P > 0);
  const long long total = (long long)N * M * C * P;
  if (total == 0) return 0;
  SGCN_REQUIRE(dout && dx && ((uintptr_t)dx & 15) == 0);   // 16-byte vector stores
  SGCN_REQUIRE(total < (1ll << 40));
  pool_bwd_kernel<<<grid1((total + 3) / 4), kHT, 0, (hipStream_t)stream>>>(dout, dx, total, C,
                                                                           M, P);
  SGCN_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
