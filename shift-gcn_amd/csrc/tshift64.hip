// Double-precision temporal shift (the reference's AT_DISPATCH_FLOATING_TYPES double
// instantiation, shift_cuda_kernel.cu:413, :455-520): forward, input gradient and the
// constrained position gradients on float64 tensors, e.g. for torch.autograd.gradcheck of
// the input gradient (the exact adjoint) or float64 conditioning studies.
//
// Not on the training hot path (fp32): one 256-thread workgroup per (b, c) plane, taps
// straight from global memory (L1/L2-resident: a plane is <= 60 KB at the model's sizes),
// per-plane double position sums merged per channel in a fixed order (deterministic).
// Arithmetic follows the reference expression order with contraction disabled, including
// `int x1 = floorf(x)` (floorf is the FLOAT function: a double x is rounded to float
// first) and `1 - dx` etc. in double.
#include "common.hpp"

#pragma clang fp contract(off)

namespace sgcn {
namespace {

constexpr int kT64 = 256;

struct Geom64 {
  int x1, y1;
  double dx, dy;
};

__device__ __forceinline__ Geom64 geom64(double x, double y) {
  Geom64 g;
  g.x1 = (int)floorf((float)x);
  g.y1 = (int)floorf((float)y);
  g.dx = x - (double)g.x1;
  g.dy = y - (double)g.y1;
  return g;
}

__device__ __forceinline__ double tap64(const double* p, int h, int w, int H, int W) {
  return (h >= 0 && w >= 0 && h < H && w < W) ? p[h * W + w] : 0.0;
}

// stride-2 bottom-backward tap (.cu:203-248): only for an even row (C++ remainder), then
// row / 2 (truncation) bounds-checked on the top grid
__device__ __forceinline__ double tap64_s2(const double* p, int h, int w, int Ht, int W) {
  if (h % 2 != 0) return 0.0;
  return tap64(p, h / 2, w, Ht, W);
}

__device__ __forceinline__ double blend64(double q11, double q21, double q12, double q22,
                                          double dx, double dy) {
  return q11 * (1 - dx) * (1 - dy) + q21 * dx * (1 - dy) + q12 * (1 - dx) * dy + q22 * dx * dy;
}

__global__ __launch_bounds__(kT64) void tshift64_fwd_kernel(const double* __restrict__ in,
                                                            double* __restrict__ out,
                                                            const double* __restrict__ xpos,
                                                            const double* __restrict__ ypos,
                                                            int C, int H, int W, int Ho,
                                                            int stride, int add_half) {
  const int plane = blockIdx.x, c = plane % C;
  const double* src = in + (size_t)plane * H * W;
  double* dst = out + (size_t)plane * Ho * W;
  const double y = add_half ? ypos[c] + 0.5 : ypos[c];
  const Geom64 g = geom64(xpos[c], y);
  for (int o = threadIdx.x; o < Ho * W; o += kT64) {
    const int h = o / W, w = o - (o / W) * W;
    const int hi = h * stride + g.y1, wi = w + g.x1;
    dst[o] = blend64(tap64(src, hi, wi, H, W), tap64(src, hi, wi + 1, H, W),
                     tap64(src, hi + 1, wi, H, W), tap64(src, hi + 1, wi + 1, H, W), g.dx, g.dy);
  }
}

__device__ __forceinline__ void block_sum2_d(double& a, double& b, double* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  __syncthreads();
  if (lane == 0) { red[2 * wid] = a; red[2 * wid + 1] = b; }
  __syncthreads();
  double sa = 0.0, sb = 0.0;
  for (int i = 0; i < nw; ++i) { sa += red[2 * i]; sb += red[2 * i + 1]; }
  a = sa;
  b = sb;
}

__global__ __launch_bounds__(kT64) void tshift64_bwd_kernel(
    const double* __restrict__ gout, const double* __restrict__ in,
    const double* __restrict__ xpos, const double* __restrict__ ypos, double* __restrict__ gin,
    double2* __restrict__ pgrad, int C, int H, int W, int Ho, int stride, int add_half) {
  __shared__ double red[2 * kT64 / 64];
  const int plane = blockIdx.x, c = plane % C;
  const double* go = gout + (size_t)plane * Ho * W;
  const double* src = in + (size_t)plane * H * W;
  double* gi = gin + (size_t)plane * H * W;
  const double x = xpos[c];
  const double y = add_half ? ypos[c] + 0.5 : ypos[c];
  // (1) input gradient over the bottom grid (.cu:78-152 stride 1, .cu:155-256 stride 2)
  const Geom64 r = geom64(-x, -y);
  for (int o = threadIdx.x; o < H * W; o += kT64) {
    const int h = o / W, w = o - (o / W) * W;
    const int h1 = h + r.y1, w1 = w + r.x1;
    double q11, q21, q12, q22;
    if (stride == 1) {
      q11 = tap64(go, h1, w1, Ho, W);
      q21 = tap64(go, h1, w1 + 1, Ho, W);
      q12 = tap64(go, h1 + 1, w1, Ho, W);
      q22 = tap64(go, h1 + 1, w1 + 1, Ho, W);
    } else {
      q11 = tap64_s2(go, h1, w1, Ho, W);
      q21 = tap64_s2(go, h1, w1 + 1, Ho, W);
      q12 = tap64_s2(go, h1 + 1, w1, Ho, W);
      q22 = tap64_s2(go, h1 + 1, w1 + 1, Ho, W);
    }
    gi[o] = blend64(q11, q21, q12, q22, r.dx, r.dy);
  }
  // (2) position products over the top grid (.cu:321-349), summed over the plane
  const Geom64 g = geom64(x, y);
  double ax = 0.0, ay = 0.0;
  for (int o = threadIdx.x; o < Ho * W; o += kT64) {
    const int h = o / W, w = o - (o / W) * W;
    const int hi = h * stride + g.y1, wi = w + g.x1;
    const double q11 = tap64(src, hi, wi, H, W), q21 = tap64(src, hi, wi + 1, H, W);
    const double q12 = tap64(src, hi + 1, wi, H, W), q22 = tap64(src, hi + 1, wi + 1, H, W);
    const double vx = (1 - g.dy) * (q21 - q11) + g.dy * (q22 - q12);
    const double vy = (1 - g.dx) * (q12 - q11) + g.dx * (q22 - q21);
    ax += vx * go[o];
    ay += vy * go[o];
  }
  block_sum2_d(ax, ay, red);
  if (threadIdx.x == 0) pgrad[plane] = make_double2(ax, ay);
}

// mean over the batch of the plane sums (.cu:501-509 up to summation order), then
// applyShiftConstraint<double> (.cu:370-395): dx/dr*0.0, dy/dr*0.01, or 0 / 1e-4 if dr == 0
__global__ __launch_bounds__(256) void tshift64_finalize_kernel(const double2* __restrict__ pg,
                                                                int B, int C,
                                                                double* __restrict__ gx,
                                                                double* __restrict__ gy) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sx = 0.0, sy = 0.0;
  for (int b = 0; b < B; ++b) {
    const double2 p = pg[(size_t)b * C + c];
    sx += p.x;
    sy += p.y;
  }
  const double Gx = sx / B, Gy = sy / B;
  const double dr = sqrt(Gy * Gy);
  if (dr != 0) {
    gx[c] = Gx / dr * 0.0;
    gy[c] = Gy / dr * 0.01;
  } else {
    gx[c] = 0.0;
    gy[c] = 0.0001;
  }
}

}  // namespace
}  // namespace sgcn

using namespace sgcn;

extern "C" {

int sgcn_tshift_fwd_f64(const double* in, double* out, const double* xpos, const double* ypos,
                        int B, int C, int H, int W, int stride, int ypos_is_raw, void* stream) {
  SGCN_REQUIRE(B >= 0 && C > 0 && H >= 0 && W > 0 && stride >= 1);
  const int Ho = H / stride;
  if (B == 0 || Ho == 0) return 0;
  SGCN_REQUIRE(in && out && xpos && ypos);
  SGCN_REQUIRE((long long)H * W < (1LL << 30) && (long long)B * C < (1LL << 31));
  tshift64_fwd_kernel<<<B * C, kT64, 0, (hipStream_t)stream>>>(
      in, out, xpos, ypos, C, H, W, Ho, stride, (ypos_is_raw && stride != 1) ? 1 : 0);
  SGCN_LAUNCH_CHECK();
  return 0;
}

size_t sgcn_tshift_bwd_f64_ws_bytes(int B, int C) { return (size_t)B * C * sizeof(double2); }

int sgcn_tshift_bwd_f64(const double* gout, const double* in, const double* xpos,
                        const double* ypos, double* gin, double* gx, double* gy, void* ws,
                        size_t ws_bytes, int B, int C, int H, int W, int stride,
                        int ypos_is_raw, void* stream) {
  SGCN_REQUIRE(B > 0 && C > 0 && H >= 0 && W > 0 && (stride == 1 || stride == 2));
  const int Ho = H / stride;
  SGCN_REQUIRE((gout || Ho == 0) && (in || H == 0) && (gin || H == 0));
  SGCN_REQUIRE(xpos && ypos && gx && gy && ws);
  SGCN_REQUIRE(ws_bytes >= sgcn_tshift_bwd_f64_ws_bytes(B, C));
  SGCN_REQUIRE((long long)H * W < (1LL << 30) && (long long)B * C < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  double2* pg = (double2*)ws;
  tshift64_bwd_kernel<<<B * C, kT64, 0, st>>>(gout, in, xpos, ypos, gin, pg, C, H, W, Ho,
                                              stride, (ypos_is_raw && stride != 1) ? 1 : 0);
  SGCN_LAUNCH_CHECK();
  tshift64_finalize_kernel<<<(C + 255) / 256, 256, 0, st>>>(pg, B, C, gx, gy);
  SGCN_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
