// Learnable fractional temporal shift on gfx950 (MI355X).
//
// Replaces the reference CUDA extension `shift_cuda`
// (model/Temporal_shift/cuda/shift_cuda_kernel.cu, shift_cuda.cpp:44-47):
//   forward : shift_cuda_forward_kernel (.cu:11-76) + launcher (.cu:405-431)
//   backward: Shift_Bottom_Backward_Stride1 / Shift_Bottom_Backward (.cu:78-256),
//             Shift_Position_Backward (.cu:277-363), the ATen mean/sum reductions
//             (.cu:501-509) and applyShiftConstraint (.cu:370-395).
//
// MI355X design (not a translation):
//  * one 256-thread workgroup per (n·m, c) plane of the (N·M, C, T, V) layout: the
//    plane is one contiguous T·V run, so the shift's integer part is an address offset
//    and all four taps of a wave are coalesced (they re-hit the same lines in L1);
//  * per-channel shift geometry is computed once per workgroup (SGPR-uniform);
//  * the backward fuses the input gradient, the position-gradient products and their
//    per-plane reduction in ONE pass: the reference's two (B,C,Ho,W) temporaries
//    (.cu:480-481, 2x245.8 MB at NTU l2) and its three ATen reductions never exist;
//    per-plane partials are combined in a fixed order by a C-thread finalize kernel,
//    so gx/gy are bit-reproducible run to run;
//  * optional fusions used by the Shift_tcn pipeline: a per-channel affine applied to
//    every in-range input tap (BatchNorm apply folded into the shift's gather), ReLU
//    masking of the input gradient, and per-plane output moments (BatchNorm stats of
//    the shift output, two-pass exact within a plane, Chan-merged in double later).
//
// Arithmetic follows the reference expression order with contraction disabled, so
// outputs are bit-identical to the oracle restatement (oracle/shift_oracle.py).
#include "common.hpp"

#pragma clang fp contract(off)

namespace sgcn {
namespace {

constexpr int kThreads = 256;

// kReverse note: every shift kernel walks its planes last to first. Its main input was
// written front to back just before it (the contraction output R, the gcn tail's H, the
// next unit's input gradient), so the last planes are still in the die-level cache; and
// the contraction that consumes its output (front to back) then starts on the planes it
// wrote last.

struct Geom {
  int x1, y1;
  float dx, dy;
};

// `int x1 = floorf(x); dx = x - x1;` (.cu:49-71)
__device__ __forceinline__ Geom make_geom(float x, float y) {
  Geom g;
  g.x1 = (int)floorf(x);
  g.y1 = (int)floorf(y);
  g.dx = x - (float)g.x1;
  g.dy = y - (float)g.y1;
  return g;
}

// q11*(1-dx)*(1-dy) + q21*dx*(1-dy) + q12*(1-dx)*dy + q22*dx*dy, left to right (.cu:73)
__device__ __forceinline__ float blend(float q11, float q21, float q12, float q22, float dx,
                                       float dy) {
  const float omdx = 1.f - dx, omdy = 1.f - dy;
  return q11 * omdx * omdy + q21 * dx * omdy + q12 * omdx * dy + q22 * dx * dy;
}

// Position of element `o` of a W-wide plane, advanced by blockDim per step without
// integer division in the loop.
struct Walker {
  int h, w, dh, dw, W;
  __device__ __forceinline__ Walker(int o0, int step, int W_) : W(W_) {
    h = o0 / W_;
    w = o0 - h * W_;
    dh = step / W_;
    dw = step - dh * W_;
  }
  __device__ __forceinline__ void next() {
    h += dh;
    w += dw;
    if (w >= W) { w -= W; ++h; }
  }
};

// Loads are issued in explicit two-phase sub-chunks of SUB elements per thread: all
// 4*SUB taps first, then the arithmetic and the stores. Interleaving a store per element
// (the output may alias the input as far as the compiler knows) serialises every tap
// load behind a vmcnt wait; batched, 4*SUB loads per thread are in flight.
constexpr int SUB = 8;

struct TapIdx {
  int o00, o01, o10, o11;  // clamped in-bounds offsets of the 4 taps
  float m00, m01, m10, m11;  // 1 where the tap is in range, else 0 (applied as a select)
};

__device__ __forceinline__ void tap_idx(int r, int c, int H, int W, TapIdx& t) {
  const bool r0 = (unsigned)r < (unsigned)H, r1 = (unsigned)(r + 1) < (unsigned)H;
  const bool c0 = (unsigned)c < (unsigned)W, c1 = (unsigned)(c + 1) < (unsigned)W;
  const int rr0 = min(max(r, 0), H - 1), rr1 = min(max(r + 1, 0), H - 1);
  const int cc0 = min(max(c, 0), W - 1), cc1 = min(max(c + 1, 0), W - 1);
  t.o00 = rr0 * W + cc0;
  t.o01 = rr0 * W + cc1;
  t.o10 = rr1 * W + cc0;
  t.o11 = rr1 * W + cc1;
  t.m00 = (r0 && c0) ? 1.f : 0.f;
  t.m01 = (r0 && c1) ? 1.f : 0.f;
  t.m10 = (r1 && c0) ? 1.f : 0.f;
  t.m11 = (r1 && c1) ? 1.f : 0.f;
}

// select without a branch: in-range -> v, else exact +0
__device__ __forceinline__ float sel(float v, float m) { return m != 0.f ? v : 0.f; }

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
template <int EPT, bool AFFINE, bool STATS>
__global__ __launch_bounds__(kThreads) void tshift_fwd_kernel(
    const float* __restrict__ in, float* __restrict__ out, const float* __restrict__ xpos,
    const float* __restrict__ ypos, const float* __restrict__ scale,
    const float* __restrict__ shift, float2* __restrict__ pstats, int C, int Hb, int W,
    int Ho, int stride, int add_half) {
  SGCN_CRIT_PRIO();
  __shared__ float red[2 * kThreads / 64];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  const float* __restrict__ src = in + (size_t)plane * Hb * W;
  float* __restrict__ dst = out + (size_t)plane * Ho * W;
  const float y = add_half ? ypos[c] + 0.5f : ypos[c];   // shift.py:17-18 (fp32 add)
  const Geom g = make_geom(xpos[c], y);
  float a = 1.f, b = 0.f;
  if (AFFINE) { a = scale[c]; b = shift[c]; }
  const int n = Ho * W;
  double run_n = 0.0, run_mean = 0.0, run_m2 = 0.0;  // block-uniform (STATS only)

  for (int base = 0; base < n; base += EPT * kThreads) {
    float v[EPT];
    Walker pos(base + threadIdx.x, kThreads, W);
#pragma unroll
    for (int s0 = 0; s0 < EPT; s0 += SUB) {
      float q[SUB][4];
      TapIdx ti[SUB];
#pragma unroll
      for (int e = 0; e < SUB; ++e) {
        tap_idx(pos.h * stride + g.y1, pos.w + g.x1, Hb, W, ti[e]);
        q[e][0] = src[ti[e].o00];
        q[e][1] = src[ti[e].o01];
        q[e][2] = src[ti[e].o10];
        q[e][3] = src[ti[e].o11];
        pos.next();
      }
#pragma unroll
      for (int e = 0; e < SUB; ++e) {
        float q11 = q[e][0], q21 = q[e][1], q12 = q[e][2], q22 = q[e][3];
        if (AFFINE) { q11 = q11 * a + b; q21 = q21 * a + b; q12 = q12 * a + b; q22 = q22 * a + b; }
        q11 = sel(q11, ti[e].m00);
        q21 = sel(q21, ti[e].m01);
        q12 = sel(q12, ti[e].m10);
        q22 = sel(q22, ti[e].m11);
        const int o = base + (s0 + e) * kThreads + threadIdx.x;
        const float val = blend(q11, q21, q12, q22, g.dx, g.dy);
        v[s0 + e] = o < n ? val : 0.f;
        if (o < n) dst[o] = val;
      }
    }
    if (STATS) {
      const int cnt = min(n - base, EPT * kThreads);
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < EPT; ++e) s += v[e];  // invalid slots hold 0
      s = block_sum(s, red);
      const float mean = s / (float)cnt;
      float m2 = 0.f;
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        const int o = base + e * kThreads + threadIdx.x;
        const float d = v[e] - mean;
        m2 += (o < n) ? d * d : 0.f;
      }
      m2 = block_sum(m2, red);
      const Moments m = merge({run_n, run_mean, run_m2}, {(double)cnt, (double)mean, (double)m2});
      run_n = m.n;
      run_mean = m.mean;
      run_m2 = m.m2;
    }
  }
  if (STATS && threadIdx.x == 0) pstats[plane] = make_float2((float)run_mean, (float)run_m2);
}

// ------------------------------------------------------------------------------------
// backward: input gradient (reverse shift) + position-gradient plane partials
// ------------------------------------------------------------------------------------
// BNP: also emit the per-plane BatchNorm-backward partials {sum gin, sum gin*xhat},
// xhat = (in - bn_mean[c]) * bn_invstd[c], of the BatchNorm that produced this shift's
// input (Shift_tcn.bn before shift_in): its separate reduction pass disappears.
template <int EPT, bool AFFINE, bool RELU_MASK, int STRIDE, bool BNP>
__global__ __launch_bounds__(kThreads) void tshift_bwd_kernel(
    const float* __restrict__ gout, const float* __restrict__ in,
    const float* __restrict__ xpos, const float* __restrict__ ypos,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ bn_mean, const float* __restrict__ bn_invstd,
    float* __restrict__ gin, float2* __restrict__ pgrad, float2* __restrict__ bn_part, int C,
    int Hb, int W, int Ho, int add_half) {
  SGCN_CRIT_PRIO();
  __shared__ float red[2 * kThreads / 64];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  float bs0 = 0.f, bs1 = 0.f, bmu = 0.f, bis = 0.f;
  if (BNP) { bmu = bn_mean[c]; bis = bn_invstd[c]; }   // this plane's channel
  const float* __restrict__ go = gout + (size_t)plane * Ho * W;
  const float* __restrict__ src = in + (size_t)plane * Hb * W;
  float* __restrict__ gi = gin + (size_t)plane * Hb * W;
  const float x = xpos[c];
  const float y = add_half ? ypos[c] + 0.5f : ypos[c];
  float a = 1.f, b = 0.f;
  if (AFFINE) { a = scale[c]; b = shift[c]; }

  // (1) grad_input over the bottom grid: bilinear sample of grad_output at (-x, -y)
  //     (.cu:108-150 stride 1; .cu:191-254 stride 2 with the even-row rule)
  if (Ho == 0) {  // empty top grid: every tap is out of range (and must not be read)
    for (int o = threadIdx.x; o < Hb * W; o += kThreads) gi[o] = 0.f;
  } else {
    const Geom r = make_geom(-x, -y);
    const int nb = Hb * W;
    for (int base = 0; base < nb; base += EPT * kThreads) {
      Walker pos(base + threadIdx.x, kThreads, W);
#pragma unroll
      for (int s0 = 0; s0 < EPT; s0 += SUB) {
        float q[SUB][4], rin[SUB];
        TapIdx ti[SUB];
#pragma unroll
        for (int e = 0; e < SUB; ++e) {
          const int h1 = pos.h + r.y1;
          const int w1 = pos.w + r.x1;
          if (STRIDE == 1) {
            tap_idx(h1, w1, Ho, W, ti[e]);
          } else {
            // h_im % 2 == 0 (C++ remainder), then h_im / 2 (truncation), bounds on the top
            // grid; exactly one of h1, h1+1 is even
            const int h2 = h1 + 1;
            const int hq1 = (h1 % 2 == 0) ? h1 / 2 : -1;
            const int hq2 = (h2 % 2 == 0) ? h2 / 2 : -1;
            TapIdx t1, t2;
            tap_idx(hq1, w1, Ho, W, t1);
            tap_idx(hq2, w1, Ho, W, t2);
            ti[e].o00 = t1.o00; ti[e].o01 = t1.o01; ti[e].m00 = t1.m00; ti[e].m01 = t1.m01;
            ti[e].o10 = t2.o00; ti[e].o11 = t2.o01; ti[e].m10 = t2.m00; ti[e].m11 = t2.m01;
          }
          q[e][0] = go[ti[e].o00];
          q[e][1] = go[ti[e].o01];
          q[e][2] = go[ti[e].o10];
          q[e][3] = go[ti[e].o11];
          if (RELU_MASK || BNP)
            rin[e] = src[min(base + (s0 + e) * kThreads + (int)threadIdx.x, nb - 1)];
          pos.next();
        }
#pragma unroll
        for (int e = 0; e < SUB; ++e) {
          const float q11 = sel(q[e][0], ti[e].m00), q21 = sel(q[e][1], ti[e].m01);
          const float q12 = sel(q[e][2], ti[e].m10), q22 = sel(q[e][3], ti[e].m11);
          float val = blend(q11, q21, q12, q22, r.dx, r.dy);
          if (RELU_MASK) val = rin[e] > 0.f ? val : 0.f;
          const int o = base + (s0 + e) * kThreads + threadIdx.x;
          if (o < nb) gi[o] = val;
          if (BNP) {
            const float gv = o < nb ? val : 0.f;
            bs0 += gv;
            bs1 += gv * ((rin[e] - bmu) * bis);
          }
        }
      }
    }
  }

  // (2) position gradients over the top grid (.cu:321-349), summed over the plane
  float ax = 0.f, ay = 0.f;
  {
    const Geom g = make_geom(x, y);
    const int nt = Ho * W;
    for (int base = 0; base < nt; base += EPT * kThreads) {
      Walker pos(base + threadIdx.x, kThreads, W);
#pragma unroll
      for (int s0 = 0; s0 < EPT; s0 += SUB) {
        float q[SUB][4], gv[SUB];
        TapIdx ti[SUB];
#pragma unroll
        for (int e = 0; e < SUB; ++e) {
          tap_idx(pos.h * STRIDE + g.y1, pos.w + g.x1, Hb, W, ti[e]);
          q[e][0] = src[ti[e].o00];
          q[e][1] = src[ti[e].o01];
          q[e][2] = src[ti[e].o10];
          q[e][3] = src[ti[e].o11];
          gv[e] = go[min(base + (s0 + e) * kThreads + (int)threadIdx.x, nt - 1)];
          pos.next();
        }
#pragma unroll
        for (int e = 0; e < SUB; ++e) {
          float q11 = q[e][0], q21 = q[e][1], q12 = q[e][2], q22 = q[e][3];
          if (AFFINE) { q11 = q11 * a + b; q21 = q21 * a + b; q12 = q12 * a + b; q22 = q22 * a + b; }
          q11 = sel(q11, ti[e].m00);
          q21 = sel(q21, ti[e].m01);
          q12 = sel(q12, ti[e].m10);
          q22 = sel(q22, ti[e].m11);
          const float vx = (1.f - g.dy) * (q21 - q11) + g.dy * (q22 - q12);
          const float vy = (1.f - g.dx) * (q12 - q11) + g.dx * (q22 - q21);
          const int o = base + (s0 + e) * kThreads + threadIdx.x;
          const float gg = o < nt ? gv[e] : 0.f;
          ax += vx * gg;
          ay += vy * gg;
        }
      }
    }
  }
  block_sum2(ax, ay, red);
  if (threadIdx.x == 0) pgrad[plane] = make_float2(ax, ay);
  if (BNP) {
    block_sum2(bs0, bs1, red);
    if (threadIdx.x == 0) bn_part[plane] = make_float2(bs0, bs1);
  }
}

// ------------------------------------------------------------------------------------
// LDS-staged variants (the product path whenever the plane fits): every element of the
// plane(s) crosses HBM exactly once with fully coalesced dword loads, and the four taps
// of each output are LDS reads (conflict-free: a wave reads 64 consecutive words).
// Same expressions in the same order as the global-tap kernels above, so the results
// are bit-identical to them (and to the oracle).
// ------------------------------------------------------------------------------------
constexpr int kFwdLdsMax = 8192;    // floats of the staged input plane (32 KiB), 256 threads
constexpr int kFwdLdsMax2 = 16384;  // ... with 512 threads (e.g. MediaPipe T=300: 9,900)
constexpr int kBwdLdsMax = 16384;   // floats of the staged gout + input planes (64 KiB)

// Zero-padded LDS planes (the stride-1 backward and the forward kernels below): an H x W
// plane is staged with row pitch WP = W + 2 (a zero column each side) between kPadRows
// zero rows above and below, element (h, w) at [(h + kPadRows) * WP + w + 1]; a tap of a
// shift with floor(x) in {-1, 0} and |floor(y)| < kPadRows then needs no range check.
constexpr int kPadRows = 4;

__host__ __device__ constexpr int ra_pad_floats(int H, int W) { return (H + 2 * kPadRows) * (W + 2); }

// zero the padding of a padded H x W plane (NT threads)
template <int NT>
__device__ __forceinline__ void zero_pad(float* lds, int H, int W) {
  const int WP = W + 2, nprow = 2 * kPadRows * WP;
  for (int i = (int)threadIdx.x; i < nprow + 2 * H; i += NT) {
    int a;
    if (i < nprow) {
      const int r = i / WP, col = i - r * WP;
      a = (r < kPadRows ? r : H + r) * WP + col;
    } else {
      const int j = i - nprow;
      a = ((j >> 1) + kPadRows) * WP + ((j & 1) ? W + 1 : 0);
    }
    lds[a] = 0.f;
  }
}

// copy n floats src -> lds (optionally x*a+b), all loads of a thread issued before any
// LDS store; n <= LPT * NT
template <int NT, int LPT, bool AFFINE>
__device__ __forceinline__ void stage_plane(const float* __restrict__ src, float* lds, int n,
                                            float a, float b) {
  float t[LPT];
#pragma unroll
  for (int e = 0; e < LPT; ++e) t[e] = src[min(e * NT + (int)threadIdx.x, n - 1)];
#pragma unroll
  for (int e = 0; e < LPT; ++e) {
    const int i = e * NT + threadIdx.x;
    if (i < n) lds[i] = AFFINE ? t[e] * a + b : t[e];
  }
}

// The W > 64 fallback of tshift_fwd_pad_kernel (every plane of the model takes that one).
template <int NT, int EPT, int LPT, bool AFFINE, bool STATS>
__global__ __launch_bounds__(NT) void tshift_fwd_lds_kernel(
    const float* __restrict__ in, float* __restrict__ out, const float* __restrict__ xpos,
    const float* __restrict__ ypos, const float* __restrict__ scale,
    const float* __restrict__ shift, float2* __restrict__ pstats, int C, int Hb, int W,
    int Ho, int stride, int add_half) {
  SGCN_CRIT_PRIO();
  extern __shared__ float pl[];   // Hb*W staged input (affine applied)
  __shared__ float red[2 * NT / 64];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  float* __restrict__ dst = out + (size_t)plane * Ho * W;
  const float y = add_half ? ypos[c] + 0.5f : ypos[c];   // shift.py:17-18 (fp32 add)
  const Geom g = make_geom(xpos[c], y);
  float a = 1.f, b = 0.f;
  if (AFFINE) { a = scale[c]; b = shift[c]; }
  stage_plane<NT, LPT, AFFINE>(in + (size_t)plane * Hb * W, pl, Hb * W, a, b);
  __syncthreads();
  const int n = Ho * W;
  double run_n = 0.0, run_mean = 0.0, run_m2 = 0.0;  // block-uniform (STATS only)
  for (int base = 0; base < n; base += EPT * NT) {
    float v[EPT];
    {
      Walker pos(base + threadIdx.x, NT, W);
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        TapIdx ti;
        tap_idx(pos.h * stride + g.y1, pos.w + g.x1, Hb, W, ti);
        const float q11 = sel(pl[ti.o00], ti.m00), q21 = sel(pl[ti.o01], ti.m01);
        const float q12 = sel(pl[ti.o10], ti.m10), q22 = sel(pl[ti.o11], ti.m11);
        const int o = base + e * NT + threadIdx.x;
        const float val = blend(q11, q21, q12, q22, g.dx, g.dy);
        v[e] = o < n ? val : 0.f;
        if (o < n) dst[o] = val;
        pos.next();
      }
    }
    if (STATS) {
      const int cnt = min(n - base, EPT * NT);
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < EPT; ++e) s += v[e];
      s = block_sum(s, red);
      const float mean = s / (float)cnt;
      float m2 = 0.f;
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        const int o = base + e * NT + threadIdx.x;
        const float d = v[e] - mean;
        m2 += o < n ? d * d : 0.f;
      }
      m2 = block_sum(m2, red);
      const Moments m = merge({run_n, run_mean, run_m2}, {(double)cnt, (double)mean, (double)m2});
      run_n = m.n;
      run_mean = m.mean;
      run_m2 = m.m2;
    }
  }
  if (STATS && threadIdx.x == 0) pstats[plane] = make_float2((float)run_mean, (float)run_m2);
}

// Forward on a zero-padded LDS plane (the product kernel for W <= 64): staged and walked on
// the joint-aligned element stride NTJ = (NT / W) * W, so a thread's joint is fixed, its
// staged elements and its outputs sit at a per-thread base plus a uniform step, and, for a
// channel whose shift stays inside the padding (every channel of a trained model), each of
// the four taps is an unconditional LDS read (the padding supplies the reference's exact
// +0 for an out-of-range tap). A channel whose shift leaves the padding takes the same
// loop with range-checked taps. Global traffic through buffer descriptors (no clamps;
// stores past the plane drop). Same expressions in the same order as tshift_fwd_kernel:
// outputs bit-identical.
//   MODE 0: the shift (sgcn_tshift_fwd), optional affine taps; STATS: two-pass
//           {mean, M2} of the whole plane (every output of the plane is in this
//           workgroup's registers).
//   MODE 1: the inference Shift_gcn tail fused into the following shift_in forward
//           (shift_gcn.py:137-141 then :67-68, BatchNorms in eval mode): the staged input
//           element is a * relu(z*zs[c*W + w] + zt[c*W + w] + res) + b, z the contraction
//           output (natural layout), res = r (RES 1, identity down) or r*rs[c] + rt[c]
//           (RES 2, down conv + eval BN), a/b = Shift_tcn.bn (eval); H is never written.
//   MODE 2: the inference unit tail fused into the shift_out forward (shift_gcn.py:72-73 +
//           161-162, eval): out = relu(S*ps[c] + pt[c] + res), S the shifted value, res = 0 /
//           r / r*rs[c] + rt[c] read at the output address; GOUT: also the next Shift_gcn's
//           gathered, masked input og[c,t,(v - c) mod V] = out[c,t,v] * gm[((v - c) mod V)*C
//           + c]. S is never written.
// A thread's joint is fixed, so the per-joint tables (zs/zt, the gather's mask and target
// joint) are per-thread constants.
template <int NT, int LPT, int MODE, bool AFFINE, bool STATS, int RES = 0, bool GOUT = false>
__global__ __launch_bounds__(NT) void tshift_fwd_pad_kernel(
    const float* __restrict__ in, float* __restrict__ out, const float* __restrict__ xpos,
    const float* __restrict__ ypos, const float* __restrict__ scale,
    const float* __restrict__ shift, float2* __restrict__ pstats, int C, int Hb, int W,
    int Ho, int stride, int add_half, const float* __restrict__ zs = nullptr,
    const float* __restrict__ zt = nullptr, const float* __restrict__ r = nullptr,
    const float* __restrict__ rs = nullptr, const float* __restrict__ rt = nullptr,
    const float* __restrict__ gm = nullptr, float* __restrict__ og = nullptr) {
  SGCN_CRIT_PRIO();
  static_assert(MODE != 1 || (AFFINE && RES >= 1 && !STATS), "pre: affine taps of relu(...)");
  static_assert(MODE != 2 || (!AFFINE && !STATS), "tail: plain taps");
  extern __shared__ float pl[];   // padded Hb x W input plane (affine applied) + 1 spare
  __shared__ float red[2 * NT / 64];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  const int WP = W + 2, GR = NT / W, NTJ = GR * W;
  const int tid = threadIdx.x;
  const bool own = tid < NTJ;
  const int w = tid % W, h0 = tid / W;
  const int nb = Hb * W, n = Ho * W;
  const unsigned vo = own ? (unsigned)tid * 4u : 0x80000000u, vstep = (unsigned)NTJ * 4u;
  float a = 1.f, b = 0.f;
  if (AFFINE) { a = scale[c]; b = shift[c]; }
  float q1 = 1.f, q2 = 0.f;   // residual BatchNorm (RES 2)
  if (RES == 2) { q1 = rs[c]; q2 = rt[c]; }
  {
    const auto ir = make_rsrc(in + (size_t)plane * nb, (unsigned)nb * 4u);
    float t[LPT], u[MODE == 1 ? LPT : 1];
#pragma unroll
    for (int e = 0; e < LPT; ++e) t[e] = bload(ir, vo + e * vstep, 0);
    if (MODE == 1) {
      const auto rr = make_rsrc(r + (size_t)plane * nb, (unsigned)nb * 4u);
#pragma unroll
      for (int e = 0; e < LPT; ++e) u[e] = bload(rr, vo + e * vstep, 0);
    }
    float zsw = 0.f, ztw = 0.f;
    if (MODE == 1) { zsw = zs[c * W + w]; ztw = zt[c * W + w]; }
    zero_pad<NT>(pl, Hb, W);
    const int lb = (h0 + kPadRows) * WP + w + 1, spare = ra_pad_floats(Hb, W);
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      float val = t[e];
      if (MODE == 1) {
        float h = t[e] * zsw + ztw;
        h += RES == 2 ? u[e] * q1 + q2 : u[e];
        val = fmaxf(h, 0.f);
      }
      pl[own && e * NTJ + tid < nb ? lb + e * GR * WP : spare] = AFFINE ? val * a + b : val;
    }
  }
  const float y = add_half ? ypos[c] + 0.5f : ypos[c];   // shift.py:17-18 (fp32 add)
  const Geom g = make_geom(xpos[c], y);
  const size_t ooff = (size_t)plane * n;
  float rv[MODE == 2 && RES ? LPT : 1];
  if (MODE == 2 && RES) {   // the residual at the output addresses, in flight over the barrier
    const auto rr = make_rsrc(r + ooff, (unsigned)n * 4u);
#pragma unroll
    for (int e = 0; e < LPT; ++e) rv[e] = bload(rr, vo + e * vstep, 0);
  }
  float sc = 1.f, sh = 0.f, gmu = 0.f;
  int du = 0;
  if (MODE == 2) {
    sc = scale[c];
    sh = shift[c];
    if (GOUT) {
      int uu = w - c % W;
      uu = uu < 0 ? uu + W : uu;
      du = uu - w;
      gmu = gm[uu * C + c];
    }
  }
  __syncthreads();
  const bool fits = g.y1 >= -kPadRows && (Ho - 1) * stride + g.y1 <= Hb + kPadRows - 2 &&
                    g.x1 >= -1 && g.x1 <= 0;
  const auto orr = make_rsrc(out + ooff, (unsigned)n * 4u);
  const auto ogr = make_rsrc(GOUT ? og + ooff : out + ooff, GOUT ? (unsigned)n * 4u : 0u);
  const int nval = own ? (n - tid + NTJ - 1) / NTJ : 0;   // this lane's elements e < nval
  float v[STATS ? LPT : 1];
  auto emit = [&](int e, float val) {
    if (MODE == 2) {
      float aa = val * sc + sh;
      if (RES == 1) aa += rv[e];
      if (RES == 2) aa += rv[e] * q1 + q2;
      val = fmaxf(aa, 0.f);
    }
    if (STATS) v[e] = e < nval ? val : 0.f;
    bstore(orr, val, vo + e * vstep, 0);
    if (GOUT) bstore(ogr, val * gmu, vo + e * vstep + (unsigned)(du * 4), 0);
  };
  if (fits) {
    // tap (0, 0) of element e: row (h0 + e*GR)*stride + y1, column w + x1; past the plane
    // (tail elements) the base clamps to the last element's (its value is discarded)
    const int la0 = (h0 * stride + g.y1 + kPadRows) * WP + w + g.x1 + 1;
    const int lmax = ((Ho - 1) * stride + g.y1 + kPadRows) * WP + W + g.x1;
    const int lstep = GR * stride * WP;
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      // (a lane that owns no element, tid >= NTJ, would start one row group past the plane;
      // an in-plane element's base never exceeds lmax, so one min clamps only the others)
      const int la = min(la0 + e * lstep, lmax);
      emit(e, blend(pl[la], pl[la + 1], pl[la + WP], pl[la + WP + 1], g.dx, g.dy));
    }
  } else {
    const bool c0 = (unsigned)(w + g.x1) < (unsigned)W, c1 = (unsigned)(w + g.x1 + 1) < (unsigned)W;
    const int cc0 = min(max(w + g.x1, 0), W - 1) + 1, cc1 = min(max(w + g.x1 + 1, 0), W - 1) + 1;
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      const int rr = (h0 + e * GR) * stride + g.y1;
      const bool r0 = (unsigned)rr < (unsigned)Hb, r1 = (unsigned)(rr + 1) < (unsigned)Hb;
      const int p0 = (min(max(rr, 0), Hb - 1) + kPadRows) * WP;
      const int p1 = (min(max(rr + 1, 0), Hb - 1) + kPadRows) * WP;
      const float q11 = (r0 && c0) ? pl[p0 + cc0] : 0.f, q21 = (r0 && c1) ? pl[p0 + cc1] : 0.f;
      const float q12 = (r1 && c0) ? pl[p1 + cc0] : 0.f, q22 = (r1 && c1) ? pl[p1 + cc1] : 0.f;
      emit(e, blend(q11, q21, q12, q22, g.dx, g.dy));
    }
  }
  if (STATS) {
    float s1 = 0.f;
#pragma unroll
    for (int e = 0; e < LPT; ++e) s1 += v[e];
    s1 = block_sum(s1, red);
    const float mean = s1 / (float)n;
    float m2 = 0.f;
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      const float d = v[e] - mean;
      m2 += e < nval ? d * d : 0.f;
    }
    m2 = block_sum(m2, red);
    if (tid == 0) pstats[plane] = make_float2(mean, m2);
  }
}

// Inference Shift_gcn tail fused into the following shift_in forward (shift_gcn.py:137-141
// then :67-68, BatchNorms in eval mode): the staged input element is
//   a * relu(z*zs[c*W + w] + zt[c*W + w] + res) + b
// with z the contraction output Z (natural layout), res = r (identity down) or
// r*rs[c] + rt[c] (down conv output + eval BN), a/b = Shift_tcn.bn (eval); the gcn
// output H is never written. Same tap arithmetic as tshift_fwd_lds_kernel.
template <int NT, int LPT, int RES>
__global__ __launch_bounds__(NT) void tshift_fwd_pre_kernel(
    const float* __restrict__ z, float* __restrict__ out, const float* __restrict__ xpos,
    const float* __restrict__ ypos, const float* __restrict__ zs, const float* __restrict__ zt,
    const float* __restrict__ r, const float* __restrict__ rs, const float* __restrict__ rt,
    const float* __restrict__ scale, const float* __restrict__ shift, int C, int Hb, int W,
    int Ho, int stride, int add_half) {
  SGCN_CRIT_PRIO();
  extern __shared__ float pl[];   // Hb*W staged input
  __shared__ float zs_s[1024], zt_s[1024];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  const int nb = Hb * W;
  const size_t ioff = (size_t)plane * nb;
  float* __restrict__ dst = out + (size_t)plane * Ho * W;
  const float y = add_half ? ypos[c] + 0.5f : ypos[c];
  const Geom g = make_geom(xpos[c], y);
  const float a = scale[c], b = shift[c];
  float q1 = 1.f, q2 = 0.f;
  if (RES == 2) { q1 = rs[c]; q2 = rt[c]; }
  for (int i = threadIdx.x; i < W; i += NT) {
    zs_s[i] = zs[c * W + i];
    zt_s[i] = zt[c * W + i];
  }
  __syncthreads();
  {
    float t[LPT], u[LPT];
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      const int i = min(e * NT + (int)threadIdx.x, nb - 1);
      t[e] = z[ioff + i];
      u[e] = r[ioff + i];
    }
    Walker pos(threadIdx.x, NT, W);
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      const int i = e * NT + threadIdx.x;
      float h = t[e] * zs_s[pos.w] + zt_s[pos.w];
      h += RES == 2 ? u[e] * q1 + q2 : u[e];
      h = fmaxf(h, 0.f);
      if (i < nb) pl[i] = h * a + b;
      pos.next();
    }
  }
  __syncthreads();
  const int n = Ho * W;
  for (int base = 0; base < n; base += LPT * NT) {
    Walker pos(base + threadIdx.x, NT, W);
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      TapIdx ti;
      tap_idx(pos.h * stride + g.y1, pos.w + g.x1, Hb, W, ti);
      const float q11 = sel(pl[ti.o00], ti.m00), q21 = sel(pl[ti.o01], ti.m01);
      const float q12 = sel(pl[ti.o10], ti.m10), q22 = sel(pl[ti.o11], ti.m11);
      const int o = base + e * NT + threadIdx.x;
      if (o < n) dst[o] = blend(q11, q21, q12, q22, g.dx, g.dy);
      pos.next();
    }
  }
}

// Inference unit tail fused into the shift_out forward (shift_gcn.py:72-73 + 161-162 with
// the BatchNorms in eval mode): out = relu(S*ps[c] + pt[c] + res), S the shifted value,
// res = 0 (RES 0), r (RES 1, identity residual) or r*rs[c] + rt[c] (RES 2, residual tcn
// conv output + eval BN), read at the output address; GOUT: also the next Shift_gcn's
// gathered, masked input og[c,t,(v - c) mod V] = out[c,t,v] * gm[((v - c) mod V)*C + c].
// S is never written. Same tap arithmetic as tshift_fwd_lds_kernel.
template <int NT, int LPT, int RES, bool GOUT>
__global__ __launch_bounds__(NT) void tshift_fwd_tail_kernel(
    const float* __restrict__ in, float* __restrict__ out, const float* __restrict__ xpos,
    const float* __restrict__ ypos, const float* __restrict__ ps, const float* __restrict__ pt,
    const float* __restrict__ r, const float* __restrict__ rs, const float* __restrict__ rt,
    const float* __restrict__ gm, float* __restrict__ og, int C, int Hb, int W, int Ho,
    int stride, int add_half) {
  SGCN_CRIT_PRIO();
  extern __shared__ float pl[];   // Hb*W staged input
  __shared__ float gm_s[GOUT ? 1024 : 1];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  const size_t ooff = (size_t)plane * Ho * W;
  const float y = add_half ? ypos[c] + 0.5f : ypos[c];
  const Geom g = make_geom(xpos[c], y);
  const float sc = ps[c], sh = pt[c];
  float q1 = 1.f, q2 = 0.f;
  if (RES == 2) { q1 = rs[c]; q2 = rt[c]; }
  const int rc = c % W;
  if (GOUT)
    for (int i = threadIdx.x; i < W; i += NT) gm_s[i] = gm[i * C + c];
  stage_plane<NT, LPT, false>(in + (size_t)plane * Hb * W, pl, Hb * W, 1.f, 0.f);
  __syncthreads();
  const int n = Ho * W;
  for (int base = 0; base < n; base += LPT * NT) {
    Walker pos(base + threadIdx.x, NT, W);
    float rv[LPT];
    if (RES) {
#pragma unroll
      for (int e = 0; e < LPT; ++e) rv[e] = r[ooff + min(base + e * NT + (int)threadIdx.x, n - 1)];
    }
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      TapIdx ti;
      tap_idx(pos.h * stride + g.y1, pos.w + g.x1, Hb, W, ti);
      const float q11 = sel(pl[ti.o00], ti.m00), q21 = sel(pl[ti.o01], ti.m01);
      const float q12 = sel(pl[ti.o10], ti.m10), q22 = sel(pl[ti.o11], ti.m11);
      const int o = base + e * NT + threadIdx.x;
      float a = blend(q11, q21, q12, q22, g.dx, g.dy) * sc + sh;
      if (RES == 1) a += rv[e];
      if (RES == 2) a += rv[e] * q1 + q2;
      a = fmaxf(a, 0.f);
      if (o < n) {
        out[ooff + o] = a;
        if (GOUT) {
          int u = pos.w - rc;
          u = u < 0 ? u + W : u;
          og[ooff + o - pos.w + u] = a * gm_s[u];
        }
      }
      pos.next();
    }
  }
}

// Stride-2 backward (the shift_out of l5 / l8), LDS-staged: both planes staged in one
// pass. JA (W <= 64): both passes walk their grids on the joint-aligned element stride
// (NT / W) * W: a thread's joint w is fixed, so the column part of every tap is a
// per-thread constant, and of the two gout rows an input row can reach (h1 / 2 and
// (h1 + 1) / 2) exactly one exists, so pass (1) reads 2 taps, not 4 (the other two are the
// exact zeros the general path selects).
template <int NT, int LPT, bool AFFINE, bool RELU_MASK, bool BNP, bool JA>
__global__ __launch_bounds__(NT) void tshift_bwd_s2_kernel(
    const float* __restrict__ gout, const float* __restrict__ in,
    const float* __restrict__ xpos, const float* __restrict__ ypos,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ bn_mean, const float* __restrict__ bn_invstd,
    float* __restrict__ gin, float2* __restrict__ pgrad, float2* __restrict__ bn_part, int C,
    int Hb, int W, int Ho, int add_half) {
  SGCN_CRIT_PRIO();
  constexpr int STRIDE = 2;
  extern __shared__ float lds[];   // [Ho*W gout][Hb*W raw input]
  __shared__ float red[4 * NT / 64];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  const int nb = Hb * W, nt = Ho * W;
  float* gs = lds;
  float* xs = lds + nt;
  float bmu = 0.f, bis = 0.f;
  if (BNP) { bmu = bn_mean[c]; bis = bn_invstd[c]; }
  const float x = xpos[c];
  const float y = add_half ? ypos[c] + 0.5f : ypos[c];
  float a = 1.f, b = 0.f;
  if (AFFINE) { a = scale[c]; b = shift[c]; }
  {  // one staging pass: both planes' loads in flight together (LPT covers nt + nb)
    const float* __restrict__ go = gout + (size_t)plane * nt;
    const float* __restrict__ src = in + (size_t)plane * nb;
    const int ntot = nt + nb;
    float t[LPT];
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      const int i = min(e * NT + (int)threadIdx.x, ntot - 1);
      t[e] = i < nt ? go[i] : src[i - nt];
    }
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      const int i = e * NT + threadIdx.x;
      if (i < ntot) lds[i] = t[e];
    }
  }
  __syncthreads();
  float* __restrict__ gi = gin + (size_t)plane * nb;

  // (1) grad_input over the bottom grid (.cu:191-254: the even-row rule)
  float bs0 = 0.f, bs1 = 0.f;
  float ax = 0.f, ay = 0.f;
  if (JA) {
    const Geom r = make_geom(-x, -y);
    const int NTJ = (NT / W) * W, GR = NT / W;
    if ((int)threadIdx.x < NTJ && nt > 0) {
      const int w = (int)threadIdx.x % W, w1 = w + r.x1;
      const bool c0 = (unsigned)w1 < (unsigned)W, c1 = (unsigned)(w1 + 1) < (unsigned)W;
      const int cc0 = min(max(w1, 0), W - 1), cc1 = min(max(w1 + 1, 0), W - 1);
      int h = (int)threadIdx.x / W;
      for (int o = threadIdx.x; o < nb; o += NTJ, h += GR) {
        // input row h reaches gout row hq = h1 / 2 (h1 = h + y1 even: taps q11, q21) or
        // (h1 + 1) / 2 (h1 odd: taps q12, q22); (h1 + 1) >> 1 is both, floor for h1 < 0
        const int h1 = h + r.y1, hq = (h1 + 1) >> 1;
        const bool ev = (h1 & 1) == 0, rok = (unsigned)hq < (unsigned)Ho;
        const int ro = min(max(hq, 0), Ho - 1) * W;
        const float t0 = (rok && c0) ? gs[ro + cc0] : 0.f;
        const float t1 = (rok && c1) ? gs[ro + cc1] : 0.f;
        float val = blend(ev ? t0 : 0.f, ev ? t1 : 0.f, ev ? 0.f : t0, ev ? 0.f : t1, r.dx, r.dy);
        const float rin = xs[o];
        if (RELU_MASK) val = rin > 0.f ? val : 0.f;
        gi[o] = val;
        if (BNP) {
          bs0 += val;
          bs1 += val * ((rin - bmu) * bis);
        }
      }
    } else if ((int)threadIdx.x < NTJ) {   // no gout rows (Ho == 0): the gradient is 0
      for (int o = threadIdx.x; o < nb; o += NTJ) gi[o] = 0.f;
    }
  } else {
    const Geom r = make_geom(-x, -y);
    Walker pos(threadIdx.x, NT, W);
    for (int o = threadIdx.x; o < nb; o += NT) {
      const int h1 = pos.h + r.y1;
      const int w1 = pos.w + r.x1;
      // h_im % 2 == 0 (C++ remainder), then h_im / 2 (truncation), bounds on the top grid;
      // exactly one of h1, h1+1 is even
      TapIdx ti;
      {
        const int h2 = h1 + 1;
        const int hq1 = (h1 % 2 == 0) ? h1 / 2 : -1;
        const int hq2 = (h2 % 2 == 0) ? h2 / 2 : -1;
        TapIdx t1, t2;
        tap_idx(hq1, w1, Ho, W, t1);
        tap_idx(hq2, w1, Ho, W, t2);
        ti.o00 = t1.o00; ti.o01 = t1.o01; ti.m00 = t1.m00; ti.m01 = t1.m01;
        ti.o10 = t2.o00; ti.o11 = t2.o01; ti.m10 = t2.m00; ti.m11 = t2.m01;
      }
      float val = 0.f;
      if (nt > 0) {
        const float q11 = sel(gs[ti.o00], ti.m00), q21 = sel(gs[ti.o01], ti.m01);
        const float q12 = sel(gs[ti.o10], ti.m10), q22 = sel(gs[ti.o11], ti.m11);
        val = blend(q11, q21, q12, q22, r.dx, r.dy);
      }
      const float rin = xs[o];
      if (RELU_MASK) val = rin > 0.f ? val : 0.f;
      gi[o] = val;
      if (BNP) {
        bs0 += val;
        bs1 += val * ((rin - bmu) * bis);
      }
      pos.next();
    }
  }

  // (2) position gradients over the top grid (.cu:321-349), summed over the plane
  if (JA) {
    const Geom g = make_geom(x, y);
    const int NTJ = (NT / W) * W, GR = NT / W;
    if ((int)threadIdx.x < NTJ) {
      const int w = (int)threadIdx.x % W, wc = w + g.x1;
      const bool c0 = (unsigned)wc < (unsigned)W, c1 = (unsigned)(wc + 1) < (unsigned)W;
      const int cc0 = min(max(wc, 0), W - 1), cc1 = min(max(wc + 1, 0), W - 1);
      int h = (int)threadIdx.x / W;
      for (int o = threadIdx.x; o < nt; o += NTJ, h += GR) {
        const int rr = h * STRIDE + g.y1;
        const bool r0 = (unsigned)rr < (unsigned)Hb, r1 = (unsigned)(rr + 1) < (unsigned)Hb;
        const int p0 = min(max(rr, 0), Hb - 1) * W, p1 = min(max(rr + 1, 0), Hb - 1) * W;
        float q11 = xs[p0 + cc0], q21 = xs[p0 + cc1], q12 = xs[p1 + cc0], q22 = xs[p1 + cc1];
        if (AFFINE) { q11 = q11 * a + b; q21 = q21 * a + b; q12 = q12 * a + b; q22 = q22 * a + b; }
        q11 = (r0 && c0) ? q11 : 0.f;
        q21 = (r0 && c1) ? q21 : 0.f;
        q12 = (r1 && c0) ? q12 : 0.f;
        q22 = (r1 && c1) ? q22 : 0.f;
        const float vx = (1.f - g.dy) * (q21 - q11) + g.dy * (q22 - q12);
        const float vy = (1.f - g.dx) * (q12 - q11) + g.dx * (q22 - q21);
        const float gg = gs[o];
        ax += vx * gg;
        ay += vy * gg;
      }
    }
  } else {
    const Geom g = make_geom(x, y);
    Walker pos(threadIdx.x, NT, W);
    for (int o = threadIdx.x; o < nt; o += NT) {
      TapIdx ti;
      tap_idx(pos.h * STRIDE + g.y1, pos.w + g.x1, Hb, W, ti);
      float q11 = xs[ti.o00], q21 = xs[ti.o01], q12 = xs[ti.o10], q22 = xs[ti.o11];
      if (AFFINE) { q11 = q11 * a + b; q21 = q21 * a + b; q12 = q12 * a + b; q22 = q22 * a + b; }
      q11 = sel(q11, ti.m00);
      q21 = sel(q21, ti.m01);
      q12 = sel(q12, ti.m10);
      q22 = sel(q22, ti.m11);
      const float vx = (1.f - g.dy) * (q21 - q11) + g.dy * (q22 - q12);
      const float vy = (1.f - g.dx) * (q12 - q11) + g.dx * (q22 - q21);
      const float gg = gs[o];
      ax += vx * gg;
      ay += vy * gg;
      pos.next();
    }
  }
  if (BNP) {   // both plane reductions behind one barrier pair
    block_sum4(ax, ay, bs0, bs1, red);
    if (threadIdx.x == 0) {
      pgrad[plane] = make_float2(ax, ay);
      bn_part[plane] = make_float2(bs0, bs1);
    }
  } else {
    block_sum2(ax, ay, red);
    if (threadIdx.x == 0) pgrad[plane] = make_float2(ax, ay);
  }
}

// Stride-1 backward on a zero-padded LDS plane: the product kernel of every stride-1
// shift backward (Shift_tcn's shift_in, plain and GBN, and the unit's shift_out, GP).
// gout is staged with row pitch WP = W + 2 (a zero column each side) between kPadRows zero
// rows above and below, so for every channel whose shift stays inside the padding
// (floor(+-x) in {-1, 0}, |floor(+-y)| <= kPadRows - 1 — every channel of a trained
// Shift-GCN, whose xpos stays near 0 and |ypos| near 1) each tap is an unconditional LDS
// read at a per-workgroup constant offset from the element: no per-element range checks,
// clamps or selects (the padding supplies the exact +0 the reference substitutes for an
// out-of-range tap). A channel whose shift leaves the padding takes the range-checked loop
// (same values). Global traffic goes through buffer descriptors: the loads
// need no clamps (past the plane they return 0) and stores past the plane are dropped.
// Elements are dealt on the joint-aligned stride NTE = (NT / W) * W (a thread's joint is
// fixed). The input gradient is bit-identical to the oracle; the position-gradient sums are
// accumulated over INPUT positions from the same gout neighbourhood (exact adjoint:
//   sum_o g[o] * dq(o)/dy = sum_i in[i] * sum_k w'_k g[i - off_k]
// only the summation order differs from the reference's sum over outputs, and the
// constraint keeps only the sign of the sum, .cu:370-395).
// BNP: also the per-plane BatchNorm-backward partials {sum gin, sum gin*xhat},
// xhat = (in - bn_mean[c]) * bn_invstd[c], of the BatchNorm that produced this shift's
// input (Shift_tcn.bn before shift_in): its separate reduction pass disappears.
//
// GP: gout is not read; it is the input gradient of the BatchNorm that
// follows this shift (Shift_tcn.bn2 inside a TCN_GCN_unit, shift_gcn.py:73,161-162),
// formed while staging: gout = k1*(gy > 0 ? gdy : 0) + k2*gx + k3 (gdy = the unit's output
// gradient, gy = its output, gx = bn2's input S, k = sgcn_bn_bwd_finalize coefficients),
// so that gradient tensor is never written.
//
// GBN (with AFFINE + BNP: Shift_tcn's shift_in inside a TCN_GCN_unit whose
// Shift_gcn has no down conv): also the backward partials of Shift_gcn.bn, the per-joint
// BatchNorm1d whose ReLU output H is this shift's input (shift_gcn.py:137-141), without a
// separate pass over (dA, H, Z). Its input gradient is g = [H > 0] * (k1*dA + k2*H + k3)
// with k = Shift_tcn.bn's backward coefficients, which need this launch's own batch-wide
// partials first; so the k-free sums are emitted per (plane, joint) instead, centred on
// Shift_tcn.bn's mean mu (k2*H + k3 = k2*(H - mu) + (k3 + k2*mu), no cancellation):
//   {sum dA, sum (H-mu), sum 1, sum dA*zh, sum (H-mu)*zh, sum zh} over t where H > 0,
//   zh = (Z - zmean[c,v]) * zinvstd[c,v]; sgcn_bn_bwd_finalize_gbn combines them.
// GBD (with GBN: the Shift_gcn HAS a down conv, whose BatchNorm2d output d is added before
// the ReLU: H = relu(bn(Z) + bnd(d)), shift_gcn.py:140-141): also the plane sums of that
// BatchNorm's backward, {sum dA, sum (H-mu), sum 1, sum dA*dh, sum (H-mu)*dh, sum dh} over
// H > 0, dh = (d - d_mean[c]) * d_invstd[c], to gdpart[j][plane] — the same six-sum form,
// finalized by sgcn_bn_bwd_finalize_gbn with V = 1 — so no sgcn_bn_bwd_reduce pass over
// (dA, H, Z, d) remains for the units with a down conv either.
template <int NT, int LPT, bool AFFINE, bool RELU_MASK, bool BNP, bool GP, bool GBN,
          bool GBD = false>
__global__ __launch_bounds__(NT) void tshift_bwd_ra_kernel(
    const float* __restrict__ gout, const float* __restrict__ in,
    const float* __restrict__ xpos, const float* __restrict__ ypos,
    const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ bn_mean, const float* __restrict__ bn_invstd,
    float* __restrict__ gin, float2* __restrict__ pgrad, float2* __restrict__ bn_part, int C,
    int H, int W, const float* __restrict__ gdy, const float* __restrict__ gy,
    const float* __restrict__ gx, const float* __restrict__ gcoef,
    const float* __restrict__ gz, const float* __restrict__ gzm,
    const float* __restrict__ gzi, float* __restrict__ gzpart, const float* __restrict__ gd = nullptr,
    const float* __restrict__ gdm = nullptr, const float* __restrict__ gdi = nullptr,
    float* __restrict__ gdpart = nullptr) {
  SGCN_CRIT_PRIO();
  static_assert(!GBN || (AFFINE && BNP && !GP), "GBN: shift_in with BNP");
  static_assert(!GBD || GBN, "GBD extends GBN");
  extern __shared__ float lds[];   // [(H + 2*kPadRows) * WP] padded gout (GBN: >= 6*NT)
  __shared__ float red[4 * NT / 64];
  const int plane = gridDim.x - 1 - blockIdx.x;   // reverse: see kReverse note
  const int c = plane % C;
  const int n = H * W, WP = W + 2;
  const int GR = NT / W, NTE = GR * W;
  const int tid = threadIdx.x;
  const bool own = tid < NTE;   // the last NT - NTE threads hold no elements
  const int w = tid % W, h0 = tid / W;
  // element e of this thread: plane offset e*NTE + tid (bytes vo + e*vstep); a lane that
  // holds no elements points past every plane (its loads return 0, its stores drop)
  const unsigned vo = own ? (unsigned)tid * 4u : 0x80000000u;
  const unsigned vstep = (unsigned)NTE * 4u, nbytes = (unsigned)n * 4u;
  const size_t poff = (size_t)plane * n;
#ifdef SGCN_DIAG_X1B_BOUND
  // timing diagnostic only (results wrong): the shift_in backward (affine taps) of a plane
  // of C >= SGCN_DIAG_X1B_BOUND channels reads no gout (the dAs read a fused epilogue saves)
  const unsigned gbytes = AFFINE && !GP && C >= SGCN_DIAG_X1B_BOUND ? 0u : nbytes;
#else
  const unsigned gbytes = nbytes;
#endif
  float t[LPT], rin_r[LPT];
  float zr[GBN ? LPT : 1], dr[GBD ? LPT : 1];
  {   // every global load of the plane in flight together
    const auto inr = make_rsrc(in + poff, nbytes);
    if (GP) {
      const auto dyr = make_rsrc(gdy + poff, nbytes);
      const auto yr = make_rsrc(gy + poff, nbytes);
      const auto xr = make_rsrc(gx + poff, nbytes);
      float u1[LPT], u2[LPT];
#pragma unroll
      for (int e = 0; e < LPT; ++e) {
        const unsigned vb = vo + e * vstep;
        t[e] = bload(dyr, vb, 0);
        u1[e] = bload(yr, vb, 0);
        u2[e] = bload(xr, vb, 0);
        rin_r[e] = bload(inr, vb, 0);
      }
      // bn2's backward coefficients, read while the plane's loads fly
      const float k1 = gcoef[c], k2 = gcoef[C + c], k3 = gcoef[2 * C + c];
#pragma unroll
      for (int e = 0; e < LPT; ++e) t[e] = k1 * (u1[e] > 0.f ? t[e] : 0.f) + k2 * u2[e] + k3;
    } else {
      const auto gr = make_rsrc(gout + poff, gbytes);
#pragma unroll
      for (int e = 0; e < LPT; ++e) {
        t[e] = bload(gr, vo + e * vstep, 0);
        rin_r[e] = bload(inr, vo + e * vstep, 0);
      }
      if (GBN) {
        // z is the gcn contraction output BEFORE its shift_out: logical joint w of this
        // thread sits at (w - c) mod W in its row (a constant in-row offset)
        const auto zrr = make_rsrc(gz + poff, nbytes);
        int wz = w - c % W;
        wz = wz < 0 ? wz + W : wz;
        const unsigned zo = vo + (unsigned)((wz - w) * 4);
#pragma unroll
        for (int e = 0; e < LPT; ++e) zr[e] = bload(zrr, zo + e * vstep, 0);
      }
      if (GBD) {   // the down conv output: natural layout, the element's own address
        const auto drr = make_rsrc(gd + poff, nbytes);
#pragma unroll
        for (int e = 0; e < LPT; ++e) dr[e] = bload(drr, vo + e * vstep, 0);
      }
    }
  }
  zero_pad<NT>(lds, H, W);
  // element (h, w) of the plane sits at lds[(h + kPadRows) * WP + w + 1]; a lane's elements
  // past the plane go to the spare float after the padded plane (branch-free stores)
  const int lbase = (h0 + kPadRows) * WP + w + 1, lstep = GR * WP;
  const int lspare = ra_pad_floats(H, W);
#pragma unroll
  for (int e = 0; e < LPT; ++e)
    lds[own && e * NTE + tid < n ? lbase + e * lstep : lspare] = t[e];
  float bmu = 0.f, bis = 0.f;
  if (BNP) { bmu = bn_mean[c]; bis = bn_invstd[c]; }
  const float x = xpos[c], y = ypos[c];
  float a = 1.f, b = 0.f;
  if (AFFINE) { a = scale[c]; b = shift[c]; }
  float zm = 0.f, zi = 0.f, dmu = 0.f, dis = 0.f;
  if (GBN) { zm = gzm[c * W + w]; zi = gzi[c * W + w]; }
  if (GBD) { dmu = gdm[c]; dis = gdi[c]; }
  __syncthreads();

  // input-gradient taps: gout at (h + r.y1 + {0,1}, w + r.x1 + {0,1}) (.cu:108-150);
  // position-gradient taps: gout at (h - g.y1 - 1 + {0,1}, w - g.x1 - 1 + {0,1}), i.e.
  // gout[i - off_k] for the forward taps off_k (the adjoint above)
  const Geom r = make_geom(-x, -y);
  const Geom g = make_geom(x, y);
  const bool fits = r.y1 >= -kPadRows && r.y1 <= kPadRows - 1 && g.y1 >= -kPadRows &&
                    g.y1 <= kPadRows - 1 && r.x1 >= -1 && r.x1 <= 0 && g.x1 >= -1 && g.x1 <= 0;
  const int kq = r.y1 * WP + r.x1, kg = (-g.y1 - 1) * WP - g.x1 - 1;
  const int nfull = n / NTE;     // elements e < nfull are inside the plane for every lane
  const int lmax = (H - 1 + kPadRows) * WP + W;   // the last element: past-the-plane bases clamp here
  const auto gir = make_rsrc(gin + poff, nbytes);
  float bs0 = 0.f, bs1 = 0.f, ax = 0.f, ay = 0.f;
  float a6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // GBN per-joint sums
  float d6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // GBD plane sums
  // one element: value, stores and sums from its eight taps (tail: the element may lie
  // past the plane — its load returned 0, its store drops, its sums are masked here)
  auto elem = [&](int e, bool tail, float q11, float q21, float q12, float q22, float G11,
                  float G21, float G12, float G22) {
    const bool ok = !tail || e * NTE + tid < n;
    float val = blend(q11, q21, q12, q22, r.dx, r.dy);
    const float rin = rin_r[e];
    if (RELU_MASK) val = rin > 0.f ? val : 0.f;
    if (tail) val = ok ? val : 0.f;
    bstore(gir, val, vo + e * vstep, 0);   // (an immediate-offset store off one base)
    if (GBN) {
      // predicated, not branched (a branch per element keeps every element's registers
      // live across the blocks): an inactive element adds exact +0 to sums that are
      // never -0, so the sums are bit-identical to skipping it; rin = 0 past the plane
      const bool act = rin > 0.f;
      const float hc = act ? rin - bmu : 0.f, zh = act ? (zr[e] - zm) * zi : 0.f;
      const float vv = act ? val : 0.f;
      a6[0] += vv;
      a6[1] += hc;
      a6[2] += act ? 1.f : 0.f;
      a6[3] = fmaf(vv, zh, a6[3]);
      a6[4] = fmaf(hc, zh, a6[4]);
      a6[5] += zh;
      if (GBD) {
        const float dh = act ? (dr[e] - dmu) * dis : 0.f;
        d6[0] += vv;
        d6[1] += hc;
        d6[2] += act ? 1.f : 0.f;
        d6[3] = fmaf(vv, dh, d6[3]);
        d6[4] = fmaf(hc, dh, d6[4]);
        d6[5] += dh;
      }
    }
    if (BNP) {
      bs0 += val;
      bs1 = fmaf(val, (rin - bmu) * bis, bs1);
    }
    const float cx = (1.f - g.dy) * (G21 - G11) + g.dy * (G22 - G12);
    const float cy = (1.f - g.dx) * (G12 - G11) + g.dx * (G22 - G21);
    float qa = AFFINE ? rin * a + b : rin;
    if (tail) qa = ok ? qa : 0.f;
    // the plane sums (position-gradient products, BatchNorm partials) are not bit-matched
    // to any reference order (their summation order is this kernel's own): fused
    ax = fmaf(qa, cx, ax);
    ay = fmaf(qa, cy, ay);
  };
  if (own && fits) {
    int l0 = lbase;
#pragma unroll
    for (int e = 0; e < LPT; ++e) {
      const bool tail = e >= nfull;
      const int lt = min(l0, lmax);   // (an in-plane element's base never exceeds lmax)
      const int la = lt + kq, lg = lt + kg;
      elem(e, tail, lds[la], lds[la + 1], lds[la + WP], lds[la + WP + 1], lds[lg + WP + 1],
           lds[lg + WP], lds[lg + 1], lds[lg]);
      // the next element's base is opaque to the compiler: its address arithmetic (and so
      // its LDS reads) cannot be hoisted into one long-lived register per element
      l0 += lstep;
      asm volatile("" : "+v"(l0));
    }
  } else if (own) {
    // range-checked taps (a shift beyond the padding; never in a trained model): a rolled
    // loop that re-reads its input elements instead of holding the staged registers
    const auto inr = make_rsrc(in + poff, nbytes);
    const auto zrr = make_rsrc(GBN ? gz + poff : in + poff, nbytes);
    int wz = w - c % W;
    wz = wz < 0 ? wz + W : wz;
    auto tap = [&](int row, int col) {
      const bool in_ = (unsigned)row < (unsigned)H && (unsigned)col < (unsigned)W;
      const int rr = min(max(row, 0), H - 1), cc = min(max(col, 0), W - 1);
      const float v = lds[(rr + kPadRows) * WP + cc + 1];
      return in_ ? v : 0.f;
    };
#pragma unroll 1
    for (int e = 0; e < LPT; ++e) {
      const int h = h0 + e * GR;
      const bool ok = e * NTE + tid < n;
      const float rin = bload(inr, vo + e * vstep, 0);
      const float zv = GBN ? bload(zrr, vo + e * vstep + (unsigned)((wz - w) * 4), 0) : 0.f;
      const int rq = h + r.y1, cq = w + r.x1, rg = h - g.y1 - 1, cg = w - g.x1 - 1;
      float val = blend(tap(rq, cq), tap(rq, cq + 1), tap(rq + 1, cq), tap(rq + 1, cq + 1),
                        r.dx, r.dy);
      if (RELU_MASK) val = rin > 0.f ? val : 0.f;
      val = ok ? val : 0.f;
      bstore(gir, val, vo + e * vstep, 0);
      if (GBN && rin > 0.f) {
        const float hc = rin - bmu, zh = (zv - zm) * zi;
        a6[0] += val;
        a6[1] += hc;
        a6[2] += 1.f;
        a6[3] = fmaf(val, zh, a6[3]);
        a6[4] = fmaf(hc, zh, a6[4]);
        a6[5] += zh;
        if (GBD) {
          const float dh = (bload(make_rsrc(gd + poff, nbytes), vo + e * vstep, 0) - dmu) * dis;
          d6[0] += val;
          d6[1] += hc;
          d6[2] += 1.f;
          d6[3] = fmaf(val, dh, d6[3]);
          d6[4] = fmaf(hc, dh, d6[4]);
          d6[5] += dh;
        }
      }
      if (BNP) {
        bs0 += val;
        bs1 += val * ((rin - bmu) * bis);
      }
      const float G11 = tap(rg + 1, cg + 1), G21 = tap(rg + 1, cg), G12 = tap(rg, cg + 1),
                  G22 = tap(rg, cg);
      const float cx = (1.f - g.dy) * (G21 - G11) + g.dy * (G22 - G12);
      const float cy = (1.f - g.dx) * (G12 - G11) + g.dx * (G22 - G21);
      float qa = AFFINE ? rin * a + b : rin;
      qa = ok ? qa : 0.f;
      ax += qa * cx;
      ay += qa * cy;
    }
  }
  if (BNP) {   // both plane reductions behind one barrier pair
    block_sum4(ax, ay, bs0, bs1, red);
    if (tid == 0) {
      pgrad[plane] = make_float2(ax, ay);
      bn_part[plane] = make_float2(bs0, bs1);
    }
  } else {
    block_sum2(ax, ay, red);
    if (tid == 0) pgrad[plane] = make_float2(ax, ay);
  }
  if (GBD) {   // the down BatchNorm's six plane sums
    block_sum4(d6[0], d6[1], d6[2], d6[3], red);
    block_sum2(d6[4], d6[5], red);
    if (tid == 0) {
      const size_t np = gridDim.x;
#pragma unroll
      for (int k = 0; k < 6; ++k) gdpart[k * np + plane] = d6[k];
    }
  }
  if (GBN) {
    // merge the GR row groups of each joint in fixed order (deterministic)
    __syncthreads();   // every LDS read of gout is done: reuse the LDS (>= 6*NT floats)
#pragma unroll
    for (int k = 0; k < 6; ++k) lds[k * NT + tid] = a6[k];
    __syncthreads();
    // one thread per (sum k, joint w): GR dependent LDS reads each instead of 6*GR
    if (tid < 6 * W) {
      const size_t np = (size_t)gridDim.x * W;
      const int k = tid / W, wk = tid - k * W;
      float sum = 0.f;
      for (int gg = 0; gg < GR; ++gg) sum += lds[k * NT + gg * W + wk];
      gzpart[k * np + (size_t)plane * W + wk] = sum;
    }
  }
}

// mean over the batch of the per-plane sums (== mean_b then sum_w, sum_h of .cu:501-509
// up to rounding), then applyShiftConstraint (.cu:370-395) with its float/double
// promotions: sqrt(dy*dy) in float (correctly rounded), quotients in float, times the
// double literals 0.0 / 0.01, stored as float; the dr == 0 branch stores 0.0 / 0.0001.
__device__ __forceinline__ void pos_finalize_body(const float2* __restrict__ pgrad, int B,
                                                  int C, float* __restrict__ gx,
                                                  float* __restrict__ gy);

__global__ __launch_bounds__(256) void tshift_pos_finalize_kernel(
    const float2* __restrict__ pgrad, int B, int C, float* __restrict__ gx,
    float* __restrict__ gy) {
  pos_finalize_body(pgrad, B, C, gx, gy);
}

// Many position-gradient finalizes in one launch (the side stream's deferred ones, flushed
// at the end of the backward); the entries are kernel arguments; blockIdx.y = entry.
struct PosBatch {
  const float2* p[SGCN_BATCH_MAX];
  float* gx[SGCN_BATCH_MAX];
  float* gy[SGCN_BATCH_MAX];
  int B[SGCN_BATCH_MAX];
  int C[SGCN_BATCH_MAX];
};
__global__ __launch_bounds__(256) void tshift_pos_finalize_many_kernel(const PosBatch t) {
  const int i = blockIdx.y;
  if ((int)blockIdx.x * 4 >= t.C[i]) return;   // whole workgroup past this entry's channels
  pos_finalize_body(t.p[i], t.B[i], t.C[i], t.gx[i], t.gy[i]);
}

__device__ __forceinline__ void pos_finalize_body(const float2* __restrict__ pgrad, int B,
                                                  int C, float* __restrict__ gx,
                                                  float* __restrict__ gy) {
  // one wave per channel, lanes striding the batch (one round trip of 4 loads for
  // B <= 256), fixed xor tree in double: deterministic
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  const int cc = min(c, C - 1);
  double ax = 0.0, ay = 0.0;
  for (int b0 = lane; b0 < B; b0 += 256) {
    float2 pv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int b = b0 + u * 64;
      pv[u] = b < B ? pgrad[(size_t)b * C + cc] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ax += (double)pv[u].x;
      ay += (double)pv[u].y;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ax += __shfl_xor(ax, o, 64);
    ay += __shfl_xor(ay, o, 64);
  }
  if (c >= C || lane != 0) return;
  const double sx = ax, sy = ay;
  const float Gx = (float)(sx / (double)B);
  const float Gy = (float)(sy / (double)B);
  const float gy2 = Gy * Gy;
  const float dr = (float)sqrt((double)gy2);
  if (dr != 0.f) {
    const float qx = (float)((double)Gx / (double)dr);
    const float qy = (float)((double)Gy / (double)dr);
    gx[c] = (float)((double)qx * 0.0);
    gy[c] = (float)((double)qy * 0.01);
  } else {
    gx[c] = 0.0f;
    gy[c] = (float)0.0001;
  }
}

template <int EPT>
void launch_fwd(bool affine, bool stats, const float* in, float* out, const float* xpos,
                const float* ypos, const float* scale, const float* shift, float2* ps, int B,
                int C, int H, int W, int Ho, int stride, int add_half, hipStream_t st) {
  dim3 grid(B * C), block(kThreads);
#define SGCN_FWD(A, S)                                                                     \
  tshift_fwd_kernel<EPT, A, S><<<grid, block, 0, st>>>(in, out, xpos, ypos, scale, shift, \
                                                      ps, C, H, W, Ho, stride, add_half)
  if (affine) {
    if (stats) SGCN_FWD(true, true); else SGCN_FWD(true, false);
  } else {
    if (stats) SGCN_FWD(false, true); else SGCN_FWD(false, false);
  }
#undef SGCN_FWD
}

// LDS path: EPT = LPT (the output plane is never larger than the staged input plane)
template <int LPT, int NT = kThreads>
void launch_fwd_lds(bool affine, bool stats, const float* in, float* out, const float* xpos,
                    const float* ypos, const float* scale, const float* shift, float2* ps,
                    int B, int C, int H, int W, int Ho, int stride, int add_half,
                    hipStream_t st) {
  dim3 grid(B * C), block(NT);
  const size_t lds = (size_t)H * W * sizeof(float);
#define SGCN_FWDL(A, S)                                                                  \
  tshift_fwd_lds_kernel<NT, LPT, LPT, A, S><<<grid, block, lds, st>>>(                    \
      in, out, xpos, ypos, scale, shift, ps, C, H, W, Ho, stride, add_half)
  if (affine) {
    if (stats) SGCN_FWDL(true, true); else SGCN_FWDL(true, false);
  } else {
    if (stats) SGCN_FWDL(false, true); else SGCN_FWDL(false, false);
  }
#undef SGCN_FWDL
}

// elements per thread of the padded joint-aligned forward kernels (W <= 64) on NT threads;
// 0 when the plane needs more than 32 per thread or more than 64 KiB of LDS
int pad_fwd_lpt(int H, int W, int nt) {
  if (W > 64) return 0;
  const int ntj = (nt / W) * W, per = (H * W + ntj - 1) / ntj;
  // 512 threads also at 12 / 20 (as ra_lpt): MediaPipe's 9,900-float planes are 20 per
  // thread, and the eval pre / tail forms held 88-95 VGPRs at 24 (two workgroups per CU)
  int lpt = per <= 8 ? 8 : (per <= 16 ? 16 : (per <= 24 ? 24 : (per <= 32 ? 32 : 0)));
  if (nt == 512 && per > 8 && per <= 12) lpt = 12;
  if (nt == 512 && per > 16 && per <= 20) lpt = 20;
  return (size_t)(ra_pad_floats(H, W) + 1) * sizeof(float) > 65536 ? 0 : lpt;
}

// padded joint-aligned forward (W <= 64): LPT elements per thread on the (NT / W) * W
// stride; false (nothing launched) when the plane needs more than 32 per thread or
// more than 64 KiB of LDS
template <int NT>
bool launch_fwd_pad(bool affine, bool stats, const float* in, float* out, const float* xpos,
                    const float* ypos, const float* scale, const float* shift, float2* ps,
                    int B, int C, int H, int W, int Ho, int stride, int add_half,
                    hipStream_t st) {
  const int lpt = pad_fwd_lpt(H, W, NT);
  const size_t lds = (size_t)(ra_pad_floats(H, W) + 1) * sizeof(float);
  if (lpt == 0) return false;
#define SGCN_FWDP(L, A, S)                                                                   \
  tshift_fwd_pad_kernel<NT, L, 0, A, S><<<B * C, NT, lds, st>>>(                             \
      in, out, xpos, ypos, scale, shift, ps, C, H, W, Ho, stride, add_half, nullptr, nullptr, \
      nullptr, nullptr, nullptr, nullptr, nullptr)
#define SGCN_FWDP_AS(L)                                                                      \
  do {                                                                                       \
    if (affine) { if (stats) SGCN_FWDP(L, true, true); else SGCN_FWDP(L, true, false); }     \
    else { if (stats) SGCN_FWDP(L, false, true); else SGCN_FWDP(L, false, false); }          \
  } while (0)
  if (lpt == 8) SGCN_FWDP_AS(8); else if (lpt == 12) SGCN_FWDP_AS(12); else if (lpt == 16) SGCN_FWDP_AS(16);
  else if (lpt == 20) SGCN_FWDP_AS(20); else if (lpt == 24) SGCN_FWDP_AS(24); else SGCN_FWDP_AS(32);
#undef SGCN_FWDP_AS
#undef SGCN_FWDP
  return true;
}

template <int EPT, int STRIDE>
void launch_bwd(bool affine, bool relu, const float* gout, const float* in, const float* xpos,
                const float* ypos, const float* scale, const float* shift, const float* bmu,
                const float* bis, float* gin, float2* pg, float2* bp, int B, int C, int H,
                int W, int Ho, int add_half, hipStream_t st) {
  dim3 grid(B * C), block(kThreads);
#define SGCN_BWD(A, R, P)                                                                    \
  tshift_bwd_kernel<EPT, A, R, STRIDE, P><<<grid, block, 0, st>>>(                            \
      gout, in, xpos, ypos, scale, shift, bmu, bis, gin, pg, bp, C, H, W, Ho, add_half)
  if (bp) {
    if (affine) {
      if (relu) SGCN_BWD(true, true, true); else SGCN_BWD(true, false, true);
    } else {
      if (relu) SGCN_BWD(false, true, true); else SGCN_BWD(false, false, true);
    }
  } else {
    if (affine) {
      if (relu) SGCN_BWD(true, true, false); else SGCN_BWD(true, false, false);
    } else {
      if (relu) SGCN_BWD(false, true, false); else SGCN_BWD(false, false, false);
    }
  }
#undef SGCN_BWD
}

constexpr int kBwdThreads = 512;

template <int LPT, bool JA>
void launch_bwd_s2(bool affine, bool relu, const float* gout, const float* in,
                   const float* xpos, const float* ypos, const float* scale,
                   const float* shift, const float* bmu, const float* bis, float* gin,
                   float2* pg, float2* bp, int B, int C, int H, int W, int Ho, int add_half,
                   hipStream_t st) {
  constexpr int NT = kBwdThreads;
  dim3 grid(B * C), block(NT);
  const size_t lds = (size_t)(H + Ho) * W * sizeof(float);
#define SGCN_BWDL(A, R, P)                                                                  \
  tshift_bwd_s2_kernel<NT, LPT, A, R, P, JA><<<grid, block, lds, st>>>(                      \
      gout, in, xpos, ypos, scale, shift, bmu, bis, gin, pg, bp, C, H, W, Ho, add_half)
  if (bp) {
    if (affine) {
      if (relu) SGCN_BWDL(true, true, true); else SGCN_BWDL(true, false, true);
    } else {
      if (relu) SGCN_BWDL(false, true, true); else SGCN_BWDL(false, false, true);
    }
  } else {
    if (affine) {
      if (relu) SGCN_BWDL(true, true, false); else SGCN_BWDL(true, false, false);
    } else {
      if (relu) SGCN_BWDL(false, true, false); else SGCN_BWDL(false, false, false);
    }
  }
#undef SGCN_BWDL
}

int pick_lpt(int n, int nt) {
  const int per = (n + nt - 1) / nt;
  return per <= 8 ? 8 : (per <= 16 ? 16 : 32);
}

// elements per thread of the joint-aligned stride-1 LDS backward kernels (stride
// (nt / W) * W); 0 = the plane does not fit 32 per thread. 512-thread workgroups also take
// 12 and 20: a thread holds ~5 VGPRs per element, and at 24 the shift_out backward (bnin)
// and the GBD backward held 141-143 VGPRs — one 512-thread workgroup per CU on MediaPipe's
// 9,900-float planes (W = 33, exactly 20 per thread); at 20 two fit (likewise 12 against 16
// for its 4,950-float T = 150 planes: three instead of two)
int ra_lpt(int n, int nt, int W) {
  const int nte = (nt / W) * W;
  if (nte <= 0 || W > 64) return 0;
  const int per = (n + nte - 1) / nte;
  if (nt == 512 && per > 8 && per <= 12) return 12;
  if (nt == 512 && per > 16 && per <= 20) return 20;
  return per <= 8 ? 8 : (per <= 16 ? 16 : (per <= 24 ? 24 : (per <= 32 ? 32 : 0)));
}

// largest stride-1 plane the joint-aligned backward kernels with affine taps (shift_in:
// plain and GBN) run on 256-thread workgroups (up to 32 elements per thread): at NTU T=300
// (7,500 floats) measured 8 % (GBN) / 4 % (plain) faster than 512 threads; the shift_out
// backward (bnin) keeps 512 threads above 4,096 floats (no difference)
constexpr int kRaSplit256 = 8192;
#ifndef SGCN_GBD_SPLIT
#define SGCN_GBD_SPLIT 1
#endif

// LDS bytes of the padded stride-1 backward (GBN reuses it for 6*NT partial sums)
size_t ra_lds_bytes(int H, int W, int nt, bool gbn) {
  const int f = ra_pad_floats(H, W);
  return (size_t)(gbn ? max(f + 1, 6 * nt) : f + 1) * sizeof(float);   // + the spare float
}
constexpr size_t kRaLdsMax = 65536;

// launch tshift_bwd_ra_kernel on nt threads (256 or 512) with LPT = ra_lpt(H*W, nt, W);
// returns false (nothing launched) when the plane does not fit its LDS or registers
template <bool AFFINE, bool RELU, bool BNP, bool GP, bool GBN, bool GBD = false>
bool launch_ra(int nt, const float* gout, const float* in, const float* xpos,
               const float* ypos, const float* scale, const float* shift, const float* bmu,
               const float* bis, float* gin, float2* pg, float2* bp, int B, int C, int H,
               int W, const float* gdy, const float* gy, const float* gx, const float* gcoef,
               const float* gz, const float* gzm, const float* gzi, float* gzpart,
               hipStream_t st, const float* gd = nullptr, const float* gdm = nullptr,
               const float* gdi = nullptr, float* gdpart = nullptr) {
  const int lpt = ra_lpt(H * W, nt, W);
  const size_t lds = ra_lds_bytes(H, W, nt, GBN);
  if (lpt == 0 || lds > kRaLdsMax) return false;
#define SGCN_RA(NT, L)                                                                         \
  tshift_bwd_ra_kernel<NT, L, AFFINE, RELU, BNP, GP, GBN, GBD><<<B * C, NT, lds, st>>>(        \
      gout, in, xpos, ypos, scale, shift, bmu, bis, gin, pg, bp, C, H, W, gdy, gy, gx, gcoef,  \
      gz, gzm, gzi, gzpart, gd, gdm, gdi, gdpart)
  if (nt == 256) {
    if (lpt == 8) SGCN_RA(256, 8); else if (lpt == 16) SGCN_RA(256, 16); else if (lpt == 24) SGCN_RA(256, 24); else SGCN_RA(256, 32);
  } else {
    if (lpt == 8) SGCN_RA(512, 8); else if (lpt == 12) SGCN_RA(512, 12); else if (lpt == 16) SGCN_RA(512, 16);
    else if (lpt == 20) SGCN_RA(512, 20); else if (lpt == 24) SGCN_RA(512, 24); else SGCN_RA(512, 32);
  }
#undef SGCN_RA
  return true;
}

int pick_ept(int n) {
  const int per = (n + kThreads - 1) / kThreads;
  return per <= 8 ? 8 : (per <= 16 ? 16 : 32);
}

}  // namespace
}  // namespace sgcn

using namespace sgcn;

extern "C" {

int sgcn_tshift_fwd(const float* in, float* out, const float* xpos, const float* ypos,
                    const float* in_scale, const float* in_shift, float* plane_stats, int B,
                    int C, int H, int W, int stride, int ypos_is_raw, void* stream) {
  SGCN_REQUIRE(B >= 0 && C > 0 && H >= 0 && W > 0 && stride >= 1);
  SGCN_REQUIRE((in_scale == nullptr) == (in_shift == nullptr));
  const int Ho = H / stride;
  if (B == 0 || Ho == 0) return 0;
  SGCN_REQUIRE(in && out && xpos && ypos);
  SGCN_REQUIRE((long long)H * W < (1LL << 30) && (long long)B * C < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const bool aff = in_scale != nullptr, stats = plane_stats != nullptr;
  float2* ps = (float2*)plane_stats;
  const int ah = (ypos_is_raw && stride != 1) ? 1 : 0;
  // padded joint-aligned kernel (W <= 64): 256 threads up to kFwdLdsMax floats, else 512
  if (H * W <= kFwdLdsMax2 &&
      (H * W <= kFwdLdsMax
           ? launch_fwd_pad<kThreads>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st)
           : launch_fwd_pad<512>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st))) {
    SGCN_LAUNCH_CHECK();
    return 0;
  }
  if (H * W <= kFwdLdsMax) {
    switch (pick_lpt(H * W, kThreads)) {
      case 8: launch_fwd_lds<8>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st); break;
      case 16: launch_fwd_lds<16>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st); break;
      default: launch_fwd_lds<32>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st); break;
    }
    SGCN_LAUNCH_CHECK();
    return 0;
  }
  if (H * W <= kFwdLdsMax2) {   // 512 threads x 32 staged elements
    launch_fwd_lds<32, 512>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st);
    SGCN_LAUNCH_CHECK();
    return 0;
  }
  switch (pick_ept(Ho * W)) {
    case 8: launch_fwd<8>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st); break;
    case 16: launch_fwd<16>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st); break;
    default: launch_fwd<32>(aff, stats, in, out, xpos, ypos, in_scale, in_shift, ps, B, C, H, W, Ho, stride, ah, st); break;
  }
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_tshift_fwd_pre(const float* z, float* out, const float* xpos, const float* ypos,
                        const float* pre_scale, const float* pre_shift, const float* r,
                        const float* r_scale, const float* r_shift, const float* in_scale,
                        const float* in_shift, int B, int C, int H, int W, int stride,
                        int ypos_is_raw, void* stream) {
  SGCN_REQUIRE(B >= 0 && C > 0 && H >= 0 && W > 0 && W <= 1024 && stride >= 1);
  SGCN_REQUIRE((r_scale == nullptr) == (r_shift == nullptr));
  SGCN_REQUIRE(H * W <= kFwdLdsMax2);   // LDS-staged planes only (caller falls back)
  const int Ho = H / stride;
  if (B == 0 || Ho == 0) return 0;
  SGCN_REQUIRE(z && out && xpos && ypos && pre_scale && pre_shift && r && in_scale &&
               in_shift && out != z);
  SGCN_REQUIRE((long long)B * C < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const int ah = (ypos_is_raw && stride != 1) ? 1 : 0;
  {   // padded joint-aligned kernel (W <= 64)
    const int nt = H * W <= kFwdLdsMax ? kThreads : 512;
    const int lpt = pad_fwd_lpt(H, W, nt);
    if (lpt) {
      const size_t plds = (size_t)(ra_pad_floats(H, W) + 1) * sizeof(float);
#define SGCN_PREP(NT, L, R)                                                                    \
  tshift_fwd_pad_kernel<NT, L, 1, true, false, R><<<B * C, NT, plds, st>>>(                    \
      z, out, xpos, ypos, in_scale, in_shift, nullptr, C, H, W, Ho, stride, ah, pre_scale,      \
      pre_shift, r, r_scale, r_shift)
#define SGCN_PREP_R(NT, L) \
  do { if (r_scale) SGCN_PREP(NT, L, 2); else SGCN_PREP(NT, L, 1); } while (0)
      if (nt == kThreads) {
        if (lpt == 8) SGCN_PREP_R(kThreads, 8); else if (lpt == 16) SGCN_PREP_R(kThreads, 16); else if (lpt == 24) SGCN_PREP_R(kThreads, 24); else SGCN_PREP_R(kThreads, 32);
      } else {
        if (lpt == 8) SGCN_PREP_R(512, 8); else if (lpt == 12) SGCN_PREP_R(512, 12); else if (lpt == 16) SGCN_PREP_R(512, 16);
        else if (lpt == 20) SGCN_PREP_R(512, 20); else if (lpt == 24) SGCN_PREP_R(512, 24); else SGCN_PREP_R(512, 32);
      }
#undef SGCN_PREP_R
#undef SGCN_PREP
      SGCN_LAUNCH_CHECK();
      return 0;
    }
  }
  const size_t lds = (size_t)H * W * sizeof(float);
#define SGCN_PRE(NT, L, R)                                                                     \
  tshift_fwd_pre_kernel<NT, L, R><<<B * C, NT, lds, st>>>(z, out, xpos, ypos, pre_scale,       \
                                                           pre_shift, r, r_scale, r_shift,     \
                                                           in_scale, in_shift, C, H, W, Ho,    \
                                                           stride, ah)
#define SGCN_PRE_R(NT, L) \
  do { if (r_scale) SGCN_PRE(NT, L, 2); else SGCN_PRE(NT, L, 1); } while (0)
  if (H * W <= kFwdLdsMax) {
    switch (pick_lpt(H * W, kThreads)) {
      case 8: SGCN_PRE_R(kThreads, 8); break;
      case 16: SGCN_PRE_R(kThreads, 16); break;
      default: SGCN_PRE_R(kThreads, 32); break;
    }
  } else {
    SGCN_PRE_R(512, 32);
  }
#undef SGCN_PRE_R
#undef SGCN_PRE
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_tshift_fwd_tail(const float* in, float* out, const float* xpos, const float* ypos,
                         const float* post_scale, const float* post_shift, const float* r,
                         const float* r_scale, const float* r_shift, const float* gather_m,
                         float* out_gathered, int B, int C, int H, int W, int stride,
                         int ypos_is_raw, void* stream) {
  SGCN_REQUIRE(B >= 0 && C > 0 && H >= 0 && W > 0 && W <= 1024 && stride >= 1);
  SGCN_REQUIRE((r_scale == nullptr) == (r_shift == nullptr) && (r || !r_scale));
  SGCN_REQUIRE((gather_m == nullptr) == (out_gathered == nullptr));
  SGCN_REQUIRE(H * W <= kFwdLdsMax2);   // LDS-staged planes only (caller falls back)
  const int Ho = H / stride;
  if (B == 0 || Ho == 0) return 0;
  SGCN_REQUIRE(in && out && xpos && ypos && post_scale && post_shift && out != in);
  SGCN_REQUIRE((long long)B * C < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const int ah = (ypos_is_raw && stride != 1) ? 1 : 0;
  const int res = r == nullptr ? 0 : (r_scale ? 2 : 1);
  const bool go = out_gathered != nullptr;
  {   // padded joint-aligned kernel (W <= 64)
    const int nt = H * W <= kFwdLdsMax ? kThreads : 512;
    const int lpt = pad_fwd_lpt(H, W, nt);
    if (lpt) {
      const size_t plds = (size_t)(ra_pad_floats(H, W) + 1) * sizeof(float);
#define SGCN_TAILP(NT, L, R, G)                                                                \
  tshift_fwd_pad_kernel<NT, L, 2, false, false, R, G><<<B * C, NT, plds, st>>>(                \
      in, out, xpos, ypos, post_scale, post_shift, nullptr, C, H, W, Ho, stride, ah, nullptr,  \
      nullptr, r, r_scale, r_shift, gather_m, out_gathered)
#define SGCN_TAILP_RG(NT, L)                                                                   \
  do {                                                                                         \
    if (res == 0) { if (go) SGCN_TAILP(NT, L, 0, true); else SGCN_TAILP(NT, L, 0, false); }    \
    else if (res == 1) { if (go) SGCN_TAILP(NT, L, 1, true); else SGCN_TAILP(NT, L, 1, false); } \
    else { if (go) SGCN_TAILP(NT, L, 2, true); else SGCN_TAILP(NT, L, 2, false); }             \
  } while (0)
      if (nt == kThreads) {
        if (lpt == 8) SGCN_TAILP_RG(kThreads, 8); else if (lpt == 16) SGCN_TAILP_RG(kThreads, 16); else if (lpt == 24) SGCN_TAILP_RG(kThreads, 24); else SGCN_TAILP_RG(kThreads, 32);
      } else {
        if (lpt == 8) SGCN_TAILP_RG(512, 8); else if (lpt == 12) SGCN_TAILP_RG(512, 12); else if (lpt == 16) SGCN_TAILP_RG(512, 16);
        else if (lpt == 20) SGCN_TAILP_RG(512, 20); else if (lpt == 24) SGCN_TAILP_RG(512, 24); else SGCN_TAILP_RG(512, 32);
      }
#undef SGCN_TAILP_RG
#undef SGCN_TAILP
      SGCN_LAUNCH_CHECK();
      return 0;
    }
  }
  const size_t lds = (size_t)H * W * sizeof(float);
#define SGCN_TAIL(NT, L, R, G)                                                                \
  tshift_fwd_tail_kernel<NT, L, R, G><<<B * C, NT, lds, st>>>(                                \
      in, out, xpos, ypos, post_scale, post_shift, r, r_scale, r_shift, gather_m,            \
      out_gathered, C, H, W, Ho, stride, ah)
#define SGCN_TAIL_RG(NT, L)                                                                   \
  do {                                                                                        \
    if (res == 0) { if (go) SGCN_TAIL(NT, L, 0, true); else SGCN_TAIL(NT, L, 0, false); }     \
    else if (res == 1) { if (go) SGCN_TAIL(NT, L, 1, true); else SGCN_TAIL(NT, L, 1, false); } \
    else { if (go) SGCN_TAIL(NT, L, 2, true); else SGCN_TAIL(NT, L, 2, false); }              \
  } while (0)
  if (H * W <= kFwdLdsMax) {
    switch (pick_lpt(H * W, kThreads)) {
      case 8: SGCN_TAIL_RG(kThreads, 8); break;
      case 16: SGCN_TAIL_RG(kThreads, 16); break;
      default: SGCN_TAIL_RG(kThreads, 32); break;
    }
  } else {
    SGCN_TAIL_RG(512, 32);
  }
#undef SGCN_TAIL_RG
#undef SGCN_TAIL
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_tshift_bwd_bnin(const float* dy, const float* y, const float* s, const float* coef,
                         const float* in, const float* xpos, const float* ypos, float* gin,
                         float* gx, float* gy, void* ws, size_t ws_bytes, int B, int C, int H,
                         int W, int ypos_is_raw, void* stream) {
  SGCN_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0);
  SGCN_REQUIRE(H * W <= kBwdLdsMax);   // LDS-staged stride-1 planes only (caller falls back)
  SGCN_REQUIRE(dy && y && s && coef && in && xpos && ypos && gin && ws);
  SGCN_REQUIRE((gx == nullptr) == (gy == nullptr));
  SGCN_REQUIRE(ws_bytes >= sgcn_tshift_bwd_ws_bytes(B, C));
  SGCN_REQUIRE((long long)B * C < (1LL << 31));
  (void)ypos_is_raw;   // stride 1: the +0.5 of shift.py:17-18 never applies
  hipStream_t st = (hipStream_t)stream;
  float2* pg = (float2*)ws;
  // 512 threads above 4K-float planes: 256 threads at NTU T = 300 measured 0.3 % slower per
  // step (profiles/r03_x1b/ab_x1b_bound.txt, variant bnin256)
  const int ntb = H * W <= 4096 ? 256 : 512;
  const bool ok = launch_ra<false, true, false, true, false>(
      ntb, nullptr, in, xpos, ypos, nullptr, nullptr, nullptr, nullptr, gin, pg, nullptr, B, C,
      H, W, dy, y, s, coef, nullptr, nullptr, nullptr, nullptr, st);
  SGCN_REQUIRE(ok);   // W <= 64, <= 32 elements per thread, padded plane <= 64 KiB (ops.ra_fits)
  SGCN_LAUNCH_CHECK();
  if (gx) tshift_pos_finalize_kernel<<<(C + 3) / 4, 256, 0, st>>>(pg, B, C, gx, gy);
  SGCN_LAUNCH_CHECK();
  return 0;
}

size_t sgcn_tshift_bwd_ws_bytes(int B, int C) { return (size_t)B * C * sizeof(float2); }

int sgcn_tshift_pos_finalize_many(const void* const* partials, float* const* gx,
                                  float* const* gy, const int* B, const int* C, int n,
                                  void* stream) {
  SGCN_REQUIRE(n >= 0 && n <= SGCN_BATCH_MAX);
  if (n == 0) return 0;
  SGCN_REQUIRE(partials && gx && gy && B && C);
  PosBatch t{};
  int max_c = 0;
  for (int i = 0; i < n; ++i) {
    SGCN_REQUIRE(partials[i] && gx[i] && gy[i] && B[i] > 0 && C[i] > 0);
    t.p[i] = (const float2*)partials[i];
    t.gx[i] = gx[i];
    t.gy[i] = gy[i];
    t.B[i] = B[i];
    t.C[i] = C[i];
    max_c = max(max_c, C[i]);
  }
  tshift_pos_finalize_many_kernel<<<dim3((max_c + 3) / 4, n), 256, 0, (hipStream_t)stream>>>(t);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_tshift_pos_finalize(const void* ws, int B, int C, float* gx, float* gy, void* stream) {
  SGCN_REQUIRE(B > 0 && C > 0 && ws && gx && gy);
  tshift_pos_finalize_kernel<<<(C + 3) / 4, 256, 0, (hipStream_t)stream>>>((const float2*)ws, B,
                                                                           C, gx, gy);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_tshift_bwd_gbn(const float* gout, const float* in, const float* xpos,
                        const float* ypos, const float* in_scale, const float* in_shift,
                        const float* bn_mean, const float* bn_invstd, float* bn_part,
                        const float* z, const float* z_mean, const float* z_invstd,
                        float* z_part, const float* d, const float* d_mean,
                        const float* d_invstd, float* d_part, float* gin, float* gx, float* gy,
                        void* ws, size_t ws_bytes, int B, int C, int H, int W, void* stream) {
  SGCN_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0 && W <= 64);
  SGCN_REQUIRE((d == nullptr) == (d_part == nullptr) && (!d || (d_mean && d_invstd)));
  SGCN_REQUIRE(H * W <= kBwdLdsMax);   // LDS-staged stride-1 planes only (caller falls back)
  SGCN_REQUIRE(gout && in && xpos && ypos && in_scale && in_shift && bn_mean && bn_invstd &&
               bn_part && z && z_mean && z_invstd && z_part && gin && ws);
  SGCN_REQUIRE((gx == nullptr) == (gy == nullptr));
  SGCN_REQUIRE(ws_bytes >= sgcn_tshift_bwd_ws_bytes(B, C));
  SGCN_REQUIRE((long long)B * C < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  float2* pg = (float2*)ws;
  float2* bp = (float2*)bn_part;
  // sgcn_tshift_bwd's stride-1 thread counts; elements per thread from the W-aligned
  // stride (NT / W) * W; 512 threads when 256 would need more than 32 per thread. With the
  // down BatchNorm's sums (GBD) a 32-element thread holds 183 VGPRs (two 256-thread
  // workgroups per CU): such planes take 512 threads x 16 (107 VGPRs, two 512-thread
  // workgroups) (SGCN_GBD_SPLIT=0: 256 threads as GBN)
  const int n = H * W;
  const int l256 = n <= kRaSplit256 ? ra_lpt(n, 256, W) : 0;
  const int ntg = l256 && !(SGCN_GBD_SPLIT && d && l256 > 24) ? 256 : kBwdThreads;
  const bool ok =
      d ? launch_ra<true, false, true, false, true, true>(
              ntg, gout, in, xpos, ypos, in_scale, in_shift, bn_mean, bn_invstd, gin, pg, bp, B,
              C, H, W, nullptr, nullptr, nullptr, nullptr, z, z_mean, z_invstd, z_part, st, d,
              d_mean, d_invstd, d_part)
        : launch_ra<true, false, true, false, true>(
              ntg, gout, in, xpos, ypos, in_scale, in_shift, bn_mean, bn_invstd, gin, pg, bp, B,
              C, H, W, nullptr, nullptr, nullptr, nullptr, z, z_mean, z_invstd, z_part, st);
  SGCN_REQUIRE(ok);   // within the largest LPT and 64 KiB of LDS (ops.ra_fits)
  SGCN_LAUNCH_CHECK();
  if (gx) tshift_pos_finalize_kernel<<<(C + 3) / 4, 256, 0, st>>>(pg, B, C, gx, gy);
  SGCN_LAUNCH_CHECK();
  return 0;
}

int sgcn_tshift_bwd(const float* gout, const float* in, const float* xpos, const float* ypos,
                    const float* in_scale, const float* in_shift, int relu_mask,
                    const float* bn_mean, const float* bn_invstd, float* bn_part, float* gin,
                    float* gx, float* gy, void* ws, size_t ws_bytes, int B, int C, int H,
                    int W, int stride, int ypos_is_raw, void* stream) {
  SGCN_REQUIRE(B > 0 && C > 0 && H >= 0 && W > 0 && (stride == 1 || stride == 2));
  SGCN_REQUIRE((in_scale == nullptr) == (in_shift == nullptr));
  const int Ho = H / stride;
  SGCN_REQUIRE((gout || Ho == 0) && (in || H == 0) && (gin || H == 0));
  SGCN_REQUIRE(xpos && ypos && ws && (gx == nullptr) == (gy == nullptr));
  SGCN_REQUIRE(!bn_part || (bn_mean && bn_invstd));
  SGCN_REQUIRE(ws_bytes >= sgcn_tshift_bwd_ws_bytes(B, C));
  SGCN_REQUIRE((long long)H * W < (1LL << 30) && (long long)B * C < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const bool aff = in_scale != nullptr, relu = relu_mask != 0;
  float2* pg = (float2*)ws;
  float2* bp = (float2*)bn_part;
  const int ah = (ypos_is_raw && stride != 1) ? 1 : 0;
  // stride 1: the padded joint-aligned LDS kernel (W <= 64, <= 32 elements per thread,
  // <= 64 KiB of LDS); small planes (T = 150 / 75) on 256 threads, so fewer lanes idle per
  // workgroup; anything else takes the global-tap kernel below
  if (stride == 1 && H > 0) {
    // (256 threads only where 32 elements per thread cover the plane, as the GBN launcher)
    const int nt1 = H * W <= kRaSplit256 && ra_lpt(H * W, 256, W) ? 256 : kBwdThreads;
    bool done;
#define SGCN_RA1(A, R, P)                                                                       done = launch_ra<A, R, P, false, false>(nt1, gout, in, xpos, ypos, in_scale, in_shift,                                                 bn_mean, bn_invstd, gin, pg, bp, B, C, H, W, nullptr,                                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,                                           nullptr, st)
    if (bp) {
      if (aff) { if (relu) SGCN_RA1(true, true, true); else SGCN_RA1(true, false, true); }
      else { if (relu) SGCN_RA1(false, true, true); else SGCN_RA1(false, false, true); }
    } else {
      if (aff) { if (relu) SGCN_RA1(true, true, false); else SGCN_RA1(true, false, false); }
      else { if (relu) SGCN_RA1(false, true, false); else SGCN_RA1(false, false, false); }
    }
#undef SGCN_RA1
    if (done) {
      SGCN_LAUNCH_CHECK();
      if (gx) tshift_pos_finalize_kernel<<<(C + 3) / 4, 256, 0, st>>>(pg, B, C, gx, gy);
      SGCN_LAUNCH_CHECK();
      return 0;
    }
  }
  if (stride == 2 && (H + Ho) * W <= kBwdLdsMax && H > 0) {
    const int lpt = pick_lpt((H + Ho) * W, kBwdThreads);
#define SGCN_BWDL_LPT(L, J)                                                                   \
  launch_bwd_s2<L, J>(aff, relu, gout, in, xpos, ypos, in_scale, in_shift, bn_mean, bn_invstd, \
                      gin, pg, bp, B, C, H, W, Ho, ah, st)
    if (W <= 64) {   // joint-aligned walk (W <= NT)
      if (lpt == 8) SGCN_BWDL_LPT(8, true); else if (lpt == 16) SGCN_BWDL_LPT(16, true);
      else SGCN_BWDL_LPT(32, true);
    } else {
      if (lpt == 8) SGCN_BWDL_LPT(8, false); else if (lpt == 16) SGCN_BWDL_LPT(16, false);
      else SGCN_BWDL_LPT(32, false);
    }
#undef SGCN_BWDL_LPT
  } else {
  const int ept = pick_ept(H * W);
#define SGCN_BWD_EPT(E)                                                                     \
  (stride == 1 ? launch_bwd<E, 1>(aff, relu, gout, in, xpos, ypos, in_scale, in_shift, \
                                  bn_mean, bn_invstd, gin, pg, bp, B, C, H, W, Ho, ah, st)                                   \
               : launch_bwd<E, 2>(aff, relu, gout, in, xpos, ypos, in_scale, in_shift, \
                                  bn_mean, bn_invstd, gin, pg, bp, B, C, H, W, Ho, ah, st))
  if (ept == 8) SGCN_BWD_EPT(8); else if (ept == 16) SGCN_BWD_EPT(16); else SGCN_BWD_EPT(32);
#undef SGCN_BWD_EPT
  }
  SGCN_LAUNCH_CHECK();
  if (gx) tshift_pos_finalize_kernel<<<(C + 3) / 4, 256, 0, st>>>(pg, B, C, gx, gy);
  SGCN_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
