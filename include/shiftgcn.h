/*
 * shiftgcn.h — C ABI of the MI355X (gfx950) Shift-GCN hot path.
 *
 * Drop-in boundary for the reference's native layer. Every entry point:
 *   - takes raw DEVICE pointers (fp32, contiguous, (N·M, C, T, V) = NCHW layout unless
 *     stated), plain int dims and an opaque hipStream_t (void*, NULL = default stream);
 *   - enqueues asynchronously on that stream only (graph-capture safe: no allocation, no
 *     host sync, no hidden state); workspace is caller-provided, sized by a *_ws_bytes()
 *     query;
 *   - returns 0 on success, SGCN_EINVAL (-22) on a bad argument (nothing enqueued), or a
 *     positive hipError_t from the launch;
 *   - is reentrant (no globals).
 * Ownership: all buffers are borrowed; nothing is allocated or freed.
 */
#ifndef SHIFTGCN_H_
#define SHIFTGCN_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGCN_EINVAL (-22)
#define SGCN_ABI_VERSION 23
/* Set in sgcn_abi_version()'s value by a diagnostic build (SGCN_PW_DIAG, SGCN_PW_STAMPS,
 * SGCN_DIAG_*: timing probes whose results are WRONG, `make diag` only); the Python loader
 * refuses such a library. */
#define SGCN_ABI_DIAG_FLAG 0x10000

/* ABI version of the loaded library (== SGCN_ABI_VERSION). 19: the measured-and-rejected
 * variants are gone (the S-free unit tail's statistics-only shift and re-formed bn2 input,
 * the re-forming temporal-shift weight gradient, per_joint = 1 / 2 rotated-store layouts).
 * 20: sgcn_tshift_bwd_gbn also takes the down conv's BatchNorm (d, d_mean, d_invstd,
 * d_part; NULL when the Shift_gcn has none); sgcn_sgd_step (the optimizer update).
 * 21: sgcn_sgd_step's per-tensor gradient scale (flags bit 1 + the float in bits 32-63: the
 * data-parallel reduction's 1/world applied inside the update, written back to the grad);
 * 22: the round-4 measured-and-rejected variants are gone (the folded BatchNorm finalizes
 * sgcn_bn_fold / sgcn_bn_bwd_fold and their consumers sgcn_tshift_fwd_fold,
 * sgcn_bn_apply_fold, sgcn_tshift_bwd_bnin_fold, sgcn_bn_bwd_apply_fold; the inference
 * epilogue sgcn_pw_fwd_bn_res; the CU-masked streams), and so are the fold structs in the
 * default kernels' argument lists.
 * 23: sgcn_sgd_step flags bit 2 (the (weight_decay, lr) column as the device address of a
 * float pair: hyper-parameters of a graph-captured step read at replay); sgcn_pw_fwd_tshift
 * takes two_row (the two-tap operand of channels with |xpos| < 2^-25). */
int sgcn_abi_version(void);

/* ------------------------------------------------------------------------------------
 * Temporal shift
 * ------------------------------------------------------------------------------------ */

/* Forward learnable fractional temporal shift.
 * Replaces `shift_cuda.forward(input, xpos, ypos, stride)`
 *   (model/Temporal_shift/cuda/shift_cuda.cpp:19-23 -> shift_cuda_kernel.cu:405-431).
 * in  : (B, C, H, W);  out: (B, C, H/stride, W);  xpos, ypos: (C) Shift parameters.
 * ypos_is_raw != 0: ypos is the raw module parameter and the +0.5 that ShiftFunction adds
 *   for stride != 1 (shift.py:17-18) is applied INSIDE the kernel as the same float32 add
 *   (the product path: no extra elementwise launch). ypos_is_raw == 0: ypos already holds
 *   the shifted value, exactly what the reference glue passes to shift_cuda.forward.
 * in_scale/in_shift: optional per-channel affine (C) applied to every in-range input tap
 *   (a fused BatchNorm apply); both NULL = identity.
 * plane_stats: optional (B*C) float2 {mean, M2} of each output plane (n = H/stride*W),
 *   consumed by sgcn_bn_finalize(); NULL = not computed.
 * Unlike the reference (at::zeros + kernel), every output element is written exactly
 * once (no memset pass). */
int sgcn_tshift_fwd(const float* in, float* out, const float* xpos, const float* ypos,
                    const float* in_scale, const float* in_shift, float* plane_stats,
                    int B, int C, int H, int W, int stride, int ypos_is_raw, void* stream);

/* Inference-mode Shift_gcn tail fused into Shift_tcn's shift_in forward (shift_gcn.py:
 * 137-141 then 67-68, BatchNorms in eval mode): out = shift(in_scale[c]*H + in_shift[c]),
 * H = relu(z*pre_scale[c*W+w] + pre_shift[c*W+w] + res) formed while staging, z the gcn
 * contraction output Z, res = r (identity down) or r*r_scale[c] + r_shift[c] (down conv
 * output with its eval BN). H is never written. H*W <= 16384 only (else SGCN_EINVAL). */
int sgcn_tshift_fwd_pre(const float* z, float* out, const float* xpos, const float* ypos,
                        const float* pre_scale, const float* pre_shift, const float* r,
                        const float* r_scale, const float* r_shift, const float* in_scale,
                        const float* in_shift, int B, int C, int H, int W, int stride,
                        int ypos_is_raw, void* stream);

/* Unit tail fused into Shift_tcn's shift_out forward (shift_gcn.py:72-73, 161-162):
 * out = relu(shift(in)*post_scale[c] + post_shift[c]
 * + res), res = 0 (r NULL), r (identity residual) or r*r_scale[c] + r_shift[c] (residual
 * tcn conv output with its eval BN), r laid out like out. gather_m/out_gathered (both or
 * neither): also out_gathered = sgcn_gcn_gather(out, gather_m) for the next unit. The
 * shifted tensor itself is never written. post_scale/post_shift are bn2's eval-mode
 * apply coefficients (sgcn_bn_eval_coef): the inference tail. Planes with H*W <= 16384
 * only (else SGCN_EINVAL: use sgcn_tshift_fwd + sgcn_bn_apply). */
int sgcn_tshift_fwd_tail(const float* in, float* out, const float* xpos, const float* ypos,
                         const float* post_scale, const float* post_shift, const float* r,
                         const float* r_scale, const float* r_shift, const float* gather_m,
                         float* out_gathered, int B, int C, int H, int W, int stride,
                         int ypos_is_raw, void* stream);

/* sgcn_tshift_bwd (stride 1, ReLU mask on `in`, no affine) whose gout is the input
 * gradient of the BatchNorm that follows the shift inside a TCN_GCN_unit (Shift_tcn.bn2,
 * shift_gcn.py:73,161-162), formed while staging: gout = k1*(y > 0 ? dy : 0) + k2*s + k3
 * with dy/y the unit's output gradient/output, s = bn2's input, coef = [3][C] {k1,k2,k3}
 * from sgcn_bn_bwd_finalize. That gradient tensor is never written. Plane limits:
 * H*W <= 16384, W <= 64, <= 32 elements per thread of the joint-aligned stride (NT / W) * W,
 * NT = 256 (H*W <= 4096) or 512 (else SGCN_EINVAL: use sgcn_bn_bwd_apply +
 * sgcn_tshift_bwd). */
int sgcn_tshift_bwd_bnin(const float* dy, const float* y, const float* s, const float* coef,
                         const float* in, const float* xpos, const float* ypos, float* gin,
                         float* gx, float* gy, void* ws, size_t ws_bytes, int B, int C, int H,
                         int W, int ypos_is_raw, void* stream);
/* Workspace bytes for sgcn_tshift_bwd (B*C float2 plane partials). */
size_t sgcn_tshift_bwd_ws_bytes(int B, int C);

/* The position-gradient step of sgcn_tshift_bwd / _bnin / _gbn on its own: gx, gy from the
 * per-plane partials those calls leave in `ws` (mean over the batch, then
 * applyShiftConstraint, .cu:370-395, 501-509). Those calls skip this step when given
 * gx = gy = NULL, so it can run later / on another stream (the positions' gradients are
 * needed only by the optimizer); ws must then stay untouched until it has run. */
int sgcn_tshift_pos_finalize(const void* ws, int B, int C, float* gx, float* gy, void* stream);

/* Backward of the temporal shift. Replaces
 * `shift_cuda.backward(grad_output, input, output, xpos, ypos, stride)`
 *   (shift_cuda.cpp:25-42 -> shift_cuda_kernel.cu:433-523).
 * gout: (B, C, H/stride, W); in: (B, C, H, W) forward input; xpos/ypos and
 * ypos_is_raw as in the forward (the reference passes the saved shifted ypos, raw = 0).
 * gin : (B, C, H, W) input gradient (reference Shift_Bottom_Backward*, .cu:78-256);
 * gx, gy: (C) position gradients = mean over batch of the summed position products
 *   (both NULL: not computed here; the partials stay in ws for sgcn_tshift_pos_finalize)
 *   (.cu:277-363, 501-509) after applyShiftConstraint (.cu:370-395).
 * in_scale/in_shift: same optional affine as the forward (the position products then
 *   use the affine taps). relu_mask != 0: gin[p] = 0 where in[p] <= 0 (fused ReLU
 *   backward for a shift whose input is a ReLU output).
 * bn_mean/bn_invstd/bn_part (optional, all or none): also write bn_part[b*C+c] =
 *   {sum gin, sum gin*(in - bn_mean[c])*bn_invstd[c]} over the plane — the
 *   sgcn_bn_bwd_reduce() partials of the BatchNorm whose output feeds this shift
 *   (Shift_tcn.bn -> shift_in), without another pass over gin and in.
 * stride must be 1 or 2 (the reference backward hard-codes 2 for stride != 1). */
int sgcn_tshift_bwd(const float* gout, const float* in, const float* xpos, const float* ypos,
                    const float* in_scale, const float* in_shift, int relu_mask,
                    const float* bn_mean, const float* bn_invstd, float* bn_part, float* gin,
                    float* gx, float* gy, void* ws, size_t ws_bytes, int B, int C, int H,
                    int W, int stride, int ypos_is_raw, void* stream);

/* Double-precision forward / backward of the temporal shift: the reference's double
 * instantiation (AT_DISPATCH_FLOATING_TYPES, shift_cuda_kernel.cu:413, :455-520), e.g. for
 * gradcheck of the input gradient. Same arguments and semantics as sgcn_tshift_fwd /
 * sgcn_tshift_bwd without the fused options; `int x1 = floorf(x)` rounds the double x to
 * float first, exactly as the reference. Workspace: sgcn_tshift_bwd_f64_ws_bytes(B, C). */
int sgcn_tshift_fwd_f64(const double* in, double* out, const double* xpos, const double* ypos,
                        int B, int C, int H, int W, int stride, int ypos_is_raw, void* stream);
size_t sgcn_tshift_bwd_f64_ws_bytes(int B, int C);
int sgcn_tshift_bwd_f64(const double* gout, const double* in, const double* xpos,
                        const double* ypos, double* gin, double* gx, double* gy, void* ws,
                        size_t ws_bytes, int B, int C, int H, int W, int stride,
                        int ypos_is_raw, void* stream);

/* Shift_tcn.shift_in backward inside a TCN_GCN_unit whose Shift_gcn has no down conv
 * (shift_gcn.py:137-141 then :66-68): exactly sgcn_tshift_bwd(stride 1, in_scale/in_shift,
 * bn_mean/bn_invstd/bn_part) — same gin, gx, gy, bn_part — and in the same launch the
 * k-free backward sums of Shift_gcn.bn (the per-joint BatchNorm1d whose ReLU output is
 * `in`): z_part[j][b*C*W + c*W + w], j = {sum gin, sum (in - mu), sum 1, sum gin*zh,
 * sum (in - mu)*zh, sum zh} over t where in > 0, zh = (z - z_mean[c*W+w]) *
 * z_invstd[c*W+w], mu = bn_mean[c]; z = that BatchNorm's input as the gcn contraction
 * stored it BEFORE its shift_out (per_joint = 3 layout: logical joint w at (w - c) mod W),
 * statistics in the per-joint local order. Feed z_part to
 * sgcn_bn_bwd_finalize_gbn; no separate sgcn_bn_bwd_reduce pass over (gin, in, z).
 * d (optional, with d_mean/d_invstd/d_part; ABI 20): a Shift_gcn WITH a down conv, whose
 * BatchNorm2d output is added before the ReLU (in = relu(bn(z) + bnd(d))): d_part[j][b*C + c]
 * = the same six sums over the plane with zh replaced by dh = (d - d_mean[c]) * d_invstd[c]
 * (d in the natural layout), finalized by sgcn_bn_bwd_finalize_gbn with V = 1 — the down
 * BatchNorm's backward sums without a reduce pass either.
 * H*W <= 16384, W <= 64 and at most 32 elements per thread of the joint-aligned stride
 * (NT / W) * W, NT = 256 (H*W <= 8192; 512 if 256 would need more than 32) or 512 (else
 * SGCN_EINVAL: use sgcn_tshift_bwd + sgcn_bn_bwd_reduce). */
int sgcn_tshift_bwd_gbn(const float* gout, const float* in, const float* xpos,
                        const float* ypos, const float* in_scale, const float* in_shift,
                        const float* bn_mean, const float* bn_invstd, float* bn_part,
                        const float* z, const float* z_mean, const float* z_invstd,
                        float* z_part, const float* d, const float* d_mean,
                        const float* d_invstd, float* d_part, float* gin, float* gx, float* gy,
                        void* ws, size_t ws_bytes, int B, int C, int H, int W, void* stream);

/* ------------------------------------------------------------------------------------
 * Pointwise (1x1) channel contraction with the joint-shift gathers fused (fp32 MFMA)
 * ------------------------------------------------------------------------------------
 * Plane operand addressing: element (b, ch, n), n = t*V + v, of a plane tensor lives at
 *   ptr[b*bstride + ch*cstride + (t*tstride)*V + ((v + rsign*ch) mod V)]
 * rsign = +1 is Shift_gcn's shift_in gather x[:, (v+c) mod V] (shift_gcn.py:108-112,127);
 * as an OUTPUT mapping rsign = +1 stores y[d, t, v] at ((v+d) mod V), which is the
 * shift_out gather z[v] = y[(v-d) mod V] (shift_gcn.py:114-118,136). tstride = 2 is the
 * strided residual conv (shift_gcn.py:35-36). */

/* Y[b][m][out(n,m)] (+)= act( sum_k A[m][k] * X'(b,k,n) + bias[m] ),  n < T*V
 * A = w: w_mcontig ? w[k*M + m] : w[m*K + k];  X'(b,k,n) = X(b,k,n) * (mask ? mask[v*K+k] : 1)
 * relu != 0 applies ReLU; accumulate != 0 adds into Y. K <= 256.
 * Forward of Shift_gcn (einsum + Linear_bias, shift_gcn.py:131-132, w = Linear_weight
 *   (C_in, C_out) m-contiguous, mask = tanh(Feature_Mask)+1), of Shift_tcn.temporal_linear
 *   (:62,69) and the down/residual convs (:84, :35); with w transposed it is their dX. */
int sgcn_pw_fwd(const float* w, int w_mcontig, const float* bias, const float* x,
                long long x_bstride, long long x_cstride, int x_tstride, int x_rsign,
                const float* mask, float* y, long long y_bstride, long long y_cstride,
                int y_tstride, int y_rsign, int relu, int accumulate, int B, int M, int K,
                int T, int V, void* stream);

/* Shift_tcn's shift_in fused into its temporal_linear (shift_gcn.py:66-70):
 *   Y[b][m][n] = act( sum_k w[m*K + k] * S_k(b, n) + bias[m] ),
 *   S_k = shift_k(in_scale[k] * X[b][k] + in_shift[k])   (stride-1 temporal shift,
 *   xpos/ypos per channel, shift_cuda_kernel.cu:11-76; in_scale/in_shift = Shift_tcn.bn's
 *   apply coefficients, both NULL = identity).
 * The shifted operand is formed from four taps of X while the contraction stages its
 * tiles (same arithmetic as sgcn_tshift_fwd, so Y is bit-identical to sgcn_tshift_fwd +
 * sgcn_pw_fwd); it is never read back from memory. x_shifted (optional, layout of x):
 * also store S there from the same registers (the weight gradient's operand, for
 * sgcn_pw_dw; NULL = not written). w is (M, K) k-contiguous (Conv2d
 * weight); relu != 0 applies ReLU. Workspace: sgcn_pw_tshift_ws_bytes(K) (the per-channel
 * shift table + one flag word). two_row (ABI 23): 0 = four taps per element; 1 = when
 * EVERY channel's xpos lies in (-2^-25, 0], two taps of the element's own column, rows
 * floor(y) and floor(y)+1 (there the .cu:73 blend reduces to q21*(1-dy) + q22*dy exactly:
 * bit-identical still); 2 = also when channels have 0 < xpos < 2^-25 (1 - dx rounds to 1;
 * the dropped dx terms weigh < 2^-25: within 3e-8 * max|tap| of sgcn_tshift_fwd). A launch
 * with any other channel uses four taps for all (decided on the device, per launch). */
size_t sgcn_pw_tshift_ws_bytes(int K);
int sgcn_pw_fwd_tshift(const float* w, const float* bias, const float* x, long long x_bstride,
                       long long x_cstride, const float* xpos, const float* ypos,
                       const float* in_scale, const float* in_shift, float* x_shifted,
                       void* ws, size_t ws_bytes, float* y, long long y_bstride,
                       long long y_cstride, int relu, int two_row, int B, int M, int K, int T,
                       int V, void* stream);

/* Workspace bytes for sgcn_pw_dw. */
size_t sgcn_pw_dw_ws_bytes(int B, int M, int Nc, int T, int V);

/* Weight gradient over every position: dW[m][c] (+)= sum_{b,n} G(b,m,n) * X'(b,c,n)
 * (stored [c][m] when dw_transpose, e.g. Linear_weight's (C_in, C_out) layout) and
 * dbias[m] (+)= sum_{b,n} G(b,m,n) (dbias may be NULL). Deterministic split-K. */
int sgcn_pw_dw(const float* g, long long g_bstride, long long g_cstride, int g_tstride,
               int g_rsign, const float* x, long long x_bstride, long long x_cstride,
               int x_tstride, int x_rsign, const float* mask, float* dw, int dw_transpose,
               int dw_accumulate, float* dbias, int dbias_accumulate, void* ws,
               size_t ws_bytes, int B, int M, int Nc, int T, int V, void* stream);

/* ------------------------------------------------------------------------------------
 * Training-mode BatchNorm (shift_gcn.py:38,55-56,85,99,137) and unit tails
 * ------------------------------------------------------------------------------------
 * per_joint = 3: Shift_gcn.bn, BatchNorm1d(V*C) over (n, t) (feature f = c*V + v here,
 * reference feature index v*C + c: pass perm_V = V to the finalizes), on the Shift_gcn
 * contraction output Z stored BEFORE its shift_out (sgcn_pw_fwd with y_rsign = 0):
 * element (c, t, v) of Z is the logical element (c, t, (v + c) mod V)
 * (shift_gcn.py:114-118,136), so the rotation is applied by these kernels' addressing
 * instead of by the contraction's stores (sgcn_moments, sgcn_bn_apply: statistics /
 * outputs / residual / coefficients at the logical position; sgcn_bn_bwd_reduce,
 * sgcn_bn_bwd_apply: Z read at the pre-rotation position, and the latter stores dZ there,
 * so the dW / dX contractions read it as a plain plane);
 * per_joint = 0: BatchNorm2d, feature = channel. Other values: SGCN_EINVAL. */

/* Bytes of the per-(b, feature) partials written by sgcn_moments / sgcn_bn_bwd_reduce. */
size_t sgcn_moments_ws_bytes(int B, int C, int V, int per_joint);

/* part[b][f] = {mean, M2} of x over the plane (or over t per joint). */
int sgcn_moments(const float* x, float* part, int B, int C, int T, int V, int per_joint,
                 void* stream);

/* Merge B partials (n_part elements each) per feature: batch mean / biased var ->
 * mean, invstd, scale = gamma*invstd, shift = beta - mean*scale (all [F], local feature
 * order); updates running_mean/var (momentum, unbiased var) and num_batches (+1) when
 * non-NULL, in the reference feature order (perm_V > 0: per-joint mapping). */

int sgcn_bn_finalize(const float* part, int B, int F, int n_part, int perm_V,
                     const float* gamma, const float* beta, float eps, float momentum,
                     float* running_mean, float* running_var, long long* num_batches,
                     float* mean, float* invstd, float* scale, float* shift, void* stream);

/* Eval-mode coefficients from running statistics: scale/shift (and, when non-NULL, the
 * running mean and 1/sqrt(running_var + eps) used by an eval-mode backward). */
int sgcn_bn_eval_coef(int F, int perm_V, const float* gamma, const float* beta,
                      const float* running_mean, const float* running_var, float eps,
                      float* mean, float* invstd, float* scale, float* shift, void* stream);

/* y = act(x*scale[f] + shift[f] + res), res = r*rscale[c] + rshift[c] (both given),
 * r (rscale NULL) or 0 (r NULL); act = ReLU if relu. y_stats (optional, B*C float2):
 * per-plane {mean, M2} of y, i.e. the sgcn_moments() partials of the NEXT BatchNorm2d's
 * input, produced without another read of y. gather_m + y_gathered (optional, both or
 * neither, exclusive with y_stats): also write y_gathered = sgcn_gcn_gather(y, gather_m),
 * the next unit's Shift_gcn input gathered and masked, from the same registers. */
int sgcn_bn_apply(const float* x, const float* scale, const float* shift, int per_joint,
                  const float* r, const float* rscale, const float* rshift, int relu,
                  float* y, float* y_stats, const float* gather_m, float* y_gathered, int B,
                  int C, int T, int V, void* stream);
/* Backward partials: g = dy * (relu ? y > 0 : 1); part[b][f] = {sum g, sum g*xhat};
 * rpart[b][c] likewise for a BatchNorm2d residual input r (NULL = none).
 * dy_coef (optional, [3][C], requires relu): dy is replaced by k1[c]*dy + k2[c]*y + k3[c],
 * i.e. the input gradient of the following BatchNorm2d (whose input is y), computed on the
 * fly instead of materialised (Shift_tcn.bn's dx feeding Shift_gcn's ReLU/BN backward). */
int sgcn_bn_bwd_reduce(const float* dy, const float* y, int relu, const float* x,
                       const float* mean, const float* invstd, int per_joint, const float* r,
                       const float* rmean, const float* rinvstd, const float* dy_coef,
                       float* part, float* rpart, int B, int C, int T, int V, void* stream);

/* dgamma/dbeta (+)= sums (reference feature order); coef[3][F] = {k1, k2, k3} such that
 * dx = k1*g + k2*x + k3: the training-mode BatchNorm input gradient (batch_stats = 1), or
 * the eval-mode one (batch_stats = 0: k2 = k3 = 0, mean/invstd = running statistics). */
int sgcn_bn_bwd_finalize(const float* part, int B, int F, long long n_total, int perm_V,
                         const float* mean, const float* invstd, const float* gamma,
                         float* dgamma, float* dbeta, int accumulate, int batch_stats,
                         float* coef, void* stream);

/* sgcn_bn_bwd_finalize for the per-joint BatchNorm1d (F = C*V features, perm_V = V) from
 * the six k-free sums of sgcn_tshift_bwd_gbn: g = k1*gin + k2*(in - mu) + (k3 + k2*mu)
 * with dy_coef = [3][C] {k1,k2,k3} (the following BatchNorm's sgcn_bn_bwd_finalize
 * coefficients) and dy_mean = [C] its mean mu (any centring value is exact; the batch
 * mean avoids cancellation); then dgamma/dbeta/coef exactly as sgcn_bn_bwd_finalize. */
int sgcn_bn_bwd_finalize_gbn(const float* part6, int B, int C, int V, long long n_total,
                             const float* dy_coef, const float* dy_mean, const float* mean,
                             const float* invstd, const float* gamma, float* dgamma,
                             float* dbeta, int accumulate, int batch_stats, float* coef,
                             void* stream);

/* dx = k1*g + k2*x + k3; dr = g (rcoef NULL, dr given) or rk1*g + rk2*r + rk3;
 * dy_coef as in sgcn_bn_bwd_reduce; per_joint 0 or 3 (see above). */
int sgcn_bn_bwd_apply(const float* dy, const float* y, int relu, const float* x,
                      const float* coef, int per_joint, const float* r, const float* rcoef,
                      const float* dy_coef, float* dx, float* dr, int B, int C, int T, int V,
                      void* stream);

/* m = tanh(Feature_Mask) + 1 (shift_gcn.py:129); n = V*C. */
int sgcn_mask_prep(const float* mask, float* m, int n, void* stream);

/* xg[b,c,t,u] = x0[b,c,t,(u + c) mod V] * m[u*C + c]: Shift_gcn's shift_in gather and
 * feature mask (shift_gcn.py:125-129; m = tanh(Feature_Mask) + 1 from sgcn_mask_prep),
 * materialised once per forward for the contraction and its weight gradient. */
int sgcn_gcn_gather(const float* x0, const float* m, float* xg, int B, int C, int T, int V,
                    void* stream);

/* Shift_gcn input side of the backward: dx[b,c,t,v] = dxt[b,c,t,u]*m[u][c] + add1 + add2
 * with u = (v - c) mod V (transpose of the shift_in gather); dmask_part[b][c][u] =
 * sum_t dxt * x0 at the gathered position. add1/add2 may be NULL.
 * prev_part (optional, B*C float2, with prev_s/prev_mean/prev_invstd): when x0 is the
 * output relu(bn2(prev_s) + residual) of the previous TCN_GCN_unit and dx is its complete
 * gradient, also write that bn2's sgcn_bn_bwd_reduce partials {sum g, sum g*xhat},
 * g = dx*(x0 > 0), xhat = (prev_s - prev_mean[c])*prev_invstd[c] — so the previous
 * unit's backward skips its reduce pass. add2_mask (optional, needs add1 and add2): add2
 * enters as add2 * (add2_mask > 0) (a unit's identity-residual gradient dout*(out > 0),
 * formed here rather than written by the unit tail's BatchNorm backward). */
int sgcn_gcn_dx_finish(const float* dxt, const float* x0, const float* m, const float* add1,
                       const float* add2, const float* add2_mask, float* dx, float* dmask_part,
                       const float* prev_s, const float* prev_mean, const float* prev_invstd,
                       float* prev_part, int B, int C, int T, int V, void* stream);

/* dmask[u][c] (+)= (sum_b dmask_part[b][c][u]) * (1 - tanh(mask[u][c])^2). */
int sgcn_mask_grad_finalize(const float* part, const float* mask, int B, int C, int V,
                            float* dmask, int accumulate, void* stream);

/* ------------------------------------------------------------------------------------
 * Ensemble head (config 4: 4-stream joint/bone/joint-motion/bone-motion inference)
 * ---------------------------------------------------------------------------------- */
/* Replaces `derive_modalities(joint_window)` (inference_pipeline.py:284-309) for a whole
 * batch, fused with Model.forward's head (shift_gcn.py:194-198) when scale/shift given.
 * joint : (N, C, T, V, M) clip batch;  parent: (V) int32 parent joint of each joint
 *   (BONE_PAIRS, inference_pipeline.py:16-22; joint 0 is its own parent -> bone 0).
 * out_* : any subset may be NULL.  bone = joint[v] - joint[parent[v]];
 *   *_motion[t] = x[t+1] - x[t] for t < T-1, 0 at t = T-1 (bone_motion = bone[t+1] -
 *   bone[t] evaluated in that order, so the fp32 results are bit-exact).
 * planes = 0: outputs in the input's (N, C, T, V, M) layout (scale/shift must be NULL);
 * planes = 1: outputs in the model's (N*M, C, T, V) plane layout, and when scale/shift
 *   ([4][M*V*C], data_bn eval coefficients of the four models, feature m*V*C + v*C + c)
 *   are given, data_bn is applied too, so the result feeds l1 directly. */
int sgcn_modalities(const float* joint, const int* parent, float* out_joint, float* out_bone,
                    float* out_joint_motion, float* out_bone_motion, const float* scale,
                    const float* shift, int planes, int N, int C, int T, int V, int M,
                    void* stream);

/* ------------------------------------------------------------------------------------
 * Model head / tail of the training step (shift_gcn.py:193-216)
 * ------------------------------------------------------------------------------------
 * Model.forward's input side is x.permute(0,4,3,1,2).view(N, M*V*C, T) -> data_bn =
 * BatchNorm1d(M*V*C) -> permute back to planes (N*M, C, T, V) (:194-198); features here
 * are in the reference order f = m*V*C + v*C + c (pass perm_V = 0 to the finalizes).
 * x is the (N, C, T, V, M) clip. */

/* Bytes of the [N][M*V*C] float2 partials of sgcn_head_moments / sgcn_head_bwd_reduce. */
size_t sgcn_head_ws_bytes(int N, int C, int V, int M);

/* part[n][f] = {mean, M2} of x over t (data_bn training statistics; merge with
 * sgcn_bn_finalize(part, N, M*V*C, T, 0, ...)). */
int sgcn_head_moments(const float* x, float* part, int N, int C, int T, int V, int M,
                      void* stream);

/* y[(n*M + m), c, t, v] = x[n, c, t, v, m] * scale[f] + shift[f]: the permute and data_bn
 * apply in one pass (scale/shift from sgcn_bn_finalize or sgcn_bn_eval_coef). */
int sgcn_head_apply(const float* x, const float* scale, const float* shift, float* y, int N,
                    int C, int T, int V, int M, void* stream);

/* part[n][f] = {sum_t g, sum_t g*(x - mean[f])*invstd[f]}, g = the plane-layout gradient of
 * y (feed sgcn_bn_bwd_finalize(part, N, M*V*C, N*T, 0, ...) for dgamma/dbeta/coef). */
int sgcn_head_bwd_reduce(const float* g, const float* x, const float* mean, const float* invstd,
                         float* part, int N, int C, int T, int V, int M, void* stream);

/* dx[n, c, t, v, m] = k1[f]*g + k2[f]*x + k3[f], coef = [3][M*V*C] from
 * sgcn_bn_bwd_finalize (only needed when the clip itself requires a gradient). */
int sgcn_head_bwd_apply(const float* g, const float* x, const float* coef, float* dx, int N,
                        int C, int T, int V, int M, void* stream);

/* out[n][c] = x.view(N, M, C, P).mean(3).mean(1) (shift_gcn.py:211-214), x the last unit's
 * (N*M, C, T', V) output, P = T'*V. */
int sgcn_pool(const float* x, float* out, int N, int M, int C, long long P, void* stream);

/* dx[n*M + m][c][p] = (dout[n][c] * (1/M)) * (1/P) (fp32 reciprocals): the pooling's
 * backward, rounded exactly as autograd's mean backward on the device. dx must be
 * 16-byte aligned. */
int sgcn_pool_bwd(const float* dout, float* dx, int N, int M, int C, long long P,
                  void* stream);

/* ------------------------------------------------------------------------------------
 * Optimizer (main.py:301-322, 414: torch.optim.SGD, dampening 0, not maximize)
 * ------------------------------------------------------------------------------------ */

/* Elements per chunk of the sgcn_sgd_step chunk map. */
int sgcn_sgd_chunk_elems(void);

/* One SGD step of every parameter tensor in ONE launch. `table` (device) holds per tensor
 * five int64 {param, grad, momentum buffer (fp32 device pointers), (float weight_decay bits)
 * | (float lr bits) << 32, flags (bit 0: the momentum buffer is new: initialised to the
 * step's d_p, torch's clone; bit 1: scale the gradient by the float whose bits are flags
 * bits 32-63 and store the scaled gradient back, i.e. GradAllReduce's deferred
 * `grad *= 1/world`; bit 2 (ABI 23): the fourth column is instead the device address of a
 * float pair {weight_decay, lr}, read by the kernel, so a graph-captured step follows
 * learning-rate changes made between replays)}; `numel` (device int32) per tensor; `chunks`
 * (device int32)
 * {tensor, first element} per chunk of at most sgcn_sgd_chunk_elems() elements. Per
 * element, torch's order: g = g*s (bit 1); d = g + wd*p (wd != 0); b = first ? d :
 * momentum*b + d (momentum != 0); d = nesterov ? d + momentum*b : b; p = p - lr*d. */
int sgcn_sgd_step(const void* table, const int* numel, const int* chunks, int n_chunks,
                  float momentum, int nesterov, void* stream);

/* Batched small launches (round 4): up to SGCN_BATCH_MAX independent instances of one
 * finalize in ONE launch; the entries travel as the kernel's arguments (no table copy).
 *   sgcn_tshift_pos_finalize_many: partials[i], gx[i], gy[i], B[i], C[i] (as
 *     sgcn_tshift_pos_finalize);
 *   sgcn_mask_prep_many: mask[i], m[i], n[i] (as sgcn_mask_prep);
 *   sgcn_mask_grad_finalize_many: part[i], mask[i], dmask[i], B[i], C[i], V[i] (as
 *     sgcn_mask_grad_finalize, accumulate 0).
 * All arrays are HOST arrays of n <= SGCN_BATCH_MAX entries. */
#define SGCN_BATCH_MAX 32
int sgcn_tshift_pos_finalize_many(const void* const* partials, float* const* gx,
                                  float* const* gy, const int* B, const int* C, int n,
                                  void* stream);
int sgcn_mask_prep_many(const float* const* mask, float* const* m, const int* count, int n,
                        void* stream);
int sgcn_mask_grad_finalize_many(const float* const* part, const float* const* mask,
                                 float* const* dmask, const int* B, const int* C,
                                 const int* V, int n, void* stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* SHIFTGCN_H_ */
