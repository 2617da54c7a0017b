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
#define SGCN_ABI_VERSION 1

/* ABI version of the loaded library (== SGCN_ABI_VERSION). */
int sgcn_abi_version(void);

/* ------------------------------------------------------------------------------------
 * Temporal shift
 * ------------------------------------------------------------------------------------ */

/* Forward learnable fractional temporal shift.
 * Replaces `shift_cuda.forward(input, xpos, ypos, stride)`
 *   (model/Temporal_shift/cuda/shift_cuda.cpp:19-23 -> shift_cuda_kernel.cu:405-431).
 * in  : (B, C, H, W);  out: (B, C, H/stride, W);  xpos, ypos: (C) raw Shift parameters.
 * The +0.5 that ShiftFunction adds to ypos for stride != 1 (shift.py:17-18) is applied
 * INSIDE the kernel as the same float32 add, so callers pass the raw parameter.
 * in_scale/in_shift: optional per-channel affine (C) applied to every in-range input tap
 *   (a fused BatchNorm apply); both NULL = identity.
 * plane_stats: optional (B*C) float2 {mean, M2} of each output plane (n = H/stride*W),
 *   consumed by sgcn_bn_finalize(); NULL = not computed.
 * Unlike the reference (at::zeros + kernel), every output element is written exactly
 * once (no memset pass). */
int sgcn_tshift_fwd(const float* in, float* out, const float* xpos, const float* ypos,
                    const float* in_scale, const float* in_shift, float* plane_stats,
                    int B, int C, int H, int W, int stride, void* stream);

/* Workspace bytes for sgcn_tshift_bwd (B*C float2 plane partials). */
size_t sgcn_tshift_bwd_ws_bytes(int B, int C);

/* Backward of the temporal shift. Replaces
 * `shift_cuda.backward(grad_output, input, output, xpos, ypos, stride)`
 *   (shift_cuda.cpp:25-42 -> shift_cuda_kernel.cu:433-523).
 * gout: (B, C, H/stride, W); in: (B, C, H, W) forward input; xpos/ypos raw (see fwd).
 * gin : (B, C, H, W) input gradient (reference Shift_Bottom_Backward*, .cu:78-256);
 * gx, gy: (C) position gradients = mean over batch of the summed position products
 *   (.cu:277-363, 501-509) after applyShiftConstraint (.cu:370-395).
 * in_scale/in_shift: same optional affine as the forward (the position products then
 *   use the affine taps). relu_mask != 0: gin[p] = 0 where in[p] <= 0 (fused ReLU
 *   backward for a shift whose input is a ReLU output).
 * stride must be 1 or 2 (the reference backward hard-codes 2 for stride != 1). */
int sgcn_tshift_bwd(const float* gout, const float* in, const float* xpos, const float* ypos,
                    const float* in_scale, const float* in_shift, int relu_mask, float* gin,
                    float* gx, float* gy, void* ws, size_t ws_bytes, int B, int C, int H,
                    int W, int stride, void* stream);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* SHIFTGCN_H_ */
