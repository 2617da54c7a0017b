// The reference training step's optimizer update (main.py:301-322, 414: torch.optim.SGD,
// momentum 0.9, nesterov, per-parameter weight decay; dampening 0) for every parameter
// tensor of the model in ONE launch.
//
// torch's multi-tensor SGD issues five foreach ops per parameter group (weight decay,
// momentum scale, momentum add, nesterov add, parameter update), each split into
// several launches: ~35 launches per step (≈0.35 ms on the critical path at NTU). Here one
// workgroup per chunk of one tensor does all five updates in registers: each element of
// the parameter, its gradient and its momentum buffer crosses HBM once.
//
// Per tensor t the caller passes (device table, rewritten every step because fresh
// gradient tensors are allocated every backward): {param, grad, momentum buffer, bits of
// (float weight_decay, float lr), flags (bit 0: the momentum buffer is new; bit 1: scale
// the gradient by the float in bits 32-63 first and store it back)} as int64, and a chunk
// map {tensor, first element} per workgroup. The scale is the data-parallel reduction's
// 1/world (shiftgcn/dist.py): the all-reduced SUM is scaled here instead of by a separate
// pass between the all-reduce and the update. Flags bit 2 (ABI 23): the (weight_decay, lr)
// column is instead the device address of that group's float pair, which the optimizer
// keeps current (shiftgcn/train.py FusedSGD): a step captured in a hipGraph then reads the
// learning rate of the replay, not the one of the capture (main.py:342-353 changes it per
// epoch).
#include "common.hpp"

namespace sgcn {
namespace {

constexpr int kSgdThreads = 256;
constexpr int kSgdChunk = 2048;   // elements per workgroup (8 per thread)

struct SgdEntry {
  long long p, g, buf, wdlr, flags;
};

__global__ __launch_bounds__(kSgdThreads) void sgd_step_kernel(
    const SgdEntry* __restrict__ table, const int* __restrict__ numel,
    const int* __restrict__ chunks, float momentum, int nesterov) {
  const int t = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const SgdEntry e = table[t];
  float* __restrict__ p = reinterpret_cast<float*>(e.p);
  // the gradient is read and (scaled) written back through one pointer: no __restrict__
  float* g = reinterpret_cast<float*>(e.g);
  float* __restrict__ buf = reinterpret_cast<float*>(e.buf);
  float wd, lr;
  if (e.flags & 4) {                                   // device-resident hyper-parameters
    const float* h = reinterpret_cast<const float*>(e.wdlr);
    wd = h[0];
    lr = h[1];
  } else {
    wd = __uint_as_float((unsigned)(e.wdlr & 0xffffffffLL));
    lr = __uint_as_float((unsigned)((unsigned long long)e.wdlr >> 32));
  }
  const bool first = (e.flags & 1) != 0;
  const bool scaled = (e.flags & 2) != 0;
  const float gs = __uint_as_float((unsigned)((unsigned long long)e.flags >> 32));
  const int end = min(numel[t], start + kSgdChunk);
  for (int i = start + (int)threadIdx.x; i < end; i += kSgdThreads) {
    const float pv = p[i];
    float d = g[i];
    if (scaled) {                                      // the reduction's grad *= 1/world
      d = d * gs;
      g[i] = d;
    }
    if (wd != 0.f) d = d + wd * pv;                    // grad + weight_decay * param
    float b;
    if (momentum != 0.f) {
      b = first ? d : buf[i] * momentum + d;           // clone on the first step
      buf[i] = b;
      d = nesterov ? d + momentum * b : b;
    }
    p[i] = pv - lr * d;                                // param - lr * d_p
  }
}

}  // namespace
}  // namespace sgcn

using namespace sgcn;

extern "C" {

int sgcn_sgd_chunk_elems(void) { return kSgdChunk; }

int sgcn_sgd_step(const void* table, const int* numel, const int* chunks, int n_chunks,
                  float momentum, int nesterov, void* stream) {
  SGCN_REQUIRE(n_chunks >= 0 && (n_chunks == 0 || (table && numel && chunks)));
  SGCN_REQUIRE(momentum >= 0.f);
  if (n_chunks == 0) return 0;
  sgd_step_kernel<<<n_chunks, kSgdThreads, 0, (hipStream_t)stream>>>(
      (const SgdEntry*)table, numel, chunks, momentum, nesterov != 0);
  SGCN_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
