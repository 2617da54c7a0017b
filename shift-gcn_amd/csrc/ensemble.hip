// Ensemble head: skeleton modality derivation fused with the model's input permute and
// (eval-mode) data_bn — one pass over the joint clip for all four streams.
//
// Reference: inference_pipeline.py:284-309 (derive_modalities: bone = joint - joint[parent]
// per BONE_PAIRS, joint/bone motion = frame differences with a zero last frame) and
// shift_gcn.py:194-198 (Model.forward head: permute (N,C,T,V,M) -> (N, M*V*C, T),
// BatchNorm1d(M*V*C), permute back to (N*M, C, T, V)).
//
// One thread per output element (n*M + m, c, t, v); consecutive threads walk v, so every
// store is coalesced and the four loads per element (frames t and t+1, joint v and its
// parent) hit the same few cache lines as the neighbouring threads' loads. The clip is
// small (NTU bs=64: 11.5 MB; ENS bs=256: 30 MB), the kernel is HBM/L2-bound and runs once
// per inference batch.
#include "common.hpp"

namespace sgcn {
namespace {

constexpr int kEnsThreads = 256;

template <bool PLANES, bool AFFINE>
__global__ void __launch_bounds__(kEnsThreads)
modalities_kernel(const float* __restrict__ joint, const int* __restrict__ parent,
                  float* __restrict__ o_joint, float* __restrict__ o_bone,
                  float* __restrict__ o_jm, float* __restrict__ o_bm,
                  const float* __restrict__ scale, const float* __restrict__ shift, int N,
                  int C, int T, int V, int M) {
  const long long total = (long long)N * M * C * T * V;
  const long long i = (long long)blockIdx.x * kEnsThreads + threadIdx.x;
  if (i >= total) return;
  // decode the OUTPUT index
  int n, m, c, t, v;
  if (PLANES) {  // (N*M, C, T, V)
    long long r = i;
    v = (int)(r % V); r /= V;
    t = (int)(r % T); r /= T;
    c = (int)(r % C); r /= C;
    m = (int)(r % M);
    n = (int)(r / M);
  } else {       // (N, C, T, V, M), the reference's on-disk / pipeline layout
    long long r = i;
    m = (int)(r % M); r /= M;
    v = (int)(r % V); r /= V;
    t = (int)(r % T); r /= T;
    c = (int)(r % C);
    n = (int)(r / C);
  }
  const int p = parent[v];
  const long long row = (((long long)n * C + c) * T) * V * M;   // (n, c, t=0, v=0, m=0)
  const long long at = row + ((long long)t * V) * M + m;
  const float jv = joint[at + (long long)v * M];
  const float jp = joint[at + (long long)p * M];
  // bone[t] = joint[t, v] - joint[t, parent]   (gen_bone_data / derive_modalities :293-294)
  const float bone = jv - jp;
  float jm = 0.f, bm = 0.f;
  if (t + 1 < T) {
    const long long at1 = at + (long long)V * M;
    const float jv1 = joint[at1 + (long long)v * M];
    const float jp1 = joint[at1 + (long long)p * M];
    jm = jv1 - jv;                       // joint_motion[t] = joint[t+1] - joint[t]  (:297-298)
    bm = (jv1 - jp1) - bone;             // bone_motion[t]  = bone[t+1]  - bone[t]   (:301-302)
  }
  float o0 = jv, o1 = bone, o2 = jm, o3 = bm;
  if (AFFINE) {
    // data_bn feature of element (n, c, t, v, m) is m*V*C + v*C + c (shift_gcn.py:195-196)
    const int F = M * V * C;
    const int f = (m * V + v) * C + c;
    o0 = o0 * scale[f] + shift[f];
    o1 = o1 * scale[F + f] + shift[F + f];
    o2 = o2 * scale[2 * F + f] + shift[2 * F + f];
    o3 = o3 * scale[3 * F + f] + shift[3 * F + f];
  }
  if (o_joint) o_joint[i] = o0;
  if (o_bone) o_bone[i] = o1;
  if (o_jm) o_jm[i] = o2;
  if (o_bm) o_bm[i] = o3;
}

}  // namespace
}  // namespace sgcn

using namespace sgcn;

extern "C" int sgcn_modalities(const float* joint, const int* parent, float* out_joint,
                               float* out_bone, float* out_joint_motion,
                               float* out_bone_motion, const float* scale,
                               const float* shift, int planes, int N, int C, int T, int V,
                               int M, void* stream) {
  SGCN_REQUIRE(N >= 0 && C > 0 && T > 0 && V > 0 && M > 0);
  SGCN_REQUIRE((scale == nullptr) == (shift == nullptr));
  SGCN_REQUIRE(!scale || planes);   // data_bn is applied in the model's plane layout
  const long long total = (long long)N * M * C * T * V;
  if (total == 0) return 0;         // empty batch: nothing to read (pointers may be NULL)
  SGCN_REQUIRE(joint && parent);
  SGCN_REQUIRE(total < (1ll << 40));
  const unsigned blocks = (unsigned)((total + kEnsThreads - 1) / kEnsThreads);
  hipStream_t st = (hipStream_t)stream;
#define SGCN_MOD(P, A)                                                                        \
  modalities_kernel<P, A><<<blocks, kEnsThreads, 0, st>>>(joint, parent, out_joint, out_bone, \
                                                          out_joint_motion, out_bone_motion,  \
                                                          scale, shift, N, C, T, V, M)
  if (planes) {
    if (scale) SGCN_MOD(true, true);
    else SGCN_MOD(true, false);
  } else {
    SGCN_MOD(false, false);
  }
#undef SGCN_MOD
  SGCN_LAUNCH_CHECK();
  return 0;
}
