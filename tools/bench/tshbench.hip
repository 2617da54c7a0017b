// Temporal shift fused into the contraction operand vs the two-launch form, through the
// public C ABI (tuning harness; not part of the product library):
//   A: sgcn_tshift_fwd(H, bn affine) -> As; sgcn_pw_fwd(As) -> R      (round-1 path)
//   B: sgcn_pw_fwd_tshift(H) -> R, two_row 0/1/2 (round 6), with and without the stored
//      operand; R and the stored operand compared with A's bit for bit (per channel)
// on the Shift_tcn shapes of the NTU model.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/tshbench.hip \
//         -Lshift-gcn_amd/shiftgcn -lshiftgcn_hip -Wl,-rpath,'$ORIGIN/../../shift-gcn_amd/shiftgcn' \
//         -o tools/bench/tshbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/shiftgcn.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
#define CR(x) do { int r = (x); if (r != 0) { printf("ABI error %d at %d\n", r, __LINE__); exit(1); } } while (0)

struct Shape { const char* name; int B, C, M, T, V; };

template <typename F>
float timeit(F&& f, hipStream_t st, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / reps;
}

int main() {
  Shape shapes[] = {
    {"l2 tcn 64->64 T300", 128, 64, 64, 300, 25},
    {"l5 tcn 128->128 T300", 128, 128, 128, 300, 25},
    {"l6 tcn 128->128 T150", 128, 128, 128, 150, 25},
    {"l8 tcn 256->256 T150", 128, 256, 256, 150, 25},
    {"l9 tcn 256->256 T75", 128, 256, 256, 75, 25},
    {"mp l2 tcn 64 T300 V33", 64, 64, 64, 300, 33},
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t maxe = (size_t)128 * 256 * 150 * 25;
  float *h, *as, *as2, *r1, *r2, *w, *bias, *xp, *yp, *sc, *sh;
  void* ws;
  CK(hipMalloc(&h, maxe * 4)); CK(hipMalloc(&as, maxe * 4)); CK(hipMalloc(&as2, maxe * 4));
  CK(hipMalloc(&r1, maxe * 4)); CK(hipMalloc(&r2, maxe * 4));
  CK(hipMalloc(&w, 256 * 256 * 4)); CK(hipMalloc(&bias, 256 * 4));
  CK(hipMalloc(&xp, 256 * 4)); CK(hipMalloc(&yp, 256 * 4));
  CK(hipMalloc(&sc, 256 * 4)); CK(hipMalloc(&sh, 256 * 4));
  CK(hipMalloc(&ws, 1 << 20));
  std::vector<float> v(maxe);
  for (size_t i = 0; i < maxe; ++i) v[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(h, v.data(), maxe * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, v.data() + 3, 256 * 256 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, v.data() + 9, 256 * 4, hipMemcpyHostToDevice));
  std::vector<float> px(256), py(256), ps(256), pb(256);
  for (int c = 0; c < 256; ++c) {
    // U(-1e-8, 1e-8)-like (shift.py:39)
    px[c] = (c % 3 == 0 ? 1e-8f : -1e-8f) * (c % 7) / 7.f;
    py[c] = ((c * 37) % 200) / 100.f - 1.f;    // U(-1,1)-like, Shift_tcn init_scale = 1
    ps[c] = 1.f + (c % 5) * 0.1f;
    pb[c] = (c % 11) * 0.01f - 0.05f;
  }
  CK(hipMemcpy(xp, px.data(), 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(yp, py.data(), 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(sc, ps.data(), 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(sh, pb.data(), 1024, hipMemcpyHostToDevice));
  for (auto& s : shapes) {
    const long long N = (long long)s.T * s.V;
    const size_t n = (size_t)s.B * s.M * N, nin = (size_t)s.B * s.C * N;
    auto A = [&]() {
      CR(sgcn_tshift_fwd(h, as, xp, yp, sc, sh, nullptr, s.B, s.C, s.T, s.V, 1, 1, st));
      CR(sgcn_pw_fwd(w, 0, bias, as, s.C * N, N, 1, 0, nullptr, r1, s.M * N, N, 1, 0, 1, 0,
                     s.B, s.M, s.C, s.T, s.V, st));
    };
    const float ta = timeit(A, st, 10);
    const float tsh = timeit([&]() {
      CR(sgcn_tshift_fwd(h, as, xp, yp, sc, sh, nullptr, s.B, s.C, s.T, s.V, 1, 1, st));
    }, st, 10);
    std::vector<float> h1(n), h2(n), a1(nin), a2(nin);
    CK(hipMemcpy(h1.data(), r1, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(a1.data(), as, nin * 4, hipMemcpyDeviceToHost));
    printf("%-24s two-launch %7.1f us (shift %6.1f + pw %6.1f)\n", s.name, ta, tsh, ta - tsh);
    for (int mode = 0; mode <= 2; ++mode) {
      const float tb = timeit([&]() {
        CR(sgcn_pw_fwd_tshift(w, bias, h, s.C * N, N, xp, yp, sc, sh, nullptr, ws, 1 << 20, r2,
                              s.M * N, N, 1, mode, s.B, s.M, s.C, s.T, s.V, st));
      }, st, 10);
      const float tbs = timeit([&]() {   // fused + the shifted operand stored (into as2)
        CR(sgcn_pw_fwd_tshift(w, bias, h, s.C * N, N, xp, yp, sc, sh, as2, ws, 1 << 20, r2,
                              s.M * N, N, 1, mode, s.B, s.M, s.C, s.T, s.V, st));
      }, st, 10);
      CK(hipMemcpy(h2.data(), r2, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(a2.data(), as2, nin * 4, hipMemcpyDeviceToHost));
      // the stored operand per channel: bit-exact, or max |diff| relative to the channel's max
      int exact_ch = 0;
      double worst = 0;
      for (int c = 0; c < s.C; ++c) {
        bool ex = true;
        double md = 0, mx = 0;
        for (int b = 0; b < s.B; ++b)
          for (long long k = 0; k < N; ++k) {
            const size_t i = ((size_t)b * s.C + c) * N + k;
            if (memcmp(&a1[i], &a2[i], 4) != 0) ex = false;
            md = fmax(md, fabs((double)a1[i] - a2[i]));
            mx = fmax(mx, fabs((double)a1[i]));
          }
        exact_ch += ex;
        worst = fmax(worst, md / (mx > 0 ? mx : 1));
      }
      const bool rok = memcmp(h1.data(), h2.data(), n * 4) == 0;
      printf("   two_row %d: fused %7.1f us  fused+store %7.1f us  operand channels exact %d/%d "
             "(worst rel %.1e)  R %s\n", mode, tb, tbs, exact_ch, s.C, worst,
             rok ? "bit-exact" : "differs");
    }
  }
  return 0;
}
