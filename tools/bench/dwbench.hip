// Weight-gradient variants of the HBM-bound 64 x 64 contractions (NTU l2-l4, B = 128 planes,
// T = 300, V = 25; tuning harness, not part of the product library): the product
// pw_dw_kernel at its split count and at 2x / 4x the workgroups, and pw_dw3 tiles with
// other chunk lengths / workgroup targets. Every variant's dW is compared with the
// product's (different split counts sum in a different order: max relative difference).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/dwbench.hip -o tools/bench/dwbench
#include "../../shift-gcn_amd/csrc/pwconv.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace sgcn;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <typename F>
float timeit(F&& launch, hipStream_t st, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1000.f / reps;
}

static double reldiff(const float* a, const float* b, int n) {
  std::vector<float> h1(n), h2(n);
  CK(hipMemcpy(h1.data(), a, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2.data(), b, n * 4, hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  for (int i = 0; i < n; ++i) { md = fmax(md, fabs(h1[i] - h2[i])); mx = fmax(mx, fabs(h1[i])); }
  return md / mx;
}

struct Ctx { hipStream_t st; float* ws; float* dwref; float* dwout; double by; const char* name;
             double fl = 0; };

template <int BM, int BN, int WM, int WN, bool MASK, bool PLAIN>
void dw_s(const Ctx& c, DwArgs a, int S, const char* tag) {
  const int N = a.T * a.V;
  const int total = a.B * ((N + kDwBK - 1) / kDwBK);
  if (S > total) S = total;
  a.chunks_per_split = (total + S - 1) / S;
  a.slab = c.ws;
  a.bslab = nullptr;
  dim3 grid(1, S);
  const size_t dyn = MASK ? (size_t)a.V * BN * 4 : 0;
  auto L = [&]() {
    pw_dw_kernel<BM, BN, WM, WN, MASK, PLAIN><<<grid, 64 * WM * WN, dyn, c.st>>>(a);
    launch_slab_reduce(a.slab, nullptr, S, a.M, a.Nc, c.dwout, 0, 0, nullptr, 0, c.st);
  };
  const float us = timeit(L, c.st, 20);
  auto K = [&]() { pw_dw_kernel<BM, BN, WM, WN, MASK, PLAIN><<<grid, 64 * WM * WN, dyn, c.st>>>(a); };
  const float uk = timeit(K, c.st, 20);
  printf("%-18s %-22s S=%5d %7.1f us (kernel %7.1f) %5.2f TB/s  diff %.1e\n", c.name, tag, S,
         us, uk, c.by / uk / 1e6, c.dwref ? reldiff(c.dwref, c.dwout, a.M * a.Nc) : 0.0);
}

template <int BKP, bool MASK, bool ROT, int BM = 64, int BN = 64, int WM = 2, int WN = 2>
void dw3_t(const Ctx& c, DwArgs a, int target, const char* tag) {
  const int P = a.B * a.T * a.V;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.Nc + BN - 1) / BN);
  const int S = dw3_splits(a.M, a.Nc, P, BKP, tiles, target);
  const int nch = (P + BKP - 1) / BKP;
  a.chunks_per_split = (nch + S - 1) / S;
  a.slab = c.ws;
  a.bslab = nullptr;
  dim3 grid(tiles, S);
  auto K = [&]() {
    pw_dw3_kernel<BM, BN, WM, WN, BKP, MASK, ROT, ROT, false><<<grid, 64 * WM * WN, 0, c.st>>>(a);
  };
  auto L = [&]() {
    K();
    launch_slab_reduce(a.slab, nullptr, S, a.M, a.Nc, c.dwout, 0, 0, nullptr, 0, c.st);
  };
  const float us = timeit(L, c.st, 20);
  const float uk = timeit(K, c.st, 20);
  printf("%-18s %-22s S=%5d %7.1f us (kernel %7.1f) %5.2f TB/s %.3f of 157.3 TF  diff %.1e\n",
         c.name, tag, S, us, uk, c.by / uk / 1e6, c.fl / uk / 1e6 / 157.3,
         reldiff(c.dwref, c.dwout, a.M * a.Nc));
}

// the 128 x 128 weight gradients (l6 / l7 at T = 150, l5's temporal_linear at T = 300)
void big(hipStream_t st, float* x, float* y, float* mask, float* ws, float* dw1, float* dw2) {
  const int B = 128, M = 128, K = 128, V = 25;
  for (int T : {150, 300}) {
    for (int msk = 0; msk < (T == 150 ? 2 : 1); ++msk) {
      const int N = T * V;
      DwArgs d{};
      d.g = {y, (long long)M * N, N, 1, msk ? 1 : 0};
      d.x = {x, (long long)K * N, N, 1, msk ? 1 : 0};
      d.mask = msk ? mask : nullptr;
      d.M = M; d.Nc = K; d.T = T; d.V = V; d.B = B;
      d.g_bytes = plane_bytes(d.g.bstride, d.g.cstride, 1, B, M, T, V);
      d.x_bytes = plane_bytes(d.x.bstride, d.x.cstride, 1, B, K, T, V);
      d.mask_bytes = msk ? (unsigned)(V * K * 4) : 0u;
      const double by = 4.0 * B * N * (M + K), fl = 2.0 * B * N * M * K;
      char name[32];
      snprintf(name, sizeof name, "128x128 T%d%s", T, msk ? " m+r" : "");
      Ctx c{st, ws, nullptr, dw1, by, name, fl};
      // product: 128 x 128, 2 x 2 waves, BKP 16, 1024 workgroups (reference for the diffs)
      {
        DwArgs a = d;
        const int S = launch_dw3(a, st, ws, false);
        auto L = [&]() { launch_dw3(a, st, ws, false); };
        const float uk = timeit(L, st, 20);
        launch_slab_reduce(ws, nullptr, S, M, K, dw1, 0, 0, nullptr, 0, st);
        CK(hipStreamSynchronize(st));
        printf("%-18s %-22s S=%5d kernel %7.1f us  %5.1f TF/s (%.3f of 157.3)\n", name,
               "product dw3", S, uk, fl / uk / 1e6, fl / uk / 1e6 / 157.3);
      }
      c.dwref = dw1;
      c.dwout = dw2;
#define V3(BKP_, BM_, BN_, WM_, WN_, TG)                                                         \
      do {                                                                                      \
        char tag[64];                                                                           \
        snprintf(tag, sizeof tag, "%dx%d w%dx%d b%d t%d", BM_, BN_, WM_, WN_, BKP_, TG);         \
        if (msk) dw3_t<BKP_, true, true, BM_, BN_, WM_, WN_>(c, d, TG, tag);                    \
        else dw3_t<BKP_, false, false, BM_, BN_, WM_, WN_>(c, d, TG, tag);                      \
      } while (0)
      V3(16, 128, 128, 2, 2, 1024);
      V3(16, 128, 128, 2, 2, 2048);
      V3(32, 128, 128, 2, 2, 1024);
      V3(16, 128, 128, 1, 2, 1024);
      V3(16, 128, 128, 2, 1, 1024);
      V3(16, 128, 128, 1, 2, 2048);
      V3(16, 128, 128, 2, 1, 2048);
      V3(32, 128, 128, 2, 1, 2048);
      V3(16, 128, 128, 4, 2, 1024);
      V3(16, 128, 64, 2, 1, 2048);
#undef V3
    }
  }
}

// the 256-row weight gradients (l9 / l10 at T = 75: 256 x 256; l8's gcn at T = 150: 256 x 128):
// the split count sets the slab traffic (S x M x Nc floats written, then read by the reduce)
void huge(hipStream_t st, float* x, float* y, float* ws, float* dw1, float* dw2) {
  const int B = 128, V = 25;
  struct S3 { int M, K, T; };
  for (S3 sh : {S3{256, 256, 75}, S3{256, 128, 150}}) {
    const int M = sh.M, K = sh.K, T = sh.T, N = T * V;
    DwArgs d{};
    d.g = {y, (long long)M * N, N, 1, 0};
    d.x = {x, (long long)K * N, N, 1, 0};
    d.M = M; d.Nc = K; d.T = T; d.V = V; d.B = B;
    d.g_bytes = plane_bytes(d.g.bstride, d.g.cstride, 1, B, M, T, V);
    d.x_bytes = plane_bytes(d.x.bstride, d.x.cstride, 1, B, K, T, V);
    const double by = 4.0 * B * N * (M + K), fl = 2.0 * B * N * M * K;
    char name[32];
    snprintf(name, sizeof name, "%dx%d T%d", M, K, T);
    Ctx c{st, ws, nullptr, dw1, by, name, fl};
    {
      DwArgs a = d;
      const int S = launch_dw3(a, st, ws, false);
      auto L = [&]() {
        launch_dw3(a, st, ws, false);
        launch_slab_reduce(ws, nullptr, S, M, K, dw1, 0, 0, nullptr, 0, st);
      };
      for (int r = 0; r < 2; ++r) {
        const float u = timeit(L, st, 20);
        printf("%-18s %-22s S=%5d %7.1f us (with reduce) %.3f of 157.3 TF\n", name, "product",
               S, u, fl / u / 1e6 / 157.3);
      }
    }
    c.dwref = dw1;
    c.dwout = dw2;
    for (int tg : {256, 384, 512, 768, 1024}) {
      char tag[64];
      snprintf(tag, sizeof tag, "target %d", tg);
      if (K == 256) dw3_t<16, false, false, 256, 256, 4, 2>(c, d, tg, tag);
      else dw3_t<16, false, false, 256, 128, 4, 2>(c, d, tg, tag);
    }
  }
}

int main(int argc, char** argv) {
  const int B = 128, M = 64, K = 64, T = 300, V = 25;
  const int N = T * V;
  const size_t ne = (size_t)B * 128 * N;   // the 128-channel T = 300 planes (big())
  hipStream_t st; CK(hipStreamCreate(&st));
  float *x, *y, *mask, *ws, *dw1, *dw2;
  CK(hipMalloc(&x, ne * 4)); CK(hipMalloc(&y, ne * 4)); CK(hipMalloc(&mask, V * K * 4));
  CK(hipMalloc(&ws, 256 << 20)); CK(hipMalloc(&dw1, 256 * 256 * 4)); CK(hipMalloc(&dw2, 256 * 256 * 4));
  std::vector<float> h(ne);
  for (size_t i = 0; i < ne; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(x, h.data(), ne * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(y, h.data() + 7, (ne - 7) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(mask, h.data(), V * K * 4, hipMemcpyHostToDevice));
  const double by = 4.0 * B * N * (M + K);
  if (argc > 1 && argv[1][0] == 'h') {
    huge(st, x, y, ws, dw1, dw2);
    printf("done\n");
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'b') {
    big(st, x, y, mask, ws, dw1, dw2);
    printf("done\n");
    return 0;
  }
  for (int shape = 0; shape < 2; ++shape) {
    const bool msk = shape == 1;
    DwArgs d{};
    d.g = {y, (long long)M * N, N, 1, msk ? 1 : 0};
    d.x = {x, (long long)K * N, N, 1, msk ? 1 : 0};
    d.mask = msk ? mask : nullptr;
    d.M = M; d.Nc = K; d.T = T; d.V = V; d.B = B;
    d.g_bytes = plane_bytes(d.g.bstride, d.g.cstride, 1, B, M, T, V);
    d.x_bytes = plane_bytes(d.x.bstride, d.x.cstride, 1, B, K, T, V);
    d.mask_bytes = msk ? (unsigned)(V * K * 4) : 0u;
    const int S0 = dw_splits(M, K, B, N, 1);
    Ctx c{st, ws, nullptr, dw1, by, msk ? "l2 gcn mask+rot" : "l2 tcn plain", 2.0 * B * N * M * K};
    if (msk) dw_s<64, 64, 2, 2, true, false>(c, d, S0, "product pw_dw");
    else dw_s<64, 64, 2, 2, false, true>(c, d, S0, "product pw_dw");
    c.dwref = dw1;
    c.dwout = dw2;
    for (int f : {2, 4}) {
      char tag[64];
      snprintf(tag, sizeof tag, "pw_dw x%d WGs", f);
      if (msk) dw_s<64, 64, 2, 2, true, false>(c, d, S0 * f, tag);
      else dw_s<64, 64, 2, 2, false, true>(c, d, S0 * f, tag);
    }
    if (!msk) dw_s<64, 64, 2, 2, false, true>(c, d, S0, "product again");   // warm state
    for (int tg : {1024, 2048, 4096}) {
      char tag[64];
      snprintf(tag, sizeof tag, "dw3 bkp16 t%d", tg);
      if (msk) dw3_t<16, true, true>(c, d, tg, tag); else dw3_t<16, false, false>(c, d, tg, tag);
      snprintf(tag, sizeof tag, "dw3 bkp32 t%d", tg);
      if (msk) dw3_t<32, true, true>(c, d, tg, tag); else dw3_t<32, false, false>(c, d, tg, tag);
      snprintf(tag, sizeof tag, "dw3 bkp64 t%d", tg);
      if (msk) dw3_t<64, true, true>(c, d, tg, tag); else dw3_t<64, false, false>(c, d, tg, tag);
    }
  }
  printf("done\n");
  return 0;
}
