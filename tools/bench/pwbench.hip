// Microbenchmark of the pointwise-contraction kernels on the unit shapes of the NTU
// model (tuning harness; not part of the product library). Includes the kernel source
// directly so template variants can be launched side by side; every variant's output is
// compared bit for bit with the product configuration's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/pwbench.hip -o tools/bench/pwbench
#include "../../shift-gcn_amd/csrc/pwconv.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace sgcn;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Shape { const char* name; int B, M, K, T, V; bool mask, rot; };

template <typename F>
float timeit(F&& launch, hipStream_t st, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 2; ++i) launch();
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1000.f / reps;
}

static std::vector<float> g_h1, g_h2;
bool same(const float* y, const float* y2, size_t n) {
  g_h1.resize(n); g_h2.resize(n);
  CK(hipMemcpy(g_h1.data(), y, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(g_h2.data(), y2, n * 4, hipMemcpyDeviceToHost));
  return memcmp(g_h1.data(), g_h2.data(), n * 4) == 0;
}

template <int BM, int BN, int WM, int WN>
void dw_variant(const char* name, const Shape& s, DwArgs a, int S, hipStream_t st, float* ws,
                float* dwref, float* dwout, double fl, double by) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.Nc + BN - 1) / BN);
  const int N = a.T * a.V;
  const int total = a.B * ((N + kDwBK - 1) / kDwBK);
  if (S > total) S = total;
  if ((size_t)S * a.M * a.Nc * 4 > ((size_t)256 << 20)) { printf("    S=%d: slab too large, skipped\n", S); return; }
  a.chunks_per_split = (total + S - 1) / S;
  a.slab = ws;
  a.bslab = nullptr;
  dim3 grid(tiles, S);
  const size_t dyn = s.mask ? (size_t)a.V * BN * 4 : 0;
  const int MN = a.M * a.Nc;
  auto L = [&]() {
    if (s.mask) pw_dw_kernel<BM, BN, WM, WN, true><<<grid, 64 * WM * WN, dyn, st>>>(a);
    else pw_dw_kernel<BM, BN, WM, WN, false><<<grid, 64 * WM * WN, 0, st>>>(a);
    launch_slab_reduce(a.slab, nullptr, S, a.M, a.Nc, dwout, 0, 0, nullptr, 0, st);
  };
  float us = timeit(L, st, 10);
  printf("%-20s %-26s S=%5d %8.1f us  %6.1f TF/s  %6.2f TB/s  %s\n", s.name, name, S, us,
         fl / us / 1e6, by / us / 1e6, dwref ? "" : "(ref)");
  if (dwref) {
    // different split counts sum in different orders: report max relative difference
    std::vector<float> h1(MN), h2(MN);
    CK(hipMemcpy(h1.data(), dwref, MN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), dwout, MN * 4, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    for (int i = 0; i < MN; ++i) { md = fmax(md, fabs(h1[i] - h2[i])); mx = fmax(mx, fabs(h1[i])); }
    printf("    max|diff|/max|ref| = %.2e\n", md / mx);
  }
}

template <int BM, int BN, int WM, int WN, bool AR = false>
void fwd_variant(const Shape& s, const FwdArgs& a, hipStream_t st, const float* yref,
                 double fl, double by) {
  if (a.M > BM || (AR && a.K > 64)) return;
  auto L = [&]() { launch_pwg<BM, BN, WM, WN, AR>(a, false, st); };
  float us = timeit(L, st, 20);
  const size_t n = (size_t)s.B * s.M * s.T * s.V;
  printf("%-20s fwd %3dx%3d w%dx%d%s         %8.1f us  %6.1f TF/s  %6.2f TB/s  %s\n", s.name,
         BM, BN, WM, WN, AR ? " AR" : "   ", us, fl / us / 1e6, by / us / 1e6,
         same(yref, a.y.ptr, n) ? "bit-exact" : "MISMATCH");
}

int main(int argc, char** argv) {
  const bool do_fwd = argc < 2 || strchr(argv[1], 'f');
  const bool do_dw = argc < 2 || strchr(argv[1], 'w');
  if (argc > 1 && strchr(argv[1], 'q')) {
    // tile quantization: the product forward at batch sizes around the model's, time per
    // 128-/256-position tile (tiles = P / BN; workgroup slots: 512 at M = 256, 768 at
    // M = 128, 1024 at M <= 64 with K <= 64)
    hipStream_t st; CK(hipStreamCreate(&st));
    const size_t maxe = (size_t)160 * 256 * 75 * 25 * 2;
    float *x, *y, *w;
    CK(hipMalloc(&x, maxe * 4)); CK(hipMalloc(&y, maxe * 4)); CK(hipMalloc(&w, 256 * 256 * 4));
    CK(hipMemset(x, 0, maxe * 4)); CK(hipMemset(w, 0, 256 * 256 * 4));
    struct Q { const char* name; int M, K, T, bn; };
    Q qs[] = {{"l9 tcn 256 T75", 256, 256, 75, 128}, {"l6 tcn 128 T150", 128, 128, 150, 128},
              {"l2 tcn 64 T300", 64, 64, 300, 256}};
    for (int rep = 0; rep < 2; ++rep)
      for (auto& q : qs)
        for (int B : {112, 120, 128, 132, 136, 140, 144, 150}) {
          const long long N = (long long)q.T * 25;
          if ((size_t)B * q.K * N > maxe || (size_t)B * q.M * N > maxe) continue;
          auto L = [&]() {
            sgcn_pw_fwd(w, 0, nullptr, x, q.K * N, N, 1, 0, nullptr, y, q.M * N, N, 1, 0, 0, 0,
                        B, q.M, q.K, q.T, 25, st);
          };
          const float us = timeit(L, st, 20);
          const double tiles = (double)B * N / q.bn;
          printf("%-18s B=%3d tiles %6.0f  %8.1f us  %6.4f us/tile  %6.1f TF/s\n", q.name, B, tiles,
                 us, us / tiles, 2.0 * B * N * q.M * q.K / us / 1e6);
        }
    return 0;
  }
  Shape shapes[] = {
    {"l2 tcn 64x64 T300", 128, 64, 64, 300, 25, false, false},
    {"l2 gcn 64x64 T300", 128, 64, 64, 300, 25, true, true},
    {"l6 tcn 128 T150", 128, 128, 128, 150, 25, false, false},
    {"l6 gcn 128 T150", 128, 128, 128, 150, 25, true, true},
    {"l9 tcn 256 T75", 128, 256, 256, 75, 25, false, false},
    {"l9 gcn 256 T75", 128, 256, 256, 75, 25, true, true},
    {"l5 tcn 128 T300", 128, 128, 128, 300, 25, false, false},
    {"l8 tcn-in 256x128 T150", 128, 256, 128, 150, 25, false, false},
    {"l5 gcn 128x64 T300", 128, 128, 64, 300, 25, true, true},
    {"l1 gcn 64x3 T300", 128, 64, 3, 300, 25, false, false},
    {"l1 dX 3x64 T300", 128, 3, 64, 300, 25, false, false},
    {"l5 dX 64x128 T300", 128, 64, 128, 300, 25, false, false},
  };
  hipStream_t st; CK(hipStreamCreate(&st));
  size_t maxe = (size_t)128 * 256 * 150 * 25;
  float *x, *y, *y2, *y3, *w, *mask, *ws, *dw1, *dw2;
  CK(hipMalloc(&x, maxe * 4)); CK(hipMalloc(&y, maxe * 4)); CK(hipMalloc(&y2, maxe * 4)); CK(hipMalloc(&y3, maxe * 4));
  CK(hipMalloc(&w, 256 * 256 * 4)); CK(hipMalloc(&mask, 64 * 256 * 4));
  CK(hipMalloc(&ws, 256 << 20)); CK(hipMalloc(&dw1, 256 * 256 * 4)); CK(hipMalloc(&dw2, 256 * 256 * 4));
  std::vector<float> h(maxe);
  for (size_t i = 0; i < maxe; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(x, h.data(), maxe * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(y, h.data() + 7, maxe * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data(), 256 * 256 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(mask, h.data(), 64 * 256 * 4, hipMemcpyHostToDevice));
  for (auto& s : shapes) {
    const long long N = (long long)s.T * s.V;
    const double P = (double)s.B * N;
    const double fl = 2.0 * P * s.M * s.K, by = 4.0 * P * (s.M + s.K);
    if (do_fwd) {
      FwdArgs a{};
      a.A = w; a.lda = s.K; a.a_mcontig = 0; a.bias = nullptr;
      a.x = {x, s.K * N, N, 1, s.rot ? 1 : 0};
      a.mask = s.mask ? mask : nullptr;
      a.y = {y2, s.M * N, N, 1, s.rot ? 1 : 0};
      a.M = s.M; a.K = s.K; a.T = s.T; a.V = s.V; a.B = s.B;
      fwd_divisors(a);
      auto L = [&]() {
        sgcn_pw_fwd(w, 0, nullptr, x, s.K * N, N, 1, s.rot ? 1 : 0, s.mask ? mask : nullptr,
                    y2, s.M * N, N, 1, s.rot ? 1 : 0, 0, 0, s.B, s.M, s.K, s.T, s.V, st);
      };
      float us = timeit(L, st, 20);
      // bit hash of the output, to compare builds (e.g. -DSGCN_PW_RPT=n) with each other
      const size_t ny = (size_t)s.B * s.M * N;
      g_h1.resize(ny);
      CK(hipMemcpy(g_h1.data(), y2, ny * 4, hipMemcpyDeviceToHost));
      unsigned long long hsh = 1469598103934665603ull;
      for (size_t i = 0; i < ny; ++i) {
        unsigned u;
        memcpy(&u, &g_h1[i], 4);
        hsh = (hsh ^ u) * 1099511628211ull;
      }
      printf("%-20s %-26s %8.1f us  %6.1f TF/s  %6.2f TB/s  hash %016llx\n", s.name,
             "fwd product", us, fl / us / 1e6, by / us / 1e6, hsh);
      if (argc > 2) {
        FwdArgs v = a;
        v.y.ptr = y3;
        v.x_bytes = plane_bytes(v.x.bstride, v.x.cstride, 1, s.B, s.K, s.T, s.V);
        v.y_bytes = plane_bytes(v.y.bstride, v.y.cstride, 1, s.B, s.M, s.T, s.V);
        v.a_bytes = (unsigned)(s.M * s.K * 4);
        v.mask_bytes = s.mask ? (unsigned)(s.V * s.K * 4) : 0u;
        fwd_variant<64, 256, 2, 4>(s, v, st, y2, fl, by);
        fwd_variant<64, 256, 2, 4, true>(s, v, st, y2, fl, by);
        fwd_variant<64, 128, 1, 4, true>(s, v, st, y2, fl, by);
        fwd_variant<64, 128, 2, 2, true>(s, v, st, y2, fl, by);
        fwd_variant<64, 256, 2, 4>(s, v, st, y2, fl, by);
        fwd_variant<64, 256, 2, 4, true>(s, v, st, y2, fl, by);
        fwd_variant<64, 128, 1, 4>(s, v, st, y2, fl, by);
        fwd_variant<64, 512, 2, 4>(s, v, st, y2, fl, by);
        fwd_variant<64, 256, 1, 4>(s, v, st, y2, fl, by);
        fwd_variant<128, 256, 2, 4>(s, v, st, y2, fl, by);
        fwd_variant<128, 128, 2, 2>(s, v, st, y2, fl, by);
        fwd_variant<128, 128, 4, 2>(s, v, st, y2, fl, by);
        fwd_variant<256, 128, 4, 2>(s, v, st, y2, fl, by);
        fwd_variant<256, 64, 4, 1>(s, v, st, y2, fl, by);
        fwd_variant<256, 128, 4, 1>(s, v, st, y2, fl, by);
        fwd_variant<256, 256, 4, 2>(s, v, st, y2, fl, by);
        fwd_variant<256, 64, 4, 2>(s, v, st, y2, fl, by);
        // 4 waves of 128 x 128 (MI = NJ = 4: 128 B of LDS fragment reads per MFMA)
        fwd_variant<256, 256, 2, 2>(s, v, st, y2, fl, by);
      }
    }
    if (do_dw) {
      // dW[m][c] = sum_p G(m,p) X(c,p): G = y (M rows), X = x (K rows)
      DwArgs d{};
      d.g = {y, s.M * N, N, 1, s.rot ? 1 : 0};
      d.x = {x, s.K * N, N, 1, s.rot ? 1 : 0};
      d.mask = s.mask ? mask : nullptr;
      d.M = s.M; d.Nc = s.K; d.T = s.T; d.V = s.V; d.B = s.B;
      const int bm = dw_tile(s.M), bn = dw_tile(s.K);
      const int tiles = ((s.M + bm - 1) / bm) * ((s.K + bn - 1) / bn);
      const int S0 = dw_splits(s.M, s.K, s.B, (int)N, tiles);
      if (bm == 128 && bn == 128) dw_variant<128, 128, 4, 2>("dw product 128x128", s, d, S0, st, ws, nullptr, dw1, fl, by);
      else dw_variant<64, 64, 2, 2>("dw product 64x64", s, d, S0, st, ws, nullptr, dw1, fl, by);
      DwArgs d3 = d;
      d3.g_bytes = plane_bytes(d.g.bstride, d.g.cstride, 1, s.B, s.M, s.T, s.V);
      d3.x_bytes = plane_bytes(d.x.bstride, d.x.cstride, 1, s.B, s.K, s.T, s.V);
      d3.mask_bytes = s.mask ? (unsigned)(s.V * s.K * 4) : 0u;
      int S3 = 0;
      const int MN = s.M * s.K;
      auto L3 = [&]() {
        S3 = launch_dw3(d3, st, ws, false);
        launch_slab_reduce(ws, nullptr, S3, s.M, s.K, dw2, 0, 0, nullptr, 0, st);
      };
      float us = timeit(L3, st, 10);
      std::vector<float> h1(MN), h2(MN);
      CK(hipMemcpy(h1.data(), dw1, MN * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), dw2, MN * 4, hipMemcpyDeviceToHost));
      double md = 0, mx = 0;
      for (int i = 0; i < MN; ++i) { md = fmax(md, fabs(h1[i] - h2[i])); mx = fmax(mx, fabs(h1[i])); }
      printf("%-20s %-26s S=%5d %8.1f us  %6.1f TF/s  %6.2f TB/s  max|diff|/max|ref| = %.2e\n",
             s.name, "dw3", S3, us, fl / us / 1e6, by / us / 1e6, md / mx);
    }
  }
  printf("done\n");
  return 0;
}
