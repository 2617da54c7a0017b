// Operand over-fetch probe of the forward contraction (verdict r03 weak #2): the NTU unit
// shapes of sgcn_pw_fwd as the model launches them, 1 warm-up + 5 timed launches each, in
// a fixed order (tools/ofetch_summary.py groups the rocprofv3 dispatches by that order).
// Built several ways by tools/gpu_ofetch.sh (tuning harness, not the product library):
//   product | -DSGCN_PW_DIAG=1 (no weight loads after stage 0: the weights' share of the
//   fetch) | -DSGCN_PW_DIAG=2 (no X loads after stage 0) | -DSGCN_PW_XPOL=2 (X loads nt) |
//   -DSGCN_PW_APOL=16 ...
// Prints per shape: average us, TF/s and the bit hash of the output.
#include "../../shift-gcn_amd/csrc/pwconv.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Shape { const char* name; int M, K, T, mc, acc; };

int main(int argc, char** argv) {
  const int B = 128, V = 25;
  Shape shapes[] = {
      {"l2 gcn 64<-64 T300", 64, 64, 300, 1, 0},
      {"l5 gcn 128<-64 T300", 128, 64, 300, 1, 0},
      {"l5 down 128<-64 T300", 128, 64, 300, 0, 0},
      {"l6 tcn 128<-128 T150", 128, 128, 150, 0, 0},
      {"l8 gcn 256<-128 T150", 256, 128, 150, 1, 0},
      {"l8 down 256<-128 T150", 256, 128, 150, 0, 0},
      {"l9 tcn 256<-256 T75", 256, 256, 75, 0, 0},
      {"l8 dX acc 128<-256 T150", 128, 256, 150, 1, 1},
  };
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  size_t maxe = (size_t)B * 256 * 150 * V;   // 122.9 M floats (491.5 MB)
  float *x, *y, *w, *bias;
  CK(hipMalloc(&x, maxe * 4));
  CK(hipMalloc(&y, maxe * 4));
  CK(hipMalloc(&w, 256 * 256 * 4));
  CK(hipMalloc(&bias, 256 * 4));
  std::vector<float> h(maxe);
  for (size_t i = 0; i < maxe; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(x, h.data(), maxe * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data() + 11, 256 * 256 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h.data() + 3, 256 * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // OFETCH_POLLUTE=1: 1 GiB written before every launch (the model's cache state: the
  // contraction's input was just written among other tensors), each launch timed alone
  const bool pollute = getenv("OFETCH_POLLUTE") && atoi(getenv("OFETCH_POLLUTE"));
  float* junk = nullptr;
  if (pollute) CK(hipMalloc(&junk, (size_t)1 << 30));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int si = 0;
  for (auto& s : shapes) {
    if (only >= 0 && si++ != only) continue;
    const long long N = (long long)s.T * V;
    const double P = (double)B * N, fl = 2.0 * P * s.M * s.K;
    auto L = [&]() {
      int rc = sgcn_pw_fwd(w, s.mc, s.acc ? nullptr : bias, x, s.K * N, N, 1, 0, nullptr, y,
                           s.M * N, N, 1, 0, 0, s.acc, B, s.M, s.K, s.T, V, st);
      if (rc) { printf("rc %d\n", rc); exit(1); }
    };
    CK(hipMemset(y, 0, (size_t)B * s.M * N * 4));
    float ms = 0.f;
    if (pollute) {
      for (int i = 0; i < 6; ++i) {
        CK(hipMemsetAsync(junk, i, (size_t)1 << 30, st));
        CK(hipEventRecord(e0, st));
        L();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float one;
        CK(hipEventElapsedTime(&one, e0, e1));
        if (i) ms += one;
      }
    } else {
      L();
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < 5; ++i) L();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    const size_t ny = (size_t)B * s.M * N;
    std::vector<float> hy(ny);
    CK(hipMemcpy(hy.data(), y, ny * 4, hipMemcpyDeviceToHost));
    unsigned long long hsh = 1469598103934665603ull;
    for (size_t i = 0; i < ny; ++i) {
      unsigned u;
      memcpy(&u, &hy[i], 4);
      hsh = (hsh ^ u) * 1099511628211ull;
    }
    const double us = ms * 1000.0 / 5;
    printf("%-26s %8.1f us  %6.1f TF/s  alg_read_MB %7.1f  alg_write_MB %7.1f  hash %016llx\n",
           s.name, us, fl / us / 1e6, 4.0 * P * (s.K + (s.acc ? s.M : 0)) / 1e6,
           4.0 * P * s.M / 1e6, hsh);
  }
  printf("done\n");
  return 0;
}
