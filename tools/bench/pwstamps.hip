// Phase timing of the forward contraction (diagnostic build: s_memtime stamps per
// workgroup at start / after the prologue / after the main loop / after the epilogue's
// stores drained). Tuning harness, not part of the product library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DSGCN_PW_STAMPS tools/bench/pwstamps.hip \
//         -o tools/bench/pwstamps
#include "../../shift-gcn_amd/csrc/pwconv.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Shape { const char* name; int B, M, K, T, V, rot; };

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  Shape shapes[] = {
    {"l2 tcn 64x64 T300", 128, 64, 64, 300, 25, 0},
    {"l2 gcn 64x64 T300 rot", 128, 64, 64, 300, 25, 1},
    {"l6 tcn 128 T150", 128, 128, 128, 150, 25, 0},
    {"l8 tcn 256x128 T150", 128, 256, 128, 150, 25, 0},
    {"l9 tcn 256 T75", 128, 256, 256, 75, 25, 0},
    {"l9 gcn 256 T75 rot", 128, 256, 256, 75, 25, 1},
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t maxe = (size_t)128 * 256 * 150 * 25;
  float *x, *y, *w, *bias;
  CK(hipMalloc(&x, maxe * 4));
  CK(hipMalloc(&y, maxe * 4));
  CK(hipMalloc(&w, 256 * 256 * 4));
  CK(hipMalloc(&bias, 256 * 4));
  CK(hipMemset(x, 0, maxe * 4));
  CK(hipMemset(w, 0, 256 * 256 * 4));
  CK(hipMemset(bias, 0, 256 * 4));
  unsigned long long* stamps;
  const size_t maxwg = 1 << 20;
  CK(hipMalloc(&stamps, maxwg * 4 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(sgcn::g_pw_stamps), &stamps, sizeof(stamps)));
  unsigned long long* where;
  CK(hipMalloc(&where, maxwg * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(sgcn::g_pw_where), &where, sizeof(where)));
  const char* dump = argc > 1 ? argv[1] : nullptr;   // per-workgroup CSV prefix
  int si = 0;
  for (auto& s : shapes) {
    const long long N = (long long)s.T * s.V;
    auto L = [&]() {
      return sgcn_pw_fwd(w, 0, bias, x, s.K * N, N, 1, s.rot, nullptr, y, s.M * N, N, 1, s.rot,
                         0, 0, s.B, s.M, s.K, s.T, s.V, st);
    };
    for (int i = 0; i < 3; ++i) CK((hipError_t)L());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    CK((hipError_t)L());
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const int BN = s.M <= 128 ? 256 : 128;
    const long long P = (long long)s.B * N;
    const int nwg = (int)((P + BN - 1) / BN);
    std::vector<unsigned long long> h((size_t)nwg * 4);
    CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> pro, mainl, epi, tot;
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int i = 0; i < nwg; ++i) {
      const unsigned long long* q = &h[(size_t)i * 4];
      pro.push_back((double)(q[1] - q[0]));
      mainl.push_back((double)(q[2] - q[1]));
      epi.push_back((double)(q[3] - q[2]));
      tot.push_back((double)(q[3] - q[0]));
      t0 = std::min(t0, q[0]);
      t1 = std::max(t1, q[3]);
    }
    if (dump) {
      std::vector<unsigned long long> hw((size_t)nwg);
      CK(hipMemcpy(hw.data(), where, hw.size() * 8, hipMemcpyDeviceToHost));
      char fn[512];
      snprintf(fn, sizeof fn, "%s_%d.csv", dump, si);
      FILE* f = fopen(fn, "w");
      fprintf(f, "wg,t0,t1,t2,t3,xcc,hwid\n");
      for (int i = 0; i < nwg; ++i) {
        const unsigned long long* q = &h[(size_t)i * 4];
        fprintf(f, "%d,%llu,%llu,%llu,%llu,%llu,%llu\n", i, q[0] - t0, q[1] - t0, q[2] - t0,
                q[3] - t0, hw[i] >> 32, hw[i] & 0xffffffffull);
      }
      fclose(f);
    }
    ++si;
    printf("%-24s %7.1f us  wg=%6d  median cycles: prologue %7.0f  main %7.0f  epilogue %7.0f"
           "  total %7.0f  (span %.0f cyc)\n", s.name, ms * 1e3, nwg, med(pro), med(mainl),
           med(epi), med(tot), (double)(t1 - t0));
  }
  return 0;
}
