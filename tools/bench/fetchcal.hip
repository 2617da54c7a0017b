// FETCH_SIZE calibration by access shape (tuning harness; not part of the product library).
// Reads one (B, C, N) fp32 tensor — every element exactly once — in the shapes the product
// kernels use, so rocprofv3 --pmc FETCH_SIZE can be compared with the known byte count:
//   flat4   : 64 lanes x 4 B consecutive (256 B per wave instruction), flattened order
//   flat16  : 64 lanes x 16 B consecutive (1 KB per wave instruction)
//   seg<K>  : pw_dw3 / pw_dw operand staging: a lane owns one of K consecutive positions
//             of a (sample, t, v) chunk, 64/K rows (channels) per wave instruction; a
//             workgroup walks its split of the positions chunk by chunk over all C rows
// Each kernel also reports its time (GB/s at the algorithmic bytes).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench/fetchcal.hip -o tools/bench/fetchcal
//   ./fetchcal [B C N] [kernel]    (kernel: all | flat4 | flat16 | seg16 | seg32)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void flat4(const float* __restrict__ x, long n, float* __restrict__ out) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void flat16(const float4* __restrict__ x, long n4, float* __restrict__ out) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// split s of the P = B*N positions, chunks of K positions; lane (rsub = lane / K, kq =
// lane % K); wave w reads rows w*(64/K) + rsub + i*(NT/K)
template <int K>
__global__ __launch_bounds__(512) void seg(const float* __restrict__ x, int B, int C, int N,
                                           int chunks_per_split, float* __restrict__ out) {
  constexpr int NT = 512, RPW = 64 / K, RSTEP = NT / K;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kq = lane % K, rsub = lane / K;
  const long P = (long)B * N;
  const long nch = (P + K - 1) / K;
  const long q0 = (long)blockIdx.x * chunks_per_split;
  const long q1 = q0 + chunks_per_split < nch ? q0 + chunks_per_split : nch;
  float s = 0.f;
  for (long q = q0; q < q1; ++q) {
    const long p = q * K + kq;
    if (p >= P) continue;
    const long b = p / N, n = p - b * N;
    const float* base = x + b * (long)C * N + n;
    for (int r = w * RPW + rsub; r < C; r += RSTEP) s += base[(long)r * N];
  }
  out[blockIdx.x * NT + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int B = argc > 3 ? atoi(argv[1]) : 128;
  const int C = argc > 3 ? atoi(argv[2]) : 384;
  const int N = argc > 3 ? atoi(argv[3]) : 3750;
  const char* which = argc > 4 ? argv[4] : (argc == 2 ? argv[1] : "all");
  const long n = (long)B * C * N;
  float *x, *out;
  CK(hipMalloc(&x, n * 4 + 64));
  CK(hipMalloc(&out, (size_t)1 << 24));
  CK(hipMemset(x, 0, n * 4));
  // evict: write a 1 GB buffer so the tensor is not cache-resident
  float* junk;
  const size_t jn = (size_t)1 << 28;
  CK(hipMalloc(&junk, jn * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    if (strcmp(which, "all") && strcmp(which, name)) return;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(junk, rep, jn * 4));
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-8s B=%d C=%d N=%d  %8.1f us  %7.1f GB/s  (%.1f MB read)\n", name, B, C, N,
             ms * 1e3, n * 4 / (ms * 1e-3) / 1e9, n * 4 / 1e6);
    }
  };
  run("flat4", [&] { flat4<<<4096, 256>>>(x, n, out); });
  run("flat16", [&] { flat16<<<4096, 256>>>((const float4*)x, n / 4, out); });
  const long P = (long)B * N;
  auto seg_launch = [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    const long nch = (P + K - 1) / K;
    const int S = 512;
    const int cps = (int)((nch + S - 1) / S);
    seg<K><<<S, 512>>>(x, B, C, N, cps, out);
  };
  run("seg16", [&] { seg_launch(std::integral_constant<int, 16>{}); });
  run("seg32", [&] { seg_launch(std::integral_constant<int, 32>{}); });
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
