// CU-masked HIP streams (hipExtStreamCreateWithCUMask): the weight-gradient side stream
// may be confined to a subset of the CUs so that its MFMA-bound contractions do not take
// CU slots from the critical path's kernels (verdict r03, weak #4; shiftgcn/fused.py).
#include "common.hpp"

extern "C" {

int sgcn_device_cu_count(int device, int* count) {
  SGCN_REQUIRE(count);
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return (int)e;
  *count = prop.multiProcessorCount;
  return 0;
}

int sgcn_stream_create_cu_mask(const unsigned* mask, int words, void** stream) {
  SGCN_REQUIRE(mask && words > 0 && stream);
  hipStream_t s = nullptr;
  hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return (int)e;
  *stream = (void*)s;
  return 0;
}

int sgcn_stream_get_cu_mask(void* stream, unsigned* mask, int words) {
  SGCN_REQUIRE(stream && mask && words > 0);
  hipError_t e = hipExtStreamGetCUMask((hipStream_t)stream, (uint32_t)words, mask);
  return e == hipSuccess ? 0 : (int)e;
}

int sgcn_stream_destroy(void* stream) {
  SGCN_REQUIRE(stream);
  hipError_t e = hipStreamDestroy((hipStream_t)stream);
  return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"
