// Runtime helpers of the kernel library: CU-masked HIP streams (spatial partitioning of the 256 CUs
// between the MFMA-bound prefill and the HBM-bound decode of the serving pipeline) and a placement
// probe that reports which XCD / CU each workgroup of a launch ran on.
//
// A CU-masked stream gets its own hardware queue whose dispatches are restricted to the CUs set in
// the mask (hipExtStreamCreateWithCUMask). Two streams with complementary masks let a decode
// graph replay and a prefill GEMM chain co-run on disjoint CUs, instead of time-slicing the whole
// chip as two plain streams do (bench/overlap_probe.py: 2-25 % overlap on plain streams).
#include "common.h"
#include <hip/hip_runtime_api.h>

DA_EXPORT int da_stream_create_cumask(unsigned nwords, const unsigned* mask, void** out) {
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, nwords, mask);
  if (e != hipSuccess) return (int)e;
  *out = (void*)s;
  return 0;
}

DA_EXPORT int da_stream_get_cumask(void* stream, unsigned nwords, unsigned* mask) {
  return (int)hipExtStreamGetCUMask((hipStream_t)stream, nwords, mask);
}

DA_EXPORT int da_stream_destroy(void* stream) { return (int)hipStreamDestroy((hipStream_t)stream); }

DA_EXPORT int da_device_cu_count(int device, int* out) {
  return (int)hipDeviceGetAttribute(out, hipDeviceAttributeMultiprocessorCount, device);
}

// One record per workgroup: {XCC id, HW_ID register (CU / SH / SE fields), wall-clock start}.
// Every workgroup spins ~`spin` cycles so that a launch of more workgroups than the mask allows
// really spreads over the permitted CUs (rather than finishing on the first few).
__global__ void placement_kernel(unsigned* out, long long spin) {
  unsigned xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) {
    unsigned* r = out + 4 * blockIdx.x;
    r[0] = __builtin_amdgcn_readfirstlane(xcc);
    r[1] = __builtin_amdgcn_readfirstlane(hwid);
    r[2] = (unsigned)t0;
    r[3] = (unsigned)(t0 >> 32);
  }
}

DA_EXPORT int da_placement_probe(void* out, int blocks, long long spin, void* stream) {
  if (blocks <= 0) return (int)hipErrorInvalidValue;
  placement_kernel<<<blocks, 64, 0, (hipStream_t)stream>>>((unsigned*)out, spin);
  DA_LAUNCH_CHECK();
}
