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

// ------------------------------------------------------------------------------------------
// Read-bandwidth probe for a CU subset (bench/cumask_bw.py): how many bytes per second can the
// CUs of a masked stream pull from HBM, by LDS-DMA into an LDS ring (mode 0: D 1-KB wave loads in
// flight per wave, no registers held) or into registers (mode 1: U 1-KB loads per wave per round)?
// The decode attention is bound by exactly this on a partition of the chip.
typedef __attribute__((address_space(3))) void* probe_lds_t;
typedef __attribute__((address_space(1))) const void* probe_g_t;

template <int D>
__global__ void __launch_bounds__(256) lds_stream_probe(const char* __restrict__ src, long long per_wg,
                                                        unsigned* out) {
  __shared__ __attribute__((aligned(16))) char ring[4][32][1024];  // 128 KB: 32 slots per wave
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const char* base = src + blockIdx.x * per_wg;
  const long long n = per_wg / 4096;  // loads per wave
  for (long long k = 0; k < n; ++k) {
    __builtin_amdgcn_global_load_lds((probe_g_t)(base + (k * 4 + w) * 1024 + lane * 16),
                                     (probe_lds_t)&ring[w][k & 31][0], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ring[w][lane & 31][lane] == 0x5a && lane == 63) out[blockIdx.x] = 1;  // keep the stream live
}

template <int U>
__global__ void __launch_bounds__(256) reg_stream_probe(const char* __restrict__ src, long long per_wg,
                                                        unsigned* out) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const char* base = src + blockIdx.x * per_wg;
  const long long n = per_wg / 4096;
  unsigned acc = 0;
  for (long long k = 0; k < n; k += U) {
    u32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long kk = k + u < n ? k + u : n - 1;
      v[u] = __builtin_nontemporal_load((const u32x4_t*)(base + (kk * 4 + w) * 1024 + lane * 16));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// mode 0: LDS-DMA ring, depth 8 / 16 / 31; mode 1: registers, U = 8 / 16. per_wg % 4096 == 0.
DA_EXPORT int da_stream_probe(const void* src, long long per_wg, int nwg, int mode, int depth, void* out,
                              void* stream) {
  if (nwg <= 0 || per_wg % 4096 || !src || !out) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const char* p = (const char*)src;
  unsigned* o = (unsigned*)out;
  if (mode == 0) {
    if (depth >= 31) lds_stream_probe<31><<<nwg, 256, 0, s>>>(p, per_wg, o);
    else if (depth >= 16) lds_stream_probe<16><<<nwg, 256, 0, s>>>(p, per_wg, o);
    else lds_stream_probe<8><<<nwg, 256, 0, s>>>(p, per_wg, o);
  } else {
    if (depth >= 16) reg_stream_probe<16><<<nwg, 256, 0, s>>>(p, per_wg, o);
    else reg_stream_probe<8><<<nwg, 256, 0, s>>>(p, per_wg, o);
  }
  DA_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// A bounded device-side delay: one wave polling the 100 MHz wall clock (s_memrealtime) for `us`
// microseconds. Tests use it to hold a stream busy deterministically (a writer's copies queued
// behind it) so that a reader on another stream provably overlaps the writer's pending work (index
// write/search race). Bounded to 10 s.
__global__ void spin_kernel(long long ticks, int* out) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0 && out) out[0] = 1;
}

DA_EXPORT int da_spin(int us, void* out, void* stream) {
  if (us < 0 || us > 10000000) return (int)hipErrorInvalidValue;
  spin_kernel<<<1, 64, 0, (hipStream_t)stream>>>((long long)us * 100, (int*)out);
  DA_LAUNCH_CHECK();
}
