// Weight prefetch into the memory-side Infinity Cache (MALL) for latency-bound decode GEMMs.
//
// At batch 1..64 the decode GEMMs stream 19-100 MB of weights each in 12-30 us: too little work to
// keep enough bytes in flight to reach HBM bandwidth (profiles/gemv_batch1_decode_r1.txt: 1.4-4.5 TB/s
// on the Phi-3 shapes). The weights of the NEXT op do not depend on activations, so a small
// workgroup count on a side stream (forked inside the captured decode graph) can read them while the
// current op runs; the dependent GEMM then hits in MALL instead of HBM. The kernel only loads: the
// result is folded into a value that is stored only when it equals an impossible sentinel, so the
// loads cannot be eliminated and nothing is written in practice.
#include "common.h"

__global__ void __launch_bounds__(256) mall_prefetch_kernel(const u32x4_t* __restrict__ p, long n16,
                                                            unsigned* __restrict__ sink, unsigned key) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned acc = 0;
  // 4 independent 16-B loads in flight per lane per iteration
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4_t a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= (a.x ^ a.y ^ a.z ^ a.w) + (b.x ^ b.y ^ b.z ^ b.w) + (c.x ^ c.y ^ c.z ^ c.w) + (d.x ^ d.y ^ d.z ^ d.w);
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == key) sink[threadIdx.x & 63] = acc;  // key is a runtime argument: loads stay live
}

DA_EXPORT int da_mall_prefetch(const void* ptr, long nbytes, int nwg, void* sink, void* stream) {
  if (((uintptr_t)ptr & 15) || nbytes < 0 || nwg <= 0) return (int)hipErrorInvalidValue;
  long n16 = nbytes / 16;
  if (n16 == 0) return 0;
  mall_prefetch_kernel<<<nwg, 256, 0, (hipStream_t)stream>>>((const u32x4_t*)ptr, n16, (unsigned*)sink,
                                                                 0x9e3779b9u);
  DA_LAUNCH_CHECK();
}
