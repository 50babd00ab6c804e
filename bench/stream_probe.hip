// Read-streaming probe for MI355X HBM: how long does it take to pull N bytes through W workgroups
// when every wave issues all of its 16-B-per-lane loads up front (the batch-1 decode-attention
// access pattern), vs a grid-stride loop with a few loads in flight? Answers "what is the floor for a
// ~35 MB read that has to finish inside one short kernel" (latency + ramp, not steady-state BW).
// Build + run (GPU box): hipcc -O3 --offload-arch=gfx950 bench/stream_probe.hip -o /tmp/sp && /tmp/sp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// each wave reads `per_wave` contiguous KiB (1 KiB per wave-instruction), all loads issued first
template <int NL>
__global__ void __launch_bounds__(256) burst(const u32x4* __restrict__ src, unsigned* out, long long waves_total) {
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wave >= waves_total) return;
  const u32x4* p = src + wave * NL * 64 + lane;
  u32x4 v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) v[i] = __builtin_nontemporal_load(p + i * 64);
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads
}

// grid-stride streaming with U loads in flight per lane
template <int U>
__global__ void __launch_bounds__(256) gstride(const u32x4* __restrict__ src, unsigned* out, long long n16) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long stride = (long long)gridDim.x * blockDim.x;
  unsigned acc = 0;
  for (long long i = tid; i < n16; i += stride * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long j = i + u * stride;
      v[u] = j < n16 ? __builtin_nontemporal_load(src + j) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename F>
static float time_us(F f, int reps = 50) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  // flush: the probe buffers are re-read each rep; each rep reads a different 256 MB window below
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const size_t total = 4ull << 30;  // 4 GiB pool: rotate windows so nothing is served from MALL
  u32x4* buf; unsigned* out;
  CK(hipMalloc(&buf, total)); CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, total));
  const size_t win = 320ull << 20;  // > 256 MB Infinity Cache
  const int nwin = (int)(total / win);
  int rot = 0;
  for (size_t mb : {9, 18, 35, 70, 140}) {
    const size_t bytes = mb << 20;
    for (int nl : {8, 24, 48}) {
      const long long waves = (long long)(bytes / (nl * 1024));
      const int wgs = (int)((waves + 3) / 4);
      auto f = [&]() {
        const u32x4* src = (const u32x4*)((char*)buf + (size_t)(rot++ % nwin) * win);
        if (nl == 8) burst<8><<<wgs, 256>>>(src, out, waves);
        else if (nl == 24) burst<24><<<wgs, 256>>>(src, out, waves);
        else burst<48><<<wgs, 256>>>(src, out, waves);
      };
      const float us = time_us(f);
      printf("{\"probe\": \"burst\", \"MB\": %zu, \"KiB_per_wave\": %d, \"wgs\": %d, \"us\": %.2f, \"TBps\": %.2f}\n", mb, nl,
             wgs, us, bytes / us / 1e6);
    }
    for (int wgs : {256, 512, 1024, 2048}) {
      const long long n16 = (long long)(bytes / 16);
      auto f = [&]() {
        const u32x4* src = (const u32x4*)((char*)buf + (size_t)(rot++ % nwin) * win);
        gstride<4><<<wgs, 256>>>(src, out, n16);
      };
      const float us = time_us(f);
      printf("{\"probe\": \"gstride4\", \"MB\": %zu, \"wgs\": %d, \"us\": %.2f, \"TBps\": %.2f}\n", mb, wgs, us,
             bytes / us / 1e6);
    }
  }
  // empty-kernel floor (launch + drain) for reference
  auto f0 = [&]() { burst<8><<<256, 256>>>((const u32x4*)buf, out, 0); };
  printf("{\"probe\": \"empty\", \"us\": %.2f}\n", time_us(f0));
  hipFree(buf); hipFree(out);
  return 0;
}
