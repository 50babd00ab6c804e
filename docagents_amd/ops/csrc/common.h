// Shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Everything here is written for 64-lane wavefronts and the gfx950 MFMA
// operand layouts documented in /opt/skills/guides/cdna_hip_programming.md §3:
//   mfma_f32_16x16x32_bf16:  A lane l -> A[l&15][8*(l>>4)+j],  B lane l -> B[8*(l>>4)+j][l&15]
//                            C lane l -> C[4*(l>>4)+i][l&15]   (i = 0..3)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DA_WAVE 64

#ifndef DA_DEBUG
#define DA_ASSERT(x) ((void)0)
#else
#define DA_ASSERT(x) assert(x)
#endif

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // 8 bf16 = one MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4_t;    // 16x16 accumulator fragment
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t; // 16-byte vector memory op
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;

typedef uint16_t bf16_t;  // storage type: raw bf16 bits

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

// Round-to-nearest-even f32 -> bf16; NaN kept NaN.
__device__ __forceinline__ bf16_t f2bf(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = multiple of 64 (<= 1024). `red` needs 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// Bijective XCD-aware remap of a flat workgroup id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): blocks that share an XCD (b % 8) get a
// contiguous range of logical tile ids so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// 32-bit mix hash (for in-kernel Gumbel noise / deterministic sampling).
__device__ __forceinline__ unsigned hash_u32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float u01(unsigned a, unsigned b, unsigned c) {
  unsigned h = hash_u32(a ^ hash_u32(b + 0x9e3779b9u * hash_u32(c + 0x632be5abu)));
  return ((h >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
}

#define DA_EXPORT extern "C" __attribute__((visibility("default")))

// Launch error plumbing: every exported launcher returns hipError_t as int.
#define DA_LAUNCH_CHECK() return (int)hipGetLastError()
