// Shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Everything here is written for 64-lane wavefronts and the gfx950 MFMA
// operand layouts documented in /opt/skills/guides/cdna_hip_programming.md §3:
//   mfma_f32_16x16x32_bf16:  A lane l -> A[l&15][8*(l>>4)+j],  B lane l -> B[8*(l>>4)+j][l&15]
//                            C lane l -> C[4*(l>>4)+i][l&15]   (i = 0..3)
//   mfma_f32_32x32x16_bf16:  A lane l -> A[l&31][8*(l>>5)+j],  B lane l -> B[8*(l>>5)+j][l&31]
//                            C lane l, reg r -> C[8*(r>>2)+4*(l>>5)+(r&3)][l&31]   (r = 0..15)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DA_WAVE 64

// Debug builds (python -m docagents_amd.ops.build --debug: -O1 -g -DDA_DEBUG) turn DA_ASSERT into
// device asserts at the kernels' indexing hot spots (cache slots / positions, top-k rows, ranges),
// for fault isolation together with AMD_SERIALIZE_KERNEL=3.
#ifndef DA_DEBUG
#define DA_ASSERT(x) ((void)0)
#else
#include <cassert>
#define DA_ASSERT(x) assert(x)
#endif

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // 8 bf16 = one MFMA A/B fragment
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;    // 16x16 accumulator fragment
typedef __attribute__((ext_vector_type(16))) float f32x16_t;  // 32x32 accumulator fragment
typedef __attribute__((ext_vector_type(4))) short s16x4_t;    // ds_read_b64_tr_b16 result
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t; // 16-byte vector memory op
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;

typedef uint16_t bf16_t;  // storage type: raw bf16 bits

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

// f32 -> bf16, round-to-nearest-even (NaN stays NaN): gfx950 has a hardware conversion
// (v_cvt_pk_bf16_f32, two values per instruction), which clang emits for __bf16 casts.
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_hw_t;

__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  const bf16x2_hw_t r = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, r);
}

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16_t mfma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------
// 16-bit element types of the kernels: bf16 (everything) and fp16 (the encoder's DTYPE=fp16 path:
// GEMMs on v_mfma_f32_*_f16, flash attention, LayerNorm / embeddings / pooling). Both are stored as
// raw 16-bit words and moved as bf16x8_t / u32x4_t registers; only the conversions and the MFMA
// opcode depend on the type, so one kernel template serves both (fp32 accumulation either way).
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_hw_t;

struct BF16T {
  static constexpr bool kF16 = false;
  __device__ static __forceinline__ float to_f(uint16_t v) { return bf2f(v); }
  __device__ static __forceinline__ uint16_t from_f(float f) { return f2bf(f); }
  __device__ static __forceinline__ unsigned pack2(float lo, float hi) { return pack_bf2(lo, hi); }
  __device__ static __forceinline__ f32x4_t mma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ f32x16_t mma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

struct F16T {
  static constexpr bool kF16 = true;
  __device__ static __forceinline__ float to_f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
  __device__ static __forceinline__ uint16_t from_f(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
  __device__ static __forceinline__ unsigned pack2(float lo, float hi) {
    const f16x2_hw_t r = {(_Float16)lo, (_Float16)hi};
    return __builtin_bit_cast(unsigned, r);
  }
  __device__ static __forceinline__ f32x4_t mma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                 0, 0, 0);
  }
  __device__ static __forceinline__ f32x16_t mma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                 0, 0, 0);
  }
};

// Exchange with lane l^32 (v_permlane32_swap, a VALU op — no LDS crossbar). Returns {own, partner}
// in some order, so callers combine both halves symmetrically (max / sum).
__device__ __forceinline__ float max_xhalf(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xhalf(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// gfx950 ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q / columns 4p..4p+3 of a
// 4x16 block of 16-bit values; lane i receives column i (row q in element q).
__device__ __forceinline__ s16x4_t lds_read_tr16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

// sum_{q < n} p[q * stride] in index order (((0 + p_0) + p_1) + ...), the loads issued 8 at a time:
// a runtime-count loop of `s += p[q * stride]` waits for each load before the next add — one
// memory round trip per term (the split-K reduce's deferred-norm sums were 6 in a row).
__device__ __forceinline__ float sum_strided(const float* __restrict__ p, int n, size_t stride) {
  float s = 0.f;
  for (int q0 = 0; q0 < n; q0 += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[(size_t)min(q0 + j, n - 1) * stride];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (q0 + j < n) s += v[j];
  }
  return s;
}

// v[e] = sum_{s < n} p[s * stride + e] (e < 8; p and stride 16-B aligned) in split order, the 16-B
// loads of 8 splits issued together (clamped): split-K reduces over 2-3 splits otherwise ran a
// remainder loop that waited for each split's loads before the next.
__device__ __forceinline__ void sum_rows8(const float* __restrict__ p, int n, size_t stride, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
  for (int s0 = 0; s0 < n; s0 += 8) {
    f32x4_t a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float* r = p + (size_t)min(s0 + j, n - 1) * stride;
      a[j] = *(const f32x4_t*)r;
      b[j] = *(const f32x4_t*)(r + 4);
    }
    // past n: + 0.f, an exact identity here (the sums start at +0 and never become -0), so the adds
    // are unconditional and no load is sunk into a branch
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool in = s0 + j < n;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += in ? a[j][e] : 0.f;
        v[4 + e] += in ? b[j][e] : 0.f;
      }
    }
  }
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

// x * sigmoid(x) with the hardware reciprocal (1 ulp) instead of an IEEE division (a 10-instruction
// scale / fma / fixup sequence per element): every caller rounds the result to bf16.
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

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
