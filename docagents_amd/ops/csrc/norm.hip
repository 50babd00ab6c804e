// Normalisation / embedding / pooling kernels (memory-bound: 16-B vector loads everywhere,
// Guideline 13). One workgroup per row, values kept in registers between the two passes so each
// row is read from HBM exactly once.
//
// Reference compute sites replaced: N1 (encoder LayerNorm / embeddings),
// N3 (`normalize`, internal/embeddings/openai.go:146-158 -> fused pooling + L2 norm), N6 (RMSNorm).
#include "common.h"

#define MAXCH 8  // max 8-element chunks per thread (D <= 8 * 8 * 256 = 16384)

template <typename T = BF16T>
__device__ __forceinline__ void load8(const bf16_t* p, float* v) {
  u32x4_t u = *(const u32x4_t*)p;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = T::to_f((bf16_t)(u[e] & 0xffff));
    v[2 * e + 1] = T::to_f((bf16_t)(u[e] >> 16));
  }
}
template <typename T = BF16T>
__device__ __forceinline__ void store8(bf16_t* p, const float* v) {
  *(u32x4_t*)p = u32x4_t{T::pack2(v[0], v[1]), T::pack2(v[2], v[3]), T::pack2(v[4], v[5]), T::pack2(v[6], v[7])};
}

// RMSNorm with optional fused residual add:
//   if resid: h = x + resid; resid <- h (residual stream updated in place); y = rms(h) * w
//   else:     y = rms(x) * w
__global__ void rmsnorm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ resid,
                               const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int D, float eps,
                               int ldx, int ldy) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (size_t)row * ldx;
  bf16_t* rr = resid ? resid + (size_t)row * D : nullptr;
  const int nch = D / 8;
  float v[MAXCH][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      load8(xr + c * 8, v[i]);
      if (rr) {
        float r[8];
        load8(rr + c * 8, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] += r[e];
        store8(rr + c * 8, v[i]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / D + eps);
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      float wv[8];
      load8(w + c * 8, wv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = v[i][e] * inv * wv[e];
      store8(y + (size_t)row * ldy + c * 8, v[i]);
    }
  }
}

// Many-row RMSNorm (prefill chunks: 57k rows of 3072): one WAVE per row, NCH 16-B chunks per lane
// (D = 64 * 8 * NCH), four rows per workgroup. The one-workgroup-per-row kernel above spends its
// time in two block barriers per 6 KB row and, at D = 3072, leaves half its threads with one chunk
// and half with two (4.2 TB/s measured in the QA prefill); here a row is a wave-level sum and every
// lane issues all its loads up front. Same math and roundings as rmsnorm_kernel.
template <int NCH>
__global__ void __launch_bounds__(256)
rmsnorm_rows_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ resid, const bf16_t* __restrict__ w,
                    bf16_t* __restrict__ y, int M, int D, float eps, int ldx, int ldy) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;  // whole wave: no barrier below
  const bf16_t* xr = x + (size_t)row * ldx;
  bf16_t* rr = resid ? resid + (size_t)row * D : nullptr;
  float v[NCH][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) load8(xr + (i * 64 + lane) * 8, v[i]);
  if (rr) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      float r[8];
      load8(rr + (i * 64 + lane) * 8, r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] += r[e];
      store8(rr + (i * 64 + lane) * 8, v[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / D + eps);
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    float wv[8];
    load8(w + (i * 64 + lane) * 8, wv);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[i][e] = v[i][e] * inv * wv[e];
    store8(y + (size_t)row * ldy + (i * 64 + lane) * 8, v[i]);
  }
}

// Optional fused fp8 output of a normalised row held in registers (v[i] = chunk threadIdx.x + i*blockDim):
// per-row e4m3 quantisation exactly like quant_fp8_rows_kernel, so the next GEMM can run on fp8
// without a separate quantisation pass over the activations.
__device__ __forceinline__ void store_row_fp8(float (&v)[MAXCH][8], int nch, int row, unsigned char* yq, int ldq,
                                              float* yscale, float* red) {
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[i][e]));
    }
  }
  amax = block_max(amax, red);
  const float sc = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) yscale[row] = sc;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][0] * inv, v[i][1] * inv, 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][2] * inv, v[i][3] * inv, lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][4] * inv, v[i][5] * inv, 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][6] * inv, v[i][7] * inv, hi, true);
      *(u32x2_t*)(yq + (size_t)row * ldq + c * 8) = u32x2_t{(unsigned)lo, (unsigned)hi};
    }
  }
}

// LayerNorm (BERT), optional residual input added first (x + resid), bias optional.
template <typename T = BF16T>
__global__ void layernorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ resid,
                                 const bf16_t* __restrict__ g, const bf16_t* __restrict__ b,
                                 bf16_t* __restrict__ y, int D, float eps, unsigned char* __restrict__ yq = nullptr,
                                 float* __restrict__ yscale = nullptr) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nch = D / 8;
  float v[MAXCH][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      load8<T>(x + (size_t)row * D + c * 8, v[i]);
      if (resid) {
        float r[8];
        load8<T>(resid + (size_t)row * D + c * 8, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] += r[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    }
  }
  const float mean = block_sum(s, red) / D;
  float var = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { float d = v[i][e] - mean; var += d * d; }
    }
  }
  var = block_sum(var, red) / D;
  const float inv = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      float gv[8], bv[8];
      load8<T>(g + c * 8, gv);
      if (b) load8<T>(b + c * 8, bv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = (v[i][e] - mean) * inv * gv[e] + (b ? bv[e] : 0.f);
      store8<T>(y + (size_t)row * D + c * 8, v[i]);
    }
  }
  if (yq) store_row_fp8(v, nch, row, yq, D, yscale, red);
}

// BERT embeddings: y = LN(word[ids[t]] + pos[positions[t]] + type[types ? types[t] : 0])
template <typename T = BF16T>
__global__ void bert_embed_ln_kernel(const int* __restrict__ ids, const int* __restrict__ positions,
                                     const int* __restrict__ types, const bf16_t* __restrict__ word,
                                     const bf16_t* __restrict__ pos, const bf16_t* __restrict__ type,
                                     const bf16_t* __restrict__ g, const bf16_t* __restrict__ b,
                                     bf16_t* __restrict__ y, int D, float eps, unsigned char* __restrict__ yq = nullptr,
                                     float* __restrict__ yscale = nullptr) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const size_t wi = (size_t)ids[row], pi = (size_t)positions[row], ti = types ? (size_t)types[row] : 0;
  const int nch = D / 8;
  float v[MAXCH][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      float a[8], p[8], t[8];
      load8<T>(word + wi * D + c * 8, a);
      load8<T>(pos + pi * D + c * 8, p);
      load8<T>(type + ti * D + c * 8, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[i][e] = a[e] + p[e] + t[e]; s += v[i][e]; }
    }
  }
  const float mean = block_sum(s, red) / D;
  float var = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { float d = v[i][e] - mean; var += d * d; }
    }
  }
  var = block_sum(var, red) / D;
  const float inv = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      float gv[8], bv[8];
      load8<T>(g + c * 8, gv);
      load8<T>(b + c * 8, bv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = (v[i][e] - mean) * inv * gv[e] + bv[e];
      store8<T>(y + (size_t)row * D + c * 8, v[i]);
    }
  }
  if (yq) store_row_fp8(v, nch, row, yq, D, yscale, red);
}

// Token embedding gather (decoder): y[t] = table[ids[t]]
__global__ void embed_kernel(const int* __restrict__ ids, const bf16_t* __restrict__ table,
                             bf16_t* __restrict__ y, int D) {
  const int row = blockIdx.x;
  const size_t id = (size_t)ids[row];
  // up to 4 chunks per thread loaded before any store (D = 3072 on 256 threads was a load, a wait,
  // a store and a second load: two table round trips in a row at the head of every decode step)
  constexpr int U = 4;
  const int nch = D / 8;
  for (int c0 = threadIdx.x; c0 < nch; c0 += U * blockDim.x) {
    u32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = *(const u32x4_t*)(table + id * D + (size_t)min(c0 + u * (int)blockDim.x, nch - 1) * 8);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * (int)blockDim.x;
      if (c < nch) *(u32x4_t*)(y + (size_t)row * D + c * 8) = v[u];
    }
  }
}

// Pooling + L2 normalisation (fp32 accumulate; zero vector left unchanged like the reference's
// `normalize`). mode 0 = CLS (first token), 1 = mean over the sequence's tokens.
// Output fp32 [B, D] and/or bf16 [B, D] (the index stores bf16).
template <typename T = BF16T>
__global__ void pool_l2norm_kernel(const bf16_t* __restrict__ h, const int* __restrict__ cu_seqlens,
                                   int D, int mode, float* __restrict__ out32,
                                   bf16_t* __restrict__ out16) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int s0 = cu_seqlens[b], s1 = cu_seqlens[b + 1];
  const int nch = D / 8;
  float v[MAXCH][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      if (mode == 0 || s1 <= s0) {
        load8<T>(h + (size_t)s0 * D + c * 8, v[i]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
        for (int t = s0; t < s1; ++t) {
          float a[8];
          load8<T>(h + (size_t)t * D + c * 8, a);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[i][e] += a[e];
        }
        const float invn = 1.f / (float)(s1 - s0);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] *= invn;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  ss = block_sum(ss, red);
  const float inv = ss > 0.f ? rsqrtf(ss) : 1.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] *= inv;
      if (out32) {
        float* o = out32 + (size_t)b * D + c * 8;
        *(f32x4_t*)o = f32x4_t{v[i][0], v[i][1], v[i][2], v[i][3]};
        *(f32x4_t*)(o + 4) = f32x4_t{v[i][4], v[i][5], v[i][6], v[i][7]};
      }
      if (out16) store8(out16 + (size_t)b * D + c * 8, v[i]);
    }
  }
}

// Per-row dynamic fp8 (OCP e4m3) quantisation for the fp8 GEMM path: scale[m] = amax(|x[m,:]|)/448,
// q = rne(x / scale) (v_cvt_pk_fp8_f32, saturating at +-448). One workgroup per row, the row kept
// in registers between the amax and the conversion pass.
__global__ void quant_fp8_rows_kernel(const bf16_t* __restrict__ x, int ldx, int K, unsigned char* __restrict__ out,
                                      int ldo, float* __restrict__ scale) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const bf16_t* xr = x + (size_t)row * ldx;
  const int nch = K / 8;
  float v[MAXCH][8];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      load8(xr + c * 8, v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[i][e]));
    }
  }
  amax = block_max(amax, red);
  const float sc = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) scale[row] = sc;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nch) {
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][0] * inv, v[i][1] * inv, 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][2] * inv, v[i][3] * inv, lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][4] * inv, v[i][5] * inv, 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][6] * inv, v[i][7] * inv, hi, true);
      *(u32x2_t*)(out + (size_t)row * ldo + c * 8) = u32x2_t{(unsigned)lo, (unsigned)hi};
    }
  }
}

static inline int row_threads(int D) {
  int ch = D / 8;
  int t = ((ch + 63) / 64) * 64;
  if (t > 256) t = 256;
  if (t < 64) t = 64;
  return t;
}
static inline bool d_ok(int D) { return D % 8 == 0 && D / 8 <= MAXCH * 256; }

DA_EXPORT int da_rmsnorm(const void* x, int ldx, void* resid, const void* w, void* y, int ldy, int M, int D,
                         float eps, void* stream) {
  if (!d_ok(D) || ldx % 8 || ldy % 8) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  // many rows of a width that is whole 512-element wave slices: one wave per row
  if (M >= 1024 && D % 512 == 0 && D / 512 <= 8) {
    const dim3 grid((M + 3) / 4);
#define RMS_ROWS(N) rmsnorm_rows_kernel<N><<<grid, 256, 0, (hipStream_t)stream>>>((const bf16_t*)x, (bf16_t*)resid, \
                      (const bf16_t*)w, (bf16_t*)y, M, D, eps, ldx, ldy)
    switch (D / 512) {
      case 4: RMS_ROWS(4); break;
      case 6: RMS_ROWS(6); break;
      case 8: RMS_ROWS(8); break;
      default: rmsnorm_kernel<<<M, row_threads(D), 0, (hipStream_t)stream>>>((const bf16_t*)x, (bf16_t*)resid,
                                                                           (const bf16_t*)w, (bf16_t*)y, D, eps,
                                                                           ldx, ldy);
    }
#undef RMS_ROWS
    DA_LAUNCH_CHECK();
  }
  rmsnorm_kernel<<<M, row_threads(D), 0, (hipStream_t)stream>>>((const bf16_t*)x, (bf16_t*)resid,
                                                                 (const bf16_t*)w, (bf16_t*)y, D, eps, ldx, ldy);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_layernorm(const void* x, const void* resid, const void* g, const void* b, void* y, int M, int D,
                           float eps, void* stream) {
  if (!d_ok(D)) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  layernorm_kernel<<<M, row_threads(D), 0, (hipStream_t)stream>>>((const bf16_t*)x, (const bf16_t*)resid,
                                                                   (const bf16_t*)g, (const bf16_t*)b,
                                                                   (bf16_t*)y, D, eps);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_bert_embed_ln(const void* ids, const void* positions, const void* types, const void* word,
                               const void* pos, const void* type, const void* g, const void* b, void* y, int T,
                               int D, float eps, void* stream) {
  if (!d_ok(D)) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  bert_embed_ln_kernel<<<T, row_threads(D), 0, (hipStream_t)stream>>>(
      (const int*)ids, (const int*)positions, (const int*)types, (const bf16_t*)word, (const bf16_t*)pos,
      (const bf16_t*)type, (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, D, eps);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_embed(const void* ids, const void* table, void* y, int T, int D, void* stream) {
  if (D % 8) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  embed_kernel<<<T, row_threads(D), 0, (hipStream_t)stream>>>((const int*)ids, (const bf16_t*)table,
                                                               (bf16_t*)y, D);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_pool_l2norm(const void* h, const void* cu_seqlens, int B, int D, int mode, void* out32,
                             void* out16, void* stream) {
  if (!d_ok(D)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  pool_l2norm_kernel<<<B, row_threads(D), 0, (hipStream_t)stream>>>((const bf16_t*)h, (const int*)cu_seqlens, D,
                                                                     mode, (float*)out32, (bf16_t*)out16);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_quant_fp8_rows(const void* x, int ldx, int M, int K, void* out, int ldo, void* scale, void* stream) {
  if (!d_ok(K) || ldx % 8 || ldo % 8) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  quant_fp8_rows_kernel<<<M, row_threads(K), 0, (hipStream_t)stream>>>((const bf16_t*)x, ldx, K, (unsigned char*)out,
                                                                       ldo, (float*)scale);
  DA_LAUNCH_CHECK();
}

// fp16 forms (the encoder's DTYPE=fp16): LayerNorm and embeddings + LayerNorm read / write fp16
// rows; pooling reads fp16 hidden states and writes fp32 and / or bf16 (the index storage type).
DA_EXPORT int da_layernorm_f16(const void* x, const void* resid, const void* g, const void* b, void* y, int M, int D,
                               float eps, void* stream) {
  if (!d_ok(D)) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  layernorm_kernel<F16T><<<M, row_threads(D), 0, (hipStream_t)stream>>>((const bf16_t*)x, (const bf16_t*)resid,
                                                                         (const bf16_t*)g, (const bf16_t*)b,
                                                                         (bf16_t*)y, D, eps);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_bert_embed_ln_f16(const void* ids, const void* positions, const void* types, const void* word,
                                   const void* pos, const void* type, const void* g, const void* b, void* y, int T,
                                   int D, float eps, void* stream) {
  if (!d_ok(D)) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  bert_embed_ln_kernel<F16T><<<T, row_threads(D), 0, (hipStream_t)stream>>>(
      (const int*)ids, (const int*)positions, (const int*)types, (const bf16_t*)word, (const bf16_t*)pos,
      (const bf16_t*)type, (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, D, eps);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_pool_l2norm_f16(const void* h, const void* cu_seqlens, int B, int D, int mode, void* out32,
                                 void* out16, void* stream) {
  if (!d_ok(D)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  pool_l2norm_kernel<F16T><<<B, row_threads(D), 0, (hipStream_t)stream>>>((const bf16_t*)h, (const int*)cu_seqlens,
                                                                           D, mode, (float*)out32, (bf16_t*)out16);
  DA_LAUNCH_CHECK();
}

// LayerNorm / BERT embeddings + LayerNorm with an additional fused fp8 (e4m3, per-row scale) output.
DA_EXPORT int da_layernorm_q(const void* x, const void* resid, const void* g, const void* b, void* y, void* yq,
                             void* yscale, int M, int D, float eps, void* stream) {
  if (!d_ok(D) || !yq || !yscale) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  layernorm_kernel<<<M, row_threads(D), 0, (hipStream_t)stream>>>((const bf16_t*)x, (const bf16_t*)resid,
                                                                   (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, D,
                                                                   eps, (unsigned char*)yq, (float*)yscale);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_bert_embed_ln_q(const void* ids, const void* positions, const void* types, const void* word,
                                 const void* pos, const void* type, const void* g, const void* b, void* y, void* yq,
                                 void* yscale, int T, int D, float eps, void* stream) {
  if (!d_ok(D) || !yq || !yscale) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  bert_embed_ln_kernel<<<T, row_threads(D), 0, (hipStream_t)stream>>>(
      (const int*)ids, (const int*)positions, (const int*)types, (const bf16_t*)word, (const bf16_t*)pos,
      (const bf16_t*)type, (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, D, eps, (unsigned char*)yq, (float*)yscale);
  DA_LAUNCH_CHECK();
}

// SwiGLU on a [M, 2F] projection whose columns are gate/up interleaved in 16-column groups (the
// w_gu row order of EPI_SWIGLU): out[m, 16j + i] = silu(g[m, 32j + i]) * u[m, 32j + 16 + i].
// Used when the gate/up GEMM runs on hipBLASLt (no SwiGLU epilogue there); one thread = 8 outputs,
// 16-B loads/stores, grid-stride over M * F / 8 chunks.
__global__ void __launch_bounds__(256)
swiglu_interleaved_kernel(const bf16_t* __restrict__ x, int ldx, bf16_t* __restrict__ y, int ldy, int M, int F) {
  const long long chunks = (long long)M * (F / 8);
  const int cpr = F / 8;
  for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < chunks;
       c += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(c / cpr), o = (int)(c % cpr) * 8;  // output column o .. o+7 (same 16-group)
    const int j = o >> 4, i = o & 15;
    const bf16_t* row = x + (size_t)m * ldx + 32 * j + i;
    const u32x4_t g = __builtin_nontemporal_load((const u32x4_t*)row);
    const u32x4_t u = __builtin_nontemporal_load((const u32x4_t*)(row + 16));
    u32x4_t r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float g0 = __uint_as_float(g[q] << 16), g1 = __uint_as_float(g[q] & 0xffff0000u);
      const float u0 = __uint_as_float(u[q] << 16), u1 = __uint_as_float(u[q] & 0xffff0000u);
      r[q] = pack_bf2(silu(g0) * u0, silu(g1) * u1);
    }
    *(u32x4_t*)(y + (size_t)m * ldy + o) = r;
  }
}

DA_EXPORT int da_swiglu_interleaved(const void* x, int ldx, void* y, int ldy, int M, int F, void* stream) {
  if (F % 16 || ldx % 8 || ldy % 8 || ldx < 2 * F || ldy < F) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const long long chunks = (long long)M * (F / 8);
  long long blocks = (chunks + 255) / 256;
  if (blocks > 256 * 32) blocks = 256 * 32;
  swiglu_interleaved_kernel<<<(int)blocks, 256, 0, (hipStream_t)stream>>>((const bf16_t*)x, ldx, (bf16_t*)y, ldy,
                                                                          M, F);
  DA_LAUNCH_CHECK();
}
