// Attention kernels for gfx950.
//
// 1) flash_attn_varlen: packed (varlen) prefill attention, bidirectional (BERT encoder, SURVEY
//    §2.4 N1) or causal with GQA (Llama-3 / Phi-3 prefill, N6/N7). Online softmax in fp32, bf16
//    MFMA (v_mfma_f32_16x16x32_bf16). "Swapped" formulation (cdna_hip_programming.md T12 / §3):
//    S^T = K·Q^T puts the query on the MFMA lane, so every softmax statistic and the O^T rescale
//    are lane-local, and the S^T accumulator registers ARE the B operand of O^T += V^T·P^T once
//    the k index is permuted consistently on both operands (no LDS round trip for P).
//    One workgroup = 4 waves x 16 queries; K tile in LDS with a 16-B row pad (conflict-free
//    ds_read_b128), V tile stored transposed in LDS for the V^T operand.
//
// 2) decode attention (one new token per sequence) over the KV cache [slot, Hkv, max_seq, D]:
//    split-KV ("flash-decoding") so a batch of long contexts fills all 256 CUs; fp32 partials
//    (unnormalised O, running max, running sum) merged by decode_combine.
#include "common.h"

template <int D>
__global__ void __launch_bounds__(256)
flash_attn_varlen_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                         int ldq, int ldk, int ldv, const int* __restrict__ cu, int H, int Hkv, int causal,
                         float scale_log2e, bf16_t* __restrict__ o, int ldo) {
  constexpr int KT = 64;                 // keys per tile
  constexpr int KSTR = D * 2 + 16;       // K row stride (bytes) in LDS
  constexpr int VSTR = KT * 2 + 8;       // V^T row stride (bytes)
  constexpr int NKK = D / 32;            // k-steps for S (over d)
  constexpr int NDT = D / 16;            // d tiles for O
  constexpr int CPR = D / 8;             // 16-B chunks per row
  __shared__ __attribute__((aligned(16))) char sK[KT * KSTR];
  __shared__ __attribute__((aligned(16))) char sVt[D * VSTR];

  const int b = blockIdx.z, h = blockIdx.y;
  const int s0 = cu[b], L = cu[b + 1] - s0;
  const int q0 = blockIdx.x * 64;
  if (q0 >= L) return;
  const int hk = h / (H / Hkv);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int qi = q0 + wid * 16 + fr;  // this lane's query (MFMA column)
  const bool qvalid = qi < L;

  bf16x8_t qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    if (qvalid) qf[kk] = *(const bf16x8_t*)(q + (size_t)(s0 + qi) * ldq + h * D + kk * 32 + fg * 8);
    else qf[kk] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }

  f32x4_t oacc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) oacc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_part = 0.f;

  const int kv_end = causal ? min(L, q0 + 64) : L;
  const int ntiles = (kv_end + KT - 1) / KT;
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kbase = kt * KT;
    // ---- stage K (row-major, padded) and V^T into LDS ----
    for (int idx = tid; idx < KT * CPR; idx += 256) {
      const int r = idx / CPR, c = idx % CPR;
      const int key = kbase + r;
      u32x4_t kvv = u32x4_t{0, 0, 0, 0}, vvv = u32x4_t{0, 0, 0, 0};
      if (key < L) {
        kvv = *(const u32x4_t*)(k + (size_t)(s0 + key) * ldk + hk * D + c * 8);
        vvv = *(const u32x4_t*)(v + (size_t)(s0 + key) * ldv + hk * D + c * 8);
      }
      *(u32x4_t*)(sK + r * KSTR + c * 16) = kvv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        *(bf16_t*)(sVt + (c * 8 + 2 * e) * VSTR + r * 2) = (bf16_t)(vvv[e] & 0xffff);
        *(bf16_t*)(sVt + (c * 8 + 2 * e + 1) * VSTR + r * 2) = (bf16_t)(vvv[e] >> 16);
      }
    }
    __syncthreads();

    // ---- S^T[key][q] for 4 key tiles of 16 ----
    f32x4_t sacc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sacc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const bf16x8_t a = *(const bf16x8_t*)(sK + (t * 16 + fr) * KSTR + kk * 64 + fg * 16);
        sacc[t] = mfma16(a, qf[kk], sacc[t]);
      }
    }
    // ---- mask + online softmax (per query = per lane column) ----
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kbase + t * 16 + fg * 4 + i;
        float s = sacc[t][i] * scale_log2e;
        if (key >= L || (causal && key > qi)) s = -INFINITY;
        sacc[t][i] = s;
        tmax = fmaxf(tmax, s);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(sacc[t][i] - m_use);
        sacc[t][i] = p;
        psum += p;
      }
    l_part = l_part * alpha + psum;
#pragma unroll
    for (int i = 0; i < NDT; ++i) oacc[i] *= alpha;

    // ---- O^T[d][q] += V^T[d][key] · P^T[key][q]; k permuted: j -> key 32c + 16(j>>2) + 4g + (j&3) ----
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8_t pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (short)f2bf(sacc[2 * c][j]);
        pb[4 + j] = (short)f2bf(sacc[2 * c + 1][j]);
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const char* rowp = sVt + (dt * 16 + fr) * VSTR;
        const u32x2_t lo = *(const u32x2_t*)(rowp + (32 * c + 4 * fg) * 2);
        const u32x2_t hi = *(const u32x2_t*)(rowp + (32 * c + 16 + 4 * fg) * 2);
        bf16x8_t va;
        va[0] = (short)(lo[0] & 0xffff); va[1] = (short)(lo[0] >> 16);
        va[2] = (short)(lo[1] & 0xffff); va[3] = (short)(lo[1] >> 16);
        va[4] = (short)(hi[0] & 0xffff); va[5] = (short)(hi[0] >> 16);
        va[6] = (short)(hi[1] & 0xffff); va[7] = (short)(hi[1] >> 16);
        oacc[dt] = mfma16(va, pb, oacc[dt]);
      }
    }
    __syncthreads();
  }

  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qvalid) {
    bf16_t* orow = o + (size_t)(s0 + qi) * ldo + h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      *(u32x2_t*)(orow + dt * 16 + fg * 4) =
          u32x2_t{pack_bf2(oacc[dt][0] * inv, oacc[dt][1] * inv), pack_bf2(oacc[dt][2] * inv, oacc[dt][3] * inv)};
    }
  }
}

// ------------------------------------------------------------------------------------------
// Decode attention: q [B, ldq] (head h at h*D), caches [slots, Hkv, max_seq, D],
// lens[b] = tokens in cache for b (current token included), slot[b] = cache slot of b.
// Partials: po [B, H, nsplit, D] fp32, pm/pl [B, H, nsplit].
template <int D, int G>
__global__ void __launch_bounds__(256)
decode_attn_kernel(const bf16_t* __restrict__ q, int ldq, const bf16_t* __restrict__ kc,
                   const bf16_t* __restrict__ vc, const int* __restrict__ lens, const int* __restrict__ slot,
                   int H, int Hkv, int max_seq, int chunk, int nsplit, float scale_log2e,
                   float* __restrict__ po, float* __restrict__ pm, float* __restrict__ pl) {
  constexpr int KT = 64;
  constexpr int PART = D / 4;            // dims per thread in the score phase
  constexpr int NP = D / 2;              // d-pairs
  constexpr int KG = 256 / NP;           // key groups in the PV phase
  __shared__ float sq[G][D];
  __shared__ float sp[G][KT];
  __shared__ float salpha[G], sm[G], sl[G];
  __shared__ float sred[KG > 0 ? KG : 1][G][D];

  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int L = lens[b];
  const int kstart = split * chunk;
  const int kend = min(L, kstart + chunk);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const size_t cbase = ((size_t)slot[b] * Hkv + hk) * (size_t)max_seq * D;

  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    sq[g][d] = bf2f(q[(size_t)b * ldq + (hk * G + g) * D + d]) * scale_log2e;
  }
  if (tid < G) { sm[tid] = -INFINITY; sl[tid] = 0.f; }
  const int dp = tid % NP, kg = tid / NP;
  float oacc[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) { oacc[g][0] = 0.f; oacc[g][1] = 0.f; }
  __syncthreads();

  for (int kb = kstart; kb < kend; kb += KT) {
    // ---- scores: 4 lanes per key, each PART dims ----
    {
      const int key = kb + (tid >> 2), part = tid & 3;
      float dots[G];
#pragma unroll
      for (int g = 0; g < G; ++g) dots[g] = 0.f;
      if (key < kend) {
        const bf16_t* kr = kc + cbase + (size_t)key * D + part * PART;
#pragma unroll
        for (int c = 0; c < PART / 8; ++c) {
          u32x4_t u = *(const u32x4_t*)(kr + c * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float kv = bf2f((bf16_t)((e & 1) ? (u[e >> 1] >> 16) : (u[e >> 1] & 0xffff)));
#pragma unroll
            for (int g = 0; g < G; ++g) dots[g] += kv * sq[g][part * PART + c * 8 + e];
          }
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d2 = dots[g] + __shfl_xor(dots[g], 1, 64);
        d2 += __shfl_xor(d2, 2, 64);
        if (part == 0) sp[g][tid >> 2] = (key < kend) ? d2 : -INFINITY;
      }
    }
    __syncthreads();
    // ---- online softmax per head (one wave per head) ----
    for (int g = wid; g < G; g += 4) {
      const float s = sp[g][lane];
      const float tmax = wave_max(s);
      const float m_old = sm[g];
      const float m_new = fmaxf(m_old, tmax);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float p = exp2f(s - m_use);
      const float psum = wave_sum(p);
      sp[g][lane] = p;
      if (lane == 0) {
        const float a = exp2f(m_old - m_use);
        salpha[g] = a;
        sl[g] = sl[g] * a + psum;
        sm[g] = m_new;
      }
    }
    __syncthreads();
    // ---- PV: thread = (d-pair, key group) ----
    if (kg < KG) {
#pragma unroll
      for (int g = 0; g < G; ++g) { oacc[g][0] *= salpha[g]; oacc[g][1] *= salpha[g]; }
      for (int kk = kg; kk < KT; kk += KG) {
        const int key = kb + kk;
        if (key >= kend) break;
        const unsigned u = *(const unsigned*)(vc + cbase + (size_t)key * D + 2 * dp);
        const float v0 = bf2f((bf16_t)(u & 0xffff)), v1 = bf2f((bf16_t)(u >> 16));
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = sp[g][kk];
          oacc[g][0] += p * v0;
          oacc[g][1] += p * v1;
        }
      }
    }
    __syncthreads();
  }
  // ---- reduce key groups, write partials ----
  if (kg < KG) {
#pragma unroll
    for (int g = 0; g < G; ++g) { sred[kg][g][2 * dp] = oacc[g][0]; sred[kg][g][2 * dp + 1] = oacc[g][1]; }
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < KG; ++j) s += sred[j][g][d];
    const int h = hk * G + g;
    po[(((size_t)b * H + h) * nsplit + split) * D + d] = s;
  }
  if (tid < G) {
    const int h = hk * G + tid;
    pm[((size_t)b * H + h) * nsplit + split] = sm[tid];
    pl[((size_t)b * H + h) * nsplit + split] = sl[tid];
  }
}

template <int D>
__global__ void decode_combine_kernel(const float* __restrict__ po, const float* __restrict__ pm,
                                      const float* __restrict__ pl, int H, int nsplit, bf16_t* __restrict__ o,
                                      int ldo) {
  const int b = blockIdx.y, h = blockIdx.x;
  const size_t base = ((size_t)b * H + h) * nsplit;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, pm[base + s]);
  const float Mu = (M == -INFINITY) ? 0.f : M;
  float lsum = 0.f;
  for (int s = 0; s < nsplit; ++s) lsum += pl[base + s] * exp2f(pm[base + s] - Mu);
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < nsplit; ++s) acc += po[(base + s) * D + d] * exp2f(pm[base + s] - Mu);
    o[(size_t)b * ldo + h * D + d] = f2bf(acc * inv);
  }
}

DA_EXPORT int da_flash_attn_varlen(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv,
                                   const void* cu_seqlens, int B, int max_seqlen, int H, int Hkv, int D, int causal,
                                   float scale, void* o, int ldo, void* stream) {
  if (H % Hkv || ldq % 8 || ldk % 8 || ldv % 8 || ldo % 4) return (int)hipErrorInvalidValue;
  if (B == 0 || max_seqlen == 0) return 0;
  dim3 grid((max_seqlen + 63) / 64, H, B);
  const float sl2e = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
#define FA_ARGS (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, ldq, ldk, ldv, (const int*)cu_seqlens, H, Hkv, \
                causal, sl2e, (bf16_t*)o, ldo
  switch (D) {
    case 64: flash_attn_varlen_kernel<64><<<grid, 256, 0, s>>>(FA_ARGS); break;
    case 96: flash_attn_varlen_kernel<96><<<grid, 256, 0, s>>>(FA_ARGS); break;
    case 128: flash_attn_varlen_kernel<128><<<grid, 256, 0, s>>>(FA_ARGS); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FA_ARGS
  DA_LAUNCH_CHECK();
}

template <int D>
static int launch_decode(int G, dim3 grid, hipStream_t s, const bf16_t* q, int ldq, const bf16_t* kc,
                         const bf16_t* vc, const int* lens, const int* slot, int H, int Hkv, int max_seq, int chunk,
                         int nsplit, float sl2e, float* po, float* pm, float* pl) {
#define DEC(GG) decode_attn_kernel<D, GG><<<grid, 256, 0, s>>>(q, ldq, kc, vc, lens, slot, H, Hkv, max_seq, chunk, \
                                                                nsplit, sl2e, po, pm, pl)
  switch (G) {
    case 1: DEC(1); break;
    case 2: DEC(2); break;
    case 4: DEC(4); break;
    case 8: DEC(8); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef DEC
  return (int)hipGetLastError();
}

// ws must hold B*H*nsplit*(D+2) floats. chunk = keys per split (multiple of 64).
DA_EXPORT int da_decode_attn(const void* q, int ldq, const void* k_cache, const void* v_cache, const void* lens,
                             const void* slot, int B, int H, int Hkv, int D, int max_seq, int chunk, int nsplit,
                             float scale, void* ws, void* o, int ldo, void* stream) {
  if (H % Hkv || chunk % 64 || nsplit < 1 || (long)chunk * nsplit < 1) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const int G = H / Hkv;
  float* po = (float*)ws;
  float* pm = po + (size_t)B * H * nsplit * D;
  float* pl = pm + (size_t)B * H * nsplit;
  dim3 grid(nsplit, Hkv, B);
  const float sl2e = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  int err;
  switch (D) {
    case 64: err = launch_decode<64>(G, grid, s, (const bf16_t*)q, ldq, (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                                     (const int*)lens, (const int*)slot, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl);
      break;
    case 96: err = launch_decode<96>(G, grid, s, (const bf16_t*)q, ldq, (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                                     (const int*)lens, (const int*)slot, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl);
      break;
    case 128: err = launch_decode<128>(G, grid, s, (const bf16_t*)q, ldq, (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                                       (const int*)lens, (const int*)slot, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  if (err) return err;
  dim3 cgrid(H, B);
  switch (D) {
    case 64: decode_combine_kernel<64><<<cgrid, 64, 0, s>>>(po, pm, pl, H, nsplit, (bf16_t*)o, ldo); break;
    case 96: decode_combine_kernel<96><<<cgrid, 128, 0, s>>>(po, pm, pl, H, nsplit, (bf16_t*)o, ldo); break;
    case 128: decode_combine_kernel<128><<<cgrid, 128, 0, s>>>(po, pm, pl, H, nsplit, (bf16_t*)o, ldo); break;
  }
  DA_LAUNCH_CHECK();
}
