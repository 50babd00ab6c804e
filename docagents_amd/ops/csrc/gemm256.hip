// 256x256-tile fp8 GEMM for prefill-sized M (C[M,N] = epi(A[M,K] . W[N,K]^T)): the encoder's fp8
// path (BASELINE config 5). bf16 prefill GEMMs run the phase-split gemm8p.hip kernel, which
// replaced this kernel's bf16 instantiation (1.42-1.51 vs 1.23-1.33 PF/s, profiles/r2).
//
// fp8 (OCP e4m3): the same 128-byte K-step and LDS image (BK = 128 fp8), one
// v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair instead of two bf16 16x16x32 (2x the bf16
// MFMA rate); each lane feeds the same 32 contiguous k-bytes of its A row and W row, so the
// instruction's internal k order pairs them consistently. Dequantisation (per-token activation
// scale x per-output-channel weight scale) is applied to the fp32 accumulators in the epilogue.
//
// MI355X-first structure (cdna_hip_programming.md §5 "glds vs register staging", T1, T2):
//  * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128 x 64 output block
//    (8 x 4 fragments of v_mfma_f32_16x16x32_bf16, 128 accumulator registers).
//  * operands staged global -> LDS with LDS-DMA (`global_load_lds_dwordx4`: 1 KiB per
//    wave-instruction, no VGPR round trip), two 64-KiB stages (A 256x64 + W 256x64 bf16).
//    The LDS image is lane-linear, so the bank-conflict XOR swizzle (16-B chunk c of row r stored
//    at chunk c ^ ((r >> 1) & 7)) is applied on the per-lane SOURCE address and undone on the
//    ds_read_b128 address (rule 21: same involution both sides).
//  * one barrier per K-step: the barrier that publishes stage kt also proves every wave finished
//    reading stage kt-1, so the LDS-DMA for tile kt+1 is issued right after it and flies under the
//    64 MFMAs per wave of tile kt. Fragment reads for the whole K-step are issued BEFORE the DMA so
//    the compiler never has to order a ds_read behind a pending LDS-DMA.
//  * bijective XCD remap + grouped-M tile order (L2 reuse of A panels / W panels per XCD).
//  * epilogue: bias / GELU / SwiGLU applied in registers, bf16 tile staged through LDS, then
//    16-B coalesced row stores with the residual add fused.
#include "gemm.h"

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* gptr_t;

namespace {
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;  // 64 KiB
constexpr int TM = 128, TN = 64;                      // per-wave output block
constexpr int SROW = TN * 2 + 16;                     // staging row stride (bytes)
constexpr int STAGING = 8 * TM * SROW;                // 144 KiB
constexpr int SMEM = (2 * STAGE > STAGING) ? 2 * STAGE : STAGING;
}  // namespace

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

template <int EPI, int FP8>
__global__ void __launch_bounds__(512)
gemm256_kernel(GemmArgs p) {
  constexpr int ES = FP8 ? 1 : 2;  // bytes per element
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA bases (M0) stay scalar
  const int wm = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fg = lane >> 4;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, ntm * ntn);
  constexpr int GROUP = 4;
  const int gid = t / (GROUP * ntn);
  const int first_m = gid * GROUP;
  const int gsz = min(ntm - first_m, GROUP);
  const int tin = t % (GROUP * ntn);
  const int m0 = (first_m + tin % gsz) * BM, n0 = (tin / gsz) * BN;

  // ---- per-lane LDS-DMA source pointers (rows clamped into range; clamped rows only feed
  //      outputs that are never stored) ----
  const char* asrc[4];
  const char* bsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wid * 4 + j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz(r);
    asrc[j] = (const char*)p.A + ((size_t)min(m0 + r, p.M - 1) * p.lda) * ES + c * 16;
    bsrc[j] = (const char*)p.W + ((size_t)min(n0 + r, p.N - 1) * p.K) * ES + c * 16;
  }
  auto issue = [&](int kt, int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(asrc[j] + kt * 128), (lds_ptr_t)(sa + (wid * 4 + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(bsrc[j] + kt * 128), (lds_ptr_t)(sb + (wid * 4 + j) * 1024), 16, 0, 0);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  {
  const int nk = p.K * ES / 128;  // 128-byte K-steps (64 bf16 or 128 fp8)
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();  // vmcnt(0) + barrier: stage kt landed for every wave; stage kt-1 fully read
    const char* sa = smem + (kt & 1) * STAGE;
    const char* sb = sa + A_BYTES;
    bf16x8_t af[2][8], bfr[2][4];
    auto read_frags = [&](int kk) {
      const int c = FP8 ? 2 * fg + kk : kk * 4 + fg;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = wm * TM + i * 16 + fr;
        af[kk][i] = *(const bf16x8_t*)(sa + r * 128 + ((c ^ swz(r)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * TN + j * 16 + fr;
        bfr[kk][j] = *(const bf16x8_t*)(sb + r * 128 + ((c ^ swz(r)) << 4));
      }
    };
    // DMA for the next stage first (branch-free: the last K-step re-stages tile nk-1 into the idle
    // buffer), so it gets the whole K-step of MFMAs to land; then all 24 fragment reads, then the
    // 64 MFMAs (measured on MI355X: ~+3 % over reads-first / compiler-interleaved orders,
    // profiles/gemm256_sched_variants_r1.txt).
    issue(min(kt + 1, nk - 1), (kt + 1) & 1);
    __builtin_amdgcn_sched_barrier(0);
    read_frags(0);
    read_frags(1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (FP8) {
      // lane group fg owns k-bytes 32fg..32fg+31 = chunks 2fg, 2fg+1 (read as "k-halves" 0 and 1
      // by read_frags with c = kk*4 + fg -> re-read here with the fp8 chunk pairing)
      typedef __attribute__((ext_vector_type(8))) int i32x8_t;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const i32x8_t a8 = __builtin_bit_cast(i32x8_t, __builtin_shufflevector(af[0][i], af[1][i], 0, 1, 2, 3, 4, 5, 6, 7,
                                                                                  8, 9, 10, 11, 12, 13, 14, 15));
          const i32x8_t b8 = __builtin_bit_cast(i32x8_t, __builtin_shufflevector(bfr[0][j], bfr[1][j], 0, 1, 2, 3, 4, 5, 6, 7,
                                                                                  8, 9, 10, 11, 12, 13, 14, 15));
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc[i][j], 0, 0, 0, 127, 0, 127);
        }
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[kk][i], bfr[kk][j], acc[i][j]);
    }
  }
  }
  __syncthreads();

  // ---- epilogue: registers -> (bias / GELU / SwiGLU) -> bf16 staging -> coalesced stores ----
  char* st = smem + wid * TM * SROW;
  const int row0 = m0 + wm * TM, col0 = n0 + wn * TN;
  if constexpr (FP8) {
    float swv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) swv[j] = p.sw[min(col0 + j * 16 + fr, p.N - 1)];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float sav = p.sa[min(row0 + i * 16 + fg * 4 + q, p.M - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j][q] *= sav * swv[j];
      }
  }
  if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int pq = 0; pq < 2; ++pq)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = silu(acc[i][2 * pq][q]) * acc[i][2 * pq + 1][q];
          *(bf16_t*)(st + (i * 16 + fg * 4 + q) * SROW + (pq * 16 + fr) * 2) = f2bf(v);
        }
  } else {
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int gc = col0 + j * 16 + fr;
        bv[j] = gc < p.N ? bf2f(p.bias[gc]) : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = acc[i][j][q] + bv[j];
          if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
          *(bf16_t*)(st + (i * 16 + fg * 4 + q) * SROW + (j * 16 + fr) * 2) = f2bf(v);
        }
  }
  __syncthreads();
  constexpr int OC = (EPI == EPI_SWIGLU) ? TN / 2 : TN;  // output columns of this wave
  constexpr int CPR = OC / 8;                            // 16-B chunks per staged row
  constexpr int RPI = 64 / CPR;
  const int cc = (lane % CPR) * 8;
  const int gcol = ((EPI == EPI_SWIGLU) ? col0 / 2 : col0) + cc;
  const int ncols = (EPI == EPI_SWIGLU) ? p.N / 2 : p.N;
  for (int rr = lane / CPR; rr < TM; rr += RPI) {
    const int gm = row0 + rr;
    if (gm >= p.M || gcol >= ncols) continue;
    u32x4_t v = *(const u32x4_t*)(st + rr * SROW + cc * 2);
    if constexpr (EPI == EPI_RESID) {
      const u32x4_t r = *(const u32x4_t*)(p.resid + (size_t)gm * p.ldr + gcol);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = bf2f((bf16_t)(v[e] & 0xffff)) + bf2f((bf16_t)(r[e] & 0xffff));
        const float hi = bf2f((bf16_t)(v[e] >> 16)) + bf2f((bf16_t)(r[e] >> 16));
        v[e] = pack_bf2(lo, hi);
      }
    }
    *(u32x4_t*)(p.C + (size_t)gm * p.ldc + gcol) = v;
  }
}

template <int FP8>
static int launch256(const GemmArgs& a, int epi, hipStream_t s, dim3 grid, dim3 block) {
  switch (epi) {
    case EPI_NONE: gemm256_kernel<EPI_NONE, FP8><<<grid, block, 0, s>>>(a); break;
    case EPI_BIAS: gemm256_kernel<EPI_BIAS, FP8><<<grid, block, 0, s>>>(a); break;
    case EPI_GELU: gemm256_kernel<EPI_GELU, FP8><<<grid, block, 0, s>>>(a); break;
    case EPI_SWIGLU: gemm256_kernel<EPI_SWIGLU, FP8><<<grid, block, 0, s>>>(a); break;
    case EPI_RESID: gemm256_kernel<EPI_RESID, FP8><<<grid, block, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

int launch_gemm256(const GemmArgs& a, int epi, hipStream_t s, int fp8) {
  if (!fp8) return (int)hipErrorInvalidValue;  // bf16: gemm8p
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn), block(512);
  return launch256<1>(a, epi, s, grid, block);
}

// fp8 GEMM entry: A [M, lda] e4m3 (row-major), W [N, K] e4m3, sa [M], sw [N] fp32 dequant scales.
DA_EXPORT int da_gemm_fp8(const void* A, int lda, const void* W, const void* sa, const void* sw, void* C, int ldc,
                          const void* bias, const void* resid, int ldr, int M, int N, int K, int epi, void* stream) {
  if (K % 128 || N % 8 || lda % 16 || ldc % 8 || !sa || !sw) return (int)hipErrorInvalidValue;
  if (epi == EPI_SWIGLU && N % 32) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = (const bf16_t*)bias; a.resid = (const bf16_t*)resid; a.ws = nullptr;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldc = ldc; a.ldr = ldr; a.k_per_split = K;
  a.sa = (const float*)sa; a.sw = (const float*)sw;
  return launch_gemm256(a, epi, (hipStream_t)stream, 1);
}
