// Shared GEMM declarations (epilogue codes and launch arguments).
#pragma once
#include "common.h"

enum Epi : int {
  EPI_NONE = 0,
  EPI_BIAS = 1,
  EPI_GELU = 2,       // bias (optional) + exact GELU (BERT)
  EPI_SWIGLU = 3,     // W rows interleaved in 16-row (gate, up) groups; out N/2 = silu(g)*u
  EPI_RESID = 4,      // bias (optional) + residual add
  EPI_PARTIAL = 5,    // fp32 split-K partial to workspace
};

struct GemmArgs {
  const bf16_t* A; const bf16_t* W; bf16_t* C;
  const bf16_t* bias; const bf16_t* resid; float* ws;
  int M, N, K, lda, ldc, ldr, k_per_split;
  const float* sa; const float* sw;  // fp8 path: per-row (A) and per-output-channel (W) scales
  const bf16_t* gamma; float eps;    // GEMV only: fused RMSNorm of the input row (gamma != null)
};

// large-tile (256x256, 8 waves, LDS-DMA staged) path; returns hipError_t.
// fp8 = 1: A and W hold OCP e4m3 bytes (lda / K in elements = bytes), C = (A.W^T) * sa[m] * sw[n].
int launch_gemm256(const GemmArgs& a, int epi, hipStream_t s, int fp8 = 0);
// 4-wave 256x256 bf16 variant (gemm256w4.hip); K % 32 == 0
int launch_gemm256w4(const GemmArgs& a, int epi, hipStream_t s);
// phase-split 256x256 bf16 kernel (gemm8p.hip); K % 64 == 0, K >= 128
int launch_gemm8p(const GemmArgs& a, int epi, hipStream_t s);
