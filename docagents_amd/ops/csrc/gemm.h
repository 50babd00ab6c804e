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
  EPI_ROPE = 6,       // QKV projection: RoPE (interleaved pairs) on q / k, k / v written to the KV cache
};

// EPI_ROPE operands: output columns [H q heads | Hkv k heads | Hkv v heads] of D; token row m goes to
// cache slot slot[m] at position pos[m] (caches [slots, Hkv, max_seq, D]); cs = [max_pos, D/2, 2].
struct RopeArgs {
  const int* pos; const int* slot; const float* cs;
  bf16_t* kc; bf16_t* vc;
  int H, Hkv, D, max_seq;
  int kv_out;  // 1: k / v columns also stored in C; 0: cache only (attention reads the cache)
};

struct GemmArgs {
  const bf16_t* A; const bf16_t* W; bf16_t* C;
  const bf16_t* bias; const bf16_t* resid; float* ws;
  int M, N, K, lda, ldc, ldr, k_per_split;
  const float* sa; const float* sw;  // fp8 path: per-row (A) and per-output-channel (W) scales
  const bf16_t* gamma; float eps;    // GEMV only: fused RMSNorm of the input row (gamma != null)
  RopeArgs rope;                     // EPI_ROPE only
  int group;  // gemm8p: row tiles per grouped-M band of the tile order (0: the default, 4)
};

// 256x256 fp8 tile (gemm256.hip): A and W hold OCP e4m3 bytes (lda / K in elements = bytes),
// C = (A.W^T) * sa[m] * sw[n]; returns hipError_t.
int launch_gemm256(const GemmArgs& a, int epi, hipStream_t s, int fp8 = 1);
// phase-split BMx256 bf16 kernel (gemm8p.hip), bm = 256 or 128; K % 64 == 0, K >= 128
int launch_gemm8p(const GemmArgs& a, int epi, hipStream_t s, int bm = 256);
// four-wave 256x256 kernel (gemm4w.hip, 128x128 per wave; the tile-13 A/B arm), bf16, no EPI_ROPE
int launch_gemm4w(const GemmArgs& a, int epi, hipStream_t s);
// row-tile height (128 / 256) for a non-RoPE prefill product of M x N (gemm8p.hip)
int gemm8p_pick_bm(int M, int N);
