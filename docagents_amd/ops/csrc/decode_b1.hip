// Batch-1 decode of a range of decoder layers as ONE persistent launch (MHA models: Phi-3-mini).
//
// The batch-1 step (the p50 cache-miss latency path) was 5 launches per layer — QKV GEMV with the
// input RMSNorm fused, decode attention (RoPE + new-token KV write fused, split-KV with in-kernel
// merge), O GEMV + residual, gate/up GEMV + SwiGLU with the norm fused, down GEMV + residual —
// each paying a kernel boundary plus a ramp in which its first weight bytes are still in flight
// (profiles/r3/check6: ~58 us per layer for 262 MB, ~4.5 TB/s). Here one launch runs every phase of
// every layer, and the seams between phases become counters in device memory:
//
//   P1 QKV      item = 12 rows (4 waves x 3)      publishes qkv rows, bumps head_cnt[head]
//   P2 attn     item = (head, split)              waits head_cnt[h]; last split merges, bumps heads
//   P3 O + x    item = 12 rows                    waits heads == H;  bumps o_cnt (per-XCD shards)
//   P4 gate/up  item = 16 rows (8 gate + 8 up)    waits o_cnt;       bumps gu_cnt
//   P5 down + x item = 4 rows (K split over 2 waves) waits gu_cnt;   bumps dn_cnt (next layer's P1)
//   P6 LM head  item = 16 rows (optional)         waits dn_cnt of the last layer
//
// What a seam costs instead of a launch: every item issues its WEIGHT loads (and an attention
// item its K/V-cache tile loads: none of them depend on this step's activations) BEFORE it waits
// for its input, so the next phase's first bytes are in flight while the previous phase drains —
// the prefetch credit of cdna_hip_programming.md §5.6 — and no phase starts from an empty pipe.
//
// Hand-off protocol (cdna_hip_programming.md §6 Guideline 16, table row 1 of MI355X_MICROARCH.md
// § visibility): every handed-off byte (qkv, attention output, residual rows, SwiGLU output,
// split partials) is STORED sc1 (write-through) and LOADED sc1 (global / buffer loads with the sc1
// bit, never flat or scalar), in 4-, 8- or 16-B granules only — the sizes that row was measured
// with — and each granule by ONE writer: a GEMV item's rows are gathered in LDS and leave as 8-B
// words, an attention head's row as 16-B chunks, and 16-bit values are read as the 4-B word that
// holds them (2-B sc1 stores from several workgroups into one line diverged after ~20 sampled
// steps on the MI355X); every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup
// barrier behind which ONE lane bumps the counter (agent-scope relaxed atomic add); ONE wave polls
// the counter relaxed with s_sleep, then the workgroup barrier. One workgroup per CU (occupancy 1). Counters are
// cumulative over the launch (target = items x (layer + 1)); the LAST workgroup to leave (an exit
// ticket every workgroup takes after its final counter access) zeroes them for the next launch.
// (A memset ahead of the launch is not enough under HIP-graph replay: measured, the second replay
// started from the first one's counters, every wait passed at once and read stale rows.) Every
// spin is bounded: a timeout sets the error word, every workgroup still takes its exit ticket, and
// the host raises (decode_b1_error) instead of hanging the GPU.
//
// Numerics: each output element is computed by the same per-lane fp32 FMA sequence and wave
// reduction as the separate kernels (gemm.hip gemv_kernel, attention.hip decode_attn_kernel
// <D, 1, 7>), so the two paths produce bit-identical tokens (tests/test_decode_b1_gpu.py).
//
// Residency: the workgroups wait on each other, so every one of them must be resident at once:
// the launcher sizes the grid as (CUs the stream may use) x (resident workgroups per CU from the
// occupancy query). Other streams' kernels only delay residency (they never wait on this one).
#include "gemm.h"

// Floating-point contraction only within one expression (a*b + c -> fma), never across statements:
// with the HIP default (fast) the backend fuses differently depending on the surrounding code, and
// the decode attention inlined into the persistent batch-1 kernel (decode_b1.hip) then differed from
// decode_attn_kernel by one bf16 ulp on some heads (measured on the MI355X, bench/b1_diverge.py).
// Both files pin the same rule, so the two compute the same bits by construction.
#pragma clang fp contract(on)

namespace {

constexpr int B1_NT = 256;          // threads per workgroup (4 waves)
constexpr int CL = 32;              // words per counter line (128 B): one counter per line
constexpr unsigned SPIN_LIMIT = 1u << 21;  // polls of ~1 us: a wait gives up after a few seconds

// sync block layout (unsigned words, each counter on its own 128-B line)
enum : int { S_ERR = 0, S_EXIT = 1, S_HEADS = 2, S_O = 3, S_GU = 11, S_DN = 19, S_HEAD = 27 };  // x CL words
// S_HEAD + h: qkv items published for head h; S_HEAD + H + h: split tickets of head h

struct B1Layer {
  const bf16_t* wqkv;  // [3 Hd, Hd] (norm gain folded)
  const bf16_t* wo;    // [Hd, Hd]
  const bf16_t* wgu;   // [2 F, Hd] gate/up interleaved in 16-row groups (norm gain folded)
  const bf16_t* wdown; // [Hd, F]
  bf16_t* kc;          // this layer's caches [slots, H, max_seq, D]
  bf16_t* vc;
};

struct B1Args {
  const B1Layer* layers;
  int l0, l1;
  bf16_t* x;           // [Hd] residual stream (in: embedding of the token; out: after layer l1 - 1)
  bf16_t* qkv;         // [3 Hd]
  bf16_t* attn;        // [Hd]
  bf16_t* act;         // [F]
  const int* lens; const int* slot; const int* pre; const int* pos; const float* cs;
  int Hd, H, F, max_seq, nsplit, chunk;
  float eps, sl2e;
  float* po; float* pm; float* pl;  // split partials [H][nsplit][D], [H][nsplit]
  unsigned* sync;
  const bf16_t* lm_head; bf16_t* logits; int V;  // optional P6
};

// ------------------------------------------------------------------ coherent accesses
__device__ __forceinline__ unsigned ld_u32(const unsigned* p) {
  return __hip_atomic_load((unsigned*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_f32(const float* p) { return __uint_as_float(ld_u32((const unsigned*)p)); }
__device__ __forceinline__ unsigned long long ld_u64(const void* p) {
  return __hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the two bf16 of the 4-B word holding element i (i even: low half)
__device__ __forceinline__ unsigned ld_pair(const bf16_t* row, int i) { return ld_u32((const unsigned*)(row + (i & ~1))); }
__device__ __forceinline__ bf16_t lo16(unsigned w) { return (bf16_t)(w & 0xffff); }
__device__ __forceinline__ bf16_t hi16(unsigned w) { return (bf16_t)(w >> 16); }
__device__ __forceinline__ void st_u32(void* p, unsigned v) {
  __hip_atomic_store((unsigned*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_f32(float* p, float v) { st_u32(p, __float_as_uint(v)); }
__device__ __forceinline__ void st_u64(void* p, unsigned long long v) {
  __hip_atomic_store((unsigned long long*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// four fp32 results -> four bf16 in one 8-B word (element 0 lowest)
__device__ __forceinline__ unsigned long long pack4(float a, float b, float c, float d) {
  return (unsigned long long)pack_bf2(a, b) | ((unsigned long long)pack_bf2(c, d) << 32);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
// 16 B of handed-off data, sc1 (aux 16): bypasses this CU's L1, which other CUs' stores never refresh
__device__ __forceinline__ u32x4_t ld16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4_t v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

__device__ __forceinline__ unsigned wave_sum_u(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (unsigned)__shfl_xor((int)v, o, 64);
  return v;
}

// Publish this workgroup's items: every storing wave drains its sc1 stores, then ONE lane adds.
__device__ __forceinline__ void publish(unsigned* ctr, unsigned n) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && n) __hip_atomic_fetch_add(ctr, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until the sum of `nsh` counter shards reaches `target`: wave 0 polls (lane i reads shard i),
// the others wait at the barrier. Returns false when the launch is aborting (timeout here or
// elsewhere): the caller leaves the kernel.
__device__ __forceinline__ bool wait_ge(unsigned* sync, int ctr_line, int nsh, unsigned target, unsigned code) {
  __shared__ int s_ok;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned* ctr = sync + ctr_line * CL;
    bool ok = true;
    for (unsigned spins = 0;; ++spins) {
      const unsigned v = wave_sum_u(lane < nsh ? ld_u32(ctr + lane * CL) : 0u);
      if (v >= target) break;
      if (ld_u32(sync + S_ERR * CL) != 0u) { ok = false; break; }
      if (spins > SPIN_LIMIT) {
        if (lane == 0) st_u32(sync + S_ERR * CL, code);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) s_ok = ok;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no load of handed-off data above the poll
  return s_ok;
}

// ------------------------------------------------------------------ GEMV item
// gemm.hip gemv_kernel's body for one 4-wave gate/up + SwiGLU item (vb), with (1) the first round's
// weight loads issued before `wait` (the phase dependency) and (2) the activation load and the
// output store coherent (sc1). Same per-lane FMA order and wave reduction as gemv_kernel. Each wave
// owns 2 gate + 2 up rows -> 2 adjacent outputs: one 4-B word, one writer.
template <int EPI, int R, int U, int KS, typename Wait>
__device__ __forceinline__ bool gemv_item(const bf16_t* A, const bf16_t* W, bf16_t* C, const bf16_t* resid, int N,
                                          int K, float eps, int vb, Wait&& wait) {
  static_assert(EPI == EPI_SWIGLU && R == 4, "the gate/up phase: 2 gate + 2 up rows per wave");
  const int lane = threadIdx.x & 63;
  const int wv = vb * 4 + (threadIdx.x >> 6);
  const int wg = wv / KS, ks = wv % KS;
  int rows[R];
  {
    const int g = wg >> 3, t = wg & 7;
#pragma unroll
    for (int r = 0; r < R; ++r) rows[r] = g * 32 + 2 * t + (r & 1) + (r >> 1) * 16;
  }
  const bf16_t* wr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = W + (size_t)min(rows[r], N - 1) * K + lane * 8;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A, K * 2);
  const bool rms = eps > 0.f;
  const int nkb = K / 512;
  const int kb0 = ks * nkb / KS, kb1 = (ks + 1) * nkb / KS;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  float ss = 0.f;
  bool first = true;
  for (int kb = kb0; kb < kb1; kb += U) {
    u32x4_t wvv[U][R], av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(kb + u, kb1 - 1) * 512;
#pragma unroll
      for (int r = 0; r < R; ++r) wvv[u][r] = __builtin_nontemporal_load((const u32x4_t*)(wr[r] + k));
    }
    if (first) {  // the weights are in flight; now the input this item depends on
      first = false;
      if (!wait()) return false;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(kb + u, kb1 - 1) * 512;
      av[u] = ld16_sc1(ra, (unsigned)(k + lane * 8) * 2u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (kb + u >= kb1) break;
      float a[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[2 * e] = bf2f((bf16_t)(av[u][e] & 0xffff));
        a[2 * e + 1] = bf2f((bf16_t)(av[u][e] >> 16));
      }
      if (rms) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ss = fmaf(a[2 * e], a[2 * e], fmaf(a[2 * e + 1], a[2 * e + 1], ss));
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[r] = fmaf(bf2f((bf16_t)(wvv[u][r][e] & 0xffff)), a[2 * e], acc[r]);
          acc[r] = fmaf(bf2f((bf16_t)(wvv[u][r][e] >> 16)), a[2 * e + 1], acc[r]);
        }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (rms) ss = wave_sum(ss);
  bool lead = true;
  if constexpr (KS == 2) {
    __shared__ float xch[4][R + 1];
    const int w = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) xch[w][r] = acc[r];
      xch[w][R] = ss;
    }
    __syncthreads();
    lead = ks == 0;
    if (lead) {
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] += xch[w + 1][r];
      ss += xch[w + 1][R];
    }
    __syncthreads();  // xch is reused by the next item
  }
  if (rms) {
    const float inv = rsqrtf(ss / K + eps);
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] *= inv;
  }
  if (lane != 0 || !lead) return true;
  const int g = wg >> 3, t = wg & 7;
  const int o = g * 16 + 2 * t;  // two adjacent outputs: one 4-B store
  if (o < N / 2) st_u32(C + o, pack_bf2(silu(acc[0]) * acc[2], silu(acc[1]) * acc[3]));
  return true;
}

// All of this workgroup's items of one GEMV phase (vb = vb0, vb0 + stride, ...), software-pipelined:
// the activation row (the same for every item of the phase) is loaded ONCE, after `wait`; each
// item's weights are requested one item ahead (two register buffers), so the next item's weight
// stream is in flight while this one's FMAs and stores run — the seam of gemv_item, where every
// item starts from an empty pipe, happens once per phase instead of once per item. Needs one load
// round per item: (K / 512) / KS == U. Same per-row FMA order and reductions as gemv_kernel.
// EPI_NONE / EPI_RESID: the item's NR = 4 R / KS contiguous rows are gathered in LDS (two buffers:
// item parity) and lane 0 of wave 0 writes them as NR / 4 8-B words (RESID: after adding the
// residual rows it reads the same way; resid may alias C) — N % NR == 0 (host-checked).
template <int EPI, int R, int U, int KS, typename Wait, typename After>
__device__ __forceinline__ bool gemv_phase(const bf16_t* A, const bf16_t* W, bf16_t* C, const bf16_t* resid, int N,
                                           int K, float eps, int vb0, int stride, int nvb, Wait&& wait,
                                           After&& after) {
  static_assert(EPI == EPI_NONE || EPI == EPI_RESID, "row outputs (the SwiGLU phase uses gemv_item)");
  constexpr int NR = 4 / KS * R;  // rows per item
  static_assert(NR % 4 == 0, "8-B output words");
  __shared__ float s_out[2][NR];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ks = KS == 2 ? (w & 1) : 0;
  const int kb0 = ks * U;  // (K / 512) == KS * U (host-checked)
  if (nvb <= 0) return true;
  auto rows_of = [&](int vb, int (&rows)[R]) {
    const int wg = (vb * 4 + w) / KS;
#pragma unroll
    for (int r = 0; r < R; ++r) rows[r] = wg * R + r;
  };
  auto issue = [&](int vb, u32x4_t (&wv)[U][R]) {
    int rows[R];
    rows_of(vb, rows);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bf16_t* wr = W + (size_t)min(rows[r], N - 1) * K + kb0 * 512 + lane * 8;
#pragma unroll
      for (int u = 0; u < U; ++u) wv[u][r] = __builtin_nontemporal_load((const u32x4_t*)(wr + u * 512));
    }
  };
  u32x4_t wa[U][R], wb[U][R], av[U];
  issue(vb0, wa);
  if (!wait()) return false;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A, K * 2);
#pragma unroll
  for (int u = 0; u < U; ++u) av[u] = ld16_sc1(ra, (unsigned)((kb0 + u) * 512 + lane * 8) * 2u);
  const bool rms = eps > 0.f;
  auto finish = [&](int vb, int par, const u32x4_t (&wv)[U][R]) {
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.f;
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float a[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[2 * e] = bf2f((bf16_t)(av[u][e] & 0xffff));
        a[2 * e + 1] = bf2f((bf16_t)(av[u][e] >> 16));
      }
      if (rms) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ss = fmaf(a[2 * e], a[2 * e], fmaf(a[2 * e + 1], a[2 * e + 1], ss));
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[r] = fmaf(bf2f((bf16_t)(wv[u][r][e] & 0xffff)), a[2 * e], acc[r]);
          acc[r] = fmaf(bf2f((bf16_t)(wv[u][r][e] >> 16)), a[2 * e + 1], acc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
    if (rms) ss = wave_sum(ss);
    bool lead = true;
    if constexpr (KS == 2) {
      __shared__ float xch[4][R + 1];
      if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) xch[w][r] = acc[r];
        xch[w][R] = ss;
      }
      __syncthreads();
      lead = ks == 0;
      if (lead) {
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] += xch[w + 1][r];
        ss += xch[w + 1][R];
      }
      __syncthreads();
    }
    if (rms) {
      const float inv = rsqrtf(ss / K + eps);
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] *= inv;
    }
    if (lane == 0 && lead) {
#pragma unroll
      for (int r = 0; r < R; ++r) s_out[par][(w / KS) * R + r] = acc[r];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int row0 = vb * NR;
      if (row0 < N) {
#pragma unroll
        for (int c = 0; c < NR; c += 4) {
          float v[4] = {s_out[par][c], s_out[par][c + 1], s_out[par][c + 2], s_out[par][c + 3]};
          if constexpr (EPI == EPI_RESID) {
            const unsigned long long rr = ld_u64(resid + row0 + c);
            const unsigned r0 = (unsigned)rr, r1 = (unsigned)(rr >> 32);
            v[0] += bf2f(lo16(r0)); v[1] += bf2f(hi16(r0)); v[2] += bf2f(lo16(r1)); v[3] += bf2f(hi16(r1));
          }
          st_u64(C + row0 + c, pack4(v[0], v[1], v[2], v[3]));
        }
      }
    }
  };
  for (int i = 0; i < nvb; i += 2) {
    if (i + 1 < nvb) issue(vb0 + (i + 1) * stride, wb);
    finish(vb0 + i * stride, 0, wa);
    after(vb0 + i * stride);
    if (i + 1 >= nvb) break;
    if (i + 2 < nvb) issue(vb0 + (i + 2) * stride, wa);
    finish(vb0 + (i + 1) * stride, 1, wb);
    after(vb0 + (i + 1) * stride);
  }
  return true;
}

// Rows per wave of the QKV / O items: 3 (12-row items) where the head width allows it — the Phi-3
// QKV projection is then 768 items = exactly 3 per workgroup on 256 CUs and the O projection 256 =
// one each (16-row items left a 2.25-item imbalance); 4 otherwise (items must not straddle heads).
template <int D>
struct B1Rows {
  static constexpr int RQ = (D % 12 == 0) ? 3 : 4;
};

// ------------------------------------------------------------------ attention item (MHA, G = 1)
// attention.hip decode_attn_kernel<D, 1, 7> (non-temporal K/V, V with K, next tile prefetched)
// for (head hk, split) of row 0, with the K/V tile loads issued BEFORE waiting for this step's q /
// new k / new v (they come from P1 of this launch: loaded sc1 after the wait). The split's partial
// goes out sc1; the last split of the head (cumulative ticket) merges them with sc1 loads and
// publishes the head's attention row.
__device__ __forceinline__ int b1_chunk(int L, int nsplit, int chunk_arg) {
  const int c = ((L + nsplit - 1) / nsplit + 63) & ~63;
  return c < chunk_arg ? c : chunk_arg;
}

template <int D>
__device__ __forceinline__ bool attn_item(const B1Args& a, const B1Layer& Ly, int hk, int split, int layer_i) {
  constexpr int KT = 64;
  constexpr int CPR = D / 8;
  constexpr int GCD = (CPR % 16 == 0) ? 16 : ((CPR % 8 == 0) ? 8 : ((CPR % 4 == 0) ? 4 : 2));
  constexpr int NSET = CPR / GCD;
  constexpr bool SHFL = (64 % CPR) == 0;
  static_assert(D <= 256, "one q element per thread");
  __shared__ float sq[D];
  __shared__ float sp[4][KT];
  __shared__ float spart[SHFL ? 1 : 4][SHFL ? 1 : KT * CPR];
  __shared__ float sacc[4 * NSET * 64 * 8];
  __shared__ float swm[4], swl[4];
  __shared__ float skn[D], svn[D], ssn;
  __shared__ int s_last;
  __shared__ __attribute__((aligned(16))) bf16_t s_ao[D];  // the head's output row, leaves as 16-B chunks
  static_assert(D % 8 == 0 && D / 8 <= B1_NT, "16-B chunks of a head row");
  const __amdgpu_buffer_rsrc_t r_attn = rsrc(a.attn + hk * D, D * 2);
  auto store_head = [&]() {  // s_ao written by threads d < D; one writer per 16-B chunk
    __syncthreads();
    if (threadIdx.x < D / 8) st16_sc1(r_attn, threadIdx.x * 16u, *(const u32x4_t*)&s_ao[threadIdx.x * 8]);
  };

  const int H = a.H, nsplit = a.nsplit, max_seq = a.max_seq;
  const int L = a.lens[0];
  DA_ASSERT(L >= 1 && L <= max_seq && a.slot[0] >= 0 && a.pos[0] == L - 1);
  const int chunk = b1_chunk(L, nsplit, a.chunk);
  const int kstart = split * chunk;
  const bool own_new = kstart <= L - 1 && L - 1 < kstart + chunk;
  const int kend = min(L - 1, kstart + chunk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const size_t cbase = ((size_t)a.slot[0] * H + hk) * (size_t)max_seq * D;
  const int P = a.pre ? a.pre[0] : 0;
  const size_t pbase = P ? ((size_t)a.pre[1] * H + hk) * (size_t)max_seq * D : cbase;
  DA_ASSERT(P % 64 == 0 && P <= L);
  const bf16_t* kc = Ly.kc;
  const bf16_t* vc = Ly.vc;
  auto ld16 = [&](const bf16_t* p) -> u32x4_t { return __builtin_nontemporal_load((const u32x4_t*)p); };
  auto tile_base = [&](const bf16_t* c, int t0) { return c + (t0 < P ? pbase : cbase) + (size_t)t0 * D; };
  auto load_kv = [&](u32x4_t (&kv)[CPR], const bf16_t* c, int t0) {
    const int nk = kend - t0;
    const int last = min(KT, nk) * CPR - 1;
    const bf16_t* kb = tile_base(c, t0);
#pragma unroll
    for (int i = 0; i < CPR; ++i) {
      const int cc = i * 64 + lane;
      kv[i] = ld16(nk > 0 ? kb + min(cc, last) * 8 : c + cbase);
    }
  };
  constexpr int HALF = D / 2;
  auto rot2 = [&](float x1, float x2, float c, float sn, int d) -> float {
    return bf2f(f2bf((d & 1) ? x2 * c + x1 * sn : x1 * c - x2 * sn));
  };
  // 1) this split's first two tiles per wave: independent of the step's activations
  u32x4_t ka[CPR], va[CPR], kb2[CPR], vb2[CPR];
  {
    const int t0 = kstart + w * KT, t1 = t0 + 4 * KT;
    load_kv(ka, kc, t0); load_kv(va, vc, t0);
    load_kv(kb2, kc, t1); load_kv(vb2, vc, t1);
  }
  // 2) q / new k / new v of head hk are P1 output of this launch
  constexpr int IQ = 4 * B1Rows<D>::RQ;
  if (!wait_ge(a.sync, S_HEAD + hk, 1, (unsigned)(3 * D / IQ) * (layer_i + 1), 0x100u + hk)) return false;
  {
    const bf16_t* row = a.qkv;
    const int qi = min(tid, D - 1), d = qi;
    const bf16_t* hp = row + hk * D;
    const unsigned wq = ld_pair(hp, d);
    const bf16_t rq1 = lo16(wq), rq2 = hi16(wq);
    const float* csp = a.cs + ((size_t)(L - 1) * HALF + (d >> 1)) * 2;
    const f32x2_t rcs = *(const f32x2_t*)csp;
    const bf16_t* kr = row + (size_t)(H + hk) * D;
    const bf16_t* vr = row + (size_t)(2 * H + hk) * D;
    const unsigned wk = ld_pair(kr, d), wv = ld_pair(vr, d);
    const bf16_t rk1 = lo16(wk), rk2 = hi16(wk), nv = (d & 1) ? hi16(wv) : lo16(wv);
    const float pc = rcs[0], ps = rcs[1];
    if (tid < D) sq[d] = rot2(bf2f(rq1), bf2f(rq2), pc, ps, d) * a.sl2e;
    if (own_new && tid < D) {
      const size_t crow = cbase + (size_t)(L - 1) * D;
      const float kv = rot2(bf2f(rk1), bf2f(rk2), pc, ps, d);
      skn[d] = kv;
      svn[d] = bf2f(nv);
      Ly.kc[crow + d] = f2bf(kv);  // for later steps (read after this launch)
      Ly.vc[crow + d] = nv;
    }
  }
  __syncthreads();
  if (own_new && w == 0) {
    float part = 0.f;
    for (int d = lane; d < D; d += 64) part += sq[d] * skn[d];
    part = wave_sum(part);
    if (lane == 0) ssn = part;
  }
  float m = -INFINITY, l = 0.f, acc[NSET][8];
#pragma unroll
  for (int s = 0; s < NSET; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[s][e] = 0.f;

  auto process = [&](const u32x4_t (&kv)[CPR], u32x4_t (&vv)[CPR], int t0) {
    const int nk = min(KT, kend - t0);
#pragma unroll
    for (int i = 0; i < CPR; ++i) {
      const int c = i * 64 + lane;
      const int dp = c % CPR;
      float kf[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        kf[2 * e] = bf2f((bf16_t)(kv[i][e] & 0xffff));
        kf[2 * e + 1] = bf2f((bf16_t)(kv[i][e] >> 16));
      }
      const f32x4_t q0 = *(const f32x4_t*)&sq[dp * 8];
      const f32x4_t q1 = *(const f32x4_t*)&sq[dp * 8 + 4];
      float part = kf[0] * q0[0] + kf[1] * q0[1] + kf[2] * q0[2] + kf[3] * q0[3] +
                   kf[4] * q1[0] + kf[5] * q1[1] + kf[6] * q1[2] + kf[7] * q1[3];
      if constexpr (SHFL) {
#pragma unroll
        for (int o = 1; o < CPR; o <<= 1) part += __shfl_xor(part, o, 64);
        if (dp == 0) sp[w][c / CPR] = part;
      } else {
        spart[w][c] = part;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
      float sc;
      if constexpr (SHFL) {
        sc = sp[w][lane];
      } else {
        sc = 0.f;
#pragma unroll
        for (int j = 0; j < CPR; ++j) sc += spart[w][lane * CPR + j];
      }
      if (lane >= nk) sc = -INFINITY;
      const float tmax = wave_max(sc);
      const float m_new = fmaxf(m, tmax);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = exp2f(m - m_use);
      const float p = exp2f(sc - m_use);
      l = l * alpha + wave_sum(p);
      m = m_new;
      sp[w][lane] = p;
#pragma unroll
      for (int st = 0; st < NSET; ++st)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[st][e] *= alpha;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < CPR; ++i) {
      const int c = i * 64 + lane;
      const int key = c / CPR;
      float vf[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        vf[2 * e] = bf2f((bf16_t)(vv[i][e] & 0xffff));
        vf[2 * e + 1] = bf2f((bf16_t)(vv[i][e] >> 16));
      }
      const float pk = sp[w][key];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[i % NSET][e] += pk * vf[e];
    }
    __builtin_amdgcn_wave_barrier();
  };
  {
    int t0 = kstart + w * KT;
    while (t0 < kend) {
      const int t1 = t0 + 4 * KT;
      process(ka, va, t0);
      if (t1 >= kend) break;
      const int t2 = t1 + 4 * KT;
      if (t2 < kend) { load_kv(ka, kc, t2); load_kv(va, vc, t2); }
      process(kb2, vb2, t1);
      if (t2 >= kend) break;
      const int t3 = t2 + 4 * KT;
      if (t3 < kend) { load_kv(kb2, kc, t3); load_kv(vb2, vc, t3); }
      t0 = t2;
    }
  }
  // merge lanes -> per-wave O through LDS (plain 16-B stores), then waves -> this split's partial
#pragma unroll
  for (int st = 0; st < NSET; ++st) {
    float* dst = &sacc[((w * NSET + st) * 64 + lane) * 8];
    *(f32x4_t*)dst = f32x4_t{acc[st][0], acc[st][1], acc[st][2], acc[st][3]};
    *(f32x4_t*)(dst + 4) = f32x4_t{acc[st][4], acc[st][5], acc[st][6], acc[st][7]};
  }
  if (lane == 0) { swm[w] = m; swl[w] = l; }
  __syncthreads();
  const size_t pidx = (size_t)hk * nsplit + split;
  for (int d = tid; d < D; d += B1_NT) {
    float M = fmaxf(fmaxf(swm[0], swm[1]), fmaxf(swm[2], swm[3]));
    if (own_new) M = fmaxf(M, ssn);
    const float Mu = (M == -INFINITY) ? 0.f : M;
    float o = 0.f, ls = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = exp2f(swm[ww] - Mu);
      float ow = 0.f;
      const int dp = d >> 3, e = d & 7;
#pragma unroll
      for (int st = 0; st < NSET; ++st) {
        const int l0 = ((dp - 64 * st) % CPR + CPR) % CPR;
#pragma unroll
        for (int j = 0; j < (64 + CPR - 1) / CPR; ++j) {
          const int ll = l0 + j * CPR;
          if (ll < 64) ow += sacc[((ww * NSET + st) * 64 + ll) * 8 + e];
        }
      }
      o += ow * f;
      ls += swl[ww] * f;
    }
    if (own_new) {
      const float f = exp2f(ssn - Mu);
      o += svn[d] * f;
      ls += f;
    }
    if (nsplit == 1) {
      s_ao[d] = f2bf(ls > 0.f ? o / ls : 0.f);
    } else {
      st_f32(a.po + pidx * D + d, o);
      if (d == 0) { st_f32(a.pm + pidx, M); st_f32(a.pl + pidx, ls); }
    }
  }
  if (nsplit == 1) store_head();
  // this split's partial is out (sc1, drained) -> ticket; the last split of the head merges
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nsplit > 1) {
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.sync + (S_HEAD + H + hk) * CL, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      s_last = (int)(old % (unsigned)nsplit) == nsplit - 1;
    }
    __syncthreads();
    if (!s_last) return true;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int d = tid; d < D; d += B1_NT) {
      const size_t base = (size_t)hk * nsplit;
      float M = -INFINITY, lsum = 0.f, o = 0.f;
      for (int s0 = 0; s0 < nsplit; s0 += 8) {
        float ms[8], ls[8], os[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int s = min(s0 + j, nsplit - 1);
          ms[j] = ld_f32(a.pm + base + s);
          ls[j] = ld_f32(a.pl + base + s);
          os[j] = ld_f32(a.po + (base + s) * D + d);
        }
        float mx = M;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (s0 + j < nsplit) mx = fmaxf(mx, ms[j]);
        const float mu = (mx == -INFINITY) ? 0.f : mx;
        const float r = (M == -INFINITY) ? 0.f : exp2f(M - mu);
        lsum *= r;
        o *= r;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (s0 + j >= nsplit) continue;
          const float f = exp2f(ms[j] - mu);
          lsum += ls[j] * f;
          o += os[j] * f;
        }
        M = mx;
      }
      s_ao[d] = f2bf(lsum > 0.f ? o / lsum : 0.f);
    }
    store_head();
  }
  publish(a.sync + S_HEADS * CL, 1u);
  return true;
}

// ------------------------------------------------------------------ the persistent kernel
template <int D>
__device__ __forceinline__ void b1_run(const B1Args& a) {
  const int G = gridDim.x, wg = blockIdx.x;
  const int Hd = a.Hd, F = a.F, H = a.H;
  unsigned* sync = a.sync;
  const int shard = wg & 7;  // per-XCD shard of the fan-in counters (dispatch round-robins XCDs)
  constexpr int RQ = B1Rows<D>::RQ, IQ = 4 * RQ;  // rows per wave / per item (QKV and O)
  // items per phase
  const int nq = 3 * Hd / IQ, no = Hd / IQ, ngu = 2 * F / 16, ndn = Hd / 4, na = H * a.nsplit;
  for (int li = a.l0; li < a.l1; ++li) {
    const B1Layer Ly = a.layers[li];
    const int lr = li - a.l0;  // layer index within this launch: counters are per launch
    // P1: QKV (input RMSNorm fused; gain folded into the weights); each item publishes its head
    auto nitems = [&](int n) { return wg < n ? (n - wg + G - 1) / G : 0; };
    auto none = [](int) {};
    if (!gemv_phase<EPI_NONE, RQ, 6, 1>(
            a.x, Ly.wqkv, a.qkv, nullptr, 3 * Hd, Hd, a.eps, wg, G, nitems(nq),
            [&]() { return lr == 0 || wait_ge(sync, S_DN, 8, (unsigned)ndn * lr, 0x200u + li); },
            [&](int vb) { publish(sync + (S_HEAD + ((vb * IQ) % Hd) / D) * CL, 1u); }))
      return;
    // P2: attention (head, split) items; each waits for its own head only
    for (int it = wg; it < na; it += G) {
      if (!attn_item<D>(a, Ly, it / a.nsplit, it % a.nsplit, lr)) return;
    }
    // P3: O projection + residual (x += attn W_o^T)
    if (!gemv_phase<EPI_RESID, RQ, 6, 1>(
            a.attn, Ly.wo, a.x, a.x, Hd, Hd, 0.f, wg, G, nitems(no),
            [&]() { return wait_ge(sync, S_HEADS, 1, (unsigned)H * (lr + 1), 0x300u + li); }, none))
      return;
    publish(sync + (S_O + shard) * CL, (unsigned)nitems(no));
    // P4: gate/up + SwiGLU (norm fused): 4 items of 96 KB each, one at a time (two buffers of
    // 4 rows x 6 KiB per lane would not fit beside the activation row)
    for (int vb = wg; vb < ngu; vb += G) {
      if (!gemv_item<EPI_SWIGLU, 4, 6, 1>(a.x, Ly.wgu, a.act, nullptr, 2 * F, Hd, a.eps, vb, [&]() {
            return vb != wg || wait_ge(sync, S_O, 8, (unsigned)no * (lr + 1), 0x400u + li);
          }))
        return;
    }
    publish(sync + (S_GU + shard) * CL, (unsigned)nitems(ngu));
    // P5: down projection + residual (K split over 2 waves)
    if (!gemv_phase<EPI_RESID, 2, 8, 2>(
            a.act, Ly.wdown, a.x, a.x, Hd, F, 0.f, wg, G, nitems(ndn),
            [&]() { return wait_ge(sync, S_GU, 8, (unsigned)ngu * (lr + 1), 0x500u + li); }, none))
      return;
    publish(sync + (S_DN + shard) * CL, (unsigned)nitems(ndn));
  }
  // P6: LM head (final RMSNorm fused) over the last layer's output
  if (a.lm_head) {
    const int nl = a.l1 - a.l0;
    const int nv = a.V / 16;
    const int n6 = wg < nv ? (nv - wg + G - 1) / G : 0;
    if (!gemv_phase<EPI_NONE, 4, 6, 1>(
            a.x, a.lm_head, a.logits, nullptr, a.V, Hd, a.eps, wg, G, n6,
            [&]() { return wait_ge(sync, S_DN, 8, (unsigned)ndn * nl, 0x600u); }, [](int) {}))
      return;
  }
}

template <int D>
__global__ void __launch_bounds__(B1_NT, 1) decode_b1_kernel(B1Args a) {
  b1_run<D>(a);
  // exit ticket (also after an early exit on a timeout): the last workgroup out zeroes every
  // counter line but the error word — all other workgroups are past their last counter access
  __shared__ int s_lastout;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.sync + S_EXIT * CL, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_lastout = old == gridDim.x - 1;
  }
  __syncthreads();
  if (s_lastout) {
    for (int i = S_EXIT + (int)threadIdx.x; i < S_HEAD + 2 * a.H; i += B1_NT) st_u32(a.sync + i * CL, 0u);
  }
}

}  // namespace

// Resident workgroups per CU of the persistent kernel (occupancy query), for the grid size.
DA_EXPORT int da_decode_b1_occupancy(int D, int* out) {
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
  if (D == 96) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_b1_kernel<96>, B1_NT, 0);
  else if (D == 64) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_b1_kernel<64>, B1_NT, 0);
  else if (D == 128) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, decode_b1_kernel<128>, B1_NT, 0);
  *out = n;
  return (int)e;
}

// Bytes of the sync block for H heads (zero before the first launch; every launch leaves its counters
// zero again, the error word excepted).
DA_EXPORT long long da_decode_b1_sync_bytes(int H) { return (long long)(S_HEAD + 2 * H) * CL * 4; }

// layers: device array of B1Layer (6 pointers each: wqkv, wo, wgu, wdown, kc, vc) for every layer;
// runs layers [l0, l1). ws: H * nsplit * (D + 2) floats. sync: da_decode_b1_sync_bytes(H) bytes
// (zero-initialised by the caller; see decode_b1_kernel's exit ticket). lm_head / logits / V: optional
// final phase (null lm_head: skip). grid: resident workgroups (CUs of the stream x occupancy).
DA_EXPORT int da_decode_b1(const void* layers, int l0, int l1, void* x, void* qkv, void* attn, void* act,
                           const void* lens, const void* slot, const void* pre, const void* pos, const void* cos_sin,
                           int Hd, int H, int D, int F, int max_seq, int nsplit, int chunk, float eps, float scale,
                           void* ws, void* sync, const void* lm_head, void* logits, int V, int grid, void* stream) {
  if (!layers || !x || !qkv || !attn || !act || !lens || !slot || !pos || !cos_sin || !ws || !sync)
    return (int)hipErrorInvalidValue;
  if (l0 < 0 || l1 <= l0 || grid < 1 || nsplit < 1 || chunk < 64 || chunk % 64) return (int)hipErrorInvalidValue;
  if (Hd != H * D || Hd % 512 || F % 512 || D % 16 || F % 16) return (int)hipErrorInvalidValue;
  // one register round of weights per item: K = 6 x 512 (hidden) and 2 x 8 x 512 (FFN): the
  // Phi-3-mini shape this launch is instantiated for (other models keep the per-kernel path)
  if (Hd / 512 != 6 || F / 512 != 16) return (int)hipErrorInvalidValue;
  if ((long long)chunk * nsplit < 1 || H > 4096) return (int)hipErrorInvalidValue;
  if (lm_head && (!logits || V < 16 || V % 16)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  B1Args a{};
  a.layers = (const B1Layer*)layers; a.l0 = l0; a.l1 = l1;
  a.x = (bf16_t*)x; a.qkv = (bf16_t*)qkv; a.attn = (bf16_t*)attn; a.act = (bf16_t*)act;
  a.lens = (const int*)lens; a.slot = (const int*)slot; a.pre = (const int*)pre; a.pos = (const int*)pos;
  a.cs = (const float*)cos_sin;
  a.Hd = Hd; a.H = H; a.F = F; a.max_seq = max_seq; a.nsplit = nsplit; a.chunk = chunk;
  a.eps = eps; a.sl2e = scale * 1.4426950408889634f;
  a.po = (float*)ws; a.pm = a.po + (size_t)H * nsplit * D; a.pl = a.pm + (size_t)H * nsplit;
  a.sync = (unsigned*)sync;
  a.lm_head = (const bf16_t*)lm_head; a.logits = (bf16_t*)logits; a.V = V;
  switch (D) {
    case 64: decode_b1_kernel<64><<<grid, B1_NT, 0, s>>>(a); break;
    case 96: decode_b1_kernel<96><<<grid, B1_NT, 0, s>>>(a); break;
    case 128: decode_b1_kernel<128><<<grid, B1_NT, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  DA_LAUNCH_CHECK();
}
