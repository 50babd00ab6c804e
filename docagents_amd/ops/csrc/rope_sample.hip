// RoPE + KV-cache write, and the fused temperature sampler with chosen-token logprob.
//
// RoPE, interleaved pairs (2i, 2i+1) rotated by theta_i * pos (the original Llama / GPT-J layout; an
// HF rotate_half checkpoint is converted by permuting the q / k rows of each head at load,
// models/llama.py to_interleaved_rope — q.k is invariant under the same permutation of both). With
// adjacent pairs a rotation never leaves a 16-B chunk, so the prefill QKV GEMM applies it in its
// epilogue (gemm8p EPI_ROPE). cos/sin come from a host-built fp32 table [max_pos, D/2, 2] so the
// kernels stay memory-bound (Appendix B: trig tables on the host, not sinf/cosf per element).
//
// The sampler replaces OpenAI's `logprobs=true, top_logprobs=1` + `calculateLLMConfidence`
// (internal/llm/openai.go:84-90,149-164): Gumbel-max sampling at
// temperature T (0.2 in the reference, openai.go:22) with an in-kernel counter-based hash RNG, and
// the chosen token's log-probability under the untempered distribution.
#include "common.h"

// qkv: [T, (H + 2*Hkv) * D] row-major (q heads, then k heads, then v heads)
// k_cache / v_cache: [num_slots, Hkv, max_seq, D]; slot[t], pos[t] give where token t goes.
// One work item per (token, 4 rotary pairs of one head) plus one per (token, 16-B chunk of V):
// grid (T, ceil(items / 256)) so a decode step's handful of tokens still spreads over many CUs.
__global__ void __launch_bounds__(256)
rope_cache_kernel(bf16_t* __restrict__ qkv, const int* __restrict__ pos, const int* __restrict__ slot,
                  const float* __restrict__ cs, bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, int H, int Hkv,
                  int D, int max_seq, int rotate_q) {
  const int t = blockIdx.x;
  const int w = blockIdx.y * blockDim.x + threadIdx.x;
  const int half = D / 2;
  const int groups = D / 8;  // one 16-B chunk = 4 consecutive rotary pairs per work item
  const int nheads = (rotate_q ? H : 0) + Hkv;
  const int nrot = nheads * groups;
  const int nv = vc ? Hkv * (D / 8) : 0;
  if (w >= nrot + nv) return;
  const int p = pos[t];
  const int ld = (H + 2 * Hkv) * D;
  bf16_t* row = qkv + (size_t)t * ld;
  const int s = slot ? slot[t] : 0;
  DA_ASSERT(p >= 0 && (!kc || p < max_seq) && s >= 0);
  if (w < nrot) {
    const int hh = w / groups, gq = w % groups;
    const int head = rotate_q ? hh : H + hh;  // head index within q|k region
    bf16_t* hp = row + head * D + gq * 8;
    const int i0 = gq * 4;
    const u32x4_t a = *(const u32x4_t*)hp;
    const f32x4_t c01 = *(const f32x4_t*)(cs + ((size_t)p * half + i0) * 2);
    const f32x4_t c23 = *(const f32x4_t*)(cs + ((size_t)p * half + i0) * 2 + 4);
    const float cc[4] = {c01[0], c01[2], c23[0], c23[2]}, sn[4] = {c01[1], c01[3], c23[1], c23[3]};
    u32x4_t r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x1 = bf2f(a[e] & 0xffff), x2 = bf2f(a[e] >> 16);
      const float o1 = x1 * cc[e] - x2 * sn[e];
      const float o2 = x2 * cc[e] + x1 * sn[e];
      r[e] = pack_bf2(o1, o2);
    }
    *(u32x4_t*)hp = r;
    if (kc && head >= H) {
      const int hk = head - H;
      *(u32x4_t*)(kc + (((size_t)s * Hkv + hk) * max_seq + p) * D + gq * 8) = r;
    }
  } else {
    const int wv = w - nrot;
    const int hk = wv / (D / 8), c = wv % (D / 8);
    const bf16_t* vrow = row + (H + Hkv) * D;
    bf16_t* dst = vc + (((size_t)s * Hkv + hk) * max_seq + p) * D + c * 8;
    *(u32x4_t*)dst = *(const u32x4_t*)(vrow + hk * D + c * 8);
  }
}

// One workgroup per row of logits [B, V] (bf16). temperature <= 0 -> greedy.
// Device-side decode bookkeeping so one decode step is graph-capturable (no host round trip):
//   ctr[b]   : per-row RNG counter (the row's position); null -> `step`
//   out_tok  : sampled token (also the next step's input token)
//   out_lp   : log softmax(logits)[tok] under the untempered distribution
//   conf     : [B, 2] running (sum exp(lp), count) -> mean token probability (llm/openai.go:149-164)
//   active   : rows still generating; cleared on EOS or when the history is full
//   pos/lens : advanced by one for active rows
//   hist     : hist[b * hist_ld + (pos[b] - start[b])] = tok (generation history)
struct SampleArgs {
  const bf16_t* logits; int V, ld; float temperature; unsigned seed, step;
  const int* ctr; int* out_tok; float* out_lp; float* conf; int* active; int* pos; int* lens;
  int* hist; const int* start; int hist_ld; int eos0, eos1, eos2, eos3;
};

// The sampler's per-row bookkeeping for the chosen token fi (logprob lp), one thread: token /
// logprob out, confidence running sums, generated-token history, position / length advance, stop
// on EOS or a full history. Every operand is read up front: as `x[b] += ...` statements behind the
// active check they were a chain of dependent memory round trips at the end of every decode step.
__device__ __forceinline__ void sample_bookkeep(const SampleArgs& a, int b, int fi, float lp) {
  const int act = a.active ? a.active[b] : 1;
  const float c0 = a.conf ? a.conf[2 * b] : 0.f, c1 = a.conf ? a.conf[2 * b + 1] : 0.f;
  const int pos = a.pos ? a.pos[b] : 0, st = a.hist ? a.start[b] : 0, len = a.lens ? a.lens[b] : 0;
  if (act == 0) return;
  a.out_tok[b] = fi;
  if (a.out_lp) a.out_lp[b] = lp;
  if (a.conf) { a.conf[2 * b] = c0 + __expf(lp); a.conf[2 * b + 1] = c1 + 1.f; }
  bool stop = (fi == a.eos0 || fi == a.eos1 || fi == a.eos2 || fi == a.eos3);
  if (a.hist) {
    const int gi = pos - st;
    if (gi >= 0 && gi < a.hist_ld) a.hist[(size_t)b * a.hist_ld + gi] = fi;
    if (gi + 1 >= a.hist_ld) stop = true;
  }
  if (a.pos) a.pos[b] = pos + 1;
  if (a.lens) a.lens[b] = len + 1;
  if (stop && a.active) a.active[b] = 0;
}

__global__ void __launch_bounds__(1024)
sample_kernel(SampleArgs a) {
  __shared__ float redf[16];
  __shared__ float bestv[16];
  __shared__ int besti[16];
  const int b = blockIdx.x;
  const bf16_t* row = a.logits + (size_t)b * a.ld;
  const int V = a.V;
  const float temperature = a.temperature;
  const float invT = temperature > 0.f ? 1.f / temperature : 0.f;
  const unsigned rs = a.ctr ? (unsigned)a.ctr[b] : a.step;
  const unsigned rkey = rs * 131071u + (unsigned)b;
  float mx = -INFINITY, bv = -INFINITY;
  int bi = 0;
  for (int c = threadIdx.x; c < V / 8; c += blockDim.x) {
    u32x4_t u = *(const u32x4_t*)(row + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = bf2f((bf16_t)((e & 1) ? (u[e >> 1] >> 16) : (u[e >> 1] & 0xffff)));
      const int v = c * 8 + e;
      mx = fmaxf(mx, x);
      float score = x;
      if (temperature > 0.f) score = x * invT - __logf(-__logf(u01(a.seed, rkey, (unsigned)v)));
      if (score > bv) { bv = score; bi = v; }
    }
  }
  for (int v = (V / 8) * 8 + threadIdx.x; v < V; v += blockDim.x) {  // tail
    const float x = bf2f(row[v]);
    mx = fmaxf(mx, x);
    float score = x;
    if (temperature > 0.f) score = x * invT - __logf(-__logf(u01(a.seed, rkey, (unsigned)v)));
    if (score > bv) { bv = score; bi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) { bestv[wid] = bv; besti[wid] = bi; }
  const float gmax = block_max(mx, redf);  // contains __syncthreads
  float s = 0.f;
  for (int v = threadIdx.x; v < V; v += blockDim.x) s += __expf(bf2f(row[v]) - gmax);
  s = block_sum(s, redf);
  if (threadIdx.x == 0) {
    float fv = bestv[0];
    int fi = besti[0];
    for (int i = 1; i < nw; ++i)
      if (bestv[i] > fv || (bestv[i] == fv && besti[i] < fi)) { fv = bestv[i]; fi = besti[i]; }
    sample_bookkeep(a, b, fi, bf2f(row[fi]) - gmax - __logf(s));
  }
}

// ---------------------------------------------------------------------------------------------
// Distributed sampling for a vocab-parallel LM head ("prefer distributed
// sampling"): each tensor-parallel rank holds logits [B, V/t] of the vocabulary slice
// [v0, v0 + V/t) and reduces it to 8 floats per row —
//   {best Gumbel score, its GLOBAL index (int bits), local max, sum exp(x - local max), logit of the
//    best, 0, 0, 0}
// — the ranks exchange only those (B x 32 B per rank instead of B x V/t bf16 logits), and
// sample_finalize_kernel picks the winner (max score, ties to the lower index, i.e. the lower
// rank), rebuilds the full log-sum-exp and runs sample_kernel's bookkeeping. The Gumbel noise is a
// function of the global index, so the token is the one sample_kernel draws from the full row.
__global__ void __launch_bounds__(1024)
sample_partial_kernel(const bf16_t* __restrict__ logits, int V, int ld, int v0, float temperature, unsigned seed,
                      unsigned step, const int* __restrict__ ctr, float* __restrict__ stats) {
  __shared__ float redf[16];
  __shared__ float bestv[16];
  __shared__ int besti[16];
  const int b = blockIdx.x;
  const bf16_t* row = logits + (size_t)b * ld;
  const float invT = temperature > 0.f ? 1.f / temperature : 0.f;
  const unsigned rs = ctr ? (unsigned)ctr[b] : step;
  const unsigned rkey = rs * 131071u + (unsigned)b;
  float mx = -INFINITY, bv = -INFINITY;
  int bi = v0;
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    const float x = bf2f(row[v]);
    mx = fmaxf(mx, x);
    float score = x;
    if (temperature > 0.f) score = x * invT - __logf(-__logf(u01(seed, rkey, (unsigned)(v0 + v))));
    if (score > bv) { bv = score; bi = v0 + v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) { bestv[wid] = bv; besti[wid] = bi; }
  const float lmax = block_max(mx, redf);
  float sacc = 0.f;
  for (int v = threadIdx.x; v < V; v += blockDim.x) sacc += __expf(bf2f(row[v]) - lmax);
  sacc = block_sum(sacc, redf);
  if (threadIdx.x == 0) {
    float fv = bestv[0];
    int fi = besti[0];
    for (int i = 1; i < nw; ++i)
      if (bestv[i] > fv || (bestv[i] == fv && besti[i] < fi)) { fv = bestv[i]; fi = besti[i]; }
    float* o = stats + (size_t)b * 8;
    o[0] = fv;
    o[1] = __int_as_float(fi);
    o[2] = lmax;
    o[3] = sacc;
    o[4] = bf2f(row[fi - v0]);
    o[5] = o[6] = o[7] = 0.f;
  }
}

// Small batches (the batch-1 decode step of the p50 path): one 1024-thread workgroup per row ran
// two passes over the 32k-entry vocabulary on ONE CU, ~21 us of a ~1.9 ms step. Here the row is cut
// into chunks of CL entries, one 256-thread workgroup per (chunk, row) produces the same 8-float
// stats as a vocab-parallel rank (sample_partial_kernel), and sample_finalize_kernel with
// ranks = chunks picks the token: the same token as sample_kernel (Gumbel noise keyed by the global
// index, ties to the lower index), the logprob's log-sum-exp combined per chunk.
constexpr int SAMPLE_CL = 1024;  // vocabulary entries per chunk: 4 per thread, kept in registers

__global__ void __launch_bounds__(256)
sample_chunk_kernel(const bf16_t* __restrict__ logits, int V, int ld, float temperature, unsigned seed,
                    unsigned step, const int* __restrict__ ctr, float* __restrict__ stats) {
  __shared__ float redf[16];
  __shared__ float bestv[16];
  __shared__ int besti[16];
  const int c = blockIdx.x, b = blockIdx.y, NC = gridDim.x;
  const int v0 = c * SAMPLE_CL;
  const bf16_t* row = logits + (size_t)b * ld;
  const float invT = temperature > 0.f ? 1.f / temperature : 0.f;
  const unsigned rs = ctr ? (unsigned)ctr[b] : step;
  const unsigned rkey = rs * 131071u + (unsigned)b;
  float mx = -INFINITY, bv = -INFINITY, xs[4];
  int bi = v0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = v0 + threadIdx.x + 256 * i;
    xs[i] = v < V ? bf2f(row[v]) : -INFINITY;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // ascending v per thread: ties keep the lower index
    const int v = v0 + threadIdx.x + 256 * i;
    if (v >= V) continue;
    mx = fmaxf(mx, xs[i]);
    float score = xs[i];
    if (temperature > 0.f) score = xs[i] * invT - __logf(-__logf(u01(seed, rkey, (unsigned)v)));
    if (score > bv) { bv = score; bi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) { bestv[wid] = bv; besti[wid] = bi; }
  const float lmax = block_max(mx, redf);
  float sacc = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) sacc += (xs[i] == -INFINITY) ? 0.f : __expf(xs[i] - lmax);
  sacc = block_sum(sacc, redf);
  if (threadIdx.x == 0) {
    float fv = bestv[0];
    int fi = besti[0];
    for (int i = 1; i < nw; ++i)
      if (bestv[i] > fv || (bestv[i] == fv && besti[i] < fi)) { fv = bestv[i]; fi = besti[i]; }
    float* o = stats + ((size_t)b * NC + c) * 8;
    o[0] = fv;
    o[1] = __int_as_float(fi);
    o[2] = lmax;
    o[3] = sacc;
    o[4] = bf2f(row[fi]);
    o[5] = o[6] = o[7] = 0.f;
  }
}

// gathered: [B][ranks][8] (the per-rank stats, rank-major within a row). One wave per row: lane r
// takes ranks r, r + 64, ... (one thread walking up to 126 ranks serially was ~12 us of the
// batch-1 step); winner = max score, ties to the lower index, as in sample_kernel.
__global__ void __launch_bounds__(64)
sample_finalize_kernel(const float* __restrict__ gathered, int B, int ranks, SampleArgs a) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b >= B) return;
  const float* g = gathered + (size_t)b * ranks * 8;
  float fv = -INFINITY, xb = 0.f, lm = -INFINITY;
  int fi = 0x7fffffff;
  for (int r = lane; r < ranks; r += 64) {
    const float* q = g + r * 8;
    const int qi = __float_as_int(q[1]);
    if (q[0] > fv || (q[0] == fv && qi < fi)) { fv = q[0]; fi = qi; xb = q[4]; }
    lm = fmaxf(lm, q[2]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(fv, o, 64), ox = __shfl_xor(xb, o, 64);
    const int oi = __shfl_xor(fi, o, 64);
    if (ov > fv || (ov == fv && oi < fi)) { fv = ov; fi = oi; xb = ox; }
  }
  const float gmax = wave_max(lm);
  float sp = 0.f;
  for (int r = lane; r < ranks; r += 64) sp += g[r * 8 + 3] * __expf(g[r * 8 + 2] - gmax);
  const float s = wave_sum(sp);
  if (lane != 0) return;
  sample_bookkeep(a, b, fi, xb - gmax - __logf(s));
}

DA_EXPORT int da_sample_partial(const void* logits, int B, int V, int ld, int v0, float temperature, unsigned seed,
                                unsigned step, const void* ctr, void* stats, void* stream) {
  if (B == 0) return 0;
  if (V <= 0 || ld < V || v0 < 0) return (int)hipErrorInvalidValue;
  sample_partial_kernel<<<B, 1024, 0, (hipStream_t)stream>>>((const bf16_t*)logits, V, ld, v0, temperature, seed,
                                                             step, (const int*)ctr, (float*)stats);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_sample_finalize(const void* gathered, int B, int ranks, void* out_tok, void* out_lp, void* conf,
                                 void* active, void* pos, void* lens, void* hist, const void* start, int hist_ld,
                                 int eos0, int eos1, int eos2, int eos3, void* stream) {
  if (hist && (!pos || !start)) return (int)hipErrorInvalidValue;
  if (ranks < 1) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  SampleArgs a{};
  a.out_tok = (int*)out_tok; a.out_lp = (float*)out_lp; a.conf = (float*)conf;
  a.active = (int*)active; a.pos = (int*)pos; a.lens = (int*)lens; a.hist = (int*)hist; a.start = (const int*)start;
  a.hist_ld = hist_ld; a.eos0 = eos0; a.eos1 = eos1; a.eos2 = eos2; a.eos3 = eos3;
  sample_finalize_kernel<<<B, 64, 0, (hipStream_t)stream>>>((const float*)gathered, B, ranks, a);
  DA_LAUNCH_CHECK();
}

// Chunked small-batch sampler (see sample_chunk_kernel): same arguments as da_sample plus a
// workspace of >= B * ceil(V / 1024) * 8 floats.
DA_EXPORT int da_sample_chunked(const void* logits, int B, int V, int ld, float temperature, unsigned seed,
                                unsigned step, const void* ctr, void* ws, void* out_tok, void* out_lp, void* conf,
                                void* active, void* pos, void* lens, void* hist, const void* start, int hist_ld,
                                int eos0, int eos1, int eos2, int eos3, void* stream) {
  if (hist && (!pos || !start)) return (int)hipErrorInvalidValue;
  if (V <= 0 || ld < V || !ws) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  const int NC = (V + SAMPLE_CL - 1) / SAMPLE_CL;
  sample_chunk_kernel<<<dim3(NC, B), 256, 0, (hipStream_t)stream>>>((const bf16_t*)logits, V, ld, temperature,
                                                                     seed, step, (const int*)ctr, (float*)ws);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  SampleArgs a{};
  a.out_tok = (int*)out_tok; a.out_lp = (float*)out_lp; a.conf = (float*)conf;
  a.active = (int*)active; a.pos = (int*)pos; a.lens = (int*)lens; a.hist = (int*)hist; a.start = (const int*)start;
  a.hist_ld = hist_ld; a.eos0 = eos0; a.eos1 = eos1; a.eos2 = eos2; a.eos3 = eos3;
  sample_finalize_kernel<<<B, 64, 0, (hipStream_t)stream>>>((const float*)ws, B, NC, a);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_rope_cache(void* qkv, const void* pos, const void* slot, const void* cos_sin, void* k_cache,
                            void* v_cache, int T, int H, int Hkv, int D, int max_seq, int rotate_q, void* stream) {
  if (D % 8 || (D / 2) % 4) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  const int items = ((rotate_q ? H : 0) + Hkv) * (D / 8) + (v_cache ? Hkv * (D / 8) : 0);
  const dim3 grid(T, (items + 255) / 256);
  rope_cache_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((bf16_t*)qkv, (const int*)pos, (const int*)slot,
                                                         (const float*)cos_sin, (bf16_t*)k_cache,
                                                         (bf16_t*)v_cache, H, Hkv, D, max_seq, rotate_q);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_sample(const void* logits, int B, int V, int ld, float temperature, unsigned seed, unsigned step,
                        const void* ctr, void* out_tok, void* out_lp, void* conf, void* active, void* pos, void* lens,
                        void* hist, const void* start, int hist_ld, int eos0, int eos1, int eos2, int eos3,
                        void* stream) {
  if (ld % 8) return (int)hipErrorInvalidValue;
  if (hist && (!pos || !start)) return (int)hipErrorInvalidValue;
  if (B == 0) return 0;
  SampleArgs a;
  a.logits = (const bf16_t*)logits; a.V = V; a.ld = ld; a.temperature = temperature; a.seed = seed; a.step = step;
  a.ctr = (const int*)ctr; a.out_tok = (int*)out_tok; a.out_lp = (float*)out_lp; a.conf = (float*)conf;
  a.active = (int*)active; a.pos = (int*)pos; a.lens = (int*)lens; a.hist = (int*)hist; a.start = (const int*)start;
  a.hist_ld = hist_ld; a.eos0 = eos0; a.eos1 = eos1; a.eos2 = eos2; a.eos3 = eos3;
  sample_kernel<<<B, 1024, 0, (hipStream_t)stream>>>(a);
  DA_LAUNCH_CHECK();
}
