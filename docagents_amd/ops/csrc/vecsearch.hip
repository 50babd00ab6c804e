// In-HBM vector index kernels: cosine similarity (dot product of L2-normalised bf16 rows) fused
// with the document filter, the similarity floor and a per-workgroup top-k select, then a
// second-pass merge. Replaces pgvector's `1 - (v <=> q) >= 0.7 ... ORDER BY ... LIMIT k` with
// `WHERE document_id = ANY(...)` (internal/store/postgres.go:218-285).
//
//  * topk_dense:  batched queries x all rows as MFMA tiles (16 rows x 16 queries per wave-MFMA),
//                 doc filter as a per-query bitmap over the shard's local doc slots. Also used for
//                 IVF coarse probing (rows = centroids) and k-means assignment (k = 1).
//  * topk_ranges: per-query row ranges (rows of a document are contiguous in the shard, and IVF
//                 lists are contiguous runs) — only the rows a query can match are read.
//  * topk_merge:  per query, select the global top-k over all workgroups' candidates (sorted desc,
//                 ties -> smaller row id first).
//  * kmeans_accum: centroid sums / counts for IVFFlat training (fp32 atomics, 256-B rows).
#include "common.h"

#define TK_MAX 32

__device__ __forceinline__ bool better(float a, int ia, float b, int ib) {
  return a > b || (a == b && ia >= 0 && (ib < 0 || ia < ib));
}

// Merge 64 new candidates (one per lane: a/ia) into a running sorted top-K list held in LDS
// (best/bidx, K entries) — executed by one full wave.
__device__ __forceinline__ void wave_merge_topk(float a, int ia, float* best, int* bidx, int K, int lane) {
  const float kth = best[K - 1];
  const int kthi = bidx[K - 1];
  // early exit: nothing beats the current k-th
  const bool cand = better(a, ia, kth, kthi) && a != -INFINITY;
  if (__ballot(cand) == 0ull) return;
  float b = lane < K ? best[lane] : -INFINITY;
  int ib = lane < K ? bidx[lane] : -1;
  float outv = -INFINITY;
  int outi = -1;
  for (int r = 0; r < K; ++r) {
    // local best of (a, b)
    float v; int vi; int which;
    if (better(a, ia, b, ib)) { v = a; vi = ia; which = 0; } else { v = b; vi = ib; which = 1; }
    if (v == -INFINITY) { vi = -1; }
    float wv = v; int wi = vi; int wl = lane;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(wv, o, 64);
      const int oi = __shfl_xor(wi, o, 64);
      const int ol = __shfl_xor(wl, o, 64);
      if (better(ov, oi, wv, wi) || (ov == wv && oi == wi && ol < wl)) { wv = ov; wi = oi; wl = ol; }
    }
    if (lane == r) { outv = wv; outi = (wv == -INFINITY) ? -1 : wi; }
    if (lane == wl) {
      if (which == 0) { a = -INFINITY; ia = -1; } else { b = -INFINITY; ib = -1; }
    }
  }
  if (lane < K) { best[lane] = outv; bidx[lane] = outi; }
}

// X [N, d] bf16 rows, slots [N] local doc slot per row (or null), Qv [Q, d] bf16, bitmap [Q, W] (or null)
// out_s / out_i : [gridDim.x, Q, K]
__global__ void __launch_bounds__(256)
topk_dense_kernel(const bf16_t* __restrict__ X, int N, int d, const int* __restrict__ slots,
                  const bf16_t* __restrict__ Qv, int Q, const unsigned* __restrict__ bitmap, int W, float thr,
                  int K, int rows_per_block, float* __restrict__ out_s, int* __restrict__ out_i) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int qstr = d * 2 + 16;
  char* sQ = smem;                                   // [16][d] bf16 padded
  float* sc = (float*)(smem + 16 * qstr);            // [16][64 + 1]
  float* best = sc + 16 * 65;                        // [16][TK_MAX]
  int* bidx = (int*)(best + 16 * TK_MAX);            // [16][TK_MAX]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int qbase = blockIdx.y * 16;
  const int nq = min(16, Q - qbase);
  for (int i = tid; i < 16 * (d / 8); i += 256) {
    const int r = i / (d / 8), c = i % (d / 8);
    u32x4_t v = u32x4_t{0, 0, 0, 0};
    if (r < nq) v = *(const u32x4_t*)(Qv + (size_t)(qbase + r) * d + c * 8);
    *(u32x4_t*)(sQ + r * qstr + c * 16) = v;
  }
  for (int i = tid; i < 16 * TK_MAX; i += 256) { best[i] = -INFINITY; bidx[i] = -1; }
  __syncthreads();

  const int rbeg = blockIdx.x * rows_per_block;
  const int rend = min(N, rbeg + rows_per_block);
  const int nkk = d / 32;
  for (int r0 = rbeg; r0 < rend; r0 += 64) {
    // ---- S[row][q] for this wave's 16 rows ----
    const int row_a = r0 + wid * 16 + fr;
    f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const bf16_t* xr = X + (size_t)(row_a < N ? row_a : 0) * d + fg * 8;
    for (int kk = 0; kk < nkk; ++kk) {
      bf16x8_t a = *(const bf16x8_t*)(xr + kk * 32);
      if (row_a >= rend) a = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      const bf16x8_t bq = *(const bf16x8_t*)(sQ + fr * qstr + kk * 64 + fg * 16);
      acc = mfma16(a, bq, acc);
    }
    const int q = fr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = wid * 16 + fg * 4 + i;
      const int row = r0 + rl;
      float s = acc[i];
      bool ok = row < rend && q < nq && s >= thr;
      if (ok && slots) {  // removed rows (slot -1) never match; the bitmap (if any) filters documents
        const int sl = slots[row];
        ok = sl >= 0 && (!bitmap || ((sl >> 5) < W && ((bitmap[(size_t)(qbase + q) * W + (sl >> 5)] >> (sl & 31)) & 1u)));
      }
      sc[q * 65 + rl] = ok ? s : -INFINITY;
    }
    __syncthreads();
    // ---- merge into running per-query top-K: wave w owns queries w, w+4, w+8, w+12 ----
    for (int qq = wid; qq < nq; qq += 4) {
      const float a = sc[qq * 65 + lane];
      wave_merge_topk(a, r0 + lane, best + qq * TK_MAX, bidx + qq * TK_MAX, K, lane);
    }
    __syncthreads();
  }
  for (int i = tid; i < nq * K; i += 256) {
    const int qq = i / K, j = i % K;
    const size_t o = ((size_t)blockIdx.x * Q + qbase + qq) * K + j;
    out_s[o] = best[qq * TK_MAX + j];
    out_i[o] = bidx[qq * TK_MAX + j];
  }
}

// ------------------------------------------------------------------------------------------------
// Streaming dense scan (d % 128 == 0): the whole-shard pass of flat search, IVF coarse probing and
// k-means assignment, built to run at HBM speed.
//
//  * Every wave is an independent worker over its own contiguous run of rows, 16 rows per MFMA
//    tile, against the workgroup's 16 queries (B fragments from LDS, one copy per workgroup).
//  * The rows stream from HBM through a ring of R groups (4 MFMA k-steps = 64 B per lane each)
//    that runs across tile boundaries: group s + R is requested as soon as group s is consumed,
//    so ~R * 4 KB per wave stay in flight (the old kernel issued one row load, waited, issued the
//    next: 3.5 TB/s on a 10M x 1024 shard).
//  * A tile's 16 x 16 scores are tested against each query's running k-th best; only rows that beat
//    it do any top-K work (TdWave below).
//  * Up to 16 queries (one query block): topk_dense_stream_kernel, every wave its own rows, the
//    rows loaded non-temporally straight into the MFMA A registers.
//  * 17..64 queries: topk_dense_mq_kernel, the workgroup's 4 waves = 4 query blocks over the SAME
//    rows: each 16-row tile is read from HBM once into LDS and feeds all four waves (B fragments of
//    a wave's 16 queries live in its registers). Query blocks as separate workgroups over the same
//    rows, even dispatched back to back to one XCD, missed in L2 and read the shard once per block
//    (batch 64: 12.1 ms vs 3.6 ms for batch 1, profiles/r5/index/).
// out [row blocks (padded to 8), Q, K]: one unsorted top-K list per (workgroup, query), ordered and
// merged by topk_merge_kernel.
constexpr int TD_G = 4;    // MFMA k-steps (of 32) per load group: 64 B per lane

// One wave's top-K state for its 16 queries over a run of 16-row tiles. Per query, 64 LDS slots:
// [0, K) the current top-K (unsorted), then one candidate sub-buffer of SB slots for each of the
// query's 4 lanes; the k-th best score sits in a register of those lanes.
//  * tile(): a lane's rows that beat the k-th best pass the doc filter / floor and go to ITS
//    sub-buffer at a lane-local count: no cross-lane traffic on the append path.
//  * cut(): once a sub-buffer could overflow on the next tile, the query's list + buffered rows (one
//    per lane, <= 64) are cut to the top K by a radix select on the ballot unit: 32 rounds of ballot
//    + popcount on an order-preserving integer image of the score find the K-th largest (ties at
//    the threshold go to the smaller row id), the winners are compacted into [0, K) by mbcnt. The
//    sorted-list merge it replaces (K rounds of a 6-level shuffle argmax per (tile, query), then
//    per 48 candidates) stalled the workgroup's load pipeline: 64 queries took 10.5 ms against
//    3.7 ms with no candidate work (bench/scan_probe.py, profiles/r5/index/).
// Lists leave unsorted; topk_merge_kernel orders them.
constexpr int TD_SL = 64;  // LDS slots per (wave, query)

__device__ __forceinline__ unsigned td_key(float v, int id) {  // larger = better; empty (id < 0) = 0
  const unsigned u = __float_as_uint(v);
  return id < 0 ? 0u : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
}
__device__ __forceinline__ float td_unkey(unsigned k) {
  return k == 0u ? -INFINITY : __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The top K of the wave's 64 (v, id) (one per lane; id < 0 = empty) into cs/ci[0, K) of a list,
// unsorted. Returns the K-th best score (-inf while fewer than K are real). Every lane must have
// read what it passes before the call (the list slots are overwritten).
__device__ __forceinline__ float td_cut(float v, int id, int K, int lane, float* cs, int* ci) {
  const unsigned key = td_key(v, id);
  unsigned T = 0;  // the K-th largest key (empty lanes have key 0)
  int need = K;
  bool act = true;
  for (int bt = 31; bt >= 0; --bt) {
    const bool one = (key >> bt) & 1u;
    const int c1 = __popcll(__ballot(act && one));
    if (c1 >= need) { T |= 1u << bt; act = act && one; }
    else { need -= c1; act = act && !one; }
  }
  // winners: every key > T, then `need` of the keys == T (smallest row ids; empties: any)
  unsigned long long sel = __ballot(key > T);
  unsigned long long eq = __ballot(key == T);
  need = K - __popcll(sel);
  if (__popcll(eq) <= need || T == 0u) {
    for (; need > 0 && eq; --need) { sel |= eq & (~eq + 1); eq &= eq - 1; }
  } else {  // exact score ties at the threshold (rare): smallest row ids first
    for (; need > 0; --need) {
      int m = ((eq >> lane) & 1ull) ? id : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o, 64));
      const unsigned long long w = __ballot(((eq >> lane) & 1ull) && id == m);
      sel |= w & (~w + 1);
      eq &= ~(w & (~w + 1));
    }
  }
  const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(sel >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)sel, 0u));
  wave_sync_lds();
  if ((sel >> lane) & 1ull) { cs[pos] = v; ci[pos] = id; }
  wave_sync_lds();
  return td_unkey(T);
}

struct TdWave {
  float* cs; int* ci;  // [16][TD_SL] scores / rows
  int K, SB, lane, fr, fg;
  float kth;  // this lane's query (fr): its current k-th best score
  int cnt;    // entries in this lane's sub-buffer

  __device__ __forceinline__ void init(float* s, int* i, int k) {
    cs = s; ci = i; K = k; SB = (TD_SL - k) / 4;  // K <= 32: SB >= 8
    lane = threadIdx.x & 63; fr = lane & 15; fg = lane >> 4;
    kth = -INFINITY; cnt = 0;
    for (int j = lane; j < 16 * TD_SL; j += 64) { cs[j] = -INFINITY; ci[j] = -1; }
  }
  // cut the lists of the queries set in `full` (bit q) back to their top K
  __device__ __forceinline__ void flush(const unsigned long long full) {
    wave_sync_lds();
    float kq = -INFINITY;  // lane q < 16: query q's new k-th best
    for (unsigned long long left = full; left; left &= left - 1) {
      const int q = __builtin_ctzll(left);
      // lane j: list slot j (< K) or sub-buffer b = (j - K) / SB entry (j - K) % SB, live below the
      // count of lane q + 16 b
      const int b = lane < K ? 0 : min((lane - K) / SB, 3), e = lane < K ? 0 : lane - K - b * SB;
      const int nb = __shfl(cnt, q + 16 * b, 64);
      const bool live = lane < K || (lane < K + 4 * SB && e < nb);
      const float v = live ? cs[q * TD_SL + lane] : -INFINITY;
      const int id = live ? ci[q * TD_SL + lane] : -1;
      const float t = td_cut(v, id, K, lane, cs + q * TD_SL, ci + q * TD_SL);
      if (lane == q) kq = t;
    }
    const float kn = __shfl(kq, fr, 64);
    if ((full >> fr) & 1ull) { kth = kn; cnt = 0; }
  }
  // a finished 16 x 16 tile: lane (fr, fg) holds rows row0 + i (row0 = tile base + 4 fg) of query fr
  // (global query index qrow); rows from `end` on are padding
  __device__ __forceinline__ void tile(const f32x4_t& acc, int row0, int end, bool qok, float thr,
                                       const int* __restrict__ slots, const unsigned* __restrict__ bitmap, int W,
                                       int qrow) {
    bool cand = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) cand |= qok && row0 + i < end && acc[i] >= thr && acc[i] > kth;
    if (!__ballot(cand)) return;  // the common case after the first tiles
    float* bs = cs + fr * TD_SL + K + fg * SB;
    int* bi = ci + fr * TD_SL + K + fg * SB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = row0 + i;
      bool ok = qok && row < end && acc[i] >= thr && acc[i] > kth;
      if (ok && slots) {  // removed rows (slot -1) never match; the bitmap filters documents
        const int sl = slots[row];
        ok = sl >= 0 && (!bitmap || ((sl >> 5) < W && ((bitmap[(size_t)qrow * W + (sl >> 5)] >> (sl & 31)) & 1u)));
      }
      if (ok) { bs[cnt] = acc[i]; bi[cnt] = row; ++cnt; }
    }
    // a lane's next tile adds <= 4: cut the queries with a sub-buffer past SB - 4
    const unsigned long long over = __ballot(cnt > SB - 4);
    if (over) flush((over | (over >> 16) | (over >> 32) | (over >> 48)) & 0xffffull);
  }
  // every list cut to its top K (unsorted) in slots [0, K)
  __device__ __forceinline__ void finish() {
    const unsigned long long rest = __ballot(cnt > 0);
    if (rest) flush((rest | (rest >> 16) | (rest >> 32) | (rest >> 48)) & 0xffffull);
  }
  // merge another wave's finished lists (same 16 queries) into this wave's
  __device__ __forceinline__ void absorb(const float* os, const int* oi, int nq) {
    wave_sync_lds();
    for (int q = 0; q < nq; ++q) {
      const float v = lane < K ? cs[q * TD_SL + lane] : lane < 2 * K ? os[q * TD_SL + lane - K] : -INFINITY;
      const int id = lane < K ? ci[q * TD_SL + lane] : lane < 2 * K ? oi[q * TD_SL + lane - K] : -1;
      td_cut(v, id, K, lane, cs + q * TD_SL, ci + q * TD_SL);
    }
  }
  // lists of queries [0, nq) -> out[o0 + q * K + j] (o0: this list's (part, first query) offset)
  __device__ __forceinline__ void store(int nq, size_t o0, float* __restrict__ os, int* __restrict__ oi) {
    wave_sync_lds();
    for (int i = lane; i < nq * K; i += 64) {
      const int q = i / K, j = i % K;
      os[o0 + i] = cs[q * TD_SL + j];
      oi[o0 + i] = ci[q * TD_SL + j];
    }
  }
};

// NG = d / 128 load groups per 16-row tile (3, 6, 8: d = 384, 768, 1024): the ring holds one whole
// tile ahead (NG * 4 KB per wave in flight), every load of the loop body unconditional (clamped),
// so the compiler's vmcnt waits stay counted.
template <int NG>
__global__ void __launch_bounds__(256)
topk_dense_stream_kernel(const bf16_t* __restrict__ X, int N, const int* __restrict__ slots,
                         const bf16_t* __restrict__ Qv, int Q, const unsigned* __restrict__ bitmap, int W, float thr,
                         int K, int rows_per_wave, int nqb, float* __restrict__ out_s, int* __restrict__ out_i) {
  constexpr int d = NG * 32 * TD_G;
  constexpr int qstr = d * 2 + 16;
  __shared__ __attribute__((aligned(16))) char sQ[16 * qstr];   // [16][d] bf16, rows padded by 16 B
  __shared__ float cs_all[4][16 * TD_SL];  // per wave: top-K lists + candidate buffers (TdWave)
  __shared__ int ci_all[4][16 * TD_SL];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  // XCD-grouped block order: blocks b and b + 8 i share an XCD; the nqb query blocks of row block rb
  // are b = (rb / 8) * 8 nqb + j * 8 + rb % 8
  const int b = blockIdx.x, per = 8 * nqb;
  const int grp = b / per, rem = b % per;
  const int qb = rem / 8, rb = grp * 8 + rem % 8;
  const int qbase = qb * 16, nq = min(16, Q - qbase);
  for (int i = tid; i < 16 * (d / 8); i += 256) {
    const int r = i / (d / 8), c = i % (d / 8);
    u32x4_t v = u32x4_t{0, 0, 0, 0};
    if (r < nq) v = *(const u32x4_t*)(Qv + (size_t)(qbase + r) * d + c * 8);
    *(u32x4_t*)(sQ + r * qstr + c * 16) = v;
  }
  TdWave st;
  st.init(cs_all[wid], ci_all[wid], K);
  __syncthreads();

  const int wbeg = (int)min((long)N, ((long)rb * 4 + wid) * rows_per_wave);
  const int wend = (int)min((long)N, (long)wbeg + rows_per_wave);
  const int ntile = (wend - wbeg + 15) / 16;
  const int lrow = N - 1;
  auto gload = [&](u32x4_t (&v)[NG][TD_G], int t) {  // tile t's fragments (rows clamped)
    const int row = min(wbeg + t * 16 + fr, lrow);
    const bf16_t* p = X + (size_t)row * d + fg * 8;
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int j = 0; j < TD_G; ++j) v[g][j] = __builtin_nontemporal_load((const u32x4_t*)(p + (g * TD_G + j) * 32));
  };
  u32x4_t ring[NG][TD_G];
  gload(ring, 0);
  const bool qok = fr < nq;
  for (int t = 0; t < ntile; ++t) {
    f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int row_next = min(wbeg + (t + 1) * 16 + fr, lrow);
    const bf16_t* pn = X + (size_t)row_next * d + fg * 8;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int j = 0; j < TD_G; ++j) {
        const int kk = g * TD_G + j;
        const bf16x8_t bq = *(const bf16x8_t*)(sQ + fr * qstr + kk * 64 + fg * 16);
        acc = mfma16(__builtin_bit_cast(bf16x8_t, ring[g][j]), bq, acc);
      }
      // group g of the NEXT tile into the slot just consumed (one tile of loads stays in flight)
#pragma unroll
      for (int j = 0; j < TD_G; ++j)
        ring[g][j] = __builtin_nontemporal_load((const u32x4_t*)(pn + (g * TD_G + j) * 32));
    }
    st.tile(acc, wbeg + t * 16 + fg * 4, wend, qok, thr, slots, bitmap, W, qbase + fr);
  }
  st.finish();
  // the 4 waves' lists -> one per workgroup (wave 0 absorbs the others'), out [rb, Q, K]
  __syncthreads();
  if (wid == 0) {
    for (int w = 1; w < 4; ++w) st.absorb(cs_all[w], ci_all[w], nq);
    st.store(nq, ((size_t)rb * Q + qbase) * K, out_s, out_i);
  }
}

// 17..64 queries per workgroup (see above). rows_per_block rows per workgroup (multiple of 16), grid
// = row blocks (padded to 8) x query groups of 64: the nqg groups of one row block are dispatched to
// one XCD back to back. A tile: 16 rows x d, 16 B per thread per load (NG loads), TD_PF tiles in
// flight in registers, written to one of two LDS buffers (16-B chunk c of row r at c ^ (r & 15): the
// 16 rows one ds_read_b128 lane group reads hit 16 distinct slots), one barrier per tile.
constexpr int TD_PF = 3;

template <int NG>
__global__ void __launch_bounds__(256, 1)
topk_dense_mq_kernel(const bf16_t* __restrict__ X, int N, const int* __restrict__ slots,
                     const bf16_t* __restrict__ Qv, int Q, const unsigned* __restrict__ bitmap, int W, float thr,
                     int K, int rows_per_block, int nqg, float* __restrict__ out_s, int* __restrict__ out_i) {
  constexpr int d = NG * 128, NK = d / 32, CPR = d / 8, RB = d * 2, TB = 16 * RB;
  static_assert(16 * CPR == 256 * NG, "one 16-B load per thread per 128 columns");
  __shared__ __attribute__((aligned(16))) char sX[2][TB];
  __shared__ float cs_all[4][16 * TD_SL];
  __shared__ int ci_all[4][16 * TD_SL];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int b = blockIdx.x, per = 8 * nqg;
  const int grp = b / per, rem = b % per;
  const int qg = rem / 8, rb = grp * 8 + rem % 8;
  const int qbase = (qg * 4 + wid) * 16, nq = max(0, min(16, Q - qbase));
  const bool qok = fr < nq;
  // this wave's B fragments: query qbase + fr, columns 32 kk + 8 fg .. + 8
  bf16x8_t bq[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk)
    bq[kk] = qok ? *(const bf16x8_t*)(Qv + (size_t)(qbase + fr) * d + kk * 32 + fg * 8)
                 : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  TdWave st;
  st.init(cs_all[wid], ci_all[wid], K);

  const int rbeg = (int)min((long)N, (long)rb * rows_per_block);
  const int rend = (int)min((long)N, (long)rbeg + rows_per_block);
  const int ntile = (rend - rbeg + 15) / 16;
  const int tl = max(ntile - 1, 0), lrow = N - 1;
  auto gload = [&](u32x4_t (&v)[NG], int t) {  // tile t (rows clamped): thread's chunks tid + 256 i
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int idx = tid + 256 * i, r = idx / CPR, c = idx % CPR;
      v[i] = __builtin_nontemporal_load((const u32x4_t*)(X + (size_t)min(rbeg + t * 16 + r, lrow) * d + c * 8));
    }
  };
  auto lstore = [&](const u32x4_t (&v)[NG], int buf) {
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const int idx = tid + 256 * i, r = idx / CPR, c = idx % CPR;
      *(u32x4_t*)(&sX[buf][r * RB + ((c ^ (r & 15)) << 4)]) = v[i];
    }
  };
  __syncthreads();  // the lists' initial values (before any load is in flight: this drains them)
  u32x4_t ring[TD_PF][NG];
#pragma unroll
  for (int u = 0; u < TD_PF; ++u) {
    gload(ring[u], min(u, tl));
    asm volatile("" ::: "memory");  // issue order = tile order (counted waits)
  }
  // whole groups of TD_PF tiles (no exit inside the unrolled group: the ring keeps fixed registers);
  // tiles past the end re-read the last one and mask every row
  for (int t0 = 0; t0 < ntile; t0 += TD_PF) {
#pragma unroll
    for (int u = 0; u < TD_PF; ++u) {
      const int t = t0 + u;
      const int buf = t & 1;
      lstore(ring[u], buf);
      gload(ring[u], min(t + TD_PF, tl));  // clamped past the end: uniform counts
      // tile t visible to every wave, and every wave is done with tile t - 2 (same buffer): a raw
      // barrier (__syncthreads() would drain the loads in flight)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const char* xr = &sX[buf][fr * RB];
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const int c = kk * 4 + fg;
        acc = mfma16(*(const bf16x8_t*)(xr + ((c ^ fr) << 4)), bq[kk], acc);
      }
      st.tile(acc, rbeg + t * 16 + fg * 4, rend, qok, thr, slots, bitmap, W, qbase + fr);
    }
  }
  st.finish();
  st.store(nq, ((size_t)rb * Q + qbase) * K, out_s, out_i);
}

// Per-query row ranges. ranges [R, 2] (start, end), range_off [Q+1]; rows_per_q_block rows of the
// query's concatenated ranges per workgroup (grid = (splits, Q)). out [splits, Q, K].
__global__ void __launch_bounds__(256)
topk_ranges_kernel(const bf16_t* __restrict__ X, int d, const int* __restrict__ slots,
                   const bf16_t* __restrict__ Qv, int Q, const int* __restrict__ ranges,
                   const int* __restrict__ range_off, const unsigned* __restrict__ bitmap, int W, float thr,
                   int K, int rows_per_split, float* __restrict__ out_s, int* __restrict__ out_i) {
  __shared__ float sc[64];
  __shared__ int sr[64];
  __shared__ float best[TK_MAX];
  __shared__ int bidx[TK_MAX];
  const int split = blockIdx.x, q = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int half = lane >> 5, l32 = lane & 31;
  if (tid < TK_MAX) { best[tid] = -INFINITY; bidx[tid] = -1; }
  // query chunks held in registers: lane handles chunks c = l32 + 32*i
  constexpr int MAXC = 16;  // d <= 32 * 8 * 16 = 4096
  const int nch = d / 8;
  float qv[MAXC][8];
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = l32 + 32 * i;
    if (c < nch) {
      u32x4_t u = *(const u32x4_t*)(Qv + (size_t)q * d + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) qv[i][e] = bf2f((bf16_t)((e & 1) ? (u[e >> 1] >> 16) : (u[e >> 1] & 0xffff)));
    }
  }
  const int rb = range_off[q], re = range_off[q + 1];
  DA_ASSERT(rb >= 0 && re >= rb);
  const int pbeg = split * rows_per_split, pend = pbeg + rows_per_split;
  __syncthreads();
  // walk the concatenated ranges; position p counts rows across this query's ranges
  int pos = 0;
  for (int r = rb; r < re; ++r) {
    const int s0 = ranges[2 * r], s1 = ranges[2 * r + 1];
    const int len = s1 - s0;
    const int lo = max(pbeg, pos), hi = min(pend, pos + len);
    for (int p0 = lo; p0 < hi; p0 += 64) {
      // 64 rows per iteration: 8 half-waves x 8 rows
      for (int j = 0; j < 8; ++j) {
        const int rl = (wid * 2 + half) * 8 + j;
        const int p = p0 + rl;
        float dot = 0.f;
        const int row = s0 + (p - pos);
        if (p < hi) {
          const bf16_t* xr = X + (size_t)row * d;
#pragma unroll
          for (int i = 0; i < MAXC; ++i) {
            const int c = l32 + 32 * i;
            if (c < nch) {
              u32x4_t u = *(const u32x4_t*)(xr + c * 8);
#pragma unroll
              for (int e = 0; e < 8; ++e)
                dot += qv[i][e] * bf2f((bf16_t)((e & 1) ? (u[e >> 1] >> 16) : (u[e >> 1] & 0xffff)));
            }
          }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
        if (l32 == 0) {
          bool ok = p < hi && dot >= thr;
          if (ok && slots) {
            const int sl = slots[row];
            ok = sl >= 0 && (!bitmap || ((sl >> 5) < W && ((bitmap[(size_t)q * W + (sl >> 5)] >> (sl & 31)) & 1u)));
          }
          sc[rl] = ok ? dot : -INFINITY;
          sr[rl] = ok ? row : -1;
        }
      }
      __syncthreads();
      if (wid == 0) wave_merge_topk(sc[lane], sr[lane], best, bidx, K, lane);
      __syncthreads();
    }
    pos += len;
    if (pos >= pend) break;
  }
  if (tid < K) {
    const size_t o = ((size_t)split * Q + q) * K + tid;
    out_s[o] = best[tid];
    out_i[o] = bidx[tid];
  }
}

// cand [P, Q, K] -> out [Q, K] sorted desc. One workgroup per query; candidates consumed in place.
__global__ void __launch_bounds__(256)
topk_merge_kernel(float* __restrict__ cs, int* __restrict__ ci, int P, int Q, int K, float* __restrict__ os,
                  int* __restrict__ oi) {
  __shared__ float rv[4];
  __shared__ int ri[4], rp[4];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = P * K;
  for (int r = 0; r < K; ++r) {
    float bv = -INFINITY; int bi = -1, bp = -1;
    for (int j = tid; j < n; j += 256) {
      const int pp = j / K, kk = j % K;
      const size_t o = ((size_t)pp * Q + q) * K + kk;
      const float v = cs[o];
      const int id = ci[o];
      if (id >= 0 && better(v, id, bv, bi)) { bv = v; bi = id; bp = (int)o; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oid = __shfl_xor(bi, o, 64), op = __shfl_xor(bp, o, 64);
      if ((oid >= 0 && better(ov, oid, bv, bi)) || (bi < 0 && oid >= 0)) { bv = ov; bi = oid; bp = op; }
    }
    if (lane == 0) { rv[wid] = bv; ri[wid] = bi; rp[wid] = bp; }
    __syncthreads();
    if (tid == 0) {
      float fv = rv[0]; int fi = ri[0], fp = rp[0];
      for (int w = 1; w < 4; ++w)
        if ((ri[w] >= 0 && better(rv[w], ri[w], fv, fi)) || (fi < 0 && ri[w] >= 0)) { fv = rv[w]; fi = ri[w]; fp = rp[w]; }
      os[(size_t)q * K + r] = fi >= 0 ? fv : -INFINITY;
      oi[(size_t)q * K + r] = fi;
      if (fp >= 0) ci[fp] = -1;  // consume
    }
    __syncthreads();
  }
}

// k-means accumulation: sums[assign[i]] += X[i] (fp32), counts[assign[i]] += 1
__global__ void kmeans_accum_kernel(const bf16_t* __restrict__ X, int N, int d, const int* __restrict__ assign,
                                    float* __restrict__ sums, float* __restrict__ counts) {
  const int row = blockIdx.x;
  if (row >= N) return;
  const int c = assign[row];
  if (c < 0) return;
  for (int j = threadIdx.x; j < d; j += blockDim.x) atomicAdd(&sums[(size_t)c * d + j], bf2f(X[(size_t)row * d + j]));
  if (threadIdx.x == 0) atomicAdd(&counts[c], 1.f);
}

DA_EXPORT size_t da_topk_dense_ws(int N, int Q, int K, int rows_per_block) {
  const int nblk = (N + rows_per_block - 1) / rows_per_block;
  return (size_t)nblk * Q * K * 8;
}

DA_EXPORT int da_topk_dense(const void* X, int N, int d, const void* slots, const void* Qv, int Q, const void* bitmap,
                            int W, float thr, int K, int rows_per_block, void* ws, void* out_s, void* out_i,
                            void* stream) {
  if (d % 32 || K < 1 || K > TK_MAX || rows_per_block % 64 || rows_per_block <= 0) return (int)hipErrorInvalidValue;
  if (Q == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = N > 0 ? (N + rows_per_block - 1) / rows_per_block : 1;
  float* cs = (float*)ws;
  int* ci = (int*)(cs + (size_t)nblk * Q * K);
  const size_t lds = 16 * (d * 2 + 16) + 16 * 65 * 4 + 16 * TK_MAX * 8;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  dim3 grid(nblk, (Q + 15) / 16);
  topk_dense_kernel<<<grid, 256, lds, s>>>((const bf16_t*)X, N, d, (const int*)slots, (const bf16_t*)Qv, Q,
                                           (const unsigned*)bitmap, W, thr, K, rows_per_block, cs, ci);
  int err = (int)hipGetLastError();
  if (err) return err;
  topk_merge_kernel<<<Q, 256, 0, s>>>(cs, ci, nblk, Q, K, (float*)out_s, (int*)out_i);
  DA_LAUNCH_CHECK();
}

// The streaming scan (d = 384, 768 or 1024): ws holds (row blocks padded to 8) * 4 * Q * K candidate
// pairs; rows_per_wave % 16 == 0. hipErrorInvalidValue for shapes it does not take (the caller
// then uses da_topk_dense).
DA_EXPORT size_t da_topk_stream_ws(int N, int Q, int K, int rows_per_wave) {
  const long nrb = ((long)N + 4L * rows_per_wave - 1) / (4L * rows_per_wave);
  const long nrb8 = (nrb + 7) / 8 * 8;
  return (size_t)nrb8 * Q * K * 8;
}

DA_EXPORT int da_topk_dense_stream(const void* X, int N, int d, const void* slots, const void* Qv, int Q,
                                   const void* bitmap, int W, float thr, int K, int rows_per_wave, void* ws,
                                   void* out_s, void* out_i, void* stream) {
  if ((d != 384 && d != 768 && d != 1024) || K < 1 || K > TK_MAX || rows_per_wave % 16 || rows_per_wave <= 0 ||
      N < 1)
    return (int)hipErrorInvalidValue;
  if (Q == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const long nrb = ((long)N + 4L * rows_per_wave - 1) / (4L * rows_per_wave);
  const int nrb8 = (int)((nrb + 7) / 8 * 8);
  const int nqb = (Q + 15) / 16, nqg = (Q + 63) / 64;  // query blocks of 16 / groups of 64
  if ((long)nrb8 * nqg > 0x7fffffffL) return (int)hipErrorInvalidValue;
  float* cs = (float*)ws;
  int* ci = (int*)(cs + (size_t)nrb8 * Q * K);
  // shared-tile kernel: one workgroup per CU over the whole shard (~N / 256 rows each; each
  // workgroup pays the early top-K fill once), never more row blocks than the workspace holds
  const int rpb = (int)max(4L * rows_per_wave, ((long)N + 256 * 16 - 1) / (256 * 16) * 16);
  const long nrb_mq = ((long)N + rpb - 1) / rpb;
  const int nrb8_mq = (int)((nrb_mq + 7) / 8 * 8);
#define TDS(NG)                                                                                         \
  do {                                                                                                  \
    if (nqb == 1)                                                                                       \
      topk_dense_stream_kernel<NG><<<nrb8, 256, 0, s>>>((const bf16_t*)X, N, (const int*)slots,         \
          (const bf16_t*)Qv, Q, (const unsigned*)bitmap, W, thr, K, rows_per_wave, 1, cs, ci);           \
    else                                                                                                \
      topk_dense_mq_kernel<NG><<<nrb8_mq * nqg, 256, 0, s>>>((const bf16_t*)X, N, (const int*)slots,    \
          (const bf16_t*)Qv, Q, (const unsigned*)bitmap, W, thr, K, rpb, nqg, cs, ci);                  \
  } while (0)
  switch (d) {
    case 384: TDS(3); break;
    case 768: TDS(6); break;
    default: TDS(8); break;
  }
#undef TDS
  int err = (int)hipGetLastError();
  if (err) return err;
  topk_merge_kernel<<<Q, 256, 0, s>>>(cs, ci, nqb == 1 ? nrb8 : nrb8_mq, Q, K, (float*)out_s, (int*)out_i);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_topk_ranges(const void* X, int d, const void* slots, const void* Qv, int Q, const void* ranges,
                             const void* range_off, const void* bitmap, int W, float thr, int K, int splits,
                             int rows_per_split, void* ws, void* out_s, void* out_i, void* stream) {
  if (d % 8 || d > 4096 || K < 1 || K > TK_MAX || splits < 1) return (int)hipErrorInvalidValue;
  if (Q == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  float* cs = (float*)ws;
  int* ci = (int*)(cs + (size_t)splits * Q * K);
  dim3 grid(splits, Q);
  topk_ranges_kernel<<<grid, 256, 0, s>>>((const bf16_t*)X, d, (const int*)slots, (const bf16_t*)Qv, Q,
                                          (const int*)ranges, (const int*)range_off, (const unsigned*)bitmap, W, thr,
                                          K, rows_per_split, cs, ci);
  int err = (int)hipGetLastError();
  if (err) return err;
  topk_merge_kernel<<<Q, 256, 0, s>>>(cs, ci, splits, Q, K, (float*)out_s, (int*)out_i);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_topk_merge(void* cand_s, void* cand_i, int P, int Q, int K, void* out_s, void* out_i, void* stream) {
  if (K < 1 || K > TK_MAX) return (int)hipErrorInvalidValue;
  if (Q == 0) return 0;
  topk_merge_kernel<<<Q, 256, 0, (hipStream_t)stream>>>((float*)cand_s, (int*)cand_i, P, Q, K, (float*)out_s,
                                                         (int*)out_i);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_kmeans_accum(const void* X, int N, int d, const void* assign, void* sums, void* counts, void* stream) {
  if (N == 0) return 0;
  kmeans_accum_kernel<<<N, 256, 0, (hipStream_t)stream>>>((const bf16_t*)X, N, d, (const int*)assign, (float*)sums,
                                                           (float*)counts);
  DA_LAUNCH_CHECK();
}
