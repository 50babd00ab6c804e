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
//  * A tile's 16 x 16 scores are tested against each query's running k-th best (a register of
//    the lanes that own that query). Rows that beat it pass the doc filter / floor and are APPENDED
//    to the query's candidate buffer in LDS (positions from a 4-lane prefix sum, no atomics); only a
//    buffer past TD_CB - 16 entries is merged into the wave's sorted top-K list (one wave merge per
//    up to 48 candidates, and the k-th best rises at each merge). Merging every (tile, query) that
//    had a candidate instead made 16 live queries VALU-bound: 10.8 ms vs 3.7 ms for one query on a
//    10M x 1024 shard (profiles/r5/index/).
//  * More than 16 queries: the grid's query blocks of one row block are dispatched to ONE XCD back
//    to back, so the shard is read from HBM once and re-read from that XCD's L2 (batch 64 reads X
//    once, not four times).
// out [row blocks (padded to 8), Q, K]: one top-K list per workgroup (its 4 waves' lists merged),
// merged by topk_merge_kernel.
constexpr int TD_G = 4;    // MFMA k-steps (of 32) per load group: 64 B per lane
constexpr int TD_CB = 48;  // candidate buffer entries per (wave, query): a tile adds <= 16

// NT: streaming (non-temporal) row loads — one query block, every row read once. With several
// query blocks the rows must stay in the XCD's L2 for the sibling blocks: non-temporal loads there
// sent every block to HBM (batch 64 = 4 blocks read 80 GB for a 20 GB shard: 15.2 ms vs 3.6 ms).
template <bool NT>
__device__ __forceinline__ u32x4_t td_load(const u32x4_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// NG = d / 128 load groups per 16-row tile (3, 6, 8: d = 384, 768, 1024): the ring holds one whole
// tile ahead (NG * 4 KB per wave in flight), every load of the loop body unconditional (clamped),
// so the compiler's vmcnt waits stay counted.
template <int NG, bool NT>
__global__ void __launch_bounds__(256)
topk_dense_stream_kernel(const bf16_t* __restrict__ X, int N, const int* __restrict__ slots,
                         const bf16_t* __restrict__ Qv, int Q, const unsigned* __restrict__ bitmap, int W, float thr,
                         int K, int rows_per_wave, int nqb, float* __restrict__ out_s, int* __restrict__ out_i) {
  constexpr int d = NG * 32 * TD_G;
  constexpr int qstr = d * 2 + 16;
  __shared__ __attribute__((aligned(16))) char sQ[16 * qstr];   // [16][d] bf16, rows padded by 16 B
  __shared__ float best_all[4][16 * TK_MAX];
  __shared__ int bidx_all[4][16 * TK_MAX];
  __shared__ float cbs_all[4][16 * TD_CB];  // candidate buffers: score, row
  __shared__ int cbi_all[4][16 * TD_CB];

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
  float* best = best_all[wid];
  int* bidx = bidx_all[wid];
  float* cbs = cbs_all[wid];
  int* cbi = cbi_all[wid];
  for (int i = lane; i < 16 * TK_MAX; i += 64) { best[i] = -INFINITY; bidx[i] = -1; }
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
      for (int j = 0; j < TD_G; ++j) v[g][j] = td_load<NT>((const u32x4_t*)(p + (g * TD_G + j) * 32));
  };
  u32x4_t ring[NG][TD_G];
  gload(ring, 0);
  float kth = -INFINITY;  // this lane's query (fr): its current k-th best score
  int cnt = 0;            // ... and the entries in its candidate buffer (same in its 4 lanes)
  const bool qok = fr < nq;
  // merge the buffers of the queries set in `full` (bit q) into their top-K lists
  auto flush = [&](unsigned long long full) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int q = 0; q < 16; ++q) {
      if (!((full >> q) & 1ull)) continue;
      const int n = __shfl(cnt, q, 64);
      const float a = lane < n ? cbs[q * TD_CB + lane] : -INFINITY;
      const int ia = lane < n ? cbi[q * TD_CB + lane] : -1;
      wave_merge_topk(a, ia, best + q * TK_MAX, bidx + q * TK_MAX, K, lane);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if ((full >> fr) & 1ull) { kth = best[fr * TK_MAX + K - 1]; cnt = 0; }
  };
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
        ring[g][j] = td_load<NT>((const u32x4_t*)(pn + (g * TD_G + j) * 32));
    }
    // ---- the tile is done: lane (fr, fg) holds rows fg*4 + i of query fr ----
    const int row0 = wbeg + t * 16 + fg * 4;
    bool cand = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) cand |= qok && row0 + i < wend && acc[i] >= thr && acc[i] > kth;
    if (__ballot(cand)) {  // early tiles, then rarely: filter, append to the buffers
      bool keep[4];
      int c = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = row0 + i;
        bool ok = qok && row < wend && acc[i] >= thr && acc[i] > kth;
        if (ok && slots) {  // removed rows (slot -1) never match; the bitmap filters documents
          const int sl = slots[row];
          ok = sl >= 0 &&
               (!bitmap || ((sl >> 5) < W && ((bitmap[(size_t)(qbase + fr) * W + (sl >> 5)] >> (sl & 31)) & 1u)));
        }
        keep[i] = ok;
        c += ok;
      }
      // inclusive prefix over the query's 4 lanes (fr, fr + 16, fr + 32, fr + 48)
      int p = c;
      const int p1 = __shfl_up(p, 16, 64);
      if (fg >= 1) p += p1;
      const int p2 = __shfl_up(p, 32, 64);
      if (fg >= 2) p += p2;
      const int total = __shfl(p, 48 + fr, 64);
      int pos = cnt + p - c;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (keep[i]) { cbs[fr * TD_CB + pos] = acc[i]; cbi[fr * TD_CB + pos] = row0 + i; ++pos; }
      cnt += total;
      const unsigned long long full = __ballot(fg == 0 && cnt > TD_CB - 16);
      if (full) flush(full);
    }
  }
  {
    const unsigned long long rest = __ballot(fg == 0 && cnt > 0);
    if (rest) flush(rest);
  }
  // the 4 waves' lists -> one per workgroup (wave 0 merges the others'), out [rb, Q, K]
  __syncthreads();
  if (wid == 0) {
    for (int q = 0; q < nq; ++q)
      for (int w = 1; w < 4; ++w)
        wave_merge_topk(lane < K ? best_all[w][q * TK_MAX + lane] : -INFINITY,
                        lane < K ? bidx_all[w][q * TK_MAX + lane] : -1, best + q * TK_MAX, bidx + q * TK_MAX, K, lane);
    for (int i = lane; i < nq * K; i += 64) {
      const int qq = i / K, j = i % K;
      const size_t o = ((size_t)rb * Q + qbase + qq) * K + j;
      out_s[o] = best[qq * TK_MAX + j];
      out_i[o] = bidx[qq * TK_MAX + j];
    }
  }
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
  const int nqb = (Q + 15) / 16;
  if ((long)nrb8 * nqb > 0x7fffffffL) return (int)hipErrorInvalidValue;
  float* cs = (float*)ws;
  int* ci = (int*)(cs + (size_t)nrb8 * Q * K);
#define TDS(NG)                                                                                          \
  do {                                                                                                   \
    if (nqb == 1)                                                                                        \
      topk_dense_stream_kernel<NG, true><<<nrb8 * nqb, 256, 0, s>>>((const bf16_t*)X, N, (const int*)slots, \
          (const bf16_t*)Qv, Q, (const unsigned*)bitmap, W, thr, K, rows_per_wave, nqb, cs, ci);          \
    else                                                                                                 \
      topk_dense_stream_kernel<NG, false><<<nrb8 * nqb, 256, 0, s>>>((const bf16_t*)X, N, (const int*)slots, \
          (const bf16_t*)Qv, Q, (const unsigned*)bitmap, W, thr, K, rows_per_wave, nqb, cs, ci);         \
  } while (0)
  switch (d) {
    case 384: TDS(3); break;
    case 768: TDS(6); break;
    default: TDS(8); break;
  }
#undef TDS
  int err = (int)hipGetLastError();
  if (err) return err;
  topk_merge_kernel<<<Q, 256, 0, s>>>(cs, ci, nrb8, Q, K, (float*)out_s, (int*)out_i);
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
