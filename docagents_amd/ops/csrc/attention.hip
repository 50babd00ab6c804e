// Attention kernels for gfx950.
//
// 1) flash_attn_v2: packed (varlen) prefill attention, bidirectional (BERT encoder)
//    or causal with GQA (Llama-3 / Phi-3 prefill, N6/N7), optionally over a shared-prefix head in
//    the KV cache. Online softmax in fp32, bf16 MFMA 32x32x16, "swapped" S^T = K.Q^T formulation
//    (details above the kernel).
//
// 2) decode attention (one new token per sequence) over the KV cache [slot, Hkv, max_seq, D]:
//    split-KV ("flash-decoding") so a batch of long contexts fills all 256 CUs; fp32 partials
//    (unnormalised O, running max, running sum) merged by decode_combine.
#include "common.h"

#include <cstdlib>

// Floating-point contraction only within one expression (a*b + c -> fma), never across statements:
// with the HIP default (fast) the backend fuses differently depending on the surrounding code, and
// the decode attention inlined into the persistent batch-1 kernel (decode_b1.hip) then differed from
// decode_attn_kernel by one bf16 ulp on some heads (measured on the MI355X, bench/b1_diverge.py).
// Both files pin the same rule, so the two compute the same bits by construction.
#pragma clang fp contract(on)

// ------------------------------------------------------------------------------------------
// flash_attn_v2: 32x32x16 MFMA, 4 waves x 32 queries (128 queries per workgroup), 64-key tiles
// double-buffered in LDS with register staging (tile t+1's global loads are in flight while tile t
// is computed; one barrier per tile).
//   S^T[key][q] = K·Q^T : A = K rows from LDS (16-B pad per row -> conflict-free ds_read_b128),
//                         B = Q^T from registers (loaded once per wave).
//   lane l owns query l&31; its 32 keys of a 64-key tile sit in the two S^T accumulators, the
//   other 32 in lane l^32 -> row max / row sum need ONE v_permlane32_swap each.
//   O^T[d][q] += V^T·P^T : B = P^T straight from the S^T registers (k index permuted), A = V^T
//                         fetched from the row-major V tile with ds_read_b64_tr_b16 (hardware
//                         transpose; row stride chosen so the 4-row x 2-group reads are
//                         bank-conflict-free).
//   scale·log2(e) is folded into the exp2 argument (one FMA per score); the O rescale is skipped
//   when no lane's running max moved; causal tiles past a wave's last query are skipped by that
//   wave (it still stages tiles and joins the barrier).
template <int D, int NW = 4, int QH = 1>
struct FA2Cfg {
  static constexpr int KT = 64, QW = 32 * QH, QB = QW * NW, NT = 64 * NW;
  static constexpr int KSTR = D * 2 + 16;                                         // bytes
  static constexpr int VSTR = (D == 64) ? 192 : (D == 128) ? 320 : D * 2;         // bytes
  static constexpr int KBUF = KT * KSTR, VBUF = KT * VSTR;
  static constexpr int CPR = D / 8, LPT = (KT * CPR + NT - 1) / NT;
  static constexpr int SMEM = 2 * (KBUF + VBUF);
};

// Shared-prefix keys (pre.len > 0): every sequence's keys are [pre.len prefix keys | its own keys];
// the prefix K/V live once in a KV-cache slot ([Hkv][max_seq][D]: head stride pre.hstride, row
// stride D), RoPE already applied. Query i of a sequence sits at key position pre.len + i (causal
// mask bottom-right aligned), so a batch whose prompts share a system-prompt head prefills that
// head once and only the suffixes here.
struct FaPrefix {
  const bf16_t* k;
  const bf16_t* v;
  long long hstride;
  int len;
  int rev;  // dispatch order (set by the launcher): bit 0 causal longest-first, bit 1 XCD-grouped
  // own keys from the KV cache (pipelined D = 96 kernel; null: from the k / v views): sequence b's
  // keys at cache[kv_slot[cu[b]], hk, kv_pos[cu[b]] + j, :] (slot_stride = Hkv * max_seq * D,
  // head stride hstride), rows D apart — the QKV epilogue then stores k / v to the cache only
  const int* kv_slot;
  const int* kv_pos;
  const bf16_t* kc;
  const bf16_t* vc;
  long long slot_stride;
};

// The (query block, head, sequence) a flash workgroup works on, from its place in the dispatch
// order. rev bit 0 (causal): the longest query blocks (most keys) first, so the kernel's tail is
// made of short blocks (longest-processing-time-first packing). rev bit 1: the query blocks of one
// (sequence, kv head) pair all run on one XCD. Workgroups are dealt round-robin over the 8 XCDs
// (linear ids g and g + 8 share one: observed dispatch, relied on for speed only), and every block
// of a pair re-reads that pair's K / V rows; grid order put a pair's blocks on all 8 XCDs, so each
// XCD's L2 fetched the same rows. Grouped, the pair's rows are fetched into one L2 and re-read
// there (pair-major per XCD: a few pairs' rows live at a time).
struct FaBlock {
  int qb, h, b;
};
__device__ __forceinline__ FaBlock fa_block(int rev, int causal, int G) {
  const int X = gridDim.x, Y = gridDim.y, Z = gridDim.z;
  const bool lpt = causal && (rev & 1);
  if ((rev & 2) && G >= 1 && Y % G == 0 && ((Y / G) * Z) % 8 == 0) {
    const int g = blockIdx.x + X * (blockIdx.y + Y * blockIdx.z);
    const int xcd = g & 7, s = g >> 3;
    const int per = X * G;                         // workgroups of one (sequence, kv head) pair
    const int pair = (s / per) * 8 + xcd, r = s % per;
    const int qi = r / G, gh = r % G;               // all G heads' longest blocks first
    const int hkv = Y / G;
    return FaBlock{lpt ? X - 1 - qi : qi, (pair % hkv) * G + gh, pair / hkv};
  }
  return FaBlock{lpt ? X - 1 - (int)blockIdx.x : (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
}

// QH = 32-query halves per wave. QH = 2: each K fragment read from LDS feeds the S MFMAs of both
// halves and each transposed V fragment the O MFMAs of both, so LDS read bytes per FLOP halve (at
// QH = 1 the LDS reads of a tile take as long as its MFMAs); the two halves' softmax VALU work is
// independent of the other half's MFMAs, so the scheduler overlaps them inside one wave.
template <int D, int NW, int QH, typename T = BF16T>
__global__ void __launch_bounds__(64 * NW, QH == 1 ? 8 / NW : 1)
flash_attn_v2_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                     int ldq, int ldk, int ldv, const int* __restrict__ cu, int H, int Hkv, int causal,
                     float c, bf16_t* __restrict__ o, int ldo, FaPrefix pre) {
  using C = FA2Cfg<D, NW, QH>;
  constexpr int KT = C::KT, NDS = D / 16, NDB = D / 32, CPR = C::CPR, LPT = C::LPT, NT = C::NT;
  constexpr bool EVEN = (KT * CPR) % NT == 0;  // every thread stages exactly LPT chunks
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const FaBlock fb = fa_block(pre.rev, causal, H / Hkv);  // dispatch order: see fa_block
  const int b = fb.b, h = fb.h, qb = fb.qb;
  const int s0 = cu[b], L = cu[b + 1] - s0;
  const int q0 = qb * C::QB;
  if (q0 >= L) return;
  const int hk = h / (H / Hkv);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int qr = lane & 31, hi = lane >> 5;
  const int wq0 = q0 + wid * C::QW;
  int qi[QH];
  bool qvalid[QH];
  bf16x8_t qf[QH][NDS];
  f32x16_t oacc[QH][NDB];
  float m_run[QH], l_part[QH];
#pragma unroll
  for (int j = 0; j < QH; ++j) {
    qi[j] = wq0 + 32 * j + qr;
    qvalid[j] = qi[j] < L;
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds) {
      if (qvalid[j]) qf[j][ds] = *(const bf16x8_t*)(q + (size_t)(s0 + qi[j]) * ldq + h * D + ds * 16 + hi * 8);
      else qf[j][ds] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < NDB; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[j][i][r] = 0.f;
    m_run[j] = -INFINITY;
    l_part[j] = 0.f;
  }

  const int P = pre.len, Lk = P + L;  // keys: [prefix | own]; own query i is key P + i
  const int kv_end = causal ? min(Lk, P + q0 + C::QB) : Lk;
  const int wave_end = causal ? min(Lk, P + wq0 + C::QW) : Lk;
  const int ntiles = (kv_end + KT - 1) / KT;

  const bf16_t* kbase_p = k + (size_t)s0 * ldk + hk * D;
  const bf16_t* vbase_p = v + (size_t)s0 * ldv + hk * D;
  if (pre.kv_slot) {  // own keys in the cache (the launcher passes ldk = ldv = D)
    const size_t off = (size_t)pre.kv_slot[s0] * pre.slot_stride + (size_t)hk * pre.hstride + (size_t)pre.kv_pos[s0] * D;
    kbase_p = pre.kc + off;
    vbase_p = pre.vc + off;
  }
  const bf16_t* kpre = pre.k + hk * pre.hstride;
  const bf16_t* vpre = pre.v + hk * pre.hstride;
  u32x4_t kst[LPT], vst[LPT];
  // Own-key tiles (all keys >= P) load through buffer resources rebuilt per tile on the scalar unit
  // (base = the tile's first key, num_records = the bytes left in the sequence: keys past the end
  // read 0), with fixed per-lane 32-bit offsets: no per-load 64-bit address math, bounds compare or
  // exec-mask branch (those were ~90 of the ~285 vector instructions of a tile).
  unsigned koff[LPT], voff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int idx = tid + NT * i, r = idx / CPR, cc = idx % CPR;
    const bool in = EVEN || idx < KT * CPR;
    koff[i] = in ? (unsigned)(r * ldk * 2 + cc * 16) : 0x80000000u;
    voff[i] = in ? (unsigned)(r * ldv * 2 + cc * 16) : 0x80000000u;
  }
  auto load_tile = [&](int t) {
    const int k0 = t * KT;
    if (k0 >= P) {
      const int o0 = k0 - P;
      const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(kbase_p + (size_t)o0 * ldk), (short)0, (L - o0) * ldk * 2, 0x00020000);
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(vbase_p + (size_t)o0 * ldv), (short)0, (L - o0) * ldv * 2, 0x00020000);
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        kst[i] = __builtin_amdgcn_raw_buffer_load_b128(rk, koff[i], 0, 0);
        vst[i] = __builtin_amdgcn_raw_buffer_load_b128(rv, voff[i], 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int idx = tid + NT * i, r = idx / CPR, cc = idx % CPR, key = t * KT + r;
      if ((EVEN || idx < KT * CPR) && key < Lk) {
        if (key >= P) {
          kst[i] = *(const u32x4_t*)(kbase_p + (size_t)(key - P) * ldk + cc * 8);
          vst[i] = *(const u32x4_t*)(vbase_p + (size_t)(key - P) * ldv + cc * 8);
        } else {
          kst[i] = *(const u32x4_t*)(kpre + (size_t)key * D + cc * 8);
          vst[i] = *(const u32x4_t*)(vpre + (size_t)key * D + cc * 8);
        }
      } else {
        kst[i] = u32x4_t{0, 0, 0, 0};
        vst[i] = u32x4_t{0, 0, 0, 0};
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* sK = smem + buf * (C::KBUF + C::VBUF);
    char* sV = sK + C::KBUF;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int idx = tid + NT * i, r = idx / CPR, cc = idx % CPR;
      if (EVEN || idx < KT * CPR) {
        *(u32x4_t*)(sK + r * C::KSTR + cc * 16) = kst[i];
        *(u32x4_t*)(sV + r * C::VSTR + cc * 16) = vst[i];
      }
    }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);
    const int kb = t * KT;
    if (kb < wave_end) {
      const char* sK = smem + cur * (C::KBUF + C::VBUF);
      const char* sV = sK + C::KBUF;
      f32x16_t sacc[QH][2];
      // all K fragments of the tile first, then the MFMAs with the two 32-key halves interleaved:
      // one LDS round trip per tile instead of one per MFMA, and back-to-back MFMAs never depend
      // on each other (a fragment-at-a-time loop serialises LDS latency + MFMA latency 12 times).
      // D = 128 (16 fragments) batches per 32-key half, which keeps it within 256 VGPRs.
#pragma unroll
      for (int j = 0; j < QH; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc[j][hh][r] = 0.f;
      if constexpr (NDS <= 6) {
        bf16x8_t kfr[2][NDS];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int ds = 0; ds < NDS; ++ds)
            kfr[hh][ds] = *(const bf16x8_t*)(sK + (hh * 32 + qr) * C::KSTR + ds * 32 + hi * 16);
#pragma unroll
        for (int ds = 0; ds < NDS; ++ds)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int j = 0; j < QH; ++j) sacc[j][hh] = T::mma32(kfr[hh][ds], qf[j][ds], sacc[j][hh]);
        // pin that order: the register-pressure scheduler otherwise re-serialises read -> MFMA pairs
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * NDS, 0);       // DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NDS * QH, 0);  // MFMAs
      } else {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          bf16x8_t kfr[NDS];
#pragma unroll
          for (int ds = 0; ds < NDS; ++ds)
            kfr[ds] = *(const bf16x8_t*)(sK + (hh * 32 + qr) * C::KSTR + ds * 32 + hi * 16);
#pragma unroll
          for (int ds = 0; ds < NDS; ++ds)
#pragma unroll
            for (int j = 0; j < QH; ++j) sacc[j][hh] = T::mma32(kfr[ds], qf[j][ds], sacc[j][hh]);
          __builtin_amdgcn_sched_group_barrier(0x100, NDS, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NDS * QH, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < QH; ++j) {
        if (kb + KT > Lk || (causal && kb + KT - 1 > P + wq0 + 32 * j)) {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int key = kb + hh * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
              if (key >= Lk || (causal && key > P + qi[j])) sacc[j][hh][r] = -INFINITY;
            }
        }
        float mx = sacc[j][0][0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sacc[j][0][r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[j][1][r]);
        mx = max_xhalf(mx);
        const float m_new = fmaxf(m_run[j], mx);
        const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
        if (__any(m_new > m_run[j])) {
          const float alpha = exp2f((m_run[j] - m_use) * c);
          l_part[j] *= alpha;
#pragma unroll
          for (int i = 0; i < NDB; ++i) oacc[j][i] *= alpha;
        }
        m_run[j] = m_new;
        const float mc = -m_use * c;
        float psum = 0.f;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(sacc[j][hh][r], c, mc));  // raw v_exp_f32
            sacc[j][hh][r] = p;
            psum += p;
          }
        l_part[j] += psum;
      }

      // O^T += V^T P^T over 4 k-steps of 16 keys: slot (hi, j) -> key 16kc + 8(j>>2) + 4hi + (j&3)
#pragma unroll
      for (int kc = 0; kc < 4; ++kc) {
        const int hh = kc >> 1, cb = (kc & 1) * 8;
        bf16x8_t pb[QH];
#pragma unroll
        for (int j = 0; j < QH; ++j) {
          const u32x4_t pw = u32x4_t{T::pack2(sacc[j][hh][cb], sacc[j][hh][cb + 1]),
                                     T::pack2(sacc[j][hh][cb + 2], sacc[j][hh][cb + 3]),
                                     T::pack2(sacc[j][hh][cb + 4], sacc[j][hh][cb + 5]),
                                     T::pack2(sacc[j][hh][cb + 6], sacc[j][hh][cb + 7])};
          pb[j] = __builtin_bit_cast(bf16x8_t, pw);
        }
        const int g = lane >> 4, li = lane & 15;
        const int row0 = kc * 16 + 4 * (g >> 1) + (li >> 2);
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const int col = db * 32 + 16 * (g & 1) + 4 * (li & 3);
          const s16x4_t lo = lds_read_tr16(sV + row0 * C::VSTR + col * 2);
          const s16x4_t hi8 = lds_read_tr16(sV + (row0 + 8) * C::VSTR + col * 2);
          const bf16x8_t va = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi8[0], hi8[1], hi8[2], hi8[3]};
#pragma unroll
          for (int j = 0; j < QH; ++j) oacc[j][db] = T::mma32(va, pb[j], oacc[j][db]);
        }
      }
    }
    if (t + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < QH; ++j) {
    const float l_tot = sum_xhalf(l_part[j]);
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if (qvalid[j]) {
      bf16_t* orow = o + (size_t)(s0 + qi[j]) * ldo + h * D;
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = db * 32 + 8 * g + 4 * hi;
          *(u32x2_t*)(orow + d) = u32x2_t{T::pack2(oacc[j][db][4 * g] * inv, oacc[j][db][4 * g + 1] * inv),
                                          T::pack2(oacc[j][db][4 * g + 2] * inv, oacc[j][db][4 * g + 3] * inv)};
        }
    }
  }
}

// ------------------------------------------------------------------------------------------
// flash_attn_pipe: the same math and fragment layouts as flash_attn_v2<D, 4, 1>, software-pipelined
// one tile deep (guide T15): the S MFMAs of tile t + 1 are issued before the softmax + P·V of tile t,
// so the softmax VALU work never waits on the MFMA results it follows (RAW) and the matrix pipe has
// independent work while a wave is in its exp/max/pack stretch. Three LDS tile buffers: tile t
// (P·V), t + 1 (S) and t + 2 (being written); one barrier per tile.
//
// SPEC = true: speculative softmax against a deferred running max (guide T13). The round-2 form put
// the S MFMAs of tile t + 1, the max / rescale branch and the exp / pack / P·V of tile t in separate
// basic blocks, so the compiler could not interleave the softmax VALU of t with the S MFMAs of t + 1
// (ISA: a 12-MFMA block with no VALU, then a 116-VALU + 32-exp block; the SIMD ran them back to back).
// With SPEC, an unmasked tile (every key visible to every query of the wave) is one straight-line
// block: S(t + 1) MFMAs interleaved with max(t), p = exp2(s·c - m_run·c) against the STALE running
// max, row sums and the bf16 pack. The reference max of a query moves only when its tile max
// overshoots it by SPEC_TAU (log2 units of p; the first tile always does), branch-free per lane;
// only the O rescale that such a move needs is a (rare, wave-uniform) branch before P·V. Masked
// tiles (causal diagonal, sequence end) take the exact path. p <= 2^SPEC_TAU keeps the fp32 sums
// and the bf16 P exact in relative terms; the result is normalised by the same l, so only rounding
// differs from SPEC = false.
//
// DMA = true (D = 96, shared prefix a multiple of 64 keys): K / V tiles arrive by LDS-DMA
// (buffer_load ... lds) instead of register staging, in rings that give each tile TWO steps of
// latency cover (staging gave one, and a step is ~0.5 us against 1-2 us of loaded HBM / L2
// latency): at the start of step t the wave issues K(t + 3) into the slot S(t) read in step t - 1
// and V(t + 2) into the slot P·V(t - 1) read; before the step's barrier it waits for K(t + 2) and
// V(t + 1) (vmcnt(6): the 3 + 3 pieces of step t may stay in flight). K rows are unpadded (192 B)
// with 16-B chunk c of row r at slot c ^ ((r >> 2) & 3) — applied on the DMA source side — so the
// 16 rows one ds_read_b128 lane group reads hit 16 distinct bank slots; V keeps its linear rows.
// No staging registers, no ds_write, no per-tile address VALU. Past the last tile the pieces are
// issued at an out-of-range offset (no memory traffic, zeros into a free slot): uniform counts.
constexpr float SPEC_TAU = 8.f;

// Three 1-KiB LDS-DMA pieces (buffer_load_dwordx4 ... lds) into LDS lds, lds + 1 KiB, lds + 2 KiB,
// lane l's 16 B from rsrc + v_i + soff. Inline asm on purpose: through the builtin, hipcc treats the
// transposed V reads (ds_read_b64_tr_b16) as possibly aliasing the DMA and drains vmcnt to 0 before
// them, which would cancel the prefetch; these ops are invisible to its counters, and the kernel
// waits for them with explicit vmcnt. No VGPR destination (register-safe); M0 is saved and
// restored inside the statement; s_nop 4 covers an SGPR operand fresh from v_readfirstlane.
__device__ __forceinline__ void dma3_lds(__amdgpu_buffer_rsrc_t rs, unsigned lds, unsigned v0, unsigned v1,
                                         unsigned v2, int soff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %4, %6 offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %4, %6 offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %3, %4, %6 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "v"(v2), "s"(rs), "s"(lds), "s"(soff)
      : "memory", "scc");
}

template <int D, bool SPEC, bool DMA>
__global__ void __launch_bounds__(256, 2)
flash_attn_pipe_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                       int ldq, int ldk, int ldv, const int* __restrict__ cu, int H, int Hkv, int causal,
                       float c, bf16_t* __restrict__ o, int ldo, FaPrefix pre) {
  using C = FA2Cfg<D, 4, 1>;
  constexpr int KT = C::KT, NDS = D / 16, NDB = D / 32, CPR = C::CPR, LPT = C::LPT, NT = C::NT;
  constexpr bool EVEN = (KT * CPR) % NT == 0;
  static_assert(NDS <= 6, "pipelined flash: D <= 96");
  static_assert(!DMA || (D == 96 && C::VSTR == D * 2), "DMA tiles: D = 96 (linear V rows)");
  constexpr int KSTR = DMA ? D * 2 : C::KSTR, KBUF = KT * KSTR, TBUF = KBUF + C::VBUF;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const FaBlock fb = fa_block(pre.rev, causal, H / Hkv);  // dispatch order: see fa_block
  const int b = fb.b, h = fb.h, qb = fb.qb;
  const int s0 = cu[b], L = cu[b + 1] - s0;
  const int q0 = qb * C::QB;
  if (q0 >= L) return;
  const int hk = h / (H / Hkv);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int qr = lane & 31, hi = lane >> 5;
  const int wq0 = q0 + wid * C::QW;
  const int qi = wq0 + qr;
  const bool qvalid = qi < L;
  bf16x8_t qf[NDS];
#pragma unroll
  for (int ds = 0; ds < NDS; ++ds)
    qf[ds] = qvalid ? *(const bf16x8_t*)(q + (size_t)(s0 + qi) * ldq + h * D + ds * 16 + hi * 8)
                    : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  f32x16_t oacc[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m_run = -INFINITY, l_part = 0.f;

  const int P = pre.len, Lk = P + L;
  const int kv_end = causal ? min(Lk, P + q0 + C::QB) : Lk;
  const int wave_end = causal ? min(Lk, P + wq0 + C::QW) : Lk;
  const int ntiles = (kv_end + KT - 1) / KT;

  const bf16_t* kbase_p = k + (size_t)s0 * ldk + hk * D;
  const bf16_t* vbase_p = v + (size_t)s0 * ldv + hk * D;
  if (pre.kv_slot) {  // own keys in the cache (the launcher passes ldk = ldv = D)
    const size_t off = (size_t)pre.kv_slot[s0] * pre.slot_stride + (size_t)hk * pre.hstride + (size_t)pre.kv_pos[s0] * D;
    kbase_p = pre.kc + off;
    vbase_p = pre.vc + off;
  }
  const bf16_t* kpre = pre.k + hk * pre.hstride;
  const bf16_t* vpre = pre.v + hk * pre.hstride;
  auto buf_of = [&](int t) { return smem + (t % 3) * TBUF; };
  u32x4_t kst[LPT], vst[LPT];
  unsigned koff[LPT], voff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int idx = tid + NT * i, r = idx / CPR, cc = idx % CPR;
    const bool in = EVEN || idx < KT * CPR;
    koff[i] = in ? (unsigned)(r * ldk * 2 + cc * 16) : 0x80000000u;
    voff[i] = in ? (unsigned)(r * ldv * 2 + cc * 16) : 0x80000000u;
  }
  // DMA pieces: wave wid fills LDS 16-B positions (3 wid + i) * 64 + lane of a tile (768 = 64 rows x
  // 12 chunks): row r, slot sl; K slot sl holds chunk sl ^ ((r >> 2) & 3), V slot sl chunk sl
  unsigned dkr[3], dkc[3], dvc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int pos = (wid * 3 + i) * 64 + lane, r = pos / 12, sl = pos % 12;
    dkr[i] = r;
    dkc[i] = (sl ^ ((r >> 2) & 3)) * 16;
    dvc[i] = sl * 16;
  }
  // tile t's K (KV = false) or V pieces into slot t % 3; t >= ntiles: out of range, no traffic
  auto dma_tile = [&](int t, bool is_v) {
    const int k0 = t * KT;
    const bf16_t* base = is_v ? vbase_p : kbase_p;
    const bf16_t* pbase = is_v ? vpre : kpre;
    const int ld = is_v ? ldv : ldk;
    const bool own = k0 >= P;
    const int o0 = k0 - P;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(own ? base + (size_t)o0 * ld : pbase + (size_t)k0 * D), (short)0,
        own ? max(L - o0, 0) * ld * 2 : (P - k0) * D * 2, 0x00020000);
    const unsigned rstride = own ? ld * 2 : D * 2;
    const int soff = t < ntiles ? 0 : 0x7ffffff0;
    typedef __attribute__((address_space(3))) char lds_char;  // LDS byte offset, not the flat address
    const unsigned dst = (unsigned)(size_t)(lds_char*)(buf_of(t) + (is_v ? KBUF : 0)) + wid * 3 * 1024;
    dma3_lds(rs, __builtin_amdgcn_readfirstlane(dst), dkr[0] * rstride + (is_v ? dvc[0] : dkc[0]),
             dkr[1] * rstride + (is_v ? dvc[1] : dkc[1]), dkr[2] * rstride + (is_v ? dvc[2] : dkc[2]), soff);
  };
  auto load_tile = [&](int t) {
    const int k0 = t * KT;
    if (k0 >= P) {
      const int o0 = k0 - P;
      const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(kbase_p + (size_t)o0 * ldk), (short)0, (L - o0) * ldk * 2, 0x00020000);
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(vbase_p + (size_t)o0 * ldv), (short)0, (L - o0) * ldv * 2, 0x00020000);
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        kst[i] = __builtin_amdgcn_raw_buffer_load_b128(rk, koff[i], 0, 0);
        vst[i] = __builtin_amdgcn_raw_buffer_load_b128(rv, voff[i], 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int idx = tid + NT * i, r = idx / CPR, cc = idx % CPR, key = t * KT + r;
      if ((EVEN || idx < KT * CPR) && key < Lk) {
        if (key >= P) {
          kst[i] = *(const u32x4_t*)(kbase_p + (size_t)(key - P) * ldk + cc * 8);
          vst[i] = *(const u32x4_t*)(vbase_p + (size_t)(key - P) * ldv + cc * 8);
        } else {
          kst[i] = *(const u32x4_t*)(kpre + (size_t)key * D + cc * 8);
          vst[i] = *(const u32x4_t*)(vpre + (size_t)key * D + cc * 8);
        }
      } else {
        kst[i] = u32x4_t{0, 0, 0, 0};
        vst[i] = u32x4_t{0, 0, 0, 0};
      }
    }
  };
  auto store_tile = [&](int t) {
    char* sK = buf_of(t);
    char* sV = sK + C::KBUF;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int idx = tid + NT * i, r = idx / CPR, cc = idx % CPR;
      if (EVEN || idx < KT * CPR) {
        *(u32x4_t*)(sK + r * C::KSTR + cc * 16) = kst[i];
        *(u32x4_t*)(sV + r * C::VSTR + cc * 16) = vst[i];
      }
    }
  };
  // byte offset of K fragment (32-key half hh, 16-dim step ds) of this lane in a K tile
  auto kfrag = [&](int hh, int ds) -> int {
    if constexpr (DMA) return (hh * 32 + qr) * KSTR + (((2 * ds + hi) ^ ((qr >> 2) & 3)) << 4);
    else return (hh * 32 + qr) * KSTR + ds * 32 + hi * 16;
  };
  // S^T of tile t: all K fragments, then the MFMAs (two independent accumulation chains)
  auto s_tile = [&](int t, f32x16_t (&sa)[2]) {
    const char* sK = buf_of(t);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int r = 0; r < 16; ++r) sa[hh][r] = 0.f;
    if constexpr (SPEC) {
      // one 32-key half at a time: 6 fragments (24 VGPRs) live instead of 12 beside the softmax of t
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        bf16x8_t kfr[NDS];
#pragma unroll
        for (int ds = 0; ds < NDS; ++ds)
          kfr[ds] = *(const bf16x8_t*)(sK + kfrag(hh, ds));
#pragma unroll
        for (int ds = 0; ds < NDS; ++ds) sa[hh] = mfma32(kfr[ds], qf[ds], sa[hh]);
      }
    } else {
      bf16x8_t kfr[2][NDS];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int ds = 0; ds < NDS; ++ds)
          kfr[hh][ds] = *(const bf16x8_t*)(sK + kfrag(hh, ds));
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) sa[hh] = mfma32(kfr[hh][ds], qf[ds], sa[hh]);
    }
  };
  // O^T += V^T P^T of tile t, P packed to bf16 (kc = 16-key step)
  auto pv_tile = [&](int t, const u32x4_t (&pw)[4]) {
    const char* sV = buf_of(t) + KBUF;
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      const bf16x8_t pb = __builtin_bit_cast(bf16x8_t, pw[kc]);
      const int g = lane >> 4, li = lane & 15;
      const int row0 = kc * 16 + 4 * (g >> 1) + (li >> 2);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const int col = db * 32 + 16 * (g & 1) + 4 * (li & 3);
        const s16x4_t lo = lds_read_tr16(sV + row0 * C::VSTR + col * 2);
        const s16x4_t hi8 = lds_read_tr16(sV + (row0 + 8) * C::VSTR + col * 2);
        const bf16x8_t va = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi8[0], hi8[1], hi8[2], hi8[3]};
        oacc[db] = mfma32(va, pb, oacc[db]);
      }
    }
  };
  // mask + online softmax + O^T += V^T P^T of tile t
  auto finish = [&](int t, f32x16_t (&sa)[2]) {
    const int kb = t * KT;
    if (kb + KT > Lk || (causal && kb + KT - 1 > P + wq0)) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb + hh * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
          if (key >= Lk || (causal && key > P + qi)) sa[hh][r] = -INFINITY;
        }
    }
    float mx = sa[0][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sa[0][r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sa[1][r]);
    mx = max_xhalf(mx);
    const float m_new = fmaxf(m_run, mx);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    if (__any(m_new > m_run)) {
      const float alpha = exp2f((m_run - m_use) * c);
      l_part *= alpha;
#pragma unroll
      for (int i = 0; i < NDB; ++i) oacc[i] *= alpha;
    }
    m_run = m_new;
    const float mc = -m_use * c;
    float psum = 0.f;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(fmaf(sa[hh][r], c, mc));
        sa[hh][r] = pv;
        psum += pv;
      }
    l_part += psum;
    u32x4_t pw[4];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      const int hh = kc >> 1, cb = (kc & 1) * 8;
      pw[kc] = u32x4_t{pack_bf2(sa[hh][cb], sa[hh][cb + 1]), pack_bf2(sa[hh][cb + 2], sa[hh][cb + 3]),
                       pack_bf2(sa[hh][cb + 4], sa[hh][cb + 5]), pack_bf2(sa[hh][cb + 6], sa[hh][cb + 7])};
    }
    pv_tile(t, pw);
  };
  // unmasked tile with a deferred running max (SPEC; see above the kernel). The caller issues the S
  // MFMAs of tile t + 1 just before, in the same basic block.
  const float spec_thr = SPEC_TAU / c;  // raw-score headroom above the reference max
  auto finish_spec = [&](int t, f32x16_t (&sa)[2]) {
    float mx = fmaxf(sa[0][0], sa[0][1]);
#pragma unroll
    for (int r = 2; r < 16; ++r) mx = fmaxf(mx, sa[0][r]);
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sa[1][r]);
    mx = max_xhalf(mx);
    // the reference max moves only when the tile max overshoots it by SPEC_TAU (log2 units of p):
    // p <= 2^SPEC_TAU; first tile: m_run = -inf -> m_new = mx, alpha = 0
    const bool up = mx > m_run + spec_thr;
    const float m_new = up ? mx : m_run;
    const float alpha = exp2f((m_run - m_new) * c);
    const float mcs = -m_new * c;
    float psum = 0.f;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(fmaf(sa[hh][r], c, mcs));
        sa[hh][r] = pv;
        psum += pv;
      }
    u32x4_t pw[4];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      const int hh = kc >> 1, cb = (kc & 1) * 8;
      pw[kc] = u32x4_t{pack_bf2(sa[hh][cb], sa[hh][cb + 1]), pack_bf2(sa[hh][cb + 2], sa[hh][cb + 3]),
                       pack_bf2(sa[hh][cb + 4], sa[hh][cb + 5]), pack_bf2(sa[hh][cb + 6], sa[hh][cb + 7])};
    }
    l_part = l_part * alpha + psum;
    m_run = m_new;
    // materialise P and l here: otherwise the compiler sinks the exp / pack work past the branch
    // into the P·V block, away from the S MFMAs of t + 1 it is meant to run beside
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) asm volatile("" : "+v"(pw[kc]));
    asm volatile("" : "+v"(l_part));
    if (__any(up)) {  // rare after the first tiles: O moves to the new reference
#pragma unroll
      for (int i = 0; i < NDB; ++i) oacc[i] *= alpha;
    }
    pv_tile(t, pw);
  };

  f32x16_t SA[2], SB[2];
  auto barrier = [&]() {  // LDS reads done + every wave here (no vmcnt drain: DMA stays in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  if constexpr (DMA) {
    dma_tile(0, false); dma_tile(0, true); dma_tile(1, false); dma_tile(1, true); dma_tile(2, false);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // K0 V0 K1 landed (V1 K2 may fly)
    barrier();
    s_tile(0, SA);
    barrier();  // every wave's S(0) reads are done before K(3) refills slot 0
  } else {
    load_tile(0);
    store_tile(0);
    if (ntiles > 1) {
      load_tile(1);
      store_tile(1);
    }
    __syncthreads();
    if (ntiles > 2) load_tile(2);
    s_tile(0, SA);
  }
  auto step = [&](int t, f32x16_t (&cur)[2], f32x16_t (&nxt)[2]) {
    if constexpr (DMA) {
      dma_tile(t + 3, false);  // slot of K(t): read by S(t) in step t - 1
      dma_tile(t + 2, true);   // slot of V(t - 1): read by P·V(t - 1) in step t - 1
    }
    const int kb = t * KT;
    const bool nx = t + 1 < ntiles && (t + 1) * KT < wave_end;
    // unmasked for every query of this wave (the smallest query sees the tile's last key)
    const bool clean = kb + KT <= Lk && (!causal || kb + KT - 1 <= P + wq0);
    if (SPEC && nx && clean) {
      s_tile(t + 1, nxt);
      finish_spec(t, cur);
    } else if (SPEC && clean && kb < wave_end) {
      finish_spec(t, cur);
    } else {
      if (nx) s_tile(t + 1, nxt);
      if (kb < wave_end) finish(t, cur);
    }
    if constexpr (DMA) {
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // K(t + 2), V(t + 1) landed
      barrier();
    } else {
      if (t + 2 < ntiles) store_tile(t + 2);   // its buffer (t - 1) % 3 was last read before the previous barrier
      if (t + 3 < ntiles) load_tile(t + 3);
      __syncthreads();
    }
  };
  for (int t = 0; t < ntiles; t += 2) {
    step(t, SA, SB);
    if (t + 1 < ntiles) step(t + 1, SB, SA);
  }
  if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing no-traffic pieces

  const float l_tot = sum_xhalf(l_part);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qvalid) {
    bf16_t* orow = o + (size_t)(s0 + qi) * ldo + h * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = db * 32 + 8 * g + 4 * hi;
        *(u32x2_t*)(orow + d) = u32x2_t{pack_bf2(oacc[db][4 * g] * inv, oacc[db][4 * g + 1] * inv),
                                        pack_bf2(oacc[db][4 * g + 2] * inv, oacc[db][4 * g + 3] * inv)};
      }
  }
}

// ------------------------------------------------------------------------------------------
// Decode attention: q [B, ldq] (head h at h*D), caches [slots, Hkv, max_seq, D],
// lens[b] = tokens in cache for b (current token included), slot[b] = cache slot of b.
// Partials: po [B, H, nsplit, D] fp32 (unnormalised, relative to pm), pm/pl [B, H, nsplit].
//
// Memory-bound streaming design: for a fixed (slot, kv head) the keys of a 64-key tile are one
// contiguous [64 x D] bf16 block, so each wave loads it as a flat byte array with fully coalesced
// 16-B-per-lane loads (1 KiB per wave-instruction) — chunk c = 64*i + lane holds key c / (D/8),
// dims 8*(c % (D/8)) .. +7. Partial dot products are reduced per key with lane shuffles when a key's
// chunks sit in one wave-instruction (D = 64, 128) or through a small per-wave LDS buffer (D = 96).
// The P*V accumulation uses the same flat chunks: lane's dim-slot for chunk i is static given
// i mod NSET, so accumulators stay in registers. Each of the 4 waves streams its own tiles with its
// own online softmax (no block barriers in the loop); the waves are merged once at the end.
// Split-KV epilogue shared by the decode kernels. A split's merged (over its 4 waves) result for
// query head h: unnormalised O row `o`, running max M (log2 domain), sum ls. With one split the
// normalised bf16 output is written directly; otherwise the fp32 partial, and the LAST split of
// (b, kv head) to finish (atomic ticket in cnt[b * Hkv + hk], reset by that split so the counters
// are zero again for the next launch / graph replay) merges all splits of its G heads — the
// separate combine launch (~5 us per layer, most of a batch-1 decode attention) is gone.
// Keys per split of a row. The grid's split count is fixed at capture (sized for the cache
// capacity, max_len), but a row holds L <= max_len keys: balanced splits (the default) spread the
// row's L keys over ALL its splits (64-key multiples) instead of filling the first ceil(L / chunk)
// and leaving the rest idle — at batch 1 and 2.9k of 4k keys, 256 working workgroups instead of 192.
__device__ __forceinline__ int dec_chunk(int L, int nsplit, int chunk_arg) {
  const int c = ((L + nsplit - 1) / nsplit + 63) & ~63;
  return c < chunk_arg ? c : chunk_arg;
}

__device__ __forceinline__ void dec_store(float o, float M, float ls, int b, int h, int d, int H, int nsplit,
                                          int split, int D, float* po, float* pm, float* pl, bf16_t* out,
                                          int ldo) {
  if (nsplit == 1) {
    out[(size_t)b * ldo + h * D + d] = f2bf(ls > 0.f ? o / ls : 0.f);
    return;
  }
  const size_t pidx = ((size_t)b * H + h) * nsplit + split;
  po[pidx * D + d] = o;
  if (d == 0) { pm[pidx] = M; pl[pidx] = ls; }
}

// XC (same-XCD exchange): every split of (b, kv head) ran on ONE XCD (the launch's workgroup ->
// XCD round-robin, see decode_attn_kernel), so partials and tickets live in ordinary (cached)
// memory: the stores reach that XCD's L2, the ticket is an L2 atomic and the merging split reads
// the partials from L2 (agent-scope loads: past its L1) — L2 round trips instead of uncached ones.
template <int D, int G, bool XC = false>
__device__ __forceinline__ void dec_finish(const float* po, const float* pm, const float* pl, int H, int Hkv,
                                           int nsplit, int b, int hk, int* cnt, bf16_t* out, int ldo, int* s_last) {
  if (nsplit == 1 || cnt == nullptr) return;  // no counters: the host launches decode_combine_kernel
  const int tid = threadIdx.x;
  // Partials and tickets live in UNCACHED memory (da_malloc_uncached: MTYPE UC, L2 bypassed), so
  // device-wide visibility needs only this workgroup's stores to have completed — no
  // __threadfence(), whose L2 write-back + invalidate of the whole cache costs more than the
  // combine launch it replaces (measured: 24.6 -> 48.4 us at batch 1).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    int* c = &cnt[b * Hkv + hk];
    const int old = XC ? __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : atomicAdd(c, 1);
    *s_last = old == nsplit - 1;
    if (*s_last) {
      if constexpr (XC) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else *c = 0;
    }
  }
  __syncthreads();
  if (!*s_last) return;
  auto ld = [](const float* p) -> float {
    if constexpr (XC) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
  };
  // One online pass over the splits, 8 splits' (m, l, o) loads issued per step: the partials sit in
  // uncached memory (~1-2 us per round trip), so a max pass + a sum pass that each walk the splits
  // one dependent load at a time cost ~2 x nsplit round trips — most of a batch-1 decode attention.
  for (int i = tid; i < G * D; i += blockDim.x) {
    const int g = i / D, d = i % D, h = hk * G + g;
    const size_t base = ((size_t)b * H + h) * nsplit;
    float M = -INFINITY, lsum = 0.f, acc = 0.f;
    for (int s0 = 0; s0 < nsplit; s0 += 8) {
      float ms[8], ls[8], os[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int s = min(s0 + j, nsplit - 1);
        ms[j] = ld(pm + base + s);
        ls[j] = ld(pl + base + s);
        os[j] = ld(po + (base + s) * D + d);
      }
      float mx = M;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (s0 + j < nsplit) mx = fmaxf(mx, ms[j]);
      const float mu = (mx == -INFINITY) ? 0.f : mx;
      const float r = (M == -INFINITY) ? 0.f : exp2f(M - mu);
      lsum *= r;
      acc *= r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (s0 + j >= nsplit) continue;
        const float f = exp2f(ms[j] - mu);
        lsum += ls[j] * f;
        acc += os[j] * f;
      }
      M = mx;
    }
    out[(size_t)b * ldo + h * D + d] = f2bf(lsum > 0.f ? acc / lsum : 0.f);
  }
}

// Fused RoPE + KV-cache write for the decode step (cs != null; MHA kernel): q is the raw qkv row
// ([q heads | k heads | v heads], row stride ldq). The kernel rotates q on its way into LDS, and
// the split holding the new token (key L-1, rope position pos[b] == L-1) takes that key's rotated
// k and v straight from the qkv row — as one extra online-softmax term, never read back from the
// cache — and writes them into the cache slot for later steps. Replaces the per-layer
// rope_cache launch of the decode step (bit-identical: the same bf16 roundings).
struct DecRope {
  bf16_t* kc;           // cache bases (writable) for the new token's k / v
  bf16_t* vc;
  const float* cs;      // [max_pos][D/2][2] (cos, sin)
  const int* pos;       // [B]
};

template <int D, int G, int VAR>
__global__ void __launch_bounds__(256)
decode_attn_kernel(const bf16_t* __restrict__ q, int ldq, const bf16_t* __restrict__ kc,
                   const bf16_t* __restrict__ vc, const int* __restrict__ lens, const int* __restrict__ slot,
                   const int* __restrict__ pre,
                   int H, int Hkv, int max_seq, int chunk_max, int nsplit, float scale_log2e,
                   float* __restrict__ po, float* __restrict__ pm, float* __restrict__ pl,
                   bf16_t* __restrict__ out, int ldo, int* __restrict__ cnt, DecRope rope) {
  constexpr int KT = 64;
  constexpr int CPR = D / 8;                       // 16-B chunks per key row
  constexpr int GCD = (CPR % 16 == 0) ? 16 : ((CPR % 8 == 0) ? 8 : ((CPR % 4 == 0) ? 4 : 2));
  constexpr int NSET = CPR / GCD;                  // distinct dim-slots per lane
  constexpr bool SHFL = (64 % CPR) == 0;           // a key's chunks live in one wave-instruction
  // 4 waves per workgroup (8, a split's tiles all in flight at once at batch 1, measured 2x slower:
  // profiles/r4/rejected_r4.txt)
  constexpr int NWV = 4, NTH = 64 * NWV;
  __shared__ float sq[G][D];
  __shared__ float sp[NWV][G][KT];
  __shared__ float spart[SHFL ? 1 : NWV][SHFL ? 1 : G * KT * CPR];
  __shared__ float so[G == 1 ? 1 : NWV][G][D];
  __shared__ float sacc[G == 1 ? NWV * NSET * 64 * 8 : 1];
  __shared__ float swm[NWV][G], swl[NWV][G];

  // VAR bit3 (XC): workgroup w of the launch runs on XCD w % 8 (round-robin dispatch; the host
  // enables XC only after a placement probe confirmed it), so (b, kv head) pair p takes the nsplit
  // workgroups w = 8 * (nsplit * (p / 8) + split) + p % 8: all of its splits on one XCD, their
  // partials exchanged through that XCD's L2 (dec_finish<XC>). Needs (B * Hkv) % 8 == 0.
  constexpr bool XC = (VAR & 8) != 0;
  int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  if constexpr (XC) {
    const int wl = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int s8 = wl >> 3, pair = (s8 / nsplit) * 8 + (wl & 7);
    split = s8 % nsplit;
    hk = pair % Hkv;
    b = pair / Hkv;
  }
  const int L = lens[b];
  DA_ASSERT(L >= 0 && L <= max_seq && slot[b] >= 0);
  const int chunk = dec_chunk(L, nsplit, chunk_max);
  const int kstart = split * chunk;
  const bool fr = rope.cs != nullptr;
  const bool own_new = fr && kstart <= L - 1 && L - 1 < kstart + chunk;  // this split holds key L-1
  const int kend = min(fr ? L - 1 : L, kstart + chunk);                  // fused: key L-1 comes from qkv
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const size_t cbase = ((size_t)slot[b] * Hkv + hk) * (size_t)max_seq * D;
  const int P = pre ? pre[2 * b] : 0;  // shared-prefix keys [0, P) live in slot pre[2b + 1]
  const size_t pbase = P ? ((size_t)pre[2 * b + 1] * Hkv + hk) * (size_t)max_seq * D : cbase;
  DA_ASSERT(P % 64 == 0 && P <= L);
  DA_ASSERT(!fr || rope.pos[b] == L - 1);
  __shared__ float skn[D], svn[D], ssn[G];

  // VAR bit0: non-temporal loads (the KV stream is read once per step); bit1: V issued together
  // with K (else after the scores: ~100 VGPRs live instead of ~200, so 4-5 waves per SIMD hide the
  // HBM latency instead of 2); bit2 (small batches, implies bit1): the wave's NEXT tile is loaded
  // before the current one is computed — at batch 1 a workgroup's few tiles are latency-bound, one
  // HBM round trip each, and occupancy buys nothing. Loads are branch-free (chunk index clamped
  // into the tile; keys >= nk get p = 0) so the compiler's vmcnt waits stay counted.
  constexpr bool NT = VAR & 1, PFT = (VAR & 4) != 0, VEARLY = PFT || (VAR & 2) != 0;
  auto ld16 = [&](const bf16_t* p) -> u32x4_t {
    if constexpr (NT) return __builtin_nontemporal_load((const u32x4_t*)p);
    else return *(const u32x4_t*)p;
  };
  auto tile_base = [&](const bf16_t* c, int t0) {
    return c + (t0 < P ? pbase : cbase) + (size_t)t0 * D;
  };
  // PFT loads are branch-free: a tile past kend reads key 0 of the row's own slot (one line, valid
  // memory, never used) so the prefetches can be issued unconditionally
  auto load_k = [&](u32x4_t (&kv)[CPR], int t0) {
    const int nk = kend - t0;
    const int last = min(KT, nk) * CPR - 1;
    const bf16_t* kb = tile_base(kc, t0);
#pragma unroll
    for (int i = 0; i < CPR; ++i) {
      const int c = i * 64 + lane;
      if constexpr (PFT) kv[i] = ld16(nk > 0 ? kb + min(c, last) * 8 : kc + cbase);
      else kv[i] = (c <= last) ? ld16(kb + c * 8) : u32x4_t{0, 0, 0, 0};
    }
  };
  auto load_v = [&](u32x4_t (&vv)[CPR], int t0) {
    const int nk = kend - t0;
    const int last = min(KT, nk) * CPR - 1;
    const bf16_t* vb = tile_base(vc, t0);
#pragma unroll
    for (int i = 0; i < CPR; ++i) {
      const int c = i * 64 + lane;
      if constexpr (PFT) vv[i] = ld16(nk > 0 ? vb + min(c, last) * 8 : vc + cbase);
      else vv[i] = (c <= last) ? ld16(vb + c * 8) : u32x4_t{0, 0, 0, 0};
    }
  };
  // RoPE (interleaved pairs (2i, 2i+1)) of one element of a head row, rounded to bf16 like the
  // rope_cache kernel / the QKV GEMM epilogue that this path replaces
  constexpr int HALF = D / 2;
  auto rot2 = [&](float x1, float x2, float c, float sn, int d) -> float {
    return bf2f(f2bf((d & 1) ? x2 * c + x1 * sn : x1 * c - x2 * sn));
  };
  auto rot = [&](const bf16_t* hp, int d, int p) -> float {
    const int i = d >> 1;
    return rot2(bf2f(hp[d & ~1]), bf2f(hp[d | 1]), rope.cs[((size_t)p * HALF + i) * 2],
                rope.cs[((size_t)p * HALF + i) * 2 + 1], d);
  };
  // PFT (small batches): the prologue's operands (this thread's q element, its RoPE partner and
  // cos / sin, the new token's k / v element) are loaded FIRST, then the first two K/V tiles of the
  // wave are requested, unconditionally (an empty tile reads one line), so the compiler's counted
  // wait for the prologue leaves the K/V stream in flight: its first HBM round trip overlaps the
  // prologue instead of following it (vmcnt retires loads in order).
  constexpr bool PRE = PFT && G * D <= 256;
  u32x4_t ka[PFT ? CPR : 1], va[PFT ? CPR : 1], kb2[PFT ? CPR : 1], vb2[PFT ? CPR : 1];
  if constexpr (PRE) {
    // straight-line, clamped loads of raw bits: no branch and no use before the K/V loads below, so
    // the wait for them is a counted vmcnt(48), not vmcnt(0) (a use inside a branch forces the latter)
    const int qi = min(tid, G * D - 1), d = qi % D;
    const bf16_t* hp = q + (size_t)b * ldq + (hk * G + qi / D) * D;
    const bf16_t rq1 = hp[d & ~1], rq2 = hp[d | 1];
    const float* csp = fr ? rope.cs + ((size_t)(L - 1) * HALF + (d >> 1)) * 2 : (const float*)hp;
    const f32x2_t rcs = *(const f32x2_t*)csp;
    const bf16_t* kr = fr ? q + (size_t)b * ldq + (size_t)(H + hk) * D : hp;
    const bf16_t* vr = fr ? q + (size_t)b * ldq + (size_t)(H + Hkv + hk) * D : hp;
    const bf16_t rk1 = kr[d & ~1], rk2 = kr[d | 1], nv = vr[d];
    const int t0 = kstart + w * KT, t1 = t0 + NWV * KT;
    load_k(ka, t0); load_v(va, t0);
    load_k(kb2, t1); load_v(vb2, t1);
    const float pc = fr ? rcs[0] : 1.f, ps = fr ? rcs[1] : 0.f;
    if (tid < G * D) {
      const float px1 = bf2f(rq1), px2 = bf2f(rq2);
      const float x = fr ? rot2(px1, px2, pc, ps, d) : ((d & 1) ? px2 : px1);
      sq[tid / D][d] = x * scale_log2e;
    }
    if (own_new && tid < D) {
      const size_t crow = cbase + (size_t)(L - 1) * D;
      const float kv = rot2(bf2f(rk1), bf2f(rk2), pc, ps, d);  // same position L - 1 -> same cos / sin
      skn[d] = kv;
      svn[d] = bf2f(nv);
      rope.kc[crow + d] = f2bf(kv);  // for later steps (read back only after this launch)
      rope.vc[crow + d] = nv;
    }
  } else {
    if constexpr (PFT) {
      const int t0 = kstart + w * KT, t1 = t0 + NWV * KT;
      load_k(ka, t0); load_v(va, t0);
      load_k(kb2, t1); load_v(vb2, t1);
    }
    for (int i = tid; i < G * D; i += NTH) {
      const int g = i / D, d = i % D;
      const bf16_t* hp = q + (size_t)b * ldq + (hk * G + g) * D;
      sq[g][d] = (fr ? rot(hp, d, L - 1) : bf2f(hp[d])) * scale_log2e;
    }
  }
  if (own_new && !PRE) {
    const size_t crow = cbase + (size_t)(L - 1) * D;
    const bf16_t* kr = q + (size_t)b * ldq + (size_t)(H + hk) * D;
    const bf16_t* vr = q + (size_t)b * ldq + (size_t)(H + Hkv + hk) * D;
    for (int d = tid; d < D; d += NTH) {
      const float kv = rot(kr, d, L - 1);
      skn[d] = kv;
      svn[d] = bf2f(vr[d]);
      rope.kc[crow + d] = f2bf(kv);  // for later steps (read back only after this launch)
      rope.vc[crow + d] = vr[d];
    }
  }
  if constexpr (G > 1) {
    for (int i = tid; i < NWV * G * D; i += NTH) (&so[0][0][0])[i] = 0.f;
  }
  __syncthreads();
  if (own_new && w == 0) {  // score of the new key for each query head of this kv head
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float part = 0.f;
      for (int d = lane; d < D; d += 64) part += sq[g][d] * skn[d];
      part = wave_sum(part);
      if (lane == 0) ssn[g] = part;
    }
  }

  float m[G], l[G], acc[G][NSET][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY; l[g] = 0.f;
#pragma unroll
    for (int s = 0; s < NSET; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][s][e] = 0.f;
  }

  auto process = [&](const u32x4_t (&kv)[CPR], u32x4_t (&vv)[CPR], int t0) {
    const int nk = min(KT, kend - t0);
    // ---- scores ----
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
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const f32x4_t q0 = *(const f32x4_t*)&sq[g][dp * 8];
        const f32x4_t q1 = *(const f32x4_t*)&sq[g][dp * 8 + 4];
        float part = kf[0] * q0[0] + kf[1] * q0[1] + kf[2] * q0[2] + kf[3] * q0[3] +
                     kf[4] * q1[0] + kf[5] * q1[1] + kf[6] * q1[2] + kf[7] * q1[3];
        if constexpr (SHFL) {
#pragma unroll
          for (int o = 1; o < CPR; o <<= 1) part += __shfl_xor(part, o, 64);
          if (dp == 0) sp[w][g][c / CPR] = part;
        } else {
          spart[w][g * KT * CPR + c] = part;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- online softmax; lane = key ----
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float sc;
      if constexpr (SHFL) {
        sc = sp[w][g][lane];
      } else {
        sc = 0.f;
#pragma unroll
        for (int j = 0; j < CPR; ++j) sc += spart[w][g * KT * CPR + lane * CPR + j];
      }
      if (lane >= nk) sc = -INFINITY;
      const float tmax = wave_max(sc);
      const float m_new = fmaxf(m[g], tmax);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = exp2f(m[g] - m_use);
      const float p = exp2f(sc - m_use);
      l[g] = l[g] * alpha + wave_sum(p);
      m[g] = m_new;
      sp[w][g][lane] = p;
#pragma unroll
      for (int st = 0; st < NSET; ++st)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][st][e] *= alpha;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- P * V ----
    asm volatile("" ::: "memory");
    if constexpr (!VEARLY) load_v(vv, t0);
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
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float pk = sp[w][g][key];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[g][i % NSET][e] += pk * vf[e];
      }
    }
    __builtin_amdgcn_wave_barrier();
  };

  if constexpr (PFT) {  // two tiles in flight per wave: ka/va and kb2/vb2 alternate
    int t0 = kstart + w * KT;
    while (t0 < kend) {
      const int t1 = t0 + NWV * KT;
      process(ka, va, t0);
      if (t1 >= kend) break;
      const int t2 = t1 + NWV * KT;
      if (t2 < kend) { load_k(ka, t2); load_v(va, t2); }
      process(kb2, vb2, t1);
      if (t2 >= kend) break;
      const int t3 = t2 + NWV * KT;
      if (t3 < kend) { load_k(kb2, t3); load_v(vb2, t3); }
      t0 = t2;
    }
  } else {
    for (int t0 = kstart + w * KT; t0 < kend; t0 += NWV * KT) {
      u32x4_t kv[CPR], vv[CPR];
      load_k(kv, t0);
      if constexpr (VEARLY) load_v(vv, t0);
      process(kv, vv, t0);
    }
  }
  // ---- merge lanes -> per-wave O, then waves -> block partial ----
  // MHA (G = 1): every lane parks its accumulators in LDS with plain 16-B stores and the output
  // threads sum the (dim-slot, lane) entries that hold their dim. LDS float atomics — 5-6 lanes per
  // address — took 7.5 us of a 20 us batch-1 launch (bench/decode_trace.py), more than the K/V stream.
  if constexpr (G == 1) {
#pragma unroll
    for (int st = 0; st < NSET; ++st) {
      float* dst = &sacc[((w * NSET + st) * 64 + lane) * 8];
      *(f32x4_t*)dst = f32x4_t{acc[0][st][0], acc[0][st][1], acc[0][st][2], acc[0][st][3]};
      *(f32x4_t*)(dst + 4) = f32x4_t{acc[0][st][4], acc[0][st][5], acc[0][st][6], acc[0][st][7]};
    }
  } else {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int st = 0; st < NSET; ++st) {
        const int dp = (lane + 64 * st) % CPR;
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(&so[w][g][dp * 8 + e], acc[g][st][e]);
      }
  }
  if (lane == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) { swm[w][g] = m[g]; swl[w][g] = l[g]; }
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += NTH) {
    const int g = i / D, d = i % D;
    float M = fmaxf(fmaxf(swm[0][g], swm[1][g]), fmaxf(swm[2][g], swm[3][g]));
#pragma unroll
    for (int ww = 4; ww < NWV; ++ww) M = fmaxf(M, swm[ww][g]);
    if (own_new) M = fmaxf(M, ssn[g]);
    const float Mu = (M == -INFINITY) ? 0.f : M;
    float o = 0.f, ls = 0.f;
#pragma unroll
    for (int ww = 0; ww < NWV; ++ww) {
      const float f = exp2f(swm[ww][g] - Mu);
      float ow;
      if constexpr (G == 1) {
        // lane l's slot st holds dims 8 * ((64 st + l) % CPR) .. +7
        // fixed trip counts: all of a wave's reads are independent and issued back to back
        ow = 0.f;
        const int dp = d >> 3, e = d & 7;
#pragma unroll
        for (int st = 0; st < NSET; ++st) {
          const int l0 = ((dp - 64 * st) % CPR + CPR) % CPR;
#pragma unroll
          for (int j = 0; j < (64 + CPR - 1) / CPR; ++j) {
            const int l = l0 + j * CPR;
            if (l < 64) ow += sacc[((ww * NSET + st) * 64 + l) * 8 + e];
          }
        }
      } else {
        ow = so[ww][g][d];
      }
      o += ow * f;
      ls += swl[ww][g] * f;
    }
    if (own_new) {  // the new token's key: weight exp2(s - M), value straight from the qkv row
      const float f = exp2f(ssn[g] - Mu);
      o += svn[d] * f;
      ls += f;
    }
    dec_store(o, M, ls, b, hk * G + g, d, H, nsplit, split, D, po, pm, pl, out, ldo);
  }
  __shared__ int s_last;
  dec_finish<D, G, XC>(po, pm, pl, H, Hkv, nsplit, b, hk, cnt, out, ldo, &s_last);
}

// ------------------------------------------------------------------------------------------
// GQA decode attention on MFMA (G = H/Hkv query heads share one KV head: Llama-3-8B G=4,
// Llama-3-70B at TP=8 G=8). The G queries of a KV head form the N=16 side of
// v_mfma_f32_16x16x32_bf16 (zero-padded), so K and V are read once per KV head instead of being
// multiplied against each query on the VALU (the G >= 2 path of decode_attn_kernel is VALU-bound).
// Per wave and 64-key tile:
//   S^T[key][g] = K·Q^T : A = K rows straight from HBM into registers (non-temporal 16-B loads),
//                         B = Q^T (registers, loaded once);
//   softmax over the 64 keys of each query column: 16 values per lane + two cross-lane steps;
//   O^T[d][g] += V^T·P^T : B = P^T from the S^T registers (k index permuted), A = V^T read from the
//                         wave's private LDS copy of the V tile with ds_read_b64_tr_b16. The V tile
//                         is a contiguous [64 x D] block of the cache, so it is copied by LDS-DMA
//                         (global_load_lds, 1 KiB per wave-instruction) with an XOR chunk swizzle
//                         on the source address that makes the transposed reads conflict-free.
template <int D>
__device__ __forceinline__ int vswz(int r) {
  return D == 128 ? ((r & 7) << 1) : (((r >> 1) & 3) << 1);
}

template <int D, int G>
__global__ void __launch_bounds__(256)
decode_attn_gqa_kernel(const bf16_t* __restrict__ q, int ldq, const bf16_t* __restrict__ kc,
                       const bf16_t* __restrict__ vc, const int* __restrict__ lens, const int* __restrict__ slot,
                   const int* __restrict__ pre,
                       int H, int Hkv, int max_seq, int chunk_max, int nsplit, float scale_log2e,
                       float* __restrict__ po, float* __restrict__ pm, float* __restrict__ pl,
                       bf16_t* __restrict__ out, int ldo, int* __restrict__ cnt) {
  static_assert(D == 64 || D == 128, "GQA MFMA decode supports head dims 64 and 128");
  constexpr int KT = 64, NDS = D / 32, NDT = D / 16, NS = D / 8;   // d-steps (S), d-tiles (O), 16-B chunks/row
  constexpr int VBYTES = KT * D * 2, NDMA = VBYTES / 1024;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef __attribute__((address_space(1))) const void* gptr_t;
  __shared__ __attribute__((aligned(16))) char sv[4 * VBYTES];
  __shared__ float swm[4][16], swl[4][16];

  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int L = lens[b];
  DA_ASSERT(L >= 0 && L <= max_seq && slot[b] >= 0);
  const int chunk = dec_chunk(L, nsplit, chunk_max);
  const int kstart = split * chunk;
  const int kend = min(L, kstart + chunk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const size_t cbase = ((size_t)slot[b] * Hkv + hk) * (size_t)max_seq * D;
  const int P = pre ? pre[2 * b] : 0;  // shared-prefix keys [0, P) live in slot pre[2b + 1]
  const size_t pbase = P ? ((size_t)pre[2 * b + 1] * Hkv + hk) * (size_t)max_seq * D : cbase;
  DA_ASSERT(P % 64 == 0 && P <= L);
  char* myv = sv + w * VBYTES;

  bf16x8_t qf[NDS];
#pragma unroll
  for (int ds = 0; ds < NDS; ++ds) {
    if (fr < G) qf[ds] = *(const bf16x8_t*)(q + (size_t)b * ldq + (hk * G + fr) * D + ds * 32 + fg * 8);
    else qf[ds] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x4_t oacc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) oacc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_part = 0.f;

  for (int t0 = kstart + w * KT; t0 < kend; t0 += 4 * KT) {
    const int nk = min(KT, kend - t0);
    const bool shared = t0 < P;
    const bf16_t* kb = kc + (shared ? pbase : cbase) + (size_t)t0 * D;
    const bf16_t* vb = vc + (shared ? pbase : cbase) + (size_t)t0 * D;
    // ---- K straight to registers (A operand rows = keys), then the V tile by LDS-DMA ----
    u32x4_t kr[4][NDS];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds) {
        const int key = min(16 * t + fr, nk - 1);
        const u32x4_t* src = (const u32x4_t*)(kb + (size_t)key * D + ds * 32 + fg * 8);
        kr[t][ds] = __builtin_nontemporal_load(src);
      }
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int P = i * 64 + lane, row = P / NS, sl = P % NS;
      const int c = sl ^ vswz<D>(row);
      const int key = min(row, nk - 1);
      // aux 2 = nt (read once per step; see decode_attn_mfma1_kernel)
      __builtin_amdgcn_global_load_lds((gptr_t)(vb + (size_t)key * D + c * 8), (lds_ptr_t)(myv + i * 1024), 16, 0, 2);
    }
    // ---- S^T = K Q^T ----
    f32x4_t sacc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sacc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds) sacc[t] = mfma16(__builtin_bit_cast(bf16x8_t, kr[t][ds]), qf[ds], sacc[t]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = 16 * t + 4 * fg + i;
        const float sc = key < nk ? sacc[t][i] * scale_log2e : -INFINITY;
        sacc[t][i] = sc;
        mx = fmaxf(mx, sc);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = max_xhalf(mx);
    const float m_new = fmaxf(m_run, mx);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(sacc[t][i] - m_use);
        sacc[t][i] = p;
        psum += p;
      }
    l_part = l_part * alpha + psum;
#pragma unroll
    for (int i = 0; i < NDT; ++i) oacc[i] *= alpha;
    // ---- O^T += V^T P^T: k-step c covers keys 32c..32c+31; slot j -> key 32c + 16(j>>2) + 4fg + (j&3) ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's V DMA landed (wave-private LDS)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const u32x4_t pw = u32x4_t{pack_bf2(sacc[2 * c][0], sacc[2 * c][1]), pack_bf2(sacc[2 * c][2], sacc[2 * c][3]),
                                 pack_bf2(sacc[2 * c + 1][0], sacc[2 * c + 1][1]),
                                 pack_bf2(sacc[2 * c + 1][2], sacc[2 * c + 1][3])};
      const bf16x8_t pb = __builtin_bit_cast(bf16x8_t, pw);
      const int q4 = fr >> 2, p4 = fr & 3;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int col = dt * 16 + 4 * p4;                      // 4 columns of this lane's address
        const int r0 = 32 * c + 4 * fg + q4, r1 = r0 + 16;
        const s16x4_t lo = lds_read_tr16(myv + r0 * (D * 2) + (((col >> 3) ^ vswz<D>(r0)) << 4) + (col & 7) * 2);
        const s16x4_t hi = lds_read_tr16(myv + r1 * (D * 2) + (((col >> 3) ^ vswz<D>(r1)) << 4) + (col & 7) * 2);
        const bf16x8_t va = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        oacc[dt] = mfma16(va, pb, oacc[dt]);
      }
    }
    // the next tile's DMA rewrites this wave's V region: finish the tr-reads first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // ---- merge the 4 waves: per-query (m, l) and O^T partials through LDS ----
  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot = sum_xhalf(l_tot);
  if (fg == 0) { swm[w][fr] = m_run; swl[w][fr] = l_tot; }
  __syncthreads();  // every wave is done with its V region
  float* so = (float*)sv;  // [4][16][D]
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) so[(w * 16 + fr) * D + dt * 16 + 4 * fg + i] = oacc[dt][i];
  __syncthreads();
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    const float M = fmaxf(fmaxf(swm[0][g], swm[1][g]), fmaxf(swm[2][g], swm[3][g]));
    const float Mu = (M == -INFINITY) ? 0.f : M;
    float o = 0.f, ls = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = exp2f(swm[ww][g] - Mu);
      o += so[(ww * 16 + g) * D + d] * f;
      ls += swl[ww][g] * f;
    }
    dec_store(o, M, ls, b, hk * G + g, d, H, nsplit, split, D, po, pm, pl, out, ldo);
  }
  __shared__ int s_last;
  dec_finish<D, G>(po, pm, pl, H, Hkv, nsplit, b, hk, cnt, out, ldo, &s_last);
}

// MHA decode attention on MFMA for few (row, kv head) pairs (batch 1..: the p50 path). The VALU
// kernel (decode_attn_kernel, G = 1) spends ~2k VALU cycles per 64-key tile on its dot products, so
// at batch 1 — 32 pairs, a few tiles per wave — it is issue-bound, not HBM-bound (profiles/r5/
// decode_mfma1/: 2.9 TB/s even with the K/V in the MALL). Here the single query is the N = 16 side of
// v_mfma_f32_16x16x32_bf16 (column 0 live, 15 zero), exactly the GQA kernel's data path with G = 1:
// K rows straight into registers (non-temporal), the V tile by LDS-DMA into a wave-private region
// (XOR chunk swizzle within groups of 4 chunks, so D = 96's 12 chunks per row stay in the row),
// S^T = K Q^T, softmax over column 0, O^T += V^T P^T with transposed LDS reads. chunk <= 512 keys per
// split (host-checked) gives every wave at most TWO tiles, and both are requested before any is
// waited for: one HBM round trip per workgroup. XC: same-XCD split exchange (see dec_finish).
template <int D>
__device__ __forceinline__ int vswz1(int r) {
  return D == 96 ? ((r >> 1) & 3) : vswz<D>(r);
}

// RP: fused RoPE + new-token KV write (DecRope, as decode_attn_kernel): q is the raw qkv row; q is
// rotated into LDS while the tiles fly, key L - 1 enters as one extra online-softmax term of the
// split that holds it (taken from the qkv row, written into the cache for later steps).
template <int D, bool XC, bool RP>
__global__ void __launch_bounds__(256)
decode_attn_mfma1_kernel(const bf16_t* __restrict__ q, int ldq, const bf16_t* __restrict__ kc,
                         const bf16_t* __restrict__ vc, const int* __restrict__ lens, const int* __restrict__ slot,
                         const int* __restrict__ pre, int H, int Hkv, int max_seq, int chunk_max, int nsplit,
                         float scale_log2e, float* __restrict__ po, float* __restrict__ pm, float* __restrict__ pl,
                         bf16_t* __restrict__ out, int ldo, int* __restrict__ cnt, DecRope rope) {
  static_assert(D == 64 || D == 96 || D == 128, "head dim");
  constexpr int KT = 64, NDS = D / 32, NDT = D / 16, NS = D / 8;
  constexpr int VBYTES = KT * D * 2, NDMA = VBYTES / 1024;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef __attribute__((address_space(1))) const void* gptr_t;
  __shared__ __attribute__((aligned(16))) char sv[4 * 2 * VBYTES];  // two tiles per wave
  __shared__ float swm[4], swl[4];

  int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  if constexpr (XC) {  // the same-XCD mapping of decode_attn_kernel
    const int wl = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int s8 = wl >> 3, pair = (s8 / nsplit) * 8 + (wl & 7);
    split = s8 % nsplit;
    hk = pair % Hkv;
    b = pair / Hkv;
  }
  const int L = lens[b];
  DA_ASSERT(L >= 0 && L <= max_seq && slot[b] >= 0);
  const int chunk = dec_chunk(L, nsplit, chunk_max);
  DA_ASSERT(chunk <= 8 * KT);
  const int kstart = split * chunk;
  const bool own_new = RP && kstart <= L - 1 && L - 1 < kstart + chunk;  // this split holds key L - 1
  const int kend = min(RP ? L - 1 : L, kstart + chunk);                  // RP: key L - 1 from the qkv row
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const size_t cbase = ((size_t)slot[b] * Hkv + hk) * (size_t)max_seq * D;
  const int P = pre ? pre[2 * b] : 0;  // shared-prefix keys [0, P) live in slot pre[2b + 1]
  const size_t pbase = P ? ((size_t)pre[2 * b + 1] * Hkv + hk) * (size_t)max_seq * D : cbase;
  DA_ASSERT(P % 64 == 0 && P <= L);
  DA_ASSERT(!RP || rope.pos[b] == L - 1);

  // ---- both tiles of this wave requested up front (branch-free: an empty tile reads key 0 of
  //      the row's own slot, valid memory whose scores are masked) ----
  const int ta = kstart + w * KT, tb = ta + 4 * KT;
  u32x4_t kr[2][4][NDS];
  auto issue = [&](int j, int t0) {
    const int nk = kend - t0;
    const bool shared = t0 < P;
    const bf16_t* kb = nk > 0 ? kc + (shared ? pbase : cbase) + (size_t)t0 * D : kc + cbase;
    const bf16_t* vb = nk > 0 ? vc + (shared ? pbase : cbase) + (size_t)t0 * D : vc + cbase;
    const int last = nk > 0 ? min(KT, nk) - 1 : 0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds) {
        const int key = min(16 * t + fr, last);
        kr[j][t][ds] = __builtin_nontemporal_load((const u32x4_t*)(kb + (size_t)key * D + ds * 32 + fg * 8));
      }
    char* myv = sv + (w * 2 + j) * VBYTES;
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int pc = i * 64 + lane, row = pc / NS, sl = pc % NS;
      const int c = sl ^ vswz1<D>(row);
      const int key = min(row, last);
      // aux 2 = nt: the KV stream is read once per step; allocating it in L2 / MALL cost the GEMVs
      // that follow ~3 % (their weights lose cache residency): profiles/r5/decode_mfma1/
      __builtin_amdgcn_global_load_lds((gptr_t)(vb + (size_t)key * D + c * 8), (lds_ptr_t)(myv + i * 1024), 16, 0, 2);
    }
  };
  issue(0, ta);
  issue(1, tb);

  bf16x8_t qf[NDS];
  [[maybe_unused]] __shared__ __attribute__((aligned(16))) bf16_t sqb[RP ? D : 1];
  [[maybe_unused]] __shared__ float skn[RP ? D : 1], svn[RP ? D : 1];
  [[maybe_unused]] __shared__ float ssn;
  if constexpr (RP) {
    // rotate q (and the new key) at position L - 1, rounded to bf16 like the rope_cache kernel
    constexpr int HALF = D / 2;
    const bf16_t* qrow = q + (size_t)b * ldq;
    if (tid < D) {
      const int d = tid, i = d >> 1;
      const float c = rope.cs[((size_t)(L - 1) * HALF + i) * 2], sn = rope.cs[((size_t)(L - 1) * HALF + i) * 2 + 1];
      auto rot = [&](const bf16_t* hp) {
        const float x1 = bf2f(hp[d & ~1]), x2 = bf2f(hp[d | 1]);
        return f2bf((d & 1) ? x2 * c + x1 * sn : x1 * c - x2 * sn);
      };
      sqb[d] = rot(qrow + hk * D);
      if (own_new) {
        const bf16_t kn = rot(qrow + (size_t)(H + hk) * D), vn = qrow[(size_t)(H + Hkv + hk) * D + d];
        skn[d] = bf2f(kn);
        svn[d] = bf2f(vn);
        const size_t crow = cbase + (size_t)(L - 1) * D;
        rope.kc[crow + d] = kn;  // for later steps (read back only after this launch)
        rope.vc[crow + d] = vn;
      }
    }
    __syncthreads();
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds)
      qf[ds] = fr == 0 ? *(const bf16x8_t*)(sqb + ds * 32 + fg * 8) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    if (own_new && w == 0) {  // score of the new key (log2 units)
      float part = 0.f;
      for (int d = lane; d < D; d += 64) part += bf2f(sqb[d]) * skn[d];
      part = wave_sum(part);
      if (lane == 0) ssn = part * scale_log2e;
    }
  } else {
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds)
      qf[ds] = fr == 0 ? *(const bf16x8_t*)(q + (size_t)b * ldq + hk * D + ds * 32 + fg * 8)
                       : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x4_t oacc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) oacc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_part = 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // both tiles' K registers and V regions landed

  auto process = [&](int j, int t0) {
    const int nk = kend - t0;
    f32x4_t sacc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sacc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < NDS; ++ds) sacc[t] = mfma16(__builtin_bit_cast(bf16x8_t, kr[j][t][ds]), qf[ds], sacc[t]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = 16 * t + 4 * fg + i;
        const float sc = key < nk ? sacc[t][i] * scale_log2e : -INFINITY;
        sacc[t][i] = sc;
        mx = fmaxf(mx, sc);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = max_xhalf(mx);
    const float m_new = fmaxf(m_run, mx);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(sacc[t][i] - m_use);
        sacc[t][i] = p;
        psum += p;
      }
    l_part = l_part * alpha + psum;
#pragma unroll
    for (int i = 0; i < NDT; ++i) oacc[i] *= alpha;
    const char* myv = sv + (w * 2 + j) * VBYTES;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const u32x4_t pw = u32x4_t{pack_bf2(sacc[2 * c][0], sacc[2 * c][1]), pack_bf2(sacc[2 * c][2], sacc[2 * c][3]),
                                 pack_bf2(sacc[2 * c + 1][0], sacc[2 * c + 1][1]),
                                 pack_bf2(sacc[2 * c + 1][2], sacc[2 * c + 1][3])};
      const bf16x8_t pb = __builtin_bit_cast(bf16x8_t, pw);
      const int q4 = fr >> 2, p4 = fr & 3;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int col = dt * 16 + 4 * p4;
        const int r0 = 32 * c + 4 * fg + q4, r1 = r0 + 16;
        const s16x4_t lo = lds_read_tr16(myv + r0 * (D * 2) + (((col >> 3) ^ vswz1<D>(r0)) << 4) + (col & 7) * 2);
        const s16x4_t hi = lds_read_tr16(myv + r1 * (D * 2) + (((col >> 3) ^ vswz1<D>(r1)) << 4) + (col & 7) * 2);
        const bf16x8_t va = bf16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        oacc[dt] = mfma16(va, pb, oacc[dt]);
      }
    }
  };
  if (ta < kend) process(0, ta);
  if (tb < kend) process(1, tb);

  // ---- merge the 4 waves (query column 0: lanes fr == 0) through LDS ----
  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot = sum_xhalf(l_tot);
  if (lane == 0) { swm[w] = m_run; swl[w] = l_tot; }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with its V regions
  float* so = (float*)sv;  // [4][D]: column 0 of each wave's O^T
  if (fr == 0) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) so[w * D + dt * 16 + 4 * fg + i] = oacc[dt][i];
  }
  __syncthreads();
  for (int d = tid; d < D; d += 256) {
    float M = fmaxf(fmaxf(swm[0], swm[1]), fmaxf(swm[2], swm[3]));
    if (own_new) M = fmaxf(M, ssn);
    const float Mu = (M == -INFINITY) ? 0.f : M;
    float o = 0.f, ls = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = exp2f(swm[ww] - Mu);
      o += so[ww * D + d] * f;
      ls += swl[ww] * f;
    }
    if (own_new) {  // the new token's key: weight exp2(s - M), value straight from the qkv row
      const float f = exp2f(ssn - Mu);
      o += svn[d] * f;
      ls += f;
    }
    dec_store(o, M, ls, b, hk, d, H, nsplit, split, D, po, pm, pl, out, ldo);
  }
  __shared__ int s_last;
  dec_finish<D, 1, XC>(po, pm, pl, H, Hkv, nsplit, b, hk, cnt, out, ldo, &s_last);
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

template <int D, int VAR>
static int launch_decode_v(int G, dim3 grid, hipStream_t s, const bf16_t* q, int ldq, const bf16_t* kc,
                           const bf16_t* vc, const int* lens, const int* slot, const int* pre, int H, int Hkv, int max_seq, int chunk,
                           int nsplit, float sl2e, float* po, float* pm, float* pl, bf16_t* out, int ldo,
                           int* cnt, DecRope rope) {
#define DEC(GG) decode_attn_kernel<D, GG, VAR><<<grid, 256, 0, s>>>(q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, \
                                                                     chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope)
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

// GQA groups (G >= 2) take the MFMA kernel: 1.8x (Llama-3-8B, G=4) to 5x (Llama-3-70B TP=8, G=8)
// over the VALU path (profiles/decode_attn_gqa_mfma_r1.json); the VALU kernel covers the other
// head dims. MHA (G = 1) decode prefetches each wave's next tile (VAR bit 2) when the launch has
// few (row, kv head) pairs (B * Hkv <= 32: latency-bound), else streams with V issued with K.
//
// Measured on MI355X (profiles/decode_attn_variants_r1.json): non-temporal K/V loads + V issued with
// K reach 6.5 TB/s for MHA (G = 1, Phi-3); with G >= 2 the extra V registers cost more occupancy
// than they buy, so those keep V after the scores (nt loads only).
constexpr int kDecPrefetchPairs = 32;

template <int D>
static int launch_decode(int G, dim3 grid, hipStream_t s, const bf16_t* q, int ldq, const bf16_t* kc,
                         const bf16_t* vc, const int* lens, const int* slot, const int* pre, int H, int Hkv, int max_seq, int chunk,
                         int nsplit, float sl2e, float* po, float* pm, float* pl, bf16_t* out, int ldo,
                         int* cnt, DecRope rope, int xc) {
  static int mfma1 = -1;
  if (mfma1 < 0) {
    const char* e = getenv("DA_DECODE_MFMA1");
    mfma1 = (e && e[0] == '0') ? 0 : 1;
  }
  if (mfma1 && G == 1 && (int)(grid.y * grid.z) <= kDecPrefetchPairs && chunk <= 512) {
    if (xc && ((grid.y * grid.z) % 8 || !cnt || nsplit < 2)) return (int)hipErrorInvalidValue;
#define M1(XCV, RPV) decode_attn_mfma1_kernel<D, XCV, RPV><<<grid, 256, 0, s>>>(q, ldq, kc, vc, lens, slot, pre, H, Hkv, \
                         max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope)
    if (xc) { if (rope.cs) M1(true, true); else M1(true, false); }
    else { if (rope.cs) M1(false, true); else M1(false, false); }
#undef M1
    return (int)hipGetLastError();
  }
  if (xc) {  // same-XCD split exchange (cached ws / counters): the prefetching MHA form only
    if (G != 1 || (int)(grid.y * grid.z) > kDecPrefetchPairs || (grid.y * grid.z) % 8 || !cnt || nsplit < 2)
      return (int)hipErrorInvalidValue;
    return launch_decode_v<D, 15>(G, grid, s, q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope);
  }
  if (G == 1) {
    if ((int)(grid.y * grid.z) <= kDecPrefetchPairs)
      return launch_decode_v<D, 7>(G, grid, s, q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope);
    return launch_decode_v<D, 3>(G, grid, s, q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope);
  }
  if (rope.cs) return (int)hipErrorInvalidValue;  // fused RoPE: MHA kernel only
  if constexpr (D == 64 || D == 128) {
    switch (G) {
      case 2: decode_attn_gqa_kernel<D, 2><<<grid, 256, 0, s>>>(q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt); break;
      case 4: decode_attn_gqa_kernel<D, 4><<<grid, 256, 0, s>>>(q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt); break;
      case 8: decode_attn_gqa_kernel<D, 8><<<grid, 256, 0, s>>>(q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt); break;
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
  return launch_decode_v<D, 1>(G, grid, s, q, ldq, kc, vc, lens, slot, pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope);
}

// ws must hold B*H*nsplit*(D+2) floats. chunk = keys per split (multiple of 64).
// pre (nullable): int32 [B][2] = (P, prefix slot) per row — keys [0, P) of row b are read from the
// prefix slot (a prompt head shared by the whole batch, stored once; P % 64 == 0 so no 64-key tile
// straddles the two sources). Every row of the batch reads the same prefix lines, so they are served
// from L2 / MALL instead of HBM.
// counters (nullable): int32 [B * Hkv], all zero, left zero by every launch -> the splits are merged
// inside the attention kernel (last split per (b, kv head)); null -> separate combine launch. With
// counters, ws and counters must be uncached allocations (da_malloc_uncached).
DA_EXPORT int da_malloc_uncached(long long bytes, void** out) {
  hipError_t e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*out, 0, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

// cos_sin / pos (both null, or both set): fused RoPE + new-token KV-cache write (MHA only; q is
// then the raw qkv row, see DecRope).
static int decode_attn_impl(const void* q, int ldq, const void* k_cache, const void* v_cache, const void* lens,
                            const void* slot, const void* pre, int B, int H, int Hkv, int D, int max_seq, int chunk,
                            int nsplit, float scale, void* ws, void* o, int ldo, void* counters, const void* cos_sin,
                            const void* pos, int xc, void* stream) {
  bf16_t* out = (bf16_t*)o;
  int* cnt = (int*)counters;
  if (H % Hkv || chunk % 64 || nsplit < 1 || (long)chunk * nsplit < 1) return (int)hipErrorInvalidValue;
  if ((cos_sin == nullptr) != (pos == nullptr) || (cos_sin && (H != Hkv || ldq < (H + 2 * Hkv) * D)))
    return (int)hipErrorInvalidValue;
  DecRope rope{(bf16_t*)k_cache, (bf16_t*)v_cache, (const float*)cos_sin, (const int*)pos};
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
                                     (const int*)lens, (const int*)slot, (const int*)pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope, xc);
      break;
    case 96: err = launch_decode<96>(G, grid, s, (const bf16_t*)q, ldq, (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                                     (const int*)lens, (const int*)slot, (const int*)pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope, xc);
      break;
    case 128: err = launch_decode<128>(G, grid, s, (const bf16_t*)q, ldq, (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                                       (const int*)lens, (const int*)slot, (const int*)pre, H, Hkv, max_seq, chunk, nsplit, sl2e, po, pm, pl, out, ldo, cnt, rope, xc);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  if (err) return err;
  if (nsplit == 1 || cnt) return 0;
  dim3 cgrid(H, B);
  switch (D) {
    case 64: decode_combine_kernel<64><<<cgrid, 64, 0, s>>>(po, pm, pl, H, nsplit, (bf16_t*)o, ldo); break;
    case 96: decode_combine_kernel<96><<<cgrid, 128, 0, s>>>(po, pm, pl, H, nsplit, (bf16_t*)o, ldo); break;
    case 128: decode_combine_kernel<128><<<cgrid, 128, 0, s>>>(po, pm, pl, H, nsplit, (bf16_t*)o, ldo); break;
  }
  DA_LAUNCH_CHECK();
}

// xc = 1: same-XCD split exchange (ws / counters in ordinary device memory; the caller has checked
// the launch's workgroup -> XCD round-robin with the placement probe). 0: uncached ws / counters.
DA_EXPORT int da_decode_attn(const void* q, int ldq, const void* k_cache, const void* v_cache, const void* lens,
                             const void* slot, const void* pre, int B, int H, int Hkv, int D, int max_seq, int chunk,
                             int nsplit, float scale, void* ws, void* o, int ldo, void* counters, const void* cos_sin,
                             const void* pos, int xc, void* stream) {
  return decode_attn_impl(q, ldq, k_cache, v_cache, lens, slot, pre, B, H, Hkv, D, max_seq, chunk, nsplit, scale, ws,
                          o, ldo, counters, cos_sin, pos, xc, stream);
}

// Dispatch order of the flash kernels (FaPrefix::rev, fa_block): causal longest query blocks first
// and the query blocks of one (sequence, kv head) pair on one XCD (737 -> 778 TF/s on the Phi-3 QA
// chunk, profiles/r4/flash_order/).
constexpr int kFaDispatch = 3;

// fp16 (the encoder's DTYPE=fp16): bidirectional or causal, no shared prefix, 4 waves x 32 queries
DA_EXPORT int da_flash_attn_f16(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv,
                                const void* cu_seqlens, int B, int max_seqlen, int H, int Hkv, int D, int causal,
                                float scale, void* o, int ldo, void* stream) {
  if (H % Hkv || ldq % 8 || ldk % 8 || ldv % 8 || ldo % 4) return (int)hipErrorInvalidValue;
  if (B == 0 || max_seqlen == 0) return 0;
  const FaPrefix pre{nullptr, nullptr, 0, 0, kFaDispatch};
  dim3 grid((max_seqlen + 127) / 128, H, B);
  hipStream_t s = (hipStream_t)stream;
#define FA_ARGS16 (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, ldq, ldk, ldv, (const int*)cu_seqlens, H, Hkv, \
                  causal, scale * 1.4426950408889634f, (bf16_t*)o, ldo, pre
  switch (D) {
    case 64: flash_attn_v2_kernel<64, 4, 1, F16T><<<grid, 256, FA2Cfg<64, 4, 1>::SMEM, s>>>(FA_ARGS16); break;
    case 96: flash_attn_v2_kernel<96, 4, 1, F16T><<<grid, 256, FA2Cfg<96, 4, 1>::SMEM, s>>>(FA_ARGS16); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FA_ARGS16
  return (int)hipGetLastError();
}

template <int NW, int QH>
static int launch_fa2(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv, const void* cu_seqlens,
                      int B, int max_seqlen, int H, int Hkv, int D, int causal, float sl2e, void* o, int ldo,
                      FaPrefix pre, hipStream_t s) {
  static bool attr_set = false;
  if constexpr (NW * QH <= 8) {
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)flash_attn_v2_kernel<128, NW, QH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                FA2Cfg<128, NW, QH>::SMEM);
      attr_set = true;
    }
  }
  dim3 grid((max_seqlen + 32 * QH * NW - 1) / (32 * QH * NW), H, B);
#define FA_ARGS (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, ldq, ldk, ldv, (const int*)cu_seqlens, H, Hkv, \
                causal, sl2e, (bf16_t*)o, ldo, pre
  switch (D) {
    case 32: flash_attn_v2_kernel<32, NW, QH><<<grid, 64 * NW, FA2Cfg<32, NW, QH>::SMEM, s>>>(FA_ARGS); break;
    case 64: flash_attn_v2_kernel<64, NW, QH><<<grid, 64 * NW, FA2Cfg<64, NW, QH>::SMEM, s>>>(FA_ARGS); break;
    // 8 waves x 64 queries exceed 256 VGPRs (spills) above D = 64: not instantiated
    case 96:
      if constexpr (NW * QH <= 8) flash_attn_v2_kernel<96, NW, QH><<<grid, 64 * NW, FA2Cfg<96, NW, QH>::SMEM, s>>>(FA_ARGS);
      else return (int)hipErrorInvalidValue;
      break;
    case 128:
      if constexpr (NW * QH <= 8) flash_attn_v2_kernel<128, NW, QH><<<grid, 64 * NW, FA2Cfg<128, NW, QH>::SMEM, s>>>(FA_ARGS);
      else return (int)hipErrorInvalidValue;
      break;
    default: return (int)hipErrorInvalidValue;
  }
#undef FA_ARGS
  return (int)hipGetLastError();
}

// Causal D = 96 (the Phi-3 prefill) runs the software-pipelined kernel (flash_attn_pipe: 576 -> 656
// TF/s; the short bidirectional BGE sequences, 8 tiles, lose to its longer pipeline fill, 617 -> 531
// at D = 64, profiles/r2/attn_bench_v5.txt) with the speculative softmax (654 -> 689 TF/s,
// profiles/r3/attn_bench_spec.txt) and LDS-DMA K / V tiles when the prefix is whole 64-key tiles and
// the operands 16-B aligned (711 TF/s); every other shape the 4-wave flash_attn_v2_kernel (8 waves
// at D = 128: Llama-3 prefill, profiles/r2/attn_bench_v4.txt).
template <int D, bool DMA>
static constexpr int fa_pipe_smem() {
  return 3 * ((DMA ? 64 * D * 2 : FA2Cfg<D, 4, 1>::KBUF) + FA2Cfg<D, 4, 1>::VBUF);
}

template <bool DMA>
static int launch_fa_pipe(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv, const void* cu_seqlens,
                          int B, int max_seqlen, int H, int Hkv, int causal, float sl2e, void* o, int ldo,
                          FaPrefix pre, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)flash_attn_pipe_kernel<96, true, DMA>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, fa_pipe_smem<96, DMA>());
    attr_set = true;
  }
  dim3 grid((max_seqlen + 127) / 128, H, B);
  flash_attn_pipe_kernel<96, true, DMA><<<grid, 256, fa_pipe_smem<96, DMA>(), s>>>(
      (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, ldq, ldk, ldv, (const int*)cu_seqlens, H, Hkv, causal, sl2e,
      (bf16_t*)o, ldo, pre);
  return (int)hipGetLastError();
}

// pre_k / pre_v: shared-prefix K/V of KV head 0 in a cache slot (nullptr / pre_len 0: none),
// pre_hstride: elements between KV heads there (max_seq * D).
// kv_slot / kv_pos (nullable; per token, int32): the sequences' own keys are read from the KV cache
// k_cache / v_cache [slots, Hkv, max_seq, D] (pre_hstride = max_seq * D) instead of k / v — causal
// D = 96 only.
DA_EXPORT int da_flash_attn_v2(const void* q, const void* k, const void* v, int ldq, int ldk, int ldv,
                               const void* cu_seqlens, int B, int max_seqlen, int H, int Hkv, int D, int causal,
                               float scale, void* o, int ldo, const void* pre_k, const void* pre_v,
                               long long pre_hstride, int pre_len, const void* kv_slot, const void* kv_pos,
                               const void* k_cache, const void* v_cache, void* stream) {
  const bool from_cache = kv_slot != nullptr;
  if (from_cache) {
    if (!causal || D != 96 || !kv_pos || !k_cache || !v_cache || pre_hstride < (long long)D ||
        pre_hstride % D || ((uintptr_t)k_cache | (uintptr_t)v_cache) % 16)
      return (int)hipErrorInvalidValue;
    k = k_cache; v = v_cache; ldk = ldv = D;  // rows D apart inside a (slot, head) block
  }
  if (H % Hkv || ldq % 8 || ldk % 8 || ldv % 8 || ldo % 4) return (int)hipErrorInvalidValue;
  if (pre_len < 0 || (pre_len > 0 && (!pre_k || !pre_v || pre_hstride < (long long)pre_len * D)))
    return (int)hipErrorInvalidValue;
  if (B == 0 || max_seqlen == 0) return 0;
  const float sl2e = scale * 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  const FaPrefix pre{(const bf16_t*)pre_k, (const bf16_t*)pre_v, pre_hstride, pre_len, kFaDispatch,
                     (const int*)kv_slot, (const int*)kv_pos, (const bf16_t*)k_cache, (const bf16_t*)v_cache,
                     from_cache ? (long long)Hkv * pre_hstride : 0LL};
  if (causal && D == 96) {
    const bool dma = pre_len % 64 == 0 && ((uintptr_t)k | (uintptr_t)v | (uintptr_t)pre_k | (uintptr_t)pre_v) % 16 == 0;
    if (dma) return launch_fa_pipe<true>(q, k, v, ldq, ldk, ldv, cu_seqlens, B, max_seqlen, H, Hkv, causal, sl2e, o, ldo, pre, s);
    return launch_fa_pipe<false>(q, k, v, ldq, ldk, ldv, cu_seqlens, B, max_seqlen, H, Hkv, causal, sl2e, o, ldo, pre, s);
  }
  if (D == 128) return launch_fa2<8, 1>(q, k, v, ldq, ldk, ldv, cu_seqlens, B, max_seqlen, H, Hkv, D, causal, sl2e, o, ldo, pre, s);
  return launch_fa2<4, 1>(q, k, v, ldq, ldk, ldv, cu_seqlens, B, max_seqlen, H, Hkv, D, causal, sl2e, o, ldo, pre, s);
}
