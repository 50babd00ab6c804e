// 256x256-tile bf16 GEMM with FOUR waves (one per SIMD), each owning a 128 x 128 output block —
// the power-capped alternative to gemm256.hip's 8-wave (128 x 64 per wave) kernel.
//
// Why (MI355X_MICROARCH 'DVFS give-back'; cdna_hip_programming.md §5.4 rule 28): prefill GEMMs run
// for seconds at the board power cap, where throughput follows energy per MFMA. A 128 x 128 wave
// block feeds 64 MFMAs (16x16x32) from 16 fragment reads per 32-deep K-step instead of 32 MFMAs from
// 12, so LDS read bytes per FLOP halve; with one wave per SIMD and its whole 512-register file,
// the next K-step's fragments are read into a second register set WHILE the current step's MFMAs
// run, so no barrier ever waits on an LDS read.
//
// Schedule (per wave; 4-slot LDS ring of 32-deep K-steps, 32 KiB each = A 256x32 + W 256x32 bf16):
//   prologue: DMA tiles 0..3 -> slots 0..3; wait tile 0; barrier; read tile 0 -> F0; wait tile 1
//   step h:   barrier B_h           (publishes tile h+1; every wave finished reading tile h)
//             DMA tile h+4 -> slot h%4   (tile h is already in registers: the slot is free)
//             read tile h+1 -> F[(h+1)%2]  ||  64 MFMAs on F[h%2]
//             lgkmcnt(0); vmcnt(16)  (tile h+2 landed; tiles h+3, h+4 stay in flight)
// RAW on the LDS-DMA data: a wave's own counted vmcnt, then a barrier the reader has passed
// (tile h+2 waited at the end of step h, read in step h+1 after B_{h+1}). WAR: slot h%4 is
// refilled only after B_h, which every wave reaches after its reads of tile h retired.
// LDS image: 64-B rows (32 bf16), 16-B chunk c of row r stored at chunk c ^ (((r >> 3) & 1) << 1)
// (conflict-free ds_read_b128 for the 16-row x 4-chunk fragment read), applied on the DMA SOURCE
// address because the LDS-DMA image is lane-linear (rule 21).
#include "gemm.h"

typedef __attribute__((address_space(3))) void* lds_ptr_t;

namespace {
constexpr int BM = 256, BN = 256, HK = 32;
constexpr int A_BYTES = BM * HK * 2, SLOT = (BM + BN) * HK * 2;  // 16 KiB, 32 KiB
constexpr int TM = 128, TN = 128;              // per-wave output block
constexpr int SROW = TN * 2 + 16;              // epilogue staging row stride (bytes)
constexpr int STAGING = 4 * TM * SROW;         // 136 KiB
constexpr int smem_bytes(int ns) { return ns * SLOT > STAGING ? ns * SLOT : STAGING; }
}  // namespace

// NS: LDS ring slots (4, or 5 = all 160 KiB of LDS). MODE 0: double fragment register set + copy;
// MODE 1: one register set, split-phase reads (no copies). MODE 2: MODE 1 without the in-loop DMA
// (timing diagnostic only: results are wrong). MODE 3: MODE 1 with register-staged loads
// (buffer_load -> VGPR -> ds_write_b128) instead of LDS-DMA.
template <int EPI, int NS, int MODE>
__global__ void __launch_bounds__(256)
gemm256w4_kernel(GemmArgs p) {
  static_assert(smem_bytes(NS) <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes(NS)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: LDS-DMA bases (M0) stay scalar
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, ntm * ntn);
  constexpr int GROUP = 4;
  const int gid = t / (GROUP * ntn);
  const int first_m = gid * GROUP;
  const int gsz = min(ntm - first_m, GROUP);
  const int tin = t % (GROUP * ntn);
  const int m0 = (first_m + tin % gsz) * BM, n0 = (tin / gsz) * BN;

  // DMA sources: each wave fills 4 x 16 rows of A and of W per slot (1 KiB per instruction), as
  // buffer_load ... lds: one 32-bit per-lane row offset (fixed for the whole K loop) + the K-step
  // as a scalar soffset, so a DMA issue carries no 64-bit address arithmetic.
  const __amdgpu_buffer_rsrc_t rsa =
      __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.A + (size_t)m0 * p.lda * 2), (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.W + (size_t)n0 * p.K * 2), (short)0, 0x7ffffff0, 0x00020000);
  unsigned avo[4], bvo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wid * 4 + j) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ (((r >> 3) & 1) << 1);
    avo[j] = (unsigned)((min(m0 + r, p.M - 1) - m0) * p.lda * 2 + c * 16);
    bvo[j] = (unsigned)((min(n0 + r, p.N - 1) - n0) * p.K * 2 + c * 16);
  }
#define W4_DMA(J, H, SA, SB)                                                                                 \
  do {                                                                                                        \
    if constexpr ((J) < 4)                                                                                    \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr_t)((SA) + (wid * 4 + (J)) * 1024), 16, avo[J], \
                                               (H) * 64, 0, 0);                                              \
    else                                                                                                      \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr_t)((SB) + (wid * 4 + (J) - 4) * 1024), 16,     \
                                               bvo[(J) - 4], (H) * 64, 0, 0);                                \
  } while (0)
  const int nh = p.K / HK;
  // Fragment reads are inline-asm ds_read_b128 so hipcc neither drains the LDS-DMA queue in front of
  // them (it cannot prove the ring slots disjoint) nor waits on them early; their completion is
  // one explicit lgkmcnt(0) that names every destination ("+v"), cdna_hip_programming.md §5.7 (ii).
  // Row base + i*16 keeps ((r >> 3) & 1) = (fr >> 3) & 1, so one address VGPR per operand serves
  // all eight reads through the 16-bit offset field.
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const unsigned rd = fr * 64 + ((fg ^ (((fr >> 3) & 1) << 1)) << 4);
  const unsigned aoff = lds0 + wm * TM * 64 + rd, boff = lds0 + A_BYTES + wn * TN * 64 + rd;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t ca[8], cb[8], na[8], nb[8];

  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto fill = [&](int h, int slot) {
    char* sa = smem + slot * SLOT;
    char* sb = sa + A_BYTES;
    W4_DMA(0, h, sa, sb); W4_DMA(1, h, sa, sb); W4_DMA(2, h, sa, sb); W4_DMA(3, h, sa, sb);
    W4_DMA(4, h, sa, sb); W4_DMA(5, h, sa, sb); W4_DMA(6, h, sa, sb); W4_DMA(7, h, sa, sb);
  };
  constexpr int VM_STEADY = (NS - 2) * 8;  // after issuing tile h+NS: tiles h+3 .. h+NS may stay in flight
// (s_nop 0: hipcc may hand this statement the address VGPRs of the LDS-DMA it just issued)
#define W4_RD(dst, addr, off) \
  asm volatile("s_nop 0\n\tds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(off))
#define W4_WAIT_READS(X, Y)                                                                           \
  asm volatile("s_waitcnt lgkmcnt(0)"                                                                 \
               : "+v"(X[0]), "+v"(X[1]), "+v"(X[2]), "+v"(X[3]), "+v"(X[4]), "+v"(X[5]), "+v"(X[6]),  \
                 "+v"(X[7]), "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2]), "+v"(Y[3]), "+v"(Y[4]), "+v"(Y[5]),  \
                 "+v"(Y[6]), "+v"(Y[7]))
#define W4_VMWAIT(N) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory")
  // one 32-deep K-step: MFMAs on (CA, CB) = tile h; fragment reads of tile h+1 into (NA, NB);
  // LDS-DMA of tile h+NS into slot fs. 8 groups of {one DMA, two reads, eight MFMAs}, order pinned.
#define W4_GROUP(I, CA, CB, NA, NB)                                                                       \
  W4_DMA(I, ft, sa, sb);                                                                                  \
  W4_RD(NA[I], ra, (I) * 1024);                                                                           \
  W4_RD(NB[I], rb, (I) * 1024);                                                                           \
  __builtin_amdgcn_sched_barrier(0);                                                                      \
  _Pragma("unroll") for (int j = 0; j < 8; ++j) acc[I][j] = mfma16(CA[I], CB[j], acc[I][j]);              \
  __builtin_amdgcn_sched_barrier(0);
#define W4_STEP(CA, CB, NA, NB)                                                                           \
  {                                                                                                       \
    bar();                                                                                                \
    const unsigned ra = aoff + rs * SLOT, rb = boff + rs * SLOT;                                          \
    const int ft = min(h + NS, nh - 1);                                                                   \
    char* sa = smem + fs * SLOT;                                                                          \
    char* sb = sa + A_BYTES;                                                                              \
    W4_GROUP(0, CA, CB, NA, NB) W4_GROUP(1, CA, CB, NA, NB) W4_GROUP(2, CA, CB, NA, NB)                   \
    W4_GROUP(3, CA, CB, NA, NB) W4_GROUP(4, CA, CB, NA, NB) W4_GROUP(5, CA, CB, NA, NB)                   \
    W4_GROUP(6, CA, CB, NA, NB) W4_GROUP(7, CA, CB, NA, NB)                                               \
    W4_WAIT_READS(NA, NB);                                                                                \
    W4_VMWAIT(VM_STEADY);                                                                                 \
    ++h;                                                                                                  \
    fs = (fs + 1 == NS) ? 0 : fs + 1;                                                                     \
    rs = (rs + 1 == NS) ? 0 : rs + 1;                                                                     \
  }

  if constexpr (MODE == 0) {
#pragma unroll
  for (int t = 0; t < NS; ++t) fill(min(t, nh - 1), t);
  W4_VMWAIT((NS - 1) * 8);                                   // tile 0
  bar();
#pragma unroll
  for (int i = 0; i < 8; ++i) W4_RD(na[i], aoff, i * 1024);
#pragma unroll
  for (int i = 0; i < 8; ++i) W4_RD(nb[i], boff, i * 1024);
  W4_WAIT_READS(na, nb);
  W4_VMWAIT((NS - 2) * 8);                                   // tile 1
  int h = 0, fs = 0, rs = 1;
  // one step per iteration + a fragment register copy: unrolling by two with the sets swapping
  // roles makes hipcc shuffle the 256 accumulators between AGPRs and VGPRs and spill in the loop
#pragma nounroll
  while (h < nh) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { ca[i] = na[i]; cb[i] = nb[i]; }
    W4_STEP(ca, cb, na, nb)
  }
  } else {
    // Copy-free split-phase schedule (one register set, 64 fragment VGPRs):
    //   phase 1: MFMAs (a_i, b_0..3) for all i  || read b_4..7 of tile h (slot published at B_{h-1})
    //   phase 2: MFMAs (a_i, b_4..7); after row i: read a_i of tile h+1; early: b_0..3 of tile h+1
    // DMA in step h: tile h+NS-1 -> the slot of tile h-1, whose last reads (b_4..7 in step h-1)
    // retired before B_h. Tile h+1 must be published at B_h (its a / b_0..3 are read in phase 2).
#define W4_NOPRD(dst, addr, off) \
  asm volatile("s_nop 1\n\tds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"(off))
#define W4_WAIT4(X) \
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(X[4]), "+v"(X[5]), "+v"(X[6]), "+v"(X[7]) : : "memory")
#define W4_WAIT12(X, Y)                                                                               \
  asm volatile("s_waitcnt lgkmcnt(0)"                                                                 \
               : "+v"(X[0]), "+v"(X[1]), "+v"(X[2]), "+v"(X[3]), "+v"(X[4]), "+v"(X[5]), "+v"(X[6]),  \
                 "+v"(X[7]), "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2]), "+v"(Y[3])                    \
               :                                                                                      \
               : "memory")
    constexpr int VM1 = (NS - 3) * 8;  // after issuing tile h+NS-1: tiles h+3 .. h+NS-1 in flight
    // MODE 3 (register staging): stg[] holds tile h+2 (loaded during step h-1); step h writes it
    // to the slot of tile h+2 (= slot of tile h-2, free) and loads tile h+3. hipcc counts these
    // loads itself (no LDS-DMA in flight), so its own vmcnt waits sit in front of each ds_write.
    u32x4_t stg[8];
    auto ld_stage = [&](int t) {
#pragma unroll
      for (int j = 0; j < 4; ++j) stg[j] = __builtin_amdgcn_raw_buffer_load_b128(rsa, avo[j], t * 64, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) stg[4 + j] = __builtin_amdgcn_raw_buffer_load_b128(rsb, bvo[j], t * 64, 0);
    };
    auto st_stage_one = [&](int j, int slot) {
      char* d = smem + slot * SLOT + (j < 4 ? 0 : A_BYTES) + (wid * 4 + (j & 3)) * 1024 + lane * 16;
      *(u32x4_t*)d = stg[j];
    };
    if constexpr (MODE == 3) {
      ld_stage(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) st_stage_one(j, 0);
      ld_stage(min(1, nh - 1));
#pragma unroll
      for (int j = 0; j < 8; ++j) st_stage_one(j, 1);
      ld_stage(min(2, nh - 1));
      __syncthreads();
    } else {
#pragma unroll
      for (int t = 0; t < NS - 1; ++t) fill(min(t, nh - 1), t);
      W4_VMWAIT((NS - 2) * 8);                                 // tile 0
      bar();
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) W4_RD(ca[i], aoff, i * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) W4_RD(cb[j], boff, j * 1024);
    W4_WAIT12(ca, cb);
    if constexpr (MODE != 3) W4_VMWAIT(VM1);                   // tile 1
    int h = 0, cs = 0;  // cs = slot of tile h
#pragma nounroll
    while (h < nh) {
      bar();                                                   // B_h
      const int ns = (cs + 1 == NS) ? 0 : cs + 1;              // slot of tile h+1
      const int fs = (cs == 0) ? NS - 1 : cs - 1;              // slot of tile h-1 (refilled)
      const int ft = min(h + NS - 1, nh - 1);
      const int ws = (cs + 2) & 3;                             // MODE 3: slot of tile h+2
      const int lt = min(h + 3, nh - 1);                       // MODE 3: tile loaded this step
      char* sa = smem + fs * SLOT;
      char* sb = sa + A_BYTES;
      const unsigned rb_cur = boff + cs * SLOT;
      const unsigned ra_nxt = aoff + ns * SLOT, rb_nxt = boff + ns * SLOT;
      // phase 1: DMA (8) + b_4..7 of tile h, 32 MFMAs on b_0..3
#define W4_P1(I)                                                                                          \
      if constexpr (MODE == 3) {                                                                          \
        st_stage_one(I, ws);                                                                              \
        if constexpr (I < 4)                                                                              \
          stg[I] = __builtin_amdgcn_raw_buffer_load_b128(rsa, avo[I], lt * 64, 0);                        \
        else                                                                                              \
          stg[I] = __builtin_amdgcn_raw_buffer_load_b128(rsb, bvo[(I) - 4], lt * 64, 0);                  \
      } else if constexpr (MODE == 4) W4_DMA(I, 0, sa, sb);                                              \
      else if constexpr (MODE != 2) W4_DMA(I, ft, sa, sb);                                               \
      if constexpr (I < 4) W4_RD(cb[4 + I], rb_cur, (4 + I) * 1024);                                      \
      __builtin_amdgcn_sched_barrier(0);                                                                  \
      _Pragma("unroll") for (int j = 0; j < 4; ++j) acc[I][j] = mfma16(ca[I], cb[j], acc[I][j]);          \
      __builtin_amdgcn_sched_barrier(0);
      W4_P1(0) W4_P1(1) W4_P1(2) W4_P1(3) W4_P1(4) W4_P1(5) W4_P1(6) W4_P1(7)
#undef W4_P1
      W4_WAIT4(cb);
      // phase 2: 32 MFMAs on b_4..7; a_i of tile h+1 after row i; b_0..3 of tile h+1 up front
#define W4_P2(I)                                                                                          \
      if constexpr (I < 4) W4_RD(cb[I], rb_nxt, (I) * 1024);                                              \
      __builtin_amdgcn_sched_barrier(0);                                                                  \
      _Pragma("unroll") for (int j = 4; j < 8; ++j) acc[I][j] = mfma16(ca[I], cb[j], acc[I][j]);          \
      __builtin_amdgcn_sched_barrier(0);                                                                  \
      W4_NOPRD(ca[I], ra_nxt, (I) * 1024);
      W4_P2(0) W4_P2(1) W4_P2(2) W4_P2(3) W4_P2(4) W4_P2(5) W4_P2(6) W4_P2(7)
#undef W4_P2
      W4_WAIT12(ca, cb);
      if constexpr (MODE != 3) W4_VMWAIT(VM1);                 // tile h+2 landed
      ++h;
      cs = ns;
    }
#undef W4_NOPRD
#undef W4_WAIT4
#undef W4_WAIT12
  }
#undef W4_STEP
#undef W4_GROUP
#undef W4_VMWAIT
#undef W4_WAIT_READS
#undef W4_RD
#undef W4_DMA
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();

  // ---- epilogue: registers -> (bias / GELU / SwiGLU) -> bf16 staging -> coalesced stores ----
  char* st = smem + wid * TM * SROW;
  const int row0 = m0 + wm * TM, col0 = n0 + wn * TN;
  if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int pq = 0; pq < 4; ++pq)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = silu(acc[i][2 * pq][q]) * acc[i][2 * pq + 1][q];
          *(bf16_t*)(st + (i * 16 + fg * 4 + q) * SROW + (pq * 16 + fr) * 2) = f2bf(v);
        }
  } else {
    float bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gc = col0 + j * 16 + fr;
      bv[j] = (p.bias && gc < p.N) ? bf2f(p.bias[gc]) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = acc[i][j][q] + bv[j];
          if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
          *(bf16_t*)(st + (i * 16 + fg * 4 + q) * SROW + (j * 16 + fr) * 2) = f2bf(v);
        }
  }
  __syncthreads();
  constexpr int OC = (EPI == EPI_SWIGLU) ? TN / 2 : TN;
  constexpr int CPR = OC / 8;
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

static int g_w4_cfg = 0;  // bit0: 5-slot ring, bit1: split-phase schedule (A/B knobs)
DA_EXPORT void da_set_gemm_w4_cfg(int v) { g_w4_cfg = v; }

template <int NS, int MODE>
static int launch_w4(const GemmArgs& a, int epi, hipStream_t s, dim3 grid, dim3 block) {
  switch (epi) {
    case EPI_NONE: gemm256w4_kernel<EPI_NONE, NS, MODE><<<grid, block, 0, s>>>(a); break;
    case EPI_BIAS: gemm256w4_kernel<EPI_BIAS, NS, MODE><<<grid, block, 0, s>>>(a); break;
    case EPI_GELU: gemm256w4_kernel<EPI_GELU, NS, MODE><<<grid, block, 0, s>>>(a); break;
    case EPI_SWIGLU: gemm256w4_kernel<EPI_SWIGLU, NS, MODE><<<grid, block, 0, s>>>(a); break;
    case EPI_RESID: gemm256w4_kernel<EPI_RESID, NS, MODE><<<grid, block, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

int launch_gemm256w4(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.K % HK) return (int)hipErrorInvalidValue;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn), block(256);
  switch (g_w4_cfg & 7) {
    case 0: return launch_w4<4, 0>(a, epi, s, grid, block);
    case 1: return launch_w4<5, 0>(a, epi, s, grid, block);
    case 2: return launch_w4<4, 1>(a, epi, s, grid, block);
    case 3: return launch_w4<5, 1>(a, epi, s, grid, block);
    case 4: return launch_w4<4, 2>(a, epi, s, grid, block);  // DIAGNOSTIC: no in-loop DMA (wrong results)
    case 5: return launch_w4<4, 3>(a, epi, s, grid, block);
    default: return launch_w4<4, 4>(a, epi, s, grid, block);  // DIAGNOSTIC: DMA always re-reads K-step 0
  }
}
