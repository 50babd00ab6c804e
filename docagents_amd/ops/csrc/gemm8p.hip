// 256x256 bf16 GEMM for prefill-sized M, phase-split ("8-phase") schedule:
//   C[M,N] = epi(A[M,K] . W[N,K]^T)
//
// MI355X-first structure (cdna_hip_programming.md §5 "The 256² 8-phase template", T1-T5; the
// schedule and its hazard proofs below are this file's own):
//  * 512 threads = 8 waves in two groups G0 (waves 0-3) and G1 (waves 4-7); every SIMD hosts one
//    wave of each group. Wave (g, wn) owns a 128x64 output block made of four 64x32 quadrants
//    Q(ih, jh): rows ih*128 + g*64 .. +64 of the tile, columns jh*128 + wn*32 .. +32.
//  * A K-tile (BK = 64) is staged as four 16 KiB half-tiles A0 (tile rows 0-127), A1 (128-255),
//    B0 (tile columns 0-127), B1 (128-255) by LDS-DMA (global_load_lds_dwordx4, lane-linear image,
//    XOR swizzle applied on the per-lane SOURCE address and undone on the ds_read_b128 address).
//    Two 64 KiB buffers: tile t lives in buffer t & 1.
//  * A K-tile is four phases; each phase = {fragment reads + DMA issue + counted waits} [barrier]
//    {16 MFMA 16x16x32 of one quadrant} [barrier]:
//        phase 0: read A0, B0 -> Q(0,0)     phase 1: read B1 -> Q(0,1)
//        phase 2: read A1     -> Q(1,1)     phase 3: (no reads) -> Q(1,0)
//    G1 runs one barrier behind G0, so on every SIMD one wave's MFMAs cover its partner's LDS reads,
//    DMA issue and waits (the read bubble that capped the lock-step gemm256 at MFMA busy 57 %).
//  * Half-tile X of tile t+2 is DMA'd into buffer t & 1 one phase after X's last read in tile t
//    (A0, B0 in phase 1; B1 in phase 2; A1 in phase 3), so each fill has 4-6 phases (~1.5 K-tiles)
//    to land instead of one K-step, with 8-14 DMAs per wave in flight across barriers (raw
//    s_barrier, counted vmcnt, never vmcnt(0) in the steady state).
//  * Hazards (global barrier index: G0's read segment of global phase p lies between barriers
//    2p-1 and 2p, its MFMA segment between 2p and 2p+1; G1's segments are one barrier later; every
//    wave ends its read segment with lgkmcnt(0)):
//      WAR: a half-tile last read in phase p is complete before barrier 2p+1 (G1), and refills are
//           issued in read segments of phase p+1 (after barrier 2p+1 for both groups).
//      RAW: every wave waits (vmcnt) for its share of a half-tile in its read segment of phase p-1
//           or earlier and reads it in phase p: G1's wait precedes barrier 2p-1, G0's read follows it.
//  * Bijective XCD remap + grouped-M tile order; epilogue (bias / GELU / SwiGLU / residual) in
//    registers, bf16 tile staged through LDS, 16-B coalesced row stores.
#include "gemm.h"

#include <type_traits>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* gptr_t;

namespace {
constexpr int BM = 256, BN = 256;
constexpr int HALF = 16384;                  // one half-tile: 128 rows x 64 bf16
constexpr int BUF = 4 * HALF;                // one K-tile
constexpr int OFF_A0 = 0, OFF_A1 = HALF, OFF_B0 = 2 * HALF, OFF_B1 = 3 * HALF;
constexpr int SROW = 64 * 2 + 16;            // epilogue staging row stride (bytes)
constexpr int STAGING = 8 * 128 * SROW;      // 144 KiB
constexpr int SMEM = (2 * BUF > STAGING) ? 2 * BUF : STAGING;
}  // namespace

#define VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

template <int EPI, int SCHED>
__global__ void __launch_bounds__(512)
gemm8p_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fg = lane >> 4;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, ntm * ntn);
  constexpr int GROUP = 4;
  const int gid = t / (GROUP * ntn);
  const int first_m = gid * GROUP;
  const int gsz = min(ntm - first_m, GROUP);
  const int tin = t % (GROUP * ntn);
  const int m0 = (first_m + tin % gsz) * BM, n0 = (tin / gsz) * BN;

  // ---- LDS-DMA sources. Wave w fills rows (2w + j) * 8 + lane / 8 of each half-tile (j = 0, 1),
  //      16-B chunk (lane & 7) ^ swz(row) of the row's 128 bytes (rows clamped into range: clamped
  //      rows only feed outputs that are never stored).
  // buffer_load ... lds: a buffer resource at the tile's first A row / W row, one 32-bit per-lane
  // row offset fixed for the whole K loop, the K-step as the scalar soffset (no per-issue VALU)
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.A + (size_t)m0 * p.lda * 2), (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.W + (size_t)n0 * p.K * 2), (short)0, 0x7ffffff0, 0x00020000);
  unsigned soff[4][2];  // [A0, A1, B0, B1][j]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = (wid * 2 + j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      soff[h][j] = (unsigned)(min(m0 + h * 128 + r, p.M - 1) - m0) * (unsigned)(p.lda * 2) + c * 16;
      soff[2 + h][j] = (unsigned)(min(n0 + h * 128 + r, p.N - 1) - n0) * (unsigned)(p.K * 2) + c * 16;
    }
  }
  const int ldsw = wid * 2048;  // wave's 2 KiB of each half-tile (wave-uniform: M0 stays scalar)
#define ISSUE(X, OFF, KT, B)                                                                                   \
  do {                                                                                                         \
    char* d_ = smem + (B) * BUF + (OFF) + ldsw;                                                                \
    __builtin_amdgcn_raw_ptr_buffer_load_lds((X) < 2 ? rsa : rsw, (lds_ptr_t)(d_), 16, soff[X][0], (KT) * 128, 0, 0); \
    __builtin_amdgcn_raw_ptr_buffer_load_lds((X) < 2 ? rsa : rsw, (lds_ptr_t)(d_ + 1024), 16, soff[X][1], (KT) * 128, 0, 0); \
  } while (0)

  // ---- fragment read offsets: row wg*64 + i*16 + fr of an A half (wn*32 + j*16 + fr of a B half),
  //      16-B chunk kk*4 + fg, swizzled by ((row >> 1) & 7) = fr >> 1 (i*16, wg*64, wn*32 keep it)
  int aoff[2], boff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int cs = ((kk * 4 + fg) ^ (fr >> 1)) << 4;
    aoff[kk] = (wg * 64 + fr) * 128 + cs;
    boff[kk] = (wn * 32 + fr) * 128 + cs;
  }

  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t ra[2][4], rb0[2][2], rb1[2][2];
  auto read_a = [&](const char* base) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) ra[kk][i] = *(const bf16x8_t*)(base + aoff[kk] + i * 2048);
  };
  auto read_b = [&](bf16x8_t (&rb)[2][2], const char* base) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) rb[kk][j] = *(const bf16x8_t*)(base + boff[kk] + j * 2048);
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lgkm0 = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
#define QUAD(IH, JH, RB)                                                                      \
  do {                                                                                        \
    __builtin_amdgcn_s_setprio(1);                                                            \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                          \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                             \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                             \
      acc[IH][JH][i][j] = mfma16(ra[kk][i], RB[kk][j], acc[IH][JH][i][j]);                    \
    __builtin_amdgcn_s_setprio(0);                                                            \
  } while (0)

  const int nk = p.K / 64;  // >= 2 (host-checked)
  using T_ = std::true_type;
  using F_ = std::false_type;

  if constexpr (SCHED == 0) {
  // ---- prologue: tiles 0 and 1 in flight; A0, B0, B1 of tile 0 landed (A1 of tile 0 is waited in
  //      phase 1 like every A1)
  ISSUE(0, OFF_A0, 0, 0); ISSUE(2, OFF_B0, 0, 0); ISSUE(3, OFF_B1, 0, 0); ISSUE(1, OFF_A1, 0, 0);
  ISSUE(0, OFF_A0, 1, 1); ISSUE(2, OFF_B0, 1, 1); ISSUE(3, OFF_B1, 1, 1); ISSUE(1, OFF_A1, 1, 1);
  VMCNT(10);
  bar();
  if (wg) bar();  // G1 runs one barrier behind

  // One K-tile. FILL = 1: tile kt + 2 exists and is issued into this buffer as its halves free up.
  // Steady-state DMA order per wave: ... A1(t) | A0 B0(t+1) | B1(t+1) | A1(t+1) | A0 B0(t+2) ...
  //   phase 1 waits A1(t)          : 12 newer (tile t+1: 8, A0 B0 of t+2: 4)  -> vmcnt(12)
  //   phase 3 waits A0 B0 B1(t+1)  : 10 newer (A1(t+1): 2, tile t+2: 8)       -> vmcnt(10)
  // Tail (no fills): phase 1 keeps tile t+1's 8 in flight (if it exists), phase 3 keeps A1(t+1)'s 2.
  auto ktile = [&](int kt, auto fill_tag, auto next_tag) __attribute__((always_inline)) {
    constexpr bool FILL = decltype(fill_tag)::value;
    constexpr bool NEXT = decltype(next_tag)::value;  // tile kt + 1 exists
    const int b = kt & 1;
    const char* base = smem + b * BUF;
    // phase 0
    read_a(base + OFF_A0);
    read_b(rb0, base + OFF_B0);
    lgkm0();
    bar();
    QUAD(0, 0, rb0);
    bar();
    // phase 1
    read_b(rb1, base + OFF_B1);
    if constexpr (FILL) { ISSUE(0, OFF_A0, kt + 2, b); ISSUE(2, OFF_B0, kt + 2, b); VMCNT(12); }
    else if constexpr (NEXT) { VMCNT(8); }
    else { VMCNT(0); }
    lgkm0();
    bar();
    QUAD(0, 1, rb1);
    bar();
    // phase 2
    read_a(base + OFF_A1);
    if constexpr (FILL) ISSUE(3, OFF_B1, kt + 2, b);
    lgkm0();
    bar();
    QUAD(1, 1, rb1);
    bar();
    // phase 3
    if constexpr (FILL) { ISSUE(1, OFF_A1, kt + 2, b); VMCNT(10); }
    else if constexpr (NEXT) { VMCNT(2); }
    bar();
    QUAD(1, 0, rb0);
    bar();
  };
  int kt = 0;
  for (; kt < nk - 2; ++kt) ktile(kt, T_{}, T_{});
  ktile(kt, F_{}, T_{});
  ktile(kt + 1, F_{}, F_{});
  } else {
  // ---- 2 phases per K-tile, 32 MFMAs (two quadrants) per segment: half the barriers per MFMA.
  //   phase A: read A0 B0 B1 -> Q(0,0) Q(0,1); issue A1(t+1) (its slot's last read: phase B of t-1)
  //   phase B: read A1       -> Q(1,1) Q(1,0); issue A0 B0 B1(t+2) (last read: phase A of t)
  //   DMA order per wave: ... A0 B0 B1(t+1) | A1(t+1) | A0 B0 B1(t+2) | A1(t+2) ...
  //   phase A waits A1(t)          : A0 B0 B1(t+1), A1(t+1) newer -> vmcnt(8)
  //   phase B waits A0 B0 B1(t+1)  : A1(t+1), A0 B0 B1(t+2) newer -> vmcnt(8) (2 in the last fill-less tile)
  ISSUE(0, OFF_A0, 0, 0); ISSUE(2, OFF_B0, 0, 0); ISSUE(3, OFF_B1, 0, 0); ISSUE(1, OFF_A1, 0, 0);
  ISSUE(0, OFF_A0, 1, 1); ISSUE(2, OFF_B0, 1, 1); ISSUE(3, OFF_B1, 1, 1);
  VMCNT(8);
  bar();
  if (wg) bar();  // G1 runs one barrier behind
  auto ktile2 = [&](int kt, auto fill_tag, auto next_tag) __attribute__((always_inline)) {
    constexpr bool FILL = decltype(fill_tag)::value;  // tile kt + 2 exists
    constexpr bool NEXT = decltype(next_tag)::value;  // tile kt + 1 exists
    const int b = kt & 1;
    const char* base = smem + b * BUF;
    read_a(base + OFF_A0);
    read_b(rb0, base + OFF_B0);
    read_b(rb1, base + OFF_B1);
    if constexpr (NEXT) { ISSUE(1, OFF_A1, kt + 1, b ^ 1); VMCNT(8); }
    else { VMCNT(0); }
    lgkm0();
    bar();
    QUAD(0, 0, rb0);
    QUAD(0, 1, rb1);
    bar();
    read_a(base + OFF_A1);
    if constexpr (FILL) { ISSUE(0, OFF_A0, kt + 2, b); ISSUE(2, OFF_B0, kt + 2, b); ISSUE(3, OFF_B1, kt + 2, b); VMCNT(8); }
    else if constexpr (NEXT) { VMCNT(2); }
    lgkm0();
    bar();
    QUAD(1, 1, rb1);
    QUAD(1, 0, rb0);
    bar();
  };
  int kt = 0;
  for (; kt < nk - 2; ++kt) ktile2(kt, T_{}, T_{});
  ktile2(kt, F_{}, T_{});
  ktile2(kt + 1, F_{}, F_{});
  }
  if (!wg) bar();  // re-align the groups
  __syncthreads();

  // ---- epilogue: registers -> (bias / GELU / SwiGLU) -> bf16 staging -> coalesced stores.
  //      Staged row lr = ih*64 + i*16 + fg*4 + q (tile row ih*128 + wg*64 + (lr & 63)),
  //      staged column lc = jh*32 + j*16 + fr (tile column jh*128 + wn*32 + (lc & 31)).
  char* st = smem + wid * 128 * SROW;
  if constexpr (EPI == EPI_SWIGLU) {
    // W rows interleaved in 16-row (gate, up) groups: j = 0 is gate, j = 1 is up of output
    // columns (n0 + jh*128 + wn*32) / 2 + fr
#pragma unroll
    for (int ih = 0; ih < 2; ++ih)
#pragma unroll
      for (int jh = 0; jh < 2; ++jh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = silu(acc[ih][jh][i][0][q]) * acc[ih][jh][i][1][q];
            *(bf16_t*)(st + (ih * 64 + i * 16 + fg * 4 + q) * SROW + (jh * 16 + fr) * 2) = f2bf(v);
          }
  } else {
    float bv[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    if (p.bias) {
#pragma unroll
      for (int jh = 0; jh < 2; ++jh)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int gc = n0 + jh * 128 + wn * 32 + j * 16 + fr;
          bv[jh][j] = gc < p.N ? bf2f(p.bias[gc]) : 0.f;
        }
    }
#pragma unroll
    for (int ih = 0; ih < 2; ++ih)
#pragma unroll
      for (int jh = 0; jh < 2; ++jh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float v = acc[ih][jh][i][j][q] + bv[jh][j];
              if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
              *(bf16_t*)(st + (ih * 64 + i * 16 + fg * 4 + q) * SROW + (jh * 32 + j * 16 + fr) * 2) = f2bf(v);
            }
  }
  __syncthreads();
  constexpr bool SW = (EPI == EPI_SWIGLU);
  constexpr int HC = SW ? 16 : 32;   // staged columns per jh half (one contiguous global run)
  constexpr int CPR = 2 * HC / 8;    // 16-B chunks per staged row
  constexpr int RPI = 64 / CPR;      // rows per store instruction
  const int ch = lane % CPR;
  const int jh = ch / (HC / 8);
  const int cc = (ch % (HC / 8)) * 8;
  const int gcol = (SW ? n0 / 2 : n0) + jh * (SW ? 64 : 128) + wn * HC + cc;
  const int ncols = SW ? p.N / 2 : p.N;
  for (int lr = lane / CPR; lr < 128; lr += RPI) {
    const int gm = m0 + (lr >> 6) * 128 + wg * 64 + (lr & 63);
    if (gm >= p.M || gcol >= ncols) continue;
    u32x4_t v = *(const u32x4_t*)(st + lr * SROW + (jh * HC + cc) * 2);
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
#undef ISSUE
#undef QUAD
}

// Schedule select for A/B runs (da_set_gemm8p_sched; DA_GEMM8P_SCHED): 0 = 4 phases per K-tile
// , 2 = 2 phases per K-tile (default: half the barriers per MFMA, +4.5 % measured).
static int g_sched = 2;
DA_EXPORT void da_set_gemm8p_sched(int v) { g_sched = v; }

template <int SCHED>
static int launch8p(const GemmArgs& a, int epi, hipStream_t s, dim3 grid, dim3 block) {
  switch (epi) {
    case EPI_NONE: gemm8p_kernel<EPI_NONE, SCHED><<<grid, block, 0, s>>>(a); break;
    case EPI_BIAS: gemm8p_kernel<EPI_BIAS, SCHED><<<grid, block, 0, s>>>(a); break;
    case EPI_GELU: gemm8p_kernel<EPI_GELU, SCHED><<<grid, block, 0, s>>>(a); break;
    case EPI_SWIGLU: gemm8p_kernel<EPI_SWIGLU, SCHED><<<grid, block, 0, s>>>(a); break;
    case EPI_RESID: gemm8p_kernel<EPI_RESID, SCHED><<<grid, block, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

int launch_gemm8p(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.K < 128 || a.K % 64) return (int)hipErrorInvalidValue;
  // buffer resources span 256 rows from the tile start (num_records 2 GiB)
  if ((size_t)256 * a.lda * 2 >= 0x7ffffff0ull || (size_t)256 * a.K * 2 >= 0x7ffffff0ull) return (int)hipErrorInvalidValue;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn), block(512);
  return g_sched == 2 ? launch8p<2>(a, epi, s, grid, block) : launch8p<0>(a, epi, s, grid, block);
}
