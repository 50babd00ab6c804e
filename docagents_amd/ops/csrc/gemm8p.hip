// BMx256 bf16 GEMM (BM = 256 or 128) for prefill-sized M, phase-split ping-pong schedule:
//   C[M,N] = epi(A[M,K] . W[N,K]^T)
//
// MI355X-first structure (cdna_hip_programming.md §5 "The 256² 8-phase template", T1-T5; the
// schedule and its hazard proofs below are this file's own):
//  * 512 threads = 8 waves in two groups G0 (waves 0-3) and G1 (waves 4-7); every SIMD hosts one
//    wave of each group. Wave (g, wn) owns a (BM/2)x64 output block made of four (BM/4)x32
//    quadrants Q(ih, jh): rows ih*BM/2 + g*BM/4 .. + BM/4, columns jh*128 + wn*32 .. +32.
//  * A K-tile (BK = 64) is staged as four half-tiles A0 (tile rows 0..BM/2-1), A1, B0 (tile columns
//    0-127), B1 (128-255) by LDS-DMA (buffer_load ... lds: lane-linear image, the bank-conflict XOR
//    swizzle applied on the per-lane SOURCE offset and undone on the ds_read_b128 address; the
//    K-step is the scalar soffset, so an issue costs no VALU). Two buffers: tile t lives in t & 1.
//  * A K-tile is two phases; each phase = {fragment reads + DMA issue + counted wait} [barrier]
//    {MFMA 16x16x32 of two quadrants} [barrier]:
//        phase A: read A0, B0, B1 -> Q(0,0), Q(0,1);   issue A1(t+1)        (slot last read: B of t-1)
//        phase B: read A1         -> Q(1,1), Q(1,0);   issue A0 B0 B1(t+2)  (slots last read: A of t)
//    G1 runs one barrier behind G0, so on every SIMD one wave's MFMAs cover its partner's LDS reads,
//    DMA issue and waits (the read bubble that capped the lock-step gemm256 at MFMA busy 57 %).
//    Measured (profiles/r2/ab_gemm8p_vs_hipblaslt.txt): 4 phases per K-tile (one quadrant per
//    segment) -4.5 %, balanced 8/4/8/4 reads -2 %: the barriers, not the LDS reads, bound a segment.
//  * Hazards (global barrier index: G0's read segment of global phase p lies between barriers
//    2p-1 and 2p, its MFMA segment between 2p and 2p+1; G1's segments are one barrier later; every
//    wave ends its read segment with lgkmcnt(0)):
//      WAR: a half-tile last read in phase p is complete before barrier 2p+1 (G1), and refills are
//           issued in read segments of phase p+1 or later (after barrier 2p+1 for both groups).
//      RAW: every wave waits (vmcnt) for its share of a half-tile in its read segment of phase p-1
//           or earlier and reads it in phase p: G1's wait precedes barrier 2p-1, G0's read follows it.
//  * Bijective XCD remap + grouped-M tile order; epilogue (bias / GELU / SwiGLU / residual) in
//    registers, bf16 tile staged through LDS, 16-B coalesced row stores. EPI_ROPE (the prefill QKV
//    projection): each 16-B chunk holds 4 interleaved rotary pairs of one head, rotated on its way
//    out, and the k / v chunks are also stored into the KV cache — the rope_cache pass folded in
//    (kv_out = 0: ONLY into the cache; the prefill attention then reads its keys there, and the
//    epilogue writes 2/3 fewer bytes of the QKV tile — the store tail is issue-bound).
//  * PERSIST: one workgroup per CU walks tile ids b, b + G, ... (G a multiple of 8: each id stays on
//    the workgroup's XCD); the staged rows go to registers, then the next tile's prologue DMA is
//    issued before this tile's stores (profiles/r5/gemm_persist/: +0.3..1 %, not for EPI_ROPE).
#include "gemm.h"

#include <cstdlib>
#include <type_traits>

typedef __attribute__((address_space(3))) void* lds_ptr_t;

namespace {
constexpr int BN = 256;
constexpr int HALF_B = 16384;                // B half-tile: 128 rows x 64 bf16
constexpr int SROW = 64 * 2 + 16;            // epilogue staging row stride (bytes)
}  // namespace

template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int EPI, int BM, typename T = BF16T, bool PERSIST = false>
__global__ void __launch_bounds__(512)
gemm8p_kernel(GemmArgs p) {
  static_assert(BM == 256 || BM == 128, "BM");
  constexpr int HALF_A = BM / 2 * 128;       // A half-tile: BM/2 rows x 64 bf16
  constexpr int OFF_A0 = 0, OFF_A1 = HALF_A, OFF_B0 = 2 * HALF_A, OFF_B1 = 2 * HALF_A + HALF_B;
  constexpr int BUF = 2 * HALF_A + 2 * HALF_B;
  constexpr int STAGING = 8 * (BM / 2) * SROW;
  constexpr int SMEM = (2 * BUF > STAGING) ? 2 * BUF : STAGING;
  constexpr int MI = BM / 64;                // 16-row fragments per quadrant
  constexpr int QR = BM / 4;                 // quadrant rows
  constexpr int NA = BM / 128;               // DMA instructions per wave per A half-tile
  // DMA instructions per wave, newest first, between a wait and the half-tile it retires:
  constexpr int CNT_AB = 2 * NA + 4;         // A1 + A0 B0 B1 of the next tiles (steady state)
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = wid >> 2, wn = wid & 3;
  const int fr = lane & 15, fg = lane >> 4;

  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN, ntiles = ntm * ntn;
  const int GROUP = p.group > 0 ? p.group : 4;
  // tile id -> (m0, n0): bijective XCD remap, then grouped-M order. PERSIST: workgroup b runs ids
  // b, b + G, b + 2G, ... (G = gridDim.x, a multiple of 8, so every id it runs maps to its own XCD)
  auto tile_of = [&](int id, int& m0_, int& n0_) __attribute__((always_inline)) {
    const int t = xcd_remap(id, ntiles);
    const int gid = t / (GROUP * ntn);
    const int first_m = gid * GROUP;
    const int gsz = min(ntm - first_m, GROUP);
    const int tin = t % (GROUP * ntn);
    m0_ = (first_m + tin % gsz) * BM;
    n0_ = (tin / gsz) * BN;
  };
  int id = blockIdx.x, m0, n0;
  tile_of(id, m0, n0);

  // ---- LDS-DMA sources: buffer resources at the tile's first A row / W row; wave w fills rows
  //      (NA*w + j) * 8 + lane / 8 of each A half-tile and (2w + j) * 8 + lane / 8 of each B half,
  //      16-B chunk (lane & 7) ^ ((row >> 1) & 7). Rows past M / N are clamped: they only feed
  //      outputs that are never stored.
  __amdgpu_buffer_rsrc_t rsa, rsw;
  unsigned aoffs[2][2], boffs[2][2];  // (fixed extents: a template-dependent array extent in a builtin argument makes hipcc's host pass drop the launch stub)
  auto sources = [&](int m0_, int n0_) __attribute__((always_inline)) {
    int sl = lane;  // (laundered like the epilogue's lane indices: recomputed per tile, not hoisted)
    if constexpr (PERSIST) asm volatile("" : "+v"(sl));
    rsa = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.A + (size_t)m0_ * p.lda * 2), (short)0, 0x7ffffff0, 0x00020000);
    rsw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.W + (size_t)n0_ * p.K * 2), (short)0, 0x7ffffff0, 0x00020000);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int r = (wid * NA + j) * 8 + (sl >> 3);
      const int c = (sl & 7) ^ ((r >> 1) & 7);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        aoffs[h][j] = (unsigned)(min(m0_ + h * (BM / 2) + r, p.M - 1) - m0_) * (unsigned)(p.lda * 2) + c * 16;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = (wid * 2 + j) * 8 + (sl >> 3);
      const int c = (sl & 7) ^ ((r >> 1) & 7);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        boffs[h][j] = (unsigned)(min(n0_ + h * 128 + r, p.N - 1) - n0_) * (unsigned)(p.K * 2) + c * 16;
    }
  };
#define ISSUE_A(H, KT, B)                                                                               \
  do {                                                                                                  \
    char* d_ = smem + (B) * BUF + ((H) ? OFF_A1 : OFF_A0) + wid * NA * 1024;                            \
    _Pragma("unroll") for (int j_ = 0; j_ < NA; ++j_)                                                   \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr_t)(d_ + j_ * 1024), 16, aoffs[H][j_], (KT) * 128, 0, 0); \
  } while (0)
#define ISSUE_B(H, KT, B)                                                                               \
  do {                                                                                                  \
    char* d_ = smem + (B) * BUF + ((H) ? OFF_B1 : OFF_B0) + wid * 2048;                                 \
    _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_)                                                    \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (lds_ptr_t)(d_ + j_ * 1024), 16, boffs[H][j_], (KT) * 128, 0, 0); \
  } while (0)
  // prologue DMA: all of K-tile 0 and A0 B0 B1 of K-tile 1
  //   (DMA order per wave: ... A0 B0 B1(t+1) | A1(t+1) | A0 B0 B1(t+2) | A1(t+2) ...)
  auto prologue = [&]() __attribute__((always_inline)) {
    ISSUE_A(0, 0, 0); ISSUE_B(0, 0, 0); ISSUE_B(1, 0, 0); ISSUE_A(1, 0, 0);
    ISSUE_A(0, 1, 1); ISSUE_B(0, 1, 1); ISSUE_B(1, 1, 1);
  };

  // ---- fragment read offsets: row wg*QR + i*16 + fr of an A half (wn*32 + j*16 + fr of a B half),
  //      16-B chunk kk*4 + fg, swizzled by ((row >> 1) & 7) = fr >> 1 (i*16, wg*QR, wn*32 keep it).
  //      (v_mfma_f32_16x16x32_bf16; the 32x32x16 shape with the same per-wave tile measured 8 %
  //      slower: the same cycles at a lower clock, profiles/r2/ab_gemm8p_mfma_shape.txt)
  int aoff[2], boff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int cs = ((kk * 4 + fg) ^ (fr >> 1)) << 4;
    aoff[kk] = (wg * QR + fr) * 128 + cs;
    boff[kk] = (wn * 32 + fr) * 128 + cs;
  }

  f32x4_t acc[2][2][MI][2];
  bf16x8_t ra[2][MI], rb0[2][2], rb1[2][2];
  auto read_a = [&](const char* base) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i) ra[kk][i] = *(const bf16x8_t*)(base + aoff[kk] + i * 2048);
  };
  auto read_b = [&](bf16x8_t (&rb)[2][2], const char* base) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) rb[kk][j] = *(const bf16x8_t*)(base + boff[kk] + j * 2048);
  };
  auto bar = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lgkm0 = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto quad = [&](auto ih_t, auto jh_t, bf16x8_t (&rb)[2][2]) __attribute__((always_inline)) {
    constexpr int IH = decltype(ih_t)::value, JH = decltype(jh_t)::value;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[IH][JH][i][j] = T::mma16(rb[kk][j], ra[kk][i], acc[IH][JH][i][j]);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  //   phase A waits A1(t)         : A0 B0 B1(t+1), A1(t+1) newer -> CNT_AB (0 in the last tile)
  //   phase B waits A0 B0 B1(t+1) : A1(t+1), A0 B0 B1(t+2) newer -> CNT_AB (NA when t+2 does not exist)
  // X: store instructions the previous tile of a persistent workgroup issued between this tile's
  // prologue DMA and K-tile 0 (X > 0 only for kt = 0): they are younger than the half-tiles kt = 0
  // waits for, so its counted waits let them stay in flight — the stores drain under the MFMAs of
  // K-tile 0 instead of before them (vmcnt retires loads, stores and LDS-DMA in issue order)
  auto ktile = [&](int kt, auto fill_tag, auto next_tag, auto x_tag) __attribute__((always_inline)) {
    constexpr bool FILL = decltype(fill_tag)::value;  // tile kt + 2 exists
    constexpr bool NEXT = decltype(next_tag)::value;  // tile kt + 1 exists
    constexpr int X = decltype(x_tag)::value;
    const int b = kt & 1;
    const char* base = smem + b * BUF;
    read_a(base + OFF_A0);
    read_b(rb0, base + OFF_B0);
    read_b(rb1, base + OFF_B1);
    if constexpr (NEXT) { ISSUE_A(1, kt + 1, b ^ 1); vmcnt<CNT_AB + X>(); }
    else { vmcnt<0>(); }
    lgkm0();
    bar();
    __builtin_amdgcn_s_setprio(1);
    quad(I0{}, I0{}, rb0);
    quad(I0{}, I1{}, rb1);
    __builtin_amdgcn_s_setprio(0);
    bar();
    read_a(base + OFF_A1);
    if constexpr (FILL) { ISSUE_A(0, kt + 2, b); ISSUE_B(0, kt + 2, b); ISSUE_B(1, kt + 2, b); vmcnt<CNT_AB + X>(); }
    else if constexpr (NEXT) { vmcnt<NA + X>(); }
    lgkm0();
    bar();
    __builtin_amdgcn_s_setprio(1);
    quad(I1{}, I1{}, rb1);
    quad(I1{}, I0{}, rb0);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const int nk = p.K / 64;  // >= 2 (host-checked)

  constexpr bool SW = (EPI == EPI_SWIGLU);
  constexpr int HC = SW ? 16 : 32;   // staged columns per jh half (one contiguous global run)
  constexpr int CPR = 2 * HC / 8;    // 16-B chunks per staged row
  constexpr int RPI = 64 / CPR;      // rows per store instruction
  constexpr int NI = (BM / 2) / RPI; // staged rows per lane
  constexpr int NB = NI < 8 ? NI : 8;
  const int ncols = SW ? p.N / 2 : p.N;

  // stores per lane of a persistent tile's epilogue (non-RoPE: one unconditional buffer store per
  // staged row; rows past M / columns past N fall outside the store's buffer range and are dropped)
  constexpr int XS = (PERSIST && EPI != EPI_ROPE) ? NI : 0;
  using X0 = std::integral_constant<int, 0>;
  using XN = std::integral_constant<int, XS>;

  sources(m0, n0);
  prologue();
  bool first = true;
  for (;;) {
    // wait for A0 B0 B1 of K-tile 0; on a persistent workgroup's later tiles the previous tile's
    // XS stores (issued after this tile's prologue DMA) may stay in flight
    if (first) vmcnt<CNT_AB>();
    else vmcnt<CNT_AB + XS>();
    bar();
    if (wg) bar();  // G1 runs one barrier behind
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (nk > 2) {
      if (first) ktile(0, T_{}, T_{}, X0{});
      else ktile(0, T_{}, T_{}, XN{});
      for (int kt = 1; kt < nk - 2; ++kt) ktile(kt, T_{}, T_{}, X0{});
      ktile(nk - 2, F_{}, T_{}, X0{});
    } else {  // nk == 2: K-tile 0 is also the last-but-one
      if (first) ktile(0, F_{}, T_{}, X0{});
      else ktile(0, F_{}, T_{}, XN{});
    }
    ktile(nk - 1, F_{}, F_{}, X0{});
    first = false;
    if (!wg) bar();  // re-align the groups
    __syncthreads();

    // lane-derived epilogue indices from a copy of the lane id the compiler cannot see through, so
    // they are recomputed here rather than hoisted out of the tile loop (live across the K-loop
    // they pushed a persistent instance past 256 VGPRs into scratch)
    int el = lane;
    if constexpr (PERSIST) asm volatile("" : "+v"(el));
    const int efr = el & 15, efg = el >> 4;
    const int ch = el % CPR;
    const int jh = ch / (HC / 8);
    const int cc = (ch % (HC / 8)) * 8;
    const int lr0 = el / CPR;
    // ---- epilogue: registers -> (bias / GELU / SwiGLU) -> bf16 staging -> coalesced stores.
    //      Staged row lr = ih*QR + i*16 + efr (tile row ih*BM/2 + wg*QR + (lr % QR)), staged
    //      columns lc = jh*32 + j*16 + 4 efg .. + 3 (tile columns jh*128 + wn*32 + (lc & 31)).
    char* st = smem + wid * (BM / 2) * SROW;
    // The MFMAs run with W as the A operand (D^T): lane (efr, efg) holds output row i*16 + efr of its
    // 16 x 16 block and the 4 CONSECUTIVE output columns 4 efg .. 4 efg + 3, so a lane stages 8 B per
    // block (one ds_write_b64 of 4 packed bf16) instead of 4 separate 2-byte writes.
    if constexpr (EPI == EPI_SWIGLU) {
      // W rows interleaved in 16-row (gate, up) groups: j = 0 is gate, j = 1 is up of output columns
      // (n0 + jh*128 + wn*32) / 2 + 4 efg + q
#pragma unroll
      for (int ih = 0; ih < 2; ++ih)
#pragma unroll
        for (int jh_ = 0; jh_ < 2; ++jh_)
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = silu(acc[ih][jh_][i][0][q]) * acc[ih][jh_][i][1][q];
            *(u32x2_t*)(st + (ih * QR + i * 16 + efr) * SROW + (jh_ * 16 + efg * 4) * 2) =
                u32x2_t{T::pack2(v[0], v[1]), T::pack2(v[2], v[3])};
          }
    } else {
      float bv[2][2][4] = {};
      if (p.bias) {
#pragma unroll
        for (int jh_ = 0; jh_ < 2; ++jh_)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int gc = n0 + jh_ * 128 + wn * 32 + j * 16 + efg * 4 + q;
              bv[jh_][j][q] = gc < p.N ? T::to_f(p.bias[gc]) : 0.f;
            }
      }
#pragma unroll
      for (int ih = 0; ih < 2; ++ih)
#pragma unroll
        for (int jh_ = 0; jh_ < 2; ++jh_)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              float v[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                v[q] = acc[ih][jh_][i][j][q] + bv[jh_][j][q];
                if constexpr (EPI == EPI_GELU) v[q] = gelu_erf(v[q]);
              }
              *(u32x2_t*)(st + (ih * QR + i * 16 + efr) * SROW + (jh_ * 32 + j * 16 + efg * 4) * 2) =
                  u32x2_t{T::pack2(v[0], v[1]), T::pack2(v[2], v[3])};
            }
    }
    __syncthreads();
    const int gcol = (SW ? n0 / 2 : n0) + jh * (SW ? 64 : 128) + wn * HC + cc;
    const bool col_ok = gcol < ncols;
    // EPI_ROPE: this lane's 8 columns lie in one head (D % 8 == 0) and hold 4 whole rotary pairs
    [[maybe_unused]] int rkind = 0, rhead = 0, rd0 = 0;
    if constexpr (EPI == EPI_ROPE) {
      const RopeArgs& R = p.rope;
      const int qw = R.H * R.D, kw = R.Hkv * R.D;
      rkind = gcol < qw ? 0 : (gcol < qw + kw ? 1 : 2);
      const int rel = gcol - (rkind == 0 ? 0 : (rkind == 1 ? qw : qw + kw));
      rhead = rel / R.D;
      rd0 = rel % R.D;
    }
    // This lane's rows lr = lane / CPR + i * RPI: the staged values of all of them go to registers
    // first (a persistent workgroup then refills the buffers with the next tile's prologue DMA
    // while this tile's stores drain), with their residual rows / RoPE positions and slots issued
    // alongside; RoPE cos / sin follow in batches of NB, all issued before any is waited for.
    int gmv[NI];
    u32x4_t vv[NI];
    [[maybe_unused]] u32x4_t rr[EPI == EPI_RESID ? NI : 1];
    [[maybe_unused]] int psv[EPI == EPI_ROPE ? NI : 1], slv[EPI == EPI_ROPE ? NI : 1];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int lr = lr0 + i * RPI;
      gmv[i] = m0 + (lr / QR) * (BM / 2) + wg * QR + (lr % QR);
      const int gmc = min(gmv[i], p.M - 1);  // loads of rows past M read a valid row, never stored
      vv[i] = *(const u32x4_t*)(st + lr * SROW + (jh * HC + cc) * 2);
      if constexpr (EPI == EPI_RESID)
        rr[i] = *(const u32x4_t*)(p.resid + (size_t)gmc * p.ldr + (col_ok ? gcol : 0));
      if constexpr (EPI == EPI_ROPE) {
        psv[i] = p.rope.pos[gmc];
        slv[i] = p.rope.slot[gmc];
      }
    }
    // output rows m0 .. M - 1 of this tile (num_records clamped below 2 GiB: a tile's rows are far
    // inside it, rows past M fall outside it)
    [[maybe_unused]] __amdgpu_buffer_rsrc_t rsc;
    if constexpr (XS > 0)
      rsc = __builtin_amdgcn_make_buffer_rsrc((void*)(p.C + (size_t)m0 * p.ldc), (short)0,
                                              (int)min((long long)(p.M - m0) * p.ldc * 2, 0x7ffffff0ll), 0x00020000);
    const int nid = id + (int)gridDim.x;
    const bool more = PERSIST && nid < ntiles;
    int nm0 = 0, nn0 = 0;
    if constexpr (PERSIST) {
      lgkm0();
      bar();  // every wave holds its staged rows: both operand buffers are free
      if (more) {
        tile_of(nid, nm0, nn0);
        sources(nm0, nn0);
        prologue();
      }
    }
#pragma unroll
    for (int i0 = 0; i0 < NI; i0 += NB) {
      if constexpr (EPI == EPI_ROPE) {
        // same bf16 roundings as GEMM -> rope_cache: rotate the bf16-rounded outputs in fp32
        const RopeArgs& R = p.rope;
        const int half = R.D / 2, i0c = rd0 / 2;
        f32x4_t c01[NB], c23[NB];
        if (rkind < 2) {
#pragma unroll
          for (int i = 0; i < NB; ++i) {
            const int ps = min(max(psv[i0 + i], 0), R.max_seq - 1);
            c01[i] = *(const f32x4_t*)(R.cs + ((size_t)ps * half + i0c) * 2);
            c23[i] = *(const f32x4_t*)(R.cs + ((size_t)ps * half + i0c) * 2 + 4);
          }
        }
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int gm = gmv[i0 + i];
          if (gm >= p.M || !col_ok) continue;
          u32x4_t v = vv[i0 + i];
          const int ps = psv[i0 + i], sl = slv[i0 + i];
          DA_ASSERT(ps >= 0 && ps < R.max_seq && sl >= 0);
          if (rkind < 2) {
            const float ccs[4] = {c01[i][0], c01[i][2], c23[i][0], c23[i][2]};
            const float sns[4] = {c01[i][1], c01[i][3], c23[i][1], c23[i][3]};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x1 = bf2f((bf16_t)(v[e] & 0xffff)), x2 = bf2f((bf16_t)(v[e] >> 16));
              const float o1 = x1 * ccs[e] - x2 * sns[e];
              const float o2 = x2 * ccs[e] + x1 * sns[e];
              v[e] = pack_bf2(o1, o2);
            }
          }
          if (rkind > 0) {
            bf16_t* cache = rkind == 1 ? R.kc : R.vc;
            *(u32x4_t*)(cache + (((size_t)sl * R.Hkv + rhead) * R.max_seq + ps) * R.D + rd0) = v;
            if (!R.kv_out) continue;  // k / v live in the cache only: no second copy in C
          }
          *(u32x4_t*)(p.C + (size_t)gm * p.ldc + gcol) = v;
        }
      } else {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int gm = gmv[i0 + i];
          if (XS == 0 && (gm >= p.M || !col_ok)) continue;
          u32x4_t v = vv[i0 + i];
          if constexpr (EPI == EPI_RESID) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = T::to_f((bf16_t)(v[e] & 0xffff)) + T::to_f((bf16_t)(rr[i0 + i][e] & 0xffff));
              const float hi = T::to_f((bf16_t)(v[e] >> 16)) + T::to_f((bf16_t)(rr[i0 + i][e] >> 16));
              v[e] = T::pack2(lo, hi);
            }
          }
          if constexpr (XS > 0) {
            // exactly one store instruction per row, whatever the row / column (the counted waits
            // of the next tile's K-tile 0 rely on it): out-of-range ones land past num_records
            const unsigned off = col_ok ? (unsigned)((gm - m0) * p.ldc + gcol) * 2u : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(v, rsc, off, 0, 0);
          } else {
            *(u32x4_t*)(p.C + (size_t)gm * p.ldc + gcol) = v;
          }
        }
      }
    }
    if (!more) break;
    id = nid; m0 = nm0; n0 = nn0;
  }
#undef ISSUE_A
#undef ISSUE_B
}

// Grouped-M band height of the tile order: 4 rows of tiles. (2-row bands ran isolated GEMMs at
// M = 65536 1.4-2.7 % faster, profiles/r4/gemm_group.txt, but the bench's QA prefill 0.8 % slower,
// profiles/r4/rejected_r4.txt: back-to-back repeats of one GEMM keep its operands cache-warm; the
// real layer sequence does not.)
static int num_cus() {
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// Persistent tile loop (a grid of one workgroup per CU, a multiple of 8 so a workgroup's tiles
// stay on its XCD) when the product has more tiles than CUs: the next tile's prologue DMA is in
// flight while this tile's stores drain, instead of a workgroup retiring and the next one paying
// launch + prologue latency (profiles/r5/gemm_epilogue/: prologue + launch ~4 % of a prefill GEMM).
// DA_GEMM8P_PERSIST=0 turns it off.
static int g_persist = -1;
static bool persist_on() {
  if (g_persist < 0) {
    const char* e = getenv("DA_GEMM8P_PERSIST");
    g_persist = (e && e[0] == '0') ? 0 : 1;
  }
  return g_persist == 1;
}

// on = 0 / 1 sets the persistent tile loop off / on for later launches, -1 only queries; returns
// the previous setting (tests run one product both ways and compare bit for bit)
DA_EXPORT int da_gemm8p_persist(int on) {
  const int prev = persist_on() ? 1 : 0;
  if (on == 0 || on == 1) g_persist = on;
  return prev;
}

template <int EPI, int BM, typename T>
static void launch8p_epi(const GemmArgs& a, int ntiles, hipStream_t s) {
  const int cus = num_cus();
  // (not EPI_ROPE: its per-row positions / slots / cos-sin next to the tile loop's state spill past
  // 256 VGPRs, and the persistent QKV projection measured 4 % slower, profiles/r5/gemm_persist/)
  if constexpr (EPI != EPI_ROPE) {
    if (persist_on() && ntiles > cus && cus >= 8) {
      gemm8p_kernel<EPI, BM, T, true><<<dim3(cus & ~7), dim3(512), 0, s>>>(a);
      return;
    }
  }
  gemm8p_kernel<EPI, BM, T, false><<<dim3(ntiles), dim3(512), 0, s>>>(a);
}

template <int BM>
static int launch8p(const GemmArgs& a0, int epi, hipStream_t s) {
  GemmArgs a = a0;
  if (a.group <= 0) a.group = 4;
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  const int nt = ntm * ntn;
  if (epi >= 100) {  // fp16 operands (the encoder's DTYPE=fp16): the BERT epilogues only
    switch (epi - 100) {
      case EPI_NONE: launch8p_epi<EPI_NONE, BM, F16T>(a, nt, s); break;
      case EPI_BIAS: launch8p_epi<EPI_BIAS, BM, F16T>(a, nt, s); break;
      case EPI_GELU: launch8p_epi<EPI_GELU, BM, F16T>(a, nt, s); break;
      case EPI_RESID: launch8p_epi<EPI_RESID, BM, F16T>(a, nt, s); break;
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
  switch (epi) {
    case EPI_NONE: launch8p_epi<EPI_NONE, BM, BF16T>(a, nt, s); break;
    case EPI_BIAS: launch8p_epi<EPI_BIAS, BM, BF16T>(a, nt, s); break;
    case EPI_GELU: launch8p_epi<EPI_GELU, BM, BF16T>(a, nt, s); break;
    case EPI_SWIGLU: launch8p_epi<EPI_SWIGLU, BM, BF16T>(a, nt, s); break;
    case EPI_RESID: launch8p_epi<EPI_RESID, BM, BF16T>(a, nt, s); break;
    case EPI_ROPE: launch8p_epi<EPI_ROPE, BM, BF16T>(a, nt, s); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// Row-tile height for a non-RoPE prefill product: the one with fewer workgroup WAVES over the
// chip's CUs, weighting a 128-row tile's time as 0.72 of a 256-row one (measured at M = 2930:
// 128-row tiles took 0.61-0.73 of the 256-row tile time, profiles/r3/gemm_ab_batch1_prefill_tiles.txt).
// At M ~ 2.6k (the batch-1 prefill of the p50 path) the O / down projections (N = 3072) then run
// 252 128-row tiles in one wave instead of 132 256-row tiles on half the chip; QA-sized chunks
// (M ~ 64k) keep 256 (the round-3 rule, 256 rows once the 256-row grid reached half the chip,
// measured 65.5 vs 74.9 us per O projection at M ~ 2.6k: profiles/r4/bm_rule/).
int gemm8p_pick_bm(int M, int N) {
  const long ntn = (N + 255) / 256;
  const long t256 = (long)((M + 255) / 256) * ntn, t128 = (long)((M + 127) / 128) * ntn;
  const int cus = num_cus();
  const long w256 = (t256 + cus - 1) / cus, w128 = (t128 + cus - 1) / cus;
  return w128 * 72 < w256 * 100 ? 128 : 256;
}

// epi + 100: the same kernel on fp16 operands / output (v_mfma_f32_16x16x32_f16)
int launch_gemm8p(const GemmArgs& a, int epi, hipStream_t s, int bm) {
  if (a.K < 128 || a.K % 64) return (int)hipErrorInvalidValue;
  // buffer resources span the tile's rows from its first one (num_records < 2 GiB)
  if ((size_t)bm * a.lda * 2 >= 0x7ffffff0ull || (size_t)256 * a.K * 2 >= 0x7ffffff0ull) return (int)hipErrorInvalidValue;
  return bm == 128 ? launch8p<128>(a, epi, s) : launch8p<256>(a, epi, s);
}

// fp16 GEMM for the encoder's DTYPE=fp16 path: C = epi(A W^T), A [M, K] / W [N, K] / C / bias /
// resid fp16, fp32 accumulation; epi NONE / BIAS / GELU / RESID. Every M on the phase-split tile
// (128-row tiles below half a chip of 256-row ones): the fp16 path has no decode-sized tiles.
DA_EXPORT int da_gemm_f16(const void* A, int lda, const void* W, void* C, int ldc, const void* bias,
                          const void* resid, int ldr, int M, int N, int K, int epi, void* stream) {
  if (M < 1 || K % 64 || K < 128 || N % 8 || lda % 8 || ldc % 8) return (int)hipErrorInvalidValue;
  if (epi != EPI_NONE && epi != EPI_BIAS && epi != EPI_GELU && epi != EPI_RESID) return (int)hipErrorInvalidValue;
  if (epi == EPI_RESID && (!resid || ldr % 8)) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = (const bf16_t*)bias; a.resid = (const bf16_t*)resid;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldc = ldc; a.ldr = ldr; a.k_per_split = K;
  return launch_gemm8p(a, 100 + epi, (hipStream_t)stream, gemm8p_pick_bm(M, N));
}
