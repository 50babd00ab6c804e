// 256x256 bf16 GEMM with FOUR waves, one per SIMD, each owning a 128x128 output block:
//   C[M,N] = epi(A[M,K] . W[N,K]^T)
//
// Why a second 256x256 kernel (VERDICT r5 "next round" #6): gemm8p.hip gives each of its 8 waves a
// 128x64 block, so per 64-deep K-tile a wave reads 16 KiB of A and 8 KiB of W fragments from LDS
// for 128x64x64 MACs; a 128x128 block reads 16 + 16 KiB for twice the MACs — 1.5x fewer LDS bytes
// per MFMA (192 -> 128 KiB of ds_read_b128 per K-tile per CU), the layout hipBLASLt's MT256x256
// kernels use (profiles/r2/pmc_hipblaslt). The price is one wave per SIMD: 256 accumulator
// registers per lane (the AGPR half of the unified 512-entry file) and no partner wave to cover
// this wave's LDS reads, DMA issue and barrier, so the overlap has to come from the instruction
// stream itself:
//  * fragment register sets, written in issue order (the MFMAs are asm volatile, so every LDS read /
//    DMA stays where it is written and hipcc counts the lgkmcnt each MFMA's operands need).
//    SCHED 3 (default; K / 64 even and >= 4): THREE sets, TWO barriers per K-tile:
//        [lgkmcnt(0) barrier B]  -> every wave has read stage t & 1 (reads came in half 2 of t-1)
//        half 1 of tile t: 64 MFMAs on set 0 (k-half 0 of t) | DMAs 0-7 of tile t+2 -> stage t & 1
//        [vmcnt(8) barrier M]    -> stage t+1 landed for every wave (tile t+2's 8 DMAs still fly)
//        half 2 of tile t: 64 MFMAs on set S1(t) (k-half 1 of t) | 32 reads of tile t+1 -> set 0 /
//                          S1(t+1) in the first 32 MFMA slots | DMAs 8-15 of tile t+2
//    with S1 alternating between sets 1 and 2 (a 2-tile unrolled loop); one DMA per 8 MFMAs over
//    the whole tile. SCHED 2: the same three sets with ONE barrier (M) per tile, so all 16 DMAs of
//    a tile go out in half 2. SCHED 0 (any K): two sets, one barrier; half 1 reads k-half 1 of t
//    beside its MFMAs, half 2 reads k-half 0 of t+1 beside the DMA. hipcc adds no vmcnt for
//    LDS-DMA before a ds_read (checked on gemm8p's ISA): the explicit waits are the only ones.
//  * measured (bench/gemm4w_ab.py, profiles/r6/gemm4w/), 32768x9216x3072: SCHED 3 1462-1472 TF/s,
//    1.5-2 % below gemm8p (1485-1500) and 4-6 % below hipBLASLt (1527-1558); SCHED 2 1390-1424,
//    SCHED 0 1370. The one-wave-per-SIMD issue stream stalls on LDS-DMA issue back-pressure (16
//    DMAs per wave in half a tile: 1297 when packed into 16 MFMA slots, +3.6 % when spread over
//    the whole tile at the price of a second barrier); gemm8p's two wave groups per SIMD cover
//    each other's stalls. Production GEMMs stay on gemm8p; this kernel is the tile-13 A/B arm.
//  * LDS: two stages of A 256x64 + W 256x64 bf16 (2 x 64 KiB), loaded by LDS-DMA
//    (buffer_load ... lds, 1 KiB per wave-instruction, 16 per wave per K-tile) with the XOR swizzle
//    of gemm8p (16-B chunk c of row r at chunk c ^ ((r >> 1) & 7), applied on the per-lane SOURCE
//    offset, undone on the read address); the epilogue stages each wave's 128x128 bf16 block
//    (4 x 34 KiB) through the same LDS.
//  * tile order: bijective XCD remap + grouped-M bands (as gemm8p).
// MFMA v_mfma_f32_16x16x32 with W as the A operand (D^T): lane (fr, fg) holds output row i*16 + fr
// of its 16x16 block and the 4 consecutive columns j*16 + 4 fg .. + 3.
#include "gemm.h"

#include <type_traits>

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// v_mfma_f32_16x16x32_bf16 (f16 for T = F16T) as asm with the accumulator tied in an AGPR
// ("+a": D = C, the register never moves). hipcc's own 16x16x32 with 256 accumulators per lane
// allocates D apart from C and copies every result back with v_accvgpr_mov (0.9-1.4 copies per
// MFMA in the K-loop, measured on this kernel's ISA); the 32x32x16 form allocates cleanly but runs ~12 % fewer FLOP/s
// on random data (MI355X_MICROARCH.md, MFMA shape and clock). Z: C = 0 (no accumulator read).
// Wait states: operands come from ds_read (no VALU -> MFMA operand hazard); accumulators are
// read only after the K-loop's closing s_nop.
template <typename T, bool Z>
__device__ __forceinline__ void mfma4w(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  if constexpr (T::kF16) {
    if constexpr (Z) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  } else {
    if constexpr (Z) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
}

namespace {
constexpr int OPND = 256 * 128;              // one operand of a stage: 256 rows x 64 bf16 (32 KiB)
constexpr int STG = 2 * OPND;                // A + W
constexpr int SROW4 = 128 * 2 + 16;          // epilogue staging row stride (bytes)
constexpr int STAGING4 = 4 * 128 * SROW4;    // 136 KiB
constexpr int SMEM4 = STAGING4 > 2 * STG ? STAGING4 : 2 * STG;
}  // namespace

template <int EPI, typename T, int SCHED = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm4w_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;

  const int ntm = (p.M + 255) / 256, ntn = (p.N + 255) / 256;
  const int GROUP = p.group > 0 ? p.group : 4;
  int m0, n0;
  {
    const int t = xcd_remap(blockIdx.x, ntm * ntn);
    const int gid = t / (GROUP * ntn);
    const int first_m = gid * GROUP;
    const int gsz = min(ntm - first_m, GROUP);
    const int tin = t % (GROUP * ntn);
    m0 = (first_m + tin % gsz) * 256;
    n0 = (tin / gsz) * 256;
  }

  // ---- LDS-DMA sources: wave w fills rows (8w + j) * 8 + lane / 8 (j < 8) of the A and the W
  //      stage, 16-B chunk (lane & 7) ^ ((row >> 1) & 7); rows past M / N are clamped (they only
  //      feed outputs that are never stored). The K-tile is the scalar soffset.
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.A + (size_t)m0 * p.lda * 2), (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)p.W + (size_t)n0 * p.K * 2), (short)0, 0x7ffffff0, 0x00020000);
  unsigned aoffs[8], woffs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = (wid * 8 + j) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    aoffs[j] = (unsigned)(min(m0 + r, p.M - 1) - m0) * (unsigned)(p.lda * 2) + c * 16;
    woffs[j] = (unsigned)(min(n0 + r, p.N - 1) - n0) * (unsigned)(p.K * 2) + c * 16;
  }

  // ---- fragment reads: A row wm*128 + i*16 + fr, W row wn*128 + j*16 + fr, 16-B chunk kk*4 + fg
  //      swizzled by (row >> 1) & 7 = fr >> 1
  int aoff[2], woff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int cs = ((kk * 4 + fg) ^ (fr >> 1)) << 4;
    aoff[kk] = (wm * 128 + fr) * 128 + cs;
    woff[kk] = OPND + (wn * 128 + fr) * 128 + cs;
  }
  // fragment register sets: SCHED 0 uses sets 0 and 1 (= k-halves 0 and 1 of the tile), SCHED 2
  // a third one (set 0 = k-half 0 of every tile, k-half 1 alternates between sets 1 and 2)
  constexpr int NSET = SCHED >= 2 ? 3 : 2;  // SCHED 2 / 3: three
  bf16x8_t fa[NSET][8], fw[NSET][8];
  f32x4_t acc[8][8];
  auto lds16 = [&](const char* q) __attribute__((always_inline)) { return *(const bf16x8_t*)q; };
  // fragment g (< 8: A block g, else W block g - 8) of k-half KK of the stage at base -> set S
  auto read_frag = [&](auto s_t, auto kk_t, int g, const char* base) __attribute__((always_inline)) {
    constexpr int S = decltype(s_t)::value, KK = decltype(kk_t)::value;
    if (g < 8) fa[S][g] = lds16(base + aoff[KK] + g * 2048);
    else fw[S][g - 8] = lds16(base + woff[KK] + (g - 8) * 2048);
  };
  // MFMA n (block i = n / 8, j = n % 8) on set S; Z: the first k-half of tile 0, C = 0
  auto mma = [&](auto s_t, auto z_t, int n) __attribute__((always_inline)) {
    constexpr int S = decltype(s_t)::value;
    mfma4w<T, decltype(z_t)::value>(acc[n >> 3][n & 7], fw[S][n & 7], fa[S][n >> 3]);
  };
  // LDS-DMA instruction g (< 8: A rows, else W rows) of tile kt into stage buf
  auto dma = [&](int g, int kt, int buf) __attribute__((always_inline)) {
    char* d = smem + buf * STG + wid * 8 * 1024 + (g < 8 ? g : OPND / 1024 + g - 8) * 1024;
    if (g < 8) __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr_t)d, 16, aoffs[g], kt * 128, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (lds_ptr_t)d, 16, woffs[g - 8], kt * 128, 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using T_ = std::true_type;
  using F_ = std::false_type;
  auto stage_sync = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  // One K-tile, in issue order (asm volatile MFMAs: every LDS read / DMA stays where it is written,
  // and hipcc counts the lgkmcnt each MFMA's operands need). FILL: tile kt + 2 exists, NEXT: tile
  // kt + 1 exists, Z: tile 0 (its first k-half starts the accumulators at C = 0).
  auto ktile = [&](int kt, auto fill_t, auto next_t, auto z_t) __attribute__((always_inline)) {
    constexpr bool FILL = decltype(fill_t)::value, NEXT = decltype(next_t)::value;
    const char* cur = smem + (kt & 1) * STG;
    // half 1: MFMAs of set0 | reads of set1 (k-half 1 of this tile), one read per 4 MFMAs
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      read_frag(I1{}, I1{}, g, cur);
#pragma unroll
      for (int q = 0; q < 4; ++q) mma(I0{}, z_t, g * 4 + q);
    }
    stage_sync();
    // half 2: MFMAs of set1 | reads of set0 (k-half 0 of tile kt + 1), DMA of tile kt + 2
    if constexpr (NEXT) {
      const char* nxt = smem + ((kt + 1) & 1) * STG;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        if constexpr (FILL) dma(g, kt + 2, kt & 1);
        read_frag(I0{}, I0{}, g, nxt);
        mma(I1{}, F_{}, 2 * g);
        mma(I1{}, F_{}, 2 * g + 1);
      }
#pragma unroll
      for (int n = 32; n < 64; ++n) mma(I1{}, F_{}, n);
    } else {
#pragma unroll
      for (int n = 0; n < 64; ++n) mma(I1{}, F_{}, n);
    }
  };
  // SCHED 2: half 1 is MFMAs only; half 2 reads BOTH k-halves of tile kt + 1 (set 0 and set S1N),
  // so the stage a barrier hands to the DMA was fully read before the previous barrier's half ended
  // (no LDS drain at the barrier). S1 / S1N: the sets holding k-half 1 of tiles kt / kt + 1.
  auto ktile3 = [&](int kt, auto fill_t, auto next_t, auto z_t, auto s1_t, auto s1n_t) __attribute__((always_inline)) {
    constexpr bool FILL = decltype(fill_t)::value, NEXT = decltype(next_t)::value;
    if constexpr (SCHED == 3) {
      // two barriers per K-tile, the DMA of tile kt + 2 spread over both halves (one per 8 MFMAs):
      // B (tile start): every wave has read stage kt & 1 (its reads came in half 2 of tile kt - 1)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int n = 0; n < 64; ++n) {
        if (FILL && n % 8 == 0) dma(n / 8, kt + 2, kt & 1);
        mma(I0{}, z_t, n);
      }
      if constexpr (NEXT) {
        // M (mid-tile): stage kt + 1 landed for every wave (the 8 DMAs of tile kt + 2 just issued
        // may stay in flight)
        if constexpr (FILL) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const char* nxt = smem + ((kt + 1) & 1) * STG;
        // read r (< 32: even -> k-half 0 frag r / 2 into set 0, odd -> k-half 1 into set S1N)
        auto rd = [&](int r) __attribute__((always_inline)) {
          if (r % 2 == 0) read_frag(I0{}, I0{}, r / 2, nxt);
          else read_frag(s1n_t, I1{}, r / 2, nxt);
        };
#pragma unroll
        for (int n = 0; n < 64; ++n) {
          if (n < 32) rd(n);  // one per MFMA, first half
          if (FILL && n % 8 == 0) dma(8 + n / 8, kt + 2, kt & 1);
          mma(s1_t, F_{}, n);
        }
      } else {
#pragma unroll
        for (int n = 0; n < 64; ++n) mma(s1_t, F_{}, n);
      }
      return;
    }
#pragma unroll
    for (int n = 0; n < 64; ++n) mma(I0{}, z_t, n);
    stage_sync();
    if constexpr (NEXT) {
      const char* nxt = smem + ((kt + 1) & 1) * STG;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        if constexpr (FILL) dma(g, kt + 2, kt & 1);
        read_frag(I0{}, I0{}, g, nxt);
        read_frag(s1n_t, I1{}, g, nxt);
#pragma unroll
        for (int q = 0; q < 4; ++q) mma(s1_t, F_{}, 4 * g + q);
      }
    } else {
#pragma unroll
      for (int n = 0; n < 64; ++n) mma(s1_t, F_{}, n);
    }
  };

  const int nk = p.K / 64;  // >= 2 (host-checked); SCHED 2: even and >= 4
#pragma unroll
  for (int g = 0; g < 16; ++g) dma(g, 0, 0);
#pragma unroll
  for (int g = 0; g < 16; ++g) dma(g, 1, 1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 (this wave's part); tile 1 in flight
  __builtin_amdgcn_s_barrier();
  if constexpr (SCHED >= 2) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      read_frag(I0{}, I0{}, g, smem);
      read_frag(I1{}, I1{}, g, smem);
    }
    ktile3(0, T_{}, T_{}, T_{}, I1{}, I2{});
    ktile3(1, T_{}, T_{}, F_{}, I2{}, I1{});
    for (int kt = 2; kt < nk - 2; kt += 2) {
      ktile3(kt, T_{}, T_{}, F_{}, I1{}, I2{});
      ktile3(kt + 1, T_{}, T_{}, F_{}, I2{}, I1{});
    }
    ktile3(nk - 2, F_{}, T_{}, F_{}, I1{}, I2{});
    ktile3(nk - 1, F_{}, F_{}, F_{}, I2{}, I1{});
  } else {
#pragma unroll
    for (int g = 0; g < 16; ++g) read_frag(I0{}, I0{}, g, smem);
    if (nk > 2) {
      ktile(0, T_{}, T_{}, T_{});
      for (int kt = 1; kt < nk - 2; ++kt) ktile(kt, T_{}, T_{}, F_{});
      ktile(nk - 2, F_{}, T_{}, F_{});
    } else {
      ktile(0, F_{}, T_{}, T_{});
    }
    ktile(nk - 1, F_{}, F_{}, F_{});
  }
  // the last MFMAs' results -> the epilogue's reads: 16 wait states (8-pass XDL needs 12), and
  // every accumulator passes through an empty asm after them so no read is scheduled above
  asm volatile("s_nop 15");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  __syncthreads();  // every wave is done with the operand stages: the staging may overwrite them

  // ---- epilogue: registers -> (bias / GELU / SwiGLU) -> bf16 staging -> coalesced 16-B stores
  char* st = smem + wid * 128 * SROW4;
  constexpr bool SW = (EPI == EPI_SWIGLU);
  if constexpr (SW) {
    // W rows interleaved in 16-row (gate, up) groups: j = 2q is gate, 2q + 1 up of the wave's
    // output columns q*16 + 4 fg .. + 3
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = silu(acc[i][2 * q][e]) * acc[i][2 * q + 1][e];
        *(u32x2_t*)(st + (i * 16 + fr) * SROW4 + (q * 16 + fg * 4) * 2) =
            u32x2_t{T::pack2(v[0], v[1]), T::pack2(v[2], v[3])};
      }
  } else {
    // bias of this lane's 4 consecutive columns per block: one 8-B load each (N % 8 == 0, so a
    // 4-column group is all in range or all out; out-of-range groups feed no stored output)
    float bv[8][4] = {};
    if (EPI != EPI_NONE && p.bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int gc = min(n0 + wn * 128 + j * 16 + fg * 4, p.N - 4);
        const u32x2_t b2 = *(const u32x2_t*)(p.bias + gc);
        bv[j][0] = T::to_f((bf16_t)(b2[0] & 0xffff)); bv[j][1] = T::to_f((bf16_t)(b2[0] >> 16));
        bv[j][2] = T::to_f((bf16_t)(b2[1] & 0xffff)); bv[j][3] = T::to_f((bf16_t)(b2[1] >> 16));
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][e] + bv[j][e];
          if constexpr (EPI == EPI_GELU) v[e] = gelu_erf(v[e]);
        }
        *(u32x2_t*)(st + (i * 16 + fr) * SROW4 + (j * 16 + fg * 4) * 2) =
            u32x2_t{T::pack2(v[0], v[1]), T::pack2(v[2], v[3])};
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's staging is written (read back by itself only)
  __builtin_amdgcn_wave_barrier();
  constexpr int OC = SW ? 64 : 128;          // output columns of this wave
  constexpr int CPR = OC / 8;                // 16-B chunks per row
  constexpr int RPI = 64 / CPR;              // rows per store instruction
  const int ncols = SW ? p.N / 2 : p.N;
  const int gcol = (SW ? (n0 + wn * 128) / 2 : n0 + wn * 128) + (lane % CPR) * 8;
  if (gcol < ncols) {
    const int row0 = m0 + wm * 128;
#pragma unroll 8
    for (int rr = lane / CPR; rr < 128; rr += RPI) {
      const int gm = row0 + rr;
      if (gm >= p.M) break;
      u32x4_t v = *(const u32x4_t*)(st + rr * SROW4 + (lane % CPR) * 16);
      if constexpr (EPI == EPI_RESID) {
        const u32x4_t r = *(const u32x4_t*)(p.resid + (size_t)gm * p.ldr + gcol);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = T::to_f((bf16_t)(v[e] & 0xffff)) + T::to_f((bf16_t)(r[e] & 0xffff));
          const float hi = T::to_f((bf16_t)(v[e] >> 16)) + T::to_f((bf16_t)(r[e] >> 16));
          v[e] = T::pack2(lo, hi);
        }
      }
      *(u32x4_t*)(p.C + (size_t)gm * p.ldc + gcol) = v;
    }
  }
}

// Schedule where K / 64 is even and >= 4: SCHED 3 (default), or via da_gemm4w_variant (the A/B of
// bench/gemm4w_ab.py): 1 = SCHED 0, 2 = SCHED 2. Other K: SCHED 0.
static int g_4w_variant = 0;
DA_EXPORT int da_gemm4w_variant(int v) {
  const int prev = g_4w_variant;
  if (v >= 0) g_4w_variant = v;
  return prev;
}

template <int EPI, typename T>
static void launch4w_e(const GemmArgs& a, int nt, hipStream_t s) {
  const int nk = a.K / 64;
  const bool three = nk >= 4 && nk % 2 == 0;
  if (three && g_4w_variant == 0) gemm4w_kernel<EPI, T, 3><<<dim3(nt), dim3(256), 0, s>>>(a);
  else if (three && g_4w_variant == 2) gemm4w_kernel<EPI, T, 2><<<dim3(nt), dim3(256), 0, s>>>(a);
  else gemm4w_kernel<EPI, T, 0><<<dim3(nt), dim3(256), 0, s>>>(a);
}

template <typename T>
static int launch4w_t(const GemmArgs& a, int epi, hipStream_t s) {
  const int nt = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  switch (epi) {
    case EPI_NONE: launch4w_e<EPI_NONE, T>(a, nt, s); break;
    case EPI_BIAS: launch4w_e<EPI_BIAS, T>(a, nt, s); break;
    case EPI_GELU: launch4w_e<EPI_GELU, T>(a, nt, s); break;
    case EPI_RESID: launch4w_e<EPI_RESID, T>(a, nt, s); break;
    case EPI_SWIGLU: launch4w_e<EPI_SWIGLU, T>(a, nt, s); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// bf16 only. K % 64 == 0, K >= 128; the buffer resources span 256 rows of A / W from the tile's
// first one (num_records < 2 GiB).
int launch_gemm4w(const GemmArgs& a0, int epi, hipStream_t s) {
  if (a0.K < 128 || a0.K % 64 || a0.M < 1) return (int)hipErrorInvalidValue;
  if ((size_t)256 * a0.lda * 2 >= 0x7ffffff0ull || (size_t)256 * a0.K * 2 >= 0x7ffffff0ull) return (int)hipErrorInvalidValue;
  GemmArgs a = a0;
  if (a.group <= 0) a.group = 4;
  return launch4w_t<BF16T>(a, epi, s);
}
