// bf16 GEMM on gfx950 MFMA with fused epilogues.
//
//   C[M, N] = epi( A[M, K] · W[N, K]^T )       (nn.Linear layout: both operands K-contiguous)
//
// Design (MI355X-first, see /opt/skills/guides/cdna_hip_programming.md §5):
//  * v_mfma_f32_16x16x32_bf16, 4 waves per workgroup, each wave owns a (BM/WM)x(BN/WN) sub-tile
//    indexed by fragment repeat (acc[FM][FN]), never by wave position.
//  * BK = 64, double-buffered LDS with register-staged prefetch (issue global loads for tile t+1
//    before the MFMAs of tile t, write them to the other LDS buffer after: Guideline 15 / T14).
//  * LDS rows are 128 B; 16-B chunks XOR-swizzled by ((row>>1)&7) so the 16 rows read by one
//    ds_read_b128 lane group land on 16 distinct slots of the 256-B bank row (conflict-free).
//  * bijective XCD remap + grouped-M tile order so neighbouring tiles share an XCD L2 (T1).
//  * epilogue staged through LDS in fp32, then 16-B coalesced stores with bias / GELU / SwiGLU /
//    residual fused (the reference outsources all of this to OpenAI).
//  * split-K writes fp32 partials; gemm_splitk_reduce applies the same epilogue.
#include "gemm.h"

template <int BM, int BN, int WM, int WN, int EPI, int PF = 1>
__global__ void __launch_bounds__(256)
gemm_bf16_kernel(GemmArgs p) {
  // PF = k-tiles in flight in registers. PF = 1: the classic register-staged double buffer (one
  // tile ahead). Decode-sized tiles (M <= 64) stream weights and are latency-bound at PF = 1 —
  // one 16-KB W tile per workgroup in flight, ~6 dependent HBM round trips per split — so they
  // keep PF tiles (up to 72 KB per workgroup) requested ahead of the MFMAs (Little's law).
  // (Weight fragments loaded straight into the MFMA B registers, skipping LDS, lost on every arm
  // measured: half-line requests, profiles/r3/rejected_r3.txt.)
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int LA = BM * 8 / 256, LB = BN * 8 / 256;  // 16-B loads per thread per tile
  static_assert(WM * WN == 4, "4 waves");
  static_assert(LA >= 1 && LB >= 1, "tile too small");
  constexpr int STAGE_FLOATS = 4 * TM * (TN + 4);
  constexpr int LDS_MAIN = 2 * (A_BYTES + B_BYTES);
  constexpr int LDS_BYTES = LDS_MAIN > STAGE_FLOATS * 4 ? LDS_MAIN : STAGE_FLOATS * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // ---- tile scheduling: XCD remap, then grouped-M ordering ----
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int nwg = ntm * ntn;
  const int t = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP = 8;
  const int gid = t / (GROUP * ntn);
  const int first_m = gid * GROUP;
  const int gsz = min(ntm - first_m, GROUP);
  const int tin = t % (GROUP * ntn);
  const int tm = first_m + tin % gsz, tn = tin / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = blockIdx.z * p.k_per_split;
  const int nk = p.k_per_split / BK;

  // ---- global -> register staging (PF slots) ----
  u32x4_t ra[PF][LA], rb[PF][LB];
  const int fr = lane & 15, fg = lane >> 4;
  // Rows past M / N are clamped, not branched around: they only feed accumulators whose outputs
  // are never stored, and branch-free loads keep the compiler's vmcnt waits counted (a load
  // under a divergent branch makes every later wait a full vmcnt(0) drain).
  auto gload = [&](u32x4_t (&xa)[LA], u32x4_t (&xb)[LB], int kt) {
    const int k0 = kbeg + kt * BK;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + 256 * i, r = idx >> 3, c = idx & 7;
      xa[i] = *(const u32x4_t*)(p.A + (size_t)min(m0 + r, p.M - 1) * p.lda + k0 + c * 8);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + 256 * i, r = idx >> 3, c = idx & 7;
      xb[i] = *(const u32x4_t*)(p.W + (size_t)min(n0 + r, p.N - 1) * p.K + k0 + c * 8);
    }
  };
  auto lstore = [&](const u32x4_t (&xa)[LA], const u32x4_t (&xb)[LB], int buf) {
    char* sa = smem + buf * (A_BYTES + B_BYTES);
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + 256 * i, r = idx >> 3, c = idx & 7;
      *(u32x4_t*)(sa + r * 128 + ((c ^ ((r >> 1) & 7)) << 4)) = xa[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + 256 * i, r = idx >> 3, c = idx & 7;
      *(u32x4_t*)(sb + r * 128 + ((c ^ ((r >> 1) & 7)) << 4)) = xb[i];
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // Loads are issued unconditionally (tile index clamped to nk - 1: the redundant tail loads hit
  // L2) so every vmcnt wait below stays counted; compute / LDS stores sit under uniform branches.
  const int kl = nk > 0 ? nk - 1 : 0;
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    gload(ra[u], rb[u], min(u, kl));
    asm volatile("" ::: "memory");  // keep issue order = tile order (counted waits stay short)
  }
  if (nk > 0) lstore(ra[0], rb[0], 0);
  __syncthreads();

  for (int kt0 = 0; kt0 < nk; kt0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int kt = kt0 + u;
      const int cur = kt & 1;
      // slot u held tile kt, already copied to LDS: refill it PF tiles ahead
      if (PF > 1 || kt + 1 < nk) gload(ra[u], rb[u], min(kt + PF, kl));
      if (kt < nk) {
        const char* sa = smem + cur * (A_BYTES + B_BYTES);
        const char* sb = sa + A_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int c = kk * 4 + fg;
          bf16x8_t af[FM], bfr[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const int r = wm * TM + i * 16 + fr;
            af[i] = *(const bf16x8_t*)(sa + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
          }
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int r = wn * TN + j * 16 + fr;
            bfr[j] = *(const bf16x8_t*)(sb + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        }
      }
      if (kt >= nk) continue;
      if (kt + 1 < nk) lstore(ra[(u + 1) % PF], rb[(u + 1) % PF], cur ^ 1);
      // LDS writes visible + buffer reads done; a raw barrier, NOT __syncthreads(): its fence
      // drains vmcnt and would cancel the PF - 1 tiles still in flight
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }

  // ---- epilogue: stage fp32 tile of this wave in LDS, then coalesced 16-B stores ----
  float* st = (float*)smem + wid * TM * (TN + 4);
  constexpr int SLD = TN + 4;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) st[(i * 16 + fg * 4 + q) * SLD + j * 16 + fr] = acc[i][j][q];
  __syncthreads();

  const int row0 = m0 + wm * TM, col0 = n0 + wn * TN;
  if constexpr (EPI == EPI_SWIGLU) {
    // output tile TM x TN/2; chunk of 8 outputs; TN/16 chunks per row
    constexpr int CPR = TN / 16;
    constexpr int RPI = 64 / CPR;
    const int oc = (lane % CPR) * 8;          // output col within wave tile
    const int grp = oc / 16, within = oc % 16;  // gate cols 32*grp+within.., up cols +16
    const int ncols_out = p.N / 2;
    const int gout = col0 / 2 + oc;
    for (int rr = lane / CPR; rr < TM; rr += RPI) {
      const int gm = row0 + rr;
      if (gm >= p.M || gout >= ncols_out) continue;
      const float* srow = st + rr * SLD + grp * 32 + within;
      unsigned packed[4];
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        float g0 = srow[e], g1 = srow[e + 1], u0 = srow[16 + e], u1 = srow[16 + e + 1];
        packed[e / 2] = pack_bf2(silu(g0) * u0, silu(g1) * u1);
      }
      *(u32x4_t*)(p.C + (size_t)gm * p.ldc + gout) = u32x4_t{packed[0], packed[1], packed[2], packed[3]};
    }
  } else {
    constexpr int CPR = TN / 8;
    constexpr int RPI = 64 / CPR;
    const int cc = (lane % CPR) * 8;
    const int gn = col0 + cc;
    for (int rr = lane / CPR; rr < TM; rr += RPI) {
      const int gm = row0 + rr;
      if (gm >= p.M || gn >= p.N) continue;
      const float* srow = st + rr * SLD + cc;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = srow[e];
      if constexpr (EPI == EPI_PARTIAL) {
        float* dst = p.ws + ((size_t)blockIdx.z * p.M + gm) * p.N + gn;
        *(f32x4_t*)dst = f32x4_t{v[0], v[1], v[2], v[3]};
        *(f32x4_t*)(dst + 4) = f32x4_t{v[4], v[5], v[6], v[7]};
        continue;
      }
      if (p.bias) {
        u32x4_t b = *(const u32x4_t*)(p.bias + gn);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += bf2f((bf16_t)(b[e] & 0xffff));
          v[2 * e + 1] += bf2f((bf16_t)(b[e] >> 16));
        }
      }
      if constexpr (EPI == EPI_GELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
      }
      if constexpr (EPI == EPI_RESID) {
        u32x4_t r = *(const u32x4_t*)(p.resid + (size_t)gm * p.ldr + gn);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += bf2f((bf16_t)(r[e] & 0xffff));
          v[2 * e + 1] += bf2f((bf16_t)(r[e] >> 16));
        }
      }
      *(u32x4_t*)(p.C + (size_t)gm * p.ldc + gn) =
          u32x4_t{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
    }
  }
}

// Split-K reduction + epilogue. One thread per 8 output elements (16-B stores).
// ssq_in (nullable): deferred RMSNorm of the product's rows — the A rows were the raw residual
// stream, so by linearity out[m, :] = inv[m] * (A W^T)[m, :], inv[m] = rsqrt(sum_p ssq_in[p][m] /
// norm_k + eps) over the producer's `parts` row sums ([parts][64] floats; gains folded into W).
__global__ void __launch_bounds__(256)
gemm_splitk_reduce(const float* __restrict__ ws, int splits, int M, int N, int epi,
                   const bf16_t* __restrict__ bias, const bf16_t* __restrict__ resid, int ldr,
                   bf16_t* __restrict__ C, int ldc, const float* __restrict__ ssq_in = nullptr, int parts = 0,
                   int norm_k = 1, float eps = 0.f) {
  const int nout = (epi == EPI_SWIGLU) ? N / 2 : N;
  const int chunks = nout / 8;
  const size_t total = (size_t)M * chunks;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(idx / chunks), oc = (int)(idx % chunks) * 8;
    float inv = 1.f;
    if (ssq_in) {  // a handful of L2-resident floats per row (fixed summation order)
      inv = rsqrtf(sum_strided(ssq_in + m, parts, 64) / norm_k + eps);
    }
    float v[8];
    if (epi == EPI_SWIGLU) {
      const int grp = oc / 16, within = oc % 16;
      const int gc = grp * 32 + within;
      float g[8], u[8];
      sum_rows8(ws + (size_t)m * N + gc, splits, (size_t)M * N, g);
      sum_rows8(ws + (size_t)m * N + gc + 16, splits, (size_t)M * N, u);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = silu(g[e] * inv) * (u[e] * inv);
    } else {
      sum_rows8(ws + (size_t)m * N + oc, splits, (size_t)M * N, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= inv;
      if (bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bf2f(bias[oc + e]);
      }
      if (epi == EPI_GELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
      }
      if (epi == EPI_RESID) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bf2f(resid[(size_t)m * ldr + oc + e]);
      }
    }
    *(u32x4_t*)(C + (size_t)m * ldc + oc) =
        u32x4_t{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
  }
}

// ------------------------------------------------------------------------------------------
// GEMV (M = 1: the batch-1 decode step that sets cache-miss latency). Pure weight streaming:
// every wave instruction loads 1 KiB of ONE weight row (64 lanes x 16 B, fully coalesced,
// non-temporal), R rows x U k-blocks of loads are in flight per wave before any FMA, the 8-wide
// dot products accumulate in fp32 per lane and each row is reduced across the wave once.
// The activation row (K bf16) is read through the caches (every wave reads the same vector).
// EPI_SWIGLU: a wave owns 2 gate rows and their 2 up rows (16-row interleave) -> 2 outputs.
// KS = 2: two neighbouring waves of a workgroup split a row's K range (long rows on narrow
// matrices: the K=8192 down projection has 3072 rows, one 16 KiB row per wave was two dependent
// HBM round trips at U=8) and combine their partial sums through LDS.
template <int EPI, int R, int U, int KS = 1>
__global__ void __launch_bounds__(256)
gemv_kernel(GemmArgs p) {
  static_assert(EPI != EPI_SWIGLU || R == 4, "SwiGLU waves own 2 gate + 2 up rows");
  static_assert(KS == 1 || KS == 2, "KS");
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);  // global wave index
  const int wg = wv / KS, ks = wv % KS;                 // row group, K part
  int rows[R];
  if constexpr (EPI == EPI_SWIGLU) {
    const int g = wg >> 3, t = wg & 7;
#pragma unroll
    for (int r = 0; r < R; ++r) rows[r] = g * 32 + 2 * t + (r & 1) + (r >> 1) * 16;
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) rows[r] = wg * R + r;
  }
  if (KS == 1 && rows[0] >= p.N) return;  // KS = 2: every wave reaches the LDS exchange below
  const bf16_t* wr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = p.W + (size_t)min(rows[r], p.N - 1) * p.K + lane * 8;
  const bf16_t* ar = p.A + lane * 8;
  const bf16_t* gr = p.gamma ? p.gamma + lane * 8 : nullptr;
  // fused RMSNorm: eps > 0 (gamma null = unit gain: the decoder folds RMSNorm gains into the
  // following weights at load, so the GEMV streams no gain vector)
  const bool rms = p.eps > 0.f;
  const int nkb = p.K / 512;
  const int kb0 = ks * nkb / KS, kb1 = (ks + 1) * nkb / KS;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  float ss = 0.f;  // fused RMSNorm: sum of squares of the raw input row (the wave's K range)
  for (int kb = kb0; kb < kb1; kb += U) {
    u32x4_t wv[U][R], av[U], gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = min(kb + u, kb1 - 1) * 512;
#pragma unroll
      for (int r = 0; r < R; ++r) wv[u][r] = __builtin_nontemporal_load((const u32x4_t*)(wr[r] + k));
      av[u] = *(const u32x4_t*)(ar + k);
      if (gr) gv[u] = *(const u32x4_t*)(gr + k);
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
      if (gr) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[2 * e] *= bf2f((bf16_t)(gv[u][e] & 0xffff));
          a[2 * e + 1] *= bf2f((bf16_t)(gv[u][e] >> 16));
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[r] = fmaf(bf2f((bf16_t)(wv[u][r][e] & 0xffff)), a[2 * e], acc[r]);
          acc[r] = fmaf(bf2f((bf16_t)(wv[u][r][e] >> 16)), a[2 * e + 1], acc[r]);
        }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (rms) ss = wave_sum(ss);
  if constexpr (KS == 2) {
    __shared__ float xch[4][R + 1];
    const int w = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) xch[w][r] = acc[r];
      xch[w][R] = ss;
    }
    __syncthreads();
    if (ks != 0 || rows[0] >= p.N) return;
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += xch[w + 1][r];
    ss += xch[w + 1][R];
  }
  if (rms) {
    const float inv = rsqrtf(ss / p.K + p.eps);
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] *= inv;
  }
  if (lane != 0) return;
  if constexpr (EPI == EPI_SWIGLU) {
    const int g = wg >> 3, t = wg & 7;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o = g * 16 + 2 * t + j;
      if (o < p.N / 2) p.C[o] = f2bf(silu(acc[j]) * acc[2 + j]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int n = rows[r];
      if (n >= p.N) continue;
      float v = acc[r];
      if (p.bias) v += bf2f(p.bias[n]);
      if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
      if constexpr (EPI == EPI_RESID) v += bf2f(p.resid[n]);
      p.C[n] = f2bf(v);
    }
  }
}

template <int R, int U, int KS = 1>
static int launch_gemv_r(const GemmArgs& a, int epi, hipStream_t s) {
  const int waves = (a.N + R - 1) / R * KS;
  dim3 grid((waves + 3) / 4), block(256);
  switch (epi) {
    case EPI_NONE: gemv_kernel<EPI_NONE, R, U, KS><<<grid, block, 0, s>>>(a); break;
    case EPI_BIAS: gemv_kernel<EPI_BIAS, R, U, KS><<<grid, block, 0, s>>>(a); break;
    case EPI_GELU: gemv_kernel<EPI_GELU, R, U, KS><<<grid, block, 0, s>>>(a); break;
    case EPI_RESID: gemv_kernel<EPI_RESID, R, U, KS><<<grid, block, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// K-blocks (512 elements = 1 KiB per row) in flight per row: the whole row when it is short
// (K = 3072: 6 blocks, one round of loads and no clamped duplicate loads), 8 per round otherwise.
static int gemv_u(int K, int /*R*/) {
  const int nkb = K / 512;
  if (nkb <= 4) return 4;
  if (nkb == 6) return 6;
  // 8, not the whole row at K = 8192: at U = 16 the compiler sinks the loads to their uses
  // (28 VGPRs, one block in flight) and the down projection drops to ~3 TB/s (measured)
  return 8;
}

template <int R>
static int launch_gemv_ru(const GemmArgs& a, int epi, hipStream_t s) {
  switch (gemv_u(a.K, R)) {
    case 6: return launch_gemv_r<R, 6>(a, epi, s);
    case 8: return launch_gemv_r<R, 8>(a, epi, s);
    default: return launch_gemv_r<R, 4>(a, epi, s);
  }
}

// Rows per wave: enough waves (>= ~4 per SIMD) that the loads in flight cover HBM latency on
// narrow matrices, 4 rows per wave (more bytes per wave) on wide ones.
static int launch_gemv(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.M != 1 || a.K % 512 || a.N % 4) return (int)hipErrorInvalidValue;
  if (epi == EPI_SWIGLU) {
    dim3 grid((a.N / 4 + 3) / 4), block(256);
    switch (gemv_u(a.K, 4)) {
      case 6: gemv_kernel<EPI_SWIGLU, 4, 6><<<grid, block, 0, s>>>(a); break;
      case 8: gemv_kernel<EPI_SWIGLU, 4, 8><<<grid, block, 0, s>>>(a); break;
      default: gemv_kernel<EPI_SWIGLU, 4, 4><<<grid, block, 0, s>>>(a); break;
    }
    return (int)hipGetLastError();
  }
  if (a.N >= 16384) return launch_gemv_ru<4>(a, epi, s);
  if (a.N >= 8192) return launch_gemv_ru<2>(a, epi, s);
  // long rows on a narrow matrix (down projection, K = 8192): two waves per row, 8 blocks each
  if (a.K >= 8192 && a.K % 1024 == 0) return launch_gemv_r<1, 8, 2>(a, epi, s);
  return launch_gemv_ru<1>(a, epi, s);
}

template <int BM, int BN, int WM, int WN, int PF = 1>
static int launch_tile(const GemmArgs& a, int epi, int splits, hipStream_t s) {
  const int ntm = (a.M + BM - 1) / BM, ntn = (a.N + BN - 1) / BN;
  dim3 grid(ntm * ntn, 1, splits), block(256);
  switch (splits > 1 ? (int)EPI_PARTIAL : epi) {
    case EPI_NONE: gemm_bf16_kernel<BM, BN, WM, WN, EPI_NONE, PF><<<grid, block, 0, s>>>(a); break;
    case EPI_BIAS: gemm_bf16_kernel<BM, BN, WM, WN, EPI_BIAS, PF><<<grid, block, 0, s>>>(a); break;
    case EPI_GELU: gemm_bf16_kernel<BM, BN, WM, WN, EPI_GELU, PF><<<grid, block, 0, s>>>(a); break;
    case EPI_SWIGLU: gemm_bf16_kernel<BM, BN, WM, WN, EPI_SWIGLU, PF><<<grid, block, 0, s>>>(a); break;
    case EPI_RESID: gemm_bf16_kernel<BM, BN, WM, WN, EPI_RESID, PF><<<grid, block, 0, s>>>(a); break;
    case EPI_PARTIAL: gemm_bf16_kernel<BM, BN, WM, WN, EPI_PARTIAL, PF><<<grid, block, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// Decode tiles (64x128 / 32x128): 4 k-tiles in flight per workgroup (register prefetch depth 4;
// 1 / 2 / 8 measured slower, profiles/decode_gemm_prefetch_sweep_r1.jsonl).
template <int BM, int BN>
static int launch_decode_tile(const GemmArgs& a, int epi, int splits, hipStream_t s) {
  return launch_tile<BM, BN, 1, 4, 4>(a, epi, splits, s);
}

// Split-K reduction fused with the residual add AND the next RMSNorm (decode layers, M <= 64):
// one workgroup per row sums the fp32 partials, adds bias + residual, writes the new residual
// stream row C, then normalises that (bf16-rounded) row: H = C * rsqrt(mean(C^2) + eps) * gamma.
// Replaces reduce + rmsnorm (two launches, two passes over the row) with one.
__global__ void __launch_bounds__(256)
splitk_reduce_resid_rmsnorm(const float* __restrict__ ws, int splits, int M, int N, const bf16_t* __restrict__ bias,
                            const bf16_t* __restrict__ resid, int ldr, bf16_t* __restrict__ C, int ldc,
                            const bf16_t* __restrict__ gamma, float eps, bf16_t* __restrict__ H, int ldh) {
  constexpr int MAXC = 4;  // N <= 8 * 256 * 4 = 8192
  __shared__ float red[16];
  const int m = blockIdx.x;
  const int nch = N / 8;
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = threadIdx.x + 256 * i;
    if (c >= nch) continue;
    const int oc = c * 8;
    sum_rows8(ws + (size_t)m * N + oc, splits, (size_t)M * N, v[i]);  // 8 splits' loads in flight
    const u32x4_t r = *(const u32x4_t*)(resid + (size_t)m * ldr + oc);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[i][2 * e] += bf2f((bf16_t)(r[e] & 0xffff)) + (bias ? bf2f(bias[oc + 2 * e]) : 0.f);
      v[i][2 * e + 1] += bf2f((bf16_t)(r[e] >> 16)) + (bias ? bf2f(bias[oc + 2 * e + 1]) : 0.f);
    }
    u32x4_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = pack_bf2(v[i][2 * e], v[i][2 * e + 1]);
      v[i][2 * e] = bf2f((bf16_t)(o[e] & 0xffff));       // normalise what the stream holds (bf16)
      v[i][2 * e + 1] = bf2f((bf16_t)(o[e] >> 16));
      ss += v[i][2 * e] * v[i][2 * e] + v[i][2 * e + 1] * v[i][2 * e + 1];
    }
    *(u32x4_t*)(C + (size_t)m * ldc + oc) = o;
  }
  const float inv = rsqrtf(block_sum(ss, red) / N + eps);
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = threadIdx.x + 256 * i;
    if (c >= nch) continue;
    const u32x4_t g = *(const u32x4_t*)(gamma + c * 8);
    u32x4_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = pack_bf2(v[i][2 * e] * inv * bf2f((bf16_t)(g[e] & 0xffff)),
                      v[i][2 * e + 1] * inv * bf2f((bf16_t)(g[e] >> 16)));
    *(u32x4_t*)(H + (size_t)m * ldh + c * 8) = o;
  }
}

// C = resid + A.W^T (+ bias) and H = RMSNorm(C) * gamma in two launches (split-K GEMM + fused
// reduce). M <= 64 (decode), N % 8 == 0, N <= 8192. ws holds splits * M * N floats.
DA_EXPORT int da_gemm_resid_rmsnorm(const void* A, int lda, const void* W, void* C, int ldc, const void* bias,
                                    const void* resid, int ldr, int M, int N, int K, int tile, int splits, void* ws,
                                    const void* gamma, float eps, void* Hout, int ldh, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (K % 64 || N % 8 || N > 8192 || lda % 8 || ldc % 8 || ldh % 8 || !ws || !gamma || !resid || !Hout)
    return (int)hipErrorInvalidValue;
  if (splits < 1 || (K / 64) % splits || M > 128 || (M > 64 && tile != 9)) return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = nullptr; a.resid = nullptr; a.ws = (float*)ws;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldc = ldc; a.ldr = ldr; a.k_per_split = K / splits;
  // tile 9 (65..128 rows): one 128x64 weight-streaming tile per 64 weight rows
  const int err = tile == 9   ? launch_tile<128, 64, 2, 2, 4>(a, EPI_PARTIAL, splits, s)
                  : tile == 2 ? launch_decode_tile<64, 128>(a, EPI_PARTIAL, splits, s)
                              : launch_decode_tile<32, 128>(a, EPI_PARTIAL, splits, s);
  if (err) return err;
  splitk_reduce_resid_rmsnorm<<<M, 256, 0, s>>>((const float*)ws, splits, M, N, (const bf16_t*)bias,
                                                (const bf16_t*)resid, ldr, (bf16_t*)C, ldc, (const bf16_t*)gamma, eps,
                                                (bf16_t*)Hout, ldh);
  DA_LAUNCH_CHECK();
}

// Split-K reduce of a residual-producing decode GEMM (33..64 rows) in the gemm_dk layer structure:
// C = resid + sum of the partials (+ bias), and per-row sums of squares of the bf16 rows C holds,
// one per 512-column part ([N / 512][64] floats: a consumer reads N / 512 floats per row). One wave
// per (row, 512 columns): no norm here, so no workgroup has to see a whole row — 64 rows x 6
// blocks instead of the 64 row-workgroups of splitk_reduce_resid_rmsnorm, whose 98 KB of partials
// per row was read by one CU.
__global__ void __launch_bounds__(64)
splitk_reduce_resid_ssq(const float* __restrict__ ws, int splits, int M, int N, const bf16_t* __restrict__ bias,
                        const bf16_t* __restrict__ resid, int ldr, bf16_t* __restrict__ C, int ldc,
                        float* __restrict__ ssq_out) {
  const int m = blockIdx.y, lane = threadIdx.x;
  const int oc = blockIdx.x * 512 + lane * 8;
  float v[8];
  sum_rows8(ws + (size_t)m * N + oc, splits, (size_t)M * N, v);
  const u32x4_t r = *(const u32x4_t*)(resid + (size_t)m * ldr + oc);
  u32x4_t o;
  float sq = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float lo = v[2 * e] + bf2f((bf16_t)(r[e] & 0xffff)) + (bias ? bf2f(bias[oc + 2 * e]) : 0.f);
    const float hi = v[2 * e + 1] + bf2f((bf16_t)(r[e] >> 16)) + (bias ? bf2f(bias[oc + 2 * e + 1]) : 0.f);
    o[e] = pack_bf2(lo, hi);
    const float bl = bf2f((bf16_t)(o[e] & 0xffff)), bh = bf2f((bf16_t)(o[e] >> 16));
    sq += bl * bl + bh * bh;  // what the stream now holds (bf16)
  }
  *(u32x4_t*)(C + (size_t)m * ldc + oc) = o;
  sq = wave_sum(sq);
  if (lane == 0) ssq_out[(size_t)blockIdx.x * 64 + m] = sq;
}

// gemm_dk's contract (DkArgs semantics, csrc/gemm_dk.hip) for 33..64 rows on the 64x128 split-K
// tiles: epi NONE / BIAS / SWIGLU with an optional deferred norm of A's rows (ssq_in: the raw
// residual stream as A, the row scale applied in the reduce), or EPI_RESID with optional per-part
// sums of squares out (ssq_out: [N / 512][64]). splits >= 2 whenever a reduce is needed; ws holds
// splits * M * N floats.
DA_EXPORT int da_gemm_dk_splitk(const void* A, int lda, const void* W, void* C, int ldc, const void* bias,
                                const void* resid, int ldr, int M, int N, int K, int epi, const float* ssq_in,
                                int ssq_parts, int norm_k, float eps, float* ssq_out, void* ws, int splits,
                                void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M < 1 || M > 64 || K % 64 || N % 16 || lda % 8 || ldc % 8 || !ws || splits < 2 || (K / 64) % splits)
    return (int)hipErrorInvalidValue;
  if (epi == EPI_SWIGLU && N % 32) return (int)hipErrorInvalidValue;
  if (epi == EPI_RESID && (!resid || ldr % 8 || ssq_in)) return (int)hipErrorInvalidValue;
  if (ssq_out && (epi != EPI_RESID || N % 512)) return (int)hipErrorInvalidValue;
  if (ssq_in && (ssq_parts < 1 || norm_k < 1 || !(eps > 0.f))) return (int)hipErrorInvalidValue;
  if (epi != EPI_NONE && epi != EPI_BIAS && epi != EPI_SWIGLU && epi != EPI_RESID) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.ws = (float*)ws;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldc = ldc; a.ldr = ldr; a.k_per_split = K / splits;
  const int err = launch_decode_tile<64, 128>(a, EPI_PARTIAL, splits, s);
  if (err) return err;
  if (epi == EPI_RESID && ssq_out) {
    splitk_reduce_resid_ssq<<<dim3(N / 512, M), 64, 0, s>>>((const float*)ws, splits, M, N, (const bf16_t*)bias,
                                                            (const bf16_t*)resid, ldr, (bf16_t*)C, ldc, ssq_out);
    DA_LAUNCH_CHECK();
  }
  const int nout = (epi == EPI_SWIGLU) ? N / 2 : N;
  const size_t work = (size_t)M * (nout / 8);
  const int blocks = (int)((work + 255) / 256);
  gemm_splitk_reduce<<<blocks, 256, 0, s>>>((const float*)ws, splits, M, N, epi, (const bf16_t*)bias,
                                             (const bf16_t*)resid, ldr, (bf16_t*)C, ldc, ssq_in, ssq_parts, norm_k,
                                             eps);
  DA_LAUNCH_CHECK();
}

// Prefill QKV projection with RoPE + KV-cache write fused into the epilogue (gemm8p EPI_ROPE);
// M >= 256 (the phase-split kernel), N == (H + 2 Hkv) * D, D % 8 == 0. kv_out = 0: the k / v
// columns of C are left unwritten (cache only).
DA_EXPORT int da_gemm_rope(const void* A, int lda, const void* W, void* C, int ldc, int M, int N, int K,
                           const void* pos, const void* slot, const void* cos_sin, void* k_cache, void* v_cache,
                           int H, int Hkv, int D, int max_seq, int kv_out, void* stream) {
  if (K % 64 || K < 128 || N % 8 || lda % 8 || ldc % 8 || D % 8 || M < 256) return (int)hipErrorInvalidValue;
  if (N != (H + 2 * Hkv) * D || !pos || !slot || !cos_sin || !k_cache || !v_cache) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldc = ldc; a.k_per_split = K;
  a.rope = RopeArgs{(const int*)pos, (const int*)slot, (const float*)cos_sin, (bf16_t*)k_cache, (bf16_t*)v_cache,
                    H, Hkv, D, max_seq, kv_out ? 1 : 0};
  const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256);
  return launch_gemm8p(a, EPI_ROPE, (hipStream_t)stream, t256 >= 256 ? 256 : 128);
}

// Tile selection: big tiles when the grid fills 256 CUs, skinny tiles (+ split-K) for decode-sized M.
// tile: 0 = auto, 1 = 128x128, 2 = 64x128, 3 = 32x128, 4 / 7 = 256x256 phase-split (gemm8p),
// 6 = GEMV (M = 1), 8 = 128x128 PF4, 9 = 128x64 PF4, 10 = 128x256 phase-split (gemm8p),
// 13 = 256x256 four-wave (gemm4w).
DA_EXPORT int da_gemm_bf16(const void* A, int lda, const void* W, void* C, int ldc,
                           const void* bias, const void* resid, int ldr,
                           int M, int N, int K, int epi, int tile, int splits, void* ws,
                           const void* rms_gamma, float rms_eps, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (K % 64 || N % 8 || lda % 8 || ldc % 8) return (int)hipErrorInvalidValue;
  if (epi == EPI_SWIGLU && N % 32) return (int)hipErrorInvalidValue;
  if (splits < 1) splits = 1;
  if ((K / 64) % splits) return (int)hipErrorInvalidValue;
  if (splits > 1 && ws == nullptr) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = (const bf16_t*)bias; a.resid = (const bf16_t*)resid; a.ws = (float*)ws;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldc = ldc; a.ldr = ldr; a.k_per_split = K / splits;
  a.gamma = (const bf16_t*)rms_gamma; a.eps = rms_eps;
  if ((rms_gamma || rms_eps > 0.f) && tile != 6) return (int)hipErrorInvalidValue;  // fused RMSNorm: GEMV only
  if (tile == 0) {
    // decode-sized M: 32x128 / 64x128 weight-streaming tiles (+ split-K, chosen by the caller);
    // 65..639 rows: the 64x128 tile over ceil(M/64) row blocks; from 640 rows the phase-split
    // kernel with the row-tile height of fewer workgroup waves (gemm8p_pick_bm; 32-layer Phi-3
    // chain and single-GEMM sweeps: bench/midm_chain.py, bench/gemm_ab.py, profiles/r2, r3)
    if (M <= 32) tile = 3;
    else if (M < 640 || splits > 1) tile = 2;
    else if (K < 128) tile = 1;
    else tile = gemm8p_pick_bm(M, N) == 256 ? 7 : 10;
  }
  if (tile == 4 || tile == 7 || tile == 10) {
    if (splits != 1 || K < 128) return (int)hipErrorInvalidValue;
    return launch_gemm8p(a, epi, s, tile == 10 ? 128 : 256);
  }
  if (tile == 13) {
    if (splits != 1 || K < 128) return (int)hipErrorInvalidValue;
    return launch_gemm4w(a, epi, s);
  }
  if (tile == 6) return launch_gemv(a, epi, s);
  int err;
  switch (tile) {
    case 1: err = launch_tile<128, 128, 2, 2>(a, epi, splits, s); break;
    case 2: err = launch_decode_tile<64, 128>(a, epi, splits, s); break;
    case 3: err = launch_decode_tile<32, 128>(a, epi, splits, s); break;
    case 8: err = launch_tile<128, 128, 2, 2, 4>(a, epi, splits, s); break;   // mid-M weight streaming
    case 9: err = launch_tile<128, 64, 2, 2, 4>(a, epi, splits, s); break;
    default: return (int)hipErrorInvalidValue;
  }
  if (err || splits == 1) return err;
  const int nout = (epi == EPI_SWIGLU) ? N / 2 : N;
  const size_t work = (size_t)M * (nout / 8);
  int blocks = (int)((work + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  gemm_splitk_reduce<<<blocks, 256, 0, s>>>((const float*)ws, splits, M, N, epi, a.bias, a.resid, ldr,
                                             a.C, ldc);
  DA_LAUNCH_CHECK();
}
