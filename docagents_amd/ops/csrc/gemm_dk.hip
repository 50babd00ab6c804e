// Decode GEMM for 2 <= M <= 64 rows with NO split-K partials (gemm_dk).
//
//   C[M, N'] = epi( rownorm(A)[M, K] . W[N, K]^T )
//
// Why: the 64x128 / 32x128 weight-streaming tiles (gemm.hip) need split-K to put enough workgroups
// on 256 CUs, and every split-K GEMM is followed by a reduce launch. In a 32-layer Phi-3 chain at
// M = 16 / 64 those reduces are 4 launches x ~4.7 us per layer — 26 % of the chain
// (rocprofv3 --kernel-trace of bench/midm_chain.py, profiles/r3/chainprof/). Here the K split lives
// INSIDE the workgroup: 4 waves each stream a quarter of K for the same BN weight rows and the four
// accumulator sets are summed through LDS at the end, so a workgroup owns finished outputs and the
// epilogue (bias / residual / SwiGLU) runs in the same launch. Narrow tiles (BN = 16..64 rows of W)
// give >= 192 workgroups without any global split.
//
// Operands go straight from global memory to the MFMA registers (v_mfma_f32_16x16x32_bf16: lane l
// holds row 16 i + (l & 15), k chunk 8 (l >> 4)); nothing is shared between the waves of a workgroup
// (disjoint K quarters), so there is no LDS staging and no barrier in the main loop. PF k-steps of
// A and W fragments are in flight per wave (counted vmcnt waits: the ring is indexed by unrolled
// slot, loads issued in k order).
//
// Deferred RMSNorm (NORM): the decode layer's norms ride here instead of in a reduce launch. The
// producer of the residual stream (EPI_RESID) writes, next to x, per-(workgroup, row) sums of squares
// of its bf16 output slice (ssq_out [parts][64]); the consumer reads x itself as A and scales each A
// fragment by inv[m] = rsqrt(sum_parts / norm_k + eps) before the MFMA (bf16-rounded exactly like
// the rmsnorm kernel's output; the RMSNorm gains are folded into W at load, models/llama.py).
#include "gemm.h"

struct DkArgs {
  const bf16_t* A; const bf16_t* W; bf16_t* C;
  const bf16_t* bias; const bf16_t* resid;
  const float* ssq_in;  // NORM: [ssq_parts][64] partial sums of squares of A's rows
  float* ssq_out;       // EPI_RESID (nullable): [gridDim.x][64] sums of squares of this tile's output rows
  int M, N, K, lda, ldc, ldr, ssq_parts, norm_k;
  float eps;
  int rb;  // row blocks of BM rows: 1, or 2 (M > BM; workgroup pairs share an XCD)
};

template <int BM, int BN, int EPI, bool NORM, int PF>
__global__ void __launch_bounds__(256)
gemm_dk_kernel(DkArgs p) {
  constexpr int FM = BM / 16, FN = BN / 16;
  constexpr int KC = 256;                      // k per chunk: one 64-deep k-tile per wave
  constexpr int ROWB = KC * 2;                 // 512 B per staged row
  constexpr int LW = BN / 8, LA = BM / 8;      // 16-B pieces per thread per chunk (32 per row)
  constexpr int CHUNK = (BN + BM) * ROWB;
  constexpr int SLD = BN + 4;
  constexpr int RED = 4 * BM * SLD * 4;
  constexpr int LDS_BYTES = 2 * CHUNK > RED ? 2 * CHUNK : RED;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  __shared__ float sinv[BM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  // row blocks (M > BM): rb = 2, and the two row blocks of an n-tile are workgroups i and i + 8 —
  // the same XCD under round-robin placement, dispatched together, so the second reads W from L2
  int tile = blockIdx.x, m0 = 0;
  if (p.rb == 2) {
    const int g = blockIdx.x >> 4, wi = blockIdx.x & 15;
    tile = g * 8 + (wi & 7);
    m0 = (wi >> 3) * BM;
  }
  if (tile * BN >= p.N || m0 >= p.M) return;  // whole-workgroup exit (grid padded to 16)
  const int n0 = tile * BN;
  const int Mb = min(BM, p.M - m0);  // rows of this block
  const int nch = p.K / KC;
  const int kl = nch - 1;

  // ---- global -> registers: whole 512-B row segments (32 lanes x 16 B per row), full lines ----
  u32x4_t rw[PF][LW], ra[PF][LA];
  auto gload = [&](u32x4_t (&xw)[LW], u32x4_t (&xa)[LA], int c) {
    const int k0 = c * KC;
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int idx = tid + 256 * i, r = idx >> 5, ch = idx & 31;
      xw[i] = __builtin_nontemporal_load((const u32x4_t*)(p.W + (size_t)min(n0 + r, p.N - 1) * p.K + k0 + ch * 8));
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + 256 * i, r = idx >> 5, ch = idx & 31;
      xa[i] = *(const u32x4_t*)(p.A + (size_t)(m0 + min(r, Mb - 1)) * p.lda + k0 + ch * 8);
    }
  };
  // LDS rows of 512 B; 16-B chunk ch of row r at slot ch ^ (r & 15): the 16 rows one ds_read_b128
  // lane group reads (same chunk) land on 16 distinct slots of a 256-B bank row
  auto lstore = [&](const u32x4_t (&xw)[LW], const u32x4_t (&xa)[LA], int buf) {
    char* sw = smem + buf * CHUNK;
    char* sa = sw + BN * ROWB;
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int idx = tid + 256 * i, r = idx >> 5, ch = idx & 31;
      *(u32x4_t*)(sw + r * ROWB + ((ch ^ (r & 15)) << 4)) = xw[i];
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + 256 * i, r = idx >> 5, ch = idx & 31;
      *(u32x4_t*)(sa + r * ROWB + ((ch ^ (r & 15)) << 4)) = xa[i];
    }
  };

#pragma unroll
  for (int u = 0; u < PF; ++u) {
    gload(rw[u], ra[u], min(u, kl));
    asm volatile("" ::: "memory");  // issue order = chunk order (counted waits)
  }
  // ---- deferred RMSNorm: inv[m] from the producer's per-part sums (fixed summation order) ----
  if constexpr (NORM) {
    // thread = (part lane, 4-row quad): a few independent 16-B loads per thread (a per-row serial
    // walk over the ~200 parts was ~25 dependent L2 round trips), partials combined in LDS in a
    // fixed order
    constexpr int RQ = BM / 4, PL = 256 / RQ;
    __shared__ f32x4_t sq4[PL][RQ];
    const int rq = tid % RQ, pl = tid / RQ;
    f32x4_t a4{0.f, 0.f, 0.f, 0.f};
    // 8 parts' loads issued before their adds (clamped; + 0 past the end is exact: sums of squares
    // are never -0): with ~192 parts on 64 part lanes, `#pragma unroll 4` left a 3-trip remainder
    // loop that waited for each load in turn
    for (int q0 = pl; q0 < p.ssq_parts; q0 += 8 * PL) {
      f32x4_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = *(const f32x4_t*)(p.ssq_in + (size_t)min(q0 + j * PL, p.ssq_parts - 1) * 64 + m0 + 4 * rq);
#pragma unroll
      for (int j = 0; j < 8; ++j) a4 += (q0 + j * PL < p.ssq_parts) ? v[j] : f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    sq4[pl][rq] = a4;
    __syncthreads();
    if (tid < BM) {
      float ss = 0.f;
      for (int q = 0; q < PL; ++q) ss += sq4[q][tid >> 2][tid & 3];
      sinv[tid] = rsqrtf(ss / p.norm_k + p.eps);
    }
  }
  lstore(rw[0], ra[0], 0);
  __syncthreads();
  float inv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) inv[i] = NORM ? sinv[min(16 * i + fr, Mb - 1)] : 1.f;

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < nch; c0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int c = c0 + u;
      const int cur = c & 1;
      // slot u held chunk c, already in LDS: refill it PF chunks ahead (clamped, branch-free)
      if (PF > 1 || c + 1 < nch) gload(rw[u], ra[u], min(c + PF, kl));
      if (c >= nch) continue;
      const char* sw = smem + cur * CHUNK;
      const char* sa = sw + BN * ROWB;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = 8 * w + 4 * kk + fg;  // this wave's k-tile of the chunk
        bf16x8_t af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int r = 16 * i + fr;
          af[i] = *(const bf16x8_t*)(sa + r * ROWB + ((ch ^ (r & 15)) << 4));
          if constexpr (NORM) {
            bf16x8_t y;
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const unsigned pk = pack_bf2(bf2f((bf16_t)af[i][e]) * inv[i], bf2f((bf16_t)af[i][e + 1]) * inv[i]);
              y[e] = (short)(pk & 0xffff);
              y[e + 1] = (short)(pk >> 16);
            }
            af[i] = y;
          }
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = 16 * j + fr;
          bfr[j] = *(const bf16x8_t*)(sw + r * ROWB + ((ch ^ (r & 15)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
      if (c + 1 < nch) lstore(rw[(u + 1) % PF], ra[(u + 1) % PF], cur ^ 1);
      // LDS writes visible + buffer reads done; a raw barrier (a __syncthreads() fence would drain
      // vmcnt and cancel the PF - 1 chunks in flight)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  float (*red)[BM][SLD] = (float (*)[BM][SLD])smem;  // the staging buffers are free now

  // ---- the four K quarters -> one tile, in wave order (deterministic) ----
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[w][16 * i + 4 * fg + q][16 * j + fr] = acc[i][j][q];
  __syncthreads();

  constexpr int BNO = EPI == EPI_SWIGLU ? BN / 2 : BN;  // output columns of the tile
  constexpr int CPR = BNO / 8;                          // 16-B output chunks per row
  static_assert(CPR >= 1 && 256 % CPR == 0, "tile");
  for (int t = tid; t < BM * CPR; t += 256) {
    const int m = t / CPR, ch = t % CPR;
    float v[8];
    if constexpr (EPI == EPI_SWIGLU) {
      const int g = ch >> 1, hh = ch & 1;
      const int gc = 32 * g + 8 * hh;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gt = red[0][m][gc + e] + red[1][m][gc + e] + red[2][m][gc + e] + red[3][m][gc + e];
        const float up = red[0][m][gc + 16 + e] + red[1][m][gc + 16 + e] + red[2][m][gc + 16 + e] +
                         red[3][m][gc + 16 + e];
        v[e] = silu(gt) * up;
      }
      const int oc = n0 / 2 + 16 * g + 8 * hh;
      if (m < Mb && oc < p.N / 2) {  // a ragged last tile (N % BN == 32) holds one gate/up group
        *(u32x4_t*)(p.C + (size_t)(m0 + m) * p.ldc + oc) =
            u32x4_t{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
      }
    } else {
      const int c = 8 * ch;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = red[0][m][c + e] + red[1][m][c + e] + red[2][m][c + e] + red[3][m][c + e];
      const int gn = n0 + c;
      const bool ok = m < Mb && gn < p.N;
      if (p.bias && ok) {
        const u32x4_t b = *(const u32x4_t*)(p.bias + gn);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += bf2f((bf16_t)(b[e] & 0xffff));
          v[2 * e + 1] += bf2f((bf16_t)(b[e] >> 16));
        }
      }
      if constexpr (EPI == EPI_RESID) {
        if (ok) {
          const u32x4_t r = *(const u32x4_t*)(p.resid + (size_t)(m0 + m) * p.ldr + gn);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[2 * e] += bf2f((bf16_t)(r[e] & 0xffff));
            v[2 * e + 1] += bf2f((bf16_t)(r[e] >> 16));
          }
        }
      }
      const u32x4_t o{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
      if (ok) *(u32x4_t*)(p.C + (size_t)(m0 + m) * p.ldc + gn) = o;
      if constexpr (EPI == EPI_RESID) {
        if (p.ssq_out) {  // sum of squares of the bf16 values the stream now holds
          float sq = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = bf2f((bf16_t)(o[e] & 0xffff)), hi = bf2f((bf16_t)(o[e] >> 16));
            sq += lo * lo + hi * hi;
          }
          if (!ok) sq = 0.f;
#pragma unroll
          for (int x = 1; x < CPR; x <<= 1) sq += __shfl_xor(sq, x, 64);
          if (ch == 0) p.ssq_out[(size_t)tile * 64 + m0 + m] = sq;
        }
      }
    }
  }
}

// Output-tile width: the widest of 64 / 32 / 16 W rows that still gives >= 192 workgroups (SwiGLU
// needs whole 32-row gate/up groups).
static int dk_bn(int N, int epi) {
  if (N / 64 >= 192) return 64;
  if (N / 32 >= 192 || epi == EPI_SWIGLU) return 32;
  return 16;
}

// Chunks in flight per workgroup: ~64 KB of W (128 / BN chunks of BN x 512 B) within ~160 VGPRs of
// register staging.
static constexpr int dk_pf(int BM, int BN) {
  int pf = 128 / BN;
  while (pf > 1 && pf * (BN + BM) / 2 > 160) pf /= 2;
  return pf;
}

template <int BM, int BN, int EPI, bool NORM>
static int dk_launch4(const DkArgs& a, hipStream_t s) {
  constexpr int PF = dk_pf(BM, BN);
  const int nt = (a.N + BN - 1) / BN;
  dim3 grid(a.rb == 2 ? (nt + 7) / 8 * 16 : nt), block(256);
  gemm_dk_kernel<BM, BN, EPI, NORM, PF><<<grid, block, 0, s>>>(a);
  return (int)hipGetLastError();
}

template <int BM, int BN, int EPI>
static int dk_launch3(const DkArgs& a, bool norm, hipStream_t s) {
  if constexpr (EPI == EPI_RESID) {  // the residual producers never take a deferred norm
    return norm ? (int)hipErrorInvalidValue : dk_launch4<BM, BN, EPI, false>(a, s);
  } else {
    return norm ? dk_launch4<BM, BN, EPI, true>(a, s) : dk_launch4<BM, BN, EPI, false>(a, s);
  }
}

template <int BM, int BN>
static int dk_launch2(const DkArgs& a, int epi, bool norm, hipStream_t s) {
  switch (epi) {
    case EPI_NONE: case EPI_BIAS: return dk_launch3<BM, BN, EPI_NONE>(a, norm, s);
    case EPI_RESID: return dk_launch3<BM, BN, EPI_RESID>(a, norm, s);
    case EPI_SWIGLU:
      if constexpr (BN >= 32) return dk_launch3<BM, BN, EPI_SWIGLU>(a, norm, s);
      return (int)hipErrorInvalidValue;
    default: return (int)hipErrorInvalidValue;
  }
}

template <int BM>
static int dk_launch1(const DkArgs& a, int epi, bool norm, hipStream_t s) {
  switch (dk_bn(a.N, epi)) {
    case 64: return dk_launch2<BM, 64>(a, epi, norm, s);
    case 32: return dk_launch2<BM, 32>(a, epi, norm, s);
    default: return dk_launch2<BM, 16>(a, epi, norm, s);
  }
}

// Number of ssq parts a RESID launch of width N writes (the consumer's ssq_parts).
DA_EXPORT int da_gemm_dk_parts(int N) { return (N + dk_bn(N, EPI_RESID) - 1) / dk_bn(N, EPI_RESID); }

// epi: EPI_NONE / EPI_BIAS / EPI_RESID / EPI_SWIGLU. ssq_in (nullable): deferred RMSNorm of A's rows
// over ssq_parts parts (norm over norm_k columns, eps); ssq_out (nullable, EPI_RESID only):
// [da_gemm_dk_parts(N)][64] floats. 1 <= M <= 64, K % 256 == 0, N % 16 == 0 (SwiGLU: N % 32 == 0).
DA_EXPORT int da_gemm_dk(const void* A, int lda, const void* W, void* C, int ldc, const void* bias,
                         const void* resid, int ldr, int M, int N, int K, int epi, const float* ssq_in, int ssq_parts,
                         int norm_k, float eps, float* ssq_out, void* stream) {
  if (M < 1 || M > 64 || K % 256 || N % 16 || lda % 8 || ldc % 8) return (int)hipErrorInvalidValue;
  if (epi == EPI_SWIGLU && N % 32) return (int)hipErrorInvalidValue;
  if (epi == EPI_RESID && (!resid || ldr % 8)) return (int)hipErrorInvalidValue;
  if (ssq_out && epi != EPI_RESID) return (int)hipErrorInvalidValue;
  if (ssq_in && (ssq_parts < 1 || norm_k < 1 || !(eps > 0.f))) return (int)hipErrorInvalidValue;
  DkArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = (const bf16_t*)bias; a.resid = (const bf16_t*)resid;
  a.ssq_in = ssq_in; a.ssq_out = ssq_out;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldc = ldc; a.ldr = ldr;
  a.ssq_parts = ssq_parts; a.norm_k = norm_k; a.eps = eps;
  const bool norm = ssq_in != nullptr;
  hipStream_t s = (hipStream_t)stream;
  a.rb = 1;
  if (M <= 16) return dk_launch1<16>(a, epi, norm, s);
  if (M <= 32) return dk_launch1<32>(a, epi, norm, s);
  // 33..64 rows: two 32-row blocks per n-tile (less A re-read per W byte than one 64-row block)
  a.rb = 2;
  return dk_launch1<32>(a, epi, norm, s);
}
