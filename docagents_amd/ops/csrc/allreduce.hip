// Custom all-reduce over xGMI for tensor-parallel decoding.
//
// MI355X nodes connect the 8 GPUs as a full mesh (7 xGMI links x ~153 GB/s per GPU). RCCL's ring
// uses one link per neighbour and pays a multi-microsecond protocol latency per call, which dominates
// the 2 x 80 small all-reduces of every Llama-3-70B TP=8 decode step. Here every rank exposes one
// registered buffer (hipIpcGetMemHandle, opened by every peer), so a kernel reads all 7 peers at once
// over all 7 links:
//
//   one-shot (latency path, decode-sized messages):
//     stage own input -> [flag barrier] -> every rank sums all W buffers in rank order -> out
//   two-shot (bandwidth path, prefill-sized messages):
//     stage -> [barrier] -> reduce own 1/W slice in place -> [barrier] -> gather all slices -> out
//
// Synchronisation is per workgroup, not grid-wide: 16-byte vector v belongs to row v / AR_TPB and
// row r is always handled by workgroup r % gridDim.x, in every phase of every call (the grid size
// is fixed per communicator). So a workgroup only waits for the same workgroup index on its peers.
// Each workgroup keeps its own call counter k in its rank's signal block (device-resident, so the
// launch is HIP-graph capturable with constant arguments); barrier values are 2k+1 / 2k+2
// (monotonic, no reset) and the staging buffer alternates by k's parity, which makes call k+2's
// writes wait for every peer to have finished reading call k.
//
// Memory ordering: staged data is made visible with a system-scope fence (L2 write-back) before the
// flag store (release, system scope) to each peer; waiting threads use system-scope acquire loads,
// then every thread issues a system-scope acquire fence before reading peer memory.
// Every wait is bounded (wall clock): a missing peer sets an error bit and the kernel finishes
// instead of hanging the GPU; the host checks the bit (XgmiAllReduce.check()).
#include <cstring>

#include "common.h"

#define AR_MAX_RANKS 8
#define AR_MAX_BLOCKS 80
#define AR_TPB 256

struct ArPtrs {
  char* p[AR_MAX_RANKS];
};

struct ArSignal {
  uint32_t flags[AR_MAX_BLOCKS][AR_MAX_RANKS];  // flags[b][w]: last barrier value peer w reached
  uint32_t cnt[AR_MAX_BLOCKS];                   // per-workgroup call counter (local only)
  uint32_t err;                                  // bit 0: a barrier timed out
  uint32_t pad[15];
};

__device__ __forceinline__ void ar_barrier(const ArPtrs& sig, ArSignal* self, int rank, int world, int b,
                                           uint32_t val, long long timeout) {
  __threadfence_system();  // this workgroup's staged writes -> memory, before any flag goes out
  __syncthreads();
  if ((int)threadIdx.x < world) {
    ArSignal* peer = (ArSignal*)sig.p[threadIdx.x];
    __hip_atomic_store(&peer->flags[b][rank], val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = &self->flags[b][threadIdx.x];
    const long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - val) < 0) {
      if (wall_clock64() - t0 > timeout) {
        __hip_atomic_fetch_or(&self->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: drop stale cached peer lines
}

template <bool BF16>
__device__ __forceinline__ void acc_add(float (&a)[8], const u32x4_t& x) {
  if (BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[2 * i] += __uint_as_float(x[i] << 16);
      a[2 * i + 1] += __uint_as_float(x[i] & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] += __uint_as_float(x[i]);
  }
}

template <bool BF16>
__device__ __forceinline__ u32x4_t acc_pack(const float (&a)[8]) {
  u32x4_t r;
  if (BF16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = pack_bf2(a[2 * i], a[2 * i + 1]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(a[i]);
  }
  return r;
}

// Sum vector v over all ranks' staging buffers, in rank order (bit-identical on every rank).
template <bool BF16>
__device__ __forceinline__ u32x4_t ar_sum(const ArPtrs& data, long long poff, long long v, int world) {
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  u32x4_t x[AR_MAX_RANKS];
#pragma unroll
  for (int w = 0; w < AR_MAX_RANKS; ++w)
    if (w < world) x[w] = ((const u32x4_t*)data.p[w])[poff + v];  // all loads in flight at once
#pragma unroll
  for (int w = 0; w < AR_MAX_RANKS; ++w)
    if (w < world) acc_add<BF16>(a, x[w]);
  return acc_pack<BF16>(a);
}

template <bool BF16>
__global__ __launch_bounds__(AR_TPB) void allreduce_kernel(ArPtrs data, ArPtrs sig, const u32x4_t* __restrict__ in,
                                                           u32x4_t* __restrict__ out, long long nvec,
                                                           long long slice, long long parity_vec, int rank,
                                                           int world, int twoshot, long long timeout) {
  const int b = blockIdx.x, G = gridDim.x, t = threadIdx.x;
  ArSignal* self = (ArSignal*)sig.p[rank];
  __shared__ uint32_t s_k;
  if (t == 0) s_k = self->cnt[b];
  __syncthreads();
  const uint32_t k = s_k;
  const long long poff = (k & 1) ? parity_vec : 0;
  u32x4_t* mine = (u32x4_t*)data.p[rank] + poff;
  const long long rows = (nvec + AR_TPB - 1) / AR_TPB;

  for (long long r = b; r < rows; r += G) {  // phase 1: stage
    const long long v = r * AR_TPB + t;
    if (v < nvec) mine[v] = in[v];
  }
  ar_barrier(sig, self, rank, world, b, 2u * k + 1u, timeout);

  if (!twoshot) {
    for (long long r = b; r < rows; r += G) {
      const long long v = r * AR_TPB + t;
      if (v < nvec) out[v] = ar_sum<BF16>(data, poff, v, world);
    }
  } else {
    const long long lo = (long long)rank * slice, hi = lo + slice < nvec ? lo + slice : nvec;
    for (long long r = b; r < rows; r += G) {  // phase 2: reduce own slice in place
      const long long v = r * AR_TPB + t;
      if (v >= lo && v < hi) {
        const u32x4_t s = ar_sum<BF16>(data, poff, v, world);
        mine[v] = s;
      }
    }
    ar_barrier(sig, self, rank, world, b, 2u * k + 2u, timeout);
    for (long long r = b; r < rows; r += G) {  // phase 3: gather every slice
      const long long v = r * AR_TPB + t;
      if (v < nvec) out[v] = ((const u32x4_t*)data.p[v / slice])[poff + v];
    }
  }
  if (t == 0) self->cnt[b] = k + 1u;
}

// ---------------------------------------------------------------------------------------------
// One-shot all-reduce with the residual-stream RMSNorm fused into its epilogue (TP decode: the
// row-parallel o / down projection's partial sums are reduced AND the next RMSNorm is applied in
// the same launch, as gemm_resid_norm does at TP = 1). The input rows are this rank's partials,
// rank 0's already including the residual (models/llama.py), so
//   x[r] = bf16(sum over ranks in rank order)      (== allreduce_kernel's output, bit for bit)
//   h[r] = bf16(x[r] * rsqrt(mean(x[r]^2) + eps) * gamma)   (== rmsnorm_kernel on x, bit for bit)
// Bit-identity with the unfused pair holds because the thread -> chunk map, the per-thread
// accumulation order and block_sum are rmsnorm_kernel's (launch with blockDim = its row_threads(D)).
// Partition: whole rows per workgroup (row r -> workgroup r % G) so the norm's reduction stays in
// one workgroup; the per-workgroup counters / barriers / staging parity are allreduce_kernel's, and
// every rank uses the same (rows, G) for a call, so the protocol invariants carry over.
#define ARN_MAXCH 8
__global__ __launch_bounds__(AR_TPB) void allreduce_rmsnorm_kernel(ArPtrs data, ArPtrs sig, const bf16_t* __restrict__ in,
                                                                   bf16_t* __restrict__ xout, bf16_t* __restrict__ hout,
                                                                   const bf16_t* __restrict__ gamma, int rows, int D,
                                                                   float eps, long long parity_vec, int rank, int world,
                                                                   long long timeout) {
  __shared__ float red[16];
  const int b = blockIdx.x, G = gridDim.x, t = threadIdx.x, bd = blockDim.x;
  ArSignal* self = (ArSignal*)sig.p[rank];
  __shared__ uint32_t s_k;
  if (t == 0) s_k = self->cnt[b];
  __syncthreads();
  const uint32_t k = s_k;
  const long long poff = (k & 1) ? parity_vec : 0;
  const int nch = D / 8;
  u32x4_t* mine = (u32x4_t*)data.p[rank] + poff;
  const u32x4_t* inv4 = (const u32x4_t*)in;
  for (int r = b; r < rows; r += G) {  // phase 1: stage own rows
    for (int c = t; c < nch; c += bd) mine[(long long)r * nch + c] = inv4[(long long)r * nch + c];
  }
  ar_barrier(sig, self, rank, world, b, 2u * k + 1u, timeout);
  for (int r = b; r < rows; r += G) {
    float v[ARN_MAXCH][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < ARN_MAXCH; ++i) {
      const int c = t + i * bd;
      if (c < nch) {
        const u32x4_t s = ar_sum<true>(data, poff, (long long)r * nch + c, world);
        *(u32x4_t*)(xout + (size_t)r * D + c * 8) = s;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[i][2 * e] = bf2f((bf16_t)(s[e] & 0xffff));
          v[i][2 * e + 1] = bf2f((bf16_t)(s[e] >> 16));
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
      }
    }
    ss = block_sum(ss, red);
    const float inv = rsqrtf(ss / D + eps);
#pragma unroll
    for (int i = 0; i < ARN_MAXCH; ++i) {
      const int c = t + i * bd;
      if (c < nch) {
        float wv[8];
        if (gamma) {
          const u32x4_t g = *(const u32x4_t*)(gamma + c * 8);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            wv[2 * e] = bf2f((bf16_t)(g[e] & 0xffff));
            wv[2 * e + 1] = bf2f((bf16_t)(g[e] >> 16));
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) wv[e] = 1.f;
        }
        float y[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = v[i][e] * inv * wv[e];
        *(u32x4_t*)(hout + (size_t)r * D + c * 8) =
            u32x4_t{pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3]), pack_bf2(y[4], y[5]), pack_bf2(y[6], y[7])};
      }
    }
    __syncthreads();  // `red` is reused by the next row's block_sum
  }
  if (t == 0) self->cnt[b] = k + 1u;
}

// rows x D bf16 (D % 8 == 0, D / 8 <= ARN_MAXCH * 256); threads = the rmsnorm kernel's row_threads(D);
// grid = min(rows, grid cap). in / xout may alias (in place); gamma may be null (unit gain).
DA_EXPORT int da_ar_allreduce_rmsnorm(const void* in, void* xout, void* hout, const void* gamma, int rows, int D,
                                      float eps, int rank, int world, void* const* data, void* const* sig,
                                      long long parity_bytes, int grid, long long timeout_ticks, hipStream_t stream) {
  if (world < 2 || world > AR_MAX_RANKS || rank < 0 || rank >= world) return (int)hipErrorInvalidValue;
  if (rows <= 0 || D % 8 || D / 8 > ARN_MAXCH * AR_TPB) return (int)hipErrorInvalidValue;
  const long long nbytes = (long long)rows * D * 2;
  if (nbytes > parity_bytes || parity_bytes % 16) return (int)hipErrorInvalidValue;
  if (grid < 1 || grid > AR_MAX_BLOCKS) return (int)hipErrorInvalidValue;
  ArPtrs d{}, s{};
  for (int w = 0; w < world; ++w) {
    d.p[w] = (char*)data[w];
    s.p[w] = (char*)sig[w];
  }
  int ch = D / 8, threads = ((ch + 63) / 64) * 64;  // == norm.hip row_threads(D)
  threads = threads > AR_TPB ? AR_TPB : (threads < 64 ? 64 : threads);
  const int g = rows < grid ? rows : grid;
  allreduce_rmsnorm_kernel<<<g, threads, 0, stream>>>(d, s, (const bf16_t*)in, (bf16_t*)xout, (bf16_t*)hout,
                                                      (const bf16_t*)gamma, rows, D, eps, parity_bytes / 16, rank,
                                                      world, timeout_ticks);
  DA_LAUNCH_CHECK();
}

DA_EXPORT int da_ar_signal_bytes() { return (int)sizeof(ArSignal); }
DA_EXPORT int da_ar_max_blocks() { return AR_MAX_BLOCKS; }
DA_EXPORT int da_ar_block_vecs() { return AR_TPB; }

// uncached != 0: hipDeviceMallocUncached (MTYPE UC). The signal block and the staging buffers are
// written by one device and polled / read by its peers over xGMI; uncached pages keep a stale line
// in any GPU's L2 from hiding a peer's flag or staged rows (coarse-grained hipMalloc memory gives no
// such guarantee across devices; same-device IPC, as in the 1-GPU tests, could never show it).
DA_EXPORT int da_ar_malloc(long long bytes, int uncached, void** out) {
  hipError_t e = uncached ? hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached)
                          : hipMalloc(out, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*out, 0, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

DA_EXPORT int da_ar_free(void* p) { return (int)hipFree(p); }

// Zero a pooled communicator buffer before its next use (signals / flags must start at 0).
DA_EXPORT int da_ar_zero(void* p, long long bytes) {
  const hipError_t e = hipMemset(p, 0, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

DA_EXPORT int da_ar_ipc_handle(void* p, void* handle_out) {
  return (int)hipIpcGetMemHandle((hipIpcMemHandle_t*)handle_out, p);
}

// Export the allocation that CONTAINS p: the runtime may hand out a buffer inside a larger block it
// keeps (seen after other exported buffers were freed: hipIpcGetMemHandle refused the pointer on one
// rank, or exported the block so that peers mapped its start, not the buffer). The importer adds
// *offset_out to the pointer hipIpcOpenMemHandle returns.
DA_EXPORT int da_ar_ipc_export(void* p, void* handle_out, long long* offset_out) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p);
  if (e != hipSuccess) return (int)e;
  *offset_out = (long long)((char*)p - (char*)base);
  return (int)hipIpcGetMemHandle((hipIpcMemHandle_t*)handle_out, (void*)base);
}

DA_EXPORT int da_ar_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

DA_EXPORT int da_ar_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

DA_EXPORT int da_ar_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

DA_EXPORT int da_ar_read_err(void* own_sig, unsigned* out) {
  return (int)hipMemcpy(out, &((ArSignal*)own_sig)->err, sizeof(unsigned), hipMemcpyDeviceToHost);
}

// wall_clock64() ticks per millisecond (the timeout unit of da_ar_allreduce).
DA_EXPORT long long da_ar_clock_khz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 100000;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) return 100000;
  return khz;
}

// Work partition of one call (host side; the kernel follows it): nvec 16-B vectors in rows of
// AR_TPB, row r owned by workgroup r % grid on every rank; two-shot slices are whole rows. Exported
// so the CPU protocol model (tests/test_xgmi_protocol.py) runs the exact partition the kernel runs.
struct ArPlan {
  long long nvec, rows, slice;
  int grid;
};
static ArPlan ar_plan(long long nbytes, int world, int grid, int twoshot) {
  ArPlan p;
  p.nvec = nbytes / 16;
  p.rows = (p.nvec + AR_TPB - 1) / AR_TPB;
  // two-shot: whole rows per slice so every slice boundary is a row boundary
  p.slice = twoshot ? (p.rows + world - 1) / world * AR_TPB : p.nvec;
  // A message with fewer rows than `grid` launches only workgroups 0..rows-1 (one row each, no
  // wrap), which keeps the row -> workgroup mapping, and every rank makes the same choice, so the
  // skipped workgroups' counters stay in step across ranks.
  p.grid = p.rows < grid ? (int)p.rows : grid;
  return p;
}

DA_EXPORT int da_ar_plan(long long nbytes, int world, int grid, int twoshot, long long* out) {
  if (nbytes <= 0 || nbytes % 16 || world < 1 || grid < 1) return (int)hipErrorInvalidValue;
  const ArPlan p = ar_plan(nbytes, world, grid, twoshot);
  out[0] = p.nvec; out[1] = p.rows; out[2] = p.slice; out[3] = p.grid;
  return 0;
}

// in/out: nbytes (multiple of 16) on this rank; data/sig: host arrays of `world` device pointers
// (own + IPC-opened peers); parity_bytes: offset of the second staging half (>= nbytes);
// grid: fixed per communicator (<= AR_MAX_BLOCKS); dtype 0 = bf16, 1 = fp32.
DA_EXPORT int da_ar_allreduce(const void* in, void* out, long long nbytes, int dtype, int rank, int world,
                              void* const* data, void* const* sig, long long parity_bytes, int twoshot, int grid,
                              long long timeout_ticks, hipStream_t stream) {
  if (world < 2 || world > AR_MAX_RANKS || rank < 0 || rank >= world) return (int)hipErrorInvalidValue;
  if (nbytes <= 0 || nbytes % 16 || nbytes > parity_bytes || parity_bytes % 16) return (int)hipErrorInvalidValue;
  if (grid < 1 || grid > AR_MAX_BLOCKS) return (int)hipErrorInvalidValue;
  ArPtrs d{}, s{};
  for (int w = 0; w < world; ++w) {
    d.p[w] = (char*)data[w];
    s.p[w] = (char*)sig[w];
  }
  const ArPlan pl = ar_plan(nbytes, world, grid, twoshot);
  const long long nvec = pl.nvec, slice = pl.slice;
  grid = pl.grid;
  if (dtype == 0)
    allreduce_kernel<true><<<grid, AR_TPB, 0, stream>>>(d, s, (const u32x4_t*)in, (u32x4_t*)out, nvec, slice,
                                                        parity_bytes / 16, rank, world, twoshot, timeout_ticks);
  else
    allreduce_kernel<false><<<grid, AR_TPB, 0, stream>>>(d, s, (const u32x4_t*)in, (u32x4_t*)out, nvec, slice,
                                                         parity_bytes / 16, rank, world, twoshot, timeout_ticks);
  DA_LAUNCH_CHECK();
}
