// Custom all-reduce over xGMI peer memory for tensor-parallel replicas inside
// one MI355X node (SURVEY.md §7.1 "comm (C++) -- custom xGMI one-shot/two-shot
// all-reduce", §7.4 item 6; reference surface: python/ray/util/collective/
// collective.py:258 allreduce over nccl_collective_group.py:188).
//
// Design (MI355X-first, not a ring):
//  * xGMI is a full mesh of point-to-point links (7 per GPU), so every rank
//    talks to every peer DIRECTLY; a ring would drive one link at a time.
//  * PUSH, not pull: a rank writes its data into the owner's receive slots
//    with plain 16-B stores through the IPC mapping (posted writes, no
//    round-trip latency per load), then publishes one flag per (block, rank).
//    All receive / gather / signal buffers are fine-grained UNCACHED device
//    memory (hipDeviceMallocUncached), so peer stores land in HBM and local
//    reads never hit a stale L2/L1 line.
//  * two-shot (large messages): rank r owns rows [r*C, (r+1)*C), C = ceil(T/N).
//      A: push row chunk p of the local input to owner p's recv[r] slot
//      -- barrier A --
//      B: reduce own chunk over the N recv slots (fixed order q = 0..N-1, so
//         every rank gets bit-identical sums), push the reduced rows into
//         EVERY rank's gather buffer (= the all-reduced output x)
//      -- barrier B --
//      C: (fused RMSNorm) h = x * rsqrt(mean(x^2) + eps) * gamma, full rows
//    Each rank sends/receives 2 x (N-1)/N of the message: the bandwidth-optimal
//    volume, spread over all 7 links at once.
//  * one-shot (small messages, latency-bound): push the whole input to every
//    peer, ONE barrier, every rank reduces all rows locally (fixed order) and
//    fuses the RMSNorm in registers.  The receive slots are double-buffered by
//    call parity, which is what makes the single barrier safe.
//  * Barriers are per BLOCK: block i of every rank runs the same rows in every
//    phase, so block i only waits for block i of its peers (no grid barrier,
//    no co-residency assumption across blocks).  Epochs are per-block counters
//    kept in device memory (valid under hipGraph replay: no frozen arguments).
//  * Every spin is bounded (wall clock): on timeout the block records an error
//    code in its signal block and exits, so a dead peer cannot hang the GPU.
#include "common.h"
#include <cstring>
#include <cstddef>
#include <stdexcept>
#include <string>
#include <vector>

namespace rdb {

constexpr int kXgMaxRanks = 8;
constexpr int kXgMaxBlocks = 256;
constexpr int kXgThreads = 256;

struct XgSignal {
  uint32_t a[kXgMaxBlocks][kXgMaxRanks];  // barrier A flags, written by peers
  uint32_t b[kXgMaxBlocks][kXgMaxRanks];  // barrier B flags, written by peers
  uint32_t counter[kXgMaxBlocks];         // per-block call epoch, owner block only
  uint32_t error;                         // != 0: a barrier timed out (1 = A, 2 = B)
  uint32_t pad[3];
};

struct XgArgs {
  char* recv[kXgMaxRanks];        // each rank's receive region: [2 parity][N src][slot] elements
  char* gather[kXgMaxRanks];      // each rank's gather buffer (the output x), [T, D]
  XgSignal* sig[kXgMaxRanks];
  const char* in;                 // local input [T, D]
  char* out_norm;                 // local RMSNorm output [T, D] (NORM only)
  const char* gamma;              // [D]
  float eps;
  int world, rank, T, D;
  long long slot_elems;           // elements per receive slot
  unsigned long long timeout_ticks;
  unsigned long long* dbg;        // optional per-block launch-view record (8 x u64 per block)
  int norm_store;                 // out_norm stores: 0 plain, 1 nontemporal, 2 sc1 (write-through)
};

template <typename T> struct Vec8;
template <> struct Vec8<bf16> { typedef bf16x8 type; };
template <> struct Vec8<f16> { typedef f16x8 type; };

__device__ __forceinline__ u32x4 ld16(const char* p) { return *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void st16(char* p, u32x4 v) { *reinterpret_cast<u32x4*>(p) = v; }
// Store of the fused-norm output (mode chosen per call, uniform branch).
__device__ __forceinline__ void st_norm(char* p, u32x4 v, int mode) {
  if (mode == 0) {
    st16(p, v);
  } else if (mode == 1) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  } else {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) __hip_atomic_store(q + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <typename T>
__device__ __forceinline__ void acc8(float (&a)[8], u32x4 raw) {
  typedef typename Vec8<T>::type V;
  const V v = __builtin_bit_cast(V, raw);
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] += (float)v[e];
}
template <typename T>
__device__ __forceinline__ u32x4 pack8(const float (&a)[8]) {
  typedef typename Vec8<T>::type V;
  V v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (T)a[e];
  return __builtin_bit_cast(u32x4, v);
}
template <typename T>
__device__ __forceinline__ void unpack8(float (&a)[8], u32x4 raw) {
  typedef typename Vec8<T>::type V;
  const V v = __builtin_bit_cast(V, raw);
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = (float)v[e];
}

// Publish "block blk of this rank reached barrier `which`" to every peer, then
// wait until every peer's block blk did.  Returns false on timeout (all threads
// agree through LDS).
__device__ bool xg_barrier(const XgArgs& a, int which, uint32_t epoch, int blk, int* s_fail) {
  const int tid = threadIdx.x;
  // every wave: its pushed stores are complete before the flag goes out
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope (peers are other agents)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid < a.world) {
      uint32_t* f = which == 0 ? &a.sig[tid]->a[blk][a.rank] : &a.sig[tid]->b[blk][a.rank];
      __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    XgSignal* me = a.sig[a.rank];
    bool ok = true;
    if (tid < a.world) {
      uint32_t* f = which == 0 ? &me->a[blk][tid] : &me->b[blk][tid];
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > a.timeout_ticks) {
          __hip_atomic_store(&me->error, (uint32_t)(which + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ok = false;
          break;
        }
      }
    }
    ok = __all(ok);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) *s_fail = ok ? 0 : 1;
  }
  __syncthreads();
  return *s_fail == 0;
}

// Block-wide sum over 256 threads (4 waves).
__device__ __forceinline__ float block_sum(float v, float* s_red) {
  v = wave_sum(v);
  const int tid = threadIdx.x;
  __syncthreads();
  if ((tid & 63) == 0) s_red[tid >> 6] = v;
  __syncthreads();
  return s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

// RMSNorm of one row held in registers (f32), written as T to dst.
template <typename T, int VPT>
__device__ __forceinline__ void norm_row(const XgArgs& a, float (&x)[VPT][8], int nvec, char* dst, float* s_red) {
  const int tid = threadIdx.x;
  float ss = 0.f;
#pragma unroll
  for (int v = 0; v < VPT; ++v)
    if (tid + v * kXgThreads < nvec)
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += x[v][e] * x[v][e];
  const float rstd = rsqrtf(block_sum(ss, s_red) / (float)a.D + a.eps);
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const int idx = tid + v * kXgThreads;
    if (idx < nvec) {
      float g[8];
      unpack8<T>(g, ld16(a.gamma + (size_t)idx * 16));
      float y[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = x[v][e] * rstd * g[e];
      st_norm(dst + (size_t)idx * 16, pack8<T>(y), a.norm_store);
    }
  }
}

template <typename T, int VPT, bool TWO_SHOT, bool NORM>
__global__ void __launch_bounds__(kXgThreads) xgmi_allreduce_kernel(XgArgs a) {
  __shared__ uint32_t s_epoch;
  __shared__ int s_fail;
  __shared__ float s_red[4];
  const int tid = threadIdx.x, blk = blockIdx.x, G = gridDim.x;
  const int N = a.world, r = a.rank;
  XgSignal* me = a.sig[r];
  if (tid == 0) s_epoch = __hip_atomic_load(&me->counter[blk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1;
  __syncthreads();
  const uint32_t epoch = s_epoch;
  const int par = epoch & 1;
  if (a.dbg && tid == 0) {  // what this block sees of its launch (kernarg / graph-replay diagnostics)
    unsigned long long* d = a.dbg + (size_t)blk * 8;
    d[0] = (unsigned long long)a.out_norm;
    d[1] = (unsigned long long)a.gamma;
    d[2] = (unsigned long long)a.in;
    d[3] = (unsigned long long)a.gather[r];
    d[4] = (unsigned long long)a.sig[r];
    d[5] = ((unsigned long long)a.T << 32) | (unsigned)a.D;
    d[6] = epoch;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    d[7] = xcc & 0xf;
  }
  // A timed-out barrier still advances this block's epoch (below), so the
  // rank stays in step with its peers; the sticky error flag poisons the
  // communicator on the host side (XgmiCommunicator.check()).
  auto finish = [&]() {
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&me->counter[blk], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  const size_t rowb = (size_t)a.D * sizeof(T);
  const int nvec = a.D / 8;
  const size_t slotb = (size_t)a.slot_elems * sizeof(T);
  // receive slot of source rank q in rank p's region, current parity
  auto slot = [&](int p, int q) -> char* { return a.recv[p] + ((size_t)par * N + q) * slotb; };

  if constexpr (TWO_SHOT) {
    const int C = (a.T + N - 1) / N;
    // ---- A: scatter row chunks to their owners ----
    for (int p = 0; p < N; ++p) {
      const int rows = min(C, a.T - p * C);
      for (int l = blk; l < rows; l += G) {
        const char* src = a.in + (size_t)(p * C + l) * rowb;
        char* dst = slot(p, r) + (size_t)l * rowb;
        u32x4 v[VPT];
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int idx = tid + i * kXgThreads;
          if (idx < nvec) v[i] = ld16(src + (size_t)idx * 16);
        }
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int idx = tid + i * kXgThreads;
          if (idx < nvec) st16(dst + (size_t)idx * 16, v[i]);
        }
      }
    }
    if (!xg_barrier(a, 0, epoch, blk, &s_fail)) { finish(); return; }
    // ---- B: reduce own chunk, all-gather the reduced rows ----
    const int my_rows = min(C, a.T - r * C);
    for (int l = blk; l < my_rows; l += G) {
      float acc[VPT][8];
#pragma unroll
      for (int i = 0; i < VPT; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[i][e] = 0.f;
      for (int q = 0; q < N; ++q) {
        const char* src = slot(r, q) + (size_t)l * rowb;
        u32x4 v[VPT];
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int idx = tid + i * kXgThreads;
          v[i] = idx < nvec ? ld16(src + (size_t)idx * 16) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int i = 0; i < VPT; ++i) acc8<T>(acc[i], v[i]);
      }
      const size_t off = (size_t)(r * C + l) * rowb;
      u32x4 pk[VPT];
#pragma unroll
      for (int i = 0; i < VPT; ++i) pk[i] = pack8<T>(acc[i]);
      for (int p = 0; p < N; ++p) {
        char* dst = a.gather[p] + off;
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int idx = tid + i * kXgThreads;
          if (idx < nvec) st16(dst + (size_t)idx * 16, pk[i]);
        }
      }
    }
    if (!xg_barrier(a, 1, epoch, blk, &s_fail)) { finish(); return; }
    // ---- C: RMSNorm over the gathered rows this block's peers pushed ----
    if constexpr (NORM) {
      for (int p = 0; p < N; ++p) {
        const int rows = min(C, a.T - p * C);
        for (int l = blk; l < rows; l += G) {
          const size_t off = (size_t)(p * C + l) * rowb;
          float x[VPT][8];
#pragma unroll
          for (int i = 0; i < VPT; ++i) {
            const int idx = tid + i * kXgThreads;
            if (idx < nvec) unpack8<T>(x[i], ld16(a.gather[r] + off + (size_t)idx * 16));
          }
          norm_row<T, VPT>(a, x, nvec, a.out_norm + off, s_red);
        }
      }
    }
  } else {
    // ---- A: push the whole local input to every peer (own rows are read in place) ----
    for (int row = blk; row < a.T; row += G) {
      const char* src = a.in + (size_t)row * rowb;
      u32x4 v[VPT];
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int idx = tid + i * kXgThreads;
        if (idx < nvec) v[i] = ld16(src + (size_t)idx * 16);
      }
      for (int p = 0; p < N; ++p) {
        if (p == r) continue;
        char* dst = slot(p, r) + (size_t)row * rowb;
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int idx = tid + i * kXgThreads;
          if (idx < nvec) st16(dst + (size_t)idx * 16, v[i]);
        }
      }
    }
    if (!xg_barrier(a, 0, epoch, blk, &s_fail)) { finish(); return; }
    // ---- B: every rank reduces every row (same order on all ranks) ----
    for (int row = blk; row < a.T; row += G) {
      float acc[VPT][8];
#pragma unroll
      for (int i = 0; i < VPT; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[i][e] = 0.f;
      for (int q = 0; q < N; ++q) {
        const char* src = (q == r ? a.in : slot(r, q)) + (size_t)row * rowb;
        u32x4 v[VPT];
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const int idx = tid + i * kXgThreads;
          v[i] = idx < nvec ? ld16(src + (size_t)idx * 16) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int i = 0; i < VPT; ++i) acc8<T>(acc[i], v[i]);
      }
      // round to T first: the norm sees exactly the x every rank returns
      float x[VPT][8];
      const size_t off = (size_t)row * rowb;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const u32x4 pk = pack8<T>(acc[i]);
        const int idx = tid + i * kXgThreads;
        if (idx < nvec) st16(a.gather[r] + off + (size_t)idx * 16, pk);
        unpack8<T>(x[i], pk);
      }
      if constexpr (NORM) norm_row<T, VPT>(a, x, nvec, a.out_norm + off, s_red);
    }
  }
  finish();
}

template <typename T, int VPT>
static void launch_vpt(const XgArgs& a, bool two_shot, bool norm, int grid, hipStream_t s) {
  if (two_shot) {
    if (norm) hipLaunchKernelGGL((xgmi_allreduce_kernel<T, VPT, true, true>), dim3(grid), dim3(kXgThreads), 0, s, a);
    else hipLaunchKernelGGL((xgmi_allreduce_kernel<T, VPT, true, false>), dim3(grid), dim3(kXgThreads), 0, s, a);
  } else {
    if (norm) hipLaunchKernelGGL((xgmi_allreduce_kernel<T, VPT, false, true>), dim3(grid), dim3(kXgThreads), 0, s, a);
    else hipLaunchKernelGGL((xgmi_allreduce_kernel<T, VPT, false, false>), dim3(grid), dim3(kXgThreads), 0, s, a);
  }
}

template <typename T>
static void launch_t(const XgArgs& a, bool two_shot, bool norm, int grid, hipStream_t s) {
  const int nvec = a.D / 8;
  if (nvec <= kXgThreads) launch_vpt<T, 1>(a, two_shot, norm, grid, s);
  else if (nvec <= 2 * kXgThreads) launch_vpt<T, 2>(a, two_shot, norm, grid, s);
  else launch_vpt<T, 4>(a, two_shot, norm, grid, s);
}

size_t xgmi_signal_bytes() { return sizeof(XgSignal); }

// dtype: 0 = bf16, 1 = f16.  Pointers are this process's views of every rank's
// buffers (IPC-mapped for peers).  The output x is written to gather[rank].
void xgmi_allreduce(int dtype, const std::vector<uintptr_t>& recv, const std::vector<uintptr_t>& gather,
                    const std::vector<uintptr_t>& sig, int rank, uintptr_t in, uintptr_t out_norm,
                    uintptr_t gamma, float eps, int T, int D, long long slot_elems, int two_shot,
                    int grid, unsigned long long timeout_ticks, uintptr_t stream, uintptr_t dbg,
                    int norm_store) {
  const int N = (int)recv.size();
  if (N < 1 || N > kXgMaxRanks || (int)gather.size() != N || (int)sig.size() != N)
    throw std::invalid_argument("xgmi_allreduce: 1..8 ranks with one recv/gather/signal buffer each");
  if (rank < 0 || rank >= N) throw std::invalid_argument("xgmi_allreduce: bad rank");
  if (D % 8 != 0 || D > 8 * 4 * kXgThreads) throw std::invalid_argument("xgmi_allreduce: D % 8 == 0, D <= 8192");
  if (T <= 0) return;
  const long long need = two_shot ? (long long)((T + N - 1) / N) * D : (long long)T * D;
  if (need > slot_elems) throw std::invalid_argument("xgmi_allreduce: message exceeds the receive slot");
  if ((in | gather[rank]) & 15) throw std::invalid_argument("xgmi_allreduce: buffers must be 16-byte aligned");
  if (out_norm && (!gamma || (out_norm & 15) || (gamma & 15)))
    throw std::invalid_argument("xgmi_allreduce: norm output / gamma must be 16-byte aligned");
  if (grid <= 0 || grid > kXgMaxBlocks) throw std::invalid_argument("xgmi_allreduce: grid must be 1..256");
  XgArgs a{};
  for (int i = 0; i < N; ++i) {
    a.recv[i] = reinterpret_cast<char*>(recv[i]);
    a.gather[i] = reinterpret_cast<char*>(gather[i]);
    a.sig[i] = reinterpret_cast<XgSignal*>(sig[i]);
  }
  a.in = reinterpret_cast<const char*>(in);
  a.out_norm = reinterpret_cast<char*>(out_norm);
  a.gamma = reinterpret_cast<const char*>(gamma);
  a.eps = eps;
  a.world = N;
  a.rank = rank;
  a.T = T;
  a.D = D;
  a.slot_elems = slot_elems;
  a.timeout_ticks = timeout_ticks;
  a.dbg = reinterpret_cast<unsigned long long*>(dbg);
  if (norm_store < 0 || norm_store > 2) throw std::invalid_argument("xgmi_allreduce: norm_store 0..2");
  a.norm_store = norm_store;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool norm = out_norm != 0;
  if (dtype == 0) launch_t<bf16>(a, two_shot != 0, norm, grid, s);
  else if (dtype == 1) launch_t<f16>(a, two_shot != 0, norm, grid, s);
  else throw std::invalid_argument("xgmi_allreduce: bf16 / f16 only");
  RDB_HIP_CHECK(hipGetLastError());
}

// ---- buffers and IPC ----------------------------------------------------------
uintptr_t xgmi_alloc_uncached(size_t bytes) {
  void* p = nullptr;
  RDB_HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
  RDB_HIP_CHECK(hipMemset(p, 0, bytes));
  RDB_HIP_CHECK(hipDeviceSynchronize());
  return reinterpret_cast<uintptr_t>(p);
}
void xgmi_free(uintptr_t p) { RDB_HIP_CHECK(hipFree(reinterpret_cast<void*>(p))); }

std::string xgmi_ipc_handle(uintptr_t p) {
  hipIpcMemHandle_t h;
  RDB_HIP_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(p)));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}
uintptr_t xgmi_ipc_open(const std::string& handle) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("xgmi_ipc_open: bad handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  void* p = nullptr;
  RDB_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<uintptr_t>(p);
}
void xgmi_ipc_close(uintptr_t p) { RDB_HIP_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(p))); }

uint32_t xgmi_read_error(uintptr_t sig) {
  uint32_t e = 0;
  RDB_HIP_CHECK(hipMemcpy(&e, reinterpret_cast<const char*>(sig) + offsetof(XgSignal, error), 4, hipMemcpyDeviceToHost));
  return e;
}

unsigned long long xgmi_ticks_per_second() {
  int dev = 0, khz = 0;
  RDB_HIP_CHECK(hipGetDevice(&dev));
  RDB_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  return (unsigned long long)(khz > 0 ? khz : 100000) * 1000ull;
}

}  // namespace rdb
