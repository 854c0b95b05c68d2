// Shared-memory data plane of ray_dynamic_batching_amd (header-only).
//
// One POSIX shm segment per serving "job" holds everything the router, the
// clients and the replica processes exchange on the hot path -- there is no RPC
// on the request path (replacing Ray's actor-RPC + plasma hops,
// core_worker.cc:2488 / plasma store).
//
//   JobHeader | ReplicaState[R] | QueueState[Q] | request rings[Q] | completion rings[C]
//
// * request ring  : MPSC (any client -> one model queue of one replica).  Bounded
//                   Vyukov queue with per-slot sequence numbers; payload inline in
//                   the slot.  The consumer can PEEK ahead and COMMIT later, so a
//                   GPU gather kernel can read payloads in place (the segment is
//                   hipHostRegister'ed) and slots are released only after the copy.
// * completion ring: MPSC (replicas -> one client).
// * QueueState    : submitted/completed counters = the queue depth the router's
//                   power-of-two choice reads with two atomic loads (replacing the
//                   probe RPC of pow_2_scheduler.py:497-598).
// * Histogram     : log-linear latency histograms updated with relaxed atomics.
// * Doorbells     : futex words in shm so an idle consumer sleeps and producers
//                   wake it across processes (no busy polling when idle).
#pragma once
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <fcntl.h>
#include <linux/futex.h>
#include <stdexcept>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace rdb {
namespace rt {

constexpr uint64_t kMagic = 0x3130424F4A424452ULL;  // "RDBJOB01"
constexpr uint32_t kVersion = 5;
constexpr uint32_t kMaxClientFlags = 512;     // clients with a liveness flag (ids beyond share none)
constexpr uint32_t kTraceCap = 8192;          // trace events per replica (power of two)
constexpr uint32_t kSnapshotBytes = 1 << 16;  // seqlock-published snapshot (routing table / plan)
constexpr int kHistSub = 32;       // sub-buckets per power of two (~3% wide)
constexpr int kHistBuckets = 1280;  // covers values up to 2^44 ns

inline int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

inline long futex_wait(std::atomic<uint32_t>* addr, uint32_t expected, int64_t timeout_ns) {
  timespec ts;
  timespec* tp = nullptr;
  if (timeout_ns >= 0) {
    ts.tv_sec = timeout_ns / 1000000000LL;
    ts.tv_nsec = timeout_ns % 1000000000LL;
    tp = &ts;
  }
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAIT, expected, tp, nullptr, 0);
}
inline void futex_wake_all(std::atomic<uint32_t>* addr) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

// ---------------------------------------------------------------------------
// Log-linear histogram: 32 sub-buckets per power of two of a nanosecond value
// (<= 12.5 % relative bucket width), range 1 ns .. ~2^40 ns.
// ---------------------------------------------------------------------------
struct Histogram {
  std::atomic<uint64_t> count;
  std::atomic<uint64_t> sum_ns;
  std::atomic<uint64_t> max_ns;
  std::atomic<uint64_t> buckets[kHistBuckets];

  static int index(uint64_t v) {
    if (v < (uint64_t)kHistSub) return (int)v;
    const int e = 63 - __builtin_clzll(v);  // >= 5
    int idx = (e - 4) * kHistSub + (int)((v >> (e - 5)) & (kHistSub - 1));
    return idx < kHistBuckets ? idx : kHistBuckets - 1;
  }
  static double lower(int idx) {
    if (idx < kHistSub) return idx;
    const int e = idx / kHistSub + 4, m = idx % kHistSub;
    return (double)(1ULL << e) * (1.0 + (double)m / kHistSub);
  }
  static double upper(int idx) { return idx < kHistSub ? idx + 1 : lower(idx + 1 < kHistBuckets ? idx + 1 : idx); }
  static double value_at(int idx) { return 0.5 * (lower(idx) + upper(idx)); }
  void record(uint64_t v) {
    count.fetch_add(1, std::memory_order_relaxed);
    sum_ns.fetch_add(v, std::memory_order_relaxed);
    uint64_t m = max_ns.load(std::memory_order_relaxed);
    while (v > m && !max_ns.compare_exchange_weak(m, v, std::memory_order_relaxed)) {}
    buckets[index(v)].fetch_add(1, std::memory_order_relaxed);
  }
  void reset() {
    count.store(0);
    sum_ns.store(0);
    max_ns.store(0);
    for (auto& b : buckets) b.store(0);
  }
  double percentile(double p) const {  // p in [0, 100]
    const uint64_t n = count.load(std::memory_order_relaxed);
    if (n == 0) return 0.0;
    const double target = p / 100.0 * (double)n;
    uint64_t acc = 0;
    for (int i = 0; i < kHistBuckets; ++i) {
      const uint64_t c = buckets[i].load(std::memory_order_relaxed);
      if (c && (double)(acc + c) >= target) {  // linear interpolation inside the bucket
        const double f = std::min(1.0, std::max(0.0, (target - (double)acc) / (double)c));
        const double v = lower(i) + f * (upper(i) - lower(i));
        return std::min(v, (double)max_ns.load(std::memory_order_relaxed));
      }
      acc += c;
    }
    return (double)max_ns.load();
  }
};

// ---------------------------------------------------------------------------
// Ring sequence-check debug mode ("a debug mode for the rings that
// checks sequence numbers"; the reference's analogue is the _RAY_TSAN_BUILD /
// sanitizer CI configs, .bazelrc:103-136).  RDB_RING_DEBUG=1 checks every
// publish / peek / commit against the Vyukov protocol's invariants:
//   publish(pos): the slot still holds the producer's reservation (seq == pos);
//   peek(pos)   : pos is not behind the consumer's tail, and the slot holds
//                 either pos (not yet published) or pos + 1 (published);
//   commit(upto): tail <= upto <= head, and every released slot is published.
// A violation is counted (process-wide), reported on stderr with the ring,
// position and sequence number, and the slot is treated as unpublished so the
// consumer never reads it; RDB_RING_DEBUG=2 aborts instead (core dump at the
// first bad access).  Off (the default) the checks cost one predictable branch.
// ---------------------------------------------------------------------------
inline int ring_debug_level() {
  static const int lvl = [] {
    const char* e = getenv("RDB_RING_DEBUG");
    return e ? atoi(e) : 0;
  }();
  return lvl;
}
struct RingDebugState {
  std::atomic<uint64_t> violations{0};
  char last[256] = {0};
};
inline RingDebugState& ring_debug_state() {
  static RingDebugState st;
  return st;
}
__attribute__((noinline, cold)) inline void ring_violation(const void* ring, const char* what, uint64_t pos,
                                                           uint64_t seq, uint64_t extra) {
  RingDebugState& st = ring_debug_state();
  st.violations.fetch_add(1, std::memory_order_relaxed);
  snprintf(st.last, sizeof(st.last), "ring %p: %s (pos=%llu seq=%llu other=%llu)", ring, what,
           (unsigned long long)pos, (unsigned long long)seq, (unsigned long long)extra);
  fprintf(stderr, "[rdb ring debug] %s\n", st.last);
  if (ring_debug_level() >= 2) abort();
}

// ---------------------------------------------------------------------------
// Bounded MPSC ring.
// ---------------------------------------------------------------------------
struct alignas(64) SlotHeader {
  std::atomic<uint64_t> seq;
  uint64_t req_id;
  int64_t t_submit_ns;
  int64_t deadline_ns;  // absolute CLOCK_MONOTONIC; 0 = none
  uint32_t len;         // payload bytes
  uint16_t kind;        // 0 = raw tensor bytes, 1 = pickled python object
  uint16_t client;      // completion ring to answer on
  uint32_t queue;       // request: target queue; completion: originating queue
  uint32_t status;      // completion status (see Status)
  int64_t t_aux_ns;     // completion: time the replica finished
};
static_assert(sizeof(SlotHeader) == 64, "slot header must be one cache line");

enum Status : uint32_t {
  ST_OK = 0,
  ST_DROPPED_STALE = 1,   // deadline could not be met (fork: scheduler.py:281-283)
  ST_ERROR = 2,           // user code / model raised
  ST_REJECTED = 3,        // replica over max_ongoing_requests
  ST_TOO_LARGE = 4,       // payload or result does not fit a slot
  ST_SHUTDOWN = 5,
  ST_REPLICA_DIED = 6,
};

struct alignas(64) RingHeader {
  uint32_t capacity;  // power of two
  uint32_t slot_bytes;
  uint64_t _pad0[7];
  alignas(64) std::atomic<uint64_t> head;
  alignas(64) std::atomic<uint64_t> tail;
  alignas(64) std::atomic<uint32_t> doorbell;
  std::atomic<uint32_t> waiters;
};

struct Ring {
  RingHeader* h = nullptr;
  char* slots = nullptr;

  static size_t bytes(uint32_t cap, uint32_t slot_bytes) {
    return sizeof(RingHeader) + (size_t)cap * slot_bytes;
  }
  void init(uint32_t cap, uint32_t slot_bytes) {
    h->capacity = cap;
    h->slot_bytes = slot_bytes;
    h->head.store(0);
    h->tail.store(0);
    h->doorbell.store(0);
    h->waiters.store(0);
    for (uint32_t i = 0; i < cap; ++i) slot(i)->seq.store(i, std::memory_order_relaxed);
  }
  SlotHeader* slot(uint64_t pos) const {
    return reinterpret_cast<SlotHeader*>(slots + (size_t)(pos & (h->capacity - 1)) * h->slot_bytes);
  }
  char* payload(SlotHeader* s) const { return reinterpret_cast<char*>(s) + sizeof(SlotHeader); }
  uint32_t max_payload() const { return h->slot_bytes - (uint32_t)sizeof(SlotHeader); }

  // Producer: reserve a slot; returns nullptr if full.  Must be followed by publish().
  SlotHeader* reserve(uint64_t* out_pos) {
    uint64_t pos = h->head.load(std::memory_order_relaxed);
    for (;;) {
      SlotHeader* s = slot(pos);
      const uint64_t seq = s->seq.load(std::memory_order_acquire);
      const int64_t dif = (int64_t)seq - (int64_t)pos;
      if (dif == 0) {
        if (h->head.compare_exchange_weak(pos, pos + 1, std::memory_order_relaxed)) {
          *out_pos = pos;
          return s;
        }
      } else if (dif < 0) {
        return nullptr;  // full
      } else {
        const uint64_t prev = pos;
        pos = h->head.load(std::memory_order_relaxed);
        if (__builtin_expect(ring_debug_level() > 0, 0) && pos == prev) {
          // head did not move, yet the slot claims a later lap: a stray
          // publish; without the check this producer spins here forever
          ring_violation(h, "reserve: free slot carries a sequence number ahead of head", pos, seq, 0);
          return nullptr;
        }
      }
    }
  }
  void publish(SlotHeader* s, uint64_t pos) {
    if (__builtin_expect(ring_debug_level() > 0, 0)) {
      const uint64_t q = s->seq.load(std::memory_order_acquire);
      if (q != pos) ring_violation(h, "publish: slot no longer holds this producer's reservation", pos, q, 0);
    }
    s->seq.store(pos + 1, std::memory_order_seq_cst);
    if (h->waiters.load(std::memory_order_seq_cst) > 0) {
      h->doorbell.fetch_add(1, std::memory_order_seq_cst);
      futex_wake_all(&h->doorbell);
    }
  }
  // Consumer side (single consumer).  peek(pos) returns the slot at absolute
  // position pos if it has been published.
  SlotHeader* peek(uint64_t pos) const {
    SlotHeader* s = slot(pos);
    const uint64_t q = s->seq.load(std::memory_order_acquire);
    if (__builtin_expect(ring_debug_level() > 0, 0)) return checked_peek(s, pos, q);
    return q == pos + 1 ? s : nullptr;
  }
  __attribute__((noinline)) SlotHeader* checked_peek(SlotHeader* s, uint64_t pos, uint64_t q) const {
    const uint64_t tail = h->tail.load(std::memory_order_acquire);
    if (pos < tail) {
      ring_violation(h, "peek behind the consumer's tail", pos, q, tail);
      return nullptr;
    }
    if (q == pos + 1) return s;
    if (q != pos) ring_violation(h, "peek: sequence number is neither free nor published for this lap", pos, q, 0);
    return nullptr;
  }
  // Release every slot in [tail, upto).
  void commit(uint64_t upto) {
    uint64_t t = h->tail.load(std::memory_order_relaxed);
    if (__builtin_expect(ring_debug_level() > 0, 0)) {
      const uint64_t head = h->head.load(std::memory_order_acquire);
      if (upto < t || upto > head) {
        ring_violation(h, "commit outside [tail, head]", upto, t, head);
        return;
      }
      for (uint64_t k = t; k < upto; ++k) {
        const uint64_t q = slot(k)->seq.load(std::memory_order_acquire);
        if (q != k + 1) {
          ring_violation(h, "commit releases an unpublished slot", k, q, 0);
          return;
        }
      }
    }
    for (; t < upto; ++t) slot(t)->seq.store(t + h->capacity, std::memory_order_release);
    h->tail.store(upto, std::memory_order_release);
  }
  uint64_t depth() const {
    return h->head.load(std::memory_order_relaxed) - h->tail.load(std::memory_order_relaxed);
  }
  // Block until the slot at `pos` is published or timeout (ns, <0 = forever).
  bool wait_for(uint64_t pos, int64_t timeout_ns, int spin = 2000) const {
    for (int i = 0; i < spin; ++i) {
      if (peek(pos)) return true;
      cpu_relax();
    }
    const int64_t deadline = timeout_ns >= 0 ? now_ns() + timeout_ns : INT64_MAX;
    for (;;) {
      h->waiters.fetch_add(1, std::memory_order_seq_cst);
      const uint32_t bell = h->doorbell.load(std::memory_order_seq_cst);
      if (peek(pos)) {
        h->waiters.fetch_sub(1, std::memory_order_seq_cst);
        return true;
      }
      int64_t left = deadline == INT64_MAX ? 50000000LL : deadline - now_ns();
      if (left <= 0) {
        h->waiters.fetch_sub(1, std::memory_order_seq_cst);
        return false;
      }
      if (left > 50000000LL) left = 50000000LL;  // re-check at least every 50 ms
      futex_wait(&h->doorbell, bell, left);
      h->waiters.fetch_sub(1, std::memory_order_seq_cst);
      if (peek(pos)) return true;
      if (deadline != INT64_MAX && now_ns() >= deadline) return false;
    }
  }
  // Wake a sleeping consumer (used for shutdown).
  void ring_bell() {
    h->doorbell.fetch_add(1, std::memory_order_seq_cst);
    futex_wake_all(&h->doorbell);
  }
};

// ---------------------------------------------------------------------------
// Job segment layout.
// ---------------------------------------------------------------------------
enum ReplicaStatus : uint32_t { RS_UNUSED = 0, RS_STARTING = 1, RS_READY = 2, RS_DRAINING = 3, RS_DEAD = 4 };

struct alignas(64) ReplicaState {
  std::atomic<uint32_t> status;
  std::atomic<uint32_t> pid;
  std::atomic<int32_t> gpu;
  std::atomic<uint32_t> restarts;
  std::atomic<int64_t> heartbeat_ns;
  std::atomic<uint64_t> batches;
  std::atomic<uint64_t> batch_items;
  std::atomic<uint64_t> padded_items;
  std::atomic<uint64_t> busy_ns;        // GPU busy time (launch -> done)
  std::atomic<uint64_t> graph_replays;
  Histogram hist_batch_size;            // raw batch sizes (value = size)
  Histogram hist_service;               // batch formation -> completion
};

constexpr int kMuxSlots = 16;
struct alignas(64) QueueState {
  std::atomic<uint32_t> active;         // 1 if a replica serves this queue
  std::atomic<uint32_t> replica;        // owning replica
  std::atomic<uint32_t> model;          // model / deployment id
  std::atomic<uint32_t> max_ongoing;    // admission bound (max_ongoing_requests)
  std::atomic<uint64_t> submitted;
  std::atomic<uint64_t> completed;
  std::atomic<uint64_t> dropped;
  std::atomic<uint64_t> errors;
  std::atomic<uint64_t> slo_violations;
  std::atomic<int64_t> slo_ns;          // per-model SLO used for violation counting
  Histogram hist_queue_wait;            // submit -> batch launch
  Histogram hist_e2e;                   // submit -> completion written
  // model multiplexing: 64-bit hashes of the multiplexed model ids this queue's
  // replica holds (0 = empty slot), published by the replica on load / evict;
  // the router prefers queues holding the requested id
  // (serve/_private/replica_scheduler/pow_2_scheduler.py:330-345, 396-443)
  std::atomic<uint64_t> mux[kMuxSlots];
};

// Per-replica trace ring (chrome-trace export, utils/tracing.py): multi-writer,
// overwrite-oldest.  Times are CLOCK_MONOTONIC ns like every other stamp here.
enum TraceKind : uint32_t { TK_FORM = 1, TK_GPU = 2, TK_COMPLETE = 3, TK_DROP = 4, TK_PY_BATCH = 5 };
struct TraceEvent {
  int64_t t0, t1;
  uint32_t kind;
  uint16_t queue, n;
  uint32_t bucket;
  std::atomic<uint32_t> seq;  // publication stamp (event index + 1)
};
struct alignas(64) TraceRing {
  std::atomic<uint64_t> head;
  TraceEvent ev[kTraceCap];
  void record(uint32_t kind, int64_t t0, int64_t t1, uint32_t queue, uint32_t n, uint32_t bucket) {
    const uint64_t i = head.fetch_add(1, std::memory_order_relaxed);
    TraceEvent& e = ev[i & (kTraceCap - 1)];
    e.seq.store(0, std::memory_order_relaxed);
    e.t0 = t0;
    e.t1 = t1;
    e.kind = kind;
    e.queue = (uint16_t)queue;
    e.n = (uint16_t)std::min<uint32_t>(n, 65535);
    e.bucket = bucket;
    e.seq.store((uint32_t)(i + 1), std::memory_order_release);
  }
};

// Seqlock-versioned snapshot (replaces Ray's long-poll / pub-sub for the
// routing table and the planner's placement: writers bump seq to odd, copy,
// bump to even; readers retry while odd or changed).
struct alignas(64) Snapshot {
  std::atomic<uint64_t> seq;
  std::atomic<uint32_t> len;
  // payload as relaxed atomic words: the concurrent copy of a seqlock is then
  // race-free in the C++ memory model (and clean under -fsanitize=thread)
  std::atomic<uint64_t> words[kSnapshotBytes / 8];
  uint64_t publish(const char* p, uint32_t n) {
    if (n > kSnapshotBytes) throw std::length_error("snapshot too large");
    uint64_t s = seq.load(std::memory_order_relaxed);
    while (!(s % 2 == 0 && seq.compare_exchange_weak(s, s + 1, std::memory_order_acquire))) {
      s = seq.load(std::memory_order_relaxed);
    }
    std::atomic_thread_fence(std::memory_order_release);
    for (uint32_t i = 0; i < (n + 7) / 8; ++i) {
      uint64_t w = 0;
      memcpy(&w, p + 8 * i, std::min<uint32_t>(8, n - 8 * i));
      words[i].store(w, std::memory_order_relaxed);
    }
    len.store(n, std::memory_order_relaxed);
    seq.store(s + 2, std::memory_order_release);
    return (s + 2) / 2;
  }
  // Returns the version (0 = never published) and fills out.
  uint64_t read(std::string& out) const {
    for (;;) {
      const uint64_t s0 = seq.load(std::memory_order_acquire);
      if (s0 & 1) continue;
      const uint32_t n = std::min<uint32_t>(len.load(std::memory_order_relaxed), kSnapshotBytes);
      out.resize(n);
      for (uint32_t i = 0; i < (n + 7) / 8; ++i) {
        const uint64_t w = words[i].load(std::memory_order_relaxed);
        memcpy(&out[8 * i], &w, std::min<uint32_t>(8, n - 8 * i));
      }
      std::atomic_thread_fence(std::memory_order_acquire);
      if (seq.load(std::memory_order_relaxed) == s0) return s0 / 2;
    }
  }
};

struct alignas(4096) JobHeader {
  std::atomic<uint64_t> magic;  // written last by the creator
  uint32_t version;
  uint32_t n_replicas;
  uint32_t n_queues;
  uint32_t n_clients;
  uint32_t req_capacity;
  uint32_t req_slot_bytes;
  uint32_t cmp_capacity;
  uint32_t cmp_slot_bytes;
  uint64_t off_replicas, off_queues, off_req, off_cmp, off_trace, off_snap, total_bytes;
  std::atomic<uint32_t> clients_registered;
  std::atomic<uint32_t> shutdown;
  std::atomic<uint64_t> next_req_id;
  std::atomic<int64_t> created_ns;
  char name[128];
  // Completion-side liveness: a client whose completion ring stayed full for a
  // whole completion timeout is marked stalled; producers then drop (and count)
  // its completions instead of blocking, until the client polls again.  One
  // wedged proxy can therefore never stall the replica's completer for others.
  std::atomic<uint64_t> cmp_dropped;
  std::atomic<uint32_t> client_stalled[kMaxClientFlags];
};
static_assert(sizeof(JobHeader) == 4096, "job header must stay one page");

struct JobConfig {
  uint32_t n_replicas = 1, n_queues = 1, n_clients = 8;
  uint32_t req_capacity = 4096, req_slot_bytes = 1024;
  uint32_t cmp_capacity = 8192, cmp_slot_bytes = 256;
  // Leave the request rings' slot pages untouched at creation: each queue's
  // consumer initialises its own ring (Job::init_req_ring) after binding those
  // pages to its GPU's NUMA node, so payloads are first-touched -- and later
  // gathered by the GPU -- on the consumer's socket, not the creator's.
  bool defer_req_rings = false;
};

// Bind [addr, addr + len) to one NUMA node (MPOL_PREFERRED; no libnuma
// needed).  Returns 0 or -errno.  A node < 0 is a no-op.
inline int mbind_preferred(void* addr, size_t len, int node) {
  if (node < 0 || node >= 1024) return 0;
  unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
  mask[node / (8 * sizeof(unsigned long))] = 1UL << (node % (8 * sizeof(unsigned long)));
  const long rc = syscall(SYS_mbind, addr, len, 1 /* MPOL_PREFERRED */, mask, (unsigned long)1024, 0);
  return rc == 0 ? 0 : -errno;
}

inline uint32_t round_pow2(uint32_t v) {
  uint32_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
inline uint32_t round_up(uint32_t v, uint32_t a) { return (v + a - 1) / a * a; }

class Job {
 public:
  Job() = default;
  ~Job() { close(); }
  Job(const Job&) = delete;
  Job& operator=(const Job&) = delete;

  // Create (and initialise) a segment; fails if it already exists unless overwrite.
  void create(const std::string& name, JobConfig cfg, bool overwrite = true) {
    name_ = name;
    cfg.req_capacity = round_pow2(cfg.req_capacity);
    cfg.cmp_capacity = round_pow2(cfg.cmp_capacity);
    cfg.req_slot_bytes = round_up(cfg.req_slot_bytes + (uint32_t)sizeof(SlotHeader), 64);
    cfg.cmp_slot_bytes = round_up(cfg.cmp_slot_bytes + (uint32_t)sizeof(SlotHeader), 64);
    const uint64_t off_rep = sizeof(JobHeader);
    const uint64_t off_q = off_rep + (uint64_t)cfg.n_replicas * sizeof(ReplicaState);
    uint64_t off_req = off_q + (uint64_t)cfg.n_queues * sizeof(QueueState);
    off_req = (off_req + 4095) & ~4095ULL;
    const uint64_t req_ring_sz = (Ring::bytes(cfg.req_capacity, cfg.req_slot_bytes) + 4095) & ~4095ULL;
    const uint64_t off_cmp = off_req + req_ring_sz * cfg.n_queues;
    const uint64_t cmp_ring_sz = (Ring::bytes(cfg.cmp_capacity, cfg.cmp_slot_bytes) + 4095) & ~4095ULL;
    const uint64_t off_trace = off_cmp + cmp_ring_sz * cfg.n_clients;
    const uint64_t off_snap = (off_trace + (uint64_t)cfg.n_replicas * sizeof(TraceRing) + 4095) & ~4095ULL;
    const uint64_t total = (off_snap + sizeof(Snapshot) + 4095) & ~4095ULL;
    if (overwrite) shm_unlink(shm_path().c_str());
    int fd = shm_open(shm_path().c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name + ": " + strerror(errno));
    if (ftruncate(fd, (off_t)total) != 0) {
      ::close(fd);
      throw std::runtime_error("ftruncate failed: " + std::string(strerror(errno)));
    }
    map(fd, total);
    created_ = true;
    JobHeader* h = hdr();
    h->version = kVersion;
    h->n_replicas = cfg.n_replicas;
    h->n_queues = cfg.n_queues;
    h->n_clients = cfg.n_clients;
    h->req_capacity = cfg.req_capacity;
    h->req_slot_bytes = cfg.req_slot_bytes;
    h->cmp_capacity = cfg.cmp_capacity;
    h->cmp_slot_bytes = cfg.cmp_slot_bytes;
    h->off_replicas = off_rep;
    h->off_queues = off_q;
    h->off_req = off_req;
    h->off_cmp = off_cmp;
    h->off_trace = off_trace;
    h->off_snap = off_snap;
    h->total_bytes = total;
    h->clients_registered.store(0);
    h->shutdown.store(0);
    h->next_req_id.store(1);
    h->created_ns.store(now_ns());
    strncpy(h->name, name.c_str(), sizeof(h->name) - 1);
    for (uint32_t q = 0; q < cfg.n_queues; ++q) {
      if (cfg.defer_req_rings) {       // header only (one page); slots wait for init_req_ring
        Ring r = req_ring(q);
        r.h->capacity = cfg.req_capacity;
        r.h->slot_bytes = cfg.req_slot_bytes;
      } else {
        req_ring(q).init(cfg.req_capacity, cfg.req_slot_bytes);
      }
    }
    for (uint32_t c = 0; c < cfg.n_clients; ++c) cmp_ring(c).init(cfg.cmp_capacity, cfg.cmp_slot_bytes);
    h->magic.store(kMagic, std::memory_order_release);
  }

  // Attach to an existing segment, waiting up to timeout for the creator.
  void attach(const std::string& name, int64_t timeout_ns = 30000000000LL) {
    name_ = name;
    const int64_t deadline = now_ns() + timeout_ns;
    int fd = -1;
    for (;;) {
      fd = shm_open(shm_path().c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && st.st_size >= (off_t)sizeof(JobHeader)) {
          map(fd, (size_t)st.st_size);
          if (hdr()->magic.load(std::memory_order_acquire) == kMagic) break;
          unmap();
        } else {
          ::close(fd);
        }
      }
      if (now_ns() > deadline) throw std::runtime_error("timed out attaching to shm job " + name);
      usleep(2000);
    }
    if (hdr()->version != kVersion) throw std::runtime_error("shm job version mismatch");
  }

  void close() {
    unmap();
    if (created_ && unlink_on_close_) shm_unlink(shm_path().c_str());
    created_ = false;
  }
  void set_unlink_on_close(bool v) { unlink_on_close_ = v; }
  bool valid() const { return base_ != nullptr; }

  JobHeader* hdr() const { return reinterpret_cast<JobHeader*>(base_); }
  ReplicaState* replica(uint32_t i) const {
    return reinterpret_cast<ReplicaState*>(base_ + hdr()->off_replicas) + i;
  }
  QueueState* queue(uint32_t i) const {
    return reinterpret_cast<QueueState*>(base_ + hdr()->off_queues) + i;
  }
  Ring req_ring(uint32_t q) const {
    const uint64_t sz = (Ring::bytes(hdr()->req_capacity, hdr()->req_slot_bytes) + 4095) & ~4095ULL;
    char* p = base_ + hdr()->off_req + sz * q;
    Ring r;
    r.h = reinterpret_cast<RingHeader*>(p);
    r.slots = p + sizeof(RingHeader);
    return r;
  }
  Ring cmp_ring(uint32_t c) const {
    const uint64_t sz = (Ring::bytes(hdr()->cmp_capacity, hdr()->cmp_slot_bytes) + 4095) & ~4095ULL;
    char* p = base_ + hdr()->off_cmp + sz * c;
    Ring r;
    r.h = reinterpret_cast<RingHeader*>(p);
    r.slots = p + sizeof(RingHeader);
    return r;
  }
  TraceRing* trace(uint32_t r) const { return reinterpret_cast<TraceRing*>(base_ + hdr()->off_trace) + r; }
  Snapshot* snapshot() const { return reinterpret_cast<Snapshot*>(base_ + hdr()->off_snap); }
  char* base() const { return base_; }
  size_t size() const { return size_; }
  const std::string& name() const { return name_; }
  // Consumer-side initialisation of request ring q (JobConfig::defer_req_rings):
  // bind its pages to `numa_node` (< 0: leave the policy alone), then write the
  // slot sequence numbers from this (CPU-pinned) process: first touch is local.
  // Must run before any producer can pick the queue.  Returns the mbind result.
  int init_req_ring(uint32_t q, int numa_node) {
    Ring r = req_ring(q);
    const uint64_t sz = (Ring::bytes(hdr()->req_capacity, hdr()->req_slot_bytes) + 4095) & ~4095ULL;
    const int rc = mbind_preferred(reinterpret_cast<char*>(r.h), sz, numa_node);
    r.init(hdr()->req_capacity, hdr()->req_slot_bytes);
    return rc;
  }
  // Byte range of the request rings (what a GPU replica pins for zero-copy H2D).
  std::pair<char*, size_t> request_region() const {
    return {base_ + hdr()->off_req, (size_t)(hdr()->off_cmp - hdr()->off_req)};
  }

 private:
  std::string shm_path() const { return "/rdb_" + name_; }
  void map(int fd, size_t sz) {
    void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap failed: " + std::string(strerror(errno)));
    base_ = reinterpret_cast<char*>(p);
    size_ = sz;
  }
  void unmap() {
    if (base_) munmap(base_, size_);
    base_ = nullptr;
    size_ = 0;
  }
  std::string name_;
  char* base_ = nullptr;
  size_t size_ = 0;
  bool created_ = false;
  bool unlink_on_close_ = true;
};

// How long a completion producer waits on a FULL completion ring before it
// declares that client stalled (RDB_COMPLETION_TIMEOUT_MS, default 2000).
// Read on the slow path only (a full ring), so tests may change it at run time.
inline int64_t completion_timeout_ns() {
  const char* e = getenv("RDB_COMPLETION_TIMEOUT_MS");
  const long long ms = e ? atoll(e) : 2000;
  return (int64_t)(ms > 0 ? ms : 2000) * 1000000LL;
}

inline bool client_stalled(const Job& job, uint32_t client) {
  return client < kMaxClientFlags && job.hdr()->client_stalled[client].load(std::memory_order_relaxed) != 0;
}
// Called by a client whenever it drains its completion ring: it is alive again.
inline void clear_client_stalled(Job& job, uint32_t client) {
  if (client < kMaxClientFlags && job.hdr()->client_stalled[client].load(std::memory_order_relaxed))
    job.hdr()->client_stalled[client].store(0, std::memory_order_relaxed);
}

// Reserve a slot on `client`'s completion ring.  Waits (spin, then yield /
// sleep) while the ring is full, but never unboundedly: after `timeout_ns` the
// client is marked stalled and nullptr is returned (the caller drops that
// completion and must still account for it).  A client already marked stalled
// gets exactly one non-blocking attempt per completion.  Also returns nullptr
// as soon as `abort()` becomes true (replica stopping / job shutdown).
template <typename Abort>
inline SlotHeader* reserve_completion(Job& job, uint32_t client, uint64_t* pos, Abort&& abort,
                                      int64_t timeout_ns = -1) {
  Ring c = job.cmp_ring(client);
  if (SlotHeader* s = c.reserve(pos)) return s;
  if (client_stalled(job, client)) {
    job.hdr()->cmp_dropped.fetch_add(1, std::memory_order_relaxed);
    return nullptr;
  }
  const int64_t t0 = now_ns();
  const int64_t limit = timeout_ns >= 0 ? timeout_ns : completion_timeout_ns();
  for (int i = 0;; ++i) {
    if (SlotHeader* s = c.reserve(pos)) return s;
    if (abort()) return nullptr;
    if (now_ns() - t0 > limit) {
      if (client < kMaxClientFlags) job.hdr()->client_stalled[client].store(1, std::memory_order_relaxed);
      job.hdr()->cmp_dropped.fetch_add(1, std::memory_order_relaxed);
      return nullptr;
    }
    if (i < 256) cpu_relax();
    else usleep(i < 4096 ? 0 : 50);
  }
}

// Complete every request still in queue q's ring (unconsumed, or consumed but
// not yet committed by a replica that died) with `status`, so its clients can
// retry elsewhere.  Used by the router on drain and by the node agent when a
// replica process dies or stops heart-beating.
inline uint64_t fail_pending(Job& job, uint32_t q, uint32_t status) {
  Ring ring = job.req_ring(q);
  QueueState* qs = job.queue(q);
  uint64_t pos = ring.h->tail.load();
  uint64_t n = 0;
  while (SlotHeader* s = ring.peek(pos)) {
    Ring c = job.cmp_ring(s->client);
    uint64_t cpos;
    SlotHeader* out = reserve_completion(job, s->client, &cpos, [] { return false; });
    if (!out) {  // stalled client: the failure notice is dropped, the request still leaves the queue
      ++pos;
      ++n;
      continue;
    }
    out->req_id = s->req_id;
    out->t_submit_ns = s->t_submit_ns;
    out->deadline_ns = s->deadline_ns;
    out->len = 0;
    out->kind = 0;
    out->client = s->client;
    out->queue = q;
    out->status = status;
    out->t_aux_ns = now_ns();
    c.publish(out, cpos);
    ++pos;
    ++n;
  }
  ring.commit(pos);
  qs->completed.fetch_add(n);
  qs->errors.fetch_add(n);
  return n;
}

// After a replica died: requests it had already consumed will never complete
// (routers re-dispatch them on the generation bump), so stop counting them as
// ongoing -- otherwise the restarted replica looks saturated forever.
inline void forget_inflight(Job& job, uint32_t q) {
  QueueState* qs = job.queue(q);
  const uint64_t sub = qs->submitted.load();
  uint64_t done = qs->completed.load();
  while (done < sub && !qs->completed.compare_exchange_weak(done, sub)) {}
}

}  // namespace rt
}  // namespace rdb
