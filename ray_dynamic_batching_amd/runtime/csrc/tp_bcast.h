// Tensor-parallel batch broadcast: a single-writer / N-reader record ring in
// its own POSIX shared-memory segment, one per TP replica group (epoch).
//
// Rank 0 of a TP replica forms each batch (first-arrival timeout over the
// replica's request ring) and publishes ONE record per batch -- (session,
// bucket, pipeline slot, n) plus the n request rows -- here; every follower
// rank reads every record in publish order, copies the rows into its pinned
// staging slot, releases the record and replays the same bucket graph (whose
// RCCL / xGMI all-reduces pair up across ranks because every rank launches the
// same graphs in the same order).  This replaces a per-batch RCCL broadcast of a
// header + the token ids and the two host syncs that reading the header needs
// (the round-5 Python loop), and idle followers sleep on a futex instead of
// joining a collective every 50 ms.
//
// Reference role: the fork's rank-0 -> worker hand-off is a Ray actor call per
// batch; the NCCL group's rendezvous is a named actor
// (python/ray/util/collective/collective_group/nccl_collective_group.py:555-577).
//
// Protocol (x86-TSO and the atomics below):
//   writer: wait until head - min(consumed[r]) < n_slots; fill slot head % n;
//           rec->seq = head + 1 (release); head = head + 1 (release); doorbell++.
//   reader r: wait until slot (next % n)->seq == next + 1 (acquire); read;
//           consumed[r] = next + 1 (release); free_bell++.
// `closed` (writer shutting down, or a peer declared the group dead) wakes
// every waiter; a closed ring never blocks again.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "shm.h"

namespace rdb {
namespace rt {

struct alignas(64) BcastHeader {
  uint64_t magic;
  uint32_t version;
  uint32_t n_slots;
  uint32_t n_readers;
  uint32_t pad0;
  uint64_t slot_bytes;                      // record header + payload capacity
  alignas(64) std::atomic<uint64_t> head;   // records published
  alignas(64) std::atomic<uint32_t> doorbell;   // futex: bumped per publish
  alignas(64) std::atomic<uint32_t> free_bell;  // futex: bumped per release
  std::atomic<uint32_t> closed;
};

struct alignas(64) BcastConsumed {           // one cache line per reader
  std::atomic<uint64_t> consumed;
  char pad[56];
};

struct alignas(64) BcastRecord {
  std::atomic<uint64_t> seq;   // publish index + 1 once the record is complete
  int32_t kind;                // BCAST_BATCH / BCAST_STOP
  int32_t a, b, c;             // engine: session, bucket index, pipeline slot
  uint32_t n;                  // requests in the batch
  uint32_t len;                // payload bytes that follow the header
  int64_t t_pub_ns;
};

enum BcastKind { BCAST_BATCH = 0, BCAST_STOP = 1 };

class TPBcast {
 public:
  static constexpr uint64_t kMagic = 0x5244425442434153ULL;   // "RDBTBCAS"
  static constexpr uint32_t kVersion = 1;
  static constexpr uint32_t kMaxReaders = 64;

  TPBcast() = default;
  ~TPBcast() { close_map(); }
  TPBcast(const TPBcast&) = delete;
  TPBcast& operator=(const TPBcast&) = delete;

  // Leader: create the segment (a stale one of the same name is replaced).
  void create(const std::string& name, uint32_t n_readers, uint32_t n_slots, uint64_t payload_bytes) {
    if (n_readers > kMaxReaders) throw std::invalid_argument("tp_bcast: at most 64 readers");
    if (n_slots < 2) throw std::invalid_argument("tp_bcast: at least 2 slots");
    name_ = name;
    const uint64_t slot_bytes = (sizeof(BcastRecord) + payload_bytes + 63) & ~63ULL;
    const size_t total = sizeof(BcastHeader) + sizeof(BcastConsumed) * kMaxReaders + slot_bytes * n_slots;
    shm_unlink(path().c_str());
    int fd = shm_open(path().c_str(), O_RDWR | O_CREAT | O_EXCL, 0600);
    if (fd < 0) throw std::runtime_error("tp_bcast: shm_open(create) failed for " + name);
    if (ftruncate(fd, (off_t)total) != 0) {
      ::close(fd);
      throw std::runtime_error("tp_bcast: ftruncate failed");
    }
    map(fd, total);
    BcastHeader* h = hdr();
    h->n_slots = n_slots;
    h->n_readers = n_readers;
    h->slot_bytes = slot_bytes;
    h->head.store(0);
    h->doorbell.store(0);
    h->free_bell.store(0);
    h->closed.store(0);
    for (uint32_t r = 0; r < kMaxReaders; ++r) consumed(r).store(0);
    for (uint32_t s = 0; s < n_slots; ++s) rec(s)->seq.store(0);
    h->version = kVersion;
    std::atomic_thread_fence(std::memory_order_release);
    reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->store(kMagic, std::memory_order_release);
    created_ = true;
  }

  // Follower: attach, waiting up to timeout for the leader to create it.
  void attach(const std::string& name, int64_t timeout_ns) {
    name_ = name;
    const int64_t deadline = now_ns() + timeout_ns;
    for (;;) {
      int fd = shm_open(path().c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && st.st_size >= (off_t)sizeof(BcastHeader)) {
          map(fd, (size_t)st.st_size);
          if (reinterpret_cast<std::atomic<uint64_t>*>(&hdr()->magic)->load(std::memory_order_acquire) == kMagic)
            break;
          close_map();
        } else {
          ::close(fd);
        }
      }
      if (now_ns() > deadline) throw std::runtime_error("tp_bcast: timed out attaching to " + name);
      usleep(2000);
    }
    if (hdr()->version != kVersion) throw std::runtime_error("tp_bcast: version mismatch");
  }

  // Remove the name once every rank has attached (the mappings stay valid):
  // nothing is left in /dev/shm when a group is SIGKILLed later.
  void unlink() { if (!name_.empty()) shm_unlink(path().c_str()); }

  uint64_t payload_capacity() const { return hdr()->slot_bytes - sizeof(BcastRecord); }
  uint32_t n_readers() const { return hdr()->n_readers; }
  bool closed() const { return hdr()->closed.load(std::memory_order_acquire) != 0; }
  void close() {
    hdr()->closed.store(1, std::memory_order_release);
    hdr()->doorbell.fetch_add(1, std::memory_order_release);
    hdr()->free_bell.fetch_add(1, std::memory_order_release);
    futex_wake_all(&hdr()->doorbell);
    futex_wake_all(&hdr()->free_bell);
  }
  uint64_t head() const { return hdr()->head.load(std::memory_order_acquire); }

  // Writer side, in two steps so the caller fills the payload in place:
  // reserve() waits for a free slot (false on close / timeout) and returns the
  // record; commit() publishes it.
  BcastRecord* reserve(int64_t timeout_ns) {
    BcastHeader* h = hdr();
    const uint64_t pos = h->head.load(std::memory_order_relaxed);
    const int64_t deadline = timeout_ns < 0 ? INT64_MAX : now_ns() + timeout_ns;
    int spin = 0;
    for (;;) {
      if (closed()) return nullptr;
      const uint32_t bell = h->free_bell.load(std::memory_order_acquire);
      uint64_t low = pos;
      for (uint32_t r = 0; r < h->n_readers; ++r) low = std::min(low, consumed(r).load(std::memory_order_acquire));
      if (pos - low < h->n_slots) break;
      if (++spin < 2000) {
        cpu_relax();
        continue;
      }
      const int64_t left = deadline - now_ns();
      if (left <= 0) return nullptr;
      futex_wait(&h->free_bell, bell, std::min<int64_t>(left, 50000000));
    }
    BcastRecord* r = rec((uint32_t)(pos % h->n_slots));
    return r;
  }
  char* payload(BcastRecord* r) const { return reinterpret_cast<char*>(r) + sizeof(BcastRecord); }
  void commit(BcastRecord* r) {
    BcastHeader* h = hdr();
    const uint64_t pos = h->head.load(std::memory_order_relaxed);
    r->t_pub_ns = now_ns();
    r->seq.store(pos + 1, std::memory_order_release);
    h->head.store(pos + 1, std::memory_order_release);
    h->doorbell.fetch_add(1, std::memory_order_release);
    futex_wake_all(&h->doorbell);
  }
  bool publish(int32_t kind, int32_t a, int32_t b, int32_t c, uint32_t n, const void* data, uint32_t len,
               int64_t timeout_ns) {
    if (len > payload_capacity()) throw std::length_error("tp_bcast: payload larger than a slot");
    BcastRecord* r = reserve(timeout_ns);
    if (!r) return false;
    r->kind = kind;
    r->a = a;
    r->b = b;
    r->c = c;
    r->n = n;
    r->len = len;
    if (len) memcpy(payload(r), data, len);
    commit(r);
    return true;
  }

  // Reader side: the next record of reader `idx` (in publish order), or null on
  // timeout / close.  The record stays valid until release(idx).
  const BcastRecord* take(uint32_t idx, int64_t timeout_ns) {
    BcastHeader* h = hdr();
    const uint64_t next = consumed(idx).load(std::memory_order_relaxed);
    BcastRecord* r = rec((uint32_t)(next % h->n_slots));
    const int64_t deadline = timeout_ns < 0 ? INT64_MAX : now_ns() + timeout_ns;
    int spin = 0;
    for (;;) {
      const uint32_t bell = h->doorbell.load(std::memory_order_acquire);
      if (r->seq.load(std::memory_order_acquire) == next + 1) return r;
      if (closed()) return nullptr;
      if (++spin < 2000) {
        cpu_relax();
        continue;
      }
      const int64_t left = deadline - now_ns();
      if (left <= 0) return nullptr;
      futex_wait(&h->doorbell, bell, std::min<int64_t>(left, 50000000));
    }
  }
  void release(uint32_t idx) {
    BcastHeader* h = hdr();
    consumed(idx).fetch_add(1, std::memory_order_release);
    h->free_bell.fetch_add(1, std::memory_order_release);
    futex_wake_all(&h->free_bell);
  }

 private:
  std::string path() const { return "/rdb_tpb_" + name_; }
  BcastHeader* hdr() const { return reinterpret_cast<BcastHeader*>(base_); }
  std::atomic<uint64_t>& consumed(uint32_t r) const {
    return reinterpret_cast<BcastConsumed*>(base_ + sizeof(BcastHeader))[r].consumed;
  }
  BcastRecord* rec(uint32_t s) const {
    char* p = base_ + sizeof(BcastHeader) + sizeof(BcastConsumed) * kMaxReaders + hdr()->slot_bytes * s;
    return reinterpret_cast<BcastRecord*>(p);
  }
  void map(int fd, size_t sz) {
    void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("tp_bcast: mmap failed");
    base_ = reinterpret_cast<char*>(p);
    size_ = sz;
  }
  void close_map() {
    if (base_) munmap(base_, size_);
    base_ = nullptr;
    size_ = 0;
  }
  std::string name_;
  char* base_ = nullptr;
  size_t size_ = 0;
  bool created_ = false;
};

}  // namespace rt
}  // namespace rdb
