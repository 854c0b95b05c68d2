// Native host runtime of ray_dynamic_batching_amd: job segments, the
// power-of-two-choices router, clients, a native load generator and the
// request consumer used by Python replicas.  Pure C++ (no HIP) so it builds and
// runs on CPU-only hosts; the GPU replica engine lives in _rdb_ops.
//
// Parity map (reference -> here):
//   serve/_private/replica_scheduler/pow_2_scheduler.py:346-654  -> Client::choose_queue
//     (two random candidates, shortest queue below max_ongoing_requests; the
//      queue length is two relaxed atomic loads instead of a probe RPC)
//   serve/_private/router.py:116-131 (max_queued_requests back-pressure) -> submit() == -1
//   util/queue.py (RayQueue actor, 3 RPCs per request) -> shm MPSC ring push
//   293-project/src/test_scheduler.py:57-96 WorkloadGenerator, venkat-code
//     patterns, milind-code request_simulator -> LoadGen (closed loop, Poisson,
//     plus rate schedules driven from Python)
#include "shm.h"
#include "tp_bcast.h"

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <deque>
#include <map>
#include <random>
#include <thread>
#include <vector>

namespace py = pybind11;
using namespace rdb::rt;

namespace {

struct XorShift {
  uint64_t s;
  explicit XorShift(uint64_t seed) : s(seed ? seed : 0x9E3779B97F4A7C15ULL) {}
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

py::dict hist_dict(const Histogram& h) {
  py::dict d;
  const uint64_t n = h.count.load();
  d["count"] = n;
  d["mean_ms"] = n ? (double)h.sum_ns.load() / n / 1e6 : 0.0;
  d["max_ms"] = (double)h.max_ns.load() / 1e6;
  d["p50_ms"] = h.percentile(50) / 1e6;
  d["p90_ms"] = h.percentile(90) / 1e6;
  d["p95_ms"] = h.percentile(95) / 1e6;
  d["p99_ms"] = h.percentile(99) / 1e6;
  d["p999_ms"] = h.percentile(99.9) / 1e6;
  return d;
}

// ---------------------------------------------------------------------------
// JobHandle: create / attach / inspect a job segment.
// ---------------------------------------------------------------------------
class JobHandle {
 public:
  JobHandle(const std::string& name, bool create, uint32_t n_replicas, uint32_t n_queues,
            uint32_t n_clients, uint32_t req_capacity, uint32_t req_slot_bytes,
            uint32_t cmp_capacity, uint32_t cmp_slot_bytes, double attach_timeout_s, bool defer_req_rings) {
    if (create) {
      JobConfig c;
      c.defer_req_rings = defer_req_rings;
      c.n_replicas = n_replicas;
      c.n_queues = n_queues;
      c.n_clients = n_clients;
      c.req_capacity = req_capacity;
      c.req_slot_bytes = req_slot_bytes;
      c.cmp_capacity = cmp_capacity;
      c.cmp_slot_bytes = cmp_slot_bytes;
      job_.create(name, c, true);
    } else {
      job_.attach(name, (int64_t)(attach_timeout_s * 1e9));
      job_.set_unlink_on_close(false);
    }
  }
  Job& job() { return job_; }
  void close() { job_.close(); }
  void unlink_on_close(bool v) { job_.set_unlink_on_close(v); }
  int init_req_ring(uint32_t q, int numa_node) {
    check_q(q);
    return job_.init_req_ring(q, numa_node);
  }

  void configure_queue(uint32_t q, uint32_t replica, uint32_t model, uint32_t max_ongoing,
                       double slo_ms, bool active) {
    check_q(q);
    QueueState* s = job_.queue(q);
    s->replica.store(replica);
    s->model.store(model);
    s->max_ongoing.store(max_ongoing);
    s->slo_ns.store((int64_t)(slo_ms * 1e6));
    s->active.store(active ? 1 : 0, std::memory_order_release);
  }
  void set_replica_status(uint32_t r, uint32_t status, int32_t gpu, uint32_t pid) {
    check_r(r);
    ReplicaState* s = job_.replica(r);
    s->gpu.store(gpu);
    s->pid.store(pid);
    s->heartbeat_ns.store(now_ns());
    s->status.store(status, std::memory_order_release);
  }
  uint32_t replica_status(uint32_t r) { check_r(r); return job_.replica(r)->status.load(); }
  uint32_t replica_generation(uint32_t r) { check_r(r); return job_.replica(r)->restarts.load(); }
  uint32_t queue_replica(uint32_t q) { check_q(q); return job_.queue(q)->replica.load(); }
  // Replica side of multiplexing: the ids (hashes) it holds, at most kMuxSlots.
  void set_queue_models(uint32_t q, std::vector<uint64_t> ids) {
    check_q(q);
    QueueState* s = job_.queue(q);
    for (int i = 0; i < kMuxSlots; ++i)
      s->mux[i].store(i < (int)ids.size() ? ids[i] : 0, std::memory_order_release);
  }
  // Test hook (router unit tests): make queue q look `depth` deep to the
  // router without enqueuing anything (submitted = completed + depth).
  // RDB_RING_DEBUG tests: add `delta` to the sequence number of the request
  // slot `ahead` positions past queue q's consumer tail (simulates a producer
  // that published the wrong lap / a stray write into the ring).
  void test_corrupt_seq(uint32_t q, uint64_t ahead, int64_t delta) {
    check_q(q);
    Ring r = job_.req_ring(q);
    SlotHeader* s = r.slot(r.h->tail.load() + ahead);
    s->seq.fetch_add((uint64_t)delta, std::memory_order_acq_rel);
  }
  void test_set_queue_depth(uint32_t q, uint64_t depth) {
    check_q(q);
    QueueState* s = job_.queue(q);
    s->submitted.store(s->completed.load() + depth, std::memory_order_release);
  }
  std::vector<uint64_t> queue_models(uint32_t q) {
    check_q(q);
    std::vector<uint64_t> out;
    for (int i = 0; i < kMuxSlots; ++i) {
      const uint64_t v = job_.queue(q)->mux[i].load(std::memory_order_acquire);
      if (v) out.push_back(v);
    }
    return out;
  }
  void heartbeat(uint32_t r) { check_r(r); job_.replica(r)->heartbeat_ns.store(now_ns()); }
  double heartbeat_age_s(uint32_t r) {
    check_r(r);
    return (now_ns() - job_.replica(r)->heartbeat_ns.load()) / 1e9;
  }
  void bump_restarts(uint32_t r) { check_r(r); job_.replica(r)->restarts.fetch_add(1); }
  void set_shutdown(bool v) {
    job_.hdr()->shutdown.store(v ? 1 : 0);
    for (uint32_t q = 0; q < job_.hdr()->n_queues; ++q) job_.req_ring(q).ring_bell();
    for (uint32_t c = 0; c < job_.hdr()->n_clients; ++c) job_.cmp_ring(c).ring_bell();
  }
  bool shutdown() { return job_.hdr()->shutdown.load() != 0; }

  uint64_t queue_depth(uint32_t q) {
    check_q(q);
    QueueState* s = job_.queue(q);
    return s->submitted.load() - s->completed.load();
  }
  py::dict queue_stats(uint32_t q) {
    check_q(q);
    QueueState* s = job_.queue(q);
    py::dict d;
    d["active"] = s->active.load();
    d["replica"] = s->replica.load();
    d["model"] = s->model.load();
    d["max_ongoing"] = s->max_ongoing.load();
    d["submitted"] = s->submitted.load();
    d["completed"] = s->completed.load();
    d["dropped"] = s->dropped.load();
    d["errors"] = s->errors.load();
    d["slo_violations"] = s->slo_violations.load();
    d["depth"] = s->submitted.load() - s->completed.load();
    d["ring_depth"] = job_.req_ring(q).depth();
    d["queue_wait"] = hist_dict(s->hist_queue_wait);
    d["e2e"] = hist_dict(s->hist_e2e);
    return d;
  }
  py::dict replica_stats(uint32_t r) {
    check_r(r);
    ReplicaState* s = job_.replica(r);
    py::dict d;
    d["status"] = s->status.load();
    d["pid"] = s->pid.load();
    d["gpu"] = s->gpu.load();
    d["restarts"] = s->restarts.load();
    d["heartbeat_age_s"] = (now_ns() - s->heartbeat_ns.load()) / 1e9;
    d["batches"] = s->batches.load();
    d["batch_items"] = s->batch_items.load();
    d["padded_items"] = s->padded_items.load();
    d["busy_ms"] = s->busy_ns.load() / 1e6;
    d["graph_replays"] = s->graph_replays.load();
    d["batch_size"] = hist_dict(s->hist_batch_size);
    d["service"] = hist_dict(s->hist_service);
    return d;
  }
  void reset_stats() {
    for (uint32_t q = 0; q < job_.hdr()->n_queues; ++q) {
      job_.queue(q)->hist_queue_wait.reset();
      job_.queue(q)->hist_e2e.reset();
    }
    for (uint32_t r = 0; r < job_.hdr()->n_replicas; ++r) {
      job_.replica(r)->hist_batch_size.reset();
      job_.replica(r)->hist_service.reset();
    }
  }
  // Fail every request still queued for a dead replica's queue so callers
  // are not left waiting (router then re-dispatches).
  // -- seqlock snapshot (routing table / plan publication)
  uint64_t publish(py::bytes b) {
    std::string s = b;
    return job_.snapshot()->publish(s.data(), (uint32_t)s.size());
  }
  py::tuple read_snapshot() {
    std::string out;
    const uint64_t v = job_.snapshot()->read(out);
    return py::make_tuple(v, py::bytes(out));
  }
  uint64_t snapshot_version() { return job_.snapshot()->seq.load() / 2; }
  // -- trace events of one replica: list of (kind, t0_ns, t1_ns, queue, n, bucket)
  py::list trace_events(uint32_t r, uint64_t since) {
    check_r(r);
    TraceRing* tr = job_.trace(r);
    const uint64_t head = tr->head.load(std::memory_order_acquire);
    uint64_t start = head > kTraceCap ? head - kTraceCap : 0;
    start = std::max(start, since);
    py::list l;
    for (uint64_t i = start; i < head; ++i) {
      const TraceEvent& e = tr->ev[i & (kTraceCap - 1)];
      if (e.seq.load(std::memory_order_acquire) != (uint32_t)(i + 1)) continue;
      l.append(py::make_tuple(e.kind, e.t0, e.t1, e.queue, e.n, e.bucket));
    }
    return l;
  }
  uint64_t trace_head(uint32_t r) { check_r(r); return job_.trace(r)->head.load(); }
  void trace_record(uint32_t r, uint32_t kind, int64_t t0, int64_t t1, uint32_t queue, uint32_t n, uint32_t bucket) {
    check_r(r);
    job_.trace(r)->record(kind, t0, t1, queue, n, bucket);
  }
  uint64_t fail_queue(uint32_t q, uint32_t status) {
    check_q(q);
    return fail_pending(job_, q, status);
  }
  py::dict info() {
    JobHeader* h = job_.hdr();
    py::dict d;
    d["name"] = std::string(h->name);
    d["n_replicas"] = h->n_replicas;
    d["n_queues"] = h->n_queues;
    d["n_clients"] = h->n_clients;
    d["req_capacity"] = h->req_capacity;
    d["req_payload_bytes"] = h->req_slot_bytes - (uint32_t)sizeof(SlotHeader);
    d["cmp_capacity"] = h->cmp_capacity;
    d["cmp_payload_bytes"] = h->cmp_slot_bytes - (uint32_t)sizeof(SlotHeader);
    d["total_bytes"] = h->total_bytes;
    d["clients_registered"] = h->clients_registered.load();
    d["completions_dropped"] = h->cmp_dropped.load();
    py::list stalled;
    for (uint32_t c = 0; c < std::min<uint32_t>(h->n_clients, kMaxClientFlags); ++c)
      if (h->client_stalled[c].load()) stalled.append(c);
    d["stalled_clients"] = stalled;
    return d;
  }
  uintptr_t base() { return reinterpret_cast<uintptr_t>(job_.base()); }
  py::tuple request_region() {
    auto r = job_.request_region();
    return py::make_tuple(reinterpret_cast<uintptr_t>(r.first), r.second);
  }

 private:
  void check_q(uint32_t q) {
    if (q >= job_.hdr()->n_queues) throw std::out_of_range("queue index out of range");
  }
  void check_r(uint32_t r) {
    if (r >= job_.hdr()->n_replicas) throw std::out_of_range("replica index out of range");
  }
  Job job_;
};

// ---------------------------------------------------------------------------
// Client: ingress side.  Routes, submits and receives completions.
// ---------------------------------------------------------------------------
struct Completion {
  uint64_t req_id;
  uint32_t status;
  uint32_t queue;
  int64_t t_submit_ns;
  int64_t t_done_ns;
  int64_t t_recv_ns;
  uint16_t kind;
  std::string payload;
};

class Client {
 public:
  Client(JobHandle& jh, int client_id, uint64_t seed) : job_(jh.job()), rng_(seed ? seed : (uint64_t)now_ns()) {
    JobHeader* h = job_.hdr();
    if (client_id < 0) client_id = (int)h->clients_registered.fetch_add(1);
    if (client_id >= (int)h->n_clients) throw std::runtime_error("too many clients for this job");
    id_ = client_id;
    cmp_ = job_.cmp_ring(id_);
    cmp_pos_ = cmp_.h->tail.load();
  }
  int id() const { return id_; }

  // Power of two choices over the active queues serving `model`, skipping
  // queues whose replica is not READY and queues at max_ongoing.  Returns -1
  // if every candidate is saturated (the caller keeps the request queued, as
  // Serve's router does while no replica has capacity).
  // Multiplexed requests (mux != 0, the hash of the model id): among the ready
  // queues with capacity, first those whose replica holds the id, then those
  // with the fewest ids loaded (a free cache slot), then any -- each tier by
  // power-of-two choice on depth (reference pow_2_scheduler.py:396-443).
  int choose_queue(uint32_t model, uint64_t mux = 0) {
    JobHeader* h = job_.hdr();
    cand_.clear();
    int serving = 0;
    for (uint32_t q = 0; q < h->n_queues; ++q) {
      QueueState* s = job_.queue(q);
      if (!s->active.load(std::memory_order_acquire) || s->model.load() != model) continue;
      ++serving;
      const uint32_t r = s->replica.load();
      if (r < h->n_replicas && job_.replica(r)->status.load(std::memory_order_relaxed) != RS_READY) continue;
      cand_.push_back(q);
    }
    const size_t n = cand_.size();
    if (serving == 0) return -2;  // no queue serves this model at all
    if (n == 0) return -1;        // queues exist but no replica is ready (starting / restarting)
    auto depth = [&](uint32_t q) {
      QueueState* s = job_.queue(q);
      return (int64_t)(s->submitted.load(std::memory_order_relaxed) - s->completed.load(std::memory_order_relaxed));
    };
    auto ok = [&](uint32_t q, int64_t d) {
      const uint32_t m = job_.queue(q)->max_ongoing.load(std::memory_order_relaxed);
      return m == 0 || d < (int64_t)m;
    };
    if (n == 1) {
      const uint32_t q = cand_[0];
      return ok(q, depth(q)) ? (int)q : -1;
    }
    if (mux != 0) {
      auto holds = [&](uint32_t q) {
        QueueState* s = job_.queue(q);
        for (int i = 0; i < kMuxSlots; ++i)
          if (s->mux[i].load(std::memory_order_relaxed) == mux) return true;
        return false;
      };
      auto loaded = [&](uint32_t q) {
        int c = 0;
        QueueState* s = job_.queue(q);
        for (int i = 0; i < kMuxSlots; ++i) c += s->mux[i].load(std::memory_order_relaxed) != 0;
        return c;
      };
      tier_.clear();
      for (uint32_t q : cand_)
        if (holds(q) && ok(q, depth(q))) tier_.push_back(q);
      if (tier_.empty()) {
        int fewest = INT32_MAX;
        for (uint32_t q : cand_)
          if (ok(q, depth(q))) fewest = std::min(fewest, loaded(q));
        for (uint32_t q : cand_)
          if (ok(q, depth(q)) && loaded(q) == fewest) tier_.push_back(q);
      }
      if (!tier_.empty()) {
        const size_t nt = tier_.size();
        const size_t ia = rng_.next() % nt;
        const size_t ib = nt > 1 ? (ia + 1 + rng_.next() % (nt - 1)) % nt : ia;   // two distinct samples
        const uint32_t a2 = tier_[ia], b2 = tier_[ib];
        return (int)(depth(a2) <= depth(b2) ? a2 : b2);
      }
      return -1;   // every candidate at max_ongoing
    }
    // Two random distinct candidates; fall back to a full scan when both are full.
    // (the second index is uniform over the other n - 1, as random.sample in
    // the reference's pow_2_scheduler.py:346-495)
    const size_t ia = rng_.next() % n;
    const size_t ib = (ia + 1 + rng_.next() % (n - 1)) % n;
    const uint32_t a = cand_[ia], b = cand_[ib];
    const int64_t da = depth(a), db = depth(b);
    const uint32_t best = da <= db ? a : b;
    const int64_t dbest = std::min(da, db);
    if (ok(best, dbest)) return (int)best;
    int64_t bd = INT64_MAX;
    int bq = -1;
    for (uint32_t q : cand_) {
      const int64_t d = depth(q);
      if (ok(q, d) && d < bd) { bd = d; bq = (int)q; }
    }
    return bq;
  }

  // Returns the request id (>0), -1 if the ring is full, -3 if too large.
  int64_t submit_raw(uint32_t queue, const char* data, uint32_t len, uint16_t kind,
                     int64_t t_submit_ns, int64_t deadline_ns, uint64_t req_id = 0) {
    Ring ring = job_.req_ring(queue);
    if (len > ring.max_payload()) return -3;
    uint64_t pos;
    SlotHeader* s = ring.reserve(&pos);
    if (!s) return -1;
    if (req_id == 0) req_id = job_.hdr()->next_req_id.fetch_add(1, std::memory_order_relaxed);
    s->req_id = req_id;
    s->t_submit_ns = t_submit_ns ? t_submit_ns : now_ns();
    s->deadline_ns = deadline_ns;
    s->len = len;
    s->kind = kind;
    s->client = (uint16_t)id_;
    s->queue = queue;
    s->status = 0;
    s->t_aux_ns = 0;
    if (len) memcpy(ring.payload(s), data, len);
    job_.queue(queue)->submitted.fetch_add(1, std::memory_order_relaxed);
    ring.publish(s, pos);
    return (int64_t)req_id;
  }

  // Drain up to max_n completions; waits up to timeout_ns for the first one.
  template <typename F>
  size_t poll_into(size_t max_n, int64_t timeout_ns, F&& fn) {
    size_t n = 0;
    clear_client_stalled(job_, (uint32_t)id_);  // polling = alive: producers may block on us again
    if (!cmp_.peek(cmp_pos_)) {
      if (timeout_ns == 0 || !cmp_.wait_for(cmp_pos_, timeout_ns, 200)) return 0;
    }
    while (n < max_n) {
      SlotHeader* s = cmp_.peek(cmp_pos_);
      if (!s) break;
      fn(s, cmp_.payload(s));
      ++cmp_pos_;
      ++n;
      if ((n & 63) == 0) cmp_.commit(cmp_pos_);
    }
    cmp_.commit(cmp_pos_);
    return n;
  }
  Ring& cmp() { return cmp_; }
  uint64_t cmp_pos() const { return cmp_pos_; }
  Job& job() { return job_; }
  XorShift& rng() { return rng_; }

 private:
  Job& job_;
  XorShift rng_;
  int id_ = 0;
  Ring cmp_;
  uint64_t cmp_pos_ = 0;
  std::vector<uint32_t> cand_, tier_;
};

// ---------------------------------------------------------------------------
// LoadGen: native request generator (closed loop or open-loop Poisson) with
// client-side end-to-end latency histograms.  One thread does submission and
// completion draining so no locks are needed on the hot path.
// ---------------------------------------------------------------------------
class LoadGen {
 public:
  LoadGen(Client& c, uint32_t model, std::vector<std::string> payloads)
      : c_(c), model_(model), payloads_(std::move(payloads)) {
    if (payloads_.empty()) throw std::invalid_argument("LoadGen needs at least one payload");
    hist_.reset();
  }
  // Submit exactly `total` requests and wait for all of them.
  //  concurrency > 0 : closed loop with that many requests in flight
  //  rate > 0        : open-loop Poisson arrivals at `rate` req/s (latency is
  //                    measured from the scheduled arrival, so client backlog counts)
  //  deadline_ms > 0 : per-request deadline (stale-drop path)
  py::dict run(uint64_t total, int concurrency, double rate, double deadline_ms, bool record,
               double timeout_s) {
    if (record) hist_.reset();
    uint64_t issued = 0, done = 0, ok = 0, dropped = 0, errors = 0, rejected = 0;
    int64_t in_flight = 0;
    std::vector<uint64_t> per_queue(c_.job().hdr()->n_queues, 0);
    const int64_t t_start = now_ns();
    const int64_t t_limit = t_start + (int64_t)(timeout_s * 1e9);
    const int64_t dl = (int64_t)(deadline_ms * 1e6);
    double next_arrival = (double)t_start;
    uint64_t backlog = 0;  // open loop: arrivals not yet accepted by the router
    std::deque<int64_t> backlog_t;
    size_t pi = 0;
    bool timed_out = false;
    auto on_done = [&](SlotHeader* s, const char*) {
      const int64_t t = now_ns();
      ++done;
      --in_flight;
      if (s->status == ST_OK) {
        ++ok;
        if (record) hist_.record((uint64_t)(t - s->t_submit_ns));
      } else if (s->status == ST_DROPPED_STALE) {
        ++dropped;
      } else {
        ++errors;
      }
      if (s->queue < per_queue.size()) per_queue[s->queue]++;
    };
    {
      py::gil_scoped_release nogil;
      while (done < total) {
        bool progress = c_.poll_into(4096, 0, on_done) > 0;
        const int64_t now = now_ns();
        if (now > t_limit) { timed_out = true; break; }
        // arrivals
        if (rate > 0) {
          while (issued + backlog < total && next_arrival <= (double)now) {
            backlog_t.push_back((int64_t)next_arrival);
            ++backlog;
            const double u = c_.rng().uniform();
            next_arrival += -std::log(1.0 - u) / rate * 1e9;
          }
        }
        // submissions
        for (;;) {
          if (issued >= total) break;
          int64_t t_sub;
          if (rate > 0) {
            if (backlog == 0) break;
            t_sub = backlog_t.front();
          } else {
            if (in_flight >= concurrency) break;
            t_sub = now;
          }
          const int q = c_.choose_queue(model_);
          if (q < 0) { ++rejected; break; }
          const std::string& p = payloads_[pi];
          const int64_t rid = c_.submit_raw((uint32_t)q, p.data(), (uint32_t)p.size(), 0, t_sub,
                                            dl > 0 ? t_sub + dl : 0);
          if (rid == -3) throw std::runtime_error("LoadGen payload larger than the request slot");
          if (rid < 0) { ++rejected; break; }
          pi = (pi + 1) % payloads_.size();
          ++issued;
          ++in_flight;
          if (rate > 0) { backlog_t.pop_front(); --backlog; }
          progress = true;
        }
        if (!progress) {
          int64_t wait = 200000;  // 200 us
          if (rate > 0 && issued < total) {
            const int64_t until = (int64_t)next_arrival - now_ns();
            wait = std::max<int64_t>(0, std::min<int64_t>(wait, until));
          }
          if (wait > 0) c_.poll_into(4096, wait, on_done);
        }
      }
    }
    const int64_t t_end = now_ns();
    py::dict d;
    d["issued"] = issued;
    d["completed"] = done;
    d["ok"] = ok;
    d["dropped"] = dropped;
    d["errors"] = errors;
    d["router_retries"] = rejected;
    d["timed_out"] = timed_out;
    d["elapsed_s"] = (t_end - t_start) / 1e9;
    d["throughput_rps"] = done ? (double)ok / ((t_end - t_start) / 1e9) : 0.0;
    d["latency"] = hist_dict(hist_);
    d["per_queue"] = per_queue;
    return d;
  }

  // Fold another generator's recorded latencies into this one (several
  // generator threads, each with its own Client / completion ring, drive one
  // node-wide measurement: bench.py at 4+ GPUs).  Call after both runs ended.
  void merge_from(const LoadGen& o) {
    hist_.count.fetch_add(o.hist_.count.load());
    hist_.sum_ns.fetch_add(o.hist_.sum_ns.load());
    uint64_t m = hist_.max_ns.load();
    const uint64_t om = o.hist_.max_ns.load();
    if (om > m) hist_.max_ns.store(om);
    for (int i = 0; i < kHistBuckets; ++i) hist_.buckets[i].fetch_add(o.hist_.buckets[i].load());
  }
  py::dict latency() const { return hist_dict(hist_); }

  // The recorded latencies as plain numbers (bucket counts, count, sum, max) so
  // that generators living in OTHER processes can be folded in: bench.py at N
  // GPUs runs one ingress per rank and merges every rank's histogram on rank 0.
  py::tuple hist_state() const {
    std::vector<uint64_t> b(kHistBuckets);
    for (int i = 0; i < kHistBuckets; ++i) b[i] = hist_.buckets[i].load();
    return py::make_tuple(b, hist_.count.load(), hist_.sum_ns.load(), hist_.max_ns.load());
  }
  void merge_state(const std::vector<uint64_t>& b, uint64_t count, uint64_t sum_ns, uint64_t max_ns) {
    if (b.size() != (size_t)kHistBuckets) throw std::invalid_argument("histogram state of the wrong size");
    hist_.count.fetch_add(count);
    hist_.sum_ns.fetch_add(sum_ns);
    if (max_ns > hist_.max_ns.load()) hist_.max_ns.store(max_ns);
    for (int i = 0; i < kHistBuckets; ++i) hist_.buckets[i].fetch_add(b[i]);
  }

 private:
  Client& c_;
  uint32_t model_;
  std::vector<std::string> payloads_;
  Histogram hist_;
};

// ---------------------------------------------------------------------------
// Consumer: request side of a Python replica (generic @serve.batch path).
// ---------------------------------------------------------------------------
// Native fake replica: one thread per served queue pops up to `max_batch`
// requests, optionally "computes" for service_us (+ per_item_us per request),
// and completes each with the first `out_bytes` of its payload.  Used as the
// FakeReplicaWrapper-style stand-in in router tests and to measure the
// runtime's own request overhead without a GPU (bench/runtime_microbench.py).
class EchoServer {
 public:
  EchoServer(JobHandle& jh, uint32_t replica, std::vector<uint32_t> queues, uint32_t max_batch,
             double service_us, double per_item_us, uint32_t out_bytes)
      : job_(jh.job()), replica_(replica), queues_(std::move(queues)), max_batch_(max_batch),
        service_ns_((int64_t)(service_us * 1e3)), per_item_ns_((int64_t)(per_item_us * 1e3)),
        out_bytes_(out_bytes) {}
  ~EchoServer() { stop(); }
  void start() {
    if (!threads_.empty()) return;
    stop_.store(false);
    job_.replica(replica_)->status.store(RS_READY);
    for (uint32_t q : queues_) threads_.emplace_back([this, q] { serve(q); });
  }
  void stop() {
    stop_.store(true);
    for (auto& t : threads_)
      if (t.joinable()) t.join();
    threads_.clear();
  }
  uint64_t served() const { return served_.load(); }

 private:
  void serve(uint32_t q) {
    Ring r = job_.req_ring(q);
    uint64_t pos = r.h->tail.load();
    ReplicaState* rs = job_.replica(replica_);
    QueueState* qs = job_.queue(q);
    std::vector<SlotHeader*> batch;
    while (!stop_.load(std::memory_order_relaxed) && !job_.hdr()->shutdown.load()) {
      rs->heartbeat_ns.store(now_ns(), std::memory_order_relaxed);
      batch.clear();
      while (batch.size() < max_batch_) {
        SlotHeader* s = r.peek(pos + batch.size());
        if (!s) break;
        batch.push_back(s);
      }
      if (batch.empty()) {
        r.wait_for(pos, 1000000, 200);
        continue;
      }
      const int64_t t0 = now_ns();
      const int64_t work = service_ns_ + per_item_ns_ * (int64_t)batch.size();
      while (work > 0 && now_ns() - t0 < work) {}
      for (SlotHeader* s : batch) {
        Ring c = job_.cmp_ring(s->client);
        uint64_t cpos;
        SlotHeader* o = reserve_completion(job_, s->client, &cpos,
                                           [this] { return stop_.load() || job_.hdr()->shutdown.load(); });
        if (!o) {
          if (stop_.load() || job_.hdr()->shutdown.load()) return;
          qs->completed.fetch_add(1, std::memory_order_relaxed);  // stalled client: dropped
          qs->errors.fetch_add(1, std::memory_order_relaxed);
          continue;
        }
        const uint32_t n = std::min<uint32_t>({s->len, out_bytes_, c.max_payload()});
        o->req_id = s->req_id;
        o->t_submit_ns = s->t_submit_ns;
        o->deadline_ns = 0;
        o->len = n;
        o->kind = 0;
        o->client = s->client;
        o->queue = q;
        o->status = ST_OK;
        o->t_aux_ns = now_ns();
        if (n) memcpy(c.payload(o), r.payload(s), n);
        qs->completed.fetch_add(1, std::memory_order_relaxed);
        qs->hist_e2e.record((uint64_t)std::max<int64_t>(0, o->t_aux_ns - s->t_submit_ns));
        c.publish(o, cpos);
      }
      pos += batch.size();
      r.commit(pos);
      rs->batches.fetch_add(1, std::memory_order_relaxed);
      rs->batch_items.fetch_add(batch.size(), std::memory_order_relaxed);
      rs->hist_batch_size.record(batch.size());
      job_.trace(replica_)->record(TK_GPU, t0, now_ns(), q, (uint32_t)batch.size(), (uint32_t)batch.size());
      served_.fetch_add(batch.size(), std::memory_order_relaxed);
    }
  }
  Job& job_;
  uint32_t replica_;
  std::vector<uint32_t> queues_;
  uint32_t max_batch_;
  int64_t service_ns_, per_item_ns_;
  uint32_t out_bytes_;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> served_{0};
  std::vector<std::thread> threads_;
};

class Consumer {
 public:
  Consumer(JobHandle& jh, std::vector<uint32_t> queues) : job_(jh.job()), queues_(std::move(queues)) {
    for (uint32_t q : queues_) {
      rings_.push_back(job_.req_ring(q));
      pos_.push_back(job_.req_ring(q).h->tail.load());
    }
  }
  // Pop up to max_n requests from the served queues (round-robin), waiting up
  // to timeout_ns for the first.  Returns list of tuples
  // (req_id, queue, client, kind, t_submit_ns, deadline_ns, payload: bytes).
  py::list pop(size_t max_n, int64_t timeout_ns) {
    std::vector<std::tuple<uint64_t, uint32_t, uint16_t, uint16_t, int64_t, int64_t, std::string>> out;
    {
      py::gil_scoped_release nogil;
      const int64_t deadline = timeout_ns >= 0 ? now_ns() + timeout_ns : INT64_MAX;
      for (;;) {
        for (size_t i = 0; i < rings_.size() && out.size() < max_n; ++i) {
          size_t k = (rr_ + i) % rings_.size();
          Ring& r = rings_[k];
          while (out.size() < max_n) {
            SlotHeader* s = r.peek(pos_[k]);
            if (!s) break;
            out.emplace_back(s->req_id, queues_[k], s->client, s->kind, s->t_submit_ns,
                             s->deadline_ns, std::string(r.payload(s), s->len));
            ++pos_[k];
          }
          r.commit(pos_[k]);
        }
        rr_ = (rr_ + 1) % std::max<size_t>(1, rings_.size());
        if (!out.empty() || job_.hdr()->shutdown.load()) break;
        const int64_t left = deadline - now_ns();
        if (left <= 0) break;
        // sleep on the first ring's doorbell (single-queue replicas are the common case)
        rings_[0].wait_for(pos_[0], std::min<int64_t>(left, 2000000), 100);
      }
    }
    py::list l;
    for (auto& t : out)
      l.append(py::make_tuple(std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t),
                              std::get<4>(t), std::get<5>(t), py::bytes(std::get<6>(t))));
    return l;
  }
  // Move up to max_n queued requests of the served queues into queue `to`
  // (planner unload: requests that reached a GPU's queue after its model was
  // drained go to a GPU that still serves the model).  Every header field is
  // preserved, so the completion reaches the ORIGINAL client under its request
  // id; the per-queue submitted counters move with the request.  Stops early
  // when the target ring is full.  Returns the number moved.
  size_t forward(uint32_t to, size_t max_n) {
    if (to >= job_.hdr()->n_queues) throw std::out_of_range("queue index");
    py::gil_scoped_release nogil;
    Ring dst = job_.req_ring(to);
    size_t moved = 0;
    for (size_t k = 0; k < rings_.size() && moved < max_n; ++k) {
      Ring& r = rings_[k];
      if (queues_[k] == to) continue;
      while (moved < max_n) {
        SlotHeader* s = r.peek(pos_[k]);
        if (!s || s->len > dst.max_payload()) break;
        uint64_t pos;
        SlotHeader* d = dst.reserve(&pos);
        if (!d) break;
        d->req_id = s->req_id;
        d->t_submit_ns = s->t_submit_ns;
        d->deadline_ns = s->deadline_ns;
        d->len = s->len;
        d->kind = s->kind;
        d->client = s->client;
        d->queue = to;
        d->status = 0;
        d->t_aux_ns = 0;
        if (s->len) memcpy(dst.payload(d), r.payload(s), s->len);
        job_.queue(to)->submitted.fetch_add(1, std::memory_order_relaxed);
        job_.queue(queues_[k])->submitted.fetch_sub(1, std::memory_order_relaxed);
        dst.publish(d, pos);
        ++pos_[k];
        ++moved;
      }
      r.commit(pos_[k]);
    }
    return moved;
  }
  // Publish a completion. Returns false if the result does not fit.
  bool complete(uint16_t client, uint64_t req_id, uint32_t queue, uint32_t status,
                int64_t t_submit_ns, py::bytes payload, uint16_t kind) {
    std::string p = payload;
    Ring c = job_.cmp_ring(client);
    bool fits = p.size() <= c.max_payload();
    if (!fits) { status = ST_TOO_LARGE; p.clear(); }
    {
      py::gil_scoped_release nogil;
      uint64_t pos;
      SlotHeader* s = reserve_completion(job_, client, &pos, [this] { return job_.hdr()->shutdown.load() != 0; });
      if (!s) {
        if (job_.hdr()->shutdown.load()) return false;
        if (kind != 2) {  // stalled client: the terminal completion is dropped but leaves the queue
          QueueState* qs = job_.queue(queue);
          qs->completed.fetch_add(1, std::memory_order_relaxed);
          qs->errors.fetch_add(1, std::memory_order_relaxed);
        }
        return false;
      }
      s->req_id = req_id;
      s->t_submit_ns = t_submit_ns;
      s->deadline_ns = 0;
      s->len = (uint32_t)p.size();
      s->kind = kind;
      s->client = client;
      s->queue = queue;
      s->status = status;
      s->t_aux_ns = now_ns();
      if (!p.empty()) memcpy(c.payload(s), p.data(), p.size());
      QueueState* qs = job_.queue(queue);
      if (kind == 2) {  // streaming item: not a terminal completion
        c.publish(s, pos);
        return fits;
      }
      qs->completed.fetch_add(1, std::memory_order_relaxed);
      if (status == ST_DROPPED_STALE) qs->dropped.fetch_add(1, std::memory_order_relaxed);
      else if (status != ST_OK) qs->errors.fetch_add(1, std::memory_order_relaxed);
      const int64_t e2e = s->t_aux_ns - t_submit_ns;
      qs->hist_e2e.record((uint64_t)std::max<int64_t>(0, e2e));
      const int64_t slo = qs->slo_ns.load(std::memory_order_relaxed);
      if (slo > 0 && e2e > slo) qs->slo_violations.fetch_add(1, std::memory_order_relaxed);
      c.publish(s, pos);
    }
    return fits;
  }
  void record_batch(uint32_t replica, uint32_t n, double queue_wait_ms_sum, uint32_t queue) {
    ReplicaState* r = job_.replica(replica);
    r->batches.fetch_add(1);
    r->batch_items.fetch_add(n);
    r->hist_batch_size.record(n);
    (void)queue_wait_ms_sum;
    (void)queue;
  }

 private:
  Job& job_;
  std::vector<uint32_t> queues_;
  std::vector<Ring> rings_;
  std::vector<uint64_t> pos_;
  size_t rr_ = 0;
};

}  // namespace

namespace rdb {
void register_node_agent(py::module_& m);
}

PYBIND11_MODULE(_rdb_runtime, m) {
  m.doc() = "ray_dynamic_batching_amd native host runtime (shm rings, router, load generator)";
  m.attr("ST_OK") = (int)ST_OK;
  m.attr("ST_DROPPED_STALE") = (int)ST_DROPPED_STALE;
  m.attr("ST_ERROR") = (int)ST_ERROR;
  m.attr("ST_REJECTED") = (int)ST_REJECTED;
  m.attr("ST_TOO_LARGE") = (int)ST_TOO_LARGE;
  m.attr("ST_SHUTDOWN") = (int)ST_SHUTDOWN;
  m.attr("ST_REPLICA_DIED") = (int)ST_REPLICA_DIED;
  m.attr("TK_FORM") = (int)TK_FORM;
  m.attr("TK_GPU") = (int)TK_GPU;
  m.attr("TK_COMPLETE") = (int)TK_COMPLETE;
  m.attr("TK_DROP") = (int)TK_DROP;
  m.attr("TK_PY_BATCH") = (int)TK_PY_BATCH;
  m.attr("RS_UNUSED") = (int)RS_UNUSED;
  m.attr("RS_STARTING") = (int)RS_STARTING;
  m.attr("RS_READY") = (int)RS_READY;
  m.attr("RS_DRAINING") = (int)RS_DRAINING;
  m.attr("RS_DEAD") = (int)RS_DEAD;
  m.def("now_ns", &now_ns);
  m.def("ring_debug_level", &ring_debug_level, "RDB_RING_DEBUG as read by this process (0 = off)");
  m.def("ring_violations", [] {
    RingDebugState& st = ring_debug_state();
    return py::make_tuple(st.violations.load(), std::string(st.last));
  }, "(count, last message) of ring sequence violations seen by this process (RDB_RING_DEBUG >= 1)");

  py::class_<JobHandle>(m, "Job")
      .def(py::init<const std::string&, bool, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                    uint32_t, uint32_t, double, bool>(),
           py::arg("name"), py::arg("create") = false, py::arg("n_replicas") = 1,
           py::arg("n_queues") = 1, py::arg("n_clients") = 8, py::arg("req_capacity") = 4096,
           py::arg("req_slot_bytes") = 1024, py::arg("cmp_capacity") = 8192,
           py::arg("cmp_slot_bytes") = 256, py::arg("attach_timeout_s") = 30.0,
           py::arg("defer_req_rings") = false)
      .def("init_req_ring", &JobHandle::init_req_ring, py::arg("queue"), py::arg("numa_node") = -1,
           "consumer-side init of a deferred request ring, its pages bound to numa_node first")
      .def("close", &JobHandle::close)
      .def("unlink_on_close", &JobHandle::unlink_on_close)
      .def("configure_queue", &JobHandle::configure_queue, py::arg("queue"), py::arg("replica"),
           py::arg("model"), py::arg("max_ongoing"), py::arg("slo_ms") = 0.0, py::arg("active") = true)
      .def("set_replica_status", &JobHandle::set_replica_status, py::arg("replica"),
           py::arg("status"), py::arg("gpu") = -1, py::arg("pid") = 0)
      .def("replica_status", &JobHandle::replica_status)
      .def("replica_generation", &JobHandle::replica_generation)
      .def("queue_replica", &JobHandle::queue_replica)
      .def("set_queue_models", &JobHandle::set_queue_models)
      .def("_test_set_queue_depth", &JobHandle::test_set_queue_depth)
      .def("_test_corrupt_seq", &JobHandle::test_corrupt_seq, py::arg("queue"), py::arg("ahead"), py::arg("delta"))
      .def("queue_models", &JobHandle::queue_models)
      .def("heartbeat", &JobHandle::heartbeat)
      .def("heartbeat_age_s", &JobHandle::heartbeat_age_s)
      .def("bump_restarts", &JobHandle::bump_restarts)
      .def("set_shutdown", &JobHandle::set_shutdown)
      .def("shutdown", &JobHandle::shutdown)
      .def("queue_depth", &JobHandle::queue_depth)
      .def("queue_stats", &JobHandle::queue_stats)
      .def("replica_stats", &JobHandle::replica_stats)
      .def("reset_stats", &JobHandle::reset_stats)
      .def("fail_queue", &JobHandle::fail_queue)
      .def("publish", &JobHandle::publish)
      .def("read_snapshot", &JobHandle::read_snapshot)
      .def("snapshot_version", &JobHandle::snapshot_version)
      .def("trace_events", &JobHandle::trace_events, py::arg("replica"), py::arg("since") = 0)
      .def("trace_head", &JobHandle::trace_head)
      .def("trace_record", &JobHandle::trace_record)
      .def("info", &JobHandle::info)
      .def("base", &JobHandle::base)
      .def("request_region", &JobHandle::request_region);

  py::class_<EchoServer>(m, "EchoServer")
      .def(py::init<JobHandle&, uint32_t, std::vector<uint32_t>, uint32_t, double, double, uint32_t>(),
           py::arg("job"), py::arg("replica"), py::arg("queues"), py::arg("max_batch") = 32,
           py::arg("service_us") = 0.0, py::arg("per_item_us") = 0.0, py::arg("out_bytes") = 8,
           py::keep_alive<1, 2>())
      .def("start", &EchoServer::start)
      .def("stop", &EchoServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("served", &EchoServer::served);

  py::class_<Client>(m, "Client")
      .def(py::init<JobHandle&, int, uint64_t>(), py::arg("job"), py::arg("client_id") = -1,
           py::arg("seed") = 0, py::keep_alive<1, 2>())
      .def_property_readonly("id", &Client::id)
      .def("choose_queue", &Client::choose_queue, py::arg("model"), py::arg("mux") = 0)
      .def("submit",
           [](Client& c, uint32_t queue, py::bytes data, uint16_t kind, double deadline_s, uint64_t req_id) {
             char* buf;
             Py_ssize_t len;
             PyBytes_AsStringAndSize(data.ptr(), &buf, &len);
             const int64_t t = now_ns();
             const int64_t dl = deadline_s > 0 ? t + (int64_t)(deadline_s * 1e9) : 0;
             return c.submit_raw(queue, buf, (uint32_t)len, kind, t, dl, req_id);
           },
           py::arg("queue"), py::arg("data"), py::arg("kind") = 0, py::arg("deadline_s") = 0.0,
           py::arg("req_id") = 0)
      .def("submit_buffer",
           [](Client& c, uint32_t queue, py::buffer data, uint16_t kind, double deadline_s, uint64_t req_id) {
             py::buffer_info bi = data.request();
             const int64_t t = now_ns();
             const int64_t dl = deadline_s > 0 ? t + (int64_t)(deadline_s * 1e9) : 0;
             return c.submit_raw(queue, static_cast<const char*>(bi.ptr),
                                 (uint32_t)(bi.size * bi.itemsize), kind, t, dl, req_id);
           },
           py::arg("queue"), py::arg("data"), py::arg("kind") = 0, py::arg("deadline_s") = 0.0,
           py::arg("req_id") = 0)
      .def("poll",
           [](Client& c, size_t max_n, double timeout_s) {
             std::vector<Completion> v;
             {
               py::gil_scoped_release nogil;
               c.poll_into(max_n, (int64_t)(timeout_s * 1e9), [&](SlotHeader* s, const char* p) {
                 v.push_back(Completion{s->req_id, s->status, s->queue, s->t_submit_ns, s->t_aux_ns,
                                        now_ns(), s->kind, std::string(p, s->len)});
               });
             }
             py::list l;
             for (auto& x : v)
               l.append(py::make_tuple(x.req_id, x.status, x.queue, x.t_submit_ns, x.t_done_ns,
                                       x.t_recv_ns, x.kind, py::bytes(x.payload)));
             return l;
           },
           py::arg("max_n") = 1024, py::arg("timeout_s") = 0.01);

  py::class_<LoadGen>(m, "LoadGen")
      .def(py::init<Client&, uint32_t, std::vector<std::string>>(), py::keep_alive<1, 2>())
      .def("run", &LoadGen::run, py::arg("total"), py::arg("concurrency") = 64,
           py::arg("rate") = 0.0, py::arg("deadline_ms") = 0.0, py::arg("record") = true,
           py::arg("timeout_s") = 600.0)
      .def("merge_from", &LoadGen::merge_from)
      .def("hist_state", &LoadGen::hist_state)
      .def("merge_state", &LoadGen::merge_state, py::arg("buckets"), py::arg("count"), py::arg("sum_ns"),
           py::arg("max_ns"))
      .def("latency", &LoadGen::latency);

  // TP batch broadcast (tp_bcast.h): the Python TP serving loop's rank-0 ->
  // follower hand-off (the GPU path uses the same ring from the native engine)
  py::class_<TPBcast>(m, "TPBcast")
      .def(py::init([](const std::string& name, bool create, uint32_t n_readers, uint32_t n_slots,
                       uint64_t payload_bytes, double attach_timeout_s) {
             auto b = std::make_unique<TPBcast>();
             if (create) {
               b->create(name, n_readers, n_slots, payload_bytes);
             } else {
               py::gil_scoped_release nogil;
               b->attach(name, (int64_t)(attach_timeout_s * 1e9));
             }
             return b;
           }),
           py::arg("name"), py::arg("create"), py::arg("n_readers") = 0, py::arg("n_slots") = 8,
           py::arg("payload_bytes") = 65536, py::arg("attach_timeout_s") = 60.0)
      .def("publish",
           [](TPBcast& b, int kind, int a, int bb, int c, uint32_t n, py::bytes payload, double timeout_s) {
             std::string d = payload;
             py::gil_scoped_release nogil;
             return b.publish(kind, a, bb, c, n, d.data(), (uint32_t)d.size(),
                              timeout_s < 0 ? -1 : (int64_t)(timeout_s * 1e9));
           },
           py::arg("kind"), py::arg("a"), py::arg("b"), py::arg("c"), py::arg("n"), py::arg("payload"),
           py::arg("timeout_s") = -1.0)
      .def("take",
           [](TPBcast& b, uint32_t reader, double timeout_s) -> py::object {
             if (reader >= b.n_readers()) throw std::out_of_range("tp_bcast: reader index");
             const BcastRecord* r;
             {
               py::gil_scoped_release nogil;
               r = b.take(reader, timeout_s < 0 ? -1 : (int64_t)(timeout_s * 1e9));
             }
             if (!r) return py::none();
             py::tuple t = py::make_tuple(r->kind, r->a, r->b, r->c, r->n,
                                          py::bytes(reinterpret_cast<const char*>(r) + sizeof(BcastRecord), r->len));
             b.release(reader);
             return t;
           },
           py::arg("reader"), py::arg("timeout_s") = -1.0)
      .def("close", &TPBcast::close)
      .def("closed", &TPBcast::closed)
      .def("unlink", &TPBcast::unlink)
      .def("head", &TPBcast::head)
      .def_property_readonly("payload_capacity", &TPBcast::payload_capacity)
      .def_property_readonly("n_readers", &TPBcast::n_readers);

  py::class_<Consumer>(m, "Consumer")
      .def(py::init<JobHandle&, std::vector<uint32_t>>(), py::keep_alive<1, 2>())
      .def("pop", &Consumer::pop, py::arg("max_n") = 64, py::arg("timeout_ns") = 10000000)
      .def("complete", &Consumer::complete, py::arg("client"), py::arg("req_id"), py::arg("queue"),
           py::arg("status"), py::arg("t_submit_ns"), py::arg("payload"), py::arg("kind") = 0)
      .def("record_batch", &Consumer::record_batch)
      .def("forward", &Consumer::forward, py::arg("to"), py::arg("max_n") = 1 << 20);
  rdb::register_node_agent(m);
}
