// Replica engine: the native dynamic-batching loop of one GPU replica.
//
// Reference behaviour being re-designed:
//   * serve/batching.py:146-197 _BatchQueue.wait_for_batch -- flush at
//     max_batch_size or batch_wait_timeout_s after the FIRST item;
//   * 293-project/src/scheduler.py:258-322 RequestQueue.get_batch -- per-model
//     queues with stale-request dropping (arrival + SLO < now + lat(b));
//   * scheduler.py:525-588 GPUWorker.execute_schedule -- one worker per GPU
//     serving several model sessions;
//   * scheduler.py:443-452 -- stack + .cuda() + synchronize around the forward.
//
// MI355X-native design:
//   launcher thread : picks the session (model queue) with the earliest head
//                     deadline (priority first), forms a batch by PEEKING the
//                     shm ring, launches on the copy stream a gather kernel that
//                     reads the payloads in place from hipHostRegister'ed shm
//                     (zero-copy H2D, padded to the bucket), then on the compute
//                     stream waits that event and replays the hipGraph captured
//                     for (session, bucket, slot), then async D2H of the outputs
//                     into pinned host memory.  `pipeline_depth` slots let the
//                     gather of batch k+1 overlap the forward of batch k.
//   completer thread: waits the batch events in FIFO order, writes the per-request
//                     results into the clients' completion rings, releases the
//                     request-ring slots and updates shm metrics.
// No Python runs in steady state.
//
// Tensor-parallel replicas (one Engine per rank process, compute_streams = 1):
//   leader (rank 0) : the loop above; after forming a batch it publishes
//                     (session, bucket, slot, n) + the n request rows to the
//                     group's broadcast ring (runtime/csrc/tp_bcast.h) before
//                     launching, then completes the requests as usual;
//   follower        : its launcher takes the records in order, copies the rows
//                     into a pinned staging slot, H2D on the copy stream, replays
//                     the SAME (session, bucket, slot) graph -- its RCCL / xGMI
//                     all-reduces pair up with the other ranks' because every
//                     rank launches the same graphs in the same order -- and its
//                     completer only retires the slot (no requests, no replica
//                     state: the group's replica slot belongs to rank 0).
//   Batch k+1 is formed, broadcast and copied while batch k computes on every rank.
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <memory>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "../../runtime/csrc/shm.h"
#include "../../runtime/csrc/tp_bcast.h"

namespace py = pybind11;
using namespace rdb::rt;

namespace rdb {
void gather_rows(uintptr_t src_ptrs, int n, int rows, int row_bytes, uintptr_t dst, uintptr_t stream);

namespace {

#define ENG_CHECK(expr)                                                                     \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("engine HIP error: ") + hipGetErrorString(_e) + \
                               " at " #expr);                                               \
  } while (0)

struct Session {
  uint32_t queue = 0;
  int max_batch = 1;
  int64_t max_wait_ns = 0;
  std::vector<int> buckets;
  int in_row_bytes = 0, out_row_bytes = 0;
  int priority = 0;
  int64_t slo_ns = 0;
  bool drop_stale = false;
  // per-bucket service estimates, written by the completer thread and read by
  // the launcher: est_ns is the GPU time of a batch that ran ALONE (seeded by
  // the latency replays, refined only by batches that overlapped no other
  // batch) and drives duty-cycle charging / backfill; est_wall_ns is the EMA of
  // the event-timed span under whatever overlap the compute streams had and
  // drives stale dropping (when a request would actually complete)
  // est_prov: the solo estimate is only a seed (timed while other sessions
  // were running, or from a first batch that overlapped another): the first
  // batch that truly runs alone REPLACES it instead of being blended in
  std::unique_ptr<std::atomic<double>[]> est_ns, est_wall_ns;
  std::unique_ptr<std::atomic<bool>[]> est_prov;
  size_t n_est = 0;
  void reset_estimates(size_t n) {
    n_est = n;
    est_ns.reset(new std::atomic<double>[n]);
    est_wall_ns.reset(new std::atomic<double>[n]);
    est_prov.reset(new std::atomic<bool>[n]);
    for (size_t i = 0; i < n; ++i) {
      est_ns[i].store(0.0, std::memory_order_relaxed);
      est_wall_ns[i].store(0.0, std::memory_order_relaxed);
      est_prov[i].store(true, std::memory_order_relaxed);
    }
  }
  double est(int bi) const { return est_ns[bi].load(std::memory_order_relaxed); }
  double est_wall(int bi) const {
    const double w = est_wall_ns[bi].load(std::memory_order_relaxed);
    return w > 0.0 ? w : est(bi);
  }
  std::vector<std::vector<hipGraphExec_t>> graphs;   // [bucket][slot]
  std::vector<std::vector<uintptr_t>> out_dev;       // [bucket][slot]
  std::vector<uintptr_t> in_dev;                     // [slot]
  std::vector<void*> host_tbl, host_out;             // [slot] pinned gather table / output staging
  Ring ring;
  uint64_t peek_pos = 0;                             // next unread position
  // duty-cycle mode (Nexus): GPU time this session may use per cycle
  int64_t duty_share_ns = 0;
  int64_t used_ns = 0;                               // charged in the current cycle
  uint64_t launched_cycle = UINT64_MAX;              // duty-cycle index of the last launch
  std::atomic<bool> active{true};                    // model loaded / unloaded by the planner
  // live load / unload (planner re-placement): batches of this session between
  // the launcher's pick and their completion; retire() waits for 0
  std::atomic<int> inflight{0};
  std::atomic<bool> retired{false};
};

enum Policy { POLICY_PRIORITY_EDF = 0, POLICY_DUTY_CYCLE = 1 };

// process-wide refcount of pinned (hipHostRegister'ed) job request regions
std::mutex& host_reg_mu() {
  static std::mutex m;
  return m;
}
std::map<void*, int>& host_reg_count() {
  static std::map<void*, int> c;
  return c;
}

struct InFlight {
  int session = -1;
  int slot = 0;
  int bucket_idx = 0;
  uint64_t pos_begin = 0, pos_end = 0;  // ring range covered (committed after completion)
  std::vector<uint64_t> req_pos;        // ring positions of the requests in batch order
  int64_t t_form_start = 0, t_launch = 0;
  bool gpu = false;
  bool solo = false;     // no other GPU batch in flight when this one launched
  uint64_t seq = 0;      // launch sequence number (launch_seq_ after this launch)
  int tp_n = 0;          // TP follower: requests in the leader's batch (stats only)
};

class Engine {
 public:
  Engine(const std::string& job_name, uint32_t replica, int pipeline_depth, bool zero_copy,
         int device, int policy, int compute_streams)
      : replica_(replica), depth_(std::max(1, pipeline_depth)), zero_copy_(zero_copy),
        device_(device), policy_(policy) {
    if (policy != POLICY_PRIORITY_EDF && policy != POLICY_DUTY_CYCLE)
      throw std::invalid_argument("policy must be 0 (priority/EDF) or 1 (duty cycle)");
    const int ns = std::max(1, std::min(compute_streams, depth_));
    job_.attach(job_name, 30000000000LL);
    job_.set_unlink_on_close(false);
    if (replica_ >= job_.hdr()->n_replicas) throw std::out_of_range("replica index");
    ENG_CHECK(hipSetDevice(device_));
    ENG_CHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
    for (int i = 0; i < ns; ++i) {
      hipStream_t st;
      ENG_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      compute_streams_.push_back(st);
    }
    if (zero_copy_) {
      auto reg = job_.request_region();
      host_base_ = reg.first;
      // Portable: several engines (one per GPU) may live in one process (the
      // SLO scheduler); only the first registers, the others reuse the mapping.
      {
        std::lock_guard<std::mutex> lk(host_reg_mu());
        int& rc = host_reg_count()[reg.first];
        if (rc == 0)
          ENG_CHECK(hipHostRegister(reg.first, reg.second, hipHostRegisterMapped | hipHostRegisterPortable));
        ++rc;
        registered_ = true;
      }
      void* dev = nullptr;
      ENG_CHECK(hipHostGetDevicePointer(&dev, reg.first, 0));
      dev_base_ = reinterpret_cast<char*>(dev);
    }
    slot_busy_.assign(depth_, false);
    // fault-injection knobs (same variables as utils/faults.py)
    auto knob = [](const char* n) { const char* v = getenv(n); return v ? atoll(v) : 0LL; };
    fault_drop_every_ = knob("RDB_FAULT_DROP_EVERY");
    fault_delay_batch_us_ = knob("RDB_FAULT_DELAY_BATCH_US");
    fault_kill_after_ = knob("RDB_FAULT_KILL_AFTER_BATCHES");
    idle_dispatch_.store(knob("RDB_IDLE_DISPATCH") != 0);
    // RDB_ENGINE_STAGGER_US (opt-in, A/B knob): when a batch is about to start on an
    // idle compute stream less than this long after another stream started from idle,
    // hold it back to that offset -- two streams that start together stay in lockstep
    // (same kernel types at the same time: profiles/stamp_timeline_r5.json), staggered
    // ones pair different kernels
    stagger_ns_ = knob("RDB_ENGINE_STAGGER_US") * 1000;
    // On the registered ring a batch's rows move with strided hipMemcpy2DAsync
    // (one per run of consecutive ring slots) instead of the gather_rows kernel,
    // so the H2D copy holds no CU: ResNet-50 closed loop 51.2k vs 49.1k img/s
    // (profiles/engine_input_copy_r6.json).  RDB_ENGINE_DMA_GATHER=0 keeps the kernel.
    {
      const char* v = getenv("RDB_ENGINE_DMA_GATHER");
      dma_gather_ = zero_copy_ && (v == nullptr || atoi(v) != 0);
    }
    stream_running_.reset(new std::atomic<int>[compute_streams_.size()]);
    for (size_t i = 0; i < compute_streams_.size(); ++i) stream_running_[i].store(0);
    for (int s = 0; s < depth_; ++s) {
      hipEvent_t a, b, c;
      ENG_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
      ENG_CHECK(hipEventCreate(&b));
      ENG_CHECK(hipEventCreate(&c));
      ev_copy_.push_back(a);
      ev_start_.push_back(b);
      ev_done_.push_back(c);
    }
  }
  ~Engine() {
    stop();
    for (auto p : tp_stage_) hipHostFree(p);
    for (auto e : ev_copy_) hipEventDestroy(e);
    for (auto e : ev_start_) hipEventDestroy(e);
    for (auto e : ev_done_) hipEventDestroy(e);
    for (auto& sp : owned_) free_host(*sp);
    if (registered_) {
      std::lock_guard<std::mutex> lk(host_reg_mu());
      void* base = job_.request_region().first;
      if (--host_reg_count()[base] == 0) {
        hipHostUnregister(base);
        host_reg_count().erase(base);
      }
    }
    if (copy_stream_) hipStreamDestroy(copy_stream_);
    for (auto st : compute_streams_) hipStreamDestroy(st);
  }

  // Sessions may be added while the engine runs (planner load of a model at a
  // batch boundary): a live-added session starts INACTIVE; the caller sets its
  // inputs / graphs and then activates it.  A retired slot (retire_session) is
  // reused; its old Session object stays allocated until the engine is destroyed
  // (the launcher may still be reading its `active` flag), only its pinned
  // buffers are freed at retirement.
  int add_session(uint32_t queue, int max_batch, double max_wait_s, std::vector<int> buckets,
                  int in_row_bytes, int out_row_bytes, int priority, double slo_ms, bool drop_stale) {
    if (queue >= job_.hdr()->n_queues) throw std::out_of_range("queue index");
    if (buckets.empty()) buckets.push_back(max_batch);
    std::sort(buckets.begin(), buckets.end());
    if (buckets.back() != max_batch) throw std::invalid_argument("largest bucket must equal max_batch");
    if (in_row_bytes % 16) throw std::invalid_argument("in_row_bytes must be a multiple of 16");
    Ring ring = job_.req_ring(queue);
    if ((uint32_t)in_row_bytes > ring.max_payload()) throw std::invalid_argument("request slot too small");
    std::lock_guard<std::mutex> api(api_mu_);
    const int n = n_sess_.load();
    for (int i = 0; i < n; ++i) {
      Session* o = sess_ptr_[i].load();
      if (o->retired.load() && o->queue == queue) throw std::invalid_argument("queue already has a retired session; reuse it");
      if (!o->retired.load() && o->queue == queue) throw std::invalid_argument("queue already served by a session");
    }
    auto sp = std::make_unique<Session>();
    Session& s = *sp;
    s.queue = queue;
    s.max_batch = max_batch;
    s.max_wait_ns = (int64_t)(max_wait_s * 1e9);
    s.buckets = buckets;
    s.in_row_bytes = in_row_bytes;
    s.out_row_bytes = out_row_bytes;
    s.priority = priority;
    s.slo_ns = (int64_t)(slo_ms * 1e6);
    s.drop_stale = drop_stale;
    s.reset_estimates(buckets.size());
    s.graphs.assign(buckets.size(), std::vector<hipGraphExec_t>(depth_, nullptr));
    s.out_dev.assign(buckets.size(), std::vector<uintptr_t>(depth_, 0));
    s.in_dev.assign(depth_, 0);
    s.ring = ring;
    s.peek_pos = ring.h->tail.load();
    s.active.store(!running_.load());
    // per-slot pinned gather tables and output staging
    for (int sl = 0; sl < depth_; ++sl) {
      void* p = nullptr;
      ENG_CHECK(hipHostMalloc(&p, sizeof(uint64_t) * max_batch, hipHostMallocDefault));
      s.host_tbl.push_back(p);
      void* o = nullptr;
      ENG_CHECK(hipHostMalloc(&o, (size_t)out_row_bytes * max_batch + 64, hipHostMallocDefault));
      s.host_out.push_back(o);
    }
    if (n >= kMaxSessions) {
      free_host(s);
      throw std::runtime_error("engine: too many sessions");
    }
    sess_ptr_[n].store(sp.get(), std::memory_order_release);
    owned_.push_back(std::move(sp));
    n_sess_.store(n + 1, std::memory_order_release);
    return n;
  }
  // Re-arm a retired session for the same queue with new graphs (a model moved
  // back onto this GPU): returns its sid, inactive until set_session_active.
  int readd_session(uint32_t queue, int max_batch, double max_wait_s, std::vector<int> buckets, int in_row_bytes,
                    int out_row_bytes, int priority, double slo_ms, bool drop_stale) {
    int old = -1;
    {
      std::lock_guard<std::mutex> api(api_mu_);
      for (int i = 0; i < n_sess_.load(); ++i)
        if (sess_ptr_[i].load()->queue == queue && sess_ptr_[i].load()->retired.load()) old = i;
    }
    if (old < 0) return add_session(queue, max_batch, max_wait_s, buckets, in_row_bytes, out_row_bytes, priority,
                                    slo_ms, drop_stale);
    if (buckets.empty()) buckets.push_back(max_batch);
    std::sort(buckets.begin(), buckets.end());
    if (buckets.back() != max_batch) throw std::invalid_argument("largest bucket must equal max_batch");
    auto sp = std::make_unique<Session>();
    Session& s = *sp;
    s.queue = queue;
    s.max_batch = max_batch;
    s.max_wait_ns = (int64_t)(max_wait_s * 1e9);
    s.buckets = buckets;
    s.in_row_bytes = in_row_bytes;
    s.out_row_bytes = out_row_bytes;
    s.priority = priority;
    s.slo_ns = (int64_t)(slo_ms * 1e6);
    s.drop_stale = drop_stale;
    s.reset_estimates(buckets.size());
    s.graphs.assign(buckets.size(), std::vector<hipGraphExec_t>(depth_, nullptr));
    s.out_dev.assign(buckets.size(), std::vector<uintptr_t>(depth_, 0));
    s.in_dev.assign(depth_, 0);
    s.ring = job_.req_ring(queue);
    s.peek_pos = s.ring.h->tail.load();
    s.active.store(false);
    for (int sl = 0; sl < depth_; ++sl) {
      void* p = nullptr;
      ENG_CHECK(hipHostMalloc(&p, sizeof(uint64_t) * max_batch, hipHostMallocDefault));
      s.host_tbl.push_back(p);
      void* o = nullptr;
      ENG_CHECK(hipHostMalloc(&o, (size_t)out_row_bytes * max_batch + 64, hipHostMallocDefault));
      s.host_out.push_back(o);
    }
    std::lock_guard<std::mutex> api(api_mu_);
    sess_ptr_[old].store(sp.get(), std::memory_order_release);   // the retired object stays owned
    owned_.push_back(std::move(sp));
    return old;
  }
  // Unload: stop picking the session, wait (bounded) until none of its batches
  // is in flight, then drop its graph handles -- after this the caller may free
  // the graphs, inputs and weights.  Requests still queued stay in the ring.
  bool retire_session(int sid, double timeout_s) {
    Session& s = sess(sid);
    const bool was_active = s.active.exchange(false, std::memory_order_seq_cst);
    const int64_t end = now_ns() + (int64_t)(timeout_s * 1e9);
    while (s.inflight.load(std::memory_order_seq_cst) != 0) {
      if (now_ns() > end) {
        s.active.store(was_active);   // could not drain: back to how it was (serving only if it was)
        return false;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    for (auto& row : s.graphs)
      for (auto& g : row) g = nullptr;
    for (auto& x : s.in_dev) x = 0;
    s.retired.store(true);
    free_host(s);
    return true;
  }
  int session_inflight(int sid) { return sess(sid).inflight.load(); }
  uint64_t session_pending(int sid) { return sess(sid).ring.depth(); }
  bool session_retired(int sid) { return sess(sid).retired.load(); }
  int num_sessions() const { return n_sess_.load(); }
  void set_input(int sid, int slot, uintptr_t dev_ptr) { sess(sid).in_dev.at(slot) = dev_ptr; }
  void set_graph(int sid, int bucket_idx, int slot, uintptr_t graph_exec, uintptr_t out_dev) {
    Session& s = sess(sid);
    s.graphs.at(bucket_idx).at(slot) = reinterpret_cast<hipGraphExec_t>(graph_exec);
    s.out_dev.at(bucket_idx).at(slot) = out_dev;
  }
  void set_latency_estimate(int sid, int bucket_idx, double ms, bool provisional) {
    Session& s = sess(sid);
    if (bucket_idx < 0 || (size_t)bucket_idx >= s.n_est) throw std::out_of_range("bucket index");
    s.est_ns[bucket_idx].store(ms * 1e6, std::memory_order_relaxed);
    s.est_prov[bucket_idx].store(provisional, std::memory_order_relaxed);
  }
  bool latency_estimate_provisional(int sid, int bucket_idx) {
    Session& s = sess(sid);
    if (bucket_idx < 0 || (size_t)bucket_idx >= s.n_est) throw std::out_of_range("bucket index");
    return s.est_prov[bucket_idx].load(std::memory_order_relaxed);
  }
  // (solo, wall) service estimates of one bucket in ms
  std::pair<double, double> latency_estimate(int sid, int bucket_idx) {
    Session& s = sess(sid);
    if (bucket_idx < 0 || (size_t)bucket_idx >= s.n_est) throw std::out_of_range("bucket index");
    return {s.est(bucket_idx) / 1e6, s.est_wall(bucket_idx) / 1e6};
  }
  // Nexus duty cycle (policy 1): every `cycle_ms` each session may use `share_ms`
  // of GPU time (= occupancy x duty cycle); budgets reset at the cycle boundary.
  void set_duty_share(int sid, double ms) { sess(sid).duty_share_ns = (int64_t)(ms * 1e6); }
  void set_duty_cycle(double ms) { duty_cycle_ns_.store((int64_t)(ms * 1e6)); }
  void set_session_active(int sid, bool on) {
    Session& s = sess(sid);
    if (on) {
      if (s.retired.load()) throw std::runtime_error("session is retired (readd_session first)");
      for (size_t b = 0; b < s.buckets.size(); ++b)
        for (int sl = 0; sl < depth_; ++sl)
          if (!s.graphs[b][sl] || !s.in_dev[sl])
            throw std::runtime_error("engine: activating a session with a missing graph/input");
    }
    s.active.store(on, std::memory_order_seq_cst);
  }
  int compute_streams() const { return (int)compute_streams_.size(); }
  void set_idle_dispatch(bool on) { idle_dispatch_.store(on, std::memory_order_relaxed); }
  // EngineConfig.stagger_us (the RDB_ENGINE_STAGGER_US knob, set before start())
  void set_stagger_us(int64_t us) { stagger_ns_ = std::max<int64_t>(0, us) * 1000; }
  int64_t stagger_us() const { return stagger_ns_ / 1000; }
  bool idle_dispatch() const { return idle_dispatch_.load(std::memory_order_relaxed); }
  void set_max_batch(int sid, int b) {
    Session& s = sess(sid);
    if (b < 1 || b > s.buckets.back()) throw std::invalid_argument("max_batch out of range");
    s.max_batch = b;
  }
  void set_max_wait(int sid, double seconds) { sess(sid).max_wait_ns = (int64_t)(seconds * 1e9); }

  void start() {
    if (running_) return;
    for (int i = 0; i < n_sess_.load(); ++i) {
      Session& s = *sess_ptr_[i].load();
      if (s.retired.load()) continue;
      for (size_t b = 0; b < s.buckets.size(); ++b)
        for (int sl = 0; sl < depth_; ++sl)
          if (!s.graphs[b][sl] || !s.in_dev[sl])
            throw std::runtime_error("engine: missing graph/input for a (session, bucket, slot)");
    }
    running_ = true;
    if (tp_role_ != TP_FOLLOWER) {   // a follower never touches the group's replica slot (rank 0 owns it)
      ReplicaState* rs = job_.replica(replica_);
      rs->gpu.store(device_);
      rs->pid.store((uint32_t)getpid());
      rs->heartbeat_ns.store(now_ns());
      rs->status.store(RS_READY, std::memory_order_release);
    }
    completer_ = std::thread([this] { completer_loop(); });
    if (tp_role_ == TP_FOLLOWER) launcher_ = std::thread([this] { follower_loop(); });
    else launcher_ = std::thread([this] { launcher_loop(); });
  }
  void stop() {
    // The threads may have ended on their own (a launcher error, a TP follower
    // after the leader's STOP) with running_ already false: they are still
    // joined here -- a joinable std::thread reaching ~Engine would terminate().
    const bool was_running = running_.exchange(false);
    if (!was_running && !launcher_.joinable() && !completer_.joinable()) return;
    for (int i = 0; i < n_sess_.load(); ++i) sess_ptr_[i].load()->ring.ring_bell();
    cv_.notify_all();
    if (launcher_.joinable()) launcher_.join();   // a TP launcher re-checks running_ every 50 ms on the ring
    if (bcast_ && !bcast_->closed()) {
      // leader (the ring's only writer, its launcher has exited): a STOP record
      // for the followers (bounded wait), then close -- which also wakes anyone
      // still blocked on the ring; a follower closing tells the leader the group broke
      if (tp_role_ == TP_LEADER) bcast_->publish(BCAST_STOP, 0, 0, 0, 0, nullptr, 0, 200000000LL);
      bcast_->close();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      stopping_completer_ = true;
    }
    cv_.notify_all();
    if (completer_.joinable()) completer_.join();
    if (tp_role_ != TP_FOLLOWER) job_.replica(replica_)->status.store(RS_DRAINING);
  }

  // ---- tensor-parallel roles (see the header comment); set after the sessions
  // and graphs are registered, before start() ----
  // Leader: create the group's broadcast ring for `n_followers` readers; a slot
  // holds one batch of the largest session's rows.
  void set_tp_leader(const std::string& name, int n_followers, int n_slots) {
    if (running_) throw std::runtime_error("set_tp_leader: engine already running");
    if (compute_streams_.size() != 1) throw std::invalid_argument("a TP engine runs ONE compute stream (graph order)");
    size_t cap = 0;
    for (int i = 0; i < n_sess_.load(); ++i) {
      Session& ss = *sess_ptr_[i].load();
      cap = std::max(cap, (size_t)ss.max_batch * (size_t)ss.in_row_bytes);
    }
    bcast_.reset(new TPBcast());
    bcast_->create(name, (uint32_t)n_followers, (uint32_t)std::max(2, n_slots), cap);
    tp_role_ = TP_LEADER;
  }
  // Follower `reader` (rank - 1): attach to the leader's ring, allocate the
  // pinned staging slots the records are copied into.
  void set_tp_follower(const std::string& name, int reader, double attach_timeout_s) {
    if (running_) throw std::runtime_error("set_tp_follower: engine already running");
    if (compute_streams_.size() != 1) throw std::invalid_argument("a TP engine runs ONE compute stream (graph order)");
    bcast_.reset(new TPBcast());
    {
      py::gil_scoped_release nogil;
      bcast_->attach(name, (int64_t)(attach_timeout_s * 1e9));
    }
    if (reader < 0 || (uint32_t)reader >= bcast_->n_readers()) throw std::out_of_range("tp follower reader index");
    tp_reader_ = (uint32_t)reader;
    const size_t cap = bcast_->payload_capacity();
    for (int sl = 0; sl < depth_; ++sl) {
      void* p = nullptr;
      ENG_CHECK(hipHostMalloc(&p, std::max<size_t>(cap, 64), hipHostMallocDefault));
      tp_stage_.push_back(p);
    }
    tp_role_ = TP_FOLLOWER;
  }
  void unlink_tp() { if (bcast_) bcast_->unlink(); }
  int tp_role() const { return tp_role_; }
  // false once stopped, failed, or (TP follower) after the leader's STOP
  bool running() const { return running_.load(); }
  uint64_t tp_published() const { return bcast_ ? bcast_->head() : 0; }
  void heartbeat() { job_.replica(replica_)->heartbeat_ns.store(now_ns()); }
  std::string error() {
    std::lock_guard<std::mutex> lk(mu_);
    return error_;
  }
  py::dict stats() {
    py::dict d;
    d["batches"] = batches_.load();
    d["requests"] = requests_.load();
    d["dropped"] = dropped_.load();
    d["padded"] = padded_.load();
    d["gpu_busy_ms"] = gpu_busy_ms_.load();
    d["backfill_batches"] = backfills_.load();
    d["completions_dropped"] = cmp_dropped_.load();
    d["error"] = error();
    return d;
  }

 private:
  Session& sess(int sid) {
    if (sid < 0 || sid >= n_sess_.load(std::memory_order_acquire)) throw std::out_of_range("session id");
    return *sess_ptr_[sid].load(std::memory_order_acquire);
  }
  static void free_host(Session& s) {
    for (auto p : s.host_tbl) hipHostFree(p);
    for (auto p : s.host_out) hipHostFree(p);
    s.host_tbl.clear();
    s.host_out.clear();
  }
  int bucket_for(const Session& s, int n) const {
    for (size_t i = 0; i < s.buckets.size(); ++i)
      if (s.buckets[i] >= n) return (int)i;
    return (int)s.buckets.size() - 1;
  }
  int64_t head_deadline(Session& s) {
    SlotHeader* h = s.ring.peek(s.peek_pos);
    if (!h) return INT64_MAX;
    if (h->deadline_ns) return h->deadline_ns;
    return h->t_submit_ns + (s.slo_ns ? s.slo_ns : 1000000000LL);
  }
  // Session choice: highest priority with work; ties -> earliest head deadline (EDF).
  int pick_session() {
    if (policy_ == POLICY_DUTY_CYCLE) return pick_duty_cycle();
    int best = -1;
    int best_pri = INT32_MIN;
    int64_t best_dl = INT64_MAX;
    const int ns = n_sess_.load(std::memory_order_acquire);
    for (int i = 0; i < ns; ++i) {
      Session& si = *sess_ptr_[i].load(std::memory_order_acquire);
      if (!si.active.load(std::memory_order_acquire)) continue;
      const int64_t dl = head_deadline(si);
      if (dl == INT64_MAX) continue;
      const int pri = si.priority;
      if (pri > best_pri || (pri == best_pri && dl < best_dl)) {
        best = (int)i;
        best_pri = pri;
        best_dl = dl;
      }
    }
    return best;
  }
  // Duty-cycle policy (fork GPUWorker.execute_schedule, scheduler.py:525-588, with
  // the cycle-end sleep sign fixed): every `cycle` each planned session runs ONE
  // batch of up to its planned size (Nexus: a session's batch per duty cycle),
  // round-robin; its GPU time is charged against its share.  When every session
  // with work has had its turn the launcher idles to the cycle boundary.
  // Sessions without a share (duty_share 0) are unconstrained (work-conserving).
  int pick_duty_cycle() {
    const int64_t cyc = duty_cycle_ns_.load(std::memory_order_relaxed);
    const int64_t now = now_ns();
    if (cyc > 0 && now - cycle_start_ns_ >= cyc) {
      cycle_start_ns_ = now - cycle_start_ns_ < 2 * cyc ? cycle_start_ns_ + cyc : now;
      ++cycle_idx_;
      for (int i = 0; i < n_sess_.load(std::memory_order_acquire); ++i) sess_ptr_[i].load()->used_ns = 0;
    }
    const size_t n = (size_t)n_sess_.load(std::memory_order_acquire);
    if (n == 0) return -1;
    bool waiting = false;
    for (size_t k = 0; k < n; ++k) {
      const size_t i = (rr_next_ + k) % n;
      Session& s = *sess_ptr_[i].load(std::memory_order_acquire);
      if (!s.active.load(std::memory_order_acquire) || !s.ring.peek(s.peek_pos)) continue;
      if (cyc > 0 && s.duty_share_ns > 0 &&
          (s.launched_cycle == cycle_idx_ || s.used_ns >= s.duty_share_ns)) {
        waiting = true;
        continue;
      }
      rr_next_ = (i + 1) % n;
      s.launched_cycle = cycle_idx_;
      return (int)i;
    }
    if (waiting) {
      // Work-conserving backfill: every session with work already had its turn.
      // Rather than idle, run another batch IF it finishes before the next
      // cycle starts (estimated), so the planned turns are never delayed; the
      // spare time goes to the session least served relative to its share
      // (used / share), so overload is split in the planned proportions.
      const int64_t left = cycle_start_ns_ + cyc - now_ns();
      int best = -1;
      double best_key = 1e300;
      for (size_t i = 0; i < n; ++i) {
        Session& s = *sess_ptr_[i].load(std::memory_order_acquire);
        if (!s.active.load(std::memory_order_acquire)) continue;
        SlotHeader* h = s.ring.peek(s.peek_pos);
        if (!h) continue;
        const uint64_t depth = s.ring.h->head.load(std::memory_order_relaxed) - s.peek_pos;
        const int bi = bucket_for(s, (int)std::min<uint64_t>(depth, (uint64_t)s.max_batch));
        if ((double)left < s.est(bi)) continue;
        const double key = (double)s.used_ns / (double)std::max<int64_t>(1, s.duty_share_ns) +
                           1e-12 * (double)(h->t_submit_ns & 0xFFFFFFF);  // tie-break: older head first
        if (key < best_key) {
          best_key = key;
          best = (int)i;
        }
      }
      if (best >= 0) {
        ++backfills_;
        return best;
      }
      if (left > 0) std::this_thread::sleep_for(std::chrono::nanoseconds(std::min<int64_t>(left, 2000000)));
    }
    return -1;
  }
  void set_error(const std::string& e) {
    std::lock_guard<std::mutex> lk(mu_);
    if (error_.empty()) error_ = e;
  }
  void write_completion(const SlotHeader* req, uint32_t queue, uint32_t status, const char* data,
                        uint32_t len, int64_t t_done) {
    Ring c = job_.cmp_ring(req->client);
    uint64_t pos;
    // Bounded: a client whose ring stays full (crashed / wedged proxy) is marked
    // stalled and loses this completion instead of stalling every other client.
    SlotHeader* s = reserve_completion(job_, req->client, &pos, [this] {
      return !running_.load(std::memory_order_relaxed) || job_.hdr()->shutdown.load(std::memory_order_relaxed);
    });
    QueueState* qs = job_.queue(queue);
    if (!s) {  // dropped: still leaves the queue's ongoing count
      qs->errors.fetch_add(1, std::memory_order_relaxed);
      qs->completed.fetch_add(1, std::memory_order_release);
      cmp_dropped_.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    if (len > c.max_payload()) { status = ST_TOO_LARGE; len = 0; }
    s->req_id = req->req_id;
    s->t_submit_ns = req->t_submit_ns;
    s->deadline_ns = req->deadline_ns;
    s->len = len;
    s->kind = 0;
    s->client = req->client;
    s->queue = queue;
    s->status = status;
    s->t_aux_ns = t_done;
    if (len) memcpy(c.payload(s), data, len);
    const int64_t e2e = t_done - req->t_submit_ns;
    if (status == ST_OK) {
      qs->hist_e2e.record((uint64_t)std::max<int64_t>(0, e2e));
      const int64_t slo = qs->slo_ns.load(std::memory_order_relaxed);
      if (slo > 0 && e2e > slo) qs->slo_violations.fetch_add(1, std::memory_order_relaxed);
    } else if (status == ST_DROPPED_STALE) {
      qs->dropped.fetch_add(1, std::memory_order_relaxed);
    } else {
      qs->errors.fetch_add(1, std::memory_order_relaxed);
    }
    qs->completed.fetch_add(1, std::memory_order_release);
    c.publish(s, pos);
  }

  void launcher_loop() {
    try {
      ENG_CHECK(hipSetDevice(device_));
      uint64_t counter = 0;
      while (running_) {
        const int slot = (int)(counter % depth_);
        {  // wait for the slot to be free
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return !slot_busy_[slot] || !running_; });
          if (!running_) break;
        }
        // wait for any work
        int sid = pick_session();
        if (sid < 0) {
          for (int i = 0; i < 4000 && sid < 0; ++i) {  // short spin
            cpu_relax();
            if ((i & 63) == 63) sid = pick_session();
          }
          if (sid < 0) {
            // sleep on the doorbell of the only active session, else poll briefly
            Session* only = nullptr;
            int n_active = 0;
            for (int i = 0; i < n_sess_.load(std::memory_order_acquire); ++i) {
              Session* c = sess_ptr_[i].load(std::memory_order_acquire);
              if (c->active.load(std::memory_order_acquire)) { only = c; ++n_active; }
            }
            if (n_active == 1) only->ring.wait_for(only->peek_pos, 20000000LL, 0);
            else if (n_active > 1) only->ring.wait_for(only->peek_pos, 200000LL, 0);
            else std::this_thread::sleep_for(std::chrono::microseconds(200));
            continue;
          }
        }
        Session& s = *sess_ptr_[sid].load(std::memory_order_acquire);
        // Dekker pair with retire_session(): count the batch first, then re-check
        // `active` (both seq_cst) -- either retire sees the count or we see the flag
        s.inflight.fetch_add(1, std::memory_order_seq_cst);
        if (!s.active.load(std::memory_order_seq_cst)) {
          s.inflight.fetch_sub(1, std::memory_order_seq_cst);
          continue;
        }
        job_.replica(replica_)->heartbeat_ns.store(now_ns(), std::memory_order_relaxed);
        roctxRangePushA("rdb:form_batch");
        InFlight f;
        f.session = sid;
        f.slot = slot;
        f.pos_begin = s.peek_pos;
        f.t_form_start = now_ns();
        const int64_t flush_at = f.t_form_start + s.max_wait_ns;
        uint64_t* tbl = reinterpret_cast<uint64_t*>(s.host_tbl[slot]);
        int n = 0;
        if (tp_role_ == TP_LEADER) tp_rows_.clear();
        while (n < s.max_batch) {
          SlotHeader* h = s.ring.peek(s.peek_pos);
          if (!h) {
            const int64_t left = flush_at - now_ns();
            if (left <= 0 || !running_) break;
            if (idle_dispatch_.load(std::memory_order_relaxed)) {
              // idle dispatch (opt-in): a partial batch goes out as soon as a
              // compute stream has no batch running, instead of waiting out the
              // first-arrival timeout while the GPU sits idle; the wait is
              // chunked so a stream going idle is noticed within ~20 us
              if (n > 0 && gpu_running_.load(std::memory_order_acquire) < (int)compute_streams_.size()) break;
              s.ring.wait_for(s.peek_pos, std::min<int64_t>(left, 20000), 2000);
              continue;
            }
            if (!s.ring.wait_for(s.peek_pos, left, 4000)) break;
            continue;
          }
          // stale-request drop (fork semantics: arrival + SLO < now + lat(batch))
          int64_t dl = h->deadline_ns;
          if (!dl && s.drop_stale && s.slo_ns) dl = h->t_submit_ns + s.slo_ns;
          if (dl) {
            const double est = s.est_wall(bucket_for(s, std::min(s.max_batch, n + 1)));
            if ((double)now_ns() + est > (double)dl) {
              write_completion(h, s.queue, ST_DROPPED_STALE, nullptr, 0, now_ns());
              dropped_.fetch_add(1, std::memory_order_relaxed);
              ++s.peek_pos;
              continue;
            }
          }
          if (fault_drop_every_ > 0 && ++fault_req_count_ % fault_drop_every_ == 0) {
            write_completion(h, s.queue, ST_REPLICA_DIED, nullptr, 0, now_ns());  // injected loss
            ++s.peek_pos;
            continue;
          }
          if (h->len != (uint32_t)s.in_row_bytes) {
            write_completion(h, s.queue, ST_ERROR, nullptr, 0, now_ns());
            ++s.peek_pos;
            continue;
          }
          if (h->kind != 0) {   // KIND_TENSOR only: a pickled call cannot be a model row
            write_completion(h, s.queue, ST_ERROR, nullptr, 0, now_ns());
            ++s.peek_pos;
            continue;
          }
          f.req_pos.push_back(s.peek_pos);
          char* payload = reinterpret_cast<char*>(h) + sizeof(SlotHeader);
          if (tp_role_ == TP_LEADER) tp_rows_.push_back(payload);
          tbl[n++] = zero_copy_ ? reinterpret_cast<uint64_t>(dev_base_ + (payload - host_base_))
                                : reinterpret_cast<uint64_t>(payload);
          ++s.peek_pos;
        }
        f.pos_end = s.peek_pos;
        roctxRangePop();
        if (n > 0) roctxRangePushA("rdb:launch");
        if (n > 0 && fault_delay_batch_us_ > 0)
          std::this_thread::sleep_for(std::chrono::microseconds(fault_delay_batch_us_));
        if (n > 0 && fault_kill_after_ > 0 && ++fault_batch_count_ > fault_kill_after_) _exit(137);
        if (n > 0) {
          const int bi = bucket_for(s, n);
          const int rows = s.buckets[bi];
          f.bucket_idx = bi;
          f.gpu = true;
          if (tp_role_ == TP_LEADER) {
            // every follower replays the same (session, bucket, slot) graph on these rows
            BcastRecord* r = nullptr;
            while (running_ && !(r = bcast_->reserve(50000000LL)))
              if (bcast_->closed()) throw std::runtime_error("tp broadcast ring closed (a follower rank is gone)");
            if (!r) {   // stopping while the followers lag: the batch is abandoned with the engine
              s.inflight.fetch_sub(1, std::memory_order_seq_cst);
              roctxRangePop();
              break;
            }
            r->kind = BCAST_BATCH;
            r->a = sid;
            r->b = bi;
            r->c = slot;
            r->n = (uint32_t)n;
            r->len = (uint32_t)((size_t)n * s.in_row_bytes);
            char* dst = bcast_->payload(r);
            for (int i = 0; i < n; ++i) memcpy(dst + (size_t)i * s.in_row_bytes, tp_rows_[i], s.in_row_bytes);
            bcast_->commit(r);
          }
          const uintptr_t in = s.in_dev[slot];
          if (dma_gather_) {
            // rows of one batch are consecutive ring slots except at the wrap:
            // one strided copy per run of equally spaced payloads
            char* dst = reinterpret_cast<char*>(in);
            int i0 = 0;
            while (i0 < n) {
              int i1 = i0 + 1;
              const int64_t pitch = n > i0 + 1 ? (int64_t)(tbl[i0 + 1] - tbl[i0]) : (int64_t)s.in_row_bytes;
              if (pitch >= s.in_row_bytes)
                while (i1 < n && (int64_t)(tbl[i1] - tbl[i1 - 1]) == pitch) ++i1;
              const char* src = host_base_ + (reinterpret_cast<char*>(tbl[i0]) - dev_base_);
              ENG_CHECK(hipMemcpy2DAsync(dst + (size_t)i0 * s.in_row_bytes, s.in_row_bytes, src,
                                         (size_t)std::max<int64_t>(pitch, s.in_row_bytes), s.in_row_bytes,
                                         i1 - i0, hipMemcpyHostToDevice, copy_stream_));
              i0 = i1;
            }
            if (rows > n)
              ENG_CHECK(hipMemsetAsync(dst + (size_t)n * s.in_row_bytes, 0,
                                       (size_t)(rows - n) * s.in_row_bytes, copy_stream_));
          } else if (zero_copy_) {
            gather_rows(reinterpret_cast<uintptr_t>(tbl), n, rows, s.in_row_bytes, in,
                        reinterpret_cast<uintptr_t>(copy_stream_));
          } else {
            for (int i = 0; i < n; ++i)
              ENG_CHECK(hipMemcpyAsync(reinterpret_cast<char*>(in) + (size_t)i * s.in_row_bytes,
                                       reinterpret_cast<void*>(tbl[i]), s.in_row_bytes,
                                       hipMemcpyHostToDevice, copy_stream_));
            if (rows > n)
              ENG_CHECK(hipMemsetAsync(reinterpret_cast<char*>(in) + (size_t)n * s.in_row_bytes, 0,
                                       (size_t)(rows - n) * s.in_row_bytes, copy_stream_));
          }
          const int si = slot % (int)compute_streams_.size();
          hipStream_t cs = compute_streams_[si];
          if (stagger_ns_ > 0 && compute_streams_.size() > 1 && stream_running_[si].load(std::memory_order_acquire) == 0) {
            // this stream starts from idle: keep it stagger_ns_ behind the last idle-start of another stream
            const int64_t t_other = last_idle_start_ns_.load(std::memory_order_acquire);
            const int64_t wait = t_other + stagger_ns_ - now_ns();
            if (last_idle_stream_.load(std::memory_order_acquire) != si && wait > 0)
              std::this_thread::sleep_for(std::chrono::nanoseconds(std::min<int64_t>(wait, stagger_ns_)));
            last_idle_start_ns_.store(now_ns(), std::memory_order_release);
            last_idle_stream_.store(si, std::memory_order_release);
          }
          ENG_CHECK(hipEventRecord(ev_copy_[slot], copy_stream_));
          ENG_CHECK(hipStreamWaitEvent(cs, ev_copy_[slot], 0));
          ENG_CHECK(hipEventRecord(ev_start_[slot], cs));
          ENG_CHECK(hipGraphLaunch(s.graphs[bi][slot], cs));
          ENG_CHECK(hipMemcpyAsync(s.host_out[slot],
                                   reinterpret_cast<void*>(s.out_dev[bi][slot]),
                                   (size_t)n * s.out_row_bytes, hipMemcpyDeviceToHost, cs));
          ENG_CHECK(hipEventRecord(ev_done_[slot], cs));
          s.used_ns += (int64_t)s.est(bi);
          padded_.fetch_add(rows - n, std::memory_order_relaxed);
          roctxRangePop();
        }
        f.t_launch = now_ns();
        {
          std::lock_guard<std::mutex> lk(mu_);
          slot_busy_[slot] = true;
          if (f.gpu) {
            f.solo = gpu_inflight_ == 0;
            f.seq = launch_seq_.fetch_add(1, std::memory_order_acq_rel) + 1;
            ++gpu_inflight_;
            gpu_running_.fetch_add(1, std::memory_order_acq_rel);
            stream_running_[slot % compute_streams_.size()].fetch_add(1, std::memory_order_acq_rel);
          }
          inflight_.push_back(std::move(f));
        }
        cv_.notify_all();
        ++counter;
      }
    } catch (const std::exception& e) {
      set_error(std::string("launcher: ") + e.what());
      job_.replica(replica_)->status.store(RS_DEAD);
      running_ = false;
      cv_.notify_all();
    }
  }

  // TP follower launcher: the leader's records, in order (see the header comment).
  void follower_loop() {
    try {
      ENG_CHECK(hipSetDevice(device_));
      while (running_) {
        const BcastRecord* r = bcast_->take(tp_reader_, 20000000LL);
        if (!r) {
          if (bcast_->closed()) break;      // the leader stopped (or the group is going down)
          continue;
        }
        if (r->kind == BCAST_STOP) {
          bcast_->release(tp_reader_);
          break;
        }
        const int sid = r->a, bi = r->b, slot = r->c, n = (int)r->n;
        if (sid < 0 || sid >= n_sess_.load(std::memory_order_acquire) || slot < 0 || slot >= depth_)
          throw std::runtime_error("tp follower: record names an unknown session / slot");
        Session& s = *sess_ptr_[sid].load(std::memory_order_acquire);
        if (bi < 0 || bi >= (int)s.buckets.size() || n < 1 || n > s.buckets[bi] ||
            r->len != (uint32_t)((size_t)n * s.in_row_bytes))
          throw std::runtime_error("tp follower: record does not match the session's buckets / row size");
        {  // the slot's previous batch must be done before its input / staging are rewritten
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return !slot_busy_[slot] || !running_; });
          if (!running_) break;
        }
        s.inflight.fetch_add(1, std::memory_order_seq_cst);
        InFlight f;
        f.session = sid;
        f.slot = slot;
        f.bucket_idx = bi;
        f.gpu = true;
        f.tp_n = n;
        f.t_form_start = now_ns();
        memcpy(tp_stage_[slot], reinterpret_cast<const char*>(r) + sizeof(BcastRecord), r->len);
        bcast_->release(tp_reader_);
        const int rows = s.buckets[bi];
        const uintptr_t in = s.in_dev[slot];
        ENG_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(in), tp_stage_[slot], (size_t)n * s.in_row_bytes,
                                 hipMemcpyHostToDevice, copy_stream_));
        if (rows > n)
          ENG_CHECK(hipMemsetAsync(reinterpret_cast<char*>(in) + (size_t)n * s.in_row_bytes, 0,
                                   (size_t)(rows - n) * s.in_row_bytes, copy_stream_));
        hipStream_t cs = compute_streams_[0];
        ENG_CHECK(hipEventRecord(ev_copy_[slot], copy_stream_));
        ENG_CHECK(hipStreamWaitEvent(cs, ev_copy_[slot], 0));
        ENG_CHECK(hipEventRecord(ev_start_[slot], cs));
        ENG_CHECK(hipGraphLaunch(s.graphs[bi][slot], cs));
        ENG_CHECK(hipEventRecord(ev_done_[slot], cs));
        f.t_launch = now_ns();
        {
          std::lock_guard<std::mutex> lk(mu_);
          slot_busy_[slot] = true;
          ++gpu_inflight_;
          gpu_running_.fetch_add(1, std::memory_order_acq_rel);
          stream_running_[0].fetch_add(1, std::memory_order_acq_rel);
          inflight_.push_back(std::move(f));
        }
        cv_.notify_all();
      }
    } catch (const std::exception& e) {
      set_error(std::string("tp follower: ") + e.what());
    }
    running_ = false;
    cv_.notify_all();
  }

  void completer_loop() {
    try {
      ENG_CHECK(hipSetDevice(device_));
      ReplicaState* rs = job_.replica(replica_);
      for (;;) {
        InFlight f;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return !inflight_.empty() || stopping_completer_; });
          if (inflight_.empty()) break;
          f = std::move(inflight_.front());
          inflight_.pop_front();
        }
        Session& s = *sess_ptr_[f.session].load(std::memory_order_acquire);
        const int n = (int)f.req_pos.size();
        if (f.gpu && tp_role_ == TP_FOLLOWER) {
          // a follower's batch: its requests belong to rank 0; only the slot is retired
          for (;;) {
            hipError_t q = hipEventQuery(ev_done_[f.slot]);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) ENG_CHECK(q);
            std::this_thread::yield();
          }
          gpu_running_.fetch_sub(1, std::memory_order_acq_rel);
          stream_running_[0].fetch_sub(1, std::memory_order_acq_rel);
          batches_.fetch_add(1, std::memory_order_relaxed);
          requests_.fetch_add(f.tp_n, std::memory_order_relaxed);
          {
            std::lock_guard<std::mutex> lk(mu_);
            slot_busy_[f.slot] = false;
            --gpu_inflight_;
          }
          s.inflight.fetch_sub(1, std::memory_order_seq_cst);
          cv_.notify_all();
          continue;
        }
        if (f.gpu) {
          // low-latency wait: spin on the event, yielding
          for (;;) {
            hipError_t q = hipEventQuery(ev_done_[f.slot]);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) ENG_CHECK(q);
            std::this_thread::yield();
          }
          gpu_running_.fetch_sub(1, std::memory_order_acq_rel);
          stream_running_[f.slot % compute_streams_.size()].fetch_sub(1, std::memory_order_acq_rel);
          const int64_t t_obs = now_ns();
          roctxRangePushA("rdb:complete");
          float ms = 0.f;
          if (hipEventElapsedTime(&ms, ev_start_[f.slot], ev_done_[f.slot]) == hipSuccess) {
            gpu_busy_ms_.store(gpu_busy_ms_.load() + ms);
            rs->busy_ns.fetch_add((uint64_t)(ms * 1e6), std::memory_order_relaxed);
            // EMAs of the service time of this bucket: the overlap-inflated
            // span always, the solo estimate only from a batch that shared the
            // GPU with no other batch from its launch to its completion
            const double v = ms * 1e6;
            std::atomic<double>& w = s.est_wall_ns[f.bucket_idx];
            const double w0 = w.load(std::memory_order_relaxed);
            w.store(w0 == 0.0 ? v : 0.9 * w0 + 0.1 * v, std::memory_order_relaxed);
            const bool solo = f.solo && launch_seq_.load(std::memory_order_acquire) == f.seq;
            std::atomic<double>& e = s.est_ns[f.bucket_idx];
            const double e0 = e.load(std::memory_order_relaxed);
            std::atomic<bool>& prov = s.est_prov[f.bucket_idx];
            if (solo && prov.load(std::memory_order_relaxed)) {
              e.store(v, std::memory_order_relaxed);          // first solo batch replaces a seed
              prov.store(false, std::memory_order_relaxed);
            } else if (e0 == 0.0) {
              e.store(v, std::memory_order_relaxed);          // overlapped: a seed, still provisional
            } else if (solo) {
              e.store(0.9 * e0 + 0.1 * v, std::memory_order_relaxed);
            }
          }
          const char* out = reinterpret_cast<const char*>(s.host_out[f.slot]);
          const int64_t t_done = now_ns();
          QueueState* qs = job_.queue(s.queue);
          for (int i = 0; i < n; ++i) {
            SlotHeader* h = s.ring.slot(f.req_pos[i]);
            qs->hist_queue_wait.record((uint64_t)std::max<int64_t>(0, f.t_launch - h->t_submit_ns));
            write_completion(h, s.queue, ST_OK, out + (size_t)i * s.out_row_bytes, s.out_row_bytes, t_done);
          }
          rs->batches.fetch_add(1, std::memory_order_relaxed);
          rs->batch_items.fetch_add(n, std::memory_order_relaxed);
          rs->padded_items.fetch_add(s.buckets[f.bucket_idx] - n, std::memory_order_relaxed);
          rs->graph_replays.fetch_add(1, std::memory_order_relaxed);
          rs->hist_batch_size.record((uint64_t)n);
          rs->hist_service.record((uint64_t)(t_done - f.t_form_start));
          batches_.fetch_add(1, std::memory_order_relaxed);
          requests_.fetch_add(n, std::memory_order_relaxed);
          TraceRing* tr = job_.trace(replica_);
          const uint32_t rows = (uint32_t)s.buckets[f.bucket_idx];
          tr->record(TK_FORM, f.t_form_start, f.t_launch, s.queue, n, rows);
          tr->record(TK_GPU, t_obs - (int64_t)(ms * 1e6), t_obs, s.queue, n, rows);
          tr->record(TK_COMPLETE, t_obs, now_ns(), s.queue, n, rows);
          roctxRangePop();
        }
        s.ring.commit(f.pos_end);
        {
          std::lock_guard<std::mutex> lk(mu_);
          slot_busy_[f.slot] = false;
          if (f.gpu) --gpu_inflight_;
        }
        s.inflight.fetch_sub(1, std::memory_order_seq_cst);
        cv_.notify_all();
      }
    } catch (const std::exception& e) {
      set_error(std::string("completer: ") + e.what());
      job_.replica(replica_)->status.store(RS_DEAD);
      running_ = false;
      cv_.notify_all();
    }
  }

  Job job_;
  uint32_t replica_;
  int depth_;
  bool zero_copy_;
  bool dma_gather_ = false;
  int device_;
  int policy_;
  bool registered_ = false;
  char* host_base_ = nullptr;
  char* dev_base_ = nullptr;
  hipStream_t copy_stream_ = nullptr;
  std::vector<hipStream_t> compute_streams_;
  std::atomic<int64_t> duty_cycle_ns_{0};
  long long fault_drop_every_ = 0, fault_delay_batch_us_ = 0, fault_kill_after_ = 0;
  long long fault_req_count_ = 0, fault_batch_count_ = 0;
  int64_t cycle_start_ns_ = 0;
  uint64_t cycle_idx_ = 0;
  std::atomic<uint64_t> backfills_{0};
  size_t rr_next_ = 0;
  std::vector<hipEvent_t> ev_copy_, ev_start_, ev_done_;
  static constexpr int kMaxSessions = 64;
  std::array<std::atomic<Session*>, kMaxSessions> sess_ptr_{};
  std::atomic<int> n_sess_{0};
  std::vector<std::unique_ptr<Session>> owned_;   // every Session ever created (api_mu_)
  std::mutex api_mu_;
  std::vector<bool> slot_busy_;
  std::deque<InFlight> inflight_;
  int gpu_inflight_ = 0;                   // GPU batches launched and not yet completed (under mu_)
  std::atomic<int> gpu_running_{0};        // GPU batches whose done-event has not fired yet
  std::unique_ptr<std::atomic<int>[]> stream_running_;   // ... per compute stream
  int64_t stagger_ns_ = 0;
  std::atomic<int64_t> last_idle_start_ns_{0};
  std::atomic<int> last_idle_stream_{-1};
  std::atomic<bool> idle_dispatch_{false}; // batch policy: dispatch partial batches onto an idle stream
  std::atomic<uint64_t> launch_seq_{0};    // GPU launches so far (solo detection)
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread launcher_, completer_;
  std::atomic<bool> running_{false};
  bool stopping_completer_ = false;
  std::string error_;
  std::atomic<uint64_t> batches_{0}, requests_{0}, dropped_{0}, padded_{0}, cmp_dropped_{0};
  std::atomic<double> gpu_busy_ms_{0.0};
  // tensor-parallel role (set_tp_leader / set_tp_follower)
  enum { TP_NONE = 0, TP_LEADER = 1, TP_FOLLOWER = 2 };
  int tp_role_ = TP_NONE;
  std::unique_ptr<TPBcast> bcast_;
  uint32_t tp_reader_ = 0;
  std::vector<void*> tp_stage_;            // follower: pinned staging per pipeline slot
  std::vector<const char*> tp_rows_;       // leader: host rows of the batch being formed
};

}  // namespace

void register_engine(py::module_& m) {
  py::class_<Engine>(m, "Engine")
      .def(py::init<const std::string&, uint32_t, int, bool, int, int, int>(), py::arg("job_name"),
           py::arg("replica"), py::arg("pipeline_depth") = 2, py::arg("zero_copy") = true,
           py::arg("device") = 0, py::arg("policy") = 0, py::arg("compute_streams") = 1)
      .def("add_session", &Engine::add_session, py::arg("queue"), py::arg("max_batch"),
           py::arg("max_wait_s"), py::arg("buckets"), py::arg("in_row_bytes"),
           py::arg("out_row_bytes"), py::arg("priority") = 0, py::arg("slo_ms") = 0.0,
           py::arg("drop_stale") = false)
      .def("set_input", &Engine::set_input)
      .def("set_graph", &Engine::set_graph)
      .def("set_latency_estimate", &Engine::set_latency_estimate, py::arg("sid"), py::arg("bucket_idx"),
           py::arg("ms"), py::arg("provisional") = false)
      .def("latency_estimate_provisional", &Engine::latency_estimate_provisional)
      .def("latency_estimate", &Engine::latency_estimate)
      .def("set_duty_share", &Engine::set_duty_share)
      .def("set_duty_cycle", &Engine::set_duty_cycle)
      .def("set_session_active", &Engine::set_session_active)
      .def("readd_session", &Engine::readd_session, py::arg("queue"), py::arg("max_batch"), py::arg("max_wait_s"),
           py::arg("buckets"), py::arg("in_row_bytes"), py::arg("out_row_bytes"), py::arg("priority") = 0,
           py::arg("slo_ms") = 0.0, py::arg("drop_stale") = false)
      .def("retire_session", &Engine::retire_session, py::arg("sid"), py::arg("timeout_s") = 10.0,
           py::call_guard<py::gil_scoped_release>())
      .def("session_inflight", &Engine::session_inflight)
      .def("session_pending", &Engine::session_pending)
      .def("session_retired", &Engine::session_retired)
      .def("num_sessions", &Engine::num_sessions)
      .def("compute_streams", &Engine::compute_streams)
      .def("set_idle_dispatch", &Engine::set_idle_dispatch)
      .def("set_stagger_us", &Engine::set_stagger_us)
      .def("set_tp_leader", &Engine::set_tp_leader, py::arg("name"), py::arg("n_followers"), py::arg("n_slots") = 8)
      .def("set_tp_follower", &Engine::set_tp_follower, py::arg("name"), py::arg("reader"),
           py::arg("attach_timeout_s") = 120.0)
      .def("unlink_tp", &Engine::unlink_tp)
      .def("tp_role", &Engine::tp_role)
      .def("running", &Engine::running)
      .def("tp_published", &Engine::tp_published)
      .def("stagger_us", &Engine::stagger_us)
      .def("idle_dispatch", &Engine::idle_dispatch)
      .def("set_max_batch", &Engine::set_max_batch)
      .def("set_max_wait", &Engine::set_max_wait)
      .def("start", &Engine::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Engine::stop, py::call_guard<py::gil_scoped_release>())
      .def("heartbeat", &Engine::heartbeat)
      .def("error", &Engine::error)
      .def("stats", &Engine::stats);
}

}  // namespace rdb
