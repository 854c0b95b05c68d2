// Node agent: the single-node replacement for the parts of Ray's raylet + GCS
// the serving stack relies on:
//
//  * Config       -- typed flag registry with RDB_<NAME> environment override
//                    (ray_config.h:72-77 / ray_config_def.h RAY_CONFIG macros).
//  * GpuAllocator -- unit-instance GPU slots: a demand >= 1 takes whole free
//                    GPUs first-fit, a fractional demand goes best-fit to the GPU
//                    with the least remaining capacity that still fits
//                    (resource_instance_set.cc:93-187), plus an HBM budget per
//                    GPU (288 GB on MI355X) so planner-packed models fit.
//  * KvStore      -- small persistent KV (config checkpoint, plan, RCCL
//                    bootstrap ids) written atomically (gcs_kv_manager,
//                    serve controller checkpoint controller.py:510-563).
//  * Supervisor   -- spawns one replica process per GPU slot (posix_spawn, own
//                    process group, log file), watches exit status and the
//                    replica's shm heartbeat, and on death fails the replica's
//                    pending requests (REPLICA_DIED -> routers retry elsewhere),
//                    bumps its generation and restarts it with exponential
//                    back-off (gcs_actor_manager.cc:1167-1361 restarts,
//                    gcs_health_check_manager.cc:79 health checks).
//  * Control RPC  -- a Unix-domain-socket line protocol (PING / STATUS / KV_*)
//                    so CLIs and other processes can query a running agent
//                    (replaces the gRPC control plane, rpc/grpc_server.h:85).
#include <fcntl.h>
#include <poll.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <spawn.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <unistd.h>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "shm.h"

extern char** environ;

namespace py = pybind11;
using namespace rdb::rt;

namespace rdb {
namespace agent {

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char b[8];
          snprintf(b, sizeof(b), "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o;
}

// ---------------------------------------------------------------------------
// Config: typed flags, env override RDB_<UPPER_NAME>.
// ---------------------------------------------------------------------------
struct Flag {
  std::string type, default_value, value, help;
  bool from_env = false;
};

class Config {
 public:
  static Config& instance() {
    static Config c;
    return c;
  }
  std::string define(const std::string& name, const std::string& type, const std::string& def,
                     const std::string& help) {
    std::lock_guard<std::mutex> lk(mu_);
    Flag f;
    f.type = type;
    f.default_value = def;
    f.help = help;
    f.value = def;
    std::string env = "RDB_";
    for (char c : name) env += (char)toupper((unsigned char)c);
    if (const char* v = getenv(env.c_str())) {
      f.value = v;
      f.from_env = true;
    }
    validate(type, f.value, name);
    auto it = flags_.find(name);
    if (it != flags_.end() && !it->second.from_env && it->second.value != it->second.default_value)
      f.value = it->second.value;  // keep an explicit set() made before (re)definition
    flags_[name] = f;
    return f.value;
  }
  std::string get(const std::string& name) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = flags_.find(name);
    if (it == flags_.end()) throw std::out_of_range("unknown config flag: " + name);
    return it->second.value;
  }
  void set(const std::string& name, const std::string& v) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = flags_.find(name);
    if (it == flags_.end()) throw std::out_of_range("unknown config flag: " + name);
    validate(it->second.type, v, name);
    it->second.value = v;
  }
  double get_double(const std::string& name) { return std::stod(get(name)); }
  py::dict all() {
    std::lock_guard<std::mutex> lk(mu_);
    py::dict d;
    for (auto& kv : flags_) {
      py::dict f;
      f["type"] = kv.second.type;
      f["value"] = kv.second.value;
      f["default"] = kv.second.default_value;
      f["help"] = kv.second.help;
      f["from_env"] = kv.second.from_env;
      d[py::str(kv.first)] = f;
    }
    return d;
  }

 private:
  Config() {
    // (name, type, default, help) -- Serve / Ray defaults where they exist
    const char* defs[][4] = {
        {"health_check_period_s", "float", "10.0", "replica health-check period (serve constants.py:107)"},
        {"health_check_timeout_s", "float", "30.0", "heartbeat age that marks a replica dead (constants.py:108)"},
        {"restart_backoff_initial_s", "float", "0.5", "first restart delay; doubles per restart"},
        {"restart_backoff_max_s", "float", "30.0", "restart delay cap"},
        {"max_restarts", "int", "-1", "restarts per replica slot, -1 = unlimited (actor max_restarts)"},
        {"control_loop_interval_s", "float", "0.1", "controller tick (serve CONTROL_LOOP_INTERVAL_S)"},
        {"replica_start_timeout_s", "float", "900", "time a replica may take to become READY"},
        {"hbm_gb_per_gpu", "float", "288", "HBM budget per GPU for placement (MI355X: 288 GB)"},
        {"agent_monitor_interval_ms", "int", "20", "supervisor poll interval"},
        {"fault_drop_every", "int", "0", "fault injection: drop every Nth request at the replica (0=off)"},
        {"fault_delay_batch_us", "int", "0", "fault injection: delay each batch by this many us"},
        {"fault_kill_after_batches", "int", "0", "fault injection: replica exits after N batches (0=off)"},
        {"fault_reject_every", "int", "0", "fault injection: router rejects every Nth submit (0=off)"},
        {"trace", "int", "0", "1 = record per-batch trace events into the shm trace ring"},
    };
    for (auto& d : defs) {
      Flag f;
      f.type = d[1];
      f.default_value = d[2];
      f.value = d[2];
      f.help = d[3];
      std::string env = "RDB_";
      for (const char* p = d[0]; *p; ++p) env += (char)toupper((unsigned char)*p);
      if (const char* v = getenv(env.c_str())) {
        f.value = v;
        f.from_env = true;
      }
      flags_[d[0]] = f;
    }
  }
  static void validate(const std::string& type, const std::string& v, const std::string& name) {
    try {
      size_t used = 0;
      if (type == "int") {
        (void)std::stoll(v, &used);
      } else if (type == "float") {
        (void)std::stod(v, &used);
      } else if (type == "bool") {
        if (v != "0" && v != "1" && v != "true" && v != "false")
          throw std::invalid_argument("bool");
        used = v.size();
      } else {
        used = v.size();
      }
      if (used != v.size()) throw std::invalid_argument("trailing");
    } catch (const std::exception&) {
      throw std::invalid_argument("config flag " + name + ": '" + v + "' is not a valid " + type);
    }
  }
  std::mutex mu_;
  std::map<std::string, Flag> flags_;
};

// ---------------------------------------------------------------------------
// GPU allocator (fixed point, 1 GPU = 10000 units like Ray's FixedPoint).
// ---------------------------------------------------------------------------
constexpr int64_t kUnit = 10000;

class GpuAllocator {
 public:
  GpuAllocator(int num_gpus, double hbm_gb_per_gpu)
      : used_(num_gpus, 0), hbm_used_(num_gpus, 0),
        hbm_total_((int64_t)std::llround(hbm_gb_per_gpu * 1e9)) {}
  // Returns {gpus, fraction} or None.
  py::object allocate(const std::string& owner, double num_gpus, double hbm_gb) {
    std::lock_guard<std::mutex> lk(mu_);
    if (allocs_.count(owner)) throw std::invalid_argument(owner + " already holds GPUs");
    const int64_t hbm = (int64_t)std::llround(hbm_gb * 1e9);
    Alloc a;
    if (num_gpus <= 0) {
      allocs_[owner] = a;
      return to_py(a);
    }
    const int64_t units = (int64_t)std::llround(num_gpus * kUnit);
    if (units >= kUnit) {
      if (units % kUnit) throw std::invalid_argument("num_gpus > 1 must be an integer");
      const int need = (int)(units / kUnit);
      const int64_t per = hbm / need;
      for (size_t g = 0; g < used_.size() && (int)a.gpus.size() < need; ++g)
        if (used_[g] == 0 && hbm_total_ - hbm_used_[g] >= per) a.gpus.push_back((int)g);
      if ((int)a.gpus.size() < need) return py::none();
      for (int g : a.gpus) {
        used_[g] = kUnit;
        hbm_used_[g] += per;
        a.units.push_back(kUnit);
        a.hbm.push_back(per);
      }
    } else {
      int best = -1;
      int64_t best_left = INT64_MAX;
      for (size_t g = 0; g < used_.size(); ++g) {
        const int64_t left = kUnit - used_[g] - units;
        if (left < 0 || hbm_total_ - hbm_used_[g] < hbm) continue;
        if (left < best_left) {
          best_left = left;
          best = (int)g;
        }
      }
      if (best < 0) return py::none();
      used_[best] += units;
      hbm_used_[best] += hbm;
      a.gpus.push_back(best);
      a.units.push_back(units);
      a.hbm.push_back(hbm);
    }
    allocs_[owner] = a;
    return to_py(a);
  }
  // Placement group (python/ray/util/placement_group.py:145, serve
  // deployment_scheduler.py:494-620): reserve ALL bundles or none (gang).
  // bundles = [(num_gpus, hbm_gb), ...]; strategy PACK / SPREAD (best effort:
  // prefer GPUs this group already uses / does not use yet), STRICT_PACK (every
  // bundle on one GPU), STRICT_SPREAD (every GPU-holding bundle on its own GPU).
  // Returns {gpus: distinct GPUs in first-use order, bundle_gpus: [[...] per
  // bundle], fraction} or None.
  py::object allocate_bundles(const std::string& owner, const std::vector<std::pair<double, double>>& bundles,
                              const std::string& strategy) {
    std::lock_guard<std::mutex> lk(mu_);
    if (allocs_.count(owner)) throw std::invalid_argument(owner + " already holds GPUs");
    const bool spread = strategy == "SPREAD" || strategy == "STRICT_SPREAD";
    const bool strict_spread = strategy == "STRICT_SPREAD", strict_pack = strategy == "STRICT_PACK";
    if (!spread && !strict_pack && strategy != "PACK")
      throw std::invalid_argument("placement strategy must be PACK, SPREAD, STRICT_PACK or STRICT_SPREAD");
    std::vector<int64_t> used = used_, hbm_used = hbm_used_;   // simulate, commit only if all fit
    Alloc a;
    std::vector<std::vector<int>> per_bundle;
    std::vector<int> mine;                                        // GPUs this group holds so far
    auto is_mine = [&](int g) { return std::find(mine.begin(), mine.end(), g) != mine.end(); };
    int pack_gpu = -1;
    for (const auto& b : bundles) {
      const int64_t units = (int64_t)std::llround(b.first * kUnit);
      const int64_t hbm = (int64_t)std::llround(b.second * 1e9);
      std::vector<int> got;
      if (units <= 0) {
        per_bundle.push_back(got);
        continue;
      }
      if (units >= kUnit) {
        if (units % kUnit) throw std::invalid_argument("bundle GPU > 1 must be an integer");
        const int need = (int)(units / kUnit);
        if (strict_pack && (bundles.size() > 1 || need > 1)) return py::none();
        const int64_t per = hbm / need;
        for (size_t g = 0; g < used.size() && (int)got.size() < need; ++g)
          if (used[g] == 0 && hbm_total_ - hbm_used[g] >= per) got.push_back((int)g);
        if ((int)got.size() < need) return py::none();
        for (int g : got) {
          used[g] = kUnit;
          hbm_used[g] += per;
          a.gpus.push_back(g);
          a.units.push_back(kUnit);
          a.hbm.push_back(per);
          if (!is_mine(g)) mine.push_back(g);
        }
      } else {
        int best = -1;
        double best_key = 1e300;
        for (size_t g = 0; g < used.size(); ++g) {
          const int64_t left = kUnit - used[g] - units;
          if (left < 0 || hbm_total_ - hbm_used[g] < hbm) continue;
          if (strict_pack && pack_gpu >= 0 && (int)g != pack_gpu) continue;
          if (strict_spread && is_mine((int)g)) continue;
          // best fit, with the group's own GPUs first (PACK) or last (SPREAD)
          const double pref = is_mine((int)g) ? (spread ? 1.0 : 0.0) : (spread ? 0.0 : 1.0);
          const double key = pref * 2.0 * kUnit + (double)left;
          if (key < best_key) {
            best_key = key;
            best = (int)g;
          }
        }
        if (best < 0) return py::none();
        used[best] += units;
        hbm_used[best] += hbm;
        a.gpus.push_back(best);
        a.units.push_back(units);
        a.hbm.push_back(hbm);
        got.push_back(best);
        if (!is_mine(best)) mine.push_back(best);
        if (strict_pack) pack_gpu = best;
      }
      per_bundle.push_back(got);
    }
    used_ = used;
    hbm_used_ = hbm_used;
    allocs_[owner] = a;
    py::dict d;
    d["gpus"] = mine;
    d["bundle_gpus"] = per_bundle;
    double frac = 0;
    for (auto u : a.units) frac += (double)u / kUnit;
    d["fraction"] = mine.size() == 1 ? std::min(1.0, frac) : (mine.empty() ? 0.0 : 1.0);
    return d;
  }
  bool release(const std::string& owner) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = allocs_.find(owner);
    if (it == allocs_.end()) return false;
    for (size_t i = 0; i < it->second.gpus.size(); ++i) {
      const int g = it->second.gpus[i];
      used_[g] = std::max<int64_t>(0, used_[g] - it->second.units[i]);
      hbm_used_[g] = std::max<int64_t>(0, hbm_used_[g] - it->second.hbm[i]);
    }
    allocs_.erase(it);
    return true;
  }
  py::list snapshot() {
    std::lock_guard<std::mutex> lk(mu_);
    py::list l;
    for (size_t g = 0; g < used_.size(); ++g) {
      py::dict d;
      d["gpu"] = (int)g;
      d["used"] = (double)used_[g] / kUnit;
      d["free"] = (double)(kUnit - used_[g]) / kUnit;
      d["hbm_used_gb"] = hbm_used_[g] / 1e9;
      d["hbm_free_gb"] = (hbm_total_ - hbm_used_[g]) / 1e9;
      py::dict holders;
      for (auto& kv : allocs_)
        for (size_t i = 0; i < kv.second.gpus.size(); ++i)
          if (kv.second.gpus[i] == (int)g) {
            const py::str k(kv.first);
            const double prev = holders.contains(k) ? holders[k].cast<double>() : 0.0;
            holders[k] = prev + (double)kv.second.units[i] / kUnit;
          }
      d["holders"] = holders;
      l.append(d);
    }
    return l;
  }
  int num_gpus() const { return (int)used_.size(); }
  std::string json() {
    std::lock_guard<std::mutex> lk(mu_);
    std::ostringstream o;
    o << "[";
    for (size_t g = 0; g < used_.size(); ++g) {
      if (g) o << ",";
      o << "{\"gpu\":" << g << ",\"used\":" << (double)used_[g] / kUnit
        << ",\"hbm_used_gb\":" << hbm_used_[g] / 1e9 << "}";
    }
    o << "]";
    return o.str();
  }

 private:
  struct Alloc {
    std::vector<int> gpus;
    std::vector<int64_t> units, hbm;
  };
  static py::dict to_py(const Alloc& a) {
    py::dict d;
    d["gpus"] = a.gpus;
    double frac = 0;
    for (auto u : a.units) frac += (double)u / kUnit;
    d["fraction"] = a.gpus.empty() ? 0.0 : (a.gpus.size() == 1 ? frac : 1.0);
    return d;
  }
  std::mutex mu_;
  std::vector<int64_t> used_, hbm_used_;
  int64_t hbm_total_;
  std::map<std::string, Alloc> allocs_;
};

// ---------------------------------------------------------------------------
// KV store: binary-safe records "<klen> <vlen>\n<key><value>\n", atomic rename.
// ---------------------------------------------------------------------------
class KvStore {
 public:
  explicit KvStore(std::string path) : path_(std::move(path)) { load(); }
  void put(const std::string& k, const std::string& v) {
    std::lock_guard<std::mutex> lk(mu_);
    data_[k] = v;
    persist();
  }
  std::optional<std::string> get(const std::string& k) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = data_.find(k);
    if (it == data_.end()) return std::nullopt;
    return it->second;
  }
  bool del(const std::string& k) {
    std::lock_guard<std::mutex> lk(mu_);
    const bool had = data_.erase(k) > 0;
    if (had) persist();
    return had;
  }
  std::vector<std::string> keys(const std::string& prefix) {
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<std::string> out;
    for (auto& kv : data_)
      if (kv.first.compare(0, prefix.size(), prefix) == 0) out.push_back(kv.first);
    return out;
  }
  const std::string& path() const { return path_; }

 private:
  void load() {
    if (path_.empty()) return;
    std::ifstream f(path_, std::ios::binary);
    if (!f) return;
    for (;;) {
      size_t kl = 0, vl = 0;
      if (!(f >> kl >> vl)) break;
      f.get();  // '\n'
      std::string k(kl, '\0'), v(vl, '\0');
      if (!f.read(&k[0], kl) || !f.read(&v[0], vl)) break;
      f.get();
      data_[k] = v;
    }
  }
  void persist() {
    if (path_.empty()) return;
    const std::string tmp = path_ + ".tmp." + std::to_string(getpid());
    {
      std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
      if (!f) throw std::runtime_error("kv: cannot write " + tmp);
      for (auto& kv : data_) {
        f << kv.first.size() << " " << kv.second.size() << "\n";
        f.write(kv.first.data(), kv.first.size());
        f.write(kv.second.data(), kv.second.size());
        f << "\n";
      }
      f.flush();
      if (!f) throw std::runtime_error("kv: write failed");
    }
    if (rename(tmp.c_str(), path_.c_str()) != 0) throw std::runtime_error("kv: rename failed");
  }
  std::string path_;
  std::mutex mu_;
  std::map<std::string, std::string> data_;
};

// ---------------------------------------------------------------------------
// Supervisor + control server.
// ---------------------------------------------------------------------------
enum ProcState { P_STARTING = 0, P_RUNNING = 1, P_BACKOFF = 2, P_EXITED = 3, P_STOPPED = 4 };
const char* state_name(int s) {
  static const char* n[] = {"STARTING", "RUNNING", "BACKOFF", "EXITED", "STOPPED"};
  return (s >= 0 && s <= 4) ? n[s] : "?";
}

struct Proc {
  int id = 0;
  std::string owner;
  std::vector<std::string> argv, env;
  std::string log_path;
  pid_t pid = -1;
  int state = P_STARTING;
  int restarts = 0;
  int max_restarts = -1;
  double backoff_initial_s = 0.5, backoff_max_s = 30.0, hb_timeout_s = 30.0;
  int64_t next_start_ns = 0, started_ns = 0;
  std::string last_exit;
  bool restart = true;
  Job* job = nullptr;
  int replica = -1;
  std::vector<uint32_t> queues;
  int group = 0;   // > 0: member of a gang-spawned process group (never restarts alone)
  int rank = -1;
  // CPU set the process starts pinned to (NUMA placement: the CPUs local to its
  // GPU, runtime/numa.py gpu_placement); every thread it starts inherits it
  std::vector<int> cpus;
  // SIGKILLed but not yet reaped: the monitor keeps calling waitpid on it and
  // the process (or its gang) restarts only once it is gone, so a new replica
  // never starts while the old one still holds its GPU memory
  pid_t zombie = -1;
};

// A gang of processes that live and die together: one tensor-parallel replica
// (rank 0 owns the replica slot in the job; ranks 1..N-1 follow it over RCCL).
// If ANY member exits (or rank 0 misses heartbeats) every member is killed, the
// replica's pending and in-flight requests are failed / re-dispatched once, the
// group's epoch is bumped (rendezvous keys of the old epoch, "tp/<owner>/...",
// are deleted from the KV) and the whole group restarts after a back-off.
// Reference: placement-group bundles of a Serve deployment
// (python/ray/serve/api.py:240-259) whose ranks rendezvous through a named
// store (collective_group/nccl_collective_group.py:555-577); Ray restarts the
// replica actor, this agent restarts the gang.
struct Group {
  int id = 0;
  std::string owner;
  std::vector<int> members;   // proc ids, rank order
  int epoch = 0;
  int state = 0;              // ProcState of the gang
  int restarts = 0;
  int max_restarts = -1;
  double backoff_initial_s = 0.5, backoff_max_s = 30.0;
  int64_t next_start_ns = 0;
  std::string last_exit;
  bool restart = true;
  Job* job = nullptr;
  int replica = -1;
  std::vector<uint32_t> queues;
};

class NodeAgent {
 public:
  NodeAgent(int num_gpus, double hbm_gb_per_gpu, const std::string& kv_path)
      : alloc_(num_gpus, hbm_gb_per_gpu > 0 ? hbm_gb_per_gpu : Config::instance().get_double("hbm_gb_per_gpu")),
        kv_(kv_path) {
    monitor_ = std::thread([this] { monitor_loop(); });
  }
  ~NodeAgent() { shutdown(5.0); }

  GpuAllocator& allocator() { return alloc_; }
  KvStore& kv() { return kv_; }

  int spawn(const std::string& owner, std::vector<std::string> argv, py::dict env_over,
            const std::string& log_path, const std::string& job_name, int replica,
            std::vector<uint32_t> queues, double hb_timeout_s, int max_restarts,
            double backoff_initial_s, double backoff_max_s, std::vector<int> cpus) {
    if (argv.empty()) throw std::invalid_argument("spawn: empty argv");
    auto p = std::make_unique<Proc>();
    p->owner = owner;
    p->argv = std::move(argv);
    std::map<std::string, std::string> env;
    for (char** e = environ; *e; ++e) {
      std::string kv(*e);
      auto eq = kv.find('=');
      if (eq != std::string::npos) env[kv.substr(0, eq)] = kv.substr(eq + 1);
    }
    for (auto item : env_over) {
      const std::string k = py::str(item.first);
      if (item.second.is_none()) env.erase(k);
      else env[k] = py::str(item.second);
    }
    for (auto& kv : env) p->env.push_back(kv.first + "=" + kv.second);
    p->log_path = log_path;
    p->replica = replica;
    p->queues = std::move(queues);
    p->hb_timeout_s = hb_timeout_s;
    p->max_restarts = max_restarts;
    p->backoff_initial_s = backoff_initial_s;
    p->backoff_max_s = backoff_max_s;
    p->cpus = std::move(cpus);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!job_name.empty()) p->job = attach_job(job_name);
      p->id = next_id_++;
      start_locked(*p);
      const int id = p->id;
      procs_[id] = std::move(p);
      return id;
    }
  }
  // Gang spawn (see Group): argvs / envs / logs per rank.  Every member gets
  // RDB_TP_RANK, RDB_TP_WORLD, RDB_TP_GROUP (= owner) and RDB_TP_EPOCH in its
  // environment; rank 0 carries the replica slot (heartbeats, queues).
  int spawn_group(const std::string& owner, std::vector<std::vector<std::string>> argvs,
                  std::vector<py::dict> envs, std::vector<std::string> logs, const std::string& job_name,
                  int replica, std::vector<uint32_t> queues, double hb_timeout_s, int max_restarts,
                  double backoff_initial_s, double backoff_max_s, std::vector<std::vector<int>> cpus) {
    const size_t n = argvs.size();
    if (n == 0) throw std::invalid_argument("spawn_group: no ranks");
    if (envs.size() != n || logs.size() != n) throw std::invalid_argument("spawn_group: argvs/envs/logs sizes differ");
    if (!cpus.empty() && cpus.size() != n) throw std::invalid_argument("spawn_group: cpus must list one set per rank");
    std::vector<std::unique_ptr<Proc>> ps;
    for (size_t r = 0; r < n; ++r) {
      if (argvs[r].empty()) throw std::invalid_argument("spawn_group: empty argv");
      auto p = std::make_unique<Proc>();
      p->owner = owner + "/rank" + std::to_string(r);
      p->argv = argvs[r];
      std::map<std::string, std::string> env;
      for (char** e = environ; *e; ++e) {
        std::string kv(*e);
        auto eq = kv.find('=');
        if (eq != std::string::npos) env[kv.substr(0, eq)] = kv.substr(eq + 1);
      }
      for (auto item : envs[r]) {
        const std::string k = py::str(item.first);
        if (item.second.is_none()) env.erase(k);
        else env[k] = py::str(item.second);
      }
      env["RDB_TP_RANK"] = std::to_string(r);
      env["RDB_TP_WORLD"] = std::to_string(n);
      env["RDB_TP_GROUP"] = owner;
      env["RDB_TP_EPOCH"] = "0";
      for (auto& kv : env) p->env.push_back(kv.first + "=" + kv.second);
      p->log_path = logs[r];
      p->replica = r == 0 ? replica : -1;
      if (r == 0) p->queues = queues;
      p->hb_timeout_s = r == 0 ? hb_timeout_s : 0.0;
      p->max_restarts = max_restarts;
      p->rank = (int)r;
      if (!cpus.empty()) p->cpus = cpus[r];
      ps.push_back(std::move(p));
    }
    std::lock_guard<std::mutex> lk(mu_);
    auto g = std::make_unique<Group>();
    g->id = next_group_++;
    g->owner = owner;
    g->max_restarts = max_restarts;
    g->backoff_initial_s = backoff_initial_s;
    g->backoff_max_s = backoff_max_s;
    g->replica = replica;
    g->queues = queues;
    if (!job_name.empty()) g->job = attach_job(job_name);
    for (auto& p : ps) {
      p->job = g->job;
      p->group = g->id;
      p->id = next_id_++;
      g->members.push_back(p->id);
      start_locked(*p);
      procs_[p->id] = std::move(p);
    }
    g->state = P_STARTING;
    const int gid = g->id;
    groups_[gid] = std::move(g);
    events_.emplace_back(gid, "group_started", owner);
    return gid;
  }
  // Stop a whole group for good.
  bool terminate_group(int gid, double grace_s) {
    std::vector<int> ids;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = groups_.find(gid);
      if (it == groups_.end()) return false;
      it->second->restart = false;
      it->second->state = P_STOPPED;
      ids = it->second->members;
    }
    bool ok = true;
    for (int id : ids) ok = terminate(id, grace_s) && ok;
    return ok;
  }
  py::dict group_info(int gid) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = groups_.find(gid);
    if (it == groups_.end()) throw std::out_of_range("unknown group id");
    const Group& g = *it->second;
    py::dict d;
    d["id"] = g.id;
    d["owner"] = g.owner;
    d["epoch"] = g.epoch;
    d["state"] = state_name(g.state);
    d["restarts"] = g.restarts;
    d["last_exit"] = g.last_exit;
    d["members"] = g.members;
    py::list pids;
    for (int id : g.members) {
      auto pit = procs_.find(id);
      pids.append(pit == procs_.end() ? -1 : (int)pit->second->pid);
    }
    d["pids"] = pids;
    return d;
  }
  // Stop a process for good (no restart): SIGTERM its group, SIGKILL after grace.
  bool terminate(int id, double grace_s) {
    pid_t pid;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = procs_.find(id);
      if (it == procs_.end()) return false;
      it->second->restart = false;
      pid = it->second->pid;
      if (pid <= 0) {
        it->second->state = P_STOPPED;
        return true;
      }
      kill(-pid, SIGTERM);
    }
    const int64_t deadline = now_ns() + (int64_t)(grace_s * 1e9);
    for (;;) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = procs_.find(id);
        if (it == procs_.end() || it->second->pid <= 0) return true;
      }
      if (now_ns() > deadline) break;
      usleep(5000);
    }
    kill(-pid, SIGKILL);
    for (int i = 0; i < 400; ++i) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = procs_.find(id);
        if (it == procs_.end() || it->second->pid <= 0) return true;
      }
      usleep(5000);
    }
    return false;
  }
  // Kill without disabling restart (chaos / fault injection: "replica killer").
  bool kill_proc(int id, int sig) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = procs_.find(id);
    if (it == procs_.end() || it->second->pid <= 0) return false;
    return kill(-it->second->pid, sig) == 0;
  }
  py::dict info(int id) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = procs_.find(id);
    if (it == procs_.end()) throw std::out_of_range("unknown process id");
    return info_locked(*it->second);
  }
  py::list list() {
    std::lock_guard<std::mutex> lk(mu_);
    py::list l;
    for (auto& kv : procs_) l.append(info_locked(*kv.second));
    return l;
  }
  py::list events() {
    std::lock_guard<std::mutex> lk(mu_);
    py::list l;
    for (auto& e : events_) l.append(py::make_tuple(std::get<0>(e), std::get<1>(e), std::get<2>(e)));
    events_.clear();
    return l;
  }
  void forget(int id) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = procs_.find(id);
    if (it != procs_.end() && it->second->pid <= 0) {
      if (it->second->zombie > 0) orphans_.push_back(it->second->zombie);   // still reaped by the monitor
      procs_.erase(it);
    }
  }
  // Drop a stopped gang and its members (a TP replica stopped or drained for
  // good); false while any member still runs.
  bool forget_group(int gid) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = groups_.find(gid);
    if (it == groups_.end()) return false;
    for (int id : it->second->members) {
      auto pit = procs_.find(id);
      if (pit != procs_.end() && pit->second->pid > 0) return false;
    }
    for (int id : it->second->members) {
      auto pit = procs_.find(id);
      if (pit == procs_.end()) continue;
      if (pit->second->zombie > 0) orphans_.push_back(pit->second->zombie);
      procs_.erase(pit);
    }
    groups_.erase(it);
    return true;
  }
  size_t num_groups() {
    std::lock_guard<std::mutex> lk(mu_);
    return groups_.size();
  }

  // -- control server
  void serve(const std::string& path) {
    if (server_.joinable()) throw std::runtime_error("control server already running");
    int fd = socket(AF_UNIX, SOCK_STREAM, 0);
    if (fd < 0) throw std::runtime_error("socket() failed");
    sockaddr_un addr{};
    addr.sun_family = AF_UNIX;
    if (path.size() >= sizeof(addr.sun_path)) throw std::invalid_argument("socket path too long");
    strncpy(addr.sun_path, path.c_str(), sizeof(addr.sun_path) - 1);
    unlink(path.c_str());
    if (bind(fd, (sockaddr*)&addr, sizeof(addr)) != 0 || listen(fd, 16) != 0) {
      close(fd);
      throw std::runtime_error("bind/listen failed on " + path);
    }
    sock_path_ = path;
    listen_fd_ = fd;
    server_ = std::thread([this] { server_loop(); });
  }
  std::string handle_command(const std::string& line) {
    std::istringstream in(line);
    std::string cmd;
    in >> cmd;
    if (cmd == "PING") return "PONG";
    if (cmd == "STATUS") return status_json();
    if (cmd == "KV_GET") {
      std::string k;
      in >> k;
      auto v = kv_.get(k);
      return v ? "OK " + *v : "NOTFOUND";
    }
    if (cmd == "KV_PUT") {
      std::string k;
      in >> k;
      std::string v;
      std::getline(in, v);
      if (!v.empty() && v[0] == ' ') v.erase(0, 1);
      kv_.put(k, v);
      return "OK";
    }
    if (cmd == "KV_DEL") {
      std::string k;
      in >> k;
      return kv_.del(k) ? "OK" : "NOTFOUND";
    }
    if (cmd == "KV_KEYS") {
      std::string prefix;
      in >> prefix;
      std::string o = "OK";
      for (auto& k : kv_.keys(prefix)) o += " " + k;
      return o;
    }
    if (cmd == "CONFIG") {
      std::string k;
      in >> k;
      try {
        return "OK " + Config::instance().get(k);
      } catch (const std::exception& e) {
        return std::string("ERR ") + e.what();
      }
    }
    return "ERR unknown command";
  }
  std::string status_json() {
    std::lock_guard<std::mutex> lk(mu_);
    std::ostringstream o;
    o << "{\"pid\":" << getpid() << ",\"gpus\":" << alloc_.json() << ",\"procs\":[";
    bool first = true;
    for (auto& kv : procs_) {
      const Proc& p = *kv.second;
      if (!first) o << ",";
      first = false;
      o << "{\"id\":" << p.id << ",\"owner\":\"" << json_escape(p.owner) << "\",\"pid\":" << p.pid
        << ",\"state\":\"" << state_name(p.state) << "\",\"restarts\":" << p.restarts
        << ",\"replica\":" << p.replica << ",\"last_exit\":\"" << json_escape(p.last_exit) << "\"}";
    }
    o << "]}";
    return o.str();
  }

  void shutdown(double grace_s) {
    if (stopped_.exchange(true)) return;
    std::vector<int> ids;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& kv : procs_) ids.push_back(kv.first);
    }
    {
      py::gil_scoped_release nogil;
      for (int id : ids) terminate(id, grace_s);
    }
    stop_.store(true);
    if (monitor_.joinable()) monitor_.join();
    if (server_.joinable()) server_.join();
    if (listen_fd_ >= 0) close(listen_fd_);
    if (!sock_path_.empty()) unlink(sock_path_.c_str());
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : jobs_) kv.second->close();
    jobs_.clear();
  }

 private:
  Job* attach_job(const std::string& name) {
    auto it = jobs_.find(name);
    if (it != jobs_.end()) return it->second.get();
    auto j = std::make_unique<Job>();
    j->attach(name, 5000000000LL);
    j->set_unlink_on_close(false);
    Job* raw = j.get();
    jobs_[name] = std::move(j);
    return raw;
  }
  void start_locked(Proc& p) {
    if (p.group > 0) {   // a (re)started gang member sees the group's current epoch
      auto git = groups_.find(p.group);
      if (git != groups_.end())
        for (auto& e : p.env)
          if (e.rfind("RDB_TP_EPOCH=", 0) == 0) e = "RDB_TP_EPOCH=" + std::to_string(git->second->epoch);
    }
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    if (!p.log_path.empty()) {
      posix_spawn_file_actions_addopen(&fa, 1, p.log_path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
      posix_spawn_file_actions_adddup2(&fa, 1, 2);
    }
    posix_spawnattr_t at;
    posix_spawnattr_init(&at);
    posix_spawnattr_setflags(&at, POSIX_SPAWN_SETPGROUP | POSIX_SPAWN_SETSIGMASK);
    posix_spawnattr_setpgroup(&at, 0);
    sigset_t none;
    sigemptyset(&none);
    posix_spawnattr_setsigmask(&at, &none);
    std::vector<char*> av, ev;
    for (auto& a : p.argv) av.push_back(const_cast<char*>(a.c_str()));
    av.push_back(nullptr);
    for (auto& e : p.env) ev.push_back(const_cast<char*>(e.c_str()));
    ev.push_back(nullptr);
    if (p.job && p.replica >= 0 && (uint32_t)p.replica < p.job->hdr()->n_replicas) {
      ReplicaState* rs = p.job->replica(p.replica);
      rs->heartbeat_ns.store(now_ns());
      rs->status.store(RS_STARTING);
    }
    // NUMA placement: the child inherits the CPU mask of the thread that spawns
    // it, so pin THIS thread to the child's set around the spawn (race-free: the
    // mask is in place before the child runs a single instruction)
    cpu_set_t saved, want;
    bool pinned = false;
    if (!p.cpus.empty()) {
      CPU_ZERO(&want);
      for (int c : p.cpus)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &want);
      if (pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) == 0 &&
          pthread_setaffinity_np(pthread_self(), sizeof(want), &want) == 0)
        pinned = true;
      else
        events_.emplace_back(p.id, "pin_failed", "cannot apply the CPU set; starting unpinned");
    }
    pid_t pid = -1;
    const int rc = posix_spawnp(&pid, av[0], &fa, &at, av.data(), ev.data());
    if (pinned) pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
    posix_spawn_file_actions_destroy(&fa);
    posix_spawnattr_destroy(&at);
    if (rc != 0) {
      p.pid = -1;
      p.state = P_EXITED;
      p.last_exit = std::string("spawn failed: ") + strerror(rc);
      events_.emplace_back(p.id, "spawn_failed", p.last_exit);
      return;
    }
    p.pid = pid;
    p.state = P_STARTING;
    p.started_ns = now_ns();
    events_.emplace_back(p.id, "started", std::to_string(pid));
  }
  void on_death_locked(Proc& p, const std::string& why) {
    p.pid = -1;
    p.last_exit = why;
    if (p.job && p.replica >= 0 && (uint32_t)p.replica < p.job->hdr()->n_replicas) {
      ReplicaState* rs = p.job->replica(p.replica);
      rs->status.store(RS_DEAD);
      for (uint32_t q : p.queues)
        if (q < p.job->hdr()->n_queues) {
          fail_pending(*p.job, q, ST_REPLICA_DIED);
          forget_inflight(*p.job, q);
        }
      rs->restarts.fetch_add(1);  // generation bump: routers reap requests lost in flight
    }
    if (!p.restart || stopped_.load()) {
      p.state = P_STOPPED;
      events_.emplace_back(p.id, "stopped", why);
      return;
    }
    if (p.max_restarts >= 0 && p.restarts >= p.max_restarts) {
      p.state = P_EXITED;
      events_.emplace_back(p.id, "exited", why);
      return;
    }
    ++p.restarts;
    const double back = std::min(p.backoff_max_s, p.backoff_initial_s * std::pow(2.0, std::min(p.restarts - 1, 20)));
    p.next_start_ns = now_ns() + (int64_t)(back * 1e9);
    p.state = P_BACKOFF;
    events_.emplace_back(p.id, "died", why + "; restart in " + std::to_string(back) + " s");
  }
  // A member of gang g died (or was killed for missed heartbeats): take the
  // whole gang down, fail the replica's requests once, bump the epoch and
  // schedule the gang's restart.
  void group_death_locked(int gid, Proc& dead, const std::string& why) {
    auto it = groups_.find(gid);
    if (it == groups_.end()) return;
    Group& g = *it->second;
    dead.pid = -1;
    dead.last_exit = why;
    // SIGKILL every member, never wait here (mu_ is held: every agent call,
    // KV rendezvous polls included, would stall for the members' exit); the
    // monitor reaps them (Proc::zombie) and the gang restarts only after that
    for (int id : g.members) {
      auto pit = procs_.find(id);
      if (pit == procs_.end() || pit->second->pid <= 0) continue;
      Proc& m = *pit->second;
      kill(-m.pid, SIGKILL);
      int st = 0;
      if (waitpid(m.pid, &st, WNOHANG) != m.pid) m.zombie = m.pid;
      m.pid = -1;
      m.last_exit = "killed with its group (rank " + std::to_string(dead.rank) + ": " + why + ")";
    }
    if (g.job && g.replica >= 0 && (uint32_t)g.replica < g.job->hdr()->n_replicas) {
      ReplicaState* rs = g.job->replica(g.replica);
      rs->status.store(RS_DEAD);
      for (uint32_t q : g.queues)
        if (q < g.job->hdr()->n_queues) {
          fail_pending(*g.job, q, ST_REPLICA_DIED);
          forget_inflight(*g.job, q);
        }
      rs->restarts.fetch_add(1);  // generation bump: routers re-dispatch what was in flight
    }
    ++g.epoch;
    for (auto& k : kv_.keys("tp/" + g.owner + "/")) kv_.del(k);
    g.last_exit = "rank " + std::to_string(dead.rank) + ": " + why;
    const bool again = g.restart && !stopped_.load() && !(g.max_restarts >= 0 && g.restarts >= g.max_restarts);
    int st_new = P_STOPPED;
    if (again) {
      ++g.restarts;
      const double back = std::min(g.backoff_max_s, g.backoff_initial_s * std::pow(2.0, std::min(g.restarts - 1, 20)));
      g.next_start_ns = now_ns() + (int64_t)(back * 1e9);
      st_new = P_BACKOFF;
      events_.emplace_back(g.id, "group_died", g.last_exit + "; restart in " + std::to_string(back) + " s");
    } else {
      st_new = g.restart ? P_EXITED : P_STOPPED;
      events_.emplace_back(g.id, "group_stopped", g.last_exit);
    }
    g.state = st_new;
    for (int id : g.members) {
      auto pit = procs_.find(id);
      if (pit == procs_.end()) continue;
      pit->second->state = st_new;
      pit->second->restarts = g.restarts;
    }
  }
  void monitor_loop() {
    const int interval_ms = std::max(1, (int)Config::instance().get_double("agent_monitor_interval_ms"));
    while (!stop_.load()) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        const int64_t now = now_ns();
        auto gone = [](pid_t z) {
          int st = 0;
          const pid_t w = waitpid(z, &st, WNOHANG);
          return w == z || (w < 0 && errno == ECHILD);
        };
        orphans_.erase(std::remove_if(orphans_.begin(), orphans_.end(), gone), orphans_.end());
        for (auto& kv : procs_) {
          Proc& p = *kv.second;
          if (p.zombie > 0 && gone(p.zombie)) p.zombie = -1;
          if (p.pid > 0) {
            int st = 0;
            const pid_t r = waitpid(p.pid, &st, WNOHANG);
            if (r == p.pid) {
              std::string why = WIFEXITED(st) ? "exit code " + std::to_string(WEXITSTATUS(st))
                                              : "signal " + std::to_string(WTERMSIG(st));
              kill(-p.pid, SIGKILL);  // reap stragglers of its process group
              if (p.group > 0) group_death_locked(p.group, p, why);
              else on_death_locked(p, why);
              continue;
            }
            if (p.job && p.replica >= 0 && (uint32_t)p.replica < p.job->hdr()->n_replicas) {
              ReplicaState* rs = p.job->replica(p.replica);
              const uint32_t s = rs->status.load();
              if (s == RS_READY) p.state = P_RUNNING;
              const double age = (now - rs->heartbeat_ns.load()) / 1e9;
              if (p.state == P_RUNNING && p.hb_timeout_s > 0 && age > p.hb_timeout_s) {
                kill(-p.pid, SIGKILL);
                int st2 = 0;
                if (waitpid(p.pid, &st2, WNOHANG) != p.pid) p.zombie = p.pid;   // reaped below, not waited for here
                const std::string why = "missed heartbeats for " + std::to_string(age) + " s";
                if (p.group > 0) group_death_locked(p.group, p, why);
                else on_death_locked(p, why);
              }
            } else if (p.state == P_STARTING) {
              p.state = P_RUNNING;
            }
          } else if (p.group == 0 && p.state == P_BACKOFF && now >= p.next_start_ns && p.zombie <= 0) {
            start_locked(p);
          }
        }
        for (auto& gkv : groups_) {   // gangs restart together
          Group& g = *gkv.second;
          if (g.state == P_STARTING) {
            bool all = true;
            for (int id : g.members) {
              auto pit = procs_.find(id);
              all = all && pit != procs_.end() && pit->second->state == P_RUNNING;
            }
            if (all) g.state = P_RUNNING;
          }
          if (g.state != P_BACKOFF || now < g.next_start_ns) continue;
          bool reaped = true;   // every old member gone (its VRAM released) before the gang restarts
          for (int id : g.members) {
            auto pit = procs_.find(id);
            reaped = reaped && (pit == procs_.end() || pit->second->zombie <= 0);
          }
          if (!reaped) continue;
          for (int id : g.members) {
            auto pit = procs_.find(id);
            if (pit != procs_.end()) start_locked(*pit->second);
          }
          g.state = P_STARTING;
          events_.emplace_back(g.id, "group_restarted", "epoch " + std::to_string(g.epoch));
        }
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(interval_ms));
    }
  }
  void server_loop() {
    while (!stop_.load()) {
      pollfd pfd{listen_fd_, POLLIN, 0};
      if (poll(&pfd, 1, 100) <= 0) continue;
      int c = accept(listen_fd_, nullptr, nullptr);
      if (c < 0) continue;
      std::string line;
      char buf[4096];
      for (;;) {
        pollfd cp{c, POLLIN, 0};
        if (poll(&cp, 1, 1000) <= 0) break;
        ssize_t n = read(c, buf, sizeof(buf));
        if (n <= 0) break;
        line.append(buf, (size_t)n);
        if (line.find('\n') != std::string::npos) break;
        if (line.size() > (1u << 20)) break;
      }
      auto nl = line.find('\n');
      if (nl != std::string::npos) line.resize(nl);
      std::string resp;
      try {
        resp = handle_command(line);
      } catch (const std::exception& e) {
        resp = std::string("ERR ") + e.what();
      }
      resp += "\n";
      size_t off = 0;
      while (off < resp.size()) {
        ssize_t w = write(c, resp.data() + off, resp.size() - off);
        if (w <= 0) break;
        off += (size_t)w;
      }
      close(c);
    }
  }
  py::dict info_locked(const Proc& p) {
    py::dict d;
    d["id"] = p.id;
    d["owner"] = p.owner;
    d["pid"] = (int)p.pid;
    d["state"] = state_name(p.state);
    d["restarts"] = p.restarts;
    d["last_exit"] = p.last_exit;
    d["replica"] = p.replica;
    d["uptime_s"] = p.pid > 0 ? (now_ns() - p.started_ns) / 1e9 : 0.0;
    return d;
  }

  GpuAllocator alloc_;
  KvStore kv_;
  std::mutex mu_;
  std::map<int, std::unique_ptr<Proc>> procs_;
  std::map<int, std::unique_ptr<Group>> groups_;
  int next_group_ = 1;
  std::map<std::string, std::unique_ptr<Job>> jobs_;
  std::deque<std::tuple<int, std::string, std::string>> events_;
  int next_id_ = 1;
  std::atomic<bool> stop_{false}, stopped_{false};
  std::thread monitor_, server_;
  int listen_fd_ = -1;
  std::string sock_path_;
  std::vector<pid_t> orphans_;   // killed processes of forgotten entries, still to be reaped
};

// Client side of the control protocol (CLI / other processes).
std::string agent_request(const std::string& path, const std::string& line, double timeout_s) {
  int fd = socket(AF_UNIX, SOCK_STREAM, 0);
  if (fd < 0) throw std::runtime_error("socket() failed");
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  strncpy(addr.sun_path, path.c_str(), sizeof(addr.sun_path) - 1);
  if (connect(fd, (sockaddr*)&addr, sizeof(addr)) != 0) {
    close(fd);
    throw std::runtime_error("cannot connect to node agent at " + path);
  }
  std::string msg = line + "\n";
  if (write(fd, msg.data(), msg.size()) != (ssize_t)msg.size()) {
    close(fd);
    throw std::runtime_error("write failed");
  }
  std::string out;
  char buf[4096];
  const int64_t deadline = now_ns() + (int64_t)(timeout_s * 1e9);
  while (out.find('\n') == std::string::npos) {
    const int left_ms = (int)std::max<int64_t>(1, (deadline - now_ns()) / 1000000);
    pollfd p{fd, POLLIN, 0};
    if (poll(&p, 1, left_ms) <= 0) break;
    ssize_t n = read(fd, buf, sizeof(buf));
    if (n <= 0) break;
    out.append(buf, (size_t)n);
  }
  close(fd);
  auto nl = out.find('\n');
  if (nl == std::string::npos) throw std::runtime_error("node agent did not answer");
  out.resize(nl);
  return out;
}

}  // namespace agent

void register_node_agent(py::module_& m) {
  using namespace agent;
  m.def("config_define", [](const std::string& n, const std::string& t, const std::string& d, const std::string& h) {
    return Config::instance().define(n, t, d, h);
  });
  m.def("config_get", [](const std::string& n) { return Config::instance().get(n); });
  m.def("config_set", [](const std::string& n, const std::string& v) { Config::instance().set(n, v); });
  m.def("config_all", []() { return Config::instance().all(); });
  m.def("agent_request", &agent_request, py::arg("path"), py::arg("line"), py::arg("timeout_s") = 5.0,
        py::call_guard<py::gil_scoped_release>());

  py::class_<GpuAllocator>(m, "GpuAllocator")
      .def(py::init<int, double>(), py::arg("num_gpus"), py::arg("hbm_gb_per_gpu") = 288.0)
      .def("allocate", &GpuAllocator::allocate, py::arg("owner"), py::arg("num_gpus"), py::arg("hbm_gb") = 0.0)
      .def("allocate_bundles", &GpuAllocator::allocate_bundles, py::arg("owner"), py::arg("bundles"),
           py::arg("strategy") = "PACK")
      .def("release", &GpuAllocator::release)
      .def("snapshot", &GpuAllocator::snapshot)
      .def_property_readonly("num_gpus", &GpuAllocator::num_gpus);

  py::class_<KvStore>(m, "KvStore")
      .def(py::init<std::string>())
      .def("put", [](KvStore& k, const std::string& key, py::bytes v) { k.put(key, std::string(v)); })
      .def("get", [](KvStore& k, const std::string& key) -> py::object {
        auto v = k.get(key);
        if (!v) return py::none();
        return py::bytes(*v);
      })
      .def("delete", &KvStore::del)
      .def("keys", &KvStore::keys, py::arg("prefix") = "")
      .def_property_readonly("path", &KvStore::path);

  py::class_<NodeAgent>(m, "NodeAgent")
      .def(py::init<int, double, const std::string&>(), py::arg("num_gpus"), py::arg("hbm_gb_per_gpu") = 0.0,
           py::arg("kv_path") = "")
      .def("allocate", [](NodeAgent& a, const std::string& o, double g, double h) { return a.allocator().allocate(o, g, h); },
           py::arg("owner"), py::arg("num_gpus"), py::arg("hbm_gb") = 0.0)
      .def("release", [](NodeAgent& a, const std::string& o) { return a.allocator().release(o); })
      .def("allocate_bundles",
           [](NodeAgent& a, const std::string& o, const std::vector<std::pair<double, double>>& b,
              const std::string& st) { return a.allocator().allocate_bundles(o, b, st); },
           py::arg("owner"), py::arg("bundles"), py::arg("strategy") = "PACK")
      .def("resources", [](NodeAgent& a) { return a.allocator().snapshot(); })
      .def("kv_put", [](NodeAgent& a, const std::string& k, py::bytes v) { a.kv().put(k, std::string(v)); })
      .def("kv_get", [](NodeAgent& a, const std::string& k) -> py::object {
        auto v = a.kv().get(k);
        if (!v) return py::none();
        return py::bytes(*v);
      })
      .def("kv_delete", [](NodeAgent& a, const std::string& k) { return a.kv().del(k); })
      .def("kv_keys", [](NodeAgent& a, const std::string& p) { return a.kv().keys(p); }, py::arg("prefix") = "")
      .def("spawn", &NodeAgent::spawn, py::arg("owner"), py::arg("argv"), py::arg("env") = py::dict(),
           py::arg("log_path") = "", py::arg("job") = "", py::arg("replica") = -1,
           py::arg("queues") = std::vector<uint32_t>{}, py::arg("health_timeout_s") = 30.0,
           py::arg("max_restarts") = -1, py::arg("backoff_initial_s") = 0.5, py::arg("backoff_max_s") = 30.0,
           py::arg("cpus") = std::vector<int>{})
      .def("terminate", &NodeAgent::terminate, py::arg("id"), py::arg("grace_s") = 5.0,
           py::call_guard<py::gil_scoped_release>())
      .def("spawn_group", &NodeAgent::spawn_group, py::arg("owner"), py::arg("argvs"), py::arg("envs"),
           py::arg("logs"), py::arg("job") = "", py::arg("replica") = -1,
           py::arg("queues") = std::vector<uint32_t>{}, py::arg("health_timeout_s") = 30.0,
           py::arg("max_restarts") = -1, py::arg("backoff_initial_s") = 0.5, py::arg("backoff_max_s") = 30.0,
           py::arg("cpus") = std::vector<std::vector<int>>{})
      .def("forget_group", &NodeAgent::forget_group, py::arg("group"))
      .def("num_groups", &NodeAgent::num_groups)
      .def("terminate_group", &NodeAgent::terminate_group, py::arg("group"), py::arg("grace_s") = 5.0,
           py::call_guard<py::gil_scoped_release>())
      .def("group_info", &NodeAgent::group_info)
      .def("kill", &NodeAgent::kill_proc, py::arg("id"), py::arg("sig") = 9)
      .def("info", &NodeAgent::info)
      .def("list", &NodeAgent::list)
      .def("events", &NodeAgent::events)
      .def("forget", &NodeAgent::forget)
      .def("serve", &NodeAgent::serve)
      .def("handle_command", &NodeAgent::handle_command)
      .def("status_json", &NodeAgent::status_json)
      .def("shutdown", &NodeAgent::shutdown, py::arg("grace_s") = 5.0);
}

}  // namespace rdb
