// Host-only stress test of the shm job segment for the sanitizer presets
// (SURVEY §5.2): P producer threads submit into one request ring, a consumer
// thread batches, peeks/commits and answers through per-producer completion
// rings, the trace ring and the seqlock snapshot are hammered concurrently.
// Built with -fsanitize=thread / -fsanitize=address,undefined by
// tests/test_sanitizers.py; exits non-zero on any lost, duplicated or
// corrupted message.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../shm.h"

using namespace rdb::rt;

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 4;
  const int N = argc > 2 ? atoi(argv[2]) : 20000;
  JobConfig cfg;
  cfg.n_replicas = 1;
  cfg.n_queues = 1;
  cfg.n_clients = (uint32_t)P;
  cfg.req_capacity = 256;
  cfg.req_slot_bytes = 64;
  cfg.cmp_capacity = 256;
  cfg.cmp_slot_bytes = 64;
  const std::string name = "ring_stress_" + std::to_string(getpid());
  Job job;
  job.create(name, cfg);
  std::atomic<bool> fail{false};
  std::atomic<int> done_producers{0};

  std::thread consumer([&] {
    Ring r = job.req_ring(0);
    uint64_t pos = 0;
    uint64_t seen = 0;
    const uint64_t total = (uint64_t)P * N;
    while (seen < total && !fail.load()) {
      uint64_t n = 0;
      while (n < 16) {
        SlotHeader* s = r.peek(pos + n);
        if (!s) break;
        ++n;
      }
      if (!n) {
        r.wait_for(pos, 1000000, 100);
        continue;
      }
      for (uint64_t i = 0; i < n; ++i) {
        SlotHeader* s = r.slot(pos + i);
        uint64_t v;
        memcpy(&v, r.payload(s), sizeof(v));
        if (v != s->req_id * 7 + 3) fail.store(true);
        Ring c = job.cmp_ring(s->client);
        uint64_t cp;
        SlotHeader* o;
        while ((o = c.reserve(&cp)) == nullptr) std::this_thread::yield();
        o->req_id = s->req_id;
        o->len = 8;
        o->client = s->client;
        memcpy(c.payload(o), &v, 8);
        c.publish(o, cp);
      }
      pos += n;
      r.commit(pos);
      seen += n;
      job.trace(0)->record(TK_GPU, 1, 2, 0, (uint32_t)n, (uint32_t)n);
    }
  });

  std::thread snap_writer([&] {
    char buf[256];
    for (int i = 0; done_producers.load() < P; ++i) {
      int len = snprintf(buf, sizeof(buf), "{\"v\":%d,\"pad\":\"%0200d\"}", i, i);
      job.snapshot()->publish(buf, (uint32_t)len);
    }
  });
  std::thread snap_reader([&] {
    std::string out;
    while (done_producers.load() < P) {
      if (job.snapshot()->read(out) && (out.empty() || out.front() != '{' || out.back() != '}')) fail.store(true);
    }
  });

  std::vector<std::thread> prods;
  for (int p = 0; p < P; ++p) {
    prods.emplace_back([&, p] {
      Ring r = job.req_ring(0);
      Ring c = job.cmp_ring((uint32_t)p);
      uint64_t cpos = 0;
      int sent = 0, got = 0;
      while (got < N && !fail.load()) {
        if (sent < N) {
          uint64_t pos;
          if (SlotHeader* s = r.reserve(&pos)) {
            s->req_id = job.hdr()->next_req_id.fetch_add(1);
            s->client = (uint16_t)p;
            s->len = 8;
            const uint64_t v = s->req_id * 7 + 3;
            memcpy(r.payload(s), &v, 8);
            r.publish(s, pos);
            ++sent;
          }
        }
        while (SlotHeader* o = c.peek(cpos)) {
          uint64_t v;
          memcpy(&v, c.payload(o), 8);
          if (v != o->req_id * 7 + 3) fail.store(true);
          ++cpos;
          ++got;
          c.commit(cpos);
        }
      }
      done_producers.fetch_add(1);
    });
  }
  for (auto& t : prods) t.join();
  consumer.join();
  snap_writer.join();
  snap_reader.join();
  const bool ok = !fail.load() && job.trace(0)->head.load() > 0;
  job.close();
  printf("%s: %d producers x %d messages\n", ok ? "OK" : "FAIL", P, N);
  return ok ? 0 : 1;
}
