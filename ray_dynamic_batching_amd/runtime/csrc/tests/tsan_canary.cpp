// Deliberate data race (tests/test_sanitizers.py only, never part of the
// runtime): proves that an instrumented extension dlopen-ed by the sanitized
// CPython launcher has its races reported -- i.e. that a clean run of the
// runtime suites means something.
#include <thread>

static long counter = 0;

extern "C" long rdb_tsan_canary(int iters) {
  auto bump = [iters] {
    for (int i = 0; i < iters; ++i) counter = counter + 1;   // unsynchronised read-modify-write
  };
  std::thread a(bump), b(bump);
  a.join();
  b.join();
  return counter;
}
