// Host-only check of host_parallel's persistent pool (runtime.hpp HostPool) and par_sort: every range runs exactly once, nested
// calls and concurrent callers (threads of one process, as shard.LocalGroup's ranks) fall back to their own
// threads, and a forked child gets a working pool.  Built by tests/test_host_pool_cpu.py; no GPU call is made.
#include <sys/wait.h>

#include <atomic>
#include <cstdio>

#include "../../siddhi_amd/csrc/runtime.hpp"

static int check(int rounds) {
  for (int r = 0; r < rounds; r++) {
    const int nth = 2 + r % 15;
    std::vector<std::atomic<int>> hit(nth);
    for (auto& h : hit) h = 0;
    std::atomic<int> inner{0};
    sg::host_parallel(nth, [&](int t) {
      hit[t]++;
      if (t == 1 && r % 7 == 0) sg::host_parallel(3, [&](int) { inner++; });   // nested: own threads
    });
    for (int t = 0; t < nth; t++)
      if (hit[t] != 1) { std::printf("range %d ran %d times (round %d)\n", t, (int)hit[t], r); return 1; }
    if (r % 7 == 0 && inner != 3) { std::printf("nested call ran %d ranges\n", (int)inner); return 1; }
  }
  return 0;
}

// par_sort: the same order as std::sort under a total order, for range counts that leave odd runs
static int check_sort() {
  uint64_t x = 88172645463325252ull;
  for (int nth : {2, 3, 5, 16}) {
    for (int64_t n : {0, 1, 4095, 4096, 100003}) {
      std::vector<std::pair<uint32_t, uint32_t>> v((size_t)n);
      for (int64_t i = 0; i < n; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v[(size_t)i] = {(uint32_t)(x % 1000), (uint32_t)i}; }
      auto w = v;
      sg::par_sort(v, [](const auto& a, const auto& b) { return a < b; }, nth);
      std::sort(w.begin(), w.end());
      if (v != w) { std::printf("par_sort differs (n=%ld nth=%d)\n", (long)n, nth); return 1; }
    }
  }
  return 0;
}

int main() {
  if (check_sort()) return 1;
  if (check(2000)) return 1;
  std::atomic<int> bad{0};
  std::vector<std::thread> callers;
  for (int c = 0; c < 4; c++) callers.emplace_back([&] { bad += check(500); });
  for (auto& t : callers) t.join();
  if (bad) return 1;
  const pid_t pid = fork();
  if (pid == 0) _exit(check(200));
  int st = 0;
  waitpid(pid, &st, 0);
  if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) { std::printf("forked child failed\n"); return 1; }
  std::printf("host pool ok\n");
  return 0;
}
