// ThreadSanitizer harness of the loopback communicator's host side (pkdtree/loopback.hpp,
// tests/test_sanitizers.py): P threads run the same random sequence of all-gathers, SUM / MIN
// reductions and all-to-all-v's with random sizes (zero-byte messages included) through one
// Hub, and every result is checked against the value computed directly; then one rank stops
// arriving and the others must get the barrier's deadline error instead of hanging. The GPU
// side of ThreadComm only adds stream-synchronised device copies around these calls.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <random>
#include <stdexcept>
#include <thread>
#include <vector>

#include "pkdtree/loopback.hpp"

using pkdtree::loopback::Hub;

namespace {

std::atomic<int> failures{0};

void check(bool ok, const char* what, int rank, int round) {
  if (!ok) {
    std::fprintf(stderr, "FAIL %s: rank %d round %d\n", what, rank, round);
    failures.fetch_add(1);
  }
}

// value rank r contributes at (round, i): every rank can recompute every other rank's data
uint32_t val(int r, int round, size_t i) { return uint32_t(r * 1000003u + round * 7919u + i * 31u + 17u); }

void run_rank(Hub& hub, int rank, int rounds, uint64_t seed) {
  const int P = hub.size();
  std::mt19937_64 rng(seed);  // same seed on every rank: the same sequence of collectives
  for (int round = 0; round < rounds; ++round) {
    const int op = int(rng() % 3);
    if (op == 0) {  // all-gather of a random (shared) size
      const size_t n = size_t(rng() % 64);
      std::vector<uint32_t> mine(n);
      for (size_t i = 0; i < n; ++i) mine[i] = val(rank, round, i);
      std::vector<char> out;
      hub.allgather(rank, mine.data(), n * 4, &out);
      const uint32_t* o = reinterpret_cast<const uint32_t*>(out.data());
      bool ok = out.size() == n * 4 * size_t(P);
      for (int r = 0; ok && r < P; ++r)
        for (size_t i = 0; i < n; ++i) ok = ok && o[size_t(r) * n + i] == val(r, round, i);
      check(ok, "allgather", rank, round);
    } else if (op == 1) {  // SUM and MIN reductions
      const size_t n = size_t(rng() % 32);
      std::vector<uint32_t> mine(n), out;
      for (size_t i = 0; i < n; ++i) mine[i] = val(rank, round, i) & 0xffffu;
      hub.reduce<uint32_t>(rank, mine.data(), n, [](uint32_t a, uint32_t b) { return a + b; }, &out);
      bool ok = out.size() == n;
      for (size_t i = 0; ok && i < n; ++i) {
        uint32_t s = 0;
        for (int r = 0; r < P; ++r) s += val(r, round, i) & 0xffffu;
        ok = out[i] == s;
      }
      check(ok, "reduce sum", rank, round);
      std::vector<int64_t> m(n), mo;
      for (size_t i = 0; i < n; ++i) m[i] = int64_t(val(rank, round, i) % 977u) - 400;
      hub.reduce<int64_t>(rank, m.data(), n, [](int64_t a, int64_t b) { return a < b ? a : b; }, &mo);
      ok = mo.size() == n;
      for (size_t i = 0; ok && i < n; ++i) {
        int64_t v = INT64_MAX;
        for (int r = 0; r < P; ++r) v = std::min<int64_t>(v, int64_t(val(r, round, i) % 977u) - 400);
        ok = mo[i] == v;
      }
      check(ok, "reduce min", rank, round);
    } else {  // all-to-all-v: rank p sends cnt(p, q) words to q (a size every rank derives)
      const uint64_t salt = rng();
      auto cnt = [&](int p, int q) { return size_t((salt >> ((p * 7 + q * 3) % 56)) % 9); };
      std::vector<size_t> sb(static_cast<size_t>(P)), so(sb), rb(sb), ro(sb);
      size_t st = 0, rt = 0;
      for (int q = 0; q < P; ++q) {
        sb[size_t(q)] = cnt(rank, q) * 4;
        so[size_t(q)] = st;
        st += sb[size_t(q)];
        rb[size_t(q)] = cnt(q, rank) * 4;
        ro[size_t(q)] = rt;
        rt += rb[size_t(q)];
      }
      std::vector<uint32_t> send(st / 4), recv(rt / 4, 0xdeadbeefu);
      for (int q = 0; q < P; ++q)
        for (size_t i = 0; i < cnt(rank, q); ++i) send[so[size_t(q)] / 4 + i] = val(rank, round, size_t(q) * 64 + i);
      hub.alltoallv(rank, send.data(), sb.data(), so.data(), recv.data(), rb.data(), ro.data());
      bool ok = true;
      for (int p = 0; p < P; ++p)
        for (size_t i = 0; i < cnt(p, rank); ++i) ok = ok && recv[ro[size_t(p)] / 4 + i] == val(p, round, size_t(rank) * 64 + i);
      check(ok, "alltoallv", rank, round);
    }
  }
}

}  // namespace

int main() {
  for (int P : {1, 2, 3, 5, 8}) {
    Hub hub(P);
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r) th.emplace_back([&, r] { run_rank(hub, r, 300, 1234 + P); });
    for (auto& t : th) t.join();
  }
  // a rank that never arrives: every other rank gets the deadline error, nobody hangs
  {
    Hub hub(3, 0.2);
    std::atomic<int> timed_out{0};
    std::vector<std::thread> th;
    for (int r = 0; r < 2; ++r)
      th.emplace_back([&] {
        try {
          hub.barrier();
        } catch (const std::runtime_error&) {
          timed_out.fetch_add(1);
        }
      });
    for (auto& t : th) t.join();
    check(timed_out.load() == 2, "barrier deadline", -1, 0);
  }
  if (failures.load()) return 1;
  std::printf("tsan loopback ok\n");
  return 0;
}
