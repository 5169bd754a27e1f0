// Host-sanitizer run of the shared-memory transport.
//
// This file and csrc/host/shm_comm.cpp are built with
// -fsanitize=address,undefined (host code only: GPU sanitizers are not
// available on this pool, and the transport is where the host-side pointer
// arithmetic lives). W forked ranks rendezvous through a c10d FileStore and run
// every collective of the transport on known data, with message sizes around
// the (deliberately small) slot and ring sizes so chunking, slot-set alternation
// and ring wrap-around all run. Exit status 0 = every rank passed every check;
// a sanitizer report aborts the rank. Driven by tests/test_sanitizers.py.
#include <sys/wait.h>
#include <unistd.h>
#include <torch/csrc/distributed/c10d/FileStore.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "host/shm_comm.h"

namespace {

using Op = c10d::ReduceOp::RedOpType;
using pdcc::host::ShmComm;

int g_rank = -1;
int g_fail = 0;

template <class T, class F>
void expect(const char* what, size_t n, const T* got, F want) {
  size_t bad = 0, first = 0;
  for (size_t i = 0; i < n; ++i)
    if (!(got[i] == want(i)) && bad++ == 0) first = i;
  if (bad) {
    ++g_fail;
    std::fprintf(stderr, "[rank %d] %s: %zu of %zu wrong (first at %zu)\n", g_rank, what, bad, n, first);
  }
}

int run(const std::string& path, int rank, int world) {
  g_rank = rank;
  auto store = c10::make_intrusive<c10d::FileStore>(path, world);
  pdcc::host::ShmConfig cfg;
  cfg.slot_bytes = 64u << 10;  // small slots and rings: many chunks, ring wrap-around
  cfg.chan_bytes = 16u << 10;
  cfg.spin_us = 50;
  cfg.timeout = std::chrono::seconds(60);
  ShmComm c(store, "san", rank, world, cfg);
  const auto to = std::chrono::milliseconds(60000);
  const double tri = world * (world + 1) / 2.0;

  for (const size_t n : {size_t{1}, size_t{1000}, size_t{16411}, size_t{40000}}) {
    std::vector<float> f(n);
    for (size_t i = 0; i < n; ++i) f[i] = float(rank + 1 + i % 5);
    c.allreduce(f.data(), n, at::kFloat, Op::SUM, to);
    expect("allreduce/sum", n, f.data(), [&](size_t i) { return float(tri + world * double(i % 5)); });

    std::vector<int64_t> p(n, rank + 2);
    c.allreduce(p.data(), n, at::kLong, Op::PRODUCT, to);
    int64_t prod = 1;
    for (int r = 0; r < world; ++r) prod *= r + 2;
    expect("allreduce/prod", n, p.data(), [&](size_t) { return prod; });

    std::vector<double> m(n);
    for (size_t i = 0; i < n; ++i) m[i] = double((rank * 7 + i) % world);
    c.allreduce(m.data(), n, at::kDouble, Op::MAX, to);
    expect("allreduce/max", n, m.data(), [&](size_t i) {
      double b = 0;
      for (int r = 0; r < world; ++r) b = std::max(b, double((r * 7 + i) % world));
      return b;
    });

    std::vector<float> rd(n, float(rank + 1));
    c.reduce(rd.data(), n, at::kFloat, Op::SUM, world - 1, to);
    if (rank == world - 1) expect("reduce", n, rd.data(), [&](size_t) { return float(tri); });

    std::vector<int32_t> b(n, rank == 0 ? 42 : -1);
    c.broadcast(b.data(), n * sizeof(int32_t), 0, to);
    expect("broadcast", n, b.data(), [](size_t) { return int32_t{42}; });

    std::vector<int32_t> in(n, rank), out(n * world, -1);
    std::vector<void*> outs(world);
    for (int r = 0; r < world; ++r) outs[r] = out.data() + r * n;
    c.allgather(in.data(), outs, n * sizeof(int32_t), to);
    expect("allgather", n * world, out.data(), [&](size_t i) { return int32_t(i / n); });

    const int groot = 1 % world;
    std::fill(out.begin(), out.end(), -1);
    std::vector<void*> gouts(world, nullptr);
    if (rank == groot) gouts = outs;
    c.gather(in.data(), gouts, n * sizeof(int32_t), groot, to);
    if (rank == groot) expect("gather", n * world, out.data(), [&](size_t i) { return int32_t(i / n); });

    std::vector<int32_t> src(n * world);
    for (size_t i = 0; i < n * world; ++i) src[i] = int32_t((i / n) * 100 + i % n);
    std::vector<const void*> ins(world, nullptr);
    if (rank == 0)
      for (int r = 0; r < world; ++r) ins[r] = src.data() + r * n;
    std::vector<int32_t> sc(n, -1);
    c.scatter(ins, sc.data(), n * sizeof(int32_t), 0, to);
    expect("scatter", n, sc.data(), [&](size_t i) { return int32_t(rank * 100 + i); });

    std::vector<float> rs_in(n * world, float(rank + 1)), rs_out(n, -1.f);
    std::vector<const void*> rs_ptr(world);
    for (int r = 0; r < world; ++r) rs_ptr[r] = rs_in.data() + r * n;
    c.reduce_scatter(rs_ptr, rs_out.data(), n, at::kFloat, Op::SUM, to);
    expect("reduce_scatter", n, rs_out.data(), [&](size_t) { return float(tri); });

    // all-to-all with uneven sizes: rank s sends (s + d + 1) * k ints, value s * 1000 + d, to rank d
    const size_t k = n / 8 + 1;
    std::vector<std::vector<int32_t>> sbuf(world), rbuf(world);
    std::vector<const void*> ip(world);
    std::vector<void*> op(world);
    std::vector<size_t> sb(world), rb(world);
    for (int d = 0; d < world; ++d) {
      sbuf[d].assign((rank + d + 1) * k, rank * 1000 + d);
      rbuf[d].assign((d + rank + 1) * k, -1);
      ip[d] = sbuf[d].data();
      sb[d] = sbuf[d].size() * sizeof(int32_t);
      op[d] = rbuf[d].data();
      rb[d] = rbuf[d].size() * sizeof(int32_t);
    }
    c.alltoall(ip, sb, op, rb, to);
    for (int s = 0; s < world; ++s)
      expect("alltoall", rbuf[s].size(), rbuf[s].data(), [&](size_t) { return int32_t(s * 1000 + rank); });

    // p2p ring (even ranks send first, odd ranks receive first: no cycle of blocked senders)
    if (world > 1) {
      const int nxt = (rank + 1) % world, prv = (rank + world - 1) % world;
      std::vector<int64_t> snd(n), rcv(n, -1);
      for (size_t i = 0; i < n; ++i) snd[i] = int64_t(rank) * 1000003 + int64_t(i);
      if (rank % 2 == 0) {
        c.send(snd.data(), n * sizeof(int64_t), nxt, to);
        c.recv(rcv.data(), n * sizeof(int64_t), prv, to);
      } else {
        c.recv(rcv.data(), n * sizeof(int64_t), prv, to);
        c.send(snd.data(), n * sizeof(int64_t), nxt, to);
      }
      expect("p2p", n, rcv.data(), [&](size_t i) { return int64_t(prv) * 1000003 + int64_t(i); });
    }
    c.barrier(to);
  }
  c.barrier(to);
  // let every peer leave its last wait before anyone exits (a finished rank looks like a dead peer)
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  return g_fail;
}

}  // namespace

int main(int argc, char** argv) {
  const int world = argc > 1 ? std::atoi(argv[1]) : 4;
  char path[] = "/tmp/pdcc_san_XXXXXX";
  const int fd = mkstemp(path);
  if (fd < 0) return 2;
  close(fd);
  unlink(path);  // the FileStore creates it
  std::vector<pid_t> kids;
  for (int r = 0; r < world; ++r) {
    const pid_t p = fork();
    if (p == 0) {
      int rc = 0;
      try {
        rc = run(path, r, world);
      } catch (const std::exception& e) {
        std::fprintf(stderr, "[rank %d] exception: %s\n", r, e.what());
        rc = 100;
      }
      std::fflush(stderr);
      _exit(std::min(rc, 100));
    }
    kids.push_back(p);
  }
  int bad = 0;
  for (const pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) ++bad;
  }
  unlink(path);
  std::printf("%s: %d of %d ranks failed\n", bad ? "FAIL" : "OK", bad, world);
  return bad ? 1 : 0;
}
