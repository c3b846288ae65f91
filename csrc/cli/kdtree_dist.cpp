// kdtree_dist — native multi-GPU driver with the reference MPI program's behaviour
// (kdtree_mpi.cpp:170-291), one process per MI355X, RCCL over xGMI instead of MPI.
//
//   kdtree_dist --gpus P [options] [SEED DIM_POINTS NUM_POINTS]
//
// The launcher process parses the configuration (eval protocol: READY, seed on stdin; debug
// protocol: argv), never touches the GPU, and forks P ranks. Rank 0 creates the RCCL unique
// id and hands it to the other ranks through pipes (MPI_Init / Comm_rank / Comm_size,
// :177-183). Then, exactly as the reference's forest decomposition:
//   * config broadcast from rank 0 (MPI_Bcast of {seed, dim, N}, :199)   -> ncclBroadcast
//   * rank r generates its generation-order slice local = N / P (remainder to the last
//     rank, :204-224) on its own GPU — jump-ahead device generator, no discard() walk —
//     plus the 10 queries (rows N .. N+9)
//   * rank r builds its own local kd-tree (HIP level-synchronous builder) with global ids
//   * every rank answers the queries on its tree; packed (d2 << 32 | id) results are
//     MIN-reduced to rank 0 (MPI_Reduce MIN of the distances, :253)             -> ncclReduce
//   * rank 0 prints the protocol lines.
// --decomp global instead builds ONE exact tree over all ranks, for any P (GlobalBuilder: the
// top levels by allreduce histograms + allgather pivot selection, one all-to-all round per
// top-level leaf of a rank, overlapped with the leaf builds; --pipeline-k adds levels); each
// rank answers the queries on its share (complete subtrees plus the top rows between them),
// rank 0 also on the boundary top rows, and the same MIN reduce combines them.
// Ranks with no points (N < P, the reference's segfault F7) contribute +inf.
// --mode reference (forest): every rank builds the reference's own quirky tree on the GPU
// (build_reference.hip) and searches it with the reference's procedure, as kdtree_mpi does.
// --save PATH writes the tree(s) (tree_io.hpp; forest: PATH.rank<r>), --leaf-threshold N caps
// the LDS subtree segments, --share-gpu puts every rank on --device (one-GPU rehearsal).
// --ranks R (forest, R >= P): R logical forest ranks over the P processes -- the reference's own
// `mpirun -np 16 --oversubscribe` (Makefile:36) on fewer GPUs; each process builds and searches
// the trees of its R / P logical slices and MIN-combines them before the reduce.
// Every collective is waited on with a watchdog (RcclComm::wait): the stream is polled and
// ncclCommGetAsyncError checked until a deadline (--timeout seconds, default 300); a stuck or
// failed collective aborts the communicator and the rank exits non-zero, after which the
// launcher stops the remaining ranks and returns non-zero.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "cli_common.hpp"
#include "ref_fallback.hpp"
#include "pkdtree/generator.hpp"
#include "pkdtree/global_builder.hpp"
#include "pkdtree/gpu_build.hpp"
#include "pkdtree/gpu_generator.hpp"
#include "pkdtree/gpu_query.hpp"
#include "pkdtree/gpu_reference.hpp"
#include "pkdtree/hip_check.hpp"
#include "pkdtree/rccl_comm.hpp"
#include "pkdtree/tree_io.hpp"

using namespace pkdtree;

namespace {

int g_rank = -1;

#define PKD_NCCL_CHECK(expr)                                                                        \
  do {                                                                                              \
    ncclResult_t r_ = (expr);                                                                       \
    if (r_ != ncclSuccess)                                                                          \
      throw std::runtime_error(std::string("rank ") + std::to_string(g_rank) + ": " #expr " -> " + \
                               ncclGetErrorString(r_));                                             \
  } while (0)

struct Config {
  int seed, dim, num_points;
};


void write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t w = ::write(fd, c, n);
    if (w <= 0) throw std::runtime_error("pipe write failed");
    c += w;
    n -= size_t(w);
  }
}
void read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t r = ::read(fd, c, n);
    if (r <= 0) throw std::runtime_error("pipe read failed (rank 0 died before sharing the RCCL id?)");
    c += r;
    n -= size_t(r);
  }
}

int run_rank(int rank, int P, int R, Config cfg, const cli::Options& o, const std::vector<int>& id_pipes,
             double timeout_s, std::chrono::high_resolution_clock::time_point tick) {
  g_rank = rank;
  if (o.share_gpu) {
    // every rank on one device (rehearsal on a one-GPU box): RCCL accepts several ranks per
    // device only when they look like different hosts, so each rank gets its own host id and
    // the ranks talk over the loopback socket transport
    ::setenv("NCCL_HOSTID", ("pkd-dist-rank" + std::to_string(rank)).c_str(), 1);
    ::setenv("NCCL_SOCKET_IFNAME", "lo", 0);
  }
  PKD_HIP_CHECK(hipSetDevice(o.share_gpu ? o.device : o.device + rank));
  // RCCL prints a version banner on stdout during initialisation; stdout carries only the
  // protocol, so fd 1 points at stderr until the communicator is up.
  std::fflush(stdout);
  const int saved_stdout = ::dup(1);
  ::dup2(2, 1);
  ncclUniqueId uid;
  if (rank == 0) {
    PKD_NCCL_CHECK(ncclGetUniqueId(&uid));
    for (int r = 1; r < P; ++r) write_all(id_pipes[size_t(2 * r + 1)], &uid, sizeof(uid));
  } else {
    read_all(id_pipes[size_t(2 * rank)], &uid, sizeof(uid));
  }
  ncclComm_t comm;
  PKD_NCCL_CHECK(ncclCommInitRank(&comm, P, uid, rank));
  std::fflush(stdout);
  ::dup2(saved_stdout, 1);
  ::close(saved_stdout);
  hipStream_t s;
  PKD_HIP_CHECK(hipStreamCreate(&s));
  // every wait on the stream is bounded and polls the communicator's asynchronous error state
  // (Comm::wait): a stuck or failed peer aborts the communicator and this rank exits non-zero
  RcclComm rcomm(comm, rank, P);
  rcomm.set_timeout(timeout_s);
  auto watchdog_wait = [&](hipStream_t st, const char* what) { rcomm.wait(st, what); };

  // MPI_Bcast of the configuration (kdtree_mpi.cpp:199): rank 0's values win.
  int* d_cfg = nullptr;
  PKD_HIP_CHECK(hipMalloc(&d_cfg, 3 * sizeof(int)));
  const int hcfg[3] = {cfg.seed, cfg.dim, cfg.num_points};
  PKD_HIP_CHECK(hipMemcpyAsync(d_cfg, hcfg, sizeof(hcfg), hipMemcpyHostToDevice, s));
  PKD_NCCL_CHECK(ncclBroadcast(d_cfg, d_cfg, 3, ncclInt32, 0, comm, s));
  int bcfg[3];
  PKD_HIP_CHECK(hipMemcpyAsync(bcfg, d_cfg, sizeof(bcfg), hipMemcpyDeviceToHost, s));
  watchdog_wait(s, "config broadcast");
  cfg = Config{bcfg[0], bcfg[1], bcfg[2]};
  const int dim = cfg.dim, Q = o.num_queries;
  const i64 N = cfg.num_points;

  // forest slices (kdtree_mpi.cpp:204-224) of the R logical ranks (the reference's mpirun -np R,
  // Makefile:36 runs 16): equal parts, remainder to the last logical rank; this process owns the
  // contiguous logical ranks [lr0, lr1) (R / P each, the first R % P one more), i.e. one
  // contiguous run of generation order, built as lr1 - lr0 independent trees
  const int lr0 = rank * (R / P) + std::min(rank, R % P), lr1 = lr0 + R / P + (rank < R % P ? 1 : 0);
  struct Slice {
    int lr;
    i64 first, n;
  };
  std::vector<Slice> slices;
  for (int lr = lr0; lr < lr1; ++lr) {
    i64 ln = N / R;
    const i64 lf = ln * lr;
    if (lr == R - 1) ln += N % R;
    slices.push_back({lr, lf, ln});
  }
  const i64 first = slices.front().first;
  i64 local = 0;
  for (const Slice& sl : slices) local += sl.n;

  const auto g0 = std::chrono::high_resolution_clock::now();
  float* d_x = nullptr;
  PKD_HIP_CHECK(hipMalloc(&d_x, size_t(std::max<i64>(local, 1) + Q) * dim * 4));
  {
    const DevGenPlan gp = devgen_plan(size_t(std::max<i64>(local, Q)) * dim);
    void* gws = nullptr;
    PKD_HIP_CHECK(hipMalloc(&gws, std::max<size_t>(1, devgen_workspace_bytes(gp))));
    if (local > 0) generate_rows_device(uint32_t(cfg.seed), dim, first, local, d_x, gws, s);
    generate_rows_device(uint32_t(cfg.seed), dim, N, Q, d_x + size_t(local) * dim, gws, s);  // the queries
    PKD_HIP_CHECK(hipStreamSynchronize(s));
    PKD_HIP_CHECK(hipFree(gws));
  }
  const auto g1 = std::chrono::high_resolution_clock::now();

  u64* d_res = nullptr;
  PKD_HIP_CHECK(hipMalloc(&d_res, size_t(Q) * 8));
  hipEvent_t e0, e1, e2;
  for (hipEvent_t* e : {&e0, &e1, &e2}) PKD_HIP_CHECK(hipEventCreate(e));
  float* d_tree = nullptr;
  u32* d_ids = nullptr;
  void* ws = nullptr;
  std::vector<std::unique_ptr<GpuBuilder>> bs;        // forest: one per logical rank of this process
  std::vector<std::unique_ptr<ReferenceBuilder>> rbs;  // --mode reference (forest): the reference's own trees
  const bool ref = o.mode == "reference";
  const bool global = o.decomp == "global";
  std::unique_ptr<GlobalBuilder> gb;
  size_t wsb_all = 0;
  if (global) {
    gb = std::make_unique<GlobalBuilder>(rcomm, N, dim, o.pipeline_k);
  } else if (local > 0) {  // allocations outside the timed region
    size_t wsb = 0;
    for (const Slice& sl : slices) {
      if (ref) {
        rbs.push_back(std::make_unique<ReferenceBuilder>(sl.n, dim));
        wsb = std::max(wsb, rbs.back()->workspace_bytes());
      } else {
        bs.push_back(std::make_unique<GpuBuilder>(sl.n, dim, BuildOptions{o.leaf_threshold, 0}));
        wsb = std::max(wsb, bs.back()->workspace_bytes());
      }
    }
    PKD_HIP_CHECK(hipMalloc(&d_tree, size_t(local) * dim * 4));
    PKD_HIP_CHECK(hipMalloc(&d_ids, size_t(local) * 4));
    PKD_HIP_CHECK(hipMalloc(&ws, std::max<size_t>(wsb, 256)));
    wsb_all = wsb;
  }
  PKD_HIP_CHECK(hipEventRecord(e0, s));
  nn_init(d_res, Q, s);
  // global 1-based ids (kdtree_mpi.cpp:223)
  // (forest: the trees of this process's logical ranks one after another, one workspace; a
  // sampled-top build that reports a band miss is redone unsampled after the queries)
  size_t ws_bytes = ws ? std::max<size_t>(wsb_all, 256) : 0;
  // returns the builder that wrote the workspace's error words (the unsampled fallback has its
  // own plan and workspace layout: the workspace is grown to it, and its error word is read)
  std::unique_ptr<GpuBuilder> fallback;
  auto build_slice = [&](size_t k, bool allow_top) -> GpuBuilder* {
    const Slice& sl = slices[k];
    const i64 off = sl.first - first;
    if (sl.n <= 0) return nullptr;
    if (ref) {  // (ties: this rank's tree from the CPU std::sort builder, before any collective)
      cli::build_reference_checked(*rbs[k], d_x + off * dim, sl.n, dim, u32(sl.first + 1), d_tree + off * dim,
                                   d_ids + off, ws, s, "kdtree_dist");
      return nullptr;
    }
    GpuBuilder* b = bs[k].get();
    if (!allow_top) {
      fallback = std::make_unique<GpuBuilder>(sl.n, dim, BuildOptions{o.leaf_threshold, 0, true, false});
      if (fallback->workspace_bytes() > ws_bytes) {
        PKD_HIP_CHECK(hipStreamSynchronize(s));
        PKD_HIP_CHECK(hipFree(ws));
        ws_bytes = fallback->workspace_bytes();
        PKD_HIP_CHECK(hipMalloc(&ws, ws_bytes));
      }
      b = fallback.get();
    }
    b->build(d_x + off * dim, nullptr, u32(sl.first + 1), d_tree + off * dim, d_ids + off, ws, s);
    return b;
  };
  u32 slice_err = 0;
  if (global) {
    gb->build(d_x, local, u32(first + 1), s);
  } else if (local > 0) {
    for (size_t k = 0; k < slices.size(); ++k) {
      GpuBuilder* wrote = build_slice(k, true);
      // the shared workspace holds one build's error words; a sampled build is checked here, on
      // this rank alone, BEFORE any collective (its rebuild must not skew the collective order)
      if (wrote && (slices.size() > 1 || wrote->sampled())) {
        u32 e = wrote->read_error(ws, s);
        if ((e & top4_band_miss_bit()) && wrote->sampled()) {
          wrote = build_slice(k, false);
          e = wrote->read_error(ws, s);
        }
        slice_err |= e;
      }
    }
  }
  PKD_HIP_CHECK(hipEventRecord(e1, s));
  const float* d_q = d_x + size_t(local) * dim;
  const bool traverse = o.query == "traverse" || (o.query == "auto" && dim <= 16);
  if (global) {
    // routed (GlobalBuilder::query): each query searched in its home block, a MIN all-reduce
    // gives it a radius, then only in the blocks that radius reaches, a second MIN all-reduce
    // (the top rows between blocks and the boundary rows are brute-forced); --query brute:
    // brute force over every block of the rank, one MIN all-reduce
    gb->query(d_q, Q, d_res, s, false,
              o.query == "brute" ? GlobalBuilder::kQueryBrute
                                 : (o.query == "traverse" ? GlobalBuilder::kQueryTraverse : GlobalBuilder::kQueryAuto));
  } else if (local > 0) {
    u64* d_one = nullptr;  // reference mode: each tree's search starts afresh, as on its own rank
    if (ref && slices.size() > 1) PKD_HIP_CHECK(hipMalloc(&d_one, size_t(Q) * 8));
    for (const Slice& sl : slices) {  // every tree of this process: MIN into the same results
      if (sl.n <= 0) continue;
      const i64 off = sl.first - first;
      const float* tp = d_tree + off * dim;
      const u32* ti = d_ids + off;
      if (ref && d_one) {
        nn_init(d_one, Q, s);
        nn_traverse_reference(tp, ti, sl.n, dim, 0, d_q, Q, d_one, s);  // kdtree_mpi.cpp:234-243
        nn_min_into(d_one, d_res, Q, s);
      } else if (ref) {
        nn_traverse_reference(tp, ti, sl.n, dim, 0, d_q, Q, d_res, s);
      } else if (traverse) {
        nn_traverse(tp, ti, sl.n, dim, 0, d_q, Q, d_res, s);
      } else {
        nn_brute(tp, ti, 0, sl.n, dim, d_q, Q, d_res, s);
      }
    }
    if (d_one) {
      PKD_HIP_CHECK(hipStreamSynchronize(s));
      (void)hipFree(d_one);
    }
  }
  // MPI_Reduce(MIN) to rank 0 (kdtree_mpi.cpp:253), the id riding along in the low bits
  PKD_NCCL_CHECK(ncclReduce(d_res, d_res, size_t(Q), ncclUint64, ncclMin, 0, comm, s));
  PKD_HIP_CHECK(hipEventRecord(e2, s));
  std::vector<u64> res(static_cast<size_t>(Q));
  PKD_HIP_CHECK(hipMemcpyAsync(res.data(), d_res, size_t(Q) * 8, hipMemcpyDeviceToHost, s));
  watchdog_wait(s, "build + queries + reduce");

  // per-rank timings, MAX-reduced (the slowest rank bounds the job)
  float bld = 0, qry = 0;
  PKD_HIP_CHECK(hipEventElapsedTime(&bld, e0, e1));
  PKD_HIP_CHECK(hipEventElapsedTime(&qry, e1, e2));
  const float gen = float(std::chrono::duration<double, std::milli>(g1 - g0).count());
  // the build's device error word rides along (MAX over ranks: non-zero iff any rank failed)
  u32 berr = global ? gb->read_error(s) : slice_err;
  if (!global && !ref && slices.size() == 1 && local > 0 && !bs[0]->sampled()) berr = bs[0]->read_error(ws, s);
  float* d_t = nullptr;
  PKD_HIP_CHECK(hipMalloc(&d_t, 4 * sizeof(float)));
  const float ht[4] = {gen, bld, qry, float(berr & 0xFFFFFFu) + (berr >> 24 ? 1.0f : 0.0f)};
  PKD_HIP_CHECK(hipMemcpyAsync(d_t, ht, sizeof(ht), hipMemcpyHostToDevice, s));
  PKD_NCCL_CHECK(ncclReduce(d_t, d_t, 4, ncclFloat32, ncclMax, 0, comm, s));
  float mt[4];
  PKD_HIP_CHECK(hipMemcpyAsync(mt, d_t, sizeof(mt), hipMemcpyDeviceToHost, s));
  watchdog_wait(s, "timing reduce");
  if (berr) std::cerr << "kdtree_dist: rank " << rank << ": device build error word 0x" << std::hex << berr << std::dec
                      << std::endl;
  if (rank == 0 && mt[3] != 0.0f) {
    std::cerr << "kdtree_dist: a rank's tree build failed; no results printed" << std::endl;
    (void)ncclCommDestroy(comm);
    return 3;
  }

  if (rank == 0) {
    for (int q = 0; q < Q; ++q) print_result_line(N + q, std::sqrt(packed_dist(res[size_t(q)])));
    if (o.debug) {
      const auto tock = std::chrono::high_resolution_clock::now();
      print_elapsed(std::chrono::duration<double>(tock - tick).count());
    }
    print_done();
    std::cout.flush();
    if (o.metrics)
      std::fprintf(stderr,
                   "{\"ranks\": %d, \"decomp\": \"%s\", \"gen_ms\": %.3f, \"build_ms\": %.3f, "
                   "\"query_reduce_ms\": %.3f, \"build_mpts_per_s\": %.2f, \"local_global_levels\": %d, "
                   "\"top_levels\": %d}\n",
                   R, o.decomp.c_str(), mt[0], mt[1], mt[2], double(N) / 1e3 / std::max(mt[1], 1e-6f),
                   bs.empty() ? 0 : bs[0]->global_levels(), gb ? gb->top_levels() : 0);
  }
  // --save: forest ranks write their own trees (<path>.rank<r>, like kdtree_mpi's independent
  // trees); the global tree is one file, every rank writing its share into its slot range
  if (!o.save.empty()) {
    const int mode = ref ? kTreeModeReference : kTreeModeExact;
    if (!global) {
      for (const Slice& sl : slices) {
        const std::string path = o.save + ".rank" + std::to_string(sl.lr);
        tree_file_create(path, sl.n, dim, 0, mode);
        const i64 off = sl.first - first;
        if (sl.n > 0) tree_file_write_device(path, sl.n, dim, 0, sl.n, d_tree + off * dim, d_ids + off, s);
      }
    } else {
      if (rank == 0) tree_file_create(o.save, N, dim, 0, mode);
      PKD_NCCL_CHECK(ncclAllReduce(d_t, d_t, 1, ncclFloat32, ncclMax, comm, s));  // barrier: the file exists
      watchdog_wait(s, "save barrier");
      tree_file_write_device(o.save, N, dim, gb->slot_lo(), gb->n_leaf(), gb->tree_pts(), gb->tree_ids(), s);
      if (rank == 0) {
        const std::vector<i64> slots = gb->top_slots();
        std::vector<float> rows(slots.size() * size_t(dim + 1));
        if (!rows.empty())
          PKD_HIP_CHECK(hipMemcpy(rows.data(), gb->top_rows(), rows.size() * 4, hipMemcpyDeviceToHost));
        for (size_t h = 0; h < slots.size(); ++h) {
          if (slots[h] < 0) continue;
          u32 id;
          std::memcpy(&id, &rows[h * size_t(dim + 1) + dim], 4);
          tree_file_write(o.save, N, dim, slots[h], 1, &rows[h * size_t(dim + 1)], &id);
        }
      }
      PKD_NCCL_CHECK(ncclAllReduce(d_t, d_t, 1, ncclFloat32, ncclMax, comm, s));  // every share written
      watchdog_wait(s, "save barrier");
    }
  }
  (void)hipFree(d_x); (void)hipFree(d_res); (void)hipFree(d_cfg); (void)hipFree(d_t);
  gb.reset();
  if (d_tree) (void)hipFree(d_tree);
  if (d_ids) (void)hipFree(d_ids);
  if (ws) (void)hipFree(ws);
  PKD_NCCL_CHECK(ncclCommDestroy(comm));
  (void)hipStreamDestroy(s);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  // --gpus / --timeout are ours; everything else goes to the shared front-end
  int P = 1, R = 0;
  double timeout_s = 300.0;
  std::vector<char*> rest{argv[0]};
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if ((a == "--gpus" || a == "--timeout") && i + 1 < argc) {
      (a == "--gpus" ? void(P = std::atoi(argv[++i])) : void(timeout_s = std::atof(argv[++i])));
    } else if (a == "--ranks" && i + 1 < argc) {
      R = std::atoi(argv[++i]);
    } else if (a.rfind("--ranks=", 0) == 0) {
      R = std::atoi(a.c_str() + 8);
    } else if (a.rfind("--gpus=", 0) == 0) {
      P = std::atoi(a.c_str() + 7);
    } else if (a.rfind("--timeout=", 0) == 0) {
      timeout_s = std::atof(a.c_str() + 10);
    } else {
      rest.push_back(argv[i]);
    }
  }
  if (P < 1 || P > 64) {
    std::cerr << "--gpus must be in [1, 64]" << std::endl;
    return 1;
  }
  if (R == 0) R = P;
  if (R < P || R > 4096) {
    std::cerr << "--ranks must be in [--gpus, 4096]" << std::endl;
    return 1;
  }
  cli::Options o = cli::parse(int(rest.size()), rest.data());
  if (R != P && o.decomp == "global") {
    std::cerr << "kdtree_dist --ranks (logical forest ranks) applies to --decomp forest" << std::endl;
    return 1;
  }
  if (o.mode != "exact" && o.decomp == "global") {
    std::cerr << "kdtree_dist --decomp global builds exact trees only (the reference's quirky tree depends on "
                 "array positions, which the redistribution does not keep); use --decomp forest"
              << std::endl;
    return 1;
  }
  const auto tick = std::chrono::high_resolution_clock::now();
  const Problem p = cli::specify(o);  // launcher: protocol I/O only, no GPU call before fork
  std::cout.flush();
  std::fflush(stdout);
  std::fflush(stderr);
  const Config cfg{p.seed, p.dim, p.num_points};

  std::vector<int> fds(size_t(2 * P), -1);
  for (int r = 1; r < P; ++r)
    if (::pipe(&fds[size_t(2 * r)]) != 0) {
      std::perror("pipe");
      return 2;
    }
  std::vector<pid_t> kids;
  for (int r = 0; r < P; ++r) {
    const pid_t pid = ::fork();
    if (pid < 0) {
      std::perror("fork");
      for (pid_t k : kids) ::kill(k, SIGTERM);
      return 2;
    }
    if (pid == 0) {
      int rc = 0;
      try {
        rc = run_rank(r, P, R, cfg, o, fds, timeout_s, tick);
      } catch (const std::exception& ex) {
        std::cerr << "kdtree_dist: " << ex.what() << std::endl;
        rc = 2;
      }
      std::cout.flush();
      std::fflush(stderr);
      ::_exit(rc);
    }
    kids.push_back(pid);
  }
  for (int fd : fds)
    if (fd >= 0) ::close(fd);
  int rc = 0;
  for (size_t done = 0; done < kids.size(); ++done) {
    int st = 0;
    const pid_t w = ::wait(&st);
    if (w < 0) break;
    const bool ok = WIFEXITED(st) && WEXITSTATUS(st) == 0;
    if (!ok && rc == 0) {
      rc = WIFEXITED(st) ? WEXITSTATUS(st) : 3;
      for (pid_t k : kids)
        if (k != w) ::kill(k, SIGTERM);  // a failed rank: stop the others (they would block in RCCL)
    }
  }
  return rc;
}
