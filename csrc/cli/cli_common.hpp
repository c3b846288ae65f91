// Shared CLI front-end for the kdtree_* executables.
//
// Reference behaviour (Utility.cpp:92-120, kdtree_sequential.cpp:140-193): with DEBUG 0 the
// program prints READY, reads the seed from stdin and uses dim=128, N=500000; with DEBUG 1
// it takes SEED DIM_POINTS NUM_POINTS from argv and prints "elapsed time". Here the mode is
// chosen at run time: three positional arguments (or --debug / KDTREE_DEBUG=1) select the
// debug protocol, none selects the eval protocol. Options start with "--" and never reach
// the positional parser, so `prog 42 3 1024` behaves exactly like the reference's DEBUG
// build.
#pragma once
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "pkdtree/protocol.hpp"

namespace pkdtree {
namespace cli {

struct Options {
  bool debug = false;
  std::string mode = "exact";      // exact | reference
  std::string query = "auto";      // auto | brute | traverse
  int threads = 0;
  int num_queries = 10;            // kdtree_sequential.cpp:144
  bool metrics = false;            // per-phase timings as one JSON line on stderr
  int device = 0;
  bool host_gen = false;           // generate on the host and copy (default: on the GPU)
  std::string decomp = "forest";   // kdtree_dist: forest (kdtree_mpi.cpp) | global (one tree)
  int pipeline_k = -1;             // kdtree_dist --decomp global: extra top levels (-1: auto)
  std::string save;                // write the tree (tree_io.hpp format); forest ranks: <save>.rank<r>
  int leaf_threshold = 0;          // largest segment of the LDS subtree kernel (0: auto from dim)
  bool share_gpu = false;          // kdtree_dist: every rank on --device (RCCL ranks as separate hosts)
  std::vector<char*> positional;   // argv[0] + positionals
};

inline Options parse(int argc, char** argv) {
  Options o;
  o.positional.push_back(argv[0]);
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&](const char* name) -> std::string {
      const std::string pre = std::string(name) + "=";
      if (a.rfind(pre, 0) == 0) return a.substr(pre.size());
      if (a == name && i + 1 < argc) return argv[++i];
      std::cerr << "missing value for " << name << std::endl;
      std::exit(1);
    };
    // "--name value" or "--name=value" (exact names: --query is not a prefix of --queries)
    auto is = [&](const char* name) { return a == name || a.rfind(std::string(name) + "=", 0) == 0; };
    if (a == "--debug") o.debug = true;
    else if (a == "--metrics-json") o.metrics = true;
    else if (is("--mode")) o.mode = val("--mode");
    else if (is("--query")) o.query = val("--query");
    else if (is("--threads")) o.threads = std::atoi(val("--threads").c_str());
    else if (is("--queries")) o.num_queries = std::atoi(val("--queries").c_str());
    else if (a == "--host-gen") o.host_gen = true;
    else if (is("--device")) o.device = std::atoi(val("--device").c_str());
    else if (is("--decomp")) o.decomp = val("--decomp");
    else if (is("--pipeline-k")) o.pipeline_k = std::atoi(val("--pipeline-k").c_str());
    else if (is("--save")) o.save = val("--save");
    else if (is("--leaf-threshold")) o.leaf_threshold = std::atoi(val("--leaf-threshold").c_str());
    else if (a == "--share-gpu") o.share_gpu = true;
    else o.positional.push_back(argv[i]);
  }
  const char* env = std::getenv("KDTREE_DEBUG");
  if (env && std::strcmp(env, "0") != 0) o.debug = true;
  if (o.positional.size() > 1) o.debug = true;
  if (o.decomp != "forest" && o.decomp != "global") {
    std::cerr << "--decomp must be forest or global" << std::endl;
    std::exit(1);
  }
  if (o.mode != "exact" && o.mode != "reference") {
    std::cerr << "--mode must be exact or reference" << std::endl;
    std::exit(1);
  }
  return o;
}

inline Problem specify(Options& o) {
  if (o.debug) return specify_problem_argv(int(o.positional.size()), o.positional.data());
  return specify_problem_stdin();
}

}  // namespace cli
}  // namespace pkdtree
