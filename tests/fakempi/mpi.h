// A file-based stand-in for the six MPI calls of the reference's kdtree_mpi.cpp
// (MPI_Init / Comm_rank / Comm_size / Type_contiguous+commit / Bcast / Reduce(MIN) / Finalize;
// SURVEY.md §2.3), so the UNMODIFIED reference MPI driver runs as P ordinary processes in a
// test: rank and size come from FAKEMPI_RANK / FAKEMPI_SIZE, messages are files in FAKEMPI_DIR
// (written to a temporary name, then renamed, so a reader never sees a partial file).
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

typedef int MPI_Comm;
typedef int MPI_Datatype;  // element size in bytes
typedef int MPI_Op;
#define MPI_COMM_WORLD 0
#define MPI_INT 4
#define MPI_FLOAT (-4)  // 4 bytes, reduced as float
#define MPI_MIN 1
#define MPI_SUCCESS 0

namespace fakempi {
inline int& rank() { static int r = 0; return r; }
inline int& size() { static int s = 1; return s; }
inline int& seq() { static int q = 0; return q; }
inline std::string dir() { const char* d = std::getenv("FAKEMPI_DIR"); return d ? d : "."; }
inline int bytes(MPI_Datatype t) { return t < 0 ? -t : t; }
inline void put(const std::string& name, const void* p, size_t n) {
  const std::string tmp = dir() + "/" + name + ".tmp", fin = dir() + "/" + name;
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f || std::fwrite(p, 1, n, f) != n) std::abort();
  std::fclose(f);
  if (std::rename(tmp.c_str(), fin.c_str()) != 0) std::abort();
}
inline void get(const std::string& name, void* p, size_t n) {
  const std::string fin = dir() + "/" + name;
  for (int i = 0; i < 600000; ++i) {  // <= 10 min
    if (FILE* f = std::fopen(fin.c_str(), "rb")) {
      const size_t got = std::fread(p, 1, n, f);
      std::fclose(f);
      if (got != n) std::abort();
      return;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  std::abort();
}
}  // namespace fakempi

inline int MPI_Init(int*, char***) {
  const char* r = std::getenv("FAKEMPI_RANK");
  const char* s = std::getenv("FAKEMPI_SIZE");
  fakempi::rank() = r ? std::atoi(r) : 0;
  fakempi::size() = s ? std::atoi(s) : 1;
  return MPI_SUCCESS;
}
inline int MPI_Comm_rank(MPI_Comm, int* r) { *r = fakempi::rank(); return MPI_SUCCESS; }
inline int MPI_Comm_size(MPI_Comm, int* s) { *s = fakempi::size(); return MPI_SUCCESS; }
inline int MPI_Type_contiguous(int count, MPI_Datatype old, MPI_Datatype* t) {
  *t = count * fakempi::bytes(old);
  return MPI_SUCCESS;
}
inline int MPI_Type_commit(MPI_Datatype*) { return MPI_SUCCESS; }
inline int MPI_Bcast(void* buf, int count, MPI_Datatype t, int root, MPI_Comm) {
  const std::string name = "bcast" + std::to_string(fakempi::seq()++);
  const size_t n = size_t(count) * fakempi::bytes(t);
  if (fakempi::rank() == root) fakempi::put(name, buf, n);
  else fakempi::get(name, buf, n);
  return MPI_SUCCESS;
}
inline int MPI_Reduce(const void* send, void* recv, int count, MPI_Datatype t, MPI_Op op, int root, MPI_Comm) {
  if (t != MPI_FLOAT || op != MPI_MIN) std::abort();  // the reference's only reduction
  const std::string name = "reduce" + std::to_string(fakempi::seq()++) + "_";
  fakempi::put(name + std::to_string(fakempi::rank()), send, size_t(count) * 4);
  if (fakempi::rank() == root) {
    std::vector<float> acc(static_cast<const float*>(send), static_cast<const float*>(send) + count), v(count);
    for (int r = 0; r < fakempi::size(); ++r) {
      fakempi::get(name + std::to_string(r), v.data(), size_t(count) * 4);
      for (int i = 0; i < count; ++i) acc[i] = v[i] < acc[i] ? v[i] : acc[i];
    }
    std::memcpy(recv, acc.data(), size_t(count) * 4);
  }
  return MPI_SUCCESS;
}
inline int MPI_Finalize() { return MPI_SUCCESS; }
