// Tree files (see pkdtree/tree_io.hpp).
#include "pkdtree/tree_io.hpp"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>


namespace pkdtree {

namespace {

constexpr size_t kHeader = 40;  // struct "<8sIIQIIQ"

void put32(unsigned char* p, u32 v) {
  for (int i = 0; i < 4; ++i) p[i] = static_cast<unsigned char>(v >> (8 * i));
}
void put64(unsigned char* p, u64 v) {
  for (int i = 0; i < 8; ++i) p[i] = static_cast<unsigned char>(v >> (8 * i));
}

void pwrite_all(int fd, const void* buf, size_t bytes, off_t off, const std::string& path) {
  const char* c = static_cast<const char*>(buf);
  while (bytes) {
    const ssize_t w = ::pwrite(fd, c, bytes, off);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) throw std::runtime_error(path + ": write failed: " + std::strerror(errno));
    c += w;
    off += w;
    bytes -= size_t(w);
  }
}

struct Fd {
  int fd;
  Fd(const std::string& path, int flags) : fd(::open(path.c_str(), flags, 0644)) {
    if (fd < 0) throw std::runtime_error(path + ": cannot open: " + std::strerror(errno));
  }
  ~Fd() { ::close(fd); }
};

}  // namespace

void tree_file_create(const std::string& path, i64 n, int dim, int depth0, int mode) {
  Fd f(path, O_WRONLY | O_CREAT | O_TRUNC);
  unsigned char h[kHeader] = {};
  std::memcpy(h, "PKDTREE\x01", 8);
  put32(h + 8, 1);
  put32(h + 12, u32(dim));
  put64(h + 16, u64(n));
  put32(h + 24, u32(depth0));
  put32(h + 28, u32(mode));
  put64(h + 32, 0);
  pwrite_all(f.fd, h, kHeader, 0, path);
  const off_t total = off_t(kHeader + size_t(n) * 4 + size_t(n) * size_t(dim) * 4);
  if (::ftruncate(f.fd, total) != 0) throw std::runtime_error(path + ": cannot size the file");
}

void tree_file_write(const std::string& path, i64 n_total, int dim, i64 slot0, i64 count, const float* pts,
                     const u32* ids) {
  if (count <= 0) return;
  if (slot0 < 0 || slot0 + count > n_total) throw std::invalid_argument("tree_file_write: slots out of range");
  Fd f(path, O_WRONLY);
  const off_t ids_off = off_t(kHeader), pts_off = off_t(kHeader + size_t(n_total) * 4);
  pwrite_all(f.fd, ids, size_t(count) * 4, ids_off + off_t(slot0) * 4, path);
  pwrite_all(f.fd, pts, size_t(count) * dim * 4, pts_off + off_t(slot0) * dim * 4, path);
}

}  // namespace pkdtree
