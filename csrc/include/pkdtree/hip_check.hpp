// Error checking for HIP calls: failures raise with file:line and the HIP error text
// (the reference ignores every error code).
#pragma once
#include <hip/hip_runtime.h>

#include <sstream>
#include <stdexcept>

#define PKD_HIP_CHECK(expr)                                                               \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      std::ostringstream _os;                                                             \
      _os << "HIP error '" << hipGetErrorString(_e) << "' (" << int(_e) << ") at "        \
          << __FILE__ << ":" << __LINE__ << " in " #expr;                                 \
      throw std::runtime_error(_os.str());                                                \
    }                                                                                     \
  } while (0)

#define PKD_LAUNCH_CHECK() PKD_HIP_CHECK(hipGetLastError())

#include <map>
#include <mutex>
#include <utility>

namespace pkdtree {

// Raise kernel `fn`'s dynamic-LDS limit to at least `bytes` on the current device. Done once per
// (kernel, device) and thread-safe, so a process that builds on several devices (or from several
// host threads) never launches a kernel whose limit was only raised on another device.
inline void ensure_dynamic_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> done;
  int dev = 0;
  PKD_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  int& have = done[{fn, dev}];
  if (have >= bytes) return;
  PKD_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  have = bytes;
}

}  // namespace pkdtree
