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
