// Device ops for the distributed (global) decomposition — filled in with global mode.
#include <hip/hip_runtime.h>
