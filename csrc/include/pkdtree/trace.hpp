// roctx ranges around host-side phases (build, level pairs, subtree, generator, queries,
// distributed phases). rocprofv3 --marker-trace shows them next to the kernel trace; with no
// tool attached a push/pop is a cheap library call. (The reference only has a DEBUG wall
// clock, kdtree_sequential.cpp:146-191)
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace pkdtree {

struct TraceRange {
  explicit TraceRange(const char* name) { roctxRangePush(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

inline void trace_push(const char* name) { roctxRangePush(name); }
inline void trace_pop() { roctxRangePop(); }

}  // namespace pkdtree
