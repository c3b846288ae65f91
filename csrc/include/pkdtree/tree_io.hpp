// On-disk tree layout (the format of parallel_kd_tree_amd/utils/io.py): little-endian header,
// then ids (u32[n]) and coordinates (f32[n][dim]) in slot order -- the implicit in-order tree,
// i.e. the reference's post-build point_list order.
//
//   magic "PKDTREE\x01" | u32 version 1 | u32 dim | u64 n | u32 depth0 | u32 mode | u64 0
//
// Writers stream from device memory in chunks (a 1 B-point tree never sits in host RAM at
// once), and several processes can fill disjoint slot ranges of one file: the distributed
// CLI's ranks each write their share, rank 0 the header and the boundary top rows.
#pragma once
#include <string>

#include "pkdtree/common.hpp"

typedef struct ihipStream_t* hipStream_t;  // as in hip_runtime_api.h (the host-only writers need no HIP)

namespace pkdtree {

constexpr int kTreeModeExact = 0, kTreeModeReference = 1;

// Creates (truncates) the file, writes the header and sizes it for n slots.
void tree_file_create(const std::string& path, i64 n, int dim, int depth0, int mode);
// Writes slots [slot0, slot0 + count) from host arrays into an existing file of n_total slots.
void tree_file_write(const std::string& path, i64 n_total, int dim, i64 slot0, i64 count, const float* pts,
                     const u32* ids);
// Same from device arrays, streamed in chunks of 16 Mi slots. Synchronises `stream`.
void tree_file_write_device(const std::string& path, i64 n_total, int dim, i64 slot0, i64 count, const float* pts,
                            const u32* ids, hipStream_t stream);

}  // namespace pkdtree
