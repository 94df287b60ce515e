// skm_output.h -- the kept-set hand-off from HBM to host arrays in key order (skm_output.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>

#include "skm.h"
#include "skm_pool.h"

namespace skm {

struct HandoffStats {
    uint64_t n = 0, chunks = 0, bytes = 0;
    double setup_s = 0;  // pinned staging + stream + events
    double wait_s = 0;   // host waiting for a piece's D2H (device sort + PCIe not yet done)
    double copy_s = 0;   // host pool copying pieces from pinned staging into the output arrays
    double total_s = 0;
    // device time (ms) summed over the chunks: selection, radix sort, gather; and the D2H pieces
    float select_ms = 0, sort_ms = 0, gather_ms = 0, d2h_ms = 0;
    uint64_t max_chunk = 0;  // k-mers of the largest chunk (sizes the device scratch)
    int wide_index = 0;      // 1: u64 arena indices (a hand-off of >= 2^32 k-mers)
};

// The n kept k-mers of a device arena (raw little-endian keys, 10-byte records; keys distinct) into
// newly allocated host arrays (*keys_out, *data_out; release with std::free), ascending by key.
// Device work runs on st; pool (may be null) copies the pinned pieces out.  Chunks are sized so
// their device scratch fits 3/4 of the memory free at the call.  index_limit / max_chunk: test
// hooks (0 = defaults 2^32 / none) that force the u64-index form and small chunks.
void kept_handoff(const uint64_t* dkeys, const skm_stored_kmer_data* ddata, uint64_t n, hipStream_t st,
                  HostPool* pool, uint64_t** keys_out, skm_stored_kmer_data** data_out, HandoffStats* stats,
                  uint64_t index_limit = 0, uint64_t max_chunk = 0);

}  // namespace skm
