// sort.h — host entry points of sort.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/otslam.h"

namespace ot {

// Stable LSD radix sort of n (key, value) pairs over key bits [0, end_bit).  Scratch slot for temp storage.
ot_status sort_pairs_u64_u32(const unsigned long long* kin, unsigned long long* kout, const unsigned* vin,
                             unsigned* vout, size_t n, int end_bit, hipStream_t stream, int scratch_slot);

// The same for 32-bit keys (rocPRIM onesweep: 8 B per pair per pass instead of 12).
ot_status sort_pairs_u32_u32(const unsigned* kin, unsigned* kout, const unsigned* vin, unsigned* vout, size_t n,
                             int end_bit, hipStream_t stream, int scratch_slot);

// Segmented form (own onesweep): the input is nseg <= 64 concatenated segments, seg[0..nseg] host offsets (seg[0] = 0,
// seg[nseg] = n); each segment is sorted stably on its own (pairs never cross a segment boundary).  dlen (device,
// nullable): segment s holds only its first dlen[s] pairs, the rest of its range is capacity (left untouched).
ot_status sort_segments_u32_u32(const unsigned* kin, unsigned* kout, const unsigned* vin, unsigned* vout,
                                const int64_t* seg, int nseg, int end_bit, hipStream_t stream, int scratch_slot,
                                const int* dlen = nullptr);


}  // namespace ot
