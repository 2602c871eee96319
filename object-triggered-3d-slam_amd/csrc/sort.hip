// sort.hip — stable device radix sort of (u64 key, u32 value) pairs (rocPRIM, LSD => stable).
// Used to put volume units in key order (export, marching cubes) and to group points by voxel key while
// keeping input-index order inside each voxel (voxel_down_sample sums in index order, like Open3D).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"
#include "sort.h"

namespace ot {

// Onesweep (one LSD pass per 8 key bits) at every size: rocPRIM's default switches to a comparison merge sort
// below 2^20 items, ~10 launches per sort independent of how few key bits are in use.
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 0>;

ot_status sort_pairs_u64_u32(const unsigned long long* kin, unsigned long long* kout, const unsigned* vin,
                             unsigned* vout, size_t n, int end_bit, hipStream_t stream, int scratch_slot) {
    if (n == 0) return OT_OK;
    size_t tmp = 0;
    OT_HIP_TRY(rocprim::radix_sort_pairs<SortConfig>(nullptr, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, stream));
    void* ws = scratch(tmp + 16, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "sort scratch allocation failed");
    OT_HIP_TRY(rocprim::radix_sort_pairs<SortConfig>(ws, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, stream));
    return OT_OK;
}

ot_status exclusive_scan_i64(const long long* in, long long* out, size_t n, hipStream_t stream, int scratch_slot) {
    if (n == 0) return OT_OK;
    size_t tmp = 0;
    OT_HIP_TRY(rocprim::exclusive_scan(nullptr, tmp, in, out, 0ll, n, rocprim::plus<long long>(), stream));
    void* ws = scratch(tmp + 16, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "scan scratch allocation failed");
    OT_HIP_TRY(rocprim::exclusive_scan(ws, tmp, in, out, 0ll, n, rocprim::plus<long long>(), stream));
    return OT_OK;
}

}  // namespace ot
