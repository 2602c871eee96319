// sort.hip — stable device radix sort of (u64 key, u32 value) pairs (own LSD onesweep; rocPRIM above 2M pairs).
// Used to put volume units in key order (export, marching cubes) and to group points by voxel key while
// keeping input-index order inside each voxel (voxel_down_sample sums in index order, like Open3D).
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"
#include "sort.h"

namespace ot {

// Onesweep (one LSD pass per 8 key bits) at every size: rocPRIM's default switches to a comparison merge sort
// below 2^20 items, ~10 launches per sort independent of how few key bits are in use.
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 0>;
// large (u64 key, u32 value) sorts: 8-bit digits with a 256-thread histogram kernel (measured: 10-bit digits, 4 passes
// instead of 5 for a 33-bit key, are slower; 11 bits do not fit the onesweep histograms of a 64-bit key in LDS)
#ifndef OT_SORT_BITS
#define OT_SORT_BITS 8
#endif
using BigSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 16>, rocprim::kernel_config<512, 16>, OT_SORT_BITS,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

// ------------------------------------------------------------------------------------------------------------
// Own stable LSD radix sort (8-bit digits), P + 2 launches for P passes:
//   k_rs_upsweep  per-tile digit histograms of every pass at once (original order)
//   k_rs_reduce   per pass: digit totals over the tiles (the upsweep zeroed them, its look-back flags, tickets)
//   k_rs_scatter  one launch per pass: tile digit counts -> publish -> stable in-tile ranks (wave ballots over the
//                 digit bits, rounds in index order) -> LDS reorder by digit -> decoupled look-back (one thread per
//                 digit; tiles take tickets in start order, so a tile only waits on running ones) -> coalesced stores
// rocPRIM's onesweep needs 3 + 3P launches (histogram memset, per pass a look-back memset and a block-id reset);
// sorts up to RS_OWN_MAX pairs are launch-bound, so the launch count is their cost; larger ones go to rocPRIM.
constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 8;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
constexpr int RS_BINS = 256;
constexpr int RS_MAXP = 8;
constexpr unsigned RS_AGG = 1u << 30, RS_PREFIX = 2u << 30, RS_VAL = (1u << 30) - 1;
// above this size rocPRIM's onesweep (1024-thread tiles) moves the data faster than these 2048-item tiles; below
// it the sorts are launch-bound and the fewer launches here win
constexpr size_t RS_OWN_MAX = (size_t)1 << 21;

struct RsPass {
    int shift;
    unsigned mask;
};
struct RsPasses {
    RsPass p[RS_MAXP];
    int np;
};

__global__ __launch_bounds__(RS_THREADS) void k_rs_upsweep(const unsigned long long* __restrict__ keys, int n, RsPasses ps,
                                                           unsigned* __restrict__ tile_hist, int ntiles,
                                                           unsigned* __restrict__ look, unsigned* __restrict__ tickets,
                                                           unsigned* __restrict__ totals) {
    __shared__ unsigned h[RS_MAXP][RS_BINS];
    const int tid = threadIdx.x;
    for (int p = 0; p < ps.np; ++p) {
        h[p][tid] = 0;
        look[((size_t)p * ntiles + blockIdx.x) * RS_BINS + tid] = 0u;  // this tile's look-back flags, every pass
    }
    if (blockIdx.x == 0) {
        if (tid < RS_MAXP) tickets[tid] = 0u;
        for (int p = 0; p < ps.np; ++p) totals[p * RS_BINS + tid] = 0u;
    }
    __syncthreads();
    const int base = blockIdx.x * RS_TILE;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const int i = base + r * RS_THREADS + tid;
        if (i < n) {
            const unsigned long long k = keys[i];
            for (int p = 0; p < ps.np; ++p) atomicAdd(&h[p][(unsigned)(k >> ps.p[p].shift) & ps.p[p].mask], 1u);
        }
    }
    __syncthreads();
    for (int p = 0; p < ps.np; ++p) tile_hist[((size_t)p * ntiles + blockIdx.x) * RS_BINS + tid] = h[p][tid];
}

__device__ inline unsigned block_exclusive_scan_256(unsigned v, unsigned* sh) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int d = 1; d < RS_BINS; d <<= 1) {
        const unsigned o = tid >= d ? sh[tid - d] : 0u;
        __syncthreads();
        sh[tid] += o;
        __syncthreads();
    }
    const unsigned incl = sh[tid];
    __syncthreads();
    return incl - v;
}

// per pass: digit totals over the tiles; grid (passes, RS_RED_BLOCKS), each block sums every RS_RED_BLOCKS-th tile
// and adds its partial totals atomically (the upsweep zeroed them)
constexpr int RS_RED_BLOCKS = 64;
__global__ __launch_bounds__(RS_THREADS) void k_rs_reduce(const unsigned* __restrict__ tile_hist, int ntiles,
                                                          unsigned* __restrict__ totals) {
    const int p = blockIdx.x, d = threadIdx.x;
    const unsigned* th = tile_hist + (size_t)p * ntiles * RS_BINS;
    unsigned acc[4] = {0u, 0u, 0u, 0u};
    int t = blockIdx.y;
    for (; t + 3 * RS_RED_BLOCKS < ntiles; t += 4 * RS_RED_BLOCKS) {
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += th[(size_t)(t + u * RS_RED_BLOCKS) * RS_BINS + d];
    }
    for (; t < ntiles; t += RS_RED_BLOCKS) acc[0] += th[(size_t)t * RS_BINS + d];
    const unsigned sum = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    if (sum) atomicAdd(&totals[p * RS_BINS + d], sum);
}

constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_CHUNK = RS_TILE / RS_WAVES;  // items per wave: a contiguous run of the tile

__global__ __launch_bounds__(RS_THREADS) void k_rs_scatter(const unsigned long long* __restrict__ kin,
                                                           const unsigned* __restrict__ vin,
                                                           unsigned long long* __restrict__ kout,
                                                           unsigned* __restrict__ vout, int n, RsPass ps,
                                                           const unsigned* __restrict__ totals, unsigned* look,
                                                           unsigned* ticket) {
    __shared__ unsigned long long s_keys[RS_TILE];
    __shared__ unsigned s_vals[RS_TILE];
    __shared__ unsigned s_start[RS_BINS], s_excl[RS_BINS], s_scan[RS_BINS];
    __shared__ unsigned s_wrun[RS_WAVES][RS_BINS];
    __shared__ int s_tile;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = (int)atomicAdd(ticket, 1u);
#pragma unroll
    for (int q = 0; q < RS_WAVES; ++q) s_wrun[q][tid] = 0u;
    __syncthreads();
    const int tile = s_tile;
    const int base = tile * RS_TILE;
    const int wbase = base + w * RS_CHUNK;  // this wave's contiguous run: items wbase + r * 64 + lane
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    unsigned long long key[RS_ITEMS];
    unsigned val[RS_ITEMS], dig[RS_ITEMS], wpos[RS_ITEMS];
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const int i = wbase + r * 64 + lane;
        const bool ok = i < n;
        key[r] = ok ? kin[i] : 0ull;
        val[r] = ok ? vin[i] : 0u;
        dig[r] = ok ? ((unsigned)(key[r] >> ps.shift) & ps.mask) : RS_BINS;
    }
    // stable ranks inside the wave's run: rounds in index order, lanes in order.  The wave's running digit
    // counts live in LDS and only this wave touches them (program order, no barriers).
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const bool ok = dig[r] < RS_BINS;
        unsigned long long eq = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (dig[r] >> b) & 1u;
            const unsigned long long bb = __ballot(bit);
            eq &= bit ? bb : ~bb;
        }
        const unsigned rk = (unsigned)__popcll(eq & lt);
        const unsigned d = ok ? dig[r] : 0u;
        const unsigned before = s_wrun[w][d];
        wpos[r] = before + rk;
        if (ok && rk == 0) s_wrun[w][d] = before + (unsigned)__popcll(eq);
    }
    __syncthreads();
    // tile digit counts (published for the look-back; tile 0: already the inclusive prefix), tile-local digit
    // starts, and each wave's offset inside a digit
    unsigned wb[RS_WAVES];
    unsigned c = 0u;
#pragma unroll
    for (int q = 0; q < RS_WAVES; ++q) {
        wb[q] = c;
        c += s_wrun[q][tid];
    }
    __hip_atomic_store(&look[(size_t)tile * RS_BINS + tid], (tile == 0 ? RS_PREFIX : RS_AGG) | c, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    const unsigned start = block_exclusive_scan_256(c, s_scan);  // contains barriers
    const unsigned goff = block_exclusive_scan_256(totals[tid], s_scan);  // global start of digit tid
    s_start[tid] = start;
#pragma unroll
    for (int q = 0; q < RS_WAVES; ++q) s_wrun[q][tid] = start + wb[q];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r)
        if (dig[r] < RS_BINS) {
            const unsigned pos = s_wrun[w][dig[r]] + wpos[r];
            s_keys[pos] = key[r];
            s_vals[pos] = val[r];
        }
    // decoupled look-back: thread d sums the digit-d counts of the preceding tiles
    unsigned excl = 0u;
    if (tile > 0) {
        for (int t = tile - 1; t >= 0;) {
            const unsigned v = __hip_atomic_load(&look[(size_t)t * RS_BINS + tid], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            const unsigned f = v & ~RS_VAL;
            if (f == 0u) continue;  // tile t has not published yet: it is running (it took an earlier ticket)
            excl += v & RS_VAL;
            if (f == RS_PREFIX) break;
            --t;
        }
        __hip_atomic_store(&look[(size_t)tile * RS_BINS + tid], RS_PREFIX | (excl + c), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    s_excl[tid] = goff + excl;
    __syncthreads();
    const int cnt = n - base < RS_TILE ? n - base : RS_TILE;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const int idx = r * RS_THREADS + tid;
        if (idx < cnt) {
            const unsigned long long k = s_keys[idx];
            const unsigned d = (unsigned)(k >> ps.shift) & ps.mask;
            const unsigned dst = s_excl[d] + (unsigned)idx - s_start[d];
            kout[dst] = k;
            vout[dst] = s_vals[idx];
        }
    }
}

ot_status sort_pairs_u64_u32(const unsigned long long* kin, unsigned long long* kout, const unsigned* vin,
                             unsigned* vout, size_t n, int end_bit, hipStream_t stream, int scratch_slot) {
    if (n == 0) return OT_OK;
#ifndef OT_SORT_ROCPRIM
    if (n <= RS_OWN_MAX) {
    if (end_bit < 1) end_bit = 1;
    RsPasses ps{};
    ps.np = (end_bit + 7) / 8;
    if (ps.np > RS_MAXP) ps.np = RS_MAXP;
    for (int p = 0; p < ps.np; ++p) {
        ps.p[p].shift = 8 * p;
        const int bits = std::min(8, end_bit - 8 * p);
        ps.p[p].mask = (1u << bits) - 1u;
    }
    const int ntiles = (int)((n + RS_TILE - 1) / RS_TILE);
    const size_t hist_words = (size_t)ps.np * ntiles * RS_BINS;
    const size_t bytes = 2 * n * (sizeof(unsigned long long) + sizeof(unsigned)) + 2 * hist_words * 4 +
                         (size_t)RS_MAXP * RS_BINS * 4 + RS_MAXP * 4 + 256;
    char* ws = (char*)scratch(bytes, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "sort scratch allocation failed");
    unsigned long long* ka = (unsigned long long*)ws;
    unsigned long long* kb = ka + n;
    unsigned* va = (unsigned*)(kb + n);
    unsigned* vb = va + n;
    unsigned* tile_hist = vb + n;
    unsigned* look = tile_hist + hist_words;
    unsigned* totals = look + hist_words;
    unsigned* tickets = totals + (size_t)RS_MAXP * RS_BINS;
    hipLaunchKernelGGL(k_rs_upsweep, dim3(ntiles), dim3(RS_THREADS), 0, stream, kin, (int)n, ps, tile_hist, ntiles,
                       look, tickets, totals);
    hipLaunchKernelGGL(k_rs_reduce, dim3(ps.np, std::min(ntiles, RS_RED_BLOCKS)), dim3(RS_THREADS), 0, stream,
                       (const unsigned*)tile_hist, ntiles, totals);
    const unsigned long long* ks = kin;
    const unsigned* vs = vin;
    for (int p = 0; p < ps.np; ++p) {
        const bool last = p == ps.np - 1;
        unsigned long long* kd = last ? kout : (p % 2 == 0 ? ka : kb);
        unsigned* vd = last ? vout : (p % 2 == 0 ? va : vb);
        hipLaunchKernelGGL(k_rs_scatter, dim3(ntiles), dim3(RS_THREADS), 0, stream, ks, vs, kd, vd, (int)n, ps.p[p],
                           (const unsigned*)(totals + p * RS_BINS), look + (size_t)p * ntiles * RS_BINS, tickets + p);
        ks = kd;
        vs = vd;
    }
    OT_LAUNCH_CHECK();
    return OT_OK;
    }
#endif
    {
    size_t tmp = 0;
    OT_HIP_TRY(rocprim::radix_sort_pairs<BigSortConfig>(nullptr, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit,
                                                        stream));
    void* ws = scratch(tmp + 16, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "sort scratch allocation failed");
    OT_HIP_TRY(rocprim::radix_sort_pairs<BigSortConfig>(ws, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, stream));
    return OT_OK;
    }
}

ot_status sort_pairs_u32_u32(const unsigned* kin, unsigned* kout, const unsigned* vin, unsigned* vout, size_t n,
                             int end_bit, hipStream_t stream, int scratch_slot) {
    if (n == 0) return OT_OK;
    if (end_bit < 1) end_bit = 1;
    size_t tmp = 0;
    OT_HIP_TRY(rocprim::radix_sort_pairs<SortConfig>(nullptr, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, stream));
    void* ws = scratch(tmp + 16, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "sort scratch allocation failed");
    OT_HIP_TRY(rocprim::radix_sort_pairs<SortConfig>(ws, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, stream));
    return OT_OK;
}

}  // namespace ot

// test hook (not part of the drop-in boundary): the library's stable radix sort on device arrays
extern "C" ot_status otx_sort_pairs_u64_u32(const unsigned long long* kin, unsigned long long* kout, const unsigned* vin,
                                           unsigned* vout, int64_t n, int32_t end_bit, void* stream) {
    if (n < 0 || (n > 0 && (!kin || !kout || !vin || !vout)) || end_bit < 1 || end_bit > 64)
        return ot::fail(OT_ERR_INVALID_ARGUMENT, "[sort] invalid arguments");
    ot_status st = ot::sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)n, end_bit, (hipStream_t)stream, 3);
    if (st != OT_OK) return st;
    OT_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return OT_OK;
}

namespace ot {

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
