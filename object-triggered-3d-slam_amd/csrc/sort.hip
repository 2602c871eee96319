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
using BigSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 16>, rocprim::kernel_config<512, 16>, 8,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

// ------------------------------------------------------------------------------------------------------------
// Own stable LSD radix sort (8- or 9-bit digits, whichever needs fewer passes), P + 2 launches for P passes:
//   k_rs_upsweep  per-tile digit histograms of every pass at once (original order)
//   k_rs_reduce   per pass and segment: digit totals over the segment's tiles (the upsweep zeroed them, its
//                 look-back flags, tickets)
//   k_rs_scatter  one launch per pass: tile digit counts -> publish -> stable in-tile ranks (wave ballots over the
//                 digit bits, rounds in index order) -> LDS reorder by digit -> decoupled look-back (one thread per
//                 digit; tiles take tickets in start order, so a tile only waits on running ones) -> coalesced stores
// Segmented form: the input is a concatenation of independent segments (a batch's frames); each is sorted in place
// (its own digit offsets, a look-back that stops at its first tile), all of them in the same launches.  Tiles never
// straddle segments.
// rocPRIM's onesweep needs 3 + 3P launches (histogram memset, per pass a look-back memset and a block-id reset);
// sorts up to RS_OWN_MAX pairs are launch-bound, so the launch count is their cost; larger unsegmented ones go to
// rocPRIM.
// D-bit digits: 2^D bins and 2^D threads per tile (one digit per thread in the histogram, scan and look-back);
// D = 8 (256 threads) or 9 (512 threads: a 25..27-bit key in 3 passes instead of 4)
template <int D>
struct Rs {
    static constexpr int BINS = 1 << D;
    static constexpr int THREADS = BINS;
    static constexpr int WAVES = THREADS / 64;
};
constexpr int RS_MAXP = 8;
constexpr int RS_MAXSEG = 64;
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
// segments: [start[s], start[s + 1]) of the input; their tiles [tile[s], tile[s + 1]).  dlen (device, nullable): the
// segment holds only its first dlen[s] items (the rest of its range is capacity; tiles past the end sort nothing)
struct RsSegs {
    int nseg;
    int start[RS_MAXSEG + 1];
    int tile[RS_MAXSEG + 1];
    const int* dlen;
};
__device__ inline int rs_seg_end(const RsSegs& sg, int s) {
    return sg.dlen ? sg.start[s] + sg.dlen[s] : sg.start[s + 1];
}

__device__ inline int rs_segment(const RsSegs& sg, int tile) {
    int s = 0;
    while (s + 1 < sg.nseg && sg.tile[s + 1] <= tile) ++s;
    return s;
}

template <typename KeyT, int RS_ITEMS, int D>
__global__ __launch_bounds__(Rs<D>::THREADS) void k_rs_upsweep(const KeyT* __restrict__ keys, RsSegs sg, RsPasses ps,
                                                           unsigned* __restrict__ tile_hist, int ntiles,
                                                           unsigned* __restrict__ look, unsigned* __restrict__ tickets,
                                                           unsigned* __restrict__ totals) {
    constexpr int RS_THREADS = Rs<D>::THREADS, RS_BINS = Rs<D>::BINS;
    constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
    __shared__ unsigned h[RS_MAXP][RS_BINS];
    const int tid = threadIdx.x;
    for (int p = 0; p < ps.np; ++p) {
        h[p][tid] = 0;
        look[((size_t)p * ntiles + blockIdx.x) * RS_BINS + tid] = 0u;  // this tile's look-back flags, every pass
    }
    if (blockIdx.x == 0) {
        if (tid < RS_MAXP) tickets[tid] = 0u;
        for (int i = 0; i < ps.np * sg.nseg; ++i) totals[(size_t)i * RS_BINS + tid] = 0u;
    }
    __syncthreads();
    const int s = rs_segment(sg, blockIdx.x);
    const int base = sg.start[s] + (blockIdx.x - sg.tile[s]) * RS_TILE;
    const int end = rs_seg_end(sg, s);
    // per lane and pass a run of equal digits, flushed into the LDS histogram when the digit changes: a lane takes
    // RS_ITEMS CONSECUTIVE keys (a histogram does not care about order), and neighbouring keys of the spatially coherent
    // inputs share their higher digits, so most passes add one run per lane instead of one LDS atomic per key (same-bin
    // LDS atomics from a whole wave serialise)
    unsigned cur[RS_MAXP], cnt[RS_MAXP];
#pragma unroll
    for (int p = 0; p < RS_MAXP; ++p) cur[p] = cnt[p] = 0u;
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const int i = base + tid * RS_ITEMS + r;
        if (i < end) {
            const KeyT k = keys[i];
#pragma unroll
            for (int p = 0; p < RS_MAXP; ++p) {
                if (p >= ps.np) break;
                const unsigned d = (unsigned)(k >> ps.p[p].shift) & ps.p[p].mask;
                if (d != cur[p]) {
                    if (cnt[p]) atomicAdd(&h[p][cur[p]], cnt[p]);
                    cur[p] = d;
                    cnt[p] = 0u;
                }
                ++cnt[p];
            }
        }
    }
#pragma unroll
    for (int p = 0; p < RS_MAXP; ++p)
        if (p < ps.np && cnt[p]) atomicAdd(&h[p][cur[p]], cnt[p]);
    __syncthreads();
    for (int p = 0; p < ps.np; ++p) tile_hist[((size_t)p * ntiles + blockIdx.x) * RS_BINS + tid] = h[p][tid];
}

template <int BINS>
__device__ inline unsigned block_exclusive_scan(unsigned v, unsigned* sh) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int d = 1; d < BINS; d <<= 1) {
        const unsigned o = tid >= d ? sh[tid - d] : 0u;
        __syncthreads();
        sh[tid] += o;
        __syncthreads();
    }
    const unsigned incl = sh[tid];
    __syncthreads();
    return incl - v;
}

// per pass and segment: digit totals over the segment's tiles; grid (passes * segments, RS_RED_BLOCKS), each block
// sums every RS_RED_BLOCKS-th tile of its segment and adds its partial totals atomically (the upsweep zeroed them)
constexpr int RS_RED_BLOCKS = 64;
template <int D>
__global__ __launch_bounds__(Rs<D>::THREADS) void k_rs_reduce(const unsigned* __restrict__ tile_hist, int ntiles, RsSegs sg,
                                                          unsigned* __restrict__ totals) {
    constexpr int RS_BINS = Rs<D>::BINS;
    const int p = blockIdx.x / sg.nseg, s = blockIdx.x % sg.nseg, d = threadIdx.x;
    const unsigned* th = tile_hist + (size_t)p * ntiles * RS_BINS;
    const int t1 = sg.tile[s + 1];
    unsigned acc[4] = {0u, 0u, 0u, 0u};
    int t = sg.tile[s] + blockIdx.y;
    for (; t + 3 * RS_RED_BLOCKS < t1; t += 4 * RS_RED_BLOCKS) {
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += th[(size_t)(t + u * RS_RED_BLOCKS) * RS_BINS + d];
    }
    for (; t < t1; t += RS_RED_BLOCKS) acc[0] += th[(size_t)t * RS_BINS + d];
    const unsigned sum = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    if (sum) atomicAdd(&totals[(size_t)blockIdx.x * RS_BINS + d], sum);
}

template <typename KeyT, int RS_ITEMS, int D>
__global__ __launch_bounds__(Rs<D>::THREADS) void k_rs_scatter(const KeyT* __restrict__ kin, const unsigned* __restrict__ vin,
                                                           KeyT* __restrict__ kout, unsigned* __restrict__ vout,
                                                           RsSegs sg, RsPass ps, const unsigned* __restrict__ totals,
                                                           unsigned* look, unsigned* ticket) {
    constexpr int RS_THREADS = Rs<D>::THREADS, RS_BINS = Rs<D>::BINS, RS_WAVES = Rs<D>::WAVES;
    constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
    constexpr int RS_CHUNK = RS_TILE / RS_WAVES;  // items per wave: a contiguous run of the tile
    __shared__ KeyT s_keys[RS_TILE];
    __shared__ unsigned s_vals[RS_TILE];
    __shared__ unsigned s_start[RS_BINS], s_excl[RS_BINS], s_scan[RS_BINS];
    __shared__ unsigned s_wrun[RS_WAVES][RS_BINS];
    __shared__ int s_tile;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = (int)atomicAdd(ticket, 1u);
#pragma unroll
    for (int q = 0; q < RS_WAVES; ++q) s_wrun[q][tid] = 0u;
    __syncthreads();
    // tickets go round-robin over the segments (ticket = i * nseg + s: tile i of segment s), so the running tiles
    // spread over every segment's independent look-back chain
    const int sgi = s_tile % sg.nseg;
    const int first = sg.tile[sgi];  // the segment's first tile
    const int tile = first + s_tile / sg.nseg;
    if (tile >= sg.tile[sgi + 1]) return;  // past the end of a shorter segment (block-uniform)
    const int base = sg.start[sgi] + (tile - first) * RS_TILE;
    const int n = rs_seg_end(sg, sgi);  // end of the segment's items
    // a tile wholly in a segment's unused capacity (dlen): nothing to move, and no tile of the segment with items
    // looks back past it (block-uniform)
    if (base >= n && tile > first) return;
    const int wbase = base + w * RS_CHUNK;  // this wave's contiguous run: items wbase + r * 64 + lane
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    KeyT key[RS_ITEMS];
    unsigned val[RS_ITEMS], dig[RS_ITEMS], wpos[RS_ITEMS];
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const int i = wbase + r * 64 + lane;
        const bool ok = i < n;
        key[r] = ok ? kin[i] : (KeyT)0;
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
        for (int b = 0; b < D; ++b) {
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
    // tile digit counts (published for the look-back; a segment's first tile: already the inclusive prefix),
    // tile-local digit starts, and each wave's offset inside a digit
    unsigned wb[RS_WAVES];
    unsigned c = 0u;
#pragma unroll
    for (int q = 0; q < RS_WAVES; ++q) {
        wb[q] = c;
        c += s_wrun[q][tid];
    }
    __hip_atomic_store(&look[(size_t)tile * RS_BINS + tid], (tile == first ? RS_PREFIX : RS_AGG) | c, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    const unsigned start = block_exclusive_scan<RS_BINS>(c, s_scan);  // contains barriers
    const unsigned goff = (unsigned)sg.start[sgi] +
                          block_exclusive_scan<RS_BINS>(totals[(size_t)sgi * RS_BINS + tid], s_scan);  // digit tid's start
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
    // decoupled look-back inside the segment: thread d sums the digit-d counts of the preceding tiles
    unsigned excl = 0u;
    if (tile > first) {
        for (int t = tile - 1; t >= first;) {
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
            const KeyT k = s_keys[idx];
            const unsigned d = (unsigned)(k >> ps.shift) & ps.mask;
            const unsigned dst = s_excl[d] + (unsigned)idx - s_start[d];
            kout[dst] = k;
            vout[dst] = s_vals[idx];
        }
    }
}

// the own sort over segments (host segment offsets seg[0..nseg], seg[0] = 0, seg[nseg] = n)
template <typename KeyT, int RS_ITEMS, int D>
static ot_status rs_sort(const KeyT* kin, KeyT* kout, const unsigned* vin, unsigned* vout, const int64_t* seg, int nseg,
                         int end_bit, hipStream_t stream, int scratch_slot, const int* dlen = nullptr) {
    constexpr int RS_THREADS = Rs<D>::THREADS, RS_BINS = Rs<D>::BINS;
    constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
    const size_t n = (size_t)seg[nseg];
    if (n == 0) return OT_OK;
    if (nseg < 1 || nseg > RS_MAXSEG || n > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[sort] too many segments");
    if (end_bit < 1) end_bit = 1;
    RsPasses ps{};
    ps.np = (end_bit + D - 1) / D;
    if (ps.np > RS_MAXP) ps.np = RS_MAXP;
    for (int p = 0; p < ps.np; ++p) {
        ps.p[p].shift = D * p;
        const int bits = std::min(D, end_bit - D * p);
        ps.p[p].mask = (1u << bits) - 1u;
    }
    RsSegs sg{};
    sg.nseg = nseg;
    sg.dlen = dlen;
    int ntiles = 0;
    for (int s = 0; s < nseg; ++s) {
        sg.start[s] = (int)seg[s];
        sg.tile[s] = ntiles;
        ntiles += (int)((seg[s + 1] - seg[s] + RS_TILE - 1) / RS_TILE);
    }
    sg.start[nseg] = (int)n;
    sg.tile[nseg] = ntiles;
    int maxt = 0;
    for (int s = 0; s < nseg; ++s) maxt = std::max(maxt, sg.tile[s + 1] - sg.tile[s]);
    const size_t hist_words = (size_t)ps.np * ntiles * RS_BINS;
    const size_t bytes = 2 * n * (sizeof(KeyT) + sizeof(unsigned)) + 2 * hist_words * 4 +
                         (size_t)RS_MAXP * nseg * RS_BINS * 4 + RS_MAXP * 4 + 512;
    char* ws = (char*)scratch(bytes, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "sort scratch allocation failed");
    KeyT* ka = (KeyT*)ws;
    KeyT* kb = ka + n;
    unsigned* va = (unsigned*)(kb + n);
    unsigned* vb = va + n;
    unsigned* tile_hist = vb + n;
    unsigned* look = tile_hist + hist_words;
    unsigned* totals = look + hist_words;
    unsigned* tickets = totals + (size_t)RS_MAXP * nseg * RS_BINS;
    hipLaunchKernelGGL((k_rs_upsweep<KeyT, RS_ITEMS, D>), dim3(ntiles), dim3(RS_THREADS), 0, stream, kin, sg, ps, tile_hist, ntiles,
                       look, tickets, totals);
    hipLaunchKernelGGL(k_rs_reduce<D>, dim3(ps.np * nseg, RS_RED_BLOCKS), dim3(RS_THREADS), 0, stream,
                       (const unsigned*)tile_hist, ntiles, sg, totals);
    const KeyT* ks = kin;
    const unsigned* vs = vin;
    for (int p = 0; p < ps.np; ++p) {
        const bool last = p == ps.np - 1;
        KeyT* kd = last ? kout : (p % 2 == 0 ? ka : kb);
        unsigned* vd = last ? vout : (p % 2 == 0 ? va : vb);
        hipLaunchKernelGGL((k_rs_scatter<KeyT, RS_ITEMS, D>), dim3(maxt * nseg), dim3(RS_THREADS), 0, stream, ks, vs, kd, vd, sg, ps.p[p],
                           (const unsigned*)(totals + (size_t)p * nseg * RS_BINS), look + (size_t)p * ntiles * RS_BINS,
                           tickets + p);
        ks = kd;
        vs = vd;
    }
    OT_LAUNCH_CHECK();
    return OT_OK;
}

ot_status sort_pairs_u64_u32(const unsigned long long* kin, unsigned long long* kout, const unsigned* vin,
                             unsigned* vout, size_t n, int end_bit, hipStream_t stream, int scratch_slot) {
    if (n == 0) return OT_OK;
    if (n <= RS_OWN_MAX) {
        const int64_t seg[2] = {0, (int64_t)n};
        if ((end_bit + 8) / 9 < (end_bit + 7) / 8)  // 9-bit digits when they save a pass
            return rs_sort<unsigned long long, 4, 9>(kin, kout, vin, vout, seg, 1, end_bit, stream, scratch_slot);
        return rs_sort<unsigned long long, 8, 8>(kin, kout, vin, vout, seg, 1, end_bit, stream, scratch_slot);
    }
    size_t tmp = 0;
    OT_HIP_TRY(rocprim::radix_sort_pairs<BigSortConfig>(nullptr, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit,
                                                        stream));
    void* ws = scratch(tmp + 16, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "sort scratch allocation failed");
    OT_HIP_TRY(rocprim::radix_sort_pairs<BigSortConfig>(ws, tmp, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, stream));
    return OT_OK;
}

constexpr int SEGSORT_ITEMS = 16;  // items per thread of the segmented sort's tiles (4096-item tiles; 2048 / 6144
                                   // measured slower)

ot_status sort_segments_u32_u32(const unsigned* kin, unsigned* kout, const unsigned* vin, unsigned* vout,
                                const int64_t* seg, int nseg, int end_bit, hipStream_t stream, int scratch_slot,
                                const int* dlen) {
    // (10-bit digits, 1024-thread tiles, 3 passes for the 28..30-bit configs[2] keys: measured slower, 624 + 85 us vs
    // 516 + 52 us per 32-frame batch for 4 passes of 8 bits)
    // 9-bit digits (512-thread tiles of the same 4096 items) when they save a pass: 25..27-bit keys in 3 passes
    if ((end_bit + 8) / 9 < (end_bit + 7) / 8)
        return rs_sort<unsigned, SEGSORT_ITEMS / 2, 9>(kin, kout, vin, vout, seg, nseg, end_bit, stream, scratch_slot,
                                                       dlen);
    return rs_sort<unsigned, SEGSORT_ITEMS, 8>(kin, kout, vin, vout, seg, nseg, end_bit, stream, scratch_slot, dlen);
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

// test hook: the segmented sort (seg: host offsets [nseg + 1])
extern "C" ot_status otx_sort_segments_u32_u32(const unsigned* kin, unsigned* kout, const unsigned* vin, unsigned* vout,
                                              const int64_t* seg, int32_t nseg, int32_t end_bit, void* stream) {
    if (!seg || nseg < 1 || nseg > 64 || end_bit < 1 || end_bit > 32 || seg[0] != 0)
        return ot::fail(OT_ERR_INVALID_ARGUMENT, "[sort] invalid arguments");
    for (int s = 0; s < nseg; ++s)
        if (seg[s + 1] < seg[s]) return ot::fail(OT_ERR_INVALID_ARGUMENT, "[sort] invalid segments");
    if (seg[nseg] > 0 && (!kin || !kout || !vin || !vout)) return ot::fail(OT_ERR_INVALID_ARGUMENT, "[sort] invalid arguments");
    ot_status st = ot::sort_segments_u32_u32(kin, kout, vin, vout, seg, nseg, end_bit, (hipStream_t)stream, 3);
    if (st != OT_OK) return st;
    OT_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return OT_OK;
}


