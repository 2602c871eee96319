// compact.h — order-preserving (stable) stream compaction for gfx950.
//
// Three launches: (1) each 256-thread workgroup counts the items its predicate keeps (4 consecutive items
// per lane, wave ballot + popcount, no atomics); (2) one workgroup scans the per-workgroup counts;
// (3) each workgroup re-evaluates the predicate and writes the kept items at
// workgroup-offset + wave-offset + lane prefix (ballot/mbcnt).  Output order == input index order, which is
// the row-major order Open3D produces for unprojection and the order numpy boolean masks keep.
#pragma once

#include <algorithm>

#include "common.h"

namespace ot {

constexpr int CMP_THREADS = 256;
constexpr int CMP_ITEMS = 4;
constexpr int CMP_TILE = CMP_THREADS * CMP_ITEMS;

// inclusive scan within a wave (64 lanes)
__device__ inline int wave_incl_scan(int v) {
    const int lane = (int)lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// exclusive scan over a 256-thread workgroup; returns the exclusive prefix and the block total
__device__ inline int block_excl_scan_256(int v, int& total) {
    __shared__ int wsum[CMP_THREADS / 64];
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    int inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < CMP_THREADS / 64; ++w) {
        int s = wsum[w];
        if (w < wid) off += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return off + inc - v;
}

template <class Pred>
__global__ __launch_bounds__(CMP_THREADS) void k_compact_count(int64_t n, Pred pred, int* block_counts) {
    const int64_t tile = (int64_t)blockIdx.x * CMP_TILE;
    int c = 0;
#pragma unroll
    for (int k = 0; k < CMP_ITEMS; ++k) {
        const int64_t i = tile + (int64_t)k * CMP_THREADS + threadIdx.x;  // lane-strided, as the emit pass
        if (i < n && pred(i)) ++c;
    }
    c = wave_sum(c);
    __shared__ int ws[CMP_THREADS / 64];
    if (lane_id() == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < CMP_THREADS / 64; ++w) t += ws[w];
        block_counts[blockIdx.x] = t;
    }
}

// single workgroup (1024 threads) exclusive scan of `n` ints in place; writes the grand total to *total
// (internal linkage: every translation unit gets its own copy)
namespace {
__global__ __launch_bounds__(1024) void k_scan_inplace(int* v, int n, int64_t* total) {
    __shared__ int wsum[16];
    __shared__ long long carry_s;
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int i = base + threadIdx.x;
        const int x = (i < n) ? v[i] : 0;
        int inc = wave_incl_scan(x);
        if (lane == 63) wsum[wid] = inc;
        __syncthreads();
        int off = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            int s = wsum[w];
            if (w < wid) off += s;
            tot += s;
        }
        const long long carry = carry_s;
        if (i < n) v[i] = (int)(carry + off + inc - x);
        __syncthreads();
        if (threadIdx.x == 0) carry_s = carry + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry_s;
}
}  // namespace


// Emit: a workgroup's tile of CMP_TILE items is walked in CMP_ITEMS lane-strided slices (item = tile + k*256 +
// lane), so consecutive lanes emit consecutive output positions and the emit functor's stores coalesce; slice k's
// kept items precede slice k+1's, which keeps the global input order.
template <class Pred, class Emit>
__global__ __launch_bounds__(CMP_THREADS) void k_compact_emit(int64_t n, Pred pred, Emit emit,
                                                              const int* block_offsets) {
    __shared__ int wsum[CMP_ITEMS][CMP_THREADS / 64];
    const int64_t tile = (int64_t)blockIdx.x * CMP_TILE;
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    bool keep[CMP_ITEMS];
    int pre[CMP_ITEMS];
#pragma unroll
    for (int k = 0; k < CMP_ITEMS; ++k) {
        const int64_t i = tile + (int64_t)k * CMP_THREADS + threadIdx.x;
        keep[k] = (i < n) && pred(i);
        int tot;
        pre[k] = wave_excl_count(keep[k], tot);
        if (lane == 0) wsum[k][wid] = tot;
    }
    __syncthreads();
    int pos = block_offsets[blockIdx.x];
#pragma unroll
    for (int k = 0; k < CMP_ITEMS; ++k) {
        int off = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < CMP_THREADS / 64; ++w) {
            const int c = wsum[k][w];
            off += (w < wid) ? c : 0;
            tot += c;
        }
        if (keep[k]) emit(tile + (int64_t)k * CMP_THREADS + threadIdx.x, (int64_t)(pos + off + pre[k]));
        pos += tot;
    }
}

// Host driver: runs the three launches on `stream` and returns the kept count on the host (synchronises).
template <class Pred, class Emit>
ot_status compact(int64_t n, Pred pred, Emit emit, hipStream_t stream, int64_t* n_out_host, int scratch_slot) {
    const int64_t nblocks = (n + CMP_TILE - 1) / CMP_TILE;
    if (n <= 0) {
        *n_out_host = 0;
        return OT_OK;
    }
    if (nblocks > (int64_t)0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "compaction input too large");
    char* ws = (char*)scratch(sizeof(int) * (size_t)nblocks + 64, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    int64_t* d_total = (int64_t*)ws;
    int* d_counts = (int*)(ws + 64);
    hipLaunchKernelGGL((k_compact_count<Pred>), dim3((unsigned)nblocks), dim3(CMP_THREADS), 0, stream, n, pred,
                       d_counts);
    hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(1024), 0, stream, d_counts, (int)nblocks, d_total);
    hipLaunchKernelGGL((k_compact_emit<Pred, Emit>), dim3((unsigned)nblocks), dim3(CMP_THREADS), 0, stream, n,
                       pred, emit, (const int*)d_counts);
    OT_LAUNCH_CHECK();
    int64_t tot = 0;
    OT_HIP_TRY(hipMemcpyAsync(&tot, d_total, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    *n_out_host = tot;
    return OT_OK;
}

// Segment heads of a sorted key array AND the segment index of every item, in one stable compaction:
// heads[s] = first position of segment s, seg[i] = segment of item i (= number of heads <= i, minus one).
namespace {
__global__ __launch_bounds__(CMP_THREADS) void k_segments_emit(int64_t n, const unsigned long long* __restrict__ keys,
                                                               const int* __restrict__ block_offsets,
                                                               int* __restrict__ heads, int* __restrict__ seg) {
    __shared__ int wsum[CMP_ITEMS][CMP_THREADS / 64];
    const int64_t tile = (int64_t)blockIdx.x * CMP_TILE;
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    bool head[CMP_ITEMS];
    int pre[CMP_ITEMS];
#pragma unroll
    for (int k = 0; k < CMP_ITEMS; ++k) {
        const int64_t i = tile + (int64_t)k * CMP_THREADS + threadIdx.x;
        head[k] = (i < n) && (i == 0 || keys[i] != keys[i - 1]);
        int tot;
        pre[k] = wave_excl_count(head[k], tot);
        if (lane == 0) wsum[k][wid] = tot;
    }
    __syncthreads();
    int pos = block_offsets[blockIdx.x];
#pragma unroll
    for (int k = 0; k < CMP_ITEMS; ++k) {
        int off = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < CMP_THREADS / 64; ++w) {
            const int c = wsum[k][w];
            off += (w < wid) ? c : 0;
            tot += c;
        }
        const int64_t i = tile + (int64_t)k * CMP_THREADS + threadIdx.x;
        const int my = pos + off + pre[k];  // segments starting before item i (exclusive)
        if (i < n) {
            if (head[k]) heads[my] = (int)i;
            seg[i] = my + (head[k] ? 1 : 0) - 1;
        }
        pos += tot;
    }
}
}  // namespace

// segment heads of a sorted key array (i == 0 or key changes) -> their positions
struct SegHeadPred {
    const unsigned long long* keys;
    __device__ bool operator()(int64_t i) const { return i == 0 || keys[i] != keys[i - 1]; }
};
struct SegHeadEmit {
    int* heads;
    __device__ void operator()(int64_t i, int64_t pos) const { heads[pos] = (int)i; }
};

// Host driver of k_segments_emit (count with SegHeadPred, scan, emit); returns the segment count (synchronises).
inline ot_status compact_segments(int64_t n, const unsigned long long* keys, int* heads, int* seg, hipStream_t stream,
                                  int64_t* n_seg_host, int scratch_slot) {
    const int64_t nblocks = (n + CMP_TILE - 1) / CMP_TILE;
    *n_seg_host = 0;
    if (n <= 0) return OT_OK;
    char* ws = (char*)scratch(sizeof(int) * (size_t)nblocks + 64, scratch_slot);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    int64_t* d_total = (int64_t*)ws;
    int* d_counts = (int*)(ws + 64);
    hipLaunchKernelGGL((k_compact_count<SegHeadPred>), dim3((unsigned)nblocks), dim3(CMP_THREADS), 0, stream, n,
                       SegHeadPred{keys}, d_counts);
    hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(1024), 0, stream, d_counts, (int)nblocks, d_total);
    hipLaunchKernelGGL(k_segments_emit, dim3((unsigned)nblocks), dim3(CMP_THREADS), 0, stream, n, keys,
                       (const int*)d_counts, heads, seg);
    OT_LAUNCH_CHECK();
    int64_t tot = 0;
    OT_HIP_TRY(hipMemcpyAsync(&tot, d_total, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    *n_seg_host = tot;
    return OT_OK;
}

// per-axis min / max of float64 [n][3] points via order-preserving u64 atomics (exact)
struct Bounds {
    unsigned long long mn[3];
    unsigned long long mx[3];
    int err;
};

// per-axis min / max of float64 [n][3] points, exact and order independent: each workgroup reduces its slice
// through the wave shuffles and LDS into one partial record; a one-workgroup pass folds the partials.
// (No same-address atomics: 1024 workgroups x 6 contended u64 atomics cost ~0.3 ms on MI355X.)
constexpr int BOUNDS_BLOCKS = 512;
namespace {
__global__ __launch_bounds__(256) void k_bounds_partial(const double* __restrict__ xyz, int64_t n,
                                                        unsigned long long* __restrict__ part) {
    unsigned long long mn[3] = {~0ull, ~0ull, ~0ull}, mx[3] = {0, 0, 0};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const unsigned long long o = dbl_to_ordered(xyz[i * 3 + a]);
            mn[a] = o < mn[a] ? o : mn[a];
            mx[a] = o > mx[a] ? o : mx[a];
        }
    }
    __shared__ unsigned long long s[4][6];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            unsigned long long t = __shfl_xor(mn[a], off, 64);
            mn[a] = t < mn[a] ? t : mn[a];
            t = __shfl_xor(mx[a], off, 64);
            mx[a] = t > mx[a] ? t : mx[a];
        }
    }
    if (lane_id() == 0)
        for (int a = 0; a < 3; ++a) {
            s[threadIdx.x >> 6][a] = mn[a];
            s[threadIdx.x >> 6][3 + a] = mx[a];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int q = threadIdx.x;
        unsigned long long v = s[0][q];
        for (int w = 1; w < 4; ++w) v = q < 3 ? (s[w][q] < v ? s[w][q] : v) : (s[w][q] > v ? s[w][q] : v);
        part[blockIdx.x * 6 + q] = v;
    }
}

__global__ __launch_bounds__(256) void k_bounds_final(const unsigned long long* __restrict__ part, int nb, Bounds* b) {
    __shared__ unsigned long long s[256][6];
    unsigned long long v[6] = {~0ull, ~0ull, ~0ull, 0, 0, 0};
    for (int i = threadIdx.x; i < nb; i += 256)
        for (int q = 0; q < 6; ++q) {
            const unsigned long long x = part[i * 6 + q];
            v[q] = q < 3 ? (x < v[q] ? x : v[q]) : (x > v[q] ? x : v[q]);
        }
    for (int q = 0; q < 6; ++q) s[threadIdx.x][q] = v[q];
    __syncthreads();
    if (threadIdx.x < 6) {
        const int q = threadIdx.x;
        unsigned long long r = s[0][q];
        for (int i = 1; i < 256; ++i) r = q < 3 ? (s[i][q] < r ? s[i][q] : r) : (s[i][q] > r ? s[i][q] : r);
        if (q < 3) b->mn[q] = r;
        else b->mx[q - 3] = r;
        if (q == 0) b->err = 0;
    }
}
}  // namespace

// Launch both passes; `part` needs BOUNDS_BLOCKS * 6 u64.
inline void launch_bounds(const double* xyz, int64_t n, Bounds* b, unsigned long long* part, hipStream_t stream) {
    const unsigned nb = (unsigned)std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), BOUNDS_BLOCKS);
    hipLaunchKernelGGL(k_bounds_partial, dim3(nb), dim3(256), 0, stream, xyz, n, part);
    hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(256), 0, stream, (const unsigned long long*)part, (int)nb, b);
}

}  // namespace ot
