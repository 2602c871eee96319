// mesh_ops.hip — TriangleMesh::ComputeVertexNormals and SamplePointsUniformly on MI355X
// (reconstruct_rgbd_filter.py:113 and :123).
//
// Normals: Open3D adds each triangle's unnormalised normal (v1-v0) x (v2-v0) to its three vertices in
// triangle order, then normalises.  To reproduce that summation order without atomics, the 3T (vertex,
// corner) pairs are radix-sorted by vertex (stable => triangle order kept) and one lane per vertex sums its
// contributions sequentially — bit-identical to the sequential CPU loop.
// Sampling: areas 0.5*|(p0-p1) x (p0-p2)| in float64; the area sum and the normalised CDF are Open3D's
// sequential recurrences (one lane, float64) so n_t = round(cdf_t * N) matches the CPU exactly; points are
// then generated in parallel, one lane per output point: binary search of its triangle in the n_t array,
// r1/r2 from a counter-based RNG (splitmix64 of seed + counter; Open3D's mt19937 is unseeded), barycentric
// a = 1 - sqrt(r1), b = sqrt(r1)(1 - r2), c = sqrt(r1) r2.
#include <atomic>
#include <cstring>
#include <functional>
#include <vector>

#include "chain.h"
#include "compact.h"
#include "sort.h"

namespace ot {

__global__ __launch_bounds__(256) void k_tri_normals(const double* __restrict__ V, const int32_t* __restrict__ T,
                                                     int64_t nt, double* __restrict__ TN,
                                                     unsigned long long* keys, unsigned* vals) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nt) return;
    const int32_t a = T[t * 3], b = T[t * 3 + 1], c = T[t * 3 + 2];
    double tn[3];
    triangle_normal(V, a, b, c, tn);
    TN[t * 3 + 0] = tn[0];
    TN[t * 3 + 1] = tn[1];
    TN[t * 3 + 2] = tn[2];
    keys[t * 3 + 0] = (unsigned long long)(unsigned)a;
    keys[t * 3 + 1] = (unsigned long long)(unsigned)b;
    keys[t * 3 + 2] = (unsigned long long)(unsigned)c;
    vals[t * 3 + 0] = (unsigned)(t * 3 + 0);
    vals[t * 3 + 1] = (unsigned)(t * 3 + 1);
    vals[t * 3 + 2] = (unsigned)(t * 3 + 2);
}

// first position of each vertex in the sorted key array (or -1 when the vertex has no triangle)
__global__ __launch_bounds__(256) void k_vertex_starts(const unsigned long long* __restrict__ skeys, int64_t m,
                                                       int* start) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    if (i == 0 || skeys[i] != skeys[i - 1]) start[skeys[i]] = (int)i;
}

__global__ __launch_bounds__(256) void k_vertex_normals(const unsigned long long* __restrict__ skeys,
                                                        const unsigned* __restrict__ svals, int64_t m,
                                                        const int* __restrict__ start, const double* __restrict__ TN,
                                                        int64_t nv, double* __restrict__ N) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= nv) return;
    double n[3] = {0.0, 0.0, 0.0};
    int64_t j = start[v];
    if (j >= 0) {
        for (; j < m && skeys[j] == (unsigned long long)v; ++j) {
            const int64_t t = svals[j] / 3;
            n[0] += TN[t * 3 + 0];
            n[1] += TN[t * 3 + 1];
            n[2] += TN[t * 3 + 2];
        }
    }
    finish_vertex_normal(n);
    N[v * 3 + 0] = n[0];
    N[v * 3 + 1] = n[1];
    N[v * 3 + 2] = n[2];
}

// ------------------------------------------------------------------------------------------- sampling
// TriangleMesh::GetTriangleArea: 0.5 * |(p0 - p1) x (p0 - p2)|, Open3D's expression order
__device__ inline double tri_area(const double* __restrict__ V, const int32_t* __restrict__ T, int64_t t) {
    const double* p0 = V + (int64_t)T[t * 3] * 3;
    const double* p1 = V + (int64_t)T[t * 3 + 1] * 3;
    const double* p2 = V + (int64_t)T[t * 3 + 2] * 3;
    double x[3], y[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        x[d] = p0[d] - p1[d];
        y[d] = p0[d] - p2[d];
    }
    const double c0 = x[1] * y[2] - x[2] * y[1];
    const double c1 = x[2] * y[0] - x[0] * y[2];
    const double c2 = x[0] * y[1] - x[1] * y[0];
    return 0.5 * sqrt((c0 * c0 + c1 * c1) + c2 * c2);
}
// bsum (nullable): the block's 256 areas are chunk blockIdx.x of the area-sum chain (CHAIN_CH values per chunk), and
// their approximate sum -- only a binade guess for the chain walk, any order will do -- is k_chain_bsum's output, formed
// here instead of in a launch of its own
__device__ inline void areas_block(const double* __restrict__ V, const int32_t* __restrict__ T, int64_t nt,
                                   double* __restrict__ area, double* __restrict__ bsum) {
    static_assert(CHAIN_CH == 256, "one areas workgroup per chain chunk");
    __shared__ double s_w[4];
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const double a = t < nt ? tri_area(V, T, t) : 0.0;
    if (t < nt) area[t] = a;
    if (!bsum) return;  // grid-uniform
    const double w = wave_sum(a);
    if (lane_id() == 0) s_w[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
}
__global__ __launch_bounds__(256) void k_tri_areas(const double* __restrict__ V, const int32_t* __restrict__ T,
                                                   int64_t nt, double* __restrict__ area, double* __restrict__ bsum) {
    areas_block(V, T, nt, area, bsum);
}
// k_tri_areas that also lands the sampler's uploaded tables (blob words -> dst) and zeroes its look-back words
// (zwords at zero) from block 0: the chains' table upload and the status memset ride on the first kernel of the chain
// instead of two launches of their own (~5 us each on one object's latency chain)
__global__ __launch_bounds__(256) void k_tri_areas_blob(const double* __restrict__ V, const int32_t* __restrict__ T,
                                                        int64_t nt, double* __restrict__ area, ArgBlob b,
                                                        unsigned long long* __restrict__ dst, int words,
                                                        unsigned long long* __restrict__ zero, int zwords,
                                                        double* __restrict__ bsum) {
    if (blockIdx.x == 0) {
        for (int i = threadIdx.x; i < words; i += 256) dst[i] = b.w[i];
        for (int i = threadIdx.x; i < zwords; i += 256) zero[i] = 0ull;
    }
    areas_block(V, T, nt, area, bsum);
}

// Open3D's sequential recurrences (GetSurfaceArea: s = (((a0 + a1) + a2) + ...), then the CDF loop
// cdf_t = a_t / s + cdf_{t-1}) are serial float64 chains whose every rounding must be reproduced.  They are
// computed exactly in parallel from one identity: while the running value s stays inside one binade
// [2^e, 2^(e+1)) (grid spacing u = 2^(e-52)), fl(s + a) = s + u * rint(a / u) for any a >= 0 that is not a tie
// (a / u exactly k + 1/2).  So inside a binade the chain is an INTEGER prefix sum of r_t = rint(a_t / u),
// independent of s.  The input is cut into 256-value chunks:
//   k_chain_bsum   approximate chunk sums (any order)            -> bsum
//   k_chain_guess  approximate exclusive prefix -> guessed binade e_b of s at each chunk start
//   k_chain_chunk  M_b = sum r_t at u_b = 2^(e_b-52), flag ties / negative / non-finite / r >= 2^53
//   k_chain_runs   runs = maximal stretches of unflagged chunks with one guessed binade (a flagged chunk is a run
//                  of its own): the inclusive prefix of M_b inside each run and every chunk's run end, in parallel
//   k_chain_walk   one wave per chain, one step per RUN instead of per 64 chunks: from the exact s (N = s / u) it
//                  accepts the longest stretch [b, k] of the run with e(s) == e_b and N + prefix <= 2^53 - 1
//                  (every intermediate sum stays inside the binade: the prefix is monotone, so the run end decides
//                  at once, else a 64-way search), records the segment (b, N, prefix base) and jumps to k + 1; any
//                  other chunk (s == 0, binade crossing, tie, wrong guess) is walked serially in Open3D's order
//   k_chain_emit   (CDF) every accepted chunk's values (N + prefix_t) * u, exact integers times 2^k, from its segment
// The guesses only decide which chunks take the fast path; every accepted value is proven exact by the walk's
// check, so any input (zeros, ties, NaN, huge ranges) gives the serial chain's bits.
constexpr int CH = CHAIN_CH;
constexpr int EX_NONE = -100000;       // no usable binade guess
constexpr long long R_MAX = 1ll << 53;

__device__ inline double pow2(int k) { return __longlong_as_double((long long)(k + 1023) << 52); }

// binade exponent of a positive finite s inside the range pow2() covers for both u and 1/u, else EX_NONE
__device__ inline int binade(double s) {
    if (!(s > 0.0) || !(s < 1e300)) return EX_NONE;
    const int e = (int)((__double_as_longlong(s) >> 52) & 0x7FF) - 1023;
    return e >= -960 ? e : EX_NONE;
}

__device__ inline void chunk_load4(const double* __restrict__ x, int64_t n, int64_t base, int lane, double v[4]) {
    const int64_t i = base + 4 * lane;
    if (i + 3 < n && ((reinterpret_cast<uintptr_t>(x) & 15) == 0)) {  // base is a multiple of 4: x's alignment decides
        const double2 p = *reinterpret_cast<const double2*>(x + i);
        const double2 q = *reinterpret_cast<const double2*>(x + i + 2);
        v[0] = p.x, v[1] = p.y, v[2] = q.x, v[3] = q.y;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = i + k < n ? x[i + k] : 0.0;
    }
}

__global__ __launch_bounds__(256) void k_chain_bsum(const ChainJob* __restrict__ jobs) {
    const ChainJob j = jobs[blockIdx.y];
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nb = (j.n + CH - 1) / CH;
    if (b >= nb) return;
    const int lane = threadIdx.x & 63;
    double v[4];
    chunk_load4(j.x, j.n, b * CH, lane, v);
    double s = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) j.bsum[b] = s;
}

// approximate exclusive prefix of the chunk sums -> guessed binade per chunk (and the prefix itself, kept in bsum):
// one 1024-thread block per chain, each thread a contiguous stretch of chunks, a wave-shuffle scan of the stretch
// totals and one of the 16 wave totals
__global__ __launch_bounds__(1024) void k_chain_guess(const ChainJob* __restrict__ jobs) {
    __shared__ double s_w[16];
    const ChainJob j = jobs[blockIdx.x];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t nb = (j.n + CH - 1) / CH, per = (nb + 1023) / 1024;
    const int64_t lo = t * per, hi = lo + per < nb ? lo + per : nb;
    double loc = 0.0;
    for (int64_t i = lo; i < hi; ++i) loc += j.bsum[i];
    double inc = loc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(inc, d);
        if (lane >= d) inc += o;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    double off = 0.0;
    for (int q = 0; q < w; ++q) off += s_w[q];
    double p = off + inc - loc;  // approximate exclusive prefix (only a guess)
    for (int64_t i = lo; i < hi; ++i) {
        j.ex[i] = binade(p);
        const double bi = j.bsum[i];
        j.bsum[i] = p;  // kept: the sampler's CDF chain guesses its binades from it (k_chain_cdf_prep)
        p += bi;
    }
}

__global__ __launch_bounds__(256) void k_chain_chunk(const ChainJob* __restrict__ jobs) {
    const ChainJob j = jobs[blockIdx.y];
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nb = (j.n + CH - 1) / CH;
    if (b >= nb) return;
    const int lane = threadIdx.x & 63;
    const int e = j.ex[b];
    bool bad = e == EX_NONE;
    long long r = 0;
    if (!bad) {
        double v[4];
        chunk_load4(j.x, j.n, b * CH, lane, v);
        const double scale = pow2(52 - e);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double m = v[k] * scale;  // exact: power-of-two scaling
            const bool ok = m >= 0.0 && m < (double)R_MAX && m - floor(m) != 0.5;
            bad |= !ok;
            r += ok ? (long long)rint(m) : 0;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
    const bool any_bad = __ballot(bad) != 0;
    if (lane == 0) {
        j.msum[b] = r < R_MAX ? r : R_MAX;  // saturated: such a chunk fails the walk's range check anyway
        j.kind[b] = any_bad ? 1 : 0;
    }
}

// The sampler's CDF chain prologue in one launch, after the area sum's walk: q_t = a_t / S (IEEE division, Open3D's
// triangle_areas[t] / surface_area), the chunk's binade guess from the SUM chain's approximate prefix at the chunk
// start over S (cdf at a chunk start ~ prefix / S: a guess only, the walk proves every accepted value), then
// k_chain_chunk's integer sum and flags -- instead of a division pass plus the chunk-sum, guess and chunk passes.
__global__ __launch_bounds__(256) void k_chain_cdf_prep(const ChainJob* __restrict__ sum_jobs,
                                                        const ChainJob* __restrict__ cdf_jobs) {
    const ChainJob js = sum_jobs[blockIdx.y], jc = cdf_jobs[blockIdx.y];
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nb = (jc.n + CH - 1) / CH;
    if (b >= nb) return;
    const int lane = threadIdx.x & 63;
    const double S = js.out[0];
    double v[4];
    chunk_load4(js.x, js.n, b * CH, lane, v);
    const int64_t i = b * CH + 4 * lane;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = v[k] / S;
    double* q = const_cast<double*>(jc.x);
    if (i + 3 < jc.n && ((reinterpret_cast<uintptr_t>(q) & 15) == 0)) {
        *reinterpret_cast<double2*>(q + i) = make_double2(v[0], v[1]);
        *reinterpret_cast<double2*>(q + i + 2) = make_double2(v[2], v[3]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k < jc.n) q[i + k] = v[k];
    }
    const int e = binade(js.bsum[b] / S);
    bool bad = e == EX_NONE;
    long long r = 0;
    if (!bad) {
        const double scale = pow2(52 - e);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (i + k >= jc.n) v[k] = 0.0;
            const double m = v[k] * scale;  // exact: power-of-two scaling
            const bool ok = m >= 0.0 && m < (double)R_MAX && m - floor(m) != 0.5;
            bad |= !ok;
            r += ok ? (long long)rint(m) : 0;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
    const bool any_bad = __ballot(bad) != 0;
    if (lane == 0) {
        jc.ex[b] = e;
        jc.msum[b] = r < R_MAX ? r : R_MAX;
        jc.kind[b] = any_bad ? 1 : 0;
    }
}

// One chunk from the exact s in Open3D's order, by integer segments: inside the binade of s every element that is
// not a tie, stays below 2^53 grid steps and keeps the running integer below 2^53 is one step of an integer prefix
// sum (the whole wave at once); the first element that breaks this is added by one exact float64 add (s + a) and the
// next segment starts after it.  A chunk costs one wave prefix per binade crossing / tie / special value instead of
// 256 dependent adds.  CDF values are stored as they are produced.  The segment is a single wave's latency chain, so
// its cross-lane steps avoid LDS: the prefix is a DPP scan inside rows of 16 plus the row totals read by readlane,
// the first bad / crossing element is found by a ballot and one readlane, and broadcasts are readlanes.
// (Round 4, measured and reverted: scanning the binade of s and the next one in one pass and resolving a crossing's
// second segment from the precomputed prefixes made the walks 57.6 / 77.6 -> 70.7 / 96.4 us per configs[3] mesh: a
// segment's cost is its dependent ballot / readlane chain, which the second grid does not remove, not its scan.)
__device__ inline long long readlane64(long long v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)v, l), hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ inline double readlane_f64(double v, int l) { return __longlong_as_double(readlane64(__double_as_longlong(v), l)); }
// the smallest per-lane index (CH when no lane has one): lanes hold ascending index ranges, so it is the value of the
// first lane that has one
__device__ inline int wave_first_idx(int idx) {
    const unsigned long long m = __ballot(idx < CH);
    return m ? __builtin_amdgcn_readlane(idx, __ffsll((long long)m) - 1) : CH;
}

// The segment arithmetic stays in float64: every grid count r = rint(a / u) and every prefix the walk keeps is an integer
// below 2^53, so float64 adds of them are exact; a prefix past the binade's limit may round, but rounding is monotone
// and the limit T = 2^53 - 1 - N is representable, so "prefix > T" is decided exactly.  No int64 conversions on the
// single wave's latency chain.
template <int CTRL>
__device__ inline double dpp_row_shr_f64(double v) {  // lanes without a source in their row of 16 read +0.0
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ inline double wave_incl_scan_f64(double v, int lane) {
    v += dpp_row_shr_f64<0x111>(v);
    v += dpp_row_shr_f64<0x112>(v);
    v += dpp_row_shr_f64<0x114>(v);
    v += dpp_row_shr_f64<0x118>(v);  // inclusive inside each row of 16
    const double r0 = readlane_f64(v, 15), r1 = readlane_f64(v, 31), r2 = readlane_f64(v, 47);
    const int row = lane >> 4;
    return v + ((row >= 1 ? r0 : 0.0) + ((row >= 2 ? r1 : 0.0) + (row >= 3 ? r2 : 0.0)));
}

template <bool CDF>
__device__ inline double chain_serial_chunk(const ChainJob& j, int64_t b, double s, const double v[4], int lane,
                                            int& ti) {
    const int64_t base = b * CH;
    const int cnt = j.n - base < CH ? (int)(j.n - base) : CH;
    int pos = 0;
    auto mark = [&](int kind, int at) {  // test hook only (j.trace is null in every product call)
        if (j.trace) {
            if (lane == 0 && ti < j.trace_cap) {
                j.trace[2 * ti] = (unsigned long long)clock64();
                j.trace[2 * ti + 1] = (unsigned long long)kind | ((unsigned long long)at << 8);
            }
            ++ti;
        }
    };
    while (pos < cnt) {  // wave-uniform
        mark(5, pos);
        const int e = binade(s);
        int stop = pos;
        if (e != EX_NONE) {
            const double scale = pow2(52 - e), u = pow2(e - 52);
            const double N = s * scale;                    // exact integer in [2^52, 2^53)
            const double T = (double)(R_MAX - 1) - N;      // exact: the largest prefix that stays in the binade
            double incl[4], loc = 0.0;
            int bad = CH;  // first element of this lane the integer step cannot take
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int idx = 4 * lane + k;
                const double m = v[k] * scale;  // exact: power-of-two scaling
                const double r = rint(m);
                const bool ok = m >= 0.0 && m < (double)R_MAX && fabs(m - r) != 0.5;
                const bool act = idx >= pos && idx < cnt;
                loc += (act && ok) ? r : 0.0;
                incl[k] = loc;
                if (act && !ok && bad == CH) bad = idx;
                if (idx >= cnt && bad == CH) bad = idx;
            }
            const double excl = wave_incl_scan_f64(loc, lane) - loc;  // exact where it matters (see above)
            const int first_bad = wave_first_idx(bad);
            int cross = CH;  // first element whose running integer leaves the binade
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                incl[k] += excl;
                const int idx = 4 * lane + k;
                if (idx >= pos && idx < first_bad && incl[k] > T && cross == CH) cross = idx;
            }
            const int first_cross = wave_first_idx(cross);
            mark(6, pos);
            stop = first_bad < first_cross ? first_bad : first_cross;
            stop = stop < cnt ? stop : cnt;
            if (stop > pos) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int idx = 4 * lane + k;
                    if (CDF && idx >= pos && idx < stop) j.out[base + idx] = (N + incl[k]) * u;
                }
                const int last = stop - 1;
                const double mine = (last & 3) == 0 ? incl[0] : (last & 3) == 1 ? incl[1] : (last & 3) == 2 ? incl[2] : incl[3];
                s = (N + readlane_f64(mine, last >> 2)) * u;
            }
        }
        if (stop < cnt) {  // one exact float64 add, in Open3D's order
            const double mine = (stop & 3) == 0 ? v[0] : (stop & 3) == 1 ? v[1] : (stop & 3) == 2 ? v[2] : v[3];
            s = readlane_f64(mine, stop >> 2) + s;
            if (CDF && lane == 0) j.out[base + stop] = s;
            ++stop;
        }
        pos = stop;
    }
    return s;
}

// one block per chain: run heads (b == 0, guessed binade changes, a flagged chunk or the chunk after one), the
// inclusive prefix of M inside each run (saturated at 2^53: the walk only compares it against < 2^53) and each
// chunk's run end -- a segmented scan, then a reverse pass for the ends
__device__ inline bool run_head(const ChainJob& j, int64_t b) {
    return b == 0 || j.kind[b] != 0 || j.kind[b - 1] != 0 || j.ex[b] != j.ex[b - 1];
}

// segmented (flag, value) combine of the run prefix: a head restarts the sum; sums saturate at 2^53
__device__ inline long long sat_add(long long a, long long b) {
    const long long c = a + b;  // both <= 2^53: no overflow
    return c < R_MAX ? c : R_MAX;
}

constexpr int RUN_ITEMS = 4;  // consecutive chunks per thread: a 1024-thread tile covers 4096 chunks
// The runs of one chain by a whole 1024-thread workgroup: set_pre(b, inclusive run prefix), set_end(b, run end).
template <class Head, class SetPre, class SetEnd>
__device__ inline void chain_runs_block(const ChainJob& j, Head run_head, SetPre set_pre, SetEnd set_end) {
    __shared__ long long s_wv[16];
    __shared__ int s_wh[16];
    __shared__ long long s_cin[16];
    __shared__ int s_wn[16];
    __shared__ int s_nin[16];
    __shared__ long long s_carry;
    __shared__ int s_next;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t nb = (j.n + CH - 1) / CH;
    constexpr int TILE = 1024 * RUN_ITEMS;
    if (t == 0) {
        s_carry = 0;
        s_next = (int)nb;
    }
    __syncthreads();
    // forward: inclusive prefix of msum inside each run (segmented scan: a head restarts the sum)
    for (int64_t t0 = 0; t0 < nb; t0 += TILE) {
        const int64_t b0 = t0 + (int64_t)t * RUN_ITEMS;
        long long lv[RUN_ITEMS];
        int lh[RUN_ITEMS];
        long long v = 0;
        int h = 0;  // a head seen so far inside this thread's chunks
#pragma unroll
        for (int k = 0; k < RUN_ITEMS; ++k) {
            const int64_t b = b0 + k;
            const bool in = b < nb;
            const bool hd = !in || run_head(b);
            const long long x = in ? j.msum[b] : 0;
            v = hd ? x : sat_add(v, x);
            h |= hd ? 1 : 0;
            lv[k] = v;
            lh[k] = h;
        }
        // exclusive segmented prefix of the thread aggregates (v, h) inside the wave
        long long iv = v;
        int ih = h;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const long long tv = __shfl_up(iv, d);
            const int th = __shfl_up(ih, d);
            if (lane >= d) {
                iv = ih ? iv : sat_add(tv, iv);
                ih = ih | th;
            }
        }
        long long ev = __shfl_up(iv, 1);
        int eh = __shfl_up(ih, 1);
        if (lane == 0) ev = 0, eh = 0;
        if (lane == 63) {
            s_wv[w] = iv;
            s_wh[w] = ih;
        }
        __syncthreads();
        if (t == 0) {  // carry into each wave: 16 serial combines
            long long c = s_carry;
            for (int i = 0; i < 16; ++i) {
                s_cin[i] = c;
                c = s_wh[i] ? s_wv[i] : sat_add(c, s_wv[i]);
            }
            s_carry = c;
        }
        __syncthreads();
        const long long cin = eh ? ev : sat_add(s_cin[w], ev);  // the running value entering this thread's chunks
#pragma unroll
        for (int k = 0; k < RUN_ITEMS; ++k)
            if (b0 + k < nb) set_pre(b0 + k, lh[k] ? lv[k] : sat_add(cin, lv[k]));
        __syncthreads();
    }
    // backward: every chunk's run end = (first head after it) - 1, tile by tile from the end (suffix minimum)
    const int64_t tiles = (nb + TILE - 1) / TILE;
    for (int64_t q = tiles - 1; q >= 0; --q) {
        const int64_t b0 = q * TILE + (int64_t)t * RUN_ITEMS;
        int ln[RUN_ITEMS];
        int nx = 0x7FFFFFFF;  // first head after each chunk, from this thread's chunks (suffix)
#pragma unroll
        for (int k = RUN_ITEMS - 1; k >= 0; --k) {
            ln[k] = nx;  // heads after chunk b0 + k inside this thread, excluding b0 + k + 1 (added next)
            const int64_t b1 = b0 + k + 1;
            if (b1 < nb && run_head(b1)) ln[k] = (int)b1;
            nx = ln[k];
        }
        // nx = first head after chunk b0 within this thread; wave exclusive suffix minimum from later lanes
        int sm = nx;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int tv = __shfl_down(sm, d);
            if (lane + d < 64) sm = tv < sm ? tv : sm;
        }
        int later = __shfl_down(sm, 1);
        if (lane == 63) later = 0x7FFFFFFF;
        if (lane == 0) s_wn[w] = sm;
        __syncthreads();
        if (t == 0) {
            int c = s_next;
            for (int i = 15; i >= 0; --i) {
                s_nin[i] = c;
                c = s_wn[i] < c ? s_wn[i] : c;
            }
            s_next = c;
        }
        __syncthreads();
        const int after = later < s_nin[w] ? later : s_nin[w];  // first head after this thread's last chunk
#pragma unroll
        for (int k = 0; k < RUN_ITEMS; ++k) {
            const int nxt = ln[k] < after ? ln[k] : after;
            if (b0 + k < nb) set_end(b0 + k, nxt - 1);
        }
        __syncthreads();
    }
}
__global__ __launch_bounds__(1024) void k_chain_runs(const ChainJob* __restrict__ jobs) {
    const ChainJob j = jobs[blockIdx.x];
    chain_runs_block(
        j, [&](int64_t b) { return run_head(j, b); }, [&](int64_t b, long long v) { j.pre[b] = v; },
        [&](int64_t b, int e) { j.rend[b] = e; });
}

// The walk's per-chunk metadata (ex, run end, run prefix, kind), staged in LDS by the whole workgroup before the one
// walking wave starts: every walk step then reads LDS instead of making dependent global round trips (the walk is a
// single wave's latency chain: one object's sampling waits on it, round 4: sum / CDF walks 86 / 118 us per configs[3]
// mesh).  Chains with more chunks than WALK_LDS_CHUNKS read global memory as before.
constexpr int WALK_LDS_CHUNKS = 7168;  // 16 B + 1 B per chunk: 119 KiB of LDS (1.8 M values)
// STAGED: the accessors index the dynamic LDS array itself, so the compiler emits LDS reads (through a generic
// pointer it had to emit flat loads, whose latency sat on every walk step: ~1.5-2.3k cycles per step, r04n trace)
extern __shared__ int4 s_walk_meta[];
template <bool STAGED>
struct WalkMeta {
    const ChainJob* j;
    int64_t nb;
    __device__ int ex(int64_t b) const {
        if constexpr (STAGED) return s_walk_meta[b].x;
        else return j->ex[b];
    }
    __device__ int rend(int64_t b) const {
        if constexpr (STAGED) return s_walk_meta[b].y;
        else return j->rend[b];
    }
    __device__ long long pre(int64_t b) const {
        if constexpr (STAGED) {
            const int4 q = s_walk_meta[b];
            return (long long)(((unsigned long long)(unsigned)q.w << 32) | (unsigned)q.z);
        } else {
            return j->pre[b];
        }
    }
    __device__ int kind(int64_t b) const {
        if constexpr (STAGED) return (int)reinterpret_cast<const signed char*>(s_walk_meta + nb)[b];
        else return j->kind[b];
    }
};

template <bool CDF, bool STAGED>
__global__ __launch_bounds__(1024) void k_chain_walk(const ChainJob* __restrict__ jobs) {
    const ChainJob j = jobs[blockIdx.x];
    const int64_t nb = (j.n + CH - 1) / CH;
    if constexpr (STAGED) {  // the whole workgroup stages the metadata and forms the runs in LDS, then one wave walks
        // (k_chain_runs folded in: its launch and the global round trip of the run prefixes and ends were on one
        // object's critical path; the CDF chain's emission still reads the prefixes from global memory)
        signed char* s_kind = reinterpret_cast<signed char*>(s_walk_meta + nb);
        for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) {
            s_walk_meta[b].x = j.ex[b];
            s_kind[b] = (signed char)j.kind[b];
        }
        __syncthreads();
        chain_runs_block(
            j,
            [&](int64_t b) {  // run_head() on the staged copies
                return b == 0 || s_kind[b] != 0 || s_kind[b - 1] != 0 || s_walk_meta[b].x != s_walk_meta[b - 1].x;
            },
            [&](int64_t b, long long v) {
                const unsigned long long pv = (unsigned long long)v;
                s_walk_meta[b].z = (int)(unsigned)pv;
                s_walk_meta[b].w = (int)(unsigned)(pv >> 32);
                if (CDF) j.pre[b] = v;
            },
            [&](int64_t b, int e) { s_walk_meta[b].y = e; });
        __syncthreads();
    }
    if (threadIdx.x >= 64) return;
    // the walking wave is one object's latency chain: it takes the issue arbiter's first pick over co-resident waves of
    // other work (another object's integrate, a mesh's vertex normals)
    __builtin_amdgcn_s_setprio(3);
    const WalkMeta<STAGED> M{&j, nb};
    const int lane = threadIdx.x;
    double s = 0.0;  // sum: 0 + a_0 + ...;  cdf: cdf_0 = q_0 + 0.0 = q_0
    int nseg = 0;
    int64_t b = 0;
    // the values of chunk vb, loaded ahead: every step issues the load of its chunk before reading the metadata, and a
    // serial chunk issues its successor's, so a chunk walked serially rarely waits for memory (a crossing chunk
    // follows a fast step; serial chunks cluster where the running value is small)
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    int64_t vb = -1;
    int ti = 0;  // trace events written (test hook only: j.trace is null in every product call)
    auto mark = [&](int kind, int64_t chunk) {
        if (j.trace) {
            if (lane == 0 && ti < j.trace_cap) {
                j.trace[2 * ti] = (unsigned long long)clock64();
                j.trace[2 * ti + 1] = (unsigned long long)kind | ((unsigned long long)chunk << 8);
            }
            ++ti;
        }
    };
    while (b < nb) {  // wave-uniform control flow: every lane holds the same s and b
        mark(0, b);
        if (vb != b) {
            chunk_load4(j.x, j.n, b * CH, lane, v);
            vb = b;
        }
        const int k_b = M.kind(b), e_b = M.ex(b), re = M.rend(b);
        const bool head = b == 0 || M.rend(b - 1) < b;
        const long long base = head ? 0 : M.pre(b - 1);
        const long long p_re = M.pre(re);
        const int e = binade(s);
        if (e != EX_NONE && k_b == 0 && e_b == e && base < R_MAX) {  // (a saturated base proves nothing)
            const long long N = (long long)(s * pow2(52 - e));  // exact integer in [2^52, 2^53)
            const long long lim = R_MAX - 1 - N + base;        // chunk c is accepted while pre[c] <= lim
            int64_t k = re;
            if (p_re > lim) {  // the binade ends inside the run: 64-way search for the last accepted chunk
                int64_t lo = b - 1, hi = re;  // pre[lo] <= lim (lo = b - 1: none yet), pre[hi] > lim
                while (hi - lo > 1) {
                    const int64_t step = (hi - lo - 1 + 63) / 64;
                    const int64_t c = lo + 1 + (int64_t)lane * step;
                    const bool ok = c < hi && M.pre(c) <= lim;
                    const unsigned long long m = __ballot(ok);
                    const int L = __popcll(m);  // the accepted probes are a prefix (pre is monotone)
                    const int64_t nlo = L ? lo + 1 + (int64_t)(L - 1) * step : lo;
                    const int64_t cL = lo + 1 + (int64_t)L * step;
                    hi = L == 0 ? lo + 1 : (cL < hi ? cL : hi);
                    lo = nlo;
                }
                k = lo;
            }
            if (k >= b) {
                mark(p_re > lim ? 2 : 1, k);
                if (CDF && lane == 0) {
                    j.seg_b[nseg] = (int)b;
                    j.seg_n[nseg] = N;
                    j.seg_base[nseg] = base;
                }
                ++nseg;
                s = (double)(N + M.pre(k) - base) * pow2(e - 52);
                b = k + 1;
                continue;
            }
        }
        // not provable from s: walk this chunk serially (its values already in flight), chunk b + 1's load issued first
        double w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = v[q];
        if (b + 1 < nb) {
            chunk_load4(j.x, j.n, (b + 1) * CH, lane, v);
            vb = b + 1;
        }
        s = chain_serial_chunk<CDF>(j, b, s, w, lane, ti);
        mark(3, b);
        if (lane == 0) j.kind[b] = 2;
        ++b;
    }
    mark(4, nb);
    if (lane == 0) {
        if (!CDF) j.out[0] = s;
        j.nseg[0] = nseg;
    }
}

__global__ __launch_bounds__(256) void k_chain_emit(const ChainJob* __restrict__ jobs) {
    const ChainJob j = jobs[blockIdx.y];
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nb = (j.n + CH - 1) / CH;
    if (b >= nb || j.kind[b] == 2) return;  // serial chunks were written by the walk
    const int lane = threadIdx.x & 63;
    // this chunk's segment: the last one starting at or before it
    int lo = 0, hi = j.nseg[0];
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (j.seg_b[mid] <= b) lo = mid;
        else hi = mid;
    }
    const int e = j.ex[b];
    const double u = pow2(e - 52), scale = pow2(52 - e);
    const long long N = j.seg_n[lo] + (j.seg_b[lo] < b ? j.pre[b - 1] - j.seg_base[lo] : 0);
    double v[4];
    chunk_load4(j.x, j.n, b * CH, lane, v);
    long long r[4], loc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        loc += (long long)rint(v[k] * scale);
        r[k] = loc;
    }
    long long incl = loc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const long long t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    const long long base = N + incl - loc;
    double o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = (double)(base + r[k]) * u;
    const int64_t i = b * CH + 4 * lane;
    if (i + 3 < j.n) {
        *reinterpret_cast<double2*>(j.out + i) = make_double2(o[0], o[1]);
        *reinterpret_cast<double2*>(j.out + i + 2) = make_double2(o[2], o[3]);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k < j.n) j.out[i + k] = o[k];
    }
}

// the chains of n_jobs independent inputs (device job table), side by side
// prologue (true): chunk sums, binade guesses, integer chunk sums and flags; false: the caller produced those
// (k_chain_cdf_prep)
template <bool CDF>
// mark (nullable): recorded on `stream` just before the walk -- a single wave per chain, the rest of the GPU idle --
// for work on another stream to start beside it (the fused extraction's vertex normals)
// bsum_done: the chunk sums were formed by the kernel that produced the values (the sampler's areas)
void launch_chains(const ChainJob* djobs, int n_jobs, int64_t max_n, hipStream_t stream, bool prologue = true,
                   hipEvent_t mark = nullptr, bool bsum_done = false) {
    const int64_t nb = (max_n + CH - 1) / CH;
    const dim3 grid((unsigned)((nb + 3) / 4), (unsigned)n_jobs);
    if (prologue) {
        if (!bsum_done) hipLaunchKernelGGL(k_chain_bsum, grid, dim3(256), 0, stream, djobs);
        hipLaunchKernelGGL(k_chain_guess, dim3(n_jobs), dim3(1024), 0, stream, djobs);
        hipLaunchKernelGGL(k_chain_chunk, grid, dim3(256), 0, stream, djobs);
    }
    // metadata staged in LDS (and the runs formed there) when every job's chunks fit (max_n bounds them all)
    const bool staged = nb <= WALK_LDS_CHUNKS;
    if (!staged) hipLaunchKernelGGL(k_chain_runs, dim3(n_jobs), dim3(1024), 0, stream, djobs);
    if (mark) (void)hipEventRecord(mark, stream);  // (a failure is the thread's last error: the caller's launch check)
    if (staged) {
        const size_t lds_bytes = (size_t)nb * 17 + 16;
        static std::atomic<bool> attr_set[2] = {false, false};
        if (!attr_set[CDF].load()) {  // above 64 KiB of dynamic LDS the kernel must opt in (once per process)
            (void)hipFuncSetAttribute((const void*)k_chain_walk<CDF, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)((size_t)WALK_LDS_CHUNKS * 17 + 16));
            attr_set[CDF].store(true);
        }
        hipLaunchKernelGGL((k_chain_walk<CDF, true>), dim3(n_jobs), dim3(1024), lds_bytes, stream, djobs);
    } else {
        hipLaunchKernelGGL((k_chain_walk<CDF, false>), dim3(n_jobs), dim3(64), 0, stream, djobs);
    }
    if (CDF) hipLaunchKernelGGL(k_chain_emit, grid, dim3(256), 0, stream, djobs);
}

void launch_sum_chains(const ChainJob* djobs, int n_jobs, int64_t max_n, hipStream_t stream) {
    launch_chains<false>(djobs, n_jobs, max_n > 0 ? max_n : 1, stream);
}

__global__ __launch_bounds__(256) void k_round_counts(const double* __restrict__ cdf, int64_t nt, int64_t N,
                                                      long long* __restrict__ ncum) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nt) return;
    long long v = (long long)round(cdf[t] * (double)N);
    ncum[t] = v < N ? v : N;
}

__device__ inline double rng_u01(unsigned long long seed, unsigned long long ctr) {
    unsigned long long z = seed + (ctr + 1ull) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// barycentric weights of point k from the counter RNG
__device__ inline void sample_bary(unsigned long long seed, int64_t k, double& a, double& b, double& c) {
    const double r1 = rng_u01(seed, (unsigned long long)(2 * k)), r2 = rng_u01(seed, (unsigned long long)(2 * k + 1));
    const double s1 = sqrt(r1);
    a = 1.0 - s1, b = s1 * (1.0 - r2), c = s1 * r2;
}

// point k of the sampling: triangle t = first index with ncum[t] > k (the CPU loop fills points [ncum[t-1], ncum[t])
// from t), barycentric weights from the counter RNG; false: rounding shortfall (Open3D leaves those points zero)
__device__ inline bool sample_triangle(const long long* __restrict__ ncum, int64_t nt, int64_t k,
                                       unsigned long long seed, int64_t& t, double& a, double& b, double& c) {
    int64_t lo = 0, hi = nt;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (ncum[mid] > k) hi = mid;
        else lo = mid + 1;
    }
    if (lo >= nt) return false;
    t = lo;
    sample_bary(seed, k, a, b, c);
    return true;
}
__device__ inline void interp3(const double* __restrict__ A, int64_t i0, int64_t i1, int64_t i2, double a, double b,
                               double c, double out[3]) {
#pragma unroll
    for (int d = 0; d < 3; ++d) out[d] = (a * A[i0 * 3 + d] + b * A[i1 * 3 + d]) + c * A[i2 * 3 + d];
}

__global__ __launch_bounds__(256) void k_sample(const double* __restrict__ V, const double* __restrict__ VN,
                                                const double* __restrict__ VC, const int32_t* __restrict__ T,
                                                const long long* __restrict__ ncum, int64_t nt, int64_t N,
                                                unsigned long long seed, double* P, double* PN, double* PC) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= N) return;
    int64_t t;
    double a, b, c;
    double x[3] = {0, 0, 0}, n[3] = {0, 0, 0}, col[3] = {0, 0, 0};
    if (sample_triangle(ncum, nt, k, seed, t, a, b, c)) {
        const int64_t i0 = T[t * 3], i1 = T[t * 3 + 1], i2 = T[t * 3 + 2];
        interp3(V, i0, i1, i2, a, b, c, x);
        if (PN) interp3(VN, i0, i1, i2, a, b, c, n);
        if (PC) interp3(VC, i0, i1, i2, a, b, c, col);
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        P[k * 3 + d] = x[d];
        if (PN) PN[k * 3 + d] = n[d];
        if (PC) PC[k * 3 + d] = col[d];
    }
}

// The sampling and the Z mask of reconstruct_rgbd_filter.py:123-132 in one pass: the points with z >= z_min (NaN
// fails, as numpy's mask) in sampling order, xyz and colours only (the reference rebuilds its cloud from those two, so
// normals are not interpolated).  A workgroup takes MZ_TILE consecutive points in a ticket order, counts the kept
// ones and finds its output offset by a decoupled look-back over the job's earlier workgroups; grid (tiles, jobs).
// one point per lane: 4 per lane (98 workgroups for 100k points, 1.5 waves per CU) left the kernel latency-bound at
// 34 us whatever its search did (r04ab-r04ad)
constexpr int MZ_ITEMS = 1, MZ_TILE = 256 * MZ_ITEMS;
struct MinZJob {
    const double* V;
    const double* VC;
    const int32_t* T;
    const long long* ncum;
    int64_t nt;
    double* P;
    double* PC;
};
__device__ inline long long round_count(const double* __restrict__ cdf, int64_t t, int64_t N) {
    const long long v = (long long)round(cdf[t] * (double)N);
    return v < N ? v : N;
}
// ncum, and per tile of MZ_TILE points the triangle of its first point (tstart[tile] = the t with ncum[t - 1] <= k0 <
// ncum[t], nt past the last count; tstart[tiles] = nt): a tile's points then search only [tstart[tile], tstart[tile + 1]]
__global__ __launch_bounds__(256) void k_round_counts_jobs(const MinZJob* __restrict__ jobs, const double* const* cdfs,
                                                           int64_t N, long long* const* ncums, int tiles,
                                                           int* __restrict__ tstart) {
    const int j = blockIdx.y;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, nt = jobs[j].nt;
    if (t >= nt) return;
    const long long c = round_count(cdfs[j], t, N), prev = t > 0 ? round_count(cdfs[j], t - 1, N) : 0;
    ncums[j][t] = c;
    int* ts = tstart + (size_t)j * (tiles + 1);
    for (long long tl = (prev + MZ_TILE - 1) / MZ_TILE; tl < tiles && tl * MZ_TILE < c; ++tl) ts[tl] = (int)t;
    if (t == nt - 1)
        for (long long tl = (c + MZ_TILE - 1) / MZ_TILE; tl <= tiles; ++tl) ts[tl] = (int)nt;
}
constexpr int MZ_LDS = 8192;  // a tile's candidate counts staged in LDS (int32) when they fit (32 KiB)
// The tile's triangle search: its points fall to triangles [t_lo, t_top] (k_round_counts_jobs' tstart), whose counts
// are staged in LDS when they fit, so each point's upper-bound search is ~13 LDS steps instead of ~20 dependent global
// loads over the whole count array (r04ab: the kernel was 34 us for 100k points of a 0.56 M-triangle mesh)
__global__ __launch_bounds__(256) void k_sample_min_z(const MinZJob* __restrict__ jobs, int64_t N,
                                                      unsigned long long seed, double z_min, int tiles,
                                                      unsigned long long* status, int* ticket,
                                                      long long* __restrict__ kept, const int* __restrict__ tstart) {
    const int j = blockIdx.y;
    const MinZJob jb = jobs[j];
    __shared__ int s_tile;
    __shared__ int wsum[MZ_ITEMS][4];
    __shared__ long long s_excl;
    __shared__ int s_nc[MZ_LDS];
    if (threadIdx.x == 0) s_tile = atomicAdd(&ticket[j], 1);
    __syncthreads();
    const int tile = s_tile;  // tiles start in ticket order: the look-back only waits on running workgroups
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    const int* ts = tstart + (size_t)j * (tiles + 1);
    const int t_lo = ts[tile], t_next = ts[tile + 1];
    const int t_top = t_next < (int)jb.nt - 1 ? t_next : (int)jb.nt - 1;  // last candidate (inclusive)
    const int cnt = t_top - t_lo + 1;                                       // <= 0: every point is a shortfall
    const bool staged = cnt > 0 && cnt <= MZ_LDS && N <= 0x7FFFFFFF;       // block-uniform
    if (staged)
        for (int i = threadIdx.x; i < cnt; i += 256) s_nc[i] = (int)jb.ncum[t_lo + i];
    __syncthreads();
    // the items' searches in lockstep (one power-of-two descent shared by the MZ_ITEMS points of a lane: the block's
    // cnt fixes its steps), then every item's triangle corners, then their vertex rows -- each phase's loads issued
    // together instead of one point's dependent chain after another's
    double x[MZ_ITEMS][3], col[MZ_ITEMS][3];
    bool keep[MZ_ITEMS], found[MZ_ITEMS];
    int pre[MZ_ITEMS];
    int64_t tt[MZ_ITEMS];
    if (staged) {
        int pos[MZ_ITEMS];
#pragma unroll
        for (int i = 0; i < MZ_ITEMS; ++i) pos[i] = -1;  // largest index with count <= k
        int step = 1;
        while (step * 2 <= cnt) step *= 2;
        for (; step > 0; step >>= 1) {
#pragma unroll
            for (int i = 0; i < MZ_ITEMS; ++i) {
                const long long k = (long long)tile * MZ_TILE + i * 256 + threadIdx.x;
                const int q = pos[i] + step;
                if (q < cnt && (long long)s_nc[q] <= k) pos[i] = q;
            }
        }
#pragma unroll
        for (int i = 0; i < MZ_ITEMS; ++i) {
            const int64_t k = (int64_t)tile * MZ_TILE + i * 256 + threadIdx.x;
            tt[i] = (int64_t)t_lo + pos[i] + 1;
            found[i] = k < N && tt[i] < jb.nt;
        }
    } else {
#pragma unroll
        for (int i = 0; i < MZ_ITEMS; ++i) {
            const int64_t k = (int64_t)tile * MZ_TILE + i * 256 + threadIdx.x;
            double a, b, c;
            found[i] = k < N && cnt > 0 && sample_triangle(jb.ncum, jb.nt, k, seed, tt[i], a, b, c);
        }
    }
    int64_t corner[MZ_ITEMS][3];
#pragma unroll
    for (int i = 0; i < MZ_ITEMS; ++i)
#pragma unroll
        for (int d = 0; d < 3; ++d) corner[i][d] = found[i] ? jb.T[tt[i] * 3 + d] : 0;
#pragma unroll
    for (int i = 0; i < MZ_ITEMS; ++i) {
        const int64_t k = (int64_t)tile * MZ_TILE + i * 256 + threadIdx.x;
#pragma unroll
        for (int d = 0; d < 3; ++d) x[i][d] = col[i][d] = 0.0;
        if (found[i]) {
            double a, b, c;
            sample_bary(seed, k, a, b, c);
            interp3(jb.V, corner[i][0], corner[i][1], corner[i][2], a, b, c, x[i]);
            if (jb.PC) interp3(jb.VC, corner[i][0], corner[i][1], corner[i][2], a, b, c, col[i]);
        }
        keep[i] = k < N && x[i][2] >= z_min;
        int tot;
        pre[i] = wave_excl_count(keep[i], tot);
        if (lane == 0) wsum[i][wid] = tot;
    }
    __syncthreads();
    int n_keep = 0;
#pragma unroll
    for (int i = 0; i < MZ_ITEMS; ++i) n_keep += wsum[i][0] + wsum[i][1] + wsum[i][2] + wsum[i][3];
    if (threadIdx.x < 64) {  // decoupled look-back by wave 0
        const long long excl = lookback_wave(status + (int64_t)j * tiles, tile, (unsigned long long)n_keep);
        if (threadIdx.x == 0) {
            s_excl = excl;
            if (tile == tiles - 1) kept[j] = excl + n_keep;
        }
    }
    __syncthreads();
    long long pos = s_excl;
#pragma unroll
    for (int i = 0; i < MZ_ITEMS; ++i) {
        int off = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            off += w < wid ? wsum[i][w] : 0;
            tot += wsum[i][w];
        }
        if (keep[i]) {
            const long long o = pos + off + pre[i];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                jb.P[o * 3 + d] = x[i][d];
                if (jb.PC) jb.PC[o * 3 + d] = col[i][d];
            }
        }
        pos += tot;
    }
}

}  // namespace ot

using namespace ot;

extern "C" {

ot_status ot_mesh_compute_vertex_normals(const double* V, int64_t nv, const int32_t* T, int64_t nt, double* out,
                                         void* stream_) {
    hipStream_t stream = S(stream_);
    if (nv < 0 || nt < 0 || (nv > 0 && (!V || !out)) || (nt > 0 && !T))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ComputeVertexNormals] invalid arguments");
    if (nv == 0) return OT_OK;
    const int64_t m = nt * 3;
    if (m > 0x7FFFFFFF || nv > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[ComputeVertexNormals] mesh too large");
    char* ws = (char*)scratch((size_t)nt * 24 + (size_t)m * (8 + 8 + 4 + 4) + (size_t)nv * 4 + 1024, 16);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    double* TN = (double*)ws;
    unsigned long long* kin = (unsigned long long*)(TN + nt * 3);
    unsigned long long* kout = kin + m;
    unsigned* vin = (unsigned*)(kout + m);
    unsigned* vout = vin + m;
    int* start = (int*)(vout + m);
    OT_HIP_TRY(hipMemsetAsync(start, 0xFF, sizeof(int) * nv, stream));
    if (nt > 0) {
        hipLaunchKernelGGL(k_tri_normals, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, V, T, nt, TN, kin,
                           vin);
        OT_LAUNCH_CHECK();
        int bits = 1;
        while (bits < 63 && (nv >> bits) != 0) ++bits;
        ot_status st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)m, bits, stream, 3);
        if (st != OT_OK) return st;
        hipLaunchKernelGGL(k_vertex_starts, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, kout, m, start);
    }
    hipLaunchKernelGGL(k_vertex_normals, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, stream, kout, vout, m, start,
                       TN, nv, out);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

ot_status ot_mesh_sample_points_uniformly(const double* V, const double* VN, const double* VC, int64_t nv,
                                          const int32_t* T, int64_t nt, int64_t n_points, uint64_t seed, double* P,
                                          double* PN, double* PC, void* stream) {
    const ot_mesh_sample_job job{V, VN, VC, nv, T, nt, P, PN, PC};
    return ot_mesh_sample_points_uniformly_after(&job, 1, n_points, seed, nullptr, stream);
}

ot_status ot_mesh_sample_points_uniformly_batch(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points,
                                                uint64_t seed, void* stream) {
    return ot_mesh_sample_points_uniformly_after(jobs, n_jobs, n_points, seed, nullptr, stream);
}

}  // extern "C"

namespace ot {
// The fused sampler runs on the caller's stream.  (Until late round 4 it ran on a per-thread stream of the device's
// greatest priority, forked from the caller's, so that a fresh mesh's vertex normals queued elsewhere were dispatched
// behind its chain; with the normals deferred until the sampling is queued, the fork's cross-queue latency is all that
// remained of it.  Test hook otx_sampler_hi_stream(1) restores it for A/B timing.)
static bool g_sampler_hi = false;
struct HiStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr;
    int dev = -1;
};
static thread_local HiStream g_hi;
// ot_mesh_sample_points_min_z_async's pending call on this thread: its tables live in this thread's scratch slot 17 and
// pinned slots 0 / 1 until ot_mesh_sample_points_min_z_wait, so no other sampling may start on the thread before
struct MinZPending {
    bool active = false;
    hipStream_t s = nullptr;  // may be the null (default) stream
    int32_t n_jobs = 0;
};
static thread_local MinZPending g_minz;
static ot_status hi_stream_fork(hipStream_t caller, hipStream_t* out) {
    int dev = 0;
    OT_HIP_TRY(hipGetDevice(&dev));
    if (!g_hi.s || g_hi.dev != dev) {  // one per thread (and device: a thread that switches devices re-creates it)
        int least = 0, greatest = 0;
        OT_HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        OT_HIP_TRY(hipStreamCreateWithPriority(&g_hi.s, hipStreamNonBlocking, greatest));
        OT_HIP_TRY(hipEventCreateWithFlags(&g_hi.fork, hipEventDisableTiming));
        g_hi.dev = dev;
    }
    OT_HIP_TRY(hipEventRecord(g_hi.fork, caller));
    OT_HIP_TRY(hipStreamWaitEvent(g_hi.s, g_hi.fork, 0));
    *out = g_hi.s;
    return OT_OK;
}

// The area sums and CDFs of every job (SamplePointsUniformly's two serial float64 chains, run side by side) into
// scratch slot 17, followed by `extra` bytes for the caller, whose leading `upload` bytes travel to the device with the
// chain table in one copy: fill(host, dev) writes them once the layout is known.  cdf[j]: the job's CDF (device);
// ncum[j]: room for its rounded counts; *extra_dev: the caller's device region.
static ot_status sample_cdfs(const ot_mesh_sample_job* jobs, int32_t n_jobs, size_t extra, size_t upload,
                             const std::function<void(char*, char*)>& fill, size_t zero_off, size_t zero_bytes,
                             hipStream_t stream, std::vector<double*>& cdf, std::vector<long long*>& ncum,
                             char** extra_dev, hipEvent_t mark = nullptr, int mark_at = 0) {
    if (g_minz.active) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] an async sampling is pending");
    size_t bytes = 256;
    int64_t max_nt = 0;
    for (int j = 0; j < n_jobs; ++j) {
        const ot_mesh_sample_job& m = jobs[j];
        if (m.n_triangles <= 0) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] Input mesh has no triangles.");
        if (!m.vertices || !m.triangles || !m.out_xyz || (m.out_normals && !m.vertex_normals) ||
            (m.out_colors && !m.vertex_colors) || m.n_vertices <= 0)
            return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] invalid arguments");
        bytes += (size_t)m.n_triangles * 32 + 256 + chain_aux_bytes(m.n_triangles);
        max_nt = m.n_triangles > max_nt ? m.n_triangles : max_nt;
    }
    const size_t table = sizeof(ChainJob) * 2 * (size_t)n_jobs;
    char* ws = (char*)scratch(bytes + table + extra + 512, 17);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    // [sum chains | CDF chains | caller's upload], sent by upload_small (kernel arguments; pinned memory serves the
    // copy fallback of large tables, and the callers synchronise before returning, so the slot is free again)
    char* up = (char*)pinned_scratch(table + upload, 0);
    if (!up) return fail(OT_ERR_HIP, "pinned allocation failed");
    ChainJob* chain = (ChainJob*)up;
    std::vector<double*> sums(n_jobs), qs(n_jobs);
    cdf.assign(n_jobs, nullptr);
    ncum.assign(n_jobs, nullptr);
    char* cur = ws;
    for (int j = 0; j < n_jobs; ++j) {
        const int64_t nt = jobs[j].n_triangles, nt2 = (nt + 1) & ~(int64_t)1;
        sums[j] = (double*)cur;
        cdf[j] = sums[j] + 8;  // 64-B offset: 16-B aligned rows for the chains' double2 loads
        qs[j] = cdf[j] + nt2;
        ncum[j] = (long long*)(qs[j] + nt2);
        cur = (char*)(ncum[j] + nt2) + 64;
        cur = (char*)(((uintptr_t)cur + 63) & ~(uintptr_t)63);
        ChainJob cs{};
        cs.x = cdf[j], cs.n = nt, cs.out = sums[j];
        cur = chain_aux(cur, nt, cs);
        ChainJob cc = cs;
        cc.x = qs[j], cc.out = cdf[j];  // the CDF overwrites the areas once q = a / s is formed
        chain[j] = cs;
        chain[n_jobs + j] = cc;
    }
    ChainJob* djobs = (ChainJob*)(((uintptr_t)cur + 63) & ~(uintptr_t)63);
    *extra_dev = (char*)djobs + table;
    if (upload) fill(up + table, *extra_dev);
    // the tables (and the caller's zeroed words) land from the first areas launch when they fit its arguments
    const size_t blob_bytes = table + upload;
    const bool blob = blob_bytes <= UPLOAD_ARG_BYTES && (zero_off & 7) == 0 && (zero_bytes & 7) == 0;
    if (!blob) {
        ot_status ust = upload_small(djobs, up, blob_bytes, stream);
        if (ust != OT_OK) return ust;
        if (zero_bytes) OT_HIP_TRY(hipMemsetAsync(*extra_dev + zero_off, 0, zero_bytes, stream));
    }
    for (int j = 0; j < n_jobs; ++j) {
        const int64_t nt = jobs[j].n_triangles;
        const dim3 grid((unsigned)((nt + 255) / 256));
        if (blob && j == 0) {
            ArgBlob b;
            std::memcpy(b.w, up, blob_bytes);
            hipLaunchKernelGGL(k_tri_areas_blob, grid, dim3(256), 0, stream, jobs[j].vertices, jobs[j].triangles, nt,
                               cdf[j], b, (unsigned long long*)djobs, (int)((blob_bytes + 7) / 8),
                               (unsigned long long*)(*extra_dev + zero_off), (int)(zero_bytes / 8), chain[j].bsum);
        } else {
            hipLaunchKernelGGL(k_tri_areas, grid, dim3(256), 0, stream, jobs[j].vertices, jobs[j].triangles, nt,
                               cdf[j], chain[j].bsum);
        }
    }
    launch_chains<false>(djobs, n_jobs, max_nt, stream, true, mark_at == 1 ? mark : nullptr, true);
    const int64_t max_nb = (max_nt + CH - 1) / CH;
    hipLaunchKernelGGL(k_chain_cdf_prep, dim3((unsigned)((max_nb + 3) / 4), (unsigned)n_jobs), dim3(256), 0, stream,
                       (const ChainJob*)djobs, (const ChainJob*)(djobs + n_jobs));
    launch_chains<true>(djobs + n_jobs, n_jobs, max_nt, stream, false, mark_at == 2 ? mark : nullptr);
    OT_LAUNCH_CHECK();
    return OT_OK;
}
}  // namespace ot

extern "C" {

ot_status ot_mesh_sample_points_uniformly_after(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points,
                                                uint64_t seed, void* inputs_ready, void* stream_) {
    hipStream_t stream = S(stream_);
    if (n_points <= 0) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] number_of_points <= 0");
    if (n_jobs < 0 || (n_jobs > 0 && !jobs)) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] invalid jobs");
    if (n_jobs == 0) return OT_OK;
    std::vector<double*> cdf;
    std::vector<long long*> ncum;
    char* extra = nullptr;
    ot_status st = sample_cdfs(jobs, n_jobs, 0, 0, nullptr, 0, 0, stream, cdf, ncum, &extra);
    if (st != OT_OK) return st;
    // the vertex normals / colours the emission interpolates may still be in flight on another stream (the facade
    // computes the normals of a fresh mesh beside the area chains above, which read only V and T)
    if (inputs_ready) OT_HIP_TRY(hipStreamWaitEvent(stream, (hipEvent_t)inputs_ready, 0));
    for (int j = 0; j < n_jobs; ++j) {
        const ot_mesh_sample_job& m = jobs[j];
        const int64_t nt = m.n_triangles;
        hipLaunchKernelGGL(k_round_counts, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, cdf[j], nt,
                           n_points, ncum[j]);
        hipLaunchKernelGGL(k_sample, dim3((unsigned)((n_points + 255) / 256)), dim3(256), 0, stream, m.vertices,
                           m.out_normals ? m.vertex_normals : nullptr, m.out_colors ? m.vertex_colors : nullptr,
                           m.triangles, ncum[j], nt, n_points, (unsigned long long)seed, m.out_xyz, m.out_normals,
                           m.out_colors);
    }
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));  // the host job table is released on return
    return OT_OK;
}

}  // extern "C"

namespace ot {
// The fused sampler's launches (on the caller's stream); the kept counts land in pinned slot 1 once it drains.  *hs:
// the stream to wait on.
static ot_status min_z_enqueue(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points, uint64_t seed,
                               double z_min, void* stream_, hipStream_t* hs, hipEvent_t mark = nullptr,
                               int mark_at = 0) {
    hipStream_t stream = S(stream_);
    if (g_sampler_hi) {
        ot_status fst = hi_stream_fork(S(stream_), &stream);
        if (fst != OT_OK) return fst;
    }
    if (n_points > ((int64_t)1 << 40)) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] too many points");
    const int64_t tiles64 = (n_points + MZ_TILE - 1) / MZ_TILE;
    if (tiles64 > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] too many points");
    const int tiles = (int)tiles64;
    // caller region: [MinZJob x n | cdf ptrs | ncum ptrs] (uploaded) | align 64 | i64 [n] (spare) | ticket i32 [n] |
    // align 64 | status u64 [n][tiles] (zeroed) | align 64 | tstart i32 [n][tiles + 1]
    const size_t up_bytes = (sizeof(MinZJob) + 16) * (size_t)n_jobs;
    const size_t zero_off = (up_bytes + 63) & ~(size_t)63;
    const size_t status_off = zero_off + (((size_t)n_jobs * 12 + 63) & ~(size_t)63);
    const size_t zero_end = status_off + (size_t)n_jobs * tiles * 8;
    const size_t tstart_off = (zero_end + 63) & ~(size_t)63;  // tstart i32 [n][tiles + 1] (every entry written)
    const size_t total = tstart_off + (size_t)n_jobs * (tiles + 1) * 4;
    std::vector<double*> cdf;
    std::vector<long long*> ncum;
    char* extra = nullptr;
    auto fill = [&](char* h, char*) {
        MinZJob* mj = (MinZJob*)h;
        const double** cp = (const double**)(mj + n_jobs);
        long long** np = (long long**)(cp + n_jobs);
        for (int j = 0; j < n_jobs; ++j) {
            const ot_mesh_sample_job& m = jobs[j];
            mj[j] = MinZJob{m.vertices, m.out_colors ? m.vertex_colors : nullptr, m.triangles, ncum[j],
                            m.n_triangles, m.out_xyz, m.out_colors};
            cp[j] = cdf[j];
            np[j] = ncum[j];
        }
    };
    // the kept counts land in pinned host memory, written by each job's last tile (no read-back copy)
    long long* kept = (long long*)pinned_scratch(sizeof(long long) * (size_t)n_jobs, 1, true);
    if (!kept) return fail(OT_ERR_HIP, "pinned allocation failed");
    for (int j = 0; j < n_jobs; ++j)
        if (jobs[j].n_triangles > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] too many triangles");
    ot_status st = sample_cdfs(jobs, n_jobs, total, up_bytes, fill, zero_off, zero_end - zero_off, stream, cdf, ncum,
                               &extra, mark, mark_at);
    if (st != OT_OK) return st;
    const MinZJob* djobs = (const MinZJob*)extra;
    const double* const* dcdf = (const double* const*)(djobs + n_jobs);
    long long* const* dncum = (long long* const*)(dcdf + n_jobs);
    int* ticket = (int*)(extra + zero_off + 8 * (size_t)n_jobs);
    unsigned long long* status = (unsigned long long*)(extra + status_off);
    int* tstart = (int*)(extra + tstart_off);
    int64_t max_nt = 0;
    for (int j = 0; j < n_jobs; ++j) max_nt = jobs[j].n_triangles > max_nt ? jobs[j].n_triangles : max_nt;
    hipLaunchKernelGGL(k_round_counts_jobs, dim3((unsigned)((max_nt + 255) / 256), n_jobs), dim3(256), 0, stream, djobs,
                       dcdf, n_points, dncum, tiles, tstart);
    hipLaunchKernelGGL(k_sample_min_z, dim3(tiles, n_jobs), dim3(256), 0, stream, djobs, n_points,
                       (unsigned long long)seed, z_min, tiles, status, ticket, kept, (const int*)tstart);
    OT_LAUNCH_CHECK();
    *hs = stream;
    return OT_OK;
}
static ot_status min_z_wait(hipStream_t hs, int32_t n_jobs, int64_t* n_kept_host) {
    OT_HIP_TRY(hipStreamSynchronize(hs));  // the kept counts (written by each job's last tile)
    const long long* kept = (const long long*)pinned_scratch(sizeof(long long) * (size_t)n_jobs, 1, true);
    for (int j = 0; j < n_jobs; ++j) n_kept_host[j] = kept[j];
    return OT_OK;
}
// the fused extraction + sampling of one volume (mc.hip ot_tsdf_extract_sample_min_z) drives the same two phases
ot_status sample_min_z_enqueue(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points, uint64_t seed,
                               double z_min, hipStream_t stream, hipStream_t* hs, hipEvent_t mark, int mark_at) {
    if (g_minz.active) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] an async sampling is pending");
    return min_z_enqueue(jobs, n_jobs, n_points, seed, z_min, (void*)stream, hs, mark, mark_at);
}
ot_status sample_min_z_wait(hipStream_t hs, int32_t n_jobs, int64_t* n_kept_host) {
    return min_z_wait(hs, n_jobs, n_kept_host);
}
}  // namespace ot

extern "C" {

static ot_status min_z_args(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points) {
    if (n_points <= 0) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] number_of_points <= 0");
    if (n_jobs < 0 || (n_jobs > 0 && !jobs)) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] invalid jobs");
    return OT_OK;
}

ot_status ot_mesh_sample_points_min_z(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points, uint64_t seed,
                                      double z_min, int64_t* n_kept_host, void* stream) {
    ot_status st = min_z_args(jobs, n_jobs, n_points);
    if (st != OT_OK) return st;
    if (n_jobs > 0 && !n_kept_host) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] invalid jobs");
    if (n_jobs == 0) return OT_OK;
    if (g_minz.active) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] an async sampling is pending");
    hipStream_t hs = nullptr;
    st = min_z_enqueue(jobs, n_jobs, n_points, seed, z_min, stream, &hs);
    if (st != OT_OK) return st;
    return min_z_wait(hs, n_jobs, n_kept_host);
}

ot_status ot_mesh_sample_points_min_z_async(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points,
                                            uint64_t seed, double z_min, void* stream) {
    ot_status st = min_z_args(jobs, n_jobs, n_points);
    if (st != OT_OK) return st;
    if (g_minz.active) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] an async sampling is pending");
    if (n_jobs == 0) return OT_OK;
    hipStream_t hs = nullptr;
    st = min_z_enqueue(jobs, n_jobs, n_points, seed, z_min, stream, &hs);
    if (st != OT_OK) return st;
    g_minz.active = true;
    g_minz.s = hs;
    g_minz.n_jobs = n_jobs;
    return OT_OK;
}

// test hook (not part of the drop-in boundary): 1 = the fused sampler on a greatest-priority stream (A/B timing)
ot_status otx_sampler_hi_stream(int32_t on) {
    g_sampler_hi = on != 0;
    return OT_OK;
}

ot_status ot_mesh_sample_points_min_z_wait(int32_t n_jobs, int64_t* n_kept_host) {
    if (n_jobs == 0 && !g_minz.active) return OT_OK;
    if (!g_minz.active || n_jobs != g_minz.n_jobs || !n_kept_host)
        return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] no pending async sampling of n_jobs jobs");
    const hipStream_t hs = g_minz.s;
    g_minz = MinZPending{};
    return min_z_wait(hs, n_jobs, n_kept_host);
}

ot_status ot_mesh_get_surface_area(const double* V, int64_t nv, const int32_t* T, int64_t nt, double* area_host,
                                   void* stream_) {
    hipStream_t stream = S(stream_);
    if (nv < 0 || nt < 0 || !area_host || (nt > 0 && (!V || !T || nv == 0)))
        return fail(OT_ERR_INVALID_ARGUMENT, "[GetSurfaceArea] invalid arguments");
    if (nt == 0) {
        *area_host = 0.0;
        return OT_OK;
    }
    const int64_t nt2 = (nt + 1) & ~(int64_t)1;
    char* ws = (char*)scratch((size_t)nt2 * 8 + chain_aux_bytes(nt) + sizeof(ChainJob) + 512, 17);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    ChainJob jb{};
    double* sum = (double*)ws;
    double* area = sum + 8;
    jb.x = area, jb.n = nt, jb.out = sum;
    char* cur = chain_aux((char*)(area + nt2), nt, jb);
    ChainJob* djob = (ChainJob*)cur;
    hipLaunchKernelGGL(k_tri_areas, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, V, T, nt, area,
                       (double*)nullptr);
    OT_HIP_TRY(hipMemcpyAsync(djob, &jb, sizeof(ChainJob), hipMemcpyHostToDevice, stream));
    launch_chains<false>(djob, 1, nt, stream);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipMemcpyAsync(area_host, sum, sizeof(double), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

// test hook (not part of the drop-in boundary): the chain walk of otx_serial_chain_f64 with its events traced into
// trace (device, 2 * cap u64: {clock64, kind | chunk << 8}; kind 0 step start, 1 run accepted, 2 accepted after the
// 64-way search, 3 serial chunk done, 4 end); *events_host: events recorded (may exceed cap)
ot_status otx_chain_walk_trace(const double* x, int64_t n, int32_t cdf, double* out, unsigned long long* trace,
                               int32_t cap, void* stream_) {
    hipStream_t stream = S(stream_);
    if (n <= 0 || !x || !out || !trace || cap <= 0 || ((uintptr_t)x & 15))
        return fail(OT_ERR_INVALID_ARGUMENT, "[chain] invalid arguments");
    char* ws = (char*)scratch(chain_aux_bytes(n) + sizeof(ChainJob) + 256, 17);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    ChainJob jb{};
    jb.x = x, jb.n = n, jb.out = out;
    ChainJob* djob = (ChainJob*)chain_aux(ws, n, jb);
    jb.trace = trace;
    jb.trace_cap = cap;
    OT_HIP_TRY(hipMemcpyAsync(djob, &jb, sizeof(ChainJob), hipMemcpyHostToDevice, stream));
    if (cdf) launch_chains<true>(djob, 1, n, stream);
    else launch_chains<false>(djob, 1, n, stream);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

// test hook (not part of the drop-in boundary): the bare chains on a device array x (16-B aligned) -- cdf != 0:
// out[t] = x_t + out[t-1] for all t (numpy.cumsum's order); cdf == 0: out[0] = ((0 + x_0) + x_1) + ...;
// serial_chunks_host (nullable): how many 256-value chunks the walk could not prove and ran serially
ot_status otx_serial_chain_f64(const double* x, int64_t n, int32_t cdf, double* out, int64_t* serial_chunks_host,
                               void* stream_) {
    hipStream_t stream = S(stream_);
    if (n <= 0 || !x || !out || ((uintptr_t)x & 15)) return fail(OT_ERR_INVALID_ARGUMENT, "[chain] invalid arguments");
    char* ws = (char*)scratch(chain_aux_bytes(n) + sizeof(ChainJob) + 256, 17);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    ChainJob jb{};
    jb.x = x, jb.n = n, jb.out = out;
    ChainJob* djob = (ChainJob*)chain_aux(ws, n, jb);
    OT_HIP_TRY(hipMemcpyAsync(djob, &jb, sizeof(ChainJob), hipMemcpyHostToDevice, stream));
    if (cdf) launch_chains<true>(djob, 1, n, stream);
    else launch_chains<false>(djob, 1, n, stream);
    OT_LAUNCH_CHECK();
    if (serial_chunks_host) {  // diagnostic: chunks the walk had to run serially (kind == 2)
        const int64_t nb = (n + CH - 1) / CH;
        std::vector<int32_t> kind((size_t)nb);
        OT_HIP_TRY(hipMemcpyAsync(kind.data(), jb.kind, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, stream));
        OT_HIP_TRY(hipStreamSynchronize(stream));
        int64_t c = 0;
        for (int32_t k : kind) c += k == 2;
        *serial_chunks_host = c;
    }
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

}  // extern "C"
