// outlier.hip — PointCloud::RemoveStatisticalOutliers / RemoveRadiusOutliers on MI355X.
//
// Neighbour search uses a uniform cell grid instead of Open3D's KD-tree (the results are defined by the
// distances, not by the search structure):
//   grid build : cell key per point -> stable radix sort (cell, index) -> cell heads -> open-addressing hash
//                (cell key -> [start, end) in the sorted order); points are re-laid out in sorted order so a
//                cell's points are contiguous in HBM.
//   ROR        : cell = radius; count |{j : d2(i, j) < r^2}| over the 27 neighbour cells (exact integers).
//   SOR        : exact k nearest neighbours by shell expansion: cells at Chebyshev ring 0, 1, 2, ... are
//                scanned into a register-resident sorted top-k list until the k-th distance is provably
//                inside the scanned cube.  Distances d2 = ((dx*dx + dy*dy) + dz*dz) (nanoflann L2 order),
//                sqrt'ed and summed in ascending order, divided by the count (std::accumulate in Open3D).
//                Cloud mean / std use a fixed-order two-level reduction in float64.
// Queries run in sorted (cell) order, so a wave's neighbourhoods overlap and stay in L2.
#include <cmath>

#include "compact.h"
#include "sort.h"

namespace ot {

struct GridDev {
    const double* sxyz;           // points in sorted order [n][3]
    const unsigned* sidx;         // sorted position -> original index
    unsigned long long* hkeys;    // cell hash keys
    int2* hval;                   // cell hash values: [start, end)
    int hash_mask;
    double origin[3];
    double h, inv_h;
};

__device__ inline int cell_coord(double v, double origin, double h) { return (int)floor((v - origin) / h); }

__device__ inline int2 grid_find(const GridDev& g, int x, int y, int z) {
    if (!key_in_range(x, y, z)) return make_int2(0, 0);
    const unsigned long long key = pack_key(x, y, z);
    unsigned slot = (unsigned)mix64(key) & (unsigned)g.hash_mask;
    for (int probe = 0; probe <= g.hash_mask; ++probe) {
        const unsigned long long k = g.hkeys[slot];
        if (k == key) return g.hval[slot];
        if (k == KEY_EMPTY) return make_int2(0, 0);
        slot = (slot + 1) & (unsigned)g.hash_mask;
    }
    return make_int2(0, 0);
}

__global__ __launch_bounds__(256) void k_cell_keys(const double* __restrict__ xyz, int64_t n, GridDev g,
                                                   unsigned long long* keys, unsigned* idx, int* err) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int x = cell_coord(xyz[i * 3 + 0], g.origin[0], g.h);
    const int y = cell_coord(xyz[i * 3 + 1], g.origin[1], g.h);
    const int z = cell_coord(xyz[i * 3 + 2], g.origin[2], g.h);
    if (!key_in_range(x, y, z)) *err = 1;
    keys[i] = pack_key(x, y, z);
    idx[i] = (unsigned)i;
}

__global__ __launch_bounds__(256) void k_grid_insert(const unsigned long long* __restrict__ skeys,
                                                     const int* __restrict__ heads, int64_t ncells, int64_t n,
                                                     GridDev g) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= ncells) return;
    const int beg = heads[c];
    const int end = (c + 1 < ncells) ? heads[c + 1] : (int)n;
    const unsigned long long key = skeys[beg];
    unsigned slot = (unsigned)mix64(key) & (unsigned)g.hash_mask;
    while (true) {  // capacity >= 2 * ncells: always terminates
        const unsigned long long old = atomicCAS(&g.hkeys[slot], KEY_EMPTY, key);
        if (old == KEY_EMPTY) {
            g.hval[slot] = make_int2(beg, end);
            return;
        }
        slot = (slot + 1) & (unsigned)g.hash_mask;
    }
}

__global__ __launch_bounds__(256) void k_gather_sorted(const double* __restrict__ xyz, const unsigned* __restrict__ sidx,
                                                       int64_t n, double* __restrict__ sxyz) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n * 3) return;
    const int64_t j = t / 3, a = t % 3;
    sxyz[t] = xyz[(int64_t)sidx[j] * 3 + a];
}

__device__ inline double d2_l2(const double* q, const double* p) {
    const double d0 = q[0] - p[0], d1 = q[1] - p[1], d2 = q[2] - p[2];
    return ((d0 * d0) + d1 * d1) + d2 * d2;
}

// ------------------------------------------------------------------------------------------------ ROR
__global__ __launch_bounds__(256) void k_ror(GridDev g, int64_t n, double r2, int nb, unsigned char* keep) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const double q[3] = {g.sxyz[j * 3], g.sxyz[j * 3 + 1], g.sxyz[j * 3 + 2]};
    const int cx = cell_coord(q[0], g.origin[0], g.h), cy = cell_coord(q[1], g.origin[1], g.h),
              cz = cell_coord(q[2], g.origin[2], g.h);
    long long cnt = 0;
    for (int dx = -1; dx <= 1; ++dx)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dz = -1; dz <= 1; ++dz) {
                const int2 se = grid_find(g, cx + dx, cy + dy, cz + dz);
                for (int k = se.x; k < se.y; ++k) cnt += d2_l2(q, g.sxyz + (int64_t)k * 3) < r2 ? 1 : 0;
            }
    keep[g.sidx[j]] = cnt > nb ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------ SOR
// Register top-k list, RIGHT-aligned: best[KMAX-kk .. KMAX-1] hold the kk smallest squared distances in
// ascending order and best[0 .. KMAX-kk-1] = -inf (never displaced).  best[KMAX-1] is therefore always the
// current k-th distance at a compile-time index, so a candidate that cannot enter costs one compare.
template <int KMAX>
__device__ inline void topk_insert(double (&best)[KMAX], double d) {
    if (!(d < best[KMAX - 1])) return;
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        if (d < best[i]) {
            const double t = best[i];
            best[i] = d;
            d = t;
        }
    }
}

template <int KMAX>
__device__ inline void scan_cell(const GridDev& g, const double q[3], int x, int y, int z, double (&best)[KMAX],
                                 int kk, long long& have) {
    const int2 se = grid_find(g, x, y, z);
    for (int m = se.x; m < se.y; ++m) {
        topk_insert<KMAX>(best, d2_l2(q, g.sxyz + (int64_t)m * 3));
        ++have;
    }
}

constexpr int SOR_RMAX = 6;  // beyond this ring a query falls back to an exact scan of every point

template <int KMAX>
__global__ __launch_bounds__(256) void k_sor_knn(GridDev g, int64_t n, int k, double* avg) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const double q[3] = {g.sxyz[j * 3], g.sxyz[j * 3 + 1], g.sxyz[j * 3 + 2]};
    const int cx = cell_coord(q[0], g.origin[0], g.h), cy = cell_coord(q[1], g.origin[1], g.h),
              cz = cell_coord(q[2], g.origin[2], g.h);
    const int kk = (int)((int64_t)k < n ? k : n);
    double best[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) best[i] = (i < KMAX - kk) ? -INFINITY : INFINITY;
    long long have = 0;
    bool done = false;
    for (int r = 0; r <= SOR_RMAX && !done; ++r) {
        // cells at Chebyshev distance exactly r
        for (int dx = -r; dx <= r; ++dx)
            for (int dy = -r; dy <= r; ++dy) {
                const bool face = (dx == -r || dx == r || dy == -r || dy == r);
                if (face) {
                    for (int dz = -r; dz <= r; ++dz) scan_cell<KMAX>(g, q, cx + dx, cy + dy, cz + dz, best, kk, have);
                } else {
                    scan_cell<KMAX>(g, q, cx + dx, cy + dy, cz - r, best, kk, have);
                    if (r > 0) scan_cell<KMAX>(g, q, cx + dx, cy + dy, cz + r, best, kk, have);
                }
            }
        if (have >= kk) {
            const double kth = best[KMAX - 1];
            // every point within distance (r - margin) * h of q lies in rings 0..r
            const double guard = (r > 0 ? (double)r - 0.01 : 0.0) * g.h;
            if (kth <= guard * guard || have >= n) done = true;
        }
    }
    if (!done) {  // isolated point: exact scan of the whole cloud
#pragma unroll
        for (int i = 0; i < KMAX; ++i) best[i] = (i < KMAX - kk) ? -INFINITY : INFINITY;
        for (int64_t m = 0; m < n; ++m) topk_insert<KMAX>(best, d2_l2(q, g.sxyz + m * 3));
    }
    double s = 0.0;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < KMAX; ++i)
        if (i >= KMAX - kk && best[i] < INFINITY) {
            s += sqrt(best[i]);
            ++cnt;
        }
    avg[g.sidx[j]] = cnt > 0 ? s / (double)cnt : -1.0;
}

// fixed-order two-level reduction: blocks reduce contiguous chunks in a fixed tree, then one block reduces
// the block partials in the same fixed order.  mode 0: sum of avg > 0 and count; mode 1: sum of (avg-mean)^2
__global__ __launch_bounds__(256) void k_sor_partial(const double* __restrict__ avg, int64_t n, int mode,
                                                     const double* __restrict__ stats, double* partial,
                                                     long long* pcount) {
    __shared__ double sd[256];
    __shared__ long long sc[256];
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t beg = (int64_t)blockIdx.x * chunk, end = beg + chunk < n ? beg + chunk : n;
    double acc = 0.0;
    long long c = 0;
    const double mean = mode == 1 ? stats[0] : 0.0;
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
        const double a = avg[i];
        if (a > 0) {
            acc += mode == 0 ? a : (a - mean) * (a - mean);
            ++c;
        }
    }
    sd[threadIdx.x] = acc;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sd[threadIdx.x] += sd[threadIdx.x + s];
            sc[threadIdx.x] += sc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = sd[0];
        pcount[blockIdx.x] = sc[0];
    }
}

__global__ __launch_bounds__(256) void k_sor_final(const double* partial, const long long* pcount, int nb, int mode,
                                                   double std_ratio, double* stats) {
    __shared__ double sd[256];
    __shared__ long long sc[256];
    double acc = 0.0;
    long long c = 0;
    for (int i = threadIdx.x; i < nb; i += 256) {
        acc += partial[i];
        c += pcount[i];
    }
    sd[threadIdx.x] = acc;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sd[threadIdx.x] += sd[threadIdx.x + s];
            sc[threadIdx.x] += sc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (mode == 0) {
            stats[2] = (double)sc[0];                  // valid
            stats[0] = sc[0] > 0 ? sd[0] / (double)sc[0] : 0.0;  // cloud mean
        } else {
            const double valid = stats[2];
            const double sdv = sqrt(sd[0] / (valid - 1.0));
            stats[1] = sdv;
            stats[3] = stats[0] + std_ratio * sdv;  // threshold
        }
    }
}

struct SorPred {
    const double* avg;
    const double* stats;
    __device__ bool operator()(int64_t i) const {
        const double a = avg[i];
        return a > 0 && a < stats[3];
    }
};
struct RorPred {
    const unsigned char* keep;
    __device__ bool operator()(int64_t i) const { return keep[i] != 0; }
};
struct IndexEmit {
    int64_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = i; }
};

// ------------------------------------------------------------------------------------ grid builder (host)
struct GridBuild {
    GridDev g;
    int64_t ncells = 0;
};

static ot_status build_grid(const double* xyz, int64_t n, double h, const double origin[3], hipStream_t stream,
                            GridBuild& out) {
    char* ws = (char*)scratch(256 + (size_t)n * (8 + 8 + 4 + 4 + 4 + 24), 8);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    int* err = (int*)ws;
    unsigned long long* kin = (unsigned long long*)(ws + 256);
    unsigned long long* kout = kin + n;
    unsigned* vin = (unsigned*)(kout + n);
    unsigned* vout = vin + n;
    int* heads = (int*)(vout + n);
    double* sxyz = (double*)(((uintptr_t)(heads + n) + 15) & ~(uintptr_t)15);
    GridDev& g = out.g;
    g.h = h;
    g.inv_h = 1.0 / h;
    for (int a = 0; a < 3; ++a) g.origin[a] = origin[a];
    OT_HIP_TRY(hipMemsetAsync(err, 0, sizeof(int), stream));
    hipLaunchKernelGGL(k_cell_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, xyz, n, g, kin, vin, err);
    OT_LAUNCH_CHECK();
    ot_status st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)n, 63, stream, 3);
    if (st != OT_OK) return st;
    int64_t ncells = 0;
    st = compact(n, SegHeadPred{kout}, SegHeadEmit{heads}, stream, &ncells, 9);
    if (st != OT_OK) return st;
    int e = 0;
    OT_HIP_TRY(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
    if (e) return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid out of range (radius too small for the extent)");
    int64_t cap = 1;
    while (cap < 2 * ncells + 2) cap <<= 1;
    char* hs = (char*)scratch((size_t)cap * (8 + 8) + 64, 10);
    if (!hs) return fail(OT_ERR_HIP, "scratch allocation failed");
    g.hkeys = (unsigned long long*)hs;
    g.hval = (int2*)(g.hkeys + cap);
    g.hash_mask = (int)(cap - 1);
    OT_HIP_TRY(hipMemsetAsync(g.hkeys, 0xFF, sizeof(unsigned long long) * cap, stream));
    hipLaunchKernelGGL(k_grid_insert, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, stream, kout, heads, ncells,
                       n, g);
    hipLaunchKernelGGL(k_gather_sorted, dim3((unsigned)((n * 3 + 255) / 256)), dim3(256), 0, stream, xyz, vout, n, sxyz);
    OT_LAUNCH_CHECK();
    g.sxyz = sxyz;
    g.sidx = vout;
    out.ncells = ncells;
    return OT_OK;
}

}  // namespace ot

using namespace ot;

static ot_status bounds_host(const double* xyz, int64_t n, hipStream_t stream, double mn[3], double mx[3]) {
    Bounds* b = (Bounds*)scratch(sizeof(Bounds) + 64, 11);
    if (!b) return fail(OT_ERR_HIP, "scratch allocation failed");
    unsigned long long* part = (unsigned long long*)scratch(sizeof(unsigned long long) * BOUNDS_BLOCKS * 6, 19);
    if (!part) return fail(OT_ERR_HIP, "scratch allocation failed");
    launch_bounds(xyz, n, b, part, stream);
    OT_LAUNCH_CHECK();
    Bounds hb;
    OT_HIP_TRY(hipMemcpyAsync(&hb, b, sizeof(Bounds), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    for (int a = 0; a < 3; ++a) {
        mn[a] = ordered_to_dbl(hb.mn[a]);
        mx[a] = ordered_to_dbl(hb.mx[a]);
    }
    return OT_OK;
}

extern "C" {

ot_status ot_remove_radius_outlier(const double* xyz, int64_t n, int32_t nb_points, double radius,
                                   int64_t* out_indices, int64_t* n_kept_host, void* stream_) {
    hipStream_t stream = S(stream_);
    if (nb_points < 1 || !(radius > 0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveRadiusOutliers] Illegal input parameters, number of points "
                                             "and radius must be positive");
    if (!n_kept_host) return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveRadiusOutliers] n_kept is NULL");
    *n_kept_host = 0;
    if (n <= 0) return OT_OK;
    if (!xyz || !out_indices || n > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveRadiusOutliers] invalid buffers");
    double mn[3], mx[3];
    ot_status st = bounds_host(xyz, n, stream, mn, mx);
    if (st != OT_OK) return st;
    GridBuild gb;
    st = build_grid(xyz, n, radius, mn, stream, gb);
    if (st != OT_OK) return st;
    unsigned char* keep = (unsigned char*)scratch((size_t)n + 64, 12);
    if (!keep) return fail(OT_ERR_HIP, "scratch allocation failed");
    hipLaunchKernelGGL(k_ror, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, gb.g, n, radius * radius,
                       (int)nb_points, keep);
    OT_LAUNCH_CHECK();
    return compact(n, RorPred{keep}, IndexEmit{out_indices}, stream, n_kept_host, 13);
}

ot_status ot_remove_statistical_outlier(const double* xyz, int64_t n, int32_t nb_neighbors, double std_ratio,
                                        int64_t* out_indices, double* out_avg_dist, int64_t* n_kept_host,
                                        void* stream_) {
    hipStream_t stream = S(stream_);
    if (nb_neighbors < 1 || !(std_ratio > 0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] Illegal input parameters, the number of "
                                             "neighbors and standard deviation ratio must be positive.");
    if (nb_neighbors > 64)
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] nb_neighbors > 64 is not supported");
    if (!n_kept_host) return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] n_kept is NULL");
    *n_kept_host = 0;
    if (n <= 0) return OT_OK;
    if (!xyz || !out_indices || n > 0x7FFFFFFF)
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] invalid buffers");
    double mn[3], mx[3];
    ot_status st = bounds_host(xyz, n, stream, mn, mx);
    if (st != OT_OK) return st;
    // cell size: volumetric first guess, then one refinement assuming surface-like (2-D) occupancy so that
    // an occupied cell holds ~k/3 points (the grid only changes speed, never the result)
    const double k = (double)nb_neighbors;
    double ext[3], vol = 1.0;
    for (int a = 0; a < 3; ++a) {
        ext[a] = std::max(mx[a] - mn[a], 1e-9);
        vol *= ext[a];
    }
    double h = std::cbrt(vol * k / (double)n);
    const double hmin = std::max(std::max(ext[0], ext[1]), ext[2]) / 1.0e6;
    h = std::max(h, hmin);
    GridBuild gb;
    st = build_grid(xyz, n, h, mn, stream, gb);
    if (st != OT_OK) return st;
    const double occ = (double)n / (double)std::max<int64_t>(gb.ncells, 1);
    const double target = std::max(k / 3.0, 2.0);
    if (occ > 2.0 * target || occ < 0.5 * target) {
        h = std::max(h * std::sqrt(target / occ), hmin);
        st = build_grid(xyz, n, h, mn, stream, gb);
        if (st != OT_OK) return st;
    }
    char* ws = (char*)scratch((size_t)n * 8 + 1024 * 16 + 256, 12);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    double* stats = (double*)ws;                  // [0] mean [1] std [2] valid [3] threshold
    double* partial = (double*)(ws + 64);         // 1024
    long long* pcount = (long long*)(ws + 64 + 1024 * 8);
    double* avg = out_avg_dist ? out_avg_dist : (double*)(ws + 256 + 1024 * 16);
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (nb_neighbors <= 32)
        hipLaunchKernelGGL(k_sor_knn<32>, dim3(grid), dim3(256), 0, stream, gb.g, n, (int)nb_neighbors, avg);
    else
        hipLaunchKernelGGL(k_sor_knn<64>, dim3(grid), dim3(256), 0, stream, gb.g, n, (int)nb_neighbors, avg);
    const int nb = (int)std::min<int64_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_sor_partial, dim3(nb), dim3(256), 0, stream, avg, n, 0, stats, partial, pcount);
    hipLaunchKernelGGL(k_sor_final, dim3(1), dim3(256), 0, stream, partial, pcount, nb, 0, std_ratio, stats);
    hipLaunchKernelGGL(k_sor_partial, dim3(nb), dim3(256), 0, stream, avg, n, 1, stats, partial, pcount);
    hipLaunchKernelGGL(k_sor_final, dim3(1), dim3(256), 0, stream, partial, pcount, nb, 1, std_ratio, stats);
    OT_LAUNCH_CHECK();
    return compact(n, SorPred{avg, stats}, IndexEmit{out_indices}, stream, n_kept_host, 13);
}

}  // extern "C"
