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
#include <vector>

#include "compact.h"
#include "sort.h"

namespace ot {

__global__ __launch_bounds__(256) void k_tri_normals(const double* __restrict__ V, const int32_t* __restrict__ T,
                                                     int64_t nt, double* __restrict__ TN,
                                                     unsigned long long* keys, unsigned* vals) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nt) return;
    const int32_t a = T[t * 3], b = T[t * 3 + 1], c = T[t * 3 + 2];
    double e1[3], e2[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        e1[d] = V[(int64_t)b * 3 + d] - V[(int64_t)a * 3 + d];
        e2[d] = V[(int64_t)c * 3 + d] - V[(int64_t)a * 3 + d];
    }
    TN[t * 3 + 0] = e1[1] * e2[2] - e1[2] * e2[1];
    TN[t * 3 + 1] = e1[2] * e2[0] - e1[0] * e2[2];
    TN[t * 3 + 2] = e1[0] * e2[1] - e1[1] * e2[0];
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
    const double sq = (n[0] * n[0] + n[1] * n[1]) + n[2] * n[2];
    if (sq > 0.0) {
        const double s = sqrt(sq);
        n[0] /= s;
        n[1] /= s;
        n[2] /= s;
    }
    if (isnan(n[0])) {
        n[0] = 0.0;
        n[1] = 0.0;
        n[2] = 1.0;
    }
    N[v * 3 + 0] = n[0];
    N[v * 3 + 1] = n[1];
    N[v * 3 + 2] = n[2];
}

// ------------------------------------------------------------------------------------------- sampling
__global__ __launch_bounds__(256) void k_tri_areas(const double* __restrict__ V, const int32_t* __restrict__ T,
                                                   int64_t nt, double* __restrict__ area) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nt) return;
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
    area[t] = 0.5 * sqrt((c0 * c0 + c1 * c1) + c2 * c2);
}

// Open3D's sequential recurrences (GetSurfaceArea: s = (((a0 + a1) + a2) + ...), then the CDF loop
// cdf_t = a_t / s + cdf_{t-1}) are serial float64 chains, kept in their exact order by ONE wave: the wave streams
// the input with coalesced 16-B-per-lane loads kept CDF_DEPTH chunks ahead, parks each 128-value chunk in LDS,
// and lane 0 runs the dependent v_add_f64 chain over it (ds_read_b128 operands).  The divisions a_t / s are a
// separate lane-parallel pass; the CDF chunk goes back through LDS to one coalesced store.  Padding adds +0.0,
// an exact no-op for these non-negative sums.
constexpr int CDF_CHUNK = 128;  // values per chunk (2 per lane)
constexpr int CDF_DEPTH = 8;    // chunks in flight

__device__ inline double2 cdf_load(const double* __restrict__ x, int64_t nt, int64_t base, int lane) {
    const int64_t i = base + 2 * lane;
    if (i + 1 < nt) return *reinterpret_cast<const double2*>(x + i);  // x is 16-B aligned, base even
    return make_double2(i < nt ? x[i] : 0.0, 0.0);
}

template <bool CDF>
__device__ inline void cdf_chunk(double2 v, double* lds, double& acc, int lane, int64_t base, int64_t nt,
                                 double* __restrict__ out) {
    reinterpret_cast<double2*>(lds)[lane] = v;
    __syncthreads();
    if (lane == 0) {
#pragma unroll 8
        for (int k = 0; k < CDF_CHUNK; k += 2) {
            const double2 p = reinterpret_cast<const double2*>(lds)[k >> 1];
            if (CDF) {
                double2 r;
                acc = p.x + acc;
                r.x = acc;
                acc = p.y + acc;
                r.y = acc;
                reinterpret_cast<double2*>(lds)[k >> 1] = r;
            } else {
                acc = acc + p.x;
                acc = acc + p.y;
            }
        }
    }
    __syncthreads();
    if (CDF) {
        const double2 r = reinterpret_cast<const double2*>(lds)[lane];
        const int64_t i = base + 2 * lane;
        if (i + 1 < nt) *reinterpret_cast<double2*>(out + i) = r;
        else if (i < nt) out[i] = r.x;
        __syncthreads();
    }
}

// one serial chain per workgroup (one wave): a single mesh, or one mesh of a batch (independent chains of
// several meshes run side by side on different CUs)
struct ChainJob {
    const double* x;
    int64_t n;
    double* out;
};

template <bool CDF>
__device__ inline void serial_chain(const double* __restrict__ x, int64_t nt, double* __restrict__ out, double* lds) {
    const int lane = threadIdx.x;
    double acc = 0.0;  // sum: s = 0 + a_0 + ...;  cdf: cdf_0 = q_0 + 0.0 = q_0 exactly
    double2 r[CDF_DEPTH];
#pragma unroll
    for (int d = 0; d < CDF_DEPTH; ++d) r[d] = cdf_load(x, nt, (int64_t)d * CDF_CHUNK, lane);
    for (int64_t base = 0; base < nt; base += (int64_t)CDF_CHUNK * CDF_DEPTH) {
#pragma unroll
        for (int d = 0; d < CDF_DEPTH; ++d) {
            const int64_t b = base + (int64_t)d * CDF_CHUNK;
            if (b < nt) cdf_chunk<CDF>(r[d], lds, acc, lane, b, nt, out);
            r[d] = cdf_load(x, nt, b + (int64_t)CDF_CHUNK * CDF_DEPTH, lane);
        }
    }
    if (!CDF && lane == 0) out[0] = acc;
}

template <bool CDF>
__global__ __launch_bounds__(64) void k_serial_chain(const double* __restrict__ x, int64_t nt, double* __restrict__ out) {
    __shared__ double lds[CDF_CHUNK];
    serial_chain<CDF>(x, nt, out, lds);
}

template <bool CDF>
__global__ __launch_bounds__(64) void k_serial_chain_batch(const ChainJob* __restrict__ jobs) {
    __shared__ double lds[CDF_CHUNK];
    const ChainJob j = jobs[blockIdx.x];
    serial_chain<CDF>(j.x, j.n, j.out, lds);
}

__global__ __launch_bounds__(256) void k_area_div(const double* __restrict__ area, int64_t nt,
                                                  const double* __restrict__ sum, double* __restrict__ q) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < nt) q[t] = area[t] / sum[0];
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

__global__ __launch_bounds__(256) void k_sample(const double* __restrict__ V, const double* __restrict__ VN,
                                                const double* __restrict__ VC, const int32_t* __restrict__ T,
                                                const long long* __restrict__ ncum, int64_t nt, int64_t N,
                                                unsigned long long seed, double* P, double* PN, double* PC) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= N) return;
    // triangle t: first index with ncum[t] > k (the CPU loop fills points [ncum[t-1], ncum[t]) from t)
    int64_t lo = 0, hi = nt;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (ncum[mid] > k) hi = mid;
        else lo = mid + 1;
    }
    if (lo >= nt) {  // rounding shortfall: left zero like Open3D's zero-initialised storage
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            P[k * 3 + d] = 0.0;
            if (PN) PN[k * 3 + d] = 0.0;
            if (PC) PC[k * 3 + d] = 0.0;
        }
        return;
    }
    const int64_t t = lo;
    const double r1 = rng_u01(seed, (unsigned long long)(2 * k)), r2 = rng_u01(seed, (unsigned long long)(2 * k + 1));
    const double s1 = sqrt(r1);
    const double a = 1.0 - s1, b = s1 * (1.0 - r2), c = s1 * r2;
    const int64_t i0 = T[t * 3], i1 = T[t * 3 + 1], i2 = T[t * 3 + 2];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        P[k * 3 + d] = (a * V[i0 * 3 + d] + b * V[i1 * 3 + d]) + c * V[i2 * 3 + d];
        if (PN) PN[k * 3 + d] = (a * VN[i0 * 3 + d] + b * VN[i1 * 3 + d]) + c * VN[i2 * 3 + d];
        if (PC) PC[k * 3 + d] = (a * VC[i0 * 3 + d] + b * VC[i1 * 3 + d]) + c * VC[i2 * 3 + d];
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
                                          double* PN, double* PC, void* stream_) {
    hipStream_t stream = S(stream_);
    if (n_points <= 0) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] number_of_points <= 0");
    if (nt <= 0) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] Input mesh has no triangles.");
    if (!V || !T || !P || (PN && !VN) || (PC && !VC) || nv <= 0)
        return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] invalid arguments");
    char* ws = (char*)scratch((size_t)nt * 32 + 256, 17);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    double* sum = (double*)ws;
    double* area = sum + 8;  // 64-B offset: 16-B aligned rows for the chain's double2 loads
    double* q = area + ((nt + 1) & ~(int64_t)1);  // 16-B aligned for the chain's double2 loads
    long long* ncum = (long long*)(q + ((nt + 1) & ~(int64_t)1));
    hipLaunchKernelGGL(k_tri_areas, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, V, T, nt, area);
    hipLaunchKernelGGL(k_serial_chain<false>, dim3(1), dim3(64), 0, stream, (const double*)area, nt, sum);
    hipLaunchKernelGGL(k_area_div, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, (const double*)area, nt,
                       (const double*)sum, q);
    hipLaunchKernelGGL(k_serial_chain<true>, dim3(1), dim3(64), 0, stream, (const double*)q, nt, area);
    hipLaunchKernelGGL(k_round_counts, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, area, nt, n_points,
                       ncum);
    hipLaunchKernelGGL(k_sample, dim3((unsigned)((n_points + 255) / 256)), dim3(256), 0, stream, V, PN ? VN : nullptr,
                       PC ? VC : nullptr, T, ncum, nt, n_points, (unsigned long long)seed, P, PN, PC);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

ot_status ot_mesh_sample_points_uniformly_batch(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points,
                                                uint64_t seed, void* stream_) {
    hipStream_t stream = S(stream_);
    if (n_points <= 0) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] number_of_points <= 0");
    if (n_jobs < 0 || (n_jobs > 0 && !jobs)) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] invalid jobs");
    if (n_jobs == 0) return OT_OK;
    size_t bytes = 256;
    for (int j = 0; j < n_jobs; ++j) {
        const ot_mesh_sample_job& m = jobs[j];
        if (m.n_triangles <= 0) return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] Input mesh has no triangles.");
        if (!m.vertices || !m.triangles || !m.out_xyz || (m.out_normals && !m.vertex_normals) ||
            (m.out_colors && !m.vertex_colors) || m.n_vertices <= 0)
            return fail(OT_ERR_INVALID_ARGUMENT, "[SamplePointsUniformly] invalid arguments");
        bytes += (size_t)m.n_triangles * 32 + 256;
    }
    char* ws = (char*)scratch(bytes + sizeof(ChainJob) * 2 * (size_t)n_jobs + 256, 17);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    std::vector<ChainJob> sum_jobs(n_jobs), cdf_jobs(n_jobs);
    std::vector<double*> areas(n_jobs), qs(n_jobs), sums(n_jobs);
    std::vector<long long*> ncums(n_jobs);
    char* cur = ws;
    for (int j = 0; j < n_jobs; ++j) {
        const int64_t nt = jobs[j].n_triangles, nt2 = (nt + 1) & ~(int64_t)1;
        sums[j] = (double*)cur;
        areas[j] = sums[j] + 8;
        qs[j] = areas[j] + nt2;
        ncums[j] = (long long*)(qs[j] + nt2);
        cur = (char*)(ncums[j] + nt2) + 64;
        cur = (char*)(((uintptr_t)cur + 63) & ~(uintptr_t)63);
        sum_jobs[j] = ChainJob{areas[j], nt, sums[j]};
        cdf_jobs[j] = ChainJob{qs[j], nt, areas[j]};
        hipLaunchKernelGGL(k_tri_areas, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, jobs[j].vertices,
                           jobs[j].triangles, nt, areas[j]);
    }
    ChainJob* djobs = (ChainJob*)(((uintptr_t)cur + 63) & ~(uintptr_t)63);
    OT_HIP_TRY(hipMemcpyAsync(djobs, sum_jobs.data(), sizeof(ChainJob) * n_jobs, hipMemcpyHostToDevice, stream));
    OT_HIP_TRY(hipMemcpyAsync(djobs + n_jobs, cdf_jobs.data(), sizeof(ChainJob) * n_jobs, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_serial_chain_batch<false>, dim3(n_jobs), dim3(64), 0, stream, (const ChainJob*)djobs);
    for (int j = 0; j < n_jobs; ++j) {
        const int64_t nt = jobs[j].n_triangles;
        hipLaunchKernelGGL(k_area_div, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, (const double*)areas[j],
                           nt, (const double*)sums[j], qs[j]);
    }
    hipLaunchKernelGGL(k_serial_chain_batch<true>, dim3(n_jobs), dim3(64), 0, stream, (const ChainJob*)(djobs + n_jobs));
    for (int j = 0; j < n_jobs; ++j) {
        const ot_mesh_sample_job& m = jobs[j];
        const int64_t nt = m.n_triangles;
        hipLaunchKernelGGL(k_round_counts, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, areas[j], nt,
                           n_points, ncums[j]);
        hipLaunchKernelGGL(k_sample, dim3((unsigned)((n_points + 255) / 256)), dim3(256), 0, stream, m.vertices,
                           m.out_normals ? m.vertex_normals : nullptr, m.out_colors ? m.vertex_colors : nullptr,
                           m.triangles, ncums[j], nt, n_points, (unsigned long long)seed, m.out_xyz, m.out_normals,
                           m.out_colors);
    }
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));  // the host job tables are released on return
    return OT_OK;
}

}  // extern "C"
