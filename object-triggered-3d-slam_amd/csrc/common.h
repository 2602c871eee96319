// common.h — shared helpers of the MI355X-native hot path (HIP, gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/otslam.h"

namespace ot {

// ------------------------------------------------------------------------------------------ errors
void set_error(const std::string& msg);
ot_status fail(ot_status code, const std::string& msg);

#define OT_HIP_TRY(expr)                                                                                   \
    do {                                                                                                   \
        hipError_t e__ = (expr);                                                                           \
        if (e__ != hipSuccess)                                                                             \
            return ::ot::fail(OT_ERR_HIP, std::string("HIP error ") + hipGetErrorString(e__) + " at " +     \
                                              __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")"); \
    } while (0)

#define OT_LAUNCH_CHECK() OT_HIP_TRY(hipGetLastError())

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ----------------------------------------------------------------------------- per-device scratch
// Grow-only scratch arena per host thread and device (capi.hip): threads driving their own streams never share a
// buffer.
void* scratch(size_t bytes, int slot);
// pinned host counterpart (per thread and device, grow-only): small tables uploaded with hipMemcpyAsync without the
// pageable staging copy; the caller must have synchronised on its previous upload from the slot before rewriting it
// coherent: fine-grained memory a kernel writes results into directly (a slot keeps the kind it was first made with)
void* pinned_scratch(size_t bytes, int slot, bool coherent = false);
// a small host table (<= UPLOAD_ARG_BYTES) to device memory in stream order, carried by the kernel arguments of one
// tiny launch instead of a copy command (measured: a ~1 KB hipMemcpyAsync from pinned memory took ~35 us on one
// object's critical path beside a running kernel); larger tables take hipMemcpyAsync.  src is consumed on return.
constexpr size_t UPLOAD_ARG_BYTES = 3072;
ot_status upload_small(void* dst, const void* src, size_t bytes, hipStream_t stream);
// the kernel-argument carrier of upload_small (also passed to a caller's own first kernel, which then stores it: one
// launch fewer on a latency chain)
struct ArgBlob {
    unsigned long long w[UPLOAD_ARG_BYTES / 8];
};
// device allocations made by the library's grow-only buffers so far (scratch arenas, filter handles): a timed
// region that allocates shows up as a change (bench.py reports it; test hook otx_alloc_count)
void note_alloc();
long long g_allocs_count();

// --------------------------------------------------------------------------------- math helpers
struct Mat4d {
    double m[16];
};
struct Mat4f {
    float m[16];
};

// Eigen generic 4x4 inverse (compute_inverse_size4 + cofactor_4x4), host side.
void inverse4(const double* m, double* r);

// ordered encoding of doubles so that unsigned integer order == numeric order (for atomicMin/Max)
__host__ __device__ inline unsigned long long dbl_to_ordered(double d) {
    unsigned long long u = __builtin_bit_cast(unsigned long long, d);
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__host__ __device__ inline double ordered_to_dbl(unsigned long long u) {
    u = (u & 0x8000000000000000ull) ? (u & 0x7FFFFFFFFFFFFFFFull) : ~u;
    return __builtin_bit_cast(double, u);
}

// packed int3 key: 21 bits per axis, biased by 2^20, x-major => numeric order == (x, y, z) lexicographic
constexpr int KEY_BITS = 21;
constexpr int KEY_BIAS = 1 << 20;
constexpr unsigned long long KEY_EMPTY = ~0ull;
__host__ __device__ inline bool key_in_range(int x, int y, int z) {
    return x >= -KEY_BIAS && x < KEY_BIAS && y >= -KEY_BIAS && y < KEY_BIAS && z >= -KEY_BIAS && z < KEY_BIAS;
}
__host__ __device__ inline unsigned long long pack_key(int x, int y, int z) {
    return ((unsigned long long)(x + KEY_BIAS) << 42) | ((unsigned long long)(y + KEY_BIAS) << 21) |
           (unsigned long long)(z + KEY_BIAS);
}
__host__ __device__ inline void unpack_key(unsigned long long k, int& x, int& y, int& z) {
    x = (int)((k >> 42) & 0x1FFFFF) - KEY_BIAS;
    y = (int)((k >> 21) & 0x1FFFFF) - KEY_BIAS;
    z = (int)(k & 0x1FFFFF) - KEY_BIAS;
}
__host__ __device__ inline unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// the frame holding element i of frame-major data with segment starts foff[0 .. nframes): the last f with
// foff[f] <= i (empty frames are skipped over)
__device__ inline int frame_of(const int* __restrict__ foff, int nframes, int64_t i) {
    int lo = 0, hi = nframes;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (foff[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

// fl(x / y) without a division, from r = fl(1 / y): q0 = fl(x r) lies within an ulp of x / y and r within half an
// ulp of 1 / y, so fl(q0 + fl(x - q0 y) r) is the correctly rounded quotient (Markstein; both fma's exact in the
// remainder) barring over/underflow, which the callers' ranges (pixel coordinates, depths, colours, counts) exclude.
// A zero x keeps its sign through q0.  Checked on the host against IEEE division over every u16 depth for 3000+
// scales (float) and 5e8 unprojection / colour / average quotients (double).
__device__ inline double div_rn(double x, double y, double r) {
    const double q0 = x * r;
    const double q = __builtin_fma(__builtin_fma(-q0, y, x), r, q0);
    return q != 0.0 ? q : q0;
}
__device__ inline float div_rn(float x, float y, float r) {
    const float q0 = x * r;
    const float q = __builtin_fmaf(__builtin_fmaf(-q0, y, x), r, q0);
    return q != 0.0f ? q : q0;
}

// ------------------------------------------------------------------------ wave / block primitives
__device__ inline unsigned lane_id() { return __lane_id(); }

// exclusive prefix of a predicate within the wave (64 lanes) and the wave total
__device__ inline int wave_excl_count(bool pred, int& total) {
    unsigned long long m = __ballot(pred);
    total = __popcll(m);
    unsigned long long lt = (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
    return __popcll(m & lt);
}

// TriangleMesh::ComputeVertexNormals' last step on the accumulated (unnormalised) sum: normalise, NaN -> (0, 0, 1)
__device__ inline void finish_vertex_normal(double n[3]) {
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
}

// triangle normal (v1 - v0) x (v2 - v0), unnormalised (Open3D ComputeTriangleNormals(false))
__device__ inline void triangle_normal(const double* __restrict__ V, int32_t a, int32_t b, int32_t c, double out[3]) {
    double e1[3], e2[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        e1[d] = V[(int64_t)b * 3 + d] - V[(int64_t)a * 3 + d];
        e2[d] = V[(int64_t)c * 3 + d] - V[(int64_t)a * 3 + d];
    }
    out[0] = e1[1] * e2[2] - e1[2] * e2[1];
    out[1] = e1[2] * e2[0] - e1[0] * e2[2];
    out[2] = e1[0] * e2[1] - e1[1] * e2[0];
}

template <typename T>
__device__ inline T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ inline int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}

// Decoupled look-back (single-pass prefix over the tiles of one chain), run by ONE whole wave of the tile's
// workgroup: publishes the tile's aggregate, reads its predecessors' status words 64 at a time (lane i: tile - 1 - i),
// folds every aggregate up to the nearest inclusive prefix, publishes its own inclusive prefix and returns the
// exclusive one (all lanes).  Status word: 0 = not yet published, LB_AGG | count, LB_PRE | inclusive prefix; the
// caller zeroes the words and starts tiles in order (tickets), so every predecessor is running or done.  A window is
// folded up to its first unpublished word and re-read from there, so a tile waits only on running predecessors.
constexpr unsigned long long LB_AGG = 1ull << 62, LB_PRE = 2ull << 62, LB_VAL = (1ull << 62) - 1;
__device__ inline long long lookback_wave(unsigned long long* st, int tile, unsigned long long agg) {
    const int lane = (int)lane_id();
    if (tile == 0) {
        if (lane == 0) __hip_atomic_store(&st[0], LB_PRE | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&st[tile], LB_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long excl = 0;
    int top = tile - 1;  // the highest predecessor not folded in yet
    while (true) {
        const int t = top - lane;
        const unsigned long long v =
            t >= 0 ? __hip_atomic_load(&st[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : LB_PRE;  // below 0: stop
        const unsigned long long pre = __ballot((v & ~LB_VAL) == LB_PRE), zero = __ballot(v == 0ull);
        const int first_pre = pre ? __ffsll((long long)pre) - 1 : 64;
        const int first_zero = zero ? __ffsll((long long)zero) - 1 : 64;
        if (first_zero < first_pre) {  // fold the published aggregates above the first gap, then wait on it
            excl += wave_sum(lane < first_zero ? (v & LB_VAL) : 0ull);
            top -= first_zero;
            continue;
        }
        excl += wave_sum(lane <= first_pre ? (v & LB_VAL) : 0ull);  // up to and including the inclusive prefix
        if (first_pre < 64) break;
        top -= 64;
    }
    if (lane == 0) __hip_atomic_store(&st[tile], LB_PRE | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (long long)excl;
}

}  // namespace ot
