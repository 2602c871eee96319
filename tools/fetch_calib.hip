// fetch_calib.hip — calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns the roofline
// kernels actually issue.  Every pattern reads (or writes) a 1-GiB buffer exactly once, far past
// the 4-MiB L2s and the 256-MiB Infinity Cache, so the compulsory HBM bytes are known: each launch's factor is
//   known bytes / (FETCH_SIZE KiB * 1024)   (resp. WRITE_SIZE).
// Patterns (one launch each, named so the counter CSV tells them apart):
//   k_cal_stream16  : 16 B per lane, coalesced dwordx4 (the guide's calibrated case: expect x2)
//   k_cal_gather8   : 8 B per lane through a buffer resource (the integrate's staged (depth, multiplier) gathers);
//                     each wave instruction consumes 4 whole 128-B lines with its lanes in a random order, and the
//                     line groups are visited in a random order (no two waves of a pass share a line)
//   k_cal_gather4   : 4 B per lane (the integrate's colour gathers), 2 whole lines per instruction, same shuffling
//   k_cal_half8     : 8 B per lane, but only the first 64 B of every 128-B line is ever read (granularity probe:
//                     known = 64 B per line if the fabric request is 64 B, 128 B if whole lines are fetched)
//   k_cal_store8    : 8 B per lane buffer stores, whole lines per instruction (the integrate's float64 colour and
//                     per-plane f32 write-back are 4-8 B per lane)
// Usage: fetch_calib [MiB]   prints one JSON line with the known byte counts per kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ inline unsigned mix32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// a bijection on [0, n) for n a power of two (odd multiplier + xor-shift on the low bits)
__device__ inline unsigned perm(unsigned i, unsigned mask) {
    i = (i * 0x9E3779B1u) & mask;
    i ^= (i >> 7) & mask;
    i = (i * 0x85EBCA6Bu) & mask;
    return i;
}

__global__ __launch_bounds__(256) void k_cal_stream16(const uint4* __restrict__ in, uint4* sink, size_t n16) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = in[i];
        acc.x ^= v.x, acc.y ^= v.y, acc.z ^= v.z, acc.w ^= v.w;
    }
    if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) sink[0] = acc;  // never true for the zero buffer
}

// group g (of G = bytes / 512) = 4 consecutive 128-B lines; wave w handles groups perm(w*k ..): lane l reads element
// (l + rot) % 64 of the group, rot random per group
__global__ __launch_bounds__(256) void k_cal_gather8(const void* base, unsigned bytes, unsigned gmask, unsigned* sink) {
    const __amdgpu_buffer_rsrc_t r = rsrc(base, bytes);
    const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const unsigned nw = gridDim.x * 4;
    unsigned acc = 0;
    for (unsigned g = wave; g <= gmask; g += nw) {
        const unsigned grp = perm(g, gmask);
        const unsigned rot = mix32(grp) & 63;
        const unsigned el = (lane * 37u + rot) & 63;  // 37 odd: a permutation of the 64 elements
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, grp * 512u + el * 8u, 0, 0);
        acc ^= v.x ^ v.y;
    }
    if (acc == 0xDEADBEEFu) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_cal_gather4(const void* base, unsigned bytes, unsigned gmask, unsigned* sink) {
    const __amdgpu_buffer_rsrc_t r = rsrc(base, bytes);
    const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const unsigned nw = gridDim.x * 4;
    unsigned acc = 0;
    for (unsigned g = wave; g <= gmask; g += nw) {  // group = 2 lines = 256 B
        const unsigned grp = perm(g, gmask);
        const unsigned rot = mix32(grp) & 63;
        const unsigned el = (lane * 37u + rot) & 63;
        acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, grp * 256u + el * 4u, 0, 0);
    }
    if (acc == 0xDEADBEEFu) sink[0] = acc;
}

// 8 lines per wave instruction, lanes 8 per line, only bytes [0, 64) of each line
__global__ __launch_bounds__(256) void k_cal_half8(const void* base, unsigned bytes, unsigned gmask, unsigned* sink) {
    const __amdgpu_buffer_rsrc_t r = rsrc(base, bytes);
    const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const unsigned nw = gridDim.x * 4;
    unsigned acc = 0;
    for (unsigned g = wave; g <= gmask; g += nw) {  // group = 8 lines = 1 KiB
        const unsigned grp = perm(g, gmask);
        const unsigned rot = mix32(grp) & 63;
        const unsigned el = (lane * 37u + rot) & 63;
        const unsigned line = el >> 3, word = el & 7;
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, grp * 1024u + line * 128u + word * 8u, 0, 0);
        acc ^= v.x ^ v.y;
    }
    if (acc == 0xDEADBEEFu) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_cal_store8(void* base, unsigned bytes, unsigned gmask) {
    const __amdgpu_buffer_rsrc_t r = rsrc(base, bytes);
    const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const unsigned nw = gridDim.x * 4;
    for (unsigned g = wave; g <= gmask; g += nw) {
        const unsigned grp = perm(g, gmask);
        const unsigned rot = mix32(grp) & 63;
        const unsigned el = (lane * 37u + rot) & 63;
        u32x2 v;
        v.x = grp;
        v.y = el;
        __builtin_amdgcn_raw_buffer_store_b64(v, r, grp * 512u + el * 8u, 0, 0);
    }
}

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atol(argv[1]) : 1024;  // power of two, <= 2048 (32-bit buffer offsets)
    const size_t bytes = mib << 20;
    if ((mib & (mib - 1)) != 0 || mib < 512 || mib > 2048) {
        fprintf(stderr, "size must be a power of two in [512, 2048] MiB\n");
        return 2;
    }
    void *a = nullptr, *b = nullptr, *sink = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 256));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    CK(hipDeviceSynchronize());
    const int grid = 4096;
    const unsigned nb = (unsigned)(bytes - 1);  // buffer-resource byte size (fits 32 bits for <= 2 GiB - 1)
    // between patterns: stream the other 1-GiB buffer through, so no pattern finds the previous one's lines cached
    auto flush = [&]() { hipLaunchKernelGGL(k_cal_stream16, dim3(grid), dim3(256), 0, 0, (const uint4*)b, (uint4*)sink, bytes / 16); };
    hipLaunchKernelGGL(k_cal_stream16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)sink, bytes / 16);
    flush();
    hipLaunchKernelGGL(k_cal_gather8, dim3(grid), dim3(256), 0, 0, a, nb, (unsigned)(bytes / 512 - 1), (unsigned*)sink);
    flush();
    hipLaunchKernelGGL(k_cal_gather4, dim3(grid), dim3(256), 0, 0, a, nb, (unsigned)(bytes / 256 - 1), (unsigned*)sink);
    flush();
    hipLaunchKernelGGL(k_cal_half8, dim3(grid), dim3(256), 0, 0, a, nb, (unsigned)(bytes / 1024 - 1), (unsigned*)sink);
    flush();
    hipLaunchKernelGGL(k_cal_store8, dim3(grid), dim3(256), 0, 0, a, nb, (unsigned)(bytes / 512 - 1));
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    // the stream16 launches: the first reads `a`, the flushes read `b` -- all 1 GiB of compulsory reads each
    printf("{\"buffer_bytes\": %zu, \"known_read_bytes\": {\"k_cal_stream16\": %zu, \"k_cal_gather8\": %zu, "
           "\"k_cal_gather4\": %zu, \"k_cal_half8_used\": %zu, \"k_cal_half8_lines\": %zu}, "
           "\"known_write_bytes\": {\"k_cal_store8\": %zu}}\n",
           bytes, bytes, bytes, bytes, bytes / 2, bytes, bytes);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    return 0;
}
