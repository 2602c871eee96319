// capi.hip — C-ABI plumbing: error reporting, version, scratch arena, host-side 4x4 inverse.
#include "common.h"
#include "srchash.h"  // generated in $(BUILD) by the Makefile

#include <atomic>
#include <cstring>
#include <mutex>
#include <vector>

namespace ot {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

ot_status fail(ot_status code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

// Grow-only per-device scratch buffers, indexed by slot (a caller-chosen small integer).  Growth happens
// with hipMalloc (synchronising) only when a larger request arrives; steady-state calls reuse the buffers.
// Per host thread: threads driving their own streams (e.g. several objects reconstructed concurrently) never
// share a buffer.  A thread's buffers live until the process ends (worker pools are long-lived).
struct Arena {
    std::vector<void*> ptr;
    std::vector<size_t> size;
};
static thread_local std::vector<Arena> g_arena;
static std::atomic<long long> g_allocs{0};

void note_alloc() { g_allocs.fetch_add(1, std::memory_order_relaxed); }
long long g_allocs_count() { return g_allocs.load(std::memory_order_relaxed); }

void* scratch(size_t bytes, int slot) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if ((int)g_arena.size() <= dev) g_arena.resize(dev + 1);
    Arena& a = g_arena[dev];
    if ((int)a.ptr.size() <= slot) {
        a.ptr.resize(slot + 1, nullptr);
        a.size.resize(slot + 1, 0);
    }
    if (a.size[slot] < bytes) {
        if (a.ptr[slot]) {
            (void)hipDeviceSynchronize();
            (void)hipFree(a.ptr[slot]);
        }
        size_t nb = bytes + bytes / 4 + 256;
        void* p = nullptr;
        if (hipMalloc(&p, nb) != hipSuccess) {
            a.ptr[slot] = nullptr;
            a.size[slot] = 0;
            return nullptr;
        }
        a.ptr[slot] = p;
        a.size[slot] = nb;
        note_alloc();
    }
    return a.ptr[slot];
}

static thread_local std::vector<Arena> g_pinned;

void* pinned_scratch(size_t bytes, int slot, bool coherent) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if ((int)g_pinned.size() <= dev) g_pinned.resize(dev + 1);
    Arena& a = g_pinned[dev];
    if ((int)a.ptr.size() <= slot) {
        a.ptr.resize(slot + 1, nullptr);
        a.size.resize(slot + 1, 0);
    }
    if (a.size[slot] < bytes) {
        if (a.ptr[slot]) (void)hipHostFree(a.ptr[slot]);  // synchronises the device
        const size_t nb = bytes + bytes / 4 + 256;
        void* p = nullptr;
        if (hipHostMalloc(&p, nb, coherent ? hipHostMallocCoherent : hipHostMallocDefault) != hipSuccess) {
            a.ptr[slot] = nullptr;
            a.size[slot] = 0;
            return nullptr;
        }
        a.ptr[slot] = p;
        a.size[slot] = nb;
        note_alloc();
    }
    return a.ptr[slot];
}

__global__ __launch_bounds__(64) void k_store_blob(ArgBlob b, unsigned long long* dst, int words) {
    for (int i = threadIdx.x; i < words; i += 64) dst[i] = b.w[i];
}

ot_status upload_small(void* dst, const void* src, size_t bytes, hipStream_t stream) {
    if (bytes == 0) return OT_OK;
    if (bytes > UPLOAD_ARG_BYTES || ((uintptr_t)dst & 7)) {
        OT_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
        return OT_OK;
    }
    ArgBlob b;
    std::memcpy(b.w, src, bytes);
    const int words = (int)((bytes + 7) / 8);  // whole words: the destination region is padded to 8 B
    hipLaunchKernelGGL(k_store_blob, dim3(1), dim3(64), 0, stream, b, (unsigned long long*)dst, words);
    OT_LAUNCH_CHECK();
    return OT_OK;
}

static inline double det3_helper(const double* m, int i1, int i2, int i3, int j1, int j2, int j3) {
    return m[i1 * 4 + j1] * (m[i2 * 4 + j2] * m[i3 * 4 + j3] - m[i2 * 4 + j3] * m[i3 * 4 + j2]);
}
static inline double cofactor4(const double* m, int i, int j) {
    const int i1 = (i + 1) % 4, i2 = (i + 2) % 4, i3 = (i + 3) % 4;
    const int j1 = (j + 1) % 4, j2 = (j + 2) % 4, j3 = (j + 3) % 4;
    const double a = det3_helper(m, i1, i2, i3, j1, j2, j3);
    const double b = det3_helper(m, i2, i3, i1, j1, j2, j3);
    const double c = det3_helper(m, i3, i1, i2, j1, j2, j3);
    return (a + b) + c;
}

// Open3D computes camera_pose = extrinsic.inverse() with Eigen's 4x4 inverse
// (CreatePointCloudFromFloatDepthImage, reached from ScalableTSDFVolume::Integrate and
// PointCloud::CreateFromRGBDImage).  Restated: cofactors, then division by the pairwise-summed determinant.
void inverse4(const double* m, double* r) {
    for (int row = 0; row < 4; ++row)
        for (int col = 0; col < 4; ++col) {
            const double c = cofactor4(m, col, row);
            r[row * 4 + col] = ((row + col) & 1) ? -c : c;
        }
    const double p0 = m[0] * r[0], p1 = m[4] * r[1], p2 = m[8] * r[2], p3 = m[12] * r[3];
    const double det = (p0 + p1) + (p2 + p3);
    for (int k = 0; k < 16; ++k) r[k] = r[k] / det;
}

}  // namespace ot

extern "C" {

const char* ot_last_error(void) { return ot::g_last_error.c_str(); }

// OT_SOURCE_HASH: _srchash.py over the sources this library was compiled from (generated by the Makefile);
// _lib.load() compares it with the sources beside the library and refuses a stale build
const char* ot_version(void) { return "otslam-mi355x 0.1.0 (gfx950) src=" OT_SOURCE_HASH; }

int32_t ot_abi_version(void) { return 1; }

}  // extern "C"

// test hook (not part of the drop-in boundary): allocations made by the library's grow-only buffers
extern "C" long long otx_alloc_count(void) { return ot::g_allocs_count(); }
