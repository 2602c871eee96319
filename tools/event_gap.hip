// Microbenchmark: GPU idle time that stream-ordered events and cross-stream waits insert between dependent kernels
// (single-object latency analysis).  Each case runs N dependent pairs of short kernels; the GPU time of
// the whole sequence (timing events around it) divided by N is compared with back-to-back kernels.  Also: the host's
// wake-up after a kernel, by hipEventSynchronize against spinning on a word the kernel stores to coherent host memory.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

__global__ void k_spin(int* buf, long long cycles) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 0) buf[blockIdx.x] += 1;
}
__global__ void k_spin_mail(int* buf, long long cycles, volatile unsigned* mail, unsigned seq) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 0) {
        buf[blockIdx.x] += 1;
        __threadfence_system();
        __hip_atomic_store((unsigned*)mail, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

struct Blob3K {
    unsigned long long w[384];
};
__global__ void k_spin_blob(int* buf, long long cycles, Blob3K b) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 0) buf[blockIdx.x] += (int)b.w[threadIdx.x];
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 200;
    const long long cyc = 2000;  // ~1 us at 2.4 GHz
    hipStream_t s, side;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    int* buf;
    CK(hipMalloc(&buf, 4096));
    CK(hipMemset(buf, 0, 4096));
    unsigned* mail;
    CK(hipHostMalloc((void**)&mail, 64, hipHostMallocCoherent));
    mail[0] = 0;
    hipEvent_t t0, t1, e, f, j;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    auto run = [&](const char* name, auto body) {
        for (int w = 0; w < 2; ++w) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, s));
            for (int i = 0; i < N; ++i) body(i);
            CK(hipEventRecord(t1, s));
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            if (w == 1) std::printf("%-44s %8.2f us per step\n", name, 1e3 * ms / N);
        }
    };
    run("2 kernels back to back", [&](int) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
    });
    Blob3K blob{};
    run("2 kernels, the 2nd with 3 KiB of arguments", [&](int) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
        hipLaunchKernelGGL(k_spin_blob, dim3(1), dim3(64), 0, s, buf, cyc, blob);
    });
    run("2 kernels + event record between", [&](int) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
        CK(hipEventRecord(e, s));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
    });
    run("2 kernels + 2 event records between", [&](int) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
        CK(hipEventRecord(e, s));
        CK(hipEventRecord(f, s));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
    });
    run("fork: 2nd kernel on side, join back", [&](int) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
        CK(hipEventRecord(f, s));
        CK(hipStreamWaitEvent(side, f, 0));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, side, buf + 64, cyc);
        CK(hipEventRecord(j, side));
        CK(hipStreamWaitEvent(s, j, 0));
    });
    run("fork + side kernel beside a main kernel", [&](int) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
        CK(hipEventRecord(f, s));
        CK(hipStreamWaitEvent(side, f, 0));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, side, buf + 64, cyc);
        CK(hipEventRecord(j, side));
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
        CK(hipStreamWaitEvent(s, j, 0));
    });
    // host round trip: kernel -> host sees completion -> host launches the next kernel
    for (int mode = 0; mode < 2; ++mode) {
        for (int w = 0; w < 2; ++w) {
            CK(hipDeviceSynchronize());
            auto h0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; ++i) {
                const unsigned seq = (unsigned)(w * N + i + 1 + mode * 4 * N);
                if (mode == 0) {
                    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, buf, cyc);
                    CK(hipEventRecord(e, s));
                    CK(hipEventSynchronize(e));
                } else {
                    hipLaunchKernelGGL(k_spin_mail, dim3(1), dim3(64), 0, s, buf, cyc, (volatile unsigned*)mail, seq);
                    while (__atomic_load_n(&mail[0], __ATOMIC_ACQUIRE) != seq) {}
                }
            }
            CK(hipDeviceSynchronize());
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
            if (w == 1)
                std::printf("%-44s %8.2f us per round trip\n", mode ? "host spins on a mailed word" : "event record + hipEventSynchronize", us / N);
        }
    }
    std::printf("DONE\n");
    return 0;
}
