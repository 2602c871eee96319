// valu_rate.hip — measured VALU throughput on gfx950 for the integrate kernel's arithmetic mix (tools only).
// Independent FMA chains, 8 waves per SIMD, every CU busy: f32 (v_fma_f32), packed f32 (v_pk_fma_f32 on float2),
// f64 (v_fma_f64), and the f32 reciprocal (v_rcp_f32).  Prints wave-instructions per SIMD-cycle-equivalent as
// FLOP/s so VERDICT r3's "packed f32 halves the VALU cost" can be checked on the hardware.
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip && ./tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;
constexpr int CH = 8;

__global__ __launch_bounds__(256) void k_f32(float* out, float a, float b) {
    float x[CH];
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(x[c]) : "v"(x[c]), "v"(a), "v"(b));
    float s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    if (s == 12345.f) out[0] = s;
}
__global__ __launch_bounds__(256) void k_pk(float* out, float a, float b) {
    f2 x[CH];
    const f2 va = {a, a}, vb = {b, b};
    for (int c = 0; c < CH; ++c) x[c] = f2{threadIdx.x * 1e-3f + c, c * 2.0f};
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = __builtin_elementwise_fma(x[c], va, vb);
    float s = 0;
    for (int c = 0; c < CH; ++c) s += x[c].x + x[c].y;
    if (s == 12345.f) out[0] = s;
}
__global__ __launch_bounds__(256) void k_f64(float* out, double a, double b) {
    double x[CH];
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = __builtin_fma(x[c], a, b);
    double s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    if (s == 12345.0) out[0] = (float)s;
}
__global__ __launch_bounds__(256) void k_rcp(float* out, float a, float b) {
    float x[CH];
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = __builtin_amdgcn_rcpf(x[c]);
    float s = 0;
    for (int c = 0; c < CH; ++c) s += x[c];
    if (s == 12345.f) out[0] = s;
}

template <typename K, typename T>
static double run(K k, T a, T b, float* out, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, a, b);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, a, b);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    float* out = nullptr;
    (void)hipMalloc(&out, 64);
    hipDeviceProp_t pr;
    (void)hipGetDeviceProperties(&pr, 0);
    const int blocks = pr.multiProcessorCount * 8;  // 8 x 4 waves per CU = 8 waves per SIMD
    const double waves = blocks * 4.0, insts = waves * ITERS * CH;
    const double simds = pr.multiProcessorCount * 4.0;
    struct {
        const char* name;
        double ms;
    } r[4] = {{"v_fma_f32", run(k_f32, 1.0001f, 0.5f, out, blocks)},
              {"v_pk_fma_f32", run(k_pk, 1.0001f, 0.5f, out, blocks)},
              {"v_fma_f64", run(k_f64, 1.0001, 0.5, out, blocks)},
              {"v_rcp_f32", run(k_rcp, 1.0f, 0.0f, out, blocks)}};
    for (auto& x : r) {
        // wave-instructions per SIMD per microsecond, and the implied clock cycles per wave-instruction at 2.4 GHz
        const double per_simd_us = insts / simds / (x.ms * 1e3);
        printf("%-14s %.3f ms  %.1f wave-insts/SIMD/us  %.2f cycles per wave-inst at 2.4 GHz\n", x.name, x.ms,
               per_simd_us, 2400.0 / per_simd_us);
    }
    return 0;
}
