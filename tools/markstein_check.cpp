// markstein_check.cpp — host proof-by-exhaustion / sampling for the reciprocal-table division of k_batch_integrate
// (csrc/tsdf.hip, FAST kernels): q0 = RN(a*y), r = fma(-b, q0, a), q = fma(r, y, q0) with y = RN(1/b) must equal the
// IEEE quotient RN(a/b) for every integer divisor b in [1, RCP_N] and every a the kernel can see.
//
// binary32 (the tsdf mean): the result scales exactly with powers of two away from underflow, so checking every
// significand of a in [1, 2) (both signs are symmetric) against every b is exhaustive.  `stride` > 1 checks every
// stride-th significand (the CPU test suite's quick mode).
// binary64 (the colour mean): `samples` random a per b -- uniform significands, exponents over the colour range
// [2^-40, 255 * 4096] -- plus a = k / b-style values next to quotient rounding boundaries.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -fopenmp markstein_check.cpp -o markstein_check
// Usage: markstein_check <stride_f32> <samples_f64_per_divisor>   prints "OK" or the first failures, exits 0 / 1.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static const int RCP_N = 4096;

static inline float q32(float a, float b, float y) {
    const float q0 = a * y;
    return std::fmaf(std::fmaf(-b, q0, a), y, q0);
}
static inline double q64(double a, double b, double y) {
    const double q0 = a * y;
    return std::fma(std::fma(-b, q0, a), y, q0);
}

static inline uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const long stride = argc > 1 ? atol(argv[1]) : 1;
    const long samples = argc > 2 ? atol(argv[2]) : 100000;
    long fails32 = 0, fails64 = 0, n32 = 0, n64 = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : fails32, fails64, n32, n64)
    for (int b = 1; b <= RCP_N; ++b) {
        const float bf = (float)b, y32 = 1.0f / bf;
        for (uint32_t m = 0; m < (1u << 23); m += (uint32_t)stride) {
            float a;
            const uint32_t bits = 0x3F800000u | m;  // [1, 2)
            std::memcpy(&a, &bits, 4);
            ++n32;
            if (q32(a, bf, y32) != a / bf) {
                if (fails32 < 5)
#pragma omp critical
                    fprintf(stderr, "f32 FAIL a=%a b=%d: %a vs %a\n", a, b, q32(a, bf, y32), a / bf);
                ++fails32;
            }
        }
        const double bd = (double)b, y64 = 1.0 / bd;
        uint64_t st = 0x1234567ull * (uint64_t)b;
        for (long i = 0; i < samples; ++i) {
            const uint64_t r = splitmix(st);
            double a;
            if (i & 1) {  // uniform significand, exponent in [-40, 20]
                const uint64_t bits = ((uint64_t)(1023 - 40 + (int)((r >> 52) % 61)) << 52) | (r & 0xFFFFFFFFFFFFFull);
                std::memcpy(&a, &bits, 8);
            } else {  // next to a rounding boundary of the quotient: a = (k + 1/2 ulp-ish) * b, then nudged
                const double k = (double)(r % (255ull * 4096ull)) + std::ldexp((double)((r >> 24) & 0xFFFF), -16);
                a = std::nextafter(k * bd, (r >> 63) ? 0.0 : 1e300);
            }
            ++n64;
            if (q64(a, bd, y64) != a / bd) {
                if (fails64 < 5)
#pragma omp critical
                    fprintf(stderr, "f64 FAIL a=%a b=%d: %a vs %a\n", a, b, q64(a, bd, y64), a / bd);
                ++fails64;
            }
        }
    }
    // the float64-colour kernel keeps one table and rounds its entries to float32 for the tsdf mean: no double
    // rounding may occur, (float)RN64(1/n) == RN32(1/n)
    long fails_dr = 0;
    for (int b = 1; b <= (1 << 20); ++b)
        if ((float)(1.0 / (double)b) != 1.0f / (float)b) ++fails_dr;
    fails32 += fails_dr;
    printf("f32 cases %ld (stride %ld) failures %ld; f64 cases %ld failures %ld; double-rounded reciprocals %ld\n", n32,
           stride, fails32, n64, fails64, fails_dr);
    if (fails32 || fails64) return 1;
    printf("OK\n");
    return 0;
}
