// chain.h — exact parallel evaluation of Open3D's serial float64 sums (kernels in mesh_ops.hip).
//
// s = ((0 + x_0) + x_1) + ... for x_t >= 0 (any input is accepted: chunks the fast path cannot prove are walked
// serially in the same order), bit-identical to the sequential loop.  Used by GetSurfaceArea / the sampling CDF
// (reconstruct_rgbd_filter.py:123) and by RemoveStatisticalOutliers' cloud mean and squared-deviation sum
// (std::accumulate / std::inner_product).
#pragma once

#include "common.h"

namespace ot {

constexpr int CHAIN_CH = 256;  // values per chunk: 64 lanes x 4

struct ChainJob {
    const double* x;  // input values (any alignment)
    int64_t n;
    double* out;      // CDF values (n), or the sum (out[0])
    double* bsum;
    int32_t* ex;
    long long* msum;
    int32_t* kind;    // 0 fast, 1 flagged by k_chain_chunk, 2 walked serially
    long long* pre;   // inclusive prefix of msum inside each run of chunks (k_chain_runs), saturated at 2^53
    int32_t* rend;    // last chunk of the run holding each chunk
    int32_t* seg_b;   // accepted segments (first chunk, exact N, prefix base) in walk order; count in *nseg
    long long* seg_n;
    long long* seg_base;
    int32_t* nseg;
    unsigned long long* trace = nullptr;  // test hook (otx_chain_walk_trace): per walk event {clock64, kind | chunk << 8}
    int trace_cap = 0;
};

// per-chain auxiliary arrays
inline size_t chain_aux_bytes(int64_t n) { return (size_t)((n + CHAIN_CH - 1) / CHAIN_CH + 1) * 64 + 512; }

inline char* chain_aux(char* cur, int64_t n, ChainJob& jb) {
    const int64_t nb = (n + CHAIN_CH - 1) / CHAIN_CH + 1;
    jb.bsum = (double*)cur;
    jb.msum = (long long*)(jb.bsum + nb);
    jb.pre = jb.msum + nb;
    jb.seg_n = jb.pre + nb;
    jb.seg_base = jb.seg_n + nb;
    jb.ex = (int32_t*)(jb.seg_base + nb);
    jb.kind = jb.ex + nb;
    jb.rend = jb.kind + nb;
    jb.seg_b = jb.rend + nb;
    jb.nseg = jb.seg_b + nb;
    cur = (char*)(jb.nseg + 2);
    return (char*)(((uintptr_t)cur + 63) & ~(uintptr_t)63);
}

// sums (out[0]) of n_jobs independent chains whose job table is on the device; max_n bounds every job's n
// (jobs with n == 0 write 0.0)
void launch_sum_chains(const ChainJob* djobs, int n_jobs, int64_t max_n, hipStream_t stream);

}  // namespace ot
