// mc.hip — ScalableTSDFVolume::ExtractTriangleMesh on MI355X (reconstruct_rgbd_filter.py:112).
//
// Canonical output order (Open3D's follows unordered_map iteration; parity compares canonical order):
//   vertices  : sorted by the edge key's (owner unit key, owner-local voxel x*256+y*16+z, axis)
//   triangles : (unit key, voxel x*256+y*16+z, tri-table order), winding (e0, e2, e1) as Open3D.
// Pipeline (one 256-lane workgroup per unit, units in key order from the rocPRIM sort):
//   k_mc_prepare   : neighbour table (+x/+y/+z combos via the block hash), id->rank, clear edge bitmasks
//   k_mc_classify  : 17^3 tile of (weight == 0, tsdf < 0) flag bytes of the unit and its +1 neighbours in LDS; per
//                    voxel cube index (any weight == 0 => skipped, like Open3D); cut edges marked in the
//                    owner unit's edge bitmask (atomicOr); per-unit triangle count
//   k_mc_count     : per-unit popcount prefix over the 384 bitmask words => vertex ids without a hash map
//   (device scans of the per-unit counts give vertex / triangle bases)
//   k_mc_vertices  : one lane per bitmask word, vertex = half + vl*key, += f0*vl/(f0+f1) on the edge axis,
//                    colour (f1*c0 + f0*c1)/(f0+f1) with c = colour/255 — Open3D's float64 expressions
//   k_mc_triangles : per-lane triangle offsets by block scan; vertex ids by popcount lookups
#include <atomic>
#include <cstring>
#include <functional>
#include <mutex>
#include "../../include/otslam_mc_tables.h"
#include "compact.h"
#include "sort.h"
#include "tsdf.h"

namespace ot {

alignas(16) __constant__ signed char c_tri[256][16];  // rows are read as one 16-B word (k_mc_emit's triangles)
__constant__ int c_eshift[12][4];
__constant__ int c_e2v[12][2];
__constant__ int c_shift[8][3];
__constant__ unsigned char c_ntri[256];  // triangles per cube configuration (from c_tri)
__constant__ unsigned c_cinfo[256];      // per cube configuration: the edges its triangles use (bits 0-11), ntri << 12
// OT_MC_EDGE_SHIFT as a compile-time table: the emission's unrolled loop over a cube's 12 edges folds each edge's shift
// into constants instead of loading it per corner (upload_tables checks it against the header's)
constexpr int kEdgeShift[12][4] = {{0, 0, 0, 0}, {1, 0, 0, 1}, {0, 1, 0, 0}, {0, 0, 0, 1}, {0, 0, 1, 0}, {1, 0, 1, 1},
                                   {0, 1, 1, 0}, {0, 0, 1, 1}, {0, 0, 0, 2}, {1, 0, 0, 2}, {1, 1, 0, 2}, {0, 1, 0, 2}};

constexpr int EWORDS = (UNIT_VOX * 3) / 32;  // 384 bitmask words per unit
constexpr int T17 = 17;

struct McDev {
    const unsigned* sorted_ids;  // rank -> id
    int* rank_of;                // id -> rank
    int* nbr;                    // [id][16] neighbour ids: [0, 8) offsets +(dx, dy, dz), [8, 16) offsets -(dx, dy, dz),
                                 // index dx*4 + dy*2 + dz, dx, dy, dz in {0, 1}
    unsigned char* cubes;        // [id][4096]
    unsigned* eflags;            // [id][384]
    int* wprefix;                // [id][384]
    long long* tri_cnt;          // [rank]
    long long* vert_cnt;         // [rank]
    long long* tri_base;         // [rank]
    long long* vert_base;        // [rank]
    unsigned short* ctri;        // [id][4096] (cube byte order): first triangle of the cube inside its unit
    int4* vk;                    // per vertex: owner unit key + edge bit (the merge key of a sharded extraction)
    int* vown = nullptr;         // per vertex: owner unit id (written with vk)
    int32_t* tk;                 // per triangle: its cube's unit key
    long long cap_v = 0x7FFFFFFFFFFFFFFFll;  // emission: rows the destination arrays hold (writes beyond are dropped:
    long long cap_t = 0x7FFFFFFFFFFFFFFFll;  // a capacity guess made before the counts are known, then redone)
};

// the marching-cubes workspace of U units, carved from one allocation (kept with the volume: MeshBuffers::ws)
static size_t mc_ws_bytes(int64_t U) {
    return (size_t)U * (4 * 8 + 4 + 16 * 4 + EWORDS * 4 * 2 + UNIT_VOX + UNIT_VOX * 2) + 16 * 256;
}
static void mc_layout(char* ws, int64_t U, McDev& m) {
    char* p = ws;
    auto take = [&](size_t n) {
        char* q = p;
        p += (n + 255) & ~(size_t)255;
        return q;
    };
    m.tri_cnt = (long long*)take(sizeof(long long) * U);
    m.vert_cnt = (long long*)take(sizeof(long long) * U);
    m.tri_base = (long long*)take(sizeof(long long) * U);
    m.vert_base = (long long*)take(sizeof(long long) * U);
    m.rank_of = (int*)take(sizeof(int) * U);
    m.nbr = (int*)take(sizeof(int) * 16 * U);
    m.eflags = (unsigned*)take(sizeof(unsigned) * EWORDS * U);
    m.wprefix = (int*)take(sizeof(int) * EWORDS * U);
    m.cubes = (unsigned char*)take((size_t)UNIT_VOX * U);
    m.ctri = (unsigned short*)take(sizeof(unsigned short) * UNIT_VOX * U);
}

__device__ inline int find_unit(const TsdfDev& d, int x, int y, int z) {
    if (!key_in_range(x, y, z)) return -1;
    const unsigned long long key = pack_key(x, y, z);
    unsigned slot = (unsigned)mix64(key) & (unsigned)d.hash_mask;
    for (int probe = 0; probe <= d.hash_mask; ++probe) {
        const unsigned long long k = d.hkeys[slot];
        if (k == key) {
            const int id = d.hvals[slot];
            return id < d.max_units ? id : -1;
        }
        if (k == KEY_EMPTY) return -1;
        slot = (slot + 1) & (unsigned)d.hash_mask;
    }
    return -1;
}

// 16 units per workgroup, 16 lanes each (one workgroup per unit spent most of its ~8 us dispatching 5.6k workgroups of
// one object's mesh): lane q < 16 of a unit looks up neighbour combination q, and the 16 lanes clear the unit's 384
// edge words with 16-B stores
constexpr int PREP_UNITS = 16;
static_assert(EWORDS % 64 == 0, "16 lanes x 16-B stores cover a unit's edge words");
__global__ __launch_bounds__(256) void k_mc_prepare(TsdfDev d, McDev m, int U) {
    const int t = threadIdx.x, q16 = t & 15;
    const int r = (int)blockIdx.x * PREP_UNITS + (t >> 4);
    if (r >= U) return;
    const int id = (int)m.sorted_ids[r];
    const int sg = q16 < 8 ? 1 : -1, q = q16 & 7;
    const int dx = sg * ((q >> 2) & 1), dy = sg * ((q >> 1) & 1), dz = sg * (q & 1);
    m.nbr[id * 16 + q16] = q == 0 ? id
                                  : find_unit(d, d.unit_keys[id * 3] + dx, d.unit_keys[id * 3 + 1] + dy,
                                              d.unit_keys[id * 3 + 2] + dz);
    if (q16 == 0) m.rank_of[id] = r;
    uint4* ef = reinterpret_cast<uint4*>(m.eflags + (size_t)id * EWORDS);
    for (int w = q16; w < EWORDS / 4; w += 16) ef[w] = make_uint4(0u, 0u, 0u, 0u);
}

__global__ __launch_bounds__(256) void k_mc_classify(TsdfDev d, McDev m) {
    // Classification needs only two predicates per voxel (weight == 0, tsdf < 0): one flag byte each in LDS
    // (4.9 KiB per 17^3 tile instead of 39 KiB of floats), so many more units are resident per CU.  (Flag bytes written
    // by k_mc_prepare from a coalesced read of each unit, and the tiles staged from them instead of the floats:
    // classify 89 -> 59 us, but prepare 8 -> 53 us, r05u -- not kept.)
    __shared__ unsigned char sB[T17 * T17 * T17];
    __shared__ unsigned sflags[EWORDS];  // this unit's own edge bits; edges owned by a +1 neighbour go to HBM directly
    __shared__ int snbr[8];
    __shared__ long long wsum[4];
    const int r = blockIdx.x;
    const int id = (int)m.sorted_ids[r];
    const int t = threadIdx.x;
    // a spatially sharded volume emits only its own units' cubes; its halo units (other ranks' border voxels,
    // ot_tsdf_import_border) are read as neighbours and own the vertices of the edges on them
    if (d.shard_world > 1 &&
        !unit_owned(d, pack_key(d.unit_keys[id * 3], d.unit_keys[id * 3 + 1], d.unit_keys[id * 3 + 2]))) {
        *reinterpret_cast<uint4*>(m.cubes + (size_t)id * UNIT_VOX + t * 16) = make_uint4(0u, 0u, 0u, 0u);
        if (t == 0) m.tri_cnt[r] = 0;
        return;
    }
    if (t < 8) snbr[t] = m.nbr[id * 16 + t];
    for (int w = t; w < EWORDS; w += 256) sflags[w] = 0u;
    __syncthreads();
    // Tile staging, every load of a lane issued before any is consumed: the unit's own 16^3 voxels as lane t's y-row
    // (z = t >> 4, x = t & 15: 16 contiguous floats, four 16-B loads per plane), then one voxel per lane of each +x /
    // +y / +z neighbour face and the 49 voxels of the three +edges and the corner (lanes 0-48).  (Round 4 staged the
    // 17^3 positions in pool order, 20 scalar load pairs per lane: 88-91 us per configs[3] object.)  A missing
    // neighbour reads as weight 0.
    const auto flag = [](float f, float w) { return (unsigned char)((w == 0.0f ? 1 : 0) | (f < 0.0f ? 2 : 0)); };
    {
        const int a = t >> 4, b = t & 15;
        const float* own = unit_base(d, id);
        const float4* tp = reinterpret_cast<const float4*>(own) + t * 4;
        const float4* wp = reinterpret_cast<const float4*>(own + UNIT_VOX) + t * 4;
        float4 tv[4], wv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tv[k] = tp[k];
            wv[k] = wp[k];
        }
        // faces: +y (lz a, lx b, ly 16), +x (lz a, lx 16, ly b), +z (lz 16, lx a, ly b)
        float fy = 0.0f, wy = 0.0f, fx = 0.0f, wx = 0.0f, fz = 0.0f, wz = 0.0f, fe = 0.0f, we = 0.0f;
        const int ny = snbr[2], nx = snbr[4], nz = snbr[1];
        if (ny >= 0) {
            fy = unit_base(d, ny)[a * 256 + b * 16];
            wy = unit_base(d, ny)[UNIT_VOX + a * 256 + b * 16];
        }
        if (nx >= 0) {
            fx = unit_base(d, nx)[a * 256 + b];
            wx = unit_base(d, nx)[UNIT_VOX + a * 256 + b];
        }
        if (nz >= 0) {
            fz = unit_base(d, nz)[a * 16 + b];
            wz = unit_base(d, nz)[UNIT_VOX + a * 16 + b];
        }
        // edges: (16, 16, lz = t) in n6, (16, ly = t - 16, 16) in n5, (lx = t - 32, 16, 16) in n3, the corner in n7
        int ne = -1, ve = 0, se = 0;
        if (t < 16) ne = snbr[6], ve = t * 256, se = (16 * T17 + 16) * T17 + t;
        else if (t < 32) ne = snbr[5], ve = t - 16, se = (16 * T17 + (t - 16)) * T17 + 16;
        else if (t < 48) ne = snbr[3], ve = (t - 32) * 16, se = ((t - 32) * T17 + 16) * T17 + 16;
        else if (t == 48) ne = snbr[7], ve = 0, se = (16 * T17 + 16) * T17 + 16;
        if (ne >= 0) {
            fe = unit_base(d, ne)[ve];
            we = unit_base(d, ne)[UNIT_VOX + ve];
        }
        const float f16[16] = {tv[0].x, tv[0].y, tv[0].z, tv[0].w, tv[1].x, tv[1].y, tv[1].z, tv[1].w,
                               tv[2].x, tv[2].y, tv[2].z, tv[2].w, tv[3].x, tv[3].y, tv[3].z, tv[3].w};
        const float w16[16] = {wv[0].x, wv[0].y, wv[0].z, wv[0].w, wv[1].x, wv[1].y, wv[1].z, wv[1].w,
                               wv[2].x, wv[2].y, wv[2].z, wv[2].w, wv[3].x, wv[3].y, wv[3].z, wv[3].w};
#pragma unroll
        for (int y = 0; y < 16; ++y) sB[(b * T17 + y) * T17 + a] = flag(f16[y], w16[y]);
        sB[(b * T17 + 16) * T17 + a] = flag(fy, wy);
        sB[(16 * T17 + b) * T17 + a] = flag(fx, wx);
        sB[(a * T17 + b) * T17 + 16] = flag(fz, wz);
        if (t <= 48) sB[se] = flag(fe, we);
    }
    __syncthreads();
    const int x = t >> 4, y = t & 15;
    long long ntri = 0;
    unsigned packed[4] = {0u, 0u, 0u, 0u};  // this lane's 16 cube bytes ([x][y][z] layout), one 16-B store
#pragma unroll
    for (int z = 0; z < UNIT_RES; ++z) {
        int cube = 0;
        bool valid = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int c = ((x + c_shift[i][0]) * T17 + (y + c_shift[i][1])) * T17 + (z + c_shift[i][2]);
            const int b = sB[c];
            if (b & 1) valid = false;
            if (b & 2) cube |= (1 << i);
        }
        if (!valid) cube = 0;
        if (cube == 255) cube = 0;
        packed[z >> 2] |= (unsigned)cube << ((z & 3) * 8);
        if (cube == 0) continue;
        ntri += c_ntri[cube];
#pragma unroll
        for (int e = 0; e < 12; ++e) {
            const int v0 = c_e2v[e][0], v1 = c_e2v[e][1];
            if (((cube >> v0) & 1) == ((cube >> v1) & 1)) continue;
            const int ox = x + c_eshift[e][0], oy = y + c_eshift[e][1], oz = z + c_eshift[e][2];
            const int nb = ((ox >> 4) << 2) | ((oy >> 4) << 1) | (oz >> 4);
            const int local = (ox & 15) * 256 + (oy & 15) * 16 + (oz & 15);
            const int bit = local * 3 + c_eshift[e][3];
            if (nb == 0) {
                atomicOr(&sflags[bit >> 5], 1u << (bit & 31));
            } else {
                const int owner = snbr[nb];
                if (owner >= 0) atomicOr(&m.eflags[(size_t)owner * EWORDS + (bit >> 5)], 1u << (bit & 31));
            }
        }
    }
    *reinterpret_cast<uint4*>(m.cubes + (size_t)id * UNIT_VOX + t * 16) = make_uint4(packed[0], packed[1], packed[2], packed[3]);
    ntri = wave_sum(ntri);
    if (lane_id() == 0) wsum[t >> 6] = ntri;
    __syncthreads();
    if (t == 0) m.tri_cnt[r] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    // neighbours' classify blocks may set bits of this unit's words too: merge, do not overwrite
    for (int w = t; w < EWORDS; w += 256) {
        const unsigned b = sflags[w];
        if (b) atomicOr(&m.eflags[(size_t)id * EWORDS + w], b);
    }
}

// per-unit exclusive popcount prefix of the 384 bitmask words: one wave per unit, 6 consecutive words per lane, 4 units
// per workgroup (one 384-thread workgroup per unit spent most of its ~10 us dispatching one object's 5.6k workgroups)
constexpr int CNT_UNITS = 4;
constexpr int CNT_PER_LANE = EWORDS / 64;
static_assert(CNT_PER_LANE == 6, "3 x 8-B loads per lane");
__global__ __launch_bounds__(64 * CNT_UNITS) void k_mc_count(McDev m, int U) {
    const int lane = (int)lane_id();
    const int r = (int)blockIdx.x * CNT_UNITS + ((int)threadIdx.x >> 6);
    if (r >= U) return;  // wave-uniform
    const int id = (int)m.sorted_ids[r];
    const uint2* ef = reinterpret_cast<const uint2*>(m.eflags + (size_t)id * EWORDS + lane * CNT_PER_LANE);
    int pc[CNT_PER_LANE], loc = 0;
#pragma unroll
    for (int k = 0; k < CNT_PER_LANE / 2; ++k) {
        const uint2 v = ef[k];
        pc[2 * k] = __popc(v.x);
        pc[2 * k + 1] = __popc(v.y);
        loc += pc[2 * k] + pc[2 * k + 1];
    }
    const int inc = wave_incl_scan(loc);
    int run = inc - loc;
    int* wp = m.wprefix + (size_t)id * EWORDS + lane * CNT_PER_LANE;
#pragma unroll
    for (int k = 0; k < CNT_PER_LANE; ++k) {
        wp[k] = run;
        run += pc[k];
    }
    if (lane == 63) m.vert_cnt[r] = inc;
}

// tsdf and colour of one voxel; colour from the float64 pool when the volume keeps it (exact: a float colour widens
// to double exactly, as Open3D's float-to-double promotion)
__device__ inline void voxel_value(const TsdfDev& d, int id, int x, int y, int z, float& f, double c[3]) {
    const float* base = unit_base(d, id);
    const int vi = z * 256 + x * 16 + y;
    f = base[vi];
    if (d.color64) {
        const double* cb = color_base<double>(d, id);
        c[0] = cb[vi];
        c[1] = cb[UNIT_VOX + vi];
        c[2] = cb[2 * UNIT_VOX + vi];
    } else {
        const float* cb = color_base<float>(d, id);
        c[0] = (double)cb[vi];
        c[1] = (double)cb[UNIT_VOX + vi];
        c[2] = (double)cb[2 * UNIT_VOX + vi];
    }
}

// exclusive scan over an NT-thread workgroup (every thread of the workgroup must call it: two barriers)
template <int NT>
__device__ inline int block_excl_scan_n(int v, int& total) {
    __shared__ int wsum[NT / 64];
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    const int inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const int s = wsum[w];
        if (w < wid) off += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return off + inc - v;
}

// one unit's vertices (rank r), EWORDS lanes.  Lane w reads edge-bitmask word w; one block scan of the words' popcounts
// lists the unit's cut edges in LDS in edge-key order (list index = the vertex's id inside the unit: the word prefixes
// count the same bits in the same order), and the lanes then take the listed vertices one each (round 6: a word's
// vertices had been one lane's serial chain while most lanes held none).  The unit's +x / +y / +z neighbour ids are
// staged in LDS (not one dependent global load per vertex before its neighbour voxel's loads).  (A wave per unit, each
// lane walking six words, measured 193 vs 109 us for the emission, r05t: fewer waves, longer chains.)
// lds: >= VLIST_BYTES
constexpr int VLIST_BYTES = UNIT_VOX * 3 * 2;  // u16 edge bit per listed vertex (<= 3 per voxel)
__device__ __forceinline__ void mc_vertices_unit(const TsdfDev& d, const McDev& m, double vl, double* V, double* VC,
                                                 int r, int w, unsigned char* lds) {
    __shared__ int s_vnbr[8];
    unsigned short* s_vl = reinterpret_cast<unsigned short*>(lds);
    const int id = (int)m.sorted_ids[r];
    if (w < 8) s_vnbr[w] = m.nbr[id * 16 + w];
    unsigned bits = m.eflags[(size_t)id * EWORDS + w];
    int nv;
    int slot = block_excl_scan_n<EWORDS>(__popc(bits), nv);  // (its barriers also publish s_vnbr)
    while (bits) {
        const int b = __ffs(bits) - 1;
        bits &= bits - 1;
        s_vl[slot++] = (unsigned short)(w * 32 + b);
    }
    __syncthreads();
    const long long vbase = m.vert_base[r];
    const int kx = d.unit_keys[id * 3], ky = d.unit_keys[id * 3 + 1], kz = d.unit_keys[id * 3 + 2];
    const double half = vl * 0.5;
    for (int i = w; i < nv; i += EWORDS) {
        const int gbit = (int)s_vl[i];
        const long long vid = vbase + i;
        const int local = gbit / 3, axis = gbit % 3;
        const int x = local >> 8, y = (local >> 4) & 15, z = local & 15;
        float f0f, f1f;
        double c0[3], c1[3];
        voxel_value(d, id, x, y, z, f0f, c0);
        int x1 = x + (axis == 0), y1 = y + (axis == 1), z1 = z + (axis == 2);
        const int nid = s_vnbr[((x1 >> 4) << 2) | ((y1 >> 4) << 1) | (z1 >> 4)];
        if (nid < 0) {  // cannot happen for a valid cube (its corners have weight > 0); never read out of bounds
            f1f = f0f;
            c1[0] = c0[0], c1[1] = c0[1], c1[2] = c0[2];
        } else {
            voxel_value(d, nid, x1 & 15, y1 & 15, z1 & 15, f1f, c1);
        }
        const int g[3] = {kx * UNIT_RES + x, ky * UNIT_RES + y, kz * UNIT_RES + z};
        double pt[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) pt[a] = half + vl * (double)g[a];
        const double f0 = fabs((double)f0f), f1 = fabs((double)f1f);
        pt[axis] += f0 * vl / (f0 + f1);
        if (vid < m.cap_v) {
#pragma unroll
            for (int a = 0; a < 3; ++a) V[vid * 3 + a] = pt[a];
            if (m.vk) m.vk[vid] = make_int4(kx, ky, kz, gbit);
            if (m.vown) m.vown[vid] = id;
            if (VC) {
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const double a0 = c0[a] / 255.0, a1 = c1[a] / 255.0;
                    VC[vid * 3 + a] = (f1 * a0 + f0 * a1) / (f0 + f1);
                }
            }
        }
    }
}

// v[e] for a per-lane e in [0, 12): a select tree (a register array indexed by a per-lane value would go to scratch)
__device__ __forceinline__ int pick12(const int (&v)[12], int e) {
    const bool b0 = e & 1, b1 = e & 2;
    const int p0 = b0 ? v[1] : v[0], p1 = b0 ? v[3] : v[2], p2 = b0 ? v[5] : v[4], p3 = b0 ? v[7] : v[6];
    const int p4 = b0 ? v[9] : v[8], p5 = b0 ? v[11] : v[10];
    const int q0 = b1 ? p1 : p0, q1 = b1 ? p3 : p2, q2 = b1 ? p5 : p4;
    return (e & 8) ? q2 : ((e & 4) ? q1 : q0);
}


// one unit's triangles (rank r).  Lanes [0, 256) own one (x, y) column of 16 cubes each for the counts: one block scan
// gives every column its first triangle and its first non-empty cube, the per-cube offsets (ctri) are written, and the
// non-empty cubes are listed in LDS in voxel order.  Then the workgroup's NT lanes take the LISTED cubes one each (round
// 6: a unit's ~10-30 surface cubes were spread over a few columns, whose lanes walked their 16 z in series while the
// rest idled; now each cube is one lane's single chain).  An NT-thread workgroup (k_mc_emit runs the triangles in its
// 384-lane workgroups) keeps every lane through every barrier (no reliance on exited waves).
// lds: >= TLIST_BYTES
constexpr int TLIST_BYTES = UNIT_VOX * 5;  // per listed cube: u32 (first triangle inside the unit << 12 | local voxel)
                                           // + its cube index byte
template <int NT>
__device__ __forceinline__ void mc_triangles_unit(const TsdfDev& d, const McDev& m, int32_t* T, int r, int t,
                                                  unsigned char* lds) {
    static_assert(NT >= 256 && NT % 64 == 0, "a unit's 256 columns need >= 256 lanes");
    const bool col = t < 256;
    __shared__ int snbr[8];
    __shared__ long long sbase[8];
    unsigned* s_list = reinterpret_cast<unsigned*>(lds);
    unsigned char* s_cube = lds + UNIT_VOX * 4;
    const int id = (int)m.sorted_ids[r];
    const int ukey[3] = {d.unit_keys[id * 3], d.unit_keys[id * 3 + 1], d.unit_keys[id * 3 + 2]};
    if (t < 8) {
        const int o = m.nbr[id * 16 + t];
        snbr[t] = o;
        sbase[t] = o >= 0 ? m.vert_base[m.rank_of[o]] : 0;
    }
    uint4 q = make_uint4(0u, 0u, 0u, 0u);
    if (col) q = *reinterpret_cast<const uint4*>(m.cubes + (size_t)id * UNIT_VOX + t * 16);
    const unsigned cw[4] = {q.x, q.y, q.z, q.w};
    int cnt = 0;  // non-empty cubes << 16 | triangles (a column's prefix of triangles < 256 * 80 < 2^16)
#pragma unroll
    for (int z = 0; z < UNIT_RES; ++z) {
        const int nt = c_ntri[(cw[z >> 2] >> ((z & 3) * 8)) & 0xFFu];
        cnt += nt + (nt ? (1 << 16) : 0);
    }
    int total;
    const int pre = block_excl_scan_n<NT>(cnt, total);  // contains __syncthreads (snbr visible after)
    if (col) {
        // per cube its first triangle inside the unit (<= 5 * 4096 < 2^16): the vertex-normal walk's index
        unsigned off[8];
        int o = pre & 0xFFFF, slot = pre >> 16;
#pragma unroll
        for (int z = 0; z < UNIT_RES; z += 2) {
            const int c0 = (int)((cw[z >> 2] >> ((z & 3) * 8)) & 0xFFu);
            const int c1 = (int)((cw[(z + 1) >> 2] >> (((z + 1) & 3) * 8)) & 0xFFu);
            const int n0 = c_ntri[c0], n1 = c_ntri[c1];
            off[z >> 1] = (unsigned)o | ((unsigned)(o + n0) << 16);
            if (n0) {
                s_list[slot] = ((unsigned)o << 12) | (unsigned)(t * 16 + z);
                s_cube[slot++] = (unsigned char)c0;
            }
            if (n1) {
                s_list[slot] = ((unsigned)(o + n0) << 12) | (unsigned)(t * 16 + z + 1);
                s_cube[slot++] = (unsigned char)c1;
            }
            o += n0 + n1;
        }
        uint4* dst = reinterpret_cast<uint4*>(m.ctri + (size_t)id * UNIT_VOX + t * 16);
        dst[0] = make_uint4(off[0], off[1], off[2], off[3]);
        dst[1] = make_uint4(off[4], off[5], off[6], off[7]);
    }
    __syncthreads();
    const int ncubes = total >> 16;
    const long long tbase = m.tri_base[r];
    // per listed cube two round trips: its table row and edge set, then the owner words and prefixes of every edge it
    // uses (the 12 edges unrolled, each shift a constant), all issued before any is used; a corner's vertex id is sbase
    // (the owner's first vertex) + the word's prefix + the set bits below its own -- the cut edges' ids are formed once
    // per cube, not once per corner
    for (int i = t; i < ncubes; i += NT) {
        const unsigned ent = s_list[i];
        const int cube = (int)s_cube[i];
        const int lv = (int)(ent & 0xFFFu);
        const int x = lv >> 8, y = (lv >> 4) & 15, z = lv & 15;
        long long out = tbase + (long long)(ent >> 12);
        const int4 row = *reinterpret_cast<const int4*>(&c_tri[cube][0]);
        const unsigned info = c_cinfo[cube];
        unsigned wb[12];
        int wp[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) {
            const int ox = x + kEdgeShift[e][0], oy = y + kEdgeShift[e][1], oz = z + kEdgeShift[e][2];
            const int o = ((ox >> 4) << 2) | ((oy >> 4) << 1) | (oz >> 4);
            const int owner = snbr[o];
            const int word = (((ox & 15) * 256 + (oy & 15) * 16 + (oz & 15)) * 3 + kEdgeShift[e][3]) >> 5;
            wb[e] = 0u;
            wp[e] = 0;
            if (((info >> e) & 1u) && owner >= 0) {
                wb[e] = m.eflags[(size_t)owner * EWORDS + word];
                wp[e] = m.wprefix[(size_t)owner * EWORDS + word];
            }
        }
        int vid[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) {
            const int ox = x + kEdgeShift[e][0], oy = y + kEdgeShift[e][1], oz = z + kEdgeShift[e][2];
            const int o = ((ox >> 4) << 2) | ((oy >> 4) << 1) | (oz >> 4);
            const int bit = ((ox & 15) * 256 + (oy & 15) * 16 + (oz & 15)) * 3 + kEdgeShift[e][3];
            const unsigned below = wb[e] & ((1u << (bit & 31)) - 1u);
            vid[e] = snbr[o] < 0 ? 0 : (int)(sbase[o] + wp[e] + __popc(below));
        }
        const int nt = (int)(info >> 12);
        const unsigned rw[4] = {(unsigned)row.x, (unsigned)row.y, (unsigned)row.z, (unsigned)row.w};
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k >= nt) break;
            const int ea = (int)((rw[(3 * k) >> 2] >> (((3 * k) & 3) * 8)) & 0xFFu);
            const int eb = (int)((rw[(3 * k + 1) >> 2] >> (((3 * k + 1) & 3) * 8)) & 0xFFu);
            const int ec = (int)((rw[(3 * k + 2) >> 2] >> (((3 * k + 2) & 3) * 8)) & 0xFFu);
            const int a = pick12(vid, ea), b = pick12(vid, eb), c = pick12(vid, ec);
            if (out < m.cap_t) {
                T[out * 3 + 0] = a;
                T[out * 3 + 1] = c;
                T[out * 3 + 2] = b;
                if (m.tk) {
                    m.tk[out * 3 + 0] = ukey[0];
                    m.tk[out * 3 + 1] = ukey[1];
                    m.tk[out * 3 + 2] = ukey[2];
                }
            }
            ++out;
        }
    }
}

constexpr int EMIT_LDS = VLIST_BYTES > TLIST_BYTES ? VLIST_BYTES : TLIST_BYTES;
__global__ __launch_bounds__(EWORDS) void k_mc_vertices(TsdfDev d, McDev m, double vl, double* V, double* VC) {
    __shared__ alignas(16) unsigned char lds[VLIST_BYTES];
    mc_vertices_unit(d, m, vl, V, VC, blockIdx.x, threadIdx.x, lds);
}
__global__ __launch_bounds__(256) void k_mc_triangles(TsdfDev d, McDev m, int32_t* T) {
    __shared__ alignas(16) unsigned char lds[TLIST_BYTES];
    mc_triangles_unit<256>(d, m, T, blockIdx.x, threadIdx.x, lds);
}
// The emission in ONE launch: workgroups [0, U) the triangles (their upper 128 lanes take part in the scan's barriers
// and in the listed cubes), [U, 2U) the vertices; the two halves' cube / vertex lists share one LDS block.  Replaces the
// vertices on the side stream beside the triangles: that fork and join cost the GPU ~25 us of idle queue time per
// extraction (tools/event_gap.hip, r05j)
__global__ __launch_bounds__(EWORDS) void k_mc_emit(TsdfDev d, McDev m, int U, double vl, double* V, double* VC,
                                                    int32_t* T) {
    __shared__ alignas(16) unsigned char lds[EMIT_LDS];
    const int b = blockIdx.x;
    if (b < U) {
        mc_triangles_unit<EWORDS>(d, m, T, b, threadIdx.x, lds);
    } else {
        mc_vertices_unit(d, m, vl, V, VC, b - U, threadIdx.x, lds);
    }
}

// TriangleMesh::ComputeVertexNormals of an extracted mesh from its marching-cubes structure: a vertex is
// a cut edge (global voxel g, axis a), and exactly the 4 cubes g - eshift(e) over the 4 edges e along a contain it.
// Their triangles are the vertex's triangles; walking the cubes in ascending triangle index (unit rank, then the cube's
// offset inside the unit) and each cube's triangles in table order adds the triangle normals in triangle order --
// Open3D's loop over the triangles -- with no sort of the 3T corners.  One lane per vertex.
// The walk is one lane's chain of dependent loads, so its loads issue in phases: the owner id (stored by the emission,
// no hash probe) -> the 4 cubes' neighbour ids -> their cube bytes, ranks and in-unit triangle offsets -> their triangle
// bases; then per cube (in triangle order) the rows of its triangles that contain the edge, then their corners.  The 4
// edges along each axis are a fixed table (no register array indexed at run time).  A cube's triangles are its first
// c_ntri[cube] table rows: the rows after the -1 terminator are ZERO-filled, and testing them for the edge would count
// phantom triangles of edge 0 (round 4's mismatch).
__constant__ unsigned char c_axis_edges[3][4] = {{0, 2, 4, 6}, {1, 3, 5, 7}, {8, 9, 10, 11}};
__global__ __launch_bounds__(256) void k_mc_vnormals(TsdfDev d, McDev m, int64_t units, const double* __restrict__ V,
                                                     const int32_t* __restrict__ T, int64_t nv, double* __restrict__ N) {
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= nv) return;
    const int4 key = m.vk[v];
    const int local = key.w / 3, axis = key.w % 3;
    const int g[3] = {key.x * UNIT_RES + (local >> 8), key.y * UNIT_RES + ((local >> 4) & 15),
                      key.z * UNIT_RES + (local & 15)};
    const int owner = m.vown ? m.vown[v] : find_unit(d, key.x, key.y, key.z);  // the emission's owner id: no probe
    if (owner < 0 || owner >= units) return;  // cannot happen for a vertex of this extraction
    int edge[4], id[4], ci[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int e = c_axis_edges[axis][k];
        const int c[3] = {g[0] - c_eshift[e][0], g[1] - c_eshift[e][1], g[2] - c_eshift[e][2]};
        // the cube's unit is the owner or one of its -x/-y/-z neighbours (arithmetic shift: floor for negatives)
        const int ox = key.x - (c[0] >> 4), oy = key.y - (c[1] >> 4), oz = key.z - (c[2] >> 4);
        edge[k] = e;
        ci[k] = ((c[0] & 15) * 16 + (c[1] & 15)) * 16 + (c[2] & 15);
        id[k] = m.nbr[owner * 16 + 8 + (ox << 2 | oy << 1 | oz)];
    }
    int cubev[4], rk[4], ct[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const bool ok = id[k] >= 0 && id[k] < units;
        cubev[k] = ok ? (int)m.cubes[(size_t)id[k] * UNIT_VOX + ci[k]] : 0;
        rk[k] = ok ? m.rank_of[id[k]] : 0;
        ct[k] = ok ? (int)m.ctri[(size_t)id[k] * UNIT_VOX + ci[k]] : 0;
    }
    long long start[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) start[k] = cubev[k] ? m.tri_base[rk[k]] + ct[k] : 0x7FFFFFFFFFFFFFFFll;
    // ascending triangle index: a 4-input sorting network (empty cubes sort last)
    auto cswap = [&](int a, int b) {
        if (start[b] < start[a]) {
            const long long ts = start[a];
            start[a] = start[b], start[b] = ts;
            const int tc = cubev[a];
            cubev[a] = cubev[b], cubev[b] = tc;
            const int te = edge[a];
            edge[a] = edge[b], edge[b] = te;
        }
    };
    cswap(0, 1);
    cswap(2, 3);
    cswap(0, 2);
    cswap(1, 3);
    cswap(1, 2);
    double n[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (cubev[i]) {  // empty cubes sorted last
            const int cube = cubev[i], e = edge[i], nt = c_ntri[cube];
            // the cube's table triangles (its first nt rows, in order) that contain the edge: rows, then corners, sum
            bool has[5];
            int row[5][3];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int t0 = c_tri[cube][3 * k], t1 = c_tri[cube][3 * k + 1], t2 = c_tri[cube][3 * k + 2];
                has[k] = k < nt && (t0 == e || t1 == e || t2 == e);
                const long long tri = start[i] + k;
#pragma unroll
                for (int r = 0; r < 3; ++r) row[k][r] = has[k] ? T[tri * 3 + r] : 0;
            }
#pragma unroll
            for (int k = 0; k < 5; ++k)
                if (has[k]) {
                    double tn[3];
                    triangle_normal(V, row[k][0], row[k][1], row[k][2], tn);
                    n[0] += tn[0];
                    n[1] += tn[1];
                    n[2] += tn[2];
                }
        }
    }
    finish_vertex_normal(n);
    N[v * 3 + 0] = n[0];
    N[v * 3 + 1] = n[1];
    N[v * 3 + 2] = n[2];
}

// the extraction's two exclusive scans (triangle and vertex counts per unit, U of each) in one launch: block 0 scans
// the triangle counts, block 1 the vertex counts, 4096 per round (4 consecutive per thread) with a carried total --
// one ~5 us launch instead of a library scan's two launches per array (U is a few thousand units).  Each block mails
// its array's total (triangles, vertices) to the volume's pinned mailbox, then `seq` to its sequence word (seqw[block]):
// the host spins on those (mail_wait), with no launch or event of its own
__global__ __launch_bounds__(1024) void k_mc_scan2(const long long* __restrict__ c0, long long* __restrict__ b0,
                                                  const long long* __restrict__ c1, long long* __restrict__ b1,
                                                  int n, long long* __restrict__ totals, unsigned* __restrict__ seqw,
                                                  unsigned seq) {
    const long long* in = blockIdx.x ? c1 : c0;
    long long* out = blockIdx.x ? b1 : b0;
    __shared__ long long wsum[16];
    __shared__ long long s_carry;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) s_carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 4096) {
        const int i0 = base + 4 * t;
        long long v[4], loc = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = i0 + k < n ? in[i0 + k] : 0;
            loc += v[k];
        }
        long long inc = loc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const long long o = __shfl_up(inc, d);
            if (lane >= d) inc += o;
        }
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        long long off = s_carry, tot = 0;
        for (int q = 0; q < 16; ++q) {
            off += q < w ? wsum[q] : 0;
            tot += wsum[q];
        }
        long long run = off + inc - loc;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (i0 + k < n) out[i0 + k] = run;
            run += v[k];
        }
        __syncthreads();
        if (t == 0) s_carry += tot;
        __syncthreads();
    }
    if (t == 0) {
        totals[blockIdx.x] = s_carry;
        __threadfence_system();  // the total reaches the host before the sequence word
        __hip_atomic_store(seqw + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static std::atomic<bool> g_tables_uploaded{false};
static bool g_mc_emit_fork = false;  // test hook otx_mc_emit_fork: the two-stream emission (round 4) for A/B timing
// ot_tsdf_extract_sample_min_z: where the vertex normals may start -- 0 right after the emission, 1 beside the area-sum
// walk, 2 beside the CDF walk (test hook otx_normals_at)
static int g_normals_at = 1;
static std::mutex g_tables_mutex;

static ot_status upload_tables() {  // once per process (one process per GPU), safe from concurrent host threads
    if (g_tables_uploaded.load(std::memory_order_acquire)) return OT_OK;
    std::lock_guard<std::mutex> lock(g_tables_mutex);
    if (g_tables_uploaded.load(std::memory_order_relaxed)) return OT_OK;
    OT_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_tri), OT_MC_TRI_TABLE, sizeof(OT_MC_TRI_TABLE)));
    OT_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_eshift), OT_MC_EDGE_SHIFT, sizeof(OT_MC_EDGE_SHIFT)));
    OT_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_e2v), OT_MC_EDGE_TO_VERT, sizeof(OT_MC_EDGE_TO_VERT)));
    OT_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_shift), OT_MC_SHIFT, sizeof(OT_MC_SHIFT)));
    unsigned char ntri[256];
    for (int c = 0; c < 256; ++c) {
        int n = 0;
        for (int k = 0; k < 15 && OT_MC_TRI_TABLE[c][k] != -1; k += 3) ++n;
        ntri[c] = (unsigned char)n;
    }
    OT_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_ntri), ntri, sizeof(ntri)));
    unsigned cinfo[256];
    for (int c = 0; c < 256; ++c) {
        unsigned em = 0u;
        for (int k = 0; k < 3 * ntri[c]; ++k) em |= 1u << OT_MC_TRI_TABLE[c][k];
        cinfo[c] = em | ((unsigned)ntri[c] << 12);
    }
    OT_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_cinfo), cinfo, sizeof(cinfo)));
    for (int e = 0; e < 12; ++e)
        for (int a = 0; a < 4; ++a)
            if (kEdgeShift[e][a] != OT_MC_EDGE_SHIFT[e][a])
                return fail(OT_ERR_INVALID_ARGUMENT, "marching cubes: kEdgeShift differs from OT_MC_EDGE_SHIFT");
    g_tables_uploaded.store(true, std::memory_order_release);
    return OT_OK;
}

template <typename T>
static ot_status grow(T*& p, int64_t& cap, int64_t need) {
    if (cap >= need && p) return OT_OK;
    if (p) OT_HIP_TRY(hipFree(p));
    p = nullptr;
    const int64_t n = std::max<int64_t>(need + need / 4, 1024);
    OT_HIP_TRY(hipMalloc(&p, sizeof(T) * (size_t)n));
    cap = n;
    return OT_OK;
}

}  // namespace ot

using namespace ot;

extern "C" {

}  // extern "C"

namespace ot {
// Marching cubes, phase 1: classify, count and scan (one read-back for the vertex / triangle totals); the structure
// (cube bytes, bases, merge-key buffers) is kept with the volume.  Phase 2 (mc_emit) writes the mesh to any
// destination while the structure is valid.
// spec (nullable): launches work that needs the structure but not the totals (a speculative emission) between the
// count kernels and the totals' read-back, so the GPU runs it while the host waits
static ot_status mc_count(ot_tsdf* vol, hipStream_t stream, int64_t* n_vertices, int64_t* n_triangles,
                          const std::function<ot_status(McDev&)>& spec = nullptr) {
    ot_status st = upload_tables();
    if (st != OT_OK) return st;
    st = wait_normals(vol, stream);  // the last mesh's deferred normals still read the structure rewritten below
    if (st != OT_OK) return st;
    int64_t U = 0;
    st = tsdf_sorted_units(vol, stream, &U);
    if (st != OT_OK) return st;
    MeshBuffers& mb = vol->mesh;
    mb.nv = mb.nt = 0;
    mb.valid = false;
    mb.internal = false;
    mb.emitted = false;
    *n_vertices = *n_triangles = 0;
    if (U == 0) return OT_OK;
    // workspace (ids are dense in [0, U)), kept with the volume after the extraction (MeshBuffers::ws)
    const size_t bytes = mc_ws_bytes(U);
    if (mb.ws_bytes < bytes) {
        if (mb.ws) {
            OT_HIP_TRY(hipStreamSynchronize(stream));
            OT_HIP_TRY(hipFree(mb.ws));
            mb.ws = nullptr;
            mb.ws_bytes = 0;
        }
        const size_t nb = bytes + bytes / 4;
        OT_HIP_TRY(hipMalloc(&mb.ws, nb));
        mb.ws_bytes = nb;
        note_alloc();
    }
    McDev m;
    m.sorted_ids = vol->sorted_ids;
    m.vk = nullptr;
    m.tk = nullptr;
    mc_layout((char*)mb.ws, U, m);
    const unsigned g = (unsigned)U;
    hipLaunchKernelGGL(k_mc_prepare, dim3((g + PREP_UNITS - 1) / PREP_UNITS), dim3(256), 0, stream, vol->dev, m, (int)U);
    hipLaunchKernelGGL(k_mc_classify, dim3(g), dim3(256), 0, stream, vol->dev, m);
    hipLaunchKernelGGL(k_mc_count, dim3((g + CNT_UNITS - 1) / CNT_UNITS), dim3(64 * CNT_UNITS), 0, stream, m, (int)U);
    OT_LAUNCH_CHECK();
    if (U > 0x7FFFFFFF) return fail(OT_ERR_CAPACITY, "[ExtractTriangleMesh] too many units");
    // the scans mail the triangle and vertex totals (hmail words 0..3)
    const unsigned seq = ++vol->mc_seq;
    hipLaunchKernelGGL(k_mc_scan2, dim3(2), dim3(1024), 0, stream, (const long long*)m.tri_cnt, m.tri_base,
                       (const long long*)m.vert_cnt, m.vert_base, (int)U, (long long*)vol->hmail,
                       vol->hmail + MAIL_SEQ_MC, seq);
    OT_LAUNCH_CHECK();
    mb.ws_units = U;
    if (spec) {  // the host waits for the read-back only, the speculative work runs behind it
        st = spec(m);
        if (st != OT_OK) return st;
    }
    // the totals' sequence words, not an event: an event between the scans and the emission idles the GPU (tsdf.h)
    st = mail_wait(vol->hmail + MAIL_SEQ_MC, seq, stream);
    if (st == OT_OK) st = mail_wait(vol->hmail + MAIL_SEQ_MC + 1, seq, stream);
    if (st != OT_OK) return st;
    long long totals[2];
    std::memcpy(totals, vol->hmail, sizeof(totals));
    const int64_t nt = totals[0], nv = totals[1];
    if (nv > 0x7FFFFFFF) return fail(OT_ERR_CAPACITY, "[ExtractTriangleMesh] more than 2^31 vertices");
    // a speculative emission may still be writing the merge-key buffers that grow() below would free: wait for it
    // (the stream already waits on the side stream's ev_join) instead of relying on hipFree's implicit synchronisation
    if (spec && (nv > mb.cap_vk || nv > mb.cap_vown || nt * 3 > mb.cap_tk)) OT_HIP_TRY(hipStreamSynchronize(stream));
    st = grow(mb.vk, mb.cap_vk, nv);  // merge keys: 16 B per vertex, 12 B per triangle
    if (st != OT_OK) return st;
    st = grow(mb.vown, mb.cap_vown, nv);
    if (st != OT_OK) return st;
    st = grow(mb.tk, mb.cap_tk, nt * 3);
    if (st != OT_OK) return st;
    mb.nv = nv;
    mb.nt = nt;
    mb.serial += 1;
    mb.valid = true;
    *n_vertices = nv;
    *n_triangles = nt;
    return OT_OK;
}

// Phase 2: vertex positions / colours and triangle indices (and the merge keys) into the given device arrays.  They
// depend on the same edge bitmasks and bases but not on each other: the vertices run on the volume's side stream
// beside the triangles (fork / join by events); the mesh is complete in stream order on return.
static ot_status mc_emit_launch(ot_tsdf* vol, McDev m, int64_t nv, double* V, double* VC, int32_t* T,
                                hipStream_t stream);
static ot_status mc_emit(ot_tsdf* vol, double* V, double* VC, int32_t* T, hipStream_t stream) {
    MeshBuffers& mb = vol->mesh;
    if (mb.nv == 0 && mb.nt == 0) return OT_OK;
    McDev m;
    m.sorted_ids = vol->sorted_ids;
    mc_layout((char*)mb.ws, mb.ws_units, m);
    m.vk = mb.vk;
    m.vown = mb.vown;
    m.tk = mb.tk;
    ot_status st = mc_emit_launch(vol, m, mb.nv, V, VC, T, stream);
    if (st == OT_OK) mb.emitted = true;
    return st;
}
// the emission kernels of structure m (U = vol->mesh.ws_units) into V / VC / T (nv: vertex rows for the NoColor zeros)
static ot_status mc_emit_launch(ot_tsdf* vol, McDev m, int64_t nv, double* V, double* VC, int32_t* T,
                                hipStream_t stream) {
    const unsigned g = (unsigned)vol->mesh.ws_units;
    ot_status st = wait_normals(vol, stream);  // the emission rewrites vk / vown, which deferred normals read
    if (st != OT_OK) return st;
    if (g_mc_emit_fork && !vol->side) {
        OT_HIP_TRY(hipStreamCreateWithFlags(&vol->side, hipStreamNonBlocking));
        OT_HIP_TRY(hipEventCreateWithFlags(&vol->ev_fork, hipEventDisableTiming));
        OT_HIP_TRY(hipEventCreateWithFlags(&vol->ev_join, hipEventDisableTiming));
    }
    double* vc = vol->color_type == OT_COLOR_RGB8 ? VC : nullptr;
    if (g_mc_emit_fork) {
        OT_HIP_TRY(hipEventRecord(vol->ev_fork, stream));
        OT_HIP_TRY(hipStreamWaitEvent(vol->side, vol->ev_fork, 0));
        hipLaunchKernelGGL(k_mc_vertices, dim3(g), dim3(EWORDS), 0, vol->side, vol->dev, m, vol->voxel_length, V, vc);
        OT_HIP_TRY(hipEventRecord(vol->ev_join, vol->side));
        hipLaunchKernelGGL(k_mc_triangles, dim3(g), dim3(256), 0, stream, vol->dev, m, T);
        OT_HIP_TRY(hipStreamWaitEvent(stream, vol->ev_join, 0));
    } else {
        if (g > 0x3FFFFFFFu) return fail(OT_ERR_CAPACITY, "[ExtractTriangleMesh] too many units");
        hipLaunchKernelGGL(k_mc_emit, dim3(2 * g), dim3(EWORDS), 0, stream, vol->dev, m, (int)g, vol->voxel_length, V,
                           vc, T);
    }
    OT_LAUNCH_CHECK();
    if (VC && vol->color_type != OT_COLOR_RGB8)
        OT_HIP_TRY(hipMemsetAsync(VC, 0, sizeof(double) * 3 * (size_t)std::min<int64_t>(nv, m.cap_v), stream));
    return OT_OK;
}
}  // namespace ot

extern "C" {

ot_status ot_tsdf_extract_triangle_mesh(ot_tsdf* vol, int64_t* n_vertices, int64_t* n_triangles, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!vol || !n_vertices || !n_triangles) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    ot_status st = mc_count(vol, stream, n_vertices, n_triangles);
    if (st != OT_OK || *n_vertices + *n_triangles == 0) return st;
    MeshBuffers& mb = vol->mesh;
    int64_t capc = mb.cap_v;
    st = grow(mb.v, mb.cap_v, mb.nv * 3);
    if (st != OT_OK) return st;
    st = grow(mb.c, capc, mb.nv * 3);
    if (st != OT_OK) return st;
    st = grow(mb.t, mb.cap_t, mb.nt * 3);
    if (st != OT_OK) return st;
    st = mc_emit(vol, mb.v, vol->color_type == OT_COLOR_RGB8 ? mb.c : nullptr, mb.t, stream);
    if (st != OT_OK) return st;
    mb.internal = true;  // ot_tsdf_fetch_triangle_mesh copies from the volume's buffers
    return OT_OK;
}

ot_status ot_tsdf_extract_triangle_mesh_count(ot_tsdf* vol, int64_t* n_vertices, int64_t* n_triangles,
                                              void* stream_) {
    if (!vol || !n_vertices || !n_triangles) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    return mc_count(vol, S(stream_), n_vertices, n_triangles);
}

ot_status ot_tsdf_extract_triangle_mesh_into(ot_tsdf* vol, double* vertices, double* vertex_colors,
                                             int32_t* triangles, int64_t capacity_vertices, int64_t capacity_triangles,
                                             int64_t* n_vertices, int64_t* n_triangles, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!vol || !n_vertices || !n_triangles || capacity_vertices < 0 || capacity_triangles < 0 ||
        (capacity_vertices > 0 && !vertices) || (capacity_triangles > 0 && !triangles))
        return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    MeshBuffers& mb = vol->mesh;
    auto spec = [&](McDev& m) -> ot_status {  // the emission into the caller's arrays, before the totals are known
        ot_status gs = grow(mb.vk, mb.cap_vk, std::max<int64_t>(capacity_vertices, 1));
        if (gs != OT_OK) return gs;
        gs = grow(mb.vown, mb.cap_vown, std::max<int64_t>(capacity_vertices, 1));
        if (gs != OT_OK) return gs;
        gs = grow(mb.tk, mb.cap_tk, std::max<int64_t>(capacity_triangles, 1) * 3);
        if (gs != OT_OK) return gs;
        m.vk = mb.vk;
        m.vown = mb.vown;
        m.tk = mb.tk;
        m.cap_v = capacity_vertices;
        m.cap_t = capacity_triangles;
        return mc_emit_launch(vol, m, capacity_vertices, vertices, vertex_colors, triangles, stream);
    };
    ot_status st = mc_count(vol, stream, n_vertices, n_triangles, spec);
    if (st != OT_OK) return st;
    if (*n_vertices <= capacity_vertices && *n_triangles <= capacity_triangles) {
        mb.emitted = true;
        return OT_OK;
    }
    return fail(OT_ERR_CAPACITY, "[ExtractTriangleMesh] the mesh exceeds the given capacity: emit it with "
                                 "ot_tsdf_emit_triangle_mesh into arrays of *n_vertices / *n_triangles rows");
}

ot_status ot_tsdf_emit_triangle_mesh(ot_tsdf* vol, double* vertices, double* vertex_colors, int32_t* triangles,
                                     void* stream_) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    const MeshBuffers& mb = vol->mesh;
    if (mb.nv == 0 && mb.nt == 0) return OT_OK;  // an empty mesh (also before any extraction)
    if (!mb.valid)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ExtractTriangleMesh] the volume changed since the extraction");
    if ((mb.nv > 0 && !vertices) || (mb.nt > 0 && !triangles))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ExtractTriangleMesh] invalid arguments");
    return mc_emit(vol, vertices, vertex_colors, triangles, S(stream_));
}

ot_status ot_tsdf_mesh_serial(const ot_tsdf* vol, int64_t* serial_host) {
    if (!vol || !serial_host) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    *serial_host = vol->mesh.valid ? vol->mesh.serial : -1;
    return OT_OK;
}

ot_status ot_tsdf_mesh_vertex_normals(ot_tsdf* vol, int64_t serial, const double* vertices, int64_t n_vertices,
                                      const int32_t* triangles, int64_t n_triangles, double* out, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!vol || (n_vertices > 0 && (!vertices || !out)) || (n_triangles > 0 && !triangles))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ComputeVertexNormals] invalid arguments");
    const MeshBuffers& mb = vol->mesh;
    if (!mb.valid || !mb.emitted || serial != mb.serial || n_vertices != mb.nv || n_triangles != mb.nt)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ComputeVertexNormals] the volume changed since this mesh was extracted");
    if (n_vertices == 0) return OT_OK;
    McDev m;
    m.sorted_ids = vol->sorted_ids;
    mc_layout((char*)mb.ws, mb.ws_units, m);
    m.vk = mb.vk;
    m.vown = mb.vown;
    m.tk = mb.tk;
    hipLaunchKernelGGL(k_mc_vnormals, dim3((unsigned)((n_vertices + 255) / 256)), dim3(256), 0, stream, vol->dev, m,
                       mb.ws_units, vertices, triangles, n_vertices, out);
    OT_LAUNCH_CHECK();
    // the walk reads the structure on `stream` (often a side stream of the caller's): later work on the volume that
    // rewrites the structure or the units waits for this point first (wait_normals in mc_count, the emission,
    // integrate, reset, growth)
    if (!vol->ev_normals) OT_HIP_TRY(hipEventCreateWithFlags(&vol->ev_normals, hipEventDisableTiming));
    OT_HIP_TRY(hipEventRecord(vol->ev_normals, stream));
    vol->normals_pending = true;
    return OT_OK;
}

// reconstruct_rgbd_filter.py:112-132 of one volume in ONE host call: extract_triangle_mesh into the caller's arrays
// (capacities guessed, as ot_tsdf_extract_triangle_mesh_into), then -- with no host work between the marching-cubes
// totals and the sampler's first launch -- sample_points_uniformly(n_points, seed) + the z >= z_min mask (the fused
// sampler, points and colours), and compute_vertex_normals of the mesh on `normals_stream` beside the sampling (the
// sampling does not read them; a reader of `normals` waits for normals_stream).  On a capacity miss nothing is sampled
// and OT_ERR_CAPACITY returns the totals (emit with ot_tsdf_emit_triangle_mesh, then sample as usual).  An empty mesh
// samples nothing (*n_kept = 0; the reference skips it: reconstruct_rgbd_filter.py:115-117).
ot_status ot_tsdf_extract_sample_min_z(ot_tsdf* vol, double* vertices, double* vertex_colors, int32_t* triangles,
                                       int64_t capacity_vertices, int64_t capacity_triangles, double* vertex_normals,
                                       void* normals_stream, int64_t n_points, uint64_t seed, double z_min,
                                       double* out_xyz, double* out_rgb, int64_t* n_vertices, int64_t* n_triangles,
                                       int64_t* n_kept, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!vol || !n_kept || !out_xyz || n_points <= 0 || (out_rgb && !vertex_colors))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ExtractTriangleMesh] invalid arguments");
    *n_kept = 0;
    ot_status st = ot_tsdf_extract_triangle_mesh_into(vol, vertices, vertex_colors, triangles, capacity_vertices,
                                                      capacity_triangles, n_vertices, n_triangles, stream_);
    if (st != OT_OK) return st;
    const int64_t nv = *n_vertices, nt = *n_triangles;
    if (nv == 0 || nt == 0) return OT_OK;
    if (!vol->ev_made) OT_HIP_TRY(hipEventCreateWithFlags(&vol->ev_made, hipEventDisableTiming));
    // ev_made: the mesh arrays are complete (the normals wait on it).  Recorded where the normals cost the sampling
    // least: just before the area-sum walk, a single wave per chain with the rest of the GPU idle (g_normals_at 1).
    // Right after the emission the normals' launch landed among the chains' wide first passes and the stream stalled
    // 27 us twice (one object 1.571 vs 1.536 ms kernel span, r05m); beside the CDF walk (2) 1.592 vs 1.587 ms wall
    const int at = vertex_normals ? g_normals_at : 0;
    if (vertex_normals && at == 0) OT_HIP_TRY(hipEventRecord(vol->ev_made, stream));
    ot_mesh_sample_job job{vertices, nullptr, out_rgb ? vertex_colors : nullptr, nv, triangles, nt, out_xyz, nullptr,
                           out_rgb};
    hipStream_t hs = nullptr;
    st = sample_min_z_enqueue(&job, 1, n_points, seed, z_min, stream, &hs, at ? vol->ev_made : nullptr, at);
    if (st != OT_OK) return st;
    if (vertex_normals) {  // queued once the sampling is (its chains' first passes are dispatched ahead of them)
        hipStream_t ns = S(normals_stream);
        OT_HIP_TRY(hipStreamWaitEvent(ns, vol->ev_made, 0));
        st = ot_tsdf_mesh_vertex_normals(vol, vol->mesh.serial, vertices, nv, triangles, nt, vertex_normals, ns);
        if (st != OT_OK) {
            int64_t dummy = 0;
            (void)sample_min_z_wait(hs, 1, &dummy);
            return st;
        }
    }
    return sample_min_z_wait(hs, 1, n_kept);
}

ot_status ot_tsdf_fetch_triangle_mesh(ot_tsdf* vol, double* vertices, double* vertex_colors, int32_t* triangles,
                                      void* stream_) {
    hipStream_t stream = S(stream_);
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    const MeshBuffers& mb = vol->mesh;
    if (!mb.internal && (mb.nv > 0 || mb.nt > 0)) {  // counted and emitted elsewhere: emit again from the structure
        if (!mb.valid)
            return fail(OT_ERR_INVALID_ARGUMENT, "[ExtractTriangleMesh] the volume changed since the extraction");
        if ((mb.nv > 0 && !vertices) || (mb.nt > 0 && !triangles))
            return fail(OT_ERR_INVALID_ARGUMENT, "[ExtractTriangleMesh] invalid arguments");
        return mc_emit(vol, vertices, vertex_colors, triangles, stream);
    }
    if (mb.nv > 0 && vertices)
        OT_HIP_TRY(hipMemcpyAsync(vertices, mb.v, sizeof(double) * 3 * mb.nv, hipMemcpyDefault, stream));
    if (mb.nv > 0 && vertex_colors) {
        if (vol->color_type == OT_COLOR_RGB8)
            OT_HIP_TRY(hipMemcpyAsync(vertex_colors, mb.c, sizeof(double) * 3 * mb.nv, hipMemcpyDefault, stream));
        else
            OT_HIP_TRY(hipMemsetAsync(vertex_colors, 0, sizeof(double) * 3 * mb.nv, stream));
    }
    if (mb.nt > 0 && triangles)
        OT_HIP_TRY(hipMemcpyAsync(triangles, mb.t, sizeof(int32_t) * 3 * mb.nt, hipMemcpyDefault, stream));
    return OT_OK;
}

// test hook: where ot_tsdf_extract_sample_min_z lets the vertex normals start (0 / 1 / 2, g_normals_at)
ot_status otx_normals_at(int32_t at) {
    if (at < 0 || at > 2) return fail(OT_ERR_INVALID_ARGUMENT, "otx_normals_at: 0, 1 or 2");
    g_normals_at = at;
    return OT_OK;
}

// test hook: 1 = the emission as two kernels on two streams (fork / join by events), 0 = one launch (default)
ot_status otx_mc_emit_fork(int32_t on) {
    g_mc_emit_fork = on != 0;
    return OT_OK;
}

// merge keys of the extracted mesh: per vertex (owner unit x, y, z, edge bit = local voxel * 3 + axis), per
// triangle its cube's unit key (x, y, z).  Device pointers; either may be NULL.
ot_status ot_tsdf_fetch_mesh_keys(ot_tsdf* vol, int32_t* vertex_keys, int32_t* triangle_units, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    const MeshBuffers& mb = vol->mesh;
    if (!mb.emitted && (mb.nv > 0 || mb.nt > 0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ExtractTriangleMesh] the mesh of the last extraction was not emitted yet");
    if (mb.nv > 0 && vertex_keys)
        OT_HIP_TRY(hipMemcpyAsync(vertex_keys, mb.vk, sizeof(int4) * mb.nv, hipMemcpyDefault, stream));
    if (mb.nt > 0 && triangle_units)
        OT_HIP_TRY(hipMemcpyAsync(triangle_units, mb.tk, sizeof(int32_t) * 3 * mb.nt, hipMemcpyDefault, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

}  // extern "C"
