// sor_sim.cpp — CPU model of k_sor_knn's lockstep work (design tool, not product code).
// Loads a float64 [n][3] .npy cloud, builds the cell grid (cell h, x-major keys, points in cell order) and
// simulates waves of 64 consecutive sorted queries scanning their candidate ranges in lockstep: per range slot the
// wave runs max-lane-length steps, and a step executes the top-k insertion chain when ANY lane inserts.
// Reports candidates per query, per-lane insertions, and wave-level step / insertion-step counts.
//   g++ -O2 -std=c++17 -o /tmp/sor_sim tools/sor_sim.cpp && /tmp/sor_sim cloud.npy k h_mult [R [zorder [flat]]]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>
#include <vector>

static std::vector<double> load_npy(const char* path, size_t& n) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    char magic[10];
    fread(magic, 1, 10, f);
    unsigned short hl = (unsigned char)magic[8] | ((unsigned char)magic[9] << 8);
    std::vector<char> hdr(hl);
    fread(hdr.data(), 1, hl, f);
    fseek(f, 0, SEEK_END);
    long sz = ftell(f) - 10 - hl;
    fseek(f, 10 + hl, SEEK_SET);
    n = sz / 24;
    std::vector<double> v(n * 3);
    fread(v.data(), 8, n * 3, f);
    fclose(f);
    return v;
}

int main(int argc, char** argv) {
    size_t n;
    auto P = load_npy(argv[1], n);
    const int K = atoi(argv[2]);
    const double hm = atof(argv[3]);  // cell = hm * 5 mm
    const int R = argc > 4 ? atoi(argv[4]) : 1;  // stage-1 block radius in cells
    const int zorder = argc > 5 ? atoi(argv[5]) : 0;  // 1: own z-cell first inside a column
    const int flat = argc > 6 ? atoi(argv[6]) : 0;  // 1: the lane's slots as one flattened lockstep stream
    // > 1: candidates in per-lane batches of this many (one gather step each), each batch sorted (a B-input network),
    // then inserted in ascending order while ANY lane of the wave still accepts its next one (a sorted batch's
    // acceptances are a prefix per lane, so a wave's insertion steps per batch = its largest prefix)
    const int batch = argc > 7 ? atoi(argv[7]) : 0;
    // > 0: accepted candidates go to a per-lane queue of this many (tested against the k-th distance of the list as
    // of the last drain); the wave drains (inserts every lane's queue, one entry per insertion step, as many steps as
    // the longest queue) when any lane's queue is full, and at the end of the query.  Same final lists.
    const int queue = argc > 8 ? atoi(argv[8]) : 0;
    long long batch_steps = 0, batch_ins_steps = 0, drain_steps = 0, drains = 0, queued = 0;
    std::vector<std::vector<double>> Q(64);
    std::vector<std::pair<long long, std::vector<double>>> pend;  // stage-1 misses: sorted position, list
    std::vector<long long> pend_wave;
    std::vector<double> un_ratio;  // unsettled queries: k-th distance / guard
    std::vector<int> un_second;    // 1: the k-th sphere crosses only the nearest face, 2: two faces, 3: more
    const double h = hm * 0.005;
    double mn[3] = {1e30, 1e30, 1e30};
    for (size_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) mn[a] = std::min(mn[a], P[i * 3 + a]);
    auto cc = [&](size_t i, int a) { return (long long)std::floor((P[i * 3 + a] - mn[a]) / h); };
    auto key = [](long long x, long long y, long long z) { return (x << 42) | (y << 21) | z; };
    std::vector<std::pair<long long, size_t>> ord(n);
    for (size_t i = 0; i < n; ++i) ord[i] = {key(cc(i, 0), cc(i, 1), cc(i, 2)), i};
    std::stable_sort(ord.begin(), ord.end(), [](auto& a, auto& b) { return a.first < b.first; });
    std::unordered_map<long long, std::pair<int, int>> cells;
    for (size_t s = 0; s < n;) {
        size_t e = s;
        while (e < n && ord[e].first == ord[s].first) ++e;
        cells[ord[s].first] = {(int)s, (int)e};
        s = e;
    }
    std::vector<double> S(n * 3);
    for (size_t s = 0; s < n; ++s)
        for (int a = 0; a < 3; ++a) S[s * 3 + a] = P[ord[s].second * 3 + a];
    auto find = [&](long long x, long long y, long long z) -> std::pair<int, int> {
        if (x < 0 || y < 0 || z < 0) return {0, 0};
        auto it = cells.find(key(x, y, z));
        return it == cells.end() ? std::pair<int, int>{0, 0} : it->second;
    };
    // per query: list of ranges (slots), columns ordered by distance class; a column = cells z-R..z+R
    const int W = 2 * R + 1;
    std::vector<std::pair<int, int>> cols;  // (dx, dy) ordered: centre, faces, rest by squared distance
    for (int dx = -R; dx <= R; ++dx)
        for (int dy = -R; dy <= R; ++dy) cols.push_back({dx, dy});
    std::stable_sort(cols.begin(), cols.end(), [](auto a, auto b) {
        return a.first * a.first + a.second * a.second < b.first * b.first + b.second * b.second;
    });
    const int nslot = (int)cols.size() * (zorder ? W : 1);
    long long trans_steps = 0, stage2_steps = 0, tot_cand = 0, tot_ins = 0, wave_steps = 0, wave_ins_steps = 0, unsettled = 0;
    std::vector<std::vector<std::pair<int, int>>> plan(64, std::vector<std::pair<int, int>>(nslot));
    std::vector<std::vector<double>> best(64, std::vector<double>(K));
    std::vector<double> lo(64 * 2), hi(64 * 2), lz(64), hz(64);
    for (size_t w0 = 0; w0 < n; w0 += 64) {
        const int nl = (int)std::min<size_t>(64, n - w0);
        for (int l = 0; l < nl; ++l) {
            const size_t j = w0 + l;
            long long x = (long long)std::floor((S[j * 3] - mn[0]) / h), y = (long long)std::floor((S[j * 3 + 1] - mn[1]) / h),
                      z = (long long)std::floor((S[j * 3 + 2] - mn[2]) / h);
            int u = 0;
            for (auto [dx, dy] : cols) {
                if (!zorder) {
                    int b = 1 << 30, e = 0;
                    for (int dz = -R; dz <= R; ++dz) {
                        auto se = find(x + dx, y + dy, z + dz);
                        if (se.second > se.first) b = std::min(b, se.first), e = std::max(e, se.second);
                    }
                    plan[l][u++] = e > 0 ? std::pair<int, int>{b, e} : std::pair<int, int>{0, 0};
                } else {
                    plan[l][u++] = find(x + dx, y + dy, z);
                    for (int r = 1; r <= R; ++r) {
                        plan[l][u++] = find(x + dx, y + dy, z - r);
                        plan[l][u++] = find(x + dx, y + dy, z + r);
                    }
                }
            }
            for (int a = 0; a < 2; ++a) {
                const double uu = (S[j * 3 + a] - mn[a]) / h, fr = uu - std::floor(uu);
                lo[l * 2 + a] = fr * h, hi[l * 2 + a] = (1 - fr) * h;
            }
            {
                const double uu = (S[j * 3 + 2] - mn[2]) / h, fr = uu - std::floor(uu);
                lz[l] = fr * h, hz[l] = (1 - fr) * h;
            }
            std::fill(best[l].begin(), best[l].end(), INFINITY);
        }
        if (flat) {  // one flattened candidate stream per lane: column transitions inside the lockstep loop
            std::vector<int> uu(nl, 0), mm(nl, 0), ee(nl, 0);
            auto advance = [&](int l) {  // next non-culled slot of lane l (culled against its current k-th)
                while (mm[l] >= ee[l] && uu[l] < nslot) {
                    const int u = uu[l]++;
                    const int ci = zorder ? u / W : u;
                    const int dx = cols[ci].first, dy = cols[ci].second;
                    double ex = dx < 0 ? lo[l * 2] + (-dx - 1) * h : (dx > 0 ? hi[l * 2] + (dx - 1) * h : 0.0);
                    double ey = dy < 0 ? lo[l * 2 + 1] + (-dy - 1) * h : (dy > 0 ? hi[l * 2 + 1] + (dy - 1) * h : 0.0);
                    if (ex * ex + ey * ey < best[l][K - 1]) mm[l] = plan[l][u].first, ee[l] = plan[l][u].second;
                }
            };
            for (;;) {
                bool live = false, any = false, trans = false;
                for (int l = 0; l < nl; ++l) {
                    if (mm[l] >= ee[l]) { advance(l); trans = true; }
                    if (mm[l] >= ee[l]) continue;
                    live = true;
                    const size_t j = w0 + l, m = mm[l]++;
                    const double d0 = S[j * 3] - S[m * 3], d1 = S[j * 3 + 1] - S[m * 3 + 1], d2 = S[j * 3 + 2] - S[m * 3 + 2];
                    const double d = (d0 * d0 + d1 * d1) + d2 * d2;
                    ++tot_cand;
                    if (d < best[l][K - 1]) {
                        any = true;
                        ++tot_ins;
                        auto& bb = best[l];
                        bb[K - 1] = d;
                        for (int i = K - 1; i > 0 && bb[i] < bb[i - 1]; --i) std::swap(bb[i], bb[i - 1]);
                    }
                }
                if (!live) break;
                ++wave_steps;
                wave_ins_steps += any;
                trans_steps += trans;
            }
        }
        for (int u = 0; u < nslot && !flat; ++u) {
            const int ci = zorder ? u / W : u;
            const int dx = cols[ci].first, dy = cols[ci].second;
            int maxlen = 0;
            std::vector<char> act(nl);
            for (int l = 0; l < nl; ++l) {
                // column cull (distance to the column's near face vs the current k-th distance)
                double ex = dx < 0 ? lo[l * 2] + (-dx - 1) * h : (dx > 0 ? hi[l * 2] + (dx - 1) * h : 0.0);
                double ey = dy < 0 ? lo[l * 2 + 1] + (-dy - 1) * h : (dy > 0 ? hi[l * 2 + 1] + (dy - 1) * h : 0.0);
                double ez = 0.0;
                if (zorder) {
                    const int dz = (u % W) == 0 ? 0 : (((u % W) - 1) % 2 == 0 ? -((u % W) + 1) / 2 : ((u % W) + 1) / 2);
                    ez = dz < 0 ? lz[l] + (-dz - 1) * h : (dz > 0 ? hz[l] + (dz - 1) * h : 0.0);
                }
                act[l] = ex * ex + ey * ey + ez * ez < best[l][K - 1];
                if (act[l]) maxlen = std::max(maxlen, plan[l][u].second - plan[l][u].first);
            }
            if (batch > 1) {
                for (int s0 = 0; s0 < maxlen; s0 += batch) {
                    int wave_ins = 0;
                    for (int l = 0; l < nl; ++l) {
                        if (!act[l]) continue;
                        const int len = plan[l][u].second - plan[l][u].first;
                        std::vector<double> bd;
                        for (int s = s0; s < s0 + batch && s < len; ++s) {
                            const size_t j = w0 + l, m = plan[l][u].first + s;
                            const double d0 = S[j * 3] - S[m * 3], d1 = S[j * 3 + 1] - S[m * 3 + 1],
                                         d2 = S[j * 3 + 2] - S[m * 3 + 2];
                            bd.push_back((d0 * d0 + d1 * d1) + d2 * d2);
                            ++tot_cand;
                        }
                        std::sort(bd.begin(), bd.end());
                        int acc = 0;
                        for (double d : bd) {
                            if (!(d < best[l][K - 1])) break;
                            ++acc;
                            ++tot_ins;
                            auto& b = best[l];
                            b[K - 1] = d;
                            for (int i = K - 1; i > 0 && b[i] < b[i - 1]; --i) std::swap(b[i], b[i - 1]);
                        }
                        wave_ins = std::max(wave_ins, acc);
                    }
                    ++batch_steps;
                    batch_ins_steps += wave_ins;
                }
                continue;
            }
            if (queue > 0) {
                auto drain = [&]() {
                    size_t mx = 0;
                    for (int l = 0; l < nl; ++l) {
                        mx = std::max(mx, Q[l].size());
                        for (double d : Q[l]) {
                            auto& b = best[l];
                            if (!(d < b[K - 1])) continue;
                            ++tot_ins;
                            b[K - 1] = d;
                            for (int i = K - 1; i > 0 && b[i] < b[i - 1]; --i) std::swap(b[i], b[i - 1]);
                        }
                        Q[l].clear();
                    }
                    drain_steps += mx;
                    drains += mx > 0;
                };
                for (int s = 0; s < maxlen; ++s) {
                    bool full = false;
                    for (int l = 0; l < nl; ++l) {
                        if (!act[l] || s >= plan[l][u].second - plan[l][u].first) continue;
                        const size_t j = w0 + l, m = plan[l][u].first + s;
                        const double d0 = S[j * 3] - S[m * 3], d1 = S[j * 3 + 1] - S[m * 3 + 1],
                                     d2 = S[j * 3 + 2] - S[m * 3 + 2];
                        const double d = (d0 * d0 + d1 * d1) + d2 * d2;
                        ++tot_cand;
                        if (d < best[l][K - 1]) {
                            Q[l].push_back(d);
                            ++queued;
                            full |= (int)Q[l].size() >= queue;
                        }
                    }
                    ++wave_steps;
                    if (full) drain();
                }
                if (u == nslot - 1) drain();
                continue;
            }
            for (int s = 0; s < maxlen; ++s) {
                bool any = false;
                for (int l = 0; l < nl; ++l) {
                    if (!act[l] || s >= plan[l][u].second - plan[l][u].first) continue;
                    const size_t j = w0 + l, m = plan[l][u].first + s;
                    const double d0 = S[j * 3] - S[m * 3], d1 = S[j * 3 + 1] - S[m * 3 + 1], d2 = S[j * 3 + 2] - S[m * 3 + 2];
                    const double d = (d0 * d0 + d1 * d1) + d2 * d2;
                    ++tot_cand;
                    if (d < best[l][K - 1]) {
                        any = true;
                        ++tot_ins;
                        auto& b = best[l];
                        b[K - 1] = d;
                        for (int i = K - 1; i > 0 && b[i] < b[i - 1]; --i) std::swap(b[i], b[i - 1]);
                    }
                }
                ++wave_steps;
                wave_ins_steps += any;
            }
        }
        long long wmax2 = 0;
        for (int l = 0; l < nl; ++l) {
            // settled if k-th <= distance to the block faces
            const size_t j = w0 + l;
            double g = 1e30;
            for (int a = 0; a < 3; ++a) {
                const double uu = (S[j * 3 + a] - mn[a]) / h, fr = uu - std::floor(uu);
                g = std::min(g, std::min(R + fr, R + 1 - fr) * h);
            }
            const bool un = !(best[l][K - 1] <= g * g);
            unsettled += un;
            if (un) {  // how far past the guard: k-th distance / guard, and the second-nearest face's guard
                double gs[6];
                int q = 0;
                for (int a = 0; a < 3; ++a) {
                    const double uu = (S[j * 3 + a] - mn[a]) / h, fr = uu - std::floor(uu);
                    gs[q++] = (R + fr) * h;
                    gs[q++] = (R + 1 - fr) * h;
                }
                std::sort(gs, gs + 6);
                const double kd = best[l][K - 1] < 1e30 ? std::sqrt(best[l][K - 1]) : 1e30;
                un_ratio.push_back(kd / g);
                un_second.push_back(kd <= gs[1] ? 1 : (kd <= gs[2] ? 2 : 3));
            }
            if (un) pend.push_back({(long long)j, best[l]}), pend_wave.push_back((long long)(w0 / 64));
            if (un) {
                long long x = (long long)std::floor((S[j * 3] - mn[0]) / h), y = (long long)std::floor((S[j * 3 + 1] - mn[1]) / h),
                          z = (long long)std::floor((S[j * 3 + 2] - mn[2]) / h);
                long long c = 0;
                const int R2 = R + 1;
                for (int dx = -R2; dx <= R2; ++dx)
                    for (int dy = -R2; dy <= R2; ++dy)
                        for (int dz = -R2; dz <= R2; ++dz) {
                            if (std::max(std::abs(dx), std::max(std::abs(dy), std::abs(dz))) != R2) continue;
                            auto se = find(x + dx, y + dy, z + dz);
                            c += se.second - se.first;
                        }
                wmax2 = std::max(wmax2, c);
            }
        }
        stage2_steps += wmax2;
    }
    const double nq = (double)n, nw = std::ceil(nq / 64);
    printf("n %zu h %.4f R %d zorder %d cells %zu (%.1f pts/cell): cand/query %.1f ins/query %.1f | per wave: steps %.1f "
           "ins-steps %.1f (%.0f%%) | unsettled %.2f%% | VALU model (12/step + 42/ins-step) per query %.1f\n",
           n, h, R, zorder, cells.size(), nq / cells.size(), tot_cand / nq, tot_ins / nq, wave_steps / nw,
           wave_ins_steps / nw, 100.0 * wave_ins_steps / std::max<long long>(wave_steps, 1), 100.0 * unsettled / nq,
           (12.0 * wave_steps + 42.0 * wave_ins_steps) / nq);
    printf("   flat %d: wave steps with a column transition %.1f\n", flat, trans_steps / nw);
    if (batch > 1) {
        const int ce = batch == 2 ? 1 : batch == 4 ? 5 : batch == 8 ? 19 : batch == 16 ? 60 : batch * batch / 2;
        printf("   batch %d: per wave %.1f batch steps, %.1f insertion steps (%.2f per batch) | VALU model "
               "(12/cand-slot x %d + %d/sort + 42/ins-step) per query %.1f\n", batch, batch_steps / nw,
               batch_ins_steps / nw, (double)batch_ins_steps / std::max<long long>(batch_steps, 1), batch, 2 * ce,
               ((12.0 * batch + 2.0 * ce) * batch_steps + 42.0 * batch_ins_steps) / nq);
    }
    if (queue > 0)
        printf("   queue %d: per wave %.1f steps, %.1f drains, %.1f drain insertion steps; queued/query %.1f (exact "
               "insertions %.1f) | VALU model (16/step + 42/drain step) per query %.1f\n", queue, wave_steps / nw,
               drains / nw, drain_steps / nw, queued / nq, tot_ins / nq, (16.0 * wave_steps + 42.0 * drain_steps) / nq);
    // Stage 2 (the 5x5x5 shell) in lockstep waves of 64 pending queries, in two list orders: "xcd" = the order stage 1's
    // atomics give (8 XCDs each walking a contiguous eighth of the waves, their waves' misses interleaved round-robin),
    // "sorted" = sorted query order (neighbouring misses share a wave)
    if (R == 1 && !pend.empty()) {
        const long long nwv = (long long)std::ceil(nq / 64);
        std::vector<std::vector<size_t>> per_x(8);
        for (size_t i = 0; i < pend.size(); ++i) per_x[std::min<long long>(7, pend_wave[i] * 8 / nwv)].push_back(i);
        std::vector<size_t> xorder;
        {
            std::vector<size_t> at(8, 0);
            bool more = true;
            while (more) {
                more = false;
                for (int x = 0; x < 8; ++x) {  // one stage-1 wave's misses from each XCD in turn
                    if (at[x] >= per_x[x].size()) continue;
                    more = true;
                    const long long w = pend_wave[per_x[x][at[x]]];
                    while (at[x] < per_x[x].size() && pend_wave[per_x[x][at[x]]] == w) xorder.push_back(per_x[x][at[x]++]);
                }
            }
        }
        std::vector<size_t> sorder(pend.size());
        for (size_t i = 0; i < pend.size(); ++i) sorder[i] = i;
        static const int cols5[25] = {12, 7, 11, 13, 17, 6, 8, 16, 18, 2, 10, 14, 22, 1, 3, 5, 9, 15, 19, 21, 23, 0, 4, 20, 24};
        for (int mode = 0; mode < 2; ++mode) {
            const auto& ord2 = mode == 0 ? xorder : sorder;
            long long st = 0, ins_st = 0, cand = 0, probes = 0;
            std::set<long long> lines_w;  // distinct 64-B lines of candidates read per wave (L1-sharing proxy)
            long long lines = 0;
            for (size_t w0 = 0; w0 < ord2.size(); w0 += 64) {
                const int nl = (int)std::min<size_t>(64, ord2.size() - w0);
                std::vector<std::vector<double>> bl(nl);
                std::vector<long long> qx(nl), qy(nl), qz(nl);
                std::vector<double> flo(nl * 3), fhi(nl * 3);
                lines_w.clear();
                for (int l = 0; l < nl; ++l) {
                    const auto& pe = pend[ord2[w0 + l]];
                    bl[l] = pe.second;
                    const size_t j = (size_t)pe.first;
                    long long c3[3];
                    for (int a = 0; a < 3; ++a) {
                        const double uu = (S[j * 3 + a] - mn[a]) / h;
                        c3[a] = (long long)std::floor(uu);
                        const double fr = uu - std::floor(uu);
                        flo[l * 3 + a] = fr * h, fhi[l * 3 + a] = (1 - fr) * h;
                    }
                    qx[l] = c3[0], qy[l] = c3[1], qz[l] = c3[2];
                }
                for (int u = 0; u < 25; ++u) {
                    const int t = cols5[u], dx = t / 5 - 2, dy = t % 5 - 2;
                    const bool inner = std::abs(dx) <= 1 && std::abs(dy) <= 1;
                    for (int part = 0; part < (inner ? 2 : 1); ++part) {
                        std::vector<std::pair<int, int>> rg(nl, {0, 0});
                        int mx = 0;
                        for (int l = 0; l < nl; ++l) {
                            const double ex = dx < 0 ? flo[l * 3] + (-dx - 1) * h : (dx > 0 ? fhi[l * 3] + (dx - 1) * h : 0.0);
                            const double ey = dy < 0 ? flo[l * 3 + 1] + (-dy - 1) * h : (dy > 0 ? fhi[l * 3 + 1] + (dy - 1) * h : 0.0);
                            double e2 = ex * ex + ey * ey;
                            if (inner) {
                                const double ez = part == 0 ? flo[l * 3 + 2] + h : fhi[l * 3 + 2] + h;
                                e2 += ez * ez;
                            }
                            if (e2 >= bl[l][K - 1]) continue;
                            ++probes;
                            int b = 1 << 30, e = 0;
                            const int z0 = inner ? (part == 0 ? -2 : 2) : -2, z1 = inner ? z0 : 2;
                            for (int dz = z0; dz <= z1; ++dz) {
                                auto se = find(qx[l] + dx, qy[l] + dy, qz[l] + dz);
                                if (se.second > se.first) b = std::min(b, se.first), e = std::max(e, se.second);
                            }
                            if (e > 0) rg[l] = {b, e}, mx = std::max(mx, e - b);
                        }
                        for (int s2 = 0; s2 < mx; ++s2) {
                            bool any = false;
                            for (int l = 0; l < nl; ++l) {
                                if (s2 >= rg[l].second - rg[l].first) continue;
                                const size_t j = (size_t)pend[ord2[w0 + l]].first, m = rg[l].first + s2;
                                lines_w.insert((long long)(m * 24 / 64));
                                const double d0 = S[j * 3] - S[m * 3], d1 = S[j * 3 + 1] - S[m * 3 + 1], d2 = S[j * 3 + 2] - S[m * 3 + 2];
                                const double d = (d0 * d0 + d1 * d1) + d2 * d2;
                                ++cand;
                                auto& bb = bl[l];
                                if (d < bb[K - 1]) {
                                    any = true;
                                    bb[K - 1] = d;
                                    for (int i = K - 1; i > 0 && bb[i] < bb[i - 1]; --i) std::swap(bb[i], bb[i - 1]);
                                }
                            }
                            ++st;
                            ins_st += any;
                        }
                    }
                }
                lines += (long long)lines_w.size();
            }
            const double np2 = (double)pend.size(), nw2 = std::ceil(np2 / 64);
            printf("   stage 2 %-6s: %zu pending, per wave %.1f steps, %.1f ins-steps, cand/query %.1f, distinct 64-B lines "
                   "per wave %.0f, column parts probed per query %.1f | VALU model per pending query %.1f\n",
                   mode == 0 ? "xcd" : "sorted", pend.size(), st / nw2, ins_st / nw2, cand / np2, lines / nw2,
                   probes / np2, (12.0 * st + 42.0 * ins_st) / np2);
        }
    }
    if (!un_ratio.empty()) {
        std::vector<double> r = un_ratio;
        std::sort(r.begin(), r.end());
        long long c1 = 0, c2 = 0;
        for (int v : un_second) c1 += v == 1, c2 += v == 2;
        printf("   unsettled: k-th / guard median %.3f p25 %.3f p75 %.3f p90 %.3f; sphere past one face only %.1f%%, two "
               "faces %.1f%%\n", r[r.size() / 2], r[r.size() / 4], r[r.size() * 3 / 4], r[r.size() * 9 / 10],
               100.0 * c1 / r.size(), 100.0 * c2 / r.size());
    }
    printf("   stage-2 wave steps per wave %.1f -> model incl. stage 2 (54/step) per query %.1f\n", stage2_steps / nw,
           (12.0 * wave_steps + 42.0 * wave_ins_steps + 54.0 * stage2_steps) / nq);
}
