// vsor_sim.cpp — CPU model of a voxel-column SOR candidate search (design tool, measured slower on the GPU: DESIGN.md §4).
//   g++ -O2 -std=c++17 -o /tmp/vsor_sim tools/vsor_sim.cpp && /tmp/vsor_sim voxel_cloud.npy k C [CZ]
// voxel-column SOR model: queries in voxel-key order, candidates = occupied voxels of columns (kx+dx, ky+dy),
// kz-C..kz+C; lockstep waves of 64.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>
#include <vector>
#include <map>
static std::vector<double> load_npy(const char* path, size_t& n) {
    FILE* f = fopen(path, "rb"); char magic[10]; if(fread(magic, 1, 10, f)){}
    unsigned short hl = (unsigned char)magic[8] | ((unsigned char)magic[9] << 8);
    std::vector<char> hdr(hl); if(fread(hdr.data(), 1, hl, f)){}
    fseek(f, 0, SEEK_END); long sz = ftell(f) - 10 - hl; fseek(f, 10 + hl, SEEK_SET);
    n = sz / 24; std::vector<double> v(n * 3); if(fread(v.data(), 8, n * 3, f)){} fclose(f); return v;
}
int main(int argc, char** argv) {
    size_t n; auto P = load_npy(argv[1], n);
    const int K = atoi(argv[2]); const int C = atoi(argv[3]); const int CZ = argc > 4 ? atoi(argv[4]) : C;
    const double vs = 0.005;
    double mn[3] = {1e30, 1e30, 1e30};
    for (size_t i = 0; i < n; ++i) for (int a = 0; a < 3; ++a) mn[a] = std::min(mn[a], P[i * 3 + a]);
    for (int a = 0; a < 3; ++a) mn[a] -= vs * 0.5;  // a voxel origin as voxel_down_sample's
    auto vc = [&](size_t i, int a) { return (long long)std::floor((P[i * 3 + a] - mn[a]) / vs); };
    auto key = [](long long x, long long y, long long z) { return (x << 42) | (y << 21) | z; };
    std::vector<std::pair<long long, size_t>> ord(n);
    for (size_t i = 0; i < n; ++i) ord[i] = {key(vc(i, 0), vc(i, 1), vc(i, 2)), i};
    std::sort(ord.begin(), ord.end());
    std::vector<double> S(n * 3); std::vector<long long> KZ(n), KX(n), KY(n);
    for (size_t s = 0; s < n; ++s) { for (int a = 0; a < 3; ++a) S[s*3+a] = P[ord[s].second*3+a];
        KX[s] = ord[s].first >> 42; KY[s] = (ord[s].first >> 21) & 0x1FFFFF; KZ[s] = ord[s].first & 0x1FFFFF; }
    std::unordered_map<long long, std::pair<int,int>> colmap;  // (x,y) -> [start,end) in sorted order
    for (size_t s = 0; s < n;) { size_t e = s; long long c = ord[s].first >> 21; while (e < n && (ord[e].first >> 21) == c) ++e; colmap[c] = {(int)s,(int)e}; s = e; }
    long long collen = 0; for (auto& kv : colmap) collen += kv.second.second - kv.second.first;
    std::vector<std::pair<int,int>> cols;
    for (int dx = -C; dx <= C; ++dx) for (int dy = -C; dy <= C; ++dy) cols.push_back({dx, dy});
    std::stable_sort(cols.begin(), cols.end(), [](auto a, auto b){ return a.first*a.first+a.second*a.second < b.first*b.first+b.second*b.second; });
    long long longcols=0, tot_cand=0, tot_ins=0, wave_steps=0, wave_ins=0, unset=0, probes=0, searchsteps=0, colslots=0;
    std::vector<std::vector<double>> best(64, std::vector<double>(K));
    for (size_t w0 = 0; w0 < n; w0 += 64) {
        int nl = (int)std::min<size_t>(64, n - w0);
        for (int l = 0; l < nl; ++l) std::fill(best[l].begin(), best[l].end(), INFINITY);
        for (auto [dx, dy] : cols) {
            std::vector<std::pair<int,int>> rg(nl); int maxlen = 0; bool anyact = false;
            for (int l = 0; l < nl; ++l) {
                size_t j = w0 + l;
                double lo0 = S[j*3] - (mn[0] + KX[j]*vs), hi0 = vs - lo0, lo1 = S[j*3+1] - (mn[1] + KY[j]*vs), hi1 = vs - lo1;
                double ex = dx < 0 ? lo0 + (-dx-1)*vs : (dx > 0 ? hi0 + (dx-1)*vs : 0), ey = dy < 0 ? lo1 + (-dy-1)*vs : (dy > 0 ? hi1 + (dy-1)*vs : 0);
                rg[l] = {0,0};
                if (!(ex*ex+ey*ey < best[l][K-1])) continue;
                anyact = true; ++probes;
                auto it = colmap.find(key(KX[j]+dx, KY[j]+dy, 0) >> 21);
                if (it == colmap.end()) continue;
                int b = it->second.first, e = it->second.second;
                // z window via binary search
                int L, R_; if (e - b <= 8) { L = b; R_ = e; } else { ++longcols; L = (int)(std::lower_bound(KZ.begin()+b, KZ.begin()+e, KZ[j]-CZ) - KZ.begin());
                R_ = (int)(std::upper_bound(KZ.begin()+b, KZ.begin()+e, KZ[j]+CZ) - KZ.begin());
                searchsteps += 2 * (long long)std::ceil(std::log2(e - b + 1)); }
                rg[l] = {L, R_}; maxlen = std::max(maxlen, R_ - L);
            }
            if (anyact) ++colslots;
            for (int s = 0; s < maxlen; ++s) {
                bool any = false;
                for (int l = 0; l < nl; ++l) {
                    if (s >= rg[l].second - rg[l].first) continue;
                    size_t j = w0 + l, m = rg[l].first + s;
                    double d0 = S[j*3]-S[m*3], d1 = S[j*3+1]-S[m*3+1], d2 = S[j*3+2]-S[m*3+2];
                    double d = (d0*d0+d1*d1)+d2*d2; ++tot_cand;
                    if (d < best[l][K-1]) { any = true; ++tot_ins; auto& bb = best[l]; bb[K-1] = d;
                        for (int i = K-1; i > 0 && bb[i] < bb[i-1]; --i) std::swap(bb[i], bb[i-1]); }
                }
                ++wave_steps; wave_ins += any;
            }
        }
        for (int l = 0; l < nl; ++l) {
            size_t j = w0 + l; double g = 1e30;
            for (int a = 0; a < 3; ++a) { long long k = a==0?KX[j]:(a==1?KY[j]:KZ[j]); int CC = a==2?CZ:C;
                double lo = S[j*3+a] - (mn[a] + k*vs); g = std::min(g, std::min(CC*vs + lo, CC*vs + vs - lo)); }
            unset += !(best[l][K-1] <= g*g);
        }
    }
    double nq = n, nw = std::ceil(nq/64);
    printf("longcols/query %.2f\n", longcols/(double)n); printf("n %zu C %d CZ %d cols %zu (mean len %.2f): cand/query %.1f ins/query %.1f | per wave: steps %.1f ins-steps %.1f (%.0f%%) colslots %.1f | probes/query %.1f search/query %.1f | unsettled %.2f%% | model (12/step+42/ins) per query %.1f\n",
        n, C, CZ, colmap.size(), (double)collen/colmap.size(), tot_cand/nq, tot_ins/nq, wave_steps/nw, wave_ins/nw, 100.0*wave_ins/std::max(1LL,wave_steps), colslots/nw, probes/nq, searchsteps/nq, 100.0*unset/nq, (12.0*wave_steps+42.0*wave_ins)/nq);
}
