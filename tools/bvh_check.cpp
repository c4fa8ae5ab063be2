// bvh_check.cpp -- development tool: builds the BVH8 of a dumped scene (tools/bvh_check.py)
// with the product builder (csrc/bvh8.cpp), traverses the dumped rays on the CPU through the
// quantised nodes (children front to back by entry distance), and reports node visits and
// triangle tests per ray, the build time and the BVH8 depth; a sample of the rays is checked
// against brute force.  usage: bvh_check <scene.bin> [greedy]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bvh8.h"

using namespace mpt;

static bool mt(const TriRec& t, const float* o, const float* d, float& tt) {
    float e1[3] = {t.e1x, t.e1y, t.e1z}, e2[3] = {t.e2x, t.e2y, t.e2z};
    float h[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    float a = e1[0] * h[0] + e1[1] * h[1] + e1[2] * h[2];
    if (a > -1e-7f && a < 1e-7f) return false;
    float f = 1.0f / a;
    float s[3] = {o[0] - t.ax, o[1] - t.ay, o[2] - t.az};
    float u = f * (s[0] * h[0] + s[1] * h[1] + s[2] * h[2]);
    if (u < 0.0f || u > 1.0f) return false;
    float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    float v = f * (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]);
    if (v < 0.0f || u + v > 1.0f) return false;
    tt = f * (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]);
    return tt > 1e-7f;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    if (argc > 2) setenv("MPT_BVH_COLLAPSE", argv[2], 1);
    FILE* f = fopen(argv[1], "rb");
    int nv, nt, nr;
    if (fread(&nv, 4, 1, f) != 1 || fread(&nt, 4, 1, f) != 1 || fread(&nr, 4, 1, f) != 1) return 3;
    std::vector<float> V(3 * (size_t)nv), R(8 * (size_t)nr);
    std::vector<int32_t> I(3 * (size_t)nt);
    if (fread(V.data(), 4, V.size(), f) != V.size() || fread(I.data(), 4, I.size(), f) != I.size() ||
        fread(R.data(), 4, R.size(), f) != R.size()) return 3;
    fclose(f);
    BVH8 b;
    auto t0 = std::chrono::steady_clock::now();
    build_bvh8(V.data(), I.data(), nt, b, 3);
    double bt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double nodes = 0, tris = 0;
    int bad = 0, checked = 0;
    for (int r = 0; r < nr; r++) {
        const float* o = &R[8 * (size_t)r];
        const float* d = o + 4;
        float inv[3];
        for (int a = 0; a < 3; a++) inv[a] = 1.0f / (std::fabs(d[a]) > 1e-30f ? d[a] : std::copysign(1e-30f, d[a]));
        float best = INFINITY;
        int bprim = -1;
        std::vector<std::pair<float, int>> stk{{0.0f, 0}};
        while (!stk.empty()) {
            auto [tn0, ni] = stk.back();
            stk.pop_back();
            if (tn0 > best) continue;
            nodes++;
            const Node8& n = b.nodes[ni];
            float sc[3] = {std::ldexp(1.0f, n.ex - 127), std::ldexp(1.0f, n.ey - 127), std::ldexp(1.0f, n.ez - 127)};
            float org[3] = {n.px, n.py, n.pz};
            const uint8_t* ql[3] = {n.qlox, n.qloy, n.qloz};
            const uint8_t* qh[3] = {n.qhix, n.qhiy, n.qhiz};
            std::vector<std::pair<float, int>> hits;
            for (int s = 0; s < 8; s++) {
                if (!((n.imask >> s) & 1) && n.meta[s] == 0) continue;
                float tn = 0.0f, tf = best;
                for (int a = 0; a < 3; a++) {
                    float lo = org[a] + ql[a][s] * sc[a], hi = org[a] + qh[a][s] * sc[a];
                    float t1 = (lo - o[a]) * inv[a], t2 = (hi - o[a]) * inv[a];
                    tn = std::max(tn, std::min(t1, t2));
                    tf = std::min(tf, std::max(t1, t2));
                }
                if (tn > tf * 1.0000009f) continue;
                hits.push_back({tn, s});
            }
            std::sort(hits.begin(), hits.end());
            // leaves first (front to back), then internal children pushed back to front
            for (auto& h : hits) {
                int s = h.second;
                if ((n.imask >> s) & 1) continue;
                int cnt = n.meta[s] >> 5, off = n.meta[s] & 31;
                for (int k = 0; k < cnt; k++) {
                    tris++;
                    const TriRec& tr = b.tris[n.tri_base + off + k];
                    float tt;
                    int prim;
                    std::memcpy(&prim, &tr.prim_bits, 4);
                    if (mt(tr, o, d, tt) && (tt < best || (tt == best && prim < bprim))) { best = tt; bprim = prim; }
                }
            }
            for (int k = (int)hits.size() - 1; k >= 0; k--) {
                int s = hits[k].second;
                if (!((n.imask >> s) & 1)) continue;
                int rank = __builtin_popcount(n.imask & ((1u << s) - 1u));
                stk.push_back({hits[k].first, (int)n.child_base + rank});
            }
        }
        if (r % 997 == 0) {   // brute force check
            checked++;
            float bb = INFINITY;
            int bp = -1;
            for (size_t t = 0; t < b.tris.size(); t++) {
                float tt;
                int prim;
                std::memcpy(&prim, &b.tris[t].prim_bits, 4);
                if (mt(b.tris[t], o, d, tt) && (tt < bb || (tt == bb && prim < bp))) { bb = tt; bp = prim; }
            }
            if (bp != bprim) bad++;
        }
    }
    printf("{\"mode\": \"%s\", \"build_s\": %.2f, \"nodes\": %zu, \"tris\": %zu, \"depth\": %d, \"nodes_per_ray\": %.3f, "
           "\"tris_per_ray\": %.3f, \"brute_force_checked\": %d, \"mismatch\": %d}\n",
           argc > 2 ? argv[2] : "default", bt, b.nodes.size(), b.tris.size(), b.depth, nodes / nr, tris / nr, checked, bad);
    return bad ? 1 : 0;
}
