// bvh8.cpp -- host BVH8 builder: binned-SAH BVH2, collapsed to 8-wide nodes, octant-ordered
// child slots (so that a ray visits slot k ^ (octant ^ 7) first, front to back),
// conservative 8-bit quantisation of child boxes.  See bvh8.h for the node format.
// Collapse: greedy (expand the child with the largest surface area, BVH2 leaves of
// max_leaf triangles), or with MPT_BVH_COLLAPSE=cost a surface-area cost minimisation over
// the whole BVH2 built down to single triangles (the dynamic programme of compressed wide
// BVH builders: each subtree takes the cheapest way to stand as 1..8 child slots -- one leaf
// of up to max_leaf triangles, one internal node, or its two children's slots).  Measured on
// the C3 city (tools/bvh_check.py, 100 k camera + bounce rays): greedy 7.37 nodes / 2.33
// triangles per ray, cost 7.57 / 2.43 (triangle / node cost 0.1 - 1.0: no better), so greedy
// stays the default; 64 / 128 SAH bins instead of 32 gain < 1 %.
#include "bvh8.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace mpt {
namespace {

struct AABB {
    float lo[3], hi[3];
    AABB() { for (int i = 0; i < 3; i++) { lo[i] = FLT_MAX; hi[i] = -FLT_MAX; } }
    void grow(const AABB& b) { for (int i = 0; i < 3; i++) { lo[i] = std::min(lo[i], b.lo[i]); hi[i] = std::max(hi[i], b.hi[i]); } }
    void grow(const float* p) { for (int i = 0; i < 3; i++) { lo[i] = std::min(lo[i], p[i]); hi[i] = std::max(hi[i], p[i]); } }
    float area() const {
        float d0 = std::max(0.0f, hi[0] - lo[0]), d1 = std::max(0.0f, hi[1] - lo[1]), d2 = std::max(0.0f, hi[2] - lo[2]);
        return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
    }
    bool valid() const { return lo[0] <= hi[0]; }
};

struct N2 { AABB box; int left = -1, right = -1, first = 0, count = 0; };

struct Builder {
    const float* v;
    const int32_t* idx;
    int n;
    int max_leaf;
    int sah_depth = 40;   // deeper than this, only balanced (median) splits
    int n_bins = 32;      // SAH bins per axis (MPT_BVH_BINS, read once per build, clamped to [2, 256])
    std::vector<AABB> tbox;
    std::vector<float> cen;
    std::vector<int> order;
    std::vector<N2> nodes;

    int build2(int begin, int end, int depth) {
        int id = (int)nodes.size();
        nodes.emplace_back();
        AABB b, cb;
        for (int i = begin; i < end; i++) { b.grow(tbox[order[i]]); cb.grow(&cen[3 * (size_t)order[i]]); }
        nodes[id].box = b;
        int cnt = end - begin;
        if (cnt <= max_leaf) { nodes[id].first = begin; nodes[id].count = cnt; return id; }
        const int NB = n_bins;
        int best_axis = -1, best_split = 0;
        float best_cost = FLT_MAX;
        // past sah_depth only balanced splits, so that the tree depth stays bounded (traversal stack)
        for (int ax = 0; ax < 3 && depth < sah_depth; ax++) {
            float ext = cb.hi[ax] - cb.lo[ax];
            if (!(ext > 0.0f)) continue;
            AABB bb[256];
            int bc[256] = {0};
            float k = NB / ext;
            for (int i = begin; i < end; i++) {
                int t = order[i];
                int bi = std::min(NB - 1, (int)((cen[3 * (size_t)t + ax] - cb.lo[ax]) * k));
                bb[bi].grow(tbox[t]);
                bc[bi]++;
            }
            float la[256];
            int lc[256];
            AABB acc;
            int ac = 0;
            for (int i = 0; i < NB; i++) { acc.grow(bb[i]); ac += bc[i]; la[i] = acc.valid() ? acc.area() : 0.0f; lc[i] = ac; }
            acc = AABB();
            ac = 0;
            for (int i = NB - 1; i > 0; i--) {
                acc.grow(bb[i]);
                ac += bc[i];
                if (lc[i - 1] == 0 || ac == 0) continue;
                float cost = la[i - 1] * lc[i - 1] + acc.area() * ac;
                if (cost < best_cost) { best_cost = cost; best_axis = ax; best_split = i; }
            }
        }
        int mid;
        if (best_axis >= 0) {
            float ext = cb.hi[best_axis] - cb.lo[best_axis];
            float k = NB / ext;
            int* m = std::partition(order.data() + begin, order.data() + end, [&](int t) {
                return std::min(NB - 1, (int)((cen[3 * (size_t)t + best_axis] - cb.lo[best_axis]) * k)) < best_split;
            });
            mid = (int)(m - order.data());
        } else {
            mid = (begin + end) / 2;   // all centroids equal: split by count
        }
        if (mid == begin || mid == end) mid = (begin + end) / 2;
        int l = build2(begin, mid, depth + 1);
        int r = build2(mid, end, depth + 1);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }
};


inline uint8_t quant_exp(float ext) {
    // smallest e with 255 * 2^e >= ext, clamped to normal floats
    int e = -126;
    if (ext > 0.0f) {
        e = (int)std::ceil(std::log2((double)ext / 255.0));
        while (std::ldexp(255.0, e) < (double)ext) e++;
        e = std::max(-126, std::min(127, e));
    }
    return (uint8_t)(e + 127);
}

}  // namespace

float scene_box_pad(const float* vertices, int num_triangles, const int32_t* indices) {
    float m = 0.0f;
    for (size_t k = 0; k < 3 * (size_t)num_triangles; k++)
        for (int i = 0; i < 3; i++) m = std::max(m, std::fabs(vertices[3 * (size_t)indices[k] + i]));
    return std::ldexp(std::max(m, 1.0f), -20);
}

void build_bvh8(const float* vertices, const int32_t* indices, int32_t num_triangles, BVH8& out, int max_leaf,
                float pad_in, int sah_depth) {
    out.nodes.clear();
    out.tris.clear();
    if (num_triangles <= 0) return;
    max_leaf = std::max(1, std::min(4, max_leaf));
    Builder b;
    b.v = vertices;
    b.idx = indices;
    b.n = num_triangles;
    b.max_leaf = max_leaf;
    b.sah_depth = sah_depth;
    if (const char* nb = std::getenv("MPT_BVH_BINS")) b.n_bins = std::max(2, std::min(256, std::atoi(nb)));
    b.tbox.resize(num_triangles);
    b.cen.resize(3 * (size_t)num_triangles);
    b.order.resize(num_triangles);
    for (int t = 0; t < num_triangles; t++) {
        for (int k = 0; k < 3; k++) b.tbox[t].grow(vertices + 3 * (size_t)indices[3 * (size_t)t + k]);
        for (int i = 0; i < 3; i++) b.cen[3 * (size_t)t + i] = 0.5f * (b.tbox[t].lo[i] + b.tbox[t].hi[i]);
        b.order[t] = t;
    }
    // Pad every triangle box by 2^-20 of the scene's largest coordinate magnitude.  The
    // Moller-Trumbore test accepts hits a rounding error outside the exact triangle (a
    // ray grazing along a wall that holds an edge of the triangle), so unpadded boxes can
    // cull a triangle the test would accept.  With the pad, box culling never changes a
    // result: traversal equals brute force (the oracle pads its boxes the same way).
    const float pad = pad_in >= 0.0f ? pad_in : scene_box_pad(vertices, num_triangles, indices);
    for (int t = 0; t < num_triangles; t++)
        for (int i = 0; i < 3; i++) { b.tbox[t].lo[i] -= pad; b.tbox[t].hi[i] += pad; }
    const char* cm = std::getenv("MPT_BVH_COLLAPSE");
    const bool greedy = !(cm && std::strcmp(cm, "cost") == 0);
    const int leaf_max = max_leaf;
    if (!greedy) b.max_leaf = 1;   // the cost collapse forms leaves from BVH2 subtrees itself
    b.nodes.reserve(2 * (size_t)num_triangles);
    int root = b.build2(0, num_triangles, 0);

    // ---- cost collapse: cost[n][i-1] = cheapest representation of subtree n as at most i
    // child slots; how[n][i-1]: 0 = as i - 1 slots, 1..7 = split (k slots left, i - k right),
    // for i = 1: 8 = one leaf slot, 9 = one internal node
    const size_t N2n = b.nodes.size();
    std::vector<float> cost;
    std::vector<uint8_t> how, split8;   // split8[n]: slots of n's left child when n is an internal BVH8 node
    std::vector<int> tri_count;
    if (!greedy) {
        const float C_NODE = 1.0f;
        const char* ct = std::getenv("MPT_BVH_CTRI");   // development A/B: triangle test cost / node test cost
        const float C_TRI = ct ? (float)std::atof(ct) : 0.3f;
        cost.assign(N2n * 8, 0.0f);
        how.assign(N2n * 8, 0);
        split8.assign(N2n, 0);
        tri_count.assign(N2n, 0);
        // children have larger indices than their parent (pre-order build): reverse order is post-order
        for (size_t ni = N2n; ni-- > 0;) {
            const N2& nd = b.nodes[ni];
            const float A = nd.box.area();
            float* c = &cost[ni * 8];
            uint8_t* h = &how[ni * 8];
            if (nd.count > 0) {
                tri_count[ni] = nd.count;
                for (int i = 0; i < 8; i++) { c[i] = A * C_TRI * (float)nd.count; h[i] = i == 0 ? 8 : 0; }
                continue;
            }
            const int l = nd.left, r = nd.right;
            tri_count[ni] = tri_count[l] + tri_count[r];
            const float* cl = &cost[(size_t)l * 8];
            const float* cr = &cost[(size_t)r * 8];
            float dist[9];
            uint8_t dk[9];
            for (int j = 2; j <= 8; j++) {
                dist[j] = FLT_MAX;
                dk[j] = 1;
                for (int k = 1; k < j; k++) {
                    const float v = cl[k - 1] + cr[j - k - 1];
                    if (v < dist[j]) { dist[j] = v; dk[j] = (uint8_t)k; }
                }
            }
            const float c_internal = A * C_NODE + dist[8];
            split8[ni] = dk[8];
            const float c_leaf = tri_count[ni] <= leaf_max ? A * C_TRI * (float)tri_count[ni] : FLT_MAX;
            c[0] = std::min(c_leaf, c_internal);
            h[0] = c_leaf <= c_internal ? 8 : 9;
            for (int i = 2; i <= 8; i++) {
                if (dist[i] < c[i - 2]) { c[i - 1] = dist[i]; h[i - 1] = dk[i]; }
                else { c[i - 1] = c[i - 2]; h[i - 1] = 0; }
            }
        }
    }
    // the child slots of a BVH8 node made from BVH2 node n: n's subtree distributed over 8
    // slots as the cost choices say; each slot is a BVH2 node (a leaf slot if its choice is
    // 'leaf' or it is a BVH2 leaf, else an internal BVH8 node)
    auto distribute = [&](int n) {
        std::vector<int> out_slots;
        std::vector<std::pair<int, int>> work{{b.nodes[n].left, split8[n]}, {b.nodes[n].right, 8 - split8[n]}};
        while (!work.empty()) {
            auto [x, j] = work.back();
            work.pop_back();
            while (j > 1 && how[(size_t)x * 8 + j - 1] == 0) j--;
            if (j == 1 || b.nodes[x].count > 0) { out_slots.push_back(x); continue; }
            const int k = how[(size_t)x * 8 + j - 1];
            work.push_back({b.nodes[x].left, k});
            work.push_back({b.nodes[x].right, j - k});
        }
        return out_slots;
    };
    auto is_leaf_slot = [&](int x) { return b.nodes[x].count > 0 || (!greedy && how[(size_t)x * 8] == 8); };
    // the triangles of a leaf slot: the BVH2 subtree's triangles, in order
    auto leaf_tris = [&](int x, std::vector<int>& tris) {
        std::vector<int> stk{x};
        while (!stk.empty()) {
            int y = stk.back();
            stk.pop_back();
            const N2& ny = b.nodes[y];
            if (ny.count > 0) { for (int k = 0; k < ny.count; k++) tris.push_back(b.order[ny.first + k]); }
            else { stk.push_back(ny.right); stk.push_back(ny.left); }
        }
    };

    // BFS over BVH8 nodes; each entry names the BVH2 node it collapses
    struct Item { int n2; int n8; int depth; };
    std::vector<Item> queue;
    out.nodes.emplace_back();
    queue.push_back({root, 0, 1});
    size_t qi = 0;
    int max_depth = 1;
    while (qi < queue.size()) {
        Item it = queue[qi++];
        max_depth = std::max(max_depth, it.depth);
        // gather up to 8 children
        std::vector<int> ch;
        const N2& r2 = b.nodes[it.n2];
        if (r2.count > 0 || (!greedy && how[(size_t)it.n2 * 8] == 8)) ch.push_back(it.n2);   // the root is one leaf
        else if (!greedy) ch = distribute(it.n2);
        else {
            ch.push_back(r2.left);
            ch.push_back(r2.right);
            while (ch.size() < 8) {
                int best = -1;
                float ba = -1.0f;
                for (int i = 0; i < (int)ch.size(); i++) {
                    const N2& c = b.nodes[ch[i]];
                    if (c.count == 0 && c.box.area() > ba) { ba = c.box.area(); best = i; }
                }
                if (best < 0) break;
                int nb = ch[best];
                ch[best] = b.nodes[nb].left;
                ch.push_back(b.nodes[nb].right);
            }
        }
        // node box and slot assignment (octant heuristic)
        AABB nb;
        for (int c : ch) nb.grow(b.nodes[c].box);
        float pc[3] = {0.5f * (nb.lo[0] + nb.hi[0]), 0.5f * (nb.lo[1] + nb.hi[1]), 0.5f * (nb.lo[2] + nb.hi[2])};
        int slot_of[8];
        int child_in_slot[8];
        for (int s = 0; s < 8; s++) child_in_slot[s] = -1;
        bool used[8] = {false};
        for (int round = 0; round < (int)ch.size(); round++) {
            float best = FLT_MAX;
            int bi = -1, bs = -1;
            for (int i = 0; i < (int)ch.size(); i++) {
                if (used[i]) continue;
                const AABB& cb = b.nodes[ch[i]].box;
                float v[3];
                for (int a = 0; a < 3; a++) v[a] = 0.5f * (cb.lo[a] + cb.hi[a]) - pc[a];
                for (int s = 0; s < 8; s++) {
                    if (child_in_slot[s] >= 0) continue;
                    float cost = -((s & 1 ? v[0] : -v[0]) + (s & 2 ? v[1] : -v[1]) + (s & 4 ? v[2] : -v[2]));
                    if (cost < best) { best = cost; bi = i; bs = s; }
                }
            }
            used[bi] = true;
            child_in_slot[bs] = bi;
            slot_of[bi] = bs;
        }
        (void)slot_of;
        Node8 nd;
        std::memset(&nd, 0, sizeof(nd));
        nd.px = nb.lo[0];
        nd.py = nb.lo[1];
        nd.pz = nb.lo[2];
        uint8_t e[3];
        for (int a = 0; a < 3; a++) e[a] = quant_exp(nb.hi[a] - nb.lo[a]);
        nd.ex = e[0];
        nd.ey = e[1];
        nd.ez = e[2];
        nd.child_base = (uint32_t)out.nodes.size();
        nd.tri_base = (uint32_t)out.tris.size();
        int internal_rank = 0;
        double p[3] = {nd.px, nd.py, nd.pz};
        for (int s = 0; s < 8; s++) {
            int ci = child_in_slot[s];
            if (ci < 0) continue;
            const N2& c = b.nodes[ch[ci]];
            uint8_t qlo[3], qhi[3];
            for (int a = 0; a < 3; a++) {
                double sc = std::ldexp(1.0, (int)e[a] - 127);
                double lo = std::floor(((double)c.box.lo[a] - p[a]) / sc);
                double hi = std::ceil(((double)c.box.hi[a] - p[a]) / sc);
                while (lo > 0 && p[a] + lo * sc > (double)c.box.lo[a]) lo -= 1;
                while (hi < 255 && p[a] + hi * sc < (double)c.box.hi[a]) hi += 1;
                lo = std::max(0.0, std::min(255.0, lo));
                hi = std::max(0.0, std::min(255.0, hi));
                qlo[a] = (uint8_t)lo;
                qhi[a] = (uint8_t)hi;
            }
            nd.qlox[s] = qlo[0]; nd.qloy[s] = qlo[1]; nd.qloz[s] = qlo[2];
            nd.qhix[s] = qhi[0]; nd.qhiy[s] = qhi[1]; nd.qhiz[s] = qhi[2];
            if (!is_leaf_slot(ch[ci])) {
                nd.imask |= (uint8_t)(1u << s);
                nd.meta[s] = (uint8_t)internal_rank++;
                out.nodes.emplace_back();
                queue.push_back({ch[ci], (int)out.nodes.size() - 1, it.depth + 1});
            } else {
                int off = (int)out.tris.size() - (int)nd.tri_base;
                std::vector<int> lt;
                leaf_tris(ch[ci], lt);
                nd.meta[s] = (uint8_t)(((int)lt.size() << 5) | off);
                for (int t : lt) {
                    const float* A = vertices + 3 * (size_t)indices[3 * (size_t)t + 0];
                    const float* B = vertices + 3 * (size_t)indices[3 * (size_t)t + 1];
                    const float* C = vertices + 3 * (size_t)indices[3 * (size_t)t + 2];
                    TriRec tr;
                    std::memset(&tr, 0, sizeof(tr));
                    tr.ax = A[0]; tr.ay = A[1]; tr.az = A[2];
                    int32_t pb = t;
                    std::memcpy(&tr.prim_bits, &pb, 4);
                    tr.e1x = B[0] - A[0]; tr.e1y = B[1] - A[1]; tr.e1z = B[2] - A[2];
                    tr.e2x = C[0] - A[0]; tr.e2y = C[1] - A[1]; tr.e2z = C[2] - A[2];
                    out.tris.push_back(tr);
                }
            }
        }
        out.nodes[it.n8] = nd;
    }
    out.depth = max_depth;
}

}  // namespace mpt
