// bvh8.h -- compressed 8-wide BVH ("BVH8") built on the host, traversed by the HIP
// kernels.  Replaces HIPRT's BVH build (HIPRTGeometry::build_bvh,
// src/HIPRT-Orochi/HIPRTScene.h:60-87, hiprtBuildFlagBitPreferHighQualityBuild) and
// the RDNA ray-tracing-unit traversal the reference relies on.
//
// Node: 80 bytes = 5 x 16-byte loads.  Child boxes are quantised to 8 bits per
// bound on a per-node power-of-two grid (conservatively rounded outward), so one
// node holds 8 children in the space of ~2.5 uncompressed BVH2 nodes.
// Triangle record: 48 bytes = vertex A, edges B-A and C-A (float32, the exact values
// the reference's Moller-Trumbore test computes, Renderer/Triangle.h:24-25) and the
// original primitive index.
#ifndef MPT_BVH8_H
#define MPT_BVH8_H

#include <cstdint>
#include <vector>

namespace mpt {

struct alignas(16) Node8 {
    float px, py, pz;          // quantisation origin (node box min)
    uint8_t ex, ey, ez;        // biased exponents: scale = 2^(e - 127)
    uint8_t imask;             // bit s: slot s is an internal child
    uint32_t child_base;       // node index of the first internal child
    uint32_t tri_base;         // index of the first triangle record of the node
    uint8_t meta[8];           // internal: rank among internal children; leaf: (count << 5) | offset; empty: 0
    uint8_t qlox[8], qloy[8], qloz[8];
    uint8_t qhix[8], qhiy[8], qhiz[8];
};
static_assert(sizeof(Node8) == 80, "Node8 must be 80 bytes");

struct alignas(16) TriRec {
    float ax, ay, az, prim_bits;   // prim index stored as int bits in the 4th lane
    float e1x, e1y, e1z, pad0;
    float e2x, e2y, e2z, pad1;
};
static_assert(sizeof(TriRec) == 48, "TriRec must be 48 bytes");

struct BVH8 {
    std::vector<Node8> nodes;
    std::vector<TriRec> tris;
    int depth = 0;
    float sah_cost = 0.0f;
};

// Builds the BVH8 over indexed triangles.  max_leaf: triangles per leaf child (<= 4).
// pad: triangle-box padding (< 0: 2^-20 of the largest coordinate of these triangles; a
// BVH over a subset of a scene passes the whole scene's pad, scene_box_pad).
// sah_depth: BVH2 depth below which SAH splits are used, balanced splits beyond (a smaller
// value gives a shallower tree: the rebuild of a BVH too deep for the traversal stack).
void build_bvh8(const float* vertices, const int32_t* indices, int32_t num_triangles, BVH8& out, int max_leaf = 3,
                float pad = -1.0f, int sah_depth = 40);
float scene_box_pad(const float* vertices, int num_triangles, const int32_t* indices);

}  // namespace mpt

#endif
