// bvh.hpp — host-side BVH build for exact culling (mesh upload time).
//
// The reference culls with an rtreego R-tree of padded face boxes
// (shared/state/mesh.go:30-50, :139, :208; shared/geom/box.go:29-68).  On the GPU the
// same role is played by a binary BVH traversed by whole waves (packet traversal), with
// one requirement the reference does not have: culling must never change a result, so
// every box is inflated far beyond the rounding error of the fp64 Möller–Trumbore test
// and of the fp64 slab test.  Build: recursive median split of the face
// centroids along the longest axis, leaves of <= kBvhLeaf faces, nodes emitted depth
// first with a skip index per node.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <array>
#include <functional>
#include <cmath>
#include <vector>

#include "mirt_internal.hpp"

namespace mirt {

struct BvhBuild {
    std::vector<BvhNode> nodes;
    std::vector<uint32_t> order;  // position -> original face index
};

// v: nv*3 vertex array, fv: nf*3 indices.  inflate: absolute padding added to every box.
inline BvhBuild build_bvh(const double* v, const uint32_t* fv, uint32_t nf, double inflate) {
    BvhBuild b;
    b.order.resize(nf);
    for (uint32_t i = 0; i < nf; ++i) b.order[i] = i;
    if (nf == 0) return b;
    std::vector<std::array<double, 3>> lo(nf), hi(nf), ce(nf);
    for (uint32_t f = 0; f < nf; ++f) {
        for (int k = 0; k < 3; ++k) {
            double a = v[3 * (size_t)fv[3 * f] + k], bb = v[3 * (size_t)fv[3 * f + 1] + k],
                   c = v[3 * (size_t)fv[3 * f + 2] + k];
            lo[f][k] = std::min(a, std::min(bb, c));
            hi[f][k] = std::max(a, std::max(bb, c));
            ce[f][k] = 0.5 * (lo[f][k] + hi[f][k]);
        }
    }
    struct Job {
        uint32_t begin, end;
        uint32_t node;
    };
    // recursive build with an explicit stack; skip indices patched after the subtree
    std::vector<uint32_t> parents_pending;
    std::function<void(uint32_t, uint32_t)> rec;
    rec = [&](uint32_t begin, uint32_t end) {
        uint32_t idx = (uint32_t)b.nodes.size();
        b.nodes.push_back(BvhNode{});
        double l[3] = {INFINITY, INFINITY, INFINITY}, h[3] = {-INFINITY, -INFINITY, -INFINITY};
        double cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = begin; i < end; ++i) {
            uint32_t f = b.order[i];
            for (int k = 0; k < 3; ++k) {
                l[k] = std::min(l[k], lo[f][k]);
                h[k] = std::max(h[k], hi[f][k]);
                cl[k] = std::min(cl[k], ce[f][k]);
                ch[k] = std::max(ch[k], ce[f][k]);
            }
        }
        for (int k = 0; k < 3; ++k) {
            b.nodes[idx].lo[k] = l[k] - inflate;
            b.nodes[idx].hi[k] = h[k] + inflate;
        }
        if (end - begin <= (uint32_t)kBvhLeaf) {
            b.nodes[idx].first = begin;
            b.nodes[idx].count = end - begin;
        } else {
            int axis = 0;
            for (int k = 1; k < 3; ++k)
                if (ch[k] - cl[k] > ch[axis] - cl[axis]) axis = k;
            uint32_t mid = begin + (end - begin) / 2;
            std::nth_element(b.order.begin() + begin, b.order.begin() + mid, b.order.begin() + end,
                             [&](uint32_t x, uint32_t y) {
                                 return ce[x][axis] < ce[y][axis] || (ce[x][axis] == ce[y][axis] && x < y);
                             });
            b.nodes[idx].count = 0;
            b.nodes[idx].first = 0;
            rec(begin, mid);
            rec(mid, end);
        }
        b.nodes[idx].skip = (uint32_t)b.nodes.size();
    };
    rec(0, nf);
    return b;
}

}  // namespace mirt
