// bvh.hpp — host-side BVH builds for exact culling (mesh upload time).
//
// The reference culls with an rtreego R-tree of padded face boxes
// (shared/state/mesh.go:30-50, :139, :208; shared/geom/box.go:29-68).  On the GPU the
// same role is played by an 8-wide BVH that whole waves walk together (packet
// traversal).  Culling must never change a result, so every box is inflated far beyond
// the rounding error of the fp64 Möller–Trumbore test and of the fp32 slab test that
// reads it.
//
// Build: SAH on all three axes (an exact sweep for nodes of <= 256 faces, else 32 bins on
// centroids) into a binary tree with leaves
// of <= kBvhLeaf faces, then collapse to 8-wide nodes by repeatedly opening the child
// with the largest surface area.  Faces are reordered so that every leaf is one
// contiguous range.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <vector>

#include "mirt_internal.hpp"

namespace mirt {

struct BvhBuild {
    std::vector<Bvh8Node> nodes;  // nodes[0] is the root
    std::vector<uint32_t> order;  // position -> original face index
    uint32_t depth = 0;           // inner levels (stack bound for traversal)
};

namespace detail {

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow(const double p[3]) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    double area() const {
        double e[3];
        for (int k = 0; k < 3; ++k) e[k] = std::max(0.0, hi[k] - lo[k]);
        return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
    }
};

struct BNode {  // binary build node
    Box box;
    int left = -1, right = -1;
    uint32_t first = 0, count = 0;  // leaf range
};

struct Builder {
    uint32_t leaf;  // max faces per leaf
    const std::vector<Box>& fbox;
    const std::vector<std::array<double, 3>>& ce;
    std::vector<uint32_t>& order;
    std::vector<BNode> nodes;

    int build(uint32_t begin, uint32_t end) {
        BNode n;
        Box cb;
        for (uint32_t i = begin; i < end; ++i) {
            n.box.grow(fbox[order[i]]);
            cb.grow(ce[order[i]].data());
        }
        const uint32_t cnt = end - begin;
        int idx = (int)nodes.size();
        nodes.push_back(n);
        if (cnt <= leaf) {
            nodes[idx].first = begin;
            nodes[idx].count = cnt;
            return idx;
        }
        // SAH split on every axis: an exact sweep over the sorted centroids for up to
        // kSweep faces, else 32 bins on the centroid extent
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
        uint32_t mid = begin + cnt / 2;
        double best = INFINITY;
        int best_axis = -1;
        uint32_t best_cut = 0;   // sweep: faces left of the cut; bins: first bin on the right
        constexpr uint32_t kSweep = 256;
        constexpr int B = 32;
        std::vector<uint32_t> tmp;
        std::vector<double> rarea;
        for (int a = 0; a < 3; ++a) {
            const double ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0)) continue;
            if (cnt <= kSweep) {
                tmp.assign(order.begin() + begin, order.begin() + end);
                std::sort(tmp.begin(), tmp.end(), [&](uint32_t x, uint32_t y) {
                    return ce[x][a] < ce[y][a] || (ce[x][a] == ce[y][a] && x < y);
                });
                rarea.assign(cnt + 1, 0.0);
                Box r;
                for (uint32_t i = cnt; i-- > 1;) {
                    r.grow(fbox[tmp[i]]);
                    rarea[i] = r.area();
                }
                Box l;
                for (uint32_t i = 1; i < cnt; ++i) {
                    l.grow(fbox[tmp[i - 1]]);
                    const double cost = l.area() * i + rarea[i] * (cnt - i);
                    if (cost < best) {
                        best = cost;
                        best_axis = a;
                        best_cut = i;
                    }
                }
            } else {
                Box bb[B];
                uint32_t bc[B] = {0};
                for (uint32_t i = begin; i < end; ++i) {
                    const uint32_t f = order[i];
                    const int b = std::min(B - 1, std::max(0, (int)((ce[f][a] - cb.lo[a]) / ext * B)));
                    bb[b].grow(fbox[f]);
                    bc[b]++;
                }
                for (int sp = 1; sp < B; ++sp) {
                    Box l, r;
                    uint32_t nl = 0, nr = 0;
                    for (int b = 0; b < sp; ++b) if (bc[b]) { l.grow(bb[b]); nl += bc[b]; }
                    for (int b = sp; b < B; ++b) if (bc[b]) { r.grow(bb[b]); nr += bc[b]; }
                    if (!nl || !nr) continue;
                    const double cost = l.area() * nl + r.area() * nr;
                    if (cost < best) {
                        best = cost;
                        best_axis = a;
                        best_cut = (uint32_t)sp;
                    }
                }
            }
        }
        if (best_axis >= 0) {
            const int a = best_axis;
            axis = a;
            if (cnt <= kSweep) {
                std::sort(order.begin() + begin, order.begin() + end, [&](uint32_t x, uint32_t y) {
                    return ce[x][a] < ce[y][a] || (ce[x][a] == ce[y][a] && x < y);
                });
                mid = begin + best_cut;
            } else {
                const double ext = cb.hi[a] - cb.lo[a];
                auto it = std::partition(order.begin() + begin, order.begin() + end, [&](uint32_t f) {
                    return std::min(B - 1, std::max(0, (int)((ce[f][a] - cb.lo[a]) / ext * B))) < (int)best_cut;
                });
                mid = (uint32_t)(it - order.begin());
            }
        }
        if (mid == begin || mid == end) {  // degenerate centroids: median by index
            mid = begin + cnt / 2;
            std::nth_element(order.begin() + begin, order.begin() + mid, order.begin() + end,
                             [&](uint32_t x, uint32_t y) {
                                 return ce[x][axis] < ce[y][axis] || (ce[x][axis] == ce[y][axis] && x < y);
                             });
        }
        int l = build(begin, mid);
        int r = build(mid, end);
        nodes[idx].left = l;
        nodes[idx].right = r;
        return idx;
    }
};

inline float round_down(double x) {
    float f = (float)x;
    return (double)f > x ? std::nextafter(f, -INFINITY) : f;
}
inline float round_up(double x) {
    float f = (float)x;
    return (double)f < x ? std::nextafter(f, INFINITY) : f;
}

}  // namespace detail

// v: nv*3 vertex array, fv: nf*3 indices.  inflate: absolute padding of every box
// (applied in fp64, then rounded outward to fp32).
inline BvhBuild build_bvh(const double* v, const uint32_t* fv, uint32_t nf, double inflate,
                          uint32_t leaf = (uint32_t)kBvhLeaf) {
    using namespace detail;
    BvhBuild out;
    out.order.resize(nf);
    for (uint32_t i = 0; i < nf; ++i) out.order[i] = i;
    std::vector<Box> fbox(nf);
    std::vector<std::array<double, 3>> ce(nf);
    for (uint32_t f = 0; f < nf; ++f) {
        for (int c = 0; c < 3; ++c) fbox[f].grow(v + 3 * (size_t)fv[3 * f + c]);
        for (int k = 0; k < 3; ++k) ce[f][k] = 0.5 * (fbox[f].lo[k] + fbox[f].hi[k]);
    }
    Builder b{std::max<uint32_t>(1, std::min<uint32_t>(leaf, 127)), fbox, ce, out.order, {}};
    if (nf == 0) {
        Bvh8Node root;
        for (int c = 0; c < 8; ++c) root.child[c] = kBvhEmpty;
        for (int k = 0; k < 3; ++k)
            for (int c = 0; c < 8; ++c) { root.lo(k, c) = INFINITY; root.hi(k, c) = -INFINITY; }
        out.nodes.push_back(root);
        return out;
    }
    b.build(0, nf);
    // collapse the binary tree into 8-wide nodes
    struct Pending { int bnode; uint32_t slot; uint32_t level; };
    std::vector<Pending> work;
    out.nodes.emplace_back();
    work.push_back({0, 0, 1});
    while (!work.empty()) {
        Pending p = work.back();
        work.pop_back();
        out.depth = std::max(out.depth, p.level);
        std::vector<int> kids;
        const BNode& bn = b.nodes[p.bnode];
        if (bn.left < 0) {
            kids.push_back(p.bnode);  // a root that is itself a leaf
        } else {
            kids.push_back(bn.left);
            kids.push_back(bn.right);
            while (kids.size() < 8) {
                int best = -1;
                double ba = -1;
                for (size_t i = 0; i < kids.size(); ++i) {
                    const BNode& k = b.nodes[kids[i]];
                    if (k.left >= 0 && k.box.area() > ba) { ba = k.box.area(); best = (int)i; }
                }
                if (best < 0) break;
                int open = kids[best];
                kids[best] = b.nodes[open].left;
                kids.push_back(b.nodes[open].right);
            }
        }
        Bvh8Node nd;  // filled locally: emplace_back below may reallocate out.nodes
        for (int c = 0; c < 8; ++c) {
            if (c >= (int)kids.size()) {
                nd.child[c] = kBvhEmpty;
                for (int k = 0; k < 3; ++k) { nd.lo(k, c) = INFINITY; nd.hi(k, c) = -INFINITY; }
                continue;
            }
            const BNode& k = b.nodes[kids[c]];
            for (int a = 0; a < 3; ++a) {
                nd.lo(a, c) = round_down(k.box.lo[a] - inflate);
                nd.hi(a, c) = round_up(k.box.hi[a] + inflate);
            }
            if (k.left < 0) {
                nd.child[c] = kBvhLeafBit | (k.count << kBvhCountShift) | k.first;
            } else {
                uint32_t slot = (uint32_t)out.nodes.size();
                nd.child[c] = slot;
                out.nodes.emplace_back();
                work.push_back({kids[c], slot, p.level + 1});
            }
        }
        out.nodes[p.slot] = nd;
    }
    return out;
}

// The kernels' node format (mirt_internal.hpp Bvh8Dev): per sign octant, the children
// sorted near to far along the octant's diagonal, bounds stored near plane first.
inline std::vector<Bvh8Dev> make_dev_nodes(const std::vector<Bvh8Node>& nodes) {
    std::vector<Bvh8Dev> out(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) {
        const Bvh8Node& n = nodes[i];
        int nk = 0;
        while (nk < 8 && n.child[nk] != kBvhEmpty) ++nk;
        for (uint32_t o = 0; o < 8; ++o) {
            Bvh8Copy& cp = out[i].oct[o];
            int ord[8];
            double key[8];
            for (int c = 0; c < nk; ++c) {
                ord[c] = c;
                key[c] = 0;
                for (int a = 0; a < 3; ++a) {
                    const double ctr = 0.5 * ((double)n.lo(a, c) + (double)n.hi(a, c));
                    key[c] += ((o >> a) & 1u) ? -ctr : ctr;
                }
            }
            std::stable_sort(ord, ord + nk, [&](int x, int y) { return key[x] < key[y]; });
            for (int slot = 0; slot < 8; ++slot) {
                const bool full = slot < nk;
                const int c = full ? ord[slot] : 0;
                for (int a = 0; a < 3; ++a) {
                    const float lo = full ? n.lo(a, c) : INFINITY, hi = full ? n.hi(a, c) : -INFINITY;
                    const bool neg = ((o >> a) & 1u) != 0;
                    cp.box[a][slot][0] = neg ? hi : lo;
                    cp.box[a][slot][1] = neg ? lo : hi;
                }
                cp.child[slot] = full ? n.child[c] : kBvhEmpty;
            }
            for (uint32_t& w : cp.pad) w = 0;
        }
    }
    return out;
}

}  // namespace mirt
