// mirt_internal.hpp — layouts shared by the host side (mirt.cpp) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mirt.h"

namespace mirt {

// Launch geometry.  Persistent workgroups of 8 waves (two per CU: the LDS mesh copy is
// 72 KiB).  A wave's unit of primary work is one 8x8 pixel block; waves take blocks
// from a sharded work queue independently of each other (see the counter layout below).
#ifndef MIRT_WG
#define MIRT_WG 512
#endif
constexpr int kWG = MIRT_WG;  // threads per workgroup of the trace kernels
// persistent workgroups resident per CU (LDS-bound: each holds the mesh; one workgroup of
// 12 or 16 waves per CU when built with MIRT_WG 768 / 1024)
constexpr int kWgPerCu = kWG >= 768 ? 1 : 1024 / kWG;  // 16 waves per CU at 128 VGPRs
constexpr int kBlk = 8;
// Doubles per triangle record in HBM and LDS: P1, E1 = P2-P1, E2 = P3-P1 (72 B).
constexpr int kTriD = 9;
// Floats per light-table record (shadow segments, kernels.hip SegPre): W1, W2, W3, A, ntL,
// cw, cA, ctL (64 B: one scalar load).
constexpr int kLtD = 16;
// Triangles one workgroup holds in LDS (73,728 B; two workgroups per CU fit in 160 KiB).
// Meshes up to this size stay resident in LDS for the life of a persistent workgroup;
// larger meshes stream through it in batches of this size.
constexpr int kLdsTris = 1024;

// 8-wide BVH node as built on the host (bvh.hpp).  Child boxes are fp32, rounded outward
// and inflated so that a ray the fp64 Möller–Trumbore test could report as a hit always
// passes the fp32 slab test (DESIGN.md §4 "Exact culling").  child[c]: kBvhEmpty, an
// inner node index, or kBvhLeafBit | count << kBvhCountShift | first (a contiguous
// triangle range).  Non-empty children come first.
struct Bvh8Node {
    float box[3][8][2];  // [axis][child][lo, hi]
    uint32_t child[8];
    float& lo(int a, int c) { return box[a][c][0]; }
    float& hi(int a, int c) { return box[a][c][1]; }
    float lo(int a, int c) const { return box[a][c][0]; }
    float hi(int a, int c) const { return box[a][c][1]; }
};
// The node as the kernels read it: one 256-byte copy per sign octant of a packet's ray
// directions (bit a set: 1/d < 0 on axis a).  In copy o the children are sorted near to
// far along the octant's diagonal (box centres projected on (+-1, +-1, +-1)) and each
// axis's bounds are stored near plane first ((hi, lo) on the negative axes), so a packet
// of that octant tests a child with no min/max sorting and pushes the nearest child last
// (it is popped first).  An empty slot is the box lo = +inf, hi = -inf stored the same way:
// every ordered test of it fails.  Copy 0 doubles as the (lo, hi) copy that packets of
// mixed signs test with the sorted slab test (they skip empty slots by their ref).  Read
// with four scalar loads (three s_load_dwordx16 of bounds, one s_load_dwordx8 of refs).
struct alignas(256) Bvh8Copy {
    float box[3][8][2];  // [axis][slot][near, far]
    uint32_t child[8];   // slot order
    uint32_t pad[8];
};
struct Bvh8Dev {
    Bvh8Copy oct[8];
};
constexpr uint32_t kBvhEmpty = 0xffffffffu;
constexpr uint32_t kBvhLeafBit = 0x80000000u;
constexpr int kBvhCountShift = 24;
constexpr uint32_t kBvhFirstMask = 0x00ffffffu;
constexpr int kBvhLeaf = 3;           // max triangles per leaf (2: +0%, 4: +2.6% frame interval)
constexpr int kBvhStack = 128;        // per-wave traversal stack entries (two VGPRs / LDS)
constexpr int kBvhMaxDepth = (kBvhStack - 1) / 7;
// A traversal pushes every entered child (leaves too): at most 7 per inner level plus the
// last node's 8, i.e. 7 depth + 1 entries.  Meshes with depth <= kBvhShallowDepth walk
// with a one-VGPR (64-entry) stack; the LDS-resident kernels require it.
constexpr int kBvhShallowDepth = 8;
// Wide traversal (shared-origin packets): up to 8 nodes per pass, one lane per child box.
// Batching is allowed only while the stack holds <= DevMesh::wide_thresh entries
// (= kBvhStack - 64 - 7 * depth), which bounds the stack by kBvhStack.
constexpr int kWideBatch = 8;

// One uploaded mesh, device pointers (shared/state/mesh.go:100-106).  Every per-face
// array is stored in BVH leaf order; fidx maps a position back to the face index of
// the uploaded mesh (reported outputs and tie-breaking use that original index).
// A BVH leaf as the view tables see it: its inflated fp32 box (the one its parent node
// holds) and its ref (kBvhLeafBit | count << kBvhCountShift | first).
struct LeafBox {
    float lo[3], hi[3];
    uint32_t ref, pad;
};

// `tri` is one allocation: [ntri * 9 tri][ntri * 6 face boxes][3 centre] (mesh_fbox,
// mesh_center), so the face boxes cost no kernel-argument bytes.
struct DevMesh {
    const double* tri;       // ntri * 9 : P1, E1, E2; then the face boxes and the centre
    const double* vnrm;      // ntri * 9 : N1, N2, N3 (normalised) if has_normals
    const uint32_t* fmat;    // ntri     : material index
    const uint32_t* fidx;    // ntri     : original face index
    const Bvh8Dev* nodes;    // root first
    const double* mats;      // nmat * 10: ka[3] kd[3] ks[3] ns
    const LeafBox* leaves;   // nleaves BVH leaves (view tables)
    uint32_t ntri;
    uint32_t has_normals;
    uint32_t depth;
    uint32_t nleaves;
    double cull_limit;       // rays whose object-space origin has a coordinate beyond this
                             // are never culled (tolerance scales with |origin|)
};
// Per BVH position: face.Bounds (mesh.go:30-50) as NewBox corners {MinCorner, MaxCorner}.
constexpr int kBoxD = 6;
__host__ __device__ inline const double* mesh_fbox(const DevMesh& m) { return m.tri + (size_t)m.ntri * kTriD; }
// centre of the mesh's bounding box (light views look at it)
__host__ __device__ inline const double* mesh_center(const DevMesh& m) {
    return m.tri + (size_t)m.ntri * (kTriD + kBoxD);
}
// wide traversal batches nodes only while the stack holds <= this many entries (< 0: never)
__host__ __device__ inline int32_t wide_thresh(const DevMesh& m) { return (int32_t)kBvhStack - 64 - 7 * (int32_t)m.depth; }

// View tables (one-object frames with an LDS-resident mesh).  A view is a point every ray
// of a packet passes through: the camera for primary rays, a light for shadow rays (a
// shadow segment runs from its hit point to the light).  With R = [F L U]^-1 for a basis
// (F, L, U) of the view, a point X (relative to the view point) lies in direction
// (s, t) = (R1.X / z, R2.X / z) at depth z = R0.X.  Per frame and view one workgroup of
// k_trace (the launch's first ones, before they stage the mesh) projects every leaf box (a box entirely in front: the bounding rectangle of its corners'
// (s, t), rounded outward with a relative margin of 2^-18; anything else: every direction)
// and sorts the leaves by their distance from the view point, then publishes the table
// (ViewHead::tag = WorkArgs::view_tag, an agent-scope release); until a wave has seen the
// tag it walks the BVH, so no wave ever waits for a table.  A packet then scans the
// table instead of walking the BVH: a leaf is tested when some live lane's direction lies
// in its rectangle and the leaf is not farther than that lane's depth bound; the scan stops
// at the first leaf farther than every live lane's bound.  Exact for the reason the block
// frustum pre-test is: a hit lies in its inflated leaf box, so its direction from the view
// point lies in the box's projection.
struct ViewLeaf {
    float s0, s1, t0, t1;  // rectangle of directions (every direction: -inf, inf, -inf, inf)
    float dmin;            // distance from the view point to the box, rounded down (+inf: never met)
    uint32_t ref;          // the BVH leaf ref
    uint32_t pad[2];
};
constexpr uint32_t kMaxViewLeaves = 512;  // meshes with more leaves walk the BVH
constexpr uint32_t kMaxViewTables = 16;   // frames x views per launch (more: the BVH walk)
// One view of one frame: 0 = the camera, 1 + l = light l.  ok = 0: no table (walk the BVH).
struct ViewHead {
    uint32_t ok;           // the table is usable (0: view point out of range, basis degenerate)
    float near_r;          // light views: leaves within this distance of the light are always tested
    uint32_t tag;          // WorkArgs::view_tag of the launch that built it (written last, release)
    uint32_t pad;
    double R[3][3];        // the view's projection rows
    double O[3];           // the view point, object space
};

// Kernel modes (mirt_set_options): exact BVH culling (default) or brute force.
enum TraceMode { kModeBvh = 0, kModeBrute = 1 };

struct DevObject {
    DevMesh m;
    double pos[3];
    double box[kBoxD];  // Object.Bounds (object.go:31-59) as NewBox corners, world space
};

// Everything per frame travels by value in the kernel-argument block (s_load'ed).
struct FrameArgs {
    double cam[3], fwd[3], left[3], up[3];
    double phw, phh;              // tan(fov/2) and phw*H/W (tracer.go:17-18)
    int32_t W, H, halfW, halfH;   // halfW = W/2 with Go integer division
    uint32_t n_objects, n_lights;
    uint32_t flags, pad;
    DevObject obj[MIRT_MAX_OBJECTS];
    double lpos[MIRT_MAX_LIGHTS][3];
    double lcol[MIRT_MAX_LIGHTS][3];
    // shadow segments of one-object frames: obj[0]'s light table, kLtD floats per light and
    // BVH position (kernels.hip SegPre, mirt.cpp light_table); NULL: no fp32 pre-classification
    const float* ltab;
    uint32_t ltab_n, ltab_pad;  // records per light (= obj[0]'s ntri)
#ifdef MIRT_FA_PAD
    uint8_t fa_pad[MIRT_FA_PAD];  // kernarg-layout experiments only
#endif
};

// A tiled frame group's share in full-height strips (k_trace only, FrameRec::xf): the rgbv
// plane is the share's TRANSFER form, written in place (k_pack_rect's layout, so no pack
// launch): pixel (i, j) of packed column k goes to word (k - k0) * ch + (j - y0) when
// x0 <= i < x1 and y0 <= j < y0 + ch, and nowhere otherwise; the launch's last workgroup
// writes the trailer {tag, words} at word `words`.  on == 0: the packed layout (every pixel
// at its packed index).
struct XferArgs {
    uint32_t on, k0, x0, x1, y0, ch, words, tag;
};
constexpr uint64_t kNoOut = ~0ull;  // out_index: a pixel the frame does not store

struct TileDesc {
    uint32_t x, y, w, h;
    uint64_t out_off;      // first packed pixel of this tile
    uint32_t region;       // k_unpack_rect: the rank region holding the tile
    uint32_t pad;          // k_unpack_rect: index of that region's first tile
};



// One 8x8 pixel block of one tile: the primary kernel's work item.  Built on the host
// per tile list (cached while the list does not change) and stored shard-major (entry
// q * per_shard + k describes block k * kQShards + q), so the consecutive tickets of a
// shard read consecutive 16-byte entries with one scalar load each.
struct alignas(16) BlockDesc {
    uint32_t out;          // packed index of the block's (0, 0) pixel
    uint32_t pxy;          // screen pixel of (0, 0): px | py << 16
    uint32_t geo;          // tile height (packed column stride) | vw << 16 | vh << 24
    uint32_t pad;
};

struct OutPlanes {
    double* rgb;
    uint8_t* rgb8;
    uint8_t* valid;
    int32_t* face;
    int32_t* object;
    uint32_t* rgbv;  // r | g << 8 | b << 16 | valid << 24 (packed multi-GPU tiles)
};

// A primary hit handed from the primary kernel to the shadow and shade kernels.
constexpr uint32_t kNoHit = 0xffffffffu;
struct HitRec {
    double h[3];     // world-space intersection
    double n[3];     // interpolated (or flat) normal
    uint64_t out;    // packed output pixel index
    uint32_t obj;    // object index (kNoHit: empty slot)
    uint32_t mat;    // material index inside that object's mesh
};

// Counters kept in device memory per call slot, zeroed before every frame.  Each counter
// owns a 128-byte line: same-line atomics serialise (~90 per microsecond on MI355X), so
// every contended counter is split kQShards ways.
//   queue(q, s): work-queue tickets of kernel q (0 primary, 1 shadow, 2 reflect) for shard s.
//     Primary block b belongs to shard b % kQShards; a wave serves the shard
//     (global wave id % kQShards) and takes one block per ticket.
//   hits(s):     hit slots of shard s.  A block with at least one hit takes 64 slots of
//     region s (capacity hit_cap = ceil(blocks / kQShards) * 64 records), slot = lane =
//     pixel of the 8x8 block, so a 64-slot shadow chunk is one block: a 2D-coherent packet.
//     Slots of pixels that missed carry obj = kNoHit.  The shadow and shade kernels walk
//     regions without any cross-shard prefix sum.
//   stat(k, s):  statistics (ray-triangle tests, BVH node/leaf visits), reduced per
//     workgroup in LDS and added once per workgroup into shard blockIdx % kStatShards.
// Each slot holds two such sets and alternates between them frame by frame: workgroup 0
// of k_primary zeroes the set the NEXT frame will use (its last user, the frame before,
// has finished: frames on one slot never overlap), so no frame needs a memset; workgroup
// 0 of k_shade folds this frame's statistics into WorkArgs::summary (and the profiling
// accumulator) once the producing kernels are done.
constexpr int kQShards = 64, kStatShards = 8, kLine = 16;
enum { kStatPrimTests = 0, kStatShadowTests, kStatPrimNodes, kStatPrimLeaves, kStatShadowNodes,
       kStatShadowLeaves, kStatHits, kStatOverflow, kStatShadowRays, kStatReflRays, kStatReflShadowRays, kStatN };
// WorkArgs::prof_acc holds the kStatN totals and then, at kProfRedo, the deferred second passes run
// (k_trace's redone blocks, the split kernels' redone items: mirt_profile.redo_items)
constexpr int kProfRedo = kStatN, kProfN = kStatN + 1;
constexpr int kQueues = 3;
__host__ __device__ constexpr int cnt_queue(int q, int s) { return (q * kQShards + s) * kLine; }
__host__ __device__ constexpr int cnt_hits(int s) { return (kQueues * kQShards + s) * kLine; }
__host__ __device__ constexpr int cnt_stat(int k, int s) {
    return ((kQueues + 1) * kQShards + k * kStatShards + s) * kLine;
}
// done(s), s < kStatShards: workgroups of the frame's last kernel finished per shard;
// done(kStatShards): shards finished (two levels keep every same-address count <= 64).
// pdone(q): primary blocks of shard q finished (k_trace).
__host__ __device__ constexpr int cnt_done(int s) {
    return ((kQueues + 1) * kQShards + kStatN * kStatShards + s) * kLine;
}
__host__ __device__ constexpr int cnt_pdone(int q) {
    return ((kQueues + 1) * kQShards + kStatN * kStatShards + kStatShards + 1 + q) * kLine;
}
constexpr int kCntN = ((kQueues + 2) * kQShards + kStatN * kStatShards + kStatShards + 1) * kLine;
typedef unsigned long long cnt_t;

// Block frustum pre-test of one-object frames (kernels.hip block_frustum).  A primary
// ray of pixel (i, j) has direction fwd + left s_i + up t_j (tracer.go:19-21), so a ray
// can only meet a root child box if (s_i, t_j) lies in the box's projection onto that
// (s, t) plane.  The host projects each root child box per frame in fp64 and rounds the
// rectangle outward with a relative margin of 2^-18; the kernel tests a block's range of
// s and t against the 8 rectangles.
struct FrustumArgs {
    float rect[8][4];      // per root child: s_lo, s_hi, t_lo, t_hi (empty child: an empty rectangle)
    double sA, sB, tA, tB; // tracer.go:19-20 offsets as affine maps: column i ~ sB - sA i, row j ~ tB - tA j
    uint32_t on;           // one object, culling on, bounded camera, W, H >= 2
    uint32_t ocert_n;      // FrameRec::ocert quads in use (0..kOcertQuads)
};
constexpr uint32_t kOcertQuads = 2;
// Object-box certificate of the primary blocks: per quad, four half-planes
// a s + b t >= c of the (s, t) plane, the projection of one face of the object's box shrunk by
// a margin.  A primary ray whose direction lies in one passes the reference's Box.Intersect of
// that box through that face's plane (tracer.go:32), so a block whose four corner directions
// all lie in one quad skips the object's gate.  (In FrameRec only: the kernarg block is full.)
struct ObjCert {
    float h[kOcertQuads][4][3];
};

// One frame of a k_trace launch (a launch traces up to kMaxFrames frames that share the mesh,
// object count, light count and options; the kernel takes FrameArgs from the first frame's).
constexpr uint32_t kMaxFrames = 8;
struct alignas(16) FrameRec {
    FrameArgs fa;
    OutPlanes out;
    FrustumArgs fr;
    ObjCert ocert;
    XferArgs xf;
    // Blocks with no pixel in [live[0], live[2]) x [live[1], live[3]) are not traced: every
    // ray of such a block misses, and the caller either cleared their outputs (a frame
    // group's whole-screen planes, launch_fill_planes) or never reads them (a share's packed
    // plane, of which k_pack_rect sends only the hit rectangle).  {0, 0, W, H}: every block.
    uint32_t live[4];
};
// k_trace's first argument: the launch's records, read in place from the kernarg segment.
struct FrameRecs {
    FrameRec r[kMaxFrames];
};

// Per-frame work description shared by the primary, shadow and shade kernels.
struct WorkArgs {
    const BlockDesc* blocks;
    uint32_t nblocks;
    uint32_t per_shard;    // BlockDesc entries per shard (ceil(nblocks / kQShards))
    uint32_t hit_cap;      // records per hit region (multiple of 64)
    HitRec* hits;          // kQShards regions of hit_cap records
    uint32_t* litw;        // per hit slot: bit l = light l reaches the hit (atomicOr by k_shadow)
    uint32_t* blkdone;     // per 64-slot hit block: lights finished (the last one shades the block)
    uint32_t wg_cap;       // k_trace: hit slots per workgroup region (chunks of 64)
    uint32_t bounces;      // configs[4] reflection extension (mirt_frame.max_bounces), 0 = off
    double* dir0;          // bounces: per hit slot, the primary ray direction (3 doubles)
    double* ph0;           // bounces: per hit slot, phong of the primary hit (3 doubles)
    // bounces: levels 1..bounces of each slot's chain, level-major ([lv - 1][slot][kReflD]):
    // the level's phong r, g, b and its obj | mat << 32 bits (k_reflect folds them innermost
    // first)
    double* refl;
    uint64_t refl_stride;  // slots per level
    // bounces, k_shadow's phong: slot s's colour goes to ph_out + ps * ph_stride with ps = s, or
    // ps = the record's `out` (the origin slot of a bounce level's record, ph_by_origin)
    double* ph_out;
    uint32_t ph_stride, ph_by_origin;
    // k_shadow's region hit counts and queue tickets (cnt_hits, cnt_queue; nullptr: `counters`):
    // a bounce level's records have counters of their own, its statistics go to `counters`
    cnt_t* qcounters;
    cnt_t* counters;
    cnt_t* counters_next;  // the other set: zeroed by k_primary for the next frame
    FrustumArgs fr;
    uint32_t dynamic;      // kDyn* bits: kernels that take work from the sharded queues (else static)
    uint32_t timeline_cap; // records the timeline buffer holds per kernel
    uint64_t* timeline;    // MIRT_OPT_TIMELINE: 8 x u64 per wave (mirt.h), else nullptr
    cnt_t* summary;        // kStatN totals of this frame (written by k_shade's last workgroup)
    cnt_t* prof_acc;       // kStatN running totals while profiling, else nullptr
    const FrameRec* frames;  // unused (k_trace reads its records from the kernarg segment)
    uint32_t nframes;
    uint32_t nblocks_frame;  // nblocks = nframes * nblocks_frame; the table describes one frame
    // view tables (k_trace, one-object frames, nullptr: none): frame f, view v at
    // views + (f * nviews + v) * nleaves, its header at view_heads[f * nviews + v]
    union {
        ViewLeaf* views;
        // split kernels (k_primary, k_shadow, k_bounce; never with view tables): their deferred
        // second passes, [0] workgroups done, [1] entries, then two words per entry
        uint32_t* split_redo;
    };
    ViewHead* view_heads;
    uint32_t nviews;         // 1 + lights
    uint32_t view_leaves;    // leaves per table
    // k_trace's queue order: per block of the table, the primary trace time of its last
    // frame on this slot (units of 64 shader cycles, 0 = unknown); blocks that took long go
    // first (order only: every block is traced the same way)
    uint16_t* block_cost;
    uint32_t view_tag;       // this launch's tag (nonzero, differs from the slot's previous launch)
    uint32_t view_pad;
    // k_trace (one-launch frames): bgcnt = the deferred second passes' list ([0] count, then
    // f << 28 | block entries) and bmap = a flag per block of the launch (zero between launches).
    // bounce waves (reflection frames without MIRT_OPT_REFLECT_CHAINS): per linear block of the table, its hit chunk
    // ((slot / 64 + 1) << 7 | hits; 0: none), written by k_primary (zeroed per frame), and the
    // hits per group of kPackGroup blocks (k_pack's prefix sums)
    uint32_t* bmap;
    uint32_t* bgcnt;
    // split kernels' primary hit chunks (k_primary without a ring; nullptr: none): per 64-slot
    // chunk, the ballot of its lanes that hit.  A missed lane's record, lit word and direction
    // are then never written (its lines stay clean): the chunk's readers (k_shadow at level 0,
    // k_pack at level 0, k_refl_fold) take validity from the mask instead of the record's obj.
    uint64_t* hmask;
    // k_primary: FrameRec::live of its frame (a block with no pixel inside is not traced: the
    // caller's planes already hold its miss values, as for k_trace)
    uint32_t live[4];
};
constexpr uint32_t kPackGroup = 64;  // source chunks per k_pack workgroup (and per counted group)
// Reflections in waves of bounces (configs[4] extension, kernels.hip k_bounce): level lv's
// hit records form region sets like the primary's (kQShards regions of hit_cap slots, region
// q holding cnt_hits(q) records of its counters, packed from the front), each record's `out`
// the origin slot (the primary hit slot whose chain it continues).
struct BounceArgs {
    const HitRec* in;       // level lv - 1 in region layout (k_pack); `out` = the origin slot
    const double* in_dir;   // per input slot: the ray that reached the hit (3 doubles)
    const cnt_t* in_cnt;    // the input's region counts
    HitRec* out;            // level lv's hits, at the input's slots (obj = kNoHit: none)
    double* out_dir;
    uint32_t* src;          // per input chunk j (region-major order): (slot / 64 + 1) << 7 | hits
    uint32_t* gcnt;         // hits per group of kPackGroup input chunks (zeroed before)
    uint32_t* chain;        // per origin slot: levels with a phong value | missed << 8
    uint32_t level;
    uint32_t pad;
};
// k_pack: a bounce level's records compacted in source-chunk order (the screen's block
// order), split evenly over the kQShards regions (region r: positions [r per, (r + 1) per)).
// The camera's part of FrameArgs (tracer.go:15-22 pixelToPoint): k_pack at level 0 makes each
// primary hit's ray direction again from its pixel, with k_primary's own operations.
struct RayGen {
    double cam[3], fwd[3], left[3], up[3];
    double phw, phh;
    int32_t halfW, halfH;
};
struct PackArgs {
    const HitRec* in;       // the source slots (level 0: the primary hit slots)
    const double* in_dir;   // the rays that reached them (level 0, nullptr: made from the pixel, rg)
    const uint32_t* src;    // source chunks in order: (slot / 64 + 1) << 7 | records (0: none)
    const uint32_t* gcnt;   // records per group of kPackGroup source chunks
    const cnt_t* in_cnt;    // level >= 1: the region counts of the chunks' level (their number); else null
    uint32_t nsrc;          // level 0: entries of src (the block table)
    uint32_t level0;        // 1: records are primary hits (their origin = their slot)
    HitRec* out;
    double* out_dir;
    uint32_t* out_litw;
    uint32_t* out_blkdone;
    cnt_t* out_cnt;         // region counts of the packed level (cnt_hits)
    const uint64_t* in_hmask;  // level 0 with WorkArgs::hmask: the source chunks' hit ballots
    RayGen rg;              // level 0 without in_dir: the frame's camera
};
constexpr int kTimelineRec = 8;
constexpr int kReflD = 4;  // doubles per slot and level of WorkArgs::refl
// WorkArgs::dynamic: kernels whose waves take work items dynamically (primary: LDS tickets
// within the workgroup; shadow / reflect: the sharded device queues).
enum { kDynPrimary = 1, kDynShadow = 2, kDynReflect = 4 };
constexpr int kBlkQ = 256;  // primary block descriptors staged in LDS per batch
// k_trace hit-chunk ring positions per workgroup (kernels.hip ring_take; 0: every chunk of
// a batch gets a fresh position); a workgroup's region holds kHitRing + its blocks' chunks.
#ifndef MIRT_HIT_RING
#define MIRT_HIT_RING 8
#endif
constexpr uint32_t kHitRing = MIRT_HIT_RING;
static_assert(kHitRing <= 32, "the ring's free positions are one 32-bit LDS word");

// Arbitrary-ray inputs/outputs for mirt_trace_rays.
struct RayIO {
    const double* orig;
    const double* dir;
    uint8_t* ok;
    double* hit;
    double* normal;
    int32_t* face;
    int32_t* object;
    uint32_t n;
};

// Device builder of one light table (kernels.hip k_light_table; lighttab.hpp records).
struct LightTabArgs {
    const double* tri;  // the mesh's P1, E1, E2 records in BVH order
    uint32_t n, nl;     // triangles, lights
    double scale;       // the mesh's largest |coordinate|
    double pos[3];      // the object's position
    double lpos[MIRT_MAX_LIGHTS][3];
    float* out;         // nl * n * kLtD floats, light-major
};
hipError_t launch_light_table(const LightTabArgs& a, hipStream_t s);
hipError_t launch_primary(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, int grid, uint32_t opts,
                          hipStream_t s);
hipError_t launch_shadow(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, int grid, uint32_t opts,
                         hipStream_t s);
struct FusedCopy;
hipError_t launch_trace(const FrameRecs& recs, const WorkArgs& wa, const FusedCopy& fc, int grid, uint32_t opts,
                        hipStream_t s);
hipError_t launch_rays(const FrameArgs& fa, const RayIO& io, int grid, uint32_t opts, hipStream_t s);
hipError_t launch_reflect(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, int grid, uint32_t opts,
                          hipStream_t s);
hipError_t launch_pack(const WorkArgs& wa, const PackArgs& pa, int grid, hipStream_t s);
bool bounce_shades();  // k_bounce traces each level's shadow rays itself (MIRT_BOUNCE_SHADE)
hipError_t launch_bounce(const FrameArgs& fa, const WorkArgs& wa, const BounceArgs& ba, int grid, uint32_t opts,
                         hipStream_t s);
hipError_t launch_refl_fold(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, const uint32_t* chain,
                            int grid, hipStream_t s);
hipError_t read_diag_counters(uint64_t* out, uint32_t n);  // MIRT_DIAG builds (zeros otherwise)
hipError_t launch_debug_fp64(int op, uint32_t n, const double* a, const double* b, double* out, hipStream_t s);
struct RectJobs {  // k_pack_rect / k_unpack_rect (and its region check): per frame of a batch
    const uint32_t* src[kMaxFrames];  // pack: the rgbv plane; unpack/check: the gathered regions
    uint32_t* dst[kMaxFrames];        // pack: the transfer buffer
    OutPlanes out[kMaxFrames];        // unpack: the framebuffer
    uint32_t rect[kMaxFrames][4];     // hit rectangle x0, y0, x1, y1 (half-open)
    uint32_t tag[kMaxFrames];         // the frame's trailer tag (transfer_tag of its index)
    uint8_t* bad[kMaxFrames];         // check: one byte per region, 1 = trailer missing or wrong
    // unpack: the framebuffer columns [ucol[f][0], ucol[f][1]) are written (the frame's hit
    // rectangle and the one its slot held before: every other column already holds misses)
    uint32_t ucol[kMaxFrames][2];
};
// Every transfer buffer ends with a two-word trailer written by k_pack_rect right after
// the data: {tag of the frame, words of data}.  The root checks it in every gathered
// region before the unpack, so a transfer of the wrong size, a stale one or one that never
// arrived fails loudly (mirt_group: MIRT_E_PEER naming the rank) instead of corrupting the
// frame.
constexpr uint32_t kTrailerWords = 2;
__host__ __device__ constexpr uint32_t transfer_tag(uint64_t frame) {
    return 0x6d697274u ^ (uint32_t)(frame * 0x9e3779b1u) ^ (uint32_t)(frame >> 32);
}
// One rank's region of the gathered plane: its tiles are d_unpack[first, first + count).
struct RegionDesc {
    uint32_t first, count;
};
// Device framebuffer -> pinned host framebuffer, the pixels of one rectangle per frame
// (mirt_group_set_host_output): the kernel stores straight into host memory over PCIe.
// Per column the kernel copies only the rows between the first and last hit of this frame
// and of the frame the host slot held before (spans: per slot and column, first | end << 16;
// every other pixel is a miss, i.e. zero, on both sides).
struct HostCopyJobs {
    const uint8_t* rgb8[kMaxFrames];
    const uint8_t* valid[kMaxFrames];
    uint8_t* hrgb8[kMaxFrames];
    uint8_t* hvalid[kMaxFrames];
    uint32_t* spans[kMaxFrames];   // the slot's W spans (device)
    uint32_t rect[kMaxFrames][4];  // columns to visit: x0, -, x1, - (half-open)
    uint32_t cur[kMaxFrames][4];   // this frame's hit rectangle (where to look for hits)
};
// k_trace's third argument: a host copy of an EARLIER launch's frames on the same stream (the
// frame group's fused host output, mirt.cpp group_flush), done by the launch's first waves
// (n = 0: none).
struct FusedCopy {
    HostCopyJobs jobs;
    uint32_t n;
    uint32_t H;
};

// Miss values into whole planes before a frame is traced (mirt_group, whole screen): per
// frame up to kFillPlanes byte ranges, each set to one byte value (0, or 0xff for the int32
// -1 of face / object).
constexpr int kFillPlanes = 6;
struct FillJobs {
    uint8_t* ptr[kMaxFrames][kFillPlanes];
    uint64_t bytes[kMaxFrames][kFillPlanes];
    uint8_t value[kMaxFrames][kFillPlanes];
};
hipError_t launch_fill_planes(const FillJobs& jobs, uint32_t nframes, uint64_t max_bytes, hipStream_t s);
hipError_t launch_copy_rect_host(const HostCopyJobs& jobs, uint32_t nframes, uint32_t H, uint32_t max_cols,
                                 hipStream_t s);
hipError_t launch_pack_rect(const TileDesc* tiles, uint32_t ntiles, const RectJobs& jobs, uint32_t nframes,
                            hipStream_t s);
// regions != nullptr: the launch also checks every region's trailer (check_region,
// bad[f][r]) before its frames are used
hipError_t launch_unpack_rect(const TileDesc* tiles, uint32_t ntiles, uint64_t max_tile_px, uint32_t H, uint64_t cap,
                              const RegionDesc* regions, uint32_t nregions, const RectJobs& jobs, uint32_t nframes,
                              hipStream_t s);
hipError_t launch_unpack(const TileDesc* tiles, uint32_t ntiles, uint64_t max_tile_px, uint32_t H, const OutPlanes& src,
                         const OutPlanes& dst, hipStream_t s);

}  // namespace mirt
