// mirt.cpp — host side of libmirt.so: context, mesh upload, per-call slots, launches.
//
// Re-entrancy: gRPC serves each BulkTrace in its own goroutine, so any
// number of threads may call mirt_trace_* concurrently on one context with different
// frames.  Each call takes a "slot" (HIP stream + workspace + events) from a pool under
// a mutex and returns it afterwards; meshes are immutable after upload.  hipSetDevice is
// called on every entry because cgo calls can land on any OS thread.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <chrono>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/mirt.h"
#include "gomath.hpp"
#include "mirt_internal.hpp"
#include "lighttab.hpp"
#include "bvh.hpp"
#include "host_internal.hpp"

using namespace mirt;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    return fail(MIRT_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

struct MeshDev {
    double* tri = nullptr;
    double* vnrm = nullptr;
    uint32_t* fmat = nullptr;
    uint32_t* fidx = nullptr;
    Bvh8Dev* nodes = nullptr;
    double* mats = nullptr;
    LeafBox* leaves = nullptr;  // the BVH's leaves (view tables)
    uint32_t nleaves = 0;
    double center[3] = {0, 0, 0};  // bounding-box centre
    uint32_t ntri = 0, nmat = 0, nnodes = 0, depth = 0;
    double scale = 1.0;  // max |coordinate| of the mesh (culling tolerances)
    Bvh8Node root{};     // host copy of the BVH root (frustum pre-test rectangles)
    // Go math.Min / math.Max of every vertex coordinate (+inf / -inf without vertices): an
    // object's box (object.go:31-59) is a function of its position and these (object_box)
    double vmin[3] = {INFINITY, INFINITY, INFINITY}, vmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool has_normals = false;
    bool live = false;
};

// Device workspace of one in-flight call.
// -DMIRT_HOST_TIMERS (diagnostic build): host time per phase of mirt_trace_frame,
// printed when the group is destroyed (tools/group_probe.py with MIRT_LIB).
#ifdef MIRT_HOST_TIMERS
#include <chrono>
static double g_ht[16];
static std::chrono::steady_clock::time_point g_ht_t;
#define HT_START() (g_ht_t = std::chrono::steady_clock::now())
#define HT(i)                                                                                   \
    do {                                                                                        \
        auto n_ = std::chrono::steady_clock::now();                                             \
        g_ht[i] += std::chrono::duration<double, std::micro>(n_ - g_ht_t).count();             \
        g_ht_t = n_;                                                                            \
    } while (0)
#else
#define HT_START() ((void)0)
#define HT(i) ((void)0)
#endif

struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool pending = false;
    bool dedicated = false;  // a frame group's slot: ordered by its stream, no done event needed
    HitRec* hits = nullptr;
    size_t hits_cap = 0;
    uint32_t* litw = nullptr;
    size_t litw_cap = 0;
    uint32_t* blkdone = nullptr;
    size_t blkdone_cap = 0;
    uint64_t* hmask = nullptr;  // split kernels: per primary hit chunk, its hit ballot (WorkArgs::hmask)
    size_t hmask_cap = 0;
    double* dir0 = nullptr;   // configs[4] reflections: primary direction per hit slot
    size_t dir0_cap = 0;
    double* ph0 = nullptr;    // configs[4] reflections: phong of the primary hit per slot
    size_t ph0_cap = 0;
    double* refl = nullptr;   // configs[4] reflections: per level and slot, phong + obj|mat
    size_t refl_cap = 0;
    // configs[4] bounce waves (k_bounce): two level buffers used alternately, the levels'
    // region counters, per origin slot the chain state
    HitRec* lhits[2] = {nullptr, nullptr};
    size_t lhits_cap[2] = {0, 0};
    double* ldir[2] = {nullptr, nullptr};
    size_t ldir_cap[2] = {0, 0};
    uint32_t* llitw[2] = {nullptr, nullptr};
    size_t llitw_cap[2] = {0, 0};
    uint32_t* lblk[2] = {nullptr, nullptr};
    size_t lblk_cap[2] = {0, 0};
    cnt_t* lcnt = nullptr;    // [bounces][kCntN]
    size_t lcnt_cap = 0;
    uint32_t* chain = nullptr;
    size_t chain_cap = 0;
    // bounce waves: a level's hits at its input's slots (k_bounce), the chunk descriptors of
    // k_pack's walk, and the block table's hit chunks (WorkArgs::bmap)
    HitRec* shits = nullptr;
    size_t shits_cap = 0;
    double* sdir = nullptr;
    size_t sdir_cap = 0;
    uint32_t* ssrc = nullptr;
    size_t ssrc_cap = 0;
    uint32_t* bmap = nullptr;
    size_t bmap_cap = 0;
    // k_trace's deferred second passes (WorkArgs::bmap / bgcnt in one-launch frames): [0] the
    // count, then kMaxFrames x nblocks list entries, then as many per-block flags; zero between
    // launches (the launch's last workgroup clears what it used)
    uint32_t* redo = nullptr;
    size_t redo_cap = 0;
    // the split kernels' deferred second passes (WorkArgs::split_redo), zero between launches
    uint32_t* sredo = nullptr;
    size_t sredo_cap = 0;
    uint32_t* gcnt = nullptr;  // [bounces + 1][groups]: records per group of kPackGroup source chunks
    size_t gcnt_cap = 0;
    uint16_t* cost = nullptr; // per block of the table: last primary trace time (WorkArgs::block_cost)
    size_t cost_cap = 0;
    cnt_t* counters = nullptr;
    TileDesc* d_tiles = nullptr;
    TileDesc* h_tiles = nullptr;  // pinned staging
    size_t tiles_cap = 0, h_tiles_cap = 0;
    // per-block work items of the last tile list traced on this slot (reused while the
    // caller keeps sending the same list: no host rebuild, no upload)
    BlockDesc* d_blocks = nullptr;
    BlockDesc* h_blocks = nullptr;  // pinned staging
    size_t blocks_cap = 0, h_blocks_cap = 0;
    std::vector<mirt_tile> blocks_key;
    std::vector<TileDesc> unpack_key;  // tile list of the last unpack (device copy in d_tiles)
    uint32_t unpack_key_H = 0;
    uint32_t blocks_W = 0, blocks_H = 0, nblocks = 0, per_shard = 0;
    // pixelToPoint per column / per row (tracer.go:19-20), cached per (fov, W, H)
    cnt_t* summary = nullptr;     // kStatN totals of the last frame (device)
    cnt_t* h_summary = nullptr;   // pinned copy for mirt_stats
    FrameRec* h_frames = nullptr; // kMaxFrames records of the next k_trace launch (its kernel argument)
    ViewLeaf* views = nullptr;    // view tables of the next k_trace launch (WorkArgs::views)
    size_t views_cap = 0;
    ViewHead* view_heads = nullptr;
    size_t view_heads_cap = 0;
    uint32_t view_tag = 0;  // the last launch's WorkArgs::view_tag
    bool dirty = false;           // counters possibly non-zero (a frame stopped half-way)
    uint32_t parity = 0;          // counter set of the next frame (two sets of kCntN)
    // device-side outputs for the host-buffer API
    void* out_buf = nullptr;
    size_t out_cap = 0;
};

struct ProfRec {
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    uint64_t pixels = 0;
    uint32_t frames = 1;
};

}  // namespace

struct mirt_ctx {
    int device = 0;
    int cus = 256;
    // k_trace / k_primary grid: at least this many 8x8 blocks per workgroup (small tile
    // lists launch fewer, fuller workgroups so frames in flight can share the chip)
    uint32_t min_blocks_per_wg = 32;
    uint32_t max_workgroups = 0;  // 0: two per CU
    std::mutex mu;
    std::vector<MeshDev> meshes;
    std::vector<std::unique_ptr<Slot>> slots;
    std::vector<Slot*> free_slots;
    uint32_t flags = 0;
    bool profiling = false;
    std::vector<ProfRec> prof_pending;
    std::vector<ProfRec> prof_free;
    cnt_t* prof_acc = nullptr;     // kProfN device totals accumulated while profiling
    uint64_t* timeline = nullptr;  // MIRT_OPT_TIMELINE buffer (2 kernels x timeline_cap waves)
    uint32_t timeline_cap = 0;
    // Light tables of one-object frames (light_table): an LRU cache of device tables keyed by
    // (mesh, object position, light set), built on the device on the stream of the first frame
    // that reads them (lt_launch), evicted only once every stream that read them has passed
    // an event recorded at eviction (lt_dead), their buffers reused for the next build.
    struct LightTab {
        uint32_t mesh = 0, nl = 0;
        double pos[3] = {0, 0, 0};
        double lpos[MIRT_MAX_LIGHTS][3] = {};
        float* d = nullptr;
        size_t bytes = 0;
        bool built = false;             // k_light_table enqueued (on `built_on`)
        hipStream_t built_on = nullptr;
        hipEvent_t ready = nullptr;     // recorded after the build
        bool ready_seen = false;        // `ready` has completed
        uint64_t last_use = 0;          // lt_clock at the last light_table() returning it
        // frame records holding the table that have not been launched yet (light_table() takes
        // a pin, lt_unpin gives it back after the launch or on the record's error path): a
        // pinned table is never evicted
        uint32_t pins = 0;
        // per stream whose frames read it: an event re-recorded after each such launch (the
        // library owns the events, so a reader stream may be destroyed meanwhile)
        std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
    };
    struct DeadTab {
        float* d = nullptr;
        size_t bytes = 0;
        std::vector<hipEvent_t> evs;    // every reader stream's last launch that read it
    };
    std::mutex lt_mu;
    std::vector<std::unique_ptr<LightTab>> ltabs;
    std::vector<DeadTab> lt_dead;
    std::vector<hipEvent_t> lt_events;  // pool
    size_t ltab_bytes = 0;              // live + dead tables
    size_t lt_cap = (size_t)4 << 30;    // mirt_set_light_cache
    uint64_t lt_clock = 0;
    uint64_t lt_stat[6] = {0, 0, 0, 0, 0, 0};  // builds, hits, evictions, fallbacks, reused buffers, entries
    // frame groups on this context: mirt_mesh_release launches their staged (open or held)
    // batches before it frees a mesh their records point at
    std::mutex groups_mu;
    std::vector<mirt_group*> groups;
};

namespace {

void mesh_free(MeshDev& m) {
    for (void* p : {(void*)m.tri, (void*)m.vnrm, (void*)m.fmat, (void*)m.fidx, (void*)m.nodes, (void*)m.mats,
                    (void*)m.leaves})
        if (p) (void)hipFree(p);
    m = MeshDev();
}

template <class T>
int dev_grow(T*& p, size_t& cap, size_t need) {
    if (need <= cap) return MIRT_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t n = std::max(need, (size_t)1);
    hipError_t e = hipMalloc((void**)&p, n * sizeof(T));
    if (e != hipSuccess) return fail(MIRT_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    cap = n;
    return MIRT_OK;
}

// Up to this many slots are created before a caller blocks on a busy one, so a caller
// enqueueing frames back to back runs ahead of the GPU instead of waiting per frame.  (32 for a
// box's concurrent orders: slower, each new slot's buffers are allocated inside the run,
// profiles/r06_box_lines.txt.)
constexpr size_t kMaxIdleBlockSlots = 8;

// First use of a slot: its event and counters.  The slot's own stream is created only by
// the synchronous entry points that use it (slot_stream): every stream takes one of the
// process's few hardware queues, which the caller's streams of frames in flight need.
int slot_init(Slot* s) {
    if (s->done) return MIRT_OK;
    HIP_TRY(hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
    HIP_TRY(hipMalloc((void**)&s->counters, 2 * kCntN * sizeof(cnt_t)));
    HIP_TRY(hipMalloc((void**)&s->summary, kStatN * sizeof(cnt_t)));
    HIP_TRY(hipHostMalloc((void**)&s->h_summary, kStatN * sizeof(cnt_t)));
    HIP_TRY(hipHostMalloc((void**)&s->h_frames, kMaxFrames * sizeof(FrameRec)));
    HIP_TRY(hipMemset(s->counters, 0, 2 * kCntN * sizeof(cnt_t)));
    return MIRT_OK;
}

void slot_free(Slot* s) {
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (void* p : {(void*)s->lhits[0], (void*)s->lhits[1], (void*)s->ldir[0], (void*)s->ldir[1], (void*)s->llitw[0],
                    (void*)s->llitw[1], (void*)s->lblk[0], (void*)s->lblk[1], (void*)s->lcnt, (void*)s->chain,
                    (void*)s->shits, (void*)s->sdir, (void*)s->ssrc, (void*)s->bmap, (void*)s->gcnt, (void*)s->redo, (void*)s->sredo})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)s->hits, (void*)s->litw, (void*)s->blkdone, (void*)s->hmask, (void*)s->dir0, (void*)s->ph0, (void*)s->refl,
                    (void*)s->cost, (void*)s->counters, (void*)s->d_tiles, (void*)s->d_blocks, (void*)s->summary, s->out_buf,
                    (void*)s->views, (void*)s->view_heads})
        if (p) (void)hipFree(p);
    if (s->h_blocks) (void)hipHostFree(s->h_blocks);
    if (s->h_tiles) (void)hipHostFree(s->h_tiles);
    if (s->h_summary) (void)hipHostFree(s->h_summary);
    if (s->h_frames) (void)hipHostFree(s->h_frames);
    if (s->done) (void)hipEventDestroy(s->done);
    if (s->stream) (void)hipStreamDestroy(s->stream);
}

// tiles (optional): the call's tile list; a free slot whose cached block table is that list's
// is preferred (concurrent BulkTrace orders of different rectangles keep their tables)
int slot_acquire(mirt_ctx* c, Slot*& out, const mirt_tile* tiles = nullptr, uint32_t n = 0) {
    {
        std::lock_guard<std::mutex> g(c->mu);
        out = nullptr;
        // prefer a free slot whose previous asynchronous work has already completed, and among
        // those one that holds this tile list's block table
        size_t pick = c->free_slots.size();
        for (size_t i = 0; i < c->free_slots.size(); ++i) {
            Slot* s = c->free_slots[i];
            if (!s->pending || hipEventQuery(s->done) == hipSuccess) {
                s->pending = false;
                const bool same = tiles && s->blocks_key.size() == n &&
                                  memcmp(s->blocks_key.data(), tiles, sizeof(mirt_tile) * n) == 0;
                if (pick == c->free_slots.size()) pick = i;
                if (same || !tiles) {
                    pick = i;
                    break;
                }
            }
        }
        if (pick < c->free_slots.size()) {
            out = c->free_slots[pick];
            c->free_slots.erase(c->free_slots.begin() + (long)pick);
        }
        if (!out && (c->free_slots.empty() || c->slots.size() < kMaxIdleBlockSlots)) {
            c->slots.emplace_back(new Slot());
            out = c->slots.back().get();
        }
        if (!out) {  // every slot busy: take the oldest free one and wait for it below
            out = c->free_slots.front();
            c->free_slots.erase(c->free_slots.begin());
        }
    }
    Slot* s = out;
    int r = slot_init(s);
    if (r != MIRT_OK) return r;
    // previous asynchronous use of this slot's staging/workspace must be finished
    if (s->pending) {
        HIP_TRY(hipEventSynchronize(s->done));
        s->pending = false;
    }
    return MIRT_OK;
}

int slot_stream(Slot* s, hipStream_t& out) {
    if (!s->stream) HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    out = s->stream;
    return MIRT_OK;
}

// Device + pinned host tile descriptors, grow-only (the slot is idle when this runs).
int tiles_grow(Slot* sl, uint32_t n) {
    int r = dev_grow(sl->d_tiles, sl->tiles_cap, n);
    if (r != MIRT_OK) return r;
    if (sl->h_tiles_cap < n) {
        if (sl->h_tiles) (void)hipHostFree(sl->h_tiles);
        sl->h_tiles = nullptr;
        sl->h_tiles_cap = 0;
        size_t cap = std::max<size_t>(n, 64);
        HIP_TRY(hipHostMalloc((void**)&sl->h_tiles, sizeof(TileDesc) * cap));
        sl->h_tiles_cap = cap;
    }
    return MIRT_OK;
}

void slot_release(mirt_ctx* c, Slot* s) {
    std::lock_guard<std::mutex> g(c->mu);
    c->free_slots.push_back(s);
}

struct SlotGuard {
    mirt_ctx* c;
    Slot* s;
    ~SlotGuard() {
        if (s) slot_release(c, s);
    }
};

// shared/state/util.go:7 boundEpsilon; rtreego.NewRect(p, len) keeps p and p + len, and
// geom.NewBox (box.go:21-26) rebuilds MaxCorner as p + ((p + len) - p).
constexpr double kBoundEpsilon = 0.0001;
static void rect_corners(const double lo[3], const double hi[3], double out[6]) {
    for (int k = 0; k < 3; ++k) {
        const double len = go_max(hi[k] - lo[k], kBoundEpsilon);
        const double q = lo[k] + len;
        out[k] = lo[k];
        out[3 + k] = lo[k] + (q - lo[k]);
    }
}
// mesh.go:30-50 face.Bounds (math.Min(a, math.Min(b, c)) per axis), as NewBox corners
static void face_box(const double* p1, const double* p2, const double* p3, double out[6]) {
    double lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = go_min(p1[k], go_min(p2[k], p3[k]));
        hi[k] = go_max(p1[k], go_max(p2[k], p3[k]));
    }
    rect_corners(lo, hi, out);
}
// object.go:31-59 Object.Bounds: min / max of pos and pos + v over the mesh's vertices.
// Rounding is monotonic, so min_v fl(pos + v) = fl(pos + min_v v) (and the Go signed-zero
// rule agrees: -0 + -0 is the only sum that is -0); the loop reduces to the mesh's vmin/vmax.
static void object_box(const double pos[3], const double vmin[3], const double vmax[3], double out[6]) {
    double lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = go_min(pos[k], pos[k] + vmin[k]);
        hi[k] = go_max(pos[k], pos[k] + vmax[k]);
    }
    rect_corners(lo, hi, out);
}
static void vertex_minmax(const double* v, uint32_t nv, double vmin[3], double vmax[3]) {
    for (int k = 0; k < 3; ++k) {
        vmin[k] = INFINITY;
        vmax[k] = -INFINITY;
    }
    for (uint32_t i = 0; i < nv; ++i)
        for (int k = 0; k < 3; ++k) {
            vmin[k] = go_min(vmin[k], v[3 * (size_t)i + k]);
            vmax[k] = go_max(vmax[k], v[3 * (size_t)i + k]);
        }
}

int check_frame(const mirt_ctx* c, const mirt_frame* f) {
    if (!f) return fail(MIRT_E_INVALID, "frame is NULL");
    if (f->n_objects > MIRT_MAX_OBJECTS)
        return fail(MIRT_E_LIMIT, "n_objects > MIRT_MAX_OBJECTS (" + std::to_string(MIRT_MAX_OBJECTS) + ")");
    if (f->n_lights > MIRT_MAX_LIGHTS)
        return fail(MIRT_E_LIMIT, "n_lights > MIRT_MAX_LIGHTS (" + std::to_string(MIRT_MAX_LIGHTS) + ")");
    if (f->n_objects && !f->objects) return fail(MIRT_E_INVALID, "objects is NULL");
    if (f->n_lights && !f->lights) return fail(MIRT_E_INVALID, "lights is NULL");
    if (f->max_bounces > MIRT_MAX_BOUNCES)
        return fail(MIRT_E_LIMIT, "max_bounces > MIRT_MAX_BOUNCES (" + std::to_string(MIRT_MAX_BOUNCES) + ")");
    for (uint32_t i = 0; i < f->n_objects; ++i) {
        uint32_t id = f->objects[i].mesh_id;
        if (id >= c->meshes.size() || !c->meshes[id].live)
            return fail(MIRT_E_INVALID, "object " + std::to_string(i) + " names unknown mesh id " + std::to_string(id));
        // the kernels' Box.Intersect needs finite corners (an object box that overflows fp64
        // would make the reference's zero-weighted dot-product terms inf * 0 = NaN)
        double bx[6];
        object_box(f->objects[i].pos, c->meshes[id].vmin, c->meshes[id].vmax, bx);
        for (int k = 0; k < 6; ++k)
            if (std::isinf(bx[k]))
                return fail(MIRT_E_LIMIT, "object " + std::to_string(i) + "'s bounding box overflows fp64");
    }
    return MIRT_OK;
}

void fill_args(const mirt_ctx* c, const mirt_frame* f, uint32_t W, uint32_t H, FrameArgs& fa, uint64_t& tris) {
    memset(&fa, 0, sizeof(fa));
    const mirt_camera& cam = f->camera;
    for (int k = 0; k < 3; ++k) {
        fa.cam[k] = cam.pos[k];
        fa.fwd[k] = cam.forward[k];
        fa.left[k] = cam.left[k];
        fa.up[k] = cam.up[k];
    }
    // tracer.go:16-18: halfWidth, halfHeight := width/2, height/2 (integer division);
    // projHalfHeight := projHalfWidth * float64(height) / float64(width)
    fa.phw = cam.proj_half_width;
    fa.phh = fa.phw * (double)H / (double)W;
    fa.W = (int32_t)W;
    fa.H = (int32_t)H;
    fa.halfW = (int32_t)(W / 2);
    fa.halfH = (int32_t)(H / 2);
    fa.n_objects = f->n_objects;
    fa.n_lights = f->n_lights;
    fa.flags = c->flags;
    tris = 0;
    for (uint32_t i = 0; i < f->n_objects; ++i) {
        const MeshDev& m = c->meshes[f->objects[i].mesh_id];
        DevObject& o = fa.obj[i];
        o.m.tri = m.tri;
        o.m.vnrm = m.vnrm;
        o.m.fmat = m.fmat;
        o.m.fidx = m.fidx;
        o.m.nodes = m.nodes;
        o.m.leaves = m.leaves;
        o.m.nleaves = m.nleaves;
        o.m.depth = m.depth;
        // culling needs bounded coordinates (fp32 slab arithmetic); beyond 2^40 never cull
        o.m.cull_limit = (m.scale <= 0x1p40) ? 256.0 * m.scale : -1.0;
        o.m.mats = m.mats;
        o.m.ntri = m.ntri;
        o.m.has_normals = m.has_normals ? 1u : 0u;
        for (int k = 0; k < 3; ++k) o.pos[k] = f->objects[i].pos[k];
        object_box(o.pos, m.vmin, m.vmax, o.box);
        tris += m.ntri;
    }
    for (uint32_t l = 0; l < f->n_lights; ++l)
        for (int k = 0; k < 3; ++k) {
            fa.lpos[l][k] = f->lights[l].pos[k];
            fa.lcol[l][k] = f->lights[l].col[k];
        }
}

// The object-box certificate of the primary blocks (FrustumArgs::ocert).  A
// face of the object's box (Object.Bounds as NewBox corners, world space, the box tracer.go:32
// tests) whose four corners all lie in front of the camera projects onto a convex quad of the
// (s, t) plane; a primary ray whose direction lies inside it meets the face's plane at a point
// of the face, ahead of the camera, so the reference's Box.Intersect (box.go:29-68) accepts it
// through that plane.  The quad is shrunk by a margin far above every rounding involved (the
// kernel's pixelToPoint + Norm, the reference's dirScale and intersection point: ~2^-50 of
// the magnitudes of the camera, the box and the ray, against 2^-24 here), and its float
// half-planes by their own rounding, so a direction inside the shrunk quad passes exactly.
// The two faces with the largest quads are kept (the kernarg block holds two).
void object_cert(const FrameArgs& fa, const double R[3][3], FrustumArgs& fr, ObjCert& oc) {
    const double* bx = fa.obj[0].box;  // {MinCorner, MaxCorner}
    double big = 1.0;
    for (int k = 0; k < 3; ++k) big = std::max({big, std::fabs(fa.cam[k]), std::fabs(bx[k]), std::fabs(bx[3 + k])});
    // the screen's (s, t) extent
    const double S = std::fabs(fr.sB) + std::fabs(fr.sA) * 2.0 * fa.halfW, T = std::fabs(fr.tB) + std::fabs(fr.tA) * 2.0 * fa.halfH;
    struct Quad {
        double area = 0.0;
        float h[4][3];
    };
    Quad best[kOcertQuads];
    for (int a = 0; a < 3; ++a)
        for (int side = 0; side < 2; ++side) {
            const int b = a == 0 ? 1 : 0, cc = a == 2 ? 1 : 2;
            double st[4][2], zmin = INFINITY;
            bool ok = true;
            for (int k = 0; k < 4; ++k) {  // corners in cyclic order over the face's other two axes
                const int ub = (k == 1 || k == 2) ? 1 : 0, uc = k >= 2 ? 1 : 0;
                double X[3];
                X[a] = bx[3 * side + a] - fa.cam[a];
                X[b] = bx[3 * ub + b] - fa.cam[b];
                X[cc] = bx[3 * uc + cc] - fa.cam[cc];
                const double mag = std::max({std::fabs(X[0]), std::fabs(X[1]), std::fabs(X[2])});
                const double z = R[0][0] * X[0] + R[0][1] * X[1] + R[0][2] * X[2];
                if (!(z > 0x1p-20 * mag) || !(mag > 0.0)) {
                    ok = false;
                    break;
                }
                zmin = std::min(zmin, z);
                st[k][0] = (R[1][0] * X[0] + R[1][1] * X[1] + R[1][2] * X[2]) / z;
                st[k][1] = (R[2][0] * X[0] + R[2][1] * X[1] + R[2][2] * X[2]) / z;
            }
            if (!ok) continue;
            double area = 0.0, cs = 0.0, ct = 0.0;
            for (int k = 0; k < 4; ++k) {
                const double* p = st[k];
                const double* q = st[(k + 1) & 3];
                area += p[0] * q[1] - q[0] * p[1];
                cs += p[0] / 4;
                ct += p[1] / 4;
            }
            area = std::fabs(area) / 2;
            const double margin = 0x1p-24 * (1.0 + S + T) * (1.0 + big / zmin);
            Quad qd;
            qd.area = area;
            for (int k = 0; k < 4; ++k) {
                const double* p = st[k];
                const double* q = st[(k + 1) & 3];
                double na = q[1] - p[1], nb = -(q[0] - p[0]);
                if (na * (cs - p[0]) + nb * (ct - p[1]) < 0) {
                    na = -na;
                    nb = -nb;
                }
                const double len = std::sqrt(na * na + nb * nb);
                if (!(len > 0.0) || !std::isfinite(len)) {
                    ok = false;
                    break;
                }
                na /= len;
                nb /= len;
                const float fa_ = (float)na, fb_ = (float)nb;
                // n . (s, t) >= n . p + margin, with the float coefficients' own rounding added
                double c0 = na * p[0] + nb * p[1] + margin;
                c0 += 0x1p-22 * (std::fabs(na) * S + std::fabs(nb) * T + std::fabs(c0)) + 0x1p-60;
                qd.h[k][0] = fa_;
                qd.h[k][1] = fb_;
                qd.h[k][2] = detail::round_up(c0);
            }
            if (!ok || !(area > 0.0) || !std::isfinite(area)) continue;
            for (uint32_t q = 0; q < kOcertQuads; ++q)
                if (area > best[q].area) {
                    for (uint32_t r = kOcertQuads - 1; r > q; --r) best[r] = best[r - 1];
                    best[q] = qd;
                    break;
                }
        }
    fr.ocert_n = 0;
    for (uint32_t q = 0; q < kOcertQuads; ++q)
        if (best[q].area > 0.0) memcpy(oc.h[fr.ocert_n++], best[q].h, sizeof(best[q].h));
}

// Rectangles of the primary kernel's whole-block frustum pre-test (mirt_internal.hpp
// FrustumArgs).  With R the inverse of the basis matrix [fwd left up], a point X (object
// space, relative to the camera) lies on the ray of (s, t) at parameter z = R0.X > 0 iff
// s = R1.X / z and t = R2.X / z.  A box entirely in front of the camera (every corner at
// z > 2^-20 |X|) projects into the bounding rectangle of its corners' (s, t); a box
// entirely behind it (z < 0 everywhere: rays start at z = 0) is never met; anything else
// is always tested.  Hits lie inside the inflated boxes, and the margin
// covers the fp64 rounding of this projection and of the kernels' rays.
void frustum_args(const mirt_ctx* c, const mirt_frame* f, const FrameArgs& fa, FrustumArgs& fr, ObjCert& oc) {
    memset(&fr, 0, sizeof(fr));
    memset(&oc, 0, sizeof(oc));
    if (fa.n_objects != 1 || (c->flags & (MIRT_OPT_NO_FRUSTUM | MIRT_OPT_BRUTE_FORCE)) || fa.halfW < 1 ||
        fa.halfH < 1)
        return;
    const DevObject& ob = fa.obj[0];
    const MeshDev& md = c->meshes[f->objects[0].mesh_id];
    double o[3], far = 0.0, big = 0.0;
    for (int k = 0; k < 3; ++k) {
        o[k] = fa.cam[k] - ob.pos[k];
        far = std::max(far, std::fabs(o[k]));
        big = std::max({big, std::fabs(fa.cam[k]), std::fabs(ob.pos[k])});
    }
    // culling off, or a camera so far out that the rays' own rounding could approach the margin
    if (!(far <= ob.m.cull_limit) || !(big <= 0x1p30)) return;
    const double F[3] = {fa.fwd[0], fa.fwd[1], fa.fwd[2]}, L[3] = {fa.left[0], fa.left[1], fa.left[2]},
                 U[3] = {fa.up[0], fa.up[1], fa.up[2]};
    // R = [F L U]^-1 by cofactors: row k of R is (column k+1 x column k+2) / det
    auto cross3 = [](const double* a, const double* b, double* r) {
        r[0] = a[1] * b[2] - a[2] * b[1];
        r[1] = a[2] * b[0] - a[0] * b[2];
        r[2] = a[0] * b[1] - a[1] * b[0];
    };
    double R[3][3];
    cross3(L, U, R[0]);
    cross3(U, F, R[1]);
    cross3(F, L, R[2]);
    const double det = F[0] * R[0][0] + F[1] * R[0][1] + F[2] * R[0][2];
    if (!(std::fabs(det) > 0.5) || !std::isfinite(det)) return;  // not a (near-)orthonormal camera basis
    for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 3; ++a) R[k][a] /= det;
    const Bvh8Node& root = md.root;
    for (int ch = 0; ch < 8; ++ch) {
        float* r = fr.rect[ch];
        r[0] = r[2] = INFINITY;  // empty: no (s, t) satisfies lo <= x <= hi
        r[1] = r[3] = -INFINITY;
        if (root.child[ch] == kBvhEmpty) continue;
        double slo = INFINITY, shi = -INFINITY, tlo = INFINITY, thi = -INFINITY;
        int front = 0, behind = 0;
        for (int k = 0; k < 8; ++k) {
            const double X[3] = {(double)((k & 1) ? root.hi(0, ch) : root.lo(0, ch)) - o[0],
                                 (double)((k & 2) ? root.hi(1, ch) : root.lo(1, ch)) - o[1],
                                 (double)((k & 4) ? root.hi(2, ch) : root.lo(2, ch)) - o[2]};
            const double mag = std::max({std::fabs(X[0]), std::fabs(X[1]), std::fabs(X[2])});
            const double z = R[0][0] * X[0] + R[0][1] * X[1] + R[0][2] * X[2];
            if (z > 0x1p-20 * mag) {
                ++front;
                const double s = (R[1][0] * X[0] + R[1][1] * X[1] + R[1][2] * X[2]) / z;
                const double t = (R[2][0] * X[0] + R[2][1] * X[1] + R[2][2] * X[2]) / z;
                slo = std::min(slo, s);
                shi = std::max(shi, s);
                tlo = std::min(tlo, t);
                thi = std::max(thi, t);
            } else if (z < 0.0) {
                ++behind;
            }
        }
        if (behind == 8) continue;  // never met
        if (front < 8 || !(std::fabs(slo) + std::fabs(shi) + std::fabs(tlo) + std::fabs(thi) < 0x1p60)) {
            r[0] = r[2] = -INFINITY;  // always tested
            r[1] = r[3] = INFINITY;
            continue;
        }
        auto widen = [](double x) { return 0x1p-18 * (1.0 + std::fabs(x)); };
        r[0] = detail::round_down(slo - widen(slo));
        r[1] = detail::round_up(shi + widen(shi));
        r[2] = detail::round_down(tlo - widen(tlo));
        r[3] = detail::round_up(thi + widen(thi));
    }
    fr.sA = fa.phw / (double)fa.halfW;
    fr.sB = fa.phw * ((double)fa.halfW - 0.5) / (double)fa.halfW;
    fr.tA = fa.phh / (double)fa.halfH;
    fr.tB = fa.phh * ((double)fa.halfH - 0.5) / (double)fa.halfH;
    fr.on = std::isfinite(fr.sA) && std::isfinite(fr.sB) && std::isfinite(fr.tA) && std::isfinite(fr.tB) ? 1u : 0u;
    if (fr.on && !(c->flags & MIRT_OPT_NO_BOX_GATE)) object_cert(fa, R, fr, oc);
}

int prof_get(mirt_ctx* c, ProfRec& r) {
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->prof_free.empty()) {
        r = c->prof_free.back();
        c->prof_free.pop_back();
        return MIRT_OK;
    }
    for (int k = 0; k < 4; ++k) HIP_TRY(hipEventCreate(&r.ev[k]));
    return MIRT_OK;
}

// Block table of a tile list: linear block number k runs over the tiles in list order and
// over each tile's blocks column-major; entry (k % kQShards) * per_shard + k / kQShards
// holds block k (shard-major, mirt_internal.hpp).  Rebuilt and uploaded only when the
// list changes.
int blocks_prepare(Slot* sl, uint32_t W, uint32_t H, const mirt_tile* tiles, uint32_t n, hipStream_t s) {
    if (sl->blocks_W == W && sl->blocks_H == H && sl->blocks_key.size() == n &&
        memcmp(sl->blocks_key.data(), tiles, sizeof(mirt_tile) * n) == 0)
        return MIRT_OK;
    sl->blocks_key.clear();
    uint64_t nb = 0;
    for (uint32_t t = 0; t < n; ++t)
        nb += (uint64_t)((tiles[t].w + kBlk - 1) / kBlk) * ((tiles[t].h + kBlk - 1) / kBlk);
    if (nb > 0x7fffffffull) return fail(MIRT_E_LIMIT, "too many 8x8 blocks in one call");
    const uint64_t per_shard = (nb + kQShards - 1) / kQShards;
    const uint64_t entries = per_shard * kQShards;
    int r = dev_grow(sl->d_blocks, sl->blocks_cap, entries);
    if (r != MIRT_OK) return r;
    if (sl->h_blocks_cap < entries) {
        if (sl->h_blocks) (void)hipHostFree(sl->h_blocks);
        sl->h_blocks = nullptr;
        sl->h_blocks_cap = 0;
        HIP_TRY(hipHostMalloc((void**)&sl->h_blocks, sizeof(BlockDesc) * entries));
        sl->h_blocks_cap = entries;
    }
    memset(sl->h_blocks, 0, sizeof(BlockDesc) * entries);
    uint64_t off = 0, k = 0;  // k: linear block number, tiles in list order, blocks column-major
    for (uint32_t t = 0; t < n; ++t) {
        const mirt_tile& tl = tiles[t];
        for (uint32_t bx = 0; bx < tl.w; bx += kBlk)
            for (uint32_t by = 0; by < tl.h; by += kBlk, ++k) {
                BlockDesc& b = sl->h_blocks[(k % kQShards) * per_shard + k / kQShards];
                b.out = (uint32_t)(off + (uint64_t)bx * tl.h + by);
                b.pxy = (tl.x + bx) | ((tl.y + by) << 16);
                b.geo = tl.h | (std::min<uint32_t>(kBlk, tl.w - bx) << 16) | (std::min<uint32_t>(kBlk, tl.h - by) << 24);
                b.pad = 0;
            }
        off += (uint64_t)tl.w * tl.h;
    }
    HIP_TRY(hipMemcpyAsync(sl->d_blocks, sl->h_blocks, sizeof(BlockDesc) * entries, hipMemcpyHostToDevice, s));
    sl->blocks_key.assign(tiles, tiles + n);
    sl->blocks_W = W;
    sl->blocks_H = H;
    sl->nblocks = (uint32_t)nb;
    sl->per_shard = (uint32_t)per_shard;
    return MIRT_OK;
}

// Validate a tile list against the screen; its pixel count.
int check_tiles(uint32_t W, uint32_t H, const mirt_tile* tiles, uint32_t n, uint64_t& pixels) {
    if (W == 0 || H == 0) return fail(MIRT_E_INVALID, "screen width/height must be > 0");
    if (n == 0 || !tiles) return fail(MIRT_E_INVALID, "empty tile list");
    pixels = 0;
    for (uint32_t t = 0; t < n; ++t) {
        const mirt_tile& tl = tiles[t];
        if (tl.w == 0 || tl.h == 0) return fail(MIRT_E_INVALID, "tile " + std::to_string(t) + " is empty");
        if ((uint64_t)tl.x + tl.w > W || (uint64_t)tl.y + tl.h > H)
            return fail(MIRT_E_INVALID, "tile " + std::to_string(t) + " exceeds the screen");
        pixels += (uint64_t)tl.w * tl.h;
    }
    if (pixels > 0xffffffffull) return fail(MIRT_E_LIMIT, "more than 2^32 pixels in one call");
    if (W > 65535 || H > 65535) return fail(MIRT_E_LIMIT, "screen width/height above 65535");
    return MIRT_OK;
}

// light_table's records on the host (mirt_debug_light_table): nl lights x n triangles of T
// (kTriD doubles each), lighttab.hpp's arithmetic (the device builder's, k_light_table).
void light_records(const double* T, uint32_t n, double scale, const double pos[3], const double (*lpos)[3], uint32_t nl,
                   float* out) {
    for (uint32_t l = 0; l < nl; ++l) {
        const LightGeom g = light_geom(lpos[l], pos, scale);
        for (uint32_t k = 0; k < n; ++k) light_record(T + (size_t)k * kTriD, g, out + ((size_t)l * n + k) * kLtD);
    }
}

// The light table of a one-object frame's shadow segments (kernels.hip SegPre, DESIGN.md
// §4.3): per light l and BVH position k, with V_i = P_i - L (object space; P2 = P1 + E1,
// P3 = P1 + E2 as the test sees them), the fp32 record
//   W1 = V2 x V3, W2 = V3 x V1, W3 = V1 x V2, A = E1 x E2, ntL = A . (L - P1), cw, cA, ctL.
// cw bounds, per unit |d|_inf, the error of every m_k = d . W_k the kernel forms in fp32
// against the exact quotient numerators of the fp64 test (fp32 rounding of W, d and the dot:
// at most 5 ulp of sum |d_i W_i|, bounded by 2^-21 = 8 ulp of |d|_inf |W|_1; the fp64 test's own rounding and the host's, 2^-36 (G + Lh)
// (G + Ed); the shadow origin's distance from the line through L, |eps| <= M, and M's
// bound over every hit on the mesh: 4 Mmax Ed), plus 2^-100 against underflow; cA the same
// for a = d . A against -inc; ctL for nt's terms that do not scale with lam.  Rounded up
// (lighttab.hpp, the arithmetic the device builder k_light_table runs).
//
// The cache (mirt_ctx::LightTab): a key (mesh, object position, lights) found is reused; a new
// key reserves a buffer (a dead table's of the same size once its readers are done, else
// hipMalloc) and is built by k_light_table on the stream of the first frame that reads it
// (lt_launch) — no host work proportional to the mesh on the issue path.  Past the cap
// (mirt_set_light_cache, default 4 GiB) the least recently used table that no unlaunched frame
// record holds (LightTab::pins: taken by light_table(), returned by lt_unpin once the record
// has been launched or dropped) is evicted: the events re-recorded after every launch that read
// it (one per reader stream, lt_after) mark the point after which its buffer is free.  Only when
// nothing is evictable (every table pinned by frames being issued) does a frame trace without a
// table; the fallbacks are counted (mirt_light_cache_stats), so a disabled prefilter is never
// silent.
hipEvent_t lt_event(mirt_ctx* c) {
    if (!c->lt_events.empty()) {
        hipEvent_t e = c->lt_events.back();
        c->lt_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    return e;
}
// Dead tables whose readers are all done: freed, or kept for a build of `want` bytes (returned).
float* lt_reap(mirt_ctx* c, size_t want) {
    float* got = nullptr;
    for (size_t i = 0; i < c->lt_dead.size();) {
        mirt_ctx::DeadTab& t = c->lt_dead[i];
        bool done = true;
        for (hipEvent_t e : t.evs) done = done && hipEventQuery(e) == hipSuccess;
        if (!done) {
            ++i;
            continue;
        }
        for (hipEvent_t e : t.evs) c->lt_events.push_back(e);
        // a buffer is kept for reuse only while the cache is within its cap (a cap lowered by
        // mirt_set_light_cache shrinks the cache as its tables die, instead of recycling them)
        if (!got && want && t.bytes == want && c->ltab_bytes <= c->lt_cap) {
            got = t.d;  // stays allocated (and counted in ltab_bytes) for the next table
            ++c->lt_stat[4];
        } else {
            (void)hipFree(t.d);
            c->ltab_bytes -= t.bytes;
        }
        c->lt_dead[i] = c->lt_dead.back();
        c->lt_dead.pop_back();
    }
    return got;
}
// Retire table i: its buffer is free once every launch that read it (or built it) is done.
void lt_evict(mirt_ctx* c, size_t i) {
    mirt_ctx::LightTab& t = *c->ltabs[i];
    mirt_ctx::DeadTab dt;
    dt.d = t.d;
    dt.bytes = t.bytes;
    for (auto& u : t.uses) dt.evs.push_back(u.second);
    if (t.ready) dt.evs.push_back(t.ready);
    c->lt_dead.push_back(std::move(dt));
    c->ltabs[i] = std::move(c->ltabs.back());
    c->ltabs.pop_back();
    ++c->lt_stat[2];
}
void lt_drop_mesh(mirt_ctx* c, uint32_t mesh) {  // the device is idle (mirt_mesh_release)
    std::lock_guard<std::mutex> g(c->lt_mu);
    for (size_t i = 0; i < c->ltabs.size();) {
        if (c->ltabs[i]->mesh != mesh) {
            ++i;
            continue;
        }
        lt_evict(c, i);
    }
    (void)lt_reap(c, 0);
}
const float* light_table(mirt_ctx* c, const mirt_frame* f, const FrameArgs& fa) {
    if (fa.n_objects != 1 || fa.n_lights == 0 ||
        (fa.flags & (MIRT_OPT_NO_PREFILTER | MIRT_OPT_BRUTE_FORCE | MIRT_OPT_NO_SEGMENT | MIRT_OPT_NO_LIGHT_TABLE)))
        return nullptr;
    const uint32_t mid = f->objects[0].mesh_id;
    std::lock_guard<std::mutex> g(c->lt_mu);
    const uint64_t now = ++c->lt_clock;
    for (auto& t : c->ltabs)
        if (t->mesh == mid && t->nl == fa.n_lights && !memcmp(t->pos, fa.obj[0].pos, sizeof(t->pos)) &&
            !memcmp(t->lpos, fa.lpos, sizeof(double) * 3 * fa.n_lights)) {
            t->last_use = now;
            ++t->pins;
            ++c->lt_stat[1];
            return t->d;
        }
    const MeshDev& m = c->meshes[mid];
    const uint32_t n = m.ntri, nl = fa.n_lights;
    if (n == 0) return nullptr;
    const size_t bytes = (size_t)nl * n * kLtD * sizeof(float);
    float* buf = lt_reap(c, bytes);
    // make room: least recently used first, never a pinned table, and no more once retired
    // tables still being read would make the room (their buffers come back to a later frame;
    // this one traces without a table meanwhile)
    while (!buf && c->ltab_bytes + bytes > c->lt_cap) {
        size_t retiring = 0;
        for (const auto& t : c->lt_dead) retiring += t.bytes;
        if (retiring >= bytes) break;
        size_t best = c->ltabs.size();
        for (size_t i = 0; i < c->ltabs.size(); ++i)
            if (c->ltabs[i]->pins == 0 &&
                (best == c->ltabs.size() || c->ltabs[i]->last_use < c->ltabs[best]->last_use))
                best = i;
        if (best == c->ltabs.size()) break;
        lt_evict(c, best);
        buf = lt_reap(c, bytes);
    }
    if (!buf) {
        if (c->ltab_bytes + bytes > c->lt_cap || hipSetDevice(c->device) != hipSuccess ||
            hipMalloc((void**)&buf, bytes) != hipSuccess) {
            ++c->lt_stat[3];  // this frame traces without the pre-classification (counted)
            return nullptr;
        }
        c->ltab_bytes += bytes;
    }
    auto lt = std::make_unique<mirt_ctx::LightTab>();
    lt->mesh = mid;
    lt->nl = nl;
    memcpy(lt->pos, fa.obj[0].pos, sizeof(lt->pos));
    memcpy(lt->lpos, fa.lpos, sizeof(double) * 3 * nl);
    lt->d = buf;
    lt->bytes = bytes;
    lt->last_use = now;
    lt->pins = 1;
    c->ltabs.push_back(std::move(lt));
    return buf;
}
// A frame record that held `tab` (light_table) was launched or dropped.
void lt_unpin(mirt_ctx* c, const float* tab) {
    if (!tab) return;
    std::lock_guard<std::mutex> g(c->lt_mu);
    for (auto& tp : c->ltabs)
        if (tp->d == tab) {
            if (tp->pins) --tp->pins;
            return;
        }
}
// The pins of up to kMaxFrames frame records, returned when the holder goes out of scope.
struct LtPins {
    mirt_ctx* c;
    const float* tab[kMaxFrames] = {};
    uint32_t n = 0;
    explicit LtPins(mirt_ctx* c_) : c(c_) {}
    void add(const float* t) { tab[n++] = t; }
    ~LtPins() {
        for (uint32_t i = 0; i < n; ++i) lt_unpin(c, tab[i]);
    }
};
// Before frames reading `tab` launch on stream s: build it there if nobody has (stream order
// then covers this stream; other streams wait for its `ready` event until it has completed),
// and remember s as a reader for eviction.
int lt_launch(mirt_ctx* c, const float* tab, hipStream_t s) {
    if (!tab) return MIRT_OK;
    std::lock_guard<std::mutex> g(c->lt_mu);
    for (auto& tp : c->ltabs) {
        mirt_ctx::LightTab& t = *tp;
        if (t.d != tab) continue;
        if (!t.built) {
            const MeshDev& m = c->meshes[t.mesh];
            LightTabArgs a{};
            a.tri = m.tri;
            a.n = m.ntri;
            a.nl = t.nl;
            a.scale = m.scale;
            memcpy(a.pos, t.pos, sizeof(a.pos));
            memcpy(a.lpos, t.lpos, sizeof(double) * 3 * t.nl);
            a.out = t.d;
            HIP_TRY(launch_light_table(a, s));
            t.ready = lt_event(c);
            if (!t.ready) return fail(MIRT_E_DEVICE, "hipEventCreate (light table)");
            HIP_TRY(hipEventRecord(t.ready, s));
            t.built = true;
            t.built_on = s;
            ++c->lt_stat[0];
        } else if (!t.ready_seen && s != t.built_on) {
            if (hipEventQuery(t.ready) == hipSuccess)
                t.ready_seen = true;
            else
                HIP_TRY(hipStreamWaitEvent(s, t.ready, 0));
        }
        return MIRT_OK;
    }
    return fail(MIRT_E_INVALID, "light table not in the cache");  // cannot happen (pinned until launched)
}
// After the frames reading `tab` were enqueued on s: the table's event for s marks their end.
int lt_after(mirt_ctx* c, const float* tab, hipStream_t s) {
    if (!tab) return MIRT_OK;
    std::lock_guard<std::mutex> g(c->lt_mu);
    for (auto& tp : c->ltabs) {
        if (tp->d != tab) continue;
        hipEvent_t e = nullptr;
        for (auto& u : tp->uses)
            if (u.first == s) e = u.second;
        if (!e) {
            if (!(e = lt_event(c))) return fail(MIRT_E_DEVICE, "hipEventCreate (light table)");
            tp->uses.emplace_back(s, e);
        }
        HIP_TRY(hipEventRecord(e, s));
        return MIRT_OK;
    }
    return MIRT_OK;
}

// One frame's launch record: its arguments, output planes and frustum rectangles.
void frame_record(const mirt_ctx* c, const mirt_frame* f, uint32_t W, uint32_t H, const OutPlanes& out, FrameRec& rec,
                  uint64_t& tris) {
    fill_args(c, f, W, H, rec.fa, tris);
    rec.fa.ltab = light_table(const_cast<mirt_ctx*>(c), f, rec.fa);
    rec.fa.ltab_n = rec.fa.ltab ? c->meshes[f->objects[0].mesh_id].ntri : 0;
    frustum_args(c, f, rec.fa, rec.fr, rec.ocert);
    rec.out = out;
    rec.xf = XferArgs{};  // the packed layout (a frame group's fused shares set their transfer form)
    rec.live[0] = rec.live[1] = 0;  // every block (a frame group narrows it to the hit rectangle)
    rec.live[2] = W;
    rec.live[3] = H;
}

// Frames whose records can share one k_trace launch (same mesh, objects, lights, options
// and frustum mode: the kernel takes those from the first record).
bool frames_batchable(const FrameRec& a, const FrameRec& b) {
    if (a.fa.n_objects != b.fa.n_objects || a.fa.n_lights != b.fa.n_lights || a.fa.flags != b.fa.flags ||
        a.fa.W != b.fa.W || a.fa.H != b.fa.H || a.fr.on != b.fr.on)
        return false;
    for (uint32_t o = 0; o < a.fa.n_objects; ++o)
        if (memcmp(&a.fa.obj[o].m, &b.fa.obj[o].m, sizeof(DevMesh)) != 0) return false;
    return true;
}

int launch_frames(mirt_ctx* c, Slot* sl, uint32_t nf, uint32_t W, uint32_t H, const mirt_tile* tiles, uint32_t n,
                  uint32_t bounces, hipStream_t s, const volatile int* cancel, uint32_t max_wg_now = 0,
                  const FusedCopy* fcopy = nullptr);

// Enqueue primary -> shadow -> shade for a tile list on stream s.
int enqueue_trace(mirt_ctx* c, Slot* sl, const mirt_frame* f, uint32_t W, uint32_t H, const mirt_tile* tiles,
                  uint32_t n, const OutPlanes& out, hipStream_t s, const volatile int* cancel, uint64_t* pixels_out,
                  uint64_t* tris_out) {
    uint64_t pixels = 0, tris = 0;
    int r = check_tiles(W, H, tiles, n, pixels);
    if (r != MIRT_OK) return r;
    frame_record(c, f, W, H, out, sl->h_frames[0], tris);
    LtPins pin(c);  // the record's light table, held until it has been launched
    pin.add(sl->h_frames[0].fa.ltab);
    if ((r = launch_frames(c, sl, 1, W, H, tiles, n, f->max_bounces, s, cancel)) != MIRT_OK) return r;
    *pixels_out = pixels;
    *tris_out = tris;
    return MIRT_OK;
}

// Launch the nf frames staged in sl->h_frames (k_trace: one launch for all of them; the
// split kernels and reflections take one frame).
int launch_frames(mirt_ctx* c, Slot* sl, uint32_t nf, uint32_t W, uint32_t H, const mirt_tile* tiles, uint32_t n,
                  uint32_t bounces, hipStream_t s, const volatile int* cancel, uint32_t max_wg_now,
                  const FusedCopy* fcopy) {
    int r = MIRT_OK;
    if (nf == 0 || nf > kMaxFrames) return fail(MIRT_E_INVALID, "1..8 frames per launch");
    const bool one_launch = !(c->flags & MIRT_OPT_SPLIT_KERNELS) && !bounces;
    if (nf > 1 && !one_launch) return fail(MIRT_E_INVALID, "several frames per launch need the single-kernel path");
    // LDS streaming of HBM meshes is k_trace's (only its launch sizes the slices)
    if (!one_launch) sl->h_frames[0].fa.flags &= ~MIRT_OPT_LDS_STREAM;
    const FrameArgs& fa = sl->h_frames[0].fa;
    const OutPlanes out = sl->h_frames[0].out;
    for (uint32_t k = 0; k < nf; ++k)  // the frames' light tables: built / waited for on s
        if ((k == 0 || sl->h_frames[k].fa.ltab != sl->h_frames[k - 1].fa.ltab) &&
            (r = lt_launch(c, sl->h_frames[k].fa.ltab, s)) != MIRT_OK)
            return r;
    if ((r = blocks_prepare(sl, W, H, tiles, n, s)) != MIRT_OK) return r;
    HT(9);
    uint64_t pixels = 0;
    for (uint32_t t = 0; t < n; ++t) pixels += (uint64_t)tiles[t].w * tiles[t].h;
    const uint32_t nl = fa.n_lights;
    const uint64_t total = (uint64_t)sl->nblocks * nf;  // every frame's blocks
    if (total > 0x7fffffffull) return fail(MIRT_E_LIMIT, "too many 8x8 blocks in one launch");
    WorkArgs wa{};
    wa.blocks = sl->d_blocks;
    wa.nblocks = (uint32_t)total;
    wa.nblocks_frame = sl->nblocks;
    wa.nframes = nf;
    wa.per_shard = sl->per_shard;
    wa.hit_cap = (uint32_t)(((uint64_t)sl->nblocks + kQShards - 1) / kQShards * 64);
    // persistent: kWgPerCu workgroups per CU
    uint64_t per_wg, max_wg;
    {
        std::lock_guard<std::mutex> g(c->mu);
        per_wg = std::max<uint32_t>(c->min_blocks_per_wg, 1);
        max_wg = c->max_workgroups ? std::min<uint64_t>(c->max_workgroups, (uint64_t)kWgPerCu * c->cus)
                                    : (uint64_t)kWgPerCu * c->cus;
    }
    // a frame group that knows how many launches are still running sizes this one for the
    // CUs they leave (a lone frame gets the whole chip)
    if (max_wg_now) max_wg = std::min<uint64_t>(max_wg_now, (uint64_t)kWgPerCu * c->cus);
    // at least min(blocks, CUs) workgroups: a small tile list (a BulkTrace order, one
    // rank's share) keeps one block per wave rather than queueing heavy blocks on few waves
    const uint64_t want = std::max<uint64_t>((total + per_wg - 1) / per_wg, std::min<uint64_t>(total, (uint64_t)c->cus));
    const int pgrid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, max_wg));
    // k_trace: workgroup w's hit region holds the kHitRing ring positions and one chunk per
    // block it owns (a chunk that finds the ring full)
    wa.wg_cap = (uint32_t)((kHitRing + (total + pgrid - 1) / pgrid) * 64);
    // k_trace (one launch): sized for any grid up to kWgPerCu per CU (G (R + ceil(total / G)) <=
    // total + G (R + 1)): a launch whose grid differs from the slot's last one
    // (MIRT_ADAPTIVE_GRID) never regrows the buffers (hipFree synchronises the device).  The split
    // kernels and the reflection levels use the kQShards regions only (no ring), which also size
    // every bounce-wave buffer below.
    const uint64_t hit_slots =
        one_launch ? std::max<uint64_t>({(uint64_t)kQShards * wa.hit_cap, (uint64_t)pgrid * wa.wg_cap,
                                         (total + (uint64_t)kWgPerCu * c->cus * (kHitRing + 1)) * 64})
                   : (uint64_t)kQShards * wa.hit_cap;
    if ((r = dev_grow(sl->hits, sl->hits_cap, hit_slots)) != MIRT_OK) return r;
    if ((r = dev_grow(sl->litw, sl->litw_cap, hit_slots)) != MIRT_OK) return r;
    if ((r = dev_grow(sl->blkdone, sl->blkdone_cap, hit_slots / 64)) != MIRT_OK) return r;
    wa.bounces = bounces;
    if (wa.bounces) {
        // the primary rays' directions: chains only (k_reflect); the bounce waves' k_pack makes
        // them again from the pixels
        const bool chains = (c->flags & MIRT_OPT_REFLECT_CHAINS) != 0;
        if (chains && (r = dev_grow(sl->dir0, sl->dir0_cap, 3 * hit_slots)) != MIRT_OK) return r;
        if ((r = dev_grow(sl->ph0, sl->ph0_cap, 3 * hit_slots)) != MIRT_OK) return r;
        if ((r = dev_grow(sl->refl, sl->refl_cap, (size_t)kReflD * bounces * hit_slots)) != MIRT_OK) return r;
        wa.dir0 = chains ? sl->dir0 : nullptr;
        wa.ph0 = sl->ph0;
        wa.refl = sl->refl;
        wa.refl_stride = hit_slots;
        wa.ph_out = sl->ph0;  // level 0 (k_shadow); the bounce levels set their own
        wa.ph_stride = 3;
        if (!(c->flags & MIRT_OPT_REFLECT_CHAINS)) {
            for (int b = 0; b < 2; ++b) {
                if ((r = dev_grow(sl->lhits[b], sl->lhits_cap[b], hit_slots)) != MIRT_OK) return r;
                if ((r = dev_grow(sl->ldir[b], sl->ldir_cap[b], 3 * hit_slots)) != MIRT_OK) return r;
                if ((r = dev_grow(sl->llitw[b], sl->llitw_cap[b], hit_slots)) != MIRT_OK) return r;
                if ((r = dev_grow(sl->lblk[b], sl->lblk_cap[b], hit_slots / 64)) != MIRT_OK) return r;
            }
            if ((r = dev_grow(sl->lcnt, sl->lcnt_cap, (size_t)(bounces + 1) * kCntN)) != MIRT_OK) return r;
            if ((r = dev_grow(sl->chain, sl->chain_cap, hit_slots)) != MIRT_OK) return r;
            if ((r = dev_grow(sl->shits, sl->shits_cap, hit_slots)) != MIRT_OK) return r;
            if ((r = dev_grow(sl->sdir, sl->sdir_cap, 3 * hit_slots)) != MIRT_OK) return r;
            if ((r = dev_grow(sl->ssrc, sl->ssrc_cap, hit_slots / 64)) != MIRT_OK) return r;
            if ((r = dev_grow(sl->bmap, sl->bmap_cap, (size_t)std::max<uint32_t>(sl->nblocks, 1))) != MIRT_OK) return r;
            const size_t ng = (std::max<size_t>(sl->nblocks, hit_slots / 64) + kPackGroup - 1) / kPackGroup;
            if ((r = dev_grow(sl->gcnt, sl->gcnt_cap, (size_t)(bounces + 1) * ng)) != MIRT_OK) return r;
            wa.bmap = sl->bmap;
            wa.bgcnt = sl->gcnt;
            HIP_TRY(hipMemsetAsync(sl->bmap, 0, (size_t)sl->nblocks * sizeof(uint32_t), s));
            HIP_TRY(hipMemsetAsync(sl->gcnt, 0, (size_t)(bounces + 1) * ng * sizeof(uint32_t), s));
        }
    }
    if (one_launch) {
        // the deferred second passes (k_trace's redo list): flags and list reuse
        // the bounce-wave fields, which one-launch frames never use
        const size_t L = (size_t)kMaxFrames * std::max<uint32_t>(sl->nblocks, 1);
        const size_t cap0 = sl->redo_cap;
        if ((r = dev_grow(sl->redo, sl->redo_cap, 1 + 2 * L)) != MIRT_OK) return r;
        if (sl->redo_cap != cap0) HIP_TRY(hipMemsetAsync(sl->redo, 0, sl->redo_cap * sizeof(uint32_t), s));
        wa.bgcnt = sl->redo;
        wa.bmap = sl->redo + 1 + L;
    }
    if (one_launch && !getenv("MIRT_NO_COST_ORDER")) {
        const size_t cap0 = sl->cost_cap;
        if ((r = dev_grow(sl->cost, sl->cost_cap, (size_t)sl->nblocks)) != MIRT_OK) return r;
        if (sl->cost_cap != cap0) HIP_TRY(hipMemsetAsync(sl->cost, 0, sl->cost_cap * sizeof(uint16_t), s));
        wa.block_cost = sl->cost;
    }
    wa.hits = sl->hits;
    wa.litw = sl->litw;
    wa.blkdone = sl->blkdone;
    wa.counters = sl->counters + (size_t)sl->parity * kCntN;
    wa.counters_next = sl->counters + (size_t)(sl->parity ^ 1u) * kCntN;
    wa.summary = sl->summary;
    wa.fr = sl->h_frames[0].fr;
    memcpy(wa.live, sl->h_frames[0].live, sizeof(wa.live));  // (k_primary: one frame per launch)
    wa.dynamic = (c->flags & MIRT_OPT_STATIC_SCHEDULE)
                     ? 0u
                     : (uint32_t)(kDynPrimary | kDynShadow | kDynReflect);
    if (c->flags & MIRT_OPT_TIMELINE) {
        std::lock_guard<std::mutex> g(c->mu);
        if (!c->timeline) {
#ifdef MIRT_ITEM_TRACE
            const uint32_t cap = (uint32_t)(c->cus * (kWG / 64)) * 32;  // item records: 32 per wave (diagnostic build)
#else
            const uint32_t cap = (uint32_t)(kWgPerCu * c->cus * (kWG / 64));
#endif
            HIP_TRY(hipMalloc((void**)&c->timeline, sizeof(uint64_t) * kTimelineRec * 2 * cap));
            c->timeline_cap = cap;
        }
        HIP_TRY(hipMemsetAsync(c->timeline, 0, sizeof(uint64_t) * kTimelineRec * 2 * c->timeline_cap, s));
        wa.timeline = c->timeline;
        wa.timeline_cap = c->timeline_cap;
    }

    ProfRec pr;
    const bool prof = c->profiling && c->prof_acc;
    if (prof && (r = prof_get(c, pr)) != MIRT_OK) return r;
    wa.prof_acc = prof ? c->prof_acc : nullptr;

    // this frame's counter set was zeroed by the previous frame's k_primary; only a frame
    // that stopped half-way leaves the sets dirty
    if (sl->dirty) HIP_TRY(hipMemsetAsync(sl->counters, 0, 2 * kCntN * sizeof(cnt_t), s));
    sl->dirty = true;
    sl->parity ^= 1u;
    const int sgrid = (int)std::max<uint64_t>(
        1, std::min<uint64_t>((pixels * std::max<uint32_t>(nl, 1) + kWG - 1) / kWG, (uint64_t)kWgPerCu * c->cus));
    if (cancel && *cancel) return fail(MIRT_E_CANCELLED, "cancelled");
    if (one_launch) {
        // one launch for the frames (k_trace); its time lands in the primary slot of the profile
        // per-view leaf tables (MIRT_OPT_VIEWS; one-object frames with an LDS-resident mesh):
        // built by k_trace's first workgroups, one per (frame, view)
        const DevMesh& m0 = fa.obj[0].m;
        const bool views = fa.n_objects == 1 && (c->flags & MIRT_OPT_VIEWS) &&
                           !(c->flags & (MIRT_OPT_BRUTE_FORCE | MIRT_OPT_NO_PREFILTER)) &&
                           m0.ntri <= (uint32_t)kLdsTris && m0.depth <= (uint32_t)kBvhShallowDepth &&
                           m0.nleaves > 0 && m0.nleaves <= kMaxViewLeaves && m0.leaves;
        uint32_t nviews = 0;
        if (views && (size_t)nf * (1 + nl) <= kMaxViewTables) {
            nviews = 1 + nl;
            if ((r = dev_grow(sl->views, sl->views_cap, (size_t)nf * nviews * m0.nleaves)) != MIRT_OK) return r;
            const size_t heads_cap = sl->view_heads_cap;
            if ((r = dev_grow(sl->view_heads, sl->view_heads_cap, (size_t)nf * nviews)) != MIRT_OK) return r;
            // a fresh buffer holds no tag (tags start at 1)
            if (sl->view_heads_cap != heads_cap)
                HIP_TRY(hipMemsetAsync(sl->view_heads, 0, sl->view_heads_cap * sizeof(ViewHead), s));
            if (++sl->view_tag == 0) sl->view_tag = 1;
            wa.view_tag = sl->view_tag;
            wa.views = sl->views;
            wa.view_heads = sl->view_heads;
            wa.nviews = nviews;
            wa.view_leaves = m0.nleaves;
        }
        // one frame: its record travels as k_trace's argument (no staging kernel ahead of it)
        HT(10);

        HT(11);
        wa.frames = nullptr;
        if (prof) HIP_TRY(hipEventRecord(pr.ev[0], s));  // the profile brackets k_trace alone
        HT(2);
        static const FusedCopy no_copy{};
        HIP_TRY(launch_trace(*(const FrameRecs*)sl->h_frames, wa, fcopy ? *fcopy : no_copy, pgrid, c->flags, s));
        HT(3);
        if (prof) {
            HIP_TRY(hipEventRecord(pr.ev[1], s));
            HIP_TRY(hipEventRecord(pr.ev[2], s));
        }
    } else {
        // the split kernels' deferred second passes: one entry per block (k_primary), per
        // (chunk, light) item (k_shadow) or per chunk (k_bounce), the launch's last workgroup
        // running them
        {
            const size_t items = std::max<size_t>({(size_t)sl->nblocks, (size_t)(wa.hit_cap / 64) * kQShards *
                                                                        std::max<uint32_t>(nl, 1), 1});
            const size_t cap0 = sl->sredo_cap;
            if ((r = dev_grow(sl->sredo, sl->sredo_cap, 2 + 2 * items)) != MIRT_OK) return r;
            if (sl->sredo_cap != cap0) HIP_TRY(hipMemsetAsync(sl->sredo, 0, sl->sredo_cap * sizeof(uint32_t), s));
            wa.split_redo = sl->sredo;
        }
        // the primary chunks' hit ballots (not with chains: k_reflect reads the records' obj)
        if (!(wa.bounces && (c->flags & MIRT_OPT_REFLECT_CHAINS)) && !getenv("MIRT_NO_HIT_BALLOT")) {
            if ((r = dev_grow(sl->hmask, sl->hmask_cap, hit_slots / 64)) != MIRT_OK) return r;
            wa.hmask = sl->hmask;
        }
        if (prof) HIP_TRY(hipEventRecord(pr.ev[0], s));
        HIP_TRY(launch_primary(fa, wa, out, pgrid, c->flags, s));
        if (prof) HIP_TRY(hipEventRecord(pr.ev[1], s));
        if (cancel && *cancel) return fail(MIRT_E_CANCELLED, "cancelled");
        // shadow rays + Phong (the wave finishing a block's last light shades it); also
        // launched with no lights, to shade every hit with the ambient term
        HIP_TRY(launch_shadow(fa, wa, out, sgrid, c->flags, s));
        if (prof) HIP_TRY(hipEventRecord(pr.ev[2], s));
        if (wa.bounces && (c->flags & MIRT_OPT_REFLECT_CHAINS)) {  // configs[4] extension: the last kernel
            if (cancel && *cancel) return fail(MIRT_E_CANCELLED, "cancelled");
            HIP_TRY(launch_reflect(fa, wa, out, sgrid, c->flags, s));
        } else if (wa.bounces) {
            // bounce waves: the primary hits packed in block order (k_pack, level 0), then per
            // level lv the reflection rays of level lv - 1's records (k_bounce, hits left at the
            // input's slots), those hits packed in order (k_pack), their shadow rays and phong
            // (k_shadow on the packed records); then the fold of every chain (the last kernel)
            HIP_TRY(hipMemsetAsync(sl->lcnt, 0, (size_t)(wa.bounces + 1) * kCntN * sizeof(cnt_t), s));
            const size_t ng = (std::max<size_t>(sl->nblocks, hit_slots / 64) + kPackGroup - 1) / kPackGroup;
            PackArgs p0{};
            p0.in = sl->hits;
            p0.in_dir = nullptr;  // made from each hit's pixel (PackArgs::rg)
            for (int k = 0; k < 3; ++k) {
                p0.rg.cam[k] = fa.cam[k];
                p0.rg.fwd[k] = fa.fwd[k];
                p0.rg.left[k] = fa.left[k];
                p0.rg.up[k] = fa.up[k];
            }
            p0.rg.phw = fa.phw;
            p0.rg.phh = fa.phh;
            p0.rg.halfW = fa.halfW;
            p0.rg.halfH = fa.halfH;
            p0.src = sl->bmap;
            p0.gcnt = sl->gcnt;
            p0.nsrc = sl->nblocks;
            p0.level0 = 1;
            p0.out = sl->lhits[0];
            p0.out_dir = sl->ldir[0];
            p0.out_litw = sl->llitw[0];
            p0.out_blkdone = sl->lblk[0];
            p0.out_cnt = sl->lcnt;
            p0.in_hmask = wa.hmask;
            HIP_TRY(launch_pack(wa, p0, (int)((sl->nblocks + kPackGroup - 1) / kPackGroup), s));
            for (uint32_t lv = 1; lv <= wa.bounces; ++lv) {
                if (cancel && *cancel) return fail(MIRT_E_CANCELLED, "cancelled");
                const int ib = (int)((lv - 1) & 1u), ob = (int)(lv & 1u);  // level lv in buffer lv % 2
                BounceArgs ba{};
                ba.in = sl->lhits[ib];
                ba.in_dir = sl->ldir[ib];
                ba.in_cnt = sl->lcnt + (size_t)(lv - 1) * kCntN;
                ba.out = sl->shits;
                ba.out_dir = sl->sdir;
                ba.src = sl->ssrc;
                ba.gcnt = sl->gcnt + (size_t)lv * ng;
                ba.chain = sl->chain;
                ba.level = lv;
                HIP_TRY(launch_bounce(fa, wa, ba, sgrid, c->flags, s));
                if (bounce_shades() && lv == wa.bounces) break;  // shaded in k_bounce, no next level
                PackArgs pk{};
                pk.in = sl->shits;
                pk.in_dir = sl->sdir;
                pk.src = sl->ssrc;
                pk.gcnt = ba.gcnt;
                pk.in_cnt = ba.in_cnt;
                pk.out = sl->lhits[ob];
                pk.out_dir = sl->ldir[ob];
                pk.out_litw = sl->llitw[ob];
                pk.out_blkdone = sl->lblk[ob];
                pk.out_cnt = sl->lcnt + (size_t)lv * kCntN;
                HIP_TRY(launch_pack(wa, pk, (int)((hit_slots / 64 + kPackGroup - 1) / kPackGroup), s));
                if (bounce_shades()) continue;
                WorkArgs wl = wa;
                wl.hits = sl->lhits[ob];
                wl.litw = sl->llitw[ob];
                wl.blkdone = sl->lblk[ob];
                wl.qcounters = pk.out_cnt;
                wl.hmask = nullptr;  // packed records: every one up to the region's count is a hit
                wl.ph_out = sl->refl + (size_t)(lv - 1) * hit_slots * kReflD;
                wl.ph_stride = kReflD;
                wl.ph_by_origin = 1;
                HIP_TRY(launch_shadow(fa, wl, out, sgrid, c->flags, s));
            }
            HIP_TRY(launch_refl_fold(fa, wa, out, sl->chain, (int)std::min<uint64_t>(4 * c->cus, 4096), s));
        }
    }
    sl->dirty = false;
    if (prof) {
        HIP_TRY(hipEventRecord(pr.ev[3], s));
        pr.pixels = pixels * nf;
        pr.frames = nf;
        std::lock_guard<std::mutex> g(c->mu);
        c->prof_pending.push_back(pr);
    }
    for (uint32_t k = 0; k < nf; ++k)  // the light tables' reader events
        if ((k == 0 || sl->h_frames[k].fa.ltab != sl->h_frames[k - 1].fa.ltab) &&
            (r = lt_after(c, sl->h_frames[k].fa.ltab, s)) != MIRT_OK)
            return r;
    if (!sl->dedicated) {
        HIP_TRY(hipEventRecord(sl->done, s));
        sl->pending = true;
    }
    return MIRT_OK;
}


int fill_stats(Slot* sl, hipStream_t s, uint64_t pixels, uint64_t tris, uint32_t nl, mirt_stats* st) {
    HIP_TRY(hipMemcpyAsync(sl->h_summary, sl->summary, kStatN * sizeof(cnt_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    memset(st, 0, sizeof(*st));
    st->primary_rays = pixels;
    st->hits = sl->h_summary[kStatHits];
    st->shadow_rays = sl->h_summary[kStatShadowRays];
    st->tri_tests = sl->h_summary[kStatPrimTests] + sl->h_summary[kStatShadowTests];
    st->reflection_rays = sl->h_summary[kStatReflRays];
    return MIRT_OK;
}

}  // namespace

extern "C" {

int mirt_abi_version(void) { return MIRT_ABI_VERSION; }
const char* mirt_last_error(void) { return g_err.c_str(); }

int mirt_create(int device, mirt_ctx** out) {
    if (!out) return fail(MIRT_E_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(MIRT_E_INVALID, "no HIP device " + std::to_string(device));
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return fail(MIRT_E_DEVICE, std::string("libmirt is built for gfx950 only; device is ") + prop.gcnArchName);
    mirt_ctx* c = new (std::nothrow) mirt_ctx();
    if (!c) return fail(MIRT_E_NOMEM, "context allocation failed");
    c->device = device;
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    *out = c;
    return MIRT_OK;
}

void mirt_destroy(mirt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (auto& sp : c->slots) slot_free(sp.get());
    for (auto* v : {&c->prof_pending, &c->prof_free})
        for (auto& r : *v) {
            for (auto e : r.ev)
                if (e) (void)hipEventDestroy(e);
        }
    (void)hipDeviceSynchronize();
    for (auto& m : c->meshes) mesh_free(m);
    for (auto& t : c->ltabs) {
        (void)hipFree(t->d);
        if (t->ready) (void)hipEventDestroy(t->ready);
        for (auto& u : t->uses) (void)hipEventDestroy(u.second);
    }
    for (auto& t : c->lt_dead) {
        (void)hipFree(t.d);
        for (hipEvent_t e : t.evs) (void)hipEventDestroy(e);
    }
    for (hipEvent_t e : c->lt_events) (void)hipEventDestroy(e);
    if (c->timeline) (void)hipFree(c->timeline);
    if (c->prof_acc) (void)hipFree(c->prof_acc);
    delete c;
}

int mirt_device(const mirt_ctx* c) { return c ? c->device : -1; }

double mirt_go_tan(double x);

int mirt_camera_init(const double pos[3], const double dir[3], double fov, mirt_camera* out) {
    if (!pos || !dir || !out) return fail(MIRT_E_INVALID, "NULL argument");
    // camera.go:35-44 with GlobalUp = (0,1,0) (environment.go:22)
    V3 d{dir[0], dir[1], dir[2]};
    V3 gup{0, 1, 0};
    if (is_zero(cross(d, gup))) return fail(MIRT_E_CAMERA, "Camera dir is parallel to global up {0 1 0}.");
    V3 f = norm(d);
    V3 l = norm(cross(d, gup));
    V3 u = cross(l, f);
    for (int k = 0; k < 3; ++k) out->pos[k] = pos[k];
    out->forward[0] = f.x; out->forward[1] = f.y; out->forward[2] = f.z;
    out->left[0] = l.x; out->left[1] = l.y; out->left[2] = l.z;
    out->up[0] = u.x; out->up[1] = u.y; out->up[2] = u.z;
    out->fov = fov;
    out->proj_half_width = mirt_go_tan(fov / 2.0);  // tracer.go:17
    return MIRT_OK;
}

// Go math.Tan (src/math/tan.go, Cephes): Cody–Waite reduction by pi/4 and a rational
// approximation.  Coefficients verified bit-for-bit against Go's published hex values
// (tests/test_host.py).  Beyond 2^29 Go switches to Payne–Hanek; camera fovs never do.
double mirt_go_tan(double x) {
    static const double P[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6, -1.79565251976484877988e7};
    static const double Q[5] = {1.0, 1.36812963470692954678e4, -1.32089234440210967447e6,
                                2.50083801823357915839e7, -5.38695755929454629881e7};
    const double PI4A = 7.85398125648498535156e-1, PI4B = 3.77489470793079817668e-8,
                 PI4C = 2.69515142907905952645e-15;
    const double M4PI = 1.27323954473516268615107010698011489627567716592365;
    if (x == 0 || x != x) return x;
    if (d_isinf(x)) return __builtin_nan("");
    bool sign = false;
    if (x < 0) {
        x = -x;
        sign = true;
    }
    if (x >= 536870912.0) return sign ? -std::tan(x) : std::tan(x);
    uint64_t j = (uint64_t)(x * M4PI);
    double y = (double)j;
    if (j & 1) {
        j++;
        y++;
    }
    double z = ((x - y * PI4A) - y * PI4B) - y * PI4C;
    double zz = z * z;
    if (zz > 1e-14)
        y = z + z * (zz * (((P[0] * zz) + P[1]) * zz + P[2]) / ((((zz + Q[1]) * zz + Q[2]) * zz + Q[3]) * zz + Q[4]));
    else
        y = z;
    if (j & 2) y = -1 / y;
    if (sign) y = -y;
    return y;
}

double mirt_go_pow(double x, double y) { return go_pow(x, y); }
// test hook: op 0 go_min(a, b), 1 go_max(a, b), 2 go_min1(a), 3 go_max0(a) (the colour
// code's constant-operand forms, pinned against the general ones by tests/test_host.py)
double mirt_go_minmax(int op, double a, double b) {
    return op == 0 ? go_min(a, b) : op == 1 ? go_max(a, b) : op == 2 ? go_min1(a) : go_max0(a);
}

void mirt_face_bounds(const double p1[3], const double p2[3], const double p3[3], double out[6]) {
    face_box(p1, p2, p3, out);
}
void mirt_object_bounds(const double* v, uint32_t nv, const double pos[3], double out[6]) {
    double vmin[3], vmax[3];
    vertex_minmax(v, nv, vmin, vmax);
    object_box(pos, vmin, vmax, out);
}

int mirt_mesh_upload(mirt_ctx* c, const double* v, uint32_t nv, const double* vn, uint32_t nn, const uint32_t* fv,
                     const uint32_t* fn, const uint32_t* fmat, uint32_t nf, const mirt_material* mats, uint32_t nm,
                     uint32_t* mesh_id) {
    if (!c || !mesh_id) return fail(MIRT_E_INVALID, "NULL context or mesh_id");
    if (nf && (!v || !fv || !fmat)) return fail(MIRT_E_INVALID, "NULL vertex/face array");
    if (nf && (!mats || nm == 0)) return fail(MIRT_E_INVALID, "faces need at least one material");
    const bool has_n = vn && nn > 0;
    if (has_n && nf && !fn) return fail(MIRT_E_INVALID, "normals given without face normal indices");
    for (uint32_t f = 0; f < nf; ++f) {
        for (int k = 0; k < 3; ++k) {
            if (fv[3 * f + k] >= nv) return fail(MIRT_E_INVALID, "face " + std::to_string(f) + " vertex out of range");
            if (has_n && fn[3 * f + k] >= nn)
                return fail(MIRT_E_INVALID, "face " + std::to_string(f) + " normal out of range");
        }
        if (fmat[f] >= nm) return fail(MIRT_E_INVALID, "face " + std::to_string(f) + " material out of range");
    }
    HIP_TRY(hipSetDevice(c->device));
    if (nf > kBvhFirstMask) return fail(MIRT_E_LIMIT, "more than 2^24 faces in one mesh");
    // Culling structure: 8-wide BVH over the faces, fp32 boxes inflated by 2^-12 of the
    // mesh's largest |coordinate|.  All per-face arrays in BVH order.
    double scale = 0;
    for (size_t i = 0; i < (size_t)nv * 3; ++i) scale = std::max(scale, std::fabs(v[i]));
    scale = std::max(scale, 1e-30);
    // MIRT_BVH_LEAF (experiments): faces per leaf, default kBvhLeaf
    const char* leaf_env = getenv("MIRT_BVH_LEAF");
    const uint32_t leaf = leaf_env && atoi(leaf_env) > 0 ? (uint32_t)atoi(leaf_env) : (uint32_t)kBvhLeaf;
    BvhBuild bvh = build_bvh(v, fv, nf, std::ldexp(scale, -12), leaf);
    if (bvh.depth > (uint32_t)kBvhMaxDepth)
        return fail(MIRT_E_LIMIT, "BVH deeper than the traversal stack (" + std::to_string(bvh.depth) + " levels)");
    // P1, E1 = P2 - P1, E2 = P3 - P1 (triangle.go:38: single fp64 subtractions, so the
    // precomputed edges are bit-identical to the per-test ones of the reference).
    std::vector<double> tri((size_t)nf * kTriD), vnrm(has_n ? (size_t)nf * kTriD : 0), mt((size_t)nm * 10);
    // the device copy of `tri` continues with the face boxes and the centre (mesh_fbox)
    std::vector<double> fbox((size_t)nf * kBoxD);
    std::vector<uint32_t> fm(nf);
    for (uint32_t pos = 0; pos < nf; ++pos) {
        const uint32_t f = bvh.order[pos];
        const double* p1 = v + 3 * (size_t)fv[3 * f];
        const double* p2 = v + 3 * (size_t)fv[3 * f + 1];
        const double* p3 = v + 3 * (size_t)fv[3 * f + 2];
        double* t = &tri[(size_t)pos * kTriD];
        for (int k = 0; k < 3; ++k) {
            t[k] = p1[k];
            t[3 + k] = p2[k] - p1[k];
            t[6 + k] = p3[k] - p1[k];
        }
        face_box(p1, p2, p3, &fbox[(size_t)pos * kBoxD]);
        if (has_n)
            for (int q = 0; q < 3; ++q)
                for (int k = 0; k < 3; ++k) vnrm[(size_t)pos * kTriD + 3 * q + k] = vn[3 * (size_t)fn[3 * f + q] + k];
        fm[pos] = fmat[f];
    }
    for (uint32_t m = 0; m < nm; ++m) {
        for (int k = 0; k < 3; ++k) {
            mt[10 * m + k] = mats[m].ka[k];
            mt[10 * m + 3 + k] = mats[m].kd[k];
            mt[10 * m + 6 + k] = mats[m].ks[k];
        }
        mt[10 * m + 9] = mats[m].ns;
    }
    const std::vector<Bvh8Dev> dev_nodes = make_dev_nodes(bvh.nodes);
    // the leaves with the boxes their parents hold, for the per-frame view tables
    std::vector<LeafBox> leaves;
    double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const Bvh8Node& n : bvh.nodes)
        for (int ch = 0; ch < 8; ++ch) {
            if (n.child[ch] == kBvhEmpty || !(n.child[ch] & kBvhLeafBit)) continue;
            LeafBox lb{};
            for (int a = 0; a < 3; ++a) {
                lb.lo[a] = n.lo(a, ch);
                lb.hi[a] = n.hi(a, ch);
                blo[a] = std::min(blo[a], (double)lb.lo[a]);
                bhi[a] = std::max(bhi[a], (double)lb.hi[a]);
            }
            lb.ref = n.child[ch];
            leaves.push_back(lb);
        }
    MeshDev md;
    md.nleaves = (uint32_t)leaves.size();
    for (int a = 0; a < 3; ++a) md.center[a] = md.nleaves ? 0.5 * (blo[a] + bhi[a]) : 0.0;
    vertex_minmax(v, nv, md.vmin, md.vmax);
    std::vector<double> dtri(tri);
    dtri.insert(dtri.end(), fbox.begin(), fbox.end());
    dtri.insert(dtri.end(), md.center, md.center + 3);
    md.ntri = nf;
    md.nmat = nm;
    md.has_normals = has_n;
    md.nnodes = (uint32_t)bvh.nodes.size();
    md.root = bvh.nodes[0];
    md.depth = bvh.depth;
    md.scale = scale;
    auto upload = [&](void** dst, const void* src, size_t bytes) -> int {
        if (bytes == 0) return MIRT_OK;
        hipError_t e = hipMalloc(dst, bytes);
        if (e != hipSuccess) return fail(MIRT_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy mesh");
        return MIRT_OK;
    };
    int r;
    if ((r = upload((void**)&md.tri, dtri.data(), dtri.size() * 8)) != MIRT_OK ||
        (r = upload((void**)&md.vnrm, vnrm.data(), vnrm.size() * 8)) != MIRT_OK ||
        (r = upload((void**)&md.fmat, fm.data(), (size_t)nf * 4)) != MIRT_OK ||
        (r = upload((void**)&md.fidx, bvh.order.data(), (size_t)nf * 4)) != MIRT_OK ||
        (r = upload((void**)&md.nodes, dev_nodes.data(), dev_nodes.size() * sizeof(Bvh8Dev))) != MIRT_OK ||
        (r = upload((void**)&md.mats, mt.data(), mt.size() * 8)) != MIRT_OK ||
        (r = upload((void**)&md.leaves, leaves.data(), leaves.size() * sizeof(LeafBox))) != MIRT_OK) {
        mesh_free(md);
        return r;
    }
    md.live = true;
    std::lock_guard<std::mutex> g(c->mu);
    *mesh_id = (uint32_t)c->meshes.size();
    c->meshes.push_back(std::move(md));
    return MIRT_OK;
}

static int group_launch_staged(mirt_group* g);

int mirt_mesh_release(mirt_ctx* c, uint32_t id) {
    if (!c) return fail(MIRT_E_INVALID, "NULL context");
    {
        // a frame group's staged records (an open batch, or one held by the lone-frame hold)
        // point at the mesh and its light tables: they are launched first, so the device sync
        // below covers them (a frame submitted before the release is traced, not dropped)
        std::lock_guard<std::mutex> gl(c->groups_mu);
        for (mirt_group* grp : c->groups) {
            int r = group_launch_staged(grp);
            if (r != MIRT_OK) return r;
        }
    }
    std::lock_guard<std::mutex> g(c->mu);
    if (id >= c->meshes.size() || !c->meshes[id].live) return fail(MIRT_E_INVALID, "unknown mesh id");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    lt_drop_mesh(c, id);  // the mesh's light tables go with it (the device is idle)
    mesh_free(c->meshes[id]);
    return MIRT_OK;
}

int mirt_set_light_cache(mirt_ctx* c, uint64_t max_bytes) {
    if (!c) return fail(MIRT_E_INVALID, "NULL context");
    std::lock_guard<std::mutex> g(c->lt_mu);
    c->lt_cap = (size_t)max_bytes;
    // shrink to the new cap now: least recently used first, never a pinned table; retired
    // buffers are freed once their readers are done (lt_reap)
    (void)lt_reap(c, 0);
    while (c->ltab_bytes > c->lt_cap) {
        size_t best = c->ltabs.size();
        for (size_t i = 0; i < c->ltabs.size(); ++i)
            if (c->ltabs[i]->pins == 0 &&
                (best == c->ltabs.size() || c->ltabs[i]->last_use < c->ltabs[best]->last_use))
                best = i;
        if (best == c->ltabs.size()) break;
        lt_evict(c, best);
        (void)lt_reap(c, 0);
    }
    return MIRT_OK;
}

int mirt_light_cache_stats(mirt_ctx* c, uint64_t out[8]) {
    if (!c || !out) return fail(MIRT_E_INVALID, "NULL argument");
    std::lock_guard<std::mutex> g(c->lt_mu);
    for (int k = 0; k < 5; ++k) out[k] = c->lt_stat[k];
    out[5] = c->ltabs.size();
    out[6] = c->ltab_bytes;
    out[7] = c->lt_cap;
    return MIRT_OK;
}

int mirt_debug_light_table_gpu(mirt_ctx* c, const double* tri, uint32_t n, double scale, const double pos[3],
                               const double* lights, uint32_t nl, float* out) {
    if (!c || (n && !tri) || !pos || (nl && !lights) || (n && nl && !out)) return fail(MIRT_E_INVALID, "NULL argument");
    if (nl > MIRT_MAX_LIGHTS) return fail(MIRT_E_LIMIT, "nl > MIRT_MAX_LIGHTS");
    if ((size_t)n * nl == 0) return MIRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    const size_t tb = (size_t)n * kTriD * sizeof(double), ob = (size_t)n * nl * kLtD * sizeof(float);
    void* d = nullptr;
    HIP_TRY(hipMalloc(&d, tb + ob));
    LightTabArgs a{};
    a.tri = (const double*)d;
    a.n = n;
    a.nl = nl;
    a.scale = scale;
    memcpy(a.pos, pos, sizeof(a.pos));
    memcpy(a.lpos, lights, sizeof(double) * 3 * nl);
    a.out = (float*)((char*)d + tb);
    hipError_t e = hipMemcpy(d, tri, tb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_light_table(a, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, a.out, ob, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "mirt_debug_light_table_gpu");
    return MIRT_OK;
}

int mirt_trace_tiles_async(mirt_ctx* c, const mirt_frame* f, uint32_t W, uint32_t H, const mirt_tile* tiles,
                           uint32_t n, const mirt_outputs* dout, void* stream, mirt_stats* st) {
    if (!c || !dout) return fail(MIRT_E_INVALID, "NULL context or outputs");
    HIP_TRY(hipSetDevice(c->device));
    int r = check_frame(c, f);
    if (r != MIRT_OK) return r;
    Slot* sl = nullptr;
    if ((r = slot_acquire(c, sl, tiles, n)) != MIRT_OK) return r;
    SlotGuard guard{c, sl};
    hipStream_t s = (hipStream_t)stream;  // NULL is the HIP null stream, as in the HIP API
    OutPlanes out{dout->rgb, dout->rgb8, dout->valid, dout->face, dout->object, dout->rgbv};
    uint64_t pixels = 0, tris = 0;
    if ((r = enqueue_trace(c, sl, f, W, H, tiles, n, out, s, nullptr, &pixels, &tris)) != MIRT_OK) {
        (void)hipStreamSynchronize(s);
        sl->pending = false;
        return r;
    }
    if (st) return fill_stats(sl, s, pixels, tris, f->n_lights, st);
    return MIRT_OK;
}

int mirt_trace_tile(mirt_ctx* c, const mirt_frame* f, uint32_t x, uint32_t y, uint32_t w, uint32_t h, uint32_t W,
                    uint32_t H, const mirt_outputs* hout, const volatile int* cancel, mirt_stats* st) {
    if (!c || !hout) return fail(MIRT_E_INVALID, "NULL context or outputs");
    HIP_TRY(hipSetDevice(c->device));
    int r = check_frame(c, f);
    if (r != MIRT_OK) return r;
    Slot* sl = nullptr;
    const mirt_tile key{x, y, w, h};
    if ((r = slot_acquire(c, sl, &key, 1)) != MIRT_OK) return r;
    SlotGuard guard{c, sl};
    const uint64_t npx = (uint64_t)w * h;
    // device staging for the requested planes: rgb(24) rgb8(3) valid(1) face(4) object(4) rgbv(4)
    const size_t need = npx * (24 + 4 + 4 + 3 + 1 + 4) + 96;
    uint8_t* base = (uint8_t*)sl->out_buf;
    size_t cap = sl->out_cap;
    if ((r = dev_grow(base, cap, need)) != MIRT_OK) return r;
    sl->out_buf = base;
    sl->out_cap = cap;
    OutPlanes out{};
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        uint8_t* p = base + off;
        off += (bytes + 15) & ~(size_t)15;
        return p;
    };
    out.rgb = hout->rgb ? (double*)carve(npx * 24) : nullptr;
    out.face = hout->face ? (int32_t*)carve(npx * 4) : nullptr;
    out.object = hout->object ? (int32_t*)carve(npx * 4) : nullptr;
    out.rgb8 = hout->rgb8 ? carve(npx * 3) : nullptr;
    out.valid = hout->valid ? carve(npx) : nullptr;
    out.rgbv = hout->rgbv ? (uint32_t*)carve(npx * 4) : nullptr;
    mirt_tile t{x, y, w, h};
    uint64_t pixels = 0, tris = 0;
    hipStream_t s = nullptr;
    if ((r = slot_stream(sl, s)) != MIRT_OK) return r;
    if ((r = enqueue_trace(c, sl, f, W, H, &t, 1, out, s, cancel, &pixels, &tris)) != MIRT_OK) {
        (void)hipStreamSynchronize(s);
        sl->pending = false;
        return r;
    }
    if (out.rgb) HIP_TRY(hipMemcpyAsync(hout->rgb, out.rgb, npx * 24, hipMemcpyDeviceToHost, s));
    if (out.rgb8) HIP_TRY(hipMemcpyAsync(hout->rgb8, out.rgb8, npx * 3, hipMemcpyDeviceToHost, s));
    if (out.valid) HIP_TRY(hipMemcpyAsync(hout->valid, out.valid, npx, hipMemcpyDeviceToHost, s));
    if (out.face) HIP_TRY(hipMemcpyAsync(hout->face, out.face, npx * 4, hipMemcpyDeviceToHost, s));
    if (out.object) HIP_TRY(hipMemcpyAsync(hout->object, out.object, npx * 4, hipMemcpyDeviceToHost, s));
    if (out.rgbv) HIP_TRY(hipMemcpyAsync(hout->rgbv, out.rgbv, npx * 4, hipMemcpyDeviceToHost, s));
    if (st) {
        if ((r = fill_stats(sl, s, pixels, tris, f->n_lights, st)) != MIRT_OK) return r;
    } else {
        HIP_TRY(hipStreamSynchronize(s));
    }
    sl->pending = false;
    if (cancel && *cancel) return fail(MIRT_E_CANCELLED, "cancelled");
    return MIRT_OK;
}

namespace {
// Unpack with per-tile packed offsets (NULL: back to back).  The slot keeps its last
// tile list on the device and skips the upload while the caller repeats it.
int unpack_impl(mirt_ctx* c, uint32_t W, uint32_t H, const mirt_tile* tiles, const uint64_t* offsets, uint32_t n,
                const mirt_outputs* packed, const mirt_outputs* fb, void* stream) {
    if (!c || !tiles || !packed || !fb || n == 0) return fail(MIRT_E_INVALID, "NULL argument or empty tile list");
    HIP_TRY(hipSetDevice(c->device));
    Slot* sl = nullptr;
    int r;
    if ((r = slot_acquire(c, sl)) != MIRT_OK) return r;
    SlotGuard guard{c, sl};
    hipStream_t s = (hipStream_t)stream;  // NULL is the HIP null stream, as in the HIP API
    const size_t cap_before = sl->tiles_cap;
    if ((r = tiles_grow(sl, n)) != MIRT_OK) return r;
    if (sl->tiles_cap != cap_before) sl->unpack_key.clear();  // reallocated: the device copy is gone
    uint64_t pixels = 0, span = 0, max_px = 0;
    std::vector<TileDesc> td(n);
    for (uint32_t t = 0; t < n; ++t) {
        if ((uint64_t)tiles[t].x + tiles[t].w > W || (uint64_t)tiles[t].y + tiles[t].h > H || !tiles[t].w ||
            !tiles[t].h)
            return fail(MIRT_E_INVALID, "tile " + std::to_string(t) + " is empty or exceeds the screen");
        const uint64_t off = offsets ? offsets[t] : pixels;
        if (off < span) return fail(MIRT_E_INVALID, "tile offsets must ascend without overlap");
        td[t] = TileDesc{tiles[t].x, tiles[t].y, tiles[t].w, tiles[t].h, off, 0, 0};
        pixels += (uint64_t)tiles[t].w * tiles[t].h;
        span = off + (uint64_t)tiles[t].w * tiles[t].h;
        max_px = std::max<uint64_t>(max_px, (uint64_t)tiles[t].w * tiles[t].h);
    }
    if (sl->unpack_key_H != H || sl->unpack_key.size() != n ||
        memcmp(sl->unpack_key.data(), td.data(), sizeof(TileDesc) * n) != 0) {
        memcpy(sl->h_tiles, td.data(), sizeof(TileDesc) * n);
        HIP_TRY(hipMemcpyAsync(sl->d_tiles, sl->h_tiles, sizeof(TileDesc) * n, hipMemcpyHostToDevice, s));
        sl->unpack_key = td;
        sl->unpack_key_H = H;
    }
    OutPlanes src{packed->rgb, packed->rgb8, packed->valid, packed->face, packed->object, packed->rgbv};
    OutPlanes dst{fb->rgb, fb->rgb8, fb->valid, fb->face, fb->object, fb->rgbv};
    HIP_TRY(launch_unpack(sl->d_tiles, n, max_px, H, src, dst, s));
    HIP_TRY(hipEventRecord(sl->done, s));
    sl->pending = true;
    return MIRT_OK;
}
}  // namespace

int mirt_unpack_tiles_async(mirt_ctx* c, uint32_t W, uint32_t H, const mirt_tile* tiles, uint32_t n,
                            const mirt_outputs* packed, const mirt_outputs* fb, void* stream) {
    return unpack_impl(c, W, H, tiles, nullptr, n, packed, fb, stream);
}

int mirt_unpack_tiles_at_async(mirt_ctx* c, uint32_t W, uint32_t H, const mirt_tile* tiles, const uint64_t* offsets,
                               uint32_t n, const mirt_outputs* packed, const mirt_outputs* fb, void* stream) {
    if (!offsets) return fail(MIRT_E_INVALID, "offsets is NULL");
    return unpack_impl(c, W, H, tiles, offsets, n, packed, fb, stream);
}

int mirt_trace_rays(mirt_ctx* c, const mirt_frame* f, uint32_t n, const double* orig, const double* dir, uint8_t* ok,
                    double* hit, double* normal, int32_t* face, int32_t* object) {
    if (!c || !orig || !dir || !ok || !hit || !normal || !face || !object)
        return fail(MIRT_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    int r = check_frame(c, f);
    if (r != MIRT_OK) return r;
    if (n == 0) return MIRT_OK;
    Slot* sl = nullptr;
    if ((r = slot_acquire(c, sl)) != MIRT_OK) return r;
    SlotGuard guard{c, sl};
    const size_t need = (size_t)n * (24 * 4 + 1 + 8) + 128;
    uint8_t* base = (uint8_t*)sl->out_buf;
    size_t cap = sl->out_cap;
    if ((r = dev_grow(base, cap, need)) != MIRT_OK) return r;
    sl->out_buf = base;
    sl->out_cap = cap;
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        uint8_t* p = base + off;
        off += (bytes + 15) & ~(size_t)15;
        return p;
    };
    RayIO io;
    io.orig = (const double*)carve((size_t)n * 24);
    io.dir = (const double*)carve((size_t)n * 24);
    io.hit = (double*)carve((size_t)n * 24);
    io.normal = (double*)carve((size_t)n * 24);
    io.face = (int32_t*)carve((size_t)n * 4);
    io.object = (int32_t*)carve((size_t)n * 4);
    io.ok = carve(n);
    io.n = n;
    hipStream_t s = nullptr;
    if ((r = slot_stream(sl, s)) != MIRT_OK) return r;
    FrameArgs fa;
    uint64_t tris;
    fill_args(c, f, 1, 1, fa, tris);
    fa.flags &= ~MIRT_OPT_LDS_STREAM;  // k_trace's option (k_rays has no slices)
    HIP_TRY(hipMemcpyAsync((void*)io.orig, orig, (size_t)n * 24, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync((void*)io.dir, dir, (size_t)n * 24, hipMemcpyHostToDevice, s));
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(((uint64_t)n + kWG - 1) / kWG, kWgPerCu * (uint64_t)c->cus));
    HIP_TRY(launch_rays(fa, io, grid, c->flags, s));
    HIP_TRY(hipMemcpyAsync(ok, io.ok, n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(hit, io.hit, (size_t)n * 24, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(normal, io.normal, (size_t)n * 24, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(face, io.face, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(object, io.object, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return MIRT_OK;
}

int mirt_profile_enable(mirt_ctx* c, int enable) {
    if (!c) return fail(MIRT_E_INVALID, "NULL context");
    HIP_TRY(hipSetDevice(c->device));
    if (enable && !c->prof_acc) {
        HIP_TRY(hipMalloc((void**)&c->prof_acc, kProfN * sizeof(cnt_t)));
        HIP_TRY(hipMemset(c->prof_acc, 0, kProfN * sizeof(cnt_t)));
    }
    c->profiling = enable != 0;
    return MIRT_OK;
}

int mirt_profile_read(mirt_ctx* c, mirt_profile* out) {
    if (!c || !out) return fail(MIRT_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    std::vector<ProfRec> recs;
    {
        std::lock_guard<std::mutex> g(c->mu);
        recs.swap(c->prof_pending);
    }
    memset(out, 0, sizeof(*out));
    std::vector<float> prim, whole;
    prim.reserve(recs.size());
    whole.reserve(recs.size());
    for (auto& r : recs) {
        HIP_TRY(hipEventSynchronize(r.ev[3]));
        float a = 0, b = 0, d = 0, t = 0;
        HIP_TRY(hipEventElapsedTime(&a, r.ev[0], r.ev[1]));
        HIP_TRY(hipEventElapsedTime(&b, r.ev[1], r.ev[2]));
        HIP_TRY(hipEventElapsedTime(&d, r.ev[2], r.ev[3]));
        HIP_TRY(hipEventElapsedTime(&t, r.ev[0], r.ev[3]));
        out->launches++;
        out->frames += r.frames;
        out->primary_ms_sum += a;
        out->shadow_ms_sum += b;
        out->reflect_ms_sum += d;
        out->frame_ms_sum += t;
        out->primary_rays += r.pixels;
        prim.push_back(a);
        whole.push_back(t);
    }
    auto median = [](std::vector<float>& v) -> double {
        if (v.empty()) return 0.0;
        size_t h = v.size() / 2;
        std::nth_element(v.begin(), v.begin() + h, v.end());
        double m = v[h];
        if (v.size() % 2 == 0) m = 0.5 * (m + *std::max_element(v.begin(), v.begin() + h));
        return m;
    };
    out->primary_ms_median = median(prim);
    out->frame_ms_median = median(whole);
    if (c->prof_acc) {
        cnt_t acc[kProfN];
        HIP_TRY(hipMemcpy(acc, c->prof_acc, sizeof(acc), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemset(c->prof_acc, 0, sizeof(acc)));
        out->hits = acc[kStatHits];
        out->shadow_rays = acc[kStatShadowRays];
        out->primary_tri_tests = acc[kStatPrimTests];
        out->shadow_tri_tests = acc[kStatShadowTests];
        out->primary_node_visits = acc[kStatPrimNodes];
        out->primary_leaf_visits = acc[kStatPrimLeaves];
        out->shadow_node_visits = acc[kStatShadowNodes];
        out->shadow_leaf_visits = acc[kStatShadowLeaves];
        out->stack_overflows = acc[kStatOverflow];
        out->reflection_rays = acc[kStatReflRays];
        out->redo_items = acc[kProfRedo];
    }
    std::lock_guard<std::mutex> g(c->mu);
    for (auto& r : recs) c->prof_free.push_back(r);
    return MIRT_OK;
}

int mirt_debug_timeline(mirt_ctx* c, uint64_t* out, uint32_t max_records) {
    if (!c || !out) return fail(MIRT_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    if (!c->timeline) return 0;
    HIP_TRY(hipDeviceSynchronize());
    std::vector<uint64_t> all((size_t)kTimelineRec * 2 * c->timeline_cap);
    HIP_TRY(hipMemcpy(all.data(), c->timeline, all.size() * 8, hipMemcpyDeviceToHost));
    uint32_t n = 0;
    for (size_t r = 0; r < (size_t)2 * c->timeline_cap && n < max_records; ++r) {
        const uint64_t* rec = &all[r * kTimelineRec];
        if (rec[2] == 0) continue;  // wave slot not launched
        memcpy(out + (size_t)n * kTimelineRec, rec, kTimelineRec * 8);
        ++n;
    }
    return (int)n;
}

int mirt_debug_light_table(const double* tri, uint32_t n, double scale, const double pos[3], const double* lights,
                           uint32_t nl, float* out) {
    if ((n && !tri) || !pos || (nl && !lights) || (n && nl && !out)) return fail(MIRT_E_INVALID, "NULL argument");
    light_records(tri, n, scale, pos, (const double(*)[3])lights, nl, out);
    return MIRT_OK;
}

int mirt_debug_counters(mirt_ctx* c, uint64_t* out, uint32_t n) {
    if (!c || !out) return fail(MIRT_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(read_diag_counters(out, n));
    return MIRT_OK;
}

int mirt_debug_fp64(mirt_ctx* c, int op, uint32_t n, const double* a, const double* b, double* out) {
    if (!c || !a || !b || !out || op < 0 || op > 4) return fail(MIRT_E_INVALID, "bad argument");
    if (n == 0) return MIRT_OK;
    HIP_TRY(hipSetDevice(c->device));
    const size_t w = op == 4 ? 6 : 1;  // op 4: six doubles per ray and per box
    double* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, (size_t)n * 8 * (2 * w + 1)));
    hipError_t e = hipMemcpy(d, a, (size_t)n * 8 * w, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + w * n, b, (size_t)n * 8 * w, hipMemcpyHostToDevice);
    double* o = d + 2 * w * (size_t)n;
    if (e == hipSuccess) e = launch_debug_fp64(op, n, d, d + w * n, o, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, o, (size_t)n * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "mirt_debug_fp64");
    return MIRT_OK;
}

int mirt_set_options(mirt_ctx* c, uint32_t flags) {
    if (!c) return fail(MIRT_E_INVALID, "NULL context");
    c->flags = flags;
    return MIRT_OK;
}

int mirt_stream_create(mirt_ctx* c, void** out) {
    if (!c || !out) return fail(MIRT_E_INVALID, "NULL argument");
    *out = nullptr;
    HIP_TRY(hipSetDevice(c->device));
    std::vector<uint32_t> mask(((uint32_t)c->cus + 31) / 32, 0u);
    for (int i = 0; i < c->cus; ++i) mask[i / 32] |= 1u << (i % 32);
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    *out = (void*)s;
    return MIRT_OK;
}

int mirt_stream_destroy(mirt_ctx* c, void* stream) {
    if (!c || !stream) return fail(MIRT_E_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return MIRT_OK;
}

int mirt_set_grid(mirt_ctx* c, uint32_t min_blocks_per_wg, uint32_t max_workgroups) {
    if (!c) return fail(MIRT_E_INVALID, "NULL context");
    if (min_blocks_per_wg == 0) return fail(MIRT_E_INVALID, "min_blocks_per_wg must be >= 1");
    std::lock_guard<std::mutex> g(c->mu);
    c->min_blocks_per_wg = min_blocks_per_wg;
    c->max_workgroups = max_workgroups;
    return MIRT_OK;
}

}  // extern "C"

// ==================================================================== multi-GPU frame group
// SURVEY.md §8(b) mirt_trace_frame: the frame split over the GPUs of one box, one process
// per GPU, the packed tiles gathered to the root over RCCL and unpacked there — the whole
// per-frame sequence in native code (the torch.distributed version in framebuffer.py costs
// ~60 us of host time per frame, tools/dist_host_probe.py).  RCCL is opened at run time
// (dlopen of librccl.so.1: the copy torch already loaded, else /opt/rocm's), so the library
// loads without it and single-GPU callers never touch it.
namespace mirt {

static Rccl load_rccl() {
    Rccl R;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        const char* e = dlerror();
        R.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
        return R;
    }
#define MIRT_RCCL_SYM(field, name)                                  \
    R.field = (decltype(R.field))dlsym(h, name);                    \
    if (!R.field) {                                                 \
        R.err = std::string("librccl.so.1 does not export ") + name; \
        return R;                                                   \
    }
    MIRT_RCCL_SYM(get_unique_id, "ncclGetUniqueId")
    MIRT_RCCL_SYM(comm_init_rank, "ncclCommInitRank")
    MIRT_RCCL_SYM(comm_destroy, "ncclCommDestroy")
    MIRT_RCCL_SYM(send, "ncclSend")
    MIRT_RCCL_SYM(recv, "ncclRecv")
    MIRT_RCCL_SYM(group_start, "ncclGroupStart")
    MIRT_RCCL_SYM(group_end, "ncclGroupEnd")
    MIRT_RCCL_SYM(error_string, "ncclGetErrorString")
#undef MIRT_RCCL_SYM
    R.comm_abort = (decltype(R.comm_abort))dlsym(h, "ncclCommAbort");
    R.comm_init_all = (decltype(R.comm_init_all))dlsym(h, "ncclCommInitAll");
    R.comm_shrink = (decltype(R.comm_shrink))dlsym(h, "ncclCommShrink");
    R.ok = true;
    return R;
}

const Rccl& rccl() {
    static const Rccl R = load_rccl();  // thread-safe one-time initialisation
    return R;
}

int set_error(int code, const std::string& msg) { return fail(code, msg); }

int trace_tiles_enqueue(mirt_ctx* c, const mirt_frame* f, uint32_t W, uint32_t H, const mirt_tile* tiles,
                        uint32_t n, const OutPlanes& out, hipStream_t s, const volatile int* cancel,
                        cnt_t* h_summary, uint64_t* pixels) {
    HIP_TRY(hipSetDevice(c->device));
    int r = check_frame(c, f);
    if (r != MIRT_OK) return r;
    Slot* sl = nullptr;
    if ((r = slot_acquire(c, sl, tiles, n)) != MIRT_OK) return r;
    SlotGuard guard{c, sl};
    uint64_t tris = 0;
    if ((r = enqueue_trace(c, sl, f, W, H, tiles, n, out, s, cancel, pixels, &tris)) != MIRT_OK) {
        (void)hipStreamSynchronize(s);
        sl->pending = false;
        return r;
    }
    // the slot's next user waits for `done` (slot_acquire): recorded again after the copy's
    // read of sl->summary
    HIP_TRY(hipMemcpyAsync(h_summary, sl->summary, kStatN * sizeof(cnt_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(sl->done, s));
    sl->pending = true;
    return MIRT_OK;
}

}  // namespace mirt

namespace {

#define RCCL_TRY(expr)                                                                           \
    do {                                                                                         \
        ncclResult_t _r = (expr);                                                                \
        if (_r != ncclSuccess) return fail(MIRT_E_DEVICE, std::string(#expr) + ": " + rccl().error_string(_r)); \
    } while (0)

// The tile deal of framebuffer.py (plan_tiles + assign): raster tiles; the tile in column c
// of tile row r goes to rank (c + s r) % world, s the smallest integer >= sqrt(world)
// coprime with world.
uint32_t deal_skew(uint32_t world) {
    uint32_t s = 1;
    auto gcd = [](uint32_t a, uint32_t b) {
        while (b) {
            const uint32_t t = a % b;
            a = b;
            b = t;
        }
        return a;
    };
    while (s * s < world || gcd(s, world) != 1) ++s;
    return s;
}

// tile_h == 0: full-height column strips (contiguous in the column-major framebuffer).
// The frame group's deal weights rank 0 down: the root also unpacks every frame (~1/32 of a
// whole frame's trace time, measured: tools/rehearsal_table.sh), so of every L = a + b (N-1)
// consecutive deal slots it takes a = b - 1 and every other rank b = round(32 / N) (N = 8:
// 3 and 4 of 31).  Slots are interleaved by stride scheduling (smallest (2 count + 1) /
// weight first, ties to the lower rank).
void deal_pattern(uint32_t world, bool weighted, std::vector<uint32_t>& P) {
    P.clear();
    const uint32_t b = weighted ? std::max<uint32_t>(1, (32 + world / 2) / world) : 1;
    const uint32_t a = b >= 2 ? b - 1 : b;
    std::vector<uint64_t> w(world, b), cnt(world, 0);
    w[0] = a;
    const uint64_t L = a + (uint64_t)b * (world - 1);
    for (uint64_t p = 0; p < L; ++p) {
        uint32_t best = 0;
        for (uint32_t q = 1; q < world; ++q)
            if ((2 * cnt[q] + 1) * w[best] < (2 * cnt[best] + 1) * w[q]) best = q;
        ++cnt[best];
        P.push_back(best);
    }
}

void plan_rank_tiles(uint32_t W, uint32_t H, uint32_t tile, uint32_t tile_h, uint32_t world, uint32_t rank,
                     std::vector<mirt_tile>& out, bool weighted = false) {
    out.clear();
    const uint32_t th = tile_h ? tile_h : H;
    const uint32_t cols = (W + tile - 1) / tile;
    std::vector<uint32_t> P;
    deal_pattern(std::max<uint32_t>(world, 1), weighted && world > 1, P);
    const uint64_t L = P.size();
    const uint32_t s = deal_skew((uint32_t)L);  // == deal_skew(world) unweighted (L == world)
    uint64_t k = 0;
    for (uint32_t y = 0; y < H; y += th)
        for (uint32_t x = 0; x < W; x += tile, ++k)
            if (world <= 1 || P[((k % cols) + (uint64_t)s * (k / cols)) % L] == rank)
                out.push_back(mirt_tile{x, y, std::min(tile, W - x), std::min(th, H - y)});
}

uint64_t tiles_pixels(const std::vector<mirt_tile>& t) {
    uint64_t n = 0;
    for (const mirt_tile& x : t) n += (uint64_t)x.w * x.h;
    return n;
}

// A stream on a hardware queue of its own whose kernels run on CUs [lo, hi) (default: all).
hipError_t stream_with_queue(int cus, hipStream_t* s, int lo = 0, int hi = -1) {
    if (hi < 0) hi = cus;
    std::vector<uint32_t> mask(((uint32_t)cus + 31) / 32, 0u);
    for (int i = lo; i < hi; ++i) mask[i / 32] |= 1u << (i % 32);
    return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

// The frame's hit rectangle [x0, x1) x [y0, y1): the pixels whose ray can meet the object.
// A ray that meets a triangle passes through a root child's box, so its (s, t) lies in that
// child's frustum rectangle (frustum_args: conservative, the block pre-test relies on it);
// pixel i's s is (float)(sB - sA i), non-increasing in i, and likewise t in j.  Frames
// without the pre-test (several objects, culling off) use the whole screen.
void hit_rect(const FrameRec& rec, uint32_t W, uint32_t H, uint32_t out[4]) {
    out[0] = 0;
    out[1] = 0;
    out[2] = W;
    out[3] = H;
    const FrustumArgs& fr = rec.fr;
    if (!fr.on) return;
    float slo = INFINITY, shi = -INFINITY, tlo = INFINITY, thi = -INFINITY;
    for (int c = 0; c < 8; ++c) {
        if (!(fr.rect[c][0] <= fr.rect[c][1]) || !(fr.rect[c][2] <= fr.rect[c][3])) continue;  // empty
        slo = std::min(slo, fr.rect[c][0]);
        shi = std::max(shi, fr.rect[c][1]);
        tlo = std::min(tlo, fr.rect[c][2]);
        thi = std::max(thi, fr.rect[c][3]);
    }
    if (!(slo <= shi)) {  // no child can be met: nothing to send
        out[2] = out[0];
        out[3] = out[1];
        return;
    }
    // first and last index whose value v(i) = (float)(B - A i) lies in [lo, hi] (v non-increasing)
    auto span = [](double A, double B, float lo, float hi, uint32_t n, uint32_t& a, uint32_t& b) {
        auto v = [&](int64_t i) { return (float)(B - A * (double)i); };
        int64_t i0 = 0, i1 = (int64_t)n - 1;
        if (std::isfinite(hi) && A > 0) {  // smallest i with v(i) <= hi
            int64_t k = (int64_t)std::max(0.0, std::min((double)n, std::floor((B - (double)hi) / A))) - 2;
            k = std::max<int64_t>(k, 0);
            while (k < (int64_t)n && v(k) > hi) ++k;
            while (k > 0 && v(k - 1) <= hi) --k;
            i0 = k;
        }
        if (std::isfinite(lo) && A > 0) {  // largest i with v(i) >= lo
            int64_t k = (int64_t)std::max(-1.0, std::min((double)n - 1, std::ceil((B - (double)lo) / A))) + 2;
            k = std::min<int64_t>(k, (int64_t)n - 1);
            while (k >= 0 && v(k) < lo) --k;
            while (k + 1 < (int64_t)n && v(k + 1) >= lo) ++k;
            i1 = k;
        }
        if (i1 < i0) {
            a = b = 0;
            return;
        }
        a = (uint32_t)i0;
        b = (uint32_t)(i1 + 1);
    };
    uint32_t x0, x1, y0, y1;
    span(fr.sA, fr.sB, slo, shi, W, x0, x1);
    span(fr.tA, fr.tB, tlo, thi, H, y0, y1);
    if (x0 >= x1 || y0 >= y1) x0 = x1 = y0 = y1 = 0;
    out[0] = x0;
    out[1] = y0;
    out[2] = x1;
    out[3] = y1;
}

// Pixels of a tile list inside a hit rectangle (k_pack_rect's transfer size in words).
uint64_t rect_pixels(const std::vector<mirt_tile>& tiles, const uint32_t R[4]) {
    uint64_t n = 0;
    for (const mirt_tile& t : tiles) {
        const uint32_t x0 = std::max(t.x, R[0]), x1 = std::min(t.x + t.w, R[2]);
        const uint32_t y0 = std::max(t.y, R[1]), y1 = std::min(t.y + t.h, R[3]);
        if (x1 > x0 && y1 > y0) n += (uint64_t)(x1 - x0) * (y1 - y0);
    }
    return n;
}

// A share of full-height strips written by k_trace in its transfer form (FrameRec::xf):
// k_pack_rect's layout of the share's columns inside R, trailer {tag, words} after the data.
// The share's tiles are in screen order, so its packed columns ascend with x.
void share_xfer(const std::vector<mirt_tile>& tiles, const uint32_t R[4], uint32_t tag, XferArgs& xf) {
    uint32_t kA = 0, kB = 0;
    for (const mirt_tile& t : tiles) {
        kA += R[0] > t.x ? std::min(t.w, R[0] - t.x) : 0u;
        kB += R[2] > t.x ? std::min(t.w, R[2] - t.x) : 0u;
    }
    const uint32_t ch = R[3] > R[1] && R[2] > R[0] ? R[3] - R[1] : 0u;
    xf.on = 1;
    xf.k0 = kA;
    xf.x0 = R[0];
    xf.x1 = R[2];
    xf.y0 = R[1];
    xf.ch = ch;
    xf.words = (kB - kA) * ch;
    xf.tag = tag;
}

// One rank's share of the deal, traced by this process: normally this rank's own; in the
// emulated world (mirt_group_emulate) every rank's, so one GPU runs the whole N-rank
// pack -> transfer -> check -> unpack chain.
struct Share {
    uint32_t q = 0;                            // deal index (0: the root's share)
    std::vector<mirt_tile> tiles;
    TileDesc* d_tiles = nullptr;               // tiles at their offsets in the share's rgbv plane
    std::vector<uint32_t*> packed;             // tiled, per frame slot: the share's rgbv plane
    std::vector<uint32_t*> sendbuf;            // tiled non-root share, per frame slot: transfer form
    std::vector<std::unique_ptr<Slot>> slots;  // per batch slot: trace workspace
};

// A launched batch (per batch slot): its frames, their slots and hit rectangles.
struct BatchRec {
    uint32_t n = 0;
    uint64_t first = 0;                        // frames first .. first + n - 1
    uint32_t j[kMaxFrames] = {};               // their frame slots
    uint32_t rect[kMaxFrames][4] = {};
    bool checked = true;                       // trailer results folded into the frame states
};

// Host copy of one frame slot's framebuffer (mirt_group_set_host_output).
struct HostFrame {
    uint8_t* rgb8 = nullptr;
    uint8_t* valid = nullptr;
    uint32_t rect[4] = {0, 0, 0, 0};           // the region last copied (the rest is zero)
};

}  // namespace

struct mirt_group {
    mirt_ctx* c = nullptr;
    int rank = 0, world = 1;
    uint32_t W = 0, H = 0, F = 1, tile = 0, tile_h = 0;
    bool tiled = false;                 // packed rgbv tiles + unpack (world > 1, or a tiled rehearsal)
    ncclComm_t comm = nullptr;          // ranks of the communicator == deal indices
    hipStream_t comm_stream = nullptr;  // every RCCL call, in issue order (the same on every rank)
    hipEvent_t ev_comm = nullptr;
    std::vector<hipStream_t> streams;   // batch slot b runs on streams[b]
    std::vector<hipEvent_t> ev_traced, ev_gathered, ev_done;
    // the deal: deal index i is rank members[i] (members[0] = 0, the root)
    std::vector<uint32_t> members;
    std::vector<std::vector<mirt_tile>> plans;  // every deal index's tiles (the transfer sizes)
    uint64_t cap = 0;                   // largest share (pixels)
    uint64_t stride = 0;                // words per gathered region / transfer buffer (cap + trailer)
    int my_index = 0;
    std::vector<Share> shares;
    std::vector<OutPlanes> fb;          // root: the framebuffers, one per frame slot
    std::vector<void*> own;             // framebuffer planes the group allocated (fbs == NULL)
    std::vector<uint32_t*> gathered;    // root, per frame slot: plan regions of `stride` words
    TileDesc* d_unpack = nullptr;       // root: every share's tiles at their region offsets
    uint32_t n_unpack = 0;
    RegionDesc* d_regions = nullptr;
    uint64_t max_tile_px = 0;
    uint8_t* h_bad = nullptr;           // root, pinned: [frame slot][region] trailer verdicts
    size_t h_bad_cap = 0;
    // modes
    uint32_t emulate = 0;               // > 1: the emulated world (mirt_group_emulate)
    uint64_t emu_drop = 0;              // emulated deal indices whose transfer is dropped (fault injection)
    bool rehearse = false;              // MIRT_GROUP_REHEARSE diagnostic (timing only: no checks)
    bool skip_unpack = false;
    bool host_out = false;
    bool d2h_sdma = false;              // MIRT_D2H=sdma: copy-engine column ranges (default: zero-copy kernel)
    // launch grid by the launches still running (MIRT_ADAPTIVE_GRID): 0 (default) fixed; 1 the
    // chip shared among them; 2 the whole chip for a launch issued when none is running (a
    // lone frame, the first of a burst), the fixed grid otherwise
    uint32_t adaptive_grid = 0;
    // Lone-frame hold (whole-screen groups of one rank; MIRT_LONE_HOLD=0 turns it off): a full
    // batch submitted while the group's last launch has ended is held, not launched.  The next
    // mirt_trace_frame launches it with the fixed grid (a burst has begun); mirt_group_wait or
    // mirt_group_frame_host launch it alone with the whole chip (kWgPerCu per CU), which a
    // caller that waits on each frame (a BulkTrace order) gets.
    bool lone_hold = false;
    bool held = false;                  // the open batch is full and held
    bool lone_next = false;             // the next group_flush launches with the whole chip
    int d2h_cus = 0;                    // CUs reserved for the host copies (0: copies on the frame stream)
    // Fused host copies (whole-screen groups of one rank with FB >= 8 launches in flight, or any
    // even FB with MIRT_FUSED_COPY=1; =0: off): FB / 2 streams (half_streams), so the F frame
    // slots cover two launches per stream, and a batch's host copy runs inside the next k_trace
    // launch on its stream (its first waves, reading framebuffers that launch does not write)
    // instead of as a kernel between the stream's traces; its ev_done is recorded after that
    // launch.
    bool half_streams = false;
    bool fused_copy = false;
    struct PendingCopy {
        bool on = false;
        uint32_t hs = 0;                // the batch's host ring slot (its ev_done)
        uint32_t cols = 0;
        FusedCopy fc{};
    };
    std::vector<PendingCopy> pend;     // per stream
    hipStream_t copy_stream = nullptr;
    std::vector<HostFrame> hfb;
    uint32_t* d_spans = nullptr;        // host output: per frame slot and column, the hit span the host holds
    // frames and batches
    uint32_t B = 1, FB = 1;
    // Host run-ahead: batch records and events form a ring of HB = FB x runahead entries, so
    // the host enqueues up to runahead x FB batches while the device runs FB at a time (one
    // per stream).  With HB = FB the host waited for batch nb - FB before enqueueing batch nb
    // and its stream sat idle from that batch's end until the host's launch reached it
    // (~20 us per stream cycle in the kernel trace).  Device resources stay per stream
    // (stream order protects them); run-ahead is off (1) for multi-frame batches, whose
    // records are staged in pinned host memory per stream slot, and for tiled groups
    // (per-slot trailer verdicts, transfers).
    uint32_t HB = 1, runahead = 1;
    uint64_t nb = 0;                    // batches launched
    uint64_t k = 0;                     // frames enqueued
    uint32_t bn = 0;                    // frames in the open batch
    uint32_t bj[kMaxFrames] = {};
    FrameRec stage[kMaxFrames];         // the open batch's records (copied per share at launch)
    uint32_t bbounces = 0;
    std::vector<BatchRec> binfo;        // per host ring slot (HB)
    std::vector<uint64_t> slot_frame;   // per frame slot: the frame it holds (~0: none)
    // per frame slot: only [dirty0, dirty1) x [dirty_y0, dirty_y1) may hold non-miss pixels
    // (whole-screen planes); a narrow frame refills those columns before it traces its hit
    // rectangle, unless the rectangle covers them (the trace rewrites every pixel in it).
    // Tiled groups (root): [dirty0, dirty1) are the columns the last unpack into the slot's
    // framebuffer may have left non-miss; the next unpack rewrites them and its own rectangle.
    std::vector<uint32_t> dirty0, dirty1, dirty_y0, dirty_y1;
    std::vector<uint64_t> slot_bad;     // per frame slot: deal indices whose transfer failed
    // fault handling (master/pool/pool.go:224-260, master/main.go:111-161)
    uint32_t timeout_ms = 0;
    bool spin_wait = false;  // MIRT_WAIT=spin: poll completion events (no blocking wait)
    uint64_t failed_mask = 0;           // ranks (not deal indices) named by the last failure
    uint64_t pending_bad = 0;           // deal indices failed since the last mirt_group_wait
    uint64_t pending_bad_frame = ~0ull;
    bool broken = false;                // a wait timed out: only mirt_group_exclude / destroy
    bool no_fused_pack = false;         // MIRT_NO_FUSED_PACK: k_pack_rect after the trace (A/B)
    hipStream_t probe_stream = nullptr;
};

namespace {

uint64_t now_us() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// The host ring (see mirt_group::HB): run-ahead only for one-frame batches of untiled groups.
void group_ring(mirt_group* g) {
    g->HB = g->FB * ((g->B == 1 && !g->tiled) ? g->runahead : 1u);
}

// Wait for a group event, within the group's deadline (0: no deadline).
// Polling: the first kSpinWaitUs are a busy poll (a frame completes within tens of
// microseconds, and a sleep would add the OS timer slack, ~50 us, to the wait), then 20 us
// sleeps between polls.
constexpr uint64_t kSpinWaitUs = 2000;
int group_wait_event(mirt_group* g, hipEvent_t ev, const char* what) {
    if (!g->timeout_ms && !g->spin_wait) {
        HIP_TRY(hipEventSynchronize(ev));
        return MIRT_OK;
    }
    const uint64_t t0 = now_us();
    const uint64_t deadline = g->timeout_ms ? t0 + (uint64_t)g->timeout_ms * 1000 : UINT64_MAX;
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return MIRT_OK;
        if (e != hipErrorNotReady) return hip_fail(e, what);
        const uint64_t now = now_us();
        if (now > deadline)
            return fail(MIRT_E_TIMEOUT, std::string(what) + ": no completion within " + std::to_string(g->timeout_ms) +
                                            " ms");
        if (now - t0 > kSpinWaitUs) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Transfer words of deal index q for a frame with hit rectangle R (data + trailer).
uint64_t transfer_words(const mirt_group* g, uint32_t q, const uint32_t R[4]) {
    return rect_pixels(g->plans[q], R) + kTrailerWords;
}

uint64_t mask_of_ranks(const mirt_group* g, uint64_t deal_mask) {
    uint64_t m = 0;
    for (size_t i = 0; i < g->members.size() && i < 64; ++i)
        if ((deal_mask >> i) & 1u) m |= 1ull << (g->members[i] & 63u);
    return m;
}

// A batch known to be complete: fold its frames' trailer verdicts into the frame states.
void batch_fold(mirt_group* g, uint32_t bs) {
    BatchRec& br = g->binfo[bs];
    if (br.checked) return;
    br.checked = true;
    if (!g->tiled || g->rank != 0 || g->rehearse || g->skip_unpack) return;
    const size_t P = g->members.size();
    for (uint32_t i = 0; i < br.n; ++i) {
        const uint32_t j = br.j[i];
        uint64_t bad = 0;
        for (size_t q = 0; q < P && q < 64; ++q)
            if (g->h_bad[(size_t)j * P + q]) bad |= 1ull << q;
        g->slot_bad[j] = bad;
        if (bad) {
            g->pending_bad |= bad;
            if (g->pending_bad_frame == ~0ull) g->pending_bad_frame = br.first + i;
        }
    }
}

std::string ranks_text(uint64_t m) {
    std::string s;
    for (int r = 0; r < 64; ++r)
        if ((m >> r) & 1u) s += (s.empty() ? "" : ",") + std::to_string(r);
    return s;
}

// After a timeout on the root: which transfers of the stuck batch never arrived intact?
// The trailers are read straight from the gathered regions on a stream of their own.
uint64_t probe_failed(mirt_group* g, uint32_t bs) {
    const BatchRec& br = g->binfo[bs];
    const size_t P = g->members.size();
    if (g->rank != 0 || !g->tiled) return 1;  // a sender only talks to the root
    uint64_t bad = 0;
    if (!g->probe_stream && hipStreamCreateWithFlags(&g->probe_stream, hipStreamNonBlocking) != hipSuccess)
        return ~0ull;
    uint32_t* h = nullptr;
    if (hipHostMalloc((void**)&h, sizeof(uint32_t) * 2 * P * kMaxFrames) != hipSuccess) return ~0ull;
    for (uint32_t i = 0; i < br.n; ++i)
        for (size_t q = 1; q < P; ++q) {
            const uint64_t words = rect_pixels(g->plans[q], br.rect[i]);
            (void)hipMemcpyAsync(h + 2 * (i * P + q), g->gathered[br.j[i]] + q * g->stride + words, 8,
                                 hipMemcpyDeviceToHost, g->probe_stream);
        }
    hipEvent_t ev = nullptr;
    bool done = false;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess &&
        hipEventRecord(ev, g->probe_stream) == hipSuccess) {
        const uint64_t deadline = now_us() + 1000000;
        while (!(done = hipEventQuery(ev) == hipSuccess) && now_us() < deadline)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (ev) (void)hipEventDestroy(ev);
    if (!done) {
        bad = ~1ull;  // the device does not answer: every peer is suspect
    } else {
        for (uint32_t i = 0; i < br.n; ++i)
            for (size_t q = 1; q < P && q < 64; ++q) {
                const uint64_t words = rect_pixels(g->plans[q], br.rect[i]);
                const uint32_t* t = h + 2 * (i * P + q);
                if (t[0] != transfer_tag(br.first + i) || t[1] != (uint32_t)words) bad |= 1ull << q;
            }
    }
    (void)hipHostFree(h);
    return bad;
}

int group_timed_out(mirt_group* g, uint32_t bs, int r) {
    if (r != MIRT_E_TIMEOUT) return r;
    const uint64_t bad = probe_failed(g, bs);
    g->failed_mask = mask_of_ranks(g, bad) & ~(g->rank == 0 ? 1ull : 0ull);
    if (g->rank != 0) g->failed_mask = 1;  // a sender waits on the root only
    g->broken = true;
    const BatchRec& br = g->binfo[bs];
    return fail(MIRT_E_TIMEOUT, "frames " + std::to_string(br.first) + ".." + std::to_string(br.first + br.n - 1) +
                                    " did not complete within " + std::to_string(g->timeout_ms) +
                                    " ms; transfers missing from rank(s) " +
                                    (g->failed_mask ? ranks_text(g->failed_mask) : std::string("none (local)")) +
                                    " (mirt_group_failed_ranks; mirt_group_exclude re-deals)");
}

// (Re)build the deal over g->members: plans, shares, buffers, the root's unpack tables.
int group_plan(mirt_group* g) {
    const uint32_t P = (uint32_t)g->members.size();
    g->plans.assign(P, {});
    uint64_t cap = 0;
    if (g->tiled) {
        for (uint32_t q = 0; q < P; ++q) {
            plan_rank_tiles(g->W, g->H, g->tile, g->tile_h, P, q, g->plans[q], true);
            if (g->plans[q].empty())
                return fail(MIRT_E_INVALID, "deal index " + std::to_string(q) + " has no tiles (tile too large for " +
                                                std::to_string(P) + " ranks)");
            cap = std::max(cap, tiles_pixels(g->plans[q]));
        }
    } else {
        g->plans[0].push_back(mirt_tile{0, 0, g->W, g->H});
        cap = (uint64_t)g->W * g->H;
    }
    const uint64_t stride = (cap + kTrailerWords + 3) & ~3ull;
    const bool grow = stride > g->stride;
    g->cap = cap;
    g->stride = std::max(g->stride, stride);
    // the shares this process traces
    std::vector<uint32_t> want;
    if (g->emulate > 1) {
        for (uint32_t q = 0; q < P; ++q) want.push_back(q);
    } else if (g->rehearse) {
        const char* rr = getenv("MIRT_GROUP_REHEARSE_RANK");
        want.push_back(rr ? (uint32_t)std::min<int>(std::max(atoi(rr), 0), (int)P - 1) : 0u);
    } else {
        want.push_back((uint32_t)g->my_index);
    }
    // keep existing shares' workspaces (slots), rebuild their tile lists and planes
    while (g->shares.size() > want.size()) {
        Share& sh = g->shares.back();
        for (auto& sl : sh.slots) slot_free(sl.get());
        for (uint32_t* p : sh.packed) (void)hipFree(p);
        for (uint32_t* p : sh.sendbuf) (void)hipFree(p);
        if (sh.d_tiles) (void)hipFree(sh.d_tiles);
        g->shares.pop_back();
    }
    g->shares.resize(want.size());
    for (size_t si = 0; si < want.size(); ++si) {
        Share& sh = g->shares[si];
        sh.q = want[si];
        sh.tiles = g->plans[sh.q];
        while (sh.slots.size() < g->F) {
            sh.slots.emplace_back(new Slot());
            sh.slots.back()->dedicated = true;
            int r = slot_init(sh.slots.back().get());
            if (r != MIRT_OK) return r;
        }
        if (!g->tiled) continue;
        if (grow || sh.packed.empty()) {
            for (uint32_t* p : sh.packed) (void)hipFree(p);
            for (uint32_t* p : sh.sendbuf) (void)hipFree(p);
            sh.packed.assign(g->F, nullptr);
            sh.sendbuf.assign(g->F, nullptr);
            for (uint32_t j = 0; j < g->F; ++j) {
                HIP_TRY(hipMalloc((void**)&sh.packed[j], g->stride * 4));
                HIP_TRY(hipMalloc((void**)&sh.sendbuf[j], g->stride * 4));
            }
        }
        std::vector<TileDesc> md;
        uint64_t o = 0;
        for (const mirt_tile& x : sh.tiles) {
            md.push_back(TileDesc{x.x, x.y, x.w, x.h, o, 0, 0});
            o += (uint64_t)x.w * x.h;
        }
        if (sh.d_tiles) (void)hipFree(sh.d_tiles);
        sh.d_tiles = nullptr;
        HIP_TRY(hipMalloc((void**)&sh.d_tiles, md.size() * sizeof(TileDesc)));
        HIP_TRY(hipMemcpy(sh.d_tiles, md.data(), md.size() * sizeof(TileDesc), hipMemcpyHostToDevice));
    }
    if (g->tiled && g->rank == 0) {
        if (grow || g->gathered.empty() || g->h_bad_cap < (size_t)g->F * P) {
            for (uint32_t* p : g->gathered) (void)hipFree(p);
            g->gathered.assign(g->F, nullptr);
        }
        // sized for the largest deal this group can hold (a deal never grows after creation)
        for (uint32_t j = 0; j < g->F; ++j)
            if (!g->gathered[j]) HIP_TRY(hipMalloc((void**)&g->gathered[j], (size_t)P * g->stride * 4));
        std::vector<TileDesc> td;
        std::vector<RegionDesc> rd;
        g->max_tile_px = 0;
        for (uint32_t q = 0; q < P; ++q) {
            const uint32_t first = (uint32_t)td.size();
            uint64_t o = 0;  // within region q
            for (const mirt_tile& x : g->plans[q]) {
                td.push_back(TileDesc{x.x, x.y, x.w, x.h, o, q, first});
                o += (uint64_t)x.w * x.h;
                g->max_tile_px = std::max<uint64_t>(g->max_tile_px, (uint64_t)x.w * x.h);
            }
            rd.push_back(RegionDesc{first, (uint32_t)(td.size() - first)});
        }
        g->n_unpack = (uint32_t)td.size();
        if (g->d_unpack) (void)hipFree(g->d_unpack);
        if (g->d_regions) (void)hipFree(g->d_regions);
        g->d_unpack = nullptr;
        g->d_regions = nullptr;
        HIP_TRY(hipMalloc((void**)&g->d_unpack, td.size() * sizeof(TileDesc)));
        HIP_TRY(hipMemcpy(g->d_unpack, td.data(), td.size() * sizeof(TileDesc), hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc((void**)&g->d_regions, rd.size() * sizeof(RegionDesc)));
        HIP_TRY(hipMemcpy(g->d_regions, rd.data(), rd.size() * sizeof(RegionDesc), hipMemcpyHostToDevice));
        if (g->h_bad_cap < (size_t)g->F * P) {
            if (g->h_bad) (void)hipHostFree(g->h_bad);
            g->h_bad = nullptr;
            g->h_bad_cap = 0;
            HIP_TRY(hipHostMalloc((void**)&g->h_bad, (size_t)g->F * P));
            g->h_bad_cap = (size_t)g->F * P;
        }
        memset(g->h_bad, 0, g->h_bad_cap);
    }
    return MIRT_OK;
}

// Creation-time agreement of the ranks (world > 1): every sender's view of the group
// {W, H, tile, tile_h, world, inflight, stride, deal checksum} must equal the root's, or
// every rank fails here instead of hanging or corrupting frames later.
uint32_t group_signature(const mirt_group* g) {
    uint32_t h = 2166136261u;
    auto mix = [&](uint32_t v) {
        for (int b = 0; b < 4; ++b) h = (h ^ ((v >> (8 * b)) & 0xffu)) * 16777619u;
    };
    mix(g->W), mix(g->H), mix(g->tile), mix(g->tile_h), mix((uint32_t)g->members.size()), mix(g->F);
    mix((uint32_t)g->stride);
    for (const auto& p : g->plans)
        for (const mirt_tile& t : p) mix(t.x), mix(t.y), mix(t.w), mix(t.h);
    return h;
}

int group_handshake(mirt_group* g) {
    const Rccl& R = rccl();
    const uint32_t P = (uint32_t)g->members.size();
    uint32_t* d = nullptr;  // [P][4] words: root receives, then sends its verdicts
    HIP_TRY(hipMalloc((void**)&d, (size_t)P * 16));
    std::vector<uint32_t> h((size_t)P * 4, 0);
    const uint32_t sig[4] = {0x6d697274u, group_signature(g), (uint32_t)g->my_index, (uint32_t)P};
    int r = MIRT_OK;
    auto step = [&](bool send_phase) -> int {
        RCCL_TRY(R.group_start());
        for (uint32_t q = 1; q < P; ++q) {
            if (g->my_index == 0) {
                if (send_phase) RCCL_TRY(R.send(d + 4 * q, 16, ncclUint8, (int)q, g->comm, g->comm_stream));
                else RCCL_TRY(R.recv(d + 4 * q, 16, ncclUint8, (int)q, g->comm, g->comm_stream));
            } else if ((uint32_t)g->my_index == q) {
                if (send_phase) RCCL_TRY(R.recv(d + 4 * q, 16, ncclUint8, 0, g->comm, g->comm_stream));
                else RCCL_TRY(R.send(d + 4 * q, 16, ncclUint8, 0, g->comm, g->comm_stream));
            }
        }
        RCCL_TRY(R.group_end());
        HIP_TRY(hipEventRecord(g->ev_comm, g->comm_stream));
        return group_wait_event(g, g->ev_comm, "group handshake");
    };
    if (g->my_index != 0) HIP_TRY(hipMemcpy(d + 4 * g->my_index, sig, 16, hipMemcpyHostToDevice));
    if ((r = step(false)) == MIRT_OK) {
        if (g->my_index == 0) {
            HIP_TRY(hipMemcpy(h.data(), d, (size_t)P * 16, hipMemcpyDeviceToHost));
            uint64_t bad = 0;
            for (uint32_t q = 1; q < P; ++q) {
                const uint32_t* s = &h[(size_t)q * 4];
                const bool ok = s[0] == sig[0] && s[1] == sig[1] && s[2] == q && s[3] == P;
                h[(size_t)q * 4] = ok ? 1u : 0u;
                if (!ok) bad |= 1ull << (q & 63u);
            }
            HIP_TRY(hipMemcpy(d, h.data(), (size_t)P * 16, hipMemcpyHostToDevice));
            r = step(true);
            if (r == MIRT_OK && bad) {
                g->failed_mask = mask_of_ranks(g, bad);
                r = fail(MIRT_E_PEER, "group handshake: rank(s) " + ranks_text(g->failed_mask) +
                                          " disagree with the root on W/H/tile/world/inflight or the deal");
            }
        } else {
            r = step(true);
            if (r == MIRT_OK) {
                uint32_t v[4];
                HIP_TRY(hipMemcpy(v, d + 4 * g->my_index, 16, hipMemcpyDeviceToHost));
                if (v[0] != 1u) {
                    g->failed_mask = 1;
                    r = fail(MIRT_E_PEER, "group handshake: the root rejected this rank's view of the group");
                }
            }
        }
    }
    (void)hipFree(d);
    return r;
}

// Device -> host copy of a frame's framebuffer: the union of this frame's hit rectangle
// and the one last copied into that host slot (outside the rectangle every pixel is a
// miss, i.e. zero, so the host planes stay exact).  Stages the frame's job; the batch's
// copies run as one k_copy_rect_host launch storing straight into pinned host memory.
void host_copy_job(mirt_group* g, uint32_t j, const uint32_t R[4], HostCopyJobs& jobs, uint32_t i, uint32_t& max_cols) {
    HostFrame& hf = g->hfb[j];
    const OutPlanes& d = g->fb[j];
    uint32_t u[4] = {R[0], R[1], R[2], R[3]};
    const bool r_empty = R[0] >= R[2] || R[1] >= R[3], p_empty = hf.rect[0] >= hf.rect[2] || hf.rect[1] >= hf.rect[3];
    if (r_empty) memcpy(u, hf.rect, sizeof(u));
    else if (!p_empty) {
        u[0] = std::min(u[0], hf.rect[0]);
        u[1] = std::min(u[1], hf.rect[1]);
        u[2] = std::max(u[2], hf.rect[2]);
        u[3] = std::max(u[3], hf.rect[3]);
    }
    memcpy(hf.rect, R, sizeof(hf.rect));
    if (u[0] >= u[2] || u[1] >= u[3]) u[0] = u[1] = u[2] = u[3] = 0;  // nothing to copy
    jobs.rgb8[i] = d.rgb8;
    jobs.valid[i] = d.valid;
    jobs.hrgb8[i] = hf.rgb8;
    jobs.hvalid[i] = hf.valid;
    jobs.spans[i] = g->d_spans + (size_t)j * g->W;
    memcpy(jobs.rect[i], u, sizeof(u));
    memcpy(jobs.cur[i], R, sizeof(jobs.cur[i]));
    max_cols = std::max(max_cols, u[2] - u[0]);
}

}  // namespace

extern "C" {

int mirt_plan_tiles(uint32_t W, uint32_t H, uint32_t tile, uint32_t tile_h, uint32_t world, uint32_t rank,
                    mirt_tile* out, uint32_t cap) {
    if (!W || !H || !tile || !world || rank >= world) return fail(MIRT_E_INVALID, "bad tile plan arguments");
    std::vector<mirt_tile> t;
    plan_rank_tiles(W, H, tile, tile_h, world, rank, t);
    if (out) {
        if (t.size() > cap) return fail(MIRT_E_LIMIT, "tile buffer too small");
        memcpy(out, t.data(), t.size() * sizeof(mirt_tile));
    }
    return (int)t.size();
}

int mirt_group_plan_tiles(uint32_t W, uint32_t H, uint32_t tile, uint32_t tile_h, uint32_t world, uint32_t rank,
                          mirt_tile* out, uint32_t cap) {
    if (!W || !H || !tile || !world || rank >= world) return fail(MIRT_E_INVALID, "bad tile plan arguments");
    std::vector<mirt_tile> t;
    plan_rank_tiles(W, H, tile, tile_h, world, rank, t, true);
    if (out) {
        if (t.size() > cap) return fail(MIRT_E_LIMIT, "tile buffer too small");
        memcpy(out, t.data(), t.size() * sizeof(mirt_tile));
    }
    return (int)t.size();
}

int mirt_group_unique_id(uint8_t* id) {
    if (!id) return fail(MIRT_E_INVALID, "id is NULL");
    if (!rccl().ok) return fail(MIRT_E_DEVICE, rccl().err);
    ncclUniqueId u;
    RCCL_TRY(rccl().get_unique_id(&u));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return MIRT_OK;
}

void mirt_group_destroy(mirt_group* g) {
    if (!g) return;
#ifdef MIRT_HOST_TIMERS
    fprintf(stderr, "host_timers_us_per_frame wait %.2f record %.2f prep %.2f launch %.2f post+gather %.2f unpack %.2f done %.2f"
                    " | hit_rect %.2f fill %.2f blocks %.2f setup %.2f stage %.2f\n",
            g_ht[0] / g->k, g_ht[1] / g->k, g_ht[2] / g->k, g_ht[3] / g->k, g_ht[4] / g->k, g_ht[5] / g->k, g_ht[6] / g->k,
            g_ht[7] / g->k, g_ht[8] / g->k, g_ht[9] / g->k, g_ht[10] / g->k, g_ht[11] / g->k);
#endif
    (void)hipSetDevice(g->c->device);
    {
        std::lock_guard<std::mutex> gl(g->c->groups_mu);
        auto& v = g->c->groups;
        v.erase(std::remove(v.begin(), v.end(), g), v.end());
    }
    // frames submitted and not launched yet (an open batch, or one held by the lone-frame hold)
    // are traced before the group goes, as mirt_group_wait would; a broken group drops them
    if (g->bn && (g->broken || group_launch_staged(g) != MIRT_OK))
        for (uint32_t i = 0; i < g->bn; ++i) lt_unpin(g->c, g->stage[i].fa.ltab);  // never launched
    g->bn = 0;
    if (g->comm) {
        // a broken group (a peer stopped answering) may have RCCL work that never ends
        if (g->broken && rccl().comm_abort) (void)rccl().comm_abort(g->comm);
        else (void)rccl().comm_destroy(g->comm);
    }
    if (!g->broken) {
        for (hipStream_t s : g->streams)
            if (s) (void)hipStreamSynchronize(s);
        if (g->comm_stream) (void)hipStreamSynchronize(g->comm_stream);
        if (g->copy_stream) (void)hipStreamSynchronize(g->copy_stream);
    }
    for (Share& sh : g->shares) {
        for (auto& sl : sh.slots) slot_free(sl.get());
        for (uint32_t* p : sh.packed) (void)hipFree(p);
        for (uint32_t* p : sh.sendbuf) (void)hipFree(p);
        if (sh.d_tiles) (void)hipFree(sh.d_tiles);
    }
    for (uint32_t* p : g->gathered)
        if (p) (void)hipFree(p);
    if (g->d_unpack) (void)hipFree(g->d_unpack);
    if (g->d_regions) (void)hipFree(g->d_regions);
    if (g->h_bad) (void)hipHostFree(g->h_bad);
    if (g->d_spans) (void)hipFree(g->d_spans);
    for (void* p : g->own) (void)hipFree(p);
    for (HostFrame& hf : g->hfb) {
        if (hf.rgb8) (void)hipHostFree(hf.rgb8);
        if (hf.valid) (void)hipHostFree(hf.valid);
    }
    for (auto* v : {&g->ev_traced, &g->ev_gathered, &g->ev_done})
        for (hipEvent_t e : *v)
            if (e) (void)hipEventDestroy(e);
    if (g->ev_comm) (void)hipEventDestroy(g->ev_comm);
    for (hipStream_t s : g->streams)
        if (s) (void)hipStreamDestroy(s);
    if (g->comm_stream) (void)hipStreamDestroy(g->comm_stream);
    if (g->copy_stream) (void)hipStreamDestroy(g->copy_stream);
    if (g->probe_stream) (void)hipStreamDestroy(g->probe_stream);
    delete g;
}

static int update_fused_copy(mirt_group* g);

int mirt_group_create(mirt_ctx* c, const uint8_t* unique_id, int rank, int world, uint32_t W, uint32_t H,
                      uint32_t tile, uint32_t tile_h, uint32_t inflight, const mirt_outputs* fbs, mirt_group** out) {
    if (!c || !out) return fail(MIRT_E_INVALID, "NULL context or out");
    *out = nullptr;
    if (world < 1 || world > 64 || rank < 0 || rank >= world) return fail(MIRT_E_INVALID, "bad rank / world (1..64)");
    if (!W || !H || W > 65535 || H > 65535) return fail(MIRT_E_INVALID, "bad screen size");
    if (inflight < 1 || inflight > 32) return fail(MIRT_E_INVALID, "inflight must be 1..32");
    if (world > 1 && !unique_id) return fail(MIRT_E_INVALID, "world > 1 needs the root's unique id");
    if (world > 1 && tile == 0) return fail(MIRT_E_INVALID, "world > 1 needs a tile size");
    const bool is_root = rank == 0;
    // the tiled path gathers packed rgbv words (uint8 colour + valid): it cannot produce
    // the fp64 colour or the diagnostic face/object planes
    if (is_root && tile > 0 && fbs)
        for (uint32_t j = 0; j < inflight; ++j)
            if (fbs[j].rgb || fbs[j].face || fbs[j].object)
                return fail(MIRT_E_INVALID, "tiled frame groups produce rgb8 / valid / rgbv only (rgb, face and "
                                            "object planes need tile == 0)");
    // the host copy (kernels.hip copy_column) scans valid planes in aligned 8-byte words: with
    // the plane 8-byte aligned, the last word never leaves the page that holds the plane's last
    // byte, and the bytes past it are masked off
    if (is_root && fbs)
        for (uint32_t j = 0; j < inflight; ++j)
            if ((uintptr_t)fbs[j].valid & 7) return fail(MIRT_E_INVALID, "valid planes must be 8-byte aligned");
    HIP_TRY(hipSetDevice(c->device));
    std::unique_ptr<mirt_group, void (*)(mirt_group*)> g(new mirt_group(), mirt_group_destroy);
    g->c = c;
    g->rank = rank;
    g->world = world;
    g->W = W;
    g->H = H;
    g->F = inflight;
    g->FB = inflight;  // one frame per launch until mirt_group_set_batch
    const char* ra = getenv("MIRT_RUNAHEAD");
    g->runahead = (uint32_t)std::min(std::max(ra ? atoi(ra) : 2, 1), 4);
    g->tile = tile;
    g->tile_h = tile_h;
    g->tiled = tile > 0;
    const char* d2h = getenv("MIRT_D2H");
    g->d2h_sdma = d2h && !strcmp(d2h, "sdma");
    const char* ag = getenv("MIRT_ADAPTIVE_GRID");
    if (ag) g->adaptive_grid = (uint32_t)std::min(std::max(atoi(ag), 0), 2);
    g->no_fused_pack = getenv("MIRT_NO_FUSED_PACK") != nullptr;
    const char* wt = getenv("MIRT_WAIT");
    if (wt) g->spin_wait = !strcmp(wt, "spin");
    // MIRT_GROUP_REHEARSE=N (timing diagnostic, world == 1 only): trace one share of an
    // N-way deal (MIRT_GROUP_REHEARSE_RANK, default 0) and unpack all N regions, the others
    // stale: the root's per-frame GPU work at N GPUs without the transfers.  Results are
    // not checked; mirt_group_emulate is the correctness mode.
    const char* reh = getenv("MIRT_GROUP_REHEARSE");
    const int plan_world = (world == 1 && g->tiled && reh && atoi(reh) > 1) ? std::min(atoi(reh), 64) : world;
    g->rehearse = plan_world != world;
    g->skip_unpack = g->rehearse && getenv("MIRT_GROUP_REHEARSE_NO_UNPACK");
    for (int q = 0; q < plan_world; ++q) g->members.push_back((uint32_t)q);
    g->my_index = rank;
    g->streams.assign(inflight, nullptr);
    const uint32_t ring = inflight * g->runahead;  // the largest HB this group can use
    g->ev_traced.assign(ring, nullptr);
    g->ev_gathered.assign(ring, nullptr);
    g->ev_done.assign(ring, nullptr);
    // host output on reserved CUs (MIRT_D2H_CUS=n): the trace kernels fill every CU's VGPR
    // file, so a copy kernel sharing their CUs waits for a frame tail to start; n CUs kept
    // for the copy stream let each frame's D2H run beside the next frames' traces
    const char* dc = getenv("MIRT_D2H_CUS");
    g->d2h_cus = dc ? std::min(std::max(atoi(dc), 0), c->cus / 2) : 0;
    // the frame streams: each with a hardware queue of its own (a CU-masked stream), so frames in
    // flight run concurrently; MIRT_PLAIN_STREAMS=1 (measurement): plain streams, which share the
    // runtime's hardware queues
    static const bool plain = getenv("MIRT_PLAIN_STREAMS") && atoi(getenv("MIRT_PLAIN_STREAMS"));
    for (uint32_t j = 0; j < inflight; ++j) {
        if (plain && !g->d2h_cus)
            HIP_TRY(hipStreamCreateWithFlags(&g->streams[j], hipStreamNonBlocking));
        else
            HIP_TRY(stream_with_queue(c->cus, &g->streams[j], 0, c->cus - g->d2h_cus));
    }
    for (uint32_t j = 0; j < ring; ++j) {
        HIP_TRY(hipEventCreateWithFlags(&g->ev_traced[j], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&g->ev_gathered[j], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&g->ev_done[j], hipEventDisableTiming));
    }
    HIP_TRY(hipEventCreateWithFlags(&g->ev_comm, hipEventDisableTiming));
    {
        const char* lh = getenv("MIRT_LONE_HOLD");
        g->lone_hold = world == 1 && !g->tiled && !(lh && !strcmp(lh, "0"));
    }
    if (g->d2h_cus) HIP_TRY(stream_with_queue(c->cus, &g->copy_stream, c->cus - g->d2h_cus, c->cus));
    g->binfo.assign(ring, BatchRec());
    group_ring(g.get());
    g->slot_frame.assign(inflight, ~0ull);
    g->slot_bad.assign(inflight, 0);
    g->dirty0.assign(inflight, 0);  // the planes' first contents are unknown: the whole screen
    g->dirty1.assign(inflight, W);
    g->dirty_y0.assign(inflight, 0);
    g->dirty_y1.assign(inflight, H);
    if (is_root && fbs) {
        for (uint32_t j = 0; j < inflight; ++j)
            g->fb.push_back(OutPlanes{fbs[j].rgb, fbs[j].rgb8, fbs[j].valid, fbs[j].face, fbs[j].object, fbs[j].rgbv});
    } else if (is_root) {
        // no framebuffers given (a caller without device memory of its own, e.g. a Go worker
        // reading frames through mirt_group_frame_host): the group owns rgb8 + valid planes
        const size_t n = (size_t)W * H;
        for (uint32_t j = 0; j < inflight; ++j) {
            OutPlanes o{};
            HIP_TRY(hipMalloc((void**)&o.rgb8, 3 * n));
            g->own.push_back(o.rgb8);
            HIP_TRY(hipMalloc((void**)&o.valid, n));
            g->own.push_back(o.valid);
            g->fb.push_back(o);
        }
    }
    if (is_root) {
        // Every framebuffer starts as a frame of misses (colour 0, valid 0, face / object -1), so a
        // slot's first frame refills nothing: before, each slot's first use filled its whole planes
        // on the frame's stream, inside the caller's first F frames (at the driver's 5 warmup and
        // 8 in flight, three 8 MB fills in the timed region, one waiting 52 us for a CU).
        const size_t n = (size_t)W * H;
        for (const OutPlanes& o : g->fb) {
            const struct { void* p; size_t bytes; int v; } planes[kFillPlanes] = {
                {o.rgb, 24 * n, 0}, {o.rgb8, 3 * n, 0}, {o.valid, n, 0}, {o.face, 4 * n, 0xff}, {o.object, 4 * n, 0xff},
                {o.rgbv, 4 * n, 0}};
            for (const auto& pl : planes)
                if (pl.p) HIP_TRY(hipMemsetAsync(pl.p, pl.v, pl.bytes, nullptr));
        }
        HIP_TRY(hipStreamSynchronize(nullptr));  // the group's streams do not order against the null stream
        g->dirty1.assign(inflight, 0);  // [0, 0): nothing to refill
        g->dirty_y1.assign(inflight, 0);
    }
    int r = group_plan(g.get());
    if (r != MIRT_OK) return r;
    if ((r = update_fused_copy(g.get())) != MIRT_OK) return r;  // the stream mapping (half_streams)
    if (world > 1) {
        if (!rccl().ok) return fail(MIRT_E_DEVICE, rccl().err);
        HIP_TRY(stream_with_queue(c->cus, &g->comm_stream));
        ncclUniqueId u;
        memcpy(u.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
        RCCL_TRY(rccl().comm_init_rank(&g->comm, world, u, rank));
        g->timeout_ms = 120000;  // the handshake never waits forever
        r = group_handshake(g.get());
        g->timeout_ms = 0;
        if (r != MIRT_OK) {
            if (r == MIRT_E_TIMEOUT) g->broken = true;
            return r;
        }
    }
    {
        std::lock_guard<std::mutex> gl(c->groups_mu);
        c->groups.push_back(g.get());
    }
    *out = g.release();
    return MIRT_OK;
}

int mirt_group_emulate(mirt_group* g, uint32_t world) {
    if (!g) return fail(MIRT_E_INVALID, "NULL group");
    if (g->k != 0) return fail(MIRT_E_INVALID, "emulate before the first frame");
    if (g->world != 1 || !g->tiled || g->rehearse)
        return fail(MIRT_E_INVALID, "emulation needs a tiled world == 1 group (not a rehearsal)");
    if (world < 1 || world > 64) return fail(MIRT_E_INVALID, "emulated world must be 1..64");
    HIP_TRY(hipSetDevice(g->c->device));
    g->emulate = world;
    g->members.clear();
    for (uint32_t q = 0; q < world; ++q) g->members.push_back(q);
    g->my_index = 0;
    return group_plan(g);
}

int mirt_group_emulate_drop(mirt_group* g, uint64_t ranks) {
    if (!g) return fail(MIRT_E_INVALID, "NULL group");
    if (g->emulate < 2) return fail(MIRT_E_INVALID, "fault injection needs an emulated world");
    if (ranks & 1u) return fail(MIRT_E_INVALID, "the root (rank 0) cannot be dropped");
    uint64_t deal = 0;  // ranks -> deal indices
    for (size_t i = 0; i < g->members.size() && i < 64; ++i)
        if ((ranks >> (g->members[i] & 63u)) & 1u) deal |= 1ull << i;
    g->emu_drop = deal;
    return MIRT_OK;
}

int mirt_group_set_timeout(mirt_group* g, uint32_t ms) {
    if (!g) return fail(MIRT_E_INVALID, "NULL group");
    g->timeout_ms = ms;
    return MIRT_OK;
}

int mirt_group_failed_ranks(const mirt_group* g, uint64_t* mask) {
    if (!g || !mask) return fail(MIRT_E_INVALID, "NULL argument");
    *mask = g->failed_mask;
    return __builtin_popcountll(g->failed_mask);
}

static int group_flush(mirt_group* g);

// The host copies still waiting for their stream's next launch (fused copies): as their own
// kernels now, each followed by its batch's ev_done.
static int flush_pending_copies(mirt_group* g) {
    if (!g->fused_copy) return MIRT_OK;
    for (uint32_t b = 0; b < g->pend.size(); ++b) {
        mirt_group::PendingCopy& p = g->pend[b];
        if (!p.on) continue;
        p.on = false;
        HIP_TRY(launch_copy_rect_host(p.fc.jobs, p.fc.n, g->H, p.cols, g->streams[b]));
        HIP_TRY(hipEventRecord(g->ev_done[p.hs], g->streams[b]));
    }
    return MIRT_OK;
}
// Whether this group runs FB / 2 streams and fuses its host copies into its launches (see
// mirt_group::fused_copy).  A change of the stream mapping drains the group first.
static int update_fused_copy(mirt_group* g) {
    const char* e = getenv("MIRT_FUSED_COPY");
    const bool force_off = e && e[0] == '0', force_on = e && e[0] == '1';
    const bool half = !g->tiled && g->world <= 1 && g->FB >= 2 && g->FB % 2 == 0 && !force_off &&
                      (force_on || g->FB >= 8);
    const bool fused = half && g->host_out && !g->copy_stream && !g->d2h_sdma;
    int r;
    if (g->fused_copy && (!fused || half != g->half_streams) && (r = flush_pending_copies(g)) != MIRT_OK) return r;
    if (half != g->half_streams && g->nb)
        for (hipStream_t s : g->streams)
            if (s) HIP_TRY(hipStreamSynchronize(s));
    g->half_streams = half;
    g->fused_copy = fused;
    if (g->pend.size() < g->FB) g->pend.assign(g->FB, mirt_group::PendingCopy());
    return MIRT_OK;
}

int mirt_group_set_host_output(mirt_group* g, int enable) {
    if (!g) return fail(MIRT_E_INVALID, "NULL group");
    if (g->rank != 0) return fail(MIRT_E_INVALID, "only the root holds framebuffers");
    HIP_TRY(hipSetDevice(g->c->device));
    int r = group_flush(g);  // the open batch keeps the setting it was staged with
    if (r != MIRT_OK) return r;
    // frames traced while the output was off never reached the host planes: the next copy
    // into each slot covers the whole screen
    if (enable && !g->host_out && !g->hfb.empty()) {
        for (HostFrame& hf : g->hfb) {
            hf.rect[0] = hf.rect[1] = 0;
            hf.rect[2] = g->W;
            hf.rect[3] = g->H;
        }
        for (uint32_t b = 0; b < g->HB; ++b)  // every column's span: the whole column
            HIP_TRY(hipStreamWaitEvent(g->streams[0], g->ev_done[b], 0));
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)g->d_spans, (int)(g->H << 16), (size_t)g->F * g->W, g->streams[0]));
        for (uint32_t b = 1; b < g->F; ++b) {
            HIP_TRY(hipEventRecord(g->ev_traced[0], g->streams[0]));
            HIP_TRY(hipStreamWaitEvent(g->streams[b], g->ev_traced[0], 0));
        }
        if (g->copy_stream) {
            HIP_TRY(hipEventRecord(g->ev_traced[0], g->streams[0]));
            HIP_TRY(hipStreamWaitEvent(g->copy_stream, g->ev_traced[0], 0));
        }
    }
    if (!enable && (r = flush_pending_copies(g)) != MIRT_OK) return r;
    g->host_out = enable != 0;
    if (g->host_out && g->hfb.empty()) {
        if (!g->fb[0].rgb8 || !g->fb[0].valid)
            return fail(MIRT_E_INVALID, "host output needs the rgb8 and valid framebuffer planes");
        g->hfb.assign(g->F, HostFrame());
        HIP_TRY(hipMalloc((void**)&g->d_spans, sizeof(uint32_t) * g->F * g->W));
        HIP_TRY(hipMemset(g->d_spans, 0, sizeof(uint32_t) * g->F * g->W));
        const size_t n = (size_t)g->W * g->H;
        for (HostFrame& hf : g->hfb) {
            HIP_TRY(hipHostMalloc((void**)&hf.rgb8, 3 * n));
            HIP_TRY(hipHostMalloc((void**)&hf.valid, n));
            memset(hf.rgb8, 0, 3 * n);
            memset(hf.valid, 0, n);
        }
    }
    return update_fused_copy(g);
}

int mirt_group_exclude(mirt_group* g, uint64_t alive, const uint8_t* new_unique_id) {
    if (!g) return fail(MIRT_E_INVALID, "NULL group");
    if (!(alive & 1u)) return fail(MIRT_E_INVALID, "the root (rank 0) must stay in the group");
    const uint32_t world = g->emulate > 1 ? g->emulate : (uint32_t)g->world;
    if (world < 64 && (alive >> world)) return fail(MIRT_E_INVALID, "alive names ranks outside the group");
    if (g->emulate <= 1 && !((alive >> g->rank) & 1u))
        return fail(MIRT_E_INVALID, "this rank is excluded: destroy its group instead");
    HIP_TRY(hipSetDevice(g->c->device));
    std::vector<uint32_t> keep;
    for (uint32_t q = 0; q < g->members.size(); ++q)
        if ((alive >> (g->members[q] & 63u)) & 1u) keep.push_back(q);  // deal indices that stay
    if (g->world > 1) {
        const Rccl& R = rccl();
        std::vector<int> excl;
        for (uint32_t q = 0; q < g->members.size(); ++q)
            if (!((alive >> (g->members[q] & 63u)) & 1u)) excl.push_back((int)q);
        ncclComm_t nc = nullptr;
        if (new_unique_id) {
            if (R.comm_abort) (void)R.comm_abort(g->comm);
            else (void)R.comm_destroy(g->comm);
            g->comm = nullptr;
            ncclUniqueId u;
            memcpy(u.internal, new_unique_id, NCCL_UNIQUE_ID_BYTES);
            int me = 0;
            for (uint32_t i = 0; i < keep.size(); ++i)
                if (keep[i] == (uint32_t)g->my_index) me = (int)i;
            RCCL_TRY(R.comm_init_rank(&nc, (int)keep.size(), u, me));
        } else {
            if (!R.comm_shrink) return fail(MIRT_E_DEVICE, "librccl has no ncclCommShrink: pass a new unique id");
            RCCL_TRY(R.comm_shrink(g->comm, excl.data(), (int)excl.size(), &nc, nullptr, NCCL_SHRINK_ABORT));
            if (R.comm_abort) (void)R.comm_abort(g->comm);
        }
        g->comm = nc;
    }
    // drain what the group still runs (the aborted communicator's kernels have ended)
    const uint32_t saved = g->timeout_ms;
    if (!g->timeout_ms) g->timeout_ms = 10000;
    for (uint32_t b = 0; b < g->F; ++b) {
        HIP_TRY(hipEventRecord(g->ev_done[b], g->streams[b]));
        int r = group_wait_event(g, g->ev_done[b], "draining the group");
        if (r != MIRT_OK) {
            g->timeout_ms = saved;
            return r;
        }
    }
    if (g->copy_stream) {
        HIP_TRY(hipEventRecord(g->ev_comm, g->copy_stream));
        int r = group_wait_event(g, g->ev_comm, "draining the host copies");
        if (r != MIRT_OK) {
            g->timeout_ms = saved;
            return r;
        }
    }
    g->timeout_ms = saved;
    std::vector<uint32_t> members;
    for (uint32_t q : keep) members.push_back(g->members[q]);
    for (uint32_t i = 0; i < keep.size(); ++i)
        if (keep[i] == (uint32_t)g->my_index) g->my_index = (int)i;
    g->members = members;
    g->emu_drop = 0;
    for (uint32_t i = 0; i < g->bn; ++i) lt_unpin(g->c, g->stage[i].fa.ltab);  // the open batch is dropped
    g->bn = 0;
    g->held = g->lone_next = false;
    g->nb = 0;
    for (BatchRec& br : g->binfo) br = BatchRec();
    for (uint64_t& f : g->slot_frame) f = ~0ull;
    for (uint64_t& b : g->slot_bad) b = 0;
    g->pending_bad = 0;
    g->pending_bad_frame = ~0ull;
    g->failed_mask = 0;
    g->broken = false;
    return group_plan(g);
}

// The staged records (an open batch, or a batch the lone-frame hold keeps) launched now: a held
// batch runs alone with the whole chip, as mirt_group_wait would run it.
static int group_launch_staged(mirt_group* g) {
    if (g->bn == 0) return MIRT_OK;
    HIP_TRY(hipSetDevice(g->c->device));
    g->lone_next = g->held;
    return group_flush(g);
}

// Launch the open batch on its slot's stream: every share's trace, then (tiled) the pack
// into the transfer form, the gather of the batch as ONE RCCL group (emulated: the same
// bytes copied on the device), and on the root the trailer check and one unpack launch.
static int group_flush(mirt_group* g) {
    if (g->bn == 0) return MIRT_OK;
    const bool lone = g->lone_next;
    g->held = g->lone_next = false;
    mirt_ctx* c = g->c;
    const uint32_t bs = (uint32_t)(g->nb % (g->half_streams ? g->FB / 2 : g->FB));  // the stream and its device slot
    const uint32_t hs = (uint32_t)(g->nb % g->HB);  // the host ring slot: records and events
    hipStream_t s = g->streams[bs];
    const bool is_root = g->rank == 0;
    const uint32_t n = g->bn;
    g->bn = 0;
    LtPins pins(c);  // the staged records' light tables, held until every share has launched
    for (uint32_t i = 0; i < n; ++i) pins.add(g->stage[i].fa.ltab);
    BatchRec& br = g->binfo[hs];
    br.n = n;
    br.first = g->k - n;
    br.checked = false;
    RectJobs jobs{};
    for (uint32_t i = 0; i < n; ++i) {
        br.j[i] = g->bj[i];
        hit_rect(g->stage[i], g->W, g->H, br.rect[i]);
        memcpy(jobs.rect[i], br.rect[i], sizeof(jobs.rect[i]));
        jobs.tag[i] = transfer_tag(br.first + i);
    }
    HT(7);
    // a sender reuses its packed planes only after their previous batch's sends are done (the
    // root's stream already waited for that gather before its unpacks)
    if (g->tiled && g->world > 1 && !is_root && g->nb >= g->FB)
        HIP_TRY(hipStreamWaitEvent(s, g->ev_gathered[(g->nb - g->FB) % g->HB], 0));
    // host copies on copy_stream: batch nb - FB last used this batch's framebuffers; its copy
    // must have read them before this batch's fill and trace rewrite them
    if (g->copy_stream && g->nb >= g->FB) HIP_TRY(hipStreamWaitEvent(s, g->ev_done[(g->nb - g->FB) % g->HB], 0));
    // adaptive grid (MIRT_ADAPTIVE_GRID, see mirt_group): mode 1, the launches still running
    // share the chip with this one; mode 2, a launch issued while none runs gets the chip
    // (kWgPerCu per CU), any other the fixed grid
    uint32_t max_wg_now = 0;
    if (g->adaptive_grid) {
        uint32_t running = 0;
        for (uint64_t b = g->nb > g->HB ? g->nb - g->HB : 0; b < g->nb; ++b)
            if (hipEventQuery(g->ev_done[b % g->HB]) == hipErrorNotReady) ++running;
        if (g->adaptive_grid == 1)
            max_wg_now = std::max<uint32_t>(1, (uint32_t)(2 * kWgPerCu * (uint64_t)c->cus / (running + 1)));
        else if (running == 0)
            max_wg_now = (uint32_t)(kWgPerCu * (uint64_t)c->cus);
    }
    if (lone) max_wg_now = (uint32_t)(kWgPerCu * (uint64_t)c->cus);
    // Blocks outside a frame's hit rectangle (every ray misses) are not traced: a share's
    // packed plane is only read inside the rectangle (k_pack_rect), and the whole-screen
    // planes get their miss values first, one fill per batch (FrameRec::live).
    bool narrow[kMaxFrames];
    {
        FillJobs fj{};
        uint64_t fill_max = 0;
        const uint64_t npx = (uint64_t)g->W * g->H;
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t* R = br.rect[i];
            narrow[i] = !(R[0] == 0 && R[1] == 0 && R[2] == g->W && R[3] == g->H);
            const uint32_t j = g->bj[i];
            if (g->tiled) continue;
            if (!narrow[i]) {  // traced whole: every pixel is written
                g->dirty0[j] = 0;
                g->dirty1[j] = g->W;
                g->dirty_y0[j] = 0;
                g->dirty_y1[j] = g->H;
                continue;
            }
            // Only columns an earlier frame of this slot may have hit can hold anything but miss
            // values (the trace writes every pixel of the blocks meeting this frame's rectangle,
            // and hit pixels lie inside it): refill those columns, whole 16-byte words (extra
            // bytes of neighbouring columns get the miss value they already hold).
            const uint32_t d0 = g->dirty0[j], d1 = g->dirty1[j], e0 = g->dirty_y0[j], e1 = g->dirty_y1[j];
            g->dirty0[j] = R[0];
            g->dirty1[j] = R[2];
            g->dirty_y0[j] = R[1];
            g->dirty_y1[j] = R[3];
            if (d1 <= d0 || e1 <= e0) continue;
            if (R[0] <= d0 && d1 <= R[2] && R[1] <= e0 && e1 <= R[3]) continue;  // rewritten by this trace
            const OutPlanes& o = g->fb[j];
            const struct { void* p; uint64_t e; uint8_t v; } planes[kFillPlanes] = {
                {o.rgb, 24, 0}, {o.rgb8, 3, 0}, {o.valid, 1, 0}, {o.face, 4, 0xff}, {o.object, 4, 0xff}, {o.rgbv, 4, 0}};
            for (int k = 0; k < kFillPlanes; ++k) {
                fj.ptr[i][k] = nullptr;
                fj.bytes[i][k] = 0;
                fj.value[i][k] = planes[k].v;
                if (!planes[k].p) continue;
                const uint64_t b0 = (uint64_t)d0 * g->H * planes[k].e & ~15ull;
                const uint64_t b1 = std::min<uint64_t>(npx * planes[k].e, ((uint64_t)d1 * g->H * planes[k].e + 15) & ~15ull);
                fj.ptr[i][k] = (uint8_t*)planes[k].p + b0;
                fj.bytes[i][k] = b1 - b0;
                fill_max = std::max(fill_max, b1 - b0);
            }
        }
        if (fill_max) HIP_TRY(launch_fill_planes(fj, n, fill_max, s));
    }
    HT(8);
    // full-height strips traced by k_trace write each share straight into its transfer form
    // (FrameRec::xf: no k_pack_rect launch, no packed plane read back)
    const bool fuse = g->tiled && (g->tile_h == 0 || g->tile_h >= g->H) && !g->bbounces &&
                      !(c->flags & MIRT_OPT_SPLIT_KERNELS) && !g->no_fused_pack;
    for (Share& sh : g->shares) {
        Slot* sl = sh.slots[bs].get();
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t j = g->bj[i];
            sl->h_frames[i] = g->stage[i];
            uint32_t* xfer = (is_root && sh.q == 0) ? g->gathered[j] : sh.sendbuf[j];
            sl->h_frames[i].out = g->tiled ? OutPlanes{nullptr, nullptr, nullptr, nullptr, nullptr,
                                                       fuse ? xfer : sh.packed[j]}
                                           : g->fb[j];
            if (fuse) share_xfer(sh.tiles, br.rect[i], jobs.tag[i], sl->h_frames[i].xf);
            if (narrow[i]) memcpy(sl->h_frames[i].live, br.rect[i], sizeof(br.rect[i]));
        }
        // fused host copies: this launch's first waves copy the stream's previous batch to the host
        // (k_trace launches only: before a reflection or split-kernel launch it runs on its own)
        const bool one_launch = !g->bbounces && !(c->flags & MIRT_OPT_SPLIT_KERNELS);
        if (g->fused_copy && g->pend[bs].on && !one_launch) {
            mirt_group::PendingCopy& p = g->pend[bs];
            p.on = false;
            HIP_TRY(launch_copy_rect_host(p.fc.jobs, p.fc.n, g->H, p.cols, s));
            HIP_TRY(hipEventRecord(g->ev_done[p.hs], s));
        }
        const FusedCopy* fcp = (g->fused_copy && g->pend[bs].on) ? &g->pend[bs].fc : nullptr;
        int r = launch_frames(c, sl, n, g->W, g->H, sh.tiles.data(), (uint32_t)sh.tiles.size(), g->bbounces, s, nullptr,
                              max_wg_now, fcp);
        if (fcp && r == MIRT_OK) {  // that batch is in host memory once this launch has ended
            g->pend[bs].on = false;
            HIP_TRY(hipEventRecord(g->ev_done[g->pend[bs].hs], s));
        }
        if (r != MIRT_OK) {
            (void)hipStreamSynchronize(s);
            return r;
        }
        if (!g->tiled) continue;
        // the share's tiles inside each frame's hit rectangle -> its transfer form (the root's
        // share straight into region 0 of the gathered plane)
        if (!fuse) {
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t j = g->bj[i];
                jobs.src[i] = sh.packed[j];
                jobs.dst[i] = (is_root && sh.q == 0) ? g->gathered[j] : sh.sendbuf[j];
            }
            HIP_TRY(launch_pack_rect(sh.d_tiles, (uint32_t)sh.tiles.size(), jobs, n, s));
        }
        if (g->emulate > 1 && sh.q != 0 && !((g->emu_drop >> sh.q) & 1u))
            for (uint32_t i = 0; i < n; ++i) {  // exactly the bytes an RCCL send would carry
                const uint32_t j = g->bj[i];
                HIP_TRY(hipMemcpyAsync(g->gathered[j] + (uint64_t)sh.q * g->stride, sh.sendbuf[j],
                                       transfer_words(g, sh.q, br.rect[i]) * 4, hipMemcpyDeviceToDevice, s));
            }
    }
    if (g->tiled && g->world > 1) {
        const Rccl& R = rccl();
        const uint32_t P = (uint32_t)g->members.size();
        HIP_TRY(hipEventRecord(g->ev_traced[hs], s));
        HIP_TRY(hipStreamWaitEvent(g->comm_stream, g->ev_traced[hs], 0));
        RCCL_TRY(R.group_start());
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t j = g->bj[i];
            if (is_root) {
                for (uint32_t q = 1; q < P; ++q)
                    RCCL_TRY(R.recv(g->gathered[j] + (uint64_t)q * g->stride, transfer_words(g, q, br.rect[i]) * 4,
                                    ncclUint8, (int)q, g->comm, g->comm_stream));
            } else {
                RCCL_TRY(R.send(g->shares[0].sendbuf[j], transfer_words(g, (uint32_t)g->my_index, br.rect[i]) * 4,
                                ncclUint8, 0, g->comm, g->comm_stream));
            }
        }
        RCCL_TRY(R.group_end());
        HIP_TRY(hipEventRecord(g->ev_gathered[hs], g->comm_stream));
        if (is_root) HIP_TRY(hipStreamWaitEvent(s, g->ev_gathered[hs], 0));
    }
    HT(4);
    if (g->tiled && is_root && !g->skip_unpack) {
        const uint32_t P = (uint32_t)g->members.size();
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t j = g->bj[i];
            jobs.src[i] = g->gathered[j];
            jobs.out[i] = g->fb[j];
            jobs.bad[i] = g->h_bad + (size_t)j * P;
            // the columns the unpack rewrites: this frame's hit rectangle and the one the slot's
            // framebuffer held (every other column holds misses already)
            const uint32_t* R = br.rect[i];
            uint32_t u0 = R[0], u1 = R[2];
            if (g->dirty1[j] > g->dirty0[j]) {
                u0 = R[2] > R[0] ? std::min(u0, g->dirty0[j]) : g->dirty0[j];
                u1 = R[2] > R[0] ? std::max(u1, g->dirty1[j]) : g->dirty1[j];
            }
            jobs.ucol[i][0] = u0;
            jobs.ucol[i][1] = u1;
            g->dirty0[j] = R[2] > R[0] ? R[0] : 0;
            g->dirty1[j] = R[2] > R[0] ? R[2] : 0;
        }
        // the regions' trailers are checked by the same launch (not in a rehearsal, whose
        // peer regions were never sent)
        HIP_TRY(launch_unpack_rect(g->d_unpack, g->n_unpack, g->max_tile_px, g->H, g->stride,
                                   g->rehearse ? nullptr : g->d_regions, P, jobs, n, s));
    }
    if (g->host_out && is_root) {
        HostCopyJobs hj{};
        uint32_t cols = 0;
        for (uint32_t i = 0; i < n; ++i) host_copy_job(g, g->bj[i], br.rect[i], hj, i, cols);
        if (cols && g->d2h_sdma) {
            // the copy engine: the whole columns of each rectangle, one contiguous range per plane
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t* u = hj.rect[i];
                if (u[0] >= u[2]) continue;
                const size_t p0 = (size_t)u[0] * g->H, np = (size_t)(u[2] - u[0]) * g->H;
                if (hj.rgb8[i])
                    HIP_TRY(hipMemcpyAsync(hj.hrgb8[i] + 3 * p0, hj.rgb8[i] + 3 * p0, 3 * np, hipMemcpyDeviceToHost, s));
                if (hj.valid[i])
                    HIP_TRY(hipMemcpyAsync(hj.hvalid[i] + p0, hj.valid[i] + p0, np, hipMemcpyDeviceToHost, s));
            }
        } else if (cols && g->copy_stream) {
            // the batch's frames are final on stream s: copy them on the reserved CUs, and let
            // the batch complete (ev_done) only once they are in host memory
            HIP_TRY(hipEventRecord(g->ev_traced[hs], s));
            HIP_TRY(hipStreamWaitEvent(g->copy_stream, g->ev_traced[hs], 0));
            HIP_TRY(launch_copy_rect_host(hj, n, g->H, cols, g->copy_stream));
            HIP_TRY(hipEventRecord(g->ev_done[hs], g->copy_stream));
            ++g->nb;
            return MIRT_OK;
        } else if (cols && g->fused_copy) {
            // copied by the stream's next launch (or flush_pending_copies), which records ev_done
            mirt_group::PendingCopy& p = g->pend[bs];
            p.on = true;
            p.hs = hs;
            p.cols = cols;
            p.fc.jobs = hj;
            p.fc.n = n;
            p.fc.H = g->H;
            HT(5);
            ++g->nb;
            return MIRT_OK;
        } else if (cols) {
            HIP_TRY(launch_copy_rect_host(hj, n, g->H, cols, s));
        }
    }
    HT(5);
    HIP_TRY(hipEventRecord(g->ev_done[hs], s));
    HT(6);
    ++g->nb;
    return MIRT_OK;
}

int mirt_group_set_batch(mirt_group* g, uint32_t frames_per_launch) {
    if (!g) return fail(MIRT_E_INVALID, "NULL group");
    if (g->k != 0) return fail(MIRT_E_INVALID, "set the batch before the first frame");
    if (frames_per_launch < 1 || frames_per_launch > kMaxFrames || frames_per_launch > g->F)
        return fail(MIRT_E_INVALID, "frames per launch must be 1..min(8, inflight)");
    if (frames_per_launch > 1 && (g->c->flags & MIRT_OPT_SPLIT_KERNELS))
        return fail(MIRT_E_INVALID, "several frames per launch need the single-kernel path (not MIRT_OPT_SPLIT_KERNELS)");
    g->B = frames_per_launch;
    g->FB = g->F / g->B;
    group_ring(g);
    return update_fused_copy(g);
}

// Nothing of the group runs: no batch launched yet, or the last one complete (its ev_done
// recorded, no host copy of it pending: a pending copy means a burst is going on).
static bool group_idle(const mirt_group* g) {
    if (g->nb == 0) return true;
    for (const mirt_group::PendingCopy& p : g->pend)
        if (p.on) return false;
    return hipEventQuery(g->ev_done[(g->nb - 1) % g->HB]) == hipSuccess;
}

int mirt_trace_frame(mirt_group* g, const mirt_frame* f, uint64_t* index) {
    if (!g || !f) return fail(MIRT_E_INVALID, "NULL group or frame");
    if (g->broken) {  // the caller must exclude the failed ranks first
        return fail(MIRT_E_PEER, "the group lost rank(s) " + ranks_text(g->failed_mask) +
                                     ": call mirt_group_exclude before tracing more frames");
    }
    mirt_ctx* c = g->c;
    HT_START();
    HIP_TRY(hipSetDevice(c->device));
    int r = check_frame(c, f);
    if (r != MIRT_OK) return r;
    const uint32_t j = (uint32_t)(g->k % g->F);
    FrameRec rec{};
    uint64_t tris = 0;
    frame_record(c, f, g->W, g->H, OutPlanes{}, rec, tris);
    HT(1);
    if (g->held && (r = group_flush(g)) != MIRT_OK) {  // a held batch: a burst has begun
        lt_unpin(c, rec.fa.ltab);
        return r;
    }
    // split kernels and reflection frames run one frame per launch
    if (g->bn > 0 && (g->bbounces || f->max_bounces || (c->flags & MIRT_OPT_SPLIT_KERNELS) ||
                      !frames_batchable(g->stage[0], rec)))
        if ((r = group_flush(g)) != MIRT_OK) {
            lt_unpin(c, rec.fa.ltab);
            return r;
        }
    const uint32_t hs = (uint32_t)(g->nb % g->HB);
    // back-pressure when a batch opens: batch nb - HB (the last user of this host ring slot)
    // must have finished; batch nb - FB, the last user of this batch's stream, device slot and
    // framebuffers, is ordered before it by the stream itself
    if (g->bn == 0 && g->nb >= g->HB) {
        if ((r = group_wait_event(g, g->ev_done[hs], "mirt_trace_frame back-pressure")) != MIRT_OK) {
            lt_unpin(c, rec.fa.ltab);
            return group_timed_out(g, hs, r);
        }
        batch_fold(g, hs);
    }
    HT(0);
    g->stage[g->bn] = rec;
    g->bj[g->bn++] = j;
    g->slot_frame[j] = g->k;
    g->slot_bad[j] = 0;
    g->bbounces = f->max_bounces;
    if (index) *index = g->k;
    ++g->k;
    if (g->bn == g->B || g->bbounces || (c->flags & MIRT_OPT_SPLIT_KERNELS)) {
        // the group has nothing running: hold the batch until the caller waits (a lone frame,
        // launched with the whole chip) or submits again (launched then, with the fixed grid)
        if (g->lone_hold && group_idle(g)) {
            g->held = true;
            return MIRT_OK;
        }
        return group_flush(g);
    }
    return MIRT_OK;
}

int mirt_group_wait(mirt_group* g, void* stream) {
    if (!g) return fail(MIRT_E_INVALID, "NULL group");
    if (g->broken) return fail(MIRT_E_PEER, "the group lost rank(s) " + ranks_text(g->failed_mask));
    HIP_TRY(hipSetDevice(g->c->device));
    g->lone_next = g->held;  // a held batch runs alone: the whole chip
    int r = group_flush(g);
    if (r == MIRT_OK) r = flush_pending_copies(g);
    if (r != MIRT_OK) return r;
    const uint64_t used = std::min<uint64_t>(g->nb, g->HB);
    for (uint64_t b = 0; b < used; ++b) {
        if (stream) {
            // a batch already complete needs no wait on the caller's stream (each wait is a
            // barrier packet on the stream's queue; after a host wait on every batch, as the
            // bench's finish does, all 16 were redundant)
            const hipError_t q = hipEventQuery(g->ev_done[b]);
            if (q != hipSuccess) {
                (void)hipGetLastError();  // (hipErrorNotReady is not an error here)
                HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, g->ev_done[b], 0));
            }
        } else {
            if ((r = group_wait_event(g, g->ev_done[b], "mirt_group_wait")) != MIRT_OK)
                return group_timed_out(g, (uint32_t)b, r);
            batch_fold(g, (uint32_t)b);
        }
    }
    if (!stream && g->comm_stream) {
        HIP_TRY(hipEventRecord(g->ev_comm, g->comm_stream));
        if ((r = group_wait_event(g, g->ev_comm, "mirt_group_wait (gathers)")) != MIRT_OK) {
            g->broken = true;
            g->failed_mask = g->rank == 0 ? 0 : 1;
            return r;
        }
    }
    if (!stream && g->pending_bad) {
        g->failed_mask = mask_of_ranks(g, g->pending_bad);
        const uint64_t fr = g->pending_bad_frame;
        g->pending_bad = 0;
        g->pending_bad_frame = ~0ull;
        return fail(MIRT_E_PEER, "frame " + std::to_string(fr) + ": the transfer of rank(s) " +
                                     ranks_text(g->failed_mask) + " is missing or inconsistent (frame skipped)");
    }
    return MIRT_OK;
}

int mirt_group_frame_host(mirt_group* g, uint64_t index, mirt_outputs* out) {
    if (!g || !out) return fail(MIRT_E_INVALID, "NULL argument");
    if (!g->host_out) return fail(MIRT_E_INVALID, "host output is off (mirt_group_set_host_output)");
    HIP_TRY(hipSetDevice(g->c->device));
    const uint32_t j = (uint32_t)(index % g->F);
    if (index >= g->k || g->slot_frame[j] != index)
        return fail(MIRT_E_INVALID, "frame " + std::to_string(index) + " is not held (enqueued frames keep their " +
                                        "slot until frame index + inflight)");
    int r;
    // the frame's own open batch, or a held batch whatever frame is asked for (a pipelined
    // caller reading frame k - 1 must not leave frame k held while it works on the host)
    if (g->held || (g->bn && index >= g->k - g->bn)) {
        if ((r = group_launch_staged(g)) != MIRT_OK) return r;
    }
    if ((r = flush_pending_copies(g)) != MIRT_OK) return r;
    // the batch holding the frame: the latest launched batch whose slot lists j
    for (uint32_t b = 0; b < g->HB; ++b) {
        const BatchRec& br = g->binfo[b];
        if (br.n && index >= br.first && index < br.first + br.n) {
            if ((r = group_wait_event(g, g->ev_done[b], "mirt_group_frame_host")) != MIRT_OK)
                return group_timed_out(g, b, r);
            batch_fold(g, b);
            break;
        }
    }
    if (g->slot_bad[j]) {
        g->failed_mask = mask_of_ranks(g, g->slot_bad[j]);
        return fail(MIRT_E_PEER, "frame " + std::to_string(index) + ": the transfer of rank(s) " +
                                     ranks_text(g->failed_mask) + " is missing or inconsistent (frame skipped)");
    }
    memset(out, 0, sizeof(*out));
    out->rgb8 = g->hfb[j].rgb8;
    out->valid = g->hfb[j].valid;
    return MIRT_OK;
}

}  // extern "C"

namespace mirt {

// The frame's hit rectangle on a W x H screen (hit_rect: conservative, every pixel outside it
// misses), for callers outside the frame group (box.cpp: an order traces and copies only its
// part inside the rectangle).  Frames without the block pre-test give the whole screen.
int frame_hit_rect(mirt_ctx* c, const mirt_frame* f, uint32_t W, uint32_t H, uint32_t out[4]) {
    int r = check_frame(c, f);
    if (r != MIRT_OK) return r;
    std::unique_ptr<FrameRec> rec(new FrameRec());
    uint64_t tris = 0;
    {
        std::lock_guard<std::mutex> g(c->mu);  // the mesh table
        fill_args(c, f, W, H, rec->fa, tris);
        frustum_args(c, f, rec->fa, rec->fr, rec->ocert);
    }
    hit_rect(*rec, W, H, out);
    return MIRT_OK;
}

}  // namespace mirt
