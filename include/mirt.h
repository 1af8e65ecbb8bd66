/*
 * mirt.h — C ABI of libmirt.so, the MI355X-native trace worker.
 *
 * Plain C, cgo-safe: no C++ types, no torch types, plain pointers and sizes.  Every
 * buffer is owned by the caller; the library copies what it needs during the call and
 * keeps no caller pointer after return (cgo pointer rules).  Every entry returns 0
 * (MIRT_OK) or a negative MIRT_E_* code, with detail in the thread-local
 * mirt_last_error().  No exception crosses the ABI.  All entries are re-entrant:
 * frame state is an argument, never global (gRPC serves each BulkTrace in its own
 * goroutine, and the master pipelines frames with different cameras).
 *
 * What each entry replaces in the reference (paths relative to its root):
 *   mirt_trace_tile      — the BulkTrace tile loop worker/distributed/main.go:67-89
 *                          calling tracer.Trace (worker/shared/tracer/tracer.go:81-91)
 *                          per pixel; also the sequential draw loop
 *                          worker/sequential/main.go:21-28 (tile = whole screen).
 *   mirt_trace_rays      — tracer.trace (tracer.go:27-50) on arbitrary rays.
 *   mirt_mesh_upload     — the immutable mesh a worker receives at Register
 *                          (shared/state/environment.go:25-62, mesh.go:100-106).
 *   mirt_frame / mirt_camera — the per-frame EnvMutables carried by WorkOrder.diff
 *                          (environment.go:65-69, camera.go:20-24, light.go:10-13).
 *   mirt_camera_init     — state.NewCamera (camera.go:35-44) + the math.Tan of
 *                          tracer.go:17.
 */
#ifndef MIRT_H
#define MIRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIRT_ABI_VERSION 7

/* error codes */
#define MIRT_OK 0
#define MIRT_E_INVALID (-1)   /* bad argument (null pointer, zero size, bad id) */
#define MIRT_E_DEVICE (-2)    /* HIP runtime / kernel launch error */
#define MIRT_E_LIMIT (-3)     /* more objects/lights than the kernel-argument block holds, or an
                                 object whose bounding box (object.go:31-59) overflows fp64: the
                                 reference still traces such a frame (its Box.Intersect evaluates
                                 inf/NaN planes, box.go:29-68); this library rejects it */
#define MIRT_E_NOMEM (-4)     /* device or host allocation failed */
#define MIRT_E_CAMERA (-5)    /* camera dir parallel to the global up vector (camera.go:37) */
#define MIRT_E_CANCELLED (-6) /* *cancel became non-zero (worker/distributed/main.go:73) */
#define MIRT_E_IO (-7)        /* scene / OBJ / MTL file could not be read or parsed */
#define MIRT_E_TIMEOUT (-8)   /* a frame group wait passed its deadline (mirt_group_set_timeout) */
#define MIRT_E_PEER (-9)      /* a rank's transfer is missing or inconsistent (mirt_group_failed_ranks) */

#define MIRT_MAX_OBJECTS 16
#define MIRT_MAX_LIGHTS 16
#define MIRT_MAX_BOUNCES 8

typedef struct mirt_ctx mirt_ctx;

/* shared/state/mesh.go:94-97 Material (colour.RGB channels as fp64 in [0,1]) */
typedef struct {
    double ka[3], kd[3], ks[3];
    double ns;
} mirt_material;

/* shared/state/object.go:17-22 Object (Pos + the mesh its id links to) */
typedef struct {
    uint32_t mesh_id;
    uint32_t reserved;
    double pos[3];
} mirt_object;

/* shared/state/light.go:10-13 Light (Col = NewRGB(u8)/255) */
typedef struct {
    double pos[3];
    double col[3];
} mirt_light;

/*
 * shared/state/camera.go:20-24 Camera.  forward/left/up exactly as NewCamera made them.
 * proj_half_width = math.Tan(fov / 2.0) as the caller computed it (tracer.go:17); a
 * Go caller passes its own math.Tan so the value is bit-identical to the reference.
 * mirt_camera_init fills it with a restatement of Go's math.Tan.
 */
typedef struct {
    double pos[3];
    double forward[3];
    double left[3];
    double up[3];
    double fov;
    double proj_half_width;
} mirt_camera;

/* shared/state/environment.go:65-69 EnvMutables */
typedef struct {
    const mirt_object *objects;
    uint32_t n_objects;
    const mirt_light *lights;
    uint32_t n_lights;
    mirt_camera camera;
    /* configs[4] EXTENSION (not in the reference): reflection bounces per primary hit,
     * 0..MIRT_MAX_BOUNCES.  0 = the reference's Trace.  Semantics in DESIGN.md §4.6:
     * c = c_add(phong, c_mul(Ks, c_reflected)), R = D - 2(D.N)N, origin hit + R*1e-4. */
    uint32_t max_bounces;
    uint32_t reserved;
} mirt_frame;

/* shared/comms/comms.proto:25-31 WorkOrder geometry */
typedef struct {
    uint32_t x, y, w, h;
} mirt_tile;

/*
 * Output planes.  Any pointer may be NULL (not produced).  Pixel (x+i, y+j) of a tile
 * lands at index i*h + j (column-major, worker/distributed/main.go:82); for a tile list
 * the tiles are packed back to back in list order.
 *   rgb    3 fp64 per pixel, the colour.RGB returned by tracer.Trace (misses: 0)
 *   rgb8   3 u8 per pixel, uint8(255*c) truncating (colour.go:59-61; misses: 0)
 *   valid  1 u8 per pixel, Trace's bool
 *   face   winning face index inside its mesh (-1 on a miss)      [diagnostic]
 *   object winning object index inside mirt_frame.objects (-1)    [diagnostic]
 *   rgbv   rgb8 and valid in ONE 32-bit word per pixel, r | g << 8 | b << 16 | valid << 24
 *          (the packed form of a multi-GPU tile buffer: one store per pixel, one
 *          contiguous plane to gather; the unpack expands it into rgb8 + valid)
 */
typedef struct {
    double *rgb;
    uint8_t *rgb8;
    uint8_t *valid;
    int32_t *face;
    int32_t *object;
    uint32_t *rgbv; /* ABI 2 */
} mirt_outputs;

/* Counters of one call; timings are device time from HIP events (0 if not recorded). */
typedef struct {
    uint64_t primary_rays;
    uint64_t shadow_rays;
    uint64_t hits;
    uint64_t tri_tests;     /* ray-triangle tests performed (brute force: rays * tris) */
    double ms_primary;      /* the frame kernel k_trace (MIRT_OPT_SPLIT_KERNELS: the primary kernel) */
    double ms_shadow;       /* MIRT_OPT_SPLIT_KERNELS: the shadow + Phong kernel (default: 0) */
    double ms_shade;        /* reserved (0) */
    double ms_total;        /* first kernel start -> last kernel end */
    uint64_t reflection_rays; /* configs[4] extension (mirt_frame.max_bounces) */
} mirt_stats;

/* Accumulated per-kernel device times while profiling is enabled (HIP events). */
typedef struct {
    uint64_t launches;
    double primary_ms_sum, shadow_ms_sum, shade_ms_sum, frame_ms_sum;
    uint64_t primary_tri_tests, shadow_tri_tests;
    uint64_t primary_rays, shadow_rays, hits;
    /* wave-level BVH traversal work (diagnostic): node boxes tested, leaves entered */
    uint64_t primary_node_visits, primary_leaf_visits, shadow_node_visits, shadow_leaf_visits;
    /* traversal stack overflows (provably impossible; a non-zero value is a library bug) */
    uint64_t stack_overflows;
    /* configs[4] extension: reflection rays traced and the reflect kernel's device time */
    uint64_t reflection_rays;
    double reflect_ms_sum;
    /* frames traced (a frame group launches up to 8 frames at once: per-frame figures
       divide by frames, per-launch kernel times by launches) */
    uint64_t frames;
    /* ABI 6: medians over the read's launches of the first kernel's and the whole launch's
       HIP-event durations (robust to a launch that waited behind an overlapped one) */
    double primary_ms_median, frame_ms_median;
    /* ABI 7: deferred second passes run by k_trace launches' last workgroups: its
       redone 8x8 blocks (the split kernels' are not counted).  They run serially in one workgroup
       at the end of a launch, so a scene that needs many makes frames slow: this makes it visible. */
    uint64_t redo_items;
} mirt_profile;

int mirt_abi_version(void);
const char *mirt_last_error(void);
/* ABI 7: a hash of the kernels, the host code that launches them and the compile flags this
 * library was built from (16 hex digits).  Profiles record it; bench.py cites a profile only
 * for the build it was taken on. */
const char *mirt_build_id(void);

/* Context bound to one HIP device (one process per GPU). */
int mirt_create(int device, mirt_ctx **out);
void mirt_destroy(mirt_ctx *ctx);
int mirt_device(const mirt_ctx *ctx);

/* camera.go:35-44 NewCamera + tracer.go:17 math.Tan(fov/2).  MIRT_E_CAMERA if dir x up = 0. */
int mirt_camera_init(const double pos[3], const double dir[3], double fov, mirt_camera *out);
/* Restatement of Go's math.Tan (pure Go, Cephes). */
double mirt_go_tan(double x);
/* Restatement of Go's math.Pow (the specular term of tracer.go:72). */
double mirt_go_pow(double x, double y);
/* Test hook: op 0 Go math.Min(a, b), 1 math.Max(a, b), 2 Min(a, 1.0), 3 Max(a, 0.0) — the
 * last two as the colour code computes them (colour.go:38-50, tracer.go:69-72). */
double mirt_go_minmax(int op, double a, double b);

/*
 * Upload one immutable mesh (shared/state/mesh.go:100-106 after MeshFromFile):
 *   v    nv*3 vertex positions (float32-parsed, widened to fp64)
 *   vn   nn*3 vertex normals, already normalised; NULL/0 => flat Normal() shading
 *   fv   nf*3 vertex indices; fn nf*3 normal indices (ignored if vn is NULL); fmat nf
 *   mats nm materials
 * Indices are range-checked here.  The mesh id is returned in *mesh_id.
 */
int mirt_mesh_upload(mirt_ctx *ctx, const double *v, uint32_t nv, const double *vn, uint32_t nn,
                     const uint32_t *fv, const uint32_t *fn, const uint32_t *fmat, uint32_t nf,
                     const mirt_material *mats, uint32_t nm, uint32_t *mesh_id);
/* Waits for the device; frames a group on this context staged and has not launched yet (an open
 * batch, a held lone frame) are launched first, so they never read a freed mesh. */
int mirt_mesh_release(mirt_ctx *ctx, uint32_t mesh_id);

/*
 * BulkTrace: trace tile (x, y, w, h) of a W x H screen into HOST buffers.  Synchronous.
 * cancel (may be NULL) is polled between kernel launches.  stats may be NULL.
 */
int mirt_trace_tile(mirt_ctx *ctx, const mirt_frame *frame, uint32_t x, uint32_t y, uint32_t w, uint32_t h,
                    uint32_t W, uint32_t H, const mirt_outputs *host_out, const volatile int *cancel,
                    mirt_stats *stats);

/*
 * Trace a list of tiles into DEVICE buffers on `stream` (a hipStream_t; NULL = the HIP
 * null stream).  Asynchronous: returns after enqueueing.  If stats is non-NULL
 * the call synchronises the stream and fills it.  Device buffers must hold
 * sum(w*h) pixels of each requested plane.
 */
int mirt_trace_tiles_async(mirt_ctx *ctx, const mirt_frame *frame, uint32_t W, uint32_t H,
                           const mirt_tile *tiles, uint32_t n_tiles, const mirt_outputs *device_out,
                           void *stream, mirt_stats *stats);

/*
 * Framebuffer assembly after a gather: scatter packed tile planes (device) into a
 * W x H column-major framebuffer (pixel (x, y) at x*H + y, the worker/sequential
 * layout).  Planes that are NULL in either struct are skipped.  Asynchronous on stream.
 */
int mirt_unpack_tiles_async(mirt_ctx *ctx, uint32_t W, uint32_t H, const mirt_tile *tiles, uint32_t n_tiles,
                            const mirt_outputs *packed, const mirt_outputs *frame_out, void *stream);
/*
 * Same, with an explicit packed offset (in pixels, ascending) per tile, so the packed
 * buffers of several ranks (each padded to a common size for the gather) are scattered
 * in ONE launch.  The device copy of the tile list is reused while the list repeats.
 */
int mirt_unpack_tiles_at_async(mirt_ctx *ctx, uint32_t W, uint32_t H, const mirt_tile *tiles,
                               const uint64_t *offsets, uint32_t n_tiles, const mirt_outputs *packed,
                               const mirt_outputs *frame_out, void *stream);

/* tracer.go:27-50 trace() on n arbitrary rays (host buffers), brute force. */
int mirt_trace_rays(mirt_ctx *ctx, const mirt_frame *frame, uint32_t n, const double *origins,
                    const double *dirs, uint8_t *ok, double *hit, double *normal, int32_t *face,
                    int32_t *object);

/* HIP-event profiling of every subsequent trace call (per-kernel device time). */
int mirt_profile_enable(mirt_ctx *ctx, int enable);
/* Synchronises outstanding profiled work, returns the sums and resets them. */
int mirt_profile_read(mirt_ctx *ctx, mirt_profile *out);

/* Ask for kernel variants (benchmark ablations).  0 = defaults. */
#define MIRT_OPT_NO_PREFILTER 1u  /* always take the true fp64 divide for r2 */
#define MIRT_OPT_BRUTE_FORCE 2u   /* test every triangle (no BVH culling), mesh streamed via LDS */
#define MIRT_OPT_STATIC_SCHEDULE 4u /* round-robin work split in every kernel (no work queues) */
#define MIRT_OPT_TIMELINE 8u        /* record per-wave start/end stamps (mirt_debug_timeline) */
#define MIRT_OPT_NO_SEGMENT 16u     /* shadow rays as full nearest-hit queries (no segment / any-hit; mesh read from HBM) */
#define MIRT_OPT_SPLIT_KERNELS 32u  /* k_primary then k_shadow (default: one k_trace launch per frame) */
#define MIRT_OPT_NO_FRUSTUM 64u     /* no whole-block frustum pre-test of primary rays */
#define MIRT_OPT_NO_OCTANT 128u     /* generic child-box test (no sign-octant variants; same decisions) */
#define MIRT_OPT_VIEWS 256u         /* per-frame view tables instead of the BVH walk (same results; slower) */
#define MIRT_OPT_REFLECT_CHAINS 512u /* reflections as per-pixel chains in one kernel (k_reflect) instead of level by level (same results) */
#define MIRT_OPT_NO_LIGHT_TABLE 1024u /* shadow segments without the fp32 light-table pre-classification (same results) */
#define MIRT_OPT_NO_BOX_GATE 2048u  /* ablation: skip the reference's Box.Intersect of the face and object boxes
                                       (box.go:29-68), i.e. brute-force semantics; DESIGN.md §4.2 */
#define MIRT_OPT_LDS_STREAM 4096u   /* meshes beyond the LDS: each wave streams the BVH-ordered triangles of the
                                       leaves its primary rays test through an LDS slice in chunks of 112 faces
                                       (k_trace; same results).  The default since ABI 7's
                                       round-5 build: the flag is accepted and changes nothing */
#define MIRT_OPT_NO_LDS_STREAM 8192u /* ablation: meshes beyond the LDS read by the primary rays straight from
                                       HBM with scalar loads (the round-4 default; same results) */
int mirt_set_options(mirt_ctx *ctx, uint32_t flags);
/*
 * Launch shape of the frame kernel: every workgroup owns at least min_blocks_per_wg 8x8
 * pixel blocks (default 32) and a frame uses at most max_workgroups workgroups (0 = the
 * default, two per CU, the most that can be resident).  With several frames in flight
 * (one stream each) fewer, fuller workgroups per frame let the frames share the chip:
 * one frame's tail runs beside the next frame's start.  Results never change.
 */
int mirt_set_grid(mirt_ctx *ctx, uint32_t min_blocks_per_wg, uint32_t max_workgroups);
/*
 * A stream on a hardware queue of its own, for one of several frames in flight.  HIP maps
 * ordinary streams onto at most GPU_MAX_HW_QUEUES queues per process (default 4) and
 * streams sharing a queue serialise; a stream created with an explicit CU mask (here:
 * every CU) always gets a new queue.  Destroy with mirt_stream_destroy.
 */
int mirt_stream_create(mirt_ctx *ctx, void **stream);
int mirt_stream_destroy(mirt_ctx *ctx, void *stream);

/*
 * Diagnostic: evaluate one fp64 primitive of the kernels on the device for n inputs
 * (host buffers) so tests can pin device arithmetic against the host bit-for-bit.
 *   op 0: sqrt(a)   op 1: a / b   op 2: Go math.Pow(a, b)   op 3: Go math.Max(a, b)
 *   op 4: box.go:29-68 Box.Intersect as the kernels evaluate it: a holds n rays (origin,
 *         direction: 6 doubles each), b n boxes ({MinCorner, MaxCorner}: 6 doubles each),
 *         out[i] = 1.0 if ray i meets box i, else 0.0
 */
int mirt_debug_fp64(mirt_ctx *ctx, int op, uint32_t n, const double *a, const double *b, double *out);

/*
 * Diagnostic: per-wave timeline of the last traced frame while MIRT_OPT_TIMELINE is set
 * (one context-wide buffer: concurrent calls overwrite each other).  Synchronises the
 * device, copies up to max_records records of 8 uint64 each into out and returns the
 * number of records (>= 0) or a negative MIRT_E_* code.  Record:
 *   [0] kernel (0 primary, 1 shadow)  [1] global wave id
 *   [2] s_memrealtime at wave start   [3] at wave end (100 MHz constant clock)
 *   [4] s_memtime at wave start       [5] at wave end (shader clock)
 *   [6] s_memrealtime after the LDS mesh staging   [7] XCC id | work items taken << 32
 */
int mirt_debug_timeline(mirt_ctx *ctx, uint64_t *out, uint32_t max_records);

/*
 * Diagnostic: wave-level event counts of a library built with -DMIRT_DIAG=1 (all zero in
 * the default build), summed since the last call and reset: per query kind (base 0:
 * primary / nearest-hit sweeps, base 8: shadow segment sweeps) [base+0] triangle tests
 * entered, [+1] past inc != 0 and the r2 pre-reject, [+2] past the r2 range check,
 * [+3] past the r3 / r2+r3 / r1 checks, [+4] hits (t >= 0); [5] / [13] BVH node visits,
 * [6] / [14] leaves tested, [15] shadow tests past the t pre-test, [22] shadow tests
 * pre-classified against a light table (those skipped by the wave: [22] - [8]).
 * Synchronises the device; n <= 32.
 */
int mirt_debug_counters(mirt_ctx *ctx, uint64_t *out, uint32_t n);

/*
 * Diagnostic (host only, no device): the kernel-argument layout the library was compiled
 * with, as the device code assumes it.  k_trace reads its second and third arguments at
 * hand-computed offsets of the kernarg segment; a CPU test compares these with the code
 * object's own argument metadata (.args[].offset / .size) for every instantiation.
 *   [0] sizeof(FrameRecs)  [1] k_trace's WorkArgs offset  [2] sizeof(WorkArgs)
 *   [3] k_trace's FusedCopy offset  [4] sizeof(FusedCopy)  [5] sizeof(FrameArgs)
 *   [6] sizeof(OutPlanes)  [7] sizeof(BounceArgs)
 * Returns the number of words written (<= n).
 */
int mirt_debug_kernarg_layout(uint64_t *out, uint32_t n);

/*
 * Diagnostic (host only, no device): the light-table records the library builds for the
 * shadow segments of a one-object frame (kernels.hip SegPre): for n triangles given as
 * P1, E1 = P2 - P1, E2 = P3 - P1 (9 doubles each, the kernels' order), a mesh whose
 * largest |coordinate| is scale, the object at pos and nl lights, writes nl * n records of
 * 16 floats (W1, W2, W3, A, ntL, cw, cA, ctL) into out.  Lets host tests check the bounds.
 */
int mirt_debug_light_table(const double *tri, uint32_t n, double scale, const double pos[3], const double *lights,
                           uint32_t nl, float *out);
/* The same records built on the device (k_light_table, the builder the cache uses). */
int mirt_debug_light_table_gpu(mirt_ctx *ctx, const double *tri, uint32_t n, double scale, const double pos[3],
                               const double *lights, uint32_t nl, float *out);

/*
 * The light-table cache of one-object frames: tables keyed by (mesh, object
 * position, light set), built on the device on the stream of the first frame that reads them,
 * least recently used evicted past max_bytes (default 4 GiB) once the streams that read them
 * have moved on.  A frame finding no room traces without a table (same results, slower) and is
 * counted.  stats: out[0] builds, [1] hits, [2] evictions, [3] frames without a table (no room),
 * [4] builds that reused an evicted buffer, [5] live tables, [6] bytes held (live + being
 * retired), [7] the cap.
 */
int mirt_set_light_cache(mirt_ctx *ctx, uint64_t max_bytes);
int mirt_light_cache_stats(mirt_ctx *ctx, uint64_t out[8]);

/*
 * Diagnostic (host only, no device): the padded boxes the reference culls with, as NewBox
 * (box.go:21-26) turns the rtreego rect into corners, written as {MinCorner, MaxCorner}:
 *   mirt_face_bounds    face.Bounds (shared/state/mesh.go:30-50) of the triangle p1 p2 p3;
 *   mirt_object_bounds  Object.Bounds (shared/state/object.go:31-59) of an object at pos
 *                       whose mesh has the nv vertices v (nv*3 doubles).
 * MaxCorner = p + ((p + len) - p) with len = max(extent, boundEpsilon): the rtreego rect stores
 * p + len and NewBox subtracts p again.  The kernels gate every candidate face and object
 * with Box.Intersect on exactly these corners.
 */
void mirt_face_bounds(const double p1[3], const double p2[3], const double p3[3], double out[6]);
void mirt_object_bounds(const double *v, uint32_t nv, const double pos[3], double out[6]);

/*
 * Multi-GPU frames (one process per GPU of a box; SURVEY.md §8(b) mirt_trace_frame).  The
 * screen is cut into tile x tile_h tiles (tile_h == 0: full-height column strips, which are
 * contiguous in the column-major framebuffer) dealt to the ranks (column c of tile row r
 * goes to rank (c + s r) % world, s the smallest integer >= sqrt(world) coprime with world); each
 * rank traces its tiles into a packed rgbv plane, RCCL (send/recv in one group, on a stream
 * of its own, frames in issue order) gathers the planes to rank 0, and rank 0 unpacks them
 * into the frame's framebuffer.  `inflight` frames overlap, frame k on stream k % inflight
 * with framebuffer fbs[k % inflight] (rank 0 only; device planes of W x H pixels; the
 * planes a caller leaves NULL are not produced; with tile > 0 only rgb8, valid and rgbv can
 * be produced — rgb, face or object planes are rejected; fbs == NULL on the root: the group
 * allocates rgb8 + valid device planes itself, for callers that read frames through
 * mirt_group_frame_host and own no device memory).  world <= 64, inflight <= 32.  world == 1 with tile == 0 traces the
 * whole screen straight into the framebuffer (no tiles, no RCCL); world == 1 with tile > 0
 * rehearses the tiled path on one GPU.
 *   mirt_group_unique_id: rank 0 makes the RCCL id (128 bytes) every rank passes in.
 *   mirt_trace_frame:     enqueue the next frame (asynchronous; *index = its number).  Lone-frame
 *                         hold (world == 1, tile == 0; MIRT_LONE_HOLD=0 turns it off): a batch
 *                         completed while the group has nothing running is HELD, not launched,
 *                         and runs at the next mirt_trace_frame (with the fixed grid: a burst has
 *                         begun) or at mirt_group_wait / mirt_group_frame_host (any index) /
 *                         mirt_mesh_release / mirt_group_destroy (alone, with the whole chip).  A
 *                         submitted frame is always traced; none of these calls drops it.
 *   mirt_group_wait:      make `stream` wait for every enqueued frame (NULL: host wait).
 *   mirt_plan_tiles:      rank's tiles of the deal (returns the count; out may be NULL).
 */
typedef struct mirt_group mirt_group;
int mirt_group_unique_id(uint8_t *id);
int mirt_group_create(mirt_ctx *ctx, const uint8_t *unique_id, int rank, int world, uint32_t W, uint32_t H,
                      uint32_t tile, uint32_t tile_h, uint32_t inflight, const mirt_outputs *fbs, mirt_group **out);
/* Frames per k_trace launch (1..min(8, inflight), default 1), before the first frame:
 * mirt_trace_frame then only stages a frame until the batch is full (or the next frame
 * differs in mesh, objects, lights or options, or mirt_group_wait flushes it); the batch's
 * frames are traced by one launch and gathered by one RCCL group.  Results are the same. */
int mirt_group_set_batch(mirt_group *g, uint32_t frames_per_launch);
int mirt_trace_frame(mirt_group *group, const mirt_frame *frame, uint64_t *index);
int mirt_group_wait(mirt_group *group, void *stream);
void mirt_group_destroy(mirt_group *group);

/*
 * Transfer integrity.  Every rank's transfer ends with a two-word trailer {frame tag, words};
 * the root checks it in every gathered region before the unpack.  A region whose trailer is
 * missing, stale or at the wrong place (a rank that did not send, sent another frame or
 * computed another size) makes the frame fail: mirt_group_wait / mirt_group_frame_host
 * return MIRT_E_PEER naming the frame and the rank(s) — the reference master skips such a
 * frame (master/main.go:153-161).  At creation (world > 1) every rank's view of the group
 * (W, H, tile, tile_h, world, inflight, the deal) is compared with the root's over RCCL;
 * a disagreement fails mirt_group_create on every rank with MIRT_E_PEER.
 */
/* Deadline of every host wait of the group, in ms (0: none, the default).  A wait past it
 * returns MIRT_E_TIMEOUT; the root then reads the trailers of the stuck frames to name the
 * ranks whose transfers never arrived (mirt_group_failed_ranks), and the group accepts no
 * frame until mirt_group_exclude.  Stream waits (mirt_group_wait with a stream) have none. */
int mirt_group_set_timeout(mirt_group *g, uint32_t ms);
/* Bit r of *mask: rank r failed the last failing call.  Returns the number of such ranks. */
int mirt_group_failed_ranks(const mirt_group *g, uint64_t *mask);
/* Re-deal over the ranks still alive (bit r of alive = rank r stays; rank 0 must): the
 * analogue of the pool removing a worker whose heartbeat failed (master/pool/pool.go:224-260)
 * and the next frame being partitioned over the remaining workers (master/main.go:96-101).
 * Every surviving rank calls it with the same mask.  The communicator is shrunk
 * (ncclCommShrink with abort) or, if new_unique_id is non-NULL, rebuilt from that id (rank 0
 * makes it with mirt_group_unique_id and the caller distributes it).  Frames not yet waited
 * for are dropped; frame indices continue. */
int mirt_group_exclude(mirt_group *g, uint64_t alive, const uint8_t *new_unique_id);
/* Correctness mode of the tiled path on ONE GPU (world == 1, tile > 0, before the first
 * frame): the group traces every rank's share of a `world`-way deal into that rank's own
 * rgbv plane, packs it into that rank's transfer buffer exactly as a peer does, copies the
 * bytes an RCCL send would carry into the root's gathered region, checks the trailers and
 * unpacks every region: the N-GPU frame assembly, bit for bit, without RCCL. */
int mirt_group_emulate(mirt_group *g, uint32_t world);
/* Fault injection in an emulated world: the transfers of these ranks (bit r = rank r, never
 * rank 0) are not copied, as if those ranks stopped answering. */
int mirt_group_emulate_drop(mirt_group *g, uint64_t ranks);

/*
 * Host output (root): after each frame the assembled rgb8 + valid framebuffer is copied to
 * pinned host memory on the frame's stream (the region the frame's hit rectangle and the
 * slot's previous one cover; every other pixel is a miss, i.e. zero), so a frame completes
 * only once it is in host memory (ms/frame includes the D2H).
 * mirt_group_frame_host waits for frame `index` (within the deadline) and returns its host
 * planes (rgb8 and valid, column-major x*H + y, owned by the group, valid until frame
 * index + inflight is enqueued); MIRT_E_PEER if the frame failed.  The setting may change
 * between frames; it applies to frames enqueued after the call.
 */
int mirt_group_set_host_output(mirt_group *g, int enable);
int mirt_group_frame_host(mirt_group *g, uint64_t index, mirt_outputs *out);
/* The deal mirt_group uses (world > 1): as mirt_plan_tiles, with rank 0 (which also unpacks
 * every frame) taking b - 1 of every L = b N - 1 deal slots and the other ranks b each,
 * b = round(32 / N) (N = 8: 3 and 4 of 31). */
int mirt_group_plan_tiles(uint32_t W, uint32_t H, uint32_t tile, uint32_t tile_h, uint32_t world, uint32_t rank,
                          mirt_tile *out, uint32_t cap);
int mirt_plan_tiles(uint32_t W, uint32_t H, uint32_t tile, uint32_t tile_h, uint32_t world, uint32_t rank,
                    mirt_tile *out, uint32_t cap);

/*
 * One process driving the GPUs of a box behind the BulkTrace contract (SURVEY.md §8(b)
 * mirt_create(n_devices)).  A reference master sees ONE drop-in worker
 * (worker/distributed/main.go:46-91) whose orders — the rectangles of the master's partition
 * (master/main.go:54-91) — are cut into `strip`-pixel-wide column strips (default 8) dealt
 * round robin over the box's device entries; each entry traces its strips, and the order is
 * assembled on entry 0 and copied into the caller's host buffers in exactly mirt_trace_tile's
 * layout (pixel (x+i, y+j) at i*h + j, every plane of mirt_outputs).  Re-entrant like
 * mirt_trace_tile: concurrent orders each take a workspace of their own.
 *   devices   n device ordinals (NULL: 0..n-1).  Entries may repeat a device (one GPU
 *             standing in for several: the same deal and assembly, device copies instead of
 *             RCCL, which refuses two ranks on one GPU).  Each entry is a context of its own.
 *   transport MIRT_BOX_RCCL (default for n > 1 distinct devices: ncclCommInitAll over them,
 *             send/recv of each entry's planes to entry 0 over xGMI), MIRT_BOX_COPY (peer
 *             copies to entry 0; the default when devices repeat or librccl lacks
 *             ncclCommInitAll), MIRT_BOX_HOST (every entry copies its strips straight into a
 *             pinned host buffer over its own link).  The bytes returned never depend on it.
 *   Meshes go to every entry through mirt_box_mesh_upload (one id for all); options through
 *   mirt_box_set_options; mirt_box_ctx(b, i) is entry i's context (read-only use: profiling,
 *   light-cache statistics).
 */
#define MIRT_BOX_RCCL 1
#define MIRT_BOX_COPY 2
#define MIRT_BOX_HOST 3
typedef struct mirt_box mirt_box;
int mirt_device_count(void);
int mirt_box_create(const int *devices, uint32_t n, mirt_box **out);
void mirt_box_destroy(mirt_box *box);
int mirt_box_size(const mirt_box *box);
mirt_ctx *mirt_box_ctx(mirt_box *box, uint32_t i);
int mirt_box_set_transport(mirt_box *box, int transport);
int mirt_box_transport(const mirt_box *box);
int mirt_box_set_strip(mirt_box *box, uint32_t strip);
int mirt_box_set_options(mirt_box *box, uint32_t flags);
int mirt_box_mesh_upload(mirt_box *box, const double *v, uint32_t nv, const double *vn, uint32_t nn,
                         const uint32_t *fv, const uint32_t *fn, const uint32_t *fmat, uint32_t nf,
                         const mirt_material *mats, uint32_t nm, uint32_t *mesh_id);
int mirt_box_mesh_release(mirt_box *box, uint32_t mesh_id);
/* BulkTrace of one order on every entry of the box; synchronous, host buffers, as mirt_trace_tile. */
int mirt_box_trace_tile(mirt_box *box, const mirt_frame *frame, uint32_t x, uint32_t y, uint32_t w, uint32_t h,
                        uint32_t W, uint32_t H, const mirt_outputs *host_out, const volatile int *cancel,
                        mirt_stats *stats);

#ifdef __cplusplus
}
#endif
#endif /* MIRT_H */
