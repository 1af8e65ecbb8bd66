/*
 * mirt_worker.c — a non-Go, non-Python caller of libmirt.so: the call sequence of the
 * drop-in GPU worker (worker/gpu in go/) in plain C, with no torch and no
 * HIP calls of its own, so the HIP runtime comes in through libmirt's RUNPATH.
 *
 *   Register   (worker/distributed/main.go:100-129): the scene -> mirt_create -> one
 *              mirt_mesh_upload per mesh.  With --gob the scene is MasterState.state, the
 *              gob-encoded Environment a master sends (mirt_scene_from_gob), and the frame
 *              is a WorkOrder.diff linked to it (mirt_scene_link_gob, main.go:56-64); without
 *              it mirt_scene_load reads scene.json (shared/state/mesh.go:109-213 semantics).
 *   BulkTrace  (worker/distributed/main.go:46-89): the master cuts the screen into one
 *              rectangle per worker (master/main.go:54-91, restated below) and each order
 *              is served concurrently — gRPC runs every BulkTrace in its own goroutine — by
 *              mirt_trace_tile into host buffers; results go back as comms.TraceResults,
 *              uint8 colours in uint32 fields, column-major i*h + j, and the master draws
 *              them (master/main.go:164-176).
 *   Frame group (mirt_trace_frame, world 1, library-owned framebuffers, host output):
 *              three frames in flight; each host frame must equal the BulkTrace frame.
 *   Box        (--box N, mirt_box_*): ONE worker driving N device entries (device i % the
 *              devices present: one GPU may stand in for a box) serves the same orders
 *              concurrently through mirt_box_trace_tile; the assembled frame must equal the
 *              one-context frame.
 *
 *   mirt_worker [--box N] <scene.json> <W> <H> <out.bin> [workers]
 *   mirt_worker [--box N] --gob <state.gob> <diff.gob> <W> <H> <out.bin> [workers]
 * Writes rgb8 (W*H*3) then valid (W*H) of the assembled frame, column-major x*H + y.
 * Exit status 0 = every check passed.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mirt.h"
#include "mirt_scene.h"

#define CHECK(call)                                                                       \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_ != MIRT_OK) {                                                             \
            fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_,       \
                    mirt_last_error());                                                   \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

#include "master_partition.h"

typedef struct {
    mirt_ctx *ctx;
    mirt_box *box;       /* non-NULL: the order is served by the box (mirt_box_trace_tile) */
    const mirt_frame *frame;
    rect order;          /* comms.WorkOrder x, y, width, height */
    uint32_t W, H;
    uint32_t *results;   /* comms.TraceResults: r, g, b per pixel (uint32 fields) */
    int rc;
} bulk_trace;

/* One BulkTrace call (worker/distributed/main.go:46-89) on its own thread. */
static int read_all(const char *path, uint8_t **data, size_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    const long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    *data = malloc(len > 0 ? (size_t)len : 1);
    *n = len > 0 && fread(*data, 1, (size_t)len, f) == (size_t)len ? (size_t)len : 0;
    fclose(f);
    return len > 0 && *n == (size_t)len ? 0 : -1;
}

static void *serve(void *p) {
    bulk_trace *b = (bulk_trace *)p;
    const size_t n = (size_t)b->order.w * b->order.h;
    uint8_t *rgb8 = malloc(3 * n), *valid = malloc(n);
    mirt_outputs out;
    memset(&out, 0, sizeof(out));
    out.rgb8 = rgb8;
    out.valid = valid;
    b->rc = b->box ? mirt_box_trace_tile(b->box, b->frame, b->order.x, b->order.y, b->order.w, b->order.h, b->W, b->H,
                                         &out, NULL, NULL)
                   : mirt_trace_tile(b->ctx, b->frame, b->order.x, b->order.y, b->order.w, b->order.h, b->W, b->H, &out,
                                     NULL, NULL);
    b->results = malloc(3 * n * sizeof(uint32_t));
    for (size_t k = 0; k < n; ++k) /* misses are (0, 0, 0) already */
        for (int c = 0; c < 3; ++c) b->results[3 * k + c] = rgb8[3 * k + c];
    free(rgb8);
    free(valid);
    return NULL;
}

/* Serve the orders concurrently (one thread each) on ctx or box and draw them into fb_rgb8
 * as the master does (master/main.go:164-176, pixel i*h + j).  Returns nonzero on a failure. */
static int serve_orders(mirt_ctx *ctx, mirt_box *box, const mirt_frame *frame, const rect *orders, int n, uint32_t W,
                        uint32_t H, uint8_t *fb_rgb8) {
    bulk_trace bt[256];
    pthread_t th[256];
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        bt[i] = (bulk_trace){ctx, box, frame, orders[i], W, H, NULL, 0};
        pthread_create(&th[i], NULL, serve, &bt[i]);
    }
    for (int i = 0; i < n; ++i) {
        pthread_join(th[i], NULL);
        if (bt[i].rc != MIRT_OK) {
            fprintf(stderr, "BulkTrace %d failed: %d (%s)\n", i, bt[i].rc, box ? "box" : "context");
            bad = 1;
            free(bt[i].results);
            continue;
        }
        const rect o = bt[i].order;
        for (uint32_t a = 0; a < o.w; ++a)
            for (uint32_t b = 0; b < o.h; ++b) {
                const size_t src = (size_t)a * o.h + b, dst = (size_t)(o.x + a) * H + (o.y + b);
                for (int c = 0; c < 3; ++c) fb_rgb8[3 * dst + c] = (uint8_t)bt[i].results[3 * src + c];
            }
        free(bt[i].results);
    }
    return bad;
}

int main(int argc, char **argv) {
    int box_n = 0;
    if (argc > 2 && strcmp(argv[1], "--box") == 0) {
        box_n = atoi(argv[2]);
        if (box_n < 1 || box_n > 64) {
            fprintf(stderr, "--box needs 1..64 entries\n");
            return 2;
        }
        argv[2] = argv[0];  /* drop the two words: argv[0] moves up */
        argv += 2;
        argc -= 2;
    }
    const int gob = argc > 1 && strcmp(argv[1], "--gob") == 0;
    char **a = argv + (gob ? 2 : 0);  /* a[1] = scene (or state.gob; a[0] = diff.gob), a[2] = W, ... */
    const int na = argc - (gob ? 2 : 0);
    if (na < 5) {
        fprintf(stderr, "usage: %s scene.json W H out.bin [workers]\n"
                        "       %s --gob state.gob diff.gob W H out.bin [workers]\n", argv[0], argv[0]);
        return 2;
    }
    const uint32_t W = (uint32_t)atoi(a[2]), H = (uint32_t)atoi(a[3]);
    uint32_t workers = na > 5 ? (uint32_t)atoi(a[5]) : 4;
    const char *out_path = a[4];
    if (mirt_abi_version() != MIRT_ABI_VERSION) {
        fprintf(stderr, "ABI %d, header %d\n", mirt_abi_version(), MIRT_ABI_VERSION);
        return 2;
    }
    /* Register: the scene and its meshes */
    mirt_scene *scene = NULL, *linked = NULL;
    if (gob) {
        uint8_t *state = NULL, *diff = NULL;
        size_t ns = 0, nd = 0;
        if (read_all(argv[2], &state, &ns) || read_all(argv[3], &diff, &nd)) {
            fprintf(stderr, "cannot read %s / %s\n", argv[2], argv[3]);
            return 2;
        }
        if (mirt_scene_from_gob(state, ns, &scene) != MIRT_OK || mirt_scene_link_gob(scene, diff, nd, &linked) != MIRT_OK) {
            fprintf(stderr, "gob: %s\n", mirt_scene_last_error());
            return 2;
        }
        free(state);
        free(diff);
    } else if (mirt_scene_load(a[1], &scene) != MIRT_OK) {
        fprintf(stderr, "scene: %s\n", mirt_scene_last_error());
        return 2;
    }
    mirt_ctx *ctx = NULL;
    CHECK(mirt_create(0, &ctx));
    const uint32_t nm = mirt_scene_mesh_count(scene);
    uint32_t *mesh_ids = calloc(nm ? nm : 1, sizeof(uint32_t));
    for (uint32_t i = 0; i < nm; ++i) {
        mirt_mesh_view v;
        CHECK(mirt_scene_mesh(scene, i, &v));
        CHECK(mirt_mesh_upload(ctx, v.vertices, v.n_vertices, v.normals, v.n_normals, v.face_v, v.face_n, v.face_mat,
                               v.n_faces, v.materials, v.n_materials, &mesh_ids[i]));
    }
    const mirt_scene *mut = gob ? linked : scene;
    const uint32_t no_all = mirt_scene_object_count(mut), nl = mirt_scene_light_count(mut);
    /* WorkOrder.diff: objects (their mesh by id), lights, camera */
    mirt_object *objs = calloc(no_all ? no_all : 1, sizeof(mirt_object));
    mirt_light *lights = calloc(nl ? nl : 1, sizeof(mirt_light));
    uint32_t no = 0;
    for (uint32_t i = 0; i < no_all; ++i) {
        CHECK(mirt_scene_object(mut, i, &objs[no]));
        if (objs[no].mesh_id == MIRT_NO_MESH) continue; /* LinkTo left its mesh nil: never hit */
        objs[no].mesh_id = mesh_ids[objs[no].mesh_id];
        ++no;
    }
    for (uint32_t i = 0; i < nl; ++i) CHECK(mirt_scene_light(mut, i, &lights[i]));
    mirt_frame frame;
    memset(&frame, 0, sizeof(frame));
    frame.objects = objs;
    frame.n_objects = no;
    frame.lights = lights;
    frame.n_lights = nl;
    CHECK(mirt_scene_camera(mut, &frame.camera));

    /* BulkTrace: the master's partition, every order on its own thread */
    rect orders[256];
    int n = 0;
    if (workers < 1 || workers > 256) workers = 4;
    (void)partition((rect){0, 0, W, H}, workers, 0, orders, &n);
    uint8_t *fb_rgb8 = calloc((size_t)W * H, 3), *fb_valid = calloc((size_t)W * H, 1);
    int bad = serve_orders(ctx, NULL, &frame, orders, n, W, H, fb_rgb8);
    /* the valid plane of the whole screen from one more call (the wire carries colours only) */
    {
        mirt_outputs out;
        memset(&out, 0, sizeof(out));
        out.valid = fb_valid;
        CHECK(mirt_trace_tile(ctx, &frame, 0, 0, W, H, W, H, &out, NULL, NULL));
    }

    /* the frame group: library-owned device framebuffers, frames copied to host memory */
    mirt_group *g = NULL;
    CHECK(mirt_group_create(ctx, NULL, 0, 1, W, H, 0, 0, 2, NULL, &g));
    CHECK(mirt_group_set_host_output(g, 1));
    CHECK(mirt_group_set_timeout(g, 10000));
    uint64_t idx[3];
    for (int k = 0; k < 3; ++k) {
        CHECK(mirt_trace_frame(g, &frame, &idx[k]));
        if (k > 0) {
            mirt_outputs h;
            CHECK(mirt_group_frame_host(g, idx[k - 1], &h));
            if (memcmp(h.rgb8, fb_rgb8, (size_t)W * H * 3) || memcmp(h.valid, fb_valid, (size_t)W * H)) {
                fprintf(stderr, "group frame %d differs from the BulkTrace frame\n", k - 1);
                bad = 1;
            }
        }
    }
    CHECK(mirt_group_wait(g, NULL));
    mirt_group_destroy(g);

    /* the box: one worker, box_n device entries, the same orders (mesh ids agree: the box
     * uploads every mesh in the same order as the context did) */
    int box_equal = -1;
    if (box_n > 0) {
        const int ndev = mirt_device_count();
        int devs[64];
        for (int i = 0; i < box_n; ++i) devs[i] = ndev > 0 ? i % ndev : 0;
        mirt_box *box = NULL;
        CHECK(mirt_box_create(devs, (uint32_t)box_n, &box));
        for (uint32_t i = 0; i < nm; ++i) {
            mirt_mesh_view v;
            uint32_t id = 0;
            CHECK(mirt_scene_mesh(scene, i, &v));
            CHECK(mirt_box_mesh_upload(box, v.vertices, v.n_vertices, v.normals, v.n_normals, v.face_v, v.face_n,
                                       v.face_mat, v.n_faces, v.materials, v.n_materials, &id));
            if (id != mesh_ids[i]) {
                fprintf(stderr, "box mesh id %u != context mesh id %u\n", id, mesh_ids[i]);
                bad = 1;
            }
        }
        uint8_t *box_rgb8 = calloc((size_t)W * H, 3);
        bad |= serve_orders(NULL, box, &frame, orders, n, W, H, box_rgb8);
        box_equal = memcmp(box_rgb8, fb_rgb8, (size_t)W * H * 3) == 0;
        if (!box_equal) {
            fprintf(stderr, "the box's frame differs from the context's\n");
            bad = 1;
        }
        free(box_rgb8);
        printf("mirt_worker: box of %d entries (transport %d), orders equal: %s\n", box_n, mirt_box_transport(box),
               box_equal ? "yes" : "NO");
        mirt_box_destroy(box);
    }

    FILE *f = fopen(out_path, "wb");
    if (!f || fwrite(fb_rgb8, 3, (size_t)W * H, f) != (size_t)W * H || fwrite(fb_valid, 1, (size_t)W * H, f) != (size_t)W * H) {
        fprintf(stderr, "cannot write %s\n", out_path);
        return 2;
    }
    fclose(f);
    mirt_destroy(ctx);
    mirt_scene_free(linked);
    mirt_scene_free(scene);
    printf("mirt_worker: %ux%u, %d BulkTrace orders on %d threads, group frames equal: %s\n", W, H, n, n,
           bad ? "NO" : "yes");
    return bad;
}
