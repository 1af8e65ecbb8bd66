/*
 * box_bench.c — throughput of the box drop-in (mirt_box_*) under the reference master's
 * traffic, measured from a native caller as the Go worker would drive it (bench.py --box).
 *
 * The reference master starts one coordinator goroutine per frame (master/main.go:264-266);
 * the coordinator cuts the screen into one rectangle per worker (master/main.go:54-91) and
 * sends each as an asynchronous BulkTrace (master/pool/pool.go:148-197), which the worker's
 * gRPC server runs in a goroutine of its own (worker/distributed/main.go:46-91).  Here K
 * coordinator slots keep K frames in flight; each slot has one thread per rectangle (the
 * goroutine serving that BulkTrace) calling mirt_box_trace_tile into the order's rgb8 buffer
 * (TraceResults carries colours only), and a slot's frame is done when all its orders are.
 *
 *   box_bench <scene.json> <W> <H> <entries> <workers> <inflight> <frames> <warmup> [out.bin]
 *
 * Entry i of the box runs on device i % (devices present).  Prints one JSON line; out.bin gets
 * the last frame's assembled rgb8 (W*H*3, column-major x*H + y) for the caller's parity check.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mirt.h"
#include "mirt_scene.h"
#include "master_partition.h"

#define CHECK(call)                                                                       \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_ != MIRT_OK) {                                                             \
            fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #call, rc_,       \
                    mirt_last_error());                                                   \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

typedef struct {
    mirt_box *box;
    const mirt_frame *frame;
    uint32_t W, H;
    rect order;
    uint32_t slot, inflight;
    uint8_t *rgb8;            /* the order's TraceResults colours, i*h + j */
    pthread_barrier_t *slot_done;  /* the slot's orders of one frame */
    pthread_barrier_t *phase;      /* every thread + main, between phases */
    volatile uint64_t *nframes;    /* frames of the current phase (0: exit) */
    mirt_stats st;
    int rc;
} order_thread;

static void *serve(void *p) {
    order_thread *t = (order_thread *)p;
    mirt_outputs out;
    memset(&out, 0, sizeof(out));
    out.rgb8 = t->rgb8;
    for (;;) {
        pthread_barrier_wait(t->phase);  /* a phase starts */
        const uint64_t n = *t->nframes;
        if (n == 0) break;
        for (uint64_t f = t->slot; f < n; f += t->inflight) {
            const int rc = mirt_box_trace_tile(t->box, t->frame, t->order.x, t->order.y, t->order.w, t->order.h, t->W,
                                               t->H, &out, NULL, &t->st);
            if (rc != MIRT_OK && t->rc == MIRT_OK) {
                t->rc = rc;
                fprintf(stderr, "order failed: %d %s\n", rc, mirt_last_error());
            }
            pthread_barrier_wait(t->slot_done);  /* the frame is complete when all its orders are */
        }
        pthread_barrier_wait(t->phase);  /* the phase ends */
    }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int main(int argc, char **argv) {
    if (argc < 9) {
        fprintf(stderr, "usage: %s scene.json W H entries workers inflight frames warmup [out.bin]\n", argv[0]);
        return 2;
    }
    const uint32_t W = (uint32_t)atoi(argv[2]), H = (uint32_t)atoi(argv[3]);
    const int entries = atoi(argv[4]), workers = atoi(argv[5]), K = atoi(argv[6]);
    const uint64_t frames = (uint64_t)atoll(argv[7]), warmup = (uint64_t)atoll(argv[8]);
    if (entries < 1 || entries > 64 || workers < 1 || workers > 64 || K < 1 || K > 64 || frames < 1) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    mirt_scene *scene = NULL;
    if (mirt_scene_load(argv[1], &scene) != MIRT_OK) {
        fprintf(stderr, "scene: %s\n", mirt_scene_last_error());
        return 2;
    }
    const int ndev = mirt_device_count();
    int devs[64];
    for (int i = 0; i < entries; ++i) devs[i] = ndev > 0 ? i % ndev : 0;
    mirt_box *box = NULL;
    CHECK(mirt_box_create(devs, (uint32_t)entries, &box));
    const uint32_t nm = mirt_scene_mesh_count(scene);
    uint32_t *ids = calloc(nm ? nm : 1, sizeof(uint32_t));
    for (uint32_t i = 0; i < nm; ++i) {
        mirt_mesh_view v;
        CHECK(mirt_scene_mesh(scene, i, &v));
        CHECK(mirt_box_mesh_upload(box, v.vertices, v.n_vertices, v.normals, v.n_normals, v.face_v, v.face_n,
                                   v.face_mat, v.n_faces, v.materials, v.n_materials, &ids[i]));
    }
    const uint32_t no = mirt_scene_object_count(scene), nl = mirt_scene_light_count(scene);
    mirt_object *objs = calloc(no ? no : 1, sizeof(mirt_object));
    mirt_light *lights = calloc(nl ? nl : 1, sizeof(mirt_light));
    for (uint32_t i = 0; i < no; ++i) {
        CHECK(mirt_scene_object(scene, i, &objs[i]));
        objs[i].mesh_id = ids[objs[i].mesh_id];
    }
    for (uint32_t i = 0; i < nl; ++i) CHECK(mirt_scene_light(scene, i, &lights[i]));
    mirt_frame frame;
    memset(&frame, 0, sizeof(frame));
    frame.objects = objs;
    frame.n_objects = no;
    frame.lights = lights;
    frame.n_lights = nl;
    CHECK(mirt_scene_camera(scene, &frame.camera));

    rect orders[64];
    int n = 0;
    (void)partition((rect){0, 0, W, H}, (uint32_t)workers, 0, orders, &n);
    const int nt = K * n;
    order_thread *th = calloc((size_t)nt, sizeof(order_thread));
    pthread_t *tid = calloc((size_t)nt, sizeof(pthread_t));
    pthread_barrier_t *slot_done = calloc((size_t)K, sizeof(pthread_barrier_t));
    pthread_barrier_t phase;
    pthread_barrier_init(&phase, NULL, (unsigned)nt + 1);
    volatile uint64_t nframes = 0;
    for (int s = 0; s < K; ++s) pthread_barrier_init(&slot_done[s], NULL, (unsigned)n);
    for (int s = 0; s < K; ++s)
        for (int p = 0; p < n; ++p) {
            order_thread *t = &th[s * n + p];
            t->box = box;
            t->frame = &frame;
            t->W = W;
            t->H = H;
            t->order = orders[p];
            t->slot = (uint32_t)s;
            t->inflight = (uint32_t)K;
            t->rgb8 = calloc((size_t)orders[p].w * orders[p].h, 3);
            t->slot_done = &slot_done[s];
            t->phase = &phase;
            t->nframes = &nframes;
            pthread_create(&tid[s * n + p], NULL, serve, t);
        }
    /* warmup phase, then the timed phase */
    double t0 = 0, t1 = 0;
    for (int ph = 0; ph < 2; ++ph) {
        nframes = ph == 0 ? (warmup ? warmup : 1) : frames;
        pthread_barrier_wait(&phase);
        if (ph == 1) t0 = now_s();
        pthread_barrier_wait(&phase);
        if (ph == 1) t1 = now_s();
    }
    nframes = 0;
    pthread_barrier_wait(&phase);
    for (int i = 0; i < nt; ++i) pthread_join(tid[i], NULL);
    int bad = 0;
    for (int i = 0; i < nt; ++i) bad |= th[i].rc != MIRT_OK;
    /* the last frame's orders (slot (frames - 1) % K) drawn as the master does (master/main.go:164-176) */
    const int last = (int)((frames - 1) % (uint64_t)K);
    uint8_t *fb = calloc((size_t)W * H, 3);
    uint64_t hits = 0, shadow = 0, tests = 0;
    for (int p = 0; p < n; ++p) {
        const order_thread *t = &th[last * n + p];
        for (uint32_t a = 0; a < t->order.w; ++a)
            memcpy(fb + 3 * ((size_t)(t->order.x + a) * H + t->order.y), t->rgb8 + 3 * (size_t)a * t->order.h,
                   3 * (size_t)t->order.h);
        hits += t->st.hits;
        shadow += t->st.shadow_rays;
        tests += t->st.tri_tests;
    }
    if (argc > 9) {
        FILE *f = fopen(argv[9], "wb");
        if (!f || fwrite(fb, 3, (size_t)W * H, f) != (size_t)W * H) bad = 1;
        if (f) fclose(f);
    }
    const double ms = 1e3 * (t1 - t0) / (double)frames;
    const uint64_t rays = (uint64_t)W * H + shadow;
    printf("{\"entries\": %d, \"transport\": %d, \"workers\": %d, \"orders_per_frame\": %d, \"inflight\": %d, "
           "\"frames\": %llu, \"warmup\": %llu, \"ms_per_frame\": %.4f, \"mrays_s\": %.1f, \"rays_per_frame\": %llu, "
           "\"hits_per_frame\": %llu, \"tri_tests_per_frame\": %llu, \"devices\": %d, \"ok\": %s}\n",
           entries, mirt_box_transport(box), workers, n, K, (unsigned long long)frames, (unsigned long long)warmup, ms,
           (double)rays / (ms * 1e3), (unsigned long long)rays, (unsigned long long)hits, (unsigned long long)tests,
           ndev, bad ? "false" : "true");
    mirt_box_destroy(box);
    mirt_scene_free(scene);
    return bad;
}
