/* master_partition.h — the reference master's screen partition (master/main.go:54-91), shared
 * by the C callers of libmirt (mirt_worker.c, box_bench.c). */
#ifndef MASTER_PARTITION_H
#define MASTER_PARTITION_H
#include <stdint.h>

typedef struct { uint32_t x, y, w, h; } rect;

/* master/main.go:54-91 partition() with workerRedundancy = 1 (master/main.go:31):
 * recursive bisection, alternating dimensions; returns the leftover workers. */
static inline uint32_t partition(rect area, uint32_t workers, uint32_t dim, rect *out, int *n) {
    const uint32_t wk = 50, hk = 50; /* widthKernel, heightKernel */
    if (workers < 2) {
        out[(*n)++] = area;
        return 0;
    }
    if (area.w <= wk && area.h <= hk) {
        out[(*n)++] = area;
        return workers - 1;
    } else if (area.w <= wk) {
        dim = 1;
    } else if (area.h <= hk) {
        dim = 0;
    }
    rect l, r;
    if (dim % 2 == 0) {
        l = (rect){area.x, area.y, area.w / 2, area.h};
        r = (rect){area.x + area.w / 2, area.y, area.w / 2 + area.w % 2, area.h};
    } else {
        l = (rect){area.x, area.y, area.w, area.h / 2};
        r = (rect){area.x, area.y + area.h / 2, area.w, area.h / 2 + area.h % 2};
    }
    const uint32_t rem = partition(l, workers / 2 + workers % 2, (dim + 1) % 2, out, n);
    return partition(r, workers / 2 + rem, (dim + 1) % 2, out, n);
}

#endif
