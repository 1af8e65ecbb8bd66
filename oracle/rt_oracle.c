/*
 * oracle/rt_oracle.c — CPU restatement of the reference's per-pixel trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libmirt.so, the Python host
 * mirror) may link, load or call this file.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it, and only as the checker / the timed CPU
 * baseline ("kind": "port").
 *
 * PARITY STATUS: UNPINNED BY THE REFERENCE.  The reference is Go; no Go toolchain
 * exists in this image or on the GPU box, its third-party deps (gwob, rtreego) are
 * not vendored, and it ships no tests or golden vectors.  This
 * restatement is pinned instead by (1) hand-derived Möller–Trumbore known-answer
 * tests, (2) an independent numpy restatement (oracle/np_oracle.py) that must agree
 * bit-for-bit, and (3) restatements of Go's math.Tan / math.Pow checked against libm.
 *
 * Arithmetic: fp64, IEEE round-to-nearest, NO contraction (build with
 * -ffp-contract=off), in exactly the operation order of the Go source, because Go
 * on amd64 (GOAMD64=v1) never fuses x*y+z.
 *
 * Follows (paths relative to the reference root):
 *   shared/geom/vector.go:14-57        vector ops           -> v_add .. v_len
 *   shared/geom/triangle.go:24-77      Normal/InterpNormal/Möller–Trumbore -> tri_*
 *   shared/geom/box.go:21-68           NewBox / Box.Intersect (R-tree culling)
 *   shared/state/object.go:31-110      Object.Bounds / Object.Intersection
 *   shared/state/mesh.go:30-50         face.Bounds
 *   shared/state/camera.go:35-44       NewCamera
 *   shared/colour/colour.go:28-61      RGB arithmetic
 *   worker/shared/tracer/tracer.go:15-91  pixelToPoint / trace / phong / Trace
 *   worker/sequential/main.go:21-28    serial i-outer, j-inner pixel loop
 *   worker/distributed/main.go:67-89   tile loop, results[i*h+j], uint8(255*c)
 * Third-party semantics restated (unpinned, not vendored in the reference):
 *   github.com/mwindels/rtreego (fork of dhconnelly/rtreego, no version pinned):
 *     Guttman R-tree, NewTree(3, 2, 5), quadratic split, SearchCondition DFS.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ vectors */
typedef struct { double x, y, z; } vec3;

static inline vec3 v_make(double x, double y, double z) { vec3 r = {x, y, z}; return r; }
/* vector.go:14-16 */
static inline vec3 v_add(vec3 a, vec3 b) { return v_make(a.x + b.x, a.y + b.y, a.z + b.z); }
/* vector.go:19-21 */
static inline vec3 v_sub(vec3 a, vec3 b) { return v_make(a.x - b.x, a.y - b.y, a.z - b.z); }
/* vector.go:24-26: Scale multiplies s * component (operand order kept) */
static inline vec3 v_scale(vec3 a, double s) { return v_make(s * a.x, s * a.y, s * a.z); }
/* vector.go:29-31: (x*x' + y*y') + z*z' */
static inline double v_dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* vector.go:34-36 */
static inline vec3 v_cross(vec3 a, vec3 b) {
    return v_make(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* vector.go:45-47 */
static inline int v_zero(vec3 a) { return a.x == 0.0 && a.y == 0.0 && a.z == 0.0; }
/* vector.go:50-53: three true divisions by the magnitude */
static inline vec3 v_norm(vec3 a) {
    double mag = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return v_make(a.x / mag, a.y / mag, a.z / mag);
}
/* vector.go:56-58 */
static inline double v_len(vec3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

/* ------------------------------------------------------- Go math restated */
/* Go math.Min / math.Max special cases (signed zero, NaN, Inf). */
static inline double go_min(double x, double y) {
    if (isinf(x) && x < 0) return x;
    if (isinf(y) && y < 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? x : y;
    return x < y ? x : y;
}
static inline double go_max(double x, double y) {
    if (isinf(x) && x > 0) return x;
    if (isinf(y) && y > 0) return y;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0 && x == y) return signbit(x) ? y : x;
    return x > y ? x : y;
}

/* Go math.Frexp: frac in [0.5, 1), handles subnormals by normalising first. */
static double go_frexp(double f, int *e) {
    *e = 0;
    if (f == 0 || isinf(f) || isnan(f)) return f;
    if (fabs(f) < 2.2250738585072014e-308) { f *= 4503599627370496.0; *e = -52; } /* 1<<52 */
    uint64_t x; memcpy(&x, &f, 8);
    *e += (int)((x >> 52) & 0x7ff) - 1022;
    x &= ~((uint64_t)0x7ff << 52);
    x |= (uint64_t)1022 << 52;
    memcpy(&f, &x, 8);
    return f;
}
/* Go math.normalize: scale a subnormal into the normal range. */
static double go_normalize(double x, int *e) {
    *e = 0;
    if (fabs(x) < 2.2250738585072014e-308) { *e = -52; return x * 4503599627370496.0; }
    return x;
}
/* Go math.Ldexp (single final rounding for subnormal results). */
static double go_ldexp(double frac, int exp) {
    if (frac == 0 || isinf(frac) || isnan(frac)) return frac;
    int e;
    frac = go_normalize(frac, &e);
    exp += e;
    uint64_t x; memcpy(&x, &frac, 8);
    exp += (int)((x >> 52) & 0x7ff) - 1023;
    if (exp < -1075) return copysign(0.0, frac);
    if (exp > 1023) return frac < 0 ? -INFINITY : INFINITY;
    double m = 1.0;
    if (exp < -1022) { exp += 53; m = 1.0 / 9007199254740992.0; }
    x &= ~((uint64_t)0x7ff << 52);
    x |= (uint64_t)(exp + 1023) << 52;
    double r; memcpy(&r, &x, 8);
    return m * r;
}
static int go_is_odd_int(double x) {
    if (fabs(x) >= 9007199254740992.0) return 0;
    double xi; double xf = modf(x, &xi);
    return xf == 0 && ((int64_t)xi & 1) == 1;
}
/*
 * Go math.Pow (pure Go on amd64): repeated squaring on the Frexp mantissa for the
 * integer part of y.  The fractional part uses Exp(yf*Log(x)); Go's amd64 Exp/Log are
 * assembly, so for non-integer exponents this (and the GPU) uses libm exp/log and
 * agrees only to a few ulp (the example scene's Ns = 10 is an integer: bit-exact).
 */
double or_go_pow(double x, double y) {
    if (y == 0 || x == 1) return 1;
    if (y == 1) return x;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0) {
        if (y < 0) return (signbit(x) && go_is_odd_int(y)) ? -INFINITY : INFINITY;
        return (signbit(x) && go_is_odd_int(y)) ? x : 0;
    }
    if (isinf(y)) {
        if (x == -1) return 1;
        if ((fabs(x) < 1) == (y > 0)) return 0;
        return INFINITY;
    }
    if (isinf(x)) {
        if (x < 0) return or_go_pow(1 / x, -y);
        return y < 0 ? 0 : INFINITY;
    }
    if (y == 0.5) return sqrt(x);
    if (y == -0.5) return 1 / sqrt(x);
    double yi; double yf = modf(fabs(y), &yi);
    if (yf != 0 && x < 0) return NAN;
    if (yi >= 9223372036854775808.0) {
        if (x == -1) return 1;
        if ((fabs(x) < 1) == (y > 0)) return 0;
        return INFINITY;
    }
    double a1 = 1.0; int ae = 0;
    if (yf != 0) {
        if (yf > 0.5) { yf--; yi++; }
        a1 = exp(yf * log(x));
    }
    int xe; double x1 = go_frexp(x, &xe);
    for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
        if (xe < -(1 << 12) || (1 << 12) < xe) {
            ae += xe;
            break;
        }
        if ((i & 1) == 1) { a1 *= x1; ae += xe; }
        x1 *= x1;
        xe <<= 1;
        if (x1 < .5) { x1 += x1; xe--; }
    }
    if (y < 0) { a1 = 1 / a1; ae = -ae; }
    return go_ldexp(a1, ae);
}

/* Go math.Tan (pure Go, Cephes coefficients; tracer.go:17 calls it once per pixel). */
static const double TAN_P[3] = {-1.30936939181383777646e4, 1.15351664838587416140e6,
                                -1.79565251976484877988e7};
static const double TAN_Q[5] = {1.0, 1.36812963470692954678e4, -1.32089234440210967447e6,
                                2.50083801823357915839e7, -5.38695755929454629881e7};
double or_go_tan(double x) {
    const double PI4A = 7.85398125648498535156e-1, PI4B = 3.77489470793079817668e-8,
                 PI4C = 2.69515142907905952645e-15;
    const double FOUR_OVER_PI = 1.27323954473516268615107010698011489627567716592365;
    if (x == 0 || isnan(x)) return x;
    if (isinf(x)) return NAN;
    int sign = 0;
    if (x < 0) { x = -x; sign = 1; }
    /* Go switches to Payne–Hanek reduction at 1<<29; camera fovs never get there. */
    if (x >= 536870912.0) return sign ? -tan(x) : tan(x);
    uint64_t j = (uint64_t)(x * FOUR_OVER_PI);
    double y = (double)j;
    if (j & 1) { j++; y++; }
    double z = ((x - y * PI4A) - y * PI4B) - y * PI4C;
    double zz = z * z;
    if (zz > 1e-14)
        y = z + z * (zz * (((TAN_P[0] * zz) + TAN_P[1]) * zz + TAN_P[2]) /
                     ((((zz + TAN_Q[1]) * zz + TAN_Q[2]) * zz + TAN_Q[3]) * zz + TAN_Q[4]));
    else
        y = z;
    if (j & 2) y = -1 / y;
    if (sign) y = -y;
    return y;
}

/* ------------------------------------------------------------- scene types */
typedef struct {
    const double *vertices;   uint32_t n_vertices;  /* nv*3, float32-parsed widened */
    const double *normals;    uint32_t n_normals;   /* nn*3, already normalised; may be 0 */
    const uint32_t *face_v;   const uint32_t *face_n; const uint32_t *face_mat;
    uint32_t n_faces;
    const double *materials;  uint32_t n_materials; /* 10 per: ka[3] kd[3] ks[3] ns */
} or_mesh;
typedef struct { uint32_t mesh; uint32_t _pad; double pos[3]; } or_object;
typedef struct { double pos[3]; double col[3]; } or_light;
typedef struct {
    const or_mesh *meshes;     uint32_t n_meshes;
    const or_object *objects;  uint32_t n_objects;
    const or_light *lights;    uint32_t n_lights;
    double cam_pos[3], cam_dir[3], fov;
} or_scene;
typedef struct { uint32_t x, y, w, h; } or_tile;
typedef struct {
    uint64_t primary_rays, shadow_rays, hits, tri_tests, box_tests;
    uint64_t reflection_rays;  /* configs[4] extension (or_set_bounces) */
} or_stats;

/* ------------------------------------------------------------- R-tree (rtreego) */
typedef struct { double p[3], q[3]; } rect;      /* rtreego Rect: p = min, q = p + lengths */
typedef struct rnode rnode;
typedef struct { rect bb; rnode *child; int32_t obj; } rentry;
struct rnode { rnode *parent; int leaf, level, n; rentry e[6]; };
typedef struct { rnode *root; int size, height; } rtree;

static rect rect_new(const double p[3], const double len[3]) {
    rect r;
    for (int i = 0; i < 3; i++) { r.p[i] = p[i]; r.q[i] = p[i] + len[i]; }
    return r;
}
static double rect_size(const rect *r) {
    double s = 1;
    for (int i = 0; i < 3; i++) s *= r->q[i] - r->p[i];
    return s;
}
static rect rect_union(const rect *a, const rect *b) {
    rect r;
    for (int i = 0; i < 3; i++) {
        r.p[i] = a->p[i] <= b->p[i] ? a->p[i] : b->p[i];
        r.q[i] = a->q[i] <= b->q[i] ? b->q[i] : a->q[i];
    }
    return r;
}
static double rect_enlargement(const rect *bb, const rect *add) {
    rect u = rect_union(bb, add);
    return rect_size(&u) - rect_size(bb);
}
static rect node_bb(const rnode *n) {
    rect r = n->e[0].bb;
    for (int i = 1; i < n->n; i++) r = rect_union(&r, &n->e[i].bb);
    return r;
}
static rnode *node_new(rnode *parent, int leaf, int level) {
    rnode *n = (rnode *)calloc(1, sizeof(rnode));
    n->parent = parent; n->leaf = leaf; n->level = level;
    return n;
}
static void node_free(rnode *n) {
    if (!n) return;
    if (!n->leaf) for (int i = 0; i < n->n; i++) node_free(n->e[i].child);
    free(n);
}
static rnode *choose_node(rnode *n, const rect *bb, int level) {
    if (n->leaf || n->level == level) return n;
    int best = 0; double bdiff = 0, barea = 0;
    for (int i = 0; i < n->n; i++) {
        double d = rect_enlargement(&n->e[i].bb, bb), a = rect_size(&n->e[i].bb);
        if (i == 0 || d < bdiff || (d == bdiff && a < barea)) { best = i; bdiff = d; barea = a; }
    }
    return choose_node(n->e[best].child, bb, level);
}
/* Guttman quadratic split, min group size m (rtreego node.split). */
static rnode *node_split(rnode *n, int m) {
    rentry all[6]; int cnt = n->n;
    memcpy(all, n->e, sizeof(rentry) * cnt);
    int s1 = 0, s2 = 1; double worst = -INFINITY;
    for (int i = 0; i < cnt; i++)
        for (int j = i + 1; j < cnt; j++) {
            rect u = rect_union(&all[i].bb, &all[j].bb);
            double d = rect_size(&u) - rect_size(&all[i].bb) - rect_size(&all[j].bb);
            if (d > worst) { worst = d; s1 = i; s2 = j; }
        }
    rnode *right = node_new(n->parent, n->leaf, n->level);
    n->n = 0;
    int used[6] = {0};
    n->e[n->n++] = all[s1]; used[s1] = 1;
    right->e[right->n++] = all[s2]; used[s2] = 1;
    rect lbb = all[s1].bb, rbb = all[s2].bb;
    int remaining = cnt - 2;
    while (remaining > 0) {
        if (n->n + remaining == m) {
            for (int i = 0; i < cnt; i++) if (!used[i]) { n->e[n->n++] = all[i]; used[i] = 1; }
            break;
        }
        if (right->n + remaining == m) {
            for (int i = 0; i < cnt; i++) if (!used[i]) { right->e[right->n++] = all[i]; used[i] = 1; }
            break;
        }
        int next = -1; double maxdiff = -1, d1b = 0, d2b = 0;
        for (int i = 0; i < cnt; i++) {
            if (used[i]) continue;
            double d1 = rect_enlargement(&lbb, &all[i].bb), d2 = rect_enlargement(&rbb, &all[i].bb);
            double diff = fabs(d1 - d2);
            if (diff > maxdiff) { maxdiff = diff; next = i; d1b = d1; d2b = d2; }
        }
        int to_left;
        if (d1b != d2b) to_left = d1b < d2b;
        else if (rect_size(&lbb) != rect_size(&rbb)) to_left = rect_size(&lbb) < rect_size(&rbb);
        else to_left = n->n <= right->n;
        if (to_left) { n->e[n->n++] = all[next]; lbb = rect_union(&lbb, &all[next].bb); }
        else { right->e[right->n++] = all[next]; rbb = rect_union(&rbb, &all[next].bb); }
        used[next] = 1; remaining--;
    }
    if (!n->leaf) {
        for (int i = 0; i < n->n; i++) n->e[i].child->parent = n;
        for (int i = 0; i < right->n; i++) right->e[i].child->parent = right;
    }
    return right;
}
static int entry_index(rnode *parent, rnode *child) {
    for (int i = 0; i < parent->n; i++) if (parent->e[i].child == child) return i;
    return -1;
}
static void rtree_insert(rtree *t, rect bb, int32_t obj) {
    rentry e; e.bb = bb; e.child = NULL; e.obj = obj;
    rnode *leaf = choose_node(t->root, &bb, 1);
    leaf->e[leaf->n++] = e;
    rnode *split = NULL;
    if (leaf->n > 5) split = node_split(leaf, 2);
    /* adjustTree */
    rnode *n = leaf, *nn = split;
    while (n != t->root) {
        rnode *parent = n->parent;
        int idx = entry_index(parent, n);
        parent->e[idx].bb = node_bb(n);
        rnode *psplit = NULL;
        if (nn) {
            rentry ne; ne.bb = node_bb(nn); ne.child = nn; ne.obj = -1;
            nn->parent = parent;
            parent->e[parent->n++] = ne;
            if (parent->n > 5) psplit = node_split(parent, 2);
        }
        n = parent; nn = psplit;
    }
    if (nn) {
        rnode *old = t->root;
        rnode *root = node_new(NULL, 0, old->level + 1);
        root->e[0].bb = node_bb(old); root->e[0].child = old; root->e[0].obj = -1;
        root->e[1].bb = node_bb(nn); root->e[1].child = nn; root->e[1].obj = -1;
        root->n = 2;
        old->parent = root; nn->parent = root;
        t->root = root; t->height++;
    }
    t->size++;
}
static void rtree_init(rtree *t) { t->root = node_new(NULL, 1, 1); t->size = 0; t->height = 1; }

/* box.go:21-26 NewBox + box.go:29-68 Box.Intersect */
static const vec3 BOX_NORMALS[6] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
static int corners_intersect(vec3 mn, vec3 mx, vec3 o, vec3 d) {
    for (int k = 0; k < 6; k++) {
        vec3 sn = BOX_NORMALS[k];
        if (v_dot(d, sn) != 0.0) {
            vec3 sp = v_dot(sn, v_make(1, 1, 1)) < 0 ? mn : mx;
            double ds = v_dot(v_sub(sp, o), sn) / v_dot(d, sn);
            if (ds >= 0.0) {
                vec3 ip = v_add(o, v_scale(d, ds));
                if (sn.x != 0.0) {
                    if ((mn.y <= ip.y && ip.y <= mx.y) && (mn.z <= ip.z && ip.z <= mx.z)) return 1;
                } else if (sn.y != 0.0) {
                    if ((mn.x <= ip.x && ip.x <= mx.x) && (mn.z <= ip.z && ip.z <= mx.z)) return 1;
                } else if (sn.z != 0.0) {
                    if ((mn.x <= ip.x && ip.x <= mx.x) && (mn.y <= ip.y && ip.y <= mx.y)) return 1;
                }
            }
        }
    }
    return 0;
}
static int box_intersect(const rect *bb, vec3 o, vec3 d) {
    vec3 mn = v_make(bb->p[0], bb->p[1], bb->p[2]);
    vec3 mx = v_make(bb->p[0] + (bb->q[0] - bb->p[0]), bb->p[1] + (bb->q[1] - bb->p[1]),
                     bb->p[2] + (bb->q[2] - bb->p[2]));
    return corners_intersect(mn, mx, o, d);
}

/* ------------------------------------------------------------------ context */
#define BOUND_EPSILON 0.0001 /* shared/state/util.go:7 */

typedef struct {
    const or_mesh *m;
    rtree faces;
    rect *fbox;           /* OR_CULL_BOXES: face.Bounds per face (mesh.go:30-50) */
} mesh_rt;
/* Culling modes (or_build):
 *   OR_CULL_BRUTE  every face and object, ascending index (no box test at all);
 *   OR_CULL_RTREE  the reference: rtreego SearchCondition over the face and object trees,
 *                  Box.Intersect on every inner-node and leaf-entry box (DFS order);
 *   OR_CULL_BOXES  every face and object in ascending index, each gated by Box.Intersect on
 *                  its OWN padded box only (face.Bounds / Object.Bounds) — the reference's
 *                  leaf-level test without rtreego's inner nodes, whose shape depends on the
 *                  unvendored tree's insertion order and split.  The GPU
 *                  computes exactly this set. */
enum { OR_CULL_BRUTE = 0, OR_CULL_RTREE = 1, OR_CULL_BOXES = 2 };
typedef struct {
    or_scene s;
    mesh_rt *meshes;
    rtree objs;           /* top-level object tree (EnvMutables.Objs) */
    rect *obox;           /* OR_CULL_BOXES: Object.Bounds per object (object.go:31-59) */
    int use_rtree;        /* the culling mode (OR_CULL_*) */
    vec3 cam_pos, cam_fwd, cam_left, cam_up;
    double fov;
    int cam_ok;
    int bounces;          /* configs[4] reflection extension: 0 = the reference */
} or_ctx;

/* camera.go:35-44 NewCamera (GlobalUp = (0,1,0), environment.go:22) */
int or_new_camera(const double pos[3], const double dir[3], double out_fwd[3], double out_left[3],
                  double out_up[3]) {
    vec3 d = v_make(dir[0], dir[1], dir[2]);
    vec3 up = v_make(0, 1, 0);
    if (v_zero(v_cross(d, up))) return -1;
    vec3 f = v_norm(d);
    vec3 l = v_norm(v_cross(d, up));
    vec3 u = v_cross(l, f);
    out_fwd[0] = f.x; out_fwd[1] = f.y; out_fwd[2] = f.z;
    out_left[0] = l.x; out_left[1] = l.y; out_left[2] = l.z;
    out_up[0] = u.x; out_up[1] = u.y; out_up[2] = u.z;
    (void)pos;
    return 0;
}

static vec3 mesh_vertex(const or_mesh *m, uint32_t i) {
    return v_make(m->vertices[3 * i], m->vertices[3 * i + 1], m->vertices[3 * i + 2]);
}
static vec3 mesh_normal(const or_mesh *m, uint32_t i) {
    return v_make(m->normals[3 * i], m->normals[3 * i + 1], m->normals[3 * i + 2]);
}

/* mesh.go:30-50 face.Bounds */
static rect face_bounds(const or_mesh *m, uint32_t f) {
    vec3 a = mesh_vertex(m, m->face_v[3 * f]), b = mesh_vertex(m, m->face_v[3 * f + 1]),
         c = mesh_vertex(m, m->face_v[3 * f + 2]);
    double p[3], len[3];
    double mn[3] = {go_min(a.x, go_min(b.x, c.x)), go_min(a.y, go_min(b.y, c.y)), go_min(a.z, go_min(b.z, c.z))};
    double mx[3] = {go_max(a.x, go_max(b.x, c.x)), go_max(a.y, go_max(b.y, c.y)), go_max(a.z, go_max(b.z, c.z))};
    for (int i = 0; i < 3; i++) { p[i] = mn[i]; len[i] = go_max(mx[i] - mn[i], BOUND_EPSILON); }
    return rect_new(p, len);
}
/* object.go:31-59 Object.Bounds */
static rect object_bounds(const or_ctx *c, uint32_t oi) {
    const or_object *o = &c->s.objects[oi];
    double mn[3] = {o->pos[0], o->pos[1], o->pos[2]}, mx[3] = {o->pos[0], o->pos[1], o->pos[2]};
    if (o->mesh < c->s.n_meshes) {
        const or_mesh *m = c->meshes[o->mesh].m;
        for (uint32_t v = 0; v < m->n_vertices; v++)
            for (int k = 0; k < 3; k++) {
                mn[k] = go_min(mn[k], o->pos[k] + m->vertices[3 * v + k]);
                mx[k] = go_max(mx[k], o->pos[k] + m->vertices[3 * v + k]);
            }
    }
    double len[3];
    for (int k = 0; k < 3; k++) len[k] = go_max(mx[k] - mn[k], BOUND_EPSILON);
    return rect_new(mn, len);
}

or_ctx *or_build(const or_scene *s, int use_rtree) {
    or_ctx *c = (or_ctx *)calloc(1, sizeof(or_ctx));
    c->s = *s;
    c->use_rtree = use_rtree;
    c->meshes = (mesh_rt *)calloc(s->n_meshes ? s->n_meshes : 1, sizeof(mesh_rt));
    for (uint32_t i = 0; i < s->n_meshes; i++) {
        c->meshes[i].m = &s->meshes[i];
        if (use_rtree == OR_CULL_RTREE) {
            rtree_init(&c->meshes[i].faces);
            for (uint32_t f = 0; f < s->meshes[i].n_faces; f++)
                rtree_insert(&c->meshes[i].faces, face_bounds(&s->meshes[i], f), (int32_t)f);
        }
        if (use_rtree != OR_CULL_BRUTE) {  /* BOXES, and the RTREE mode's veto audit */
            c->meshes[i].fbox = (rect *)malloc(sizeof(rect) * (s->meshes[i].n_faces + 1));
            for (uint32_t f = 0; f < s->meshes[i].n_faces; f++) c->meshes[i].fbox[f] = face_bounds(&s->meshes[i], f);
        }
    }
    if (use_rtree == OR_CULL_RTREE) {
        rtree_init(&c->objs);
        for (uint32_t o = 0; o < s->n_objects; o++) rtree_insert(&c->objs, object_bounds(c, o), (int32_t)o);
    }
    if (use_rtree != OR_CULL_BRUTE) {
        c->obox = (rect *)malloc(sizeof(rect) * (s->n_objects + 1));
        for (uint32_t o = 0; o < s->n_objects; o++) c->obox[o] = object_bounds(c, o);
    }
    c->cam_pos = v_make(s->cam_pos[0], s->cam_pos[1], s->cam_pos[2]);
    double f[3], l[3], u[3];
    c->cam_ok = or_new_camera(s->cam_pos, s->cam_dir, f, l, u) == 0;
    c->cam_fwd = v_make(f[0], f[1], f[2]);
    c->cam_left = v_make(l[0], l[1], l[2]);
    c->cam_up = v_make(u[0], u[1], u[2]);
    c->fov = s->fov;
    return c;
}
int or_camera_ok(const or_ctx *c) { return c->cam_ok; }
void or_free(or_ctx *c) {
    if (!c) return;
    if (c->use_rtree == OR_CULL_RTREE) {
        for (uint32_t i = 0; i < c->s.n_meshes; i++) node_free(c->meshes[i].faces.root);
        node_free(c->objs.root);
    }
    for (uint32_t i = 0; i < c->s.n_meshes; i++) free(c->meshes[i].fbox);
    free(c->obox);
    free(c->meshes);
    free(c);
}

/* ------------------------------------------------------- Möller–Trumbore */
/* triangle.go:37-77.  Returns 1 on hit with the intersection point and (r1,r2,r3). */
static int tri_intersection(vec3 p1, vec3 p2, vec3 p3, vec3 o, vec3 d, vec3 *hit, double bc[3]) {
    vec3 p1p2 = v_sub(p2, p1), p1p3 = v_sub(p3, p1), neg = v_scale(d, -1);
    double inc = v_dot(p1p2, v_cross(p1p3, neg));
    if (inc != 0.0) {
        vec3 p1or = v_sub(o, p1);
        double r2 = v_dot(p1or, v_cross(p1p3, neg)) / inc;
        if (0.0 <= r2 && r2 <= 1.0) {
            double r3 = v_dot(p1p2, v_cross(p1or, neg)) / inc;
            if (0.0 <= r2 + r3 && r2 + r3 <= 1.0) {
                double r1 = 1.0 - r2 - r3;
                if (r1 >= 0.0 && r2 >= 0.0 && r3 >= 0.0) {
                    double t = v_dot(p1p2, v_cross(p1p3, p1or)) / inc;
                    if (t >= 0.0) {
                        *hit = v_add(o, v_scale(d, t));
                        bc[0] = r1; bc[1] = r2; bc[2] = r3;
                        return 1;
                    }
                }
            }
        }
    }
    return 0;
}
/* Exported for known-answer tests. */
int or_triangle_intersection(const double p1[3], const double p2[3], const double p3[3], const double o[3],
                             const double d[3], double hit[3], double bc[3]) {
    vec3 h = {0, 0, 0};
    int r = tri_intersection(v_make(p1[0], p1[1], p1[2]), v_make(p2[0], p2[1], p2[2]), v_make(p3[0], p3[1], p3[2]),
                             v_make(o[0], o[1], o[2]), v_make(d[0], d[1], d[2]), &h, bc);
    hit[0] = h.x; hit[1] = h.y; hit[2] = h.z;
    return r;
}

typedef struct {
    int ok;
    vec3 hit, normal;
    uint32_t mat, face, obj;
} hitrec;

typedef struct {
    uint32_t *stack_face; /* scratch for R-tree candidates */
    uint64_t tri_tests, box_tests;
} scratch;

/* rtreego SearchCondition DFS (order = entry order in each node) */
typedef struct { vec3 o, d; uint32_t *out; uint32_t n; uint64_t *box_tests; } searchq;
static void rt_search(const rnode *n, searchq *q) {
    for (int i = 0; i < n->n; i++) {
        (*q->box_tests)++;
        if (!box_intersect(&n->e[i].bb, q->o, q->d)) continue;
        if (n->leaf) q->out[q->n++] = (uint32_t)n->e[i].obj;
        else rt_search(n->e[i].child, q);
    }
}

/* object.go:63-110 Object.Intersection */
static void object_intersection(const or_ctx *c, uint32_t oi, vec3 ro, vec3 rd, hitrec *out, scratch *sc) {
    const or_object *ob = &c->s.objects[oi];
    vec3 pos = v_make(ob->pos[0], ob->pos[1], ob->pos[2]);
    int has = 0; double best = 0;
    vec3 bip = {0, 0, 0}, bn = {0, 0, 0};
    uint32_t bmat = 0, bface = 0;
    ro = v_sub(ro, pos);
    if (ob->mesh < c->s.n_meshes) {
        const or_mesh *m = c->meshes[ob->mesh].m;
        uint32_t ncand;
        const uint32_t *cand = NULL;
        const rect *fbox = c->use_rtree == OR_CULL_BOXES ? c->meshes[ob->mesh].fbox : NULL;
        if (c->use_rtree == OR_CULL_RTREE) {
            searchq q = {ro, rd, sc->stack_face, 0, &sc->box_tests};
            rt_search(c->meshes[ob->mesh].faces.root, &q);
            ncand = q.n; cand = sc->stack_face;
        } else {
            ncand = m->n_faces;
        }
        int has_normals = m->n_normals > 0;
        for (uint32_t k = 0; k < ncand; k++) {
            uint32_t f = cand ? cand[k] : k;
            if (fbox) {  /* OR_CULL_BOXES: the face's own box (object.go:76, box.go:29-68) */
                sc->box_tests++;
                if (!box_intersect(&fbox[f], ro, rd)) continue;
            }
            vec3 p1 = mesh_vertex(m, m->face_v[3 * f]), p2 = mesh_vertex(m, m->face_v[3 * f + 1]),
                 p3 = mesh_vertex(m, m->face_v[3 * f + 2]);
            vec3 ip; double bc[3];
            sc->tri_tests++;
            if (tri_intersection(p1, p2, p3, ro, rd, &ip, bc)) {
                vec3 nrm;
                if (has_normals) {
                    vec3 n1 = mesh_normal(m, m->face_n[3 * f]), n2 = mesh_normal(m, m->face_n[3 * f + 1]),
                         n3 = mesh_normal(m, m->face_n[3 * f + 2]);
                    /* triangle.go:29-31 InterpNormal */
                    nrm = v_norm(v_add(v_add(v_scale(n1, bc[0]), v_scale(n2, bc[1])), v_scale(n3, bc[2])));
                } else {
                    /* triangle.go:24-26 Normal */
                    nrm = v_norm(v_cross(v_sub(p2, p1), v_sub(p3, p1)));
                }
                double dist = v_len(v_sub(ro, ip));
                if (!has || dist < best) {
                    has = 1; best = dist; bip = ip; bn = nrm; bmat = m->face_mat[f]; bface = f;
                }
            }
        }
    }
    out->ok = has;
    out->hit = v_add(bip, pos);
    out->normal = bn;
    out->mat = bmat;
    out->face = bface;
    out->obj = oi;
}

/* tracer.go:27-50 trace: nearest object by |hit - Cam.Pos| (also for shadow rays) */
static hitrec trace(const or_ctx *c, vec3 ro, vec3 rd, scratch *sc) {
    hitrec best; memset(&best, 0, sizeof(best));
    double bestd = 0;
    uint32_t cands[64];
    uint32_t *cl = NULL; uint32_t nc;
    if (c->use_rtree == OR_CULL_RTREE) {
        cl = c->s.n_objects <= 64 ? cands : (uint32_t *)malloc(sizeof(uint32_t) * c->s.n_objects);
        searchq q = {ro, rd, cl, 0, &sc->box_tests};
        rt_search(c->objs.root, &q);
        nc = q.n;
    } else {
        nc = c->s.n_objects;
    }
    for (uint32_t k = 0; k < nc; k++) {
        uint32_t oi = cl ? cl[k] : k;
        if (c->use_rtree == OR_CULL_BOXES) {  /* the object's own box (tracer.go:32) */
            sc->box_tests++;
            if (!box_intersect(&c->obox[oi], ro, rd)) continue;
        }
        hitrec h;
        object_intersection(c, oi, ro, rd, &h, sc);
        if (h.ok) {
            double d = v_len(v_sub(h.hit, c->cam_pos));
            if (!best.ok || d < bestd) { best = h; bestd = d; }
        }
    }
    if (cl && cl != cands) free(cl);
    return best;
}

/* colour.go:38-50 */
typedef struct { double r, g, b; } rgb;
static inline rgb c_add(rgb a, rgb b) { rgb o = {go_min(a.r + b.r, 1.0), go_min(a.g + b.g, 1.0), go_min(a.b + b.b, 1.0)}; return o; }
static inline rgb c_scale(rgb a, double s) {
    rgb o = {go_max(0.0, go_min(s * a.r, 1.0)), go_max(0.0, go_min(s * a.g, 1.0)), go_max(0.0, go_min(s * a.b, 1.0))};
    return o;
}
static inline rgb c_mul(rgb a, rgb b) { rgb o = {a.r * b.r, a.g * b.g, a.b * b.b}; return o; }

/* tracer.go:53-77 phong */
static rgb phong(const or_ctx *c, const hitrec *h, scratch *sc, uint64_t *shadow_rays) {
    const or_mesh *m = c->meshes[c->s.objects[h->obj].mesh].m;
    const double *mt = &m->materials[10 * h->mat];
    rgb ka = {mt[0], mt[1], mt[2]}, kd = {mt[3], mt[4], mt[5]}, ks = {mt[6], mt[7], mt[8]};
    double ns = mt[9];
    rgb col = ka;
    for (uint32_t li = 0; li < c->s.n_lights; li++) {
        const or_light *L = &c->s.lights[li];
        vec3 lpos = v_make(L->pos[0], L->pos[1], L->pos[2]);
        rgb lcol = {L->col[0], L->col[1], L->col[2]};
        vec3 ldir = v_norm(v_sub(lpos, h->hit));
        (*shadow_rays)++;
        hitrec sh = trace(c, v_add(h->hit, v_scale(ldir, 0.0001)), ldir, sc);
        if (!sh.ok || v_len(v_sub(lpos, h->hit)) < v_len(v_sub(sh.hit, h->hit))) {
            vec3 refl = v_sub(v_scale(h->normal, 2 * v_dot(ldir, h->normal)), ldir);
            vec3 camdir = v_norm(v_sub(c->cam_pos, h->hit));
            col = c_add(col, c_mul(c_scale(kd, go_max(v_dot(ldir, h->normal), 0.0)), lcol));
            col = c_add(col, c_mul(c_scale(ks, or_go_pow(go_max(v_dot(refl, camdir), 0.0), ns)), lcol));
        }
    }
    return col;
}

/* tracer.go:15-22 pixelToPoint (Go int division for half sizes) */
static vec3 pixel_to_point(const or_ctx *c, int i, int j, int width, int height) {
    int hw = width / 2, hh = height / 2;
    double phw = or_go_tan(c->fov / 2.0);
    double phh = phw * (double)height / (double)width;
    vec3 ioff = v_scale(c->cam_left, phw * ((double)(hw - i) - 0.5) / (double)hw);
    vec3 joff = v_scale(c->cam_up, phh * ((double)(hh - j) - 0.5) / (double)hh);
    return v_add(v_add(v_add(c->cam_pos, c->cam_fwd), ioff), joff);
}

/*
 * configs[4] reflection extension (NOT in the reference; BASELINE.json / SURVEY.md §8(d)
 * define it by the build):  at a hit reached along direction D,
 *   c = c_add(phong(hit), c_mul(Ks, c_reflected)),
 *   c_reflected = the same rule at the nearest hit of trace(hit + R 1e-4, R) (black on a
 *   miss), R = D - 2 (D.N) N computed as sub(D, scale(N, 2 dot(D, N))), not normalised;
 * recursion stops after `bounces` reflections (the deepest level is plain phong).  trace
 * and phong are the reference's (tracer.go:27-77), camera-distance object choice included.
 */
static rgb shade_reflect(const or_ctx *c, const hitrec *h, vec3 d_in, int depth, scratch *sc, uint64_t *shadow_rays,
                         uint64_t *refl_rays) {
    rgb ph = phong(c, h, sc, shadow_rays);
    if (depth >= c->bounces) return ph;
    vec3 R = v_sub(d_in, v_scale(h->normal, 2 * v_dot(d_in, h->normal)));
    (*refl_rays)++;
    hitrec h2 = trace(c, v_add(h->hit, v_scale(R, 0.0001)), R, sc);
    rgb cr = {0, 0, 0};
    if (h2.ok) cr = shade_reflect(c, &h2, R, depth + 1, sc, shadow_rays, refl_rays);
    const double *mt = &c->meshes[c->s.objects[h->obj].mesh].m->materials[10 * h->mat];
    rgb ks = {mt[6], mt[7], mt[8]};
    return c_add(ph, c_mul(ks, cr));
}

/* tracer.go:81-91 Trace */
typedef struct { int valid; rgb c; uint32_t face, obj; } pixel_out;
static pixel_out trace_pixel(const or_ctx *c, int i, int j, int W, int H, scratch *sc, uint64_t *shadow_rays,
                             uint64_t *refl_rays) {
    pixel_out p; memset(&p, 0, sizeof(p));
    vec3 sp = pixel_to_point(c, i, j, W, H);
    vec3 d = v_norm(v_sub(sp, c->cam_pos));
    hitrec h = trace(c, c->cam_pos, d, sc);
    if (h.ok) {
        p.valid = 1;
        p.c = c->bounces > 0 ? shade_reflect(c, &h, d, 0, sc, shadow_rays, refl_rays) : phong(c, &h, sc, shadow_rays);
        p.face = h.face;
        p.obj = h.obj;
    }
    return p;
}

void or_set_bounces(or_ctx *c, int bounces) { c->bounces = bounces < 0 ? 0 : bounces; }

/* --------------------------------------------------------- tile driver */
typedef struct {
    const or_ctx *c;
    const or_tile *tiles; uint32_t ntiles;
    const uint64_t *tile_off;
    uint32_t W, H;
    int tid, nthreads, shade;
    uint8_t *valid; double *rgb; uint8_t *rgb8; int32_t *face; int32_t *obj;
    uint64_t primary, shadow, hits, tri, box, refl;
    uint32_t max_faces;
} job;

static void *run_job(void *arg) {
    job *jb = (job *)arg;
    scratch sc; sc.tri_tests = 0; sc.box_tests = 0;
    sc.stack_face = (uint32_t *)malloc(sizeof(uint32_t) * (jb->max_faces + 1));
    uint64_t shadow = 0, refl = 0;
    for (uint32_t t = 0; t < jb->ntiles; t++) {
        const or_tile *tl = &jb->tiles[t];
        /* worker/distributed/main.go:67-89: i over width (outer), j over height (inner) */
        for (uint32_t i = (uint32_t)jb->tid; i < tl->w; i += (uint32_t)jb->nthreads) {
            for (uint32_t j = 0; j < tl->h; j++) {
                uint64_t idx = jb->tile_off[t] + (uint64_t)i * tl->h + j;
                pixel_out p;
                jb->primary++;
                if (jb->shade) {
                    p = trace_pixel(jb->c, (int)(tl->x + i), (int)(tl->y + j), (int)jb->W, (int)jb->H, &sc, &shadow,
                                    &refl);
                } else {
                    memset(&p, 0, sizeof(p));
                    vec3 sp = pixel_to_point(jb->c, (int)(tl->x + i), (int)(tl->y + j), (int)jb->W, (int)jb->H);
                    hitrec h = trace(jb->c, jb->c->cam_pos, v_norm(v_sub(sp, jb->c->cam_pos)), &sc);
                    p.valid = h.ok; p.face = h.face; p.obj = h.obj;
                }
                if (p.valid) jb->hits++;
                if (jb->valid) jb->valid[idx] = (uint8_t)p.valid;
                if (jb->rgb) {
                    jb->rgb[3 * idx] = p.c.r; jb->rgb[3 * idx + 1] = p.c.g; jb->rgb[3 * idx + 2] = p.c.b;
                }
                if (jb->rgb8) {
                    /* colour.go:59-61 RGB(): uint8(255 * c), truncating */
                    jb->rgb8[3 * idx] = (uint8_t)(255 * p.c.r);
                    jb->rgb8[3 * idx + 1] = (uint8_t)(255 * p.c.g);
                    jb->rgb8[3 * idx + 2] = (uint8_t)(255 * p.c.b);
                }
                if (jb->face) jb->face[idx] = p.valid ? (int32_t)p.face : -1;
                if (jb->obj) jb->obj[idx] = p.valid ? (int32_t)p.obj : -1;
            }
        }
    }
    jb->shadow = shadow;
    jb->refl = refl;
    jb->tri = sc.tri_tests;
    jb->box = sc.box_tests;
    free(sc.stack_face);
    return NULL;
}

/*
 * Trace a list of tiles.  Output for tile t starts at sum_{u<t} w_u*h_u pixels and is
 * column-major inside the tile (results[i*h + j], worker/distributed/main.go:82).  A
 * single tile (0,0,W,H) is the worker/sequential framebuffer in (i, j) order.
 * shade=0 traces primary rays only (configs[0]: "primary-rays-only").
 */
int or_trace_tiles(const or_ctx *c, uint32_t W, uint32_t H, const or_tile *tiles, uint32_t ntiles, int nthreads,
                   int shade, uint8_t *valid, double *rgb, uint8_t *rgb8, int32_t *face, int32_t *obj,
                   or_stats *st) {
    if (!c->cam_ok) return -1;
    if (nthreads < 1) nthreads = 1;
    uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (ntiles + 1));
    off[0] = 0;
    for (uint32_t t = 0; t < ntiles; t++) off[t + 1] = off[t] + (uint64_t)tiles[t].w * tiles[t].h;
    uint32_t maxf = 0;
    for (uint32_t i = 0; i < c->s.n_meshes; i++) if (c->s.meshes[i].n_faces > maxf) maxf = c->s.meshes[i].n_faces;
    job *jobs = (job *)calloc((size_t)nthreads, sizeof(job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        job *jb = &jobs[t];
        jb->c = c; jb->tiles = tiles; jb->ntiles = ntiles; jb->tile_off = off; jb->W = W; jb->H = H;
        jb->tid = t; jb->nthreads = nthreads; jb->shade = shade;
        jb->valid = valid; jb->rgb = rgb; jb->rgb8 = rgb8; jb->face = face; jb->obj = obj;
        jb->max_faces = maxf;
    }
    if (nthreads == 1) run_job(&jobs[0]);
    else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run_job, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    if (st) {
        memset(st, 0, sizeof(*st));
        for (int t = 0; t < nthreads; t++) {
            st->primary_rays += jobs[t].primary; st->shadow_rays += jobs[t].shadow; st->hits += jobs[t].hits;
            st->reflection_rays += jobs[t].refl;
            st->tri_tests += jobs[t].tri; st->box_tests += jobs[t].box;
        }
    }
    free(jobs); free(th); free(off);
    return 0;
}

/* tracer.go:27-50 trace() on arbitrary rays (for known-answer tests of the nearest-hit rule). */
int or_trace_rays(const or_ctx *c, uint32_t n, const double *orig, const double *dir, uint8_t *ok, double *hit,
                  double *normal, int32_t *face, int32_t *obj) {
    uint32_t maxf = 0;
    for (uint32_t i = 0; i < c->s.n_meshes; i++) if (c->s.meshes[i].n_faces > maxf) maxf = c->s.meshes[i].n_faces;
    scratch sc; sc.tri_tests = 0; sc.box_tests = 0;
    sc.stack_face = (uint32_t *)malloc(sizeof(uint32_t) * (maxf + 1));
    for (uint32_t r = 0; r < n; r++) {
        hitrec h = trace(c, v_make(orig[3 * r], orig[3 * r + 1], orig[3 * r + 2]),
                         v_make(dir[3 * r], dir[3 * r + 1], dir[3 * r + 2]), &sc);
        ok[r] = (uint8_t)h.ok;
        hit[3 * r] = h.hit.x; hit[3 * r + 1] = h.hit.y; hit[3 * r + 2] = h.hit.z;
        normal[3 * r] = h.normal.x; normal[3 * r + 1] = h.normal.y; normal[3 * r + 2] = h.normal.z;
        face[r] = h.ok ? (int32_t)h.face : -1;
        obj[r] = h.ok ? (int32_t)h.obj : -1;
    }
    free(sc.stack_face);
    return 0;
}

/*
 * Audit of the R-tree mode against OR_CULL_BOXES, per ray (OR_CULL_RTREE contexts only):
 *   veto[r]  candidates the rtreego tree prunes although their OWN box passes Box.Intersect
 *            and they would count: faces Möller–Trumbore accepts whose leaf entry passes but
 *            an ancestor inner-node box fails, plus objects whose own box passes, with such
 *            a face, pruned by the object tree;
 *   ties[r]  objects on the ray where two distinct accepted faces share the minimum
 *            distance (the R-tree's DFS order and the ascending index may pick different
 *            winners: object.go:97's strict `<` keeps the first visited).
 * The two culling modes can only differ on a ray where one of the two is non-zero.
 */
static int face_accepts(const or_mesh *m, uint32_t f, vec3 ro, vec3 rd, double *dist) {
    vec3 p1 = mesh_vertex(m, m->face_v[3 * f]), p2 = mesh_vertex(m, m->face_v[3 * f + 1]),
         p3 = mesh_vertex(m, m->face_v[3 * f + 2]);
    vec3 ip; double bc[3];
    if (!tri_intersection(p1, p2, p3, ro, rd, &ip, bc)) return 0;
    *dist = v_len(v_sub(ro, ip));
    return 1;
}
int or_rtree_audit(const or_ctx *c, uint32_t n, const double *orig, const double *dir, uint32_t *veto,
                   uint32_t *ties) {
    if (c->use_rtree != OR_CULL_RTREE) return -1;
    uint32_t maxf = 0;
    for (uint32_t i = 0; i < c->s.n_meshes; i++) if (c->s.meshes[i].n_faces > maxf) maxf = c->s.meshes[i].n_faces;
    uint32_t *cand = (uint32_t *)malloc(sizeof(uint32_t) * (maxf + 1));
    uint8_t *mark = (uint8_t *)malloc(maxf + 1);
    uint32_t *ocand = (uint32_t *)malloc(sizeof(uint32_t) * (c->s.n_objects + 1));
    uint8_t *omark = (uint8_t *)malloc(c->s.n_objects + 1);
    uint64_t bt = 0;
    for (uint32_t r = 0; r < n; r++) {
        vec3 o = v_make(orig[3 * r], orig[3 * r + 1], orig[3 * r + 2]);
        vec3 d = v_make(dir[3 * r], dir[3 * r + 1], dir[3 * r + 2]);
        uint32_t nv = 0, nt = 0;
        searchq oq = {o, d, ocand, 0, &bt};
        rt_search(c->objs.root, &oq);
        memset(omark, 0, c->s.n_objects + 1);
        for (uint32_t k = 0; k < oq.n; k++) omark[ocand[k]] = 1;
        for (uint32_t oi = 0; oi < c->s.n_objects; oi++) {
            const or_object *ob = &c->s.objects[oi];
            if (ob->mesh >= c->s.n_meshes) continue;
            const or_mesh *m = c->meshes[ob->mesh].m;
            vec3 ro = v_sub(o, v_make(ob->pos[0], ob->pos[1], ob->pos[2]));
            const rect *fbox = c->meshes[ob->mesh].fbox;
            /* both modes skip an object whose own box fails (its leaf entry is that box) */
            if (!box_intersect(&c->obox[oi], o, d)) continue;
            const int pruned = !omark[oi];
            searchq fq = {ro, d, cand, 0, &bt};
            rt_search(c->meshes[ob->mesh].faces.root, &fq);
            memset(mark, 0, m->n_faces + 1);
            for (uint32_t k = 0; k < fq.n; k++) mark[cand[k]] = 1;
            int has = 0, tie = 0; double best = 0;
            for (uint32_t f = 0; f < m->n_faces; f++) {
                double dist;
                if (!box_intersect(&fbox[f], ro, d) || !face_accepts(m, f, ro, d, &dist)) continue;
                if (!mark[f] || pruned) nv++;  /* pruned above its own box */
                if (!mark[f] || pruned) continue;
                if (!has || dist < best) { has = 1; best = dist; tie = 0; }
                else if (dist == best) tie = 1;
            }
            nt += (uint32_t)tie;
        }
        veto[r] = nv;
        ties[r] = nt;
    }
    free(cand); free(mark); free(ocand); free(omark);
    return 0;
}

/* The corners box_intersect uses (box.go:21-26 NewBox on the rtreego rect): {MinCorner,
 * MaxCorner} of face.Bounds (mesh.go:30-50) and Object.Bounds (object.go:31-59). */
static void rect_out(const rect *bb, double out[6]) {
    for (int k = 0; k < 3; k++) { out[k] = bb->p[k]; out[3 + k] = bb->p[k] + (bb->q[k] - bb->p[k]); }
}
int or_face_box(const or_ctx *c, uint32_t mesh, uint32_t f, double out[6]) {
    if (mesh >= c->s.n_meshes || f >= c->s.meshes[mesh].n_faces) return -1;
    rect r = face_bounds(&c->s.meshes[mesh], f);
    rect_out(&r, out);
    return 0;
}
int or_object_box(const or_ctx *c, uint32_t oi, double out[6]) {
    if (oi >= c->s.n_objects) return -1;
    rect r = object_bounds(c, oi);
    rect_out(&r, out);
    return 0;
}
/* box.go:29-68 on n rays against one box given as NewBox corners (known-answer tests). */
int or_box_intersect(const double box[6], uint32_t n, const double *orig, const double *dir, uint8_t *out) {
    vec3 mn = v_make(box[0], box[1], box[2]), mx = v_make(box[3], box[4], box[5]);
    for (uint32_t i = 0; i < n; i++)
        out[i] = (uint8_t)corners_intersect(mn, mx, v_make(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]),
                                            v_make(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]));
    return 0;
}
