// kernels.hip — CDNA4 (gfx950) kernels of the trace worker.
//
// Replaces, per pixel of a tile, worker/shared/tracer/tracer.go:81-91 Trace:
//   k_primary   pixelToPoint + primary dir (tracer.go:15-22, 83-86), nearest hit over
//               every object (tracer.go:27-50, object.go:63-110, triangle.go:37-77),
//               miss outputs, wave-aggregated compaction of the hits.
//   k_secondary shadow rays of phong (tracer.go:60-64): one lane per (hit, light); or
//               arbitrary rays for mirt_trace_rays (tracer.go:27-50).
//   k_shade     Phong (tracer.go:53-77) with colour.go:38-50 clamping and the
//               uint8(255*c) packing of worker/distributed/main.go:79-86.
//   k_unpack    framebuffer assembly after the multi-GPU gather.
//
// Mapping: one lane = one ray; a wave traces an 8x8 pixel block (coherent rays).
// Triangles are read wave-uniformly (LDS broadcast when the mesh is LDS-resident).
// Two sweep modes per object:
//   kModeBrute  every triangle, in LDS batches (the north star's brute force);
//   kModeBvh    (default) the whole wave walks the mesh's BVH together (packet
//               traversal, stackless skip pointers, wave-uniform node loads); a node is
//               entered when ANY lane's ray hits its inflated box.  Culling never
//               changes a result: boxes are inflated far beyond the fp64 rounding of
//               both tests, and the nearest rule is order-free (below).
//
// Numerics: fp64, -ffp-contract=off, the reference's operation order, true IEEE
// division, correctly rounded sqrt.  Hit/miss, the winning face and the colour are
// bit-identical to the CPU restatement (oracle/rt_oracle.c).
#include "gomath.hpp"
#include "mirt_internal.hpp"
#include "diag.hpp"
#include "lighttab.hpp"

namespace mirt {

// Wave-uniform reads of immutable device data (BVH nodes, triangles streamed from HBM)
// go through the constant address space so hipcc emits scalar s_load into SGPRs.
typedef const __attribute__((address_space(4))) double* cdptr;
typedef const __attribute__((address_space(4))) Bvh8Dev* cnptr;
typedef unsigned int u32x16 __attribute__((ext_vector_type(16)));
typedef const __attribute__((address_space(4))) u32x16* cv16ptr;
typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(4))) u32x8* cv8ptr;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) u32x4* cv4ptr;

__device__ __forceinline__ V3 vload(const double* p) { return V3{p[0], p[1], p[2]}; }
__device__ __forceinline__ void vstore(double* p, V3 v) {
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}

// Sound pre-reject for the first barycentric test of triangle.go:50-53:
//   r2 = fl(n / d);  test 0 <= r2 <= 1   (d finite, non-zero).
// Returns true only when that test certainly FAILS, without dividing:
//  * n * copysign(2^1000, d) < -|d|  <=>  n, d of opposite signs and |n| 2^1000 > |d|,
//    i.e. q < -2^-1000: fl(q) is negative and not -0.  The product is exact, or
//    overflows to -inf, which only happens when |q| > 2^-1000 as well.
//  * |n| > fl(|d| (1 + 2^-50)): |q| > 1 + 2^-51, so fl(q) is outside [-1, 1] — out
//    whatever the sign.  For a subnormal |d| the product may round to |d|, and then
//    |n| > |d| already means |q| >= 1 + 2^-52; overflow to +inf never rejects.
__device__ __forceinline__ bool r2_certainly_out(double n, double d) {
    const double k = __builtin_copysign(0x1p1000, d);
    return (n * k < -__builtin_fabs(d)) | (__builtin_fabs(n) > __builtin_fabs(d) * (1.0 + 0x1p-50));
}

// MIRT_DIAG (diagnostic builds only): wave-level event counts (how many waves reach each
// stage of the triangle test, per query kind), read with mirt_debug_counters.  Counted by
// the wave's first active lane into 8 shards.
constexpr int kDiagN = 32;
__device__ unsigned long long g_diag[8 * kDiagN];
__device__ __forceinline__ void diag(int k) {
    if (MIRT_DIAG) {
        const uint64_t ex = __builtin_amdgcn_read_exec();
        if ((threadIdx.x & 63) == (uint32_t)__builtin_ctzll(ex))
            atomicAdd(&g_diag[(blockIdx.x & 7) * kDiagN + k], 1ull);
    }
}

// Sound pre-reject for t >= 0 (triangle.go:67-71): true only when fl(n / d) is certainly
// negative (q < -2^-1000, the first half of r2_certainly_out's argument), i.e. t < 0.
__device__ __forceinline__ bool t_certainly_negative(double n, double d) {
    return n * __builtin_copysign(0x1p1000, d) < -__builtin_fabs(d);
}

// Möller–Trumbore exactly as triangle.go:37-77, on (p1or = O - P1, E1, E2), returning
// only the hit decision and the ray parameter.  neg = D * -1 (triangle.go:38).
//   DG: diagnostic counter base (MIRT_DIAG builds).
//   TPRE (shadow segments, whose rays leave the surface: the triangles they start on and
//   those behind them have t < 0): t's numerator is computed up front and a certainly
//   negative t rejects before any divide.  The conditions are a conjunction of pure tests,
//   so their order changes no result.
template <bool PREFILTER, int DG = 0, bool TPRE = false>
__device__ __forceinline__ bool mt_test(V3 p1or, V3 e1, V3 e2, V3 neg, double& t_out) {
    diag(DG + 0);
    V3 c = cross(e2, neg);
    double inc = dot(e1, c);
    if (inc != 0.0) {
        double nt = 0.0;
        double n2 = dot(p1or, c);
        if (PREFILTER && r2_certainly_out(n2, inc)) return false;
        if (PREFILTER && TPRE) {
            diag(DG + 7);
            nt = dot(e1, cross(e2, p1or));
            if (t_certainly_negative(nt, inc)) return false;
        }
        diag(DG + 1);
        if (PREFILTER) {
            // Divide-free classification of the barycentric conditions:
            // with q2 = n2/inc, q3 = n3/inc exact, q2, q3 >= 2^-40 and q2 + q3 <= 1 - 2^-40
            // make every rounded condition hold; q3 < -2^-40 or q2 + q3 > 1 + 2^-40 (q2 is
            // within [-2^-1000, 1 + 2^-51] past the pre-reject) make one fail.  Only lanes in
            // neither case take the divides.  |inc| >= 2^-900 keeps 2^-40 |inc| exact; an
            // infinite n3 or sum decides correctly, an overflowing bound only stays undecided,
            // and NaN lands in neither case.
            const double n3 = dot(e1, cross(p1or, neg));
            const double ai = __builtin_fabs(inc);
            const double p2 = inc < 0.0 ? -n2 : n2, p3 = inc < 0.0 ? -n3 : n3;
            const double m = 0x1p-40 * ai, sum = p2 + p3;
            const bool sane = ai >= 0x1p-900;
            const bool in = sane && p2 >= m && p3 >= m && sum <= ai - 0x1p-39 * ai;
            const bool out = sane && (p3 < -m || sum > ai + 0x1p-39 * ai);
            if (out) return false;
            if (!in) {  // tracer.go / triangle.go:50-66 as written
                diag(DG + 2);
                const double r2 = n2 / inc;
                if (!(0.0 <= r2 && r2 <= 1.0)) return false;
                const double r3 = n3 / inc;
                if (!(0.0 <= r2 + r3 && r2 + r3 <= 1.0)) return false;
                const double r1 = 1.0 - r2 - r3;
                if (!(r1 >= 0.0 && r2 >= 0.0 && r3 >= 0.0)) return false;
            }
            diag(DG + 3);
            const double t = (TPRE ? nt : dot(e1, cross(e2, p1or))) / inc;
            if (t >= 0.0) {
                diag(DG + 4);
                t_out = t;
                return true;
            }
            return false;
        }
        double r2 = n2 / inc;
        if (0.0 <= r2 && r2 <= 1.0) {
            diag(DG + 2);
            double r3 = dot(e1, cross(p1or, neg)) / inc;
            if (0.0 <= r2 + r3 && r2 + r3 <= 1.0) {
                double r1 = 1.0 - r2 - r3;
                if (r1 >= 0.0 && r2 >= 0.0 && r3 >= 0.0) {
                    diag(DG + 3);
                    double t = dot(e1, cross(e2, p1or)) / inc;
                    if (t >= 0.0) {
                        diag(DG + 4);
                        t_out = t;
                        return true;
                    }
                }
            }
        }
    }
    return false;
}

// Full triangle.go:37-77 for the winner (barycentrics needed for InterpNormal).
__device__ __forceinline__ bool mt_full(V3 p1or, V3 e1, V3 e2, V3 neg, double& t, double& r1, double& r2,
                                        double& r3) {
    V3 c = cross(e2, neg);
    double inc = dot(e1, c);
    if (inc != 0.0) {
        r2 = dot(p1or, c) / inc;
        if (0.0 <= r2 && r2 <= 1.0) {
            r3 = dot(e1, cross(p1or, neg)) / inc;
            if (0.0 <= r2 + r3 && r2 + r3 <= 1.0) {
                r1 = 1.0 - r2 - r3;
                if (r1 >= 0.0 && r2 >= 0.0 && r3 >= 0.0) {
                    t = dot(e1, cross(e2, p1or)) / inc;
                    if (t >= 0.0) return true;
                }
            }
        }
    }
    return false;
}

// Stage triangles [base, base+n) into LDS.  REL: store p1or = ro - P1 instead of P1
// (primary rays share one origin per object, so object.go:71 + triangle.go:48's
// subtraction is done once per triangle instead of once per ray; same fp64 value).
template <bool REL>
__device__ __forceinline__ void stage_tris(double* __restrict__ s, const double* __restrict__ g, uint32_t base,
                                           uint32_t n, V3 ro) {
    for (uint32_t k = threadIdx.x; k < n; k += kWG) {
        const double* t = g + (size_t)(base + k) * kTriD;
        double* d = s + (size_t)k * kTriD;
        if (REL) {
            d[0] = ro.x - t[0];
            d[1] = ro.y - t[1];
            d[2] = ro.z - t[2];
        } else {
            d[0] = t[0];
            d[1] = t[1];
            d[2] = t[2];
        }
#pragma unroll
        for (int q = 3; q < kTriD; ++q) d[q] = t[q];
    }
}

// Nearest-hit state of one object sweep.  object.go:97-103 keeps the first candidate
// (in its iteration order) reaching the minimum distance, with strict `<`.  With faces
// visited in ascending index order that is: the lowest face index among the hits at
// the minimum distance — except that a NaN distance on the lowest-indexed hit wins (no
// later `<` beats NaN) and a NaN anywhere else never wins.  `consider` computes exactly
// that in ANY visiting order, so culling/reordering cannot change the result.
// (no bools: a bool that lives across the test's divergent stages is a lane mask the compiler
// merges with three scalar instructions at every join, a word in a VGPR is merged by the exec
// mask for free; the flags are a sentinel and bits of words the state holds anyway)
struct Best {
    double d;           // the minimum non-NaN distance (if has())
    uint32_t face;      // lowest original face index at that distance; ~0u: no non-NaN hit yet
    uint32_t pos;       // its position in the BVH-ordered arrays
    uint32_t first;     // lowest original face index of any hit (0xffffffff: none)
    // that hit's position; bit 30: its distance is NaN; bit 31: some hit's distance is NaN (the
    // box gate: the winner alone does not decide).  Positions are < 2^24, and the flags packed
    // here keep two VGPRs fewer live through the sweep.
    uint32_t first_pos;
    __device__ __forceinline__ bool has() const { return face != 0xffffffffu; }
    __device__ __forceinline__ uint32_t first_nan() const { return (first_pos >> 30) & 1u; }
    __device__ __forceinline__ uint32_t any_nan() const { return MIRT_BOX_GATE == 4 ? 0u : first_pos >> 31; }
};
__device__ __forceinline__ void best_init(Best& b) {
    b.d = 0;
    b.face = 0xffffffffu;
    b.pos = 0;
    b.first = 0xffffffffu;
    b.first_pos = 0;
}
__device__ __forceinline__ void consider(Best& b, double dist, uint32_t face, uint32_t pos) {
    const bool isnan_d = dist != dist;
    if (face < b.first) {
        b.first = face;
        b.first_pos = pos | (isnan_d ? 0x40000000u : 0u) | (b.first_pos & 0x80000000u);
    }
    if (MIRT_BOX_GATE != 4) b.first_pos |= isnan_d ? 0x80000000u : 0u;  // (4: measurement build without it)
    if (!isnan_d && (!b.has() || dist < b.d || (dist == b.d && face < b.face))) {
        b.d = dist;
        b.face = face;
        b.pos = pos;
    }
}
__device__ __forceinline__ bool best_result(const Best& b, uint32_t& face, uint32_t& pos) {
    if (b.first == 0xffffffffu) return false;
    if (b.first_nan() || !b.has()) {
        face = b.first;
        pos = b.first_pos & 0x3fffffffu;
    } else {
        face = b.face;
        pos = b.pos;
    }
    return true;
}

// ---------------------------------------------------------------- the reference's box test
// shared/geom/box.go:29-68 Box.Intersect of the ray (o, d) with a box given as NewBox's
// corners bx = {MinCorner[3], MaxCorner[3]} (finite: the host builds them, mirt.cpp
// face_box / object_box).  The reference ORs six planes; for the plane of normal +-e_A with
// d_A != 0 it computes dirScale = (corner - o).n / d.n and checks the other two coordinates
// of o + dirScale d against the rectangle.  With finite corners that is exactly
//   ds = (corner_A - o_A) / d_A >= 0  and  lo_B <= o_B + ds d_B <= hi_B  (B != A):
// x * 1 = x, (-a) / (-b) = a / b, and a zero-weighted term of the dot products is +-0 unless
// a coordinate of o is not finite, where it is NaN and fails the plane — as the non-finite
// coordinate of o + ds d fails the rectangle here.  (d.n != 0 is d_A != 0 for finite d; a NaN
// d fails every plane both ways.)  The planes are pure tests, so any order gives the
// reference's boolean.
__device__ __forceinline__ double v3c(V3 v, int a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; }
// A box's corners in registers (loaded once per test: the object's from the kernel arguments,
// a face's from the mesh; a pointer that could be either would take the kernel argument's
// address, which copies the arguments to scratch).  Indexed with constants only (a run-time
// index would move the array to LDS or scratch).
struct Box6 {
    double v[kBoxD];
};
__device__ __forceinline__ Box6 box_load(const double* p) {
    Box6 b;
#pragma unroll
    for (int k = 0; k < kBoxD; ++k) b.v[k] = p[k];
    return b;
}
// plane `HI` (MaxCorner, normal +e_A) or not (MinCorner, -e_A) of axis A (box.go:33-60)
template <int A>
__device__ __forceinline__ bool box_plane(const Box6& bx, V3 o, V3 d, bool hi) {
    constexpr int B = A == 0 ? 1 : 0, C = A == 2 ? 1 : 2;
    const double da = v3c(d, A);
    const double ds = ((hi ? bx.v[3 + A] : bx.v[A]) - v3c(o, A)) / da;  // box.go:42
    const double ib = v3c(o, B) + ds * v3c(d, B), ic = v3c(o, C) + ds * v3c(d, C);  // box.go:47
    return da != 0.0 && ds >= 0.0 && bx.v[B] <= ib && ib <= bx.v[3 + B] && bx.v[C] <= ic && ic <= bx.v[3 + C];
}
// The far (FAR) or near plane of axis A: +e_A for d_A > 0 is the far one, -e_A for d_A < 0.
template <int A, bool FAR>
__device__ __forceinline__ bool box_side(const Box6& bx, V3 o, V3 d) {
    return box_plane<A>(bx, o, d, (v3c(d, A) > 0.0) == FAR);
}
// A pointer the compiler cannot prove loop-invariant: loads through it stay at their use
// instead of being hoisted to the kernel's start and held in SGPRs across the work loop.
template <typename T>
__device__ __forceinline__ const T* at_use(const T* p) {
    asm volatile("" : "+s"(p));
    return p;
}
// Box.Intersect for the lanes `on` (false on the others).  A ray that meets a box leaves it
// through the far plane of some axis (+e_a for d_a > 0, -e_a for d_a < 0).  The wave first
// tries the far plane of the axis its first lane's direction leans on most (a wave-uniform
// axis: one branch to straight-line code), then the other two far planes, each only while a
// lane is unproven, and last the three near planes (a ray through an edge, or one that misses
// the box: the rare path).  Same boolean as the reference's: every plane is tried for every
// lane the earlier planes did not prove.  (Trying the near and far planes in a fixed order
// after the lean axis cost 3-10 far-plane evaluations per wave on the driver's frame, this
// order 1.3-3: tests/gate_order_model.py.)
__device__ __forceinline__ bool box_gate(const Box6& bx, V3 o, V3 d, bool on) {
    if (MIRT_BOX_GATE == 3) return on;  // measurement build: every box passes (the structure kept)
    if (__ballot(on) == 0) return false;
    const double ax = __builtin_fabs(d.x), ay = __builtin_fabs(d.y), az = __builtin_fabs(d.z);
    const int lean = (ax >= ay && ax >= az) ? 0 : ay >= az ? 1 : 2;
    const int a = __builtin_amdgcn_readfirstlane(lean);
    bool r = false;
    diag(24);  // gates evaluated (wave-level)
    if (on) r = a == 0 ? box_side<0, true>(bx, o, d) : a == 1 ? box_side<1, true>(bx, o, d) : box_side<2, true>(bx, o, d);
    // the other far planes (A is a constant once unrolled; A == a was tried)
#pragma unroll
    for (int A = 0; A < 3; ++A) {
        if (A == a || __ballot(on && !r) == 0) continue;
        diag(25);  // further far planes evaluated
        if (on && !r) r = A == 0 ? box_side<0, true>(bx, o, d) : A == 1 ? box_side<1, true>(bx, o, d) : box_side<2, true>(bx, o, d);
    }
#pragma unroll
    for (int A = 0; A < 3; ++A) {
        if (__ballot(on && !r) == 0) break;
        diag(26);  // near planes evaluated
        if (on && !r) r = A == 0 ? box_side<0, false>(bx, o, d) : A == 1 ? box_side<1, false>(bx, o, d) : box_side<2, false>(bx, o, d);
    }
    if (__ballot(on && !r) != 0) diag(27);  // waves with a lane whose box fails
    return r;
}
// The same boolean in a fixed order (the second pass's per-candidate test, inside the sweep):
// the three far planes, then the three near ones, each while a lane is unproven.
__device__ __forceinline__ bool box_gate_small(const Box6& bx, V3 o, V3 d, bool on) {
    bool r = false;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        if (__ballot(on && !r) == 0) break;
        if (on && !r)
            r = q == 0 ? box_side<0, true>(bx, o, d) : q == 1 ? box_side<1, true>(bx, o, d) : q == 2 ? box_side<2, true>(bx, o, d)
              : q == 3 ? box_side<0, false>(bx, o, d) : q == 4 ? box_side<1, false>(bx, o, d) : box_side<2, false>(bx, o, d);
    }
    return r;
}

// Shadow segments' fp32 pre-classification against a light table.  A
// shadow ray runs along the line through its light L: o = L - lam d + eps, |eps| tiny.
// For the triangle (P1, P1 + E1, P1 + E2) and V_i = P_i - L, the reference's barycentric
// quotients are r_k = m_k / a with m_k = d . W_k (W_1 = V_2 x V_3, W_2 = V_3 x V_1,
// W_3 = V_1 x V_2) and a = d . A, A = E1 x E2 (so inc = -a), and its t numerator is
// nt = A . (o - P1) = ntL - lam a with ntL = A . (L - P1).  The light table holds W_1..3,
// A, ntL and error bounds per (light, triangle) in fp32, computed on the host (mirt.cpp
// light_records); the kernel forms m_k, a and nt with a few fp32 FMAs and rejects a lane
// only when the bounds prove that the fp64 test of triangle.go:37-77 fails:
//   |a| > Ea and some m_k certainly of the other sign (a barycentric < 0), or nt certainly
//   of a's sign (t < 0);   E = |d|_inf cw, Ea = |d|_inf cA, Et = 2 |lam| |d|_inf cA + ctL
//   (nt's error from lam a is at most 7 ulp of |lam| |d|_inf |A|_1; cA holds 10).
// A wave whose lanes are all rejected skips the triangle; the others run the fp64 test
// unchanged on the lanes not rejected, so the results are the same bits.
struct SegPre {
    float dx, dy, dz;  // d in fp32
    float ninf;        // |d|_inf
    float lam, lamn;   // lam = |L - hit| - 1e-4, 2 |lam| |d|_inf
};
__device__ __forceinline__ SegPre seg_pre(V3 d, double lh) {
    SegPre p;
    p.dx = (float)d.x;
    p.dy = (float)d.y;
    p.dz = (float)d.z;
    p.ninf = fmaxf(fmaxf(fabsf(p.dx), fabsf(p.dy)), fabsf(p.dz));
    p.lam = (float)(lh - 1e-4);
    p.lamn = 2.0f * fabsf(p.lam) * p.ninf;
    return p;
}
__device__ __forceinline__ float dot32(const float* w, const SegPre& p) {
    return __builtin_fmaf(w[2], p.dz, __builtin_fmaf(w[1], p.dy, w[0] * p.dx));
}
// true: the fp64 test of this lane certainly fails (see SegPre).  w: the record in SGPRs.
__device__ __forceinline__ bool seg_reject(const SegPre& p, const float* w) {
    const float m1 = dot32(w, p), m2 = dot32(w + 3, p), m3 = dot32(w + 6, p), a = dot32(w + 9, p);
    const float E = p.ninf * w[13], Ea = p.ninf * w[14];
    const float nt = __builtin_fmaf(-p.lam, a, w[12]);
    const float Et = __builtin_fmaf(p.lamn, w[14], w[15]);
    const float lo = fminf(fminf(m1, m2), m3), hi = fmaxf(fmaxf(m1, m2), m3);
    const bool pos = (a > Ea) & ((lo < -E) | (nt > Et));
    const bool neg = (a < -Ea) & ((hi > E) | (nt < -Et));
    return pos | neg;
}

// Test n triangles at positions pos0.. of the BVH-ordered arrays; `src` points at the
// record of position pos0 (in LDS or in HBM).
//   lt (shadow segments; NULL: none): the light table at position pos0 (kLtD floats per
//   triangle), sp the lane's SegPre, live the lanes whose result still matters.
//   GATE (a trace's second pass, trace_nearest / shadow_lit_single): a candidate counts only
//   if its face box (fbox, BVH order) passes the reference's Box.Intersect (object.go:76).
template <bool REL, bool PREFILTER, int DG = 0, bool TPRE = false, bool LT3 = true, bool GATE = false,
          typename SrcPtr>
__device__ __forceinline__ void test_range(SrcPtr src, const uint32_t* __restrict__ fidx, uint32_t pos0,
                                           uint32_t n, V3 ro, V3 d, V3 neg, Best& b, uint32_t& wtests,
                                           const float* lt = nullptr, const SegPre* sp = nullptr, bool live = true,
                                           const double* fbox = nullptr) {
    wtests += n;  // wave-uniform: triangles this wave tests (x active lanes = tests)
    if (MIRT_EXP_NO_TRI_TESTS || (MIRT_EXP_NO_SHADOW_TESTS && TPRE)) return;
    // the fp64 test of triangle i on the lanes `maybe` leaves
    auto test = [&](uint32_t i, bool maybe) {
        const uint32_t k = pos0 + i;
        const auto t = src + (size_t)i * kTriD;
        V3 p1or = REL ? V3{t[0], t[1], t[2]} : sub(ro, V3{t[0], t[1], t[2]});
        V3 e1{t[3], t[4], t[5]};
        V3 e2{t[6], t[7], t[8]};
        double tt;
        // k is wave-uniform: a scalar load (lgkmcnt), issued ahead of the test
        const uint32_t fk = ((const __attribute__((address_space(4))) uint32_t*)fidx)[k];
        bool acc = maybe && mt_test<PREFILTER, DG, TPRE>(p1or, e1, e2, neg, tt);
        if (GATE) acc = box_gate_small(box_load(fbox + (size_t)k * kBoxD), ro, d, acc);
        if (acc) {
            V3 ip = add(ro, scale(d, tt));  // triangle.go:69
            consider(b, len(sub(ro, ip)), fk, k);  // object.go:97
        }
    };
    // light-table classification of triangle i from its record (in SGPRs)
    auto classify = [&](const u32x16& a16) {
        float w[kLtD];
#pragma unroll
        for (int q = 0; q < kLtD; ++q) w[q] = __uint_as_float(a16[q]);
        diag(22);  // light-table classifications (shadow)
        return live & !seg_reject(*sp, w);  // (no short circuit: straight-line code)
    };
    if (TPRE && PREFILTER && lt) {
        // two triangles per step, both records loaded up front (one scalar-load wait per pair);
        // a wave whose lanes all reject a triangle skips its fp64 record
        if (LT3 && n == 3) {  // the default leaf: all three records up front
            const u32x16 r0 = ((cv16ptr)lt)[0];
            const u32x16 r1 = ((cv16ptr)(lt + kLtD))[0];
            const u32x16 r2 = ((cv16ptr)(lt + 2 * kLtD))[0];
            const bool m0 = classify(r0), m1 = classify(r1), m2 = classify(r2);
            if (__ballot(m0) != 0) test(0, m0);
            if (__ballot(m1) != 0) test(1, m1);
            if (__ballot(m2) != 0) test(2, m2);
            return;
        }
        for (uint32_t i = 0; i < n; i += 2) {
            const bool two = i + 1 < n;
            const u32x16 r0 = ((cv16ptr)(lt + (size_t)i * kLtD))[0];
            const u32x16 r1 = ((cv16ptr)(lt + (size_t)(two ? i + 1 : i) * kLtD))[0];
            const bool m0 = classify(r0);
            const bool m1 = two & classify(r1);
            if (__ballot(m0) != 0) test(i, m0);
            if (__ballot(m1) != 0) test(i + 1, m1);
        }
    } else if (TPRE && GATE) {  // a second pass (rare): the least code
#pragma unroll 1
        for (uint32_t i = 0; i < n; ++i) test(i, true);
    } else if (TPRE) {
        // unrolled by two by hand, as the classified loop above
        for (uint32_t i = 0; i < n; i += 2) {
            test(i, true);
            if (i + 1 < n) test(i + 1, true);
        }
    } else if (GATE) {  // a second pass (rare): the least code
#pragma unroll 1
        for (uint32_t i = 0; i < n; ++i) test(i, true);
    } else {
#pragma unroll 2
        for (uint32_t i = 0; i < n; ++i) test(i, true);
    }
}

struct Visits {
    uint32_t tests;     // triangles tested by the wave (x active lanes = ray-triangle tests)
    uint32_t nodes;     // BVH nodes whose children the wave tested
    uint32_t leaves;    // leaves the wave entered
    uint32_t overflow;  // wide-traversal stack overflows (never expected; tests assert 0)
};
// Per-wave totals over a whole persistent kernel.  At the end every wave parks its totals
// in LDS and one lane of the workgroup adds the sums into shard blockIdx % kStatShards:
// one atomic per statistic per workgroup (see the counter layout in mirt_internal.hpp).
struct WaveStats {
    cnt_t tests;                               // lane tests: can pass 2^32 per wave (brute force)
    uint32_t nodes, leaves, hits, overflow;    // wave-level counts (fewer live SGPRs)
};
// MIRT_PHASE_TIMING (diagnostic builds only): shader-clock cycles per phase of the primary
// blocks, reported in the timeline record instead of the wave's start/end clocks.
struct PhaseClock {
    uint64_t acc[4] = {0, 0, 0, 0};
    uint64_t t = 0;
    __device__ __forceinline__ void start() {
        if (MIRT_PHASE_TIMING) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void lap(int k) {
        if (MIRT_PHASE_TIMING) {
            const uint64_t n = __builtin_amdgcn_s_memtime();
            acc[k] += n - t;
            t = n;
        }
    }
};

// threadIdx.x made opaque to the compiler (FRESH): k_trace's end (statistics, summary) recomputes
// its byte offsets instead of keeping the start's 64-bit copy live through the whole work loop
// (that copy was k_trace's only spilled VGPR pair; in k_shadow the same change spilled 3 more)
template <bool FRESH>
__device__ __forceinline__ uint32_t tid_fresh() {
    uint32_t t = threadIdx.x;
    if (FRESH) asm volatile("" : "+v"(t));
    return t;
}
// The wave's index in its workgroup, said to be wave-uniform (it is): loop indices and work
// items derived from it live in SGPRs.  Held as a VGPR, they had been spilled across the work
// loops: k_shadow's 27 spilled VGPRs and k_bounce's 5 were these indices, shard cursors included.
__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
template <bool FRESH = false>
__device__ __forceinline__ void stats_flush(cnt_t* counters, cnt_t (*red)[4], int stat_tests, int stat_nodes,
                                            int stat_leaves, int stat_hits, const WaveStats& w) {
    const uint32_t tid = tid_fresh<FRESH>();
    const uint32_t wave = tid >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[wave][0] = w.tests;
        red[wave][1] = w.nodes;
        red[wave][2] = w.leaves;
        red[wave][3] = w.hits;
    }
    __syncthreads();
    // returning atomics: once the wave's vmcnt drains they have been performed, which is
    // what frame_fold's done count relies on (no L2-flushing fence needed)
    if ((threadIdx.x & 63) == 0 && w.overflow) {
        const cnt_t old = atomicAdd(&counters[cnt_stat(kStatOverflow, 0)], w.overflow);
        asm volatile("" ::"v"(old));
    }
    if (tid < 4) {
        cnt_t sum = 0;
        for (int k = 0; k < kWG / 64; ++k) sum += red[k][tid];
        const int stat = tid == 0 ? stat_tests : tid == 1 ? stat_nodes
                       : tid == 2 ? stat_leaves : stat_hits;  // < 0: not recorded
        if (sum && stat >= 0) {
            const cnt_t old = atomicAdd(&counters[cnt_stat(stat, blockIdx.x % kStatShards)], sum);
            asm volatile("" ::"v"(old));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Wave-uniform traversal stack in VGPR lanes: entry i lives in lane i % 64 of word i / 64
// (DEEP: two words, 128 entries; else one word, 64 entries, for trees of depth <=
// kBvhShallowDepth).  Push and pop are v_writelane / v_readlane with the SGPR stack pointer:
// no memory traffic and no LDS latency on the node-to-node dependency chain.
// A 64-bit value every lane holds the same of, in SGPRs (no instruction where it is there already)
__device__ __forceinline__ uint64_t u64_uniform(uint64_t v) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32;
}
template <bool DEEP>
struct WaveStack {
    int a = 0, b = 0;
    uint32_t sp = 0;
    __device__ __forceinline__ void put(uint32_t ref) {  // write the entry above the top
        ref = __builtin_amdgcn_readfirstlane(ref);  // (scalar already, except in an out-of-line pass)
        sp = __builtin_amdgcn_readfirstlane(sp);
        if (!DEEP || sp < 64)
            asm("v_writelane_b32 %0, %1, m0" : "+v"(a) : "s"(ref), "{m0}"(sp));
        else
            asm("v_writelane_b32 %0, %1, m0" : "+v"(b) : "s"(ref), "{m0}"(sp - 64));
    }
    __device__ __forceinline__ void push(uint32_t ref) {
        put(ref);
        ++sp;
    }
    // Child push without a branch: the ref is written above the top unconditionally and
    // kept (sp += 1) iff some live lane's ray enters the child, i.e. (m & live) != 0:
    // s_and_b64 sets SCC exactly then and s_addc_u32 adds it.
    __device__ __forceinline__ void push_if(uint32_t ref, uint64_t m, uint64_t live) {
        put(ref);
        // (scalar already in the kernels; an out-of-line second pass needs them said so)
        m = u64_uniform(m);
        live = u64_uniform(live);
        sp = __builtin_amdgcn_readfirstlane(sp);
        uint64_t t;
        asm volatile("s_and_b64 %1, %2, %3\n\ts_addc_u32 %0, %0, 0" : "+s"(sp), "=&s"(t) : "s"(m), "s"(live) : "scc");
    }
    __device__ __forceinline__ uint32_t pop() {
        --sp;
        return (uint32_t)(!DEEP || sp < 64 ? __builtin_amdgcn_readlane(a, (int)sp)
                                           : __builtin_amdgcn_readlane(b, (int)(sp - 64)));
    }
};

// fp32 ray of the conservative slab tests: origin, 1/D with zero or tiny components
// replaced by +-2^60 (so (bound - o) * inv is never 0 * inf), and o * inv.
struct Ray32 {
    float ox, oy, oz, ix, iy, iz, oix, oiy, oiz;
};
// 1/d from v_rcp_f64 refined by one Newton step (relative error far below fp32's 2^-24;
// the slab tests only need ~2^-20).
__device__ __forceinline__ float inv32(double d) {
    if (!(__builtin_fabs(d) >= 0x1p-60)) return __builtin_copysignf(0x1p60f, (float)d);  // tiny, zero or NaN
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
    return __builtin_fabs(r) > 0x1p60 ? __builtin_copysignf(0x1p60f, (float)d) : (float)r;
}
__device__ __forceinline__ Ray32 ray32(V3 ro, V3 d) {
    Ray32 r;
    r.ox = (float)ro.x;
    r.oy = (float)ro.y;
    r.oz = (float)ro.z;
    r.ix = inv32(d.x);
    r.iy = inv32(d.y);
    r.iz = inv32(d.z);
    r.oix = r.ox * r.ix;
    r.oiy = r.oy * r.iy;
    r.oiz = r.oz * r.iz;
    return r;
}
// One copy of a node in SGPRs: three s_load_dwordx16 + one s_load_dwordx8.  Words
// 16 a + 2 c (+1): near (far) bound of slot c on axis a (copy 0: lo, hi), 48..55 refs.
struct NodeRegs {
    u32x16 w0, w1, w2;
    u32x8 w3;  // the child refs (the copy's last 8 words are padding, never loaded)
    __device__ __forceinline__ uint32_t word(int i) const {
        return i < 16 ? w0[i] : i < 32 ? w1[i - 16] : i < 48 ? w2[i - 32] : w3[i - 48];
    }
    __device__ __forceinline__ float lo(int a, int c) const { return __uint_as_float(word(a * 16 + 2 * c)); }
    __device__ __forceinline__ float hi(int a, int c) const { return __uint_as_float(word(a * 16 + 2 * c + 1)); }
    __device__ __forceinline__ uint32_t child(int c) const { return word(48 + c); }
};
// oct (packet_octant): the copy of that sign octant; mixed packets (kOctMixed = 8) read
// copy 0, whose pairs are (lo, hi).
__device__ __forceinline__ NodeRegs load_node(cnptr nd, uint32_t oct = 0) {
    const cv16ptr p = (cv16ptr)&nd->oct[oct & 7u];
    return NodeRegs{p[0], p[1], p[2], ((cv8ptr)p)[6]};
}

// Ray vs child c's box, t >= 0 half-line.  Boxes are inflated by 2^-12 of the mesh
// scale, which covers the fp32 rounding of every quantity here for origins within the
// cull limit (256 x scale) by a factor > 4.
template <bool SEG>
__device__ __forceinline__ bool slab32(const NodeRegs& nd, int c, const Ray32& r, float tmax) {
    const float ax = __builtin_fmaf(nd.lo(0, c), r.ix, -r.oix), bx = __builtin_fmaf(nd.hi(0, c), r.ix, -r.oix);
    const float ay = __builtin_fmaf(nd.lo(1, c), r.iy, -r.oiy), by = __builtin_fmaf(nd.hi(1, c), r.iy, -r.oiy);
    const float az = __builtin_fmaf(nd.lo(2, c), r.iz, -r.oiz), bz = __builtin_fmaf(nd.hi(2, c), r.iz, -r.oiz);
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return tn <= (SEG ? fminf(tf, tmax) : tf);
}

// The same test as a lane mask (v_cmp straight into SGPRs: no per-lane bool to pack).
typedef float f32x2 __attribute__((ext_vector_type(2)));
// {lo, hi} * a[SA] - b[SB] in one v_pk_fma_f32: the box pair is an SGPR operand and
// op_sel broadcasts one dword of each ray pair to both halves (no per-child moves).
#define MIRT_PK_SLAB(SA, SB)                                                                         \
    template <>                                                                                      \
    __device__ __forceinline__ f32x2 pk_slab<SA, SB>(f32x2 box, f32x2 a, f32x2 b) {                  \
        f32x2 t;                                                                                     \
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0," #SA "," #SB "] op_sel_hi:[1," #SA "," #SB      \
            "] neg_lo:[0,0,1] neg_hi:[0,0,1]"                                                        \
            : "=v"(t) : "s"(box), "v"(a), "v"(b));                                                   \
        return t;                                                                                    \
    }
template <int SA, int SB>
__device__ __forceinline__ f32x2 pk_slab(f32x2 box, f32x2 a, f32x2 b);
__device__ __forceinline__ float a_min(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float a_max(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float a_min3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float a_max3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
MIRT_PK_SLAB(0, 1)
MIRT_PK_SLAB(1, 0)
#undef MIRT_PK_SLAB
template <bool SEG>
__device__ __forceinline__ uint64_t slab_mask(const NodeRegs& nd, int c, const Ray32& r, float tmax) {
    // both planes of an axis in one packed FMA; ray pairs (ix, iy), (iz, oix), (oiy, oiz)
    const f32x2 p0 = {r.ix, r.iy}, p1 = {r.iz, r.oix}, p2 = {r.oiy, r.oiz};
    const f32x2 tx = pk_slab<0, 1>((f32x2){nd.lo(0, c), nd.hi(0, c)}, p0, p1);
    const f32x2 ty = pk_slab<1, 0>((f32x2){nd.lo(1, c), nd.hi(1, c)}, p0, p2);
    const f32x2 tz = pk_slab<0, 1>((f32x2){nd.lo(2, c), nd.hi(2, c)}, p1, p2);
    // min/max as asm too: the compiler would otherwise canonicalize each asm result first
    // (no NaN reaches here: 1/D is clamped to +-2^60, bounds and origins are finite)
    const float tn = a_max3(a_min(tx.x, tx.y), a_min(ty.x, ty.y), a_max(a_min(tz.x, tz.y), 0.0f));
    float tf = a_min3(a_max(tx.x, tx.y), a_max(ty.x, ty.y), a_max(tz.x, tz.y));
    if (SEG) tf = a_min(tf, tmax);
    return __builtin_amdgcn_fcmpf(tn, tf, 5 /* FCMP_OLE: tn <= tf */);
}

// Sign octant of a packet: bit a set = every live lane's fp32 1/d is negative on axis a;
// kOctMixed = live lanes disagree on some axis.  With a uniform octant each axis's near and
// far plane are known without comparing them: for 1/d > 0, fma(lo, 1/d, -o/d) <=
// fma(hi, 1/d, -o/d) because lo <= hi and rounding is monotonic (reversed for 1/d < 0).
// Every node also stores each axis's bounds as (hi, lo) pairs (Bvh8Node::sbox); a packet
// loads, per axis, the copy whose first word is its near plane, and a child test needs no
// min/max sorting: 7 VALU instead of 13 (8 instead of 14 for segments), bit-for-bit the
// same decision as slab_mask (MIRT_OPT_NO_OCTANT: the sorted test only).
constexpr uint32_t kOctMixed = 8;
__device__ __forceinline__ uint32_t packet_octant(const Ray32& r, bool live) {
    const uint64_t lm = __ballot(live);
    const uint64_t nx = __ballot(live && r.ix < 0.0f), ny = __ballot(live && r.iy < 0.0f),
                   nz = __ballot(live && r.iz < 0.0f);
    if ((nx && nx != lm) || (ny && ny != lm) || (nz && nz != lm)) return kOctMixed;
    return (nx ? 1u : 0u) | (ny ? 2u : 0u) | (nz ? 4u : 0u);
}
// Child c's box with each axis pair loaded near-plane first (load_node with the octant).
template <bool SEG>
__device__ __forceinline__ uint64_t slab_mask_ordered(const NodeRegs& nd, int c, const Ray32& r, float tmax) {
    const f32x2 p0 = {r.ix, r.iy}, p1 = {r.iz, r.oix}, p2 = {r.oiy, r.oiz};
    const f32x2 tx = pk_slab<0, 1>((f32x2){nd.lo(0, c), nd.hi(0, c)}, p0, p1);
    const f32x2 ty = pk_slab<1, 0>((f32x2){nd.lo(1, c), nd.hi(1, c)}, p0, p2);
    const f32x2 tz = pk_slab<0, 1>((f32x2){nd.lo(2, c), nd.hi(2, c)}, p1, p2);
    const float tn = a_max3(tx.x, ty.x, a_max(tz.x, 0.0f));
    const float tf = SEG ? a_min3(tx.y, ty.y, a_min(tz.y, tmax)) : a_min3(tx.y, ty.y, tz.y);
    return __builtin_amdgcn_fcmpf(tn, tf, 5 /* FCMP_OLE */);
}
// Bit c = some live lane's ray meets child c.
template <bool ORDERED, bool SEG>
__device__ __forceinline__ uint32_t children_entered(const NodeRegs& nd, const Ray32& r, float tmax, uint64_t fmask,
                                                     uint64_t lmask) {
    uint32_t entered = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        if (nd.child(c) == kBvhEmpty) continue;
        const uint64_t m = ORDERED ? slab_mask_ordered<SEG>(nd, c, r, tmax) : slab_mask<SEG>(nd, c, r, tmax);
        if (((m | fmask) & lmask) != 0) entered |= 1u << c;
    }
    return entered;
}

// Wave-uniform walk of one object's 8-wide BVH (packet traversal).  A child is entered
// when ANY live lane's ray meets its box; entered children (inner nodes and leaves alike)
// go on the wave's register stack, the nearest one on top (node copies are sorted near
// to far for the packet's sign octant), and the walk pops them one at a time: a leaf is
// tested, an inner node loaded and its children tested.
//   Nearest query (!SEG): once a lane holds a candidate at distance b.d, boxes it would
//   enter beyond tmax = f32((b.d + M) (1 + 2^-20)), M = 2^-36 (1 + b.d + |ro|), are
//   skipped for it: every candidate inside such a box lies farther than b.d (the argument
//   of the segment bound below), so it can neither win nor tie.
//   SEG (segment query): a lane also skips boxes it enters beyond its tmax, and retires
//   once its nearest candidate is closer than `resolve` (the caller's decision is then
//   made); the walk ends when no live lane is left.
// Packets with a lane whose object-space origin is beyond the cull limit (the inflation
// argument needs a bounded origin) enter every child.
//   GATE: candidates pass their face box (fbox) first (test_range; a trace's second pass).
// ---------------------------------------------------------------- LDS triangle streaming
// north_star's "triangle data streamed through LDS in batches", for a mesh beyond the LDS
// (MIRT_OPT_LDS_STREAM, one-object frames, k_trace): each wave keeps a window of kStreamTris + 1
// consecutive faces of the BVH-ordered triangle array in its own LDS slice.  A leaf the window
// holds is tested from LDS; otherwise the wave first loads the window around the leaf (centred
// on it, so leaves visited after it on either side in BVH order are likely inside) with vector
// loads, 16 bytes per lane per load (1.8 KB in 2 loads), then tests it from LDS.  The records are
// copied, not recomputed: the same bits are tested either way.  Window size (round 6, configs[3],
// three runs each, profiles/r06_ab_stream_window.txt): 112 faces (8 KB) 1.112 ms device per frame
// at an 84% window hit rate, 48 faces 1.094, 32 faces 1.098, 24 faces 1.085, 16 faces 1.095.
#ifndef MIRT_STREAM_TRIS
#define MIRT_STREAM_TRIS 24
#endif
constexpr uint32_t kStreamTris = MIRT_STREAM_TRIS;  // even
constexpr size_t kStreamSlice = (size_t)(kStreamTris + 1) * kTriD;  // doubles per wave (an odd base rounds down)
constexpr size_t kStreamBytes = (kWG / 64) * kStreamSlice * sizeof(double);
// each wave's window start (~0: none); k_trace resets it before its waves start
__shared__ uint32_t g_stream_base[kWG / 64];
extern __shared__ __attribute__((aligned(16))) double g_lds_mesh[];
__device__ __forceinline__ const double* stream_leaf(cdptr tri, uint32_t ntri, uint32_t first, uint32_t cnt) {
    const uint32_t wave = wave_id();
    double* slice = g_lds_mesh + (size_t)wave * kStreamSlice;
    uint32_t base = __builtin_amdgcn_readfirstlane(g_stream_base[wave]);
    diag(23);  // leaves served through the window (MIRT_DIAG builds)
    if (base == ~0u || first < base || first + cnt > base + kStreamTris + 1 || first + cnt > ntri) {
        diag(31);  // window reloads (8 KB each)
        // an even start (16-byte aligned: 72-byte faces), at most ntri - kStreamTris, so the
        // kStreamTris + 1 faces from it cover the leaf
        base = first > kStreamTris / 2 ? first - kStreamTris / 2 : 0u;
        if (ntri > kStreamTris && base > ntri - kStreamTris) base = ntri - kStreamTris;
        base &= ~1u;
        const uint32_t n = min(kStreamTris + 1, ntri - base), nd = n * kTriD;
        const double2* src = (const double2*)(tri + (size_t)base * kTriD);
        double2* dst = (double2*)slice;
        asm volatile("" ::: "memory");  // every lane's reads of the previous window come first
        for (uint32_t i = threadIdx.x & 63; i < nd / 2; i += 64) dst[i] = src[i];
        if ((nd & 1) && (threadIdx.x & 63) == 0) slice[nd - 1] = tri[(size_t)base * kTriD + nd - 1];
        if ((threadIdx.x & 63) == 0) g_stream_base[wave] = base;
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slice is written before it is read
    }
    return slice + (size_t)(first - base) * kTriD;
}

template <bool REL, bool PREFILTER, bool SEG, bool LT3 = true, bool GATE = false, typename SrcPtr>
__device__ __forceinline__ void bvh_sweep(const DevMesh& m, SrcPtr src, V3 ro, V3 d, V3 neg, bool lane_on, Best& b,
                                          Visits& vis, float tmax = 0.0f, double resolve = 0.0, bool octant = true,
                                          const float* lt = nullptr, const SegPre* sp = nullptr,
                                          const double* fbox = nullptr, bool stream = false) {
    // LDS-resident meshes (the host guarantees depth <= kBvhShallowDepth) use a one-VGPR stack
    constexpr bool DEEP = !__is_same(SrcPtr, const double*);
    const Ray32 r = ray32(ro, d);
    const double far = fmax(fmax(__builtin_fabs(ro.x), __builtin_fabs(ro.y)), __builtin_fabs(ro.z));
    const bool all = __ballot(lane_on && !(far <= m.cull_limit)) != 0;  // wave-uniform
    bool live = lane_on;
    const uint32_t oct = octant && !all ? packet_octant(r, lane_on) : kOctMixed;  // wave-uniform
    float tm = SEG ? tmax : __builtin_inff();
    const double Mbase = 0x1p-36 * (1.0 + far);
    WaveStack<DEEP> stk;
    stk.push(0u);  // the root
    do {
        const uint32_t ref = stk.pop();
        if (ref & kBvhLeafBit) {
            const uint32_t first = ref & kBvhFirstMask, cnt = (ref & ~kBvhLeafBit) >> kBvhCountShift;
            ++vis.leaves;
            diag(SEG ? 14 : 6);
            const float* lt_leaf = lt ? lt + (size_t)first * kLtD : nullptr;
            if (DEEP && stream)  // an HBM mesh through the wave's LDS window (stream is a constant)
                test_range<REL, PREFILTER, SEG ? 8 : 0, SEG, LT3, GATE>(stream_leaf((cdptr)src, m.ntri, first, cnt), m.fidx,
                                                                     first, cnt, ro, d, neg, b, vis.tests, lt_leaf, sp, live,
                                                                     fbox);
            else
                test_range<REL, PREFILTER, SEG ? 8 : 0, SEG, LT3, GATE>(src + (size_t)first * kTriD, m.fidx, first, cnt, ro,
                                                                     d, neg, b, vis.tests, lt_leaf, sp, live, fbox);
            if (SEG) {
                live = live && !(b.has() && b.d < resolve);
                if (__ballot(live) == 0) break;
            } else if (b.has()) {
                tm = (float)(b.d + (Mbase + 0x1p-36 * b.d)) * (1.0f + 0x1p-20f);
            }
            continue;
        }
        const NodeRegs nd = load_node((cnptr)m.nodes + ref, oct);
        ++vis.nodes;
        diag(SEG ? 13 : 5);
        const uint64_t lm = __ballot(live);
        if (oct != kOctMixed) {
            // far first: slot 0, the nearest, ends on top.  Empty slots come last in a copy,
            // so slots 4..7 (2..3) are skipped at once when slot 4 (2) is empty; the test of
            // any other empty slot fails (its box is lo = +inf, hi = -inf).
            if (nd.child(4) != kBvhEmpty) {
#pragma unroll
                for (int c = 7; c >= 4; --c) stk.push_if(nd.child(c), slab_mask_ordered<true>(nd, c, r, tm), lm);
            }
            if (nd.child(2) != kBvhEmpty) {
#pragma unroll
                for (int c = 3; c >= 2; --c) stk.push_if(nd.child(c), slab_mask_ordered<true>(nd, c, r, tm), lm);
            }
#pragma unroll
            for (int c = 1; c >= 0; --c) stk.push_if(nd.child(c), slab_mask_ordered<true>(nd, c, r, tm), lm);
        } else if (!all) {
#pragma unroll
            for (int c = 7; c >= 0; --c) {
                if (nd.child(c) == kBvhEmpty) continue;
                stk.push_if(nd.child(c), slab_mask<true>(nd, c, r, tm), lm);
            }
        } else {
#pragma unroll
            for (int c = 7; c >= 0; --c)
                if (nd.child(c) != kBvhEmpty) stk.push(nd.child(c));
        }
    } while (stk.sp != 0);
}

// The LDS-resident mesh (RESIDENT kernels): dynamic shared memory sized to the mesh at
// launch, 72 B per face, after the kernel's static LDS (the launch passes 0 bytes otherwise).
extern __shared__ __attribute__((aligned(16))) double g_lds_mesh[];

// (build-time switches: diag.hpp)
#define MIRT_TRACE_KERNEL __global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(MIRT_WAVES_PER_EU)))
// k_reflect keeps a whole bounce (ray, hit, normal) live through its shadow queries.  At 2
// waves per SIMD (256 VGPRs, one 512-thread workgroup per CU) nothing spills (168 VGPRs),
// but configs[4] ran 30% slower (1.28-1.31 vs 0.98-1.01 ms per frame, tools/ab_bench.sh):
// the occupancy is worth more than the 17-77 spilled VGPRs (<= 160 B of scratch per lane,
// mostly outside the traversal loops) it costs at 4.
#define MIRT_REFLECT_KERNEL \
    __global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(MIRT_REFLECT_WAVES_PER_EU)))

// ---------------------------------------------------------------- wide traversal
// Wave reductions over 64 lanes (DPP row shifts + row broadcasts; every lane active,
// lanes without data hold the identity).  Result read from lane 63: wave-uniform.
template <bool MIN, int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ float dpp_step(float v) {
    const float id = MIN ? __builtin_inff() : -__builtin_inff();
    const int t = __builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), CTRL, ROW_MASK, BANK_MASK, false);
    return MIN ? fminf(v, __int_as_float(t)) : fmaxf(v, __int_as_float(t));
}
template <bool MIN>
__device__ __forceinline__ float wave_reduce(float v) {
    v = dpp_step<MIN, 0x111, 0xf, 0xf>(v);  // row_shr:1
    v = dpp_step<MIN, 0x112, 0xf, 0xf>(v);  // row_shr:2
    v = dpp_step<MIN, 0x113, 0xf, 0xf>(v);  // row_shr:3
    v = dpp_step<MIN, 0x114, 0xf, 0xe>(v);  // row_shr:4
    v = dpp_step<MIN, 0x118, 0xf, 0xc>(v);  // row_shr:8
    v = dpp_step<MIN, 0x142, 0xa, 0xf>(v);  // row_bcast:15
    v = dpp_step<MIN, 0x143, 0xc, 0xf>(v);  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// A packet of rays through one common point C (object space): the camera for primary
// rays, the light for shadow rays walked backwards.  Lane ray: C + s * e_lane with s in
// [smin, smax].  The cone keeps, per axis, the range of the lanes' fp32 1/e; a child box
// is entered iff the interval slab test passes:
//   (bound - C) * (1/e) is linear in 1/e, so over the packet every lane's plane crossing
//   lies between the values at the two endpoints of the range; the per-axis minimum of
//   those four products bounds every lane's near crossing from below and the maximum
//   bounds its far crossing from above.  If any lane's ray meets the box, the bounds pass.
// fp32 rounding is covered by the 2^-12 x scale box inflation exactly as for the per-lane
// test.  all = accept everything (origin beyond the cull limit, or a lane
// with a non-finite direction).
struct Cone {
    float ixlo, ixhi, iylo, iyhi, izlo, izhi;      // range of 1/e over live lanes
    float cxlo, cxhi, cylo, cyhi, czlo, czhi;      // C * each endpoint
    float smin, smax;
    bool all, none;
};
__device__ __forceinline__ float u_f(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ float u_lane(float x, uint32_t lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), (int)lane));
}
__device__ __forceinline__ Cone make_cone(V3 corig, float ix, float iy, float iz, bool live, bool force,
                                          float smin_lane, float smax_lane, double cull_limit) {
    Cone c;
    c.none = __ballot(live) == 0;
    const float cx = u_f((float)corig.x), cy = u_f((float)corig.y), cz = u_f((float)corig.z);
    const double far = fmax(fmax(__builtin_fabs(corig.x), __builtin_fabs(corig.y)), __builtin_fabs(corig.z));
    const bool bad = live && (force || !(__builtin_fabsf(ix) <= 0x1p61f && __builtin_fabsf(iy) <= 0x1p61f &&
                                         __builtin_fabsf(iz) <= 0x1p61f && smax_lane >= smin_lane));
    c.all = __ballot(bad) != 0 || !(u_f((float)far) <= (float)cull_limit && far <= cull_limit);
    const float inf = __builtin_inff();
    c.ixlo = wave_reduce<true>(live ? ix : inf);
    c.ixhi = wave_reduce<false>(live ? ix : -inf);
    c.iylo = wave_reduce<true>(live ? iy : inf);
    c.iyhi = wave_reduce<false>(live ? iy : -inf);
    c.izlo = wave_reduce<true>(live ? iz : inf);
    c.izhi = wave_reduce<false>(live ? iz : -inf);
    c.cxlo = cx * c.ixlo;
    c.cxhi = cx * c.ixhi;
    c.cylo = cy * c.iylo;
    c.cyhi = cy * c.iyhi;
    c.czlo = cz * c.izlo;
    c.czhi = cz * c.izhi;
    c.smin = wave_reduce<true>(live ? smin_lane : inf);
    c.smax = wave_reduce<false>(live ? smax_lane : -inf);
    return c;
}
__device__ __forceinline__ bool cone_box(const Cone& c, float lx, float ly, float lz, float hx, float hy, float hz) {
    const float l0 = __builtin_fmaf(lx, c.ixlo, -c.cxlo), l1 = __builtin_fmaf(lx, c.ixhi, -c.cxhi);
    const float h0 = __builtin_fmaf(hx, c.ixlo, -c.cxlo), h1 = __builtin_fmaf(hx, c.ixhi, -c.cxhi);
    const float m0 = __builtin_fmaf(ly, c.iylo, -c.cylo), m1 = __builtin_fmaf(ly, c.iyhi, -c.cyhi);
    const float k0 = __builtin_fmaf(hy, c.iylo, -c.cylo), k1 = __builtin_fmaf(hy, c.iyhi, -c.cyhi);
    const float p0 = __builtin_fmaf(lz, c.izlo, -c.czlo), p1 = __builtin_fmaf(lz, c.izhi, -c.czhi);
    const float q0 = __builtin_fmaf(hz, c.izlo, -c.czlo), q1 = __builtin_fmaf(hz, c.izhi, -c.czhi);
    const float nx = fminf(fminf(l0, l1), fminf(h0, h1)), fx = fmaxf(fmaxf(l0, l1), fmaxf(h0, h1));
    const float ny = fminf(fminf(m0, m1), fminf(k0, k1)), fy = fmaxf(fmaxf(m0, m1), fmaxf(k0, k1));
    const float nz = fminf(fminf(p0, p1), fminf(q0, q1)), fz = fmaxf(fmaxf(p0, p1), fmaxf(q0, q1));
    const float tn = fmaxf(fmaxf(nx, ny), fmaxf(nz, c.smin));
    const float tf = fminf(fminf(fx, fy), fminf(fz, c.smax));
    return tn <= tf;
}

// Per-lane test of one box held in SGPRs (leaf boxes accepted by the cone: skip the
// leaf when no lane's own ray meets it).
template <bool SEG>
__device__ __forceinline__ bool lane_box(const Ray32& r, float lx, float ly, float lz, float hx, float hy, float hz,
                                         float tmax) {
    const float ax = __builtin_fmaf(lx, r.ix, -r.oix), bx = __builtin_fmaf(hx, r.ix, -r.oix);
    const float ay = __builtin_fmaf(ly, r.iy, -r.oiy), by = __builtin_fmaf(hy, r.iy, -r.oiy);
    const float az = __builtin_fmaf(lz, r.iz, -r.oiz), bz = __builtin_fmaf(hz, r.iz, -r.oiz);
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), 0.0f));
    const float tf = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return tn <= (SEG ? fminf(tf, tmax) : tf);
}

// Walk one object's BVH for a shared-origin packet.  Each pass pops up to kWideBatch
// nodes from the wave's LDS stack `stk`; lane L tests child L % 8 of node L / 8 against
// the cone; accepted inner children are pushed (one ds_write per lane), accepted leaves
// are tested per lane (box, then triangles).  Lanes whose own origin is beyond the cull
// limit force every leaf (and the cone accepts everything for them via `all`).
//   SEG: as bvh_sweep (retire lanes whose nearest candidate is below `resolve`, skip
//   leaf boxes entered beyond tmax).
template <bool REL, bool PREFILTER, bool SEG, typename SrcPtr>
__device__ __forceinline__ void bvh_wide(const DevMesh& m, SrcPtr src, uint32_t* __restrict__ stk, const Cone& cone,
                                         const Ray32& r, bool force, V3 ro, V3 d, V3 neg, bool lane_on, Best& b,
                                         Visits& vis, uint32_t& overflow, float tmax = 0.0f, double resolve = 0.0) {
    if (cone.none) return;
    const uint32_t lane = threadIdx.x & 63;
    bool live = lane_on;
    uint32_t sp = 1;
    if (lane == 0) stk[0] = 0;  // root
    while (sp > 0) {
        uint32_t k = ((int32_t)sp <= wide_thresh(m)) ? min(sp, (uint32_t)kWideBatch) : 1u;
        const uint32_t slot = lane >> 3, c = lane & 7;
        const bool on = slot < k;
        uint32_t node = 0;
        if (on) node = stk[sp - 1 - slot];
        sp -= k;
        vis.nodes += k;
        float lx = 0, ly = 0, lz = 0, hx = 0, hy = 0, hz = 0;
        uint32_t ref = kBvhEmpty;
        if (on) {
            const float* nb = (const float*)&m.nodes[node].oct[0];  // copy 0: (lo, hi) pairs
            ref = ((const uint32_t*)nb)[48 + c];
            lx = nb[2 * c];
            ly = nb[16 + 2 * c];
            lz = nb[32 + 2 * c];
            hx = nb[2 * c + 1];
            hy = nb[16 + 2 * c + 1];
            hz = nb[32 + 2 * c + 1];
        }
        const bool acc = ref != kBvhEmpty && (cone.all || cone_box(cone, lx, ly, lz, hx, hy, hz));
        const bool is_leaf = (ref & kBvhLeafBit) != 0;
        const uint64_t inner = __ballot(acc && !is_leaf);
        uint64_t leaves = __ballot(acc && is_leaf);
        const uint32_t npush = __popcll(inner);
        if (sp + npush > (uint32_t)kBvhStack) {  // cannot happen (wide_thresh bound); counted
            ++overflow;
            break;
        }
        if (acc && !is_leaf) stk[sp + __popcll(inner & ((1ull << lane) - 1ull))] = ref;
        sp += npush;
        while (leaves) {
            const uint32_t bit = __ffsll((unsigned long long)leaves) - 1;
            leaves &= leaves - 1;
            const uint32_t lref = __builtin_amdgcn_readlane(ref, bit);
#if MIRT_LEAF_LANE_TEST
            const float blx = u_lane(lx, bit), bly = u_lane(ly, bit), blz = u_lane(lz, bit);
            const float bhx = u_lane(hx, bit), bhy = u_lane(hy, bit), bhz = u_lane(hz, bit);
            if (__ballot(live && (force || lane_box<SEG>(r, blx, bly, blz, bhx, bhy, bhz, tmax))) == 0) continue;
#endif
            const uint32_t first = lref & kBvhFirstMask, cnt = (lref & ~kBvhLeafBit) >> kBvhCountShift;
            ++vis.leaves;
            test_range<REL, PREFILTER>(src + (size_t)first * kTriD, m.fidx, first, cnt, ro, d, neg, b, vis.tests);
            if (SEG) live = live && !(b.has() && b.d < resolve);
        }
        if (SEG && __ballot(live) == 0) break;
    }
}

// Packet walk of a view table (ViewLeaf) instead of the BVH, for rays that all pass through
// the view point.  Lane state: its direction (ls, lt) in the view's (s, t) plane, or unb
// (every direction), and its depth bound zl (a leaf farther from the view point than zl
// cannot hold a candidate of the lane).  (cs0, cs1) x (ct0, ct1) bounds the live lanes'
// directions (wave-uniform).  A leaf is tested when some live lane's direction lies in its
// rectangle within its depth bound; leaves come nearest first, so the walk ends at the first
// leaf beyond every live lane's bound.
//   !SEG (primary rays, view = the camera): zl is bvh_sweep's nearest-query bound, tightened
//   as the lane finds candidates.  SEG (shadow segments, view = the light): zl is fixed,
//   lanes retire as in bvh_sweep.
template <bool PREFILTER, bool SEG, typename SrcPtr>
__device__ __forceinline__ void view_sweep(const DevMesh& m, SrcPtr src, const ViewLeaf* __restrict__ vt, uint32_t n,
                                           float ls, float lt, bool unb, float cs0, float cs1, float ct0, float ct1,
                                           float zl, V3 ro, V3 d, V3 neg, bool lane_on, Best& b, Visits& vis,
                                           double resolve = 0.0, float tseg = 0.0f) {
    const uint32_t lane = threadIdx.x & 63;
    bool live = lane_on;
    // the lane's own ray against a candidate leaf's box, as bvh_sweep's slab test (primary:
    // bounded by the nearest-query bound zl; segments: by tseg)
    const Ray32 r32 = ray32(ro, d);
    const double Mbase =
        0x1p-36 * (1.0 + fmax(fmax(__builtin_fabs(ro.x), __builtin_fabs(ro.y)), __builtin_fabs(ro.z)));
    bool done = false;
    for (uint32_t p0 = 0; p0 < n && !done; p0 += 64) {
        const uint32_t j = p0 + lane;
        float4 a = make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff());
        float dm = __builtin_inff();
        uint32_t ref = 0, lix = 0;
        if (j < n) {
            const float4* q = (const float4*)(vt + j);
            a = q[0];
            const float4 c = q[1];
            dm = c.x;
            ref = __float_as_uint(c.y);
            lix = __float_as_uint(c.z);
        }
        ++vis.nodes;
        uint64_t cand = __ballot(j < n && a.x <= cs1 && a.y >= cs0 && a.z <= ct1 && a.w >= ct0);
        while (cand) {
            const uint32_t bit = (uint32_t)__builtin_ctzll(cand);
            cand &= cand - 1;
            const float dmin = u_lane(dm, bit);
            if (__ballot(live && dmin <= zl) == 0) {  // this leaf and every later one: beyond all lanes
                done = true;
                break;
            }
            const float s0 = u_lane(a.x, bit), s1 = u_lane(a.y, bit), t0 = u_lane(a.z, bit), t1 = u_lane(a.w, bit);
            if (__ballot(live && dmin <= zl && (unb || (ls >= s0 && ls <= s1 && lt >= t0 && lt <= t1))) == 0) continue;
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)ref, (int)bit);
            const uint32_t li = (uint32_t)__builtin_amdgcn_readlane((int)lix, (int)bit);
            const LeafBox* lb = m.leaves + li;
            if (__ballot(live && lane_box<true>(r32, lb->lo[0], lb->lo[1], lb->lo[2], lb->hi[0], lb->hi[1], lb->hi[2],
                                                SEG ? tseg : zl)) == 0)
                continue;
            const uint32_t first = r & kBvhFirstMask, cnt = (r & ~kBvhLeafBit) >> kBvhCountShift;
            ++vis.leaves;
            diag(SEG ? 14 : 6);
            test_range<false, PREFILTER, SEG ? 8 : 0, SEG>(src + (size_t)first * kTriD, m.fidx, first, cnt, ro, d, neg, b,
                                                        vis.tests);
            if (SEG) {
                live = live && !(b.has() && b.d < resolve);
                if (__ballot(live) == 0) {
                    done = true;
                    break;
                }
            } else if (b.has()) {
                zl = fminf(zl, (float)(b.d + (Mbase + 0x1p-36 * b.d)) * (1.0f + 0x1p-20f));
            }
        }
    }
}

struct Nearest {
    bool ok;
    uint32_t obj, face, mat;
    V3 hit, normal;
};

// Winner recompute for one object: world hit, normal (InterpNormal or Normal),
// material.  Same arithmetic as the sweep, so the same hit point.
__device__ __forceinline__ void winner(const DevObject& ob, uint32_t pos, V3 ro, V3 d, V3 neg, V3& world,
                                       V3& normal, uint32_t& mat, bool want_normal) {
    const double* t = ob.m.tri + (size_t)pos * kTriD;
    V3 p1 = vload(t), e1 = vload(t + 3), e2 = vload(t + 6);
    double tt = 0, r1 = 0, r2 = 0, r3 = 0;
    mt_full(sub(ro, p1), e1, e2, neg, tt, r1, r2, r3);
    V3 ip = add(ro, scale(d, tt));
    world = add(ip, V3{ob.pos[0], ob.pos[1], ob.pos[2]});  // object.go:109
    if (want_normal) {
        if (ob.m.has_normals) {
            const double* nn = ob.m.vnrm + (size_t)pos * kTriD;
            // triangle.go:29-31: ((N1*r1 + N2*r2) + N3*r3).Norm()
            normal = norm(add(add(scale(vload(nn), r1), scale(vload(nn + 3), r2)), scale(vload(nn + 6), r3)));
        } else {
            // triangle.go:24-26: (P2-P1) x (P3-P1) normalised
            normal = norm(cross(e1, e2));
        }
        mat = ob.m.fmat[pos];
    }
}

// tracer.go:27-50: nearest over objects by |hit - Cam.Pos| (also for shadow rays),
// first object in order wins ties (strict <).
//   RESIDENT: object 0's mesh sits in LDS (`lds`), relative (p1or) when REL.
//   BRUTE:    sweep every triangle instead of walking the BVH.
//   COMMON:   every lane's ray starts at o (primary rays): wide cone traversal.
//   vt (one-object frames, LDS-resident, !REL): the camera's view table; (ls, lt) the lane's
//   direction and crect the block's range of directions (view_sweep).
//   The reference searches only objects whose box the ray meets (tracer.go:32) and only faces
//   whose box it meets (object.go:76), by Box.Intersect (box.go:29-68) on the padded boxes of
//   shared/state (rtreego's inner nodes are not replicated).  The sweep keeps
//   every candidate (the culling is exact) and the boxes are applied to its outcome: an object
//   box that fails removes the object; a winner whose face box passes, with no NaN distance
//   around (whose first-hit rule could elect another face), is the nearest gated candidate
//   itself.  Should some lane's winner fail its face box, `redo` is set (wave-uniform; the
//   result is then meaningless) and the caller runs its work item again with pass2, where every
//   candidate is gated before it counts (an LDS-resident mesh swept whole, an HBM mesh through
//   its BVH).  The retry lives in the callers' work loops: a loop around the sweep here cost
//   ~5% of the frame (VALU and SALU of the restructured sweep, tools/ab_valu.sh).
//   obj_sure (wave-uniform): the object's box is known to pass for every lane (a primary block
//   inside the object-box certificate, block_obj_cert), so its gate is skipped.
//   MIRT_OPT_NO_BOX_GATE: no boxes (brute-force semantics).
template <bool REL, bool PREFILTER, bool BRUTE, bool COMMON = false, int HBM1 = 0>
__device__ __forceinline__ Nearest trace_nearest(const FrameArgs& fa, const double* __restrict__ lds, bool resident, V3 o, V3 d,
                                 bool lane_on, bool want_normal, Visits& vis, bool pass2, bool& redo,
                                 bool obj_sure = false, uint32_t* __restrict__ stk = nullptr, const ViewLeaf* vt = nullptr, uint32_t vn = 0,
                                 float ls = 0.0f, float lt = 0.0f, float4 crect = float4{0.0f, 0.0f, 0.0f, 0.0f}) {
    Nearest best;
    best.ok = false;
    best.obj = best.face = best.mat = 0;
    best.hit = best.normal = V3{0, 0, 0};
    double bestcd = 0;
    V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    const bool gating = MIRT_BOX_GATE && !(fa.flags & MIRT_OPT_NO_BOX_GATE);
    bool again = false;
    // (HBM1: the one-object HBM-mesh kernels, launched by the host for those frames only)
    const uint32_t nobj = HBM1 ? 1u : fa.n_objects;
    for (uint32_t oi = 0; oi < nobj; ++oi) {
        const DevObject& ob = fa.obj[oi];
        V3 ro = sub(o, V3{ob.pos[0], ob.pos[1], ob.pos[2]});  // object.go:71
        V3 neg = scale(d, -1);  // triangle.go:38 rDir.Scale(-1)
        Best b;
        best_init(b);
        const uint32_t ntri = ob.m.ntri;
        if (pass2) {
            // every candidate gated: an LDS-resident mesh (<= kLdsTris faces) is swept whole,
            // which keeps the gate's code out of the BVH walk; an HBM mesh walks its BVH
            if (resident)
                test_range<REL, PREFILTER, 0, false, true, true>(lds, ob.m.fidx, 0, ntri, ro, d, neg, b, vis.tests,
                                                               nullptr, nullptr, true, mesh_fbox(ob.m));
            else if (BRUTE)
                test_range<false, PREFILTER, 0, false, true, true>((cdptr)ob.m.tri, ob.m.fidx, 0, ntri, ro, d, neg, b,
                                                                 vis.tests, nullptr, nullptr, true, mesh_fbox(ob.m));
            else
                bvh_sweep<false, PREFILTER, false, true, true>(ob.m, (cdptr)ob.m.tri, ro, d, neg, lane_on, b, vis, 0.0f,
                                                               0.0, !(fa.flags & MIRT_OPT_NO_OCTANT), nullptr, nullptr,
                                                               mesh_fbox(ob.m), HBM1 == 2);
        } else if (BRUTE) {
            if (resident)
                test_range<REL, PREFILTER>(lds, ob.m.fidx, 0, ntri, ro, d, neg, b, vis.tests);
            else  // every triangle straight from HBM (waves run independently: no LDS staging)
                test_range<false, PREFILTER>((cdptr)ob.m.tri, ob.m.fidx, 0, ntri, ro, d, neg, b, vis.tests);
        } else if (COMMON) {
            const Ray32 r = ray32(ro, d);
            const double far = fmax(fmax(__builtin_fabs(ro.x), __builtin_fabs(ro.y)), __builtin_fabs(ro.z));
            const bool force = !(far <= ob.m.cull_limit);
            const Cone cone = make_cone(ro, r.ix, r.iy, r.iz, lane_on, force, 0.0f, __builtin_inff(), ob.m.cull_limit);
            if (resident)
                bvh_wide<REL, PREFILTER, false>(ob.m, lds, stk, cone, r, force, ro, d, neg, lane_on, b, vis, vis.overflow);
            else
                bvh_wide<false, PREFILTER, false>(ob.m, (cdptr)ob.m.tri, stk, cone, r, force, ro, d, neg, lane_on, b, vis,
                                                  vis.overflow);
        } else if (resident && !REL && vt) {
            view_sweep<PREFILTER, false>(ob.m, lds, vt, vn, ls, lt, false, crect.x, crect.y, crect.z, crect.w,
                                         __builtin_inff(), ro, d, neg, lane_on, b, vis);
        } else if (resident) {
            bvh_sweep<REL, PREFILTER, false>(ob.m, lds, ro, d, neg, lane_on, b, vis, 0.0f, 0.0,
                                             !(fa.flags & MIRT_OPT_NO_OCTANT));
        } else {
            bvh_sweep<false, PREFILTER, false>(ob.m, (cdptr)ob.m.tri, ro, d, neg, lane_on, b, vis, 0.0f, 0.0,
                                               !(fa.flags & MIRT_OPT_NO_OCTANT), nullptr, nullptr, nullptr, HBM1 == 2);
        }
        uint32_t face = 0, pos = 0;
        bool got = lane_on && best_result(b, face, pos);
        if (gating) {
            // the object's box (tracer.go:32), then, in a first pass, the winner's face box
            // (object.go:76): one box_gate serves both (a loop, so its code is not repeated)
            bool fok = true;
            if (obj_sure) diag(30);  // object gates the block certificate skips
#pragma unroll 1
            for (int k = obj_sure ? 1 : 0; k < (pass2 ? 1 : 2); ++k) {  // obj_sure: the block's certificate
                Box6 bx;
                if (k == 0)
                    bx = Box6{{ob.box[0], ob.box[1], ob.box[2], ob.box[3], ob.box[4], ob.box[5]}};
                else
                    bx = box_load(mesh_fbox(ob.m) + (size_t)pos * kBoxD);
                const bool r = box_gate(bx, k == 0 ? o : ro, d, got);
                if (k == 0)
                    got = r;
                else
                    fok = r;
            }
            if (!pass2) again = again || (got && (!fok || b.any_nan()));
        }
        if (got) {
            V3 world, normal{0, 0, 0};
            uint32_t mat = 0;
            winner(ob, pos, ro, d, neg, world, normal, mat, want_normal);
            double cd = len(sub(world, cam));  // tracer.go:38
            if (!best.ok || cd < bestcd) {
                best.ok = true;
                bestcd = cd;
                best.obj = oi;
                best.face = face;
                best.mat = mat;
                best.hit = world;
                best.normal = normal;
            }
        }
    }
    if (MIRT_BOX_GATE == 2) {  // measurement build: gates evaluated, no second pass
        vis.overflow += __ballot(again) != 0;
        again = false;
    }
    redo = __ballot(again) != 0;
    if (redo) diag(28);  // nearest queries run again (pass 2)
    return best;
}
// trace_nearest with its second pass in place, for callers without a work loop to retry in
// (k_rays, the reflection chains, k_bounce's own shadows).
template <bool REL, bool PREFILTER, bool BRUTE, int HBM1 = 0>
__device__ __forceinline__ Nearest trace_nearest_settled(const FrameArgs& fa, const double* __restrict__ lds,
                                                         bool resident, V3 o, V3 d, bool lane_on, bool want_normal,
                                                         Visits& vis) {
    bool redo = false;
    Nearest r;
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        r = trace_nearest<REL, PREFILTER, BRUTE, false, HBM1>(fa, lds, resident, o, d, lane_on, want_normal, vis, pass == 1,
                                                               redo);
        if (!redo) break;
    }
    return r;
}

// Shadow ray of a one-object frame as a segment query (exact; DESIGN.md §4 "Shadow
// segments").  Only tracer.go:64's lit flag leaves the kernel:
//   lit = !shaded || |L - hit| < |occluder - hit|,   occluder = nearest hit from o.
// With lh = |L - hit| and |o - hit| = 1e-4 (+ rounding), a candidate at distance dist from
// o lies within dist + 1e-4 + M of hit, and the nearest is no farther, so
//   dist < lh - 1e-4 - M  =>  not lit (the lane retires: any-hit);
//   every candidate beyond lh + 1e-4 + M  =>  lit, so boxes entered beyond that are culled;
// otherwise the nearest candidate found is the true nearest and the reference comparison
// runs unchanged.  M bounds every fp64 rounding involved with a wide margin.
//   vt / vh (LDS-resident): the light's view table and header (view_sweep from the light).
//   LT3: a three-face leaf loads its three light-table records at once (k_trace; the split
//   k_shadow loads two per step, which spills fewer VGPRs there)
//   The reference's boxes (trace_nearest) are applied to what the decision rests on: a lane
//   that retired rests on its candidate b.pos (a gated candidate nearer than `resolve` proves
//   "not lit" whatever else the boxes remove); a lane whose candidates all lie beyond the light
//   (no NaN distance) is lit under any gating; else it rests on the winner, which must pass
//   with no NaN distance around.  An object box that fails leaves no candidate (lit).  A face
//   box that fails sets `redo` (wave-uniform; the result is then meaningless): the caller runs
//   the work item again with pass2, where every candidate is gated before it counts.  The
//   retry lives in the callers' own work loops, so the sweep's code is not wrapped in a second
//   loop (that cost 12 spilled VGPRs in k_trace).
template <bool PREFILTER, bool LT3 = true, int HBM1 = 0>
__device__ __forceinline__ bool shadow_lit_single(const FrameArgs& fa, const double* __restrict__ lds, bool resident,
                                                  uint32_t* __restrict__ stk, V3 hit, V3 o, V3 d, V3 lpos, uint32_t li,
                                                  bool lane_on, Visits& vis, bool pass2, bool& redo,
                                                  const ViewLeaf* vt = nullptr, uint32_t vn = 0,
                                                  const ViewHead* vh = nullptr) {
    const DevObject& ob = fa.obj[0];
    const V3 pos{ob.pos[0], ob.pos[1], ob.pos[2]};
    const V3 ro = sub(o, pos);  // object.go:71
    const V3 neg = scale(d, -1);
    const double lh = len(sub(lpos, hit));
    const double mag = fmax(fmax(fmax(__builtin_fabs(o.x), __builtin_fabs(o.y)), __builtin_fabs(o.z)),
                            fmax(fmax(__builtin_fabs(pos.x), __builtin_fabs(pos.y)), __builtin_fabs(pos.z)));
    const double M = 0x1p-36 * (1.0 + lh + mag);
    const double resolve = lh - 1e-4 - M;
    const float tmax = (float)(lh + 1e-4 + M) * (1.0f + 0x1p-20f);
    const bool gating = MIRT_BOX_GATE && !(fa.flags & MIRT_OPT_NO_BOX_GATE);
    redo = false;
    Best b;
    best_init(b);
    // Culling cone: the packet's rays walked backwards from the light, L + s * (-d), over
    // s in [-(2e-4 + M), lh]: it covers o + t * d for t in [0, tmax] (o, L and d are
    // collinear up to fp64 rounding, far inside the box inflation).
    const Ray32 r = ray32(ro, d);
    const double far = fmax(fmax(__builtin_fabs(ro.x), __builtin_fabs(ro.y)), __builtin_fabs(ro.z));
    const bool force = !(far <= ob.m.cull_limit);
    const float smin = -(float)(2e-4 + M) * (1.0f + 0x1p-20f);
    const float smax = (float)lh * (1.0f + 0x1p-20f);
    Cone cone;
    if (MIRT_SHADOW_WIDE) cone = make_cone(sub(lpos, pos), -r.ix, -r.iy, -r.iz, lane_on, force, smin, smax, ob.m.cull_limit);
    if (pass2) {
        // every candidate gated (as trace_nearest's pass 2): an LDS-resident mesh swept whole,
        // an HBM mesh through its BVH
        if (resident)
            test_range<false, PREFILTER, 8, true, false, true>(lds, ob.m.fidx, 0, ob.m.ntri, ro, d, neg, b, vis.tests,
                                                             nullptr, nullptr, lane_on, mesh_fbox(ob.m));
        else
            bvh_sweep<false, PREFILTER, true, LT3, true>(ob.m, (cdptr)ob.m.tri, ro, d, neg, lane_on, b, vis, tmax,
                                                         resolve, !(fa.flags & MIRT_OPT_NO_OCTANT), nullptr, nullptr,
                                                         mesh_fbox(ob.m), false);
    } else if (MIRT_SHADOW_WIDE) {
        if (resident)
            bvh_wide<false, PREFILTER, true>(ob.m, lds, stk, cone, r, force, ro, d, neg, lane_on, b, vis, vis.overflow,
                                             tmax, resolve);
        else
            bvh_wide<false, PREFILTER, true>(ob.m, (cdptr)ob.m.tri, stk, cone, r, force, ro, d, neg, lane_on, b, vis,
                                             vis.overflow, tmax, resolve);
    } else if (resident && vt) {
        // the lane's direction from the light: its hit point relative to the view point (every
        // point of the segment short of the light lies in that direction)
        const double* R0 = vh->R[0];
        const double* R1 = vh->R[1];
        const double* R2 = vh->R[2];
        const V3 X = sub(sub(hit, pos), V3{vh->O[0], vh->O[1], vh->O[2]});
        const double z = R0[0] * X.x + R0[1] * X.y + R0[2] * X.z;
        const double mag = fmax(fmax(__builtin_fabs(X.x), __builtin_fabs(X.y)), __builtin_fabs(X.z));
        const bool unb = !(z > 0x1p-20 * mag);
        float ls = 0.0f, lt = 0.0f;
        if (!unb) {
            ls = (float)((R1[0] * X.x + R1[1] * X.y + R1[2] * X.z) / z);
            lt = (float)((R2[0] * X.x + R2[1] * X.y + R2[2] * X.z) / z);
        }
        const bool any_unb = __ballot(lane_on && unb) != 0;
        const float inf = __builtin_inff();
        float cs0 = -inf, cs1 = inf, ct0 = -inf, ct1 = inf;
        if (!any_unb) {
            const bool on = lane_on;
            cs0 = wave_reduce<true>(on ? ls : inf);
            cs1 = wave_reduce<false>(on ? ls : -inf);
            ct0 = wave_reduce<true>(on ? lt : inf);
            ct1 = wave_reduce<false>(on ? lt : -inf);
        }
        // a candidate of the segment lies within |L - hit| of the light (or within near_r)
        const float zl = (float)(lh + (double)vh->near_r) * (1.0f + 0x1p-20f);
        view_sweep<PREFILTER, true>(ob.m, lds, vt, vn, ls, lt, unb, cs0, cs1, ct0, ct1, zl, ro, d, neg, lane_on, b, vis,
                                    resolve, tmax);
    } else {
        // the light's fp32 table (SegPre): per lane d, |d|_inf and the distance along d
        const float* lt = fa.ltab && li < fa.n_lights ? fa.ltab + (size_t)li * fa.ltab_n * kLtD : nullptr;
        SegPre sp;
        if (lt) sp = seg_pre(d, lh);
        if (resident)
            bvh_sweep<false, PREFILTER, true, LT3>(ob.m, lds, ro, d, neg, lane_on, b, vis, tmax, resolve,
                                                  !(fa.flags & MIRT_OPT_NO_OCTANT), lt, &sp);
        else
            bvh_sweep<false, PREFILTER, true, LT3>(ob.m, (cdptr)ob.m.tri, ro, d, neg, lane_on, b, vis, tmax, resolve,
                                                  !(fa.flags & MIRT_OPT_NO_OCTANT), lt, &sp, nullptr, HBM1 == 2 && MIRT_STREAM_SHADOW);
    }
    if (gating) {
        uint32_t face = 0, p = 0;
        const bool retired = b.has() && b.d < resolve;
        const bool far_lit = !retired && b.has() && !b.any_nan() && b.d > lh + 1e-4 + M;
        const bool need = lane_on && best_result(b, face, p) && !far_lit;
        // the object's box (tracer.go:32), then, in a first pass, the face box the decision
        // rests on (object.go:76)
        const uint32_t fpos = retired ? b.pos : p;
        const bool ok = box_gate(Box6{{ob.box[0], ob.box[1], ob.box[2], ob.box[3], ob.box[4], ob.box[5]}}, o, d, need);
        bool fok = true;
        if (!pass2) {
            V3 o2 = o;  // (object-space origin made again here, not kept live through the sweep)
            asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
            fok = box_gate(box_load(at_use(mesh_fbox(ob.m)) + (size_t)fpos * kBoxD), sub(o2, pos), d, ok);
        }
        if (need && !ok) best_init(b);
        if (!pass2) {
            redo = __ballot(ok && (!fok || (!retired && b.any_nan()))) != 0;
            if (redo) diag(29);  // segment queries run again (pass 2)
            if (MIRT_BOX_GATE == 2) {  // measurement build: gates evaluated, no second pass
                vis.overflow += redo;
                redo = false;
            }
        }
    }
    if (b.has() && b.d < resolve) return false;
    // the nearest candidate (not a NaN-distance first hit, which wins regardless) lies beyond
    // lh + 1e-4 + M from o: the occluder is farther from hit than the light
    if (b.has() && !b.first_nan() && b.d > lh + 1e-4 + M) return true;
    uint32_t face, p;
    if (!best_result(b, face, p)) return true;
    V3 world, normal;
    uint32_t mat;
    V3 o3 = o;
    asm volatile("" : "+v"(o3.x), "+v"(o3.y), "+v"(o3.z));
    winner(ob, p, sub(o3, pos), d, scale(d, -1), world, normal, mat, false);
    return lh < len(sub(world, hit));
}
// shadow_lit_single with its retry in place, for callers that hold per-lane chain state
// (k_reflect, k_bounce with MIRT_BOUNCE_SHADE) rather than a work queue.
template <bool PREFILTER, bool LT3 = true, int HBM1 = 0>
__device__ __forceinline__ bool shadow_lit_single_settled(const FrameArgs& fa, const double* __restrict__ lds,
                                                          bool resident, uint32_t* __restrict__ stk, V3 hit, V3 o, V3 d,
                                                          V3 lpos, uint32_t li, bool lane_on, Visits& vis) {
    bool redo = false;
    bool lit = shadow_lit_single<PREFILTER, LT3, HBM1>(fa, lds, resident, stk, hit, o, d, lpos, li, lane_on, vis, false, redo);
    if (redo)
        lit = shadow_lit_single<PREFILTER, LT3, HBM1>(fa, lds, resident, stk, hit, o, d, lpos, li, lane_on, vis, true, redo);
    return lit;
}

// A hit pixel's packed word: uint8(255 c) per channel (colour.go:59-61), valid = 1.
__device__ __forceinline__ uint32_t pack_rgbv(const RGB& c) {
    return (uint32_t)c_u8(c.r) | ((uint32_t)c_u8(c.g) << 8) | ((uint32_t)c_u8(c.b) << 16) | (1u << 24);
}

// ---------------------------------------------------------------- Phong
// tracer.go:53-76 for one hit; bit l of lit = light l reaches the point.
__device__ __forceinline__ RGB phong(const FrameArgs& fa, const double* __restrict__ mt, V3 hit, V3 n, uint32_t lit) {
    RGB ka{mt[0], mt[1], mt[2]}, kd{mt[3], mt[4], mt[5]}, ks{mt[6], mt[7], mt[8]};
    const double ns = mt[9];
    const V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    RGB col = ka;  // tracer.go:56
    // tracer.go:66 does not depend on the light: computed once (same value for every light)
    const V3 camdir = lit ? norm(sub(cam, hit)) : V3{0, 0, 0};
    for (uint32_t l = 0; l < (MIRT_EXP_NO_PHONG ? 0u : fa.n_lights); ++l) {
        if (!((lit >> l) & 1u)) continue;
        const V3 lpos{fa.lpos[l][0], fa.lpos[l][1], fa.lpos[l][2]};
        const RGB lcol{fa.lcol[l][0], fa.lcol[l][1], fa.lcol[l][2]};
        const V3 ldir = norm(sub(lpos, hit));                         // tracer.go:61
        const V3 refl = sub(scale(n, 2 * dot(ldir, n)), ldir);        // tracer.go:65
        col = c_add(col, c_mul(c_scale(kd, go_max0(dot(ldir, n))), lcol));                // :69
        col = c_add(col, c_mul(c_scale(ks, go_pow(go_max0(dot(refl, camdir)), ns)), lcol));  // :72
    }
    return col;
}

// ---------------------------------------------------------------- frame statistics
// Called by every workgroup of the frame's last kernel after its statistics are flushed:
// the last workgroup (two-level done count, <= 64 same-address atomics per level) folds
// the statistic shards into WorkArgs::summary and the profiling accumulator.  Shards are
// read with atomics (device-coherent across the XCDs' L2s).
// The launch's last workgroup (the done counters, one atomic per workgroup and shard): true in
// every thread of that workgroup only.
__device__ __forceinline__ bool launch_last(const WorkArgs& wa) {
    __shared__ bool last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's statistics atomics performed
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t sh = blockIdx.x % kStatShards;
        const uint32_t in_shard = (gridDim.x - sh + kStatShards - 1) / kStatShards;
        bool l = atomicAdd(&wa.counters[cnt_done(sh)], (cnt_t)1) == (cnt_t)in_shard - 1;
        if (l) {
            const uint32_t shards = min((uint32_t)kStatShards, gridDim.x);
            l = atomicAdd(&wa.counters[cnt_done(kStatShards)], (cnt_t)1) == (cnt_t)shards - 1;
        }
        last = l;
    }
    __syncthreads();
    return last;
}
// The frame's statistics totals, by the launch's last workgroup.
template <bool FRESH = false>
__device__ __forceinline__ void frame_summary(const FrameArgs& fa, const WorkArgs& wa, bool last) {
    const uint32_t tid = tid_fresh<FRESH>();
    if (!last || tid >= kStatN) return;
    const int st = (int)tid;
    cnt_t sum = 0;
    for (int sh = 0; sh < kStatShards; ++sh)
        sum += atomicAdd(&wa.counters[cnt_stat(st == kStatShadowRays ? kStatHits : st, sh)], (cnt_t)0);
    if (st == kStatShadowRays) {  // one per light per primary hit, plus those of reflection hits
        sum *= fa.n_lights;
        for (int sh = 0; sh < kStatShards; ++sh)
            sum += atomicAdd(&wa.counters[cnt_stat(kStatReflShadowRays, sh)], (cnt_t)0);
    }
    wa.summary[st] = sum;
    if (wa.prof_acc && sum) atomicAdd(&wa.prof_acc[st], sum);
}
__device__ __forceinline__ void frame_fold(const FrameArgs& fa, const WorkArgs& wa) {
    frame_summary(fa, wa, launch_last(wa));
}

// ---------------------------------------------------------------- work distribution
// A wave serves queue shard q = (global wave id) % kQShards (several shards in turn when
// fewer than kQShards waves run).  dynamic: each ticket of the shard's counter is one work
// item, the next ticket is requested before the current item is traced so the atomic's
// latency hides behind the work; static: items q, q + kQShards, ... split round-robin
// among the waves of the shard (ablation).
struct ShardCursor {
    uint32_t gw, nw;  // global wave id, waves in the grid
    __device__ __forceinline__ ShardCursor() {
        // wave-uniform, said so: every index derived from it (shard, rank, item, chunk) then
        // lives in SGPRs instead of VGPRs held (and in k_shadow spilled) across the item loop
        gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (kWG / 64) + (threadIdx.x >> 6));
        nw = gridDim.x * (kWG / 64);
    }
    __device__ __forceinline__ uint32_t first_shard() const { return nw >= (uint32_t)kQShards ? gw % kQShards : gw; }
    __device__ __forceinline__ uint32_t shard_step() const { return nw >= (uint32_t)kQShards ? kQShards : nw; }
    // static mode: this wave's rank among the waves serving its shard, and their count
    __device__ __forceinline__ uint32_t rank() const { return nw >= (uint32_t)kQShards ? gw / kQShards : 0; }
    __device__ __forceinline__ uint32_t peers() const {
        if (nw < (uint32_t)kQShards) return 1;
        const uint32_t q = gw % kQShards;
        return nw / kQShards + (q < nw % kQShards ? 1 : 0);
    }
};
// MIRT_OPT_TIMELINE: per-wave stamps (mirt.h mirt_debug_timeline).
struct WaveClock {
    uint64_t real0, clk0, staged = 0;
    bool real0_override = false;
    uint64_t phase_setup = 0, phase_trace = 0;
    __device__ __forceinline__ WaveClock() {
        real0 = __builtin_amdgcn_s_memrealtime();
        clk0 = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void mark_staged() { staged = __builtin_amdgcn_s_memrealtime(); }
    __device__ __forceinline__ void record(const WorkArgs& wa, uint32_t kernel, uint32_t items) const {
        const uint64_t real1 = __builtin_amdgcn_s_memrealtime(), clk1 = __builtin_amdgcn_s_memtime();
        const uint32_t gw = blockIdx.x * (kWG / 64) + wave_id();
        const uint32_t lane = threadIdx.x & 63;
        if (gw >= wa.timeline_cap || lane >= kTimelineRec) return;
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
        const uint64_t v[kTimelineRec] = {kernel, gw, real0, real1, real0_override ? phase_setup : clk0,
                                          real0_override ? phase_trace : clk1, staged, xcc | ((uint64_t)items << 32)};
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < kTimelineRec; ++k) x = lane == (uint32_t)k ? v[k] : x;
        wa.timeline[((size_t)kernel * wa.timeline_cap + gw) * kTimelineRec + lane] = x;
    }
};

// MIRT_ITEM_TRACE (diagnostic builds only, with MIRT_OPT_TIMELINE): one record per work
// item of k_trace instead of one per wave — {kind, workgroup, start, end (100 MHz), start,
// end (shader clock), wave tests, nodes | hits << 32} — appended through a counter held in
// the buffer's first record (tools/item_trace.py).
struct ItemClock {
    uint64_t real0 = 0, clk0 = 0;
    __device__ __forceinline__ void start() {
        if (MIRT_ITEM_TRACE) {
            real0 = __builtin_amdgcn_s_memrealtime();
            clk0 = __builtin_amdgcn_s_memtime();
        }
    }
    uint32_t k = 0;  // records written by this wave (fixed region of kItemRecs per wave: no atomics)
    static constexpr uint32_t kItemRecs = 32;
    __device__ __forceinline__ void record(const WorkArgs& wa, uint32_t kind, uint64_t tests, uint64_t nodes,
                                           uint64_t hits, uint64_t phases = 0) {
        if (!MIRT_ITEM_TRACE || !wa.timeline) return;
        const uint64_t real1 = __builtin_amdgcn_s_memrealtime(), clk1 = __builtin_amdgcn_s_memtime();
        const uint32_t lane = threadIdx.x & 63;
        const uint32_t gw = blockIdx.x * (kWG / 64) + wave_id();
        const uint32_t idx = gw * kItemRecs + k;
        ++k;
        if (k > kItemRecs || idx >= 2 * wa.timeline_cap || lane >= kTimelineRec) return;
        const uint64_t v[kTimelineRec] = {kind, blockIdx.x, real0, real1, clk1 - clk0, phases, tests, nodes | (hits << 32)};
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < kTimelineRec; ++k) x = lane == (uint32_t)k ? v[k] : x;
        wa.timeline[(size_t)idx * kTimelineRec + lane] = x;
    }
};

// One ticket of counter c, issued by lane 0; resolve() broadcasts it (waits for the atomic).
// Queue, hit-slot and primary-done counters are used through the low 32-bit word of
// their line: a 32-bit returning atomic lands in one VGPR (a 64-bit one whose unused high
// half gets reused forces an immediate wait for the atomic).
__device__ __forceinline__ uint32_t* lo32(cnt_t* c) { return (uint32_t*)c; }
__device__ __forceinline__ uint32_t ticket_issue(cnt_t* c) {
    uint32_t t = 0;
    if ((threadIdx.x & 63) == 0) t = atomicAdd(lo32(c), 1u);
    return t;
}
__device__ __forceinline__ uint32_t ticket_resolve(uint32_t t) { return __builtin_amdgcn_readfirstlane(t); }
// Work items of shard q when item k of the shard is global item k * kQShards + q.
__device__ __forceinline__ uint32_t shard_items(uint32_t n, uint32_t q) {
    return n > q ? (n - q + kQShards - 1) / kQShards : 0u;
}

// ---------------------------------------------------------------- hit slots
// A HitRec is eight 64-bit words: h[3], n[3], out, obj | mat << 32.
__device__ __forceinline__ void st64(uint64_t* p, uint64_t v) { *p = v; }
// A constant made at its store (as store_black's zero): k_primary had hoisted the miss slot's
// kNoHit word and the -1 of the face and object planes out of its loops and spilled them.
template <typename T>
__device__ __forceinline__ T at_store(T v) {
    asm volatile("" : "+v"(v));
    return v;
}
// A miss's fp64 colour (three zeros), its zero made at the store: a zero hoisted out of the
// block loops would stay live across the traversal, and k_trace spilled it to scratch.
__device__ __forceinline__ void store_black(double* p) {
    uint64_t z = 0;
    asm volatile("" : "+v"(z));
    uint64_t* q = (uint64_t*)p;
    q[0] = z;
    q[1] = z;
    q[2] = z;
}
__device__ __forceinline__ uint64_t ld64(const uint64_t* p) { return *p; }
__device__ __forceinline__ void st32(uint32_t* p, uint32_t v) { *p = v; }
__device__ __forceinline__ double bitsd(uint64_t x) { return __longlong_as_double((long long)x); }

// Descriptor of block k of shard q (shard-major table; scalar load; zero if past the end).
__device__ __forceinline__ BlockDesc block_desc(const WorkArgs& wa, uint32_t q, uint32_t k) {
    // readfirstlane: the index is provably uniform, so this is one s_load_dwordx4 (lgkmcnt),
    // not a vector load whose vmcnt wait would also wait for the in-flight ticket atomic
    const uint32_t kk = __builtin_amdgcn_readfirstlane(min(k, wa.per_shard - 1));
    const uint32_t qq = __builtin_amdgcn_readfirstlane(q);
    const u32x4 v = ((cv4ptr)wa.blocks)[(size_t)qq * wa.per_shard + kk];
    return k < wa.per_shard ? BlockDesc{v[0], v[1], v[2], v[3]} : BlockDesc{0, 0, 0, 0};
}

// ---------------------------------------------------------------- block frustum
// Whole-block pre-test (one-object frames, mirt_internal.hpp FrustumArgs): the block's
// rays span s in [s(px + vw - 1), s(px)] and t in [t(py + vh - 1), t(py)]; lane c < 8
// checks that range against root child c's projected rectangle (staged in LDS).  A block
// none of whose rectangles it overlaps cannot hit the object.  Bit c set: child c may be
// met by a ray of the block.
__device__ __forceinline__ void stage_frustum(float4* __restrict__ rects, const FrustumArgs& fr) {
    if (threadIdx.x < 8)
        rects[threadIdx.x] = make_float4(fr.rect[threadIdx.x][0], fr.rect[threadIdx.x][1], fr.rect[threadIdx.x][2],
                                         fr.rect[threadIdx.x][3]);
}
__device__ __forceinline__ uint32_t block_frustum(const FrustumArgs& fr, const float4* __restrict__ rects,
                                                  uint32_t px, uint32_t py, uint32_t vw, uint32_t vh) {
    const uint32_t lane = threadIdx.x & 63;
    const float4 r = rects[lane & 7];
    const float s0 = (float)(fr.sB - fr.sA * (double)px), s1 = (float)(fr.sB - fr.sA * (double)(px + vw - 1));
    const float t0 = (float)(fr.tB - fr.tA * (double)py), t1 = (float)(fr.tB - fr.tA * (double)(py + vh - 1));
    const bool meet = lane < 8 && fminf(s0, s1) <= r.y && fmaxf(s0, s1) >= r.x && fminf(t0, t1) <= r.w &&
                      fmaxf(t0, t1) >= r.z;
    return (uint32_t)__ballot(meet);
}
// The same predicate evaluated by one thread over all 8 rectangles: true iff
// block_frustum(...) != 0 for that block.
__device__ __forceinline__ bool block_may_meet(const FrustumArgs& fr, const float4* __restrict__ rects, uint32_t px,
                                               uint32_t py, uint32_t vw, uint32_t vh) {
    const float s0 = (float)(fr.sB - fr.sA * (double)px), s1 = (float)(fr.sB - fr.sA * (double)(px + vw - 1));
    const float t0 = (float)(fr.tB - fr.tA * (double)py), t1 = (float)(fr.tB - fr.tA * (double)(py + vh - 1));
    bool meet = false;
    for (int c = 0; c < 8; ++c) {
        const float4 r = rects[c];
        meet |= fminf(s0, s1) <= r.y && fmaxf(s0, s1) >= r.x && fminf(t0, t1) <= r.w && fmaxf(t0, t1) >= r.z;
    }
    return meet;
}

// The object-box certificate (FrameRec::ocert, mirt.cpp object_cert): true iff the four
// corner directions of the block's (s, t) range lie inside one certificate quad, so every ray
// of the block passes the object's Box.Intersect (the quad is convex; its margin covers the
// difference between the affine (s, t) of a pixel here and the kernel's pixelToPoint).  One
// thread per block, at staging.
__device__ __forceinline__ bool block_obj_cert(const FrameRec& rec, uint32_t px, uint32_t py, uint32_t vw, uint32_t vh) {
    const FrustumArgs& fr = rec.fr;
    const double s0 = fr.sB - fr.sA * (double)px, s1 = fr.sB - fr.sA * (double)(px + vw - 1);
    const double t0 = fr.tB - fr.tA * (double)py, t1 = fr.tB - fr.tA * (double)(py + vh - 1);
    for (uint32_t q = 0; q < fr.ocert_n && q < kOcertQuads; ++q) {
        bool in = true;
        for (int k = 0; k < 4; ++k) {
            const double a = rec.ocert.h[q][k][0], b = rec.ocert.h[q][k][1], c = rec.ocert.h[q][k][2];
            in = in && a * s0 + b * t0 >= c && a * s0 + b * t1 >= c && a * s1 + b * t0 >= c && a * s1 + b * t1 >= c;
        }
        if (in) return true;
    }
    return false;
}

// ---------------------------------------------------------------- primary block
// One 8x8 pixel block: raygen (tracer.go:15-22, :86), nearest hit, outputs of misses,
// and, if any lane hit, 64 hit slots of region q (slot = lane) with their lit word and
// the block's light counter zeroed.  REL: the LDS mesh is stored relative to the camera.
// Hit chunks of a workgroup-local region (k_trace): LDS allocation counter and ready
// flags, slot index of the region's chunk 0.
struct LocalChunks {
    uint32_t* count;
    uint32_t* ready;
    size_t base;
    uint8_t* frame_of;  // per chunk: its frame within the launch (k_trace)
    uint32_t frame;
    uint32_t* ring;     // free positions of the hit-chunk ring (bit p: position p free)
    uint16_t* pos;      // per chunk: its position in the region (< kHitRing: a ring position)
    uint32_t* key;      // per chunk: its block's redo key (frame << 28 | block), redo_mark
};

// Hit-chunk ring (k_trace): a chunk takes the lowest free one of kHitRing positions of the
// workgroup's region and gives it back once shaded, so a frame's hit records dirty a few
// ring positions per workgroup instead of one fresh 4 KB chunk per hit block (the L2
// write-back of those lines was most of the frame's HBM writes).  A chunk that finds the
// ring full takes position kHitRing + its index in the batch (never shared).
__device__ __forceinline__ uint32_t ring_take(uint32_t* ring, uint32_t c) {
    uint32_t p = kHitRing + c;
    if (kHitRing > 0) {
        uint32_t m = __hip_atomic_load(ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (m) {
            const uint32_t b = __builtin_ctz(m), bit = 1u << b;
            const uint32_t old = atomicAnd(ring, ~bit);
            if (old & bit) {
                p = b;
                break;
            }
            m = old & ~bit;
        }
    }
    return p;
}
//   pass2 / returns: trace_nearest's retry.  true = the block must run again with pass2 (its
//   result rested on a face box that fails: nothing was written); false = done.
// The output word of a block's pixel (lx, ly): its packed index bd.out + lx * th + ly, or, for
// a share written in its transfer form (k_trace's FrameRec::xf, full-height strips: th = H),
// the word k_pack_rect would have copied it to; kNoOut for a pixel outside the hit rectangle.
// The primary ray's direction at pixel (i, j): tracer.go:15-22 pixelToPoint, then tracer.go:86
// (p - Cam.Pos).Norm(), in the reference's fp64 operations.  A is FrameArgs (k_primary, k_trace)
// or RayGen (k_pack at level 0, which makes the direction again instead of reading it): one
// function, so both get the same bits.
template <class A>
__device__ __forceinline__ V3 primary_dir(const A& a, uint32_t i, uint32_t j) {
    const V3 cam{a.cam[0], a.cam[1], a.cam[2]};
    const double si = a.phw * ((double)(a.halfW - (int32_t)i) - 0.5) / (double)a.halfW;
    const double sj = a.phh * ((double)(a.halfH - (int32_t)j) - 0.5) / (double)a.halfH;
    const V3 p = add(add(add(cam, V3{a.fwd[0], a.fwd[1], a.fwd[2]}), scale(V3{a.left[0], a.left[1], a.left[2]}, si)),
                     scale(V3{a.up[0], a.up[1], a.up[2]}, sj));
    return norm(sub(p, cam));
}
__device__ __forceinline__ uint64_t out_index(const XferArgs* xf, const BlockDesc& bd, uint32_t lx, uint32_t ly,
                                              uint32_t th) {
    if (!xf || !xf->on) return (uint64_t)bd.out + (uint64_t)lx * th + ly;
    const uint32_t i = (bd.pxy & 0xffffu) + lx, j = (bd.pxy >> 16) + ly;
    const uint32_t k0 = (bd.out - (bd.pxy >> 16)) / th;  // the block's first packed column
    if (i < xf->x0 || i >= xf->x1 || j < xf->y0 || j - xf->y0 >= xf->ch) return kNoOut;
    return (uint64_t)(k0 + lx - xf->k0) * xf->ch + (j - xf->y0);
}

template <bool REL, bool PREFILTER, bool BRUTE, int HBM1 = 0>
__device__ __forceinline__ bool primary_block(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out,
                                              const double* __restrict__ lds, uint32_t* __restrict__ stk, bool resident,
                                              const BlockDesc& bd, uint32_t q, WaveStats& ws, PhaseClock& pc,
                                              bool pass2, bool frustum = false, const float4* __restrict__ frect = nullptr,
                                              const LocalChunks* lc = nullptr, uint32_t classified = 0,
                                              const ViewLeaf* vt = nullptr, uint32_t vn = 0,
                                              const FrustumArgs* vfr = nullptr, uint32_t blk = ~0u,
                                              const XferArgs* xf = nullptr) {
    pc.start();
    const uint32_t lane = threadIdx.x & 63;
    const V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    const uint32_t lx = lane >> 3, ly = lane & 7;
    const uint32_t px = bd.pxy & 0xffffu, py = bd.pxy >> 16, th = bd.geo & 0xffffu;
    const uint32_t vw = (bd.geo >> 16) & 0xffu, vh = bd.geo >> 24;
    const bool active = lx < vw && ly < vh;
    // classified (k_trace staging, block_may_meet): 1 culled, 2 may meet, 0 test here; bit 4:
    // the block lies in the object-box certificate (block_obj_cert)
    if (frustum && ((classified & 3) == 1 || ((classified & 3) == 0 && block_frustum(wa.fr, frect, px, py, vw, vh) == 0))) {
        ++ws.nodes;
        diag(21);
        const uint64_t oidx = out_index(xf, bd, lx, ly, th);
        if (active && oidx != kNoOut && !MIRT_SKIP_MISS_STORES) {  // every ray misses (tracer.go:88-90: colour zero)
            if (out.valid) out.valid[oidx] = 0;
            if (out.face) out.face[oidx] = -1;
            if (out.object) out.object[oidx] = -1;
            if (out.rgb) store_black(out.rgb + 3 * oidx);
            if (out.rgb8) {
                out.rgb8[3 * oidx] = 0;
                out.rgb8[3 * oidx + 1] = 0;
                out.rgb8[3 * oidx + 2] = 0;
            }
            if (out.rgbv) out.rgbv[oidx] = 0u;
        }
        pc.lap(2);
        return false;
    }
    const uint32_t i = px + (active ? lx : 0), j = py + (active ? ly : 0);

    // tracer.go:15-22 pixelToPoint with the reference's fp64 operations (computed, not
    // loaded: a vector load here would wait for the previous block's stores, which share
    // its in-order memory counter), then tracer.go:86 (p - Cam.Pos).Norm()
    V3 d = primary_dir(fa, i, j);

    Visits vis{0, 0, 0, 0};
    // view table walk: the lane's direction (s_i, t_j) and the block's range (block_frustum's)
    float ls = 0.0f, lt = 0.0f;
    float4 crect{0.0f, 0.0f, 0.0f, 0.0f};
    if (vt) {
        ls = (float)(vfr->sB - vfr->sA * (double)i);
        lt = (float)(vfr->tB - vfr->tA * (double)j);
        const float s0 = (float)(vfr->sB - vfr->sA * (double)px), s1 = (float)(vfr->sB - vfr->sA * (double)(px + vw - 1));
        const float t0 = (float)(vfr->tB - vfr->tA * (double)py), t1 = (float)(vfr->tB - vfr->tA * (double)(py + vh - 1));
        crect = float4{fminf(s0, s1), fmaxf(s0, s1), fminf(t0, t1), fmaxf(t0, t1)};
    }
    pc.lap(0);
    bool redo = false;
    Nearest nh = trace_nearest<REL, PREFILTER, BRUTE, MIRT_PRIMARY_WIDE, HBM1>(fa, lds, resident, cam, d,
                                                                         active && !MIRT_EXP_NO_PRIMARY_TRACE, true, vis,
                                                                         pass2, redo, (classified & 4) != 0, stk, vt, vn, ls, lt, crect);
    pc.lap(1);
    ws.tests += (cnt_t)vis.tests * __popcll(__ballot(active));
    ws.nodes += vis.nodes;
    ws.leaves += vis.leaves;
    ws.overflow += vis.overflow;
    if (redo) return true;  // wave-uniform: nothing written yet

    const uint64_t oidx = out_index(xf, bd, lx, ly, th);
    const bool is_hit = active && nh.ok;
    // hit slots first: the slot allocation's returning atomic is waited for before this
    // block's output stores are issued (the wait would otherwise cover them too)
    const uint64_t mask = __ballot(is_hit);
    if (mask) {
        ws.hits += __popcll(mask);
        uint32_t base = 0, rp = 0;
        if (lane == 0) {
            if (lc) {
                base = atomicAdd(lc->count, 1u);
                rp = ring_take(lc->ring, base);
                lc->pos[base] = (uint16_t)rp;  // LDS, in order before the ready flag
                lc->key[base] = blk;
            } else {
                base = atomicAdd(lo32(&wa.counters[cnt_hits(q)]), 64u);
            }
        }
        base = __builtin_amdgcn_readfirstlane(base);
        rp = __builtin_amdgcn_readfirstlane(rp);
        // (the lane offset made here: base + lane hoisted out of the block loop stays live
        // across the traversal as a 64-bit pair, and k_trace spilled it to scratch)
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
        const size_t slot = lc ? (size_t)(lc->base + (size_t)rp * 64) + ln : (size_t)q * wa.hit_cap + base + lane;
        // bounce waves: the block's hit chunk, for k_pack's walk in block order
        if (!lc && wa.bmap && blk != ~0u && lane == 0) {
            wa.bmap[blk] = (uint32_t)(((size_t)q * wa.hit_cap + base) / 64 + 1) << 7 | (uint32_t)__popcll(mask);
            atomicAdd(&wa.bgcnt[blk / kPackGroup], (uint32_t)__popcll(mask));
        }
        uint64_t* w = (uint64_t*)&wa.hits[slot];
        // the chunk's hit ballot (split kernels): its missed lanes write nothing below
        const bool ballot = !lc && wa.hmask;
        if (ballot && lane == 0) st64(&wa.hmask[slot / 64], mask);
        if (is_hit) {
            st64(w + 0, dbits(nh.hit.x));
            st64(w + 1, dbits(nh.hit.y));
            st64(w + 2, dbits(nh.hit.z));
            st64(w + 3, dbits(nh.normal.x));
            st64(w + 4, dbits(nh.normal.y));
            st64(w + 5, dbits(nh.normal.z));
            st64(w + 6, oidx);
            st64(w + 7, (uint64_t)nh.obj | ((uint64_t)nh.mat << 32));
            // the reflect kernel's incoming D (reflection frames run the split kernels: k_trace,
            // the caller with local chunks, never sees one, launch_frames)
            if (!lc && wa.bounces && wa.dir0) vstore(wa.dir0 + 3 * slot, d);  // (chains: k_reflect reads it)
        } else if (!ballot) {
            st64(w + 7, at_store((uint64_t)kNoHit));
        }
        if (is_hit || !ballot) st32(&wa.litw[slot], 0u);
        if (lane == 0) st32(&wa.blkdone[slot / 64], 0u);
        if (lc) {
            // publish to the workgroup: the chunk's stores have reached L2 (shared by every
            // wave of this CU) before its ready flag is raised in LDS
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                lc->frame_of[base] = (uint8_t)lc->frame;  // LDS, in order before the flag
                __hip_atomic_store(&lc->ready[base], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    if (active && oidx != kNoOut) {
        if (out.valid) out.valid[oidx] = is_hit ? 1 : 0;
        if (out.face) out.face[oidx] = is_hit ? (int32_t)nh.face : at_store(-1);
        if (out.object) out.object[oidx] = is_hit ? (int32_t)nh.obj : at_store(-1);
        if (!is_hit) {
            if (out.rgb) store_black(out.rgb + 3 * oidx);
            if (out.rgb8) {
                out.rgb8[3 * oidx] = 0;
                out.rgb8[3 * oidx + 1] = 0;
                out.rgb8[3 * oidx + 2] = 0;
            }
            if (out.rgbv) out.rgbv[oidx] = 0u;  // a hit's word is written by the wave that shades it
        }
    }
    pc.lap(2);
    return false;
}

// ---------------------------------------------------------------- view tables (ViewLeaf)
// the float next to finite f towards -inf / +inf
__device__ __forceinline__ float f32_prev(float f) {
    const uint32_t b = __float_as_uint(f);
    return f == 0.0f ? -0x1p-149f : __uint_as_float((int32_t)b > 0 ? b - 1u : b + 1u);
}
__device__ __forceinline__ float f32_next(float f) { return -f32_prev(-f); }
// x rounded to float downwards / upwards (NaN stays NaN)
__device__ __forceinline__ float f32_down(double x) {
    const float f = (float)x;
    return ((double)f > x && __builtin_isfinite(f)) ? f32_prev(f) : ((double)f > x ? 0x1.fffffep127f : f);
}
__device__ __forceinline__ float f32_up(double x) {
    const float f = (float)x;
    return ((double)f < x && __builtin_isfinite(f)) ? f32_next(f) : ((double)f < x ? -0x1.fffffep127f : f);
}
__device__ __forceinline__ void cross3(const double* a, const double* b, double* r) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = a[2] * b[0] - a[0] * b[2];
    r[2] = a[0] * b[1] - a[1] * b[0];
}
// R = [F L U]^-1 by cofactors (row k: column k+1 x column k+2, / det), as the host's
// frustum_args; false for a basis far from orthonormal.
__device__ bool view_rows(const double F[3], const double L[3], const double U[3], double R[3][3]) {
    cross3(L, U, R[0]);
    cross3(U, F, R[1]);
    cross3(F, L, R[2]);
    const double det = F[0] * R[0][0] + F[1] * R[0][1] + F[2] * R[0][2];
    if (!(__builtin_fabs(det) > 0.5) || !(__builtin_fabs(det) < 2.0)) return false;
    for (int k = 0; k < 3; ++k)
        for (int a = 0; a < 3; ++a) R[k][a] /= det;
    return true;
}
// One workgroup per (frame, view): the view's basis and point, every leaf's rectangle of
// directions and distance, the table sorted by distance (bitonic, in the LDS scratch), then
// published: every thread's stores fenced at agent scope, then the header's tag stored with
// release semantics (readers: view_ready).  Conditions as the host's
// frustum pre-test: the view point within the mesh's cull limit and below 2^30, a box
// entirely in front (every corner at z > 2^-20 |X|) gets its corners' bounding rectangle
// widened by 2^-18 (1 + |x|), a box entirely behind the camera is never met, anything else
// (and, for a light, any box within near_r of it: a shadow segment ends 1e-4 past the light)
// gets every direction.
constexpr uint32_t kViewSort = kMaxViewLeaves;
// k_trace's queue buckets: unknown cost, 8 log2 classes of the last primary trace time
// (units of 64 shader cycles; >= 2^12, i.e. >= ~110 us, first), and the culled blocks.
constexpr int kQueueBuckets = 10;
struct ViewScratch {
    ViewLeaf tmp[kViewSort];
    float key[kViewSort];
    uint32_t idx[kViewSort];
    double R[3][3], O[3];
    uint32_t ok;
    float near_r;
};
constexpr size_t kViewScratchBytes = sizeof(ViewScratch);
__device__ void build_view(const FrameRec& rec, uint32_t v, ViewLeaf* __restrict__ out, ViewHead* __restrict__ head,
                           void* scratch, uint32_t tag) {
    ViewScratch& sc = *(ViewScratch*)scratch;
    float* const key = sc.key;
    uint32_t* const idx = sc.idx;
    ViewLeaf* const tmp = sc.tmp;
    double (*const sR)[3] = sc.R;
    double* const sO = sc.O;
    const FrameArgs& fa = rec.fa;
    const DevMesh& m = fa.obj[0].m;
    const uint32_t n = m.nleaves;
    if (threadIdx.x == 0) {
        double O[3], big = 0.0, far = 0.0;
        const double* P = v == 0 ? fa.cam : fa.lpos[v - 1];
        for (int k = 0; k < 3; ++k) {
            O[k] = P[k] - fa.obj[0].pos[k];
            big = fmax(big, fmax(__builtin_fabs(P[k]), __builtin_fabs(fa.obj[0].pos[k])));
            far = fmax(far, __builtin_fabs(O[k]));
        }
        bool ok = far <= m.cull_limit && big <= 0x1p30 && n <= kMaxViewLeaves && (v > 0 || rec.fr.on);
        double R[3][3] = {};
        if (ok && v == 0) {
            ok = view_rows(fa.fwd, fa.left, fa.up, R);
        } else if (ok) {  // a light: look from it at the mesh's centre
            const double* mc = mesh_center(m);
            double F[3] = {mc[0] - O[0], mc[1] - O[1], mc[2] - O[2]};
            const double fl = sqrt(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]);
            if (fl > 0x1p-40 * (1.0 + far)) {
                for (int k = 0; k < 3; ++k) F[k] /= fl;
            } else {
                F[0] = 0.0, F[1] = 0.0, F[2] = 1.0;
            }
            const int a = (__builtin_fabs(F[0]) <= __builtin_fabs(F[1]) && __builtin_fabs(F[0]) <= __builtin_fabs(F[2])) ? 0
                          : (__builtin_fabs(F[1]) <= __builtin_fabs(F[2]) ? 1 : 2);
            const double A[3] = {a == 0 ? 1.0 : 0.0, a == 1 ? 1.0 : 0.0, a == 2 ? 1.0 : 0.0};
            double Lb[3], U[3];
            cross3(A, F, Lb);
            const double ll = sqrt(Lb[0] * Lb[0] + Lb[1] * Lb[1] + Lb[2] * Lb[2]);
            for (int k = 0; k < 3; ++k) Lb[k] /= ll;
            cross3(F, Lb, U);
            ok = view_rows(F, Lb, U, R);
        }
        for (int k = 0; k < 3; ++k) {
            sO[k] = O[k];
            for (int a = 0; a < 3; ++a) sR[k][a] = R[k][a];
        }
        sc.ok = ok ? 1u : 0u;
        sc.near_r = v == 0 ? 0.0f : f32_up(2.5e-4 + 0x1p-26 * (1.0 + far + m.cull_limit));
        head->ok = sc.ok;
        head->near_r = sc.near_r;
        for (int k = 0; k < 3; ++k) {
            head->O[k] = O[k];
            for (int a = 0; a < 3; ++a) head->R[k][a] = R[k][a];
        }
    }
    __syncthreads();
    const float inf = __builtin_inff();
    const float s_near = sc.near_r;
    uint32_t n2 = 1;
    while (n2 < n) n2 <<= 1;
    const uint32_t nt = sc.ok ? n2 : 0u;  // an unusable view publishes its header only
    for (uint32_t j = threadIdx.x; j < nt; j += blockDim.x) {
        if (j >= n) {
            key[j] = inf;
            idx[j] = 0xffffffffu;
            continue;
        }
        const LeafBox lb = m.leaves[j];
        double slo = inf, shi = -inf, tlo = inf, thi = -inf, d2 = 0.0;
        int front = 0, behind = 0;
        for (int a = 0; a < 3; ++a) {
            const double g = fmax(fmax((double)lb.lo[a] - sO[a], 0.0), sO[a] - (double)lb.hi[a]);
            d2 += g * g;
        }
        for (int k = 0; k < 8; ++k) {
            const double X[3] = {(double)((k & 1) ? lb.hi[0] : lb.lo[0]) - sO[0],
                                 (double)((k & 2) ? lb.hi[1] : lb.lo[1]) - sO[1],
                                 (double)((k & 4) ? lb.hi[2] : lb.lo[2]) - sO[2]};
            const double mag = fmax(fmax(__builtin_fabs(X[0]), __builtin_fabs(X[1])), __builtin_fabs(X[2]));
            const double z = sR[0][0] * X[0] + sR[0][1] * X[1] + sR[0][2] * X[2];
            if (z > 0x1p-20 * mag) {
                ++front;
                const double ss = (sR[1][0] * X[0] + sR[1][1] * X[1] + sR[1][2] * X[2]) / z;
                const double tt = (sR[2][0] * X[0] + sR[2][1] * X[1] + sR[2][2] * X[2]) / z;
                slo = fmin(slo, ss);
                shi = fmax(shi, ss);
                tlo = fmin(tlo, tt);
                thi = fmax(thi, tt);
            } else if (z < 0.0) {
                ++behind;
            }
        }
        ViewLeaf r;
        r.ref = lb.ref;
        r.pad[0] = j;  // the leaf's box: DevMesh::leaves[j]
        r.pad[1] = 0;
        const float dmin = f32_down(sqrt(d2) * (1.0 - 0x1p-30));
        r.dmin = dmin;
        const bool never = v == 0 && behind == 8;
        const bool every = front < 8 || !(__builtin_fabs(slo) + __builtin_fabs(shi) + __builtin_fabs(tlo) +
                                              __builtin_fabs(thi) < 0x1p60) ||
                           (v > 0 && dmin <= s_near);
        if (never) {
            r.dmin = inf;
            r.s0 = r.t0 = inf;
            r.s1 = r.t1 = -inf;
        } else if (every) {
            r.s0 = r.t0 = -inf;
            r.s1 = r.t1 = inf;
        } else {
            r.s0 = f32_down(slo - 0x1p-18 * (1.0 + __builtin_fabs(slo)));
            r.s1 = f32_up(shi + 0x1p-18 * (1.0 + __builtin_fabs(shi)));
            r.t0 = f32_down(tlo - 0x1p-18 * (1.0 + __builtin_fabs(tlo)));
            r.t1 = f32_up(thi + 0x1p-18 * (1.0 + __builtin_fabs(thi)));
        }
        tmp[j] = r;
        key[j] = r.dmin;
        idx[j] = j;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= nt; k <<= 1)  // bitonic sort by distance, ascending
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (uint32_t i = threadIdx.x; i < n2; i += blockDim.x) {
                const uint32_t x = i ^ jj;
                if (x > i) {
                    const bool up = (i & k) == 0;
                    const bool gt = key[i] > key[x] || (key[i] == key[x] && idx[i] > idx[x]);
                    if (gt == up) {
                        const float tk = key[i];
                        key[i] = key[x];
                        key[x] = tk;
                        const uint32_t ti = idx[i];
                        idx[i] = idx[x];
                        idx[x] = ti;
                    }
                }
            }
            __syncthreads();
        }
    if (sc.ok)
        for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) out[j] = tmp[idx[j]];
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&head->tag, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// The workgroup's copies of the launch's view headers (k_trace's LDS): state 0 = not seen
// published yet, 1 = published and usable, 2 = published, not usable.
struct ViewCache {
    ViewHead* head;
    uint32_t* state;
};
// Table q of this launch if it is published and usable, else nullptr (the caller walks the
// BVH).  The first wave of a workgroup to see the builder's tag (an agent-scope acquire
// after it) copies the header into the workgroup's LDS and publishes that to its peers; the
// table itself is read after that acquire.
__device__ __forceinline__ const ViewHead* view_lookup(const WorkArgs& wa, uint32_t q, const ViewCache& vc) {
    uint32_t st = __hip_atomic_load(&vc.state[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (st == 0) {
        if (__hip_atomic_load(&wa.view_heads[q].tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != wa.view_tag)
            return nullptr;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        // lanes 0..9 copy one 8-byte word of ok / near_r / R / O each, past the scalar cache
        const uint32_t lane = threadIdx.x & 63;
        const unsigned long long* src = (const unsigned long long*)&wa.view_heads[q];
        unsigned long long* dst = (unsigned long long*)&vc.head[q];
        constexpr uint32_t kWords = sizeof(ViewHead) / 8;
        if (lane < kWords)
            dst[lane] = __hip_atomic_load((unsigned long long*)src + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st = __hip_atomic_load((uint32_t*)&wa.view_heads[q].ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 1u : 2u;
        __hip_atomic_store(&vc.state[q], st, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return st == 1 ? &vc.head[q] : nullptr;
}




// ---------------------------------------------------------------- deferred second passes
// k_trace's second passes never run inside its work loop, whose registers and
// code they would take (an inlined second pass cost ~5% of the frame, one out of line ~11 MB
// of scratch traffic per frame, although neither runs on the benchmark's scenes).  A block
// whose primary first pass asks for one is recorded and skipped; a shadow item that asks for
// one records its chunk's block and publishes its first-pass bit (the block's pixels are all
// recomputed).  The launch's last workgroup then traces every recorded block again from its
// pixels, every query with its second pass in place (redo_block), and overwrites its outputs.
// Keys: frame << 28 | block index in the frame's table.  Flags (WorkArgs::bmap) dedupe the
// list (WorkArgs::bgcnt); device-scope atomics throughout (the list crosses XCDs).
__device__ __forceinline__ void redo_mark(const WorkArgs& wa, uint32_t key) {
    if ((threadIdx.x & 63) == 0) {
        const uint32_t fi = (key >> 28) * wa.nblocks_frame + (key & 0x0fffffffu);
        if (__hip_atomic_fetch_or(&wa.bmap[fi], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
            const uint32_t i = __hip_atomic_fetch_add(&wa.bgcnt[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&wa.bgcnt[1 + i], key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------- shadow item
// 64 hit slots (chunk c of region q) x light l: shadow rays from hit + 1e-4 L
// (tracer.go:61-64), the lit bit published by atomicOr, and Phong (tracer.go:53-76) by
// the wave that finishes the chunk's last light.  n_lights == 0: one pass that shades.
//   vf: the chunk's frame within the launch (its view tables, k_trace), ~0u: none.
//   pass2 / returns: shadow_lit_single's retry.  true = the item must run again with pass2
//   (nothing was published: no lit bit, no count, no shading); false = done.
template <bool PREFILTER, bool BRUTE, bool LT3 = true, int HBM1 = 0, bool SPLIT = false>
__device__ __forceinline__ bool shadow_item(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out,
                                            const double* __restrict__ lds, uint32_t* __restrict__ stk, bool resident,
                                            bool segment, size_t chunk, uint32_t l, WaveStats& ws, bool pass2,
                                            uint32_t vf = ~0u, const ViewCache* vc = nullptr, uint32_t lim = 64,
                                            uint32_t* ring = nullptr, uint32_t rpos = ~0u, uint32_t defer = ~0u) {
    // (a fresh lane index: its derived per-lane offsets are recomputed per item instead of being
    // hoisted out of the caller's item loop and held, or spilled, across every item)
    const uint32_t lane = tid_fresh<true>() & 63;
    const uint32_t nl = max(fa.n_lights, 1u);
    const size_t slot = chunk + lane;
    const uint64_t* w = (const uint64_t*)&wa.hits[slot];
    // lim: the chunk's records (a bounce level's last chunk of a region is partial); a chunk
    // with a hit ballot (WorkArgs::hmask) has no record at its missed lanes
    bool active;
    if (SPLIT && wa.hmask) {  // (k_shadow only: k_trace's chunks carry no ballot)
        const uint64_t hm = u64_uniform(wa.hmask[chunk / 64]);
        active = lane < lim && ((hm >> lane) & 1u);
    } else {
        active = lane < lim && (uint32_t)ld64(w + 7) != kNoHit;
    }
    V3 o{0, 0, 0}, d{1, 0, 0}, hit{0, 0, 0};
    const V3 lpos{fa.lpos[l][0], fa.lpos[l][1], fa.lpos[l][2]};
    if (active) {
        hit = V3{bitsd(ld64(w)), bitsd(ld64(w + 1)), bitsd(ld64(w + 2))};
        V3 ldir = norm(sub(lpos, hit));     // tracer.go:61
        o = add(hit, scale(ldir, 0.0001));  // tracer.go:64
        d = ldir;
    }
    Visits vis{0, 0, 0, 0};
    bool is_lit = false;
    if (fa.n_lights == 0) {
        // no lights: nothing to trace, the pass only shades (ambient)
    } else if (MIRT_EXP_NO_SHADOW_TRACE) {
        is_lit = true;
    } else if (segment) {
        const ViewLeaf* vt = nullptr;
        const ViewHead* vh = nullptr;
        if (vf != ~0u && wa.views && vc) {
            const uint32_t q = vf * wa.nviews + 1 + l;
            vh = view_lookup(wa, q, *vc);
            if (vh) vt = wa.views + (size_t)q * wa.view_leaves;
        }
        bool redo = false;
        is_lit = shadow_lit_single<PREFILTER, LT3, HBM1>(fa, lds, resident, stk, hit, o, d, lpos, l, active, vis, pass2, redo, vt,
                                                   wa.view_leaves, vh);
        if (redo && defer != ~0u) {  // k_trace: the block is traced again at the launch's end
            redo_mark(wa, defer);
            redo = false;
        }
        if (redo) {  // wave-uniform; the first pass's visits still count
            ws.tests += (cnt_t)vis.tests * __popcll(__ballot(active));
            ws.nodes += vis.nodes;
            ws.leaves += vis.leaves;
            ws.overflow += vis.overflow;
            return true;
        }
    } else {
        bool redo = false;
        Nearest r = trace_nearest<false, PREFILTER, BRUTE, false, HBM1>(fa, lds, resident, o, d, active, false, vis, pass2,
                                                                          redo);
        if (redo && defer != ~0u) {  // k_trace: the block is traced again at the launch's end
            redo_mark(wa, defer);
            redo = false;
        }
        if (redo) {  // wave-uniform: the item runs again with pass2 (nothing published)
            ws.tests += (cnt_t)vis.tests * __popcll(__ballot(active));
            ws.nodes += vis.nodes;
            ws.leaves += vis.leaves;
            ws.overflow += vis.overflow;
            return true;
        }
        // tracer.go:64: lit iff !shaded || |L - hit| < |occluder - hit|
        is_lit = !r.ok || len(sub(lpos, hit)) < len(sub(r.hit, hit));
    }
    ws.tests += (cnt_t)vis.tests * __popcll(__ballot(active));
    ws.nodes += vis.nodes;
    ws.leaves += vis.leaves;
    ws.overflow += vis.overflow;
    // publish this light's bit, then count the light done for the chunk; device-scope
    // atomics are coherent across XCDs and the wait orders the two atomics (the slot index is
    // recomputed here: nothing of the item's start stays live across the traversal)
    const size_t slot_b = chunk + (tid_fresh<true>() & 63);
    if (active && is_lit) {
        const uint32_t old =
            __hip_atomic_fetch_or(&wa.litw[slot_b], 1u << l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(old));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t done = 0;
    if (lane == 0) done = atomicAdd(&wa.blkdone[chunk / 64], 1u);
    done = __builtin_amdgcn_readfirstlane(done);
    if (done != nl - 1) return false;
    // Phong of the lane's hit (tracer.go:53-76) once its lit word is complete, and its outputs.
    // The record is read again here (hit point and obj | mat too, through a slot index the
    // compiler cannot reuse from the item's start): none of it stays live across the traversal,
    // which in k_shadow had spilled it to scratch.
    auto shade = [&](uint64_t& oidx) {
        const size_t s2 = chunk + (tid_fresh<true>() & 63);
        const uint64_t* w2 = (const uint64_t*)&wa.hits[s2];
        const uint32_t lit = atomicOr(&wa.litw[s2], 0u);
        const V3 h2{bitsd(ld64(w2)), bitsd(ld64(w2 + 1)), bitsd(ld64(w2 + 2))};
        const V3 n{bitsd(ld64(w2 + 3)), bitsd(ld64(w2 + 4)), bitsd(ld64(w2 + 5))};
        oidx = ld64(w2 + 6);
        const uint64_t w7b = ld64(w2 + 7);
        const uint32_t obj = (uint32_t)w7b, mat = (uint32_t)(w7b >> 32);
        return phong(fa, fa.obj[obj].m.mats + (size_t)mat * 10, h2, n, lit);
    };
    auto store = [&](uint64_t oidx, const RGB& col) {
        // k_trace (ring != nullptr) of a share in its transfer form: a hit lies inside its
        // frame's hit rectangle, so this is never taken (the split kernels have no such frames)
        if (ring && oidx == kNoOut) return;
        if (wa.bounces) {  // the level's phong: the reflection fold combines the levels and writes the pixel
            double* e = wa.ph_out + (wa.ph_by_origin ? (size_t)oidx : slot_b) * wa.ph_stride;
            e[0] = col.r;
            e[1] = col.g;
            e[2] = col.b;
            return;
        }
        if (out.rgb) {
            out.rgb[3 * oidx] = col.r;
            out.rgb[3 * oidx + 1] = col.g;
            out.rgb[3 * oidx + 2] = col.b;
        }
        if (out.rgb8) {
            out.rgb8[3 * oidx] = c_u8(col.r);
            out.rgb8[3 * oidx + 1] = c_u8(col.g);
            out.rgb8[3 * oidx + 2] = c_u8(col.b);
        }
        if (out.rgbv) out.rgbv[oidx] = pack_rgbv(col);
    };
    // ring (k_trace): the position goes back to the workgroup's ring once every access to the
    // chunk has completed: the other lights' waves counted themselves done after theirs, and
    // this wave's loads were consumed by phong (the wait has nothing else to wait for: the
    // output stores are issued after the release)
    if (ring && rpos < kHitRing) {
        RGB col{0, 0, 0};
        uint64_t oidx = 0;
        if (active) col = shade(oidx);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) atomicOr(ring, 1u << rpos);
        if (active) store(oidx, col);
        return false;
    }
    if (!active) return false;
    uint64_t oidx = 0;
    const RGB col = shade(oidx);
    store(oidx, col);
    return false;
}

// ---------------------------------------------------------------- primary kernel
// RESIDENT (host-decided): one object whose mesh fits in LDS; it is staged once per
// persistent workgroup, relative to the camera (p1or), and every sweep reads LDS.
// Out-of-line second passes (see k_trace's): helpers.
template <typename T>
__device__ __forceinline__ T* uni_ptr(T* p) {
    return (T*)u64_uniform((uint64_t)p);
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ void stats_add(WaveStats& a, const WaveStats& b) {
    a.tests += b.tests;
    a.nodes += b.nodes;
    a.leaves += b.leaves;
    a.hits += b.hits;
    a.overflow += b.overflow;
}

// Kernel arguments: the split kernels take theirs by value (the compiler places them); k_trace
// reads its records and its second and third arguments at the offsets kTraceWaOffset /
// kTraceFcOffset below, which tests/test_kernarg_layout.py checks against the code object's
// metadata.  A segment past 4 KB is not a hazard: the vertex-light soups pass with FrameArgs
// 32 and 224 bytes larger (split kernels' segments of 4096 and 4288 bytes).
constexpr size_t kalign(size_t x, size_t a) { return (x + a - 1) & ~(a - 1); }

// The split kernels' deferred second passes (as k_trace's): a work item whose
// first pass asks for one records itself (two words) and publishes nothing; the launch's last
// workgroup runs every recorded item again with the second pass in place, after its own work.
// WorkArgs::split_redo: [0] workgroups done, [1] entries, then the entries; the last
// workgroup zeroes both counts, so the buffer is clean for the next launch.
__device__ __forceinline__ void split_redo_push(const WorkArgs& wa, uint32_t a, uint32_t b) {
    if ((threadIdx.x & 63) == 0) {
        const uint32_t i = __hip_atomic_fetch_add(&wa.split_redo[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&wa.split_redo[2 + 2 * i], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&wa.split_redo[3 + 2 * i], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// Called once by every workgroup after its work: true in the launch's last one, which then
// reads the entries (n = the count, or 0 elsewhere).
__device__ __forceinline__ uint32_t split_redo_last(const WorkArgs& wa) {
    __shared__ uint32_t s_n;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's entries are stored
    __syncthreads();
    if (threadIdx.x == 0) {
        s_n = 0;
        if (__hip_atomic_fetch_add(&wa.split_redo[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1)
            s_n = 0x80000000u | __hip_atomic_load(&wa.split_redo[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return s_n;
}
__device__ __forceinline__ uint32_t split_redo_entry(const WorkArgs& wa, uint32_t e, int w) {
    return __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&wa.split_redo[2 + 2 * e + w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void split_redo_reset(const WorkArgs& wa, uint32_t last) {
    __syncthreads();
    if (threadIdx.x == 0 && last) {
        __hip_atomic_store(&wa.split_redo[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&wa.split_redo[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
template <bool PREFILTER, bool BRUTE, bool RESIDENT>
MIRT_TRACE_KERNEL void k_primary(const FrameArgs fa, const WorkArgs wa, OutPlanes out) {
    double* const lds = g_lds_mesh;  // RESIDENT: the mesh (dynamic LDS sized at launch)
    __shared__ uint32_t wstk[kWG / 64][MIRT_PRIMARY_WIDE ? kBvhStack : 1];
    __shared__ cnt_t red[kWG / 64][4];
    __shared__ float4 frect[8];  // frustum rectangles
    __shared__ uint32_t bq[kBlkQ][3];  // this workgroup's block descriptors (out, pxy, geo)
    __shared__ uint32_t bq_next;
    WaveClock clock;
    uint32_t taken = 0;
    const V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    if (blockIdx.x == 0)  // the next frame's counter set (see mirt_internal.hpp)
        for (int i = threadIdx.x; i < kCntN; i += kWG) wa.counters_next[i] = 0;
    const bool use_frustum = !BRUTE && MIRT_BLOCK_FRUSTUM && wa.fr.on;
    if (use_frustum) stage_frustum(frect, wa.fr);
    if (RESIDENT) {
        const DevObject& ob = fa.obj[0];
        stage_tris<true>(lds, ob.m.tri, 0, ob.m.ntri, sub(cam, V3{ob.pos[0], ob.pos[1], ob.pos[2]}));
    }
    WaveStats ws{0, 0, 0, 0, 0};
    PhaseClock pc;
    // Workgroup w owns blocks w, w + G, w + 2G, ... (G = grid size): a regular lattice over
    // the frame, so every workgroup gets about the same share of the object's footprint.
    // Its descriptors are staged in LDS (kBlkQ at a time) and its waves take them with an
    // LDS ticket: block costs differ by orders of magnitude (culled or not, hit or not), and
    // an LDS atomic balances them without touching the vector memory counter.
    // MIRT_OPT_STATIC_SCHEDULE: wave v of the workgroup takes entries v, v + 8, ... instead.
    const uint32_t G = gridDim.x, wave = wave_id();
    const uint32_t mine = wa.nblocks > blockIdx.x ? (wa.nblocks - blockIdx.x + G - 1) / G : 0u;
    const bool dyn = (wa.dynamic & kDynPrimary) != 0;
    for (uint32_t c0 = 0; c0 < mine; c0 += kBlkQ) {
        const uint32_t nc = min(mine - c0, (uint32_t)kBlkQ);
        for (uint32_t t = threadIdx.x; t < nc; t += kWG) {
            const uint32_t b = blockIdx.x + (c0 + t) * G;
            const u32x4 v = ((const u32x4*)wa.blocks)[(size_t)(b % kQShards) * wa.per_shard + b / kQShards];
            bq[t][0] = v[0];
            bq[t][1] = v[1];
            bq[t][2] = v[2];
        }
        if (threadIdx.x == 0) bq_next = kWG / 64;  // entries 0..7 go to waves 0..7 without a ticket
        if (c0 == 0) clock.mark_staged();
        __syncthreads();
        uint32_t t = wave;
        while (t < nc) {
            const BlockDesc bd{(uint32_t)__builtin_amdgcn_readfirstlane(bq[t][0]),
                               (uint32_t)__builtin_amdgcn_readfirstlane(bq[t][1]),
                               (uint32_t)__builtin_amdgcn_readfirstlane(bq[t][2]), 0u};
            const uint32_t b = blockIdx.x + (c0 + t) * G;
            // WorkArgs::live: a block with no pixel in the frame's live rectangle is skipped
            const uint32_t px = bd.pxy & 0xffffu, py = bd.pxy >> 16, vw = (bd.geo >> 16) & 0xffu, vh = bd.geo >> 24;
            if (px < wa.live[2] && px + vw > wa.live[0] && py < wa.live[3] && py + vh > wa.live[1]) {
                ++taken;
                if (primary_block<RESIDENT, PREFILTER, BRUTE>(fa, wa, out, lds, wstk[wave], RESIDENT, bd, b % kQShards, ws,
                                                              pc, false, use_frustum, frect, nullptr, 0, nullptr, 0, nullptr, b))
                    split_redo_push(wa, b, 0u);  // the same block again, every candidate box-gated, at the launch's end
            }
            pc.lap(3);
            if (dyn) {
                uint32_t nt = 0;
                if ((threadIdx.x & 63) == 0) nt = atomicAdd(&bq_next, 1u);
                t = __builtin_amdgcn_readfirstlane(nt);
            } else {
                t += kWG / 64;
            }
        }
        __syncthreads();  // every wave is done with this batch before it is restaged
    }
    if (mine == 0) {
        __syncthreads();
        clock.mark_staged();
    }
    if (wa.split_redo) {  // the deferred second passes, in the launch's last workgroup
        const uint32_t last = split_redo_last(wa);
        for (uint32_t e = wave; e < (last & 0x7fffffffu); e += kWG / 64) {
            const uint32_t b = split_redo_entry(wa, e, 0);
            const u32x4 v = ((const u32x4*)wa.blocks)[(size_t)(b % kQShards) * wa.per_shard + b / kQShards];
            const BlockDesc bd{(uint32_t)__builtin_amdgcn_readfirstlane(v[0]), (uint32_t)__builtin_amdgcn_readfirstlane(v[1]),
                               (uint32_t)__builtin_amdgcn_readfirstlane(v[2]), 0u};
            primary_block<RESIDENT, PREFILTER, BRUTE>(fa, wa, out, lds, wstk[wave], RESIDENT, bd, b % kQShards, ws, pc, true,
                                                      use_frustum, frect, nullptr, 0, nullptr, 0, nullptr, b);
        }
        split_redo_reset(wa, last);
    }
    stats_flush(wa.counters, red, kStatPrimTests, kStatPrimNodes, kStatPrimLeaves, kStatHits, ws);
    if (MIRT_PHASE_TIMING) {  // record [4], [5], [6] = cycles in setup+raygen, trace, outputs
        clock.clk0 = 0;
        clock.staged = pc.acc[3];
        clock.real0_override = true;
        clock.phase_trace = pc.acc[2];
        clock.phase_setup = pc.acc[0] + pc.acc[1];
    }
    if (wa.timeline) clock.record(wa, 0, taken);
}

// ---------------------------------------------------------------- shadow kernel
// Work item: the 64 slots of one hit block x one light.  Tickets of shard q enumerate
// (light, chunk) of region q.
template <bool PREFILTER, bool BRUTE, bool RESIDENT>
__global__ __launch_bounds__(kWG) __attribute__((amdgpu_waves_per_eu(MIRT_SHADOW_WAVES_PER_EU)))
void k_shadow(const FrameArgs fa, const WorkArgs wa, OutPlanes out) {
    double* const lds = g_lds_mesh;  // RESIDENT: the mesh (dynamic LDS sized at launch)
    __shared__ uint32_t wstk[kWG / 64][MIRT_SHADOW_WIDE ? kBvhStack : 1];
    __shared__ cnt_t red[kWG / 64][4];
    // segment query for one-object frames (BVH kernels only; brute force stays literal)
    // RESIDENT implies one object and no MIRT_OPT_NO_SEGMENT (is_resident): a constant there
    const bool segment = RESIDENT ? !BRUTE : (!BRUTE && fa.n_objects == 1 && !(fa.flags & MIRT_OPT_NO_SEGMENT));
    WaveClock clock;
    uint32_t taken = 0;
    if (RESIDENT) {
        stage_tris<false>(lds, fa.obj[0].m.tri, 0, fa.obj[0].m.ntri, V3{0, 0, 0});
        __syncthreads();
    }
    clock.mark_staged();
    const ShardCursor sc;
    WaveStats ws{0, 0, 0, 0, 0};
    const uint32_t nl = max(fa.n_lights, 1u);
    cnt_t* const qctr = wa.qcounters ? wa.qcounters : wa.counters;
    for (uint32_t q = sc.first_shard(); q < (uint32_t)kQShards; q += sc.shard_step()) {
        const uint32_t nrec = __builtin_amdgcn_readfirstlane(*lo32(&qctr[cnt_hits(q)])), nch = (nrec + 63) / 64;
        const uint32_t items = nch * nl, peers = sc.peers();
        cnt_t* qc = &qctr[cnt_queue(1, q)];
        // item rank is this wave's (static); with the queue on, items peers + ticket follow,
        // each ticket taken while the previous item is traced
        const bool dyn = (wa.dynamic & kDynShadow) && items > peers;
        uint32_t k = sc.rank(), nxt = 0;
        while (k < items) {
            nxt = dyn ? ticket_issue(qc) : 0;
            ++taken;
            const uint32_t l = k / nch, c = k - l * nch;
            if (shadow_item<PREFILTER, BRUTE, MIRT_SHADOW_LT3, 0, true>(fa, wa, out, lds, wstk[wave_id()], RESIDENT, segment,
                                                              (size_t)q * wa.hit_cap + (size_t)c * 64, l, ws, false, ~0u,
                                                              nullptr, min(64u, nrec - c * 64)))
                // the same item again, every candidate box-gated, at the launch's end (not counted
                // done, so its chunk is shaded then)
                split_redo_push(wa, (uint32_t)((size_t)q * wa.hit_cap / 64 + c), l | min(64u, nrec - c * 64) << 8);
            k = dyn ? peers + ticket_resolve(nxt) : k + peers;
        }
    }
#ifndef MIRT_EXP_NO_SPLIT_REDO
    if (wa.split_redo) {  // the deferred second passes, in the launch's last workgroup
        const uint32_t last = split_redo_last(wa);
        for (uint32_t e = wave_id(); e < (last & 0x7fffffffu); e += kWG / 64) {
            const uint32_t ch = split_redo_entry(wa, e, 0), w1 = split_redo_entry(wa, e, 1);
            shadow_item<PREFILTER, BRUTE, MIRT_SHADOW_LT3, 0, true>(fa, wa, out, lds, wstk[wave_id()], RESIDENT, segment,
                                                          (size_t)ch * 64, w1 & 0xffu, ws, true, ~0u, nullptr, w1 >> 8);
        }
        split_redo_reset(wa, last);
    }
#endif
    stats_flush(wa.counters, red, kStatShadowTests, kStatShadowNodes, kStatShadowLeaves, -1, ws);
    if (wa.timeline) clock.record(wa, 1, taken);
    if (!wa.bounces) frame_fold(fa, wa);  // otherwise the reflection fold is the frame's last kernel
}

// ---------------------------------------------------------------- one-launch frame
// k_trace: the whole frame in ONE persistent launch, primary blocks and their shadow
// items handled inside the workgroup that owns the blocks.  Workgroup w owns the same
// lattice of blocks as in k_primary and a private hit region (WorkArgs::wg_cap slots);
// its waves take primary blocks and shadow items (chunk, light) with LDS tickets,
// preferring shadow items so the region stays hot in this XCD's L2.  A chunk is
// published through an LDS ready flag once its stores have reached L2 (every wave of the
// workgroup shares that L2, so no device-scope coherence is needed).  One mesh staging,
// no second launch, and the shadow work of early blocks fills the primary tail.  The mesh
// is staged in absolute coordinates (the shadow rays' origins differ per lane).
// The launch's frame records, read through the constant address space: the kernel never
// writes them, so their loads stay scalar and are not repeated after the kernel's stores.
typedef const __attribute__((address_space(4))) FrameRec ConstFrameRec;
// k_trace's arguments: every frame record of the launch (FrameRecs, only the first nframes
// meaningful), then the work description.  A launch's kernarg segment of up to 28 KB costs the
// host what a 4 KB one does (tools/launch_cost: 4.9 us at 4 KB, 5.6 at 28 KB) and the records reach the kernel
// with no staging copy (a k_stage_frames launch per batch before); frame_rec finds record f at
// offset f * sizeof(FrameRec) of the segment.
static_assert(sizeof(FrameRecs) + sizeof(WorkArgs) <= 32 * 1024, "k_trace arguments exceed the measured kernarg size");
__device__ __forceinline__ const FrameRec& frame_rec(const FrameRec* frames, uint32_t f) {
    return *(const FrameRec*)((ConstFrameRec*)frames + f);
}

// recs: the launch's frame records (the first kernel argument, read in place from the kernarg
// segment through the constant address space).
// VIEWS: the instantiation that uses view tables (MIRT_OPT_VIEWS); the default one has no
// view code at all (present, it cost 6 spilled VGPRs and 1.7% of the frame interval).
// One recorded block traced again from its pixels (redo_mark), every query with its second pass
// in place: primary_block's raygen, the nearest hit, one shadow query per light and phong
// (shadow_item's arithmetic, lane by lane), and all of the block's outputs.
template <bool PREFILTER, bool BRUTE, bool RESIDENT, int HBM1 = 0>
__device__ __forceinline__ void redo_block(const FrameArgs& fa, const OutPlanes& out, const BlockDesc& bd,
                                           const XferArgs* xf) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lx = lane >> 3, ly = lane & 7;
    const uint32_t px = bd.pxy & 0xffffu, py = bd.pxy >> 16, th = bd.geo & 0xffffu;
    const uint32_t vw = (bd.geo >> 16) & 0xffu, vh = bd.geo >> 24;
    const bool active = lx < vw && ly < vh;
    const uint32_t i = px + (active ? lx : 0), j = py + (active ? ly : 0);
    const V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    // tracer.go:15-22, :86 (primary_block's operations)
    const double si = fa.phw * ((double)(fa.halfW - (int32_t)i) - 0.5) / (double)fa.halfW;
    const double sj = fa.phh * ((double)(fa.halfH - (int32_t)j) - 0.5) / (double)fa.halfH;
    V3 p = add(add(add(cam, V3{fa.fwd[0], fa.fwd[1], fa.fwd[2]}), scale(V3{fa.left[0], fa.left[1], fa.left[2]}, si)),
               scale(V3{fa.up[0], fa.up[1], fa.up[2]}, sj));
    const V3 d = norm(sub(p, cam));
    Visits vis{0, 0, 0, 0};
    const Nearest nh =
        trace_nearest_settled<false, PREFILTER, BRUTE, HBM1>(fa, g_lds_mesh, RESIDENT, cam, d, active, true, vis);
    const bool hit = active && nh.ok;
    const bool segment = RESIDENT ? !BRUTE : (!BRUTE && fa.n_objects == 1 && !(fa.flags & MIRT_OPT_NO_SEGMENT));
    uint32_t lit = 0;
    for (uint32_t l = 0; l < fa.n_lights; ++l) {
        const V3 lpos{fa.lpos[l][0], fa.lpos[l][1], fa.lpos[l][2]};
        V3 o{0, 0, 0}, sd{1, 0, 0};
        if (hit) {
            sd = norm(sub(lpos, nh.hit));      // tracer.go:61
            o = add(nh.hit, scale(sd, 0.0001));  // tracer.go:64
        }
        bool is_lit;
        if (segment) {
            is_lit = shadow_lit_single_settled<PREFILTER, true, HBM1>(fa, g_lds_mesh, RESIDENT, nullptr, nh.hit, o, sd, lpos,
                                                                        l, hit, vis);
        } else {
            const Nearest r =
                trace_nearest_settled<false, PREFILTER, BRUTE, HBM1>(fa, g_lds_mesh, RESIDENT, o, sd, hit, false, vis);
            is_lit = !r.ok || len(sub(lpos, nh.hit)) < len(sub(r.hit, nh.hit));
        }
        if (hit && is_lit) lit |= 1u << l;
    }
    const uint64_t oidx = out_index(xf, bd, lx, ly, th);
    if (!active || oidx == kNoOut) return;
    if (out.valid) out.valid[oidx] = hit ? 1 : 0;
    if (out.face) out.face[oidx] = hit ? (int32_t)nh.face : -1;
    if (out.object) out.object[oidx] = hit ? (int32_t)nh.obj : -1;
    RGB col{0, 0, 0};
    if (hit) col = phong(fa, fa.obj[nh.obj].m.mats + (size_t)nh.mat * 10, nh.hit, nh.normal, lit);
    if (out.rgb) {
        out.rgb[3 * oidx] = col.r;
        out.rgb[3 * oidx + 1] = col.g;
        out.rgb[3 * oidx + 2] = col.b;
    }
    if (out.rgb8) {
        out.rgb8[3 * oidx] = c_u8(col.r);
        out.rgb8[3 * oidx + 1] = c_u8(col.g);
        out.rgb8[3 * oidx + 2] = c_u8(col.b);
    }
    if (out.rgbv) out.rgbv[oidx] = hit ? pack_rgbv(col) : 0u;
}

// One entry of k_trace's redo list (redo_mark), out of line: a call at the kernel's end, where
// nothing of the work loop is live, keeps the second passes' code and registers out of the
// kernel body (its SGPR allocation).  Arguments are made scalar again, the frame records and
// the work description read through the constant address space.
typedef const __attribute__((address_space(4))) WorkArgs ConstWorkArgs;
constexpr size_t kTraceWaOffset = kalign(sizeof(FrameRecs), alignof(WorkArgs));  // k_trace's second argument
template <bool PREFILTER, bool BRUTE, bool RESIDENT, int HBM1 = 0>
__device__ __attribute__((noinline)) void trace_redo_entry(const FrameRec* frames, const WorkArgs* wap, uint32_t e) {
    frames = uni_ptr(frames);
    const WorkArgs& wa = *(const WorkArgs*)(ConstWorkArgs*)uni_ptr(wap);
    e = uni32(e);
    const uint32_t key = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&wa.bgcnt[1 + e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t f = key >> 28, qbl = key & 0x0fffffffu;
    const u32x4 qv = ((const u32x4*)wa.blocks)[(size_t)(qbl % kQShards) * wa.per_shard + qbl / kQShards];
    const BlockDesc bd{(uint32_t)__builtin_amdgcn_readfirstlane(qv[0]), (uint32_t)__builtin_amdgcn_readfirstlane(qv[1]),
                       (uint32_t)__builtin_amdgcn_readfirstlane(qv[2]), 0u};
    const FrameRec& fr = frame_rec(frames, f);
    redo_block<PREFILTER, BRUTE, RESIDENT, HBM1>(fr.fa, fr.out, bd, &fr.xf);
    if ((threadIdx.x & 63) == 0)
        __hip_atomic_store(&wa.bmap[f * wa.nblocks_frame + qbl], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bytes [a, b) of src -> dst with the same alignment on both sides (same layout): head
// bytes, 16-byte words, tail bytes; one wave.
__device__ __forceinline__ void copy_span(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t a,
                                          uint64_t b, uint32_t lane) {
    const uint64_t a16 = min(b, (a + 15) & ~15ull), b16 = max(a16, b & ~15ull);
    if (a + lane < a16) dst[a + lane] = src[a + lane];
    for (uint64_t i = a16 + 16 * lane; i < b16; i += 16 * 64) *(uint4*)(dst + i) = *(const uint4*)(src + i);
    if (b16 + lane < b) dst[b16 + lane] = src[b16 + lane];
}
// One column x of frame f of a host copy job (k_copy_rect_host, k_trace's fused copy): one wave.
__device__ __forceinline__ void copy_column(const HostCopyJobs& jobs, uint32_t f, uint32_t x, uint32_t H, uint32_t lane) {
    const uint32_t* C = jobs.cur[f];
    uint32_t a = 1, b = 0;  // this frame's hit rows [a, b) (empty: a > b)
    if (x >= C[0] && x < C[2] && C[1] < C[3]) {
        // the column's rows [C[1], C[3]) of the valid plane in aligned 8-byte words, 512 rows per
        // wave-wide step and the steps' loads independent (no chain of dependent loads through the
        // rectangle: an edge column's few hit rows can lie anywhere in it).  The plane is 8-byte
        // aligned (mirt_group_create checks caller planes; library planes are hipMalloc'ed), so the
        // last word stays inside the page of the plane's last byte; its bytes past `end` are masked.
        const uint64_t x0 = (uint64_t)x * H, beg = x0 + C[1], end = x0 + C[3];
        const uint8_t* plane = jobs.valid[f];
        uint32_t lo = ~0u, hi = 0;  // this lane's first / last hit row + 1 (none: lo = ~0u)
#pragma unroll 4
        for (uint64_t p = (beg & ~7ull) + 8 * lane; p < end; p += 8 * 64) {
            uint64_t w = *(const uint64_t*)(plane + p);
            if (p < beg) w &= ~0ull << (8 * (beg - p));
            if (end - p < 8) w &= (1ull << (8 * (end - p))) - 1;
            if (w) {
                const uint32_t r = (uint32_t)((int64_t)p - (int64_t)x0);
                lo = min(lo, r + (uint32_t)__builtin_ctzll(w) / 8);
                hi = max(hi, r + (uint32_t)(63 - __builtin_clzll(w)) / 8 + 1);
            }
        }
        for (int o = 32; o; o >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
        }
        if (lo != ~0u) {
            a = lo;
            b = hi;
        }
    }
    const uint32_t prev = jobs.spans[f][x];
    const uint32_t a0 = prev & 0xffffu, b0 = prev >> 16;
    uint32_t u0 = a0, u1 = b0;
    if (a < b) {
        u0 = a0 < b0 ? min(a, a0) : a;
        u1 = a0 < b0 ? max(b, b0) : b;
    }
    if (u0 < u1) {
        // the spans widened to whole 16-byte words inside the column: the device plane is current at
        // every pixel of the frame (misses included), so the extra bytes are this frame's too, and
        // the head and tail single-byte stores over PCIe go (they remain only at a column's ends)
        const uint64_t c0 = (uint64_t)x * H, p0 = c0 + u0, p1 = c0 + u1;
        auto widen = [](uint64_t a, uint64_t b, uint64_t lo, uint64_t hi, uint64_t& wa, uint64_t& wb) {
            wa = max(lo, a & ~15ull);
            wb = min(hi, (b + 15) & ~15ull);
        };
        uint64_t a, b;
        widen(3 * p0, 3 * p1, 3 * c0, 3 * (c0 + H), a, b);
        copy_span(jobs.rgb8[f], jobs.hrgb8[f], a, b, lane);
        widen(p0, p1, c0, c0 + H, a, b);
        copy_span(jobs.valid[f], jobs.hvalid[f], a, b, lane);
    }
    if (lane == 0) jobs.spans[f][x] = a < b ? (a | (b << 16)) : 0u;
}
// k_trace's third argument (FusedCopy), read in place from the kernarg segment.
constexpr size_t kTraceFcOffset = kalign(kTraceWaOffset + sizeof(WorkArgs), alignof(FusedCopy));
static_assert(kTraceFcOffset + sizeof(FusedCopy) <= 32 * 1024, "k_trace arguments exceed the measured kernarg size");
}  // namespace mirt
// The layout above as the device code assumes it; tests/test_kernarg_layout.py checks it against
// the code object's argument metadata for every kernel instantiation.
extern "C" int mirt_debug_kernarg_layout(uint64_t* out, uint32_t n) {
    using namespace mirt;
    const uint64_t v[8] = {sizeof(FrameRecs), kTraceWaOffset,   sizeof(WorkArgs),  kTraceFcOffset,
                           sizeof(FusedCopy), sizeof(FrameArgs), sizeof(OutPlanes), sizeof(BounceArgs)};
    if (!out) return MIRT_E_INVALID;
    const uint32_t k = n < 8 ? n : 8;
    for (uint32_t i = 0; i < k; ++i) out[i] = v[i];
    return (int)k;
}
namespace mirt {
template <bool PREFILTER, bool BRUTE, bool RESIDENT, bool VIEWS = false, int HBM1 = 0>
MIRT_TRACE_KERNEL void k_trace(const FrameRecs recs, const WorkArgs wa, const FusedCopy fc) {
    const FrameArgs& fa = recs.r[0].fa;
    // (recs is the first kernel argument: offset 0 of the kernarg segment; taking its address
    // would copy it to scratch)
    const FrameRec* const frames = (const FrameRec*)(ConstFrameRec*)__builtin_amdgcn_kernarg_segment_ptr();
    double* const lds = g_lds_mesh;  // RESIDENT: the mesh (dynamic LDS sized at launch)
    __shared__ uint32_t wstk[kWG / 64][(MIRT_PRIMARY_WIDE || MIRT_SHADOW_WIDE) ? kBvhStack : 1];
    __shared__ cnt_t red[kWG / 64][4];
    __shared__ float4 frect[kMaxFrames][8];
    __shared__ uint32_t bq[kBlkQ][3];
    __shared__ uint8_t bq_cull[kBlkQ];   // 1: the block frustum pre-test culled it at staging
    __shared__ uint8_t bq_frame[kBlkQ];  // the block's frame within the launch
    __shared__ uint32_t bq_bl[kBlkQ];    // the block's index in the frame's table (WorkArgs::block_cost)
    __shared__ uint32_t s_bucket[kQueueBuckets];
    __shared__ uint8_t chunk_frame[kBlkQ];
    __shared__ uint32_t ready[kBlkQ];
    __shared__ uint16_t chunk_pos[kBlkQ];  // each chunk's position in the region (ring_take)
    __shared__ uint32_t chunk_key[kBlkQ];  // each chunk's block (redo_mark)
    __shared__ uint32_t s_prim, s_pdone, s_chunks, s_item, s_front, s_back, s_ring;
    __shared__ ViewHead s_vhead[VIEWS ? kMaxViewTables : 1];
    __shared__ uint32_t s_vstate[VIEWS ? kMaxViewTables : 1];
    const ViewCache vc{s_vhead, s_vstate};
    // RESIDENT implies one object and no MIRT_OPT_NO_SEGMENT (is_resident): a constant there
    const bool segment = (RESIDENT || HBM1) ? !BRUTE : (!BRUTE && fa.n_objects == 1 && !(fa.flags & MIRT_OPT_NO_SEGMENT));
    WaveClock clock;
    uint32_t taken = 0;
    if (blockIdx.x == 0)  // the next frame's counter set (see mirt_internal.hpp)
        for (int i = threadIdx.x; i < kCntN; i += kWG) wa.counters_next[i] = 0;
    const uint32_t NF = wa.nframes, nbf = wa.nblocks_frame;  // the host checks NF <= kMaxFrames
    const bool use_frustum = !BRUTE && MIRT_BLOCK_FRUSTUM && wa.fr.on;  // same for every frame (host)
    if (use_frustum && threadIdx.x < 8 * NF) {
        const float* r = frame_rec(frames, threadIdx.x >> 3).fr.rect[threadIdx.x & 7];
        frect[threadIdx.x >> 3][threadIdx.x & 7] = make_float4(r[0], r[1], r[2], r[3]);
    }
    if (VIEWS && threadIdx.x < kMaxViewTables) s_vstate[threadIdx.x] = 0;  // read after the batch barrier
    if (VIEWS && RESIDENT && wa.views && blockIdx.x < NF * wa.nviews) {
        // the launch's first workgroups build the view tables in the mesh's LDS, then stage it
        const uint32_t q = blockIdx.x, f = q / wa.nviews;
        build_view(frame_rec(frames, f), q - f * wa.nviews, wa.views + (size_t)q * wa.view_leaves, wa.view_heads + q, lds,
                   wa.view_tag);
        __syncthreads();
    }
    if (fc.n) {
        // the host copy of an earlier launch's frames on this stream (a column per wave; that
        // launch has ended: stream order), before this workgroup's tracing: fire and forget
        const FusedCopy* cp = at_use((const FusedCopy*)((const char*)__builtin_amdgcn_kernarg_segment_ptr() + kTraceFcOffset));
        const uint32_t nw = gridDim.x * (kWG / 64), gw = blockIdx.x * (kWG / 64) + wave_id();
        for (uint32_t f = 0; f < cp->n; ++f)
            for (uint32_t x = cp->jobs.rect[f][0] + gw; x < cp->jobs.rect[f][2]; x += nw)
                copy_column(cp->jobs, f, x, cp->H, threadIdx.x & 63);
    }
    if (RESIDENT) stage_tris<false>(lds, fa.obj[0].m.tri, 0, fa.obj[0].m.ntri, V3{0, 0, 0});
    if (HBM1 == 2 && threadIdx.x < kWG / 64) g_stream_base[threadIdx.x] = ~0u;  // no window yet (read after the batch barrier)
    uint32_t* stk = wstk[wave_id()];
    WaveStats wp{0, 0, 0, 0, 0}, wsh{0, 0, 0, 0, 0};
    PhaseClock pc;
    const uint32_t nl = max(fa.n_lights, 1u);
    constexpr uint32_t kNone = 0xffffffffu;
    // every wait is bounded (~1 s): should progress ever stall, the wave records it in the
    // overflow statistic (tests assert 0) and leaves, so the kernel always drains
    constexpr uint32_t kSpinLimit = 1u << 24;
    uint32_t spins = 0;
    const uint32_t G = gridDim.x;
    const uint32_t mine = wa.nblocks > blockIdx.x ? (wa.nblocks - blockIdx.x + G - 1) / G : 0u;
    const size_t chunk0 = (size_t)blockIdx.x * wa.wg_cap;  // slot of the region's position 0
    auto lds_ld = [](uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto lds_inc = [](uint32_t* p) {
        uint32_t t = 0;
        if ((threadIdx.x & 63) == 0) t = atomicAdd(p, 1u);
        return (uint32_t)__builtin_amdgcn_readfirstlane(t);
    };
    ItemClock ic;
    // Blocks the frustum pre-test cannot cull go to the front of the workgroup's queue:
    // their primary trace and shadow items are the long single-wave chains, and starting
    // them first keeps the cheap culled blocks as filler instead of delaying a chain to the
    // end of the workgroup's life (the frame's tail; with a small tile list, its latency).
    const bool classify = use_frustum;
    const bool partition = classify && !(fa.flags & MIRT_OPT_STATIC_SCHEDULE);
    if (classify) __syncthreads();  // the frustum rectangles are staged
    for (uint32_t c0 = 0; c0 < mine; c0 += kBlkQ) {
        const uint32_t nc = min(mine - c0, (uint32_t)kBlkQ);
        // Queue order, by buckets filled in one pass (nc <= kBlkQ <= kWG: one entry per
        // thread): blocks that may meet the object before culled ones; with cost estimates
        // (WorkArgs::block_cost) unknown ones first, then by their last primary trace time,
        // longest first (log2 buckets), so the long single-wave chains start at once.
        static_assert(kBlkQ <= kWG, "one queue entry per thread");
        if (threadIdx.x == 0) {
            s_front = 0;
            s_back = nc;  // every queued block goes to [0, s_front)
        }
        if (threadIdx.x < kQueueBuckets) s_bucket[threadIdx.x] = 0;
        __syncthreads();
        const uint32_t t = threadIdx.x;
        uint32_t cls = ~0u, qbl = 0, qf = 0;
        u32x4 qv{0u, 0u, 0u, 0u};
        bool culled = false, ocert = false;
        if (t < nc) {
            const uint32_t b = blockIdx.x + (c0 + t) * G;  // over every frame's blocks
            qf = b / nbf;
            qbl = b - qf * nbf;
            qv = ((const u32x4*)wa.blocks)[(size_t)(qbl % kQShards) * wa.per_shard + qbl / kQShards];
            ready[t] = 0;
            // FrameRec::live: a block with no pixel in the frame's live rectangle is not queued
            const uint32_t px = qv[1] & 0xffffu, py = qv[1] >> 16, vw = (qv[2] >> 16) & 0xffu, vh = qv[2] >> 24;
            const uint32_t* lv = frame_rec(frames, qf).live;
            if (px < lv[2] && px + vw > lv[0] && py < lv[3] && py + vh > lv[1]) {
                if (classify) {
                    culled = !block_may_meet(frame_rec(frames, qf).fr, frect[qf], px, py, vw, vh);
                    ocert = !culled && block_obj_cert(frame_rec(frames, qf), px, py, vw, vh);
                }
                if (!partition) {
                    cls = 0;
                } else if (culled) {
                    cls = kQueueBuckets - 1;
                } else if (wa.block_cost) {
                    const uint32_t est = wa.block_cost[qbl];
                    const int lg = est ? 31 - __builtin_clz(est) : 0;
                    cls = est == 0 ? 0u : 1u + (uint32_t)min(kQueueBuckets - 3, max(0, 12 - lg));
                } else {
                    cls = 0;
                }
            }
        }
        if (cls != ~0u) atomicAdd(&s_bucket[cls], 1u);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int k = 0; k < kQueueBuckets; ++k) {
                const uint32_t c = s_bucket[k];
                s_bucket[k] = acc;
                acc += c;
            }
            s_front = acc;
        }
        __syncthreads();
        if (cls != ~0u) {
            const uint32_t slot = atomicAdd(&s_bucket[cls], 1u);
            bq_bl[slot] = qbl;
            bq[slot][0] = qv[0];
            bq[slot][1] = qv[1];
            bq[slot][2] = qv[2];
            bq_cull[slot] = classify ? (culled ? 1 : 2 | (ocert ? 4 : 0)) : 0;  // 0: not classified
            bq_frame[slot] = (uint8_t)qf;
        }
        if (threadIdx.x == 0) {
            s_prim = s_pdone = s_chunks = s_item = 0;
            s_ring = kHitRing >= 32 ? ~0u : (1u << kHitRing) - 1u;  // every ring position free
        }
        if (c0 == 0) clock.mark_staged();
        __syncthreads();
        // queued blocks: [0, s_front) and [s_back, nc); ticket q is entry q or q - nfront + s_back
        const uint32_t nfront = s_front, back0 = s_back, nq = nfront + (nc - back0);
        LocalChunks lc{&s_chunks, ready, chunk0, chunk_frame, 0, &s_ring, chunk_pos, chunk_key};
        uint32_t pend = kNone;  // a shadow ticket held (possibly for a chunk not yet allocated)
        for (;;) {
            // 1. a shadow item of an allocated chunk
            const uint32_t avail = lds_ld(&s_chunks) * nl;
            if (pend == kNone && lds_ld(&s_item) < avail) pend = lds_inc(&s_item);
            if (pend != kNone && pend < avail) {
                const uint32_t c = pend / nl, l = pend - c * nl;
                while (lds_ld(&ready[c]) == 0 && ++spins < kSpinLimit) {
                    diag(17);
                    __builtin_amdgcn_s_sleep(1);
                }
                if (spins >= kSpinLimit) break;
                // the chunk's LDS records (position, frame) are read after its ready flag: the
                // producer wrote them first, and LDS operations complete in order
                asm volatile("" ::: "memory");
                ++taken;
                diag(19);
                ic.start();
                const WaveStats before = wsh;
                const uint32_t cf = __builtin_amdgcn_readfirstlane(chunk_frame[c]);
                const FrameRec& fr = frame_rec(frames, cf);
                const uint32_t cp = __builtin_amdgcn_readfirstlane(chunk_pos[c]);
                const uint32_t ck = __builtin_amdgcn_readfirstlane(chunk_key[c]);
                shadow_item<PREFILTER, BRUTE, true, HBM1>(fr.fa, wa, fr.out, lds, stk, RESIDENT, segment, chunk0 + (size_t)cp * 64, l, wsh,
                                              false, RESIDENT ? cf : ~0u, VIEWS ? &vc : nullptr, 64, &s_ring, cp, ck);
                ic.record(wa, 1, wsh.tests - before.tests, wsh.nodes - before.nodes, 0);
                pend = kNone;
                continue;
            }
            // 2. a primary block
            if (lds_ld(&s_prim) < nq) {
                const uint32_t q = lds_inc(&s_prim);
                if (q < nq) {
                    const uint32_t t = q < nfront ? q : q - nfront + back0;
                    const BlockDesc bd{(uint32_t)__builtin_amdgcn_readfirstlane(bq[t][0]),
                                       (uint32_t)__builtin_amdgcn_readfirstlane(bq[t][1]),
                                       (uint32_t)__builtin_amdgcn_readfirstlane(bq[t][2]), 0u};
                    ++taken;
                    diag(20);
                    ic.start();
                    const WaveStats before = wp;
                    const uint64_t ph0 = pc.acc[0], ph1 = pc.acc[1];
                    const uint32_t f = __builtin_amdgcn_readfirstlane(bq_frame[t]);
                    const FrameRec& fr = frame_rec(frames, f);
                    lc.frame = f;
                    // the camera's view table of this frame, once published (and usable)
                    const ViewLeaf* vt = nullptr;
                    if (VIEWS && RESIDENT && wa.views && fr.fr.on && view_lookup(wa, f * wa.nviews, vc))
                        vt = wa.views + (size_t)f * wa.nviews * wa.view_leaves;
                    const uint64_t cost0 = wa.block_cost ? __builtin_amdgcn_s_memtime() : 0;
                    const uint32_t cls = __builtin_amdgcn_readfirstlane(bq_cull[t]);
                    const uint32_t key = f << 28 | __builtin_amdgcn_readfirstlane(bq_bl[t]);
                    if (primary_block<false, PREFILTER, BRUTE, HBM1>(fr.fa, wa, fr.out, lds, stk, RESIDENT, bd, 0, wp, pc, false,
                                                               use_frustum, frect[f], &lc, cls, vt, wa.view_leaves, &fr.fr,
                                                               key, &fr.xf))
                        redo_mark(wa, key);  // traced again, from its pixels, at the launch's end
                    if (wa.block_cost && (threadIdx.x & 63) == 0) {  // this trace's time, for the slot's next frame
                        const uint64_t dc = (__builtin_amdgcn_s_memtime() - cost0) >> 6;
                        wa.block_cost[bq_bl[t]] = (uint16_t)(dc < 1 ? 1 : (dc > 65535 ? 65535 : dc));
                    }
                    ic.record(wa, 0, wp.tests - before.tests, wp.nodes - before.nodes, wp.hits - before.hits,
                              (pc.acc[0] - ph0) | ((pc.acc[1] - ph1) << 32));
                    lds_inc(&s_pdone);  // after the block's chunk (if any) was allocated
                    continue;
                }
            }
            // 3. nothing available now: leave once every block is done and no item is left
            if (lds_ld(&s_pdone) >= nq) {
                const uint32_t total = lds_ld(&s_chunks) * nl;
                if (pend == kNone) {
                    if (lds_ld(&s_item) >= total) break;
                    pend = lds_inc(&s_item);
                }
                if (pend >= total) break;
                continue;
            }
            if (++spins >= kSpinLimit) break;
            diag(18);
            __builtin_amdgcn_s_sleep(1);
        }
        // every wave is done with this batch (each chunk shaded, its ring position free)
        // before it is restaged; the next batch reuses the region from position 0
        __syncthreads();
    }
    if (mine == 0) clock.mark_staged();
    if (spins >= kSpinLimit) wp.overflow += 1;
    __syncthreads();
    stats_flush<true>(wa.counters, red, kStatPrimTests, kStatPrimNodes, kStatPrimLeaves, kStatHits, wp);
    __syncthreads();
    stats_flush<true>(wa.counters, red, kStatShadowTests, kStatShadowNodes, kStatShadowLeaves, -1, wsh);
    if (wa.timeline && !MIRT_ITEM_TRACE) clock.record(wa, 0, taken);
    const bool last = launch_last(wa);
    if (last && wa.bgcnt) {
        // the deferred second passes (redo_mark): every other workgroup is done
        const uint32_t n = __hip_atomic_load(&wa.bgcnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t e = wave_id(); e < n; e += kWG / 64)
            trace_redo_entry<PREFILTER, BRUTE, RESIDENT, HBM1>(
                frames, (const WorkArgs*)((const char*)__builtin_amdgcn_kernarg_segment_ptr() + kTraceWaOffset), e);
        __syncthreads();
        if (threadIdx.x == 0 && n) {
            __hip_atomic_store(&wa.bgcnt[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (wa.prof_acc) atomicAdd(&wa.prof_acc[kProfRedo], (cnt_t)n);  // mirt_profile.redo_items
        }
    }
    if (last && threadIdx.x == 0)  // the trailers of the shares written in their transfer form
        for (uint32_t f = 0; f < wa.nframes; ++f) {
            const FrameRec& fr = frame_rec(frames, f);
            if (fr.xf.on && fr.out.rgbv) {
                fr.out.rgbv[fr.xf.words] = fr.xf.tag;
                fr.out.rgbv[fr.xf.words + 1] = fr.xf.words;
            }
        }
    frame_summary<true>(fa, wa, last);
}

// ---------------------------------------------------------------- reflections (configs[4])
// EXTENSION, not in the reference (oracle: rt_oracle.c shade_reflect).
// Work item: the 64 slots of one hit block.  Each lane follows its own bounce chain:
// R = D - 2 (D.N) N, nearest hit of trace(hit + R 1e-4, R), phong there with shadow
// rays; then the levels are combined innermost first, c_k = c_add(ph_k, c_mul(Ks_k,
// c_(k+1))), a miss contributing black, the deepest level (k = bounces) plain phong.
// Level 0's phong comes from the shadow kernel (WorkArgs::ph0).
template <bool PREFILTER, bool BRUTE, bool RESIDENT>
MIRT_REFLECT_KERNEL void k_reflect(const FrameArgs fa, const WorkArgs wa, OutPlanes out) {
    double* const lds = g_lds_mesh;  // RESIDENT: the mesh (dynamic LDS sized at launch)
    __shared__ cnt_t red[kWG / 64][4];
    // RESIDENT implies one object and no MIRT_OPT_NO_SEGMENT (is_resident): a constant there
    const bool segment = RESIDENT ? !BRUTE : (!BRUTE && fa.n_objects == 1 && !(fa.flags & MIRT_OPT_NO_SEGMENT));
    if (RESIDENT) {
        stage_tris<false>(lds, fa.obj[0].m.tri, 0, fa.obj[0].m.ntri, V3{0, 0, 0});
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63;
    const ShardCursor sc;
    WaveStats ws{0, 0, 0, 0, 0};
    cnt_t refl_rays = 0, refl_shadow = 0;
    const uint32_t B = min(wa.bounces, (uint32_t)MIRT_MAX_BOUNCES);
    for (uint32_t q = sc.first_shard(); q < (uint32_t)kQShards; q += sc.shard_step()) {
        const uint32_t nch = *lo32(&wa.counters[cnt_hits(q)]) / 64;
        cnt_t* qc = &wa.counters[cnt_queue(2, q)];
        uint32_t k = (wa.dynamic & kDynReflect) ? ticket_resolve(ticket_issue(qc)) : sc.rank();
        while (k < nch) {
            const uint32_t nxt = (wa.dynamic & kDynReflect) ? ticket_issue(qc) : 0;
            const size_t slot = (size_t)q * wa.hit_cap + (size_t)k * 64 + lane;
            const HitRec rec = wa.hits[slot];
            const bool active = rec.obj != kNoHit;
            // Only the current bounce is live; each level's phong and material go to
            // WorkArgs::refl and are folded back innermost first below (a per-lane array of
            // every level, indexed at run time, lived in scratch: 55-71 spilled VGPRs).
            V3 D{1, 0, 0}, hit{0, 0, 0}, N{0, 0, 1};
            uint32_t levels = 0;   // levels with a phong value
            bool missed = false;   // the chain ended on a miss (else on the depth limit)
            if (active) {
                D = vload(wa.dir0 + 3 * slot);
                hit = vload(rec.h);
                N = vload(rec.n);
                levels = 1;
            }
            bool on = active;
            for (uint32_t lv = 1; lv <= B; ++lv) {
                if (__ballot(on) == 0) break;
                const V3 R = sub(D, scale(N, 2 * dot(D, N)));
                const V3 o = add(hit, scale(R, 0.0001));
                Visits vis{0, 0, 0, 0};
                const Nearest r = trace_nearest_settled<false, PREFILTER, BRUTE>(fa, lds, RESIDENT, o, R, on, true, vis);
                refl_rays += __popcll(__ballot(on));
                ws.tests += (cnt_t)vis.tests * __popcll(__ballot(on));
                ws.nodes += vis.nodes;
                ws.leaves += vis.leaves;
                ws.overflow += vis.overflow;
                if (on && !r.ok) {
                    missed = true;
                    on = false;
                }
                uint32_t lit = 0;
                refl_shadow += (cnt_t)__popcll(__ballot(on)) * fa.n_lights;
                for (uint32_t l = 0; l < fa.n_lights; ++l) {  // tracer.go:60-64 at the reflected hit
                    const V3 lpos{fa.lpos[l][0], fa.lpos[l][1], fa.lpos[l][2]};
                    V3 so{0, 0, 0}, sd{1, 0, 0};
                    if (on) {
                        sd = norm(sub(lpos, r.hit));
                        so = add(r.hit, scale(sd, 0.0001));
                    }
                    Visits sv{0, 0, 0, 0};
                    bool is_lit;
                    if (segment) {
                        is_lit = shadow_lit_single_settled<PREFILTER>(fa, lds, RESIDENT, nullptr, r.hit, so, sd, lpos, l, on, sv);
                    } else {
                        const Nearest sr = trace_nearest_settled<false, PREFILTER, BRUTE>(fa, lds, RESIDENT, so, sd, on, false, sv);
                        is_lit = !sr.ok || len(sub(lpos, r.hit)) < len(sub(sr.hit, r.hit));
                    }
                    lit |= (uint32_t)is_lit << l;
                    ws.tests += (cnt_t)sv.tests * __popcll(__ballot(on));
                    ws.nodes += sv.nodes;
                    ws.leaves += sv.leaves;
                    ws.overflow += sv.overflow;
                }
                if (on) {  // the level's phong and material wait in WorkArgs::refl for the fold
                    const RGB ph = phong(fa, fa.obj[r.obj].m.mats + (size_t)r.mat * 10, r.hit, r.normal, lit);
                    double* const e = wa.refl + ((size_t)(lv - 1) * wa.refl_stride + slot) * kReflD;
                    e[0] = ph.r;
                    e[1] = ph.g;
                    e[2] = ph.b;
                    e[3] = bitsd((uint64_t)r.obj | ((uint64_t)r.mat << 32));
                    levels = lv + 1;
                    D = R;
                    hit = r.hit;
                    N = r.normal;
                }
            }
            if (active) {
                // c_L = ph_L (a chain that ended on a miss: c_add(ph_L, c_mul(Ks_L, black))),
                // then c_k = c_add(ph_k, c_mul(Ks_k, c_(k+1))) down to level 0
                const uint32_t L = levels - 1;
                auto level = [&](uint32_t lv, RGB& ph, RGB& ks) {
                    uint32_t obj = rec.obj, mat = rec.mat;
                    if (lv == 0) {
                        ph = RGB{wa.ph0[3 * slot], wa.ph0[3 * slot + 1], wa.ph0[3 * slot + 2]};
                    } else {
                        const double* e = wa.refl + ((size_t)(lv - 1) * wa.refl_stride + slot) * kReflD;
                        ph = RGB{e[0], e[1], e[2]};
                        const uint64_t om = dbits(e[3]);
                        obj = (uint32_t)om;
                        mat = (uint32_t)(om >> 32);
                    }
                    const double* mt = fa.obj[obj].m.mats + (size_t)mat * 10;
                    ks = RGB{mt[6], mt[7], mt[8]};
                };
                RGB ph, ks;
                level(L, ph, ks);
                RGB c = missed ? c_add(ph, c_mul(ks, RGB{0, 0, 0})) : ph;  // c_reflected = black
                for (int lv = (int)L - 1; lv >= 0; --lv) {
                    level((uint32_t)lv, ph, ks);
                    c = c_add(ph, c_mul(ks, c));
                }
                if (out.rgb) {
                    out.rgb[3 * rec.out] = c.r;
                    out.rgb[3 * rec.out + 1] = c.g;
                    out.rgb[3 * rec.out + 2] = c.b;
                }
                if (out.rgb8) {
                    out.rgb8[3 * rec.out] = c_u8(c.r);
                    out.rgb8[3 * rec.out + 1] = c_u8(c.g);
                    out.rgb8[3 * rec.out + 2] = c_u8(c.b);
                }
                if (out.rgbv) out.rgbv[rec.out] = pack_rgbv(c);
            }
            k = (wa.dynamic & kDynReflect) ? ticket_resolve(nxt) : k + sc.peers();
        }
    }
    // reflection rays and their shadow rays as two extra statistics (per workgroup)
    WaveStats extra{refl_rays, (uint32_t)refl_shadow, 0, 0, 0};  // per wave: well below 2^32
    stats_flush(wa.counters, red, kStatShadowTests, kStatShadowNodes, kStatShadowLeaves, -1, ws);
    __syncthreads();
    stats_flush(wa.counters, red, kStatReflRays, kStatReflShadowRays, -1, -1, extra);
    frame_fold(fa, wa);
}

// Reflections in waves of bounces (the default; MIRT_OPT_REFLECT_CHAINS runs k_reflect above,
// which follows each lane's whole chain).  k_pack first lays the primary hits out in block
// order; per level lv = 1..bounces k_bounce traces one reflection ray per record of level
// lv - 1 (R = D - 2 (D.N) N from hit + 1e-4 R, the nearest hit of tracer.go:27-50) and leaves
// its hits at the input's slots, k_pack compacts them in order, so a wave of 64 records holds
// 64 live rays from a few neighbouring blocks (the chain kernel kept a lane per primary hit
// through every level: 41% of its lanes had a ray at level 1, ~12% at level 4); k_shadow then
// traces level lv's shadow rays and stores its
// phong at the origin slot; k_refl_fold combines the levels per pixel, innermost first.
// One input chunk of a bounce level (k_bounce): its reflection rays' nearest hits, the level's
// records at the input's slots.  true: a second pass is needed (nothing written).
template <bool PREFILTER, bool BRUTE, bool RESIDENT>
__device__ __forceinline__ bool bounce_chunk(const FrameArgs& fa, const WorkArgs& wa, const BounceArgs& ba,
                                             const double* __restrict__ lds, uint32_t q, uint32_t k, uint32_t n,
                                             uint32_t cp, bool pass2, WaveStats& ws, cnt_t& rays, cnt_t& shadow_rays) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lv = ba.level;
        const size_t slot = (size_t)q * wa.hit_cap + (size_t)k * 64 + lane;
        const bool inb = k * 64 + lane < n;
        const HitRec rec = ba.in[inb ? slot : (size_t)q * wa.hit_cap + (size_t)k * 64];
        const bool active = inb && rec.obj != kNoHit;
        const size_t origin = (size_t)rec.out;  // k_pack: the primary hit slot of the chain
        V3 D{1, 0, 0}, hit{0, 0, 0}, N{0, 0, 1};
        if (active) {
            D = vload(ba.in_dir + 3 * slot);
            hit = vload(rec.h);
            N = vload(rec.n);
        }
        const V3 R = sub(D, scale(N, 2 * dot(D, N)));
        const V3 o = add(hit, scale(R, 0.0001));
        Visits vis{0, 0, 0, 0};
        bool redo = false;
        const Nearest r = trace_nearest<false, PREFILTER, BRUTE>(fa, lds, RESIDENT, o, R, active, true, vis, pass2, redo);
        if (redo) {  // wave-uniform: nothing written yet
            ws.tests += (cnt_t)vis.tests * __popcll(__ballot(active));
            ws.nodes += vis.nodes;
            ws.leaves += vis.leaves;
            return true;
        }
        rays += __popcll(__ballot(active));
        ws.tests += (cnt_t)vis.tests * __popcll(__ballot(active));
        ws.nodes += vis.nodes;
        ws.leaves += vis.leaves;
        ws.overflow += vis.overflow;
        const bool got = active && r.ok;
        if (active) ba.chain[origin] = got ? lv + 1 : (lv | 256u);  // levels with phong | missed
        const uint64_t m = __ballot(got);
        shadow_rays += (cnt_t)__popcll(m) * fa.n_lights;
        if (MIRT_BOUNCE_SHADE && m) {
            // the level's shadow rays and phong in this wave (tracer.go:53-77 at the hit;
            // the packed lanes are mostly live): no k_shadow launch per level
            const bool segment = RESIDENT ? !BRUTE : (!BRUTE && fa.n_objects == 1 && !(fa.flags & MIRT_OPT_NO_SEGMENT));
            uint32_t lit = 0;
            for (uint32_t l = 0; l < fa.n_lights; ++l) {
                const V3 lpos{fa.lpos[l][0], fa.lpos[l][1], fa.lpos[l][2]};
                V3 so{0, 0, 0}, sd{1, 0, 0};
                if (got) {
                    sd = norm(sub(lpos, r.hit));
                    so = add(r.hit, scale(sd, 0.0001));
                }
                Visits sv{0, 0, 0, 0};
                bool is_lit;
                if (segment) {
                    is_lit = shadow_lit_single_settled<PREFILTER>(fa, lds, RESIDENT, nullptr, r.hit, so, sd, lpos, l, got, sv);
                } else {
                    const Nearest sr = trace_nearest_settled<false, PREFILTER, BRUTE>(fa, lds, RESIDENT, so, sd, got, false, sv);
                    is_lit = !sr.ok || len(sub(lpos, r.hit)) < len(sub(sr.hit, r.hit));
                }
                lit |= (uint32_t)is_lit << l;
                ws.tests += (cnt_t)sv.tests * __popcll(m);
                ws.nodes += sv.nodes;
                ws.leaves += sv.leaves;
                ws.overflow += sv.overflow;
            }
            if (got) {
                const RGB ph = phong(fa, fa.obj[r.obj].m.mats + (size_t)r.mat * 10, r.hit, r.normal, lit);
                double* const e = wa.refl + ((size_t)(lv - 1) * wa.refl_stride + origin) * kReflD;
                e[0] = ph.r;
                e[1] = ph.g;
                e[2] = ph.b;
            }
        }
        // the level's hits stay at the input's slots; k_pack compacts them in order
        uint64_t* w = (uint64_t*)&ba.out[slot];
        if (got) {
            st64(w + 0, dbits(r.hit.x));
            st64(w + 1, dbits(r.hit.y));
            st64(w + 2, dbits(r.hit.z));
            st64(w + 3, dbits(r.normal.x));
            st64(w + 4, dbits(r.normal.y));
            st64(w + 5, dbits(r.normal.z));
            st64(w + 6, (uint64_t)origin);
            st64(w + 7, (uint64_t)r.obj | ((uint64_t)r.mat << 32));
            vstore(ba.out_dir + 3 * slot, R);
            wa.refl[((size_t)(lv - 1) * wa.refl_stride + origin) * kReflD + 3] =
                bitsd((uint64_t)r.obj | ((uint64_t)r.mat << 32));
        } else {
            st64(w + 7, (uint64_t)kNoHit);
        }
        if (lane == 0) {
            const uint32_t j = q * cp + k;
            ba.src[j] = (uint32_t)(((size_t)q * wa.hit_cap + (size_t)k * 64) / 64 + 1) << 7 | (uint32_t)__popcll(m);
            if (m) atomicAdd(&ba.gcnt[j / kPackGroup], (uint32_t)__popcll(m));
        }
    return false;
}
template <bool PREFILTER, bool BRUTE, bool RESIDENT>
MIRT_TRACE_KERNEL void k_bounce(const FrameArgs fa, const WorkArgs wa, const BounceArgs ba) {
    double* const lds = g_lds_mesh;
    __shared__ cnt_t red[kWG / 64][4];
    if (RESIDENT) {
        stage_tris<false>(lds, fa.obj[0].m.tri, 0, fa.obj[0].m.ntri, V3{0, 0, 0});
        __syncthreads();
    }
    const ShardCursor sc;
    WaveStats ws{0, 0, 0, 0, 0};
    cnt_t rays = 0, shadow_rays = 0;
    // chunks per region of the input, as k_pack published it (high word of its region counts):
    // input chunk (q, k) is source chunk q * cp + k of k_pack
    const uint32_t cp = (uint32_t)(ba.in_cnt[cnt_hits(0)] >> 32);
    for (uint32_t q = sc.first_shard(); q < (uint32_t)kQShards; q += sc.shard_step()) {
        const uint32_t n = *lo32((cnt_t*)&ba.in_cnt[cnt_hits(q)]), nch = (n + 63) / 64;
        for (uint32_t k = sc.rank(); k < nch;) {
            if (bounce_chunk<PREFILTER, BRUTE, RESIDENT>(fa, wa, ba, lds, q, k, n, cp, false, ws, rays, shadow_rays))
                split_redo_push(wa, q, k);  // the same chunk again, every candidate box-gated, at the launch's end
            k += sc.peers();
        }
    }
    if (wa.split_redo) {  // the deferred second passes, in the launch's last workgroup
        const uint32_t last = split_redo_last(wa);
        for (uint32_t e = wave_id(); e < (last & 0x7fffffffu); e += kWG / 64) {
            const uint32_t q = split_redo_entry(wa, e, 0), k = split_redo_entry(wa, e, 1);
            const uint32_t n = *lo32((cnt_t*)&ba.in_cnt[cnt_hits(q)]);
            bounce_chunk<PREFILTER, BRUTE, RESIDENT>(fa, wa, ba, lds, q, k, n, cp, true, ws, rays, shadow_rays);
        }
        split_redo_reset(wa, last);
    }
    WaveStats extra{rays, (uint32_t)shadow_rays, 0, 0, 0};  // per wave: well below 2^32
    stats_flush(wa.counters, red, kStatShadowTests, kStatShadowNodes, kStatShadowLeaves, -1, ws);
    __syncthreads();
    stats_flush(wa.counters, red, kStatReflRays, kStatReflShadowRays, -1, -1, extra);
}

// k_pack (bounce waves): the records of a level compacted in source-chunk order — level 0
// the primary hit blocks in block-table order (column-major 8x8 blocks: neighbours on the
// screen), each later level in its input's order, so a wave of 64 records holds the rays of a
// few adjacent blocks — and dealt evenly over the kQShards regions.  Every workgroup sums the
// chunk counts before its range (and the total) itself: no scan kernel, no second launch.
constexpr int kPackWG = 256;
static_assert(kPackGroup == 64, "k_pack: one source chunk per lane of wave 0");
__device__ __forceinline__ void pack_chunk(const WorkArgs& wa, const PackArgs& pa, uint32_t e, uint32_t off, uint32_t per,
                                           uint32_t lane, uint32_t blk) {
    if ((e & 127u) == 0) return;
    const size_t cs = (size_t)((e >> 7) - 1) * 64;
    const size_t from = cs + lane;
    const uint64_t* w = (const uint64_t*)&pa.in[from];
    // primary chunks with a hit ballot: nothing is read at a missed lane
    const uint64_t m = pa.in_hmask ? u64_uniform(pa.in_hmask[cs / 64]) : __ballot((uint32_t)ld64(w + 7) != kNoHit);
    if (!((m >> lane) & 1u)) return;
    const uint64_t w7 = ld64(w + 7);
    const uint32_t p = off + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    const uint32_t r = p / per, idx = p - r * per;
    const size_t dst = (size_t)r * wa.hit_cap + idx;
    uint64_t v[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) v[q] = ld64(w + q);
    V3 dir;
    if (pa.in_dir) {
        dir = vload(pa.in_dir + 3 * from);
    } else {  // level 0: the primary ray again, from the block's pixel (lane = 8 lx + ly, primary_block)
        const uint32_t pxy = ((const uint32_t*)wa.blocks)[4 * ((size_t)(blk % kQShards) * wa.per_shard + blk / kQShards) + 1];
        dir = primary_dir(pa.rg, (pxy & 0xffffu) + (lane >> 3), (pxy >> 16) + (lane & 7));
    }
    uint64_t* d = (uint64_t*)&pa.out[dst];
#pragma unroll
    for (int q = 0; q < 6; ++q) st64(d + q, v[q]);
    st64(d + 6, pa.level0 ? (uint64_t)from : ld64(w + 6));
    st64(d + 7, w7);
    vstore(pa.out_dir + 3 * dst, dir);
    st32(&pa.out_litw[dst], 0u);
    st32(&pa.out_blkdone[dst / 64], 0u);  // (every record of the chunk: the same zero)
}
__global__ __launch_bounds__(kPackWG) void k_pack(const WorkArgs wa, const PackArgs pa) {
    __shared__ uint32_t s_red[2][kPackWG / 64];
    __shared__ uint32_t s_off[kPackGroup], s_src[kPackGroup];
    __shared__ uint32_t s_nsrc;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) {
        uint32_t n = pa.nsrc;
        if (pa.in_cnt) {
            n = 0;
            for (int q = 0; q < kQShards; ++q) n += (*lo32((cnt_t*)&pa.in_cnt[cnt_hits(q)]) + 63) / 64;
        }
        s_nsrc = n;
    }
    __syncthreads();
    // workgroup w packs source chunks [64 w, 64 w + 64); the records before them and in total
    // come from the producers' per-group counts
    const uint32_t nsrc = s_nsrc, ng = (nsrc + kPackGroup - 1) / kPackGroup;
    const uint32_t j0 = min(nsrc, blockIdx.x * kPackGroup), j1 = min(nsrc, j0 + kPackGroup);
    uint32_t pre = 0, tot = 0;
    for (uint32_t g = tid; g < ng; g += kPackWG) {
        const uint32_t c = pa.gcnt[g];
        tot += c;
        if (g < blockIdx.x) pre += c;
    }
    for (int o = 32; o > 0; o >>= 1) {
        pre += __shfl_xor(pre, o);
        tot += __shfl_xor(tot, o);
    }
    if (lane == 0) {
        s_red[0][wave] = pre;
        s_red[1][wave] = tot;
    }
    if (wave == 0) {  // the group's chunks: exclusive scan of their counts
        const uint32_t e = j0 + lane < j1 ? pa.src[j0 + lane] : 0u, c = e & 127u;
        uint32_t x = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        s_off[lane] = x - c;
        s_src[lane] = e;
    }
    __syncthreads();
    pre = tot = 0;
    for (int k = 0; k < kPackWG / 64; ++k) {
        pre += s_red[0][k];
        tot += s_red[1][k];
    }
    const uint32_t per = ((tot + 63) / 64 + kQShards - 1) / kQShards * 64;  // records per region
    if (blockIdx.x == 0 && tid < (uint32_t)kQShards) {
        // the region's records (low word) and every region's capacity in chunks (high word: the
        // chunk stride k_bounce maps input chunks to source chunks with)
        const uint32_t a = tid * per;
        pa.out_cnt[cnt_hits(tid)] = (cnt_t)(tot > a ? min(per, tot - a) : 0u) | ((cnt_t)(per / 64) << 32);
    }
    for (uint32_t t = wave; t < j1 - j0; t += kPackWG / 64) pack_chunk(wa, pa, s_src[t], pre + s_off[t], per, lane, j0 + t);
}
bool bounce_shades() { return MIRT_BOUNCE_SHADE != 0; }
hipError_t launch_pack(const WorkArgs& wa, const PackArgs& pa, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_pack, dim3(std::max(grid, 1)), dim3(kPackWG), 0, s, wa, pa);
    return hipGetLastError();
}

// The frame's last kernel on the bounce path: per primary hit slot, c_L = ph_L (a chain that
// ended on a miss: c_add(ph_L, c_mul(Ks_L, black))), then c_k = c_add(ph_k, c_mul(Ks_k,
// c_(k+1))) down to level 0 (rt_oracle.c shade_reflect), and the pixel's outputs.
__global__ __launch_bounds__(256) void k_refl_fold(const FrameArgs fa, const WorkArgs wa, OutPlanes out,
                                                   const uint32_t* __restrict__ chain) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * 4 + wave_id(), nw = gridDim.x * 4;
    // one walk over every region's chunks (a loop per region left most waves idle per region)
    __shared__ uint32_t s_first[kQShards + 1];
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int q = 0; q < kQShards; ++q) {
            s_first[q] = acc;
            acc += *lo32(&wa.counters[cnt_hits(q)]) / 64;
        }
        s_first[kQShards] = acc;
    }
    __syncthreads();
    for (uint32_t g = gw, q = 0; g < s_first[kQShards]; g += nw) {
        while (g >= s_first[q + 1]) ++q;
        const uint32_t k = g - s_first[q];
        {
            const size_t slot = (size_t)q * wa.hit_cap + (size_t)k * 64 + lane;
            if (wa.hmask && !((u64_uniform(wa.hmask[slot / 64]) >> lane) & 1u)) continue;
            const HitRec& rec = wa.hits[slot];
            if (!wa.hmask && rec.obj == kNoHit) continue;
            const uint32_t st = chain[slot], L = (st & 0xffu) - 1;
            auto level = [&](uint32_t l, RGB& ph, RGB& ks) {
                uint32_t obj = rec.obj, mat = rec.mat;
                if (l == 0) {
                    ph = RGB{wa.ph0[3 * slot], wa.ph0[3 * slot + 1], wa.ph0[3 * slot + 2]};
                } else {
                    const double* e = wa.refl + ((size_t)(l - 1) * wa.refl_stride + slot) * kReflD;
                    ph = RGB{e[0], e[1], e[2]};
                    const uint64_t om = dbits(e[3]);
                    obj = (uint32_t)om;
                    mat = (uint32_t)(om >> 32);
                }
                const double* mt = fa.obj[obj].m.mats + (size_t)mat * 10;
                ks = RGB{mt[6], mt[7], mt[8]};
            };
            RGB ph, ks;
            level(L, ph, ks);
            RGB c = (st >> 8) ? c_add(ph, c_mul(ks, RGB{0, 0, 0})) : ph;  // c_reflected = black
            for (int l = (int)L - 1; l >= 0; --l) {
                level((uint32_t)l, ph, ks);
                c = c_add(ph, c_mul(ks, c));
            }
            const uint64_t oidx = rec.out;
            if (out.rgb) {
                out.rgb[3 * oidx] = c.r;
                out.rgb[3 * oidx + 1] = c.g;
                out.rgb[3 * oidx + 2] = c.b;
            }
            if (out.rgb8) {
                out.rgb8[3 * oidx] = c_u8(c.r);
                out.rgb8[3 * oidx + 1] = c_u8(c.g);
                out.rgb8[3 * oidx + 2] = c_u8(c.b);
            }
            if (out.rgbv) out.rgbv[oidx] = pack_rgbv(c);
        }
    }
    frame_fold(fa, wa);
}

// ---------------------------------------------------------------- arbitrary rays
template <bool PREFILTER, bool BRUTE, bool RESIDENT>
MIRT_TRACE_KERNEL void k_rays(const FrameArgs fa, RayIO io) {
    double* const lds = g_lds_mesh;  // RESIDENT: the mesh (dynamic LDS sized at launch)
    if (RESIDENT) {
        stage_tris<false>(lds, fa.obj[0].m.tri, 0, fa.obj[0].m.ntri, V3{0, 0, 0});
        __syncthreads();
    }
    const uint64_t nchunks = ((uint64_t)io.n + kWG - 1) / kWG;
    for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
        const uint64_t item = chunk * kWG + threadIdx.x;
        const bool active = item < io.n;
        V3 o{0, 0, 0}, d{1, 0, 0};
        if (active) {
            o = vload(io.orig + 3 * item);
            d = vload(io.dir + 3 * item);
        }
        Visits vis{0, 0, 0, 0};
        Nearest r = trace_nearest_settled<false, PREFILTER, BRUTE>(fa, lds, RESIDENT, o, d, active, true, vis);
        if (active) {
            io.ok[item] = r.ok ? 1 : 0;
            vstore(io.hit + 3 * item, r.ok ? r.hit : V3{0, 0, 0});
            vstore(io.normal + 3 * item, r.ok ? r.normal : V3{0, 0, 0});
            io.face[item] = r.ok ? (int32_t)r.face : -1;
            io.object[item] = r.ok ? (int32_t)r.obj : -1;
        }
    }
}

// ---------------------------------------------------------------- unpack
// packed tile-major planes -> W x H framebuffer, pixel (x, y) at x*H + y.  One workgroup
// per tile (grid-stride over tiles): the tile's descriptor is one scalar load, and the
// tile's column runs are contiguous in both layouts.  A packed rgbv plane with 4-aligned
// columns (tile height, tile row and H multiples of 4: the 32-px multi-GPU tiles) goes four
// pixels per thread — one 16-byte load, the rgb8 run as three dwords, the valid run as one
// — instead of byte stores; anything else goes pixel by pixel.  Planes absent from the
// source are not written.
__device__ __forceinline__ void unpack_pixel(const OutPlanes& src, const OutPlanes& dst, uint64_t p, uint64_t q) {
    if (src.valid && dst.valid) dst.valid[q] = src.valid[p];
    if (src.face && dst.face) dst.face[q] = src.face[p];
    if (src.object && dst.object) dst.object[q] = src.object[p];
    if (src.rgb && dst.rgb) {
        dst.rgb[3 * q] = src.rgb[3 * p];
        dst.rgb[3 * q + 1] = src.rgb[3 * p + 1];
        dst.rgb[3 * q + 2] = src.rgb[3 * p + 2];
    }
    if (src.rgb8 && dst.rgb8) {
        dst.rgb8[3 * q] = src.rgb8[3 * p];
        dst.rgb8[3 * q + 1] = src.rgb8[3 * p + 1];
        dst.rgb8[3 * q + 2] = src.rgb8[3 * p + 2];
    }
    if (src.rgbv) {  // packed word -> rgb8 + valid (and/or a packed framebuffer)
        const uint32_t v = src.rgbv[p];
        if (dst.rgbv) dst.rgbv[q] = v;
        if (dst.valid && !src.valid) dst.valid[q] = (uint8_t)(v >> 24);
        if (dst.rgb8 && !src.rgb8) {
            dst.rgb8[3 * q] = (uint8_t)v;
            dst.rgb8[3 * q + 1] = (uint8_t)(v >> 8);
            dst.rgb8[3 * q + 2] = (uint8_t)(v >> 16);
        }
    }
}
// Grid: x runs over tiles, y over 1024-pixel chunks of a tile (a chunk per workgroup, a
// 4-pixel group per thread), so a frame of few large tiles (full-height strips) still
// spreads over thousands of short workgroups instead of a few long per-tile loops.
constexpr uint32_t kUnpackChunk = 1024;
__global__ __launch_bounds__(256) void k_unpack(const TileDesc* __restrict__ tiles, uint32_t ntiles, uint32_t H,
                                                OutPlanes src, OutPlanes dst) {
    const bool only_rgbv = src.rgbv && !src.rgb && !src.rgb8 && !src.valid && !src.face && !src.object;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t tt = __builtin_amdgcn_readfirstlane(t);
        const TileDesc td = tiles[tt];
        const uint32_t n = td.w * td.h;  // w, h <= 65535
        for (uint32_t c0 = blockIdx.y * kUnpackChunk; c0 < n; c0 += gridDim.y * kUnpackChunk) {
            if (only_rgbv && (td.h & 3u) == 0 && (td.y & 3u) == 0 && (H & 3u) == 0 && (td.out_off & 3u) == 0) {
                const uint32_t local = c0 + threadIdx.x * 4;
                if (local >= n) continue;
                const uint32_t lx = local / td.h, ly = local - lx * td.h;
                const uint64_t q = (uint64_t)(td.x + lx) * H + (td.y + ly);  // multiple of 4
                const uint4 v = *(const uint4*)(src.rgbv + td.out_off + local);
                if (dst.rgbv) *(uint4*)(dst.rgbv + q) = v;
                if (dst.valid)
                    *(uint32_t*)(dst.valid + q) = (v.x >> 24) | ((v.y >> 24) << 8) | ((v.z >> 24) << 16) | ((v.w >> 24) << 24);
                if (dst.rgb8) {  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3 (3q is a multiple of 4)
                    uint32_t* o = (uint32_t*)(dst.rgb8 + 3 * q);
                    o[0] = (v.x & 0xffffffu) | (v.y << 24);
                    o[1] = ((v.y >> 8) & 0xffffu) | (v.z << 16);
                    o[2] = ((v.z >> 16) & 0xffu) | ((v.w & 0xffffffu) << 8);
                }
            } else {
                const uint32_t end = min(n, c0 + kUnpackChunk);
                for (uint32_t local = c0 + threadIdx.x; local < end; local += blockDim.x) {
                    const uint32_t lx = local / td.h, ly = local - lx * td.h;
                    unpack_pixel(src, dst, td.out_off + local, (uint64_t)(td.x + lx) * H + (td.y + ly));
                }
            }
        }
    }
}

// ---------------------------------------------------------------- diagnostics
__global__ __launch_bounds__(256) void k_debug_fp64(int op, uint32_t n, const double* __restrict__ a,
                                                    const double* __restrict__ b, double* __restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double r;
    if (op == 4) {  // box.go:29-68 as the kernels evaluate it: ray i = a[6i..], box i = b[6i..]
        const double* ray = a + 6 * (size_t)i;
        out[i] = box_gate(box_load(b + 6 * (size_t)i), V3{ray[0], ray[1], ray[2]}, V3{ray[3], ray[4], ray[5]}, true) ? 1.0 : 0.0;
        return;
    }
    switch (op) {
        case 0: r = sqrt(a[i]); break;
        case 1: r = a[i] / b[i]; break;
        case 2: r = go_pow(a[i], b[i]); break;
        default: r = go_max(a[i], b[i]); break;
    }
    out[i] = r;
}

// ---------------------------------------------------------------- launchers
// opts: MIRT_OPT_* bits (mirt.h); resident: one object whose mesh fits in LDS.
#define MIRT_DISPATCH(KERNEL)                                                                      \
    do {                                                                                           \
        const bool pre = !(opts & MIRT_OPT_NO_PREFILTER), brute = (opts & MIRT_OPT_BRUTE_FORCE) != 0; \
        if (resident) {                                                                            \
            if (pre && !brute) KERNEL(true, false, true);                                          \
            else if (pre) KERNEL(true, true, true);                                                \
            else if (!brute) KERNEL(false, false, true);                                           \
            else KERNEL(false, true, true);                                                        \
        } else {                                                                                   \
            if (pre && !brute) KERNEL(true, false, false);                                         \
            else if (pre) KERNEL(true, true, false);                                               \
            else if (!brute) KERNEL(false, false, false);                                          \
            else KERNEL(false, true, false);                                                       \
        }                                                                                          \
    } while (0)

// (the MIRT_OPT_NO_SEGMENT ablation runs the general kernels, so the resident ones carry
// only the segment query for shadow rays)
static bool is_resident(const FrameArgs& fa) {
    return MIRT_LDS_MESH && fa.n_objects == 1 && fa.obj[0].m.ntri <= (uint32_t)kLdsTris &&
           fa.obj[0].m.depth <= (uint32_t)kBvhShallowDepth && !(fa.flags & MIRT_OPT_NO_SEGMENT);
}
// dynamic LDS bytes of a RESIDENT launch: the mesh
static size_t mesh_lds_bytes(const FrameArgs& fa) { return (size_t)fa.obj[0].m.ntri * kTriD * sizeof(double); }

hipError_t launch_primary(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, int grid, uint32_t opts,
                          hipStream_t s) {
    const bool resident = is_resident(fa);
    const size_t dyn = resident ? mesh_lds_bytes(fa) : 0;
#define K_PRIM(P, B, R) hipLaunchKernelGGL((k_primary<P, B, R>), dim3(grid), dim3(kWG), (R) ? dyn : 0, s, fa, wa, out)
    MIRT_DISPATCH(K_PRIM);
#undef K_PRIM
    return hipGetLastError();
}

hipError_t launch_shadow(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, int grid, uint32_t opts,
                         hipStream_t s) {
    const bool resident = is_resident(fa);
    const size_t dyn = resident ? mesh_lds_bytes(fa) : 0;
#define K_SHADOW(P, B, R) hipLaunchKernelGGL((k_shadow<P, B, R>), dim3(grid), dim3(kWG), (R) ? dyn : 0, s, fa, wa, out)
    MIRT_DISPATCH(K_SHADOW);
#undef K_SHADOW
    return hipGetLastError();
}

hipError_t launch_rays(const FrameArgs& fa, const RayIO& io, int grid, uint32_t opts, hipStream_t s) {
    const bool resident = is_resident(fa);
    const size_t dyn = resident ? mesh_lds_bytes(fa) : 0;
#define K_RAYS(P, B, R) hipLaunchKernelGGL((k_rays<P, B, R>), dim3(grid), dim3(kWG), (R) ? dyn : 0, s, fa, io)
    MIRT_DISPATCH(K_RAYS);
#undef K_RAYS
    return hipGetLastError();
}

hipError_t launch_reflect(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, int grid, uint32_t opts,
                          hipStream_t s) {
    const bool resident = is_resident(fa);
    const size_t dyn = resident ? mesh_lds_bytes(fa) : 0;
#define K_REFLECT(P, B, R) hipLaunchKernelGGL((k_reflect<P, B, R>), dim3(grid), dim3(kWG), (R) ? dyn : 0, s, fa, wa, out)
    MIRT_DISPATCH(K_REFLECT);
#undef K_REFLECT
    return hipGetLastError();
}

hipError_t launch_bounce(const FrameArgs& fa, const WorkArgs& wa, const BounceArgs& ba, int grid, uint32_t opts,
                         hipStream_t s) {
    const bool resident = is_resident(fa);
    const size_t dyn = resident ? mesh_lds_bytes(fa) : 0;
#define K_BOUNCE(P, B, R) hipLaunchKernelGGL((k_bounce<P, B, R>), dim3(grid), dim3(kWG), (R) ? dyn : 0, s, fa, wa, ba)
    MIRT_DISPATCH(K_BOUNCE);
#undef K_BOUNCE
    return hipGetLastError();
}

hipError_t launch_refl_fold(const FrameArgs& fa, const WorkArgs& wa, const OutPlanes& out, const uint32_t* chain,
                            int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_refl_fold, dim3(std::max(grid, 1)), dim3(256), 0, s, fa, wa, out, chain);
    return hipGetLastError();
}

hipError_t launch_trace(const FrameRecs& recs, const WorkArgs& wa, const FusedCopy& fc, int grid, uint32_t opts,
                        hipStream_t s) {
    const FrameArgs& fa = recs.r[0].fa;
    // MIRT_FORCE_STREAM=1 (experiment): LDS-sized meshes too take the streamed HBM path, whose
    // workgroups hold ~23 KB of LDS instead of the whole mesh
    static const bool force_stream = [] {
        const char* e = getenv("MIRT_FORCE_STREAM");
        return e && e[0] == '1';
    }();
    const bool resident = is_resident(fa) && !force_stream;
    // an HBM mesh streamed through LDS (the default; MIRT_OPT_NO_LDS_STREAM reads it with scalar
    // loads): one chunk slice per wave
    // a one-object frame of an HBM mesh with segment shadows and the default test (HBM1 > 0: the
    // kernel takes the object count and the shadow mode as constants), streamed through LDS or not
    const bool one_hbm = !resident && fa.n_objects == 1 && !(fa.flags & MIRT_OPT_NO_SEGMENT) &&
                         !(opts & (MIRT_OPT_BRUTE_FORCE | MIRT_OPT_NO_PREFILTER)) && MIRT_HBM1;
    const bool stream = one_hbm && !(fa.flags & MIRT_OPT_NO_LDS_STREAM);
    const size_t dyn = resident ? std::max(mesh_lds_bytes(fa), wa.views ? kViewScratchBytes : (size_t)0)
                                : (stream ? kStreamBytes : 0);
#define K_TRACE(P, B, R) hipLaunchKernelGGL((k_trace<P, B, R>), dim3(grid), dim3(kWG), dyn, s, recs, wa, fc)
    if (wa.views && resident && !(opts & (MIRT_OPT_BRUTE_FORCE | MIRT_OPT_NO_PREFILTER)))
        hipLaunchKernelGGL((k_trace<true, false, true, true>), dim3(grid), dim3(kWG), dyn, s, recs, wa, fc);
    else if (stream)
        hipLaunchKernelGGL((k_trace<true, false, false, false, 2>), dim3(grid), dim3(kWG), dyn, s, recs, wa, fc);
    else if (one_hbm)
        hipLaunchKernelGGL((k_trace<true, false, false, false, 1>), dim3(grid), dim3(kWG), dyn, s, recs, wa, fc);
    else
        MIRT_DISPATCH(K_TRACE);
#undef K_TRACE
    return hipGetLastError();
}

hipError_t launch_unpack(const TileDesc* tiles, uint32_t ntiles, uint64_t max_tile_px, uint32_t H, const OutPlanes& src,
                         const OutPlanes& dst, hipStream_t s) {
    const uint32_t gx = ntiles < 8192u ? (ntiles ? ntiles : 1u) : 8192u;
    const uint64_t chunks = (max_tile_px + kUnpackChunk - 1) / kUnpackChunk;
    const uint32_t gy = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(chunks, std::max<uint64_t>(1, 16384 / gx)));
    hipLaunchKernelGGL(k_unpack, dim3(gx, gy), dim3(256), 0, s, tiles, ntiles, H, src, dst);
    return hipGetLastError();
}

// The transfer form of the multi-GPU frame (mirt_group): for each of a rank's tiles only
// its pixels inside the frame's hit rectangle (mirt.cpp hit_rect: no pixel outside it can
// meet the object), column-major per tile, tiles back to back, as rgbv words.  Every rank
// derives the same rectangle from the same frame, so the sizes need no exchange.
__device__ __forceinline__ uint32_t tile_rect(const TileDesc& td, const uint32_t* R, uint32_t& cx0, uint32_t& cy0,
                                              uint32_t& cw, uint32_t& ch) {
    cx0 = max(td.x, R[0]);
    cy0 = max(td.y, R[1]);
    const uint32_t cx1 = min(td.x + td.w, R[2]), cy1 = min(td.y + td.h, R[3]);
    cw = cx1 > cx0 ? cx1 - cx0 : 0u;
    ch = cy1 > cy0 ? cy1 - cy0 : 0u;
    return cw * ch;
}
// words of tiles [first, t) inside R (tiles of one rank are contiguous in the table): the
// wave's lanes take every 64th tile, then a butterfly sum (every wave computes it)
__device__ __forceinline__ uint64_t rect_offset(const TileDesc* __restrict__ tiles, uint32_t first, uint32_t t,
                                                const uint32_t* R) {
    uint32_t acc = 0;  // < W * H < 2^32
    for (uint32_t u = first + (threadIdx.x & 63); u < t; u += 64) {
        uint32_t a, b, c, d;
        acc += tile_rect(tiles[u], R, a, b, c, d);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    return acc;
}
// grid x: the rank's tiles, z: the frame of the batch
__global__ __launch_bounds__(256) void k_pack_rect(const TileDesc* __restrict__ tiles, uint32_t ntiles, RectJobs jobs) {
    const uint32_t f = blockIdx.z;
    const uint32_t* R = jobs.rect[f];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t tt = __builtin_amdgcn_readfirstlane(t);
        const TileDesc td = tiles[tt];
        uint32_t cx0, cy0, cw, ch;
        const uint32_t n = tile_rect(td, R, cx0, cy0, cw, ch);
        if (n == 0) continue;
        const uint64_t off = rect_offset(tiles, 0, tt, R);
        const uint32_t* __restrict__ src = jobs.src[f] + td.out_off;
        uint32_t* __restrict__ dst = jobs.dst[f] + off;
        for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) {
            const uint32_t lx = p / ch, ly = p - lx * ch;
            dst[p] = src[(uint64_t)(cx0 - td.x + lx) * td.h + (cy0 - td.y + ly)];
        }
    }
    // the trailer right after the data: {frame tag, words} (mirt_internal.hpp kTrailerWords)
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        const uint64_t total = rect_offset(tiles, 0, ntiles, R);
        if (threadIdx.x == 0) {
            jobs.dst[f][total] = jobs.tag[f];
            jobs.dst[f][total + 1] = (uint32_t)total;
        }
    }
}

// Root, before the unpack: region r of the gathered plane must end with the trailer of this
// frame at the word count its tiles give inside the hit rectangle; writes bad[f][r]
// (host-visible).  One wave; run by k_unpack_rect's workgroups (x, 0, f) for the regions x,
// x + gridDim.x, ...
__device__ __forceinline__ void check_region(const TileDesc* __restrict__ tiles, const RegionDesc& rd, uint32_t r,
                                             uint64_t stride, const RectJobs& jobs, uint32_t f) {
    const uint64_t total = rect_offset(tiles, rd.first, rd.first + rd.count, jobs.rect[f]);
    if ((threadIdx.x & 63) == 0) {
        const uint32_t* t = jobs.src[f] + (uint64_t)r * stride + total;
        const bool ok = total + kTrailerWords <= stride && t[0] == jobs.tag[f] && t[1] == (uint32_t)total;
        jobs.bad[f][r] = ok ? 0 : 1;
    }
}
hipError_t launch_pack_rect(const TileDesc* tiles, uint32_t ntiles, const RectJobs& jobs, uint32_t nframes,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_pack_rect, dim3(ntiles ? ntiles : 1u, 1, nframes), dim3(256), 0, s, tiles, ntiles, jobs);
    return hipGetLastError();
}

// Gathered regions (rank r at word r * cap) -> framebuffer planes; pixels outside the hit
// rectangle are misses; only the columns [ucol[f][0], ucol[f][1]) are written (every other
// column of the slot's framebuffer holds misses already).  Grid as k_unpack (x: tile, y:
// 1024-pixel chunk), z: frame.  With regions, the workgroups of y == 0 first check the
// regions' trailers (the check of a frame never waits for its unpack: both only read src).
__global__ __launch_bounds__(256) void k_unpack_rect(const TileDesc* __restrict__ tiles, uint32_t ntiles, uint32_t H,
                                                     uint64_t cap, const RegionDesc* __restrict__ regions,
                                                     uint32_t nregions, RectJobs jobs) {
    const uint32_t f = blockIdx.z;
    const uint32_t* R = jobs.rect[f];
    const OutPlanes dst = jobs.out[f];
    if (regions && blockIdx.y == 0 && threadIdx.x < 64)
        for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x)
            check_region(tiles, regions[r], r, cap, jobs, f);
    const uint32_t u0 = jobs.ucol[f][0], u1 = jobs.ucol[f][1];
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t tt = __builtin_amdgcn_readfirstlane(t);
        const TileDesc td = tiles[tt];
        if (td.x + td.w <= u0 || td.x >= u1) continue;  // no column of this tile can change
        uint32_t cx0, cy0, cw, ch;
        tile_rect(td, R, cx0, cy0, cw, ch);
        const uint64_t off = rect_offset(tiles, td.pad, tt, R);  // pad: the region's first tile
        const uint32_t* __restrict__ src = jobs.src[f] + (uint64_t)td.region * cap + off;
        const uint32_t n = td.w * td.h;
        const bool fast = (td.h & 3u) == 0 && (td.y & 3u) == 0 && (H & 3u) == 0;
        for (uint32_t c0 = blockIdx.y * kUnpackChunk; c0 < n; c0 += gridDim.y * kUnpackChunk) {
            if (fast) {  // 4 pixels of one column per thread: 16-byte / 4-byte aligned stores
                const uint32_t local = c0 + threadIdx.x * 4;
                if (local >= n) continue;
                const uint32_t lx = local / td.h, ly = local - lx * td.h;
                const uint32_t X = td.x + lx, Y = td.y + ly;
                if (X < u0 || X >= u1) continue;
                const bool xin = X >= cx0 && X < cx0 + cw;
                uint32_t v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t y = Y + k;
                    v[k] = xin && y >= cy0 && y < cy0 + ch ? src[(uint64_t)(X - cx0) * ch + (y - cy0)] : 0u;
                }
                const uint64_t q = (uint64_t)X * H + Y;  // multiple of 4
                if (dst.rgbv) *(uint4*)(dst.rgbv + q) = make_uint4(v[0], v[1], v[2], v[3]);
                if (dst.valid)
                    *(uint32_t*)(dst.valid + q) = (v[0] >> 24) | ((v[1] >> 24) << 8) | ((v[2] >> 24) << 16) |
                                                  ((v[3] >> 24) << 24);
                if (dst.rgb8) {  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
                    uint32_t* o = (uint32_t*)(dst.rgb8 + 3 * q);
                    o[0] = (v[0] & 0xffffffu) | (v[1] << 24);
                    o[1] = ((v[1] >> 8) & 0xffffu) | (v[2] << 16);
                    o[2] = ((v[2] >> 16) & 0xffu) | ((v[3] & 0xffffffu) << 8);
                }
                continue;
            }
            const uint32_t end = min(n, c0 + kUnpackChunk);
            for (uint32_t local = c0 + threadIdx.x; local < end; local += blockDim.x) {
                const uint32_t lx = local / td.h, ly = local - lx * td.h;
                const uint32_t X = td.x + lx, Y = td.y + ly;
                if (X < u0 || X >= u1) continue;
                const bool in = X >= cx0 && X < cx0 + cw && Y >= cy0 && Y < cy0 + ch;
                const uint32_t v = in ? src[(uint64_t)(X - cx0) * ch + (Y - cy0)] : 0u;
                const uint64_t q = (uint64_t)X * H + Y;
                if (dst.rgbv) dst.rgbv[q] = v;
                if (dst.valid) dst.valid[q] = (uint8_t)(v >> 24);
                if (dst.rgb8) {
                    dst.rgb8[3 * q] = (uint8_t)v;
                    dst.rgb8[3 * q + 1] = (uint8_t)(v >> 8);
                    dst.rgb8[3 * q + 2] = (uint8_t)(v >> 16);
                }
            }
        }
    }
}
hipError_t launch_unpack_rect(const TileDesc* tiles, uint32_t ntiles, uint64_t max_tile_px, uint32_t H, uint64_t cap,
                              const RegionDesc* regions, uint32_t nregions, const RectJobs& jobs, uint32_t nframes,
                              hipStream_t s) {
    const uint32_t gx = ntiles < 8192u ? (ntiles ? ntiles : 1u) : 8192u;
    const uint64_t chunks = (max_tile_px + kUnpackChunk - 1) / kUnpackChunk;
    const uint32_t gy = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(chunks, std::max<uint64_t>(1, 16384 / gx)));
    hipLaunchKernelGGL(k_unpack_rect, dim3(gx, gy, nframes), dim3(256), 0, s, tiles, ntiles, H, cap, regions, nregions,
                       jobs);
    return hipGetLastError();
}

// grid x: groups of 4 columns (one wave each), z: frame.  Column x holds rows contiguously
// in both planes (x * H + y).  The column's hit span is found from the valid plane inside
// this frame's hit rectangle (64 rows per step, from each end inwards: the rows inside the
// span are never read); the rows of its union with the span the host slot held are
// copied.  Waves are independent (no barrier), so a column's wave retires as soon as its
// copy is issued.
__global__ __launch_bounds__(256) void k_copy_rect_host(HostCopyJobs jobs, uint32_t H) {
    const uint32_t f = blockIdx.z, lane = threadIdx.x & 63;
    const uint32_t* R = jobs.rect[f];
    for (uint32_t x = R[0] + blockIdx.x * 4 + wave_id(); x < R[2]; x += gridDim.x * 4) copy_column(jobs, f, x, H, lane);
}
hipError_t launch_copy_rect_host(const HostCopyJobs& jobs, uint32_t nframes, uint32_t H, uint32_t max_cols,
                                 hipStream_t s) {
    const uint32_t gx = std::max<uint32_t>(1, std::min<uint32_t>((max_cols + 3) / 4, 1024));
    hipLaunchKernelGGL(k_copy_rect_host, dim3(gx, 1, nframes), dim3(256), 0, s, jobs, H);
    return hipGetLastError();
}

// Copy a launch's frame records from pinned host memory to the device (one workgroup; a
// hipMemcpyAsync of a few KB from pinned memory held the host until the stream got there).
// launch_fill_planes: grid x over 64 KiB chunks, y over planes, z over frames; 16-byte
// stores (planes are hipMalloc'd, so 256-byte aligned), the tail byte by byte.
__global__ __launch_bounds__(256) void k_fill_planes(FillJobs jobs) {
    const uint32_t f = blockIdx.z, p = blockIdx.y;
    uint8_t* dst = jobs.ptr[f][p];
    if (!dst) return;
    const uint64_t n = jobs.bytes[f][p];
    const uint32_t v8 = jobs.value[f][p];
    const uint32_t w = v8 | v8 << 8 | v8 << 16 | v8 << 24;
    const uint4 q = make_uint4(w, w, w, w);
    const uint64_t n16 = n / 16;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        ((uint4*)dst)[i] = q;
    if (blockIdx.x == 0 && threadIdx.x < (n & 15)) dst[n16 * 16 + threadIdx.x] = (uint8_t)v8;
}

hipError_t launch_fill_planes(const FillJobs& jobs, uint32_t nframes, uint64_t max_bytes, hipStream_t s) {
    if (nframes == 0 || max_bytes == 0) return hipSuccess;
    const uint32_t gx = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((max_bytes / 16 + 4095) / 4096, 1024));
    hipLaunchKernelGGL(k_fill_planes, dim3(gx, kFillPlanes, nframes), dim3(256), 0, s, jobs);
    return hipGetLastError();
}

// One light table, one thread per (light, triangle) record, on the stream of
// the first frame that reads it (mirt.cpp lt_launch): lighttab.hpp's arithmetic, the host
// builder's bits.
__global__ __launch_bounds__(256) void k_light_table(const LightTabArgs a) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)a.n * a.nl) return;
    const uint32_t l = (uint32_t)(i / a.n);
    const size_t k = i - (size_t)l * a.n;
    const LightGeom g = light_geom(a.lpos[l], a.pos, a.scale);
    float r[kLtD];
    light_record(a.tri + k * kTriD, g, r);
    float4* o = (float4*)(a.out + i * kLtD);
#pragma unroll
    for (int q = 0; q < kLtD / 4; ++q) o[q] = make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
}
hipError_t launch_light_table(const LightTabArgs& a, hipStream_t s) {
    const size_t n = (size_t)a.n * a.nl;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_light_table, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_debug_fp64(int op, uint32_t n, const double* a, const double* b, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_fp64, dim3((n + 255) / 256), dim3(256), 0, s, op, n, a, b, out);
    return hipGetLastError();
}

hipError_t read_diag_counters(uint64_t* out, uint32_t n) {
    unsigned long long h[8 * kDiagN];
    hipError_t e = hipMemcpyFromSymbol(h, HIP_SYMBOL(g_diag), sizeof(h), 0, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    for (uint32_t k = 0; k < n && k < (uint32_t)kDiagN; ++k) {
        out[k] = 0;
        for (int sh = 0; sh < 8; ++sh) out[k] += h[sh * kDiagN + k];
    }
    for (auto& x : h) x = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_diag), h, sizeof(h), 0, hipMemcpyHostToDevice);
}

}  // namespace mirt
