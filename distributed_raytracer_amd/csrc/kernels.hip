// kernels.hip — CDNA4 (gfx950) kernels of the trace worker.
//
// Replaces, per pixel of a tile, worker/shared/tracer/tracer.go:81-91 Trace:
//   k_primary   pixelToPoint + primary dir (tracer.go:15-22, 83-86), brute-force
//               nearest hit over every triangle of every object (tracer.go:27-50,
//               object.go:63-110, triangle.go:37-77), miss outputs, hit compaction.
//   k_secondary shadow rays of phong (tracer.go:60-64): one lane per (hit, light), or
//               arbitrary rays for mirt_trace_rays (tracer.go:27-50).
//   k_shade     Phong (tracer.go:53-77) with the colour clamping of colour.go:38-50 and
//               uint8(255*c) packing (colour.go:59-61, worker/distributed/main.go:79-86).
//   k_unpack    framebuffer assembly after the multi-GPU gather.
//
// Mapping: one lane = one ray, wave64 over an 8x8 pixel block (coherent branches).
// Triangles are staged cooperatively into LDS (72 B each) and read wave-uniformly, i.e.
// as LDS broadcasts; meshes of <= kLdsTris triangles stay LDS-resident for the life of
// a persistent workgroup.  The running nearest hit is a per-lane (distance, face) pair;
// the winner's normal/material are recomputed once after the sweep (bit-identical).
//
// Numerics: fp64, built with -ffp-contract=off, the reference's operation order, true
// IEEE division, correctly rounded sqrt.  Hit/miss and the nearest-hit choice are
// therefore bit-identical to the CPU restatement.
#include "gomath.hpp"
#include "mirt_internal.hpp"

namespace mirt {

__device__ __forceinline__ V3 vload(const double* p) { return V3{p[0], p[1], p[2]}; }
__device__ __forceinline__ void vstore(double* p, V3 v) {
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}

// Sound pre-reject for the first barycentric test of triangle.go:50-53:
//   r2 = fl(n / d);  test 0 <= r2 <= 1.
// Returns true only when that test certainly FAILS, without dividing.  Valid for
// 2^-900 <= |d| <= 2^900 (outside: never rejects, the exact path decides):
//  * opposite signs and |n| * 2^1000 > |d|: q < -2^-1000, so fl(q) < 0 (not -0);
//  * same signs and |n| > fl(|d| (1 + 2^-50)) >= |d| (1 + 2^-51): fl(q) > 1.
// Scaling by 2^1000 is exact (or overflows to +inf, which is also a correct reject).
__device__ __forceinline__ bool r2_certainly_out(double n, double d) {
    double an = __builtin_fabs(n), ad = __builtin_fabs(d);
    bool in_range = ad >= 0x1p-900 && ad <= 0x1p900;
    bool opp = (n < 0.0) != (d < 0.0);
    bool neg_out = n != 0.0 && opp && an * 0x1p1000 > ad;
    bool big_out = !opp && an > ad * (1.0 + 0x1p-50);
    return in_range && (neg_out || big_out);
}

// Möller–Trumbore exactly as triangle.go:37-77, on (p1or = O - P1, E1, E2), returning
// only the hit decision and the ray parameter.  neg = D * -1 (triangle.go:38).
template <bool PREFILTER>
__device__ __forceinline__ bool mt_test(V3 p1or, V3 e1, V3 e2, V3 neg, double& t_out) {
    V3 c = cross(e2, neg);
    double inc = dot(e1, c);
    if (inc != 0.0) {
        double n2 = dot(p1or, c);
        if (PREFILTER && r2_certainly_out(n2, inc)) return false;
        double r2 = n2 / inc;
        if (0.0 <= r2 && r2 <= 1.0) {
            double r3 = dot(e1, cross(p1or, neg)) / inc;
            if (0.0 <= r2 + r3 && r2 + r3 <= 1.0) {
                double r1 = 1.0 - r2 - r3;
                if (r1 >= 0.0 && r2 >= 0.0 && r3 >= 0.0) {
                    double t = dot(e1, cross(e2, p1or)) / inc;
                    if (t >= 0.0) {
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

// Stage triangles [base, base+n) of a mesh into LDS.  REL: store p1or = ro - P1 instead
// of P1 (primary rays share one origin per object, so object.go:71 + triangle.go:48's
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

// Sweep n staged triangles for one ray; object.go:97-103 nearest rule (strict <, the
// first face reaching the minimum distance wins in ascending face order).
template <bool REL, bool PREFILTER>
__device__ __forceinline__ void sweep(const double* __restrict__ s, uint32_t n, uint32_t base, V3 ro, V3 d, V3 neg,
                                      bool& has, double& bestd, uint32_t& bface) {
#pragma unroll 2
    for (uint32_t k = 0; k < n; ++k) {
        const double* t = s + (size_t)k * kTriD;
        V3 p1or = REL ? V3{t[0], t[1], t[2]} : sub(ro, V3{t[0], t[1], t[2]});
        V3 e1{t[3], t[4], t[5]};
        V3 e2{t[6], t[7], t[8]};
        double tt;
        if (mt_test<PREFILTER>(p1or, e1, e2, neg, tt)) {
            V3 ip = add(ro, scale(d, tt));         // triangle.go:69
            double dist = len(sub(ro, ip));        // object.go:97
            if (!has || dist < bestd) {
                has = true;
                bestd = dist;
                bface = base + k;
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
__device__ __forceinline__ void winner(const DevObject& ob, uint32_t f, V3 ro, V3 d, V3 neg, V3& world,
                                       V3& normal, uint32_t& mat, bool want_normal) {
    const double* t = ob.m.tri + (size_t)f * kTriD;
    V3 p1 = vload(t), e1 = vload(t + 3), e2 = vload(t + 6);
    double tt = 0, r1 = 0, r2 = 0, r3 = 0;
    mt_full(sub(ro, p1), e1, e2, neg, tt, r1, r2, r3);
    V3 ip = add(ro, scale(d, tt));
    world = add(ip, V3{ob.pos[0], ob.pos[1], ob.pos[2]});  // object.go:109
    if (want_normal) {
        if (ob.m.has_normals) {
            const double* nn = ob.m.vnrm + (size_t)f * kTriD;
            // triangle.go:29-31: ((N1*r1 + N2*r2) + N3*r3).Norm()
            normal = norm(add(add(scale(vload(nn), r1), scale(vload(nn + 3), r2)), scale(vload(nn + 6), r3)));
        } else {
            // triangle.go:24-26: (P2-P1) x (P3-P1) normalised
            normal = norm(cross(e1, e2));
        }
        mat = ob.m.fmat[f];
    }
}

// tracer.go:27-50: nearest over objects by |hit - Cam.Pos| (also for shadow rays).
// REL (primary rays only) requires every lane of the workgroup to share `o`.
template <bool REL, bool PREFILTER>
__device__ Nearest trace_nearest(const FrameArgs& fa, double* __restrict__ lds, bool resident, V3 o, V3 d,
                                 bool want_normal) {
    Nearest best;
    best.ok = false;
    best.obj = best.face = best.mat = 0;
    best.hit = best.normal = V3{0, 0, 0};
    double bestcd = 0;
    V3 neg = scale(d, -1);  // triangle.go:38 rDir.Scale(-1)
    V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    for (uint32_t oi = 0; oi < fa.n_objects; ++oi) {
        const DevObject& ob = fa.obj[oi];
        V3 ro = sub(o, V3{ob.pos[0], ob.pos[1], ob.pos[2]});  // object.go:71
        bool has = false;
        double bestd = 0;
        uint32_t bface = 0;
        const uint32_t ntri = ob.m.ntri;
        if (resident) {
            sweep<REL, PREFILTER>(lds, ntri, 0, ro, d, neg, has, bestd, bface);
        } else {
            for (uint32_t base = 0; base < ntri; base += kLdsTris) {
                uint32_t n = min((uint32_t)kLdsTris, ntri - base);
                __syncthreads();
                stage_tris<REL>(lds, ob.m.tri, base, n, ro);
                __syncthreads();
                sweep<REL, PREFILTER>(lds, n, base, ro, d, neg, has, bestd, bface);
            }
        }
        if (has) {
            V3 world, normal{0, 0, 0};
            uint32_t mat = 0;
            winner(ob, bface, ro, d, neg, world, normal, mat, want_normal);
            double cd = len(sub(world, cam));  // tracer.go:38
            if (!best.ok || cd < bestcd) {
                best.ok = true;
                bestcd = cd;
                best.obj = oi;
                best.face = bface;
                best.mat = mat;
                best.hit = world;
                best.normal = normal;
            }
        }
    }
    return best;
}

__device__ __forceinline__ uint32_t find_tile(const TileDesc* __restrict__ tiles, uint32_t ntiles, uint32_t unit) {
    uint32_t lo = 0, hi = ntiles - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi + 1) >> 1;
        if (tiles[mid].unit_begin <= unit)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

// ---------------------------------------------------------------- primary
template <bool PREFILTER>
__global__ __launch_bounds__(kWG, 4) void k_primary(const FrameArgs fa, const TileDesc* __restrict__ tiles,
                                                     uint32_t ntiles, uint32_t total_units, OutPlanes out,
                                                     HitRec* __restrict__ hits, uint32_t* __restrict__ counters) {
    __shared__ __attribute__((aligned(16))) double lds[kLdsTris * kTriD];
    const bool resident = fa.n_objects == 1 && fa.obj[0].m.ntri <= (uint32_t)kLdsTris;
    V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    if (resident) {
        const DevObject& ob = fa.obj[0];
        stage_tris<true>(lds, ob.m.tri, 0, ob.m.ntri, sub(cam, V3{ob.pos[0], ob.pos[1], ob.pos[2]}));
        __syncthreads();
    }
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t unit = blockIdx.x; unit < total_units; unit += gridDim.x) {
        const uint32_t ti = find_tile(tiles, ntiles, unit);
        const TileDesc td = tiles[ti];
        const uint32_t lu = unit - td.unit_begin;
        const uint32_t ux = lu % td.units_w, uy = lu / td.units_w;
        // lane -> (x, y) with y fastest so a wave's writes are 8 runs of 8 contiguous pixels
        const uint32_t lx = ux * kUnitW + (wave & 3) * 8 + (lane >> 3);
        const uint32_t ly = uy * kUnitH + (wave >> 2) * 8 + (lane & 7);
        const bool active = lx < td.w && ly < td.h;
        const int i = (int)(td.x + (active ? lx : 0)), j = (int)(td.y + (active ? ly : 0));

        // tracer.go:15-22 pixelToPoint, then tracer.go:86 dir = (p - Cam.Pos).Norm()
        const double si = fa.phw * ((double)(fa.halfW - i) - 0.5) / (double)fa.halfW;
        const double sj = fa.phh * ((double)(fa.halfH - j) - 0.5) / (double)fa.halfH;
        V3 p = add(add(add(cam, V3{fa.fwd[0], fa.fwd[1], fa.fwd[2]}), scale(V3{fa.left[0], fa.left[1], fa.left[2]}, si)),
                   scale(V3{fa.up[0], fa.up[1], fa.up[2]}, sj));
        V3 d = norm(sub(p, cam));

        Nearest nh = trace_nearest<true, PREFILTER>(fa, lds, resident, cam, d, true);

        const uint64_t oidx = td.out_off + (uint64_t)lx * td.h + ly;
        const bool is_hit = active && nh.ok;
        if (active) {
            if (out.valid) out.valid[oidx] = is_hit ? 1 : 0;
            if (out.face) out.face[oidx] = is_hit ? (int32_t)nh.face : -1;
            if (out.object) out.object[oidx] = is_hit ? (int32_t)nh.obj : -1;
            if (!is_hit) {
                if (out.rgb) {
                    out.rgb[3 * oidx] = 0.0;
                    out.rgb[3 * oidx + 1] = 0.0;
                    out.rgb[3 * oidx + 2] = 0.0;
                }
                if (out.rgb8) {
                    out.rgb8[3 * oidx] = 0;
                    out.rgb8[3 * oidx + 1] = 0;
                    out.rgb8[3 * oidx + 2] = 0;
                }
            }
        }
        // wave-aggregated compaction of hits
        const uint64_t mask = __ballot(is_hit);
        if (mask) {
            const uint32_t cnt = __popcll(mask);
            const uint32_t leader = __ffsll((unsigned long long)mask) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(&counters[kCntHits], cnt);
            base = __shfl(base, leader);
            if (is_hit) {
                const uint32_t rank = __popcll(mask & ((1ull << lane) - 1ull));
                HitRec& hr = hits[base + rank];
                vstore(hr.h, nh.hit);
                vstore(hr.n, nh.normal);
                hr.out = oidx;
                hr.obj = nh.obj;
                hr.mat = nh.mat;
            }
        }
    }
}

// ---------------------------------------------------------------- secondary rays
template <int MODE, bool PREFILTER>
__global__ __launch_bounds__(kWG, 4) void k_secondary(const FrameArgs fa, const HitRec* __restrict__ hits,
                                                       const uint32_t* __restrict__ counters,
                                                       uint8_t* __restrict__ lit, RayIO io) {
    __shared__ __attribute__((aligned(16))) double lds[kLdsTris * kTriD];
    const bool resident = fa.n_objects == 1 && fa.obj[0].m.ntri <= (uint32_t)kLdsTris;
    if (resident) {
        stage_tris<false>(lds, fa.obj[0].m.tri, 0, fa.obj[0].m.ntri, V3{0, 0, 0});
        __syncthreads();
    }
    const uint32_t nh = MODE == kModeShadow ? counters[kCntHits] : io.n;
    const uint64_t items = MODE == kModeShadow ? (uint64_t)nh * fa.n_lights : (uint64_t)io.n;
    const uint64_t nchunks = (items + kWG - 1) / kWG;
    for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
        const uint64_t item = chunk * kWG + threadIdx.x;
        const bool active = item < items;
        V3 o{0, 0, 0}, d{1, 0, 0};
        uint32_t h = 0, l = 0;
        V3 hit{0, 0, 0}, lpos{0, 0, 0};
        if (active) {
            if (MODE == kModeShadow) {
                // consecutive lanes = consecutive hits of one light: coherent rays
                l = (uint32_t)(item / nh);
                h = (uint32_t)(item - (uint64_t)l * nh);
                hit = vload(hits[h].h);
                lpos = V3{fa.lpos[l][0], fa.lpos[l][1], fa.lpos[l][2]};
                V3 ldir = norm(sub(lpos, hit));       // tracer.go:61
                o = add(hit, scale(ldir, 0.0001));    // tracer.go:64
                d = ldir;
            } else {
                o = vload(io.orig + 3 * item);
                d = vload(io.dir + 3 * item);
            }
        }
        Nearest r = trace_nearest<false, PREFILTER>(fa, lds, resident, o, d, MODE == kModeRays);
        if (active) {
            if (MODE == kModeShadow) {
                // tracer.go:64: lit iff !shaded || |L - hit| < |occluder - hit|
                const bool is_lit = !r.ok || len(sub(lpos, hit)) < len(sub(r.hit, hit));
                lit[(uint64_t)l * nh + h] = is_lit ? 1 : 0;
            } else {
                io.ok[item] = r.ok ? 1 : 0;
                vstore(io.hit + 3 * item, r.ok ? r.hit : V3{0, 0, 0});
                vstore(io.normal + 3 * item, r.ok ? r.normal : V3{0, 0, 0});
                io.face[item] = r.ok ? (int32_t)r.face : -1;
                io.object[item] = r.ok ? (int32_t)r.obj : -1;
            }
        }
    }
}

// ---------------------------------------------------------------- shade
__global__ __launch_bounds__(256) void k_shade(const FrameArgs fa, const HitRec* __restrict__ hits,
                                               const uint32_t* __restrict__ counters,
                                               const uint8_t* __restrict__ lit, OutPlanes out) {
    const uint32_t nh = counters[kCntHits];
    V3 cam{fa.cam[0], fa.cam[1], fa.cam[2]};
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += gridDim.x * blockDim.x) {
        const HitRec hr = hits[h];
        const DevMesh& m = fa.obj[hr.obj].m;
        const double* mt = m.mats + (size_t)hr.mat * 10;
        RGB ka{mt[0], mt[1], mt[2]}, kd{mt[3], mt[4], mt[5]}, ks{mt[6], mt[7], mt[8]};
        const double ns = mt[9];
        const V3 hit = vload(hr.h), n = vload(hr.n);
        RGB c = ka;  // tracer.go:56
        for (uint32_t l = 0; l < fa.n_lights; ++l) {
            if (!lit[(uint64_t)l * nh + h]) continue;
            const V3 lpos{fa.lpos[l][0], fa.lpos[l][1], fa.lpos[l][2]};
            const RGB lcol{fa.lcol[l][0], fa.lcol[l][1], fa.lcol[l][2]};
            const V3 ldir = norm(sub(lpos, hit));                         // tracer.go:61
            const V3 refl = sub(scale(n, 2 * dot(ldir, n)), ldir);        // tracer.go:65
            const V3 camdir = norm(sub(cam, hit));                        // tracer.go:66
            c = c_add(c, c_mul(c_scale(kd, go_max(dot(ldir, n), 0.0)), lcol));                // :69
            c = c_add(c, c_mul(c_scale(ks, go_pow(go_max(dot(refl, camdir), 0.0), ns)), lcol));  // :72
        }
        if (out.rgb) {
            out.rgb[3 * hr.out] = c.r;
            out.rgb[3 * hr.out + 1] = c.g;
            out.rgb[3 * hr.out + 2] = c.b;
        }
        if (out.rgb8) {
            out.rgb8[3 * hr.out] = c_u8(c.r);
            out.rgb8[3 * hr.out + 1] = c_u8(c.g);
            out.rgb8[3 * hr.out + 2] = c_u8(c.b);
        }
    }
}

// ---------------------------------------------------------------- unpack
// packed tile-major planes -> W x H framebuffer, pixel (x, y) at x*H + y.
__global__ __launch_bounds__(256) void k_unpack(const TileDesc* __restrict__ tiles, uint32_t ntiles, uint64_t npix,
                                                uint32_t H, OutPlanes src, OutPlanes dst) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npix;
         p += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = ntiles - 1;
        while (lo < hi) {
            uint32_t mid = (lo + hi + 1) >> 1;
            if (tiles[mid].out_off <= p)
                lo = mid;
            else
                hi = mid - 1;
        }
        const TileDesc td = tiles[lo];
        const uint64_t local = p - td.out_off;
        const uint32_t lx = (uint32_t)(local / td.h), ly = (uint32_t)(local - (uint64_t)lx * td.h);
        const uint64_t q = (uint64_t)(td.x + lx) * H + (td.y + ly);
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
    }
}

// ---------------------------------------------------------------- diagnostics
__global__ __launch_bounds__(256) void k_debug_fp64(int op, uint32_t n, const double* __restrict__ a,
                                                    const double* __restrict__ b, double* __restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double r;
    switch (op) {
        case 0: r = sqrt(a[i]); break;
        case 1: r = a[i] / b[i]; break;
        case 2: r = go_pow(a[i], b[i]); break;
        default: r = go_max(a[i], b[i]); break;
    }
    out[i] = r;
}

// ---------------------------------------------------------------- launchers
hipError_t launch_debug_fp64(int op, uint32_t n, const double* a, const double* b, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_fp64, dim3((n + 255) / 256), dim3(256), 0, s, op, n, a, b, out);
    return hipGetLastError();
}

hipError_t launch_primary(const FrameArgs& fa, const TileDesc* tiles, uint32_t ntiles, uint32_t total_units,
                          const OutPlanes& out, HitRec* hits, uint32_t* counters, int grid, bool prefilter,
                          hipStream_t s) {
    if (prefilter)
        hipLaunchKernelGGL(k_primary<true>, dim3(grid), dim3(kWG), 0, s, fa, tiles, ntiles, total_units, out, hits,
                           counters);
    else
        hipLaunchKernelGGL(k_primary<false>, dim3(grid), dim3(kWG), 0, s, fa, tiles, ntiles, total_units, out, hits,
                           counters);
    return hipGetLastError();
}

hipError_t launch_shadow(const FrameArgs& fa, const HitRec* hits, const uint32_t* counters, uint8_t* lit, int grid,
                         bool prefilter, hipStream_t s) {
    RayIO none{};
    if (prefilter)
        hipLaunchKernelGGL((k_secondary<kModeShadow, true>), dim3(grid), dim3(kWG), 0, s, fa, hits, counters, lit,
                           none);
    else
        hipLaunchKernelGGL((k_secondary<kModeShadow, false>), dim3(grid), dim3(kWG), 0, s, fa, hits, counters, lit,
                           none);
    return hipGetLastError();
}

hipError_t launch_rays(const FrameArgs& fa, const RayIO& io, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_secondary<kModeRays, true>), dim3(grid), dim3(kWG), 0, s, fa, (const HitRec*)nullptr,
                       (const uint32_t*)nullptr, (uint8_t*)nullptr, io);
    return hipGetLastError();
}

hipError_t launch_shade(const FrameArgs& fa, const HitRec* hits, const uint32_t* counters, const uint8_t* lit,
                        const OutPlanes& out, uint64_t /*lit_stride*/, int grid, hipStream_t s) {
    hipLaunchKernelGGL(k_shade, dim3(grid), dim3(256), 0, s, fa, hits, counters, lit, out);
    return hipGetLastError();
}

hipError_t launch_unpack(const TileDesc* tiles, uint32_t ntiles, uint64_t npix, uint32_t H, const OutPlanes& src,
                         const OutPlanes& dst, hipStream_t s) {
    uint64_t blocks = (npix + 255) / 256;
    int grid = (int)(blocks < 4096 ? (blocks ? blocks : 1) : 4096);
    hipLaunchKernelGGL(k_unpack, dim3(grid), dim3(256), 0, s, tiles, ntiles, npix, H, src, dst);
    return hipGetLastError();
}

}  // namespace mirt
