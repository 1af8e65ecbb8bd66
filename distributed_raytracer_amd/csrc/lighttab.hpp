// lighttab.hpp — one record of a shadow-segment light table, shared by the
// host builder (mirt_debug_light_table) and the device builder (kernels.hip k_light_table):
// the same fp64 operations in the same order on both sides (-ffp-contract=off), so the
// tables are bit-identical wherever they are built (tests/test_light_table.py).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mirt {

// Per light: Lo = L - pos (object space), Lh >= |L - hit| over every hit on the mesh and
// Mmax >= the kernel's M (shadow_lit_single) for every hit; R = the mesh's |hit| bound.
struct LightGeom {
    double Lo[3], Lh, Mmax;
};
__host__ __device__ inline LightGeom light_geom(const double L[3], const double pos[3], double scale) {
    LightGeom g;
    const double R = 2.0 * sqrt(3.0) * scale + 1.0;  // |hit| in object space, with slack
    const double pinf = fmax(fmax(fabs(pos[0]), fabs(pos[1])), fabs(pos[2]));
    for (int q = 0; q < 3; ++q) g.Lo[q] = L[q] - pos[q];
    g.Lh = sqrt(g.Lo[0] * g.Lo[0] + g.Lo[1] * g.Lo[1] + g.Lo[2] * g.Lo[2]) + R;  // >= |L - hit|
    g.Mmax = 0x1p-36 * (2.0 + g.Lh + pinf + R);
    return g;
}

// x rounded to float, then one float up (std::nextafter((float)x, +inf)): NaN and +inf stay.
__host__ __device__ inline float f32_round_up(double x) {
    const float f = (float)x;
    if (f != f || f == __builtin_inff()) return f;
    if (f == 0.0f) return 0x1p-149f;
    uint32_t b;
    __builtin_memcpy(&b, &f, 4);
    b = f > 0.0f ? b + 1u : b - 1u;
    float r;
    __builtin_memcpy(&r, &b, 4);
    return r;
}

// The 16-float record of triangle t (P1, E1, E2: 9 doubles) for one light:
//   W1 = V2 x V3, W2 = V3 x V1, W3 = V1 x V2 (V_i = P_i - L), A = E1 x E2, ntL = A . (L - P1),
//   cw, cA, ctL (error bounds, rounded up; see mirt.cpp light_table).
__host__ __device__ inline void light_record(const double* t, const LightGeom& g, float* r) {
    auto n1 = [](const double* v) { return fabs(v[0]) + fabs(v[1]) + fabs(v[2]); };
    auto cross = [](const double* a, const double* b, double* o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    double V[3][3], W[3][3], A[3], e21[3];
    for (int q = 0; q < 3; ++q) {
        V[0][q] = t[q] - g.Lo[q];
        V[1][q] = V[0][q] + t[3 + q];
        V[2][q] = V[0][q] + t[6 + q];
        e21[q] = t[6 + q] - t[3 + q];
    }
    cross(V[1], V[2], W[0]);
    cross(V[2], V[0], W[1]);
    cross(V[0], V[1], W[2]);
    cross(t + 3, t + 6, A);
    const double ntL = -(A[0] * V[0][0] + A[1] * V[0][1] + A[2] * V[0][2]);
    const double G = fmax(fmax(n1(V[0]), n1(V[1])), n1(V[2]));
    const double Ed = fmax(fmax(n1(t + 3), n1(t + 6)), n1(e21));
    const double Wm = fmax(fmax(n1(W[0]), n1(W[1])), n1(W[2]));
    const double cw = 1.25 * (0x1p-21 * Wm + 0x1p-36 * (G + g.Lh) * (G + Ed) + 4.0 * g.Mmax * Ed) + 0x1p-100;
    const double cA = 1.25 * (0x1p-21 * n1(A) + 0x1p-44 * Ed * Ed) + 0x1p-100;
    const double ctL = 1.25 * (0x1p-22 * fabs(ntL) + n1(A) * g.Mmax + 0x1p-36 * (G + g.Lh) * Ed * Ed) + 0x1p-100;
    for (int w = 0; w < 3; ++w)
        for (int q = 0; q < 3; ++q) r[3 * w + q] = (float)W[w][q];
    for (int q = 0; q < 3; ++q) r[9 + q] = (float)A[q];
    r[12] = (float)ntL;
    r[13] = f32_round_up(cw);
    r[14] = f32_round_up(cA);
    r[15] = f32_round_up(ctL);
}

}  // namespace mirt
