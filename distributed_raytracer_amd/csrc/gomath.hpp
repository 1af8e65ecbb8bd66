// gomath.hpp — fp64 vector ops and Go math semantics, compiled for host and gfx950.
//
// Every function restates the reference's arithmetic in its exact operation order;
// the whole library is built with -ffp-contract=off so that no x*y+z is fused (Go on
// amd64 at GOAMD64=v1 never fuses).  Divisions stay true IEEE divisions (never a
// reciprocal multiply) and sqrt stays the correctly rounded square root.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

#define MIRT_HD __host__ __device__ __forceinline__

namespace mirt {

struct V3 {
    double x, y, z;
};

MIRT_HD V3 v3(double x, double y, double z) { return V3{x, y, z}; }
// shared/geom/vector.go:14-16
MIRT_HD V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
// vector.go:19-21
MIRT_HD V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
// vector.go:24-26 — s * component
MIRT_HD V3 scale(V3 a, double s) { return V3{s * a.x, s * a.y, s * a.z}; }
// vector.go:29-31 — (x*x' + y*y') + z*z'
MIRT_HD double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vector.go:34-36
MIRT_HD V3 cross(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// vector.go:45-47
MIRT_HD bool is_zero(V3 a) { return a.x == 0.0 && a.y == 0.0 && a.z == 0.0; }
// vector.go:56-58
MIRT_HD double len(V3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
// vector.go:50-53 — three true divisions by the magnitude
MIRT_HD V3 norm(V3 a) {
    double mag = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return V3{a.x / mag, a.y / mag, a.z / mag};
}

MIRT_HD uint64_t dbits(double d) {
    uint64_t u;
    __builtin_memcpy(&u, &d, 8);
    return u;
}
MIRT_HD double dfrom(uint64_t u) {
    double d;
    __builtin_memcpy(&d, &u, 8);
    return d;
}
MIRT_HD bool d_isnan(double x) { return x != x; }
MIRT_HD bool d_isinf(double x) { return (dbits(x) & 0x7fffffffffffffffull) == 0x7ff0000000000000ull; }
MIRT_HD bool d_signbit(double x) { return (dbits(x) >> 63) != 0; }

// Go math.Min / math.Max (signed zeros, NaN, Inf handled like Go).
MIRT_HD double go_min(double x, double y) {
    if ((d_isinf(x) && x < 0) || (d_isinf(y) && y < 0)) return -__builtin_inf();
    if (d_isnan(x) || d_isnan(y)) return __builtin_nan("");
    if (x == 0 && x == y) return d_signbit(x) ? x : y;
    return x < y ? x : y;
}
MIRT_HD double go_max(double x, double y) {
    if ((d_isinf(x) && x > 0) || (d_isinf(y) && y > 0)) return __builtin_inf();
    if (d_isnan(x) || d_isnan(y)) return __builtin_nan("");
    if (x == 0 && x == y) return d_signbit(x) ? y : x;
    return x > y ? x : y;
}

// The constant-operand forms the colour code uses, with Go's results for every input:
//   go_min(a, 1.0):  NaN -> NaN, else the smaller (no signed-zero case: 1 is not zero)
//   go_max(x, 0.0) and go_max(0.0, x):  NaN -> NaN, x > 0 -> x, else +0 (both zeros give
//   +0: Go returns the operand without the sign bit)
// (tests/test_host.py pins them against go_min / go_max over special and random values.)
MIRT_HD double go_min1(double a) { return a >= 1.0 ? 1.0 : a; }
MIRT_HD double go_max0(double x) { return x <= 0.0 ? 0.0 : x; }

// Go math.Frexp / normalize / Ldexp (bit manipulation; exact).
MIRT_HD double go_frexp(double f, int& e) {
    e = 0;
    if (f == 0 || d_isinf(f) || d_isnan(f)) return f;
    double af = f < 0 ? -f : f;
    if (af < 2.2250738585072014e-308) {
        f *= 4503599627370496.0;
        e = -52;
    }
    uint64_t x = dbits(f);
    e += (int)((x >> 52) & 0x7ff) - 1022;
    x &= ~(0x7ffull << 52);
    x |= 1022ull << 52;
    return dfrom(x);
}
MIRT_HD double go_ldexp(double frac, int exp) {
    if (frac == 0 || d_isinf(frac) || d_isnan(frac)) return frac;
    double af = frac < 0 ? -frac : frac;
    if (af < 2.2250738585072014e-308) {
        frac *= 4503599627370496.0;
        exp -= 52;
    }
    uint64_t x = dbits(frac);
    exp += (int)((x >> 52) & 0x7ff) - 1023;
    if (exp < -1075) return d_signbit(frac) ? -0.0 : 0.0;
    if (exp > 1023) return frac < 0 ? -__builtin_inf() : __builtin_inf();
    double m = 1.0;
    if (exp < -1022) {
        exp += 53;
        m = 1.0 / 9007199254740992.0;
    }
    x &= ~(0x7ffull << 52);
    x |= (uint64_t)(exp + 1023) << 52;
    return m * dfrom(x);
}

MIRT_HD double go_trunc(double x) {
    // exact integer part of |x| < 2^63 (Go math.Modf's int part)
    return (double)(int64_t)x;
}
MIRT_HD bool go_is_odd_int(double x) {
    double ax = x < 0 ? -x : x;
    if (ax >= 9007199254740992.0) return false;
    double xi = go_trunc(x);
    return xi == x && (((int64_t)xi) & 1) == 1;
}

// exp(yf * log(x)) of go_pow's fractional exponent, out of line: inlined, its polynomial
// constants are hoisted out of the kernels' work loops into registers and spilled to
// scratch, although the suzanne materials (integer Ns) never take this path.
__host__ __device__ __attribute__((noinline)) inline double go_pow_frac(double yf, double x) {
    return exp(yf * log(x));
}

// Go math.Pow.  The integer part of y is applied by repeated squaring on the Frexp
// mantissa (bit-exact with Go); a fractional part uses exp(yf*log(x)), which matches Go
// only to a few ulp (Go's amd64 Exp/Log are assembly).  tracer.go:72 uses it with the
// material's Ns (10 in example/suzanne.mtl: integer, so bit-exact).
MIRT_HD double go_pow(double x, double y) {
    if (y == 0 || x == 1) return 1;
    if (y == 1) return x;
    // Small integer exponents of a base in [2^-60, 16] (tracer.go:72's Ns): Go's repeated
    // squaring on the Frexp mantissa only rescales every operand by powers of two, which
    // changes no rounding while all products stay normal (here x^y lies in [2^-960, 2^64]
    // and the squares below 2^128), so squaring x itself in the same order gives the same
    // bits and Go's final Ldexp is exact.
    if (y >= 2.0 && y <= 16.0 && x >= 0x1p-60 && x <= 16.0 && y == (double)(int)y) {
        double a = 1.0, p = x;
        for (int i = (int)y; i != 0; i >>= 1) {
            if (i & 1) a *= p;
            p *= p;
        }
        return a;
    }
    if (d_isnan(x) || d_isnan(y)) return __builtin_nan("");
    if (x == 0) {
        if (y < 0) return (d_signbit(x) && go_is_odd_int(y)) ? -__builtin_inf() : __builtin_inf();
        return (d_signbit(x) && go_is_odd_int(y)) ? x : 0.0;
    }
    double ax = x < 0 ? -x : x;
    if (d_isinf(y)) {
        if (x == -1) return 1;
        if ((ax < 1) == (y > 0)) return 0;
        return __builtin_inf();
    }
    if (d_isinf(x)) {
        if (x < 0) {
            // Pow(1/x, -y) with 1/-Inf = -0
            return go_pow(-0.0, -y);
        }
        return y < 0 ? 0.0 : __builtin_inf();
    }
    if (y == 0.5) return sqrt(x);
    if (y == -0.5) return 1 / sqrt(x);
    double ay = y < 0 ? -y : y;
    if (ay >= 9223372036854775808.0) {
        if (x == -1) return 1;
        if ((ax < 1) == (y > 0)) return 0;
        return __builtin_inf();
    }
    double yi = go_trunc(ay);
    double yf = ay - yi;
    if (yf != 0 && x < 0) return __builtin_nan("");
    double a1 = 1.0;
    int ae = 0;
    if (yf != 0) {
        if (yf > 0.5) {
            yf--;
            yi++;
        }
        a1 = go_pow_frac(yf, x);
    }
    int xe;
    double x1 = go_frexp(x, xe);
    for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
        if (xe < -(1 << 12) || (1 << 12) < xe) {
            ae += xe;
            break;
        }
        if ((i & 1) == 1) {
            a1 *= x1;
            ae += xe;
        }
        x1 *= x1;
        xe <<= 1;
        if (x1 < .5) {
            x1 += x1;
            xe--;
        }
    }
    if (y < 0) {
        a1 = 1 / a1;
        ae = -ae;
    }
    return go_ldexp(a1, ae);
}

// shared/colour/colour.go:38-50
struct RGB {
    double r, g, b;
};
MIRT_HD RGB c_add(RGB a, RGB b) {  // go_min(x, 1.0) per channel
    return RGB{go_min1(a.r + b.r), go_min1(a.g + b.g), go_min1(a.b + b.b)};
}
MIRT_HD RGB c_scale(RGB a, double s) {  // go_max(0.0, go_min(s * x, 1.0)) per channel
    return RGB{go_max0(go_min1(s * a.r)), go_max0(go_min1(s * a.g)), go_max0(go_min1(s * a.b))};
}
MIRT_HD RGB c_mul(RGB a, RGB b) { return RGB{a.r * b.r, a.g * b.g, a.b * b.b}; }
// colour.go:59-61 RGB(): uint8(255 * c), Go truncates toward zero
MIRT_HD uint8_t c_u8(double c) { return (uint8_t)(255 * c); }

}  // namespace mirt
