// geo_math.h — f32 transcendentals with a fixed, fully specified evaluation
// order (explicit fmaf, no contraction), so that the gfx950 kernel and a
// host build of the same sequence produce bit-identical results.
//
// Why: the per-pixel hit-classification mask must match the CPU path pixel
// for pixel (BASELINE.json north_star).  ROCm OCML and glibc differ by a few
// ULP in asinf/atan2f/sinf, enough to flip pixels on the photon-ring edge.
// Only IEEE-exact operations are used: + - * / sqrt fma rint fabs copysign
// min max and compares; compile with -ffp-contract=off and correctly rounded
// f32 divide/sqrt (hipcc default, pinned by -fhip-fp32-correctly-rounded-divide-sqrt).
//
// Algorithms: the general-purpose forms (point path, observer): Cody-Waite
// reduction by pi/2 plus Cephes-style minimax polynomials (sin/cos on
// [-pi/4, pi/4], asin on [0, 1/2], atan on [-(sqrt2-1), sqrt2-1]); the
// per-pixel sky-direction forms (end of file): reduction by pi, acos/pi as
// sqrt(1 - |x|) P(|x|), atan2 in turns.  Accuracy is checked against libm in
// tests/test_math.py (<= 3 ulp / 2e-7 abs on the ranges used).
#pragma once

#if defined(__HIP__)  // HIP language mode (hipcc compiles .cpp as HIP too)
#include <hip/hip_runtime.h>
#define GEO_HD __host__ __device__ __forceinline__
#define GEO_HDM __host__ __device__ __forceinline__  // member functions
#else
#define GEO_HD static inline
#define GEO_HDM inline
#endif

// Makes the compiler forget what it knows about a VGPR value (no code).
#if defined(__HIP_DEVICE_COMPILE__)
#define GEO_OPAQUE(x) asm volatile("" : "+v"(x))
#else
#define GEO_OPAQUE(x) ((void)0)
#endif
// Gives a variable an arbitrary defined value at no cost (device: whatever
// its VGPR holds; host: 0) — for registers that are always written before a
// read that matters.
#if defined(__HIP_DEVICE_COMPILE__)
#define GEO_UNSET(x) asm volatile("" : "=v"(x))  // volatile: not CSEd into one value (copied 14 ways)
#else
#define GEO_UNSET(x) ((x) = 0)
#endif

namespace geo {

constexpr float kPi = 3.14159265358979323846f;
constexpr float kPi2 = 1.57079632679489661923f;   // PI/2 (shader.wgsl:23 M_PI_2)
constexpr float kPi4 = 0.785398163397448309616f;
constexpr float kTwoOverPi = 0.636619772367581343076f;
constexpr float kInvPi = 0.318309886183790671538f;
constexpr float kInvTwoPi = 0.159154943091895335769f;

GEO_HD float fmaf_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// In an arm of a lane-divergent branch that must stay a branch (a volatile
// asm cannot be speculated, so the arm is not if-converted into work every
// lane would do).
#if defined(__HIP_DEVICE_COMPILE__)
#define GEO_COLD_ARM() asm volatile("")
#else
#define GEO_COLD_ARM() ((void)0)
#endif

// Correctly rounded sqrt, equal to __builtin_sqrtf for every input.  On the
// device, hipcc's correctly rounded sequence wraps the +-1-ulp correction of
// v_sqrt_f32 in a 2^32 pre-scale for x < 2^-96 and a class fix-up for
// +-0/+inf (~17 VALU).  Here: s = x rsq(x) corrected once by its residual,
// s + (x - s^2) rsq(x)/2, which is correctly rounded for every finite
// x >= 2^-96 (5 VALU + the range test; exhaustively checked against
// __builtin_sqrtf over all 2^32 inputs, tests/test_gpu_math.py).  Smaller,
// zero, NaN and infinite inputs take the builtin.  The fast sequence runs on
// every lane with no exec-mask change, and the out-of-range lanes are redone
// in a wave-uniform branch that a typical wave never takes (a divergent
// if/else costs ~6 scalar instructions of exec juggling per call, ~10 calls
// a pixel).
GEO_HD float sqrtf_(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const bool ok = __builtin_amdgcn_fmed3f(x, 0x1p-96f, 0x1.fffffep127f) == x;  // NaN, +inf fail
    const float y = __builtin_amdgcn_rsqf(x);
    const float s0 = x * y;
    const float hy = 0.5f * y;
    float r = __builtin_fmaf(__builtin_fmaf(-s0, s0, x), hy, s0);
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
        GEO_COLD_ARM();
        r = ok ? r : __builtin_sqrtf(x);
    }
    return r;
#else
    return __builtin_sqrtf(x);
#endif
}
// Correctly rounded reciprocal, equal to 1.0f / x (hipcc's correctly rounded
// division, ~11 VALU) for every input.  For normal |x| < 2^126 the Markstein
// step r + r(1 - x r) on the 1-ulp v_rcp_f32 seed is correctly rounded (3
// VALU; checked against the builtin for all 2^32 inputs on the GPU,
// tests/test_gpu_math.py; outside that range the seed's result is denormal,
// zero or infinite and the step is not exact).  The range test is one
// v_med3_f32 + compare (NaN fails it); other lanes take the builtin in a
// wave-uniform branch, as in sqrtf_.
GEO_HD float rcpf_(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float ax = __builtin_fabsf(x);
    const bool ok = __builtin_amdgcn_fmed3f(ax, 0x1p-126f, 0x1.fffffep125f) == ax;
    const float r0 = __builtin_amdgcn_rcpf(x);
    float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
        GEO_COLD_ARM();
        r = ok ? r : 1.0f / x;
    }
    return r;
#else
    return 1.0f / x;
#endif
}
// The quotient of the specification: a times the correctly rounded
// reciprocal of b (two IEEE roundings, within 1 ulp of a / b).  On gfx950
// that is rcpf_'s 5 VALU plus one multiply instead of the ~11 of a
// correctly rounded division; the oracle mirrors it as a * (1.0f / b).
GEO_HD float divf_(float a, float b) { return a * rcpf_(b); }
GEO_HD float clampf_(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
// max(a, b) with a NaN `a` mapped to b (used to clamp radicands at 0).
GEO_HD float fmaxf_(float a, float b) { return a > b ? a : b; }

// sin and cos of x, |x| < ~1e4.
// rint(t) and (int)rint(t) & 3 for |t| < 2^22 by the 1.5 * 2^23 shifter: t + M
// rounds t to an integer (ties to even, as rintf) in the low mantissa bits, so
// j = (t + M) - M exactly and the quadrant is the sum's low 2 bits (M = 0 mod
// 4); full-rate adds where v_rndne_f32 and v_cvt_i32_f32 are half-rate.
GEO_HD void sincosf_(float x, float* s, float* c) {
    constexpr float kShifter = 12582912.0f;  // 1.5 * 2^23
    const float tj = x * kTwoOverPi + kShifter;
    const float j = tj - kShifter;
    uint32_t tb;
    __builtin_memcpy(&tb, &tj, 4);
    const int q = (int)(tb & 3u);
    float r = fmaf_(-j, 1.5703125f, x);
    r = fmaf_(-j, 4.837512969970703125e-4f, r);
    r = fmaf_(-j, 7.54978995489188216e-8f, r);
    const float z = r * r;
    const float ps = fmaf_(fmaf_(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float sn = fmaf_(ps * z, r, r);
    const float pc = fmaf_(fmaf_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                           4.166664568298827e-2f);
    const float cs = fmaf_(pc * z, z, fmaf_(-0.5f, z, 1.0f));
    const float sa = (q & 1) ? cs : sn;
    const float ca = (q & 1) ? sn : cs;
    *s = (q & 2) ? -sa : sa;
    *c = ((q + 1) & 2) ? -ca : ca;
}

// asin(x) for x in [-1, 1]: |x| clamped to 1 by one v_min_f32 (a NaN x
// becomes |x| = 1, i.e. +-pi/2 by its sign bit; a compare-and-select clamp
// kept the NaN: 4 VALU for no case a frame produces), the sign restored by
// the final copysign.
GEO_HD float asinf_(float x) {
    const float a = __builtin_fminf(__builtin_fabsf(x), 1.0f);
    const bool big = a > 0.5f;
    const float z = big ? 0.5f * (1.0f - a) : a * a;
    // the square root only where it is used: a wave with no |x| > 1/2 lane
    // branches over it (the compiler would otherwise take it on every lane)
    float s = a;
    if (big) {
        GEO_COLD_ARM();
        s = sqrtf_(z);
    }
    const float p = fmaf_(fmaf_(fmaf_(fmaf_(4.2163199048e-2f, z, 2.4181311049e-2f), z,
                                      4.5470025998e-2f), z, 7.4953002686e-2f), z,
                          1.6666752422e-1f);
    float r = fmaf_(p * z, s, s);
    r = big ? fmaf_(-2.0f, r, kPi2) : r;
    return __builtin_copysignf(r, x);
}

// atan2(y, x); atan2(0, 0) = 0.
GEO_HD float atan2f_(float y, float x) {
    const float ay = __builtin_fabsf(y);
    const float ax = __builtin_fabsf(x);
    const bool big = ay > 2.414213562373095f * ax;
    const bool mid = ay > 0.4142135623730950f * ax;
    const float num = big ? -ax : (mid ? ay - ax : ay);
    const float den = big ? ay : (mid ? ay + ax : ax);
    const float y0 = big ? kPi2 : (mid ? kPi4 : 0.0f);
    const float t = den > 0.0f ? divf_(num, den) : 0.0f;
    const float z = t * t;
    const float p = fmaf_(fmaf_(fmaf_(8.05374449538e-2f, z, -1.38776856032e-1f), z,
                                1.99777106478e-1f), z, -3.33329491539e-1f);
    float r = y0 + fmaf_(p * z, t, t);
    r = (x < 0.0f) ? kPi - r : r;
    return __builtin_copysignf(r, y);
}

// acos(x) for x in [-1, 1] (clamped), from the asin kernel:
// |x| <= 1/2: pi/2 - asin(x); else 2 asin(sqrt((1 - |x|)/2)) (reflected for x < 0).
GEO_HD float acosf_(float x) {
    x = clampf_(x, -1.0f, 1.0f);
    const float a = __builtin_fabsf(x);
    if (a <= 0.5f) return kPi2 - asinf_(x);
    const float z = 0.5f * (1.0f - a);
    const float s = sqrtf_(z);
    const float p = fmaf_(fmaf_(fmaf_(fmaf_(4.2163199048e-2f, z, 2.4181311049e-2f), z,
                                      4.5470025998e-2f), z, 7.4953002686e-2f), z,
                          1.6666752422e-1f);
    const float r = 2.0f * fmaf_(p * z, s, s);
    return x > 0.0f ? r : kPi - r;
}

GEO_HD float atanf_(float x) { return atan2f_(x, 1.0f); }

// ---- The per-pixel sky-direction transcendentals (round 6) ----
// Specified for what they feed: angles in turns and half-turns, absolute
// error <= 2e-7 (tools/fit_sky_polys.py fits the polynomials;
// tests/test_math.py checks the error), against a UV bar of 1e-4.  The
// general-purpose forms above stay for the point path and the observer.

// sqrt(max(x, 2^-96)), correctly rounded, for x in [0, 1]: sqrtf_'s fast
// sequence with the range test replaced by the max (x = 0 gives 2^-48; the
// nonzero x here are >= 2^-24), so no branch.
GEO_HD float sqrt_unit_(float x) {
    const float xm = __builtin_fmaxf(x, 0x1p-96f);
#if defined(__HIP_DEVICE_COMPILE__)
    const float y = __builtin_amdgcn_rsqf(xm);
    const float s0 = xm * y;
    const float hy = 0.5f * y;
    return __builtin_fmaf(__builtin_fmaf(-s0, s0, xm), hy, s0);
#else
    return __builtin_sqrtf(xm);
#endif
}

// sin and cos of x, |x| < 2^21: j = rint(x / pi) by the 1.5 * 2^23 shifter
// (one fma; its sum's low mantissa bit is j's parity), r = x - j pi in two
// Cody-Waite parts (|r| <= pi/2 + 1 ulp; pi - P1 - P2 = 5e-12), cubic
// polynomials in r^2, and both signs flipped for odd j by an XOR of the
// parity bit.  17 VALU.
GEO_HD void sincos_sky_(float x, float* s, float* c) {
    constexpr float kShifter = 12582912.0f;  // 1.5 * 2^23
    const float tj = fmaf_(x, kInvPi, kShifter);
    const float j = tj - kShifter;
    uint32_t tb;
    __builtin_memcpy(&tb, &tj, 4);
    const uint32_t flip = tb << 31;
    float r = fmaf_(-j, 3.140625f, x);
    r = fmaf_(-j, 9.67653584666550159e-4f, r);
    const float z = r * r;
    const float ps = fmaf_(fmaf_(fmaf_(2.600061634e-06f, z, -1.980661764e-04f), z, 8.333017118e-03f), z,
                           -1.666665673e-01f);
    const float sn = fmaf_(r * z, ps, r);
    const float pc = fmaf_(fmaf_(fmaf_(2.319447049e-05f, z, -1.385593088e-03f), z, 4.166398942e-02f), z,
                           -4.999993145e-01f);
    const float cs = fmaf_(z, pc, 1.0f);
    uint32_t sb, cb;
    __builtin_memcpy(&sb, &sn, 4);
    __builtin_memcpy(&cb, &cs, 4);
    sb ^= flip;
    cb ^= flip;
    __builtin_memcpy(s, &sb, 4);
    __builtin_memcpy(c, &cb, 4);
}

// acos(x) / pi in [0, 1] for x in [-1, 1] (|x| clamped to 1 by one
// v_min_f32; a NaN x gives |x| = 1): h = sqrt(1 - |x|) P(|x|) with P of
// degree 6, and 1 - h for x < 0.  h <= 0.5 + 1 ulp, so the result is in
// [0, 1] for every input.  No branch; 18 VALU.
GEO_HD float acos_pi_(float x) {
    const float a = __builtin_fminf(__builtin_fabsf(x), 1.0f);
    const float s = sqrt_unit_(1.0f - a);
    float p = fmaf_(8.312922437e-04f, a, -3.820668207e-03f);
    p = fmaf_(p, a, 8.837061934e-03f);
    p = fmaf_(p, a, -1.565995067e-02f);
    p = fmaf_(p, a, 2.827732079e-02f);
    p = fmaf_(p, a, -6.830646098e-02f);
    p = fmaf_(p, a, 4.999999702e-01f);
    const float h = s * p;
    return x < 0.0f ? 1.0f - h : h;
}

// atan2(y, x) / (2 pi) taken into [0, 1] (the sky's U before its clamp):
// atan2f_'s reduction to |t| <= tan(pi/8) with its offsets in turns, a cubic
// polynomial in t^2 with 1 / (2 pi) folded in, then the half-plane and
// lower-half reflections (x < 0: 1/2 - r; y < 0: 1 - r).  atan2(+-0, 0) = 0;
// a NaN y gives NaN (the caller's clamp maps it to 0).
GEO_HD float atan2_turns_(float y, float x) {
    const float ay = __builtin_fabsf(y);
    const float ax = __builtin_fabsf(x);
    const bool big = ay > 2.414213562373095f * ax;
    const bool mid = ay > 0.4142135623730950f * ax;
    const float num = big ? -ax : (mid ? ay - ax : ay);
    const float den = big ? ay : (mid ? ay + ax : ax);
    const float y0 = big ? 0.25f : (mid ? 0.125f : 0.0f);
    const float t = den > 0.0f ? divf_(num, den) : 0.0f;
    const float z = t * t;
    const float p = fmaf_(fmaf_(fmaf_(-1.715674624e-02f, z, 3.116416559e-02f), z, -5.302115157e-02f), z,
                          1.591545641e-01f);
    const float r = fmaf_(t, p, y0);
    const float h = x < 0.0f ? 0.5f - r : r;
    return y < 0.0f ? 1.0f - h : h;
}

}  // namespace geo
