// geo_pixel.h — the per-pixel f32 path: camera ray, relativistic aberration,
// null-geodesic RK4 + Newton sphere crossing, sky-sphere UV, bilinear sample.
//
// Restates, per pixel and in f32:
//   fs_main                SR/schwarzschild_sphere_shader/shader.wgsl:57-106
//   solve_ray_fan (1 node) SR/simulation/sphere_ray_tracer.rs:35-56
//   solve_geodesic         SR/simulation/sphere_ray_tracer.rs:60-193
// with the node angle theta replaced by the pixel's own angle to the black
// hole.
//
// Evaluation order is fixed (explicit fmaf, no contraction); the CPU oracle
// (oracle/geo_oracle.c, geo_oracle_pixel_f32) restates the same sequence
// independently and tests/ require bit-identical mask, UV, steps and RGBA.
// Any change here must be mirrored there.
#pragma once

#include <stdint.h>

#include "geo_math.h"

namespace geo {

constexpr float kNoValue = 15.0f;          // SphereRayTracer::NO_VALUE, sphere_ray_tracer.rs:22
constexpr float kBlackHoleLambda = -7.0f;  // hit_black_hole threshold, shader.wgsl:88
constexpr int kNewtonIters = 3;            // final_newton_refinements, sphere_ray_tracer.rs:129
constexpr float kSixth = 1.0f / 6.0f;
constexpr float kAdaptiveDefaultTol = 1e-6f;  // GEO_ADAPTIVE_DEFAULT_TOL
constexpr uint32_t kAdaptiveMaxGrowth = 16u;   // GEO_ADAPTIVE_MAX_GROWTH

// Integration kinds (frame-uniform, chosen on the host):
constexpr int kCurvedOut = 0;  // rs > 0, observer outside the horizon (r > rs), step in [2^-10, 1/2]
constexpr int kCurvedIn = 1;   // rs > 0, any other observer or step: the reference's tests as written
constexpr int kFlat = 2;       // rs = 0: straight lines

// Frame-constant scalars derived from the scene, evaluated identically on
// every lane (and by the oracle).  Names follow sphere_ray_tracer.rs:60-132.
struct PixelConsts {
    float rs, sphere_r, r, step;
    uint32_t max_steps;
    float hh, h6;          // step/2 (step_half :130), step/6
    float hh2, hhh, h2_6;  // step^2/4, step^2/2, step^2/6
    float r3_2;            // 3*rs/2 (:109)
    float sphere_u;        // 1/sphere_r (:131)
    float schwarz_u;       // 1/rs (:132)
    float u0;              // 1/r (:122)
    float h_over_r2;       // (1 - rs/r)/(r*r) (:123)
    float inv_r2;          // 1/(r*r)
    float bound;           // 0.9*min(u0, 1/max(sphere_r, r3_2)) (:127)
    float e_out;           // sqrt(1 - rs/r) (solve_ray_fan :48)
    float e_in;            // sqrt(-1 + rs/r) (:44)
    float barrier_thresh;  // 4/(27 rs^2) (:107)
    bool r_inside_h;       // r < rs (:42)
    bool outside;          // r > rs (:62)
    bool sphere_outside;   // sphere_r > rs (:63)
    bool inside_sphere;    // r < sphere_r (:64)
    bool diff_sides;       // different_sides_3r_2 (:110)
    bool rs_nonzero;
    // frame-uniform parts of the radial cases (:67-104) and pre-filters (:113-117)
    float radial_falling, radial_outgoing;  // result for rotation < 1e-10, by `falling`
    bool radial_by_energy;                  // radial result decided by energy > 0 instead
    bool pf_always, pf_falling, pf_outgoing, pf_eneg, pf_barrier;
    // device forms of the same tests (geodesic_init): the barrier term as one
    // compare, `inv_b2 < barrier_lim` (-inf when pf_barrier is off), and the
    // squared outside-horizon energy
    float barrier_lim, e_out2;
    // pf_always | pf_falling << 1 | pf_outgoing << 2 as one aligned word: the
    // kernel reads it with one scalar load (the bool bytes above sit at
    // unaligned kernarg offsets, which hipcc fetches with vector loads)
    uint32_t pf_bits;
    // frame-uniform parts of the stop test and the initial loop test, folded
    // on the host (gfx9 has no scalar float compares, so the kernel would
    // evaluate them in VALU on every lane): StopTest's interval [stop_lo,
    // stop_hi] and stop_bits = above0 (U0 > SU) | (max_steps != 0 && u0 > 0) << 2
    float stop_lo, stop_hi;
    uint32_t stop_bits;
    int kind;  // the frame's integration kind (geodesic_kind)
    // the integrator's scaled state U = scale*u (scale = 3 rs/2, or 1 for rs = 0)
    float scale, U0, SU, BD, HU;
    float ub_k;  // scale * (e_out * u0): outside the horizon UB0 = ub_k |sin theta| / cos theta
    float SUp;  // next float above SU: (U > SU) == (U >= SUp) for every float U
    // GEO_MODE_ADAPTIVE step control (geodesic_angle_adaptive), scaled like U
    float tolU;  // scale * tol: reject a step whose error estimate exceeds it
    float tolG;  // tolU / 64: double the step after one whose estimate is below it
    float hmax;  // GEO_ADAPTIVE_MAX_GROWTH * step
};



// Next float above a positive finite x.
GEO_HD float next_up_(float x) {
    uint32_t b;
    __builtin_memcpy(&b, &x, 4);
    b += 1u;
    __builtin_memcpy(&x, &b, 4);
    return x;
}

// median of three; for lo <= hi: med3(x, lo, hi) == x  <=>  lo <= x <= hi, and
// a NaN x never compares equal.
GEO_HD float med3_(float x, float lo, float hi) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_fmed3f(x, lo, hi);
#else
    const float m = x > lo ? x : lo;  // NaN x -> lo
    return m < hi ? m : hi;
#endif
}

// c ? a : b for a lane condition c and frame-uniform a, b, as scalar lane-mask
// ops: lane_mask_(c) is the wave's ballot of c (taken where c is computed: a
// ballot of a condition from an earlier block costs two VALU to rebuild it),
// lane_select_ picks by it with an inverse ballot.  hipcc otherwise selects
// the flag bytes per lane in VGPRs.
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint64_t LaneMask;
GEO_HD LaneMask lane_mask_(bool c) { return __builtin_amdgcn_ballot_w64(c); }
GEO_HD bool lane_select_(LaneMask m, bool a, bool b) {
    return __builtin_amdgcn_inverse_ballot_w64((a ? m : 0ull) | (b ? ~m : 0ull));
}
#else
typedef bool LaneMask;
GEO_HD LaneMask lane_mask_(bool c) { return c; }
GEO_HD bool lane_select_(LaneMask m, bool a, bool b) { return m ? a : b; }
#endif

// Step sizes for which the interval stop test of kCurvedOut is exact
// ("Exact group test"): a state entering U > HU from the
// interval always has U' > 0 there (the reference's horizon test `u > 1/rs &&
// u' > 0`, :134, then holds at once) and every later state stays above HU.
// Proved for one f32 RK4 step with h in [2^-10, 1/2]; other steps take the
// general kCurvedIn test.
constexpr float kHorizonStepMin = 0x1p-10f;
constexpr float kHorizonStepMax = 0.5f;

// tol: GEO_MODE_ADAPTIVE local error tolerance in u (<= 0: the default 1e-6).
GEO_HD PixelConsts make_consts(float rs, float sphere_r, float r, float step, uint32_t max_steps,
                               float tol = 0.0f) {
    PixelConsts k;
    k.rs = rs;
    k.sphere_r = sphere_r;
    k.r = r;
    k.step = step;
    k.max_steps = max_steps;
    k.hh = step * 0.5f;
    k.h6 = step / 6.0f;
    k.hh2 = (step * step) * 0.25f;
    k.hhh = (step * step) * 0.5f;
    k.h2_6 = (step * step) / 6.0f;
    k.r3_2 = 1.5f * rs;
    k.sphere_u = 1.0f / sphere_r;
    k.schwarz_u = 1.0f / rs;
    k.u0 = 1.0f / r;
    k.h_over_r2 = (1.0f - rs / r) / (r * r);
    k.inv_r2 = 1.0f / (r * r);
    const float um = 1.0f / (sphere_r > k.r3_2 ? sphere_r : k.r3_2);
    k.bound = 0.9f * (k.u0 < um ? k.u0 : um);
    k.e_out = __builtin_sqrtf(1.0f - rs / r);
    k.e_in = __builtin_sqrtf(-1.0f + rs / r);
    k.barrier_thresh = 4.0f / (27.0f * rs * rs);
    k.r_inside_h = r < rs;
    k.outside = r > rs;
    k.sphere_outside = sphere_r > rs;
    k.inside_sphere = r < sphere_r;
    const float dr = r - k.r3_2;
    k.diff_sides = ((r < k.r3_2) != (sphere_r < k.r3_2)) && (__builtin_fabsf(dr) > 1e-10f);
    k.rs_nonzero = rs != 0.0f;
    // radial rays (:67-104)
    k.radial_by_energy = false;
    if (k.inside_sphere) {
        if (k.outside) {
            k.radial_falling = k.rs_nonzero ? kNoValue : kPi;
            k.radial_outgoing = 0.0f;
        } else if (k.sphere_outside) {
            k.radial_by_energy = true;  // energy > 0 ? 0 : NO_VALUE
            k.radial_falling = k.radial_outgoing = 0.0f;
        } else {
            k.radial_falling = k.radial_outgoing = 0.0f;
        }
    } else {
        k.radial_falling = k.sphere_outside ? 0.0f : kNoValue;
        k.radial_outgoing = kNoValue;
    }
    // pre-filters (:113-117): NO_VALUE when any term holds
    k.pf_always = k.inside_sphere && !k.sphere_outside;
    k.pf_eneg = !k.outside && k.sphere_outside;     // & energy < 0
    k.pf_barrier = k.rs > 0.0f && k.diff_sides;     // & 1/b^2 < 4/(27 rs^2)
    k.pf_falling = r < k.r3_2 && k.inside_sphere;   // & falling
    k.pf_outgoing = r > k.r3_2 && !k.inside_sphere; // & !falling
    k.barrier_lim = k.pf_barrier ? k.barrier_thresh : -__builtin_inff();
    k.e_out2 = k.e_out * k.e_out;
    k.pf_bits = (k.pf_always ? 1u : 0u) | (k.pf_falling ? 2u : 0u) | (k.pf_outgoing ? 4u : 0u);
    k.scale = k.rs_nonzero ? k.r3_2 : 1.0f;
    k.U0 = k.scale * k.u0;
    k.SU = k.scale * k.sphere_u;
    k.BD = k.scale * k.bound;
    k.HU = k.scale * k.schwarz_u;
    k.ub_k = k.scale * (k.e_out * k.u0);
    k.SUp = next_up_(k.SU);
    {
        const bool above0 = k.U0 > k.SU;
        k.kind = !k.rs_nonzero ? kFlat
                 : (k.outside && step >= kHorizonStepMin && step <= kHorizonStepMax) ? kCurvedOut
                                                                                       : kCurvedIn;
        k.stop_lo = above0 ? k.SUp : k.BD;
        k.stop_hi = above0 ? k.HU : k.SU;
        k.stop_bits = (above0 ? 1u : 0u) | ((max_steps != 0u && k.u0 > 0.0f) ? 4u : 0u);
    }
    k.tolU = k.scale * (tol > 0.0f ? tol : kAdaptiveDefaultTol);
    k.tolG = k.tolU * (1.0f / 64.0f);
    k.hmax = step * (float)kAdaptiveMaxGrowth;
    return k;
}

// kFlat for rs = 0; kCurvedOut outside the horizon for the steps its stop
// test is exact for (kHorizonStepMin..Max); kCurvedIn (the reference's full
// per-step tests) otherwise, which is exact for any frame.
GEO_HD int geodesic_kind(const PixelConsts& k) { return k.kind; }

// The integrator works on the scaled state U = c u (c = 3 rs/2): RK4 commutes
// with a linear rescaling of the state, and c f(u) = c(-u + c u^2) becomes
//   F(U) = U (U - 1) = fma(U, U, -U)                     (one FMA),
// or F(U) = -U in flat space (rs = 0, scale 1).  The sphere, escape and
// horizon thresholds are scaled alike (SU, BD, HU); Newton's ratio
// (u - su)/ub is scale-free.
template <int KIND>
GEO_HD float F_(float U) {
    if constexpr (KIND == kFlat)
        return -U;
    else
        return fmaf_(U, U, -U);
}

// One classic RK4 step of U'' = F(U) (sphere_ray_tracer.rs:137-146) in 14
// VALU ops.  The reference's stage values are evaluated in algebraically
// identical forms that need neither a_ub, b_ub nor c_ub:
//   a = U + h/2 UB            b = a + h^2/4 F(U)        [= U + h/2 a_ub]
//   U_h = U + h UB            c = U_h + h^2/2 F(a)      [= U + h b_ub]
//   next_U  = U_h + h^2/6 (F(U) + F(a) + F(b))          [= U + h/6 (UB + 2a_ub + 2b_ub + c_ub)]
//   next_UB = UB + h/6 (F(U) + 2 F(a) + 2 F(b) + F(c))
// hh = h/2, hh2 = h^2/4, hhh = h^2/2, h6 = h/6, h2_6 = h^2/6.
template <int KIND>
GEO_HD void rk4_step(float U, float UB, float h, float hh, float hh2, float hhh, float h6, float h2_6,
                     float* NU, float* NUB) {
    const float fu = F_<KIND>(U);
    const float au = fmaf_(hh, UB, U);
    const float uh = fmaf_(h, UB, U);
    const float fa = F_<KIND>(au);
    const float bu = fmaf_(hh2, fu, au);
    const float fb = F_<KIND>(bu);
    const float cu = fmaf_(hhh, fa, uh);
    const float fc = F_<KIND>(cu);
    const float fab = fa + fb;
    *NU = fmaf_(h2_6, fu + fab, uh);
    *NUB = fmaf_(h6, fmaf_(2.0f, fab, fu) + fc, UB);
}

// The horizon half of the loop test (:134), `u > 1/rs && ub > 0`.  For an
// observer outside the horizon it reduces to `u > 1/rs`: beyond the photon
// sphere u'' > 0, so a ray from r > rs reaches u > 1/rs only while ub > 0.
// (The oracle keeps the full test; tests require bit equality.)
template <int KIND>
GEO_HD bool horizon_(float NU, float NUB, float HU) {
    if constexpr (KIND == kCurvedOut)
        return NU > HU;
    else if constexpr (KIND == kCurvedIn)
        return (NU > HU) & (NUB > 0.0f);
    else
        return false;
}

// Newton on the step length from the steeper end (:150-182), from the
// pre-step state (U, UB) and the post-step state (NU, NUB) of step `it`.
template <int KIND>
GEO_HD float newton_angle(const PixelConsts& k, float U, float UB, float NU, float NUB, uint32_t it) {
    float ns, wu, wub;
    if (__builtin_fabsf(UB) > __builtin_fabsf(NUB)) {
        ns = 0.0f;
        wu = U;
        wub = UB;
    } else {
        ns = k.step;
        wu = NU;
        wub = NUB;
    }
    for (int n = 0; n < kNewtonIters; ++n) {
        ns = ns - divf_(wu - k.SU, wub);
        const float n2 = ns * ns;
        const float n6 = ns * kSixth;
        rk4_step<KIND>(U, UB, ns, ns * 0.5f, n2 * 0.25f, n2 * 0.5f, n6, ns * n6, &wu, &wub);
    }
    return (float)(it - 1u) * k.step + ns;
}

// Ray set-up of solve_ray_fan + solve_geodesic (sphere_ray_tracer.rs:38-132)
// for (st, ct) = (sin theta, cos theta >= 0) of the central-frame direction
// and rct = rcpf_(ct), which the pixel shares with its sky direction (sky_uv).
// Returns false with the traveled angle in *early (radial case, pre-filter
// or failed initial loop test); else the scaled initial state (U, UB).
//
// KIND is the frame-uniform integration kind (geodesic_kind).  Outside the
// horizon (kCurvedOut, kFlat) the energy is the frame constant e_out and the
// pf_eneg term and the energy-decided radial case cannot occur (both need
// r <= rs), so the per-lane tests are the compares on st and 1/b^2 alone
// (their lane masks combine with the frame-uniform flags in scalar ops).
template <int KIND>
GEO_HD bool geodesic_init(const PixelConsts& k, float st, float ct, float rct, float* early, float* U0,
                          float* UB0) {
    // solve_ray_fan per node (:38-49)
    const float rotation = k.r * ct;
    bool falling;
    float energy, e2;
    if (KIND == kCurvedIn && k.r_inside_h) {
        falling = false;
        energy = (-st) * k.e_in;
        e2 = energy * energy;
    } else {
        falling = st > 0.0f;
        energy = k.e_out;
        e2 = k.e_out2;
    }
    const LaneMask falling_m = lane_mask_(falling);
    // radial rays (:67-104), frame-uniform table
    if (rotation < 1e-10f) {
        *early = (KIND == kCurvedIn && k.radial_by_energy) ? (energy > 0.0f ? 0.0f : kNoValue)
                                                           : (falling ? k.radial_falling : k.radial_outgoing);
        return false;
    }
    // 1/b^2 with b = rotation/energy = r ct/energy (:61), from the pixel's 1/ct
    const float inv_b2 = e2 * ((rct * rct) * k.inv_r2);
    // pre-filters (:106-119), frame-uniform terms precomputed
    const bool eneg = KIND == kCurvedIn && k.pf_eneg && energy < 0.0f;
    const bool pf_always = (k.pf_bits & 1u) != 0, pf_falling = (k.pf_bits & 2u) != 0,
               pf_outgoing = (k.pf_bits & 4u) != 0;
    if (pf_always || eneg || inv_b2 < k.barrier_lim || lane_select_(falling_m, pf_falling, pf_outgoing)) {
        *early = kNoValue;
        return false;
    }
    // RK4 init (:122-132), scaled: UB = c u'0, u'0 = sqrt(1/b^2 - (1 - rs/r)/r^2).
    // Outside the horizon E^2 = 1 - rs/r, so the radicand is (E/r)^2 tan^2
    // theta and UB = (c E/r) |st|/ct (ub_k = c E/r): no cancellation where
    // the literal difference loses every digit (|theta| << 1, a tangential
    // ray: up to 4e-4 rad of traveled angle in f32 against the f64 literal
    // form), and no square root.  Inside the horizon both radicand terms are
    // positive and the literal form stays (clamped at 0: the reference
    // yields NaN there only for |theta| < ~1e-8, never at a fan node).
    float UB;
    if (KIND == kCurvedIn && k.r_inside_h) {
        float ub = sqrtf_(fmaxf_(0.0f, inv_b2 - k.h_over_r2));
        if (!falling) ub = -ub;
        UB = k.scale * ub;
    } else {
        UB = (k.ub_k * __builtin_fabsf(st)) * rct;
        if (!falling) UB = -UB;
    }
    // loop test of :134-135 on the initial state (u' > 0 <=> UB > 0;
    // schwarz_u = +inf for rs = 0; u0 > schwarz_u needs r < rs)
    if ((KIND == kCurvedIn && k.u0 > k.schwarz_u && UB > 0.0f) || !(k.stop_bits & 4u)) {
        *early = kNoValue;
        return false;
    }
    *U0 = k.U0;
    *UB0 = UB;
    return true;
}

// The lanes of the wave for which p holds (a uniform SGPR mask), and the
// rarely taken arm of a branch that must stay a branch: a volatile asm cannot
// be speculated, so the compiler cannot turn the arm into a select that every
// group would pay for.
#if defined(__HIP_DEVICE_COMPILE__)
GEO_HD uint64_t ballot_(bool p) { return __builtin_amdgcn_ballot_w64(p); }
GEO_HD bool in_ballot_(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
#define GEO_RARE() asm volatile("")
#else
GEO_HD uint64_t ballot_(bool p) { return p ? 1u : 0u; }
GEO_HD bool in_ballot_(uint64_t m) { return m != 0; }
#define GEO_RARE() ((void)0)
#endif

// Stop flag of one accepted step (reference order: crossing :150, escape
// :184, loop test :134-135).  The integration ends at the first crossing, so
// "above the sphere" (U > SU) is fixed for the whole integration and frame-
// uniform (U0 vs SU).  Outside the horizon the flag is then ONE interval test
// (v_med3_f32 + compare):
//   inside the sphere (U0 > SU): stop <=> NU not in [SU+, HU]
//       (crossing outward | horizon; escape NU < BD < SU is a crossing too)
//   outside (U0 <= SU):          stop <=> NU not in [BD, SU]
//       (crossing inward | escape; the horizon HU > SU is a crossing too)
// `!(NU >= BD)` is (NU < BD) or NaN and, with BD > 0, also covers the `u > 0`
// test.  NaN always stops.  The horizon half of the reference's loop test,
// `u > 1/rs && u' > 0`, is `NU > HU` alone for kCurvedOut: a state that
// enters U > HU from the interval has U' > 0 for the RK4 map at the steps
// kCurvedOut admits ("Exact group test").  kCurvedIn keeps
// the reference's tests as written.
template <int KIND>
struct StopTest {
    float SU, BD, HU, lo, hi;
    float vmin;  // above0 ? 0 : -inf (exact())
    bool above0;
    GEO_HDM explicit StopTest(const PixelConsts& k)
        : SU(k.SU), BD(k.BD), HU(k.HU), lo(k.stop_lo), hi(k.stop_hi),
          vmin((k.stop_bits & 1u) != 0 ? 0.0f : -__builtin_inff()), above0((k.stop_bits & 1u) != 0) {}
    GEO_HDM bool operator()(float NU, float NUB) const {
        if constexpr (KIND == kCurvedIn)
            return ((NU > SU) != above0) | !(NU >= BD) | ((NU > HU) & (NUB > 0.0f));
        else
            return med3_(NU, lo, hi) != NU;
    }
    // The same flag with the horizon's `u' > 0` evaluated, for a stepper the
    // kCurvedOut argument does not cover (the adaptive RK5(4) map, whose step
    // grows to 16 h): NU < lo | NaN | (NU > hi & NUB > vmin), where vmin = 0
    // inside the sphere (the horizon test) and -inf outside it (NU > hi = SU
    // is a crossing; a NaN NUB comes with a NaN NU).  Three compares, each
    // balloted on its own.
    GEO_HDM bool exact(float NU, float NUB) const {
        if constexpr (KIND == kCurvedOut)
            return !(NU >= lo) | ((NU > hi) & (NUB > vmin));
        else
            return (*this)(NU, NUB);
    }
    // exact() as a wave mask in two parts, for the adaptive loop: out_mask,
    // a superset (kCurvedOut: NU outside [lo, hi] or NaN, one v_med3_f32 and
    // a compare per attempt), then exact_refine, taken only when out_mask
    // has lanes: out & exact_refine == exact, because a state outside the
    // interval stops iff it is below lo (or NaN) or its U' exceeds vmin.
    // hipcc rebuilds a compound condition through a VGPR before its ballot,
    // so the compares are balloted one by one.
    GEO_HDM uint64_t out_mask(float NU) const {
        if constexpr (KIND == kCurvedOut)
            return ballot_(med3_(NU, lo, hi) != NU);
        else
            return ~0ull;
    }
    GEO_HDM uint64_t exact_refine(float NU, float NUB) const {
        if constexpr (KIND == kCurvedOut)
            return ballot_(!(NU >= lo)) | ballot_(NUB > vmin);
        else
            return ballot_((*this)(NU, NUB));
    }
};


template <int G, int KIND>
GEO_HD void group_steps_(float u, float b, float h, float hh, float hh2, float hhh, float h6, float h2_6,
                         float (&ou)[G], float (&ob)[G]) {
#pragma unroll
    for (int j = 0; j < G; ++j)
        rk4_step<KIND>(j ? ou[j - 1] : u, j ? ob[j - 1] : b, h, hh, hh2, hhh, h6, h2_6, &ou[j], &ob[j]);
}

// IEEE minNum/maxNum of three floats (a NaN operand yields the min/max of the
// others) as one v_min3_f32 / v_max3_f32.  hipcc lowers fminf chains on
// loop-carried values with a canonicalising v_max_f32 x, x per operand first
// (2 extra VALU per group, measured); the states are arithmetic results, never
// signaling NaNs, so the canonicalisation is a no-op here.
GEO_HD float min3_(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return __builtin_fminf(__builtin_fminf(a, b), c);
#endif
}
GEO_HD float max3_(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
#endif
}

// The exit test of a group of G RK4 steps, exact: it holds iff the per-step
// StopTest holds for one of the group's G states (the group's start state is
// inside the interval, or the previous group would have stopped).  Three
// forms, chosen per frame:
//   kTestLow  (kCurvedOut/kFlat, observer inside the sphere): the minimum of
//             states 1..G-1 below lo, or state G outside [lo, hi] (or NaN).
//             A state above hi = HU needs no test of its own: it has U' > 0,
//             and U > HU with U' >= 0 maps to U' >= U, U'' >= U' under the
//             f32 RK4 map (all stage values exceed 1, so every F >= 0), so
//             state G is above HU too.  A NaN state makes every later state
//             NaN, state G included, which the range test sees (the minimum
//             ignores NaN operands).
//   kTestBoth (kCurvedOut/kFlat, observer outside the sphere): the minimum
//             below lo or the maximum above hi (the ray can graze the sphere,
//             entering and leaving within a group), or state G outside.
//   kTestEach (kCurvedIn): the reference's compound test on every state.
// Round 2 tested state G alone, which is exact only while no state leaves the
// interval and comes back within a group; a near-radial outgoing ray at a
// large step breaks that (RK4 overshoots U = 0, where F(U) = U^2 - U > 0
// turns it back: seed 70751).  For G = 4 the minimum is one v_min3_f32: 4
// VALU per group against 2 for state G alone.
// hipcc takes the ballot of a single compare as its mask but rebuilds any
// other condition through a VGPR (two VALU), so the compares are balloted one
// by one and ORed in scalar ops; the compound test is ORed first and balloted
// once.
constexpr int kTestLow = 0;
constexpr int kTestBoth = 1;
constexpr int kTestEach = 2;

template <int G, int KIND, int TEST>
GEO_HD uint64_t group_stop_(const StopTest<KIND>& stop_at, const float (&ou)[G], const float (&ob)[G]) {
    if constexpr (TEST == kTestEach || G == 1) {
        bool s = false;
#pragma unroll
        for (int j = 0; j < G; ++j) s = s | stop_at(ou[j], ob[j]);
        return ballot_(s);
    } else {
        // states 1..G-1 (ou[0..G-2]): their minimum (and maximum)
        float mn = ou[0], mx = ou[0];
        int j = 1;
        for (; j + 2 <= G - 1; j += 2) {
            mn = min3_(mn, ou[j], ou[j + 1]);
            if constexpr (TEST == kTestBoth) mx = max3_(mx, ou[j], ou[j + 1]);
        }
        for (; j < G - 1; ++j) {
            mn = __builtin_fminf(mn, ou[j]);
            if constexpr (TEST == kTestBoth) mx = __builtin_fmaxf(mx, ou[j]);
        }
        const float last = ou[G - 1];
        uint64_t m = ballot_(mn < stop_at.lo) | ballot_(med3_(last, stop_at.lo, stop_at.hi) != last);
        if constexpr (TEST == kTestBoth) m |= ballot_(mx > stop_at.hi);
        return m;
    }
}

// The lower half of kTestLow alone: the minimum of all G states below lo (a
// NaN state is left to a later test: NaN propagates).  The pair loop's A
// groups take this test (3 VALU instead of 4) and leave a stop above hi to
// the B group's full test (run_groups_pp): a state above hi = HU keeps every
// later state above it (group_stop_'s kTestLow argument), so B's last state is
// above hi, or NaN, too.
template <int G>
GEO_HD uint64_t group_low_(float lo, const float (&ou)[G]) {
    float mn = ou[0];
    int j = 1;
    for (; j + 2 <= G; j += 2) mn = min3_(mn, ou[j], ou[j + 1]);
    for (; j < G; ++j) mn = min3_(mn, ou[j], ou[j]);
    return ballot_(mn < lo);
}

// The group loop: G RK4 steps per exit test; returns the steps before the
// stopping group (or `all` when the budget of whole groups runs out), with the
// group's G + 1 states in su_/sb_.  A lane that stops inside a group discards
// the rest of it (the oracle keeps the literal per-step loop; tests require
// bit equality).
//
// The loop alternates two register sets, group A stepping from X into
// a_1..a_G and group B from a_G into b_1..b_{G-1}, X, so neither ends with a
// start-state move.  Its exit is wave-uniform (every lane done, or the
// budget): a lane that stops is masked off and keeps its stopping group's
// states in whichever set that group wrote; after the loop one select per
// state puts them in su_/sb_.
template <int G, int KIND, int TEST>
GEO_HD uint32_t run_groups_pp(const StopTest<KIND>& stop_at, uint32_t ngroups, uint32_t all, float h, float hh,
                              float hh2, float hhh, float h6, float h2_6, float (&su_)[G + 1], float (&sb_)[G + 1]) {
    float xu = su_[0], xb = sb_[0];  // X: group A's start, group B's end
    float au[G], ab[G], bu[G], bb[G];  // a_1..a_G; b_1..b_{G-1} (b_G is X)
    // Every element read after the loop as a state of the lane's stopping
    // group was written by that group; the others are selected but unused
    // (a lane on the budget continues from su_[0] alone).  Defined without
    // instructions: an empty asm output (14 v_mov otherwise).
#pragma unroll
    for (int j = 0; j < G; ++j) {
        GEO_UNSET(au[j]);
        GEO_UNSET(ab[j]);
        GEO_UNSET(bu[j]);
        GEO_UNSET(bb[j]);
    }
    // Groups q = 0, 2, 4, ... are A groups, 1, 3, ... B groups.  A lane that
    // stops in group q records it = q G (a multiple of G below `all`), so the
    // set its states sit in is (it / G) & 1 after the loop.
    //
    // The lanes still integrating are the wave-uniform mask `live`, which is
    // also the exec mask of the group steps: no per-lane flag, so the loop's
    // scalar work is the masked regions, one AND per stop test and a branch
    // (`hit`, uniform) past the rare block where lanes stop.
    uint64_t live = ballot_(true);
    uint32_t it = all;
    uint32_t q = 0;
    // One exit test per A+B pair of groups: a group whose lanes are all done
    // runs with an empty exec mask, which the masked region's execz branch
    // skips, so the pair needs no test between its groups; an odd budget's
    // last group is an A group after the loop.  The loop has one exit edge
    // (hipcc's structurizer turns a second one into lane-mask flags at the
    // latch): an empty `live` zeroes the pair counter instead of breaking.
    uint32_t rem = ngroups >> 1;
    while (rem != 0) {
        if (in_ballot_(live)) group_steps_<G, KIND>(xu, xb, h, hh, hh2, hhh, h6, h2_6, au, ab);
        uint64_t hit = (TEST == kTestLow ? group_low_<G>(stop_at.lo, au) : group_stop_<G, KIND, TEST>(stop_at, au, ab)) &
                       live;
        --rem;
        if (hit != 0) {
            if (in_ballot_(hit)) {
                GEO_RARE();
                it = q * (uint32_t)G;
            }
            live &= ~hit;
            rem = live == 0 ? 0u : rem;  // (the B group below then runs on an empty exec mask: skipped)
        }
        if (in_ballot_(live)) {
            float ou[G], ob[G];
            group_steps_<G, KIND>(au[G - 1], ab[G - 1], h, hh, hh2, hhh, h6, h2_6, ou, ob);
#pragma unroll
            for (int j = 0; j < G - 1; ++j) {
                bu[j] = ou[j];
                bb[j] = ob[j];
            }
            xu = ou[G - 1];
            xb = ob[G - 1];
        }
        float tu[G], tb[G];
#pragma unroll
        for (int j = 0; j < G - 1; ++j) {
            tu[j] = bu[j];
            tb[j] = bb[j];
        }
        tu[G - 1] = xu;
        tb[G - 1] = xb;
        hit = group_stop_<G, KIND, TEST>(stop_at, tu, tb) & live;
        q += 2u;
        // `live` empties only where lanes stop, so its test sits in that
        // branch: a pair without stops ends in the counter's compare alone
        if (hit != 0) {
            uint64_t in_a = 0;
            if constexpr (TEST == kTestLow) {
                // A stops above hi (or at a NaN), left to this test: a_G is
                // then above hi or NaN.  The A group's start state X is B's
                // end now; the replay (geodesic_finish) reads it only as the
                // state before a first stop at a_1, where any value above SU
                // gives the same result (no crossing; a NaN a_1 gives NaN
                // either way), so hi stands in for it.
                in_a = hit & ~ballot_(au[G - 1] <= stop_at.hi);
                if (in_a != 0) {
                    if (in_ballot_(in_a)) {
                        GEO_RARE();
                        it = (q - 2u) * (uint32_t)G;
                        xu = stop_at.hi;
                    }
                }
            }
            if (in_ballot_(hit & ~in_a)) {
                GEO_RARE();
                it = (q - 1u) * (uint32_t)G;
            }
            live &= ~hit;
            rem = live == 0 ? 0u : rem;
        }
    }
    if ((ngroups & 1u) != 0 && live != 0) {
        if (in_ballot_(live)) group_steps_<G, KIND>(xu, xb, h, hh, hh2, hhh, h6, h2_6, au, ab);
        const uint64_t hit = group_stop_<G, KIND, TEST>(stop_at, au, ab) & live;
        if (in_ballot_(hit)) {
            GEO_RARE();
            it = q * (uint32_t)G;
        }
        ++q;
    }
    // the set holding the stopping group (B: start a_G, then b_1..b_{G-1}, X);
    // a lane on the budget continues from the last group's end state, which
    // sits where a B group's start state (a_G, after an A group) or an A
    // group's (X, after a B group) does
    const bool in_b = it < all ? ((it / (uint32_t)G) & 1u) != 0 : (q & 1u) != 0;
    su_[0] = in_b ? au[G - 1] : xu;
    sb_[0] = in_b ? ab[G - 1] : xb;
#pragma unroll
    for (int j = 0; j < G - 1; ++j) {
        su_[j + 1] = in_b ? bu[j] : au[j];
        sb_[j + 1] = in_b ? bb[j] : ab[j];
    }
    su_[G] = in_b ? xu : au[G - 1];
    sb_[G] = in_b ? xb : ab[G - 1];
    return it;
}

// After the group loop: from the G + 1 states of the lane's stopping group
// and `it` = the steps before it (or the whole-group budget), the first
// stopping step, the budget tail of fewer than G steps, the crossing test and
// Newton (sphere_ray_tracer.rs:150-191).  *steps = executed main-loop RK4
// steps.
template <int G, int KIND>
GEO_HD float geodesic_finish(const PixelConsts& k, const StopTest<KIND>& stop_at, uint32_t it,
                             float (&su_)[G + 1], float (&sb_)[G + 1], uint32_t* steps) {
    const uint32_t ms = k.max_steps;
    // Opaque copies: the per-step flags are recomputed from the state rather
    // than carried out of the loop as lane masks.
#pragma unroll
    for (int j = 0; j <= G; ++j) {
        GEO_OPAQUE(su_[j]);
        GEO_OPAQUE(sb_[j]);
    }
    GEO_OPAQUE(it);
    float ou = su_[0], oub = sb_[0], nu = su_[0], nub = sb_[0];
    if (it + (uint32_t)G <= ms) {
        // stopped inside the group: the first step j whose flag holds
        bool found = false;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const bool sj = !found && stop_at(su_[j + 1], sb_[j + 1]);
            if (sj) {
                ou = su_[j]; oub = sb_[j]; nu = su_[j + 1]; nub = sb_[j + 1];
                it += (uint32_t)j + 1u;
            }
            found = found | sj;
        }
    } else {
        // budget exit: fewer than G steps left, one test per step
        float cu = su_[0], cb = sb_[0];
        for (uint32_t r = it; r < ms; ++r) {
            rk4_step<KIND>(cu, cb, k.step, k.hh, k.hh2, k.hhh, k.h6, k.h2_6, &nu, &nub);
            ou = cu;
            oub = cb;
            ++it;
            if (stop_at(nu, nub)) break;
            cu = nu;
            cb = nub;
            ou = nu;  // no crossing if the budget ends here
            oub = nub;
        }
    }
    *steps = it;
    if ((nu > k.SU) == (ou > k.SU)) return kNoValue;  // stopped without a crossing
    return newton_angle<KIND>(k, ou, oub, nu, nub, it);
}

// RK4 steps per exit test: 4 is the fastest on gfx950 (G = 5, 6, 8 +0.4, +5,
// +6 % on config 3: the steps a lane wastes in its stopping group outweigh the
// saved tests; DESIGN.md §4, tools/ubench/loop_ab.hip at 3cd1aa2)
constexpr int kGroup = 4;

// Traveled angle of the ray at angle theta to the black hole, or kNoValue.
// *steps = executed main-loop RK4 steps.  KIND: the integration kind
// (geodesic_kind); LOOP = RK4 steps per exit test.
template <int KIND, int LOOP = kGroup>
GEO_HD float geodesic_angle_v(const PixelConsts& k, float st, float ct, float rct, uint32_t* steps) {
    *steps = 0;
    float U, UB, early;
    if (!geodesic_init<KIND>(k, st, ct, rct, &early, &U, &UB)) return early;
    float h = k.step, hh = k.hh, hh2 = k.hh2, hhh = k.hhh, h6 = k.h6, h2_6 = k.h2_6;
    // Main loop (:134-191), restructured for the wave64 VALU: per step the
    // lane-exit flag is StopTest (crossing | escape | horizon); the budget
    // (:135) is wave-uniform.
    StopTest<KIND> stop_at(k);
    // The loop's frame constants in VGPRs: on gfx950 a VALU op that reads an
    // SGPR issues at about half the rate of an all-VGPR one
    // (tools/ubench/op_rates.hip), and 6 of the step's 14 ops read one.
    GEO_OPAQUE(h);
    GEO_OPAQUE(hh);
    GEO_OPAQUE(hh2);
    GEO_OPAQUE(hhh);
    GEO_OPAQUE(h6);
    GEO_OPAQUE(h2_6);
    GEO_OPAQUE(stop_at.lo);
    GEO_OPAQUE(stop_at.hi);
    // G RK4 steps per exit test (the budget in whole groups is a wave-uniform
    // bound)
    constexpr int G = LOOP;
    const uint32_t ms = k.max_steps;
    const uint32_t ngroups = ms / (uint32_t)G;
    float su_[G + 1], sb_[G + 1];
    su_[0] = U;
    sb_[0] = UB;
#pragma unroll
    for (int j = 1; j <= G; ++j) {
        su_[j] = U;
        sb_[j] = UB;
    }
    // per lane: steps before its stopping group (budget: all)
    uint32_t it;
    if constexpr (KIND == kCurvedIn)
        it = run_groups_pp<G, KIND, kTestEach>(stop_at, ngroups, ngroups * (uint32_t)G, h, hh, hh2, hhh, h6, h2_6,
                                               su_, sb_);
    else if (stop_at.above0)  // frame-uniform
        it = run_groups_pp<G, KIND, kTestLow>(stop_at, ngroups, ngroups * (uint32_t)G, h, hh, hh2, hhh, h6, h2_6,
                                              su_, sb_);
    else
        it = run_groups_pp<G, KIND, kTestBoth>(stop_at, ngroups, ngroups * (uint32_t)G, h, hh, hh2, hhh, h6, h2_6,
                                               su_, sb_);
    return geodesic_finish<G, KIND>(k, stop_at, it, su_, sb_, steps);
}

// Runtime-dispatched form (host tests); the kernel instantiates per kind.
GEO_HD float geodesic_angle(const PixelConsts& k, float st, float ct, uint32_t* steps) {
    const float rct = rcpf_(ct);
    switch (geodesic_kind(k)) {
        case kCurvedOut: return geodesic_angle_v<kCurvedOut>(k, st, ct, rct, steps);
        case kCurvedIn: return geodesic_angle_v<kCurvedIn>(k, st, ct, rct, steps);
        default: return geodesic_angle_v<kFlat>(k, st, ct, rct, steps);
    }
}

// ---- GEO_MODE_ADAPTIVE (config 5; a build extension, not in the reference) ----
//
// Dormand-Prince RK5(4) (J. Comput. Appl. Math. 6 (1980) 19-26, RK5(4)7M) on
// the scaled state, in Nystrom form: for (U, V)' = (V, F(U)) the stage values
// are U_i = U + c_i h V + h^2 sum_j (A^2)_ij G_j with G_j = F(U_j), so no stage
// V is formed; the 5th-order solution is
//   NU = U + h V + h^2 sum_j (bA)_j G_j,   NV = V + h sum_j b_j G_j,
// and the embedded error estimate in U is h^2 sum_j ((b - b*)A)_j G_j (stage 7,
// the FSAL stage, does not enter it).  Coefficients: exact rationals rounded
// once to f32 (tools/dp5_coeffs.py); zeros dropped ((A^2)_{i,i-1} = b2 =
// (bA)_2 = (bA)_6 = (eA)_2 = 0, c6 = 1).  44 VALU ops per attempt.
namespace dp5 {
constexpr float c2 = 0x1.99999ap-3f, c3 = 0x1.333334p-2f, c4 = 0x1.99999ap-1f, c5 = 0x1.c71c72p-1f;
constexpr float a31 = 0x1.70a3d8p-5f;
constexpr float a41 = -0x1.eb851ep-2f, a42 = 0x1.99999ap-1f;
constexpr float a51 = -0x1.dde5dcp+0f, a52 = 0x1.a5de0ep+1f, a53 = -0x1.08b37cp+0f;
constexpr float a61 = -0x1.026c9cp+1f, a62 = 0x1.08ba2ep+2f, a63 = -0x1.b26c9cp+0f, a64 = 0x1.45d174p-4f;
constexpr float q1 = 0x1.755556p-4f, q3 = 0x1.420338p-2f, q4 = 0x1.0aaaaap-3f, q5 = -0x1.256f18p-5f;
constexpr float b1 = 0x1.755556p-4f, b3 = 0x1.cc049ap-2f, b4 = 0x1.4d5556p-1f, b5 = -0x1.4a1cfcp-2f,
                b6 = 0x1.0c30c4p-3f;
constexpr float e1 = 0x1.5b9754p-9f, e3 = -0x1.938a4p-8f, e4 = 0x1.4da74p-7f, e5 = -0x1.be0506p-9f,
                e6 = -0x1.ad1ad2p-9f;
}  // namespace dp5

// One attempt: 5th-order (NU, NV) and the error sum SE (error = |SE| h^2).
// Stage values as U_i = (U + c_i hV) + h^2 S_i with hV = h V and h^2 formed
// once (c6 = 1 shares U + hV with NU): 44 VALU per attempt.
template <int KIND>
GEO_HD void dp5_step(float U, float V, float h, float hh, float* NU, float* NV, float* SE) {
    using namespace dp5;
    const float hv = h * V;
    const float g1 = F_<KIND>(U);
    const float u2 = fmaf_(c2, hv, U);
    const float g2 = F_<KIND>(u2);
    const float u3 = fmaf_(hh, a31 * g1, fmaf_(c3, hv, U));
    const float g3 = F_<KIND>(u3);
    const float u4 = fmaf_(hh, fmaf_(a42, g2, a41 * g1), fmaf_(c4, hv, U));
    const float g4 = F_<KIND>(u4);
    const float u5 = fmaf_(hh, fmaf_(a53, g3, fmaf_(a52, g2, a51 * g1)), fmaf_(c5, hv, U));
    const float g5 = F_<KIND>(u5);
    const float w = U + hv;
    const float u6 = fmaf_(hh, fmaf_(a64, g4, fmaf_(a63, g3, fmaf_(a62, g2, a61 * g1))), w);
    const float g6 = F_<KIND>(u6);
    *NU = fmaf_(hh, fmaf_(q5, g5, fmaf_(q4, g4, fmaf_(q3, g3, q1 * g1))), w);
    *NV = fmaf_(h, fmaf_(b6, g6, fmaf_(b5, g5, fmaf_(b4, g4, fmaf_(b3, g3, b1 * g1)))), V);
    *SE = fmaf_(e6, g6, fmaf_(e5, g5, fmaf_(e4, g4, fmaf_(e3, g3, e1 * g1))));
}

// Traveled angle with error-controlled steps, or kNoValue; *steps = step
// attempts (accepted + rejected).  Same ray set-up, stop order and Newton
// sphere crossing as the fixed-step path (sphere_ray_tracer.rs:60-193), with
// the RK5 map in place of RK4.  Step control is power-of-two so every step
// is an exact multiple of the initial one:
//   |SE| h^2 > tolU           reject, h /= 2
//   |SE| h^2 < tolU/64        accept, then h = min(2h, hmax)  (5th order: x32)
//   otherwise                 accept, keep h
//
// The loop is wave-uniform: every lane that entered it attempts a step per
// iteration, with no per-lane exit and no exec-mask bookkeeping; the lanes
// still integrating are the scalar mask `live`.  A lane that stops (an
// accepted step's stop test) records its step's start (U, V, h, ang) and end
// (NU, NV) in a rarely taken block, leaves `live`, and keeps stepping
// harmlessly (its registers are no longer read).  The loop ends when `live`
// is empty or the budget is spent.  Round 2's per-lane `break` cost 26 SALU
// and ~10 VALU of mask and state bookkeeping per attempt.
template <int KIND>
GEO_HD float geodesic_angle_adaptive(const PixelConsts& k, float st, float ct, float rct, uint32_t* steps) {
    *steps = 0;
    float U, V, early;
    if (!geodesic_init<KIND>(k, st, ct, rct, &early, &U, &V)) return early;
    const StopTest<KIND> stop_at(k);
    const uint32_t ms = k.max_steps;
    float h = k.step, ang = 0.0f;
    // the stopping step: start (sU, sV, sh, sang) and end (sNU, sNV)
    float sU, sV, sh, sang, sNU, sNV;
    GEO_UNSET(sU);
    GEO_UNSET(sV);
    GEO_UNSET(sh);
    GEO_UNSET(sang);
    GEO_UNSET(sNU);
    GEO_UNSET(sNV);
    // attempts up to and including the lane's stop; 0: no stop (the budget)
    uint32_t it = 0;
    uint64_t live = ballot_(true);
    // one exit edge (an empty `live` ends the count instead of a break: hipcc
    // turns a second exit into lane-mask flags at the latch)
    for (uint32_t n = 1; n <= ms; ++n) {
        float NU, NV, SE;
        const float hh = h * h;
        dp5_step<KIND>(U, V, h, hh, &NU, &NV, &SE);
        const float err = __builtin_fabsf(SE) * hh;
        const bool acc = !(err > k.tolU);
        uint64_t hit = ballot_(acc) & stop_at.out_mask(NU) & live;
        if (hit != 0) hit &= stop_at.exact_refine(NU, NV);
        if (hit != 0) {
            if (in_ballot_(hit)) {
                GEO_RARE();
                sU = U;
                sV = V;
                sh = h;
                sang = ang;
                sNU = NU;
                sNV = NV;
                it = n;
            }
            live &= ~hit;
            n = live == 0 ? ms : n;
        }
        // the new step as h times 2, 1 or 1/2 (exact: the same bits as h + h,
        // h and h * 0.5), one multiply after two selects of the factor; the
        // cap as a growth test (h = step 2^j, so h < hmax implies 2h <= hmax)
        const float grow = (err < k.tolG && h < k.hmax) ? 2.0f : 1.0f;
        U = acc ? NU : U;
        V = acc ? NV : V;
        ang = acc ? ang + h : ang;
        h = h * (acc ? grow : 0.5f);
    }
    *steps = it != 0 ? it : ms;
    if (it == 0 || (sNU > k.SU) == (sU > k.SU)) return kNoValue;
    // Newton on the step length from the steeper end (:150-182)
    float ns, wu, wv;
    if (__builtin_fabsf(sV) > __builtin_fabsf(sNV)) {
        ns = 0.0f; wu = sU; wv = sV;
    } else {
        ns = sh; wu = sNU; wv = sNV;
    }
    for (int n = 0; n < kNewtonIters; ++n) {
        ns = ns - divf_(wu - k.SU, wv);
        float se;
        dp5_step<KIND>(sU, sV, ns, ns * ns, &wu, &wv, &se);
    }
    return sang + ns;
}

// 3x3 part of a column-major mat4 times v (w = 0).
GEO_HD void mat3_mul(const float* m, float x, float y, float z, float* ox, float* oy, float* oz) {
    *ox = fmaf_(m[8], z, fmaf_(m[4], y, m[0] * x));
    *oy = fmaf_(m[9], z, fmaf_(m[5], y, m[1] * x));
    *oz = fmaf_(m[10], z, fmaf_(m[6], y, m[2] * x));
}

// shader.wgsl:60-75 — pixel (px, py) of a width x height frame to the
// direction in the black-hole-central frame (unit up to rounding).
//
// Camera ray (:60-64): the pixel centre's NDC, nx = (2 px + 1 - W)/W and
// ny = (H - 2 py - 1)/H (full-screen quad, basic_sphere_buffer.rs:63-83),
// scaled by the FOV column w and rotated by display_to_movement's 3 x 3 part:
//   d = M0 (-ny M0[12], -nx M0[13], M0[14]) = py A + px B + C,
// affine in the integer pixel coordinates.  A, B, C are frame constants
// (CameraConsts, evaluated in f64 and rounded once to f32, on the host), so
// a pixel's ray is two FMAs per component.
//
// The aberration (:69-70), sin(l') = (s - k)/(1 - s k) with phi kept, is
// applied as the boost along z it is: for the unnormalised ray d, |d| = L,
//   e_z = (d_z - k L)/(L - k d_z),   e_xy = d_xy sqrt(1 - k^2)/(L - k d_z),
// (|e| = 1), so steps 2-5 need one sqrt, one reciprocal and no
// transcendental.  kt = sqrt(1 - k^2) is a frame constant (aberration_kt).
// movement_to_central (:72-74) is skipped where it is exactly the identity
// (the Unmoving and FrozenFall states, observer.rs:243-246): a product with
// it can turn -0 into +0, so the skip is part of the specification.
GEO_HD float aberration_kt(float psi_k) { return __builtin_sqrtf(fmaf_(-psi_k, psi_k, 1.0f)); }

struct CameraConsts {
    float a[3], b[3], c[3];  // d = py a + px b + c
    bool m1_identity;        // movement_to_central's 3 x 3 part is exactly the identity
};

// Host (f64, then one rounding per constant; the oracle evaluates the same
// expressions).  m0 = display_to_movement, m1 = movement_to_central.
GEO_HD CameraConsts camera_consts(const float* m0, const float* m1, uint32_t width, uint32_t height) {
    CameraConsts cc;
    const double w = (double)width, h = (double)height;
    const double sx = 2.0 / w, ox = (1.0 - w) / w;   // nx = px sx + ox
    const double sy = -2.0 / h, oy = (h - 1.0) / h;  // ny = py sy + oy
    for (int i = 0; i < 3; ++i) {
        const double p = -(double)m0[12] * (double)m0[i];     // d_i's ny coefficient
        const double q = -(double)m0[13] * (double)m0[4 + i]; // d_i's nx coefficient
        const double r = (double)m0[14] * (double)m0[8 + i];
        cc.a[i] = (float)(sy * p);
        cc.b[i] = (float)(sx * q);
        cc.c[i] = (float)((oy * p + ox * q) + r);
    }
    cc.m1_identity = m1[0] == 1.0f && m1[1] == 0.0f && m1[2] == 0.0f && m1[4] == 0.0f && m1[5] == 1.0f &&
                     m1[6] == 0.0f && m1[8] == 0.0f && m1[9] == 0.0f && m1[10] == 1.0f;
    return cc;
}

GEO_HD void pixel_central_dir(const CameraConsts& cc, const float* m1, float psi_k, float kt, uint32_t px,
                              uint32_t py, float* c2x, float* c2y, float* c2z) {
    const float fx = (float)px, fy = (float)py;
    const float dx = fmaf_(fy, cc.a[0], fmaf_(fx, cc.b[0], cc.c[0]));
    const float dy = fmaf_(fy, cc.a[1], fmaf_(fx, cc.b[1], cc.c[1]));
    const float dz = fmaf_(fy, cc.a[2], fmaf_(fx, cc.b[2], cc.c[2]));
    const float len = sqrtf_(fmaf_(dz, dz, fmaf_(dy, dy, dx * dx)));
    const float id = rcpf_(fmaf_(-psi_k, dz, len));
    const float g = kt * id;
    const float ex = dx * g, ey = dy * g, ez = fmaf_(-psi_k, len, dz) * id;
    if (cc.m1_identity) {
        *c2x = ex;
        *c2y = ey;
        *c2z = ez;
    } else {
        mat3_mul(m1, ex, ey, ez, c2x, c2y, c2z);  // to_cart, then movement_to_central (:72-74)
    }
}

// floor(x) as an int32 for |x| < 2^31 (the sampler's texel coordinates):
// one v_cvt_flr_i32_f32 on the device, where hipcc emits v_floor_f32 +
// v_cvt_i32_f32 (two half-rate opcodes) for the cast of floorf.
GEO_HD int32_t floor_i32_(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
#else
    return (int32_t)__builtin_floorf(x);
#endif
}

// Fan lookup (shader.wgsl:77-84); i+1 clamped to n-1 (weight 0 there).
// (pi/2 - asin(st)) / pi is acos(st) / pi, computed as such (acos_pi_, in
// [0, 1] for every input, so the node index is in [0, n-1] with no clamp).
// On the device, with the same bits: the index by v_cvt_flr_i32_f32 and the
// weight by v_fract_f32 (t - floor(t), exact for t >= 0).
struct FanPos {
    uint32_t i, i1;  // nodes
    float w;         // weight of node i1
};
GEO_HD FanPos fan_pos(uint32_t n, float st) {
    const float t = acos_pi_(st) * (float)(n - 1u);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t i = (uint32_t)floor_i32_(t);
    const float w = __builtin_amdgcn_fractf(t);
#else
    const float fl = __builtin_floorf(t);
    const uint32_t i = (uint32_t)fl;
    const float w = t - fl;
#endif
    const uint32_t i1 = (i + 1u < n) ? i + 1u : n - 1u;
    return FanPos{i, i1, w};
}
GEO_HD float fan_at(const float* fan, const FanPos& p) { return fan[p.i] * (1.0f - p.w) + fan[p.i1] * p.w; }
GEO_HD float fan_lerp(const float* fan, uint32_t n, float st) { return fan_at(fan, fan_pos(n, st)); }

// sin theta of the central-frame direction, c2z clamped to [-1, 1] (to_polar's
// asin argument, :75) by one v_med3_f32 (a NaN becomes -1, where a compare-
// and-select clamp would keep it: 4 VALU for no case a frame produces; c2z
// is an arithmetic result, so never a signaling NaN, which med3 would quiet).
GEO_HD float central_sin(float c2z) { return med3_(c2z, -1.0f, 1.0f); }

// |(c2x, c2y)| = cos theta of the central-frame direction (to_polar, :75).
GEO_HD float central_rho(float c2x, float c2y) { return sqrtf_(fmaf_(c2y, c2y, c2x * c2x)); }

// shader.wgsl:90-100 — (phi of c2, lambda') to sky-sphere (U, V); rho = central_rho, rrho = rcpf_(rho).
GEO_HD void sky_uv(const float* m2, float c2x, float c2y, float rho, float rrho, float lam, float* U, float* V) {
    float sl, cl;
    sincos_sky_(lam, &sl, &cl);
    // to_cart(phi, lam) with (cos phi, sin phi) = (c2x, c2y)/rho
    float ex = cl, ey = 0.0f;
    if (rho > 0.0f) {
        const float w = cl * rrho;
        ex = c2x * w;
        ey = c2y * w;
    }
    float x, y, z;
    mat3_mul(m2, ex, ey, sl, &x, &y, &z);
    // polar.x / 2pi wrapped into [0, 1] and 1/2 - polar.y / pi = acos(z) / pi
    // (:95-100).  U is clamped with NaN -> 0 by one v_med3_f32 (the med3 of a
    // NaN is the IEEE min of the other two, 0; atan2_turns_ never returns -0);
    // V is in [0, 1] for every z (acos_pi_).
    *U = med3_(atan2_turns_(y, x), 0.0f, 1.0f);
    *V = acos_pi_(z);
}

// Packed channel pairs of the bilinear sample: R|B and G|A in the two 16-bit
// halves of a u32 (no field overflows).
GEO_HD uint32_t rb_(uint32_t t) { return t & 0x00FF00FFu; }
GEO_HD uint32_t ga_(uint32_t t) { return (t >> 8) & 0x00FF00FFu; }
// Operands < 2^24 (packed pairs <= 0x00FF00FF, weights <= 256): the 24-bit
// multiply (v_mul_u32_u24 / v_mad_u32_u24, full rate) gives the same low 32
// bits as v_mul_lo_u32 (quarter rate), which is what hipcc picks otherwise.
GEO_HD uint32_t mul24_(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__umul24(a, b);
#else
    return a * b;
#endif
}
GEO_HD uint32_t lerp2_(uint32_t a, uint32_t b, uint32_t ia, uint32_t wb) { return mul24_(a, ia) + mul24_(b, wb); }
GEO_HD uint32_t div255_(uint32_t v) {  // round(v / 255) for v <= 255 * 255
    const uint32_t p = v + 128u;
    return (p + (p >> 8)) >> 8;
}
GEO_HD uint32_t blend255_(uint32_t c, uint32_t a) { return div255_(c * a); }  // round(c*a/255)

// The texel quad (ix0, iy0), (ix0+1, iy0), (ix0, iy0+1), (ix0+1, iy0+1) of a
// tw x th equirect, U wrapping and V clamping; ix0 in [-1, tw-1] and iy0 in
// [-1, th-1] for U, V in [0, 1].  fetch(i): texel i of the row-major texture.
template <typename Fetch>
struct WrapClampQuad {
    Fetch fetch;
    uint32_t tw, th;
    GEO_HDM void operator()(int ix0, int iy0, uint32_t (&t)[4]) const {
        const int w = (int)tw, h = (int)th;
        if (ix0 < 0) ix0 += w;
        if (ix0 >= w) ix0 -= w;
        const int ix1 = (ix0 + 1 == w) ? 0 : ix0 + 1;
        int iy1 = iy0 + 1;
        iy0 = iy0 < 0 ? 0 : (iy0 > h - 1 ? h - 1 : iy0);
        iy1 = iy1 < 0 ? 0 : (iy1 > h - 1 ? h - 1 : iy1);
        const uint32_t r0 = (uint32_t)iy0 * tw, r1 = (uint32_t)iy1 * tw;
        t[0] = fetch(r0 + (uint32_t)ix0);
        t[1] = fetch(r0 + (uint32_t)ix1);
        t[2] = fetch(r1 + (uint32_t)ix0);
        t[3] = fetch(r1 + (uint32_t)ix1);
    }
};

// The padded copy of a tw x th equirect the device samples: (tw + 2) x (th + 2)
// texels, texel (x, y) of the texture at padded (x + 1, y + 1), column -1 =
// column tw - 1 and column tw = column 0 (U wraps), row -1 = row 0 and row th =
// row th - 1 (V clamps).  Every quad WrapClampQuad reads for U, V in [0, 1] is
// then the plain 2 x 2 block at padded index (iy0 + 1) (tw + 2) + ix0 + 1: no
// wrap or clamp logic, and on the device the four loads share one offset.
// rgba8: the row-major texture, 4 bytes per texel (any alignment).
GEO_HD void pad_sky(const uint8_t* rgba8, uint32_t tw, uint32_t th, uint32_t* dst) {
    const uint32_t pw = tw + 2u;
    for (uint32_t py = 0; py < th + 2u; ++py) {
        const uint32_t y = py == 0u ? 0u : (py > th ? th - 1u : py - 1u);
        const uint8_t* row = rgba8 + (size_t)y * tw * 4u;
        uint32_t* out = dst + (size_t)py * pw;
        __builtin_memcpy(out + 1, row, (size_t)tw * 4u);
        out[0] = out[tw];       // column tw - 1
        out[tw + 1u] = out[1];  // column 0
    }
}

// Level 0 of the padded sky again as row pairs (the device's bilinear reads
// this copy): padded texels (x, y) and (x, y + 1) side by side in 8 bytes,
// rows y = 0 .. th, so the quad at padded (x, y) is the 16 bytes at
// 2 ((y (tw + 2) + x)) texels: one 16-byte load, one 128-B line.  pad: the
// padded level (pad_sky), dst: 2 (th + 1) (tw + 2) texels.
GEO_HD void pair_sky_rows(const uint32_t* pad, uint32_t tw, uint32_t th, uint32_t* dst) {
    const uint32_t pw = tw + 2u;
    for (uint32_t y = 0; y <= th; ++y)
        for (uint32_t x = 0; x < pw; ++x) {
            dst[2u * ((size_t)y * pw + x)] = pad[(size_t)y * pw + x];
            dst[2u * ((size_t)y * pw + x) + 1u] = pad[(size_t)(y + 1u) * pw + x];
        }
}

// The G|A channels of a texel into the two 16-bit halves (bytes 1 and 3 to
// bytes 0 and 2): one v_perm_b32 on the device.
GEO_HD uint32_t ga_perm_(uint32_t t) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(0u, t, 0x0c030c01u);
#else
    return ga_(t);
#endif
}

// LOD-0 bilinear sample of an RGBA8 equirect (U wraps, V clamps) with 8-bit
// sub-texel weights, as texture units do, on packed channel pairs; quad(ix0,
// iy0, t) supplies the texel quad (WrapClampQuad, or a padded-copy reader).
// Texel coordinates in 1/256 texel units: n = floor(U tw 256 - 128) =
// floor(256 x) for x = U tw - 1/2, so ix0 = n >> 8 (arithmetic, -1 for
// x < 0) and the weight is n & 255 (one fma, one v_cvt_flr_i32_f32, two
// integer ops per axis).  tw256 = tw * 256 as a float (exact, tw < 2^24).
template <typename Quad>
GEO_HD uint32_t sample_sky_quad_f(const Quad& quad, float tw256, float th256, float U, float V) {
    const int32_t nx = floor_i32_(fmaf_(U, tw256, -128.0f));
    const int32_t ny = floor_i32_(fmaf_(V, th256, -128.0f));
    const uint32_t wx = (uint32_t)nx & 255u;
    const uint32_t wy = (uint32_t)ny & 255u;
    uint32_t t[4];
    quad(nx >> 8, ny >> 8, t);
    const uint32_t t00 = t[0], t10 = t[1], t01 = t[2], t11 = t[3];
    const uint32_t iwx = 256u - wx, iwy = 256u - wy;
    // horizontal (fields <= 255*256), truncated to 8 bits, then vertical, rounded;
    // (x >> 8) & 0x00FF00FF is ga_perm_'s byte move (one v_perm_b32)
    const uint32_t trb = ga_perm_(lerp2_(rb_(t00), rb_(t10), iwx, wx));
    const uint32_t brb = ga_perm_(lerp2_(rb_(t01), rb_(t11), iwx, wx));
    const uint32_t tga = ga_perm_(lerp2_(ga_perm_(t00), ga_perm_(t10), iwx, wx));
    const uint32_t bga = ga_perm_(lerp2_(ga_perm_(t01), ga_perm_(t11), iwx, wx));
    const uint32_t crb = ga_perm_(lerp2_(trb, brb, iwy, wy) + 0x00800080u);
    const uint32_t cga = ga_perm_(lerp2_(tga, bga, iwy, wy) + 0x00800080u);
    return crb | (cga << 8);
}
template <typename Quad>
GEO_HD uint32_t sample_sky_quad(const Quad& quad, uint32_t tw, uint32_t th, float U, float V) {
    return sample_sky_quad_f(quad, (float)tw * 256.0f, (float)th * 256.0f, U, V);
}

template <typename Fetch>
GEO_HD uint32_t sample_sky_raw(Fetch fetch, uint32_t tw, uint32_t th, float U, float V) {
    return sample_sky_quad(WrapClampQuad<Fetch>{fetch, tw, th}, tw, th, U, V);
}

// The reference's alpha blend (BlendState::ALPHA_BLENDING, pipeline.rs:49) in
// 8-bit fixed point of a sample s over the target pixel d:
//   rgb = round((s.rgb a + d.rgb (255 - a)) / 255),  alpha = round(a + d.a (255 - a) / 255).
GEO_HD uint32_t composite_(uint32_t s, uint32_t d) {
    const uint32_t a = s >> 24, ia = 255u - a;
    const uint32_t r = div255_((s & 0xFFu) * a + (d & 0xFFu) * ia);
    const uint32_t g = div255_(((s >> 8) & 0xFFu) * a + ((d >> 8) & 0xFFu) * ia);
    const uint32_t b = div255_(((s >> 16) & 0xFFu) * a + ((d >> 16) & 0xFFu) * ia);
    const uint32_t al = div255_(a * 255u + (d >> 24) * ia);
    return r | (g << 8) | (b << 16) | (al << 24);
}

// ---- GEO_FLAG_MIPS: the reference's mip-mapped sky (textureSample) ----
//
// The reference samples a 4-level mip chain (Texture::new_with_mipmaps(...,
// 4), basic_sphere_buffer.rs:31-36) with implicit derivatives (textureSample,
// shader.wgsl:101).  Its mip generator and sampler live in the absent
// wgpu_renderer submodule, so this specification fixes them:
//   * level l is max(1, w >> l) x max(1, h >> l); texel (x, y) of level l+1 =
//     the rounded mean (a + b + c + d + 2) >> 2 per channel of the 2 x 2 block
//     (2x..2x+1, 2y..2y+1) of level l, indices clamped to level l (box filter);
//   * the footprint from the UV differences across the pixel's 2 x 2 quad
//     (frame-aligned: x pairs 2i, 2i+1; y pairs 2j, 2j+1), each row's and
//     each column's own difference (WGSL leaves coarse or fine to the
//     implementation), U unwrapped as textureSample sees it (the seam takes the
//     coarsest level, as in the reference);
//   * rho2 = max((dU/dx W)^2 + (dV/dx H)^2, (dU/dy W)^2 + (dV/dy H)^2) in
//     level-0 texels, lambda = log2(rho2)/2 clamped to [0, 3] and taken in
//     1/256 steps (lod_q8); trilinear: bilinear samples of levels floor(lambda)
//     and floor(lambda) + 1 (U wraps, V clamps, as level 0), blended with the
//     8-bit weight frac(lambda) like the vertical bilinear lerp.
constexpr int kSkyMipLevels = 4;

GEO_HD uint32_t mip_dim(uint32_t d, int l) {
    const uint32_t r = d >> l;
    return r ? r : 1u;
}

// Level l + 1 of a w x h level (row-major RGBA8 texels as u32): the rounded
// 2 x 2 box mean, block indices clamped to the level.
GEO_HD void mip_down(const uint32_t* src, uint32_t w, uint32_t h, uint32_t* dst) {
    const uint32_t w2 = mip_dim(w, 1), h2 = mip_dim(h, 1);
    for (uint32_t y = 0; y < h2; ++y) {
        const uint32_t y0 = 2u * y < h ? 2u * y : h - 1u, y1 = 2u * y + 1u < h ? 2u * y + 1u : h - 1u;
        for (uint32_t x = 0; x < w2; ++x) {
            const uint32_t x0 = 2u * x < w ? 2u * x : w - 1u, x1 = 2u * x + 1u < w ? 2u * x + 1u : w - 1u;
            const uint32_t t00 = src[(size_t)y0 * w + x0], t10 = src[(size_t)y0 * w + x1];
            const uint32_t t01 = src[(size_t)y1 * w + x0], t11 = src[(size_t)y1 * w + x1];
            uint32_t o = 0;
            for (int c = 0; c < 4; ++c) {
                const uint32_t sh = 8u * (uint32_t)c;
                const uint32_t sum = ((t00 >> sh) & 255u) + ((t10 >> sh) & 255u) + ((t01 >> sh) & 255u) +
                                     ((t11 >> sh) & 255u) + 2u;
                o |= (sum >> 2) << sh;
            }
            dst[(size_t)y * w2 + x] = o;
        }
    }
}

// log2(1 + t), t in [0, 1): fixed polynomial, max error 1.9e-4 (far below
// the 1/512 resolution of lod_q8's lambda).
GEO_HD float log2_1p_(float t) {
    return t * fmaf_(t, fmaf_(t, fmaf_(t, -0x1.59455ap-4f, 0x1.4b69f0p-2f), -0x1.5b2e8ap-1f), 0x1.7044aep+0f);
}

// 256 lambda, lambda = log2(rho2)/2 clamped to [0, kSkyMipLevels - 1]:
// rho2 <= 1 (magnification) or NaN gives 0, rho2 >= 2^6 gives 768.
GEO_HD uint32_t lod_q8(float rho2) {
    if (!(rho2 > 1.0f)) return 0u;
    if (!(rho2 < 64.0f)) return 256u * (uint32_t)(kSkyMipLevels - 1);
    uint32_t b;
    __builtin_memcpy(&b, &rho2, 4);
    const float e = (float)((int32_t)(b >> 23) - 127);  // 0..5
    const uint32_t mb = (b & 0x007FFFFFu) | 0x3F800000u;
    float m;
    __builtin_memcpy(&m, &mb, 4);
    const float l2 = e + log2_1p_(m - 1.0f);  // log2(rho2) in [0, 6]
    const int32_t q = floor_i32_(l2 * 128.0f);
    const uint32_t qmax = 256u * (uint32_t)(kSkyMipLevels - 1);
    return q < 0 ? 0u : ((uint32_t)q < qmax ? (uint32_t)q : qmax);
}

// The squared footprint in level-0 texels from the quad differences.
GEO_HD float mip_rho2(float dux, float dvx, float duy, float dvy, float w, float h) {
    const float ax = dux * w, bx = dvx * h, ay = duy * w, by = dvy * h;
    const float rx = fmaf_(bx, bx, ax * ax), ry = fmaf_(by, by, ay * ay);
    return rx > ry ? rx : ry;
}

// The trilinear blend of two level samples with the 8-bit weight f (packed
// channel pairs, as the vertical bilinear lerp).
GEO_HD uint32_t mip_blend(uint32_t s0, uint32_t s1, uint32_t f) {
    const uint32_t i = 256u - f;
    const uint32_t rb = ga_perm_(lerp2_(rb_(s0), rb_(s1), i, f) + 0x00800080u);
    const uint32_t ga = ga_perm_(lerp2_(ga_perm_(s0), ga_perm_(s1), i, f) + 0x00800080u);
    return rb | (ga << 8);
}

// The blend of a sample over the cleared target (sample_sky_qf's epilogue).
GEO_HD uint32_t over_clear(uint32_t s, bool opaque) {
    if (opaque) return s | 0xFF000000u;
    const uint32_t a = s >> 24;
    return blend255_(s & 0xFFu, a) | (blend255_((s >> 8) & 0xFFu, a) << 8) | (blend255_((s >> 16) & 0xFFu, a) << 16) |
           0xFF000000u;
}

// A sample over the cleared target (0,0,0,1) (renderer.rs:233-238): rgb*a/255,
// alpha 1.  `opaque` (every texel alpha 255, checked on upload) skips the
// blend, which is exact there.
template <typename Quad>
GEO_HD uint32_t sample_sky_qf(const Quad& quad, float tw256, float th256, bool opaque, float U, float V) {
    return over_clear(sample_sky_quad_f(quad, tw256, th256, U, V), opaque);
}
template <typename Quad>
GEO_HD uint32_t sample_sky_q(const Quad& quad, uint32_t tw, uint32_t th, bool opaque, float U, float V) {
    return sample_sky_qf(quad, (float)tw * 256.0f, (float)th * 256.0f, opaque, U, V);
}
template <typename Fetch>
GEO_HD uint32_t sample_sky(Fetch fetch, uint32_t tw, uint32_t th, bool opaque, float U, float V) {
    return sample_sky_q(WrapClampQuad<Fetch>{fetch, tw, th}, tw, th, opaque, U, V);
}

constexpr uint32_t kBlackRGBA = 0xFF000000u;  // clear colour (0,0,0,1), renderer.rs:233-238

}  // namespace geo
