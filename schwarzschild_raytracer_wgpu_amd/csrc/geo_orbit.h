// geo_orbit.h — f64 vector/matrix helpers, polar transformations and the
// massive-particle Orbit, shared by the host observer (observer.cpp) and the
// accretion-disk point kernels (geo_points.hip).  Restates, in the reference's
// evaluation order:
//   polar transformations   SR/simulation/polar_transformations.rs:7-51
//   Orbit                   SR/simulation/orbit.rs:12-237
// and the glam 0.25 operations they use (column-major DMat3, mul_vec3 as
// x*vx + y*vy + z*vz, normalize = v * (1/|v|), from_rotation_x/z,
// DVec3::angle_between = acos(clamp(dot / sqrt(|a|^2 |b|^2)))).
// f64 libm calls: glibc on the host, the device math library on gfx950 (the
// two may differ by an ulp; tests compare orbits with a tolerance).
#pragma once

#include <math.h>

#include "geo_math.h"

namespace geo64 {

struct V3 {
    double x, y, z;
};
GEO_HD V3 v3(double x, double y, double z) { return V3{x, y, z}; }
GEO_HD V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
GEO_HD V3 scale(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
GEO_HD double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
GEO_HD double length(V3 a) { return ::sqrt(dot(a, a)); }
GEO_HD V3 normalize(V3 a) { return scale(a, 1.0 / length(a)); }
GEO_HD V3 cross(V3 a, V3 b) { return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
GEO_HD V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
GEO_HD double angle_between(V3 a, V3 b) {
    double c = dot(a, b) / ::sqrt(dot(a, a) * dot(b, b));
    c = c < -1.0 ? -1.0 : (c > 1.0 ? 1.0 : c);
    return ::acos(c);
}
GEO_HD double signum(double x) { return __builtin_signbit(x) ? -1.0 : 1.0; }  // Rust f64::signum (non-NaN)

// Column-major 3x3 (glam DMat3): c[0] = x_axis, c[1] = y_axis, c[2] = z_axis.
struct M3 {
    V3 c[3];
};
GEO_HD M3 from_cols(V3 x, V3 y, V3 z) { return M3{{x, y, z}}; }
GEO_HD M3 identity() { return from_cols(v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1)); }
GEO_HD V3 mul(const M3& m, V3 v) {
    V3 r = scale(m.c[0], v.x);
    r = add(r, scale(m.c[1], v.y));
    r = add(r, scale(m.c[2], v.z));
    return r;
}
GEO_HD M3 mul(const M3& a, const M3& b) { return from_cols(mul(a, b.c[0]), mul(a, b.c[1]), mul(a, b.c[2])); }
GEO_HD M3 mul(const M3& a, double s) { return from_cols(scale(a.c[0], s), scale(a.c[1], s), scale(a.c[2], s)); }
GEO_HD M3 transpose(const M3& m) {
    return from_cols(v3(m.c[0].x, m.c[1].x, m.c[2].x), v3(m.c[0].y, m.c[1].y, m.c[2].y),
                     v3(m.c[0].z, m.c[1].z, m.c[2].z));
}
GEO_HD M3 from_diagonal(V3 d) { return from_cols(v3(d.x, 0, 0), v3(0, d.y, 0), v3(0, 0, d.z)); }
GEO_HD M3 from_rotation_x(double a) {
    const double s = ::sin(a), c = ::cos(a);
    return from_cols(v3(1, 0, 0), v3(0, c, s), v3(0, -s, c));
}
GEO_HD M3 from_rotation_z(double a) {
    const double s = ::sin(a), c = ::cos(a);
    return from_cols(v3(c, s, 0), v3(-s, c, 0), v3(0, 0, 1));
}

// polar_transformations.rs:7-51
GEO_HD V3 carthesic_to_polar(V3 v) {
    V3 p = v3(0, 0, 0);
    p.x = length(v);
    if (p.x != 0.) {
        p.y = ::atan2(v.y, v.x);
        p.z = ::asin(v.z / p.x);
    }
    return p;
}
GEO_HD V3 polar_to_carthesic(V3 p) {
    return v3(p.x * ::cos(p.y) * ::cos(p.z), p.x * ::sin(p.y) * ::cos(p.z), p.x * ::sin(p.z));
}
GEO_HD V3 polar2_to_carthesic(double phi, double theta) {
    return v3(::cos(phi) * ::cos(theta), ::sin(phi) * ::cos(theta), ::sin(theta));
}
GEO_HD V3 trans_polar_vec(V3 polar, const M3& t) { return carthesic_to_polar(mul(t, polar_to_carthesic(polar))); }
GEO_HD M3 look_to_vec_mat(V3 look_to) {
    const V3 z = normalize(look_to);
    V3 xp = carthesic_to_polar(z);
    xp.z -= M_PI_2;
    const V3 x = polar_to_carthesic(xp);
    const V3 y = cross(z, x);
    return from_cols(x, y, z);
}

// orbit.rs:12-237
struct Orbit {
    double schwarz_r, start_phi, tilt_angle, orbit_angle;
    M3 plane_tilt_mat;
    double energy, rotation, r, u, u_bar, last_r;
    bool has_hit_singularity;

    // Orbit::new (:29-82); false = None (start inside the horizon)
    GEO_HDM static bool make(double schwarz_r, V3 position, V3 desired_direction, double rotation, Orbit* o) {
        const double r = length(position);
        if (r <= schwarz_r) return false;
        if (rotation < schwarz_r * 1e-5) rotation = 0.;
        o->schwarz_r = schwarz_r;
        o->u = 1. / r;
        o->energy = ::sqrt((1. - schwarz_r / r) * (1. + rotation * rotation / (r * r)));
        const V3 plane_normal = cross(position, desired_direction);
        double tilt_angle = angle_between(plane_normal, v3(0, 0, 1));
        const double pos_phi = ::atan2(position.y, position.x);
        if (tilt_angle < 1e-10 || M_PI - tilt_angle < 1e-10) {
            tilt_angle = 0.;
            o->start_phi = 0.;
            o->orbit_angle = pos_phi;
            o->plane_tilt_mat = identity();
        } else {
            const V3 horizontal_cut = cross(v3(0, 0, 1), plane_normal);
            double orbit_angle = angle_between(horizontal_cut, position);
            if (position.z < 0.) orbit_angle = 2. * M_PI - orbit_angle;
            o->orbit_angle = orbit_angle;
            o->start_phi = ::atan2(horizontal_cut.y, horizontal_cut.x);
            o->plane_tilt_mat = from_rotation_x(tilt_angle);
        }
        o->tilt_angle = tilt_angle;
        o->rotation = rotation;
        o->r = r;
        o->u_bar = 0.;
        o->last_r = r;
        o->has_hit_singularity = false;
        return true;
    }

    // :84-135
    GEO_HDM void do_step(double time_step) {
        if (has_hit_singularity) return;
        if (rotation == 0.) {
            const double next_r = 2. * r - last_r - time_step * time_step * schwarz_r / (2. * r * r);
            if (next_r < 0.) {
                has_hit_singularity = true;
            } else {
                last_r = r;
                r = next_r;
            }
            return;
        }
        const double l = rotation;
        double delta_phi = time_step * l * u * u / 2.;
        double next_u = u + delta_phi * u_bar;
        delta_phi = time_step * l / 4. * (u * u + next_u * next_u);
        next_u = u + delta_phi * u_bar;
        delta_phi = time_step * l / 4. * (u * u + next_u * next_u);
        next_u = u + delta_phi * u_bar;
        delta_phi = time_step * l / 4. * (u * u + next_u * next_u);
        if (next_u > 50.) {
            has_hit_singularity = true;
            return;
        }
        const double frag = 1. + ::floor(delta_phi * 100.);
        const unsigned step_fragments = frag > 1000. ? 1000u : (unsigned)frag;
        for (unsigned i = 0; i < step_fragments; ++i) {
            do_angle_step(delta_phi / (double)step_fragments);
            if (has_hit_singularity) return;
        }
    }

    // :137-167
    GEO_HDM void do_angle_step(double delta_phi) {
        const double l = rotation, uu = u, ub = u_bar, rs = schwarz_r;
        const double a_u = uu + delta_phi / 2. * ub;
        const double a_u_bar = ub + delta_phi / 2. * (rs * (1. / (2. * l * l) + 3. / 2. * uu * uu) - uu);
        const double b_u = uu + delta_phi / 2. * a_u_bar;
        const double b_u_bar = ub + delta_phi / 2. * (rs * (1. / (2. * l * l) + 3. / 2. * a_u * a_u) - a_u);
        const double c_u = uu + delta_phi * b_u_bar;
        const double c_u_bar = ub + delta_phi * (rs * (1. / (2. * l * l) + 3. / 2. * b_u * b_u) - b_u);
        const double next_u = uu + delta_phi * (ub / 6. + a_u_bar / 3. + b_u_bar / 3. + c_u_bar / 6.);
        const double next_u_bar =
            ub + delta_phi * (rs / (2. * l * l) +
                              3. * rs / 2. * (uu * uu / 6. + a_u * a_u / 3. + b_u * b_u / 3. + c_u * c_u / 6.) -
                              (uu + 2. * a_u + 2. * b_u + c_u) / 6.);
        u = next_u;
        u_bar = next_u_bar;
        if (__builtin_isinf(u) || u > 100.) {
            has_hit_singularity = true;
        } else {
            r = 1. / u;
            orbit_angle += delta_phi;
        }
    }

    GEO_HDM double h_r() const { return 1. - schwarz_r / r; }

    // :174-182
    GEO_HDM V3 get_position() const {
        V3 p = trans_polar_vec(v3(r, orbit_angle, 0.), plane_tilt_mat);
        p.y += start_phi;
        return polar_to_carthesic(p);
    }

    // :185-198
    GEO_HDM V3 get_velocity() const {
        const double falling = rotation == 0. ? -signum(r - last_r) : signum(u_bar);
        return v3(energy / h_r(), -falling * ::sqrt(energy * energy - h_r() * (1. + rotation * rotation / (r * r))),
                  rotation / (r * r));
    }

    // :201-208
    GEO_HDM double current_tilt_angle() const {
        const V3 p = trans_polar_vec(v3(r, orbit_angle, 0.), plane_tilt_mat);
        return tilt_angle * ::cos(p.y);
    }

    GEO_HDM bool is_singular() const { return has_hit_singularity; }
    GEO_HDM bool is_central_fall() const { return rotation == 0.; }
};

}  // namespace geo64
