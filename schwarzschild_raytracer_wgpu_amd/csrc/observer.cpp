// observer.cpp — host side of the camera/uniform API (f64), C++ restatement of
//   Observer                    SR/simulation/observer.rs:42-297
//   polar transformations       SR/simulation/polar_transformations.rs:7-51
//   Orbit (observer orbits)     SR/simulation/orbit.rs:12-237
// producing the 208-byte TransformationPipeline (observer.rs:21-28) that
// geo_render_rows consumes.  The glam 0.25 operations used by the reference
// (column-major DMat3, mul_vec3 as x*vx + y*vy + z*vz, normalize = v * (1/|v|),
// from_rotation_x/z) are restated with the same evaluation order.
#include <cmath>
#include <cstring>
#include <new>

#include "../../include/geo/geo.h"

namespace {

struct V3 {
    double x, y, z;
};
inline V3 v3(double x, double y, double z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 scale(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline double length(V3 a) { return std::sqrt(dot(a, a)); }
inline V3 normalize(V3 a) { return scale(a, 1.0 / length(a)); }
inline V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
inline V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
// glam DVec3::angle_between: acos_approx(dot / sqrt(|a|^2 |b|^2)), clamped.
inline double angle_between(V3 a, V3 b) {
    double c = dot(a, b) / std::sqrt(dot(a, a) * dot(b, b));
    c = c < -1.0 ? -1.0 : (c > 1.0 ? 1.0 : c);
    return std::acos(c);
}

// Column-major 3x3 (glam DMat3): c[0] = x_axis, c[1] = y_axis, c[2] = z_axis.
struct M3 {
    V3 c[3];
};
inline M3 from_cols(V3 x, V3 y, V3 z) { return M3{{x, y, z}}; }
inline M3 identity() { return from_cols(v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1)); }
inline V3 mul(const M3& m, V3 v) {
    V3 r = scale(m.c[0], v.x);
    r = add(r, scale(m.c[1], v.y));
    r = add(r, scale(m.c[2], v.z));
    return r;
}
inline M3 mul(const M3& a, const M3& b) { return from_cols(mul(a, b.c[0]), mul(a, b.c[1]), mul(a, b.c[2])); }
inline M3 mul(const M3& a, double s) { return from_cols(scale(a.c[0], s), scale(a.c[1], s), scale(a.c[2], s)); }
inline M3 transpose(const M3& m) {
    return from_cols(v3(m.c[0].x, m.c[1].x, m.c[2].x), v3(m.c[0].y, m.c[1].y, m.c[2].y),
                     v3(m.c[0].z, m.c[1].z, m.c[2].z));
}
inline M3 from_diagonal(V3 d) { return from_cols(v3(d.x, 0, 0), v3(0, d.y, 0), v3(0, 0, d.z)); }
inline M3 from_rotation_x(double a) {
    const double s = std::sin(a), c = std::cos(a);
    return from_cols(v3(1, 0, 0), v3(0, c, s), v3(0, -s, c));
}
inline M3 from_rotation_z(double a) {
    const double s = std::sin(a), c = std::cos(a);
    return from_cols(v3(c, s, 0), v3(-s, c, 0), v3(0, 0, 1));
}

// polar_transformations.rs:7-51
V3 carthesic_to_polar(V3 v) {
    V3 p = v3(0, 0, 0);
    p.x = length(v);
    if (p.x != 0.) {
        p.y = std::atan2(v.y, v.x);
        p.z = std::asin(v.z / p.x);
    }
    return p;
}
V3 polar_to_carthesic(V3 p) {
    return v3(p.x * std::cos(p.y) * std::cos(p.z), p.x * std::sin(p.y) * std::cos(p.z), p.x * std::sin(p.z));
}
V3 polar2_to_carthesic(double phi, double theta) {
    return v3(std::cos(phi) * std::cos(theta), std::sin(phi) * std::cos(theta), std::sin(theta));
}
V3 trans_polar_vec(V3 polar, const M3& t) { return carthesic_to_polar(mul(t, polar_to_carthesic(polar))); }
M3 look_to_vec_mat(V3 look_to) {
    const V3 z = normalize(look_to);
    V3 xp = carthesic_to_polar(z);
    xp.z -= M_PI_2;
    const V3 x = polar_to_carthesic(xp);
    const V3 y = cross(z, x);
    return from_cols(x, y, z);
}

inline double signum(double x) { return std::signbit(x) ? -1.0 : 1.0; }  // Rust f64::signum (non-NaN)

// orbit.rs:12-237
struct Orbit {
    double schwarz_r, start_phi, tilt_angle, orbit_angle;
    M3 plane_tilt_mat;
    double energy, rotation, r, u, u_bar, last_r;
    bool has_hit_singularity;

    static bool make(double schwarz_r, V3 position, V3 desired_direction, double rotation, Orbit* o) {
        const double r = length(position);
        if (r <= schwarz_r) return false;
        if (rotation < schwarz_r * 1e-5) rotation = 0.;
        o->schwarz_r = schwarz_r;
        o->u = 1. / r;
        o->energy = std::sqrt((1. - schwarz_r / r) * (1. + rotation * rotation / (r * r)));
        const V3 plane_normal = cross(position, desired_direction);
        double tilt_angle = angle_between(plane_normal, v3(0, 0, 1));
        const double pos_phi = std::atan2(position.y, position.x);
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
            o->start_phi = std::atan2(horizontal_cut.y, horizontal_cut.x);
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

    void do_step(double time_step) {
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
        double frag = 1. + std::floor(delta_phi * 100.);
        unsigned step_fragments = frag > 1000. ? 1000u : (unsigned)frag;
        for (unsigned i = 0; i < step_fragments; ++i) {
            do_angle_step(delta_phi / (double)step_fragments);
            if (has_hit_singularity) return;
        }
    }

    void do_angle_step(double delta_phi) {
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
        if (std::isinf(u) || u > 100.) {
            has_hit_singularity = true;
        } else {
            r = 1. / u;
            orbit_angle += delta_phi;
        }
    }

    double h_r() const { return 1. - schwarz_r / r; }

    V3 get_position() const {
        V3 p = trans_polar_vec(v3(r, orbit_angle, 0.), plane_tilt_mat);
        p.y += start_phi;
        return polar_to_carthesic(p);
    }

    V3 get_velocity() const {
        const double falling = rotation == 0. ? -signum(r - last_r) : signum(u_bar);
        return v3(energy / h_r(),
                  -falling * std::sqrt(energy * energy - h_r() * (1. + rotation * rotation / (r * r))),
                  rotation / (r * r));
    }

    double current_tilt_angle() const {
        const V3 p = trans_polar_vec(v3(r, orbit_angle, 0.), plane_tilt_mat);
        return tilt_angle * std::cos(p.y);
    }

    bool is_singular() const { return has_hit_singularity; }
    bool is_central_fall() const { return rotation == 0.; }
};

constexpr double kSafeFracPi2 = M_PI_2 - 0.0001;  // observer.rs:9

}  // namespace

struct geo_observer {
    double schwarz_r;
    V3 position;
    double cam_phi, cam_theta;
    bool has_orbit;
    Orbit orbit;
    int state;
    double time_speedup, energy, mouse_sensitivity;
    double fov_scaling[4];
    M3 standard_to_movement, movement_to_central, central_to_uv;
    double psi;

    double h_r() const { return 1. - schwarz_r / length(position); }

    V3 unmoving_velocity() const {
        V3 v = v3(0, 0, 0);
        if (length(position) > schwarz_r) {
            v.x = 1. / std::sqrt(h_r());
            v.y = 0.;
        } else {
            v.x = 0.;
            v.y = -std::sqrt(-h_r());
        }
        return v;
    }
    V3 frozen_fall_velocity() const {
        if (energy * energy < h_r()) return unmoving_velocity();
        return v3(energy / h_r(), std::sqrt(energy * energy - h_r()), 0.);
    }
    V3 velocity() const {
        switch (state) {
            case GEO_OBSERVER_UNMOVING: return unmoving_velocity();
            case GEO_OBSERVER_FROZEN_FALL: return frozen_fall_velocity();
            default: return has_orbit ? orbit.get_velocity() : unmoving_velocity();
        }
    }
    bool is_singular() const {
        if (std::fabs(length(position) - schwarz_r) < 1e-10) return true;
        if (state == GEO_OBSERVER_ORBITING) return has_orbit ? orbit.is_singular() : true;
        return length(position) < 1e-10;
    }
};

extern "C" {

int geo_observer_create(double schwarz_r, double fov, double width, double height, geo_observer** out) {
    if (!out || !(height > 0.) || !(width > 0.)) return GEO_EINVAL;
    geo_observer* o = new (std::nothrow) geo_observer();
    if (!o) return GEO_ENOMEM;
    const double ratio = width / height;
    o->schwarz_r = schwarz_r;
    o->position = v3(25., 0., 1.);
    o->cam_phi = M_PI;
    o->cam_theta = 0.;
    o->has_orbit = false;
    o->state = GEO_OBSERVER_FROZEN_FALL;
    o->time_speedup = 1.;
    o->energy = 1.;
    o->mouse_sensitivity = fov / height;
    o->fov_scaling[0] = std::tan(fov / 2.);
    o->fov_scaling[1] = std::tan(fov / 2.) * ratio;
    o->fov_scaling[2] = 1.;
    o->fov_scaling[3] = 1.;
    o->standard_to_movement = identity();
    o->movement_to_central = identity();
    o->central_to_uv = identity();
    o->psi = 1.;
    *out = o;
    return GEO_OK;
}

void geo_observer_destroy(geo_observer* o) { delete o; }

int geo_observer_set_position(geo_observer* o, double x, double y, double z) {
    if (!o) return GEO_EINVAL;
    o->position = v3(x, y, z);
    return GEO_OK;
}

int geo_observer_get_position(const geo_observer* o, double* xyz) {
    if (!o || !xyz) return GEO_EINVAL;
    xyz[0] = o->position.x;
    xyz[1] = o->position.y;
    xyz[2] = o->position.z;
    return GEO_OK;
}

int geo_observer_set_camera(geo_observer* o, double phi, double theta) {
    if (!o) return GEO_EINVAL;
    o->cam_phi = phi;
    o->cam_theta = theta;
    return GEO_OK;
}

int geo_observer_set_energy(geo_observer* o, double energy) {
    if (!o) return GEO_EINVAL;
    o->energy = energy;
    return GEO_OK;
}

int geo_observer_set_state(geo_observer* o, int state) {
    if (!o || (state != GEO_OBSERVER_UNMOVING && state != GEO_OBSERVER_FROZEN_FALL)) return GEO_EINVAL;
    o->state = state;
    return GEO_OK;
}

int geo_observer_start_orbit(geo_observer* o, double rotation) {
    if (!o) return GEO_EINVAL;
    const V3 direction = v3(-o->position.y, o->position.x, 0.);
    Orbit orb;
    if (!Orbit::make(o->schwarz_r, o->position, direction, rotation, &orb)) {
        o->has_orbit = false;  // Orbit::new returned None; state unchanged (observer.rs:164-168)
        return GEO_ESTATE;
    }
    o->orbit = orb;
    o->has_orbit = true;
    o->state = GEO_OBSERVER_ORBITING;
    return GEO_OK;
}

int geo_observer_get_state(const geo_observer* o) { return o ? o->state : GEO_EINVAL; }

double geo_observer_radial_position(const geo_observer* o) { return o ? length(o->position) : NAN; }

int geo_observer_update_position(geo_observer* o, double fwd, double left, double up, double dt) {
    if (!o) return GEO_EINVAL;
    if (o->state == GEO_OBSERVER_ORBITING) {
        if (!o->has_orbit) return GEO_ESTATE;
        o->orbit.do_step(o->time_speedup * dt);
        o->position = o->orbit.get_position();
    } else {
        const double movement_step = 0.051;
        const V3 d = mul(mul(from_rotation_z(o->cam_phi), movement_step), v3(fwd, left, up));
        o->position = add(o->position, d);
    }
    return GEO_OK;
}

int geo_observer_move_camera(geo_observer* o, double dx, double dy) {
    if (!o) return GEO_EINVAL;
    o->cam_phi += dx * o->mouse_sensitivity;
    o->cam_theta += dy * o->mouse_sensitivity;
    if (o->cam_theta < -kSafeFracPi2)
        o->cam_theta = -kSafeFracPi2;
    else if (o->cam_theta > kSafeFracPi2)
        o->cam_theta = kSafeFracPi2;
    return GEO_OK;
}

int geo_observer_update_screen_format(geo_observer* o, double width, double height) {
    if (!o || !(height > 0.)) return GEO_EINVAL;
    const double ratio = width / height;
    const double t = o->fov_scaling[0];
    o->fov_scaling[0] = t;
    o->fov_scaling[1] = t * ratio;
    o->fov_scaling[2] = 1.;
    o->fov_scaling[3] = 1.;
    return GEO_OK;
}

int geo_observer_is_singular(const geo_observer* o) { return o ? (o->is_singular() ? 1 : 0) : GEO_EINVAL; }

// observer.rs:197-262
int geo_observer_calc_transformation_pipeline(geo_observer* o, geo_frame* out) {
    if (!o || !out) return GEO_EINVAL;
    const double r = length(o->position);
    if (!o->is_singular()) {
        const V3 vel = o->velocity();
        if (r > o->schwarz_r)
            o->psi = vel.x * vel.x * o->h_r();
        else
            o->psi = -vel.y * vel.y / o->h_r();
        if (o->psi - 1. < 1e-10) o->psi = 1.;
        const M3 standard_to_central = transpose(look_to_vec_mat(neg(o->position)));
        if (o->state == GEO_OBSERVER_ORBITING && o->has_orbit && !o->orbit.is_central_fall()) {
            const double tilt_angle = o->orbit.current_tilt_angle();
            const double plane_angle1 =
                std::acos(-vel.x * vel.y * signum(r - o->schwarz_r) /
                          std::sqrt((1. + r * r * vel.z * vel.z) * o->psi * (o->psi - 1.)));
            double plane_angle2;
            if (r > o->schwarz_r)
                plane_angle2 = std::acos(-vel.y / std::sqrt(o->h_r() * (o->psi - 1.)));
            else
                plane_angle2 = std::acos(-vel.x * std::sqrt(-o->h_r() / (o->psi - 1.)));
            const M3 orbit_plane_tilt = from_rotation_z(-tilt_angle);
            const M3 tilted_center_to_movement1 = from_rotation_x(-plane_angle1);
            const M3 movement2_to_tilted_center = from_rotation_x(plane_angle2);
            o->standard_to_movement = mul(mul(tilted_center_to_movement1, orbit_plane_tilt), standard_to_central);
            o->movement_to_central = mul(transpose(orbit_plane_tilt), movement2_to_tilted_center);
        } else {
            o->standard_to_movement = standard_to_central;
            o->movement_to_central = identity();
        }
        o->central_to_uv = mul(look_to_vec_mat(o->position), from_diagonal(v3(1., -1., 1.)));
    }
    const M3 camera_to_standard = look_to_vec_mat(polar2_to_carthesic(o->cam_phi, o->cam_theta));
    const M3 cam = mul(o->standard_to_movement, camera_to_standard);
    // DMat4::from_mat3 + w_axis = fov_scaling, as_mat4().to_cols_array()
    float* d = out->display_to_movement;
    for (int c = 0; c < 3; ++c) {
        d[c * 4 + 0] = (float)cam.c[c].x;
        d[c * 4 + 1] = (float)cam.c[c].y;
        d[c * 4 + 2] = (float)cam.c[c].z;
        d[c * 4 + 3] = 0.f;
    }
    for (int i = 0; i < 4; ++i) d[12 + i] = (float)o->fov_scaling[i];
    // Mat4::from_mat3(DMat3::as_mat3())
    const M3* src[2] = {&o->movement_to_central, &o->central_to_uv};
    float* dst[2] = {out->movement_to_central, out->central_to_uv};
    for (int k = 0; k < 2; ++k) {
        for (int c = 0; c < 3; ++c) {
            dst[k][c * 4 + 0] = (float)src[k]->c[c].x;
            dst[k][c * 4 + 1] = (float)src[k]->c[c].y;
            dst[k][c * 4 + 2] = (float)src[k]->c[c].z;
            dst[k][c * 4 + 3] = 0.f;
        }
        dst[k][12] = 0.f;
        dst[k][13] = 0.f;
        dst[k][14] = 0.f;
        dst[k][15] = 1.f;
    }
    out->psi_factor_and_position[0] = (float)std::sqrt((o->psi - 1.) / o->psi);
    out->psi_factor_and_position[1] = (float)o->position.x;
    out->psi_factor_and_position[2] = (float)o->position.y;
    out->psi_factor_and_position[3] = (float)o->position.z;
    return GEO_OK;
}

}  // extern "C"
