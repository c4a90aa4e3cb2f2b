// observer.cpp — host side of the camera/uniform API (f64), C++ restatement of
//   Observer                    SR/simulation/observer.rs:42-297
// producing the 208-byte TransformationPipeline (observer.rs:21-28) that
// geo_render_rows consumes.  Polar transformations, the glam helpers and the
// Orbit (orbit.rs) live in geo_orbit.h, shared with the point-cloud kernels.
#include <cmath>
#include <cstring>
#include <new>

#include "../../include/geo/geo.h"
#include "geo_orbit.h"

namespace {

using namespace geo64;

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
