// sr.hpp — the reference's host-side types, in C++17, over libgeo's C-ABI.
//
// The reference's host is Rust (schwarzschild_raytracer/src, `SR/` below);
// this image has no Rust toolchain, so the host side above the C-ABI is C++,
// mirroring the reference's types, names, argument meaning and error
// behaviour one for one:
//
//   sr::Observer                      Observer            SR/simulation/observer.rs:42-296
//   sr::TransformationPipeline        TransformationPipeline  observer.rs:21-28 (== geo_frame, 208 B)
//   sr::SphereRayTracer               SphereRayTracer     SR/simulation/sphere_ray_tracer.rs:12-56
//   sr::RayConnector                  RayConnector        SR/simulation/ray_connector.rs:6-157
//   sr::SchwarzschildSphereShaderDraw the per-sphere plugin trait
//                                                         SR/schwarzschild_sphere_shader/schwarzschild_sphere_shader_draw.rs:3-6
//   sr::BasicSphereBuffer             BasicSphereBuffer   .../sphere_buffer/basic_sphere_buffer.rs:12-100
//   sr::PointCloud                    PointCloud (+ its two point meshes)
//                                                         SR/schwarzschild_point_shader/point_cloud.rs:7-156
//   sr::RenderPass                    the wgpu::RenderPass the draws record into
//   sr::Renderer                      Renderer::{render, update, resize, get_*}
//                                                         SR/renderer/renderer.rs:21-296
//
// Errors: the reference unwraps (a failure panics); here every failing
// libgeo call throws sr::Error carrying the geo_status.  GPU work is
// asynchronous on the pass's HIP stream, as wgpu queues are; calls that
// return host values (solve_ray_fan, RayConnector::update_ray, read_frame)
// synchronise.  Only HIP's C runtime API is used, for device memory.
//
// Build (any C++17 compiler):
//   g++ -std=c++17 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include app.cpp
//       -L schwarzschild_raytracer_wgpu_amd -lgeo -L /opt/rocm/lib -lamdhip64
#pragma once

#include <hip/hip_runtime_api.h>

#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "geo.h"

namespace sr {

constexpr double kPi = 3.14159265358979323846;

struct Error : std::runtime_error {
    int status;
    Error(const std::string& what, int st) : std::runtime_error(what + ": " + geo_status_str(st)), status(st) {}
};

inline void check(int st, const char* what) {
    if (st != GEO_OK) throw Error(what, st);
}
inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Error(std::string(what) + " (" + hipGetErrorString(e) + ")", GEO_EHIP);
}

struct Vec3 {  // glam::Vec3
    float x, y, z;
};
struct DVec3 {  // glam::DVec3
    double x, y, z;
};

using TransformationPipeline = geo_frame;

// One libgeo context (a device plus the texture / ray fan it holds): the
// per-sphere bind groups of the reference.
class Context {
   public:
    explicit Context(int device = 0) : device_(device) {
        geo_ctx* c = nullptr;
        check(geo_ctx_create(device, &c), "geo_ctx_create");
        h_.reset(c);
    }
    geo_ctx* get() const { return h_.get(); }
    int device() const { return device_; }

   private:
    struct Del {
        void operator()(geo_ctx* c) const { geo_ctx_destroy(c); }
    };
    std::unique_ptr<geo_ctx, Del> h_;
    int device_;
};

// A device allocation of n elements of T (hipMalloc / hipFree).
template <typename T>
class DeviceBuffer {
   public:
    DeviceBuffer() = default;
    explicit DeviceBuffer(size_t n) : n_(n) {
        void* p = nullptr;
        if (n) hip_check(hipMalloc(&p, n * sizeof(T)), "hipMalloc");
        p_.reset(static_cast<T*>(p));
    }
    T* data() const { return p_.get(); }
    size_t size() const { return n_; }

   private:
    struct Del {
        void operator()(T* p) const { (void)hipFree(p); }
    };
    std::unique_ptr<T, Del> p_;
    size_t n_ = 0;
};

// ---- Observer (observer.rs) --------------------------------------------
class Observer {
   public:
    // Observer::new (observer.rs:68-87)
    Observer(double schwarz_r, double fov, double width, double height) : schwarz_r_(schwarz_r) {
        geo_observer* o = nullptr;
        check(geo_observer_create(schwarz_r, fov, width, height, &o), "geo_observer_create");
        h_.reset(o);
    }
    double get_radial_position() const { return geo_observer_radial_position(h_.get()); }
    DVec3 get_position() const {
        double p[3];
        check(geo_observer_get_position(h_.get(), p), "geo_observer_get_position");
        return {p[0], p[1], p[2]};
    }
    // desired_direction = (forward, left, up) (observer.rs:103-125)
    void update_position(DVec3 desired_direction, double dt) {
        check(geo_observer_update_position(h_.get(), desired_direction.x, desired_direction.y, desired_direction.z,
                                           dt),
              "geo_observer_update_position");
    }
    // start_orbit (observer.rs:162-171): the reference only starts an orbit when
    // Orbit::new succeeds; returns whether it did
    bool start_orbit(double rotation) {
        const int st = geo_observer_start_orbit(h_.get(), rotation);
        if (st == GEO_ESTATE) return false;
        check(st, "geo_observer_start_orbit");
        return true;
    }
    void start_frozen_fall() { check(geo_observer_set_state(h_.get(), GEO_OBSERVER_FROZEN_FALL), "start_frozen_fall"); }
    void start_unmoving() { check(geo_observer_set_state(h_.get(), GEO_OBSERVER_UNMOVING), "start_unmoving"); }
    bool is_singular() const { return geo_observer_is_singular(h_.get()) != 0; }
    TransformationPipeline calc_transformation_pipeline() {
        TransformationPipeline t;
        check(geo_observer_calc_transformation_pipeline(h_.get(), &t), "calc_transformation_pipeline");
        return t;
    }
    void update_screen_format(double width, double height) {
        check(geo_observer_update_screen_format(h_.get(), width, height), "update_screen_format");
    }
    void move_camera(double horizontal_pixels, double vertical_pixels) {
        check(geo_observer_move_camera(h_.get(), horizontal_pixels, vertical_pixels), "move_camera");
    }
    double get_schwarz_r() const { return schwarz_r_; }
    // reset_to_start (observer.rs:292-296)
    void reset_to_start() {
        set_position({25.0, 0.0, 0.0});
        set_camera(kPi, 0.0);
        start_frozen_fall();
    }
    // not in the reference's public API (its fields are private): explicit
    // pose for tests and benchmarks
    void set_position(DVec3 p) { check(geo_observer_set_position(h_.get(), p.x, p.y, p.z), "set_position"); }
    void set_camera(double phi, double theta) { check(geo_observer_set_camera(h_.get(), phi, theta), "set_camera"); }
    void set_energy(double e) { check(geo_observer_set_energy(h_.get(), e), "set_energy"); }

   private:
    struct Del {
        void operator()(geo_observer* o) const { geo_observer_destroy(o); }
    };
    std::unique_ptr<geo_observer, Del> h_;
    double schwarz_r_;
};

// ---- SphereRayTracer (sphere_ray_tracer.rs) ----------------------------
class SphereRayTracer {
   public:
    static constexpr double NO_VALUE = GEO_NO_VALUE;  // :22

    // SphereRayTracer::new (:24-33): 2 * nr_nodes_half fan nodes; the f64
    // fan itself is computed on the GPU (geo_solve_ray_fan)
    SphereRayTracer(double sphere_r, double schwarz_r, uint32_t max_iter, double default_step, size_t nr_nodes_half,
                    std::shared_ptr<Context> ctx = nullptr)
        : ctx_(ctx ? std::move(ctx) : std::make_shared<Context>(0)),
          sphere_r_(sphere_r),
          schwarz_r_(schwarz_r),
          max_iter_(max_iter),
          default_step_(default_step),
          grid_(2 * nr_nodes_half, (float)NO_VALUE) {}

    // solve_ray_fan (:35-56): the fan of pi/2 - traveled angle at radius r;
    // also becomes the context's fan (the reference's update_ray_fan upload)
    const std::vector<float>& solve_ray_fan(double r) {
        check(geo_solve_ray_fan(ctx_->get(), sphere_r_, schwarz_r_, max_iter_, default_step_, (uint32_t)grid_.size(),
                                r, grid_.data(), nullptr),
              "geo_solve_ray_fan");
        return grid_;
    }
    // The fan at radius r into the context only, asynchronous on `stream`
    // (no host copy, so a frame loop does not synchronise); the host grid
    // is not updated.
    void update_device_fan(double r, void* stream = nullptr) {
        check(geo_solve_ray_fan(ctx_->get(), sphere_r_, schwarz_r_, max_iter_, default_step_, (uint32_t)grid_.size(),
                                r, nullptr, stream),
              "geo_solve_ray_fan");
    }
    const std::shared_ptr<Context>& context() const { return ctx_; }

   private:
    std::shared_ptr<Context> ctx_;
    double sphere_r_, schwarz_r_;
    uint32_t max_iter_;
    double default_step_;
    std::vector<float> grid_;
};

// ---- RayConnector (ray_connector.rs) ------------------------------------
// One connector, on the device (a batch of one of geo_rays); update_ray and
// reset_ray return [x, y, z, incoming angle] as the reference does.
class RayConnector {
   public:
    RayConnector(float schwarz_r, Vec3 pos, bool less_than_180, std::shared_ptr<Context> ctx = nullptr)
        : ctx_(ctx ? std::move(ctx) : std::make_shared<Context>(0)), out_(4) {
        const float p[3] = {pos.x, pos.y, pos.z};
        geo_rays* r = nullptr;
        check(geo_rays_create(ctx_->get(), schwarz_r, 1, less_than_180 ? GEO_RAYS_NEAR : GEO_RAYS_FAR, p, &r),
              "geo_rays_create");
        h_.reset(r);
    }
    std::array<float, 4> reset_ray(Vec3 other_position) { return call(other_position, 0, 1); }
    std::array<float, 4> update_ray(Vec3 other_position, uint32_t iterations) {
        return call(other_position, iterations, 0);
    }
    void set_position(Vec3 new_pos) {
        const float p[3] = {new_pos.x, new_pos.y, new_pos.z};
        check(geo_rays_set_positions(h_.get(), p), "geo_rays_set_positions");
    }

   private:
    std::array<float, 4> call(Vec3 o, uint32_t iterations, int reset) {
        const float other[3] = {o.x, o.y, o.z};
        check(geo_rays_update(h_.get(), other, 0, iterations, reset, out_.data(), nullptr), "geo_rays_update");
        std::array<float, 4> v;
        hip_check(hipMemcpy(v.data(), out_.data(), sizeof(v), hipMemcpyDeviceToHost), "hipMemcpy");
        return v;
    }
    struct Del {
        void operator()(geo_rays* r) const { geo_rays_destroy(r); }
    };
    std::shared_ptr<Context> ctx_;
    std::unique_ptr<geo_rays, Del> h_;
    DeviceBuffer<float> out_;
};

// ---- the render pass and the per-sphere plugin trait --------------------
// What a draw records into: the colour target (device RGBA8, width x height),
// the group-0 uniform, and the stream.  `cleared` is true until the first
// sphere draws: the reference clears to (0,0,0,1) (renderer.rs:233-238) and
// blends every sphere over the target (pipeline.rs:49); over a fresh clear
// that is libgeo's plain draw, later spheres use GEO_FLAG_COMPOSITE.
struct RenderPass {
    uint8_t* target;
    uint32_t width, height;
    TransformationPipeline uniform;
    void* stream;
    bool cleared;
};

class SchwarzschildSphereShaderDraw {  // schwarzschild_sphere_shader_draw.rs:3-6
   public:
    virtual ~SchwarzschildSphereShaderDraw() = default;
    virtual void draw(RenderPass& render_pass) const = 0;
};

// RGBA8 image (row-major), the reference's image::DynamicImage as uploaded
struct Image {
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> rgba;
};

// ---- BasicSphereBuffer (basic_sphere_buffer.rs) -------------------------
class BasicSphereBuffer : public SchwarzschildSphereShaderDraw {
   public:
    static constexpr size_t NR_NODES_HALF = 200;     // :42-51: 400 fan nodes
    static constexpr uint32_t MAX_ITER = 1000;
    static constexpr double STEP = kPi / 100.0;

    // BasicSphereBuffer::new (:21-60): the sphere's texture (group 2) and its
    // ray tracer; mode GEO_MODE_DIRECT integrates every pixel's own geodesic,
    // GEO_MODE_FAN lerps the reference's 400-node fan (shader.wgsl:77-84).
    // mipmaps: sample the texture's 4-level mip chain trilinearly as the
    // reference's textureSample does (Texture::new_with_mipmaps(..., 4),
    // GEO_FLAG_MIPS); off, the level-0 bilinear sample the benchmark measures.
    // ring_f64: the capture band's lanes integrate in f64 (GEO_FLAG_RING_F64:
    // direct or adaptive mode, the level-0 sampler, the pass's first sphere).
    BasicSphereBuffer(int device, double sphere_radius, double schwarz_radius, const Image& texture_image,
                      uint32_t mode = GEO_MODE_DIRECT, uint32_t max_iter = MAX_ITER, double step = STEP,
                      bool mipmaps = false, bool ring_f64 = false)
        : ctx_(std::make_shared<Context>(device)),
          ray_tracer_(sphere_radius, schwarz_radius, max_iter, step, NR_NODES_HALF, ctx_),
          sphere_radius_(sphere_radius),
          schwarz_radius_(schwarz_radius),
          max_iter_(max_iter),
          step_(step),
          mode_(mode),
          mipmaps_(mipmaps),
          ring_f64_(ring_f64) {
        check(geo_set_sky(ctx_->get(), texture_image.rgba.data(), texture_image.width, texture_image.height),
              "geo_set_sky");
    }

    // update_ray_fan (:85-88); the direct mode integrates per pixel, so the
    // radius is all it needs.  In fan mode the fan is solved into the
    // sphere's context on `stream` (the stream its draws run on: the
    // Renderer's), as the reference writes it into the sphere's fan texture.
    void update_ray_fan(double radial_position, void* stream = nullptr) {
        radial_position_ = radial_position;
        if (mode_ == GEO_MODE_FAN) ray_tracer_.update_device_fan(radial_position, stream);
    }

    // SchwarzschildSphereShaderDraw::draw (:92-100) + fs_main over the pass's target
    void draw(RenderPass& pass) const override {
        if (!(radial_position_ > 0.0)) throw Error("BasicSphereBuffer::draw before update_ray_fan", GEO_ESTATE);
        geo_scene s;
        s.rs = (float)schwarz_radius_;
        s.sphere_r = (float)sphere_radius_;
        s.r_obs = (float)radial_position_;
        s.step = (float)step_;
        s.max_steps = max_iter_;
        s.mode = mode_;
        s.flags = (pass.cleared ? 0u : GEO_FLAG_COMPOSITE) | (mipmaps_ ? GEO_FLAG_MIPS : 0u) |
                  (ring_f64_ ? GEO_FLAG_RING_F64 : 0u);
        s.tol = 0.0f;
        check(geo_render_rows(ctx_->get(), &pass.uniform, &s, pass.width, pass.height, 0, pass.height, pass.target,
                              nullptr, nullptr, nullptr, nullptr, pass.stream),
              "geo_render_rows");
        pass.cleared = false;
    }
    const std::shared_ptr<Context>& context() const { return ctx_; }

   private:
    std::shared_ptr<Context> ctx_;
    SphereRayTracer ray_tracer_;
    double sphere_radius_, schwarz_radius_;
    uint32_t max_iter_;
    double step_;
    uint32_t mode_;
    bool mipmaps_;
    bool ring_f64_;
    double radial_position_ = 0.0;
};

// ---- PointCloud (point_cloud.rs) and its point meshes --------------------
class PointCloud {
   public:
    // PointCloud::new (:20-65)
    PointCloud(int device, const std::vector<Vec3>& model_vertices, float schwarz_r, Vec3 observer_pos,
               bool activate_farside, bool activate_orbits, uint64_t seed = 0)
        : ctx_(std::make_shared<Context>(device)), n_((uint32_t)model_vertices.size()), farside_(activate_farside) {
        std::vector<float> xyz(3 * model_vertices.size());
        for (size_t i = 0; i < model_vertices.size(); ++i) {
            xyz[3 * i] = model_vertices[i].x;
            xyz[3 * i + 1] = model_vertices[i].y;
            xyz[3 * i + 2] = model_vertices[i].z;
        }
        const float o[3] = {observer_pos.x, observer_pos.y, observer_pos.z};
        geo_points* p = nullptr;
        check(geo_points_create(ctx_->get(), schwarz_r, xyz.data(), n_, o, activate_farside ? 1 : 0,
                                activate_orbits ? 1 : 0, seed, &p),
              "geo_points_create");
        h_.reset(p);
    }

    // the model generators (:67-115), exposed so a caller can keep the vertices
    static std::vector<Vec3> spiral_model() {  // new_spiral (:67-81)
        const size_t n = 10000;
        std::vector<Vec3> pts(n);
        for (size_t i = 0; i < n; ++i) {
            const float t = (float)i / (float)n * (6.28318530717958647692f + 0.05f);
            const float r = 16.0f + 2.0f * t;
            pts[i] = {-r * std::cos(10.0f * t), -r * std::sin(10.0f * t), 0.001f};
        }
        return pts;
    }
    // new_accretion_disk (:83-99): points at r in [16, 26), |theta| < 0.1.  The
    // reference draws from an OS-seeded fastrand stream; here a seeded wyrand
    // stream (the same generator family).
    static std::vector<Vec3> accretion_disk_model(uint64_t seed = 0, size_t n = 5000) {
        uint64_t s = seed ^ 0x5C4Aull;
        auto f64 = [&s]() {
            s += 0xA0761D6478BD642Full;
            const __uint128_t t = (__uint128_t)s * (s ^ 0xE7037ED1A0B428DBull);
            const uint64_t v = (uint64_t)(t >> 64) ^ (uint64_t)t;
            return (double)(v >> 11) * 0x1.0p-53;
        };
        std::vector<Vec3> pts(n);
        for (size_t i = 0; i < n; ++i) {
            const double r = 16.0 + 10.0 * f64();
            const double phi = f64() * 2.0 * kPi;
            const double theta = 0.2 * (f64() - 0.5);
            // polar_to_carthesic (polar_transformations.rs)
            pts[i] = {(float)(r * std::cos(phi) * std::cos(theta)), (float)(r * std::sin(phi) * std::cos(theta)),
                      (float)(r * std::sin(theta))};
        }
        return pts;
    }
    static std::vector<Vec3> heart_model() {  // new_heart (:101-115)
        const size_t n = 4000;
        std::vector<Vec3> pts(n);
        for (size_t i = 0; i < n; ++i) {
            const float t = (float)i / (float)n * 6.28318530717958647692f;
            const float st = std::sin(t);
            pts[i] = {11.0f, 16.0f * st * st * st,
                      13.0f * std::cos(t) - 5.0f * std::cos(2.0f * t) - 2.0f * std::cos(3.0f * t) -
                          std::cos(4.0f * t)};
        }
        return pts;
    }
    static PointCloud new_spiral(int device, float schwarz_r, Vec3 observer_pos, bool activate_farside) {
        return PointCloud(device, spiral_model(), schwarz_r, observer_pos, activate_farside, false);
    }
    static PointCloud new_accretion_disk(int device, float schwarz_r, Vec3 observer_pos, bool activate_farside,
                                         uint64_t seed = 0, size_t n = 5000) {
        return PointCloud(device, accretion_disk_model(seed, n), schwarz_r, observer_pos, activate_farside, true,
                          seed);
    }
    static PointCloud new_heart(int device, float schwarz_r, Vec3 observer_pos, bool activate_farside) {
        return PointCloud(device, heart_model(), schwarz_r, observer_pos, activate_farside, false);
    }

    // update (:117-148): orbits and respawns, then update_ray(observer, 1);
    // dt in seconds; asynchronous on `stream` (a side stream overlaps it with
    // the sphere draws; draw() orders itself after it)
    void update(Vec3 observer_pos, double dt, void* stream = nullptr) {
        const float o[3] = {observer_pos.x, observer_pos.y, observer_pos.z};
        check(geo_points_update(h_.get(), o, dt, stream), "geo_points_update");
    }
    // get_vertices / get_vertices_farside (:150-156): host copies, [x, y, z, angle]
    std::vector<std::array<float, 4>> get_vertices(bool farside = false) const {
        const float* d = geo_points_vertices(h_.get(), farside ? 1 : 0);
        if (!d) throw Error("get_vertices_farside of a cloud without a far side", GEO_EINVAL);
        std::vector<std::array<float, 4>> v(n_);
        hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        hip_check(hipMemcpy(v.data(), d, v.size() * sizeof(v[0]), hipMemcpyDeviceToHost), "hipMemcpy");
        return v;
    }
    // the point meshes' draw (schwarzschild_point_shader/shader.wgsl:36-74):
    // the near-side vertices, then the far-side ones
    // (geo_points_draw).  The draw waits for the last update() and the next
    // update() for the draw, on whichever streams they run, so update() may
    // take a side stream and overlap the sphere draws.
    void draw(RenderPass& pass) const {
        check(geo_points_draw(h_.get(), &pass.uniform, pass.width, pass.height, 0, pass.height, pass.target, nullptr,
                              pass.stream),
              "geo_points_draw");
    }
    uint32_t len() const { return n_; }
    bool has_farside() const { return farside_; }

   private:
    struct Del {
        void operator()(geo_points* p) const { geo_points_destroy(p); }
    };
    std::shared_ptr<Context> ctx_;
    std::unique_ptr<geo_points, Del> h_;
    uint32_t n_;
    bool farside_;
};

// ---- Renderer (renderer.rs) ---------------------------------------------
// Owns the observer and the colour target (the surface texture of the
// reference's present loop, here device RGBA8 that read_frame copies out).
class Renderer {
   public:
    // Renderer::new (renderer.rs:48-139): observer with the reference's
    // schwarz_r and fov at the surface size
    Renderer(uint32_t width, uint32_t height, double schwarz_r = 10.0, double fov = kPi / 2, void* stream = nullptr)
        : observer_(schwarz_r, fov, width, height),
          width_(width),
          height_(height),
          target_((size_t)width * height * 4),
          stream_(stream) {}

    // update (:152-161): the observer moves with the controller's input
    // (none here) for dt seconds
    void update(double dt, DVec3 desired_direction = {0.0, 0.0, 0.0}) {
        observer_.update_position(desired_direction, dt);
    }
    // resize (:141-150)
    void resize(uint32_t width, uint32_t height) {
        if (width == 0 || height == 0) return;
        width_ = width;
        height_ = height;
        target_ = DeviceBuffer<uint8_t>((size_t)width * height * 4);
        observer_.update_screen_format(width, height);
    }
    // render (:208-264): clear to (0,0,0,1), the uniform, every sphere's draw
    // in order, then the point meshes.  Asynchronous.
    void render(const std::vector<const SchwarzschildSphereShaderDraw*>& sphere_shader_meshes,
                const std::vector<const PointCloud*>& point_meshes) {
        RenderPass pass{target_.data(), width_, height_, observer_.calc_transformation_pipeline(), stream_, true};
        if (sphere_shader_meshes.empty())
            hip_check(hipMemsetD32Async((hipDeviceptr_t)target_.data(), 0xFF000000u, (size_t)width_ * height_,
                                        (hipStream_t)stream_),
                      "hipMemsetD32Async");
        for (const SchwarzschildSphereShaderDraw* s : sphere_shader_meshes) s->draw(pass);
        for (const PointCloud* p : point_meshes) p->draw(pass);
        last_uniform_ = pass.uniform;
    }
    // the presented frame: width*height RGBA8, row-major (synchronises)
    std::vector<uint8_t> read_frame() const {
        std::vector<uint8_t> out((size_t)width_ * height_ * 4);
        hip_check(hipStreamSynchronize((hipStream_t)stream_), "hipStreamSynchronize");
        hip_check(hipMemcpy(out.data(), target_.data(), out.size(), hipMemcpyDeviceToHost), "hipMemcpy");
        return out;
    }
    double get_schwarz_r() const { return observer_.get_schwarz_r(); }        // :285-287
    double get_radial_position() const { return observer_.get_radial_position(); }  // :289-291
    Vec3 get_position() const {                                                // :293-296
        const DVec3 p = observer_.get_position();
        return {(float)p.x, (float)p.y, (float)p.z};
    }
    Observer& observer() { return observer_; }
    const TransformationPipeline& last_uniform() const { return last_uniform_; }
    uint32_t width() const { return width_; }
    uint32_t height() const { return height_; }
    uint8_t* target() const { return target_.data(); }

   private:
    Observer observer_;
    uint32_t width_, height_;
    DeviceBuffer<uint8_t> target_;
    void* stream_;
    TransformationPipeline last_uniform_{};
};

}  // namespace sr
