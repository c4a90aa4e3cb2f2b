// The reference's own tests (SR/simulation/tests.rs) through the C++ host
// mirror (include/geo/sr.hpp) over libgeo, plus one presented frame.
//
//   sr_reference_tests tests          tests.rs:8-79, same names, loops, tolerances
//   sr_reference_tests frame W H DIR  Renderer::render of the sky sphere (+ the
//                                     heart point cloud): FNV-1a of both frames;
//                                     DIR/model.f32 = the cloud's model vertices
//
// tests/test_cpp_host.py builds it (CPU) and runs it (GPU), comparing the
// fan with the oracle and the frames with the oracle / the Python host.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "geo/sr.hpp"

namespace {

sr::Vec3 sub(sr::Vec3 a, sr::Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
sr::Vec3 neg(sr::Vec3 a) { return {-a.x, -a.y, -a.z}; }
// glam::Vec3::angle_between: acos(dot / sqrt(|a|^2 |b|^2))
float angle_between(sr::Vec3 a, sr::Vec3 b) {
    const float d = a.x * b.x + a.y * b.y + a.z * b.z;
    const float l = std::sqrt((a.x * a.x + a.y * a.y + a.z * a.z) * (b.x * b.x + b.y * b.y + b.z * b.z));
    float c = d / l;
    c = c > 1.0f ? 1.0f : (c < -1.0f ? -1.0f : c);
    return std::acos(c);
}

// tests.rs:8-13 (asserts nothing in the reference; the fan is printed for the
// caller to compare with the oracle)
bool sphere_geodesics_test() {
    sr::SphereRayTracer sphere(100., 10., 100, sr::kPi / 100., 10);
    const std::vector<float>& result = sphere.solve_ray_fan(25.);
    std::printf("sphere_geodesics_test fan");
    for (float v : result) std::printf(" %a", v);
    std::printf("\n");
    return result.size() == 20;
}

// tests.rs:15-38
bool ray_connector_euclidian_test() {
    const int NR_TESTS = 100;
    int counter = 0;
    auto ctx = std::make_shared<sr::Context>(0);
    for (int i = 0; i < NR_TESTS; ++i) {
        const sr::Vec3 pos{20.f, 0.f, 0.1f};
        const float angle = (float)i / (float)NR_TESTS * 3.14159265358979323846f;
        const sr::Vec3 observer_pos{19.f * std::cos(angle), 19.f * std::sin(angle), 0.f};
        sr::RayConnector ray_connector(0., pos, true, ctx);
        const float euclidian_angle = angle_between(sub(pos, observer_pos), neg(observer_pos));
        const std::array<float, 4> output = ray_connector.reset_ray(observer_pos);
        const float error = std::fabs(euclidian_angle - output[3]);
        if (error < 5e-4f)
            counter += 1;
        else
            std::printf("Failed with error %g at angle %g\n", error, angle);
    }
    std::printf("ray_connector_euclidian_test %d/%d\n", counter, NR_TESTS);
    return counter == NR_TESTS;
}

// tests.rs:40-79
bool ray_connector_euclidian_tracing_test() {
    const int NR_TESTS = 60;
    int counter = 0;
    auto ctx = std::make_shared<sr::Context>(0);
    const sr::Vec3 pos{20.f, 0.f, 0.1f};
    sr::RayConnector ray_connector(5., pos, true, ctx);
    sr::RayConnector control(5., pos, true, ctx);
    sr::RayConnector ray_connector_far(5., pos, false, ctx);
    sr::RayConnector control_far(5., pos, false, ctx);
    for (int i = 0; i < NR_TESTS; ++i) {
        const float angle = (float)i / (float)NR_TESTS * 6.28318530717958647692f;
        const sr::Vec3 observer_pos{7.f * std::cos(angle), 7.f * std::sin(angle), 0.f};
        const auto output = ray_connector.update_ray(observer_pos, 1);
        const auto output2 = control.update_ray(observer_pos, 5);
        const auto output_far = ray_connector_far.update_ray(observer_pos, 1);
        const auto output2_far = control_far.update_ray(observer_pos, 5);
        const float error = std::fabs(output2[3] - output[3]);
        const float error_far = std::fabs(output2_far[3] - output_far[3]);
        if (error < 5e-4f)
            counter += 1;
        else
            std::printf("Failed with error %g at angle %g\n", error, angle);
        if (error_far < 5e-4f)
            counter += 1;
        else
            std::printf("Failed with error %g at angle %g for the farside ray\n", error_far, angle);
    }
    std::printf("ray_connector_euclidian_tracing_test %d/%d\n", counter, 2 * NR_TESTS);
    return counter == 2 * NR_TESTS;
}

uint64_t fnv1a(const std::vector<uint8_t>& b) {
    uint64_t h = 1469598103934665603ull;
    for (uint8_t x : b) h = (h ^ x) * 1099511628211ull;
    return h;
}

// the synthetic 512x256 sky of examples/render_frame.c
sr::Image test_sky() {
    sr::Image im;
    im.width = 512;
    im.height = 256;
    im.rgba.resize((size_t)im.width * im.height * 4);
    for (uint32_t y = 0; y < im.height; ++y)
        for (uint32_t x = 0; x < im.width; ++x) {
            uint8_t* t = &im.rgba[4 * ((size_t)y * im.width + x)];
            t[0] = (uint8_t)((x * 7u) ^ (y * 13u));
            t[1] = (uint8_t)(x + y);
            t[2] = (uint8_t)(x * y);
            t[3] = 255;
        }
    return im;
}

int frame(uint32_t W, uint32_t H, const std::string& dir) {
    // the reference's default scene scaled to rs = 1 (lib.rs:72, observer.rs:70-81)
    sr::Renderer renderer(W, H, 1.0, sr::kPi / 2);
    renderer.observer().set_position({2.5, 0.0, 0.1});
    sr::BasicSphereBuffer sky(0, 50.0, 1.0, test_sky(), GEO_MODE_DIRECT, 2048);
    sky.update_ray_fan(renderer.get_radial_position());
    renderer.render({&sky}, {});
    const uint64_t h_sky = fnv1a(renderer.read_frame());

    sr::PointCloud heart = sr::PointCloud::new_heart(0, 1.0f, renderer.get_position(), true);
    heart.update(renderer.get_position(), 1.0 / 60.0);
    renderer.render({&sky}, {&heart});
    const uint64_t h_all = fnv1a(renderer.read_frame());
    // the model the cloud was built from, for the Python host's twin frame
    FILE* f = std::fopen((dir + "/model.f32").c_str(), "wb");
    if (!f) return 1;
    for (const sr::Vec3& v : sr::PointCloud::heart_model()) {
        const float xyz[3] = {v.x, v.y, v.z};
        std::fwrite(xyz, sizeof(float), 3, f);
    }
    std::fclose(f);
    std::printf("frame sky fnv1a %016llx\nframe sky+points fnv1a %016llx\n", (unsigned long long)h_sky,
                (unsigned long long)h_all);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "tests";
    try {
        if (mode == "tests") {
            const bool a = sphere_geodesics_test();
            const bool b = ray_connector_euclidian_test();
            const bool c = ray_connector_euclidian_tracing_test();
            std::printf("%s\n", a && b && c ? "all passed" : "FAILED");
            return a && b && c ? 0 : 1;
        }
        if (mode == "frame" && argc > 4) return frame((uint32_t)std::atoi(argv[2]), (uint32_t)std::atoi(argv[3]), argv[4]);
        std::fprintf(stderr, "usage: %s tests | frame W H DIR\n", argv[0]);
        return 2;
    } catch (const sr::Error& e) {
        std::fprintf(stderr, "sr::Error: %s\n", e.what());
        return 3;
    }
}
