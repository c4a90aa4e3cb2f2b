// The reference's per-frame loop (SR/lib.rs State::update + State::render,
// lib.rs:287-300 and 413-419) in C++ over libgeo, through the host mirror
// include/geo/sr.hpp: the observer falls, each sphere's ray fan is updated to
// the new radius, the accretion disk's orbits and RayConnectors are advanced,
// and the renderer draws the sky sphere and the disk's two point meshes.
//
// Build:
//   g++ -std=c++17 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include examples/frame_loop.cpp
//       -L schwarzschild_raytracer_wgpu_amd -lgeo -L /opt/rocm/lib -lamdhip64 -o frame_loop
//   ./frame_loop [W H FRAMES out.ppm OVERLAP(1|0) MODE(direct|fan)]
//
// MODE fan draws the sky the way the reference displays it: each frame solves
// the sphere's 400-node f64 ray fan on the GPU (stream-ordered, no host copy)
// and the shader lerps into it; direct (default) integrates every pixel.
//
// Prints frames/s of the whole loop (host + GPU, K frames back to back) and
// writes the last frame.  Scene: the reference's, scaled to rs = 1 (its
// schwarz_r = 10 scene divided by 10): sky r = 50 with a synthetic equirect
// texture, observer FrozenFall from (2.5, 0, 0.1), 5000-point disk.
#include <chrono>
#include <string>
#include <cstdio>
#include <cstdlib>

#include "geo/sr.hpp"

int main(int argc, char** argv) {
    const uint32_t W = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1920u;
    const uint32_t H = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1080u;
    const int frames = argc > 3 ? std::atoi(argv[3]) : 300;
    const char* out = argc > 4 ? argv[4] : "frame_loop.ppm";
    const bool overlap = argc > 5 ? std::atoi(argv[5]) != 0 : true;
    // "fan": the reference's display path (a 400-node f64 fan per frame, lerped per pixel)
    const bool fan = argc > 6 && std::string(argv[6]) == "fan";
    try {
        sr::Image sky;
        sky.width = 2048;
        sky.height = 1024;
        sky.rgba.resize((size_t)sky.width * sky.height * 4);
        for (uint32_t y = 0; y < sky.height; ++y)
            for (uint32_t x = 0; x < sky.width; ++x) {  // 8-degree lat/long checkerboard
                uint8_t* t = &sky.rgba[4 * ((size_t)y * sky.width + x)];
                const bool c = (((x * 360u / sky.width) / 8u) + ((y * 180u / sky.height) / 8u)) & 1u;
                t[0] = c ? 230 : 40;
                t[1] = c ? 200 : 60;
                t[2] = c ? 120 : 160;
                t[3] = 255;
            }

        sr::Renderer renderer(W, H, 1.0, sr::kPi / 2);
        renderer.observer().set_position({2.5, 0.0, 0.1});
        sr::BasicSphereBuffer first_sphere(0, 50.0, 1.0, sky, fan ? GEO_MODE_FAN : GEO_MODE_DIRECT);
        sr::PointCloud first_point_cloud =
            sr::PointCloud::new_accretion_disk(0, 1.0f, renderer.get_position(), true);

        // The disk update is latency-bound (one lane per connector, sequential
        // 48-node solves): on a side stream it overlaps the VALU-bound sky
        // draw; PointCloud::draw waits for it (geo_points_draw).
        hipStream_t side = nullptr, fan_stream = nullptr;
        if (overlap) sr::hip_check(hipStreamCreateWithFlags(&side, hipStreamNonBlocking), "hipStreamCreate");
        // Fan mode: the frame's fan on its own stream.  The context double-buffers
        // the fan and orders solves and draws with events, so this frame's fan
        // overlaps the previous frame's draws and its own draw still waits for it.
        if (overlap && fan)
            sr::hip_check(hipStreamCreateWithFlags(&fan_stream, hipStreamNonBlocking), "hipStreamCreate");
        const double dt = 1.0 / 60.0;
        auto frame = [&]() {
            // State::update (lib.rs:287-300)
            renderer.update(dt);
            const double r = renderer.get_radial_position();
            first_sphere.update_ray_fan(r, fan_stream);
            first_point_cloud.update(renderer.get_position(), dt, side);
            // State::render (lib.rs:413-419): the first sphere and both point meshes
            renderer.render({&first_sphere}, {&first_point_cloud});
        };
        for (int i = 0; i < 30; ++i) frame();
        sr::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < frames; ++i) frame();
        sr::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

        const std::vector<uint8_t> rgba = renderer.read_frame();
        FILE* f = std::fopen(out, "wb");
        if (!f) return 1;
        std::fprintf(f, "P6\n%u %u\n255\n", W, H);
        for (size_t i = 0; i < (size_t)W * H; ++i) std::fwrite(&rgba[4 * i], 1, 3, f);
        std::fclose(f);
        std::printf("%ux%u%s%s: %d frames in %.3f s = %.1f frames/s (%.4f ms/frame); observer r = %.4f\n", W, H,
                    fan ? " fan mode" : "", overlap ? (fan ? " (disk update and fans on side streams)" : " (disk update on a side stream)") : "", frames, s, frames / s,
                    s / frames * 1e3,
                    renderer.get_radial_position());
        if (side) sr::hip_check(hipStreamDestroy(side), "hipStreamDestroy");
        if (fan_stream) sr::hip_check(hipStreamDestroy(fan_stream), "hipStreamDestroy");
        return 0;
    } catch (const sr::Error& e) {
        std::fprintf(stderr, "sr::Error: %s\n", e.what());
        return 3;
    }
}
