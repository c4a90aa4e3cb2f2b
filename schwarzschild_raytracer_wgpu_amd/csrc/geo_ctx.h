// geo_ctx.h — the device context shared by the libgeo translation units
// (geo_render.hip: sky, fan, step counters; geo_points.hip: point clouds).
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

struct geo_ctx {
    int device;
    int num_cus;
    uint32_t* sky;
    uint32_t sky_w, sky_h;
    bool sky_opaque;
    float* fan;
    uint32_t fan_cap, n_fan;
    unsigned long long* step_slots;
};

// Makes `dev` current for the scope of a C-ABI call, restoring the caller's device.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
