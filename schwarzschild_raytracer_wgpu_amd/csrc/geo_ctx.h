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
    // Ray fan, double-buffered so that a frame's fan can be solved on a side
    // stream while the previous frame's fan-mode draws still read the other
    // buffer.  fan[fan_cur] is the context's fan (fan_cur < 0: none).  Each
    // buffer's last writer (geo_solve_ray_fan) and readers (fan-mode renders,
    // a chained event: every render waits, after its launch, for the previous
    // reader) are events, so a solve into a buffer waits for the draws that
    // read it and a draw waits for the solve that wrote its buffer, whatever
    // streams they run on.
    float* fan[2];
    uint32_t fan_cap, n_fan[2];
    int fan_cur;
    hipEvent_t fan_written[2], fan_read[2];
    bool fan_written_rec[2], fan_read_rec[2];
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
