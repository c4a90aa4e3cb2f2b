// geo_ctx.h — the device context shared by the libgeo translation units
// (geo_render.hip: sky, fan, step counters; geo_points.hip: point clouds).
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

struct geo_ctx {
    int device;
    int num_cus;
    // The sky's mip chain (geo::kSkyMipLevels levels, geo::mip_down), each
    // level padded (geo::pad_sky) and stored one after another in `sky`:
    // level l at byte sky_lvl_off[l], (sky_lvl_w[l] + 2) x (sky_lvl_h[l] + 2)
    // texels; level 0 first, so a level-0 render reads `sky` as before.
    uint32_t* sky;
    uint32_t sky_w, sky_h;
    bool sky_opaque;
    static constexpr int kSkyLevels = 4;
    uint32_t sky_lvl_w[kSkyLevels], sky_lvl_h[kSkyLevels], sky_lvl_off[kSkyLevels];
    uint32_t sky_total_bytes;
    uint32_t sky_pairs_off;  // kSkyPairs: byte offset of level 0's row pairs in `sky` (geo_render.hip)
    // Ray fan, double-buffered so that a frame's fan can be solved on a side
    // stream while the previous frame's fan-mode draws still read the other
    // buffer.  fan[fan_cur] is the context's fan (fan_cur < 0: none).  Each
    // buffer's last writer (geo_solve_ray_fan, on fan_writer[b]) and readers
    // (fan-mode renders) are tracked so that a solve into a buffer waits for
    // the draws that read it and a draw waits for the solve that wrote its
    // buffer, whatever streams they run on, with no event work for what
    // stream order already gives:
    //   * a draw on the writer's stream neither waits for the solve nor
    //     records an event: its slot's bit in fan_read_slots[b] stands for it
    //     (render_done of that slot completes after it);
    //   * a draw on another stream waits for fan_written[b] and joins the
    //     chained reader event fan_read[b] (recorded after its launch; when
    //     the previous recorder ran on another stream the draw first waits for
    //     it, so the event covers every recorded reader);
    //   * a solve into b waits for the writer, the chain and the slots' events
    //     that are not on its own stream, then starts b's record afresh.
    float* fan[2];
    uint32_t fan_cap, n_fan[2];
    int fan_cur;
    hipEvent_t fan_written[2], fan_read[2];
    bool fan_written_rec[2], fan_read_rec[2];
    hipStream_t fan_writer[2], fan_reader[2];  // streams of the last solve, of the last chain record
    uint32_t fan_read_slots[2];               // render slots (bits) whose unrecorded draws read the buffer
    // Sharded step counters: set 0 is the GEO_FLAG_DEFER_STEPS accumulator
    // (geo_steps_flush folds it); a render with a steps_total of its own
    // counts into one of kStepCallSets per-call sets, taken round-robin, and
    // folds it into its total on its stream.  A set is taken again only after
    // its previous fold (step_set_free), so renders on different streams never
    // fold each other's counts.
    unsigned long long* step_slots;
    static constexpr int kStepCallSets = 4;
    hipEvent_t step_set_free[kStepCallSets];
    bool step_set_rec[kStepCallSets];
    int step_set_next;
    // The last render of this context on each stream it has rendered on, so
    // that a sky upload or a fan regrow waits for the renders that may read
    // the buffer it replaces, and for nothing else (a device-wide wait would
    // also wait for other contexts' work and for collectives in flight that
    // need peers, which can hang a rank).  More than kRenderStreams streams:
    // a new stream takes slot render_next after waiting for that slot's event,
    // so the event it records covers the evicted stream's render too.
    static constexpr int kRenderStreams = 8;
    hipStream_t render_stream[kRenderStreams];
    hipEvent_t render_done[kRenderStreams];
    int n_render_streams, render_next;
    // Workgroup dispatch order ("Longest-first dispatch").
    // GEO_DISPATCH_LONGEST_FIRST: every `dispatch_period`-th render of a grid
    // records each tile's cost (its waves' largest step counts, atomically
    // added into tile_cost) and two small kernels after it rebuild the order
    // from those costs, most expensive tile first, into the order buffer the
    // current one is not in; later renders of the same grid (learn_key)
    // dispatch in that order.  The rebuild runs on the context's own
    // learn_stream, after every render of the context issued before it
    // (render_done of every slot, waited for on learn_stream only), so no
    // render still reads the buffer it overwrites and no render stream ever
    // waits for another (such a wait can sit behind a collective).
    // Renders adopt the new order only once the host has seen the rebuild
    // complete (hipEventQuery, never a wait), so none waits for it either; a
    // recording render is deferred while a rebuild is pending (the rebuild
    // consumes and zeroes the costs).
    // GEO_DISPATCH_EXPLICIT: geo_set_tile_order's order for its grid.
    // Orders are packed (y << 16 | x) per workgroup.
    int dispatch_mode;
    uint32_t dispatch_period, since_learn;  // renders of the grid since its last recording one
    uint32_t learn_key[9];
    bool learn_valid;   // learn_key names a grid
    int order_cur;      // order[order_cur] is the grid's order (-1: none yet)
    uint32_t* order[2];
    uint32_t* tile_cost;  // per tile of the learned grid; zero between rebuilds
    uint32_t* class_hist;
    uint32_t tile_cap;    // tiles the buffers hold
    uint32_t explicit_x, explicit_y;  // GEO_DISPATCH_EXPLICIT's grid
    hipEvent_t order_written;   // the last rebuild, on learn_stream
    hipStream_t learn_stream;   // created by the first rebuild
    bool rebuild_pending;       // issued, not yet seen complete by the host
    bool rebuild_keep;          // its order is still wanted (same grid and mode since)
    int rebuild_nb;             // the order buffer it writes
    unsigned long long costs_recorded, orders_adopted;  // geo_dispatch_stats
    // geo_time_next_render: events for the next render's kernel dispatch
    hipEvent_t time_start, time_stop;
#if defined(GEO_WAVE_LOG)
    unsigned long long* wave_log;  // diagnostic build only (geo_debug_set_wave_log)
#endif
};

// Makes `dev` current for the scope of a C-ABI call, restoring the caller's
// device.  It also clears the thread's last-error state first: the call's
// launches are checked with hipGetLastError, which would otherwise report an
// error left by an unrelated earlier HIP call of the caller (e.g. an elapsed
// time asked of an unrecorded event) as this call's failure.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        (void)hipGetLastError();
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
