// geo_render.hip — gfx950 kernels and the device half of the libgeo C-ABI.
//
//   geo_render_kernel<MODE>  per-pixel fs_main + solve_geodesic (fixed RK4, fan lerp,
//                            or error-controlled RK5(4): GEO_MODE_ADAPTIVE)
//                            (SR/schwarzschild_sphere_shader/shader.wgsl:57-106,
//                             SR/simulation/sphere_ray_tracer.rs:35-193)
//   geo_fan_kernel           SphereRayTracer::solve_ray_fan in f64, one lane per node
//                            (sphere_ray_tracer.rs:35-193)
//   geo_steps_finalize       folds the sharded step counters into the caller's u64
//
// Work decomposition: one 256-thread workgroup per 32x8 pixel tile, each
// wave64 a 16x4 block (compact 2-D footprint = coherent step counts), 2 x 2
// of them (a tile row spans one 128-B sky line);
// the frame uniform rides in the kernarg segment (SGPRs, wave-uniform), the
// ray fan (fan mode) is read from its cache-resident device copy; per-lane
// ray state lives in VGPRs.  The hot loop
// is pure FP32 VALU — no MFMA, no LDS, no memory traffic.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <type_traits>
#include <vector>

#include "../../include/geo/geo.h"
#include "geo_ctx.h"
#include "geo_band.h"
#include "geo_pixel.h"

// Work decomposition (measured): 32 x 8-pixel workgroup tiles
// of 2 x 2 waves of 16 x 4 pixels.  A tile row spans 32 sky texels = one
// 128-B line, so neighbouring waves share their sky lines in one CU instead of
// fetching them on up to 4 XCDs' L2s (102.8 -> 59.5 MB of L2 fabric reads per
// 4K frame against 8 x 32 tiles; config 3 -2 to -5 %, config 5 -2 %, config 2
// -1.5 %; 16 x 16, 64 x 8 and 32 x 16 in between); the 16 x 4 wave shape is
// -0.5 % on config 3 against 8 x 8, 32 x 2 is +2.5 % (steps diverge more
// within a wave).  Tiles keep the hardware's round-robin placement over the
// XCDs: runs of consecutive tiles per XCD were slower on every config.  The
// fan (fan mode) is read from its cache-resident device copy: staging it in
// LDS per workgroup put a load and a barrier before every block's pixel work
// (+6 % per 4K fan-mode frame).

namespace {

constexpr int kWaveW = 16;             // a wave64 covers a compact 16x4 block (few divergent
constexpr int kWaveRows = 64 / kWaveW;  // steps per wave; tools/ubench/loop_ab.hip at 3cd1aa2)
constexpr int kWavesX = 2;              // waves side by side in a tile
constexpr int kTileW = kWaveW * kWavesX;
constexpr int kTileH = 8;               // a block kTileW x kTileH
constexpr int kBlock = kTileW * kTileH;  // 256 threads = 4 waves (32 x 8, 2 x 2 waves of 16 x 4;
                                         // twice as tall with two pixels per lane, lane_rows)
static_assert(kTileH % kWaveRows == 0 && kBlock % 64 == 0, "tile of whole waves");
// band heights are multiples of 8 (the C-ABI's contract, geo.h), so a wave's
// rows never straddle a band for any wave shape up to 8 rows
constexpr uint32_t kBandRowAlign = 8;
static_assert(kBandRowAlign % kWaveRows == 0, "a wave's rows lie in one band");
constexpr uint32_t kMaxFan = 4096;       // fan nodes (16 KiB)
constexpr uint32_t kDefaultDispatchPeriod = 16;  // renders of a grid per re-learned order
// a tile's out-of-loop work in steps of its mode's loop (the set-up, Newton
// crossing and sky epilogue: ~330 VALU against 14 per RK4 step, ~420 against
// ~57 per RK5(4) attempt), added to each wave's recorded cost
constexpr uint32_t kCostOverheadDirect = 24, kCostOverheadAdaptive = 8;
constexpr int kStepSlots = 256;          // sharded step counters (one per 128-B line)
constexpr int kSlotStride = 16;          // u64 per slot = 128 B (own cache line)
constexpr size_t kSlotSetU64 = (size_t)kStepSlots * kSlotStride;  // one set of sharded counters
constexpr int kSlotSets = 1 + geo_ctx::kStepCallSets;            // the DEFER accumulator + per-call sets

// The per-frame part of a launch: the uniform and the camera constants the
// host derives from it (a second kernel argument, FrameBatch, one per frame
// of a batched launch, geo_render_band_set_frames).
struct FrameK {
    geo_frame frame;
    geo::CameraConsts cam;  // the pixel's camera ray (geo::camera_consts)
    float kt;               // geo::aberration_kt
};
constexpr uint32_t kMaxBatchFrames = GEO_MAX_BATCH_FRAMES;
// A batch's frames may each have their own observer radius (their scenes
// differ in r_obs only, geo_render_band_set_batch): the scene constants of
// each frame ride along (the integration kind is shared); a single-frame
// launch reads RenderArgs::k.
template <uint32_t NF>
struct FrameBatch {
    FrameK f[NF];
    geo::PixelConsts k[NF];
    float ring_kx[NF];  // GEO_FLAG_RING_F64: frame z's band factor (geo::band_kx; 0: no band)
};
template <>
struct FrameBatch<1> {
    FrameK f[1];
};

struct RenderArgs {
    geo::PixelConsts k;  // scene constants, evaluated once on the host (IEEE f32, same bits)
    uint32_t width, height, row0, nrows;
    uint32_t tile_y0;  // first tile row of this launch (launch_tiles)
    uint32_t tiles_x, launch_tiles;  // the frame's tiles per row; the tiles of this launch (wave_blocks)
    uint32_t persist_blocks;         // kFanPersist: workgroups of the fan draw's grid
    // dispatch order (geo_ctx): workgroup i draws tile
    // (order[i] & 0xFFFF, order[i] >> 16); null = row-major
    const uint32_t* tile_order;
    // a cost-recording render: each wave adds its largest step count plus
    // cost_overhead (its out-of-loop work, in steps) into its tile's entry
    unsigned int* tile_cost;
    uint32_t cost_overhead;
    // local row lr -> row0 + b*band_stride + (lr - b*band_rows), b = lr / band_rows
    // = umulhi(lr, band_magic) (band_rows_magic)
    uint32_t band_rows, band_magic, band_stride;
    uint32_t sky_opaque;
    uint32_t composite;  // GEO_FLAG_COMPOSITE
    const uint32_t* sky;  // padded (geo::pad_sky): (sky_w + 2) x (sky_h + 2) texels
    uint32_t sky_w, sky_h;
    float sky_w256, sky_h256;  // sky_w * 256, sky_h * 256 (exact; geo::sample_sky_quad_f)
    uint32_t sky_pitch_b, sky_bytes;
    // GEO_FLAG_MIPS: level l's byte offset, pitch and sizes * 256; level 0's
    // size for the footprint; the whole chain's bytes
    uint32_t mip_off[geo::kSkyMipLevels], mip_pitch[geo::kSkyMipLevels];
    float mip_w256[geo::kSkyMipLevels], mip_h256[geo::kSkyMipLevels];
    float sky_wf, sky_hf;
    uint32_t sky_total_bytes;
    uint32_t sky_pairs_off, sky_pairs_pitch;  // kSkyPairs: level 0's row pairs (PairSkyQuad)
    const float* fan;
    uint32_t n_fan;
    uint32_t* out_rgba;
    uint8_t* out_mask;
    float2* out_uv;
    uint32_t* out_steps;
    unsigned long long* step_slots;
    uint64_t out_frame_px;  // batched launch: pixels from one frame's output to the next (colour only)
#if defined(GEO_WAVE_LOG)
    // diagnostic build only (tools/wave_timeline.py): per wave, in launch
    // order, {start, end} (s_memrealtime, 100 MHz), {HW_ID, XCC_ID}, {tile,
    // the wave's largest step count}
    unsigned long long* wave_log;
#endif
};

// MODE: GEO_MODE_DIRECT / GEO_MODE_FAN / GEO_MODE_ADAPTIVE; KIND: geo::kCurvedOut/kCurvedIn/kFlat
// (frame-uniform integration kind, geo::geodesic_kind; ignored in fan mode).
// Max of v over the 64 lanes of a fully active wave (the same DPP scan).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Sum of v over the 64 lanes of a fully active wave (DPP inclusive scan:
// row_shr 1/2/4/8 within rows of 16, then row_bcast 15/31; lane 63 holds it).
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// The texel quad from the context's padded sky (geo::pad_sky): the 2 x 2 block
// at padded texel (ix0 + 1, iy0 + 1), by four buffer loads from one 32-bit
// byte offset (one v_mad_u32_u24): +4 B for the right column as the immediate
// offset, +pitch for the lower row as the scalar offset.  Against the wrap/clamp
// quad on the unpadded texture this drops the wrap and clamp selects, the
// quarter-rate v_mul_lo_u32 row products and the 64-bit address adds; the
// texels are the same (geo_set_sky limits the padded sky to < 2^31 bytes).
constexpr int kBufferRsrcWord3 = 0x00020000;  // gfx9 buffer resource: raw 32-bit dwords
struct PaddedSkyQuad {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t pitch_b;  // bytes per padded row, (sky_w + 2) * 4
    __device__ __forceinline__ void operator()(int ix0, int iy0, uint32_t (&t)[4]) const {
        const uint32_t off = __umul24((uint32_t)(iy0 + 1), pitch_b) + ((uint32_t)(ix0 + 1) << 2);
        t[0] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
        t[1] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4u, 0, 0);
        t[2] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, (int)pitch_b, 0);
        t[3] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4u, (int)pitch_b, 0);
    }
};

// A/B variant (GEO_SKY_PAIRS=1): level 0 also stored as row pairs
// (geo::pair_sky_rows), so a bilinear quad is 16 contiguous bytes, one
// buffer_load_dwordx4 and one 128-B line, where the row-major quad spans two
// rows, two lines.  Measured against PaddedSkyQuad: the fan draw -0.5 to
// -1 % (one box read the 1080p draw -8 %), config 3 +0.2 to +0.8 %, the ring
// overhead up by half a point (profiles/r06zk_sky_pairs_ab.txt,
// profiles/r06zl_sky_pairs_ab.txt), for a second copy of level 0 in device
// memory: not kept.
#if defined(GEO_SKY_PAIRS)
constexpr bool kSkyPairs = GEO_SKY_PAIRS != 0;
#else
constexpr bool kSkyPairs = false;
#endif
struct PairSkyQuad {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t base, pitch_b;  // the pairs' byte offset in the sky buffer; bytes per pair row, (sky_w + 2) * 8
    __device__ __forceinline__ void operator()(int ix0, int iy0, uint32_t (&t)[4]) const {
        const uint32_t off = base + __umul24((uint32_t)(iy0 + 1), pitch_b) + ((uint32_t)(ix0 + 1) << 3);
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
        t[0] = v[0];  // (x, y)
        t[2] = v[1];  // (x, y + 1)
        t[1] = v[2];  // (x + 1, y)
        t[3] = v[3];  // (x + 1, y + 1)
    }
};
__device__ __forceinline__ auto level0_quad(const RenderArgs& a) {
    if constexpr (kSkyPairs)
        return PairSkyQuad{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(a.sky), 0, (int)a.sky_total_bytes,
                                                             kBufferRsrcWord3),
                           a.sky_pairs_off, a.sky_pairs_pitch};
    else
        return PaddedSkyQuad{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(a.sky), 0, (int)a.sky_bytes,
                                                               kBufferRsrcWord3),
                             a.sky_pitch_b};
}

// The texel quad of one mip level of the padded chain (geo_ctx::sky): like
// PaddedSkyQuad at a per-lane level, so base and pitch are vector values.
struct LevelQuad {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t base, pitch_b;
    __device__ __forceinline__ void operator()(int ix0, int iy0, uint32_t (&t)[4]) const {
        const uint32_t off = base + __umul24((uint32_t)(iy0 + 1), pitch_b) + ((uint32_t)(ix0 + 1) << 2);
        t[0] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
        t[1] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4u, 0, 0);
        t[2] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + pitch_b, 0, 0);
        t[3] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + pitch_b + 4u, 0, 0);
    }
};

template <typename T>
__device__ __forceinline__ T level_sel(const T (&v)[geo::kSkyMipLevels], uint32_t l) {
    static_assert(geo::kSkyMipLevels == 4, "four levels");
    return l == 0u ? v[0] : (l == 1u ? v[1] : (l == 2u ? v[2] : v[3]));
}

// The trilinear sample (GEO_FLAG_MIPS, geo_pixel.h): levels floor(lambda) and
// the next, blended with frac(lambda) in 8 bits.  A zero weight returns
// level floor(lambda) alone: mip_blend(s0, s1, 0) == s0 bit for bit (each
// channel (256 s0 + 128) >> 8), so the second level is fetched only under the
// lanes that blend.  A wave magnified everywhere (rho2 <= 1, so lambda = 0,
// on every active lane: most of a 4K frame of a 4096 x 2048 sky) skips the
// level of detail and samples level 0 with its base and pitch as scalars, as
// the level-0 path does.
__device__ __forceinline__ uint32_t sample_trilinear(const RenderArgs& a, float rho2, float U, float V) {
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(a.sky), 0,
                                                                           (int)a.sky_total_bytes, kBufferRsrcWord3);
    if (geo::ballot_(rho2 > 1.0f) == 0)  // lod_q8 is 0 unless rho2 > 1
        return geo::sample_sky_quad_f(LevelQuad{rsrc, a.mip_off[0], a.mip_pitch[0]}, a.mip_w256[0], a.mip_h256[0], U,
                                      V);
    const uint32_t q = geo::lod_q8(rho2);
    const uint32_t l0 = q >> 8, f = q & 255u;
    const uint32_t s0 = geo::sample_sky_quad_f(LevelQuad{rsrc, level_sel(a.mip_off, l0), level_sel(a.mip_pitch, l0)},
                                               level_sel(a.mip_w256, l0), level_sel(a.mip_h256, l0), U, V);
    if (f == 0u) return s0;
    const uint32_t l1 = l0 + 1u < (uint32_t)geo::kSkyMipLevels ? l0 + 1u : l0;
    const uint32_t s1 = geo::sample_sky_quad_f(LevelQuad{rsrc, level_sel(a.mip_off, l1), level_sel(a.mip_pitch, l1)},
                                               level_sel(a.mip_w256, l1), level_sel(a.mip_h256, l1), U, V);
    return geo::mip_blend(s0, s1, f);
}

// The value of v in lane ^ 1 (DPP quad_perm [1, 0, 3, 2]) and in lane ^ 16
// (ds_swizzle, bit mode: and 0x1F, xor 0x10, within 32-lane halves): the
// x and y partners of the pixel's 2 x 2 quad in the 16 x 4 wave.
__device__ __forceinline__ float lane_xor1(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_xor16(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
}

// Epilogue of one pixel (shader.wgsl:88-105): black-hole test, sky UV,
// bilinear sample, blend and the optional outputs at index o.
// bh: the mask (lam < -7, or the band's f64 decision, GEO_FLAG_RING_F64).
__device__ __forceinline__ void shade_pixel_bh(const RenderArgs& a, const float* central_to_uv, float c2x, float c2y,
                                               float ct, float rct, float lam, bool bh, uint32_t steps, size_t o) {
    // A black-hole pixel is discarded (shader.wgsl:88): it needs its UV
    // only when the caller asks for it, so a wave inside the shadow skips
    // the sincos/atan2/asin and the sample (config 3 -0.3 %, config 5 -4.4 %)
    float U = 0.0f, V = 0.0f;
    if (!bh || a.out_uv)
        geo::sky_uv(central_to_uv, c2x, c2y, ct, rct, lam, &U, &V);
    const auto quad = level0_quad(a);
    if (a.composite) {
        // over the previous spheres; a discarded pixel keeps the target
        if (!bh) {
            const uint32_t s = geo::sample_sky_quad_f(quad, a.sky_w256, a.sky_h256, U, V);
            a.out_rgba[o] = a.sky_opaque ? s : geo::composite_(s, a.out_rgba[o]);
        }
    } else {
        a.out_rgba[o] = bh ? geo::kBlackRGBA : geo::sample_sky_qf(quad, a.sky_w256, a.sky_h256, a.sky_opaque != 0, U, V);
    }
    if (a.out_mask) a.out_mask[o] = bh ? 1 : 0;
    if (a.out_uv) a.out_uv[o] = make_float2(U, V);
    if (a.out_steps) a.out_steps[o] = steps;
}
__device__ __forceinline__ void shade_pixel(const RenderArgs& a, const float* central_to_uv, float c2x, float c2y,
                                            float ct, float rct, float lam, uint32_t steps, size_t o) {
    shade_pixel_bh(a, central_to_uv, c2x, c2y, ct, rct, lam, lam < geo::kBlackHoleLambda, steps, o);
}

// GEO_FLAG_RING_F64's kernel argument: the band's f64 constants (geo_band.h);
// empty in the other instantiations.
template <bool RING>
struct BandArg {};
template <>
struct BandArg<true> {
    geo::BandConsts k;
};
// The band's constants reach the band's lanes through LDS: the kernel copies
// them there from its argument segment at its start (one dword per thread,
// one barrier).  Kernel arguments are loaded at the kernel's entry and held
// in SGPRs to their last use: read in the band branch they took the kernel
// to 106 SGPRs (6 waves per SIMD instead of 8); from LDS they are loaded
// where the band's lanes use them.
constexpr uint32_t kBandDwords = (uint32_t)(sizeof(geo::BandConsts) / 4u);
// A ring render launches one wave per workgroup (the tile's four waves as
// four workgroups): a wave with band lanes lives two to three times as long
// as its tile's others, and a 4-wave workgroup keeps its finished waves'
// slots from the next workgroup until it ends (config 3 +8.4 -> +7.4 %,
// config 2 +15.0 -> +13.1 % over the plain frame, profiles/r06e_ring_wave_blocks_ab.txt).
constexpr bool kRingWaveBlocks = true;
// The same for a plain one-frame direct-mode render (tiles differ ~30x in
// cost, and its waves' lifetimes within a tile differ too): config 3
// -0.7 %, config 2 -1 % per frame; the adaptive mode measured +0.8 % and
// keeps 4-wave workgroups (profiles/r06h_all_wave_blocks_ab.txt)
constexpr bool kDirectWaveBlocks = true;
// The four waves of a tile on one XCD (its L2 holds the tile's sky lines):
// against four consecutive workgroups (on four XCDs), config 3 -0.6 to
// -0.8 %, config 2 -0.8 % (profiles/r06k_wave_block_layout_ab.txt)
#if defined(GEO_WB_XCD)
constexpr bool kWaveBlocksXcd = GEO_WB_XCD != 0;
#else
constexpr bool kWaveBlocksXcd = true;
#endif
#if defined(GEO_ADAPTIVE_WAVE_BLOCKS)  // A/B variant
constexpr bool kAdaptiveWaveBlocks = true;
#else
constexpr bool kAdaptiveWaveBlocks = false;
#endif
__host__ __device__ constexpr bool wave_blocks(int mode, bool mips, uint32_t nf, bool ring) {
    return (ring && kRingWaveBlocks && nf == 1) ||
           (!mips && nf == 1 &&
            ((kDirectWaveBlocks && mode == GEO_MODE_DIRECT) || (kAdaptiveWaveBlocks && mode == GEO_MODE_ADAPTIVE)));
}
#if defined(GEO_FAN_PERSIST)  // A/B variant: the fan-mode draw on a persistent grid
constexpr bool kFanPersist = true;
#else
constexpr bool kFanPersist = false;
#endif
// WB's 1-D grid for a launch of n tiles (n <= kMaxWaveBlockTiles: at most 2^31 workgroups)
constexpr uint32_t kMaxWaveBlockTiles = 1u << 26;
inline uint32_t wave_block_count(uint32_t n) { return kWaveBlocksXcd ? (n + 7u) / 8u * 32u : 4u * n; }
static_assert(sizeof(geo::BandConsts) % 8u == 0 && kBandDwords / 2u <= 64u, "one 8-byte word per thread");

// GEO_FLAG_MIPS epilogue: the pixel's UV and its quad footprint rho2 are
// known; the trilinear sample in place of the level-0 one.
__device__ __forceinline__ void shade_pixel_mips(const RenderArgs& a, float lam, float U, float V, float rho2,
                                                 uint32_t steps, size_t o) {
    const bool bh = lam < geo::kBlackHoleLambda;
    if (a.composite) {
        if (!bh) {
            const uint32_t s = sample_trilinear(a, rho2, U, V);
            a.out_rgba[o] = a.sky_opaque ? s : geo::composite_(s, a.out_rgba[o]);
        }
    } else {
        a.out_rgba[o] = bh ? geo::kBlackRGBA : geo::over_clear(sample_trilinear(a, rho2, U, V), a.sky_opaque != 0);
    }
    if (a.out_mask) a.out_mask[o] = bh ? 1 : 0;
    if (a.out_uv) a.out_uv[o] = make_float2(U, V);
    if (a.out_steps) a.out_steps[o] = steps;
}

// The pixel's traveled-angle result lambda' (pi/2 - angle) by mode.
template <int MODE, int KIND>
__device__ __forceinline__ float pixel_lambda(const RenderArgs& a, const geo::PixelConsts& k, float st, float ct,
                                              float rct, uint32_t* steps) {
    if constexpr (MODE == GEO_MODE_FAN) {
        *steps = 0;
        return geo::fan_lerp(a.fan, a.n_fan, st);
    } else if constexpr (MODE == GEO_MODE_ADAPTIVE) {
        return geo::kPi2 - geo::geodesic_angle_adaptive<KIND>(k, st, ct, rct, steps);
    } else {
        return geo::kPi2 - geo::geodesic_angle_v<KIND>(k, st, ct, rct, steps);
    }
}

// The scene constants of frame z of the launch.
template <uint32_t NF>
__device__ __forceinline__ const geo::PixelConsts& frame_consts(const RenderArgs& a, const FrameBatch<NF>& fb,
                                                                uint32_t z) {
    if constexpr (NF > 1)
        return fb.k[z];
    else
        return a.k;
}

// Pixels per lane: a fan-mode lane (level-0 sampler) draws two, rows
// kWaveRows apart, so one wave covers 16 x 8 pixels and each lane's loads of
// the second pixel overlap the first's (the fan lerp and the texel quads are
// the kernel's latency; its VALU work is short).  The mip-mapped fan draw
// measured the same either way (profiles/r03v_fan_mips_ab.txt) and keeps one.
// Four pixels per lane (a 32 x 32 tile, 47 VGPRs) measured the same as two
// (4K draw 0.0373 vs 0.0370 ms, 3 x 3 interleaved, profiles/r04g_fan_lr_ab.txt):
// the draw's waves are not short of independent work.
#if defined(GEO_FAN_LANE_ROWS)  // A/B variant
constexpr uint32_t kFanLaneRows = GEO_FAN_LANE_ROWS;
#else
constexpr uint32_t kFanLaneRows = 2;
#endif
__host__ __device__ constexpr uint32_t lane_rows(int mode, bool mips) {
    return mode == GEO_MODE_FAN && !mips ? kFanLaneRows : 1u;
}

// The fan-mode draw of one 32 x (8 LR) tile, LR pixels per lane (lane_rows)
// kWaveRows rows apart: every pixel's ray, then every fan lerp (2 LR loads in
// flight), then every epilogue.  Pixels k and k + 1 (k even) lie in one
// 8-row-aligned group of the wave's rows, so in one band (band heights are
// multiples of 8): the band mapping is per group, in scalar ops.
template <uint32_t LR>
__device__ __forceinline__ void fan_tile(const RenderArgs& a, const FrameK& f, size_t obase, uint2 tile, uint32_t wave,
                                         uint32_t lane) {
    static_assert(LR % 2 == 0 && LR * kWaveRows % 8 == 0, "pixel pairs fill 8-row groups");
    const uint32_t px = tile.x * kTileW + (wave % kWavesX) * kWaveW + lane % kWaveW;
    const uint32_t wl0 = tile.y * (kTileH * LR) + (wave / kWavesX) * (kWaveRows * LR);
    const uint32_t r = lane / kWaveW;
    uint32_t ly[LR], py[LR];
#pragma unroll
    for (uint32_t k = 0; k < LR; k += 2) {
        const uint32_t g0 = wl0 + (k / 2) * 8u;  // 8-row-aligned local row of pixels k, k + 1
        const uint32_t band = __umulhi(g0, a.band_magic);
        const uint32_t p0 = a.row0 + band * a.band_stride + (g0 - band * a.band_rows) + r;
        ly[k] = g0 + r;
        ly[k + 1] = g0 + r + kWaveRows;
        py[k] = p0;
        py[k + 1] = p0 + kWaveRows;
    }
#if defined(GEO_FAN_PROBE) && (GEO_FAN_PROBE & 4)  // diagnostic: the stores alone
#pragma unroll
    for (uint32_t k = 0; k < LR; ++k)
        if (px < a.width && ly[k] < a.nrows && py[k] < a.height) a.out_rgba[obase + (size_t)ly[k] * a.width + px] = py[k];
    return;
#endif
    float c2x[LR], c2y[LR], st[LR], ct[LR], rct[LR], lam[LR];
#pragma unroll
    for (uint32_t k = 0; k < LR; ++k) {
        float c2z;
        geo::pixel_central_dir(f.cam, f.frame.movement_to_central, f.frame.psi_factor_and_position[0], f.kt, px,
                               py[k], &c2x[k], &c2y[k], &c2z);
        st[k] = geo::central_sin(c2z);
        ct[k] = geo::central_rho(c2x[k], c2y[k]);
        rct[k] = geo::rcpf_(ct[k]);
    }
    geo::FanPos fp[LR];
#pragma unroll
    for (uint32_t k = 0; k < LR; ++k) fp[k] = geo::fan_pos(a.n_fan, st[k]);
#pragma unroll
    for (uint32_t k = 0; k < LR; ++k) {
#if defined(GEO_FAN_PROBE) && (GEO_FAN_PROBE & 2)  // diagnostic: no fan loads
        lam[k] = st[k] + fp[k].w;
#else
        lam[k] = geo::fan_at(a.fan, fp[k]);
#endif
    }
    bool in[LR], bh[LR];
    bool all_bh = true;
#pragma unroll
    for (uint32_t k = 0; k < LR; ++k) {
        in[k] = px < a.width && ly[k] < a.nrows && py[k] < a.height;
        bh[k] = lam[k] < geo::kBlackHoleLambda;
        all_bh = all_bh && bh[k];
    }
    if (!a.composite && !a.out_uv && !a.out_mask && !a.out_steps) {
        // the plain draw: every UV, then every texel quad (4 LR loads in
        // flight), then the stores; a wave with no sky pixel stores the
        // clear colour only
        uint32_t rgba[LR];
#pragma unroll
        for (uint32_t k = 0; k < LR; ++k) rgba[k] = geo::kBlackRGBA;
        if (geo::ballot_(!all_bh) != 0) {
            float U[LR], V[LR];
#pragma unroll
            for (uint32_t k = 0; k < LR; ++k)
                geo::sky_uv(f.frame.central_to_uv, c2x[k], c2y[k], ct[k], rct[k], lam[k], &U[k], &V[k]);
            const auto quad = level0_quad(a);
            uint32_t smp[LR];
#pragma unroll
            for (uint32_t k = 0; k < LR; ++k) {
#if defined(GEO_FAN_PROBE) && (GEO_FAN_PROBE & 1)  // diagnostic: no texel loads
                smp[k] = __float_as_uint(U[k]) ^ __float_as_uint(V[k]);
                (void)quad;
#elif defined(GEO_FAN_PROBE) && (GEO_FAN_PROBE & 8)  // diagnostic: every lane samples near one texel
                smp[k] = geo::sample_sky_quad_f(quad, a.sky_w256, a.sky_h256, 0.5f + U[k] * 1e-6f, 0.5f);
#else
                smp[k] = geo::sample_sky_quad_f(quad, a.sky_w256, a.sky_h256, U[k], V[k]);
#endif
            }
#pragma unroll
            for (uint32_t k = 0; k < LR; ++k)
                rgba[k] = bh[k] ? geo::kBlackRGBA : geo::over_clear(smp[k], a.sky_opaque != 0);
        }
#pragma unroll
        for (uint32_t k = 0; k < LR; ++k)
            if (in[k]) a.out_rgba[obase + (size_t)ly[k] * a.width + px] = rgba[k];
    } else {
#pragma unroll
        for (uint32_t k = 0; k < LR; ++k)
            if (in[k])
                shade_pixel(a, f.frame.central_to_uv, c2x[k], c2y[k], ct[k], rct[k], lam[k], 0u,
                            obase + (size_t)ly[k] * a.width + px);
    }
}

// NF: frames of the launch (FrameBatch; 1, or up to kMaxBatchFrames with the
// frame in blockIdx.z and its output a.out_frame_px pixels after the last's).
// RING: GEO_FLAG_RING_F64 (geo_band.h): the lanes of the capture-orbit band
// take their traveled angle from the f64 path instead of the f32 one.
template <int MODE, int KIND, bool MIPS, uint32_t NF, bool RING>
__global__ __launch_bounds__(kBlock) void geo_render_kernel(const RenderArgs a, const FrameBatch<NF> fb,
                                                            const BandArg<RING && NF == 1> bk) {
#if defined(GEO_WAVE_LOG)
    const unsigned long long t_wave0 = __builtin_amdgcn_s_memrealtime();
#endif
    constexpr uint32_t LR = lane_rows(MODE, MIPS);
    const uint32_t z = NF > 1 ? blockIdx.z : 0u;
    const FrameK& f = fb.f[z];
    const size_t obase = NF > 1 ? (size_t)z * a.out_frame_px : 0;
    // WB (wave_blocks): one wave per workgroup, on a 1-D grid: workgroup L
    // draws wave w of the tile at dispatch position p (p indexes the order,
    // or the launch's tiles row-major).  kWaveBlocksXcd: the hardware deals
    // workgroups to the 8 XCDs round-robin (L mod 8), so the four waves of a
    // tile are put 8 apart (p = 8 (L / 32) + L mod 8, w = (L / 8) mod 4) and
    // share their XCD's L2 for the tile's sky lines; the grid is padded to
    // whole groups of 8 tiles.  Otherwise p = L / 4, w = L mod 4.
    constexpr bool WB = wave_blocks(MODE, MIPS, NF, RING);
    uint32_t pos, wave;
    if constexpr (WB) {
        const uint32_t L = blockIdx.x;
        pos = kWaveBlocksXcd ? ((L >> 5) << 3) + (L & 7u) : L >> 2;
        wave = kWaveBlocksXcd ? (L >> 3) & 3u : L & 3u;
        if (pos >= a.launch_tiles) return;  // the padding of the last group (a whole workgroup)
    } else {
        pos = blockIdx.y * gridDim.x + blockIdx.x;
        wave = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
    }
    const uint32_t tiles_x = WB ? a.tiles_x : gridDim.x;
    uint2 tile;
    if (a.tile_order) {
        const uint32_t t = a.tile_order[pos];  // one scalar load
        tile = make_uint2(t & 0xFFFFu, t >> 16);
    } else if constexpr (WB) {
        tile = make_uint2(pos % tiles_x, a.tile_y0 + pos / tiles_x);
    } else {
        tile = make_uint2(blockIdx.x, a.tile_y0 + blockIdx.y);
    }
    const uint32_t lane = threadIdx.x & 63u;
    // RING: the band's constants in LDS (kBandDwords): a one-frame launch
    // copies them from its kernel arguments; a batched launch (RB) derives
    // frame z's in a wave's own slot when the wave has band lanes
    constexpr bool RB = RING && NF > 1;
    __shared__ double band_lds[RING ? (RB ? kBlock / 64u : 1u) * (kBandDwords / 2u) : 1u];
    if constexpr (RING && NF == 1) {
        // one 8-byte word per thread (kBandDwords / 2 <= 64)
        if (threadIdx.x < kBandDwords / 2u)
            reinterpret_cast<uint2*>(band_lds)[threadIdx.x] = reinterpret_cast<const uint2*>(&bk.k)[threadIdx.x];
        __syncthreads();
    }
    const uint32_t px = tile.x * kTileW + (wave % kWavesX) * kWaveW + lane % kWaveW;
    // local row -> frame row.  band_rows is a multiple of 8 (checked on the
    // host): each wave's rows (at most 8) lie in one band and the mapping is
    // wave-uniform (scalar ops; the band index by a multiply-high,
    // band_rows_magic).
    const uint32_t wl0 = tile.y * (kTileH * LR) + (wave / kWavesX) * (kWaveRows * LR);
    const uint32_t ly = wl0 + lane / kWaveW;
    const uint32_t band = __umulhi(wl0, a.band_magic);
    const uint32_t py = a.row0 + band * a.band_stride + (wl0 - band * a.band_rows) + (ly - wl0);
    uint32_t steps = 0;
    uint32_t cost_scale = 1u;  // RING: 2 on the band's lanes (their steps are f64)
    (void)cost_scale;
    const bool in_frame = px < a.width && ly < a.nrows && py < a.height;
    if constexpr (LR > 1) {
        if constexpr (kFanPersist) {
            // a persistent grid (its tiles all cost the same): workgroup b
            // draws tiles b, b + G, ... of the launch
            for (uint32_t t = blockIdx.x; t < a.launch_tiles; t += gridDim.x)
                fan_tile<LR>(a, f, obase, make_uint2(t % a.tiles_x, a.tile_y0 + t / a.tiles_x), wave, lane);
        } else {
            fan_tile<LR>(a, f, obase, tile, wave, lane);
        }
    } else if constexpr (!MIPS) {
        if (in_frame) {
            float c2x, c2y, c2z;
            geo::pixel_central_dir(f.cam, f.frame.movement_to_central, f.frame.psi_factor_and_position[0], f.kt, px,
                                   py, &c2x, &c2y, &c2z);
            const float st = geo::central_sin(c2z);
            const float ct = geo::central_rho(c2x, c2y);
            const float rct = geo::rcpf_(ct);  // shared by the ray's 1/b^2 and its sky direction
            if constexpr (RING) {
                // the band's lanes skip the f32 integration (its loop runs on
                // the other lanes) and take lambda' and the mask from the f64
                // path; both then draw the sky from the f32 ray
                double* const bslot = band_lds + (RB ? wave * (kBandDwords / 2u) : 0u);
                const geo::BandConsts& bkl = *reinterpret_cast<const geo::BandConsts*>(bslot);
                float kx;
                if constexpr (RB)
                    kx = fb.ring_kx[z];
                else
                    kx = bkl.kx;
                const bool band = geo::in_band(kx, ct);
#if defined(GEO_RING_PRIO)  // A/B variant: a wave with band lanes issues first
                if (geo::ballot_(band) != 0) __builtin_amdgcn_s_setprio(GEO_RING_PRIO);
#endif
                float lam = 0.0f;
                bool bh = false;
                if (!band) {
                    lam = pixel_lambda<MODE, KIND>(a, frame_consts(a, fb, z), st, ct, rct, &steps);
                    bh = lam < geo::kBlackHoleLambda;
                }
                if (geo::ballot_(band) != 0) {
                    if constexpr (RB) {
                        // frame z's constants, written by the wave's first
                        // active lane (lanes outside the frame are off here)
                        // into the wave's slot (the same f64 operations as the
                        // host's geo::band_consts), then read by the band's lanes
                        if (lane == (uint32_t)__builtin_amdgcn_readfirstlane((int)lane)) {
                            const geo::PixelConsts& kz = fb.k[z];
                            geo::band_consts_into(*reinterpret_cast<geo::BandConsts*>(bslot), f.frame, kz.rs,
                                                  kz.sphere_r, kz.r, kz.step, kz.max_steps, a.width, a.height);
                        }
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                    if (band) {
                        GEO_COLD_ARM();
                        const double l = geo::band_lambda(bkl, px, py, &steps);
                        lam = (float)l;
                        bh = l < (double)geo::kBlackHoleLambda;
                        cost_scale = 2u;  // an f64 step issues as two f32 ones
                    }
                }
                shade_pixel_bh(a, f.frame.central_to_uv, c2x, c2y, ct, rct, lam, bh, steps,
                               obase + (size_t)ly * a.width + px);
            } else {
                const float lam = pixel_lambda<MODE, KIND>(a, frame_consts(a, fb, z), st, ct, rct, &steps);
                shade_pixel(a, f.frame.central_to_uv, c2x, c2y, ct, rct, lam, steps,
                            obase + (size_t)ly * a.width + px);
            }
        }
    } else {
        // Every lane traces its pixel, the ones outside the frame or the
        // requested rows too (the helpers of the frame-aligned 2 x 2 quads,
        // as a fragment shader's): the footprint needs all four UVs of a quad.
        // Black-hole pixels keep their UV as well (textureSample runs before
        // the discard, shader.wgsl:101-104).
        float c2x, c2y, c2z;
        geo::pixel_central_dir(f.cam, f.frame.movement_to_central, f.frame.psi_factor_and_position[0], f.kt, px, py,
                               &c2x, &c2y, &c2z);
        const float st = geo::central_sin(c2z);
        const float ct = geo::central_rho(c2x, c2y);
        const float rct = geo::rcpf_(ct);
        const float lam = pixel_lambda<MODE, KIND>(a, frame_consts(a, fb, z), st, ct, rct, &steps);
        // A pixel's UV is read by its own sample and by its quad partners'
        // footprints, all in this wave: a wave wholly inside the shadow reads
        // none (unless the caller asks for UV) and skips the UV and the
        // footprint (a wave-uniform branch)
        float U = 0.0f, V = 0.0f, rho2 = 0.0f;
        if (geo::ballot_(!(lam < geo::kBlackHoleLambda)) != 0 || a.out_uv) {
            geo::sky_uv(f.frame.central_to_uv, c2x, c2y, ct, rct, lam, &U, &V);
            const float ux = lane_xor1(U), vx = lane_xor1(V), uy = lane_xor16(U), vy = lane_xor16(V);
            rho2 = geo::mip_rho2(U - ux, V - vx, U - uy, V - vy, a.sky_wf, a.sky_hf);
        }
        if (in_frame)
            shade_pixel_mips(a, lam, U, V, rho2, steps, obase + (size_t)ly * a.width + px);
        else
            steps = 0;
    }
    if constexpr (MODE != GEO_MODE_FAN) {
        if (a.step_slots) {
            // One atomic per wave (all 64 lanes active here; a wave's sum fits
            // u32: 64 x 2^20 steps at most) into one of kStepSlots sharded
            // slots.  No block barrier, so a wave that finishes early frees
            // its slot at once.
            const uint32_t total = wave_sum_u32(steps);
            const uint32_t slot = (tile.x * (kBlock / 64) + wave) % kStepSlots;
            if ((threadIdx.x & 63) == 0 && total)
                atomicAdd(&a.step_slots[slot * kSlotStride], (unsigned long long)total);
        }
        if (a.tile_cost && z == 0u) {
            // a wave holds its slot until its slowest lane stops: the tile's
            // cost is the sum of its waves' largest step counts (frame 0's
            // of a batch: the order is per tile)
            // (RING: a wave runs its f32 lanes' loop, then its band lanes'
            // f64 loop at about twice the cost per step)
            const uint32_t wmax = RING ? wave_max_u32(cost_scale == 1u ? steps : 0u) +
                                             2u * wave_max_u32(cost_scale == 1u ? 0u : steps)
                                       : wave_max_u32(steps);
            if ((threadIdx.x & 63) == 0)
                atomicAdd(&a.tile_cost[tile.y * tiles_x + tile.x], wmax + a.cost_overhead);
        }
    }
#if defined(GEO_WAVE_LOG)
    if (a.wave_log) {
        const uint32_t wmax = wave_max_u32(steps);
        const unsigned long long t_wave1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) {
            const size_t wg = (size_t)blockIdx.z * (WB ? a.launch_tiles : gridDim.x * gridDim.y) + pos;  // the tile, in launch order
            unsigned long long* p = a.wave_log + (wg * (kBlock / 64) + wave) * 4;
            const uint32_t hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);    // HW_REG_XCC_ID[3:0]
            p[0] = t_wave0;
            p[1] = t_wave1;
            p[2] = hw_id | ((unsigned long long)xcc << 32);
            p[3] = (tile.x | (tile.y << 16)) | ((unsigned long long)wmax << 32);
        }
    }
#endif
}

// ---- longest-first dispatch: the order from recorded tile costs ---------
// Cost classes of an eighth of an octave (the octave and the next three
// bits of the cost, 256 classes), dispatched from the highest class down;
// within a class, tile order.  Two
// kernels: per-chunk class histograms, then each chunk's tiles scattered to
// their positions (and their costs cleared for the next recording).
// eighth-octave classes: on an 8-rank share of the 4K frame the learned
// order runs 0.0316 ms against 0.0325 with half octaves and 0.0314 for the
// exact LPT order (profiles/r04e_cost_class_ab.txt)
constexpr uint32_t kSubOctaveBits = 3;
constexpr int kCostClasses = 32 << kSubOctaveBits;
constexpr uint32_t kOrderChunk = 1024;  // tiles per workgroup

// class = (octave << bits) + the top `bits` mantissa bits below the leading one
__device__ __forceinline__ uint32_t cost_class(uint32_t c) {
    if (c == 0u) return 0u;
    const uint32_t o = 31u - (uint32_t)__clz(c);
    const uint32_t m = (c << (31u - o)) >> (31u - kSubOctaveBits) & ((1u << kSubOctaveBits) - 1u);
    return (o << kSubOctaveBits) + m;
}

__global__ __launch_bounds__(256) void geo_order_hist(const uint32_t* __restrict__ cost, uint32_t n,
                                                      uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kCostClasses];
    if (threadIdx.x < kCostClasses) h[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t lo = blockIdx.x * kOrderChunk, hi = min(n, lo + kOrderChunk);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += 256u) atomicAdd(&h[cost_class(cost[i])], 1u);
    __syncthreads();
    if (threadIdx.x < kCostClasses) hist[blockIdx.x * kCostClasses + threadIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(256) void geo_order_scatter(uint32_t* __restrict__ cost, uint32_t n,
                                                         const uint32_t* __restrict__ hist, uint32_t tiles_x,
                                                         uint32_t* __restrict__ order) {
    __shared__ uint32_t tot[kCostClasses], base[kCostClasses];
    const uint32_t c = threadIdx.x;
    if (c < kCostClasses) {
        uint32_t t = 0u, mine = 0u;
        for (uint32_t g = 0; g < gridDim.x; ++g) {
            const uint32_t v = hist[g * kCostClasses + c];
            t += v;
            if (g < blockIdx.x) mine += v;
        }
        tot[c] = t;
        base[c] = mine;
    }
    __syncthreads();
    if (c < kCostClasses) {
        uint32_t above = 0u;  // tiles of the higher classes, dispatched first
        for (uint32_t k = c + 1u; k < (uint32_t)kCostClasses; ++k) above += tot[k];
        base[c] += above;
    }
    __syncthreads();
    const uint32_t lo = blockIdx.x * kOrderChunk, hi = min(n, lo + kOrderChunk);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += 256u) {
        const uint32_t pos = atomicAdd(&base[cost_class(cost[i])], 1u);
        order[pos] = ((i / tiles_x) << 16) | (i % tiles_x);
        cost[i] = 0u;
    }
}

// Frame row y of frame f comes from rank r = (y / band_rows) % world, local
// row ((y / band_rows) / world) * band_rows + y % band_rows of that rank's
// packed bands (geo_render_bands' layout).  One thread per 16 B (W % 4 == 0)
// or per pixel.
template <typename T>
__global__ __launch_bounds__(256) void geo_assemble_kernel(const uint8_t* __restrict__ src, size_t rank_stride,
                                                           size_t frame_stride, uint32_t world, uint32_t band_rows,
                                                           uint32_t row_units, uint32_t height,
                                                           uint8_t* __restrict__ dst) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    const uint32_t y = blockIdx.y;
    const uint32_t f = blockIdx.z;
    if (x >= row_units) return;
    const uint32_t b = y / band_rows;
    const uint32_t r = b % world;
    const size_t lrow = (size_t)(b / world) * band_rows + y % band_rows;
    const size_t row_bytes = (size_t)row_units * sizeof(T);
    const T* s = reinterpret_cast<const T*>(src + r * rank_stride + f * frame_stride + lrow * row_bytes);
    T* d = reinterpret_cast<T*>(dst + ((size_t)f * height + y) * row_bytes);
    d[x] = s[x];
}

// The same from RGB24-packed bands (geo_pack_rgb; alpha restored to 255):
// one thread per 4 pixels (12 B in, 16 B out), W % 4 == 0.
__global__ __launch_bounds__(256) void geo_assemble_rgb_kernel(const uint8_t* __restrict__ src, size_t rank_stride,
                                                               size_t frame_stride, uint32_t world,
                                                               uint32_t band_rows, uint32_t quads, uint32_t height,
                                                               uint8_t* __restrict__ dst) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    const uint32_t y = blockIdx.y;
    const uint32_t f = blockIdx.z;
    if (x >= quads) return;
    const uint32_t b = y / band_rows;
    const uint32_t r = b % world;
    const size_t lrow = (size_t)(b / world) * band_rows + y % band_rows;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src + r * rank_stride + f * frame_stride +
                                                         lrow * (size_t)quads * 12u) + 3u * x;
    const uint32_t w0 = s[0], w1 = s[1], w2 = s[2];  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
    uint4 o;
    o.x = (w0 & 0x00FFFFFFu) | 0xFF000000u;
    o.y = (w0 >> 24) | ((w1 & 0xFFFFu) << 8) | 0xFF000000u;
    o.z = (w1 >> 16) | ((w2 & 0xFFu) << 16) | 0xFF000000u;
    o.w = (w2 >> 8) | 0xFF000000u;
    reinterpret_cast<uint4*>(dst + ((size_t)f * height + y) * (size_t)quads * 16u)[x] = o;
}

// The lead layout (geo_assemble_lead): cycles of lead*band_rows rows of rank 0
// followed by one band_rows band per peer.  QUAD: one thread per 4 pixels
// (16 B out; peers' rows RGBA8 or RGB24), else one per pixel (RGBA8 only).
// The row's source (rank 0's own bands or a peer's) is block-uniform.
template <bool QUAD>
__global__ __launch_bounds__(256) void geo_assemble_lead_kernel(
    const uint8_t* __restrict__ lead_src, size_t lead_frame_stride, uint32_t lead_rows,
    const uint8_t* __restrict__ src, size_t rank_stride, size_t frame_stride, uint32_t world, uint32_t band_rows,
    uint32_t units, uint32_t height, uint32_t src_bpp, uint8_t* __restrict__ dst) {
    using T = typename std::conditional<QUAD, uint4, uint32_t>::type;
    constexpr uint32_t kPix = QUAD ? 4u : 1u;  // pixels per unit
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    const uint32_t y = blockIdx.y;
    const uint32_t f = blockIdx.z;
    if (x >= units) return;
    const uint32_t cycle = lead_rows + (world - 1u) * band_rows;
    const uint32_t c = y / cycle, off = y % cycle;
    const size_t rgba_row = (size_t)units * sizeof(T);
    T* d = reinterpret_cast<T*>(dst + ((size_t)f * height + y) * rgba_row);
    if (off < lead_rows) {
        const size_t lrow = (size_t)c * lead_rows + off;
        d[x] = reinterpret_cast<const T*>(lead_src + f * lead_frame_stride + lrow * rgba_row)[x];
        return;
    }
    const uint32_t o2 = off - lead_rows;
    const uint32_t r = 1u + o2 / band_rows;
    const size_t lrow = (size_t)c * band_rows + o2 % band_rows;
    const uint8_t* row = src + r * rank_stride + f * frame_stride + lrow * (size_t)units * kPix * src_bpp;
    if constexpr (QUAD) {
        if (src_bpp == 3u) {
            const uint32_t* s = reinterpret_cast<const uint32_t*>(row) + 3u * x;
            const uint32_t w0 = s[0], w1 = s[1], w2 = s[2];  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
            uint4 o;
            o.x = (w0 & 0x00FFFFFFu) | 0xFF000000u;
            o.y = (w0 >> 24) | ((w1 & 0xFFFFu) << 8) | 0xFF000000u;
            o.z = (w1 >> 16) | ((w2 & 0xFFu) << 16) | 0xFF000000u;
            o.w = (w2 >> 8) | 0xFF000000u;
            d[x] = o;
            return;
        }
    }
    d[x] = reinterpret_cast<const T*>(row)[x];
}

// RGBA8 -> RGB24 (alpha dropped: every frame pixel is opaque after the clear),
// 4 pixels per thread.
__global__ __launch_bounds__(256) void geo_pack_rgb_kernel(const uint4* __restrict__ src, uint64_t quads,
                                                           uint32_t* __restrict__ dst) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= quads) return;
    const uint4 p = src[i];
    uint32_t* d = dst + 3u * i;
    d[0] = (p.x & 0x00FFFFFFu) | (p.y << 24);
    d[1] = ((p.y >> 8) & 0xFFFFu) | (p.z << 16);
    d[2] = ((p.z >> 16) & 0xFFu) | (p.w << 8);
}

__global__ __launch_bounds__(kStepSlots) void geo_steps_finalize(unsigned long long* slots,
                                                                  unsigned long long* total) {
    __shared__ unsigned long long s[kStepSlots / 64];
    const int i = threadIdx.x;
    unsigned long long v = slots[i * kSlotStride];
    slots[i * kSlotStride] = 0;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((i & 63) == 0) s[i >> 6] = v;
    __syncthreads();
    if (i == 0) {
        unsigned long long t = 0;
        for (int j = 0; j < kStepSlots / 64; ++j) t += s[j];
        *total += t;
    }
}

// f64 restatement of SphereRayTracer::solve_geodesic (sphere_ray_tracer.rs:60-193),
// operation for operation (no contraction).  The radial cases and
// pre-filters (:60-119): false with the result in *early, else the initial
// u' (:123).
__device__ bool solve_geodesic_f64_init(double sphere_r, double schwarz_r, double r, double energy, double rotation,
                                        bool r_falling, double* early, double* u_bar0) {
    const double NO_VALUE = GEO_NO_VALUE;
    const double PI = 3.14159265358979323846;
    const double b = rotation / energy;
    const bool outside = r > schwarz_r;
    const bool sphere_outside = sphere_r > schwarz_r;
    const bool inside_sphere = r < sphere_r;
    if (rotation < 1e-10) {
        if (inside_sphere) {
            if (outside)
                *early = r_falling ? (schwarz_r == 0. ? PI : NO_VALUE) : 0.;
            else
                *early = sphere_outside ? (energy > 0. ? 0. : NO_VALUE) : 0.;
        } else {
            *early = (sphere_outside && r_falling) ? 0. : NO_VALUE;
        }
        return false;
    }
    const bool barrier_3r_2 = (schwarz_r > 0.) && 1. / (b * b) < 4. / (27. * schwarz_r * schwarz_r);
    const double r3_2 = 3. * schwarz_r / 2.;
    const bool different_sides_3r_2 = ((r < r3_2) != (sphere_r < r3_2)) && fabs(r - r3_2) > 1e-10;
    if ((inside_sphere && !sphere_outside) || (!outside && sphere_outside && energy < 0.) ||
        (barrier_3r_2 && different_sides_3r_2) || (r < r3_2 && inside_sphere && r_falling) ||
        (r > r3_2 && !inside_sphere && !r_falling)) {
        *early = NO_VALUE;
        return false;
    }
    *u_bar0 = (r_falling ? 1. : -1.) * sqrt(1. / (b * b) - (1. - schwarz_r / r) / (r * r));
    return true;
}

// The f64 solve (sphere_ray_tracer.rs:121-193), restructured for latency.
// A fan is one lane per node, 400 lanes = 7 waves, so its time is
// the longest node's dependent chain: the literal loop spends ~60 f64
// instructions per step (two f64 divisions by 6 among them), this one the
// scaled 14-op RK4 of the f32 kernel (geo_pixel.h rk4_step) in f64 --
// U = c u, c = 3 rs/2 (1 for rs = 0), F(U) = U(U - 1) (-U in flat space),
// the thresholds scaled alike, Newton's ratio scale-free.  It is the same
// algorithm (stages, tests, Newton) with a different rounding of the f64
// intermediates: the fan agrees with the literal f64 restatement to within
// one f32 ulp (tests/test_gpu_parity.py, the fan tolerance).
template <bool FLAT>
__device__ __forceinline__ double fan_F(double U) {
    return FLAT ? -U : __builtin_fma(U, U, -U);
}
template <bool FLAT>
__device__ __forceinline__ void fan_rk4(double U, double V, double h, double hh, double hh2, double hhh, double h6,
                                        double h2_6, double* NU, double* NV) {
    const double fu = fan_F<FLAT>(U);
    const double au = __builtin_fma(hh, V, U);
    const double uh = __builtin_fma(h, V, U);
    const double fa = fan_F<FLAT>(au);
    const double bu = __builtin_fma(hh2, fu, au);
    const double fb = fan_F<FLAT>(bu);
    const double cu = __builtin_fma(hhh, fa, uh);
    const double fc = fan_F<FLAT>(cu);
    const double fab = fa + fb;
    *NU = __builtin_fma(h2_6, fu + fab, uh);
    *NV = __builtin_fma(h6, __builtin_fma(2.0, fab, fu) + fc, V);
}
// One step of the literal loop's tests (:134, :150, :184) from (U, V) to
// (NU, NV): 0 continue, 1 crossing (Newton), 2 stop without a value.
template <bool FLAT>
__device__ __forceinline__ int fan_test(double U, double V, double NU, double SU, double BD, double HU) {
    if (!FLAT && U > HU && V > 0.) return 2;  // the loop test on the pre-step state (:134)
    if ((NU > SU) != (U > SU)) return 1;
    if (NU < BD) return 2;
    return 0;
}
// A lane's chain of RK4 steps is the fan's critical path, so the exit branch
// (which waits for the newest state's compares) is taken once per kFanGroup
// steps: the group's flags are formed without branches, and a group that
// stops is replayed step by step from its start (the same arithmetic, so the
// same result as testing every step).  Groups of 8 and 16 are +-4 % and up
// to +22 %.
constexpr int kFanGroup = 4;
template <bool FLAT>
__device__ double fan_integrate(double sphere_r, double schwarz_r, uint32_t max_iter, double step, double r,
                                double u_bar0) {
    const double NO_VALUE = GEO_NO_VALUE;
    const double r3_2 = 3. * schwarz_r / 2.;
    const double c = FLAT ? 1. : r3_2;
    const double u0 = 1. / r;
    const double SU = c / sphere_r;                                      // sphere_u
    const double BD = c * (0.9 * fmin(u0, 1. / fmax(sphere_r, r3_2)));  // bound
    const double HU = FLAT ? __builtin_inf() : c / schwarz_r;           // schwarz_u
    const double h = step, hh = step / 2., hh2 = step * step / 4., hhh = step * step / 2., h6 = step / 6.,
                 h2_6 = step * step / 6.;
    double U = c * u0, V = c * u_bar0;
    if (!(U > 0.)) return NO_VALUE;
    double angle = 0.;
    uint32_t it = 0;
    // whole groups while the budget allows; a stopping group falls through
    // to the per-step loop below from its start state
    while (it + kFanGroup <= max_iter) {
        double su[kFanGroup + 1], sv[kFanGroup + 1];
        su[0] = U;
        sv[0] = V;
        bool stop = false;
#pragma unroll
        for (int j = 0; j < kFanGroup; ++j) {
            fan_rk4<FLAT>(su[j], sv[j], h, hh, hh2, hhh, h6, h2_6, &su[j + 1], &sv[j + 1]);
            stop |= fan_test<FLAT>(su[j], sv[j], su[j + 1], SU, BD, HU) != 0;
        }
        if (stop) break;
        U = su[kFanGroup];
        V = sv[kFanGroup];
#pragma unroll
        for (int j = 0; j < kFanGroup; ++j) angle += step;  // the literal accumulation (:190)
        it += kFanGroup;
    }
    for (; it < max_iter; ++it) {
        double NU, NV;
        fan_rk4<FLAT>(U, V, h, hh, hh2, hhh, h6, h2_6, &NU, &NV);
        const int t = fan_test<FLAT>(U, V, NU, SU, BD, HU);
        if (t == 2) return NO_VALUE;
        if (t == 1) {
            // Newton on the step length from the steeper end (:150-182)
            double ns, wu, wv;
            if (fabs(V) > fabs(NV)) {
                ns = 0.;
                wu = U;
                wv = V;
            } else {
                ns = h;
                wu = NU;
                wv = NV;
            }
            for (int n = 0; n < 3; ++n) {
                ns -= (wu - SU) / wv;
                const double n2 = ns * ns;
                fan_rk4<FLAT>(U, V, ns, ns / 2., n2 / 4., n2 / 2., ns / 6., n2 / 6., &wu, &wv);
            }
            return angle + ns;
        }
        U = NU;
        V = NV;
        angle += step;
    }
    // budget exhausted; the literal loop re-tests the final state only
    // against :134 and `u > 0`, both of which end without a value too
    return NO_VALUE;
}

__global__ void geo_fan_kernel(double sphere_r, double schwarz_r, uint32_t max_iter, double step,
                               uint32_t n, double r, float* fan) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double PI = 3.14159265358979323846;
    const double FRAC_PI_2 = 1.57079632679489661923;
    // solve_ray_fan (sphere_ray_tracer.rs:37-53)
    const double theta = FRAC_PI_2 - PI * (double)i / ((double)n - 1.);
    const double rotation = r * cos(theta);
    bool r_falling;
    double energy;
    if (r < schwarz_r) {
        r_falling = false;
        energy = sin(-theta) * sqrt(-1. + schwarz_r / r);
    } else {
        r_falling = theta > 0.;
        energy = sqrt(1. - schwarz_r / r);
    }
    double angle, u_bar0;
    if (solve_geodesic_f64_init(sphere_r, schwarz_r, r, energy, rotation, r_falling, &angle, &u_bar0)) {
        angle = schwarz_r == 0. ? fan_integrate<true>(sphere_r, schwarz_r, max_iter, step, r, u_bar0)
                                : fan_integrate<false>(sphere_r, schwarz_r, max_iter, step, r, u_bar0);
    }
    fan[i] = (float)(FRAC_PI_2 - angle);
}

}  // namespace


extern "C" {

int geo_abi_version(void) { return GEO_ABI_VERSION; }

const char* geo_status_str(int status) {
    switch (status) {
        case GEO_OK: return "ok";
        case GEO_EINVAL: return "invalid argument";
        case GEO_EHIP: return "HIP runtime error";
        case GEO_ENOMEM: return "out of memory";
        case GEO_ENODEV: return "no such HIP device";
        case GEO_ESTATE: return "call out of order";
        default: return "unknown status";
    }
}

// The context's ordering events: no timestamps, and no system-scope fence
// (they order device work on one device and let the host wait for it; a
// system-scope release after every render writes back the caches again and
// cost ~2 % per 4K frame)
constexpr unsigned kCtxEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;

int geo_ctx_create(int device, geo_ctx** out) {
    if (!out) return GEO_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return GEO_ENODEV;
    DeviceGuard g(device);
    if (!g.ok) return GEO_EHIP;
    geo_ctx* c = new (std::nothrow) geo_ctx();
    if (!c) return GEO_ENOMEM;
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete c;
        return GEO_EHIP;
    }
    c->num_cus = prop.multiProcessorCount;
    c->fan_cur = -1;
    bool ok = true;
    for (int b = 0; b < 2 && ok; ++b)
        ok = hipEventCreateWithFlags(&c->fan_written[b], kCtxEventFlags) == hipSuccess &&
             hipEventCreateWithFlags(&c->fan_read[b], kCtxEventFlags) == hipSuccess;
    for (int i = 0; i < geo_ctx::kStepCallSets && ok; ++i)
        ok = hipEventCreateWithFlags(&c->step_set_free[i], kCtxEventFlags) == hipSuccess;
    for (int i = 0; i < geo_ctx::kRenderStreams && ok; ++i)
        ok = hipEventCreateWithFlags(&c->render_done[i], kCtxEventFlags) == hipSuccess;
    if (ok) ok = hipEventCreateWithFlags(&c->order_written, kCtxEventFlags) == hipSuccess;
    c->dispatch_mode = GEO_DISPATCH_LONGEST_FIRST;
    c->dispatch_period = kDefaultDispatchPeriod;
    c->order_cur = -1;
    int st = ok ? GEO_OK : GEO_EHIP;
    if (ok && hipMalloc(&c->step_slots, sizeof(unsigned long long) * kSlotSetU64 * kSlotSets) != hipSuccess) {
        c->step_slots = nullptr;
        st = GEO_ENOMEM;
    }
    if (st == GEO_OK &&
        hipMemset(c->step_slots, 0, sizeof(unsigned long long) * kSlotSetU64 * kSlotSets) != hipSuccess)
        st = GEO_EHIP;
    if (st != GEO_OK) {
        if (c->step_slots) (void)hipFree(c->step_slots);
        for (int b = 0; b < 2; ++b) {
            if (c->fan_written[b]) (void)hipEventDestroy(c->fan_written[b]);
            if (c->fan_read[b]) (void)hipEventDestroy(c->fan_read[b]);
        }
        for (int i = 0; i < geo_ctx::kStepCallSets; ++i)
            if (c->step_set_free[i]) (void)hipEventDestroy(c->step_set_free[i]);
        for (int i = 0; i < geo_ctx::kRenderStreams; ++i)
            if (c->render_done[i]) (void)hipEventDestroy(c->render_done[i]);
        if (c->order_written) (void)hipEventDestroy(c->order_written);
        delete c;
        return st;
    }
    *out = c;
    return GEO_OK;
}

// The context's renders (and step flushes) in flight, on every stream it has
// rendered on: after this, nothing of the context's reads the sky, the fan
// buffers or the step counters.
static int wait_renders(geo_ctx* c) {
    for (int i = 0; i < c->n_render_streams; ++i)
        if (hipEventSynchronize(c->render_done[i]) != hipSuccess) return GEO_EHIP;
    return GEO_OK;
}

// The fan buffer b's last writer and readers (geo_ctx: the chained event and
// the slots of the draws that recorded none).
static int wait_fan(geo_ctx* c, int b) {
    if (c->fan_written_rec[b] && hipEventSynchronize(c->fan_written[b]) != hipSuccess) return GEO_EHIP;
    if (c->fan_read_rec[b] && hipEventSynchronize(c->fan_read[b]) != hipSuccess) return GEO_EHIP;
    for (int i = 0; i < c->n_render_streams; ++i)
        if ((c->fan_read_slots[b] >> i & 1u) && hipEventSynchronize(c->render_done[i]) != hipSuccess) return GEO_EHIP;
    return GEO_OK;
}

// Buffer b holds no pending writer or reader (after a host wait for them).
static void fan_forget(geo_ctx* c, int b) {
    c->fan_written_rec[b] = c->fan_read_rec[b] = false;
    c->fan_writer[b] = c->fan_reader[b] = nullptr;
    c->fan_read_slots[b] = 0;
}

// The slot whose event tracks the context's work on stream s
// (geo_ctx::render_done): the caller's next kernel on s records it as its stop
// event (hipExtLaunchKernelGGL), which rides on the dispatch's own completion
// signal instead of a marker packet after it (a marker per frame cost ~1 % of
// the event-timed 4K kernel).  With every slot taken, the least recently
// claimed one is evicted after a HOST wait for its event (a
// device-side wait would tie the caller's stream to an unrelated stream's
// work, which may sit behind a collective); that wait is the only blocking
// step, and only a context rendering on more than kRenderStreams streams
// reaches it.  -1 on a HIP error.
static int render_slot(geo_ctx* c, hipStream_t s) {
    int i = 0;
    while (i < c->n_render_streams && c->render_stream[i] != s) ++i;
    if (i == c->n_render_streams) {
        if (c->n_render_streams < geo_ctx::kRenderStreams) {
            ++c->n_render_streams;
        } else {
            i = c->render_next;
            c->render_next = (i + 1) % geo_ctx::kRenderStreams;
            if (hipEventSynchronize(c->render_done[i]) != hipSuccess) return -1;
            // the evicted stream's draws are done: no fan buffer waits for them
            for (int b = 0; b < 2; ++b) c->fan_read_slots[b] &= ~(1u << i);
        }
        c->render_stream[i] = s;
    }
    return i;
}

static hipEvent_t render_event(geo_ctx* c, hipStream_t s) {
    const int i = render_slot(c, s);
    return i < 0 ? nullptr : c->render_done[i];
}

void geo_ctx_destroy(geo_ctx* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    // work in flight may still read the buffers or record the events: the
    // context's own work, not the device's (no device-wide wait, see geo_ctx)
    (void)wait_renders(c);
    for (int b = 0; b < 2; ++b) (void)wait_fan(c, b);
    for (int i = 0; i < geo_ctx::kStepCallSets; ++i)
        if (c->step_set_rec[i]) (void)hipEventSynchronize(c->step_set_free[i]);
    if (c->sky) (void)hipFree(c->sky);
    for (int b = 0; b < 2; ++b) {
        if (c->fan[b]) (void)hipFree(c->fan[b]);
        (void)hipEventDestroy(c->fan_written[b]);
        (void)hipEventDestroy(c->fan_read[b]);
    }
    for (int i = 0; i < geo_ctx::kStepCallSets; ++i) (void)hipEventDestroy(c->step_set_free[i]);
    for (int i = 0; i < geo_ctx::kRenderStreams; ++i) (void)hipEventDestroy(c->render_done[i]);
    if (c->step_slots) (void)hipFree(c->step_slots);
    if (c->learn_valid || c->tile_cap) (void)hipEventSynchronize(c->order_written);
    if (c->learn_stream) (void)hipStreamDestroy(c->learn_stream);
    for (int b = 0; b < 2; ++b)
        if (c->order[b]) (void)hipFree(c->order[b]);
    if (c->tile_cost) (void)hipFree(c->tile_cost);
    if (c->class_hist) (void)hipFree(c->class_hist);
    (void)hipEventDestroy(c->order_written);
    delete c;
}

int geo_set_sky(geo_ctx* c, const uint8_t* rgba8, uint32_t w, uint32_t h) {
    static_assert(geo_ctx::kSkyLevels == geo::kSkyMipLevels, "one mip chain");
    if (!c || !rgba8 || w == 0 || h == 0 || w > (1u << 20) || h > (1u << 20)) return GEO_EINVAL;
    // the padded chain must stay below 2^31 bytes (32-bit buffer offsets, PaddedSkyQuad / LevelQuad)
    uint32_t lw[geo_ctx::kSkyLevels], lh[geo_ctx::kSkyLevels], loff[geo_ctx::kSkyLevels];
    uint64_t total = 0;
    for (int l = 0; l < geo_ctx::kSkyLevels; ++l) {
        lw[l] = geo::mip_dim(w, l);
        lh[l] = geo::mip_dim(h, l);
        loff[l] = (uint32_t)total;
        total += ((uint64_t)lw[l] + 2u) * ((uint64_t)lh[l] + 2u) * 4u;
        if (total >= (1ull << 31)) return GEO_EINVAL;
    }
    const uint64_t pairs_off = total;  // kSkyPairs: level 0's row pairs after the chain
    if (kSkyPairs) {
        total += ((uint64_t)w + 2u) * ((uint64_t)h + 1u) * 8u;
        if (total >= (1ull << 31)) return GEO_EINVAL;
    }
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    // the chain on the host: level 0 = the texture, level l + 1 = the 2 x 2
    // box mean of level l (geo::mip_down), each padded for wrap/clamp
    std::vector<uint32_t> lvl((size_t)w * h), next;
    std::memcpy(lvl.data(), rgba8, (size_t)w * h * 4);
    std::vector<uint32_t> pad(total / 4u);
    for (int l = 0; l < geo_ctx::kSkyLevels; ++l) {
        if (l > 0) {
            next.resize((size_t)lw[l] * lh[l]);
            geo::mip_down(lvl.data(), lw[l - 1], lh[l - 1], next.data());
            lvl.swap(next);
        }
        geo::pad_sky(reinterpret_cast<const uint8_t*>(lvl.data()), lw[l], lh[l], pad.data() + loff[l] / 4u);
    }
    if (kSkyPairs) geo::pair_sky_rows(pad.data(), w, h, pad.data() + pairs_off / 4u);
    // Renders of this context still running on any of the caller's streams
    // (non-blocking ones do not order against a blocking copy) may be reading
    // the current sky: let them finish before it is overwritten or freed.  A
    // sky change is a set-up call (the reference builds its texture once,
    // basic_sphere_buffer.rs:29-36), so the wait costs nothing per frame.
    if (wait_renders(c) != GEO_OK) return GEO_EHIP;
    if (c->sky && c->sky_total_bytes != (uint32_t)total) {
        (void)hipFree(c->sky);
        c->sky = nullptr;
        c->sky_w = c->sky_h = 0;
    }
    if (!c->sky && hipMalloc(&c->sky, total) != hipSuccess) {
        c->sky = nullptr;
        c->sky_w = c->sky_h = 0;
        return GEO_ENOMEM;
    }
    if (hipMemcpy(c->sky, pad.data(), total, hipMemcpyHostToDevice) != hipSuccess) {
        // the buffer's contents are unknown now: no sky (renders return GEO_ESTATE until the next upload)
        (void)hipFree(c->sky);
        c->sky = nullptr;
        c->sky_w = c->sky_h = 0;
        return GEO_EHIP;
    }
    c->sky_w = w;
    c->sky_h = h;
    c->sky_total_bytes = (uint32_t)total;
    c->sky_pairs_off = (uint32_t)pairs_off;
    for (int l = 0; l < geo_ctx::kSkyLevels; ++l) {
        c->sky_lvl_w[l] = lw[l];
        c->sky_lvl_h[l] = lh[l];
        c->sky_lvl_off[l] = loff[l];
    }
    bool opaque = true;
    const size_t bytes = (size_t)w * h * 4;
    for (size_t i = 3; i < bytes && opaque; i += 4) opaque = rgba8[i] == 255;
    c->sky_opaque = opaque;  // the means of opaque texels are opaque: every level
    return GEO_OK;
}

// Both fan buffers hold at least n nodes.  Growing them waits for the device
// (renders in flight may read the old buffers); 400-node fans never regrow.
static int ensure_fan(geo_ctx* c, uint32_t n) {
    if (c->fan[0] && c->fan_cap >= n) return GEO_OK;
    for (int b = 0; b < 2; ++b)
        if (wait_fan(c, b) != GEO_OK) return GEO_EHIP;
    for (int b = 0; b < 2; ++b) {
        if (c->fan[b]) (void)hipFree(c->fan[b]);
        c->fan[b] = nullptr;
        c->n_fan[b] = 0;
        fan_forget(c, b);
    }
    c->fan_cap = 0;
    c->fan_cur = -1;
    if (hipMalloc(&c->fan[0], sizeof(float) * n) != hipSuccess) return GEO_ENOMEM;
    if (hipMalloc(&c->fan[1], sizeof(float) * n) != hipSuccess) {
        (void)hipFree(c->fan[0]);
        c->fan[0] = nullptr;
        return GEO_ENOMEM;
    }
    c->fan_cap = n;
    return GEO_OK;
}

// The buffer a new fan goes to (the one the current fan is not in), ordered
// on stream s after its previous writer and readers (on s itself by stream
// order).
static int fan_next(geo_ctx* c, hipStream_t s) {
    const int b = c->fan_cur < 0 ? 0 : 1 - c->fan_cur;
    if (c->fan_written_rec[b] && c->fan_writer[b] != s && hipStreamWaitEvent(s, c->fan_written[b], 0) != hipSuccess)
        return -1;
    if (c->fan_read_rec[b] && c->fan_reader[b] != s && hipStreamWaitEvent(s, c->fan_read[b], 0) != hipSuccess)
        return -1;
    for (int i = 0; i < c->n_render_streams; ++i)
        if ((c->fan_read_slots[b] >> i & 1u) && c->render_stream[i] != s &&
            hipStreamWaitEvent(s, c->render_done[i], 0) != hipSuccess)
            return -1;
    return b;
}

int geo_set_fan(geo_ctx* c, const float* fan, uint32_t n) {
    if (!c || !fan || n < 2 || n > kMaxFan) return GEO_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    int st = ensure_fan(c, n);
    if (st) return st;
    // a synchronous upload: into the free buffer once its last solve and
    // draws are done
    const int b = c->fan_cur < 0 ? 0 : 1 - c->fan_cur;
    if (wait_fan(c, b) != GEO_OK) return GEO_EHIP;
    if (hipMemcpy(c->fan[b], fan, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess) return GEO_EHIP;
    fan_forget(c, b);  // written and read by nothing in flight
    c->n_fan[b] = n;
    c->fan_cur = b;
    return GEO_OK;
}

int geo_solve_ray_fan(geo_ctx* c, double sphere_r, double schwarz_r, uint32_t max_iter, double step,
                      uint32_t nr_nodes, double r, float* fan_out, void* stream) {
    if (!c || nr_nodes < 2 || nr_nodes > kMaxFan || !(step > 0.)) return GEO_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    int st = ensure_fan(c, nr_nodes);
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
    const int b = fan_next(c, s);
    if (b < 0) return GEO_EHIP;
    hipLaunchKernelGGL(geo_fan_kernel, dim3((nr_nodes + 63) / 64), dim3(64), 0, s, sphere_r,
                       schwarz_r, max_iter, step, nr_nodes, r, c->fan[b]);
    if (hipGetLastError() != hipSuccess) return GEO_EHIP;
    if (hipEventRecord(c->fan_written[b], s) != hipSuccess) return GEO_EHIP;
    // the solve is ordered after every earlier reader of b: later waits for
    // b's readers start afresh, and a wait for the solve covers the old ones
    fan_forget(c, b);
    c->fan_written_rec[b] = true;
    c->fan_writer[b] = s;
    c->n_fan[b] = nr_nodes;
    c->fan_cur = b;
    if (fan_out) {
        if (hipMemcpyAsync(fan_out, c->fan[b], sizeof(float) * nr_nodes, hipMemcpyDeviceToHost, s) !=
            hipSuccess)
            return GEO_EHIP;
        if (hipStreamSynchronize(s) != hipSuccess) return GEO_EHIP;
    }
    return GEO_OK;
}

// floor(lr / d) == umulhi(lr, m) for every local row lr < 2^20: d a power of
// two, m = 2^32 / d exactly; otherwise m = floor(2^32 / d) + 1, whose error
// lr (m - 2^32/d) / 2^32 < lr / 2^32 stays below 1/d while lr d < 2^32
// (d <= 4096, checked by the caller).
static uint32_t band_rows_magic(uint32_t d) {
    return (d & (d - 1u)) == 0u ? (uint32_t)((1ull << 32) / d) : (uint32_t)((1ull << 32) / d + 1u);
}

// One frame's tiles: grid.y is limited to 65535, so a taller tile grid (more
// than 524280 rows; the C-ABI takes 2^20) goes out as several launches, each
// with its first tile row in tile_y0.  The kernel's mapping is the same.
constexpr uint32_t kMaxGridY = 65535;
extern "C++" {
// The last launch records `done` (render_event) as its stop event; a timed
// render (geo_time_next_render) puts the caller's start event on the first
// launch's dispatch and its stop event on the last one's, and records `done`
// after it.
template <int MODE, int KIND, uint32_t NF>
static int launch_tiles(RenderArgs a, const FrameBatch<NF>& fb, uint32_t nframes, bool mips, uint32_t tiles_x,
                        uint32_t tiles_y, hipStream_t s, hipEvent_t done, hipEvent_t t_start, hipEvent_t t_stop,
                        const geo::BandConsts* band) {
    a.tiles_x = tiles_x;
    // rows of tiles per launch: the 2-D grid's y limit, and WB's 1-D limit
    const bool wb = NF == 1 && !mips && (band ? kRingWaveBlocks : wave_blocks(MODE, false, 1, false));
    const uint32_t max_ny = wb ? std::min(kMaxGridY, kMaxWaveBlockTiles / tiles_x) : kMaxGridY;
    for (uint32_t y0 = 0; y0 < tiles_y; y0 += max_ny) {
        a.tile_y0 = y0;
        const uint32_t ny = tiles_y - y0 < max_ny ? tiles_y - y0 : max_ny;
        a.launch_tiles = tiles_x * ny;
        const bool last = y0 + ny >= tiles_y;
        hipEvent_t start = y0 == 0 ? t_start : nullptr;
        hipEvent_t stop = last ? (t_stop ? t_stop : done) : nullptr;
        dim3 grid(tiles_x, ny, nframes);
        if (MODE == GEO_MODE_FAN && kFanPersist && !mips)
            grid = dim3(std::min(a.launch_tiles, a.persist_blocks), 1, nframes);
        if constexpr (NF == 1) {
            if constexpr (MODE != GEO_MODE_FAN && KIND != geo::kFlat) {
                if (band) {  // GEO_FLAG_RING_F64 (one frame, level-0 sampler)
                    BandArg<true> bk;
                    bk.k = *band;
                    if (kRingWaveBlocks)
                        hipExtLaunchKernelGGL((geo_render_kernel<MODE, KIND, false, 1, true>),
                                              dim3(wave_block_count(a.launch_tiles)), dim3(64), 0, s, start, stop, 0,
                                              a, fb, bk);
                    else
                        hipExtLaunchKernelGGL((geo_render_kernel<MODE, KIND, false, 1, true>), grid, dim3(kBlock), 0,
                                              s, start, stop, 0, a, fb, bk);
                    if (hipGetLastError() != hipSuccess) return GEO_EHIP;
                    continue;
                }
            }
            if (mips)
                hipExtLaunchKernelGGL((geo_render_kernel<MODE, KIND, true, 1, false>), grid, dim3(kBlock), 0, s,
                                      start, stop, 0, a, fb, BandArg<false>{});
            else if (wave_blocks(MODE, false, 1, false))
                hipExtLaunchKernelGGL((geo_render_kernel<MODE, KIND, false, 1, false>),
                                      dim3(wave_block_count(a.launch_tiles)), dim3(64), 0, s, start, stop, 0, a, fb,
                                      BandArg<false>{});
            else
                hipExtLaunchKernelGGL((geo_render_kernel<MODE, KIND, false, 1, false>), grid, dim3(kBlock), 0, s,
                                      start, stop, 0, a, fb, BandArg<false>{});
        } else {
            bool done_ring = false;
            if constexpr (MODE != GEO_MODE_FAN && KIND != geo::kFlat) {
                if (band) {  // GEO_FLAG_RING_F64 in a batch: fb.ring_kx, the constants derived per wave
                    hipExtLaunchKernelGGL((geo_render_kernel<MODE, KIND, false, NF, true>), grid, dim3(kBlock), 0, s,
                                          start, stop, 0, a, fb, BandArg<false>{});
                    done_ring = true;
                }
            }
            if (!done_ring)
                hipExtLaunchKernelGGL((geo_render_kernel<MODE, KIND, false, NF, false>), grid, dim3(kBlock), 0, s,
                                      start, stop, 0, a, fb, BandArg<false>{});
        }
        if (hipGetLastError() != hipSuccess) return GEO_EHIP;
    }
    if (t_stop && hipEventRecord(done, s) != hipSuccess) return GEO_EHIP;
    return GEO_OK;
}

// One frame (FrameBatch<1>, the kernel arguments as before batching), or a
// batch of 2 .. kMaxBatchFrames in one launch (FrameBatch<kMaxBatchFrames>,
// the frame in blockIdx.z; no mip-mapped sampler).  band: GEO_FLAG_RING_F64's
// constants (frame 0), or null; a batch carries each frame's band factor
// (ring_kx, 0 where the frame has no capture orbit) and its kernel derives
// the constants per wave from the frame and its scene constants.
static_assert(sizeof(RenderArgs) + sizeof(FrameBatch<kMaxBatchFrames>) <= 4096, "kernel arguments fit 4 KiB");
static_assert(sizeof(RenderArgs) + sizeof(FrameBatch<1>) + sizeof(BandArg<true>) <= 4096,
              "kernel arguments fit 4 KiB");
template <int MODE, int KIND>
static int launch_frames(const RenderArgs& a, const FrameK* fk, const geo::PixelConsts* pk, uint32_t nframes,
                         bool mips, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s, hipEvent_t done,
                         hipEvent_t t_start, hipEvent_t t_stop, const geo::BandConsts* band = nullptr) {
    if (nframes == 1) {
        FrameBatch<1> fb;
        fb.f[0] = fk[0];
        return launch_tiles<MODE, KIND, 1>(a, fb, 1, mips, tiles_x, tiles_y, s, done, t_start, t_stop, band);
    }
    FrameBatch<kMaxBatchFrames> fb;
    std::memset(&fb, 0, sizeof(fb));
    for (uint32_t i = 0; i < nframes; ++i) {
        fb.f[i] = fk[i];
        fb.k[i] = pk[i];
        fb.ring_kx[i] = (band && pk[i].rs > 0.0f && pk[i].r > pk[i].rs) ? geo::band_kx(pk[i].rs, pk[i].r) : 0.0f;
    }
    return launch_tiles<MODE, KIND, kMaxBatchFrames>(a, fb, nframes, false, tiles_x, tiles_y, s, done, t_start,
                                                     t_stop, band);
}
}

// The order buffers hold at least n tiles (both orders, the costs, the class
// histograms).  Growing them waits for the context's renders and rebuilds,
// and forgets the learned order.
static int ensure_tiles(geo_ctx* c, uint32_t n) {
    if (c->tile_cap >= n) return GEO_OK;
    if (wait_renders(c) != GEO_OK || hipEventSynchronize(c->order_written) != hipSuccess) return GEO_EHIP;
    for (int b = 0; b < 2; ++b) {
        if (c->order[b]) (void)hipFree(c->order[b]);
        c->order[b] = nullptr;
    }
    if (c->tile_cost) (void)hipFree(c->tile_cost);
    if (c->class_hist) (void)hipFree(c->class_hist);
    c->tile_cost = c->class_hist = nullptr;
    c->tile_cap = 0;
    c->order_cur = -1;
    c->learn_valid = false;
    c->rebuild_pending = false;  // order_written synchronised above
    const size_t chunks = (n + kOrderChunk - 1) / kOrderChunk;
    if (hipMalloc(&c->order[0], n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->order[1], n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->tile_cost, n * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->class_hist, chunks * kCostClasses * sizeof(uint32_t)) != hipSuccess) {
        for (int b = 0; b < 2; ++b)
            if (c->order[b]) (void)hipFree(c->order[b]);
        if (c->tile_cost) (void)hipFree(c->tile_cost);
        if (c->class_hist) (void)hipFree(c->class_hist);
        c->order[0] = c->order[1] = c->tile_cost = c->class_hist = nullptr;
        return GEO_ENOMEM;
    }
    if (hipMemset(c->tile_cost, 0, n * sizeof(uint32_t)) != hipSuccess) return GEO_EHIP;
    c->tile_cap = n;
    return GEO_OK;
}

// A render call refused before render_impl: the timing pair of
// geo_time_next_render is dropped too (it belongs to that call alone).
static int invalid_call(geo_ctx* c) {
    if (c) c->time_start = c->time_stop = nullptr;
    return GEO_EINVAL;
}

// frames: nframes uniforms (1 .. kMaxBatchFrames); frame f's output starts
// out_frame_stride bytes after frame f - 1's (a batch draws colour only).
// scene_per_frame: `scene` points at nframes scenes, frame f's at scene[f]
// (they may differ in r_obs only); otherwise one scene for every frame.
static int render_impl(geo_ctx* c, const geo_frame* frames, uint32_t nframes, size_t out_frame_stride,
                       const geo_scene* scene, bool scene_per_frame, uint32_t width, uint32_t height, uint32_t row0, uint32_t nrows,
                       uint32_t band_rows, uint32_t band_stride, uint8_t* out_rgba8, uint8_t* out_mask,
                       float* out_uv, uint32_t* out_steps, unsigned long long* steps_total, void* stream) {
    // geo_time_next_render's events belong to this render alone, on every
    // exit path: a call that fails validation drops them (a later render
    // must not record the caller's pair)
    const hipEvent_t t_start = c->time_start, t_stop = c->time_stop;
    c->time_start = c->time_stop = nullptr;
    if (scene->mode != GEO_MODE_DIRECT && scene->mode != GEO_MODE_FAN && scene->mode != GEO_MODE_ADAPTIVE)
        return GEO_EINVAL;
    if ((scene->flags & ~(GEO_FLAG_DEFER_STEPS | GEO_FLAG_COMPOSITE | GEO_FLAG_MIPS | GEO_FLAG_RING_F64)) != 0)
        return GEO_EINVAL;
    const bool ring_flag = (scene->flags & GEO_FLAG_RING_F64) != 0;
    if (ring_flag && (scene->mode == GEO_MODE_FAN || (scene->flags & (GEO_FLAG_COMPOSITE | GEO_FLAG_MIPS)) != 0))
        return GEO_EINVAL;
    // frame-aligned 2 x 2 quads: the rows a wave covers start on even frame rows
    const bool mips = (scene->flags & GEO_FLAG_MIPS) != 0;
    if (mips && ((row0 | band_stride) & 1u) != 0) return GEO_EINVAL;
    if (nframes == 0 || nframes > kMaxBatchFrames) return GEO_EINVAL;
    if (nframes > 1 && (mips || out_mask || out_uv || out_steps || out_frame_stride % 4u != 0 ||
                        out_frame_stride < (size_t)nrows * width * 4u))
        return GEO_EINVAL;
    const bool adaptive = scene->mode == GEO_MODE_ADAPTIVE;
    // tol: 0 (default) or a positive finite tolerance in the adaptive mode, 0 otherwise
    if (adaptive ? !(scene->tol >= 0.0f && scene->tol <= 3.0e38f) : scene->tol != 0.0f) return GEO_EINVAL;
    const bool defer = (scene->flags & GEO_FLAG_DEFER_STEPS) != 0;
    if (scene->max_steps > (1u << 24)) return GEO_EINVAL;  // a wave's step sum must fit u32
    if (defer && steps_total) return GEO_EINVAL;
    if (!c->sky) return GEO_ESTATE;
    if (scene->mode == GEO_MODE_FAN && (c->fan_cur < 0 || c->n_fan[c->fan_cur] < 2)) return GEO_ESTATE;
    // bound > 0 (escape test folding, geo_pixel.h) needs r_obs > 0 and sphere_r > 0
    if (scene->mode != GEO_MODE_FAN &&
        (!(scene->step > 0.0f) || !(scene->r_obs > 0.0f) || !(scene->sphere_r > 0.0f) || !(scene->rs >= 0.0f)))
        return GEO_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    RenderArgs a;
    FrameK fk[kMaxBatchFrames];
    geo::PixelConsts pk[kMaxBatchFrames];
    for (uint32_t i = 0; i < nframes; ++i) {
        const geo_frame& fr = frames[i];
        std::memcpy(&fk[i].frame, &fr, sizeof(geo_frame));
        fk[i].cam = geo::camera_consts(fr.display_to_movement, fr.movement_to_central, width, height);
        fk[i].kt = geo::aberration_kt(fr.psi_factor_and_position[0]);
        const geo_scene& si = scene_per_frame ? scene[i] : *scene;
        if (i > 0 && scene_per_frame) {
            // one launch, one sampler, one integration: every field but r_obs
            // agrees with frame 0's (a fan-mode batch draws one fan: r_obs too)
            if (si.rs != scene->rs || si.sphere_r != scene->sphere_r || si.step != scene->step ||
                si.max_steps != scene->max_steps || si.mode != scene->mode || si.flags != scene->flags ||
                si.tol != scene->tol || (scene->mode == GEO_MODE_FAN && si.r_obs != scene->r_obs) ||
                !(si.r_obs > 0.0f))
                return GEO_EINVAL;
        }
        pk[i] = geo::make_consts(si.rs, si.sphere_r, si.r_obs, si.step, si.max_steps, si.tol);
        if (geo::geodesic_kind(pk[i]) != geo::geodesic_kind(pk[0])) return GEO_EINVAL;
    }
    a.out_frame_px = out_frame_stride / 4u;
    a.persist_blocks = (uint32_t)c->num_cus * 8u;  // 8 workgroups of 4 waves per CU: every wave slot
#if defined(GEO_WAVE_LOG)
    a.wave_log = c->wave_log;
#endif
    a.k = pk[0];
    a.width = width;
    a.height = height;
    a.row0 = row0;
    a.nrows = nrows;
    a.band_rows = band_rows;
    a.band_magic = band_rows_magic(band_rows);
    a.band_stride = band_stride;
    a.sky_opaque = c->sky_opaque ? 1u : 0u;
    a.composite = (scene->flags & GEO_FLAG_COMPOSITE) ? 1u : 0u;
    const uint32_t tiles_x = (width + kTileW - 1) / kTileW;
    const uint32_t tile_h = kTileH * lane_rows(scene->mode, mips);
    const uint32_t tiles_y = (nrows + tile_h - 1) / tile_h;
    a.sky = c->sky;
    a.sky_w = c->sky_w;
    a.sky_h = c->sky_h;
    a.sky_w256 = (float)c->sky_w * 256.0f;
    a.sky_h256 = (float)c->sky_h * 256.0f;
    a.sky_pitch_b = (c->sky_w + 2u) * 4u;
    a.sky_bytes = a.sky_pitch_b * (c->sky_h + 2u);
    for (int l = 0; l < geo::kSkyMipLevels; ++l) {
        a.mip_off[l] = c->sky_lvl_off[l];
        a.mip_pitch[l] = (c->sky_lvl_w[l] + 2u) * 4u;
        a.mip_w256[l] = (float)c->sky_lvl_w[l] * 256.0f;
        a.mip_h256[l] = (float)c->sky_lvl_h[l] * 256.0f;
    }
    a.sky_wf = (float)c->sky_w;
    a.sky_hf = (float)c->sky_h;
    a.sky_total_bytes = c->sky_total_bytes;
    a.sky_pairs_off = c->sky_pairs_off;
    a.sky_pairs_pitch = (c->sky_w + 2u) * 8u;
    a.tile_order = nullptr;
    a.tile_cost = nullptr;
    a.cost_overhead = adaptive ? kCostOverheadAdaptive : kCostOverheadDirect;
    const int fb = c->fan_cur;
    a.fan = fb < 0 ? nullptr : c->fan[fb];
    a.n_fan = fb < 0 ? 0u : c->n_fan[fb];
    a.out_rgba = reinterpret_cast<uint32_t*>(out_rgba8);
    a.out_mask = out_mask;
    a.out_uv = reinterpret_cast<float2*>(out_uv);
    a.out_steps = out_steps;
    hipStream_t s = (hipStream_t)stream;
    // counters: the context's accumulator (DEFER), or a per-call set free of
    // any earlier call's fold (steps_total; not in fan mode, which has none)
    int call_set = -1;
    a.step_slots = defer ? c->step_slots : nullptr;
    if (steps_total && scene->mode != GEO_MODE_FAN) {
        call_set = c->step_set_next;
        c->step_set_next = (call_set + 1) % geo_ctx::kStepCallSets;
        if (c->step_set_rec[call_set] && hipStreamWaitEvent(s, c->step_set_free[call_set], 0) != hipSuccess)
            return GEO_EHIP;
        a.step_slots = c->step_slots + (size_t)(1 + call_set) * kSlotSetU64;
    }
    // GEO_FLAG_RING_F64 (geo_band.h): the band's lanes take the f64 path; no
    // capture orbit (rs = 0, or the observer inside the horizon): the plain draw
    bool ring = ring_flag && scene->rs > 0.0f && scene->r_obs > scene->rs;
    if (ring_flag && scene_per_frame)  // a batch: any frame with a capture orbit (each gets its own factor)
        for (uint32_t i = 1; i < nframes; ++i) ring = ring || (scene[i].rs > 0.0f && scene[i].r_obs > scene[i].rs);
    const int slot = render_slot(c, s);
    if (slot < 0) return GEO_EHIP;
    const hipEvent_t done = c->render_done[slot];
    // The dispatch order (geo_ctx): a learned or explicit order for exactly
    // this grid, one launch, not in fan mode (its tiles all cost the same).
    bool record = false;
    // (one launch for the whole grid: the 2-D grid's y limit, and WB's tile count)
    if (scene->mode != GEO_MODE_FAN && tiles_y <= kMaxGridY && (uint64_t)tiles_x * tiles_y <= kMaxWaveBlockTiles) {
        if (c->dispatch_mode == GEO_DISPATCH_EXPLICIT) {
            if (c->order_cur >= 0 && tiles_x == c->explicit_x && tiles_y == c->explicit_y)
                a.tile_order = c->order[c->order_cur];
        } else if (c->dispatch_mode == GEO_DISPATCH_LONGEST_FIRST) {
            // (a GEO_FLAG_RING_F64 render learns its own order: its band's tiles cost more)
            const uint32_t key[9] = {width, height, row0, nrows, band_rows, band_stride, scene->mode,
                                     (mips ? 1u : 0u) | (ring ? 2u : 0u), tiles_x * tiles_y};
            if (!c->learn_valid || std::memcmp(key, c->learn_key, sizeof(key)) != 0) {
                std::memcpy(c->learn_key, key, sizeof(key));
                c->learn_valid = true;
                c->order_cur = -1;
                c->rebuild_keep = false;  // a rebuild still running learned another grid
                c->since_learn = c->dispatch_period;
            }
            // adopt a finished rebuild: a host query, never a wait
            if (c->rebuild_pending) {
                const hipError_t q = hipEventQuery(c->order_written);
                if (q == hipSuccess) {
                    c->rebuild_pending = false;
                    if (c->rebuild_keep) {
                        c->order_cur = c->rebuild_nb;
                        ++c->orders_adopted;
                    }
                } else if (q != hipErrorNotReady) {
                    return GEO_EHIP;
                }
            }
            // every period-th render of the grid records (period 1: every
            // render), or the first one after that whose predecessor's
            // rebuild has been adopted
            if (c->since_learn < c->dispatch_period) ++c->since_learn;
            record = c->since_learn >= c->dispatch_period && !c->rebuild_pending;
            if (record) c->since_learn = 0u;
            if (record) {
                int est = ensure_tiles(c, tiles_x * tiles_y);
                if (est) return est;
                if (!c->learn_valid) {  // the growth forgot the key: this render learns it again
                    std::memcpy(c->learn_key, key, sizeof(key));
                    c->learn_valid = true;
                }
                a.tile_cost = c->tile_cost;
            }
            if (c->order_cur >= 0) a.tile_order = c->order[c->order_cur];
        }
    }
    geo::BandConsts band_k;  // (one frame; a batch derives its frames' constants on the device)
    if (ring && nframes == 1) band_k = geo::band_consts(frames[0], *scene, width, height);
    const geo::BandConsts* band = ring ? &band_k : nullptr;
    int st;
    if (scene->mode == GEO_MODE_FAN) {
        // after the solve that wrote the buffer (geo_ctx: on the solve's own
        // stream by stream order, with no event work: the reader is its
        // slot's bit); on another stream this render then joins the buffer's
        // chain of readers (the wait is queued after the launch, so it holds
        // back only later work on s, never this render)
        // (a buffer uploaded by geo_set_fan has no writer in flight: its next
        // writer waits for its readers on the host, so they need no event)
        const bool by_slot = !c->fan_written_rec[fb] || c->fan_writer[fb] == s;
        if (!by_slot && hipStreamWaitEvent(s, c->fan_written[fb], 0) != hipSuccess) return GEO_EHIP;
        st = launch_frames<GEO_MODE_FAN, geo::kCurvedOut>(a, fk, pk, nframes, mips, tiles_x, tiles_y, s, done, t_start, t_stop);
        if (st) return st;
        if (by_slot) {
            c->fan_read_slots[fb] |= 1u << slot;
        } else {
            if (c->fan_read_rec[fb] && c->fan_reader[fb] != s &&
                hipStreamWaitEvent(s, c->fan_read[fb], 0) != hipSuccess)
                return GEO_EHIP;
            if (hipEventRecord(c->fan_read[fb], s) != hipSuccess) return GEO_EHIP;
            c->fan_read_rec[fb] = true;
            c->fan_reader[fb] = s;
        }
    } else if (adaptive) {
        switch (geo::geodesic_kind(a.k)) {
            case geo::kCurvedOut: st = launch_frames<GEO_MODE_ADAPTIVE, geo::kCurvedOut>(a, fk, pk, nframes, mips, tiles_x, tiles_y, s, done, t_start, t_stop, band); break;
            case geo::kCurvedIn: st = launch_frames<GEO_MODE_ADAPTIVE, geo::kCurvedIn>(a, fk, pk, nframes, mips, tiles_x, tiles_y, s, done, t_start, t_stop, band); break;
            default: st = launch_frames<GEO_MODE_ADAPTIVE, geo::kFlat>(a, fk, pk, nframes, mips, tiles_x, tiles_y, s, done, t_start, t_stop);
        }
    } else {
        switch (geo::geodesic_kind(a.k)) {
            case geo::kCurvedOut: st = launch_frames<GEO_MODE_DIRECT, geo::kCurvedOut>(a, fk, pk, nframes, mips, tiles_x, tiles_y, s, done, t_start, t_stop, band); break;
            case geo::kCurvedIn: st = launch_frames<GEO_MODE_DIRECT, geo::kCurvedIn>(a, fk, pk, nframes, mips, tiles_x, tiles_y, s, done, t_start, t_stop, band); break;
            default: st = launch_frames<GEO_MODE_DIRECT, geo::kFlat>(a, fk, pk, nframes, mips, tiles_x, tiles_y, s, done, t_start, t_stop);
        }
    }
    if (st) return st;
    if (record) {
        // rebuild the order into the buffer not in use, on the context's
        // learn stream, after every render of the context issued so far (this
        // one included: its launch recorded render_done[slot]); earlier
        // renders on any stream may still read that buffer
        ++c->costs_recorded;
        if (!c->learn_stream && hipStreamCreateWithFlags(&c->learn_stream, hipStreamNonBlocking) != hipSuccess) {
            c->learn_stream = nullptr;
            return GEO_EHIP;
        }
        hipStream_t ls = c->learn_stream;
        const int nb = c->order_cur < 0 ? 0 : 1 - c->order_cur;
        for (int i = 0; i < c->n_render_streams; ++i)
            if (hipStreamWaitEvent(ls, c->render_done[i], 0) != hipSuccess) return GEO_EHIP;
        const uint32_t n = tiles_x * tiles_y;
        const uint32_t chunks = (n + kOrderChunk - 1) / kOrderChunk;
        hipLaunchKernelGGL(geo_order_hist, dim3(chunks), dim3(256), 0, ls, c->tile_cost, n, c->class_hist);
        hipLaunchKernelGGL(geo_order_scatter, dim3(chunks), dim3(256), 0, ls, c->tile_cost, n, c->class_hist, tiles_x,
                           c->order[nb]);
        if (hipGetLastError() != hipSuccess) return GEO_EHIP;
        if (hipEventRecord(c->order_written, ls) != hipSuccess) return GEO_EHIP;
        c->rebuild_pending = true;
        c->rebuild_keep = true;
        c->rebuild_nb = nb;
    }
    if (call_set >= 0) {
        hipLaunchKernelGGL(geo_steps_finalize, dim3(1), dim3(kStepSlots), 0, s, a.step_slots, steps_total);
        if (hipGetLastError() != hipSuccess) return GEO_EHIP;
        if (hipEventRecord(c->step_set_free[call_set], s) != hipSuccess) return GEO_EHIP;
        c->step_set_rec[call_set] = true;
    }
    return GEO_OK;
}

int geo_assemble_bands(geo_ctx* c, const uint8_t* src, size_t rank_stride, size_t frame_stride, uint32_t world,
                       uint32_t band_rows, uint32_t width, uint32_t height, uint32_t nframes, uint32_t src_bpp,
                       uint8_t* dst, void* stream) {
    if (!c || !src || !dst || world == 0 || band_rows == 0 || width == 0 || height == 0 || nframes == 0 ||
        height > 65535u || nframes > 65535u || (src_bpp != 3u && src_bpp != 4u))
        return GEO_EINVAL;
    if (src_bpp == 3u && (width % 4u != 0 || rank_stride % 4u != 0 || frame_stride % 4u != 0 ||
                          (uintptr_t)src % 4u != 0 || (uintptr_t)dst % 16u != 0))
        return GEO_EINVAL;
    const size_t row_bytes = (size_t)width * src_bpp;
    const size_t nb_max = ((size_t)(height + band_rows - 1) / band_rows + world - 1) / world;
    if (frame_stride < nb_max * band_rows * row_bytes || rank_stride < (size_t)nframes * frame_stride)
        return GEO_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    hipStream_t s = (hipStream_t)stream;
    if (src_bpp == 3u) {
        const uint32_t quads = width / 4u;
        hipLaunchKernelGGL(geo_assemble_rgb_kernel, dim3((quads + 255u) / 256u, height, nframes), dim3(256), 0, s,
                           src, rank_stride, frame_stride, world, band_rows, quads, height, dst);
        return hipGetLastError() == hipSuccess ? GEO_OK : GEO_EHIP;
    }
    const bool wide = (width % 4u) == 0 && (rank_stride % 16u) == 0 && (frame_stride % 16u) == 0 &&
                      ((uintptr_t)src % 16u) == 0 && ((uintptr_t)dst % 16u) == 0;
    const uint32_t units = wide ? width / 4u : width;
    const dim3 grid((units + 255u) / 256u, height, nframes);
    if (wide)
        hipLaunchKernelGGL(geo_assemble_kernel<uint4>, grid, dim3(256), 0, s, src, rank_stride, frame_stride, world,
                           band_rows, units, height, dst);
    else
        hipLaunchKernelGGL(geo_assemble_kernel<uint32_t>, grid, dim3(256), 0, s, src, rank_stride, frame_stride,
                           world, band_rows, units, height, dst);
    return hipGetLastError() == hipSuccess ? GEO_OK : GEO_EHIP;
}

int geo_assemble_shares(geo_ctx* c, const uint8_t* lead_src, size_t lead_frame_stride, uint32_t lead_rows,
                        const uint8_t* src, size_t rank_stride, size_t frame_stride, uint32_t world,
                        uint32_t band_rows, uint32_t width, uint32_t height, uint32_t nframes, uint32_t src_bpp,
                        uint8_t* dst, void* stream) {
    if (!c || !lead_src || !dst || world == 0 || lead_rows == 0 || band_rows == 0 || width == 0 || height == 0 ||
        nframes == 0 || height > 65535u || nframes > 65535u || (src_bpp != 3u && src_bpp != 4u))
        return GEO_EINVAL;
    // 16-B units need width % 4 == 0 and aligned buffers; RGB24 peers need them
    const size_t lead_align = width % 4u == 0 ? 16u : 4u;
    if (src_bpp == 3u && width % 4u != 0) return GEO_EINVAL;
    if ((uint64_t)lead_rows + (uint64_t)(world - 1u) * band_rows > (1u << 20)) return GEO_EINVAL;
    const uint32_t cycle = lead_rows + (world - 1u) * band_rows;
    // rank 0 has ceil(H / cycle) bands; rank 1, the first peer, the most of the peers
    const size_t nb0 = (height + cycle - 1u) / cycle;
    const size_t nb1 = height > lead_rows ? (height - lead_rows + cycle - 1u) / cycle : 0;
    if (lead_frame_stride < nb0 * lead_rows * (size_t)width * 4u) return GEO_EINVAL;
    if (lead_frame_stride % lead_align != 0 || (uintptr_t)lead_src % lead_align != 0 ||
        (uintptr_t)dst % lead_align != 0)
        return GEO_EINVAL;
    if (world > 1u) {
        if ((nb1 > 0 && !src) || frame_stride < nb1 * band_rows * (size_t)width * src_bpp ||
            rank_stride < (size_t)nframes * frame_stride)
            return GEO_EINVAL;
        const size_t align = src_bpp == 4u ? lead_align : 4u;
        if (rank_stride % align != 0 || frame_stride % align != 0 || (uintptr_t)src % align != 0) return GEO_EINVAL;
    }
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    hipStream_t s = (hipStream_t)stream;
    if (width % 4u == 0) {
        const uint32_t quads = width / 4u;
        hipLaunchKernelGGL(geo_assemble_lead_kernel<true>, dim3((quads + 255u) / 256u, height, nframes), dim3(256),
                           0, s, lead_src, lead_frame_stride, lead_rows, src, rank_stride, frame_stride, world,
                           band_rows, quads, height, src_bpp, dst);
    } else {
        hipLaunchKernelGGL(geo_assemble_lead_kernel<false>, dim3((width + 255u) / 256u, height, nframes), dim3(256),
                           0, s, lead_src, lead_frame_stride, lead_rows, src, rank_stride, frame_stride, world,
                           band_rows, width, height, src_bpp, dst);
    }
    return hipGetLastError() == hipSuccess ? GEO_OK : GEO_EHIP;
}

int geo_assemble_lead(geo_ctx* c, const uint8_t* lead_src, size_t lead_frame_stride, uint32_t lead,
                      const uint8_t* src, size_t rank_stride, size_t frame_stride, uint32_t world,
                      uint32_t band_rows, uint32_t width, uint32_t height, uint32_t nframes, uint32_t src_bpp,
                      uint8_t* dst, void* stream) {
    if (lead == 0 || (uint64_t)lead * band_rows > (1u << 20)) return GEO_EINVAL;
    return geo_assemble_shares(c, lead_src, lead_frame_stride, lead * band_rows, src, rank_stride, frame_stride,
                               world, band_rows, width, height, nframes, src_bpp, dst, stream);
}

int geo_pack_rgb(geo_ctx* c, const uint8_t* rgba, uint64_t npixels, uint8_t* rgb, void* stream) {
    if (!c || !rgba || !rgb || npixels == 0 || npixels % 4u != 0 || (uintptr_t)rgba % 16u != 0 ||
        (uintptr_t)rgb % 4u != 0)
        return GEO_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    const uint64_t quads = npixels / 4u;
    hipLaunchKernelGGL(geo_pack_rgb_kernel, dim3((unsigned)((quads + 255u) / 256u)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const uint4*>(rgba), quads, reinterpret_cast<uint32_t*>(rgb));
    return hipGetLastError() == hipSuccess ? GEO_OK : GEO_EHIP;
}

int geo_steps_flush(geo_ctx* c, unsigned long long* steps_total, void* stream) {
    if (!c || !steps_total) return GEO_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    const hipEvent_t done = render_event(c, (hipStream_t)stream);
    if (!done) return GEO_EHIP;
    hipExtLaunchKernelGGL(geo_steps_finalize, dim3(1), dim3(kStepSlots), 0, (hipStream_t)stream, nullptr, done, 0,
                          c->step_slots, steps_total);
    return hipGetLastError() == hipSuccess ? GEO_OK : GEO_EHIP;
}

int geo_time_next_render(geo_ctx* c, void* start_event, void* stop_event) {
    if (!c || !start_event || !stop_event) return GEO_EINVAL;
    c->time_start = (hipEvent_t)start_event;
    c->time_stop = (hipEvent_t)stop_event;
    return GEO_OK;
}

int geo_set_dispatch(geo_ctx* c, int mode, uint32_t period) {
    if (!c || (mode != GEO_DISPATCH_ROW_MAJOR && mode != GEO_DISPATCH_LONGEST_FIRST) || period == 0 ||
        period > (1u << 20))
        return GEO_EINVAL;
    c->dispatch_mode = mode;
    c->dispatch_period = period;
    c->learn_valid = false;  // learn again from the next render
    c->order_cur = -1;
    c->rebuild_keep = false;
    return GEO_OK;
}

#if defined(GEO_WAVE_LOG)
// Diagnostic build only: renders log every wave's span into `log` (4 u64 per
// wave of the launch's grid, device memory; NULL stops logging).
int geo_debug_set_wave_log(geo_ctx* c, void* log) {
    if (!c) return GEO_EINVAL;
    c->wave_log = (unsigned long long*)log;
    return GEO_OK;
}
#endif

int geo_dispatch_stats(geo_ctx* c, unsigned long long* costs_recorded, unsigned long long* orders_adopted) {
    if (!c) return GEO_EINVAL;
    if (costs_recorded) *costs_recorded = c->costs_recorded;
    if (orders_adopted) *orders_adopted = c->orders_adopted;
    return GEO_OK;
}

int geo_set_tile_order(geo_ctx* c, uint32_t tiles_x, uint32_t tiles_y, const uint32_t* order) {
    if (!c) return GEO_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return GEO_EHIP;
    if (!order) {  // row-major
        c->dispatch_mode = GEO_DISPATCH_ROW_MAJOR;
        c->learn_valid = false;
        c->order_cur = -1;
        c->rebuild_keep = false;
        return GEO_OK;
    }
    if (tiles_x == 0 || tiles_y == 0 || tiles_x > 0xFFFFu || tiles_y > kMaxGridY) return GEO_EINVAL;
    const size_t n = (size_t)tiles_x * tiles_y;
    if (n > 0xFFFFFFFFu) return GEO_EINVAL;
    std::vector<uint8_t> seen(n, 0);  // a permutation of the grid's tiles
    for (size_t i = 0; i < n; ++i) {
        const uint32_t x = order[i] & 0xFFFFu, y = order[i] >> 16;
        if (x >= tiles_x || y >= tiles_y || seen[(size_t)y * tiles_x + x]) return GEO_EINVAL;
        seen[(size_t)y * tiles_x + x] = 1;
    }
    int st = ensure_tiles(c, (uint32_t)n);
    if (st) return st;
    // renders in flight may read either buffer, a rebuild may write one
    if (wait_renders(c) != GEO_OK || hipEventSynchronize(c->order_written) != hipSuccess) return GEO_EHIP;
    c->rebuild_pending = false;
    if (hipMemcpy(c->order[0], order, n * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
        c->order_cur = -1;
        return GEO_EHIP;
    }
    c->dispatch_mode = GEO_DISPATCH_EXPLICIT;
    c->explicit_x = tiles_x;
    c->explicit_y = tiles_y;
    c->order_cur = 0;
    c->learn_valid = false;
    return GEO_OK;
}

int geo_render_rows(geo_ctx* c, const geo_frame* frame, const geo_scene* scene, uint32_t width,
                    uint32_t height, uint32_t row0, uint32_t nrows, uint8_t* out_rgba8,
                    uint8_t* out_mask, float* out_uv, uint32_t* out_steps,
                    unsigned long long* steps_total, void* stream) {
    if (!c || !frame || !scene || !out_rgba8 || width == 0 || height == 0 || nrows == 0)
        return invalid_call(c);
    if ((uint64_t)row0 + nrows > height || width > (1u << 20) || height > (1u << 20))
        return invalid_call(c);
    // one band covering every row (2^21 >= nrows)
    return render_impl(c, frame, 1, 0, scene, false, width, height, row0, nrows, 1u << 21, 1u << 21, out_rgba8, out_mask,
                       out_uv, out_steps, steps_total, stream);
}

int geo_render_bands(geo_ctx* c, const geo_frame* frame, const geo_scene* scene, uint32_t width,
                     uint32_t height, uint32_t band_rows, uint32_t band0, uint32_t band_step,
                     uint32_t nbands, uint8_t* out_rgba8, uint8_t* out_mask, float* out_uv,
                     uint32_t* out_steps, unsigned long long* steps_total, void* stream) {
    if (!c || !frame || !scene || !out_rgba8 || width == 0 || height == 0 || band_rows == 0 ||
        nbands == 0 || band_step == 0 || band_rows < kBandRowAlign || (band_rows & (band_rows - 1)) != 0)
        return invalid_call(c);
    if (width > (1u << 20) || height > (1u << 20)) return invalid_call(c);
    const uint64_t first = (uint64_t)band0 * band_rows;
    const uint64_t last = first + (uint64_t)(nbands - 1) * band_step * band_rows;
    const uint64_t nrows = (uint64_t)nbands * band_rows;
    if (first >= height || last >= height || nrows > (1u << 20)) return invalid_call(c);
    return render_impl(c, frame, 1, 0, scene, false, width, height, (uint32_t)first, (uint32_t)nrows,
                       band_rows, band_step * band_rows, out_rgba8, out_mask, out_uv,
                       out_steps, steps_total, stream);
}

// The band set's arguments, checked (geo_render_band_set, geo_render_band_set_frames).
static bool band_set_ok(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row0, uint32_t row_stride,
                        uint32_t nbands) {
    // band_rows: a multiple of 8, at most 4096 unless a power of two (band_rows_magic)
    if (width == 0 || height == 0 || band_rows == 0 || nbands == 0 || row_stride < band_rows ||
        band_rows % kBandRowAlign != 0 || ((band_rows & (band_rows - 1)) != 0 && band_rows > 4096u))
        return false;
    if (width > (1u << 20) || height > (1u << 20)) return false;
    const uint64_t last = (uint64_t)row0 + (uint64_t)(nbands - 1) * row_stride;
    const uint64_t nrows = (uint64_t)nbands * band_rows;
    return row0 < height && last < height && nrows <= (1u << 20);
}

int geo_render_band_set(geo_ctx* c, const geo_frame* frame, const geo_scene* scene, uint32_t width,
                        uint32_t height, uint32_t band_rows, uint32_t row0, uint32_t row_stride, uint32_t nbands,
                        uint8_t* out_rgba8, uint8_t* out_mask, float* out_uv, uint32_t* out_steps,
                        unsigned long long* steps_total, void* stream) {
    if (!c || !frame || !scene || !out_rgba8 || !band_set_ok(width, height, band_rows, row0, row_stride, nbands))
        return invalid_call(c);
    return render_impl(c, frame, 1, 0, scene, false, width, height, row0, nbands * band_rows, band_rows, row_stride,
                       out_rgba8, out_mask, out_uv, out_steps, steps_total, stream);
}

int geo_render_band_set_frames(geo_ctx* c, const geo_frame* frames, uint32_t nframes, const geo_scene* scene,
                               uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row0,
                               uint32_t row_stride, uint32_t nbands, uint8_t* out_rgba8, size_t out_frame_stride,
                               unsigned long long* steps_total, void* stream) {
    if (!c || !frames || !scene || !out_rgba8 || nframes == 0 || nframes > kMaxBatchFrames ||
        !band_set_ok(width, height, band_rows, row0, row_stride, nbands))
        return invalid_call(c);
    return render_impl(c, frames, nframes, out_frame_stride, scene, false, width, height, row0, nbands * band_rows,
                       band_rows, row_stride, out_rgba8, nullptr, nullptr, nullptr, steps_total, stream);
}

int geo_render_band_set_batch(geo_ctx* c, const geo_frame* frames, const geo_scene* scenes, uint32_t nframes,
                              uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row0, uint32_t row_stride,
                              uint32_t nbands, uint8_t* out_rgba8, size_t out_frame_stride,
                              unsigned long long* steps_total, void* stream) {
    if (!c || !frames || !scenes || !out_rgba8 || nframes == 0 || nframes > kMaxBatchFrames ||
        !band_set_ok(width, height, band_rows, row0, row_stride, nbands))
        return invalid_call(c);
    return render_impl(c, frames, nframes, out_frame_stride, scenes, true, width, height, row0, nbands * band_rows,
                       band_rows, row_stride, out_rgba8, nullptr, nullptr, nullptr, steps_total, stream);
}

}  // extern "C"
