// gsr_common.h -- shared device math, buffer layouts and launch declarations
// of the MI355X-native Gaussian rasterizer (gfx950 / CDNA4, wave64).
//
// Buffer layouts are computed on the host from (P, num_rendered, W, H) alone,
// exactly like the reference re-derives its chunk pointers
// (rasterizer_impl.cu:155-194, rasterizer_impl.h:21-73), so gsr_backward can
// find every array again without any header read-back.
#pragma once
#include <string>

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gsr {

constexpr int TILE_X = 16;  // config.h:16-17 (BLOCK_X/BLOCK_Y); parity needs 16x16 tiles
constexpr int TILE_Y = 16;
constexpr int TILE_PIX = TILE_X * TILE_Y;
// Count-matrix rows (one preprocess / duplicate workgroup each): 1024 Gaussians, or 512 when rows of 1024
// would put fewer than two on every CU -- config 3's 293 rows on 256 CUs left 37 CUs with two workgroups'
// work (tracking preprocess 20.3 -> 16.7 us with 586 rows of 512); config 4's 977 rows stay at 1024 (its
// count matrix would double: column scan 16 -> 31 us).  The choice is a pure function of (P, CU count):
// GeomLayout::make and every kernel read it as a shift (Camera::pre_shift).
constexpr int PRE_BLOCK = 1024;  // the largest row (workgroup size bound, LDS arrays)
__host__ __device__ inline int pre_shift_for(int P, int cus) { return ((P + 1023) >> 10) < 2 * cus ? 9 : 10; }
int geom_pre_shift(int P);  // pre_shift_for(P, CU count of the current device) (gsr_capi.hip)
int current_device_cus();   // the current device's CU count (gsr_capi.hip)
constexpr int MAX_LDS_TILES = 16384; // tile histogram in LDS up to 64 KB; global atomics beyond
constexpr int SORT_THREADS = 256;
constexpr int SORT_ITEMS = 8;        // keys per thread per radix pass
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;
constexpr int RADIX = 256;
constexpr int RENDER_BATCH = 256;    // Gaussians staged in LDS per batch
constexpr int INST_REC_MAX = 12;     // backward per-instance record: at most 12 floats (RecLayout)
constexpr int TILE_CTR_STRIDE = 64;  // per-tile atomic counters one 256-B line apart (spread over L2 channels)

// ---------------------------------------------------------------- layouts --
__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// One 64-byte render record per Gaussian (four float4, one cache-line fetch per
// gather in the render kernels; the SoA form cost ~6 line fetches per instance),
// stored in the form the render loops evaluate (copied to LDS as is):
//   q0 = (x, y, K_AC * conic A, K_AC * conic C)   pixel coordinates; K_AC = -log2(e)/2
//   q1 = (K_B * conic B, opacity, depth, workgroup-local instance offset bits); K_B = -log2(e)
//   q2 = (r, g, b, tile rect lo bits)   rect lo = x0 | y0 << 16
//   q3 = (colors2 r, g, b, tile rect hi bits)   rect hi = x1 | y1 << 16; colors2 = 0 unless dual
constexpr int RR_F4 = 4;
struct GeomLayout {       // per-Gaussian state ("geomBuffer")
    size_t rr;            // float4 [P][4] render records
    size_t clamp;         // u32    [P]  SH clamp bits (r, g, b)
    size_t bin;           // uint4  [P]  (rect lo, rect hi, depth bits, tiles) for duplicate
    size_t tiles;         // u32    [P]  tiles touched
    size_t offsets;       // u32    [P]  exclusive instance offset (also in q1.w)
    size_t blocksums;     // u32    [nb] exclusive scan of the per-workgroup instance totals
    size_t wgsum;         // u32    [nb] per-workgroup instance totals (bit 31: prefiltered violation)
    size_t wgcull;        // u32    [nb] per-workgroup culled-instance totals (Camera::cull; point_list's tail)
    size_t counters;      // u32    [8]  [0]=num_rendered [1]=prefiltered violation [2]=longest tile list
                          //             [3]=sort cap [4]=colscan arrival counter
    size_t total;
    int nb;     // count-matrix rows
    int shift;  // log2 Gaussians per row
    static GeomLayout make(int P) { return make(P, geom_pre_shift(P)); }
    static GeomLayout make(int P, int shift) {
        GeomLayout L;
        size_t o = 0, p = (size_t)(P > 0 ? P : 1);
        L.shift = shift;
        L.nb = (P + (1 << shift) - 1) >> shift;
        L.rr = o; o = align_up(o + 16 * RR_F4 * p, 256);
        L.clamp = o; o = align_up(o + 4 * p, 256);
        L.bin = o; o = align_up(o + 16 * p, 256);
        L.tiles = o; o = align_up(o + 4 * p, 256);
        L.offsets = o; o = align_up(o + 4 * p, 256);
        L.blocksums = o; o = align_up(o + 4 * (size_t)(L.nb > 0 ? L.nb : 1), 256);
        L.wgsum = o; o = align_up(o + 4 * (size_t)(L.nb > 0 ? L.nb : 1), 256);
        L.wgcull = o; o = align_up(o + 4 * (size_t)(L.nb > 0 ? L.nb : 1), 256);
        L.counters = o; o = align_up(o + 32, 256);
        L.total = o;
        return L;
    }
};

struct ImgLayout {        // per-pixel / per-tile state ("imgBuffer")
    size_t final_T;       // f32   [N]
    size_t n_contrib;     // u32   [N]
    size_t ranges;        // uint2 [tiles]  [start, end) of each tile's sorted list
    size_t order;         // u32   [tiles]  render schedule: workgroup i renders tile order[i] (tile_plan)
    size_t tile_count;    // u32   [2*tiles*TILE_CTR_STRIDE] instance counters, then bucket cursors (one memset)
    size_t rowmax;        // u32   [tiles*16] per 4x4 block (tile_px/tile_py order): the longest n_contrib
    size_t total;
    static ImgLayout make(int W, int H) {
        ImgLayout L;
        size_t N = (size_t)W * H;
        size_t T = (size_t)((W + TILE_X - 1) / TILE_X) * ((H + TILE_Y - 1) / TILE_Y);
        size_t o = 0;
        L.final_T = o; o = align_up(o + 4 * (N ? N : 1), 256);
        L.n_contrib = o; o = align_up(o + 4 * (N ? N : 1), 256);
        L.ranges = o; o = align_up(o + 8 * (T ? T : 1), 256);
        L.order = o; o = align_up(o + 4 * (T ? T : 1), 256);
        L.tile_count = o; o = align_up(o + 8 * (size_t)TILE_CTR_STRIDE * (T ? T : 1), 256);
        L.rowmax = o; o = align_up(o + 64 * (T ? T : 1), 256);
        L.total = o;
        return L;
    }
};

inline int higher_msb(uint32_t n) {  // rasterizer_impl.cu:35-50 (bits needed for tile ids)
    int b = 0;
    while (b < 32 && (n >> b) != 0) b++;
    return b;
}

constexpr int TILE_SORT_CAP = 4096;  // longest tile list render_fwd sorts (4 chunks of 1024 keys)

struct BinLayout {        // per-instance state ("binningBuffer")
    size_t point_list;    // u64 [I] PointEntry (mask << 32 | Gaussian id) in (tile, depth, id) order -- offset 0
    size_t keys[2];       // u64 [I] bucketed (depth<<32 | id) keys / radix ping-pong (tile<<32 | depth)
    size_t vals[2];       // u32 [I] radix ping-pong values (fallback path only)
    size_t gid;           // u32 [I] Gaussian id of each unsorted instance (fallback path only)
    size_t hist;          // u32 [RADIX * nsb] + [RADIX] digit totals (fallback path only)
    size_t total;
    int nsb;              // radix-sort workgroups
    int npass;            // 8-bit LSD passes over bits [0, 32 + msb(tiles))
    int final_buf;        // which ping-pong half holds the sorted keys/vals
    static BinLayout make(int I, int W, int H) {
        BinLayout L;
        size_t n = (size_t)(I > 0 ? I : 1);
        uint32_t tiles = (uint32_t)(((W + TILE_X - 1) / TILE_X) * ((H + TILE_Y - 1) / TILE_Y));
        int bits = 32 + higher_msb(tiles);
        L.npass = (bits + 7) / 8;
        L.final_buf = L.npass & 1;
        L.nsb = (int)((n + SORT_TILE - 1) / SORT_TILE);
        size_t o = 0;
        L.point_list = o; o = align_up(o + 8 * n, 256);
        L.keys[0] = o; o = align_up(o + 8 * n, 256);
        L.keys[1] = o; o = align_up(o + 8 * n, 256);
        L.vals[0] = o; o = align_up(o + 4 * n, 256);
        L.vals[1] = o; o = align_up(o + 4 * n, 256);
        L.gid = o; o = align_up(o + 4 * n, 256);
        L.hist = o; o = align_up(o + 4 * ((size_t)RADIX * L.nsb + RADIX), 256);  // + digit totals
        L.total = o;
        return L;
    }
};

// ------------------------------------------------------------ parameters --
// A launch's device-side switch (the gated geometry reuse of gsr_forward_reuse_if_equal): the comparison
// kernel stores the call's epoch e into *p when the geometry differs; the kernel runs iff (*p == e) == run.
// The word is not cleared first: whatever it held is not e (epochs are unique per call), which reads as
// "equal" only if the comparison found no difference.  p == nullptr: always runs.  Read once per
// workgroup, before anything else.
struct Gate {
    const uint32_t* p = nullptr;
    uint32_t e = 0;
    uint32_t run = 1;
    __device__ __forceinline__ bool off() const { return p != nullptr && ((*p == e) != (run != 0u)); }
};

struct Camera {
    int W, H;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    int gx, gy;  // tile grid
    const float* view;
    const float* proj;
    const float* campos;
    const float* bg;
    float scale_modifier;
    int sh_degree;
    int prefiltered;
    // Render schedule: render workgroup i renders tile tile_order[i] (a permutation written by
    // the binning's workgroup 0, tile_plan; nullptr = row-major).  sched_cus: the device's CU
    // count, the round size of the plan.
    const uint32_t* tile_order = nullptr;
    uint32_t* tile_order_out = nullptr;
    // Per-block last-contributor maxima (ImgLayout::rowmax): written by render_fwd, read by render_bwd
    // (its batch range and row-list bounds without a reduction over n_contrib first); nullptr = not kept
    uint32_t* rowmax = nullptr;
    int sched_cus = 256;
    int pre_shift = 10;  // log2 Gaussians per count-matrix row (GeomLayout::shift)
    // Tile culling (the fused tracking forward, static mode): a (Gaussian, tile) instance whose alpha >= 1/255
    // ellipse reaches no 4x4 block of the tile (block_mask_exact == 0, conservative) is left out of the tile's
    // bucket -- it would be sorted and staged but never evaluated, and its record would be zero.  Its record
    // slot stays (slots are rect-indexed); bin[i].w carries the Gaussian's live-tile mask, which gauss_bwd
    // reads to skip the unwritten slots.  Results are bitwise those of the unculled lists; num_rendered
    // (the record count) is unchanged, the tile ranges are shorter.
    int cull = 0;
    // point_list's tail [L, num_rendered) of a culled binning: 1 the culled instances themselves (the dynamic
    // forward, whose buffers the caller reads like the reference's), 0 padding ids (static mode)
    int tail_exact = 0;
    Gate gate;  // (preprocess, duplicate_bucket and render_fwd return at once when it is off)
    // Host snapshot (the dynamic forward's bucketed binning only): the duplicate's workgroup 0 stores counters[0..7]
    // into this mapped, coherent pinned host buffer once they are final -- in place of a 32-B device-to-host copy
    // launched behind it (4 us of the stream per forward) -- and the host's event follows the duplicate
    uint32_t* host_snap = nullptr;
};
// bin[i].w: bit k set = rect tile k (row-major in the rect) has an instance in its bucket; all ones when
// nothing is culled (or the rect has more than 32 tiles)
__device__ __forceinline__ bool tile_live(uint32_t live, uint32_t k) { return k >= 32u || ((live >> k) & 1u); }
// culled instances among rect tiles [0, k) (k <= the Gaussian's tile count): positions in point_list's tail
__device__ __forceinline__ uint32_t culled_below(uint32_t live, uint32_t k) {
    const uint32_t m = k >= 32u ? 0xFFFFFFFFu : ((1u << k) - 1u);
    return (uint32_t)__popc(~live & m);
}
// Wave priority by remaining work (GSR_PRIO_SCHED): the instruction arbiter favours older
// waves, so on a CU the last-dispatched tile used to run alone at the end at one wave per
// SIMD; raising the priority of the waves with the most work left keeps the CU's tiles
// finishing together (a dynamic longest-remaining-first among co-resident tiles).
#ifndef GSR_PRIO_SCHED
#define GSR_PRIO_SCHED 1
#endif
// Levels at 70 / 45 / 22 % of the frame's mean tile list (`mean4` = 4 x mean, from num_rendered) when every tile
// is resident at once (config 3: 1200 tiles, 1280 workgroup slots; 200 / 100 / 50 % measured 3 us slower
// there), and at 200 / 100 / 50 % when the tiles take several dispatch rounds (config 4: 3225 tiles; the
// single-round levels measured 392 against 383 us for render_bwd): `multi` = more tiles than 5 per CU.
__device__ __forceinline__ void prio_by_remaining(int remaining, uint32_t mean4, bool multi) {
#if GSR_PRIO_SCHED
    const uint32_t r = 4u * (uint32_t)remaining;  // compare r / mean4 against the level thresholds (x 100)
    const uint32_t t3 = multi ? 200u : 70u, t2 = multi ? 100u : 45u, t1 = multi ? 50u : 22u;
    if (100u * r > t3 * mean4) __builtin_amdgcn_s_setprio(3);
    else if (100u * r > t2 * mean4) __builtin_amdgcn_s_setprio(2);
    else if (100u * r > t1 * mean4) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#endif
}
__device__ __forceinline__ bool sched_multi_round(const Camera& cam) { return cam.gx * cam.gy > 5 * cam.sched_cus; }
__device__ __forceinline__ uint32_t sched_mean4(const Camera& cam, const uint32_t* counters) {
    const uint32_t nt = (uint32_t)(cam.gx * cam.gy);
    return max(1u, (uint32_t)(4ull * counters[0] / (nt ? nt : 1u)));
}
// the tile a render workgroup (1D grid over the tiles) works on
__device__ __forceinline__ int sched_tile(const Camera& cam) {
    return cam.tile_order ? (int)cam.tile_order[blockIdx.x] : (int)blockIdx.x;
}

// SplaTAM's tracking transform (gsr_track_transform_fwd) fused into preprocess: the world-frame
// map + the frame's pose in; preprocess forms the camera-frame rendervars itself and also writes
// them to GaussIn's means3D / rotations / opacities / scales / colors2 (then outputs) for the
// backward.  mw == nullptr: no transform (GaussIn holds the rendervars).
struct TrackXf {
    const float* mw = nullptr;  // means_world [P,3]
    const float* ur = nullptr;  // unnorm_rotations [P,4]
    const float* lo = nullptr;  // logit_opacities [P,1]
    const float* ls = nullptr;  // log_scales [P,scols]
    int scols = 1;
    const float* cq = nullptr;  // the frame's quaternion column (stride qs)
    const float* ct = nullptr;  // the frame's translation column (stride qs)
    int qs = 1;
    const float* w2c = nullptr;  // [16] row-major (depth colours)
    int store = 1;               // 0: the rendervars are not stored (the tracking backward recomputes them)
};

struct GaussIn {
    TrackXf xf;
    int P, M;
    const float* means3D;
    const float* shs;
    const float* colors;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D;
    const float* colors2;  // second precomputed colour set of a dual render (else nullptr)
    int sh_staged;         // SH colours already in bin[i].xyz / clamp (sh_eval_kernel, gsr_sh.hip)
    const uint8_t* alive = nullptr;  // optional per-Gaussian mask, 0 = pruned (gsr_forward_dual_static_alive)
};

struct GeomPtrs {
    float4* rr;
    uint32_t* clamp;
    uint4* bin;
    uint32_t* tiles;
    uint32_t* offsets;
    uint32_t* blocksums;
    uint32_t* counters;
    uint32_t* wgsum;
    uint32_t* wgcull;
    static GeomPtrs at(void* base, const GeomLayout& L) {
        char* b = (char*)base;
        return {(float4*)(b + L.rr), (uint32_t*)(b + L.clamp), (uint4*)(b + L.bin), (uint32_t*)(b + L.tiles),
                (uint32_t*)(b + L.offsets), (uint32_t*)(b + L.blocksums), (uint32_t*)(b + L.counters),
                (uint32_t*)(b + L.wgsum), (uint32_t*)(b + L.wgcull)};
    }
};

// Render record accessors
struct RenderRec {
    float4 q0, q1, q2, q3;
};
__device__ __forceinline__ RenderRec load_rr(const float4* __restrict__ rr, uint32_t i) {
    const float4* r = rr + (size_t)RR_F4 * i;
    return {r[0], r[1], r[2], r[3]};
}
__device__ __forceinline__ uint2 rr_rect(const RenderRec& r) {
    return make_uint2(__float_as_uint(r.q2.w), __float_as_uint(r.q3.w));
}
// instance offset of Gaussian i: scanned workgroup base + workgroup-local part (q1.w)
__device__ __forceinline__ uint32_t rr_offset(const RenderRec& r, const uint32_t* blocksums, uint32_t i, int shift) {
    return blocksums[i >> shift] + __float_as_uint(r.q1.w);
}

// ------------------------------------------------------------ device math --
// The functions below restate forward.cu / backward.cu / auxiliary.h in
// standard notation.  They keep the operation order of oracle/gsr_oracle.c and
// disable FMA contraction so that preprocess outputs (radii, tile rects) are
// bit-identical to the float32 oracle.

__constant__ static const float kSH_C0 = 0.28209479177387814f;
__constant__ static const float kSH_C1 = 0.4886025119029199f;
__constant__ static const float kSH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                                             -1.0925484305920792f, 0.5462742152960396f};
__constant__ static const float kSH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                             0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                             -0.5900435899266435f};

__device__ __forceinline__ float3 xform4x3(float3 p, const float* m) {  // auxiliary.h:58-66
#pragma clang fp contract(off)
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}

__device__ __forceinline__ float4 xform4x4(float3 p, const float* m) {  // auxiliary.h:68-77
#pragma clang fp contract(off)
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

__device__ __forceinline__ float ndc2pix(float v, int S) {  // auxiliary.h:41-44 (double literals)
    return (float)((((double)v + 1.0) * S - 1.0) * 0.5);
}

__device__ __forceinline__ void get_rect(float px, float py, int r, int gx, int gy, int& x0, int& y0, int& x1,
                                         int& y1) {  // auxiliary.h:46-56
#pragma clang fp contract(off)
    float fr = (float)r;
    int a = (int)((px - fr) / (float)TILE_X);
    int b = (int)((py - fr) / (float)TILE_Y);
    float cx = px + fr; cx = cx + (float)TILE_X; cx = cx - 1.0f;
    float cy = py + fr; cy = cy + (float)TILE_Y; cy = cy - 1.0f;
    int c = (int)(cx / (float)TILE_X);
    int d = (int)(cy / (float)TILE_Y);
    a = max(a, 0); b = max(b, 0); c = max(c, 0); d = max(d, 0);
    x0 = min(a, gx); y0 = min(b, gy); x1 = min(c, gx); y1 = min(d, gy);
}

// Sigma = R S^2 R^T, R from the un-normalised quaternion (forward.cu:118-152)
__device__ __forceinline__ void rot_from_quat(float4 q, float R[3][3]) {
#pragma clang fp contract(off)
    float r = q.x, x = q.y, y = q.z, z = q.w;
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

__device__ __forceinline__ void cov3d_fwd(float3 s3, float mod, float4 q, float cov[6]) {
#pragma clang fp contract(off)
    float R[3][3];
    rot_from_quat(q, R);
    float s[3] = {mod * s3.x, mod * s3.y, mod * s3.z};
    float M[3][3];
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
        for (int i = 0; i < 3; i++) M[k][i] = s[k] * R[i][k];
    float S[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) S[i][j] = M[0][i] * M[0][j] + M[1][i] * M[1][j] + M[2][i] * M[2][j];
    cov[0] = S[0][0]; cov[1] = S[0][1]; cov[2] = S[0][2];
    cov[3] = S[1][1]; cov[4] = S[1][2]; cov[5] = S[2][2];
}

struct Proj {
    float tx, ty, tz, xmul, ymul;
    float Mx[2][3];  // J V3
    float a, b, c;   // cov2D (+0.3 low-pass on the diagonal)
};

// forward.cu:74-113 (EWA, with the +-1.3 tanfov clamp) in standard notation
__device__ __forceinline__ void cov2d_fwd(float3 mean, float fx, float fy, float tanx, float tany, const float c3[6],
                                          const float* view, Proj& o) {
#pragma clang fp contract(off)
    float3 t = xform4x3(mean, view);
    float limx = 1.3f * tanx, limy = 1.3f * tany;
    float txtz = t.x / t.z, tytz = t.y / t.z;
    o.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    o.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    o.tx = t.x; o.ty = t.y; o.tz = t.z;
    float J00 = fx / t.z, J02 = -(fx * t.x) / (t.z * t.z);
    float J11 = fy / t.z, J12 = -(fy * t.y) / (t.z * t.z);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        o.Mx[0][k] = J00 * view[4 * k + 0] + J02 * view[4 * k + 2];
        o.Mx[1][k] = J11 * view[4 * k + 1] + J12 * view[4 * k + 2];
    }
    float S[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float u0[3], u1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        u0[k] = S[k][0] * o.Mx[0][0] + S[k][1] * o.Mx[0][1] + S[k][2] * o.Mx[0][2];
        u1[k] = S[k][0] * o.Mx[1][0] + S[k][1] * o.Mx[1][1] + S[k][2] * o.Mx[1][2];
    }
    float a = o.Mx[0][0] * u0[0] + o.Mx[0][1] * u0[1] + o.Mx[0][2] * u0[2];
    float b = o.Mx[0][0] * u1[0] + o.Mx[0][1] * u1[1] + o.Mx[0][2] * u1[2];
    float c = o.Mx[1][0] * u1[0] + o.Mx[1][1] * u1[1] + o.Mx[1][2] * u1[2];
    o.a = a + 0.3f;
    o.b = b;
    o.c = c + 0.3f;
}

// conic = inverse of the (dilated) 2D covariance (forward.cu:219-224), shared by
// preprocess and the backward (which recomputes it rather than storing it):
// one contraction-free sequence, so both get the same bits.  Returns det.
__device__ __forceinline__ float conic_of(const Proj& pj, float& ca, float& cb, float& cc) {
#pragma clang fp contract(off)
    const float det = pj.a * pj.c - pj.b * pj.b;
    const float det_inv = 1.f / det;
    ca = pj.c * det_inv;
    cb = -pj.b * det_inv;
    cc = pj.a * det_inv;
    return det;
}

// forward.cu:20-71 (one channel at a time, same order as the oracle)
__device__ __forceinline__ void sh_fwd(int deg, float3 pos, const float* campos, const float* sh, float rgb[3],
                                       unsigned& clamped_bits) {
#pragma clang fp contract(off)
    float dx = pos.x - campos[0], dy = pos.y - campos[1], dz = pos.z - campos[2];
    float len = sqrtf(dx * dx + dy * dy + dz * dz);
    float x = dx / len, y = dy / len, z = dz / len;
    clamped_bits = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
#define S(k) sh[3 * (k) + ch]
        float res = kSH_C0 * S(0);
        if (deg > 0) {
            res = res - kSH_C1 * y * S(1) + kSH_C1 * z * S(2) - kSH_C1 * x * S(3);
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                res = res + (kSH_C2[0] * xy * S(4) + kSH_C2[1] * yz * S(5) + kSH_C2[2] * (2.f * zz - xx - yy) * S(6) +
                             kSH_C2[3] * xz * S(7) + kSH_C2[4] * (xx - yy) * S(8));
                if (deg > 2) {
                    res = res + (kSH_C3[0] * y * (3.f * xx - yy) * S(9) + kSH_C3[1] * xy * z * S(10) +
                                 kSH_C3[2] * y * (4.f * zz - xx - yy) * S(11) +
                                 kSH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy) * S(12) +
                                 kSH_C3[4] * x * (4.f * zz - xx - yy) * S(13) + kSH_C3[5] * z * (xx - yy) * S(14) +
                                 kSH_C3[6] * x * (xx - 3.f * yy) * S(15));
                }
            }
        }
#undef S
        res = res + 0.5f;
        if (res < 0.f) clamped_bits |= 1u << ch;
        rgb[ch] = fmaxf(res, 0.f);
    }
}

// Render-record form of the conic (written by preprocess, staged to LDS as is):
// prescaled so that
//   p2 = A' dx^2 + B' dx dy + C' dy^2 = log2(e) * power      (forward.cu:341)
// feeds v_exp_f32 (exp2) directly, laid out as
//   sa = q0 = (x, y, A', C'),  sb = q1 = (B', opacity, depth, -)
// so (x, y) - pixel and (A', C') * (dx, dy) are packed-f32 pairs.  Forward and
// backward read the same values and evaluate p2 through the same contraction-
// free sequence, so both see bit-identical alphas (the backward recovers T by
// dividing by 1 - alpha and must take exactly the forward's decisions).
constexpr float kLog2e = 1.4426950408889634f;
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr float K_AC = -0.5f * kLog2e;  // render-record scale of conic A and C
constexpr float K_B = -kLog2e;          // render-record scale of conic B
__device__ __forceinline__ v2f pix_delta(float4 sa, v2f pix) {
#pragma clang fp contract(off)
    return v2f{sa.x, sa.y} - pix;
}
// p2 = (A' dx) dx + (C' dy) dy, then + (B' dx) dy: forward.cu:341's order (the two square terms, of one
// sign, summed first; the cross term last), as FMAs on the packed (A' dx, C' dy).  The forward and the
// backward evaluate the same expression, so their alpha decisions agree bit for bit.  (Round 4 evaluated
// dx (A' dx + B' dy) + C' dy^2, one VALU less; its per-element gradient errors moved away from the
// float32 reference arithmetic's: config 4's worst dscales element 0.127 of its float32 error scale against
// 0.05 -- tools/alpha_forms.py replays both orders in the CPU oracle, profiles/r7_alpha_forms_cpu.txt.)
__device__ __forceinline__ float eval_p2(float4 sa, float4 sb, v2f d) {
#pragma clang fp contract(off)
    const v2f t = v2f{sa.z, sa.w} * d;  // (A' dx, C' dy)
    return __builtin_fmaf(sb.x * d.x, d.y, __builtin_fmaf(t.x, d.x, t.y * d.y));
}

// Pixel of thread tid within its 16x16 tile: wave w covers the 8x8 quadrant
// (w & 1, w >> 1); inside it, 16-lane row r covers the 4x4 block (r & 1, r >> 1),
// lanes row-major.  Tile block b = 4w + r is at block column 2(w & 1) + (r & 1),
// block row 2(w >> 1) + (r >> 1).  Small square footprints cull round Gaussians
// tightly (pixel-pair evaluations per instance on the config-3 frame, AABB cull:
// 16x4 strips 105, 8x8 quadrants 90, 4x4 blocks 48; tools/tile_balance.py).
__device__ __forceinline__ int tile_px(int tid) { return 8 * ((tid >> 6) & 1) + 4 * ((tid >> 4) & 1) + (tid & 3); }
__device__ __forceinline__ int tile_py(int tid) { return 8 * (tid >> 7) + 4 * ((tid >> 5) & 1) + ((tid >> 2) & 3); }

// Ellipse half-extents of the region where o * exp(-0.5 d^T Q d) >= 1/255
// (forward.cu:341-351), with margins that exceed the float32 error of
// evaluating `power` (grows with the conic's eccentricity kappa), so culling
// never changes a result.  Returns false for anything unusual (non-finite
// values, non-positive-definite conic, extreme eccentricity): no culling.
// Sets never = true when alpha <= o < 1/255 (never blended).
__device__ __forceinline__ bool alpha_extent(float4 a, float4 b, float& hx, float& hy, bool& never) {
    // conic from the render-record scaling (a few ulp off the preprocess values; the
    // margins below are orders of magnitude larger)
    const float A = a.z * (1.f / K_AC), B = b.x * (1.f / K_B), C = a.w * (1.f / K_AC), o = b.y;
    const float det = A * C - B * B;
    never = false;
    if (!(det > 0.f) || !(A > 0.f) || !isfinite(det) || !isfinite(a.x) || !isfinite(a.y) || !isfinite(o))
        return false;
    const float kappa = A * C / det;  // 1 / (1 - rho^2) >= 1
    if (!(kappa < 1e4f)) return false;
    const float t = 255.f * o;
    if (t < 0.999f) {
        never = true;
        return true;
    }
    const float tau = fmaxf(__logf(t), 0.f) * (1.001f + 4e-6f * kappa) + 1e-3f;
    hx = sqrtf(2.f * tau * C / det) * 1.001f + 0.01f;
    hy = sqrtf(2.f * tau * A / det) * 1.001f + 0.01f;
    return true;
}

// 16-bit mask of the 4x4-pixel blocks of a tile (bit 4w + r, layout of
// tile_px / tile_py) that a Gaussian can contribute to.
__device__ __forceinline__ uint32_t block_mask(float4 a, float4 b, float x0, float y0) {
    float hx = 0.f, hy = 0.f;
    bool never;
    if (!alpha_extent(a, b, hx, hy, never)) return 0xFFFFu;
    if (never) return 0u;
    const float xl = a.x - hx, xh = a.x + hx, yl = a.y - hy, yh = a.y + hy;
    uint32_t mx = 0, my = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        mx |= (xh >= x0 + 4.f * c && xl <= x0 + 4.f * c + 3.f) ? 1u << c : 0u;
        my |= (yh >= y0 + 4.f * c && yl <= y0 + 4.f * c + 3.f) ? 1u << c : 0u;
    }
    uint32_t m = 0;
#pragma unroll
    for (int bi = 0; bi < 16; bi++) {
        const int w = bi >> 2, r = bi & 3;
        const int cx = 2 * (w & 1) + (r & 1), cy = 2 * (w >> 1) + (r >> 1);
        m |= ((mx >> cx) & (my >> cy) & 1u) << bi;
    }
    return m;
}

// Sorted tile list entries: (4x4-block mask << 32) | Gaussian id.  The sort writes
// plain ids; render_fwd computes the ellipse-exact block_mask_exact of every entry
// it stages (one per thread, from the render record it loads anyway) and writes
// it into the entry's high half, where render_bwd (which only stages entries
// render_fwd staged) reads it.
typedef uint64_t PointEntry;
__device__ __forceinline__ uint32_t pe_id(PointEntry p) { return (uint32_t)p; }
__device__ __forceinline__ uint32_t pe_mask(PointEntry p) { return (uint32_t)(p >> 32); }

// block_mask with the ellipse instead of its bounding box: per block row the
// x-extent of the alpha >= 1/255 ellipse q(u) = A ux^2 + 2B ux uy + C uy^2 <= 2 tau
// over the row's y-span is exact (the left boundary (-B uy - sqrt(2 tau A - det
// uy^2)) / A is convex in uy, so its minimum over an interval is the leftmost
// point uy = B sqrt(2 tau / (det C)) clamped to the interval; symmetrically on
// the right); margins cover the float32 error.  ~10 % fewer pixel-pair
// evaluations than the box on a frame (tools/tile_balance.py).
// The per-Gaussian half of block_mask_exact.  hx < 0: no culling (full mask);
// hy < 0: never blended (empty mask).  The reciprocals, logarithm and square roots are the
// hardware's (v_rcp / v_log / v_sqrt_f32, ~1 ulp; the correctly rounded library forms cost ~10
// instructions each): the margins (x 1.001, + 1e-3 on tau, + 0.01 / 0.02 px) exceed their error by
// four orders of magnitude.
struct MaskGeom {
    float ax, ay, hx, hy, B, inv_A, twoA_tau, det, us, eps;
};
constexpr int MASK_GEOM_F = 10;
__device__ __forceinline__ MaskGeom mask_geom(float4 a, float4 b) {
    MaskGeom g;
    g.ax = a.x;
    g.ay = a.y;
    const float A = a.z * (1.f / K_AC), B = b.x * (1.f / K_B), C = a.w * (1.f / K_AC), o = b.y;
    const float det = A * C - B * B;
    const float rdet = __builtin_amdgcn_rcpf(det);
    const float kappa = A * C * rdet;  // 1 / (1 - rho^2) >= 1
    // anything unusual (non-finite values, a conic that is not positive definite, extreme eccentricity): no culling
    const bool bad = !(det > 0.f) || !(A > 0.f) || !isfinite(det) || !isfinite(a.x) || !isfinite(a.y) ||
                     !isfinite(o) || !(kappa < 1e4f);
    const float t = 255.f * o;
    const bool never = t < 0.999f;  // alpha <= o < 1/255: never blended
    // tau = ln(255 o), with the margin of the float32 error of `power` (grows with kappa)
    const float tau = fmaxf(__builtin_amdgcn_logf(t) * 0.69314718f, 0.f) * (1.001f + 4e-6f * kappa) + 1e-3f;
    const float k2 = 2.f * tau * rdet;
    const float hx = __builtin_amdgcn_sqrtf(k2 * C) * 1.001f + 0.01f;
    const float hy = __builtin_amdgcn_sqrtf(k2 * A) * 1.001f + 0.01f;
    g.hx = bad ? -1.f : (never ? 0.f : hx);
    g.hy = bad ? 0.f : (never ? -1.f : hy);
    g.B = B;
    g.det = det;
    g.twoA_tau = 2.f * tau * A;
    g.inv_A = __builtin_amdgcn_rcpf(A);
    g.us = B * __builtin_amdgcn_sqrtf(k2 * __builtin_amdgcn_rcpf(C));  // uy of the leftmost point (rightmost: -us)
    g.eps = 0.02f + 0.002f * hx;
    return g;
}
// Block row r (pixel centres y0 + 4r .. + 3): the ellipse's x-extent over the row's y-span
// [lo, hi] is [xmin, xmax]; the row's blocks are the columns c with x0 + 4c <= xmax and
// xmin <= x0 + 4c + 3, i.e. c in [ceil((xmin - x0 - 3) / 4), floor((xmax - x0) / 4)] (a rounding of
// the scaled differences can only widen that range: the mask stays conservative).
__device__ __forceinline__ uint32_t mask_of_geom(const MaskGeom& g, float x0, float y0) {
    if (g.hx < 0.f) return 0xFFFFu;
    if (g.hy < 0.f) return 0u;
    const float dy0 = y0 - g.ay;
    const float xa = g.ax - g.eps, xb = g.ax + g.eps;
    const float qx = -0.25f * (x0 + 3.f), px = -0.25f * x0;
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const float ylo = dy0 + 4.f * r, yhi = ylo + 3.f;
        const bool row = yhi >= -g.hy && ylo <= g.hy;  // the row meets the ellipse's y-span
        const float lo = fmaxf(ylo, -g.hy), hi = fminf(yhi, g.hy);
        const float ul = __builtin_amdgcn_fmed3f(g.us, lo, hi), ur = __builtin_amdgcn_fmed3f(-g.us, lo, hi);
        const float wl = __builtin_amdgcn_sqrtf(fmaxf(__builtin_fmaf(-g.det * ul, ul, g.twoA_tau), 0.f));
        const float wr = __builtin_amdgcn_sqrtf(fmaxf(__builtin_fmaf(-g.det * ur, ur, g.twoA_tau), 0.f));
        const float xmin = xa - __builtin_fmaf(g.B, ul, wl) * g.inv_A;
        const float xmax = xb + __builtin_fmaf(-g.B, ur, wr) * g.inv_A;
        // column range, clamped to [0, 4) / [-1, 3] in float before the conversion
        const int clo = (int)__builtin_amdgcn_fmed3f(ceilf(__builtin_fmaf(xmin, 0.25f, qx)), 0.f, 4.f);
        const int chi = (int)__builtin_amdgcn_fmed3f(floorf(__builtin_fmaf(xmax, 0.25f, px)), -1.f, 3.f);
        const uint32_t cm = row ? ((1u << (chi + 1)) - 1u) & ~((1u << clo) - 1u) : 0u;  // (chi + 1, clo in [0, 4])
        // block (column c, row r) -> bit 4w + rr, w = 2 (r >> 1) + (c >> 1), rr = 2 (r & 1) + (c & 1)
        const int base = 8 * (r >> 1) + 2 * (r & 1);
        m |= ((cm & 3u) << base) | ((cm >> 2) << (base + 4));
    }
    return m;
}
// Whether the ellipse can reach the tile at all (Camera::cull): mask_of_geom's test with the tile's whole
// pixel-centre span [y0, y0 + 15] as one row and [x0, x0 + 15] as one column -- a superset of the union of its
// sixteen block tests (it also admits the unit gaps between block rows / columns), so conservative like them
#ifndef GSR_CULL_EXACT
#define GSR_CULL_EXACT 0  // 1: the sixteen block tests (block_mask_exact != 0) instead
#endif
__device__ __forceinline__ bool tile_reached(const MaskGeom& g, float x0, float y0) {
    if (g.hx < 0.f) return true;
    if (g.hy < 0.f) return false;
    const float ylo = y0 - g.ay, yhi = ylo + 15.f;
    if (!(yhi >= -g.hy && ylo <= g.hy)) return false;
    const float lo = fmaxf(ylo, -g.hy), hi = fminf(yhi, g.hy);
    const float ul = __builtin_amdgcn_fmed3f(g.us, lo, hi), ur = __builtin_amdgcn_fmed3f(-g.us, lo, hi);
    const float wl = __builtin_amdgcn_sqrtf(fmaxf(__builtin_fmaf(-g.det * ul, ul, g.twoA_tau), 0.f));
    const float wr = __builtin_amdgcn_sqrtf(fmaxf(__builtin_fmaf(-g.det * ur, ur, g.twoA_tau), 0.f));
    const float xmin = (g.ax - g.eps) - __builtin_fmaf(g.B, ul, wl) * g.inv_A;
    const float xmax = (g.ax + g.eps) + __builtin_fmaf(-g.B, ur, wr) * g.inv_A;
    return xmax >= x0 && xmin <= x0 + 15.f;
}
__device__ __forceinline__ uint32_t block_mask_exact(float4 a, float4 b, float x0, float y0) {
    return mask_of_geom(mask_geom(a, b), x0, y0);
}
// 4-bit mask of the 8x8-pixel wave quadrants of a tile (bit w: pixel centres
// x0+8(w&1) .. +7, y0+8(w>>1) .. +7) that a Gaussian can contribute to.
__device__ __forceinline__ uint32_t quad_mask(float4 a, float4 b, float x0, float y0) {
    float hx = 0.f, hy = 0.f;
    bool never;
    if (!alpha_extent(a, b, hx, hy, never)) return 0xFu;
    if (never) return 0u;
    const float xl = a.x - hx, xh = a.x + hx, yl = a.y - hy, yh = a.y + hy;
    const uint32_t mx = (xh >= x0 && xl <= x0 + 7.f ? 1u : 0u) | (xh >= x0 + 8.f && xl <= x0 + 15.f ? 2u : 0u);
    const uint32_t my = (yh >= y0 && yl <= y0 + 7.f ? 1u : 0u) | (yh >= y0 + 8.f && yl <= y0 + 15.f ? 2u : 0u);
    // bit w = x half (w & 1) and y half (w >> 1)
    return (mx * (my & 1u)) | ((mx * (my >> 1)) << 2);
}

// inclusive scan over the 64 lanes: six DPP adds (row_shr 1 / 2 / 4 / 8 with bank masks: the in-row prefix; row_bcast 15 / 31 carry it across
// rows) instead of six lane shuffles through the LDS crossbar
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xe, true);   // row_shr:4 (banks 1-3)
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xc, true);   // row_shr:8 (banks 2-3)
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
    return v;
}
// number of set bits of `mask` below this lane (v_mbcnt_lo / hi)
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Ordered list of the batch entries whose quadrant mask has bit `w` (one wave
// builds its own list; ballot + popcount compaction, order preserved).
__device__ __forceinline__ int build_wave_list(const uint8_t* s_mask, int cnt, int w, int jmin, uint16_t* list) {
    const int lane = __lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
    int n = 0;
    for (int c = 0; c < cnt; c += 64) {
        const int j = c + lane;
        const bool bit = j < cnt && j >= jmin && ((s_mask[j] >> w) & 1u);
        const uint64_t bal = __ballot(bit);
        if (bit) list[n + __popcll(bal & lt)] = (uint16_t)j;
        n += __popcll(bal);
    }
    return n;
}

// The four ordered lists of a wave's 16-lane rows: list[r] gets the batch
// entries whose 16-bit block mask has bit 4w + r (ballot + popcount
// compaction, order preserved), skipping entries j < jmin[r].  Every list is
// then padded with `pad` (the index of a staged dummy entry that never blends)
// up to the returned length: the longest list rounded up to 4, so the rows of
// a wave step through their lists in lockstep with no validity tests.
// jmul scales the stored j (the walk may take it as an LDS byte offset; j * jmul must stay below 2^16).
template <typename MaskOf>
__device__ __forceinline__ int build_row_lists_by(MaskOf mask_of, int cnt, int w, const int (&jmin)[4],
                                                  uint16_t* list, int stride, uint16_t pad, uint32_t jmul = 1u) {
    const int lane = __lane_id();
    int n[4] = {0, 0, 0, 0};
    for (int c = 0; c < cnt; c += 64) {
        const int j = c + lane;
        const uint32_t m = j < cnt ? (mask_of(j) >> (4 * w)) & 0xFu : 0u;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            // the row's lanes as an SGPR mask: its lane prefix by v_mbcnt, the store predicated on it
            const uint64_t bal = __builtin_amdgcn_uicmp((m >> r) & 1u, 0u, 33 /* ne */) &
                                 __builtin_amdgcn_sicmp(j, jmin[r], 39 /* sge */);
            if (__builtin_amdgcn_inverse_ballot_w64(bal))
                list[r * stride + n[r] + (int)lanes_below(bal)] = (uint16_t)((uint32_t)j * jmul);
            n[r] += __popcll(bal);
        }
    }
    const int len = (max(max(n[0], n[1]), max(n[2], n[3])) + 3) & ~3;
#pragma unroll
    for (int r = 0; r < 4; r++)
        for (int p = n[r] + lane; p < len; p += 64) list[r * stride + p] = pad;
    return len;
}
__device__ __forceinline__ int build_row_lists(const uint16_t* s_mask, int cnt, int w, const int (&jmin)[4],
                                               uint16_t* list, int stride, uint16_t pad, uint32_t jmul = 1u) {
    return build_row_lists_by([&](int j) { return (uint32_t)s_mask[j]; }, cnt, w, jmin, list, stride, pad, jmul);
}

// Four consecutive entries of this lane's (padded) row list, per lane (VGPR).
struct RowGroup4 {
    int j[4];
};
__device__ __forceinline__ RowGroup4 load_row_group4(const uint16_t* row_list, int i) {
    const uint2 q = *reinterpret_cast<const uint2*>(&row_list[i]);
    RowGroup4 g;
    g.j[0] = (int)(q.x & 0xFFFFu);
    g.j[1] = (int)(q.x >> 16);
    g.j[2] = (int)(q.y & 0xFFFFu);
    g.j[3] = (int)(q.y >> 16);
    return g;
}

// Per-wave row lists of one batch: row r of wave w (tile block b = 4w + r) lists the entries j
// (< cnt) whose block mask has bit b and that lie before the block's last contributor (j >=
// jmin[r]), as (j | slot << 16) with slot = the entry's slot for block b; every wave also forms
// the batch's slot bases (exclusive scan of the masks' popcounts, redundantly per wave) and
// returns cnt = the longest prefix of the cmax staged entries whose slots fit in `budget`.
// Lists are padded to a common multiple of 4 with `pad`.  Wave 0 publishes the bases.
struct SlotLists {
    int len, cnt;
};
// jmul / smul scale the stored j and slot (the walk may take them as LDS byte offsets: j * record
// size, slot * slot size; both must stay below 2^16).
__device__ __forceinline__ SlotLists build_row_slot_lists(const uint16_t* s_mask, uint16_t* s_base, int cmax,
                                                         int budget, int w, const int (&jmin)[4], uint32_t* list,
                                                         int stride, uint32_t pad, uint32_t jmul = 1u,
                                                         uint32_t smul = 1u) {
    const int lane = __lane_id();
    const uint32_t below_w = (1u << (4 * w)) - 1u;  // blocks of the waves before this one
    int n[4] = {0, 0, 0, 0};
    uint32_t carry = 0;
    int cnt = 0;
    for (int c = 0; c < cmax; c += 64) {
        const int j = c + lane;
        const uint32_t mf = j < cmax ? (uint32_t)s_mask[j] : 0u;
        const uint32_t pc = __popc(mf);
        // inclusive prefix of the popcounts over the batch (DPP scan), the chunk total from lane 63
        const uint32_t incl = carry + wave_incl_scan(pc);
        const uint32_t base = incl - pc;
        const uint64_t fits = __builtin_amdgcn_sicmp(j, cmax, 40 /* slt */) &
                              __builtin_amdgcn_uicmp(incl, (uint32_t)budget, 37 /* ule */);
        cnt += __popcll(fits);
        carry = __builtin_amdgcn_readlane(incl, 63);
        if (w == 0 && __builtin_amdgcn_inverse_ballot_w64(fits)) s_base[j] = (uint16_t)base;
        const uint32_t m = (mf >> (4 * w)) & 0xFu;
        // the entry's word for the wave's first block; block r adds the slots of blocks r' < r it reaches
        const uint32_t w0 = __umul24((uint32_t)j, jmul) | (__umul24(base + __popc(mf & below_w), smul) << 16);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            // compare masks straight from v_cmp (a __ballot of a combined bool costs a select and a compare
            // more per row)
            const uint64_t bal = __builtin_amdgcn_uicmp((m >> r) & 1u, 0u, 33 /* ne */) &
                                 __builtin_amdgcn_sicmp(j, jmin[r], 39 /* sge */) & fits;
            if (__builtin_amdgcn_inverse_ballot_w64(bal))
                list[r * stride + n[r] + (int)lanes_below(bal)] = w0 + (__umul24(__popc(m & ((1u << r) - 1u)), smul) << 16);
            n[r] += __popcll(bal);
        }
    }
    const int len = (max(max(n[0], n[1]), max(n[2], n[3])) + 3) & ~3;
#pragma unroll
    for (int r = 0; r < 4; r++)
        for (int p = n[r] + lane; p < len; p += 64) list[r * stride + p] = pad;
    return {len, cnt};
}
// Four consecutive (j | slot << 16) words of this lane's row list.
__device__ __forceinline__ uint4 load_slot_group4(const uint32_t* row_list, int i) {
    return *reinterpret_cast<const uint4*>(&row_list[i]);
}

// In-kernel device-clock timing of one launch (graph-capturable, no extra
// kernels): clk = [start, sum of durations, launches, groups done, then 16 group
// counters KCLOCK_GROUP_STRIDE words apart].  The first workgroup stamps the
// start; workgroups count themselves done in 16 counters on separate cache lines
// (one counter for all 1200 workgroups serialised ~10 us of same-address
// atomics at the end of the launch), the last of each group counts the group,
// and the last group adds (now - start) and resets the counters for the next
// launch.  wall_clock64 runs at 100 MHz.
constexpr int KCLOCK_GROUP_STRIDE = 32;  // u64 words (256 B)
constexpr int KCLOCK_WORDS = 4 + 16 * KCLOCK_GROUP_STRIDE;
// Diagnostics build only (-DGSR_WGTIME=1, tools/wgtime.py; never in libgsr.so): every render
// workgroup records [start, end, HW_ID, XCC_ID] in its translation unit's g_wgtime table.
#ifndef GSR_WGTIME
#define GSR_WGTIME 0
#endif
#define GSR_WGTIME_MAX 16384
#if GSR_WGTIME
#define GSR_WGTIME_TABLE static __device__ unsigned long long g_wgtime[GSR_WGTIME_MAX][4];
#define GSR_WGTIME_MARK(end_)                                                                              \
    do {                                                                                                   \
        if (end_) __syncthreads();                                                                         \
        const unsigned b_ = blockIdx.y * gridDim.x + blockIdx.x;                                           \
        if (threadIdx.x == 0 && b_ < GSR_WGTIME_MAX) {                                                     \
            g_wgtime[b_][(end_) ? 1 : 0] = wall_clock64();                                                 \
            if (!(end_)) {                                                                                 \
                g_wgtime[b_][2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                     \
                g_wgtime[b_][3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);                    \
            }                                                                                              \
        }                                                                                                  \
    } while (0)
#else
#define GSR_WGTIME_TABLE
#define GSR_WGTIME_MARK(end_) do {} while (0)
#endif

__device__ __forceinline__ void kclock_begin(unsigned long long* clk) {
    if (clk && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        __hip_atomic_store(&clk[0], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Relaxed agent-scope atomics throughout: a release/acquire fence per workgroup
// costs an L2 writeback each on this multi-XCD part (~4% of the tracking step).
// Only workgroup 0 (the one that stamped the start) releases, and only the last
// one acquires.
__device__ __forceinline__ void kclock_end(unsigned long long* clk) {  // every thread of the block calls this
    if (!clk) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned nb = gridDim.x * gridDim.y, b = blockIdx.y * gridDim.x + blockIdx.x, g = b & 15u;
        const unsigned ngroups = nb < 16u ? nb : 16u;
        const unsigned gsize = nb / 16u + (g < nb % 16u ? 1u : 0u);
        unsigned long long* gc = clk + 4 + g * KCLOCK_GROUP_STRIDE;
        if (b == 0) __atomic_thread_fence(__ATOMIC_RELEASE);
        if (__hip_atomic_fetch_add(gc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
            __hip_atomic_store(gc, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_fetch_add(&clk[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1) {
                __atomic_thread_fence(__ATOMIC_ACQUIRE);
                const unsigned long long t0 = __hip_atomic_load(&clk[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                clk[1] += wall_clock64() - t0;
                clk[2] += 1;
                __hip_atomic_store(&clk[3], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// Cross-workgroup hand-off inside one launch without a release fence (an agent-
// scope release is an L2 writeback per workgroup on this multi-XCD part): the
// producers publish with agent-scope atomic stores (written through to the
// coherence point), wait for them (vmcnt 0), and count themselves done with one
// relaxed atomic; the last workgroup to arrive reads with agent-scope atomic
// loads and resets the counter for the next launch.
__device__ __forceinline__ void st_agent(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The last workgroup's fixed-order gather of per-workgroup partials: thread t adds values
// k < N of part[stride * b + k] for b = t, t + nt, t + 2 nt, ... in that order -- the same
// sums, bit for bit, as the plain loop (v starts at +0, and the out-of-range slots add +0),
// but CH partials' loads are in flight per memory round trip (the plain loop waited for each
// agent-scope load before issuing the next iteration's).
template <int N, int CH>
__device__ __forceinline__ void gather_partials(const float* part, int stride, int nb, int t, int nt,
                                                float (&v)[N]) {
    for (int b0 = t; b0 < nb; b0 += CH * nt) {
        float buf[CH][N];
#pragma unroll
        for (int u = 0; u < CH; u++) {
            const int b = b0 + u * nt;
#pragma unroll
            for (int k = 0; k < N; k++) buf[u][k] = b < nb ? ld_agent(part + (size_t)stride * b + k) : 0.f;
        }
#pragma unroll
        for (int u = 0; u < CH; u++)
#pragma unroll
            for (int k = 0; k < N; k++) v[k] += buf[u][k];
    }
}
// Same for large grids: 16 group counters (workgroup id mod 16, 64 B apart)
// and a top counter, so no single address takes more than ~nb/16 atomics
// (same-address atomics serialise: one counter for 1024 workgroups cost
// ~15 us).  ctr: ARRIVE_GROUPED_WORDS words, zero before the first launch.
constexpr int ARRIVE_STRIDE = 16;
constexpr int ARRIVE_GROUPED_WORDS = 17 * ARRIVE_STRIDE;
__device__ __forceinline__ bool last_block_arrive_grouped(uint32_t* ctr) {
    __shared__ uint32_t s_last2;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0)
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t nb = gridDim.x * gridDim.y * gridDim.z;
        const uint32_t b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, g = b & 15u;
        const uint32_t ngroups = nb < 16u ? nb : 16u, gsize = nb / 16u + (g < nb % 16u ? 1u : 0u);
        uint32_t* gc = ctr + ARRIVE_STRIDE * (1 + g);
        uint32_t last = 0;
        if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
            __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1) {
                __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        s_last2 = last;
    }
    __syncthreads();
    return s_last2 != 0u;
}

// Every thread of the workgroup calls this after its st_agent stores; true in
// the last workgroup of the grid to arrive (then *counter is back to 0).
__device__ __forceinline__ bool last_block_arrive(uint32_t* counter) {
    __shared__ uint32_t s_last;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0): this thread's stores have landed
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t nb = gridDim.x * gridDim.y * gridDim.z;
        const uint32_t old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == nb - 1 ? 1u : 0u;
        if (old == nb - 1) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return s_last != 0u;
}

// --------------------------------------------------------- wave64 helpers --
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

// Sum over each 16-lane row; every lane of the row receives the row total.
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x124>(v);  // row_ror:4
    v += dpp_mov<0x128>(v);  // row_ror:8
    return v;
}

// v_permlane32_swap: lanes 0-31 <- a(l)+a(l+32), lanes 32-63 <- b(l-32)+b(l)
__device__ __forceinline__ float swapsum32(float a, float b) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// v_permlane16_swap: within each 32-lane half, row0 <- a.r0+a.r1, row1 <- b.r0+b.r1
__device__ __forceinline__ float swapsum16(float a, float b) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Transposed wave reduction of 9 values: ~30 VALU instead of 9 full
// butterflies.  On return, for row = lane/16:
//   r0 row {0,1,2,3} holds the wave totals of v{0,2,1,3}
//   r1 row {0,1,2,3} holds the wave totals of v{4,6,5,7}
//   r8 row 0 holds the wave total of v8
__device__ __forceinline__ void wave_reduce9(const float v[9], float& r0, float& r1, float& r8) {
    float s01 = swapsum32(v[0], v[1]);
    float s23 = swapsum32(v[2], v[3]);
    float s45 = swapsum32(v[4], v[5]);
    float s67 = swapsum32(v[6], v[7]);
    float s8 = swapsum32(v[8], 0.f);
    float t0 = swapsum16(s01, s23);
    float t1 = swapsum16(s45, s67);
    float t2 = swapsum16(s8, 0.f);
    r0 = row16_sum(t0);
    r1 = row16_sum(t1);
    r8 = row16_sum(t2);
}
__device__ __forceinline__ int reduce9_slot_r0(int row) { return (row == 0) ? 0 : (row == 1 ? 2 : (row == 2 ? 1 : 3)); }

// Four consecutive entries of a wave's quadrant list as wave-uniform (SGPR)
// indices; entries past n repeat the first one and are flagged invalid.
struct Group4 {
    int j[4];
    bool valid[4];
};
__device__ __forceinline__ Group4 load_group4(const uint16_t* list, int i, int n) {
    const uint2 q = *reinterpret_cast<const uint2*>(&list[i]);
    const uint32_t q0 = __builtin_amdgcn_readfirstlane(q.x), q1 = __builtin_amdgcn_readfirstlane(q.y);
    Group4 g;
    g.j[0] = (int)(q0 & 0xFFFFu);
    g.j[1] = (int)(q0 >> 16);
    g.j[2] = (int)(q1 & 0xFFFFu);
    g.j[3] = (int)(q1 >> 16);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        g.valid[k] = i + k < n;
        if (!g.valid[k]) g.j[k] = g.j[0];
    }
    return g;
}

// Transposed reduction of 4 items x 9 values (v[item*9 + q]) over the 64 lanes:
// 18 permlane32 + 9 permlane16 swaps and 36 DPP adds (~2.5 VALU per value).
// On return row rho (= lane / 16) of r[q] holds, in all its 16 lanes, the wave
// total of value q of item rho.
__device__ __forceinline__ void wave_reduce4x9(const float (&v)[36], float (&r)[9]) {
    float r1[18];
#pragma unroll
    for (int n = 0; n < 18; n++) r1[n] = swapsum32(v[n], v[n + 18]);
#pragma unroll
    for (int m = 0; m < 9; m++) r[m] = row16_sum(swapsum16(r1[m], r1[m + 9]));
}

// Same for 2 items x 9 values (v[item*9 + q]).  On return, for row rho:
//   r[m] (m < 4) holds value q = m + 4*(rho & 1) of item rho >> 1,
//   r[4] holds value 8 of item rho >> 1 in rows 0 and 2 (rows 1, 3: zero).
__device__ __forceinline__ void wave_reduce2x9(const float (&v)[18], float (&r)[5]) {
    float r1[9];
#pragma unroll
    for (int q = 0; q < 9; q++) r1[q] = swapsum32(v[q], v[q + 9]);
#pragma unroll
    for (int m = 0; m < 4; m++) r[m] = row16_sum(swapsum16(r1[m], r1[m + 4]));
    r[4] = row16_sum(swapsum16(r1[8], 0.f));
}

// Transposed reduction of N values (N a multiple of 4) over the 64 lanes.
// On return row rho (= lane / 16) of r[m] (m < N/4) holds the wave total of
// v[m + rho * N / 4] in all 16 lanes of the row.
// Sums over each 16-lane row of 4 entries x NV values (v[e * NV + m], entry-major),
// transposed: a step pairs every lane with a partner differing in one lane class
// bit; the lane keeps one half of its values and adds the partner's copy of that
// half (2 selects + 1 DPP add per kept value), so each step halves what a lane
// holds.  Partners: row_ror:8 (lane ^ 8), row_half_mirror (i <-> 7 - i, which
// flips class bit 4), quad_perm [2,3,0,1] (^ 2), quad_perm [1,0,3,2] (^ 1).  The
// first two steps split the entries: lane class e = 2 (lane>>3 & 1) + (lane>>2 & 1)
// ends up with NV values of entry e; further transposed steps split m while the
// count stays even, plain DPP adds finish the rest.  Cost ~2.8 VALU per value
// against 4 for four plain DPP steps per value.
#ifndef GSR_DPP_BANKMASK
#define GSR_DPP_BANKMASK 1
#endif
#ifndef GSR_REDUCE_PIN
#define GSR_REDUCE_PIN 1
#endif
template <int NV>
struct RowReduce {
    static constexpr int V = 4 * NV;
    static constexpr int S = (V / 4) % 2 ? 2 : ((V / 8) % 2 ? 3 : 4);  // transposed steps (>= 2)
    static constexpr int R = V >> S;                                     // values per lane at the end
    // lanes that hold (and write) distinct results: class bits of the plain steps are 0
    static constexpr int WRITER_MASK = S == 2 ? 3 : (S == 3 ? 1 : 0);
};

template <int N, int CTRL>
__device__ __forceinline__ void row_tstep(const float* c, float* out, bool hi) {
#pragma unroll
    for (int i = 0; i < N / 2; i++) {
        const float keep = hi ? c[i + N / 2] : c[i];
        const float send = hi ? c[i] : c[i + N / 2];
        out[i] = keep + dpp_mov<CTRL>(send);
    }
}

// The same step for partners in the other half of a 4-lane-bank pair (row_ror:8: banks
// {0,1} <-> {2,3}; row_half_mirror: banks {0,2} <-> {1,3}): two v_add_f32_dpp whose
// bank masks write complementary lane halves -- lanes of the low half add the pair's c[i],
// lanes of the high half c[i + N/2] -- instead of two selects and one DPP add per value.
// Each pair is its own asm block and starts with s_nop 1: the VALU-write -> DPP-read hazard of its
// inputs needs 2 wait states, and the compiler, which does not see the DPP inside, may schedule the
// VALU that writes an input right before any of the blocks (a single s_nop ahead of the first block
// once let a select land between two blocks and the DPP read the stale register: the Fisher kernel's
// opacity column at 4 waves/SIMD).  Requires full EXEC.
template <int N>
__device__ __forceinline__ void row_tstep_ror8(const float* c, float* out) {
    static_assert(N % 2 == 0, "even value count");
#pragma unroll
    for (int i = 0; i < N / 2; i++)
        asm volatile("s_nop 1\n\t"
                     "v_add_f32_dpp %0, %1, %1 row_ror:8 row_mask:0xf bank_mask:0x3\n\t"
                     "v_add_f32_dpp %0, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xc"
                     : "=&v"(out[i]) : "v"(c[i]), "v"(c[i + N / 2]));
}
template <int N>
__device__ __forceinline__ void row_tstep_mirror(const float* c, float* out) {
    static_assert(N % 2 == 0, "even value count");
#pragma unroll
    for (int i = 0; i < N / 2; i++)
        asm volatile("s_nop 1\n\t"
                     "v_add_f32_dpp %0, %1, %1 row_half_mirror row_mask:0xf bank_mask:0x5\n\t"
                     "v_add_f32_dpp %0, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xa"
                     : "=&v"(out[i]) : "v"(c[i]), "v"(c[i + N / 2]));
}

// r[i] = row total of value (entry row_entry(lane), m = row_m0<NV>(lane) + i)
template <int NV>
__device__ __forceinline__ void row_reduce(const float (&v)[4 * NV], float (&r)[RowReduce<NV>::R], int lane) {
    using RR = RowReduce<NV>;
    constexpr int V = RR::V;
    float a[V / 2], b[V / 4];
#if GSR_DPP_BANKMASK
    row_tstep_ror8<V>(v, a);                    // row_ror:8, bank-masked pair adds
    row_tstep_mirror<V / 2>(a, b);              // row_half_mirror, bank-masked pair adds
#else
    row_tstep<V, 0x128>(v, a, lane & 8);        // row_ror:8
    row_tstep<V / 2, 0x141>(a, b, lane & 4);    // row_half_mirror
#endif
    if constexpr (RR::S == 2) {
#pragma unroll
        for (int i = 0; i < RR::R; i++) {
            float t = b[i] + dpp_mov<0x4E>(b[i]);
            r[i] = t + dpp_mov<0xB1>(t);
        }
    } else if constexpr (RR::S == 3) {
        float c[V / 8];
        row_tstep<V / 4, 0x4E>(b, c, lane & 2);
#pragma unroll
        for (int i = 0; i < RR::R; i++) r[i] = c[i] + dpp_mov<0xB1>(c[i]);
    } else {
        float c[V / 8];
        row_tstep<V / 4, 0x4E>(b, c, lane & 2);
        row_tstep<V / 8, 0xB1>(c, r, lane & 1);
    }
#if GSR_REDUCE_PIN
    // the totals formed here, in every lane: otherwise the compiler sinks the plain steps' adds into the
    // caller's writer-lane branch, where a DPP read of a disabled lane is invalid, so each step becomes
    // v_mov_b32_dpp (outside) + v_add_f32 (inside) instead of one v_add_f32_dpp (same operands, same sum)
#pragma unroll
    for (int i = 0; i < RR::R; i++) asm volatile("" : "+v"(r[i]));
#endif
}
__device__ __forceinline__ int row_entry(int lane) { return 2 * ((lane >> 3) & 1) + ((lane >> 2) & 1); }
template <int NV>
__device__ __forceinline__ int row_m0(int lane) {
    using RR = RowReduce<NV>;
    int m0 = 0;
    if (RR::S >= 3 && (lane & 2)) m0 += NV / 2;
    if (RR::S >= 4 && (lane & 1)) m0 += NV / 4;
    return m0;
}

template <int N>
__device__ __forceinline__ void wave_reduce_n(const float (&v)[N], float (&r)[N / 4]) {
    static_assert(N % 4 == 0, "pad to a multiple of 4");
    float r1[N / 2];
#pragma unroll
    for (int n = 0; n < N / 2; n++) r1[n] = swapsum32(v[n], v[n + N / 2]);
#pragma unroll
    for (int m = 0; m < N / 4; m++) r[m] = row16_sum(swapsum16(r1[m], r1[m + N / 4]));
}


__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Lanes of the wave whose 8-bit digit equals mine (valid lanes only).
__device__ __forceinline__ uint64_t wave_match8(uint32_t d, bool valid) {
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        uint64_t bal = __ballot(valid && ((d >> b) & 1u));
        m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    return m;
}

// Unsorted instance slot of (Gaussian g, tile tx,ty): duplicateWithKeys order
// (rasterizer_impl.cu:98-109) = offsets[g] + row-major index inside g's tile rect.
__device__ __forceinline__ uint32_t instance_slot(uint2 rect, uint32_t off, uint32_t tx, uint32_t ty) {
    const uint32_t x0 = rect.x & 0xFFFFu, y0 = rect.x >> 16, w = (rect.y & 0xFFFFu) - x0;
    return off + (ty - y0) * w + (tx - x0);
}

// ------------------------------------------------------- kernel launchers --
hipError_t launch_preprocess(const Camera& cam, const GaussIn& g, GeomPtrs geo, int* radii, uint32_t* counts,
                             bool lds_hist, int ntiles, int nb, hipStream_t s, unsigned long long* clk = nullptr);
hipError_t launch_tile_colscan(uint32_t* counts, int nb, int ntiles, uint32_t* tot, GeomPtrs geo, uint2* ranges,
                               uint32_t* status, bool tail, hipStream_t s, unsigned long long* clk = nullptr,
                               Gate gate = Gate{});
hipError_t launch_exclusive_scan(uint32_t* data, uint32_t n, uint32_t* total, hipStream_t s);
hipError_t launch_scan_counts(GeomPtrs geo, int nb, const uint32_t* tile_count, int tile_stride, int ntiles,
                              uint2* ranges, uint32_t* status, hipStream_t s);
hipError_t launch_duplicate(const Camera& cam, int P, GeomPtrs geo, uint64_t* keys, uint32_t* gid,
                            int nb, hipStream_t s);
// Speculative launches: kernels exit early when the device-side counters show
// num_rendered > cap_inst or a tile list longer than cap_tile (the host then
// re-launches with an exact buffer).  Pass UINT32_MAX to disable the guard.
struct SpecGuard {
    const uint32_t* counters;  // GeomLayout counters: [0] num_rendered, [2] longest tile list
    uint32_t cap_inst, cap_tile;
    __device__ __forceinline__ bool overflow() const {
        return counters[0] > cap_inst || counters[2] > cap_tile;
    }
};
// Backward-side check that the forward state is valid for a binning layout of
// `cap_inst` instances: counters[3] holds the longest tile list the sort path
// that produced point_list handles (TILE_SORT_CAP for render_fwd's tile sort,
// 0xffffffff for the radix fallback), set by the forward.  Only a static-mode
// forward can leave it failing; the backward kernels then do no work (no
// out-of-bounds access) and the gradients are zero.
struct BwdGuard {
    const uint32_t* counters;
    uint32_t cap_inst;
    __device__ __forceinline__ bool overflow() const {
        return counters[0] > cap_inst || counters[2] > counters[3];
    }
};
// Static-mode status rows are sticky across calls (HIP-graph replays): [0] and [2] keep the
// maximum num_rendered / longest tile list seen, [1] ORs the prefiltered violations, [3] the
// longest list the tile sort handles.  An overflow in any replay therefore stays visible until
// the caller zeroes the row.
__device__ __forceinline__ void status_merge(uint32_t* st, uint32_t n, uint32_t viol, uint32_t longest,
                                             uint32_t sort_cap) {
    if (n) atomicMax(st + 0, n);
    if (viol) atomicOr(st + 1, viol);
    if (longest) atomicMax(st + 2, longest);
    if (sort_cap) atomicMax(st + 3, sort_cap);
}
// lds_hist: the colscan ran without its scan tail; every workgroup scans the
// workgroup and tile totals (`tot`) itself, workgroup 0 writes ranges,
// counters and `status` (static mode; may be null).
// Row-major render schedule (the paths that do not run tile_plan).
hipError_t launch_identity_order(uint32_t* order, int ntiles, hipStream_t s);
hipError_t launch_duplicate_bucket(const Camera& cam, int P, GeomPtrs geo, uint2* ranges, const uint32_t* tot,
                                   uint32_t* cursor, bool lds_hist, int ntiles, uint64_t* keys, uint64_t* point_list,
                                   int nb, SpecGuard guard, uint32_t* status, hipStream_t s, unsigned long long* clk = nullptr);
hipError_t launch_radix_sort(uint64_t* keys[2], uint32_t* vals[2], uint32_t* hist, uint32_t n, int nsb, int npass,
                             hipStream_t s);
hipError_t launch_gather_ids(const uint32_t* vals, const uint32_t* gid, uint64_t* point_list, uint32_t n,
                             hipStream_t s);
// SplaTAM's tracking L1 loss (get_loss tracking=True, scripts/splatam.py:262-296) and its
// gradient images formed in the dual forward's per-pixel epilogue (gsr_track_forward_dual_static):
// the same mask / sums / sign gradient as gsr_track_l1_fwd_bwd, without reading the images back.
struct TrackL1 {
    const float* gt_im;     // [3,H,W]
    const float* gt_depth;  // [1,H,W]
    float sil_thres, w_im, w_depth;
    const float* seed;      // dL/dloss (device scalar, read when the kernel runs)
    float* dL_dim;          // [3,H,W]
    float* dL_dds;          // [3,H,W] (channels 1, 2 written as zero)
    float* part;            // zero-filled scratch: 2 partials per tile + arrival counters
    float* loss;            // device scalar
};
int track_l1_fused_scratch_floats(int ntiles);
// keys: the unsorted tile buckets (render_fwd sorts each tile's bucket into point_list in
// its prologue; the keys are scratch afterwards); nullptr when point_list is already
// sorted (radix fallback)
hipError_t launch_render_fwd(const Camera& cam, const uint2* ranges, uint64_t* point_list,
                             uint64_t* keys, GeomPtrs geo,
                             const float* colors2, float* final_T, uint32_t* n_contrib, float* out_color,
                             float* out_color2, float* out_depth, SpecGuard guard, hipStream_t s,
                             unsigned long long* clk = nullptr, const TrackL1* l1 = nullptr);
hipError_t launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* vis, hipStream_t s);
// the tracking iteration's forward (+ L1) and render backward in one launch (gsr_backward.hip); inst receives
// the pose-fused gauss_bwd's per-instance records (track_records_floats)
hipError_t launch_render_track(const Camera& cam, const uint2* ranges, uint64_t* point_list, uint64_t* keys,
                               GeomPtrs geo, float* final_T, uint32_t* n_contrib, float* out_color,
                               float* out_color2, float* out_depth, SpecGuard guard, const TrackL1& l1, float* inst,
                               hipStream_t s, unsigned long long* clk = nullptr);
int track_records_stride();  // floats per instance record of the tracking render backward (6)
// geometry reuse (gsr_forward_reuse): the render records' colours replaced by `colors` [P,3]
hipError_t launch_recolour(int P, const float* colors, GeomPtrs geo, hipStream_t s, Gate gate = Gate{});
// gated geometry reuse: geom [0, counters) + counters[0..3] and the radii from the previous call, the render
// records' colour quarter replaced by this call's colours (recolour fused into the copy)
hipError_t launch_reuse_copy(Gate gate, const void* prev_geom, void* geom, size_t geom_bytes, size_t tiles_offset,
                             const float* colors, const int* prev_radii, int* radii, int P, hipStream_t s);
// *word = e when any pair differs bitwise (word not cleared: see Gate)
hipError_t launch_epoch_mismatch(const struct EqualPairs& q, uint32_t* word, uint32_t e, hipStream_t s);
struct EqualPairs {
    int npairs;
    const float* a[8];
    const float* b[8];
    long long n[8];
};
hipError_t launch_bitwise_equal(const EqualPairs& q, int* flag, hipStream_t s);
// Per-(tile, Gaussian) instance record of the power-1 backward: the per-pair sums
// the launched render_bwd variant forms, packed (no slots for absent terms):
// [hx, hy, hxx, hxy, hyy | G dL/dalpha (o_op) | dch dp (o_c1, 3) | dch dq (o_c2, n_c2)]
// padded to an even count (float2 stores); 6 floats (24 B) for SplaTAM tracking.
struct RecLayout {
    int stride;                 // floats per record (even)
    int o_op, o_c1, o_c2, n_c2; // offsets, -1 when absent
};
RecLayout bwd_rec_layout(unsigned need, bool dual);
hipError_t launch_render_bwd(const Camera& cam, const uint2* ranges, const uint64_t* point_list, GeomPtrs geo,
                             const float* final_T, const uint32_t* n_contrib, const float* dL_dpix,
                             const float* colors2, const float* dL_dpix2, unsigned need, float* inst, BwdGuard guard,
                             hipStream_t s, unsigned long long* clk = nullptr);
// which optional per-pair sums render_bwd forms (the geometric ones always)
constexpr unsigned NEED_OPACITY = 1u, NEED_COLORS = 2u, NEED_COLORS2 = 4u;
constexpr unsigned NEED_DL2_CH0_ONLY = 8u;  // dL_dpix2 channels 1, 2 are promised zero
struct GradsOut {
    float* dmeans2D;
    float* dcolors;
    float* dopacity;
    float* dmeans3D;
    float* dcov3D;
    float* dsh;
    float* dscales;
    float* drot;
    float* dcolors2;  // second colour set of a dual render (nullptr otherwise)
};
// Tracking (gsr_track_backward_dual): the pose gradient -- and the pose Adam step -- fused into
// gauss_bwd, whose per-Gaussian dL/dmeans_cam, dL/d[z,1,z^2] and (anisotropic) dL/drotation
// never leave registers.  Same maths as track_transform_bwd_kernel (gsr_glue.hip).
struct PoseFuse {
    const float* means_world;  // [P,3]
    const float* unnorm_rot;   // [P,4]
    int scols;                 // 1: isotropic map (rotation does not depend on the pose)
    float* cam_q;              // frame's quaternion column (stride qs)
    float* cam_t;              // frame's translation column (stride qs)
    int qs;
    const float* w2c;          // [16] row-major, depth colours
    float* part;               // zero-filled scratch: 16 * nblocks partials + arrival counters
    float* adam_state;         // 15 floats (nullptr: write dq / dt instead)
    double lr_q, lr_t, beta1, beta2, eps;
    float* dq;                 // gradient outputs when adam_state == nullptr
    float* dt;
    const uint32_t* guard = nullptr;  // the forward's counters + capacity (Adam skipped on an overflow)
    uint32_t cap = 0;
    const float* loss = nullptr;      // best-candidate selection (PoseAdam::loss / best)
    float* best = nullptr;
    // log_scales [P, scols]: recompute each Gaussian's camera-frame mean / rotation / scale from the
    // world-frame map and the (pre-step) pose instead of reading GaussIn's arrays (the forward ran the
    // transform inside preprocess without storing them); nullptr: read GaussIn
    const float* ls = nullptr;
};
int pose_fuse_scratch_floats(int P);
hipError_t launch_gauss_bwd(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, const float* inst,
                            RecLayout rec, const GradsOut& out, BwdGuard guard, hipStream_t s,
                            const PoseFuse* pose = nullptr, unsigned long long* clk = nullptr);
hipError_t launch_selftest_reduce9(const float* in, float* out, hipStream_t s);
// gsr_sh.hip: SH colour stages with LDS-staged, coalesced coefficient traffic
bool sh_staged(const Camera& cam, const GaussIn& g);
hipError_t launch_sh_eval(const Camera& cam, const GaussIn& g, GeomPtrs geo, hipStream_t s);
// torch.optim.Adam's element update (foreach form: exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2)
// .addcmul_(g, g, 1-b2); p.addcdiv_(exp_avg, sqrt(exp_avg_sq)/sqrt(bc2) + eps, -lr/bc1)) -- the one
// definition the mapping step and the SH-stage colour step share, with no FP contraction (each
// operation rounded, like torch's separate kernels): the two kernels had contracted differently and
// diverged by an ulp from the second step on.
// Streams read or written once per iteration (optimizer parameters and moments, SH coefficients): with
// GSR_NT_STREAMS the loads and stores carry the nontemporal hint (the guide's streaming form: tools/micro/stream
// measures 6.33 TB/s for nontemporal float4 copies against 5.77 TB/s plain); the values are the same bits.
#ifndef GSR_NT_STREAMS
#define GSR_NT_STREAMS 1  // (config-4 mapping: sh_bwd 231 -> 204, map_transform_bwd 90 -> 67, sh_eval 69 -> 36 us)
#endif
typedef float gsr_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float ld_stream(const float* p) {
    if constexpr (GSR_NT_STREAMS != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ void st_stream(float* p, float v) {
    if constexpr (GSR_NT_STREAMS != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ float4 ld_stream(const float4* p) {
    if constexpr (GSR_NT_STREAMS != 0) {
        const gsr_f4v v = __builtin_nontemporal_load(reinterpret_cast<const gsr_f4v*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
    if constexpr (GSR_NT_STREAMS != 0) {
        const gsr_f4v w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<gsr_f4v*>(p));
    } else {
        *p = v;
    }
}

__device__ __forceinline__ float adam_update_elem(float p, float g, float& m, float& v, float ss, float w1, float beta2,
                                           float omb2, float bc2_sqrt, float eps) {
#pragma clang fp contract(off)
    const float mm = m + w1 * (g - m);
    float v2 = v * beta2;
    v2 = v2 + omb2 * g * g;
    const float denom = sqrtf(v2) / bc2_sqrt + eps;
    m = mm;
    v = v2;
    return p + ss * (mm / denom);
}

// The mapping optimizer's colour group applied to the SH coefficients inside sh_bwd (m == nullptr: none):
// torch.optim.Adam's element update with the scalars formed on the host like the other fused steps.
struct ShAdam {
    float* m = nullptr;
    float* v = nullptr;
    float ss = 0.f, w1 = 0.f, beta2 = 0.f, omb2 = 0.f, bc2_sqrt = 1.f, eps = 0.f;
    const uint32_t* guard = nullptr;  // the forward's status row / counters: skip the step on an overflow
    uint32_t cap = 0;
    uint32_t* halted = nullptr;       // gsr_map_adam.halted (sticky skip)
};
hipError_t launch_sh_bwd(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, const float* drgb,
                         float* dmeans3D, float* dsh, BwdGuard guard, hipStream_t s, const ShAdam& sa = ShAdam{});
// error reporting shared by the C entry points (gsr_last_error)
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* where);
// backward_power != 1 (the vendored renderCUDAFused semantics, backward.cu:850-1140)
// backward_power == 2 through per-instance second moments (gsr_backward.hip, gauss_bwd_mom_kernel)
int moments_record_floats(bool sh);
hipError_t launch_render_bwd_moments(const Camera& cam, const uint2* ranges, const uint64_t* point_list, GeomPtrs geo,
                                     const float* final_T, const uint32_t* n_contrib, const float* dL_dpix, bool sh,
                                     float* inst, BwdGuard guard, hipStream_t s);
hipError_t launch_gauss_bwd_moments(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii,
                                    const float* inst, const GradsOut& out, BwdGuard guard, hipStream_t s);
constexpr int JAC_FLOATS = 84;  // per-Gaussian linear chain pack, see gsr_backward_power.hip
constexpr int JAC_CONIC = 80;   // conic (A, B, C) inside the pack
int power_record_floats(int nsh);  // values stored per instance record
hipError_t launch_gauss_jac(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, float* jac,
                            hipStream_t s);
hipError_t launch_render_bwd_power(const Camera& cam, const GaussIn& g, const uint2* ranges,
                                   const uint64_t* point_list, GeomPtrs geo, const float* jac, const float* final_T,
                                   const uint32_t* n_contrib, const float* dL_dpix, int power, float* rec,
                                   BwdGuard guard, hipStream_t s);
// Fisher-selective backward_power path (dL/dmeans3D + dL/dopacity only, colours precomputed):
// gauss_mpack (3x5 chain matrix per Gaussian, MPACK_FLOATS), render_bwd_fisher (4-float records), sums
constexpr int MPACK_FLOATS = 16;
hipError_t launch_gauss_mpack(const Camera& cam, const GaussIn& g, const int* radii, float* mpack, hipStream_t s);
hipError_t launch_render_bwd_fisher(const Camera& cam, const uint2* ranges, const uint64_t* point_list, GeomPtrs geo,
                                    const float* mpack, const float* final_T, const uint32_t* n_contrib,
                                    const float* dL_dpix, int power, float* rec, BwdGuard guard, hipStream_t s);
hipError_t launch_gauss_bwd_fisher(int P, GeomPtrs geo, const int* radii, const float* rec, float* dmeans3D,
                                   float* dopacity, BwdGuard guard, hipStream_t s);
hipError_t launch_gauss_bwd_power(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii,
                                  const float* rec, const GradsOut& out, BwdGuard guard, hipStream_t s);

}  // namespace gsr
