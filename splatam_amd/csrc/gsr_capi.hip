// gsr_capi.hip -- extern "C" entry points of libgsr.so (see include/gsr.h).
//
// Host orchestration of one rasterization, the counterpart of
// CudaRasterizer::Rasterizer::{forward,backward,markVisible}
// (rasterizer_impl.cu:141-434).  Everything is enqueued on the caller's
// stream; the only host synchronisation is the read-back of num_rendered
// (the reference's cudaMemcpy at rasterizer_impl.cu:282), done through a
// pinned per-thread staging word.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gsr.h"
#include "../../include/gsr_glue.h"
#include "gsr_common.h"

#ifndef GSR_TILE_CULL
#define GSR_TILE_CULL 1  // Camera::cull for gsr_settings.binning == GSR_BINNING_CULLED (0: A/B builds without culling)
#endif
using namespace gsr;

namespace {
thread_local std::string g_last_error;
}  // namespace

namespace gsr {
int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* where) {
    return fail(GSR_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}
}  // namespace gsr

namespace {

struct Pinned {  // per-thread staging of the device counters + the event after the scan
    uint32_t* p = nullptr;   // (mapped, coherent: the bucketed duplicate stores into it, Camera::host_snap)
    uint32_t* dp = nullptr;  // its device address
    hipEvent_t ev = nullptr;
    ~Pinned() {
        if (p) (void)hipHostFree(p);
        if (ev) (void)hipEventDestroy(ev);
    }
};
// Host-side state is kept per device (the device of the launch stream), so one process (or one
// thread) may serve several GPUs: the pinned counter staging + its event (per thread and device),
// the binning-capacity hint (per device) and the stage timing (per device).
constexpr int kMaxDevices = 64;
int stream_device(hipStream_t s) {
    thread_local hipStream_t last_s = nullptr;
    thread_local int last_d = -1;
    if (last_d >= 0 && s == last_s && s != nullptr) return last_d;
    int d = 0;
    if (hipStreamGetDevice(s, &d) != hipSuccess && hipGetDevice(&d) != hipSuccess) d = 0;
    (void)hipGetLastError();
    if (d < 0 || d >= kMaxDevices) d = 0;
    last_s = s;
    last_d = d;
    return d;
}
int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDevices) d = 0;
    return d;
}
thread_local Pinned g_pinned[kMaxDevices];
// GSR_SNAP_COPY=1: the counters reach the host by a copy launched after the duplicate (A/B switch of Camera::host_snap)
const bool g_snap_copy = getenv("GSR_SNAP_COPY") && atoi(getenv("GSR_SNAP_COPY")) != 0;
struct RatioHint {
    std::atomic<double> v{3.0};  // last num_rendered / P (binning capacity hint)
};
RatioHint g_inst_ratio[kMaxDevices];
std::atomic<int> g_cus[kMaxDevices];  // CU count per device (render schedule round size), 0 = unknown
int device_cus(int dev) {
    int n = g_cus[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    (void)hipGetLastError();
    g_cus[dev].store(n, std::memory_order_relaxed);
    return n;
}

Camera make_camera(const gsr_settings* s) {
    Camera c;
    c.W = s->image_width;
    c.H = s->image_height;
    c.tan_fovx = s->tan_fovx;
    c.tan_fovy = s->tan_fovy;
    c.focal_y = (float)c.H / (2.0f * s->tan_fovy);  // rasterizer_impl.cu:222-223
    c.focal_x = (float)c.W / (2.0f * s->tan_fovx);
    c.gx = (c.W + TILE_X - 1) / TILE_X;
    c.gy = (c.H + TILE_Y - 1) / TILE_Y;
    c.view = s->viewmatrix;
    c.proj = s->projmatrix;
    c.campos = s->campos;
    c.bg = s->bg;
    c.scale_modifier = s->scale_modifier;
    c.sh_degree = s->sh_degree;
    c.prefiltered = s->prefiltered;
    return c;
}

GaussIn make_gauss(const gsr_gaussians* g) {
    GaussIn o;
    o.P = g->P;
    o.M = g->shs ? g->M : 0;
    o.means3D = g->means3D;
    o.shs = (g->shs && g->M > 0) ? g->shs : nullptr;
    o.colors = g->colors_precomp;
    o.opacities = g->opacities;
    o.scales = g->scales;
    o.rotations = g->rotations;
    o.cov3D = g->cov3D_precomp;
    o.colors2 = nullptr;
    o.sh_staged = 0;
    o.alive = nullptr;
    return o;
}

int validate(const gsr_settings* s, const gsr_gaussians* g, bool forward) {
    if (!s || !g) return fail(GSR_ERR_INVALID_ARG, "null settings or gaussians");
    if (g->P < 0) return fail(GSR_ERR_INVALID_ARG, "P must be >= 0");
    if (s->binning != GSR_BINNING_CULLED && s->binning != GSR_BINNING_REFERENCE)
        return fail(GSR_ERR_INVALID_ARG, "settings.binning must be GSR_BINNING_CULLED or GSR_BINNING_REFERENCE");
    if (s->image_width <= 0 || s->image_height <= 0) return fail(GSR_ERR_INVALID_ARG, "image size must be positive");
    if (s->image_width > 16 * 65535 || s->image_height > 16 * 65535)
        return fail(GSR_ERR_INVALID_ARG, "image too large for 16-bit tile coordinates");
    if (g->P == 0) return GSR_OK;
    if (!g->means3D) return fail(GSR_ERR_INVALID_ARG, "means3D is required");
    if (forward && !g->opacities) return fail(GSR_ERR_INVALID_ARG, "opacities are required");
    if (!s->viewmatrix || !s->projmatrix || !s->bg) return fail(GSR_ERR_INVALID_ARG, "camera matrices / bg missing");
    const bool has_sh = g->shs && g->M > 0;
    if (!g->colors_precomp && !has_sh)
        return fail(GSR_ERR_INVALID_ARG, "Please provide excatly one of either SHs or precomputed colors!");
    if (!g->colors_precomp && !s->campos) return fail(GSR_ERR_INVALID_ARG, "campos required for SH colours");
    if (has_sh && (s->sh_degree < 0 || s->sh_degree > 3 || (s->sh_degree + 1) * (s->sh_degree + 1) > g->M))
        return fail(GSR_ERR_INVALID_ARG, "sh_degree must be in [0,3] with (deg+1)^2 <= M");
    const bool has_sr = g->scales && g->rotations;
    if (!has_sr && !g->cov3D_precomp)
        return fail(GSR_ERR_INVALID_ARG,
                    "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    return GSR_OK;
}

void* obtain(gsr_alloc_fn alloc, void* ctx, int kind, size_t bytes) {
    void* p = alloc(ctx, kind, bytes);
    return p;
}

// ---- optional per-stage timing with hipEvents on the launch stream --------
struct TimedRec {
    int stage;
    long long units;
    hipEvent_t a, b;
};
struct Timing {
    bool on = false;
    // device-clock mode (graph-capturable): stamp kernels around the stages in `mask`
    // accumulate wall_clock64() ticks on the device: [start, sum, count, -] per stage
    bool clock = false;
    unsigned mask = 0;
    unsigned long long* dclock = nullptr;
    std::vector<TimedRec> recs;
    std::vector<hipEvent_t> pool;
    double ms[GSR_NUM_STAGES] = {};
    long long launches[GSR_NUM_STAGES] = {};
    long long units[GSR_NUM_STAGES] = {};
    ~Timing() {
        for (auto& r : recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
    hipEvent_t take() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
};
// Per device, not thread-local: torch runs autograd backward on its own thread.
Timing g_timing[kMaxDevices];
std::mutex g_timing_mu;

// resets as kernels: plain kernel nodes when captured in a HIP graph (small memcpy /
// memset nodes misbehaved on re-replay here)
__global__ void zero_words_kernel(uint32_t* __restrict__ p, size_t n) {
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) p[k] = 0u;
}
// zero-fill as a kernel (a memset node in a captured graph was not re-executed on replay)
hipError_t zero_async(void* p, size_t bytes, hipStream_t s) {
    const size_t n = bytes / 4;
    if (n == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<size_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(zero_words_kernel, dim3(blocks), dim3(256), 0, s, (uint32_t*)p, n);
    return hipGetLastError();
}

size_t kclock_bytes() { return (size_t)KCLOCK_WORDS * sizeof(unsigned long long) * GSR_NUM_STAGES; }

__global__ void stamp_begin_kernel(unsigned long long* c) { c[0] = wall_clock64(); }
__global__ void stamp_end_kernel(unsigned long long* c) {
    c[1] += wall_clock64() - c[0];
    c[2] += 1;
}

// Inside a stream capture an event record is only an internal dependency unless
// it is external: then it becomes a graph node re-recorded at every replay, so the
// stage times read after replays are those of the last replay.
hipError_t record_event(hipEvent_t e, hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive)
        return hipEventRecordWithFlags(e, s, hipEventRecordExternal);
    return hipEventRecord(e, s);
}

struct StageTimer {  // brackets the launches of one stage
    TimedRec rec{};
    hipStream_t s;
    bool on;
    unsigned long long* dc = nullptr;
    unsigned long long* kc = nullptr;  // in-kernel clock slot (stages whose kernel stamps itself)
    // in_kernel: the stage is one launch that takes kclock() and stamps itself
    // (kclock_begin / kclock_end), so no stamp kernels are added around it
    Timing& T;
    StageTimer(int stage, long long units, hipStream_t s_, bool in_kernel = false)
        : s(s_), on(false), T(g_timing[stream_device(s_)]) {
        on = T.on;
        if (!on) return;
        if (T.clock) {
            on = false;
            if ((T.mask >> stage) & 1u) {
                if (in_kernel) {
                    kc = T.dclock + (size_t)KCLOCK_WORDS * stage;
                } else {
                    dc = T.dclock + (size_t)KCLOCK_WORDS * stage;
                    hipLaunchKernelGGL(stamp_begin_kernel, dim3(1), dim3(1), 0, s, dc);
                }
            }
            return;
        }
        rec.stage = stage; rec.units = units;
        {
            std::lock_guard<std::mutex> lk(g_timing_mu);
            rec.a = T.take(); rec.b = T.take();
        }
        (void)record_event(rec.a, s);
    }
    unsigned long long* kclock() const { return kc; }
    ~StageTimer() {
        if (dc) hipLaunchKernelGGL(stamp_end_kernel, dim3(1), dim3(1), 0, s, dc);
        if (!on) return;
        (void)record_event(rec.b, s);
        std::lock_guard<std::mutex> lk(g_timing_mu);
        T.recs.push_back(rec);
    }
};

// The speculative launches learn their work units only after the host sync.
void g_timing_units(int dev, int stage, long long units) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    Timing& T = g_timing[dev];
    for (auto it = T.recs.rbegin(); it != T.recs.rend(); ++it)
        if (it->stage == stage) { it->units = units; break; }
}

void timing_drain(Timing& T) {  // caller holds g_timing_mu
    for (auto& r : T.recs) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            T.ms[r.stage] += ms;
            T.launches[r.stage] += 1;
            T.units[r.stage] += r.units;
        }
        T.pool.push_back(r.a);
        T.pool.push_back(r.b);
    }
    T.recs.clear();
    (void)hipGetLastError();  // an event that was never recorded must not leave a sticky error for torch
}

}  // namespace

namespace gsr {
int geom_pre_shift(int P) { return pre_shift_for(P, device_cus(current_device())); }
int current_device_cus() { return device_cus(current_device()); }
}  // namespace gsr

extern "C" {

int gsr_abi_version(void) { return GSR_ABI_VERSION; }

const char* gsr_last_error(void) { return g_last_error.c_str(); }

size_t gsr_geom_buffer_bytes(int P) { return GeomLayout::make(P).total; }
size_t gsr_geom_counters_offset(int P) { return GeomLayout::make(P).counters; }
size_t gsr_binning_buffer_bytes(int num_rendered, int W, int H) { return BinLayout::make(num_rendered, W, H).total; }
size_t gsr_image_buffer_bytes(int W, int H) { return ImgLayout::make(W, H).total; }

// gsr_forward_reuse_if_equal's inputs: the device comparison and the previous call's state
struct ReuseIn {
    EqualPairs pairs;
    int prev_num_rendered;
    const void* prev_geom;
    void* prev_binning;
    void* prev_image;
    const int* prev_radii;
    int* reused;
};

// the reuse form's render: the previous call's sorted lists (no sort), ranges, schedule and image buffer (its
// final_T / n_contrib rewritten with the same values), this call's records (the copied geometry)
static hipError_t launch_reuse_render(const Camera& cam, Gate gate, const ImgLayout& IL, const ReuseIn* reuse,
                                      const GeomPtrs& geo, float* out_color, float* out_depth, hipStream_t stream) {
    Camera cr = cam;
    cr.gate = gate;
    char* pib = (char*)reuse->prev_image;
    cr.tile_order = (const uint32_t*)(pib + IL.order);
    cr.rowmax = (uint32_t*)(pib + IL.rowmax);
    const SpecGuard rg{geo.counters, (uint32_t)reuse->prev_num_rendered, 0xFFFFFFFFu};
    return launch_render_fwd(cr, (const uint2*)(pib + IL.ranges), (uint64_t*)reuse->prev_binning, nullptr, geo,
                             nullptr, (float*)(pib + IL.final_T), (uint32_t*)(pib + IL.n_contrib), out_color, nullptr,
                             out_depth, rg, stream);
}

// colors2 != NULL: dual render (second colour set composited in the same pass, out_color2)
// capacity > 0: static mode -- binning buffer of `capacity` instances, no host
// synchronisation at all (graph-capturable); the device counters are copied to
// `status` and the call returns `capacity` (the layout size for the backward).
static int forward_impl(const gsr_settings* settings, const gsr_gaussians* gaussians, const float* colors2,
                        float* out_color, float* out_color2, float* out_depth, int* radii, gsr_alloc_fn alloc,
                        void* alloc_ctx, void* stream_, int capacity = 0, uint32_t* status = nullptr,
                        const TrackL1* l1 = nullptr, const TrackXf* xf = nullptr, float* track_inst = nullptr,
                        const uint8_t* alive = nullptr, const ReuseIn* reuse = nullptr) {
    int rc = validate(settings, gaussians, true);
    if (track_inst && (!l1 || !colors2 || capacity <= 0))
        return fail(GSR_ERR_INVALID_ARG, "the fused render backward needs the static dual forward with the L1 loss");
    if (rc != GSR_OK) return rc;
    if (!alloc) return fail(GSR_ERR_INVALID_ARG, "allocator callback required");
    // the fused tracking render may leave its images unstored (all three image pointers NULL): its loss and
    // backward consume them in registers
    const bool no_images = track_inst && !out_color && !out_color2 && !out_depth;
    if (!no_images) {
        if (!out_color || !out_depth) return fail(GSR_ERR_INVALID_ARG, "output image pointers required");
        if (colors2 && !out_color2) return fail(GSR_ERR_INVALID_ARG, "out_color2 required with colors2");
    }
    if (colors2 && gaussians->P > 0 && !gaussians->means3D) return fail(GSR_ERR_INVALID_ARG, "means3D is required");
    hipStream_t stream = (hipStream_t)stream_;
    const int dev = stream_device(stream);
    Pinned& pin = g_pinned[dev];
    Camera cam = make_camera(settings);
    GaussIn g = make_gauss(gaussians);
    g.colors2 = colors2;  // packed into the render records by preprocess (dual render)
    g.alive = alive;
    if (xf) g.xf = *xf;   // tracking transform fused into preprocess (g's arrays are then its outputs)
    const int P = g.P, W = cam.W, H = cam.H;
    const GeomLayout GL = GeomLayout::make(P);
    cam.pre_shift = GL.shift;
    const ImgLayout IL = ImgLayout::make(W, H);
    void* geom = obtain(alloc, alloc_ctx, GSR_BUF_GEOM, GL.total);
    void* img = obtain(alloc, alloc_ctx, GSR_BUF_IMAGE, IL.total);
    if (!geom || !img) return fail(GSR_ERR_ALLOC, "allocator returned NULL (geom/image buffer)");
    const GeomPtrs geo = GeomPtrs::at(geom, GL);
    char* ib = (char*)img;
    float* final_T = (float*)(ib + IL.final_T);
    uint32_t* n_contrib = (uint32_t*)(ib + IL.n_contrib);
    uint2* ranges = (uint2*)(ib + IL.ranges);
    uint32_t* tile_count = (uint32_t*)(ib + IL.tile_count);
    const int ntiles = cam.gx * cam.gy;
    uint32_t* order = (uint32_t*)(ib + IL.order);
    cam.tile_order = order;   // render schedule (tile_plan in the bucketed duplicate, else row-major)
    cam.rowmax = (uint32_t*)(ib + IL.rowmax);
    cam.sched_cus = device_cus(dev);
    uint32_t* cursor = tile_count + (size_t)ntiles * TILE_CTR_STRIDE;
    hipError_t e;
    // tile counts: per-workgroup LDS histograms + column scan (transient count matrix in SCRATCH),
    // or global atomics on padded counters when the histogram does not fit in LDS
    const bool lds_hist = ntiles <= MAX_LDS_TILES;
    uint32_t* cmat = nullptr;
    uint32_t* tile_tot = nullptr;
    if (lds_hist && P > 0) {
        cmat = (uint32_t*)obtain(alloc, alloc_ctx, GSR_BUF_SCRATCH, 4 * ((size_t)GL.nb * ntiles + ntiles));
        if (!cmat) return fail(GSR_ERR_ALLOC, "allocator returned NULL (tile count matrix)");
        tile_tot = cmat + (size_t)GL.nb * ntiles;
    } else if ((e = zero_async(tile_count, 8 * (size_t)ntiles * TILE_CTR_STRIDE, stream)) != hipSuccess) {
        return hip_fail(e, "memset tile counts");
    }
    static const bool force_radix_env = getenv("GSR_FORCE_RADIX") && atoi(getenv("GSR_FORCE_RADIX")) != 0;
    const bool force_radix = force_radix_env && capacity <= 0;
    // tile culling: a per-call choice (gsr_settings.binning), no process-wide mode
    cam.cull = (GSR_TILE_CULL && settings->binning != GSR_BINNING_REFERENCE) ? 1 : 0;
    cam.tail_exact = capacity <= 0 ? 1 : 0;  // (include/gsr.h: the culled instances, or padding in static mode)
    auto ensure_pinned = [&]() -> int {
        if (!pin.p) {
            // (portable: the buffer serves the launches on device `dev`, whatever device is current here)
            if ((e = hipHostMalloc((void**)&pin.p, 32,
                                   hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable)) != hipSuccess)
                return hip_fail(e, "hipHostMalloc");
            if ((e = hipHostGetDevicePointer((void**)&pin.dp, pin.p, 0)) != hipSuccess)
                return hip_fail(e, "hipHostGetDevicePointer");
        }
        if (!pin.ev) {  // created on the stream's device (the caller's current device is that device)
            int cur = 0;
            (void)hipGetDevice(&cur);
            if (cur != dev) (void)hipSetDevice(dev);
            e = hipEventCreateWithFlags(&pin.ev, hipEventDisableTiming);
            if (cur != dev) (void)hipSetDevice(cur);
            if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
        }
        return GSR_OK;
    };
    // num_rendered & co. to pinned host memory (eager mode): copied here, or (stored_by_kernel) already stored by
    // the launch just enqueued (Camera::host_snap)
    auto snapshot_counters = [&](bool stored_by_kernel) -> int {
        if (int r = ensure_pinned(); r != GSR_OK) return r;
        if (!stored_by_kernel &&
            (e = hipMemcpyAsync(pin.p, geo.counters, 32, hipMemcpyDeviceToHost, stream)) != hipSuccess)
            return hip_fail(e, "copy num_rendered");
        if ((e = hipEventRecord(pin.ev, stream)) != hipSuccess) return hip_fail(e, "record num_rendered");
        return GSR_OK;
    };
    // gated geometry reuse (gsr_forward_reuse_if_equal): the device compares this call's geometry with the
    // previous call's, both forms are enqueued with every launch gated on the result (counters[5]), and the
    // host learns which one ran from the counter copy it waits on anyway -- no second synchronisation.  (A
    // speculative form -- the reuse enqueued unconditionally, the host waiting on the comparison right after
    // it, the full forward only on a difference -- measured slower on the unchanged caller: its early wait
    // stalls the host before the call's render is enqueued, profiles/r10i_unit_reuse_forms.txt)
    const bool can_reuse = reuse && capacity <= 0 && !colors2 && !track_inst && !l1 && !xf && lds_hist &&
                           !force_radix && P > 0 && !sh_staged(cam, g);
    const bool gated = can_reuse;
    if (reuse && reuse->reused) *reuse->reused = 0;
    Gate eq_gate;
    uint32_t epoch = 0;
    if (gated) {
        // the comparison word is counters[5] of this call's geometry buffer, not cleared: the comparison stores
        // this call's epoch there on a difference, and no earlier content can equal the epoch (unique per call)
        static std::atomic<uint32_t> g_epoch{0};
        do epoch = g_epoch.fetch_add(1u, std::memory_order_relaxed) + 1u; while (epoch == 0u);
        uint32_t* word = geo.counters + 5;
        if ((e = launch_epoch_mismatch(reuse->pairs, word, epoch, stream)) != hipSuccess)
            return hip_fail(e, "geometry comparison");
        cam.gate = Gate{word, epoch, 1u};  // the full forward runs when the geometry differs ...
        eq_gate = Gate{word, epoch, 0u};   // ... the reuse form when it is equal
        if ((e = launch_reuse_copy(eq_gate, reuse->prev_geom, geom, GL.counters, GL.tiles, g.colors,
                                   reuse->prev_radii, radii, P, stream)) != hipSuccess)
            return hip_fail(e, "geometry reuse");
    }
    // the bucketed duplicate's workgroup 0 writes the render schedule (tile_plan); the other paths
    // render in row-major order
    Camera cplan = cam;
    cplan.tile_order_out = (lds_hist && !force_radix) ? order : nullptr;
    if ((!lds_hist || force_radix) && P > 0 && (e = launch_identity_order(order, ntiles, stream)) != hipSuccess)
        return hip_fail(e, "render schedule");
    // the bucketed duplicate does the instance / tile scans itself (lds_hist); otherwise a
    // scan launch does them, and the counters are final right after it
    const bool scan_in_duplicate = lds_hist && !force_radix;
    if (P > 0) {
        if (!radii) return fail(GSR_ERR_INVALID_ARG, "radii output required");
        {
            // (stage clocks in the device-clock mode: preprocess_kernel stamps itself; sh_eval is not timed)
            StageTimer t(GSR_STAGE_PREPROCESS, P, stream, true);
            if (sh_staged(cam, g)) {  // SH colours with coalesced coefficient reads, ahead of preprocess
                if ((e = launch_sh_eval(cam, g, geo, stream)) != hipSuccess) return hip_fail(e, "sh_eval");
                g.sh_staged = 1;
            }
            if ((e = launch_preprocess(cam, g, geo, radii, lds_hist ? cmat : tile_count, lds_hist, ntiles, GL.nb,
                                       stream, t.kclock())) != hipSuccess)
                return hip_fail(e, "preprocess");
        }
        {
            // the tile-count scans that give the ranges (the "ranges" stage of the bucketed path)
            StageTimer t(GSR_STAGE_RANGES, ntiles, stream, lds_hist);
            if (lds_hist) {  // column scan (+ instance / tile scans in the same launch unless scan_in_duplicate)
                if ((e = launch_tile_colscan(cmat, GL.nb, ntiles, tile_tot, geo, ranges,
                                             capacity > 0 ? status : nullptr, !scan_in_duplicate, stream,
                                             t.kclock(), cam.gate)) != hipSuccess)
                    return hip_fail(e, "tile count scan");
            } else if ((e = launch_scan_counts(geo, GL.nb, tile_count, TILE_CTR_STRIDE, ntiles, ranges,
                                               capacity > 0 ? status : nullptr, stream)) != hipSuccess) {
                return hip_fail(e, "scan");
            }
        }
        if (capacity <= 0 && !scan_in_duplicate && (rc = snapshot_counters(false)) != GSR_OK) return rc;
    } else {
        if ((e = zero_async(ranges, sizeof(uint2) * (size_t)ntiles, stream)) != hipSuccess)
            return hip_fail(e, "memset ranges");
    }
    if (P == 0) {  // rasterize_points.cu:67-81: zero outputs, forward not run (the sticky status keeps its rows)
        void* bin = obtain(alloc, alloc_ctx, GSR_BUF_BINNING, BinLayout::make(0, W, H).total);
        if (!bin) return fail(GSR_ERR_ALLOC, "allocator returned NULL (binning buffer)");
        if (l1) {  // the zero silhouette masks every pixel: loss 0 and zero gradient images, as get_loss gives
            const size_t img3 = sizeof(float) * 3 * (size_t)W * H;
            if ((e = zero_async(l1->loss, sizeof(float), stream)) != hipSuccess ||
                (l1->dL_dim && (e = zero_async(l1->dL_dim, img3, stream)) != hipSuccess) ||
                (l1->dL_dds && (e = zero_async(l1->dL_dds, img3, stream)) != hipSuccess))
                return hip_fail(e, "zero loss");
        }
        if (no_images) return 0;
        if ((e = zero_async(out_color, sizeof(float) * 3 * (size_t)W * H, stream)) != hipSuccess ||
            (e = zero_async(out_depth, sizeof(float) * (size_t)W * H, stream)) != hipSuccess ||
            (colors2 && (e = zero_async(out_color2, sizeof(float) * 3 * (size_t)W * H, stream)) != hipSuccess))
            return hip_fail(e, "zero outputs");
        return 0;
    }
    // Speculative binning + render: the binning buffer is sized from the last
    // calls' instances-per-Gaussian ratio, so everything is enqueued before the
    // host waits on num_rendered (the reference blocks right after the scan,
    // rasterizer_impl.cu:282, leaving the GPU idle while it launches the rest).
    const double ratio = g_inst_ratio[dev].v.load(std::memory_order_relaxed);
    const uint32_t cap = capacity > 0 ? (uint32_t)capacity
                                      : (uint32_t)std::min(2.0e9, std::max(1024.0, 1.5 * ratio * P));
    auto bin_ptrs = [&](void* bin, const BinLayout& BL, uint64_t** keys, uint32_t** vals, uint32_t*& gid,
                        uint64_t*& point_list, uint32_t*& hist) {
        char* bb = (char*)bin;
        keys[0] = (uint64_t*)(bb + BL.keys[0]);
        keys[1] = (uint64_t*)(bb + BL.keys[1]);
        vals[0] = (uint32_t*)(bb + BL.vals[0]);
        vals[1] = (uint32_t*)(bb + BL.vals[1]);
        gid = (uint32_t*)(bb + BL.gid);
        point_list = (uint64_t*)(bb + BL.point_list);
        hist = (uint32_t*)(bb + BL.hist);
    };
    uint64_t* keys[2];
    uint32_t* vals[2];
    uint32_t *gid, *hist;
    uint64_t* point_list;
    bool speculated = false;
    if (!force_radix) {
        const BinLayout SL = BinLayout::make((int)cap, W, H);
        void* bin = obtain(alloc, alloc_ctx, GSR_BUF_BINNING, SL.total);
        if (!bin) return fail(GSR_ERR_ALLOC, "allocator returned NULL (binning buffer)");
        bin_ptrs(bin, SL, keys, vals, gid, point_list, hist);
        const SpecGuard guard{geo.counters, cap, (uint32_t)TILE_SORT_CAP};
        const bool dup_snap = capacity <= 0 && scan_in_duplicate && !g_snap_copy;
        if (dup_snap) {
            if ((rc = ensure_pinned()) != GSR_OK) return rc;
            cplan.host_snap = pin.dp;
        }
        {
            StageTimer t(GSR_STAGE_DUPLICATE, P, stream, true);
            if ((e = launch_duplicate_bucket(cplan, P, geo, ranges, tile_tot, lds_hist ? cmat : cursor, lds_hist,
                                             ntiles, keys[0], point_list, GL.nb, guard,
                                             capacity > 0 ? status : nullptr,
                                             stream, t.kclock())) != hipSuccess)
                return hip_fail(e, "duplicate");
        }
        if (capacity <= 0 && scan_in_duplicate && (rc = snapshot_counters(dup_snap)) != GSR_OK) return rc;
        if (track_inst) {  // forward + L1 + the tracking render backward, one launch (render_track_kernel)
            StageTimer t(GSR_STAGE_RENDER_FWD, 0, stream, true);
            if ((e = launch_render_track(cam, ranges, point_list, keys[0], geo, no_images ? nullptr : final_T,
                                         n_contrib, out_color,
                                         out_color2, out_depth, guard, *l1, track_inst, stream, t.kclock())) !=
                hipSuccess)
                return hip_fail(e, "render (fused tracking forward + backward)");
        } else {
            StageTimer t(GSR_STAGE_RENDER_FWD, 0, stream, true);
            if ((e = launch_render_fwd(cam, ranges, point_list, keys[0], geo, colors2, final_T, n_contrib,
                                       out_color, out_color2, out_depth, guard, stream, t.kclock(), l1)) !=
                hipSuccess)
                return hip_fail(e, "render");
        }
        if (gated) {  // the reuse form's render: the previous call's sorted lists (no sort) and image buffer
            if ((e = launch_reuse_render(cam, eq_gate, IL, reuse, geo, out_color, out_depth, stream)) != hipSuccess)
                return hip_fail(e, "render (geometry reuse)");
        }
        speculated = true;
    }
    if (capacity > 0) {  // static mode: report, never wait (an overflow shows in status, outputs invalid)
        return (int)cap;
    }
    if ((e = hipEventSynchronize(pin.ev)) != hipSuccess) return hip_fail(e, "sync num_rendered");
    if (gated && pin.p[5] != epoch) {  // equal geometry: the reuse form ran (num_rendered is the previous call's)
        *reuse->reused = 1;
        return reuse->prev_num_rendered;
    }
    const uint32_t I = pin.p[0];
    const uint32_t longest = pin.p[2];
    if (pin.p[1] != 0)
        return fail(GSR_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    if (I > 0x7fffffffu) return fail(GSR_ERR_INVALID_ARG, "num_rendered overflows int32");
    g_inst_ratio[dev].v.store(P > 0 ? std::max(0.05, (double)I / P) : 1.0, std::memory_order_relaxed);
    const bool spec_ok = speculated && I <= cap && longest <= (uint32_t)TILE_SORT_CAP;
    if (spec_ok) {
        g_timing_units(dev, GSR_STAGE_SORT, I);
        g_timing_units(dev, GSR_STAGE_RENDER_FWD, I);
        return (int)I;
    }
    // exact re-launch (capacity overflow, a tile longer than the LDS sort, or forced radix)
    const BinLayout BL = BinLayout::make((int)I, W, H);
    void* bin = obtain(alloc, alloc_ctx, GSR_BUF_BINNING, BL.total);
    if (!bin) return fail(GSR_ERR_ALLOC, "allocator returned NULL (binning buffer)");
    bin_ptrs(bin, BL, keys, vals, gid, point_list, hist);
    const SpecGuard none{geo.counters, 0xffffffffu, 0xffffffffu};
    const bool tile_sorted = I > 0 && longest <= (uint32_t)TILE_SORT_CAP && !force_radix;
    cplan.host_snap = nullptr;  // (the host has read this call's counters: nothing may store into them later)
    if (tile_sorted) {
        {
            StageTimer t(GSR_STAGE_DUPLICATE, P, stream, true);
            if ((e = launch_duplicate_bucket(cplan, P, geo, ranges, tile_tot, lds_hist ? cmat : cursor, lds_hist,
                                             ntiles, keys[0], point_list, GL.nb, none, nullptr, stream,
                                             t.kclock())) !=
                hipSuccess)
                return hip_fail(e, "duplicate");
        }
    } else if (I > 0) {
        // fallback for tiles longer than the LDS sort: global stable LSD radix sort of (tile, depth)
        if ((e = hipMemsetD32Async((hipDeviceptr_t)(geo.counters + 3), 0xffffffffu, 1, stream)) != hipSuccess)
            return hip_fail(e, "sort path flag");
        {
            StageTimer t(GSR_STAGE_DUPLICATE, P, stream);
            if ((e = launch_duplicate(cam, P, geo, keys[0], gid, GL.nb, stream)) != hipSuccess)
                return hip_fail(e, "duplicate");
        }
        {
            StageTimer t(GSR_STAGE_SORT, I, stream);
            if ((e = launch_radix_sort(keys, vals, hist, I, BL.nsb, BL.npass, stream)) != hipSuccess)
                return hip_fail(e, "radix sort");
        }
        {
            StageTimer t(GSR_STAGE_RANGES, I, stream);
            if ((e = launch_gather_ids(vals[BL.final_buf], gid, point_list, I, stream)) != hipSuccess)
                return hip_fail(e, "gather ids");
        }
    }
    {
        StageTimer t(GSR_STAGE_RENDER_FWD, I, stream, true);
        if ((e = launch_render_fwd(cam, ranges, point_list, tile_sorted ? keys[0] : nullptr, geo, colors2,
                                   final_T, n_contrib, out_color, out_color2, out_depth, none, stream, t.kclock(),
                                   l1)) != hipSuccess)
            return hip_fail(e, "render");
    }
    return (int)I;
}

static int backward_impl(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                         const float* dL_dout_color, const float* colors2, const float* dL_dout_color2,
                         int num_rendered, const void* geom_buffer, const void* binning_buffer,
                         const void* image_buffer, int power, const gsr_grads* grads, float* dcolors2,
                         int dl2_channels, gsr_alloc_fn alloc, void* alloc_ctx, void* stream_,
                         const PoseFuse* pose = nullptr, const ShAdam* sh_adam = nullptr,
                         const float* pre_inst = nullptr) {
    int rc = validate(settings, gaussians, false);
    if (dl2_channels != 1 && dl2_channels != 3) return fail(GSR_ERR_INVALID_ARG, "dl2_channels must be 1 or 3");
    if (rc != GSR_OK) return rc;
    // (with pre-formed records -- the fused tracking render's -- the gradient images are not read)
    if (colors2 && !dL_dout_color2 && !pre_inst) return fail(GSR_ERR_INVALID_ARG, "dual backward needs dL_dout_color2");
    if (colors2 && power != 1) return fail(GSR_ERR_INVALID_ARG, "dual render supports backward_power == 1 only");
    if (!grads) return fail(GSR_ERR_INVALID_ARG, "grads required");
    if (num_rendered < 0) return fail(GSR_ERR_INVALID_ARG, "num_rendered must be >= 0");
    hipStream_t stream = (hipStream_t)stream_;
    Camera cam = make_camera(settings);
    const GaussIn g = make_gauss(gaussians);
    if (sh_adam && (power != 1 || !sh_staged(cam, g)))  // checked before any work is enqueued
        return fail(GSR_ERR_INVALID_ARG, "sh_adam needs staged SH colours (M == (D+1)^2) and power 1");
    const int P = g.P;
    if (P == 0) return GSR_OK;
    if (!geom_buffer || !image_buffer || !radii || (!dL_dout_color && !pre_inst))
        return fail(GSR_ERR_INVALID_ARG, "missing forward state");
    // the forward's render schedule (a permutation of the tiles; any order gives the same results)
    cam.tile_order = (const uint32_t*)((const char*)image_buffer + ImgLayout::make(cam.W, cam.H).order);
    cam.rowmax = (uint32_t*)((char*)const_cast<void*>(image_buffer) + ImgLayout::make(cam.W, cam.H).rowmax);
    cam.sched_cus = device_cus(current_device());  // (wave priority levels: one or several dispatch rounds)
    const GeomLayout GL = GeomLayout::make(P);
    cam.pre_shift = GL.shift;
    const ImgLayout IL = ImgLayout::make(cam.W, cam.H);
    const BinLayout BL = BinLayout::make(num_rendered, cam.W, cam.H);
    const GeomPtrs geo = GeomPtrs::at(const_cast<void*>(geom_buffer), GL);
    const char* ib = (const char*)image_buffer;
    const float* final_T = (const float*)(ib + IL.final_T);
    const uint32_t* n_contrib = (const uint32_t*)(ib + IL.n_contrib);
    const uint2* ranges = (const uint2*)(ib + IL.ranges);
    hipError_t e;
    GradsOut out{grads->dmeans2D, grads->dcolors, grads->dopacity, grads->dmeans3D,
                 grads->dcov3D,   grads->dsh,     grads->dscales,  grads->drotations};
    if (!out.dmeans3D && !pose) return fail(GSR_ERR_INVALID_ARG, "dmeans3D output pointer required");
    if (power != 1 && !out.dmeans2D && !out.dcolors && !out.dcov3D && !out.dscales && !out.drot && !out.dsh) {
        // Fisher-selective path: only dL/dmeans3D (+ dL/dopacity), the gradients the fork's Fisher
        // scoring reads (scripts/ros_handler.py:884-889)
        if (g.shs) return fail(GSR_ERR_INVALID_ARG, "backward_power != 1 with only dmeans3D / dopacity requested "
                                                    "needs precomputed colours (no SH)");
        if (num_rendered > 0 && !binning_buffer) return fail(GSR_ERR_INVALID_ARG, "missing binning buffer");
        if (!alloc) return fail(GSR_ERR_INVALID_ARG, "allocator callback required");
        const size_t mp_bytes = align_up(sizeof(float) * MPACK_FLOATS * (size_t)P, 256);
        const size_t rec_bytes = sizeof(float) * 4 * (size_t)num_rendered;
        char* scratch = (char*)obtain(alloc, alloc_ctx, GSR_BUF_SCRATCH, mp_bytes + rec_bytes);
        if (!scratch) return fail(GSR_ERR_ALLOC, "allocator returned NULL (backward scratch)");
        float* mpack = (float*)scratch;
        float* rec = (float*)(scratch + mp_bytes);
        const BwdGuard guard{geo.counters, (uint32_t)num_rendered};
        {
            StageTimer t(GSR_STAGE_GAUSS_BWD, P, stream);
            if ((e = launch_gauss_mpack(cam, g, radii, mpack, stream)) != hipSuccess)
                return hip_fail(e, "gaussian chain matrix");
        }
        if (num_rendered > 0) {
            const uint64_t* point_list = (const uint64_t*)((const char*)binning_buffer + BL.point_list);
            StageTimer t(GSR_STAGE_RENDER_BWD, num_rendered, stream);
            if ((e = launch_render_bwd_fisher(cam, ranges, point_list, geo, mpack, final_T, n_contrib, dL_dout_color,
                                              power, rec, guard, stream)) != hipSuccess)
                return hip_fail(e, "render backward (fisher)");
        }
        StageTimer t(GSR_STAGE_GAUSS_BWD, P, stream);
        if ((e = launch_gauss_bwd_fisher(P, geo, radii, rec, out.dmeans3D, out.dopacity, guard, stream)) != hipSuccess)
            return hip_fail(e, "gaussian backward (fisher)");
        return GSR_OK;
    }
    if (power == 2) {
        // backward_power == 2 (the fork's Fisher / Hessian scoring, scripts/ros_handler.py:839-902): each
        // pair's squared outputs are quadratic forms of its base values, so render_bwd forms per-instance
        // second moments and gauss_bwd_mom applies the forms per Gaussian (gsr_backward.hip).  Outputs
        // not requested (NULL) are skipped; dmeans3D is always formed.
        const bool sh = g.shs != nullptr;
        if (sh && (cam.sh_degree < 0 || cam.sh_degree > 3))
            return fail(GSR_ERR_INVALID_ARG, "unsupported sh_degree for backward_power != 1");
        if (num_rendered > 0 && !binning_buffer) return fail(GSR_ERR_INVALID_ARG, "missing binning buffer");
        if (!alloc) return fail(GSR_ERR_INVALID_ARG, "allocator callback required");
        const size_t rec_bytes = sizeof(float) * (size_t)moments_record_floats(sh) * (size_t)num_rendered;
        float* rec = nullptr;
        if (rec_bytes > 0) {
            rec = (float*)obtain(alloc, alloc_ctx, GSR_BUF_SCRATCH, rec_bytes);
            if (!rec) return fail(GSR_ERR_ALLOC, "allocator returned NULL (backward scratch)");
        }
        const BwdGuard guard{geo.counters, (uint32_t)num_rendered};
        if (num_rendered > 0) {
            const uint64_t* point_list = (const uint64_t*)((const char*)binning_buffer + BL.point_list);
            StageTimer t(GSR_STAGE_RENDER_BWD, num_rendered, stream);
            if ((e = launch_render_bwd_moments(cam, ranges, point_list, geo, final_T, n_contrib, dL_dout_color, sh, rec,
                                               guard, stream)) != hipSuccess)
                return hip_fail(e, "render backward (moments)");
        }
        StageTimer t(GSR_STAGE_GAUSS_BWD, P, stream);
        if ((e = launch_gauss_bwd_moments(cam, g, geo, radii, rec, out, guard, stream)) != hipSuccess)
            return hip_fail(e, "gaussian backward (moments)");
        return GSR_OK;
    }
    if (power != 1) {
        if (!out.dmeans2D || !out.dcolors || !out.dopacity || !out.dcov3D || !out.dscales || !out.drot)
            return fail(GSR_ERR_INVALID_ARG, "backward_power != 1 needs every gradient output pointer, or only "
                                             "dmeans3D (+ dopacity)");
        // per-pair powf before summation (renderCUDAFused, backward.cu:850-1140): gsr_backward_power.hip
        const int nsh = g.shs ? (cam.sh_degree + 1) * (cam.sh_degree + 1) : 0;
        const int nvp = power_record_floats(nsh);
        if (nvp < 0) return fail(GSR_ERR_INVALID_ARG, "unsupported sh_degree for backward_power != 1");
        if (num_rendered > 0 && !binning_buffer) return fail(GSR_ERR_INVALID_ARG, "missing binning buffer");
        if (!alloc) return fail(GSR_ERR_INVALID_ARG, "allocator callback required");
        const size_t jac_bytes = (sizeof(float) * JAC_FLOATS * (size_t)P + 255) / 256 * 256;
        const size_t rec_bytes = sizeof(float) * (size_t)nvp * (size_t)num_rendered;
        char* scratch = (char*)obtain(alloc, alloc_ctx, GSR_BUF_SCRATCH, jac_bytes + rec_bytes);
        if (!scratch) return fail(GSR_ERR_ALLOC, "allocator returned NULL (backward scratch)");
        float* jac = (float*)scratch;
        float* rec = (float*)(scratch + jac_bytes);
        {
            StageTimer t(GSR_STAGE_GAUSS_BWD, P, stream);
            if ((e = launch_gauss_jac(cam, g, geo, radii, jac, stream)) != hipSuccess)
                return hip_fail(e, "gaussian jacobian");
        }
        if (num_rendered > 0) {
            const uint64_t* point_list = (const uint64_t*)((const char*)binning_buffer + BL.point_list);
            StageTimer t(GSR_STAGE_RENDER_BWD, num_rendered, stream);
            if ((e = launch_render_bwd_power(cam, g, ranges, point_list, geo, jac, final_T, n_contrib, dL_dout_color,
                                             power, rec, BwdGuard{geo.counters, (uint32_t)num_rendered}, stream)) !=
                hipSuccess)
                return hip_fail(e, "render backward (power)");
        }
        StageTimer t(GSR_STAGE_GAUSS_BWD, P, stream);
        if ((e = launch_gauss_bwd_power(cam, g, geo, radii, rec, out, BwdGuard{geo.counters, (uint32_t)num_rendered},
                                        stream)) != hipSuccess)
            return hip_fail(e, "gaussian backward (power)");
        return GSR_OK;
    }
    float* inst = nullptr;
    // SH colours feed dL/dmeans3D through the view direction, so their sums are needed with SH
    // pose-fused tracking backward: the pose needs the geometric sums and the depth colours only
    const unsigned need = pose ? (NEED_COLORS2 | NEED_DL2_CH0_ONLY)
                               : (out.dopacity ? NEED_OPACITY : 0u) | ((out.dcolors || g.shs) ? NEED_COLORS : 0u) |
                                     (dcolors2 ? NEED_COLORS2 : 0u) | (dl2_channels == 1 ? NEED_DL2_CH0_ONLY : 0u);
    const RecLayout rec = bwd_rec_layout(need, colors2 != nullptr);
    // staged SH backward: gauss_bwd leaves dL/dcolor in a scratch array, sh_bwd turns it into dsh and the
    // view-direction term of dL/dmeans3D (gsr_sh.hip)
    const bool shs_staged = sh_staged(cam, g);
    // pre_inst: the records were formed by the fused tracking render (render_track_kernel)
    const size_t rec_bytes = pre_inst ? 0 : align_up(sizeof(float) * rec.stride * (size_t)num_rendered, 256);
    const size_t scratch_bytes = (num_rendered > 0 ? rec_bytes : 0) + (shs_staged ? sizeof(float) * 3 * (size_t)P : 0);
    char* scratch = nullptr;
    if (scratch_bytes > 0) {
        if (!alloc) return fail(GSR_ERR_INVALID_ARG, "allocator callback required");
        scratch = (char*)obtain(alloc, alloc_ctx, GSR_BUF_SCRATCH, scratch_bytes);
        if (!scratch) return fail(GSR_ERR_ALLOC, "allocator returned NULL (backward scratch)");
    }
    float* drgb = shs_staged ? (float*)(scratch + (num_rendered > 0 ? rec_bytes : 0)) : nullptr;
    if (pre_inst) {
        if (!pose || rec.stride != track_records_stride())
            return fail(GSR_ERR_INVALID_ARG, "precomputed records are the pose-fused tracking backward's only");
        inst = const_cast<float*>(pre_inst);
    } else if (num_rendered > 0) {
        if (!binning_buffer) return fail(GSR_ERR_INVALID_ARG, "missing binning buffer");
        inst = (float*)scratch;
        const char* bb = (const char*)binning_buffer;
        const uint64_t* point_list = (const uint64_t*)(bb + BL.point_list);
        StageTimer t(GSR_STAGE_RENDER_BWD, num_rendered, stream, true);
        if ((e = launch_render_bwd(cam, ranges, point_list, geo, final_T, n_contrib, dL_dout_color, colors2,
                                   dL_dout_color2, need, inst, BwdGuard{geo.counters, (uint32_t)num_rendered},
                                   stream, t.kclock())) != hipSuccess)
            return hip_fail(e, "render backward");
    }
    out.dcolors2 = dcolors2;
    {
        // (device-clock mode: gauss_bwd_kernel stamps itself; a staged sh_bwd after it is not timed)
        StageTimer t(GSR_STAGE_GAUSS_BWD, P, stream, true);
        const BwdGuard guard{geo.counters, (uint32_t)num_rendered};
        GaussIn gc = g;
        GradsOut oc = out;
        if (shs_staged) {  // the chain without SH: dL/dcolor to scratch, dsh by sh_bwd below
            gc.shs = nullptr;
            gc.M = 0;
            oc.dcolors = drgb;
            oc.dsh = nullptr;
        }
        PoseFuse pc;
        if (pose) {
            pc = *pose;
            pc.guard = geo.counters;
        }
        if ((e = launch_gauss_bwd(cam, gc, geo, radii, inst, rec, oc, guard, stream, pose ? &pc : nullptr,
                                  t.kclock())) != hipSuccess)
            return hip_fail(e, "gaussian backward");
        // the colour step guards on this call's own forward counters (not a sticky status row: an
        // overflow in an earlier replay must not skip the steps of later valid iterations)
        ShAdam sa = sh_adam ? *sh_adam : ShAdam{};
        if (sh_adam) {
            sa.guard = geo.counters;
            sa.cap = (uint32_t)num_rendered;
        }
        if (shs_staged && (e = launch_sh_bwd(cam, g, geo, radii, drgb, out.dmeans3D, out.dsh, guard, stream, sa)) !=
                              hipSuccess)
            return hip_fail(e, "sh backward");
    }
    return GSR_OK;
}

int gsr_track_forward_scratch_floats(int image_width, int image_height) {
    const int gx = (image_width + TILE_X - 1) / TILE_X, gy = (image_height + TILE_Y - 1) / TILE_Y;
    return track_l1_fused_scratch_floats(gx * gy > 0 ? gx * gy : 1);
}

int gsr_track_forward_dual_static(const gsr_settings* settings, const gsr_gaussians* gaussians, const float* colors2,
                                  int capacity, unsigned* status, float* out_color, float* out_color2,
                                  float* out_depth, int* radii, const float* gt_im, const float* gt_depth,
                                  float sil_thres, float w_im, float w_depth, const float* dL_dloss, float* loss,
                                  float* dL_dim, float* dL_ddepth_sil, float* scratch, gsr_alloc_fn alloc,
                                  void* alloc_ctx, void* stream) {
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    if (capacity <= 0 || !status) return fail(GSR_ERR_INVALID_ARG, "static mode needs capacity > 0 and status");
    if (!gt_im || !gt_depth || !dL_dloss || !loss || !dL_dim || !dL_ddepth_sil || !scratch)
        return fail(GSR_ERR_INVALID_ARG, "track_forward_dual_static: null pointer");
    const TrackL1 l1{gt_im, gt_depth, sil_thres, w_im, w_depth, dL_dloss, dL_dim, dL_ddepth_sil, scratch, loss};
    return forward_impl(settings, gaussians, colors2, out_color, out_color2, out_depth, radii, alloc, alloc_ctx,
                        stream, capacity, status, &l1);
}

static int track_forward_xf(const gsr_settings* settings, const gsr_gaussians* gaussians, float* colors2,
                            const gsr_track_xform* xform, int capacity, unsigned* status, float* out_color,
                            float* out_color2, float* out_depth, int* radii, const float* gt_im, const float* gt_depth,
                            float sil_thres, float w_im, float w_depth, const float* dL_dloss, float* loss,
                            float* dL_dim, float* dL_ddepth_sil, float* scratch, gsr_alloc_fn alloc, void* alloc_ctx,
                            void* stream, float* inst_records);

int gsr_track_forward_dual_static_xf(const gsr_settings* settings, const gsr_gaussians* gaussians, float* colors2,
                                     const gsr_track_xform* xform, int capacity, unsigned* status, float* out_color,
                                     float* out_color2, float* out_depth, int* radii, const float* gt_im,
                                     const float* gt_depth, float sil_thres, float w_im, float w_depth,
                                     const float* dL_dloss, float* loss, float* dL_dim, float* dL_ddepth_sil,
                                     float* scratch, gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    return track_forward_xf(settings, gaussians, colors2, xform, capacity, status, out_color, out_color2, out_depth,
                            radii, gt_im, gt_depth, sil_thres, w_im, w_depth, dL_dloss, loss, dL_dim, dL_ddepth_sil,
                            scratch, alloc, alloc_ctx, stream, nullptr);
}

int gsr_track_records_floats(int capacity) { return track_records_stride() * (capacity > 1 ? capacity : 1); }

int gsr_track_forward_backward_dual_static_xf(const gsr_settings* settings, const gsr_gaussians* gaussians,
                                              float* colors2, const gsr_track_xform* xform, int capacity,
                                              unsigned* status, float* out_color, float* out_color2,
                                              float* out_depth, int* radii, const float* gt_im,
                                              const float* gt_depth, float sil_thres, float w_im, float w_depth,
                                              const float* dL_dloss, float* loss, float* scratch,
                                              float* inst_records, gsr_alloc_fn alloc, void* alloc_ctx,
                                              void* stream) {
    if (!inst_records) return fail(GSR_ERR_INVALID_ARG, "track_forward_backward_dual_static_xf: null records");
    // the gradient images are not formed (the backward runs from the registers); the L1 epilogue's
    // pointers to them are never dereferenced.  out_color, out_color2 and out_depth all NULL: the rendered
    // images (and final_T / n_contrib / the block maxima of the image buffer) are not stored either
    return track_forward_xf(settings, gaussians, colors2, xform, capacity, status, out_color, out_color2, out_depth,
                            radii, gt_im, gt_depth, sil_thres, w_im, w_depth, dL_dloss, loss, nullptr, nullptr,
                            scratch, alloc, alloc_ctx, stream, inst_records);
}

static int track_forward_xf(const gsr_settings* settings, const gsr_gaussians* gaussians, float* colors2,
                            const gsr_track_xform* xform, int capacity, unsigned* status, float* out_color,
                            float* out_color2, float* out_depth, int* radii, const float* gt_im, const float* gt_depth,
                            float sil_thres, float w_im, float w_depth, const float* dL_dloss, float* loss,
                            float* dL_dim, float* dL_ddepth_sil, float* scratch, gsr_alloc_fn alloc, void* alloc_ctx,
                            void* stream, float* inst_records) {
    if (!xform || !gaussians) return fail(GSR_ERR_INVALID_ARG, "track_forward_dual_static_xf: null pointer");
    const gsr_track_xform& x = *xform;
    if ((x.scale_cols != 1 && x.scale_cols != 3) || x.q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "track_forward_dual_static_xf: bad sizes");
    if (gaussians->P > 0 && (!x.means_world || !x.unnorm_rot || !x.logit_opac || !x.log_scales || !x.cam_q ||
                             !x.cam_t || !x.w2c || !gaussians->means3D || !gaussians->rotations ||
                             !gaussians->opacities || !gaussians->scales || !colors2))
        return fail(GSR_ERR_INVALID_ARG, "track_forward_dual_static_xf: null pointer");
    if (gaussians->shs || gaussians->cov3D_precomp)
        return fail(GSR_ERR_INVALID_ARG, "track_forward_dual_static_xf: precomputed colours, scales / rotations only");
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    if (capacity <= 0 || !status) return fail(GSR_ERR_INVALID_ARG, "static mode needs capacity > 0 and status");
    // (the fused forward + backward, inst_records set, forms no gradient images: dL_dim / dL_ddepth_sil NULL)
    if (!gt_im || !gt_depth || !dL_dloss || !loss || (!inst_records && (!dL_dim || !dL_ddepth_sil)) || !scratch)
        return fail(GSR_ERR_INVALID_ARG, "track_forward_dual_static_xf: null pointer");
    TrackXf xf;
    xf.mw = x.means_world; xf.ur = x.unnorm_rot; xf.lo = x.logit_opac; xf.ls = x.log_scales;
    xf.scols = x.scale_cols; xf.cq = x.cam_q; xf.ct = x.cam_t; xf.qs = x.q_stride; xf.w2c = x.w2c;
    xf.store = x.store_rendervars != 0;
    const TrackL1 l1{gt_im, gt_depth, sil_thres, w_im, w_depth, dL_dloss, dL_dim, dL_ddepth_sil, scratch, loss};
    return forward_impl(settings, gaussians, colors2, out_color, out_color2, out_depth, radii, alloc, alloc_ctx,
                        stream, capacity, status, &l1, &xf, inst_records, x.alive);
}

int gsr_forward_dual_static_xf(const gsr_settings* settings, const gsr_gaussians* gaussians, float* colors2,
                               const gsr_track_xform* xform, int capacity, unsigned* status, float* out_color,
                               float* out_color2, float* out_depth, int* radii, gsr_alloc_fn alloc, void* alloc_ctx,
                               void* stream) {
    if (!xform || !gaussians) return fail(GSR_ERR_INVALID_ARG, "forward_dual_static_xf: null pointer");
    const gsr_track_xform& x = *xform;
    if ((x.scale_cols != 1 && x.scale_cols != 3) || x.q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "forward_dual_static_xf: bad sizes");
    if (!x.store_rendervars) return fail(GSR_ERR_INVALID_ARG, "forward_dual_static_xf: store_rendervars must be 1");
    if (gaussians->shs || gaussians->cov3D_precomp)
        return fail(GSR_ERR_INVALID_ARG, "forward_dual_static_xf: precomputed colours, scales / rotations only");
    if (gaussians->P > 0 && (!x.means_world || !x.unnorm_rot || !x.logit_opac || !x.log_scales || !x.cam_q ||
                             !x.cam_t || !x.w2c || !gaussians->means3D || !gaussians->rotations ||
                             !gaussians->opacities || !gaussians->scales || !gaussians->colors_precomp))
        return fail(GSR_ERR_INVALID_ARG, "forward_dual_static_xf: null pointer");
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    if (capacity <= 0 || !status) return fail(GSR_ERR_INVALID_ARG, "static mode needs capacity > 0 and status");
    TrackXf xf;
    xf.mw = x.means_world; xf.ur = x.unnorm_rot; xf.lo = x.logit_opac; xf.ls = x.log_scales;
    xf.scols = x.scale_cols; xf.cq = x.cam_q; xf.ct = x.cam_t; xf.qs = x.q_stride; xf.w2c = x.w2c;
    xf.store = true;
    return forward_impl(settings, gaussians, colors2, out_color, out_color2, out_depth, radii, alloc, alloc_ctx,
                        stream, capacity, status, nullptr, &xf, nullptr, x.alive);
}

int gsr_track_backward_scratch_floats(int P) { return pose_fuse_scratch_floats(P < 1 ? 1 : P); }

static int track_backward(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                          const float* colors2, const float* dL_dout_color, const float* dL_dout_color2,
                          int num_rendered, const void* geom_buffer, const void* binning_buffer,
                          const void* image_buffer, const float* means_world, const float* unnorm_rot,
                          int scale_cols, float* cam_q, float* cam_t, int q_stride, const float* w2c, double lr_q,
                          double lr_t, double beta1, double beta2, double eps, float* adam_state, float* dL_dcam_q,
                          float* dL_dcam_t, float* scratch, const gsr_pose_track* track, const float* log_scales,
                          gsr_alloc_fn alloc, void* alloc_ctx, void* stream, const float* inst_records);

int gsr_track_backward_dual(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                            const float* colors2, const float* dL_dout_color, const float* dL_dout_color2,
                            int num_rendered, const void* geom_buffer, const void* binning_buffer,
                            const void* image_buffer, const float* means_world, const float* unnorm_rot,
                            int scale_cols, float* cam_q, float* cam_t, int q_stride, const float* w2c, double lr_q,
                            double lr_t, double beta1, double beta2, double eps, float* adam_state,
                            float* dL_dcam_q, float* dL_dcam_t, float* scratch, const gsr_pose_track* track,
                            const float* log_scales, gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    return track_backward(settings, gaussians, radii, colors2, dL_dout_color, dL_dout_color2, num_rendered,
                          geom_buffer, binning_buffer, image_buffer, means_world, unnorm_rot, scale_cols, cam_q, cam_t,
                          q_stride, w2c, lr_q, lr_t, beta1, beta2, eps, adam_state, dL_dcam_q, dL_dcam_t, scratch,
                          track, log_scales, alloc, alloc_ctx, stream, nullptr);
}

int gsr_track_backward_dual_records(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                                    const float* colors2, int num_rendered, const void* geom_buffer,
                                    const void* binning_buffer, const void* image_buffer, const float* means_world,
                                    const float* unnorm_rot, int scale_cols, float* cam_q, float* cam_t, int q_stride,
                                    const float* w2c, double lr_q, double lr_t, double beta1, double beta2,
                                    double eps, float* adam_state, float* dL_dcam_q, float* dL_dcam_t,
                                    float* scratch, const gsr_pose_track* track, const float* log_scales,
                                    const float* inst_records, gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    if (!inst_records) return fail(GSR_ERR_INVALID_ARG, "track_backward_dual_records: null records");
    // (the gradient images are not read: the records already hold the render backward's sums)
    return track_backward(settings, gaussians, radii, colors2, nullptr, nullptr, num_rendered, geom_buffer,
                          binning_buffer, image_buffer, means_world, unnorm_rot, scale_cols, cam_q, cam_t, q_stride,
                          w2c, lr_q, lr_t, beta1, beta2, eps, adam_state, dL_dcam_q, dL_dcam_t, scratch, track,
                          log_scales, alloc, alloc_ctx, stream, inst_records);
}

static int track_backward(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                          const float* colors2, const float* dL_dout_color, const float* dL_dout_color2,
                          int num_rendered, const void* geom_buffer, const void* binning_buffer,
                          const void* image_buffer, const float* means_world, const float* unnorm_rot,
                          int scale_cols, float* cam_q, float* cam_t, int q_stride, const float* w2c, double lr_q,
                          double lr_t, double beta1, double beta2, double eps, float* adam_state, float* dL_dcam_q,
                          float* dL_dcam_t, float* scratch, const gsr_pose_track* track, const float* log_scales,
                          gsr_alloc_fn alloc, void* alloc_ctx, void* stream, const float* inst_records) {
    if (!gaussians || (scale_cols != 1 && scale_cols != 3) || q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "track_backward_dual: bad sizes");
    if (!colors2 || !means_world || !unnorm_rot || !cam_q || !cam_t || !w2c || !scratch ||
        (!adam_state && (!dL_dcam_q || !dL_dcam_t)))
        return fail(GSR_ERR_INVALID_ARG, "track_backward_dual: null pointer");
    if (scale_cols != 1 && !gaussians->rotations)
        return fail(GSR_ERR_INVALID_ARG, "track_backward_dual: anisotropic maps need the rendered rotations");
    PoseFuse pf{means_world, unnorm_rot, scale_cols, cam_q, cam_t, q_stride, w2c, scratch, adam_state,
                lr_q, lr_t, beta1, beta2, eps, dL_dcam_q, dL_dcam_t};
    pf.cap = (uint32_t)num_rendered;  // pf.guard = the forward's counters (backward_impl)
    pf.ls = log_scales;               // recompute the rendervars (forward without stored rendervars)
    if (track) {
        pf.loss = track->loss;
        pf.best = track->best;
    }
    gsr_grads none{};
    return backward_impl(settings, gaussians, radii, dL_dout_color, colors2, dL_dout_color2, num_rendered,
                         geom_buffer, binning_buffer, image_buffer, 1, &none, nullptr, 1, alloc, alloc_ctx, stream,
                         &pf, nullptr, inst_records);
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* visible, void* stream) {
    (void)projmatrix;
    if (P < 0) return fail(GSR_ERR_INVALID_ARG, "P must be >= 0");
    if (P == 0) return GSR_OK;
    if (!means3D || !viewmatrix || !visible) return fail(GSR_ERR_INVALID_ARG, "null pointer");
    hipError_t e = launch_mark_visible(P, means3D, viewmatrix, visible, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "mark_visible");
    return GSR_OK;
}


int gsr_timing_enable(int on) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    Timing& T = g_timing[current_device()];
    timing_drain(T);
    T.on = on != 0;
    T.clock = on >= GSR_TIMING_CLOCK;
    T.mask = (unsigned)on & 0xFFu;
    for (int i = 0; i < GSR_NUM_STAGES; i++) { T.ms[i] = 0.0; T.launches[i] = 0; T.units[i] = 0; }
    if (T.clock) {
        hipError_t e;
        if (!T.dclock && (e = hipMalloc((void**)&T.dclock, kclock_bytes())) != hipSuccess)
            return hip_fail(e, "timing clock buffer");
        if ((e = hipMemset(T.dclock, 0, kclock_bytes())) != hipSuccess) return hip_fail(e, "timing clock reset");
    }
    return GSR_OK;
}

int gsr_timing_read(double* ms, long long* launches, long long* units, int n) {
    std::lock_guard<std::mutex> lk(g_timing_mu);
    Timing& T = g_timing[current_device()];
    timing_drain(T);
    if (T.clock && T.dclock) {
        std::vector<unsigned long long> h((size_t)KCLOCK_WORDS * GSR_NUM_STAGES);
        int dev = 0, khz = 0;
        hipError_t e;
        if ((e = hipMemcpy(h.data(), T.dclock, kclock_bytes(), hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "timing clock read");
        if ((e = hipGetDevice(&dev)) != hipSuccess ||
            (e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev)) != hipSuccess || khz <= 0)
            return fail(GSR_ERR_HIP, "wall clock rate unavailable");
        for (int i = 0; i < GSR_NUM_STAGES; i++) {
            T.ms[i] = (double)h[(size_t)KCLOCK_WORDS * i + 1] / (double)khz;
            T.launches[i] = (long long)h[(size_t)KCLOCK_WORDS * i + 2];
        }
    }
    for (int i = 0; i < n && i < GSR_NUM_STAGES; i++) {
        if (ms) ms[i] = T.ms[i];
        if (launches) launches[i] = T.launches[i];
        if (units) units[i] = T.units[i];
    }
    return GSR_NUM_STAGES;
}

// Test hook: validates the wave64 permlane/DPP reduction on the device.
int gsr_selftest_reduce9(const float* in_dev, float* out_dev, void* stream) {
    hipError_t e = launch_selftest_reduce9(in_dev, out_dev, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "selftest");
    return GSR_OK;
}

int gsr_forward(const gsr_settings* settings, const gsr_gaussians* gaussians, float* out_color, float* out_depth,
                int* radii, gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    return forward_impl(settings, gaussians, nullptr, out_color, nullptr, out_depth, radii, alloc, alloc_ctx, stream);
}

int gsr_forward_reuse(const gsr_settings* settings, const gsr_gaussians* gaussians, int num_rendered,
                      const void* prev_geom, void* binning_buffer, void* image_buffer, const int* prev_radii,
                      float* out_color, float* out_depth, int* radii, gsr_alloc_fn alloc, void* alloc_ctx,
                      void* stream_) {
    int rc = validate(settings, gaussians, true);
    if (rc != GSR_OK) return rc;
    if (!alloc) return fail(GSR_ERR_INVALID_ARG, "allocator callback required");
    if (!gaussians->colors_precomp || (gaussians->shs && gaussians->M > 0))
        return fail(GSR_ERR_INVALID_ARG, "geometry reuse needs precomputed colours (no SH)");
    if (gaussians->P <= 0 || num_rendered < 0 || !prev_geom || !binning_buffer || !image_buffer || !prev_radii ||
        !out_color || !out_depth || !radii)
        return fail(GSR_ERR_INVALID_ARG, "geometry reuse needs the previous call's state and the outputs");
    hipStream_t stream = (hipStream_t)stream_;
    const int dev = stream_device(stream);
    Camera cam = make_camera(settings);
    const GaussIn g = make_gauss(gaussians);
    const int P = g.P;
    const GeomLayout GL = GeomLayout::make(P);
    cam.pre_shift = GL.shift;
    const ImgLayout IL = ImgLayout::make(cam.W, cam.H);
    void* geom = obtain(alloc, alloc_ctx, GSR_BUF_GEOM, GL.total);
    if (!geom) return fail(GSR_ERR_ALLOC, "allocator returned NULL (geom buffer)");
    const GeomPtrs geo = GeomPtrs::at(geom, GL);
    char* ib = (char*)image_buffer;
    cam.tile_order = (const uint32_t*)(ib + IL.order);
    cam.rowmax = (uint32_t*)(ib + IL.rowmax);
    cam.sched_cus = device_cus(dev);
    hipError_t e;
    {
        StageTimer t(GSR_STAGE_PREPROCESS, P, stream);
        if ((e = hipMemcpyAsync(geom, prev_geom, GL.total, hipMemcpyDeviceToDevice, stream)) != hipSuccess ||
            (e = hipMemcpyAsync(radii, prev_radii, sizeof(int) * (size_t)P, hipMemcpyDeviceToDevice, stream)) !=
                hipSuccess)
            return hip_fail(e, "copy previous geometry");
        if ((e = launch_recolour(P, g.colors, geo, stream)) != hipSuccess) return hip_fail(e, "recolour");
    }
    // the previous render_fwd left point_list sorted (with its block masks): no sort, any list length
    const SpecGuard guard{geo.counters, (uint32_t)num_rendered, 0xFFFFFFFFu};
    {
        StageTimer t(GSR_STAGE_RENDER_FWD, num_rendered, stream, true);
        if ((e = launch_render_fwd(cam, (const uint2*)(ib + IL.ranges), (uint64_t*)binning_buffer, nullptr, geo,
                                   nullptr, (float*)(ib + IL.final_T), (uint32_t*)(ib + IL.n_contrib), out_color,
                                   nullptr, out_depth, guard, stream, t.kclock())) != hipSuccess)
            return hip_fail(e, "render");
    }
    return num_rendered;
}

int gsr_forward_reuse_if_equal(const gsr_settings* settings, const gsr_gaussians* gaussians, int npairs,
                               const float* const* a, const float* const* b, const long long* n,
                               int prev_num_rendered, const void* prev_geom, void* prev_binning, void* prev_image,
                               const int* prev_radii, float* out_color, float* out_depth, int* radii, int* reused,
                               gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    if (!gaussians || !gaussians->colors_precomp || (gaussians->shs && gaussians->M > 0) || gaussians->cov3D_precomp)
        return fail(GSR_ERR_INVALID_ARG, "geometry reuse needs precomputed colours (no SH, no cov3D)");
    if (npairs < 1 || npairs > 8 || !a || !b || !n || !reused)
        return fail(GSR_ERR_INVALID_ARG, "gsr_forward_reuse_if_equal: 1..8 pairs and `reused`");
    if (prev_num_rendered < 0 || !prev_geom || !prev_binning || !prev_image || !prev_radii)
        return fail(GSR_ERR_INVALID_ARG, "geometry reuse needs the previous call's state");
    ReuseIn r{};
    r.pairs.npairs = npairs;
    for (int k = 0; k < npairs; k++) {
        if (n[k] < 0 || (n[k] > 0 && (!a[k] || !b[k])))
            return fail(GSR_ERR_INVALID_ARG, "gsr_forward_reuse_if_equal: pair");
        r.pairs.a[k] = a[k];
        r.pairs.b[k] = b[k];
        r.pairs.n[k] = n[k];
    }
    r.prev_num_rendered = prev_num_rendered;
    r.prev_geom = prev_geom;
    r.prev_binning = prev_binning;
    r.prev_image = prev_image;
    r.prev_radii = prev_radii;
    r.reused = reused;
    return forward_impl(settings, gaussians, nullptr, out_color, nullptr, out_depth, radii, alloc, alloc_ctx, stream,
                        0, nullptr, nullptr, nullptr, nullptr, nullptr, &r);
}

int gsr_bitwise_equal(int npairs, const float* const* a, const float* const* b, const long long* n, int* flag,
                      void* stream) {
    if (npairs < 0 || npairs > 8 || (npairs > 0 && (!a || !b || !n)) || !flag)
        return fail(GSR_ERR_INVALID_ARG, "gsr_bitwise_equal: 0..8 pairs and a flag");
    EqualPairs q{};
    q.npairs = npairs;
    for (int k = 0; k < npairs; k++) {
        if (n[k] < 0 || (n[k] > 0 && (!a[k] || !b[k]))) return fail(GSR_ERR_INVALID_ARG, "gsr_bitwise_equal: pair");
        q.a[k] = a[k];
        q.b[k] = b[k];
        q.n[k] = n[k];
    }
    hipError_t e = zero_async(flag, sizeof(int), (hipStream_t)stream);  // (kernel: valid under capture too)
    if (e == hipSuccess) e = launch_bitwise_equal(q, flag, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "bitwise_equal");
    return GSR_OK;
}

int gsr_forward_dual(const gsr_settings* settings, const gsr_gaussians* gaussians, const float* colors2,
                     float* out_color, float* out_color2, float* out_depth, int* radii, gsr_alloc_fn alloc,
                     void* alloc_ctx, void* stream) {
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    return forward_impl(settings, gaussians, colors2, out_color, out_color2, out_depth, radii, alloc, alloc_ctx,
                        stream);
}

int gsr_forward_static(const gsr_settings* settings, const gsr_gaussians* gaussians, int capacity, unsigned* status,
                       float* out_color, float* out_depth, int* radii, gsr_alloc_fn alloc, void* alloc_ctx,
                       void* stream) {
    if (capacity <= 0 || !status) return fail(GSR_ERR_INVALID_ARG, "static mode needs capacity > 0 and status");
    return forward_impl(settings, gaussians, nullptr, out_color, nullptr, out_depth, radii, alloc, alloc_ctx, stream,
                        capacity, status);
}

int gsr_forward_dual_static(const gsr_settings* settings, const gsr_gaussians* gaussians, const float* colors2,
                            int capacity, unsigned* status, float* out_color, float* out_color2, float* out_depth,
                            int* radii, gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    if (capacity <= 0 || !status) return fail(GSR_ERR_INVALID_ARG, "static mode needs capacity > 0 and status");
    return forward_impl(settings, gaussians, colors2, out_color, out_color2, out_depth, radii, alloc, alloc_ctx,
                        stream, capacity, status);
}

int gsr_forward_dual_static_alive(const gsr_settings* settings, const gsr_gaussians* gaussians, const float* colors2,
                                  int capacity, unsigned* status, float* out_color, float* out_color2,
                                  float* out_depth, int* radii, const unsigned char* alive, gsr_alloc_fn alloc,
                                  void* alloc_ctx, void* stream) {
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    if (capacity <= 0 || !status) return fail(GSR_ERR_INVALID_ARG, "static mode needs capacity > 0 and status");
    if (!alive && gaussians && gaussians->P > 0) return fail(GSR_ERR_INVALID_ARG, "alive mask required");
    return forward_impl(settings, gaussians, colors2, out_color, out_color2, out_depth, radii, alloc, alloc_ctx,
                        stream, capacity, status, nullptr, nullptr, nullptr, alive);
}

int gsr_backward(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                 const float* dL_dout_color, int num_rendered, const void* geom_buffer, const void* binning_buffer,
                 const void* image_buffer, int power, const gsr_grads* grads, gsr_alloc_fn alloc, void* alloc_ctx,
                 void* stream) {
    return backward_impl(settings, gaussians, radii, dL_dout_color, nullptr, nullptr, num_rendered, geom_buffer,
                         binning_buffer, image_buffer, power, grads, nullptr, 3, alloc, alloc_ctx, stream);
}

int gsr_backward_dual(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                      const float* colors2, const float* dL_dout_color, const float* dL_dout_color2,
                      int num_rendered, const void* geom_buffer, const void* binning_buffer,
                      const void* image_buffer, const gsr_grads* grads, float* dcolors2, int dl2_channels,
                      gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    return backward_impl(settings, gaussians, radii, dL_dout_color, colors2, dL_dout_color2, num_rendered,
                         geom_buffer, binning_buffer, image_buffer, 1, grads, dcolors2, dl2_channels, alloc, alloc_ctx,
                         stream);
}

int gsr_backward_dual_sh_adam(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                              const float* colors2, const float* dL_dout_color, const float* dL_dout_color2,
                              int num_rendered, const void* geom_buffer, const void* binning_buffer,
                              const void* image_buffer, const gsr_grads* grads, float* dcolors2, int dl2_channels,
                              const gsr_map_adam* sh_adam, gsr_alloc_fn alloc, void* alloc_ctx, void* stream) {
    if (!colors2) return fail(GSR_ERR_INVALID_ARG, "colors2 required");
    if (!sh_adam || !gaussians || !gaussians->shs || sh_adam->step < 1 || !sh_adam->exp_avg[4] ||
        !sh_adam->exp_avg_sq[4])
        return fail(GSR_ERR_INVALID_ARG, "backward_dual_sh_adam: SH colours and the colour group's state required");
    // the scalars exactly as gsr_map_transform_bwd_adam forms them (python floats -> float)
    ShAdam sa;
    const double bc1 = 1.0 - pow(sh_adam->beta1, (double)sh_adam->step);
    sa.m = sh_adam->exp_avg[4];
    sa.v = sh_adam->exp_avg_sq[4];
    sa.ss = (float)(-sh_adam->lr[4] / bc1);
    sa.w1 = (float)(1.0 - sh_adam->beta1);
    sa.beta2 = (float)sh_adam->beta2;
    sa.omb2 = (float)(1.0 - sh_adam->beta2);
    sa.bc2_sqrt = (float)sqrt(1.0 - pow(sh_adam->beta2, (double)sh_adam->step));
    sa.eps = (float)sh_adam->eps;
    sa.halted = sh_adam->halted;
    // sa.guard / sa.cap: the forward's own counters (backward_impl); sh_adam->status is not read
    return backward_impl(settings, gaussians, radii, dL_dout_color, colors2, dL_dout_color2, num_rendered,
                         geom_buffer, binning_buffer, image_buffer, 1, grads, dcolors2, dl2_channels, alloc, alloc_ctx,
                         stream, nullptr, &sa);
}

}  // extern "C"
