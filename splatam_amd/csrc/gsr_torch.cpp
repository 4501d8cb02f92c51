// gsr_torch.cpp -- the native torch binding of the drop-in path's two per-iteration calls:
// RasterizeGaussiansCUDA / RasterizeGaussiansBackwardCUDA (rasterize_points.cu:35-115, 117-196), the
// tensor -> pointer marshalling SURVEY.md 8(b) describes, over the C ABI of include/gsr.h.
//
// splatam_amd/_C.py's ctypes binding does the same work for every entry point; for these two it
// spent ~45 us (forward) and ~27 us (backward) of host time per call in Python (argument checks, ctypes
// structs, the allocator callback into Python), which the unchanged caller -- two renders forward and
// backward per SplaTAM iteration, host-bound -- pays in full.  Here the same checks, error messages,
// buffers and results cost a few microseconds.  Semantics mirror _C.rasterize_gaussians (dynamic mode,
// capacity 0) and _C.rasterize_gaussians_backward exactly; _C.py dispatches to this module for them.
#include <cstdlib>
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <array>
#include <optional>
#include <string>
#include <vector>

#include "gsr.h"

namespace {

// The buffers the library asks for during one call (GSR_BUF_*), as torch tensors on the call's device
struct Bufs {
    at::Device dev{at::kCPU};
    std::array<at::Tensor, 4> t;
};

void* alloc_cb(void* ctx, int kind, size_t nbytes) {
    auto* b = static_cast<Bufs*>(ctx);
    if (kind < 0 || kind >= 4) return nullptr;
    try {
        at::Tensor t = at::empty({(int64_t)(nbytes > 0 ? nbytes : 1)}, at::TensorOptions().dtype(at::kByte).device(b->dev));
        b->t[kind] = t;
        return t.data_ptr();
    } catch (...) {
        return nullptr;
    }
}

[[noreturn]] void raise_rc(const char* what) {
    throw std::runtime_error(std::string(what) + ": " + gsr_last_error());
}

std::string dtype_name(const at::Tensor& t) {
    std::string s = c10::toString(t.scalar_type());
    return "torch." + (s == "Float" ? std::string("float32") : s == "Double" ? std::string("float64")
                       : s == "Half" ? std::string("float16") : s == "Int" ? std::string("int32")
                       : s == "Long" ? std::string("int64") : s);
}

// _C._dev_f32: contiguous float32 on `dev`, or an undefined tensor for an empty one (-> NULL)
at::Tensor dev_f32(const at::Tensor& t, const at::Device& dev, const char* name) {
    if (!t.defined() || t.numel() == 0) return at::Tensor();
    if (t.scalar_type() != at::kFloat)
        throw std::runtime_error(std::string(name) + ": expected scalar type Float but found " + dtype_name(t));
    at::Tensor r = t.device() == dev ? t : t.to(dev);
    return r.contiguous();
}

// _C._cam_f32: the camera tensors are the same objects on every call of an iteration and SplaTAM passes
// the matrices as transposed views, so the contiguous copy is reused while the source tensor is alive and
// unmodified (weak reference + version counter), on the same stream, never during stream capture.
// GSR_CAM_CACHE=0 disables it, as for the ctypes path (_C._CAM_CACHE).
const bool g_cam_cache_on = [] {
    const char* v = std::getenv("GSR_CAM_CACHE");
    return !(v && std::string(v) == "0");
}();
struct CamEntry {
    c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl> src;
    int64_t version;
    hipStream_t stream;
    at::Tensor copy;
};
thread_local std::vector<CamEntry> g_cam;

at::Tensor cam_f32(const at::Tensor& t, const at::Device& dev, const char* name, hipStream_t s) {
    if (!t.defined() || t.numel() == 0) return at::Tensor();
    if (t.scalar_type() == at::kFloat && t.device() == dev && t.is_contiguous()) return t;
    if (!g_cam_cache_on) return dev_f32(t, dev, name);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return dev_f32(t, dev, name);
    const c10::TensorImpl* impl = t.unsafeGetTensorImpl();
    for (auto& e : g_cam) {
        auto p = e.src.lock();
        if (p.get() == impl && e.version == t._version() && e.stream == s && e.copy.device() == dev) return e.copy;
    }
    at::Tensor c = dev_f32(t, dev, name);
    if (g_cam.size() >= 64) {  // drop the dead entries; still full: drop the oldest half (bounded either way)
        std::vector<CamEntry> live;
        for (auto& e : g_cam)
            if (!e.src.expired()) live.push_back(e);
        if (live.size() >= 64) live.erase(live.begin(), live.begin() + 32);
        g_cam.swap(live);
    }
    g_cam.push_back(CamEntry{c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>(t.getIntrusivePtr()),
                             t._version(), s, c});
    return c;
}

const float* fptr(const at::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }

struct Cam {
    gsr_settings s{};
    std::array<at::Tensor, 4> keep;
};

Cam settings(const at::Tensor& bg, const at::Tensor& view, const at::Tensor& proj, const at::Tensor& campos,
             double tanfovx, double tanfovy, int64_t H, int64_t W, double scale_modifier, int64_t degree,
             bool prefiltered, const at::Device& dev, hipStream_t st) {
    Cam c;
    c.keep = {cam_f32(bg, dev, "bg", st), cam_f32(view, dev, "viewmatrix", st), cam_f32(proj, dev, "projmatrix", st),
              cam_f32(campos, dev, "campos", st)};
    c.s.image_height = (int)H;
    c.s.image_width = (int)W;
    c.s.tan_fovx = (float)tanfovx;
    c.s.tan_fovy = (float)tanfovy;
    c.s.bg = fptr(c.keep[0]);
    c.s.scale_modifier = (float)scale_modifier;
    c.s.viewmatrix = fptr(c.keep[1]);
    c.s.projmatrix = fptr(c.keep[2]);
    c.s.sh_degree = (int)degree;
    c.s.campos = fptr(c.keep[3]);
    c.s.prefiltered = prefiltered ? 1 : 0;
    return c;
}

struct Gauss {
    gsr_gaussians g{};
    std::array<at::Tensor, 7> keep;
};

Gauss gaussians(const at::Tensor& means3D, const at::Tensor& sh, const at::Tensor& colors, const at::Tensor& opacity,
                const at::Tensor& scales, const at::Tensor& rotations, const at::Tensor& cov3D, const at::Device& dev) {
    Gauss r;
    const int64_t P = means3D.size(0);
    const int64_t M = (sh.defined() && sh.numel() > 0 && sh.dim() >= 2 && sh.size(0) != 0) ? sh.size(1) : 0;
    r.keep = {dev_f32(means3D, dev, "means3D"), M ? dev_f32(sh, dev, "sh") : at::Tensor(), dev_f32(colors, dev, "colors"),
              dev_f32(opacity, dev, "opacity"), dev_f32(scales, dev, "scales"), dev_f32(rotations, dev, "rotations"),
              dev_f32(cov3D, dev, "cov3D_precomp")};
    r.g.P = (int)P;
    r.g.M = (int)M;
    r.g.means3D = fptr(r.keep[0]);
    r.g.shs = fptr(r.keep[1]);
    r.g.colors_precomp = fptr(r.keep[2]);
    r.g.opacities = fptr(r.keep[3]);
    r.g.scales = fptr(r.keep[4]);
    r.g.rotations = fptr(r.keep[5]);
    r.g.cov3D_precomp = fptr(r.keep[6]);
    return r;
}

// Geometry reuse across consecutive calls (_C.py's rules, here for the native path): SplaTAM renders RGB and
// then depth / silhouette of the same Gaussians from the same camera (scripts/splatam.py:255,259).  When the
// host checks pass -- means3D and the camera tensors the very same objects at the same versions, equal scalar
// settings, precomputed colours, no SH / cov3D, the previous call's rotations / opacities / scales and buffers
// alive and unmodified -- the call goes through gsr_forward_reuse_if_equal, which compares this call's
// rotations / opacities / scales with the previous call's on the device and gates the reuse and the full
// forward on the result, with the one host wait gsr_forward makes anyway.  GSR_GEOM_CACHE=0 (or
// set_geom_cache(False)) disables it.
using WeakT = c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>;
bool g_geom_cache = [] {
    const char* v = std::getenv("GSR_GEOM_CACHE");
    return !(v && std::string(v) == "0");
}();
std::array<int64_t, 3> g_reuse_stats{0, 0, 0};  // hits, misses, misses on content (device comparison)

struct Ref {  // a weak reference + the version it had
    std::optional<WeakT> w;
    int64_t version = 0;
    static Ref of(const at::Tensor& t) {
        Ref r;
        if (t.defined()) {
            r.w.emplace(t.getIntrusivePtr());
            r.version = t._version();
        }
        return r;
    }
    bool same(const at::Tensor& t) const {  // the same object, unmodified (both undefined: same)
        if (!t.defined() || !w) return !t.defined() && !w;
        auto p = w->lock();
        return p.get() == t.unsafeGetTensorImpl() && t._version() == version;
    }
    at::Tensor get() const {  // the referenced tensor at its recorded version, or undefined
        if (!w) return at::Tensor();
        auto p = w->lock();
        if (!p) return at::Tensor();
        at::Tensor t(std::move(p));
        return t._version() == version ? t : at::Tensor();
    }
};
struct PrevCall {
    int dev = -1;
    hipStream_t stream = nullptr;
    int64_t P = 0, H = 0, W = 0, degree = 0;
    double tanfovx = 0, tanfovy = 0, scale_modifier = 0;
    bool prefiltered = false;
    std::array<Ref, 5> shared;  // means3D, bg, viewmatrix, projmatrix, campos (the caller's objects)
    std::array<Ref, 3> others;  // rotations, opacities, scales as passed down
    std::array<Ref, 3> bufs;    // geom, binning, image
    Ref radii;
    int num_rendered = 0;
};
thread_local std::vector<PrevCall> g_prev;

// _C.rasterize_gaussians, dynamic mode
std::tuple<int64_t, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> rasterize_gaussians(
    const at::Tensor& background, const at::Tensor& means3D, const at::Tensor& colors, const at::Tensor& opacity,
    const at::Tensor& scales, const at::Tensor& rotations, double scale_modifier, const at::Tensor& cov3D_precomp,
    const at::Tensor& viewmatrix, const at::Tensor& projmatrix, double tan_fovx, double tan_fovy, int64_t image_height,
    int64_t image_width, const at::Tensor& sh, int64_t degree, const at::Tensor& campos, bool prefiltered) {
    if (means3D.dim() != 2 || means3D.size(1) != 3)
        throw std::runtime_error("means3D must have dimensions (num_points, 3)");
    const at::Device dev = means3D.device();
    if (!dev.is_cuda())
        throw std::runtime_error("splatam_amd rasterizer runs on ROCm devices only (no CPU fallback); means3D is on " +
                                 dev.str());
    const int64_t P = means3D.size(0), H = image_height, W = image_width;
    const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
    if (P == 0) {
        at::Tensor empty = at::empty({0}, at::TensorOptions().dtype(at::kByte).device(dev));
        return {0, at::zeros({3, H, W}, f32), at::zeros({0}, at::TensorOptions().dtype(at::kInt).device(dev)), empty,
                empty.clone(), empty.clone(), at::zeros({1, H, W}, f32)};
    }
    c10::DeviceGuard guard(dev);
    const hipStream_t st = c10::hip::getCurrentHIPStream(dev.index()).stream();
    Cam c = settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, H, W, scale_modifier, degree,
                     prefiltered, dev, st);
    Gauss g = gaussians(means3D, sh, colors, opacity, scales, rotations, cov3D_precomp, dev);
    at::Tensor out_color = at::empty({3, H, W}, f32);
    at::Tensor out_depth = at::empty({1, H, W}, f32);
    at::Tensor radii = at::empty({P}, at::TensorOptions().dtype(at::kInt).device(dev));
    Bufs b;
    b.dev = dev;
    const bool reusable = g_geom_cache && g.g.colors_precomp && g.g.M == 0 && !g.g.cov3D_precomp && g.g.opacities &&
                          g.g.scales && g.g.rotations;
    if (!reusable) {
        const int n = gsr_forward(&c.s, &g.g, out_color.data_ptr<float>(), out_depth.data_ptr<float>(),
                                  radii.data_ptr<int>(), alloc_cb, &b, st);
        if (n < 0) raise_rc("rasterize_gaussians");
        return {(int64_t)n, out_color, radii, b.t[GSR_BUF_GEOM], b.t[GSR_BUF_BINNING], b.t[GSR_BUF_IMAGE], out_depth};
    }
    const std::array<const at::Tensor*, 5> shared = {&means3D, &background, &viewmatrix, &projmatrix, &campos};
    const std::array<at::Tensor, 3> others = {g.keep[5], g.keep[3], g.keep[4]};
    PrevCall* pc = nullptr;
    for (auto& e : g_prev)
        if (e.dev == dev.index()) pc = &e;
    bool hit = pc && pc->stream == st && pc->P == P && pc->H == H && pc->W == W && pc->degree == degree &&
               pc->tanfovx == tan_fovx && pc->tanfovy == tan_fovy && pc->scale_modifier == scale_modifier &&
               pc->prefiltered == prefiltered;
    for (int k = 0; hit && k < 5; k++) hit = pc->shared[k].same(*shared[k]);
    std::array<at::Tensor, 3> po, pb;
    at::Tensor prad;
    for (int k = 0; hit && k < 3; k++) {
        po[k] = pc->others[k].get();
        pb[k] = pc->bufs[k].get();
        hit = po[k].defined() && pb[k].defined() && po[k].sizes() == others[k].sizes();
    }
    if (hit) {
        prad = pc->radii.get();
        hit = prad.defined();
    }
    int n;
    if (hit) {
        const float* pa[3];
        const float* pbp[3];
        long long pn[3];
        for (int k = 0; k < 3; k++) {
            pa[k] = others[k].data_ptr<float>();
            pbp[k] = po[k].data_ptr<float>();
            pn[k] = (long long)others[k].numel();
        }
        int reused = 0;
        n = gsr_forward_reuse_if_equal(&c.s, &g.g, 3, pa, pbp, pn, pc->num_rendered, pb[0].data_ptr(), pb[1].data_ptr(),
                                       pb[2].data_ptr(), prad.data_ptr<int>(), out_color.data_ptr<float>(),
                                       out_depth.data_ptr<float>(), radii.data_ptr<int>(), &reused, alloc_cb, &b, st);
        if (n < 0) raise_rc("rasterize_gaussians (geometry reuse)");
        if (reused) {  // this call's geometry buffer; the previous call's binning and image buffers
            g_reuse_stats[0]++;
            return {(int64_t)n, out_color, radii, b.t[GSR_BUF_GEOM], pb[1], pb[2], out_depth};
        }
        g_reuse_stats[1]++;
        g_reuse_stats[2]++;
    } else {
        g_reuse_stats[1]++;
        n = gsr_forward(&c.s, &g.g, out_color.data_ptr<float>(), out_depth.data_ptr<float>(), radii.data_ptr<int>(),
                        alloc_cb, &b, st);
        if (n < 0) raise_rc("rasterize_gaussians");
    }
    if (!pc) {
        g_prev.emplace_back();
        pc = &g_prev.back();
    }
    PrevCall& r = *pc;
    r.dev = dev.index();
    r.stream = st;
    r.P = P, r.H = H, r.W = W, r.degree = degree;
    r.tanfovx = tan_fovx, r.tanfovy = tan_fovy, r.scale_modifier = scale_modifier;
    r.prefiltered = prefiltered;
    for (int k = 0; k < 5; k++) r.shared[k] = Ref::of(*shared[k]);
    for (int k = 0; k < 3; k++) r.others[k] = Ref::of(others[k]);
    r.bufs = {Ref::of(b.t[GSR_BUF_GEOM]), Ref::of(b.t[GSR_BUF_BINNING]), Ref::of(b.t[GSR_BUF_IMAGE])};
    r.radii = Ref::of(radii);
    r.num_rendered = n;
    return {(int64_t)n, out_color, radii, b.t[GSR_BUF_GEOM], b.t[GSR_BUF_BINNING], b.t[GSR_BUF_IMAGE], out_depth};
}

void set_geom_cache(bool on) { g_geom_cache = on; }
std::vector<int64_t> reuse_stats() { return {g_reuse_stats[0], g_reuse_stats[1], g_reuse_stats[2]}; }

// _C.rasterize_gaussians_backward (needs: 8 flags or an empty list = every gradient)
std::vector<at::Tensor> rasterize_gaussians_backward(
    const at::Tensor& background, const at::Tensor& means3D, const at::Tensor& radii, const at::Tensor& colors,
    const at::Tensor& scales, const at::Tensor& rotations, double scale_modifier, const at::Tensor& cov3D_precomp,
    const at::Tensor& viewmatrix, const at::Tensor& projmatrix, double tan_fovx, double tan_fovy,
    const at::Tensor& dL_dout_color, const at::Tensor& sh, int64_t degree, const at::Tensor& campos,
    const at::Tensor& geomBuffer, int64_t R, const at::Tensor& binningBuffer, const at::Tensor& imageBuffer,
    int64_t power, std::vector<bool> needs) {
    const at::Device dev = means3D.device();
    const int64_t P = means3D.size(0);
    const int64_t H = dL_dout_color.size(1), W = dL_dout_color.size(2);
    const int64_t M = (sh.defined() && sh.numel() > 0 && sh.size(0) != 0) ? sh.size(1) : 0;
    const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
    if (!needs.empty() && power != 1) {  // honoured only for the Fisher-selective request (ros_handler.py:884-889)
        const bool fisher = M == 0 && colors.defined() && colors.numel() > 0 && !needs[0] && !needs[1] && !needs[4] &&
                            !needs[5] && !needs[6] && !needs[7];
        if (!fisher) needs.clear();
    }
    if (needs.empty()) needs.assign(8, true);
    needs[3] = true;  // dmeans3D is always produced
    const std::array<std::vector<int64_t>, 8> shapes = {std::vector<int64_t>{P, 3}, {P, 3}, {P, 1}, {P, 3}, {P, 6},
                                                        {P, M, 3}, {P, 3}, {P, 4}};
    std::vector<at::Tensor> out(8);
    for (int k = 0; k < 8; k++)
        if (needs[k]) out[k] = at::empty(shapes[k], f32);
    if (P == 0) return out;
    c10::DeviceGuard guard(dev);
    const hipStream_t st = c10::hip::getCurrentHIPStream(dev.index()).stream();
    Cam c = settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, H, W, scale_modifier, degree,
                     false, dev, st);
    // opacities are not an input of the backward (rasterize_points.cu:117-139): they live in geomBuffer
    Gauss g = gaussians(means3D, sh, colors, at::Tensor(), scales, rotations, cov3D_precomp, dev);
    at::Tensor dpix = dev_f32(dL_dout_color, dev, "dL_dout_color");
    at::Tensor radii_c = radii.to(dev, at::kInt).contiguous();
    auto ptr = [](const at::Tensor& t) -> float* { return (t.defined() && t.numel() > 0) ? t.data_ptr<float>() : nullptr; };
    gsr_grads gr{ptr(out[0]), ptr(out[1]), ptr(out[2]), ptr(out[3]), ptr(out[4]), ptr(out[5]), ptr(out[6]), ptr(out[7])};
    Bufs b;
    b.dev = dev;
    const int rc = gsr_backward(&c.s, &g.g, radii_c.data_ptr<int>(), dpix.data_ptr<float>(), (int)R,
                                geomBuffer.data_ptr(), binningBuffer.numel() ? binningBuffer.data_ptr() : nullptr,
                                imageBuffer.data_ptr(), (int)power, &gr, alloc_cb, &b, st);
    if (rc < 0) raise_rc("rasterize_gaussians_backward");
    return out;  // the scratch buffer returns to torch's caching allocator (stream-ordered) with `b`
}

}  // namespace

PYBIND11_MODULE(_gsr_torch, m) {
    m.doc() = "native torch binding of gsr_forward / gsr_backward (the drop-in path's per-iteration calls)";
    m.def("rasterize_gaussians", &rasterize_gaussians);
    m.def("rasterize_gaussians_backward", &rasterize_gaussians_backward);
    m.def("set_geom_cache", &set_geom_cache);
    m.def("reuse_stats", &reuse_stats);
}
