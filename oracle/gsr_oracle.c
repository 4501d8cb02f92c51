/*
 * oracle/gsr_oracle.c -- CPU restatement of the SplaTAM differentiable Gaussian
 * rasterizer (diff-gaussian-rasterization-w-depth, vendored copy under
 * /root/reference/hessian-diff-gaussian-rasterization-w-depth).
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path (splatam_amd/) never links or calls it.
 *
 * Parity status: the reference CUDA extension cannot be built or run in this
 * container (no nvcc, no NVIDIA GPU) and ships no golden vectors, so kernel
 * numerics are "parity unpinned" against the reference binary.  This
 * restatement follows the .cu sources line by line (citations per function)
 * and is cross-checked in tests/ against torch.autograd through a dense
 * formulation and against finite differences in float64.
 *
 * Built twice (see oracle/Makefile):  -DREAL=float  -> oracle/_build/libgsr_oracle_f32.so
 *                                     -DREAL=double -> oracle/_build/libgsr_oracle_f64.so
 * Compiled with -ffp-contract=off so float32 results follow IEEE op by op.
 *
 * Semantics notes:
 *   - forward: forward.cu:155-256 (preprocess), forward.cu:261-393 (render),
 *     rasterizer_impl.cu:70-138,198-339 (binning / sort / ranges);
 *   - backward, mode GSR_ORACLE_UPSTREAM: the upstream decomposition that the
 *     un-vendored diff_gaussian_rasterization runs (backward.cu:586-748 render,
 *     144-274 cov2D, 412-475 cov3D, 480-530 preprocess, 20-139 SH);
 *   - backward, mode GSR_ORACLE_FUSED: the vendored renderCUDAFused semantics
 *     (backward.cu:850-1140): the full chain per (pixel, Gaussian) pair and
 *     powf(value, power) applied per pair before summation.  The two vendored
 *     SH bugs (backward.cu:1067 offset M*gid instead of 3*M*gid, and
 *     backward.cu:1117 dropping SH grads when D==0) are NOT replicated.
 *
 * Threads (OpenMP): preprocess over Gaussians, render / backward over tiles.
 * Results do not depend on the thread count: the backward sums each pair's
 * terms into the record of its (tile, Gaussian) instance (pixels of a tile in
 * order), then each Gaussian's records in instance order.  oracle_set_threads
 * (0 = OpenMP default) sets the count.
 *
 * Threshold proximity (test support): the forward flags every pixel with an
 * evaluated pair whose alpha lies within a relative ALPHA_BAND of 1/255 or
 * whose test_T lies within a relative T_BAND of 1e-4 (a float32 implementation
 * may decide such a pair the other way) with bit 0, a T = 0.5 crossing within
 * T_BAND (the median depth's decision) with bit 1, and `unstable` marks every Gaussian
 * evaluated at a flagged pixel (its gradient depends on that decision through
 * T and the accumulated colour).  Per-element gradient checks skip them.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef REAL
#define REAL float
#endif
typedef REAL real;

#define BLOCK_X 16
#define BLOCK_Y 16

#define GSR_ORACLE_UPSTREAM 0
#define GSR_ORACLE_FUSED 1
#define ALPHA_BAND 2e-5
#define T_BAND 1e-4

static int g_threads = 0; /* 0: OpenMP default (OMP_NUM_THREADS / all cores) */
void oracle_set_threads(int n) { g_threads = n < 0 ? 0 : n; }
int oracle_threads(void);
static int nthreads(void)
{
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}

/* auxiliary.h:22-39 */
static const real SH_C0 = (real)0.28209479177387814;
static const real SH_C1 = (real)0.4886025119029199;
static const real SH_C2[5] = {(real)1.0925484305920792, (real)-1.0925484305920792,
                              (real)0.31539156525252005, (real)-1.0925484305920792,
                              (real)0.5462742152960396};
static const real SH_C3[7] = {(real)-0.5900435899266435, (real)2.890611442640554,
                              (real)-0.4570457994644658, (real)0.3731763325901154,
                              (real)-0.4570457994644658, (real)1.445305721320277,
                              (real)-0.5900435899266435};

typedef struct { real x, y, z; } v3;

static inline real rmin(real a, real b) { return a < b ? a : b; }
static inline real rmax(real a, real b) { return a > b ? a : b; }
#if defined(REAL_IS_DOUBLE)
#define RSQRT(x) sqrt(x)
#define REXP(x) exp(x)
#define RCEIL(x) ceil(x)
#define RPOW(x, p) pow((x), (p))
#else
#define RSQRT(x) sqrtf(x)
#define REXP(x) expf(x)
#define RCEIL(x) ceilf(x)
#define RPOW(x, p) powf((x), (p))
#endif

/* forward.cu:341,349 / backward.cu:681-684: power = -0.5 (A dx^2 + C dy^2) - B dx dy, G = exp(power).
 * GSR_ORACLE_ALPHA_FORM (float32 experiment builds only, tools/alpha_forms.py; never the oracle the tests
 * use) evaluates it the way a GPU render-record variant does instead: the conic prescaled by -log2(e)/2,
 * -log2(e) in float, power as log2(e) * power in the variant's FMA order, G = exp2f. */
#if defined(GSR_ORACLE_ALPHA_FORM) && !defined(REAL_IS_DOUBLE)
static inline float alpha_power(const float* co, float dx, float dy)
{
    const float l2e = 1.4426950408889634f, kac = -0.5f * l2e, kb = -l2e;
    const float A = kac * co[0], B = kb * co[1], C = kac * co[2];
    (void)A; (void)B; (void)C;
#if GSR_ORACLE_ALPHA_FORM == 1 /* dx (A' dx + B' dy) + C' dy^2 */
    return fmaf(fmaf(B, dy, A * dx), dx, (C * dy) * dy);
#elif GSR_ORACLE_ALPHA_FORM == 3 /* (B' dx) dy + (A' dx dx + C' dy dy) */
    return fmaf(B * dx, dy, fmaf(A * dx, dx, (C * dy) * dy));
#elif GSR_ORACLE_ALPHA_FORM == 5 /* the reference order with the exact -1/2 folded, times log2(e) */
    const float a = -0.5f * co[0], c = -0.5f * co[2], b = -co[1];
    return (((a * dx) * dx + (c * dy) * dy) + (b * dx) * dy) * l2e;
#else
#error unknown GSR_ORACLE_ALPHA_FORM
#endif
}
#define POWER_OF(co, dx, dy) alpha_power((co), (dx), (dy))
#define GEXP(p) exp2f(p)
#else
#define POWER_OF(co, dx, dy) ((real)-0.5 * ((co)[0] * (dx) * (dx) + (co)[2] * (dy) * (dy)) - (co)[1] * (dx) * (dy))
#define GEXP(p) REXP(p)
#endif

/* auxiliary.h:41-44: evaluated in double because of the 1.0 / 0.5 literals */
static inline real ndc2pix(real v, int S) { return (real)((((double)v + 1.0) * S - 1.0) * 0.5); }

/* auxiliary.h:46-56 */
static void get_rect(real px, real py, int r, int gx, int gy, int* x0, int* y0, int* x1, int* y1)
{
    real fr = (real)r;
    int a = (int)((px - fr) / (real)BLOCK_X);
    int b = (int)((py - fr) / (real)BLOCK_Y);
    real cx = px + fr; cx = cx + (real)BLOCK_X; cx = cx - (real)1;
    real cy = py + fr; cy = cy + (real)BLOCK_Y; cy = cy - (real)1;
    int c = (int)(cx / (real)BLOCK_X);
    int d = (int)(cy / (real)BLOCK_Y);
    a = a > 0 ? a : 0; b = b > 0 ? b : 0; c = c > 0 ? c : 0; d = d > 0 ? d : 0;
    *x0 = a < gx ? a : gx; *y0 = b < gy ? b : gy;
    *x1 = c < gx ? c : gx; *y1 = d < gy ? d : gy;
}

/* auxiliary.h:58-77 (column-major 4x4, m[4c+r]) */
static inline v3 xform4x3(v3 p, const real* m)
{
    v3 t;
    t.x = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
    t.y = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
    t.z = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
    return t;
}
static inline void xform4x4(v3 p, const real* m, real* o)
{
    o[0] = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
    o[1] = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
    o[2] = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
    o[3] = m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15];
}

/* forward.cu:118-152: Sigma = R S^2 R^T, R from the UN-normalised quaternion (w,x,y,z),
 * stored upper triangle [xx,xy,xz,yy,yz,zz].  Written in standard (row-major) notation. */
static void cov3d_fwd(const real* s3, real mod, const real* q, real* cov)
{
    real r = q[0], x = q[1], y = q[2], z = q[3];
    real R[3][3];
    R[0][0] = (real)1 - (real)2 * (y * y + z * z); R[0][1] = (real)2 * (x * y - r * z); R[0][2] = (real)2 * (x * z + r * y);
    R[1][0] = (real)2 * (x * y + r * z); R[1][1] = (real)1 - (real)2 * (x * x + z * z); R[1][2] = (real)2 * (y * z - r * x);
    R[2][0] = (real)2 * (x * z - r * y); R[2][1] = (real)2 * (y * z + r * x); R[2][2] = (real)1 - (real)2 * (x * x + y * y);
    real s[3] = {mod * s3[0], mod * s3[1], mod * s3[2]};
    /* M = S R^T :  M[k][i] = s_k R[i][k];  Sigma_ij = sum_k M[k][i] M[k][j] */
    real M[3][3];
    for (int k = 0; k < 3; k++)
        for (int i = 0; i < 3; i++) M[k][i] = s[k] * R[i][k];
    real S[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) S[i][j] = M[0][i] * M[0][j] + M[1][i] * M[1][j] + M[2][i] * M[2][j];
    cov[0] = S[0][0]; cov[1] = S[0][1]; cov[2] = S[0][2];
    cov[3] = S[1][1]; cov[4] = S[1][2]; cov[5] = S[2][2];
}

/* forward.cu:74-113: EWA projection, cov2D = (J V) Sigma (J V)^T + 0.3 I.
 * Returns (a, b, c) and the intermediates needed by the backward. */
typedef struct {
    real tx, ty, tz;          /* view-space mean after the +-1.3 tanfov clamp of x,y */
    real xmul, ymul;          /* backward.cu:175-176: 0 where the clamp is active   */
    real Mx[2][3];            /* M = J V3 (2x3) */
    real a, b, c;             /* cov2D entries after the +0.3 low-pass */
    int near;                 /* tx/tz or ty/tz within a relative 1e-5 of the clamp limit */
} proj_t;

static void cov2d_fwd(v3 mean, real fx, real fy, real tanx, real tany, const real* cov3, const real* view, proj_t* o)
{
    v3 t = xform4x3(mean, view);
    real limx = (real)1.3 * tanx, limy = (real)1.3 * tany;
    real txtz = t.x / t.z, tytz = t.y / t.z;
    o->xmul = (txtz < -limx || txtz > limx) ? (real)0 : (real)1;
    o->ymul = (tytz < -limy || tytz > limy) ? (real)0 : (real)1;
    o->near = fabs(fabs((double)txtz) / limx - 1.0) <= 1e-5 || fabs(fabs((double)tytz) / limy - 1.0) <= 1e-5;
    t.x = rmin(limx, rmax(-limx, txtz)) * t.z;
    t.y = rmin(limy, rmax(-limy, tytz)) * t.z;
    o->tx = t.x; o->ty = t.y; o->tz = t.z;
    real J00 = fx / t.z, J02 = -(fx * t.x) / (t.z * t.z);
    real J11 = fy / t.z, J12 = -(fy * t.y) / (t.z * t.z);
    for (int k = 0; k < 3; k++) {
        /* V3[r][k] = view[4k + r] */
        o->Mx[0][k] = J00 * view[4 * k + 0] + J02 * view[4 * k + 2];
        o->Mx[1][k] = J11 * view[4 * k + 1] + J12 * view[4 * k + 2];
    }
    real S[3][3] = {{cov3[0], cov3[1], cov3[2]}, {cov3[1], cov3[3], cov3[4]}, {cov3[2], cov3[4], cov3[5]}};
    real u0[3], u1[3];
    for (int k = 0; k < 3; k++) {
        u0[k] = S[k][0] * o->Mx[0][0] + S[k][1] * o->Mx[0][1] + S[k][2] * o->Mx[0][2];
        u1[k] = S[k][0] * o->Mx[1][0] + S[k][1] * o->Mx[1][1] + S[k][2] * o->Mx[1][2];
    }
    real a = o->Mx[0][0] * u0[0] + o->Mx[0][1] * u0[1] + o->Mx[0][2] * u0[2];
    real b = o->Mx[0][0] * u1[0] + o->Mx[0][1] * u1[1] + o->Mx[0][2] * u1[2];
    real c = o->Mx[1][0] * u1[0] + o->Mx[1][1] * u1[1] + o->Mx[1][2] * u1[2];
    o->a = a + (real)0.3;
    o->b = b;
    o->c = c + (real)0.3;
}

/* forward.cu:20-71: SH -> RGB (+0.5, clamp >= 0, per-channel clamped flags) */
static void sh_fwd(int deg, int M, v3 pos, const real* campos, const real* sh, real* rgb, unsigned char* clamped,
                   unsigned char* near)
{
    real dx = pos.x - campos[0], dy = pos.y - campos[1], dz = pos.z - campos[2];
    real len = RSQRT(dx * dx + dy * dy + dz * dz);
    real x = dx / len, y = dy / len, z = dz / len;
    (void)M;
    for (int ch = 0; ch < 3; ch++) {
#define S(k) sh[3 * (k) + ch]
        real res = SH_C0 * S(0);
        if (deg > 0) {
            res = res - SH_C1 * y * S(1) + SH_C1 * z * S(2) - SH_C1 * x * S(3);
            if (deg > 1) {
                real xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                res = res + (SH_C2[0] * xy * S(4) + SH_C2[1] * yz * S(5) +
                             SH_C2[2] * ((real)2 * zz - xx - yy) * S(6) + SH_C2[3] * xz * S(7) +
                             SH_C2[4] * (xx - yy) * S(8));
                if (deg > 2) {
                    res = res + (SH_C3[0] * y * ((real)3 * xx - yy) * S(9) + SH_C3[1] * xy * z * S(10) +
                                 SH_C3[2] * y * ((real)4 * zz - xx - yy) * S(11) +
                                 SH_C3[3] * z * ((real)2 * zz - (real)3 * xx - (real)3 * yy) * S(12) +
                                 SH_C3[4] * x * ((real)4 * zz - xx - yy) * S(13) +
                                 SH_C3[5] * z * (xx - yy) * S(14) + SH_C3[6] * x * (xx - (real)3 * yy) * S(15));
                }
            }
        }
#undef S
        res = res + (real)0.5;
        clamped[ch] = res < (real)0;
        if (near && fabs((double)res) <= 1e-5) *near = 1; /* the clamp decision sits on its threshold */
        rgb[ch] = rmax(res, (real)0);
    }
}

/* ------------------------------------------------------------------------- */
/* Forward                                                                    */
/* ------------------------------------------------------------------------- */

typedef struct {
    int P, D, M, W, H;
    const real* bg;            /* [3] */
    const real* means3D;       /* [P,3] */
    const real* shs;           /* [P,M,3] or NULL */
    const real* colors;        /* [P,3] or NULL */
    const real* opacities;     /* [P] */
    const real* scales;        /* [P,3] or NULL */
    const real* rotations;     /* [P,4] or NULL */
    const real* cov3D_precomp; /* [P,6] or NULL */
    real scale_modifier;
    const real* view;          /* [16] */
    const real* proj;          /* [16] */
    const real* campos;        /* [3] */
    real tan_fovx, tan_fovy;
} oracle_in;

typedef struct {
    /* caller-provided outputs */
    real* out_color;  /* [3,H,W] */
    real* out_depth;  /* [H,W]   */
    int* radii;       /* [P]     */
    real* means2D;    /* [P,2]   */
    real* depths;     /* [P]     */
    real* conic_opacity; /* [P,4] */
    real* rgb;        /* [P,3]  (colors used for rendering) */
    unsigned char* clamped; /* [P,3] */
    int* tiles_touched;  /* [P] */
    real* final_T;    /* [H*W] */
    int* n_contrib;   /* [H*W] */
    int* ranges;      /* [tiles,2] */
    /* allocated here, freed by oracle_free_list */
    int* point_list;  /* [num_rendered] gaussian ids in (tile, depth, id) order */
    /* optional (NULL: not computed): threshold proximity, see the header */
    unsigned char* unstable_pix; /* [H*W] */
    unsigned char* unstable;     /* [P]   */
} oracle_fwd_out;

typedef struct { uint32_t tile; real depth; int id; } inst_t;

static int inst_cmp(const void* pa, const void* pb)
{
    const inst_t* a = (const inst_t*)pa;
    const inst_t* b = (const inst_t*)pb;
    if (a->tile != b->tile) return a->tile < b->tile ? -1 : 1;
    if (a->depth != b->depth) return a->depth < b->depth ? -1 : 1;
    /* cub's LSD radix sort is stable: equal keys keep the unsorted (Gaussian-id) order */
    return a->id < b->id ? -1 : (a->id > b->id);
}

/* forward.cu:155-256 (preprocessCUDA); auxiliary.h:139-164 (in_frustum) */
static void preprocess(const oracle_in* in, oracle_fwd_out* o, int gx, int gy, real fx, real fy)
{
#pragma omp parallel for schedule(static) num_threads(nthreads())
    for (int i = 0; i < in->P; i++) {
        o->radii[i] = 0;
        o->tiles_touched[i] = 0;
        v3 p = {in->means3D[3 * i], in->means3D[3 * i + 1], in->means3D[3 * i + 2]};
        real hom[4];
        xform4x4(p, in->proj, hom);
        real pw = (real)1 / (hom[3] + (real)0.0000001);
        v3 pv = xform4x3(p, in->view);
        if (pv.z <= (real)0.001) continue;
        real ppx = hom[0] * pw, ppy = hom[1] * pw;
        real cov3[6];
        const real* c3;
        if (in->cov3D_precomp) c3 = in->cov3D_precomp + 6 * i;
        else { cov3d_fwd(in->scales + 3 * i, in->scale_modifier, in->rotations + 4 * i, cov3); c3 = cov3; }
        proj_t pj;
        cov2d_fwd(p, fx, fy, in->tan_fovx, in->tan_fovy, c3, in->view, &pj);
        real det = pj.a * pj.c - pj.b * pj.b;
        if (det == (real)0) continue;
        real det_inv = (real)1 / det;
        real ca = pj.c * det_inv, cb = -pj.b * det_inv, cc = pj.a * det_inv;
        real mid = (real)0.5 * (pj.a + pj.c);
        real l1 = mid + RSQRT(rmax((real)0.1, mid * mid - det));
        real l2 = mid - RSQRT(rmax((real)0.1, mid * mid - det));
        real rad = RCEIL((real)3 * RSQRT(rmax(l1, l2)));
        real px = ndc2pix(ppx, in->W), py = ndc2pix(ppy, in->H);
        int x0, y0, x1, y1;
        get_rect(px, py, (int)rad, gx, gy, &x0, &y0, &x1, &y1);
        if ((x1 - x0) * (y1 - y0) == 0) continue;
        unsigned char nr = (unsigned char)pj.near;
        if (!in->colors) sh_fwd(in->D, in->M, p, in->campos, in->shs + (size_t)3 * in->M * i, o->rgb + 3 * i, o->clamped + 3 * i, &nr);
        else { for (int c = 0; c < 3; c++) { o->rgb[3 * i + c] = in->colors[3 * i + c]; o->clamped[3 * i + c] = 0; } }
        if (o->unstable) o->unstable[i] = nr;
        o->depths[i] = pv.z;
        o->radii[i] = (int)rad;
        o->means2D[2 * i] = px; o->means2D[2 * i + 1] = py;
        o->conic_opacity[4 * i] = ca; o->conic_opacity[4 * i + 1] = cb; o->conic_opacity[4 * i + 2] = cc;
        o->conic_opacity[4 * i + 3] = in->opacities[i];
        o->tiles_touched[i] = (y1 - y0) * (x1 - x0);
    }
}

/* forward.cu:261-393 (renderCUDA), one tile at a time, pixels sequential */
static long long render_tile(const oracle_in* in, oracle_fwd_out* o, int tx, int ty, int start, int end)
{
    long long evals = 0;
    for (int ly = 0; ly < BLOCK_Y; ly++)
        for (int lx = 0; lx < BLOCK_X; lx++) {
            int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
            if (px >= in->W || py >= in->H) continue;
            real T = 1, C[3] = {0, 0, 0}, D = (real)15;
            int contributor = 0, last = 0;
            unsigned char near = 0;
            for (int k = start; k < end; k++) {
                contributor++;
                evals++;
                int g = o->point_list[k];
                real dx = o->means2D[2 * g] - (real)px, dy = o->means2D[2 * g + 1] - (real)py;
                const real* co = o->conic_opacity + 4 * g;
                real power = POWER_OF(co, dx, dy);
                if (power > (real)0) continue;
                real alpha = rmin((real)0.99, co[3] * GEXP(power));
                if (fabs((double)alpha * 255.0 - 1.0) <= ALPHA_BAND) near = 1;
                if (alpha < (real)1 / (real)255) continue;
                real test_T = T * ((real)1 - alpha);
                if (fabs((double)test_T * 1e4 - 1.0) <= T_BAND) near = 1;
                if (test_T < (real)0.0001) break; /* done = true: no further entries are visited */
                for (int c = 0; c < 3; c++) C[c] += o->rgb[3 * g + c] * alpha * T;
                if (fabs((double)test_T * 2.0 - 1.0) <= T_BAND || fabs((double)T * 2.0 - 1.0) <= T_BAND) near |= 2;
                if (T > (real)0.5 && test_T < (real)0.5) D = o->depths[g];
                T = test_T;
                last = contributor;
            }
            int pid = py * in->W + px;
            o->final_T[pid] = T;
            o->n_contrib[pid] = last;
            for (int c = 0; c < 3; c++) o->out_color[c * in->H * in->W + pid] = C[c] + T * in->bg[c];
            o->out_depth[pid] = D;
            if (o->unstable_pix) o->unstable_pix[pid] = near;
        }
    return evals;
}

/* rasterizer_impl.cu:198-339 (Rasterizer::forward). Returns num_rendered. */
int oracle_forward(const oracle_in* in, oracle_fwd_out* o, long long* pair_evals)
{
    int W = in->W, H = in->H;
    real fy = (real)H / ((real)2 * in->tan_fovy);
    real fx = (real)W / ((real)2 * in->tan_fovx);
    int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    if (o->unstable) memset(o->unstable, 0, (size_t)in->P);
    preprocess(in, o, gx, gy, fx, fy);
    /* rasterizer_impl.cu:277-309: scan, duplicateWithKeys, stable sort by (tile, depth) */
    long long I = 0;
    for (int i = 0; i < in->P; i++) I += o->tiles_touched[i];
    inst_t* inst = (inst_t*)malloc(sizeof(inst_t) * (size_t)(I > 0 ? I : 1));
    long long off = 0;
    for (int i = 0; i < in->P; i++) {
        if (o->radii[i] <= 0) continue;
        int x0, y0, x1, y1;
        get_rect(o->means2D[2 * i], o->means2D[2 * i + 1], o->radii[i], gx, gy, &x0, &y0, &x1, &y1);
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                inst[off].tile = (uint32_t)(y * gx + x);
                inst[off].depth = o->depths[i];
                inst[off].id = i;
                off++;
            }
    }
    qsort(inst, (size_t)I, sizeof(inst_t), inst_cmp);
    o->point_list = (int*)malloc(sizeof(int) * (size_t)(I > 0 ? I : 1));
    for (long long k = 0; k < I; k++) o->point_list[k] = inst[k].id;
    /* rasterizer_impl.cu:116-138 + 311 (identifyTileRanges) */
    memset(o->ranges, 0, sizeof(int) * 2 * (size_t)gx * gy);
    for (long long k = 0; k < I; k++) {
        uint32_t t = inst[k].tile;
        if (k == 0 || inst[k - 1].tile != t) o->ranges[2 * t] = (int)k;
        if (k == I - 1 || inst[k + 1].tile != t) o->ranges[2 * t + 1] = (int)(k + 1);
    }
    free(inst);
    long long ev = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : ev) num_threads(nthreads())
    for (int t = 0; t < gx * gy; t++)
        ev += render_tile(in, o, t % gx, t / gx, o->ranges[2 * t], o->ranges[2 * t + 1]);
    if (pair_evals) *pair_evals = ev;
    if (o->unstable_pix && o->unstable) {
        /* every Gaussian with a (near-)contributing pair at a flagged pixel, up to the (near-)terminating
         * pair: its per-pair terms there depend on the flagged decision through T and the accumulated colour */
        for (int pid = 0; pid < W * H; pid++) {
            if (!(o->unstable_pix[pid] & 1)) continue;
            int px = pid % W, py = pid / W, t = (py / BLOCK_Y) * gx + px / BLOCK_X;
            int start = o->ranges[2 * t], end = o->ranges[2 * t + 1];
            double T = 1.0;
            for (int k = start; k < end; k++) {
                int g = o->point_list[k];
                double dx = (double)o->means2D[2 * g] - px, dy = (double)o->means2D[2 * g + 1] - py;
                const real* co = o->conic_opacity + 4 * g;
                double pw = -0.5 * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                if (pw > 0) continue;
                double a = co[3] * exp(pw);
                if (a > 0.99) a = 0.99;
                if (a * 255.0 < 1.0 - 2 * ALPHA_BAND) continue;
                o->unstable[g] = 1;
                if (a * 255.0 < 1.0) continue;
                T *= 1.0 - a;
                if (T * 1e4 < 1.0 - 2 * T_BAND) break;
            }
        }
    }
    return (int)I;
}

void oracle_free_list(oracle_fwd_out* o)
{
    free(o->point_list);
    o->point_list = NULL;
}

/* ------------------------------------------------------------------------- */
/* Backward                                                                   */
/* ------------------------------------------------------------------------- */

typedef struct {
    real* dmeans2D;  /* [P,3] */
    real* dcolors;   /* [P,3] */
    real* dopacity;  /* [P]   */
    real* dmeans3D;  /* [P,3] */
    real* dcov3D;    /* [P,6] */
    real* dsh;       /* [P,M,3] or NULL */
    real* dscales;   /* [P,3] */
    real* drot;      /* [P,4] */
} oracle_grads;

/* Per-Gaussian chain from the 2D quantities of one Gaussian to every
 * per-Gaussian output.  g2[0..1] = dL/dmean2D (NDC units), g2[2..4] = dL/dconic
 * (A, B/2, C as stored in float4 .x .y .w), g2[5] = dL/dopacity, g2[6..8] = dL/dcolor.
 * Outputs out[]: 0..2 dmean3D, 3..8 dcov3D, 9..11 dscale, 12..15 drot, 16.. dsh (3 per coeff).
 * backward.cu:144-274 (cov2D), 412-475 (cov3D), 480-530 (preprocess), 20-139 (SH). */
#define NOUT_FIXED 16
static void chain(const oracle_in* in, const oracle_fwd_out* fo, int g, const real* g2, real fx, real fy, real* out)
{
    int nsh = in->shs ? (in->D + 1) * (in->D + 1) : 0;
    for (int k = 0; k < NOUT_FIXED + 3 * nsh; k++) out[k] = 0;
    v3 m = {in->means3D[3 * g], in->means3D[3 * g + 1], in->means3D[3 * g + 2]};
    real cov3[6];
    const real* c3;
    if (in->cov3D_precomp) c3 = in->cov3D_precomp + 6 * g;
    else { cov3d_fwd(in->scales + 3 * g, in->scale_modifier, in->rotations + 4 * g, cov3); c3 = cov3; }
    /* --- computeCov2DCUDA (backward.cu:144-274) --- */
    proj_t pj;
    cov2d_fwd(m, fx, fy, in->tan_fovx, in->tan_fovy, c3, in->view, &pj);
    real a = pj.a, b = pj.b, c = pj.c;
    real gA = g2[2], gBh = g2[3], gC = g2[4];
    real denom = a * c - b * b;
    real dL_da = 0, dL_db = 0, dL_dc = 0;
    real denom2inv = (real)1 / ((denom * denom) + (real)0.0000001);
    real dcov[6] = {0, 0, 0, 0, 0, 0};
    if (denom2inv != (real)0) {
        dL_da = denom2inv * (-c * c * gA + (real)2 * b * c * gBh + (denom - a * c) * gC);
        dL_dc = denom2inv * (-a * a * gC + (real)2 * a * b * gBh + (denom - a * c) * gA);
        dL_db = denom2inv * (real)2 * (b * c * gA - (denom + (real)2 * b * b) * gBh + a * b * gC);
        /* dL/dSigma = M^T G M with G = [[da, db/2],[db/2, dc]]; off-diagonals counted twice */
        const real (*Mx)[3] = (const real(*)[3])pj.Mx;
        for (int i = 0; i < 3; i++)
            for (int j = i; j < 3; j++) {
                real v = Mx[0][i] * Mx[0][j] * dL_da + Mx[1][i] * Mx[1][j] * dL_dc +
                         (real)0.5 * (Mx[0][i] * Mx[1][j] + Mx[1][i] * Mx[0][j]) * dL_db;
                int idx = (i == 0) ? j : (i == 1 ? 2 + j : 5);
                dcov[idx] = (i == j) ? v : (real)2 * v;
            }
    }
    for (int k = 0; k < 6; k++) out[3 + k] = dcov[k];
    /* dL/dM = 2 G M Sigma (M = J V3, 2x3) */
    real S[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    real MS[2][3];
    for (int r = 0; r < 2; r++)
        for (int k = 0; k < 3; k++) MS[r][k] = pj.Mx[r][0] * S[0][k] + pj.Mx[r][1] * S[1][k] + pj.Mx[r][2] * S[2][k];
    real dM[2][3];
    for (int k = 0; k < 3; k++) {
        dM[0][k] = (real)2 * dL_da * MS[0][k] + dL_db * MS[1][k];
        dM[1][k] = (real)2 * dL_dc * MS[1][k] + dL_db * MS[0][k];
    }
    /* dL/dJ = dL/dM V3^T ; V3[r][k] = view[4k+r] */
    const real* V = in->view;
    real dJ00 = dM[0][0] * V[0] + dM[0][1] * V[4] + dM[0][2] * V[8];
    real dJ02 = dM[0][0] * V[2] + dM[0][1] * V[6] + dM[0][2] * V[10];
    real dJ11 = dM[1][0] * V[1] + dM[1][1] * V[5] + dM[1][2] * V[9];
    real dJ12 = dM[1][0] * V[2] + dM[1][1] * V[6] + dM[1][2] * V[10];
    real tz = (real)1 / pj.tz, tz2 = tz * tz, tz3 = tz2 * tz;
    real dtx = pj.xmul * -fx * tz2 * dJ02;
    real dty = pj.ymul * -fy * tz2 * dJ12;
    real dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + ((real)2 * fx * pj.tx) * tz3 * dJ02 + ((real)2 * fy * pj.ty) * tz3 * dJ12;
    /* transformVec4x3Transpose (auxiliary.h:89-97) */
    out[0] = V[0] * dtx + V[1] * dty + V[2] * dtz;
    out[1] = V[4] * dtx + V[5] * dty + V[6] * dtz;
    out[2] = V[8] * dtx + V[9] * dty + V[10] * dtz;
    /* --- preprocessCUDA bwd (backward.cu:480-530): mean via the projection --- */
    const real* pr = in->proj;
    real hom[4];
    xform4x4(m, pr, hom);
    real mw = (real)1 / (hom[3] + (real)0.0000001);
    real mul1 = (pr[0] * m.x + pr[4] * m.y + pr[8] * m.z + pr[12]) * mw * mw;
    real mul2 = (pr[1] * m.x + pr[5] * m.y + pr[9] * m.z + pr[13]) * mw * mw;
    real gx2 = g2[0], gy2 = g2[1];
    out[0] += (pr[0] * mw - pr[3] * mul1) * gx2 + (pr[1] * mw - pr[3] * mul2) * gy2;
    out[1] += (pr[4] * mw - pr[7] * mul1) * gx2 + (pr[5] * mw - pr[7] * mul2) * gy2;
    out[2] += (pr[8] * mw - pr[11] * mul1) * gx2 + (pr[9] * mw - pr[11] * mul2) * gy2;
    /* --- SH bwd (backward.cu:20-139) --- */
    if (in->shs) {
        const real* sh = in->shs + (size_t)3 * in->M * g;
        real dox = m.x - in->campos[0], doy = m.y - in->campos[1], doz = m.z - in->campos[2];
        real len = RSQRT(dox * dox + doy * doy + doz * doz);
        real x = dox / len, y = doy / len, z = doz / len;
        real dRGB[3];
        for (int ch = 0; ch < 3; ch++) dRGB[ch] = fo->clamped[3 * g + ch] ? (real)0 : g2[6 + ch];
        real* dsh = out + NOUT_FIXED;
        real ddir[3] = {0, 0, 0};
        int D = in->D;
        for (int ch = 0; ch < 3; ch++) {
#define SH(k) sh[3 * (k) + ch]
            real dRGBdx = 0, dRGBdy = 0, dRGBdz = 0;
            dsh[3 * 0 + ch] = SH_C0 * dRGB[ch];
            if (D > 0) {
                dsh[3 * 1 + ch] = -SH_C1 * y * dRGB[ch];
                dsh[3 * 2 + ch] = SH_C1 * z * dRGB[ch];
                dsh[3 * 3 + ch] = -SH_C1 * x * dRGB[ch];
                dRGBdx = -SH_C1 * SH(3);
                dRGBdy = -SH_C1 * SH(1);
                dRGBdz = SH_C1 * SH(2);
                if (D > 1) {
                    real xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                    dsh[3 * 4 + ch] = SH_C2[0] * xy * dRGB[ch];
                    dsh[3 * 5 + ch] = SH_C2[1] * yz * dRGB[ch];
                    dsh[3 * 6 + ch] = SH_C2[2] * ((real)2 * zz - xx - yy) * dRGB[ch];
                    dsh[3 * 7 + ch] = SH_C2[3] * xz * dRGB[ch];
                    dsh[3 * 8 + ch] = SH_C2[4] * (xx - yy) * dRGB[ch];
                    dRGBdx += SH_C2[0] * y * SH(4) + SH_C2[2] * (real)2 * -x * SH(6) + SH_C2[3] * z * SH(7) + SH_C2[4] * (real)2 * x * SH(8);
                    dRGBdy += SH_C2[0] * x * SH(4) + SH_C2[1] * z * SH(5) + SH_C2[2] * (real)2 * -y * SH(6) + SH_C2[4] * (real)2 * -y * SH(8);
                    dRGBdz += SH_C2[1] * y * SH(5) + SH_C2[2] * (real)2 * (real)2 * z * SH(6) + SH_C2[3] * x * SH(7);
                    if (D > 2) {
                        dsh[3 * 9 + ch] = SH_C3[0] * y * ((real)3 * xx - yy) * dRGB[ch];
                        dsh[3 * 10 + ch] = SH_C3[1] * xy * z * dRGB[ch];
                        dsh[3 * 11 + ch] = SH_C3[2] * y * ((real)4 * zz - xx - yy) * dRGB[ch];
                        dsh[3 * 12 + ch] = SH_C3[3] * z * ((real)2 * zz - (real)3 * xx - (real)3 * yy) * dRGB[ch];
                        dsh[3 * 13 + ch] = SH_C3[4] * x * ((real)4 * zz - xx - yy) * dRGB[ch];
                        dsh[3 * 14 + ch] = SH_C3[5] * z * (xx - yy) * dRGB[ch];
                        dsh[3 * 15 + ch] = SH_C3[6] * x * (xx - (real)3 * yy) * dRGB[ch];
                        dRGBdx += SH_C3[0] * SH(9) * (real)3 * (real)2 * xy + SH_C3[1] * SH(10) * yz +
                                  SH_C3[2] * SH(11) * (real)-2 * xy + SH_C3[3] * SH(12) * (real)-3 * (real)2 * xz +
                                  SH_C3[4] * SH(13) * ((real)-3 * xx + (real)4 * zz - yy) +
                                  SH_C3[5] * SH(14) * (real)2 * xz + SH_C3[6] * SH(15) * (real)3 * (xx - yy);
                        dRGBdy += SH_C3[0] * SH(9) * (real)3 * (xx - yy) + SH_C3[1] * SH(10) * xz +
                                  SH_C3[2] * SH(11) * ((real)-3 * yy + (real)4 * zz - xx) +
                                  SH_C3[3] * SH(12) * (real)-3 * (real)2 * yz + SH_C3[4] * SH(13) * (real)-2 * xy +
                                  SH_C3[5] * SH(14) * (real)-2 * yz + SH_C3[6] * SH(15) * (real)-3 * (real)2 * xy;
                        dRGBdz += SH_C3[1] * SH(10) * xy + SH_C3[2] * SH(11) * (real)4 * (real)2 * yz +
                                  SH_C3[3] * SH(12) * (real)3 * ((real)2 * zz - xx - yy) +
                                  SH_C3[4] * SH(13) * (real)4 * (real)2 * xz + SH_C3[5] * SH(14) * (xx - yy);
                    }
                }
            }
#undef SH
            ddir[0] += dRGBdx * dRGB[ch];
            ddir[1] += dRGBdy * dRGB[ch];
            ddir[2] += dRGBdz * dRGB[ch];
        }
        /* dnormvdv (auxiliary.h:107-117) */
        real sum2 = dox * dox + doy * doy + doz * doz;
        real invsum32 = (real)1 / RSQRT(sum2 * sum2 * sum2);
        out[0] += ((sum2 - dox * dox) * ddir[0] - doy * dox * ddir[1] - doz * dox * ddir[2]) * invsum32;
        out[1] += (-dox * doy * ddir[0] + (sum2 - doy * doy) * ddir[1] - doz * doy * ddir[2]) * invsum32;
        out[2] += (-dox * doz * ddir[0] - doy * doz * ddir[1] + (sum2 - doz * doz) * ddir[2]) * invsum32;
    }
    /* --- computeCov3D bwd (backward.cu:412-475) --- */
    if (in->scales) {
        const real* q = in->rotations + 4 * g;
        real r = q[0], x = q[1], y = q[2], z = q[3];
        real R[3][3];
        R[0][0] = (real)1 - (real)2 * (y * y + z * z); R[0][1] = (real)2 * (x * y - r * z); R[0][2] = (real)2 * (x * z + r * y);
        R[1][0] = (real)2 * (x * y + r * z); R[1][1] = (real)1 - (real)2 * (x * x + z * z); R[1][2] = (real)2 * (y * z - r * x);
        R[2][0] = (real)2 * (x * z - r * y); R[2][1] = (real)2 * (y * z + r * x); R[2][2] = (real)1 - (real)2 * (x * x + y * y);
        real s[3];
        for (int k = 0; k < 3; k++) s[k] = in->scale_modifier * in->scales[3 * g + k];
        real Gs[3][3] = {{dcov[0], (real)0.5 * dcov[1], (real)0.5 * dcov[2]},
                         {(real)0.5 * dcov[1], dcov[3], (real)0.5 * dcov[4]},
                         {(real)0.5 * dcov[2], (real)0.5 * dcov[4], dcov[5]}};
        /* Sigma = M^T M with M = S R^T (M[k][i] = s_k R[i][k]);  dL/dM = 2 M Gs */
        real Mm[3][3], dMm[3][3];
        for (int k = 0; k < 3; k++)
            for (int i = 0; i < 3; i++) Mm[k][i] = s[k] * R[i][k];
        for (int k = 0; k < 3; k++)
            for (int j = 0; j < 3; j++) dMm[k][j] = (real)2 * (Mm[k][0] * Gs[0][j] + Mm[k][1] * Gs[1][j] + Mm[k][2] * Gs[2][j]);
        /* dL/ds_k = sum_i dM[k][i] R[i][k]  (the reference does not multiply by scale_modifier) */
        for (int k = 0; k < 3; k++) out[9 + k] = dMm[k][0] * R[0][k] + dMm[k][1] * R[1][k] + dMm[k][2] * R[2][k];
        /* dL/dR[i][k] = dM[k][i] s_k */
        real dR[3][3];
        for (int i = 0; i < 3; i++)
            for (int k = 0; k < 3; k++) dR[i][k] = dMm[k][i] * s[k];
        out[12] = (real)2 * z * (dR[1][0] - dR[0][1]) + (real)2 * y * (dR[0][2] - dR[2][0]) + (real)2 * x * (dR[2][1] - dR[1][2]);
        out[13] = (real)2 * y * (dR[0][1] + dR[1][0]) + (real)2 * z * (dR[0][2] + dR[2][0]) + (real)2 * r * (dR[2][1] - dR[1][2]) - (real)4 * x * (dR[1][1] + dR[2][2]);
        out[14] = (real)2 * x * (dR[0][1] + dR[1][0]) + (real)2 * r * (dR[0][2] - dR[2][0]) + (real)2 * z * (dR[1][2] + dR[2][1]) - (real)4 * y * (dR[0][0] + dR[2][2]);
        out[15] = (real)2 * r * (dR[1][0] - dR[0][1]) + (real)2 * x * (dR[0][2] + dR[2][0]) + (real)2 * y * (dR[1][2] + dR[2][1]) - (real)4 * z * (dR[0][0] + dR[1][1]);
    }
}

static inline real apply_power(real v, int p) { return p == 1 ? v : RPOW(v, (real)p); }

/* Per-pixel back-to-front pass (backward.cu:586-748 / 850-1040).  Every
 * contributing pair's terms go to the record of its (tile, Gaussian) instance
 * (its index k in point_list): upstream mode the 9 per-pair 2D quantities,
 * fused mode the per-pair chain outputs after powf.  Tiles run in parallel,
 * the pixels of a tile in order; the records are then added per Gaussian in
 * instance order, so the sums do not depend on the thread count. */
#define NV_FUSED_FIXED 22 /* dcolors 3, dmeans2D 2, dmeans3D 3, dcov3D 6, dscales 3, drot 4, dopacity 1 */
int oracle_backward(const oracle_in* in, const oracle_fwd_out* fo, const real* dL_dpix, int mode, int power,
                    oracle_grads* go, long long* pair_evals, long long* pair_contrib, oracle_grads* gs)
{
    /* gs (upstream mode, optional): per-element error scale of every gradient -- the
     * chain's Jacobian in absolute value applied to the per-Gaussian sums of |per-pair
     * term| (a float32 sum of those terms is accurate to a small multiple of
     * eps * scale whatever the cancellation); NULL skips it. */
    int P = in->P, W = in->W, H = in->H;
    real fy = (real)H / ((real)2 * in->tan_fovy);
    real fx = (real)W / ((real)2 * in->tan_fovx);
    int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    int nsh = in->shs ? (in->D + 1) * (in->D + 1) : 0;
    if (mode == GSR_ORACLE_UPSTREAM && power != 1) return -1;
    /* zero all outputs (rasterize_points.cu:151-159) */
    memset(go->dmeans2D, 0, sizeof(real) * 3 * (size_t)P);
    memset(go->dcolors, 0, sizeof(real) * 3 * (size_t)P);
    memset(go->dopacity, 0, sizeof(real) * (size_t)P);
    memset(go->dmeans3D, 0, sizeof(real) * 3 * (size_t)P);
    memset(go->dcov3D, 0, sizeof(real) * 6 * (size_t)P);
    if (go->dsh) memset(go->dsh, 0, sizeof(real) * 3 * (size_t)in->M * P);
    memset(go->dscales, 0, sizeof(real) * 3 * (size_t)P);
    memset(go->drot, 0, sizeof(real) * 4 * (size_t)P);
    if (gs) {
        if (mode != GSR_ORACLE_UPSTREAM) return -1;
        memset(gs->dmeans2D, 0, sizeof(real) * 3 * (size_t)P);
        memset(gs->dcolors, 0, sizeof(real) * 3 * (size_t)P);
        memset(gs->dopacity, 0, sizeof(real) * (size_t)P);
        memset(gs->dmeans3D, 0, sizeof(real) * 3 * (size_t)P);
        memset(gs->dcov3D, 0, sizeof(real) * 6 * (size_t)P);
        if (gs->dsh) memset(gs->dsh, 0, sizeof(real) * 3 * (size_t)in->M * P);
        memset(gs->dscales, 0, sizeof(real) * 3 * (size_t)P);
        memset(gs->drot, 0, sizeof(real) * 4 * (size_t)P);
    }
    long long I = 0;
    for (int t = 0; t < gx * gy; t++)
        if (fo->ranges[2 * t + 1] > I) I = fo->ranges[2 * t + 1];
    const int NVS = mode == GSR_ORACLE_UPSTREAM ? 9 : NV_FUSED_FIXED + 3 * nsh;
    const int NV = (mode == GSR_ORACLE_UPSTREAM && gs) ? 18 : NVS; /* + the |term| sums */
    real* rec = (real*)calloc((size_t)(I > 0 ? I : 1) * NV, sizeof(real));
    if (!rec) return -2;
    real ddelx = (real)(0.5 * W), ddely = (real)(0.5 * H);
    real bgdot_w[3] = {in->bg[0], in->bg[1], in->bg[2]};
    long long ev = 0, ct = 0;
#pragma omp parallel num_threads(nthreads()) reduction(+ : ev, ct)
    {
        real* outbuf = (real*)malloc(sizeof(real) * (NOUT_FIXED + 48));
#pragma omp for schedule(dynamic, 4)
        for (int t = 0; t < gx * gy; t++) {
            int tx = t % gx, ty = t / gx;
            int start = fo->ranges[2 * t], end = fo->ranges[2 * t + 1];
            for (int ly = 0; ly < BLOCK_Y; ly++)
                for (int lx = 0; lx < BLOCK_X; lx++) {
                    int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                    if (px >= W || py >= H) continue;
                    int pid = py * W + px;
                    real T_final = fo->final_T[pid];
                    real T = T_final;
                    int contributor = end - start;
                    int last = fo->n_contrib[pid];
                    real accum[3] = {0, 0, 0}, last_color[3] = {0, 0, 0}, last_alpha = 0;
                    real dpix[3];
                    for (int c = 0; c < 3; c++) dpix[c] = dL_dpix[c * H * W + pid];
                    real bg_dot = bgdot_w[0] * dpix[0] + bgdot_w[1] * dpix[1] + bgdot_w[2] * dpix[2];
                    for (int k = end - 1; k >= start; k--) {
                        contributor--;
                        if (contributor >= last) continue;
                        ev++;
                        int g = fo->point_list[k];
                        real dx = fo->means2D[2 * g] - (real)px, dy = fo->means2D[2 * g + 1] - (real)py;
                        const real* co = fo->conic_opacity + 4 * g;
                        real power_ = POWER_OF(co, dx, dy);
                        if (power_ > (real)0) continue;
                        real G = GEXP(power_);
                        real alpha = rmin((real)0.99, co[3] * G);
                        if (alpha < (real)1 / (real)255) continue;
                        ct++;
                        T = T / ((real)1 - alpha);
                        real dchannel_dcolor = alpha * T;
                        real g2[9];
                        real dL_dalpha = 0;
                        for (int c = 0; c < 3; c++) {
                            real col = fo->rgb[3 * g + c];
                            accum[c] = last_alpha * last_color[c] + ((real)1 - last_alpha) * accum[c];
                            last_color[c] = col;
                            dL_dalpha += (col - accum[c]) * dpix[c];
                            g2[6 + c] = dchannel_dcolor * dpix[c];
                        }
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final / ((real)1 - alpha)) * bg_dot;
                        real dL_dG = co[3] * dL_dalpha;
                        real gdx = G * dx, gdy = G * dy;
                        real dG_ddelx = -gdx * co[0] - gdy * co[1];
                        real dG_ddely = -gdy * co[2] - gdx * co[1];
                        g2[0] = dL_dG * dG_ddelx * ddelx;
                        g2[1] = dL_dG * dG_ddely * ddely;
                        g2[2] = (real)-0.5 * gdx * dx * dL_dG;
                        g2[3] = (real)-0.5 * gdx * dy * dL_dG;
                        g2[4] = (real)-0.5 * gdy * dy * dL_dG;
                        g2[5] = G * dL_dalpha;
                        real* r = rec + (size_t)k * NV;
                        if (mode == GSR_ORACLE_UPSTREAM) {
                            for (int q = 0; q < 9; q++) r[q] += g2[q];
                            if (NV == 18)
                                for (int q = 0; q < 9; q++) r[9 + q] += g2[q] < 0 ? -g2[q] : g2[q];
                        } else {
                            /* backward.cu:1040-1137: chain per pair, powf per pair, then sum */
                            chain(in, fo, g, g2, fx, fy, outbuf);
                            for (int c = 0; c < 3; c++) r[c] += apply_power(g2[6 + c], power);
                            r[3] += apply_power(g2[0], power);
                            r[4] += apply_power(g2[1], power);
                            for (int c = 0; c < 3; c++) r[5 + c] += apply_power(outbuf[c], power);
                            for (int c = 0; c < 6; c++) r[8 + c] += apply_power(outbuf[3 + c], power);
                            if (in->scales) {
                                for (int c = 0; c < 3; c++) r[14 + c] += apply_power(outbuf[9 + c], power);
                                for (int c = 0; c < 4; c++) r[17 + c] += apply_power(outbuf[12 + c], power);
                            }
                            r[21] += apply_power(g2[5], power);
                            for (int c = 0; c < 3 * nsh; c++) r[22 + c] += apply_power(outbuf[NOUT_FIXED + c], power);
                        }
                    }
                }
        }
        free(outbuf);
    }
    /* per-Gaussian sums of the instance records, in instance order */
    real* acc = (real*)calloc((size_t)(P > 0 ? P : 1) * NV, sizeof(real));
    for (long long k = 0; k < I; k++) {
        int g = fo->point_list[k];
        real* a = acc + (size_t)g * NV;
        const real* r = rec + (size_t)k * NV;
        for (int q = 0; q < NV; q++) a[q] += r[q];
    }
    free(rec);
    if (mode == GSR_ORACLE_UPSTREAM) {
#pragma omp parallel num_threads(nthreads())
        {
            real* outbuf = (real*)malloc(sizeof(real) * (NOUT_FIXED + 48));
#pragma omp for schedule(static)
            for (int g = 0; g < P; g++) {
                if (fo->radii[g] <= 0) continue;
                const real* a2 = acc + (size_t)NV * g;
                go->dmeans2D[3 * g] = a2[0];
                go->dmeans2D[3 * g + 1] = a2[1];
                go->dopacity[g] = a2[5];
                for (int c = 0; c < 3; c++) go->dcolors[3 * g + c] = a2[6 + c];
                chain(in, fo, g, a2, fx, fy, outbuf);
                for (int c = 0; c < 3; c++) go->dmeans3D[3 * g + c] = outbuf[c];
                for (int c = 0; c < 6; c++) go->dcov3D[6 * g + c] = outbuf[3 + c];
                if (go->dsh && nsh > 0)
                    for (int c = 0; c < 3 * nsh; c++) go->dsh[(size_t)3 * in->M * g + c] = outbuf[NOUT_FIXED + c];
                if (in->scales) {
                    for (int c = 0; c < 3; c++) go->dscales[3 * g + c] = outbuf[9 + c];
                    for (int c = 0; c < 4; c++) go->drot[4 * g + c] = outbuf[12 + c];
                }
                if (NV == 18) { /* error scale: |J| applied to the |term| sums (chain is linear in g2) */
                    const real* s2 = acc + (size_t)18 * g + 9;
                    real sc[NOUT_FIXED + 48], e[9], col[NOUT_FIXED + 48];
                    const int no = NOUT_FIXED + 3 * nsh;
                    for (int q = 0; q < no; q++) sc[q] = 0;
                    for (int q = 0; q < 9; q++) {
                        if (s2[q] == 0) continue;
                        for (int u = 0; u < 9; u++) e[u] = u == q ? 1 : 0;
                        chain(in, fo, g, e, fx, fy, col);
                        for (int o2 = 0; o2 < no; o2++) sc[o2] += (col[o2] < 0 ? -col[o2] : col[o2]) * s2[q];
                    }
                    gs->dmeans2D[3 * g] = s2[0];
                    gs->dmeans2D[3 * g + 1] = s2[1];
                    gs->dopacity[g] = s2[5];
                    for (int c = 0; c < 3; c++) gs->dcolors[3 * g + c] = s2[6 + c];
                    for (int c = 0; c < 3; c++) gs->dmeans3D[3 * g + c] = sc[c];
                    for (int c = 0; c < 6; c++) gs->dcov3D[6 * g + c] = sc[3 + c];
                    if (gs->dsh && nsh > 0)
                        for (int c = 0; c < 3 * nsh; c++) gs->dsh[(size_t)3 * in->M * g + c] = sc[NOUT_FIXED + c];
                    if (in->scales) {
                        for (int c = 0; c < 3; c++) gs->dscales[3 * g + c] = sc[9 + c];
                        for (int c = 0; c < 4; c++) gs->drot[4 * g + c] = sc[12 + c];
                    }
                }
            }
            free(outbuf);
        }
    } else {
        for (int g = 0; g < P; g++) {
            const real* a = acc + (size_t)NV * g;
            for (int c = 0; c < 3; c++) go->dcolors[3 * g + c] = a[c];
            go->dmeans2D[3 * g] = a[3];
            go->dmeans2D[3 * g + 1] = a[4];
            for (int c = 0; c < 3; c++) go->dmeans3D[3 * g + c] = a[5 + c];
            for (int c = 0; c < 6; c++) go->dcov3D[6 * g + c] = a[8 + c];
            for (int c = 0; c < 3; c++) go->dscales[3 * g + c] = a[14 + c];
            for (int c = 0; c < 4; c++) go->drot[4 * g + c] = a[17 + c];
            go->dopacity[g] = a[21];
            if (go->dsh && nsh > 0)
                for (int c = 0; c < 3 * nsh; c++) go->dsh[(size_t)3 * in->M * g + c] = a[22 + c];
        }
    }
    free(acc);
    if (pair_evals) *pair_evals = ev;
    if (pair_contrib) *pair_contrib = ct;
    return 0;
}

/* rasterizer_impl.cu:54-67 (checkFrustum) */
void oracle_mark_visible(int P, const real* means3D, const real* view, unsigned char* visible)
{
    for (int i = 0; i < P; i++) {
        v3 p = {means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
        v3 pv = xform4x3(p, view);
        visible[i] = pv.z > (real)0.001;
    }
}

int oracle_real_size(void) { return (int)sizeof(real); }
int oracle_threads(void) { return nthreads(); }
