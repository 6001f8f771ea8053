/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see of2d_oracle.h).
 *
 * A from-scratch C restatement of the arithmetic of tjwdraper/OpticalFlow2d,
 * operation for operation in the same fp32 order, so that it reproduces the
 * reference bit for bit when compiled with -O2 -ffp-contract=off on x86-64.
 * Citations are `file:line` relative to the reference repository root.
 *
 * Conventions restated from the reference:
 *  - fields are contiguous, idx = i + j*dimx, x (= i) is the fast axis
 *    (src/Field.tpp:13);
 *  - an Image is float, a Motion is interleaved {x,y} float pairs
 *    (src/Motion.h:7, src/coord2d.h:149);
 *  - coord2d<float>::operator/ throws "Divide by zero exception" when the
 *    divisor is 0 (src/coord2d.h:95-108) — emulated with setjmp/longjmp;
 *  - std::pow(float,int) promotes to double (C++11 <cmath>), so Motion::norm
 *    and Motion::maxabs square in double (src/Motion.cpp:42-58);
 *  - exp(float) in Kernel.cpp resolves to the float overload (libstdc++
 *    <math.h> exports std::exp), i.e. expf (src/Kernel.cpp:61).
 */
#include "of2d_oracle.h"

#include <math.h>
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float x, y;
} v2;

/* ------------------------------------------------------------------ errors */
static jmp_buf *g_jb = NULL;
static char g_err[512];

static void raise_err(const char *msg) {
    snprintf(g_err, sizeof g_err, "%s", msg);
    if (g_jb) longjmp(*g_jb, 1);
    fprintf(stderr, "oracle: uncaught error: %s\n", msg);
    abort();
}

const char *oracle_last_error(void) { return g_err; }

/* ------------------------------------------------------------------ printing */
static int g_capture = 0;
static char *g_out = NULL;
static size_t g_out_len = 0, g_out_cap = 0;

void oracle_capture_output(int on) { g_capture = on; }
void oracle_clear_output(void) {
    g_out_len = 0;
    if (g_out) g_out[0] = 0;
}
const char *oracle_captured_output(void) { return g_out ? g_out : ""; }

/* mexPrintf stand-in for the oracle's own output (not a reference build) */
static void oprintf(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (n < 0) return;
    if ((size_t)n >= sizeof buf) n = sizeof buf - 1;
    if (!g_capture) {
        fputs(buf, stdout);
        return;
    }
    if (g_out_len + (size_t)n + 1 > g_out_cap) {
        size_t nc = g_out_cap ? g_out_cap * 2 : 4096;
        while (nc < g_out_len + (size_t)n + 1) nc *= 2;
        g_out = (char *)realloc(g_out, nc);
        g_out_cap = nc;
    }
    memcpy(g_out + g_out_len, buf, (size_t)n + 1);
    g_out_len += (size_t)n;
}

/* ------------------------------------------------------------------ coord2d */
static inline v2 V(float x, float y) {
    v2 r;
    r.x = x;
    r.y = y;
    return r;
}
static inline v2 vadd(v2 a, v2 b) { return V(a.x + b.x, a.y + b.y); }
static inline v2 vsub(v2 a, v2 b) { return V(a.x - b.x, a.y - b.y); }
static inline v2 vmul(v2 a, float s) { return V(a.x * s, a.y * s); }
/* src/coord2d.h:95-100 */
static inline v2 vdiv(v2 a, float s) {
    if (s == 0) raise_err("Divide by zero exception");
    return V(a.x / s, a.y / s);
}

/* loop order knob: every pointwise pass below is order independent; the
 * reference walks i outer / j inner (strided).  The SOR sweep always walks in
 * reference order because its result depends on it. */
static int g_refloop = 0;
void oracle_set_reference_loop_order(int on) { g_refloop = on; }

#define FOR_IJ(DX, DY, ...)                                                  \
    do {                                                                      \
        if (g_refloop) {                                                      \
            for (unsigned i = 0; i < (unsigned)(DX); i++)                     \
                for (unsigned j = 0; j < (unsigned)(DY); j++) {               \
                    unsigned idx = i + j * (unsigned)(DX);                    \
                    __VA_ARGS__                                               \
                }                                                             \
        } else {                                                              \
            for (unsigned j = 0; j < (unsigned)(DY); j++)                     \
                for (unsigned i = 0; i < (unsigned)(DX); i++) {               \
                    unsigned idx = i + j * (unsigned)(DX);                    \
                    __VA_ARGS__                                               \
                }                                                             \
        }                                                                     \
    } while (0)

/* ------------------------------------------------------------------ gradients.h */
/* src/gradients.h:9-19 */
static inline float pdx_f(const float *f, unsigned idx, unsigned i, unsigned dx) {
    if (i == 0) return f[idx + 1] - f[idx];
    if (i == dx - 1) return f[idx] - f[idx - 1];
    return (f[idx + 1] - f[idx - 1]) / 2.0f;
}
/* src/gradients.h:21-32 */
static inline float pdy_f(const float *f, unsigned idx, unsigned j, unsigned dx, unsigned dy) {
    if (j == 0) return f[idx + dx] - f[idx];
    if (j == dy - 1) return f[idx] - f[idx - dx];
    return (f[idx + dx] - f[idx - dx]) / 2.0f;
}
static inline v2 pdx_v(const v2 *f, unsigned idx, unsigned i, unsigned dx) {
    if (i == 0) return vsub(f[idx + 1], f[idx]);
    if (i == dx - 1) return vsub(f[idx], f[idx - 1]);
    return vdiv(vsub(f[idx + 1], f[idx - 1]), 2.0f);
}
static inline v2 pdy_v(const v2 *f, unsigned idx, unsigned j, unsigned dx, unsigned dy) {
    if (j == 0) return vsub(f[idx + dx], f[idx]);
    if (j == dy - 1) return vsub(f[idx], f[idx - dx]);
    return vdiv(vsub(f[idx + dx], f[idx - dx]), 2.0f);
}
/* src/gradients.h:71-80 */
static inline v2 qlap_v(const v2 *f, unsigned idx, unsigned i, unsigned j, unsigned dx,
                        unsigned dy) {
    if (i == 0 || i == dx - 1 || j == 0 || j == dy - 1) return V(0.0f, 0.0f);
    return vdiv(vadd(vadd(vadd(f[idx - 1], f[idx + 1]), f[idx - dx]), f[idx + dx]), 4.0f);
}

/* ------------------------------------------------------------------ Field ops */
/* Logger norm precision knob (test infrastructure).  0: the reference's
 * Motion::norm, a sequential FLOAT running sum (below).  1: the same
 * magnitudes summed in double and divided as the GPU path does (registration.cpp
 * logger_error: (float)sum / (float)n), i.e. the Logger error the reference
 * would compute without fp32 running-sum rounding; the GPU's fp64 tree sums
 * of fp32 per-lane partials agree with it to ~1e-7 relative.  Only the
 * convergence fixtures (tests/golden/make_convergence.py) use 1. */
static int g_logger_fp64 = 0;
void oracle_set_logger_fp64(int on) { g_logger_fp64 = on; }

/* src/Motion.cpp:42-49: float accumulation of a double magnitude */
static float motion_norm(const v2 *u, unsigned n) {
    if (g_logger_fp64) {
        double s = 0.0;
        for (unsigned i = 0; i < n; i++) {
            double px = (double)u[i].x, py = (double)u[i].y;
            s += sqrt(px * px + py * py);
        }
        return (float)s / (float)n;
    }
    float norm = 0.0f;
    for (unsigned i = 0; i < n; i++) {
        double px = (double)u[i].x, py = (double)u[i].y;
        norm = (float)((double)norm + sqrt(px * px + py * py));
    }
    return norm / (float)n;
}
/* src/Motion.cpp:51-58 (squares .y twice, as the reference does) */
static float motion_maxabs(const v2 *u, unsigned n) {
    float m = 0.0f;
    for (unsigned i = 0; i < n; i++) {
        double py = (double)u[i].y;
        float normsq = (float)(py * py + py * py);
        m = (m < normsq) ? normsq : m; /* std::max(m, normsq) */
    }
    return sqrtf(m);
}

float oracle_motion_norm(const float *u, int n) { return motion_norm((const v2 *)u, (unsigned)n); }
/* the float running sum of src/Motion.cpp:43-46 before the division by n
 * (checker of the device's of2d_motion_norms) */
float oracle_motion_norm_sum(const float *u, int n) {
    float norm = 0.0f;
    for (unsigned i = 0; i < (unsigned)n; i++) {
        double px = (double)u[2 * i], py = (double)u[2 * i + 1];
        norm = (float)((double)norm + sqrt(px * px + py * py));
    }
    return norm;
}
float oracle_motion_maxabs(const float *u, int n) {
    return motion_maxabs((const v2 *)u, (unsigned)n);
}

/* src/Image.cpp:96-104 */
static float image_min(const float *I, unsigned n) {
    float m = I[0];
    for (unsigned i = 1; i < n; i++)
        if (I[i] < m) m = I[i];
    return m;
}
float oracle_image_min(const float *I, int n) { return image_min(I, (unsigned)n); }

/* src/Field.tpp:75-143 (T = float) */
static void downsample_f(const float *in, unsigned dxi, unsigned dyi, float *out, unsigned dxo,
                         unsigned dyo) {
    if (dxo > dxi || dyo > dyi) raise_err("Error in Field<T>::downSample: dimensions");
    if (dxo == 0 || dyo == 0) raise_err("Divide by zero exception");
    unsigned fx = dxi / dxo, fy = dyi / dyo, sizein = dxi * dyi;
    FOR_IJ(dxo, dyo, {
        unsigned idxin = i * fx + j * fy * dxi;
        float val = 0.0f;
        int p = 0;
        for (unsigned ii = 0; ii < fx; ii++)
            for (unsigned jj = 0; jj < fy; jj++) {
                unsigned k = idxin + ii + jj * dxi;
                if (k >= sizein) continue;
                val += in[k];
                p++;
            }
        if (p != 0) out[idx] = val / (float)p;
    });
}
static void downsample_v(const v2 *in, unsigned dxi, unsigned dyi, v2 *out, unsigned dxo,
                         unsigned dyo) {
    if (dxo > dxi || dyo > dyi) raise_err("Error in Field<T>::downSample: dimensions");
    if (dxo == 0 || dyo == 0) raise_err("Divide by zero exception");
    unsigned fx = dxi / dxo, fy = dyi / dyo, sizein = dxi * dyi;
    FOR_IJ(dxo, dyo, {
        unsigned idxin = i * fx + j * fy * dxi;
        v2 val = V(0.0f, 0.0f);
        int p = 0;
        for (unsigned ii = 0; ii < fx; ii++)
            for (unsigned jj = 0; jj < fy; jj++) {
                unsigned k = idxin + ii + jj * dxi;
                if (k >= sizein) continue;
                val = vadd(val, in[k]);
                p++;
            }
        if (p != 0) out[idx] = vdiv(val, (float)p);
    });
}

/* src/Field.tpp:145-206 (bilinear, renormalised by the valid weight) */
#define UPSAMPLE_BODY(T, MUL, ADD, DIV, ASSIGN)                                   \
    float px = (float)i * (float)dxi / (float)dxo;                                \
    int ddx = (int)floorf(px);                                                    \
    float fxx = px - (float)ddx;                                                  \
    float py = (float)j * (float)dyi / (float)dyo;                                \
    int ddy = (int)floorf(py);                                                    \
    float fyy = py - (float)ddy;                                                  \
    unsigned idxO = (unsigned)ddx + (unsigned)ddy * dxi;                          \
    if (idxO >= sizein) continue;                                                 \
    T val = MUL(MUL(in[idxO], (1 - fxx)), (1 - fyy));                             \
    float weight = (1 - fxx) * (1 - fyy);                                         \
    if ((unsigned)ddx < dxi - 1) {                                                \
        val = ADD(val, MUL(MUL(in[idxO + 1], fxx), (1 - fyy)));                   \
        weight += fxx * (1 - fyy);                                                \
    }                                                                             \
    if ((unsigned)ddy < dyi - 1) {                                                \
        val = ADD(val, MUL(MUL(in[idxO + dxi], (1 - fxx)), fyy));                 \
        weight += (1 - fxx) * fyy;                                                \
    }                                                                             \
    if ((unsigned)ddx < dxi - 1 && (unsigned)ddy < dyi - 1) {                     \
        val = ADD(val, MUL(MUL(in[idxO + 1 + dxi], fxx), fyy));                   \
        weight += fxx * fyy;                                                      \
    }                                                                             \
    if (weight != 0) ASSIGN;

static inline float fmul_(float a, float b) { return a * b; }
static inline float fadd_(float a, float b) { return a + b; }

static void upsample_f(const float *in, unsigned dxi, unsigned dyi, float *out, unsigned dxo,
                       unsigned dyo) {
    if (dxo < dxi || dyo < dyi) raise_err("Error in Field<T>::upSample: dimensions");
    unsigned sizein = dxi * dyi;
    /* (float)i * dimin.x: unsigned promoted to float (Field.tpp:172) */
    FOR_IJ(dxo, dyo, { UPSAMPLE_BODY(float, fmul_, fadd_, _, out[idx] = val / weight) });
}
static void upsample_v(const v2 *in, unsigned dxi, unsigned dyi, v2 *out, unsigned dxo,
                       unsigned dyo) {
    if (dxo < dxi || dyo < dyi) raise_err("Error in Field<T>::upSample: dimensions");
    unsigned sizein = dxi * dyi;
    FOR_IJ(dxo, dyo, { UPSAMPLE_BODY(v2, vmul, vadd, _, out[idx] = vdiv(val, weight)) });
}

/* src/Motion.cpp:61-85 / 87-111: resample then rescale by the dimension ratio */
static void motion_upsample(const v2 *in, unsigned dxi, unsigned dyi, v2 *out, unsigned dxo,
                            unsigned dyo) {
    upsample_v(in, dxi, dyi, out, dxo, dyo);
    float rx = (float)dxo / (float)dxi, ry = (float)dyo / (float)dyi;
    unsigned n = dxo * dyo;
    for (unsigned i = 0; i < n; i++) {
        out[i].x *= rx;
        out[i].y *= ry;
    }
}
static void motion_downsample(const v2 *in, unsigned dxi, unsigned dyi, v2 *out, unsigned dxo,
                              unsigned dyo) {
    downsample_v(in, dxi, dyi, out, dxo, dyo);
    float rx = (float)dxo / (float)dxi, ry = (float)dyo / (float)dyi;
    unsigned n = dxo * dyo;
    for (unsigned i = 0; i < n; i++) {
        out[i].x *= rx;
        out[i].y *= ry;
    }
}

/* src/Image.cpp:119-182: pull-back bilinear warp; out-of-range keeps the pixel */
static void warp2d(float *I, const v2 *u, unsigned dx, unsigned dy) {
    unsigned n = dx * dy;
    float *tmp = (float *)malloc(n * sizeof(float));
    memcpy(tmp, I, n * sizeof(float));
    FOR_IJ(dx, dy, {
        float px = (float)(int)i + u[idx].x;
        int ddx = (int)floorf(px);
        float fxx = px - (float)ddx;
        float py = (float)(int)j + u[idx].y;
        int ddy = (int)floorf(py);
        float fyy = py - (float)ddy;
        if (ddx < 0 || (unsigned)ddx >= dx || ddy < 0 || (unsigned)ddy >= dy) continue;
        int idxO = ddx + ddy * (int)dx;
        float val = tmp[idxO] * (1 - fxx) * (1 - fyy);
        float weight = (1 - fxx) * (1 - fyy);
        if ((unsigned)ddx < dx - 1) {
            val += tmp[idxO + 1] * fxx * (1 - fyy);
            weight += fxx * (1 - fyy);
        }
        if ((unsigned)ddy < dy - 1) {
            val += tmp[idxO + (int)dx] * (1 - fxx) * fyy;
            weight += (1 - fxx) * fyy;
        }
        if ((unsigned)ddx < dx - 1 && (unsigned)ddy < dy - 1) {
            val += tmp[idxO + 1 + (int)dx] * fxx * fyy;
            weight += fxx * fyy;
        }
        if (weight != 0) I[idx] = val / weight;
    });
    free(tmp);
}
void oracle_warp2d(float *I, const float *u, int dimx, int dimy) {
    warp2d(I, (const v2 *)u, (unsigned)dimx, (unsigned)dimy);
}

/* src/Motion.cpp:113-178: composition u(x) <- v(x) + u(x + v(x)) */
static void accumulate(v2 *u, const v2 *v, unsigned dx, unsigned dy) {
    unsigned n = dx * dy;
    v2 *tot = (v2 *)malloc(n * sizeof(v2));
    memcpy(tot, u, n * sizeof(v2));
    FOR_IJ(dx, dy, {
        float px = (float)i + v[idx].x;
        int ddx = (int)floorf(px);
        float fxx = px - (float)ddx;
        float py = (float)j + v[idx].y;
        int ddy = (int)floorf(py);
        float fyy = py - (float)ddy;
        if (ddx < 0 || (unsigned)ddx >= dx || ddy < 0 || (unsigned)ddy >= dy) continue;
        u[idx] = v[idx];
        int idxO = ddx + ddy * (int)dx;
        v2 val = vmul(vmul(tot[idxO], (1 - fxx)), (1 - fyy));
        float weight = (1 - fxx) * (1 - fyy);
        if ((unsigned)ddx < dx - 1) {
            val = vadd(val, vmul(vmul(tot[idxO + 1], fxx), (1 - fyy)));
            weight += fxx * (1 - fyy);
        }
        if ((unsigned)ddy < dy - 1) {
            val = vadd(val, vmul(vmul(tot[idxO + (int)dx], (1 - fxx)), fyy));
            weight += (1 - fxx) * fyy;
        }
        if ((unsigned)ddx < dx - 1 && (unsigned)ddy < dy - 1) {
            val = vadd(val, vmul(vmul(tot[idxO + 1 + (int)dx], fxx), fyy));
            weight += fxx * fyy;
        }
        if (weight != 0) u[idx] = vadd(u[idx], vdiv(val, weight));
    });
    free(tot);
}
void oracle_accumulate(float *u, const float *v, int dimx, int dimy) {
    accumulate((v2 *)u, (const v2 *)v, (unsigned)dimx, (unsigned)dimy);
}

/* src/Kernel.cpp:45-73: kw x kw Gaussian, expf in float, normalised in double */
void oracle_gaussian_kernel(int kw, float sigma, double *k) {
    int cx = (int)(((unsigned)kw - 1u) / 2u), cy = cx;
    double weight = 0;
    for (int i = 0; i < kw; i++)
        for (int j = 0; j < kw; j++) {
            int idx = i + j * kw;
            float num = (float)(-((i - cx) * (i - cx) + (j - cy) * (j - cy)));
            k[idx] = (double)expf(num / (2 * sigma * sigma));
            weight += k[idx];
        }
    for (int i = 0; i < kw * kw; i++) k[i] /= weight;
}

/* src/Field.tpp:208-269: taps valid iff the LINEAR index is in [0, N) */
static void convolute_v(v2 *f, unsigned dx, unsigned dy, const double *k, int kw) {
    unsigned n = dx * dy;
    int cx = (int)(((unsigned)kw - 1u) / 2u), cy = cx;
    v2 *tmp = (v2 *)malloc(n * sizeof(v2));
    memcpy(tmp, f, n * sizeof(v2));
    FOR_IJ(dx, dy, {
        v2 val = V(0.0f, 0.0f);
        double weight = 0.0f;
        for (int ii = -cx; ii <= cx; ii++)
            for (int jj = -cy; jj <= cy; jj++) {
                unsigned lin = (unsigned)((int)i + ii) + (unsigned)((int)j + jj) * dx;
                if (lin >= n) continue; /* negative wraps to a huge unsigned */
                int ik = (ii + cx) + (jj + cy) * kw;
                val = vadd(val, vmul(tmp[(int)idx + ii + jj * (int)dx], (float)k[ik]));
                weight += k[ik];
            }
        if (weight != 0) f[idx] = vdiv(val, (float)weight);
    });
    free(tmp);
}
static void convolute_f(float *f, unsigned dx, unsigned dy, const double *k, int kw) {
    unsigned n = dx * dy;
    int cx = (int)(((unsigned)kw - 1u) / 2u), cy = cx;
    float *tmp = (float *)malloc(n * sizeof(float));
    memcpy(tmp, f, n * sizeof(float));
    FOR_IJ(dx, dy, {
        float val = 0.0f; /* Field.tpp:240 leaves T val uninitialised for float */
        double weight = 0.0f;
        for (int ii = -cx; ii <= cx; ii++)
            for (int jj = -cy; jj <= cy; jj++) {
                unsigned lin = (unsigned)((int)i + ii) + (unsigned)((int)j + jj) * dx;
                if (lin >= n) continue;
                int ik = (ii + cx) + (jj + cy) * kw;
                /* float * double promotes: val += (double) product */
                val = (float)((double)val + (double)tmp[(int)idx + ii + jj * (int)dx] * k[ik]);
                weight += k[ik];
            }
        if (weight != 0) f[idx] = (float)((double)val / weight);
    });
    free(tmp);
}
void oracle_convolute_motion(float *u, int dimx, int dimy, const double *k, int kw) {
    convolute_v((v2 *)u, (unsigned)dimx, (unsigned)dimy, k, kw);
}
void oracle_convolute_image(float *I, int dimx, int dimy, const double *k, int kw) {
    convolute_f(I, (unsigned)dimx, (unsigned)dimy, k, kw);
}

void oracle_downsample_image(const float *in, int a, int b, float *out, int c, int d) {
    downsample_f(in, (unsigned)a, (unsigned)b, out, (unsigned)c, (unsigned)d);
}
void oracle_upsample_image(const float *in, int a, int b, float *out, int c, int d) {
    upsample_f(in, (unsigned)a, (unsigned)b, out, (unsigned)c, (unsigned)d);
}
void oracle_downsample_motion(const float *in, int a, int b, float *out, int c, int d) {
    motion_downsample((const v2 *)in, (unsigned)a, (unsigned)b, (v2 *)out, (unsigned)c,
                      (unsigned)d);
}
void oracle_upsample_motion(const float *in, int a, int b, float *out, int c, int d) {
    motion_upsample((const v2 *)in, (unsigned)a, (unsigned)b, (v2 *)out, (unsigned)c,
                    (unsigned)d);
}

/* src/Image.cpp:189-218 */
static void jacobian(const v2 *u, unsigned dx, unsigned dy, float *jac) {
    FOR_IJ(dx, dy, {
        v2 dudx = pdx_v(u, idx, i, dx);
        v2 dudy = pdy_v(u, idx, j, dx, dy);
        jac[idx] = (1.0f + dudx.x) * (1.0f + dudy.y) - dudx.y * dudy.x;
    });
}
void oracle_jacobian(const float *u, int dimx, int dimy, float *jac) {
    jacobian((const v2 *)u, (unsigned)dimx, (unsigned)dimy, jac);
}

/* src/Motion.cpp:253-277: scaling and squaring */
static void motion_exp(v2 *u, unsigned dx, unsigned dy) {
    unsigned n = dx * dy;
    float l = 1 + log2f(motion_maxabs(u, n));
    float c = ceilf(l);
    /* static_cast<int> of -inf/NaN is INT_MIN on x86-64 (cvttss2si) */
    int nsq = (c == c && c > -2147483648.0f && c < 2147483648.0f) ? (int)c : (int)0x80000000;
    if (nsq < 0) nsq = 0;
    if (nsq == 0) return;
    float scale = (float)pow(2, -nsq);
    for (unsigned i = 0; i < n; i++) {
        u[i].x *= scale;
        u[i].y *= scale;
    }
    v2 *tmp = (v2 *)malloc(n * sizeof(v2));
    for (int s = 0; s < nsq; s++) {
        memcpy(tmp, u, n * sizeof(v2));
        accumulate(u, tmp, dx, dy);
    }
    free(tmp);
}
void oracle_motion_exp(float *u, int dimx, int dimy) {
    motion_exp((v2 *)u, (unsigned)dimx, (unsigned)dimy);
}

/* ------------------------------------------------------------------ solvers */
/* src/regularization/IterativeSolver.cpp:22-56 */
static void spatial_derivative(const float *I, unsigned dx, unsigned dy, v2 *dI) {
    FOR_IJ(dx, dy, { dI[idx] = V(pdx_f(I, idx, i, dx), pdy_f(I, idx, j, dx, dy)); });
}
void oracle_spatial_derivative(const float *I, int dimx, int dimy, float *dI) {
    spatial_derivative(I, (unsigned)dimx, (unsigned)dimy, (v2 *)dI);
}
void oracle_temporal_derivative(const float *Iref, const float *Imov, int n, float *It) {
    for (int i = 0; i < n; i++) It[i] = Imov[i] - Iref[i];
}

/* src/regularization/OpticalFlow/OpticalFlow.cpp:15-39 */
static void get_force(v2 *f, const v2 *u, const v2 *dI, const float *It, unsigned n) {
    for (unsigned idx = 0; idx < n; idx++)
        f[idx] = vmul(dI[idx], It[idx] + u[idx].x * dI[idx].x + u[idx].y * dI[idx].y);
}
void oracle_get_force(const float *u, const float *dI, const float *It, int n, float *f) {
    get_force((v2 *)f, (const v2 *)u, (const v2 *)dI, It, (unsigned)n);
}

void oracle_qlaplacian(const float *u, int dimx, int dimy, float *q) {
    unsigned dx = (unsigned)dimx, dy = (unsigned)dimy;
    const v2 *U = (const v2 *)u;
    v2 *Q = (v2 *)q;
    FOR_IJ(dx, dy, { Q[idx] = qlap_v(U, idx, i, j, dx, dy); });
}

/* src/regularization/OpticalFlow/OpticalFlowDiffusion.cpp:19-84 */
static void hs_update(v2 *u, v2 *q, v2 *f, const v2 *dI, const float *It, unsigned dx,
                      unsigned dy, float alpha) {
    unsigned n = dx * dy;
    FOR_IJ(dx, dy, { q[idx] = qlap_v(u, idx, i, j, dx, dy); });
    get_force(f, q, dI, It, n);
    const float alphasq = alpha * alpha;
    FOR_IJ(dx, dy, {
        u[idx] = vsub(q[idx], vdiv(f[idx], alphasq + dI[idx].x * dI[idx].x +
                                               dI[idx].y * dI[idx].y));
    });
}

int oracle_hs_update(float *u, const float *dI, const float *It, int dimx, int dimy,
                     float alpha) {
    unsigned n = (unsigned)dimx * (unsigned)dimy;
    v2 *q = (v2 *)malloc(n * sizeof(v2)), *f = (v2 *)malloc(n * sizeof(v2));
    jmp_buf jb, *prev = g_jb;
    int rc = 0;
    g_jb = &jb;
    if (setjmp(jb) == 0)
        hs_update((v2 *)u, q, f, (const v2 *)dI, It, (unsigned)dimx, (unsigned)dimy, alpha);
    else
        rc = -1;
    g_jb = prev;
    free(q);
    free(f);
    return rc;
}

/* src/Logger.cpp:32-51 */
typedef struct {
    v2 *prev, *diff;
    unsigned n;
    int iter;
    float *error;
    int verbose;
} logger;

static void logger_init(logger *L, unsigned n, int niter, int verbose) {
    L->prev = (v2 *)calloc(n, sizeof(v2));
    L->diff = (v2 *)calloc(n, sizeof(v2));
    L->n = n;
    L->iter = 0;
    L->error = (float *)calloc((size_t)niter + 1, sizeof(float));
    L->verbose = verbose;
}
static void logger_free(logger *L) {
    free(L->prev);
    free(L->diff);
    free(L->error);
}
static void logger_update(logger *L, const v2 *u) {
    for (unsigned i = 0; i < L->n; i++) L->diff[i] = vsub(u[i], L->prev[i]);
    float prevnorm = motion_norm(L->prev, L->n);
    L->error[L->iter] = (prevnorm == 0 ? 0.0f : motion_norm(L->diff, L->n) / prevnorm);
    memcpy(L->prev, u, L->n * sizeof(v2));
    if (L->verbose) oprintf("Iteration: %d\tError:%.4f\n", L->iter, (double)L->error[L->iter]);
    L->iter++;
}
static float logger_err(const logger *L) { return L->error[L->iter - 1]; }

int oracle_hs_loop(float *u, const float *dI, const float *It, int dimx, int dimy, float alpha,
                   int niter, int fixed, float *errs) {
    unsigned n = (unsigned)dimx * (unsigned)dimy;
    v2 *q = (v2 *)malloc(n * sizeof(v2)), *f = (v2 *)malloc(n * sizeof(v2));
    logger L;
    logger_init(&L, n, niter, 0);
    jmp_buf jb, *prev = g_jb;
    int rc = 0, iter;
    g_jb = &jb;
    if (setjmp(jb) == 0) {
        for (iter = 0; iter < niter; iter++) {
            hs_update((v2 *)u, q, f, (const v2 *)dI, It, (unsigned)dimx, (unsigned)dimy, alpha);
            logger_update(&L, (const v2 *)u);
            if (errs) errs[iter] = logger_err(&L);
            if (!fixed && logger_err(&L) < 0.001f && iter > 1) {
                iter++;
                break;
            }
        }
        rc = iter;
    } else {
        rc = -1;
    }
    g_jb = prev;
    logger_free(&L);
    free(q);
    free(f);
    return rc;
}

/* The HS loop of oracle_hs_loop (fixed iterations) on `nthreads` OpenMP
 * threads, for bench.py's all-cores CPU baseline only.  The Jacobi update is
 * order independent (q is computed from the old u over the whole grid before u
 * is written, OpticalFlowDiffusion.cpp:43-55), so threads over j-lines give the
 * same u bit for bit (tests/test_oracle.py).  The Logger norms are summed per
 * thread in fp32 (the reference's sequential order within each thread's
 * j-lines) and combined in thread order: the errors round differently from the
 * single sequential sum, the motion does not depend on them. */
int oracle_hs_loop_mt(float *uf, const float *dIf, const float *It, int dimx, int dimy,
                      float alpha, int niter, int nthreads, float *errs) {
    const unsigned dx = (unsigned)dimx, dy = (unsigned)dimy, n = dx * dy;
    v2 *u = (v2 *)uf;
    const v2 *dI = (const v2 *)dIf;
    const int nt = nthreads > 0 ? nthreads : 1;
    v2 *q = (v2 *)malloc(n * sizeof(v2)), *prev = (v2 *)calloc(n, sizeof(v2));
    float *part = (float *)calloc(2 * (size_t)nt, sizeof(float));
    if (!q || !prev || !part) {
        free(q);
        free(prev);
        free(part);
        return -1;
    }
    const float alphasq = alpha * alpha;
    for (int it = 0; it < niter; it++) {
        /* slots of threads the runtime did not start stay 0 (OMP_DYNAMIC,
         * thread limits): every slot is reset per iteration */
        memset(part, 0, 2 * (size_t)nt * sizeof(float));
#pragma omp parallel num_threads(nt)
        {
#pragma omp for schedule(static)
            for (unsigned j = 0; j < dy; j++)
                for (unsigned i = 0; i < dx; i++) {
                    unsigned idx = i + j * dx;
                    q[idx] = qlap_v(u, idx, i, j, dx, dy);
                }
            float sd = 0.0f, sp = 0.0f;
#pragma omp for schedule(static)
            for (unsigned j = 0; j < dy; j++)
                for (unsigned i = 0; i < dx; i++) {
                    unsigned idx = i + j * dx;
                    v2 f = vmul(dI[idx], It[idx] + q[idx].x * dI[idx].x + q[idx].y * dI[idx].y);
                    u[idx] = vsub(q[idx], vdiv(f, alphasq + dI[idx].x * dI[idx].x +
                                                      dI[idx].y * dI[idx].y));
                    v2 d = vsub(u[idx], prev[idx]);
                    double px = prev[idx].x, py = prev[idx].y, ex = d.x, ey = d.y;
                    sp = (float)((double)sp + sqrt(px * px + py * py));
                    sd = (float)((double)sd + sqrt(ex * ex + ey * ey));
                    prev[idx] = u[idx];
                }
#ifdef _OPENMP
            extern int omp_get_thread_num(void);
            const int t = omp_get_thread_num();
#else
            const int t = 0;
#endif
            part[2 * t] = sd;
            part[2 * t + 1] = sp;
        }
        float sd = 0.0f, sp = 0.0f;
        for (int t = 0; t < nt; t++) {
            sd += part[2 * t];
            sp += part[2 * t + 1];
        }
        if (errs) errs[it] = (sp == 0.0f) ? 0.0f : (sd / (float)n) / (sp / (float)n);
    }
    free(q);
    free(prev);
    free(part);
    return niter;
}

/* src/regularization/Demons/Demons.cpp:34-63 */
static void demons_force(v2 *c, const v2 *dI, const float *It, unsigned n, float sigma_i,
                         float sigma_x) {
    const float sigma_xsq = sigma_x * sigma_x;
    const float sigma_isq = sigma_i * sigma_i;
    for (unsigned idx = 0; idx < n; idx++) {
        float den = dI[idx].x * dI[idx].x + dI[idx].y * dI[idx].y +
                    It[idx] * It[idx] * sigma_isq / sigma_xsq;
        c[idx] = vmul(vdiv(vmul(dI[idx], It[idx]), den), -1.0f);
    }
}
int oracle_demons_force(const float *dI, const float *It, int n, float sigma_i, float sigma_x,
                        float *c) {
    jmp_buf jb, *prev = g_jb;
    int rc = 0;
    g_jb = &jb;
    if (setjmp(jb) == 0)
        demons_force((v2 *)c, (const v2 *)dI, It, (unsigned)n, sigma_i, sigma_x);
    else
        rc = -1;
    g_jb = prev;
    return rc;
}

/* src/regularization/OpticalFlow/OpticalFlowFluid.cpp:7-41 (in place, i outer) */
static void sor_sweep(v2 *x, const v2 *b, unsigned dx, unsigned dy, float mu, float lambda,
                      float omega) {
    const unsigned sx = 1, sy = dx;
    if (dx < 3 || dy < 3) return;
    for (unsigned i = 1; i < dx - 1; i++)
        for (unsigned j = 1; j < dy - 1; j++) {
            unsigned idx = i * sx + j * sy;
            x[idx].x = (1.0f - omega) * x[idx].x +
                       omega / (-6 * mu - 2 * lambda) *
                           (b[idx].x -
                            mu * (x[idx + sx].x + x[idx - sx].x + x[idx + sy].x + x[idx - sy].x) -
                            (mu + lambda) * (x[idx + sx].x + x[idx - sx].x +
                                             0.25f * (x[idx + sx + sy].y - x[idx - sx + sy].y -
                                                      x[idx + sx - sy].y + x[idx - sx - sy].y)));
            x[idx].y = (1.0f - omega) * x[idx].y +
                       omega / (-6 * mu - 2 * lambda) *
                           (b[idx].y -
                            mu * (x[idx + sx].y + x[idx - sx].y + x[idx + sy].y + x[idx - sy].y) -
                            (mu + lambda) * (x[idx + sx].y + x[idx - sx].y +
                                             0.25f * (x[idx + sx + sy].x - x[idx - sx + sy].x -
                                                      x[idx + sx - sy].x + x[idx - sx - sy].x)));
        }
}
void oracle_sor_sweep(float *x, const float *b, int dimx, int dimy, float mu, float lambda,
                      float omega) {
    sor_sweep((v2 *)x, (const v2 *)b, (unsigned)dimx, (unsigned)dimy, mu, lambda, omega);
}

/* src/regularization/OpticalFlow/OpticalFlowFluid.cpp:60-90 */
static void fluid_increment(const v2 *mo, const v2 *vel, unsigned dx, unsigned dy, v2 *R) {
    FOR_IJ(dx, dy, {
        v2 v = vel[idx];
        v2 dudx = pdx_v(mo, idx, i, dx);
        v2 dudy = pdy_v(mo, idx, j, dx, dy);
        R[idx] = vsub(vsub(v, vmul(dudx, v.x)), vmul(dudy, v.y));
    });
}
void oracle_fluid_increment(const float *u, const float *v, int dimx, int dimy, float *R) {
    fluid_increment((const v2 *)u, (const v2 *)v, (unsigned)dimx, (unsigned)dimy, (v2 *)R);
}

/* ------------------------------------------------------------------ naive DCT
 * Curvature's FFTW plans (OpticalFlowCurvature.cpp:118-121) restated from the
 * published FFTW r2r definitions (FFTW 3.x manual, "1d Real-even DFTs"):
 *   REDFT10: Y_k = 2 sum_j X_j cos(pi (j+1/2) k / n)
 *   REDFT01: Y_k = X_0 + 2 sum_{j>=1} X_j cos(pi j (k+1/2) / n)
 * applied separably over a row-major n0 x n1 array.  Parity UNPINNED: FFTW's
 * fast algorithms round differently; no FFTW exists in this image. */
static void dct_axis(double *a, unsigned n0, unsigned n1, int axis, int kind) {
    unsigned n = axis ? n1 : n0, m = axis ? n0 : n1;
    double *col = (double *)malloc(n * sizeof(double)), *res = (double *)malloc(n * sizeof(double));
    for (unsigned t = 0; t < m; t++) {
        for (unsigned j = 0; j < n; j++) col[j] = axis ? a[t * n1 + j] : a[j * n1 + t];
        for (unsigned k = 0; k < n; k++) {
            double s = 0;
            if (kind == 10) {
                for (unsigned j = 0; j < n; j++)
                    s += 2.0 * col[j] * cos(M_PI * ((double)j + 0.5) * (double)k / (double)n);
            } else {
                s = col[0];
                for (unsigned j = 1; j < n; j++)
                    s += 2.0 * col[j] * cos(M_PI * (double)j * ((double)k + 0.5) / (double)n);
            }
            res[k] = s;
        }
        for (unsigned k = 0; k < n; k++) {
            if (axis)
                a[t * n1 + k] = res[k];
            else
                a[k * n1 + t] = res[k];
        }
    }
    free(col);
    free(res);
}

/* separable 2-D transform of a row-major n0 x n1 array, axis 1 then axis 0
 * (kind 10: REDFT10, kind 1: REDFT01), as Curvature applies it */
void oracle_dct2d(double *a, int n0, int n1, int kind) {
    dct_axis(a, (unsigned)n0, (unsigned)n1, 1, kind);
    dct_axis(a, (unsigned)n0, (unsigned)n1, 0, kind);
}

/* ------------------------------------------------------------------ registration */
enum { R_DIFFUSION = 0, R_CURVATURE, R_ELASTIC, R_THIRION, R_DIFFEO, R_FLUID };

typedef struct {
    int kind;
    unsigned dx, dy, n;
    v2 *gradI; /* IterativeSolver */
    float *It;
    v2 *force; /* OpticalFlow */
    v2 *qdiff; /* Diffusion */
    float alpha;
    float mu, lambda, omega; /* Elastic / Fluid */
    v2 *velocity, *increment;
    float timestep;
    float *Iwar; /* Demons */
    v2 *corr;
    float sigma_i, sigma_x, sigma_diff, sigma_fluid;
    int kw, accum;
    double *kdiff, *kfluid;
    double *rhs_x, *rhs_y, *eig; /* Curvature */
    float tau;
} solver;

struct oracle_reg {
    int nscales, nrefine, reg, verbose, fixed;
    int *niter;
    unsigned *dx, *dy;
    float **Iref, **Imov;
    v2 **motion;
    solver *sol;
    int *iters;
    int niters_log, niters_cap;
    float *last_err;
    int last_err_n;
};

static void solver_init(solver *s, int reg, unsigned dx, unsigned dy, const float *p,
                        unsigned np) {
    memset(s, 0, sizeof *s);
    s->kind = reg;
    s->dx = dx;
    s->dy = dy;
    s->n = dx * dy;
    unsigned n = s->n;
    s->gradI = (v2 *)calloc(n, sizeof(v2));
    s->It = (float *)calloc(n, sizeof(float));
    switch (reg) {
    case R_DIFFUSION: /* ImageRegistrationOpticalFlow.cpp:22-31 */
        s->force = (v2 *)calloc(n, sizeof(v2));
        s->qdiff = (v2 *)calloc(n, sizeof(v2));
        s->alpha = p[0];
        break;
    case R_CURVATURE: /* :32-48, OpticalFlowCurvature.cpp:6-30, 99-122 */
        s->force = (v2 *)calloc(n, sizeof(v2));
        s->alpha = p[0];
        s->tau = (np == 1) ? 1.0f : p[1];
        s->rhs_x = (double *)calloc(n, sizeof(double));
        s->rhs_y = (double *)calloc(n, sizeof(double));
        s->eig = (double *)calloc(n, sizeof(double));
        {
            const double PI_ = 3.14159265;
            for (unsigned pp = 0; pp < dx; pp++)
                for (unsigned q = 0; q < dy; q++) {
                    unsigned idx = pp * dy + q;
                    double lam = -4 + 2 * cos(pp * PI_ / dx) + 2 * cos(q * PI_ / dy);
                    s->eig[idx] = 1.0f / (1.0f + (double)(s->tau * s->alpha) * pow(lam, 2));
                }
        }
        break;
    case R_ELASTIC: /* :49-66 */
        s->force = (v2 *)calloc(n, sizeof(v2));
        s->mu = p[0];
        s->lambda = p[1];
        s->omega = (np != 3) ? 0.66f : p[2];
        break;
    case R_FLUID: /* ImageRegistrationFluid.cpp:17-34, OpticalFlowFluid.cpp:43-52 */
        s->force = (v2 *)calloc(n, sizeof(v2));
        s->mu = p[0];
        s->lambda = p[1];
        s->omega = (np != 3) ? (float)0.66 : p[2];
        s->velocity = (v2 *)calloc(n, sizeof(v2));
        s->increment = (v2 *)calloc(n, sizeof(v2));
        break;
    case R_THIRION:
    case R_DIFFEO: /* ImageRegistrationDemons.cpp:20-55, Demons.cpp:4-24 */
        s->sigma_i = p[0];
        s->sigma_x = p[1];
        s->sigma_diff = p[2];
        s->sigma_fluid = p[3];
        s->kw = (int)(unsigned)p[4];
        s->accum = (reg == R_THIRION) ? (int)p[5] : 0;
        s->Iwar = (float *)calloc(n, sizeof(float));
        s->corr = (v2 *)calloc(n, sizeof(v2));
        s->kdiff = (double *)calloc((size_t)s->kw * s->kw, sizeof(double));
        s->kfluid = (double *)calloc((size_t)s->kw * s->kw, sizeof(double));
        oracle_gaussian_kernel(s->kw, s->sigma_diff, s->kdiff);
        oracle_gaussian_kernel(s->kw, s->sigma_fluid, s->kfluid);
        break;
    }
}

static void solver_free(solver *s) {
    free(s->gradI);
    free(s->It);
    free(s->force);
    free(s->qdiff);
    free(s->velocity);
    free(s->increment);
    free(s->Iwar);
    free(s->corr);
    free(s->kdiff);
    free(s->kfluid);
    free(s->rhs_x);
    free(s->rhs_y);
    free(s->eig);
}

/* IterativeSolver::set_derivatives (IterativeSolver.cpp:53-56) */
static void set_derivatives(solver *s, const float *Iref, const float *Imov) {
    spatial_derivative(Imov, s->dx, s->dy, s->gradI);
    for (unsigned i = 0; i < s->n; i++) s->It[i] = Imov[i] - Iref[i];
}

static void get_update(solver *s, v2 *u, const float *Iref, const float *Imov) {
    unsigned dx = s->dx, dy = s->dy, n = s->n;
    switch (s->kind) {
    case R_DIFFUSION: /* OpticalFlowDiffusion.cpp:43-55 */
        hs_update(u, s->qdiff, s->force, s->gradI, s->It, dx, dy, s->alpha);
        break;
    case R_ELASTIC: /* OpticalFlowElastic.cpp:13-19 */
        get_force(s->force, u, s->gradI, s->It, n);
        sor_sweep(u, s->force, dx, dy, s->mu, s->lambda, s->omega);
        break;
    case R_FLUID: { /* OpticalFlowFluid.cpp:123-140 */
        get_force(s->force, u, s->gradI, s->It, n);
        sor_sweep(s->velocity, s->force, dx, dy, s->mu, s->lambda, s->omega);
        fluid_increment(u, s->velocity, dx, dy, s->increment);
        const float dumax = 0.65f;
        s->timestep = dumax / motion_maxabs(s->increment, n);
        oprintf("Dumax: %.3f\tMaxabs increment: %.3f\t Timestep: %.3f\n", (double)dumax,
                (double)motion_maxabs(s->increment, n), (double)s->timestep);
        if (s->timestep >= 65.0f) return;
        for (unsigned i = 0; i < n; i++) u[i] = vadd(u[i], vmul(s->increment[i], s->timestep));
        break;
    }
    case R_CURVATURE: { /* OpticalFlowCurvature.cpp:209-232 */
        get_force(s->force, u, s->gradI, s->It, n);
        for (unsigned i = 0; i < dx; i++)
            for (unsigned j = 0; j < dy; j++) {
                unsigned rm = i * dy + j, cm = i + j * dx;
                s->rhs_x[rm] = (double)(u[cm].x - s->tau * s->force[cm].x);
                s->rhs_y[rm] = (double)(u[cm].y - s->tau * s->force[cm].y);
            }
        dct_axis(s->rhs_x, dx, dy, 1, 10);
        dct_axis(s->rhs_x, dx, dy, 0, 10);
        dct_axis(s->rhs_y, dx, dy, 1, 10);
        dct_axis(s->rhs_y, dx, dy, 0, 10);
        for (unsigned i = 0; i < n; i++) {
            s->rhs_x[i] *= s->eig[i];
            s->rhs_y[i] *= s->eig[i];
        }
        dct_axis(s->rhs_x, dx, dy, 1, 1);
        dct_axis(s->rhs_x, dx, dy, 0, 1);
        dct_axis(s->rhs_y, dx, dy, 1, 1);
        dct_axis(s->rhs_y, dx, dy, 0, 1);
        for (unsigned i = 0; i < dx; i++)
            for (unsigned j = 0; j < dy; j++) {
                unsigned rm = i * dy + j, cm = i + j * dx;
                u[cm] = vdiv(V((float)s->rhs_x[rm], (float)s->rhs_y[rm]), 4.0f * (float)n);
            }
        break;
    }
    case R_THIRION:
    case R_DIFFEO: /* DemonsThirions.cpp:18-42, DemonsDiffeomorphic.cpp:15-35 */
        memcpy(s->Iwar, Imov, n * sizeof(float));
        warp2d(s->Iwar, u, dx, dy);
        set_derivatives(s, Iref, s->Iwar);
        demons_force(s->corr, s->gradI, s->It, n, s->sigma_i, s->sigma_x);
        convolute_v(s->corr, dx, dy, s->kfluid, s->kw);
        if (s->kind == R_DIFFEO) {
            motion_exp(s->corr, dx, dy);
            accumulate(u, s->corr, dx, dy);
        } else if (s->accum == 0) {
            accumulate(u, s->corr, dx, dy);
        } else if (s->accum == 1) {
            for (unsigned i = 0; i < n; i++) u[i] = vadd(u[i], s->corr[i]);
        }
        convolute_v(u, dx, dy, s->kdiff, s->kw);
        break;
    }
}

static void log_iters(oracle_reg *r, int it) {
    if (r->niters_log == r->niters_cap) {
        r->niters_cap = r->niters_cap ? 2 * r->niters_cap : 64;
        r->iters = (int *)realloc(r->iters, (size_t)r->niters_cap * sizeof(int));
    }
    r->iters[r->niters_log++] = it;
}

static void keep_errors(oracle_reg *r, const logger *L) {
    free(r->last_err);
    r->last_err_n = L->iter;
    r->last_err = (float *)malloc(((size_t)L->iter + 1) * sizeof(float));
    memcpy(r->last_err, L->error, (size_t)L->iter * sizeof(float));
}

/* ImageRegistration{OpticalFlow,Demons,Fluid}::estimate_motion_at_current_resolution */
static void estimate_level(oracle_reg *r, int s) {
    solver *S = &r->sol[s];
    unsigned dx = r->dx[s], dy = r->dy[s], n = dx * dy;
    int niter = r->niter[s];
    v2 *motion = r->motion[s];
    const float *Iref = r->Iref[s];
    const float *Imov = r->Imov[s];
    float *Iaux = (float *)calloc(n, sizeof(float));
    float *jac = (float *)calloc(n, sizeof(float));
    v2 *est = (v2 *)calloc(n, sizeof(v2));
    int demons = (r->reg == R_THIRION || r->reg == R_DIFFEO);
    int fluid = (r->reg == R_FLUID);
    for (int refine = 0; refine < r->nrefine; refine++) {
        memcpy(Iaux, Imov, n * sizeof(float));
        warp2d(Iaux, motion, dx, dy);
        logger L;
        logger_init(&L, n, niter, r->verbose);
        if (!demons) set_derivatives(S, Iref, Iaux);
        int iter, done = 0;
        for (iter = 0; iter < niter; iter++) {
            get_update(S, est, Iref, Iaux);
            logger_update(&L, est);
            if (!r->fixed && logger_err(&L) < 0.001f && iter > 1) {
                done = iter + 1;
                break;
            }
            if (fluid) { /* ImageRegistrationFluid.cpp:107-124 */
                jacobian(est, dx, dy, jac);
                if (image_min(jac, n) < 0.5) {
                    oprintf("Regridding on iteration: %d\tMin Jacobian: %.3f\n", iter,
                            (double)image_min(jac, n));
                    accumulate(motion, est, dx, dy);
                    memset(est, 0, n * sizeof(v2));
                    memcpy(Iaux, Imov, n * sizeof(float));
                    warp2d(Iaux, motion, dx, dy);
                    set_derivatives(S, Iref, Iaux);
                }
            }
        }
        if (!done) done = iter;
        log_iters(r, done);
        keep_errors(r, &L);
        logger_free(&L);
        accumulate(motion, est, dx, dy);
        memset(est, 0, n * sizeof(v2));
    }
    free(Iaux);
    free(jac);
    free(est);
}

/* ImageRegistration.cpp:6-47 (the rule is 71 printed '%', i.e. 142 in the literal) */
#define BANNER_RULE "%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%"
static void banner(oracle_reg *r, const float *p, unsigned np) {
    oprintf("%s\n", BANNER_RULE);
    oprintf("Optical flow image registration started... (2D C++ implementation)...\n");
    oprintf("Registration parameters:\n");
    oprintf("dimensions:\t\t\t\t(%d %d)\n", r->dx[0], r->dy[0]);
    oprintf("niter:\t\t\t\t\t(%d", r->niter[0]);
    for (int s = 1; s < r->nscales + 1; s++) oprintf(" %d", r->niter[s]);
    oprintf(")\n");
    oprintf("nscales:\t\t\t\t%d\n", r->nscales);
    oprintf("nrefine:\t\t\t\t%d\n", r->nrefine);
    switch (r->reg) {
    case 0: oprintf("regularisation:\t\t\t\tDiffusion\n"); break;
    case 1: oprintf("regularisation:\t\t\t\tCurvature\n"); break;
    case 2: oprintf("regularisation:\t\t\t\tElastic\n"); break;
    case 3: oprintf("regularisation:\t\t\t\tThirions Demons\n"); break;
    case 4: oprintf("regularisation:\t\t\t\tDiffeomorphic Demons\n"); break;
    case 5: oprintf("regularisation:\t\t\t\tFluid\n"); break;
    }
    if (np == 1) {
        oprintf("reg. param:\t\t\t\t%.2f\n", (double)p[0]);
    } else {
        oprintf("reg. params:\t\t\t\t(%.2f", (double)p[0]);
        for (unsigned q = 1; q < np; q++) oprintf(" %.2f", (double)p[q]);
        oprintf(")\n");
    }
    oprintf("%s\n\n", BANNER_RULE);
}

/* ImageRegistrationOpticalFlow.cpp:8-12, ImageRegistrationDemons.cpp:7-10,
 * ImageRegistrationFluid.cpp:5-7 */
static int valid_params(int reg, unsigned np) {
    switch (reg) {
    case R_DIFFUSION: return np == 1;
    case R_CURVATURE: return np >= 1 && np <= 2;
    case R_ELASTIC: return np >= 2 && np <= 3;
    case R_THIRION: return np == 6;
    case R_DIFFEO: return np == 5;
    case R_FLUID: return np >= 2 && np <= 3;
    }
    return 0;
}

static void reg_free(oracle_reg *r) {
    if (!r) return;
    for (int s = 0; s <= r->nscales; s++) {
        if (r->Iref) free(r->Iref[s]);
        if (r->Imov) free(r->Imov[s]);
        if (r->motion) free(r->motion[s]);
        if (r->sol && r->sol[s].n) solver_free(&r->sol[s]);
    }
    free(r->Iref);
    free(r->Imov);
    free(r->motion);
    free(r->sol);
    free(r->niter);
    free(r->dx);
    free(r->dy);
    free(r->iters);
    free(r->last_err);
    free(r);
}

int oracle_create(oracle_reg **out, int dimx, int dimy, const int *niter, int nscales, int reg,
                  const float *p, unsigned np, int nrefine, int verbose) {
    *out = NULL;
    if (reg < 0 || reg > 5) {
        snprintf(g_err, sizeof g_err, "Error: invalid regularisation given\n");
        return 1;
    }
    if (nscales < 0 || dimx <= 0 || dimy <= 0) {
        snprintf(g_err, sizeof g_err, "Error: invalid dimensions\n");
        return 1;
    }
    oracle_reg *r = (oracle_reg *)calloc(1, sizeof *r);
    r->nscales = nscales;
    r->nrefine = nrefine;
    r->reg = reg;
    r->verbose = verbose;
    r->niter = (int *)malloc((size_t)(nscales + 1) * sizeof(int));
    memcpy(r->niter, niter, (size_t)(nscales + 1) * sizeof(int));
    r->dx = (unsigned *)calloc((size_t)nscales + 1, sizeof(unsigned));
    r->dy = (unsigned *)calloc((size_t)nscales + 1, sizeof(unsigned));
    /* ImageRegistration.cpp:56-61: dim(dimin.x/scale, dimin.y/scale), float scale */
    for (int s = nscales; s >= 0; s--) {
        float scale = (float)pow(2, s);
        r->dx[s] = (unsigned)((float)(unsigned)dimx / scale);
        r->dy[s] = (unsigned)((float)(unsigned)dimy / scale);
    }
    r->Iref = (float **)calloc((size_t)nscales + 1, sizeof(float *));
    r->Imov = (float **)calloc((size_t)nscales + 1, sizeof(float *));
    r->motion = (v2 **)calloc((size_t)nscales + 1, sizeof(v2 *));
    for (int s = nscales; s >= 0; s--) {
        unsigned n = r->dx[s] * r->dy[s];
        r->Iref[s] = (float *)calloc(n ? n : 1, sizeof(float));
        r->Imov[s] = (float *)calloc(n ? n : 1, sizeof(float));
        r->motion[s] = (v2 *)calloc(n ? n : 1, sizeof(v2));
    }
    banner(r, p, np);
    if (!valid_params(reg, np)) {
        snprintf(g_err, sizeof g_err,
                 "Invalid number of regularisation parameters for given regularisation method.\n");
        r->sol = NULL;
        reg_free(r);
        return 1;
    }
    r->sol = (solver *)calloc((size_t)nscales + 1, sizeof(solver));
    for (int s = nscales; s >= 0; s--) solver_init(&r->sol[s], reg, r->dx[s], r->dy[s], p, np);
    *out = r;
    return 0;
}

void oracle_destroy(oracle_reg *r) { reg_free(r); }
void oracle_set_fixed_iters(oracle_reg *r, int on) { r->fixed = on; }

/* ImageRegistration.cpp:103-121 + Image::set_image (Image.cpp:15-29) */
int oracle_set_images(oracle_reg *r, const double *ref, const double *mov) {
    unsigned n0 = r->dx[0] * r->dy[0];
    jmp_buf jb, *prev = g_jb;
    int rc = 0;
    g_jb = &jb;
    if (setjmp(jb) == 0) {
        for (unsigned i = 0; i < n0; i++) r->Iref[0][i] = (float)ref[i];
        for (int s = r->nscales; s >= 1; s--)
            downsample_f(r->Iref[0], r->dx[0], r->dy[0], r->Iref[s], r->dx[s], r->dy[s]);
        for (unsigned i = 0; i < n0; i++) r->Imov[0][i] = (float)mov[i];
        for (int s = r->nscales; s >= 1; s--)
            downsample_f(r->Imov[0], r->dx[0], r->dy[0], r->Imov[s], r->dx[s], r->dy[s]);
    } else {
        rc = 2;
    }
    g_jb = prev;
    return rc;
}

/* ImageRegistration.cpp:133-156 */
int oracle_estimate(oracle_reg *r) {
    jmp_buf jb, *prev = g_jb;
    int rc = 0;
    g_jb = &jb;
    r->niters_log = 0;
    if (setjmp(jb) == 0) {
        for (int s = r->nscales; s >= 0; s--) {
            if (s > 0 && s < r->nscales)
                motion_downsample(r->motion[0], r->dx[0], r->dy[0], r->motion[s], r->dx[s],
                                  r->dy[s]);
            estimate_level(r, s);
            if (s > 0)
                motion_upsample(r->motion[s], r->dx[s], r->dy[s], r->motion[0], r->dx[0],
                                r->dy[0]);
        }
    } else {
        rc = 2;
    }
    g_jb = prev;
    return rc;
}

/* Motion::copy_motion_to_input (Motion.cpp:23-39): planar [x-plane; y-plane] */
int oracle_get_motion(oracle_reg *r, double *out) {
    unsigned n = r->dx[0] * r->dy[0];
    for (unsigned i = 0; i < n; i++) {
        out[i] = (double)r->motion[0][i].x;
        out[i + n] = (double)r->motion[0][i].y;
    }
    return 0;
}

/* WrapperOpticalFlow2d.cpp:120-137 */
int oracle_warp(oracle_reg *r, const double *mov, double *out) {
    unsigned n = r->dx[0] * r->dy[0];
    float *I = (float *)malloc(n * sizeof(float));
    for (unsigned i = 0; i < n; i++) I[i] = (float)mov[i];
    warp2d(I, r->motion[0], r->dx[0], r->dy[0]);
    for (unsigned i = 0; i < n; i++) out[i] = (double)I[i];
    free(I);
    return 0;
}

int oracle_iterations(const oracle_reg *r, int *out, int cap) {
    int n = r->niters_log < cap ? r->niters_log : cap;
    for (int i = 0; i < n; i++) out[i] = r->iters[i];
    return r->niters_log;
}

int oracle_last_errors(const oracle_reg *r, float *out, int cap) {
    int n = r->last_err_n < cap ? r->last_err_n : cap;
    for (int i = 0; i < n; i++) out[i] = r->last_err[i];
    return r->last_err_n;
}
