// field_kernels.hip — once-per-refine / once-per-level field primitives for
// gfx950: boundary conversions, pyramid resampling, bilinear warp, image
// gradients, motion composition.  Each restates one reference loop pixel for
// pixel in the same fp32 operation order (-ffp-contract=off), so results are
// bit-identical to the reference.  All are HBM-bound gathers/streams; one
// thread per pixel, 64-wide rows of the pitched layout per wave.
#include "of2d_device.h"

namespace of2d {

namespace {
constexpr int kBx = 64, kBy = 4;
inline dim3 grid2d(int dx, int dy) { return dim3((dx + kBx - 1) / kBx, (dy + kBy - 1) / kBy); }
#define OF2D_PX_PROLOGUE(DX, DY)                          \
    const int i = blockIdx.x * kBx + threadIdx.x;         \
    const int j = blockIdx.y * kBy + threadIdx.y;         \
    if (i >= (DX) || j >= (DY)) return;
}  // namespace

// ------------------------------------------------------------ boundary I/O
// Image::set_image (src/Image.cpp:15-29): (float) im[idx]
__global__ void d2f_kernel(const double *__restrict__ in, int dimx, int dimy,
                           float *__restrict__ out, int P) {
    OF2D_PX_PROLOGUE(dimx, dimy)
    out[(long)j * P + i] = (float)in[(long)j * dimx + i];
}
void launch_d2f(const double *in, int dimx, int dimy, float *out, int P, int row_offset,
                hipStream_t st) {
    (void)row_offset;
    hipLaunchKernelGGL(d2f_kernel, grid2d(dimx, dimy), dim3(kBx, kBy), 0, st, in, dimx, dimy,
                       out, P);
    OF2D_HIP(hipGetLastError());
}

// Image::copy_image_to_input (src/Image.cpp:36-50)
__global__ void f2d_kernel(const float *__restrict__ in, int P, int dimx, int dimy,
                           double *__restrict__ out) {
    OF2D_PX_PROLOGUE(dimx, dimy)
    out[(long)j * dimx + i] = (double)in[(long)j * P + i];
}
void launch_f2d(const float *in, int P, int dimx, int dimy, double *out, hipStream_t st) {
    hipLaunchKernelGGL(f2d_kernel, grid2d(dimx, dimy), dim3(kBx, kBy), 0, st, in, P, dimx, dimy,
                       out);
    OF2D_HIP(hipGetLastError());
}

// Motion::copy_motion_to_input (src/Motion.cpp:23-39): planar, x-plane first
__global__ void motion_to_planar_kernel(const float2 *__restrict__ m, int P, int dimx, int dimy,
                                        double *__restrict__ out) {
    OF2D_PX_PROLOGUE(dimx, dimy)
    const float2 v = m[(long)j * P + i];
    const long n = (long)dimx * dimy, k = (long)j * dimx + i;
    out[k] = (double)v.x;
    out[k + n] = (double)v.y;
}
void launch_motion_to_planar(const float2 *m, int P, int dimx, int dimy, double *out,
                             hipStream_t st) {
    hipLaunchKernelGGL(motion_to_planar_kernel, grid2d(dimx, dimy), dim3(kBx, kBy), 0, st, m, P,
                       dimx, dimy, out);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ pyramid
// Field<float>::downSample (src/Field.tpp:75-143): box average over the
// integer factor dimin/dimout, ii outer / jj inner, taps past the end skipped.
__global__ void downsample_image_kernel(const float *__restrict__ in, int dxi, int dyi, int Pi,
                                        float *__restrict__ out, int dxo, int dyo, int Po) {
    OF2D_PX_PROLOGUE(dxo, dyo)
    const int fx = dxi / dxo, fy = dyi / dyo;
    float val = 0.0f;
    int p = 0;
    for (int ii = 0; ii < fx; ii++)
        for (int jj = 0; jj < fy; jj++) {
            const int y = j * fy + jj;
            if (y >= dyi) continue;  // linear index >= sizein
            val += in[(long)y * Pi + i * fx + ii];
            p++;
        }
    if (p != 0) out[(long)j * Po + i] = val / (float)p;
}
void launch_downsample_image(const float *in, int dxi, int dyi, int Pi, float *out, int dxo,
                             int dyo, int Po, hipStream_t st) {
    if (dxo <= 0 || dyo <= 0 || dxo > dxi || dyo > dyi)
        throw std::invalid_argument(
            "Error in Image::downSample(const Image& im): Error in Field<T>::downSample(const "
            "FIeld<T>& fieldin): input has to have same dimensions as target\n");
    hipLaunchKernelGGL(downsample_image_kernel, grid2d(dxo, dyo), dim3(kBx, kBy), 0, st, in, dxi,
                       dyi, Pi, out, dxo, dyo, Po);
    OF2D_HIP(hipGetLastError());
}

// Motion::downSample (src/Motion.cpp:87-111): Field<vector2d>::downSample then
// every component scaled by dimout/dimin (float ratio).
__global__ void downsample_motion_kernel(const float2 *__restrict__ in, int dxi, int dyi, int Pi,
                                         float2 *__restrict__ out, int dxo, int dyo, int Po,
                                         float rx, float ry) {
    OF2D_PX_PROLOGUE(dxo, dyo)
    const int fx = dxi / dxo, fy = dyi / dyo;
    float vx = 0.0f, vy = 0.0f;
    int p = 0;
    for (int ii = 0; ii < fx; ii++)
        for (int jj = 0; jj < fy; jj++) {
            const int y = j * fy + jj;
            if (y >= dyi) continue;
            const float2 a = in[(long)y * Pi + i * fx + ii];
            vx = vx + a.x;
            vy = vy + a.y;
            p++;
        }
    float2 o = out[(long)j * Po + i];
    if (p != 0) o = make_float2(vx / (float)p, vy / (float)p);
    o.x *= rx;
    o.y *= ry;
    out[(long)j * Po + i] = o;
}
void launch_downsample_motion(const float2 *in, int dxi, int dyi, int Pi, float2 *out, int dxo,
                              int dyo, int Po, hipStream_t st) {
    if (dxo <= 0 || dyo <= 0 || dxo > dxi || dyo > dyi)
        throw std::invalid_argument(
            "Error in Motion::downSample(const Motion& im): Error in Field<T>::downSample(const "
            "FIeld<T>& fieldin): input has to have same dimensions as target\n");
    const float rx = (float)dxo / (float)dxi, ry = (float)dyo / (float)dyi;
    hipLaunchKernelGGL(downsample_motion_kernel, grid2d(dxo, dyo), dim3(kBx, kBy), 0, st, in, dxi,
                       dyi, Pi, out, dxo, dyo, Po, rx, ry);
    OF2D_HIP(hipGetLastError());
}

// Motion::upSample (src/Motion.cpp:61-85) = Field<vector2d>::upSample
// (src/Field.tpp:145-206, bilinear renormalised by the valid weight) then
// every component scaled by dimout/dimin.
__global__ void upsample_motion_kernel(const float2 *__restrict__ in, int dxi, int dyi, int Pi,
                                       float2 *__restrict__ out, int dxo, int dyo, int Po,
                                       float rx, float ry) {
    OF2D_PX_PROLOGUE(dxo, dyo)
    float2 o = out[(long)j * Po + i];
    const float px = (float)i * (float)dxi / (float)dxo;
    const int dx = (int)floorf(px);
    const float fx = px - (float)dx;
    const float py = (float)j * (float)dyi / (float)dyo;
    const int dy = (int)floorf(py);
    const float fy = py - (float)dy;
    const unsigned lin = (unsigned)dx + (unsigned)dy * (unsigned)dxi;
    if (lin < (unsigned)dxi * (unsigned)dyi) {
        const float2 *b = in + (long)dy * Pi + dx;
        float vx = (b[0].x * (1 - fx)) * (1 - fy);
        float vy = (b[0].y * (1 - fx)) * (1 - fy);
        float w = (1 - fx) * (1 - fy);
        const bool ax = (unsigned)dx < (unsigned)(dxi - 1);
        const bool ay = (unsigned)dy < (unsigned)(dyi - 1);
        if (ax) {
            vx = vx + (b[1].x * fx) * (1 - fy);
            vy = vy + (b[1].y * fx) * (1 - fy);
            w += fx * (1 - fy);
        }
        if (ay) {
            vx = vx + (b[Pi].x * (1 - fx)) * fy;
            vy = vy + (b[Pi].y * (1 - fx)) * fy;
            w += (1 - fx) * fy;
        }
        if (ax && ay) {
            vx = vx + (b[Pi + 1].x * fx) * fy;
            vy = vy + (b[Pi + 1].y * fx) * fy;
            w += fx * fy;
        }
        if (w != 0) o = make_float2(vx / w, vy / w);
    }
    o.x *= rx;
    o.y *= ry;
    out[(long)j * Po + i] = o;
}
void launch_upsample_motion(const float2 *in, int dxi, int dyi, int Pi, float2 *out, int dxo,
                            int dyo, int Po, hipStream_t st) {
    if (dxo < dxi || dyo < dyi)
        throw std::invalid_argument(
            "Error in Motion::upSample(const Motion& mo): Error in Field<T>::downSample(const "
            "FIeld<T>& fieldin): input has to have same dimensions as target\n");
    const float rx = (float)dxo / (float)dxi, ry = (float)dyo / (float)dyi;
    hipLaunchKernelGGL(upsample_motion_kernel, grid2d(dxo, dyo), dim3(kBx, kBy), 0, st, in, dxi,
                       dyi, Pi, out, dxo, dyo, Po, rx, ry);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ warp
// Image::warp2d (src/Image.cpp:119-182): pull-back bilinear sample of src at
// (i + u.x, j + u.y); out-of-range floor keeps the original pixel; at the
// right/top edge only in-range taps are used, renormalised by their weight.
//
// Branch-free: the taps are loaded unconditionally (an out-of-range tap
// pattern reads element 0; g[1], g[P], g[P+1] of an in-image pixel stay in the
// allocation: pitch padding and the zeroed ghost j-line below the last row)
// and the reference's conditional terms are selects.
__device__ __forceinline__ float warp_px(const float *__restrict__ src, float2 m, float own, int i,
                                         int j, int dimx, int dimy, int P) {
    const float px = (float)i + m.x;
    const int dx = (int)floorf(px);
    const float fx = px - (float)dx;
    const float py = (float)j + m.y;
    const int dy = (int)floorf(py);
    const float fy = py - (float)dy;
    const bool ok = !(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy);
    const bool ax = dx < dimx - 1, ay = dy < dimy - 1;
    const float *b = src + (ok ? ((unsigned)dy * (unsigned)P + (unsigned)dx) : 0u);
    const float t00 = b[0], t10 = b[1], t01 = b[P], t11 = b[P + 1];
    float val = (t00 * (1 - fx)) * (1 - fy);
    float w = (1 - fx) * (1 - fy);
    const float v10 = val + (t10 * fx) * (1 - fy), w10 = w + fx * (1 - fy);
    val = ax ? v10 : val;
    w = ax ? w10 : w;
    const float v01 = val + (t01 * (1 - fx)) * fy, w01 = w + (1 - fx) * fy;
    val = ay ? v01 : val;
    w = ay ? w01 : w;
    const float v11 = val + (t11 * fx) * fy, w11 = w + fx * fy;
    val = (ax && ay) ? v11 : val;
    w = (ax && ay) ? w11 : w;
    // val / w is val itself when w rounds to exactly 1 (demons_kernels.hip
    // warp_batch): divide only in the waves where some lane needs it
    float q = val;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(ok && w != 1.0f) != 0, 0)) q = val / w;
    return (ok && w != 0) ? q : own;
}
__global__ void warp_kernel(const float *__restrict__ src, const float2 *__restrict__ u,
                            float *__restrict__ dst, int dimx, int dimy, int P) {
    OF2D_PX_PROLOGUE(dimx, dimy)
    const long idx = (long)j * P + i;
    dst[idx] = warp_px(src, u[idx], src[idx], i, j, dimx, dimy, P);
}
void launch_warp(const float *src, const float2 *u, float *dst, int dimx, int dimy, int P,
                 hipStream_t st) {
    hipLaunchKernelGGL(warp_kernel, grid2d(dimx, dimy), dim3(kBx, kBy), 0, st, src, u, dst, dimx,
                       dimy, P);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ gradients
// IterativeSolver::set_derivatives (IterativeSolver.cpp:22-56):
//   dI = (partial_x, partial_y)(Iaux)  gradients.h:9-32 (central /2.0f,
//   one-sided on the borders); It = Iaux - Iref.
__global__ void gradients_kernel(const float *__restrict__ Iref, const float *__restrict__ Ia,
                                 float2 *__restrict__ dI, float *__restrict__ It, int dimx,
                                 int nrows, int P, int row0, int dimy) {
    OF2D_PX_PROLOGUE(dimx, nrows)
    const long idx = (long)j * P + i;
    const int jg = row0 + j;  // global j-line: border rule uses the global index
    float gx, gy;
    if (i == 0)
        gx = Ia[idx + 1] - Ia[idx];
    else if (i == dimx - 1)
        gx = Ia[idx] - Ia[idx - 1];
    else
        gx = (Ia[idx + 1] - Ia[idx - 1]) / 2.0f;
    if (jg == 0)
        gy = Ia[idx + P] - Ia[idx];
    else if (jg == dimy - 1)
        gy = Ia[idx] - Ia[idx - P];
    else
        gy = (Ia[idx + P] - Ia[idx - P]) / 2.0f;
    dI[idx] = make_float2(gx, gy);
    It[idx] = Ia[idx] - Iref[idx];
}
void launch_gradients_rows(const float *Iref, const float *Iaux, float2 *dI, float *It, int dimx,
                           int nrows, int P, int row0, int dimy, hipStream_t st) {
    hipLaunchKernelGGL(gradients_kernel, grid2d(dimx, nrows), dim3(kBx, kBy), 0, st, Iref, Iaux,
                       dI, It, dimx, nrows, P, row0, dimy);
    OF2D_HIP(hipGetLastError());
}
void launch_gradients(const float *Iref, const float *Iaux, float2 *dI, float *It, int dimx,
                      int dimy, int P, hipStream_t st) {
    launch_gradients_rows(Iref, Iaux, dI, It, dimx, dimy, P, 0, dimy, st);
}

// ------------------------------------------------------------ composition
// Motion::accumulate (src/Motion.cpp:113-178): u(x) <- v(x) + u_old(x + v(x))
// (bilinear, renormalised); out-of-range keeps u_old(x).
// Branch-free as warp_kernel.
__device__ __forceinline__ float2 accumulate_px(const float2 *__restrict__ mo, float2 c,
                                                float2 own, int i, int j, int dimx, int dimy,
                                                int P) {
    const float px = (float)i + c.x;
    const int dx = (int)floorf(px);
    const float fx = px - (float)dx;
    const float py = (float)j + c.y;
    const int dy = (int)floorf(py);
    const float fy = py - (float)dy;
    const bool ok = !(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy);
    const bool ax = dx < dimx - 1, ay = dy < dimy - 1, axy = ax && ay;
    const float2 *b = mo + (ok ? ((unsigned)dy * (unsigned)P + (unsigned)dx) : 0u);
    const float2 t00 = b[0], t10 = b[1], t01 = b[P], t11 = b[P + 1];
    float vx = (t00.x * (1 - fx)) * (1 - fy);
    float vy = (t00.y * (1 - fx)) * (1 - fy);
    float w = (1 - fx) * (1 - fy);
    const float x10 = vx + (t10.x * fx) * (1 - fy), y10 = vy + (t10.y * fx) * (1 - fy);
    const float w10 = w + fx * (1 - fy);
    vx = ax ? x10 : vx;
    vy = ax ? y10 : vy;
    w = ax ? w10 : w;
    const float x01 = vx + (t01.x * (1 - fx)) * fy, y01 = vy + (t01.y * (1 - fx)) * fy;
    const float w01 = w + (1 - fx) * fy;
    vx = ay ? x01 : vx;
    vy = ay ? y01 : vy;
    w = ay ? w01 : w;
    const float x11 = vx + (t11.x * fx) * fy, y11 = vy + (t11.y * fx) * fy;
    const float w11 = w + fx * fy;
    vx = axy ? x11 : vx;
    vy = axy ? y11 : vy;
    w = axy ? w11 : w;
    float2 q = make_float2(c.x + vx, c.y + vy);  // vx / 1.0f is vx
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(ok && w != 1.0f) != 0, 0))
        q = make_float2(c.x + vx / w, c.y + vy / w);
    return ok ? (w != 0 ? q : c) : own;
}
__global__ void accumulate_kernel(const float2 *__restrict__ mo, const float2 *__restrict__ v,
                                  float2 *__restrict__ mn, int dimx, int dimy, int P) {
    OF2D_PX_PROLOGUE(dimx, dimy)
    const long idx = (long)j * P + i;
    mn[idx] = accumulate_px(mo, v[idx], mo[idx], i, j, dimx, dimy, P);
}
void launch_accumulate(const float2 *m_old, const float2 *v, float2 *m_new, int dimx, int dimy,
                       int P, hipStream_t st) {
    hipLaunchKernelGGL(accumulate_kernel, grid2d(dimx, dimy), dim3(kBx, kBy), 0, st, m_old, v,
                       m_new, dimx, dimy, P);
    OF2D_HIP(hipGetLastError());
}

// Fluid regridding (ImageRegistrationFluid.cpp:108-124) in one pass: the
// motion accumulates the estimate (Motion::accumulate), the next estimate
// starts at zero (a second buffer: the Logger keeps the old one), and the
// moving image is warped by the new motion (Image::warp2d); per pixel the
// operations of accumulate_kernel then warp_kernel.
__global__ void regrid_kernel(const float2 *__restrict__ mo, const float2 *__restrict__ est,
                              float2 *__restrict__ est0, float2 *__restrict__ mn,
                              const float *__restrict__ Imov, float *__restrict__ Iaux, int dimx,
                              int dimy, int P) {
    OF2D_PX_PROLOGUE(dimx, dimy)
    const long idx = (long)j * P + i;
    const float2 m = accumulate_px(mo, est[idx], mo[idx], i, j, dimx, dimy, P);
    mn[idx] = m;
    est0[idx] = make_float2(0.0f, 0.0f);
    Iaux[idx] = warp_px(Imov, m, Imov[idx], i, j, dimx, dimy, P);
}
void launch_regrid(const float2 *m_old, const float2 *est, float2 *est0, float2 *m_new,
                   const float *Imov, float *Iaux, int dimx, int dimy, int P, hipStream_t st) {
    hipLaunchKernelGGL(regrid_kernel, grid2d(dimx, dimy), dim3(kBx, kBy), 0, st, m_old, est, est0,
                       m_new, Imov, Iaux, dimx, dimy, P);
    OF2D_HIP(hipGetLastError());
}

// The device-decided form (Registration::loop_fluid): the regrid runs only
// after an iteration whose report decided one (kFluidRegridWord), the motion
// fields are picked by the flipped index (the accumulated motion goes to
// motion[mcur]), and the estimate is not touched: the next iteration reads it
// as zero (fluid_zero_est) and as the Logger's prev.  Per pixel the operations
// of regrid_kernel.
__global__ void regrid_if_kernel(float2 *__restrict__ m0, float2 *__restrict__ m1,
                                 const float2 *__restrict__ est, const float *__restrict__ Imov,
                                 float *__restrict__ Iaux, int dimx, int dimy, int P,
                                 FluidCtl ctl) {
    if (fluid_stopped(ctl) || !fluid_zero_est(ctl)) return;
    const bool c1 = ctl.w[kFluidMcurWord] != 0u;
    const float2 *mo = c1 ? m0 : m1;
    float2 *mn = c1 ? m1 : m0;
    // kBx x kBy pixel blocks in a grid-stride loop (a capped grid: most
    // launches are no-ops)
    const int nbx = (dimx + kBx - 1) / kBx, nb = nbx * ((dimy + kBy - 1) / kBy);
    for (int t = blockIdx.x; t < nb; t += gridDim.x) {
        const int i = (t % nbx) * kBx + threadIdx.x, j = (t / nbx) * kBy + threadIdx.y;
        if (i >= dimx || j >= dimy) continue;
        const long idx = (long)j * P + i;
        const float2 m = accumulate_px(mo, est[idx], mo[idx], i, j, dimx, dimy, P);
        mn[idx] = m;
        Iaux[idx] = warp_px(Imov, m, Imov[idx], i, j, dimx, dimy, P);
    }
}
void launch_regrid_if(float2 *m0, float2 *m1, const float2 *est, const float *Imov, float *Iaux,
                      int dimx, int dimy, int P, hipStream_t st, FluidCtl ctl) {
    if (!ctl.w) throw std::invalid_argument("launch_regrid_if: control words");
    const dim3 g = grid2d(dimx, dimy);
    hipLaunchKernelGGL(regrid_if_kernel, dim3(std::min((int)(g.x * g.y), kCappedGrid)),
                       dim3(kBx, kBy), 0, st, m0, m1, est, Imov, Iaux, dimx, dimy, P, ctl);
    OF2D_HIP(hipGetLastError());
}

// Motion::accumulate of an estimate onto a ZERO motion field (the end of the
// single-level refine loop, ImageRegistrationOpticalFlow.cpp:138): the
// interpolated old motion is 0, so u = est + 0 where (x + est) is inside the
// global grid and u = 0 (the old value) where it falls outside.  Slab variant:
// rows [0, nrows) are global j-lines row0.. of a dimy-line grid.
__global__ void compose_zero_kernel(const float2 *__restrict__ v, float2 *__restrict__ out,
                                    int dimx, int nrows, int P, int row0, int dimy) {
    OF2D_PX_PROLOGUE(dimx, nrows)
    const long idx = (long)j * P + i;
    const float2 c = v[idx];
    const float px = (float)i + c.x;
    const int dx = (int)floorf(px);
    const float py = (float)(row0 + j) + c.y;
    const int dy = (int)floorf(py);
    float2 o = make_float2(0.0f, 0.0f);
    if (!(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy)) o = make_float2(c.x + 0.0f, c.y + 0.0f);
    out[idx] = o;
}
void launch_compose_zero(const float2 *v, float2 *out, int dimx, int nrows, int P, int row0,
                         int dimy, hipStream_t st) {
    hipLaunchKernelGGL(compose_zero_kernel, grid2d(dimx, nrows), dim3(kBx, kBy), 0, st, v, out,
                       dimx, nrows, P, row0, dimy);
    OF2D_HIP(hipGetLastError());
}

// Field<vector2d>::operator+= (src/Field.tpp:272-287): additive Demons update
__global__ void add_motion_kernel(const float2 *__restrict__ a, const float2 *__restrict__ b,
                                  float2 *__restrict__ o, int dimx, int dimy, int P) {
    OF2D_PX_PROLOGUE(dimx, dimy)
    const long idx = (long)j * P + i;
    const float2 x = a[idx], y = b[idx];
    o[idx] = make_float2(x.x + y.x, x.y + y.y);
}
void launch_add_motion(const float2 *a, const float2 *b, float2 *out, int dimx, int dimy, int P,
                       hipStream_t st) {
    hipLaunchKernelGGL(add_motion_kernel, grid2d(dimx, dimy), dim3(kBx, kBy), 0, st, a, b, out,
                       dimx, dimy, P);
    OF2D_HIP(hipGetLastError());
}

}  // namespace of2d
