// demons_kernels.hip — Thirion's / diffeomorphic Demons iteration for gfx950.
//
// DemonsThirions::get_update (src/regularization/Demons/DemonsThirions.cpp:18-42),
// per iteration, in three passes over HBM:
//   K1 demons_force_kernel   Iwar = warp2d(Imov, u) at the pixel and its four
//                            neighbours (Image.cpp:119-182), dI = grad(Iwar),
//                            It = Iwar - Iref (IterativeSolver.cpp:22-56),
//                            c = -dI*It / (|dI|^2 + It^2 si^2/sx^2) (Demons.cpp:34-63)
//                            -> corr.  24 B/px + gathers.
//   K2 smooth_compose_kernel corr <- corr (*) G(sigma_fluid)   (Field.tpp:209-269)
//                            then u_mid = accumulate(u, corr)  (Motion.cpp:113-178)
//                            or u + corr (Addition) -> u_mid.  24 B/px + gathers.
//   K3 smooth_norm_kernel    u_new = u_mid (*) G(sigma_diffusion) plus the
//                            Logger partials against u (prev).  24 B/px.
// The Gaussian smoothing is the reference's DIRECT kw x kw convolution, staged
// through LDS, with its exact semantics: a tap is valid iff its LINEAR index
// lies in [0, N) (so taps past an x-edge wrap into the neighbouring j-line),
// the sum runs ii (x) outer / jj (y) inner in fp32 with (float) weights, and
// it is normalised by the fp64 sum of the valid weights cast to float.  A
// separable form cannot reproduce that rounding; the direct form is still
// HBM-bound at kw = 5 (25 LDS reads of 8 B per output pixel), so the exact
// form is the one shipped.
#include "of2d_device.h"

namespace of2d {

namespace {
constexpr int kCx = 64;  // conv tile: 64 px wide
constexpr int kCy = 16;  // 16 j-lines high (4 per thread row)
constexpr int kCThreadsY = 4;
static_assert(kCy / kCThreadsY == 4, "conv4 computes four j-lines per thread");

// warp2d value of Imov at pixel (a, b) with motion u (Image.cpp:137-174)
__device__ __forceinline__ float warped_at(const float *__restrict__ Imov,
                                           const float2 *__restrict__ u, int a, int b, int dimx,
                                           int dimy, int P) {
    const long idx = (long)b * P + a;
    const float2 m = u[idx];
    float out = Imov[idx];
    const float px = (float)a + m.x;
    const int dx = (int)floorf(px);
    const float fx = px - (float)dx;
    const float py = (float)b + m.y;
    const int dy = (int)floorf(py);
    const float fy = py - (float)dy;
    if (!(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy)) {
        const float *q = Imov + (long)dy * P + dx;
        float val = (q[0] * (1 - fx)) * (1 - fy);
        float w = (1 - fx) * (1 - fy);
        const bool ax = dx < dimx - 1, ay = dy < dimy - 1;
        if (ax) {
            val += (q[1] * fx) * (1 - fy);
            w += fx * (1 - fy);
        }
        if (ay) {
            val += (q[P] * (1 - fx)) * fy;
            w += (1 - fx) * fy;
        }
        if (ax && ay) {
            val += (q[P + 1] * fx) * fy;
            w += fx * fy;
        }
        if (w != 0) out = val / w;
    }
    return out;
}
}  // namespace

// Block: 64 x 4 threads, a 64 x kFy output tile (kFy/4 j-lines per thread).
// The warped image is computed ONCE per pixel of the tile plus a one-pixel
// halo into LDS (1.16 warps per output pixel instead of 5), then the central
// differences, It and the force come from LDS.
constexpr int kFy = 16;
__global__ __launch_bounds__(256) void demons_force_kernel(
    const float *__restrict__ Iref, const float *__restrict__ Imov, const float2 *__restrict__ u,
    float2 *__restrict__ corr, int dimx, int dimy, int P, float sigma_isq, float sigma_xsq,
    unsigned *__restrict__ status) {
    constexpr int TW = 64 + 2, TH = kFy + 2;
    __shared__ float w[TH][TW];
    const int x0 = blockIdx.x * 64, y0 = blockIdx.y * kFy;
    const int tid = threadIdx.y * 64 + threadIdx.x;
    // warp the tile + halo, all loads of a thread's slots issued together
    // (the same arithmetic as warped_at / Image.cpp:137-174)
    constexpr int NS = (TW * TH + 255) / 256;
    float2 m[NS];
    float own[NS];
    long idx[NS];
    bool in[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) {
        const int s = tid + 256 * q, r = s / TW, c = s - r * TW;
        const int a = x0 - 1 + c, b = y0 - 1 + r;
        in[q] = s < TW * TH && a >= 0 && a < dimx && b >= 0 && b < dimy;
        idx[q] = (long)b * P + a;
        m[q] = in[q] ? u[idx[q]] : make_float2(0.0f, 0.0f);
        own[q] = in[q] ? Imov[idx[q]] : 0.0f;
    }
    float t00[NS], t10[NS], t01[NS], t11[NS], fx[NS], fy[NS];
    bool ok[NS], ax[NS], ay[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) {
        const int s = tid + 256 * q, r = s / TW, c = s - r * TW;
        const int a = x0 - 1 + c, b = y0 - 1 + r;
        const float px = (float)a + m[q].x;
        const int dx = (int)floorf(px);
        fx[q] = px - (float)dx;
        const float py = (float)b + m[q].y;
        const int dy = (int)floorf(py);
        fy[q] = py - (float)dy;
        ok[q] = in[q] && !(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy);
        ax[q] = dx < dimx - 1;
        ay[q] = dy < dimy - 1;
        const float *g = Imov + (long)dy * P + dx;
        t00[q] = ok[q] ? g[0] : 0.0f;
        t10[q] = ok[q] && ax[q] ? g[1] : 0.0f;
        t01[q] = ok[q] && ay[q] ? g[P] : 0.0f;
        t11[q] = ok[q] && ax[q] && ay[q] ? g[P + 1] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < NS; q++) {
        if (!in[q]) continue;
        const int s = tid + 256 * q, r = s / TW, c = s - r * TW;
        float out = own[q];
        if (ok[q]) {
            const float gx = fx[q], gy = fy[q];
            float val = (t00[q] * (1 - gx)) * (1 - gy);
            float wt = (1 - gx) * (1 - gy);
            if (ax[q]) {
                val += (t10[q] * gx) * (1 - gy);
                wt += gx * (1 - gy);
            }
            if (ay[q]) {
                val += (t01[q] * (1 - gx)) * gy;
                wt += (1 - gx) * gy;
            }
            if (ax[q] && ay[q]) {
                val += (t11[q] * gx) * gy;
                wt += gx * gy;
            }
            if (wt != 0) out = val / wt;
        }
        w[r][c] = out;
    }
    __syncthreads();
    const int i = x0 + threadIdx.x;
    if (i >= dimx) return;
    const int c = threadIdx.x + 1;
    bool zero = false;
    // the wave index is uniform (64-thread rows): scalar row arithmetic
    for (int rr = (int)__builtin_amdgcn_readfirstlane(threadIdx.y); rr < kFy; rr += 4) {
        const int j = y0 + rr;
        if (j >= dimy) break;
        const int r = rr + 1;
        const float w0 = w[r][c];
        float gx, gy;
        if (i == 0)
            gx = w[r][c + 1] - w0;
        else if (i == dimx - 1)
            gx = w0 - w[r][c - 1];
        else
            gx = (w[r][c + 1] - w[r][c - 1]) / 2.0f;
        if (j == 0)
            gy = w[r + 1][c] - w0;
        else if (j == dimy - 1)
            gy = w0 - w[r - 1][c];
        else
            gy = (w[r + 1][c] - w[r - 1][c]) / 2.0f;
        const long idx = (long)j * P + i;
        const float it = w0 - Iref[idx];
        // Demons.cpp:57: dI * It / (dI.x^2 + dI.y^2 + It*It*sigma_isq/sigma_xsq) * -1
        const float den = (gx * gx + gy * gy) + ((it * it) * sigma_isq) / sigma_xsq;
        zero |= den == 0.0f;
        corr[idx] = make_float2(((gx * it) / den) * -1.0f, ((gy * it) / den) * -1.0f);
    }
    if (zero) atomicOr(status, kStatusDivZero);
}

void launch_demons_force(const float *Iref, const float *Imov, const float2 *u, float2 *corr,
                         int dimx, int dimy, int P, float sigma_isq, float sigma_xsq,
                         unsigned *status, hipStream_t st) {
    hipLaunchKernelGGL(demons_force_kernel, dim3((dimx + 63) / 64, (dimy + kFy - 1) / kFy),
                       dim3(64, 4), 0, st, Iref, Imov, u, corr, dimx, dimy, P, sigma_isq,
                       sigma_xsq, status);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ convolution
// One LDS tile of (kCx + 2cx) x (kCy + 2cy) float2 addressed by LINEAR index:
// slot (r, c) holds field[L] with L = (y0 - cy + r) * dimx + (x0 - cx + c), the
// reference's idx + ii*step.x + jj*step.y (Field.tpp:254), zero where L is
// outside [0, N).
struct ConvArgs {
    const float *kf;   // (float) k[idxkernel], kw*kw, idx = (ii+cx) + (jj+cy)*kw
    const double *kd;  // k[idxkernel] as double (boundary weight sums)
    int kw, cx, cy;
    double wfull;  // sum of all weights in the reference's order (interior pixels)
};

template <int KW>
__device__ __forceinline__ void conv_load_tile(float2 *tile, const float2 *__restrict__ f,
                                               int dimx, int dimy, int P, int x0, int y0,
                                               int cx_rt, int cy_rt) {
    const int cx = KW > 0 ? (KW - 1) / 2 : cx_rt, cy = KW > 0 ? (KW - 1) / 2 : cy_rt;
    const int TW = kCx + 2 * cx, TH = kCy + 2 * cy;
    const long N = (long)dimx * dimy;
    const int tid = threadIdx.y * 64 + threadIdx.x;
    // slot (r, c) <- f[L], L = row * dimx + col with col within cx of [0, dimx):
    // the j-line of L is row - 1, row or row + 1 (no 64-bit division)
    auto fetch = [&](int s) {
        const int r = s / TW, c = s - r * TW;
        int row = y0 - cy + r, col = x0 - cx + c;
        while (col < 0) {  // once unless cx > dimx
            col += dimx;
            row -= 1;
        }
        while (col >= dimx) {
            col -= dimx;
            row += 1;
        }
        const long L = (long)row * dimx + col;
        return (L >= 0 && L < N) ? f[(long)row * P + col] : make_float2(0.0f, 0.0f);
    };
    if constexpr (KW > 0) {
        // compile-time tile: every load of the thread in flight at once
        constexpr int TWc = kCx + 2 * ((KW - 1) / 2), THc = kCy + 2 * ((KW - 1) / 2);
        constexpr int NS = (TWc * THc + 255) / 256;
        float2 v[NS];
#pragma unroll
        for (int q = 0; q < NS; q++) {
            const int s = tid + 256 * q;
            v[q] = s < TWc * THc ? fetch(s) : make_float2(0.0f, 0.0f);
        }
#pragma unroll
        for (int q = 0; q < NS; q++) {
            const int s = tid + 256 * q;
            if (s < TWc * THc) tile[s] = v[q];
        }
    } else {
        for (int s = tid; s < TW * TH; s += 256) tile[s] = fetch(s);
    }
}

// value of the reference's convolution at (i, j) from the LDS tile; returns
// false when the weight sum is 0 (then the reference leaves the pixel as is)
// KW > 0: kernel width known at compile time (taps unrolled, weights in
// scalar registers); KW == 0: runtime width.
template <int KW>
__device__ __forceinline__ bool conv_px(const float2 *tile, const ConvArgs &a, int i, int j,
                                        int tx, int ty, int dimx, long N, float2 &out) {
    const int kw = KW > 0 ? KW : a.kw;
    const int cx = KW > 0 ? (KW - 1) / 2 : a.cx, cy = KW > 0 ? (KW - 1) / 2 : a.cy;
    const int TW = kCx + 2 * cx;
    const long lin = (long)j * dimx + i;
    const bool interior = (lin - cx - (long)cy * dimx >= 0) && (lin + cx + (long)cy * dimx < N);
    float vx = 0.0f, vy = 0.0f;
    double weight = 0.0;
    if (interior) {
#pragma unroll
        for (int ii = -cx; ii <= cx; ii++)
#pragma unroll
            for (int jj = -cy; jj <= cy; jj++) {
                const float2 t = tile[(ty + cy + jj) * TW + (tx + cx + ii)];
                const float k = a.kf[(ii + cx) + (jj + cy) * kw];
                vx = vx + t.x * k;
                vy = vy + t.y * k;
            }
        weight = a.wfull;
    } else {
#pragma unroll
        for (int ii = -cx; ii <= cx; ii++)
#pragma unroll
            for (int jj = -cy; jj <= cy; jj++) {
                const unsigned L = (unsigned)(i + ii) + (unsigned)(j + jj) * (unsigned)dimx;
                if ((long)L >= N) continue;  // Field.tpp:245-247 (unsigned compare)
                const float2 t = tile[(ty + cy + jj) * TW + (tx + cx + ii)];
                const int ik = (ii + cx) + (jj + cy) * kw;
                vx = vx + t.x * a.kf[ik];
                vy = vy + t.y * a.kf[ik];
                weight += a.kd[ik];
            }
    }
    if (weight == 0) return false;
    const float wf = (float)weight;  // coord2d::operator/(const T&) with T = float
    out = make_float2(vx / wf, vy / wf);
    return true;
}

// The convolution at four consecutive j-lines j0..j0+3 of column i.  When the
// width is known and all four pixels are interior, the 4 + 2c tile values of
// each tap column are read once and shared by the four outputs (each output
// still sums ii outer / jj inner, the reference's order); otherwise per pixel.
template <int KW>
__device__ __forceinline__ void conv4(const float2 *tile, const ConvArgs &a, int i, int j0,
                                      int tx, int ty0, int dimx, int dimy, long N, float2 res[4],
                                      bool has[4]) {
    if constexpr (KW > 0) {
        constexpr int c = (KW - 1) / 2, TW = kCx + 2 * c;
        const long lin0 = (long)j0 * dimx + i, lin3 = (long)(j0 + 3) * dimx + i;
        if (j0 + 3 < dimy && lin0 - c - (long)c * dimx >= 0 && lin3 + c + (long)c * dimx < N) {
            float vx[4] = {0.0f, 0.0f, 0.0f, 0.0f}, vy[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int ii = -c; ii <= c; ii++) {
                float2 col[4 + 2 * c];
#pragma unroll
                for (int q = 0; q < 4 + 2 * c; q++) col[q] = tile[(ty0 + q) * TW + (tx + c + ii)];
#pragma unroll
                for (int k = 0; k < 4; k++)
#pragma unroll
                    for (int jj = -c; jj <= c; jj++) {
                        const float kk = a.kf[(ii + c) + (jj + c) * KW];
                        vx[k] = vx[k] + col[k + c + jj].x * kk;
                        vy[k] = vy[k] + col[k + c + jj].y * kk;
                    }
            }
            const float wf = (float)a.wfull;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                has[k] = a.wfull != 0;
                res[k] = make_float2(vx[k] / wf, vy[k] / wf);
            }
            return;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        has[k] = false;
        if (j0 + k < dimy) has[k] = conv_px<KW>(tile, a, i, j0 + k, tx, ty0 + k, dimx, N, res[k]);
    }
}

// mode 0: Composition (Motion::accumulate), 1: Addition (Field::operator+=),
// 2: neither (DemonsThirions.cpp:33-38 with another value), 3: store corr only
template <int KW>
__global__ __launch_bounds__(256) void smooth_compose_kernel(
    const float2 *__restrict__ corr, const float2 *__restrict__ u, float2 *__restrict__ out,
    int dimx, int dimy, int P, ConvArgs a, int mode) {
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    const int x0 = blockIdx.x * kCx, y0 = blockIdx.y * kCy;
    conv_load_tile<KW>(tile, corr, dimx, dimy, P, x0, y0, a.cx, a.cy);
    __syncthreads();
    const long N = (long)dimx * dimy;
    const int i = x0 + threadIdx.x;
    if (i >= dimx) return;
    // four consecutive j-lines per thread; the wave index is uniform
    const int r0 = (int)__builtin_amdgcn_readfirstlane(threadIdx.y) * (kCy / kCThreadsY);
    float2 sm[4];
    bool has[4];
    conv4<KW>(tile, a, i, y0 + r0, threadIdx.x, r0, dimx, dimy, N, sm, has);
    float2 cv[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int j = y0 + r0 + k;
        cv[k] = make_float2(0.0f, 0.0f);
        if (j < dimy) cv[k] = has[k] ? sm[k] : corr[(long)j * P + i];
    }
    if (mode == 0) {
        // Motion::accumulate (Motion.cpp:113-178): u(x) <- c(x) + u_old(x + c(x)),
        // bilinear with in-range taps renormalised; out of range keeps u_old(x).
        // All gathers of the four pixels are issued before any is used.
        float2 own[4], t00[4], t10[4], t01[4], t11[4];
        float fx[4], fy[4];
        bool ok[4], ax[4], ay[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int j = y0 + r0 + k;
            const bool in = j < dimy;
            own[k] = in ? u[(long)j * P + i] : make_float2(0.0f, 0.0f);
            const float px = (float)i + cv[k].x;
            const int dx = (int)floorf(px);
            fx[k] = px - (float)dx;
            const float py = (float)j + cv[k].y;
            const int dy = (int)floorf(py);
            fy[k] = py - (float)dy;
            ok[k] = in && !(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy);
            ax[k] = dx < dimx - 1;
            ay[k] = dy < dimy - 1;
            const float2 *b = u + (long)dy * P + dx;
            const float2 z = make_float2(0.0f, 0.0f);
            t00[k] = ok[k] ? b[0] : z;
            t10[k] = ok[k] && ax[k] ? b[1] : z;
            t01[k] = ok[k] && ay[k] ? b[P] : z;
            t11[k] = ok[k] && ax[k] && ay[k] ? b[P + 1] : z;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int j = y0 + r0 + k;
            if (j >= dimy) break;
            const float2 c = cv[k];
            float2 o = own[k];
            if (ok[k]) {
                o = c;
                const float gx = fx[k], gy = fy[k];
                float vx = (t00[k].x * (1 - gx)) * (1 - gy);
                float vy = (t00[k].y * (1 - gx)) * (1 - gy);
                float w = (1 - gx) * (1 - gy);
                if (ax[k]) {
                    vx = vx + (t10[k].x * gx) * (1 - gy);
                    vy = vy + (t10[k].y * gx) * (1 - gy);
                    w += gx * (1 - gy);
                }
                if (ay[k]) {
                    vx = vx + (t01[k].x * (1 - gx)) * gy;
                    vy = vy + (t01[k].y * (1 - gx)) * gy;
                    w += (1 - gx) * gy;
                }
                if (ax[k] && ay[k]) {
                    vx = vx + (t11[k].x * gx) * gy;
                    vy = vy + (t11[k].y * gx) * gy;
                    w += gx * gy;
                }
                if (w != 0) o = make_float2(c.x + vx / w, c.y + vy / w);
            }
            out[(long)j * P + i] = o;
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int j = y0 + r0 + k;
        if (j >= dimy) break;
        const long idx = (long)j * P + i;
        const float2 c = cv[k];
        float2 o;
        if (mode == 3) {
            o = c;
        } else if (mode == 1) {
            const float2 m = u[idx];
            o = make_float2(m.x + c.x, m.y + c.y);
        } else {
            o = u[idx];
        }
        out[idx] = o;
    }
}

// u_new = u_mid (*) G(sigma_diffusion); Logger partials sum ||u_new - prev||,
// sum ||prev|| per block (fixed order)
template <int KW>
__global__ __launch_bounds__(256) void smooth_norm_kernel(const float2 *__restrict__ umid,
                                                          const float2 *__restrict__ prev,
                                                          float2 *__restrict__ out, int dimx,
                                                          int dimy, int P, ConvArgs a,
                                                          double *__restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    const int x0 = blockIdx.x * kCx, y0 = blockIdx.y * kCy;
    conv_load_tile<KW>(tile, umid, dimx, dimy, P, x0, y0, a.cx, a.cy);
    __syncthreads();
    const long N = (long)dimx * dimy;
    const int i = x0 + threadIdx.x;
    double sd = 0.0, sp = 0.0;
    if (i < dimx) {
        const int r0 = (int)__builtin_amdgcn_readfirstlane(threadIdx.y) * (kCy / kCThreadsY);
        float2 sm[4];
        bool has[4];
        conv4<KW>(tile, a, i, y0 + r0, threadIdx.x, r0, dimx, dimy, N, sm, has);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int j = y0 + r0 + k;
            if (j >= dimy) break;
            const long idx = (long)j * P + i;
            const float2 v = has[k] ? sm[k] : umid[idx];
            out[idx] = v;
            const float2 pv = prev[idx];
            const float ex = v.x - pv.x, ey = v.y - pv.y;
            sd += (double)__builtin_sqrtf(ex * ex + ey * ey);
            sp += (double)__builtin_sqrtf(pv.x * pv.x + pv.y * pv.y);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        sd += __shfl_down(sd, off);
        sp += __shfl_down(sp, off);
    }
    __shared__ double red[2][4];
    if (threadIdx.x == 0) {
        red[0][threadIdx.y] = sd;
        red[1][threadIdx.y] = sp;
    }
    __syncthreads();
    if (threadIdx.x == 0 && threadIdx.y == 0) {
        const long blk = (long)blockIdx.y * gridDim.x + blockIdx.x;
        partial[2 * blk] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        partial[2 * blk + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}

inline size_t conv_lds_bytes(int cx, int cy) {
    return sizeof(float2) * (size_t)(kCx + 2 * cx) * (kCy + 2 * cy);
}
dim3 conv_grid(int dimx, int dimy) { return dim3((dimx + kCx - 1) / kCx, (dimy + kCy - 1) / kCy); }
int conv_nblocks(int dimx, int dimy) {
    const dim3 g = conv_grid(dimx, dimy);
    return int(g.x * g.y);
}

void launch_smooth_compose(const float2 *corr, const float2 *u, float2 *out, int dimx, int dimy,
                           int P, const float *kf, const double *kd, int kw, double wfull,
                           int mode, hipStream_t st) {
    const int c = (kw - 1) / 2;
    ConvArgs a{kf, kd, kw, c, c, wfull};
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, conv_grid(dimx, dimy), dim3(64, kCThreadsY),
                           conv_lds_bytes(c, c), st, corr, u, out, dimx, dimy, P, a, mode);
    };
    switch (kw) {
        case 3: go(smooth_compose_kernel<3>); break;
        case 5: go(smooth_compose_kernel<5>); break;
        case 7: go(smooth_compose_kernel<7>); break;
        default: go(smooth_compose_kernel<0>); break;
    }
    OF2D_HIP(hipGetLastError());
}

void launch_smooth_norm(const float2 *umid, const float2 *prev, float2 *out, int dimx, int dimy,
                        int P, const float *kf, const double *kd, int kw, double wfull,
                        double *partial, hipStream_t st) {
    const int c = (kw - 1) / 2;
    ConvArgs a{kf, kd, kw, c, c, wfull};
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, conv_grid(dimx, dimy), dim3(64, kCThreadsY),
                           conv_lds_bytes(c, c), st, umid, prev, out, dimx, dimy, P, a, partial);
    };
    switch (kw) {
        case 3: go(smooth_norm_kernel<3>); break;
        case 5: go(smooth_norm_kernel<5>); break;
        case 7: go(smooth_norm_kernel<7>); break;
        default: go(smooth_norm_kernel<0>); break;
    }
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ exp (diffeomorphic)
// Motion::maxabs (Motion.cpp:51-58, squares .y twice) -> per-block max of
// (float)(2*y^2) in float; the last reduction and the scaling-and-squaring
// count nsquares = max(0, (int)ceil(1 + log2(sqrt(max)))) (Motion.cpp:253-261)
// are done by one block of exp_prepare_kernel.
__global__ __launch_bounds__(256) void maxabs_partial_kernel(const float2 *__restrict__ f,
                                                             int dimx, int dimy, int P,
                                                             float *__restrict__ part) {
    float m = 0.0f;
    const long n = (long)dimx * dimy;
    for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < n; k += (long)gridDim.x * 256) {
        const long j = k / dimx, i = k - j * dimx;
        const double y = (double)f[j * P + i].y;
        const float s = (float)(y * y + y * y);
        m = (m < s) ? s : m;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_down(m, off);
        m = (m < o) ? o : m;
    }
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int w = 1; w < 4; w++) r = (r < red[w]) ? red[w] : r;
        part[blockIdx.x] = r;
    }
}

__global__ void exp_prepare_kernel(const float *__restrict__ part, int nparts,
                                   int *__restrict__ nsq_out, float *__restrict__ maxabs_out,
                                   int nsq_max, unsigned *__restrict__ status) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float m = 0.0f;
    for (int b = 0; b < nparts; b++) m = (m < part[b]) ? part[b] : m;
    const float ma = sqrtf(m);
    const float c = ceilf(1.0f + log2f(ma));
    int nsq = (c == c && c > -2147483648.0f && c < 2147483648.0f) ? (int)c : (int)0x80000000;
    if (nsq < 0) nsq = 0;
    if (nsq > nsq_max) atomicOr(status, kStatusExpBound);
    *nsq_out = nsq;
    *maxabs_out = ma;
}

// Field<vector2d>::operator*=(pow(2, -nsq)) when nsq > 0
__global__ void exp_scale_kernel(float2 *__restrict__ f, int dimx, int dimy, int P,
                                 const int *__restrict__ nsq) {
    const int n = *nsq;
    if (n == 0) return;
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    if (i >= dimx || j >= dimy) return;
    const float s = ldexpf(1.0f, -n);  // (float) std::pow(2, -nsquares), exact
    float2 v = f[(long)j * P + i];
    v.x *= s;
    v.y *= s;
    f[(long)j * P + i] = v;
}

// one squaring u <- u o u (Motion.cpp:268-272: Mtmp = *this; this->accumulate(*Mtmp)),
// active only while s < nsq; otherwise copies src to dst
__global__ void exp_square_kernel(const float2 *__restrict__ mo, float2 *__restrict__ mn,
                                  int dimx, int dimy, int P, const int *__restrict__ nsq, int s) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    if (i >= dimx || j >= dimy) return;
    const long idx = (long)j * P + i;
    const float2 c = mo[idx];
    if (s >= *nsq) {
        mn[idx] = c;
        return;
    }
    float2 out = c;
    const float px = (float)i + c.x;
    const int dx = (int)floorf(px);
    const float fx = px - (float)dx;
    const float py = (float)j + c.y;
    const int dy = (int)floorf(py);
    const float fy = py - (float)dy;
    if (!(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy)) {
        const float2 *b = mo + (long)dy * P + dx;
        float vx = (b[0].x * (1 - fx)) * (1 - fy);
        float vy = (b[0].y * (1 - fx)) * (1 - fy);
        float w = (1 - fx) * (1 - fy);
        const bool ax = dx < dimx - 1, ay = dy < dimy - 1;
        if (ax) {
            vx = vx + (b[1].x * fx) * (1 - fy);
            vy = vy + (b[1].y * fx) * (1 - fy);
            w += fx * (1 - fy);
        }
        if (ay) {
            vx = vx + (b[P].x * (1 - fx)) * fy;
            vy = vy + (b[P].y * (1 - fx)) * fy;
            w += (1 - fx) * fy;
        }
        if (ax && ay) {
            vx = vx + (b[P + 1].x * fx) * fy;
            vy = vy + (b[P + 1].y * fx) * fy;
            w += fx * fy;
        }
        if (w != 0) out = make_float2(c.x + vx / w, c.y + vy / w);
    }
    mn[idx] = out;
}

void launch_motion_exp(float2 *f, float2 *scratch, int dimx, int dimy, int P, int nsq_max,
                       float *d_part, int nparts, int *d_nsq, float *d_maxabs, unsigned *status,
                       float2 **result, hipStream_t st) {
    hipLaunchKernelGGL(maxabs_partial_kernel, dim3(nparts), dim3(256), 0, st, f, dimx, dimy, P,
                       d_part);
    hipLaunchKernelGGL(exp_prepare_kernel, dim3(1), dim3(64), 0, st, d_part, nparts, d_nsq,
                       d_maxabs, nsq_max, status);
    const dim3 g((dimx + 63) / 64, (dimy + 3) / 4), b(64, 4);
    hipLaunchKernelGGL(exp_scale_kernel, g, b, 0, st, f, dimx, dimy, P, d_nsq);
    float2 *src = f, *dst = scratch;
    for (int s = 0; s < nsq_max; s++) {
        hipLaunchKernelGGL(exp_square_kernel, g, b, 0, st, src, dst, dimx, dimy, P, d_nsq, s);
        std::swap(src, dst);
    }
    *result = src;
    OF2D_HIP(hipGetLastError());
}

}  // namespace of2d
