// demons_kernels.hip — Thirion's / diffeomorphic Demons iteration for gfx950.
//
// DemonsThirions::get_update (src/regularization/Demons/DemonsThirions.cpp:18-42)
// per iteration:
//   K1 force                 Iwar = warp2d(Imov, u) (Image.cpp:119-182),
//                            dI = grad(Iwar), It = Iwar - Iref
//                            (IterativeSolver.cpp:22-56),
//                            c = -dI*It / (|dI|^2 + It^2 si^2/sx^2) (Demons.cpp:34-63)
//   K2 smooth + update       c <- c (*) G(sigma_fluid)   (Field.tpp:209-269)
//                            then u_mid = accumulate(u, c) (Motion.cpp:113-178)
//                            or u + c (Addition)
//   K3 smooth_norm_kernel    u_new = u_mid (*) G(sigma_diffusion) plus the
//                            Logger partials against u (prev).  24 B/px.
// K1 + K2 run as ONE kernel (demons_fused_kernel) on every tile whose
// convolution taps stay inside the image's x range: the warped image and the
// correction of the tile plus its halo live only in LDS, so the pass reads u,
// Imov, Iref and writes u_mid (24 B/px) instead of 48 B/px through a corr
// field.  The edge tile columns, whose taps wrap into the neighbouring j-line,
// take the unfused force + smooth_compose kernels.
// The Gaussian smoothing is the reference's DIRECT kw x kw convolution with
// its exact semantics: a tap is valid iff its LINEAR index lies in [0, N) (so
// taps past an x-edge wrap into the neighbouring j-line), the sum runs ii (x)
// outer / jj (y) inner in fp32 with (float) weights, and it is normalised by
// the fp64 sum of the valid weights cast to float.  A separable form cannot
// reproduce that rounding, so the direct form is the one shipped; its x and y
// components are summed as one packed pair (v_pk_mul_f32 + v_pk_add_f32 round
// exactly like the scalar multiply and add).
#include "of2d_device.h"

#include <cmath>

namespace of2d {

namespace {
constexpr int kCx = 64;  // conv tile: 64 px wide
constexpr int kCThreadsY = 4;
// j-lines per thread of the product smoothing kernels (the tile is
// kCThreadsY * kCr j-lines high): a taller tile loads fewer halo rows per
// output and shares each LDS tap column between more outputs
// waves-per-SIMD floor of the fused kernel (tools/ A/B builds set it)
#ifndef OF2D_DEMONS_WPE
#define OF2D_DEMONS_FUSED_ATTR
#else
#define OF2D_DEMONS_FUSED_ATTR __attribute__((amdgpu_waves_per_eu(OF2D_DEMONS_WPE)))
#endif
#ifndef OF2D_DEMONS_CR
#define OF2D_DEMONS_CR 8
#endif
constexpr int kCr = OF2D_DEMONS_CR;
// warped slots per thread per gather batch of the fused kernel (tools/ A/B
// builds override it)
// warped slots per thread per gather batch of the fused kernel
#ifndef OF2D_DEMONS_BW
#define OF2D_DEMONS_BW 6
#endif
// fused kernel's output tile: OF2D_DEMONS_TX columns (threads across) x
// OF2D_DEMONS_TY thread rows of kCr j-lines (A/B builds: 128 x 4, 64 x 8)
#ifndef OF2D_DEMONS_TX
#define OF2D_DEMONS_TX 64
#endif
#ifndef OF2D_DEMONS_TY
#define OF2D_DEMONS_TY 4
#endif
typedef float v2f __attribute__((ext_vector_type(2)));

// warp2d values of Imov at B pixels (a[q], b[q]) with motion u
// (Image.cpp:137-174); in[q] = the pixel is valid and inside the image (res[q]
// is meaningful only then).  Every load of the batch is issued before any is
// used, and none is conditional: a slot outside the image, or a tap pattern
// outside it, reads element 0, and the taps g[1], g[P], g[P+1] of an in-image
// pixel stay inside the allocation (pitch padding and the zeroed ghost j-line
// below the last row, of2d_device.h); the reference's conditional terms are
// selects between the sums with and without the term, so no exec-mask branch
// is needed and every kept value is the reference's.
template <int B>
__device__ __forceinline__ void warp_batch(const float *__restrict__ Imov,
                                           const float2 *__restrict__ u, const int a[B],
                                           const int b[B], const bool valid[B], int dimx, int dimy,
                                           int P, float res[B], bool in[B]) {
    float2 m[B];
    float own[B];
#pragma unroll
    for (int q = 0; q < B; q++) {
        // bitwise, not short-circuit: no exec-mask branches around the loads
        in[q] = valid[q] & ((unsigned)a[q] < (unsigned)dimx) & ((unsigned)b[q] < (unsigned)dimy);
        const unsigned idx = in[q] ? ((unsigned)b[q] * (unsigned)P + (unsigned)a[q]) : 0u;
        m[q] = u[idx];
        own[q] = Imov[idx];
    }
    float t00[B], t10[B], t01[B], t11[B], fx[B], fy[B];
    bool ok[B], ax[B], ay[B];
#pragma unroll
    for (int q = 0; q < B; q++) {
        const float px = (float)a[q] + m[q].x;
        const int dx = (int)floorf(px);
        fx[q] = px - (float)dx;
        const float py = (float)b[q] + m[q].y;
        const int dy = (int)floorf(py);
        fy[q] = py - (float)dy;
        ok[q] = in[q] && !(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy);
        ax[q] = dx < dimx - 1;
        ay[q] = dy < dimy - 1;
        const float *g = Imov + (ok[q] ? ((unsigned)dy * (unsigned)P + (unsigned)dx) : 0u);
        t00[q] = g[0];
        t10[q] = g[1];
        t01[q] = g[P];
        t11[q] = g[P + 1];
    }
#pragma unroll
    for (int q = 0; q < B; q++) {
        const float gx = fx[q], gy = fy[q];
        float val = (t00[q] * (1 - gx)) * (1 - gy);
        float wt = (1 - gx) * (1 - gy);
        const float v10 = val + (t10[q] * gx) * (1 - gy), w10 = wt + gx * (1 - gy);
        val = ax[q] ? v10 : val;
        wt = ax[q] ? w10 : wt;
        const float v01 = val + (t01[q] * (1 - gx)) * gy, w01 = wt + (1 - gx) * gy;
        val = ay[q] ? v01 : val;
        wt = ay[q] ? w01 : wt;
        const bool axy = ax[q] && ay[q];
        const float v11 = val + (t11[q] * gx) * gy, w11 = wt + gx * gy;
        val = axy ? v11 : val;
        wt = axy ? w11 : wt;
        // val / wt is val itself when wt rounds to exactly 1 (an interior tap
        // pattern: 99.7 % of the lanes at 4096^2), so the division runs only
        // for the slot batches in which some lane of the wave needs it
        float r = val;
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(ok[q] && wt != 1.0f) != 0, 0)) r = val / wt;
        res[q] = (ok[q] && wt != 0) ? r : (in[q] ? own[q] : 0.0f);
    }
}

// Demons.cpp:57: dI * It / (dI.x^2 + dI.y^2 + It*It*sigma_isq/sigma_xsq) * -1
// SXP: sigma_xsq is a power of two 2^k (|k| <= 126; the default sigma_x = 0.25
// gives 2^-4) and `sxq` holds its reciprocal 2^-k: t * 2^-k and t / 2^k are the
// same exact value, correctly rounded by both (denormals preserved), so the
// multiply gives the division's bits.  Otherwise `sxq` is sigma_xsq.
template <bool SXP = false>
__device__ __forceinline__ float2 demons_corr(float gx, float gy, float it, float sigma_isq,
                                              float sxq, bool &zero) {
    const float t = (it * it) * sigma_isq;
    const float den = (gx * gx + gy * gy) + (SXP ? t * sxq : t / sxq);
    zero |= den == 0.0f;
    return make_float2(((gx * it) / den) * -1.0f, ((gy * it) / den) * -1.0f);
}

// x tile of a launch over a subset of the tile columns: block columns
// [0, ntl) are tiles [0, ntl), the others the last tiles of a gxt-tile row
__device__ __forceinline__ int tile_x(int ntl, int gxt) {
    const int b = (int)blockIdx.x;
    return b < ntl ? b : gxt - ((int)gridDim.x - b);
}

// d = 2^k with |k| <= 126: *r = 2^-k (exact, normal) and true
bool pow2_reciprocal(float d, float *r) {
    int e = 0;
    const float m = std::frexp(d, &e);  // d = m 2^e, m in [0.5, 1)
    if (m != 0.5f || e - 1 < -126 || e - 1 > 126) return false;
    *r = std::ldexp(1.0f, 1 - e);
    return true;
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
    unsigned *__restrict__ status, int ntl, int gxt) {
    constexpr int TW = 64 + 2, TH = kFy + 2;
    __shared__ float w[TH][TW];
    const int x0 = tile_x(ntl, gxt) * 64, y0 = blockIdx.y * kFy;
    const int tid = threadIdx.y * 64 + threadIdx.x;
    // warp the tile + halo (slots outside the image are never read)
    constexpr int NS = (TW * TH + 255) / 256;
    {
        int a[NS], b[NS];
        bool valid[NS], in[NS];
        float res[NS];
#pragma unroll
        for (int q = 0; q < NS; q++) {
            const int s = tid + 256 * q, r = s / TW;
            a[q] = x0 - 1 + (s - r * TW);
            b[q] = y0 - 1 + r;
            valid[q] = s < TW * TH;
        }
        warp_batch<NS>(Imov, u, a, b, valid, dimx, dimy, P, res, in);
#pragma unroll
        for (int q = 0; q < NS; q++) {
            const int s = tid + 256 * q, r = s / TW;
            if (in[q]) w[r][s - r * TW] = res[q];
        }
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
        corr[idx] = demons_corr(gx, gy, w0 - Iref[idx], sigma_isq, sigma_xsq, zero);
    }
    if (zero) atomicOr(status, kStatusDivZero);
}

void launch_demons_force(const float *Iref, const float *Imov, const float2 *u, float2 *corr,
                         int dimx, int dimy, int P, float sigma_isq, float sigma_xsq,
                         unsigned *status, hipStream_t st) {
    const int gx = (dimx + 63) / 64;
    hipLaunchKernelGGL(demons_force_kernel, dim3(gx, (dimy + kFy - 1) / kFy), dim3(64, 4), 0, st,
                       Iref, Imov, u, corr, dimx, dimy, P, sigma_isq, sigma_xsq, status, gx, gx);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ convolution
// One LDS tile of (kCx + 2cx) x (kCThreadsY * R + 2cy) float2 addressed by
// LINEAR index: slot (r, c) holds field[L] with L = (y0 - cy + r) * dimx +
// (x0 - cx + c), the reference's idx + ii*step.x + jj*step.y (Field.tpp:254),
// zero where L is outside [0, N).
struct ConvArgs {
    const float *kf;   // (float) k[idxkernel], kw*kw, idx = (ii+cx) + (jj+cy)*kw
    const double *kd;  // k[idxkernel] as double (boundary weight sums)
    int kw, cx, cy;
    double wfull;  // sum of all weights in the reference's order (interior pixels)
};

template <int KW, int R = kCr>
__device__ __forceinline__ void conv_load_tile(float2 *tile, const float2 *__restrict__ f,
                                               int dimx, int dimy, int P, int x0, int y0,
                                               int cx_rt, int cy_rt) {
    constexpr int CY = kCThreadsY * R;  // tile height without the halo
    const int cx = KW > 0 ? (KW - 1) / 2 : cx_rt, cy = KW > 0 ? (KW - 1) / 2 : cy_rt;
    const int TW = kCx + 2 * cx, TH = CY + 2 * cy;
    const long N = (long)dimx * dimy;
    const int tid = threadIdx.y * 64 + threadIdx.x;
    // x-interior tile (block-uniform): no tap column leaves [0, dimx), so L is
    // in [0, N) iff its j-line is
    const bool xin = x0 - cx >= 0 && x0 + kCx + cx <= dimx;
    // slot (r, c) <- f[L], L = row * dimx + col with col within cx of [0, dimx):
    // the j-line of L is row - 1, row or row + 1 (no 64-bit division)
    auto fetch = [&](int s) {
        const int r = s / TW, c = s - r * TW;
        int row = y0 - cy + r, col = x0 - cx + c;
        if (xin)
            return (unsigned)row < (unsigned)dimy ? f[(long)row * P + col]
                                                  : make_float2(0.0f, 0.0f);
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
        constexpr int TWc = kCx + 2 * ((KW - 1) / 2), THc = CY + 2 * ((KW - 1) / 2);
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
template <int KW, int TX = kCx>
__device__ __forceinline__ bool conv_px(const float2 *tile, const ConvArgs &a, int i, int j,
                                        int tx, int ty, int dimx, long N, float2 &out) {
    const int kw = KW > 0 ? KW : a.kw;
    const int cx = KW > 0 ? (KW - 1) / 2 : a.cx, cy = KW > 0 ? (KW - 1) / 2 : a.cy;
    const int TW = TX + 2 * cx;
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

// every tap of the R pixels (i, j0..j0+R-1) has its linear index in [0, N)
template <int KW, int R>
__device__ __forceinline__ bool conv_rows_interior(int i, int j0, int dimx, int dimy, long N) {
    constexpr int c = KW > 0 ? (KW - 1) / 2 : 0;
    const long lin0 = (long)j0 * dimx + i, linl = (long)(j0 + R - 1) * dimx + i;
    return j0 + R - 1 < dimy && lin0 - c - (long)c * dimx >= 0 && linl + c + (long)c * dimx < N;
}

// The convolution at R consecutive j-lines j0..j0+R-1 of column i.  When the
// width is known and all R pixels are interior, the R + 2c tile values of
// each tap column are read once and shared by the R outputs (each output
// still sums ii outer / jj inner, the reference's order), x and y as one
// packed pair (PK) or as two scalars; otherwise per pixel.
// W1: the interior weight sum (float)wfull is exactly 1 (a normalised kernel,
// the reference's set_gaussian / set_average), so acc / wf is acc itself
template <int KW, int R, bool PK, bool W1 = false, int TX = kCx>
__device__ __forceinline__ void convR(const float2 *tile, const ConvArgs &a, int i, int j0,
                                      int tx, int ty0, int dimx, int dimy, long N, float2 res[R],
                                      bool has[R]) {
    if constexpr (KW > 0) {
        constexpr int c = (KW - 1) / 2, TW = TX + 2 * c;
        if (conv_rows_interior<KW, R>(i, j0, dimx, dimy, N)) {
            v2f acc[R];
#pragma unroll
            for (int k = 0; k < R; k++) acc[k] = v2f{0.0f, 0.0f};
#pragma unroll
            for (int ii = -c; ii <= c; ii++) {
                v2f col[R + 2 * c];
#pragma unroll
                for (int q = 0; q < R + 2 * c; q++) {
                    const float2 t = tile[(ty0 + q) * TW + (tx + c + ii)];
                    col[q] = v2f{t.x, t.y};
                }
#pragma unroll
                for (int k = 0; k < R; k++)
#pragma unroll
                    for (int jj = -c; jj <= c; jj++) {
                        const float kk = a.kf[(ii + c) + (jj + c) * KW];
                        if constexpr (PK) {
                            acc[k] = acc[k] + col[k + c + jj] * v2f{kk, kk};
                        } else {
                            acc[k].x = acc[k].x + col[k + c + jj].x * kk;
                            acc[k].y = acc[k].y + col[k + c + jj].y * kk;
                        }
                    }
            }
            const float wf = (float)a.wfull;
#pragma unroll
            for (int k = 0; k < R; k++) {
                has[k] = W1 || a.wfull != 0;
                res[k] = W1 ? make_float2(acc[k].x, acc[k].y)
                            : make_float2(acc[k].x / wf, acc[k].y / wf);
            }
            return;
        }
    }
#pragma unroll
    for (int k = 0; k < R; k++) {
        has[k] = false;
        if (j0 + k < dimy)
            has[k] = conv_px<KW, TX>(tile, a, i, j0 + k, tx, ty0 + k, dimx, N, res[k]);
    }
}

// Motion::accumulate (Motion.cpp:113-178) at pixels (i, j0..j0+G-1) with
// increments cv: u(x) <- c(x) + u_old(x + c(x)), bilinear with in-range taps
// renormalised; out of range keeps u_old(x).  Every gather of the G pixels is
// issued before any is used; as in warp_batch, no load is conditional (an
// out-of-range tap pattern reads element 0) and the conditional terms are
// selects.
template <int G>
__device__ __forceinline__ void compose_px(const float2 *__restrict__ u, int i, int j0, int dimx,
                                           int dimy, int P, const float2 cv[G], float2 o[G]) {
    float2 own[G], t00[G], t10[G], t01[G], t11[G];
    float fx[G], fy[G];
    bool ok[G], ax[G], ay[G];
#pragma unroll
    for (int k = 0; k < G; k++) {
        const int j = j0 + k;
        const bool in = j < dimy;
        own[k] = u[in ? ((unsigned)j * (unsigned)P + (unsigned)i) : 0u];
        const float px = (float)i + cv[k].x;
        const int dx = (int)floorf(px);
        fx[k] = px - (float)dx;
        const float py = (float)j + cv[k].y;
        const int dy = (int)floorf(py);
        fy[k] = py - (float)dy;
        ok[k] = in && !(dx < 0 || dx >= dimx || dy < 0 || dy >= dimy);
        ax[k] = dx < dimx - 1;
        ay[k] = dy < dimy - 1;
        const float2 *b = u + (ok[k] ? ((unsigned)dy * (unsigned)P + (unsigned)dx) : 0u);
        t00[k] = b[0];
        t10[k] = b[1];
        t01[k] = b[P];
        t11[k] = b[P + 1];
    }
#pragma unroll
    for (int k = 0; k < G; k++) {
        const float2 c = cv[k];
        const float gx = fx[k], gy = fy[k];
        const v2f wx0 = v2f{1 - gx, 1 - gx}, wx1 = v2f{gx, gx};
        const v2f wy0 = v2f{1 - gy, 1 - gy}, wy1 = v2f{gy, gy};
        // (t * wx) * wy per component, added in the reference's tap order
        v2f v = (v2f{t00[k].x, t00[k].y} * wx0) * wy0;
        float w = (1 - gx) * (1 - gy);
        const v2f v10 = v + (v2f{t10[k].x, t10[k].y} * wx1) * wy0;
        const float w10 = w + gx * (1 - gy);
        v = ax[k] ? v10 : v;
        w = ax[k] ? w10 : w;
        const v2f v01 = v + (v2f{t01[k].x, t01[k].y} * wx0) * wy1;
        const float w01 = w + (1 - gx) * gy;
        v = ay[k] ? v01 : v;
        w = ay[k] ? w01 : w;
        const bool axy = ax[k] && ay[k];
        const v2f v11 = v + (v2f{t11[k].x, t11[k].y} * wx1) * wy1;
        const float w11 = w + gx * gy;
        v = axy ? v11 : v;
        w = axy ? w11 : w;
        // v / w is v itself when w rounds to exactly 1 (as in warp_batch)
        float2 q = make_float2(c.x + v.x, c.y + v.y);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(ok[k] && w != 1.0f) != 0, 0))
            q = make_float2(c.x + v.x / w, c.y + v.y / w);
        o[k] = ok[k] ? (w != 0 ? q : c) : own[k];
    }
}

// the motion update of DemonsThirions.cpp:33-38 at (i, j0..j0+R-1) from the
// smoothed correction cv.  mode 0: Composition (Motion::accumulate), 1:
// Addition (Field::operator+=), 2: neither (another enum value), 3: store the
// smoothed correction itself (diffeomorphic: exp and compose follow)
template <int R>
__device__ __forceinline__ void store_update(const float2 *__restrict__ u,
                                             float2 *__restrict__ out, int i, int j0, int dimx,
                                             int dimy, int P, const float2 cv[R], int mode) {
    static_assert(R % 4 == 0, "compose batches of four");
    if (mode == 0) {
#pragma unroll
        for (int h = 0; h < R; h += 4) {
            float2 o[4];
            compose_px<4>(u, i, j0 + h, dimx, dimy, P, cv + h, o);
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (j0 + h + k < dimy) out[(long)(j0 + h + k) * P + i] = o[k];
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < R; k++) {
        const int j = j0 + k;
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

// K2 from a correction field in HBM: smoothing + motion update (store_update)
template <int KW, int R = kCr, bool PK = true>
__global__ __launch_bounds__(256) void smooth_compose_kernel(
    const float2 *__restrict__ corr, const float2 *__restrict__ u, float2 *__restrict__ out,
    int dimx, int dimy, int P, ConvArgs a, int mode, int ntl, int gxt) {
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int CY = kCThreadsY * R;
    const int x0 = tile_x(ntl, gxt) * kCx, y0 = blockIdx.y * CY;
    conv_load_tile<KW, R>(tile, corr, dimx, dimy, P, x0, y0, a.cx, a.cy);
    __syncthreads();
    const long N = (long)dimx * dimy;
    const int i = x0 + threadIdx.x;
    if (i >= dimx) return;
    // R consecutive j-lines per thread; the wave index is uniform
    const int r0 = (int)__builtin_amdgcn_readfirstlane(threadIdx.y) * R;
    float2 sm[R];
    bool has[R];
    convR<KW, R, PK>(tile, a, i, y0 + r0, threadIdx.x, r0, dimx, dimy, N, sm, has);
    float2 cv[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
        const int j = y0 + r0 + k;
        cv[k] = make_float2(0.0f, 0.0f);
        if (j < dimy) cv[k] = has[k] ? sm[k] : corr[(long)j * P + i];
    }
    store_update<R>(u, out, i, y0 + r0, dimx, dimy, P, cv, mode);
}

// K1 + K2 for a 64 x CY tile.  1. the warped image over the tile plus a
// (c + 1)-pixel halo into LDS; 2. the correction over the tile plus a c-pixel
// halo into LDS (the halo is recomputed by the neighbouring tiles); 3. the
// sigma_fluid convolution and the motion update.  Per pixel the arithmetic of
// demons_force_kernel + smooth_compose_kernel: bit-identical.
// Tiles at the x edges hold, in the halo columns past the edge, the pixels the
// reference's LINEAR tap indices reach there: column x < 0 of j-line y is
// pixel (x + dimx, y - 1), column x >= dimx is (x - dimx, y + 1) (Field.tpp:254,
// idx + ii).  Every slot is warped, differentiated and corrected as the pixel
// it holds (one-sided gradients at that pixel's own borders, whose missing
// neighbour is exactly the column across the seam), so the convolution reads
// the reference's tap values from LDS like anywhere else.  Needs one wrap at
// most: dimx >= 2 * 64 (launch_demons_update).
// FAST: (float)ca.wfull == 1 and sigma_xsq a power of two whose reciprocal
// `sxq` carries (convR W1, demons_corr SXP); otherwise `sxq` is sigma_xsq
// TX x (TY R) output tile: TX (64 or 128) threads across (one or two waves
// per tile row of threads), TY thread rows of R j-lines each
template <int KW, int R, bool FAST, int TX = kCx, int TY = kCThreadsY>
__global__ __launch_bounds__(TX * TY) OF2D_DEMONS_FUSED_ATTR void demons_fused_kernel(
    const float *__restrict__ Iref, const float *__restrict__ Imov, const float2 *__restrict__ u,
    float2 *__restrict__ out, int dimx, int dimy, int P, float sigma_isq, float sxq,
    ConvArgs ca, int mode, unsigned *__restrict__ status, int bx0) {
    constexpr int c = (KW - 1) / 2;
    constexpr int NT = TX * TY;  // threads
    constexpr int CY = TY * R;
    constexpr int CW = TX + 2 * c, CH = CY + 2 * c;  // correction tile
    constexpr int WW = CW + 2, WH = CH + 2;          // warped-image tile
    __shared__ float wt[WH * WW];
    __shared__ __attribute__((aligned(16))) float2 ct[CH * CW];
    const int x0 = ((int)blockIdx.x + bx0) * TX, y0 = blockIdx.y * CY;
    const int tid = threadIdx.y * TX + threadIdx.x;
    // block-uniform: the warped tile crosses an x edge (its slots past it
    // hold the wrapped pixels)
    const bool xedge = x0 - c - 1 < 0 || x0 + TX + c + 1 > dimx;
    auto wrap = [&](int &x, int &y) __attribute__((always_inline)) {
        const int lo = x < 0, hi = x >= dimx;
        x += lo ? dimx : (hi ? -dimx : 0);
        y += hi - lo;
    };
    {
        // 1. slot s <-> pixel (x0 - c - 1 + s % WW, y0 - c - 1 + s / WW)
        // (wrapped), in batches of BW slots per thread
        constexpr int NW = (WW * WH + NT - 1) / NT, BW = OF2D_DEMONS_BW;
#pragma unroll
        for (int q0 = 0; q0 < NW; q0 += BW) {
            int a[BW], b[BW];
            bool valid[BW], in[BW];
            float res[BW];
#pragma unroll
            for (int q = 0; q < BW; q++) {
                const int s = tid + NT * (q0 + q), r = s / WW;
                a[q] = x0 - c - 1 + (s - r * WW);
                b[q] = y0 - c - 1 + r;
                if (xedge) wrap(a[q], b[q]);
                valid[q] = q0 + q < NW && s < WW * WH;
            }
            warp_batch<BW>(Imov, u, a, b, valid, dimx, dimy, P, res, in);
#pragma unroll
            for (int q = 0; q < BW; q++)
                if (valid[q]) wt[tid + NT * (q0 + q)] = in[q] ? res[q] : 0.0f;
        }
    }
    // 2. correction slot (r, cc) <-> pixel (x0 - c + cc, y0 - c + r), cc < CW,
    // enumerated at the warped tile's pitch WW (index s = r * WW + cc; the
    // lanes with cc >= CW idle): a wave's reads of wt are then one contiguous
    // run with no row seam inside a 32-lane group (no LDS bank conflicts), and
    // its writes of ct stay contiguous.  Iref of the slots is loaded while
    // the warp tile completes.
    // (unconditional loads: a slot outside the image reads element 0 and keeps
    // 0, so the loads issue back to back instead of one branch each)
    constexpr int NC = (WW * CH + NT - 1) / NT;
    float iref[NC];
#pragma unroll
    for (int q = 0; q < NC; q++) {
        const int s = tid + NT * q, r = s / WW, cc = s - r * WW;
        int i = x0 - c + cc, j = y0 - c + r;
        if (xedge) wrap(i, j);
        const bool ok = (s < WW * CH) & (cc < CW) & ((unsigned)j < (unsigned)dimy);
        const float t = Iref[ok ? ((unsigned)j * (unsigned)P + (unsigned)i) : 0u];
        iref[q] = ok ? t : 0.0f;
    }
    __syncthreads();
    {
        // j-lines outside the image hold 0 (their linear index is outside [0, N))
        bool zero = false;
        // block-uniform: every slot has both x and both y neighbours in the
        // image (central differences of gradients.h:9-32 everywhere)
        const bool tin = x0 - c >= 1 && x0 - c + CW <= dimx - 1 && y0 - c >= 1 &&
                         y0 - c + CH <= dimy - 1;
        if (tin) {
#pragma unroll
            for (int q = 0; q < NC; q++) {
                const int s = tid + NT * q, r = s / WW, cc = s - r * WW;
                if (s < WW * CH && cc < CW) {
                    const float *w = wt + (r + 1) * WW + (cc + 1);
                    const float gx = (w[1] - w[-1]) / 2.0f, gy = (w[WW] - w[-WW]) / 2.0f;
                    ct[r * CW + cc] =
                        demons_corr<FAST>(gx, gy, w[0] - iref[q], sigma_isq, sxq, zero);
                }
            }
        } else {
#pragma unroll
        for (int q = 0; q < NC; q++) {
            const int s = tid + NT * q, r = s / WW, cc = s - r * WW;
            if (s < WW * CH && cc < CW) {
                int i = x0 - c + cc, j = y0 - c + r;
                if (xedge) wrap(i, j);
                float2 cv = make_float2(0.0f, 0.0f);
                if ((unsigned)j < (unsigned)dimy) {
                    const float *w = wt + (r + 1) * WW + (cc + 1);
                    const float w0 = w[0];
                    float gx, gy;
                    if (i == 0)
                        gx = w[1] - w0;
                    else if (i == dimx - 1)
                        gx = w0 - w[-1];
                    else
                        gx = (w[1] - w[-1]) / 2.0f;
                    if (j == 0)
                        gy = w[WW] - w0;
                    else if (j == dimy - 1)
                        gy = w0 - w[-WW];
                    else
                        gy = (w[WW] - w[-WW]) / 2.0f;
                    cv = demons_corr<FAST>(gx, gy, w0 - iref[q], sigma_isq, sxq, zero);
                }
                ct[r * CW + cc] = cv;
            }
        }
        }
        if (zero) atomicOr(status, kStatusDivZero);
    }
    __syncthreads();
    // 3. R consecutive j-lines per thread (the columns of the tile inside the
    // image: the last tile may be partial)
    const long N = (long)dimx * dimy;
    const int i = x0 + threadIdx.x;
    if (i >= dimx) return;  // no barrier follows
    const int r0 = (int)__builtin_amdgcn_readfirstlane(threadIdx.y) * R;
    float2 sm[R];
    bool has[R];
    convR<KW, R, true, FAST, TX>(ct, ca, i, y0 + r0, threadIdx.x, r0, dimx, dimy, N, sm, has);
    float2 cv[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
        cv[k] = make_float2(0.0f, 0.0f);
        if (y0 + r0 + k < dimy) cv[k] = has[k] ? sm[k] : ct[(r0 + k + c) * CW + threadIdx.x + c];
    }
    store_update<R>(u, out, i, y0 + r0, dimx, dimy, P, cv, mode);
}

// u_new = u_mid (*) G(sigma_diffusion); Logger partials sum ||u_new - prev||,
// sum ||prev|| per block (fixed order).  The partials feed the fp64 Logger
// mode only (fixed iterations, logger_fp64; the default mode takes the
// reference's float sums from seqnorm_kernels.hip and launches NORM = false):
// an approximation of Motion::norm's float running sum at any precision, so
// the magnitudes take the hardware square root (<= 1 ulp) rather than the
// correctly rounded sequence.  The R previous-motion loads of a thread are
// issued together after the convolution, whose registers they reuse.
template <int KW, int R = kCr, bool PK = true, bool W1 = false, bool NORM = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KW == 7 ? 7 : 8))) void smooth_norm_kernel(const float2 *__restrict__ umid,
                                                          const float2 *__restrict__ prev,
                                                          float2 *__restrict__ out, int dimx,
                                                          int dimy, int P, ConvArgs a,
                                                          double *__restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) float2 tile[];
    constexpr int CY = kCThreadsY * R;
    const int x0 = blockIdx.x * kCx, y0 = blockIdx.y * CY;
    conv_load_tile<KW, R>(tile, umid, dimx, dimy, P, x0, y0, a.cx, a.cy);
    __syncthreads();
    const long N = (long)dimx * dimy;
    const int i = x0 + threadIdx.x;
    double sd = 0.0, sp = 0.0;
    if (i < dimx) {
        const int r0 = (int)__builtin_amdgcn_readfirstlane(threadIdx.y) * R;
        const int j0 = y0 + r0;
        float2 sm[R];
        bool has[R];
        convR<KW, R, PK, W1>(tile, a, i, j0, threadIdx.x, r0, dimx, dimy, N, sm, has);
        // every output of the thread is the convolution's: no fallback loads
        // of u_mid (the loads below are skipped by branch, not by select)
        const bool conv_all = W1 && KW > 0 && conv_rows_interior<KW, R>(i, j0, dimx, dimy, N);
        float2 pv[R];
        if (NORM) {
#pragma unroll
            for (int k = 0; k < R; k++)
                pv[k] = prev[j0 + k < dimy ? (unsigned)(j0 + k) * (unsigned)P + (unsigned)i : 0u];
        }
#pragma unroll
        for (int k = 0; k < R; k++) {
            const int j = j0 + k;
            if (j >= dimy) break;
            const unsigned idx = (unsigned)j * (unsigned)P + (unsigned)i;
            float2 v = sm[k];
            if (!conv_all && !has[k]) v = umid[idx];
            out[idx] = v;
            if (NORM) {
                const float ex = v.x - pv[k].x, ey = v.y - pv[k].y;
                sd += (double)__builtin_amdgcn_sqrtf(ex * ex + ey * ey);
                sp += (double)__builtin_amdgcn_sqrtf(pv[k].x * pv[k].x + pv[k].y * pv[k].y);
            }
        }
    }
    if (!NORM) return;
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

inline size_t conv_lds_bytes(int cx, int cy, int R = kCr) {
    return sizeof(float2) * (size_t)(kCx + 2 * cx) * (kCThreadsY * R + 2 * cy);
}
inline dim3 conv_grid_r(int dimx, int dimy, int R) {
    return dim3((dimx + kCx - 1) / kCx, (dimy + kCThreadsY * R - 1) / (kCThreadsY * R));
}
dim3 conv_grid(int dimx, int dimy) { return conv_grid_r(dimx, dimy, kCr); }
int conv_nblocks(int dimx, int dimy) {
    const dim3 g = conv_grid(dimx, dimy);
    return int(g.x * g.y);
}

namespace {
// smooth_compose over `gridx` block columns: tiles [0, ntl) and the last
// gridx - ntl tiles of the gxt-tile row
void smooth_compose_tiles(const float2 *corr, const float2 *u, float2 *out, int dimx, int dimy,
                          int P, const ConvArgs &a, int mode, int gridx, int ntl, int gxt,
                          hipStream_t st) {
    const dim3 g(gridx, conv_grid(dimx, dimy).y);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, g, dim3(64, kCThreadsY), conv_lds_bytes(a.cx, a.cy), st, corr, u,
                           out, dimx, dimy, P, a, mode, ntl, gxt);
    };
    switch (a.kw) {
        case 3: go(smooth_compose_kernel<3>); break;
        case 5: go(smooth_compose_kernel<5>); break;
        case 7: go(smooth_compose_kernel<7>); break;
        default: go(smooth_compose_kernel<0>); break;
    }
    OF2D_HIP(hipGetLastError());
}
}  // namespace

void launch_smooth_compose(const float2 *corr, const float2 *u, float2 *out, int dimx, int dimy,
                           int P, const float *kf, const double *kd, int kw, double wfull,
                           int mode, hipStream_t st) {
    const int c = (kw - 1) / 2;
    const ConvArgs a{kf, kd, kw, c, c, wfull};
    const int gx = conv_grid(dimx, dimy).x;
    smooth_compose_tiles(corr, u, out, dimx, dimy, P, a, mode, gx, gx, gx, st);
}

void launch_demons_update(const float *Iref, const float *Imov, const float2 *u, float2 *corr,
                          float2 *out, int dimx, int dimy, int P, float sigma_isq,
                          float sigma_xsq, const float *kf, const double *kd, int kw,
                          double wfull, int mode, unsigned *status, hipStream_t st) {
    const int c = (kw - 1) / 2;
    const ConvArgs a{kf, kd, kw, c, c, wfull};
    const int gx = (dimx + kCx - 1) / kCx;
    // the fused kernel takes every tile, the x-edge ones included, when its
    // width is compiled in and no tile wraps more than once (dimx >= 128)
    if (!(kw == 3 || kw == 5 || kw == 7) || dimx < 2 * kCx) {
        launch_demons_force(Iref, Imov, u, corr, dimx, dimy, P, sigma_isq, sigma_xsq, status, st);
        smooth_compose_tiles(corr, u, out, dimx, dimy, P, a, mode, gx, gx, gx, st);
        return;
    }
    float rsx = 0.0f;
    const bool fast = (float)wfull == 1.0f && pow2_reciprocal(sigma_xsq, &rsx);
    constexpr int TX = OF2D_DEMONS_TX, TY = OF2D_DEMONS_TY;
    // one wrap at most per tile: the tile narrower than half the image
    if (dimx < 2 * TX) {
        launch_demons_force(Iref, Imov, u, corr, dimx, dimy, P, sigma_isq, sigma_xsq, status, st);
        smooth_compose_tiles(corr, u, out, dimx, dimy, P, a, mode, gx, gx, gx, st);
        return;
    }
    const dim3 g((dimx + TX - 1) / TX, (dimy + TY * kCr - 1) / (TY * kCr));
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, g, dim3(TX, TY), 0, st, Iref, Imov, u, out, dimx, dimy, P,
                           sigma_isq, fast ? rsx : sigma_xsq, a, mode, status, 0);
    };
    switch (kw * 2 + fast) {
        case 6: go(demons_fused_kernel<3, kCr, false, TX, TY>); break;
        case 7: go(demons_fused_kernel<3, kCr, true, TX, TY>); break;
        case 10: go(demons_fused_kernel<5, kCr, false, TX, TY>); break;
        case 11: go(demons_fused_kernel<5, kCr, true, TX, TY>); break;
        case 15: go(demons_fused_kernel<7, kCr, true, TX, TY>); break;
        default: go(demons_fused_kernel<7, kCr, false, TX, TY>); break;
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
    const bool w1 = (float)wfull == 1.0f;
    // no partials wanted (the Logger's float sums come from seqnorm): no norms
    if (!partial) {
        switch (w1 ? kw : -kw) {
            case 3: go(smooth_norm_kernel<3, kCr, true, true, false>); break;
            case -3: go(smooth_norm_kernel<3, kCr, true, false, false>); break;
            case 5: go(smooth_norm_kernel<5, kCr, true, true, false>); break;
            case -5: go(smooth_norm_kernel<5, kCr, true, false, false>); break;
            case 7: go(smooth_norm_kernel<7, kCr, true, true, false>); break;
            case -7: go(smooth_norm_kernel<7, kCr, true, false, false>); break;
            default: go(smooth_norm_kernel<0, kCr, true, false, false>); break;
        }
        OF2D_HIP(hipGetLastError());
        return;
    }
    switch (w1 ? kw : -kw) {
        case 3: go(smooth_norm_kernel<3, kCr, true, true>); break;
        case -3: go(smooth_norm_kernel<3>); break;
        case 5: go(smooth_norm_kernel<5, kCr, true, true>); break;
        case -5: go(smooth_norm_kernel<5>); break;
        case 7: go(smooth_norm_kernel<7, kCr, true, true>); break;
        case -7: go(smooth_norm_kernel<7>); break;
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
