// hs_jacobi_impl.h — the fused Horn-Schunck Jacobi kernels the product
// launches (hs_kernels.hip): one, two and three iterations per pass.  The
// measured variants that are not launched (four iterations per pass, the
// pre-OPT row step, diagnostic modes) live in tools/hs_variants_impl.h with
// the tuning harness.
//
// Restates, fused into one pass over HBM, the three full-grid passes of
// OpticalFlowDiffusion::get_update (src/regularization/OpticalFlow/
// OpticalFlowDiffusion.cpp:43-55):
//   q  = qlaplacian(u_old)                  gradients.h:72-80, OpticalFlowDiffusion.cpp:19-40
//   f  = dI * ((It + q.x*dI.x) + q.y*dI.y)  OpticalFlow.cpp:15-39 (called with q)
//   u' = q - f / ((alpha^2 + dI.x^2) + dI.y^2)   OpticalFlowDiffusion.cpp:57-84
// plus the per-pixel magnitudes of Logger::update_error (Logger.cpp:32-51,
// Motion.cpp:42-49): sum ||u'-u|| and sum ||u|| (prev == u_old for HS).
//
// Geometry: a wave owns a strip of 64*PXL px (PXL consecutive px per lane,
// 16-B loads) and marches ROWS j-lines down it, keeping u at j-1, j, j+1 in
// registers; x-neighbours come from the adjacent lanes by DPP wave shifts
// (the strip's two edge lanes load one float2 each).  WAVES waves of a block
// march consecutive row bands of the same strip.
#pragma once

#include "of2d_device.h"
#include <type_traits>


// the intermediate iterates of the MID triple (read again by the Logger's
// pass): default cache policy (0) or non-temporal (1).  Non-temporal, like the
// pass's loads, so the MALL keeps the triple's gradient fields: 4096^2 texture
// convergence 132 -> 124-126 us per iteration, procedural unchanged
// (profiles/r05q_ahead_ab.log)
#ifndef OF2D_HS_MID_NT
#define OF2D_HS_MID_NT 1
#endif

namespace of2d {
namespace hs {

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ float4 ld4(const float4 *p) {
    if constexpr (NT) {
        const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
template <bool NT>
__device__ __forceinline__ float2 ld2(const float2 *p) {
    if constexpr (NT) {
        const v2f v = __builtin_nontemporal_load(reinterpret_cast<const v2f *>(p));
        return make_float2(v.x, v.y);
    } else {
        return *p;
    }
}
template <bool NT>
__device__ __forceinline__ void st4(float4 *p, float4 v) {
    if constexpr (NT) {
        v4f w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<v4f *>(p));
    } else {
        *p = v;
    }
}

// lane i <- lane i-1 / lane i+1 by DPP (wave_shr:1 / wave_shl:1): a VALU op,
// not an LDS permute; the lane without a source (0 / 63) reads 0 and is
// patched or unused by the callers
__device__ __forceinline__ float dpp_from_left(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float dpp_from_right(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, true));
}

// |v| for the Logger sums: v_sqrt_f32 (within 1 ulp).  The norms only feed the
// fp64 convergence sums, which already differ from the reference's sequential
// fp32 sum in rounding (tests compare errors at a stated tolerance); the
// motion itself never depends on them.
__device__ __forceinline__ double norm_d(float x, float y) {
    return (double)__builtin_amdgcn_sqrtf(x * x + y * y);
}

// q = 0 on the border (gradients.h:73-76) as a bit mask, so the compiler
// keeps the stencil branch-free (a select here became divergent branches)
__device__ __forceinline__ float2 zero_if(bool z, float2 q) {
    const int keep = z ? 0 : -1;
    return make_float2(__int_as_float(__float_as_int(q.x) & keep),
                       __int_as_float(__float_as_int(q.y) & keep));
}

__device__ __forceinline__ float2 update_px(float2 q, float gx, float gy, float it,
                                            float alphasq, unsigned &bad) {
    const float s = (it + q.x * gx) + q.y * gy;      // OpticalFlow.cpp:33
    const float fx = gx * s, fy = gy * s;            // coord2d * float
    const float den = (alphasq + gx * gx) + gy * gy;  // OpticalFlowDiffusion.cpp:78
    bad |= (den == 0.0f) ? 1u : 0u;                  // coord2d.h:95-100 throws
    return make_float2(q.x - fx / den, q.y - fy / den);
}

// ---------------------------------------------------------------------------
// fp32 division without the range-scaling steps.  The compiler expands the
// IEEE quotient a / b as
//   bs = div_scale(b, b, a); as, vcc = div_scale(a, b, a); r = rcp(bs)
//   r = fma(fma(-bs, r, 1), r, r); q = as * r; q = fma(fma(-bs, q, as), r, q)
//   q = div_fmas(fma(-bs, q, as), r, q, vcc); a / b = div_fixup(q, b, a)
// div_scale returns its operand unchanged and clears vcc unless a or b is 0,
// b is denormal, 1/b or a/b would be denormal, |a| < 2^-103, or a/b is within
// 2^96 of the overflow threshold.  With b in [2^-40, 2^40) and a in 0 or
// [2^-80, 2^50] none of these holds except a == 0, and for a == 0 (and for
// inf / NaN operands) div_fixup returns the special value from b and a alone.
// In that range the sequence below is therefore the compiler's sequence on
// the same values: bit-identical quotients, with the reciprocal refinement
// (which depends on b only) shared by every division by the same b.
__device__ __forceinline__ float recip_refined(float b) {
    const float r0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, r0, 1.0f), r0, r0);
}
// (ax / b, ay / b) for b with refined reciprocal r, both components packed
__device__ __forceinline__ float2 div2_unscaled(float ax, float ay, float b, float r) {
    const v2f a = {ax, ay}, nb = {-b, -b}, rr = {r, r};
    v2f q = a * rr;
    v2f e = __builtin_elementwise_fma(nb, q, a);
    q = __builtin_elementwise_fma(e, rr, q);
    e = __builtin_elementwise_fma(nb, q, a);
    q = __builtin_elementwise_fma(e, rr, q);
    return make_float2(__builtin_amdgcn_div_fixupf(q.x, b, ax),
                       __builtin_amdgcn_div_fixupf(q.y, b, ay));
}
// frexp exponent of v within [lo, hi] (0, inf and NaN have exponent 0)
template <int LO, int HI>
__device__ __forceinline__ bool exp_in(float v) {
    return (unsigned)(__builtin_amdgcn_frexp_expf(v) - LO) <= (unsigned)(HI - LO);
}

// What the unscaled division needs from the gradients, checked once per field
// instead of per row step: every gradient the Jacobi kernels can read (the whole
// allocation, ghost j-lines and padding included) in 0 or [2^-30, 2^20) and its
// denominator (alpha^2 + gx^2) + gy^2 in [2^-40, 2^40), else range_flag |= 1.
// Also the reference's divide-by-zero test (coord2d.h:95-100) on the image
// pixels, the only pixels whose division the reference performs: status |=
// kStatusDivZero if a denominator is 0 — dI is fixed for the whole loop, so
// this is the test every iteration would repeat.
template <int = 0>
__global__ void hs_precheck_kernel(const float2 *__restrict__ base, long count, int P, int ghost,
                                   int dimx, int dimy, float alphasq,
                                   unsigned *__restrict__ range_flag,
                                   unsigned *__restrict__ status) {
    bool bad = false, zero = false;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (long)gridDim.x * blockDim.x) {
        const float2 g = base[i];
        const float den = (alphasq + g.x * g.x) + g.y * g.y;
        bad |= !(exp_in<-29, 20>(g.x) && exp_in<-29, 20>(g.y) && exp_in<-39, 40>(den));
        const long row = i / P - ghost;
        const int col = (int)(i % P);
        zero |= den == 0.0f && row >= 0 && row < dimy && col < dimx;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(range_flag, 1u);
    if (__any(zero) && (threadIdx.x & 63) == 0) atomicOr(status, kStatusDivZero);
}

// u rows as PXL float2 per lane
template <int PXL>
struct Row {
    float2 v[PXL];
};

template <int PXL, bool NT>
__device__ __forceinline__ Row<PXL> load_row(const float2 *row, int x) {
    Row<PXL> r;
    const float4 *p = reinterpret_cast<const float4 *>(row + x);
#pragma unroll
    for (int k = 0; k < PXL / 2; k++) {
        const float4 a = ld4<NT>(p + k);
        r.v[2 * k] = make_float2(a.x, a.y);
        r.v[2 * k + 1] = make_float2(a.z, a.w);
    }
    return r;
}

template <int ROWS, int PXL, int WAVES, bool NT_LD, bool NT_ST, bool NT_G = NT_LD>
__global__ __launch_bounds__(64 * WAVES) void jacobi_kernel(
    const float2 *__restrict__ uo, float2 *__restrict__ un, const float2 *__restrict__ dI,
    const float *__restrict__ It, int P, int dimx, int nrows, int row0, int dimy, float alphasq,
    double *__restrict__ partial, unsigned *__restrict__ status) {
    static_assert(PXL == 2 || PXL == 4, "PXL");
    constexpr int STRIP = 64 * PXL;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = blockIdx.x * STRIP + PXL * lane;
    const int jbeg = (blockIdx.y * WAVES + wave) * ROWS;
    const int jend = min(jbeg + ROWS, nrows);

    double sdiff = 0.0, sprev = 0.0;
    unsigned bad = 0;
    if (jbeg < nrows) {
        const bool need_l = (lane == 0) && (x > 0) && (x < dimx - 1);
        const bool need_r = (lane == 63) && (x + PXL < dimx);
        Row<PXL> um = load_row<PXL, NT_LD>(uo + (long)(jbeg - 1) * P, x);  // ghost j-line ok
        Row<PXL> uc = load_row<PXL, NT_LD>(uo + (long)jbeg * P, x);
        for (int j = jbeg; j < jend; ++j) {
            const Row<PXL> up = load_row<PXL, NT_LD>(uo + (long)(j + 1) * P, x);
            Row<PXL> g = load_row<PXL, NT_G>(dI + (long)j * P, x);
            float t[PXL];
            if constexpr (PXL == 2) {
                const float2 tt = ld2<NT_G>(reinterpret_cast<const float2 *>(It + (long)j * P + x));
                t[0] = tt.x;
                t[1] = tt.y;
            } else {
                const float4 tt = ld4<NT_G>(reinterpret_cast<const float4 *>(It + (long)j * P + x));
                t[0] = tt.x;
                t[1] = tt.y;
                t[2] = tt.z;
                t[3] = tt.w;
            }
            float2 left, right;
            left.x = dpp_from_left(uc.v[PXL - 1].x);
            left.y = dpp_from_left(uc.v[PXL - 1].y);
            right.x = dpp_from_right(uc.v[0].x);
            right.y = dpp_from_right(uc.v[0].y);
            if (need_l) left = uo[(long)j * P + x - 1];
            if (need_r) right = uo[(long)j * P + x + PXL];
            const int jg = row0 + j;
            const bool yb = (jg == 0) || (jg == dimy - 1);
            float2 nw[PXL];
#pragma unroll
            for (int k = 0; k < PXL; k++) {
                const float2 l = (k == 0) ? left : uc.v[k - 1];
                const float2 r = (k == PXL - 1) ? right : uc.v[k + 1];
                float2 q;
                // gradients.h:77-79: (((u[i-1] + u[i+1]) + u[j-1]) + u[j+1]) / 4.0f
                q.x = (((l.x + r.x) + um.v[k].x) + up.v[k].x) / 4.0f;
                q.y = (((l.y + r.y) + um.v[k].y) + up.v[k].y) / 4.0f;
                const int xi = x + k;
                q = zero_if(yb || xi == 0 || xi == dimx - 1, q);  // :73-76
                unsigned b = 0;
                nw[k] = update_px(q, g.v[k].x, g.v[k].y, t[k], alphasq, b);
                if (xi < dimx) {
                    bad |= b;
                    sdiff += norm_d(nw[k].x - uc.v[k].x, nw[k].y - uc.v[k].y);
                    sprev += norm_d(uc.v[k].x, uc.v[k].y);
                }
            }
            float2 *dst = un + (long)j * P + x;
            if (x + PXL <= dimx) {
#pragma unroll
                for (int k = 0; k < PXL / 2; k++)
                    st4<NT_ST>(reinterpret_cast<float4 *>(dst) + k,
                               make_float4(nw[2 * k].x, nw[2 * k].y, nw[2 * k + 1].x,
                                           nw[2 * k + 1].y));
            } else {
#pragma unroll
                for (int k = 0; k < PXL; k++)
                    if (x + k < dimx) dst[k] = nw[k];
            }
            um = uc;
            uc = up;
        }
    }
    // fixed-order block reduction -> one (diff, prev) pair per block
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        sdiff += __shfl_down(sdiff, off);
        sprev += __shfl_down(sprev, off);
    }
    __shared__ double red[2][WAVES];
    if (lane == 0) {
        red[0][wave] = sdiff;
        red[1][wave] = sprev;
    }
    if (__any(bad) && lane == 0) atomicOr(status, kStatusDivZero);
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            a += red[0][w];
            b += red[1][w];
        }
        const long blk = (long)blockIdx.y * gridDim.x + blockIdx.x;
        partial[2 * blk] = a;
        partial[2 * blk + 1] = b;
    }
}

// ---------------------------------------------------------------------------
// Two Jacobi iterations per pass over HBM (temporal blocking).  Same per-pixel
// arithmetic as jacobi_kernel, applied twice: u1 = step(u), u2 = step(u1).
// A wave loads a strip of 64*PXL px starting PXL px left of its 62*PXL output
// columns (lanes 1..62 own PXL px each; lanes 0 and 63 are the halo that u1
// needs), so no edge lane loads anything extra and every load stays 16-B
// aligned.  Down the strip it keeps u at rows j..j+2 and u1 at rows j-1..j+1
// in registers: one u row, one dI row and one It row in, one u2 row out per
// step, 28 B per pixel for TWO iterations (+ the 4 / 2 halo rows of a ROWS
// band and the 2 halo lanes).  Rows outside [0, dimy) are read from the
// clamped ghost lines and never feed a pixel of the image (the border rule
// zeroes q there).  Logger partials of both iterations over the owned pixels:
// partial[2*blk..] for the first, partial2[2*blk..] for the second.
template <int PXL>
constexpr int hs2_out() {
    return 62 * PXL;
}

// XCD-aware block order: the hardware deals workgroup w to XCD w % 8, so
// logical block L = (w % 8) * ceil(n / 8) + w / 8 puts runs of consecutive
// strips (which share the 128-B lines at their unaligned borders and, a band
// row further, their halo rows) on one XCD and its L2.  Returns false for the
// padding workgroups of the last XCD.
__device__ __forceinline__ bool xcd_block(int gx, int gy, int &bx, int &by) {
    const int n = gx * gy, per = (n + 7) / 8;
    const int w = (int)blockIdx.x;
    const int L = (w % 8) * per + w / 8;
    if (L >= n) return false;
    bx = L % gx;
    by = L / gx;
    return true;
}

template <int ROWS, int WAVES, int PXL = 2, bool XCD = false>
__global__ __launch_bounds__(64 * WAVES) void jacobi2_kernel(
    const float2 *__restrict__ uo, float2 *__restrict__ un, const float2 *__restrict__ dI,
    const float *__restrict__ It, int P, int dimx, int nrows, int row0, int dimy, float alphasq,
    int glo, int ghi, double *__restrict__ partial, double *__restrict__ partial2,
    unsigned *__restrict__ status, int band0, int gx, int gy) {
    // XCD: a 1-D grid of 8 * ceil(gx * gy / 8) workgroups remapped by
    // xcd_block; otherwise a gx x gy grid
    int bx = (int)blockIdx.x, by = (int)blockIdx.y;
    if constexpr (XCD) {
        if (!xcd_block(gx, gy, bx, by)) return;
    }
    static_assert(PXL == 2 || PXL == 4, "PXL");
    // band0: this launch covers row bands band0 .. band0 + gridDim.y - 1 (a
    // band = WAVES * ROWS j-lines), so a slab can run its interior bands while
    // the halo exchange that only the outer bands read is in flight
    // glo / ghi: first / one-past-last local row whose u, dI and It may be
    // read (ghost j-lines included); rows outside are clamped into it
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = bx * hs2_out<PXL>() - PXL + PXL * lane;  // this lane's px x..x+PXL-1
    const bool own = lane >= 1 && lane <= 62 && x < dimx;
    const bool xin = x >= 0 && x + PXL <= P;  // the lane's px lie inside the pitched row
    const int band = band0 + by;
    const int jbeg = (band * WAVES + wave) * ROWS;
    const int jend = min(jbeg + ROWS, nrows);
    double sd1 = 0.0, sp1 = 0.0, sd2 = 0.0, sp2 = 0.0;
    unsigned bad = 0;
    auto cl = [&](int j) { return min(max(j, glo), ghi - 1); };
    // lanes whose px lie outside the pitched row read a clamped in-row group
    // instead (their values only reach the halo lanes 0 / 63)
    const int xl = xin ? x : (x < 0 ? 0 : P - PXL);
    auto ldu = [&](int j) { return load_row<PXL, true>(uo + (long)cl(j) * P, xl); };
    auto ldg = [&](int j, Row<PXL> &g, float t[PXL]) {
        g = load_row<PXL, false>(dI + (long)cl(j) * P, xl);
        const float *tp = It + (long)cl(j) * P + xl;
        if constexpr (PXL == 2) {
            const float2 tt = *reinterpret_cast<const float2 *>(tp);
            t[0] = tt.x;
            t[1] = tt.y;
        } else {
            const float4 tt = *reinterpret_cast<const float4 *>(tp);
            t[0] = tt.x;
            t[1] = tt.y;
            t[2] = tt.z;
            t[3] = tt.w;
        }
    };
    // one Jacobi step at row j from rows (m, c, p) of its input
    auto stepr = [&](int j, const Row<PXL> &m, const Row<PXL> &c, const Row<PXL> &p,
                     const Row<PXL> &g, const float t[PXL], unsigned &b) {
        float2 left, right;
        left.x = dpp_from_left(c.v[PXL - 1].x);
        left.y = dpp_from_left(c.v[PXL - 1].y);
        right.x = dpp_from_right(c.v[0].x);
        right.y = dpp_from_right(c.v[0].y);
        const int jg = row0 + j;
        const bool yb = (jg == 0) || (jg == dimy - 1);
        Row<PXL> o;
#pragma unroll
        for (int k = 0; k < PXL; k++) {
            const float2 l = (k == 0) ? left : c.v[k - 1];
            const float2 r = (k == PXL - 1) ? right : c.v[k + 1];
            float2 q;
            q.x = (((l.x + r.x) + m.v[k].x) + p.v[k].x) / 4.0f;
            q.y = (((l.y + r.y) + m.v[k].y) + p.v[k].y) / 4.0f;
            const int xi = x + k;
            q = zero_if(yb || xi == 0 || xi == dimx - 1, q);
            o.v[k] = update_px(q, g.v[k].x, g.v[k].y, t[k], alphasq, b);
        }
        return o;
    };
    // px k of the lane inside the image: a select, not a product (padding may
    // hold 0/0 when alpha = 0)
    auto norms = [&](const Row<PXL> &nw, const Row<PXL> &od, double &sd, double &sp) {
#pragma unroll
        for (int k = 0; k < PXL; k++) {
            const double d = norm_d(nw.v[k].x - od.v[k].x, nw.v[k].y - od.v[k].y);
            const double q = norm_d(od.v[k].x, od.v[k].y);
            const bool in = x + k < dimx;
            sd += in ? d : 0.0;
            sp += in ? q : 0.0;
        }
    };
    if (jbeg < nrows) {
        // u rows jbeg-2 .. jbeg+1; u1 rows jbeg-1, jbeg
        Row<PXL> a0 = ldu(jbeg - 2), a1 = ldu(jbeg - 1), a2 = ldu(jbeg), a3 = ldu(jbeg + 1);
        Row<PXL> gm, gc;
        float tm[PXL], tc[PXL];
        ldg(jbeg - 1, gm, tm);
        ldg(jbeg, gc, tc);
        unsigned bx = 0;  // halo rows: flagged by the waves that own them
        Row<PXL> v0 = stepr(jbeg - 1, a0, a1, a2, gm, tm, bx);  // u1 row j-1
        Row<PXL> v1 = stepr(jbeg, a1, a2, a3, gc, tc, bx);      // u1 row j
        // a2 = u row j, a3 = u row j+1; the loads of step j+1 are issued during
        // step j (one row of software prefetch)
        Row<PXL> nu = ldu(jbeg + 2), ng;
        float nt[PXL];
        ldg(jbeg + 1, ng, nt);
        for (int j = jbeg; j < jend; ++j) {
            const Row<PXL> a4 = nu;
            const Row<PXL> gp = ng;
            float tp[PXL];
#pragma unroll
            for (int k = 0; k < PXL; k++) tp[k] = nt[k];
            if (j + 1 < jend) {
                nu = ldu(j + 3);
                ldg(j + 2, ng, nt);
            }
            unsigned b1 = 0, b2 = 0;
            const Row<PXL> v2 = stepr(j + 1, a2, a3, a4, gp, tp, b1);  // u1 row j+1
            const Row<PXL> w = stepr(j, v0, v1, v2, gc, tc, b2);       // u2 row j
            if (own) {
                norms(v1, a2, sd1, sp1);  // first iteration at row j: u1 against u
                norms(w, v1, sd2, sp2);   // second: u2 against u1
                // the denominator depends on dI only, so the second iteration's
                // zero test at (x, j) is also the first one's
                bad |= b2;
                float2 *dst = un + (long)j * P + x;
                if (x + PXL <= dimx) {
#pragma unroll
                    for (int k = 0; k < PXL / 2; k++)
                        st4<true>(reinterpret_cast<float4 *>(dst) + k,
                                  make_float4(w.v[2 * k].x, w.v[2 * k].y, w.v[2 * k + 1].x,
                                              w.v[2 * k + 1].y));
                } else {
#pragma unroll
                    for (int k = 0; k < PXL; k++)
                        if (x + k < dimx) dst[k] = w.v[k];
                }
            }
            v0 = v1;
            v1 = v2;
            a2 = a3;
            a3 = a4;
            gc = gp;
#pragma unroll
            for (int k = 0; k < PXL; k++) tc[k] = tp[k];
        }
    }
    // fixed-order block reductions -> (diff, prev) per iteration per block
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        sd1 += __shfl_down(sd1, off);
        sp1 += __shfl_down(sp1, off);
        sd2 += __shfl_down(sd2, off);
        sp2 += __shfl_down(sp2, off);
    }
    __shared__ double red[4][WAVES];
    if (lane == 0) {
        red[0][wave] = sd1;
        red[1][wave] = sp1;
        red[2][wave] = sd2;
        red[3][wave] = sp2;
    }
    if (__any(bad) && lane == 0) atomicOr(status, kStatusDivZero);
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0, c = 0.0, d = 0.0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) {
            a += red[0][w];
            b += red[1][w];
            c += red[2][w];
            d += red[3][w];
        }
        const long blk = (long)band * gx + bx;
        partial[2 * blk] = a;
        partial[2 * blk + 1] = b;
        partial2[2 * blk] = c;
        partial2[2 * blk + 1] = d;
    }
}

// ---------------------------------------------------------------------------
// Three Jacobi iterations per pass (u1 = step(u), u2 = step(u1), u3 = step(u2)):
// the pair kernel's scheme one level deeper.  A wave loads 128 px starting
// 4 px left of its 120 output columns (lanes 2..61 own 2 px each; lanes 0-1
// and 62-63 are the halo the first two steps need), keeps u at rows j..j+3,
// u1 at j..j+2 and u2 at j-1..j+1 in registers, and per step reads one u row,
// one dI and one It row and writes one u3 row: 28 B per pixel for THREE
// iterations (+ the 6 / 4 halo rows of a band).  Bit-identical to three
// single steps.  Logger partials of the three iterations: partial, partial2,
// partial3.  Measured in tools/hs_variants.hip ("two"): ~10 % less time per
// iteration than the pair kernel at 4096^2 (47.6 vs 52.7 us) — the kernels are
// now issue/latency-bound more than HBM-bound.  band0 as in jacobi2_kernel.
// ROWS > 0: j-lines per wave fixed at compile time; ROWS == 0: `rows` (chosen
// by the launcher so that the grid fills whole rounds of resident blocks)
// Issue priority by progress (PRIO > 0).  The SIMD arbiter issues VALU by
// priority, then age, so with equal priorities the four co-resident waves of a
// SIMD finish in dispatch order and the youngest runs its last rows with the
// SIMD nearly empty (tools/hs_variants stamps).  Waves that have done less
// of their band run at higher priority, which keeps the four abreast.
template <int PRIO>
__device__ __forceinline__ void progress_prio(int done, int total) {
    if constexpr (PRIO == 1) {
        const int q = (done * 16) / total;  // scalar
        if (q < 8)
            __builtin_amdgcn_s_setprio(3);
        else if (q < 12)
            __builtin_amdgcn_s_setprio(2);
        else if (q < 14)
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
    } else if constexpr (PRIO == 3) {
        const int q = (done * 3) / total;
        if (q < 1)
            __builtin_amdgcn_s_setprio(2);
        else if (q < 2)
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
    } else if constexpr (PRIO == 4) {
        const int q = (done * 20) / total;
        if (q < 6)
            __builtin_amdgcn_s_setprio(3);
        else if (q < 11)
            __builtin_amdgcn_s_setprio(2);
        else if (q < 16)
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
    } else if constexpr (PRIO == 2) {
        const int q = (done * 4) / total;
        if (q < 1)
            __builtin_amdgcn_s_setprio(3);
        else if (q < 2)
            __builtin_amdgcn_s_setprio(2);
        else if (q < 3)
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
    }
}

// Row step: border masks behind a wave-uniform branch (only strips and rows
// that touch the image border apply them), the division range test on min /
// max of |sc| (zeros take the IEEE path), the x-neighbour lane shifts folded
// into the first add of each sum (v_add_f32 with DPP).  The division by the
// denominator is the unscaled exact sequence (div2_unscaled) when the
// gradient field passed hs_precheck_kernel's range test (range_flag == 0).
// ALT: odd waves march their band upward (from its last j-line to its first),
// even waves downward, so the two waves on either side of every band boundary
// of a block read the shared halo j-lines at about the same time (both at the
// start or both at the end of their bands) and the second read hits in L2;
// with one direction the halo rows of a band boundary are read a whole band
// apart, from HBM twice.  The stencil is symmetric in j and every output
// depends only on input values: bit-identical either way.
// GI: the gradients are not read from dI but derived in the kernel from the
// image they were taken of, Iaux (IterativeSolver::spatial_derivative,
// IterativeSolver.cpp:22-56, gradients.h:9-32: the same float operations, so
// the same bits as dI): per row step one Iaux row (4 B/px) replaces one dI row
// (8 B/px), 24 instead of 28 B per pixel and launch.  The x-neighbours of a
// lane's two Iaux px come by DPP from the adjacent lanes like those of u; the
// j-neighbours are the Iaux rows before and after in the march.  Iaux needs
// the same ghost j-lines as u (rows glo .. ghi-1 readable).  Worth it when dI
// and It do not stay resident in the 256 MB MALL between launches (the
// launchers' callers decide, of2d_device.h hs3_gradients_from_image).
// MID: the two intermediate iterates u1, u2 of the owned rows are stored too
// (to m1, m2): the reference-exact Logger needs every iterate in memory
// (registration.cpp run_chunked_exact), 16 B/px more per launch.
template <int ROWS, int WAVES, bool XCD, int MINB, int UNR, int PRIO, bool ALT, bool GI,
          bool MID>
__device__ __forceinline__ void jacobi3_body(
    const float2 *__restrict__ uo, float2 *__restrict__ un, const float2 *__restrict__ dI,
    const float *__restrict__ It, int P, int dimx, int nrows, int row0, int dimy, float alphasq,
    int glo, int ghi, double *__restrict__ partial, double *__restrict__ partial2,
    double *__restrict__ partial3, unsigned *__restrict__ status, int band0, int gx, int gy,
    int rows, const unsigned *__restrict__ range_flag, int jlo, int jhi,
    const float *__restrict__ Ia, float2 *__restrict__ m1, float2 *__restrict__ m2) {
    int bx = (int)blockIdx.x, by = (int)blockIdx.y;
    if constexpr (XCD) {
        if (!xcd_block(gx, gy, bx, by)) return;
    }
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane lets the compiler keep the row
    // arithmetic in scalar registers (buffer loads with scalar row offsets
    // measured 5 % slower than these global loads)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int x = bx * kHs3Out - 4 + 2 * lane;  // this lane's px x, x+1
    const bool own = lane >= 2 && lane <= 61 && x < dimx;
    const bool xin = x >= 0 && x + 2 <= P;
    // block row `by` of this launch covers j-lines from jlo (default: band0's
    // first line) up to jhi (default nrows); its Logger partials go to slot
    // (band0 + by) * gx + bx
    const int band = band0 + by;
    if (jlo < 0) jlo = band0 * WAVES * rows;
    if (jhi < 0) jhi = nrows;
    const int jbeg = jlo + (by * WAVES + wave) * rows;
    const int jend = min(jbeg + rows, jhi);
    // Logger magnitudes accumulate in fp32 per lane (<= 2 * rows values of one
    // wave), in fp64 from the lane sums on; they only feed the convergence test
    float s1d = 0.0f, s1p = 0.0f, s2d = 0.0f, s2p = 0.0f, s3d = 0.0f, s3p = 0.0f;
    unsigned bad = 0;
    auto cl = [&](int j) { return min(max(j, glo), ghi - 1); };
    const int xl = xin ? x : (x < 0 ? 0 : P - 2);
    auto ldu = [&](int j) { return load_row<2, true>(uo + (long)cl(j) * P, xl); };
    // one row of gradients with the denominator (alpha^2 + gx^2) + gy^2
    // (OpticalFlowDiffusion.cpp:78), which the three steps share
    struct G {
        Row<2> g;
        float t[2], den[2], rcp[2];
    };
    // the gradient field is in the unscaled-division range (hs_precheck_kernel)
    const bool grange = range_flag && *range_flag == 0;
    // GI: raw rows of Iaux and It
    auto ldia = [&](int j) {
        return ld2<false>(reinterpret_cast<const float2 *>(Ia + (long)cl(j) * P + xl));
    };
    auto ldit = [&](int j) {
        return ld2<false>(reinterpret_cast<const float2 *>(It + (long)cl(j) * P + xl));
    };
    auto ldg = [&](int j) {
        G r;
        r.g = load_row<2, false>(dI + (long)cl(j) * P, xl);
        const float2 tt = ld2<false>(reinterpret_cast<const float2 *>(It + (long)cl(j) * P + xl));
        r.t[0] = tt.x;
        r.t[1] = tt.y;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            r.den[k] = (alphasq + r.g.v[k].x * r.g.v[k].x) + r.g.v[k].y * r.g.v[k].y;
            r.rcp[k] = recip_refined(r.den[k]);
        }
        return r;
    };
    // any lane of this wave on an x-border pixel: wave-uniform
    const bool xedge_w = __builtin_amdgcn_ballot_w64(x == 0 || x == dimx - 1 || x + 1 == 0 ||
                                                     x + 1 == dimx - 1) != 0;
    // GI: the gradient row of j-line j from the Iaux rows j-1 (im), j (ic),
    // j+1 (ip) and the It row (t); the border rule of gradients.h:9-32 with
    // the global j
    auto mkg = [&](int j, float2 im, float2 ic, float2 ip, float2 t) {
        G r;
        const float lft = dpp_from_left(ic.y);   // Iaux[x - 1]
        const float rgt = dpp_from_right(ic.x);  // Iaux[x + 2]
        // partial_x: (f[i+1] - f[i-1]) / 2.0f, one-sided at i = 0 / dimx - 1
        float gx0 = (ic.y - lft) / 2.0f, gx1 = (rgt - ic.x) / 2.0f;
        if (xedge_w) {
            if (x == 0)
                gx0 = ic.y - ic.x;
            else if (x == dimx - 1)
                gx0 = ic.x - lft;
            if (x + 1 == dimx - 1) gx1 = ic.y - ic.x;
        }
        // partial_y with the global j-line (wave-uniform)
        const int jg = row0 + j;
        float gy0, gy1;
        if (jg == 0) {
            gy0 = ip.x - ic.x;
            gy1 = ip.y - ic.y;
        } else if (jg == dimy - 1) {
            gy0 = ic.x - im.x;
            gy1 = ic.y - im.y;
        } else {
            gy0 = (ip.x - im.x) / 2.0f;
            gy1 = (ip.y - im.y) / 2.0f;
        }
        r.g.v[0] = make_float2(gx0, gy0);
        r.g.v[1] = make_float2(gx1, gy1);
        r.t[0] = t.x;
        r.t[1] = t.y;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            r.den[k] = (alphasq + r.g.v[k].x * r.g.v[k].x) + r.g.v[k].y * r.g.v[k].y;
            r.rcp[k] = recip_refined(r.den[k]);
        }
        return r;
    };
    auto stepr_opt = [&](int j, const Row<2> &m, const Row<2> &c, const Row<2> &p, const G &g) {
        // (l + r) per component with the lane shift folded into the add
        // (the empty asm keeps the SLP vectorizer from pairing x and y into a
        // packed add, which has no DPP form; the adds then absorb the moves)
        float sx0 = dpp_from_left(c.v[1].x) + c.v[1].x;
        float sy0 = dpp_from_left(c.v[1].y) + c.v[1].y;
        float sx1 = dpp_from_right(c.v[0].x) + c.v[0].x;
        float sy1 = dpp_from_right(c.v[0].y) + c.v[0].y;
        asm("" : "+v"(sx0), "+v"(sy0), "+v"(sx1), "+v"(sy1));
        const int jg = row0 + j;
        const bool yb = (jg == 0) || (jg == dimy - 1);
        v2f q[2];
        q[0] = ((v2f{sx0, sy0} + v2f{m.v[0].x, m.v[0].y}) + v2f{p.v[0].x, p.v[0].y}) / 4.0f;
        q[1] = ((v2f{sx1, sy1} + v2f{m.v[1].x, m.v[1].y}) + v2f{p.v[1].x, p.v[1].y}) / 4.0f;
        if (yb || xedge_w) {
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int xi = x + k;
                const float2 z = zero_if(yb || xi == 0 || xi == dimx - 1, make_float2(q[k].x, q[k].y));
                q[k] = v2f{z.x, z.y};
            }
        }
        float sc[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const v2f pr = q[k] * v2f{g.g.v[k].x, g.g.v[k].y};
            sc[k] = (g.t[k] + pr.x) + pr.y;
        }
        Row<2> o;
        const float mn = fminf(fabsf(sc[0]), fabsf(sc[1])), mx = fmaxf(fabsf(sc[0]), fabsf(sc[1]));
        if (grange && __builtin_amdgcn_ballot_w64(!(mn >= 0x1p-50f && mx < 0x1p30f)) == 0) {
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const float gx = g.g.v[k].x, gy = g.g.v[k].y;
                const float2 f = div2_unscaled(gx * sc[k], gy * sc[k], g.den[k], g.rcp[k]);
                o.v[k] = make_float2(q[k].x - f.x, q[k].y - f.y);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const float gx = g.g.v[k].x, gy = g.g.v[k].y;
                const float fx = gx * sc[k], fy = gy * sc[k];
                o.v[k] = make_float2(q[k].x - fx / g.den[k], q[k].y - fy / g.den[k]);
            }
        }
        return o;
    };
    // the triple kernel needs no per-pixel zero test: hs_precheck_kernel made
    // it once for the field (dI is fixed), so the flag word stays unused
    auto stepr = [&](int j, const Row<2> &m, const Row<2> &c, const Row<2> &p, const G &g,
                     unsigned &) { return stepr_opt(j, m, c, p, g); };
    const bool in1 = x + 1 < dimx;
    auto mag = [](float a, float b) { return __builtin_amdgcn_sqrtf(a * a + b * b); };
    auto norms = [&](const Row<2> &nw, const Row<2> &od, float &sd, float &sp) {
        sd += mag(nw.v[0].x - od.v[0].x, nw.v[0].y - od.v[0].y);
        sp += mag(od.v[0].x, od.v[0].y);
        const float d1 = mag(nw.v[1].x - od.v[1].x, nw.v[1].y - od.v[1].y);
        const float p1 = mag(od.v[1].x, od.v[1].y);
        sd += in1 ? d1 : 0.0f;  // a select, not a product: padding may hold 0/0
        sp += in1 ? p1 : 0.0f;
    };
    // one band, marched in direction D (+1: j-lines jbeg..jend-1, -1: jend-1..jbeg);
    // position s of the march is j-line J(s), "ahead" is the next position
    auto march = [&](auto dirc) __attribute__((always_inline)) {
        constexpr int D = decltype(dirc)::value;
        const int n = jend - jbeg;
        auto J = [&](int sp) { return D > 0 ? jbeg + sp : jend - 1 - sp; };
        // stepr with the j-1 / j+1 rows taken from behind / ahead by direction
        auto S = [&](int sp, const Row<2> &bh, const Row<2> &c, const Row<2> &ah, const G &g,
                     unsigned &b) {
            return D > 0 ? stepr(J(sp), bh, c, ah, g, b) : stepr(J(sp), ah, c, bh, g, b);
        };
        unsigned bx_ = 0;  // halo rows: flagged by the waves that own them
        const Row<2> a0 = ldu(J(-3)), a1 = ldu(J(-2)), a2 = ldu(J(-1));
        Row<2> uj = ldu(J(0)), uj1 = ldu(J(1)), uj2 = ldu(J(2));
        // GI: the gradient row at position sp from the Iaux rows at positions
        // sp-1 (behind), sp, sp+1 (ahead), in j order by direction
        auto MG = [&](int sp, float2 bh, float2 c, float2 ah, float2 t) {
            return D > 0 ? mkg(J(sp), bh, c, ah, t) : mkg(J(sp), ah, c, bh, t);
        };
        G gm2, gm1, gj, gj1;
        float2 i1, i2, i3, nt;  // GI: Iaux at positions sp+1, sp+2, sp+3; It at sp+2
        if constexpr (GI) {
            const float2 im3 = ldia(J(-3)), im2 = ldia(J(-2)), im1 = ldia(J(-1)),
                         i0 = ldia(J(0));
            i1 = ldia(J(1));
            i2 = ldia(J(2));
            gm2 = MG(-2, im3, im2, im1, ldit(J(-2)));
            gm1 = MG(-1, im2, im1, i0, ldit(J(-1)));
            gj = MG(0, im1, i0, i1, ldit(J(0)));
            gj1 = MG(1, i0, i1, i2, ldit(J(1)));
        } else {
            gm2 = ldg(J(-2));
            gm1 = ldg(J(-1));
            gj = ldg(J(0));
            gj1 = ldg(J(1));
        }
        // u1 at positions -2 .. 1, u2 at -1, 0
        const Row<2> p0 = S(-2, a0, a1, a2, gm2, bx_);
        const Row<2> p1 = S(-1, a1, a2, uj, gm1, bx_);
        Row<2> vj = S(0, a2, uj, uj1, gj, bx_);
        Row<2> vj1 = S(1, uj, uj1, uj2, gj1, bx_);
        Row<2> wm1 = S(-1, p0, p1, vj, gm1, bx_);
        Row<2> wj = S(0, p1, vj, vj1, gj, bx_);
        // an owned row of an intermediate iterate (MID)
        auto stmid = [&](float2 *m, int sp, const Row<2> &v) __attribute__((always_inline)) {
            float2 *dst = m + (long)J(sp) * P + x;
            if (x + 2 <= dimx)
                st4<OF2D_HS_MID_NT != 0>(reinterpret_cast<float4 *>(dst),
                                         make_float4(v.v[0].x, v.v[0].y, v.v[1].x, v.v[1].y));
            else
                dst[0] = v.v[0];
        };
        if constexpr (MID) {
            if (own) {
                stmid(m1, 0, vj);
                if (n > 1) stmid(m1, 1, vj1);
                stmid(m2, 0, wj);
            }
        }
        Row<2> nu = ldu(J(3));
        G ng;
        if constexpr (GI) {
            i3 = ldia(J(3));
            nt = ldit(J(2));
        } else {
            ng = ldg(J(2));
        }
        // one output row; the window shifts by renaming, which the unrolled
        // copies below turn into register renames instead of moves
        auto body = [&](int sp, bool pref) __attribute__((always_inline)) {
            const Row<2> a3 = nu;  // u at position sp+3
            G gj2;                 // gradients at position sp+2
            if constexpr (GI) {
                gj2 = MG(sp + 2, i1, i2, i3, nt);
                i1 = i2;
                i2 = i3;
            } else {
                gj2 = ng;
            }
            if (pref) {
                nu = ldu(J(sp + 4));
                if constexpr (GI) {
                    i3 = ldia(J(sp + 4));
                    nt = ldit(J(sp + 3));
                } else {
                    ng = ldg(J(sp + 3));
                }
            }
            unsigned b1 = 0, b3 = 0;
            const Row<2> vj2 = S(sp + 2, uj1, uj2, a3, gj2, b1);  // u1
            const Row<2> wj1 = S(sp + 1, vj, vj1, vj2, gj1, b1);  // u2
            const Row<2> z = S(sp, wm1, wj, wj1, gj, b3);         // u3
            if (MID && own) {
                if (sp + 2 < n) stmid(m1, sp + 2, vj2);
                if (sp + 1 < n) stmid(m2, sp + 1, wj1);
            }
            if (own) {
                if constexpr (!MID) {  // MID: the exact Logger takes its own norms
                    norms(vj, uj, s1d, s1p);
                    norms(wj, vj, s2d, s2p);
                    norms(z, wj, s3d, s3p);
                }
                bad |= b3;  // the denominator depends on dI only: one test per pixel
                float2 *dst = un + (long)J(sp) * P + x;
                if (x + 2 <= dimx)
                    st4<true>(reinterpret_cast<float4 *>(dst),
                              make_float4(z.v[0].x, z.v[0].y, z.v[1].x, z.v[1].y));
                else
                    dst[0] = z.v[0];
            }
            uj = uj1;
            uj1 = uj2;
            uj2 = a3;
            vj = vj1;
            vj1 = vj2;
            wm1 = wj;
            wj = wj1;
            gj = gj1;
            gj1 = gj2;
        };
        int sp = 0;
        for (; sp + UNR < n; sp += UNR) {
            progress_prio<PRIO>(sp, n);
#pragma unroll
            for (int k = 0; k < UNR; k++) body(sp + k, true);
        }
        for (; sp < n; ++sp) body(sp, sp + 1 < n);
    };
    if (jbeg < jend) {
        if (ALT && (wave & 1))
            march(std::integral_constant<int, -1>{});
        else
            march(std::integral_constant<int, 1>{});
    }
    if constexpr (MID) {  // no Logger partials (seqnorm_kernels.hip takes the norms)
        if (__any(bad) && lane == 0) atomicOr(status, kStatusDivZero);
        return;
    }
    double d1d = s1d, d1p = s1p, d2d = s2d, d2p = s2p, d3d = s3d, d3p = s3p;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        d1d += __shfl_down(d1d, off);
        d1p += __shfl_down(d1p, off);
        d2d += __shfl_down(d2d, off);
        d2p += __shfl_down(d2p, off);
        d3d += __shfl_down(d3d, off);
        d3p += __shfl_down(d3p, off);
    }
    __shared__ double red[6][WAVES];
    if (lane == 0) {
        red[0][wave] = d1d;
        red[1][wave] = d1p;
        red[2][wave] = d2d;
        red[3][wave] = d2p;
        red[4][wave] = d3d;
        red[5][wave] = d3p;
    }
    if (__any(bad) && lane == 0) atomicOr(status, kStatusDivZero);
    __syncthreads();
    if (threadIdx.x == 0) {
        double r[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < WAVES; ++w)
#pragma unroll
            for (int q = 0; q < 6; q++) r[q] += red[q][w];
        const long blk = (long)band * gx + bx;
        partial[2 * blk] = r[0];
        partial[2 * blk + 1] = r[1];
        partial2[2 * blk] = r[2];
        partial2[2 * blk + 1] = r[3];
        partial3[2 * blk] = r[4];
        partial3[2 * blk + 1] = r[5];
    }
}

template <int ROWS, int WAVES, bool XCD = true, int MINB = 1, int UNR = 4, int PRIO = 0,
          bool ALT = false, bool GI = false>
__global__ __launch_bounds__(64 * WAVES, MINB) void jacobi3_kernel(
    const float2 *__restrict__ uo, float2 *__restrict__ un, const float2 *__restrict__ dI,
    const float *__restrict__ It, int P, int dimx, int nrows, int row0, int dimy, float alphasq,
    int glo, int ghi, double *__restrict__ partial, double *__restrict__ partial2,
    double *__restrict__ partial3, unsigned *__restrict__ status, int band0, int gx, int gy,
    int rows = ROWS, const unsigned *__restrict__ range_flag = nullptr, int jlo = -1,
    int jhi = -1, const float *__restrict__ Ia = nullptr) {
    jacobi3_body<ROWS, WAVES, XCD, MINB, UNR, PRIO, ALT, GI, false>(
        uo, un, dI, It, P, dimx, nrows, row0, dimy, alphasq, glo, ghi, partial, partial2, partial3,
        status, band0, gx, gy, rows, range_flag, jlo, jhi, Ia, nullptr, nullptr);
}
// the same storing the intermediate iterates u1, u2 to m1, m2 (MID)
template <int ROWS, int WAVES, bool XCD = true, int MINB = 1, int UNR = 4, int PRIO = 0,
          bool ALT = false, bool GI = false>
__global__ __launch_bounds__(64 * WAVES, MINB) void jacobi3_mid_kernel(
    const float2 *__restrict__ uo, float2 *__restrict__ un, const float2 *__restrict__ dI,
    const float *__restrict__ It, int P, int dimx, int nrows, int row0, int dimy, float alphasq,
    int glo, int ghi, double *__restrict__ partial, double *__restrict__ partial2,
    double *__restrict__ partial3, unsigned *__restrict__ status, int band0, int gx, int gy,
    int rows, const unsigned *__restrict__ range_flag, int jlo, int jhi,
    const float *__restrict__ Ia, float2 *__restrict__ m1, float2 *__restrict__ m2,
    const int *__restrict__ stop, int stop_t0) {
    // the loop broke before this triple's first iteration (seqnorm_decide):
    // nothing of it is read
    if (stop && *stop < stop_t0) return;
    jacobi3_body<ROWS, WAVES, XCD, MINB, UNR, PRIO, ALT, GI, true>(
        uo, un, dI, It, P, dimx, nrows, row0, dimy, alphasq, glo, ghi, partial, partial2, partial3,
        status, band0, gx, gy, rows, range_flag, jlo, jhi, Ia, m1, m2);
}

template <int ROWS, int WAVES>
inline dim3 grid3_for(int dimx, int nrows) {
    return dim3((dimx + kHs3Out - 1) / kHs3Out, (nrows + ROWS * WAVES - 1) / (ROWS * WAVES));
}

template <int ROWS, int WAVES, int PXL = 2>
inline dim3 grid2_for(int dimx, int nrows) {
    return dim3((dimx + hs2_out<PXL>() - 1) / hs2_out<PXL>(),
                (nrows + ROWS * WAVES - 1) / (ROWS * WAVES));
}

template <int ROWS, int PXL, int WAVES>
inline dim3 grid_for(int P, int nrows) {
    return dim3(P / (64 * PXL), (nrows + ROWS * WAVES - 1) / (ROWS * WAVES));
}

}  // namespace hs
}  // namespace of2d
