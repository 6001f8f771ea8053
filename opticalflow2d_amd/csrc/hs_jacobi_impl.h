// hs_jacobi_impl.h — the fused Horn-Schunck Jacobi step as a template, shared
// by the product kernel (hs_kernels.hip) and the tuning harness
// (tools/hs_variants.hip).
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
// registers; x-neighbours come from the adjacent lanes by cross-lane shuffles
// (the strip's two edge lanes load one float2 each).  WAVES waves of a block
// march consecutive row bands of the same strip.
#pragma once

#include "of2d_device.h"

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

__device__ __forceinline__ float2 update_px(float2 q, float gx, float gy, float it,
                                            float alphasq, unsigned &bad) {
    const float s = (it + q.x * gx) + q.y * gy;      // OpticalFlow.cpp:33
    const float fx = gx * s, fy = gy * s;            // coord2d * float
    const float den = (alphasq + gx * gx) + gy * gy;  // OpticalFlowDiffusion.cpp:78
    bad |= (den == 0.0f) ? 1u : 0u;                  // coord2d.h:95-100 throws
    return make_float2(q.x - fx / den, q.y - fy / den);
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
            left.x = __shfl_up(uc.v[PXL - 1].x, 1);
            left.y = __shfl_up(uc.v[PXL - 1].y, 1);
            right.x = __shfl_down(uc.v[0].x, 1);
            right.y = __shfl_down(uc.v[0].y, 1);
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
                if (yb || xi == 0 || xi == dimx - 1) q = make_float2(0.0f, 0.0f);  // :73-76
                unsigned b = 0;
                nw[k] = update_px(q, g.v[k].x, g.v[k].y, t[k], alphasq, b);
                if (xi < dimx) {
                    bad |= b;
                    const float ex = nw[k].x - uc.v[k].x, ey = nw[k].y - uc.v[k].y;
                    sdiff += (double)__builtin_sqrtf(ex * ex + ey * ey);
                    sprev += (double)__builtin_sqrtf(uc.v[k].x * uc.v[k].x + uc.v[k].y * uc.v[k].y);
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

template <int ROWS, int PXL, int WAVES>
inline dim3 grid_for(int P, int nrows) {
    return dim3(P / (64 * PXL), (nrows + ROWS * WAVES - 1) / (ROWS * WAVES));
}

}  // namespace hs
}  // namespace of2d
