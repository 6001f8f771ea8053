// hs_kernels.hip — the Horn-Schunck Jacobi step for gfx950 (north-star kernel).
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
// Algorithmic traffic: read u 8 B + dI 8 B + It 4 B, write u' 8 B = 28 B/px.
// Each wave owns a 128-px strip (2 px per lane, 16-B loads) and marches
// kHsRows j-lines down it keeping the rows j-1, j, j+1 of u in registers, so
// every row of u is fetched once per wave (+2 halo rows per kHsRows); the
// x-neighbours come from the adjacent lanes by cross-lane shuffles, only the
// strip's two edge lanes load one extra float2 each.  fp32 arithmetic in the
// reference's order, compiled with -ffp-contract=off (no FMA contraction) and
// IEEE division, so every pixel is bit-identical to the reference.
#include "of2d_device.h"

namespace of2d {

__device__ __forceinline__ float2 hs_update_px(float2 q, float gx, float gy, float it,
                                               float alphasq, unsigned &bad) {
    const float s = (it + q.x * gx) + q.y * gy;      // OpticalFlow.cpp:33
    const float fx = gx * s, fy = gy * s;            // coord2d * float
    const float den = (alphasq + gx * gx) + gy * gy;  // OpticalFlowDiffusion.cpp:78
    bad |= (den == 0.0f) ? 1u : 0u;                  // coord2d.h:95-100 throws
    return make_float2(q.x - fx / den, q.y - fy / den);
}

__global__ __launch_bounds__(256) void hs_jacobi_kernel(
    const float2 *__restrict__ uo, float2 *__restrict__ un, const float2 *__restrict__ dI,
    const float *__restrict__ It, int P, int dimx, int nrows, int row0, int dimy, float alphasq,
    double *__restrict__ partial, unsigned *__restrict__ status) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = blockIdx.x * kHsStrip + 2 * lane;
    const int jbeg = (blockIdx.y * kHsWaves + wave) * kHsRows;
    const int jend = min(jbeg + kHsRows, nrows);

    double sdiff = 0.0, sprev = 0.0;
    unsigned bad = 0;
    if (jbeg < nrows) {
        const long Pq = P >> 1;  // float4 per row
        const long xq = x >> 1;
        const float4 *U = reinterpret_cast<const float4 *>(uo);
        const float4 *G = reinterpret_cast<const float4 *>(dI);
        const float2 *T = reinterpret_cast<const float2 *>(It);
        const bool v0 = x < dimx, v1 = x + 1 < dimx;
        const bool xb0 = (x == 0) || (x == dimx - 1);
        const bool xb1 = (x + 1 == dimx - 1);
        const bool need_l = (lane == 0) && (x > 0) && (x < dimx - 1);
        const bool need_r = (lane == 63) && (x + 2 < dimx);

        float4 um = U[(long)(jbeg - 1) * Pq + xq];  // row -1 is a ghost j-line
        float4 uc = U[(long)jbeg * Pq + xq];
#pragma unroll 4
        for (int j = jbeg; j < jend; ++j) {
            const float4 up = U[(long)(j + 1) * Pq + xq];  // row nrows is a ghost j-line
            const float4 g = G[(long)j * Pq + xq];
            const float2 t = T[((long)j * P + x) >> 1];
            float lx = __shfl_up(uc.z, 1), ly = __shfl_up(uc.w, 1);
            float rx = __shfl_down(uc.x, 1), ry = __shfl_down(uc.y, 1);
            if (need_l) {
                const float2 e = uo[(long)j * P + x - 1];
                lx = e.x;
                ly = e.y;
            }
            if (need_r) {
                const float2 e = uo[(long)j * P + x + 2];
                rx = e.x;
                ry = e.y;
            }
            const int jg = row0 + j;
            const bool yb = (jg == 0) || (jg == dimy - 1);
            // gradients.h:77-79: (((u[i-1] + u[i+1]) + u[j-1]) + u[j+1]) / 4.0f
            float2 q0, q1;
            q0.x = (((lx + uc.z) + um.x) + up.x) / 4.0f;
            q0.y = (((ly + uc.w) + um.y) + up.y) / 4.0f;
            q1.x = (((uc.x + rx) + um.z) + up.z) / 4.0f;
            q1.y = (((uc.y + ry) + um.w) + up.w) / 4.0f;
            if (yb || xb0) q0 = make_float2(0.0f, 0.0f);  // gradients.h:73-76
            if (yb || xb1) q1 = make_float2(0.0f, 0.0f);
            unsigned b0 = 0, b1 = 0;
            const float2 n0 = hs_update_px(q0, g.x, g.y, t.x, alphasq, b0);
            const float2 n1 = hs_update_px(q1, g.z, g.w, t.y, alphasq, b1);
            float2 *dst = un + (long)j * P + x;
            if (v1) {
                *reinterpret_cast<float4 *>(dst) = make_float4(n0.x, n0.y, n1.x, n1.y);
            } else if (v0) {
                *dst = n0;
            }
            if (v0) {
                bad |= b0;
                const float ex = n0.x - uc.x, ey = n0.y - uc.y;
                sdiff += (double)__builtin_sqrtf(ex * ex + ey * ey);
                sprev += (double)__builtin_sqrtf(uc.x * uc.x + uc.y * uc.y);
            }
            if (v1) {
                bad |= b1;
                const float ex = n1.x - uc.z, ey = n1.y - uc.w;
                sdiff += (double)__builtin_sqrtf(ex * ex + ey * ey);
                sprev += (double)__builtin_sqrtf(uc.z * uc.z + uc.w * uc.w);
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
    __shared__ double red[2][kHsWaves];
    if (lane == 0) {
        red[0][wave] = sdiff;
        red[1][wave] = sprev;
    }
    if (__any(bad) && lane == 0) atomicOr(status, kStatusDivZero);
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int w = 0; w < kHsWaves; ++w) {
            a += red[0][w];
            b += red[1][w];
        }
        const long blk = (long)blockIdx.y * gridDim.x + blockIdx.x;
        partial[2 * blk] = a;
        partial[2 * blk + 1] = b;
    }
}

void launch_hs_jacobi(const float2 *u_old, float2 *u_new, const float2 *dI, const float *It,
                      int P, int dimx, int nrows, int row0, int dimy, float alphasq,
                      double *partial, unsigned *status, hipStream_t st) {
    if (P % kHsStrip != 0 || nrows <= 0 || dimx > P)
        throw std::invalid_argument("launch_hs_jacobi: bad geometry");
    hipLaunchKernelGGL(hs_jacobi_kernel, hs_grid(P, nrows), dim3(256), 0, st, u_old, u_new, dI,
                       It, P, dimx, nrows, row0, dimy, alphasq, partial, status);
    OF2D_HIP(hipGetLastError());
}

// partial: [C][nblocks][2]; one block per iteration, fixed summation order.
__global__ __launch_bounds__(256) void reduce_partials_kernel(const double *__restrict__ partial,
                                                              int nblocks,
                                                              double *__restrict__ sums) {
    const double *p = partial + (size_t)blockIdx.x * nblocks * 2;
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nblocks; i += 256) {
        a += p[2 * i];
        b += p[2 * i + 1];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        b += __shfl_down(b, off);
    }
    __shared__ double red[2][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wave] = a;
        red[1][wave] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        sums[2 * blockIdx.x] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        sums[2 * blockIdx.x + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}

void launch_reduce_partials(const double *partial, int nblocks, int C, double *sums,
                            hipStream_t st) {
    if (C <= 0) return;
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(C), dim3(256), 0, st, partial, nblocks, sums);
    OF2D_HIP(hipGetLastError());
}

}  // namespace of2d
