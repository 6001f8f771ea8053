// curvature_kernels.hip — OpticalFlowCurvature::get_update on gfx950.
//
// OpticalFlowCurvature.cpp:149-167: rhs = u - tau * f (float, stored as
// double), a 2-D DCT-II (FFTW REDFT10 on both axes), multiplication by the
// eigenvalues of (1 + tau*alpha*L^2) (:6-30), a 2-D DCT-III (REDFT01), and
// u = (float)rhs / (4.0f * n) (:106-125).
//
// FFTW is absent from this image, so the transforms are the r2r definitions
// themselves, evaluated as fp64 GEMMs against cosine matrices on the MFMA
// units (v_mfma_f64_16x16x4_f64):
//   forward  T = X C1^T (axis y),  Y = (C0 T) .* E (axis x, eigenvalues fused)
//   inverse  S = Y D1^T,           Z = D0 S
// with X the rhs as a column-major dimx x dimy matrix (element (i, j) at
// i + j*ld, i.e. the pitched field layout) and C/D the REDFT10/REDFT01
// matrices.  The axis order is the oracle's (y first).  fp64 throughout, so
// the only departure from FFTW is the summation order (parity at tolerance).
#include "of2d_device.h"

namespace of2d {

namespace {
typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int kGT = 64;   // block tile (M and N)
constexpr int kGK = 16;   // K per LDS stage
constexpr int kLdsPad = 2;  // doubles of padding per LDS row
}  // namespace

// C[m + n*ldc] = sum_k A[m + k*lda] * B[k + n*ldb]  (column-major), times
// E[m + n*lde] when E != nullptr; batch z offsets A, B, C by their strides.
// 4 waves in 2 x 2, each wave a 32 x 32 sub-tile of 2 x 2 MFMA tiles.  The
// MFMA is fed B^T as its A operand and A^T as its B operand, so the result
// comes out transposed: accumulator r of lane l is row m = l % 16 of column
// n = l / 16 + 4r (checked by tools/dgemm_check.hip), and a store of 16 lanes
// is one 128-B column segment.
__global__ __launch_bounds__(256) void dgemm_nn_kernel(int M, int N, int K,
                                                       const double *__restrict__ A, long lda,
                                                       long sA, const double *__restrict__ B,
                                                       long ldb, long sB, double *__restrict__ C,
                                                       long ldc, long sC,
                                                       const double *__restrict__ E, long lde) {
    __shared__ double As[kGK][kGT + kLdsPad];  // As[k][m]
    __shared__ double Bs[kGK][kGT + kLdsPad];  // Bs[k][n]
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int m0 = blockIdx.x * kGT, n0 = blockIdx.y * kGT;
    A += blockIdx.z * sA;
    B += blockIdx.z * sB;
    C += blockIdx.z * sC;
    v4d acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = v4d{0.0, 0.0, 0.0, 0.0};

    // global -> LDS assignment: A: m = t % 64, k = t / 64 + 4q; B: k = t % 16, n = t / 16 + 16q
    const int am = t & 63, ak = t >> 6;
    const int bk = t & 15, bn = t >> 4;
    for (int k0 = 0; k0 < K; k0 += kGK) {
        double ra[4], rb[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int m = m0 + am, k = k0 + ak + 4 * q;
            ra[q] = (m < M && k < K) ? A[m + (long)k * lda] : 0.0;
            const int kb = k0 + bk, n = n0 + bn + 16 * q;
            rb[q] = (kb < K && n < N) ? B[kb + (long)n * ldb] : 0.0;
        }
        __syncthreads();  // previous stage's reads are done
#pragma unroll
        for (int q = 0; q < 4; q++) {
            As[ak + 4 * q][am] = ra[q];
            Bs[bk][bn + 16 * q] = rb[q];
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < kGK / 4; ks++) {
            const int kk = 4 * ks + (lane >> 4);
            double fa[2], fb[2];
#pragma unroll
            for (int a = 0; a < 2; a++) fa[a] = As[kk][wm * 32 + a * 16 + (lane & 15)];
#pragma unroll
            for (int b = 0; b < 2; b++) fb[b] = Bs[kk][wn * 32 + b * 16 + (lane & 15)];
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(fb[b], fa[a], acc[a][b], 0, 0, 0);
        }
    }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = m0 + wm * 32 + a * 16 + (lane & 15);
                const int n = n0 + wn * 32 + b * 16 + (lane >> 4) + 4 * r;
                if (m < M && n < N) {
                    double v = acc[a][b][r];
                    if (E) v *= E[m + (long)n * lde];
                    C[m + (long)n * ldc] = v;
                }
            }
}

void launch_dgemm(int M, int N, int K, const double *A, long lda, long sA, const double *B,
                  long ldb, long sB, double *C, long ldc, long sC, const double *E, long lde,
                  int batch, hipStream_t st) {
    const dim3 g((M + kGT - 1) / kGT, (N + kGT - 1) / kGT, batch);
    hipLaunchKernelGGL(dgemm_nn_kernel, g, dim3(256), 0, st, M, N, K, A, lda, sA, B, ldb, sB, C,
                       ldc, sC, E, lde);
    OF2D_HIP(hipGetLastError());
}

// rhs = u - tau * f with f = dI * ((It + u.x dI.x) + u.y dI.y) (OpticalFlow.cpp:15-39,
// OpticalFlowCurvature.cpp:75-97): float arithmetic, stored as double planes x | y
__global__ void curv_rhs_kernel(const float2 *__restrict__ u, const float2 *__restrict__ dI,
                                const float *__restrict__ It, float tau, int dimx, int dimy,
                                int P, double *__restrict__ X, long plane) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    if (i >= dimx || j >= dimy) return;
    const long idx = (long)j * P + i;
    const float2 m = u[idx], g = dI[idx];
    const float sc = (It[idx] + m.x * g.x) + m.y * g.y;
    const float fx = g.x * sc, fy = g.y * sc;
    X[idx] = (double)(m.x - tau * fx);
    X[plane + idx] = (double)(m.y - tau * fy);
}
void launch_curv_rhs(const float2 *u, const float2 *dI, const float *It, float tau, int dimx,
                     int dimy, int P, double *X, long plane, hipStream_t st) {
    hipLaunchKernelGGL(curv_rhs_kernel, dim3((dimx + 63) / 64, (dimy + 3) / 4), dim3(64, 4), 0,
                       st, u, dI, It, tau, dimx, dimy, P, X, plane);
    OF2D_HIP(hipGetLastError());
}

// u' = vector2d(Z.x, Z.y) / (4.0f * n) (OpticalFlowCurvature.cpp:106-125: the
// double -> float conversion, then coord2d::operator/ in float), plus the
// Logger partials sum ||u' - u||, sum ||u|| per 64 x 4 block
__global__ __launch_bounds__(256) void curv_construct_kernel(const double *__restrict__ Z,
                                                             long plane,
                                                             const float2 *__restrict__ u,
                                                             float2 *__restrict__ out, float div,
                                                             int dimx, int dimy, int P,
                                                             double *__restrict__ partial) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    double sd = 0.0, sp = 0.0;
    if (i < dimx && j < dimy) {
        const long idx = (long)j * P + i;
        const float2 n = make_float2((float)Z[idx] / div, (float)Z[plane + idx] / div);
        const float2 o = u[idx];
        out[idx] = n;
        const float ex = n.x - o.x, ey = n.y - o.y;
        sd = (double)__builtin_sqrtf(ex * ex + ey * ey);
        sp = (double)__builtin_sqrtf(o.x * o.x + o.y * o.y);
    }
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
int curv_nblocks(int dimx, int dimy) { return ((dimx + 63) / 64) * ((dimy + 3) / 4); }
void launch_curv_construct(const double *Z, long plane, const float2 *u, float2 *out, float div,
                           int dimx, int dimy, int P, double *partial, hipStream_t st) {
    hipLaunchKernelGGL(curv_construct_kernel, dim3((dimx + 63) / 64, (dimy + 3) / 4), dim3(64, 4),
                       0, st, Z, plane, u, out, div, dimx, dimy, P, partial);
    OF2D_HIP(hipGetLastError());
}

}  // namespace of2d
