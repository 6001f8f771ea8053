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
#include <algorithm>

#include "hs_jacobi_impl.h"

namespace of2d {

// Tuned on MI355X with tools/hs_variants.hip (profiles/r01_hs_variants.log):
// 32 j-lines per wave, 2 px per lane, 4 waves per block, non-temporal loads of
// u (read once, not reused before it is overwritten) and non-temporal stores of
// u'; dI / It keep the default cache policy.
using HsKernel = decltype(&hs::jacobi_kernel<kHsRows, kHsPxl, kHsWaves, true, true, false>);
static const HsKernel kHsJacobi = &hs::jacobi_kernel<kHsRows, kHsPxl, kHsWaves, true, true, false>;

// Two iterations per launch (tools/hs_variants.hip "two": 32 j-lines, 4 waves
// fastest; 51 us per iteration against 79 us for the single step at 4096^2).
// XCD-aware block order (1-D launch grid remapped in the kernel): ~2 % faster
static const auto kHsJacobi2 = &hs::jacobi2_kernel<kHs2Rows, kHs2Waves, 2, true>;
static_assert(kHs2Out == hs::hs2_out<2>(), "hs2_grid and the kernel disagree on the strip");

void launch_hs_jacobi2(const float2 *u_old, float2 *u_new, const float2 *dI, const float *It,
                       int P, int dimx, int nrows, int row0, int dimy, float alphasq, int glo,
                       int ghi, double *partial, double *partial2, unsigned *status,
                       hipStream_t st, int band_lo, int band_hi) {
    if (P % kHsStrip != 0 || nrows <= 0 || dimx > P || dimx < 2 || glo > -1 || ghi < nrows + 1)
        throw std::invalid_argument("launch_hs_jacobi2: bad geometry");
    const int nb = hs2_nbands(nrows);
    if (band_lo < 0) band_lo = 0;
    if (band_hi < 0) band_hi = nb;
    if (band_lo > band_hi || band_hi > nb) throw std::invalid_argument("launch_hs_jacobi2: bands");
    if (band_lo == band_hi) return;
    dim3 g = hs2_grid(dimx, nrows);
    g.y = band_hi - band_lo;
    const dim3 gl(8 * ((g.x * g.y + 7) / 8));
    hipLaunchKernelGGL(kHsJacobi2, gl, dim3(64 * kHs2Waves), 0, st, u_old, u_new, dI, It, P,
                       dimx, nrows, row0, dimy, alphasq, glo, ghi, partial, partial2, status,
                       band_lo, (int)g.x, (int)g.y);
    OF2D_HIP(hipGetLastError());
}

// 4 resident 4-wave blocks per CU (<= 128 VGPRs), loop unrolled 4x, unscaled
// exact division where its range holds, issue priority by progress (the four
// waves of a SIMD finish together: 89.8 -> 83.6 us per launch at 4096^2,
// tools/hs_variants prio), fewer VALU per row step (border masks behind a
// wave-uniform branch, DPP folded into adds) and alternating
// march directions, so the waves on either side of a band boundary read its
// halo j-lines together (83.8 -> 82.9 us, tools/hs_variants opt)
static const auto kHsJacobi3 = &hs::jacobi3_kernel<0, kHs3Waves, true, 4, 4, 1, true>;
// the same with the gradients derived from Iaux in the kernel (GI: 24 B/px)
static const auto kHsJacobi3I = &hs::jacobi3_kernel<0, kHs3Waves, true, 4, 4, 1, true, true>;
// both, storing the intermediate iterates too (MID: +16 B/px)
static const auto kHsJacobi3M = &hs::jacobi3_mid_kernel<0, kHs3Waves, true, 4, 4, 1, true, false>;
static const auto kHsJacobi3IM = &hs::jacobi3_mid_kernel<0, kHs3Waves, true, 4, 4, 1, true, true>;

void launch_hs_jacobi3(const float2 *u_old, float2 *u_new, const float2 *dI, const float *It,
                       int P, int dimx, int nrows, int row0, int dimy, float alphasq, int glo,
                       int ghi, double *partial, double *partial2, double *partial3,
                       unsigned *status, const unsigned *range_flag, hipStream_t st,
                       int band_lo, int band_hi, const float *Ia, float2 *u1, float2 *u2,
                       const int *stop, int stop_t0, int slots) {
    if (P % kHsStrip != 0 || nrows <= 0 || dimx > P || dimx < 2 || glo > -1 || ghi < nrows + 1)
        throw std::invalid_argument("launch_hs_jacobi3: bad geometry");
    if (!u1 != !u2) throw std::invalid_argument("launch_hs_jacobi3: u1 and u2 go together");
    if (!range_flag) throw std::invalid_argument("launch_hs_jacobi3: no range flag");
    const int rows = hs3_rows(dimx, nrows, slots);
    const int nb = (nrows + kHs3Waves * rows - 1) / (kHs3Waves * rows);
    if (band_lo < 0) band_lo = 0;
    if (band_hi < 0) band_hi = nb;
    if (band_lo > band_hi || band_hi > nb) throw std::invalid_argument("launch_hs_jacobi3: bands");
    if (band_lo == band_hi) return;
    dim3 g((dimx + kHs3Out - 1) / kHs3Out, nb);
    g.y = band_hi - band_lo;
    const dim3 gl(8 * ((g.x * g.y + 7) / 8));
    if (u1)
        hipLaunchKernelGGL(Ia ? kHsJacobi3IM : kHsJacobi3M, gl, dim3(64 * kHs3Waves), 0, st, u_old,
                           u_new, dI, It, P, dimx, nrows, row0, dimy, alphasq, glo, ghi, partial,
                           partial2, partial3, status, band_lo, (int)g.x, (int)g.y, rows,
                           range_flag, -1, -1, Ia, u1, u2, stop, stop_t0);
    else
        hipLaunchKernelGGL(Ia ? kHsJacobi3I : kHsJacobi3, gl, dim3(64 * kHs3Waves), 0, st, u_old,
                           u_new, dI, It, P, dimx, nrows, row0, dimy, alphasq, glo, ghi, partial,
                           partial2, partial3, status, band_lo, (int)g.x, (int)g.y, rows,
                           range_flag, -1, -1, Ia);
    OF2D_HIP(hipGetLastError());
}

int launch_hs_jacobi3_window(const float2 *u_old, float2 *u_new, const float2 *dI,
                             const float *It, int P, int dimx, int nrows, int row0, int dimy,
                             float alphasq, int glo, int ghi, int jlo, int jhi,
                             int rows_per_wave, int slot_band0, double *partial,
                             double *partial2, double *partial3, unsigned *status,
                             const unsigned *range_flag, hipStream_t st, const float *Ia) {
    if (P % kHsStrip != 0 || nrows <= 0 || dimx > P || dimx < 2 || glo > -1 || ghi < nrows + 1 ||
        jlo < 0 || jhi > nrows || jlo >= jhi || rows_per_wave < 1 || slot_band0 < 0)
        throw std::invalid_argument("launch_hs_jacobi3_window: bad geometry");
    if (!range_flag) throw std::invalid_argument("launch_hs_jacobi3_window: no range flag");
    const int gx = (dimx + kHs3Out - 1) / kHs3Out;
    const int per_band = kHs3Waves * rows_per_wave;
    const int gy = (jhi - jlo + per_band - 1) / per_band;
    const dim3 gl(8 * ((gx * gy + 7) / 8));
    hipLaunchKernelGGL(Ia ? kHsJacobi3I : kHsJacobi3, gl, dim3(64 * kHs3Waves), 0, st, u_old,
                       u_new, dI, It, P, dimx, nrows, row0, dimy, alphasq, glo, ghi, partial,
                       partial2, partial3, status, slot_band0, gx, gy, rows_per_wave, range_flag,
                       jlo, jhi, Ia);
    OF2D_HIP(hipGetLastError());
    return gy;
}

void launch_hs_precheck(const float2 *base, size_t count, int P, int ghost, int dimx, int dimy,
                        float alphasq, unsigned *range_flag, unsigned *status, hipStream_t st) {
    OF2D_HIP(hipMemsetAsync(range_flag, 0, sizeof(unsigned), st));
    const long n = (long)count;
    const unsigned blocks = (unsigned)std::min<long>(2048, (n + 255) / 256);
    hipLaunchKernelGGL(hs::hs_precheck_kernel<>, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st,
                       base, n, P, ghost, dimx, dimy, alphasq, range_flag, status);
    OF2D_HIP(hipGetLastError());
}

void launch_hs_jacobi(const float2 *u_old, float2 *u_new, const float2 *dI, const float *It,
                      int P, int dimx, int nrows, int row0, int dimy, float alphasq,
                      double *partial, unsigned *status, hipStream_t st) {
    if (P % kHsStrip != 0 || nrows <= 0 || dimx > P)
        throw std::invalid_argument("launch_hs_jacobi: bad geometry");
    hipLaunchKernelGGL(kHsJacobi, hs_grid(P, nrows), dim3(64 * kHsWaves), 0, st, u_old, u_new,
                       dI, It, P, dimx, nrows, row0, dimy, alphasq, partial, status);
    OF2D_HIP(hipGetLastError());
}

// partial: [C][nblocks][2]; one 1024-thread block per iteration, fixed
// summation order (strided per-thread sums, wave trees, then the 16 waves in
// order).
__global__ __launch_bounds__(1024) void reduce_partials_kernel(const double *__restrict__ partial,
                                                               int stride, int nblocks,
                                                               double *__restrict__ sums) {
    const double *p = partial + (size_t)blockIdx.x * stride * 2;
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nblocks; i += 1024) {
        a += p[2 * i];
        b += p[2 * i + 1];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        b += __shfl_down(b, off);
    }
    __shared__ double red[2][16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wave] = a;
        red[1][wave] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; w++) {
            a += red[0][w];
            b += red[1][w];
        }
        sums[2 * blockIdx.x] = a;
        sums[2 * blockIdx.x + 1] = b;
    }
}

void launch_reduce_partials(const double *partial, int nblocks, int C, double *sums,
                            hipStream_t st, int stride) {
    if (C <= 0) return;
    if (stride < 0) stride = nblocks;
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(C), dim3(1024), 0, st, partial, stride,
                       nblocks, sums);
    OF2D_HIP(hipGetLastError());
}

namespace {
struct RankPtrs {
    const double *p[kMaxLocalRanks];
};
}  // namespace
__global__ void sum_ranks_kernel(RankPtrs src, int n, long count, double *__restrict__ out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    double a = src.p[0][i];
    for (int r = 1; r < n; r++) a += src.p[r][i];
    out[i] = a;
}
void launch_sum_ranks(const double *const *src, int n, size_t count, double *out,
                      hipStream_t st) {
    if (n < 1 || n > kMaxLocalRanks) throw std::invalid_argument("launch_sum_ranks: n");
    if (count == 0) return;
    RankPtrs p{};
    for (int r = 0; r < n; r++) p.p[r] = src[r];
    hipLaunchKernelGGL(sum_ranks_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st,
                       p, n, (long)count, out);
    OF2D_HIP(hipGetLastError());
}

// halo j-lines between slabs of one device (slab.cpp local_exchange): 16-B
// words, a few blocks, so that the copy finds CU slots beside the triples at
// once (the runtime's copy kernel is 256 blocks: 24 us per 98 KB copy beside
// 8 ranks' triples, profiles/r05f_ranks_attribution.txt)
__global__ __launch_bounds__(256) void copy_lines_kernel(const float2 *__restrict__ src,
                                                         float2 *__restrict__ dst, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        dst[i] = src[i];
}
void launch_copy_lines(void *dst, const void *src, size_t bytes, hipStream_t st) {
    if (bytes % 8 != 0 || (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) % 8)
        throw std::invalid_argument("launch_copy_lines: 8-B aligned whole float2s");
    const long n = (long)(bytes / 8);
    if (n == 0) return;
    const unsigned blocks = (unsigned)std::min<long>(16, (n + 255) / 256);
    hipLaunchKernelGGL(copy_lines_kernel, dim3(blocks), dim3(256), 0, st,
                       static_cast<const float2 *>(src), static_cast<float2 *>(dst), n);
    OF2D_HIP(hipGetLastError());
}

void PartialRuns::add(int t, int len, int nblocks) {
    if (!runs.empty() && runs.back().t0 + runs.back().len == t && runs.back().nblocks == nblocks)
        runs.back().len += len;
    else
        runs.push_back({t, len, nblocks});
}
void PartialRuns::reduce(const double *partial, int stride, double *sums, hipStream_t st) const {
    for (const Run &r : runs)
        launch_reduce_partials(partial + (size_t)r.t0 * stride * 2, r.nblocks, r.len,
                               sums + 2 * (size_t)r.t0, st, stride);
}

}  // namespace of2d
