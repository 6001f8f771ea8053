// hs_variants.hip — tuning harness for the HS Jacobi kernel (not part of the
// product).  Times template variants of of2d::hs::jacobi_kernel on a 4096^2
// grid with HIP events, checks every variant bit-identical to the first, and
// times a copy probe with the same traffic mix (read 8+8+4 B, write 8 B per
// px, no stencil) as the achievable ceiling.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 \
//         -I opticalflow2d_amd/csrc tools/hs_variants.hip -o tools/hs_variants
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// wave start / end stamps of the triple kernel (mode "stamps"): 100 MHz
// s_memrealtime, XCC id and HW_ID, one record of 4 words per wave
__device__ unsigned long long *g_stamps = nullptr;
#define OF2D_HS3_STAMP_BEGIN const unsigned long long stamp0_ = __builtin_amdgcn_s_memrealtime();
#define OF2D_HS3_STAMP_END                                                              \
    if (g_stamps && (threadIdx.x & 63) == 0) {                                          \
        const unsigned long long t1_ = __builtin_amdgcn_s_memrealtime();                \
        const unsigned w_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);        \
        g_stamps[4 * w_] = stamp0_;                                                     \
        g_stamps[4 * w_ + 1] = t1_;                                                     \
        g_stamps[4 * w_ + 2] = __builtin_amdgcn_s_getreg((3 << 11) | 20);              \
        g_stamps[4 * w_ + 3] = __builtin_amdgcn_s_getreg((31 << 11) | 4);              \
    }
#include "hs_variants_impl.h"  // the variant zoo (product kernels: csrc/hs_jacobi_impl.h)

using namespace of2d;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void probe_kernel(const float4 *__restrict__ u, const float4 *__restrict__ g,
                             const float2 *__restrict__ t, float4 *__restrict__ o, long n2) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long stride = (long)gridDim.x * blockDim.x;
    for (; i < n2; i += stride) {
        const float4 a = u[i], b = g[i];
        const float2 c = t[i];
        o[i] = make_float4(a.x + b.x * c.x, a.y + b.y, a.z + b.z * c.y, a.w + b.w);
    }
}

struct Bufs {
    float2 *u0, *u1, *dI;
    float *It;
    double *partial;
    unsigned *status;
    unsigned *rflag;  // hs_precheck_kernel's range flag for dI
    int P, dimx, dimy;
};

template <int ROWS, int PXL, int WAVES, bool NTL, bool NTS, bool NTG = NTL>
float run(const Bufs &b, int iters, float2 *out_host, const char *name, double bytes) {
    dim3 g = hs::grid_for<ROWS, PXL, WAVES>(b.P, b.dimy);
    auto k = hs::jacobi_kernel<ROWS, PXL, WAVES, NTL, NTS, NTG>;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    // warm-up
    for (int it = 0; it < 3; it++)
        hipLaunchKernelGGL(k, g, dim3(64 * WAVES), 0, 0, (it & 1) ? b.u1 : b.u0,
                           (it & 1) ? b.u0 : b.u1, b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy,
                           0.01f, b.partial, b.status);
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; it++)
        hipLaunchKernelGGL(k, g, dim3(64 * WAVES), 0, 0, (it & 1) ? b.u1 : b.u0,
                           (it & 1) ? b.u0 : b.u1, b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy,
                           0.01f, b.partial, b.status);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / iters;
    // deterministic check run: 5 iterations from zero
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 5; it++)
        hipLaunchKernelGGL(k, g, dim3(64 * WAVES), 0, 0, (it & 1) ? b.u1 : b.u0,
                           (it & 1) ? b.u0 : b.u1, b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy,
                           0.01f, b.partial, b.status);
    CK(hipMemcpy(out_host, b.u1, sizeof(float2) * (size_t)b.P * b.dimy, hipMemcpyDeviceToHost));
    printf("%-28s grid=%5ux%-4u  %8.2f us  %7.1f GB/s  %5.1f%% of 8 TB/s\n", name, g.x, g.y, us,
           bytes / us / 1e3, bytes / us / 1e3 / 80.0);
    return (float)us;
}

// two iterations per launch (hs::jacobi2_kernel): timed per ITERATION, and
// checked bit for bit against 6 single steps of the product kernel
template <int ROWS, int WAVES, int PXL = 2, bool XCD = false>
int run2(const Bufs &b, int iters, const char *name, double bytes) {
    const dim3 g = hs::grid2_for<ROWS, WAVES, PXL>(b.dimx, b.dimy);
    auto k = hs::jacobi2_kernel<ROWS, WAVES, PXL, XCD>;
    const dim3 gl = XCD ? dim3(8 * ((g.x * g.y + 7) / 8)) : g;  // launch grid
    auto k1 = hs::jacobi_kernel<32, 2, 4, true, true, false>;
    const dim3 g1 = hs::grid_for<32, 2, 4>(b.P, b.dimy);
    double *p2 = b.partial + 2 * 65536 / 2;
    auto launch2 = [&](const float2 *in, float2 *out) {
        hipLaunchKernelGGL(k, gl, dim3(64 * WAVES), 0, 0, in, out, b.dI, b.It, b.P, b.dimx, b.dimy,
                           0, b.dimy, 0.01f, -1, b.dimy + 1, b.partial, p2, b.status, 0, (int)g.x,
                           (int)g.y);
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 3; it++) launch2((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters / 2; it++) launch2((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / (2 * (iters / 2));
    const size_t cnt = (size_t)b.P * b.dimy;
    std::vector<float2> A(cnt), B(cnt);
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 6; it++)
        hipLaunchKernelGGL(k1, g1, dim3(256), 0, 0, (it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1,
                           b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy, 0.01f, b.partial, b.status);
    CK(hipMemcpy(A.data(), b.u0, sizeof(float2) * cnt, hipMemcpyDeviceToHost));
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 3; it++) launch2((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipMemcpy(B.data(), b.u1, sizeof(float2) * cnt, hipMemcpyDeviceToHost));
    // the slab's overlapped form: interior bands first, then the two outer ones
    {
        const int nb = (int)g.y;
        auto split = [&](const float2 *in, float2 *out) {
            auto bands = [&](int lo, int hi) {
                dim3 gg = g;
                gg.y = hi - lo;
                const dim3 ggl = XCD ? dim3(8 * ((gg.x * gg.y + 7) / 8)) : gg;
                hipLaunchKernelGGL(k, ggl, dim3(64 * WAVES), 0, 0, in, out, b.dI, b.It, b.P,
                                   b.dimx, b.dimy, 0, b.dimy, 0.01f, -1, b.dimy + 1, b.partial,
                                   p2, b.status, lo, (int)gg.x, (int)gg.y);
            };
            if (nb >= 3) {
                bands(1, nb - 1);
                bands(0, 1);
                bands(nb - 1, nb);
            } else {
                bands(0, nb);
            }
        };
        std::vector<float2> Cb(cnt);
        CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
        CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
        for (int it = 0; it < 3; it++) split((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
        CK(hipMemcpy(Cb.data(), b.u1, sizeof(float2) * cnt, hipMemcpyDeviceToHost));
        if (memcmp(Cb.data(), B.data(), sizeof(float2) * cnt) != 0) {
            printf("   band-split launches differ from the full launch\n");
            return 1;
        }
    }
    long bad = 0;
    for (int j = 0; j < b.dimy; j++)
        for (int i = 0; i < b.dimx; i++) {
            const float2 x = A[(size_t)j * b.P + i], y = B[(size_t)j * b.P + i];
            if (memcmp(&x, &y, sizeof x) != 0 && bad++ < 3)
                printf("   mismatch at (%d,%d): %.9g %.9g vs %.9g %.9g\n", i, j, x.x, x.y, y.x, y.y);
        }
    printf("%-28s grid=%5ux%-4u  %8.2f us/iter  %7.1f GB/s-equiv  %s\n", name, g.x, g.y, us,
           bytes / us / 1e3, bad ? "MISMATCH" : "bit-identical to 6 single steps");
    return bad ? 1 : 0;
}

// three iterations per launch: timed per ITERATION, checked against 6 single steps
template <int ROWS, int WAVES, int MINB = 1, int UNR = 4, bool FD = true>
int run3(const Bufs &b, int iters, const char *name, double bytes) {
    const dim3 g = hs::grid3_for<ROWS, WAVES>(b.dimx, b.dimy);
    const dim3 gl(8 * ((g.x * g.y + 7) / 8));
    auto k = hs::jacobi3_kernel<ROWS, WAVES, true, MINB, UNR, FD>;
    auto k1 = hs::jacobi_kernel<32, 2, 4, true, true, false>;
    const dim3 g1 = hs::grid_for<32, 2, 4>(b.P, b.dimy);
    double *p2 = b.partial + 2 * 16384, *p3 = b.partial + 4 * 16384;
    auto launch3 = [&](const float2 *in, float2 *out) {
        hipLaunchKernelGGL(k, gl, dim3(64 * WAVES), 0, 0, in, out, b.dI, b.It, b.P, b.dimx, b.dimy,
                           0, b.dimy, 0.01f, -1, b.dimy + 1, b.partial, p2, p3, b.status, 0,
                           (int)g.x, (int)g.y, ROWS, b.rflag, -1, -1);
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 3; it++) launch3((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipEventRecord(e0, 0));
    const int nl = iters / 3;
    for (int it = 0; it < nl; it++) launch3((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / (3 * nl);
    const size_t cnt = (size_t)b.P * b.dimy;
    std::vector<float2> A(cnt), B(cnt);
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 6; it++)
        hipLaunchKernelGGL(k1, g1, dim3(256), 0, 0, (it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1,
                           b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy, 0.01f, b.partial, b.status);
    CK(hipMemcpy(A.data(), b.u0, sizeof(float2) * cnt, hipMemcpyDeviceToHost));
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 2; it++) launch3((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipMemcpy(B.data(), b.u0, sizeof(float2) * cnt, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int j = 0; j < b.dimy; j++)
        for (int i = 0; i < b.dimx; i++) {
            const float2 x = A[(size_t)j * b.P + i], y = B[(size_t)j * b.P + i];
            if (memcmp(&x, &y, sizeof x) != 0 && bad++ < 3)
                printf("   mismatch at (%d,%d): %.9g %.9g vs %.9g %.9g\n", i, j, x.x, x.y, y.x, y.y);
        }
    printf("%-28s grid=%5ux%-4u  %8.2f us/iter  %7.1f GB/s-equiv  %s\n", name, g.x, g.y, us,
           bytes / us / 1e3, bad ? "MISMATCH" : "bit-identical to 6 single steps");
    return bad ? 1 : 0;
}

template <int PRIO, int DIAG = 0, int OPT = 0, bool ALT = false>
float time_prio(const Bufs &b, int nl, int rr = 0);

// the product triple kernel (PRIO 1) timed per iteration
int run3p(const Bufs &b, int iters, const char *name, double bytes) {
    const int gx = (b.dimx + kHs3Out - 1) / kHs3Out;
    const int r = hs3_rows(b.dimx, b.dimy);
    const int gy = (b.dimy + 4 * r - 1) / (4 * r);
    const int nl = iters / 3;
    const float us = time_prio<1, 0, 1, true>(b, nl) / 3.0f;
    printf("%-34s %4d blocks r=%-3d %8.2f us/iter (%6.2f us/launch)\n", name, 8 * ((gx * gy + 7) / 8),
           r, us, 3 * us);
    return 0;
}

// back-to-back launches of the four-step kernel (per launch, events)
template <int MINB, bool ALT, int UNR = 4>
float time_quad(const Bufs &b, int nl, int r) {
    const int gx = (b.dimx + kHs3Out - 1) / kHs3Out;
    const int gy = (b.dimy + 4 * r - 1) / (4 * r);
    auto k = hs::jacobi4_kernel<0, 4, true, MINB, UNR, 1, ALT>;
    double *p2 = b.partial + 2 * 16384, *p3 = b.partial + 4 * 16384, *p4 = b.partial + 6 * 16384;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto go = [&](int it) {
        hipLaunchKernelGGL(k, dim3(8 * ((gx * gy + 7) / 8)), dim3(256), 0, 0, (it & 1) ? b.u1 : b.u0,
                           (it & 1) ? b.u0 : b.u1, b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy,
                           0.01f, -1, b.dimy + 1, b.partial, p2, p3, p4, b.status, 0, gx, gy, r,
                           b.rflag, -1, -1);
    };
    for (int it = 0; it < 4; it++) go(it);
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < nl; it++) go(it);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 1000.0f * ms / nl;
}

// four iterations per launch (jacobi4_kernel), `r` j-lines per wave: timed per
// ITERATION, checked against 8 single steps
template <int WAVES, int MINB, int PRIO = 1, int UNR = 4, bool ALT = false>
int run4(const Bufs &b, int iters, int r, const char *name, double bytes) {
    const int gx = (b.dimx + kHs3Out - 1) / kHs3Out;
    const int gy = (b.dimy + WAVES * r - 1) / (WAVES * r);
    const dim3 gl(8 * ((gx * gy + 7) / 8));
    auto k = hs::jacobi4_kernel<0, WAVES, true, MINB, UNR, PRIO, ALT>;
    auto k1 = hs::jacobi_kernel<32, 2, 4, true, true, false>;
    const dim3 g1 = hs::grid_for<32, 2, 4>(b.P, b.dimy);
    double *p2 = b.partial + 2 * 16384, *p3 = b.partial + 4 * 16384, *p4 = b.partial + 6 * 16384;
    auto launch4 = [&](const float2 *in, float2 *out) {
        hipLaunchKernelGGL(k, gl, dim3(64 * WAVES), 0, 0, in, out, b.dI, b.It, b.P, b.dimx, b.dimy,
                           0, b.dimy, 0.01f, -1, b.dimy + 1, b.partial, p2, p3, p4, b.status, 0,
                           gx, gy, r, b.rflag, -1, -1);
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 3; it++) launch4((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipEventRecord(e0, 0));
    const int nl = iters / 4;
    for (int it = 0; it < nl; it++) launch4((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / (4 * nl);
    const size_t cnt = (size_t)b.P * b.dimy;
    std::vector<float2> A(cnt), B(cnt);
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 8; it++)
        hipLaunchKernelGGL(k1, g1, dim3(256), 0, 0, (it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1,
                           b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy, 0.01f, b.partial, b.status);
    CK(hipMemcpy(A.data(), b.u0, sizeof(float2) * cnt, hipMemcpyDeviceToHost));
    CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
    for (int it = 0; it < 2; it++) launch4((it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1);
    CK(hipMemcpy(B.data(), b.u0, sizeof(float2) * cnt, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int j = 0; j < b.dimy; j++)
        for (int i = 0; i < b.dimx; i++) {
            const float2 x = A[(size_t)j * b.P + i], y = B[(size_t)j * b.P + i];
            if (memcmp(&x, &y, sizeof x) != 0 && bad++ < 3)
                printf("   mismatch at (%d,%d): %.9g %.9g vs %.9g %.9g\n", i, j, x.x, x.y, y.x, y.y);
        }
    printf("%-34s %4u blocks r=%-3d %8.2f us/iter (%6.2f us/launch)  %s\n", name, gl.x, r, us,
           4 * us, bad ? "MISMATCH" : "bit-identical to 8 single steps");
    return bad ? 1 : 0;
}

// The slab's overlapped launch (slab.cpp fused): interior j-lines [E, n-E) on
// one stream with a block budget that leaves room for the two 16-line edge
// launches on a second stream.  Timed per three iterations against the full
// launch, and checked bit-identical to it.
int run_split(const Bufs &b, int iters) {
    using namespace of2d::hs;
    const int gx = (b.dimx + kHs3Out - 1) / kHs3Out;
    // edge j-lines (HV_E, a multiple of 4; the product uses 16) and the
    // interior's block budget as slab_geometry sets it (8 slots for RCCL)
    const int E = getenv("HV_E") ? atoi(getenv("HV_E")) : 16, RE = E / 4;
    const int ni = b.dimy - 2 * E;
    const int ri = hs3_rows(b.dimx, ni, 1024 - 2 * gx - 8);
    const int gyi = (ni + 4 * ri - 1) / (4 * ri);
    const int rf = hs3_rows(b.dimx, b.dimy);
    const int gyf = (b.dimy + 4 * rf - 1) / (4 * rf);
    auto k = jacobi3_kernel<0, 4, true, 4, 4, true, 1, 0, 1, true>;  // the product kernel
    double *p2 = b.partial + 2 * 16384, *p3 = b.partial + 4 * 16384;
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t ei, ee, e0, e1;
    CK(hipEventCreateWithFlags(&ei, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ee, hipEventDisableTiming));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto win = [&](hipStream_t st, const float2 *in, float2 *out, int jlo, int jhi, int r,
                   int slot) {
        const int gy = (jhi - jlo + 4 * r - 1) / (4 * r);
        hipLaunchKernelGGL(k, dim3(8 * ((gx * gy + 7) / 8)), dim3(256), 0, st, in, out, b.dI, b.It,
                           b.P, b.dimx, b.dimy, 0, b.dimy, 0.01f, -1, b.dimy + 1, b.partial, p2,
                           p3, b.status, slot, gx, gy, r, b.rflag, jlo, jhi);
    };
    auto full = [&](const float2 *in, float2 *out) { win(s1, in, out, 0, b.dimy, rf, 0); };
    // the earlier slab scheme: interior bands, then the first and the last band,
    // all on one stream
    auto serial = [&](const float2 *in, float2 *out) {
        win(s1, in, out, 4 * rf, (gyf - 1) * 4 * rf, rf, 1);
        win(s1, in, out, 0, 4 * rf, rf, 0);
        win(s1, in, out, (gyf - 1) * 4 * rf, b.dimy, rf, gyf - 1);
    };
    auto split = [&](const float2 *in, float2 *out) {
        CK(hipStreamWaitEvent(s2, ei, 0));  // previous interior
        CK(hipStreamWaitEvent(s1, ee, 0));  // previous edges
        win(s1, in, out, E, b.dimy - E, ri, 0);
        CK(hipEventRecord(ei, s1));
        win(s2, in, out, 0, E, RE, gyi);
        win(s2, in, out, b.dimy - E, b.dimy, RE, gyi + 1);
        CK(hipEventRecord(ee, s2));
    };
    const size_t cnt = (size_t)b.P * b.dimy;
    std::vector<float2> A(cnt), B(cnt);
    std::vector<float2> C(cnt);
    float ms[3];
    for (int mode = 0; mode < 3; mode++) {
        CK(hipDeviceSynchronize());
        CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
        CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * (size_t)b.P * (b.dimy + 2)));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(ei, s1));
        CK(hipEventRecord(ee, s2));
        auto go = [&](int it) {
            const float2 *in = (it & 1) ? b.u1 : b.u0;
            float2 *out = (it & 1) ? b.u0 : b.u1;
            if (mode == 0)
                full(in, out);
            else if (mode == 1)
                split(in, out);
            else
                serial(in, out);
        };
        for (int it = 0; it < 2; it++) go(it);
        CK(hipStreamWaitEvent(s1, ee, 0));
        CK(hipStreamSynchronize(s1));
        CK(hipMemcpy(mode == 0 ? A.data() : mode == 1 ? B.data() : C.data(), b.u0,
                     sizeof(float2) * cnt, hipMemcpyDeviceToHost));
        CK(hipEventRecord(e0, s1));
        CK(hipStreamWaitEvent(s2, e0, 0));
        for (int it = 0; it < iters; it++) go(it);
        CK(hipStreamWaitEvent(s1, ee, 0));
        CK(hipEventRecord(e1, s1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[mode], e0, e1));
    }
    long bad = 0;
    for (size_t i = 0; i < cnt; i++)
        if (memcmp(&A[i], &B[i], sizeof(float2)) != 0 || memcmp(&A[i], &C[i], sizeof(float2)) != 0)
            bad++;
    printf("full launch  %3d x %d rows  %8.2f us / 3 iterations\n", gyf, rf, 1000.0 * ms[0] / iters);
    printf("split launch %3d x %d rows + 2 x %d-line edges (second stream)  %8.2f us / 3 iterations  %s\n",
           gyi, ri, E, 1000.0 * ms[1] / iters, bad ? "MISMATCH" : "bit-identical to the full launch");
    printf("serial bands (interior, first, last on one stream)  %8.2f us / 3 iterations\n",
           1000.0 * ms[2] / iters);
    return bad ? 1 : 0;
}

// One stamped launch of the product triple kernel (runtime rows per wave, as
// launch_hs_jacobi3 picks them) after a warm-up: when each wave starts and
// ends, so the tail (waves idle while the slowest finish) can be read off.
template <int PRIO>
int run_stamps(const Bufs &b) {
    using namespace of2d::hs;
    const int gx = (b.dimx + kHs3Out - 1) / kHs3Out;
    const int r = hs3_rows(b.dimx, b.dimy);
    const int gy = (b.dimy + 4 * r - 1) / (4 * r);
    const int nblk = 8 * ((gx * gy + 7) / 8);
    auto k = jacobi3_kernel<0, 4, true, 4, 4, true, PRIO>;
    double *p2 = b.partial + 2 * 16384, *p3 = b.partial + 4 * 16384;
    auto go = [&](int it) {
        hipLaunchKernelGGL(k, dim3(nblk), dim3(256), 0, 0, (it & 1) ? b.u1 : b.u0,
                           (it & 1) ? b.u0 : b.u1, b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy,
                           0.01f, -1, b.dimy + 1, b.partial, p2, p3, b.status, 0, gx, gy, r,
                           b.rflag, -1, -1);
    };
    const size_t nw = (size_t)nblk * 4;
    unsigned long long *d;
    CK(hipMalloc(&d, sizeof(unsigned long long) * 4 * nw));
    CK(hipMemset(d, 0, sizeof(unsigned long long) * 4 * nw));
    for (int it = 0; it < 40; it++) go(it);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < 100; it++) go(it);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(4 * nw);
    printf("stamps PRIO=%d: %d x %d blocks (%d rows per wave), %zu waves; %.2f us per launch "
           "(100 launches, events)\n", PRIO, gx, gy, r, nw, 10.0 * ms);
    for (int rep = 0; rep < 3; rep++) {
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d, sizeof d));
        go(rep);
        CK(hipDeviceSynchronize());
        unsigned long long *z = nullptr;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &z, sizeof z));
        CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 4 * nw, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, t1 = 0;
        std::vector<double> st, en, du;
        double xsum[8] = {0}, xmax[8] = {0};
        int xn[8] = {0};
        for (size_t w = 0; w < nw; w++)
            if (h[4 * w + 1]) {
                t0 = std::min(t0, h[4 * w]);
                t1 = std::max(t1, h[4 * w + 1]);
            }
        for (size_t w = 0; w < nw; w++) {
            if (!h[4 * w + 1]) continue;
            const double a = (h[4 * w] - t0) * 0.01, e = (h[4 * w + 1] - t0) * 0.01;  // us
            st.push_back(a);
            en.push_back(e);
            du.push_back(e - a);
            const int x = (int)(h[4 * w + 2] & 7);
            xsum[x] += e - a;
            xmax[x] = std::max(xmax[x], e);
            xn[x]++;
        }
        auto pct = [](std::vector<double> v, double p) {
            std::sort(v.begin(), v.end());
            return v[(size_t)(p * (v.size() - 1))];
        };
        printf(" launch %d: span %.1f us, %zu waves stamped\n", rep, (t1 - t0) * 0.01, du.size());
        printf("  start  p0 %.1f p50 %.1f p90 %.1f p100 %.1f\n", pct(st, 0), pct(st, .5),
               pct(st, .9), pct(st, 1));
        printf("  end    p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f\n", pct(en, 0),
               pct(en, .1), pct(en, .5), pct(en, .9), pct(en, 1));
        printf("  dur    p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f\n", pct(du, 0),
               pct(du, .1), pct(du, .5), pct(du, .9), pct(du, 1));
        double busy = 0;
        for (double v : du) busy += v;
        printf("  wave-slot occupancy over the span: %.3f\n", busy / (du.size() * (t1 - t0) * 0.01));
        if (rep == 2) {  // mean duration by strip, by band, and the spread inside a CU
            std::vector<double> sb(gx, 0), sg(gy, 0);
            std::vector<int> nb(gx, 0), ng(gy, 0);
            std::map<unsigned, std::vector<double>> cu;
            const int per = (gx * gy + 7) / 8;
            for (size_t w = 0; w < nw; w++) {
                if (!h[4 * w + 1]) continue;
                const int blk = (int)(w / 4), L = (blk % 8) * per + blk / 8;
                const double dd = (h[4 * w + 1] - h[4 * w]) * 0.01;
                sb[L % gx] += dd;
                nb[L % gx]++;
                sg[L / gx] += dd;
                ng[L / gx]++;
                const unsigned hw = (unsigned)h[4 * w + 3];
                cu[((unsigned)h[4 * w + 2] << 16) | (hw >> 8)].push_back(dd);
            }
            printf("  by strip:");
            for (int i = 0; i < gx; i++) printf(" %.0f", nb[i] ? sb[i] / nb[i] : 0.0);
            printf("\n  by band:");
            for (int i = 0; i < gy; i++) printf(" %.0f", ng[i] ? sg[i] / ng[i] : 0.0);
            double within = 0, across = 0, gm = 0;
            int nn = 0;
            std::vector<double> cm;
            for (auto &kv : cu) {
                double m = 0;
                for (double v : kv.second) m += v;
                m /= kv.second.size();
                cm.push_back(m);
                for (double v : kv.second) within += (v - m) * (v - m), nn++;
                gm += m;
            }
            gm /= cm.size();
            for (double m : cm) across += (m - gm) * (m - gm);
            printf("\n  %zu CUs: std within a CU %.1f us, std of CU means %.1f us\n", cm.size(),
                   sqrt(within / nn), sqrt(across / cm.size()));
        }
        for (int x = 0; x < 8; x++)
            if (xn[x])
                printf("  xcc %d: %4d waves, mean dur %.1f us, last end %.1f us\n", x, xn[x],
                       xsum[x] / xn[x], xmax[x]);
    }
    CK(hipFree(d));
    return 0;
}

// Back-to-back launches of the product triple kernel with the progress
// priority schemes, interleaved in rounds so clock drift hits all alike.
template <int PRIO, int DIAG, int OPT, bool ALT>
float time_prio(const Bufs &b, int nl, int rr) {
    using namespace of2d::hs;
    const int gx = (b.dimx + kHs3Out - 1) / kHs3Out;
    const int r = rr > 0 ? rr : hs3_rows(b.dimx, b.dimy);
    const int gy = (b.dimy + 4 * r - 1) / (4 * r);
    const int nblk = 8 * ((gx * gy + 7) / 8);
    auto k = jacobi3_kernel<0, 4, true, 4, 4, true, PRIO, DIAG, OPT, ALT>;
    double *p2 = b.partial + 2 * 16384, *p3 = b.partial + 4 * 16384;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto go = [&](int it) {
        hipLaunchKernelGGL(k, dim3(nblk), dim3(256), 0, 0, (it & 1) ? b.u1 : b.u0,
                           (it & 1) ? b.u0 : b.u1, b.dI, b.It, b.P, b.dimx, b.dimy, 0, b.dimy,
                           0.01f, -1, b.dimy + 1, b.partial, p2, p3, b.status, 0, gx, gy, r,
                           b.rflag, -1, -1);
    };
    for (int it = 0; it < 4; it++) go(it);
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < nl; it++) go(it);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 1000.0f * ms / nl;
}

int run_prio(const Bufs &b) {
    const char *names[] = {"prio0", "prio1", "prio2", "prio1 no-logger", "prio0 no-logger", "prio1 nt-grad"};
    std::vector<std::vector<float>> t(6);
    for (int round = 0; round < 6; round++) {
        t[0].push_back(time_prio<0>(b, 200));
        t[1].push_back(time_prio<1>(b, 200));
        t[2].push_back(time_prio<2>(b, 200));
        t[3].push_back(time_prio<1, 1>(b, 200));
        t[4].push_back(time_prio<0, 1>(b, 200));
        t[5].push_back(time_prio<1, 2>(b, 200));
    }
    for (int v = 0; v < 6; v++) {
        printf("%s:", names[v]);
        for (float x : t[v]) printf(" %.2f", x);
        std::vector<float> s = t[v];
        std::sort(s.begin(), s.end());
        printf("  median %.2f us/launch\n", s[s.size() / 2]);
    }
    return 0;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 200;
    Bufs b;
    b.dimx = b.dimy = n;
    b.P = (n + 255) / 256 * 256 + (argc > 4 ? atoi(argv[4]) : 0);  // optional pitch padding
    const size_t rows = (size_t)n + 2;
    float2 *base0, *base1, *based;
    float *baset;
    CK(hipMalloc(&base0, sizeof(float2) * b.P * rows + 4096));
    CK(hipMalloc(&base1, sizeof(float2) * b.P * rows + 4096));
    CK(hipMalloc(&based, sizeof(float2) * b.P * rows + 4096));
    CK(hipMalloc(&baset, sizeof(float) * b.P * rows + 4096));
    b.u0 = base0 + b.P;
    b.u1 = base1 + b.P;
    b.dI = based + b.P;
    b.It = baset + b.P;
    CK(hipMalloc(&b.partial, sizeof(double) * 2 * 65536));
    CK(hipMalloc(&b.status, 64));
    std::vector<float> h((size_t)b.P * rows * 2);
    srand(1);
    for (auto &v : h) v = (rand() / (float)RAND_MAX) - 0.5f;
    if (getenv("HV_TEX")) {  // bench-like inputs: gradients of a smooth texture pair
        auto tex = [](double x, double y) {
            return 0.5 + 0.1 * (sin(0.11 * x + 0.07 * y) + sin(0.05 * x - 0.13 * y + 1.0) +
                                sin(0.23 * x + 0.19 * y + 2.0));
        };
        std::vector<float> g((size_t)b.P * rows * 2, 0.0f), t((size_t)b.P * rows, 0.0f);
        for (int j = 0; j < n; j++)
            for (int i = 0; i < n; i++) {
                const size_t o = (size_t)(j + 1) * b.P + i;
                g[2 * o] = (float)((tex(i + 1 - 1.5, j + 0.75) - tex(i - 1 - 1.5, j + 0.75)) / 2);
                g[2 * o + 1] = (float)((tex(i - 1.5, j + 1 + 0.75) - tex(i - 1.5, j - 1 + 0.75)) / 2);
                t[o] = (float)(tex(i - 1.5, j + 0.75) - tex(i, j));
            }
        CK(hipMemcpy(based, g.data(), sizeof(float2) * b.P * rows, hipMemcpyHostToDevice));
        CK(hipMemcpy(baset, t.data(), sizeof(float) * b.P * rows, hipMemcpyHostToDevice));
        printf("inputs: smooth texture pair (HV_TEX)\n");
    } else {
        CK(hipMemcpy(based, h.data(), sizeof(float2) * b.P * rows, hipMemcpyHostToDevice));
        CK(hipMemcpy(baset, h.data(), sizeof(float) * b.P * rows, hipMemcpyHostToDevice));
    }
    b.rflag = b.status + 8;
    CK(hipMemset(b.status, 0, 64));
    hipLaunchKernelGGL(hs::hs_precheck_kernel<>, dim3(1024), dim3(256), 0, 0, based,
                       (long)b.P * (long)rows, b.P, 1, b.dimx, b.dimy, 0.01f, b.rflag, b.status);
    unsigned hflag = 0;
    CK(hipMemcpy(&hflag, b.rflag, sizeof hflag, hipMemcpyDeviceToHost));
    printf("gradient range flag %u (0: unscaled division in range)\n", hflag);
    const double bytes = 28.0 * n * n;
    printf("grid %d^2, %d launches per variant, %.1f MB per launch\n", n, iters, bytes / 1e6);

    // probe: same traffic mix, no stencil
    {
        const long n2 = (long)b.P * n / 2;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int grid : {2048, 4096, 8192}) {
            hipLaunchKernelGGL(probe_kernel, dim3(grid), dim3(256), 0, 0, (const float4 *)b.u0,
                               (const float4 *)b.dI, (const float2 *)b.It, (float4 *)b.u1, n2);
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < iters; it++)
                hipLaunchKernelGGL(probe_kernel, dim3(grid), dim3(256), 0, 0,
                                   (const float4 *)((it & 1) ? b.u1 : b.u0), (const float4 *)b.dI,
                                   (const float2 *)b.It, (float4 *)((it & 1) ? b.u0 : b.u1), n2);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = 1000.0 * ms / iters;
            printf("probe grid=%-6d                   %8.2f us  %7.1f GB/s  %5.1f%% of 8 TB/s\n",
                   grid, us, bytes / us / 1e3, bytes / us / 1e3 / 80.0);
        }
    }

    const size_t cnt = (size_t)b.P * n;
    std::vector<float2> ref(cnt), got(cnt);
    int bad = 0;
#define V(R, X, W, NL, NS)                                                                 \
    do {                                                                                   \
        run<R, X, W, NL, NS>(b, iters, got.data(), #R "r " #X "px " #W "w nl" #NL " ns" #NS, \
                             bytes);                                                      \
        if (first) {                                                                       \
            ref = got;                                                                     \
            first = false;                                                                 \
        } else if (memcmp(ref.data(), got.data(), cnt * sizeof(float2)) != 0) {            \
            printf("   ^^^ MISMATCH\n");                                                   \
            bad++;                                                                         \
        }                                                                                  \
    } while (0)
    bool first = true;
#define V3(R, X, W, NL, NS, NG)                                                            \
    do {                                                                                   \
        run<R, X, W, NL, NS, NG>(b, iters, got.data(),                                     \
                                 #R "r " #X "px " #W "w u" #NL " st" #NS " g" #NG, bytes); \
        if (first) {                                                                       \
            ref = got;                                                                     \
            first = false;                                                                 \
        } else if (memcmp(ref.data(), got.data(), cnt * sizeof(float2)) != 0) {            \
            printf("   ^^^ MISMATCH\n");                                                  \
            bad++;                                                                         \
        }                                                                                  \
    } while (0)
    const bool product_only = argc > 3 && strcmp(argv[3], "product") == 0;
    if (argc > 3 && strcmp(argv[3], "pair") == 0)  // the product pair kernel (PMC runs)
        return run2<32, 4, 2, true>(b, iters, "two-step 32r 4w xcd (product)", bytes);
    if (argc > 3 && strcmp(argv[3], "prio") == 0) return run_prio(b);
    if (argc > 3 && strcmp(argv[3], "stamps") == 0)
        return run_stamps<0>(b) | run_stamps<1>(b) | run_stamps<2>(b) | run_stamps<0>(b);
    if (argc > 3 && strcmp(argv[3], "split") == 0)  // the slab's overlapped interior / edges
        return run_split(b, iters);
    if (argc > 3 && strcmp(argv[3], "triple") == 0)  // the product triple kernel (PMC runs)
        return run3<36, 4, 4, 4, true>(b, iters, "three-step 36r 4w xcd (product at 4096^2)", bytes);
    if (argc > 3 && strcmp(argv[3], "opt") == 0) {  // product triple kernel: OPT 0 vs 1
        // bit-identity: 7 launches of each from zero, whole field compared
        const int gx = (b.dimx + kHs3Out - 1) / kHs3Out;
        const int r = hs3_rows(b.dimx, b.dimy);
        const int gy = (b.dimy + 4 * r - 1) / (4 * r);
        double *p2 = b.partial + 2 * 16384, *p3 = b.partial + 4 * 16384;
        const size_t cnt = (size_t)b.P * (b.dimy + 2);
        std::vector<float2> A(cnt), B(cnt);
        typedef void (*K3)(const float2 *, float2 *, const float2 *, const float *, int, int, int,
                           int, int, float, int, int, double *, double *, double *, unsigned *,
                           int, int, int, int, const unsigned *, int, int);
        const K3 ks[3] = {hs::jacobi3_kernel<0, 4, true, 4, 4, true, 1, 0, 0, false>,
                          hs::jacobi3_kernel<0, 4, true, 4, 4, true, 1, 0, 0, true>,
                          hs::jacobi3_kernel<0, 4, true, 4, 4, true, 1, 0, 1, true>};
        const char *kn[3] = {"product", "ALT (alternating march)", "ALT + OPT 1"};
        bool same = true;
        for (int o = 0; o < 3; o++) {
            CK(hipMemset(b.u0 - b.P, 0, sizeof(float2) * cnt));
            CK(hipMemset(b.u1 - b.P, 0, sizeof(float2) * cnt));
            for (int it = 0; it < 7; it++)
                hipLaunchKernelGGL(ks[o], dim3(8 * ((gx * gy + 7) / 8)), dim3(256), 0, 0,
                                   (it & 1) ? b.u1 : b.u0, (it & 1) ? b.u0 : b.u1, b.dI, b.It, b.P,
                                   b.dimx, b.dimy, 0, b.dimy, 0.01f, -1, b.dimy + 1, b.partial, p2,
                                   p3, b.status, 0, gx, gy, r, b.rflag, -1, -1);
            CK(hipMemcpy(o ? B.data() : A.data(), b.u1 - b.P, sizeof(float2) * cnt,
                         hipMemcpyDeviceToHost));
            if (o) {
                const bool eq = memcmp(A.data(), B.data(), sizeof(float2) * cnt) == 0;
                printf("%s after 21 iterations: %s\n", kn[o], eq ? "bit-identical to the product" : "MISMATCH");
                same = same && eq;
            }
        }
        for (int w = 0; w < 3; w++) time_prio<1>(b, 200);
        std::vector<float> t[3];
        for (int round = 0; round < 6; round++) {
            t[0].push_back(time_prio<1, 0, 0, false>(b, 200));
            t[1].push_back(time_prio<1, 0, 0, true>(b, 200));
            t[2].push_back(time_prio<1, 0, 1, true>(b, 200));
        }
        for (int v = 0; v < 3; v++) {
            printf("%-26s:", kn[v]);
            for (float x : t[v]) printf(" %.2f", x);
            std::sort(t[v].begin(), t[v].end());
            printf("  median %.2f us/launch\n", t[v][t[v].size() / 2]);
        }
        return same ? 0 : 1;
    }
    if (argc > 3 && strcmp(argv[3], "rows") == 0) {  // product kernel, j-lines per wave swept
        const int rs[] = {0, 36, 40, 50, 56, 64, 80, 100, 128};
        for (int w = 0; w < 2; w++) time_prio<1, 0, 1, true>(b, 50);
        for (int round = 0; round < 2; round++)
            for (int r : rs) {
                const int rr = r ? r : hs3_rows(b.dimx, b.dimy);
                const int gx = (b.dimx + kHs3Out - 1) / kHs3Out, gy = (b.dimy + 4 * rr - 1) / (4 * rr);
                printf("rows %3d%s: %6d blocks  %8.2f us/launch\n", rr, r ? "" : " (hs3_rows)",
                       gx * gy, time_prio<1, 0, 1, true>(b, iters / 3, rr));
            }
        return 0;
    }
    if (argc > 3 && strcmp(argv[3], "quad") == 0) {  // four iterations per launch vs the triple
        int b4 = 0;
        for (int w = 0; w < 3; w++)  // past the clock transient of sustained load
            run3<36, 4, 4, 4, true>(b, iters, "(warm-up) three-step", bytes);
        if (getenv("HV_WARM")) {  // sustained back-to-back timing (no host sync between)
            time_prio<1, 0, 1, true>(b, 1500);
            for (int round = 0; round < 3; round++) {
                const float t3 = time_prio<1, 0, 1, true>(b, 600) / 3.0f;
                const float t4 = time_quad<3, true>(b, 450, 36) / 4.0f;
                const float t4b = time_quad<4, true, 1>(b, 450, 36) / 4.0f;
                printf("warm round %d: triple %.2f us/iter, quad minb3 %.2f, quad minb4 unr1 %.2f\n",
                       round, t3, t4, t4b);
            }
            return 0;
        }
        for (int round = 0; round < 2; round++) {
            b4 |= run3p(b, iters, "three-step (product)", bytes);
            b4 |= run4<4, 3, 1, 4, true>(b, iters, 36, "four-step minb3 alt", bytes);
            b4 |= run4<4, 3, 1, 4, true>(b, iters, 64, "four-step minb3 alt", bytes);
            b4 |= run4<4, 4, 1, 2, true>(b, iters, 36, "four-step minb4 unr2 alt", bytes);
            b4 |= run4<4, 4, 1, 1, true>(b, iters, 36, "four-step minb4 unr1 alt", bytes);
            b4 |= run4<4, 3, 1, 2, true>(b, iters, 36, "four-step minb3 unr2 alt", bytes);
        }
        return b4;
    }
    if (argc > 3 && strcmp(argv[3], "two") == 0) {
        int b2 = 0;
        V3(32, 2, 4, true, true, false);
        b2 |= run2<32, 4>(b, iters, "two-step 32r 4w", bytes);
        b2 |= run3<36, 4, 1, 4, false>(b, iters, "three-step 36r 4w unr4", bytes);
        b2 |= run3<36, 4, 1, 4, true>(b, iters, "three-step 36r 4w unr4 fd", bytes);
        b2 |= run3<36, 4, 4, 4, true>(b, iters, "three-step 36r 4w unr4 fd minb4", bytes);
        b2 |= run3<36, 4, 4, 2, true>(b, iters, "three-step 36r 4w unr2 fd minb4", bytes);
        b2 |= run3<36, 4, 3, 4, true>(b, iters, "three-step 36r 4w unr4 fd minb3", bytes);
        b2 |= run3<36, 4, 1, 4, false>(b, iters, "three-step 36r 4w unr4 (again)", bytes);
        b2 |= run2<32, 4, 2, true>(b, iters, "two-step 32r 4w xcd", bytes);
        b2 |= run2<32, 2, 2, true>(b, iters, "two-step 32r 2w xcd", bytes);
        b2 |= run2<16, 4, 2, true>(b, iters, "two-step 16r 4w xcd", bytes);
        b2 |= run2<32, 4>(b, iters, "two-step 32r 4w (again)", bytes);
        return b2;
    }
    V3(32, 2, 4, true, true, false);  // the product configuration (hs_kernels.hip)
    if (product_only) return 0;
    V3(32, 2, 4, false, true, false);
    V3(24, 2, 4, false, true, false);
    V3(40, 2, 4, false, true, false);
    V3(48, 2, 4, false, true, false);
    V3(32, 2, 2, false, true, false);
    V3(32, 2, 8, false, true, false);
    V3(24, 4, 2, false, true, false);
    V3(48, 4, 2, false, true, false);
    V3(32, 2, 4, true, true, false);
    V3(32, 2, 4, false, true, true);
    V3(32, 2, 4, true, false, false);
    V3(32, 4, 4, true, true, false);
    V3(64, 2, 2, false, true, false);
    V3(32, 2, 1, false, true, false);
    printf("%s\n", bad ? "SOME VARIANTS MISMATCH" : "all variants bit-identical");
    return bad ? 1 : 0;
}
