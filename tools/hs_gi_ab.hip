// hs_gi_ab.hip — A/B harness (not part of the product): the triple Jacobi
// kernel reading the gradient field dI (28 B/px per launch) against the same
// kernel deriving the gradients from Iaux in the kernel (GI, 24 B/px), at
// several unroll depths.  Checks every variant bit-identical to the product
// kernel (motion after 21 iterations and the Logger partials), then times
// them interleaved in rounds after a sustained warm-up.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 \
//         -I opticalflow2d_amd/csrc tools/hs_gi_ab.hip -Lopticalflow2d_amd -lof2d \
//         -Wl,-rpath,'$ORIGIN/../opticalflow2d_amd' -o tools/hs_gi_ab
//   tools/hs_gi_ab [dimx=4096] [launches=300] [rounds=5] [variant (PMC mode) | -1] [dimy=dimx]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hs_jacobi_impl.h"

using namespace of2d;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

// streaming probes with the two kernels' access mixes and no stencil (2 px
// per thread): u float4 + dI float4 + It float2 in, float4 out (28 B/px), and
// u float4 + Iaux float2 + It float2 in, float4 out (24 B/px).  Their known
// byte counts calibrate FETCH_SIZE / WRITE_SIZE for each mix, and their time
// is the achievable ceiling for that mix at this grid.
__global__ void probe_field_kernel(const float4 *__restrict__ u, const float4 *__restrict__ g,
                                   const float2 *__restrict__ t, float4 *__restrict__ o, long n2) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
         i += (long)gridDim.x * blockDim.x) {
        const float4 a = u[i], b = g[i];
        const float2 c = t[i];
        o[i] = make_float4(a.x + b.x * c.x, a.y + b.y, a.z + b.z * c.y, a.w + b.w);
    }
}
__global__ void probe_image_kernel(const float4 *__restrict__ u, const float2 *__restrict__ ia,
                                   const float2 *__restrict__ t, float4 *__restrict__ o, long n2) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
         i += (long)gridDim.x * blockDim.x) {
        const float4 a = u[i];
        const float2 b = ia[i], c = t[i];
        o[i] = make_float4(a.x + b.x * c.x, a.y + b.y, a.z + b.x * c.y, a.w + b.y);
    }
}

typedef void (*K3)(const float2 *, float2 *, const float2 *, const float *, int, int, int, int,
                   int, float, int, int, double *, double *, double *, unsigned *, int, int, int,
                   int, const unsigned *, int, int, const float *);

struct Variant {
    const char *name;
    K3 k;
    bool gi;
    int cap;  // resident 4-wave blocks per round (blocks per CU x 256)
};

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;  // dimx
    const int ny = argc > 5 ? atoi(argv[5]) : n;    // dimy
    const int launches = argc > 2 ? atoi(argv[2]) : 300;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const int P = pitch_for(n);
    const size_t cnt = (size_t)P * (ny + 2) + kPitchAlign;
    const float alphasq = 0.1f * 0.1f;
    float2 *u0, *u1, *dI;
    float *Ia, *Ir, *It;
    CK(hipMalloc(&u0, cnt * 8));
    CK(hipMalloc(&u1, cnt * 8));
    CK(hipMalloc(&dI, cnt * 8));
    CK(hipMalloc(&Ia, cnt * 4));
    CK(hipMalloc(&Ir, cnt * 4));
    CK(hipMalloc(&It, cnt * 4));
    CK(hipMemset(dI, 0, cnt * 8));
    CK(hipMemset(It, 0, cnt * 4));
    // smooth texture pair, the moving image shifted by (1.5, -0.75)
    std::vector<float> a(cnt, 0.0f), r(cnt, 0.0f);
    auto tex = [](double x, double y) {
        return 0.5 + 0.1 * (sin(0.11 * x + 0.07 * y) + sin(0.05 * x - 0.13 * y + 1.0) +
                            sin(0.23 * x + 0.19 * y + 2.0));
    };
    for (int j = 0; j < ny; j++)
        for (int i = 0; i < n; i++) {
            const size_t o = (size_t)(j + 1) * P + i;
            r[o] = (float)tex(i, j);
            a[o] = (float)tex(i - 1.5, j + 0.75);
        }
    CK(hipMemcpy(Ia, a.data(), cnt * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(Ir, r.data(), cnt * 4, hipMemcpyHostToDevice));
    float2 *pu0 = u0 + P, *pu1 = u1 + P, *pdI = dI + P;
    float *pIa = Ia + P, *pIr = Ir + P, *pIt = It + P;
    hipStream_t st = 0;
    launch_gradients(pIr, pIa, pdI, pIt, n, ny, P, st);
    unsigned *status, *rflag;
    CK(hipMalloc(&status, 256));
    CK(hipMemset(status, 0, 256));
    rflag = status + kRangeFlagWord;
    launch_hs_precheck(dI, cnt, P, 1, n, ny, alphasq, rflag, status, st);
    unsigned hf[2] = {0, 0};
    CK(hipMemcpy(hf, status, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hf + 1, rflag, 4, hipMemcpyDeviceToHost));
    printf("grid %d x %d P %d: status %u range flag %u\n", n, ny, P, hf[0], hf[1]);
    const int gx = (n + kHs3Out - 1) / kHs3Out;
    const int nbmax = gx * ((ny + 15) / 16);
    double *part;
    CK(hipMalloc(&part, sizeof(double) * 6 * nbmax));
    // (the prefetch-depth and branch-free probes of profiles/r02_d_*, r02_e_*
    // were template variants of the same kernel, removed from the product header)
    const Variant vs[] = {
        {"dI  unr4 4/CU (product, field)", hs::jacobi3_kernel<0, 4, true, 4, 4, 1, true, false>, false, 1024},
        {"GI  unr4 4/CU (product, image)", hs::jacobi3_kernel<0, 4, true, 4, 4, 1, true, true>, true, 1024},
        {"GI  unr2 4/CU", hs::jacobi3_kernel<0, 4, true, 4, 2, 1, true, true>, true, 1024},
    };
    const int nv = sizeof vs / sizeof vs[0];
    // the partial slots are indexed by the variant's own block count, so the
    // Logger partials are compared between variants of the same geometry only
    auto geom = [&](const Variant &v, int &rows, int &gy) {
        rows = hs3_rows(n, ny, v.cap);
        gy = (ny + 4 * rows - 1) / (4 * rows);
    };
    auto launch = [&](const Variant &v, const float2 *in, float2 *out) {
        int rows, gy;
        geom(v, rows, gy);
        const int nb = gx * gy;
        hipLaunchKernelGGL(v.k, dim3(8 * ((nb + 7) / 8)), dim3(256), 0, st, in, out, pdI, pIt, P,
                           n, ny, 0, ny, alphasq, -1, ny + 1, part, part + 2 * nb, part + 4 * nb,
                           status, 0, gx, gy, rows, rflag, -1, -1, v.gi ? pIa : nullptr);
    };
    // probes over the pitched rows (P * ny px, 2 px per thread)
    const long n2 = (long)P * ny / 2;
    auto probes = [&](int reps) {
        for (int k = 0; k < reps; k++) {
            hipLaunchKernelGGL(probe_field_kernel, dim3(8192), dim3(256), 0, st, (const float4 *)pu0,
                               (const float4 *)pdI, (const float2 *)pIt, (float4 *)pu1, n2);
            hipLaunchKernelGGL(probe_image_kernel, dim3(8192), dim3(256), 0, st, (const float4 *)pu1,
                               (const float2 *)pIa, (const float2 *)pIt, (float4 *)pu0, n2);
        }
    };
    if (argc > 4 && atoi(argv[4]) == -2) {  // PMC mode: the probes only
        probes(launches);
        CK(hipDeviceSynchronize());
        printf("probes: %d launches each, %ld px\n", launches, 2 * n2);
        return 0;
    }
    if (argc > 4 && atoi(argv[4]) >= 0) {  // PMC mode: `launches` launches of variant argv[4] only
        const int v = atoi(argv[4]);
        for (int w = 0; w < launches; w++) launch(vs[v], (w & 1) ? pu1 : pu0, (w & 1) ? pu0 : pu1);
        CK(hipDeviceSynchronize());
        printf("%s: %d launches\n", vs[v].name, launches);
        return 0;
    }
    // bit identity: 7 launches (21 iterations) from zero motion
    std::vector<float2> ref(cnt), got(cnt);
    std::vector<double> pref(6 * nbmax), pgot(6 * nbmax);
    int bad = 0;
    for (int v = 0; v < nv; v++) {
        CK(hipMemset(u0, 0, cnt * 8));
        CK(hipMemset(u1, 0, cnt * 8));
        for (int it = 0; it < 7; it++) launch(vs[v], (it & 1) ? pu1 : pu0, (it & 1) ? pu0 : pu1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), u1, cnt * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pgot.data(), part, pgot.size() * 8, hipMemcpyDeviceToHost));
        if (v == 0) {
            ref = got;
            pref = pgot;
            continue;
        }
        long diff = 0;
        for (int j = 0; j < ny; j++)
            diff += memcmp(&ref[(size_t)(j + 1) * P], &got[(size_t)(j + 1) * P], 8 * (size_t)n) != 0;
        int rows, gy;
        geom(vs[v], rows, gy);
        const bool same_geom = vs[v].cap == vs[0].cap;
        const bool peq = !same_geom || memcmp(pref.data(), pgot.data(), 6 * gx * gy * 8) == 0;
        printf("%-28s: rows %d, 21 iterations %s, Logger partials %s\n", vs[v].name, rows,
               diff ? "MISMATCH" : "bit-identical",
               same_geom ? (peq ? "identical" : "DIFFER") : "(other band geometry)");
        bad += (diff != 0) + !peq;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 3 * launches; w++) launch(vs[0], (w & 1) ? pu1 : pu0, (w & 1) ? pu0 : pu1);
    std::vector<std::vector<float>> t(nv);
    for (int rd = 0; rd < rounds; rd++)
        for (int v = 0; v < nv; v++) {
            CK(hipEventRecord(e0, st));
            for (int w = 0; w < launches; w++)
                launch(vs[v], (w & 1) ? pu1 : pu0, (w & 1) ? pu0 : pu1);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(1000.0f * ms / launches);
        }
    {
        probes(20);
        float ms;
        for (int which = 0; which < 2; which++) {
            CK(hipEventRecord(e0, st));
            for (int k = 0; k < launches; k++) {
                if (which == 0)
                    hipLaunchKernelGGL(probe_field_kernel, dim3(8192), dim3(256), 0, st,
                                       (const float4 *)pu0, (const float4 *)pdI,
                                       (const float2 *)pIt, (float4 *)pu1, n2);
                else
                    hipLaunchKernelGGL(probe_image_kernel, dim3(8192), dim3(256), 0, st,
                                       (const float4 *)pu0, (const float2 *)pIa,
                                       (const float2 *)pIt, (float4 *)pu1, n2);
            }
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = 1000.0 * ms / launches, b = (which ? 24.0 : 28.0) * P * ny;
            printf("probe %-22s: %.2f us/launch, %.0f GB/s (%d B/px, no stencil)\n",
                   which ? "u+Iaux+It (image mix)" : "u+dI+It (field mix)", us, b / us / 1e3,
                   which ? 24 : 28);
        }
    }
    for (int v = 0; v < nv; v++) {
        printf("%-28s:", vs[v].name);
        for (float x : t[v]) printf(" %.2f", x);
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2];
        const double bytes = (vs[v].gi ? 24.0 : 28.0) * n * ny;
        printf("  median %.2f us/launch (%.2f us/iter, %.0f GB/s of its own %d B/px)\n", med,
               med / 3, bytes / med / 1e3, vs[v].gi ? 24 : 28);
    }
    return bad ? 1 : 0;
}
