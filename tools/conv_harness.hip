// Demons kernel harness at 4096^2 (or argv[1]): checks the fused correction
// update (launch_demons_update) bit for bit against the unfused force +
// smooth_compose pair, then times the shipped kernels and tile / packing
// variants of the smoothing kernels against a same-traffic copy floor,
// interleaved in rounds so that clock drift hits every variant alike.
//   hipcc -O3 -ffp-contract=off -std=c++17 --offload-arch=gfx950 \
//         -I opticalflow2d_amd/csrc tools/conv_harness.hip -o tools/conv_harness
#include "../opticalflow2d_amd/csrc/demons_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

using namespace of2d;

// the floor: read a, b (8 B each), write c (8 B), per 64 x 16 block
__global__ __launch_bounds__(256) void copy_floor(const float2 *__restrict__ a,
                                                  const float2 *__restrict__ b,
                                                  float2 *__restrict__ c, int dimx, int dimy,
                                                  int P) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    for (int k = 0; k < 4; k++) {
        const int j = blockIdx.y * 16 + threadIdx.y * 4 + k;
        if (i < dimx && j < dimy) {
            const long idx = (long)j * P + i;
            const float2 x = a[idx], y = b[idx];
            c[idx] = make_float2(x.x + y.x, x.y + y.y);
        }
    }
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 4096;
    const int ny = argc > 2 ? atoi(argv[2]) : n;
    const int P = pitch_for(n);
    const size_t cnt = (size_t)(ny + 2) * P;
    std::vector<float2> h(cnt);
    std::vector<float> hi(cnt);
    unsigned x = 1;
    for (size_t k = 0; k < cnt; k++) {
        x = x * 1664525u + 1013904223u;
        // small motions (|u| < 1.5 px), as in a converging registration
        h[k] = make_float2(((x >> 8) & 1023) / 1024.0f * 3.0f - 1.5f,
                           ((x >> 18) & 1023) / 1024.0f * 3.0f - 1.5f);
        hi[k] = ((x >> 4) & 4095) / 4096.0f;
    }
    float2 *A, *B, *C, *D;
    float *I1, *I2;
    hipMalloc(&A, cnt * 8);
    hipMalloc(&B, cnt * 8);
    hipMalloc(&C, cnt * 8);
    hipMalloc(&D, cnt * 8);
    hipMalloc(&I1, cnt * 4);
    hipMalloc(&I2, cnt * 4);
    hipMemcpy(A, h.data(), cnt * 8, hipMemcpyHostToDevice);
    hipMemcpy(B, h.data(), cnt * 8, hipMemcpyHostToDevice);
    hipMemcpy(I1, hi.data(), cnt * 4, hipMemcpyHostToDevice);
    std::reverse(hi.begin(), hi.end());
    hipMemcpy(I2, hi.data(), cnt * 4, hipMemcpyHostToDevice);
    float2 *a = A + P, *b = B + P, *c = C + P, *d = D + P;
    float *iref = I1 + P, *imov = I2 + P;
    const int kw = 5;
    // a normalised Gaussian (sigma 2), weights as Kernel::set_gaussian stores them
    std::vector<double> kd(kw * kw);
    double ksum = 0;
    for (int q = 0; q < kw * kw; q++) {
        const int di = q % kw - 2, dj = q / kw - 2;
        kd[q] = std::exp(-(di * di + dj * dj) / 8.0);
        ksum += kd[q];
    }
    std::vector<float> kf(kw * kw);
    double wfull = 0;
    for (int q = 0; q < kw * kw; q++) {
        kd[q] /= ksum;
        kf[q] = (float)kd[q];
    }
    for (int ii = 0; ii < kw; ii++)
        for (int jj = 0; jj < kw; jj++) wfull += kd[ii + jj * kw];
    float *dkf;
    double *dkd, *part;
    unsigned *status;
    hipMalloc(&dkf, 100);
    hipMalloc(&dkd, 200);
    hipMalloc(&status, 4);
    hipMemset(status, 0, 4);
    const dim3 g2 = conv_grid_r(n, ny, 2);
    hipMalloc(&part, 16 * (size_t)g2.x * g2.y);
    hipMemcpy(dkf, kf.data(), kf.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dkd, kd.data(), kd.size() * 8, hipMemcpyHostToDevice);
    const ConvArgs ca{dkf, dkd, kw, 2, 2, wfull};
    const float si = 1.0f, sx = 0.25f;

    // 1. the fused update against force + smooth_compose, every mode
    int bad = 0;
    for (int mode = 0; mode < 4; mode++) {
        launch_demons_force(iref, imov, a, d, n, ny, P, si * si, sx * sx, status, 0);
        launch_smooth_compose(d, a, c, n, ny, P, dkf, dkd, kw, wfull, mode, 0);
        std::vector<float2> want((size_t)ny * P), got((size_t)ny * P);
        hipMemcpy(want.data(), c, want.size() * 8, hipMemcpyDeviceToHost);
        hipMemset(C, 0, cnt * 8);
        launch_demons_update(iref, imov, a, d, c, n, ny, P, si * si, sx * sx, dkf, dkd, kw, wfull,
                             mode, status, 0);
        hipMemcpy(got.data(), c, got.size() * 8, hipMemcpyDeviceToHost);
        long nb = 0;
        for (int j = 0; j < ny; j++)
            for (int i = 0; i < n; i++) {
                const size_t k = (size_t)j * P + i;
                if (memcmp(&want[k], &got[k], 8) != 0 && nb++ < 3)
                    printf("  mode %d mismatch at (%d,%d): %.9g %.9g vs %.9g %.9g\n", mode, i, j,
                           want[k].x, want[k].y, got[k].x, got[k].y);
            }
        int nl, nr;
        const int ni = demons_edge_tiles(n, kw, &nl, &nr);
        printf("fused update mode %d (%d interior + %d/%d edge tile columns): %s\n", mode, ni, nl,
               nr, nb ? "MISMATCH" : "bit-identical to force + smooth_compose");
        bad |= nb != 0;
    }
    if (hipGetLastError() != hipSuccess) {
        printf("launch error\n");
        return 1;
    }

    // 2. timings
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct V {
        const char *name;
        std::function<void()> fn;
        std::vector<float> us;
    };
    auto norm = [&](auto kern, int R) {
        return [=] {
            hipLaunchKernelGGL(kern, conv_grid_r(n, ny, R), dim3(64, 4), conv_lds_bytes(2, 2, R),
                               0, a, b, c, n, ny, P, ca, part);
        };
    };
    auto comp = [&](auto kern, int R, int mode) {
        const int gx = (n + 63) / 64;
        return [=] {
            hipLaunchKernelGGL(kern, conv_grid_r(n, ny, R), dim3(64, 4), conv_lds_bytes(2, 2, R),
                               0, d, a, c, n, ny, P, ca, mode, gx, gx);
        };
    };
    std::vector<V> vs;
    vs.push_back({"copy floor (24 B/px)",
                  [&] {
                      hipLaunchKernelGGL(copy_floor, dim3(n / 64, (ny + 15) / 16), dim3(64, 4), 0, 0,
                                         a, b, c, n, ny, P);
                  },
                  {}});
    vs.push_back({"force", [&] {
                      launch_demons_force(iref, imov, a, d, n, ny, P, si * si, sx * sx, status, 0);
                  }, {}});
    vs.push_back({"compose R4 scalar", comp(smooth_compose_kernel<5, 4, false>, 4, 0), {}});
    vs.push_back({"compose R8 packed", comp(smooth_compose_kernel<5, 8, true>, 8, 0), {}});
    vs.push_back({"force + compose R8", [&] {
                      launch_demons_force(iref, imov, a, d, n, ny, P, si * si, sx * sx, status, 0);
                      launch_smooth_compose(d, a, c, n, ny, P, dkf, dkd, kw, wfull, 0, 0);
                  }, {}});
    vs.push_back({"fused update (shipped)", [&] {
                      launch_demons_update(iref, imov, a, d, c, n, ny, P, si * si, sx * sx, dkf,
                                           dkd, kw, wfull, 0, status, 0);
                  }, {}});
    vs.push_back({"norm R4 scalar", norm(smooth_norm_kernel<5, 4, false>, 4), {}});
    vs.push_back({"norm R4 packed", norm(smooth_norm_kernel<5, 4, true>, 4), {}});
    vs.push_back({"norm R8 scalar", norm(smooth_norm_kernel<5, 8, false>, 8), {}});
    vs.push_back({"norm R8 packed (shipped)", norm(smooth_norm_kernel<5, 8, true>, 8), {}});
    const int reps = 30;
    for (int round = 0; round < 5; round++) {
        for (auto &v : vs) {
            for (int r = 0; r < 3; r++) v.fn();
            hipEventRecord(e0, 0);
            for (int r = 0; r < reps; r++) v.fn();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            v.us.push_back(ms * 1e3f / reps);
        }
    }
    if (hipGetLastError() != hipSuccess) {
        printf("launch error\n");
        return 1;
    }
    printf("grid %d x %d, kw %d, median of 5 rounds of %d launches\n", n, ny, kw, reps);
    for (auto &v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double us = v.us[v.us.size() / 2];
        printf("%-28s %8.1f us  %6.2f TB/s at 24 B/px\n", v.name, us, 24.0 * n * ny / us / 1e6);
    }
    return bad;
}
