// Demons smoothing timing harness: the shipped smooth_norm / smooth_compose
// kernels against a same-traffic copy floor at 4096^2.
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -I opticalflow2d_amd/csrc \
//         tools/conv_harness.hip -o tools/conv_harness
#include "../opticalflow2d_amd/csrc/demons_kernels.hip"

#include <cstdio>
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
    const int P = pitch_for(n);
    const size_t cnt = (size_t)(n + 2) * P;
    std::vector<float2> h(cnt);
    unsigned x = 1;
    for (auto &v : h) {
        x = x * 1664525u + 1013904223u;
        v = make_float2(((x >> 8) & 1023) / 1024.0f - 0.5f, ((x >> 18) & 1023) / 1024.0f - 0.5f);
    }
    float2 *A, *B, *C;
    hipMalloc(&A, cnt * 8);
    hipMalloc(&B, cnt * 8);
    hipMalloc(&C, cnt * 8);
    hipMemcpy(A, h.data(), cnt * 8, hipMemcpyHostToDevice);
    hipMemcpy(B, h.data(), cnt * 8, hipMemcpyHostToDevice);
    float2 *a = A + P, *b = B + P, *c = C + P;
    const int kw = 5;
    std::vector<float> kf(kw * kw, 0.04f);
    std::vector<double> kd(kw * kw, 0.04);
    float *dkf;
    double *dkd, *part;
    hipMalloc(&dkf, 100);
    hipMalloc(&dkd, 200);
    hipMalloc(&part, 16 * (size_t)conv_nblocks(n, n));
    hipMemcpy(dkf, kf.data(), kf.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dkd, kd.data(), kd.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto fn) {
        for (int r = 0; r < 3; r++) fn();
        hipEventRecord(e0, 0);
        const int reps = 50;
        for (int r = 0; r < reps; r++) fn();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / reps;
        printf("%-28s %8.1f us  %6.2f TB/s (24 B/px)\n", name, us, 24.0 * n * n / us / 1e6);
    };
    timeit("copy floor", [&] {
        hipLaunchKernelGGL(copy_floor, conv_grid(n, n), dim3(64, 4), 0, 0, a, b, c, n, n, P);
    });
    timeit("smooth_norm kw5", [&] {
        launch_smooth_norm(a, b, c, n, n, P, dkf, dkd, kw, 1.0, part, 0);
    });
    timeit("smooth_compose kw5 mode0", [&] {
        launch_smooth_compose(a, b, c, n, n, P, dkf, dkd, kw, 1.0, 0, 0);
    });
    timeit("smooth_compose kw5 mode3", [&] {
        launch_smooth_compose(a, b, c, n, n, P, dkf, dkd, kw, 1.0, 3, 0);
    });
    return 0;
}
