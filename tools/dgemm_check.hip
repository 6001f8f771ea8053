// Checks dgemm_nn_kernel (curvature_kernels.hip) against a CPU product on
// ragged shapes.  hipcc -O3 --offload-arch=gfx950 tools/dgemm_check.hip -o tools/dgemm_check
#include "../opticalflow2d_amd/csrc/curvature_kernels.hip"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace of2d;

struct Case {
    int M, N, K;
    long lda, sA, ldb, sB, ldc, sC;
    bool useE;
};

int main() {
    const long pl = 128L * 96;
    Case cases[] = {{64, 64, 64, 67, 0, 65, 0, 69, 0, false},
                    {70, 37, 37, 73, 0, 38, 0, 75, 0, false},
                    {5, 4, 4, 8, 0, 5, 0, 9, 0, false},
                    {130, 96, 130, 133, 0, 131, 0, 135, 0, false},
                    {128, 128, 16, 131, 0, 17, 0, 133, 0, false},
                    // the curvature pipeline's calls at 96 x 96 (pitch 128, x|y planes)
                    {96, 96, 96, 128, pl, 96, 0, 128, pl, false},
                    {96, 96, 96, 128, 0, 128, pl, 128, pl, true},
                    {128, 40, 128, 128, 0, 128, 128L * 40, 128, 128L * 40, true}};
    int bad = 0;
    for (auto &c : cases) {
        const int M = c.M, N = c.N, K = c.K, batch = 2;
        std::vector<double> A(c.lda * K + c.sA), B(c.ldb * N + c.sB), C(c.ldc * N + c.sC, -7.0),
            R(C.size(), -7.0), E((size_t)c.ldc * N);
        unsigned x = 7;
        auto rnd = [&]() { x = x * 1664525u + 1013904223u; return (x >> 8) * (1.0 / 16777216.0) - 0.5; };
        for (auto &v : A) v = rnd();
        for (auto &v : B) v = rnd();
        for (auto &v : E) v = rnd();
        for (int z = 0; z < batch; z++)
            for (int n = 0; n < N; n++)
                for (int m = 0; m < M; m++) {
                    double acc = 0;
                    for (int k = 0; k < K; k++)
                        acc += A[z * c.sA + m + k * c.lda] * B[z * c.sB + k + n * c.ldb];
                    if (c.useE) acc *= E[m + n * c.ldc];
                    R[z * c.sC + m + n * c.ldc] = acc;
                }
        double *dA, *dB, *dC, *dE;
        hipMalloc(&dA, A.size() * 8);
        hipMalloc(&dB, B.size() * 8);
        hipMalloc(&dC, C.size() * 8);
        hipMalloc(&dE, E.size() * 8);
        hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dC, C.data(), C.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dE, E.data(), E.size() * 8, hipMemcpyHostToDevice);
        launch_dgemm(M, N, K, dA, c.lda, c.sA, dB, c.ldb, c.sB, dC, c.ldc, c.sC,
                     c.useE ? dE : nullptr, c.ldc, batch, 0);
        hipMemcpy(C.data(), dC, C.size() * 8, hipMemcpyDeviceToHost);
        double err = 0;
        long first = -1;
        for (size_t q = 0; q < C.size(); q++) {
            const double d = std::fabs(C[q] - R[q]);
            if (d > err) err = d;
            if (d > 1e-12 && first < 0) first = (long)q;
        }
        printf("M=%d N=%d K=%d batch=%d E=%d max err %.3e", M, N, K, batch, (int)c.useE, err);
        if (first >= 0) printf("  first bad flat %ld got %f want %f", first, C[first], R[first]);
        printf("\n");
        bad += err > 1e-12;
        hipFree(dA);
        hipFree(dB);
        hipFree(dC);
        hipFree(dE);
    }
    return bad ? 1 : 0;
}
