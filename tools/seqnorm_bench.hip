// Timing harness of the device Logger norms (seqnorm_kernels.hip) in
// isolation, fed as the registration loop feeds them: K synthetic
// Horn-Schunck-like iterates u_k = A (1 - r^k) + noise at n x n (A smooth),
// the updates (u_{k-1}, u_k) in batches of B on two sets of workspaces, each
// stage of each batch timed by HIP events on one stream: the pass, the check
// + fix, the walk.
//   hipcc --offload-arch=gfx950 -O2 tools/seqnorm_bench.hip -o tools/seqnorm_bench \
//         -Lopticalflow2d_amd -lof2d -Wl,-rpath,'$ORIGIN/../opticalflow2d_amd'
//   tools/seqnorm_bench [n] [K] [B] [r]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../opticalflow2d_amd/csrc/of2d_device.h"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

__device__ float hashf(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return (float)(x >> 8) * (1.0f / 16777216.0f) - 0.5f;
}

__global__ void gen(float2 *u, int n, int P, float w, unsigned seed) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
    if (i >= n) return;
    const float x = (float)i / n, y = (float)j / n;
    const float ax = 1.5f * __sinf(6.3f * x + 2.0f * y) + 0.4f * __cosf(17.0f * y);
    const float ay = 1.2f * __cosf(5.1f * y - 3.0f * x) + 0.3f * __sinf(23.0f * x);
    const unsigned h = (unsigned)(j * n + i) * 2u + seed * 0x9e3779b9u;
    u[(size_t)j * P + i] = make_float2(ax * w + 1e-3f * hashf(h), ay * w + 1e-3f * hashf(h + 1));
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int K = argc > 2 ? std::atoi(argv[2]) : 12;
    const int B = argc > 3 ? std::atoi(argv[3]) : 3;
    const float decay = argc > 4 ? (float)std::atof(argv[4]) : 0.8f;  // |u_k - u_{k-1}| ratio
    const int P = (n + 127) / 128 * 128;
    std::vector<float2 *> u(K + 1);
    for (auto &p : u) {
        CK(hipMalloc(&p, (size_t)P * n * sizeof(float2)));
        CK(hipMemset(p, 0, (size_t)P * n * sizeof(float2)));
    }
    for (int k = 1; k <= K; k++) {
        float r = 1.0f;
        for (int q = 0; q < k; q++) r *= decay;
        hipLaunchKernelGGL(gen, dim3((n + 255) / 256, n), dim3(256), 0, 0, u[k], n, P, 1.0f - r, k);
    }
    std::vector<void *> ws(6);
    for (auto &w : ws) CK(hipMalloc(&w, of2d::seqnorm_workspace_bytes(n, n)));
    float *out;
    CK(hipMalloc(&out, 2 * K * sizeof(float)));
    int *dbg;
    CK(hipMalloc(&dbg, 10 * K * sizeof(int)));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int ng = (K + B - 1) / B;
    std::vector<hipEvent_t> ev(4 * ng);
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (int rep = 0; rep < 2; rep++) {  // rep 0 warms up (and leaves the profiles)
        for (int t = 0, g = 0; t < K; g++) {
            of2d::SeqnormBatch S;
            S.K = std::min(B, K - t);
            for (int i = 0; i <= S.K; i++) S.u[i] = u[t + i];
            for (int i = 0; i < S.K; i++) {
                S.ws[i] = ws[3 * (g & 1) + i];
                S.use_profile[i] = rep > 0 || g >= 2;
                S.out[i] = out + 2 * (t + i);
                S.dbg[i] = dbg + 10 * (t + i);
            }
            hipEvent_t *e = &ev[4 * g];
            CK(hipEventRecord(e[0], st));
            of2d::launch_seqnorm_pass(S, n, n, P, st);
            CK(hipEventRecord(e[1], st));
            of2d::launch_seqnorm_refine(S, n, n, P, st);
            CK(hipEventRecord(e[2], st));
            of2d::launch_seqnorm_walk(S, n, n, P, st);
            CK(hipEventRecord(e[3], st));
            if (rep > 0 && std::getenv("SNB_WS")) {
                CK(hipStreamSynchronize(st));
                for (int i = 0; i < S.K; i++) {
                    unsigned q[12];
                    of2d::seqnorm_ws_stats(S.ws[i], n, n, q);
                    std::printf("  update %d ws %d: listed %u prof %u %u | seg %u %u multi %u %u none %u %u\n",
                                t + i, 3 * (g & 1) + i, q[0], q[1], q[2], q[4], q[5], q[6], q[7],
                                q[8], q[9]);
                }
            }
            t += S.K;
        }
        CK(hipStreamSynchronize(st));
    }
    std::vector<float> h(2 * K);
    std::vector<int> d(10 * K);
    CK(hipMemcpy(h.data(), out, h.size() * sizeof(float), hipMemcpyDeviceToHost));
    CK(hipMemcpy(d.data(), dbg, d.size() * sizeof(int), hipMemcpyDeviceToHost));
    std::printf("seqnorm_bench %d^2, %d updates in batches of %d, decay %.3f\n", n, K, B, decay);
    std::printf("batch   pass  refine    walk (us) | per update: sums, resolves, raw, listed, made\n");
    double tot[3] = {0, 0, 0};
    for (int g = 0; g < ng; g++) {
        float t[3];
        for (int s = 0; s < 3; s++) {
            CK(hipEventElapsedTime(&t[s], ev[4 * g + s], ev[4 * g + s + 1]));
            tot[s] += t[s];
        }
        std::printf("%5d %7.1f %7.1f %7.1f |", g, 1e3 * t[0], 1e3 * t[1], 1e3 * t[2]);
        for (int k = g * B; k < std::min(K, g * B + B); k++)
            std::printf(" [%.6g %.6g  %d %d  %d %d  %d  %d %d]", h[2 * k], h[2 * k + 1], d[10 * k],
                        d[10 * k + 1], d[10 * k + 2], d[10 * k + 3], d[10 * k + 4], d[10 * k + 8],
                        d[10 * k + 9]);
        std::printf("\n");
    }
    std::printf("per update: pass %.1f refine %.1f walk %.1f us\n", 1e3 * tot[0] / K,
                1e3 * tot[1] / K, 1e3 * tot[2] / K);
    return 0;
}
