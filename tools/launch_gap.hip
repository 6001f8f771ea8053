// launch_gap.hip — what separates two dependent back-to-back kernels on one
// stream (the HS triple kernel's inter-launch gap).
//
// Same grid as the HS triple kernel at 4096^2 (1016 blocks of 256 threads),
// four bodies: empty; read 128 MB; read 128 MB + write 128 MB with
// non-temporal stores (the triple kernel's u' policy); the same with default
// stores.  Each is launched back to back nlaunch times, timed with events
// around the whole run (per-launch = kernel + gap), and as graphs of the same
// launches.  Run under rocprofv3 --kernel-trace to split kernel from gap.
//   hipcc --offload-arch=gfx950 -O3 -o tools/launch_gap tools/launch_gap.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

constexpr int kBlocks = 1016, kThreads = 256;
constexpr size_t kN = (size_t)4096 * 4096 / 2;  // float4 = 2 px of float2: 128 MB

__global__ void k_empty(float4 *, const float4 *, size_t) {}

typedef float v4f __attribute__((ext_vector_type(4)));

template <int MODE>  // 1 read, 2 read + NT write, 3 read + write
__global__ __launch_bounds__(kThreads) void k_stream(float4 *dst, const float4 *src, size_t n) {
    float4 acc = make_float4(0, 0, 0, 0);
    for (size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (size_t)gridDim.x * kThreads) {
        const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(src) + i);
        if (MODE == 1) {
            acc.x += v.x;
        } else if (MODE == 2) {
            __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(dst) + i);
        } else {
            reinterpret_cast<v4f *>(dst)[i] = v;
        }
    }
    if (MODE == 1 && acc.x == 12345.0f) dst[0] = acc;
}

template <class K>
void run(const char *name, K kern, float4 *a, float4 *b, int nlaunch, hipStream_t st) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 50; w++) hipLaunchKernelGGL(kern, dim3(kBlocks), dim3(kThreads), 0, st, a, b, kN);
    CK(hipEventRecord(e0, st));
    for (int k = 0; k < nlaunch; k++)
        hipLaunchKernelGGL(kern, dim3(kBlocks), dim3(kThreads), 0, st, (k & 1) ? a : b,
                           (k & 1) ? b : a, kN);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // the same launches captured as one graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int k = 0; k < nlaunch; k++)
        hipLaunchKernelGGL(kern, dim3(kBlocks), dim3(kThreads), 0, st, (k & 1) ? a : b,
                           (k & 1) ? b : a, kN);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float gms = 0;
    CK(hipEventElapsedTime(&gms, e0, e1));
    printf("%-28s stream %8.2f us/launch   graph %8.2f us/launch\n", name, 1000.0 * ms / nlaunch,
           1000.0 * gms / nlaunch);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
}

int main(int argc, char **argv) {
    const int nlaunch = argc > 1 ? atoi(argv[1]) : 330;
    float4 *a, *b;
    CK(hipMalloc(&a, kN * sizeof(float4)));
    CK(hipMalloc(&b, kN * sizeof(float4)));
    CK(hipMemset(a, 0, kN * sizeof(float4)));
    CK(hipMemset(b, 0, kN * sizeof(float4)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    run("empty", k_empty, a, b, nlaunch, st);
    run("read 128 MB", k_stream<1>, a, b, nlaunch, st);
    run("read + NT write 128 MB", k_stream<2>, a, b, nlaunch, st);
    run("read + write 128 MB", k_stream<3>, a, b, nlaunch, st);
    CK(hipFree(a));
    CK(hipFree(b));
    return 0;
}
