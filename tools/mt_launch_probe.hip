// mt_launch_probe.hip — the launch pattern of the in-process slab group
// (slab.cpp local_exchange) without any of the library: N host threads, one
// non-blocking stream each, all on device 0; per step every thread launches a
// streaming kernel over its own buffer, records a "ready" event from a ring,
// waits (host atomic counters, then hipStreamWaitEvent) for its neighbours'
// ready events, launches a 16-block copy kernel from the neighbour's buffer
// into its own, records "done", and waits for the neighbours' done events.
// Used to tell whether a crash under `rocprofv3 --kernel-trace` needs the
// library's code at all.
//
//   tools/mt_launch_probe [threads=8] [steps=3000] [mib_per_thread=64] [serial]
// (serial: the same streams and sequence issued from one host thread)
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

__global__ __launch_bounds__(256) void stream_kernel(const float4 *__restrict__ a,
                                                     float4 *__restrict__ b, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        float4 v = a[i];
        v.x += 1.0f;
        b[i] = v;
    }
}
__global__ __launch_bounds__(256) void copy_kernel(const float2 *__restrict__ s,
                                                   float2 *__restrict__ d, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        d[i] = s[i];
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 8;
    const int steps = argc > 2 ? std::atoi(argv[2]) : 3000;
    const long mib = argc > 3 ? std::atol(argv[3]) : 64;
    constexpr int kR = 4;
    const long n4 = mib * (1 << 20) / 16;
    const long halo = 3 * 4096;  // float2s per exchange (three 4096-px lines)
    CK(hipSetDevice(0));
    std::vector<float4 *> a(n), b(n);
    std::vector<hipStream_t> st(n);
    std::vector<hipEvent_t> evr(n * kR), evd(n * kR);
    for (int r = 0; r < n; r++) {
        CK(hipMalloc(&a[r], n4 * 16));
        CK(hipMalloc(&b[r], n4 * 16));
        CK(hipMemset(a[r], 0, n4 * 16));
        CK(hipMemset(b[r], 0, n4 * 16));
        CK(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
        for (int k = 0; k < kR; k++) {
            CK(hipEventCreateWithFlags(&evr[r * kR + k], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&evd[r * kR + k], hipEventDisableTiming));
        }
    }
    CK(hipDeviceSynchronize());
    if (const char *m = std::getenv("MT_PROBE_MAPS")) {  // to symbolise a crash's frames
        FILE *in = std::fopen("/proc/self/maps", "r"), *out = std::fopen(m, "w");
        if (in && out) {
            char buf[4096];
            size_t k;
            while ((k = std::fread(buf, 1, sizeof buf, in)) > 0) std::fwrite(buf, 1, k, out);
        }
        if (in) std::fclose(in);
        if (out) std::fclose(out);
    }
    std::vector<std::atomic<long>> ready(n), done(n);
    for (int r = 0; r < n; r++) ready[r] = 0, done[r] = 0;
    auto wait = [](const std::atomic<long> &c, long x) {
        while (c.load(std::memory_order_acquire) <= x) std::this_thread::yield();
    };
    const auto t0 = std::chrono::steady_clock::now();
    if (argc > 4 && std::string(argv[4]) == "serial") {
        // the same per-stream sequence from ONE host thread (phases in rank
        // order per step: every wait below is on an event already recorded)
        for (long x = 0; x < steps; x++) {
            const int k = (int)(x % kR);
            for (int r = 0; r < n; r++) {
                float4 *in = (x & 1) ? b[r] : a[r], *out = (x & 1) ? a[r] : b[r];
                hipLaunchKernelGGL(stream_kernel, dim3(128), dim3(256), 0, st[r], in, out, n4);
                CK(hipGetLastError());
                CK(hipEventRecord(evr[r * kR + k], st[r]));
            }
            for (int r = 0; r < n; r++) {
                float4 *out = (x & 1) ? a[r] : b[r];
                for (int q : {r - 1, r + 1}) {
                    if (q < 0 || q >= n) continue;
                    CK(hipStreamWaitEvent(st[r], evr[q * kR + k], 0));
                    const float2 *src = reinterpret_cast<const float2 *>((x & 1) ? a[q] : b[q]);
                    float2 *dst = reinterpret_cast<float2 *>(out) + (q < r ? 0 : halo);
                    hipLaunchKernelGGL(copy_kernel, dim3(16), dim3(256), 0, st[r], src, dst, halo);
                    CK(hipGetLastError());
                }
                CK(hipEventRecord(evd[r * kR + k], st[r]));
            }
            for (int r = 0; r < n; r++)
                for (int q : {r - 1, r + 1})
                    if (q >= 0 && q < n) CK(hipStreamWaitEvent(st[r], evd[q * kR + k], 0));
        }
        CK(hipDeviceSynchronize());
        const double s =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("mt_launch_probe: %d streams x %d steps from one thread, %.3f s, ok\n", n,
                    steps, s);
        return 0;
    }
    std::vector<std::thread> th;
    for (int r = 0; r < n; r++)
        th.emplace_back([&, r] {
            CK(hipSetDevice(0));
            for (long x = 0; x < steps; x++) {
                const int k = (int)(x % kR);
                float4 *in = (x & 1) ? b[r] : a[r], *out = (x & 1) ? a[r] : b[r];
                hipLaunchKernelGGL(stream_kernel, dim3(128), dim3(256), 0, st[r], in, out, n4);
                CK(hipGetLastError());
                CK(hipEventRecord(evr[r * kR + k], st[r]));
                ready[r].store(x + 1, std::memory_order_release);
                for (int q : {r - 1, r + 1}) {
                    if (q < 0 || q >= n) continue;
                    wait(ready[q], x);
                    CK(hipStreamWaitEvent(st[r], evr[q * kR + k], 0));
                    const float2 *src = reinterpret_cast<const float2 *>((x & 1) ? a[q] : b[q]);
                    float2 *dst = reinterpret_cast<float2 *>(out) + (q < r ? 0 : halo);
                    hipLaunchKernelGGL(copy_kernel, dim3(16), dim3(256), 0, st[r], src, dst, halo);
                    CK(hipGetLastError());
                }
                CK(hipEventRecord(evd[r * kR + k], st[r]));
                done[r].store(x + 1, std::memory_order_release);
                for (int q : {r - 1, r + 1}) {
                    if (q < 0 || q >= n) continue;
                    wait(done[q], x);
                    CK(hipStreamWaitEvent(st[r], evd[q * kR + k], 0));
                }
            }
            CK(hipStreamSynchronize(st[r]));
        });
    for (auto &t : th) t.join();
    const double s =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("mt_launch_probe: %d threads x %d steps on one device, %.3f s, ok\n", n, steps, s);
    for (int r = 0; r < n; r++) {
        CK(hipFree(a[r]));
        CK(hipFree(b[r]));
        for (int k = 0; k < kR; k++) {
            CK(hipEventDestroy(evr[r * kR + k]));
            CK(hipEventDestroy(evd[r * kR + k]));
        }
        CK(hipStreamDestroy(st[r]));
    }
    return 0;
}
