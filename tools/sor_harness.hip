// SOR wavefront timeline harness: runs the SOR sweep (sor_block_kernel) on a synthetic
// {v, b} field and prints per-strip start/end times and polled batches.
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -I opticalflow2d_amd/csrc \
//         tools/sor_harness.hip -o tools/sor_harness
//   tools/sor_harness DIMX DIMY [REPS]
// (-DOF2D_SOR_GLEAD=N: granule vectors N batches ahead)
#include "../opticalflow2d_amd/csrc/fluid_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace of2d;

int main(int argc, char **argv) {
    const int dimx = argc > 1 ? atoi(argv[1]) : 8192, dimy = argc > 2 ? atoi(argv[2]) : 8192;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int waves = kSorGLead;  // printed as the variant
    const int P = pitch_for(dimx), ns = sor_nstrips(dimx);
    const size_t rows = (size_t)sor_rows(dimx, dimy) + 1;
    std::vector<float4> h((size_t)rows * P);
    unsigned x = 12345;
    for (auto &q : h) {
        auto rnd = [&]() { x = x * 1664525u + 1013904223u; return (x >> 8) * (1.0f / 16777216.0f) - 0.5f; };
        q = make_float4(rnd(), rnd(), rnd(), rnd());
    }
    float4 *vb;
    void *H;
    unsigned *ticket, *status;
    unsigned long long *trace;
    OF2D_HIP(hipMalloc(&vb, h.size() * sizeof(float4)));
    OF2D_HIP(hipMemcpy(vb, h.data(), h.size() * sizeof(float4), hipMemcpyHostToDevice));
    OF2D_HIP(hipMalloc(&H, sor_granule_bytes(dimx, dimy)));
    OF2D_HIP(hipMemset(H, 0, sor_granule_bytes(dimx, dimy)));
    OF2D_HIP(hipMalloc(&ticket, 4));
    OF2D_HIP(hipMalloc(&status, 4));
    OF2D_HIP(hipMemset(ticket, 0, 4));
    OF2D_HIP(hipMemset(status, 0, 4));
    OF2D_HIP(hipMalloc(&trace, 32 * (size_t)ns));
    // zero motion / gradients / It for the pack (b = 0; the pack only tags
    // granule region 0 and rewrites vb.zw)
    float2 *zf;
    OF2D_HIP(hipMalloc(&zf, (size_t)dimy * P * sizeof(float2)));
    OF2D_HIP(hipMemset(zf, 0, (size_t)dimy * P * sizeof(float2)));
    float4 *vb0 = vb;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> tr(4 * (size_t)ns);
    for (int r = 0; r < reps; r++) {
        const unsigned epoch = r + 1;
        // column-0 granules for strip 0 (what sor_pack writes)
        launch_sor_pack(vb0, zf, zf, (const float *)zf, nullptr, dimx, dimy, P, H, epoch, 0);
        hipEventRecord(e0, 0);
        launch_sor_traced(vb0, dimx, dimy, P, 0.25f, 0.0f, 0.66f, H, epoch, ticket, status, trace, 0);
        hipEventRecord(e1, 0);
        OF2D_HIP(hipDeviceSynchronize());
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned st;
        OF2D_HIP(hipMemcpy(&st, status, 4, hipMemcpyDeviceToHost));
        OF2D_HIP(hipMemcpy(tr.data(), trace, tr.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, t1 = 0, polls = 0;
        for (int i = 0; i < ns; i++) {
            t0 = std::min(t0, tr[4 * i]);
            t1 = std::max(t1, tr[4 * i + 1]);
            polls += tr[4 * i + 2];
        }
        const double steps = dimy + 126.0;
        const double lag = ns > 1 ? (tr[4 * (ns - 1)] - tr[0]) * 0.01 / (ns - 1) : 0;  // us
        double dur = 0;
        for (int i = 0; i < ns; i++) dur += (tr[4 * i + 1] - tr[4 * i]) * 0.01;
        dur /= ns;
        printf("glead %d %dx%d strips %d: %.3f ms (timeline %.3f ms)  start lag %.2f us/strip  strip %.1f us"
               " = %.1f ns/step  polled batches %llu  status %u\n",
               waves, dimx, dimy, ns, ms, (t1 - t0) * 1e-5, lag, dur, dur * 1e3 / steps, polls, st);
        // strip 0 never waits for a neighbour: its cycles per step and clock
        printf("  strip 0: %.1f cycles/step, clock %.3f GHz\n", tr[3] / steps,
               tr[3] / ((tr[1] - tr[0]) * 10.0));
        if (r == reps - 1 && ns > 1) {
            printf("  strip: start_us end_us polls\n");
            for (int i = 0; i < ns; i += std::max(1, ns / 12))
                printf("  %4d: %9.2f %9.2f %llu\n", i, (tr[4 * i] - t0) * 0.01,
                       (tr[4 * i + 1] - t0) * 0.01, tr[4 * i + 2]);
        }
    }
    // final field after `reps` sweeps from the seeded start: identical for
    // every WAVES value when the sweeps are exact
    OF2D_HIP(hipMemcpy(h.data(), vb, h.size() * sizeof(float4), hipMemcpyDeviceToHost));
    unsigned long long hsh = 1469598103934665603ull;
    for (const auto &q : h) {
        unsigned u[4];
        memcpy(u, &q, 16);
        for (int k = 0; k < 4; k++) hsh = (hsh ^ u[k]) * 1099511628211ull;
    }
    printf("glead %d %dx%d reps %d: field hash %016llx\n", waves, dimx, dimy, reps, hsh);
    return 0;
}
