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
#include <algorithm>
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
#ifdef OF2D_SOR_HTRACE
    const size_t ntr = 4 * (size_t)ns + (size_t)ns * kSorHtMax;
#else
    const size_t ntr = 4 * (size_t)ns;
#endif
    OF2D_HIP(hipMalloc(&trace, 8 * ntr));
    // zero motion / gradients / It for the pack (b = 0; the pack only tags
    // granule region 0 and rewrites vb.zw)
    float2 *zf;
    OF2D_HIP(hipMalloc(&zf, (size_t)dimy * P * sizeof(float2)));
    OF2D_HIP(hipMemset(zf, 0, (size_t)dimy * P * sizeof(float2)));
    float4 *vb0 = vb;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> tr(ntr);
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
#ifdef OF2D_SOR_HTRACE
        // hand-off slack: strip I's batch b (ghost rows up to sb + 9) checked
        // ready at T_c(I, b); its producer I-1 publishes row sb + 9 at step
        // sb + 132, i.e. in its batch b + 16 (4.5 steps in)
        if (r == reps - 1 && ns > 12) {
            const int nb = (dimy + 125 + 3) / kSorB + 1;
            auto T = [&](int I, int b) { return tr[4 * ns + (size_t)I * kSorHtMax + b]; };
            std::vector<double> slack, period, lagv;
            long np = 0, nt = 0;
            for (int I = 5; I < ns - 5; I++)
                for (int b = 24; b + 40 < nb; b++) {
                    const unsigned long long c = T(I, b), pr = T(I - 1, b + 16);
                    const unsigned long long m = ~(1ull << 63);
                    slack.push_back(((long long)(c & m) - (long long)(pr & m)) * 0.01);
                    period.push_back(((long long)(T(I, b + 1) & m) - (long long)(c & m)) * 0.01);
                    lagv.push_back(((long long)(c & m) - (long long)(T(I - 1, b) & m)) * 0.01);
                    np += (c >> 63) & 1;
                    nt++;
                }
            auto pct = [](std::vector<double> v, double q) {
                std::sort(v.begin(), v.end());
                return v.empty() ? 0.0 : v[(size_t)(q * (v.size() - 1))];
            };
            printf("  handoff: slack us p10 %.2f p50 %.2f p90 %.2f | batch period us p50 %.3f p90 %.3f |"
                   " strip lag us p50 %.2f | polled %.1f %%\n",
                   pct(slack, 0.1), pct(slack, 0.5), pct(slack, 0.9), pct(period, 0.5),
                   pct(period, 0.9), pct(lagv, 0.5), 100.0 * np / std::max(1l, nt));
            // slack early and late in the sweep, and where the strips poll
            std::vector<double> e, l;
            long pe = 0, pl = 0, pm = 0;
            for (int I = 5; I < ns - 5; I++) {
                const unsigned long long m = ~(1ull << 63);
                e.push_back(((long long)(T(I, 24) & m) - (long long)(T(I - 1, 40) & m)) * 0.01);
                l.push_back(((long long)(T(I, nb - 60) & m) - (long long)(T(I - 1, nb - 44) & m)) * 0.01);
                for (int b = 0; b < nb; b++)
                    if (T(I, b) >> 63) (b < 24 ? pe : (b + 60 < nb ? pm : pl))++;
            }
            printf("  slack us: batch 24 p50 %.2f, batch nb-60 p50 %.2f | polls per strip: first 24 batches %.1f,"
                   " middle %.1f, last 60 %.1f\n",
                   pct(e, 0.5), pct(l, 0.5), (double)pe / (ns - 10), (double)pm / (ns - 10),
                   (double)pl / (ns - 10));
            // one strip's batch periods around its polls
            const int I = ns / 2;
            printf("  strip %d periods (us, * = polled):", I);
            for (int b = 100; b < 160; b++)
                printf(" %.2f%s", ((T(I, b + 1) & ~(1ull << 63)) - (T(I, b) & ~(1ull << 63))) * 0.01,
                       (T(I, b) >> 63) ? "*" : "");
            printf("\n");
        }
#endif
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
