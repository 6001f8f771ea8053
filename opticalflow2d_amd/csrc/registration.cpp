// registration.cpp — device-resident registration driver (host C++ over HIP).
//
// Mirrors the control flow of the reference drivers:
//   ImageRegistration::ImageRegistration / estimate_motion   src/ImageRegistration.cpp:49-156
//   ImageRegistrationOpticalFlow::estimate_motion_at_current_resolution
//                                                            src/ImageRegistrationOpticalFlow.cpp:97-151
//   ImageRegistrationDemons::...                             src/ImageRegistrationDemons.cpp:86-137
//   ImageRegistrationFluid::...                              src/ImageRegistrationFluid.cpp:67-142
// The iteration loop is speculative: the host enqueues a chunk of iterations
// without waiting, the fused Logger norms of the whole chunk come back in one
// 16-B-per-iteration read, and the convergence test of Logger.cpp /
// ImageRegistrationOpticalFlow.cpp:131-134 is evaluated on the host.  The
// motion estimate rotates through three buffers, so the chunk's start state is
// never overwritten: when the break fires inside a chunk the iterations up to
// the break are replayed from that state (deterministic, bit-identical).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <hip/hip_ext.h>

#include "of2d_host.h"
#include "of2d_solvers.h"

// the walks' cost counters per iteration to stderr (resolves, raw segments,
// listed tiles, walk clocks; tools/seqnorm_diag.py): a diagnostic build only,
// tools/build_variant.sh sndebug registration.cpp -DOF2D_SN_DEBUG=1
#ifndef OF2D_SN_DEBUG
#define OF2D_SN_DEBUG 0
#endif

namespace of2d {

float logger_error(double sum_diff, double sum_prev, double npx) {
    const float n = (float)npx;
    const float prevnorm = (float)sum_prev / n;
    const float diffnorm = (float)sum_diff / n;
    return prevnorm == 0 ? 0.0f : diffnorm / prevnorm;
}

void HostScratch::ensure(int n) {
    if (n <= cap) return;
    if (sums) (void)hipHostFree(sums);
    if (flt) (void)hipHostFree(flt);
    if (seqh) (void)hipHostFree(seqh);
    if (!status) OF2D_HIP(hipHostMalloc(&status, 64 * sizeof(unsigned)));
    if (!report)
        OF2D_HIP(hipHostMalloc(&report, sizeof(FluidReport) * kFluidReports,
                               hipHostMallocCoherent | hipHostMallocMapped));
    OF2D_HIP(hipHostMalloc(&sums, sizeof(double) * 4 * n));
    OF2D_HIP(hipHostMalloc(&flt, sizeof(float) * 4 * n));
    OF2D_HIP(hipHostMalloc(&seqh, sizeof(float) * 4 * (n + 3),
                           hipHostMallocCoherent | hipHostMallocMapped));
    cap = n;
}
HostScratch::~HostScratch() {
    if (sums) (void)hipHostFree(sums);
    if (flt) (void)hipHostFree(flt);
    if (seqh) (void)hipHostFree(seqh);
    if (status) (void)hipHostFree(status);
    if (report) (void)hipHostFree(report);
}

bool valid_regularisation_parameters(int reg, unsigned np) {
    switch (reg) {
        case 0: return np == 1;
        case 1: return np >= 1 && np <= 2;
        case 2: return np >= 2 && np <= 3;
        case 3: return np == 6;
        case 4: return np == 5;
        case 5: return np >= 2 && np <= 3;
    }
    return false;
}

std::vector<double> gaussian_kernel(int kw, float sigma) {
    std::vector<double> k((size_t)kw * kw);
    const int cx = (int)(((unsigned)kw - 1u) / 2u), cy = cx;
    double weight = 0;
    for (int i = 0; i < kw; i++)
        for (int j = 0; j < kw; j++) {
            const int idx = i + j * kw;
            const float num = (float)(-((i - cx) * (i - cx) + (j - cy) * (j - cy)));
            k[idx] = (double)expf(num / (2 * sigma * sigma));
            weight += k[idx];
        }
    for (auto &v : k) v /= weight;
    return k;
}

static const char kRule[] =
    "%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%%";  // 71 x '%'

Registration::Registration(int dimx, int dimy, int nscales, const int *niter, int nrefine,
                           int reg, const float *params, unsigned nparams, int verbose)
    : dimx_(dimx), dimy_(dimy), nscales_(nscales), nrefine_(nrefine), reg_(reg),
      verbose_(verbose) {
    if (reg < 0 || reg > 5) throw std::invalid_argument("Error: invalid regularisation given\n");
    if (dimx <= 0 || dimy <= 0 || nscales < 0)
        throw std::invalid_argument("Error: invalid image dimensions\n");
    // the kernels index a field's elements with 32-bit unsigned offsets (the
    // reference's own indices are unsigned int, src/Field.tpp:13)
    if (!field_fits_u32(dimx, dimy, 3))
        throw std::invalid_argument("Error: image too large (a field must have < 2^32 elements)\n");
    niter_.assign(niter, niter + nscales + 1);
    params_.assign(params, params + nparams);
    // ImageRegistration.cpp:56-61: dim(dimin.x/scale, dimin.y/scale) with float scale
    ldx_.resize(nscales + 1);
    ldy_.resize(nscales + 1);
    for (int s = nscales; s >= 0; s--) {
        const float scale = (float)std::pow(2, s);
        ldx_[s] = (int)(unsigned)((float)(unsigned)dimx / scale);
        ldy_[s] = (int)(unsigned)((float)(unsigned)dimy / scale);
    }
    // ImageRegistration::display_registration_parameters (ImageRegistration.cpp:6-47),
    // printed before the parameter check exactly like the reference (:80, then set_solver)
    print("%s\n", kRule + 0);
    print("Optical flow image registration started... (2D C++ implementation)...\n");
    print("Registration parameters:\n");
    print("dimensions:\t\t\t\t(%d %d)\n", ldx_[0], ldy_[0]);
    print("niter:\t\t\t\t\t(%d", niter_[0]);
    for (int s = 1; s < nscales + 1; s++) print(" %d", niter_[s]);
    print(")\n");
    print("nscales:\t\t\t\t%d\n", nscales);
    print("nrefine:\t\t\t\t%d\n", nrefine);
    static const char *names[] = {"Diffusion", "Curvature", "Elastic", "Thirions Demons",
                                  "Diffeomorphic Demons", "Fluid"};
    print("regularisation:\t\t\t\t%s\n", names[reg]);
    if (nparams == 1) {
        print("reg. param:\t\t\t\t%.2f\n", (double)params[0]);
    } else if (nparams > 1) {
        print("reg. params:\t\t\t\t(%.2f", (double)params[0]);
        for (unsigned p = 1; p < nparams; p++) print(" %.2f", (double)params[p]);
        print(")\n");
    }
    print("%s\n\n", kRule);
    if (!valid_regularisation_parameters(reg, nparams))
        throw std::invalid_argument(
            "Invalid number of regularisation parameters for given regularisation method.\n");
    for (int s = 0; s <= nscales; s++)
        if (ldx_[s] <= 0 || ldy_[s] <= 0)
            throw std::invalid_argument("Error: pyramid level with zero size\n");
    if (reg == 3 || reg == 4) {  // Demons.cpp:19-23
        const int kw = (int)(unsigned)params[4];
        if (kw < 1) throw std::invalid_argument("Error: Demons kernel width must be >= 1\n");
        kdiff_ = gaussian_kernel(kw, params[2]);
        kfluid_ = gaussian_kernel(kw, params[3]);
    }
}

Registration::~Registration() {
    multi_release();
    if (d_stage_) (void)hipFree(d_stage_);
    if (d_partial_) (void)hipFree(d_partial_);
    if (d_sums_) (void)hipFree(d_sums_);
    if (d_status_) (void)hipFree(d_status_);
    if (d_scalar_) (void)hipFree(d_scalar_);
    lv_.clear();
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    if (ev_join_) (void)hipEventDestroy(ev_join_);
    if (sn_st_) (void)hipStreamDestroy(sn_st_);
    if (fx_st_) (void)hipStreamDestroy(fx_st_);
    for (hipStream_t w : wk_st_)
        if (w) (void)hipStreamDestroy(w);
    for (int k = 0; k < kExactEv; k++) {
        if (ev_step_[k]) (void)hipEventDestroy(ev_step_[k]);
        if (ev_fix_[k]) (void)hipEventDestroy(ev_fix_[k]);
        if (ev_pass_[k]) (void)hipEventDestroy(ev_pass_[k]);
        if (ev_walk_[k]) (void)hipEventDestroy(ev_walk_[k]);
    }
    if (hs_st_) (void)hipStreamDestroy(hs_st_);
    if (st_) (void)hipStreamDestroy(st_);
}

void Registration::set_option(const std::string &key, double v) {
    if (key == "fixed_iters")
        fixed_ = v != 0;
    else if (key == "logger_fp64")
        logger_fp64_ = v != 0;
    else if (key == "ngpus") {
        if (v < 1 || v > kMaxLocalRanks)
            throw std::invalid_argument("option 'ngpus' must be in [1, 16]");
        if ((int)v != ngpus_) multi_release();
        ngpus_ = (int)v;
    }
    else if (key == "ngpus_share") {
        if ((v != 0) != share_) multi_release();
        share_ = v != 0;
    }
    else if (key == "chunk") {
        if (ready_) throw std::invalid_argument("option 'chunk' must be set before first use");
        chunk_ = std::max(1, (int)v);
        chunk_set_ = true;
    }
    else if (key == "hs_gradients_from_image")
        gi_ = v < 0 ? -1 : (v != 0 ? 1 : 0);
    else if (key == "slab_split")
        split_ = v < 0 ? -1 : (v != 0 ? 1 : 0);
    else if (key == "device") {
        if (ready_) throw std::invalid_argument("option 'device' must be set before first use");
        device_ = (int)v;
    } else
        throw std::invalid_argument("unknown option: " + key);
}

void Registration::ensure_device() {
    if (ready_) {
        OF2D_HIP(hipSetDevice(home_));  // the entry point's DeviceScope restores the caller's
        return;
    }
    if (device_ >= 0) OF2D_HIP(hipSetDevice(device_));
    OF2D_HIP(hipGetDevice(&home_));
    OF2D_HIP(hipGetDeviceCount(&ndev_));
    OF2D_HIP(hipDeviceGetAttribute(&ncu_, hipDeviceAttributeMultiprocessorCount, home_));
    int prio_lo = 0, pr = 0;
    OF2D_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &pr));
    OF2D_HIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    // HS's exact loop on CU-masked streams (OF2D_SN_CUMASK; a device or
    // runtime without CU masks gets unmasked streams)
    // (hipExtStreamCreateWithCUMask makes BLOCKING streams: they order against
    // the null stream, so the library keeps its own null-stream calls — the
    // synchronous hipMemcpy / hipMemset of setup and read-back — off the loop)
    std::vector<uint32_t> big((ncu_ + 31) / 32, 0u), small(big.size(), 0u);
    bool masked = false;
    if (OF2D_SN_CUMASK > 0 && OF2D_SN_CUMASK < ncu_) {
        for (int c = 0; c < ncu_; c++) {
            if (c < OF2D_SN_CUMASK) small[c / 32] |= 1u << (c % 32);
            else big[c / 32] |= 1u << (c % 32);
        }
        masked = hipExtStreamCreateWithCUMask(&hs_st_, (uint32_t)big.size(), big.data()) ==
                     hipSuccess &&
                 hipExtStreamCreateWithCUMask(&sn_st_, (uint32_t)big.size(), big.data()) ==
                     hipSuccess;
        if (!masked) {
            (void)hipGetLastError();
            for (hipStream_t *q : {&hs_st_, &sn_st_})
                if (*q) (void)hipStreamDestroy(*q);
            hs_st_ = sn_st_ = nullptr;
        }
    }
    if (masked) {
        tri_slots_ = 4 * (ncu_ - OF2D_SN_CUMASK);
    } else {
        OF2D_HIP(hipStreamCreateWithFlags(&sn_st_, hipStreamNonBlocking));
    }
    if (masked && OF2D_SN_CUMASK_WALK) {
        OF2D_HIP(hipStreamCreateWithPriority(&fx_st_, hipStreamNonBlocking, pr));
        for (hipStream_t &w : wk_st_)
            OF2D_HIP(hipExtStreamCreateWithCUMask(&w, (uint32_t)small.size(), small.data()));
    } else {
        // the fix and the walks at high priority: they are the latency chain that
        // gates the steps (ring) and passes (workspaces) a few groups later, and
        // wait for CUs behind the bandwidth kernels otherwise (4096^2 procedural
        // convergence 148 -> 128 us per iteration, profiles/r04m_exact_pipeline_ab.log)
        OF2D_HIP(hipStreamCreateWithPriority(&fx_st_, hipStreamNonBlocking, pr));
        for (hipStream_t &w : wk_st_)
            OF2D_HIP(hipStreamCreateWithPriority(&w, hipStreamNonBlocking, pr));
    }
    for (int k = 0; k < kExactEv; k++) {
        OF2D_HIP(hipEventCreateWithFlags(&ev_step_[k], hipEventDisableTiming));
        OF2D_HIP(hipEventCreateWithFlags(&ev_fix_[k], hipEventDisableTiming));
        OF2D_HIP(hipEventCreateWithFlags(&ev_pass_[k], hipEventDisableTiming));
        OF2D_HIP(hipEventCreateWithFlags(&ev_walk_[k], hipEventDisableTiming));
    }
    OF2D_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
    OF2D_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    lv_.resize(nscales_ + 1);
    size_t maxnb = 1;
    for (int s = 0; s <= nscales_; s++) {
        Level &L = lv_[s];
        L.dx = ldx_[s];
        L.dy = ldy_[s];
        L.P = pitch_for(L.dx);
        L.Iref.alloc(L.dx, L.dy);
        L.Imov.alloc(L.dx, L.dy);
        L.Iaux.alloc(L.dx, L.dy);
        L.It.alloc(L.dx, L.dy);
        L.motion[0].alloc(L.dx, L.dy);
        L.motion[1].alloc(L.dx, L.dy);
        L.dI.alloc(L.dx, L.dy);
        for (int b = 0; b < 3; b++) L.est[b].alloc(L.dx, L.dy);  // [3..]: exact-norm ring
        solvers::alloc_level(L, reg_);
        maxnb = std::max(maxnb, (size_t)solvers::max_partial_blocks(L, reg_));
    }
    stage_count_ = (size_t)dimx_ * dimy_ * 2;
    OF2D_HIP(hipMalloc(&d_stage_, stage_count_ * sizeof(double)));
    partial_count_ = (size_t)chunk_ * maxnb * 2;
    OF2D_HIP(hipMalloc(&d_partial_, partial_count_ * sizeof(double)));
    OF2D_HIP(hipMalloc(&d_sums_, sizeof(double) * 4 * (size_t)std::max(chunk_, 64)));
    OF2D_HIP(hipMalloc(&d_status_, 64 * sizeof(unsigned)));
    OF2D_HIP(hipMemset(d_status_, 0, 64 * sizeof(unsigned)));
    OF2D_HIP(hipMalloc(&d_scalar_, (16 + 256) * sizeof(float)));
    OF2D_HIP(hipDeviceSynchronize());  // null-stream memset vs the non-blocking stream
    hs_.ensure(std::max(chunk_, 64));
    for (auto &w : d_seqws_) w.alloc(seqnorm_workspace_bytes(dimx_, dimy_));
    d_seq_.alloc(4 * (size_t)(std::max(chunk_, 64) + 3));  // two blocks of run_exact_pipelined
    ready_ = true;
}

// ImageRegistration::set_reference_image / set_moving_image (:103-121)
void Registration::set_images(const double *ref, const double *mov) {
    DeviceScope scope;  // the caller's device again on return
    ensure_device();
    const size_t n0 = (size_t)dimx_ * dimy_;
    Level &L0 = lv_[0];
    for (int which = 0; which < 2; which++) {
        const double *src = which ? mov : ref;
        OF2D_HIP(hipMemcpyAsync(d_stage_, src, n0 * sizeof(double), hipMemcpyHostToDevice, st_));
        Field<float> &dst0 = which ? L0.Imov : L0.Iref;
        launch_d2f(d_stage_, dimx_, dimy_, dst0.p, L0.P, 0, st_);
        for (int s = nscales_; s >= 1; s--) {
            Field<float> &dst = which ? lv_[s].Imov : lv_[s].Iref;
            launch_downsample_image(dst0.p, L0.dx, L0.dy, L0.P, dst.p, lv_[s].dx, lv_[s].dy,
                                    lv_[s].P, st_);
        }
    }
    // Horn-Schunck's iterate ring for the exact Logger (run_exact_pipelined),
    // allocated here rather than inside the first estimate's loop: 13 more
    // fields per level (the other solvers allocate theirs at first use)
    if (reg_ == 0 && exact_norms())
        for (Level &L : lv_)
            for (int b = 3; b <= kRing; b++)
                if (!L.est[b].p) L.est[b].alloc(L.dx, L.dy);
    OF2D_HIP(hipStreamSynchronize(st_));
}

void Registration::check_status() {
    OF2D_HIP(hipMemcpyAsync(hs_.status, d_status_, sizeof(unsigned), hipMemcpyDeviceToHost, st_));
    OF2D_HIP(hipStreamSynchronize(st_));
    check_reported_status(hs_.status[0]);
}

// a status word already read back (after the stream's sync)
void Registration::check_reported_status(unsigned st) {
    if (st) OF2D_HIP(hipMemsetAsync(d_status_, 0, sizeof(unsigned), st_));
    if (st & kStatusDivZero) throw std::runtime_error("Divide by zero exception");
    if (st & kStatusSpinTimeout)
        throw DeviceError("internal error: SOR strip hand-off timed out (results discarded)");
    if (st & kStatusExpBound)
        throw DeviceError("internal error: scaling-and-squaring count above its bound");
}

// ImageRegistration::estimate_motion (:133-156)
void Registration::estimate() {
    DeviceScope scope;  // the caller's device again on return
    ensure_device();
    iters_.clear();
    OF2D_HIP(hipMemsetAsync(d_status_, 0, 64 * sizeof(unsigned), st_));
    Level &L0 = lv_[0];
    for (int s = nscales_; s >= 0; s--) {
        Level &L = lv_[s];
        if (s > 0 && s < nscales_)
            launch_downsample_motion(L0.cur_motion(), L0.dx, L0.dy, L0.P, L.cur_motion(), L.dx,
                                     L.dy, L.P, st_);
        estimate_level(s);
        if (s > 0)
            launch_upsample_motion(L.cur_motion(), L.dx, L.dy, L.P, L0.cur_motion(), L0.dx,
                                   L0.dy, L0.P, st_);
    }
    OF2D_HIP(hipStreamSynchronize(st_));
}

// estimate_motion_at_current_resolution of the three drivers
void Registration::estimate_level(int s) {
    Level &L = lv_[s];
    const int niter = niter_[s];
    const bool demons = (reg_ == 3 || reg_ == 4);
    for (int refine = 0; refine < nrefine_; refine++) {
        // *Iaux = *Imov; Iaux->warp2d(*motion)
        launch_warp(L.Imov.p, L.cur_motion(), L.Iaux.p, L.dx, L.dy, L.P, st_);
        // HS over several devices: the ranks take their gradients themselves
        // (the slabs need >= 3 j-lines each: coarser levels run on one device)
        const int nr = ranks();
        const bool multi = reg_ == 0 && nr > 1 && L.dy >= 3 * nr && L.dx >= 3;
        if (!demons && !multi)
            launch_gradients(L.Iref.p, L.Iaux.p, L.dI.p, L.It.p, L.dx, L.dy, L.P, st_);
        L.est[0].zero(st_);  // motion_est starts at zero (reset() at :141 / new Motion)
        int fin = 0, it = 0;
        switch (reg_) {
            case 0: it = multi ? loop_hs_multi(s, params_[0], fin) : loop_hs(L, niter, params_[0], fin); break;
            case 1: it = loop_curvature(L, niter, fin); break;
            case 2: it = loop_elastic(L, niter, fin); break;
            case 3:
            case 4: it = loop_demons(L, niter, fin); break;
            case 5: it = loop_fluid(L, niter); break;
        }
        iters_.push_back(it);
        // motion->accumulate(*motion_est)
        launch_accumulate(L.motion[L.mcur].p, L.est[fin].p, L.motion[1 - L.mcur].p, L.dx, L.dy,
                          L.P, st_);
        L.mcur ^= 1;
    }
}

void Registration::seqnorm(const Level &L, const float2 *cur, const float2 *prev, int t,
                           const int *stop, int t0) {
    // the profile of the last call predicts this one when it was on the same grid
    const bool use_prof = seq_dx_[0] == L.dx && seq_dy_[0] == L.dy;
    seq_dx_[0] = L.dx;
    seq_dy_[0] = L.dy;
    if (!stop) {
        launch_seqnorm(cur, prev, L.dx, L.dy, L.P, d_seqws_[0].p, use_prof,
                       d_seq_.p + 2 * (size_t)t, nullptr, st_);
        return;
    }
    // launch_seqnorm's three stages, each returning at once past the loop's
    // break (*stop < t0: an iteration the host enqueued ahead of its decision)
    SeqnormBatch B;
    B.K = 1;
    B.u[0] = prev;
    B.u[1] = cur;
    B.ws[0] = d_seqws_[0].p;
    B.use_profile[0] = use_prof;
    B.stop = stop;
    B.t0 = t0;
    launch_seqnorm_pass(B, L.dx, L.dy, L.P, st_);
    launch_seqnorm_refine(B, L.dx, L.dy, L.P, st_);
    B.use_profile[0] = false;
    B.out[0] = d_seq_.p + 2 * (size_t)t;
    launch_seqnorm_walk(B, L.dx, L.dy, L.P, st_);
}

// The chunked loop of run_chunked with the reference's float norms for the
// solvers without a triple (Demons, Elastic, Curvature: single steps).  Every
// iterate must be in memory for its norms, so the iterations run in groups of
// up to three single steps into a ring of the kRing buffers other than the
// chunk's start buffer a (kept for a replay).  The norms of a group run behind
// its steps as one batch (seqnorm_kernels.hip: pair i = iterates t + i - 1,
// t + i): the bandwidth pass on sn_st_, the check and fix on fx_st_ and the
// latency-bound walk on wk_st_[g mod 3], so group g's walk overlaps the steps,
// passes and walks of the groups after it.  Group g works on workspace set
// g mod kSeqSets, whose last walk (group g - kSeqSets) left the profile that
// predicts it (the check corrects the prediction with the fp64 prefix and the
// fix remakes the few tiles it missed); the walk makes the segment entries of
// the tiles it resolves itself.  Iterate m's buffer is read by the walks of
// iterations m - 1 and m; iterate m + kRing rewrites it after both.  HS takes
// run_exact_pipelined.
int Registration::run_chunked_exact(Level &L, int niter, int nb, const StepFn &step,
                                    int &final_buf, const StepFn3M &step3m) {
    if (step3m) return run_exact_pipelined(L, niter, step, final_buf, step3m);
    const double npx = (double)L.dx * L.dy;
    last_err_.clear();
    constexpr int R = kRing;
    static_assert(R + 1 <= (int)(sizeof(L.est) / sizeof(L.est[0])), "ring");
    for (int b = 3; b <= R; b++)
        if (!L.est[b].p) L.est[b].alloc(L.dx, L.dy);
    auto ring = [&](int a, int t) {  // the (t mod R)-th buffer other than a
        const int i = t % R;
        return i < a ? i : i + 1;
    };
    auto src_of = [&](int a, int t) { return t == 0 ? a : ring(a, t - 1); };
    auto ev = [](hipEvent_t *e, int g) { return e[g % kExactEv]; };
    constexpr bool sn_debug = OF2D_SN_DEBUG != 0;
    constexpr int kDbg = 10;
    DevArray<int> dbg;
    if (sn_debug) dbg.alloc(kDbg * (size_t)chunk_);
    // a new loop: each workspace's first call starts from a fresh state
    bool walked[kSeqWs] = {};
    std::vector<int> group_of((size_t)chunk_);
    int a = 0, k0 = 0, g = 0;
    while (k0 < niter) {
        const int C = std::min(chunk_, niter - k0);
        const int g0 = g;  // the chunk's first group
        for (int t = 0; t < C; g++) {
            const int k = std::min(3, C - t);
            for (int m = t; m < t + k; m++) group_of[m] = g;
            // the buffers of iterates t + 1 .. t + k held iterates t + 1 - R ..
            // t + k - R, read by the walks of iterations t - R .. t + k - R
            for (int q = std::max(t - R, 0), last = -1; q <= t + k - R; q++)
                if (group_of[q] != last) {
                    last = group_of[q];
                    OF2D_HIP(hipStreamWaitEvent(st_, ev(ev_walk_, last), 0));
                }
            for (int m = t; m < t + k; m++)
                step(L.est[src_of(a, m)].p, L.est[ring(a, m)].p, d_partial_ + (size_t)m * nb * 2);
            OF2D_HIP(hipEventRecord(ev(ev_step_, g), st_));
            SeqnormBatch B;
            B.K = k;
            B.u[0] = L.est[src_of(a, t)].p;
            for (int i = 0; i < k; i++) {
                const int w = 3 * (g % kSeqSets) + i;
                B.u[i + 1] = L.est[ring(a, t + i)].p;
                B.ws[i] = d_seqws_[w].p;
                B.use_profile[i] = walked[w] && seq_dx_[w] == L.dx && seq_dy_[w] == L.dy;
                seq_dx_[w] = L.dx;
                seq_dy_[w] = L.dy;
                walked[w] = true;
                B.out[i] = d_seq_.p + 2 * (size_t)(t + i);
                B.dbg[i] = sn_debug ? dbg.p + kDbg * (size_t)(t + i) : nullptr;
            }
            enqueue_norms(B, L, g);
            t += k;
        }
        // the last walk of each walk stream
        for (int q = std::max(g - kWalkers, g0); q < g; q++)
            OF2D_HIP(hipStreamWaitEvent(st_, ev(ev_walk_, q), 0));
        OF2D_HIP(hipMemcpyAsync(hs_.flt, d_seq_.p, sizeof(float) * 2 * C, hipMemcpyDeviceToHost,
                                st_));
        check_status();  // synchronises st_ (and with it every norm of the chunk)
        if (sn_debug) print_sn_debug(L, dbg.p, k0, 0, C);
        for (int t = 0; t < C; t++) {
            const int k = k0 + t;
            const float err = logger_error(hs_.flt[2 * t], hs_.flt[2 * t + 1], npx);
            last_err_.push_back(err);
            if (verbose_) print("Iteration: %d\tError:%.4f\n", k, (double)err);
            if (err < 0.001f && k > 1) {  // ImageRegistrationOpticalFlow.cpp:131-134
                // iteration t's buffer was reused by iteration t + R: replay
                if (t + R <= C - 1)
                    for (int r = 0; r <= t; r++)
                        step(L.est[src_of(a, r)].p, L.est[ring(a, r)].p, d_partial_);
                final_buf = ring(a, t);
                return k + 1;
            }
        }
        a = ring(a, C - 1);
        k0 += C;
    }
    final_buf = a;
    return niter;
}

// One group's norms behind its steps (ev_step_[g] recorded on st_): the pass
// on sn_st_ once group g - kSeqSets's walk has left the workspaces, the check
// and fix on fx_st_, the walk on wk_st_[g mod 3]; with B.stop, seqnorm_decide
// after the walk (the sums' copy to seqh_out).  Records ev_walk_[g].
void Registration::enqueue_norms(const SeqnormBatch &B, const Level &L, int g, double npx,
                                 float *seqh_out, bool passed) {
    auto ev = [](hipEvent_t *e, int q) { return e[q % kExactEv]; };
    if (!passed) {
        OF2D_HIP(hipStreamWaitEvent(sn_st_, ev(ev_step_, g), 0));
        if (g >= kSeqSets) OF2D_HIP(hipStreamWaitEvent(sn_st_, ev(ev_walk_, g - kSeqSets), 0));
        launch_seqnorm_pass(B, L.dx, L.dy, L.P, sn_st_);
        OF2D_HIP(hipEventRecord(ev(ev_pass_, g), sn_st_));
    }
    OF2D_HIP(hipStreamWaitEvent(fx_st_, ev(ev_pass_, g), 0));
    launch_seqnorm_refine(B, L.dx, L.dy, L.P, fx_st_);
    OF2D_HIP(hipEventRecord(ev(ev_fix_, g), fx_st_));
    hipStream_t wk = wk_st_[g % kWalkers];
    OF2D_HIP(hipStreamWaitEvent(wk, ev(ev_fix_, g), 0));
    launch_seqnorm_walk(B, L.dx, L.dy, L.P, wk);
    if (B.stop)
        launch_seqnorm_decide(B.out[0], B.K, B.t0, npx, const_cast<int *>(B.stop), seqh_out, wk);
    OF2D_HIP(hipEventRecord(ev(ev_walk_, g), wk));
}

// OF2D_SN_DEBUG builds: iterations [k0 + lo, k0 + hi)'s walk counters (dbg[10 * t])
void Registration::print_sn_debug(const Level &L, const int *dbg, int k0, int lo, int hi) {
    constexpr int kDbg = 10;
    std::vector<int> h(kDbg * (size_t)hi);
    OF2D_HIP(hipMemcpy(h.data(), dbg, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int t = lo; t < hi; t++)
        std::fprintf(stderr,
                     "seqnorm %dx%d it %d: resolves %d %d raw %d %d listed %d walk %d %d "
                     "res %d made %d %d\n",
                     L.dx, L.dy, k0 + t, h[kDbg * t], h[kDbg * t + 1], h[kDbg * t + 2],
                     h[kDbg * t + 3], h[kDbg * t + 4], h[kDbg * t + 5], h[kDbg * t + 6],
                     h[kDbg * t + 7], h[kDbg * t + 8], h[kDbg * t + 9]);
}

// HS's loop with the reference's float norms, pipelined from chunk to chunk.
// The iterations run in triples (step3m: all three iterates stored) into the
// ring est[1 .. kRing] (iterate j >= 1 in est[1 + (j - 1) mod kRing], iterate
// 0 in est[0]), each triple's norms as one batch (enqueue_norms).  The break
// is also taken on the device: after each walk seqnorm_decide applies the
// reference's test to the batch's errors and keeps the first breaking
// iteration in the stop word, and every later triple and norm kernel returns
// at once.  So the host enqueues block b + 1 (chunk_ iterations, whole
// triples) before it reads block b's sums, and the streams never drain
// between blocks; and a break never needs a replay: the triple that would
// overwrite the final iterate t + 1 (with iterate t + 1 + kRing) waits for
// the walk of iteration t and then finds the stop word set.  The tail of one
// or two single steps (niter not a multiple of three; the single step does
// not read the stop word) is enqueued after every earlier block is decided.
int Registration::run_exact_pipelined(Level &L, int niter, const StepFn &step, int &final_buf,
                                      const StepFn3M &step3m) {
    if (hs_st_) {
        // the loop on the masked stream: it runs after st_'s work so far, and
        // st_ runs after the loop (every launch below goes to st_)
        OF2D_HIP(hipEventRecord(ev_fork_, st_));
        OF2D_HIP(hipStreamWaitEvent(hs_st_, ev_fork_, 0));
        std::swap(st_, hs_st_);
        struct Back {
            Registration *r;
            ~Back() {
                std::swap(r->st_, r->hs_st_);
                (void)hipEventRecord(r->ev_join_, r->hs_st_);
                (void)hipStreamWaitEvent(r->st_, r->ev_join_, 0);
            }
        } back{this};
        return run_exact_pipelined_on(L, niter, step, final_buf, step3m);
    }
    return run_exact_pipelined_on(L, niter, step, final_buf, step3m);
}
int Registration::run_exact_pipelined_on(Level &L, int niter, const StepFn &step, int &final_buf,
                                         const StepFn3M &step3m) {
    const double npx = (double)L.dx * L.dy;
    last_err_.clear();
    constexpr int R = kRing;
    static_assert(R + 1 <= (int)(sizeof(L.est) / sizeof(L.est[0])), "ring");
    for (int b = 1; b <= R; b++)
        if (!L.est[b].p) L.est[b].alloc(L.dx, L.dy);
    auto slot = [](int j) { return j == 0 ? 0 : 1 + (j - 1) % R; };
    auto ev = [](hipEvent_t *e, int q) { return e[q % kExactEv]; };
    int *stop = reinterpret_cast<int *>(d_status_ + kStopWord);
    OF2D_HIP(hipMemsetAsync(stop, 0x7f, sizeof(int), st_));  // no break yet
    constexpr int kNoStop = 0x7f7f7f7f;
    // a block: whole triples, few enough groups that no event of a block being
    // read is recorded again before it is (two blocks in flight: the host
    // enqueues one ahead of the one it reads; deeper queues measured no better,
    // profiles/r05q_ahead_ab.log)
    constexpr int kInFlight = 2;
    const int cb = chunk_set_ ? chunk_ : OF2D_SN_BLOCK;
    const int blk = std::min(3 * ((cb + 2) / 3), 3 * (kExactEv / kInFlight - 4));
    const int ring2 = kInFlight * blk;  // the sums' ring: the blocks in flight
    hs_.ensure(std::max(std::max(chunk_, 64), ring2));
    if (d_seq_.n < 2 * (size_t)ring2) d_seq_.alloc(2 * (size_t)ring2);
    constexpr bool sn_debug = OF2D_SN_DEBUG != 0;
    constexpr int kDbg = 10;
    DevArray<int> dbg;
    if (sn_debug) dbg.alloc(kDbg * (size_t)ring2);
    bool walked[kSeqWs] = {};  // a new loop: each workspace starts from a fresh state
    // this loop's tag in the checks' stamps (a stamp of an earlier loop never
    // matches one of this loop's iterations)
    const unsigned epoch = (++exact_epoch_ & 0xfffu) << 20;
    std::vector<int> grp_of((size_t)std::max(niter, 1));
    int g = 0;
    // iterations [t, t + k) as group g (t a multiple of three)
    auto enqueue_group = [&](int t, int k) {
        for (int m = t; m < t + k; m++) grp_of[m] = g;
        // iterates t + 1 .. t + k overwrite iterates t + 1 - R .. t + k - R,
        // read by the walks of iterations t - R .. t + k - R
        for (int q = std::max(t - R, 0), last = -1; q <= t + k - R; q++)
            if (grp_of[q] != last) {
                last = grp_of[q];
                OF2D_HIP(hipStreamWaitEvent(st_, ev(ev_walk_, last), 0));
            }
        if (k == 3)
            step3m(L.est[slot(t)].p, L.est[slot(t + 1)].p, L.est[slot(t + 2)].p,
                   L.est[slot(t + 3)].p, t, -1, -1);
        else
            for (int m = t; m < t + k; m++) step(L.est[slot(m)].p, L.est[slot(m + 1)].p, d_partial_);
        SeqnormBatch B;
        B.K = k;
        B.stop = stop;
        B.t0 = t;
        B.u[0] = L.est[slot(t)].p;
        for (int i = 0; i < k; i++) {
            const int w = 3 * (g % kSeqSets) + i;
            B.u[i + 1] = L.est[slot(t + 1 + i)].p;
            B.ws[i] = d_seqws_[w].p;
            B.use_profile[i] = walked[w] && seq_dx_[w] == L.dx && seq_dy_[w] == L.dy;
            seq_dx_[w] = L.dx;
            seq_dy_[w] = L.dy;
            walked[w] = true;
            B.out[i] = d_seq_.p + 2 * (size_t)((t + i) % ring2);
            B.dbg[i] = sn_debug ? dbg.p + kDbg * (size_t)((t + i) % ring2) : nullptr;
            for (int q = 1; q <= 3; q++)  // the pair's workspaces in groups g - 1 .. g - 3
                if (g - q >= 0) B.near[i][q - 1] = d_seqws_[3 * ((g - q) % kSeqSets) + i].p;
        }
        B.epoch = epoch;
        OF2D_HIP(hipEventRecord(ev(ev_step_, g), st_));
        enqueue_norms(B, L, g, npx, hs_.seqh + 2 * (size_t)(t % ring2));
        g++;
    };
    const int ntrip = niter / 3 * 3;
    const int nbt = (ntrip + blk - 1) / blk;  // blocks of triples
    const int nblocks = nbt + (niter > ntrip ? 1 : 0);  // and the tail
    auto lo_of = [&](int b) { return b < nbt ? b * blk : ntrip; };
    auto hi_of = [&](int b) { return b < nbt ? std::min((b + 1) * blk, ntrip) : niter; };
    std::vector<int> gbeg(nblocks + 1, 0);
    auto enqueue_block = [&](int b) {
        gbeg[b] = g;
        if (b < nbt)
            for (int t = lo_of(b); t < hi_of(b); t += 3) enqueue_group(t, 3);
        else
            enqueue_group(ntrip, niter - ntrip);
        gbeg[b + 1] = g;
    };
    // the other streams' work before st_'s next (the next loop rewrites the
    // ring and the stop word), the status, and the device's break against the
    // host's
    auto finish = [&](int tbreak) {
        std::vector<hipStream_t> side = {sn_st_, fx_st_};
        for (hipStream_t w : wk_st_) side.push_back(w);
        for (hipStream_t s : side) {
            OF2D_HIP(hipEventRecord(ev_join_, s));
            OF2D_HIP(hipStreamWaitEvent(st_, ev_join_, 0));
        }
        OF2D_HIP(hipMemcpyAsync(hs_.status + 1, stop, sizeof(int), hipMemcpyDeviceToHost, st_));
        check_status();  // synchronises st_
        const int dev = static_cast<int>(hs_.status[1]);
        if (dev != (tbreak >= 0 ? tbreak : kNoStop))
            throw DeviceError("internal error: the device's Logger break (" + std::to_string(dev) +
                              ") is not the host's (" + std::to_string(tbreak) + ")");
    };
    // blocks enqueued so far (of the nbt blocks of triples); the host keeps
    // one block queued beyond the one it reads
    int enq = 0;
    if (nblocks > 0) enqueue_block(enq++);
    for (int b = 0; b < nblocks; b++) {
        while (enq < nbt && enq <= b + 1) enqueue_block(enq++);
        // block b's sums: the last walk of each walk stream, then its decide
        for (int q = std::max(gbeg[b + 1] - kWalkers, gbeg[b]); q < gbeg[b + 1]; q++)
            OF2D_HIP(hipEventSynchronize(ev(ev_walk_, q)));
        if (sn_debug) {
            for (int t = lo_of(b); t < hi_of(b); t++) {
                std::vector<int> h(kDbg);
                OF2D_HIP(hipMemcpy(h.data(), dbg.p + kDbg * (size_t)(t % ring2), kDbg * sizeof(int),
                                   hipMemcpyDeviceToHost));
                std::fprintf(stderr,
                             "seqnorm %dx%d it %d: resolves %d %d raw %d %d listed %d walk %d %d "
                             "res %d made %d %d\n",
                             L.dx, L.dy, t, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8],
                             h[9]);
            }
        }
        for (int t = lo_of(b); t < hi_of(b); t++) {
            const float *sm = hs_.seqh + 2 * (size_t)(t % ring2);
            const float err = logger_error(sm[0], sm[1], npx);
            last_err_.push_back(err);
            if (verbose_) print("Iteration: %d\tError:%.4f\n", t, (double)err);
            if (err < 0.001f && t > 1) {  // ImageRegistrationOpticalFlow.cpp:131-134
                finish(t);
                final_buf = slot(t + 1);
                return t + 1;
            }
        }
        if (b + 1 == nbt && nblocks > nbt) enqueue_block(nbt);  // the tail, after the rest
    }
    finish(-1);
    final_buf = slot(niter);
    return niter;
}

// Speculative chunked iteration loop shared by every solver whose iteration
// reads motion_est from one buffer and writes the next iterate to another
// (HS, Demons, Elastic, Curvature).  step(src, dst, partial) enqueues one
// get_update plus the fused Logger partials (nb blocks x {diff, prev}).  With
// step2 (HS), iterations run in pairs fused into one pass, alternating between
// the two buffers other than the chunk's start buffer a, and a single step
// fills an odd tail.  a is never written inside a chunk, so a break at
// iteration t is replayed from it with single steps (iteration t reads
// src_of(a, t) and writes dst_of(a, t)).
int Registration::run_chunked(Level &L, int niter, int nb, const StepFn &step, int &final_buf,
                              const StepFn2 &step2, const StepFn3 &step3, const int *nblk,
                              const StepFn3M &step3m) {
    if (exact_norms()) return run_chunked_exact(L, niter, nb, step, final_buf, step3m);
    const double npx = (double)L.dx * L.dy;
    last_err_.clear();
    if (fixed_ && d_all_.n < 2 * (size_t)niter) {
        d_all_.alloc(2 * (size_t)niter);
        hs_.ensure((niter + 1) / 2);  // 4 doubles per unit of capacity
    }
    const bool use2 = bool(step2), use3 = bool(step3);
    int a = 0, k0 = 0;
    auto src_of = [](int a_, int t) { return t == 0 ? a_ : (t % 2 == 1 ? (a_ + 1) % 3 : (a_ + 2) % 3); };
    auto dst_of = [](int a_, int t) { return t % 2 == 0 ? (a_ + 1) % 3 : (a_ + 2) % 3; };
    while (k0 < niter) {
        const int C = std::min(chunk_, niter - k0);
        auto part = [&](int t) { return d_partial_ + (size_t)t * nb * 2; };
        int end = -1;  // pairs: the buffer holding the chunk's last iterate
        PartialRuns runs;  // which kernel wrote how many block partials per row
        if (use2) {
            // fused launches (triples, then a pair / single tail) alternate
            // between the two buffers other than a
            auto other = [&](int b) { return b == (a + 1) % 3 ? (a + 2) % 3 : (a + 1) % 3; };
            int cur = a, t = 0;
            while (t < C) {
                const int nxt = other(cur);
                if (use3 && C - t >= 3) {
                    step3(L.est[cur].p, L.est[nxt].p, part(t), part(t + 1), part(t + 2));
                    runs.add(t, 3, nblk ? nblk[2] : nb);
                    t += 3;
                } else if (C - t >= 2) {
                    step2(L.est[cur].p, L.est[nxt].p, part(t), part(t + 1));
                    runs.add(t, 2, nblk ? nblk[1] : nb);
                    t += 2;
                } else {
                    step(L.est[cur].p, L.est[nxt].p, part(t));
                    runs.add(t, 1, nblk ? nblk[0] : nb);
                    t += 1;
                }
                cur = nxt;
            }
            end = cur;
        } else {
            for (int t = 0; t < C; t++) step(L.est[src_of(a, t)].p, L.est[dst_of(a, t)].p, part(t));
            runs.add(0, C, nblk ? nblk[0] : nb);
        }
        if (fixed_) {
            // no break to decide: every chunk's sums stay on the device and are
            // read back once after the loop (no host round trip per chunk)
            runs.reduce(d_partial_, nb, d_all_.p + 2 * (size_t)k0, st_);
            a = use2 ? end : dst_of(a, C - 1);
            k0 += C;
            continue;
        }
        runs.reduce(d_partial_, nb, d_sums_, st_);
        OF2D_HIP(hipMemcpyAsync(hs_.sums, d_sums_, sizeof(double) * 2 * C, hipMemcpyDeviceToHost,
                                st_));
        check_status();  // synchronises the stream; throws the reference's runtime_error
        for (int t = 0; t < C; t++) {
            const int k = k0 + t;
            const float err = logger_error(hs_.sums[2 * t], hs_.sums[2 * t + 1], npx);
            last_err_.push_back(err);
            if (verbose_) print("Iteration: %d\tError:%.4f\n", k, (double)err);
            if (!fixed_ && err < 0.001f && k > 1) {  // ImageRegistrationOpticalFlow.cpp:131-134
                // dst(t) was overwritten by iteration t+2, or (pairs) never
                // written: replay single steps from the chunk's start buffer a
                if (use2 || t + 2 <= C - 1)
                    for (int r = 0; r <= t; r++)
                        step(L.est[src_of(a, r)].p, L.est[dst_of(a, r)].p, d_partial_);
                final_buf = dst_of(a, t);
                return k + 1;
            }
        }
        a = use2 ? end : dst_of(a, C - 1);
        k0 += C;
    }
    if (fixed_ && niter > 0) {
        OF2D_HIP(hipMemcpyAsync(hs_.sums, d_all_.p, sizeof(double) * 2 * niter,
                                hipMemcpyDeviceToHost, st_));
        check_status();
        for (int k = 0; k < niter; k++) {
            const float err = logger_error(hs_.sums[2 * k], hs_.sums[2 * k + 1], npx);
            last_err_.push_back(err);
            if (verbose_) print("Iteration: %d\tError:%.4f\n", k, (double)err);
        }
    }
    final_buf = a;
    return niter;
}

// HS iteration loop (ImageRegistrationOpticalFlow.cpp:117-135) with fused Logger
int Registration::loop_hs(Level &L, int niter, float alpha, int &final_buf) {
    const float alphasq = alpha * alpha;  // OpticalFlowDiffusion.cpp:70
    // partial rows long enough for every HS kernel; each row is reduced over
    // the blocks of the kernel that wrote it
    const int nb = hs_partial_blocks(L.P, L.dx, L.dy);
    const int nblk[3] = {hs_nblocks(L.P, L.dy), hs2_nblocks(L.dx, L.dy),
                         hs3_nblocks(L.dx, L.dy)};
    const bool pairs = L.dx >= 2;
    unsigned *range_flag = d_status_ + kRangeFlagWord;
    if (pairs)
        launch_hs_precheck(L.dI.base, L.dI.count, L.P, 1, L.dx, L.dy, alphasq, range_flag,
                           d_status_, st_);
    return run_chunked(
        L, niter, nb,
        [&](const float2 *src, float2 *dst, double *partial) {
            launch_hs_jacobi(src, dst, L.dI.p, L.It.p, L.P, L.dx, L.dy, 0, L.dy, alphasq, partial,
                             d_status_, st_);
        },
        final_buf,
        pairs ? StepFn2([&](const float2 *src, float2 *dst, double *p1, double *p2) {
            // one ghost j-line above and below the level's fields (rows beyond
            // are clamped onto it; they only feed pixels outside the image)
            launch_hs_jacobi2(src, dst, L.dI.p, L.It.p, L.P, L.dx, L.dy, 0, L.dy, alphasq, -1,
                              L.dy + 1, p1, p2, d_status_, st_);
        })
              : StepFn2(),
        pairs ? StepFn3([&](const float2 *src, float2 *dst, double *p1, double *p2, double *p3) {
            // past the MALL the gradients are derived from Iaux in the kernel
            // (dI was taken of it; hs3_gradients_from_image)
            launch_hs_jacobi3(src, dst, L.dI.p, L.It.p, L.P, L.dx, L.dy, 0, L.dy, alphasq, -1,
                              L.dy + 1, p1, p2, p3, d_status_, range_flag, st_, -1, -1,
                              (gi_ < 0 ? hs3_gradients_from_image(L.dx, L.dy) : gi_ != 0)
                                  ? L.Iaux.p
                                  : nullptr);
        })
              : StepFn3(),
        nblk,
        pairs ? StepFn3M([&](const float2 *src, float2 *d1, float2 *d2, float2 *d3, int t0,
                             int band_lo, int band_hi) {
            // the exact Logger's triples: every iterate stored (partials unused)
            launch_hs_jacobi3(src, d3, L.dI.p, L.It.p, L.P, L.dx, L.dy, 0, L.dy, alphasq, -1,
                              L.dy + 1, d_partial_, d_partial_ + (size_t)nb * 2,
                              d_partial_ + (size_t)nb * 4, d_status_, range_flag, st_, band_lo,
                              band_hi,
                              (gi_ < 0 ? hs3_exact_gradients_from_image(L.dx, L.dy) : gi_ != 0)
                                  ? L.Iaux.p
                                  : nullptr,
                              d1, d2, reinterpret_cast<const int *>(d_status_ + kStopWord), t0,
                              tri_slots_);
        })
              : StepFn3M());
}

// WrapperOpticalFlow2d.cpp:105-117 -> Motion::copy_motion_to_input
void Registration::get_motion(double *out) {
    DeviceScope scope;  // the caller's device again on return
    ensure_device();
    Level &L0 = lv_[0];
    launch_motion_to_planar(L0.cur_motion(), L0.P, dimx_, dimy_, d_stage_, st_);
    OF2D_HIP(hipMemcpyAsync(out, d_stage_, sizeof(double) * 2 * dimx_ * dimy_,
                            hipMemcpyDeviceToHost, st_));
    OF2D_HIP(hipStreamSynchronize(st_));
}

// WrapperOpticalFlow2d.cpp:120-137: Imov.set_image; Imov.warp2d(motion[0])
void Registration::warp(const double *in, double *out) {
    DeviceScope scope;  // the caller's device again on return
    ensure_device();
    Level &L0 = lv_[0];
    const size_t n0 = (size_t)dimx_ * dimy_;
    OF2D_HIP(hipMemcpyAsync(d_stage_, in, n0 * sizeof(double), hipMemcpyHostToDevice, st_));
    Field<float> a, b;
    a.alloc(dimx_, dimy_);
    b.alloc(dimx_, dimy_);
    launch_d2f(d_stage_, dimx_, dimy_, a.p, L0.P, 0, st_);
    launch_warp(a.p, L0.cur_motion(), b.p, dimx_, dimy_, L0.P, st_);
    launch_f2d(b.p, L0.P, dimx_, dimy_, d_stage_, st_);
    OF2D_HIP(hipMemcpyAsync(out, d_stage_, n0 * sizeof(double), hipMemcpyDeviceToHost, st_));
    OF2D_HIP(hipStreamSynchronize(st_));
}

}  // namespace of2d
