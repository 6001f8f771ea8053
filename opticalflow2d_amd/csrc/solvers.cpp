// solvers.cpp — solver-specific buffers and iteration loops for the
// regularisations other than Horn-Schunck.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "of2d_host.h"
#include "of2d_solvers.h"

namespace of2d {
namespace solvers {

void alloc_level(Level &L, int reg) {
    switch (reg) {
        case 3:
        case 4:  // Demons.cpp:9-10 (Iwar lives in the force kernel's registers)
            L.corr.alloc(L.dx, L.dy);
            L.tmp.alloc(L.dx, L.dy);
            if (reg == 4) {
                L.force.alloc(L.dx, L.dy);      // exp scratch
                L.increment.alloc(L.dx, L.dy);  // u o exp(c)
            }
            break;
        case 2:  // OpticalFlow::force + Logger prev; SOR hand-off buffers
        case 5:  // + OpticalFlowFluid velocity / increment (OpticalFlowFluid.cpp:50-51)
            L.force.alloc(L.dx, L.dy);
            L.tmp.alloc(L.dx, L.dy);
            L.sorH.alloc(sor_granule_bytes(L.dx, L.dy) / sizeof(unsigned long long));
            L.sorTicket.alloc(reg == 5 ? 1 + (size_t)sor_nstrips(L.dx) : 1);
            if (reg == 5) L.sorCtr.alloc(2);
            L.part.alloc((size_t)increment_nblocks(L.dx, L.dy));
            L.vb.alloc(L.dx, sor_rows(L.dx, L.dy));  // skewed v | b rows; Fluid: v is the velocity
            if (reg == 5) L.increment.alloc(L.dx, L.dy);
            break;
        case 1:  // OpticalFlowCurvature.cpp:36-56 (the force is fused into the rhs kernel)
            L.cbuf[0].alloc(2 * (size_t)L.P * L.dy);
            L.cbuf[1].alloc(2 * (size_t)L.P * L.dy);
            break;
        default:
            break;
    }
}

int max_partial_blocks(const Level &L, int reg) {
    if (reg == 3 || reg == 4) return conv_nblocks(L.dx, L.dy);
    if (reg == 2 || reg == 5) return increment_nblocks(L.dx, L.dy);
    if (reg == 1) return curv_nblocks(L.dx, L.dy);
    return hs_partial_blocks(L.P, L.dx, L.dy);
}

}  // namespace solvers

// Device copies of the two Gaussian kernels: float weights for the sums,
// double weights for boundary weight sums, and the interior weight sum in the
// reference's summation order (Field.tpp:242-256).
struct DemonsKernels {
    float *kf = nullptr;
    double *kd = nullptr;
    int kw = 0;
    double wfull_fluid = 0, wfull_diff = 0;
    ~DemonsKernels() {
        if (kf) (void)hipFree(kf);
        if (kd) (void)hipFree(kd);
    }
};

static double full_weight(const std::vector<double> &k, int kw) {
    const int c = (kw - 1) / 2;
    double w = 0.0;
    for (int ii = -c; ii <= c; ii++)
        for (int jj = -c; jj <= c; jj++) w += k[(ii + c) + (jj + c) * kw];
    return w;
}

// ImageRegistrationDemons::estimate_motion_at_current_resolution loop body
// (ImageRegistrationDemons.cpp:109-121) with DemonsThirions::get_update
// (DemonsThirions.cpp:18-42) / DemonsDiffeomorphic::get_update (:15-35)
int Registration::loop_demons(Level &L, int niter, int &final_buf) {
    const int kw = (int)(unsigned)params_[4];
    if (!demons_k_) {
        demons_k_ = std::make_shared<DemonsKernels>();
        const size_t n = (size_t)kw * kw;
        std::vector<float> kf(2 * n);
        std::vector<double> kd(2 * n);
        for (size_t t = 0; t < n; t++) {
            kf[t] = (float)kfluid_[t];
            kd[t] = kfluid_[t];
            kf[n + t] = (float)kdiff_[t];
            kd[n + t] = kdiff_[t];
        }
        OF2D_HIP(hipMalloc(&demons_k_->kf, sizeof(float) * 2 * n));
        OF2D_HIP(hipMalloc(&demons_k_->kd, sizeof(double) * 2 * n));
        OF2D_HIP(hipMemcpy(demons_k_->kf, kf.data(), sizeof(float) * 2 * n, hipMemcpyHostToDevice));
        OF2D_HIP(hipMemcpy(demons_k_->kd, kd.data(), sizeof(double) * 2 * n, hipMemcpyHostToDevice));
        demons_k_->kw = kw;
        demons_k_->wfull_fluid = full_weight(kfluid_, kw);
        demons_k_->wfull_diff = full_weight(kdiff_, kw);
    }
    const DemonsKernels &K = *demons_k_;
    const size_t n = (size_t)kw * kw;
    // Demons.cpp:48-49
    const float sigma_xsq = params_[1] * params_[1];
    const float sigma_isq = params_[0] * params_[0];
    const bool diffeo = (reg_ == 4);
    int mode = 3;
    if (!diffeo) {
        const int accum = (int)params_[5];  // static_cast<MotionAccumulation>((int) regparams[5])
        mode = accum == 0 ? 0 : (accum == 1 ? 1 : 2);
    }
    // scaling-and-squaring bound: |c| <= 1/(2 sqrt(k)), k = sigma_i^2/sigma_x^2 (AM-GM on
    // Demons.cpp:57's denominator), smoothing keeps the bound, maxabs <= sqrt(2)|c|
    int nsq_max = 32;
    if (diffeo) {
        const double k = (double)sigma_isq / (double)sigma_xsq;
        if (k > 0 && std::isfinite(k)) {
            const double ma = std::sqrt(2.0) / (2.0 * std::sqrt(k));
            nsq_max = std::max(0, (int)std::ceil(1.0 + std::log2(ma)) + 2);
            nsq_max = std::min(nsq_max, 32);
        }
    }
    const int nb = conv_nblocks(L.dx, L.dy);
    const int nparts = 256;
    // the default Logger mode sums the reference's float norms itself
    // (run_chunked_exact): the smoothing pass then computes no partials
    const bool partials = !exact_norms();
    return run_chunked(
        L, niter, nb,
        [&](const float2 *src, float2 *dst, double *partial) {
            // force, correspondence->convolute and the motion update in one
            // pass over the x-interior tiles (diffeomorphic: the smoothed
            // correspondence itself, then exp() and motion->accumulate)
            launch_demons_update(L.Iref.p, L.Iaux.p, src, L.corr.p, L.tmp.p, L.dx, L.dy, L.P,
                                 sigma_isq, sigma_xsq, K.kf, K.kd, kw, K.wfull_fluid,
                                 diffeo ? 3 : mode, d_status_, st_);
            const float2 *umid = L.tmp.p;
            if (diffeo) {
                float2 *cexp = nullptr;
                launch_motion_exp(L.tmp.p, L.force.p, L.dx, L.dy, L.P, nsq_max, d_scalar_ + 16,
                                  nparts, reinterpret_cast<int *>(d_scalar_), d_scalar_ + 1,
                                  d_status_, &cexp, st_);
                launch_accumulate(src, cexp, L.increment.p, L.dx, L.dy, L.P, st_);
                umid = L.increment.p;
            }
            launch_smooth_norm(umid, src, dst, L.dx, L.dy, L.P, K.kf + n, K.kd + n, kw,
                               K.wfull_diff, partials ? partial : nullptr, st_);
        },
        final_buf);
}

// ImageRegistrationFluid::estimate_motion_at_current_resolution loop body
// (ImageRegistrationFluid.cpp:94-125) with OpticalFlowFluid::get_update
// (OpticalFlowFluid.cpp:123-140).  The reference prints a line every
// iteration and may break or regrid after any iteration; both decisions are
// taken on the device (launch_fluid_report_decide: the stop word, the regrid
// word, the motion index) and every kernel of an iteration reads them, so the
// host enqueues kFluidAhead iterations ahead of the report it reads and prints
// the lines from the reports afterwards, in order; the GPU never waits for the
// host between iterations (it did: ~20-28 us per iteration).
// Iterations enqueued past a break return at once.  After a regrid the next
// iteration reads its estimate as zero while the buffer keeps the old
// estimate as the Logger's prev (fluid_zero_est), so no buffer changes role
// on the device's decision: iteration i reads buf[i & 1] and writes
// buf[(i + 1) & 1].
int Registration::loop_fluid(Level &L, int niter) {
    const float mu = params_[0], lambda = params_[1];
    const float omega = params_.size() == 3 ? params_[2] : (float)0.66;  // OpticalFlowFluid.h:10
    L.tmp.zero(st_);  // Logger::prev starts at zero (Logger.cpp:13, new per refine)
    float *scal = d_scalar_ + 8;  // [0] maxabs, [1] dt, [2] min jacobian
    const int nb = increment_nblocks(L.dx, L.dy);
    const double npx = (double)L.dx * L.dy;
    const bool exact = exact_norms();
    last_err_.clear();
    if (niter <= 0) return 0;
    // control words: no break yet, no regrid, the level's motion index
    OF2D_HIP(hipMemsetAsync(d_status_ + kStopWord, 0x7f, sizeof(int), st_));
    OF2D_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_status_ + kFluidRegridWord), 0,
                               1, st_));
    OF2D_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_status_ + kFluidMcurWord),
                               L.mcur, 1, st_));
    const int *stop = reinterpret_cast<const int *>(d_status_ + kStopWord);
    float2 *buf[2] = {L.est[0].p, L.force.p};
    static_assert(kFluidAhead + 2 <= kFluidReports && kFluidAhead + 2 <= kExactEv, "rings");
    // iteration i's device work, up to its report in host memory
    auto enqueue = [&](int i) {
        const FluidCtl c{d_status_, i};
        float2 *in = buf[i & 1], *out = buf[(i + 1) & 1];
        // get_force(force, motion) into vb's b, then the SOR sweep of the
        // velocity (v): the first iteration packs it, later ones find it packed
        // by the previous fluid_step (or repacked by the regrid pass)
        const unsigned ep = ++epoch_;
        if (i == 0)
            launch_sor_pack(L.vb.p, in, L.dI.p, L.It.p, nullptr, L.dx, L.dy, L.P, L.sorH.p, ep,
                            st_);
        else  // after a regrid: gradients of the new warped image + force of est = 0
            launch_regrid_pack(L.Iref.p, L.Iaux.p, L.dI.p, L.It.p, L.vb.p, L.dx, L.dy, L.P,
                               L.sorH.p, ep, st_, c);
        if (sor_increment_workers() != 0) {  // the increment rides behind the sweep
            launch_sor_increment(L.vb.p, L.dx, L.dy, L.P, mu, lambda, omega, L.sorH.p, ep,
                                 L.sorTicket.p, L.sorCtr.p, in, L.increment.p, L.part.p, scal,
                                 d_status_, st_, c);
        } else {
            launch_sor(L.vb.p, L.dx, L.dy, L.P, mu, lambda, omega, L.sorH.p, ep, L.sorTicket.p,
                       d_status_, st_, c);
            launch_increment(in, L.vb.p, L.increment.p, L.dx, L.dy, L.P, L.part.p, scal, st_, c);
        }
        // integrate, Logger, Jacobian and the next iteration's force in one
        // pass; the Logger's prev is L.tmp (zero) in the first iteration, the
        // input buffer's content after (the estimate, or after a regrid the
        // pre-regrid estimate, Logger.cpp:45)
        launch_fluid_step(in, L.increment.p, out, i == 0 ? L.tmp.p : nullptr, scal, L.dI.p,
                          L.It.p, L.vb.p, L.dx, L.dy, L.P, L.sorH.p, ep + 1, d_partial_, L.part.p,
                          st_, c);
        if (exact) seqnorm(L, out, i == 0 ? L.tmp.p : in, 0, stop, i);
        // sums, maxabs, dt, min Jacobian, status, the error and the decisions
        // straight into the host-mapped report; then the regrid if decided
        launch_fluid_report_decide(d_partial_, nb, L.part.p, scal, exact ? d_seq_.p : nullptr,
                                   npx, fixed_, hs_.report + i % kFluidReports, st_, c);
        launch_regrid_if(L.motion[0].p, L.motion[1].p, out, L.Imov.p, L.Iaux.p, L.dx, L.dy, L.P,
                         st_, c);
        OF2D_HIP(hipEventRecord(ev_step_[i % kExactEv], st_));
    };
    int enq = 0, iter;
    for (iter = 0; iter < niter; iter++) {
        while (enq < niter && enq <= iter + kFluidAhead) enqueue(enq++);
        OF2D_HIP(hipEventSynchronize(ev_step_[iter % kExactEv]));
        const FluidReport &r = hs_.report[iter % kFluidReports];
        check_reported_status(r.status);
        print("Dumax: %.3f\tMaxabs increment: %.3f\t Timestep: %.3f\n", (double)0.65f,
              (double)r.maxabs, (double)r.dt);
        last_err_.push_back(r.err);
        if (verbose_) print("Iteration: %d\tError:%.4f\n", iter, (double)r.err);
        if (r.flags & kFluidBreak) {
            iter++;
            break;
        }
        if (r.flags & kFluidRegrid)
            print("Regridding on iteration: %d\tMin Jacobian: %.3f\n", iter, (double)r.jmin);
    }
    // the iterations enqueued past a break are no-ops; then the level's state
    // as the host loop left it: L.est[0] the last estimate (zero after a final
    // regrid, which the next iteration would have read as zero), L.mcur the
    // accumulated motion
    OF2D_HIP(hipMemcpyAsync(hs_.status + 2, d_status_ + kFluidRegridWord, 2 * sizeof(unsigned),
                            hipMemcpyDeviceToHost, st_));
    OF2D_HIP(hipStreamSynchronize(st_));
    if (buf[iter & 1] != L.est[0].p) std::swap(L.est[0], L.force);
    if (hs_.status[2]) L.est[0].zero(st_);
    L.mcur = hs_.status[3] ? 1 : 0;
    return iter;
}

// ImageRegistrationOpticalFlow loop (:123-135) with OpticalFlowElastic::get_update
// (OpticalFlowElastic.cpp:13-19): force from the motion, then the SOR sweep of
// the motion itself (in place).  Chunked like HS; the chunk's start state is
// snapshot so a break inside the chunk is replayed from it.
int Registration::loop_elastic(Level &L, int niter, int &final_buf) {
    const float mu = params_[0], lambda = params_[1];
    const float omega = params_.size() == 3 ? params_[2] : 0.66f;  // OpticalFlowElastic.h:9
    float2 *est = L.est[0].p;
    float2 *snap = L.est[1].p;
    float2 *prev = L.tmp.p;
    L.tmp.zero(st_);
    const int nb = increment_nblocks(L.dx, L.dy);
    const double npx = (double)L.dx * L.dy;
    // get_force(force, motion) then the SOR sweep of the motion itself: pack
    // {u, force} into vb, sweep, unpack (the unpack is fused into the Logger pass)
    auto update = [&]() {
        const unsigned ep = ++epoch_;
        launch_sor_pack(L.vb.p, est, L.dI.p, L.It.p, est, L.dx, L.dy, L.P, L.sorH.p, ep, st_);
        launch_sor(L.vb.p, L.dx, L.dy, L.P, mu, lambda, omega, L.sorH.p, ep, L.sorTicket.p,
                   d_status_, st_);
    };
    last_err_.clear();
    final_buf = 0;
    const bool exact = exact_norms();
    int k0 = 0;
    while (k0 < niter) {
        const int C = std::min(chunk_, niter - k0);
        OF2D_HIP(hipMemcpyAsync(L.est[1].base, L.est[0].base, L.est[0].bytes(),
                                hipMemcpyDeviceToDevice, st_));
        for (int t = 0; t < C; t++) {
            update();
            // the logger pass moves the new motion into est and prev: the
            // exact norms read the previous motion from a copy
            if (exact)
                OF2D_HIP(hipMemcpyAsync(L.force.base, L.tmp.base, L.tmp.bytes(),
                                        hipMemcpyDeviceToDevice, st_));
            launch_logger(L.vb.p, est, prev, L.dx, L.dy, L.P, d_partial_ + (size_t)t * nb * 2,
                          st_);
            if (exact) seqnorm(L, est, L.force.p, t);
        }
        if (exact) {
            OF2D_HIP(hipMemcpyAsync(hs_.flt, d_seq_.p, sizeof(float) * 2 * C,
                                    hipMemcpyDeviceToHost, st_));
        } else {
            launch_reduce_partials(d_partial_, nb, C, d_sums_, st_);
            OF2D_HIP(hipMemcpyAsync(hs_.sums, d_sums_, sizeof(double) * 2 * C,
                                    hipMemcpyDeviceToHost, st_));
        }
        check_status();
        for (int t = 0; t < C; t++) {
            const int k = k0 + t;
            const float err = exact ? logger_error(hs_.flt[2 * t], hs_.flt[2 * t + 1], npx)
                                    : logger_error(hs_.sums[2 * t], hs_.sums[2 * t + 1], npx);
            last_err_.push_back(err);
            if (verbose_) print("Iteration: %d\tError:%.4f\n", k, (double)err);
            if (!fixed_ && err < 0.001f && k > 1) {
                if (t < C - 1) {  // replay up to the break from the chunk's start state
                    OF2D_HIP(hipMemcpyAsync(L.est[0].base, L.est[1].base, L.est[0].bytes(),
                                            hipMemcpyDeviceToDevice, st_));
                    for (int r = 0; r <= t; r++) {
                        update();
                        launch_logger(L.vb.p, est, prev, L.dx, L.dy, L.P, d_partial_, st_);
                    }
                    check_status();
                }
                (void)snap;
                return k + 1;
            }
        }
        k0 += C;
    }
    return niter;
}

// Curvature (OpticalFlowCurvature.cpp:144-167) inside the ImageRegistrationOpticalFlow
// loop.  The transform matrices and eigenvalues depend only on the level's
// dimensions and the parameters, so they are built once per level on the host
// in double (the reference's eigenvalue expression, OpticalFlowCurvature.cpp:6-30;
// the REDFT10 / REDFT01 definitions for the transforms) and uploaded.
namespace {
void build_curvature(Level &L, float alpha, float tau, hipStream_t st) {
    if (L.cE.p) return;
    const int n0 = L.dx, n1 = L.dy, P = L.P;
    const double PI_ = 3.14159265;  // OpticalFlowCurvature.cpp:4
    std::vector<double> h;
    auto upload = [&](DevArray<double> &d) {
        d.alloc(h.size());
        OF2D_HIP(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice,
                                st));
        OF2D_HIP(hipStreamSynchronize(st));
    };
    // REDFT10 along an axis of length n: Y_k = sum_j 2 cos(pi (j + 1/2) k / n) X_j
    auto c10 = [](int k, int j, int n) {
        return 2.0 * std::cos(M_PI * ((double)j + 0.5) * (double)k / (double)n);
    };
    // REDFT01: Y_k = X_0 + sum_{j>=1} 2 cos(pi j (k + 1/2) / n) X_j
    auto c01 = [](int k, int j, int n) {
        return j == 0 ? 1.0 : 2.0 * std::cos(M_PI * (double)j * ((double)k + 0.5) / (double)n);
    };
    // right factors (axis y), column-major n1 x n1: M^T[j][q] = M[q][j]
    h.assign((size_t)n1 * n1, 0.0);
    for (int q = 0; q < n1; q++)
        for (int j = 0; j < n1; j++) h[j + (size_t)q * n1] = c10(q, j, n1);
    upload(L.cC1T);
    for (int q = 0; q < n1; q++)
        for (int j = 0; j < n1; j++) h[j + (size_t)q * n1] = c01(q, j, n1);
    upload(L.cD1T);
    // left factors (axis x), column-major n0 x n0 with leading dimension P
    h.assign((size_t)P * n0, 0.0);
    for (int i = 0; i < n0; i++)
        for (int k = 0; k < n0; k++) h[k + (size_t)i * P] = c10(k, i, n0);
    upload(L.cC0);
    for (int i = 0; i < n0; i++)
        for (int k = 0; k < n0; k++) h[k + (size_t)i * P] = c01(k, i, n0);
    upload(L.cD0);
    // eigenvalues 1 / (1 + tau alpha (-4 + 2 cos(p pi / nx) + 2 cos(q pi / ny))^2)
    h.assign((size_t)P * n1, 0.0);
    const float ta = tau * alpha;
    for (int p = 0; p < n0; p++)
        for (int q = 0; q < n1; q++) {
            const double lam = -4 + 2 * std::cos((unsigned)p * PI_ / (unsigned)n0) +
                               2 * std::cos((unsigned)q * PI_ / (unsigned)n1);
            h[p + (size_t)q * P] = 1.0f / (1.0f + ta * std::pow(lam, 2));
        }
    upload(L.cE);
}
}  // namespace

int Registration::loop_curvature(Level &L, int niter, int &final_buf) {
    const float alpha = params_[0];
    const float tau = params_.size() == 1 ? 1.0f : params_[1];  // OpticalFlowCurvature.h:8
    build_curvature(L, alpha, tau, st_);
    const int n0 = L.dx, n1 = L.dy, P = L.P;
    const long plane = (long)P * n1;
    const float div = 4.0f * (float)((unsigned)n0 * (unsigned)n1);  // 4.0f*sizein
    double *X = L.cbuf[0].p, *T = L.cbuf[1].p;
    return run_chunked(
        L, niter, curv_nblocks(n0, n1),
        [&](const float2 *src, float2 *dst, double *partial) {
            launch_curv_rhs(src, L.dI.p, L.It.p, tau, n0, n1, P, X, plane, st_);
            // forward REDFT10 x REDFT10 (axis y, then axis x with the eigenvalues)
            launch_dgemm(n0, n1, n1, X, P, plane, L.cC1T.p, n1, 0, T, P, plane, nullptr, 0, 2,
                         st_);
            launch_dgemm(n0, n1, n0, L.cC0.p, P, 0, T, P, plane, X, P, plane, L.cE.p, P, 2, st_);
            // inverse REDFT01 x REDFT01
            launch_dgemm(n0, n1, n1, X, P, plane, L.cD1T.p, n1, 0, T, P, plane, nullptr, 0, 2,
                         st_);
            launch_dgemm(n0, n1, n0, L.cD0.p, P, 0, T, P, plane, X, P, plane, nullptr, 0, 2, st_);
            launch_curv_construct(X, plane, src, dst, div, n0, n1, P, partial, st_);
        },
        final_buf);
}

}  // namespace of2d
