// solvers.cpp — solver-specific buffers and iteration loops for the
// regularisations other than Horn-Schunck.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

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
        case 2:
            L.force.alloc(L.dx, L.dy);
            break;
        case 5:
            L.force.alloc(L.dx, L.dy);
            L.velocity.alloc(L.dx, L.dy);
            L.increment.alloc(L.dx, L.dy);
            L.jac.alloc(L.dx, L.dy);
            L.tmp.alloc(L.dx, L.dy);
            break;
        case 1:
            L.force.alloc(L.dx, L.dy);
            break;
        default:
            break;
    }
}

int max_partial_blocks(const Level &L, int reg) {
    if (reg == 3 || reg == 4) return conv_nblocks(L.dx, L.dy);
    return hs_nblocks(L.P, L.dy);
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
    return run_chunked(
        L, niter, nb,
        [&](const float2 *src, float2 *dst, double *partial) {
            launch_demons_force(L.Iref.p, L.Iaux.p, src, L.corr.p, L.dx, L.dy, L.P, sigma_isq,
                                sigma_xsq, d_status_, st_);
            const float2 *umid = L.tmp.p;
            if (!diffeo) {
                launch_smooth_compose(L.corr.p, src, L.tmp.p, L.dx, L.dy, L.P, K.kf, K.kd, kw,
                                      K.wfull_fluid, mode, st_);
            } else {
                // correspondence->convolute; correspondence->exp(); motion->accumulate
                launch_smooth_compose(L.corr.p, src, L.tmp.p, L.dx, L.dy, L.P, K.kf, K.kd, kw,
                                      K.wfull_fluid, 3, st_);
                float2 *cexp = nullptr;
                launch_motion_exp(L.tmp.p, L.force.p, L.dx, L.dy, L.P, nsq_max, d_scalar_ + 16,
                                  nparts, reinterpret_cast<int *>(d_scalar_), d_scalar_ + 1,
                                  d_status_, &cexp, st_);
                launch_accumulate(src, cexp, L.increment.p, L.dx, L.dy, L.P, st_);
                umid = L.increment.p;
            }
            launch_smooth_norm(umid, src, dst, L.dx, L.dy, L.P, K.kf + n, K.kd + n, kw,
                               K.wfull_diff, partial, st_);
        },
        final_buf);
}

int Registration::loop_fluid(Level &, int) {
    throw std::runtime_error("Fluid: not implemented yet");
}
int Registration::loop_elastic(Level &, int, int &) {
    throw std::runtime_error("Elastic: not implemented yet");
}
int Registration::loop_curvature(Level &, int, int &) {
    throw std::runtime_error("Curvature: not implemented yet");
}

}  // namespace of2d
