// ranks.cpp — Horn-Schunck over several devices inside ONE process: the
// drop-in boundary's multi-GPU path (of2d_set_option "ngpus", the gateway's
// ninth init argument).
//
// A MATLAB / Octave caller runs one process (WrapperOpticalFlow2d.cpp:13 keeps
// a process-global singleton), so the ranks here are the row slabs of the
// multi-GPU solver (slab.cpp) in an in-process group: rank r owns j-lines
// [row_begin, row_end) (of2d_slab_bounds) of every HS level's iteration loop
// on device (device + r) mod count, and runs that loop from a host thread of
// its own, as the solver's processes would over RCCL.  Everything around the
// loop stays on the registration's device — pyramid, warp2d, accumulate
// (ImageRegistrationOpticalFlow.cpp:97-151) — and per refine the ranks pull
// their rows of Iref and the warped Iaux (plus three halo j-lines each side)
// by peer copy, take their gradients, iterate, and the motion estimate's rows
// come back.
//
// The slab solver brings the loop's performance path to every rank: fused
// triples with three-line halos exchanged beside the interior bands
// (fixed_iters / logger_fp64), triples that store all three iterates and the
// reference's Logger chained through the ranks (default: each rank's norms in
// batches of three updates, the prediction offsets and the exact walks passed
// from rank to rank, so the break falls on the one-device iteration), and one
// host thread per rank enqueueing whole chunks, meeting the others only at the
// halo and chain hand-offs.  Results are the one-device results bit for bit
// (the qlaplacian border rule takes the global j, gradients.h:73).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <thread>

#include "../../include/of2d.h"
#include "of2d_host.h"

namespace of2d {

// slab.cpp internals for this path
void slab_set_images_device(of2d_slab *s, const float *Iref, const float *Iaux, int srcP,
                            int src_dev);
void slab_copy_estimate(of2d_slab *s, float2 *dst, int dst_dev);

struct MultiHS {
    int dx = 0, dy = 0, home = 0;
    float alpha = 0.0f;
    of2d_slab_group *grp = nullptr;
    std::vector<of2d_slab *> slabs;
    std::vector<int> rb;  // each rank's first j-line
    ~MultiHS() {
        for (of2d_slab *s : slabs)
            if (s) of2d_slab_destroy(s);
        if (grp) of2d_slab_group_destroy(grp);
    }
};

namespace {
// peer access between every pair of the devices used (the halo copies, the
// chained Logger's reads of the neighbour's memory, the fp64 mode's sums)
void enable_peers(const std::vector<int> &devs) {
    for (int a : devs)
        for (int b : devs) {
            if (a == b) continue;
            int ok = 0;
            OF2D_HIP(hipDeviceCanAccessPeer(&ok, a, b));
            if (!ok)
                throw std::invalid_argument("ngpus: devices " + std::to_string(a) + " and " +
                                            std::to_string(b) + " have no peer access");
            OF2D_HIP(hipSetDevice(a));
            const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) OF2D_HIP(e);
            (void)hipGetLastError();  // clear an "already enabled"
        }
}

// a slab call's failure as the registration reports it
void rethrow(int rc, const std::string &msg) {
    if (rc == OF2D_ERR_INVALID_ARGUMENT) throw std::invalid_argument(msg);
    if (rc == OF2D_ERR_DEVICE) throw DeviceError(msg);
    throw std::runtime_error(msg);
}
}  // namespace

void Registration::multi_release() {
    DeviceScope scope;  // destroying a slab switches to its device
    lv_multi_.clear();
}

MultiHS &Registration::multi_for(int s, float alpha) {
    if ((int)lv_multi_.size() <= s) lv_multi_.resize(s + 1);
    if (lv_multi_[s] && lv_multi_[s]->alpha == alpha) return *lv_multi_[s];
    DeviceScope scope;  // switched per rank below
    const Level &L = lv_[s];
    auto m = std::make_shared<MultiHS>();
    m->dx = L.dx;
    m->dy = L.dy;
    m->home = home_;
    m->alpha = alpha;
    int count = 0;
    OF2D_HIP(hipGetDeviceCount(&count));
    const int n = ranks();
    if (n > kMaxLocalRanks) throw std::invalid_argument("ngpus: at most 16 ranks");
    std::vector<int> devs;
    for (int k = 0; k < n; k++) {
        const int d = (m->home + k) % count;
        if (std::find(devs.begin(), devs.end(), d) == devs.end()) devs.push_back(d);
    }
    enable_peers(devs);
    if (of2d_slab_group_create(&m->grp, n) != OF2D_OK)
        throw std::invalid_argument("ngpus: bad rank count");
    for (int k = 0; k < n; k++) {
        of2d_slab *sl = nullptr;
        const int rc = of2d_slab_create_local(&sl, L.dx, L.dy, alpha, k, n, (m->home + k) % count,
                                              m->grp);
        if (rc != OF2D_OK) rethrow(rc, std::string("ngpus: ") + of2d_slab_last_error(nullptr));
        m->slabs.push_back(sl);
        int b = 0, e = 0;
        (void)of2d_slab_bounds(L.dy, k, n, &b, &e);
        m->rb.push_back(b);
    }
    lv_multi_[s] = m;
    return *m;
}

// ImageRegistrationOpticalFlow::estimate_motion_at_current_resolution's
// iteration loop (:117-135) over the ranks; Iaux is the warped moving image of
// this refine (on the registration's device).  The result goes to L.est[0].
int Registration::loop_hs_multi(int s, float alpha, int &final_buf) {
    Level &L = lv_[s];
    const int niter = niter_[s];
    MultiHS &M = multi_for(s, alpha);
    const int n = (int)M.slabs.size();
    last_err_.clear();
    OF2D_HIP(hipStreamSynchronize(st_));  // Iref and the warped Iaux are ready
    for (of2d_slab *sl : M.slabs) {
        auto opt = [&](const char *key, double v) {
            const int rc = of2d_slab_set_option(sl, key, v);
            if (rc != OF2D_OK) rethrow(rc, of2d_slab_last_error(sl));
        };
        opt("logger_fp64", logger_fp64_ ? 1.0 : 0.0);
        opt("hs_gradients_from_image", gi_);
        opt("split", split_);
        slab_set_images_device(sl, L.Iref.p, L.Iaux.p, L.P, M.home);
    }
    // every rank's loop from a thread of its own (each enqueues whole chunks
    // and meets its neighbours at the halo and Logger-chain hand-offs)
    std::vector<int> done(n, 0), rc(n, OF2D_OK);
    std::vector<std::string> msg(n);
    {
        std::vector<std::thread> th;
        for (int k = 0; k < n; k++)
            th.emplace_back([&, k] {
                rc[k] = of2d_slab_run(M.slabs[k], niter, fixed_ ? 1 : 0, &done[k]);
                if (rc[k] != OF2D_OK) msg[k] = of2d_slab_last_error(M.slabs[k]);
            });
        for (auto &t : th) t.join();
    }
    OF2D_HIP(hipSetDevice(M.home));
    for (int k = 0; k < n; k++)
        if (rc[k] != OF2D_OK) {
            // a rank that threw left the group's per-rank counters (halo
            // exchanges, Logger-chain groups) out of step with the others':
            // the next run starts from new slabs
            const int code = rc[k];
            const std::string m = msg[k];
            multi_release();
            rethrow(code, m);
        }
    // the Logger errors are global: every rank holds the same
    const int ne = of2d_slab_last_errors(M.slabs[0], nullptr, 0);
    last_err_.assign(std::max(ne, 0), 0.0f);
    if (ne > 0) of2d_slab_last_errors(M.slabs[0], last_err_.data(), ne);
    if (verbose_)
        for (int k = 0; k < ne; k++) print("Iteration: %d\tError:%.4f\n", k, (double)last_err_[k]);
    // the ranks' rows of motion_est back into L.est[0] on the registration's device
    for (int k = 0; k < n; k++)
        slab_copy_estimate(M.slabs[k], L.est[0].p + (size_t)M.rb[k] * L.P, M.home);
    OF2D_HIP(hipSetDevice(M.home));
    final_buf = 0;
    return done[0];
}

}  // namespace of2d
