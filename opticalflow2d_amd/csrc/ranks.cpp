// ranks.cpp — Horn-Schunck over several devices inside ONE process: the
// drop-in boundary's multi-GPU path (of2d_set_option "ngpus", the gateway's
// ninth init argument).
//
// A MATLAB / Octave caller runs one process (WrapperOpticalFlow2d.cpp:13 keeps
// a process-global singleton), so the ranks here are row slabs driven by the
// registration's own host thread, not processes: rank r owns j-lines
// [row_begin, row_end) (of2d_slab_bounds) of every HS level's iteration loop
// on device (device + r) mod count.  Everything around the loop stays on the
// registration's device — pyramid, warp2d, accumulate
// (ImageRegistrationOpticalFlow.cpp:97-151) — and per refine the ranks pull
// their rows of Iref and the warped Iaux (plus one halo j-line each side, for
// the gradients) by peer copy, iterate, and the result rows come back.
//
// One host thread enqueues every rank's work in program order, so each
// cross-rank dependency is an event recorded before it is waited on:
//   halo      before step t a rank copies its neighbours' boundary rows of
//             u_{t-1} into its own ghost j-lines (after their step t-1)
//   Logger    reference-exact (default): each rank's seqnorm tables with the
//             fp64 totals of the ranks before it as the prediction offset
//             (chained rank by rank: a rank reads only its neighbours'
//             memory, the pairs whose peer access multi_for enables), then
//             the walks chained in rank order, rank r starting from rank r-1's
//             exact running sums — the linear order of Motion::norm
//             (Motion.cpp:42-49) crosses the slabs in rank order, so the sums
//             are the one-device sums bit for bit; fp64 (logger_fp64) / fixed
//             iterations: per-rank partial sums, added on the host in rank
//             order
//   reuse     step t writes the ring buffer of iterate t-4: it waits for the
//             readers of that iterate (its own norms of t-4 / t-3 and the
//             neighbours' halo copies before their step t-3)
// The iterations are single Jacobi steps (the one-device default for exact
// norms too); the qlaplacian border rule uses the global j (gradients.h:73), so
// the motion is the one-device motion bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "../../include/of2d.h"
#include "of2d_host.h"

namespace of2d {

struct RankSlab {
    int dev = 0, rb = 0, re = 0, nrows = 0, P = 0;
    hipStream_t st = nullptr, sn = nullptr, wk = nullptr;
    Field<float2> u[5];
    Field<float2> dI;
    Field<float> It, Iref, Iaux;
    DevArray<double> partial, sums, poff;
    DevArray<double> nxt;  // [4][2]: poff + this slab's total per iteration slot (t & 3)
    DevArray<unsigned> status;
    DevArray<unsigned char> ws[2];
    DevArray<float> seq;
    const double *tot[2] = {nullptr, nullptr};
    bool walked[2] = {false, false};
    hipEvent_t ev_step[4] = {}, ev_fix[4] = {}, ev_walk[4] = {}, ev_off[4] = {};
    ~RankSlab() {
        (void)hipSetDevice(dev);
        for (hipStream_t s : {st, sn, wk})
            if (s) (void)hipStreamSynchronize(s);
        for (int k = 0; k < 4; k++)
            for (hipEvent_t e : {ev_step[k], ev_fix[k], ev_walk[k], ev_off[k]})
                if (e) (void)hipEventDestroy(e);
        for (hipStream_t s : {st, sn, wk})
            if (s) (void)hipStreamDestroy(s);
    }
};

struct MultiHS {
    int dx = 0, dy = 0, home = 0;
    std::vector<std::unique_ptr<RankSlab>> r;
};

namespace {
void enable_peer(int a, int b) {
    if (a == b) return;
    OF2D_HIP(hipSetDevice(a));
    const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) OF2D_HIP(e);
    (void)hipGetLastError();  // clear an "already enabled"
}
// dst (on device dd) <- src (on device sd), bytes, on stream st of device dd
void copy(void *dst, int dd, const void *src, int sd, size_t bytes, hipStream_t st) {
    if (dd == sd)
        OF2D_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    else
        OF2D_HIP(hipMemcpyPeerAsync(dst, dd, src, sd, bytes, st));
}
}  // namespace

void Registration::multi_release() {
    DeviceScope scope;  // ~RankSlab switches to each rank's device
    lv_multi_.clear();
}

MultiHS &Registration::multi_for(int s) {
    if ((int)lv_multi_.size() <= s) lv_multi_.resize(s + 1);
    if (lv_multi_[s]) return *lv_multi_[s];
    const Level &L = lv_[s];
    auto m = std::make_shared<MultiHS>();
    m->dx = L.dx;
    m->dy = L.dy;
    DeviceScope scope;  // switched per rank below
    m->home = home_;
    int count = 0;
    OF2D_HIP(hipGetDeviceCount(&count));
    const int n = ngpus_;
    if (n > kMaxLocalRanks) throw std::invalid_argument("ngpus: at most 16 ranks");
    for (int k = 0; k < n; k++) {
        auto R = std::make_unique<RankSlab>();
        R->dev = (m->home + k) % count;
        if (of2d_slab_bounds(L.dy, k, n, &R->rb, &R->re) != OF2D_OK)
            throw std::invalid_argument("ngpus: bad partition");
        R->nrows = R->re - R->rb;
        if (R->nrows < 1) throw std::invalid_argument("ngpus: more ranks than j-lines");
        R->P = L.P;
        enable_peer(R->dev, m->home);
        enable_peer(m->home, R->dev);
        if (k > 0) {
            enable_peer(R->dev, m->r[k - 1]->dev);
            enable_peer(m->r[k - 1]->dev, R->dev);
        }
        OF2D_HIP(hipSetDevice(R->dev));
        for (hipStream_t *s : {&R->st, &R->sn, &R->wk})
            OF2D_HIP(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
        for (int e = 0; e < 4; e++)
            for (hipEvent_t *ev : {&R->ev_step[e], &R->ev_fix[e], &R->ev_walk[e], &R->ev_off[e]})
                OF2D_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        for (auto &f : R->u) f.alloc(L.dx, R->nrows);  // one ghost j-line each side: the halo
        R->dI.alloc(L.dx, R->nrows);
        R->It.alloc(L.dx, R->nrows);
        R->Iref.alloc(L.dx, R->nrows);
        R->Iaux.alloc(L.dx, R->nrows);
        const int nb = hs_nblocks(L.P, R->nrows);
        R->partial.alloc((size_t)nb * 2 * chunk_);
        R->sums.alloc(2 * (size_t)chunk_);
        R->poff.alloc(2);
        R->nxt.alloc(8);
        R->status.alloc(64);
        for (auto &w : R->ws) w.alloc(seqnorm_workspace_bytes(L.dx, R->nrows));
        R->seq.alloc(2 * (size_t)chunk_);
        m->r.push_back(std::move(R));
    }
    OF2D_HIP(hipSetDevice(m->home));
    lv_multi_[s] = m;
    return *m;
}

// ImageRegistrationOpticalFlow::estimate_motion_at_current_resolution's
// iteration loop (:117-135) over the ranks; Iaux is the warped moving image of
// this refine (on the registration's device).  The result goes to L.est[0].
int Registration::loop_hs_multi(int s, float alpha, int &final_buf) {
    Level &L = lv_[s];
    const int niter = niter_[s];
    MultiHS &M = multi_for(s);
    const int n = (int)M.r.size(), home = M.home;
    const float alphasq = alpha * alpha;  // OpticalFlowDiffusion.cpp:70
    const double npx = (double)L.dx * L.dy;
    const bool exact = exact_norms();
    const size_t rowb = (size_t)L.P * sizeof(float2);
    last_err_.clear();
    // the refine's images, rows [rb - 1, re + 1) clipped, into every rank
    OF2D_HIP(hipEventRecord(ev_fork_, st_));
    for (auto &Rp : M.r) {
        RankSlab &R = *Rp;
        OF2D_HIP(hipSetDevice(R.dev));
        OF2D_HIP(hipStreamWaitEvent(R.st, ev_fork_, 0));
        const int lo = std::max(R.rb - 1, 0), hi = std::min(R.re + 1, L.dy);
        const size_t off = (size_t)lo * L.P, bytes = (size_t)(hi - lo) * L.P * sizeof(float);
        const long loc = (long)(lo - R.rb) * L.P;
        copy(R.Iref.p + loc, R.dev, L.Iref.p + off, home, bytes, R.st);
        copy(R.Iaux.p + loc, R.dev, L.Iaux.p + off, home, bytes, R.st);
        // IterativeSolver::set_derivatives on the owned rows (the halo rows
        // feed the one-sided / central y differences at the slab edges)
        launch_gradients_rows(R.Iref.p, R.Iaux.p, R.dI.p, R.It.p, L.dx, R.nrows, L.P, R.rb, L.dy,
                              R.st);
        R.u[0].zero(R.st);  // motion_est starts at zero (:107, :141)
        OF2D_HIP(hipMemsetAsync(R.status.p, 0, 64 * sizeof(unsigned), R.st));
        R.walked[0] = R.walked[1] = false;
    }
    for (auto &Rp : M.r) {  // the first halo copies read the neighbours' zeroed buffers
        OF2D_HIP(hipSetDevice(Rp->dev));
        OF2D_HIP(hipStreamSynchronize(Rp->st));
    }
    auto ring = [](int a, int t) {
        const int i = t & 3;
        return i < a ? i : i + 1;
    };
    auto src_of = [&](int a, int t) { return t == 0 ? a : ring(a, t - 1); };
    // one Jacobi step of every rank from buffer `in` to `out` (halo first);
    // t >= 0: iteration t of the chunk (events, reuse waits), -1: a replay
    auto step_all = [&](int in, int out, int t, bool partials) {
        for (int k = 0; k < n; k++) {
            RankSlab &R = *M.r[k];
            OF2D_HIP(hipSetDevice(R.dev));
            if (t >= 4) {  // `out` held iterate t - 4: its readers first
                if (exact) OF2D_HIP(hipStreamWaitEvent(R.st, R.ev_walk[(t - 3) & 3], 0));
                for (int q : {k - 1, k + 1})
                    if (q >= 0 && q < n)
                        OF2D_HIP(hipStreamWaitEvent(R.st, M.r[q]->ev_step[(t - 3) & 3], 0));
            }
            float2 *u = R.u[in].p;
            if (k > 0) {  // the last owned row above -> ghost row -1
                const RankSlab &A = *M.r[k - 1];
                if (t > 0) OF2D_HIP(hipStreamWaitEvent(R.st, A.ev_step[(t - 1) & 3], 0));
                copy(u - L.P, R.dev, A.u[in].p + (size_t)(A.nrows - 1) * L.P, A.dev, rowb, R.st);
            }
            if (k < n - 1) {  // the first owned row below -> ghost row nrows
                const RankSlab &B = *M.r[k + 1];
                if (t > 0) OF2D_HIP(hipStreamWaitEvent(R.st, B.ev_step[(t - 1) & 3], 0));
                copy(u + (size_t)R.nrows * L.P, R.dev, B.u[in].p, B.dev, rowb, R.st);
            }
            const int nb = hs_nblocks(L.P, R.nrows);
            launch_hs_jacobi(u, R.u[out].p, R.dI.p, R.It.p, L.P, L.dx, R.nrows, R.rb, L.dy,
                             alphasq,
                             R.partial.p + (partials ? (size_t)std::max(t, 0) * nb * 2 : 0),
                             R.status.p, R.st);
            if (t >= 0) OF2D_HIP(hipEventRecord(R.ev_step[t & 3], R.st));
        }
        if (t < 0)  // a replay: every rank's step done before the next one's halo
            for (auto &Rp : M.r) {
                OF2D_HIP(hipSetDevice(Rp->dev));
                OF2D_HIP(hipStreamSynchronize(Rp->st));
            }
    };
    // the reference's float norms of iteration t, rank by rank
    auto norms = [&](int in, int out, int t, int kglob) {
        const int w = kglob & 1;
        bool use_prof[kMaxLocalRanks];
        for (int k = 0; k < n; k++) {
            RankSlab &R = *M.r[k];
            OF2D_HIP(hipSetDevice(R.dev));
            OF2D_HIP(hipStreamWaitEvent(R.sn, R.ev_step[t & 3], 0));
            if (t >= 2) OF2D_HIP(hipStreamWaitEvent(R.sn, R.ev_walk[(t - 2) & 3], 0));
            // the workspace's last walk (two iterations back) predicts this one
            use_prof[k] = R.walked[w];
            R.walked[w] = true;
            launch_seqnorm_pass(R.u[out].p, R.u[in].p, L.dx, R.nrows, L.P, R.ws[w].p,
                                use_prof[k], R.sn);
            R.tot[w] = seqnorm_total(L.dx, R.nrows, L.P, R.ws[w].p, R.sn);
        }
        // the offsets chained in rank order: rank k reads only rank k - 1's
        // slot t & 3, which rank k - 1 rewrites four iterations later, after
        // rank k has read it (the wait on rank k's ev_off of t - 4)
        for (int k = 0; k < n; k++) {
            RankSlab &R = *M.r[k];
            OF2D_HIP(hipSetDevice(R.dev));
            const double *prev_nxt = nullptr;
            if (k > 0) {
                OF2D_HIP(hipStreamWaitEvent(R.sn, M.r[k - 1]->ev_off[t & 3], 0));
                prev_nxt = M.r[k - 1]->nxt.p + 2 * (t & 3);
            }
            if (k < n - 1 && t >= 4) OF2D_HIP(hipStreamWaitEvent(R.sn, M.r[k + 1]->ev_off[t & 3], 0));
            launch_seqnorm_offset_chain(prev_nxt, &R.tot[w], 1, R.poff.p, R.nxt.p + 2 * (t & 3),
                                        R.sn);
            OF2D_HIP(hipEventRecord(R.ev_off[t & 3], R.sn));
            launch_seqnorm_refine(R.u[out].p, R.u[in].p, L.dx, R.nrows, L.P, R.ws[w].p,
                                  use_prof[k], R.poff.p, R.sn);
            OF2D_HIP(hipEventRecord(R.ev_fix[t & 3], R.sn));
        }
        for (int k = 0; k < n; k++) {
            RankSlab &R = *M.r[k];
            OF2D_HIP(hipSetDevice(R.dev));
            OF2D_HIP(hipStreamWaitEvent(R.wk, R.ev_fix[t & 3], 0));
            const float *s_in = nullptr;
            if (k > 0) {
                OF2D_HIP(hipStreamWaitEvent(R.wk, M.r[k - 1]->ev_walk[t & 3], 0));
                s_in = M.r[k - 1]->seq.p + 2 * (size_t)t;
            }
            launch_seqnorm_walk(R.u[out].p, R.u[in].p, L.dx, R.nrows, L.P, R.ws[w].p, s_in,
                                R.seq.p + 2 * (size_t)t, nullptr, R.wk);
            OF2D_HIP(hipEventRecord(R.ev_walk[t & 3], R.wk));
        }
    };
    auto check_status_all = [&] {
        unsigned st = 0;
        for (auto &Rp : M.r) {
            OF2D_HIP(hipSetDevice(Rp->dev));
            OF2D_HIP(hipMemcpyAsync(hs_.status, Rp->status.p, sizeof(unsigned),
                                    hipMemcpyDeviceToHost, Rp->st));
            OF2D_HIP(hipStreamSynchronize(Rp->st));
            st |= hs_.status[0];
        }
        OF2D_HIP(hipSetDevice(home));
        if (st & kStatusDivZero) throw std::runtime_error("Divide by zero exception");
    };
    int a = 0, k0 = 0, done = -1, fin = 0;
    while (k0 < niter && done < 0) {
        const int C = std::min(chunk_, niter - k0);
        for (int t = 0; t < C; t++) {
            step_all(src_of(a, t), ring(a, t), t, !exact);
            if (exact) norms(src_of(a, t), ring(a, t), t, k0 + t);
        }
        // the chunk's Logger sums on the host
        std::vector<double> sums(2 * (size_t)C, 0.0);
        if (exact) {
            RankSlab &Z = *M.r[n - 1];  // the last rank's walk holds the global sums
            OF2D_HIP(hipSetDevice(Z.dev));
            OF2D_HIP(hipMemcpyAsync(hs_.flt, Z.seq.p, sizeof(float) * 2 * C,
                                    hipMemcpyDeviceToHost, Z.wk));
            OF2D_HIP(hipStreamSynchronize(Z.wk));
            for (int i = 0; i < 2 * C; i++) sums[i] = hs_.flt[i];
        } else {
            for (auto &Rp : M.r) {  // per rank in a fixed order, then rank order
                RankSlab &R = *Rp;
                OF2D_HIP(hipSetDevice(R.dev));
                launch_reduce_partials(R.partial.p, hs_nblocks(L.P, R.nrows), C, R.sums.p, R.st);
                OF2D_HIP(hipMemcpyAsync(hs_.sums, R.sums.p, sizeof(double) * 2 * C,
                                        hipMemcpyDeviceToHost, R.st));
                OF2D_HIP(hipStreamSynchronize(R.st));
                for (int i = 0; i < 2 * C; i++) sums[i] += hs_.sums[i];
            }
        }
        for (auto &Rp : M.r) {  // every rank's work of the chunk is done
            OF2D_HIP(hipSetDevice(Rp->dev));
            for (hipStream_t q : {Rp->st, Rp->sn, Rp->wk}) OF2D_HIP(hipStreamSynchronize(q));
        }
        check_status_all();
        for (int t = 0; t < C; t++) {
            const int k = k0 + t;
            const float err = logger_error(sums[2 * t], sums[2 * t + 1], npx);
            last_err_.push_back(err);
            if (verbose_) print("Iteration: %d\tError:%.4f\n", k, (double)err);
            if (!fixed_ && err < 0.001f && k > 1) {  // ImageRegistrationOpticalFlow.cpp:131-134
                if (t + 4 <= C - 1)  // iteration t's buffer was reused: replay
                    for (int q = 0; q <= t; q++) step_all(src_of(a, q), ring(a, q), -1, false);
                fin = ring(a, t);
                done = k + 1;
                break;
            }
        }
        if (done < 0) {
            a = ring(a, C - 1);
            k0 += C;
        }
    }
    if (done < 0) {
        fin = a;
        done = niter;
    }
    // the ranks' rows of motion_est back into L.est[0] on the registration's device
    for (auto &Rp : M.r) {
        RankSlab &R = *Rp;
        OF2D_HIP(hipSetDevice(R.dev));
        copy(L.est[0].p + (size_t)R.rb * L.P, home, R.u[fin].p, R.dev,
             (size_t)R.nrows * L.P * sizeof(float2), R.st);
        OF2D_HIP(hipStreamSynchronize(R.st));
    }
    OF2D_HIP(hipSetDevice(home));
    final_buf = 0;
    return done;
}

}  // namespace of2d
