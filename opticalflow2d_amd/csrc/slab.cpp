// slab.cpp — row-slab Horn-Schunck over RCCL (the multi-GPU north-star path).
//
// The global dimx x dimy grid is cut into contiguous slabs of j-lines (the
// memory-slow axis), one per process/GPU.  Iterations run in TRIPLES fused into
// one pass (hs::jacobi3_kernel; a pair or single step fills a chunk's tail):
// the pass computes the first iteration on the owned rows plus two halo rows
// on each side, the second with one, the third on the owned rows, so each slab
// keeps three ghost j-lines of u above and below and, before every fused
// launch of K iterations, sends its first K owned j-lines to the rank above
// and its last K to the rank below (ncclSend/ncclRecv, one group) — the same
// bytes per iteration as a one-line exchange per step, a third of the
// messages.  The exchange runs on its own stream while the interior row bands
// compute; only the outer bands wait for it.  The gradients of the halo rows
// are computed locally from three image halo rows (set_images).  The Logger's
// norms (Logger.cpp:32-51) are fused into the stencil kernels per block,
// reduced per rank, and all-reduced once per chunk of iterations (two doubles
// per iteration) — the host then applies the reference's break test
// (ImageRegistrationOpticalFlow.cpp:131-134).  The border rule of
// gradients::qlaplacian uses the GLOBAL j (gradients.h:73), so the slab result
// equals the single-grid result bit for bit.
//
// The slab path registers with zero initial motion, one level, one refine:
// warp2d by a zero field is the identity (src/Image.cpp:144-173 with fx=fy=0),
// so Iaux == Imov and the gradients are taken of Imov directly.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <thread>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/of2d.h"
#include "of2d_host.h"

#define OF2D_NCCL(call)                                                                   \
    do {                                                                                  \
        ncclResult_t r_ = (call);                                                         \
        if (r_ != ncclSuccess)                                                            \
            throw ::of2d::DeviceError(std::string("RCCL error: ") + ncclGetErrorString(r_)); \
    } while (0)

namespace of2d {
struct SlabExact;  // the reference-exact Logger's state (below)
}

struct of2d_slab {
    int dimx = 0, dimy = 0, rank = 0, nranks = 1, rb = 0, re = 0, nrows = 0, P = 0;
    // convergence-on runs: the Logger's norms as the reference takes them
    // (float running sums in linear order across the slabs, SlabExact), or
    // fp64 sums of the fused partials ("logger_fp64"); fixed_iters runs take
    // no break and always use the fp64 sums.  -1 (auto): the reference's norms
    // except over RCCL with two or more ranks, whose chained walks (ncclSend /
    // ncclRecv on two communicators split from the halo one, beside it on
    // other streams) have not run on hardware: there the fp64 sums unless the
    // caller sets 0
    int logger_fp64 = -1;
    // triples split into interior / edge launches (slab_geometry): -1 when a
    // neighbour is on another device or behind RCCL, 0 never, 1 whenever the
    // slab is tall enough (option "split": tests run the multi-device launch
    // order on co-located slabs)
    int split = -1;
    // a rehearsal of the RCCL halo on one GPU (option "rccl_self_halo", tests
    // only): a one-rank communicator sends its boundary j-lines to itself into
    // a scratch buffer at every exchange, and its triples take the split
    // launches, so ncclGroupStart / ncclSend / ncclRecv run on comm_st between
    // the interior and edge launches as on an N-rank communicator; the motion
    // is untouched (the scratch is never read)
    int self_halo = 0;
    float *d_selfx = nullptr;
    of2d::SlabExact *ex = nullptr;
    int device = 0;
    float alpha = 0.0f;
    hipStream_t st = nullptr;
    hipStream_t comm_st = nullptr;  // the halo exchange, overlapped with interior bands
    // split launches (slab.cpp fused): the latest work on st that comm_st must
    // see (an interior launch, or a pair / single step) and the latest edge
    // launches on comm_st that st must see
    hipEvent_t ev_int = nullptr, ev_edge = nullptr;
    ncclComm_t comm = nullptr;
    of2d_slab_group *grp = nullptr;  // in-process transport instead of RCCL
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;  // its all-reduce handshakes
    // its halo handshakes (local_exchange): a ring of event pairs, one per
    // exchange in flight, and the exchanges it has enqueued over its life
    static constexpr int kXr = 4;
    hipEvent_t ev_xr[kXr] = {}, ev_xd[kXr] = {};
    long nx = 0;
    double *d_red = nullptr;  // its all-reduce result staging
    of2d::Field<float2> u[3];
    of2d::Field<float2> dI;
    of2d::Field<float> It, Iref, Imov;
    double *d_partial = nullptr, *d_sums = nullptr, *d_stage = nullptr;
    double *d_all = nullptr;  // fixed_iters: the sums of every iteration of a run
    size_t all_cap = 0;
    unsigned *d_status = nullptr;
    of2d::HostScratch hs;
    int chunk = 33;  // eleven fused triples per chunk
    // a fixed-iteration run has no break to replay, so its chunks only set how
    // often the partial rows are reduced: 33 triples per reduction launch
    int chunk_fixed = 99;
    int chunk_cap() const { return chunk > chunk_fixed ? chunk : chunk_fixed; }
    int fin = 0;    // buffer holding the final motion
    int start = 0;  // zeroed buffer the next run starts from (motion_est->reset())
    // a run began and has not re-zeroed `start` (it threw midway): the next
    // run zeroes it first
    bool start_dirty = false;
    // the triple kernel takes the gradients from Iaux (= Imov) instead of dI:
    // -1 by slab size (of2d::hs3_gradients_from_image), 0 / 1 forced
    int gi = -1;
    // set_images' divide-by-zero test (dI is fixed per image pair): this rank's
    // result, and whether the ranks have voted on it yet (first run after
    // set_images; set_images itself need not be called by all ranks together)
    bool divzero_local = false, divzero_voted = false, divzero = false;
    double last_ms = 0.0;
    std::vector<float> errs;
    std::string err;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // the triple launches of the first kTriTimed chunks of a run, bracketed by
    // event pairs on st (after the edge launches have joined it): the dominant
    // kernel's own launch time inside the run, for the roofline report
    static constexpr int kTriTimed = 64;
    hipEvent_t ev_tri[2 * kTriTimed] = {};
    int tri_pairs = 0, tri_launches = 0;
    double tri_us = 0.0;  // average per triple launch of the last run
    int tri_n = 0;        // triple launches that average covers
    // the halo's cost, sampled on the first kHaloTimed split triples of a run
    // (five events each, so that the other launches keep no extra packets):
    // st before / after its wait on the previous edge launches (the stall the
    // halo puts on the interior), comm_st before / after the exchange and after
    // the two edge launches
    static constexpr int kHaloTimed = 8;
    hipEvent_t ev_halo[5 * kHaloTimed] = {};
    int halo_n = 0;  // sampled in this run so far
    double halo_us[3] = {};  // last run: stall, exchange, edges (us per sampled launch)
    int halo_samples = 0;
};

// The ranks of one grid inside ONE process, one host thread per rank: halos
// and the Logger all-reduce move by device copies ordered with events, and the
// host threads meet at a barrier per exchange.  Same slab code, same launches,
// same halo lines as the RCCL path; it exists so that the decomposition can run
// on a single GPU, where RCCL refuses two ranks on one device.
struct of2d_slab_group {
    int n = 0;
    // exact Logger: per rank, the groups whose offset / walk it has enqueued
    // (the next rank waits for its neighbour's count before waiting on the
    // neighbour's event); groups are counted over the slabs' lifetime
    std::unique_ptr<std::atomic<long>[]> off_done, walk_done;
    // halo exchanges (local_exchange): per rank, the exchanges whose ready /
    // done record it has enqueued, and the buffer it published for each slot
    std::unique_ptr<std::atomic<long>[]> xr_ready, xr_done;
    std::vector<const void *> xptr;  // [rank * kXr + slot]
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    std::vector<of2d_slab *> slabs;
    std::vector<const void *> ptr;  // per rank: the buffer published for this exchange
    std::vector<char> flag;          // per rank: any_rank's vote
    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        const long my = gen;
        if (++arrived == n) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return gen != my; }))
            throw std::runtime_error("slab group: a rank did not reach the exchange");
    }
};

namespace {
thread_local std::string g_create_err;

template <class F>
int sguard(of2d_slab *s, F &&f) {
    try {
        // every entry point binds the calling thread to the slab's device (a
        // caller may have switched it since create)
        if (s && s->P > 0) OF2D_HIP(hipSetDevice(s->device));
        f();
        if (s) s->err.clear();
        return OF2D_OK;
    } catch (const std::invalid_argument &e) {
        if (s) s->err = e.what();
        return OF2D_ERR_INVALID_ARGUMENT;
    } catch (const of2d::DeviceError &e) {
        if (s) s->err = e.what();
        return OF2D_ERR_DEVICE;
    } catch (const std::exception &e) {
        if (s) s->err = e.what();
        return OF2D_ERR_RUNTIME;
    }
}

// in-process group: wait until `cnt` (a rank's count of enqueued records)
// passes x
void wait_count(const std::atomic<long> &cnt, long x, const char *what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0; cnt.load(std::memory_order_acquire) <= x; spin++) {
        if (spin > 64) std::this_thread::yield();
        if ((spin & 1023) == 1023 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
            throw std::runtime_error(std::string("slab group: a rank did not reach the ") + what);
    }
}

// in-process transport, point to point: every rank publishes `u` once its
// boundary lines are final (its ready record of exchange x), pulls its
// neighbours' lines into its own ghost lines, and does not run ahead until the
// neighbours have pulled from it (their done records).  The host threads meet
// only their neighbours and only to see an event RECORDED (enqueued), never
// completed, so each runs ahead enqueueing whole chunks; the event pairs are a
// ring of kXr, which is safe from x + 1 on: a rank publishes done(x) after
// its wait on the neighbour's ready(x) was enqueued, and waits for the
// neighbours' done(x) before its exchange x + 1.
void local_exchange(of2d_slab *s, float2 *u, int lines, size_t cnt, hipStream_t st) {
    of2d_slab_group *g = s->grp;
    constexpr int kXr = of2d_slab::kXr;
    const long P = s->P;
    const size_t bytes = cnt * sizeof(float);
    const long x = s->nx++;
    const int k = (int)(x % kXr);
    for (int r = 0; r < s->nranks; r++)
        if (!g->slabs[r]) throw std::invalid_argument("slab group: not every rank was created");
    OF2D_HIP(hipEventRecord(s->ev_xr[k], st));
    g->xptr[(size_t)s->rank * kXr + k] = u;
    g->xr_ready[s->rank].store(x + 1, std::memory_order_release);
    const int nbr[2] = {s->rank - 1, s->rank + 1};
    for (int q : nbr) {
        if (q < 0 || q >= s->nranks) continue;
        wait_count(g->xr_ready[q], x, "halo exchange");
        const of2d_slab *o = g->slabs[q];
        const float2 *src = static_cast<const float2 *>(g->xptr[(size_t)q * kXr + k]);
        OF2D_HIP(hipStreamWaitEvent(st, o->ev_xr[k], 0));
        // its last lines into the ghost lines above row 0, or its first lines
        // below the last row
        float2 *dst = q < s->rank ? u - lines * P : u + (long)s->nrows * P;
        const float2 *from = q < s->rank ? src + (long)(o->nrows - lines) * P : src;
        if (o->device == s->device)  // a few blocks, beside the other ranks' triples
            of2d::launch_copy_lines(dst, from, bytes, st);
        else
            OF2D_HIP(hipMemcpyAsync(dst, from, bytes, hipMemcpyDeviceToDevice, st));
    }
    OF2D_HIP(hipEventRecord(s->ev_xd[k], st));
    g->xr_done[s->rank].store(x + 1, std::memory_order_release);
    for (int q : nbr) {
        if (q < 0 || q >= s->nranks) continue;
        wait_count(g->xr_done[q], x, "halo exchange");
        OF2D_HIP(hipStreamWaitEvent(st, g->slabs[q]->ev_xd[k], 0));
    }
}

// `lines` (1..3) boundary j-lines to each neighbour, on stream `st`
void halo_exchange(of2d_slab *s, float2 *u, int lines, hipStream_t st) {
    const long P = s->P;
    // lines are contiguous at pitch P: 2 floats per px, the padding travels too
    const size_t cnt = 2 * ((size_t)(lines - 1) * P + (size_t)s->dimx);
    if (s->nranks == 1) {
        if (!(s->self_halo && s->comm)) return;
        const size_t cap = 2 * ((size_t)2 * P + (size_t)s->dimx);  // three lines
        if (!s->d_selfx) OF2D_HIP(hipMalloc(&s->d_selfx, 2 * cap * sizeof(float)));
        for (int side = 0; side < 2; side++) {  // one peer op pair per group, as below
            OF2D_NCCL(ncclGroupStart());
            OF2D_NCCL(ncclSend(side ? u + (long)(s->nrows - lines) * P : u, cnt, ncclFloat, 0,
                               s->comm, st));
            OF2D_NCCL(ncclRecv(s->d_selfx + side * cap, cnt, ncclFloat, 0, s->comm, st));
            OF2D_NCCL(ncclGroupEnd());
        }
        return;
    }
    if (s->grp) return local_exchange(s, u, lines, cnt, st);
    OF2D_NCCL(ncclGroupStart());
    if (s->rank > 0) {
        OF2D_NCCL(ncclSend(u, cnt, ncclFloat, s->rank - 1, s->comm, st));
        OF2D_NCCL(ncclRecv(u - lines * P, cnt, ncclFloat, s->rank - 1, s->comm, st));
    }
    if (s->rank < s->nranks - 1) {
        OF2D_NCCL(ncclSend(u + (long)(s->nrows - lines) * P, cnt, ncclFloat, s->rank + 1,
                           s->comm, st));
        OF2D_NCCL(ncclRecv(u + (long)s->nrows * P, cnt, ncclFloat, s->rank + 1, s->comm, st));
    }
    OF2D_NCCL(ncclGroupEnd());
}

// true on every rank if `mine` is true on any rank (host-side; synchronises)
bool any_rank(of2d_slab *s, bool mine) {
    if (s->nranks == 1 && !s->comm) return mine;
    if (s->grp) {
        of2d_slab_group *g = s->grp;
        g->flag[s->rank] = mine;
        g->barrier();
        bool any = false;
        for (char f : g->flag) any = any || f;
        g->barrier();  // nobody votes again before everyone has read
        return any;
    }
    unsigned v = mine ? 1u : 0u;
    unsigned *w = s->d_status + of2d::kRangeFlagWord + 1;
    OF2D_HIP(hipMemcpyAsync(w, &v, sizeof v, hipMemcpyHostToDevice, s->st));
    OF2D_NCCL(ncclAllReduce(w, w, 1, ncclUint32, ncclMax, s->comm, s->st));
    OF2D_HIP(hipMemcpyAsync(&v, w, sizeof v, hipMemcpyDeviceToHost, s->st));
    OF2D_HIP(hipStreamSynchronize(s->st));
    return v != 0;
}

// sum of `count` doubles over the ranks, in place, on stream `st`
void allreduce_sums(of2d_slab *s, double *buf, size_t count, hipStream_t st) {
    if (s->nranks == 1 && !s->comm) return;
    if (!s->grp) {
        OF2D_NCCL(ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, s->comm, st));
        return;
    }
    // in-process: every rank adds all ranks' buffers in rank order into its
    // own staging, then copies it back once every rank has read every buffer
    of2d_slab_group *g = s->grp;
    OF2D_HIP(hipEventRecord(s->ev_ready, st));
    g->ptr[s->rank] = buf;
    g->barrier();
    std::vector<const double *> src(s->nranks);
    for (int r = 0; r < s->nranks; r++) {
        if (r != s->rank) OF2D_HIP(hipStreamWaitEvent(st, g->slabs[r]->ev_ready, 0));
        src[r] = static_cast<const double *>(g->ptr[r]);
    }
    of2d::launch_sum_ranks(src.data(), s->nranks, count, s->d_red, st);
    OF2D_HIP(hipEventRecord(s->ev_done, st));
    g->barrier();
    for (int r = 0; r < s->nranks; r++)
        if (r != s->rank) OF2D_HIP(hipStreamWaitEvent(st, g->slabs[r]->ev_done, 0));
    OF2D_HIP(hipMemcpyAsync(buf, s->d_red, count * sizeof(double), hipMemcpyDeviceToDevice, st));
}
// Launch geometry of a slab's triples.  With neighbours on other devices (or
// over RCCL) and at least 3E j-lines the launch is split (see fused in
// of2d_slab_run): interior j-lines [E, nrows-E) with a block budget that leaves room for the two edge launches
// of E = 16 j-lines (4 waves x 4 lines, one block per strip) and for the RCCL
// send/recv kernel (kCommBlocks) to be resident beside it.  At 4096 x 4096 per
// rank: 27 x 38-line interior bands (945 blocks) + 2 x 35 edge blocks, 104 us
// per three iterations against 99 us for the unsplit launch
// (tools/hs_variants split; the earlier interior-then-outer-bands order on one
// stream took 149 us).
struct SlabGeometry {
    bool split = false;
    int slots = 1024;  // block slots of an unsplit triple (triple_slots)
    int E = 16, re = 4;  // edge j-lines, j-lines per wave in an edge launch
    int ri = 0, bi = 0;  // interior j-lines per wave and block rows
    int n3 = 0;          // block partials a triple writes
    int nb = 0;          // partial row length for every kernel of the slab
};
bool use_gi(const of2d_slab *s) {
    return s->gi < 0 ? of2d::hs3_gradients_from_image(s->dimx, s->nrows) : s->gi != 0;
}
// the exact-Logger loop's triples (run_exact): its passes stream the iterates
// beside them (of2d::hs3_exact_gradients_from_image)
bool use_gi_exact(const of2d_slab *s) {
    return s->gi < 0 ? of2d::hs3_exact_gradients_from_image(s->dimx, s->nrows) : s->gi != 0;
}
// the motion buffer holding neither the result nor the next run's zeroed start
int scratch_buffer(const of2d_slab *s) {
    for (int b = 0; b < 3; b++)
        if (b != s->fin && b != s->start) return b;
    return 0;
}

// room for the per-iteration sums of a fixed_iters run of niter iterations
void reserve_sums(of2d_slab *s, int niter) {
    if (s->all_cap >= 2 * (size_t)niter) return;
    if (s->d_all) OF2D_HIP(hipFree(s->d_all));
    s->d_all = nullptr;
    s->all_cap = 0;
    OF2D_HIP(hipMalloc(&s->d_all, sizeof(double) * 2 * (size_t)niter));
    s->all_cap = 2 * (size_t)niter;
    s->hs.ensure((niter + 1) / 2);  // 4 doubles per unit of capacity
}

// an exchange partner of this slab is on another device, or behind RCCL (the
// split launches hide the exchange's latency; between slabs of one device it
// is a local copy of a few lines, cheaper than the edge launches: 16 of 11.5
// us per triple at 8 ranks on one device, profiles/r04n_ranks8_fixed_kernel_stats.csv)
bool remote_neighbour(const of2d_slab *s) {
    if (!s->grp) return s->nranks > 1;
    for (int q : {s->rank - 1, s->rank + 1})
        if (q >= 0 && q < s->nranks && s->grp->slabs[q] && s->grp->slabs[q]->device != s->device)
            return true;
    return false;
}

// the slab is tall enough for the interior / edge split (two E-line edges and
// an interior of at least E lines)
bool can_split_shape(const of2d_slab *s) {
    return s->nrows >= 3 * SlabGeometry().E && s->dimx >= 2;
}
bool can_split(const of2d_slab *s) {
    return (s->nranks > 1 || (s->self_halo && s->comm)) && can_split_shape(s);
}
// Block slots a whole-slab triple may take: the device's 1024 (4 per CU), or,
// with k > 1 slabs of an in-process group on this device, 1024 / min(k, 4) —
// their triples run side by side (up to four at once, one per hardware
// queue), so each takes longer bands in fewer blocks instead of a whole
// device's worth of short ones (512-row slabs of 4096: 245 blocks of 19-line
// bands rather than 910 of 5-line bands, whose halo rows and prologue
// double the work per pixel; profiles/r05f_ranks_attribution.txt)
#ifndef OF2D_SLAB_SHARE_Q
#define OF2D_SLAB_SHARE_Q 2  // slabs assumed to run side by side (A/B knob; 1: none)
#endif
int triple_slots(const of2d_slab *s) {
    if (!s->grp) return 1024;
    int k = 0;
    for (const of2d_slab *o : s->grp->slabs)
        if (o && o->device == s->device) k++;
    return k > 1 ? 1024 / std::min(k, OF2D_SLAB_SHARE_Q) : 1024;
}
SlabGeometry slab_geometry_as(const of2d_slab *s, bool split, int slots = 1024,
                              bool any_ranks = false) {
    SlabGeometry g;
    const int gx = (s->dimx + of2d::kHs3Out - 1) / of2d::kHs3Out;
    g.split = split && (any_ranks ? can_split_shape(s) : can_split(s));
    g.slots = slots;
    if (g.split) {
        const int ni = s->nrows - 2 * g.E;
        constexpr int kCommBlocks = 8;
        g.ri = of2d::hs3_rows(s->dimx, ni, std::max(gx, 1024 - 2 * gx - kCommBlocks));
        g.bi = (ni + of2d::kHs3Waves * g.ri - 1) / (of2d::kHs3Waves * g.ri);
        g.n3 = gx * (g.bi + 2);
    } else {
        const int r = of2d::hs3_rows(s->dimx, s->nrows, slots);
        g.n3 = gx * ((s->nrows + of2d::kHs3Waves * r - 1) / (of2d::kHs3Waves * r));
    }
    g.nb = std::max(of2d::hs_partial_blocks(s->P, s->dimx, s->nrows), g.n3);
    return g;
}
SlabGeometry slab_geometry(const of2d_slab *s) {
    return slab_geometry_as(s, s->split > 0 || (s->split < 0 && remote_neighbour(s)),
                            triple_slots(s));
}
// partial-row length for every geometry: the allocation at create, before the
// group's other slabs (whose devices decide the split and the slots) or the
// options are known (the split shape whatever the rank count: rccl_self_halo
// splits a one-rank slab)
int partial_blocks_cap(const of2d_slab *s) {
    int nb = slab_geometry_as(s, true, 1024, true).nb;
    for (int slots : {1024, 512, 341, 256}) nb = std::max(nb, slab_geometry_as(s, false, slots).nb);
    return nb;
}
// convergence-on runs take the reference's float running sums (run_exact)
bool exact_logger(const of2d_slab *s) {
    if (s->logger_fp64 >= 0) return s->logger_fp64 == 0;
    return !(s->comm && s->nranks > 1);
}
}  // namespace

// ---------------------------------------------------------------- exact Logger
// The reference's Logger norms over the slabs (Motion.cpp:42-49 as
// Logger::update_error takes them, Logger.cpp:32-51): one float running sum in
// the global linear order, which crosses the slabs in rank order.  As on one
// device (Registration::run_chunked_exact) every iterate stays in memory: the
// iterations run in groups of up to three (a triple launch that stores all
// three iterates, with its 3-line halo, or single steps with 1-line halos)
// into a ring of kExR buffers, and each group's norms are one batch of
// seqnorm launches (seqnorm_kernels.hip) over this slab's rows:
//   sn  the pass, the slab's fp64 totals, the prediction offsets chained in
//       rank order (rank r receives r - 1's running fp64 totals and sends its
//       own on), the check / fix (which work only for norms without a usable
//       profile)
//   wk  the walk, chained in rank order: rank r starts from rank r - 1's
//       exact running sums after its last term and passes its own on, so the
//       last rank's walk ends with the reference's sums bit for bit
// Over RCCL the chains are ncclRecv / ncclSend of 2K doubles / floats on
// communicators of their own (one per stream: comm keeps the halo); in an
// in-process group the next rank waits for its neighbour's event and reads its
// device memory.  At each chunk's end the last rank's sums decide the break
// on every rank (ncclBroadcast / a read of its memory).
namespace of2d {
constexpr int kExR = 12;   // ring buffers besides the chunk's start buffer
constexpr int kExEv = 16;  // event / slot ring per group
struct SlabExact {
    Field<float2> extra[kExR + 1 - 3];  // buffers 3 .. kExR (0 .. 2 are the slab's u)
    DevArray<unsigned char> ws[6];      // two sets of three workspaces
    bool walked[6] = {};
    hipStream_t sn = nullptr, wk = nullptr;
    hipEvent_t ev_step[kExEv] = {}, ev_fix[kExEv] = {}, ev_walk[kExEv] = {}, ev_off[kExEv] = {};
    DevArray<double> poff;    // [3][2] this group's prediction offsets
    DevArray<double> nxt;     // [kExEv][3][2] offsets + this slab's totals, per group slot
    DevArray<double> nxt_in;  // [kExEv][3][2] the previous rank's (RCCL)
    DevArray<float> seq;      // [chunk][2] exact running sums after this slab
    DevArray<float> sin;      // [kExEv][3][2] the previous rank's (RCCL)
    ncclComm_t comm_sn = nullptr, comm_wk = nullptr;
    long gseq = 0;  // groups enqueued over the slab's life (the same on every rank)
    int dev = 0;
    ~SlabExact() {
        (void)hipSetDevice(dev);
        for (hipStream_t q : {sn, wk})
            if (q) (void)hipStreamSynchronize(q);
        if (comm_sn) ncclCommDestroy(comm_sn);
        if (comm_wk) ncclCommDestroy(comm_wk);
        for (int k = 0; k < kExEv; k++)
            for (hipEvent_t e : {ev_step[k], ev_fix[k], ev_walk[k], ev_off[k]})
                if (e) (void)hipEventDestroy(e);
        for (hipStream_t q : {sn, wk})
            if (q) (void)hipStreamDestroy(q);
    }
};
}  // namespace of2d

namespace {
using of2d::kExEv;
using of2d::kExR;
void slab_prepare(of2d_slab *s);

of2d::Field<float2> &exbuf(of2d_slab *s, int k) { return k < 3 ? s->u[k] : s->ex->extra[k - 3]; }

// first exact run: the ring, workspaces, streams, events and (RCCL) the two
// chain communicators, split from the halo communicator by every rank together
void exact_setup(of2d_slab *s) {
    if (s->ex) return;
    auto *E = new of2d::SlabExact();
    s->ex = E;
    E->dev = s->device;
    for (auto &f : E->extra) f.alloc(s->dimx, s->nrows, 3);
    for (auto &w : E->ws) w.alloc(of2d::seqnorm_workspace_bytes(s->dimx, s->nrows));
    OF2D_HIP(hipStreamCreateWithFlags(&E->sn, hipStreamNonBlocking));
    OF2D_HIP(hipStreamCreateWithFlags(&E->wk, hipStreamNonBlocking));
    for (int k = 0; k < kExEv; k++)
        for (hipEvent_t *e : {&E->ev_step[k], &E->ev_fix[k], &E->ev_walk[k], &E->ev_off[k]})
            OF2D_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    E->poff.alloc(6);
    E->nxt.alloc(6 * kExEv);
    E->nxt_in.alloc(6 * kExEv);
    E->seq.alloc(2 * (size_t)s->chunk);
    E->sin.alloc(6 * kExEv);
    if (s->comm && s->nranks > 1) {
        OF2D_NCCL(ncclCommSplit(s->comm, 0, s->rank, &E->comm_sn, nullptr));
        OF2D_NCCL(ncclCommSplit(s->comm, 0, s->rank, &E->comm_wk, nullptr));
    }
}

// in-process group: wait until rank r has enqueued group g's record of `done`
void wait_rank(const std::atomic<long> &done, long g) { wait_count(done, g, "Logger chain"); }

// The convergence-on run with the reference's Logger; *done = iterations
int run_exact(of2d_slab *s, int niter) {
    exact_setup(s);
    of2d::SlabExact &E = *s->ex;
    of2d_slab_group *grp = s->grp;
    const bool rccl = E.comm_sn != nullptr;
    const int n = s->nranks, r = s->rank;
    const of2d_slab *up = grp && r > 0 ? grp->slabs[r - 1] : nullptr;
    const float alphasq = s->alpha * s->alpha;
    const double npx = (double)s->dimx * s->dimy;
    const int nb = slab_geometry(s).nb;
    unsigned *range_flag = s->d_status + of2d::kRangeFlagWord;
    const float *ia = use_gi_exact(s) ? s->Imov.p : nullptr;
    for (bool &w : E.walked) w = false;  // a new loop: no profile yet
    auto ring = [](int a, int t) {  // the (t mod kExR)-th buffer other than a
        const int i = t % kExR;
        return i < a ? i : i + 1;
    };
    auto src_of = [&](int a, int t) { return t == 0 ? a : ring(a, t - 1); };
    auto ev = [](hipEvent_t *e, long g) { return e[g % kExEv]; };
    auto part = [&](int t) { return s->d_partial + (size_t)t * nb * 2; };
    // one step from buffer `in` to `out` with its 1-line halo (chunk tails, replays)
    auto single = [&](int in, int out, double *partial) {
        float2 *uin = exbuf(s, in).p;
        halo_exchange(s, uin, 1, s->st);
        of2d::launch_hs_jacobi(uin, exbuf(s, out).p, s->dI.p, s->It.p, s->P, s->dimx, s->nrows,
                               s->rb, s->dimy, alphasq, partial, s->d_status, s->st);
    };
    std::vector<long> group_of((size_t)s->chunk);
    int a = s->start, k0 = 0;
    while (k0 < niter) {
        const int C = std::min(s->chunk, niter - k0);
        long g = 0;
        for (int t = 0; t < C; t += 0) {
            const int k = std::min(3, C - t);
            g = E.gseq++;
            for (int m = t; m < t + k; m++) group_of[m] = g;
            // the buffers of iterates t .. t + k - 1 held iterates t - kExR ..,
            // last read by the walk of iterate t + k - kExR's group
            if (t + k - kExR >= 0)
                OF2D_HIP(hipStreamWaitEvent(s->st, ev(E.ev_walk, group_of[t + k - kExR]), 0));
            if (k == 3) {
                float2 *uin = exbuf(s, src_of(a, t)).p;
                halo_exchange(s, uin, 3, s->st);
                of2d::launch_hs_jacobi3(uin, exbuf(s, ring(a, t + 2)).p, s->dI.p, s->It.p, s->P,
                                        s->dimx, s->nrows, s->rb, s->dimy, alphasq, -3,
                                        s->nrows + 3, part(t), part(t + 1), part(t + 2),
                                        s->d_status, range_flag, s->st, -1, -1, ia,
                                        exbuf(s, ring(a, t)).p, exbuf(s, ring(a, t + 1)).p,
                                        nullptr, 0, slab_geometry(s).slots);
            } else {
                for (int m = t; m < t + k; m++) single(src_of(a, m), ring(a, m), part(m));
            }
            OF2D_HIP(hipEventRecord(ev(E.ev_step, g), s->st));
            // the group's norms as one batch on this slab's rows
            of2d::SeqnormBatch B;
            B.K = k;
            B.u[0] = exbuf(s, src_of(a, t)).p;
            const double *tot[3];
            for (int i = 0; i < k; i++) {
                const int w = 3 * (int)(g & 1) + i;
                B.u[i + 1] = exbuf(s, ring(a, t + i)).p;
                B.ws[i] = E.ws[w].p;
                B.use_profile[i] = E.walked[w];
                E.walked[w] = true;
                B.p_off[i] = E.poff.p + 2 * i;
                B.out[i] = E.seq.p + 2 * (size_t)(t + i);
            }
            OF2D_HIP(hipStreamWaitEvent(E.sn, ev(E.ev_step, g), 0));
            // workspace set g & 1: group g - 2's walk has read it and left its profile
            if (g >= 2) OF2D_HIP(hipStreamWaitEvent(E.sn, ev(E.ev_walk, g - 2), 0));
            of2d::launch_seqnorm_pass(B, s->dimx, s->nrows, s->P, E.sn);
            for (int i = 0; i < k; i++)
                tot[i] = of2d::seqnorm_total(s->dimx, s->nrows, s->P, B.ws[i], E.sn);
            double *nxt = E.nxt.p + 6 * (g % kExEv);
            const double *prev_nxt = nullptr;
            if (r > 0 && rccl) {
                double *in = E.nxt_in.p + 6 * (g % kExEv);
                OF2D_NCCL(ncclRecv(in, 2 * k, ncclDouble, r - 1, E.comm_sn, E.sn));
                prev_nxt = in;
            } else if (r > 0 && grp) {
                wait_rank(grp->off_done[r - 1], g);
                OF2D_HIP(hipStreamWaitEvent(E.sn, ev(up->ex->ev_off, g), 0));
                prev_nxt = up->ex->nxt.p + 6 * (g % kExEv);
            }
            of2d::launch_seqnorm_offset_chain(prev_nxt, tot, k, E.poff.p, nxt, E.sn);
            if (rccl && r < n - 1)
                OF2D_NCCL(ncclSend(nxt, 2 * k, ncclDouble, r + 1, E.comm_sn, E.sn));
            OF2D_HIP(hipEventRecord(ev(E.ev_off, g), E.sn));
            if (grp) grp->off_done[r].store(g + 1, std::memory_order_release);
            of2d::launch_seqnorm_refine(B, s->dimx, s->nrows, s->P, E.sn);
            OF2D_HIP(hipEventRecord(ev(E.ev_fix, g), E.sn));
            OF2D_HIP(hipStreamWaitEvent(E.wk, ev(E.ev_fix, g), 0));
            if (r > 0 && rccl) {
                float *in = E.sin.p + 6 * (g % kExEv);
                OF2D_NCCL(ncclRecv(in, 2 * k, ncclFloat, r - 1, E.comm_wk, E.wk));
                for (int i = 0; i < k; i++) B.s_in[i] = in + 2 * i;
            } else if (r > 0 && grp) {
                wait_rank(grp->walk_done[r - 1], g);
                OF2D_HIP(hipStreamWaitEvent(E.wk, ev(up->ex->ev_walk, g), 0));
                for (int i = 0; i < k; i++) B.s_in[i] = up->ex->seq.p + 2 * (size_t)(t + i);
            }
            of2d::launch_seqnorm_walk(B, s->dimx, s->nrows, s->P, E.wk);
            if (rccl && r < n - 1)
                OF2D_NCCL(ncclSend(E.seq.p + 2 * (size_t)t, 2 * k, ncclFloat, r + 1, E.comm_wk,
                                   E.wk));
            OF2D_HIP(hipEventRecord(ev(E.ev_walk, g), E.wk));
            if (grp) grp->walk_done[r].store(g + 1, std::memory_order_release);
            t += k;
        }
        // the chunk's global sums: the last rank's walks
        if (rccl)
            OF2D_NCCL(ncclBroadcast(E.seq.p, E.seq.p, 2 * (size_t)C, ncclFloat, n - 1, E.comm_wk,
                                    E.wk));
        OF2D_HIP(hipStreamSynchronize(E.wk));
        OF2D_HIP(hipStreamSynchronize(E.sn));
        const of2d_slab *last = grp ? grp->slabs[n - 1] : s;
        if (grp) grp->barrier();  // every rank's walks of the chunk are done
        OF2D_HIP(hipMemcpy(s->hs.flt, last->ex->seq.p, sizeof(float) * 2 * C,
                           hipMemcpyDeviceToHost));
        if (grp) grp->barrier();  // read before the last rank's next chunk rewrites it
        OF2D_HIP(hipMemcpyAsync(s->hs.status, s->d_status, sizeof(unsigned),
                                hipMemcpyDeviceToHost, s->st));
        OF2D_HIP(hipStreamSynchronize(s->st));
        if (s->hs.status[0] & of2d::kStatusDivZero)
            throw std::runtime_error("Divide by zero exception");
        for (int t = 0; t < C; t++) {
            const int kk = k0 + t;
            const float e = of2d::logger_error(s->hs.flt[2 * t], s->hs.flt[2 * t + 1], npx);
            s->errs.push_back(e);
            if (e < 0.001f && kk > 1) {  // ImageRegistrationOpticalFlow.cpp:131-134
                // iteration t's buffer was reused by iteration t + kExR: replay
                // (every rank: the sums are global)
                if (t + kExR <= C - 1)
                    for (int q = 0; q <= t; q++) single(src_of(a, q), ring(a, q), s->d_partial);
                s->fin = ring(a, t);
                return kk + 1;
            }
        }
        a = ring(a, C - 1);
        k0 += C;
    }
    s->fin = a;
    return niter;
}
}  // namespace

extern "C" {

int of2d_slab_bounds(int dimy, int rank, int nranks, int *row_begin, int *row_end) {
    if (dimy <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || !row_begin || !row_end)
        return OF2D_ERR_INVALID_ARGUMENT;
    const int base = dimy / nranks, rem = dimy % nranks;
    *row_begin = rank * base + std::min(rank, rem);
    *row_end = *row_begin + base + (rank < rem ? 1 : 0);
    return OF2D_OK;
}

int of2d_rccl_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }

int of2d_rccl_get_unique_id(void *out, int len) {
    if (!out || len < (int)sizeof(ncclUniqueId)) return OF2D_ERR_INVALID_ARGUMENT;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return OF2D_ERR_DEVICE;
    std::memcpy(out, &id, sizeof id);
    return OF2D_OK;
}

static int slab_create(of2d_slab **out, int dimx, int dimy, float alpha, int rank, int nranks,
                       int device, const void *uid, int id_len, of2d_slab_group *grp) {
    if (!out) return OF2D_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    auto *s = new of2d_slab();
    int rc = sguard(s, [&] {
        if (dimx < 3 || dimy < 3) throw std::invalid_argument("slab: grid too small");
        if (of2d_slab_bounds(dimy, rank, nranks, &s->rb, &s->re) != OF2D_OK)
            throw std::invalid_argument("slab: bad rank/nranks");
        s->nrows = s->re - s->rb;
        if (s->nrows < 3) throw std::invalid_argument("slab: fewer than 3 j-lines per rank");
        if (!of2d::field_fits_u32(dimx, s->nrows, 3))
            throw std::invalid_argument("slab: a field must have < 2^32 elements");
        s->dimx = dimx;
        s->dimy = dimy;
        s->rank = rank;
        s->nranks = nranks;
        s->alpha = alpha;
        s->device = device;
        s->P = of2d::pitch_for(dimx);
        OF2D_HIP(hipSetDevice(device));
        OF2D_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
        OF2D_HIP(hipEventCreate(&s->ev0));
        OF2D_HIP(hipEventCreate(&s->ev1));
        for (auto &e : s->ev_tri) OF2D_HIP(hipEventCreate(&e));
        for (auto &e : s->ev_halo) OF2D_HIP(hipEventCreate(&e));
        OF2D_HIP(hipStreamCreateWithFlags(&s->comm_st, hipStreamNonBlocking));
        OF2D_HIP(hipEventCreateWithFlags(&s->ev_int, hipEventDisableTiming));
        OF2D_HIP(hipEventCreateWithFlags(&s->ev_edge, hipEventDisableTiming));
        for (auto &f : s->u) f.alloc(dimx, s->nrows, 3);  // three ghost j-lines each side
        s->dI.alloc(dimx, s->nrows, 2);
        s->It.alloc(dimx, s->nrows, 2);
        s->Iref.alloc(dimx, s->nrows, 3);
        s->Imov.alloc(dimx, s->nrows, 3);
        const int nb = partial_blocks_cap(s);
        OF2D_HIP(hipMalloc(&s->d_partial, sizeof(double) * 2 * (size_t)nb * s->chunk_cap()));
        OF2D_HIP(hipMalloc(&s->d_sums, sizeof(double) * 2 * s->chunk));
        OF2D_HIP(hipMalloc(&s->d_status, 64 * sizeof(unsigned)));
        OF2D_HIP(hipMemset(s->d_status, 0, 64 * sizeof(unsigned)));
        OF2D_HIP(hipDeviceSynchronize());  // null-stream memset vs the non-blocking stream
        OF2D_HIP(hipMalloc(&s->d_stage, sizeof(double) * 2 * (size_t)dimx * (s->nrows + 6)));
        s->hs.ensure(s->chunk);
        reserve_sums(s, 3000);  // 48 KB: a fixed_iters run of 3000 iterations needs no allocation
        if (grp) {
            if (grp->n != nranks) throw std::invalid_argument("slab: group size != nranks");
            OF2D_HIP(hipEventCreateWithFlags(&s->ev_ready, hipEventDisableTiming));
            OF2D_HIP(hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming));
            for (int k = 0; k < of2d_slab::kXr; k++) {
                OF2D_HIP(hipEventCreateWithFlags(&s->ev_xr[k], hipEventDisableTiming));
                OF2D_HIP(hipEventCreateWithFlags(&s->ev_xd[k], hipEventDisableTiming));
            }
            OF2D_HIP(hipMalloc(&s->d_red, sizeof(double) * 2 * (size_t)s->chunk_cap()));
            std::lock_guard<std::mutex> lk(grp->m);
            if (grp->slabs[rank]) throw std::invalid_argument("slab: rank already in the group");
            grp->slabs[rank] = s;
            s->grp = grp;
        } else if (nranks > 1 || uid) {
            // nranks == 1 with an id: a one-rank communicator, so that the RCCL
            // calls (init, all-reduces) run on a one-GPU box too
            if (!uid || id_len < (int)sizeof(ncclUniqueId))
                throw std::invalid_argument("slab: RCCL unique id required for nranks > 1");
            ncclUniqueId id;
            std::memcpy(&id, uid, sizeof id);
            OF2D_NCCL(ncclCommInitRank(&s->comm, nranks, id, rank));
        }
    });
    if (rc != OF2D_OK) {
        g_create_err = s->err;
        of2d_slab_destroy(s);
        return rc;
    }
    *out = s;
    return OF2D_OK;
}

int of2d_slab_create(of2d_slab **out, int dimx, int dimy, float alpha, int rank, int nranks,
                     int device, const void *uid, int id_len) {
    return slab_create(out, dimx, dimy, alpha, rank, nranks, device, uid, id_len, nullptr);
}

int of2d_slab_group_create(of2d_slab_group **out, int nranks) {
    if (!out || nranks < 1 || nranks > of2d::kMaxLocalRanks) return OF2D_ERR_INVALID_ARGUMENT;
    auto *g = new of2d_slab_group();
    g->n = nranks;
    g->slabs.assign(nranks, nullptr);
    g->ptr.assign(nranks, nullptr);
    g->flag.assign(nranks, 0);
    g->xptr.assign((size_t)nranks * of2d_slab::kXr, nullptr);
    g->xr_ready.reset(new std::atomic<long>[nranks]);
    g->xr_done.reset(new std::atomic<long>[nranks]);
    g->off_done.reset(new std::atomic<long>[nranks]);
    g->walk_done.reset(new std::atomic<long>[nranks]);
    for (int r = 0; r < nranks; r++) {
        g->xr_ready[r] = 0;
        g->xr_done[r] = 0;
        g->off_done[r] = 0;
        g->walk_done[r] = 0;
    }
    *out = g;
    return OF2D_OK;
}

int of2d_slab_group_destroy(of2d_slab_group *g) {
    if (!g) return OF2D_ERR_INVALID_ARGUMENT;
    for (of2d_slab *s : g->slabs)
        if (s) return OF2D_ERR_STATE;  // destroy the slabs first
    delete g;
    return OF2D_OK;
}

int of2d_slab_create_local(of2d_slab **out, int dimx, int dimy, float alpha, int rank,
                           int nranks, int device, of2d_slab_group *g) {
    if (!g) return OF2D_ERR_INVALID_ARGUMENT;
    return slab_create(out, dimx, dimy, alpha, rank, nranks, device, nullptr, 0, g);
}

int of2d_slab_set_images(of2d_slab *s, const double *Iref_rows, const double *Imov_rows) {
    if (!s || !Iref_rows || !Imov_rows) return OF2D_ERR_INVALID_ARGUMENT;
    return sguard(s, [&] {
        // rows [rb-3, re+3) clipped to [0, dimy) -> local rows [-up3, nrows+dn3)
        const int up3 = std::min(3, s->rb), dn3 = std::min(3, s->dimy - s->re);
        const int rows = s->nrows + up3 + dn3;
        for (int which = 0; which < 2; which++) {
            const double *src = which ? Imov_rows : Iref_rows;
            of2d::Field<float> &dst = which ? s->Imov : s->Iref;
            OF2D_HIP(hipMemcpyAsync(s->d_stage, src, sizeof(double) * s->dimx * rows,
                                    hipMemcpyHostToDevice, s->st));
            of2d::launch_d2f(s->d_stage, s->dimx, rows, dst.p - (long)up3 * s->P, s->P, 0,
                             s->st);
        }
        slab_prepare(s);
    });
}
}  // extern "C"

namespace of2d {
void slab_set_images_device(of2d_slab *s, const float *Iref, const float *Iaux, int srcP,
                            int src_dev) {
    if (srcP != s->P) throw std::invalid_argument("slab: image pitch differs from the slab's");
    DeviceScope scope(s->device);
    const int lo = std::max(s->rb - 3, 0), hi = std::min(s->re + 3, s->dimy);
    const size_t bytes = sizeof(float) * (size_t)(hi - lo) * s->P;
    const long dst = (long)(lo - s->rb) * s->P;
    for (int which = 0; which < 2; which++) {
        const float *src = (which ? Iaux : Iref) + (size_t)lo * s->P;
        float *d = (which ? s->Imov : s->Iref).p + dst;
        if (src_dev == s->device)
            OF2D_HIP(hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToDevice, s->st));
        else
            OF2D_HIP(hipMemcpyPeerAsync(d, s->device, src, src_dev, bytes, s->st));
    }
    slab_prepare(s);
}

void slab_copy_estimate(of2d_slab *s, float2 *dst, int dst_dev) {
    DeviceScope scope(s->device);
    const size_t bytes = sizeof(float2) * (size_t)s->nrows * s->P;
    if (dst_dev == s->device)
        OF2D_HIP(hipMemcpyAsync(dst, s->u[s->fin].p, bytes, hipMemcpyDeviceToDevice, s->st));
    else
        OF2D_HIP(hipMemcpyPeerAsync(dst, dst_dev, s->u[s->fin].p, s->device, bytes, s->st));
    OF2D_HIP(hipStreamSynchronize(s->st));
}
}  // namespace of2d

namespace {
// the images are in the slab (rows [rb-3, re+3) clipped): gradients, zeroed
// motion and the division tests, as every image pair needs them
void slab_prepare(of2d_slab *s) {
    {
        // IterativeSolver::set_derivatives(Iref, Iaux = Imov) on the owned rows
        // plus the two halo rows on each side that the fused kernels' first
        // steps need
        const int up2 = std::min(2, s->rb), dn2 = std::min(2, s->dimy - s->re);
        const long o = -(long)up2 * s->P;
        of2d::launch_gradients_rows(s->Iref.p + o, s->Imov.p + o, s->dI.p + o, s->It.p + o,
                                    s->dimx, s->nrows + up2 + dn2, s->P, s->rb - up2, s->dimy,
                                    s->st);
        for (auto &f : s->u) f.zero(s->st);
        s->fin = 0;
        s->start = 0;
        s->start_dirty = false;
        // the triple kernel's division range and the reference's divide-by-zero
        // test (coord2d.h:95-100), once per image pair: dI is fixed for every
        // iteration of every run on these images, so the test each iteration
        // would make is known now; run() throws on all ranks together instead
        // of one rank leaving the others in an exchange
        unsigned *range_flag = s->d_status + of2d::kRangeFlagWord;
        OF2D_HIP(hipMemsetAsync(s->d_status, 0, sizeof(unsigned), s->st));
        of2d::launch_hs_precheck(s->dI.base, s->dI.count, s->P, 2, s->dimx, s->nrows,
                                 s->alpha * s->alpha, range_flag, s->d_status, s->st);
        OF2D_HIP(hipMemcpyAsync(s->hs.status, s->d_status, sizeof(unsigned),
                                hipMemcpyDeviceToHost, s->st));
        OF2D_HIP(hipStreamSynchronize(s->st));
        s->divzero_local = (s->hs.status[0] & of2d::kStatusDivZero) != 0;
        s->divzero_voted = false;
        OF2D_HIP(hipMemsetAsync(s->d_status, 0, sizeof(unsigned), s->st));
        OF2D_HIP(hipStreamSynchronize(s->st));
    }
}
}  // namespace

extern "C" {

int of2d_slab_reserve(of2d_slab *s, int niter) {
    if (!s || niter < 0) return OF2D_ERR_INVALID_ARGUMENT;
    return sguard(s, [&] { reserve_sums(s, niter); });
}

int of2d_slab_run(of2d_slab *s, int niter, int fixed_iters, int *iters_done) {
    if (!s) return OF2D_ERR_INVALID_ARGUMENT;
    return sguard(s, [&] {
        const float alphasq = s->alpha * s->alpha;
        const SlabGeometry G = slab_geometry(s);
        // partial rows long enough for every kernel; each row is reduced over
        // the blocks of the kernel that wrote it
        const int nb = G.nb;
        const int n1 = of2d::hs_nblocks(s->P, s->nrows), n2 = of2d::hs2_nblocks(s->dimx, s->nrows),
                  n3 = G.n3;
        const double npx = (double)s->dimx * s->dimy;
        unsigned *range_flag = s->d_status + of2d::kRangeFlagWord;
        // Iaux == Imov (zero initial motion); its three ghost j-lines hold the
        // neighbours' image rows, as the gradients of the halo rows need
        const float *ia = use_gi(s) ? s->Imov.p : nullptr;
        auto src_of = [](int a, int t) { return t == 0 ? a : (t % 2 == 1 ? (a + 1) % 3 : (a + 2) % 3); };
        auto dst_of = [](int a, int t) { return t % 2 == 0 ? (a + 1) % 3 : (a + 2) % 3; };
        // st runs after the latest edge launches / comm_st after the latest st
        // work.  Only split launches use comm_st: without them a wait and a
        // record around every launch would put two barrier packets between
        // consecutive kernels (~4-6 us per launch)
        auto join_st = [&] {
            if (G.split) OF2D_HIP(hipStreamWaitEvent(s->st, s->ev_edge, 0));
        };
        auto mark_st = [&] {
            if (G.split) OF2D_HIP(hipEventRecord(s->ev_int, s->st));
        };
        auto win3 = [&](hipStream_t st, int in, int out, int jlo, int jhi, int rpw, int slot,
                        double *p1, double *p2, double *p3) {
            of2d::launch_hs_jacobi3_window(s->u[in].p, s->u[out].p, s->dI.p, s->It.p, s->P,
                                           s->dimx, s->nrows, s->rb, s->dimy, alphasq, -3,
                                           s->nrows + 3, jlo, jhi, rpw, slot, p1, p2, p3,
                                           s->d_status, range_flag, st, ia);
        };
        // K (2 or 3) iterations in one pass from buffer `in` to buffer `out`.
        // One rank: one launch.  With neighbours, triples are split: the
        // interior j-lines [E, nrows-E) on st need no halo and start at once;
        // the exchange and the two E-line edge launches run beside them on
        // comm_st (the interior's block budget leaves room for them), so the
        // halo costs the edges' few row steps, not a serialised launch.  The
        // interior of launch k reads rows E-3..E-1 of `in`, written by the
        // edges of launch k-1 (st waits ev_edge); the edges read rows
        // E..E+2, written by the interior of launch k-1 (comm_st waits ev_int,
        // recorded before this launch's interior).  Pairs and single steps
        // (chunk tails, replays) exchange and launch on st.
        auto fused = [&](int K, int in, int out, double *p1, double *p2, double *p3) {
            float2 *uin = s->u[in].p;
            if (K == 3 && G.split) {
                hipEvent_t *eh = s->halo_n < of2d_slab::kHaloTimed
                                     ? s->ev_halo + 5 * s->halo_n++ : nullptr;
                OF2D_HIP(hipStreamWaitEvent(s->comm_st, s->ev_int, 0));
                if (eh) OF2D_HIP(hipEventRecord(eh[0], s->st));
                join_st();
                if (eh) OF2D_HIP(hipEventRecord(eh[1], s->st));
                win3(s->st, in, out, G.E, s->nrows - G.E, G.ri, 0, p1, p2, p3);
                mark_st();
                if (eh) OF2D_HIP(hipEventRecord(eh[2], s->comm_st));
                halo_exchange(s, uin, 3, s->comm_st);
                if (eh) OF2D_HIP(hipEventRecord(eh[3], s->comm_st));
                win3(s->comm_st, in, out, 0, G.E, G.re, G.bi, p1, p2, p3);
                win3(s->comm_st, in, out, s->nrows - G.E, s->nrows, G.re, G.bi + 1, p1, p2, p3);
                if (eh) OF2D_HIP(hipEventRecord(eh[4], s->comm_st));
                OF2D_HIP(hipEventRecord(s->ev_edge, s->comm_st));
                return;
            }
            join_st();
            halo_exchange(s, uin, K, s->st);
            if (K == 3)
                of2d::launch_hs_jacobi3(uin, s->u[out].p, s->dI.p, s->It.p, s->P, s->dimx,
                                        s->nrows, s->rb, s->dimy, alphasq, -3, s->nrows + 3, p1,
                                        p2, p3, s->d_status, range_flag, s->st, -1, -1, ia,
                                        nullptr, nullptr, nullptr, 0, G.slots);
            else
                of2d::launch_hs_jacobi2(uin, s->u[out].p, s->dI.p, s->It.p, s->P, s->dimx,
                                        s->nrows, s->rb, s->dimy, alphasq, -3, s->nrows + 3, p1,
                                        p2, s->d_status, s->st);
            mark_st();
        };
        // a single step from buffer `in` to `out`
        auto single = [&](int in, int out, double *partial) {
            float2 *uin = s->u[in].p;
            join_st();
            halo_exchange(s, uin, 1, s->st);
            of2d::launch_hs_jacobi(uin, s->u[out].p, s->dI.p, s->It.p, s->P, s->dimx, s->nrows,
                                   s->rb, s->dimy, alphasq, partial, s->d_status, s->st);
            mark_st();
        };
        auto step = [&](int a, int t, double *partial) {
            single(src_of(a, t), dst_of(a, t), partial);
        };
        if (!s->P) throw std::invalid_argument("slab: set_images first");
        if (!s->divzero_voted) {
            s->divzero = any_rank(s, s->divzero_local);
            s->divzero_voted = true;
        }
        if (s->divzero) throw std::runtime_error("Divide by zero exception");
        if (fixed_iters) reserve_sums(s, niter);  // no-op after of2d_slab_reserve
        OF2D_HIP(hipMemsetAsync(s->d_status, 0, sizeof(unsigned), s->st));
        s->errs.clear();
        s->tri_pairs = 0;
        s->tri_launches = 0;
        s->halo_n = 0;
        OF2D_HIP(hipEventRecord(s->ev0, s->st));
        mark_st();  // comm_st starts after everything enqueued so far
        OF2D_HIP(hipStreamWaitEvent(s->comm_st, s->ev_int, 0));
        OF2D_HIP(hipEventRecord(s->ev_edge, s->comm_st));
        // motion_est starts at zero: buffer `start` was zeroed by set_images or
        // at the end of the previous run (below), unless that run threw midway
        if (s->start_dirty) s->u[s->start].zero(s->st);
        s->start_dirty = true;
        int a = s->start, k0 = 0, done = -1;
        if (!fixed_iters && exact_logger(s)) {
            done = run_exact(s, niter);
            if (s->fin >= 3) {  // into a buffer of u[] (get_motion, the next run's start)
                const int x = (s->start + 1) % 3;
                OF2D_HIP(hipMemcpyAsync(s->u[x].p, exbuf(s, s->fin).p,
                                        sizeof(float2) * (size_t)s->nrows * s->P,
                                        hipMemcpyDeviceToDevice, s->st));
                s->fin = x;
            }
            k0 = niter;  // skips the fused-partials loop
        }
        while (k0 < niter && done < 0) {
            const int C = std::min(fixed_iters ? s->chunk_fixed : s->chunk, niter - k0);
            auto part = [&](int t) { return s->d_partial + (size_t)t * nb * 2; };
            // triples (then a pair / single tail) alternate between the two
            // buffers other than the chunk's start buffer a, which stays intact
            // for a replay
            of2d::PartialRuns runs;
            auto other = [&](int b) { return b == (a + 1) % 3 ? (a + 2) % 3 : (a + 1) % 3; };
            int cur = a, tp = 0;
            // time this chunk's triples (the first kTriTimed chunks of the run)
            const bool timed = C >= 3 && s->tri_pairs < of2d_slab::kTriTimed;
            if (timed) {
                join_st();
                OF2D_HIP(hipEventRecord(s->ev_tri[2 * s->tri_pairs], s->st));
            }
            while (tp < C) {
                const int nxt = other(cur);
                if (C - tp >= 3) {
                    fused(3, cur, nxt, part(tp), part(tp + 1), part(tp + 2));
                    runs.add(tp, 3, n3);
                    tp += 3;
                    if (timed && C - tp < 3) {  // the chunk's last triple
                        join_st();
                        OF2D_HIP(hipEventRecord(s->ev_tri[2 * s->tri_pairs + 1], s->st));
                        s->tri_pairs++;
                        s->tri_launches += C / 3;
                    }
                } else if (C - tp == 2) {
                    fused(2, cur, nxt, part(tp), part(tp + 1), nullptr);
                    runs.add(tp, 2, n2);
                    tp += 2;
                } else {
                    single(cur, nxt, part(tp));
                    runs.add(tp, 1, n1);
                    tp += 1;
                }
                cur = nxt;
            }
            if (fixed_iters) {
                // no break to decide: keep every chunk's sums on the device and
                // read them back once after the run (no host sync per chunk)
                double *sums = s->d_all + 2 * (size_t)k0;
                join_st();  // the edge launches' partials
                runs.reduce(s->d_partial, nb, sums, s->st);
                allreduce_sums(s, sums, 2 * (size_t)C, s->st);
                a = cur;
                k0 += C;
                continue;
            }
            join_st();
            runs.reduce(s->d_partial, nb, s->d_sums, s->st);
            allreduce_sums(s, s->d_sums, 2 * (size_t)C, s->st);
            OF2D_HIP(hipMemcpyAsync(s->hs.sums, s->d_sums, sizeof(double) * 2 * C,
                                    hipMemcpyDeviceToHost, s->st));
            OF2D_HIP(hipMemcpyAsync(s->hs.status, s->d_status, sizeof(unsigned),
                                    hipMemcpyDeviceToHost, s->st));
            OF2D_HIP(hipStreamSynchronize(s->st));
            if (s->hs.status[0] & of2d::kStatusDivZero)
                throw std::runtime_error("Divide by zero exception");
            for (int t = 0; t < C; t++) {
                const int k = k0 + t;
                const float e = of2d::logger_error(s->hs.sums[2 * t], s->hs.sums[2 * t + 1], npx);
                s->errs.push_back(e);
                if (!fixed_iters && e < 0.001f && k > 1) {
                    // replay single steps from the chunk's start buffer up to the
                    // break (pairs never wrote iteration t's own buffer; all ranks
                    // agree: the sums are global)
                    for (int r = 0; r <= t; r++) step(a, r, s->d_partial);
                    s->fin = dst_of(a, t);
                    done = k + 1;
                    break;
                }
            }
            if (done < 0) {
                a = cur;
                k0 += C;
            }
        }
        if (done < 0) {
            s->fin = a;
            done = niter;
        }
        join_st();
        if (fixed_iters && niter > 0) {
            OF2D_HIP(hipMemcpyAsync(s->hs.sums, s->d_all, sizeof(double) * 2 * niter,
                                    hipMemcpyDeviceToHost, s->st));
            OF2D_HIP(hipMemcpyAsync(s->hs.status, s->d_status, sizeof(unsigned),
                                    hipMemcpyDeviceToHost, s->st));
            OF2D_HIP(hipStreamSynchronize(s->st));
            if (s->hs.status[0] & of2d::kStatusDivZero)
                throw std::runtime_error("Divide by zero exception");
            for (int t = 0; t < niter; t++)
                s->errs.push_back(
                    of2d::logger_error(s->hs.sums[2 * t], s->hs.sums[2 * t + 1], npx));
        }
        OF2D_HIP(hipEventRecord(s->ev1, s->st));
        // ImageRegistrationOpticalFlow.cpp:141 motion_est->reset() after the
        // loop: zero a buffer other than the result for the next run; it runs
        // behind ev1 and is not waited for here
        s->start = (s->fin + 2) % 3;
        s->u[s->start].zero(s->st);
        s->start_dirty = false;
        OF2D_HIP(hipEventSynchronize(s->ev1));
        float ms = 0.0f;
        OF2D_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        s->last_ms = ms;
        double tri_ms = 0.0;
        for (int p = 0; p < s->tri_pairs; p++) {
            float m = 0.0f;
            OF2D_HIP(hipEventElapsedTime(&m, s->ev_tri[2 * p], s->ev_tri[2 * p + 1]));
            tri_ms += m;
        }
        s->tri_n = s->tri_launches;
        s->tri_us = s->tri_launches ? 1000.0 * tri_ms / s->tri_launches : 0.0;
        for (double &h : s->halo_us) h = 0.0;
        for (int p = 0; p < s->halo_n; p++) {
            const hipEvent_t *eh = s->ev_halo + 5 * p;
            const int from[3] = {0, 2, 3}, to[3] = {1, 3, 4};
            for (int q = 0; q < 3; q++) {
                float m = 0.0f;
                OF2D_HIP(hipEventElapsedTime(&m, eh[from[q]], eh[to[q]]));
                s->halo_us[q] += 1000.0 * m / s->halo_n;
            }
        }
        s->halo_samples = s->halo_n;
        if (iters_done) *iters_done = done;
    });
}

int of2d_slab_get_motion(of2d_slab *s, double *out) {
    if (!s || !out) return OF2D_ERR_INVALID_ARGUMENT;
    return sguard(s, [&] {
        // motion->accumulate(*motion_est) onto the zero initial motion, then planar
        // output (Motion::copy_motion_to_input); the scratch buffer is the one
        // holding neither fin nor the next run's zeroed start
        float2 *tmp = s->u[scratch_buffer(s)].p;
        of2d::launch_compose_zero(s->u[s->fin].p, tmp, s->dimx, s->nrows, s->P, s->rb, s->dimy,
                                  s->st);
        of2d::launch_motion_to_planar(tmp, s->P, s->dimx, s->nrows, s->d_stage, s->st);
        OF2D_HIP(hipMemcpyAsync(out, s->d_stage, sizeof(double) * 2 * s->dimx * s->nrows,
                                hipMemcpyDeviceToHost, s->st));
        OF2D_HIP(hipStreamSynchronize(s->st));
    });
}

int of2d_slab_time_kernel(of2d_slab *s, int nlaunch, double *avg_us) {
    if (!s || nlaunch <= 0 || !avg_us) return OF2D_ERR_INVALID_ARGUMENT;
    return sguard(s, [&] {
        if (!s->P) throw std::invalid_argument("slab: set_images first");
        const float alphasq = s->alpha * s->alpha;
        // the triple kernel (three iterations per launch) over the slab's whole
        // geometry: a warm-up launch, then nlaunch back-to-back launches between
        // two events.  Every launch reads the zeroed start buffer and writes the
        // scratch buffer, so the last run's result (fin) and the next run's start
        // survive; the partials go to the run's partial buffer, re-written by
        // every run before it is read
        const int nb = slab_geometry(s).nb;
        double *p1 = s->d_partial, *p2 = p1 + (size_t)nb * 2, *p3 = p1 + (size_t)nb * 4;
        const int in = s->start, out = scratch_buffer(s);
        auto go = [&] {
            of2d::launch_hs_jacobi3(s->u[in].p, s->u[out].p, s->dI.p, s->It.p, s->P, s->dimx,
                                    s->nrows, s->rb, s->dimy, alphasq, -3, s->nrows + 3, p1, p2,
                                    p3, s->d_status, s->d_status + of2d::kRangeFlagWord, s->st,
                                    -1, -1, use_gi(s) ? s->Imov.p : nullptr, nullptr, nullptr,
                                    nullptr, 0, slab_geometry(s).slots);
        };
        go();
        OF2D_HIP(hipEventRecord(s->ev0, s->st));
        for (int k = 0; k < nlaunch; k++) go();
        OF2D_HIP(hipEventRecord(s->ev1, s->st));
        OF2D_HIP(hipEventSynchronize(s->ev1));
        float ms = 0.0f;
        OF2D_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        *avg_us = 1000.0 * ms / nlaunch;
    });
}

int of2d_slab_info(const of2d_slab *s, int *info, int n) {
    if (!s || !info || n < 1) return -OF2D_ERR_INVALID_ARGUMENT;
    int rccl = 0;
    if (s->comm && ncclCommCount(s->comm, &rccl) != ncclSuccess) return -OF2D_ERR_DEVICE;
    const int halo_lines = s->nranks > 1 ? 3 : 0;
    const int v[] = {s->nranks, rccl, s->grp ? 1 : 0, s->rb, s->re, s->dimx, s->P,
                     halo_lines, slab_geometry(s).split ? 1 : 0, use_gi(s) ? 1 : 0,
                     exact_logger(s) ? 1 : 0};
    const int k = std::min(n, (int)(sizeof v / sizeof v[0]));
    for (int i = 0; i < k; i++) info[i] = v[i];
    return k;
}

int of2d_slab_set_option(of2d_slab *s, const char *key, double value) {
    if (!s || !key) return OF2D_ERR_INVALID_ARGUMENT;
    if (std::strcmp(key, "logger_fp64") == 0) {
        s->logger_fp64 = value < 0.0 ? -1 : (value != 0.0 ? 1 : 0);
        return OF2D_OK;
    }
    if (std::strcmp(key, "split") == 0) {
        s->split = value < 0.0 ? -1 : (value != 0.0 ? 1 : 0);
        return OF2D_OK;
    }
    if (std::strcmp(key, "rccl_self_halo") == 0) {
        if (value != 0.0 && !(s->comm && s->nranks == 1)) {
            s->err = "slab: rccl_self_halo needs a one-rank RCCL communicator";
            return OF2D_ERR_INVALID_ARGUMENT;
        }
        s->self_halo = value != 0.0;
        return OF2D_OK;
    }
    if (std::strcmp(key, "hs_gradients_from_image") == 0) {
        s->gi = value < 0.0 ? -1 : (value != 0.0 ? 1 : 0);
        return OF2D_OK;
    }
    s->err = std::string("slab: unknown option ") + key;
    return OF2D_ERR_INVALID_ARGUMENT;
}

int of2d_slab_last_run_kernel_us(const of2d_slab *s, double *avg_us, int *nlaunch) {
    if (!s || !avg_us || !nlaunch) return OF2D_ERR_INVALID_ARGUMENT;
    *avg_us = s->tri_us;
    *nlaunch = s->tri_n;
    return OF2D_OK;
}

int of2d_slab_last_run_halo_us(const of2d_slab *s, double *us3, int *nsampled) {
    if (!s || !us3 || !nsampled) return OF2D_ERR_INVALID_ARGUMENT;
    for (int q = 0; q < 3; q++) us3[q] = s->halo_us[q];
    *nsampled = s->halo_samples;
    return OF2D_OK;
}

int of2d_slab_last_errors(const of2d_slab *s, float *out, int n) {
    if (!s || (n > 0 && !out)) return -OF2D_ERR_INVALID_ARGUMENT;
    const int k = std::min(n, (int)s->errs.size());
    for (int i = 0; i < k; i++) out[i] = s->errs[i];
    return (int)s->errs.size();
}

int of2d_slab_last_run_ms(const of2d_slab *s, double *ms) {
    if (!s || !ms) return OF2D_ERR_INVALID_ARGUMENT;
    *ms = s->last_ms;
    return OF2D_OK;
}

int of2d_slab_destroy(of2d_slab *s) {
    if (!s) return OF2D_ERR_INVALID_ARGUMENT;
    if (s->st) (void)hipStreamSynchronize(s->st);
    if (s->comm_st) (void)hipStreamSynchronize(s->comm_st);
    if (s->ex) {
        (void)hipSetDevice(s->device);
        for (auto &f : s->ex->extra) f.release();
        delete s->ex;
    }
    if (s->comm) ncclCommDestroy(s->comm);
    if (s->grp) {
        std::lock_guard<std::mutex> lk(s->grp->m);
        s->grp->slabs[s->rank] = nullptr;
    }
    if (s->ev_ready) (void)hipEventDestroy(s->ev_ready);
    if (s->ev_done) (void)hipEventDestroy(s->ev_done);
    for (int k = 0; k < of2d_slab::kXr; k++) {
        if (s->ev_xr[k]) (void)hipEventDestroy(s->ev_xr[k]);
        if (s->ev_xd[k]) (void)hipEventDestroy(s->ev_xd[k]);
    }
    if (s->d_red) (void)hipFree(s->d_red);
    if (s->d_partial) (void)hipFree(s->d_partial);
    if (s->d_sums) (void)hipFree(s->d_sums);
    if (s->d_all) (void)hipFree(s->d_all);
    if (s->d_selfx) (void)hipFree(s->d_selfx);
    if (s->d_status) (void)hipFree(s->d_status);
    if (s->d_stage) (void)hipFree(s->d_stage);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    for (auto &e : s->ev_tri)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : s->ev_halo)
        if (e) (void)hipEventDestroy(e);
    if (s->ev_int) (void)hipEventDestroy(s->ev_int);
    if (s->ev_edge) (void)hipEventDestroy(s->ev_edge);
    for (auto &f : s->u) f.release();
    s->dI.release();
    s->It.release();
    s->Iref.release();
    s->Imov.release();
    if (s->comm_st) (void)hipStreamDestroy(s->comm_st);
    if (s->st) (void)hipStreamDestroy(s->st);
    delete s;
    return OF2D_OK;
}

const char *of2d_slab_last_error(const of2d_slab *s) {
    return s ? s->err.c_str() : g_create_err.c_str();
}

}  // extern "C"
