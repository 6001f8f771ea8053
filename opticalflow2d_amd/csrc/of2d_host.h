// of2d_host.h — host-side driver of libof2d.so (C++ above the C-ABI).
//
// Registration mirrors the reference's ImageRegistration hierarchy
// (src/ImageRegistration.{h,cpp}, src/ImageRegistration{OpticalFlow,Demons,
// Fluid}.cpp): a pyramid of nscales+1 levels, nrefine warp-refine passes per
// level, and an iteration loop per refine whose body is the solver's
// get_update (src/regularization/**).  Everything below the C-ABI is device
// resident: images, gradients, motion fields and Logger norms live in HBM and
// the host only enqueues kernels and reads back a few bytes per chunk of
// iterations to take the convergence decision.
#pragma once

#include <algorithm>
#include <cstdarg>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "of2d_device.h"

namespace of2d {

struct DemonsKernels;
struct MultiHS;
void print(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

// ------------------------------------------------------------ device buffer
// A pitched field with one ghost j-line above row 0 and one below the last
// row; `p` points at row 0.  Zero-initialised like Field<T>::Field
// (src/Field.tpp:15-18).
template <class T>
struct Field {
    T *base = nullptr;
    T *p = nullptr;
    int dimx = 0, dimy = 0, P = 0;
    size_t count = 0;
    Field() = default;
    Field(const Field &) = delete;
    Field &operator=(const Field &) = delete;
    Field(Field &&o) noexcept { *this = std::move(o); }
    Field &operator=(Field &&o) noexcept {
        std::swap(base, o.base);
        std::swap(p, o.p);
        std::swap(dimx, o.dimx);
        std::swap(dimy, o.dimy);
        std::swap(P, o.P);
        std::swap(count, o.count);
        return *this;
    }
    ~Field() { release(); }
    void alloc(int dx, int dy, int ghost = 1) {
        release();
        dimx = dx;
        dimy = dy;
        P = pitch_for(dx);
        count = (size_t)(dy + 2 * ghost) * P + kPitchAlign;
        OF2D_HIP(hipMalloc(&base, count * sizeof(T)));
        // the null-stream memset is unordered with the driver's non-blocking
        // stream: finish it before anything is enqueued there
        OF2D_HIP(hipMemset(base, 0, count * sizeof(T)));
        OF2D_HIP(hipDeviceSynchronize());
        p = base + (size_t)ghost * P;
    }
    void release() {
        if (base) (void)hipFree(base);
        base = p = nullptr;
        count = 0;
    }
    void zero(hipStream_t st) { OF2D_HIP(hipMemsetAsync(base, 0, count * sizeof(T), st)); }
    size_t bytes() const { return count * sizeof(T); }
};

// A plain device array (no ghost lines)
template <class T>
struct DevArray {
    T *p = nullptr;
    size_t n = 0;
    DevArray() = default;
    DevArray(const DevArray &) = delete;
    DevArray &operator=(const DevArray &) = delete;
    DevArray(DevArray &&o) noexcept { *this = std::move(o); }
    DevArray &operator=(DevArray &&o) noexcept {
        std::swap(p, o.p);
        std::swap(n, o.n);
        return *this;
    }
    ~DevArray() {
        if (p) (void)hipFree(p);
    }
    void alloc(size_t count) {
        if (p) (void)hipFree(p);
        n = count;
        OF2D_HIP(hipMalloc(&p, sizeof(T) * (count ? count : 1)));
        OF2D_HIP(hipMemset(p, 0, sizeof(T) * (count ? count : 1)));
        OF2D_HIP(hipDeviceSynchronize());  // see Field::alloc
    }
};

// the Fluid loop's report ring (iterations enqueued ahead of the host's read)
constexpr int kFluidReports = 8;
// iterations the Fluid loop enqueues beyond the one whose report it reads
constexpr int kFluidAhead = 3;
// Pinned host scratch for the per-chunk read-back
struct HostScratch {
    double *sums = nullptr;
    unsigned *status = nullptr;
    float *flt = nullptr;
    float *seqh = nullptr;  // coherent, mapped: seqnorm_decide's copy of the exact sums
    FluidReport *report = nullptr;  // [kFluidReports], hipHostMallocCoherent
    int cap = 0;
    void ensure(int n);
    ~HostScratch();
};

// Per-iteration Logger norms -> error, exactly the reference's float formula
// (Logger.cpp:37-39, Motion.cpp:47) applied to fp64 sums.
float logger_error(double sum_diff, double sum_prev, double npx);

// The reference-exact Logger's pipeline depth (Registration, below): iterate
// ring buffers, workspace sets and walk streams (build knobs for A/B runs)
#ifndef OF2D_SN_RING
#define OF2D_SN_RING 15
#endif
#ifndef OF2D_SN_SETS
#define OF2D_SN_SETS 4
#endif
#ifndef OF2D_SN_WALKERS
#define OF2D_SN_WALKERS 3
#endif
constexpr int kMaxEst = OF2D_SN_RING + 1 > 16 ? OF2D_SN_RING + 1 : 16;
// CUs kept from the bandwidth kernels of HS's exact loop (its triples and
// passes run on streams with a CU mask without them), so that the loop's
// latency chain (check, entries, walks) finds free slots: 4096^2 procedural
// 141-142 -> 128-131 us per iteration with 8-32 CUs kept, texture unchanged
// (profiles/r05e_conv_cumask_ab.log; the chain's streams on those CUs only
// was slower: r05d).  0 = no mask.
#ifndef OF2D_SN_CUMASK
#define OF2D_SN_CUMASK 16
#endif
// iterations per host decision block of HS's exact loop (the "chunk" option
// overrides it): the host enqueues one block ahead of its decision, so a
// break leaves at most two blocks of no-op launches behind it (each group's
// seven kernels chained by events: ~90 us a group at 4096^2).  12 instead of
// 33: texture pair 162-165 -> 149 us per iteration, procedural 126-127 ->
// 123-125 (profiles/r05h_chunk_ab.log); 9: 140-142 / 120-121 against 12's
// 143-146 / 122-124, 6: 143-145 / 123 (profiles/r05i_blk_ab.log)
#ifndef OF2D_SN_BLOCK
#define OF2D_SN_BLOCK 9
#endif
// 1: the walks on the reserved CUs, the check and entries on every CU (a walk
// block beside the triple's and pass's blocks slows them more than the walk
// gains there: 4096^2 convergence on, texture 142-144 -> 132-136, procedural
// 118-120 -> 114-116 us per iteration; 8, 24 or 32 reserved CUs the same,
// profiles/r05m_cuwalk_ab.log)
#ifndef OF2D_SN_CUMASK_WALK
#define OF2D_SN_CUMASK_WALK 1
#endif

struct Level {
    int dx = 0, dy = 0, P = 0;
    Field<float> Iref, Imov, Iaux, It, Iwar, jac;
    Field<float2> motion[2];
    int mcur = 0;
    Field<float2> dI;
    Field<float2> est[kMaxEst];  // [3] .. [kRing]: only for the exact-norm loop's ring
    Field<float2> force, velocity, increment, corr, tmp;
    DevArray<double> cbuf[2];              // Curvature: two x|y double plane pairs (pitch P)
    DevArray<double> cC1T, cC0, cD1T, cD0;  // Curvature: REDFT10 / REDFT01 matrices
    DevArray<double> cE;                    // Curvature: eigenvalues (pitch P)
    Field<float4> vb;                   // SOR working array {v, b} (Fluid: persistent velocity)
    DevArray<unsigned long long> sorH;  // SOR strip hand-off granules
    DevArray<unsigned> sorTicket;       // SOR strip ticket (multiple of nstrips between sweeps);
                                        // Fluid: then per strip its last finished epoch
    DevArray<unsigned long long> sorCtr;  // Fluid sweep + increment: role ticket, tile counter
    DevArray<float> part;               // per-block float partials (max / min reductions)
    float2 *cur_motion() { return motion[mcur].p; }
};

class Registration {
   public:
    Registration(int dimx, int dimy, int nscales, const int *niter, int nrefine, int reg,
                 const float *params, unsigned nparams, int verbose);
    ~Registration();
    void set_images(const double *ref, const double *mov);
    void estimate();
    void get_motion(double *out);
    void warp(const double *in, double *out);
    void set_option(const std::string &key, double v);
    const std::vector<int> &iterations() const { return iters_; }
    const std::vector<float> &last_errors() const { return last_err_; }
    int dimx() const { return dimx_; }
    int dimy() const { return dimy_; }

    using StepFn = std::function<void(const float2 *src, float2 *dst, double *partial)>;
    // two iterations in one pass: partial / partial2 receive the Logger partials
    // of the first / second (nb blocks each, as the single step's)
    using StepFn2 = std::function<void(const float2 *src, float2 *dst, double *partial,
                                       double *partial2)>;
    using StepFn3 = std::function<void(const float2 *src, float2 *dst, double *partial,
                                       double *partial2, double *partial3)>;
    // three iterations in one pass, every iterate stored (d1, d2, d3)
    // (t0: the triple's first iteration, for the stop word of run_exact_pipelined)
    // (band_lo / band_hi: the triple's row bands this launch covers, -1 all)
    using StepFn3M = std::function<void(const float2 *src, float2 *d1, float2 *d2, float2 *d3,
                                        int t0, int band_lo, int band_hi)>;

   private:
    // nblk[k]: block partials written by step (k = 0), step2 (1), step3 (2)
    int run_chunked(Level &L, int niter, int nb, const StepFn &step, int &final_buf,
                    const StepFn2 &step2 = nullptr, const StepFn3 &step3 = nullptr,
                    const int *nblk = nullptr, const StepFn3M &step3m = nullptr);
    void ensure_device();
    void estimate_level(int s);
    int loop_hs(Level &L, int niter, float alpha, int &final_buf);
    int loop_demons(Level &L, int niter, int &final_buf);
    int loop_fluid(Level &L, int niter);
    int loop_elastic(Level &L, int niter, int &final_buf);
    int loop_curvature(Level &L, int niter, int &final_buf);
    // HS over ngpus_ row slabs in this process (ranks.cpp)
    int loop_hs_multi(int s, float alpha, int &final_buf);
    MultiHS &multi_for(int s, float alpha);
    void multi_release();
    int ngpus_ = 1;
    // ranks may share a device (option "ngpus_share"; tests of the
    // decomposition on one GPU); otherwise at most one rank per device: a
    // device's rows in one slab, as splitting them only adds halo work
    bool share_ = false;
    int ndev_ = 1;
    int ranks() const { return share_ ? ngpus_ : std::min(ngpus_, ndev_); }
    std::vector<std::shared_ptr<MultiHS>> lv_multi_;
    void check_status();
    void check_reported_status(unsigned st);

    int dimx_, dimy_, nscales_, nrefine_, reg_, verbose_;
    std::vector<int> niter_;
    std::vector<float> params_;
    std::vector<int> ldx_, ldy_;
    std::vector<Level> lv_;
    bool fixed_ = false;
    // Logger norms: the reference's float running sums (seqnorm, default) or
    // fp64 sums of the fused partials (logger_fp64; fixed_iters runs always)
    bool logger_fp64_ = false;
    bool exact_norms() const { return !fixed_ && !logger_fp64_; }
    // enqueue the exact norms of one Logger update into d_seq_[2t], [2t + 1]
    // (synchronous loops: Elastic, Fluid; workspace 0, on st_)
    // (stop, t0: the batch returns at once when *stop < t0, Fluid's loop)
    void seqnorm(const Level &L, const float2 *cur, const float2 *prev, int t,
                 const int *stop = nullptr, int t0 = 0);
    // run_chunked with the reference's float norms (single steps in groups of
    // up to three into a ring, each group's norms as one batch on the norm
    // streams); with step3m, run_exact_pipelined
    int run_chunked_exact(Level &L, int niter, int nb, const StepFn &step, int &final_buf,
                          const StepFn3M &step3m = nullptr);
    // HS: triples, blocks of iterations enqueued one ahead of the host's
    // decision, the break also taken on the device (the stop word)
    int run_exact_pipelined(Level &L, int niter, const StepFn &step, int &final_buf,
                            const StepFn3M &step3m);
    int run_exact_pipelined_on(Level &L, int niter, const StepFn &step, int &final_buf,
                               const StepFn3M &step3m);
    // a group's norms behind its steps: pass on sn_st_, check and fix on
    // fx_st_, walk (and with B.stop seqnorm_decide) on wk_st_[g mod 3]
    // (passed: the batch's pass is already enqueued and ev_pass_[g] recorded)
    void enqueue_norms(const SeqnormBatch &B, const Level &L, int g, double npx = 0.0,
                       float *seqh_out = nullptr, bool passed = false);
    void print_sn_debug(const Level &L, const int *dbg, int k0, int lo, int hi);
    hipStream_t sn_st_ = nullptr, fx_st_ = nullptr, wk_st_[OF2D_SN_WALKERS] = {};
    int ncu_ = 256;        // compute units of the device
    // HS's exact loop runs its triples on hs_st_ (in place of st_ for the
    // loop) and its passes on sn_st_, both masked (OF2D_SN_CUMASK; null: no
    // mask), with tri_slots_ resident triple blocks
    hipStream_t hs_st_ = nullptr;
    int tri_slots_ = 1024;
    static constexpr int kExactEv = 64;  // event ring per group (two blocks in flight)
    // workspace sets: group g's walk is read (its profile) by group g + kSeqSets
    static constexpr int kSeqSets = OF2D_SN_SETS;
    static constexpr int kSeqWs = 3 * kSeqSets;
    // iterate buffers: a step waits for the walks kRing / 3 groups back, so
    // kRing / 3 groups of steps, passes and walks are in flight
    static constexpr int kRing = OF2D_SN_RING;
    static_assert(kRing + 1 <= kMaxEst, "Level::est holds the ring");
    static constexpr int kWalkers = OF2D_SN_WALKERS;  // walk streams
    hipEvent_t ev_step_[kExactEv] = {}, ev_pass_[kExactEv] = {}, ev_fix_[kExactEv] = {},
               ev_walk_[kExactEv] = {};
    DevArray<unsigned char> d_seqws_[kSeqWs];  // seqnorm workspaces (level 0 size)
    DevArray<float> d_seq_;                    // per-iteration exact sums of a chunk
    int seq_dx_[kSeqWs] = {}, seq_dy_[kSeqWs] = {};  // grid of each workspace's last call
    int chunk_ = 33;  // eleven fused triples per chunk
    bool chunk_set_ = false;  // the option was given (HS's exact loop then uses it too)
    unsigned exact_epoch_ = 0;  // run_exact_pipelined loops so far (the checks' stamps)
    int gi_ = -1;     // triple kernel: dI from Iaux (1), from dI (0), by size (-1)
    int split_ = -1;  // ranks' triples: interior / edge split (slab option "split")
    int device_ = -1;  // option "device" (-1: the current device at first use)
    int home_ = -1;    // the registration's device, fixed at first use
    bool ready_ = false;
    hipStream_t st_ = nullptr;
    hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
    double *d_stage_ = nullptr;  // double staging for boundary copies
    size_t stage_count_ = 0;
    double *d_partial_ = nullptr;
    DevArray<double> d_all_;  // fixed_iters: every iteration's Logger sums of a level
    size_t partial_count_ = 0;
    double *d_sums_ = nullptr;
    unsigned *d_status_ = nullptr;
    float *d_scalar_ = nullptr;
    HostScratch hs_;
    std::vector<int> iters_;
    std::vector<float> last_err_;
    // Demons kernels (Kernel::set_gaussian, src/Kernel.cpp:45-73)
    std::vector<double> kdiff_, kfluid_;
    std::shared_ptr<DemonsKernels> demons_k_;
    unsigned epoch_ = 0;  // SOR hand-off epoch, strictly increasing per sweep
};

// Validation of nparams per regularisation (ImageRegistrationOpticalFlow.cpp:8-12,
// ImageRegistrationDemons.cpp:7-10, ImageRegistrationFluid.cpp:5-7)
bool valid_regularisation_parameters(int reg, unsigned nparams);

// Kernel::set_gaussian (src/Kernel.cpp:45-73): expf in float, normalised in double
std::vector<double> gaussian_kernel(int kw, float sigma);

}  // namespace of2d
