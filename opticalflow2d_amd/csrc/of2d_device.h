// of2d_device.h — shared definitions for the gfx950 kernels and the host
// driver of libof2d.so.
//
// HBM layout (DESIGN.md "Data layout"): every field of a pyramid level is a
// pitched, row-major (j-line major, x fastest) array whose pitch P is dimx
// rounded up to a multiple of 128 elements, with one zeroed ghost j-line above
// row 0 and one below row dimy-1.  Images are float (4 B/px), motion fields
// interleaved float2 (8 B/px) — the reference's layout (src/Field.tpp:13,
// src/Motion.h:7) plus padding, so 2-px float4 loads of a motion row and 4-px
// float4 loads of an image row are 16-B aligned.
#pragma once

#include <vector>

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace of2d {

constexpr int kPitchAlign = 128;  // elements

inline int pitch_for(int dimx) { return (dimx + kPitchAlign - 1) / kPitchAlign * kPitchAlign; }
// a pitched field of dimy + 2 * ghost j-lines (plus the alignment slack) has
// fewer than 2^32 elements: the gather kernels' unsigned 32-bit offsets hold
inline bool field_fits_u32(int dimx, int dimy, int ghost) {
    return ((unsigned long long)dimy + 2ull * ghost) * (unsigned long long)pitch_for(dimx) +
               kPitchAlign < (1ull << 32);
}

struct DeviceError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define OF2D_HIP(call)                                                                    \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            throw ::of2d::DeviceError(std::string("HIP error: ") + hipGetErrorString(e_) + \
                                      " at " __FILE__ ":" + std::to_string(__LINE__));   \
    } while (0)

// Restores the calling thread's current device when the scope ends (normally
// or by an exception); bind() switches it meanwhile.  The multi-device paths
// switch devices per rank, and a caller's own device must survive every entry
// point.
class DeviceScope {
   public:
    DeviceScope() { (void)hipGetDevice(&prev_); }
    explicit DeviceScope(int dev) : DeviceScope() { bind(dev); }
    ~DeviceScope() {
        if (prev_ >= 0) (void)hipSetDevice(prev_);
    }
    void bind(int dev) { OF2D_HIP(hipSetDevice(dev)); }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;

   private:
    int prev_ = -1;
};

// status bits written by kernels (one word per context, zeroed per call)
constexpr unsigned kStatusDivZero = 1u;
constexpr unsigned kStatusExpBound = 2u;  // scaling-and-squaring count above the host bound
constexpr unsigned kStatusSpinTimeout = 4u;  // a bounded inter-workgroup wait gave up

// ---------------------------------------------------------------- HS Jacobi
// Each wave marches kHsRows j-lines of a kHsStrip-px strip (kHsPxl px per
// lane); a block is kHsWaves waves stacked in y (hs_jacobi_impl.h).
constexpr int kHsRows = 32;
constexpr int kHsPxl = 2;
constexpr int kHsStrip = 64 * kHsPxl;
constexpr int kHsWaves = 4;
inline dim3 hs_grid(int P, int nrows) {
    return dim3(P / kHsStrip, (nrows + kHsRows * kHsWaves - 1) / (kHsRows * kHsWaves));
}
inline int hs_nblocks(int P, int nrows) {
    dim3 g = hs_grid(P, nrows);
    return int(g.x * g.y);
}

// One Jacobi step of OpticalFlowDiffusion::get_update with the Logger's norm
// partials fused (sum ||u_new-u_old||, sum ||u_old|| per block, fp64).
// Row pointers address the first owned row; rows -1 and nrows must be valid
// memory (ghost j-lines).  row0 is the global j of the first owned row.
void launch_hs_jacobi(const float2 *u_old, float2 *u_new, const float2 *dI, const float *It,
                      int P, int dimx, int nrows, int row0, int dimy, float alphasq,
                      double *partial, unsigned *status, hipStream_t st);
// Two Jacobi iterations per launch (temporal blocking, hs::jacobi2_kernel):
// u_new = step(step(u_old)), bit-identical to two launch_hs_jacobi calls.
// Rows [glo, ghi) (relative to the first owned row; ghost j-lines included)
// are readable: u and dI/It outside the owned rows feed the first step's halo
// row on each side.  Logger partials of the first iteration go to partial,
// of the second to partial2 (hs2_nblocks blocks each).
constexpr int kHs2Out = 124;  // output columns per wave (hs_jacobi_impl.h)
constexpr int kHs2Rows = 32;
constexpr int kHs2Waves = 4;
inline dim3 hs2_grid(int dimx, int nrows) {
    return dim3((dimx + kHs2Out - 1) / kHs2Out,
                (nrows + kHs2Rows * kHs2Waves - 1) / (kHs2Rows * kHs2Waves));
}
inline int hs2_nblocks(int dimx, int nrows) {
    dim3 g = hs2_grid(dimx, nrows);
    return int(g.x * g.y);
}
// band_lo / band_hi: the row bands (kHs2Rows * kHs2Waves j-lines each) this
// launch covers; -1 / -1 = all of them.
inline int hs2_nbands(int nrows) {
    return (nrows + kHs2Rows * kHs2Waves - 1) / (kHs2Rows * kHs2Waves);
}
void launch_hs_jacobi2(const float2 *u_old, float2 *u_new, const float2 *dI, const float *It,
                       int P, int dimx, int nrows, int row0, int dimy, float alphasq, int glo,
                       int ghi, double *partial, double *partial2, unsigned *status,
                       hipStream_t st, int band_lo = -1, int band_hi = -1);
// Three Jacobi iterations per launch (hs::jacobi3_kernel): bit-identical to
// three launch_hs_jacobi calls; rows [glo, ghi) readable as for the pair
// kernel (the first two steps also cover two / one halo rows each side).
constexpr int kHs3Out = 120;  // output columns per wave (hs_jacobi_impl.h)
constexpr int kHs3Waves = 4;
// j-lines per wave.  A block's time is about (rows + 2) row steps (the
// prologue computes the halo rows of the first two iterations), and the 4-wave
// blocks (4 resident per CU, 256 CUs: `cap` = 1024 block slots, less when
// another launch is to run beside it) run in rounds, so the choice minimises
// rounds x (rows + 2) over rows in [4, 64], fewest rows on ties.  4096^2: 36
// (1015 blocks, one round; 32 gave 1120 blocks and a 9 % second round);
// 16384^2: 50 (11 rounds of 1006-1024 blocks, against 59 and 9.4 rounds);
// grids too small to fill one round get short bands and more blocks.
inline int hs3_rows(int dimx, int nrows, int cap = 1024) {
    const long gx = (dimx + kHs3Out - 1) / kHs3Out;
    int best = 4;
    long best_t = -1;
    for (int r = 4; r <= 64; r++) {
        const long bands = (nrows + kHs3Waves * r - 1) / (kHs3Waves * r);
        const long rounds = (gx * bands + cap - 1) / cap;
        const long t = rounds * (r + 2);
        if (best_t < 0 || t < best_t) {
            best_t = t;
            best = r;
        }
        if (bands == 1) break;  // more rows per wave change nothing
    }
    return best;
}
inline int hs3_nbands(int dimx, int nrows) {
    const int r = kHs3Waves * hs3_rows(dimx, nrows);
    return (nrows + r - 1) / r;
}
inline dim3 hs3_grid(int dimx, int nrows) {
    return dim3((dimx + kHs3Out - 1) / kHs3Out, hs3_nbands(dimx, nrows));
}
inline int hs3_nblocks(int dimx, int nrows) {
    dim3 g = hs3_grid(dimx, nrows);
    return int(g.x * g.y);
}
// range_flag: the word launch_hs_precheck wrote for this dI (required: the
// kernel leaves the divide-by-zero test to it)
// The triple kernel reads dI + It (12 B/px) at every launch.  While both fit
// in the 256 MB MALL (Infinity Cache) they stay resident between launches
// and reading them costs no HBM bandwidth; past that the launch is HBM-bound
// and deriving dI from Iaux in the kernel (GI, 4 B/px instead of 8) saves a
// seventh of its bytes.  Measured per launch (profiles/r02_d_gi_pf_ab*.log):
// 4096^2 81.4 (dI) vs 81.1 us (GI), 16384^2 1553 vs 1335 us.
constexpr double kMallBytes = 256.0 * 1024 * 1024;
inline bool hs3_gradients_from_image(int dimx, int nrows) {
    return 12.0 * dimx * nrows > kMallBytes;
}
// HS's exact-Logger loop streams more than the triple: per three iterations
// the MID triple (u0 in, three iterates out) and the Logger pass (four
// iterates in, non-temporal) move 64 B/px beside the gradients' 12, so dI + It
// stay in the MALL only where all of it fits (4096^2: GI and the pass's
// non-temporal loads 140 -> 131 us per iteration texture, 118 -> 107
// procedural, profiles/r05o_gi_nt_ab.log)
inline bool hs3_exact_gradients_from_image(int dimx, int nrows) {
    return 76.0 * dimx * nrows > kMallBytes;
}
// Ia (Iaux, the image dI was taken of) non-null: the kernel derives the
// gradients from it (24 instead of 28 B/px per launch, same bits); null: it
// reads dI
void launch_hs_jacobi3(const float2 *u_old, float2 *u_new, const float2 *dI, const float *It,
                       int P, int dimx, int nrows, int row0, int dimy, float alphasq, int glo,
                       int ghi, double *partial, double *partial2, double *partial3,
                       unsigned *status, const unsigned *range_flag, hipStream_t st,
                       int band_lo = -1, int band_hi = -1, const float *Ia = nullptr,
                       float2 *u1 = nullptr, float2 *u2 = nullptr, const int *stop = nullptr,
                       int stop_t0 = 0, int slots = 1024);
// (slots: resident 4-wave blocks the launch may have, for its j-lines per
// wave, hs3_rows; 1024 = every CU of the device)
// (u1, u2 non-null: the first two iterates of the owned rows are stored there
// too, for the reference-exact Logger; +16 B/px; with stop, the launch does
// nothing when *stop < stop_t0: the loop broke before the triple's first
// iteration stop_t0, seqnorm_decide)
// Once per gradient field, before the triple kernel runs on it
// (hs_jacobi_impl.h hs_precheck_kernel): zeroes *range_flag, then sets it if
// any gradient / denominator of the allocation [base, base + count) lies
// outside the unscaled-division range, and ORs kStatusDivZero into *status if
// an image pixel's denominator is 0.  ghost: j-lines before row 0 in base.
// The triple kernel over j-lines [jlo, jhi) of the level, rows_per_wave
// j-lines per wave, Logger partials from slot band `slot_band0` on (slot =
// (slot_band0 + block row) * gx + strip): the slab's interior / edge launches.
// Returns the launch's block rows.
int launch_hs_jacobi3_window(const float2 *u_old, float2 *u_new, const float2 *dI,
                             const float *It, int P, int dimx, int nrows, int row0, int dimy,
                             float alphasq, int glo, int ghi, int jlo, int jhi,
                             int rows_per_wave, int slot_band0, double *partial,
                             double *partial2, double *partial3, unsigned *status,
                             const unsigned *range_flag, hipStream_t st,
                             const float *Ia = nullptr);
void launch_hs_precheck(const float2 *base, size_t count, int P, int ghost, int dimx, int dimy,
                        float alphasq, unsigned *range_flag, unsigned *status, hipStream_t st);
constexpr int kRangeFlagWord = 32;  // word of the 64-word status buffers holding range_flag
constexpr int kStopWord = 33;  // the exact-Logger loop's break (seqnorm_decide)
// the Fluid loop's device-side decisions (Registration::loop_fluid, FluidCtl):
// the iteration just decided regridded (the next iteration's estimate reads as
// zero, its Logger prev is the buffer's content), and which of the level's two
// motion fields holds the accumulated motion
constexpr int kFluidRegridWord = 34;
constexpr int kFluidMcurWord = 35;
// A Fluid iteration's kernels and its place in the loop: w = the 64-word
// status buffer (kStopWord: the first breaking iteration, 0x7f7f7f7f none;
// kFluidRegridWord, kFluidMcurWord), it = the iteration.  Every kernel of an
// iteration past the break returns at once; w == nullptr: no control words
// (the kernels' plain behaviour, other callers)
struct FluidCtl {
    unsigned *w = nullptr;
    int it = 0;
};
// blocks of the launches that the control words usually make no-ops (the
// regrid's): grid-stride loops over a capped grid, so an idle launch costs a
// few microseconds instead of dispatching a block per tile
constexpr int kCappedGrid = 2048;
// (plain loads: the words are written by earlier kernels of the same stream)
__device__ __forceinline__ bool fluid_stopped(const FluidCtl &c) {
    return c.w && (int)c.w[kStopWord] < c.it;
}
// the iteration's input estimate is the zero field of a regrid (its buffer
// still holds the pre-regrid estimate, the Logger's prev)
__device__ __forceinline__ bool fluid_zero_est(const FluidCtl &c) {
    return c.w && c.w[kFluidRegridWord] != 0u;
}
// partial-row length that fits every HS kernel (single, pair, triple)
inline int hs_partial_blocks(int P, int dimx, int nrows) {
    int nb = hs_nblocks(P, nrows);
    nb = nb > hs2_nblocks(dimx, nrows) ? nb : hs2_nblocks(dimx, nrows);
    return nb > hs3_nblocks(dimx, nrows) ? nb : hs3_nblocks(dimx, nrows);
}
// Sum C iterations' per-block partials in a fixed order: sums[2t+{0,1}] =
// {sum ||diff||, sum ||prev||} for t < C.
// out[i] = sum over r < n of src[r][i], added in rank order (the in-process
// slab group's all-reduce, slab.cpp); n <= kMaxLocalRanks
constexpr int kMaxLocalRanks = 16;
// device-to-device copy of whole float2s on one device, by a few blocks
void launch_copy_lines(void *dst, const void *src, size_t bytes, hipStream_t st);
void launch_sum_ranks(const double *const *src, int n, size_t count, double *out, hipStream_t st);
// Row t of `partial` starts at t * stride * 2 doubles (stride = nblocks if < 0).
void launch_reduce_partials(const double *partial, int nblocks, int C, double *sums,
                            hipStream_t st, int stride = -1);
// The launches of one chunk: runs of consecutive iterations whose kernels wrote
// the same number of block partials, so that rows are reduced over exactly the
// blocks that wrote them (no zero fill of the partial rows per chunk).
struct PartialRuns {
    struct Run {
        int t0, len, nblocks;
    };
    std::vector<Run> runs;
    void add(int t, int len, int nblocks);
    void reduce(const double *partial, int stride, double *sums, hipStream_t st) const;
};

// ---------------------------------------------------------------- Logger norms
// The reference's Motion::norm (src/Motion.cpp:42-49) bit for bit: the float
// running sum S <- (float)((double)S + sqrt((double)x^2 + (double)y^2)) over
// the pixels in linear order, of |cur - prev| (out[0]) and |prev| (out[1])
// (Logger::update_error, src/Logger.cpp:32-51; seqnorm_kernels.hip).  out[]
// holds the sums, not yet divided by N.  ws: seqnorm_workspace_bytes; it also
// keeps each call's running-sum profile, which the next call on the same grid
// uses as its prediction when use_profile is set (the result is exact either
// way; a poor prediction costs time).  dbg (optional, int[10]): the walk's
// cost counters (resolves, raw segments, listed tiles, clocks, tiles given
// its own segment entries).
constexpr int kSnTile = 4096;  // consecutive terms per tile
size_t seqnorm_workspace_bytes(int dimx, int dimy);
void launch_seqnorm(const float2 *cur, const float2 *prev, int dimx, int dimy, int P, void *ws,
                    bool use_profile, float *out, int *dbg, hipStream_t st);
// the two halves of launch_seqnorm: the bandwidth passes (tables) and the
// latency-bound walk, so that a pipeline can run them on separate streams
// (the walk reads what tables wrote; tables reads the profile the last walk
// on the same workspace wrote)
void launch_seqnorm_tables(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                           void *ws, bool use_profile, hipStream_t st);
// s_in (optional, device float[2]): the exact running sums of the terms
// before this grid — a row slab's norms continue its predecessor's
void launch_seqnorm_walk(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                         void *ws, const float *s_in, float *out, int *dbg, hipStream_t st);
// launch_seqnorm_tables in parts for row slabs: the pass over the slab, its
// fp64 total (returned: device double[2] inside ws), the predecessors' totals
// chained in rank order for K pairs (poff = the previous rank's nxt, or 0
// without one; nxt = poff + tot: device double[K][2] each, prev_nxt
// peer-readable), and the
// check / fix with that offset (p_off, device double[2], optional)
void launch_seqnorm_pass(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                         void *ws, bool use_profile, hipStream_t st);
const double *seqnorm_total(int dimx, int dimy, int P, void *ws, hipStream_t st);
void launch_seqnorm_offset_chain(const double *prev_nxt, const double *const *tot, int K,
                                 double *poff, double *nxt, hipStream_t st);
void launch_seqnorm_refine(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                           void *ws, bool use_profile, const double *p_off, hipStream_t st);
// A batch of K <= 3 consecutive Logger updates of one loop: pair i is
// (prev, cur) = (u[i], u[i + 1]) on workspace ws[i] (its own profile), so the
// pass reads the K + 1 iterates once (a Jacobi triple's four arrays for three
// updates) and each of check, fix and walk is one launch for the batch.
struct SeqnormBatch {
    int K = 1;
    const float2 *u[4] = {};
    void *ws[3] = {};
    bool use_profile[3] = {};
    const double *p_off[3] = {};  // refine: a row slab's predecessors' fp64 sums
    const float *s_in[3] = {};    // walk: a row slab's predecessors' exact sums
    float *out[3] = {};           // walk: the sums of pair i (device float[2])
    int *dbg[3] = {};             // walk: cost counters (int[10]), optional
    // the loop's break word (launch_seqnorm_decide): with it, every kernel of
    // the batch returns at once when *stop < t0 (t0: the batch's first
    // iteration)
    const int *stop = nullptr;
    int t0 = 0;
    // the pass (launch_seqnorm_pass) over tiles [tile_lo, tile_hi) only
    // (tile_hi 0: every tile); the launch with tile_lo 0 resets the check's list
    unsigned tile_lo = 0, tile_hi = 0;
    // the pass's scale prediction (OF2D_SN_NEAR): workspaces of pair i in the
    // three groups before this one (their checks' fp64 totals, taken when the
    // check has stamped them with `epoch` + its iteration + 1), null: none
    void *near[3][3] = {};
    unsigned epoch = 0;  // the loop's tag in the stamps' high 12 bits
};
// the Logger errors of a walked batch (pair i's sums at seq[2i], seq[2i + 1]),
// as logger_error does on the host: the first iteration t0 + i > 1 whose
// error is below 0.001 into *stop (atomicMin); the sums copied to host
// (mapped host memory, float[2K])
void launch_seqnorm_decide(const float *seq, int K, int t0, double npx, int *stop, float *host,
                           hipStream_t st);
// diagnostics (tools/seqnorm_bench; synchronous): the workspace's list count
// and profile flags (cnt[0..3]), then per norm the tiles with segment entries,
// with more than one candidate, with none (out[12])
void seqnorm_ws_stats(const void *ws, int dimx, int dimy, unsigned *out);
void launch_seqnorm_pass(const SeqnormBatch &b, int dimx, int dimy, int P, hipStream_t st);
void launch_seqnorm_refine(const SeqnormBatch &b, int dimx, int dimy, int P, hipStream_t st);
void launch_seqnorm_walk(const SeqnormBatch &b, int dimx, int dimy, int P, hipStream_t st);

// ---------------------------------------------------------------- fields
void launch_d2f(const double *in, int dimx, int dimy, float *out, int P, int row_offset,
                hipStream_t st);
void launch_f2d(const float *in, int P, int dimx, int dimy, double *out, hipStream_t st);
void launch_motion_to_planar(const float2 *m, int P, int dimx, int dimy, double *out,
                             hipStream_t st);
void launch_downsample_image(const float *in, int dxi, int dyi, int Pi, float *out, int dxo,
                             int dyo, int Po, hipStream_t st);
void launch_downsample_motion(const float2 *in, int dxi, int dyi, int Pi, float2 *out, int dxo,
                              int dyo, int Po, hipStream_t st);
void launch_upsample_motion(const float2 *in, int dxi, int dyi, int Pi, float2 *out, int dxo,
                            int dyo, int Po, hipStream_t st);
void launch_warp(const float *src, const float2 *u, float *dst, int dimx, int dimy, int P,
                 hipStream_t st);
void launch_gradients(const float *Iref, const float *Iaux, float2 *dI, float *It, int dimx,
                      int dimy, int P, hipStream_t st);
// slab variant: rows [0, nrows) of a slab whose first row is global j-line row0;
// rows -1 and nrows are ghost j-lines holding the neighbours' image rows
void launch_gradients_rows(const float *Iref, const float *Iaux, float2 *dI, float *It, int dimx,
                           int nrows, int P, int row0, int dimy, hipStream_t st);
void launch_accumulate(const float2 *m_old, const float2 *v, float2 *m_new, int dimx, int dimy,
                       int P, hipStream_t st);
// Fluid regridding: m_new <- accumulate(m_old, est), est0 <- 0 over the image
// pixels (ghost lines and pitch padding are never written), Iaux <- warp(Imov, m_new)
void launch_regrid(const float2 *m_old, const float2 *est, float2 *est0, float2 *m_new,
                   const float *Imov, float *Iaux, int dimx, int dimy, int P, hipStream_t st);
void launch_compose_zero(const float2 *v, float2 *out, int dimx, int nrows, int P, int row0,
                         int dimy, hipStream_t st);
void launch_add_motion(const float2 *a, const float2 *b, float2 *out, int dimx, int dimy, int P,
                       hipStream_t st);

// ---------------------------------------------------------------- Demons
void launch_demons_force(const float *Iref, const float *Imov, const float2 *u, float2 *corr,
                         int dimx, int dimy, int P, float sigma_isq, float sigma_xsq,
                         unsigned *status, hipStream_t st);
dim3 conv_grid(int dimx, int dimy);
int conv_nblocks(int dimx, int dimy);
// One correction update (DemonsThirions.cpp:20-38): force, sigma_fluid
// smoothing and the motion update (mode as launch_smooth_compose) -> out.
// One fused launch over every tile (demons_fused_kernel; the x-edge tiles hold
// the wrapped tap pixels) for kw 3 / 5 / 7 and dimx >= 128; otherwise the
// unfused kernels through corr (scratch).
void launch_demons_update(const float *Iref, const float *Imov, const float2 *u, float2 *corr,
                          float2 *out, int dimx, int dimy, int P, float sigma_isq,
                          float sigma_xsq, const float *kf, const double *kd, int kw,
                          double wfull, int mode, unsigned *status, hipStream_t st);
// mode 0 Composition, 1 Addition, 2 no update, 3 store the smoothed corr only
void launch_smooth_compose(const float2 *corr, const float2 *u, float2 *out, int dimx, int dimy,
                           int P, const float *kf, const double *kd, int kw, double wfull,
                           int mode, hipStream_t st);
void launch_smooth_norm(const float2 *umid, const float2 *prev, float2 *out, int dimx, int dimy,
                        int P, const float *kf, const double *kd, int kw, double wfull,
                        double *partial, hipStream_t st);
// Motion::exp (Motion.cpp:253-277) on f; *result is f or scratch
void launch_motion_exp(float2 *f, float2 *scratch, int dimx, int dimy, int P, int nsq_max,
                       float *d_part, int nparts, int *d_nsq, float *d_maxabs, unsigned *status,
                       float2 **result, hipStream_t st);

// ---------------------------------------------------------------- Curvature
// C = A B (column-major fp64, MFMA), times E elementwise when E != nullptr;
// batch z offsets A, B, C by sA, sB, sC elements
void launch_dgemm(int M, int N, int K, const double *A, long lda, long sA, const double *B,
                  long ldb, long sB, double *C, long ldc, long sC, const double *E, long lde,
                  int batch, hipStream_t st);
// X planes (x at 0, y at `plane`, pitch P) <- (double)(u - tau * force(u))
void launch_curv_rhs(const float2 *u, const float2 *dI, const float *It, float tau, int dimx,
                     int dimy, int P, double *X, long plane, hipStream_t st);
int curv_nblocks(int dimx, int dimy);
// out <- (float)Z / div, Logger partials against u
void launch_curv_construct(const double *Z, long plane, const float2 *u, float2 *out, float div,
                           int dimx, int dimy, int P, double *partial, hipStream_t st);

// ---------------------------------------------------------------- Fluid / Elastic
int sor_nstrips(int dimx);
// The SOR working array vb is stored skewed along the Gauss-Seidel wavefront:
// pixel (i, j) at row 2i + j, column i (fluid_kernels.hip).  A row is 16 P
// bytes: P float2 values of the field being relaxed (v), then P float2
// right-hand sides (b), so the passes that write only b (the force) or read
// only v write / read contiguous runs of 8-B elements.  It has
// sor_rows(dimx, dimy) rows; the last kSorPadRows are padding for lanes that
// run past the image (as do the kSorPadRows above and below each granule region).
constexpr int kSorPadRows = 256;
// float2 index of v(i, j) / b(i, j) in vb
__host__ __device__ inline long sor_v(int i, int j, int P) { return (2L * i + j) * 2L * P + i; }
__host__ __device__ inline long sor_b(int i, int j, int P) { return sor_v(i, j, P) + P; }
inline int sor_rows(int dimx, int dimy) { return 2 * dimx + dimy + kSorPadRows; }
long sor_granule_stride(int dimy);
// (nstrips + 1) regions of 16-B granules, zeroed once
size_t sor_granule_bytes(int dimx, int dimy);
// in-place Gauss-Seidel SOR sweep (OpticalFlowFluid.cpp:7-41), wavefront-exact,
// on the skewed vb (v and b halves per row, sor_rows rows of 16 P bytes).
// epoch: > every earlier epoch on H, the same epoch as the sor_pack before it;
// ticket: per-H counter, a multiple of nstrips before the launch.
void launch_sor(float4 *vb, int dimx, int dimy, int P, float mu, float lambda, float omega,
                void *H, unsigned epoch, unsigned *ticket, unsigned *status, hipStream_t st,
                FluidCtl ctl = {});
// vb's b <- force(u, dI, It); if v != nullptr also vb's v <- v; granule region
// 0 <- column 0 of v tagged with epoch
void launch_sor_pack(float4 *vb, const float2 *u, const float2 *dI, const float *It,
                     const float2 *v, int dimx, int dimy, int P, void *H, unsigned epoch,
                     hipStream_t st);
// after a regrid: dI, It <- gradients of Iaux (set_derivatives) and vb's b <-
// force of a zero estimate, granule region 0 <- column 0 of v tagged epoch
void launch_regrid_pack(const float *Iref, const float *Iaux, float2 *dI, float *It, float4 *vb,
                        int dimx, int dimy, int P, void *H, unsigned epoch, hipStream_t st,
                        FluidCtl ctl = {});
void launch_force(const float2 *u, const float2 *dI, const float *It, float2 *f, int dimx,
                  int dimy, int P, hipStream_t st);
int increment_nblocks(int dimx, int dimy);
// the Fluid sweep with the increment behind it (fluid_kernels.hip SorInc): the
// sweep of launch_sor plus launch_increment's R, partials and scal in one
// launch (+ the timestep reduction).  ticket: 1 + nstrips words of the level
// (the sweep ticket, then per strip its last finished epoch), zero at
// allocation; ctr: 2 counters, zero at allocation.  Falls back to launch_sor
// + launch_increment where too few CUs are left for workers; with
// sor_increment_workers() == 0 (OF2D_SOR_NCONS=0) the caller runs those.
int sor_increment_workers();
void launch_sor_increment(float4 *vb, int dimx, int dimy, int P, float mu, float lambda,
                          float omega, void *H, unsigned epoch, unsigned *ticket,
                          unsigned long long *ctr, const float2 *u, float2 *R, float *part,
                          float *scal, unsigned *status, hipStream_t st, FluidCtl ctl = {});
// R and scal[0] = maxabs(R), scal[1] = 0.65f / maxabs
void launch_increment(const float2 *u, const float4 *vel, float2 *R, int dimx, int dimy, int P,
                      float *part, float *scal, hipStream_t st, FluidCtl ctl = {});
// uo <- u + R dt (dt < 65) or u; Logger partials of uo against prev (against u
// when prev is null); per-block Jacobian minima of uo into jpart (their min:
// launch_fluid_report); vb's b <- force(uo) and granule region 0 tagged with
// `epoch` for the next sweep (fluid_kernels.hip fluid_step_kernel)
void launch_fluid_step(const float2 *u, const float2 *R, float2 *uo, const float2 *prev,
                       const float *scal, const float2 *dI, const float *It, float4 *vb, int dimx,
                       int dimy, int P, void *H, unsigned epoch, double *lpart, float *jpart,
                       hipStream_t st, FluidCtl ctl = {});
// Per-iteration report a kernel writes straight into host memory (fine-grained
// pinned, so no copy launches): the Fluid loop's Logger sums, maxabs, dt,
// min Jacobian and status word
struct FluidReport {
    double sums[2];
    float maxabs, dt, jmin;
    unsigned status;
    float seq[2];   // the reference's float Logger sums (exact mode)
    float err;      // the Logger error as the host computes it (logger_error)
    unsigned flags;  // kFluidBreak, kFluidRegrid; kFluidDone once written
};
constexpr unsigned kFluidBreak = 1u, kFluidRegrid = 2u, kFluidDone = 4u;
// The end of a Fluid iteration's device work: the nb Logger partial pairs
// reduced as launch_reduce_partials does (same order, same bits), the minimum
// of the nb Jacobian partials into scal[2], and {sums, scal[0..2], *status}
// written to the host-mapped FluidReport (one launch instead of reduce + min +
// three copies)
void launch_fluid_report(const double *lpart, int nb, const float *jpart, float *scal,
                         const unsigned *status, FluidReport *report, hipStream_t st);
// ... and the iteration's decisions on the device (ImageRegistrationFluid.cpp:
// 99-124): err from the exact float sums `seq` (the reference's Logger) or from
// the fp64 sums (seq null), the break (!fixed, err < 0.001f, it > 1: the stop
// word), the regrid (no break and min Jacobian < 0.5: kFluidRegridWord, and the
// motion index flips); the report carries them for the host's lines
void launch_fluid_report_decide(const double *lpart, int nb, const float *jpart, float *scal,
                                const float *seq, double npx, bool fixed, FluidReport *report,
                                hipStream_t st, FluidCtl ctl);
// the regrid of an iteration that decided one (kFluidRegridWord; a no-op
// otherwise): motion[mcur'] <- accumulate(motion[1 - mcur'], est) with mcur'
// the flipped index, Iaux <- warp2d(Imov, new motion); est is left as it is
// (the next iteration reads it as zero and as the Logger's prev)
void launch_regrid_if(float2 *m0, float2 *m1, const float2 *est, const float *Imov, float *Iaux,
                      int dimx, int dimy, int P, hipStream_t st, FluidCtl ctl);
void launch_logger(const float4 *vb, float2 *u, float2 *prev, int dimx, int dimy, int P,
                   double *partial, hipStream_t st);

}  // namespace of2d
