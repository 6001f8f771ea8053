/*
 * of2d.h — C-ABI of the MI355X-native OpticalFlow2d registration library
 * (libof2d.so).  Plain pointers and sizes only; every entry point returns an
 * int status (OF2D_OK = 0) and never throws across the boundary.
 *
 * The boundary replaces the reference's MEX entry point and the operator
 * plug-in point underneath it:
 *
 *   reference                                   replaced by
 *   -----------------------------------------   ---------------------------------
 *   mexFunction (WrapperOpticalFlow2d.cpp:18-20) of2d_gateway (same 5 modes)
 *   init branch            (:23-83)              of2d_create
 *   register branch        (:86-102)             of2d_set_images + of2d_estimate
 *   get-motion branch      (:105-117)            of2d_get_motion
 *   warp branch            (:120-137)            of2d_warp
 *   close branch           (:140-147)            of2d_destroy
 *   ImageRegistration::estimate_motion
 *     (src/ImageRegistration.cpp:133-156) and every
 *     IterativeSolver::get_update
 *     (src/regularization/IterativeSolver.h:22)  of2d_estimate (device-resident)
 *   enum Regularisation/Verbose/MotionAccumulation
 *     (src/SolverOptions.h:4-8)                  OF2D_REG_* / OF2D_VERBOSE_* /
 *                                                OF2D_ACCUM_* (same values)
 *
 * Array layout at the boundary is the reference's: column-major with x fast,
 * idx = i + j*dimx (src/Field.tpp:13; MATLAB [dimx, dimy]); images are double
 * [dimx*dimy]; a motion field is planar double [dimx*dimy*2], x-plane first
 * (src/Motion.cpp:23-39).
 */
#ifndef OF2D_H
#define OF2D_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define OF2D_OK 0
#define OF2D_ERR_INVALID_ARGUMENT 1 /* std::invalid_argument / mexErrMsgTxt on bad input */
#define OF2D_ERR_RUNTIME 2          /* std::runtime_error, e.g. "Divide by zero exception" */
#define OF2D_ERR_DEVICE 3           /* HIP / RCCL failure */
#define OF2D_ERR_STATE 4            /* call sequence not allowed (mexErrMsgTxt :149-151) */

/* ---- SolverOptions.h:4-8, identical integer values ---- */
enum of2d_regularisation {
    OF2D_REG_DIFFUSION = 0,
    OF2D_REG_CURVATURE = 1,
    OF2D_REG_ELASTIC = 2,
    OF2D_REG_THIRIONS_DEMONS = 3,
    OF2D_REG_DIFFEOMORPHIC_DEMONS = 4,
    OF2D_REG_FLUID = 5
};
enum of2d_verbose { OF2D_VERBOSE_OFF = 0, OF2D_VERBOSE_ON = 1 };
enum of2d_motion_accumulation { OF2D_ACCUM_COMPOSITION = 0, OF2D_ACCUM_ADDITION = 1 };

typedef struct of2d_ctx of2d_ctx;

/* Text the reference prints with mexPrintf (parameter banner
 * ImageRegistration.cpp:6-47, Logger lines Logger.cpp:62-69, Fluid lines
 * OpticalFlowFluid.cpp:94, ImageRegistrationFluid.cpp:110) goes through this
 * hook; NULL restores the default (stdout).  Process-global. */
typedef void (*of2d_print_fn)(const char *text, void *user);
void of2d_set_print_hook(of2d_print_fn fn, void *user);

/* ---- registration object (replaces the init branch, :23-83) ----
 * niter has nscales+1 entries (finest level first, :35-38); regparams has
 * nparams entries whose meaning follows the reference per regularisation
 * (ImageRegistrationOpticalFlow.cpp:8-68, ImageRegistrationDemons.cpp:7-57,
 * ImageRegistrationFluid.cpp:5-36).  Invalid nparams fails with
 * OF2D_ERR_INVALID_ARGUMENT and the reference's message. */
int of2d_create(of2d_ctx **out, int dimx, int dimy, const int *niter, int nscales, int reg,
                const float *regparams, unsigned nparams, int nrefine, int verbose);
/* register branch (:86-102): images are double [dimx*dimy] */
int of2d_set_images(of2d_ctx *ctx, const double *Iref, const double *Imov);
int of2d_estimate(of2d_ctx *ctx);
/* get-motion branch (:105-117): out is double [dimx*dimy*2], planar */
int of2d_get_motion(of2d_ctx *ctx, double *out);
/* warp branch (:120-137): out is double [dimx*dimy] */
int of2d_warp(of2d_ctx *ctx, const double *Imov, double *out);
/* close branch (:140-147) */
int of2d_destroy(of2d_ctx *ctx);
const char *of2d_last_error(const of2d_ctx *ctx);
/* iterations executed per (level, refine) of the last of2d_estimate, in
 * execution order (coarsest level first); returns the number of entries */
int of2d_iterations_executed(const of2d_ctx *ctx, int *out, int cap);
/* per-iteration Logger error (Logger.cpp:32-51) of the last loop executed */
int of2d_last_errors(const of2d_ctx *ctx, float *out, int cap);
/* Options that the reference does not have (bench / deployment only):
 *   "fixed_iters" (0/1): run every iteration, no convergence break
 *   "chunk" (>=1): iterations enqueued between host convergence checks
 *   "device" (>=0): HIP device ordinal, must be set before of2d_set_images
 *   "hs_gradients_from_image" (-1 auto = default, 0, 1): as for the slab
 *   solver (of2d_slab_set_option); bit-identical results either way
 *   "ngpus" (1 = default .. 16): Horn-Schunck levels run as that many row
 *   slabs, rank r on device (device + r) mod count, in this process (halos and
 *   the Logger's running sums cross the ranks by peer copies; the pyramid,
 *   warps and accumulation stay on the registration's device).  Results are
 *   the one-device results bit for bit with the default Logger norms.  Levels
 *   with fewer j-lines than ranks run on one device.  Ranks beyond the device
 *   count are merged (a device runs one slab of rows; splitting it only adds
 *   halo work) unless "ngpus_share" is set.
 *   "ngpus_share" (0 = default / 1): ranks may share a device, (device + r)
 *   mod count for every r < ngpus (the decomposition on fewer devices than
 *   ranks: tests, timings of the path's overhead on one GPU).
 *   "slab_split" (-1 auto = default, 0, 1): the ranks' slab option "split"
 *   (of2d_slab_set_option).
 *   "logger_fp64" (0 = default / 1): 0 computes the Logger norms as the
 *   reference does (float running sums, of2d_motion_norms), so the break of
 *   ImageRegistrationOpticalFlow.cpp:131-134 falls on the reference's
 *   iteration at every size; 1 sums the magnitudes in fp64 (faster: the fused
 *   multi-iteration kernels stay on; at >= 4096^2 the break can move by a few
 *   iterations).  fixed_iters runs take no break and use the fp64 sums. */
int of2d_set_option(of2d_ctx *ctx, const char *key, double value);

/* ---- gateway: the process-global singleton of WrapperOpticalFlow2d.cpp:13.
 * Mode is keyed on (nlhs, nrhs, singleton present) exactly like mexFunction:
 *   init (0,8,no)  prhs = {[dimx dimy], niter, nscales, reg, regparams,
 *                          nparams, nrefine, verbose}
 *   init (0,9,no)  the same plus ngpus (of2d_set_option "ngpus"): not in the
 *                  reference, which has no multi-device mode
 *   register (0,2,yes) prhs = {Iref, Imov}
 *   get (1,0,yes)  plhs[0] = double [dimx*dimy*2]
 *   warp (1,1,yes) prhs = {Imov}, plhs[0] = double [dimx*dimy]
 *   close (0,0,yes)
 * anything else: OF2D_ERR_STATE with the reference's message (:149-151).
 * plhs buffers are caller-allocated; of2d_gateway_output_numel tells the size. */
int of2d_gateway(int nlhs, double **plhs, int nrhs, const double *const *prhs);
size_t of2d_gateway_output_numel(int nlhs, int nrhs);
int of2d_gateway_output_dims(int nlhs, int nrhs, size_t *dims, int *ndims);
const char *of2d_gateway_last_error(void);

/* ---- row-slab Horn-Schunck solver (multi-GPU north-star path) ----
 * One process per GPU.  Global grid dimx x dimy is split into contiguous slabs
 * of j-lines; rank r owns rows [row_begin, row_end) (of2d_slab_bounds).  The
 * halo (K j-lines to each neighbour before every fused launch of K = 3, 2 or 1
 * iterations) travels over RCCL, overlapped with the interior row bands.  A
 * slab needs >= 3 j-lines.
 * nranks == 1 needs no unique id (pass NULL); with one, a one-rank RCCL
 * communicator carries the Logger all-reduces (exercises RCCL on one GPU). */
int of2d_slab_bounds(int dimy, int rank, int nranks, int *row_begin, int *row_end);
int of2d_rccl_unique_id_size(void);
int of2d_rccl_get_unique_id(void *out, int len);
typedef struct of2d_slab of2d_slab;
int of2d_slab_create(of2d_slab **out, int dimx, int dimy, float alpha, int rank, int nranks,
                     int device, const void *rccl_unique_id, int id_len);
/* images: rows [row_begin-3, row_end+3) clipped to [0, dimy), double, x fast
 * (three halo rows: iterations run fused in threes, whose first step also
 * covers two halo j-lines on each side) */
int of2d_slab_set_images(of2d_slab *s, const double *Iref_rows, const double *Imov_rows);
/* The slab's per-run setup lives outside of2d_slab_run: set_images computes the
 * gradients and the divide-by-zero / division-range test (dI is fixed per image
 * pair), and every run ends by zeroing the buffer the next run starts from
 * (motion_est->reset(), ImageRegistrationOpticalFlow.cpp:141), enqueued behind
 * the run's end event.  of2d_slab_reserve sizes the per-iteration Logger sums
 * of a fixed_iters run of niter iterations (3000 are reserved at create), so a
 * run allocates nothing. */
int of2d_slab_reserve(of2d_slab *s, int niter);
/* runs niter Jacobi iterations (HS, Logger, convergence unless fixed_iters)
 * from zero motion (ImageRegistrationOpticalFlow.cpp:123-135); *iters_done
 * receives the iterations executed */
int of2d_slab_run(of2d_slab *s, int niter, int fixed_iters, int *iters_done);
/* owned rows of the motion, planar double [dimx*nrows*2] */
int of2d_slab_get_motion(of2d_slab *s, double *out);
/* average duration (microseconds) of one launch of the Jacobi kernel (the
 * fused kernel: THREE iterations per launch, over the whole slab in one
 * launch) over nlaunch launches, timed with HIP events on the stream it is
 * launched on.  The launches read the zeroed start buffer and write scratch:
 * the last run's motion (of2d_slab_get_motion) is left intact. */
int of2d_slab_time_kernel(of2d_slab *s, int nlaunch, double *avg_us);
/* slab facts for reports: info[0..10] = {nranks, ranks of the RCCL
 * communicator (ncclCommCount; 0 without one), in-process group (0/1),
 * row_begin, row_end, dimx, pitch (elements), halo j-lines exchanged per fused
 * launch, interior/edge split (0/1), triple kernel derives dI from Iaux (0/1),
 * Logger of a convergence-on run (1: the reference's float running sums,
 * 0: fp64 sums — "logger_fp64" resolved)}; returns the number of entries
 * written */
int of2d_slab_info(const of2d_slab *s, int *info, int n);
/* the Logger errors of the last of2d_slab_run's iterations (the global ones:
 * the same on every rank), up to n into out; returns how many there are */
int of2d_slab_last_errors(const of2d_slab *s, float *out, int n);
/* wall time (ms, HIP events) of the last of2d_slab_run on this rank */
int of2d_slab_last_run_ms(const of2d_slab *s, double *ms);
/* the triple kernel's own average launch time (us) inside the last run,
 * from HIP events bracketing the back-to-back triple launches of each of its
 * first 64 chunks on the solver's stream (halo exchange included for N > 1),
 * and the number of launches that average covers */
int of2d_slab_last_run_kernel_us(const of2d_slab *s, double *avg_us, int *nlaunch);
/* the halo's cost inside the last run, sampled with HIP events on the first 8
 * split triples (interior launch beside the exchange and two edge launches):
 * us3[0] the solver stream's wait for the previous launch's edges before the
 * interior may start (the stall the halo puts on the critical stream),
 * us3[1] the exchange on the halo stream (ncclGroupStart .. ncclGroupEnd of
 * the sends / receives, or the in-process copies, including the wait for the
 * neighbours), us3[2] the two edge launches; averages per sampled launch, and
 * *nsampled the launches sampled (0 when the run had no split triples) */
int of2d_slab_last_run_halo_us(const of2d_slab *s, double *us3, int *nsampled);
/* options (no reference counterpart):
 *   "hs_gradients_from_image" (-1 auto = default, 0, 1): the triple kernel
 *   derives dI from Iaux in the kernel (24 B/px per launch) instead of reading
 *   dI (28); auto does so when dI + It (12 B/px) exceed the 256 MB MALL;
 *   bit-identical either way
 *   "logger_fp64" (-1 auto = default, 0, 1): as of2d_set_option's; 0 takes
 *   the convergence-on Logger norms as the reference does (one float running
 *   sum over the slabs in rank order, so the break falls on the one-grid
 *   reference's iteration), 1 sums the fused fp64 partials (fixed_iters runs
 *   always do); auto is 0 except on an RCCL communicator of two or more
 *   ranks, where the rank-to-rank chain of the running sums (two more
 *   communicators on two more streams) has not run on hardware: 1 there,
 *   unless 0 is set
 *   "split" (-1 auto = default, 0, 1): triples as an interior launch beside
 *   the halo exchange and two edge launches (auto: when a neighbour is on
 *   another device or behind RCCL), never, or whenever the slab has >= 48
 *   j-lines AND a halo to exchange — two or more ranks, or a one-rank
 *   communicator with "rccl_self_halo" (tests of the multi-device launch
 *   order on one device; a one-rank slab without either stays unsplit
 *   whatever is set); bit-identical either way
 *   "rccl_self_halo" (0 = default, 1; a one-rank RCCL communicator only):
 *   every halo exchange also sends the slab's boundary j-lines to rank 0
 *   itself (ncclSend / ncclRecv in a group, into a scratch buffer that is never
 *   read), and "split" 1 then splits the one-rank slab: the RCCL halo calls
 *   of an N-rank run, rehearsed on one GPU; bit-identical */
int of2d_slab_set_option(of2d_slab *s, const char *key, double value);
int of2d_slab_destroy(of2d_slab *s);
const char *of2d_slab_last_error(const of2d_slab *s);
/* In-process slab group: the nranks slabs of one grid in ONE process, driven by
 * one host thread per rank, exchanging the same halo lines and Logger sums by
 * device copies (ordered with HIP events, the threads meeting at a barrier per
 * exchange) instead of RCCL.  Same slab code and launches as the RCCL path; it
 * lets the decomposition run on a single GPU, where RCCL refuses two ranks on
 * one device (tests/test_gpu_slab_local.py).  nranks <= 16.  Create the group,
 * then one slab per rank with of2d_slab_create_local; call of2d_slab_run on all
 * ranks concurrently; destroy the slabs before the group. */
typedef struct of2d_slab_group of2d_slab_group;
int of2d_slab_group_create(of2d_slab_group **out, int nranks);
int of2d_slab_group_destroy(of2d_slab_group *g);
int of2d_slab_create_local(of2d_slab **out, int dimx, int dimy, float alpha, int rank,
                           int nranks, int device, of2d_slab_group *g);

/* ---- kernel-level test entry: the Logger's norms ----
 * Motion::norm (src/Motion.cpp:42-49) as Logger::update_error (src/Logger.cpp:
 * 32-51) takes it: the float running sums, in linear order, of
 * sqrt((double)x^2 + (double)y^2) over (cur - prev) -> sums[2k] and over prev
 * -> sums[2k+1] (not divided by dimx*dimy), bit-identical to the reference's.
 * cur / prev: npairs host fields of float [dimx*dimy*2] each, interleaved x, y
 * per pixel (coord2d), idx = i + j*dimx; the pairs run in order on one
 * workspace, so pair k's walk predicts pair k+1's, as in a Logger loop.
 * stats (optional, int[8*npairs], cost figures, not results): per pair the
 * tiles the device walk resolved below tile level (|cur - prev|, |prev|), the
 * 64-term segments it stepped term by term (same order), the tiles whose
 * entries were recomputed, the walk's wall-clock ticks at 100 MHz (same
 * order) and those of the |cur - prev| walk's resolves. */
int of2d_motion_norms(const float *cur, const float *prev, int dimx, int dimy, int npairs,
                      float *sums, int *stats);
/* The Logger norms of a chain of iterates u[0 .. niter] (niter + 1 fields of
 * dimx*dimy*2 floats): sums[2k], sums[2k + 1] are those of the update from
 * u[k] to u[k + 1], as of2d_motion_norms gives them, computed the way the
 * registration loop batches them: `batch` (1..3) consecutive updates per
 * batch, whose pass reads each iterate once, on four sets of workspaces in
 * rotation (batch g's profile is batch g - 4's, Registration::kSeqSets).  The
 * launches run in order on one stream: the sums match the registration's,
 * its stream schedule (walks on three streams, the stop word) is not
 * reproduced.  stats as of2d_motion_norms, per update.  Not in the
 * reference: a test entry for the batched device norms. */
int of2d_motion_norms_chain(const float *u, int dimx, int dimy, int niter, int batch,
                            float *sums, int *stats);

/* ---- library info ---- */
const char *of2d_version(void);
int of2d_device_count(int *count);

#ifdef __cplusplus
}
#endif
#endif
