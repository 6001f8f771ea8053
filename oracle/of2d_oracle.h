/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, -ffp-contract=off) of the reference registration
 * path of tjwdraper/OpticalFlow2d.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / CPU
 * baseline.  The product path (libof2d.so) never links or calls it.
 *
 * Every function cites the reference file:line it restates.
 * Parity pinning: see oracle/README.md (primitives pinned bitwise against the
 * reference's own coord2d.h / gradients.h / Kernel.cpp compiled from
 * /root/reference into oracle/_ref/; whole-path HS pinned by the reference
 * outputs recorded in SURVEY.md §8c).
 */
#ifndef OF2D_ORACLE_H
#define OF2D_ORACLE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_reg oracle_reg;

/* ---- registration object (mirrors ImageRegistration* driven by mexFunction) ---- */
int oracle_create(oracle_reg **out, int dimx, int dimy, const int *niter, int nscales,
                  int reg, const float *regparams, unsigned nparams, int nrefine,
                  int verbose);
int oracle_set_images(oracle_reg *r, const double *ref, const double *mov);
int oracle_estimate(oracle_reg *r);
int oracle_get_motion(oracle_reg *r, double *out_planar);
int oracle_warp(oracle_reg *r, const double *mov, double *out);
void oracle_destroy(oracle_reg *r);
const char *oracle_last_error(void);
/* iterations executed per (level, refine) in execution order; returns count */
int oracle_iterations(const oracle_reg *r, int *out, int cap);
/* 1 = run every iteration (no convergence break) — bench-only knob */
void oracle_set_fixed_iters(oracle_reg *r, int on);
/* per-iteration Logger errors of the last loop executed (float), returns count */
int oracle_last_errors(const oracle_reg *r, float *out, int cap);

/* printed text (banner, verbose lines, Fluid lines) captured instead of stdout */
void oracle_capture_output(int on);
const char *oracle_captured_output(void);
void oracle_clear_output(void);

/* ---- primitives (interleaved motion = float[2*N], x fastest) ---- */
void oracle_spatial_derivative(const float *I, int dimx, int dimy, float *dI);
void oracle_temporal_derivative(const float *Iref, const float *Imov, int n, float *It);
void oracle_qlaplacian(const float *u, int dimx, int dimy, float *q);
/* one OpticalFlowDiffusion::get_update, in place on u; returns 0 or -1 (div by zero) */
int oracle_hs_update(float *u, const float *dI, const float *It, int dimx, int dimy, float alpha);
/* HS iteration loop as in ImageRegistrationOpticalFlow.cpp:123-135 (u starts as given);
 * returns iterations executed or -1 on error; errs[] receives Logger errors */
int oracle_hs_loop(float *u, const float *dI, const float *It, int dimx, int dimy, float alpha,
                   int niter, int fixed, float *errs);
int oracle_hs_loop_mt(float *u, const float *dI, const float *It, int dimx, int dimy,
                      float alpha, int niter, int nthreads, float *errs);
float oracle_motion_norm(const float *u, int n);
float oracle_motion_norm_sum(const float *u, int n);
float oracle_motion_maxabs(const float *u, int n);
void oracle_warp2d(float *I, const float *u, int dimx, int dimy);
void oracle_accumulate(float *u, const float *v, int dimx, int dimy);
void oracle_gaussian_kernel(int kw, float sigma, double *k);
void oracle_convolute_motion(float *u, int dimx, int dimy, const double *k, int kw);
void oracle_convolute_image(float *I, int dimx, int dimy, const double *k, int kw);
void oracle_downsample_image(const float *in, int dx_in, int dy_in, float *out, int dx_out, int dy_out);
void oracle_upsample_image(const float *in, int dx_in, int dy_in, float *out, int dx_out, int dy_out);
void oracle_downsample_motion(const float *in, int dx_in, int dy_in, float *out, int dx_out, int dy_out);
void oracle_upsample_motion(const float *in, int dx_in, int dy_in, float *out, int dx_out, int dy_out);
int oracle_demons_force(const float *dI, const float *It, int n, float sigma_i, float sigma_x,
                        float *c);
void oracle_jacobian(const float *u, int dimx, int dimy, float *jac);
float oracle_image_min(const float *I, int n);
void oracle_motion_exp(float *u, int dimx, int dimy);
/* one in-place SOR sweep (OpticalFlowFluid.cpp:7-41 == OpticalFlowElastic.cpp:21-55) */
void oracle_sor_sweep(float *x, const float *b, int dimx, int dimy, float mu, float lambda,
                      float omega);
void oracle_get_force(const float *u, const float *dI, const float *It, int n, float *f);
void oracle_dct2d(double *a, int n0, int n1, int kind);
void oracle_fluid_increment(const float *u, const float *v, int dimx, int dimy, float *R);

/* thread/loop-order knob for the CPU baseline: 1 = reference loop order
 * (i outer, j inner, strided), 0 = row order (same results, faster) */
void oracle_set_reference_loop_order(int on);
void oracle_set_logger_fp64(int on);

#ifdef __cplusplus
}
#endif
#endif
