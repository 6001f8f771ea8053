// capi.cpp — the extern "C" boundary of libof2d.so (include/of2d.h).
//
// Every entry point catches the C++ exceptions of the driver and turns them
// into a status code plus the reference's message, so nothing throws across
// the ABI.  The gateway reproduces mexFunction's five modes over the same
// process-global singleton (WrapperOpticalFlow2d.cpp:13-155).
#include "../../include/of2d.h"

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "of2d_host.h"

struct of2d_ctx {
    std::unique_ptr<of2d::Registration> reg;
    std::string err;
};

namespace {
of2d_print_fn g_print = nullptr;
void *g_print_user = nullptr;
std::mutex g_print_mu;
thread_local std::string g_gateway_err;

template <class F>
int guarded(std::string &err, F &&f) {
    try {
        f();
        err.clear();
        return OF2D_OK;
    } catch (const std::invalid_argument &e) {
        err = e.what();
        return OF2D_ERR_INVALID_ARGUMENT;
    } catch (const of2d::DeviceError &e) {
        err = e.what();
        return OF2D_ERR_DEVICE;
    } catch (const std::exception &e) {
        err = e.what();
        return OF2D_ERR_RUNTIME;
    } catch (...) {
        err = "unknown error";
        return OF2D_ERR_RUNTIME;
    }
}
}  // namespace

namespace of2d {
void print(const char *fmt, ...) {
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    std::lock_guard<std::mutex> lk(g_print_mu);
    if (g_print)
        g_print(buf, g_print_user);
    else {
        fputs(buf, stdout);
        fflush(stdout);
    }
}
}  // namespace of2d

extern "C" {

void of2d_set_print_hook(of2d_print_fn fn, void *user) {
    std::lock_guard<std::mutex> lk(g_print_mu);
    g_print = fn;
    g_print_user = user;
}

const char *of2d_version(void) { return "opticalflow2d_amd 0.1 (gfx950)"; }

int of2d_device_count(int *count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (count) *count = (e == hipSuccess) ? n : 0;
    return e == hipSuccess ? OF2D_OK : OF2D_ERR_DEVICE;
}

int of2d_create(of2d_ctx **out, int dimx, int dimy, const int *niter, int nscales, int reg,
                const float *regparams, unsigned nparams, int nrefine, int verbose) {
    if (!out) return OF2D_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    auto *c = new of2d_ctx();
    std::string err;
    int rc = guarded(err, [&] {
        if (!niter) throw std::invalid_argument("niter is NULL");
        if (nparams > 0 && !regparams) throw std::invalid_argument("regparams is NULL");
        static const float zero = 0.0f;
        c->reg.reset(new of2d::Registration(dimx, dimy, nscales, niter, nrefine, reg,
                                            nparams ? regparams : &zero, nparams, verbose));
    });
    if (rc != OF2D_OK) {
        g_gateway_err = err;
        delete c;
        return rc;
    }
    *out = c;
    return OF2D_OK;
}

int of2d_set_images(of2d_ctx *ctx, const double *Iref, const double *Imov) {
    if (!ctx || !Iref || !Imov) return OF2D_ERR_INVALID_ARGUMENT;
    return guarded(ctx->err, [&] { ctx->reg->set_images(Iref, Imov); });
}

int of2d_estimate(of2d_ctx *ctx) {
    if (!ctx) return OF2D_ERR_INVALID_ARGUMENT;
    return guarded(ctx->err, [&] { ctx->reg->estimate(); });
}

int of2d_get_motion(of2d_ctx *ctx, double *out) {
    if (!ctx || !out) return OF2D_ERR_INVALID_ARGUMENT;
    return guarded(ctx->err, [&] { ctx->reg->get_motion(out); });
}

int of2d_warp(of2d_ctx *ctx, const double *Imov, double *out) {
    if (!ctx || !Imov || !out) return OF2D_ERR_INVALID_ARGUMENT;
    return guarded(ctx->err, [&] { ctx->reg->warp(Imov, out); });
}

int of2d_destroy(of2d_ctx *ctx) {
    if (!ctx) return OF2D_ERR_INVALID_ARGUMENT;
    std::string err;
    int rc = guarded(err, [&] { ctx->reg.reset(); });
    delete ctx;
    return rc;
}

const char *of2d_last_error(const of2d_ctx *ctx) {
    return ctx ? ctx->err.c_str() : g_gateway_err.c_str();
}

int of2d_iterations_executed(const of2d_ctx *ctx, int *out, int cap) {
    if (!ctx) return -1;
    const auto &v = ctx->reg->iterations();
    for (int i = 0; i < (int)v.size() && i < cap; i++) out[i] = v[i];
    return (int)v.size();
}

int of2d_last_errors(const of2d_ctx *ctx, float *out, int cap) {
    if (!ctx) return -1;
    const auto &v = ctx->reg->last_errors();
    for (int i = 0; i < (int)v.size() && i < cap; i++) out[i] = v[i];
    return (int)v.size();
}

int of2d_set_option(of2d_ctx *ctx, const char *key, double value) {
    if (!ctx || !key) return OF2D_ERR_INVALID_ARGUMENT;
    return guarded(ctx->err, [&] { ctx->reg->set_option(key, value); });
}

int of2d_motion_norms(const float *cur, const float *prev, int dimx, int dimy, int npairs,
                      float *sums, int *stats) {
    if (!cur || !prev || !sums || dimx <= 0 || dimy <= 0 || npairs <= 0)
        return OF2D_ERR_INVALID_ARGUMENT;
    std::string err;
    int rc = guarded(err, [&] {
        of2d::Field<float2> c, p;
        c.alloc(dimx, dimy);
        p.alloc(dimx, dimy);
        const size_t n = (size_t)dimx * dimy * 2;
        const size_t row = (size_t)dimx * sizeof(float2), pitch = (size_t)c.P * sizeof(float2);
        of2d::DevArray<unsigned char> ws;
        ws.alloc(of2d::seqnorm_workspace_bytes(dimx, dimy));
        of2d::DevArray<float> out;
        out.alloc(2 * (size_t)npairs);
        // the walk's counters: the 8 of the ABI, then 2 more (tools)
        constexpr int kSnDbg = 10;
        of2d::DevArray<int> dbg;
        dbg.alloc(kSnDbg * (size_t)npairs);
        for (int k = 0; k < npairs; k++) {
            // one workspace: each pair's walk predicts the next (its profile)
            OF2D_HIP(hipMemcpy2D(c.p, pitch, cur + k * n, row, row, dimy, hipMemcpyHostToDevice));
            OF2D_HIP(hipMemcpy2D(p.p, pitch, prev + k * n, row, row, dimy, hipMemcpyHostToDevice));
            of2d::launch_seqnorm(c.p, p.p, dimx, dimy, c.P, ws.p, k > 0, out.p + 2 * k,
                                 dbg.p + kSnDbg * k, nullptr);
        }
        OF2D_HIP(hipMemcpy(sums, out.p, 2 * sizeof(float) * npairs, hipMemcpyDeviceToHost));
        if (stats)
            OF2D_HIP(hipMemcpy2D(stats, 8 * sizeof(int), dbg.p, kSnDbg * sizeof(int),
                                 8 * sizeof(int), npairs, hipMemcpyDeviceToHost));
    });
    if (rc != OF2D_OK) g_gateway_err = err;
    return rc;
}

int of2d_motion_norms_chain(const float *u, int dimx, int dimy, int niter, int batch,
                            float *sums, int *stats) {
    if (!u || !sums || dimx <= 0 || dimy <= 0 || niter <= 0 || batch < 1 || batch > 3)
        return OF2D_ERR_INVALID_ARGUMENT;
    std::string err;
    int rc = guarded(err, [&] {
        const size_t n = (size_t)dimx * dimy * 2;
        std::vector<of2d::Field<float2>> f((size_t)niter + 1);
        for (size_t k = 0; k <= (size_t)niter; k++) {
            f[k].alloc(dimx, dimy);
            const size_t row = (size_t)dimx * sizeof(float2), pitch = (size_t)f[k].P * sizeof(float2);
            OF2D_HIP(hipMemcpy2D(f[k].p, pitch, u + k * n, row, row, dimy, hipMemcpyHostToDevice));
        }
        // four sets of three workspaces rotated per batch, as the registration
        // loops (Registration::kSeqSets): batch g's profile is batch g - 4's
        constexpr int kSets = 4;
        of2d::DevArray<unsigned char> ws[3 * kSets];
        bool used[3 * kSets] = {};
        for (auto &w : ws) w.alloc(of2d::seqnorm_workspace_bytes(dimx, dimy));
        of2d::DevArray<float> out;
        out.alloc(2 * (size_t)niter);
        constexpr int kSnDbg = 10;
        of2d::DevArray<int> dbg;
        dbg.alloc(kSnDbg * (size_t)niter);
        for (int t = 0, g = 0; t < niter; g++) {
            of2d::SeqnormBatch B;
            B.K = std::min(batch, niter - t);
            for (int i = 0; i <= B.K; i++) B.u[i] = f[(size_t)t + i].p;
            for (int i = 0; i < B.K; i++) {
                const int w = 3 * (g % kSets) + i;
                B.ws[i] = ws[w].p;
                B.use_profile[i] = used[w];
                used[w] = true;
                B.out[i] = out.p + 2 * (size_t)(t + i);
                B.dbg[i] = dbg.p + kSnDbg * (size_t)(t + i);
            }
            of2d::launch_seqnorm_pass(B, dimx, dimy, f[0].P, nullptr);
            of2d::launch_seqnorm_refine(B, dimx, dimy, f[0].P, nullptr);
            of2d::launch_seqnorm_walk(B, dimx, dimy, f[0].P, nullptr);
            t += B.K;
        }
        OF2D_HIP(hipMemcpy(sums, out.p, 2 * sizeof(float) * niter, hipMemcpyDeviceToHost));
        if (stats)
            OF2D_HIP(hipMemcpy2D(stats, 8 * sizeof(int), dbg.p, kSnDbg * sizeof(int),
                                 8 * sizeof(int), niter, hipMemcpyDeviceToHost));
    });
    if (rc != OF2D_OK) g_gateway_err = err;
    return rc;
}

// ------------------------------------------------------------------ gateway
// static ImageRegistration *myImageRegistration (WrapperOpticalFlow2d.cpp:13)
static of2d_ctx *g_single = nullptr;
static int g_dimx = 0, g_dimy = 0;

size_t of2d_gateway_output_numel(int nlhs, int nrhs) {
    if (!g_single || nlhs != 1) return 0;
    if (nrhs == 0) return (size_t)g_dimx * g_dimy * 2;
    if (nrhs == 1) return (size_t)g_dimx * g_dimy;
    return 0;
}

int of2d_gateway_output_dims(int nlhs, int nrhs, size_t *dims, int *ndims) {
    if (!g_single || nlhs != 1 || (nrhs != 0 && nrhs != 1)) {
        if (ndims) *ndims = 0;
        return OF2D_ERR_STATE;
    }
    dims[0] = (size_t)g_dimx;  // dim_motion_mw / dim_image_mw (:74-78)
    dims[1] = (size_t)g_dimy;
    if (nrhs == 0) {
        dims[2] = 2;
        *ndims = 3;
    } else {
        *ndims = 2;
    }
    return OF2D_OK;
}

const char *of2d_gateway_last_error(void) { return g_gateway_err.c_str(); }

int of2d_gateway(int nlhs, double **plhs, int nrhs, const double *const *prhs) {
    // init (:23-83); a ninth input (this library's, not the reference's) is
    // the number of devices HS runs on (of2d_set_option "ngpus")
    if (nlhs == 0 && (nrhs == 8 || nrhs == 9) && g_single == nullptr) {
        const int dimx = (int)prhs[0][0], dimy = (int)prhs[0][1];
        const int nscales = (int)prhs[2][0];
        if (nscales < 0) {
            g_gateway_err = "Error: invalid number of scales\n";
            return OF2D_ERR_INVALID_ARGUMENT;
        }
        std::vector<int> niter(nscales + 1);
        for (int s = 0; s < nscales + 1; s++) niter[s] = (int)prhs[1][s];
        const int reg = (int)prhs[3][0];
        const unsigned nparams = (unsigned)prhs[5][0];
        std::vector<float> rp(nparams ? nparams : 1, 0.0f);
        for (unsigned p = 0; p < nparams; p++) rp[p] = (float)prhs[4][p];
        const int nrefine = (int)prhs[6][0];
        const int verbose = (int)prhs[7][0];
        of2d_ctx *c = nullptr;
        int rc = of2d_create(&c, dimx, dimy, niter.data(), nscales, reg, rp.data(), nparams,
                             nrefine, verbose);
        if (rc != OF2D_OK) return rc;  // message already in g_gateway_err
        if (nrhs == 9) {
            rc = of2d_set_option(c, "ngpus", prhs[8][0]);
            if (rc != OF2D_OK) {
                g_gateway_err = c->err;
                of2d_destroy(c);
                return rc;
            }
        }
        g_single = c;
        g_dimx = dimx;
        g_dimy = dimy;
        g_gateway_err.clear();
        return OF2D_OK;
    }
    // register (:86-102)
    if (nlhs == 0 && nrhs == 2 && g_single != nullptr) {
        int rc = of2d_set_images(g_single, prhs[0], prhs[1]);
        if (rc == OF2D_OK) rc = of2d_estimate(g_single);
        g_gateway_err = g_single->err;
        return rc;
    }
    // get motion (:105-117)
    if (nlhs == 1 && nrhs == 0 && g_single != nullptr) {
        int rc = of2d_get_motion(g_single, plhs[0]);
        g_gateway_err = g_single->err;
        return rc;
    }
    // warp (:120-137)
    if (nlhs == 1 && nrhs == 1 && g_single != nullptr) {
        int rc = of2d_warp(g_single, prhs[0], plhs[0]);
        g_gateway_err = g_single->err;
        return rc;
    }
    // close (:140-147)
    if (nlhs == 0 && nrhs == 0 && g_single != nullptr) {
        int rc = of2d_destroy(g_single);
        g_single = nullptr;
        g_dimx = g_dimy = 0;
        return rc;
    }
    g_gateway_err = "Error: invalid number of input and output variables gives.\n";
    return OF2D_ERR_STATE;
}

}  // extern "C"
