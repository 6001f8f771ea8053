// mex_driver.cpp — plays MATLAB for tests: implements tests/stub/mex.h and
// calls the adapter's mexFunction (opticalflow2d_amd/mex/OpticalFlow2dMex.cpp)
// the way the interpreter does for `OpticalFlow2d(...)`: it wraps every input
// in an mxArray, passes nlhs/nrhs, owns plhs[0] afterwards, and turns
// mexErrMsgTxt into an error result.  ctypes entry points: mexdrv_*.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "mex.h"

namespace {
std::string g_err, g_out;
}

double *mxGetPr(const mxArray *a) { return const_cast<double *>(a->data.data()); }

mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity cx) {
    if (cls != mxDOUBLE_CLASS || cx != mxREAL) throw std::invalid_argument("stub: real double only");
    auto *a = new mxArray();
    size_t n = 1;
    for (mwSize k = 0; k < ndim; k++) {
        a->dims.push_back(dims[k]);
        n *= dims[k];
    }
    a->data.assign(n, 0.0);
    return a;
}

void mexErrMsgTxt(const char *msg) { throw mex_error(msg); }

int mexPrintf(const char *fmt, ...) {
    char buf[4096];
    va_list ap;
    va_start(ap, fmt);
    int n = vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_out += buf;
    return n;
}

extern "C" {

// OpticalFlow2d(in{0..nrhs-1}) with nlhs outputs.  Input k is a column-major
// double array of in_numel[k] values (shape is irrelevant to the gateway: it
// reads mxGetPr only, like WrapperOpticalFlow2d.cpp).  On success returns 0
// and, for nlhs == 1, copies plhs[0] (up to out_cap values) into out and its
// dims into out_dims / out_ndims.  mexErrMsgTxt -> returns 1 (message in
// mexdrv_last_error).
int mexdrv_call(int nlhs, int nrhs, const double *const *in, const size_t *in_numel, double *out,
                size_t out_cap, size_t *out_dims, int *out_ndims) {
    std::vector<std::unique_ptr<mxArray>> prhs_own;
    std::vector<const mxArray *> prhs;
    for (int k = 0; k < nrhs; k++) {
        auto a = std::make_unique<mxArray>();
        a->dims = {in_numel[k], 1};
        a->data.assign(in[k], in[k] + in_numel[k]);
        prhs.push_back(a.get());
        prhs_own.push_back(std::move(a));
    }
    mxArray *plhs[1] = {nullptr};
    g_err.clear();
    int rc = 0;
    try {
        mexFunction(nlhs, plhs, nrhs, prhs.empty() ? nullptr : prhs.data());
    } catch (const mex_error &e) {
        g_err = e.what();
        rc = 1;
    } catch (const std::exception &e) {  // would be a crash in MATLAB
        g_err = std::string("uncaught C++ exception: ") + e.what();
        rc = 2;
    }
    std::unique_ptr<mxArray> res(plhs[0]);
    if (out_ndims) *out_ndims = 0;
    if (res) {
        if (out_ndims) *out_ndims = (int)res->dims.size();
        for (size_t k = 0; k < res->dims.size() && out_dims && k < 3; k++) out_dims[k] = res->dims[k];
        if (out) std::memcpy(out, res->data.data(), sizeof(double) * std::min(out_cap, res->data.size()));
    }
    return rc;
}

const char *mexdrv_last_error(void) { return g_err.c_str(); }
const char *mexdrv_printed(void) { return g_out.c_str(); }
void mexdrv_clear_printed(void) { g_out.clear(); }

}  // extern "C"
