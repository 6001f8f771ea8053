// OpticalFlow2dMex.cpp — the MEX entry point over libof2d.so.
//
// Drop-in replacement for the reference's WrapperOpticalFlow2d.cpp:18-155:
// same function name in MATLAB/Octave (OpticalFlow2d), same five call modes,
// same error strings.  All mode logic and the process-global singleton live in
// the library (of2d_gateway); this adapter only converts mxArray <-> double*.
// Build (needs a real MATLAB/Octave mex.h, not available in this image):
//   mkoctfile --mex -o OpticalFlow2d.mex OpticalFlow2dMex.cpp
//     -I<repo>/include -L<repo>/opticalflow2d_amd -lof2d   (one command line)
#include <mex.h>

#include <vector>

#include "of2d.h"

static void mex_print(const char *text, void *) { mexPrintf("%s", text); }

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
    static bool hooked = false;
    if (!hooked) {
        of2d_set_print_hook(mex_print, nullptr);
        hooked = true;
    }
    std::vector<const double *> in(nrhs > 0 ? nrhs : 1, nullptr);
    for (int k = 0; k < nrhs; k++) in[k] = mxGetPr(prhs[k]);
    double *out = nullptr;
    if (nlhs == 1) {
        size_t dims[3];
        int nd = 0;
        if (of2d_gateway_output_dims(nlhs, nrhs, dims, &nd) == OF2D_OK) {
            mwSize mdims[3] = {(mwSize)dims[0], (mwSize)dims[1], nd == 3 ? (mwSize)dims[2] : 1};
            plhs[0] = mxCreateNumericArray(nd, mdims, mxDOUBLE_CLASS, mxREAL);
            out = mxGetPr(plhs[0]);
        }
    }
    double *outs[1] = {out};
    if (of2d_gateway(nlhs, outs, nrhs, in.data()) != OF2D_OK)
        mexErrMsgTxt(of2d_gateway_last_error());
}
