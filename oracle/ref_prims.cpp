// ORACLE PIN HARNESS — TEST INFRASTRUCTURE ONLY.
//
// Compiled by oracle/Makefile against the reference's own, self-contained
// source files where they lie under /root/reference (no copies, no stand-in
// headers):
//   src/coord2d.h   (value type, operator/ throw semantics)
//   src/gradients.h (partial_x / partial_y / qlaplacian templates)
//   src/Kernel.h, src/Kernel.cpp (Gaussian weights)
// Every other reference translation unit includes <mex.h> (src/Field.tpp:5),
// which this image lacks, so the whole MEX path is unbuildable here (see
// DESIGN.md "Oracle and parity pinning").  This harness exposes the buildable
// primitives through extern "C" so tests can compare oracle/of2d_oracle.c with
// them bit for bit.  The loops below only drive the reference templates over a
// field; they restate no arithmetic of their own except where marked
// "C++ semantics probe" (expressions evaluated with the reference's coord2d
// type so that C++ promotion rules, not our restatement, decide the rounding).
#include <src/coord2d.h>
#include <src/gradients.h>
#include <src/Kernel.h>

#include <cmath>
#include <cstring>
#include <stdexcept>

extern "C" {

int ref_gaussian(unsigned kw, float sigma, double *out) {
    Kernel k(kw);
    k.set_gaussian(sigma);
    std::memcpy(out, k.get_kernel(), sizeof(double) * kw * kw);
    return 0;
}

// gradients::partial_x / partial_y over an Image (T = float)
void ref_spatial_derivative(float *I, unsigned dimx, unsigned dimy, float *dI) {
    dim d(dimx, dimy);
    for (unsigned j = 0; j < dimy; j++)
        for (unsigned i = 0; i < dimx; i++) {
            unsigned idx = i + j * dimx;
            dI[2 * idx + 0] = gradients::partial_x(I, idx, i, d);
            dI[2 * idx + 1] = gradients::partial_y(I, idx, j, d);
        }
}

// gradients::partial_x / partial_y over a Motion (T = vector2d)
void ref_motion_partials(float *u, unsigned dimx, unsigned dimy, float *dudx, float *dudy) {
    dim d(dimx, dimy);
    vector2d *U = reinterpret_cast<vector2d *>(u);
    for (unsigned j = 0; j < dimy; j++)
        for (unsigned i = 0; i < dimx; i++) {
            unsigned idx = i + j * dimx;
            vector2d a = gradients::partial_x(U, idx, i, d);
            vector2d b = gradients::partial_y(U, idx, j, d);
            dudx[2 * idx] = a.x;
            dudx[2 * idx + 1] = a.y;
            dudy[2 * idx] = b.x;
            dudy[2 * idx + 1] = b.y;
        }
}

// gradients::qlaplacian over a Motion
void ref_qlaplacian(float *u, unsigned dimx, unsigned dimy, float *q) {
    dim d(dimx, dimy);
    vector2d *U = reinterpret_cast<vector2d *>(u);
    for (unsigned j = 0; j < dimy; j++)
        for (unsigned i = 0; i < dimx; i++) {
            unsigned idx = i + j * dimx;
            vector2d r = gradients::qlaplacian(U, idx, i, j, d);
            q[2 * idx] = r.x;
            q[2 * idx + 1] = r.y;
        }
}

// coord2d<float>::operator/ — returns 1 when the reference throws
int ref_coord2d_div(float x, float y, float a, float *out) {
    try {
        vector2d r = vector2d(x, y) / a;
        out[0] = r.x;
        out[1] = r.y;
        return 0;
    } catch (const std::runtime_error &) {
        return 1;
    }
}

// C++ semantics probe: the per-pixel HS update expression
// (OpticalFlow.cpp:33 then OpticalFlowDiffusion.cpp:78) evaluated with the
// reference's coord2d type on a precomputed quasi-Laplacian q.
int ref_hs_pointwise(const float *q, const float *dI, const float *It, unsigned n, float alpha,
                     float *u) {
    const vector2d *Q = reinterpret_cast<const vector2d *>(q);
    const vector2d *D = reinterpret_cast<const vector2d *>(dI);
    vector2d *U = reinterpret_cast<vector2d *>(u);
    const float alphasq = alpha * alpha;
    try {
        for (unsigned idx = 0; idx < n; idx++) {
            vector2d dIv = D[idx];
            vector2d f = dIv * (It[idx] + Q[idx].x * D[idx].x + Q[idx].y * D[idx].y);
            vector2d qv = Q[idx];
            U[idx] = qv - f / (alphasq + D[idx].x * D[idx].x + D[idx].y * D[idx].y);
        }
    } catch (const std::runtime_error &) {
        return 1;
    }
    return 0;
}

// C++ semantics probe: Motion::norm's accumulation (Motion.cpp:43-47) —
// std::pow(float, int) in C++17.
float ref_norm_probe(const float *u, unsigned n) {
    const vector2d *U = reinterpret_cast<const vector2d *>(u);
    float norm = 0.0f;
    for (unsigned i = 0; i < n; i++) norm += std::sqrt(std::pow(U[i].x, 2) + std::pow(U[i].y, 2));
    return norm / n;
}

// C++ semantics probe: Motion::maxabs (Motion.cpp:52-57)
float ref_maxabs_probe(const float *u, unsigned n) {
    const vector2d *U = reinterpret_cast<const vector2d *>(u);
    float maxabs = 0.0f;
    for (unsigned i = 0; i < n; i++) {
        float normsq = std::pow(U[i].y, 2) + std::pow(U[i].y, 2);
        maxabs = std::max(maxabs, normsq);
    }
    return std::sqrt(maxabs);
}

}  // extern "C"
