// solvers.cpp — solver-specific buffers and iteration loops for the
// regularisations other than Horn-Schunck.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "of2d_host.h"
#include "of2d_solvers.h"

namespace of2d {
namespace solvers {

void alloc_level(Level &L, int reg) {
    (void)L;
    (void)reg;
}

int max_partial_blocks(const Level &L, int reg) {
    (void)reg;
    return hs_nblocks(L.P, L.dy);
}

}  // namespace solvers

int Registration::loop_demons(Level &, int, int &) {
    throw std::runtime_error("Thirion/Diffeomorphic Demons: not implemented yet");
}
int Registration::loop_fluid(Level &, int) {
    throw std::runtime_error("Fluid: not implemented yet");
}
int Registration::loop_elastic(Level &, int, int &) {
    throw std::runtime_error("Elastic: not implemented yet");
}
int Registration::loop_curvature(Level &, int, int &) {
    throw std::runtime_error("Curvature: not implemented yet");
}

}  // namespace of2d
