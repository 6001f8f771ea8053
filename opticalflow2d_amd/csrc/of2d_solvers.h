// of2d_solvers.h — per-regularisation device buffers and kernel launchers
// beyond Horn-Schunck (Demons, Fluid, Elastic, Curvature).
#pragma once

#include "of2d_host.h"

namespace of2d {
namespace solvers {

// allocate the solver-specific fields of a level (IterativeSolver / OpticalFlow /
// Demons / OpticalFlowFluid constructors)
void alloc_level(Level &L, int reg);
// largest number of per-block Logger partials one iteration writes at this level
int max_partial_blocks(const Level &L, int reg);

}  // namespace solvers
}  // namespace of2d
