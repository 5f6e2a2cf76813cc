// heat2d_amd — device-side collectives of the engine that are not part of the stencil launch
// interface (kernels.h): kept in their own header so that changing them rebuilds only the engine
// and kernels.hip, not the 44 stencil translation units.
#pragma once

#include "kernels.h"

namespace h2d {

// The IPC all-reduce of a fused convergence check (launch_ipc_allreduce) that first sums this
// rank's `nparts` per-wave residual partials in one fixed order (lane-strided, then the wave) into
// *local — the reduce kernel and the all-reduce kernel in ONE launch (one kernel boundary less per
// check on the direct pipeline).
void launch_ipc_allreduce_parts(const double* parts, int nparts, double* local, double* out, char* const* d_blocks,
                                int me, int nranks, int parity, unsigned long long target, size_t count_off,
                                size_t slot_off, int max_ranks, long long max_polls, unsigned int* timed_out,
                                unsigned int* timed_out_host, const unsigned long long* stop, const DecideArgs& decide,
                                hipStream_t s);

}  // namespace h2d
