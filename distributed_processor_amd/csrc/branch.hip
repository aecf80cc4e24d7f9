// branch.hip -- launches of branch_kernel (branch_kernel.h) for the STATE /
// READOUT measurement models; the DEMOD instantiations are compiled in
// branch_demod.hip (a separate translation unit, built in parallel).
#include "branch_kernel.h"

namespace dpemu {

hipError_t launch_branch_demod(const KParams &p, int feat, uint32_t blocks, hipStream_t stream);

hipError_t launch_branch(const KParams &p, int feat, hipStream_t stream)
{
    const uint32_t blocks = (uint32_t)((p.n_lanes + BLOCK - 1) / BLOCK);
    if (blocks == 0) return hipSuccess;
    if (feat & FEAT_DEMOD) return launch_branch_demod(p, feat, blocks, stream);
    switch (feat & (FEAT_FPROC | FEAT_LUT | FEAT_SYNC | FEAT_REGS | FEAT_PROG_LDS)) {
#define CASE(F) case F: return launch_branch_f<F>(p, blocks, stream);
#define CASES(L) CASE(L) CASE(L | FEAT_FPROC) CASE(L | FEAT_SYNC) CASE(L | FEAT_FPROC | FEAT_SYNC) \
                 CASE(L | FEAT_LUT) CASE(L | FEAT_LUT | FEAT_SYNC)
    CASES(0) CASES(FEAT_REGS) CASES(FEAT_PROG_LDS) CASES(FEAT_REGS | FEAT_PROG_LDS)
#undef CASES
#undef CASE
    }
    return hipErrorInvalidValue;
}

}  // namespace dpemu
