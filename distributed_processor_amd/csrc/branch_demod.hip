// branch_demod.hip -- branch_kernel (branch_kernel.h) with the readout
// demodulation model (FEAT_DEMOD: meas_model DPEMU_MEAS_DEMOD, lane.h
// demod_readout), every program feature combination.
#include "branch_kernel.h"

namespace dpemu {

hipError_t launch_branch_demod(const KParams &p, int feat, uint32_t blocks, hipStream_t stream)
{
    switch (feat & (FEAT_FPROC | FEAT_LUT | FEAT_SYNC | FEAT_REGS | FEAT_PROG_LDS | FEAT_DEMOD)) {
#define CASE(F) case F: return launch_branch_f<F>(p, blocks, stream);
#define CASES(L) CASE(L) CASE(L | FEAT_FPROC) CASE(L | FEAT_SYNC) CASE(L | FEAT_FPROC | FEAT_SYNC) \
                 CASE(L | FEAT_LUT) CASE(L | FEAT_LUT | FEAT_SYNC)
    CASES(FEAT_DEMOD) CASES(FEAT_DEMOD | FEAT_REGS) CASES(FEAT_DEMOD | FEAT_PROG_LDS)
    CASES(FEAT_DEMOD | FEAT_REGS | FEAT_PROG_LDS)
#undef CASES
#undef CASE
    }
    return hipErrorInvalidValue;
}

}  // namespace dpemu
