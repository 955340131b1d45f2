// The LDS-halo forward with bf16 activations (C4's fused Conv -> BN -> ReLU chain): its own compiler job.
#include "conv_kernels.h"

int halo_fwd_16(const HaloFwdArgs& a, int dt) {
    switch (dt) {
        case 1: return halo_fwd_run<__bf16, float>(a);
        case 2: return halo_fwd_run<float, __bf16>(a);
        case 3: return halo_fwd_run<__bf16, __bf16>(a);
        default: return (int)hipErrorInvalidValue;
    }
}
