// conv3x3 eval forward with the output transform fused into the LDS-halo conv's epilogue (its own compiler job):
// the residual shortcut add, FiLM, or MaxPool2d(2) of a Conv -> BatchNorm (folded) -> ReLU layer.  Kernels:
// conv_kernels.h (EpiStoreW<..., FUSE = true>).
#include "conv_kernels.h"

CDM_API int cdm_conv3x3_fwd_x16_fused(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx,
                                      const float* amax_x, const float* amax_w, const float* bias, float* y, int ldy,
                                      int Cout, int kc, float* amax_y, int kind, const float* sc_x, const float* sc_w,
                                      const float* sc_b, int split, const float* fa, int fan, const float* fb, int fbn,
                                      int nterm, void* stream) {
    const int M = N * H * W;
    if (!x16_ok(nterm) || !x16_amax_ok(nterm, amax_x, amax_w) || kc != 16 || W != H || (W != 32 && W != 64) ||
        Cin % 16 || Cout % 128 || ldx % 4 || (H * W) % HBM_ || (unsigned long long)M * (unsigned)ldx * 4ull >= (1ull << 32))
        return (int)hipErrorInvalidValue;
    if (kind == FUSE_RESID ? (!sc_x || !sc_w || !sc_b) : kind == FUSE_FILM ? (!fa || !fb) : kind != FUSE_POOL)
        return (int)hipErrorInvalidValue;
    EpiStoreW<4, float, false, true> e{y, ldy, 0, bias, Cout, EPI_RELU, nullptr, 0, M, Cout, amax_y};
    e.fz.kind = kind; e.fz.hw = H * W; e.fz.W = W;
    e.fz.x = sc_x; e.fz.w = sc_w; e.fz.b = sc_b; e.fz.split = split;
    e.fz.fa = fa; e.fz.fan = fan; e.fz.fb = fb; e.fz.fbn = fbn;
    return launch_conv_halo_w(W, x, N, H, Cin, ldx, reinterpret_cast<const __bf16*>(wx), Cout, amax_x, amax_w, e, nterm,
                              S(stream));
}
