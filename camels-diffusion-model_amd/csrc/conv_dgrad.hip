// conv3x3 dgrad of a Conv -> BatchNorm -> ReLU layer, BN backward in the LDS-halo staging: C ABI.  Kernels: conv_kernels.h.
#include "conv_kernels.h"

// conv3x3 dgrad of a Conv -> BatchNorm -> ReLU layer with the BN backward fused into the halo staging: the conv
// input dy = bn_bwd_elem(g, y, coefficients) is computed per staged element (dy never materialised).  C = BN
// channels (the dgrad's input channels), Cout = the dgrad's output channels.  W == H in {32, 64, 128}, C % 16 == 0,
// C <= 256; wx = cdm_split_f16x2 of the kc = 16 packed dgrad weights; max|dy| <= *amax_dy (cdm_bn_bwd_amax_bound).
// dy_out (optional): the dy computed in the staging is also stored there ([pix][C] at g's row stride ldg, g's element
// type), for the layer's weight gradient (cdm_conv3x3_wgrad_x16_ex with dy = dy_out and no BN coefficients).
CDM_API int cdm_conv3x3_dgrad_x16_bnbwd_dy(const float* g, int ldg, const float* y, int ldy, const float* s,
                                           const float* t, const float* mean, const float* invstd, const float* A,
                                           const float* B, const float* Cc, int N, int H, int W, int C, const void* wx,
                                           const float* amax_dy, const float* amax_w, float* out, int ldo, int Cout,
                                           int flags, float* amax_out, void* dy_out, int nterm, int dt, void* stream) {
    if (!x16_ok(nterm) || W != H || !halo_width_ok(W, nterm) || W > 128 || C % 16 || C > 256 || ldg % 4 || ldy % 4 ||
        (H * W) % HBM_ || !x16_amax_ok(nterm, amax_dy, amax_w) || (dt && nterm != 1))
        return (int)hipErrorInvalidValue;
    const int M = N * H * W;
    PreBnBwd pre{y, ldy, {s, t, mean, invstd, A, B, Cc}};
    pre.dyo = dy_out;
    const __bf16* b = reinterpret_cast<const __bf16*>(wx);
    // dt bit 0: g and y are bf16, bit 1: the output (the producer's g) is stored as bf16
    auto run = [&](auto xtag, auto otag) {
        using XT = decltype(xtag);
        using OT = decltype(otag);
        if constexpr (std::is_same<OT, float>::value) {   // an accumulating dgrad: the load-ahead epilogue
            if ((flags & EPI_ACCUM) && W <= 64) {
                const EpiStoreW<4, float, true> ea{out, ldo, 0, nullptr, Cout, flags, nullptr, 0, M, Cout, amax_out};
                return launch_conv_halo_w(W, reinterpret_cast<const XT*>(g), N, H, C, ldg, b, Cout, amax_dy, amax_w, ea,
                                          nterm, S(stream), pre);
            }
        }
        const EpiStoreW<4, OT> eh{reinterpret_cast<OT*>(out), ldo, 0, nullptr, Cout, flags, nullptr, 0, M, Cout,
                                  amax_out};
        return launch_conv_halo_w(W, reinterpret_cast<const XT*>(g), N, H, C, ldg, b, Cout, amax_dy, amax_w, eh, nterm,
                                  S(stream), pre);
    };
    switch (dt & 3) {
        case 1: return run(__bf16{}, float{});
        case 2: return run(float{}, __bf16{});
        case 3: return run(__bf16{}, __bf16{});
        default: return run(float{}, float{});
    }
}
CDM_API int cdm_conv3x3_dgrad_x16_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s,
                                        const float* t, const float* mean, const float* invstd, const float* A,
                                        const float* B, const float* Cc, int N, int H, int W, int C, const void* wx,
                                        const float* amax_dy, const float* amax_w, float* out, int ldo, int Cout,
                                        int flags, float* amax_out, int nterm, int dt, void* stream) {
    return cdm_conv3x3_dgrad_x16_bnbwd_dy(g, ldg, y, ldy, s, t, mean, invstd, A, B, Cc, N, H, W, C, wx, amax_dy, amax_w,
                                          out, ldo, Cout, flags, amax_out, nullptr, nterm, dt, stream);
}
CDM_API int cdm_conv3x3_dgrad_h3_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s,
                                       const float* t, const float* mean, const float* invstd, const float* A,
                                       const float* B, const float* Cc, int N, int H, int W, int C, const void* wx,
                                       const float* amax_dy, const float* amax_w, float* out, int ldo, int Cout,
                                       int flags, float* amax_out, void* stream) {
    return cdm_conv3x3_dgrad_x16_bnbwd(g, ldg, y, ldy, s, t, mean, invstd, A, B, Cc, N, H, W, C, wx, amax_dy, amax_w,
                                       out, ldo, Cout, flags, amax_out, NT_H3, 0, stream);
}
