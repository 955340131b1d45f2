// conv3x3 forward on the 16-bit matrix cores (LDS-halo kernel, split-GEMM fallback): C ABI.  Kernels: conv_kernels.h.
#include "conv_kernels.h"

// conv3x3 forward on the 16-bit matrix cores in arithmetic nterm (split terms, see gemm_x3_kernel);
// wx = the split packed weights (cdm_split_bf16x3 / cdm_split_f16x2, same K order kc as cdm_pack_conv3x3).
static int conv3x3_fwd_split(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx, const float* amax_x,
                             const float* amax_w, const float* bias, float* y, int ldy, int Cout, int flags,
                             float* stats, int stats_ld, int kc, int nterm, float* amax_y, hipStream_t st,
                             const float* pre_s = nullptr, const float* pre_t = nullptr, int* ymm = nullptr,
                             int ymm_ld = 0, int dt = 0) {
    if (Cin % 4 || Cout % 4 || (kc != 0 && kc != 16) || (kc == 16 && Cin % 16)) return (int)hipErrorInvalidValue;
    const int M = N * H * W, K = 9 * Cin;
    MkPre mb{reinterpret_cast<const __bf16*>(wx), Cout, amax_w};
    EpiStore ep{y, ldy, 0, bias, Cout, flags, stats, stats_ld, M, Cout, amax_y};
    const bool halo = kc == 16 && W == H && halo_width_ok(W, nterm) && ldx % 4 == 0 && (H * W) % HBM_ == 0 &&
                      (unsigned long long)M * (unsigned)ldx * 4ull < (1ull << 32);   // 32-bit halo source offsets
    if ((pre_s || ymm) && (!halo || (ymm && !stats) || (pre_s && (!pre_t || Cin > 256))))
        return (int)hipErrorInvalidValue;      // the fused BN-ReLU input / max-min epilogue: LDS-halo path only
    if (dt && (!halo || nterm != 1)) return (int)hipErrorInvalidValue;   // bf16 activations: C4's LDS-halo path only
    if (halo) {   // LDS-halo path; dt bit 0: x (the BN-ReLU source) is bf16, bit 1: y is stored as bf16
        const HaloFwdArgs a{x, N, H, W, Cin, ldx, wx, amax_x, amax_w, bias, y, ldy, Cout, flags, stats, stats_ld, nterm,
                            amax_y, st, pre_s, pre_t, ymm, ymm_ld};
        return (dt & 3) ? halo_fwd_16(a, dt & 3) : halo_fwd_run<float, float>(a);
    }
    if (Cin == 128 && Cout == 128 && H == 64 && W == 64 && kc == 16) {
        using LA = LdIm2colA<128, 16, 64>;
        return launch_gemm_x3<RowK<LA>::template T, StagePre, EpiStore, true>(
            MkRowK<LA>{LA{x, H, W, Cin, ldx, M, K}, amax_x}, mb, ep, M, Cout, K, 1, nterm, st);
    }
    if (kc == 16) {
        using LA = LdIm2colA<0, 16>;
        return launch_gemm_x3<RowK<LA>::template T, StagePre, EpiStore, true>(
            MkRowK<LA>{LA{x, H, W, Cin, ldx, M, K}, amax_x}, mb, ep, M, Cout, K, 1, nterm, st);
    }
    using LA = LdIm2colA<0, 0>;
    return launch_gemm_x3<RowK<LA>::template T, StagePre, EpiStore, true>(
        MkRowK<LA>{LA{x, H, W, Cin, ldx, M, K}, amax_x}, mb, ep, M, Cout, K, 1, nterm, st);
}

// timing ablations of the h3 LDS-halo kernel (W = H = 64, kc = 16; tools/conv_ablation.py only)
CDM_API int cdm_conv3x3_halo_ablate(int abl, const float* x, int N, int H, int Cin, int ldx, const void* wx,
                                    const float* amax_x, const float* amax_w, float* y, int ldy, int Cout,
                                    void* stream) {
    if (H != 64 || Cin % 16 || ldx % 4) return (int)hipErrorInvalidValue;
    const int M = N * H * 64, mtiles = M / HBM_;
    if ((unsigned long long)M * (unsigned)ldx * 4ull >= (1ull << 32)) return (int)hipErrorInvalidValue;
    const int tpb = (abl >> 16) > 0 ? (abl >> 16) : 1;   // tiles per block in the high bits (0 -> 1)
    abl &= 0xffff;
    const EpiStoreW<4> eh{y, ldy, 0, nullptr, Cout, 0, nullptr, 0, M, Cout};
    const __bf16* b = reinterpret_cast<const __bf16*>(wx);
    dim3 grid((mtiles + tpb - 1) / tpb, (Cout + GBN - 1) / GBN, 1);
    hipStream_t s = S(stream);
#define CDM_ABL(A) hipLaunchKernelGGL((conv3x3_halo_x3_kernel<NT_H3, 64, EpiStoreW<4>, true, A>), grid, dim3(HTHREADS), 0, \
                                      s, x, H, Cin, ldx, b, Cout, amax_x, amax_w, eh, PreNone{}, mtiles, tpb)
    switch (abl) {
        case 0: CDM_ABL(0); break;
        case 1: CDM_ABL(1); break;
        case 2: CDM_ABL(2); break;
        case 4: CDM_ABL(4); break;
        case 8: CDM_ABL(8); break;
        case 12: CDM_ABL(12); break;
        case 14: CDM_ABL(14); break;
        case 16: CDM_ABL(16); break;
        case 32: CDM_ABL(32); break;
        case 17: CDM_ABL(17); break;
        case 3: CDM_ABL(3); break;
        case 5: CDM_ABL(5); break;
        case 9: CDM_ABL(9); break;
        case 13: CDM_ABL(13); break;
        case 21: CDM_ABL(21); break;
        case 25: CDM_ABL(25); break;
        case 29: CDM_ABL(29); break;
        case 33: CDM_ABL(33); break;
        case 45: CDM_ABL(45); break;
        case 16385: CDM_ABL(16385); break;
        case 16445: CDM_ABL(16445); break;
        case 60: CDM_ABL(60); break;
        case 61: CDM_ABL(61); break;
        case 62: CDM_ABL(62); break;
        case 65: CDM_ABL(65); break;
        case 129: CDM_ABL(129); break;
        case 257: CDM_ABL(257); break;
        case 513: CDM_ABL(513); break;
        case 769: CDM_ABL(769); break;
        case 1025: CDM_ABL(1025); break;
        default: return (int)hipErrorInvalidValue;
    }
#undef CDM_ABL
    return cdm_status();
}

CDM_API int cdm_conv3x3_fwd_x3(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx3,
                               const float* bias, float* y, int ldy, int Cout, int flags, float* stats, int stats_ld,
                               int kc, int nterm, void* stream) {
    if (nterm != 1 && nterm != 3 && nterm != 6) return (int)hipErrorInvalidValue;
    return conv3x3_fwd_split(x, N, H, W, Cin, ldx, wx3, nullptr, nullptr, bias, y, ldy, Cout, flags, stats, stats_ld, kc,
                             nterm, nullptr, S(stream));
}

CDM_API int cdm_conv3x3_fwd_x16(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx,
                                const float* amax_x, const float* amax_w, const float* bias, float* y, int ldy,
                                int Cout, int flags, float* stats, int stats_ld, int kc, float* amax_y, int nterm,
                                int dt, void* stream) {
    if (!x16_ok(nterm) || !x16_amax_ok(nterm, amax_x, amax_w)) return (int)hipErrorInvalidValue;
    return conv3x3_fwd_split(x, N, H, W, Cin, ldx, wx, amax_x, amax_w, bias, y, ldy, Cout, flags, stats, stats_ld, kc,
                             nterm, amax_y, S(stream), nullptr, nullptr, nullptr, 0, dt);
}
CDM_API int cdm_conv3x3_fwd_h3(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx, const float* amax_x,
                               const float* amax_w, const float* bias, float* y, int ldy, int Cout, int flags,
                               float* stats, int stats_ld, int kc, float* amax_y, void* stream) {
    return cdm_conv3x3_fwd_x16(x, N, H, W, Cin, ldx, wx, amax_x, amax_w, bias, y, ldy, Cout, flags, stats, stats_ld, kc,
                               amax_y, NT_H3, 0, stream);
}

// cdm_conv3x3_fwd_h3 + two fusions of the train-mode Conv -> BatchNorm -> ReLU chain (LDS-halo path only):
//   pre_s / pre_t (optional): the input is relu(x * pre_s[c] + pre_t[c]) of the previous layer's pre-norm output x
//                             (its BN apply runs in this conv's staging; *amax_x must bound that z)
//   ymm (optional, needs stats): per output channel max / min of y as ordered-int keys, ymm[c] / ymm[ymm_ld + c]
//                             (cleared by the caller to INT_MIN / INT_MAX), for the next layer's exact max|z|
CDM_API int cdm_conv3x3_fwd_x16_ex(const float* x, int N, int H, int W, int Cin, int ldx, const float* pre_s,
                                   const float* pre_t, const void* wx, const float* amax_x, const float* amax_w,
                                   const float* bias, float* y, int ldy, int Cout, int flags, float* stats,
                                   int stats_ld, int kc, float* amax_y, int* ymm, int ymm_ld, int nterm, int dt,
                                   void* stream) {
    if (!x16_ok(nterm) || !x16_amax_ok(nterm, amax_x, amax_w)) return (int)hipErrorInvalidValue;
    return conv3x3_fwd_split(x, N, H, W, Cin, ldx, wx, amax_x, amax_w, bias, y, ldy, Cout, flags, stats, stats_ld, kc,
                             nterm, amax_y, S(stream), pre_s, pre_t, ymm, ymm_ld, dt);
}
CDM_API int cdm_conv3x3_fwd_h3_ex(const float* x, int N, int H, int W, int Cin, int ldx, const float* pre_s,
                                  const float* pre_t, const void* wx, const float* amax_x, const float* amax_w,
                                  const float* bias, float* y, int ldy, int Cout, int flags, float* stats, int stats_ld,
                                  int kc, float* amax_y, int* ymm, int ymm_ld, void* stream) {
    return cdm_conv3x3_fwd_x16_ex(x, N, H, W, Cin, ldx, pre_s, pre_t, wx, amax_x, amax_w, bias, y, ldy, Cout, flags,
                                  stats, stats_ld, kc, amax_y, ymm, ymm_ld, NT_H3, 0, stream);
}
