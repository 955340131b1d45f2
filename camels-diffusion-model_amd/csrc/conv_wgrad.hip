// conv3x3 weight gradient (kernel-row and transposed-read kernels, split-GEMM fallback): C ABI.  Kernels: conv_kernels.h.
#include "conv_kernels.h"

// the staggered wave order of the kernel-row weight gradient ($CDM_WGRAD_STAGGER, default 5 since round 6).  Round 3's
// form was slower (C2 train step 52.11-52.42 -> 52.88-53.05 ms, C4 32.26-32.52 -> 33.38-33.61 ms, profiles/
// r3_ab_wgrad_stagger.txt): the staging-first wave waited on the K step's loads it had just issued.  Round 6: that wave
// loads one K step further ahead — same-box A/B, 3 rounds, C2 48.10-48.16 -> 47.02-47.09 ms and C4 25.63-25.68 ->
// 25.24-25.27 ms per train step, slabs and sums bit-identical (profiles/r6_ab_wgrad_stagger_early.txt).  Bit 2 (default
// value 5 = 1 | 4): the MFMA-first half, too, loads the step after next once it has staged (before the barrier rather
// than after it): C2 46.75-46.77 -> 46.16-46.26 ms, C4 neutral (25.24-26.05 -> 25.44-25.71), bit-identical
// (profiles/r6_ab_wgrad_ahead.txt)
static int wgrad_ks4() {
    static const int v = [] { const char* e = getenv("CDM_WGRAD_KS4"); return e ? atoi(e) : 1; }();
    return v;
}
static int wgrad_ks1() {   // $CDM_WGRAD_KS1=1: 16-pixel K steps for the fp32-activation forms (A/B timing only)
    static const int v = [] { const char* e = getenv("CDM_WGRAD_KS1"); return e ? atoi(e) : 0; }();
    return v;
}
// 64-pixel K steps for h3 too, on the 64^2 layers ($CDM_WGRAD_KS4H3=0: 32): 133 KiB of LDS (gfx950 has 160 per CU) and
// 254 VGPRs without spills; same-box A/B after the schedule changes, 3 rounds: C2 44.94-45.11 -> 44.66-44.78 ms
// (profiles/r6_ab_wgrad_ks4h3.txt; 16-pixel steps: 45.70-45.77 -> 47.33-47.38, profiles/r6_ab_wgrad_ks1.txt)
static int wgrad_ks4h3() {
    static const int v = [] { const char* e = getenv("CDM_WGRAD_KS4H3"); return e ? atoi(e) : 1; }();
    return v;
}
static int wgrad_stagger() {
    static const int v = [] { const char* e = getenv("CDM_WGRAD_STAGGER"); return e ? atoi(e) : 5; }();
    return v;
}

// Two staging schedules of this kernel were measured and dropped (bit-identical outputs, same-box A/B,
// profiles/r3_ab_deep_staging.txt, r3_ab_wgrad_interleave.txt): the K step two ahead loaded into a second register set
// (BN coefficients moved to LDS to make room): C2 51.07-51.22 -> 51.87-52.01 ms per step, C4 neutral; the same with the
// next step's staging interleaved into the MFMAs' scheduling region (sched_group_barrier: 1 MFMA, 2 LDS reads, 5 VALU
// per gap): C2 49.78-49.91 -> 51.19-51.68 ms, C4 neutral.
template <int KS, class PRE = PreNone, class PX = PreNone, class GT = float, class XT = float>
static int launch_wgrad_row(const GT* dy, int lddy, int Cout, const XT* x, int H, int W, int Cin, int ldx, int K,
                            int sp, const float* amax_dy, const float* amax_x, float* slab, int nterm, hipStream_t st,
                            PRE pre = PRE{}, PX px = PX{}) {
    constexpr bool F32 = std::is_same<GT, float>::value && std::is_same<XT, float>::value;
    const int ktiles = K / (16 * KS), per = (ktiles + sp - 1) / sp;
    dim3 grid((Cout / 128) * 3 * (Cin / 128) * ((ktiles + per - 1) / per));
    if (!F32 && nterm != 1) return (int)hipErrorInvalidValue;   // bf16 activations: the one-term (C4) arithmetic only
    if constexpr (KS == 4) {   // 64-pixel K steps: the one-term bf16 images (66 KiB of LDS), or h3 ($CDM_WGRAD_KS4H3: 133 KiB)
        if constexpr (F32) {
            if (nterm == NT_H3) {
                hipLaunchKernelGGL((wgrad3x3_row_kernel<NT_H3, 4, PRE, PX>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H,
                                   W, Cin, ldx, ktiles, per, amax_dy, amax_x, slab, pre, px, wgrad_stagger());
                return cdm_status();
            }
        }
        if (nterm != 1) return (int)hipErrorInvalidValue;
        hipLaunchKernelGGL((wgrad3x3_row_kernel<1, 4, PRE, PX, GT, XT>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H, W,
                           Cin, ldx, ktiles, per, amax_dy, amax_x, slab, pre, px, wgrad_stagger());
        return cdm_status();
    } else {
    if constexpr (!F32) {
        hipLaunchKernelGGL((wgrad3x3_row_kernel<1, KS, PRE, PX, GT, XT>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H,
                           W, Cin, ldx, ktiles, per, amax_dy, amax_x, slab, pre, px, wgrad_stagger());
        return cdm_status();
    } else {
    if constexpr (PX::kind != 0) {            // the fused X transform: the 16-bit arithmetics (h3, bf16)
        if (nterm == NT_H3)
            hipLaunchKernelGGL((wgrad3x3_row_kernel<NT_H3, KS, PRE, PX>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H,
                               W, Cin, ldx, ktiles, per, amax_dy, amax_x, slab, pre, px, wgrad_stagger());
        else if (nterm == 1)
            hipLaunchKernelGGL((wgrad3x3_row_kernel<1, KS, PRE, PX>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H, W,
                               Cin, ldx, ktiles, per, amax_dy, amax_x, slab, pre, px, wgrad_stagger());
        else
            return (int)hipErrorInvalidValue;
        return cdm_status();
    }
    switch (nterm) {
        case 1: hipLaunchKernelGGL((wgrad3x3_row_kernel<1, KS, PRE>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H, W, Cin, ldx,
                                   ktiles, per, amax_dy, amax_x, slab, pre, PreNone{}, wgrad_stagger()); break;
        case 3: hipLaunchKernelGGL((wgrad3x3_row_kernel<3, KS, PRE>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H, W, Cin, ldx,
                                   ktiles, per, amax_dy, amax_x, slab, pre, PreNone{}, wgrad_stagger()); break;
        case NT_H3: hipLaunchKernelGGL((wgrad3x3_row_kernel<NT_H3, KS, PRE>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H, W,
                                       Cin, ldx, ktiles, per, amax_dy, amax_x, slab, pre, PreNone{}, wgrad_stagger()); break;
        case 6: hipLaunchKernelGGL((wgrad3x3_row_kernel<6, KS, PRE>), grid, dim3(512), 0, st, dy, lddy, Cout, x, H, W, Cin, ldx,
                                   ktiles, per, amax_dy, amax_x, slab, pre, PreNone{}, wgrad_stagger()); break;
        default: return (int)hipErrorInvalidValue;
    }
    return cdm_status();
    }
    }
}

// conv3x3 weight gradient on the 16-bit matrix cores (same slab contract as cdm_conv3x3_wgrad); W % 8 == 0
static int conv3x3_wgrad_split(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin,
                               int ldx, const float* amax_dy, const float* amax_x, int splits, float* slab, int nterm,
                               hipStream_t st, int variant = 0) {
    if (Cin % 4 || Cout % 4 || W % 8) return (int)hipErrorInvalidValue;
    const int M = Cout, NN = 9 * Cin, K = N * H * W;
    const int sp = effective_splits(K, splits);
    EpiStore ep{slab, NN, (long long)M * NN, nullptr, 1, 0, nullptr, 0, M, NN};
    const bool row_ok = Cin % 128 == 0 && Cout % 128 == 0 && lddy % 4 == 0 && ldx % 4 == 0;
    if ((variant == 0 || variant == 3) && row_ok) {   // kernel-row path (3 taps per block): KS = 2, else 1
        if (variant == 0 && W % 32 == 0 && effective_splits(K, splits, 32) == sp && !wgrad_ks1())
            return launch_wgrad_row<2>(dy, lddy, Cout, x, H, W, Cin, ldx, K, sp, amax_dy, amax_x, slab, nterm, st);
        if (W % 16 == 0 && effective_splits(K, splits, 16) == sp)
            return launch_wgrad_row<1>(dy, lddy, Cout, x, H, W, Cin, ldx, K, sp, amax_dy, amax_x, slab, nterm, st);
    }
    if (variant != 2 && Cin % 128 == 0 && Cout % 128 == 0 && W % 16 == 0 && lddy % 4 == 0 && ldx % 4 == 0 &&
        effective_splits(K, splits, 16) == sp) {   // transposed-read path
        const int ktiles = K / 16, per = (ktiles + sp - 1) / sp;
        dim3 grid((M / GBM) * (NN / GBN) * ((ktiles + per - 1) / per));
        switch (nterm) {
            case 1: hipLaunchKernelGGL(wgrad3x3_tr_x3_kernel<1>, grid, dim3(GTHREADS), 0, st, dy, lddy, Cout, x, H, W, Cin,
                                       ldx, K, per, amax_dy, amax_x, ep); break;
            case 3: hipLaunchKernelGGL(wgrad3x3_tr_x3_kernel<3>, grid, dim3(GTHREADS), 0, st, dy, lddy, Cout, x, H, W, Cin,
                                       ldx, K, per, amax_dy, amax_x, ep); break;
            case NT_H3: hipLaunchKernelGGL(wgrad3x3_tr_x3_kernel<NT_H3>, grid, dim3(GTHREADS), 0, st, dy, lddy, Cout, x, H,
                                           W, Cin, ldx, K, per, amax_dy, amax_x, ep); break;
            case 6: hipLaunchKernelGGL(wgrad3x3_tr_x3_kernel<6>, grid, dim3(GTHREADS), 0, st, dy, lddy, Cout, x, H, W, Cin,
                                       ldx, K, per, amax_dy, amax_x, ep); break;
            default: return (int)hipErrorInvalidValue;
        }
        return cdm_status();
    }
    return launch_gemm_x3<ColK<LdDenseAT>::template T, ColK<LdIm2colB>::template T, EpiStore, false>(
        MkColK<LdDenseAT>{LdDenseAT{dy, lddy, M, K}, amax_dy}, MkColK<LdIm2colB>{LdIm2colB{x, H, W, Cin, ldx, K, NN}, amax_x},
        ep, M, NN, K, sp, nterm, st);
}

CDM_API int cdm_conv3x3_wgrad_x3(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin,
                                 int ldx, int splits, float* slab, int nterm, void* stream) {
    if (nterm != 1 && nterm != 3 && nterm != 6) return (int)hipErrorInvalidValue;
    return conv3x3_wgrad_split(dy, lddy, Cout, x, N, H, W, Cin, ldx, nullptr, nullptr, splits, slab, nterm, S(stream));
}

CDM_API int cdm_conv3x3_wgrad_x16(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin,
                                  int ldx, const float* amax_dy, const float* amax_x, int splits, float* slab, int nterm,
                                  void* stream) {
    if (!x16_ok(nterm) || !x16_amax_ok(nterm, amax_dy, amax_x)) return (int)hipErrorInvalidValue;
    return conv3x3_wgrad_split(dy, lddy, Cout, x, N, H, W, Cin, ldx, amax_dy, amax_x, splits, slab, nterm, S(stream));
}
CDM_API int cdm_conv3x3_wgrad_h3(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin,
                                 int ldx, const float* amax_dy, const float* amax_x, int splits, float* slab,
                                 void* stream) {
    return cdm_conv3x3_wgrad_x16(dy, lddy, Cout, x, N, H, W, Cin, ldx, amax_dy, amax_x, splits, slab, NT_H3, stream);
}

// measurement entry: variant 0 = kernel-row kernel, 32-pixel K steps (default path), 1 = per-tap kernel,
// 2 = generic split GEMM, 3 = kernel-row kernel with 16-pixel K steps
CDM_API int cdm_conv3x3_wgrad_h3_variant(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W,
                                         int Cin, int ldx, const float* amax_dy, const float* amax_x, int splits,
                                         float* slab, int variant, void* stream) {
    if (!amax_dy || !amax_x || variant < 0 || variant > 3) return (int)hipErrorInvalidValue;
    return conv3x3_wgrad_split(dy, lddy, Cout, x, N, H, W, Cin, ldx, amax_dy, amax_x, splits, slab, NT_H3, S(stream),
                               variant);
}

// conv3x3 weight gradient of a Conv -> BatchNorm -> ReLU layer with the BN backward fused into the dY staging of
// the kernel-row kernel (same slab contract as cdm_conv3x3_wgrad_h3).  Cin % 128 == Cout % 128 == 0, W % 16 == 0.
CDM_API int cdm_conv3x3_wgrad_x16_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s,
                                        const float* t, const float* mean, const float* invstd, const float* A,
                                        const float* B, const float* Cc, int Cout, const float* x, int N, int H, int W,
                                        int Cin, int ldx, const float* amax_dy, const float* amax_x, int splits,
                                        float* slab, int nterm, int dt, void* stream) {
    if (!x16_ok(nterm) || Cin % 128 || Cout % 128 || W % 16 || ldg % 4 || ldy % 4 || ldx % 4 ||
        !x16_amax_ok(nterm, amax_dy, amax_x) || (dt && nterm != 1))
        return (int)hipErrorInvalidValue;
    const int K = N * H * W, sp = effective_splits(K, splits);
    const PreBnBwd pre{y, ldy, {s, t, mean, invstd, A, B, Cc}};
    // dt bit 0: g and y are bf16, bit 1: x is bf16
    auto run = [&](auto gtag, auto xtag) {
        using GT = decltype(gtag);
        using XT = decltype(xtag);
        const GT* gg = reinterpret_cast<const GT*>(g);
        const XT* xx = reinterpret_cast<const XT*>(x);
        if (W % 32 == 0 && effective_splits(K, splits, 32) == sp)
            return launch_wgrad_row<2>(gg, ldg, Cout, xx, H, W, Cin, ldx, K, sp, amax_dy, amax_x, slab, nterm, S(stream),
                                       pre);
        if (effective_splits(K, splits, 16) == sp)
            return launch_wgrad_row<1>(gg, ldg, Cout, xx, H, W, Cin, ldx, K, sp, amax_dy, amax_x, slab, nterm, S(stream),
                                       pre);
        return (int)hipErrorInvalidValue;
    };
    switch (dt & 3) {
        case 1: return run(__bf16{}, float{});
        case 2: return run(float{}, __bf16{});
        case 3: return run(__bf16{}, __bf16{});
        default: return run(float{}, float{});
    }
}
CDM_API int cdm_conv3x3_wgrad_h3_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s,
                                       const float* t, const float* mean, const float* invstd, const float* A,
                                       const float* B, const float* Cc, int Cout, const float* x, int N, int H, int W,
                                       int Cin, int ldx, const float* amax_dy, const float* amax_x, int splits,
                                       float* slab, void* stream) {
    return cdm_conv3x3_wgrad_x16_bnbwd(g, ldg, y, ldy, s, t, mean, invstd, A, B, Cc, Cout, x, N, H, W, Cin, ldx, amax_dy,
                                       amax_x, splits, slab, NT_H3, 0, stream);
}

// the kernel-row weight gradient with both staging fusions selectable: g / y / BN coefficients (optional, all or
// none: the dY operand is the BN backward of g, as cdm_conv3x3_wgrad_h3_bnbwd) and x_s / x_t (optional: the X operand
// is relu(x * x_s[c] + x_t[c]) of the previous layer's pre-norm output).  Cin % 128 == Cout % 128 == 0, W % 16 == 0.
CDM_API int cdm_conv3x3_wgrad_x16_ex(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                                     const float* mean, const float* invstd, const float* A, const float* B,
                                     const float* Cc, int Cout, const float* x, int N, int H, int W, int Cin, int ldx,
                                     const float* x_s, const float* x_t, const float* x_g, int ldxg,
                                     const float* x_mean, const float* x_invstd, float* x_sums,
                                     const float* amax_dy, const float* amax_x, int splits, float* slab, int nterm,
                                     int dt, void* stream) {
    if (!x16_ok(nterm) || Cin % 128 || Cout % 128 || W % 16 || ldg % 4 || ldx % 4 ||
        !x16_amax_ok(nterm, amax_dy, amax_x) || (x_s && !x_t) || (y && ldy % 4) ||
        (x_sums && (!x_s || !x_g || ldxg % 4 || !x_mean || !x_invstd)) || (dt && nterm != 1))
        return (int)hipErrorInvalidValue;
    const int K = N * H * W, sp = effective_splits(K, splits);
    const bool ks2 = W % 32 == 0 && effective_splits(K, splits, 32) == sp && !wgrad_ks1();
    // 64-pixel K steps for bf16 activations ($CDM_WGRAD_KS4=0: 32): with fp32 activations they measured 1.81x slower
    // per launch than 32 (1284 vs 710 us, 22 VGPRs spilled, profiles/r3_c4_ks4.txt); the bf16 staging registers are
    // half as wide (249 VGPRs, no spill): C4 29.64-29.89 -> 29.31-29.44 ms per step (profiles/r4_ab_dy_store_ks4.txt)
    const bool ks4 = wgrad_ks4() && W % 64 == 0 && effective_splits(K, splits, 64) == sp;
    const bool ks4h3 = nterm == NT_H3 && wgrad_ks4h3() && W % 64 == 0 && effective_splits(K, splits, 64) == sp;
    if (!ks2 && effective_splits(K, splits, 16) != sp) return (int)hipErrorInvalidValue;
    const PreBnBwd pre{y, ldy, {s, t, mean, invstd, A, B, Cc}};
    const PreBnRelu px{{x_s, x_t}};
    const PreBnReluSums pxs{{x_s, x_t}, x_g, ldxg, x_mean, x_invstd, x_sums};
    hipStream_t st = S(stream);
    // dt bit 0: g (and y) are bf16, bit 1: x (and x_g) are bf16
    auto run = [&](auto gtag, auto xtag) {
        using GT = decltype(gtag);
        using XT = decltype(xtag);
        const GT* gg = reinterpret_cast<const GT*>(g);
        const XT* xx = reinterpret_cast<const XT*>(x);
        constexpr bool BF = !(std::is_same<GT, float>::value && std::is_same<XT, float>::value);
#define CDM_WG(KS_, PRE_, PX_) launch_wgrad_row<KS_>(gg, ldg, Cout, xx, H, W, Cin, ldx, K, sp, amax_dy, amax_x, slab, \
                                                     nterm, st, PRE_, PX_)
        auto wgk = [&](auto pre_, auto px_) -> int {
            if constexpr (BF) {
                if (ks4) return CDM_WG(4, pre_, px_);
            } else {
                if (ks4h3) return CDM_WG(4, pre_, px_);
            }
            return ks2 ? CDM_WG(2, pre_, px_) : CDM_WG(1, pre_, px_);
        };
#define CDM_WGK(PRE_, PX_) wgk(PRE_, PX_)
        if (x_sums) {   // the producer's BN-backward sums ride along (x_sums[splits][5][Cin])
            if (y) return CDM_WGK(pre, pxs);
            return CDM_WGK(PreNone{}, pxs);
        }
        if (y && x_s) return CDM_WGK(pre, px);
        if (y) return CDM_WGK(pre, PreNone{});
        if (x_s) return CDM_WGK(PreNone{}, px);
        return CDM_WGK(PreNone{}, PreNone{});
#undef CDM_WGK
#undef CDM_WG
    };
    switch (dt & 3) {
        case 1: return run(__bf16{}, float{});
        case 2: return run(float{}, __bf16{});
        case 3: return run(__bf16{}, __bf16{});
        default: return run(float{}, float{});
    }
}
CDM_API int cdm_conv3x3_wgrad_h3_ex(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                                    const float* mean, const float* invstd, const float* A, const float* B,
                                    const float* Cc, int Cout, const float* x, int N, int H, int W, int Cin, int ldx,
                                    const float* x_s, const float* x_t, const float* amax_dy, const float* amax_x,
                                    int splits, float* slab, void* stream) {
    return cdm_conv3x3_wgrad_x16_ex(g, ldg, y, ldy, s, t, mean, invstd, A, B, Cc, Cout, x, N, H, W, Cin, ldx, x_s, x_t,
                                    nullptr, 0, nullptr, nullptr, nullptr, amax_dy, amax_x, splits, slab, NT_H3, 0, stream);
}
