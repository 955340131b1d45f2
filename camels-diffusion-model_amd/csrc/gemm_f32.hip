// Generic fp32 / split-16-bit GEMMs (up0, ConvT 2x2, Linear / conv fallbacks), weight splits and packs, operand
// maxima and slab reductions.  Kernel templates: conv_kernels.h.
#include "conv_kernels.h"

namespace cdm {

// b [K][N] fp32 (ld ldb)  ->  out [ceil(K/16)][3][N][16] bf16 split terms (k >= K zero-filled)
__global__ void split_bf16x3_kernel(const float* __restrict__ b, long long ldb, int K, int N, __bf16* __restrict__ out) {
    const int ktiles = (K + XBK - 1) / XBK;
    const long long total = (long long)ktiles * N * XBK;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long long)gridDim.x * blockDim.x) {
        const int kk = (int)(q % XBK); const long long r = q / XBK;
        const int n = (int)(r % N); const int kt = (int)(r / N);
        const int k = kt * XBK + kk;
        const float x = k < K ? b[(long long)k * ldb + n] : 0.f;
        const __bf16 h = (__bf16)x;
        const float r1 = x - (float)h;
        const __bf16 m = (__bf16)r1;
        const __bf16 l = (__bf16)(r1 - (float)m);
        __bf16* o = out + (((long long)kt * 3) * N + n) * XBK + kk;
        o[0] = h; o[(long long)N * XBK] = m; o[2LL * N * XBK] = l;
    }
}

// b [K][N] fp32 (ld ldb) -> out [ceil(K/16)][3][N][16]: fp16 hi / lo of b * s (planes 0, 1), s = op_scale(max|b|)
__global__ void split_f16x2_kernel(const float* __restrict__ b, long long ldb, int K, int N, const float* amax,
                                   __bf16* __restrict__ out) {
    const float sc = op_scale<NT_H3>(amax);
    const int ktiles = (K + XBK - 1) / XBK;
    const long long total = (long long)ktiles * N * XBK;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long long)gridDim.x * blockDim.x) {
        const int kk = (int)(q % XBK); const long long r = q / XBK;
        const int n = (int)(r % N); const int kt = (int)(r / N);
        const int k = kt * XBK + kk;
        const float v = (k < K ? b[(long long)k * ldb + n] : 0.f) * sc;
        const _Float16 h = (_Float16)v;
        __bf16* o = out + (((long long)kt * 3) * N + n) * XBK + kk;
        o[0] = __builtin_bit_cast(__bf16, h);
        o[(long long)N * XBK] = __builtin_bit_cast(__bf16, (_Float16)(v - (float)h));
    }
}

// ---- batched train-mode weight repack of every 3x3 conv (one amax launch + one pack-and-split launch per step
//      instead of ~7 small launches per layer): OIHW W -> the h3 split images the halo conv reads, directly ----
struct PackSplitJob {
    const float* W;          // OIHW [Cout][Cin][3][3]
    int Cin, Cout, kc;       // kc: K order (16 = channel-chunk-major, 0 = tap-major), as cdm_pack_conv3x3
    int mode;                // 0: the h3 split (fp16 hi / lo of W * 2^(14 - e)), 1: one bf16 term (C4; plane 0 only)
    __bf16* wpk_x;           // fwd operand  [ceil(9 Cin / 16)][3][Cout][16]  (K = tap/ci, N = co)
    __bf16* wdg_x;           // dgrad operand [ceil(9 Cout / 16)][3][Cin][16] (K = tap'/co, N = ci), W flipped
    float* amax;             // max|W| (the split scale of both images)
};
static __device__ __forceinline__ void unk(int k, int C, int kc, int& tap, int& c) {   // inverse of kidx
    if (kc <= 0) { tap = k / C; c = k - tap * C; return; }
    const int cc = k / (9 * kc), rem = k - cc * 9 * kc;
    tap = rem / kc; c = cc * kc + (rem - tap * kc);
}
__global__ __launch_bounds__(256) void pack_amax_batch_kernel(const PackSplitJob* __restrict__ jobs) {
    const PackSplitJob j = jobs[blockIdx.y];
    const long long total = (long long)j.Cout * j.Cin * 9;
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(j.W[i]));
    block_amax_commit(m, j.amax);
}
__global__ __launch_bounds__(256) void pack_split_batch_kernel(const PackSplitJob* __restrict__ jobs) {
    const PackSplitJob j = jobs[blockIdx.y >> 1];
    const bool dg = blockIdx.y & 1;
    __bf16* out = dg ? j.wdg_x : j.wpk_x;
    if (!out) return;
    const int K = 9 * (dg ? j.Cout : j.Cin), N = dg ? j.Cin : j.Cout;
    const bool one = j.mode == 1;
    const float sc = one ? 1.f : op_scale<NT_H3>(j.amax);
    const int ktiles = (K + XBK - 1) / XBK;
    const long long total = (long long)ktiles * N * XBK;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long long)gridDim.x * blockDim.x) {
        const int kk = (int)(q % XBK); const long long r = q / XBK;
        const int n = (int)(r % N); const int kt = (int)(r / N);
        const int k = kt * XBK + kk;
        float v = 0.f;
        if (k < K) {
            int tap, c;
            if (!dg) { unk(k, j.Cin, j.kc, tap, c); v = j.W[((long long)n * j.Cin + c) * 9 + tap]; }          // W[co=n][ci=c]
            else     { unk(k, j.Cout, j.kc, tap, c); v = j.W[((long long)c * j.Cin + n) * 9 + (8 - tap)]; }  // W[co=c][ci=n]
        }
        __bf16* o = out + (((long long)kt * 3) * N + n) * XBK + kk;
        if (one) {          // the hi plane of cdm_split_bf16x3 (the one-term arithmetic reads no other)
            o[0] = (__bf16)v;
            continue;
        }
        v *= sc;
        const _Float16 h = (_Float16)v;
        o[0] = __builtin_bit_cast(__bf16, h);
        o[(long long)N * XBK] = __builtin_bit_cast(__bf16, (_Float16)(v - (float)h));
    }
}

// out = max(out, max |x[r*ld + c]|) over r < rows, c < C  (atomic max on the float's bits; NaN ignored)
__global__ void amax_kernel(const float* __restrict__ x, long long rows, int C, long long ld, unsigned* out) {
    float m = 0.f;
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (C % 4 == 0 && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        const int C4 = C / 4;
        const long long total = rows * C4;
        for (long long q = t0; q < total; q += stride) {
            const long long r = q / C4; const int c = (int)(q - r * C4) * 4;
            const float4 v = *reinterpret_cast<const float4*>(x + r * ld + c);
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
    } else {
        const long long total = rows * C;
        for (long long q = t0; q < total; q += stride) {
            const long long r = q / C; const int c = (int)(q - r * C);
            m = fmaxf(m, fabsf(x[r * ld + c]));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    __shared__ float wm[8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wm[w] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, wm[i]);
        atomicMax(out, __float_as_uint(m));
    }
}

// ============================== slab reduction / permutation ==============================
// out[m*s_m + (n / csplit)*s_hi + (n % csplit)*s_lo] (+)= sum_z slab[z][m][n]
__global__ void slab_reduce_kernel(const float* __restrict__ slab, int splits, int M, int N, float* out,
                                   long long s_m, long long s_hi, long long s_lo, int csplit, int accumulate,
                                   float scale) {
    const long long total = (long long)M * N;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        float v = 0.f;
        for (int z = 0; z < splits; ++z) v += slab[(long long)z * total + idx];
        v *= scale;
        const int m = (int)(idx / N), n = (int)(idx - (long long)m * N);
        const int hi = n / csplit, lo = n - hi * csplit;
        float* p = out + m * s_m + hi * s_hi + lo * s_lo;
        *p = accumulate ? *p + v : v;
    }
}

// the same reduction for N % 4 == 0: a block = 32 float4 columns x 8 split groups; each thread sums every 8th
// split of its 4 columns with two independent accumulators (memory-level parallelism), the 8 groups are folded
// through LDS in a fixed order (deterministic).  HBM-bound on the slab read (the scalar kernel above is bound by
// the latency of its serial split loop).
__global__ __launch_bounds__(256) void slab_reduce4_kernel(const float* __restrict__ slab, int splits, int M, int N,
                                                           float* out, long long s_m, long long s_hi, long long s_lo,
                                                           int csplit, int accumulate, float scale) {
    __shared__ float4 red[8][32];
    const long long total4 = (long long)M * N / 4;
    const int col = threadIdx.x & 31, zg = threadIdx.x >> 5;
    const long long i4 = (long long)blockIdx.x * 32 + col;
    float4 a0 = f4zero(), a1 = f4zero();
    if (i4 < total4) {
        const float4* p = reinterpret_cast<const float4*>(slab) + i4;
        int z = zg;
        for (; z + 8 < splits; z += 16) {
            const float4 u = p[(long long)z * total4], v = p[(long long)(z + 8) * total4];
            a0.x += u.x; a0.y += u.y; a0.z += u.z; a0.w += u.w;
            a1.x += v.x; a1.y += v.y; a1.z += v.z; a1.w += v.w;
        }
        if (z < splits) {
            const float4 u = p[(long long)z * total4];
            a0.x += u.x; a0.y += u.y; a0.z += u.z; a0.w += u.w;
        }
    }
    red[zg][col] = make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
    __syncthreads();
    if (zg == 0 && i4 < total4) {
        float4 v = red[0][col];
#pragma unroll
        for (int k = 1; k < 8; ++k) { const float4 u = red[k][col]; v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w; }
        const float vv[4] = {v.x * scale, v.y * scale, v.z * scale, v.w * scale};
        const long long idx = i4 * 4;
        const int m = (int)(idx / N), n0 = (int)(idx - (long long)m * N);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = n0 + e, hi = n / csplit, lo = n - hi * csplit;
            float* q = out + m * s_m + hi * s_hi + lo * s_lo;
            *q = accumulate ? *q + vv[e] : vv[e];
        }
    }
}

}  // namespace cdm

// ---------------------------------------------------------------------------------------------
// C ABI (declared in include/cdm_hip.h)
// ---------------------------------------------------------------------------------------------
template <int BK, int KC, bool XCD>
static int conv3x3_fwd_bk(const float* x, int N, int H, int W, int Cin, int ldx, const float* wpk, const float* bias,
                          float* y, int ldy, int Cout, int flags, float* stats, int stats_ld, hipStream_t st) {
    const int M = N * H * W, K = 9 * Cin;
    LdDenseB lb{wpk, Cout, K, Cout};
    EpiStore ep{y, ldy, 0, bias, Cout, flags, stats, stats_ld, M, Cout};
    if (Cin == 128 && Cout == 128 && H == 64 && W == 64) {   // the hot conv: own instantiation
        LdIm2colA<128, KC, 64> la{x, H, W, Cin, ldx, M, K};
        return launch_gemm<LdIm2colA<128, KC, 64>, LdDenseB, EpiStore, false, BK, XCD>(la, lb, ep, M, Cout, K, 1, st);
    }
    if (Cin == 128 && Cout == 128) {
        LdIm2colA<128, KC> la{x, H, W, Cin, ldx, M, K};
        return launch_gemm<LdIm2colA<128, KC>, LdDenseB, EpiStore, false, BK, XCD>(la, lb, ep, M, Cout, K, 1, st);
    }
    LdIm2colA<0, KC> la{x, H, W, Cin, ldx, M, K};
    return launch_gemm<LdIm2colA<0, KC>, LdDenseB, EpiStore, false, BK, XCD>(la, lb, ep, M, Cout, K, 1, st);
}

// kc = K order of the packed weights (cdm_pack_conv3x3): 16 = channel-chunk-major (needs Cin % 16 == 0),
// 0 = tap-major.  Both run with the XCD-aware M-tile remap.
CDM_API int cdm_conv3x3_fwd(const float* x, int N, int H, int W, int Cin, int ldx, const float* wpk,
                            const float* bias, float* y, int ldy, int Cout, int flags, float* stats, int stats_ld,
                            int kc, void* stream) {
    if (Cin % 4 || Cout % 4 || (kc != 0 && kc != 16) || (kc == 16 && Cin % 16)) return (int)hipErrorInvalidValue;
    if (kc == 16)
        return conv3x3_fwd_bk<16, 16, true>(x, N, H, W, Cin, ldx, wpk, bias, y, ldy, Cout, flags, stats, stats_ld,
                                            S(stream));
    return conv3x3_fwd_bk<16, 0, true>(x, N, H, W, Cin, ldx, wpk, bias, y, ldy, Cout, flags, stats, stats_ld,
                                       S(stream));
}

// tuning entry point: 0 = default (BK16, tap-major K), 1 = BK32, 2 = XCD remap,
// 3 = channel-chunk-major K (needs the kc=16 weight pack), 4 = 2 + 3
CDM_API int cdm_conv3x3_fwd_variant(int variant, const float* x, int N, int H, int W, int Cin, int ldx,
                                    const float* wpk, const float* bias, float* y, int ldy, int Cout, int flags,
                                    float* stats, int stats_ld, void* stream) {
    if (Cin % 4 || Cout % 4) return (int)hipErrorInvalidValue;
    hipStream_t st = S(stream);
    switch (variant) {
        case 1: return conv3x3_fwd_bk<32, 0, false>(x, N, H, W, Cin, ldx, wpk, bias, y, ldy, Cout, flags, stats, stats_ld, st);
        case 2: return conv3x3_fwd_bk<16, 0, true>(x, N, H, W, Cin, ldx, wpk, bias, y, ldy, Cout, flags, stats, stats_ld, st);
        case 3: if (Cin % 16) return (int)hipErrorInvalidValue;
                return conv3x3_fwd_bk<16, 16, false>(x, N, H, W, Cin, ldx, wpk, bias, y, ldy, Cout, flags, stats, stats_ld, st);
        case 4: if (Cin % 16) return (int)hipErrorInvalidValue;
                return conv3x3_fwd_bk<16, 16, true>(x, N, H, W, Cin, ldx, wpk, bias, y, ldy, Cout, flags, stats, stats_ld, st);
        default: return conv3x3_fwd_bk<16, 0, false>(x, N, H, W, Cin, ldx, wpk, bias, y, ldy, Cout, flags, stats, stats_ld, st);
    }
}

static int split_blocks(int K, int N) {
    const long long total = (long long)((K + XBK - 1) / XBK) * N * XBK;
    long long blocks = (total + 255) / 256;
    return (int)(blocks > 8192 ? 8192 : (blocks < 1 ? 1 : blocks));
}

CDM_API int cdm_split_bf16x3(const float* b, long long ldb, int K, int N, void* out, void* stream) {
    hipLaunchKernelGGL(split_bf16x3_kernel, dim3(split_blocks(K, N)), dim3(256), 0, S(stream), b, ldb, K, N,
                       reinterpret_cast<__bf16*>(out));
    return cdm_status();
}

CDM_API int cdm_split_f16x2(const float* b, long long ldb, int K, int N, const float* amax, void* out, void* stream) {
    if (!amax) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(split_f16x2_kernel, dim3(split_blocks(K, N)), dim3(256), 0, S(stream), b, ldb, K, N, amax,
                       reinterpret_cast<__bf16*>(out));
    return cdm_status();
}

// A kernel, not hipMemsetAsync: on this ROCm a memset captured into a hipGraph did not reliably clear its buffer on
// later replays (tools/graph_probe.py: a 192-float memset node replayed after the buffer was rewritten left
// garbage), which made replayed sampling steps inherit stale h3 operand maxima.  Every clear on a captured path
// goes through this kernel.
__global__ void fill_f32_kernel(float* p, long long n, float v) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}
static int fill_f32(float* p, long long n, float v, hipStream_t s) {
    if (n <= 0) return 0;
    long long blocks = (n + 255) / 256;
    blocks = blocks > 4096 ? 4096 : blocks;
    hipLaunchKernelGGL(fill_f32_kernel, dim3((int)blocks), dim3(256), 0, s, p, n, v);
    return cdm_status();
}
CDM_API int cdm_zero_f32(float* p, long long n, void* stream) { return fill_f32(p, n, 0.f, S(stream)); }

/* every 3x3 conv's train-mode weight images in two launches: max|W| per job (into job.amax, cleared first by the
   caller, e.g. cdm_zero_f32 over a slot array), then the h3 split images straight from OIHW W */
CDM_API int cdm_pack_split_conv3x3_batch(const void* jobs_dev, int njobs, long long max_w_elems, void* stream) {
    if (njobs <= 0 || njobs > 32768) return (int)hipErrorInvalidValue;
    const PackSplitJob* jobs = reinterpret_cast<const PackSplitJob*>(jobs_dev);
    long long bx = (max_w_elems + 255) / 256;
    bx = bx > 64 ? 64 : (bx < 1 ? 1 : bx);
    hipLaunchKernelGGL(pack_amax_batch_kernel, dim3((unsigned)bx, njobs), dim3(256), 0, S(stream), jobs);
    int e = cdm_status(); if (e) return e;
    long long sx = (max_w_elems * 3 / 2 + 255) / 256;       // split images pad K to 16: ~1 element per weight
    sx = sx > 256 ? 256 : (sx < 1 ? 1 : sx);
    hipLaunchKernelGGL(pack_split_batch_kernel, dim3((unsigned)sx, 2 * njobs), dim3(256), 0, S(stream), jobs);
    return cdm_status();
}

CDM_API int cdm_amax_f32(const float* x, long long rows, int C, long long ld, float* out, int accumulate,
                         void* stream) {
    if (rows < 0 || C < 0 || ld < C) return (int)hipErrorInvalidValue;
    if (!accumulate) {
        const int e = fill_f32(out, 1, 0.f, S(stream));
        if (e) return e;
    }
    const long long total = rows * (long long)C;
    if (total == 0) return 0;
    long long blocks = (total / 4 + 255) / 256;
    blocks = blocks > 2048 ? 2048 : (blocks < 1 ? 1 : blocks);
    hipLaunchKernelGGL(amax_kernel, dim3((int)blocks), dim3(256), 0, S(stream), x, rows, C, ld,
                       reinterpret_cast<unsigned*>(out));
    return cdm_status();
}

CDM_API int cdm_convT2x2_fwd(const float* x, int N, int H, int W, int Cin, int ldx, const float* wpk,
                             const float* bias, float* y, int ldy, int Cout, float* amax, void* stream) {
    if (Cin % 4 || Cout % 4) return (int)hipErrorInvalidValue;
    const int M = N * H * W, K = Cin, NN = 4 * Cout;
    LdDenseA la{x, ldx, M, K};
    LdDenseB lb{wpk, NN, K, NN};
    EpiConvT2x2 ep{y, ldy, bias, H, W, Cout, M, NN, amax};
    return launch_gemm<LdDenseA, LdDenseB, EpiConvT2x2, false>(la, lb, ep, M, NN, K, 1, S(stream));
}

// the same on the fp16 matrix cores (h3: scaled hi/lo split, see split_terms); wx = cdm_split_f16x2 of wpk
CDM_API int cdm_convT2x2_fwd_x16(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx,
                                 const float* amax_x, const float* amax_w, const float* bias, float* y, int ldy,
                                 int Cout, float* amax_y, int nterm, void* stream) {
    if (!x16_ok(nterm) || Cin % 4 || Cout % 4 || !x16_amax_ok(nterm, amax_x, amax_w)) return (int)hipErrorInvalidValue;
    const int M = N * H * W, K = Cin, NN = 4 * Cout;
    EpiConvT2x2 ep{y, ldy, bias, H, W, Cout, M, NN, amax_y};
    // the two-deep prefetch form where the shape allows ($CDM_CONVT_DEEP=0: gemm_x3, read per call for A/B tests)
    const char* dv = getenv("CDM_CONVT_DEEP");
    if ((!dv || atoi(dv) != 0) && M % GBM == 0 && NN % GBN == 0 && K % (2 * XBK) == 0 && ldx % 4 == 0 &&
        (nterm == NT_H3 || nterm == 1)) {
        const dim3 grid(M / GBM, NN / GBN);
        const __bf16* wb = reinterpret_cast<const __bf16*>(wx);
        // transposed accumulators + 16-byte scatter stores ($CDM_CONVT_TRO=1; needs 16-byte aligned output rows and
        // whole 8-column groups per sub-pixel): bit-identical but 213 -> 219 us per launch in the sampling step and C2
        // +0.15 ms (profiles/r6_ab_convT_tro.txt) — the dword-store epilogue was not store-issue bound; off
        static const int tro_env = [] { const char* e = getenv("CDM_CONVT_TRO"); return e ? atoi(e) : 0; }();
        const bool tro = tro_env && Cout % 8 == 0 && ldy % 4 == 0 && reinterpret_cast<uintptr_t>(y) % 16 == 0;
        if (tro) {
            const EpiConvT2x2T et{y, ldy, bias, H, W, Cout, M, NN, amax_y};
            if (nterm == NT_H3)
                hipLaunchKernelGGL((gemm_deep_kernel<NT_H3, DeepDenseA, EpiConvT2x2T, 3, true>), grid, dim3(GTHREADS), 0,
                                   S(stream), DeepDenseA{x, ldx}, wb, NN, amax_x, amax_w, et, K);
            else
                hipLaunchKernelGGL((gemm_deep_kernel<1, DeepDenseA, EpiConvT2x2T, 3, true>), grid, dim3(GTHREADS), 0,
                                   S(stream), DeepDenseA{x, ldx}, wb, NN, amax_x, amax_w, et, K);
            return cdm_status();
        }
        if (nterm == NT_H3)
            hipLaunchKernelGGL((gemm_deep_kernel<NT_H3, DeepDenseA, EpiConvT2x2, 3>), grid, dim3(GTHREADS), 0,
                               S(stream), DeepDenseA{x, ldx}, wb, NN, amax_x, amax_w, ep, K);
        else
            hipLaunchKernelGGL((gemm_deep_kernel<1, DeepDenseA, EpiConvT2x2, 3>), grid, dim3(GTHREADS), 0, S(stream),
                               DeepDenseA{x, ldx}, wb, NN, amax_x, amax_w, ep, K);
        return cdm_status();
    }
    return launch_gemm_x3<RowK<LdDenseA>::template T, StagePre, EpiConvT2x2, true>(
        MkRowK<LdDenseA>{LdDenseA{x, ldx, M, K}, amax_x}, MkPre{reinterpret_cast<const __bf16*>(wx), NN, amax_w}, ep,
        M, NN, K, 1, nterm, S(stream));
}
CDM_API int cdm_convT2x2_fwd_h3(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx,
                                const float* amax_x, const float* amax_w, const float* bias, float* y, int ldy,
                                int Cout, float* amax_y, void* stream) {
    return cdm_convT2x2_fwd_x16(x, N, H, W, Cin, ldx, wx, amax_x, amax_w, bias, y, ldy, Cout, amax_y, NT_H3, stream);
}

// dX[n,h,w,ci] (+)= sum_{ij,co} dY[n,2h+i,2w+j,co] * W[ci][co][ij];  H, W are the INPUT (small) grid
CDM_API int cdm_convT2x2_dgrad(const float* dy, int N, int H, int W, int Cout, int lddy, const float* wpkT,
                               float* dx, int lddx, int Cin, int flags, void* stream) {
    if (Cin % 4 || Cout % 4) return (int)hipErrorInvalidValue;
    const int M = N * H * W, K = 4 * Cout;
    LdConvT2x2GatherA la{dy, H, W, Cout, lddy, M, K};
    LdDenseB lb{wpkT, Cin, K, Cin};
    EpiStore ep{dx, lddx, 0, nullptr, 1, flags, nullptr, 0, M, Cin};
    return launch_gemm<LdConvT2x2GatherA, LdDenseB, EpiStore, false>(la, lb, ep, M, Cin, K, 1, S(stream));
}

// h3 ConvT 2x2 dgrad: A = gathered dY (k = (ij, co), max|dY| = *amax_dy), B = cdm_split_f16x2 of the packed
// wpkT [4 Cout][Cin] with max|W| = *amax_w
CDM_API int cdm_convT2x2_dgrad_x16(const float* dy, int N, int H, int W, int Cout, int lddy, const void* wx,
                                   const float* amax_dy, const float* amax_w, float* dx, int lddx, int Cin, int flags,
                                   int nterm, void* stream) {
    if (!x16_ok(nterm) || Cin % 4 || Cout % 4 || !x16_amax_ok(nterm, amax_dy, amax_w)) return (int)hipErrorInvalidValue;
    const int M = N * H * W, K = 4 * Cout;
    EpiStore ep{dx, lddx, 0, nullptr, 1, flags, nullptr, 0, M, Cin};
    // the two-deep prefetch form ($CDM_CONVT_DEEP=0: gemm_x3); a 16-k tile stays inside one sub-pixel (Cout % 16)
    const char* dv = getenv("CDM_CONVT_DEEP");
    if ((!dv || atoi(dv) != 0) && M % GBM == 0 && Cin % GBN == 0 && Cout % 16 == 0 && K % (2 * XBK) == 0 &&
        lddy % 4 == 0 && (nterm == NT_H3 || nterm == 1)) {
        const dim3 grid(M / GBM, Cin / GBN);
        const __bf16* wb = reinterpret_cast<const __bf16*>(wx);
        const DeepConvT2x2GatherA al{dy, H, W, Cout, lddy};
        // two resident blocks per CU ($CDM_CONVT_DGRAD_MINB=3: three): the 3-block form spills 36-50 VGPRs at its 168 cap;
        // 199 without spill at two — bit-identical, 219 -> 209 us (h3), 203 -> 161 us (bf16) per launch, same-box trace
        // A/B (profiles/r6_ab_convT_dgrad_minb.txt)
        static const int mb2 = [] { const char* e = getenv("CDM_CONVT_DGRAD_MINB"); return e ? atoi(e) != 3 : 1; }();
        if (mb2) {
            if (nterm == NT_H3)
                hipLaunchKernelGGL((gemm_deep_kernel<NT_H3, DeepConvT2x2GatherA, EpiStore, 2>), grid, dim3(GTHREADS), 0,
                                   S(stream), al, wb, Cin, amax_dy, amax_w, ep, K);
            else
                hipLaunchKernelGGL((gemm_deep_kernel<1, DeepConvT2x2GatherA, EpiStore, 2>), grid, dim3(GTHREADS), 0,
                                   S(stream), al, wb, Cin, amax_dy, amax_w, ep, K);
            return cdm_status();
        }
        if (nterm == NT_H3)
            hipLaunchKernelGGL((gemm_deep_kernel<NT_H3, DeepConvT2x2GatherA, EpiStore, 3>), grid, dim3(GTHREADS), 0,
                               S(stream), al, wb, Cin, amax_dy, amax_w, ep, K);
        else
            hipLaunchKernelGGL((gemm_deep_kernel<1, DeepConvT2x2GatherA, EpiStore, 3>), grid, dim3(GTHREADS), 0,
                               S(stream), al, wb, Cin, amax_dy, amax_w, ep, K);
        return cdm_status();
    }
    return launch_gemm_x3<RowK<LdConvT2x2GatherA>::template T, StagePre, EpiStore, true>(
        MkRowK<LdConvT2x2GatherA>{LdConvT2x2GatherA{dy, H, W, Cout, lddy, M, K}, amax_dy},
        MkPre{reinterpret_cast<const __bf16*>(wx), Cin, amax_w}, ep, M, Cin, K, 1, nterm, S(stream));
}
CDM_API int cdm_convT2x2_dgrad_h3(const float* dy, int N, int H, int W, int Cout, int lddy, const void* wx,
                                  const float* amax_dy, const float* amax_w, float* dx, int lddx, int Cin, int flags,
                                  void* stream) {
    return cdm_convT2x2_dgrad_x16(dy, N, H, W, Cout, lddy, wx, amax_dy, amax_w, dx, lddx, Cin, flags, NT_H3, stream);
}

// h3 ConvT 2x2 weight gradient (same slab contract as cdm_convT2x2_wgrad); W % 8 == 0
CDM_API int cdm_convT2x2_wgrad_x16(const float* x, int N, int H, int W, int Cin, int ldx, const float* dy, int Cout,
                                   int lddy, const float* amax_x, const float* amax_dy, int splits, float* slab,
                                   int nterm, void* stream) {
    if (!x16_ok(nterm) || Cin % 4 || Cout % 4 || W % 8 || !x16_amax_ok(nterm, amax_x, amax_dy))
        return (int)hipErrorInvalidValue;
    const int M = Cin, NN = 4 * Cout, K = N * H * W;
    const int sp = effective_splits(K, splits);
    EpiStore ep{slab, NN, (long long)M * NN, nullptr, 1, 0, nullptr, 0, M, NN};
    static const bool tr = [] { const char* e = getenv("CDM_CONVT_WGRAD_TR"); return !e || atoi(e) != 0; }();
    if (tr && Cin % 128 == 0 && Cout % 128 == 0 && W % 16 == 0 && ldx % 4 == 0 && lddy % 4 == 0 &&
        effective_splits(K, splits, 16) == sp) {
        // the transposed-read staging of the 3x3 weight gradient with the ConvT sub-pixel map ($CDM_CONVT_WGRAD_TR=0:
        // the generic GEMM below)
        const int ktiles = K / 16, per = (ktiles + sp - 1) / sp;
        dim3 grid((M / GBM) * (NN / GBN) * ((ktiles + per - 1) / per));
        if (nterm == NT_H3)
            hipLaunchKernelGGL((wgrad3x3_tr_x3_kernel<NT_H3, 1, true>), grid, dim3(GTHREADS), 0, S(stream), x, ldx, Cin,
                               dy, H, W, Cout, lddy, K, per, amax_x, amax_dy, ep);
        else
            hipLaunchKernelGGL((wgrad3x3_tr_x3_kernel<1, 1, true>), grid, dim3(GTHREADS), 0, S(stream), x, ldx, Cin, dy, H,
                               W, Cout, lddy, K, per, amax_x, amax_dy, ep);
        return cdm_status();
    }
    return launch_gemm_x3<ColK<LdDenseAT>::template T, ColK<LdConvT2x2GatherB>::template T, EpiStore, false>(
        MkColK<LdDenseAT>{LdDenseAT{x, ldx, M, K}, amax_x},
        MkColK<LdConvT2x2GatherB>{LdConvT2x2GatherB{dy, H, W, Cout, lddy, K, NN}, amax_dy}, ep, M, NN, K, sp, nterm,
        S(stream));
}
CDM_API int cdm_convT2x2_wgrad_h3(const float* x, int N, int H, int W, int Cin, int ldx, const float* dy, int Cout,
                                  int lddy, const float* amax_x, const float* amax_dy, int splits, float* slab,
                                  void* stream) {
    return cdm_convT2x2_wgrad_x16(x, N, H, W, Cin, ldx, dy, Cout, lddy, amax_x, amax_dy, splits, slab, NT_H3, stream);
}

// C[m][n] = A[m][k] . B[k][n] (+bias[n % bias_mod]).  splits > 1: writes raw partials to slab[z][M][N].
CDM_API int cdm_gemm_f32(const float* a, long long lda, int M, int K, const float* b, long long ldb, int N,
                         float* c, long long ldc, const float* bias, int bias_mod, int flags, int splits,
                         float* slab, void* stream) {
    if (K % 4 || N % 4) return (int)hipErrorInvalidValue;
    LdDenseA la{a, lda, M, K};
    LdDenseB lb{b, ldb, K, N};
    const int sp = effective_splits(K, splits);
    if (sp > 1) {
        EpiStore ep{slab, N, (long long)M * N, nullptr, 1, 0, nullptr, 0, M, N};
        return launch_gemm<LdDenseA, LdDenseB, EpiStore, false>(la, lb, ep, M, N, K, sp, S(stream));
    }
    EpiStore ep{c, ldc, 0, bias, bias_mod > 0 ? bias_mod : 1, flags, nullptr, 0, M, N};
    return launch_gemm<LdDenseA, LdDenseB, EpiStore, false>(la, lb, ep, M, N, K, 1, S(stream));
}

CDM_API int cdm_gemm_splits(int K, int splits) { return effective_splits(K, splits); }

// C[m][n] = A[m][k] . B[k][n] + bias[n % bias_mod] on the 16-bit matrix cores (nterm: NT_H3 or one bf16 term);
// wx = the split image of B (cdm_split_f16x2 / cdm_split_bf16x3 of [K][N]); h3: max|A| = *amax_a, max|B| = *amax_w.
// amax_c (optional): running max|C|.  up0's ConvTranspose2d(k = h/4) on the 1x1 map (ContextUnet.py:26-30).
CDM_API int cdm_gemm_x16(const float* a, long long lda, int M, int K, const void* wx, const float* amax_a,
                         const float* amax_w, int N, float* c, long long ldc, const float* bias, int bias_mod,
                         float* amax_c, int nterm, void* stream) {
    if (!x16_ok(nterm) || !x16_amax_ok(nterm, amax_a, amax_w) || K % 4 || N % 4 || lda % 4)
        return (int)hipErrorInvalidValue;
    EpiStore ep{c, ldc, 0, bias, bias_mod > 0 ? bias_mod : 1, 0, nullptr, 0, M, N, amax_c};
    return launch_gemm_x3<RowK<LdDenseA>::template T, StagePre, EpiStore, true>(
        MkRowK<LdDenseA>{LdDenseA{a, lda, M, K}, amax_a}, MkPre{reinterpret_cast<const __bf16*>(wx), N, amax_w}, ep, M,
        N, K, 1, nterm, S(stream));
}

// slab[z][co][tap*Cin+ci] = partial sum over a pixel range of dY[pix][co] * X[pix+tap][ci]
CDM_API int cdm_conv3x3_wgrad(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin,
                              int ldx, int splits, float* slab, void* stream) {
    if (Cin % 4 || Cout % 4) return (int)hipErrorInvalidValue;
    const int M = Cout, NN = 9 * Cin, K = N * H * W;
    LdDenseAT la{dy, lddy, M, K};
    LdIm2colB lb{x, H, W, Cin, ldx, K, NN};
    const int sp = effective_splits(K, splits);
    EpiStore ep{slab, NN, (long long)M * NN, nullptr, 1, 0, nullptr, 0, M, NN};
    return launch_gemm<LdDenseAT, LdIm2colB, EpiStore, true>(la, lb, ep, M, NN, K, sp, S(stream));
}

// slab[z][ci][ij*Cout+co] = partial over input pixels of X[pix][ci] * dY[n,2h+i,2w+j,co]
CDM_API int cdm_convT2x2_wgrad(const float* x, int N, int H, int W, int Cin, int ldx, const float* dy, int Cout,
                               int lddy, int splits, float* slab, void* stream) {
    if (Cin % 4 || Cout % 4) return (int)hipErrorInvalidValue;
    const int M = Cin, NN = 4 * Cout, K = N * H * W;
    LdDenseAT la{x, ldx, M, K};
    LdConvT2x2GatherB lb{dy, H, W, Cout, lddy, K, NN};
    const int sp = effective_splits(K, splits);
    EpiStore ep{slab, NN, (long long)M * NN, nullptr, 1, 0, nullptr, 0, M, NN};
    return launch_gemm<LdDenseAT, LdConvT2x2GatherB, EpiStore, true>(la, lb, ep, M, NN, K, sp, S(stream));
}

// slab[z][m][n] = partial over k of a[k][m] * b[k][n]   (A^T B; up0 / Linear weight gradients)
CDM_API int cdm_gemm_tn_f32(const float* a, long long lda, int M, int K, const float* b, long long ldb, int N,
                            int splits, float* slab, void* stream) {
    if (M % 4 || N % 4) return (int)hipErrorInvalidValue;
    LdDenseAT la{a, lda, M, K};
    LdDenseB lb{b, ldb, K, N};
    const int sp = effective_splits(K, splits);
    EpiStore ep{slab, N, (long long)M * N, nullptr, 1, 0, nullptr, 0, M, N};
    return launch_gemm<LdDenseAT, LdDenseB, EpiStore, true>(la, lb, ep, M, N, K, sp, S(stream));
}

CDM_API int cdm_slab_reduce(const float* slab, int splits, int M, int N, float* out, long long s_m, long long s_hi,
                            long long s_lo, int csplit, int accumulate, float scale, void* stream) {
    const long long total = (long long)M * N;
    if (N % 4 == 0 && splits >= 8) {
        const long long blocks4 = (total / 4 + 31) / 32;
        hipLaunchKernelGGL(slab_reduce4_kernel, dim3((unsigned)blocks4), dim3(256), 0, S(stream), slab, splits, M, N, out,
                           s_m, s_hi, s_lo, csplit > 0 ? csplit : N, accumulate, scale);
        return cdm_status();
    }
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(blocks), dim3(256), 0, S(stream), slab, splits, M, N, out, s_m, s_hi,
                       s_lo, csplit > 0 ? csplit : N, accumulate, scale);
    return cdm_status();
}