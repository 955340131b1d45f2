// up0 of ContextUnet on large maps (ContextUnet.py:26-27: ConvTranspose2d(2nf, 2nf, h/4, h/4) on the 1x1 to_vec map;
// config 5 at 256x256: kernel 64x64, 2nf = 512 -> 1.07 G weights = 4.3 GB fp32).  With B <= 16 rows the layer is a
// skinny GEMM bound by one read (forward) / one write (weight gradient) of the weight tensor, so it runs as VALU fp32
// FMA kernels over the weights in the reference layout W[ci][co][kh][kw] (no per-step repack of 4.3 GB):
//   forward      y[n][ij][co]  = b[co] + sum_ci x[n][ci] W[ci][co][ij]        (y NHWC, ij = kh*k + kw)
//   weight grad  dW[ci][co][ij] = sum_n x[n][ci] dy[n][ij][co]
// Summation in fp32 FMA, ci (forward) / n (weight grad) ascending.
// Forward block: 256 threads = 16 output channels (co) x 16 quads of 4 consecutive ij (W read as float4 along ij, 256 B
// row pieces; 4.5 TB/s measured); weight-gradient block: 4 co x 64 quads (1 KB row pieces per wave store).  x^T [ci][16]
// sits in LDS and is read as broadcast float4.
#include "cdm_common.h"

namespace cdm {

constexpr int U0_NB = 16;     // rows (samples) per pass
constexpr int U0_CMAX = 512;  // channels (2 n_feat) held in LDS

static __device__ __forceinline__ void u0_stage_x(const float* __restrict__ x, int B, int C, int n0, float* xs) {
    for (int i = threadIdx.x; i < C * U0_NB; i += blockDim.x) {
        const int ci = i / U0_NB, n = i - ci * U0_NB;
        xs[i] = n0 + n < B ? x[(long long)(n0 + n) * C + ci] : 0.f;
    }
}

// grid (KK / 64, C / 16); every pass of 16 samples re-reads W (B > 16: config-5 CFG sampling, 2 passes)
__global__ __launch_bounds__(256) void up0_fwd_kernel(const float* __restrict__ x, int B, int C,
                                                      const float* __restrict__ W, int KK,
                                                      const float* __restrict__ bias, float* __restrict__ y) {
    __shared__ __attribute__((aligned(16))) float xs[U0_CMAX * U0_NB];
    __shared__ float tile[64 * 17];                 // [ij][co] of one sample (+1 pad)
    const int tid = threadIdx.x, q = tid & 15, cl = tid >> 4;
    const int co0 = blockIdx.y * 16, co = co0 + cl, ij0 = blockIdx.x * 64;
    const float* wp = W + (long long)co * KK + ij0 + q * 4;
    const long long ws = (long long)C * KK;
    const float bco = bias ? bias[co] : 0.f;
    for (int n0 = 0; n0 < B; n0 += U0_NB) {
        __syncthreads();
        u0_stage_x(x, B, C, n0, xs);
        __syncthreads();
        float acc[U0_NB][4];
#pragma unroll
        for (int n = 0; n < U0_NB; ++n)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[n][k] = 0.f;
#pragma unroll 4
        for (int ci = 0; ci < C; ++ci) {
            const float4 w4 = ld4(wp + ci * ws);
            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int n4 = 0; n4 < U0_NB / 4; ++n4) {
                const float4 xv = *reinterpret_cast<const float4*>(xs + ci * U0_NB + n4 * 4);
                const float xe[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[n4 * 4 + e][k] = fmaf(xe[e], wv[k], acc[n4 * 4 + e][k]);
            }
        }
        // per sample: [64 ij][16 co] through LDS, stored as 64-byte channel runs of y (NHWC)
        const int r = tid >> 2, c4 = (tid & 3) * 4;
#pragma unroll
        for (int n = 0; n < U0_NB; ++n) {
            if (n0 + n >= B) break;   // uniform
#pragma unroll
            for (int k = 0; k < 4; ++k) tile[(q * 4 + k) * 17 + cl] = acc[n][k] + bco;
            __syncthreads();
            const float4 v = make_float4(tile[r * 17 + c4], tile[r * 17 + c4 + 1], tile[r * 17 + c4 + 2],
                                         tile[r * 17 + c4 + 3]);
            st4(y + ((long long)(n0 + n) * KK + ij0 + r) * C + co0 + c4, v);
            __syncthreads();
        }
    }
}

// grid (KK / 256, C / 4); one pass over the samples (B <= 16): dy of the block's [16 n][256 ij][4 co] tile in registers,
// then one float4 of dW per ci and thread — a wave writes 1 KB of one dW row per ci (16 co x 64 ij blocks, 256 B row
// pieces, streamed the 4.3 GB out at 1.7 TB/s)
__global__ __launch_bounds__(256) void up0_wgrad_kernel(const float* __restrict__ x, int B, int C,
                                                        const float* __restrict__ dy, int KK, float* __restrict__ dW) {
    __shared__ __attribute__((aligned(16))) float xs[U0_CMAX * U0_NB];
    const int tid = threadIdx.x, q = tid & 63, cl = tid >> 6;
    const int co = blockIdx.y * 4 + cl, ij = blockIdx.x * 256 + q * 4;
    u0_stage_x(x, B, C, 0, xs);
    float d[U0_NB][4];
#pragma unroll
    for (int n = 0; n < U0_NB; ++n)
#pragma unroll
        for (int k = 0; k < 4; ++k) d[n][k] = n < B ? dy[((long long)n * KK + ij + k) * C + co] : 0.f;
    __syncthreads();
    float* op = dW + (long long)co * KK + ij;
    const long long ws = (long long)C * KK;
#pragma unroll 2
    for (int ci = 0; ci < C; ++ci) {
        float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int n4 = 0; n4 < U0_NB / 4; ++n4) {
            const float4 xv = *reinterpret_cast<const float4*>(xs + ci * U0_NB + n4 * 4);
            const float xe[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = fmaf(xe[e], d[n4 * 4 + e][k], o[k]);
        }
        st4(op + ci * ws, make_float4(o[0], o[1], o[2], o[3]));
    }
}

// input gradient: dx[n][ci] = sum_k dyT[n][k] W[ci][k], k = (co, ij) (dyT = dy transposed per sample to [n][co][ij]).
// Block: 64 ci x one K range of KR; thread = (ci group of 8: tid >> 5, k lane: tid & 31) owns acc[8 ci][16 n] over the
// k = k0 + 4 lane + 128 s of its range: per k step 8 float4 of W (each 32-lane half-wave reads 512 contiguous bytes of
// one W row) and the 16 n rows of dyT at the same k (shared by the 8 ci groups through L1), 512 FMAs.  W is read
// exactly once; the 32 k lanes fold through shuffles at the end; per-split partials slab[split][n < B][ci].
constexpr int U0D_KR = 32768;
__global__ __launch_bounds__(256, 2) void up0_dgrad_kernel(const float* __restrict__ dyT, int B, int C,
                                                           const float* __restrict__ W, long long K,
                                                           float* __restrict__ slab) {
    const int tid = threadIdx.x, kl = tid & 31, cg = tid >> 5;
    const int ci0 = blockIdx.x * 64 + cg * 8;
    const long long k0 = (long long)blockIdx.y * U0D_KR, k1 = min(K, k0 + U0D_KR);
    float acc[8][U0_NB];
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int n = 0; n < U0_NB; ++n) acc[c][n] = 0.f;
    for (long long k = k0 + kl * 4; k < k1; k += 128) {
        float4 w[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) w[c] = ld4(W + (long long)(ci0 + c) * K + k);
#pragma unroll
        for (int n = 0; n < U0_NB; ++n) {
            const float4 d = n < B ? ld4(dyT + (long long)n * K + k) : f4zero();
#pragma unroll
            for (int c = 0; c < 8; ++c)
                acc[c][n] = fmaf(d.w, w[c].w, fmaf(d.z, w[c].z, fmaf(d.y, w[c].y, fmaf(d.x, w[c].x, acc[c][n]))));
        }
    }
    // fold the 32 k lanes (lanes 0-31 and 32-63 of a wave are different ci groups)
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int n = 0; n < U0_NB; ++n) {
            float v = acc[c][n];
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
            acc[c][n] = v;
        }
    if (kl == 0) {
        float* out = slab + (long long)blockIdx.y * B * C;
#pragma unroll
        for (int n = 0; n < U0_NB; ++n) {
            if (n >= B) break;
#pragma unroll
            for (int c = 0; c < 8; ++c) out[n * C + ci0 + c] = acc[c][n];
        }
    }
}

static bool u0_shape_ok(int C, int KK) { return C % 16 == 0 && C <= U0_CMAX && KK % 64 == 0; }
static bool u0_wgrad_shape_ok(int C, int KK) { return C % 16 == 0 && C <= U0_CMAX && KK % 256 == 0; }

CDM_API int cdm_up0_fwd(const float* x, int B, int C, const float* W, int KK, const float* bias, float* y,
                        void* stream) {
    if (B < 1 || !u0_shape_ok(C, KK)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(up0_fwd_kernel, dim3(KK / 64, C / 16), dim3(256), 0, (hipStream_t)stream, x, B, C, W, KK, bias,
                       y);
    return cdm_status();
}

// slab [ceil(C*KK / 32768)][B][C] of per-K-range partials; cdm_slab_reduce folds them
CDM_API int cdm_up0_dgrad(const float* dyT, int B, int C, const float* W, int KK, float* slab, void* stream) {
    if (B < 1 || B > U0_NB || C % 64 || C > U0_CMAX || KK % 64) return (int)hipErrorInvalidValue;
    const long long K = (long long)C * KK;
    hipLaunchKernelGGL(up0_dgrad_kernel, dim3(C / 64, (unsigned)((K + U0D_KR - 1) / U0D_KR)), dim3(256), 0,
                       (hipStream_t)stream, dyT, B, C, W, K, slab);
    return cdm_status();
}
CDM_API int cdm_up0_dgrad_splits(int C, int KK) { return (int)(((long long)C * KK + U0D_KR - 1) / U0D_KR); }

CDM_API int cdm_up0_wgrad(const float* x, int B, int C, const float* dy, int KK, float* dW, void* stream) {
    if (B < 1 || B > U0_NB || !u0_wgrad_shape_ok(C, KK)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(up0_wgrad_kernel, dim3(KK / 256, C / 4), dim3(256), 0, (hipStream_t)stream, x, B, C, dy, KK,
                       dW);
    return cdm_status();
}

}  // namespace cdm
