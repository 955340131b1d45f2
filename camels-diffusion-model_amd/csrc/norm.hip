// Normalisation, pooling and FiLM kernels (HBM-bound, float4 over channels, NHWC).
//
// Reference ops covered (diffusion_utilities.py / ContextUnet.py):
//   BatchNorm2d + ReLU            diffusion_utilities.py:28-29,35-36  (train: batch stats, eval: running stats)
//   random 1x1 shortcut + add     diffusion_utilities.py:54-55
//   MaxPool2d(2)                  diffusion_utilities.py:109
//   GroupNorm(8) + ReLU           ContextUnet.py:28-29,37-38
//   FiLM  cemb*h + temb           ContextUnet.py:57-58
//
// Statistics are produced as per-(image, chunk-of-pixels) partial sums in an fp32 "slab"
// [N][nchunks][R][C] (the conv epilogue writes the same layout with R = 2 and 128-pixel chunks),
// then folded in fp64 by a tiny finalize kernel.  Deterministic: no atomics anywhere.
#include "cdm_common.h"

#include <type_traits>

namespace cdm {

struct NormP {              // z_pre = y*s + t ; xhat = (y - mean)*invstd
    const float* s; const float* t; int sn;                  // index n*sn + c
    const float* mean; const float* invstd; int mn; int cpg;  // index n*mn + c/cpg
};
struct FilmP { const float* a; int an; const float* b; int bn; };  // out = a[n*an+c]*u + b[n*bn+c]
// + w[c]*x[n,p] + b[c] (C_in = 1), or + b[c] + sum_k w[c][k] x[n,p][k] over xc image channels (x pixel stride ldx)
struct ResidP { const float* x; const float* w; const float* b; int split; int xc = 1; int ldx = 1; };

// -------------------------------------------------------------------------------------------------
// generic per-(n,c) partial reduction over pixel chunks
// -------------------------------------------------------------------------------------------------
template <int R>
struct Acc4 { float4 v[R]; };

struct StatsF {  // R=2: sum, sum of squares
    static constexpr int R = 2;
    const float* y; int ldy; int HW;
    __device__ __forceinline__ void operator()(int n, int p, int c, Acc4<2>& a) const {
        const float4 v = ld4(y + ((long long)n * HW + p) * ldy + c);
        a.v[0].x += v.x; a.v[0].y += v.y; a.v[0].z += v.z; a.v[0].w += v.w;
        a.v[1].x += v.x * v.x; a.v[1].y += v.y * v.y; a.v[1].z += v.z * v.z; a.v[1].w += v.w * v.w;
    }
};

struct SumF {  // R=1: plain sum (bias gradients)
    static constexpr int R = 1;
    const float* g; int ldg; int HW;
    __device__ __forceinline__ void operator()(int n, int p, int c, Acc4<1>& a) const {
        const float4 v = ld4(g + ((long long)n * HW + p) * ldg + c);
        a.v[0].x += v.x; a.v[0].y += v.y; a.v[0].z += v.z; a.v[0].w += v.w;
    }
};

// Recompute one element's forward pieces.
static __device__ __forceinline__ void norm_elem(const NormP& np, int n, int c, float y, float& zpre, float& xhat) {
    zpre = fmaf(y, np.s[n * np.sn + c], np.t[n * np.sn + c]);
    const int gi = n * np.mn + c / np.cpg;
    xhat = (y - np.mean[gi]) * np.invstd[gi];
}

// R=5 backward sums for  out = [pool|film]( relu( norm(y) ) ):
//   S1 = sum g_pre, S2 = sum g_pre*xhat, S3 = sum g_out*u (FiLM), S4 = sum g_out (FiLM), S5 = sum xhat
template <bool POOL, bool FILM>
struct NormBwdF {
    static constexpr int R = 5;
    const float* g; int ldg;      // grad wrt the op output (pooled grid when POOL)
    const float* y; int ldy;      // pre-norm activations (full grid)
    int H, W;                     // full grid
    NormP np; FilmP fp;
    __device__ __forceinline__ void operator()(int n, int p, int c4, Acc4<5>& a) const {
        float* acc = reinterpret_cast<float*>(a.v);  // acc[r*4 + j]
        if constexpr (POOL) {
            const int Wo = W >> 1, ho = p / Wo, wo = p - ho * Wo;
            const float4 gv = ld4(g + ((long long)n * (H >> 1) * Wo + p) * ldg + c4);
            float4 yv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                yv[e] = ld4(y + ((long long)(n * H + 2 * ho + (e >> 1)) * W + 2 * wo + (e & 1)) * ldy + c4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c4 + j;
                float zp[4], xh[4], best = -INFINITY; int arg = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    norm_elem(np, n, c, f4get(yv[e], j), zp[e], xh[e]);
                    const float z = relu_f(zp[e]);
                    if (z > best || isnan(z)) { best = z; arg = e; }
                }
                const float gj = f4get(gv, j);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float gpre = (e == arg && zp[e] > 0.f) ? gj : 0.f;
                    acc[0 * 4 + j] += gpre; acc[1 * 4 + j] += gpre * xh[e]; acc[4 * 4 + j] += xh[e];
                }
            }
        } else {
            const float4 gv = ld4(g + ((long long)n * H * W + p) * ldg + c4);
            const float4 yv = ld4(y + ((long long)n * H * W + p) * ldy + c4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c4 + j;
                float zp, xh; norm_elem(np, n, c, f4get(yv, j), zp, xh);
                float gz = f4get(gv, j);
                if constexpr (FILM) {
                    const float u = relu_f(zp);
                    acc[2 * 4 + j] += gz * u; acc[3 * 4 + j] += gz;
                    gz *= fp.a[n * fp.an + c];
                }
                const float gpre = zp > 0.f ? gz : 0.f;
                acc[0 * 4 + j] += gpre; acc[1 * 4 + j] += gpre * xh; acc[4 * 4 + j] += xh;
            }
        }
    }
};

// grid (nchunks, N); block 256.  Covers pixels [chunk*csize, min(HWp, ...)) of image n.
template <class F>
__global__ __launch_bounds__(256) void chan_reduce_kernel(F f, int HWp, int C, int csize, float* slab) {
    constexpr int R = F::R;
    __shared__ float red[256 * 4 * R];
    const int C4 = C >> 2;
    const int P = 256 / C4;
    const int tid = threadIdx.x, c4 = tid % C4, pl = tid / C4;
    const int n = blockIdx.y, chunk = blockIdx.x;
    const int p0 = chunk * csize, p1 = min(HWp, p0 + csize);
    Acc4<R> a;
#pragma unroll
    for (int r = 0; r < R; ++r) a.v[r] = f4zero();
    if (pl < P)
        for (int p = p0 + pl; p < p1; p += P) f(n, p, c4 * 4, a);
    // LDS tree over the P pixel lanes
    if (pl < P) {
#pragma unroll
        for (int r = 0; r < R; ++r) st4(&red[(pl * R + r) * C + c4 * 4], a.v[r]);
    }
    __syncthreads();
    float* out = slab + ((long long)n * gridDim.x + chunk) * R * C;
    for (int idx = tid; idx < R * C; idx += 256) {
        float s = 0.f;
        for (int q = 0; q < P; ++q) s += red[q * R * C + idx];
        out[idx] = s;
    }
}

template <class F>
static int launch_reduce(const F& f, int N, int HWp, int C, int csize, float* slab, hipStream_t s) {
    if (C % 4 || C > 1024) return (int)hipErrorInvalidValue;
    const int nchunks = (HWp + csize - 1) / csize;
    hipLaunchKernelGGL(chan_reduce_kernel<F>, dim3(nchunks, N), dim3(256), 0, s, f, HWp, C, csize, slab);
    return cdm_status();
}

// -------------------------------------------------------------------------------------------------
// stage 1 of every slab fold: part[s][r][c] = sum over tiles of split s of slab[t][r][c]   (fp64)
// grid (ceil(C/64), S); 256 threads = 64 channels x 4 tile lanes (coalesced over channels)
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void slab_colsum_kernel(const float* __restrict__ slab, int ntiles, int R, int C,
                                                          double* __restrict__ part, int per) {
    __shared__ double red[4][64];
    const int cl = threadIdx.x & 63, lane = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int t0 = blockIdx.y * per, t1 = min(ntiles, t0 + per);
    for (int r = 0; r < R; ++r) {
        double acc = 0.0;
        if (c < C) {
            // the same serial order of additions, its loads issued 8 at a time (the loop was load-latency bound)
            int t = t0 + lane;
            for (; t + 28 < t1; t += 32) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = slab[((long long)(t + 4 * u) * R + r) * C + c];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += (double)v[u];
            }
            for (; t < t1; t += 4) acc += (double)slab[((long long)t * R + r) * C + c];
        }
        red[lane][cl] = acc;
        __syncthreads();
        if (lane == 0 && c < C)
            part[((long long)blockIdx.y * R + r) * C + c] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------------------
// finalize kernels (fold the fp64 partials)
// -------------------------------------------------------------------------------------------------
// BatchNorm (train): per channel over all ntiles = N*nchunks partials.  Updates running stats like
// torch (momentum 0.1, unbiased running var), increments num_batches_tracked (int64) once.
// Block = 16 channels x 16 lanes over the S partials (strided), folded through LDS in a fixed order.
__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const double* part, int S, int R, int C, double count,
                                       const float* gamma, const float* beta, float* rmean, float* rvar,
                                       long long* nbt, float momentum, float eps, float* mean, float* invstd,
                                       float* scale, float* shift, const int* ymm, int ymm_ld, float* amax_z) {
    __shared__ double rs[16][17], rq[16][17];
    const int cl = threadIdx.x & 15, ln = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + cl;
    if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
    {
        double s = 0.0, q = 0.0;
        if (c < C) {
            int t = ln;
            for (; t + 48 < S; t += 64) {   // loads 4 partials ahead, additions in the serial order
                double vs[4], vq[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    vs[u] = part[((long long)(t + 16 * u) * R + 0) * C + c];
                    vq[u] = part[((long long)(t + 16 * u) * R + 1) * C + c];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) { s += vs[u]; q += vq[u]; }
            }
            for (; t < S; t += 16) {
                s += part[((long long)t * R + 0) * C + c];
                q += part[((long long)t * R + 1) * C + c];
            }
        }
        rs[ln][cl] = s; rq[ln][cl] = q;
    }
    __syncthreads();
    if (ln != 0 || c >= C) return;
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) { s += rs[k][cl]; q += rq[k][cl]; }
    const double mu = s / count;
    double var = q / count - mu * mu;
    if (var < 0.0) var = 0.0;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    mean[c] = (float)mu; invstd[c] = is;
    const float sc = gamma[c] * is;
    const float sh = beta[c] - (float)mu * sc;
    scale[c] = sc; shift[c] = sh;
    if (ymm) {   // exact max over the layer of z = relu(fmaf(y, sc, sh)): monotone in y, so at max y or min y
        const float yx = sc >= 0.f ? fkey_inv(ymm[c]) : fkey_inv(ymm[ymm_ld + c]);
        const float zm = relu_f(fmaf(yx, sc, sh));
        atomicMax(reinterpret_cast<unsigned*>(amax_z), __float_as_uint(zm));
    }
    if (rmean) {
        const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
        rmean[c] = (float)((double)momentum * mu + (1.0 - (double)momentum) * (double)rmean[c]);
        rvar[c] = (float)((double)momentum * unb + (1.0 - (double)momentum) * (double)rvar[c]);
    }
}

// BatchNorm (eval): scale/shift from running stats.
__global__ void bn_eval_coeffs_kernel(int C, const float* gamma, const float* beta, const float* rmean,
                                      const float* rvar, float eps, float* mean, float* invstd, float* scale,
                                      float* shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float is = 1.0f / sqrtf(rvar[c] + eps);
    const float sc = gamma[c] * is;
    mean[c] = rmean[c]; invstd[c] = is; scale[c] = sc; shift[c] = beta[c] - rmean[c] * sc;
}

// eval-mode BatchNorm inside the train-structured forward (gradients through model.eval()): the coefficients of
// bn_eval_coeffs_kernel and, for a fused (BN-ReLU staged) layer under h3, the exact max of z = relu(y s + t) from the
// conv epilogue's per-channel max / min keys (as bn_fwd_finalize_kernel); running statistics untouched
__global__ void bn_frozen_fwd_kernel(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                     float eps, float* mean, float* invstd, float* scale, float* shift, const int* ymm,
                                     int ymm_ld, float* amax_z) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float is = 1.0f / sqrtf(rvar[c] + eps);
    const float sc = gamma[c] * is, sh = beta[c] - rmean[c] * sc;
    mean[c] = rmean[c]; invstd[c] = is; scale[c] = sc; shift[c] = sh;
    if (ymm) {
        const float yx = sc >= 0.f ? fkey_inv(ymm[c]) : fkey_inv(ymm[ymm_ld + c]);
        atomicMax(reinterpret_cast<unsigned*>(amax_z), __float_as_uint(relu_f(fmaf(yx, sc, sh))));
    }
}

// GroupNorm: block per image n; partials slab[n][nchunks][R][C].
// one block per (sample n, group g): the group's (chunk, channel) partials strided over 256 threads, fp64, then a
// fixed-order tree (deterministic).  (One thread per group walking every chunk took ~1 ms per launch at C5's
// 256^2 maps: 512 chunks x 8 channels serially, 16 blocks.)
__global__ __launch_bounds__(256) void gn_fwd_finalize_kernel(const float* slab, int nchunks, int R, int C, int G,
                                       double count, const float* gamma, const float* beta, float eps, float* mean,
                                       float* invstd, float* scale, float* shift) {
    const int n = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
    const int cpg = C / G;
    __shared__ double rs[256], rq[256];
    __shared__ float sm, si;
    double s = 0.0, q = 0.0;
    for (int i = tid; i < nchunks * cpg; i += 256) {
        const int k = i / cpg, c = g * cpg + (i - k * cpg);
        const float* p = slab + (((long long)n * nchunks + k) * R) * C + c;
        s += p[0]; q += p[C];
    }
    rs[tid] = s; rq[tid] = q;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) { rs[tid] += rs[tid + o]; rq[tid] += rq[tid + o]; }
        __syncthreads();
    }
    if (tid == 0) {
        const double mu = rs[0] / count;
        double var = rq[0] / count - mu * mu;
        if (var < 0.0) var = 0.0;
        sm = (float)mu; si = (float)(1.0 / sqrt(var + (double)eps));
        mean[n * G + g] = sm; invstd[n * G + g] = si;
    }
    __syncthreads();
    for (int c = g * cpg + tid; c < (g + 1) * cpg; c += 256) {
        const float sc = gamma[c] * si;
        scale[n * C + c] = sc; shift[n * C + c] = beta[c] - sm * sc;
    }
}

// BatchNorm backward: dgamma/dbeta (assign), dy = A*gpre + B + Cc*xhat coefficients, conv bias grad.
// frozen (eval-mode BatchNorm, running statistics): y_hat does not depend on the batch, so dy = gamma invstd g_pre only
// (A = gamma invstd, B = Cc = 0) and dbias = A S1 — the backward of torch's batch_norm(training=False)
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* part, int S, int C, double count,
                                       const float* gamma, const float* invstd, float* dgamma, float* dbeta, float* A,
                                       float* B, float* Cc, float* dbias, int frozen) {
    __shared__ double r1[16][17], r2[16][17], r5[16][17];
    const int cl = threadIdx.x & 15, ln = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + cl;
    {
        double s1 = 0.0, s2 = 0.0, s5 = 0.0;
        if (c < C) {
            int t = ln;
            for (; t + 48 < S; t += 64) {   // loads 4 partials ahead, additions in the serial order
                double v1[4], v2[4], v5[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double* p = part + (long long)(t + 16 * u) * 5 * C;
                    v1[u] = p[0 * C + c]; v2[u] = p[1 * C + c]; v5[u] = p[4 * C + c];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) { s1 += v1[u]; s2 += v2[u]; s5 += v5[u]; }
            }
            for (; t < S; t += 16) {
                const double* p = part + (long long)t * 5 * C;
                s1 += p[0 * C + c]; s2 += p[1 * C + c]; s5 += p[4 * C + c];
            }
        }
        r1[ln][cl] = s1; r2[ln][cl] = s2; r5[ln][cl] = s5;
    }
    __syncthreads();
    if (ln != 0 || c >= C) return;
    double s1 = 0.0, s2 = 0.0, s5 = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) { s1 += r1[k][cl]; s2 += r2[k][cl]; s5 += r5[k][cl]; }
    const double a = (double)gamma[c] * (double)invstd[c];
    const double b = frozen ? 0.0 : -a * s1 / count, cc = frozen ? 0.0 : -a * s2 / count;
    dgamma[c] = (float)s2; dbeta[c] = (float)s1;
    A[c] = (float)a; B[c] = (float)b; Cc[c] = (float)cc;
    if (dbias) dbias[c] = (float)(a * s1 + b * count + cc * s5);
}

// GroupNorm backward: block per image n. Writes per-(n,c) coefficients and per-(n,c) parameter
// partials pdg/pdb/pdbias[n][c] (summed over n by a follow-up column reduction) and FiLM sums.
// one block per (sample n, group g) as the forward finalize: thread t sums channel g*cpg + t % cpg over the chunks
// t / cpg, t / cpg + 256 / cpg, ... (fp64); the per-channel sums are then folded in thread order (deterministic),
// and the group sums sum_c gamma_c * (channel sum) follow from them.
__global__ __launch_bounds__(256) void gn_bwd_finalize_kernel(const float* slab, int nchunks, int C, int G,
                                       double count_g, int HW, const float* gamma, const float* invstd, float* A,
                                       float* B, float* Cc, float* pdg, float* pdb, float* pdbias) {
    const int n = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, cpg = C / G;
    __shared__ double r1[256], r2[256], r5[256];
    __shared__ double ch1[64], ch2[64], ch5[64], gs[2];
    const int per = 256 / cpg;                      // threads per channel (cpg <= 64: launch check)
    const int cl = tid % cpg, c = g * cpg + cl;
    double s1 = 0.0, s2 = 0.0, s5 = 0.0;
    if (tid < per * cpg)
        for (int k = tid / cpg; k < nchunks; k += per) {
            const float* p = slab + ((long long)n * nchunks + k) * 5 * C + c;
            s1 += p[0]; s2 += p[C]; s5 += p[4 * C];
        }
    r1[tid] = s1; r2[tid] = s2; r5[tid] = s5;
    __syncthreads();
    if (tid < cpg) {
        double a = 0.0, b = 0.0, e = 0.0;
        for (int j = 0; j < per; ++j) { a += r1[j * cpg + tid]; b += r2[j * cpg + tid]; e += r5[j * cpg + tid]; }
        ch1[tid] = a; ch2[tid] = b; ch5[tid] = e;
    }
    __syncthreads();
    if (tid == 0) {
        double a1 = 0.0, a2 = 0.0;
        for (int j = 0; j < cpg; ++j) { a1 += (double)gamma[g * cpg + j] * ch1[j]; a2 += (double)gamma[g * cpg + j] * ch2[j]; }
        gs[0] = a1; gs[1] = a2;
    }
    __syncthreads();
    if (tid < cpg) {
        const double is = invstd[n * G + g];
        const double a = (double)gamma[c] * is, b = -is * gs[0] / count_g, cc = -is * gs[1] / count_g;
        A[n * C + c] = (float)a; B[n * C + c] = (float)b; Cc[n * C + c] = (float)cc;
        pdg[n * C + c] = (float)ch2[tid]; pdb[n * C + c] = (float)ch1[tid];
        pdbias[n * C + c] = (float)(a * ch1[tid] + b * (double)HW + cc * ch5[tid]);
    }
}

// out[n][c] = sum over chunks of slab[n][k][r][c]   (FiLM dcemb / dtemb, per-sample sums)
__global__ void slab_sum_nc_kernel(const float* slab, int N, int nchunks, int R, int r, int C, float* out) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= N * C) return;
    const int n = idx / C, c = idx - n * C;
    double s = 0.0;
    for (int k = 0; k < nchunks; ++k) s += slab[(((long long)n * nchunks + k) * R + r) * C + c];
    out[idx] = (float)s;
}

// out[c] (+)= sum_n in[n][c]
// up to three independent column sums in one launch (blockIdx.y selects the pair); 64 columns per block, the rows
// split over the 4 waves (8 loads in flight per lane), folded in a fixed order: deterministic
struct ColSum3 { const float* in[3]; float* out[3]; };
__global__ __launch_bounds__(256) void col_sum_kernel(ColSum3 cs, int N, int C, int accumulate) {
    __shared__ double red[4][64];
    const float* in = cs.in[blockIdx.y];
    float* out = cs.out[blockIdx.y];
    const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
    double s = 0.0;
    if (c < C) {
        int n = grp;
        for (; n + 28 < N; n += 32) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = in[(long long)(n + 4 * k) * C + c];
#pragma unroll
            for (int k = 0; k < 8; ++k) s += v[k];
        }
        for (; n < N; n += 4) s += in[(long long)n * C + c];
    }
    red[grp][cl] = s;
    __syncthreads();
    if (grp == 0 && c < C) {
        const float r = (float)(red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]);
        out[c] = accumulate ? out[c] + r : r;
    }
}

// -------------------------------------------------------------------------------------------------
// elementwise forward apply:  out = [pool]( [film]( relu(y*s+t) ) [+ resid] )
// -------------------------------------------------------------------------------------------------
// RESID: 0 none, 1 the C_in = 1 shortcut w[c] x[p] + b[c], 2 the in_channels > 1 shortcut (a dot over rp.xc channels;
// a template value of its own: a run-time branch in the C_in = 1 form cost it 2.5x, 218 -> 544 us per 64^2 apply)
template <bool POOL, bool FILM, int RESID, bool RELU>
__global__ __launch_bounds__(256) void norm_apply_fwd_kernel(const float* y, int ldy, int N, int H, int W, int C,
                                                             NormP np, FilmP fp, ResidP rp, float* out, int ldo,
                                                             float* amax) {
    const int C4 = C >> 2;
    float am = 0.f;
    const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
    const long long total = (long long)N * Ho * Wo * C4;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4) * 4;
        const long long pix = idx / C4;                  // n*Ho*Wo + p
        const int n = (int)(pix / (Ho * Wo));
        const int p = (int)(pix - (long long)n * Ho * Wo);
        float o[4];
        if constexpr (POOL) {
            const int ho = p / Wo, wo = p - ho * Wo;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = -INFINITY;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float4 v = ld4(y + ((long long)(n * H + 2 * ho + (e >> 1)) * W + 2 * wo + (e & 1)) * ldy + c4);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float z = fmaf(f4get(v, j), np.s[n * np.sn + c4 + j], np.t[n * np.sn + c4 + j]);
                    if (RELU) z = relu_f(z);
                    if (z > o[j] || isnan(z)) o[j] = z;
                }
            }
        } else {
            const float4 v = ld4(y + pix * ldy + c4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c4 + j;
                float z = fmaf(f4get(v, j), np.s[n * np.sn + c], np.t[n * np.sn + c]);
                if (RELU) z = relu_f(z);
                if constexpr (FILM) z = fp.a[n * fp.an + c] * z + fp.b[n * fp.bn + c];
                if constexpr (RESID == 1) {
                    const int sel = n >= rp.split ? C : 0;
                    z = rp.w[sel + c] * rp.x[pix] + rp.b[sel + c] + z;
                } else if constexpr (RESID == 2) {   // in_channels > 1: the 1x1 shortcut's dot over the image channels
                    const int sel = n >= rp.split ? C : 0;
                    const float* wr = rp.w + (long long)(sel + c) * rp.xc;
                    const float* xr = rp.x + pix * rp.ldx;
                    float r = rp.b[sel + c];
                    for (int k = 0; k < rp.xc; ++k) r = fmaf(wr[k], xr[k], r);
                    z = r + z;
                }
                o[j] = z;
            }
        }
        st4(out + pix * ldo + c4, make_float4(o[0], o[1], o[2], o[3]));
        am = fmaxf(am, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
    }
    if (amax) block_amax_commit(am, amax);
}

// elementwise backward apply: dy = A*g_pre + B + Cc*xhat   (full grid; pooled / FiLM'd g_out recomputed)
template <bool POOL, bool FILM>
__global__ __launch_bounds__(256) void norm_apply_bwd_kernel(const float* g, int ldg, const float* y, int ldy, int N,
                                                             int H, int W, int C, NormP np, FilmP fp, const float* A,
                                                             const float* B, const float* Cc, int cn, float* dy,
                                                             int lddy, float* amax) {
    const int C4 = C >> 2;
    float am = 0.f;
    const int Ho = POOL ? H / 2 : H, Wo = POOL ? W / 2 : W;
    const long long total = (long long)N * Ho * Wo * C4;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4) * 4;
        const long long pix = idx / C4;
        const int n = (int)(pix / (Ho * Wo));
        const int p = (int)(pix - (long long)n * Ho * Wo);
        const float4 gv = ld4(g + pix * ldg + c4);
        if constexpr (POOL) {
            const int ho = p / Wo, wo = p - ho * Wo;
            float4 yv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                yv[e] = ld4(y + ((long long)(n * H + 2 * ho + (e >> 1)) * W + 2 * wo + (e & 1)) * ldy + c4);
            float out[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c4 + j;
                float zp[4], xh[4], best = -INFINITY; int arg = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    norm_elem(np, n, c, f4get(yv[e], j), zp[e], xh[e]);
                    const float z = relu_f(zp[e]);
                    if (z > best || isnan(z)) { best = z; arg = e; }
                }
                const float a = A[n * cn + c], b = B[n * cn + c], cc = Cc[n * cn + c];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float gpre = (e == arg && zp[e] > 0.f) ? f4get(gv, j) : 0.f;
                    out[e][j] = fmaf(cc, xh[e], fmaf(a, gpre, b));
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                st4(dy + ((long long)(n * H + 2 * ho + (e >> 1)) * W + 2 * wo + (e & 1)) * lddy + c4,
                    make_float4(out[e][0], out[e][1], out[e][2], out[e][3]));
#pragma unroll
                for (int j = 0; j < 4; ++j) am = fmaxf(am, fabsf(out[e][j]));
            }
        } else {
            const float4 yv = ld4(y + pix * ldy + c4);
            float out[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c4 + j;
                const int si = n * np.sn + c, gi = n * np.mn + c / np.cpg;
                float gz = f4get(gv, j);
                if constexpr (FILM) gz *= fp.a[n * fp.an + c];
                out[j] = bn_bwd_elem(gz, f4get(yv, j), np.s[si], np.t[si], np.mean[gi], np.invstd[gi], A[n * cn + c],
                                     B[n * cn + c], Cc[n * cn + c]);
            }
            st4(dy + pix * lddy + c4, make_float4(out[0], out[1], out[2], out[3]));
#pragma unroll
            for (int j = 0; j < 4; ++j) am = fmaxf(am, fabsf(out[j]));
        }
    }
    if (amax) block_amax_commit(am, amax);
}

// dense BatchNorm backward of a bf16-activation (C4) layer as its own pass: dy = bn_bwd_elem(g, y) with the fused
// staging's expression, g / y of element type GT, dy stored as OT (bf16: the value the fused dgrad staging would have
// rounded to).  8 channels per thread (16-byte bf16 loads).  The dgrad and weight gradient then stage dy as a plain
// operand (the LDS-halo forward schedule, halo two chunks ahead, which the fused BN-backward staging cannot hold).
template <class GT, class OT>
__global__ __launch_bounds__(256) void bn_bwd_dy_kernel(const GT* __restrict__ g, int ldg, const GT* __restrict__ y,
                                                        int ldy, long long P, int C, const float* __restrict__ s,
                                                        const float* __restrict__ t, const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, const float* __restrict__ A,
                                                        const float* __restrict__ B, const float* __restrict__ Cc,
                                                        OT* __restrict__ dy, int lddy) {
    const int C8 = C >> 3;
    const long long total = P * C8;
    const long long stride = (long long)gridDim.x * blockDim.x;
    // the grid stride is a multiple of C8 (host: C8 divides 256), so a thread keeps its channel octet: its 72
    // coefficients are loaded once, not per element (the per-element scalar loads held the pass at 3.8 TB/s)
    const long long idx0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int c8 = (int)(idx0 % C8) * 8;
    float cf[7][8];
    {
        const float* src[7] = {s, t, mean, invstd, A, B, Cc};
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const float4 a = ld4(src[k] + c8), b = ld4(src[k] + c8 + 4);
            cf[k][0] = a.x; cf[k][1] = a.y; cf[k][2] = a.z; cf[k][3] = a.w;
            cf[k][4] = b.x; cf[k][5] = b.y; cf[k][6] = b.z; cf[k][7] = b.w;
        }
    }
    for (long long idx = idx0; idx < total; idx += stride) {
        const long long pix = idx / C8;
        const float4 g0 = Act<GT>::to4(Act<GT>::load4(g + pix * ldg + c8));
        const float4 g1 = Act<GT>::to4(Act<GT>::load4(g + pix * ldg + c8 + 4));
        const float4 y0 = Act<GT>::to4(Act<GT>::load4(y + pix * ldy + c8));
        const float4 y1 = Act<GT>::to4(Act<GT>::load4(y + pix * ldy + c8 + 4));
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float gv = j < 4 ? f4get(g0, j) : f4get(g1, j - 4), yv = j < 4 ? f4get(y0, j) : f4get(y1, j - 4);
            o[j] = bn_bwd_elem(gv, yv, cf[0][j], cf[1][j], cf[2][j], cf[3][j], cf[4][j], cf[5][j], cf[6][j]);
        }
        OT* d = dy + pix * lddy + c8;
        if constexpr (std::is_same<OT, float>::value) {
            st4(d, make_float4(o[0], o[1], o[2], o[3]));
            st4(d + 4, make_float4(o[4], o[5], o[6], o[7]));
        } else {
            typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
            *reinterpret_cast<bf16x8_t*>(d) = bf16x8_t{(__bf16)o[0], (__bf16)o[1], (__bf16)o[2], (__bf16)o[3],
                                                       (__bf16)o[4], (__bf16)o[5], (__bf16)o[6], (__bf16)o[7]};
        }
    }
}

// upper bound of max|dy| for the fused BN backward (dy never materialised): per channel
// |A| max|g| + |B| + |Cc| (max|y| + |mean|) invstd >= |A g_pre + B + Cc xhat|; max over channels into *out
__global__ __launch_bounds__(256) void bn_bwd_amax_bound_kernel(int C, const float* A, const float* B, const float* Cc,
                                                                const float* mean, const float* invstd,
                                                                const float* amax_g, const float* amax_y, float* out) {
    const float G = *amax_g, Y = *amax_y;
    float m = 0.f;
    for (int c = threadIdx.x; c < C; c += blockDim.x)
        m = fmaxf(m, fabsf(A[c]) * G + fabsf(B[c]) + fabsf(Cc[c]) * (Y + fabsf(mean[c])) * invstd[c]);
    block_amax_commit(m, out);
}

static inline int ew_blocks(long long total) {
    long long b = (total + 255) / 256;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (int)b;
}

}  // namespace cdm

using namespace cdm;
static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------ C ABI ------------------------------------------------
CDM_API int cdm_reduce_stats(const float* y, int ldy, int N, int HW, int C, int csize, float* slab, void* stream) {
    return launch_reduce(StatsF{y, ldy, HW}, N, HW, C, csize, slab, S(stream));
}

// cdm_reduce_stats (the same per-lane sums and fold order) + optional per-channel max / min of y as ordered-int keys
// (atomic max into ymm[c], min into ymm[ymm_ld + c]): the BN statistics of the C_in = 1 init conv, whose train-mode
// BN-ReLU apply then runs in the next conv's staging (bn_fwd_finalize turns the keys into the exact max|z|).
// A block covers U0S_CG consecutive chunks of one image (one slab partial per chunk) and issues its max / min atomics
// once: one block per chunk put 2 M atomics on the 2C key addresses at bs = 256 (~120 us of contention).
constexpr int U0S_CG = 8;
__global__ __launch_bounds__(256) void stats_mm_kernel(const float* __restrict__ y, int ldy, int HW, int C, int csize,
                                                       int nchunks, float* __restrict__ slab, int* ymm, int ymm_ld) {
    __shared__ float red[256 * 4 * 2];
    __shared__ float rmx[256 * 4], rmn[256 * 4];
    const int C4 = C >> 2;
    const int P = 256 / C4;
    const int tid = threadIdx.x, c4 = tid % C4, pl = tid / C4;
    const int n = blockIdx.y;
    float4 hi = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY), lo = make_float4(INFINITY, INFINITY, INFINITY, INFINITY);
    const int cend = min(nchunks, (int)(blockIdx.x + 1) * U0S_CG);
    for (int chunk = blockIdx.x * U0S_CG; chunk < cend; ++chunk) {
        const int p0 = chunk * csize, p1 = min(HW, p0 + csize);
        Acc4<2> a;
        a.v[0] = f4zero(); a.v[1] = f4zero();
        auto take = [&](const float4 v) {   // one read of y per element: StatsF's sums + max / min
            a.v[0].x += v.x; a.v[0].y += v.y; a.v[0].z += v.z; a.v[0].w += v.w;
            a.v[1].x += v.x * v.x; a.v[1].y += v.y * v.y; a.v[1].z += v.z * v.z; a.v[1].w += v.w * v.w;
            hi = make_float4(fmaxf(hi.x, v.x), fmaxf(hi.y, v.y), fmaxf(hi.z, v.z), fmaxf(hi.w, v.w));
            lo = make_float4(fminf(lo.x, v.x), fminf(lo.y, v.y), fminf(lo.z, v.z), fminf(lo.w, v.w));
        };
        if (pl < P) {
            const float* yb = y + (long long)n * HW * ldy + c4 * 4;
            int p = p0 + pl;
            for (; p + 7 * P < p1; p += 8 * P) {   // 8 loads in flight, taken in the serial order (same sums)
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = ld4(yb + (long long)(p + u * P) * ldy);
#pragma unroll
                for (int u = 0; u < 8; ++u) take(v[u]);
            }
            for (; p < p1; p += P) take(ld4(yb + (long long)p * ldy));
        }
        __syncthreads();   // red is reused per chunk
        if (pl < P) {
#pragma unroll
            for (int r = 0; r < 2; ++r) st4(&red[(pl * 2 + r) * C + c4 * 4], a.v[r]);
        }
        __syncthreads();
        float* out = slab + ((long long)n * nchunks + chunk) * 2 * C;
        for (int idx = tid; idx < 2 * C; idx += 256) {
            float sacc = 0.f;
            for (int q = 0; q < P; ++q) sacc += red[q * 2 * C + idx];
            out[idx] = sacc;
        }
    }
    if (!ymm) return;
    if (pl < P) {
        st4(&rmx[pl * C + c4 * 4], hi);
        st4(&rmn[pl * C + c4 * 4], lo);
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        float mx = -INFINITY, mn = INFINITY;
        for (int q = 0; q < P; ++q) { mx = fmaxf(mx, rmx[q * C + c]); mn = fminf(mn, rmn[q * C + c]); }
        atomicMax(ymm + c, fkey(mx));
        atomicMin(ymm + ymm_ld + c, fkey(mn));
    }
}

CDM_API int cdm_reduce_stats_mm(const float* y, int ldy, int N, int HW, int C, int csize, float* slab, int* ymm,
                                int ymm_ld, void* stream) {
    if (C % 4 || C > 1024) return (int)hipErrorInvalidValue;
    const int nchunks = (HW + csize - 1) / csize;
    hipLaunchKernelGGL(stats_mm_kernel, dim3((nchunks + U0S_CG - 1) / U0S_CG, N), dim3(256), 0, S(stream), y, ldy, HW,
                       C, csize, nchunks, slab, ymm, ymm_ld);
    return cdm_status();
}

CDM_API int cdm_reduce_sum(const float* g, int ldg, int N, int HW, int C, int csize, float* slab, void* stream) {
    return launch_reduce(SumF{g, ldg, HW}, N, HW, C, csize, slab, S(stream));
}

// mode: 0 plain, 1 pooled g (2x2 max pool after the relu), 2 FiLM after the relu
CDM_API int cdm_norm_bwd_reduce(int mode, const float* g, int ldg, const float* y, int ldy, int N, int H, int W, int C,
                                const float* s, const float* t, int sn, const float* mean, const float* invstd, int mn,
                                int cpg, const float* film_a, int film_an, int csize, float* slab, void* stream) {
    NormP np{s, t, sn, mean, invstd, mn, cpg};
    FilmP fp{film_a, film_an, nullptr, 0};
    if (mode == 1)
        return launch_reduce(NormBwdF<true, false>{g, ldg, y, ldy, H, W, np, fp}, N, (H / 2) * (W / 2), C, csize, slab,
                             S(stream));
    if (mode == 2)
        return launch_reduce(NormBwdF<false, true>{g, ldg, y, ldy, H, W, np, fp}, N, H * W, C, csize, slab, S(stream));
    return launch_reduce(NormBwdF<false, false>{g, ldg, y, ldy, H, W, np, fp}, N, H * W, C, csize, slab, S(stream));
}

CDM_API int cdm_slab_colsum(const float* slab, int ntiles, int R, int C, double* part, int splits, void* stream) {
    if (splits < 1) splits = 1;
    const int per = (ntiles + splits - 1) / splits;
    hipLaunchKernelGGL(slab_colsum_kernel, dim3((C + 63) / 64, splits), dim3(256), 0, S(stream), slab, ntiles, R, C, part,
                       per);
    return cdm_status();
}

CDM_API int cdm_bn_fwd_finalize(const double* part, int nparts, int R, int C, double count, const float* gamma,
                                const float* beta, float* rmean, float* rvar, long long* nbt, float momentum, float eps,
                                float* mean, float* invstd, float* scale, float* shift, const int* ymm, int ymm_ld,
                                float* amax_z, void* stream) {
    if (ymm && !amax_z) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, S(stream), part, nparts, R, C, count,
                       gamma, beta, rmean, rvar, nbt, momentum, eps, mean, invstd, scale, shift, ymm, ymm_ld, amax_z);
    return cdm_status();
}
__global__ void fill_i32_kernel(int* p, long long n, int v) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}
CDM_API int cdm_fill_i32(int* p, long long n, int v, void* stream) {
    if (n <= 0) return 0;
    long long b = (n + 255) / 256;
    hipLaunchKernelGGL(fill_i32_kernel, dim3((int)(b > 4096 ? 4096 : b)), dim3(256), 0, S(stream), p, n, v);
    return cdm_status();
}

CDM_API int cdm_bn_fwd_frozen(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                              float eps, float* mean, float* invstd, float* scale, float* shift, const int* ymm,
                              int ymm_ld, float* amax_z, void* stream) {
    if (ymm && !amax_z) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_frozen_fwd_kernel, dim3((C + 255) / 256), dim3(256), 0, S(stream), C, gamma, beta, rmean, rvar,
                       eps, mean, invstd, scale, shift, ymm, ymm_ld, amax_z);
    return cdm_status();
}
CDM_API int cdm_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                               float eps, float* mean, float* invstd, float* scale, float* shift, void* stream) {
    hipLaunchKernelGGL(bn_eval_coeffs_kernel, dim3((C + 255) / 256), dim3(256), 0, S(stream), C, gamma, beta, rmean, rvar,
                       eps, mean, invstd, scale, shift);
    return cdm_status();
}

CDM_API int cdm_gn_fwd_finalize(const float* slab, int N, int nchunks, int R, int C, int G, double count,
                                const float* gamma, const float* beta, float eps, float* mean, float* invstd,
                                float* scale, float* shift, void* stream) {
    if (G > 64) return (int)hipErrorInvalidValue;
    if (C % G) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(gn_fwd_finalize_kernel, dim3(N, G), dim3(256), 0, S(stream), slab, nchunks, R, C, G, count,
                       gamma, beta, eps, mean, invstd, scale, shift);
    return cdm_status();
}

CDM_API int cdm_bn_bwd_finalize(const double* part, int nparts, int C, double count, const float* gamma,
                                const float* invstd, float* dgamma, float* dbeta, float* A, float* B, float* Cc,
                                float* dbias, void* stream) {
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, S(stream), part, nparts, C, count,
                       gamma, invstd, dgamma, dbeta, A, B, Cc, dbias, 0);
    return cdm_status();
}
CDM_API int cdm_bn_bwd_finalize_frozen(const double* part, int nparts, int C, double count, const float* gamma,
                                       const float* invstd, float* dgamma, float* dbeta, float* A, float* B, float* Cc,
                                       float* dbias, void* stream) {
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, S(stream), part, nparts, C, count,
                       gamma, invstd, dgamma, dbeta, A, B, Cc, dbias, 1);
    return cdm_status();
}

CDM_API int cdm_gn_bwd_finalize(const float* slab, int N, int nchunks, int C, int G, double count_g, int HW,
                                const float* gamma, const float* invstd, float* A, float* B, float* Cc, float* pdg,
                                float* pdb, float* pdbias, void* stream) {
    if (C % G || C / G > 64) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(N, G), dim3(256), 0, S(stream), slab, nchunks, C, G, count_g, HW,
                       gamma, invstd, A, B, Cc, pdg, pdb, pdbias);
    return cdm_status();
}

CDM_API int cdm_slab_sum_nc(const float* slab, int N, int nchunks, int R, int r, int C, float* out, void* stream) {
    hipLaunchKernelGGL(slab_sum_nc_kernel, dim3((N * C + 255) / 256), dim3(256), 0, S(stream), slab, N, nchunks, R, r, C,
                       out);
    return cdm_status();
}

CDM_API int cdm_col_sum(const float* in, int N, int C, float* out, int accumulate, void* stream) {
    ColSum3 cs{{in, nullptr, nullptr}, {out, nullptr, nullptr}};
    hipLaunchKernelGGL(col_sum_kernel, dim3((C + 63) / 64, 1), dim3(256), 0, S(stream), cs, N, C, accumulate);
    return cdm_status();
}
CDM_API int cdm_col_sum3(const float* in0, float* out0, const float* in1, float* out1, const float* in2, float* out2,
                         int N, int C, void* stream) {
    const int k = in2 ? 3 : (in1 ? 2 : 1);
    ColSum3 cs{{in0, in1, in2}, {out0, out1, out2}};
    hipLaunchKernelGGL(col_sum_kernel, dim3((C + 63) / 64, k), dim3(256), 0, S(stream), cs, N, C, 0);
    return cdm_status();
}

// flags: 1 pool, 2 film, 4 resid, 8 relu
CDM_API int cdm_norm_apply_fwd(int flags, const float* y, int ldy, int N, int H, int W, int C, const float* s,
                               const float* t, int sn, const float* film_a, int film_an, const float* film_b,
                               int film_bn, const float* rx, const float* rw, const float* rb, int rsplit, float* out,
                               int ldo, float* amax, void* stream) {
    if (C % 4) return (int)hipErrorInvalidValue;
    NormP np{s, t, sn, nullptr, nullptr, 0, 1};
    FilmP fp{film_a, film_an, film_b, film_bn};
    ResidP rp{rx, rw, rb, rsplit};
    const bool pool = flags & 1, film = flags & 2, resid = flags & 4, relu = flags & 8;
    const long long total = (long long)N * (pool ? (H / 2) * (W / 2) : H * W) * (C / 4);
    const int nb = ew_blocks(total);
#define CDM_APPLY(P, F, Rz, Rl) \
    hipLaunchKernelGGL((norm_apply_fwd_kernel<P, F, Rz, Rl>), dim3(nb), dim3(256), 0, S(stream), y, ldy, N, H, W, C, np, fp, rp, out, ldo, amax)
    if (pool) {
        if (film || resid) return (int)hipErrorInvalidValue;
        if (relu) CDM_APPLY(true, false, 0, true); else CDM_APPLY(true, false, 0, false);
    } else if (film) {
        if (resid) return (int)hipErrorInvalidValue;
        if (relu) CDM_APPLY(false, true, 0, true); else CDM_APPLY(false, true, 0, false);
    } else if (resid) {
        if (relu) CDM_APPLY(false, false, 1, true); else CDM_APPLY(false, false, 1, false);
    } else {
        if (relu) CDM_APPLY(false, false, 0, true); else CDM_APPLY(false, false, 0, false);
    }
#undef CDM_APPLY
    return cdm_status();
}

// the residual apply of ResidualConvBlock(in_channels > 1, C, is_res) (diffusion_utilities.py:45-55 with the fresh 1x1
// shortcut of :54): out = [relu](y s + t) + rb[c] + sum_k rw[c][k] rx[p][k], k < xc image channels at pixel stride ldx
// (rw / rb: [2][C][xc] / [2][C] when rsplit < N, the CFG halves' two draws)
CDM_API int cdm_norm_apply_fwd_resid_c(int relu, const float* y, int ldy, int N, int H, int W, int C, const float* s,
                                       const float* t, const float* rx, int ldx, int xc, const float* rw, const float* rb,
                                       int rsplit, float* out, int ldo, float* amax, void* stream) {
    if (C % 4 || xc < 1 || ldx < xc) return (int)hipErrorInvalidValue;
    NormP np{s, t, 0, nullptr, nullptr, 0, 1};
    FilmP fp{nullptr, 0, nullptr, 0};
    ResidP rp{rx, rw, rb, rsplit, xc, ldx};
    const int nb = ew_blocks((long long)N * H * W * (C / 4));
    if (relu)
        hipLaunchKernelGGL((norm_apply_fwd_kernel<false, false, 2, true>), dim3(nb), dim3(256), 0, S(stream), y, ldy, N,
                           H, W, C, np, fp, rp, out, ldo, amax);
    else
        hipLaunchKernelGGL((norm_apply_fwd_kernel<false, false, 2, false>), dim3(nb), dim3(256), 0, S(stream), y, ldy,
                           N, H, W, C, np, fp, rp, out, ldo, amax);
    return cdm_status();
}

CDM_API int cdm_norm_apply_bwd(int mode, const float* g, int ldg, const float* y, int ldy, int N, int H, int W, int C,
                               const float* s, const float* t, int sn, const float* mean, const float* invstd, int mn,
                               int cpg, const float* film_a, int film_an, const float* A, const float* B,
                               const float* Cc, int cn, float* dy, int lddy, float* amax, void* stream) {
    if (C % 4) return (int)hipErrorInvalidValue;
    NormP np{s, t, sn, mean, invstd, mn, cpg};
    FilmP fp{film_a, film_an, nullptr, 0};
    const long long total = (long long)N * (mode == 1 ? (H / 2) * (W / 2) : H * W) * (C / 4);
    const int nb = ew_blocks(total);
    if (mode == 1)
        hipLaunchKernelGGL((norm_apply_bwd_kernel<true, false>), dim3(nb), dim3(256), 0, S(stream), g, ldg, y, ldy, N, H, W,
                           C, np, fp, A, B, Cc, cn, dy, lddy, amax);
    else if (mode == 2)
        hipLaunchKernelGGL((norm_apply_bwd_kernel<false, true>), dim3(nb), dim3(256), 0, S(stream), g, ldg, y, ldy, N, H,
                           W, C, np, fp, A, B, Cc, cn, dy, lddy, amax);
    else
        hipLaunchKernelGGL((norm_apply_bwd_kernel<false, false>), dim3(nb), dim3(256), 0, S(stream), g, ldg, y, ldy, N, H,
                           W, C, np, fp, A, B, Cc, cn, dy, lddy, amax);
    return cdm_status();
}

CDM_API int cdm_bn_bwd_dy(const void* g, int ldg, const void* y, int ldy, long long P, int C, const float* s,
                          const float* t, const float* mean, const float* invstd, const float* A, const float* B,
                          const float* Cc, void* dy, int lddy, int dt, void* stream) {
    // dt bit 0: g and y are bf16, bit 1: dy is stored as bf16
    if (C <= 0 || C % 8 || 256 % (C / 8) || ldg % 8 || ldy % 8 || lddy % 8 || P < 0) return (int)hipErrorInvalidValue;
    if (P == 0) return 0;
    const int nb = ew_blocks(P * (C / 8));
    auto run = [&](auto gtag, auto otag) {
        using GT = decltype(gtag);
        using OT = decltype(otag);
        hipLaunchKernelGGL((bn_bwd_dy_kernel<GT, OT>), dim3(nb), dim3(256), 0, S(stream),
                           reinterpret_cast<const GT*>(g), ldg, reinterpret_cast<const GT*>(y), ldy, P, C, s, t, mean,
                           invstd, A, B, Cc, reinterpret_cast<OT*>(dy), lddy);
        return cdm_status();
    };
    switch (dt & 3) {
        case 1: return run(__bf16{}, float{});
        case 2: return run(float{}, __bf16{});
        case 3: return run(__bf16{}, __bf16{});
        default: return run(float{}, float{});
    }
}

CDM_API int cdm_bn_bwd_amax_bound(int C, const float* A, const float* B, const float* Cc, const float* mean,
                                  const float* invstd, const float* amax_g, const float* amax_y, float* amax_dy,
                                  void* stream) {
    if (!amax_g || !amax_y || !amax_dy) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bn_bwd_amax_bound_kernel, dim3(1), dim3(256), 0, S(stream), C, A, B, Cc, mean, invstd, amax_g,
                       amax_y, amax_dy);
    return cdm_status();
}
