// Small / HBM-bound kernels of the ContextUnet DDPM hot path (gfx950).
//
//   conv3x3 with C_in = 1   init_conv.conv1 (diffusion_utilities.py:27 via ContextUnet.py:14)
//   conv3x3 with C_out = 1  out.3 (ContextUnet.py:39)
//   AvgPool2d(h/4) + GELU   to_vec (ContextUnet.py:17)
//   EmbedFC x4              Linear -> GELU -> Linear (diffusion_utilities.py:118-145)
//   perturb_input           code/train_diffusion_condition.py:202-203
//   F.mse_loss (+grad)      code/train_diffusion_condition.py:227
//   denoise_add_noise + CFG code/train_diffusion_condition.py:274-279,318-329 (+ on-device snapshots :331-332)
//   torch.optim.Adam        code/train_diffusion_condition.py:200 (single-tensor Adam arithmetic)
//   weight repacking        OIHW / [Cin][Cout][kh][kw] -> GEMM-ready layouts (+ eval-mode BN fold)
#include "cdm_common.h"

namespace cdm {

static inline int nblocks(long long total, int per = 256, int cap = 8192) {
    long long b = (total + per - 1) / per;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (int)b;
}

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based; used for training noise / timesteps and sampler z)
// ------------------------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };
static __device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                            uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return U4{c0, c1, c2, c3};
}
static __device__ __forceinline__ float u01(uint32_t v) { return ((float)(v >> 8) + 0.5f) * (1.0f / 16777216.0f); }
static __device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
    const float u1 = u01(a), u2 = u01(b);
    const float r = sqrtf(-2.0f * logf(u1));
    float s, c; sincosf(6.283185307179586f * u2, &s, &c);
    z0 = r * c; z1 = r * s;
}
// normal for element e of stream `sub`
static __device__ __forceinline__ float philox_normal(unsigned long long seed, uint32_t sub, long long e) {
    const U4 v = philox((uint32_t)(e >> 2), (uint32_t)((unsigned long long)e >> 34), sub, 0x5EEDu,
                        (uint32_t)seed, (uint32_t)(seed >> 32));
    float z0, z1, z2, z3;
    box_muller(v.x, v.y, z0, z1); box_muller(v.z, v.w, z2, z3);
    const int j = (int)(e & 3);
    return j == 0 ? z0 : (j == 1 ? z1 : (j == 2 ? z2 : z3));
}

__global__ void philox_uniform_kernel(float* out, long long n, float lo, float hi, unsigned long long seed, uint32_t sub,
                                      const int* sub_dev) {
    if (sub_dev) sub += (uint32_t)*sub_dev;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q * 4 < n; q += (long long)gridDim.x * blockDim.x) {
        const U4 v = philox((uint32_t)q, (uint32_t)((unsigned long long)q >> 32), sub, 0x0417u, (uint32_t)seed,
                            (uint32_t)(seed >> 32));
        const uint32_t r[4] = {v.x, v.y, v.z, v.w};
        for (int j = 0; j < 4; ++j) if (q * 4 + j < n) out[q * 4 + j] = lo + (hi - lo) * u01(r[j]);
    }
}

__global__ void philox_normal_kernel(float* out, long long n, unsigned long long seed, uint32_t sub, const int* sub_dev) {
    if (sub_dev) sub += (uint32_t)*sub_dev;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q * 4 < n; q += (long long)gridDim.x * blockDim.x) {
        const U4 v = philox((uint32_t)q, (uint32_t)((unsigned long long)q >> 32), sub, 0x5EEDu, (uint32_t)seed,
                            (uint32_t)(seed >> 32));
        float z[4];
        box_muller(v.x, v.y, z[0], z[1]); box_muller(v.z, v.w, z[2], z[3]);
        for (int j = 0; j < 4; ++j) if (q * 4 + j < n) out[q * 4 + j] = z[j];
    }
}

// t[n] in [lo, hi] uniformly (torch.randint(1, T+1) equivalent distribution)
__global__ void philox_randint_kernel(int* out, int n, int lo, int hi, unsigned long long seed, uint32_t sub,
                                      const int* sub_dev) {
    if (sub_dev) sub += (uint32_t)*sub_dev;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const U4 v = philox((uint32_t)i, 0x71u, sub, 0xA11Cu, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint64_t r = ((uint64_t)v.x << 32) | v.y;
    out[i] = lo + (int)(r % (uint64_t)(hi - lo + 1));
}

// ------------------------------------------------------------------------------------------------
// conv3x3, C_in = 1:  y[p][co] = b[co] + sum_tap x[p+tap] * wt[tap][co]   (wt = pack_conv3x3 output, Cin = 1)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_cin1_fwd_kernel(const float* x, int N, int H, int W, const float* w9,
                                                            const float* bias, float* y, int ldy, int C, int relu,
                                                            float* amax) {
    // lanes span channels (one float4 each; a pixel's C channels are one coalesced row), the 9 input
    // taps are wave-uniform broadcast loads, the 9x4 weights of a lane stay in registers.
    // amax (optional): running max|y| for the consuming h3 conv's operand scale (block_amax_commit)
    const int C4 = C >> 2, PP = 256 / C4;
    const int c4 = (threadIdx.x % C4) * 4, pl = threadIdx.x / C4;
    float am = 0.f;
    const bool active = pl < PP;      // (every thread reaches the block max at the end: it synchronises the block)
    float wr[9][4], bb[4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) wr[tap][j] = active ? w9[tap * C + c4 + j] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) bb[j] = active ? bias[c4 + j] : 0.f;
    const long long P = active ? (long long)N * H * W : 0;
    // U pixels per thread and iteration, their 9 U input taps loaded before any is used: the loop was one L2 round
    // trip per pixel (186 us for 537 MB of output at bs=256, 2.9 TB/s)
    constexpr int U = 4;
    const long long step = (long long)gridDim.x * PP;
    for (long long pix0 = (long long)blockIdx.x * PP + pl; pix0 < P; pix0 += step * U) {
        float xv[U][9];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long pix = pix0 + u * step;
            const int n = (int)(pix / (H * W)), rem = (int)(pix - (long long)n * H * W), h = rem / W, w = rem - h * W;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int hh = h + tap / 3 - 1, ww = w + tap % 3 - 1;
                xv[u][tap] = (pix < P && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                                 ? x[((long long)n * H + hh) * W + ww] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long pix = pix0 + u * step;
            if (pix >= P) break;
            float o[4] = {bb[0], bb[1], bb[2], bb[3]};
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = fmaf(xv[u][tap], wr[tap][j], o[j]);
            if (relu) {
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = relu_f(o[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) am = fmaxf(am, fabsf(o[j]));
            st4(y + pix * ldy + c4, make_float4(o[0], o[1], o[2], o[3]));
        }
    }
    if (amax) block_amax_commit(am, amax);
}

// Row form of conv_cin1_fwd_kernel (and, below, of conv_cout1_dgrad_kernel): a block owns one image row (n, h), its
// three source rows (zero-padded, W + 2 wide) staged once in LDS, lanes over channel quads and pixels of the row.  The
// flat-pixel kernels spend a 64-bit division and nine bounds-checked global loads per pixel and lane and write at
// ~2.8 TB/s; here the output row is a plain coalesced stream.  The same fmaf sequence over the taps (zeros where the
// image ends, as there): bit-identical results.  W <= ROWK_MAXW (the flat kernels serve wider maps).
constexpr int ROWK_MAXW = 2048;
__global__ __launch_bounds__(256) void conv_cin1_fwd_row_kernel(const float* __restrict__ x, int H, int W,
                                                                const float* __restrict__ w9,
                                                                const float* __restrict__ bias, float* __restrict__ y,
                                                                int ldy, int C, int relu, float* amax) {
    extern __shared__ float xs[];   // [3][W + 2]
    const int n = blockIdx.x / H, h = blockIdx.x - n * H, WP = W + 2;
    const int C4 = C >> 2, PP = 256 / C4;
    const int c4 = (threadIdx.x % C4) * 4, pl = threadIdx.x / C4;
    const bool active = pl < PP;
    // weights and the source rows requested together (one memory round trip before the barrier, not two)
    const int cw = active ? c4 : 0;
    float wr[9][4], bb[4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        const float4 v = ld4(w9 + tap * C + cw);
        wr[tap][0] = v.x; wr[tap][1] = v.y; wr[tap][2] = v.z; wr[tap][3] = v.w;
    }
    {
        const float4 v = ld4(bias + cw);
        bb[0] = v.x; bb[1] = v.y; bb[2] = v.z; bb[3] = v.w;
    }
    for (int i = threadIdx.x; i < 3 * WP; i += 256) {
        const int r = i / WP, col = i - r * WP, hh = h + r - 1, ww = col - 1;
        const bool in = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        const float v = x[in ? ((long long)n * H + hh) * W + ww : 0];
        xs[i] = in ? v : 0.f;
    }
    __syncthreads();
    float am = 0.f;
    float* yr = y + ((long long)n * H + h) * W * ldy;
    for (int w = active ? pl : W; w < W; w += PP) {
        float o[4] = {bb[0], bb[1], bb[2], bb[3]};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const float xv = xs[(tap / 3) * WP + w + tap % 3];
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = fmaf(xv, wr[tap][j], o[j]);
        }
        if (relu) {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = relu_f(o[j]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) am = fmaxf(am, fabsf(o[j]));
        st4(yr + (long long)w * ldy + c4, make_float4(o[0], o[1], o[2], o[3]));
    }
    if (amax) block_amax_commit(am, amax);
}

// BN backward of the init conv's Conv -> BatchNorm -> ReLU applied while reading its dy (FUSED): dy is never written
struct Cin1BnBwd { const float* y; int ldy; const float* p[7]; };   // s, t, mean, invstd, A, B, Cc

// per-(n, chunk) partials R = 10: r<9 -> sum dy[p][c]*x[p+tap_r], r=9 -> sum dy[p][c]
// FUSED: dy = bn_bwd_elem(g, y) from the grad g of the ReLU output and the pre-norm y (the expression of
// norm_apply_bwd_kernel: bit-identical dy, no 537 MB write + read of it at bs=256)
template <bool FUSED>
__global__ __launch_bounds__(256) void conv_cin1_wgrad_kernel(const float* dy, int lddy, const float* x, int H, int W,
                                                              int C, int csize, float* slab, Cin1BnBwd bn) {
    constexpr int R = 10;
    __shared__ float red[256 * 4 * R];
    const int C4 = C >> 2, P = 256 / C4, tid = threadIdx.x, c4 = (tid % C4) * 4, pl = tid / C4;
    const int n = blockIdx.y, chunk = blockIdx.x, HW = H * W;
    const int p0 = chunk * csize, p1 = min(HW, p0 + csize);
    float acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[r][j] = 0.f;
    if (pl < P) {
        for (int p = p0 + pl; p < p1; p += P) {
            const int h = p / W, w = p - h * W;
            float4 g = ld4(dy + ((long long)n * HW + p) * lddy + c4);
            if constexpr (FUSED) {
                const float4 yv = ld4(bn.y + ((long long)n * HW + p) * bn.ldy + c4);
                float gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    gv[j] = bn_bwd_elem(gv[j], f4get(yv, j), bn.p[0][c4 + j], bn.p[1][c4 + j], bn.p[2][c4 + j],
                                        bn.p[3][c4 + j], bn.p[4][c4 + j], bn.p[5][c4 + j], bn.p[6][c4 + j]);
                g = make_float4(gv[0], gv[1], gv[2], gv[3]);
            }
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int hh = h + tap / 3 - 1, ww = w + tap % 3 - 1;
                const float xv = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) ? x[(long long)n * HW + hh * W + ww] : 0.f;
                acc[tap][0] += g.x * xv; acc[tap][1] += g.y * xv; acc[tap][2] += g.z * xv; acc[tap][3] += g.w * xv;
            }
            acc[9][0] += g.x; acc[9][1] += g.y; acc[9][2] += g.z; acc[9][3] += g.w;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) st4(&red[(pl * R + r) * C + c4], make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]));
    }
    __syncthreads();
    float* out = slab + ((long long)n * gridDim.x + chunk) * R * C;
    for (int idx = tid; idx < R * C; idx += 256) {
        float s = 0.f;
        for (int q = 0; q < P; ++q) s += red[q * R * C + idx];
        out[idx] = s;
    }
}

// out[r*s_r + c*s_c] (+)= sum_s part[s][r0+r][c]  for r < rn   (part = fp64 partials of cdm_slab_colsum)
// 64 outputs per block, the S partials split over the 4 waves and folded in a fixed order (deterministic)
__global__ __launch_bounds__(256) void slab_sum_all_kernel(const double* part, int S, int R, int r0, int rn, int C,
                                                           float* out, long long s_r, long long s_c, int accumulate) {
    __shared__ double red[4][64];
    const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6, idx = blockIdx.x * 64 + cl;
    double s = 0.0;
    int r = 0, c = 0;
    if (idx < rn * C) {
        r = idx / C; c = idx - r * C;
        const double* src = part + (long long)(r0 + r) * C + c;
        for (int t = grp; t < S; t += 4) s += src[(long long)t * R * C];
    }
    red[grp][cl] = s;
    __syncthreads();
    if (grp == 0 && idx < rn * C) {
        const double tot = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
        float* p = out + r * s_r + c * s_c;
        *p = accumulate ? *p + (float)tot : (float)tot;
    }
}

// ------------------------------------------------------------------------------------------------
// conv3x3, C_out = 1 (out.3):  eps[p] = b + sum_{tap,ci} z[p+tap][ci] * w[ci][tap]   (w == OIHW[0] flattened)
// One wave per 64 consecutive pixels; the C channels are split over 4 waves and reduced in LDS.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_cout1_fwd_kernel(const float* z, int ldz, int N, int H, int W, int C,
                                                             const float* w, const float* bias, float* out) {
    // lanes span channels (float4 each, coalesced 9 tap rows per pixel), per-lane 9x4 weights in
    // registers, per-pixel dot product folded over the C/4 lanes through LDS.
    __shared__ float part[256];
    const int C4 = C >> 2, PP = 256 / C4;
    const int c4 = (threadIdx.x % C4) * 4, pl = threadIdx.x / C4;
    float wr[9][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) wr[tap][j] = (pl < PP) ? w[(c4 + j) * 9 + tap] : 0.f;
    const long long P = (long long)N * H * W;
    for (long long base = (long long)blockIdx.x * PP; base < P; base += (long long)gridDim.x * PP) {
        const long long pix = base + pl;
        float s = 0.f;
        if (pl < PP && pix < P) {
            const int n = (int)(pix / (H * W)), rem = (int)(pix - (long long)n * H * W), h = rem / W, wx = rem - h * W;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int hh = h + tap / 3 - 1, ww = wx + tap % 3 - 1;
                if ((unsigned)hh >= (unsigned)H || (unsigned)ww >= (unsigned)W) continue;
                const float4 v = ld4(z + (((long long)n * H + hh) * W + ww) * ldz + c4);
                s = fmaf(v.x, wr[tap][0], s); s = fmaf(v.y, wr[tap][1], s);
                s = fmaf(v.z, wr[tap][2], s); s = fmaf(v.w, wr[tap][3], s);
            }
        }
        part[threadIdx.x] = s;
        __syncthreads();
        if (threadIdx.x < PP && base + threadIdx.x < P) {
            float acc = bias[0];
            for (int q = 0; q < C4; ++q) acc += part[threadIdx.x * C4 + q];
            out[base + threadIdx.x] = acc;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// image gradient of the init conv (ResidualConvBlock(1, nf, is_res) under autograd, diffusion_utilities.py:45-55):
//   dx[p] = sum_{tap,c} W1[c][8 - tap] dy1[p + tap][c]  (conv1's input gradient: the tap-flipped 3x3 conv, C_out = 1)
//         + sum_c scw[sel][c] gres[p][c]               (the random 1x1 shortcut's input gradient; sel = n >= split)
// dy1 = bn_bwd_elem(g1, y1, ...) of conv1's BatchNorm + ReLU, applied while reading (bn.y == nullptr: g1 is dy1).
// Same thread layout as conv_cout1_fwd_kernel: lanes over channels (float4), per-pixel sums folded through LDS.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_cin1_dgrad_kernel(const float* g1, int ldg, Cin1BnBwd bn, const float* w9,
                                                              const float* gres, int ldr, const float* scw, int split,
                                                              int N, int H, int W, int C, float* dx) {
    __shared__ float part[256];
    const int C4 = C >> 2, PP = 256 / C4;
    const int c4 = (threadIdx.x % C4) * 4, pl = threadIdx.x / C4;
    float wr[9][4], cf[7][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) wr[tap][j] = (pl < PP) ? w9[(c4 + j) * 9 + (8 - tap)] : 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) cf[k][j] = (bn.y && pl < PP) ? bn.p[k][c4 + j] : 0.f;
    const long long P = (long long)N * H * W;
    for (long long base = (long long)blockIdx.x * PP; base < P; base += (long long)gridDim.x * PP) {
        const long long pix = base + pl;
        float s = 0.f;
        if (pl < PP && pix < P) {
            const int n = (int)(pix / (H * W)), rem = (int)(pix - (long long)n * H * W), h = rem / W, wx = rem - h * W;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int hh = h + tap / 3 - 1, ww = wx + tap % 3 - 1;
                if ((unsigned)hh >= (unsigned)H || (unsigned)ww >= (unsigned)W) continue;
                const long long q = ((long long)n * H + hh) * W + ww;
                float4 v = ld4(g1 + q * ldg + c4);
                if (bn.y) {
                    const float4 yv = ld4(bn.y + q * bn.ldy + c4);
                    float gv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        gv[j] = bn_bwd_elem(gv[j], f4get(yv, j), cf[0][j], cf[1][j], cf[2][j], cf[3][j], cf[4][j],
                                            cf[5][j], cf[6][j]);
                    v = make_float4(gv[0], gv[1], gv[2], gv[3]);
                }
                s = fmaf(v.x, wr[tap][0], s); s = fmaf(v.y, wr[tap][1], s);
                s = fmaf(v.z, wr[tap][2], s); s = fmaf(v.w, wr[tap][3], s);
            }
            if (gres) {
                const float* sw = scw + (n >= split ? C : 0) + c4;
                const float4 r = ld4(gres + pix * ldr + c4);
                s = fmaf(r.x, sw[0], s); s = fmaf(r.y, sw[1], s); s = fmaf(r.z, sw[2], s); s = fmaf(r.w, sw[3], s);
            }
        }
        part[threadIdx.x] = s;
        __syncthreads();
        if (threadIdx.x < PP && base + threadIdx.x < P) {
            float acc = 0.f;
            for (int q = 0; q < C4; ++q) acc += part[threadIdx.x * C4 + q];
            dx[base + threadIdx.x] = acc;
        }
        __syncthreads();
    }
}

// Band form (W | 256, C % 16 == 0): a block owns R = 256/W whole output rows of one image.  The R + 2 input
// rows of the band are staged through LDS 16 channels at a time (coalesced 64-byte pixel pieces); each thread
// reduces its halo pixels to the 9 per-tap partial sums s[tap][q] = sum_c z[q][c] w[c][tap] (the weights are
// wave-uniform: scalar loads), and every output pixel then adds its 9 neighbours' partials.  z is read from
// HBM once (+2/R halo rows) instead of 9 times through the caches.
// gs / gt (optional, per (sample, channel) [N][C]): the input is relu(z gs + gt) of the pre-norm z (out.1's GroupNorm +
// ReLU applied while staging, the fmaf of norm_apply_fwd: bit-identical to the applied tensor; padding stays zero)
// HPM: halo pixels the LDS images hold, (R + 2) W rounded up to 64: 384 for W <= 64 (40 KiB of LDS, 4 blocks per CU;
// the W-independent 768-pixel images took 80 KiB, 2 blocks per CU, half the loads in flight: 2.3 TB/s), 512 for W = 128,
// 768 for W = 256
// FULL = false (default): 256 threads, up to HPM / 256 halo pixels per thread in the tap reduction (at 384 pixels the
// SIMDs holding waves 0-1 do twice the FMAs of the others).  FULL ($CDM_COUT1_FULL=1): HPM threads, one halo pixel
// each — balanced SIMDs, but same-box 182 vs 164 us per C2 step (profiles/r4_ab_cout1_threads.txt)
// SL: channels per LDS slab, 16 (default) or 32 ($CDM_COUT1_SLAB=32, C % 32 == 0: a pixel's slab piece is then one
// whole 128-byte line — measured no faster, 144-149 vs 137-160 us at the bench shape, profiles/r5_cout1_probe.jsonl).
// The tap partials st alias the slab image once the last slab is reduced (LDS 26 KiB at SL = 16).
template <int HPM, bool FULL = true, int SL = 16>
__global__ __launch_bounds__(FULL ? HPM : 256) void conv_cout1_fwd_band_kernel(const float* __restrict__ z, int ldz, int H, int W,
                                                                  int C, const float* __restrict__ w,
                                                                  const float* __restrict__ bias,
                                                                  float* __restrict__ out,
                                                                  const float* __restrict__ gs,
                                                                  const float* __restrict__ gt) {
    constexpr int NTHR = FULL ? HPM : 256;
    constexpr int KQ = (HPM + NTHR - 1) / NTHR;       // halo pixels per thread in the tap reduction
    constexpr int PPX = SL / 4;                       // float4 pieces per halo pixel and slab
    constexpr int ZT = HPM * (SL + 1), STN = 9 * HPM;
    __shared__ float sm[ZT > STN ? ZT : STN];
    float* zt = sm;                                   // [halo px][SL ch + 1 pad]
    float* st = sm;                                   // [tap][halo px] (after the slab loop)
    const int R = 256 / W, HP = (R + 2) * W;
    // XCD-contiguous band order: the bands of an image run on one XCD, so the halo rows a band shares with its
    // neighbours come from that XCD's L2 (round-robin order fetched 1.68x the algorithmic bytes)
    const int L = xcd_logical_block();
    const int bands = H / R, n = L / bands, h0 = (L - n * bands) * R;
    const int tid = threadIdx.x;
    float acc[KQ][9];
#pragma unroll
    for (int k = 0; k < KQ; ++k)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[k][t] = 0.f;
    // staging: piece i of this thread = (halo pixel q4 / PPX, channels 4 (q4 % PPX)..+3) of the current slab;
    // the next slabs' pieces are loaded into registers while this slab is reduced
    constexpr int PQ = HPM * PPX / NTHR;              // HPM * PPX pieces over the threads
    const float* src[PQ];
#pragma unroll
    for (int i = 0; i < PQ; ++i) {
        const int q4 = tid + i * NTHR, q = q4 / PPX, part = q4 % PPX;
        const int hh = h0 - 1 + q / W, ww = q - (q / W) * W;
        src[i] = (q < HP && (unsigned)hh < (unsigned)H) ? z + (((long long)n * H + hh) * W + ww) * ldz + part * 4
                                                        : nullptr;
    }
    // two register sets: the slab two ahead is in flight while one slab is reduced (round 5: one slab of look-ahead
    // left each block waiting on its loads once per slab, 3.3 TB/s on the C2 out.3 forward)
    float4 pre[2][PQ];
    auto gload = [&](float4 (&dst)[PQ], int c0) {
#pragma unroll
        for (int i = 0; i < PQ; ++i) dst[i] = src[i] ? ld4(src[i] + c0) : f4zero();
    };
    auto slab = [&](const float4 (&cur)[PQ], float4 (&nxt)[PQ], int c0) {
        float ks[4] = {1.f, 1.f, 1.f, 1.f}, kt[4] = {0.f, 0.f, 0.f, 0.f};
        if (gs) {   // this thread's 4 channels (q4 % PPX == tid % PPX for every piece)
            const int cb = n * C + c0 + (tid % PPX) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) { ks[j] = gs[cb + j]; kt[j] = gt[cb + j]; }
        }
#pragma unroll
        for (int i = 0; i < PQ; ++i) {
            const int q4 = tid + i * NTHR;
            if (q4 / PPX < HP) {
                float v[4] = {cur[i].x, cur[i].y, cur[i].z, cur[i].w};
                if (gs && src[i]) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = relu_f(fmaf(v[j], ks[j], kt[j]));
                }
                float* d = zt + (q4 / PPX) * (SL + 1) + (q4 % PPX) * 4;
                d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3];
            }
        }
        __syncthreads();
        if (c0 + 2 * SL < C) gload(nxt, c0 + 2 * SL);    // cur's registers are free: the slab after next
#pragma unroll
        for (int k = 0; k < KQ; ++k) {
            const int q = tid + k * NTHR;
            if (q < HP) {
#pragma unroll
                for (int c = 0; c < SL; ++c) {
                    const float v = zt[q * (SL + 1) + c];
                    // taps in pairs on the packed fp32 FMA (v_pk_fma_f32: the same fmaf per element, half the
                    // VALU issue; the reduction is VALU-bound on the SIMDs whose waves hold two halo pixels)
                    const float* wc = w + (c0 + c) * 9;
#pragma unroll
                    for (int t = 0; t < 8; t += 2) {
                        const f32x2 r = __builtin_elementwise_fma(f32x2{v, v}, f32x2{wc[t], wc[t + 1]},
                                                                  f32x2{acc[k][t], acc[k][t + 1]});
                        acc[k][t] = r[0]; acc[k][t + 1] = r[1];
                    }
                    acc[k][8] = fmaf(v, wc[8], acc[k][8]);
                }
            }
        }
        __syncthreads();
    };
    gload(pre[0], 0);
    if (SL < C) gload(pre[1], SL);
    for (int c0 = 0; c0 < C; c0 += 2 * SL) {   // C % SL == 0 (host check)
        slab(pre[0], pre[0], c0);
        if (c0 + SL < C) slab(pre[1], pre[1], c0 + SL);
    }
#pragma unroll
    for (int k = 0; k < KQ; ++k) {
        const int q = tid + k * NTHR;
        if (q < HP) {
#pragma unroll
            for (int t = 0; t < 9; ++t) st[t * HP + q] = acc[k][t];
        }
    }
    __syncthreads();
    // output pixel (h0 + r, c): sum over taps of the partial of halo pixel (r + ky, c + kx - 1)
    if (FULL && tid >= 256) return;
    const int r = tid / W, c = tid - r * W;
    float o = bias[0];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int cc = c + kx - 1;
            if ((unsigned)cc < (unsigned)W) o += st[(ky * 3 + kx) * HP + (r + ky) * W + cc];
        }
    out[((long long)n * H + h0 + r) * W + c] = o;
}

// dz[p'][ci] = sum_tap deps[p' - tap + 1] * w[ci][tap]   (lanes span channels, deps taps broadcast)
__global__ __launch_bounds__(256) void conv_cout1_dgrad_kernel(const float* deps, int N, int H, int W, int C,
                                                               const float* w, float* dz, int lddz) {
    const int C4 = C >> 2, PP = 256 / C4;
    const int c4 = (threadIdx.x % C4) * 4, pl = threadIdx.x / C4;
    if (pl >= PP) return;
    float wr[9][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) wr[tap][j] = w[(c4 + j) * 9 + tap];
    const long long P = (long long)N * H * W;
    constexpr int U = 4;   // U pixels per thread and iteration, all 9 U deps taps in flight together (as conv_cin1_fwd)
    const long long step = (long long)gridDim.x * PP;
    for (long long pix0 = (long long)blockIdx.x * PP + pl; pix0 < P; pix0 += step * U) {
        float gv[U][9];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long pix = pix0 + u * step;
            const int n = (int)(pix / (H * W)), rem = (int)(pix - (long long)n * H * W), h = rem / W, wx = rem - h * W;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int hh = h - (tap / 3 - 1), ww = wx - (tap % 3 - 1);
                gv[u][tap] = (pix < P && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                                 ? deps[((long long)n * H + hh) * W + ww] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long pix = pix0 + u * step;
            if (pix >= P) break;
            float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int j = 0; j < 4; ++j) o[j] = fmaf(gv[u][tap], wr[tap][j], o[j]);
            st4(dz + pix * lddz + c4, make_float4(o[0], o[1], o[2], o[3]));
        }
    }
}

// row form of conv_cout1_dgrad_kernel (as conv_cin1_fwd_row_kernel): deps rows h+1, h, h-1 of image n in LDS
__global__ __launch_bounds__(256) void conv_cout1_dgrad_row_kernel(const float* __restrict__ deps, int H, int W, int C,
                                                                   const float* __restrict__ w, float* __restrict__ dz,
                                                                   int lddz) {
    extern __shared__ float gs[];   // [3][W + 2]: gs[r][col] = deps[h + 1 - r][col - 1]
    const int n = blockIdx.x / H, h = blockIdx.x - n * H, WP = W + 2;
    const int C4 = C >> 2, PP = 256 / C4;
    const int c4 = (threadIdx.x % C4) * 4, pl = threadIdx.x / C4;
    const bool active = pl < PP;
    // weights and the source rows requested together (one memory round trip before the barrier, not two)
    const int cw = active ? c4 : 0;
    float wr[9][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) wr[tap][j] = w[(cw + j) * 9 + tap];
    for (int i = threadIdx.x; i < 3 * WP; i += 256) {
        const int r = i / WP, col = i - r * WP, hh = h + 1 - r, ww = col - 1;
        const bool in = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        const float v = deps[in ? ((long long)n * H + hh) * W + ww : 0];
        gs[i] = in ? v : 0.f;
    }
    __syncthreads();
    float* dr = dz + ((long long)n * H + h) * W * lddz;
    for (int x = active ? pl : W; x < W; x += PP) {
        float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            // deps[h - (ky - 1)][x - (kx - 1)] = gs[ky][x + 2 - kx]
            const float gv = gs[(tap / 3) * WP + x + 2 - tap % 3];
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = fmaf(gv, wr[tap][j], o[j]);
        }
        st4(dr + (long long)x * lddz + c4, make_float4(o[0], o[1], o[2], o[3]));
    }
}

// out.3 weight gradient, band form: dW[c][tap] = sum_p deps[p] z[p + off_tap][c] = sum_q z[q][c] deps[q - off_tap].
// A block owns R whole rows of one image; every z pixel q of the band is read from HBM once (float4 per lane,
// C/4 lanes per pixel: one coalesced row), and its 9 contributions use the deps values around it, staged with a
// zero border in LDS (no bounds tests).  Per-block partials [9][C] (fixed-order LDS fold over the pixel lanes).
// gs / gt (optional, per (sample, channel) [N][C]): z = relu(y gs + gt) of the pre-norm y (out.1's GroupNorm + ReLU,
// the fmaf of norm_apply_fwd: bit-identical to the applied tensor) — z is then never written by the forward
__global__ __launch_bounds__(256) void conv_cout1_wgrad_band_kernel(const float* __restrict__ deps,
                                                                    const float* __restrict__ z, int ldz, int H, int W,
                                                                    int C, int R, float* __restrict__ slab,
                                                                    const float* __restrict__ gs,
                                                                    const float* __restrict__ gt) {
    extern __shared__ float sm[];                        // deps band [(R+2)][(W+2)], then the fold [PL][9][C]
    const int bands = H / R, n = blockIdx.x / bands, h0 = (blockIdx.x - n * bands) * R;
    const int C4 = C >> 2, PL = 256 / C4, tid = threadIdx.x, c4 = (tid % C4) * 4, pl = tid / C4;
    const int DW = W + 2, DN = (R + 2) * DW;
    float* dl = sm;
    float* red = sm + ((DN + 3) & ~3);
    for (int i = tid; i < DN; i += 256) {
        const int rr = i / DW, cc = i - rr * DW, hh = h0 - 1 + rr, ww = cc - 1;
        dl[i] = ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) ? deps[((long long)n * H + hh) * W + ww] : 0.f;
    }
    __syncthreads();
    float acc[9][4];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[t][j] = 0.f;
    float ks[4] = {1.f, 1.f, 1.f, 1.f}, kt[4] = {0.f, 0.f, 0.f, 0.f};
    if (gs) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { ks[j] = gs[n * C + c4 + j]; kt[j] = gt[n * C + c4 + j]; }
    }
    if (pl < PL) {
        const float* zb = z + ((long long)n * H + h0) * W * ldz + c4;
        for (int q = pl; q < R * W; q += PL) {
            const int r = q / W, c = q - r * W;
            float4 v = ld4(zb + (long long)q * ldz);
            if (gs) {
                v.x = relu_f(fmaf(v.x, ks[0], kt[0])); v.y = relu_f(fmaf(v.y, ks[1], kt[1]));
                v.z = relu_f(fmaf(v.z, ks[2], kt[2])); v.w = relu_f(fmaf(v.w, ks[3], kt[3]));
            }
            // output pixel p = q - off, off = (ky - 1, kx - 1): deps at band row r + 2 - ky, column c + 2 - kx
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const float g = dl[(r + 2 - ky) * DW + (c + 2 - kx)];
                    const int t = ky * 3 + kx;
                    acc[t][0] = fmaf(g, v.x, acc[t][0]); acc[t][1] = fmaf(g, v.y, acc[t][1]);
                    acc[t][2] = fmaf(g, v.z, acc[t][2]); acc[t][3] = fmaf(g, v.w, acc[t][3]);
                }
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) st4(&red[(pl * 9 + t) * C + c4], make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]));
    }
    __syncthreads();
    float* out = slab + (long long)blockIdx.x * 9 * C;
    for (int idx = tid; idx < 9 * C; idx += 256) {
        float s = 0.f;
        for (int q = 0; q < PL; ++q) s += red[q * 9 * C + idx];
        out[idx] = s;
    }
}

// partials R = 9: r = tap: sum_p deps[p] * z[p+tap][c]
__global__ __launch_bounds__(256) void conv_cout1_wgrad_kernel(const float* deps, const float* z, int ldz, int H,
                                                               int W, int C, int csize, float* slab) {
    constexpr int R = 9;
    __shared__ float red[256 * 4 * R];
    const int C4 = C >> 2, P = 256 / C4, tid = threadIdx.x, c4 = (tid % C4) * 4, pl = tid / C4;
    const int n = blockIdx.y, chunk = blockIdx.x, HW = H * W;
    const int p0 = chunk * csize, p1 = min(HW, p0 + csize);
    float acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[r][j] = 0.f;
    if (pl < P) {
        for (int p = p0 + pl; p < p1; p += P) {
            const int h = p / W, w = p - h * W;
            const float g = deps[(long long)n * HW + p];
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int hh = h + tap / 3 - 1, ww = w + tap % 3 - 1;
                if ((unsigned)hh >= (unsigned)H || (unsigned)ww >= (unsigned)W) continue;
                const float4 v = ld4(z + ((long long)n * HW + hh * W + ww) * ldz + c4);
                acc[tap][0] += g * v.x; acc[tap][1] += g * v.y; acc[tap][2] += g * v.z; acc[tap][3] += g * v.w;
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) st4(&red[(pl * R + r) * C + c4], make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]));
    }
    __syncthreads();
    float* out = slab + ((long long)n * gridDim.x + chunk) * R * C;
    for (int idx = tid; idx < R * C; idx += 256) {
        float s = 0.f;
        for (int q = 0; q < P; ++q) s += red[q * R * C + idx];
        out[idx] = s;
    }
}

// ------------------------------------------------------------------------------------------------
// AvgPool2d(h/4) + GELU
// ------------------------------------------------------------------------------------------------
__global__ void avgpool_gelu_fin_kernel(const float* sums, int N, int C, float inv_hw, float* hpre, float* hv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * C) return;
    const float m = sums[i] * inv_hw;
    hpre[i] = m; hv[i] = (float)gelu_d((double)m);   // GELU rounded once (see embed_fwd_kernel)
}
// dst[n,p,c] += dhv[n][c] * gelu'(hpre[n][c]) / HW
__global__ void avgpool_gelu_bwd_kernel(const float* dhv, const float* hpre, int N, int HW, int C, float inv_hw,
                                       float* dst, int ldd) {
    const int C4 = C >> 2;
    const long long total = (long long)N * HW * C4;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int c4 = (int)(idx % C4) * 4;
        const long long pix = idx / C4;
        const int n = (int)(pix / HW);
        float4 d = ld4(dst + pix * ldd + c4);
        float v[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = n * C + c4 + j;
            v[j] += dhv[k] * gelu_grad_f(hpre[k]) * inv_hw;
        }
        st4(dst + pix * ldd + c4, make_float4(v[0], v[1], v[2], v[3]));
    }
}

// ------------------------------------------------------------------------------------------------
// EmbedFC x4:  out = W2 gelu(W1 x + b1) + b2    (one launch for all four MLPs)
// ------------------------------------------------------------------------------------------------
struct MlpDesc {
    const float* x; int rows; int in_dim; int E;
    const float* w1; const float* b1; const float* w2; const float* w2t; const float* b2;
    float* pre; float* h; float* out;
    const float* dout; float* dpre; float* dw1; float* db1; float* dw2; float* db2;
};
struct Mlp4 { MlpDesc m[4]; };

// Evaluated in fp64 and rounded once (the embeddings are a few thousand values per step): the same inputs give the
// same embedding at every step of a sampling run (c is fixed, t moves slowly), so any rounding bias of an fp32
// evaluation is repeated 1500 times and accumulates coherently along the trajectory; rounded once, the embedding
// is within half an ulp of the exact value (tools/t1500_steps.py: the fp32 kernel's c / t embedding errors were 1.7x /
// 6.6x the reference's, coherent over the run).  pre / h (kept for the backward) are the rounded fp64 values.
__global__ __launch_bounds__(256) void embed_fwd_kernel(Mlp4 P) {
    const MlpDesc& d = P.m[blockIdx.y];
    const int b = blockIdx.x;
    if (b >= d.rows) return;
    __shared__ double hs[1024];
    for (int j = threadIdx.x; j < d.E; j += 256) {
        double s = d.b1[j];
        for (int k = 0; k < d.in_dim; ++k) s = fma((double)d.w1[j * d.in_dim + k], (double)d.x[b * d.in_dim + k], s);
        const double g = gelu_d(s);
        if (d.pre) { d.pre[(long long)b * d.E + j] = (float)s; d.h[(long long)b * d.E + j] = (float)g; }
        hs[j] = g;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < d.E; j += 256) {
        double s = d.b2[j];
        for (int i = 0; i < d.E; ++i) s = fma((double)d.w2t[(long long)i * d.E + j], hs[i], s);
        d.out[(long long)b * d.E + j] = (float)s;
    }
}

// dpre[b][i] = gelu'(pre[b][i]) * sum_j dout[b][j] w2[j][i]
__global__ __launch_bounds__(256) void embed_bwd_act_kernel(Mlp4 P) {
    const MlpDesc& d = P.m[blockIdx.y];
    const int b = blockIdx.x;
    if (b >= d.rows) return;                       // block-uniform
    __shared__ float drow[1024];                   // dout row b (E <= 1024, checked by cdm_embed_bwd)
    for (int j = threadIdx.x; j < d.E; j += 256) drow[j] = d.dout[(long long)b * d.E + j];
    __syncthreads();
    for (int i = threadIdx.x; i < d.E; i += 256) {
        float s = 0.f;
        // same sequential fma chain as before; unrolled so the w2 loads of 8 steps are in flight together
#pragma unroll 8
        for (int j = 0; j < d.E; ++j) s = fmaf(drow[j], d.w2[(long long)j * d.E + i], s);
        d.dpre[(long long)b * d.E + i] = s * gelu_grad_f(d.pre[(long long)b * d.E + i]);
    }
}

// parameter grads (assign): dw2[j][i], db2[j], dw1[i][k], db1[i]; each a sequential fp64 sum over the rows (the
// product of two fp32 values is exact in fp64, so fma and multiply-add give the same bits).  dw2 (E x E outputs, the
// bulk) in 64 x 64 tiles: the block stages 64 rows of dout and h through LDS and each thread carries 4 x 4 outputs, 16
// independent fp64 chains (the per-output form waited on one global load per row: 40 us per C2 step, latency-bound);
// blocks past the tiles take db2, dw1, db1 one output per thread.  30 us per C2 step; 32 x 32 tiles (160 blocks, 4
// chains per thread) measured 67 us (fp64 FMA latency with a quarter of the chains, profiles/r4_train_step_*).
constexpr int EMB_T = 64;
static __host__ __device__ inline int embed_tiles(int E) { return ((E + EMB_T - 1) / EMB_T) * ((E + EMB_T - 1) / EMB_T); }
__global__ __launch_bounds__(256) void embed_bwd_param_kernel(Mlp4 P) {
    const MlpDesc& d = P.m[blockIdx.y];
    const int E = d.E, I = d.in_dim, rows = d.rows;
    const int nt = embed_tiles(E);
    const int tid = threadIdx.x;
    if ((int)blockIdx.x < nt) {
        __shared__ __attribute__((aligned(16))) float ds_[EMB_T][EMB_T], hs_[EMB_T][EMB_T];
        const int tpr = (E + EMB_T - 1) / EMB_T;
        const int j0 = (blockIdx.x / tpr) * EMB_T, i0 = (blockIdx.x % tpr) * EMB_T;
        const int tj = (tid >> 4) * 4, ti = (tid & 15) * 4;
        double s[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) s[a][c] = 0.0;
        for (int b0 = 0; b0 < rows; b0 += EMB_T) {
            const int nb = min(EMB_T, rows - b0);
            // the chunk's 2 x 16 loads per thread issued together (then stored): one memory latency per chunk
            float dv_[EMB_T * EMB_T / 256], hv_[EMB_T * EMB_T / 256];
#pragma unroll
            for (int u = 0; u < EMB_T * EMB_T / 256; ++u) {
                const int q = tid + u * 256, r = q / EMB_T, c = q - r * EMB_T;
                const bool ok = r < nb;
                dv_[u] = ok && j0 + c < E ? d.dout[(long long)(b0 + r) * E + j0 + c] : 0.f;
                hv_[u] = ok && i0 + c < E ? d.h[(long long)(b0 + r) * E + i0 + c] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < EMB_T * EMB_T / 256; ++u) {
                const int q = tid + u * 256, r = q / EMB_T, c = q - r * EMB_T;
                ds_[r][c] = dv_[u];
                hs_[r][c] = hv_[u];
            }
            __syncthreads();
            for (int r = 0; r < nb; ++r) {
                const float4 dv = *reinterpret_cast<const float4*>(&ds_[r][tj]);
                const float4 hv = *reinterpret_cast<const float4*>(&hs_[r][ti]);
                const double dd[4] = {dv.x, dv.y, dv.z, dv.w}, hh[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int c = 0; c < 4; ++c) s[a][c] = fma(dd[a], hh[c], s[a][c]);
            }
            __syncthreads();
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int j = j0 + tj + a, i = i0 + ti + c;
                if (j < E && i < E) d.dw2[(long long)j * E + i] = (float)s[a][c];
            }
        return;
    }
    const long long n_rest = (long long)E + (long long)E * I + E;
    const long long idx = (long long)(blockIdx.x - nt) * blockDim.x + tid;
    if (idx >= n_rest) return;
    double s = 0.0;
    if (idx < E) {
        const int j = (int)idx;
#pragma unroll 32
        for (int b = 0; b < rows; ++b) s += d.dout[(long long)b * E + j];
        d.db2[j] = (float)s;
    } else if (idx < E + (long long)E * I) {
        const long long q = idx - E;
        const int i = (int)(q / I), k = (int)(q - (long long)i * I);
#pragma unroll 32
        for (int b = 0; b < rows; ++b) s += (double)d.dpre[(long long)b * E + i] * d.x[b * I + k];
        d.dw1[q] = (float)s;
    } else {
        const int i = (int)(idx - E - (long long)E * I);
#pragma unroll 32
        for (int b = 0; b < rows; ++b) s += d.dpre[(long long)b * E + i];
        d.db1[i] = (float)s;
    }
}

// input gradient of two EmbedFCs fed the same input (timeembed1/2 by t, contextembed1/2 by c; ContextUnet.py:51-54):
// dx[b][k] = sum_i dpre_a[b][i] w1_a[i][k] + sum_i dpre_b[b][i] w1_b[i][k]   (one thread per (b, k), sequential fp32)
__global__ __launch_bounds__(256) void embed_input_grad_kernel(const float* dpre_a, const float* w1_a, int Ea,
                                                               const float* dpre_b, const float* w1_b, int Eb, int rows,
                                                               int in_dim, float* dx) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * in_dim) return;
    const int b = idx / in_dim, k = idx - b * in_dim;
    float s = 0.f;
    for (int i = 0; i < Ea; ++i) s = fmaf(dpre_a[(long long)b * Ea + i], w1_a[i * in_dim + k], s);
    float s2 = 0.f;
    for (int i = 0; i < Eb; ++i) s2 = fmaf(dpre_b[(long long)b * Eb + i], w1_b[i * in_dim + k], s2);
    dx[idx] = s + s2;
}

// ------------------------------------------------------------------------------------------------
// diffusion elementwise math
// ------------------------------------------------------------------------------------------------
// x_pert = sqrt(ab[t]) x + (1 - ab[t]) noise ; temb_in = float(t)/float(T)
// t per sample (t != NULL) or one device-side step index (*cur_i) for the whole batch; in the latter case the
// noise is row (T - i) of a table with row stride nstride (nstride = 0: a single noise buffer).
// `omab` may be any noise-coefficient table (the paper ELBO uses sqrt(1 - ab)).
__global__ void perturb_kernel(const float* x, const float* noise, const int* t, const int* cur_i, long long nstride,
                               const float* sab, const float* omab, int N, int HW, int T, float* out, float* tin) {
#pragma clang fp contract(off)  // keep the reference's separate fp32 roundings (bit-exact)
    const long long total = (long long)N * HW;
    const int ci = cur_i ? *cur_i : 0;
    const float* nz = cur_i ? noise + (long long)(T - ci) * nstride : noise;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const int n = (int)(i / HW);
        const int ti = cur_i ? ci : t[n];
        out[i] = sab[ti] * x[i] + omab[ti] * nz[i];
        if (tin && i - (long long)n * HW == 0) tin[n] = (float)ti / (float)T;
    }
}

// acc[n] += (mean_p (pred - noise)^2 * mul[i]) / div[i]   i = t[n] (per-sample steps) or *cur_i; one block per
// sample, fixed reduction order (deterministic)
// NLL term (code/train_diffusion_elbo.py:133-141): mul = 1, div = 2 b_t;  paper ELBO (:112-125): mul = w_t, div = 10
__global__ __launch_bounds__(256) void mse_accum_kernel(const float* pred, const float* noise, long long nstride, int T,
                                                        int HW, const int* t, const int* cur_i, const float* mul,
                                                        const float* div, float* acc) {
#pragma clang fp contract(off)
    const int n = blockIdx.x, i = t ? t[n] : *cur_i;
    const float* nz = t ? noise : noise + (long long)(T - i) * nstride;
    float s = 0.f;
    for (int p = threadIdx.x; p < HW; p += 256) {
        const float d = pred[(long long)n * HW + p] - nz[(long long)n * HW + p];
        s += d * d;
    }
    __shared__ float red[4];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float mse = (red[0] + red[1] + red[2] + red[3]) / (float)HW;
        acc[n] += (mse * mul[i]) / div[i];
    }
}

// per-block partials: [0] sum (pred-noise)^2, [1] sum dpred ; dpred = 2(pred-noise)/numel
__global__ __launch_bounds__(256) void mse_kernel(const float* pred, const float* noise, long long n, float scale,
                                                  float* dpred, float* partial) {
    float s0 = 0.f, s1 = 0.f;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float d = pred[i] - noise[i];
        const float g = d * scale;
        dpred[i] = g;
        s0 += d * d; s1 += g;
    }
    __shared__ float r0[4], r1[4];
    s0 = wave_sum(s0); s1 = wave_sum(s1);
    if ((threadIdx.x & 63) == 0) { r0[threadIdx.x >> 6] = s0; r1[threadIdx.x >> 6] = s1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[blockIdx.x * 2 + 0] = r0[0] + r0[1] + r0[2] + r0[3];
        partial[blockIdx.x * 2 + 1] = r1[0] + r1[1] + r1[2] + r1[3];
    }
}
// loss = sum0 / numel (written to loss_out), dbias = sum1 (written to dbias_out); nonfinite (optional) counts
// the steps whose loss is NaN / inf (the trainer's failure guard, read once per epoch: no per-step host sync)
__global__ void mse_finalize_kernel(const float* partial, int nb, double inv_numel, float* loss_out, float* dbias_out,
                                    int* nonfinite) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double a = 0.0, b = 0.0;
    for (int i = 0; i < nb; ++i) { a += partial[2 * i]; b += partial[2 * i + 1]; }
    const float loss = (float)(a * inv_numel);
    if (loss_out) *loss_out = loss;
    if (dbias_out) *dbias_out = (float)b;
    if (nonfinite && !isfinite(loss)) *nonfinite += 1;
}

// Sampler step prologue (device-side step counter, so one captured step replays for every i):
//   i = *ctr; *ctr = i - 1; cur[0] = i; t_cur = (float)((double)i / T); shortcut rows for step i.
__global__ void sample_prologue_kernel(int* ctr, int T, int* cur_i, float* t_cur, const float* sc_table, int sc_row,
                                       float* sc_cur) {
    const int i = *ctr;
    __syncthreads();
    if (threadIdx.x == 0) { *ctr = i - 1; *cur_i = i; *t_cur = (float)((double)i / (double)T); }
    if (sc_table)
        for (int k = threadIdx.x; k < sc_row; k += blockDim.x) sc_cur[k] = sc_table[(long long)(T - i) * sc_row + k];
}

// x <- (x - eps*coef[i]) / sa[i] + sb[i]*z ;  eps = eu + w (ec - eu) when cfg (model batch = 2n)
// z = 0 at i == 1; z from z_table[(T-i)][e] when given, else Philox(seed, stream i).
// Writes x into both halves of the model-input buffer (x2 may alias x), and a snapshot when slot[i] >= 0.
__global__ void denoise_kernel(const float* xin, float* x, float* x2, long long numel, const float* eps, int cfg,
                               float w, const int* cur_i, const float* coef, const float* sa, const float* sb,
                               const float* z_table, long long zstride, unsigned long long seed,
                               const long long* seed_dev, const int* snap_slot, float* snaps, int T) {
#pragma clang fp contract(off)  // keep the reference's separate fp32 roundings (bit-exact)
    const int i = *cur_i;
    const float cf = coef[i], a = sa[i], b = sb[i];
    const int slot = snap_slot ? snap_slot[i] : -1;
    // per-run key: seed ^ *seed_dev (drawn from torch's CUDA generator before every run, so consecutive sampling
    // calls get fresh z, as the reference's randn_like on the device does)
    const unsigned long long sd = seed_dev ? seed ^ (unsigned long long)seed_dev[0] : seed;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < numel; e += (long long)gridDim.x * blockDim.x) {
        float ep = eps[e];
        if (cfg) { const float eu = eps[numel + e]; ep = eu + w * (ep - eu); }
        float z = 0.f;
        if (i > 1) z = z_table ? z_table[(long long)(T - i) * zstride + e] : philox_normal(sd, (uint32_t)i, e);
        const float mean = (xin[e] - ep * cf) / a;   // same op order / roundings as the reference
        const float v = mean + b * z;
        x[e] = v;
        if (x2) { x2[e] = v; x2[numel + e] = v; }
        if (slot >= 0) snaps[(long long)slot * numel + e] = v;
    }
}

// ------------------------------------------------------------------------------------------------
// Adam = torch.optim.Adam's single-tensor step (torch/optim/adam.py _single_tensor_adam, the path the
// reference's CPU run takes; code/train_diffusion_condition.py:200,229), with lr / step in device memory so
// a captured step replays.
// state (double[4]): [0] lr (a Python float, as torch keeps it), [1] step count, [2] -step_size rounded to
//                    fp32, [3] sqrt(bias_correction2) rounded to fp32
// bc (double[nbc][2]): 1 - beta1**step and (1 - beta2**step)**0.5 for step = 1..nbc, evaluated on the host
//                    with torch's own Python-double expressions (the last row is exactly {1, 1}; steps past
//                    nbc reuse it, which is exact since both powers have underflowed below 2^-54 there)
// Elementwise roundings follow torch's CPU kernels (probed against torch 2.10 AVX-512):
//   exp_avg.lerp_(g, 1-b1)           lerp_vec: fmadd(w, g - m, m)                 -> one fma
//   exp_avg_sq.mul_(b2)              v * float(b2)
//              .addcmul_(g, g, 1-b2)   self + (c * g) * g, contracted to fma(c*g, g, self)
//   denom = sqrt(v) / bc2s + eps     div by the fp32-cast scalar, add (alpha = 1)
//   param.addcdiv_(m, denom, -ss)    self + (value * m) / denom
// The one deliberate difference: sqrtf here is correctly rounded; torch's vectorised CPU sqrt is not always
// (<= 1 ulp), so p differs from torch CPU by <= 1 ulp of the update on those elements (test_gpu_trainer.py).
// ------------------------------------------------------------------------------------------------
__global__ void adam_prep_kernel(double* state, const double* bc, int nbc) {
    const double step = state[1] + 1.0;
    state[1] = step;
    const int k = (int)(step < (double)nbc ? step : (double)nbc) - 1;
    state[2] = (double)(float)(-(state[0] / bc[2 * k]));     // value=-step_size, Scalar -> float
    state[3] = (double)(float)bc[2 * k + 1];                  // bias_correction2_sqrt, wrapped scalar -> float
}
__global__ void adam_kernel(float* p, const float* g, float* m, float* v, long long n, const double* state, float beta1c,
                            float beta2, float beta2c, float eps, float gscale) {
#pragma clang fp contract(off)  // only the explicit fmaf below fuse, as in torch's CPU kernels
    const float nss = (float)state[2], bc2s = (float)state[3];
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float gi = g[i] * gscale;             // 1/world for the summed data-parallel gradient
        float mi = m[i];
        mi = fmaf(beta1c, gi - mi, mi);                   // exp_avg.lerp_(grad, 1 - beta1)
        float vi = v[i] * beta2;                          // exp_avg_sq.mul_(beta2)
        vi = fmaf(beta2c * gi, gi, vi);                   //   .addcmul_(grad, grad, 1 - beta2)
        const float denom = sqrtf(vi) / bc2s + eps;       // (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
        p[i] = p[i] + (nss * mi) / denom;                 // param.addcdiv_(exp_avg, denom, -step_size)
        m[i] = mi; v[i] = vi;
    }
}

// ------------------------------------------------------------------------------------------------
// weight packing
// ------------------------------------------------------------------------------------------------
// conv3x3 OIHW W[co][ci][tap] ->  wpk[(tap*Cin + ci)*Cout + co] (* fold[co]),  wdg[(tap*Cout+co)*Cin+ci] = W[co][ci][8-tap]
// fold (eval BN): s = gamma/sqrt(rv+eps), bpk = (b - rm)*s + beta
// kc > 0: channel-chunk-major K order k = ((ci/kc)*9 + tap)*kc + ci%kc  (must match LdIm2colA<.., KC>)
static __device__ __forceinline__ long long kidx(int tap, int ci, int C, int kc) {
    if (kc <= 0) return (long long)tap * C + ci;
    const int cc = ci / kc;
    return ((long long)cc * 9 + tap) * kc + (ci - cc * kc);
}
__global__ void pack_conv3x3_kernel(const float* W, const float* b, int Cin, int Cout, const float* gamma,
                                    const float* beta, const float* rm, const float* rv, float eps, float* wpk,
                                    float* bpk, float* wdg, int kc) {
    const long long total = (long long)Cout * Cin * 9;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int tap = (int)(idx % 9);
        const long long q = idx / 9;
        const int ci = (int)(q % Cin), co = (int)(q / Cin);
        const float wv = W[idx];
        float s = 1.f;
        if (gamma) s = gamma[co] / sqrtf(rv[co] + eps);
        if (wpk) wpk[kidx(tap, ci, Cin, kc) * Cout + co] = wv * s;
        if (wdg) wdg[kidx(8 - tap, co, Cout, kc) * Cin + ci] = wv;
        if (bpk && idx < Cout) {
            const int c = (int)idx;
            bpk[c] = gamma ? (b[c] - rm[c]) * (gamma[c] / sqrtf(rv[c] + eps)) + beta[c] : b[c];
        }
    }
}

// ConvTranspose weight W[ci][co][kk] ->  wt[ci][kk*Cout + co],  wtT[(kk*Cout + co)][ci]
// out[b][c][r] = in[b][r][c] for `batch` R x C matrices: 64 x 64 tiles through LDS (reads coalesced along c,
// writes along r; the +1 pad keeps the column reads conflict-free)
__global__ __launch_bounds__(256) void transpose_tiled_kernel(const float* __restrict__ in, long long R, long long C,
                                                              float* __restrict__ out) {
    __shared__ float t[64][65];
    const long long tilesC = (C + 63) / 64;
    const long long b = blockIdx.y;
    const long long r0 = (blockIdx.x / tilesC) * 64, c0 = (blockIdx.x % tilesC) * 64;
    const float* ib = in + b * R * C;
    float* ob = out + b * R * C;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const long long r = r0 + ty + 4 * k, c = c0 + tx;
        if (r < R && c < C) t[ty + 4 * k][tx] = ib[r * C + c];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const long long c = c0 + ty + 4 * k, r = r0 + tx;
        if (r < R && c < C) ob[c * R + r] = t[tx][ty + 4 * k];
    }
}

__global__ void pack_convT_kernel(const float* W, int Cin, int Cout, int KK, float* wt, float* wtT) {
    const long long total = (long long)Cin * Cout * KK;
    for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int kk = (int)(idx % KK);
        const long long q = idx / KK;
        const int co = (int)(q % Cout), ci = (int)(q / Cout);
        const float v = W[idx];
        const long long col = (long long)kk * Cout + co;
        if (wt) wt[(long long)ci * KK * Cout + col] = v;
        if (wtT) wtT[col * Cin + ci] = v;
    }
}

}  // namespace cdm

using namespace cdm;
static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------ C ABI ------------------------------------------------
CDM_API int cdm_philox_normal(float* out, long long n, unsigned long long seed, unsigned int sub, const int* sub_dev,
                              void* stream) {
    hipLaunchKernelGGL(philox_normal_kernel, dim3(nblocks((n + 3) / 4)), dim3(256), 0, S(stream), out, n, seed, sub, sub_dev);
    return cdm_status();
}
CDM_API int cdm_philox_uniform(float* out, long long n, float lo, float hi, unsigned long long seed, unsigned int sub,
                               const int* sub_dev, void* stream) {
    hipLaunchKernelGGL(philox_uniform_kernel, dim3(nblocks((n + 3) / 4)), dim3(256), 0, S(stream), out, n, lo, hi, seed, sub,
                       sub_dev);
    return cdm_status();
}
CDM_API int cdm_philox_randint(int* out, int n, int lo, int hi, unsigned long long seed, unsigned int sub,
                               const int* sub_dev, void* stream) {
    hipLaunchKernelGGL(philox_randint_kernel, dim3((n + 255) / 256), dim3(256), 0, S(stream), out, n, lo, hi, seed, sub,
                       sub_dev);
    return cdm_status();
}
static int row_kernels() {   // $CDM_ROW_KERNELS: 1 (default) the row forms of the C_in = 1 / C_out = 1 kernels, 0 flat
    static const int v = [] { const char* e = getenv("CDM_ROW_KERNELS"); return e ? atoi(e) : 1; }();
    return v;
}
CDM_API int cdm_conv3x3_cin1_fwd(const float* x, int N, int H, int W, const float* w9, const float* bias, float* y,
                                 int ldy, int C, int relu, float* amax, void* stream) {
    if (C % 4) return (int)hipErrorInvalidValue;
    if (C > 1024) return (int)hipErrorInvalidValue;
    const long long P = (long long)N * H * W;
    if (row_kernels() && W <= ROWK_MAXW && (long long)N * H <= 0x7fffffffll) {
        hipLaunchKernelGGL(conv_cin1_fwd_row_kernel, dim3((unsigned)(N * H)), dim3(256), 3 * (W + 2) * sizeof(float),
                           S(stream), x, H, W, w9, bias, y, ldy, C, relu, amax);
        return cdm_status();
    }
    hipLaunchKernelGGL(conv_cin1_fwd_kernel, dim3(nblocks(P, 256 / (C / 4), 4096)), dim3(256), 0, S(stream), x, N, H, W, w9,
                       bias, y, ldy, C, relu, amax);
    return cdm_status();
}
CDM_API int cdm_conv3x3_cin1_wgrad(const float* dy, int lddy, const float* x, int N, int H, int W, int C, int csize,
                                   float* slab, void* stream) {
    if (C % 4 || C > 1024) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(conv_cin1_wgrad_kernel<false>, dim3((H * W + csize - 1) / csize, N), dim3(256), 0, S(stream), dy,
                       lddy, x, H, W, C, csize, slab, Cin1BnBwd{});
    return cdm_status();
}
// cdm_conv3x3_cin1_wgrad of a Conv -> BatchNorm -> ReLU layer with its BN backward applied while reading dy: g = grad of
// the ReLU output, y = pre-norm activations, s / t / mean / invstd / A / B / Cc per channel (as cdm_norm_apply_bwd mode 0)
CDM_API int cdm_conv3x3_cin1_wgrad_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s,
                                         const float* t, const float* mean, const float* invstd, const float* A,
                                         const float* B, const float* Cc, const float* x, int N, int H, int W, int C,
                                         int csize, float* slab, void* stream) {
    if (C % 4 || C > 1024 || ldg % 4 || ldy % 4) return (int)hipErrorInvalidValue;
    const Cin1BnBwd bn{y, ldy, {s, t, mean, invstd, A, B, Cc}};
    hipLaunchKernelGGL(conv_cin1_wgrad_kernel<true>, dim3((H * W + csize - 1) / csize, N), dim3(256), 0, S(stream), g,
                       ldg, x, H, W, C, csize, slab, bn);
    return cdm_status();
}
CDM_API int cdm_slab_sum_all(const double* part, int nparts, int R, int r0, int rn, int C, float* out, long long s_r,
                             long long s_c, int accumulate, void* stream) {
    hipLaunchKernelGGL(slab_sum_all_kernel, dim3((rn * C + 63) / 64), dim3(256), 0, S(stream), part, nparts, R, r0, rn, C,
                       out, s_r, s_c, accumulate);
    return cdm_status();
}
static int launch_cout1_band(const float* z, int ldz, int N, int H, int W, int C, const float* w, const float* bias,
                             float* out, const float* gs, const float* gt, hipStream_t st) {
    const dim3 grid(N * (H / (256 / W)));
    const int hp = (256 / W + 2) * W;           // halo pixels of a band
    static const int full = [] { const char* e = getenv("CDM_COUT1_FULL"); return e ? atoi(e) : 0; }();
    // 32-channel slabs on request ($CDM_COUT1_SLAB=32, read per call for A/B tests; not for 768-pixel bands: spills)
    const char* sv = getenv("CDM_COUT1_SLAB");
    if (!full && C % 32 == 0 && hp <= 512 && sv && atoi(sv) == 32) {
        if (hp <= 384)
            hipLaunchKernelGGL((conv_cout1_fwd_band_kernel<384, false, 32>), grid, dim3(256), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
        else
            hipLaunchKernelGGL((conv_cout1_fwd_band_kernel<512, false, 32>), grid, dim3(256), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
        return cdm_status();
    }
    if (!full) {
        if (hp <= 384)
            hipLaunchKernelGGL((conv_cout1_fwd_band_kernel<384, false>), grid, dim3(256), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
        else if (hp <= 512)
            hipLaunchKernelGGL((conv_cout1_fwd_band_kernel<512, false>), grid, dim3(256), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
        else
            hipLaunchKernelGGL((conv_cout1_fwd_band_kernel<768, false>), grid, dim3(256), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
        return cdm_status();
    }
    if (hp <= 384)
        hipLaunchKernelGGL(conv_cout1_fwd_band_kernel<384>, grid, dim3(384), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
    else if (hp <= 512)
        hipLaunchKernelGGL(conv_cout1_fwd_band_kernel<512>, grid, dim3(512), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
    else
        hipLaunchKernelGGL(conv_cout1_fwd_band_kernel<768>, grid, dim3(768), 0, st, z, ldz, H, W, C, w, bias, out, gs, gt);
    return cdm_status();
}
CDM_API int cdm_conv3x3_cout1_fwd(const float* z, int ldz, int N, int H, int W, int C, const float* w, const float* bias,
                                  float* out, void* stream) {
    if (C % 4 || C > 1024) return (int)hipErrorInvalidValue;
    const long long P = (long long)N * H * W;
    if (C % 16 == 0 && W <= 256 && 256 % W == 0 && H % (256 / W) == 0 && ldz % 4 == 0)
        return launch_cout1_band(z, ldz, N, H, W, C, w, bias, out, nullptr, nullptr, S(stream));
    hipLaunchKernelGGL(conv_cout1_fwd_kernel, dim3(nblocks(P, 256 / (C / 4), 8192)), dim3(256), 0, S(stream), z, ldz, N, H,
                       W, C, w, bias, out);
    return cdm_status();
}
// out.3 on out.1's pre-norm output y with its GroupNorm + ReLU (per (n, c) scale gs / shift gt, [N][C]) applied while
// staging: the band form only (C % 16 == 0, W | 256, (256 / W) | H)
CDM_API int cdm_conv3x3_cout1_fwd_gn(const float* y, int ldy, int N, int H, int W, int C, const float* gs,
                                     const float* gt, const float* w, const float* bias, float* out, void* stream) {
    if (C % 16 || C > 1024 || W > 256 || 256 % W || H % (256 / W) || ldy % 4 || !gs || !gt)
        return (int)hipErrorInvalidValue;
    return launch_cout1_band(y, ldy, N, H, W, C, w, bias, out, gs, gt, S(stream));
}
CDM_API int cdm_conv3x3_cin1_dgrad(const float* g1, int ldg, const float* y1, int ldy, const float* s, const float* t,
                                   const float* mean, const float* invstd, const float* A, const float* B,
                                   const float* Cc, const float* w9, const float* gres, int ldr, const float* scw,
                                   int split, int N, int H, int W, int C, float* dx, void* stream) {
    if (C % 4 || C > 1024 || ldg % 4 || (y1 && ldy % 4) || (gres && (ldr % 4 || !scw))) return (int)hipErrorInvalidValue;
    if (y1 && !(s && t && mean && invstd && A && B && Cc)) return (int)hipErrorInvalidValue;
    const Cin1BnBwd bn{y1, ldy, {s, t, mean, invstd, A, B, Cc}};
    const long long P = (long long)N * H * W;
    hipLaunchKernelGGL(conv_cin1_dgrad_kernel, dim3(nblocks(P, 256 / (C / 4), 8192)), dim3(256), 0, S(stream), g1, ldg,
                       bn, w9, gres, ldr, scw, split, N, H, W, C, dx);
    return cdm_status();
}
CDM_API int cdm_conv3x3_cout1_dgrad(const float* deps, int N, int H, int W, int C, const float* w, float* dz, int lddz,
                                    void* stream) {
    if (C % 4 || C > 1024) return (int)hipErrorInvalidValue;
    const long long P = (long long)N * H * W;
    if (row_kernels() && W <= ROWK_MAXW && (long long)N * H <= 0x7fffffffll) {
        hipLaunchKernelGGL(conv_cout1_dgrad_row_kernel, dim3((unsigned)(N * H)), dim3(256), 3 * (W + 2) * sizeof(float),
                           S(stream), deps, H, W, C, w, dz, lddz);
        return cdm_status();
    }
    hipLaunchKernelGGL(conv_cout1_dgrad_kernel, dim3(nblocks(P, 256 / (C / 4), 4096)), dim3(256), 0, S(stream), deps, N, H,
                       W, C, w, dz, lddz);
    return cdm_status();
}
CDM_API int cdm_conv3x3_cout1_wgrad_gn(const float* deps, const float* y, int ldy, int N, int H, int W, int C,
                                       const float* gs, const float* gt, int csize, float* slab, void* stream) {
    // band form only: R = -csize whole rows per block, partials [N * H / R][9][C]; gs / gt null: y is z itself
    if (C % 4 || C > 1024 || csize >= 0 || (gs && !gt)) return (int)hipErrorInvalidValue;
    const int R = -csize;
    const size_t lds = (((size_t)(R + 2) * (W + 2) + 3) & ~(size_t)3) * 4 + (size_t)(256 / (C / 4)) * 9 * C * 4;
    if (H % R || ldy % 4 || lds > 64 * 1024) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(conv_cout1_wgrad_band_kernel, dim3(N * (H / R)), dim3(256), lds, S(stream), deps, y, ldy, H, W, C,
                       R, slab, gs, gt);
    return cdm_status();
}
CDM_API int cdm_conv3x3_cout1_wgrad(const float* deps, const float* z, int ldz, int N, int H, int W, int C, int csize,
                                    float* slab, void* stream) {
    if (C % 4 || C > 1024) return (int)hipErrorInvalidValue;
    if (csize < 0)                    // band form: R = -csize whole rows per block, partials [N * H / R][9][C]
        return cdm_conv3x3_cout1_wgrad_gn(deps, z, ldz, N, H, W, C, nullptr, nullptr, csize, slab, stream);
    hipLaunchKernelGGL(conv_cout1_wgrad_kernel, dim3((H * W + csize - 1) / csize, N), dim3(256), 0, S(stream), deps, z,
                       ldz, H, W, C, csize, slab);
    return cdm_status();
}
CDM_API int cdm_avgpool_gelu_fin(const float* sums, int N, int C, int HW, float* hpre, float* hv, void* stream) {
    hipLaunchKernelGGL(avgpool_gelu_fin_kernel, dim3((N * C + 255) / 256), dim3(256), 0, S(stream), sums, N, C,
                       1.0f / (float)HW, hpre, hv);
    return cdm_status();
}
CDM_API int cdm_avgpool_gelu_bwd(const float* dhv, const float* hpre, int N, int HW, int C, float* dst, int ldd,
                                 void* stream) {
    if (C % 4) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(avgpool_gelu_bwd_kernel, dim3(nblocks((long long)N * HW * (C / 4))), dim3(256), 0, S(stream), dhv,
                       hpre, N, HW, C, 1.0f / (float)HW, dst, ldd);
    return cdm_status();
}
CDM_API int cdm_embed_fwd(const Mlp4* P, void* stream) {
    int rows = 1;
    for (int k = 0; k < 4; ++k) { rows = P->m[k].rows > rows ? P->m[k].rows : rows; if (P->m[k].E > 1024) return (int)hipErrorInvalidValue; }
    hipLaunchKernelGGL(embed_fwd_kernel, dim3(rows, 4), dim3(256), 0, S(stream), *P);
    return cdm_status();
}
CDM_API int cdm_embed_input_grad(const float* dpre_a, const float* w1_a, int Ea, const float* dpre_b,
                                 const float* w1_b, int Eb, int rows, int in_dim, float* dx, void* stream) {
    if (rows < 0 || in_dim < 1 || Ea < 0 || Eb < 0) return (int)hipErrorInvalidValue;
    if (rows == 0) return 0;
    hipLaunchKernelGGL(embed_input_grad_kernel, dim3((rows * in_dim + 255) / 256), dim3(256), 0, S(stream), dpre_a, w1_a,
                       Ea, dpre_b, w1_b, Eb, rows, in_dim, dx);
    return cdm_status();
}
CDM_API int cdm_embed_bwd(const Mlp4* P, void* stream) {
    int rows = 1;
    for (int k = 0; k < 4; ++k) { rows = P->m[k].rows > rows ? P->m[k].rows : rows; if (P->m[k].E > 1024) return (int)hipErrorInvalidValue; }
    hipLaunchKernelGGL(embed_bwd_act_kernel, dim3(rows, 4), dim3(256), 0, S(stream), *P);
    int e = cdm_status(); if (e) return e;
    int nbx = 1;
    for (int k = 0; k < 4; ++k) {
        const MlpDesc& m = P->m[k];
        const long long rest = 2LL * m.E + (long long)m.E * m.in_dim;
        const int b = embed_tiles(m.E) + (int)((rest + 255) / 256);
        nbx = b > nbx ? b : nbx;
    }
    hipLaunchKernelGGL(embed_bwd_param_kernel, dim3(nbx, 4), dim3(256), 0, S(stream), *P);
    return cdm_status();
}
CDM_API int cdm_perturb(const float* x, const float* noise, const int* t, const int* cur_i, long long nstride,
                        const float* sab, const float* omab, int N, int HW, int T, float* out, float* tin, void* stream) {
    if (!t && !cur_i) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(perturb_kernel, dim3(nblocks((long long)N * HW)), dim3(256), 0, S(stream), x, noise, t, cur_i,
                       nstride, sab, omab, N, HW, T, out, tin);
    return cdm_status();
}
CDM_API int cdm_mse_accum(const float* pred, const float* noise, long long nstride, int T, int N, int HW, const int* t,
                          const int* cur_i, const float* mul, const float* div, float* acc, void* stream) {
    if (!t && !cur_i) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(mse_accum_kernel, dim3(N), dim3(256), 0, S(stream), pred, noise, nstride, T, HW, t, cur_i, mul,
                       div, acc);
    return cdm_status();
}
CDM_API int cdm_mse(const float* pred, const float* noise, long long n, double grad_numel, float* dpred, float* partial,
                    int nb, float* loss_out, float* dbias_out, int* nonfinite, void* stream) {
    if (!(grad_numel > 0.0)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(mse_kernel, dim3(nb), dim3(256), 0, S(stream), pred, noise, n, (float)(2.0 / grad_numel), dpred,
                       partial);
    int e = cdm_status(); if (e) return e;
    hipLaunchKernelGGL(mse_finalize_kernel, dim3(1), dim3(64), 0, S(stream), partial, nb, 1.0 / (double)n, loss_out,
                       dbias_out, nonfinite);
    return cdm_status();
}
CDM_API int cdm_sample_prologue(int* ctr, int T, int* cur_i, float* t_cur, const float* sc_table, int sc_row, float* sc_cur,
                                void* stream) {
    hipLaunchKernelGGL(sample_prologue_kernel, dim3(1), dim3(256), 0, S(stream), ctr, T, cur_i, t_cur, sc_table, sc_row,
                       sc_cur);
    return cdm_status();
}
CDM_API int cdm_denoise(const float* xin, float* x, float* x2, long long numel, const float* eps, int cfg, float w,
                        const int* cur_i, const float* coef, const float* sa, const float* sb, const float* z_table,
                        long long zstride, unsigned long long seed, const long long* seed_dev, const int* snap_slot,
                        float* snaps, int T, void* stream) {
    hipLaunchKernelGGL(denoise_kernel, dim3(nblocks(numel)), dim3(256), 0, S(stream), xin, x, x2, numel, eps, cfg, w, cur_i,
                       coef, sa, sb, z_table, zstride, seed, seed_dev, snap_slot, snaps, T);
    return cdm_status();
}
CDM_API int cdm_adam(float* p, const float* g, float* m, float* v, long long n, double* state, const double* bc,
                     int nbc, double beta1, double beta2, double eps, float grad_scale, void* stream) {
    if (nbc < 1) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(1), 0, S(stream), state, bc, nbc);
    int e = cdm_status(); if (e) return e;
    hipLaunchKernelGGL(adam_kernel, dim3(nblocks(n, 256, 16384)), dim3(256), 0, S(stream), p, g, m, v, n, state,
                       (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps, grad_scale);
    return cdm_status();
}
CDM_API int cdm_pack_conv3x3(const float* W, const float* b, int Cin, int Cout, const float* gamma, const float* beta,
                             const float* rm, const float* rv, float eps, float* wpk, float* bpk, float* wdg, int kc,
                             void* stream) {
    if (kc && ((wpk && Cin % kc) || (wdg && Cout % kc))) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(pack_conv3x3_kernel, dim3(nblocks((long long)Cout * Cin * 9)), dim3(256), 0, S(stream), W, b, Cin,
                       Cout, gamma, beta, rm, rv, eps, wpk, bpk, wdg, kc);
    return cdm_status();
}
static void transpose_tiled(const float* in, long long batch, long long R, long long C, float* out, hipStream_t s) {
    const long long tiles = ((R + 63) / 64) * ((C + 63) / 64);
    hipLaunchKernelGGL(transpose_tiled_kernel, dim3((unsigned)tiles, (unsigned)batch), dim3(256), 0, s, in, R, C, out);
}

CDM_API int cdm_pack_convT(const float* W, int Cin, int Cout, int KK, float* wt, float* wtT, void* stream) {
    if (wt) {
        // wt[ci] = W[ci]^T  ([Cout][KK] -> [KK][Cout]);  wtT = wt^T ([Cin][KK*Cout] -> [KK*Cout][Cin])
        if (KK > 1) transpose_tiled(W, Cin, Cout, KK, wt, S(stream));
        else if (hipMemcpyAsync(wt, W, sizeof(float) * (size_t)Cin * Cout, hipMemcpyDeviceToDevice, S(stream)) != hipSuccess)
            return cdm_status();
        if (wtT) transpose_tiled(wt, 1, Cin, (long long)KK * Cout, wtT, S(stream));
        return cdm_status();
    }
    hipLaunchKernelGGL(pack_convT_kernel, dim3(nblocks((long long)Cin * Cout * KK)), dim3(256), 0, S(stream), W, Cin, Cout,
                       KK, wt, wtT);
    return cdm_status();
}
CDM_API int cdm_transpose(const float* in, int R, int C, float* out, void* stream) {
    transpose_tiled(in, 1, R, C, out, S(stream));
    return cdm_status();
}
/* in [batch][R][C] -> out [batch][C][R] */
CDM_API int cdm_transpose_batched(const float* in, int batch, int R, int C, float* out, void* stream) {
    transpose_tiled(in, batch, R, C, out, S(stream));
    return cdm_status();
}
__global__ void counter_add_kernel(int* c, int d) { if (threadIdx.x == 0) *c += d; }
CDM_API int cdm_counter_add(int* ctr, int delta, void* stream) {
    hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, S(stream), ctr, delta);
    return cdm_status();
}
CDM_API int cdm_device_sync() { return (int)hipDeviceSynchronize(); }
CDM_API int cdm_abi_version() { return 1; }
