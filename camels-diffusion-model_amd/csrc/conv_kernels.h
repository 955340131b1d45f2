#pragma once
// Kernel templates of the 16-bit / fp32 MFMA conv and GEMM family, shared by the translation units
// gemm_f32.hip (generic GEMMs, ConvT, splits, reductions), conv_fwd.hip (LDS-halo forward), conv_dgrad.hip
// (LDS-halo BN-backward dgrad) and conv_wgrad.hip (kernel-row weight gradient): one header, four compiler jobs.
// fp32 MFMA (v_mfma_f32_32x32x2_f32) implicit-GEMM family for gfx950.
//
// One templated main loop serves every contraction on the ContextUnet path:
//   conv3x3 fwd            C[pix][co]      = im2col(X)[pix][tap,ci] . Wp[tap,ci][co]
//   conv3x3 dgrad          same kernel, X := dY, Wp := flipped/transposed weights
//   convT 2x2 fwd          C[pix][ij,co]   = X[pix][ci] . Wt[ci][ij,co]        (scatter epilogue)
//   convT 2x2 dgrad        C[pix][ci]      = gather(dY)[pix][ij,co] . WtT[ij,co][ci]
//   up0 (convT k=H/4 1x1)  C[n][ij,co]     = hv[n][ci] . W0[ci][ij,co]
//   *_wgrad (split-K)      C[m][n]         = sum_pix A^T[pix][m] . B[pix][n] -> fp32 partial slabs
// Reference ops: nn.Conv2d(.,.,3,1,1) diffusion_utilities.py:27,34 / ContextUnet.py:36,39;
// nn.ConvTranspose2d(in,out,2,2) diffusion_utilities.py:86; ConvTranspose2d(k=h/4) ContextUnet.py:27.
//
// Tile: 128x128 per 256-thread workgroup (4 waves as 2x2, each wave 64x64 = 2x2 MFMA 32x32
// accumulators = 64 AGPRs), BK in {16,32}, LDS double buffer staged through registers (the global
// loads for tile t+1 are issued before the MFMAs of tile t, written to LDS after them: T14).
// LDS images are k-major ([k][m], [k][n]) so every MFMA operand read is one conflict-free
// ds_read_b32 of 32 consecutive floats per half-wave.  Partial-tile bounds are handled by the
// loaders (zero fill) and the epilogues (masked stores), so any M and N%4==0, K%4==0 work.
#include "cdm_common.h"
#include <cstdlib>
#include <type_traits>

namespace cdm {

constexpr int GBM = 128;
constexpr int GBN = 128;
constexpr int GTHREADS = 256;

// ============================== A loaders, k-contiguous: A(m, k..k+3) ==============================
struct LdDenseA {  // A[m][k] = a[m*lda + k]
    const float* a; long long lda; int M, K;
    struct Row { const float* p; };
    __device__ __forceinline__ Row row(int m) const { return Row{m < M ? a + (long long)m * lda : nullptr}; }
    __device__ __forceinline__ float4 load(const Row& r, int k) const {
        return (r.p && k < K) ? ld4(r.p + k) : f4zero();
    }
};

// K order: KC == 0 -> k = tap*C + ci (tap-major);  KC > 0 -> k = (cc*9 + tap)*KC + cj, ci = cc*KC + cj
// (channel-chunk-major: the 9 taps of one KC-channel slab are consecutive K tiles, so they re-read the
//  same ~17 KB input slab from L1/L2 instead of re-streaming the block's whole 131 KB input 9 times).
template <int CT, int KC = 0, int HT = 0>  // CT/HT > 0: channels / square map size known at compile time
struct LdIm2colA {  // 3x3, stride 1, pad 1; m = (n,h,w)
    const float* x; int Hrt, Wrt, Crt, ldx, M, K;
    struct Row { int n, h, w; bool ok; };
    __device__ __forceinline__ Row row(int m) const {
        const int H = HT > 0 ? HT : Hrt, W = HT > 0 ? HT : Wrt;
        Row r; r.ok = m < M; const int hw = H * W; r.n = m / hw; const int rem = m - r.n * hw;
        r.h = rem / W; r.w = rem - r.h * W; return r;
    }
    __device__ __forceinline__ float4 load(const Row& r, int k) const {
        if (!r.ok || k >= K) return f4zero();
        const int C = CT > 0 ? CT : Crt;
        const int H = HT > 0 ? HT : Hrt, W = HT > 0 ? HT : Wrt;
        int tap, ci;
        if constexpr (KC > 0) {
            const int cc = k / (9 * KC), rem = k - cc * 9 * KC;
            tap = rem / KC; ci = cc * KC + (rem - tap * KC);
        } else {
            tap = k / C; ci = k - tap * C;
        }
        const int ky = tap / 3, kx = tap - ky * 3;
        const int hh = r.h + ky - 1, ww = r.w + kx - 1;
        if ((unsigned)hh >= (unsigned)H || (unsigned)ww >= (unsigned)W) return f4zero();
        return ld4(x + ((long long)(r.n * H + hh) * W + ww) * ldx + ci);
    }
};

struct LdConvT2x2GatherA {  // dgrad of convT 2x2: m = (n,h,w) on the INPUT grid, k = (i*2+j)*Co + co
    const float* dy; int H, W, Co, lddy, M, K;   // dy is [N, 2H, 2W, Co] (ld lddy)
    struct Row { int n, h, w; bool ok; };
    __device__ __forceinline__ Row row(int m) const {
        Row r; r.ok = m < M; const int hw = H * W; r.n = m / hw; const int rem = m - r.n * hw;
        r.h = rem / W; r.w = rem - r.h * W; return r;
    }
    __device__ __forceinline__ float4 load(const Row& r, int k) const {
        if (!r.ok || k >= K) return f4zero();
        const int ij = (k >= Co) + (k >= 2 * Co) + (k >= 3 * Co), co = k - ij * Co;   // k < K = 4 Co: no division
        const int oh = 2 * r.h + (ij >> 1), ow = 2 * r.w + (ij & 1);
        return ld4(dy + ((long long)(r.n * 2 * H + oh) * (2 * W) + ow) * lddy + co);
    }
};

// ============================== A loader, m-contiguous: A(m..m+3, k) (wgrad) ==============================
struct LdDenseAT {  // A(m, k) = a[k*lda + m]  (a is [K][M] row-major, e.g. dY[pix][co])
    const float* a; long long lda; int M, K;
    __device__ __forceinline__ float4 loadT(int k, int m) const {
        return (k < K && m < M) ? ld4(a + (long long)k * lda + m) : f4zero();
    }
    // split-bf16 path: 8 consecutive k at one m (K % 8 == 0)
    struct Col { int m; };
    __device__ __forceinline__ Col col(int m) const { return Col{m}; }
    __device__ __forceinline__ void load8(const Col& c, int k, float (&o)[8]) const {
        const bool ok = c.m < M && k < K;
        const float* p = a + (long long)k * lda + c.m;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = ok ? p[(long long)j * lda] : 0.f;
    }
};

// ============================== B loaders, n-contiguous: B(k, n..n+3) ==============================
struct LdDenseB {  // B[k][n] = b[k*ldb + n]
    const float* b; long long ldb; int K, N;
    struct Col { int n; };
    __device__ __forceinline__ Col col(int n) const { return Col{n}; }
    __device__ __forceinline__ float4 load(const Col& c, int k) const {
        return (k < K && c.n < N) ? ld4(b + (long long)k * ldb + c.n) : f4zero();
    }
};

struct LdIm2colB {  // conv3x3 wgrad: B(k = pix, n = tap*C + ci) = X[pix shifted by tap][ci]
    const float* x; int H, W, C, ldx, K, N;
    struct Col { int dy, dx, ci; bool ok; };
    __device__ __forceinline__ Col col(int n) const {
        Col c; c.ok = n < N; const int tap = n / C; c.ci = n - tap * C;
        const int ky = tap / 3; c.dy = ky - 1; c.dx = tap - ky * 3 - 1; return c;
    }
    __device__ __forceinline__ float4 load(const Col& c, int k) const {
        if (!c.ok || k >= K) return f4zero();
        const int hw = H * W; const int n = k / hw; const int rem = k - n * hw;
        const int h = rem / W, w = rem - h * W;
        const int hh = h + c.dy, ww = w + c.dx;
        if ((unsigned)hh >= (unsigned)H || (unsigned)ww >= (unsigned)W) return f4zero();
        return ld4(x + ((long long)(n * H + hh) * W + ww) * ldx + c.ci);
    }
    // split-bf16 path: 8 consecutive pixels k..k+7 (one image row, W % 8 == 0) at one column
    __device__ __forceinline__ void load8(const Col& c, int k, float (&o)[8]) const {
        const int hw = H * W; const int n = k / hw; const int rem = k - n * hw;
        const int h = rem / W, w0 = rem - h * W;
        const int hh = h + c.dy;
        const bool rowok = c.ok && k < K && (unsigned)hh < (unsigned)H;
        const float* p = x + ((long long)(n * H + hh) * W + w0 + c.dx) * ldx + c.ci;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ww = w0 + j + c.dx;
            o[j] = (rowok && (unsigned)ww < (unsigned)W) ? p[(long long)j * ldx] : 0.f;
        }
    }
};

struct LdConvT2x2GatherB {  // convT 2x2 wgrad: B(k = input pix (n,h,w), n = ij*Co + co) = dY[n,2h+i,2w+j,co]
    const float* dy; int H, W, Co, lddy, K, N;
    struct Col { int i, j, co; bool ok; };
    __device__ __forceinline__ Col col(int n) const {
        Col c; c.ok = n < N; const int ij = n / Co; c.co = n - ij * Co; c.i = ij >> 1; c.j = ij & 1; return c;
    }
    __device__ __forceinline__ float4 load(const Col& c, int k) const {
        if (!c.ok || k >= K) return f4zero();
        const int hw = H * W; const int n = k / hw; const int rem = k - n * hw;
        const int h = rem / W, w = rem - h * W;
        return ld4(dy + ((long long)(n * 2 * H + 2 * h + c.i) * (2 * W) + 2 * w + c.j) * lddy + c.co);
    }
    // split-bf16 / h3 path: 8 consecutive input pixels k..k+7 (one image row, W % 8 == 0) at one column
    __device__ __forceinline__ void load8(const Col& c, int k, float (&o)[8]) const {
        const bool ok = c.ok && k < K;
        const int hw = H * W; const int n = k / hw; const int rem = k - n * hw;
        const int h = rem / W, w0 = rem - h * W;
        const float* p = dy + ((long long)(n * 2 * H + 2 * h + c.i) * (2 * W) + 2 * w0 + c.j) * lddy + c.co;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = ok ? p[(long long)(2 * j) * lddy] : 0.f;
    }
};

// ============================== epilogues ==============================
// Accumulator element (i, j, r) of a wave sits at row  mw + 32i + (r&3) + 8(r>>2) + 4(lane>>5)
//                                             column nw + 32j + (lane&31).
#define CDM_FOR_ACC(...) CDM_FOR_ACC_N(2, __VA_ARGS__)
#define CDM_FOR_ACC_N(NI, ...)                                                             \
    _Pragma("unroll") for (int i = 0; i < NI; ++i)                                          \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                           \
    _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                        \
        const int m = mw + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);              \
        const int n = nw + 32 * j + (lane & 31);                                             \
        __VA_ARGS__                                                                          \
    }

enum { EPI_RELU = 1, EPI_ACCUM = 2 };

// Eval-mode output transforms fused into the conv epilogue (EpiStoreW<..., FUSE = true>; the norm_apply_fwd forms of
// diffusion_utilities.py:54-55 / :109 and ContextUnet.py:57-58 after a BatchNorm folded into the weights), applied to
// v = relu(acc + bias):
//   RESID  out = w[c] x[pix] + b[c] + v  (the random 1x1 shortcut of the C_in = 1 image; set 1 for images >= split)
//   FILM   out = a[img][c] v + b[img][c]
//   POOL   out[pooled pixel] = max over the 2x2 window (MaxPool2d(2): NaN wins), image width 32 or 64
enum { FUSE_RESID = 1, FUSE_FILM = 2, FUSE_POOL = 3 };
struct EpiFuse {
    int kind = 0;
    int hw = 1, W = 1;                      // pixels per image and image width of the conv's output grid
    const float* x = nullptr; const float* w = nullptr; const float* b = nullptr; int split = 0;   // RESID
    const float* fa = nullptr; int fan = 0; const float* fb = nullptr; int fbn = 0;                 // FILM
};

// WM = waves along M (2: 128-row block, 4: 256-row block); stats per 128-row tile.  OT = the stored element type (bf16:
// C4's fused-chain activations and gradients; the statistics / maxima are those of the stored, rounded values)
template <int WM = 2, class OT = float, bool ACC = false, bool FUSE = false>
struct EpiStoreW {  // y[m*ldy + n] (+)= acc + bias[n % bias_mod]; optional per-tile column stats
    OT* y; long long ldy; long long zstride; const float* bias; int bias_mod; int flags;
    float* stats; int stats_ld;  // stats[tile][0|1][stats_ld]: sum / sum of squares of the stored value
    int M, N;
    float* amax = nullptr;       // optional running max|stored value| (block_amax_commit)
    int* ymm = nullptr;          // optional per-column max / min of the stored value, ordered-int keys (fkey):
    int ymm_ld = 0;              //   ymm[n] (atomic max), ymm[ymm_ld + n] (atomic min); needs stats
    EpiFuse fz{};                // FUSE: the eval-mode output transform (LDS-halo conv, whole 256-pixel tiles)

    // Addresses of a wave tile's 64 accumulator elements (i, j, r) — row mw + 32 i + (r & 3) + 8 (r >> 2) + 4 (lane >> 5),
    // column nw + 32 j + (lane & 31) — as a wave-uniform base (scalar arithmetic: mw / nw are wave-uniform, made so for
    // the compiler by readfirstlane) plus ONE lane byte offset shared by all 64 of them.  Written as y + (long long)m *
    // ldy + n per element, every address cost two v_mul_lo_u32 and a v_mad_u64_u32 (quarter-rate VALU) — the bulk of
    // the epilogue's issue time, which no MFMA overlaps (round 6).
    struct WaveAddr {
        OT* base; long long ldy; unsigned lb;
        __device__ __forceinline__ OT* at(int i, int j, int r) const {
            return reinterpret_cast<OT*>(reinterpret_cast<char*>(base + (long long)(32 * i + (r & 3) + 8 * (r >> 2)) * ldy
                                                                 + 32 * j) + lb);
        }
    };
    __device__ __forceinline__ WaveAddr wave_addr(OT* yb, int mw, int nw, int lane) const {
        const int mu = __builtin_amdgcn_readfirstlane(mw), nu = __builtin_amdgcn_readfirstlane(nw);
        return WaveAddr{yb + (long long)mu * ldy + nu, ldy,
                        (unsigned)(4 * (lane >> 5) * (int)ldy + (lane & 31)) * (unsigned)sizeof(OT)};
    }

    // FUSE (eval forward, conv3x3_halo_x3_kernel): relu(acc + bias), then fz's transform; the whole block tile is in
    // range (host: M % 256 == 0, N % 128 == 0) and a 256-pixel tile lies in one image (hw % 256 == 0).  POOL: at
    // W = 32 a wave's two row blocks are two image rows (the 2x2 window is in registers); at W = 64 a wave holds one
    // image row and its vertical neighbour is wave wm ^ 1 (exchanged through scratch, 16 KiB per round, two rounds).
    __device__ __forceinline__ void fused(f32x16 (&acc)[2][2], int mw, int nw, int lane, int wm, int wn,
                                          float* scratch) const {
        const int img = mw / fz.hw;
        float bj[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) bj[j] = bias ? bias[nw + 32 * j + (lane & 31)] : 0.f;
        float am = 0.f;
        if (fz.kind == FUSE_POOL) {
            float hp[2][2][8];   // horizontal pairs (rows r, r + 1 of an accumulator: pixels d, d + 1)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const float a = relu_f(acc[i][j][2 * k] + bj[j]), b = relu_f(acc[i][j][2 * k + 1] + bj[j]);
                        hp[i][j][k] = (b > a || isnan(b)) ? b : a;
                        am = fmaxf(am, hp[i][j][k]);
                    }
            const int hw4 = fz.hw >> 2, Wo = fz.W >> 1;
            auto put = [&](int i, int j, int k, float v) {   // pooled value of the window at accumulator (i, j, 2k)
                const int m = mw + 32 * i + (2 * k & 3) + 8 * (2 * k >> 2) + 4 * (lane >> 5);
                const int p = m - img * fz.hw, h = p / fz.W, c = p - h * fz.W;
                const long long o = (long long)img * hw4 + (h >> 1) * Wo + (c >> 1);
                Act<OT>::store(y + o * ldy + nw + 32 * j + (lane & 31), Act<OT>::round(v));
            };
            if (fz.W == 32) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const float a = hp[0][j][k], b = hp[1][j][k];
                        put(0, j, k, (b > a || isnan(b)) ? b : a);
                    }
            } else {
                float* xs = scratch + ((wm >> 1) * 2 + wn) * 16 * 64;   // [pair][wn][16 values][64 lanes]
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if (wm & 1) {
#pragma unroll
                        for (int j = 0; j < 2; ++j)
#pragma unroll
                            for (int k = 0; k < 8; ++k) xs[(j * 8 + k) * 64 + lane] = hp[i][j][k];
                    }
                    __syncthreads();
                    if (!(wm & 1)) {
#pragma unroll
                        for (int j = 0; j < 2; ++j)
#pragma unroll
                            for (int k = 0; k < 8; ++k) {
                                const float a = hp[i][j][k], b = xs[(j * 8 + k) * 64 + lane];
                                put(i, j, k, (b > a || isnan(b)) ? b : a);
                            }
                    }
                    __syncthreads();
                }
            }
        } else {
            // every coefficient and shortcut input loaded ahead of the first store: y may alias them as far as the
            // compiler knows, so a load written next to its use waits behind the previous store (RESID cost the
            // 64^2 init conv 300 us per launch that way)
            const int sel = img >= fz.split ? N : 0;
            const bool resid = fz.kind == FUSE_RESID;
            float ca[2], cb[2], xv[2][16];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = nw + 32 * j + (lane & 31);
                ca[j] = resid ? fz.w[sel + n] : fz.fa[img * fz.fan + n];
                cb[j] = resid ? fz.b[sel + n] : fz.fb[img * fz.fbn + n];
            }
            if (resid) {
                const float* xb = fz.x + __builtin_amdgcn_readfirstlane(mw);
                const unsigned lx = (unsigned)(4 * (lane >> 5)) * 4u;
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        xv[i][r] = *reinterpret_cast<const float*>(
                            reinterpret_cast<const char*>(xb + 32 * i + (r & 3) + 8 * (r >> 2)) + lx);
            }
            const WaveAddr wa = wave_addr(y, mw, nw, lane);
            CDM_FOR_ACC({
                float v = relu_f(acc[i][j][r] + bj[j]);
                if (resid) v = fmaf(ca[j], xv[i][r], cb[j]) + v;
                else v = fmaf(ca[j], v, cb[j]);
                v = Act<OT>::round(v);
                Act<OT>::store(wa.at(i, j, r), v);
                am = fmaxf(am, fabsf(v));
            })
        }
        if (amax) block_amax_commit(am, amax);
    }

    __device__ __forceinline__ void operator()(f32x16 (&acc)[2][2], int mw, int nw, int lane, int wm, int wn,
                                               float* scratch, int tid) const {
        if constexpr (FUSE) {
            fused(acc, mw, nw, lane, wm, wn, scratch);
            return;
        }
        OT* yz = y + (long long)blockIdx.z * zstride;      // 0 when the kernel applied its own (remapped) slab
        float cs[2] = {0.f, 0.f}, cq[2] = {0.f, 0.f};
        float cmx[2] = {-INFINITY, -INFINITY}, cmn[2] = {INFINITY, INFINITY};
        float am = 0.f;
        if (mw - wm * 64 + WM * 64 <= M && (nw - wn * 64) + GBN <= N) {
            // whole block tile in range (the hot shapes): no per-element bounds branches, bias hoisted (one
            // column per lane and j)
            float bj[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bj[j] = bias ? bias[(nw + 32 * j + (lane & 31)) % bias_mod] : 0.f;
            const bool relu = flags & EPI_RELU;
            const bool accum = flags & EPI_ACCUM;
            const WaveAddr wa = wave_addr(yz, mw, nw, lane);
            if constexpr (ACC) {
                // accumulate (a compile-time variant: the interleaved form below waited on one load per element — the
                // compiler cannot prove the addresses disjoint — +0.5 ms per accumulating 64^2 dgrad, profiles/
                // r4_train_step_sequence_c2.txt; holding the old values in the shared epilogue made every conv spill):
                // the 16 old values of a 32 x 32 block are loaded before its first store
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        float old[16];
#pragma unroll
                        for (int r = 0; r < 16; ++r) old[r] = Act<OT>::load(wa.at(i, j, r));
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            float v = acc[i][j][r] + bj[j] + old[r];
                            if (relu) v = relu_f(v);
                            v = Act<OT>::round(v);
                            Act<OT>::store(wa.at(i, j, r), v);
                            cs[j] += v; cq[j] += v * v;
                            am = fmaxf(am, fabsf(v));
                            cmx[j] = fmaxf(cmx[j], v); cmn[j] = fminf(cmn[j], v);
                        }
                    }
            } else {
                // the runtime accumulate flag hoisted out of the 64 elements (a uniform branch per element split the
                // epilogue into 64 basic blocks, each with its own vmcnt(0) wait)
                // (and the column statistics, when the launch records none: the eval forwards)
                auto body = [&](auto accum_tag, auto stats_tag) {
                    CDM_FOR_ACC({
                        float v = acc[i][j][r] + bj[j];
                        if constexpr (decltype(accum_tag)::value) v += Act<OT>::load(wa.at(i, j, r));
                        if (relu) v = relu_f(v);
                        v = Act<OT>::round(v);
                        Act<OT>::store(wa.at(i, j, r), v);
                        am = fmaxf(am, fabsf(v));
                        if constexpr (decltype(stats_tag)::value) {
                            cs[j] += v; cq[j] += v * v;
                            cmx[j] = fmaxf(cmx[j], v); cmn[j] = fminf(cmn[j], v);
                        }
                    })
                };
                if (accum) body(std::true_type{}, std::true_type{});
                else if (stats) body(std::false_type{}, std::true_type{});
                else body(std::false_type{}, std::false_type{});
            }
        } else {
            CDM_FOR_ACC({
                if (m < M && n < N) {
                    float v = acc[i][j][r];
                    if (bias) v += bias[n % bias_mod];
                    OT* p = yz + (long long)m * ldy + n;
                    if (flags & EPI_ACCUM) v += Act<OT>::load(p);
                    if (flags & EPI_RELU) v = relu_f(v);
                    v = Act<OT>::round(v);
                    Act<OT>::store(p, v);
                    cs[j] += v; cq[j] += v * v;
                    am = fmaxf(am, fabsf(v));
                    cmx[j] = fmaxf(cmx[j], v); cmn[j] = fminf(cmn[j], v);
                }
            })
        }
        if (amax) block_amax_commit(am, amax);
        if (!stats) return;
#pragma unroll
        for (int j = 0; j < 2; ++j) { cs[j] += __shfl_xor(cs[j], 32, 64); cq[j] += __shfl_xor(cq[j], 32, 64); }
        __syncthreads();  // scratch aliases the operand LDS
        if (lane < 32) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = wn * 64 + 32 * j + lane;
                scratch[(wm * 2 + 0) * GBN + c] = cs[j];
                scratch[(wm * 2 + 1) * GBN + c] = cq[j];
            }
        }
        __syncthreads();
        if (tid < GBN * (WM / 2)) {   // tile t of the block's WM/2 128-row tiles sums waves 2t and 2t+1
            const int t = tid / GBN, c = tid - t * GBN;
            const int n = (nw - wn * 64) + c;
            if (n < N) {
                float* st = stats + (long long)((mw - wm * 64) / GBM + t) * 2 * stats_ld;
                st[n] = scratch[(4 * t + 0) * GBN + c] + scratch[(4 * t + 2) * GBN + c];
                st[stats_ld + n] = scratch[(4 * t + 1) * GBN + c] + scratch[(4 * t + 3) * GBN + c];
            }
        }
        if (!ymm) return;
        // column max / min over the block (the next layer's exact max|relu(y s + t)|, see bn_fwd_finalize)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            cmx[j] = fmaxf(cmx[j], __shfl_xor(cmx[j], 32, 64));
            cmn[j] = fminf(cmn[j], __shfl_xor(cmn[j], 32, 64));
        }
        __syncthreads();
        if (lane < 32) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = wn * 64 + 32 * j + lane;
                scratch[wm * GBN + c] = cmx[j];
                scratch[(WM + wm) * GBN + c] = cmn[j];
            }
        }
        __syncthreads();
        if (tid < GBN) {
            const int n = (nw - wn * 64) + tid;
            if (n < N) {
                float mx = scratch[tid], mn = scratch[WM * GBN + tid];
#pragma unroll
                for (int w = 1; w < WM; ++w) {
                    mx = fmaxf(mx, scratch[w * GBN + tid]);
                    mn = fminf(mn, scratch[(WM + w) * GBN + tid]);
                }
                atomicMax(ymm + n, fkey(mx));
                atomicMin(ymm + ymm_ld + n, fkey(mn));
            }
        }
    }

    // tall wave tiles (conv3x3_halo_x3_kernel, ABL 8192; 2 waves along M of the 256-row block): the wave holds rows
    // mw..mw+127 (4 row blocks of 32) x columns nw..nw+63, i.e. exactly one 128-row stats tile, written directly
    __device__ __forceinline__ void tall(f32x16 (&acc)[4][2], int mw, int nw, int lane, int wm, int wn, float* scratch,
                                         int tid) const {
        static_assert(WM == 4, "tall tiles: a 256-row block");
        constexpr int NWM = 2;   // waves along M
        OT* yz = y + (long long)blockIdx.z * zstride;
        // column sums per half (row blocks 0-1, 2-3), added as the 64 x 64 form adds its two waves: identical stats
        float cs[2][2] = {{0.f, 0.f}, {0.f, 0.f}}, cq[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
        float cmx[2] = {-INFINITY, -INFINITY}, cmn[2] = {INFINITY, INFINITY};
        float am = 0.f;
        const bool relu = flags & EPI_RELU;
        const bool accum = flags & EPI_ACCUM;
        if (mw + 128 <= M && (nw - wn * 64) + GBN <= N) {
            float bj[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bj[j] = bias ? bias[(nw + 32 * j + (lane & 31)) % bias_mod] : 0.f;
            if constexpr (ACC) {   // the load-ahead accumulate (see operator())
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        float old[16];
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int m = mw + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                            old[r] = Act<OT>::load(yz + (long long)m * ldy + nw + 32 * j + (lane & 31));
                        }
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int m = mw + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                            const int n = nw + 32 * j + (lane & 31);
                            float v = acc[i][j][r] + bj[j] + old[r];
                            if (relu) v = relu_f(v);
                            v = Act<OT>::round(v);
                            Act<OT>::store(yz + (long long)m * ldy + n, v);
                            cs[i >> 1][j] += v; cq[i >> 1][j] += v * v;
                            am = fmaxf(am, fabsf(v));
                            cmx[j] = fmaxf(cmx[j], v); cmn[j] = fminf(cmn[j], v);
                        }
                    }
            } else {
                CDM_FOR_ACC_N(4, {
                    float v = acc[i][j][r] + bj[j];
                    if (accum) v += Act<OT>::load(yz + (long long)m * ldy + n);
                    if (relu) v = relu_f(v);
                    v = Act<OT>::round(v);
                    Act<OT>::store(yz + (long long)m * ldy + n, v);
                    cs[i >> 1][j] += v; cq[i >> 1][j] += v * v;
                    am = fmaxf(am, fabsf(v));
                    cmx[j] = fmaxf(cmx[j], v); cmn[j] = fminf(cmn[j], v);
                })
            }
        } else {
            CDM_FOR_ACC_N(4, {
                if (m < M && n < N) {
                    float v = acc[i][j][r];
                    if (bias) v += bias[n % bias_mod];
                    OT* p = yz + (long long)m * ldy + n;
                    if (accum) v += Act<OT>::load(p);
                    if (relu) v = relu_f(v);
                    v = Act<OT>::round(v);
                    Act<OT>::store(p, v);
                    cs[i >> 1][j] += v; cq[i >> 1][j] += v * v;
                    am = fmaxf(am, fabsf(v));
                    cmx[j] = fmaxf(cmx[j], v); cmn[j] = fminf(cmn[j], v);
                }
            })
        }
        if (amax) block_amax_commit(am, amax);
        if (!stats) return;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                cs[h][j] += __shfl_xor(cs[h][j], 32, 64);
                cq[h][j] += __shfl_xor(cq[h][j], 32, 64);
            }
        if (lane < 32) {
            float* st = stats + (long long)(mw / GBM) * 2 * stats_ld;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = nw + 32 * j + lane;
                if (n < N) { st[n] = cs[0][j] + cs[1][j]; st[stats_ld + n] = cq[0][j] + cq[1][j]; }
            }
        }
        if (!ymm) return;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            cmx[j] = fmaxf(cmx[j], __shfl_xor(cmx[j], 32, 64));
            cmn[j] = fminf(cmn[j], __shfl_xor(cmn[j], 32, 64));
        }
        __syncthreads();  // scratch aliases the operand LDS
        if (lane < 32) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int c = wn * 64 + 32 * j + lane;
                scratch[wm * GBN + c] = cmx[j];
                scratch[(NWM + wm) * GBN + c] = cmn[j];
            }
        }
        __syncthreads();
        if (tid < GBN) {
            const int n = (nw - wn * 64) + tid;
            if (n < N) {
                float mx = scratch[tid], mn = scratch[NWM * GBN + tid];
#pragma unroll
                for (int w = 1; w < NWM; ++w) {
                    mx = fmaxf(mx, scratch[w * GBN + tid]);
                    mn = fminf(mn, scratch[(NWM + w) * GBN + tid]);
                }
                atomicMax(ymm + n, fkey(mx));
                atomicMin(ymm + ymm_ld + n, fkey(mn));
            }
        }
    }
};
using EpiStore = EpiStoreW<2>;
template <class EP> struct IsEpiStoreW : std::false_type {};
template <int WM, class OT, bool ACC, bool FUSE> struct IsEpiStoreW<EpiStoreW<WM, OT, ACC, FUSE>> : std::true_type {};

// EpiConvT2x2 for the transposed accumulators of gemm_deep_kernel<..., TRO = true>: acc[i][j][r] = C[m][n] at m = mw + 32 i +
// (lane & 31), n = nw + 32 j + (r & 3) + 8 (r >> 2) + 4 (lane >> 5).  Four consecutive n (r = 4q..4q+3) are four consecutive
// output channels of one sub-pixel ij (Co % 8 == 0: an 8-aligned column group never straddles two sub-pixels, so ij is
// wave-uniform), stored as one float4; needs y, ldy 16-byte aligned and M % 128 == N % 128 == 0 (host checks).
struct EpiConvT2x2T {
    float* y; long long ldy; const float* bias; int H, W, Co, M, N;
    float* amax = nullptr;
    __device__ __forceinline__ void operator()(f32x16 (&acc)[2][2], int mw, int nw, int lane, int, int, float*,
                                               int) const {
        float am = 0.f;
        const int hw = H * W, nu = __builtin_amdgcn_readfirstlane(nw), lh = 4 * (lane >> 5);
        float* px[2];   // the lane's input pixel m -> its output 2x2 block's first pixel
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = mw + 32 * i + (lane & 31), b = m / hw, rem = m - b * hw, h = rem / W, w = rem - h * W;
            px[i] = y + ((long long)(b * 2 * H + 2 * h) * (2 * W) + 2 * w) * ldy + lh;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int nb = nu + 32 * j + 8 * q, ij = nb / Co, co = nb - ij * Co;   // wave-uniform
                const long long off = ((long long)(ij >> 1) * (2 * W) + (ij & 1)) * ldy + co;
                const float* bp = bias + co + lh;   // (the packed parameter buffer: not 16-byte aligned in general)
                const float4 bv = bias ? make_float4(bp[0], bp[1], bp[2], bp[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const float4 v = make_float4(acc[i][j][4 * q] + bv.x, acc[i][j][4 * q + 1] + bv.y,
                                                 acc[i][j][4 * q + 2] + bv.z, acc[i][j][4 * q + 3] + bv.w);
                    *reinterpret_cast<float4*>(px[i] + off) = v;
                    am = fmaxf(am, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
                }
            }
        if (amax) block_amax_commit(am, amax);
    }
};

struct EpiConvT2x2 {  // row m = (n,h,w) input pixel, col = ij*Co + co  ->  y[n, 2h+i, 2w+j, co] = acc + b[co]
    float* y; long long ldy; const float* bias; int H, W, Co, M, N;
    float* amax = nullptr;       // optional running max|y| (block_amax_commit)
    // Integer divisions only per lane and row block / column (6 per lane, not 2 per element: the per-element form
    // spent more issue cycles on v_rcp_iflag / v_mul_lo sequences than the K = Cin main loop on MFMAs).  The 16 rows
    // of an accumulator are mw + 32 i + 4 (lane >> 5) + {0..3, 8..11, 16..19, 24..27}: (b, h, w) advance by carry.
    __device__ __forceinline__ void operator()(f32x16 (&acc)[2][2], int mw, int nw, int lane, int, int,
                                               float*, int) const {
        float am = 0.f;
        const int hw = H * W;
        long long coff[2];   // output offset of column n inside its 2x2 block: (ij >> 1) rows, (ij & 1) pixels, co
        float bj[2];
        bool nok[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = nw + 32 * j + (lane & 31);
            nok[j] = n < N;
            const int ij = nok[j] ? n / Co : 0, co = nok[j] ? n - ij * Co : 0;
            coff[j] = ((long long)(ij >> 1) * (2 * W) + (ij & 1)) * ldy + co;
            bj[j] = bias ? bias[co] : 0.f;
        }
        if ((W == 16 || W % 32 == 0) && hw % 32 == 0 && mw + 64 <= M && nw + 64 <= N) {
            // (round 6) the wave's two 32-pixel row blocks each lie in one image and span at most two input rows (W =
            // 16: rows d < 16 and d >= 16; W >= 32: one row), so element r of a lane is its row block's first pixel
            // plus a wave-uniform output offset: one 64-bit lane pointer per row block, scalar offsets per element
            // (the carry walk below formed a 64-bit index product per element)
            const int mu = __builtin_amdgcn_readfirstlane(mw);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int mb = mu + 32 * i + 4 * (lane >> 5);
                const int b = mb / hw, rem = mb - b * hw, h = rem / W, w = rem - h * W;
                const float* pl0 = y + ((long long)(b * 2 * H + 2 * h) * (2 * W) + 2 * w) * ldy;
                float* pl = const_cast<float*>(pl0);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int d = (r & 3) + 8 * (r >> 2);
                    const long long dd = (W >= 32 || d < 16) ? 2 * d : 4 * W + 2 * (d - 16);   // output pixels
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const float v = acc[i][j][r] + bj[j];
                        pl[dd * ldy + coff[j]] = v;
                        am = fmaxf(am, fabsf(v));
                    }
                }
            }
            if (amax) block_amax_commit(am, amax);
            return;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int mb = mw + 32 * i + 4 * (lane >> 5);
            int b = mb / hw;
            const int rem = mb - b * hw;
            int h = rem / W, w = rem - h * W;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int d = (r & 3) + 8 * (r >> 2);
                if (r > 0) {
                    w += d - ((r - 1) & 3) - 8 * ((r - 1) >> 2);
                    while (w >= W) {
                        w -= W;
                        if (++h == H) { h = 0; ++b; }
                    }
                }
                if (mb + d < M) {
                    const long long pb = ((long long)(b * 2 * H + 2 * h) * (2 * W) + 2 * w) * ldy;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        if (nok[j]) {
                            const float v = acc[i][j][r] + bj[j];
                            y[pb + coff[j]] = v;
                            am = fmaxf(am, fabsf(v));
                        }
                    }
                }
            }
        }
        if (amax) block_amax_commit(am, amax);
    }
};

// ============================== the main loop ==============================
template <class LA, class LB, class EP, bool A_MCONTIG, int BK, bool XCD_REMAP = false>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_f32_kernel(LA la, LB lb, EP ep, int K, int kt_per_split) {
    constexpr int PADA = A_MCONTIG ? 4 : 2;   // k-major A image: stride == 2 (mod 32) -> conflict-free b32 transpose writes
    constexpr int SA = GBM + PADA, SB = GBN + 4;
    constexpr int A_LD = GBM * BK / 4 / GTHREADS;
    constexpr int B_LD = GBN * BK / 4 / GTHREADS;
    constexpr int TPR = BK / 4;               // threads per A row in the k-contiguous loader
    __shared__ __attribute__((aligned(16))) float smem[2 * BK * SA + 2 * BK * SB];
    float (*As)[BK][SA] = reinterpret_cast<float (*)[BK][SA]>(smem);
    float (*Bs)[BK][SB] = reinterpret_cast<float (*)[BK][SB]>(smem + 2 * BK * SA);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    int bx = blockIdx.x;
    if constexpr (XCD_REMAP) {   // blocks b, b+8, ... share an XCD: give each XCD a contiguous run of M tiles
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = bx & 7, j = bx >> 3;
        bx = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    const int m0 = bx * GBM, n0 = blockIdx.y * GBN;
    const int ktiles = (K + BK - 1) / BK;
    const int kt0 = blockIdx.z * kt_per_split;
    const int kt1 = min(ktiles, kt0 + kt_per_split);

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[A_LD], rb[B_LD];
    // per-thread fixed coordinates (row / column decompositions hoisted out of the K loop)
    typename LB::Col bcol = lb.col(n0 + (tid % 32) * 4);
    [[maybe_unused]] auto arows = [&]() {
        if constexpr (!A_MCONTIG) {
            struct Rows { typename LA::Row r[A_LD]; } rs;
#pragma unroll
            for (int i = 0; i < A_LD; ++i) rs.r[i] = la.row(m0 + tid / TPR + i * (GTHREADS / TPR));
            return rs;
        } else {
            return 0;
        }
    }();
    auto gload = [&](int kt) {
        const int k0 = kt * BK;
        if constexpr (!A_MCONTIG) {
#pragma unroll
            for (int i = 0; i < A_LD; ++i) ra[i] = la.load(arows.r[i], k0 + (tid % TPR) * 4);
        } else {
#pragma unroll
            for (int i = 0; i < A_LD; ++i) ra[i] = la.loadT(k0 + tid / 32 + i * 8, m0 + (tid % 32) * 4);
        }
#pragma unroll
        for (int i = 0; i < B_LD; ++i) rb[i] = lb.load(bcol, k0 + tid / 32 + i * 8);
    };
    auto sstore = [&](int buf) {
        if constexpr (!A_MCONTIG) {
#pragma unroll
            for (int i = 0; i < A_LD; ++i) {
                const int rr = tid / TPR + i * (GTHREADS / TPR), kq = (tid % TPR) * 4;
                As[buf][kq + 0][rr] = ra[i].x; As[buf][kq + 1][rr] = ra[i].y;
                As[buf][kq + 2][rr] = ra[i].z; As[buf][kq + 3][rr] = ra[i].w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < A_LD; ++i) st4(&As[buf][tid / 32 + i * 8][(tid % 32) * 4], ra[i]);
        }
#pragma unroll
        for (int i = 0; i < B_LD; ++i) st4(&Bs[buf][tid / 32 + i * 8][(tid % 32) * 4], rb[i]);
    };

    if (kt0 < kt1) { gload(kt0); sstore(0); }
    __syncthreads();
    int cur = 0;
    const int am = wm * 64 + (lane & 31), bn = wn * 64 + (lane & 31), kh = lane >> 5;
    for (int kt = kt0; kt < kt1; ++kt) {
        const bool more = kt + 1 < kt1;
        if (more) gload(kt + 1);
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const float a0 = As[cur][kk + kh][am], a1 = As[cur][kk + kh][am + 32];
            const float b0 = Bs[cur][kk + kh][bn], b1 = Bs[cur][kk + kh][bn + 32];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (more) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    ep(acc, m0 + wm * 64, n0 + wn * 64, lane, wm, wn, smem, tid);
}

template <class LA, class LB, class EP, bool A_MCONTIG, int BK = 16, bool XCD_REMAP = false>
static int launch_gemm(const LA& la, const LB& lb, const EP& ep, int M, int N, int K, int splits, hipStream_t s) {
    const int ktiles = (K + BK - 1) / BK;
    if (splits < 1) splits = 1;
    if (splits > ktiles) splits = ktiles > 0 ? ktiles : 1;
    const int per = (ktiles + splits - 1) / splits;
    splits = ktiles > 0 ? (ktiles + per - 1) / per : 1;
    dim3 grid((M + GBM - 1) / GBM, (N + GBN - 1) / GBN, splits);
    hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, EP, A_MCONTIG, BK, XCD_REMAP>), grid, dim3(GTHREADS), 0, s, la, lb, ep, K,
                       per);
    return cdm_status();
}

// split count actually used by launch_gemm for a requested value (host helper, mirrored in Python)
static int effective_splits(int K, int splits, int BK = 16) {
    const int ktiles = (K + BK - 1) / BK;
    if (splits < 1) splits = 1;
    if (splits > ktiles) splits = ktiles > 0 ? ktiles : 1;
    const int per = (ktiles + splits - 1) / splits;
    return ktiles > 0 ? (ktiles + per - 1) / per : 1;
}

// ============================== split-bf16 main loop (fp32-accurate, bf16 MFMA) ==============================
// fp32 GEMM on the bf16 matrix cores: every fp32 operand x is split into bf16 terms
//   x = hi + mid + lo (+ <= 2^-24 |x|),  hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid)
// and a.b is accumulated (fp32, in the MFMA) from the NT largest cross terms, smallest first:
//   NT = 6: mm, lh, hl, mh, hm, hh    (dropped: ml, lm, ll <= 2^-24 |ab|  -> fp32-class error)
//   NT = 3: mh, hm, hh                (~2^-16 relative; bf16x3)
//   NT = 1: hh                        (plain bf16 operands, fp32 accumulate)
//   NT = 4 (NT_H3): fp16 two-term split, 3 products on v_mfma_f32_32x32x16_f16 (fp32-class, see below)
// NT_H3: x is first scaled by a per-tensor power of two s = 2^(14 - e), max|x| < 2^e (exact), so the
// whole tensor sits inside fp16's normal range, then x*s = hi + lo + O(2^-22 |x*s|) with hi = f16(x*s),
// lo = f16(x*s - hi): 11 + 11 significand bits.  a.b ~ hh + hl + lh (dropped ll <= 2^-22 |ab|); the
// accumulator is multiplied back by 1/(s_a s_b) (exact).  Representation error per product is 2^-22
// relative vs fp32's 2^-24 rounding of each product — below the fp32 accumulation error of a K >= 64
// dot product — at half the matrix-core work of NT = 6.  max|x| comes from cdm_amax_f32 (device scalar,
// read by the kernel: no host sync).  Elements < 2^-28 max|x| lose significand bits (fp16 subnormals);
// their absolute error stays < 2^-39 max|x|.
// v_mfma_f32_32x32x16_bf16 retires 16x the MACs of v_mfma_f32_32x32x2_f32 per cycle, so NT = 6 moves
// 2.67x the fp32-MFMA rate through the matrix cores.
// LDS images are [term][row][16 k] bf16, 32 bytes per row, no padding; the two 16-byte k-halves of a
// row are XOR-swizzled by row bit 3 (xoff below).  With the gfx950 LDS lane groups this makes every
// access conflict-free: fragment ds_read_b128 (4 x 16 lanes, 256-byte banks), the A ds_write_b64
// (4 x 16 lanes = 4 rows x 32 B, 128-byte banks) and the B / k-strided ds_write_b128 (8 x 8 lanes = 4 rows
// x 2 halves).  (PMC on the previous 48-byte padded stride: 33 % of LDS cycles were bank conflicts.)
// Operand stagers (global -> registers -> split -> LDS), one per operand:
//   StageRowK  rows are k-contiguous fp32 (im2col / dense A): float4 along k, split, ds_write_b64 x terms
//   StagePre   pre-split bf16 [K/16][3][rows][16] (packed weights, cdm_split_bf16x3): 16-byte copies
//   StageColK  k-strided fp32 (wgrad: k = pixel, rows = channels): 8 scalar loads along k at one row
//              (lanes on consecutive rows -> coalesced), split, ds_write_b128 x terms
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
// 16-byte staging registers: a native vector, not HIP's uint4 struct — a struct copy lowers to a memcpy that SROA
// leaves in an alloca, which AMDGPUPromoteAlloca then moves into LDS (every staged piece took a global -> LDS slot ->
// register -> LDS round trip with a vmcnt(0) wait next to its load)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int NT_H3 = 4;

// the power-of-two operand scale of NT_H3 (1 for the bf16 arithmetics or a missing / degenerate max)
template <int NT>
static __device__ __forceinline__ float op_scale(const float* amax) {
    if constexpr (NT != NT_H3) {
        return 1.f;
    } else {
        if (!amax) return 1.f;
        const float m = *amax;
        if (!(m > 0.f) || m > 3.0e38f) return 1.f;
        int e;
        frexpf(m, &e);                               // m = f 2^e, f in [0.5, 1)  ->  m 2^(14-e) < 2^14
        return ldexpf(1.f, min(126, max(-126, 14 - e)));
    }
}

// one 32x32x16 product on the matrix cores in the arithmetic NT (operands are 16-bit images either way)
template <int NT>
static __device__ __forceinline__ f32x16 xmfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
    if constexpr (NT == NT_H3)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// acc *= 1 / (s_a s_b) for NT_H3 (two exact power-of-two multiplies)
template <int NT>
static __device__ __forceinline__ void unscale(f32x16 (&acc)[2][2], float sa, float sb) {
    if constexpr (NT == NT_H3) {
        const float ia = 1.f / sa, ib = 1.f / sb;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = (acc[i][j][r] * ia) * ib;
    }
}
constexpr int XBK = 16;
constexpr int XPLANE = GBM * XBK;     // elements per term plane (GBM == GBN == 128 rows x 16 k)

// element offset of (row, k) in a term plane: 16 bf16 per row, k-halves swapped on odd row-octets
static __device__ __forceinline__ int xoff(int row, int k) {
    return row * XBK + ((((k >> 3) ^ (row >> 3)) & 1) << 3) + (k & 7);
}

template <int NT> struct XTerms { static constexpr int NS = NT >= 6 ? 3 : (NT >= 3 ? 2 : 1); };

// x -> NS 16-bit terms (bf16 hi/mid/lo, or for NT_H3 the fp16 hi/lo of x * sc, bit-stored as __bf16)
template <int NT, int E>
static __device__ __forceinline__ void split_terms(const float (&x)[E], float sc, __bf16 (&h)[E], __bf16 (&m)[E],
                                                   __bf16 (&l)[E]) {
    constexpr int NS = XTerms<NT>::NS;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if constexpr (NT == NT_H3) {
            const float v = x[e] * sc;
            const _Float16 hi = (_Float16)v;
            h[e] = __builtin_bit_cast(__bf16, hi);
            m[e] = __builtin_bit_cast(__bf16, (_Float16)(v - (float)hi));
        } else {
            h[e] = (__bf16)x[e];
            if constexpr (NS > 1) {
                const float r = x[e] - (float)h[e];
                m[e] = (__bf16)r;
                if constexpr (NS > 2) l[e] = (__bf16)(r - (float)m[e]);
            }
        }
    }
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// h3 split of the pair (a, b), packed as the LDS images hold it (low half = a): hi = f16(sc x), lo = f16(sc x - hi),
// each by one v_fma_mix{lo,hi}_f16 that forms the scaled product inside the instruction and writes its packed half
// directly: 4 VALU per pair.  The compiler's own code for split_terms<NT_H3> + packing rounded hi twice (a mix for the
// residual, a v_cvt_pk_f16_f32 of two separately multiplied products for the store: 7 VALU per pair; round 6).  The
// same roundings (sc x is exact: sc is a power of two; each term is one RNE fp16 rounding of an exact fma), so the
// terms are bit-identical to split_terms<NT_H3> except hi(-0) = +0 (value-equal).
static __device__ __forceinline__ void h3_pair(float a, float b, float sc, unsigned& hp, unsigned& lp) {
    asm("v_fma_mixlo_f16 %0, %2, %3, 0\n\t"
        "v_fma_mixhi_f16 %0, %2, %4, 0\n\t"
        "v_fma_mixlo_f16 %1, %2, %3, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %1, %2, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(hp), "=&v"(lp)
        : "v"(sc), "v"(a), "v"(b));
}

// x[0..3] (4 consecutive k of one row) -> its NS term images, 2 elements per dword: t[term] = {k0 | k1, k2 | k3}
template <int NT>
static __device__ __forceinline__ void split_pk4(const float (&x)[4], float sc, u32x2 (&t)[3]) {
    if constexpr (NT == NT_H3) {
        unsigned h0, h1, l0, l1;
        h3_pair(x[0], x[1], sc, h0, l0);
        h3_pair(x[2], x[3], sc, h1, l1);
        t[0] = u32x2{h0, h1};
        t[1] = u32x2{l0, l1};
    } else {
        constexpr int NS = XTerms<NT>::NS;
        __bf16 h[4], m[4], l[4];
        split_terms<NT>(x, sc, h, m, l);
        t[0] = __builtin_bit_cast(u32x2, bf16x4{h[0], h[1], h[2], h[3]});
        if constexpr (NS > 1) t[1] = __builtin_bit_cast(u32x2, bf16x4{m[0], m[1], m[2], m[3]});
        if constexpr (NS > 2) t[2] = __builtin_bit_cast(u32x2, bf16x4{l[0], l[1], l[2], l[3]});
    }
}

template <class LD, int NT>
struct StageRowK {
    static constexpr int NS = XTerms<NT>::NS;
    static constexpr int LDN = GBM * XBK / 4 / GTHREADS;   // 2 float4 per thread
    LD ld;
    const float* amax;
    float sc;
    typename LD::Row row[LDN];
    float4 r[LDN];
    __device__ __forceinline__ float sc_of() const { return op_scale<NT>(amax); }
    __device__ __forceinline__ void init(int tid, int r0) {
        sc = op_scale<NT>(amax);
#pragma unroll
        for (int i = 0; i < LDN; ++i) row[i] = ld.row(r0 + tid / 4 + i * (GTHREADS / 4));
    }
    __device__ __forceinline__ void gload(int tid, int kt) {
#pragma unroll
        for (int i = 0; i < LDN; ++i) r[i] = ld.load(row[i], kt * XBK + (tid % 4) * 4);
    }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int i = 0; i < LDN; ++i) r[i] = f4zero();
    }
    __device__ __forceinline__ void sstore(int tid, __bf16* base) const {
#pragma unroll
        for (int i = 0; i < LDN; ++i) {
            const float x[4] = {r[i].x, r[i].y, r[i].z, r[i].w};
            u32x2 tm[3];
            split_pk4<NT>(x, sc, tm);
            __bf16* d = base + xoff(tid / 4 + i * (GTHREADS / 4), (tid % 4) * 4);
#pragma unroll
            for (int k = 0; k < NS; ++k) *reinterpret_cast<u32x2*>(d + k * XPLANE) = tm[k];
        }
    }
};

template <int NT>
struct StagePre {
    static constexpr int NS = XTerms<NT>::NS;
    const __bf16* p; int rows;           // [ktiles][3][rows][16]
    const float* amax;                   // NT_H3: max|W| the terms were split with (cdm_split_f16x2)
    float sc;
    int rr, kh; bool ok;
    u32x4 r[NS];
    __device__ __forceinline__ float sc_of() const { return op_scale<NT>(amax); }
    __device__ __forceinline__ void init(int tid, int r0) {
        sc = op_scale<NT>(amax);
        rr = r0 + (tid >> 1); kh = (tid & 1) * 8; ok = rr < rows;
    }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int t = 0; t < NS; ++t) r[t] = u32x4{0, 0, 0, 0};
    }
    __device__ __forceinline__ void gload(int, int kt) {
#pragma unroll
        for (int t = 0; t < NS; ++t)
            r[t] = ok ? *reinterpret_cast<const u32x4*>(p + (((long long)kt * 3 + t) * rows + rr) * XBK + kh)
                      : u32x4{0, 0, 0, 0};
    }
    __device__ __forceinline__ void sstore(int tid, __bf16* base) const {
        __bf16* d = base + xoff(tid >> 1, (tid & 1) * 8);
#pragma unroll
        for (int t = 0; t < NS; ++t) *reinterpret_cast<u32x4*>(d + t * XPLANE) = r[t];
    }
};

template <class LD, int NT>
struct StageColK {
    static constexpr int NS = XTerms<NT>::NS;
    LD ld;
    const float* amax;
    float sc;
    typename LD::Col col;
    float r[8];
    // thread -> (row tid>>1, k-half tid&1): an 8-lane store group covers 4 rows x 2 halves (conflict-free)
    __device__ __forceinline__ float sc_of() const { return op_scale<NT>(amax); }
    __device__ __forceinline__ void init(int tid, int r0) { sc = op_scale<NT>(amax); col = ld.col(r0 + (tid >> 1)); }
    __device__ __forceinline__ void gload(int tid, int kt) { ld.load8(col, kt * XBK + (tid & 1) * 8, r); }
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = 0.f;
    }
    __device__ __forceinline__ void sstore(int tid, __bf16* base) const {
        __bf16 h[8], m[8], l[8];
        split_terms<NT>(r, sc, h, m, l);
        __bf16* d = base + xoff(tid >> 1, (tid & 1) * 8);
        *reinterpret_cast<bf16x8*>(d) = bf16x8{h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]};
        if constexpr (NS > 1)
            *reinterpret_cast<bf16x8*>(d + XPLANE) = bf16x8{m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]};
        if constexpr (NS > 2)
            *reinterpret_cast<bf16x8*>(d + 2 * XPLANE) = bf16x8{l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7]};
    }
};

// SA: operand A stager (rows = M), SB: operand B stager (rows = N); split-K over blockIdx.z.  KS 16-deep K
// tiles share one barrier interval (one stager copy per tile; tiles past the split's end are zero-filled).
// (KS = 2 measured: ConvT 2x2 fwd 602 -> 695 us, 64 KiB LDS costs a block per CU — KS = 1 ships)
// order == 1 (operand-sharing block order): the flat block id, dealt round-robin over the 8 XCDs by the dispatcher,
// is remapped XCD-contiguous and decomposed column-tile fastest, then row tile, then K split, so the blocks that
// read the same A rows (and, split-K, the same K range of B) run together on one XCD and share its L2: with the
// grid's natural order (column tile = blockIdx.y, dispatched after every row tile) A was re-read from HBM once per
// column tile.  order == 0: XCD_REMAP of the row tile only (the previous schedule).
// MINB: the launch-bounds minimum of resident blocks (2: the compiler settles at 3 waves per SIMD, 155 VGPRs; 4: 4
// waves per SIMD, <= 128 VGPRs — the ConvT forward fits without spills).
template <class SA, class SB, class EP, int NT, bool XCD_REMAP, int KS = 1, int MINB = 2>
__global__ __launch_bounds__(GTHREADS, MINB) void gemm_x3_kernel(SA sa0, SB sb0, EP ep, int K, int kt_per_split,
                                                              int order) {
    constexpr int NS = XTerms<NT>::NS;
    constexpr int TILE = NS * XPLANE;                 // bf16 per operand per K tile
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * KS * TILE];
    __bf16* As = smem;                        // [buf][ks][term][row][16 k] (xoff swizzle)
    __bf16* Bs = smem + 2 * KS * TILE;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (order == 1) {
        const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
        const int L = bx + gx * (by + gy * bz), q = nwg >> 3, r = nwg & 7, xcd = L & 7, j = L >> 3;
        int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
        by = l % gy; l /= gy;
        bx = l % gx; bz = l / gx;
    } else if constexpr (XCD_REMAP) {
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = bx & 7, j = bx >> 3;
        bx = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
    }
    const int m0 = bx * GBM, n0 = by * GBN;
    const int ktiles = (K + XBK - 1) / XBK;
    const int kt0 = bz * kt_per_split;
    const int kt1 = min(ktiles, kt0 + kt_per_split);

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    SA sa[KS];
    SB sb[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        sa[ks] = sa0; sb[ks] = sb0;
        sa[ks].init(tid, m0); sb[ks].init(tid, n0);
    }
    auto gload = [&](int kt) {          // K tiles kt .. kt+KS-1 (zeros past the split's end)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (kt + ks < kt1) { sa[ks].gload(tid, kt + ks); sb[ks].gload(tid, kt + ks); }
            else { sa[ks].zero(); sb[ks].zero(); }
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            sa[ks].sstore(tid, As + (buf * KS + ks) * TILE);
            sb[ks].sstore(tid, Bs + (buf * KS + ks) * TILE);
        }
    };
    if (kt0 < kt1) { gload(kt0); sstore(0); }
    __syncthreads();
    int cur = 0;
    const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31), kh = (lane >> 5) * 8;
    int aoff[2], boff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) { aoff[i] = xoff(ar + 32 * i, kh); boff[i] = xoff(br + 32 * i, kh); }
    for (int kt = kt0; kt < kt1; kt += KS) {
        const bool more = kt + KS < kt1;
        if (more) gload(kt + KS);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const __bf16* a = As + (cur * KS + ks) * TILE;
            const __bf16* b = Bs + (cur * KS + ks) * TILE;
            bf16x8 fa[2][NS], fb[2][NS];
#pragma unroll
            for (int t = 0; t < NS; ++t)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    fa[i][t] = *reinterpret_cast<const bf16x8*>(a + t * XPLANE + aoff[i]);
                    fb[i][t] = *reinterpret_cast<const bf16x8*>(b + t * XPLANE + boff[i]);
                }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    f32x16 c = acc[i][j];
                    if constexpr (NT >= 6) {
                        c = xmfma<NT>(fa[i][1], fb[j][1], c);   // mm
                        c = xmfma<NT>(fa[i][2], fb[j][0], c);   // lh
                        c = xmfma<NT>(fa[i][0], fb[j][2], c);   // hl
                    }
                    if constexpr (NT >= 3) {
                        c = xmfma<NT>(fa[i][1], fb[j][0], c);   // mh (NT_H3: lo.hi)
                        c = xmfma<NT>(fa[i][0], fb[j][1], c);   // hm (NT_H3: hi.lo)
                    }
                    acc[i][j] = xmfma<NT>(fa[i][0], fb[j][0], c);  // hh
                }
        }
        if (more) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    unscale<NT>(acc, sa0.sc_of(), sb0.sc_of());
    EP e = ep;
    if constexpr (IsEpiStoreW<EP>::value) { e.y += (long long)bz * e.zstride; e.zstride = 0; }   // this split's slab
    e(acc, m0 + wm * 64, n0 + wn * 64, lane, wm, wn, reinterpret_cast<float*>(smem), tid);
}

// Dense-A x pre-split-B GEMM with a two-deep register prefetch (the ConvT 2x2 forward: K = Cin = 256 / 512, so a
// block's whole life is 16-32 K tiles, and gemm_x3's one-deep prefetch left every tile waiting on the HBM latency of
// the A loads issued one tile earlier — 12 MFMAs per wave per tile cannot cover it).  Tiles kt + 1 and kt + 2 are
// in flight while tile kt computes: two register sets, the loop unrolled by two so each set has a fixed role.
// Same block tile, LDS images, fragment order and MFMA order per K tile as gemm_x3_kernel<StageRowK<LdDenseA>,
// StagePre> (bit-identical results); every load unconditional (M % 128 == 0, N % 128 == 0, K % 32 == 0: the
// host checks), the last tiles re-load tile nk - 1 instead of branching.
// AL: the A addresses — base(m) the row's origin, off(kt) the block-uniform element offset of K tile kt (16 k)
struct DeepDenseA {          // A[m][k] = a[m lda + k]
    const float* a; long long lda;
    __device__ __forceinline__ const float* base(int m) const { return a + (long long)m * lda; }
    __device__ __forceinline__ long long off(int kt) const { return (long long)kt * XBK; }
};
struct DeepConvT2x2GatherA { // the ConvT 2x2 input gradient (LdConvT2x2GatherA): m = (n, h, w), k = (i 2 + j) Co + co
    const float* dy; int H, W, Co; long long lddy;
    __device__ __forceinline__ const float* base(int m) const {
        const int hw = H * W, n = m / hw, rem = m - n * hw, h = rem / W, w = rem - h * W;
        return dy + ((long long)(n * 2 * H + 2 * h) * (2 * W) + 2 * w) * lddy;
    }
    __device__ __forceinline__ long long off(int kt) const {   // a 16-k tile lies in one sub-pixel (Co % 16 == 0)
        const int k0 = kt * XBK, ij = k0 / Co, co = k0 - ij * Co;
        return ((long long)(ij >> 1) * (2 * W) + (ij & 1)) * lddy + co;
    }
};
// TRO (round 6): the MFMAs take B as their first operand, so each accumulator holds the tile transposed — a lane keeps one
// row m (pixel) and, for r = 4q..4q+3, four consecutive columns n: the epilogue (EpiConvT2x2T) stores 16 bytes per
// instruction instead of 4 (the scatter epilogue issued 64 dword stores per lane per tile, which nothing overlapped)
template <int NT, class AL, class EP, int MINB, bool TRO = false>
__global__ __launch_bounds__(GTHREADS, MINB) void gemm_deep_kernel(AL al, const __bf16* __restrict__ bp, int N,
                                                                  const float* amax_a, const float* amax_b, EP ep,
                                                                  int K) {
    constexpr int NS = XTerms<NT>::NS;
    constexpr int TILE = NS * XPLANE;
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * 2 * TILE];
    __bf16* As = smem;                 // [buf][term][row][16 k] (xoff swizzle)
    __bf16* Bs = smem + 2 * TILE;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // operand-sharing order (gemm_x3 order 1): XCD-contiguous flat ids, column tile fastest
    const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy;
    int bx, by;
    {
        const int L = blockIdx.x + gx * blockIdx.y, q = nwg >> 3, r = nwg & 7, xcd = L & 7, j = L >> 3;
        const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
        by = l % gy; bx = l / gy;
    }
    const int m0 = bx * GBM, n0 = by * GBN, nk = K / XBK;
    const float sa = op_scale<NT>(amax_a), sb = op_scale<NT>(amax_b);
    const float* arow[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) arow[i] = al.base(m0 + tid / 4 + i * (GTHREADS / 4)) + (tid % 4) * 4;
    const __bf16* brow = bp + (long long)(n0 + (tid >> 1)) * XBK + (tid & 1) * 8;
    const long long bstride = (long long)N * XBK;   // one term plane of a K tile ([ktiles][3][N][16])
    struct Regs { float4 a[2]; u32x4 b[NS]; };
    auto gload = [&](Regs& R, int kt) {
        const long long ko = al.off(kt);
#pragma unroll
        for (int i = 0; i < 2; ++i) R.a[i] = ld4(arow[i] + ko);
#pragma unroll
        for (int t = 0; t < NS; ++t) R.b[t] = *reinterpret_cast<const u32x4*>(brow + ((long long)kt * 3 + t) * bstride);
    };
    auto sstore = [&](const Regs& R, int buf) {
        __bf16* ab = As + buf * TILE;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float x[4] = {R.a[i].x, R.a[i].y, R.a[i].z, R.a[i].w};
            __bf16 h[4], m[4], l[4];
            split_terms<NT>(x, sa, h, m, l);
            __bf16* d = ab + xoff(tid / 4 + i * (GTHREADS / 4), (tid % 4) * 4);
            *reinterpret_cast<bf16x4*>(d) = bf16x4{h[0], h[1], h[2], h[3]};
            if constexpr (NS > 1) *reinterpret_cast<bf16x4*>(d + XPLANE) = bf16x4{m[0], m[1], m[2], m[3]};
            if constexpr (NS > 2) *reinterpret_cast<bf16x4*>(d + 2 * XPLANE) = bf16x4{l[0], l[1], l[2], l[3]};
        }
        __bf16* d = Bs + buf * TILE + xoff(tid >> 1, (tid & 1) * 8);
#pragma unroll
        for (int t = 0; t < NS; ++t) *reinterpret_cast<u32x4*>(d + t * XPLANE) = R.b[t];
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31), kh = (lane >> 5) * 8;
    int aoff[2], boff[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) { aoff[i] = xoff(ar + 32 * i, kh); boff[i] = xoff(br + 32 * i, kh); }
    auto mm = [&](int buf) {
        const __bf16* ab = As + buf * TILE;
        const __bf16* bb = Bs + buf * TILE;
        bf16x8 fa[2][NS], fb[2][NS];
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                fa[i][t] = *reinterpret_cast<const bf16x8*>(ab + t * XPLANE + aoff[i]);
                fb[i][t] = *reinterpret_cast<const bf16x8*>(bb + t * XPLANE + boff[i]);
            }
        auto mf = [&](const bf16x8& x, const bf16x8& w, const f32x16& c) {   // x: the A fragment (rows m)
            if constexpr (TRO) return xmfma<NT>(w, x, c);
            else return xmfma<NT>(x, w, c);
        };
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x16 c = acc[i][j];
                if constexpr (NT >= 6) {
                    c = mf(fa[i][1], fb[j][1], c);
                    c = mf(fa[i][2], fb[j][0], c);
                    c = mf(fa[i][0], fb[j][2], c);
                }
                if constexpr (NT >= 3) {
                    c = mf(fa[i][1], fb[j][0], c);
                    c = mf(fa[i][0], fb[j][1], c);
                }
                acc[i][j] = mf(fa[i][0], fb[j][0], c);
            }
    };
    Regs R0, R1;
    gload(R0, 0);
    gload(R1, 1);
    sstore(R0, 0);
    __syncthreads();
    // top of an iteration: LDS buffer 0 holds tile kt, R1 tile kt + 1 (in flight)
    for (int kt = 0; kt < nk; kt += 2) {
        gload(R0, min(kt + 2, nk - 1));
        mm(0);
        sstore(R1, 1);
        __syncthreads();
        gload(R1, min(kt + 3, nk - 1));
        mm(1);
        if (kt + 2 < nk) sstore(R0, 0);
        __syncthreads();
    }
    unscale<NT>(acc, sa, sb);
    ep(acc, m0 + wm * 64, n0 + wn * 64, lane, wm, wn, reinterpret_cast<float*>(smem), tid);
}

// $CDM_GEMM_MINB: 4 or 2 resident blocks per CU asked of the compiler; default 4 for h3 (profiles/r3_ab_gemm_minb.txt),
// 2 for the one-term bf16 arithmetic, whose 4-block form spills 51 VGPRs (with the bf16 knobs below, same-box A/B:
// C4 27.95-28.02 -> 27.73-27.75 ms per step, profiles/r4_ab_c4_knobs.txt)
static int gemm_minb(int nterm) {
    static const int v = [] { const char* e = getenv("CDM_GEMM_MINB"); return e ? atoi(e) : 0; }();
    return v > 0 ? v : (nterm == 1 ? 2 : 4);
}

static int gemm_order() {   // $CDM_GEMM_ORDER: 1 operand-sharing block order (default), 0 grid order
    static const int v = [] { const char* e = getenv("CDM_GEMM_ORDER"); return e ? atoi(e) : 1; }();
    return v;
}

// SA<NS>/SB<NS> are stager templates; splits as launch_gemm (K-tile ranges over blockIdx.z)
template <template <int> class SAT, template <int> class SBT, class EP, bool XCD_REMAP, class MkA, class MkB>
static int launch_gemm_x3(MkA mka, MkB mkb, const EP& ep, int M, int N, int K, int splits, int nterm,
                          hipStream_t s) {
    const int ktiles = (K + XBK - 1) / XBK;
    if (splits < 1) splits = 1;
    if (splits > ktiles) splits = ktiles > 0 ? ktiles : 1;
    const int per = (ktiles + splits - 1) / splits;
    splits = ktiles > 0 ? (ktiles + per - 1) / per : 1;
    dim3 grid((M + GBM - 1) / GBM, (N + GBN - 1) / GBN, splits);
    const int order = gemm_order();
    switch (nterm) {
        case 1:
            if (gemm_minb(1) == 4)
                hipLaunchKernelGGL((gemm_x3_kernel<SAT<1>, SBT<1>, EP, 1, XCD_REMAP, 1, 4>), grid, dim3(GTHREADS), 0, s,
                                   mka.template make<1>(), mkb.template make<1>(), ep, K, per, order);
            else
                hipLaunchKernelGGL((gemm_x3_kernel<SAT<1>, SBT<1>, EP, 1, XCD_REMAP>), grid, dim3(GTHREADS), 0, s,
                                   mka.template make<1>(), mkb.template make<1>(), ep, K, per, order);
            break;
        case 3: hipLaunchKernelGGL((gemm_x3_kernel<SAT<3>, SBT<3>, EP, 3, XCD_REMAP>), grid, dim3(GTHREADS), 0, s,
                                   mka.template make<3>(), mkb.template make<3>(), ep, K, per, order); break;
        case NT_H3:
            if (gemm_minb(NT_H3) == 4)
                hipLaunchKernelGGL((gemm_x3_kernel<SAT<NT_H3>, SBT<NT_H3>, EP, NT_H3, XCD_REMAP, 1, 4>), grid,
                                   dim3(GTHREADS), 0, s, mka.template make<NT_H3>(), mkb.template make<NT_H3>(), ep, K,
                                   per, order);
            else
                hipLaunchKernelGGL((gemm_x3_kernel<SAT<NT_H3>, SBT<NT_H3>, EP, NT_H3, XCD_REMAP>), grid,
                                   dim3(GTHREADS), 0, s, mka.template make<NT_H3>(), mkb.template make<NT_H3>(), ep, K,
                                   per, order);
            break;
        case 6: hipLaunchKernelGGL((gemm_x3_kernel<SAT<6>, SBT<6>, EP, 6, XCD_REMAP>), grid, dim3(GTHREADS), 0, s,
                                   mka.template make<6>(), mkb.template make<6>(), ep, K, per, order); break;
        default: return (int)hipErrorInvalidValue;
    }
    return cdm_status();
}

template <class LD> struct MkRowK {
    LD ld; const float* amax = nullptr;
    template <int NT> StageRowK<LD, NT> make() const { StageRowK<LD, NT> s; s.ld = ld; s.amax = amax; return s; }
};
template <class LD> struct MkColK {
    LD ld; const float* amax = nullptr;
    template <int NT> StageColK<LD, NT> make() const { StageColK<LD, NT> s; s.ld = ld; s.amax = amax; return s; }
};
struct MkPre {
    const __bf16* p; int rows; const float* amax = nullptr;
    template <int NT> StagePre<NT> make() const { StagePre<NT> s; s.p = p; s.rows = rows; s.amax = amax; return s; }
};
template <class LD> struct RowK { template <int NT> using T = StageRowK<LD, NT>; };
template <class LD> struct ColK { template <int NT> using T = StageColK<LD, NT>; };

// Optional staging pre-op of a conv operand.  PreBnBwd: the operand is dy of a Conv -> BatchNorm -> ReLU layer,
// computed while staging from the grad g of the ReLU output and the pre-norm activations y (bn_bwd_elem, the
// expression of norm_apply_bwd_kernel): dy is never written to HBM (no 537 MB write + 2 reads per layer).
struct PreNone { static constexpr bool on = false; static constexpr int kind = 0; };
struct PreBnBwd {
    static constexpr bool on = true;
    static constexpr int kind = 1;
    const float* y; int ldy;   // pre-norm activations [pix][C]
    const float* p[7];         // per channel: scale s, shift t, mean, invstd, A, B, Cc
    void* dyo = nullptr;       // LDS-halo dgrad only (optional): the dy it computes is also stored here, element type and
                               // row stride those of g, each element once (the block's own rows, column block 0), for
                               // the layer's weight gradient to read instead of recomputing it from g and y
};
// PreBnRelu: the operand is z = relu(y s + t) of a Conv -> BatchNorm -> ReLU layer (train mode), computed while
// staging from the layer's pre-norm output y: z is never written (the apply kernel's 537 MB write + read at 64^2).
// Zero padding stays zero (only in-image pieces are transformed).  Same fmaf as norm_apply_fwd: bit-identical.
struct PreBnRelu {
    static constexpr bool on = false;
    static constexpr int kind = 2;
    const float* p[2];         // per input channel: scale s, shift t
};
static __device__ __forceinline__ float bn_relu_elem(float y, float s, float t) { return relu_f(fmaf(y, s, t)); }
// PreBnReluSums (kernel-row weight gradient only): the X operand as PreBnRelu, and in addition the producer layer's
// BatchNorm-backward channel sums, accumulated while its pre-norm output y is staged anyway: with g = the gradient wrt
// relu(y s + t) (this conv's input, already written by this layer's dgrad), g_pre = (y s + t > 0 ? g : 0) and
// xhat = (y - mean) invstd:  S1 = sum g_pre, S2 = sum g_pre xhat, S5 = sum xhat per channel (the mode-0 sums of
// cdm_norm_bwd_reduce, whose pass over g and y this replaces).  Each X pixel is staged by the 3 kernel-row blocks x
// the co tiles of its split and summed by exactly one of them (spread evenly, see the kernel); one partial per block,
// sums[(split * 3 + ky) * gx + co tile][5][Cin] (rows 2, 3 zero).
struct PreBnReluSums {
    static constexpr bool on = false;
    static constexpr int kind = 3;
    const float* p[2];         // per input channel: scale s, shift t
    const float* g; int ldg;   // grad wrt this conv's input relu(y s + t)
    const float* mean; const float* invstd;
    float* sums;
};


// ============================== LDS-halo conv3x3 on the split-bf16 matrix cores ==============================
// conv3x3 (stride 1, pad 1) forward / dgrad for Cin % 16 == 0 (channel-chunk-major K, kc = 16) and image
// width WT in {32, 64} (128, 256 with the two-term h3 arithmetic).  A block owns tpb consecutive tiles of 256
// output pixels (a tile = 256/WT whole image rows) x 128 output channels, one tile after the other, 8 waves as 4 (M) x 2 (N), each wave 64x64.  Per 16-channel chunk the block stages its
// input rows plus the 1-pixel halo ((256/WT + 2) x (WT + 2) pixels x 16 ch) ONCE into LDS, split into
// bf16 terms, and the 9 taps of that chunk read their A fragments straight out of the halo tile at
// shifted addresses: no im2col re-reads (the generic path re-reads every input element 9x through
// L1/L2).  B (pre-split weights) streams one kernel row (3 taps, 36 KiB) per barrier, double-buffered,
// so each barrier interval holds 72 MFMAs per wave and the fragment reads of tap t+1 overlap the MFMAs
// of tap t; 256-row blocks halve the per-pixel weight re-reads of the 128-row kernel.
// LDS (x6, WT 64): halo 2 x 3 x 396 px x 32 B + B 2 x 3 taps x 3 terms x 4 KiB = 146 KiB (1 block / CU).
constexpr int HBM_ = 256;          // output pixels per block
constexpr int HTHREADS = 512;

// ABL: timing-ablation bits for tools/conv_ablation.py (1 = shipped for NS <= 2; x6 keeps 0: its registers do not fit
// the second fragment set): 1 fragment prefetch (the next
// tap's fragments are read during the current tap's MFMAs: 0.94 -> 0.84 ms), 2 every MFMA issued twice, 4 B
// staged once (stale afterwards), 8 halo stored without the term split, 16 no barriers in the main loop,
// 32 halo loaded for the first chunk only, 64 / 128 prefetch schedules: 2 reads per MFMA gap / all reads after the
// tap's first MFMA, 256 staggered halo split (waves 0-3 split + store the next chunk's halo after their last kernel
// row's MFMAs, waves 4-7 before them, so each SIMD pairs one wave's VALU with its partner's MFMAs), 512 static
// priority 1 for waves 4-7, 16384 epilogue skipped (behind a never-taken branch: the MFMAs stay live; round 6: 0.753 ->
// 0.672 ms at 16 tiles per block — the epilogue's 537 MB of y, stored by every block at the same time, drains at ~6.6
// TB/s with no MFMA running; issuing the next chunk's loads ahead of those stores measured slower, 0.822 -> 0.833 ms)
// XT: element type of the source x (and of PRE's y): bf16 for C4's fused-chain activations / gradients
template <int NT, int WT, class EP, bool XCD_REMAP, int ABL = (NT >= 6 ? 0 : 1), class PRE = PreNone, class XT = float>
__global__ __launch_bounds__((ABL & 8192) ? 256 : HTHREADS, 1) void conv3x3_halo_x3_kernel(const XT* __restrict__ x, int H, int Cin,
                                                                      int ldx, const __bf16* __restrict__ wx3,
                                                                      int Cout, const float* amax_x,
                                                                      const float* amax_w, EP ep, PRE pre,
                                                                      int mtiles, int tpb, int stgd = 0) {
    // stgd: bit 0 the staggered halo split (halo_stagger), bit 1 waves 4-7 at priority 1; bits 8+: the start delay of
    // every other block in 10 ns
    // ticks (halo_delay: desynchronises the blocks' epilogue store bursts)
    const int stg = stgd & 1;
    constexpr bool bearly = true;   // B of the next chunk's first kernel row fetched in row 1 (round 6, profiles/r6_ab_halo_bearly.txt)
    constexpr int NS = XTerms<NT>::NS;
    // TALL (ABL 8192, one bf16 term only): 4 waves (one per SIMD, 512 registers each: the accumulators live in AGPRs) as
    // 2 (M) x 2 (N) of 128 x 64 — 4 row blocks of 32 pixels per wave.  The one-term MFMA reads 1 KiB of fragments per
    // 32x32x16 product from LDS at 64 x 64 (the CU's LDS rate at full MFMA rate); 128 x 64 reads 0.75 KiB.  Same
    // 256-pixel x 128-channel block tile and LDS images as the 8-wave form; launched with 256 threads.  Measured (round
    // 4, profiles/r4_ab_halo_tall.txt): bit-identical C4 train steps, but 29.3 vs 27.5 ms — one wave per SIMD leaves
    // the staging and barrier waits uncovered (forward 64^2 414 vs 326 us).  Kept as an ablation bit, not dispatched.
    constexpr bool TALL = (ABL & 8192) != 0;
    static_assert(!TALL || NS == 1, "tall wave tiles: the one-term images only");
    constexpr int MI = TALL ? 4 : 2;                  // 32-row blocks per wave
    constexpr int NTH = TALL ? 256 : HTHREADS;        // threads per block
    constexpr int HB = HBM_;                          // output pixels per tile
    constexpr int ROWS = HB / WT, HR = ROWS + 2, HC = WT + 2, HPX = HR * HC;
    constexpr int HQ = (HPX * 4 + NTH - 1) / NTH;   // float4 halo pieces per thread
    // halo planes padded to HQ x 512 pieces where LDS allows: every piece then has a slot (past-the-halo pieces
    // write unused padding), so the split + store has no branches and can share a scheduling region with MFMAs
    constexpr int HPXA = HQ * NTH / 4;
    // ONEB (ABL 2048, one bf16 term only): B of all 9 taps of a chunk in one buffer, one barrier per chunk (36 MFMAs per
    // wave between barriers instead of 12; the one-term chunk is too short to pay three barrier drains)
    constexpr bool ONEB = (ABL & 2048) != 0;
    static_assert(!ONEB || NS == 1, "one barrier per chunk: the one-term images only");
    constexpr int BGR = ONEB ? 3 : 1;                 // B groups (kernel rows) per buffer
    // DEEP (ABL 4096, with ONEB, forward staging only): the halo of chunk q+2 is loaded while chunk q computes and
    // chunk q+1 (loaded one chunk earlier) is stored, so a halo load has two chunks to arrive instead of one (the
    // one-term chunk is short against HBM latency); two halo register sets, Cin % 32 == 0
    constexpr bool DEEP = (ABL & 4096) != 0;
    static_assert(!DEEP || (ONEB && !PRE::on), "two-deep halo prefetch: one-term forward staging only");
    constexpr bool HPAD = (2 * NS * HPXA * XBK + 2 * 3 * BGR * NS * XPLANE) * 2 + 7 * 256 * 4 <= 160 * 1024;
    constexpr int HPLANE = (HPAD ? HPXA : HPX) * XBK;   // bf16 per halo term plane
    constexpr int BPL = 3 * NS;                       // B planes per group (3 taps x NS terms)
    constexpr int BQ = (BGR * BPL * 256 + NTH - 1) / NTH;  // 16-byte B pieces per thread
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * NS * HPLANE + 2 * BGR * BPL * XPLANE];
    __bf16* Hs = smem;                                // [buf][term][halo pixel][16 ch] (xoff swizzle)
    __bf16* Bs = smem + 2 * NS * HPLANE;              // [buf][tap dx][term][col][16 k] (xoff swizzle)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    if ((ABL & 512) || (stgd & 2)) {   // static priority for the second-dispatched half (stgd bit 1: $CDM_HALO_PRIO)
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    // the block's tpb 256-pixel tiles, run one after the other: the next tile's first halo and B are fetched
    // during the current tile's last chunk, so only a block's first tile waits on HBM latency before its MFMAs.
    // XCD-aware: XCD x owns a contiguous tile range and its cnt blocks step through it together (tile
    // base + k * cnt + j), so the blocks running at one time hold consecutive tiles whose halo rows meet in L2
    // (tiles 2j, 2j+1 per block instead put the two rows shared by tiles 2j+1 and 2j+2 in different phases:
    // measured 1.6x the HBM fetch bytes)
    int t_first = blockIdx.x * tpb, t_step = 1;
    if constexpr (XCD_REMAP) {
        const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
        const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, cnt = xcd < r ? q + 1 : q;
        t_first = start * tpb + j;
        t_step = cnt;
    }
    if (t_first >= mtiles) return;   // cannot happen for grid.x = ceil(mtiles / tpb); uniform per block
    if (const unsigned dly = (unsigned)stgd >> 8; dly && ((blockIdx.x >> 3) & 1)) {
        // every other block of each XCD starts dly x 10 ns late (s_memrealtime: 100 MHz), so that half the CUs store
        // their tile's y while the other half compute (all blocks otherwise reach every epilogue together and the
        // chip's write bandwidth, not the MFMAs, paces those microseconds)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < dly) __builtin_amdgcn_s_sleep(4);
    }
    const int n0 = blockIdx.y * GBN;
    const int hw = H * WT;
    const int nchunks = Cin / 16, ngroups = nchunks * 3;
    const float sx = op_scale<NT>(amax_x);
    // BN-backward pre-op: the block's per-channel coefficients, staged once (Cin <= 256)
    constexpr int NCOEF = PRE::kind == 1 ? 7 : (PRE::kind == 2 ? 2 : 0);
    __shared__ __attribute__((aligned(16))) float bcs[NCOEF ? NCOEF * 256 : 4];
    if constexpr (NCOEF > 0) {
        for (int i = tid; i < NCOEF * Cin; i += NTH) {
            const int k = i / Cin;
            bcs[i] = pre.p[k][i - k * Cin];
        }
        __syncthreads();
    }

    f32x16 acc[MI][2];

    // ---- halo staging: piece q = (halo pixel q>>2, channels 4(q&3)..+3); addresses fixed per block ----
    // Every global load of the main loop is issued unconditionally (pieces outside the image load a valid dummy
    // address and are zeroed where they are stored): with loads under branches the compiler can no longer count
    // them and waits for vmcnt(0) — the B stores of a kernel row then waited on the next chunk's halo (HBM latency)
    // and the halo split on the B loads just issued.
    using RawX = typename Act<XT>::Raw;
    constexpr unsigned XSZ = sizeof(XT);
    RawX hreg[HQ];
    // chunk-0 source of piece j as a 32-bit byte offset from the uniform base x (pre.y): scalar base + lane offset
    // loads, one VGPR per piece instead of a 64-bit pointer (the PreBnBwd variant spilled with two pointers per piece).
    // Offsets stay below 2^32: the host checks N H W ldx * 4 bytes < 2^32 (cdm_conv3x3 entry points).
    unsigned hxo[HQ];               // (a dummy in-bounds offset 0 + channel quad when !hin[j])
    bool hin[HQ];                   // piece j is inside the image (else zero padding / past the halo)
    int hdst[HQ];                   // its LDS offset within a term plane
    RawX yreg[PRE::on ? HQ : 1];    // PreBnBwd: the pre-norm activations of piece j
    unsigned hyo[PRE::on ? HQ : 1];
    auto setup_tile = [&](int t) {  // halo source offsets of tile t
        const int m0 = t * HB, img = m0 / hw, h0 = (m0 - img * hw) / WT;
#pragma unroll
        for (int j = 0; j < HQ; ++j) {
            const int q = tid + j * NTH;
            const int hp = q >> 2, c4 = q & 3;
            const int hr = hp / HC, hc = hp - hr * HC;
            const int ih = h0 - 1 + hr, iw = hc - 1;
            const bool in = q < HPX * 4 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)WT;
            const unsigned pix = in ? (unsigned)((img * H + ih) * WT + iw) : 0u;
            hin[j] = in;
            hxo[j] = (pix * (unsigned)ldx + (unsigned)c4 * 4u) * XSZ;
            if constexpr (PRE::on) hyo[j] = (pix * (unsigned)pre.ldy + (unsigned)c4 * 4u) * XSZ;
        }
    };
#pragma unroll
    for (int j = 0; j < HQ; ++j) {
        const int q = tid + j * NTH;
        hdst[j] = (HPAD || q < HPX * 4) ? xoff(q >> 2, (q & 3) * 4) : -1;
    }
    setup_tile(t_first);
    // a halo register set and its in-image mask (DEEP: the mask travels with the set across a tile change)
    auto gload_halo_to = [&](RawX (&dst)[HQ], unsigned& mask, int cc) {
        const char* xb = reinterpret_cast<const char*>(x + cc * 16);
        mask = 0u;
#pragma unroll
        for (int j = 0; j < HQ; ++j) {
            dst[j] = Act<XT>::load4(xb + hxo[j]);
            mask |= (hin[j] ? 1u : 0u) << j;
        }
    };
    auto gload_halo = [&](int cc) {
        if constexpr (ABL & 32) {
            if (cc > 0) return;
        }
        const char* xb = reinterpret_cast<const char*>(x + cc * 16);
#pragma unroll
        for (int j = 0; j < HQ; ++j) hreg[j] = Act<XT>::load4(xb + hxo[j]);
        if constexpr (PRE::on) {
            const char* yb = reinterpret_cast<const char*>(pre.y) + (size_t)cc * 16 * XSZ;   // pre.y holds XT elements
#pragma unroll
            for (int j = 0; j < HQ; ++j) yreg[j] = Act<XT>::load4(yb + hyo[j]);
        }
    };
    // inb(j): piece j lies inside the image (else zero padding)
    auto store_halo_impl = [&](const RawX (&src)[HQ], auto inb, __bf16* base, int cc) {
        float cf[NCOEF ? NCOEF : 1][4];   // coefficients of this thread's 4 channels (q & 3 == tid & 3 for every j)
        if constexpr (NCOEF > 0) {
            const int cb = cc * 16 + (tid & 3) * 4;
#pragma unroll
            for (int k = 0; k < NCOEF; ++k) {
                const float4 v = *reinterpret_cast<const float4*>(bcs + k * Cin + cb);
                cf[k][0] = v.x; cf[k][1] = v.y; cf[k][2] = v.z; cf[k][3] = v.w;
            }
        }
#pragma unroll
        for (int j = 0; j < HQ; ++j) {
            if (HPAD || hdst[j] >= 0) {
                const float4 sv = Act<XT>::to4(src[j]);
                float xv[4] = {sv.x, sv.y, sv.z, sv.w};
                if constexpr (PRE::kind == 1) {
                    const float4 yv = Act<XT>::to4(yreg[j]);
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        xv[e] = bn_bwd_elem(xv[e], f4get(yv, e), cf[0][e], cf[1][e], cf[2][e], cf[3][e],
                                            cf[4][e], cf[5][e], cf[6][e]);
                    if (pre.dyo != nullptr && blockIdx.y == 0) {   // block-uniform
                        // piece j's halo pixel (hr, hc) is one of the tile's own output pixels: rows 1..ROWS, columns
                        // 1..WT of the halo (always inside the image); hxo[j] addresses it in g, same layout as dyo
                        const int q = tid + j * NTH, hp = q >> 2, hr = hp / HC, hc = hp - hr * HC;
                        if (q < HPX * 4 && hr >= 1 && hr <= ROWS && hc >= 1 && hc <= WT) {
                            char* o = reinterpret_cast<char*>(pre.dyo) + hxo[j] + (size_t)cc * 16 * XSZ;
                            if constexpr (std::is_same<XT, float>::value)
                                *reinterpret_cast<float4*>(o) = make_float4(xv[0], xv[1], xv[2], xv[3]);
                            else
                                *reinterpret_cast<bf16x4*>(o) = bf16x4{(__bf16)xv[0], (__bf16)xv[1], (__bf16)xv[2],
                                                                       (__bf16)xv[3]};
                        }
                    }
                } else if constexpr (PRE::kind == 2) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) xv[e] = bn_relu_elem(xv[e], cf[0][e], cf[1][e]);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) xv[e] = inb(j) ? xv[e] : 0.f;   // zero padding (transform not applied)
                u32x2 tm[3];
                if constexpr (ABL & 8) {
                    const u32x2 raw{__float_as_uint(xv[0]), __float_as_uint(xv[1])};
                    tm[0] = raw; tm[1] = u32x2{__float_as_uint(xv[2]), __float_as_uint(xv[3])}; tm[2] = raw;
                } else {
                    split_pk4<NT>(xv, sx, tm);
                }
                __bf16* d = base + hdst[j];
#pragma unroll
                for (int k = 0; k < NS; ++k) *reinterpret_cast<u32x2*>(d + k * HPLANE) = tm[k];
            }
        }
    };
    auto store_halo = [&](__bf16* base, int cc) { store_halo_impl(hreg, [&](int j) { return hin[j]; }, base, cc); };
    auto store_halo_set = [&](const RawX (&src)[HQ], unsigned mask, __bf16* base, int cc) {
        store_halo_impl(src, [&](int j) { return ((mask >> j) & 1u) != 0u; }, base, cc);
    };
    // ---- B staging: piece q = (plane q>>8 = dx*NS + t, col (q&255)>>1, k-half q&1) of group g ----
    // two register sets for B: the groups dy = 1 and dy = 2 of a chunk are both fetched at the chunk's start,
    // ahead of the next chunk's halo, so the per-group B waits never wait for the (HBM-latency) halo loads:
    // the halo has the whole chunk (3 barrier intervals) to arrive (vmcnt counts in issue order)
    u32x4 bregA[BQ], bregB[BQ];
    // unconditional loads (see the halo): a piece past the group loads an in-bounds dummy and is not stored; a
    // column >= Cout (Cout % 128 != 0) loads a copy of column Cout - 1: its accumulators are never stored (a select
    // here would be hoisted to the load by the scheduler and wait on it)
    // per-lane byte offsets of the pieces within a group (fixed per block); the group offset is uniform, so each
    // load is a scalar-base + 32-bit lane-offset address (no 64-bit multiplies in the loop)
    unsigned bpo[BQ];
#pragma unroll
    for (int j = 0; j < BQ; ++j) {
        const int q = tid + j * NTH;
        // ONEB: plane pl = kernel row * BPL + tap (NS == 1); group gr of the chunk at the global group stride
        const int plg = min(q >> 8, BGR * BPL - 1), gr = plg / BPL, pl = plg - gr * BPL;
        const int dx = pl / NS, t = pl - dx * NS, half = q & 1;
        const int n = min(n0 + ((q & 255) >> 1), Cout - 1);
        bpo[j] = (unsigned)((gr * 9 * Cout + (dx * 3 + t) * Cout + n) * XBK + half * 8) * 2u;
    }
    auto gload_b = [&](int g, u32x4 (&breg)[BQ]) {
        const char* gb = reinterpret_cast<const char*>(wx3) + (long long)g * (9 * XBK * 2) * Cout;
#pragma unroll
        for (int j = 0; j < BQ; ++j) breg[j] = *reinterpret_cast<const u32x4*>(gb + bpo[j]);
    };
    int bstores = 0;
    auto store_b = [&](int boff, const u32x4 (&breg)[BQ]) {   // into Bs + boff
        if constexpr (ABL & 4) {
            if (bstores++ >= 2) return;
        }
        // an opaque offset: the compiler can no longer prove the stores disjoint from the current kernel row's
        // fragment reads, so it keeps them after those reads instead of pulling them (and their load waits) up
        // among the first MFMAs
        asm volatile("" : "+s"(boff));
        __bf16* base = Bs + boff;
#pragma unroll
        for (int j = 0; j < BQ; ++j) {
            const int q = tid + j * NTH;
            if (q < BGR * BPL * 256)
                *reinterpret_cast<u32x4*>(base + (q >> 8) * XPLANE + xoff((q & 255) >> 1, (q & 1) * 8)) = breg[j];
        }
    };

    // per-lane halo pixel of each A fragment row (tap (0,0) origin)
    const int kh = (lane >> 5) * 8;
    int hp0[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int p = wm * (32 * MI) + 32 * i + (lane & 31);
        const int r = p / WT, c = p - r * WT;
        hp0[i] = r * HC + c;
    }
    int boff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) boff[j] = xoff(wn * 64 + 32 * j + (lane & 31), kh);
    // A fragment offset of tap (dy, dx), row block i (fixed per lane); TALL computes them per kernel row instead
    // (36 registers held across the loop would not fit beside the 128 accumulators)
    int aoff[3][3][TALL ? 1 : 2];
    if constexpr (!TALL) {
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                for (int i = 0; i < 2; ++i) aoff[dy][dx][i] = xoff(hp0[i] + dy * HC + dx, kh);
    }
    auto afrag = [&](int dy, int dx, int i) {
        if constexpr (TALL) return xoff(hp0[i] + dy * HC + dx, kh);
        else return aoff[dy][dx][i];
    };

    auto hmfma = [&](const bf16x8& fa_, const bf16x8& fb_, const f32x16& c_) {
        if constexpr (ABL & 2) return xmfma<NT>(fa_, fb_, xmfma<NT>(fa_, fb_, c_));
        else return xmfma<NT>(fa_, fb_, c_);
    };
    // the 3 taps (dx) of kernel row dy of the current chunk: fragments from the halo image a and B group b
    // vtag = std::integral_constant<int, V>: V > 0 interleaves V VALU instructions (and a DS write every 4th MFMA)
    // into every MFMA gap — the halo split of the next chunk, placed in the same scheduling region (ABL 1024)
    auto compute = [&](int dy, const __bf16* a, const __bf16* b, auto vtag) {
        constexpr int V = decltype(vtag)::value;
        int nmf = 0;
        auto mf1 = [&]() {   // one MFMA slot of the pinned schedule
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if constexpr (V > 0) {
                __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
                // the LDS writes after the last fragment read (they may alias it): in the last tap
                if (++nmf > 24 && (nmf & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
            }
        };
        // register double buffer: the fragments of tap dx+1 are read while the MFMAs of tap dx issue
        bf16x8 FA[2][MI][NS], FB[2][2][NS];
        auto ldfrag = [&](int buf, int dx) {
#pragma unroll
            for (int t = 0; t < NS; ++t)
#pragma unroll
                for (int i = 0; i < MI; ++i) {
                    FA[buf][i][t] = *reinterpret_cast<const bf16x8*>(a + t * HPLANE + afrag(dy, dx, i));
                    if (i < 2) FB[buf][i][t] = *reinterpret_cast<const bf16x8*>(b + (dx * NS + t) * XPLANE + boff[i]);
                }
        };
        constexpr bool PREFETCH = ABL & 1;
        if constexpr (PREFETCH) ldfrag(0, 0);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            if constexpr (PREFETCH) {
                if (dx < 2) ldfrag((dx + 1) & 1, dx + 1);
            } else {
                ldfrag(dx & 1, dx);
            }
            const auto& fa = FA[dx & 1];
            const auto& fb = FB[dx & 1];
            // term-major: the hh products issue first, the cross terms after
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = hmfma(fa[i][0], fb[j][0], acc[i][j]);
            if constexpr (NT >= 3) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[i][j] = hmfma(fa[i][0], fb[j][1], acc[i][j]);
                        acc[i][j] = hmfma(fa[i][1], fb[j][0], acc[i][j]);
                    }
            }
            if constexpr (NT >= 6) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[i][j] = hmfma(fa[i][1], fb[j][1], acc[i][j]);
                        acc[i][j] = hmfma(fa[i][0], fb[j][2], acc[i][j]);
                        acc[i][j] = hmfma(fa[i][2], fb[j][0], acc[i][j]);
                    }
            }
        }
        if constexpr (PREFETCH) {
            // pin the interleave: the next tap's fragment reads go one per MFMA gap of the current tap
            constexpr int MF = 2 * MI * (NT >= 6 ? 6 : (NT >= 3 ? 3 : 1)), RD = (MI + 2) * NS;
            if constexpr (V > 0) __builtin_amdgcn_sched_group_barrier(0x020, BQ, 0);   // next B loads first
            __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);          // tap 0 fragments
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                if constexpr (ABL & 64) {          // two reads per gap: the next tap's fragments land early
#pragma unroll
                    for (int k = 0; k < RD / 2; ++k) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, MF - RD / 2, 0);
                } else if constexpr (ABL & 128) {  // all reads after the tap's first MFMA
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, MF - 1, 0);
                } else {
#pragma unroll
                    for (int k = 0; k < RD; ++k) {
                        mf1();
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                    if constexpr (V > 0) {
#pragma unroll
                        for (int k = 0; k < MF - RD; ++k) mf1();
                    } else {
                        __builtin_amdgcn_sched_group_barrier(0x008, MF - RD, 0);
                    }
                }
            }
            if constexpr (V > 0) {                                        // last tap
#pragma unroll
                for (int k = 0; k < MF; ++k) mf1();
            } else {
                __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
            }
        }
    };
    using V0 = std::integral_constant<int, 0>;
    using VH = std::integral_constant<int, (ABL & 1024) ? 4 : 0>;

    auto sync = [&]() {
        if constexpr (!(ABL & 16)) __syncthreads();
    };
    gload_halo(0);
    gload_b(0, bregA);
    store_halo(Hs, 0);
    store_b(0, bregA);
    __syncthreads();
    int hb = 0, bb = 0;
    // DEEP: set X holds the chunk after the current one (stored at the end of the current chunk), set Y receives the
    // one after that; the roles alternate per chunk (nchunks is even, so they line up across tiles)
    RawX hX[DEEP ? HQ : 1], hY[DEEP ? HQ : 1];
    unsigned mX = 0u, mY = 0u;
    if constexpr (DEEP) gload_halo_to(hX, mX, 1);
    for (int kt = 0, t = t_first; kt < tpb && t < mtiles; ++kt, t += t_step) {
    const bool nextt = kt + 1 < tpb && t + t_step < mtiles;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    if constexpr (DEEP) {
    // chunk cc: B of chunk q+1 and the halo of chunk q+2 are loaded (across the tile end: the next tile's chunks 0 / 1),
    // the MFMAs of chunk q run, then chunk q+1 (halo from the set loaded one chunk earlier) is stored
    auto step = [&](int cc, const RawX (&hs)[HQ], unsigned ms, RawX (&hl)[HQ], unsigned& ml) {
        const bool morec = cc + 1 < nchunks;
        const bool has1 = morec || nextt;               // chunk q+1 exists in this block
        const __bf16* a = Hs + hb * NS * HPLANE;
        const __bf16* bcur = Bs + bb * 3 * BPL * XPLANE;
        gload_b(morec ? (cc + 1) * 3 : 0, bregA);
        if (cc + 2 == nchunks && nextt) setup_tile(t + t_step);
        // chunk q+2: this tile's cc + 2, or the next tile's cc + 2 - nchunks (a dummy reload past the block's end)
        gload_halo_to(hl, ml, cc + 2 < nchunks ? cc + 2 : cc + 2 - nchunks);
        compute(0, a, bcur, V0{});
        compute(1, a, bcur + BPL * XPLANE, V0{});
        compute(2, a, bcur + 2 * BPL * XPLANE, V0{});
        if (has1) {
            store_halo_set(hs, ms, Hs + (hb ^ 1) * NS * HPLANE, morec ? cc + 1 : 0);
            store_b((bb ^ 1) * 3 * BPL * XPLANE, bregA);
        }
        sync();
        bb ^= 1;
        hb ^= 1;
    };
    for (int cc = 0; cc < nchunks; cc += 2) {
        step(cc, hX, mX, hY, mY);
        step(cc + 1, hY, mY, hX, mX);
    }
    } else if constexpr (ONEB) {
    for (int cc = 0; cc < nchunks; ++cc) {
        const bool morec = cc + 1 < nchunks;
        const __bf16* a = Hs + hb * NS * HPLANE;
        const __bf16* bcur = Bs + bb * 3 * BPL * XPLANE;
        // the next chunk's 9 taps of B and its halo (or the next tile's first chunk): a whole chunk to arrive
        gload_b(morec ? (cc + 1) * 3 : 0, bregA);
        if (!morec && nextt) setup_tile(t + t_step);
        gload_halo(morec ? cc + 1 : 0);
        compute(0, a, bcur, V0{});
        compute(1, a, bcur + BPL * XPLANE, V0{});
        // staggered (stg): waves 4-7 split + store the next chunk before the last kernel row's MFMAs, waves 0-3 after
        // them (both buffers idle since the previous chunk's barrier)
        const bool early = stg && __builtin_amdgcn_readfirstlane(wave) >= NTH / 128;   // wave-uniform (scalar branch)
        if (morec && early) { store_halo(Hs + (hb ^ 1) * NS * HPLANE, cc + 1); store_b((bb ^ 1) * 3 * BPL * XPLANE, bregA); }
        compute(2, a, bcur + 2 * BPL * XPLANE, V0{});
        if (morec && !early) { store_halo(Hs + (hb ^ 1) * NS * HPLANE, cc + 1); store_b((bb ^ 1) * 3 * BPL * XPLANE, bregA); }
        sync();
        bb ^= 1;
        hb ^= 1;
    }
    } else {
    for (int cc = 0; cc < nchunks; ++cc) {
        const bool morec = cc + 1 < nchunks;
        const int g0 = cc * 3;
        const __bf16* a = Hs + hb * NS * HPLANE;
        // dy = 0: fetch B of dy = 1 and dy = 2, then the next chunk's halo (or the next tile's first)
        gload_b(g0 + 1, bregA);
        gload_b(g0 + 2, bregB);
        if (!morec && nextt) setup_tile(t + t_step);
        gload_halo(morec ? cc + 1 : 0);   // (a dummy reload of chunk 0 after the block's last chunk)
        compute(0, a, Bs + bb * BPL * XPLANE, V0{});
        store_b((bb ^ 1) * BPL * XPLANE, bregA);
        sync();
        bb ^= 1;
        // dy = 1 (bearly: B of the next chunk's dy = 0 fetched here, into the register set stored in dy = 0, so it has a
        // whole group's MFMAs to arrive instead of being stored right after the MFMAs it was issued before)
        if constexpr (bearly) gload_b(morec ? g0 + 3 : 0, bregA);
        compute(1, a, Bs + bb * BPL * XPLANE, V0{});
        store_b((bb ^ 1) * BPL * XPLANE, bregB);
        sync();
        bb ^= 1;
        // dy = 2: fetch B of the next chunk's dy = 0; split + store the next halo (buffer idle since chunk cc-1)
        // ahead of this group's MFMAs, so its VALU work interleaves with them; B after them (just issued)
        if constexpr (!bearly) gload_b(morec ? g0 + 3 : 0, bregA);
        // staggered split (ABL 256, or stg at run time: $CDM_HALO_STAGGER): waves 0-3 split + store the next halo
        // after this kernel row's MFMAs, waves 4-7 before them, so each SIMD pairs one wave's VALU with its partner's
        // MFMAs (wave-uniform)
        const bool late = ((ABL & 256) || stg) && wave < NTH / 128;
        // (round 6) after the block's last chunk these stores write the next tile's chunk 0 (halo and B, fetched during
        // this chunk; setup_tile moved the halo offsets) into the buffers its first chunk reads — the work the post-loop
        // stores did — so the stores need no `more chunks` condition (each condition was one more basic block splitting
        // the MFMAs' scheduling region; after the last tile they rewrite idle buffers)
        const int cn = morec ? cc + 1 : 0;
        if constexpr (!(ABL & 1024)) {
            if (!late) store_halo(Hs + (hb ^ 1) * NS * HPLANE, cn);
        }
        compute(2, a, Bs + bb * BPL * XPLANE, VH{});
        if constexpr (ABL & 1024) {
            // after the MFMAs in program order (its LDS writes may alias the fragment reads) but in their scheduling
            // region: the split's VALU fills the MFMA gaps
            store_halo(Hs + (hb ^ 1) * NS * HPLANE, cn);
        }
        if (late) store_halo(Hs + (hb ^ 1) * NS * HPLANE, cn);
        store_b((bb ^ 1) * BPL * XPLANE, bregA);
        sync();
        bb ^= 1;
        hb ^= 1;
    }
    }
    if constexpr (!TALL) unscale<NT>(acc, sx, op_scale<NT>(amax_w));   // (one term: unscaled)
    if constexpr (ONEB && !DEEP) {   // (the three-barrier schedule stored them in its last kernel row)
        if (nextt) {   // the next tile's chunk 0 (its loads were issued during the last chunk) into the halo / B buffers
            // idle since the last chunk's closing barrier, ahead of the epilogue: its prefetch registers die before the
            // epilogue and the epilogue needs no barrier pair after it
            store_halo(Hs + hb * NS * HPLANE, 0);
            store_b(bb * BGR * BPL * XPLANE, bregA);
        }
    }
    // epilogue scratch (stats / max-min: 4 KiB): the other halo buffer (>= 24 KiB), last read by the final chunk
    // before its closing barrier
    if constexpr (TALL)
        ep.tall(acc, t * HB + wm * 128, n0 + wn * 64, lane, wm, wn, reinterpret_cast<float*>(Hs + (hb ^ 1) * NS * HPLANE),
                tid);
    else if constexpr (ABL & 16384) {   // timing ablation: the epilogue skipped (kept live behind a never-taken branch)
        if (acc[0][0][0] == 1.2345e-30f)
            ep(acc, t * HB + wm * 64, n0 + wn * 64, lane, wm, wn, reinterpret_cast<float*>(Hs + (hb ^ 1) * NS * HPLANE),
               tid);
    } else
        ep(acc, t * HB + wm * 64, n0 + wn * 64, lane, wm, wn, reinterpret_cast<float*>(Hs + (hb ^ 1) * NS * HPLANE), tid);
    if (nextt) __syncthreads();
    }
}

// ============================== conv3x3 weight gradient, split-bf16, transposed LDS reads ==============================
// dW[co][tap*Cin + ci] (per split-K slab) = sum_pix dY[pix][co] * X[pix shifted by tap][ci]; K = pixels.
// Both operands are stored pixel-major in HBM (channels contiguous), i.e. k-strided for the MFMA.  They
// are staged exactly as they arrive — float4 along channels, split into bf16 terms, one [16 pix][128 ch]
// image per term (256-byte rows, 16-byte chunks XOR-swizzled by row: conflict-free stores and reads) —
// and the k-contiguous MFMA fragments are produced by the hardware transpose read ds_read_b64_tr_b16
// (two per fragment).  Block: 128 co x 128 columns of one tap (Cin % 128 == 0, Cout % 128 == 0), 4 waves
// 2x2 of 64x64, split-K over blockIdx.z.  The 16 pixels of a K step lie in one image row (W % 16 == 0),
// so the tap shift is one bounds test per pixel.  KS K steps (16 pixels each) share one barrier interval.
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
static __device__ __forceinline__ int trswz(int row, int ch) {   // byte offset of 16-B chunk ch in row
    return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}

// CT (round 5): the ConvTranspose2d(k = 2, s = 2) weight gradient on the same staging (diffusion_utilities.py:86):
// dW[ci][ij][co] = sum_{n,h,w} X[n,h,w][ci] dY[n,2h+i,2w+j][co] — "dy" is then the ConvT input X (rows M = its
// channels), "x" its output gradient dY read at the sub-pixel (i, j) = (tap >> 1, tap & 1) of each input pixel (N =
// 4 taps x its channels), H / W the input grid; the slab layout [z][ci][ij * Cout + co] of cdm_convT2x2_wgrad.  Both
// operands are staged pixel-major as they arrive and read transposed, instead of the generic GEMM's 8 scalar
// k-strided loads per column (0.19 of the h3 ceiling, round 4).
template <int NT, int KS = 1, bool CT = false>   // KS = 2 measured neutral (1.06 vs 1.07 ms per 309 GF)
__global__ __launch_bounds__(GTHREADS, 2) void wgrad3x3_tr_x3_kernel(const float* __restrict__ dy, int lddy, int Cout,
                                                                     const float* __restrict__ x, int H, int W, int Cin,
                                                                     int ldx, int K, int kt_per_split,
                                                                     const float* amax_dy, const float* amax_x,
                                                                     EpiStore ep) {
    constexpr int NS = XTerms<NT>::NS;
    constexpr int IMG = 16 * 128;                     // bf16 per [16 pix][128 ch] term image
    constexpr int STEP = 2 * NS * IMG;                // bf16 per K step (both operands, all terms)
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * KS * STEP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // 1-D grid, split-major logical order L = z*T + tile, remapped so that each XCD (hardware block b -> XCD b%8)
    // runs a contiguous range of L: the T tiles of one split share their dY / X pixel range in that XCD's L2.
    constexpr int NTAP = CT ? 4 : 9;
    const int gx = Cout / GBM, T = gx * (NTAP * Cin / GBN);
    int L;
    {
        const int nwg = gridDim.x, q8 = nwg >> 3, r8 = nwg & 7, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
        L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + j;
    }
    const int bz = L / T, tl = L - bz * T;
    const int m0 = (tl % gx) * GBM, n0 = (tl / gx) * GBN;
    const int tap = n0 / Cin, ci0 = n0 - tap * Cin;
    const int ky = tap / 3, sdy = ky - 1, sdx = tap - ky * 3 - 1;
    const int ti = tap >> 1, tj = tap & 1;            // CT: the sub-pixel of the output gradient
    const int ktiles = K / 16;
    const int kt0 = bz * kt_per_split;
    const int kt1 = min(ktiles, kt0 + kt_per_split);
    const float sdy_ = op_scale<NT>(amax_dy), sx_ = op_scale<NT>(amax_x);

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // staging map: thread -> pixel rows kk = (tid>>5) + 8i, channel quad c4 = (tid&31)*4
    const int kq = tid >> 5, c4 = (tid & 31) * 4;
    const int hw = H * W;
    // running image coordinates of the K step's first pixel
    int p0 = kt0 * 16;
    int pn = p0 / hw, ph = (p0 - pn * hw) / W, pw = p0 - pn * hw - ph * W;
    // DEEP2 (CT, KS = 1; round 6): two register sets, the K step two ahead in flight while one computes — a ConvT K step
    // is 12 MFMAs per wave, far too short to cover the HBM latency of loads issued one step ahead
    constexpr bool DEEP2 = CT && KS == 1;
    float4 ra[KS][2], rb[KS][2], ra2[DEEP2 ? KS : 1][2], rb2[DEEP2 ? KS : 1][2];
    auto gload_to = [&](float4 (&ra)[KS][2], float4 (&rb)[KS][2], int kt) {   // the KS K steps from kt (zero past kt1)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const bool ok = kt + ks < kt1;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int kk = kq + 8 * i;
                const long long pix = (long long)(pn * H + ph) * W + pw + kk;
                ra[ks][i] = ok ? ld4(dy + pix * lddy + m0 + c4) : f4zero();
                if constexpr (CT) {
                    const long long opix = (long long)(pn * 2 * H + 2 * ph + ti) * (2 * W) + 2 * (pw + kk) + tj;
                    rb[ks][i] = ok ? ld4(x + opix * ldx + ci0 + c4) : f4zero();
                } else {
                    const int hh = ph + sdy, ww = pw + kk + sdx;
                    rb[ks][i] = (ok && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
                                    ? ld4(x + ((long long)(pn * H + hh) * W + ww) * ldx + ci0 + c4)
                                    : f4zero();
                }
            }
            pw += 16;
            if (pw >= W) { pw = 0; if (++ph == H) { ph = 0; ++pn; } }
        }
    };
    auto gload = [&](int kt) { gload_to(ra, rb, kt); };
    auto sstore_from = [&](const float4 (&ra)[KS][2], const float4 (&rb)[KS][2], __bf16* base0) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int op = 0; op < 2; ++op)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                __bf16* base = base0 + ks * STEP;
                const float4 v = op ? rb[ks][i] : ra[ks][i];
                const float xv[4] = {v.x, v.y, v.z, v.w};
                u32x2 tm[3];
                split_pk4<NT>(xv, op ? sx_ : sdy_, tm);
                const int kk = kq + 8 * i;
                char* d = reinterpret_cast<char*>(base + op * NS * IMG) + trswz(kk, c4 >> 3) + (c4 & 7) * 2;
#pragma unroll
                for (int k = 0; k < NS; ++k) *reinterpret_cast<u32x2*>(d + k * IMG * 2) = tm[k];
            }
    };
    auto sstore = [&](__bf16* base0) { sstore_from(ra, rb, base0); };
    // transposed-read addresses: lane 4q+p of 16-lane group g supplies row kb+q, columns c0+4p..+3
    const int g = (lane >> 4) & 3, q = (lane >> 2) & 3, pq = lane & 3;
    const int kb = 8 * (g >> 1) + q;
    int aoff[2][2], boff[2][2];   // [i][half] byte offsets within a term image
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ca = wm * 64 + 32 * i + 16 * (g & 1) + 4 * pq, cb = wn * 64 + 32 * i + 16 * (g & 1) + 4 * pq;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            aoff[i][hf] = trswz(kb + 4 * hf, ca >> 3) + (ca & 7) * 2;
            boff[i][hf] = trswz(kb + 4 * hf, cb >> 3) + (cb & 7) * 2;
        }
    }

    auto mma_at = [&](int cur) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
        const char* a = reinterpret_cast<const char*>(smem + (cur * KS + ks) * STEP);
        const char* b = a + NS * IMG * 2;
        bf16x8 fa[2][NS], fb[2][NS];
#pragma unroll
        for (int t = 0; t < NS; ++t)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const bf16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + t * IMG * 2 + aoff[i][0]));
                const bf16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + t * IMG * 2 + aoff[i][1]));
                const bf16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(b + t * IMG * 2 + boff[i][0]));
                const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(b + t * IMG * 2 + boff[i][1]));
                fa[i][t] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
                fb[i][t] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
            }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                f32x16 c = acc[i][j];
                if constexpr (NT >= 6) {
                    c = xmfma<NT>(fa[i][1], fb[j][1], c);
                    c = xmfma<NT>(fa[i][2], fb[j][0], c);
                    c = xmfma<NT>(fa[i][0], fb[j][2], c);
                }
                if constexpr (NT >= 3) {
                    c = xmfma<NT>(fa[i][1], fb[j][0], c);
                    c = xmfma<NT>(fa[i][0], fb[j][1], c);
                }
                acc[i][j] = xmfma<NT>(fa[i][0], fb[j][0], c);
            }
        }
    };
    if constexpr (DEEP2) {
        if (kt0 < kt1) { gload_to(ra, rb, kt0); sstore_from(ra, rb, smem); }
        if (kt0 + 1 < kt1) gload_to(ra2, rb2, kt0 + 1);
        __syncthreads();
        int cur = 0;
        for (int kt = kt0; kt < kt1; kt += 2) {   // set (ra, rb): even steps, (ra2, rb2): odd steps
            if (kt + 2 < kt1) gload_to(ra, rb, kt + 2);
            mma_at(cur);
            if (kt + 1 < kt1) sstore_from(ra2, rb2, smem + (cur ^ 1) * STEP);
            __syncthreads();
            cur ^= 1;
            if (kt + 1 >= kt1) break;
            if (kt + 3 < kt1) gload_to(ra2, rb2, kt + 3);
            mma_at(cur);
            if (kt + 2 < kt1) sstore_from(ra, rb, smem + (cur ^ 1) * STEP);
            __syncthreads();
            cur ^= 1;
        }
    } else {
        if (kt0 < kt1) { gload(kt0); sstore(smem); }
        __syncthreads();
        int cur = 0;
        for (int kt = kt0; kt < kt1; kt += KS) {
            const bool more = kt + KS < kt1;
            if (more) gload(kt + KS);
            mma_at(cur);
            if (more) sstore(smem + (cur ^ 1) * KS * STEP);
            __syncthreads();
            cur ^= 1;
        }
    }
    unscale<NT>(acc, sdy_, sx_);
    EpiStore e = ep;                       // this block's split slab (the epilogue would index blockIdx.z)
    e.y += (long long)bz * ep.zstride;
    e.zstride = 0;
    e(acc, m0 + wm * 64, n0 + wn * 64, lane, wm, wn, reinterpret_cast<float*>(smem), tid);
}

// Weight gradient by kernel row: a block owns 128 co x 128 ci x the 3 taps (ky, kx = 0..2) of one kernel row.
// Per K step (16 pixels of one image row) it stages dY [16 pix][128 co] and the input row segment with its
// 1-pixel halo X [18 pix][128 ci] once; the 3 taps read B from the same X image at row offsets 0 / 1 / 2 (the
// kx shift), so each dY fragment feeds 3 taps and X is staged once instead of three times (2.5x less LDS
// traffic per MFMA than the per-tap kernel above).  8 waves = 2 (co) x 4 (ci), wave tile 64 co x 32 ci x 3
// taps (6 accumulators).  Split-K over pixel ranges; writes slab[z][co][tap*Cin+ci] like the per-tap kernel.
template <int NT, int KS = 1, class PRE = PreNone, class PX = PreNone, class GT = float, class XT = float>
                                // GT / XT: element types of dy (g and PRE's y) / of x (and PX's g): bf16 for C4's
                                // fused-chain activations and gradients
                                // KS: 16-pixel K steps per barrier (W % (16 KS) == 0);
                                // KS = 2: 1.09x KS = 1; KS = 4 (133 KiB of LDS under h3): C2 -0.7 % (round 6)
                                // PRE = PreBnBwd: dy computed from g (the dy argument) and y while staging
                                // PX = PreBnRelu: X = relu(y s + t) computed from the previous layer's y (the x argument)
__global__ __launch_bounds__(512, 1) void wgrad3x3_row_kernel(const GT* __restrict__ dy, int lddy, int Cout,
                                                              const XT* __restrict__ x, int H, int W, int Cin,
                                                              int ldx, int ktiles, int kt_per_split,
                                                              const float* amax_dy, const float* amax_x,
                                                              float* __restrict__ slab, PRE pre, PX px, int stg) {
    constexpr int NS = XTerms<NT>::NS;
    constexpr int RA = 16 * KS, RB = RA + 2;          // image rows (pixels): dY, X with its halo
    constexpr int IA = RA * 128, IB = RB * 128;       // bf16 per term image
    constexpr int STEP = NS * (IA + IB);
    // the PreBnReluSums fold reuses the staging buffers as [16 rows][3][128] floats: at least 12288 bf16 of them
    // (one bf16 term with 16-pixel K steps stages only 8704)
    constexpr int SMEM = (PX::kind == 3 && 2 * STEP < 2 * 16 * 3 * 128) ? 2 * 16 * 3 * 128 : 2 * STEP;
    __shared__ __attribute__((aligned(16))) __bf16 smem[SMEM];
    // wave made provably uniform (readfirstlane): the schedule branches on it, and the K-step position (pn, ph, pw)
    // advanced inside those branches must stay scalar — as tid >> 6 the compiler treated it as divergent, kept the
    // position in VGPRs and wrapped every buffer load in a readfirstlane waterfall loop
    // UNI per form, as measured (profiles/r6_ab_wgrad_uniform.txt, r6_ab_wgrad_uniform_bf16.txt): h3, and the one-term
    // forms with the producer sums (both operand types alike, or 32-pixel steps) or 64-pixel steps without them (-2 to
    // -7 % per launch); the other one-term forms keep the divergent index and the three-path loop below (+6 to +24 %
    // with the uniform one)
    constexpr bool SUMSF = PX::kind == 3;
    constexpr bool UNI = NT == NT_H3 || (SUMSF && (std::is_same<GT, XT>::value || KS == 2)) || (!SUMSF && KS == 4);
    const int tid = threadIdx.x, lane = tid & 63, wave = UNI ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
    const int wm = wave & 1, wn = wave >> 1;
    const int gx = Cout / 128, T = gx * 3 * (Cin / 128);
    int L;   // split-major logical order, XCD-contiguous ranges (as the per-tap kernel)
    {
        const int nwg = gridDim.x, q8 = nwg >> 3, r8 = nwg & 7, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
        L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + j;
    }
    const int bz = L / T, tl = L - bz * T;
    const int m0 = (tl % gx) * 128, r2 = tl / gx, ky = r2 % 3, ci0 = (r2 / 3) * 128;
    const int kt0 = bz * kt_per_split, kt1 = min(ktiles, kt0 + kt_per_split);   // in units of KS steps
    const float sa = op_scale<NT>(amax_dy), sb = op_scale<NT>(amax_x);

    f32x16 acc[3][2];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][i][r] = 0.f;

    // staging map: thread -> image row sr (pixel), channel quad c4; threads 0..63 also stage X rows 16, 17
    const int sr = tid >> 5, c4 = (tid & 31) * 4;
    const int hw = H * W;
    const int p0 = kt0 * RA;
    int pn = p0 / hw, ph = (p0 - pn * hw) / W, pw = p0 - pn * hw - ph * W;
    using RawG = typename Act<GT>::Raw;
    using RawX = typename Act<XT>::Raw;
    RawG ra[KS];
    RawX rb[KS], rb1 = Act<XT>::zero();
    bool vb[KS], vb1 = false;       // PX: which X pieces lie inside the image (padding stays zero)
    float xs[4], xt[4];             // PX coefficients of this thread's 4 input channels ci0 + c4
    if constexpr (PX::kind >= 2) {
        const float4 a = ld4(px.p[0] + ci0 + c4), b = ld4(px.p[1] + ci0 + c4);
        xs[0] = a.x; xs[1] = a.y; xs[2] = a.z; xs[3] = a.w; xt[0] = b.x; xt[1] = b.y; xt[2] = b.z; xt[3] = b.w;
    }
    // PreBnReluSums: every X pixel (image row hh, column c) of this ci tile is staged by all 3 x gx blocks of the
    // split holding its output pixel(s); it is summed by exactly one of them, spread evenly: the kernel-row block
    // ky = hh % 3 (ky = 1 for the last image row, where hh % 3 == 0 stages no output row) and, per K step q
    // (global RA-pixel step), the co tile q % gx.  The flag is per K step (block-uniform), set by gload.
    constexpr bool SUMS = PX::kind == 3;
    bool sum_step = false;
    float xm[4], xi[4], s1[4], s2[4], s5[4];
    RawX gr[SUMS ? KS : 1], gr1 = Act<XT>::zero();
    if constexpr (SUMS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { s1[e] = 0.f; s2[e] = 0.f; s5[e] = 0.f; }
        const float4 a = ld4(px.mean + ci0 + c4), b = ld4(px.invstd + ci0 + c4);
        xm[0] = a.x; xm[1] = a.y; xm[2] = a.z; xm[3] = a.w; xi[0] = b.x; xi[1] = b.y; xi[2] = b.z; xi[3] = b.w;
    }
    RawG ya[PRE::on ? KS : 1];
    float cf[PRE::on ? 7 : 1][4];   // PreBnBwd coefficients of this thread's 4 output channels m0 + c4
    if constexpr (PRE::on) {
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const float4 v = ld4(pre.p[k] + m0 + c4);
            cf[k][0] = v.x; cf[k][1] = v.y; cf[k][2] = v.z; cf[k][3] = v.w;
        }
    }
    // K-step loads as buffer loads: the step's pixel (pn, ph, pw) is wave-uniform, so each operand's address is a
    // uniform base (scalar arithmetic, a new resource per step) + a per-lane byte offset that is the same for every step
    // (pixel sr + 16 k of the step, channel quad c4); padding pieces (outside the image, and the sums' skipped pieces)
    // take offset BUF_OOB and read zeros.  Round 6: the per-load 64-bit index products (two v_mul_lo_u32 and a
    // v_mad_u64_u32, quarter-rate) and the exec-masked zero fills were the bulk of this VALU-issue-bound loop's non-MFMA
    // instructions.
    // (two-term h3 only: for the one-term bf16 kernels it measured slower, 26.53 -> 26.99 ms per C4 step; C2 48.61 ->
    // 48.42 ms, profiles/r6_ab_wgrad_bufld.txt)
    constexpr bool BUFLD = NT == NT_H3;
    unsigned odg[KS], ody[KS], oxk[KS], ogk[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        odg[k] = (unsigned)((sr + 16 * k) * lddy + c4) * (unsigned)sizeof(GT);
        if constexpr (PRE::on) ody[k] = (unsigned)((sr + 16 * k) * pre.ldy + c4) * (unsigned)sizeof(GT);
        oxk[k] = (unsigned)((sr + 16 * k) * ldx + c4) * (unsigned)sizeof(XT);
        if constexpr (SUMS) ogk[k] = (unsigned)((sr + 16 * k) * px.ldg + c4) * (unsigned)sizeof(XT);
    }
    const unsigned ox1 = (unsigned)((RA + sr) * ldx + c4) * (unsigned)sizeof(XT);
    unsigned og1 = 0u;
    if constexpr (SUMS) og1 = (unsigned)((RA + sr) * px.ldg + c4) * (unsigned)sizeof(XT);
    auto gload = [&]() {   // the K step at (pn, ph, pw), then advance by RA pixels
        const int hh = ph + ky - 1;
        const bool rowok = (unsigned)hh < (unsigned)H;
        const long long xrow = (long long)(pn * H + hh) * W;
        if constexpr (SUMS) {
            const int ks = (hh == H - 1 && hh % 3 == 0) ? 1 : hh % 3;
            const long long q = ((long long)(pn * H + ph) * W + pw) / RA;
            sum_step = rowok && ky == ks && (int)(q % gx) == (m0 >> 7);
        }
        if constexpr (BUFLD) {
            const long long pix0 = (long long)(pn * H + ph) * W + pw;            // the step's first output pixel
            const long long xp0 = xrow + pw - 1;                                 // its X image's first pixel (halo)
            const auto rdy = buf_rsrc(dy + pix0 * lddy + m0);
            const auto rx = buf_rsrc(x + xp0 * ldx + ci0);
    #pragma unroll
            for (int k = 0; k < KS; ++k) {
                ra[k] = Act<GT>::bload4(rdy, odg[k]);
                if constexpr (PRE::on)
                    ya[k] = Act<GT>::bload4(buf_rsrc(reinterpret_cast<const GT*>(pre.y) + pix0 * pre.ldy + m0), ody[k]);
                const int w0 = pw - 1 + sr + 16 * k;
                vb[k] = rowok && (unsigned)w0 < (unsigned)W;
                rb[k] = Act<XT>::bload4(rx, vb[k] ? oxk[k] : BUF_OOB);
                if constexpr (SUMS) {   // central rows 1..RA of the X image (the step's own columns, inside the image)
                    const auto rg = buf_rsrc(reinterpret_cast<const XT*>(px.g) + xp0 * px.ldg + ci0);
                    gr[k] = Act<XT>::bload4(rg, (sum_step && (k > 0 || sr >= 1)) ? ogk[k] : BUF_OOB);
                }
            }
            if (tid < 64) {   // (wave 0: a uniform branch)
                const int w1 = pw + RA - 1 + sr;
                vb1 = rowok && w1 < W;
                rb1 = Act<XT>::bload4(rx, vb1 ? ox1 : BUF_OOB);
                if constexpr (SUMS) {
                    const auto rg = buf_rsrc(reinterpret_cast<const XT*>(px.g) + xp0 * px.ldg + ci0);
                    gr1 = Act<XT>::bload4(rg, (sum_step && tid < 32) ? og1 : BUF_OOB);
                }
            }
        } else {   // one-term (C4): plain loads (the buffer form measured 26.53 -> 26.99 ms per C4 step)
    #pragma unroll
            for (int k = 0; k < KS; ++k) {
                const long long pix = (long long)(pn * H + ph) * W + pw + sr + 16 * k;
                ra[k] = Act<GT>::load4(dy + pix * lddy + m0 + c4);
                if constexpr (PRE::on) ya[k] = Act<GT>::load4(reinterpret_cast<const GT*>(pre.y) + pix * pre.ldy + m0 + c4);
                const int w0 = pw - 1 + sr + 16 * k;
                vb[k] = rowok && (unsigned)w0 < (unsigned)W;
                rb[k] = vb[k] ? Act<XT>::load4(x + (xrow + w0) * ldx + ci0 + c4) : Act<XT>::zero();
                if constexpr (SUMS) {   // central rows 1..RA of the X image (the step's own columns, inside the image)
                    gr[k] = (sum_step && (k > 0 || sr >= 1))
                                ? Act<XT>::load4(reinterpret_cast<const XT*>(px.g) + (xrow + w0) * px.ldg + ci0 + c4)
                                : Act<XT>::zero();
                }
            }
            if (tid < 64) {
                const int w1 = pw + RA - 1 + sr;
                vb1 = rowok && w1 < W;
                rb1 = vb1 ? Act<XT>::load4(x + (xrow + w1) * ldx + ci0 + c4) : Act<XT>::zero();
                if constexpr (SUMS)
                    gr1 = (sum_step && tid < 32)
                              ? Act<XT>::load4(reinterpret_cast<const XT*>(px.g) + (xrow + w1) * px.ldg + ci0 + c4)
                              : Act<XT>::zero();
            }
        }
        pw += RA;
        if (pw >= W) { pw = 0; if (++ph == H) { ph = 0; ++pn; } }
    };
    // (lane conditions as selects, not branches: a divergent `if` around a piece cost an exec save / restore and four
    // register copies per piece; the pieces a condition drops were loaded as zeros, BUF_OOB)
    auto xsum = [&](const float4& v, const float4& gv, bool on) {     // PreBnReluSums: one central piece
        // (contraction off, the fused products spelled out: the compiler's free fmul + fadd fusion decided differently
        // in the two inlined copies of the staging (the wave schedules), so the sums' last bits depended on the schedule)
#pragma clang fp contract(off)
        if constexpr (SUMS) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float y = f4get(v, e);
                const float zp = fmaf(y, xs[e], xt[e]);
                const float xh = (y - xm[e]) * xi[e];
                const float gp = zp > 0.f ? f4get(gv, e) : 0.f;   // (g is 0 where !on: nothing to mask in s1, s2)
                s1[e] += gp; s2[e] = fmaf(gp, xh, s2[e]); s5[e] += on ? xh : 0.f;
            }
        }
    };
    auto xpre = [&](const float4& v, bool valid) -> float4 {   // PX transform at staging time (after the load wait)
        if constexpr (PX::kind >= 2) {
            if constexpr (BUFLD)
                return make_float4(valid ? bn_relu_elem(v.x, xs[0], xt[0]) : 0.f,
                                   valid ? bn_relu_elem(v.y, xs[1], xt[1]) : 0.f,
                                   valid ? bn_relu_elem(v.z, xs[2], xt[2]) : 0.f,
                                   valid ? bn_relu_elem(v.w, xs[3], xt[3]) : 0.f);
            else if (valid)
                return make_float4(bn_relu_elem(v.x, xs[0], xt[0]), bn_relu_elem(v.y, xs[1], xt[1]),
                                   bn_relu_elem(v.z, xs[2], xt[2]), bn_relu_elem(v.w, xs[3], xt[3]));
        }
        return v;   // (padding pieces were loaded as zeros)
    };
    auto put = [&](char* img, int row, const float4& v, float sc, int ielems) {
        const float xv[4] = {v.x, v.y, v.z, v.w};
        u32x2 tm[3];
        split_pk4<NT>(xv, sc, tm);
        char* d = img + trswz(row, c4 >> 3) + (c4 & 7) * 2;
#pragma unroll
        for (int k = 0; k < NS; ++k) *reinterpret_cast<u32x2*>(d + k * ielems * 2) = tm[k];
    };
    // one-term bf16 operands without a staging transform are copied as they arrive (no convert round trip)
    constexpr bool RAWG = NT == 1 && !PRE::on && std::is_same<GT, __bf16>::value;
    constexpr bool RAWX = NT == 1 && PX::kind == 0 && std::is_same<XT, __bf16>::value;
    auto sstore = [&](__bf16* buf) {
        char* a = reinterpret_cast<char*>(buf);
        char* b = a + NS * IA * 2;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            if constexpr (PRE::on) {
                const float4 yf = Act<GT>::to4(ya[k]), gf = Act<GT>::to4(ra[k]);
                const float yv[4] = {yf.x, yf.y, yf.z, yf.w};
                float gv[4] = {gf.x, gf.y, gf.z, gf.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    gv[e] = bn_bwd_elem(gv[e], yv[e], cf[0][e], cf[1][e], cf[2][e], cf[3][e], cf[4][e], cf[5][e],
                                        cf[6][e]);
                put(a, sr + 16 * k, make_float4(gv[0], gv[1], gv[2], gv[3]), sa, IA);
            } else if constexpr (RAWG) {   // bf16 dy (stored by the dgrad) into the one-term image: a plain copy
                *reinterpret_cast<uint2*>(a + trswz(sr + 16 * k, c4 >> 3) + (c4 & 7) * 2) = ra[k];
            } else {
                put(a, sr + 16 * k, Act<GT>::to4(ra[k]), sa, IA);
            }
            if constexpr (RAWX) {
                *reinterpret_cast<uint2*>(b + trswz(sr + 16 * k, c4 >> 3) + (c4 & 7) * 2) = rb[k];
            } else {
                const float4 xk = Act<XT>::to4(rb[k]);
                if constexpr (SUMS) {
                    // (sum_step: block-uniform; the lane condition sr >= 1 only splits wave 0 at k = 0)
                    if constexpr (BUFLD) {
                        if (sum_step) xsum(xk, Act<XT>::to4(gr[k]), k > 0 || sr >= 1);
                    } else {
                        if (sum_step && (k > 0 || sr >= 1)) xsum(xk, Act<XT>::to4(gr[k]), true);
                    }
                }
                put(b, sr + 16 * k, xpre(xk, vb[k]), sb, IB);
            }
        }
        if constexpr (RAWX) {
            if (tid < 64) *reinterpret_cast<uint2*>(b + trswz(RA + sr, c4 >> 3) + (c4 & 7) * 2) = rb1;
        } else {
            const float4 x1 = Act<XT>::to4(rb1);
            if constexpr (SUMS) {
                if constexpr (BUFLD) {
                    if (sum_step && tid < 64) xsum(x1, Act<XT>::to4(gr1), tid < 32);   // (wave 0 only: uniform)
                } else {
                    if (sum_step && tid < 32) xsum(x1, Act<XT>::to4(gr1), true);
                }
            }
            if (tid < 64) put(b, RA + sr, xpre(x1, vb1), sb, IB);
        }
    };
    // transposed-read addresses (see the per-tap kernel); tap t reads X rows shifted by t
    const int g = (lane >> 4) & 3, q = (lane >> 2) & 3, pq = lane & 3;
    const int kb = 8 * (g >> 1) + q;
    // (the swizzle depends on row & 15 only: K sub-step k adds the constant 16 k rows = 4096 k bytes)
    int aoff[2][2], boff[3][2];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int ca = wm * 64 + 32 * i + 16 * (g & 1) + 4 * pq;
            aoff[i][hf] = trswz(kb + 4 * hf, ca >> 3) + (ca & 7) * 2;
        }
        const int cb = wn * 32 + 16 * (g & 1) + 4 * pq;
#pragma unroll
        for (int t = 0; t < 3; ++t) boff[t][hf] = trswz(kb + 4 * hf + t, cb >> 3) + (cb & 7) * 2;
    }

    // the MFMAs of the K step staged in buffer cur_
    auto mma_at = [&](int cur_) {
        const char* a = reinterpret_cast<const char*>(smem + cur_ * STEP);
        const char* b = a + NS * IA * 2;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
        bf16x8 fa[2][NS];
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const bf16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + s * IA * 2 + aoff[i][0] + 4096 * k));
                const bf16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + s * IA * 2 + aoff[i][1] + 4096 * k));
                fa[i][s] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
            }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            bf16x8 fb[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                const bf16x4 b0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(b + s * IB * 2 + boff[t][0] + 4096 * k));
                const bf16x4 b1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(b + s * IB * 2 + boff[t][1] + 4096 * k));
                fb[s] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                f32x16 c = acc[t][i];
                if constexpr (NT >= 6) {
                    c = xmfma<NT>(fa[i][1], fb[1], c);
                    c = xmfma<NT>(fa[i][2], fb[0], c);
                    c = xmfma<NT>(fa[i][0], fb[2], c);
                }
                if constexpr (NT >= 3) {
                    c = xmfma<NT>(fa[i][1], fb[0], c);
                    c = xmfma<NT>(fa[i][0], fb[1], c);
                }
                acc[t][i] = xmfma<NT>(fa[i][0], fb[0], c);
            }
        }
        }
    };
    // stg: the two waves of each SIMD (w, w + 4) run the step in opposite orders — one stages the next K step
    // (VALU: BN transforms, term split, LDS writes) while the other issues its MFMAs, instead of both alternating in
    // lock-step between the barriers.  The staging-first wave loads one K step further ahead (its registers are free
    // once it has staged), so its staging finds the data in flight since the previous step's MFMAs (round 3's form
    // loaded at the top of the step and waited out the whole HBM latency there).
    const bool early = (stg & 1) && wave >= 4;
    if ((stg & 2) && wave >= 4) __builtin_amdgcn_s_setprio(1);   // stg bit 1: the staging-first half at priority 1
    // stg bit 2: the MFMA-first half also loads the K step after next as soon as it has staged (before the barrier; the
    // default: loading at the top of the step after the barrier measured C2 46.16-46.26 -> 46.75-46.77 ms)
    const bool ahead = UNI || early || (stg & 4);
    if (kt0 < kt1) { gload(); sstore(smem); }
    if (ahead && kt0 + 1 < kt1) gload();
    __syncthreads();
    int cur = 0;
    if constexpr (UNI) {
        // one copy of the MFMAs on a single path, the staging on wave-uniform branches around it.  Round 6: with the
        // MFMAs on three paths and the wave index divergent, the K-step position (pn, ph, pw) advanced on those paths
        // sat in VGPRs — a readfirstlane waterfall loop around every buffer load — and the compiler shuffled the 96
        // accumulators between register sets at every join (96 v_mov per step): C2's sums form 769 -> 685 us per launch
        for (int kt = kt0; kt < kt1; ++kt) {
            const bool more = kt + 1 < kt1;
            if (early) {
                if (more) sstore(smem + (cur ^ 1) * STEP);
                if (kt + 2 < kt1) gload();
            }
            mma_at(cur);
            if (!early) {   // (always ahead: a third load site cost 100+ register copies per step)
                if (more) sstore(smem + (cur ^ 1) * STEP);
                if (kt + 2 < kt1) gload();
            }
            __syncthreads();
            cur ^= 1;
        }
    } else {
        for (int kt = kt0; kt < kt1; ++kt) {
            const bool more = kt + 1 < kt1;
            auto mma = [&]() { mma_at(cur); };
            if (early) {
                if (more) sstore(smem + (cur ^ 1) * STEP);
                if (kt + 2 < kt1) gload();
                mma();
            } else if (ahead) {
                mma();
                if (more) sstore(smem + (cur ^ 1) * STEP);
                if (kt + 2 < kt1) gload();
            } else {
                if (more) gload();
                mma();
                if (more) sstore(smem + (cur ^ 1) * STEP);
            }
            __syncthreads();
            cur ^= 1;
        }
    }
    if constexpr (SUMS) {   // fold the 16 pixel rows of each channel quad (fixed order): one partial per block,
        float* red = reinterpret_cast<float*>(smem);        // [16 rows][3][128 ch] in the idle staging buffers
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            red[(sr * 3 + 0) * 128 + c4 + e] = s1[e];
            red[(sr * 3 + 1) * 128 + c4 + e] = s2[e];
            red[(sr * 3 + 2) * 128 + c4 + e] = s5[e];
        }
        __syncthreads();
        if (tid < 128) {   // sums[(split * 3 + ky) * gx + co tile][5][Cin]
            float a1 = 0.f, a2 = 0.f, a5 = 0.f;
            for (int r = 0; r < 16; ++r) {
                a1 += red[(r * 3 + 0) * 128 + tid]; a2 += red[(r * 3 + 1) * 128 + tid];
                a5 += red[(r * 3 + 2) * 128 + tid];
            }
            float* o = px.sums + ((long long)(bz * 3 + ky) * gx + (m0 >> 7)) * 5 * Cin + ci0 + tid;
            o[0] = a1; o[Cin] = a2; o[2 * Cin] = 0.f; o[3 * Cin] = 0.f; o[4 * Cin] = a5;
        }
    }
    float ia = 1.f, ib = 1.f;
    if constexpr (NT == NT_H3) { ia = 1.f / sa; ib = 1.f / sb; }
    const int NN = 9 * Cin;
    // wave-uniform base + one lane byte offset for all 96 stores (per-element 64-bit index products were quarter-rate
    // VALU; see EpiStoreW::WaveAddr)
    float* sz = slab + (long long)bz * Cout * NN + (long long)(m0 + __builtin_amdgcn_readfirstlane(wm) * 64) * NN
              + ky * 3 * Cin + ci0 + __builtin_amdgcn_readfirstlane(wn) * 32;
    const unsigned lb = (unsigned)(4 * (lane >> 5) * NN + (lane & 31)) * 4u;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float* p = sz + (long long)(32 * i + (r & 3) + 8 * (r >> 2)) * NN + t * Cin;
                *reinterpret_cast<float*>(reinterpret_cast<char*>(p) + lb) =
                    NT == NT_H3 ? (acc[t][i][r] * ia) * ib : acc[t][i][r];
            }
    }
}

// tiles per block of the LDS-halo conv (round 3: one round of 256 blocks, up to 16 tiles; round 2: >= 512 blocks, at most 8).  Kernel level
// (tools/conv_ablation.py, h3 128->128 @64^2, B=256, one box): 1 tile 0.872 ms, 2: 0.854, 4: 0.848, 8: 0.843,
// 16: 0.834.  Bench, same box, 2 runs each (tpb 1 -> this policy): C2 train 4296 -> 4355 img/s, sampling 15.94 ->
// 15.71 ms per step (CFG 31.95 -> 31.50), C4 bf16 train 6416 -> 6478, sample 9.69 -> 9.46 ms, C5 train 70.7 ->
// 71.2 img/s, sample 69.4 -> 67.6 ms.  The tiles of a block are interleaved across its XCD (see the kernel).
static int halo_tpb(int mtiles, int ntiles, int nterm, int wt) {
    (void)nterm; (void)wt;
    static const int forced = [] { const char* e = getenv("CDM_HALO_TPB"); return e ? atoi(e) : 0; }();
    if (forced > 0) return forced;   // A/B timing override (tools), never set by the product
    // the block count the tiles are dealt to: 256 = one round of one block per CU (up to 16 tiles per block).  Same-box
    // A/B, 2 rounds (profiles/r3_ab_grid_blocks.txt): vs 512 (two rounds, up to 8 tiles) C2 train step 51.32 -> 51.13 ms,
    // C4 31.82 -> 31.70 ms ($CDM_HALO_BLOCKS overrides)
    static const int blocks = [] { const char* e = getenv("CDM_HALO_BLOCKS"); return e ? atoi(e) : 256; }();
    const int maxt = blocks <= 256 ? 16 : 8;
    const int t = (mtiles * ntiles) / (blocks > 0 ? blocks : 512);
    return t < 1 ? 1 : (t > maxt ? maxt : t);
}

// the staggered halo split of the LDS-halo conv: on for h3, off for the one-term bf16 images ($CDM_HALO_STAGGER=0 / 1
// forces it).  Same-box A/B, 2 rounds (profiles/r3_ab_halo_stagger.txt): C2 (h3) train step 51.92-51.95 -> 51.34-51.44
// ms; C4 (bf16) 32.20-32.21 -> 32.26-32.40 ms (its halo split is a plain conversion: nothing left to hide)
static int halo_stagger(int nterm) {   // default on for h3 and (round 4, profiles/r4_ab_c4_knobs.txt) for bf16
    static const int v = [] { const char* e = getenv("CDM_HALO_STAGGER"); return e ? atoi(e) : -1; }();
    // + the block start delay (bits 8+, 10 ns ticks; $CDM_HALO_DELAY)
    static const int d = [] { const char* e = getenv("CDM_HALO_DELAY"); return e ? atoi(e) : 0; }();
    // + static priority 1 for waves 4-7 (bit 1; $CDM_HALO_PRIO, measured neutral: off, profiles/r6_ab_wave_priority.txt).
    // (B fetched one kernel row earlier is compiled in since round 6: as a runtime switch, bit 2, it had measured
    // sampling 13.37-13.40 -> 13.15-13.18 ms per step, profiles/r6_ab_halo_bearly.txt; as a constant a further 13.08-13.20
    // -> 12.87-12.95 and C2 45.10-45.31 -> 44.72-44.83 ms, profiles/r6_ab_halo_bearly_const.txt — the switch's second
    // load site and its branches had cost that much)
    static const int p = [] { const char* e = getenv("CDM_HALO_PRIO"); return e ? atoi(e) : 0; }();
    return (v >= 0 ? v : ((nterm == NT_H3 || nterm == 1) ? 1 : 0)) | (p ? 2 : 0) | (d << 8);
}

// the one-barrier-per-chunk schedule of the one-term (bf16) LDS-halo conv ($CDM_HALO_ONEB=0: three barriers per chunk)
static int halo_oneb() {
    static const int v = [] { const char* e = getenv("CDM_HALO_ONEB"); return e ? atoi(e) : 1; }();
    return v;
}

static int halo_oneb_bwd() {   // the bf16 BN-backward dgrad, one barrier per chunk: default on since round 4 (bf16
                               // g / y; profiles/r4_ab_c4_knobs.txt)
    static const int v = [] { const char* e = getenv("CDM_HALO_ONEB_BWD"); return e ? atoi(e) : 1; }();
    return v;
}

// the two-chunk-deep halo prefetch of the one-term forward halo conv ($CDM_HALO_DEEP=0: one chunk ahead)
static int halo_deep() {
    static const int v = [] { const char* e = getenv("CDM_HALO_DEEP"); return e ? atoi(e) : 1; }();
    return v;
}

// XT / OT: element types of the source (x, PRE's y) and of the stored output; bf16 only with the one-term (C4)
// arithmetic
template <int WT, class PRE = PreNone, class XT = float, class OT = float, bool ACC = false, bool FUSE = false>
static int launch_conv_halo(const XT* x, int N, int H, int Cin, int ldx, const __bf16* wx3, int Cout,
                            const float* amax_x, const float* amax_w, const EpiStoreW<4, OT, ACC, FUSE>& ep, int nterm,
                            hipStream_t s, PRE pre = PRE{}, int tpb = 0) {
    using EP = EpiStoreW<4, OT, ACC, FUSE>;
    constexpr bool F32 = std::is_same<XT, float>::value && std::is_same<OT, float>::value;
    const int M = N * H * WT, mtiles = M / HBM_;
    // the kernel addresses the halo sources (x, pre.y) by 32-bit byte offsets from their base
    if ((unsigned long long)M * (unsigned)ldx * sizeof(XT) >= (1ull << 32)) return (int)hipErrorInvalidValue;
    if constexpr (PRE::kind == 1) {
        if ((unsigned long long)M * (unsigned)pre.ldy * sizeof(XT) >= (1ull << 32)) return (int)hipErrorInvalidValue;
    }
    if (!F32 && nterm != 1) return (int)hipErrorInvalidValue;
    if (tpb < 1) tpb = halo_tpb(mtiles, (Cout + GBN - 1) / GBN, nterm, WT);
    dim3 grid((mtiles + tpb - 1) / tpb, (Cout + GBN - 1) / GBN, 1);
    if constexpr (WT > 64) {
        // wide rows (C5: 128 / 256 columns): a block is 256 / WT whole rows, halo (256/WT + 2) x (WT + 2);
        // LDS fits the two-term (h3) image only (WT 256: 2 x 2 x 774 px x 32 B + 48 KiB B = 145 KiB)
        if constexpr (!F32) {
            return (int)hipErrorInvalidValue;
        } else {
            if (nterm != NT_H3) return (int)hipErrorInvalidValue;
            hipLaunchKernelGGL((conv3x3_halo_x3_kernel<NT_H3, WT, EP, true, 1, PRE>), grid, dim3(HTHREADS), 0, s,
                               x, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, pre, mtiles, tpb, halo_stagger(nterm));
            return cdm_status();
        }
    } else {
    switch (nterm) {
        case 1:
            if constexpr (!PRE::on) {
                if (halo_oneb() && halo_deep() && Cin % 32 == 0) {
                    hipLaunchKernelGGL((conv3x3_halo_x3_kernel<1, WT, EP, true, 1 | 2048 | 4096, PRE, XT>),
                                       grid, dim3(HTHREADS), 0, s, x, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, pre,
                                       mtiles, tpb, halo_stagger(nterm));
                    break;
                }
            }
            // (the BN-backward staging form spills 12 VGPRs with the 9-tap B set: one barrier per chunk only by request)
            if (PRE::on ? halo_oneb_bwd() : halo_oneb())
                hipLaunchKernelGGL((conv3x3_halo_x3_kernel<1, WT, EP, true, 1 | 2048, PRE, XT>), grid, dim3(HTHREADS),
                                   0, s, x, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, pre, mtiles, tpb, halo_stagger(nterm));
            else
                hipLaunchKernelGGL((conv3x3_halo_x3_kernel<1, WT, EP, true, 1, PRE, XT>), grid, dim3(HTHREADS), 0, s,
                                   x, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, pre, mtiles, tpb, halo_stagger(nterm));
            break;
        default:
            if constexpr (F32) {
                if (nterm == NT_H3) {
                    hipLaunchKernelGGL((conv3x3_halo_x3_kernel<NT_H3, WT, EP, true, 1, PRE>), grid, dim3(HTHREADS), 0,
                                       s, x, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, pre, mtiles, tpb, halo_stagger(nterm));
                } else if constexpr (!FUSE) {   // the x3 / x6 arithmetics: no fused eval epilogue
                    switch (nterm) {
                        case 3: hipLaunchKernelGGL((conv3x3_halo_x3_kernel<3, WT, EP, true, 1, PRE>), grid, dim3(HTHREADS), 0, s, x, H,
                                                   Cin, ldx, wx3, Cout, amax_x, amax_w, ep, pre, mtiles, tpb, halo_stagger(nterm)); break;
                        case 6: hipLaunchKernelGGL((conv3x3_halo_x3_kernel<6, WT, EP, true, 0, PRE>), grid, dim3(HTHREADS), 0, s, x, H,
                                                   Cin, ldx, wx3, Cout, amax_x, amax_w, ep, pre, mtiles, tpb, halo_stagger(nterm)); break;
                        default: return (int)hipErrorInvalidValue;
                    }
                } else {
                    return (int)hipErrorInvalidValue;
                }
            } else {
                return (int)hipErrorInvalidValue;
            }
    }
    return cdm_status();
    }
}

// LDS-halo conv of a W x W image (W in {32, 64}; 128 / 256 with the h3 arithmetic only)
template <class PRE = PreNone, class XT = float, class OT = float, bool ACC = false, bool FUSE = false>
static int launch_conv_halo_w(int W, const XT* x, int N, int H, int Cin, int ldx, const __bf16* wx3, int Cout,
                              const float* amax_x, const float* amax_w, const EpiStoreW<4, OT, ACC, FUSE>& ep, int nterm,
                              hipStream_t s, PRE pre = PRE{}) {
    if constexpr (FUSE) {   // the fused eval epilogue: 32^2 / 64^2 maps (C2 / C4)
        switch (W) {
            case 32: return launch_conv_halo<32, PRE, XT, OT, ACC, FUSE>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep,
                                                                         nterm, s, pre);
            case 64: return launch_conv_halo<64, PRE, XT, OT, ACC, FUSE>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep,
                                                                         nterm, s, pre);
            default: return (int)hipErrorInvalidValue;
        }
    } else if constexpr (ACC) {   // the accumulating (load-ahead epilogue) variant: the dgrads at 32^2 / 64^2 only
        switch (W) {
            case 32: return launch_conv_halo<32, PRE, XT, OT, ACC>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, nterm,
                                                                   s, pre);
            case 64: return launch_conv_halo<64, PRE, XT, OT, ACC>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, nterm,
                                                                   s, pre);
            default: return (int)hipErrorInvalidValue;
        }
    } else {
    switch (W) {
        case 32: return launch_conv_halo<32, PRE, XT, OT>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, nterm, s, pre);
        case 64: return launch_conv_halo<64, PRE, XT, OT>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, nterm, s, pre);
        case 128: return launch_conv_halo<128, PRE, XT, OT>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, nterm, s, pre);
        case 256:   // the BN-backward staging registers do not fit next to the 7 halo pieces of a 256-wide row
            if constexpr (PRE::on) return (int)hipErrorInvalidValue;
            else return launch_conv_halo<256, PRE, XT, OT>(x, N, H, Cin, ldx, wx3, Cout, amax_x, amax_w, ep, nterm, s, pre);
        default: return (int)hipErrorInvalidValue;
    }
    }
}
static bool halo_width_ok(int W, int nterm) {
    return W == 32 || W == 64 || ((W == 128 || W == 256) && nterm == NT_H3);
}

}  // namespace cdm

using namespace cdm;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// The "x16" entry points run the LDS-halo / kernel-row / split-GEMM kernels in either 16-bit arithmetic
// (nterm = NT_H3: fp32-class scaled fp16 hi/lo; nterm = 1: one bf16 term, the C4 mixed-precision configuration),
// with every train-mode fusion available to both; the *_h3 names are the same calls with nterm = NT_H3.  The operand
// maxima (amax_*) scale the h3 operands only and may be null for nterm = 1.
static inline bool x16_ok(int nterm) { return nterm == NT_H3 || nterm == 1; }
static inline bool x16_amax_ok(int nterm, const void* a, const void* b) { return nterm != NT_H3 || (a && b); }

// The LDS-halo forward of cdm_conv3x3_fwd_x16 / _ex for one pair of source / output element types (XT, OT): the
// fp32 pair is instantiated in conv_fwd.hip, the bf16 pairs of C4's fused chain in conv_fwd16.hip (halo_fwd_16).
struct HaloFwdArgs {
    const float* x; int N, H, W, Cin, ldx; const void* wx; const float* amax_x; const float* amax_w; const float* bias;
    float* y; int ldy, Cout, flags; float* stats; int stats_ld; int nterm; float* amax_y; hipStream_t st;
    const float* pre_s; const float* pre_t; int* ymm; int ymm_ld;
};
template <class XT, class OT>
static int halo_fwd_run(const HaloFwdArgs& a) {
    const int M = a.N * a.H * a.W;
    const __bf16* b = reinterpret_cast<const __bf16*>(a.wx);
    const XT* xx = reinterpret_cast<const XT*>(a.x);
    if constexpr (std::is_same<OT, float>::value) {   // an accumulating dgrad: the load-ahead epilogue
        if ((a.flags & EPI_ACCUM) && !a.pre_s && !a.stats && !a.ymm && a.W <= 64) {
            const EpiStoreW<4, float, true> ea{a.y, a.ldy, 0, a.bias, a.Cout, a.flags, nullptr, 0, M, a.Cout, a.amax_y};
            return launch_conv_halo_w(a.W, xx, a.N, a.H, a.Cin, a.ldx, b, a.Cout, a.amax_x, a.amax_w, ea, a.nterm, a.st);
        }
    }
    EpiStoreW<4, OT> eh{reinterpret_cast<OT*>(a.y), a.ldy, 0, a.bias, a.Cout, a.flags, a.stats, a.stats_ld, M, a.Cout,
                        a.amax_y};
    eh.ymm = a.ymm; eh.ymm_ld = a.ymm_ld;
    if (a.pre_s)
        return launch_conv_halo_w(a.W, xx, a.N, a.H, a.Cin, a.ldx, b, a.Cout, a.amax_x, a.amax_w, eh, a.nterm, a.st,
                                  PreBnRelu{{a.pre_s, a.pre_t}});
    return launch_conv_halo_w(a.W, xx, a.N, a.H, a.Cin, a.ldx, b, a.Cout, a.amax_x, a.amax_w, eh, a.nterm, a.st);
}
int halo_fwd_16(const HaloFwdArgs& a, int dt);   // conv_fwd16.hip: dt 1 (bf16 x), 2 (bf16 y), 3 (both)
