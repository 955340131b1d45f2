/*
 * cdm_hip.h — C ABI of libcdm_hip.so, the MI355X (gfx950) kernels behind the ContextUnet DDPM
 * hot path.  Plain pointers and sizes only (no torch types).  Every function returns 0 on success
 * or a hipError_t code; launches go on the caller's stream (`stream` is a hipStream_t, NULL =
 * default stream); the library never allocates, never synchronises and keeps no global state, so
 * every call can be captured into a hipGraph.
 *
 * The reference has no FFI: its boundary is the Python module API.  Each entry point
 * below names the reference operation it replaces (paths relative to the reference repo root).
 * Layout: activations NHWC fp32, (N,H,W,C) with a pixel stride `ld*` >= C so that channel slices
 * of concatenation buffers are addressable (replaces torch.cat, diffusion_utilities.py:96 and
 * ContextUnet.py:59).  Weights are the reference OIHW / ConvTranspose [Cin][Cout][kh][kw] tensors
 * repacked by cdm_pack_* into GEMM layouts.
 */
#ifndef CDM_HIP_H
#define CDM_HIP_H
#ifdef __cplusplus
extern "C" {
#endif

#define CDM_EPI_RELU 1
#define CDM_EPI_ACCUM 2

int cdm_abi_version(void);
int cdm_device_sync(void);

/* ---- contractions (fp32 MFMA 32x32x2; csrc/gemm_f32.hip) -------------------------------------- */
/* nn.Conv2d(Cin,Cout,3,1,1) forward (diffusion_utilities.py:27,34; ContextUnet.py:36) and, with
 * flipped weights, its input gradient.  y (+)= conv(x) + bias; stats[tile][2][stats_ld] receives
 * per-128-pixel column sums / sums of squares (BatchNorm2d batch statistics, diffusion_utilities.py:28).
 * kc must equal the kc the weights were packed with (cdm_pack_conv3x3). */
int cdm_conv3x3_fwd(const float* x, int N, int H, int W, int Cin, int ldx, const float* wpk, const float* bias,
                    float* y, int ldy, int Cout, int flags, float* stats, int stats_ld, int kc, void* stream);
/* same, selecting a kernel variant (tuning: 0 default, 1 BK32, 2 XCD remap, 3 chunked K, 4 = 2+3) */
int cdm_conv3x3_fwd_variant(int variant, const float* x, int N, int H, int W, int Cin, int ldx, const float* wpk,
                            const float* bias, float* y, int ldy, int Cout, int flags, float* stats, int stats_ld,
                            void* stream);
/* conv3x3 forward, fp32-accurate on the bf16 matrix cores: operands split into nterm-term bf16 sums
 * (nterm 6 = fp32-class, 3 = bf16x3, 1 = bf16); wx3 from cdm_split_bf16x3 of the packed weights.
 * Same semantics as cdm_conv3x3_fwd (nn.Conv2d(.,.,3,1,1) diffusion_utilities.py:27,34). */
int cdm_conv3x3_fwd_x3(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx3, const float* bias,
                       float* y, int ldy, int Cout, int flags, float* stats, int stats_ld, int kc, int nterm,
                       void* stream);
/* conv3x3 weight gradient on the split-bf16 path: same slab contract as cdm_conv3x3_wgrad; W % 8 == 0 */
int cdm_conv3x3_wgrad_x3(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin, int ldx,
                         int splits, float* slab, int nterm, void* stream);
/* fp32 [K][N] (ld ldb) -> [ceil(K/16)][3][N][16] bf16 split terms hi/mid/lo */
int cdm_split_bf16x3(const float* b, long long ldb, int K, int N, void* out, void* stream);
/* fp32-class conv3x3 on the fp16 matrix cores ("h3"): each operand is scaled by a power of two derived
 * from its max |.| (device scalars amax_x / amax_w, see cdm_amax_f32) and split into fp16 hi + lo;
 * 3 cross products (hh, hl, lh) per MAC, fp32 accumulate, exact unscale.  wx from cdm_split_f16x2 of
 * the packed weights with the same amax_w.  Same semantics as cdm_conv3x3_fwd. */
int cdm_conv3x3_fwd_h3(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx, const float* amax_x,
                       const float* amax_w, const float* bias, float* y, int ldy, int Cout, int flags, float* stats,
                       int stats_ld, int kc, float* amax_y, void* stream);
/* cdm_conv3x3_fwd_h3 with the train-mode Conv -> BatchNorm -> ReLU fusions (LDS-halo shapes only):
 * pre_s / pre_t (optional): the input is relu(x * pre_s[c] + pre_t[c]) computed while staging (x = the previous
 * layer's pre-norm output; its BatchNorm apply is never materialised; *amax_x must be max of that input);
 * ymm (optional, needs stats): per output channel max / min of y as ordered-int keys ymm[c] / ymm[ymm_ld + c],
 * cleared by the caller to INT_MIN / INT_MAX (cdm_fill_i32); cdm_bn_fwd_finalize turns them into max|z| */
int cdm_conv3x3_fwd_h3_ex(const float* x, int N, int H, int W, int Cin, int ldx, const float* pre_s, const float* pre_t,
                          const void* wx, const float* amax_x, const float* amax_w, const float* bias, float* y, int ldy,
                          int Cout, int flags, float* stats, int stats_ld, int kc, float* amax_y, int* ymm, int ymm_ld,
                          void* stream);
/* eval-mode conv3x3 of a Conv -> BatchNorm (folded into wx / bias) -> ReLU layer with its output transform in the
 * LDS-halo epilogue (csrc/conv_fwd_eval.hip; W == H in {32, 64}, kc = 16, Cout % 128 == 0), v = relu(conv + bias):
 *   kind 1 (resid, diffusion_utilities.py:54-55): y[p][c] = sc_w[s][c] sc_x[p] + sc_b[s][c] + v, s = image >= split
 *   kind 2 (FiLM, ContextUnet.py:57-58):           y[p][c] = fa[image * fan + c] v + fb[image * fbn + c]
 *   kind 3 (MaxPool2d(2), diffusion_utilities.py:109): y = the [N][H/2][W/2] pooled map (row stride ldy)
 * amax_y (h3): running max|y|.  Replaces cdm_conv3x3_fwd_x16 + cdm_norm_apply_fwd of the eval forward. */
int cdm_conv3x3_fwd_x16_fused(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx,
                              const float* amax_x, const float* amax_w, const float* bias, float* y, int ldy, int Cout,
                              int kc, float* amax_y, int kind, const float* sc_x, const float* sc_w, const float* sc_b,
                              int split, const float* fa, int fan, const float* fb, int fbn, int nterm, void* stream);
/* timing ablations of the h3 LDS-halo conv (64x64 maps, no bias / stats; tools/conv_ablation.py): abl bits
 * 1 fragment prefetch, 2 MFMAs doubled, 4 B staged once, 8 halo without the term split (results meaningless);
 * bits 16+: tiles per block (0 -> 1) */
int cdm_conv3x3_halo_ablate(int abl, const float* x, int N, int H, int Cin, int ldx, const void* wx,
                            const float* amax_x, const float* amax_w, float* y, int ldy, int Cout, void* stream);
int cdm_conv3x3_wgrad_h3(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin, int ldx,
                         const float* amax_dy, const float* amax_x, int splits, float* slab, void* stream);
/* measurement entry of the h3 weight gradient: variant 0 = kernel-row kernel (3 taps per block, 32-pixel K steps,
 * the default), 1 = per-tap kernel, 2 = generic split GEMM, 3 = kernel-row kernel with 16-pixel K steps; same
 * slab contract */
int cdm_conv3x3_wgrad_h3_variant(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin,
                                 int ldx, const float* amax_dy, const float* amax_x, int splits, float* slab,
                                 int variant, void* stream);
/* Conv -> BatchNorm -> ReLU backward with the BN backward fused into the conv staging (dy never written):
 * dy = A (y s + t > 0 ? g : 0) + B + Cc (y - mean) invstd per element (the expression of cdm_norm_apply_bwd
 * mode 0, bit-identical), s/t/mean/invstd/A/B/Cc per channel.  dgrad: LDS-halo kernel, W == H in {32, 64, 128},
 * C % 16 == 0, C <= 256, C = BN channels, Cout = dgrad output channels, wx = split packed dgrad weights;
 * wgrad: kernel-row kernel (Cin, Cout % 128 == 0, W % 16 == 0), same slab contract as cdm_conv3x3_wgrad_h3.
 * max|dy| <= *amax_dy from cdm_bn_bwd_amax_bound. */
int cdm_conv3x3_dgrad_h3_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                               const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                               int N, int H, int W, int C, const void* wx, const float* amax_dy, const float* amax_w,
                               float* out, int ldo, int Cout, int flags, float* amax_out, void* stream);
int cdm_conv3x3_wgrad_h3_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                               const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                               int Cout, const float* x, int N, int H, int W, int Cin, int ldx, const float* amax_dy,
                               const float* amax_x, int splits, float* slab, void* stream);
/* the kernel-row weight gradient with both staging fusions selectable: y (+ s, t, mean, invstd, A, B, Cc) non-null:
 * dY = the BatchNorm backward of g (as cdm_conv3x3_wgrad_h3_bnbwd), else dY = g; x_s / x_t non-null: the X operand
 * is relu(x * x_s[c] + x_t[c]).  Cin % 128 == Cout % 128 == 0, W % 16 == 0. */
int cdm_conv3x3_wgrad_h3_ex(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                            const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                            int Cout, const float* x, int N, int H, int W, int Cin, int ldx, const float* x_s,
                            const float* x_t, const float* amax_dy, const float* amax_x, int splits, float* slab,
                            void* stream);
/* ---- the 16-bit-arithmetic ("x16") forms of the h3 entry points above and of the h3 ConvT 2x2 calls below ----------
 * identical contracts plus a trailing `nterm`: NT_H3 = 4 (fp32-class scaled fp16 hi/lo, = the *_h3 call) or 1 (one
 * bf16 term per operand, fp32 accumulate: BASELINE configuration C4, bf16 mixed precision, with every train-mode
 * Conv -> BatchNorm -> ReLU fusion of the h3 path).  For nterm = 1 the weight images come from cdm_split_bf16x3 (plane
 * 0 is read) and the amax_* operand maxima are ignored (may be null).  Reference ops: nn.Conv2d(.,.,3,1,1)
 * diffusion_utilities.py:27,34 and its autograd; nn.ConvTranspose2d(Cin, Cout, 2, 2) diffusion_utilities.py:86. */
/* dt (the x16 conv entry points): bf16 activation storage of C4's fused Conv -> BatchNorm -> ReLU chain, one-term
 * (nterm = 1) arithmetic only.  Forward / dgrad: bit 0 = the source (x or g, and the BN staging's y) holds bf16, bit 1 =
 * the output is stored as bf16 (statistics / maxima of the stored values).  Weight gradient: bit 0 = g / dy (and y) are
 * bf16, bit 1 = x (and x_g) are bf16.  dt = 0: fp32 everywhere (every other arithmetic). */
int cdm_conv3x3_fwd_x16(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx, const float* amax_x,
                        const float* amax_w, const float* bias, float* y, int ldy, int Cout, int flags, float* stats,
                        int stats_ld, int kc, float* amax_y, int nterm, int dt, void* stream);
int cdm_conv3x3_fwd_x16_ex(const float* x, int N, int H, int W, int Cin, int ldx, const float* pre_s, const float* pre_t,
                           const void* wx, const float* amax_x, const float* amax_w, const float* bias, float* y,
                           int ldy, int Cout, int flags, float* stats, int stats_ld, int kc, float* amax_y, int* ymm,
                           int ymm_ld, int nterm, int dt, void* stream);
int cdm_conv3x3_wgrad_x16(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin, int ldx,
                          const float* amax_dy, const float* amax_x, int splits, float* slab, int nterm, void* stream);
int cdm_conv3x3_dgrad_x16_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                                const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                                int N, int H, int W, int C, const void* wx, const float* amax_dy, const float* amax_w,
                                float* out, int ldo, int Cout, int flags, float* amax_out, int nterm, int dt,
                                void* stream);
/* the same, also storing the dy it computes into dy_out ([pix][C], g's row stride ldg and element type) for the
 * layer's weight gradient (cdm_conv3x3_wgrad_x16_ex with g = dy_out, y = null): the BN backward is evaluated once per
 * element instead of again in each of the weight gradient's 3 kernel-row blocks. */
int cdm_conv3x3_dgrad_x16_bnbwd_dy(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                                   const float* mean, const float* invstd, const float* A, const float* B,
                                   const float* Cc, int N, int H, int W, int C, const void* wx, const float* amax_dy,
                                   const float* amax_w, float* out, int ldo, int Cout, int flags, float* amax_out,
                                   void* dy_out, int nterm, int dt, void* stream);
int cdm_conv3x3_wgrad_x16_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                                const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                                int Cout, const float* x, int N, int H, int W, int Cin, int ldx, const float* amax_dy,
                                const float* amax_x, int splits, float* slab, int nterm, int dt, void* stream);
/* cdm_conv3x3_wgrad_x16_ex also takes (x_g, ldxg, x_mean, x_invstd, x_sums), all optional (x_sums null: off): with
 * x_s / x_t given, the BatchNorm-backward channel sums of the layer that produced x are accumulated while x is staged:
 * g_pre = (x x_s + x_t > 0 ? x_g : 0), xhat = (x - x_mean) x_invstd; x_sums[(split * 3 + kernel row) * (Cout / 128) +
 * co tile][5][Cin] (one partial per block, splits = effective split count) rows 0 = sum g_pre, 1 = sum g_pre xhat,
 * 4 = sum xhat (rows 2, 3 zero) — the slab of cdm_norm_bwd_reduce mode 0 with 3 Cout/128 tiles per split
 * (x_g = the gradient wrt this conv's input, written by this layer's dgrad before this call). */
int cdm_conv3x3_wgrad_x16_ex(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                             const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                             int Cout, const float* x, int N, int H, int W, int Cin, int ldx, const float* x_s,
                             const float* x_t, const float* x_g, int ldxg, const float* x_mean, const float* x_invstd,
                             float* x_sums, const float* amax_dy, const float* amax_x, int splits, float* slab,
                             int nterm, int dt, void* stream);
int cdm_convT2x2_fwd_x16(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx, const float* amax_x,
                         const float* amax_w, const float* bias, float* y, int ldy, int Cout, float* amax_y, int nterm,
                         void* stream);
int cdm_convT2x2_dgrad_x16(const float* dy, int N, int H, int W, int Cout, int lddy, const void* wx,
                           const float* amax_dy, const float* amax_w, float* dx, int lddx, int Cin, int flags, int nterm,
                           void* stream);
int cdm_convT2x2_wgrad_x16(const float* x, int N, int H, int W, int Cin, int ldx, const float* dy, int Cout, int lddy,
                           const float* amax_x, const float* amax_dy, int splits, float* slab, int nterm, void* stream);
/* fp32 [K][N] (ld ldb) -> [ceil(K/16)][3][N][16]: planes 0/1 = fp16 hi/lo of b * 2^(14-e), max|b| = *amax < 2^e */
int cdm_split_f16x2(const float* b, long long ldb, int K, int N, const float* amax, void* out, void* stream);
/* batched train-mode repack: jobs_dev = device array of njobs records
 *   { const float* W (OIHW); int Cin, Cout, kc, pad; bf16* wpk_x; bf16* wdg_x (may be null); float* amax; }
 * (64-bit pointers, 48 bytes per record); writes max|W| (atomic max into a cleared *amax) and the two h3 split
 * images of cdm_pack_conv3x3 + cdm_split_f16x2 directly from W.  max_w_elems = the largest Cout * Cin * 9. */
int cdm_pack_split_conv3x3_batch(const void* jobs_dev, int njobs, long long max_w_elems, void* stream);
/* *out = max(accumulate ? *out : 0, max |x[r*ld + c]|), r < rows, c < C (atomic max, graph-capturable) */
int cdm_amax_f32(const float* x, long long rows, int C, long long ld, float* out, int accumulate, void* stream);
/* ---- sample statistics (csrc/stats.hip) --------------------------------------------------------
 * power[b][u][v] = |sum_{x,y} img[b][x][y] e^{-2 pi i (u x + v y) / N}|^2 * scale, fp64 (direct DFT; T = scratch of
 * B*N*N complex doubles).  scale 1/N^2 = np.fft.fftn(norm="ortho") of power_spectrum, diffusion_utilities.py:322;
 * scale 1 = np.fft.fft2 of calculate_power_spectrum_2d, sample_power_spectra.py:128. */
int cdm_dft2_power(const float* img, int B, int N, double scale, void* T, double* power, void* stream);
/* power[b] = |fftn(box[b])|^2 * scale, fp64, for B row-major boxes of rank 1..3 with extents dims[0..rank) (host
 * array): one direct-DFT pass per axis; T0, T1 = scratch of B * prod(dims) complex doubles each.  The 3-D and non-square
 * branches of power_spectrum (diffusion_utilities.py:316-336). */
int cdm_dftn_power(const float* box, int B, int rank, const int* dims, double scale, void* T0, void* T1, double* power,
                   void* stream);
/* cdm_dftn_power for fp64 boxes: power_spectrum of a float64 numpy box, whose np.fft.fftn runs on the fp64 values
 * (diffusion_utilities.py:322) — no fp32 rounding of the input. */
int cdm_dftn_power_f64(const double* box, int B, int rank, const int* dims, double scale, void* T0, void* T1,
                       double* power, void* stream);
/* out[b][k] = sum_{i = off[k]}^{off[k+1]-1} power[b][idx[i]] in list order (the reference's binning loops,
 * diffusion_utilities.py:352-356 / sample_power_spectra.py:157-163, with the bin geometry built on the host) */
int cdm_bin_sum(const double* power, int B, long long NN, const int* off, const int* idx, int nbins, double* out,
                void* stream);
/* out[b] = np.histogram(x[b], edges[0..nbins], density=True)[0]  (train_diffusion.py:205-207) */
int cdm_histogram_density(const float* x, int B, long long P, const double* edges, int nbins, double* out,
                          void* stream);
/* ---- CAMELS map preprocessing (csrc/data.hip; code/train_diffusion_condition.py:137-144) ----------------------- */
/* out[0], out[1] = min, max of x[0..n) (keys = 2 unsigned of scratch; order-independent atomics) */
int cdm_minmax_f32(const float* x, long long n, unsigned* keys, float* out, void* stream);
/* dst[N][O][O] = bilinear(O x O, align_corners=False)((log10(shift(src) / max) - min) / (max - min)) of src[N][S][S],
 * with minmax = cdm_minmax_f32 of the whole raw dataset (every step of the reference is monotone) */
int cdm_camels_maps(const float* src, int N, int S, int O, const float* minmax, float* dst, void* stream);
/* p[0..n) = 0 (a fill kernel: graph-capturable; a captured hipMemsetAsync did not clear reliably on replay) */
int cdm_zero_f32(float* p, long long n, void* stream);
/* Producers below (cdm_norm_apply_fwd / _bwd, cdm_convT2x2_fwd, cdm_conv3x3_fwd_h3 amax_y) take an optional
 * float* amax: when non-null they atomically max the |values| they store into it, so the next h3 conv gets
 * its operand's max without a separate pass. */
/* nn.ConvTranspose2d(Cin,Cout,2,2) forward (diffusion_utilities.py:86); H,W = input grid. */
int cdm_convT2x2_fwd(const float* x, int N, int H, int W, int Cin, int ldx, const float* wpk, const float* bias,
                     float* y, int ldy, int Cout, float* amax, void* stream);
/* the same on the fp16 matrix cores (h3); wx = cdm_split_f16x2 of wpk [Cin][4*Cout] with max|wpk| = *amax_w */
int cdm_convT2x2_fwd_h3(const float* x, int N, int H, int W, int Cin, int ldx, const void* wx, const float* amax_x,
                        const float* amax_w, const float* bias, float* y, int ldy, int Cout, float* amax_y,
                        void* stream);
/* its input gradient (autograd of diffusion_utilities.py:86). */
int cdm_convT2x2_dgrad(const float* dy, int N, int H, int W, int Cout, int lddy, const float* wpkT, float* dx,
                       int lddx, int Cin, int flags, void* stream);
/* dense C = A.B (+bias[n % bias_mod]): up0 ConvTranspose2d(2nf,2nf,h/4,h/4) on a 1x1 map (ContextUnet.py:27)
 * and its input gradient (split-K partial slabs when splits > 1). */
int cdm_gemm_f32(const float* a, long long lda, int M, int K, const float* b, long long ldb, int N, float* c,
                 long long ldc, const float* bias, int bias_mod, int flags, int splits, float* slab, void* stream);
int cdm_gemm_splits(int K, int splits);
/* C[m][n] = A[m][k] . B[k][n] + bias[n % bias_mod] on the 16-bit matrix cores (nterm 4 = h3, 1 = bf16); wx = the split
 * image of B [K][N] (cdm_split_f16x2 with max|B| in *amax_w / cdm_split_bf16x3); h3: max|A| = *amax_a; amax_c
 * (optional): running max|C|.  The up0 ConvTranspose2d(k = h/4) of the 1x1 map (ContextUnet.py:26-30). */
int cdm_gemm_x16(const float* a, long long lda, int M, int K, const void* wx, const float* amax_a, const float* amax_w,
                 int N, float* c, long long ldc, const float* bias, int bias_mod, float* amax_c, int nterm,
                 void* stream);
/* weight gradients (autograd of the layers above), split-K partial slabs [splits][M][N]. */
int cdm_conv3x3_wgrad(const float* dy, int lddy, int Cout, const float* x, int N, int H, int W, int Cin, int ldx,
                      int splits, float* slab, void* stream);
int cdm_convT2x2_wgrad(const float* x, int N, int H, int W, int Cin, int ldx, const float* dy, int Cout, int lddy,
                       int splits, float* slab, void* stream);
/* h3 variants of the ConvT 2x2 backward: dgrad with wx = cdm_split_f16x2 of wpkT [4 Cout][Cin] (max|W| = *amax_w)
 * and max|dy| = *amax_dy; wgrad with max|x| = *amax_x, max|dy| = *amax_dy (W % 8 == 0).  Same semantics. */
int cdm_convT2x2_dgrad_h3(const float* dy, int N, int H, int W, int Cout, int lddy, const void* wx,
                          const float* amax_dy, const float* amax_w, float* dx, int lddx, int Cin, int flags,
                          void* stream);
int cdm_convT2x2_wgrad_h3(const float* x, int N, int H, int W, int Cin, int ldx, const float* dy, int Cout, int lddy,
                          const float* amax_x, const float* amax_dy, int splits, float* slab, void* stream);
int cdm_gemm_tn_f32(const float* a, long long lda, int M, int K, const float* b, long long ldb, int N, int splits,
                    float* slab, void* stream);
/* out[m*s_m + (n/csplit)*s_hi + (n%csplit)*s_lo] (+)= scale * sum_z slab[z][m][n] */
int cdm_slab_reduce(const float* slab, int splits, int M, int N, float* out, long long s_m, long long s_hi,
                    long long s_lo, int csplit, int accumulate, float scale, void* stream);

/* ---- normalisation / pooling / FiLM (csrc/norm.hip) ------------------------------------------- */
/* per-(image, pixel-chunk) partial sums (slab[N][chunks][R][C]) */
int cdm_reduce_stats(const float* y, int ldy, int N, int HW, int C, int csize, float* slab, void* stream);
/* cdm_reduce_stats (identical slab) + optional (ymm != NULL) per-channel max / min of y as ordered-int keys, atomic max
 * into ymm[c] / min into ymm[ymm_ld + c] (cleared by the caller to INT_MIN / INT_MAX): the C_in = 1 init conv's
 * BatchNorm statistics when its BN-ReLU apply runs in the next conv's staging. */
int cdm_reduce_stats_mm(const float* y, int ldy, int N, int HW, int C, int csize, float* slab, int* ymm, int ymm_ld,
                        void* stream);
int cdm_reduce_sum(const float* g, int ldg, int N, int HW, int C, int csize, float* slab, void* stream);
/* BatchNorm2d / GroupNorm(8) + ReLU (+MaxPool2d(2) | +FiLM) backward sums (mode 0 plain, 1 pool, 2 FiLM) */
int cdm_norm_bwd_reduce(int mode, const float* g, int ldg, const float* y, int ldy, int N, int H, int W, int C,
                        const float* s, const float* t, int sn, const float* mean, const float* invstd, int mn,
                        int cpg, const float* film_a, int film_an, int csize, float* slab, void* stream);
/* stage 1 of every slab fold: part[s][r][c] = sum_{tiles of split s} slab[t][r][c] in fp64 (parallel) */
int cdm_slab_colsum(const float* slab, int ntiles, int R, int C, double* part, int splits, void* stream);
/* BatchNorm2d train statistics + running-stat update (diffusion_utilities.py:28,35; momentum 0.1, eps 1e-5) */
int cdm_bn_fwd_finalize(const double* part, int nparts, int R, int C, double count, const float* gamma,
                        const float* beta, float* rmean, float* rvar, long long* nbt, float momentum, float eps,
                        float* mean, float* invstd, float* scale, float* shift, const int* ymm, int ymm_ld,
                        float* amax_z, void* stream);
/* (ymm optional: the per-channel max / min keys of the layer's y from cdm_conv3x3_fwd_h3_ex; amax_z then receives
 *  the exact max over the layer of relu(fmaf(y, scale, shift)) by an atomic max, for the consumer's h3 scale) */
/* p[0..n) = v */
int cdm_fill_i32(int* p, long long n, int v, void* stream);
/* BatchNorm2d eval (running statistics) */
int cdm_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                       float* mean, float* invstd, float* scale, float* shift, void* stream);
/* GroupNorm(8, C) statistics (ContextUnet.py:28,37) */
int cdm_gn_fwd_finalize(const float* slab, int N, int nchunks, int R, int C, int G, double count, const float* gamma,
                        const float* beta, float eps, float* mean, float* invstd, float* scale, float* shift,
                        void* stream);
int cdm_bn_bwd_finalize(const double* part, int nparts, int C, double count, const float* gamma, const float* invstd,
                        float* dgamma, float* dbeta, float* A, float* B, float* Cc, float* dbias, void* stream);
/* eval-mode BatchNorm in the train-structured forward / backward (gradients through model.eval(), the reference's
 * batch_norm(training=False) under autograd): coefficients from the running statistics (running stats and
 * num_batches_tracked untouched; ymm / amax_z as cdm_bn_fwd_finalize), and the backward finalize with the batch terms
 * dropped (A = gamma invstd, B = Cc = 0, dgamma = S2, dbeta = S1, dbias = A S1) */
int cdm_bn_fwd_frozen(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                      float* mean, float* invstd, float* scale, float* shift, const int* ymm, int ymm_ld, float* amax_z,
                      void* stream);
int cdm_bn_bwd_finalize_frozen(const double* part, int nparts, int C, double count, const float* gamma,
                               const float* invstd, float* dgamma, float* dbeta, float* A, float* B, float* Cc,
                               float* dbias, void* stream);
int cdm_gn_bwd_finalize(const float* slab, int N, int nchunks, int C, int G, double count_g, int HW,
                        const float* gamma, const float* invstd, float* A, float* B, float* Cc, float* pdg, float* pdb,
                        float* pdbias, void* stream);
int cdm_slab_sum_nc(const float* slab, int N, int nchunks, int R, int r, int C, float* out, void* stream);
int cdm_col_sum(const float* in, int N, int C, float* out, int accumulate, void* stream);
/* up to three column sums out_k[c] = sum_n in_k[n][c] in one launch (in1 / in2 may be null) */
int cdm_col_sum3(const float* in0, float* out0, const float* in1, float* out1, const float* in2, float* out2, int N,
                 int C, void* stream);
/* out = [MaxPool2d(2)]([cemb*](ReLU(y*s+t))[+temb])[+ 1x1 shortcut(x)]  — flags 1 pool, 2 FiLM, 4 resid, 8 relu
 * (BN/GN apply diffusion_utilities.py:28-29; MaxPool2d :109; random shortcut :54-55; FiLM ContextUnet.py:57-58) */
int cdm_norm_apply_fwd(int flags, const float* y, int ldy, int N, int H, int W, int C, const float* s, const float* t,
                       int sn, const float* film_a, int film_an, const float* film_b, int film_bn, const float* rx,
                       const float* rw, const float* rb, int rsplit, float* out, int ldo, float* amax, void* stream);
/* the same residual apply for in_channels = xc > 1 (ContextUnet.py:6,14 — init_conv = ResidualConvBlock(in_channels,
 * n_feat, is_res=True), the 1x1 shortcut of diffusion_utilities.py:54-55 over xc channels):
 * out = [relu](y*s+t) + rb[c] + sum_k rw[c][k] rx[p*ldx + k]; rw [2][C][xc] / rb [2][C] when rsplit < N */
int cdm_norm_apply_fwd_resid_c(int relu, const float* y, int ldy, int N, int H, int W, int C, const float* s,
                               const float* t, const float* rx, int ldx, int xc, const float* rw, const float* rb,
                               int rsplit, float* out, int ldo, float* amax, void* stream);
int cdm_norm_apply_bwd(int mode, const float* g, int ldg, const float* y, int ldy, int N, int H, int W, int C,
                       const float* s, const float* t, int sn, const float* mean, const float* invstd, int mn, int cpg,
                       const float* film_a, int film_an, const float* A, const float* B, const float* Cc, int cn,
                       float* dy, int lddy, float* amax, void* stream);
/* *amax_dy = max(*amax_dy, max_c |A| max|g| + |B| + |Cc| (max|y| + |mean|) invstd): an upper bound of max|dy| of
 * the fused BN backward (from the producers' max|g| = *amax_g and max|y| = *amax_y); one block */
/* dense BatchNorm backward of a bf16-activation (C4) layer as its own pass: dy[p][c] = the fused staging's
 * bn_bwd_elem(g, y) (s, t, mean, invstd, A, B, Cc per channel), P pixels x C channels (C % 8 == 0); dt bit 0: g and y
 * are bf16, bit 1: dy is stored as bf16 (round to nearest even) */
int cdm_bn_bwd_dy(const void* g, int ldg, const void* y, int ldy, long long P, int C, const float* s, const float* t,
                  const float* mean, const float* invstd, const float* A, const float* B, const float* Cc, void* dy,
                  int lddy, int dt, void* stream);
int cdm_bn_bwd_amax_bound(int C, const float* A, const float* B, const float* Cc, const float* mean,
                          const float* invstd, const float* amax_g, const float* amax_y, float* amax_dy, void* stream);

/* ---- small ops (csrc/misc.hip) ---------------------------------------------------------------- */
/* init_conv.conv1: Conv2d(1, nf, 3, 1, 1) (ContextUnet.py:14 -> diffusion_utilities.py:27) */
int cdm_conv3x3_cin1_fwd(const float* x, int N, int H, int W, const float* wt, const float* bias, float* y, int ldy,
                         int C, int relu, float* amax, void* stream);   /* amax: optional running max|y| (atomic) */
int cdm_conv3x3_cin1_wgrad(const float* dy, int lddy, const float* x, int N, int H, int W, int C, int csize,
                           float* slab, void* stream);
/* cdm_conv3x3_cin1_wgrad of the init conv's Conv -> BatchNorm -> ReLU with its BN backward applied while reading: g =
 * grad of the ReLU output, y = pre-norm activations, per-channel s, t, mean, invstd, A, B, Cc as cdm_norm_apply_bwd
 * mode 0 (bit-identical dy, never written).  Replaces the autograd BatchNorm2d backward + Conv2d weight grad of
 * ContextUnet.py:14 (init_conv.conv1, diffusion_utilities.py:26-30). */
int cdm_conv3x3_cin1_wgrad_bnbwd(const float* g, int ldg, const float* y, int ldy, const float* s, const float* t,
                                 const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                                 const float* x, int N, int H, int W, int C, int csize, float* slab, void* stream);
int cdm_slab_sum_all(const double* part, int nparts, int R, int r0, int rn, int C, float* out, long long s_r,
                     long long s_c, int accumulate, void* stream);
/* out.3: Conv2d(nf, 1, 3, 1, 1) (ContextUnet.py:39) */
int cdm_conv3x3_cout1_fwd(const float* z, int ldz, int N, int H, int W, int C, const float* w, const float* bias,
                          float* out, void* stream);
/* out.3 on out.1's pre-norm output y with its GroupNorm + ReLU applied while staging (gs / gt per (sample, channel),
 * [N][C]; bit-identical to cdm_norm_apply_fwd then cdm_conv3x3_cout1_fwd): eval forwards (ContextUnet.py:37-39).
 * C % 16 == 0, W | 256, (256 / W) | H. */
int cdm_conv3x3_cout1_fwd_gn(const float* y, int ldy, int N, int H, int W, int C, const float* gs, const float* gt,
                             const float* w, const float* bias, float* out, void* stream);
/* image gradient of the init conv (ResidualConvBlock(1, nf, is_res) under autograd, diffusion_utilities.py:45-55):
 * dx[n][p] = sum_{tap,c} w9[c][8 - tap] dy1[p + tap][c] + sum_c scw[(n >= split) * C + c] gres[p][c], w9 = conv1's OIHW
 * weights [C][1][3][3]; dy1 = the BatchNorm + ReLU backward of g1 with y1 and the coefficients of cdm_norm_apply_bwd
 * mode 0 (y1 == NULL: g1 is dy1); gres = the gradient of the block output (NULL: no shortcut term). */
int cdm_conv3x3_cin1_dgrad(const float* g1, int ldg, const float* y1, int ldy, const float* s, const float* t,
                           const float* mean, const float* invstd, const float* A, const float* B, const float* Cc,
                           const float* w9, const float* gres, int ldr, const float* scw, int split, int N, int H,
                           int W, int C, float* dx, void* stream);
int cdm_conv3x3_cout1_dgrad(const float* deps, int N, int H, int W, int C, const float* w, float* dz, int lddz,
                            void* stream);
/* weight gradient partials: csize > 0: per (image, csize-pixel chunk) [N][chunks][9][C]; csize = -R (band form, H % R
 * == 0): one block per R whole rows, every z pixel read once, partials [N * H / R][9][C] */
int cdm_conv3x3_cout1_wgrad(const float* deps, const float* z, int ldz, int N, int H, int W, int C, int csize,
                            float* slab, void* stream);
/* band form (csize = -R) on out.1's pre-norm output y with its GroupNorm + ReLU (per (n, c) gs / gt, [N][C]) applied
 * while staging: z = relu(y gs + gt), bit-identical to the applied tensor, never materialised */
int cdm_conv3x3_cout1_wgrad_gn(const float* deps, const float* y, int ldy, int N, int H, int W, int C, const float* gs,
                               const float* gt, int csize, float* slab, void* stream);
/* to_vec: AvgPool2d(h/4) + GELU (ContextUnet.py:17) */
int cdm_avgpool_gelu_fin(const float* sums, int N, int C, int HW, float* hpre, float* hv, void* stream);
int cdm_avgpool_gelu_bwd(const float* dhv, const float* hpre, int N, int HW, int C, float* dst, int ldd, void* stream);
/* EmbedFC x4 (diffusion_utilities.py:118-145); `P` points to a host struct cdm_mlp4 (see csrc/misc.hip MlpDesc) */
int cdm_embed_fwd(const void* P, void* stream);
/* input gradient of the two EmbedFCs fed one input (t: timeembed1/2, c: contextembed1/2; ContextUnet.py:51-54):
 * dx[b][k] = sum_i dpre_a[b][i] w1_a[i][k] + sum_i dpre_b[b][i] w1_b[i][k]  (dpre from cdm_embed_bwd, w1 [E][in_dim]) */
int cdm_embed_input_grad(const float* dpre_a, const float* w1_a, int Ea, const float* dpre_b, const float* w1_b, int Eb,
                         int rows, int in_dim, float* dx, void* stream);
int cdm_embed_bwd(const void* P, void* stream);
/* perturb_input (code/train_diffusion_condition.py:202-203) + t/T for the time embedding (:225).
 * t: per-sample steps, or cur_i: one device-side step for the batch with noise row (T - *cur_i)*nstride. */
int cdm_perturb(const float* x, const float* noise, const int* t, const int* cur_i, long long nstride,
                const float* sab, const float* omab, int N, int HW, int T, float* out, float* tin, void* stream);
/* per-sample weighted MSE accumulation of the likelihood / ELBO estimators
 * (code/train_diffusion_elbo.py:74-149; code/train_diffusion_paper.py:77-183):
 * acc[n] += (mean (pred - noise)^2 * mul[i]) / div[i], i = t[n] or *cur_i (noise row (T - i)*nstride) */
int cdm_mse_accum(const float* pred, const float* noise, long long nstride, int T, int N, int HW, const int* t,
                  const int* cur_i, const float* mul, const float* div, float* acc, void* stream);
/* F.mse_loss + its gradient (code/train_diffusion_condition.py:227): loss = mean over the n elements, dpred =
 * 2 (pred - noise) / grad_numel (grad_numel = n, or the data-parallel count of a ragged global batch);
 * nonfinite (optional): += 1 when the loss is NaN / inf (SURVEY §5 failure guard; read once per epoch) */
int cdm_mse(const float* pred, const float* noise, long long n, double grad_numel, float* dpred, float* partial, int nb,
            float* loss_out, float* dbias_out, int* nonfinite, void* stream);
/* sampler: per-step prologue (device step counter) and denoise_add_noise + CFG combine
 * (code/train_diffusion_condition.py:274-279, 312-333) */
int cdm_sample_prologue(int* ctr, int T, int* cur_i, float* t_cur, const float* sc_table, int sc_row, float* sc_cur,
                        void* stream);
/* z: z_table[(T - i) * zstride + e] when given, else Philox keyed by seed ^ *seed_dev (seed_dev optional: a
 * per-run device value, so one captured graph draws a fresh z sequence on every run) */
int cdm_denoise(const float* xin, float* x, float* x2, long long numel, const float* eps, int cfg, float w,
                const int* cur_i, const float* coef, const float* sa, const float* sb, const float* z_table,
                long long zstride, unsigned long long seed, const long long* seed_dev, const int* snap_slot,
                float* snaps, int T, void* stream);
/* randn_like / randint / the per-forward random 1x1 shortcut draw (diffusion_utilities.py:54), on-device Philox.
 * The stream id is sub (+ *sub_dev when given: a device counter advanced by cdm_counter_add, so a captured
 * step draws fresh numbers on every replay). */
int cdm_philox_normal(float* out, long long n, unsigned long long seed, unsigned int sub, const int* sub_dev,
                      void* stream);
int cdm_philox_uniform(float* out, long long n, float lo, float hi, unsigned long long seed, unsigned int sub,
                       const int* sub_dev, void* stream);
int cdm_philox_randint(int* out, int n, int lo, int hi, unsigned long long seed, unsigned int sub, const int* sub_dev,
                       void* stream);
int cdm_counter_add(int* ctr, int delta, void* stream);
/* torch.optim.Adam step (code/train_diffusion_condition.py:200,229) with torch's CPU roundings.
 * state (double[4], device) = {lr, step count, scratch, scratch}; bc (double[nbc][2], device) = host-evaluated
 * {1 - beta1**s, (1 - beta2**s)**0.5} for s = 1..nbc (steps past nbc reuse the last row, which must be {1, 1}).
 * grad_scale multiplies g (1/world for a summed data-parallel gradient). */
int cdm_adam(float* p, const float* g, float* m, float* v, long long n, double* state, const double* bc, int nbc,
             double beta1, double beta2, double eps, float grad_scale, void* stream);
/* weight repacking (+ eval-mode BatchNorm folding) */
/* kc = 0: K order tap-major (k = tap*C + ci); kc = 16: channel-chunk-major (k = ((ci/16)*9 + tap)*16 + ci%16),
 * the order cdm_conv3x3_fwd(kc = 16) consumes (wdg is chunked over Cout).  ConvTranspose packing: */
int cdm_pack_conv3x3(const float* W, const float* b, int Cin, int Cout, const float* gamma, const float* beta,
                     const float* rm, const float* rv, float eps, float* wpk, float* bpk, float* wdg, int kc,
                     void* stream);
int cdm_pack_convT(const float* W, int Cin, int Cout, int KK, float* wt, float* wtT, void* stream);
int cdm_transpose(const float* in, int R, int C, float* out, void* stream);
/* batched: in [batch][R][C] -> out [batch][C][R] (64x64 LDS tiles) */
int cdm_transpose_batched(const float* in, int batch, int R, int C, float* out, void* stream);

/* up0 on large maps (ContextUnet.py:26-27, ConvTranspose2d(C, C, k, k) on the 1x1 to_vec map, KK = k*k), VALU fp32
 * kernels over the weights in the reference layout W[ci][co][KK] (no repack): forward y[n][KK][C] (NHWC) =
 * bias + x[n][:] W (any B >= 1, one read of W per 16 samples); weight gradient dW[ci][co][KK] = x^T dy with
 * dy [B][KK][C] (NHWC), B <= 16 (assigns).  C % 16 == 0, C <= 512, KK % 64 == 0 (weight gradient: KK % 256 == 0). */
int cdm_up0_fwd(const float* x, int B, int C, const float* W, int KK, const float* bias, float* y, void* stream);
int cdm_up0_wgrad(const float* x, int B, int C, const float* dy, int KK, float* dW, void* stream);
/* input gradient dx[n][ci] = sum_k dyT[n][k] W[ci][k] over k = (co, ij), dyT = dy transposed per sample to [B][C][KK]
 * (B <= 16, C % 64 == 0): per-K-range partials slab [cdm_up0_dgrad_splits(C, KK)][B][C], folded by cdm_slab_reduce */
int cdm_up0_dgrad(const float* dyT, int B, int C, const float* W, int KK, float* slab, void* stream);
int cdm_up0_dgrad_splits(int C, int KK);

#ifdef __cplusplus
}
#endif
#endif /* CDM_HIP_H */
