// CAMELS map preprocessing on the device: code/train_diffusion_condition.py:137-144
// (== code/train_diffusion.py:106-113), in the dtype of the maps file (fp32):
//     mn = min(x); if mn <= 0: x = x - mn + 1e-8;  x = x / max(x);  x = log10(x);
//     x = (x - min(x)) / (max(x) - min(x));  F.interpolate(x[:, None], (64, 64), mode="bilinear")
// Every step is a monotone map of the raw values, so every later min / max is the image of the raw min / max:
// one min/max reduction over the raw maps (order-independent atomics -> deterministic), then one fused pass
// that normalises the (up to) 4 source pixels of each output pixel and interpolates them with torch's
// bilinear weights (align_corners=False, no antialias).  The raw maps are read once.
#include "cdm_common.h"

namespace cdm {

// float <-> order-preserving unsigned key
static __device__ __forceinline__ unsigned fkey(float f) {
    const unsigned b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
static __device__ __forceinline__ float fval(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ void minmax_init_kernel(unsigned* keys) {
    keys[0] = 0xffffffffu;   // running min key
    keys[1] = 0u;            // running max key
}

__global__ void minmax_kernel(const float* __restrict__ x, long long n, unsigned* keys) {
    unsigned kmin = 0xffffffffu, kmax = 0u;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned k = fkey(x[i]);
        kmin = min(kmin, k); kmax = max(kmax, k);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kmin = min(kmin, (unsigned)__shfl_xor((int)kmin, o, 64));
        kmax = max(kmax, (unsigned)__shfl_xor((int)kmax, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&keys[0], kmin);
        atomicMax(&keys[1], kmax);
    }
}

__global__ void minmax_finalize_kernel(const unsigned* keys, float* out) {
    out[0] = fval(keys[0]);
    out[1] = fval(keys[1]);
}

// one output pixel per thread: dst[n][oy][ox] from src[n][S][S]
__global__ void camels_maps_kernel(const float* __restrict__ src, int N, int S, int O, const float* __restrict__ mm,
                                   float* __restrict__ dst) {
    const float mn = mm[0], mx = mm[1];
    const bool shift = mn <= 0.f;
    // the images of the raw extremes under shift / scale / log10 (monotone)
    const float tmax = shift ? (mx - mn) + 1e-8f : mx;
    const float tmin = shift ? (mn - mn) + 1e-8f : mn;
    const float umin = log10f(tmin / tmax), umax = log10f(tmax / tmax);
    const float den = umax - umin;
    const float scale = (float)S / (float)O;
    const long long total = (long long)N * O * O;
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long long)gridDim.x * blockDim.x) {
        const int n = (int)(q / (O * O)), rem = (int)(q - (long long)n * O * O), oy = rem / O, ox = rem - oy * O;
        // torch area_pixel_compute_source_index (align_corners=False, linear): max(scale*(o+0.5)-0.5, 0)
        const float hr = fmaxf(scale * (oy + 0.5f) - 0.5f, 0.f), wr = fmaxf(scale * (ox + 0.5f) - 0.5f, 0.f);
        const int h1 = (int)hr, w1 = (int)wr;
        const int hp = h1 < S - 1 ? 1 : 0, wp = w1 < S - 1 ? 1 : 0;
        const float l1h = hr - h1, l0h = 1.f - l1h, l1w = wr - w1, l0w = 1.f - l1w;
        const float* s = src + (long long)n * S * S;
        auto norm = [&](int y, int x) {
            float v = s[(long long)y * S + x];
            if (shift) v = (v - mn) + 1e-8f;
            v = log10f(v / tmax);
            return (v - umin) / den;
        };
        const float v00 = norm(h1, w1), v01 = norm(h1, w1 + wp), v10 = norm(h1 + hp, w1), v11 = norm(h1 + hp, w1 + wp);
        dst[q] = l0h * (l0w * v00 + l1w * v01) + l1h * (l0w * v10 + l1w * v11);
    }
}

}  // namespace cdm

using namespace cdm;

static inline hipStream_t SD(void* s) { return reinterpret_cast<hipStream_t>(s); }

CDM_API int cdm_minmax_f32(const float* x, long long n, unsigned* keys, float* out, void* stream) {
    if (n <= 0) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(minmax_init_kernel, dim3(1), dim3(1), 0, SD(stream), keys);
    long long blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(minmax_kernel, dim3((unsigned)blocks), dim3(256), 0, SD(stream), x, n, keys);
    hipLaunchKernelGGL(minmax_finalize_kernel, dim3(1), dim3(1), 0, SD(stream), keys, out);
    return cdm_status();
}

CDM_API int cdm_camels_maps(const float* src, int N, int S, int O, const float* minmax, float* dst, void* stream) {
    if (N < 0 || S < 1 || O < 1) return (int)hipErrorInvalidValue;
    if (N == 0) return 0;
    long long blocks = ((long long)N * O * O + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(camels_maps_kernel, dim3((unsigned)blocks), dim3(256), 0, SD(stream), src, N, S, O, minmax, dst);
    return cdm_status();
}
