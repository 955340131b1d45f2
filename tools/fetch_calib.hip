// Calibration of rocprofv3 FETCH_SIZE against known byte counts in the access patterns of the conv kernels
// (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of the bytes of a wide coalesced streaming read; other widths are
// uncalibrated).  Each pattern reads a [1 M px][128 ch] fp32 tensor (537 MB, > the 256 MB Infinity Cache) exactly
// once; a 1 GiB write between launches evicts it from L2 and the Infinity Cache.
//   0 wide     : 16 B per lane, consecutive lanes consecutive (1 KiB per wave instruction)
//   1 halo     : the LDS-halo conv's staging: 4 lanes per pixel read 64 B (16 channels) of its 512-B row, the 8
//                channel chunks of a pixel in 8 passes (chunk-major, as the conv's K loop), 256-pixel tiles
//   2 halo6    : as 1, plus the conv's halo rows: each 4-row tile also reads the row above and below (6/4 = 1.5x the
//                bytes of pattern 1 requested; the excess is what L2 does or does not absorb)
//   3 rowfull  : the weight gradient's staging: 32 lanes per pixel read its whole 512-B row
//
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fc -o fc -- tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int C = 128, W = 64, H = 64, N = 256;
constexpr long long PIX = (long long)N * H * W;

__global__ __launch_bounds__(512) void wide(const float4* __restrict__ x, long long n4, float* out) {
    float s = 0.f;
    for (long long i = blockIdx.x * 512ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 512) {
        const float4 v = x[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

// one block per 256-pixel tile (4 image rows); HALO: rows h0-1 .. h0+4 (66 columns incl. padding skipped)
template <bool HALO>
__global__ __launch_bounds__(512) void halo(const float* __restrict__ x, float* out) {
    // XCD-contiguous tiles (as the conv's remap): blocks b and b + 8 share an XCD and hold consecutive tiles
    const int tile = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3), img = tile / (H / 4), h0 = (tile % (H / 4)) * 4;
    const int r0 = HALO ? -1 : 0, r1 = HALO ? 5 : 4;
    float s = 0.f;
    for (int cc = 0; cc < C / 16; ++cc) {
        for (int q = threadIdx.x; q < (r1 - r0) * W * 4; q += 512) {
            const int p = q >> 2, c4 = q & 3, hr = h0 + r0 + p / W, w = p % W;
            if ((unsigned)hr >= (unsigned)H) continue;
            const float4 v = *reinterpret_cast<const float4*>(x + ((long long)(img * H + hr) * W + w) * C + cc * 16 + c4 * 4);
            s += v.x + v.y + v.z + v.w;
        }
        __syncthreads();
    }
    if (s == 1234.5f) out[0] = s;
}

__global__ __launch_bounds__(512) void rowfull(const float* __restrict__ x, float* out) {
    const long long p0 = (long long)blockIdx.x * 256;
    float s = 0.f;
    for (int k = 0; k < 256; k += 16) {
        const long long p = p0 + k + (threadIdx.x >> 5);
        const float4 v = *reinterpret_cast<const float4*>(x + p * C + (threadIdx.x & 31) * 4);
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

__global__ void scrub(float4* p, long long n4) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) p[i] = make_float4(1, 2, 3, 4);
}

int main() {
    float *x, *out, *junk;
    const long long bytes = PIX * C * 4, jbytes = 1ll << 30;
    if (hipMalloc(&x, bytes) || hipMalloc(&out, 64) || hipMalloc(&junk, jbytes)) return 1;
    hipMemset(x, 0, bytes);
    const int tiles = (int)(PIX / 256);
    for (int rep = 0; rep < 2; ++rep) {
        for (int pat = 0; pat < 4; ++pat) {
            hipLaunchKernelGGL(scrub, dim3(4096), dim3(256), 0, 0, (float4*)junk, jbytes / 16);
            if (pat == 0) hipLaunchKernelGGL(wide, dim3(4096), dim3(512), 0, 0, (const float4*)x, bytes / 16, out);
            if (pat == 1) hipLaunchKernelGGL(halo<false>, dim3(tiles), dim3(512), 0, 0, x, out);
            if (pat == 2) hipLaunchKernelGGL(halo<true>, dim3(tiles), dim3(512), 0, 0, x, out);
            if (pat == 3) hipLaunchKernelGGL(rowfull, dim3(tiles), dim3(512), 0, 0, x, out);
        }
    }
    if (hipDeviceSynchronize()) return 2;
    printf("fetch_calib: tensor %lld bytes; patterns wide / halo / halo6 (requests 1.5x) / rowfull\n", bytes);
    return 0;
}
