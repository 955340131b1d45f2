// Microbenchmark: does the 16x16x32 f16 MFMA shape sustain more fp32-equivalent work than 32x32x16 in the conv's
// inner-loop pattern (fragments re-read from swizzled LDS images every tap, 2 waves per SIMD, random operands)?
//   hipcc --offload-arch=gfx950 -O3 mfma_shape.hip -o mfma_shape && ./mfma_shape
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int LDS_BYTES = 96 * 1024;

__device__ __forceinline__ int swz(int row, int half) { return row * 32 + ((half ^ ((row >> 3) & 1)) << 4); }

// 32x32x16: per "tap" 2x2 tiles x 3 products (hh, hl, lh), fragments: A 2 tiles x 2 terms, B 2 x 2
__global__ __launch_bounds__(512, 1) void k32(const uint4* src, float* out, int iters) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    for (int i = threadIdx.x; i < LDS_BYTES / 16; i += 512) reinterpret_cast<uint4*>(sm)[i] = src[(blockIdx.x * 97 + i) % 65536];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f32x16 acc[2][2] = {};
    const int kh = lane >> 5;
    for (int it = 0; it < iters; ++it) {
        const int base = ((it * 7 + wave * 3) & 15) * 2048;
        f16x8 a[2][2], b[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                a[i][t] = *reinterpret_cast<const f16x8*>(sm + base + t * 16384 + swz(32 * i + (lane & 31), kh));
                b[i][t] = *reinterpret_cast<const f16x8*>(sm + 49152 + base + t * 8192 + swz(32 * i + (lane & 31), kh));
            }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][0], b[j][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][0], b[j][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][1], b[j][0], acc[i][j], 0, 0, 0);
            }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) s += acc[i][j][r];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

// 16x16x32: per "tap" 4x4 tiles; 1 MFMA [hi|lo] x [hi|hi] (hh + lh) per tile, plus every second tap one paired
// [hi_t|hi_u] x [lo_t|lo_u] (hl of two taps) per tile: 1.5 MFMA-16x16x32 per tile per tap = the same MACs as k32
__global__ __launch_bounds__(512, 1) void k16(const uint4* src, float* out, int iters) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    for (int i = threadIdx.x; i < LDS_BYTES / 16; i += 512) reinterpret_cast<uint4*>(sm)[i] = src[(blockIdx.x * 97 + i) % 65536];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f32x4 acc[4][4] = {};
    const int kg = lane >> 4, r16 = lane & 15;
    for (int it = 0; it < iters; it += 2) {           // two taps per iteration
#pragma unroll
        for (int tap = 0; tap < 2; ++tap) {
            const int base = (((it + tap) * 7 + wave * 3) & 15) * 2048;
            f16x8 a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a[i] = *reinterpret_cast<const f16x8*>(sm + base + (kg >> 1) * 16384 + swz(16 * i + r16, kg & 1));
                b[i] = *reinterpret_cast<const f16x8*>(sm + 49152 + base + swz(16 * i + r16, kg & 1));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        const int b0 = ((it * 7 + wave * 3) & 15) * 2048, b1 = (((it + 1) * 7 + wave * 3) & 15) * 2048;
        f16x8 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a[i] = *reinterpret_cast<const f16x8*>(sm + ((kg >> 1) ? b1 : b0) + swz(16 * i + r16, kg & 1));
            b[i] = *reinterpret_cast<const f16x8*>(sm + 49152 + ((kg >> 1) ? b1 : b0) + 8192 + swz(16 * i + r16, kg & 1));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) s += acc[i][j][r];
    out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
    const int blocks = 1024, iters = 4000;
    std::vector<uint16_t> h(65536 * 8);
    std::mt19937 rng(1);
    for (auto& v : h) { _Float16 f = (_Float16)((rng() % 20001) / 10000.0f - 1.0f); v = *reinterpret_cast<uint16_t*>(&f); }
    uint4* d; float* o;
    hipMalloc(&d, h.size() * 2); hipMalloc(&o, blocks * 512 * 4);
    hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipFuncSetAttribute((const void*)k32, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute((const void*)k16, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    // MACs per tap per wave: 32x32x16 x 12 = 196608 (both kernels)
    const double flop = 2.0 * 196608.0 * iters * 8 * blocks;
    for (int rep = 0; rep < 3; ++rep) {
        for (int k = 0; k < 2; ++k) {
            for (int w = 0; w < 2; ++w) {
                if (k == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(512), LDS_BYTES, 0, d, o, iters);
                else hipLaunchKernelGGL(k16, dim3(blocks), dim3(512), LDS_BYTES, 0, d, o, iters);
            }
            hipEventRecord(e0);
            const int n = 5;
            for (int w = 0; w < n; ++w) {
                if (k == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(512), LDS_BYTES, 0, d, o, iters);
                else hipLaunchKernelGGL(k16, dim3(blocks), dim3(512), LDS_BYTES, 0, d, o, iters);
            }
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); ms /= n;
            printf("%s: %.3f ms  %.0f TF/s f16-MFMA work\n", k == 0 ? "32x32x16" : "16x16x32", ms, flop / ms / 1e9);
        }
    }
    return 0;
}
