// Streaming-write ceiling on MI355X for the C_in = 1 / C_out = 1 conv writers (537 MB of fp32 output per launch at
// bs = 256, 64x64, 128 channels; larger than the 256 MB Infinity Cache):
//   0 store      : float4 stores, grid-stride, consecutive lanes consecutive 16 B (1 KiB per wave instruction)
//   1 store_nt   : the same with nontemporal stores
//   2 copy       : float4 copy of a 537 MB tensor (read + write)
//   3 read       : float4 read of the same tensor (sum kept live)
//   4 rowblock   : the row kernels' write pattern: block b writes its own 32 KiB (one 64-pixel x 128-channel row),
//                  8 iterations of 4 KiB, no compute
//   5 rowblock_w : 4 plus the row kernels' prologue: 36 weight loads per lane (stride 9, as conv_cout1_dgrad_row)
//
//   hipcc --offload-arch=gfx950 -O3 tools/write_bw.hip -o tools/write_bw && tools/write_bw
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr long long BYTES = 256ll * 64 * 64 * 128 * 4;

__global__ __launch_bounds__(256) void store(float4* p, long long n4, float v) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256)
        p[i] = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
}
__global__ __launch_bounds__(256) void store_nt(float4* p, long long n4, float v) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        float* q = reinterpret_cast<float*>(p + i);
        __builtin_nontemporal_store(v, q);
        __builtin_nontemporal_store(v + 1.f, q + 1);
        __builtin_nontemporal_store(v + 2.f, q + 2);
        __builtin_nontemporal_store(v + 3.f, q + 3);
    }
}
__global__ __launch_bounds__(256) void copy(const float4* __restrict__ a, float4* __restrict__ b, long long n4) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void read(const float4* __restrict__ a, long long n4, float* out) {
    float s = 0.f;
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

__global__ __launch_bounds__(256) void rowblock(float4* p, float v) {
    float4* q = p + (long long)blockIdx.x * 2048;
#pragma unroll 1
    for (int it = 0; it < 8; ++it) q[it * 256 + threadIdx.x] = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
}
__global__ __launch_bounds__(256) void rowblock_w(float4* p, const float* __restrict__ w) {
    const int c4 = (threadIdx.x & 31) * 4;
    float wr[9][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) wr[tap][j] = w[(c4 + j) * 9 + tap];
    float4* q = p + (long long)blockIdx.x * 2048;
#pragma unroll 1
    for (int it = 0; it < 8; ++it) {
        float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = fmaf((float)(it + tap), wr[tap][j], o[j]);
        q[it * 256 + threadIdx.x] = make_float4(o[0], o[1], o[2], o[3]);
    }
}

int main() {
    float4 *a, *b;
    float* out;
    if (hipMalloc(&a, BYTES) || hipMalloc(&b, BYTES) || hipMalloc(&out, 64)) return 1;
    hipMemset(a, 0, BYTES);
    hipMemset(b, 0, BYTES);
    const long long n4 = BYTES / 16;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[6] = {"store", "store_nt", "copy", "read", "rowblock", "rowblock_w"};
    for (int grid : {4096, 16384}) {
        for (int pat = 0; pat < 6; ++pat) {
            float best = 1e30f;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(e0, 0);
                if (pat == 0) hipLaunchKernelGGL(store, dim3(grid), dim3(256), 0, 0, b, n4, (float)rep);
                if (pat == 1) hipLaunchKernelGGL(store_nt, dim3(grid), dim3(256), 0, 0, b, n4, (float)rep);
                if (pat == 2) hipLaunchKernelGGL(copy, dim3(grid), dim3(256), 0, 0, a, b, n4);
                if (pat == 3) hipLaunchKernelGGL(read, dim3(grid), dim3(256), 0, 0, a, n4, out);
                if (pat == 4) hipLaunchKernelGGL(rowblock, dim3(BYTES / 32768), dim3(256), 0, 0, b, (float)rep);
                if (pat == 5) hipLaunchKernelGGL(rowblock_w, dim3(BYTES / 32768), dim3(256), 0, 0, b, (const float*)a);
                hipEventRecord(e1, 0);
                if (hipEventSynchronize(e1)) return 2;
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep > 0 && ms < best) best = ms;
            }
            const double bytes = pat == 2 ? 2.0 * BYTES : (double)BYTES;
            printf("%-9s grid %5d: %8.1f us  %.2f TB/s (bytes moved / time)\n", names[pat], grid, best * 1e3,
                   bytes / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
