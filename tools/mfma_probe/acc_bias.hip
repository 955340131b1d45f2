// Accumulation bias of v_mfma_f32_32x32x16_f16 and what folding partial sums in fp32 VALU does to it.
// One wave per 32x32 output tile, C = A B with K = 2304 (a 256-channel 3x3 conv's reduction, 144 MFMAs of K = 16), fp16-
// exact operands so the only error is the fp32 accumulation.  Modes:
//   G = 0   the shipped form: every MFMA accumulates into the running C
//   G > 0   every G MFMAs go into zeroed partial accumulators, folded into C by v_add_f32 (round-to-nearest-even);
//           G = 27 is the h3 forward conv's 16-channel chunk (9 taps x 3 products), G = 1 folds after every MFMA
// Errors against the fp64 product on the host: mean / rms (0 for unbiased rounding), mean / mean|C|, relative L2.
//   hipcc --offload-arch=gfx950 -O3 acc_bias.hip -o acc_bias && ./acc_bias
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int K = 2304, NB = 512, M = 32 * NB;

// A: M x K row-major fp16; Bt: 32 x K (B transposed) fp16; C: M x 32 fp32
__global__ __launch_bounds__(64) void acc_probe(const _Float16* A, const _Float16* Bt, float* C, int G) {
    const int lane = threadIdx.x, b = blockIdx.x, kh = lane >> 5;
    const _Float16* pa = A + (long long)(32 * b + (lane & 31)) * K + 8 * kh;
    const _Float16* pb = Bt + (long long)(lane & 31) * K + 8 * kh;
    f32x16 c = {}, part = {};
    for (int s = 0; s < K / 16; ++s) {
        const f16x8 a = *reinterpret_cast<const f16x8*>(pa + 16 * s);
        const f16x8 v = *reinterpret_cast<const f16x8*>(pb + 16 * s);
        if (G == 0) {
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, v, c, 0, 0, 0);
        } else {
            part = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, v, part, 0, 0, 0);
            if ((s + 1) % G == 0 || s + 1 == K / 16) {
#pragma unroll
                for (int r = 0; r < 16; ++r) { c[r] += part[r]; part[r] = 0.f; }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) C[(long long)(32 * b + (r & 3) + 8 * (r >> 2) + 4 * kh) * 32 + (lane & 31)] = c[r];
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> uni(0.f, 1.f);
    std::normal_distribution<float> nrm(0.f, 1.f);
    std::vector<_Float16> A((size_t)M * K), Bt((size_t)32 * K);
    std::vector<double> ref((size_t)M * 32);
    std::vector<float> C((size_t)M * 32);
    _Float16 *dA, *dB;
    float* dC;
    CK(hipMalloc(&dA, A.size() * 2)); CK(hipMalloc(&dB, Bt.size() * 2)); CK(hipMalloc(&dC, C.size() * 4));
    for (int signs = 0; signs < 2; ++signs) {
        for (auto& v : A) v = (_Float16)(signs ? nrm(rng) : uni(rng));
        for (auto& v : Bt) v = (_Float16)uni(rng);
        for (int i = 0; i < M; ++i)
            for (int j = 0; j < 32; ++j) {
                double s = 0.0;
                const _Float16* a = &A[(size_t)i * K];
                const _Float16* b = &Bt[(size_t)j * K];
                for (int k = 0; k < K; ++k) s += (double)(float)a[k] * (double)(float)b[k];
                ref[(size_t)i * 32 + j] = s;
            }
        CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, Bt.data(), Bt.size() * 2, hipMemcpyHostToDevice));
        for (int G : {0, 1, 3, 9, 27, 48}) {
            hipLaunchKernelGGL(acc_probe, dim3(NB), dim3(64), 0, 0, dA, dB, dC, G);
            CK(hipGetLastError());
            CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
            double se = 0, se2 = 0, sr2 = 0, sac = 0;
            long long neg = 0;
            for (size_t i = 0; i < C.size(); ++i) {
                const double e = (double)C[i] - ref[i];
                se += e; se2 += e * e; sr2 += ref[i] * ref[i]; sac += std::fabs(ref[i]); neg += e < 0;
            }
            const double n = (double)C.size();
            printf("{\"operands\": \"%s\", \"fold_every\": %d, \"mean_over_rms\": %.5f, \"mean_over_meanabsC\": %.4e, "
                   "\"rel_l2\": %.4e, \"frac_negative\": %.4f}\n",
                   signs ? "fp16-exact, A of both signs" : "fp16-exact, positive", G, se / n / std::sqrt(se2 / n),
                   se / n / (sac / n), std::sqrt(se2 / sr2), neg / n);
        }
    }
    CK(hipFree(dA)); CK(hipFree(dB)); CK(hipFree(dC));
    return 0;
}
