// Shared definitions for the CDNA4 (gfx950) ContextUnet DDPM kernels.
// Layout convention: every activation is NHWC fp32; a tensor view is (ptr, N, H, W, C, ldc) where
// element (n,h,w,c) lives at ptr[((n*H + h)*W + w)*ldc + c].  ldc > C addresses a channel slice of
// a wider buffer, which is how the reference's torch.cat calls (diffusion_utilities.py:96,
// ContextUnet.py:59) are eliminated: producers write straight into their slice.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CDM_API extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) float f32x2;

static __device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

static __device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
static __device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// ---- activation element types (C4 mixed precision stores the fused Conv -> BN -> ReLU chain's y and g as bf16) ----
// Act<T>::Raw is what a 4-channel piece occupies in registers between its load and its use (loads stay raw so the
// conversion does not force a wait at the load site); to4() widens it (bf16 -> fp32 is exact); round() is the value a
// store of v keeps.
template <class T> struct Act;
// raw buffer resource over [base, base + 2^31 - 16): a load at byte offset BUF_OOB or beyond returns zeros (the range
// check of a stride-0 buffer), which turns a masked / padded load into an unconditional one with a selected offset
constexpr unsigned BUF_OOB = 0x80000000u;
static __device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7FFFFFF0, 0x00020000);
}
template <> struct Act<float> {
    typedef float4 Raw;
    static __device__ __forceinline__ Raw load4(const void* p) { return *reinterpret_cast<const float4*>(p); }
    static __device__ __forceinline__ Raw bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
        return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
    }
    static __device__ __forceinline__ float4 to4(const Raw& r) { return r; }
    static __device__ __forceinline__ Raw zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
    static __device__ __forceinline__ float round(float v) { return v; }
    static __device__ __forceinline__ void store(float* p, float v) { *p = v; }
    static __device__ __forceinline__ float load(const float* p) { return *p; }
};
template <> struct Act<__bf16> {
    typedef uint2 Raw;
    static __device__ __forceinline__ Raw load4(const void* p) { return *reinterpret_cast<const uint2*>(p); }
    static __device__ __forceinline__ Raw bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        const u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
        return make_uint2(v.x, v.y);
    }
    static __device__ __forceinline__ float4 to4(const Raw& r) {
        return make_float4(__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u), __uint_as_float(r.y << 16),
                           __uint_as_float(r.y & 0xffff0000u));
    }
    static __device__ __forceinline__ Raw zero() { return make_uint2(0u, 0u); }
    static __device__ __forceinline__ float round(float v) { return (float)(__bf16)v; }
    static __device__ __forceinline__ void store(__bf16* p, float v) { *p = (__bf16)v; }
    static __device__ __forceinline__ float load(const __bf16* p) { return (float)*p; }
};

static __device__ __forceinline__ float f4get(const float4& v, int j) {
    return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// ReLU with torch's NaN semantics (torch.relu(nan) = nan; fmaxf would return 0 and hide a diverged step from the
// trainer's non-finite-loss guard): IEEE 754-2019 maximum, gfx950's v_maximum3_f32 — one VALU instruction instead of
// a compare + select (-0 maps to +0, the only difference from x < 0 ? 0 : x, value-equal)
static __device__ __forceinline__ float relu_f(float x) { return __builtin_elementwise_maximum(x, 0.f); }

// float <-> int key with the same order (signed int compare): atomicMax / atomicMin of floats on an int slot
static __device__ __forceinline__ int fkey(float f) { const int i = __float_as_int(f); return i >= 0 ? i : i ^ 0x7FFFFFFF; }
static __device__ __forceinline__ float fkey_inv(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

// exact (erf) GELU, as torch.nn.GELU() default (diffusion_utilities.py:130, ContextUnet.py:17)
static __device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// GELU evaluated in fp64 (rounded once by the caller): the per-step embeddings / to_vec (csrc/misc.hip)
static __device__ __forceinline__ double gelu_d(double x) { return 0.5 * x * (1.0 + erf(x * 0.70710678118654752440)); }
static __device__ __forceinline__ float gelu_grad_f(float x) {
    const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
    return cdf + x * pdf;
}

static inline int cdm_status() { return (int)hipGetLastError(); }

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

static __device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// *out = max(*out, block max of m) for non-negative m (atomic max on the float's bits).  Every thread of
// the block must call it (it synchronises the block).  Producers use it to hand the h3 convolutions the
// max|.| of the tensor they write (csrc/gemm_f32.hip, NT_H3) without a separate pass over it.
static __device__ __forceinline__ void block_amax_commit(float m, float* out) {
    __shared__ float red[16];
    m = wave_max(m);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) red[w] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)((blockDim.x + 63) >> 6); ++i) m = fmaxf(m, red[i]);
        // *out only grows, so a block whose max does not exceed a value read from it has nothing to add: the atomic
        // is skipped (a stale read only costs an unneeded atomic).  With one atomic per block on one address, the
        // C_in = 1 forward's 16 384 blocks took 198 us against 94 us for the same kernel with no max requested.
        const unsigned cur = __hip_atomic_load(reinterpret_cast<unsigned*>(out), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        if (__float_as_uint(m) > cur) atomicMax(reinterpret_cast<unsigned*>(out), __float_as_uint(m));
    }
}

// BatchNorm (+ReLU) backward of one element.  norm_apply_bwd_kernel and the fused conv staging
// (gemm_f32.hip, PreBnBwd) both use this one expression, so the fused and unfused paths produce
// bit-identical dy:   z_pre = y s + t,  xhat = (y - mean) invstd,  dy = A (z_pre > 0 ? g : 0) + B + Cc xhat
static __device__ __forceinline__ float bn_bwd_elem(float g, float y, float s, float t, float mean, float invstd,
                                                    float a, float b, float cc) {
    const float zp = fmaf(y, s, t);
    const float xh = (y - mean) * invstd;
    return fmaf(cc, xh, fmaf(a, zp > 0.f ? g : 0.f, b));
}

// XCD-aware block order: consecutive hardware block ids go round-robin over the 8 XCDs (each with its own L2);
// this returns a logical index such that XCD x owns one contiguous range of logical blocks, so neighbouring work
// items (e.g. image bands sharing halo rows) run on one XCD and meet in its L2.  A bijection on [0, gridDim.x).
static __device__ __forceinline__ int xcd_logical_block() {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
}
