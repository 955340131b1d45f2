// Sample statistics of generated maps: power spectrum P(k) of 2-D / 3-D boxes and per-map PDF.
//
// Reference: power_spectrum  code/diffusion_utilities.py:302-368 (np.fft.fftn norm="ortho", bins round(k/dk))
//            calculate_power_spectrum_2d  code/sample_power_spectra.py:112-165 (np.fft.fft2, log bins)
//            compare_distributions  code/train_diffusion.py:196-215 (np.histogram(..., density=True))
// All arithmetic is fp64, like numpy's.  The DFT is evaluated directly (two passes of N-term complex dot
// products against an exact twiddle table, sincospi) — O(N^3) per map, ~0.3 MFLOP at N = 64, so a batch of
// 256 maps is a few microseconds of fp64 VALU; no FFT library.  The radial binning sums each bin's power in
// the order the caller's index list gives (CSR), so the reference's flat-order sums are reproduced exactly.
#include "cdm_common.h"

#include <type_traits>

namespace cdm {

// pass 1: T[b][x][v] = sum_y img[b][x][y] * w^(v*y),  w = exp(-2 pi i / N); one block per (b, x), thread v
__global__ void dft_rows_kernel(const float* __restrict__ img, int N, double2* __restrict__ T) {
    extern __shared__ double sm[];
    double* row = sm;            // [N]
    double* cs = sm + N;         // [N] cos(2 pi k / N)
    double* sn = sm + 2 * N;     // [N] sin(2 pi k / N)
    const long long base = (long long)blockIdx.x * N;          // (b*N + x) * N
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        row[k] = (double)img[base + k];
        double s, c;
        sincospi(2.0 * k / N, &s, &c);
        cs[k] = c; sn[k] = s;
    }
    __syncthreads();
    for (int v = threadIdx.x; v < N; v += blockDim.x) {
        double re = 0.0, im = 0.0;
        int idx = 0;
        for (int y = 0; y < N; ++y) {             // w^(v y): angle index (v*y) mod N, accumulated
            re = fma(row[y], cs[idx], re);
            im = fma(-row[y], sn[idx], im);
            idx += v; if (idx >= N) idx -= N;
        }
        T[base + v] = make_double2(re, im);
    }
}

// pass 2: F[b][u][v] = sum_x T[b][x][v] * w^(u*x);  power = |F|^2 * scale.  One block per (b, u), thread v.
__global__ void dft_cols_power_kernel(const double2* __restrict__ T, int N, double scale, double* __restrict__ power) {
    extern __shared__ double sm[];
    double* cs = sm;
    double* sn = sm + N;
    const int b = blockIdx.x / N, u = blockIdx.x - b * N;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        double s, c;
        sincospi(2.0 * k / N, &s, &c);
        cs[k] = c; sn[k] = s;
    }
    __syncthreads();
    const double2* Tb = T + (long long)b * N * N;
    for (int v = threadIdx.x; v < N; v += blockDim.x) {
        double re = 0.0, im = 0.0;
        int idx = 0;
        for (int x = 0; x < N; ++x) {
            const double2 t = Tb[(long long)x * N + v];
            const double c = cs[idx], s = sn[idx];          // (t.re + i t.im)(c - i s)
            re = fma(t.x, c, fma(t.y, s, re));
            im = fma(t.y, c, fma(-t.x, s, im));
            idx += u; if (idx >= N) idx -= N;
        }
        power[((long long)b * N + u) * N + v] = (re * re + im * im) * scale;
    }
}

// Any-rank boxes (power_spectrum's 3-D branch and non-square 2-D boxes, diffusion_utilities.py:316-336): the DFT
// along one axis of a complex fp64 array viewed as [outer][n][inner], one thread per output element (o, k, i):
// out[o][k][i] = sum_j in[o][j][i] w^(k j).  Successive calls over every axis give fftn.  The input of the first pass is
// the real box (re only: fp32, or fp64 as numpy's fftn of a float64 array computes); the last pass may write
// |F|^2 * scale instead of F.  RealT = void: complex fp64 input (the later passes).
template <typename RealT, bool POWER_OUT>
__global__ __launch_bounds__(256) void dft_axis_kernel(const void* __restrict__ in_, int outer, int n, long long inner,
                                                       double scale, void* __restrict__ out_) {
    extern __shared__ double tw[];            // [2n]: cos, sin of 2 pi k / n
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        double s, c;
        sincospi(2.0 * k / n, &s, &c);
        tw[k] = c; tw[n + k] = s;
    }
    __syncthreads();
    const long long total = (long long)outer * n * inner;
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const long long i = e % inner;
    const long long ok = e / inner;
    const int k = (int)(ok % n);
    const long long o = ok / n;
    const long long base = o * n * inner + i;
    double re = 0.0, im = 0.0;
    int idx = 0;
    for (int j = 0; j < n; ++j) {             // w^(k j): angle index (k*j) mod n, accumulated
        const double c = tw[idx], sn = tw[n + idx];
        if constexpr (!std::is_void_v<RealT>) {
            const double v = (double)static_cast<const RealT*>(in_)[base + (long long)j * inner];
            re = fma(v, c, re);
            im = fma(-v, sn, im);
        } else {                              // (a + i b)(c - i s)
            const double2 v = static_cast<const double2*>(in_)[base + (long long)j * inner];
            re = fma(v.x, c, fma(v.y, sn, re));
            im = fma(v.y, c, fma(-v.x, sn, im));
        }
        idx += k; if (idx >= n) idx -= n;
    }
    if constexpr (POWER_OUT)
        static_cast<double*>(out_)[e] = (re * re + im * im) * scale;
    else
        static_cast<double2*>(out_)[e] = make_double2(re, im);
}

// out[b][k] = sum over i in idx[off[k] .. off[k+1]) (in that order) of power[b][idx[i]]; one block per map
__global__ void bin_sum_kernel(const double* __restrict__ power, long long NN, const int* __restrict__ off,
                               const int* __restrict__ idx, int nbins, double* __restrict__ out) {
    const double* p = power + (long long)blockIdx.x * NN;
    for (int k = threadIdx.x; k < nbins; k += blockDim.x) {
        double s = 0.0;
        for (int i = off[k]; i < off[k + 1]; ++i) s += p[idx[i]];
        out[(long long)blockIdx.x * nbins + k] = s;
    }
}

// numpy.histogram(x[b], edges, density=True): counts with edges[i] <= v < edges[i+1] (the last bin closed),
// values outside [edges[0], edges[nb]] dropped; density = n / diff(edges) / sum(n).  One block per map.
__global__ void histogram_density_kernel(const float* __restrict__ x, long long P, const double* __restrict__ edges,
                                         int nb, double* __restrict__ out) {
    extern __shared__ unsigned char smraw[];
    double* e = reinterpret_cast<double*>(smraw);                         // [nb + 1]
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(e + nb + 1);   // [nb]
    for (int i = threadIdx.x; i <= nb; i += blockDim.x) e[i] = edges[i];
    for (int i = threadIdx.x; i < nb; i += blockDim.x) cnt[i] = 0ull;
    __syncthreads();
    const float* xb = x + (long long)blockIdx.x * P;
    const double lo = e[0], hi = e[nb];
    for (long long q = threadIdx.x; q < P; q += blockDim.x) {
        const double v = (double)xb[q];
        if (!(v >= lo && v <= hi)) continue;
        int bin;
        if (v == hi) {
            bin = nb - 1;
        } else {                                   // largest i with e[i] <= v  (searchsorted side='right' - 1)
            int a = 0, c = nb;                     // e[a] <= v < e[c]
            while (c - a > 1) {
                const int m = (a + c) >> 1;
                if (e[m] <= v) a = m; else c = m;
            }
            bin = a;
        }
        atomicAdd(&cnt[bin], 1ull);
    }
    __syncthreads();
    __shared__ unsigned long long total;
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < nb; ++i) t += cnt[i];
        total = t;
    }
    __syncthreads();
    const double tot = (double)total;
    for (int i = threadIdx.x; i < nb; i += blockDim.x)
        out[(long long)blockIdx.x * nb + i] = (double)cnt[i] / (e[i + 1] - e[i]) / tot;
}

}  // namespace cdm

using namespace cdm;

static inline hipStream_t SS(void* s) { return reinterpret_cast<hipStream_t>(s); }

// |DFT2(img[b])|^2 * scale for B maps of N x N fp32 (row-major); T = scratch of B*N*N complex doubles
CDM_API int cdm_dft2_power(const float* img, int B, int N, double scale, void* T, double* power, void* stream) {
    if (B < 0 || N < 1 || N > 4096) return (int)hipErrorInvalidValue;
    if (B == 0) return 0;
    const int th = N < 256 ? ((N + 63) / 64) * 64 : 256;
    hipLaunchKernelGGL(dft_rows_kernel, dim3(B * N), dim3(th), 3 * N * sizeof(double), SS(stream), img, N,
                       reinterpret_cast<double2*>(T));
    hipLaunchKernelGGL(dft_cols_power_kernel, dim3(B * N), dim3(th), 2 * N * sizeof(double), SS(stream),
                       reinterpret_cast<const double2*>(T), N, scale, power);
    return cdm_status();
}

// |fftn(box[b])|^2 * scale for B row-major boxes of rank 1..3 with extents dims[0..rank); T0 / T1 = scratch of
// B * prod(dims) complex doubles each (ping-pong between the axis passes)
template <typename RealT>
static int dftn_power(const RealT* box, int B, int rank, const int* dims, double scale, void* T0, void* T1,
                      double* power, void* stream) {
    if (B < 0 || rank < 1 || rank > 3) return (int)hipErrorInvalidValue;
    long long n_all = 1;
    for (int a = 0; a < rank; ++a) {
        if (dims[a] < 1 || dims[a] > 4096) return (int)hipErrorInvalidValue;
        n_all *= dims[a];
    }
    if (B == 0) return 0;
    const long long total = (long long)B * n_all;
    const dim3 grid((unsigned)((total + 255) / 256));
    long long inner = n_all;
    const void* src = box;
    void* bufs[2] = {T0, T1};
    for (int a = 0; a < rank; ++a) {          // axis a: [B * prod(dims[:a])][dims[a]][prod(dims[a+1:])]
        const int n = dims[a];
        inner /= n;
        const int outer = (int)(total / ((long long)n * inner));
        const size_t sm = 2 * (size_t)n * sizeof(double);
        const bool first = a == 0, last = a == rank - 1;
        void* dst = last ? (void*)power : bufs[a & 1];
        if (first && last)
            hipLaunchKernelGGL((dft_axis_kernel<RealT, true>), grid, dim3(256), sm, SS(stream), src, outer, n, inner,
                               scale, dst);
        else if (first)
            hipLaunchKernelGGL((dft_axis_kernel<RealT, false>), grid, dim3(256), sm, SS(stream), src, outer, n, inner,
                               scale, dst);
        else if (last)
            hipLaunchKernelGGL((dft_axis_kernel<void, true>), grid, dim3(256), sm, SS(stream), src, outer, n, inner,
                               scale, dst);
        else
            hipLaunchKernelGGL((dft_axis_kernel<void, false>), grid, dim3(256), sm, SS(stream), src, outer, n, inner,
                               scale, dst);
        int e = cdm_status(); if (e) return e;
        src = dst;
    }
    return 0;
}

CDM_API int cdm_dftn_power(const float* box, int B, int rank, const int* dims, double scale, void* T0, void* T1,
                           double* power, void* stream) {
    return dftn_power(box, B, rank, dims, scale, T0, T1, power, stream);
}

// the same for fp64 boxes (np.fft.fftn of a float64 array: no fp32 rounding of the input)
CDM_API int cdm_dftn_power_f64(const double* box, int B, int rank, const int* dims, double scale, void* T0, void* T1,
                               double* power, void* stream) {
    return dftn_power(box, B, rank, dims, scale, T0, T1, power, stream);
}

CDM_API int cdm_bin_sum(const double* power, int B, long long NN, const int* off, const int* idx, int nbins,
                        double* out, void* stream) {
    if (B < 0 || nbins < 1) return (int)hipErrorInvalidValue;
    if (B == 0) return 0;
    hipLaunchKernelGGL(bin_sum_kernel, dim3(B), dim3(256), 0, SS(stream), power, NN, off, idx, nbins, out);
    return cdm_status();
}

CDM_API int cdm_histogram_density(const float* x, int B, long long P, const double* edges, int nbins, double* out,
                                  void* stream) {
    if (B < 0 || nbins < 1 || nbins > 4000) return (int)hipErrorInvalidValue;
    if (B == 0) return 0;
    const size_t sm = (size_t)(nbins + 1) * sizeof(double) + (size_t)nbins * sizeof(unsigned long long);
    hipLaunchKernelGGL(histogram_density_kernel, dim3(B), dim3(256), sm, SS(stream), x, P, edges, nbins, out);
    return cdm_status();
}
