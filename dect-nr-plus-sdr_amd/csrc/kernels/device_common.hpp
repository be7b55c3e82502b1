// Device helpers shared by the DECT NR+ kernels: complex arithmetic, LDS Stockham FFT
// (radix 4/2/3, autosort, one workgroup per transform), block reductions.
#pragma once

#include "experiments.hpp"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace dnrp::dev {

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // a * conj(b)
    return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float cnorm(float2 a) { return a.x * a.x + a.y * a.y; }

// exp(j*phi) for a double phase: exact reduction to revolutions in [-1/2, 1/2] in double, then the
// hardware sin/cos (v_sin_f32 / v_cos_f32 take revolutions; ~1e-6 absolute error). No slow
// large-argument path, so no register-hungry Payne-Hanek code next to the hot loops.
__device__ __forceinline__ float2 phasor(double phi) {
    const double rev = phi * 0.15915494309189533577;  // 1 / (2 pi)
    const float r = static_cast<float>(rev - rint(rev));
    return make_float2(__builtin_amdgcn_cosf(r), __builtin_amdgcn_sinf(r));
}

// Copy x[q0 + i], i in [0, n), into dst[i] (zero outside [0, S)) with U loads in flight per thread
// (tid / nt: this thread's index in the copying group, a wavefront or the workgroup). A plain
// strided loop issues one load and waits for it every iteration.
template <int U, class T, class F>
__device__ __forceinline__ void stage_gen(T* dst, uint32_t n, uint32_t tid, uint32_t nt, F&& load) {
    for (uint32_t base = 0; base < n; base += nt * U) {
        T v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t i = base + tid + j * nt;
            v[j] = i < n ? load(i) : T{};
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t i = base + tid + j * nt;
            if (i < n) dst[i] = v[j];
        }
    }
}

template <int U>
__device__ __forceinline__ void stage_span(float2* dst, const float2* __restrict__ x, int64_t q0, uint32_t n, int64_t S,
                                           uint32_t tid, uint32_t nt) {
    stage_gen<U>(dst, n, tid, nt, [&](uint32_t i) {
        const int64_t q = q0 + i;
        return (q >= 0 && q < S) ? x[q] : make_float2(0.f, 0.f);
    });
}

// same with a lower bound: x[q] valid for q in [lo, S) (RX windows whose packet starts before the
// window, fine_peak < 0: zero history there, never a read before the window row)
template <int U>
__device__ __forceinline__ void stage_span_lo(float2* dst, const float2* __restrict__ x, int64_t q0, uint32_t n,
                                              int64_t lo, int64_t S, uint32_t tid, uint32_t nt) {
    stage_gen<U>(dst, n, tid, nt, [&](uint32_t i) {
        const int64_t q = q0 + i;
        return (q >= lo && q < S) ? x[q] : make_float2(0.f, 0.f);
    });
}

// stage_span_lo for one wavefront whose whole span [q0, q0 + n] lies inside the valid range: two
// samples per lane and load (16 B, 8-B aligned: the unaligned dwordx4 form, nontemporal), half the load
// instructions of the float2 form and 16-B LDS writes; x[q0 + n] may be read, never written
template <int U>
__device__ __forceinline__ void stage_span_x2(float2* dst, const float2* __restrict__ x, int64_t q0, uint32_t n,
                                              uint32_t lane) {
    for (uint32_t base = 0; base < n; base += 128 * U) {
        float4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t i = base + 2 * lane + 128 * j;
            v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            // nontemporal: bypasses only the L1, the samples are not re-read by this wave
            typedef float f4u __attribute__((ext_vector_type(4), aligned(8)));
            if (i < n) {
                const f4u t = __builtin_nontemporal_load(reinterpret_cast<const f4u*>(x + q0 + i));
                v[j] = make_float4(t.x, t.y, t.z, t.w);
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t i = base + 2 * lane + 128 * j;
            if (i + 1 < n) *reinterpret_cast<float4*>(dst + i) = v[j];
            else if (i < n) dst[i] = make_float2(v[j].x, v[j].y);
        }
    }
}

template <int U, class T>
__device__ __forceinline__ void stage_copy(T* dst, const T* __restrict__ src, uint32_t n, uint32_t tid, uint32_t nt) {
    stage_gen<U>(dst, n, tid, nt, [&](uint32_t i) { return src[i]; });
}

// FFT plan passed by value: radix sequence (each 2, 3 or 4), product = N
struct fft_plan {
    uint32_t N;
    uint32_t nr;
    uint32_t radix[16];
};

// R-point DFT in registers, SIGN = -1 forward, +1 inverse (unnormalised)
template <int SIGN>
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = csub(a1, a3);
    // t3 * (SIGN * j)
    const float2 t3j = SIGN < 0 ? make_float2(t3.y, -t3.x) : make_float2(-t3.y, t3.x);
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3j);
    a3 = csub(t1, t3j);
}

// Stockham autosort passes on LDS ping-pong buffers; tw[j] = exp(-2*pi*i*j/N) (forward table).
// nb transforms stored back to back (x[b*N .. b*N+N)) run in the same passes.
// Returns the buffer holding the result. Whole workgroup participates; ends with a barrier.
template <int SIGN>
__device__ float2* fft_lds(float2* x_, float2* y_, const float2* __restrict__ tw, const fft_plan& p, uint32_t nb = 1) {
    const uint32_t N = p.N;
    uint32_t Ns = 1;
    for (uint32_t s = 0; s < p.nr; ++s) {
        const uint32_t R = p.radix[s];
        const uint32_t NR = N / R;
        const uint32_t tstep = N / (Ns * R);
        for (uint32_t jb = threadIdx.x; jb < nb * NR; jb += blockDim.x) {
            const uint32_t b = jb / NR, j = jb - b * NR;
            const float2* x = x_ + b * N;
            float2* y = y_ + b * N;
            const uint32_t k = j % Ns;
            const uint32_t od = (j / Ns) * Ns * R + k;
            if (R == 4) {
                float2 a0 = x[j], a1 = x[j + NR], a2 = x[j + 2 * NR], a3 = x[j + 3 * NR];
                if (Ns > 1) {
                    const uint32_t e = k * tstep;
                    float2 w1 = tw[e % N], w2 = tw[(2 * e) % N], w3 = tw[(3 * e) % N];
                    if (SIGN > 0) {
                        w1 = cconj(w1);
                        w2 = cconj(w2);
                        w3 = cconj(w3);
                    }
                    a1 = cmul(a1, w1);
                    a2 = cmul(a2, w2);
                    a3 = cmul(a3, w3);
                }
                dft4<SIGN>(a0, a1, a2, a3);
                y[od] = a0;
                y[od + Ns] = a1;
                y[od + 2 * Ns] = a2;
                y[od + 3 * Ns] = a3;
            } else if (R == 2) {
                float2 a0 = x[j], a1 = x[j + NR];
                if (Ns > 1) {
                    float2 w1 = tw[(k * tstep) % N];
                    if (SIGN > 0) w1 = cconj(w1);
                    a1 = cmul(a1, w1);
                }
                y[od] = cadd(a0, a1);
                y[od + Ns] = csub(a0, a1);
            } else {  // R == 3
                float2 a0 = x[j], a1 = x[j + NR], a2 = x[j + 2 * NR];
                if (Ns > 1) {
                    const uint32_t e = k * tstep;
                    float2 w1 = tw[e % N], w2 = tw[(2 * e) % N];
                    if (SIGN > 0) {
                        w1 = cconj(w1);
                        w2 = cconj(w2);
                    }
                    a1 = cmul(a1, w1);
                    a2 = cmul(a2, w2);
                }
                // W3 = exp(SIGN * 2 pi i / 3)
                const float c3 = -0.5f, s3 = SIGN * 0.86602540378443864676f;
                const float2 s = cadd(a1, a2), d = csub(a1, a2);
                const float2 m = make_float2(a0.x + c3 * s.x, a0.y + c3 * s.y);
                const float2 jd = make_float2(-s3 * d.y, s3 * d.x);  // s3 * j * d
                y[od] = cadd(a0, s);
                y[od + Ns] = cadd(m, jd);
                y[od + 2 * Ns] = csub(m, jd);
            }
        }
        __syncthreads();
        float2* t = x_;
        x_ = y_;
        y_ = t;
        Ns *= R;
    }
    return x_;
}

// Power-of-two sizes (every u>=2 / b in {1,2,4,8,16} FFT of tx_rx.hpp:67-69): radix-4 Stockham
// passes with shift/mask index arithmetic (no integer division) + one radix-2 pass for odd log2.
// tw: forward twiddle table of N entries (LDS or global), tw[j] = exp(-2 pi i j / N).
template <int SIGN>
__device__ float2* fft_pow2(float2* x_, float2* y_, const float2* tw, uint32_t log2N, uint32_t nb = 1) {
    const uint32_t N = 1u << log2N;
    uint32_t s = 0;  // log2(Ns)
    for (; s + 2 <= log2N; s += 2) {
        const uint32_t NR = N >> 2, kmask = (1u << s) - 1u, tsh = log2N - s - 2;
        for (uint32_t jb = threadIdx.x; jb < nb * NR; jb += blockDim.x) {
            const uint32_t j = jb & (NR - 1u), bo = (jb >> (log2N - 2)) << log2N;
            const float2* x = x_ + bo;
            float2* y = y_ + bo;
            const uint32_t k = j & kmask;
            const uint32_t od = ((j - k) << 2) + k;
            float2 a0 = x[j], a1 = x[j + NR], a2 = x[j + 2 * NR], a3 = x[j + 3 * NR];
            if (s) {
                const uint32_t e = k << tsh;
                float2 w1 = tw[e], w2 = tw[2 * e], w3 = tw[3 * e];
                if (SIGN > 0) {
                    w1 = cconj(w1);
                    w2 = cconj(w2);
                    w3 = cconj(w3);
                }
                a1 = cmul(a1, w1);
                a2 = cmul(a2, w2);
                a3 = cmul(a3, w3);
            }
            dft4<SIGN>(a0, a1, a2, a3);
            y[od] = a0;
            y[od + (1u << s)] = a1;
            y[od + (2u << s)] = a2;
            y[od + (3u << s)] = a3;
        }
        __syncthreads();
        float2* t = x_;
        x_ = y_;
        y_ = t;
    }
    if (s < log2N) {  // final radix-2 pass, Ns = N/2
        const uint32_t NR = N >> 1, kmask = (1u << s) - 1u;
        for (uint32_t jb = threadIdx.x; jb < nb * NR; jb += blockDim.x) {
            const uint32_t j = jb & (NR - 1u), bo = (jb >> (log2N - 1)) << log2N;
            const float2* x = x_ + bo;
            float2* y = y_ + bo;
            const uint32_t k = j & kmask;
            const uint32_t od = ((j - k) << 1) + k;
            const float2 a0 = x[j];
            float2 a1 = x[j + NR];
            float2 w = tw[k];
            if (SIGN > 0) w = cconj(w);
            a1 = cmul(a1, w);
            y[od] = cadd(a0, a1);
            y[od + (1u << s)] = csub(a0, a1);
        }
        __syncthreads();
        float2* t = x_;
        x_ = y_;
        y_ = t;
    }
    return x_;
}

// dispatch: power-of-two fast path, generic mixed radix otherwise
template <int SIGN>
__device__ __forceinline__ float2* fft_any(float2* x, float2* y, const float2* tw, const fft_plan& p, uint32_t nb = 1) {
    if ((p.N & (p.N - 1)) == 0) return fft_pow2<SIGN>(x, y, tw, 31u - __clz(p.N), nb);
    return fft_lds<SIGN>(x, y, tw, p, nb);
}

// Batched FFT whose last pass hands its outputs to store(b, n, v) (transform b, output index n)
// instead of writing the ping-pong buffer, e.g. straight into a cyclic-prefixed time-domain layout.
// The input must be in x; pass i reads x when i is even, so with fft_num_passes() = P the last pass
// reads x iff P is odd: the caller places the input so that the store target is never read.
__host__ __device__ inline uint32_t fft_num_passes(const fft_plan& p) {
    if ((p.N & (p.N - 1)) == 0) {
        uint32_t lg = 0;
        while ((1u << lg) < p.N) ++lg;
        return (lg + 1) / 2;
    }
    return p.nr;
}

template <int SIGN, class Store>
__device__ void fft_store(float2* x_, float2* y_, const float2* tw, const fft_plan& p, uint32_t nb, Store store) {
    const uint32_t N = p.N;
    if ((N & (N - 1)) == 0) {
        const uint32_t log2N = 31u - __clz(N);
        uint32_t s = 0;
        for (; s + 2 <= log2N; s += 2) {
            const bool last = (s + 2 == log2N);
            const uint32_t NR = N >> 2, kmask = (1u << s) - 1u, tsh = log2N - s - 2;
            for (uint32_t jb = threadIdx.x; jb < nb * NR; jb += blockDim.x) {
                const uint32_t j = jb & (NR - 1u), b = jb >> (log2N - 2), bo = b << log2N;
                const float2* x = x_ + bo;
                const uint32_t k = j & kmask;
                const uint32_t od = ((j - k) << 2) + k;
                float2 a0 = x[j], a1 = x[j + NR], a2 = x[j + 2 * NR], a3 = x[j + 3 * NR];
                if (s) {
                    const uint32_t e = k << tsh;
                    float2 w1 = tw[e], w2 = tw[2 * e], w3 = tw[3 * e];
                    if (SIGN > 0) {
                        w1 = cconj(w1);
                        w2 = cconj(w2);
                        w3 = cconj(w3);
                    }
                    a1 = cmul(a1, w1);
                    a2 = cmul(a2, w2);
                    a3 = cmul(a3, w3);
                }
                dft4<SIGN>(a0, a1, a2, a3);
                if (last) {
                    store(b, od, a0);
                    store(b, od + (1u << s), a1);
                    store(b, od + (2u << s), a2);
                    store(b, od + (3u << s), a3);
                } else {
                    float2* y = y_ + bo;
                    y[od] = a0;
                    y[od + (1u << s)] = a1;
                    y[od + (2u << s)] = a2;
                    y[od + (3u << s)] = a3;
                }
            }
            __syncthreads();
            float2* t = x_;
            x_ = y_;
            y_ = t;
        }
        if (s < log2N) {  // final radix-2 pass
            const uint32_t NR = N >> 1, kmask = (1u << s) - 1u;
            for (uint32_t jb = threadIdx.x; jb < nb * NR; jb += blockDim.x) {
                const uint32_t j = jb & (NR - 1u), b = jb >> (log2N - 1), bo = b << log2N;
                const float2* x = x_ + bo;
                const uint32_t k = j & kmask;
                const uint32_t od = ((j - k) << 1) + k;
                const float2 a0 = x[j];
                float2 w = tw[k];
                if (SIGN > 0) w = cconj(w);
                const float2 a1 = cmul(x[j + NR], w);
                store(b, od, cadd(a0, a1));
                store(b, od + (1u << s), csub(a0, a1));
            }
            __syncthreads();
        }
        return;
    }
    uint32_t Ns = 1;
    for (uint32_t s = 0; s < p.nr; ++s) {
        const bool last = (s + 1 == p.nr);
        const uint32_t R = p.radix[s];
        const uint32_t NR = N / R;
        const uint32_t tstep = N / (Ns * R);
        for (uint32_t jb = threadIdx.x; jb < nb * NR; jb += blockDim.x) {
            const uint32_t b = jb / NR, j = jb - b * NR;
            const float2* x = x_ + b * N;
            float2* y = y_ + b * N;
            const uint32_t k = j % Ns;
            const uint32_t od = (j / Ns) * Ns * R + k;
            float2 o[4];
            if (R == 4) {
                float2 a0 = x[j], a1 = x[j + NR], a2 = x[j + 2 * NR], a3 = x[j + 3 * NR];
                if (Ns > 1) {
                    const uint32_t e = k * tstep;
                    float2 w1 = tw[e % N], w2 = tw[(2 * e) % N], w3 = tw[(3 * e) % N];
                    if (SIGN > 0) {
                        w1 = cconj(w1);
                        w2 = cconj(w2);
                        w3 = cconj(w3);
                    }
                    a1 = cmul(a1, w1);
                    a2 = cmul(a2, w2);
                    a3 = cmul(a3, w3);
                }
                dft4<SIGN>(a0, a1, a2, a3);
                o[0] = a0;
                o[1] = a1;
                o[2] = a2;
                o[3] = a3;
            } else if (R == 2) {
                float2 a0 = x[j], a1 = x[j + NR];
                if (Ns > 1) {
                    float2 w1 = tw[(k * tstep) % N];
                    if (SIGN > 0) w1 = cconj(w1);
                    a1 = cmul(a1, w1);
                }
                o[0] = cadd(a0, a1);
                o[1] = csub(a0, a1);
            } else {
                float2 a0 = x[j], a1 = x[j + NR], a2 = x[j + 2 * NR];
                if (Ns > 1) {
                    const uint32_t e = k * tstep;
                    float2 w1 = tw[e % N], w2 = tw[(2 * e) % N];
                    if (SIGN > 0) {
                        w1 = cconj(w1);
                        w2 = cconj(w2);
                    }
                    a1 = cmul(a1, w1);
                    a2 = cmul(a2, w2);
                }
                const float c3 = -0.5f, s3 = SIGN * 0.86602540378443864676f;
                const float2 sm = cadd(a1, a2), d = csub(a1, a2);
                const float2 m = make_float2(a0.x + c3 * sm.x, a0.y + c3 * sm.y);
                const float2 jd = make_float2(-s3 * d.y, s3 * d.x);
                o[0] = cadd(a0, sm);
                o[1] = cadd(m, jd);
                o[2] = csub(m, jd);
            }
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) {
                if (r >= R) break;
                if (last)
                    store(b, od + r * Ns, o[r]);
                else
                    y[od + r * Ns] = o[r];
            }
        }
        __syncthreads();
        float2* t = x_;
        x_ = y_;
        y_ = t;
        Ns *= R;
    }
}

// ---------------------------------------------------------------------------------------------
// One-wavefront 1024-point FFT (N_b_DFT_os = 1024: u,b = 8,16 / 4,16 / ... at os 1).
// Lane t holds v[m] = x[t + 64 m] on entry and v[m] = X[t + 64 m] on exit. Stockham passes
// radix 16 (Ns = 1), radix 16 (Ns = 16) and radix 4 (Ns = 256, four butterflies per lane): the
// first pass starts from registers, two exchanges go through the wave's own LDS buffer xb
// (>= 1088 float2, index padded i + i/16: conflict-free b64 writes, <= 2-way reads), no workgroup
// barrier. tw: forward twiddles exp(-2 pi i j / 1024) (LDS or global).
constexpr uint32_t WFFT_XB = 1024 + 64;

// exchange slot of element i: padded i + i / 16 (default: conflict-free b64 writes of pass 1 and 2,
// 2-way ds_read_b64 conflicts in passes 2 and 3 -- slots 0 and 32 of a half-wave share a bank) or, with
// XS_WFFT_SWZ (experiments.hpp), i ^ ((i >> 4) & 15): conflict-free for all four exchange patterns, but the XOR makes
// the slot lane-dependent per instruction (address VALU instead of immediate offsets)
__device__ __forceinline__ uint32_t wfft_pad(uint32_t i) { return experiment(XS_WFFT_SWZ) ? (i ^ ((i >> 4) & 15u)) : i + (i >> 4); }

template <int SIGN>
__device__ __forceinline__ float2 wfft_tw(const float2* tw, uint32_t e) {
    const float2 w = tw[e];
    return SIGN > 0 ? cconj(w) : w;
}

// X[k1 + 4 k2] = sum_r x[r] W16^(r k), r = c + 4 a (decimation in time, twiddles W16^(c k1))
template <int SIGN>
__device__ __forceinline__ void dft16(float2 (&v)[16]) {
    constexpr float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f, R2 = 0.70710678118654752440f;
#pragma unroll
    for (int c = 0; c < 4; ++c) dft4<SIGN>(v[c], v[c + 4], v[c + 8], v[c + 12]);  // A[c][k1] at v[c + 4 k1]
    // W16^(c k1), SIGN-signed angle 2 pi c k1 / 16
    auto rot = [](float2 a, float cs, float sn) {  // a * (cs + SIGN*j*sn)
        const float s = SIGN * sn;
        return make_float2(a.x * cs - a.y * s, a.x * s + a.y * cs);
    };
    v[1 + 4 * 1] = rot(v[1 + 4 * 1], C1, S1);
    v[1 + 4 * 2] = rot(v[1 + 4 * 2], R2, R2);
    v[1 + 4 * 3] = rot(v[1 + 4 * 3], S1, C1);
    v[2 + 4 * 1] = rot(v[2 + 4 * 1], R2, R2);
    v[2 + 4 * 2] = rot(v[2 + 4 * 2], 0.f, 1.f);
    v[2 + 4 * 3] = rot(v[2 + 4 * 3], -R2, R2);
    v[3 + 4 * 1] = rot(v[3 + 4 * 1], S1, C1);
    v[3 + 4 * 2] = rot(v[3 + 4 * 2], -R2, R2);
    v[3 + 4 * 3] = rot(v[3 + 4 * 3], -C1, -S1);
    float2 o[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        float2 a0 = v[4 * k1], a1 = v[4 * k1 + 1], a2 = v[4 * k1 + 2], a3 = v[4 * k1 + 3];
        dft4<SIGN>(a0, a1, a2, a3);  // over c -> k2
        o[k1] = a0;
        o[k1 + 4] = a1;
        o[k1 + 8] = a2;
        o[k1 + 12] = a3;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = o[k];
}

// In-place radix-4 decimation-in-time FFT of N = 4^p points on one buffer: the input sits at base-4
// digit-reversed positions, pass s (quarter Q = 4^(s/2)) combines four Q-point transforms per
// butterfly with the twiddles W_N^(r k N/(4Q)) of fft_pow2's pass s, output in natural order. Every
// butterfly reads and writes its own four slots (no second buffer: half the LDS of fft_pow2).
// PAD: slot i at x[i + i / 32] (the stride-4 accesses of the first passes and the digit-reversed
// input writes on distinct banks: the caller allocates N + N / 32 slots and indexes through r4pad)
__device__ __forceinline__ uint32_t r4pad(uint32_t i) { return i + (i >> 5); }

template <int SIGN, bool PAD = false>
__device__ void fft_r4_inplace(float2* x_, const float2* tw, uint32_t log2N) {
    auto x = [&](uint32_t i) -> float2& { return x_[PAD ? r4pad(i) : i]; };
    const uint32_t NB = 1u << (log2N - 2);
    for (uint32_t s = 0; s < log2N; s += 2) {
        const uint32_t Q = 1u << s, tsh = log2N - s - 2;
        for (uint32_t j = threadIdx.x; j < NB; j += blockDim.x) {
            const uint32_t k = j & (Q - 1u), i0 = ((j >> s) << (s + 2)) + k;
            float2 a0 = x(i0), a1 = x(i0 + Q), a2 = x(i0 + 2 * Q), a3 = x(i0 + 3 * Q);
            if (s) {
                const uint32_t e = k << tsh;
                float2 w1 = tw[e], w2 = tw[2 * e], w3 = tw[3 * e];
                if (SIGN > 0) {
                    w1 = cconj(w1);
                    w2 = cconj(w2);
                    w3 = cconj(w3);
                }
                a1 = cmul(a1, w1);
                a2 = cmul(a2, w2);
                a3 = cmul(a3, w3);
            }
            dft4<SIGN>(a0, a1, a2, a3);
            x(i0) = a0;
            x(i0 + Q) = a1;
            x(i0 + 2 * Q) = a2;
            x(i0 + 3 * Q) = a3;
        }
        __syncthreads();
    }
}

// fft_r4_inplace<SIGN, true> for a compile-time size (sync_fine's 4096 points): the same butterflies
// and twiddles in the same order, so bit-identical results. The passes unrolled, so each butterfly's
// four padded slots are one base address plus immediate offsets (Q constant; for Q = 16 the second
// half of a 64-slot group lies one pad slot further), and two butterflies per thread and trip (j and
// j + nt) with both butterflies' slot and twiddle loads issued before either is computed: one memory
// latency per pass instead of two at NB = 2 nt. Twiddles through a buffer resource (32-bit offsets).
template <uint32_t S, uint32_t LOG2N, class F>
__device__ __forceinline__ void r4_passes(F& pass) {  // pass(integral_constant<S>) for S = 0, 2, .. < LOG2N
    if constexpr (S < LOG2N) {
        pass(std::integral_constant<uint32_t, S>{});
        r4_passes<S + 2, LOG2N>(pass);
    }
}

template <int SIGN, uint32_t LOG2N>
__device__ void fft_r4_inplace_ct(float2* x_, const float2* tw) {
    constexpr uint32_t NB = 1u << (LOG2N - 2);
    const uint32_t nt = blockDim.x;
    const __amdgpu_buffer_rsrc_t twr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(tw), 0, static_cast<int>((1u << LOG2N) * 8u), 0x00020000);
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    auto pass = [&](auto sc) {
        constexpr uint32_t s = decltype(sc)::value, Q = 1u << s, tsh = LOG2N - s - 2;
        static_assert(Q >= 32 || 4 * Q <= 32 || Q == 16, "pad offsets");
        // padded slot of i0 + r Q relative to r4pad(i0), i0 = 4 Q m + k with k < Q
        auto off = [](int r) -> uint32_t {
            if constexpr (Q >= 32) return r * Q + r * (Q / 32);
            else if constexpr (Q == 16) return r * Q + (r >= 2 ? 1u : 0u);
            else return r * Q;
        };
        for (uint32_t j0 = threadIdx.x; j0 < NB; j0 += 2 * nt) {
            const bool two = j0 + nt < NB;
            float2 a[2][4], w[2][3];
            float2* p[2];
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const uint32_t j = b && two ? j0 + nt : j0;
                const uint32_t k = j & (Q - 1u);
                p[b] = x_ + r4pad(((j >> s) << (s + 2)) + k);
#pragma unroll
                for (int r = 0; r < 4; ++r) a[b][r] = p[b][off(r)];
                if constexpr (s > 0) {
                    const uint32_t e8 = (k << tsh) * 8u;
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        const u2 v = __builtin_amdgcn_raw_buffer_load_b64(twr, (r + 1) * e8, 0, 0);
                        w[b][r] = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
                    }
                }
            }
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                if constexpr (s > 0) {
#pragma unroll
                    for (int r = 0; r < 3; ++r) a[b][r + 1] = cmul(a[b][r + 1], SIGN > 0 ? cconj(w[b][r]) : w[b][r]);
                }
                dft4<SIGN>(a[b][0], a[b][1], a[b][2], a[b][3]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) p[0][off(r)] = a[0][r];
            if (two) {
#pragma unroll
                for (int r = 0; r < 4; ++r) p[1][off(r)] = a[1][r];
            }
        }
        __syncthreads();
    };
    r4_passes<0, LOG2N>(pass);
}

// 8-point DFT in registers (natural order in and out): two 4-point DFTs of the even and odd inputs
// and the W8^m butterflies, W8 = exp(SIGN 2 pi i / 8)
template <int SIGN>
__device__ __forceinline__ void dft8(float2 (&a)[8]) {
    constexpr float R2 = 0.70710678118654752440f;
    float2 e0 = a[0], e1 = a[2], e2 = a[4], e3 = a[6], o0 = a[1], o1 = a[3], o2 = a[5], o3 = a[7];
    dft4<SIGN>(e0, e1, e2, e3);
    dft4<SIGN>(o0, o1, o2, o3);
    // W8^1 = (1 + SIGN j) / sqrt 2, W8^2 = SIGN j, W8^3 = (-1 + SIGN j) / sqrt 2
    const float2 w1 = SIGN < 0 ? make_float2(R2 * (o1.x + o1.y), R2 * (o1.y - o1.x)) : make_float2(R2 * (o1.x - o1.y), R2 * (o1.x + o1.y));
    const float2 w2 = SIGN < 0 ? make_float2(o2.y, -o2.x) : make_float2(-o2.y, o2.x);
    const float2 w3 = SIGN < 0 ? make_float2(R2 * (o3.y - o3.x), -R2 * (o3.x + o3.y)) : make_float2(-R2 * (o3.x + o3.y), R2 * (o3.x - o3.y));
    a[0] = cadd(e0, o0);
    a[4] = csub(e0, o0);
    a[1] = cadd(e1, w1);
    a[5] = csub(e1, w1);
    a[2] = cadd(e2, w2);
    a[6] = csub(e2, w2);
    a[3] = cadd(e3, w3);
    a[7] = csub(e3, w3);
}

// 4096-point in-place radix-8 decimation-in-time FFT by 512 threads (one butterfly per thread and
// pass, four passes instead of fft_r4_inplace_ct's six): the input at base-8 digit-reversed slots
// (rev8), output in natural order, slot i at x[r8pad(i)] (r8pad: the stride-8 butterfly reads, the
// stride-512 digit-reversed writes and the stride-64 / -512 groups on distinct bank pairs)
__device__ __forceinline__ uint32_t r8pad(uint32_t i) { return i + (i >> 3) + (i >> 9); }
__device__ __forceinline__ uint32_t rev8(uint32_t i) {  // 12 bits = 4 base-8 digits
    return ((i & 7u) << 9) | (((i >> 3) & 7u) << 6) | (((i >> 6) & 7u) << 3) | (i >> 9);
}
constexpr uint32_t R8_SLOTS = 4096 + 512 + 8;

template <int SIGN>
__device__ void fft_r8_4096(float2* x_, const float2* tw) {
    const uint32_t j = threadIdx.x;  // blockDim.x == 512 (caller)
    const __amdgpu_buffer_rsrc_t twr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(tw), 0, 4096 * 8, 0x00020000);
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    auto pass = [&](auto sc) {
        constexpr uint32_t s = decltype(sc)::value, Q = 1u << s, tsh = 12 - s - 3;
        const uint32_t k = j & (Q - 1u), i0 = ((j >> s) << (s + 3)) + k;
        float2 a[8], w[7];
#pragma unroll
        for (int r = 0; r < 8; ++r) a[r] = x_[r8pad(i0 + r * Q)];
        if constexpr (s > 0) {
            const uint32_t e8 = (k << tsh) * 8u;
#pragma unroll
            for (int r = 0; r < 7; ++r) {
                const u2 v = __builtin_amdgcn_raw_buffer_load_b64(twr, (r + 1) * e8, 0, 0);
                w[r] = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
            }
#pragma unroll
            for (int r = 0; r < 7; ++r) a[r + 1] = cmul(a[r + 1], SIGN > 0 ? cconj(w[r]) : w[r]);
        }
        dft8<SIGN>(a);
#pragma unroll
        for (int r = 0; r < 8; ++r) x_[r8pad(i0 + r * Q)] = a[r];
        __syncthreads();
    };
    pass(std::integral_constant<uint32_t, 0>{});
    pass(std::integral_constant<uint32_t, 3>{});
    pass(std::integral_constant<uint32_t, 6>{});
    pass(std::integral_constant<uint32_t, 9>{});
}

// base-4 digit reversal of the log2N / 2 digits of i (fft_r4_inplace's input position)
__device__ __forceinline__ uint32_t rev4(uint32_t i, uint32_t log2N) {
    const uint32_t b = __brev(i) >> (32 - log2N);
    return ((b & 0x55555555u) << 1) | ((b >> 1) & 0x55555555u);
}

template <int SIGN>
__device__ __forceinline__ void wave_fft1024(float2 (&v)[16], float2* xb, const float2* tw, uint32_t lane) {
    // pass 1: radix 16, Ns = 1, butterfly j = lane on x[j + 64 r] -> y[16 j + k]
    dft16<SIGN>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) xb[wfft_pad(16 * lane + k)] = v[k];
    __builtin_amdgcn_wave_barrier();
    // pass 2: radix 16, Ns = 16: reads y[j + 64 r], twiddle W256^(r kk), writes z[(j/16) 256 + kk + 16 k]
    const uint32_t kk = lane & 15u;
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = xb[wfft_pad(lane + 64 * r)];
#pragma unroll
    for (int r = 1; r < 16; ++r) v[r] = cmul(v[r], wfft_tw<SIGN>(tw, 4 * r * kk));
    dft16<SIGN>(v);
    __builtin_amdgcn_wave_barrier();
    const uint32_t zb = (lane >> 4) * 256 + kk;
#pragma unroll
    for (int k = 0; k < 16; ++k) xb[wfft_pad(zb + 16 * k)] = v[k];
    __builtin_amdgcn_wave_barrier();
    // pass 3: radix 4, Ns = 256: butterflies j = lane + 64 b read z[j + 256 r], twiddle W1024^(r j),
    // write X[j + 256 r] = X[lane + 64 (b + 4 r)] -> v[b + 4 r]
    float2 o[16];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t j = lane + 64 * b;
        float2 a0 = xb[wfft_pad(j)], a1 = xb[wfft_pad(j + 256)], a2 = xb[wfft_pad(j + 512)], a3 = xb[wfft_pad(j + 768)];
        a1 = cmul(a1, wfft_tw<SIGN>(tw, j));
        a2 = cmul(a2, wfft_tw<SIGN>(tw, 2 * j));
        a3 = cmul(a3, wfft_tw<SIGN>(tw, 3 * j));
        dft4<SIGN>(a0, a1, a2, a3);
        o[b] = a0;
        o[b + 4] = a1;
        o[b + 8] = a2;
        o[b + 12] = a3;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = o[m];
}

// Same transform with two twiddle loads per lane instead of 27: pass 2 needs W^(4 kk r), r = 1..15,
// = powers of one loaded W^(4 kk) (binary-power products, chain depth <= 4); pass 3 needs W^(j),
// W^(2j), W^(3j) for j = lane + 64 b, and W^(lane + 64 b) = W^lane * exp(SIGN i pi b / 8) with
// compile-time constants. Fewer live registers where the FFT sits inside a loop; results differ from
// wave_fft1024 by a few float ulps of the twiddles (~1e-7 relative).
// w1 = W^(4 (lane & 15)), wl = W^lane (SIGN-signed): the caller may keep them in registers
template <int SIGN>
__device__ __forceinline__ void wave_fft1024_rt(float2 (&v)[16], float2* xb, float2 w1, float2 wl, uint32_t lane) {
    constexpr float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f, R2 = 0.70710678118654752440f;
    dft16<SIGN>(v);
#pragma unroll
    for (int k = 0; k < 16; ++k) xb[wfft_pad(16 * lane + k)] = v[k];
    __builtin_amdgcn_wave_barrier();
    const uint32_t kk = lane & 15u;
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = xb[wfft_pad(lane + 64 * r)];
    {
        float2 w[16];
        w[1] = w1;
        w[2] = cmul(w1, w1);
        w[4] = cmul(w[2], w[2]);
        w[8] = cmul(w[4], w[4]);
        w[3] = cmul(w[2], w1);
        w[5] = cmul(w[4], w1);
        w[6] = cmul(w[4], w[2]);
        w[7] = cmul(w[4], w[3]);
        w[9] = cmul(w[8], w1);
        w[10] = cmul(w[8], w[2]);
        w[11] = cmul(w[8], w[3]);
        w[12] = cmul(w[8], w[4]);
        w[13] = cmul(w[8], w[5]);
        w[14] = cmul(w[8], w[6]);
        w[15] = cmul(w[8], w[7]);
#pragma unroll
        for (int r = 1; r < 16; ++r) v[r] = cmul(v[r], w[r]);
    }
    dft16<SIGN>(v);
    __builtin_amdgcn_wave_barrier();
    const uint32_t zb = (lane >> 4) * 256 + kk;
#pragma unroll
    for (int k = 0; k < 16; ++k) xb[wfft_pad(zb + 16 * k)] = v[k];
    __builtin_amdgcn_wave_barrier();
    float2 o[16];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t j = lane + 64 * b;
        const float cb = b == 0 ? 1.f : b == 1 ? C1 : b == 2 ? R2 : S1;
        const float sb = b == 0 ? 0.f : b == 1 ? S1 : b == 2 ? R2 : C1;
        const float2 e1 = b == 0 ? wl : cmul(wl, make_float2(cb, SIGN * sb));
        const float2 e2 = cmul(e1, e1), e3 = cmul(e2, e1);
        float2 a0 = xb[wfft_pad(j)], a1 = xb[wfft_pad(j + 256)], a2 = xb[wfft_pad(j + 512)], a3 = xb[wfft_pad(j + 768)];
        a1 = cmul(a1, e1);
        a2 = cmul(a2, e2);
        a3 = cmul(a3, e3);
        dft4<SIGN>(a0, a1, a2, a3);
        o[b] = a0;
        o[b + 4] = a1;
        o[b + 8] = a2;
        o[b + 12] = a3;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = o[m];
}

template <int SIGN>
__device__ __forceinline__ void wave_fft1024_rt(float2 (&v)[16], float2* xb, const float2* tw, uint32_t lane) {
    wave_fft1024_rt<SIGN>(v, xb, wfft_tw<SIGN>(tw, 4 * (lane & 15u)), wfft_tw<SIGN>(tw, lane), lane);
}

// block-wide sum of a double, result valid in all threads (blockDim.x multiple of 64, <= 1024)
// three block sums with one set of barriers (each value summed exactly as block_sum sums it);
// red holds >= 3 * waves doubles
__device__ __forceinline__ void block_sum3(double& a, double& b, double& c, double* red) {
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
        c += __shfl_xor(c, o);
    }
    const uint32_t w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        red[w] = a;
        red[nw + w] = b;
        red[2 * nw + w] = c;
    }
    __syncthreads();
    double sa = 0.0, sb = 0.0, sc = 0.0;
    for (uint32_t i = 0; i < nw; ++i) {
        sa += red[i];
        sb += red[nw + i];
        sc += red[2 * nw + i];
    }
    __syncthreads();
    a = sa;
    b = sb;
    c = sc;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const uint32_t w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (uint32_t i = 0; i < nw; ++i) s += red[i];
    __syncthreads();
    return s;
}

}  // namespace dnrp::dev
