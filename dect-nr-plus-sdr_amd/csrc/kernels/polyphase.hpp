// Register-blocked rational polyphase resampler (resampler_t, lib/src/phy/resample/resampler.cpp:330-454).
//
// Output m of an L/M resampler with group delay D reads inputs p(m) - d, d = 0..HL, weighted by
// h[ph(m) + d*L], where t = D + m*M, p = t / L, ph = t % L. For an "aligned" output m_b with
// ph(m_b) = 0 the L outputs m_b .. m_b+L-1 have the compile-time phases (k*M) % L and newest inputs
// p(m_b) + (k*M) / L, so one thread computes a whole block of L outputs from the
// W = HL + 1 + ((L-1)*M)/L window inputs starting at p(m_b) - HL.
//
// The loop runs input-major: window input i (one LDS read) updates all L accumulators with the
// taps g[i][k] = h[ph_k + (HL + o_k - i) * L] (zero outside output k's FIR span), a [W][LP] table
// in LDS that every lane reads at the same address (16-B broadcasts, LP = 4*ceil(L/4)). Live state
// is L accumulators plus one input and one tap row, the loop is not unrolled across inputs, and
// nothing can be hoisted into registers: small VGPR footprint whatever the filter length.
// Aligned outputs are m_b = m_star + L*q, whose newest input is p_star + M*q.
#pragma once

#include "device_common.hpp"

namespace dnrp::dev {

typedef float v4f __attribute__((ext_vector_type(4)));

template <int L, int M, int HL>
struct pp_block {
    static constexpr int W = HL + 1 + ((L - 1) * M) / L;  // window inputs per block
    static constexpr int LP = (L + 3) / 4 * 4;             // padded tap row length

    // xw: LDS window (xw[i] = input p_b - HL + i); g: LDS taps [W][LP]; y[k] = output m_b + k
    __device__ static __forceinline__ void run(const float2* xw, const float* g, float2 (&y)[L]) {
#pragma unroll
        for (int k = 0; k < L; ++k) y[k] = make_float2(0.f, 0.f);
        const v4f* rows = reinterpret_cast<const v4f*>(g);
#pragma unroll 2
        for (int i = 0; i < W; ++i) {
            const float2 xv = xw[i];
            v4f t[LP / 4];
#pragma unroll
            for (int c = 0; c < LP / 4; ++c) t[c] = rows[i * (LP / 4) + c];
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const float tv = t[k / 4][k % 4];
                y[k].x = fmaf(xv.x, tv, y[k].x);
                y[k].y = fmaf(xv.y, tv, y[k].y);
            }
        }
    }

    // B blocks per lane sharing every tap-row read: block b's window starts at xw[b].
    // LDS bytes per FMA fall from (16 LP/4 + 8) / (2L) to (16 LP/4 + 8 B) / (2 L B).
    template <int B>
    __device__ static __forceinline__ void run_multi(const float2* const (&xw)[B], const float* g, float2 (&y)[B][L]) {
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int k = 0; k < L; ++k) y[b][k] = make_float2(0.f, 0.f);
        const v4f* rows = reinterpret_cast<const v4f*>(g);
#pragma unroll 2
        for (int i = 0; i < W; ++i) {
            v4f t[LP / 4];
#pragma unroll
            for (int c = 0; c < LP / 4; ++c) t[c] = rows[i * (LP / 4) + c];
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const float2 xv = xw[b][i];
#pragma unroll
                for (int k = 0; k < L; ++k) {
                    const float tv = t[k / 4][k % 4];
                    y[b][k].x = fmaf(xv.x, tv, y[b][k].x);
                    y[b][k].y = fmaf(xv.y, tv, y[b][k].y);
                }
            }
        }
    }
};

// Output-major form of the same block: the W window inputs are read from LDS into registers once
// (16-B reads where the window start is even), then every output k accumulates exactly its HL + 1
// taps h[ph_k + d L] — compile-time indices, no zero taps (the input-major table carries
// W * L - (HL + 1) * L zeros: 32 % of the FMAs for 9/10, 26 % for 10/9). The taps are read
// through the constant address space: uniform scalar loads into SGPRs, no LDS traffic at all.
// Summation order d = HL .. 0 (oldest input first) matches pp_block::run bit for bit.
typedef const __attribute__((address_space(4))) float* ctap_ptr;

template <int L, int M, int HL>
struct pp_direct {
    static constexpr int W = HL + 1 + ((L - 1) * M) / L;

    template <bool EVEN>
    __device__ static __forceinline__ void load(const float2* xw, float2 (&x)[W]) {
        if constexpr (EVEN) {
            const float4* x4 = reinterpret_cast<const float4*>(xw);
#pragma unroll
            for (int i = 0; i < W / 2; ++i) {
                const float4 v = x4[i];
                x[2 * i] = make_float2(v.x, v.y);
                x[2 * i + 1] = make_float2(v.z, v.w);
            }
            if constexpr (W & 1) x[W - 1] = xw[W - 1];
        } else {
#pragma unroll
            for (int i = 0; i < W; ++i) x[i] = xw[i];
        }
    }

    __device__ static __forceinline__ void run(const float2 (&x)[W], ctap_ptr h, float2 (&y)[L]) {
#pragma unroll
        for (int k = 0; k < L; ++k) y[k] = make_float2(0.f, 0.f);
        // tap-row order: the L taps of delay d are contiguous (h[ph_k + d L], ph_k a permutation of
        // 0..L-1), one short scalar load each, so only ~L taps are live in SGPRs at a time
        uint64_t hp = reinterpret_cast<uint64_t>(h);
#pragma unroll
        for (int d = HL; d >= 0; --d) {
            // opaque tap pointer per row: stops the compiler from hoisting all (HL + 1) L tap loads
            // ahead of the FMAs (more SGPRs than a wave has -> spills through VGPR lanes)
            if ((HL - d) % 2 == 0) asm volatile("" : "+s"(hp));
            const ctap_ptr hr = reinterpret_cast<ctap_ptr>(hp);
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const int o = (k * M) / L, ph = (k * M) % L;
                const float t = hr[ph + d * L];
                y[k].x = fmaf(x[HL + o - d].x, t, y[k].x);
                y[k].y = fmaf(x[HL + o - d].y, t, y[k].y);
            }
        }
    }
};

}  // namespace dnrp::dev

namespace dnrp::dev {

// pp_direct with the taps as compile-time constants (TP: a generated taps_* struct, build/gen/
// taps_gen.hpp): every tap is an immediate materialised into an SGPR next to its FMA, zero taps
// (the filter's padding to a multiple of L) vanish, and no SGPRs or LDS hold a tap table. The host
// checks its run-time taps against TP::h bit for bit before choosing a kernel built on this.
template <class TP>
struct pp_const {
    static constexpr int L = TP::L, M = TP::M, HL = TP::HL;
    static constexpr int W = HL + 1 + ((L - 1) * M) / L;

    __device__ static __forceinline__ void run(const float2 (&x)[W], float2 (&y)[L]) {
#pragma unroll
        for (int k = 0; k < L; ++k) y[k] = make_float2(0.f, 0.f);
#pragma unroll
        for (int d = HL; d >= 0; --d) {
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const int o = (k * M) / L, ph = (k * M) % L;
                constexpr_if_nonzero(TP::h[ph + d * L], x[HL + o - d], y[k]);
            }
        }
    }

    // the same sums with the window read from LDS as it is consumed: input i is loaded LOOK delay
    // rows before its first use (d = HL + o_max - i), so about o_max + 1 + LOOK inputs are live instead
    // of all W (the register budget of occupancy-bound callers); bit-identical to run()
    template <int LOOK = 2>
    __device__ static __forceinline__ void run_lds(const float2* xw, float2 (&y)[L]) {
        constexpr int OM = ((L - 1) * M) / L;
        float2 x[W];
#pragma unroll
        for (int i = 0; i <= OM + LOOK && i < W; ++i) x[i] = xw[i];
#pragma unroll
        for (int k = 0; k < L; ++k) y[k] = make_float2(0.f, 0.f);
#pragma unroll
        for (int d = HL; d >= 0; --d) {
            // the input that becomes needed LOOK rows from now; a compiler barrier every other row
            // keeps the loads where they are (hoisted, all W would be live again)
            constexpr_load(xw, x, HL + OM - d + LOOK + 1);
            if ((HL - d) % 2 == 1) asm volatile("" ::: "memory");
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const int o = (k * M) / L, ph = (k * M) % L;
                constexpr_if_nonzero(TP::h[ph + d * L], x[HL + o - d], y[k]);
            }
        }
    }

    // the same sums input-major from LDS: window input i (ascending, in 16-B pairs; xw 16-B aligned)
    // updates every output k whose span holds it (d = HL + o_k - i), so output k still sums
    // d = HL .. 0 in order, bit-identical to run(); live state is the L sums and one input pair. The
    // sums are pinned after every pair, or the compiler sinks each output's FMAs into its consumer and
    // holds the whole window again.
    // PAIRS: 16-B reads of input pairs (xw 16-B aligned), else 8-B reads (any float2 alignment)
    template <bool PAIRS = true>
    __device__ static __forceinline__ void run_imaj(const float2* xw, float2 (&y)[L]) {
        static_assert(L == 9 || L == 10, "pin list");
#pragma unroll
        for (int k = 0; k < L; ++k) y[k] = make_float2(0.f, 0.f);
        auto pair = [&](int j) -> float4 {
            if constexpr (PAIRS) return reinterpret_cast<const float4*>(xw)[j];
            const float2 a = xw[2 * j], b = 2 * j + 1 < W ? xw[2 * j + 1] : make_float2(0.f, 0.f);
            return make_float4(a.x, a.y, b.x, b.y);
        };
        float4 nxt = pair(0);
#pragma unroll
        for (int j = 0; 2 * j < W; ++j) {
            const float4 cur = nxt;
            if (2 * j + 2 < W) nxt = pair(j + 1);
            asm volatile("" ::: "memory");  // one pair ahead, not the whole window
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int i = 2 * j + e;
                if (i >= W) continue;
                const float2 xi = e ? make_float2(cur.z, cur.w) : make_float2(cur.x, cur.y);
#pragma unroll
                for (int k = 0; k < L; ++k) {
                    const int o = (k * M) / L, ph = (k * M) % L, d = HL + o - i;
                    if (d < 0 || d > HL) continue;
                    constexpr_if_nonzero(TP::h[ph + d * L], xi, y[k]);
                }
            }
            if constexpr (L == 9)
                asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]),
                             "+v"(y[8]));
            else
                asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]),
                             "+v"(y[8]), "+v"(y[9]));
        }
    }

  private:
    __device__ static __forceinline__ void constexpr_load(const float2* xw, float2 (&x)[W], const int i) {
        if (i > ((L - 1) * M) / L && i < W) x[i] = xw[i];
    }
    __device__ static __forceinline__ void constexpr_if_nonzero(const float t, const float2 xv, float2& acc) {
        if (t != 0.f) {  // compile-time after unrolling: padding taps cost nothing (fma(x, 0, a) == a)
            acc.x = fmaf(xv.x, t, acc.x);
            acc.y = fmaf(xv.y, t, acc.y);
        }
    }
};

}  // namespace dnrp::dev

namespace dnrp::dev {

// ---- polyphase blocks on the matrix cores (split fp16, three passes)
// 16 polyphase blocks of L outputs as one v_mfma_f32_16x16x32_f16 per pass and component:
//   C[q][c] = sum_i X[q][i] G[i][c],  X[q][i] = window input i of block q (16 x 32), G = the block
//   taps (32 x 16: G[i][c] = h[ph_c + (HL + o_c - i) L] inside output c's FIR span, else 0).
// Every f32 operand is split into fp16 hi + lo (x = hi + lo to ~2^-20 relative, hi rounded toward
// zero); the product keeps hi*hi + hi*lo + lo*hi (the dropped lo*lo is ~2^-20 of it), accumulated in
// f32 -- about 1e-6 relative against the f32 FMA chain of pp_direct. The window samples are stored as
// split words in the block's LDS buffer: slot s = {HI = (re_hi, im_hi), LO = (re_lo, im_lo)} in the
// 8 bytes a float2 takes, so the buffer keeps its layout.
// Lane l: A rows (blocks) l & 15, k = 8 (l >> 4) + j (j = 0..7); B rows k, column (output) l & 15;
// C column l & 15, rows 4 (l >> 4) + r (MI355X guide, 16x16x32 operand / accumulator maps).
typedef _Float16 mf_h8 __attribute__((ext_vector_type(8)));
typedef __fp16 mf_h2 __attribute__((ext_vector_type(2)));  // v_cvt_pkrtz_f16_f32 result
typedef float mf_f4 __attribute__((ext_vector_type(4)));
typedef uint32_t mf_u2 __attribute__((ext_vector_type(2)));
typedef uint32_t mf_u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint2 mf_split(float2 v) {  // -> {HI, LO} words of one complex sample
    const mf_h2 hi = __builtin_amdgcn_cvt_pkrtz(v.x, v.y);
    const mf_h2 lo = __builtin_amdgcn_cvt_pkrtz(v.x - static_cast<float>(hi.x), v.y - static_cast<float>(hi.y));
    return make_uint2(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo));
}

// A operands of one lane: 8 consecutive split slots s[0..7] -> (re_hi, im_hi, re_lo, im_lo) half8 each
__device__ __forceinline__ void mf_operands(const uint2 (&s)[8], mf_h8& rh, mf_h8& ih, mf_h8& rl, mf_h8& il) {
    uint4 a, b, c, d;
    uint32_t* pa = &a.x;
    uint32_t* pb = &b.x;
    uint32_t* pc = &c.x;
    uint32_t* pd = &d.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint2 s0 = s[2 * j], s1 = s[2 * j + 1];
        pa[j] = __builtin_amdgcn_perm(s1.x, s0.x, 0x05040100u);  // re_hi of samples 2j, 2j+1
        pb[j] = __builtin_amdgcn_perm(s1.x, s0.x, 0x07060302u);  // im_hi
        pc[j] = __builtin_amdgcn_perm(s1.y, s0.y, 0x05040100u);  // re_lo
        pd[j] = __builtin_amdgcn_perm(s1.y, s0.y, 0x07060302u);  // im_lo
    }
    rh = __builtin_bit_cast(mf_h8, a);
    ih = __builtin_bit_cast(mf_h8, b);
    rl = __builtin_bit_cast(mf_h8, c);
    il = __builtin_bit_cast(mf_h8, d);
}

// 16 blocks: w = the lane's 8 window slots (block l & 15, window inputs 8 (l >> 4) ..), gh / gl =
// the lane's taps (hi / lo). Returns the real and imaginary accumulators (C rows 4 (l >> 4) + r).
__device__ __forceinline__ void mf_blocks(const uint2 (&w)[8], const mf_h8& gh, const mf_h8& gl, mf_f4& cr, mf_f4& ci) {
    mf_h8 rh, ih, rl, il;
    mf_operands(w, rh, ih, rl, il);
    const mf_f4 z = {0.f, 0.f, 0.f, 0.f};
    cr = __builtin_amdgcn_mfma_f32_16x16x32_f16(rh, gh, z, 0, 0, 0);
    ci = __builtin_amdgcn_mfma_f32_16x16x32_f16(ih, gh, z, 0, 0, 0);
    cr = __builtin_amdgcn_mfma_f32_16x16x32_f16(rh, gl, cr, 0, 0, 0);
    ci = __builtin_amdgcn_mfma_f32_16x16x32_f16(ih, gl, ci, 0, 0, 0);
    cr = __builtin_amdgcn_mfma_f32_16x16x32_f16(rl, gh, cr, 0, 0, 0);
    ci = __builtin_amdgcn_mfma_f32_16x16x32_f16(il, gh, ci, 0, 0, 0);
}

}  // namespace dnrp::dev
