// Batched turbo decoding of PDC code blocks on gfx950 (see fec_dev.hpp). Three kernels:
//   fec_dematch_kernel  workgroup = wave of code blocks: rate de-matching (srsran_rm_turbo_rx_lut_ role,
//                       pdc_enc.cpp:359-360) straight into the wave's [k][lane] soft streams
//   fec_tdec_kernel     wavefront = up to 64 code blocks of one size K, lane = code block: the
//                       iterations of the host decoder (fec.cpp Tdec / map_decode) with CRC early stop
//   fec_tbcrc_kernel    wavefront = packet with C > 1: transport-block CRC24A (pdc_enc.cpp:478-488),
//                       16-B pieces per lane joined by GF(2) shifts
// and the encoder: fec_encode_kernel (wavefront = code block) + fec_pack_kernel (scratch -> d rows).
#include "fec_dev.hpp"

#ifndef FEC_BWD_AHEAD
#define FEC_BWD_AHEAD 1  // backward-pass windows prefetched (2: 256 VGPRs + spills, no gain)
#endif
#ifndef FEC_FWD_AHEAD
#define FEC_FWD_AHEAD 2  // forward-pass windows prefetched (A/B: 1 -> 2 tdec 54.6 -> 46.3 ms, 3 no gain)
#endif

namespace dnrp::dev {

__global__ void __launch_bounds__(256) fec_dematch_kernel(FecArgs A) {
    // workgroup = wave of up to 64 same-size code blocks; thread (row r, lane l): list entries
    // q = r, r + 4, ... of code block l. The 64 lanes of a wavefront write one 128-B [k][lane] row
    // per entry; their reads walk 64 LLR rows in step (L1-resident lines).
    const FecWave w = A.waves[blockIdx.x];
    const uint32_t l = threadIdx.x & 63u, r = threadIdx.x >> 6;
    const uint32_t K = w.K, nvalid = 3 * (K + 4);
    const bool active = l < w.n;
    const FecCb cb = A.cbs[w.first_cb + (active ? l : 0)];
    const uint32_t* valid = A.tab + w.valid_off;
    int16_t* base = A.work16 + w.data_off;
    const int16_t* llr = A.llr + cb.llr_off;
    // tail slot of (stream, t = index - K), as fec.cpp Tdec::load orders them
    const uint8_t tslot[3][4] = {{0, 4, 6, 10}, {3, 2, 9, 8}, {1, 5, 7, 11}};
    // HARQ: a block that passed its CRC in an earlier transmission is neither combined nor decoded
    // (pdc_enc.cpp:346-406); the others add the new soft bits to their softbuffer
    const bool harq = A.sb != nullptr && active && !A.flags[cb.flag_off];
    for (uint32_t q = r; q < nvalid; q += 4) {
        const uint32_t e = valid[q], st = e >> 16, idx = e & 0xFFFF;
        // soft bits j = j0, j0 + nvalid, ... land on list entry q; summed in j order with int16
        // saturation like the host's sequential accumulation (starting from the softbuffer value)
        int16_t* sbe = harq ? A.sb + cb.sb_off + (size_t)st * (K + 4) + idx : nullptr;
        int32_t sum = harq ? *sbe : 0;
        if (active) {
            uint32_t j = q >= cb.start ? q - cb.start : q + nvalid - cb.start;
            for (; j < cb.E; j += nvalid) sum = min(32767, max(-32768, sum + (int32_t)llr[j]));
        }
        if (harq) *sbe = (int16_t)sum;
        if (idx < K) base[(size_t)st * K * 64 + (size_t)idx * 64 + l] = (int16_t)sum;
        else A.tail[(size_t)blockIdx.x * 12 * 64 + tslot[st][idx - K] * 64 + l] = sum;
    }
    // decoder 2's extrinsic needs no zero fill: the first iteration's decoder 1 reads none
}

// One trellis step of the forward recursion (state s = 4 s1 + 2 s2 + s3; next n = (a, s1, s2),
// predecessors s = (s1, s2, s3) for s3 = 0, 1 with input u = a ^ s2 ^ s3, parity p = a ^ s1 ^ s3).
__device__ __forceinline__ void fwd_step(int32_t (&a)[8], int32_t A, int32_t B) {
    int32_t nxt[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        const int an = n >> 2, s1 = (n >> 1) & 1, s2 = n & 1;
        int32_t best = FEC_NEG;
#pragma unroll
        for (int s3 = 0; s3 < 2; ++s3) {
            const int s = (s1 << 2) | (s2 << 1) | s3;
            const int u = an ^ s2 ^ s3, p = an ^ s1 ^ s3;
            best = max(best, a[s] + (u ? A : 0) + (p ? B : 0));
        }
        nxt[n] = best;
    }
    int32_t mx = nxt[0];
#pragma unroll
    for (int n = 1; n < 8; ++n) mx = max(mx, nxt[n]);
#pragma unroll
    for (int n = 0; n < 8; ++n) a[n] = max(nxt[n] - mx, FEC_NEG);
}

// QPP interleaver pi(i) = (f1 i + f2 i^2) mod K on wave-uniform values: direct evaluation at a
// window start, then pi(i+1) = pi(i) + d(i), d(i+1) = d(i) + 2 f2 (mod K)
struct Qpp {
    uint32_t K, f1, f2;
    __device__ uint32_t at(uint32_t i) const {
        return (uint32_t)(((uint64_t)f1 * i + (uint64_t)f2 * ((uint64_t)i * i % K)) % K);
    }
    __device__ uint32_t delta(uint32_t i) const {  // pi(i+1) - pi(i) mod K = f1 + f2 (2 i + 1)
        return (uint32_t)(((uint64_t)f1 + (uint64_t)f2 * (2ull * i + 1)) % K);
    }
};

// inputs of step k: decoder 1 reads natural order (its a priori = decoder 2's extrinsic, stored in
// natural order), decoder 2 the QPP row pi = pi(k)
template <int DEC>
__device__ __forceinline__ void inputs(const int16_t* base, uint32_t K, uint32_t k, uint32_t pi, uint32_t l, int32_t* a,
                                       int32_t* b) {
    const int16_t *sys = base, *p1 = base + (size_t)K * 64, *p2 = base + (size_t)2 * K * 64;
    const int16_t *le1 = base + (size_t)3 * K * 64, *le2 = base + (size_t)4 * K * 64;
    if (DEC != 2) {  // DEC 0: decoder 1 of the first iteration, whose a priori is zero
        *a = (int32_t)sys[(size_t)k * 64 + l] + (DEC == 1 ? (int32_t)le2[(size_t)k * 64 + l] : 0);
        *b = p1[(size_t)k * 64 + l];
    } else {
        *a = (int32_t)sys[(size_t)pi * 64 + l] + le1[(size_t)pi * 64 + l];
        *b = p2[(size_t)k * 64 + l];
    }
}

// loads of the FEC_WIN steps from k0 (pi values of the window in pis[] for decoder 2)
template <int DEC>
__device__ __forceinline__ void load_win(const int16_t* base, const Qpp& q, uint32_t k0, uint32_t l, int32_t* a,
                                         int32_t* b, uint32_t* pis) {
    uint32_t pi = DEC == 2 ? q.at(k0) : 0, d = DEC == 2 ? q.delta(k0) : 0;
#pragma unroll
    for (int t = 0; t < (int)FEC_WIN; ++t) {
        pis[t] = pi;
        inputs<DEC>(base, q.K, k0 + t, pi, l, &a[t], &b[t]);
        if (DEC == 2) {
            pi += d;
            pi = pi >= q.K ? pi - q.K : pi;
            d += 2 * q.f2 % q.K;
            d = d >= q.K ? d - q.K : d;
        }
    }
}

// One constituent decoder (fec.cpp map_decode): forward pass with checkpoints, backward pass with
// the windows' forward metrics recomputed in registers; extrinsic out (and, for decoder 2, the
// hard decisions of the full LLR at the de-interleaved positions).
template <int DEC>
__device__ void map_decode(const FecArgs& A, const FecWave& w, uint32_t wave, int16_t* base, uint32_t l) {
    const uint32_t K = w.K, nw = K / FEC_WIN;
    int32_t* ck = A.ck + w.ck_off;
    int32_t a[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) a[s] = s == 0 ? 0 : FEC_NEG;
    // software pipeline: the inputs of the next FEC_FWD_AHEAD windows are in flight while this
    // window is computed
    const Qpp q{K, w.f1, w.f2};
    uint32_t pis[FEC_WIN];
    int32_t Ab[FEC_FWD_AHEAD][FEC_WIN], Bb[FEC_FWD_AHEAD][FEC_WIN];
#pragma unroll
    for (int d = 0; d < FEC_FWD_AHEAD; ++d)
        if (d * FEC_WIN < K) load_win<DEC>(base, q, d * FEC_WIN, l, Ab[d], Bb[d], pis);
    for (uint32_t k0 = 0; k0 < K; k0 += FEC_WIN) {
        int32_t Ak[FEC_WIN], Bk[FEC_WIN];
#pragma unroll
        for (int t = 0; t < (int)FEC_WIN; ++t) Ak[t] = Ab[0][t], Bk[t] = Bb[0][t];
#pragma unroll
        for (int d = 0; d + 1 < FEC_FWD_AHEAD; ++d)
#pragma unroll
            for (int t = 0; t < (int)FEC_WIN; ++t) Ab[d][t] = Ab[d + 1][t], Bb[d][t] = Bb[d + 1][t];
        if (k0 + FEC_FWD_AHEAD * FEC_WIN < K)
            load_win<DEC>(base, q, k0 + FEC_FWD_AHEAD * FEC_WIN, l, Ab[FEC_FWD_AHEAD - 1], Bb[FEC_FWD_AHEAD - 1], pis);
#pragma unroll
        for (int s = 0; s < 8; ++s) ck[((size_t)(k0 / FEC_WIN) * 8 + s) * 64 + l] = a[s];
#pragma unroll
        for (int t = 0; t < (int)FEC_WIN; ++t) fwd_step(a, Ak[t], Bk[t]);
    }
    // backward through the termination
    const int32_t* tl = A.tail + (size_t)wave * 12 * 64 + (DEC == 2 ? 6 : 0) * 64 + l;
    int32_t be[8], bn[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) be[s] = s == 0 ? 0 : FEC_NEG;
    for (int t = 2; t >= 0; --t) {
        const int32_t tx = tl[t * 64], tz = tl[(3 + t) * 64];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int s1 = (s >> 2) & 1, s2 = (s >> 1) & 1, s3 = s & 1;
            const int u = s2 ^ s3;  // input = feedback: a = 0
            const int p = s1 ^ s3;
            const int nx = (s1 << 1) | s2;
            bn[s] = be[nx] + (u ? tx : 0) + (p ? tz : 0);
        }
        int32_t mx = bn[0];
#pragma unroll
        for (int s = 1; s < 8; ++s) mx = max(mx, bn[s]);
#pragma unroll
        for (int s = 0; s < 8; ++s) be[s] = max(bn[s] - mx, FEC_NEG);
    }
    int16_t* le_out = base + (size_t)(DEC == 2 ? 4 : 3) * K * 64;
    uint8_t* bits = A.bits + w.data_off / 5;
    // the checkpoints and inputs of the FEC_BWD_AHEAD windows below the current one, prefetched
    int32_t cb_[FEC_BWD_AHEAD][8], Ab2[FEC_BWD_AHEAD][FEC_WIN], Bb2[FEC_BWD_AHEAD][FEC_WIN];
    uint32_t pb[FEC_BWD_AHEAD][FEC_WIN], pw[FEC_WIN];
#pragma unroll
    for (int d = 0; d < FEC_BWD_AHEAD; ++d) {
        const int32_t wd = (int32_t)nw - 1 - d;
        if (wd >= 0) {
#pragma unroll
            for (int s = 0; s < 8; ++s) cb_[d][s] = ck[((size_t)wd * 8 + s) * 64 + l];
            load_win<DEC>(base, q, wd * FEC_WIN, l, Ab2[d], Bb2[d], pb[d]);
        }
    }
    for (int32_t wi = (int32_t)nw - 1; wi >= 0; --wi) {
        int32_t aw[FEC_WIN][8], Aw[FEC_WIN], Bw[FEC_WIN];
#pragma unroll
        for (int s = 0; s < 8; ++s) aw[0][s] = cb_[0][s];
#pragma unroll
        for (int t = 0; t < (int)FEC_WIN; ++t) Aw[t] = Ab2[0][t], Bw[t] = Bb2[0][t], pw[t] = pb[0][t];
#pragma unroll
        for (int d = 0; d + 1 < FEC_BWD_AHEAD; ++d) {
#pragma unroll
            for (int s = 0; s < 8; ++s) cb_[d][s] = cb_[d + 1][s];
#pragma unroll
            for (int t = 0; t < (int)FEC_WIN; ++t) Ab2[d][t] = Ab2[d + 1][t], Bb2[d][t] = Bb2[d + 1][t], pb[d][t] = pb[d + 1][t];
        }
        if (wi - FEC_BWD_AHEAD >= 0) {
            const int32_t wd = wi - FEC_BWD_AHEAD;
#pragma unroll
            for (int s = 0; s < 8; ++s) cb_[FEC_BWD_AHEAD - 1][s] = ck[((size_t)wd * 8 + s) * 64 + l];
            load_win<DEC>(base, q, wd * FEC_WIN, l, Ab2[FEC_BWD_AHEAD - 1], Bb2[FEC_BWD_AHEAD - 1], pb[FEC_BWD_AHEAD - 1]);
        }
#pragma unroll
        for (int t = 0; t < (int)FEC_WIN; ++t) {
            if (t + 1 < (int)FEC_WIN) {
#pragma unroll
                for (int s = 0; s < 8; ++s) aw[t + 1][s] = aw[t][s];
                fwd_step(aw[t + 1], Aw[t], Bw[t]);
            }
        }
#pragma unroll
        for (int t = FEC_WIN - 1; t >= 0; --t) {
            const uint32_t k = wi * FEC_WIN + t;
            const int32_t Ak = Aw[t], Bk = Bw[t];
            int32_t m1 = INT32_MIN, m0 = INT32_MIN;
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int s1 = (s >> 2) & 1, s2 = (s >> 1) & 1, s3 = s & 1;
                int32_t b = INT32_MIN;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int an = u ^ s2 ^ s3, p = an ^ s1 ^ s3;
                    const int nx = (an << 2) | (s1 << 1) | s2;
                    const int32_t g = (u ? Ak : 0) + (p ? Bk : 0);
                    const int32_t v = aw[t][s] + g + be[nx];
                    if (u) m1 = max(m1, v); else m0 = max(m0, v);
                    b = max(b, g + be[nx]);
                }
                bn[s] = b;
            }
            const int32_t llr = m1 - m0;
            const int32_t e = min(32767, max(-32767, ((llr - Ak) * 3) >> 2));
            if (DEC != 2) {
                le_out[(size_t)k * 64 + l] = (int16_t)e;
            } else {  // natural order: decoder 1's a priori and the hard decisions at pi(k)
                le_out[(size_t)pw[t] * 64 + l] = (int16_t)e;
                bits[(size_t)pw[t] * 64 + l] = llr > 0;
            }
            int32_t mx = bn[0];
#pragma unroll
            for (int s = 1; s < 8; ++s) mx = max(mx, bn[s]);
#pragma unroll
            for (int s = 0; s < 8; ++s) be[s] = max(bn[s] - mx, FEC_NEG);
        }
    }
}

#ifndef DNRP_FEC_WPE
#define DNRP_FEC_WPE 2
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DNRP_FEC_WPE))) fec_tdec_kernel(FecArgs A) {
    // by value: the stores below may alias A.waves as far as the compiler knows, a reference would
    // make it reload the wave's fields after every store
    const FecWave w = A.waves[blockIdx.x];
    const uint32_t l = threadIdx.x;
    const bool active = l < w.n;
    const FecCb cb = A.cbs[w.first_cb + (active ? l : 0)];
    int16_t* base = A.work16 + w.data_off;
    const uint8_t* bits = A.bits + w.data_off / 5;
    const bool kept = A.sb != nullptr && active && A.flags[cb.flag_off];  // HARQ: decoded earlier
    bool done = !active || kept, ok = kept;
    uint32_t used = 0, mask = 0;
    for (uint32_t it = A.it_first; it <= A.max_iter; ++it) {
        if (__all(done)) break;
        if (!done) {
            if (it == 1)
                map_decode<0>(A, w, blockIdx.x, base, l);
            else
                map_decode<1>(A, w, blockIdx.x, base, l);
            map_decode<2>(A, w, blockIdx.x, base, l);
            used = it;
            // register after all K bits: 0 for a CRC24 block; for the PLCF's CRC16 the register the
            // mask it was sent with leaves (none / closed loop 0x5555 / beamforming 0xAAAA / both
            // 0xFFFF, pcc_enc.cpp:170-183) = mask * x^16 mod g: 0, 0xFB1A, 0xE615, 0x1D0F
            const uint32_t W = cb.poly == 0x1021u ? 16u : 24u, msk = (1u << W) - 1;
            uint32_t reg = 0;
            for (uint32_t k = 0; k < w.K; ++k) {
                const uint32_t top = (reg >> (W - 1)) & 1;
                reg = (reg << 1) & msk;
                if (top ^ bits[(size_t)k * 64 + l]) reg ^= cb.poly;
            }
            ok = W == 24 ? reg == 0 : (reg == 0 || reg == 0xFB1Au || reg == 0xE615u || reg == 0x1D0Fu);
            mask = W == 24 ? 0u : (reg == 0xFB1Au ? 1u : (reg == 0xE615u ? 2u : (reg == 0x1D0Fu ? 3u : 0u)));
            if (ok && it >= A.min_iter) done = true;
        }
    }
    if (!active) return;
    if (!done && !A.final_pass) {  // undecided: its streams and extrinsic stay for the continuation
        A.cb_out[w.first_cb + l] = (used << 4) | 8u;
        return;
    }
    ok = done && ok;
    if (kept) {  // its bytes from the earlier decode stay in the output row
        A.cb_out[w.first_cb + l] = 1u;
        return;
    }
    if (A.sb != nullptr && ok) A.flags[cb.flag_off] = 1;
    for (uint32_t j = 0; j < cb.out_bytes; ++j) {
        uint32_t v = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) v = (v << 1) | bits[(size_t)(8 * j + t) * 64 + l];
        A.tb[cb.tb_off + j] = (uint8_t)v;
    }
    A.cb_out[w.first_cb + l] = (used << 4) | (mask << 1) | (ok ? 1u : 0u);
}

// GF(2)[x] helpers for joining segment CRCs (zero initial register, no final XOR, so the CRC is
// linear): crc(A || B) = crc(A) x^{|B|} + crc(B) mod g, and leading zero bits do not change it.
// W-bit CRCs with polynomial g = x^W + poly.
template <int W>
__device__ __forceinline__ uint32_t mulmod(uint32_t a, uint32_t b, uint32_t poly) {
    constexpr uint32_t M = (1u << W) - 1u;
    uint32_t r = 0;
#pragma unroll
    for (int i = W - 1; i >= 0; --i) {
        const uint32_t top = (r >> (W - 1)) & 1u;
        r = (r << 1) & M;
        if (top) r ^= poly;
        if ((b >> i) & 1u) r ^= a;
    }
    return r;
}
template <int W>
__device__ uint32_t xpow(uint64_t n, uint32_t poly) {  // x^n mod g
    uint32_t r = 1, b = 2;
    while (n) {
        if (n & 1) r = mulmod<W>(r, b, poly);
        b = mulmod<W>(b, b, poly);
        n >>= 1;
    }
    return r;
}
template <int W>
__device__ __forceinline__ uint32_t xshift(uint32_t n, uint32_t poly) {  // x^n mod g by n shifts (small n)
    constexpr uint32_t M = (1u << W) - 1u;
    uint32_t r = 1;
    for (uint32_t i = 0; i < n; ++i) r = ((r << 1) & M) ^ (((r >> (W - 1)) & 1u) ? poly : 0u);
    return r;
}
constexpr uint32_t CRC24A_POLY = 0x864CFB, CRC24B_POLY = 0x800063, CRC16_POLY = 0x1021;

// Transport-block CRC24A (pdc_enc.cpp:478-488). The TB is read in 1-KiB blocks, one coalesced 16-B
// piece per lane; each lane's CRC (byte table in LDS) of its piece is joined with its neighbours' in a
// 6-level tree (multipliers x^128 .. x^4096, equal-length segments), and the running CRC takes the
// block by crc x^(8 len) + block. A short last block is front-padded (leading zeros leave a CRC
// unchanged), so its segments keep equal lengths.
__global__ void __launch_bounds__(64) fec_tbcrc_kernel(FecTbArgs A) {
    __shared__ uint32_t T[256];
    const uint32_t p = blockIdx.x, l = threadIdx.x;
    for (uint32_t v = l; v < 256; v += 64) {  // byte table of CRC24A: T[v] = crc of byte v
        uint32_t r = v << 16;
        for (int t = 0; t < 8; ++t) r = ((r << 1) & 0xFFFFFFu) ^ (((r >> 23) & 1u) ? CRC24A_POLY : 0u);
        T[v] = r;
    }
    __syncthreads();
    const uint8_t* d = A.tb + A.tb_off[p];
    const uint32_t nb = A.nbytes[p];
    uint32_t lv[7];
    lv[0] = xshift<24>(128, CRC24A_POLY);
#pragma unroll
    for (int t = 0; t < 6; ++t) lv[t + 1] = mulmod<24>(lv[t], lv[t], CRC24A_POLY);  // x^256 .. x^8192
    uint32_t crc = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint32_t len = min(1024u, nb - b0);
        const int32_t s0 = static_cast<int32_t>(16 * l) - static_cast<int32_t>(1024 - len);  // piece start in the block
        uint32_t r = 0;
        if (s0 >= 0 && (((uintptr_t)(d + b0 + s0)) & 15u) == 0) {  // whole aligned piece: one 16-B load
            const uint4 v = *reinterpret_cast<const uint4*>(d + b0 + s0);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 4; ++k) r = ((r << 8) & 0xFFFFFFu) ^ T[((r >> 16) ^ (w[q] >> (8 * k))) & 0xFFu];
        } else {
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int32_t i = s0 + t;
                if (i >= 0) r = ((r << 8) & 0xFFFFFFu) ^ T[((r >> 16) ^ d[b0 + i]) & 0xFFu];
            }
        }
#pragma unroll
        for (int t = 0; t < 6; ++t) {
            const uint32_t o = __shfl_down(r, 1u << t);
            if ((l & ((2u << t) - 1u)) == 0) r = mulmod<24>(r, lv[t], CRC24A_POLY) ^ o;
        }
        const uint32_t blk = __shfl(r, 0);
        crc = mulmod<24>(crc, len == 1024 ? lv[6] : xpow<24>(8ull * len, CRC24A_POLY), CRC24A_POLY) ^ blk;
    }
    if (l == 0) {
        if (A.crc_out) {
            A.crc_out[p] = crc;
        } else {
            const uint32_t rx = ((uint32_t)d[nb] << 16) | ((uint32_t)d[nb + 1] << 8) | d[nb + 2];
            A.ok[p] = crc == rx;
        }
    }
}

// ---- encoder (fec.cpp dnrp_pdc_encode: pdc_enc.cpp:148-229; dnrp_pcc_encode: pcc_enc.cpp:166-212) ----
// One wavefront per code block, its bits shared by the lanes as MSB-first 32-bit words in LDS: c (the
// block: TB bits, then the TB CRC24A / PLCF CRC16 ^ mask, then the code-block CRC24B), and the three
// coded streams d0 = c, d1 = z, d2 = z' with their tails (TS 36.212 §5.1.3.2). Each constituent
// encoder runs lane-parallel: lane l encodes bits [l Lc, (l + 1) Lc) once from the zero state, the
// entry states follow from an affine prefix scan over the lanes (state map M = A^Lc), and a second
// pass from the true entry state writes the parity words. Rate matching: 64 consecutive output bits
// per step -- list entries (start + j) mod 3 (K + 4) read coalesced, the bits gathered from LDS, one
// ballot -- kept one 8-B word per lane and stored 512 B at a time into the packed scratch, each code
// block at a 64-bit aligned offset; fec_pack_kernel splices the blocks into the d rows.
constexpr uint32_t FEC_ENC_WAVES = 4;
// bits per lane of a K-bit block (multiple of 32, <= 96 for K <= 6144); host: fec_enc_chunk too
constexpr uint32_t FEC_ENC_WORDS = (6144 + 4 + 31) / 32 + 1;

__device__ __forceinline__ uint32_t lbit(const uint32_t* w, uint32_t k) { return (w[k >> 5] >> (31u - (k & 31u))) & 1u; }

// RSC step, state s = s1 | s2 << 1 | s3 << 2: a = u ^ s2 ^ s3, z = a ^ s1 ^ s3, next = (a, s1, s2)
__device__ __forceinline__ uint32_t rsc_step(uint32_t& s, uint32_t u) {
    const uint32_t s1 = s & 1u, s2 = (s >> 1) & 1u, s3 = (s >> 2) & 1u, a = u ^ s2 ^ s3;
    s = a | (s1 << 1) | (s2 << 2);
    return a ^ s1 ^ s3;
}
struct gf2m3 {  // 3x3 GF(2) matrix as its three 3-bit columns
    uint32_t c0, c1, c2;
    __device__ uint32_t apply(uint32_t s) const { return ((s & 1u) ? c0 : 0u) ^ ((s & 2u) ? c1 : 0u) ^ ((s & 4u) ? c2 : 0u); }
    __device__ gf2m3 sq() const { return {apply(c0), apply(c1), apply(c2)}; }
};

// one constituent encoder over K input bits in(i): parity words of bits [i0, i0 + n) into z (the lane's
// whole words: Lc is a multiple of 32, at most 96), returns the encoder's final state (every lane).
// The lane's input bits are gathered once into registers; mA: the state map M = A^Lc (host, per K)
template <class In>
__device__ __forceinline__ uint32_t rsc_wave(In in, uint32_t K, uint32_t Lc, uint32_t mA, uint32_t lane, uint32_t* z) {
    const uint32_t i0 = lane * Lc, n = i0 < K ? min(Lc, K - i0) : 0u;
    uint32_t xw[3] = {0u, 0u, 0u};
    uint32_t s = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t u = in(i0 + i);
        xw[i >> 5] |= u << (31u - (i & 31u));
        rsc_step(s, u);
    }
    // the inclusive affine scan v_l = F_l + M v_{l-1} over the lanes
    gf2m3 M{mA & 7u, (mA >> 3) & 7u, (mA >> 6) & 7u};
    uint32_t v = s;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d);
        if (lane >= d) v ^= M.apply(o);
        M = M.sq();
    }
    uint32_t st = __shfl_up(v, 1u);
    if (lane == 0) st = 0;
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
        if (32 * q >= n) break;
        const uint32_t x = xw[q], nb = min(32u, n - 32 * q);
        uint32_t w = 0;
        for (uint32_t t = 0; t < nb; ++t) w = (w << 1) | rsc_step(st, (x >> (31u - t)) & 1u);
        z[(i0 >> 5) + q] = w << (32u - nb);
    }
    // the encoder's final state: the last lane's, after its own (possibly short) chunk
    return __shfl(st, (K - 1) / Lc);
}

__global__ void __launch_bounds__(64 * FEC_ENC_WAVES) fec_encode_kernel(FecEncArgs A, uint32_t n_cb) {
    __shared__ uint32_t lds[FEC_ENC_WAVES][4][FEC_ENC_WORDS];
    __shared__ unsigned long long stage[FEC_ENC_WAVES][64];  // direct mode: a batch of output words
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t ci = blockIdx.x * FEC_ENC_WAVES + wv;
    if (ci >= n_cb) return;  // uniform per wave; no workgroup barrier below
    const FecEncCb cb = A.cbs[ci];
    uint32_t* cw = lds[wv][0];
    uint32_t* d1 = lds[wv][1];
    uint32_t* d2 = lds[wv][2];
    uint32_t* d0 = lds[wv][3];
    const uint32_t K = cb.K, D = K + 4, nw = (D + 31) / 32;
    for (uint32_t i = lane; i < FEC_ENC_WORDS; i += 64) cw[i] = d0[i] = d1[i] = d2[i] = 0u;
    const uint8_t* tb = A.tb + cb.tb_off;
    const uint32_t tbytes = cb.tbs >> 3;
    // the CRC after the TB: PLCF CRC16 ^ mask over its 40 / 80 bits (every lane), else the TB's CRC24A
    uint32_t tcrc;
    if (cb.crc16) {
        uint32_t r16 = 0;
        for (uint32_t pos = 0; pos < cb.tbs; ++pos) {
            const uint32_t top = (r16 >> 15) & 1u;
            r16 = (r16 << 1) & 0xFFFFu;
            if (top ^ ((tb[pos >> 3] >> (7 - (pos & 7))) & 1u)) r16 ^= CRC16_POLY;
        }
        tcrc = r16 ^ cb.mask;
    } else {
        tcrc = A.tbcrc[cb.pkt];
    }
    const uint32_t clen = cb.crc16 ? 16u : 24u;
    __builtin_amdgcn_wave_barrier();
    // c words [0, rlen): TB bits from bit rp, the TB / PLCF CRC bits after bit tbs
    for (uint32_t i = lane; 32 * i < cb.rlen; i += 64) {
        const uint32_t pos = cb.rp + 32 * i, b0 = pos >> 3, sh = pos & 7u;
        uint64_t v = 0;
#pragma unroll
        for (int t = 0; t < 5; ++t) v = (v << 8) | (b0 + t < tbytes ? tb[b0 + t] : 0u);
        uint32_t w = static_cast<uint32_t>(v >> (8 - sh));
        if (pos + 32 > cb.tbs)  // the word reaches the CRC after the TB
            for (uint32_t t = 0; t < 32; ++t) {
                const uint32_t q = pos + t;
                if (q >= cb.tbs && q < cb.tbs + clen) w |= ((tcrc >> (clen - 1 - (q - cb.tbs))) & 1u) << (31 - t);
            }
        const uint32_t valid = min(32u, cb.rlen - 32 * i);
        cw[i] = valid == 32 ? w : w & ~(0xFFFFFFFFu >> valid);
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t Lc = fec_enc_chunk(K);
    if (cb.crc24b) {
        // CRC24B over c[0, rlen), front-padded to 64 Lc bits so the lanes' segments are equal
        const int32_t off = static_cast<int32_t>(64 * Lc) - static_cast<int32_t>(cb.rlen);
        uint32_t r = 0;
        for (uint32_t t = 0; t < Lc; ++t) {
            const int32_t k = static_cast<int32_t>(lane * Lc + t) - off;
            if (k < 0) continue;
            const uint32_t top = (r >> 23) & 1u;
            r = (r << 1) & 0xFFFFFFu;
            if (top ^ lbit(cw, static_cast<uint32_t>(k))) r ^= CRC24B_POLY;
        }
        uint32_t mlt = xshift<24>(Lc, CRC24B_POLY);
#pragma unroll
        for (int t = 0; t < 6; ++t) {
            const uint32_t o = __shfl_down(r, 1u << t);
            if ((lane & ((2u << t) - 1u)) == 0) r = mulmod<24>(r, mlt, CRC24B_POLY) ^ o;
            mlt = mulmod<24>(mlt, mlt, CRC24B_POLY);
        }
        const uint32_t crc = __shfl(r, 0);
        if (lane < 24) {
            const uint32_t k = cb.rlen + lane;
            atomicOr(&cw[k >> 5], ((crc >> (23 - lane)) & 1u) << (31u - (k & 31u)));
        }
        __builtin_amdgcn_wave_barrier();
    }
    // d0 = c (bits < K)
    for (uint32_t i = lane; i < nw; i += 64) d0[i] = cw[i];
    // encoder 1 (natural order) -> d1, encoder 2 on the QPP rows c[pi(i)] -> d2
    const uint32_t f1 = rsc_wave([&](uint32_t i) { return lbit(cw, i); }, K, Lc, cb.mA, lane, d1);
    const uint32_t f2x2 = 2 * cb.f2 % K;
    uint32_t pi = 0, dl = 0, inext = 0xFFFFFFFFu;
    auto qpp = [&](uint32_t i) {  // i runs consecutively per lane: recurrence after the first index
        if (i != inext) {
            pi = static_cast<uint32_t>(((uint64_t)cb.f1 * i + (uint64_t)cb.f2 * ((uint64_t)i * i % K)) % K);
            dl = static_cast<uint32_t>(((uint64_t)cb.f1 + (uint64_t)cb.f2 * (2ull * i + 1)) % K);
        }
        const uint32_t r = pi;
        pi += dl;
        pi = pi >= K ? pi - K : pi;
        dl += f2x2;
        dl = dl >= K ? dl - K : dl;
        inext = i + 1;
        return r;
    };
    const uint32_t f2 = rsc_wave([&](uint32_t i) { return lbit(cw, qpp(i)); }, K, Lc, cb.mA, lane, d2);
    __builtin_amdgcn_wave_barrier();
    // trellis termination (TS 36.212 §5.1.3.2.2): x / z of three feedback steps per encoder
    if (lane == 0) {
        uint32_t x1[3], z1[3], x2[3], z2[3], s = f1;
        for (int t = 0; t < 3; ++t) {
            const uint32_t s1 = s & 1u, s2 = (s >> 1) & 1u, s3 = (s >> 2) & 1u;
            x1[t] = s2 ^ s3, z1[t] = s1 ^ s3;
            s = (s1 << 1) | (s2 << 2);
        }
        s = f2;
        for (int t = 0; t < 3; ++t) {
            const uint32_t s1 = s & 1u, s2 = (s >> 1) & 1u, s3 = (s >> 2) & 1u;
            x2[t] = s2 ^ s3, z2[t] = s1 ^ s3;
            s = (s1 << 1) | (s2 << 2);
        }
        const uint32_t t0[4] = {x1[0], z1[1], x2[0], z2[1]}, t1[4] = {z1[0], x1[2], z2[0], x2[2]},
                       t2[4] = {x1[1], z1[2], x2[1], z2[2]};
        for (int t = 0; t < 4; ++t) {
            const uint32_t k = K + t, sh = 31u - (k & 31u);
            d0[k >> 5] |= t0[t] << sh;
            d1[k >> 5] |= t1[t] << sh;
            d2[k >> 5] |= t2[t] << sh;
        }
    }
    __builtin_amdgcn_wave_barrier();
    // rate matching: output bit j = stream[st][idx] of list entry (start + j) mod 3 D
    const uint32_t* valid = A.tab + cb.valid_off;
    const uint32_t nvalid = 3 * D;
    unsigned long long* out = reinterpret_cast<unsigned long long*>(A.ebits) + (cb.oo >> 6);
    const uint32_t nm = (cb.E + 63) / 64;
    uint32_t base = cb.start;  // list index of output bit 64 m
    unsigned long long acc = 0;
    for (uint32_t m = 0; m < nm; ++m) {
        uint32_t q = base + lane;
        q = q >= nvalid ? q - nvalid : q;
        const uint32_t j = 64 * m + lane;
        uint32_t bit = 0;
        if (j < cb.E) {
            const uint32_t ent = valid[q], st = ent >> 16, idx = ent & 0xFFFFu;
            bit = lbit(st == 0 ? d0 : st == 1 ? d1 : d2, idx);
        }
        const unsigned long long bal = __ballot(bit);
        // ballot bit i = output bit 64 m + i -> bytes in stream order, MSB first
        const unsigned long long v = __builtin_bswap64(__builtin_bitreverse64(bal));
        if ((m & 63u) == lane) acc = v;
        if ((m & 63u) == 63u || m + 1 == nm) {
            if (!A.d) {
                if (lane <= (m & 63u)) out[(m & ~63u) + lane] = acc;
            } else {
                // direct: the block's bytes straight into its packet's d row (whole bytes, host-checked),
                // 64 consecutive bytes per store instruction through the wave's LDS stage
                stage[wv][lane] = acc;
                __builtin_amdgcn_wave_barrier();
                const uint8_t* sb = reinterpret_cast<const uint8_t*>(stage[wv]);
                const uint32_t b0 = 8 * (m & ~63u), nbt = min(512u, cb.E / 8 - b0);
                uint8_t* dst = A.d + (size_t)cb.pkt * A.d_stride + cb.pstart / 8 + b0;
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k)
                    if (64 * k + lane < nbt) dst[64 * k + lane] = sb[64 * k + lane];
                __builtin_amdgcn_wave_barrier();
            }
        }
        base += 64;
        base = base >= nvalid ? base - nvalid : base;  // nvalid >= 3 (40 + 4) > 64
    }
}

// packed scratch (each code block from a 64-bit aligned bit offset) -> MSB-first d rows: thread =
// output byte of a packet; the code block holding each of its bits by the packet's block starts
__global__ void __launch_bounds__(256) fec_pack_kernel(FecPackArgs A) {
    const uint8_t* scr = A.ebits;
    for (uint32_t p = blockIdx.y; p < A.n; p += gridDim.y) {  // packets grid-stride: any n
        const uint32_t G = A.G[p], nb = (G + 7) / 8, c0 = A.cb_first[p], c1 = A.cb_first[p + 1];
        for (uint32_t B = blockIdx.x * blockDim.x + threadIdx.x; B < nb; B += gridDim.x * blockDim.x) {
            const uint32_t j0 = 8 * B;
            uint32_t lo = c0, hi = c1 - 1;  // last block starting at or before j0
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (A.pstart[mid] <= j0) lo = mid;
                else hi = mid - 1;
            }
            uint32_t r = lo;
            const uint32_t end = r + 1 < c1 ? A.pstart[r + 1] : G;
            uint32_t v;
            if ((A.pstart[r] & 7u) == 0 && j0 + 8 <= end) {  // whole byte of one block, byte-aligned
                v = scr[(A.oo[r] + (j0 - A.pstart[r])) >> 3];
            } else {
                v = 0;
                for (uint32_t t = 0; t < 8; ++t) {
                    const uint32_t j = j0 + t;
                    uint32_t bit = 0;
                    if (j < G) {
                        while (r + 1 < c1 && j >= A.pstart[r + 1]) ++r;
                        const uint64_t q = A.oo[r] + (j - A.pstart[r]);
                        bit = (scr[q >> 3] >> (7u - (q & 7u))) & 1u;
                    }
                    v = (v << 1) | bit;
                }
            }
            A.d[(size_t)p * A.d_stride + B] = (uint8_t)v;
        }
    }
}

int launch_fec_encode(const FecEncArgs& a, uint32_t n_cb, hipStream_t s) {
    if (n_cb == 0) return 0;
    hipLaunchKernelGGL(fec_encode_kernel, dim3((n_cb + FEC_ENC_WAVES - 1) / FEC_ENC_WAVES), dim3(64 * FEC_ENC_WAVES), 0, s,
                       a, n_cb);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_fec_pack(const FecPackArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    const uint32_t gx = (a.max_bytes + 255) / 256 < 256 ? (a.max_bytes + 255) / 256 : 256;
    hipLaunchKernelGGL(fec_pack_kernel, dim3(gx > 0 ? gx : 1, a.n < 65535u ? a.n : 65535u), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// continuation gather: the soft streams, decoder 2's extrinsic and the tails of the undecided code
// blocks, [k][old lane] of their old waves -> [k][new lane] of dense new waves of the same size
__global__ void __launch_bounds__(256) fec_compact_kernel(FecCompactArgs A) {
    const FecWave w = A.dst_waves[blockIdx.x];
    const uint32_t l = threadIdx.x & 63u, r = threadIdx.x >> 6, K = w.K;
    if (l >= w.n) return;
    const uint32_t so = A.src_of[w.first_cb + l], sw = so >> 6, sl = so & 63u;
    const FecWave ow = A.src_waves[sw];
    const int16_t* src = A.src16 + ow.data_off;
    int16_t* dst = A.dst16 + w.data_off;
    for (uint32_t k = r; k < K; k += 4) {
#pragma unroll
        for (int st = 0; st < 5; ++st) {
            if (st == 3) continue;  // decoder 1's extrinsic is recomputed
            dst[(size_t)st * K * 64 + (size_t)k * 64 + l] = src[(size_t)st * K * 64 + (size_t)k * 64 + sl];
        }
    }
    if (r == 0)
        for (int t = 0; t < 12; ++t)
            A.dst_tail[(size_t)blockIdx.x * 12 * 64 + t * 64 + l] = A.src_tail[(size_t)sw * 12 * 64 + t * 64 + sl];
}

int launch_fec_compact(const FecCompactArgs& a, uint32_t n_waves, hipStream_t s) {
    if (n_waves == 0) return 0;
    hipLaunchKernelGGL(fec_compact_kernel, dim3(n_waves), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_fec_dematch(const FecArgs& a, hipStream_t s) {
    if (a.n_cb == 0) return 0;
    hipLaunchKernelGGL(fec_dematch_kernel, dim3(a.n_waves), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_fec_tdec(const FecArgs& a, uint32_t n_waves, hipStream_t s) {
    if (n_waves == 0) return 0;
    hipLaunchKernelGGL(fec_tdec_kernel, dim3(n_waves), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_fec_tbcrc(const FecTbArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    hipLaunchKernelGGL(fec_tbcrc_kernel, dim3(a.n), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dnrp::dev
