// Batched turbo decoding of PDC code blocks on gfx950 (see fec_dev.hpp). Three kernels:
//   fec_dematch_kernel  workgroup = wave of code blocks: rate de-matching (srsran_rm_turbo_rx_lut_ role,
//                       pdc_enc.cpp:359-360) straight into the wave's [k][lane] soft streams
//   fec_tdec_kernel     wavefront = up to 64 code blocks of one size K, lane = code block: the
//                       iterations of the host decoder (fec.cpp Tdec / map_decode) with CRC early stop
//   fec_tbcrc_kernel    wavefront = packet with C > 1: transport-block CRC24A (pdc_enc.cpp:478-488),
//                       segment CRCs per lane joined by GF(2) shifts
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

// GF(2)[x] / CRC24A helpers for joining segment CRCs: crc(A || B) = crc(A) x^{|B|} + crc(B)
__device__ __forceinline__ uint32_t mulmod24(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 23; i >= 0; --i) {
        const uint32_t top = (r >> 23) & 1;
        r = (r << 1) & 0xFFFFFF;
        if (top) r ^= 0x864CFB;
        if ((b >> i) & 1) r ^= a;
    }
    return r;
}
__device__ uint32_t xpow24(uint64_t n) {  // x^n mod g
    uint32_t r = 1, b = 2;  // 1 and x
    while (n) {
        if (n & 1) r = mulmod24(r, b);
        b = mulmod24(b, b);
        n >>= 1;
    }
    return r;
}

__global__ void __launch_bounds__(64) fec_tbcrc_kernel(FecTbArgs A) {
    const uint32_t p = blockIdx.x, l = threadIdx.x;
    const uint8_t* d = A.tb + A.tb_off[p];
    const uint32_t nb = A.nbytes[p], seg = (nb + 63) / 64;
    const uint32_t lo = min(nb, l * seg), hi = min(nb, lo + seg);
    uint32_t reg = 0;
    for (uint32_t i = lo; i < hi; ++i) {
        const uint32_t byte = d[i];
        for (int t = 7; t >= 0; --t) {
            const uint32_t top = (reg >> 23) & 1;
            reg = (reg << 1) & 0xFFFFFF;
            if (top ^ ((byte >> t) & 1)) reg ^= 0x864CFB;
        }
    }
    __shared__ uint32_t part[64];
    part[l] = reg;
    __syncthreads();
    if (l == 0) {
        uint32_t crc = 0;
        for (uint32_t j = 0; j < 64; ++j) {
            const uint32_t a = min(nb, j * seg), b = min(nb, a + seg);
            if (b > a) crc = mulmod24(crc, xpow24(8ull * (b - a))) ^ part[j];
        }
        if (A.crc_out) {
            A.crc_out[p] = crc;
        } else {
            const uint32_t rx = ((uint32_t)d[nb] << 16) | ((uint32_t)d[nb + 1] << 8) | d[nb + 2];
            A.ok[p] = crc == rx;
        }
    }
}

// ---- encoder (fec.cpp dnrp_pdc_encode: pdc_enc.cpp:148-229) ---------------------------------------
// wavefront = up to 64 code blocks of one size, lane = code block: b bits -> CRC24B -> both
// constituent encoders (the second on the QPP rows, addresses by the scalar recurrence) with trellis
// termination -> rate matching into the unpacked bit scratch
__global__ void __launch_bounds__(64) fec_encode_kernel(FecEncArgs A) {
    const FecWave w = A.waves[blockIdx.x];
    const uint32_t l = threadIdx.x, K = w.K, D = K + 4;
    const bool active = l < w.n;
    const FecEncCb cb = A.cbs[w.first_cb + (active ? l : 0)];
    uint8_t* c = A.cd + w.data_off;
    uint8_t* d0 = c + (size_t)K * 64;
    uint8_t* d1 = d0 + (size_t)D * 64;
    uint8_t* d2 = d1 + (size_t)D * 64;
    const uint8_t* tb = A.tb + cb.tb_off;
    uint32_t tcrc;
    if (cb.crc16) {  // PLCF CRC16 over its 40 / 80 bits, masked (closed loop / beamforming)
        uint32_t r16 = 0;
        for (uint32_t pos = 0; pos < cb.tbs; ++pos) {
            const uint32_t top = (r16 >> 15) & 1u;
            r16 = (r16 << 1) & 0xFFFFu;
            if (top ^ ((tb[pos >> 3] >> (7 - (pos & 7))) & 1u)) r16 ^= 0x1021u;
        }
        tcrc = r16 ^ cb.mask;
    } else {
        tcrc = A.tbcrc[cb.pkt];
    }
    const uint32_t tcrc_top = cb.crc16 ? 15u : 23u;
    // c = b[rp, rp + rlen) (+ CRC24B), encoder 1 on the fly
    uint32_t reg = 0, s1 = 0, s2 = 0, s3 = 0, byte = 0;
    for (uint32_t k = 0; k < K; ++k) {
        uint32_t bit;
        if (k < cb.rlen) {
            const uint32_t pos = cb.rp + k;
            if ((k == 0 || (pos & 7) == 0) && pos < cb.tbs) byte = tb[pos >> 3];  // one load per byte
            bit = pos < cb.tbs ? (byte >> (7 - (pos & 7))) & 1u : (tcrc >> (tcrc_top - (pos - cb.tbs))) & 1u;
            const uint32_t top = (reg >> 23) & 1u;
            reg = (reg << 1) & 0xFFFFFF;
            if (top ^ bit) reg ^= 0x800063;
        } else {
            bit = (reg >> (23 - (k - cb.rlen))) & 1u;  // the code-block CRC (crc24b blocks only)
        }
        c[(size_t)k * 64 + l] = (uint8_t)bit;
        d0[(size_t)k * 64 + l] = (uint8_t)bit;
        const uint32_t a = bit ^ s2 ^ s3;
        d1[(size_t)k * 64 + l] = (uint8_t)(a ^ s1 ^ s3);
        s3 = s2, s2 = s1, s1 = a;
    }
    uint32_t x1[3], z1[3];
    for (int t = 0; t < 3; ++t) {
        x1[t] = s2 ^ s3, z1[t] = s1 ^ s3;
        s3 = s2, s2 = s1, s1 = 0;
    }
    // encoder 2 on c[pi(i)] (each lane reads back only its own column)
    const Qpp q{K, w.f1, w.f2};
    uint32_t pi = 0, dl = q.delta(0);
    const uint32_t f2x2 = 2 * w.f2 % K;
    s1 = s2 = s3 = 0;
    for (uint32_t i = 0; i < K; ++i) {
        const uint32_t a = c[(size_t)pi * 64 + l] ^ s2 ^ s3;
        d2[(size_t)i * 64 + l] = (uint8_t)(a ^ s1 ^ s3);
        s3 = s2, s2 = s1, s1 = a;
        pi += dl;
        pi = pi >= K ? pi - K : pi;
        dl += f2x2;
        dl = dl >= K ? dl - K : dl;
    }
    uint32_t x2[3], z2[3];
    for (int t = 0; t < 3; ++t) {
        x2[t] = s2 ^ s3, z2[t] = s1 ^ s3;
        s3 = s2, s2 = s1, s1 = 0;
    }
    // tails (TS 36.212 §5.1.3.2.2; fec.cpp turbo_encode)
    const uint32_t t0[4] = {x1[0], z1[1], x2[0], z2[1]}, t1[4] = {z1[0], x1[2], z2[0], x2[2]},
                   t2[4] = {x1[1], z1[2], x2[1], z2[2]};
    for (int t = 0; t < 4; ++t) {
        d0[(size_t)(K + t) * 64 + l] = (uint8_t)t0[t];
        d1[(size_t)(K + t) * 64 + l] = (uint8_t)t1[t];
        d2[(size_t)(K + t) * 64 + l] = (uint8_t)t2[t];
    }
    if (!active) return;
    // rate matching: bit j <- circular-buffer list entry (start + j) mod 3 (K + 4)
    const uint32_t* valid = A.tab + w.valid_off;
    const uint32_t nvalid = 3 * D;
    uint8_t* e = A.ebits + cb.e_off;
    uint32_t qv = cb.start;
    for (uint32_t j = 0; j < cb.E; ++j) {
        const uint32_t ent = valid[qv], st = ent >> 16, idx = ent & 0xFFFF;
        e[j] = d0[(size_t)st * D * 64 + (size_t)idx * 64 + l];
        if (++qv == nvalid) qv = 0;
    }
}

__global__ void __launch_bounds__(256) fec_pack_kernel(FecPackArgs A) {
    for (uint32_t p = blockIdx.y; p < A.n; p += gridDim.y) {  // packets grid-stride: any n
        const uint32_t G = A.G[p], nb = (G + 7) / 8;
        const uint8_t* e = A.ebits + A.e_off[p];
        for (uint32_t B = blockIdx.x * blockDim.x + threadIdx.x; B < nb; B += gridDim.x * blockDim.x) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) v = (v << 1) | (8 * B + t < G ? e[8 * B + t] : 0u);
            A.d[(size_t)p * A.d_stride + B] = (uint8_t)v;
        }
    }
}

int launch_fec_encode(const FecEncArgs& a, uint32_t n_waves, hipStream_t s) {
    if (n_waves == 0) return 0;
    hipLaunchKernelGGL(fec_encode_kernel, dim3(n_waves), dim3(64), 0, s, a);
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
