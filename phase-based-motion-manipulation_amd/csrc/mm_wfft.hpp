// mm_wfft.hpp — one-wavefront Stockham FFT (gfx950, wave64), no workgroup barriers.
//
// One length-N complex sequence per WAVE: lane l holds v[m] = x[l + 64 m],
// m = 0..P-1 (P = N/64), before and after fft<>().  That layout is coalesced
// for global loads/stores of a column or row (64 lanes x 8 B per m).
//
// Passes are radix R0 = min(16, P) (radix 16 = 4x4 in registers) plus one
// remainder pass; N = 2048 runs 16*16*8 with two LDS exchanges (the
// workgroup-per-sequence FFT of mm_fft.hpp needs three, each with two
// __syncthreads).  A pass of radix R handles Q = P/R butterflies per lane,
// j = l + 64 q, whose inputs x[j + t*N/R] are registers q + Q*t; Stockham-style
// it writes y[(j/Ns)*Ns*R + j%Ns + t*Ns].  The last pass writes j + t*N/R,
// i.e. register q + Q*t again: no final LDS trip.
//
// Exchanges go through a per-wave LDS buffer in E phases of N/E entries: phase
// e writes the outputs of butterflies q in [eQ/E, (e+1)Q/E) (they land in
// [eN/E, (e+1)N/E)) and reads registers m in [eP/E, (e+1)P/E).  E = 2 halves
// the buffer (8.7 KB at N = 2048), doubling the waves LDS admits per CU.
// LDS ops of one wave execute in order, so a wave-level fence/barrier (a code
// motion barrier, no s_barrier) is all the synchronisation there is.
#pragma once
#include "mm_fft.hpp"

namespace mm {
namespace wf {

constexpr int ilog2(int x)
{
    int r = 0;
    while ((1 << r) < x) ++r;
    return r;
}

template <int LOG2N> struct Plan {
    static constexpr int N = 1 << LOG2N;
    static constexpr int P = N / 64;                               // points per lane
    static constexpr int RB = ilog2(P) < 4 ? ilog2(P) : 4;         // log2 main radix
    static constexpr int R0 = 1 << RB;
    static constexpr int NFULL = LOG2N / RB;                       // full-radix passes
    static constexpr int NP = NFULL + (LOG2N % RB ? 1 : 0);        // passes
    static constexpr int radix(int p) { return p < NFULL ? R0 : (1 << (LOG2N % RB)); }
    static constexpr int ns(int p) { return p == 0 ? 1 : ns(p - 1) * radix(p - 1); }
    // twiddle bases of pass p: one if its Ns <= 64 (r = lane & (Ns-1) for every q)
    static constexpr int nbase(int p) { return p == 0 ? 0 : (ns(p) <= 64 ? 1 : P / radix(p)); }
    static constexpr int base_slot(int p) { return p == 0 ? 0 : base_slot(p - 1) + nbase(p - 1); }
    static constexpr int NBASE = base_slot(NP);
    // largest E (<= cap) dividing Q of every pass that exchanges
    static constexpr int max_phases(int cap)
    {
        int e = cap;
        for (int p = 0; p + 1 < NP; ++p)
            while (e > 1 && (P / radix(p)) % e) e /= 2;
        return e;
    }
};

template <int LOG2N> constexpr int pad_shift() { return Plan<LOG2N>::RB; }
// one complex of padding every R0 entries: minimal (2-way, ds_*_b64) bank
// conflicts for the Ns = 1 and Ns = R0 write patterns and the l + 64 m reads
template <int LOG2N> __device__ __forceinline__ int pad(int i) { return i + (i >> pad_shift<LOG2N>()); }
template <int LOG2N, int E> constexpr int buf_complex()
{
    return (1 << LOG2N) / E + (1 << LOG2N) / E / Plan<LOG2N>::R0;
}

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// W16^e * a, W16 = exp(DIR * 2*pi*i / 16), e in {1,2,3,4,6,9}
template <int DIR, int EXP>
__device__ __forceinline__ c2 rot16(c2 a)
{
    constexpr float C = 0.92387953251128674f, S = 0.38268343236508977f, H = 0.70710678118654752f;
    constexpr float cr = EXP == 1 ? C : EXP == 2 ? H : EXP == 3 ? S : EXP == 4 ? 0.0f
                       : EXP == 6 ? -H : -C;
    constexpr float si = EXP == 1 ? S : EXP == 2 ? H : EXP == 3 ? C : EXP == 4 ? 1.0f
                       : EXP == 6 ? H : -S;
    if constexpr (EXP == 4) return mul_i<DIR>(a);
    else return mul_p(a, c2{cr, DIR * si}, c2{-DIR * si, cr});
}

// 16-point DFT, natural order in and out: 4 x DFT4, twiddles W16^(n2 k1), 4 x DFT4.
template <int DIR>
__device__ __forceinline__ void dft16(c2 *u)
{
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4<DIR>(u[n2], u[n2 + 4], u[n2 + 8], u[n2 + 12]);
    // u[n2 + 4 k1] = a[n2][k1]
    u[5] = rot16<DIR, 1>(u[5]);
    u[9] = rot16<DIR, 2>(u[9]);
    u[13] = rot16<DIR, 3>(u[13]);
    u[6] = rot16<DIR, 2>(u[6]);
    u[10] = rot16<DIR, 4>(u[10]);
    u[14] = rot16<DIR, 6>(u[14]);
    u[7] = rot16<DIR, 3>(u[7]);
    u[11] = rot16<DIR, 6>(u[11]);
    u[15] = rot16<DIR, 9>(u[15]);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) dft4<DIR>(u[4 * k1], u[4 * k1 + 1], u[4 * k1 + 2], u[4 * k1 + 3]);
    // u[4 k1 + k2] = X[k1 + 4 k2]: transpose the 4x4 register tile
    c2 t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = u[i];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) u[k1 + 4 * k2] = t[4 * k1 + k2];
}

template <int R, int DIR>
__device__ __forceinline__ void dft(c2 *u)
{
    if constexpr (R == 16) dft16<DIR>(u);
    else if constexpr (R == 8) dft8<DIR>(u);
    else if constexpr (R == 4) dft4<DIR>(u[0], u[1], u[2], u[3]);
    else dft2<DIR>(u[0], u[1]);
}

// Twiddle bases of every pass, issued up front (latency hides under pass 0).
template <int LOG2N, int DIR, int PI = 1>
__device__ __forceinline__ void load_bases(c2 *wb, int lane, const c2 *__restrict__ tw)
{
    using PL = Plan<LOG2N>;
    if constexpr (PI < PL::NP) {
        constexpr int NS = PL::ns(PI), R = PL::radix(PI);
        constexpr int stride = PL::N / (NS * R);   // table stride of W_{NS*R}
        constexpr int NB = PL::nbase(PI), SLOT = PL::base_slot(PI);
#pragma unroll
        for (int q = 0; q < NB; ++q)
            wb[SLOT + q] = twiddle<DIR>(tw, ((lane + 64 * q) & (NS - 1)) * stride);
        load_bases<LOG2N, DIR, PI + 1>(wb, lane, tw);
    }
}

template <int LOG2N, int DIR, int E, int PI>
__device__ __forceinline__ void pass(c2 (&v)[Plan<LOG2N>::P], int lane, c2 *buf, const c2 *wb)
{
    using PL = Plan<LOG2N>;
    constexpr int N = PL::N, P = PL::P, R = PL::radix(PI), NS = PL::ns(PI), Q = P / R;
    constexpr bool LAST = PI == PL::NP - 1;
    constexpr int SLOT = PL::base_slot(PI);
    c2 o[P];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        // one butterfly at a time: stops the scheduler from hoisting every
        // butterfly's twiddle powers (that alone cost ~60 VGPRs at N = 2048)
        __builtin_amdgcn_sched_barrier(0);
        c2 u[R];
#pragma unroll
        for (int t = 0; t < R; ++t) u[t] = v[q + Q * t];
        if constexpr (NS > 1) apply_twiddles<R>(u, wb[SLOT + (NS <= 64 ? 0 : q)]);
        dft<R, DIR>(u);
#pragma unroll
        for (int t = 0; t < R; ++t) {
            if constexpr (LAST) v[q + Q * t] = u[t];
            else o[q * R + t] = u[t];
        }
    }
    if constexpr (!LAST) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
#pragma unroll
            for (int q = e * Q / E; q < (e + 1) * Q / E; ++q) {
                const int j = lane + 64 * q;
                const int base = (j / NS) * NS * R + (j & (NS - 1)) - e * (N / E);
                // NS = 1: base is a multiple of R = R0, so pad(base + t) = pad(base) + t;
                // NS >= R0: NS t is a multiple of R0, so pad adds NS t / R0
                constexpr int step = NS == 1 ? 1 : NS + NS / PL::R0;
                c2 *row = buf + pad<LOG2N>(base);
#pragma unroll
                for (int t = 0; t < R; ++t) row[t * step] = o[q * R + t];
            }
            wave_sync();
            // pad(lane + 64 m) = pad(lane) + m (64 + 64 / R0)
            const c2 *col = buf + pad<LOG2N>(lane);
#pragma unroll
            for (int m = e * P / E; m < (e + 1) * P / E; ++m)
                v[m] = col[(m - e * P / E) * (64 + 64 / PL::R0)];
            wave_sync();
        }
    }
}

template <int LOG2N, int DIR, int E, int PI>
__device__ __forceinline__ void pass_loop(c2 (&v)[Plan<LOG2N>::P], int lane, c2 *buf, const c2 *wb)
{
    if constexpr (PI < Plan<LOG2N>::NP) {
        pass<LOG2N, DIR, E, PI>(v, lane, buf, wb);
        pass_loop<LOG2N, DIR, E, PI + 1>(v, lane, buf, wb);
    }
}

// Unnormalised DFT of the wave's sequence (DIR = -1 forward, +1 inverse).
// buf: buf_complex<LOG2N, E>() entries private to this wave.
template <int LOG2N, int DIR, int E>
__device__ __forceinline__ void fft(c2 (&v)[Plan<LOG2N>::P], int lane, c2 *buf,
                                    const c2 *__restrict__ tw)
{
    static_assert(Plan<LOG2N>::max_phases(E) == E, "E must divide every exchanging pass's Q");
    constexpr int NB = Plan<LOG2N>::NBASE > 0 ? Plan<LOG2N>::NBASE : 1;
    c2 wb[NB];
    load_bases<LOG2N, DIR>(wb, lane, tw);
    pass_loop<LOG2N, DIR, E, 0>(v, lane, buf, wb);
}

}  // namespace wf
}  // namespace mm
