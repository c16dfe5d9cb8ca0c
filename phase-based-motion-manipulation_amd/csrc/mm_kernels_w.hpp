// mm_kernels_w.hpp — wave-per-sequence variants of the FFT kernels (gfx950).
//
// Same math and data layout as mm_kernels.hpp; each length-N FFT is owned by
// ONE wavefront (mm_wfft.hpp: 32 points per lane at N = 2048, LDS exchanges
// synchronised at wave level), so no kernel here executes a workgroup barrier.
#pragma once
#include "mm_kernels.hpp"
#include "mm_wfft.hpp"

namespace mm {

// K2 runs at 2 waves/SIMD (F_{t-1} in registers), where LDS admits a full
// column buffer per wave (8 x 17.4 KB at N = 2048): E = 1 exchange phase.
template <int LOG2N> constexpr int k2_phases() { return 1; }
template <int LOG2N> constexpr int k2_waves_per_simd() { return LOG2N <= 9 ? 3 : 2; }

// =========================================================================
// K2 (wave form): column FFT -> spectral op vs F_{t-1} -> column IFFT -> Q
// =========================================================================
// Workgroup b = one wave = (column f = b mod N/2, sub-chunk s = b div N/2).
// Sub-chunk s owns frames [s*n/nsub, (s+1)*n/nsub) of the launch; it starts
// from F_{a-1}, recomputed from G[a-1] (one extra forward FFT: the state is a
// pure function of the previous INPUT frame), so the nsub waves
// of a column run independently.  F_{t-1} stays in registers across frames.
// Column f = 0 packs the two real-input columns 0 and N/2 as z = G0 + i GN
// (see k_cols); their spectra are Hermitian in fy, so only fy <= N/2 is
// carried and the rest mirrored.
template <int LOG2N>
__device__ __forceinline__ void load_column(c2 (&v)[wf::Plan<LOG2N>::P], const c2 *Gc,
                                            const c2 *GN, int lane, const Geo &g, bool packed)
{
    constexpr int P = wf::Plan<LOG2N>::P;
#pragma unroll
    for (int m = 0; m < P; ++m) {   // unconditional clamped loads, then select
        const int rr = lane + 64 * m - g.y0;
        const int rc = min(max(rr, 0), g.H - 1);
        const c2 a = Gc[rc];
        const float bn = packed ? GN[rc].x : 0.0f;
        const bool in = rr >= 0 && rr < g.H;
        v[m] = in ? (packed ? mk(a.x, bn) : a) : mk(0.0f, 0.0f);
    }
}

// Z = F0 + i FN (natural layout in v) -> all of Z to buf, then per bin
// fy < N/2 (m < P/2): F0 = (Z + conj Zm)/2, FN = (Z - conj Zm)/2i with
// Zm = Z[(N - fy) mod N] (fy = 0 pairs with itself); fy = N/2 (lane 0,
// m = P/2) is its own partner.  The caller syncs before reusing buf.
template <int LOG2N>
__device__ __forceinline__ void stash_pair(const c2 (&v)[wf::Plan<LOG2N>::P], int lane, c2 *buf)
{
    constexpr int P = wf::Plan<LOG2N>::P;
#pragma unroll
    for (int m = 0; m < P; ++m) buf[wf::pad<LOG2N>(lane + 64 * m)] = v[m];
    wf::wave_sync();
}
__device__ __forceinline__ void split_pair(c2 z, c2 zm, c2 &f0, c2 &fN)
{
    f0 = mk(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
    fN = mk(0.5f * (z.y + zm.y), -0.5f * (z.x - zm.x));
}
template <int LOG2N>
__device__ __forceinline__ c2 partner(int fy, const c2 *buf)
{
    constexpr int N = 1 << LOG2N;
    return buf[wf::pad<LOG2N>((N - fy) & (N - 1))];
}

// Frame range of one wave and where its F_{t-1} comes from.
struct K2Range {
    int fa, fb;      // frames [fa, fb) of the launch
    int first;       // first frame that produces output
    int src;         // G frame whose spectrum seeds F_{t-1}, or -1: state_in
};
__device__ __forceinline__ K2Range k2_range(int s, int nsub, int nframes, int first_passthrough)
{
    K2Range r;
    r.fa = s * nframes / nsub;
    r.fb = (s + 1) * nframes / nsub;
    r.first = r.fa;
    r.src = -1;
    if (s > 0) {
        r.src = r.fa - 1;                 // sub-chunk > 0: F_{a-1} from G[a-1]
    } else if (first_passthrough) {
        r.src = r.fa;                     // passthrough frame: F_a only, no output
        r.first = r.fa + 1;
    }
    return r;
}

// Ordinary column f (1 <= f < N/2).
template <int LOG2N, int MODE>
__device__ __forceinline__ void cols_plain(const c2 *__restrict__ G, size_t g_stride,
                                           c2 *__restrict__ Q, size_t q_stride,
                                           const c2 *state_in, c2 *state_out, int f, K2Range r,
                                           bool last, const Geo &g, const Spec &sp,
                                           const c2 *__restrict__ tw, c2 *buf)
{
    using PL = wf::Plan<LOG2N>;
    constexpr int N = PL::N, P = PL::P, E = k2_phases<LOG2N>();
    const int lane0 = threadIdx.x;
    const c2 *G0 = G + (size_t)f * g.H;
    c2 pv[P];   // F_{t-1}[fy], fy = lane + 64 m
    if (r.src >= 0) {
        load_column<LOG2N>(pv, G0 + (size_t)r.src * g_stride, G0, lane0, g, false);
        wf::fft<LOG2N, -1, E>(pv, lane0, buf, tw);
    } else {
#pragma unroll
        for (int m = 0; m < P; ++m)
            pv[m] = state_in ? state_in[(size_t)f * N + lane0 + 64 * m] : mk(0.0f, 0.0f);
    }
    for (int fr = r.first; fr < r.fb; ++fr) {
        // opaque per-iteration lane index: keeps LICM from hoisting every
        // lane-derived address and twiddle of both FFTs out of the frame loop
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        c2 v[P];
        load_column<LOG2N>(v, G0 + (size_t)fr * g_stride, G0, lane, g, false);
        wf::fft<LOG2N, -1, E>(v, lane, buf, tw);
#pragma unroll
        for (int m = 0; m < P; ++m) {
            // one bin at a time: keeps the op instances from being interleaved
            __builtin_amdgcn_sched_barrier(0);
            const c2 a = spectral_op<LOG2N, MODE>(v[m], pv[m], f, lane + 64 * m, sp);
            pv[m] = v[m];
            v[m] = a;
        }
        __builtin_amdgcn_sched_barrier(0);
        wf::fft<LOG2N, +1, E>(v, lane, buf, tw);
        c2 *Qc = Q + (size_t)fr * q_stride;   // pair-interleaved Q (q_index)
#pragma unroll
        for (int m = 0; m < P; ++m) {
            const int k = (lane + 64 * m - g.rb + 2 * N) & (N - 1);
            if (k < g.Hn) Qc[q_index(g, k, f)] = v[m];
        }
    }
    if (last) {
        c2 *S0 = state_out + (size_t)f * N;
#pragma unroll
        for (int m = 0; m < P; ++m) S0[lane0 + 64 * m] = pv[m];
    }
}

// The real-input columns 0 and N/2 as one complex column z = G0 + i GN.
template <int LOG2N, int MODE>
__device__ __forceinline__ void cols_packed(const c2 *__restrict__ G, size_t g_stride,
                                            c2 *__restrict__ Q, size_t q_stride,
                                            const c2 *state_in, c2 *state_out, K2Range r,
                                            bool last, const Geo &g, const Spec &sp,
                                            const c2 *__restrict__ tw, c2 *buf)
{
    using PL = wf::Plan<LOG2N>;
    constexpr int N = PL::N, P = PL::P, H = P / 2, E = k2_phases<LOG2N>();
    const int lane0 = threadIdx.x;
    const c2 *G0 = G, *GN = G + (size_t)(N / 2) * g.H;
    // pv[m] = F0_{t-1}[fy], pv[m + H] = FN_{t-1}[fy] for fy = lane + 64 m < N/2;
    // fy = N/2 of both in pm0/pmN (lane 0)
    c2 pv[P];
    c2 pm0 = mk(0.0f, 0.0f), pmN = mk(0.0f, 0.0f);
    if (r.src >= 0) {
        c2 v[P];
        load_column<LOG2N>(v, G0 + (size_t)r.src * g_stride, GN + (size_t)r.src * g_stride, lane0,
                           g, true);
        wf::fft<LOG2N, -1, E>(v, lane0, buf, tw);
        stash_pair<LOG2N>(v, lane0, buf);
#pragma unroll
        for (int m = 0; m < H; ++m)
            split_pair(v[m], partner<LOG2N>(lane0 + 64 * m, buf), pv[m], pv[m + H]);
        split_pair(v[H], v[H], pm0, pmN);
        wf::wave_sync();
    } else if (state_in) {
        const c2 *S0 = state_in, *SN = state_in + (size_t)(N / 2) * N;
#pragma unroll
        for (int m = 0; m < H; ++m) {
            pv[m] = S0[lane0 + 64 * m];
            pv[m + H] = SN[lane0 + 64 * m];
        }
        pm0 = S0[N / 2];
        pmN = SN[N / 2];
    } else {
#pragma unroll
        for (int m = 0; m < P; ++m) pv[m] = mk(0.0f, 0.0f);
    }
    for (int fr = r.first; fr < r.fb; ++fr) {
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        c2 v[P];
        load_column<LOG2N>(v, G0 + (size_t)fr * g_stride, GN + (size_t)fr * g_stride, lane, g,
                           true);
        wf::fft<LOG2N, -1, E>(v, lane, buf, tw);
        // A0 + i AN for fy < N/2 stays in registers; conj(A0) + i conj(AN) goes
        // to buf[fy] (the Z[fy] there was read by this lane already; the other
        // lanes read only the upper half), read back by bin N - fy.
        stash_pair<LOG2N>(v, lane, buf);
#pragma unroll
        for (int m = 0; m < H; ++m) {
            __builtin_amdgcn_sched_barrier(0);
            const int fy = lane + 64 * m;
            c2 f0, fN;
            split_pair(v[m], partner<LOG2N>(fy, buf), f0, fN);
            const c2 a0 = spectral_op<LOG2N, MODE>(f0, pv[m], 0, fy, sp);
            const c2 an = spectral_op<LOG2N, MODE>(fN, pv[m + H], N / 2, fy, sp);
            pv[m] = f0;
            pv[m + H] = fN;
            v[m] = mk(a0.x - an.y, a0.y + an.x);
            buf[wf::pad<LOG2N>(fy)] = mk(a0.x + an.y, an.x - a0.y);
        }
        __builtin_amdgcn_sched_barrier(0);
        c2 mid0, midN;
        split_pair(v[H], v[H], mid0, midN);
        const c2 a0m = spectral_op<LOG2N, MODE>(mid0, pm0, 0, N / 2, sp);
        const c2 anm = spectral_op<LOG2N, MODE>(midN, pmN, N / 2, N / 2, sp);
        pm0 = mid0;
        pmN = midN;
        wf::wave_sync();
#pragma unroll
        for (int m = H; m < P; ++m) {
            const int fy = lane + 64 * m;   // > N/2 except lane 0, m = H
            const c2 w = buf[wf::pad<LOG2N>(fy == N / 2 ? 0 : N - fy)];
            v[m] = fy == N / 2 ? mk(a0m.x - anm.y, a0m.y + anm.x) : w;
        }
        wf::wave_sync();
        wf::fft<LOG2N, +1, E>(v, lane, buf, tw);
        c2 *Qc = Q + (size_t)fr * q_stride;   // pair-interleaved Q (q_index)
#pragma unroll
        for (int m = 0; m < P; ++m) {   // inverse of A0 + i AN: real parts Q0 + i QN
            const int k = (lane + 64 * m - g.rb + 2 * N) & (N - 1);
            if (k < g.Hn) {
                Qc[q_index(g, k, 0)] = mk(v[m].x, 0.0f);
                Qc[q_index(g, k, N / 2)] = mk(v[m].y, 0.0f);
            }
        }
    }
    if (last) {   // full Hermitian columns: F[N - fy] = conj F[fy] (bitwise, see split_pair)
        c2 *S0 = state_out, *SN = state_out + (size_t)(N / 2) * N;
#pragma unroll
        for (int m = 0; m < H; ++m) {
            const int fy = lane0 + 64 * m;
            S0[fy] = pv[m];
            SN[fy] = pv[m + H];
            if (fy > 0) {
                S0[N - fy] = mk(pv[m].x, -pv[m].y);
                SN[N - fy] = mk(pv[m + H].x, -pv[m + H].y);
            }
        }
        if (lane0 == 0) {
            S0[N / 2] = pm0;
            SN[N / 2] = pmN;
        }
    }
}

template <int LOG2N, int MODE>
__global__ __launch_bounds__(64, k2_waves_per_simd<LOG2N>())
void k_cols_w(const c2 *__restrict__ G, size_t g_stride, c2 *__restrict__ Q, size_t q_stride,
              const c2 *state_in, c2 *state_out, int nframes, int first_passthrough, int nsub,
              Geo g, Spec sp, const c2 *__restrict__ tw)
{
    constexpr int N = 1 << LOG2N;
    __shared__ c2 buf[wf::buf_complex<LOG2N, k2_phases<LOG2N>()>()];
    const int f = blockIdx.x % (N / 2), s = blockIdx.x / (N / 2);
    const K2Range r = k2_range(s, nsub, nframes, first_passthrough);
    if (f == 0)
        cols_packed<LOG2N, MODE>(G, g_stride, Q, q_stride, state_in, state_out, r, s == nsub - 1,
                                 g, sp, tw, buf);
    else
        cols_plain<LOG2N, MODE>(G, g_stride, Q, q_stride, state_in, state_out, f, r,
                                s == nsub - 1, g, sp, tw, buf);
}

}  // namespace mm
