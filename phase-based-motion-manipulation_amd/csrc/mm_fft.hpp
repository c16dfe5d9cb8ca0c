// mm_fft.hpp — register/LDS Stockham FFT for one length-N complex sequence per
// "FFT group" of T = N/8 threads (gfx950, wave64).
//
// Replaces the reference's per-stage radix-2 dispatches (FFT.compute:213-276,
// driven 11+11 times per 2D FFT from MotionMagnificationProcessor.cs:522-549)
// with log8(N) register passes and LDS exchanges inside one kernel.
//
// Layout contract ("L0"): thread t of the group holds v[j] = x[t + j*T],
// j = 0..7, both before and after fft_regs<>().  A pass of radix R processes
// B = 8/R butterflies per thread; butterfly b = t + q*T reads x[b + m*N/R]
// (= register q + m*B) and, Stockham-style, writes y[(b/Ns)*Ns*R + b%Ns + m*Ns].
// After the last pass (Ns*R == N) that index is t + (q+m*B)*T, i.e. register
// q + m*B again, so the result stays in registers with no final LDS trip.
#pragma once
#include <hip/hip_runtime.h>

namespace mm {

// Complex value: a 2 x f32 vector, so that it lives in an aligned VGPR pair
// and the complex arithmetic issues as packed FP32 (VOP3P v_pk_add_f32 /
// v_pk_mul_f32 / v_pk_fma_f32: two lanes' worth of f32 work per wave64
// instruction at the issue cost of one scalar v_fma_f32 — 4.2 cycles per
// wave-instruction either way, profiles/r02_valu_calib.json).  Plain sums and
// differences use the vector operators (the compiler emits v_pk_add_f32 with
// neg modifiers); products and the +-i rotations, whose operands must be
// swizzled, are written as single VOP3P instructions with op_sel / neg
// modifiers (the compiler's own lowering of those swizzles adds v_pk_mov and
// negations).
typedef float c2 __attribute__((ext_vector_type(2)));

__host__ __device__ __forceinline__ c2 mk(float x, float y) { c2 r = {x, y}; return r; }
__device__ __forceinline__ c2 add(c2 a, c2 b) { return a + b; }
__device__ __forceinline__ c2 sub(c2 a, c2 b) { return a - b; }
__device__ __forceinline__ c2 scale(c2 a, float s) { return a * s; }

// x + i*DIR*y: DIR = +1 -> (x.x - y.y, x.y + y.x); DIR = -1 -> (x.x + y.y, x.y - y.x)
template <int DIR>
__device__ __forceinline__ c2 add_i(c2 x, c2 y)
{
    c2 d;
    if constexpr (DIR > 0)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(d) : "v"(x), "v"(y));
    else
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(x), "v"(y));
    return d;
}
// x - i*DIR*y
template <int DIR>
__device__ __forceinline__ c2 sub_i(c2 x, c2 y) { return add_i<-DIR>(x, y); }

// a * w = (ax wx - ay wy, ax wy + ay wx): t = (ax wx, ax wy), then
// d = (-ay wy + t.x, ay wx + t.y)
__device__ __forceinline__ c2 mul(c2 a, c2 w)
{
    c2 t, d;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
        : "=v"(d) : "v"(a), "v"(w), "v"(t));
    return d;
}
// a * w in plain C, for the spectral ops: their factors come straight from
// transcendental instructions (v_sin/v_cos), and a transcendental result read
// by the next instruction needs a wait state that the compiler inserts for
// its own instructions but not in front of inline asm (an asm mul() there read
// stale values on gfx950).  The FFT's asm operands come from loads and plain
// VALU results only.
__device__ __forceinline__ c2 mul_c(c2 a, c2 w)
{
    return mk(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}
// a * conj(w) = (ax wx + ay wy, ay wx - ax wy): the inverse FFT's twiddles
// from the forward bases without a conjugated copy
__device__ __forceinline__ c2 mul_conj(c2 a, c2 w)
{
    c2 t, d;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[0,0,1]"
        : "=v"(d) : "v"(a), "v"(w), "v"(t));
    return d;
}
// a * w^DIR-convention: the forward (DIR < 0) FFT multiplies by the table's
// W_N^k, the inverse by its conjugate
template <int DIR>
__device__ __forceinline__ c2 mul_tw(c2 a, c2 w) { return DIR < 0 ? mul(a, w) : mul_conj(a, w); }

// LDS read of one complex value that the backend must not pair with another
// into ds_read2_b64: on gfx950 a ds_read2_b64 takes 8 LDS cycles per
// wave-instruction (two accesses in 4 x 16-lane groups over 32 banks) where
// two ds_read_b64 take 4 (2 x 32 lanes over 64 banks; MI355X_MICROARCH.md
// §LDS), and the exchange reads are the FFTs' LDS-bound part.  A volatile
// access is never merged (SILoadStoreOptimizer skips ordered references).
#ifndef MM_LDS_NOPAIR
#define MM_LDS_NOPAIR 1
#endif
__device__ __forceinline__ c2 lds_ld(const c2 *p)
{
    if constexpr (MM_LDS_NOPAIR) {
        typedef __attribute__((address_space(3))) const volatile c2 lds_vc2;
        return *(lds_vc2 *)(p);   // (generic -> LDS address space: a ds_read_b64)
    } else {
        return *p;
    }
}

// LDS index padding: one complex every 8 (bank-conflict-free Stockham writes
// for Ns = 1 and Ns = 8 with ds_write_b64).
__device__ __forceinline__ int pad8(int i) { return i + (i >> 3); }
template <int N> constexpr int lds_complex() { return N + N / 8; }

template <int DIR>
__device__ __forceinline__ void dft2(c2 &a, c2 &b)
{
    c2 t = a;
    a = add(t, b);
    b = sub(t, b);
}

template <int DIR>
__device__ __forceinline__ void dft4(c2 &x0, c2 &x1, c2 &x2, c2 &x3)
{
    const c2 s0 = x0 + x2, d0 = x0 - x2;
    const c2 s1 = x1 + x3, t = x1 - x3;
    x0 = s0 + s1;
    x2 = s0 - s1;
    x1 = add_i<DIR>(d0, t);
    x3 = sub_i<DIR>(d0, t);
}

template <int DIR>
__device__ __forceinline__ void dft8(c2 *v)
{
    constexpr float h = 0.70710678118654752f;
    c2 a0 = v[0] + v[4], b0 = v[0] - v[4];
    c2 a1 = v[1] + v[5], b1 = v[1] - v[5];
    c2 a2 = v[2] + v[6], b2 = v[2] - v[6];
    c2 a3 = v[3] + v[7], b3 = v[3] - v[7];
    // b[n] *= W8^n, W8 = exp(DIR*i*pi/4) = h (1 + i DIR); W8^2 = i*DIR folds into
    // the DFT4 below, W8^3 = h (-1 + i DIR) = -h (b - i DIR b) / b
    b1 = add_i<DIR>(b1, b1) * h;
    b3 = sub_i<DIR>(b3, b3) * (-h);
    dft4<DIR>(a0, a1, a2, a3);
    // DFT4 of (b0, b1, i DIR b2, b3)
    const c2 s0 = add_i<DIR>(b0, b2), d0 = sub_i<DIR>(b0, b2);
    const c2 s1 = b1 + b3, t = b1 - b3;
    v[0] = a0; v[2] = a1; v[4] = a2; v[6] = a3;
    v[1] = s0 + s1;
    v[5] = s0 - s1;
    v[3] = add_i<DIR>(d0, t);
    v[7] = sub_i<DIR>(d0, t);
}

// u[m] *= w^m (m < R, R <= 16) for the forward FFT (DIR < 0), u[m] *=
// conj(w)^m for the inverse: w is always the forward base, its powers are
// products (<= 4 roundings), and only the final multiply conjugates.
template <int R, int DIR>
__device__ __forceinline__ void apply_twiddles(c2 *u, c2 w1)
{
    if constexpr (R >= 2) u[1] = mul_tw<DIR>(u[1], w1);
    if constexpr (R >= 4) {
        const c2 w2 = mul(w1, w1);
        const c2 w3 = mul(w2, w1);
        u[2] = mul_tw<DIR>(u[2], w2);
        u[3] = mul_tw<DIR>(u[3], w3);
        if constexpr (R >= 8) {
            const c2 w4 = mul(w2, w2);
            u[4] = mul_tw<DIR>(u[4], w4);
            u[5] = mul_tw<DIR>(u[5], mul(w1, w4));
            u[6] = mul_tw<DIR>(u[6], mul(w2, w4));
            u[7] = mul_tw<DIR>(u[7], mul(w3, w4));
            if constexpr (R >= 16) {
                const c2 w8 = mul(w4, w4);
                u[8] = mul_tw<DIR>(u[8], w8);
                u[9] = mul_tw<DIR>(u[9], mul(w1, w8));
                u[10] = mul_tw<DIR>(u[10], mul(w2, w8));
                u[11] = mul_tw<DIR>(u[11], mul(w3, w8));
                const c2 w12 = mul(w4, w8);
                u[12] = mul_tw<DIR>(u[12], w12);
                u[13] = mul_tw<DIR>(u[13], mul(w1, w12));
                u[14] = mul_tw<DIR>(u[14], mul(w2, w12));
                u[15] = mul_tw<DIR>(u[15], mul(w3, w12));
            }
        }
    }
}

// The same multiplies with the powers w^1 .. w^7 of one radix-8 pass read from
// an LDS table (tw_tab_build: identical products, so identical values):
// p[k NS] holds (w^{2k+1}, w^{2k+2}), k = 0..3 (the last .zw unused).
template <int DIR, int NS>
__device__ __forceinline__ void apply_twiddles_tt(c2 *u, const float4 *p)
{
    const float4 a = p[0], b = p[NS], c = p[2 * NS], d = p[3 * NS];
    u[1] = mul_tw<DIR>(u[1], mk(a.x, a.y));
    u[2] = mul_tw<DIR>(u[2], mk(a.z, a.w));
    u[3] = mul_tw<DIR>(u[3], mk(b.x, b.y));
    u[4] = mul_tw<DIR>(u[4], mk(b.z, b.w));
    u[5] = mul_tw<DIR>(u[5], mk(c.x, c.y));
    u[6] = mul_tw<DIR>(u[6], mk(c.z, c.w));
    u[7] = mul_tw<DIR>(u[7], mk(d.x, d.y));
}

constexpr int fft_passes_v(int log2n) { return log2n / 3 + (log2n % 3 ? 1 : 0); }
// twiddle-base slots P*4 + q (preload_twiddles): 16 up to N = 4096 (4
// passes), 20 at N = 8192 (5 passes); unused slots are constant (1, 0) and
// compile away
constexpr int kTwSlots = 20;
template <int LOG2N> constexpr int fft_passes() { return fft_passes_v(LOG2N); }
constexpr int pass_radix_v(int log2n, int p) { return (p < log2n / 3) ? 8 : (log2n % 3 == 2 ? 4 : 2); }
template <int LOG2N, int P> constexpr int pass_radix() { return pass_radix_v(LOG2N, P); }
constexpr int pass_ns_v(int log2n, int p) { return p == 0 ? 1 : pass_ns_v(log2n, p - 1) * pass_radix_v(log2n, p - 1); }

// Twiddle buffer: the N-entry W_N table (tw_entries_v: kept as a function so
// the buffer layout has one definition).  A pass-table variant (each
// butterfly's powers loaded as one row) issued fewer VALU instructions but ran
// slower: its per-pass load latency sits on the short row kernels' critical
// path; powers are products of one preloaded base instead.
constexpr int tw_entries_v(int log2n) { return 1 << log2n; }

// Base twiddle W_{Ns R}^r of butterfly q of pass P (one load from the table
// tw[k] = exp(-2 pi i k / N)), for every pass, issued at FFT start so the
// latency hides under pass 0: slot P*4 + q.  Always the forward base: the
// inverse conjugates in its multiplies (mul_tw).
// TWST: stride of the table actually passed (a W_{N*TWST} table serves a
// length-N transform at indices times TWST).
template <int LOG2N, int P = 1, int TWST = 1>
__device__ __forceinline__ void preload_twiddles(c2 (&wb)[kTwSlots], int t, const c2 *__restrict__ tw)
{
    if constexpr (P < fft_passes<LOG2N>()) {
        constexpr int N = 1 << LOG2N, T = N / 8, R = pass_radix<LOG2N, P>(), B = 8 / R;
        constexpr int NS = pass_ns_v(LOG2N, P), TWS = N / (NS * R);
#pragma unroll
        for (int q = 0; q < B; ++q) wb[P * 4 + q] = tw[((t + q * T) & (NS - 1)) * TWS * TWST];
        preload_twiddles<LOG2N, P + 1, TWST>(wb, t, tw);
    }
}

// LDS layout of the exchange after pass P: index i lives at
// xpad(i) = i + A*(i >> S), chosen per pass (tools/lds_banks.py models the
// gfx950 bank rules: ds_write_b64 in 4 groups of 16 lanes over 32 banks,
// ds_read_b64 in 2 groups of 32 lanes over 64 banks).  Ns = 1 (8b + m
// writes): pad8, the only linear form without write conflicts (its reads
// stay 2-way on a few lanes); Ns = 8: A = 4, S = 5, conflict-free both ways;
// Ns >= 64: none needed.  Against pad8 on every pass: 1.11x instead of
// 1.56x the conflict-free LDS cycles at N = 512..4096.  Every layout fits
// N + N/8 entries (lds_complex), and xpad(base + off) = xpad(base) +
// xpad(off) for the offsets used, so LDS offsets stay immediates.
constexpr int xpad_s(int log2n, int ns) { return log2n < 9 || ns == 1 ? 3 : (ns == 8 ? 5 : 30); }
constexpr int xpad_a(int log2n, int ns) { return log2n < 9 || ns == 1 ? 1 : (ns == 8 ? 4 : 0); }
template <int LOG2N, int NS>
__host__ __device__ constexpr int xpad(int i) { return i + xpad_a(LOG2N, NS) * (i >> xpad_s(LOG2N, NS)); }

// Twiddle-power table of the inner 512-point transform (passes 1 and 2, radix
// 8, NS = 8 and 64): pass P's powers of base index i at tt[tw_tab_off(P) +
// k NS + i], k = 0..3 (float4 = two powers).  4.5 KB of LDS.
__host__ __device__ constexpr int tw_tab_off(int p) { return p == 1 ? 0 : 4 * 8; }
constexpr int tw_tab_float4() { return 4 * 8 + 4 * 64; }
// Fills the table: entry i < 8 is pass 1's base W_64^i, i >= 8 pass 2's
// W_512^(i-8), read from the W_N table at stride C (preload_twiddles_wl's
// bases) and raised with apply_twiddles' exact products.  Threads tid of nthr.
__device__ __forceinline__ void tw_tab_build(float4 *tt, int tid, int nthr, const c2 *__restrict__ tw, int C)
{
    for (int e = tid; e < 8 + 64; e += nthr) {
        const bool p1 = e < 8;
        const int i = p1 ? e : e - 8, ns = p1 ? 8 : 64;
        const c2 w1 = tw[(p1 ? i * 8 : i) * C];
        const c2 w2 = mul(w1, w1), w3 = mul(w2, w1), w4 = mul(w2, w2);
        const c2 w5 = mul(w1, w4), w6 = mul(w2, w4), w7 = mul(w3, w4);
        float4 *o = tt + (p1 ? tw_tab_off(1) : tw_tab_off(2)) + i;
        o[0] = make_float4(w1.x, w1.y, w2.x, w2.y);
        o[ns] = make_float4(w3.x, w3.y, w4.x, w4.y);
        o[2 * ns] = make_float4(w5.x, w5.y, w6.x, w6.y);
        o[3 * ns] = make_float4(w7.x, w7.y, 0.0f, 0.0f);
    }
}

// One Stockham pass (radix R, stride Ns).  B = 8/R butterflies per thread;
// butterfly b = t + q*T reads x[b + m*N/R] (= register q + m*B) and writes
// y[(b/Ns)*Ns*R + b%Ns + m*Ns].
// Exchange synchronisation: WSYNC = false -> workgroup barriers (the group
// spans several waves); true -> the group lies within one wave, whose LDS
// operations execute in program order, so only the compiler's ordering of
// the writes before the reads is needed (wave_barrier: no s_barrier).
template <bool WSYNC>
__device__ __forceinline__ void xsync()
{
    if constexpr (WSYNC) __builtin_amdgcn_wave_barrier();
    else __syncthreads();
}

// TT: the pass's twiddle powers come from the LDS table tt (tw_tab_build)
// instead of products of the base wb[P*4 + q]
template <int LOG2N, int P, int DIR, bool WSYNC = false, bool TT = false>
__device__ __forceinline__ void fft_pass(c2 (&v)[8], int t, c2 *lds, const c2 (&wb)[kTwSlots],
                                         const float4 *tt = nullptr)
{
    constexpr int N = 1 << LOG2N, T = N / 8, R = pass_radix<LOG2N, P>(), B = 8 / R;
    constexpr int NS = pass_ns_v(LOG2N, P);
    constexpr bool LAST = P == fft_passes<LOG2N>() - 1;
#pragma unroll
    for (int q = 0; q < B; ++q) {
        const int b = t + q * T;
        c2 u[R];
#pragma unroll
        for (int m = 0; m < R; ++m) u[m] = v[q + m * B];
        if constexpr (NS > 1) {
            if constexpr (TT && R == 8) apply_twiddles_tt<DIR, NS>(u, tt + tw_tab_off(P) + (b & (NS - 1)));
            else apply_twiddles<R, DIR>(u, wb[P * 4 + q]);
        }
        if constexpr (R == 8) dft8<DIR>(u);
        else if constexpr (R == 4) dft4<DIR>(u[0], u[1], u[2], u[3]);
        else dft2<DIR>(u[0], u[1]);
        if constexpr (LAST) {
#pragma unroll
            for (int m = 0; m < R; ++m) v[q + m * B] = u[m];
        } else {
            // xpad(base + m Ns) = xpad(base) + xpad(m Ns): immediate LDS offsets
            c2 *row = lds + xpad<LOG2N, NS>((b / NS) * NS * R + (b & (NS - 1)));
#pragma unroll
            for (int m = 0; m < R; ++m) row[xpad<LOG2N, NS>(m * NS)] = u[m];
        }
    }
    if constexpr (!LAST) {
        xsync<WSYNC>();
        if constexpr (T % 32 == 0) {   // xpad(t + j T) = xpad(t) + xpad(j T)
            const c2 *col = lds + xpad<LOG2N, NS>(t);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = lds_ld(col + xpad<LOG2N, NS>(j * T));
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = lds_ld(lds + xpad<LOG2N, NS>(t + j * T));
        }
        xsync<WSYNC>();
    }
}

template <int LOG2N, int DIR, int P, bool WSYNC = false, bool TT = false>
__device__ __forceinline__ void fft_pass_loop(c2 (&v)[8], int t, c2 *lds, const c2 (&wb)[kTwSlots],
                                              const float4 *tt = nullptr)
{
    if constexpr (P < fft_passes<LOG2N>()) {
        fft_pass<LOG2N, P, DIR, WSYNC, TT>(v, t, lds, wb, tt);
        fft_pass_loop<LOG2N, DIR, P + 1, WSYNC, TT>(v, t, lds, wb, tt);
    }
}

// Unnormalised DFT of the group's sequence, DIR=-1 forward, DIR=+1 inverse.
// Every thread of the WORKGROUP must call this (it contains __syncthreads).
// Ends with a barrier, LDS free on return.  tw: twiddle buffer (tw_entries_v).
template <int LOG2N, int DIR>
__device__ __forceinline__ void fft_regs(c2 (&v)[8], int t, c2 *lds, const c2 *__restrict__ tw)
{
    c2 wb[kTwSlots];
    preload_twiddles<LOG2N>(wb, t, tw);
    fft_pass_loop<LOG2N, DIR, 0>(v, t, lds, wb);
}

// Slot i = P*4 + q of the twiddle-base array is used by pass P's butterfly q.
constexpr bool tw_slot_used(int log2n, int i)
{
    return i / 4 >= 1 && i / 4 < fft_passes_v(log2n) && i % 4 < 8 / pass_radix_v(log2n, i / 4);
}

// Same, with the (forward) twiddle bases already in registers
// (preload_twiddles): for loops that must not issue loads between frames.
template <int LOG2N, int DIR>
__device__ __forceinline__ void fft_regs_w(c2 (&v)[8], int t, c2 *lds, const c2 (&wf)[kTwSlots])
{
    fft_pass_loop<LOG2N, DIR, 0>(v, t, lds, wf);
}

// ---- wave-local FFT: one barrier per transform ------------------------------
// For N >= 1024 a group of T = N/8 threads spans C = N/512 waves.  N = C x M,
// M = 512 = 64 lanes x 8 points: an outer C-point stage across the waves (in
// registers: thread t holds, for each of its H = 8/C values n2 = t + 64 C h,
// all C elements n2 + M n1 in registers h + H n1), ONE cross-wave exchange
// through LDS, and an inner M-point Stockham FFT per wave whose two exchanges
// are wave-local (no s_barrier).  Against the all-workgroup Stockham form (six
// barriers per transform at N = 2048) this removes five barrier waits and
// their skew; the LDS bytes moved are the same.
//   fft_dif: natural order in (v[j] = x[t + jT]), bin-permuted out:
//            v[j] = X[w + C (l + 64 j)], w = t / 64, l = t % 64 (fft_bin).
//   fft_dit: bin-permuted in, natural order out (the inverse of that layout).
// For N <= 512 (C = 1) both are the plain Stockham transform, synchronised per
// wave (a group lies within one wave).
// LDS: C regions of fft_region() complex values (= lds_complex<N>() in all);
// region w is wave w's for the inner transform.  On return from either, other
// waves may still use their regions: __syncthreads() before any use of the
// group's LDS by another wave.
// C waves per transform for 1024 <= N <= 4096; N = 8192 (T = 1024 threads,
// 16 waves: more than a thread's 8 values for the outer stage) runs the
// all-workgroup Stockham transform in natural order, as C = 1
constexpr int fft_c_v(int log2n) { return log2n >= 9 && log2n <= 12 ? 1 << (log2n - 9) : 1; }
constexpr int fft_inner_v(int log2n) { return log2n >= 9 ? 9 : log2n; }
constexpr int fft_region_v(int log2n) { return (1 << fft_inner_v(log2n)) + (1 << fft_inner_v(log2n)) / 8; }

// Slot i of the fft_dif / fft_dit twiddle-base array is in use.
constexpr bool tw_slot_used_wl(int log2n, int i)
{
    return fft_c_v(log2n) == 1 ? tw_slot_used(log2n, i)
                               : (i == 4 || i == 8 || (i >= 12 && i < 12 + 8 / fft_c_v(log2n)));
}

// bin of register j of thread t after fft_dif (and before fft_dit)
template <int LOG2N>
__device__ __forceinline__ int fft_bin(int t, int j)
{
    constexpr int C = fft_c_v(LOG2N), T = (1 << LOG2N) / 8;
    if constexpr (C == 1) return t + j * T;
    else return (t >> 6) + C * ((t & 63) + 64 * j);
}

// LDS slot of bin f in a bin-indexed exchange after fft_dif (all N bins):
// bins f = w (mod C) contiguous, residue regions N/C + 8 apart.  fft_dif's
// layout writes (lane l of wave w: bins w + C (l + 64 j)) land on consecutive
// slots, and natural-order reads of 32 lanes (f = c + l, c = 0 mod C) spread
// the C residues 16 banks apart: both conflict-free on gfx950 (pad8 on f:
// 2-way writes and reads; tools/lds_banks.py).  N + 8 C slots (<= lds_complex).
template <int LOG2N>
__host__ __device__ constexpr int zslot(int f)
{
    constexpr int C = fft_c_v(LOG2N), N = 1 << LOG2N;
    return C == 1 ? f : (f % C) * (N / C + 8) + f / C;
}
// The same for entries e = 0..N/2 (half spectra): regions N/(2C) + 8 apart,
// C (N/(2C) + 8) slots
template <int LOG2N>
__host__ __device__ constexpr int zslot_h(int e)
{
    constexpr int C = fft_c_v(LOG2N), N = 1 << LOG2N;
    return C == 1 ? e : (e % C) * (N / (2 * C) + 8) + e / C;
}
template <int LOG2N> constexpr int zslot_h_size()
{
    return fft_c_v(LOG2N) == 1 ? (1 << LOG2N) / 2 + 1 : (1 << LOG2N) / 2 + 8 * fft_c_v(LOG2N);
}

// Twiddle bases of fft_dif / fft_dit (forward direction): the inner passes'
// (slots 4, 8, from the W_N table at stride C) and, for C > 1, the outer
// stage's W_N^{n2} for the thread's H values n2 (slots 12 + h).
template <int LOG2N>
__device__ __forceinline__ void preload_twiddles_wl(c2 (&wb)[kTwSlots], int t, const c2 *__restrict__ tw)
{
    constexpr int C = fft_c_v(LOG2N);
    if constexpr (C == 1) {
        preload_twiddles<LOG2N>(wb, t, tw);
    } else {
        preload_twiddles<9, 1, C>(wb, t & 63, tw);
#pragma unroll
        for (int h = 0; h < 8 / C; ++h) wb[12 + h] = tw[t + 64 * C * h];
    }
}

template <int C, int DIR>
__device__ __forceinline__ void dft_c(c2 *u)
{
    if constexpr (C == 8) dft8<DIR>(u);
    else if constexpr (C == 4) dft4<DIR>(u[0], u[1], u[2], u[3]);
    else dft2<DIR>(u[0], u[1]);
}

template <int LOG2N, int DIR, bool TT = false>
__device__ __forceinline__ void fft_dif(c2 (&v)[8], int t, c2 *lds, const c2 (&wb)[kTwSlots],
                                        const float4 *tt = nullptr)
{
    constexpr int C = fft_c_v(LOG2N), H = 8 / C, RS = fft_region_v(LOG2N);
    if constexpr (C == 1) {   // one wave per transform (N <= 512), or the whole workgroup (N = 8192)
        fft_pass_loop<LOG2N, DIR, 0, ((1 << LOG2N) / 8 <= 64)>(v, t, lds, wb);
    } else {
#pragma unroll
        for (int h = 0; h < H; ++h) {
            c2 u[C];
#pragma unroll
            for (int m = 0; m < C; ++m) u[m] = v[h + H * m];
            dft_c<C, DIR>(u);                       // over n1 -> k1
            apply_twiddles<C, DIR>(u, wb[12 + h]);  // Y[k1] *= W_N^{n2 k1}
            const int n2 = t + 64 * C * h;
#pragma unroll
            for (int m = 0; m < C; ++m) lds[m * RS + n2] = u[m];
        }
        __syncthreads();
        const int w = t >> 6, l = t & 63;
        c2 *reg = lds + w * RS;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = lds_ld(reg + l + 64 * j);
        __builtin_amdgcn_wave_barrier();
        fft_pass_loop<9, DIR, 0, true, TT>(v, l, reg, wb, tt);
    }
}

template <int LOG2N, int DIR, bool TT = false>
__device__ __forceinline__ void fft_dit(c2 (&v)[8], int t, c2 *lds, const c2 (&wb)[kTwSlots],
                                        const float4 *tt = nullptr)
{
    constexpr int C = fft_c_v(LOG2N), H = 8 / C, RS = fft_region_v(LOG2N);
    if constexpr (C == 1) {   // one wave per transform (N <= 512), or the whole workgroup (N = 8192)
        fft_pass_loop<LOG2N, DIR, 0, ((1 << LOG2N) / 8 <= 64)>(v, t, lds, wb);
    } else {
        const int w = t >> 6, l = t & 63;
        c2 *reg = lds + w * RS;
        fft_pass_loop<9, DIR, 0, true, TT>(v, l, reg, wb, tt);   // over k2 -> n2, region w
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 8; ++j) reg[l + 64 * j] = v[j];
        __syncthreads();
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int n2 = t + 64 * C * h;
            c2 u[C];
#pragma unroll
            for (int m = 0; m < C; ++m) u[m] = lds_ld(lds + m * RS + n2);
            apply_twiddles<C, DIR>(u, wb[12 + h]);  // y[k1] *= W_N^{DIR n2 k1}
            dft_c<C, DIR>(u);                       // over k1 -> n1
#pragma unroll
            for (int m = 0; m < C; ++m) v[h + H * m] = u[m];
        }
    }
}

}  // namespace mm
