// mm_steer.hpp — MM_MODE_STEERABLE (extension f2): oriented
// local-phase subbands with a per-coefficient temporal filter.  Spec and CPU
// oracle: oracle/steerable_ref.py (no reference counterpart; parity of the
// shared stages is pinned by its S = 0 identity with the reference path).
//
// Per frame, after K1 (row FFTs -> G):
//   k_cols_fwd : G columns -> F, the half spectrum (f <= N/2, all fy)
//   k_sb_cols  : one column kx of F (Hermitian mirror for kx > N/2) times each
//                band mask  m_i a_o / N^2  (o < O/2) and the residual mask
//                (m_0 + m_{L-1}) / N^2 -> column IFFT -> T[band][k][kx] (row-major)
//                for the Hn list rows the crop + blur need
//   k_sb_rows  : one list row k: per band the row IFFT -> local coefficient
//                s(x); in the W+4 columns the blur reads, phase filter vs the
//                state, s' = s e^{i S P} (gated |s| < tau), y += 2 Re s';
//                residual y += Re s;  |y| -> horizontal 5-tap blur -> Yh
// then K4 (k_compose) as in the other modes.
#pragma once
#include "mm_kernels.hpp"

namespace mm {

// GeneratePyramidFilters (PyramidOperations.compute:25-87) for level i at radius fr.
__device__ __forceinline__ float level_mask(float fr, int i, const Spec &sp)
{
    if (i == 0)
        return fr > sp.maxF ? 1.0f : (fr > sp.hp_lo ? smooth01((fr - sp.hp_lo) * sp.hp_inv) : 0.0f);
    if (i == sp.L - 1)
        return fr < sp.minF ? 1.0f : (fr < sp.lp_hi ? 1.0f - smooth01((fr - sp.minF) * sp.lp_inv) : 0.0f);
    return (fr >= sp.lo[i] && fr <= sp.hi[i])
               ? 0.5f * (1.0f + __cosf(2.0f * kPi * ((fr - sp.lo[i]) * sp.inv_w[i] - 0.5f)))
               : 0.0f;
}

__device__ __forceinline__ float pow4(float x) { x *= x; return x * x; }

// normalize_phase (PyramidPhaseDifference.compute:47-54) for |x| < 3 pi
__device__ __forceinline__ float wrap_pi(float x)
{
    if (x > kPi) x -= 2.0f * kPi;
    if (x < -kPi) x += 2.0f * kPi;
    return x;
}

// signed true frequency / N of index k: k < N/2 -> k, else k - N (N/2 -> -1/2)
template <int N> __device__ __forceinline__ float sfreq(int k)
{
    return (float)(k < N / 2 ? k : k - N) * (1.0f / (float)N);
}

// Band b (< nb) of column kx is identically zero when the column lies outside
// the band's annulus: every bin has fr >= |fx| (exact in fp32: fx = k/N and
// sqrt of the exact square), and level_mask is 0 for fr > hi.  Both band
// kernels apply this same test: k_sb_cols skips such columns (no FFT, no
// store) and k_sb_rows reads zeros for them (no load).  For L = 5 the two
// inner levels' bands are zero in 55 % and 85 % of the columns.
template <int N>
__device__ __forceinline__ bool band_col_zero(int b, int nb, int nmid, int kx, const Spec &sp)
{
    return b < nb && fabsf(sfreq<N>(kx)) > sp.hi[1 + b % nmid];
}

// -------------------------------------------------------------------------
// F of every chunk frame: column FFTs of K1's G, stored as Fb[fr][f][fy].
// -------------------------------------------------------------------------
template <int LOG2N>
__global__ __launch_bounds__(wg_threads<LOG2N>())
void k_cols_fwd(const c2 *__restrict__ G, size_t g_stride, c2 *__restrict__ Fb, size_t f_stride,
                int total_cols, Geo g, const c2 *__restrict__ tw)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = groups_per_wg<LOG2N>();
    constexpr int F = N / 2 + 1;
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = GPW == 1 ? 0 : threadIdx.x / T, t = GPW == 1 ? threadIdx.x : threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const int logical = blockIdx.x * GPW + grp;
    const bool valid = logical < total_cols;
    const int fr = valid ? logical / F : 0, f = valid ? logical % F : 0;
    const c2 *Gc = G + (size_t)fr * g_stride + (size_t)f * g.Hg;   // (H rows of Hg: K1 writes row pairs)
    c2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int rr = t + j * T - g.y0;
        const c2 a = Gc[min(max(rr, 0), g.H - 1)];
        v[j] = (rr >= 0 && rr < g.H) ? a : mk(0.0f, 0.0f);
    }
    fft_regs<LOG2N, -1>(v, t, lds, tw);
    if (valid) {
        c2 *out = Fb + (size_t)fr * f_stride + (size_t)f * N;
#pragma unroll
        for (int j = 0; j < 8; ++j) out[t + j * T] = v[j];
    }
}

// Band rows T[b] (k_sb_cols -> k_sb_rows), t_rows(Hn) x N complex per band.
// MM_SB_RROWS = R: list rows in groups of R, (k, kx) at (k/R) R N + R kx + k%R,
// so that a workgroup's GPW columns of a row group are one 8 R GPW-byte piece
// (R = 4, GPW = 1: 32 B, a quarter of the lines per store instruction and four
// times the piece of the row-major layout), and k_sb_rows reads its row at an
// 8 R-byte stride (the group's other rows are the neighbouring row
// workgroups', on the same XCD).  R = 1: row-major, (k, kx) at k N + kx.
// Same call (profiles/r06h_sb_rows_layout_ab.txt), C3 O = 8 DIFF frames/s:
// R 1 / 2 at GPW 2: 940 / 1,094; R 2 / 4 / 8 at GPW 1: 966 / 1,135 / 1,046.
#ifndef MM_SB_RROWS
#define MM_SB_RROWS 4
#endif
constexpr int kSbR = MM_SB_RROWS;
static_assert(kSbR == 1 || kSbR == 2 || kSbR == 4 || kSbR == 8, "MM_SB_RROWS: 1, 2, 4 or 8");
template <int N> __device__ __forceinline__ size_t t_row(int k)   // offset of (k, 0)
{
    return (size_t)(k / kSbR) * (kSbR * N) + k % kSbR;
}
constexpr int t_col_stride() { return kSbR; }                     // between (k, kx) and (k, kx+1)
// rows per band in T (whole row groups)
__host__ __device__ constexpr int t_rows(int hn) { return (hn + kSbR - 1) / kSbR * kSbR; }
// k_sb_cols staging: column c's rows at c S + k (MM_SB_STG_CM = 1), S = the
// rows rounded up to 16 mod 32 entries from N = 1024 on: the rows' 8-B
// writes (16 consecutive rows per lane group) are conflict-free, and so are
// the float4 reads of a row group's columns (S 2 = 32 mod 64 dwords puts
// column 1 on the other half of the banks; tools/lds_banks.py "sb_stg").
// MM_SB_STG_CM = 0: row-group-major (k / R) R GPW + R c + k % R (2-way
// conflicted writes).
#ifndef MM_SB_STG_CM
#define MM_SB_STG_CM 1
#endif
__host__ __device__ constexpr int sb_stg_stride(int hn, int n)
{
    return MM_SB_STG_CM && n >= 1024 ? (t_rows(hn) + 15) / 32 * 32 + 16 : t_rows(hn);
}

// -------------------------------------------------------------------------
// Band columns: T[b][k][kx] = IFFT_col(F m_i a_o / N^2)[canvas row rb + k]
// -------------------------------------------------------------------------
// GPW >= 2 columns per workgroup (same-XCD blocks own consecutive columns):
// each band's columns are transposed through LDS and leave as one
// 8 R GPW-byte piece per row group of T (t_row), which k_sb_rows then reads
// row by row (a column-major T made those reads 8-B gathers: 16x L2->L1
// traffic).  The store piece is what bounds this kernel: 8 B (one column per
// workgroup) / 16 B (R = 1) / 32 B (R = 2) per lane: C3 O = 8 k_sb_cols 1,020 /
// 594 / 434 us per frame (profiles/r06h_sb_rows_layout_ab.txt).  The band loop
// issues no loads (twiddle bases hoisted), so its stores are never waited for.
#ifndef MM_SB_COLS_WL
#define MM_SB_COLS_WL 1
#endif
template <int LOG2N>
__global__ __launch_bounds__(sb_threads<LOG2N>()) __attribute__((amdgpu_waves_per_eu(4)))
void k_sb_cols(const c2 *__restrict__ Fb, c2 *__restrict__ Tb, size_t band_stride, Geo g, Spec sp,
               const c2 *__restrict__ tw, int stg_own, size_t f_stride, size_t t_stride)
{
    // blockIdx.y: the frame of the launch's frames (k_sb_rows' group of NF),
    // its F at Fb + y f_stride, its band rows at Tb + y t_stride
    Fb += blockIdx.y * f_stride;
    Tb += blockIdx.y * t_stride;
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = sb_groups<LOG2N>();
    constexpr bool SB_WL = MM_SB_COLS_WL && fft_c_v(LOG2N) > 1;
    constexpr bool DIRECT = SB_WL && sb_direct<LOG2N>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = T % 64 == 0 ? __builtin_amdgcn_readfirstlane(threadIdx.x / T) : threadIdx.x / T;
    const int t0 = threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    // columns near kx = 0 and N carry more bands than those near N/2
    // (band_col_zero): interleave column runs over the XCDs.  Runs of 64
    // blocks (128 columns): each XCD then owns a heavy and a light part of the
    // spectrum in each of the launch's two workgroup rounds (same-call at 1080p,
    // O = 8: k_sb_cols 117.4 (runs of 8) -> 105.7-105.8 us per frame; 2 / 4 /
    // 16 / 32 / 128: 121.0-121.5 / 115.5-116.0 / 114.5-114.9 / 116.2-116.6 /
    // 127.6)
#ifndef MM_SB_COLS_RUN
#define MM_SB_COLS_RUN 64
#endif
    // (heavy runs first, 0, last, 1, last - 1, ...: C3 k_sb_cols 436 -> 457 us
    // per frame, profiles/r06h_sb_rows_layout_ab.txt)
    const int blk = xcd_interleave<MM_SB_COLS_RUN>(blockIdx.x, gridDim.x);
    const int kx_raw = blk * GPW + grp;
    const bool valid = kx_raw < N;               // small N: more groups than columns
    const int kx = valid ? kx_raw : N - 1;
    const bool mir = kx > N / 2;
    const c2 *Fc = Fb + (size_t)(mir ? N - kx : kx) * N;
    const float fxs = sfreq<N>(kx);
    c2 v0[8];
    float fr[8], cx[8], sy[8], isum[8];
    // the inverse column transform is the wave-local fft_dit (one workgroup
    // barrier instead of six at N = 2048): its input is in fft_bin order, so
    // register j of lane t holds bin ky = fft_bin(t, j) (the F column is read
    // once, in that order), and its output is in natural row order as before
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int ky = SB_WL ? fft_bin<LOG2N>(t0, j) : t0 + j * T;
        c2 a = Fc[mir ? (N - ky) & (N - 1) : ky];     // F(-f) = conj F(f) (real input)
        if (mir) a.y = -a.y;
        v0[j] = scale(a, sp.inv_nn);
        const float fys = sfreq<N>(ky);
        const float r2 = fxs * fxs + fys * fys;
        fr[j] = __builtin_amdgcn_sqrtf(r2);
        const bool flat = kx == N / 2 || ky == N / 2 || r2 == 0.0f;   // a_o = 1/O
        const float ir = flat ? 0.0f : 1.0f / fr[j];
        cx[j] = fxs * ir;
        sy[j] = fys * ir;
        // O = 6, 8: sum_k max(0, cos(theta - 2 pi k / O))^4 = 3 O / 16 for every
        // theta (cos^4 = 3/8 + cos 2x / 2 + cos 4x / 8, and the O equally spaced
        // lobes cancel the harmonics 2 and 4 when O divides neither; the max(0, .)
        // keeps exactly half of the sum, the lobes o and o + O/2 being opposite).
        // The constant replaces the per-bin O-term sum (same value to fp32
        // rounding; k_sb_cols -6 %, O = 8 DIFF +3 % same-call,
        // profiles/r05f_sb_isum_ab.txt).  O = 4 keeps the sum (harmonic 4 stays).
        if (sp.O > 4) {
            isum[j] = flat ? -1.0f : 16.0f / (3.0f * (float)sp.O);
            continue;
        }
        float sum = 0.0f;
        for (int k = 0; k < sp.O; ++k) sum += pow4(fmaxf(0.0f, cx[j] * sp.ang_c[k] + sy[j] * sp.ang_s[k]));
        isum[j] = flat ? -1.0f : 1.0f / sum;
    }
    c2 wtw[kTwSlots];
#pragma unroll
    for (int i = 0; i < kTwSlots; ++i) wtw[i] = mk(1.0f, 0.0f);
    if constexpr (SB_WL) preload_twiddles_wl<LOG2N>(wtw, t0, tw);
    else preload_twiddles<LOG2N>(wtw, t0, tw);
    const int nmid = sp.L >= 3 ? sp.L - 2 : 0;
    const int nb = nmid * (sp.O / 2);
    const int kx0 = blk * GPW;
    // staging [Hn][GPW]: its own LDS area after the exchange buffers when
    // stg_own (the launch sized the LDS for it), else over them
    c2 *stg = stg_own ? lds_all + GPW * lds_complex<N>() : lds_all;
    // Bands level-major (b = o nmid + i - 1 as before): the radial mask of a
    // level is evaluated once for its O/2 orientation bands, which then only
    // add the angular factor (the same expressions per band: bitwise the
    // band-major loop's values).  The residual band (b = nb) runs last.
    float rm[8];
    int nbuf = 0;   // DIRECT: exchange buffer of the next band run
    for (int lb = 0; lb <= nb; ++lb) {
        const int i = lb < nb ? 1 + lb / (sp.O / 2) : 0, o = lb < nb ? lb % (sp.O / 2) : 0;
        const int b = lb < nb ? o * nmid + (i - 1) : nb;
        // opaque lane index and twiddle bases per band: keeps LICM from
        // hoisting the FFT addressing and twiddle powers into live registers
        int t = t0;
        asm volatile("" : "+v"(t));
        c2 wt[kTwSlots];
#pragma unroll
        for (int q = 0; q < kTwSlots; ++q) {
            wt[q] = wtw[q];
            if (SB_WL ? tw_slot_used_wl(LOG2N, q) : tw_slot_used(LOG2N, q)) asm volatile("" : "+v"(wt[q]));
        }
        // workgroup-uniform: skip the band where all its columns are zero
        bool all_zero = true;
        for (int c = 0; c < GPW && kx0 + c < N; ++c) all_zero &= band_col_zero<N>(b, nb, nmid, kx0 + c, sp);
        if (all_zero) continue;   // (then every band of this level: o = 0 skips them all)
        if (lb < nb && o == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) rm[j] = level_mask(fr[j], i, sp);
        }
        c2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float m;
            if (b == nb) {   // residual: levels 0 and L-1, no orientation
                m = level_mask(fr[j], 0, sp) + (sp.L > 1 ? level_mask(fr[j], sp.L - 1, sp) : 0.0f);
            } else {
                const float ao = isum[j] < 0.0f
                                     ? 1.0f / (float)sp.O
                                     : pow4(fmaxf(0.0f, cx[j] * sp.ang_c[o] + sy[j] * sp.ang_s[o])) * isum[j];
                m = rm[j] * ao;
            }
            v[j] = scale(v0[j], m);
        }
        if constexpr (DIRECT) {
            // one column: rows t + jT leave from registers as 8-B values;
            // the two exchange buffers alternate, so no barrier guards the
            // next band's writes against this band's cross-wave reads
            fft_dit<LOG2N, +1>(v, t, lds_all + nbuf * lds_complex<N>(), wt);
            nbuf ^= 1;
            c2 *out = Tb + (size_t)b * band_stride + (size_t)kx * t_col_stride();
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = (t + j * T - g.rb + 2 * N) & (N - 1);
                if (valid && k < g.Hn) out[t_row<N>(k)] = v[j];
            }
            continue;
        }
        if constexpr (SB_WL) {
            fft_dit<LOG2N, +1>(v, t, lds, wt);
            // staging over the exchange buffers: every wave past its reads first
            if (!stg_own) __syncthreads();
        } else {
            fft_regs_w<LOG2N, +1>(v, t, lds, wt);   // ends with a barrier after its last exchange read
        }
        // staging: column-major (c S + k, MM_SB_STG_CM) or in T's order (row
        // group m's GPW columns x R rows at m R GPW)
        const int S = sb_stg_stride(g.Hn, N);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = (t + j * T - g.rb + 2 * N) & (N - 1);
            if (k < g.Hn)
                stg[MM_SB_STG_CM ? grp * S + k : (k / kSbR) * (kSbR * GPW) + kSbR * grp + k % kSbR] = v[j];
        }
        __syncthreads();
        c2 *out = Tb + (size_t)b * band_stride;
        const int groups = t_rows(g.Hn) / kSbR;
        if constexpr (MM_SB_STG_CM && kSbR > 1 && GPW <= N) {   // R GPW / 2 float4 per row group
            // float4 q of row group m: column q / (R/2), rows 2 (q % (R/2)) ..
            // +1 of the group (a last partial group's missing rows are stale
            // staging, written to T's pad rows, which k_sb_rows never reads)
            constexpr int PW = kSbR * GPW / 2, H2 = kSbR / 2;
            for (int e = grp * T + t; e < groups * PW; e += GPW * T) {
                const int m = e / PW, q = e - m * PW, c = q / H2, h = q - c * H2;
                *reinterpret_cast<float4 *>(out + (size_t)m * (kSbR * N) + kSbR * kx0 + 2 * q) =
                    *reinterpret_cast<const float4 *>(stg + c * S + m * kSbR + 2 * h);
            }
        } else if constexpr (MM_SB_STG_CM) {    // R = 1, or tiny N (fewer columns than groups)
            for (int e = grp * T + t; e < groups * kSbR * GPW; e += GPW * T) {
                const int m = e / (kSbR * GPW), o = e - m * (kSbR * GPW), c = o / kSbR, kk = o - c * kSbR;
                if (kx0 + c < N) out[(size_t)m * (kSbR * N) + kSbR * (kx0 + c) + kk] = stg[c * S + m * kSbR + kk];
            }
        } else if constexpr (kSbR > 1 && GPW <= N) {   // whole pieces: R GPW / 2 float4 per row group
            // (a last partial group's missing rows are stale staging, written
            // to T's pad rows, which k_sb_rows never reads)
            constexpr int PW = kSbR * GPW / 2;
            for (int e = grp * T + t; e < groups * PW; e += GPW * T) {
                const int m = e / PW, part = e - m * PW;
                *reinterpret_cast<float4 *>(out + (size_t)m * (kSbR * N) + kSbR * kx0 + 2 * part) =
                    reinterpret_cast<const float4 *>(stg)[e];
            }
        } else if constexpr (kSbR > 1) {       // tiny N: fewer columns than groups
            for (int e = grp * T + t; e < groups * kSbR * GPW; e += GPW * T) {
                const int m = e / (kSbR * GPW), c = (e / kSbR) % GPW, kk = e % kSbR;
                if (kx0 + c < N) out[(size_t)m * (kSbR * N) + kSbR * (kx0 + c) + kk] = stg[e];
            }
        } else if constexpr (GPW >= 2 && GPW <= N) {   // whole pieces: GPW / 2 float4 per row
            constexpr int PW = GPW / 2;
            for (int e = grp * T + t; e < g.Hn * PW; e += GPW * T) {
                const int k = e / PW, part = e - k * PW;
                *reinterpret_cast<float4 *>(out + (size_t)k * N + kx0 + 2 * part) =
                    reinterpret_cast<const float4 *>(stg)[e];
            }
        } else {                    // tiny N: fewer columns than groups
            for (int e = grp * T + t; e < g.Hn * GPW; e += GPW * T) {
                const int k = e / GPW, c = e - k * GPW;
                if (kx0 + c < N) out[(size_t)k * N + kx0 + c] = stg[e];
            }
        }
        // the next band's FFT rewrites the buffers (an own staging area: the
        // next band's staging writes follow its FFT's barrier)
        if (!stg_own) __syncthreads();
    }
}

// -------------------------------------------------------------------------
// Band rows: local phase filter, amplification, synthesis, |.|, H blur -> Yh
// -------------------------------------------------------------------------
// State planes (floats): phi[b][k][xi], u_h[...], u_l[...] for the Wc = W+4
// canvas columns x0-2 .. x0+W+1 the horizontal blur reads (xi = x - (x0-2)
// mod N).  reset: first frame (phi <- arg s, u <- 0, nothing amplified).
// Band b+1's row loads are issued before band b's state stores, so the FFT's
// wait for them does not wait for those stores (one in-order vmcnt); band
// b+1's state loads follow the stores and are consumed only after its FFT,
// when the stores have long completed.  The pointers are not restrict so
// that the compiler keeps this order.
// IIR: the temporal filter as a template parameter, so that the DIFF kernel
// carries one state plane's registers, not three: 120 VGPRs (3 planes, 4
// waves per SIMD) -> <= 96 (5 waves per SIMD).  At 1080p the Hn = 1,084 rows
// are 1,084 four-wave workgroups: at 4 waves per SIMD 1,024 of them run at
// once and the last 60 make a second round of the whole row time; at 5 they
// all fit one round.
// NF consecutive frames per launch (1 or 2): a workgroup runs band b of
// frame 0, then band b of frame 1 against frame 0's new state still in
// registers, and writes the state planes once per NF frames (the DIFF planes
// are read and written once per pair instead of per frame: 200 -> 100 MB per
// 1080p frame at O = 8).  The same expressions in the same order as NF = 1:
// bitwise the per-frame outputs.  Frame f's band rows at Tb + f * t_stride,
// its Yh at Yh + f * yh_stride; reset applies to frame 0 (the stream's first
// frame: it seeds the state and passes through); write_mask bit f: frame f's
// Yh is wanted.
#ifndef MM_SB_OFF32
#define MM_SB_OFF32 1
#endif
#ifndef MM_SB_IIR_GROUPS
#define MM_SB_IIR_GROUPS 0
#endif
// k_sb_rows' twiddle bases loaded per band from the (L1-resident) table
// instead of ~20 VGPRs held across the band loop: IIR (its band loop then
// fits 128 VGPRs without spills: 1080p O = 8 IIR 4.43k -> 4.52k frames/s,
// profiles/r06h_sb_rows_layout_ab.txt); MM_SB_TWLD_DIFF for DIFF (at 6 waves
// per SIMD, 80 VGPRs, it spills 18)
#ifndef MM_SB_TWLD_IIR
#define MM_SB_TWLD_IIR 1
#endif
#ifndef MM_SB_TWLD_DIFF
#define MM_SB_TWLD_DIFF 0
#endif
template <bool IIR> constexpr bool kSbRowsTwLd = IIR ? MM_SB_TWLD_IIR : MM_SB_TWLD_DIFF;
template <int LOG2N, bool IIR, int NF>
__global__ __launch_bounds__(sb_rows_threads<LOG2N>())
__attribute__((amdgpu_waves_per_eu(IIR || NF > 2 || sb_rows_threads<LOG2N>() >= 1024 ? 4 : 5)))
void k_sb_rows(const c2 *Tb, size_t band_stride, size_t t_stride, float *__restrict__ Yh, size_t yh_stride,
               float *st_phi, float *st_uh, float *st_ul,
               int reset, int write_mask, Geo g, Spec sp, Blur5 bw, const c2 *__restrict__ tw, int ngroups)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = sb_rows_groups<LOG2N>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    // (the group index wave-uniform: the row's band and state bases stay scalar)
    const int grp = GPW == 1 ? 0 : (T % 64 == 0 ? __builtin_amdgcn_readfirstlane(threadIdx.x / T) : threadIdx.x / T);
    const int t0 = GPW == 1 ? threadIdx.x : threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const int logical = xcd_remap(blockIdx.x, gridDim.x) * GPW + grp;
    const bool valid = logical < g.Hn;
    const int k = valid ? logical : g.Hn - 1;   // list row (canvas row rb + k)
    // state / synthesis window: canvas columns x0 - 2 .. x0 + Wy + 1 (the blur's
    // reach around the Yh columns; Wy = W + 1 for odd W: the crop's second texel)
    const int Wc = g.Wy + 4, xs = g.x0 - 2;
    const int nmid = sp.L >= 3 ? sp.L - 2 : 0;
    const int nb = nmid * (sp.O / 2);
    constexpr bool iir = IIR;
    c2 wtw[kTwSlots];
#pragma unroll
    for (int i = 0; i < kTwSlots; ++i) wtw[i] = mk(1.0f, 0.0f);
    if constexpr (!kSbRowsTwLd<IIR>) preload_twiddles<LOG2N>(wtw, t0, tw);   // forward bases; fft_regs_w conjugates
    // row k of band b of frame f (contiguous) and its state: loaded one row ahead
    c2 v[8];
    float pp[8], puh[8], pul[8];
    // ngroups groups of NF frames per launch, one after the other in every
    // workgroup (its row's state goes to memory between groups and comes back
    // to the same lanes): fewer kernel boundaries than a launch per group.
    // Group gi: band rows at Tb + gi NF t_stride, Yh at Yh + gi NF yh_stride,
    // write_mask bits gi NF .., reset for group 0 only.
    const c2 *Tg = Tb;
    int rz = reset;
    auto load_row = [&](int f, int b, int t) {
        // (row base per workgroup, 32-bit lane offsets: no 64-bit address
        // math per element, MM_SB_OFF32)
        const c2 *row = Tg + (size_t)f * t_stride + (size_t)b * band_stride + t_row<N>(k);
#pragma unroll
        for (int j = 0; j < 8; ++j)   // band_col_zero columns were never written: 0
            v[j] = band_col_zero<N>(b, nb, nmid, t + j * T, sp)
                       ? mk(0.0f, 0.0f)
                       : (MM_SB_OFF32 ? ld_off<c2>(row, (unsigned)((t + j * T) * t_col_stride()) * 8u)
                                      : row[(t + j * T) * t_col_stride()]);
    };
    auto load_state = [&](int b, int t) {
        if (b < nb && !rz) {
            const size_t rs = ((size_t)b * g.Hn + k) * Wc;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int xi = min((t + j * T - xs + N) & (N - 1), Wc - 1);
                if (MM_SB_OFF32) {
                    pp[j] = ld_off<float>(st_phi + rs, (unsigned)xi * 4u);
                    if (iir) {
                        puh[j] = ld_off<float>(st_uh + rs, (unsigned)xi * 4u);
                        pul[j] = ld_off<float>(st_ul + rs, (unsigned)xi * 4u);
                    }
                } else {
                    pp[j] = st_phi[rs + xi];
                    if (iir) {
                        puh[j] = st_uh[rs + xi];
                        pul[j] = st_ul[rs + xi];
                    }
                }
            }
        }
    };
    // (IIR: one group per launch; its three state planes leave no registers
    // for the loop: 34 B of spills inside the band loop, k_sb_rows +6 %)
    const int ngr = IIR && !MM_SB_IIR_GROUPS ? 1 : ngroups;
    for (int gi = 0; gi < ngr; ++gi) {
    Tg = Tb + (size_t)gi * NF * t_stride;
    rz = gi == 0 ? reset : 0;
    const int wmask = write_mask >> (gi * NF);
    float *Yg = Yh + (size_t)gi * NF * yh_stride;
    if (gi > 0) __syncthreads();   // the previous group's blur reads of the LDS are done
    {
        int t = t0;
        asm volatile("" : "+v"(t));
        load_row(0, 0, t);
        load_state(0, t);
    }
    float y[NF][8];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int j = 0; j < 8; ++j) y[f][j] = 0.0f;
    for (int b = 0; b <= nb; ++b) {
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            int t = t0;
            asm volatile("" : "+v"(t));
            c2 wt[kTwSlots];
            if constexpr (kSbRowsTwLd<IIR>) {
                // (IIR: the twiddle bases from the L1-resident table per band
                // instead of ~20 VGPRs held across the band loop)
#pragma unroll
                for (int i = 0; i < kTwSlots; ++i) wt[i] = mk(1.0f, 0.0f);
                preload_twiddles<LOG2N>(wt, t, tw);
            } else {
#pragma unroll
                for (int i = 0; i < kTwSlots; ++i) {
                    wt[i] = wtw[i];
                    if (tw_slot_used(LOG2N, i)) asm volatile("" : "+v"(wt[i]));
                }
            }
            fft_regs_w<LOG2N, +1>(v, t, lds, wt);
            if (b == nb) {   // residual: Hermitian, real output
#pragma unroll
                for (int j = 0; j < 8; ++j) y[f][j] += v[j].x;
                if (f + 1 < NF) load_row(f + 1, nb, t);
                continue;
            }
            // this band's new state and amplified synthesis, in registers
            const bool rst = f == 0 && rz;               // the stream's first frame
            const bool wr = ((wmask >> f) & 1) != 0;
            float nph[8], nuh[8], nul[8];
            // local phases two bins at a time (packed FP32, fast_atan2's values)
            float phs[8];
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const c2 p2 = fast_atan2_x2(v[j].y, v[j].x, v[j + 1].y, v[j + 1].x);
                phs[j] = p2.x;
                phs[j + 1] = p2.y;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float ph = phs[j];
                float P = 0.0f, uh = 0.0f, ul = 0.0f;
                if (!rst) {
                    if (!iir) {
                        P = wrap_pi(pp[j] - ph);              // prev - cur, as the reference
                    } else {
                        const float d = wrap_pi(ph - pp[j]);
                        uh = (1.0f - sp.r_high) * (puh[j] + d);
                        ul = (1.0f - sp.r_low) * (pul[j] + d);
                        P = ul - uh;
                    }
                }
                nph[j] = ph;
                nuh[j] = uh;
                nul[j] = ul;
                c2 s2 = v[j];
                if (wr && v[j].x * v[j].x + v[j].y * v[j].y >= sp.tau2) {
                    const float rev = P * sp.S_rev;
                    s2 = mul_c(v[j], mk(__builtin_amdgcn_cosf(rev), __builtin_amdgcn_sinf(rev)));
                }
                const int xi = (t + j * T - xs + N) & (N - 1);
                if (xi < Wc) y[f][j] += 2.0f * s2.x;
            }
            if (f + 1 < NF) {
                // the next frame's row of this band; its previous state is this
                // frame's new one, still in registers
                load_row(f + 1, b, t);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    pp[j] = nph[j];
                    if (iir) {
                        puh[j] = nuh[j];
                        pul[j] = nul[j];
                    }
                }
                continue;
            }
            load_row(0, b + 1, t);
            __builtin_amdgcn_sched_barrier(0);   // row loads of b+1 ahead of the stores of b
            if (valid) {
                const size_t rs = ((size_t)b * g.Hn + k) * Wc;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int xi = (t + j * T - xs + N) & (N - 1);
                    if (xi < Wc) {
                        if (MM_SB_OFF32) {
                            st_off<float>(st_phi + rs, (unsigned)xi * 4u, nph[j]);
                            if (iir) {
                                st_off<float>(st_uh + rs, (unsigned)xi * 4u, nuh[j]);
                                st_off<float>(st_ul + rs, (unsigned)xi * 4u, nul[j]);
                            }
                        } else {
                            st_phi[rs + xi] = nph[j];
                            if (iir) {
                                st_uh[rs + xi] = nuh[j];
                                st_ul[rs + xi] = nul[j];
                            }
                        }
                    }
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            load_state(b + 1, t);
        }
    }
    // |y| (ConvertComplexMagToTex) then the horizontal half of ApplyAntiAliasing
    float *raw = reinterpret_cast<float *>(lds);
    const bool interior = g.x0 >= 2 && g.x0 + g.Wy + 2 <= N;
    // (an opaque lane index: the blur's addressing is not hoisted out of the
    // group loop into registers live across the band loop)
    int tb = t0;
    asm volatile("" : "+v"(tb));
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        if (!((wmask >> f) & 1)) continue;        // uniform
        if (f > 0) __syncthreads();               // the previous frame's blur reads are done
#pragma unroll
        for (int j = 0; j < 8; ++j) raw[tb + j * T] = fabsf(y[f][j]);
        __syncthreads();
        if (valid) {
            float *out = Yg + (size_t)f * yh_stride + (size_t)k * g.Wy;
            for (int X = tb; X < g.Wy; X += T) {
                const int c = g.x0 + X;
                float acc;
                if (interior) {
                    acc = bw.w0 * raw[c] + bw.w1 * (raw[c - 1] + raw[c + 1]) + bw.w2 * (raw[c - 2] + raw[c + 2]);
                } else {
                    acc = bw.w0 * raw[wrap_idx(c, N, g.edge)];
                    acc += bw.w1 * (raw[wrap_idx(c - 1, N, g.edge)] + raw[wrap_idx(c + 1, N, g.edge)]);
                    acc += bw.w2 * (raw[wrap_idx(c - 2, N, g.edge)] + raw[wrap_idx(c + 2, N, g.edge)]);
                }
                out[X] = acc;
            }
        }
    }
    }   // groups
}

}  // namespace mm
