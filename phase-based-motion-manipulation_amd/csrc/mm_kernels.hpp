// mm_kernels.hpp — the three HIP kernels of one magnified frame (gfx950).
//
// Data flow per frame (N = padded square size, F = N/2+1 half-spectrum columns):
//   K1 k_rows_fwd : RGBA frame --(luma, stretch+pad bilinear, Hann window)-->
//                   real rows --(paired real FFT)--> G[f][row]       (f < F)
//   K2 k_cols     : G column --FFT--> F_t --(pyramid phase op vs F_{t-1})-->
//                   A --IFFT--> Q[f][row]; F_t becomes the state.  One WG owns
//                   a column for a whole chunk of frames, so F_{t-1} stays in
//                   registers between frames.
//   K3 k_rows_inv : Q rows --(paired C2R IFFT)--> |z| --(5-tap H blur)--> ring
//                   of rows in LDS --(5-tap V blur, YIQ recombine, YIQ->RGB,
//                   saturate, crop)--> RGBA frame
// Reference stages replaced (MotionMagnificationProcessor.cs:145-206): a4-a18 of
// SURVEY.md §8(a).  The pyramid levels are applied pointwise in frequency
// (SURVEY.md §7): arg(m_i F) = arg F for real m_i >= 0, so one atan2/sincos per
// bin serves every level.
#pragma once
#include "mm_fft.hpp"
#include <stdint.h>

namespace mm {

constexpr int kMaxLevels = 16;
constexpr float kPi = 3.14159265359f;  // PyramidOperations.compute:5

struct Tap4 {         // composite stretch+pad bilinear taps incl. Hann factor
    int idx[4];
    float w[4];
};

struct Geo {
    int W, H, N;
    int x0, y0;       // image placement inside the canvas (PadTexture .cs:360-363)
    int rb;           // canvas row of Q list index 0 (= y0 - 2)
    int Hn;           // rows kept in Q (= min(H + 4, N))
    int Hq;           // Q column stride (Hn rounded to even)
    int edge;         // 0 repeat, 1 clamp
};

struct Spec {
    int L;
    float minF, maxF, S, tau, inv_nn;
    float lo[kMaxLevels], hi[kMaxLevels];
};

struct Blur5 { float w0, w1, w2; };  // taps at 0, +-1, +-2 texels

template <int LOG2N> constexpr int fft_T() { return (1 << LOG2N) / 8; }
template <int LOG2N> constexpr int groups_per_wg() { return fft_T<LOG2N>() >= 256 ? 1 : 256 / fft_T<LOG2N>(); }
template <int LOG2N> constexpr int wg_threads() { return groups_per_wg<LOG2N>() * fft_T<LOG2N>(); }

__device__ __forceinline__ int wrap_idx(int i, int n, int edge)
{
    if (edge) return i < 0 ? 0 : (i >= n ? n - 1 : i);
    int r = i % n;
    return r < 0 ? r + n : r;
}

// Same-XCD blocks (b % 8 equal under round-robin dispatch) get consecutive ids.
__device__ __forceinline__ int xcd_remap(int b, int nb)
{
    int q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// ---- pixel access -------------------------------------------------------
template <int FMT> struct Pix;
template <> struct Pix<0> {           // RGBA8 UNORM
    static constexpr int bpp = 4;
    __device__ static float4 load(const uint8_t *base, size_t i)
    {
        uint32_t u = reinterpret_cast<const uint32_t *>(base)[i];
        const float s = 1.0f / 255.0f;
        return make_float4((float)(u & 255u) * s, (float)((u >> 8) & 255u) * s,
                           (float)((u >> 16) & 255u) * s, (float)(u >> 24) * s);
    }
    __device__ static void store(uint8_t *base, size_t i, float r, float g, float b)
    {
        uint32_t R = (uint32_t)(r * 255.0f + 0.5f), G = (uint32_t)(g * 255.0f + 0.5f),
                 B = (uint32_t)(b * 255.0f + 0.5f);
        reinterpret_cast<uint32_t *>(base)[i] = R | (G << 8) | (B << 16) | (255u << 24);
    }
};
template <> struct Pix<1> {           // RGBA32F
    static constexpr int bpp = 16;
    __device__ static float4 load(const uint8_t *base, size_t i)
    {
        return reinterpret_cast<const float4 *>(base)[i];
    }
    __device__ static void store(uint8_t *base, size_t i, float r, float g, float b)
    {
        reinterpret_cast<float4 *>(base)[i] = make_float4(r, g, b, 1.0f);
    }
};

// RGBToYIQ.shader:46-50 rows
__device__ __forceinline__ float luma(float4 c) { return 0.299f * c.x + 0.587f * c.y + 0.114f * c.z; }
__device__ __forceinline__ float chroma_i(float4 c) { return 0.596f * c.x + -0.274f * c.y + -0.322f * c.z; }
__device__ __forceinline__ float chroma_q(float4 c) { return 0.211f * c.x + -0.523f * c.y + 0.312f * c.z; }
__device__ __forceinline__ float sat(float v) { return fminf(fmaxf(v, 0.0f), 1.0f); }

// =========================================================================
// K1: luma rows -> half spectra of row pairs
// =========================================================================
template <int LOG2N, int FMT>
__global__ __launch_bounds__(wg_threads<LOG2N>())
void k_rows_fwd(const uint8_t *__restrict__ frames, size_t frame_bytes, int pairs_per_frame,
                int total_pairs, Geo g, const Tap4 *__restrict__ colTab,
                const Tap4 *__restrict__ rowTab, const c2 *__restrict__ tw,
                c2 *__restrict__ G, size_t g_stride)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = groups_per_wg<LOG2N>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = threadIdx.x / T, t = threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const int logical = xcd_remap(blockIdx.x, gridDim.x) * GPW + grp;
    const bool valid = logical < total_pairs;
    const int frame = valid ? logical / pairs_per_frame : 0;
    const int ra = valid ? 2 * (logical % pairs_per_frame) : 0;  // image row of pair
    const uint8_t *img = frames + (size_t)frame * frame_bytes;

    // vertical part of the separable resample: V_a, V_b over all source columns
    float *V = reinterpret_cast<float *>(lds);
    if (valid) {
        const Tap4 ta = rowTab[ra], tb = rowTab[ra + 1];
        for (int i = t; i < g.W; i += T) {
            float va = 0.0f, vb = 0.0f;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                va += ta.w[m] * luma(Pix<FMT>::load(img, (size_t)ta.idx[m] * g.W + i));
                vb += tb.w[m] * luma(Pix<FMT>::load(img, (size_t)tb.idx[m] * g.W + i));
            }
            V[i] = va;
            V[g.W + i] = vb;
        }
    }
    __syncthreads();
    c2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = t + j * T - g.x0;
        float ya = 0.0f, yb = 0.0f;
        if (valid && i >= 0 && i < g.W) {
            const Tap4 tc = colTab[i];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                ya += tc.w[c] * V[tc.idx[c]];
                yb += tc.w[c] * V[g.W + tc.idx[c]];
            }
        }
        v[j] = mk(ya, yb);
    }
    __syncthreads();
    fft_regs<LOG2N, -1>(v, t, lds, tw);
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[pad8(t + j * T)] = v[j];
    __syncthreads();
    if (!valid) return;
    c2 *Gf = G + (size_t)frame * g_stride;
    auto split_store = [&](int f) {
        c2 zf = lds[pad8(f)], zm = lds[pad8((N - f) & (N - 1))];
        // Y_a = (Z[f] + conj Z[N-f]) / 2 ;  Y_b = (Z[f] - conj Z[N-f]) / 2i
        float4 o;
        o.x = 0.5f * (zf.x + zm.x);
        o.y = 0.5f * (zf.y - zm.y);
        o.z = 0.5f * (zf.y + zm.y);
        o.w = -0.5f * (zf.x - zm.x);
        *reinterpret_cast<float4 *>(Gf + (size_t)f * g.H + ra) = o;
    };
#pragma unroll
    for (int j = 0; j < 4; ++j) split_store(t + j * T);
    if (t == 0) split_store(N / 2);
}

// =========================================================================
// K2: column FFT -> pyramid phase magnification -> column IFFT
// =========================================================================
__device__ __forceinline__ float smooth01(float x)   // HLSL smoothstep(0,1,x)
{
    float t = sat(x);
    return t * t * (3.0f - 2.0f * t);
}

// Radial masks of GeneratePyramidFilters (PyramidOperations.compute:25-87) and the
// per-level gate/phase rule of ProcessPyramidPhaseDifference
// (PyramidPhaseDifference.compute:58-101), summed over levels
// (AccumulatePyramidLevel, PyramidOperations.compute:111-128), for one bin.
template <int LOG2N>
__device__ __forceinline__ c2 pyramid_op(c2 c, c2 p, int fx, int fy, const Spec &sp)
{
    constexpr int N = 1 << LOG2N;
    const float ux = (float)fx / (float)N;
    const float uy = (float)(fy <= N / 2 ? fy : N - fy) / (float)N;
    const float fr = sqrtf(ux * ux + uy * uy);
    const float cm = sqrtf(c.x * c.x + c.y * c.y);
    const float pm = sqrtf(p.x * p.x + p.y * p.y);
    const float mn = fminf(cm, pm);
    float mpass = 0.0f, mmag = 0.0f;
    for (int i = 0; i < sp.L; ++i) {
        float m = 0.0f;
        if (i == 0) {
            if (fr > sp.maxF) m = 1.0f;
            else if (fr > sp.maxF * 0.8f) m = smooth01((fr - sp.maxF * 0.8f) / (sp.maxF * 0.2f));
        } else if (i == sp.L - 1) {
            if (fr < sp.minF) m = 1.0f;
            else if (fr < sp.minF * 1.2f) m = 1.0f - smooth01((fr - sp.minF) / (sp.minF * 0.2f));
        } else {
            const float lo = sp.lo[i], hi = sp.hi[i];
            if (fr >= lo && fr <= hi) {
                const float nrm = (fr - lo) / (hi - lo);
                m = 0.5f * (1.0f + cosf(2.0f * kPi * (nrm - 0.5f)));
            }
        }
        if (m > 0.0f) {
            if (i == 0 || i == sp.L - 1 || m * mn < sp.tau) mpass += m;
            else mmag += m;
        }
    }
    c2 a = scale(c, mpass);
    if (mmag > 0.0f) {
        // delta = wrap(arg p - arg c) = arg(p * conj c)
        const float dre = p.x * c.x + p.y * c.y;
        const float dim = p.y * c.x - p.x * c.y;
        const float d = atan2f(dim, dre);
        float s, co;
        sincosf(sp.S * d, &s, &co);
        a = add(a, scale(mul(c, mk(co, s)), mmag));
    }
    return scale(a, sp.inv_nn);
}

template <int LOG2N>
__global__ __launch_bounds__(wg_threads<LOG2N>())
void k_cols(const c2 *__restrict__ G, size_t g_stride, c2 *__restrict__ Q, size_t q_stride,
            const c2 *state_in, c2 *state_out, int nframes, int first_passthrough,
            Geo g, Spec sp, const c2 *__restrict__ tw)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = groups_per_wg<LOG2N>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = threadIdx.x / T, t = threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const int f_raw = blockIdx.x * GPW + grp;
    const bool valid = f_raw <= N / 2;
    const int f = valid ? f_raw : N / 2;

    c2 prev[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        prev[j] = state_in ? state_in[(size_t)f * N + t + j * T] : mk(0.0f, 0.0f);

    for (int fr = 0; fr < nframes; ++fr) {
        const c2 *Gc = G + (size_t)fr * g_stride + (size_t)f * g.H;
        c2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int rr = t + j * T - g.y0;
            v[j] = (rr >= 0 && rr < g.H) ? Gc[rr] : mk(0.0f, 0.0f);
        }
        fft_regs<LOG2N, -1>(v, t, lds, tw);
        if (fr == 0 && first_passthrough) {
#pragma unroll
            for (int j = 0; j < 8; ++j) prev[j] = v[j];
            continue;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const c2 a = pyramid_op<LOG2N>(v[j], prev[j], f, t + j * T, sp);
            prev[j] = v[j];
            v[j] = a;
        }
        fft_regs<LOG2N, +1>(v, t, lds, tw);
        if (valid) {
            c2 *Qc = Q + (size_t)fr * q_stride + (size_t)f * g.Hq;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = (t + j * T - g.rb + 2 * N) & (N - 1);
                if (k < g.Hn) Qc[k] = v[j];
            }
        }
    }
    if (valid && state_out) {
#pragma unroll
        for (int j = 0; j < 8; ++j) state_out[(size_t)f * N + t + j * T] = prev[j];
    }
}

// =========================================================================
// K3: row C2R IFFT -> |z| -> blur -> YIQ recombine -> RGB -> crop
// =========================================================================
template <int LOG2N> constexpr int k3_rows_per_step() { return 2 * groups_per_wg<LOG2N>(); }
template <int LOG2N> constexpr int k3_ring() { return k3_rows_per_step<LOG2N>() + 4; }

template <int LOG2N, int FMT>
__global__ __launch_bounds__(wg_threads<LOG2N>())
void k_rows_inv(const c2 *__restrict__ Q, size_t q_stride, const uint8_t *__restrict__ frames_in,
                uint8_t *__restrict__ frames_out, size_t frame_bytes, int frame0,
                int bands_per_frame, int BR, Geo g, Blur5 bw, const Tap4 *__restrict__ colTab,
                const Tap4 *__restrict__ rowTab, const c2 *__restrict__ tw)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = groups_per_wg<LOG2N>();
    constexpr int NT = wg_threads<LOG2N>();
    constexpr int P = k3_rows_per_step<LOG2N>(), RING = k3_ring<LOG2N>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = threadIdx.x / T, t = threadIdx.x % T;
    c2 *scratch = lds_all;                                   // GPW FFT areas
    c2 *lds = scratch + grp * lds_complex<N>();
    float *ring = reinterpret_cast<float *>(scratch + GPW * lds_complex<N>());
    float *scr_f = reinterpret_cast<float *>(scratch);

    const int band = blockIdx.x % bands_per_frame;
    const int frame = frame0 + blockIdx.x / bands_per_frame;
    const int i0 = band * BR;
    const int i1 = min(i0 + BR, g.H);
    const int kend = i1 + 4;                       // list rows [i0, kend)
    const c2 *Qf = Q + (size_t)frame * q_stride;
    const uint8_t *img = frames_in + (size_t)frame * frame_bytes;
    uint8_t *outp = frames_out + (size_t)frame * frame_bytes;

    int next_emit = i0;
    for (int s = i0; s < kend; s += P) {
        // ---- paired C2R inverse row FFTs ---------------------------------
        const int ka = s + 2 * grp, kb = ka + 1;
        const bool ha = ka < kend, hb = kb < kend;
        const int qa_row = ka % N, qb_row = kb % N;
        c2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int fq = t + j * T;
            const bool mirror = fq > N / 2;
            const int ff = mirror ? N - fq : fq;
            c2 qa = ha ? Qf[(size_t)ff * g.Hq + qa_row] : mk(0.0f, 0.0f);
            c2 qb = hb ? Qf[(size_t)ff * g.Hq + qb_row] : mk(0.0f, 0.0f);
            if (ff == 0 || ff == N / 2) { qa.y = 0.0f; qb.y = 0.0f; }
            if (mirror) { qa.y = -qa.y; qb.y = -qb.y; }
            v[j] = mk(qa.x - qb.y, qa.y + qb.x);     // Z = Qa + i Qb
        }
        fft_regs<LOG2N, +1>(v, t, lds, tw);
        // raw |z| rows of this group into its own scratch area
        float *raw = reinterpret_cast<float *>(lds);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            raw[t + j * T] = fabsf(v[j].x);
            raw[N + t + j * T] = fabsf(v[j].y);
        }
        __syncthreads();
        // ---- horizontal blur of the new rows into the ring ----------------
        for (int e = threadIdx.x; e < P * g.W; e += NT) {
            const int rl = e / g.W, X = e - rl * g.W;
            const int k = s + rl;
            if (k >= kend) continue;
            const float *rw = reinterpret_cast<const float *>(scratch + (rl >> 1) * lds_complex<N>()) + (rl & 1) * N;
            const int c = g.x0 + X;
            float acc = bw.w0 * rw[wrap_idx(c, N, g.edge)];
            acc += bw.w1 * (rw[wrap_idx(c - 1, N, g.edge)] + rw[wrap_idx(c + 1, N, g.edge)]);
            acc += bw.w2 * (rw[wrap_idx(c - 2, N, g.edge)] + rw[wrap_idx(c + 2, N, g.edge)]);
            ring[(k % RING) * g.W + X] = acc;
        }
        __syncthreads();
        // ---- emit finished output rows -------------------------------------
        const int avail = min(s + P, kend);        // list rows < avail are in the ring
        while (next_emit < i1 && next_emit + 4 < avail) {
            const int i = next_emit;
            const Tap4 tr = rowTab[i];
            float *VI = scr_f, *VQ = scr_f + g.W;
            for (int x = threadIdx.x; x < g.W; x += NT) {
                float vi = 0.0f, vq = 0.0f;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float4 px = Pix<FMT>::load(img, (size_t)tr.idx[m] * g.W + x);
                    vi += tr.w[m] * chroma_i(px);
                    vq += tr.w[m] * chroma_q(px);
                }
                VI[x] = vi;
                VQ[x] = vq;
            }
            __syncthreads();
            // canvas row Y = y0 + i; a blur tap at wrapped/clamped canvas row cy
            // is the band's sequential list row in [i, i+4] congruent to cy - rb.
            const int Y = g.y0 + i;
            int sl[5];
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                const int cy = wrap_idx(Y + d - 2, N, g.edge);
                const int kk = (cy - g.rb + 2 * N) & (N - 1);
                const int kseq = i + ((kk - i + 2 * N) & (N - 1));
                sl[d] = (kseq % RING) * g.W;
            }
            for (int X = threadIdx.x; X < g.W; X += NT) {
                float yb = bw.w0 * ring[sl[2] + X];
                yb += bw.w1 * (ring[sl[1] + X] + ring[sl[3] + X]);
                yb += bw.w2 * (ring[sl[0] + X] + ring[sl[4] + X]);
                const Tap4 tc = colTab[X];
                float ci = 0.0f, cq = 0.0f;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    ci += tc.w[c] * VI[tc.idx[c]];
                    cq += tc.w[c] * VQ[tc.idx[c]];
                }
                // YIQToRGB.shader:51-76 + saturate
                const float r = sat(1.0f * yb + 0.956f * ci + 0.621f * cq);
                const float gg = sat(1.0f * yb + -0.272f * ci + -0.647f * cq);
                const float b = sat(1.0f * yb + -1.106f * ci + 1.703f * cq);
                Pix<FMT>::store(outp, (size_t)i * g.W + X, r, gg, b);
            }
            __syncthreads();
            ++next_emit;
        }
    }
}

// =========================================================================
// synthetic stream, RGBA8
// =========================================================================
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_synth(uint8_t *out, int W, int H, int t0, int count, uint64_t seed, int gray)
{
    const size_t npx = (size_t)W * H;
    const size_t total = npx * count;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total;
         e += (size_t)gridDim.x * blockDim.x) {
        const int fr = (int)(e / npx);
        const size_t p = e - (size_t)fr * npx;
        const int y = (int)(p / W), x = (int)(p - (size_t)y * W);
        const double two_pi = 6.283185307179586;
        const double d = 0.5 * sin(two_pi * 0.05 * (t0 + fr));
        const double sx = sin(two_pi * (x + d) / 37.0), cy = cos(two_pi * y / 53.0);
        const double gc[3] = {1.0, 0.8, 0.6};
        uint32_t packed = 255u << 24;
        for (int ch = 0; ch < 3; ++ch) {
            const int cc = gray ? 0 : ch;
            const uint64_t h = splitmix64(seed ^ ((uint64_t)p * 3u + (uint64_t)cc));
            const double u = (double)(h >> 40) * (1.0 / 16777216.0);
            double v = 0.4 + 0.3 * sx * cy * gc[cc] + 0.15 * u;
            v = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
            packed |= (uint32_t)floor(v * 255.0 + 0.5) << (8 * ch);
        }
        reinterpret_cast<uint32_t *>(out)[e] = packed;
    }
}

}  // namespace mm
