// mm_kernels.hpp — the three HIP kernels of one magnified frame (gfx950).
//
// Data flow per frame (N = padded square size, F = N/2+1 half-spectrum columns):
//   K1 k_rows_fwd : RGBA frame --(luma, stretch+pad bilinear, Hann window)-->
//                   real rows --(paired real FFT)--> G[f][row]       (f < F)
//   K2 k_cols     : G column --FFT--> F_t --(pyramid phase op vs F_{t-1})-->
//                   A --IFFT--> Q[row/2][f][row%2]; F_t becomes the state.
//                   One FFT group owns a column for a whole chunk of frames, so
//                   F_{t-1} stays in registers between frames.
//   K3 k_rows_inv : Q rows --(paired C2R IFFT)--> |z| --(5-tap H blur)--> Yh
//   K4 k_compose  : Yh --(5-tap V blur)--, input --(I/Q resample)--> YIQ->RGB,
//                   saturate, crop --> RGBA frame
// Reference stages replaced (MotionMagnificationProcessor.cs:145-206): a4-a18 of
// SURVEY.md §8(a).  The pyramid levels are applied pointwise in frequency
// (SURVEY.md §7): arg(m_i F) = arg F for real m_i >= 0, so one atan2/sincos per
// bin serves every level.
#pragma once
#include "mm_fft.hpp"
#include "mm_srgb.hpp"
#include <stdint.h>
#include <type_traits>

namespace mm {

constexpr int kMaxLevels = 16;
constexpr float kPi = 3.14159265359f;  // PyramidOperations.compute:5

struct Tap4 {         // composite stretch+pad bilinear taps incl. Hann factor
    int idx[4];
    float w[4];
};

struct Geo {
    int W, H, N;
    int x0, y0;       // image placement inside the canvas (PadTexture .cs:360-363):
                      // floor((N - W) / 2); for odd N - W the quad's left edge is at
                      // x0 + 0.5 and CropTexture samples between two texels
    int ox, oy;       // W, H odd (k_compose_odd)
    int Hg;           // rows per G column (H rounded up to even: K1 writes row pairs)
    int Wy;           // Yh columns (W + ox: the crop's second texel)
    int rb;           // canvas row of Q list index 0 (= y0 - 2)
    int Hn;           // rows kept in Q (= min(H + 4, N))
    int Hq;           // Hn rounded up to whole Q tiles (TK rows)
    int Qs;           // Q bins per tile row (N/2 + 2; q_index)
    int TK;           // rows per Q tile (q_tile_v)
    int edge;         // 0 repeat, 1 clamp
};

struct Spec {
    int mode;               // MM_MODE_PYRAMID (0) | MM_MODE_STANDARD (1)
    // standard mode band-pass (PhaseDifferenceComputeShader.compute:88-122)
    int bp_apply;
    float bp_low, bp_high, bp_steep, bp_sens, bp_edge;
    float bp_inv_low, bp_inv_1mhigh, bp_inv_band;
    int L;
    float minF, maxF, S, tau2, inv_nn;
    float S_rev;            // S / (2 pi): phase scale in revolutions (v_sin/v_cos)
    int S_pow;              // |S| when S is an integer, else -1 (k_cols SP: the power form)
    float S_sgn;            // sign of S (+1 / -1) for the power form
    float tau2_nn;          // tau2 * inv_nn^2 (gate on masks pre-scaled by inv_nn)
    float hp_lo, hp_inv;    // high-pass ramp start maxF*0.8, 1/(maxF*0.2)
    float lp_hi, lp_inv;    // low-pass ramp end minF*1.2, 1/(minF*0.2)
    float lo[kMaxLevels], hi[kMaxLevels], inv_w[kMaxLevels];  // middle bands
    // MM_MODE_STEERABLE (mm_steer.hpp): orientations, filter, IIR coefficients,
    // orientation unit vectors (cos, sin of 2 pi k / O)
    int O, filt;
    float r_low, r_high;
    float ang_c[8], ang_s[8];
};

struct Blur5 { float w0, w1, w2; };  // taps at 0, +-1, +-2 texels

constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x / 2); }
template <int LOG2N> constexpr int fft_T() { return (1 << LOG2N) / 8; }
template <int LOG2N> constexpr int groups_per_wg() { return fft_T<LOG2N>() >= 256 ? 1 : 256 / fft_T<LOG2N>(); }
template <int LOG2N> constexpr int wg_threads() { return groups_per_wg<LOG2N>() * fft_T<LOG2N>(); }
// at least MIN FFT groups per workgroup (within 1024 threads)
constexpr int groups_at_least_v(int log2n, int min)
{
    const int T = (1 << log2n) / 8, base = T >= 256 ? 1 : 256 / T;
    if (base >= min) return base;
    int g = min;
    while (g > base && T * g > 1024) g /= 2;
    return g;
}
template <int LOG2N, int MIN> constexpr int groups_at_least() { return groups_at_least_v(LOG2N, MIN); }
#ifndef MM_K1_GROUPS
#define MM_K1_GROUPS 2
#endif
#ifndef MM_K2_GROUPS
#define MM_K2_GROUPS 2
#endif
#ifndef MM_K3_GROUPS
#define MM_K3_GROUPS 1
#endif
// K3 runs one Q tile (TK = 2 * groups rows) per workgroup
template <int LOG2N> constexpr int k3_groups() { return groups_at_least<LOG2N, MM_K3_GROUPS>(); }
template <int LOG2N> constexpr int k3_threads() { return k3_groups<LOG2N>() * fft_T<LOG2N>(); }
// (MM_Q_TILE_8K: rows per Q tile at N = 8192, where K3 runs one row pair per
// workgroup: 4 gives K2 32-B Q pieces from its one column per workgroup.
// 5120x2880 same-call, tiles of 2 / 4 / 8 rows: K2 193-196 / 185 / 179-184 us,
// K3 31 / 35 / 45 us per frame, 3.04-3.11k / 3.13k / 3.04-3.10k frames/s,
// profiles/r06k_q_tile_8k_ab.txt)
#ifndef MM_Q_TILE_8K
#define MM_Q_TILE_8K 4
#endif
constexpr int q_tile_v(int log2n) { return log2n == 13 ? MM_Q_TILE_8K : 2 * groups_at_least_v(log2n, MM_K3_GROUPS); }
template <int LOG2N> constexpr int q_tile() { return q_tile_v(LOG2N); }
// K1 runs >= 2 row pairs per workgroup so that G receives 32-B pieces
template <int LOG2N> constexpr int k1_groups() { return groups_at_least<LOG2N, MM_K1_GROUPS>(); }
template <int LOG2N> constexpr int k1_threads() { return k1_groups<LOG2N>() * fft_T<LOG2N>(); }
// LAT: short launches (one frame: the drop-in call) run one row pair per
// workgroup, so that twice as many workgroups spread over the CUs and none
// waits behind another's latency chain (G then leaves as 16-B pieces)
template <int LOG2N, bool LAT> constexpr int k1_gpw() { return LAT && fft_T<LOG2N>() >= 64 ? 1 : k1_groups<LOG2N>(); }

__device__ __forceinline__ int wrap_idx(int i, int n, int edge)
{
    if (edge) return i < 0 ? 0 : (i >= n ? n - 1 : i);
    int r = i % n;
    return r < 0 ? r + n : r;
}

// Wrap an index known to lie in [-1, n] (resample taps) with the edge mode.
__device__ __forceinline__ int wrap_near(int i, int n, int edge)
{
    if (i < 0) return edge ? 0 : i + n;
    if (i >= n) return edge ? n - 1 : i - n;
    return i;
}

// Same-XCD blocks (b % 8 equal under round-robin dispatch) get consecutive ids.
__device__ __forceinline__ int xcd_remap(int b, int nb)
{
    int q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Like xcd_remap, but each XCD owns runs of G consecutive blocks spread over the
// whole range (run k on XCD k % 8): same-XCD neighbours still share L2 lines,
// and work that varies smoothly with the block index is balanced over XCDs.
// Falls back to xcd_remap when nb is not a multiple of 8 G.
template <int G>
__device__ __forceinline__ int xcd_interleave(int b, int nb)
{
    if (nb % (8 * G) != 0) return xcd_remap(b, nb);
    const int x = b % 8, q = b / 8;
    return ((q / G) * 8 + x) * G + q % G;
}

// Access at a 32-bit BYTE offset from a (workgroup-uniform) base: matches the
// scalar-base + 32-bit vector-offset form of global loads/stores (an index
// scaled as zext(i) * sizeof(T) needs 64-bit address math per access).
template <class T>
__device__ __forceinline__ T ld_off(const void *base, unsigned byte_off)
{
    return *reinterpret_cast<const T *>(reinterpret_cast<const uint8_t *>(base) + byte_off);
}
template <class T>
__device__ __forceinline__ void st_off(void *base, unsigned byte_off, T v)
{
    *reinterpret_cast<T *>(reinterpret_cast<uint8_t *>(base) + byte_off) = v;
}

// Stores of whole 128-B lines that nothing reads back soon (output frames, Yh
// rows): non-temporal, so that they stream out under the kernel instead of
// sitting dirty in L2 for the write-back at the end of the kernel (same-call:
// K34 -4 %, one-frame K3 / K4 -5 % / -7 %).  The partial-line hand-off stores
// (G, Q) stay write-back: their pieces are merged in L2 (non-temporal there:
// K1 3x, K2 1.8x slower, profiles/r03g_nt_ab.txt).
template <class T>
__device__ __forceinline__ void st_stream(void *base, unsigned byte_off, T v)
{
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    void *p = reinterpret_cast<uint8_t *>(base) + byte_off;
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    if constexpr (sizeof(T) == 16) {
        u32x4 w;
        __builtin_memcpy(&w, &v, 16);
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
    } else if constexpr (sizeof(T) == 8) {
        u32x2 w;
        __builtin_memcpy(&w, &v, 8);
        __builtin_nontemporal_store(w, reinterpret_cast<u32x2 *>(p));
    } else {
        static_assert(sizeof(T) == 4, "st_stream: 4, 8 or 16 bytes");
        unsigned w;
        __builtin_memcpy(&w, &v, 4);
        __builtin_nontemporal_store(w, reinterpret_cast<unsigned *>(p));
    }
}

// |z| rows of the row IFFTs (K3 four-wide path, K34, K34o) start kZShift
// floats into their LDS row, so that the blur taps c-2 .. c+5 of an aligned
// quad c = x0 + 4q (x0 % 4 == 0) are two 16-B aligned ds_read_b128.
constexpr int kZShift = 2;

// Q hand-off (K2 -> K3): element (row k, bin f) of a frame, stored in tiles of
// TK rows: [k/TK][f][k%TK], Qs bins per tile row.  A K2 workgroup's columns of
// one tile are contiguous (GPW*TK*8 bytes: whole 128-B lines at TK = 8), and
// K3's TK/2 row pairs of a bin are one contiguous TK*8-byte block.
__device__ __forceinline__ size_t q_index(const Geo &g, int k, int f)
{
    return ((size_t)(k / g.TK) * g.Qs + f) * g.TK + (k % g.TK);
}

#ifdef MM_ASM_MARKS
#define MM_MARK(x) asm volatile("; " x)
#else
#define MM_MARK(x)
#endif

// ---- pixel access -------------------------------------------------------
template <int FMT> struct Pix;
template <> struct Pix<0> {           // RGBA8 UNORM
    static constexpr int bpp = 4;
    using raw_t = uint32_t;             // keep loads raw in registers, convert at use
    __device__ static raw_t raw(const uint8_t *base, size_t i)
    {
        return reinterpret_cast<const uint32_t *>(base)[i];
    }
    __device__ static float4 cvt(raw_t u)
    {
        const float s = 1.0f / 255.0f;
        return make_float4((float)(u & 255u) * s, (float)((u >> 8) & 255u) * s,
                           (float)((u >> 16) & 255u) * s, (float)(u >> 24) * s);
    }
    __device__ static float4 load(const uint8_t *base, size_t i) { return cvt(raw(base, i)); }
    __device__ static uint32_t pack(float r, float g, float b)
    {
        uint32_t R = (uint32_t)(r * 255.0f + 0.5f), G = (uint32_t)(g * 255.0f + 0.5f),
                 B = (uint32_t)(b * 255.0f + 0.5f);
        return R | (G << 8) | (B << 16) | (255u << 24);
    }
    __device__ static void store(uint8_t *base, unsigned i, float r, float g, float b)
    {
        st_stream<uint32_t>(base, i * 4u, pack(r, g, b));
    }
    // r, g, b in code units (255 x the UNORM value), unclamped: three
    // v_cvt_pk_u8_f32, each rounding to nearest and clamping to 0 .. 255 into
    // its byte lane (the compose kernels' pack, kOut255)
    __device__ static uint32_t pack255(float r, float g, float b)
    {
        const uint32_t a = __builtin_amdgcn_cvt_pk_u8_f32(r, 0u, 0xff000000u);
        return __builtin_amdgcn_cvt_pk_u8_f32(b, 2u, __builtin_amdgcn_cvt_pk_u8_f32(g, 1u, a));
    }
};
template <> struct Pix<1> {           // RGBA32F
    static constexpr int bpp = 16;
    using raw_t = float4;
    __device__ static raw_t raw(const uint8_t *base, size_t i)
    {
        return reinterpret_cast<const float4 *>(base)[i];
    }
    __device__ static float4 cvt(raw_t v) { return v; }
    __device__ static float4 load(const uint8_t *base, size_t i) { return raw(base, i); }
    __device__ static void store(uint8_t *base, unsigned i, float r, float g, float b)
    {
        st_stream<float4>(base, i * 16u, make_float4(r, g, b, 1.0f));
    }
};
// RGBA16F: linear half floats, as the reference camera's HDR render target
// (ARGBHalf: Assets/Scenes/SampleScene.unity:663 m_HDR, linear colour space
// ProjectSettings/ProjectSettings.asset:50) hands them to OnRenderImage
// (.cs:101).  Values above 1 pass unclipped up to the reference's saturate
// (YIQToRGB.shader); the output is rounded to half (round to nearest even).
template <> struct Pix<2> {
    static constexpr int bpp = 8;
    using raw_t = uint2;
    __device__ static raw_t raw(const uint8_t *base, size_t i)
    {
        return reinterpret_cast<const uint2 *>(base)[i];
    }
    __device__ static float h2f(unsigned bits)
    {
        return (float)__builtin_bit_cast(_Float16, (unsigned short)(bits & 0xffffu));
    }
    __device__ static unsigned f2h(float v)
    {
        return (unsigned)__builtin_bit_cast(unsigned short, (_Float16)v);
    }
    __device__ static float4 cvt(raw_t u)
    {
        return make_float4(h2f(u.x), h2f(u.x >> 16), h2f(u.y), h2f(u.y >> 16));
    }
    __device__ static uint2 pack(float r, float g, float b)
    {
        return make_uint2(f2h(r) | f2h(g) << 16, f2h(b) | 0x3C00u << 16);   // alpha 1.0
    }
    __device__ static void store(uint8_t *base, unsigned i, float r, float g, float b)
    {
        st_stream<uint2>(base, i * 8u, pack(r, g, b));
    }
};
// RGBA8 sRGB: an 8-bit sRGB render target under Unity's Linear colour space
// is sampled as linear light and encoded on write, so the pipeline sees
// linear values.  Decode: the exact 256-entry table (tools/gen_srgb.py);
// encode of a saturated value: 255 srgb(v) rounded, found from the pow
// approximation and corrected by one step against the exact thresholds
// kSrgbThr (the approximation is within one code of the exact one).
template <> struct Pix<3> {
    static constexpr int bpp = 4;
    using raw_t = uint32_t;
    __device__ static raw_t raw(const uint8_t *base, size_t i)
    {
        return reinterpret_cast<const uint32_t *>(base)[i];
    }
    __device__ static float4 cvt(raw_t u)
    {
        return make_float4(kSrgbDec[u & 255u], kSrgbDec[(u >> 8) & 255u], kSrgbDec[(u >> 16) & 255u],
                           (float)(u >> 24) * (1.0f / 255.0f));
    }
    __device__ static uint32_t enc(float v)
    {
        const float s = v <= 0.0031308f ? 12.92f * v : 1.055f * __powf(v, 1.0f / 2.4f) - 0.055f;
        int b = min(max((int)(s * 255.0f + 0.5f), 0), 255);
        b += v >= kSrgbThr[b + 1] ? 1 : 0;
        b -= v < kSrgbThr[b] ? 1 : 0;
        return (uint32_t)b;
    }
    __device__ static uint32_t pack(float r, float g, float b)
    {
        return enc(r) | (enc(g) << 8) | (enc(b) << 16) | (255u << 24);
    }
    __device__ static void store(uint8_t *base, unsigned i, float r, float g, float b)
    {
        st_stream<uint32_t>(base, i * 4u, pack(r, g, b));
    }
};
// saturated before the store: the UNORM destinations (RGBA8, RGBA8 sRGB)
template <int FMT> constexpr bool kUnorm = FMT == 0 || FMT == 3;
// MM_OUT255=1 (diagnostic): RGBA8 compose in code units.  The chroma
// conversion drops its 1/255, the vertical luma blur carries 255 in its
// weights, and YIQToRGB's saturate and the x255 + round of the UNORM write
// become the clamp and round-to-nearest-even of v_cvt_pk_u8_f32
// (Pix<0>::pack255; tools/cvtpk_probe.hip): 3 VALU per pixel instead of 10,
// K34 -10 % VALU, parity green, but 4 spills at its 128-VGPR bound at
// N = 2048: same-call K34 6.09 -> 6.24 us per frame at 1080p, equal at 2160p
// (profiles/r06f_out255_ab.txt).  Off by default.
#ifndef MM_OUT255
#define MM_OUT255 0
#endif
template <int FMT> constexpr bool kOut255 = MM_OUT255 && FMT == 0;
// the vertical blur weights of the compose (255 x for kOut255; scalar
// registers like the kernel argument they come from, not 3 VGPRs)
__device__ __forceinline__ float uniform_f(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}
template <int FMT> __device__ __forceinline__ Blur5 vblur_w(Blur5 b)
{
    if constexpr (kOut255<FMT>)
        return Blur5{uniform_f(b.w0 * 255.0f), uniform_f(b.w1 * 255.0f), uniform_f(b.w2 * 255.0f)};
    else return b;
}

// RGBToYIQ.shader:46-50 rows
__device__ __forceinline__ float luma(float4 c) { return 0.299f * c.x + 0.587f * c.y + 0.114f * c.z; }
__device__ __forceinline__ float chroma_i(float4 c) { return 0.596f * c.x + -0.274f * c.y + -0.322f * c.z; }
__device__ __forceinline__ float chroma_q(float4 c) { return 0.211f * c.x + -0.523f * c.y + 0.312f * c.z; }
__device__ __forceinline__ float sat(float v) { return fminf(fmaxf(v, 0.0f), 1.0f); }

// Y of a raw pixel (RGBA8: 1/255 folded into the RGBToYIQ row).
// K1's luma in units of kLumaUnit<FMT>: RGBA8 as the exact integer
// 299 R + 587 G + 114 B (two v_dot4_u32_u8: 299 = 256 + 43, 587 = 2 * 256 + 75,
// and one convert; RGBToYIQ's 0.299/0.587/0.114 of R/255 ... times 255000),
// whose unit 1/255000 folds into the resample weights; RGBA32F as luma().
template <int FMT> constexpr float kLumaUnit = FMT == 0 ? 1.0f / 255000.0f : 1.0f;
template <int FMT>
__device__ __forceinline__ float luma_units(typename Pix<FMT>::raw_t u)
{
    if constexpr (FMT == 0) {
        const unsigned hi = __builtin_amdgcn_udot4(u, 0x00000201u, 0u, false);    // R + 2 G
        return (float)__builtin_amdgcn_udot4(u, 0x00724B2Bu, hi << 8, false);   // + 43 R + 75 G + 114 B
    } else {
        return luma(Pix<FMT>::cvt(u));
    }
}

// (I, Q) of a raw pixel.  RGBA8: the 1/255 of the UNORM read is folded into the
// RGBToYIQ coefficients (3 byte converts + 6 FMAs).
template <int FMT>
__device__ __forceinline__ float2 chroma_iq(typename Pix<FMT>::raw_t u)
{
    if constexpr (FMT == 0) {
        constexpr float k = 1.0f / 255.0f;
        const float r = (float)(u & 255u), gg = (float)((u >> 8) & 255u), b = (float)((u >> 16) & 255u);
        return make_float2((0.596f * k) * r + (-0.274f * k) * gg + (-0.322f * k) * b,
                           (0.211f * k) * r + (-0.523f * k) * gg + (0.312f * k) * b);
    } else {
        const float4 c = Pix<FMT>::cvt(u);
        return make_float2(chroma_i(c), chroma_q(c));
    }
}

// Packed-FP32 pixel math of the compose stage (K4 and K34 share it, so the
// fused and unfused outputs stay bitwise equal): (I, Q) is one c2, and every
// weighted sum is written in the same left-to-right order as its scalar form,
// so each lane computes the scalar form's fma chain exactly (v_pk_fma_f32 /
// v_pk_mul_f32 with a broadcast scalar operand: half the VALU instructions).
template <int FMT>
__device__ __forceinline__ c2 chroma_iq2(typename Pix<FMT>::raw_t u)
{
    if constexpr (FMT == 0) {
        constexpr float k = kOut255<FMT> ? 1.0f : 1.0f / 255.0f;
        const float r = (float)(u & 255u), gg = (float)((u >> 8) & 255u), b = (float)((u >> 16) & 255u);
        return mk(0.596f * k, 0.211f * k) * r + mk(-0.274f * k, -0.523f * k) * gg + mk(-0.322f * k, 0.312f * k) * b;
    } else {
        const float4 c = Pix<FMT>::cvt(u);
        return mk(0.596f, 0.211f) * c.x + mk(-0.274f, -0.523f) * c.y + mk(-0.322f, 0.312f) * c.z;
    }
}

// YIQToRGB.shader:51-76 + saturate for one pixel: R and G as one pair, B alone
// (B as two FMAs: written as 1 yb + ..., the contraction fused the 1 yb
// product and left a multiply and a subtract)
// (kOut255: yb, cc and the result in code units, the saturate left to the pack)
template <int FMT>
__device__ __forceinline__ void yiq_rgb(float yb, c2 cc, float &rr, float &gg, float &bb)
{
    const c2 rg = mk(yb, yb) + mk(0.956f, -0.272f) * cc.x + mk(0.621f, -0.647f) * cc.y;
    const float b = fmaf(1.703f, cc.y, fmaf(-1.106f, cc.x, yb));
    if constexpr (kOut255<FMT>) {
        rr = rg.x; gg = rg.y; bb = b;
    } else {
        rr = sat(rg.x); gg = sat(rg.y); bb = sat(b);
    }
}
// the compose kernels' packed pixel and single-pixel store of yiq_rgb's result
template <int FMT> __device__ __forceinline__ uint32_t out_pack(float r, float g, float b)
{
    if constexpr (kOut255<FMT>) return Pix<FMT>::pack255(r, g, b);
    else return Pix<FMT>::pack(r, g, b);
}
template <int FMT> __device__ __forceinline__ void out_store(uint8_t *base, unsigned i, float r, float g, float b)
{
    if constexpr (kOut255<FMT>) st_stream<uint32_t>(base, i * 4u, Pix<FMT>::pack255(r, g, b));
    else Pix<FMT>::store(base, i, r, g, b);
}

// =========================================================================
// K1: luma rows -> half spectra of row pairs
// =========================================================================
// GEN (odd W or H): the composite taps of a pixel span i-2 .. i+1 and are
// read as unmerged Tap4 entries (colT / rowT) instead of the 3-tap tables.
#ifndef MM_K1_COOP
#define MM_K1_COOP 1   // batch form: the two row pairs' source rows loaded once
#endif
template <int LOG2N, int FMT, bool GEN = false, bool LAT = false>
__global__ __launch_bounds__((k1_gpw<LOG2N, LAT>() * fft_T<LOG2N>()))
void k_rows_fwd(const uint8_t *__restrict__ frames, size_t frame_bytes, int pairs_per_frame,
                int total_pairs, Geo g, const float4 *__restrict__ colW3,
                const float4 *__restrict__ rowW3, const Tap4 *__restrict__ colT,
                const Tap4 *__restrict__ rowT, const c2 *__restrict__ tw,
                c2 *__restrict__ G, size_t g_stride)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = k1_gpw<LOG2N, LAT>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    // group index: wave-uniform (scalar) when a group spans whole waves
    const int grp = GPW == 1 ? 0 : (T % 64 == 0 ? __builtin_amdgcn_readfirstlane(threadIdx.x / T)
                                               : threadIdx.x / T);
    const int t = GPW == 1 ? threadIdx.x : threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const int lblk = xcd_remap(blockIdx.x, gridDim.x) * GPW;   // block's first pair
    const int logical = lblk + grp;
    const bool valid = logical < total_pairs;
    const int frame = valid ? logical / pairs_per_frame : 0;
    const int ra = valid ? 2 * (logical % pairs_per_frame) : 0;  // image row of pair
    const uint8_t *img = frames + (size_t)frame * frame_bytes;

    // vertical part of the separable resample: V_a, V_b over all source columns.
    // Taps of image row r lie on source rows r-1..r+1 (w3 tables), so the pair
    // (ra, ra+1) reads the 4 source rows ra-1..ra+2.
    float *V = reinterpret_cast<float *>(lds);   // GEN: [2][W] (rows a, b)
    c2 *V2 = lds;                                 // 3-tap path: [W] (row a, row b) pairs
    using raw_t = typename Pix<FMT>::raw_t;
    constexpr int BPP = Pix<FMT>::bpp;
    // one-pair workgroups (LAT: short launches, latency-bound) issue the
    // column taps and twiddles with the pixel loads instead of one dependent
    // round trip each after them (batch launches: K1 +5 %, registers held
    // across the loads)
    c2 wb[kTwSlots];
    float4 cw[8];
    if constexpr (LAT && !GEN) {
        preload_twiddles_wl<LOG2N>(wb, t, tw);
#pragma unroll
        for (int j = 0; j < 8; ++j) cw[j] = colW3[min(max(t + j * T - g.x0, 0), g.W - 1)];
    }
    // RGBA8 / RGBA16F: all 32 pixel loads of the thread in one batch; RGBA32F
    // (4x the registers of RGBA8): two batches of 16
    constexpr int UB = BPP == 16 ? 4 : 8;
    if constexpr (GEN) {
        if (valid) {
            Tap4 ta = rowT[ra];
            Tap4 tb = ra + 1 < g.H ? rowT[ra + 1] : ta;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                ta.w[m] *= kLumaUnit<FMT>;
                tb.w[m] = ra + 1 < g.H ? tb.w[m] * kLumaUnit<FMT> : 0.0f;   // the zero row of odd H
            }
            unsigned pa[4], pb[4];   // source row byte offsets
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                pa[m] = (unsigned)(wrap_near(ta.idx[m], g.H, g.edge) * g.W * BPP);
                pb[m] = (unsigned)(wrap_near(tb.idx[m], g.H, g.edge) * g.W * BPP);
            }
            for (int i = t; i < g.W; i += T) {
                float va = 0.0f, vb = 0.0f;
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    va += ta.w[m] * luma_units<FMT>(ld_off<raw_t>(img, pa[m] + (unsigned)i * BPP));
                    vb += tb.w[m] * luma_units<FMT>(ld_off<raw_t>(img, pb[m] + (unsigned)i * BPP));
                }
                V[i] = va;
                V[g.W + i] = vb;
            }
        }
    } else if (MM_K1_COOP && GPW == 2 && !LAT && pairs_per_frame % 2 == 0) {
        // Batch form, the two groups' row pairs in one frame (uniform test):
        // the workgroup's 4 rows r0 .. r0+3 read the 6 source rows r0-1 ..
        // r0+4 once, shared (each group alone read 4: 8 row loads for 4
        // rows); thread tid of the 2T does N/(2T) columns for both groups.
        // Same lumas and the same packed expressions per group as below: the
        // V2 values are bitwise the per-group form's.
        if (valid) {
            const int r0 = ra - 2 * grp;   // group 0's pair (same frame: pairs_per_frame even)
            c2 w[2][3];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                float4 wa = rowW3[r0 + 2 * q], wb = rowW3[r0 + 2 * q + 1];
                wa.x *= kLumaUnit<FMT>, wa.y *= kLumaUnit<FMT>, wa.z *= kLumaUnit<FMT>;
                wb.x *= kLumaUnit<FMT>, wb.y *= kLumaUnit<FMT>, wb.z *= kLumaUnit<FMT>;
                w[q][0] = mk(wa.x, wb.x);
                w[q][1] = mk(wa.y, wb.y);
                w[q][2] = mk(wa.z, wb.z);
            }
            const uint8_t *rowp[6];   // workgroup-uniform source row pointers
#pragma unroll
            for (int d = 0; d < 6; ++d) rowp[d] = img + (unsigned)(wrap_near(r0 - 1 + d, g.H, g.edge) * g.W * BPP);
            constexpr int CT = N / (2 * T);          // columns per thread (W <= N)
            constexpr int CB = BPP == 16 ? 1 : CT;   // columns per load batch
            c2 *V2g1 = lds_all + lds_complex<N>();
#pragma unroll
            for (int h = 0; h < CT / CB; ++h) {
                __builtin_amdgcn_sched_barrier(0);
                raw_t px[CB][6];
#pragma unroll
                for (int u = 0; u < CB; ++u) {
                    const unsigned off = (unsigned)min((int)threadIdx.x + (h * CB + u) * 2 * T, g.W - 1) * BPP;
#pragma unroll
                    for (int d = 0; d < 6; ++d) px[u][d] = ld_off<raw_t>(rowp[d], off);
                }
#pragma unroll
                for (int u = 0; u < CB; ++u) {
                    const int i = (int)threadIdx.x + (h * CB + u) * 2 * T;
                    float l[6];
#pragma unroll
                    for (int d = 0; d < 6; ++d) l[d] = luma_units<FMT>(px[u][d]);
                    if (i < g.W) {
                        lds_all[i] = w[0][0] * mk(l[0], l[1]) + w[0][1] * mk(l[1], l[2]) + w[0][2] * mk(l[2], l[3]);
                        V2g1[i] = w[1][0] * mk(l[2], l[3]) + w[1][1] * mk(l[3], l[4]) + w[1][2] * mk(l[4], l[5]);
                    }
                }
            }
        }
    } else if (valid) {
        // odd H: the last pair's second row is outside the image (zero)
        float4 wa = rowW3[ra], wb = ra + 1 < g.H ? rowW3[ra + 1] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        wa.x *= kLumaUnit<FMT>, wa.y *= kLumaUnit<FMT>, wa.z *= kLumaUnit<FMT>;
        wb.x *= kLumaUnit<FMT>, wb.y *= kLumaUnit<FMT>, wb.z *= kLumaUnit<FMT>;
        // rows a and b as one packed pair: (a, b) = (wa.x, wb.x) (l0, l1) +
        // (wa.y, wb.y) (l1, l2) + (wa.z, wb.z) (l2, l3), per lane the scalar
        // forms' fma chains (half the VALU instructions, one 8-B LDS store)
        const c2 w0 = mk(wa.x, wb.x), w1 = mk(wa.y, wb.y), w2 = mk(wa.z, wb.z);
        const uint8_t *rowp[4];   // workgroup-uniform source row pointers
#pragma unroll
        for (int d = 0; d < 4; ++d) rowp[d] = img + (unsigned)(wrap_near(ra - 1 + d, g.H, g.edge) * g.W * BPP);
        // W <= N = 8T: at most 8 columns per thread
#pragma unroll
        for (int h = 0; h < 8 / UB; ++h) {
            __builtin_amdgcn_sched_barrier(0);
            raw_t px[UB][4];
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const unsigned off = (unsigned)min(t + (h * UB + u) * T, g.W - 1) * BPP;
#pragma unroll
                for (int d = 0; d < 4; ++d) px[u][d] = ld_off<raw_t>(rowp[d], off);
            }
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const int i = t + (h * UB + u) * T;
                float l[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) l[d] = luma_units<FMT>(px[u][d]);
                if (i < g.W) V2[i] = w0 * mk(l[0], l[1]) + w1 * mk(l[1], l[2]) + w2 * mk(l[2], l[3]);
            }
        }
    }
    __syncthreads();
    // all 8 colW3 loads in one batch (two batches of 4: one more dependent
    // L2 round trip per pair, K1 +5 %)
    c2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = t + j * T - g.x0;                    // image column
        const int ic = min(max(i, 0), g.W - 1);
        float ya = 0.0f, yb = 0.0f;
        if constexpr (GEN) {
            const Tap4 tc = colT[ic];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int c = wrap_near(tc.idx[m], g.W, g.edge);
                ya += tc.w[m] * V[c];
                yb += tc.w[m] * V[g.W + c];
            }
        } else {
            const float4 w = LAT ? cw[j] : colW3[ic];   // weights of source columns i-1, i, i+1; .w: wrapped
            const unsigned nb = __float_as_uint(w.w);          // (i-1) | (i+1) << 16
            const int cl = nb & 0xffffu, cr = nb >> 16;
            const c2 y2 = w.x * V2[cl] + w.y * V2[ic] + w.z * V2[cr];   // (ya, yb)
            ya = y2.x;
            yb = y2.y;
        }
        const bool in = valid && i >= 0 && i < g.W;
        v[j] = in ? mk(ya, yb) : mk(0.0f, 0.0f);
    }
    if constexpr (!LAT || GEN) preload_twiddles_wl<LOG2N>(wb, t, tw);
    __syncthreads();
    fft_dif<LOG2N, -1>(v, t, lds, wb);
    __syncthreads();   // every wave done with its LDS region
#pragma unroll
    for (int j = 0; j < 8; ++j) lds[zslot<LOG2N>(fft_bin<LOG2N>(t, j))] = v[j];
    __syncthreads();
    // half spectra of rows (ra, ra+1) at bins f = t + jT (j < 4) and N/2 (j = 4)
    auto split = [&](int f) {
        c2 zf = lds[zslot<LOG2N>(f)], zm = lds[zslot<LOG2N>((N - f) & (N - 1))];
        // Y_a = (Z[f] + conj Z[N-f]) / 2 ;  Y_b = (Z[f] - conj Z[N-f]) / 2i
        float4 o;
        o.x = 0.5f * (zf.x + zm.x);
        o.y = 0.5f * (zf.y - zm.y);
        o.z = 0.5f * (zf.y + zm.y);
        o.w = -0.5f * (zf.x - zm.x);
        return o;
    };
    float4 o[5];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = split(t + j * T);
    o[4] = split(N / 2);
    // G[f][row] is row-contiguous per bin.  With whole row-pair groups per
    // frame in the workgroup (uniform test), the GPW pairs' values of a bin are
    // transposed through LDS and leave as one 16*GPW-byte piece (consecutive
    // rows); else every group stores its own 16-B pieces.
    if (GPW == 1 || pairs_per_frame % GPW != 0) {
        if (!valid) return;
        c2 *Gf = G + (size_t)frame * g_stride;
#pragma unroll
        for (int j = 0; j < 4; ++j) st_off<float4>(Gf, (unsigned)((t + j * T) * g.Hg + ra) * 8u, o[j]);
        if (t == 0) st_off<float4>(Gf, (unsigned)((N / 2) * g.Hg + ra) * 8u, o[4]);
        return;
    }
    __syncthreads();   // split reads done before the staging overwrites the buffers
    // [GPW][SS] (group-major, SS = N/2+1 rounded up to 8 mod 16 float4: the two
    // groups' entries of a bin 32 banks apart) when GPW == 2; [N/2 + 1][GPW]
    // otherwise (small N: many groups, no room for padding)
    float4 *stg = reinterpret_cast<float4 *>(lds_all);
    constexpr int SS = (N / 2 + 1 + 7) / 16 * 16 + 8;
    constexpr bool GM = GPW == 2 && 2 * SS * 2 <= 2 * lds_complex<N>();
    auto sidx = [&](int f, int c) { return GM ? c * SS + f : f * GPW + c; };
#pragma unroll
    for (int j = 0; j < 4; ++j) stg[sidx(t + j * T, grp)] = o[j];
    if (t == 0) stg[sidx(N / 2, grp)] = o[4];
    __syncthreads();
    if (lblk >= total_pairs) return;   // whole block past the end (total % GPW == 0)
    const int fr0 = lblk / pairs_per_frame, ra0 = 2 * (lblk % pairs_per_frame);
    c2 *Gf = G + (size_t)fr0 * g_stride;
    for (int e = threadIdx.x; e < (N / 2 + 1) * GPW; e += GPW * T) {
        const int f = e / GPW, c = e - f * GPW;
        st_off<float4>(Gf, (unsigned)(f * g.Hg + ra0 + 2 * c) * 8u, stg[sidx(f, c)]);
    }
}

// =========================================================================
// K2: column FFT -> pyramid phase magnification -> column IFFT
// =========================================================================
__device__ __forceinline__ float smooth01(float x)   // HLSL smoothstep(0,1,x)
{
    float t = sat(x);
    return t * t * (3.0f - 2.0f * t);
}

// atan2 for the phase difference: octant reduction + degree-15 odd minimax
// polynomial on [0,1] (|err| <= 1.5e-7 rad; the phase scale S multiplies it).
__device__ __forceinline__ float fast_atan2(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    // max3 with the smallest normal float: atan2(0, 0) = 0 without a select
    // (0 * rcp(2^-126) = 0); no nonzero argument of the ops is that small
    // (mn by the octant compare, not fminf: its NaN canonicalisation costs two
    // more instructions on operands the compiler cannot prove canonical)
    const bool steep = ay > ax;
    const float mx = fmaxf(fmaxf(ax, ay), 1.17549435e-38f), mn = steep ? ax : ay;
    const float a = mn * __builtin_amdgcn_rcpf(mx);
    const float s = a * a;
    float r = -0.00405455008149147f;
    r = r * s + 0.021862903609871864f;
    r = r * s - 0.055912263691425323f;
    r = r * s + 0.09642193466424942f;
    r = r * s - 0.1390862911939621f;
    r = r * s + 0.19946566224098206f;
    r = r * s - 0.33329859375953674f;
    r = r * s + 0.9999993443489075f;
    r *= a;
    if (steep) r = 1.57079632679489662f - r;
    if (x < 0.0f) r = 3.14159265358979324f - r;
    return copysignf(r, y);
}

// fast_atan2 of two arguments at once: the polynomial, its reconstruction
// constant and the scale run as packed FP32 (v_pk_fma_f32: a fused
// multiply-add per half, so both results are fast_atan2's bit for bit); the
// octant selects stay scalar (VOP3P has no abs modifier)
__device__ __forceinline__ c2 fast_atan2_x2(float y0, float x0, float y1, float x1)
{
    const float ax0 = fabsf(x0), ay0 = fabsf(y0), ax1 = fabsf(x1), ay1 = fabsf(y1);
    const bool st0 = ay0 > ax0, st1 = ay1 > ax1;
    const float a0 = (st0 ? ax0 : ay0) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(ax0, ay0), 1.17549435e-38f));
    const float a1 = (st1 ? ax1 : ay1) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(ax1, ay1), 1.17549435e-38f));
    const c2 a = mk(a0, a1), sq = a * a;
    c2 r = mk(-0.00405455008149147f, -0.00405455008149147f);
    r = r * sq + mk(0.021862903609871864f, 0.021862903609871864f);
    r = r * sq - mk(0.055912263691425323f, 0.055912263691425323f);
    r = r * sq + mk(0.09642193466424942f, 0.09642193466424942f);
    r = r * sq - mk(0.1390862911939621f, 0.1390862911939621f);
    r = r * sq + mk(0.19946566224098206f, 0.19946566224098206f);
    r = r * sq - mk(0.33329859375953674f, 0.33329859375953674f);
    r = r * sq + mk(0.9999993443489075f, 0.9999993443489075f);
    const c2 ra = r * a;
    const c2 rs = mk(1.57079632679489662f, 1.57079632679489662f) - ra;
    float t0 = st0 ? rs.x : ra.x, t1 = st1 ? rs.y : ra.y;
    if (x0 < 0.0f) t0 = 3.14159265358979324f - t0;
    if (x1 < 0.0f) t1 = 3.14159265358979324f - t1;
    return mk(copysignf(t0, y0), copysignf(t1, y1));
}

// Radial masks of GeneratePyramidFilters (PyramidOperations.compute:25-87) and the
// per-level gate/phase rule of ProcessPyramidPhaseDifference
// (PyramidPhaseDifference.compute:58-101), summed over levels
// (AccumulatePyramidLevel, PyramidOperations.compute:111-128), for one bin:
//   A = c * [ sum_{pass} m_i + sum_{mag} m_i * e^{i S wrap(arg p - arg c)} ] / N^2
// Levels 0 and L-1 always pass; a middle level passes where |m c| or |m p| < tau.
template <int LOG2N>
__device__ __forceinline__ c2 pyramid_op(c2 c, c2 p, int fx, int fy, const Spec &sp)
{
    constexpr int N = 1 << LOG2N;
    const float ux = (float)fx * (1.0f / (float)N);
    const float uy = (float)(fy <= N / 2 ? fy : N - fy) * (1.0f / (float)N);
    const float fr = __builtin_amdgcn_sqrtf(ux * ux + uy * uy);
    const float mn2 = fminf(c.x * c.x + c.y * c.y, p.x * p.x + p.y * p.y);
    // level 0: high-pass
    float mpass = fr > sp.maxF ? 1.0f : (fr > sp.hp_lo ? smooth01((fr - sp.hp_lo) * sp.hp_inv) : 0.0f);
    // level L-1: low-pass
    if (sp.L > 1)
        mpass += fr < sp.minF ? 1.0f : (fr < sp.lp_hi ? 1.0f - smooth01((fr - sp.minF) * sp.lp_inv) : 0.0f);
    float mmag = 0.0f;
    for (int i = 1; i < sp.L - 1; ++i) {
        if (fr >= sp.lo[i] && fr <= sp.hi[i]) {
            const float m = 0.5f * (1.0f + __cosf(2.0f * kPi * ((fr - sp.lo[i]) * sp.inv_w[i] - 0.5f)));
            if (m * m * mn2 < sp.tau2) mpass += m;
            else mmag += m;
        }
    }
    c2 a = scale(c, mpass * sp.inv_nn);
    if (mmag > 0.0f) {
        // delta = wrap(arg p - arg c) = arg(p * conj c)
        const float d = fast_atan2(p.y * c.x - p.x * c.y, p.x * c.x + p.y * c.y);
        const float ph = sp.S * d;
        const float k = mmag * sp.inv_nn;
        a = add(a, scale(mul_c(c, mk(__cosf(ph), __sinf(ph))), k));
    }
    return a;
}

// ProcessPhaseDifference (PhaseDifferenceComputeShader.compute:124-179) for one
// bin of the unmasked spectrum (standard mode, .cs:208-232):
//   A = c * e^{i S w(sf) wrap(arg p - arg c)} / N^2, or c / N^2 if |c| or |p| < tau,
// w = calculate_bandpass_weight(calculate_spatial_frequency) (:74-122).
template <int LOG2N>
__device__ __forceinline__ c2 standard_op(c2 c, c2 p, int fx, int fy, const Spec &sp)
{
    constexpr int N = 1 << LOG2N;
    const float ux = (float)fx * (1.0f / (float)N);
    const float uy = (float)(fy <= N / 2 ? fy : N - fy) * (1.0f / (float)N);
    const float sf = fminf(__builtin_amdgcn_sqrtf(ux * ux + uy * uy) / 0.707f, 1.0f);
    const float mn2 = fminf(c.x * c.x + c.y * c.y, p.x * p.x + p.y * p.y);
    if (mn2 < sp.tau2) return scale(c, sp.inv_nn);
    float w = 1.0f;
    if (sp.bp_apply) {
        if (sf < sp.bp_low) w *= __powf(sf * sp.bp_inv_low, sp.bp_steep);
        if (sf > sp.bp_high) w *= __powf((1.0f - sf) * sp.bp_inv_1mhigh, sp.bp_steep);
        w *= sp.bp_sens;
        if (sf > sp.bp_low && sf < sp.bp_high)
            w *= 1.0f + sp.bp_edge * __sinf(kPi * (sf - sp.bp_low) * sp.bp_inv_band);
        w = fmaxf(w, 0.0f);
    }
    const float d = fast_atan2(p.y * c.x - p.x * c.y, p.x * c.x + p.y * c.y);
    const float ph = (d * w) * sp.S;
    return scale(mul_c(c, mk(__cosf(ph), __sinf(ph))), sp.inv_nn);
}

template <int LOG2N, int MODE>
__device__ __forceinline__ c2 spectral_op(c2 c, c2 p, int fx, int fy, const Spec &sp)
{
    if constexpr (MODE == 0) return pyramid_op<LOG2N>(c, p, fx, fy, sp);
    else return standard_op<LOG2N>(c, p, fx, fy, sp);
}

// ---- frame-invariant part of the spectral op: per-bin LDS table ---------
// A thread owns the same bins of one column for every frame of a launch, so
// what depends only on (fx, fy) is evaluated once per launch into LDS (N/2+1
// entries: every mask is symmetric in fy) instead of once per bin and frame.
//   MM_K2_PYR_TAB (pyramid): x = m_a, the first middle-band mask nonzero at
//     the bin; y = -(m_a + hp + lp), minus the bin's mask sum (hp, lp: the
//     always-passed levels 0 and L-1), when at most one band is nonzero (sign
//     bit set, -0.0 included), else y = m_b, the second band, and hp + lp is
//     evaluated inline (a divergent branch that only waves holding such bins
//     take; none for L <= 5 at default bands).
//     The host checks that no 3 bands overlap.
//   MM_MODE_STANDARD: (w, 0), w = calculate_bandpass_weight (:74-122).
constexpr int MM_K2_PYR_TAB = 2;
// MM_K2_PYR_TAB2: MM_K2_PYR_TAB for band layouts whose neighbouring middle
// bands overlap (L = 6 at the default 0.05 / 0.45: the C3 configuration).
// Waves holding a two-band bin run pyramid_op_2band_x2 (branch-free, the
// bins' whole mask sums from a second LDS array) instead of the generic
// one-bin-at-a-time op; the table is MM_K2_PYR_TAB's.  A separate kernel
// instance, so that the one-band layouts' kernel keeps its registers.
constexpr int MM_K2_PYR_TAB2 = 4;
template <int MODE> constexpr bool k2_tabled()
{
    return MODE == MM_K2_PYR_TAB || MODE == MM_K2_PYR_TAB2;
}
template <int MODE> constexpr bool k2_msum() { return MODE == MM_K2_PYR_TAB2; }
template <int MODE> constexpr bool k2_one_band_op() { return MODE == MM_K2_PYR_TAB || MODE == MM_K2_PYR_TAB2; }

template <int LOG2N, int MODE>
__device__ __forceinline__ float2 bin_static(int fx, int fyy, const Spec &sp)
{
    constexpr int N = 1 << LOG2N;
    const float ux = (float)fx * (1.0f / (float)N);
    const float uy = (float)fyy * (1.0f / (float)N);
    const float fr = __builtin_amdgcn_sqrtf(ux * ux + uy * uy);
    if constexpr (MODE == MM_MODE_STANDARD) {
        const float sf = fminf(fr / 0.707f, 1.0f);
        float w = 1.0f;
        if (sp.bp_apply) {
            if (sf < sp.bp_low) w *= __powf(sf * sp.bp_inv_low, sp.bp_steep);
            if (sf > sp.bp_high) w *= __powf((1.0f - sf) * sp.bp_inv_1mhigh, sp.bp_steep);
            w *= sp.bp_sens;
            if (sf > sp.bp_low && sf < sp.bp_high)
                w *= 1.0f + sp.bp_edge * __sinf(kPi * (sf - sp.bp_low) * sp.bp_inv_band);
            w = fmaxf(w, 0.0f);
        }
        return make_float2(w, 0.0f);
    } else {
        float mfix = fr > sp.maxF ? 1.0f : (fr > sp.hp_lo ? smooth01((fr - sp.hp_lo) * sp.hp_inv) : 0.0f);
        if (sp.L > 1)
            mfix += fr < sp.minF ? 1.0f : (fr < sp.lp_hi ? 1.0f - smooth01((fr - sp.minF) * sp.lp_inv) : 0.0f);
        float ma = 0.0f, mb = 0.0f;
        for (int i = 1; i < sp.L - 1; ++i) {
            if (fr >= sp.lo[i] && fr <= sp.hi[i]) {
                const float m = 0.5f * (1.0f + __cosf(2.0f * kPi * ((fr - sp.lo[i]) * sp.inv_w[i] - 0.5f)));
                if (m != 0.0f) {
                    if (ma == 0.0f) ma = m;
                    else mb = m;
                }
            }
        }
        // one band: y = -(m_a + hp + lp), the bin's whole mask sum (sign bit set,
        // -0.0 included); two bands: y = m_b > 0
        return make_float2(ma, mb != 0.0f ? mb : -(ma + mfix));
    }
}

// The bin's whole mask sum (every level, the K2 tables' second array): the
// pass weight of the two-band op.  For a one-band bin it is -y of
// bin_static's entry bit for bit (the same sum, ma + hp + lp).
template <int LOG2N>
__device__ __forceinline__ float bin_mask_sum(int fx, int fyy, const Spec &sp)
{
    constexpr int N = 1 << LOG2N;
    const float ux = (float)fx * (1.0f / (float)N);
    const float uy = (float)fyy * (1.0f / (float)N);
    const float fr = __builtin_amdgcn_sqrtf(ux * ux + uy * uy);
    float mfix = fr > sp.maxF ? 1.0f : (fr > sp.hp_lo ? smooth01((fr - sp.hp_lo) * sp.hp_inv) : 0.0f);
    if (sp.L > 1)
        mfix += fr < sp.minF ? 1.0f : (fr < sp.lp_hi ? 1.0f - smooth01((fr - sp.minF) * sp.lp_inv) : 0.0f);
    float ma = 0.0f, mb = 0.0f;
    for (int i = 1; i < sp.L - 1; ++i) {
        if (fr >= sp.lo[i] && fr <= sp.hi[i]) {
            const float m = 0.5f * (1.0f + __cosf(2.0f * kPi * ((fr - sp.lo[i]) * sp.inv_w[i] - 0.5f)));
            if (m != 0.0f) {
                if (ma == 0.0f) ma = m;
                else mb = m;
            }
        }
    }
    return mb != 0.0f ? (ma + mb) + mfix : ma + mfix;
}

// atan2 for a nonzero argument (the magnified bins: |u| = |p||c| > 0 there)
__device__ __forceinline__ float atan2_nz(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    const float a = fminf(ax, ay) * __builtin_amdgcn_rcpf(fmaxf(ax, ay));
    const float s = a * a;
    float r = -0.00405455008149147f;
    r = r * s + 0.021862903609871864f;
    r = r * s - 0.055912263691425323f;
    r = r * s + 0.09642193466424942f;
    r = r * s - 0.1390862911939621f;
    r = r * s + 0.19946566224098206f;
    r = r * s - 0.33329859375953674f;
    r = r * s + 0.9999993443489075f;
    r *= a;
    if (ay > ax) r = 1.57079632679489662f - r;
    if (x < 0.0f) r = 3.14159265358979324f - r;
    return copysignf(r, y);
}

// pyramid_op with the middle bands from the table.  Table entries are the
// masks times inv_nn = 1/N^2 (a power of two, so every product and sum below
// is the unscaled one times inv_nn exactly, and the gate m^2 mn2 < tau^2 reads
// (m inv_nn)^2 mn2 < tau^2 inv_nn^2 with the same outcome):
//   A = c * [mpass + mmag e^{i S delta}],  delta = arg(p conj c)
template <int LOG2N>
__device__ __forceinline__ c2 pyramid_op_t(c2 c, c2 p, int fx, int fy, const Spec &sp, float2 mt)
{
    constexpr int N = 1 << LOG2N;
    const float mn2 = fminf(c.x * c.x + c.y * c.y, p.x * p.x + p.y * p.y);
    float mpass, mb;
    if (__builtin_signbit(mt.y)) {   // static hp + lp from the table
        mpass = -mt.y - mt.x;
        mb = 0.0f;
    } else {                         // two bands at this bin: hp + lp inline
        const float ux = (float)fx * (1.0f / (float)N);
        const float uy = (float)(fy <= N / 2 ? fy : N - fy) * (1.0f / (float)N);
        const float fr = __builtin_amdgcn_sqrtf(ux * ux + uy * uy);
        mpass = fr > sp.maxF ? 1.0f : (fr > sp.hp_lo ? smooth01((fr - sp.hp_lo) * sp.hp_inv) : 0.0f);
        if (sp.L > 1)
            mpass += fr < sp.minF ? 1.0f : (fr < sp.lp_hi ? 1.0f - smooth01((fr - sp.minF) * sp.lp_inv) : 0.0f);
        mpass *= sp.inv_nn;
        mb = mt.y;
    }
    float mmag = 0.0f;
    if (mt.x * mt.x * mn2 < sp.tau2_nn) mpass += mt.x;
    else mmag += mt.x;
    if (mb * mb * mn2 < sp.tau2_nn) mpass += mb;
    else mmag += mb;
    c2 w = mk(mpass, 0.0f);
    if (mmag > 0.0f) {
        // S * delta in revolutions straight into v_sin / v_cos
        const float rev = atan2_nz(p.y * c.x - p.x * c.y, p.x * c.x + p.y * c.y) * sp.S_rev;
        w = mk(mmag * __builtin_amdgcn_cosf(rev) + mpass, mmag * __builtin_amdgcn_sinf(rev));
    }
    return mul_c(c, w);
}

// pyramid_op_t for a bin with at most one middle band (table entry y < 0,
// the usual case: bands touch only where their masks are 0), without
// branches or selects on the phase factor, so that the compiler interleaves
// several bins' dependency chains (atan2 polynomial, v_sin/v_cos) instead of
// branching around each one under an exec mask:
//   w = mpass + mmag e^{i S delta},  mmag = gated ? 0 : m_a,  mpass = sum - mmag
// (mmag = 0 gives w = (mpass, 0) exactly: cos/sin are finite for every
// argument, fast_atan2(0, 0) = 0).  u = p conj c and c w use the packed
// multiplies (their operands are plain VALU results, never a transcendental's).
__device__ __forceinline__ c2 pyramid_op_1band(c2 c, c2 p, const Spec &sp, float2 mt)
{
    const float mn2 = fminf(c.x * c.x + c.y * c.y, p.x * p.x + p.y * p.y);
    const float mmag = mt.x * mt.x * mn2 < sp.tau2_nn ? 0.0f : mt.x;
    const float mpass = -mt.y - mmag;
    const c2 u = mul_conj(p, c);
    const float rev = fast_atan2(u.y, u.x) * sp.S_rev;
    const float cw = __builtin_amdgcn_cosf(rev), sw = __builtin_amdgcn_sinf(rev);
    return mul(c, mk(mmag * cw + mpass, mmag * sw));
}

// pyramid_op_1band for two bins at once: the same operations, with the
// atan2 polynomial, its reconstruction and the scale to revolutions of both
// bins in packed FP32 (one v_pk_fma per step for two bins; v_pk_fma_f32 is a
// fused multiply-add per half, so every value is the scalar form's bit for
// bit).  Only the per-bin octant selects stay scalar (no abs modifier on
// VOP3P sources).
__device__ __forceinline__ void pyramid_op_1band_x2(c2 &v0, c2 &p0, float2 mt0, c2 &v1, c2 &p1, float2 mt1,
                                                    const Spec &sp)
{
    const c2 c0 = v0, c1 = v1;
    const float mn0 = fminf(c0.x * c0.x + c0.y * c0.y, p0.x * p0.x + p0.y * p0.y);
    const float mn1 = fminf(c1.x * c1.x + c1.y * c1.y, p1.x * p1.x + p1.y * p1.y);
    const float mmag0 = mt0.x * mt0.x * mn0 < sp.tau2_nn ? 0.0f : mt0.x;
    const float mmag1 = mt1.x * mt1.x * mn1 < sp.tau2_nn ? 0.0f : mt1.x;
    const float mpass0 = -mt0.y - mmag0, mpass1 = -mt1.y - mmag1;
    const c2 u0 = mul_conj(p0, c0), u1 = mul_conj(p1, c1);
    // octant reduction per bin (fast_atan2's expressions)
    const float ax0 = fabsf(u0.x), ay0 = fabsf(u0.y), ax1 = fabsf(u1.x), ay1 = fabsf(u1.y);
    const bool st0 = ay0 > ax0, st1 = ay1 > ax1;
    const float a0 = (st0 ? ax0 : ay0) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(ax0, ay0), 1.17549435e-38f));
    const float a1 = (st1 ? ax1 : ay1) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(ax1, ay1), 1.17549435e-38f));
    const c2 a = mk(a0, a1), sq = a * a;
    c2 r = mk(-0.00405455008149147f, -0.00405455008149147f);
    r = r * sq + mk(0.021862903609871864f, 0.021862903609871864f);
    r = r * sq - mk(0.055912263691425323f, 0.055912263691425323f);
    r = r * sq + mk(0.09642193466424942f, 0.09642193466424942f);
    r = r * sq - mk(0.1390862911939621f, 0.1390862911939621f);
    r = r * sq + mk(0.19946566224098206f, 0.19946566224098206f);
    r = r * sq - mk(0.33329859375953674f, 0.33329859375953674f);
    r = r * sq + mk(0.9999993443489075f, 0.9999993443489075f);
    const c2 ra = r * a;
    const c2 rs = mk(1.57079632679489662f, 1.57079632679489662f) - ra;
    float t0 = st0 ? rs.x : ra.x, t1 = st1 ? rs.y : ra.y;
    if (u0.x < 0.0f) t0 = 3.14159265358979324f - t0;
    if (u1.x < 0.0f) t1 = 3.14159265358979324f - t1;
    const c2 rev = mk(copysignf(t0, u0.y), copysignf(t1, u1.y)) * mk(sp.S_rev, sp.S_rev);
    const float cw0 = __builtin_amdgcn_cosf(rev.x), sw0 = __builtin_amdgcn_sinf(rev.x);
    const float cw1 = __builtin_amdgcn_cosf(rev.y), sw1 = __builtin_amdgcn_sinf(rev.y);
    v0 = mul(c0, mk(mmag0 * cw0 + mpass0, mmag0 * sw0));
    v1 = mul(c1, mk(mmag1 * cw1 + mpass1, mmag1 * sw1));
    p0 = c0;
    p1 = c1;
}

// pyramid_op_1band_x2 for waves that hold a bin with TWO middle bands (the
// L = 6 layouts: neighbouring raised-cosine bands overlap), branch-free like
// the one-band op instead of the generic per-bin path: each band is gated on
// its own (PyramidPhaseDifference.compute:82-86 per level),
//   w = msum - mmag + mmag e^{i S delta},  mmag = [m_a not gated] m_a + [m_b not gated] m_b,
// msum = the bin's whole mask sum (table's second array).  A one-band bin
// (mt.y < 0) has m_b = 0, whose gate always holds: the one-band op's values
// bit for bit (msum == -mt.y).
__device__ __forceinline__ void pyramid_op_2band_x2(c2 &v0, c2 &p0, float2 mt0, float ms0, c2 &v1, c2 &p1,
                                                    float2 mt1, float ms1, const Spec &sp)
{
    const c2 c0 = v0, c1 = v1;
    const float mn0 = fminf(c0.x * c0.x + c0.y * c0.y, p0.x * p0.x + p0.y * p0.y);
    const float mn1 = fminf(c1.x * c1.x + c1.y * c1.y, p1.x * p1.x + p1.y * p1.y);
    const float mb0 = fmaxf(mt0.y, 0.0f), mb1 = fmaxf(mt1.y, 0.0f);
    const float mmag0 = (mt0.x * mt0.x * mn0 < sp.tau2_nn ? 0.0f : mt0.x) + (mb0 * mb0 * mn0 < sp.tau2_nn ? 0.0f : mb0);
    const float mmag1 = (mt1.x * mt1.x * mn1 < sp.tau2_nn ? 0.0f : mt1.x) + (mb1 * mb1 * mn1 < sp.tau2_nn ? 0.0f : mb1);
    const float mpass0 = ms0 - mmag0, mpass1 = ms1 - mmag1;
    const c2 u0 = mul_conj(p0, c0), u1 = mul_conj(p1, c1);
    const float ax0 = fabsf(u0.x), ay0 = fabsf(u0.y), ax1 = fabsf(u1.x), ay1 = fabsf(u1.y);
    const bool st0 = ay0 > ax0, st1 = ay1 > ax1;
    const float a0 = (st0 ? ax0 : ay0) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(ax0, ay0), 1.17549435e-38f));
    const float a1 = (st1 ? ax1 : ay1) * __builtin_amdgcn_rcpf(fmaxf(fmaxf(ax1, ay1), 1.17549435e-38f));
    const c2 a = mk(a0, a1), sq = a * a;
    c2 r = mk(-0.00405455008149147f, -0.00405455008149147f);
    r = r * sq + mk(0.021862903609871864f, 0.021862903609871864f);
    r = r * sq - mk(0.055912263691425323f, 0.055912263691425323f);
    r = r * sq + mk(0.09642193466424942f, 0.09642193466424942f);
    r = r * sq - mk(0.1390862911939621f, 0.1390862911939621f);
    r = r * sq + mk(0.19946566224098206f, 0.19946566224098206f);
    r = r * sq - mk(0.33329859375953674f, 0.33329859375953674f);
    r = r * sq + mk(0.9999993443489075f, 0.9999993443489075f);
    const c2 ra = r * a;
    const c2 rs = mk(1.57079632679489662f, 1.57079632679489662f) - ra;
    float t0 = st0 ? rs.x : ra.x, t1 = st1 ? rs.y : ra.y;
    if (u0.x < 0.0f) t0 = 3.14159265358979324f - t0;
    if (u1.x < 0.0f) t1 = 3.14159265358979324f - t1;
    const c2 rev = mk(copysignf(t0, u0.y), copysignf(t1, u1.y)) * mk(sp.S_rev, sp.S_rev);
    const float cw0 = __builtin_amdgcn_cosf(rev.x), sw0 = __builtin_amdgcn_sinf(rev.x);
    const float cw1 = __builtin_amdgcn_cosf(rev.y), sw1 = __builtin_amdgcn_sinf(rev.y);
    v0 = mul(c0, mk(mmag0 * cw0 + mpass0, mmag0 * sw0));
    v1 = mul(c1, mk(mmag1 * cw1 + mpass1, mmag1 * sw1));
    p0 = c0;
    p1 = c1;
}

// the same for one bin (the packed group's one-at-a-time ops)
__device__ __forceinline__ c2 pyramid_op_2band(c2 c, c2 p, const Spec &sp, float2 mt, float ms)
{
    const float mn2 = fminf(c.x * c.x + c.y * c.y, p.x * p.x + p.y * p.y);
    const float mb = fmaxf(mt.y, 0.0f);
    const float mmag = (mt.x * mt.x * mn2 < sp.tau2_nn ? 0.0f : mt.x) + (mb * mb * mn2 < sp.tau2_nn ? 0.0f : mb);
    const float mpass = ms - mmag;
    const c2 u = mul_conj(p, c);
    const float rev = fast_atan2(u.y, u.x) * sp.S_rev;
    const float cw = __builtin_amdgcn_cosf(rev), sw = __builtin_amdgcn_sinf(rev);
    return mul(c, mk(mmag * cw + mpass, mmag * sw));
}

// The power form of the phase factor (k_cols SP > 0: an integer phase scale
// S with |S| == SP fixed at compile time).  For an integer S
//   e^{i S wrap(arg p - arg c)} = e^{i S (arg p - arg c)} = z^S,
//   z = p conj(c) / (|p| |c|)
// (wrap subtracts a multiple of 2 pi, which an integer S maps to a multiple of
// 2 pi: PyramidPhaseDifference.compute:47-54, 92-98), so the atan2 polynomial,
// its octant logic and sin / cos become one rsq and a fixed chain of complex
// squarings and products, two bins per packed op: |S| = 25 is 4 squarings + 2
// products, 10 is 3 + 1.  S < 0: conj(z)^|S| (the sign on z's imaginary part).
// Same value up to fp32 rounding (tests/test_k2_pow.py against the atan2 form
// and the oracle).  Opt-in (MM_K2_POW=1): it trades the atan2 polynomial and
// 3 transcendentals per bin for 1 rsq and 12 packed ops per bin (|S| = 25),
// +15 VALU per 8 bins at 16 fewer transcendental issue slots, and measured
// slower same-call (1080p k_cols 8.38 -> 8.58-8.61 us, C3 38.6-39.0 ->
// 39.1-39.4: the squaring chain is one long dependency per bin pair).  Range: |p| |c| < 2^64 (the product of the squared norms is
// scaled by 2^-64 before the rsq; any RGBA8 frame is below 2^25 per bin), and
// a bin with |p|^2 |c|^2 < 2^-62 gets z = u 2^31 instead of u / |u| (such a bin
// is gated unless tau < 2^-31 / (m N M)).

// (x + i y)^E for two bins at once (one per lane of x and y)
template <int E>
__device__ __forceinline__ void cpow_x2(c2 &x, c2 &y)
{
    static_assert(E >= 1, "exponent");
    if constexpr (E % 2 == 0) {
        cpow_x2<E / 2>(x, y);
        const c2 xx = x * x - y * y, yy = (x + x) * y;
        x = xx;
        y = yy;
    } else if constexpr (E > 1) {
        c2 rx = x, ry = y;
        cpow_x2<E - 1>(rx, ry);
        const c2 xx = rx * x - ry * y, yy = rx * y + ry * x;
        x = xx;
        y = yy;
    }
}

// pyramid_op_1band_x2 (TWO: pyramid_op_2band_x2, with the bins' mask sums
// ms0, ms1) in the power form, E = |S|
template <int E, bool TWO>
__device__ __forceinline__ void pyramid_op_pow_x2(c2 &v0, c2 &p0, float2 mt0, float ms0, c2 &v1, c2 &p1,
                                                  float2 mt1, float ms1, const Spec &sp)
{
    const c2 c0 = v0, c1 = v1;
    const float cn0 = c0.x * c0.x + c0.y * c0.y, pn0 = p0.x * p0.x + p0.y * p0.y;
    const float cn1 = c1.x * c1.x + c1.y * c1.y, pn1 = p1.x * p1.x + p1.y * p1.y;
    const float mn0 = fminf(cn0, pn0), mn1 = fminf(cn1, pn1);
    float mmag0, mmag1, mpass0, mpass1;
    if constexpr (TWO) {
        const float mb0 = fmaxf(mt0.y, 0.0f), mb1 = fmaxf(mt1.y, 0.0f);
        mmag0 = (mt0.x * mt0.x * mn0 < sp.tau2_nn ? 0.0f : mt0.x) + (mb0 * mb0 * mn0 < sp.tau2_nn ? 0.0f : mb0);
        mmag1 = (mt1.x * mt1.x * mn1 < sp.tau2_nn ? 0.0f : mt1.x) + (mb1 * mb1 * mn1 < sp.tau2_nn ? 0.0f : mb1);
        mpass0 = ms0 - mmag0;
        mpass1 = ms1 - mmag1;
    } else {
        mmag0 = mt0.x * mt0.x * mn0 < sp.tau2_nn ? 0.0f : mt0.x;
        mmag1 = mt1.x * mt1.x * mn1 < sp.tau2_nn ? 0.0f : mt1.x;
        mpass0 = -mt0.y - mmag0;
        mpass1 = -mt1.y - mmag1;
    }
    const c2 u0 = mul_conj(p0, c0), u1 = mul_conj(p1, c1);
    // 1 / (|u| 2^-32) = rsq(|c|^2 |p|^2 2^-64), then the 2^-32 back
    const c2 q = (mk(cn0, cn1) * mk(0x1p-64f, 0x1p-64f)) * mk(pn0, pn1);
    const c2 r = mk(__builtin_amdgcn_rsqf(fmaxf(q.x, 0x1p-126f)), __builtin_amdgcn_rsqf(fmaxf(q.y, 0x1p-126f))) *
                 mk(0x1p-32f, 0x1p-32f);
    c2 x = mk(u0.x, u1.x) * r, y = mk(u0.y, u1.y) * (r * mk(sp.S_sgn, sp.S_sgn));
    cpow_x2<E>(x, y);
    v0 = mul(c0, mk(mmag0 * x.x + mpass0, mmag0 * y.x));
    v1 = mul(c1, mk(mmag1 * x.y + mpass1, mmag1 * y.y));
    p0 = c0;
    p1 = c1;
}

// one bin (the packed group's one-at-a-time ops): the two-bin form with the
// second lane a copy
template <int E, bool TWO>
__device__ __forceinline__ c2 pyramid_op_pow1(c2 c, c2 p, const Spec &sp, float2 mt, float ms)
{
    c2 v0 = c, p0 = p, v1 = c, p1 = p;
    pyramid_op_pow_x2<E, TWO>(v0, p0, mt, ms, v1, p1, mt, ms, sp);
    return v0;
}
template <int MODE>
__device__ __forceinline__ c2 standard_op_t(c2 c, c2 p, const Spec &sp, float2 mt)
{
    const float mn2 = fminf(c.x * c.x + c.y * c.y, p.x * p.x + p.y * p.y);
    if (mn2 < sp.tau2) return scale(c, sp.inv_nn);
    const float d = fast_atan2(p.y * c.x - p.x * c.y, p.x * c.x + p.y * c.y);
    const float ph = (d * mt.x) * sp.S;
    return scale(mul_c(c, mk(__cosf(ph), __sinf(ph))), sp.inv_nn);
}

template <int LOG2N> constexpr int k2_tab_entries() { return (1 << LOG2N) / 2 + 1; }
// Per-bin table slot of entry e (0 <= e <= N/2): entries e = w (mod C) are
// contiguous (slot (e mod C) Q + e / C, Q = ceil(entries / C)), so that a
// wave's bins fy = w + C (l + 64 j) (fft_bin: one residue w per wave) read
// consecutive slots, and the mirrored bins N - fy consecutive slots backwards:
// no bank conflicts (natural order: lanes 8 C bytes apart, 4-way at C = 4).
template <int LOG2N> constexpr int k2_tab_q() { return (k2_tab_entries<LOG2N>() + fft_c_v(LOG2N) - 1) / fft_c_v(LOG2N); }
template <int LOG2N> constexpr int k2_tab_slots() { return k2_tab_q<LOG2N>() * fft_c_v(LOG2N); }
template <int LOG2N>
__host__ __device__ constexpr int k2_tix(int e)
{
    constexpr int C = fft_c_v(LOG2N);
    return C == 1 ? e : (e % C) * k2_tab_q<LOG2N>() + e / C;
}

// MODE: MM_MODE_PYRAMID (dynamic masks), MM_MODE_STANDARD or MM_K2_PYR_TAB (tables)
template <int LOG2N, int MODE>
__device__ __forceinline__ c2 k2_op(c2 c, c2 p, int fx, int fy, const Spec &sp, const float2 *tab)
{
    constexpr int N = 1 << LOG2N;
    if constexpr (MODE == MM_MODE_PYRAMID) {
        return pyramid_op<LOG2N>(c, p, fx, fy, sp);
    } else {
        const float2 mt = tab[k2_tix<LOG2N>(fy <= N / 2 ? fy : N - fy)];
        if constexpr (MODE == MM_MODE_STANDARD) return standard_op_t<MODE>(c, p, sp, mt);
        else return pyramid_op_t<LOG2N>(c, p, fx, fy, sp, mt);
    }
}

// k_cols runs at least two columns per workgroup, so that a Q row receives one
// 16-B (or wider) piece per workgroup instead of one 8-B value per column
// two columns per k_cols workgroup (whole 32-B Q pieces per tile row).  At
// N = 4096 that is 16 waves with 123-148 KB of LDS, one workgroup per CU for
// the whole launch; one column per workgroup there (8 waves, <= 62 KB without
// the packed group's arrays, MM_K2_PKALL: two per CU) measured slower
// same-call (C3 k_cols 37.5 -> 38.6-39.0 us per frame: 16-B Q pieces), so it
// is a build option only (-DMM_K2_GROUPS_4K=1).
#ifndef MM_K2_GROUPS_4K
#define MM_K2_GROUPS_4K 2
#endif
template <int LOG2N> constexpr int k2_groups()
{
    return LOG2N >= 13 ? 1 : LOG2N >= 12 ? MM_K2_GROUPS_4K : groups_at_least<LOG2N, MM_K2_GROUPS>();
}
// the steerable band-column kernel: one column per workgroup where one
// transform fills a workgroup (N >= 2048), else the transforms a 256-thread
// workgroup holds; its staged pieces are 32 B through the band rows' row
// groups of 4 (MM_SB_RROWS, mm_steer.hpp), and the workgroups of a CU run
// independently (two columns in one 1,024-thread workgroup synchronised 16
// waves per barrier: C3 O = 8 k_sb_cols 434 -> 380 us, 1080p 81.7 -> 69.4,
// profiles/r06h_sb_rows_layout_ab.txt).  MM_SB_MIN_GROUPS = 2 / 4: two / four
// columns per workgroup (four at N = 2048: 130 us, one workgroup per CU in
// two rounds).  MM_SB_GPW1 = 1: one column with direct 8-B stores and a
// double-buffered exchange (no staging: C3 1,020 us).
#ifndef MM_SB_GPW1
#define MM_SB_GPW1 0
#endif
#ifndef MM_SB_MIN_GROUPS
#define MM_SB_MIN_GROUPS 1
#endif
template <int LOG2N> constexpr int sb_groups() { return groups_at_least<LOG2N, MM_SB_GPW1 ? 1 : MM_SB_MIN_GROUPS>(); }
// k_sb_cols with one column per workgroup: the band loop alternates two
// exchange buffers (the next band's transform never waits for this one's
// cross-wave reads) and stores from registers (no staging)
// the steerable band-row kernel: row transforms per workgroup (MM_SB_ROWS2_4K
// = 1: two at N = 4096, rows k, k+1 of one band-row group reading the same
// 32-B sectors in one 1,024-thread workgroup: C3 k_sb_rows 465 -> 568 us,
// profiles/r06h_sb_rows_layout_ab.txt; off)
#ifndef MM_SB_ROWS2_4K
#define MM_SB_ROWS2_4K 0
#endif
template <int LOG2N> constexpr int sb_rows_groups()
{
    return LOG2N == 12 && MM_SB_ROWS2_4K ? 2 : groups_per_wg<LOG2N>();
}
template <int LOG2N> constexpr int sb_rows_threads() { return sb_rows_groups<LOG2N>() * fft_T<LOG2N>(); }
template <int LOG2N> constexpr bool sb_direct() { return MM_SB_GPW1 && sb_groups<LOG2N>() == 1 && fft_c_v(LOG2N) > 1; }
template <int LOG2N> constexpr int sb_threads() { return sb_groups<LOG2N>() * fft_T<LOG2N>(); }
// K2's Q staging buffer (c2 slots written by rows, read back as float4
// pieces): slot i lives at i ^ (((i >> 4) & 1) << 1), i.e. float4 r at
// r ^ ((r >> 3) & 1).  The row writes of a 16-lane group (every other float4
// of a 16-float4 span) then cover all 32 banks once (linear: 2-way), and the
// ds_read_b128 groups still read 16 distinct 4-bank slots (tools/lds_banks.py).
#ifndef MM_K2_NOSWZ
__device__ __forceinline__ int k2_stg_swz(int i) { return i ^ (((i >> 4) & 1) << 1); }
__device__ __forceinline__ int k2_stg_swz4(int r) { return r ^ ((r >> 3) & 1); }
#else   // diagnostic: linear staging
__device__ __forceinline__ int k2_stg_swz(int i) { return i; }
__device__ __forceinline__ int k2_stg_swz4(int r) { return r; }
#endif
template <int LOG2N> constexpr int k2_threads() { return k2_groups<LOG2N>() * fft_T<LOG2N>(); }
// dynamic LDS of k_cols: per group the FFT exchange buffer and its column's
// per-bin table, plus for column N/2 (packed group only) its table, its
// previous spectrum (bins 0..N/2) and its staged Q values (one float per row).
// Above 64 KiB at N = 2048 (77.8 KiB): two workgroups still fit a CU's 160 KiB.
// The inner 512-point passes of k_cols's column FFTs take their twiddle
// powers from an LDS table (tw_tab_build) instead of 6 products per pass
// (MM_K2_TWTAB=1; default 0: same-call K2 8.08 -> 8.21 us/frame with the
// table, profiles/r03k_k2_twtab_ab.txt: the LDS reads cost more than the
// 48 VALU products per wave-frame they replace)
#ifndef MM_K2_TWTAB
#define MM_K2_TWTAB 0
#endif
template <int LOG2N> constexpr bool k2_twtab() { return MM_K2_TWTAB && fft_c_v(LOG2N) > 1; }
// Dedicated Q staging (k_cols_body stg_c2): the list rows [0, Hq) of the
// workgroup's GPW columns, [Hq/TK][GPW][TK] c2 (k2_stg_swz stays inside
// 32-slot blocks), when it fits beside two workgroups per CU (1080p: 17 KB);
// else 0 (aliased with the exchange buffers).
template <int LOG2N, int MODE> constexpr size_t k2_lds_bytes(bool with_packed = true);
template <int LOG2N, int MODE> inline int k2_stg_c2(int Hq, bool with_packed = true)
{
    const int c = (Hq * k2_groups<LOG2N>() + 31) / 32 * 32;
    return k2_lds_bytes<LOG2N, MODE>(with_packed) + sizeof(c2) * (size_t)c <= 81920 ? c : 0;
}

// bytes of n columns' mask-sum arrays ([TS] floats each, rounded up to 16 B;
// pyramid tables with overlapping bands only)
template <int LOG2N, int MODE> constexpr size_t k2_msum_bytes(int n)
{
    return k2_msum<MODE>() ? ((sizeof(float) * (size_t)n * k2_tab_slots<LOG2N>()) + 15) / 16 * 16 : 0;
}
// k_cols' dynamic LDS, in layout order: the GPW exchange buffers, the GPW
// columns' tables and mask sums, the inner twiddle table (TT); then what only
// the packed group (block 0) uses: column N/2's table and mask sums and ldsX.
// A launch without block 0 (its frames all in k_cols_tail) omits that last part.
template <int LOG2N, int MODE> constexpr size_t k2_lds_bytes(bool with_packed)
{
    return (size_t)k2_groups<LOG2N>() *
               (sizeof(c2) * lds_complex<(1 << LOG2N)>() + sizeof(float2) * k2_tab_slots<LOG2N>()) +
           k2_msum_bytes<LOG2N, MODE>(k2_groups<LOG2N>()) +
           (k2_twtab<LOG2N>() ? sizeof(float4) * tw_tab_float4() : 0) +
           (with_packed ? sizeof(float2) * k2_tab_slots<LOG2N>() + k2_msum_bytes<LOG2N, MODE>(1) + sizeof(c2) * 4
                        : 0);
}

// Columns f = 1..N/2-1 get one FFT group each.  The two real columns f = 0 and
// f = N/2 (row DFT bins that are real for real rows, so their column spectra are
// Hermitian in fy) share group 0 of block 0 as one complex column z = G0 + i*GN.
// The grid is then exactly N/2 groups (512 two-column workgroups at N=2048: one
// resident round at 2 WGs/CU, no one-group tail).  After the forward FFT the
// packed group unpacks F0, FN from Z(fy), Z(N-fy) (partner bins through LDS)
// and runs the same number of ops per thread as any other group: a thread's
// bins fy < N/2 (j < 4) carry column 0's op at fy, its bins fy > N/2 carry
// column N/2's op at N - fy; the two real bins of column N/2 (0 and N/2) are
// one extra op each for threads T/4 and 3T/4 (F_{t-1} and the result in ldsX).
// A second exchange recombines A = A0 + i AN per bin.
// (The packed block is the kernel's critical path: every block is resident at
// once, so its extra work is the kernel's.)
#ifndef MM_K2_OPG
#define MM_K2_OPG 2   // bins of the branch-free op interleaved per scheduling group (8, 4: K2 +1.6 %, +0.9 %)
#endif
#ifdef MM_K2_STAMPS
// Diagnostic build only: per-wave cycle totals of the frame-loop phases
// (s_memtime deltas), written by lane 0 with a vector store after the loop.
__device__ unsigned long long mm_k2_stamps[4096 * 8 * 8];
__device__ unsigned long long mm_k2_entry[4096 * 8];   // s_memrealtime at entry, per wave
__device__ unsigned long long mm_k2_exit[4096 * 8];    // ... after the last Q stores completed (vmcnt 0)
#define K2_STAMP(i)                                                      \
    do {                                                                 \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();      \
        st_acc[i] += n_ - st_prev;                                       \
        st_prev = n_;                                                    \
    } while (0)
#else
#define K2_STAMP(i) do { } while (0)
#endif
//
// The frame loop is instantiated twice (BLK0): block 0, whose group 0 is the
// packed group, runs the extra exchanges; every other block runs a loop with
// none of that code, so its register allocation is not shaped by the packed
// group's live values.
// The temporal state is G_{t-1}, K1's row spectra of the previous input frame
// (previousSourceTexture, .cs:142): every launch first runs `Gprev` through
// the forward transform as a passthrough frame (fr = -1), which sets F_{t-1}
// in registers bit for bit as the frame loop would have, then frames
// 0 .. nframes-1 of G, whose Q go to Q + fr * q_stride.
// A per-bin table entry from LDS as its own ds_read_b64 (lds_ld: not paired
// into a ds_read2_b64, which costs twice the LDS cycles on gfx950)
__device__ __forceinline__ float2 tab_ld(const float2 *p)
{
    const c2 v = lds_ld(reinterpret_cast<const c2 *>(p));
    return make_float2(v.x, v.y);
}

template <int LOG2N, int MODE, bool BLK0, int SP = 0>
__device__ __forceinline__ void k_cols_body(const c2 *G, size_t g_stride, const c2 *Gprev, c2 *Q,
                                            size_t q_stride, int nframes, const Geo &g,
                                            const Spec &sp, const c2 *__restrict__ tw,
                                            const float2 *__restrict__ ktab, const float *__restrict__ kmsum,
                                            int stg_c2, int blk, int nb_prio = 0)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = k2_groups<LOG2N>();
    constexpr int TS = k2_tab_slots<LOG2N>();
#ifdef MM_K2_STAMPS
    const unsigned long long st_entry = __builtin_amdgcn_s_memrealtime();
#endif
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    // group index: wave-uniform (scalar) when a group spans whole waves
    const int grp = T % 64 == 0 ? __builtin_amdgcn_readfirstlane(threadIdx.x / T) : threadIdx.x / T;
    const int t0 = threadIdx.x % T;
    // stg_c2 > 0: a dedicated Q staging area of that many c2 at the start of
    // the LDS (k2_stg_c2, when it fits beside two workgroups per CU), the FFT
    // exchange buffers and tables after it; 0: the staging aliases the
    // exchange buffers (two more workgroup barriers per frame)
    c2 *xbase = lds_all + stg_c2;
    c2 *lds = xbase + grp * lds_complex<N>();
    float2 *tabs = reinterpret_cast<float2 *>(xbase + GPW * lds_complex<N>());
    float2 *tab0 = tabs + grp * TS;
    // column N/2: F_{t-1} at its real bins 0 and N/2 and their results (two
    // threads of the packed group).  Its Q values are staged with column 0's:
    // the packed group's staging slot of a row holds (Q0, QN) (the inverse of
    // A0 + i AN; both real), split into the two columns' pieces at the store.
    // the bins' whole mask sums (tabled pyramid modes; two-band waves read them)
    float *ms0 = reinterpret_cast<float *>(tabs + GPW * TS) + grp * TS;
    uint8_t *lds_tail = reinterpret_cast<uint8_t *>(tabs + GPW * TS) + k2_msum_bytes<LOG2N, MODE>(GPW);
    float4 *ttab = reinterpret_cast<float4 *>(lds_tail);   // inner passes' twiddle powers (TT)
    if constexpr (k2_twtab<LOG2N>()) lds_tail += sizeof(float4) * tw_tab_float4();
    // packed group only (k2_lds_bytes with_packed): column N/2's table, mask sums, ldsX
    float2 *tabN = reinterpret_cast<float2 *>(lds_tail);
    float *msN = reinterpret_cast<float *>(tabN + TS);
    c2 *ldsX = reinterpret_cast<c2 *>(reinterpret_cast<uint8_t *>(msN) + k2_msum_bytes<LOG2N, MODE>(1));
    const int f_raw = blk * GPW + grp;
    const bool valid = f_raw < N / 2;
    const int f = valid ? f_raw : N / 2 - 1;
    constexpr bool blk0 = BLK0;               // block 0 runs the extra exchanges
    const bool packed = blk0 && grp == 0;     // group owning columns 0 and N/2

    // G column of a frame.  Rows outside the image get an out-of-range buffer
    // offset: the range check returns 0 for them without a memory access (the
    // zero padding of PadTexture, .cs:358-381).  A frame's loads are issued
    // before the previous frame's Q stores, so the wait for them never waits
    // for those stores (one in-order vmcnt).  (Loading one frame ahead, 16
    // more VGPRs, measured no faster: the frame loop is bound by its barrier
    // and dependency-chain latencies, not by this load's.)
    c2 ga[8];
    float gb[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    // (buffer loads: 32-bit offsets, and kept in order with the buffer stores)
    // One buffer resource per column, its range the H image rows: row t + jT - y0
    // at byte offset (t - y0) 8 + j T 8, and rows outside the image (negative
    // offsets wrap to huge ones) fail the range check without any compare.
    auto load_g = [&](int fr, int t) {
        const int gfr = __builtin_amdgcn_readfirstlane(fr);   // uniform; -1: Gprev
        const c2 *Gc = gfr < 0 ? Gprev : G + (size_t)gfr * g_stride;
        const auto grs = __builtin_amdgcn_make_buffer_rsrc(const_cast<c2 *>(Gc) + (size_t)f * g.Hg, 0,
                                                           g.H * (int)sizeof(c2), 0x00020000);
        const unsigned o0 = (unsigned)(t - g.y0) * 8u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(grs, o0 + (unsigned)(j * T * 8), 0, 0);
            ga[j] = mk(__uint_as_float(a.x), __uint_as_float(a.y));
        }
        if constexpr (blk0) {   // column N/2 (real) for the packed group's block only
            const auto nrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<c2 *>(Gc) + (size_t)(N / 2) * g.Hg, 0,
                                                               g.H * (int)sizeof(c2), 0x00020000);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                gb[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(nrs, o0 + (unsigned)(j * T * 8), 0, 0));
        }
    };
#ifndef MM_K2_NOGAHEAD
    // the prime's G_{t-1} loads first: their HBM latency overlaps the twiddle
    // loads and the table copy instead of following its barrier (one-frame
    // calls pay the prologue and the prime on every call)
    load_g(-1, t0);
#endif
    // twiddle bases of both FFTs, loaded once (issued under the table copy): no loads inside a frame but G's
    constexpr bool TT = k2_twtab<LOG2N>();
    c2 wtw[kTwSlots];
#pragma unroll
    for (int i = 0; i < kTwSlots; ++i) wtw[i] = mk(1.0f, 0.0f);
    if constexpr (TT) {   // outer-stage bases only; the inner passes read ttab
#pragma unroll
        for (int h = 0; h < 8 / fft_c_v(LOG2N); ++h) wtw[12 + h] = tw[t0 + 64 * fft_c_v(LOG2N) * h];
        tw_tab_build(ttab, threadIdx.x, GPW * T, tw, fft_c_v(LOG2N));
        if constexpr (MODE == MM_MODE_PYRAMID) __syncthreads();
    } else {
        preload_twiddles_wl<LOG2N>(wtw, t0, tw);
    }
    if constexpr (MODE != MM_MODE_PYRAMID) {
        // the column's table, evaluated once per parameter set by k_k2_table
        // (slot order): a copy instead of N/2+1 bin_static per group and launch
        const float2 *src0 = ktab + (size_t)f * TS;
        for (int e = t0; e < TS; e += T) tab0[e] = src0[e];
        if (packed) {
            const float2 *srcN = ktab + (size_t)(N / 2) * TS;
            for (int e = t0; e < TS; e += T) tabN[e] = srcN[e];
        }
        if constexpr (k2_msum<MODE>()) {
            const float *m0 = kmsum + (size_t)f * TS;
            for (int e = t0; e < TS; e += T) ms0[e] = m0[e];
            if (packed) {
                const float *mN = kmsum + (size_t)(N / 2) * TS;
                for (int e = t0; e < TS; e += T) msN[e] = mN[e];
            }
        }
        __syncthreads();
    }

    // waves whose bins all have at most one middle band (frame-invariant,
    // uniform) take the branch-free op
    // packed group: bin j's op column (0 or N/2) and bin within it
    auto pk_col0 = [&](int j, int fy) { return j < 4 || fy == N / 2; };
    bool wave_two_band = true;
    if constexpr (k2_tabled<MODE>()) {
        bool two = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int fy = fft_bin<LOG2N>(t0, j);
            if (packed && !pk_col0(j, fy)) two |= !__builtin_signbit(tabN[k2_tix<LOG2N>(N - fy)].y);
            else two |= !__builtin_signbit(tab0[k2_tix<LOG2N>(fy <= N / 2 ? fy : N - fy)].y);
        }
        if (packed && t0 == 0)
            two |= !__builtin_signbit(tabN[k2_tix<LOG2N>(0)].y) || !__builtin_signbit(tabN[k2_tix<LOG2N>(N / 2)].y);
        wave_two_band = __any(two);
    }
    // F_{t-1}: set by the passthrough frame fr = -1 (Gprev)
    c2 prev[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) prev[j] = mk(0.0f, 0.0f);

    // per-bin table bases of a regular group's bins (regular_op): bin j is
    // fy = fy0 + j N/8 (fy0 = fft_bin(t, 0)), table entry fy for j < 4, N - fy
    // for j >= 4; N/8 is a multiple of C, so both are slots of two
    // frame-invariant bases plus immediates (k2_tix): entry fy0 + m C at slot
    // k2_tix(fy0) + m, entry M - fy0 (M a multiple of C) at slot
    // k2_tix(C - w) - 1 - fy0 / C + M / C for w = fy0 mod C > 0.
    // (hoisted out of the frame loop where registers allow: N >= 2048, TK == 2;
    // smaller N recompute them per frame from the opaque lane index)
    constexpr bool HOIST = q_tile<LOG2N>() == 2;
    const int hfy0 = fft_bin<LOG2N>(t0, 0);
    const int hw = hfy0 % fft_c_v(LOG2N);
    const float2 *tlo0 = tab0 + k2_tix<LOG2N>(hfy0);
    const float2 *thi0 = tab0 + (hw ? k2_tix<LOG2N>(fft_c_v(LOG2N) - hw) - 1 : 0) - hfy0 / fft_c_v(LOG2N);

    constexpr int TK = q_tile<LOG2N>(), BLK = GPW * TK / 2;   // float4 per tile row
    constexpr int NST = (N * GPW / 2 + GPW * T - 1) / (GPW * T);   // store slots per thread (Hq <= N)
    const int fb = blk * GPW, nq = (g.Hq / TK) * BLK;
    c2 *stg = lds_all;   // staged Q pieces of a frame: [row pair][GPW][TK]
    const bool stg_ded = stg_c2 > 0;
    bool staged = false;   // stg holds the previous frame's pieces (uniform)
    // Canvas-row staging (TK == 2, rb even, no list row wrapping: every
    // geometry but H close to N): the inverse transform's rows n = t + jT go
    // to LDS unconditionally at slot(n) = ((n/2) GPW + grp) TK + n%2 (one base
    // + immediates, no per-row checks), and the Q stores read list row pair kt
    // at canvas pair kt + rb/2.  Otherwise list-row staging (rows of [0, Hq)).
    const bool cstage = !stg_ded && TK == 2 && (g.rb & 1) == 0 && g.rb >= 0 && g.rb + g.Hq <= N;
    const int rd_off = cstage ? (g.rb / 2) * GPW : 0;   // float4 pieces
    // frame-invariant per-thread Q store offsets (loop invariant: computed
    // from t0, not the opaque t below); a frame with nothing staged stores
    // through an empty buffer range instead
    unsigned so_st[NST];
#pragma unroll
    for (int i = 0; i < NST; ++i) {
        const int e = grp * T + t0 + i * GPW * T;
        const int kt = e / BLK, r = e - kt * BLK;
        const bool ok = e < nq && (GPW <= N / 2 || fb + (2 * r) / TK < N / 2);   // tiny N: fewer columns than groups
        so_st[i] = ok ? (unsigned)((kt * g.Qs + fb) * TK + 2 * r) * 8u : 0x80000000u;
    }
    // (k2_stg_swz: float4 r at r ^ ((r >> 3) & 1); + i GPW T keeps bit 3)
    const float4 *rd_base = reinterpret_cast<const float4 *>(stg) + k2_stg_swz4(grp * T + t0 + rd_off);

    // One straight path per iteration: G loads of frame fr, then the Q stores
    // of frame fr-1 from the staging buffer (exactly NST buffer stores per
    // thread; slots past the end are dropped by the range check), then frame
    // fr, whose first use of the loads waits with vmcnt(NST) and never for the
    // stores.
#ifdef MM_K2_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
    st_acc[7] = __builtin_amdgcn_s_memrealtime();   // loop start (100 MHz, device-wide)
#endif
    // One frame of the loop.  The prime (fr = -1) runs as its own instance
    // ahead of the loop, so the frame loop itself is compiled with no
    // passthrough branch: in one shared body the branch merge made the
    // compiler copy the FFT outputs twice per frame (once for the merge, once
    // into the loop-carried F_{t-1}: 32 v_mov; K2 -2 % at 1080p, -3 % at
    // 2160p same-call).  The prime keeps a RUNTIME passthrough test (fr is
    // made opaque): an instance specialised on a constant fr = -1 computed an
    // F_{t-1} 1 ulp away from the in-loop one, which broke the bitwise
    // equality of one-frame calls, tails, ring hand-offs and batches.
    // OPK: the regular groups' op, fixed per loop instance (the one-band op or
    // the rest, chosen once per wave: wave_two_band is frame-invariant), so the
    // register allocation of the one-band loop is not shaped by the generic
    // op's live values; -1: chosen per frame at run time (block 0)
    auto frame_iter = [&](const int fr, auto opk_c) __attribute__((always_inline)) -> bool {
        constexpr int OPK = decltype(opk_c)::value;
        // Opaque per-iteration copy of the lane index: stops LICM from hoisting
        // every t-derived LDS address and twiddle of both FFTs out of the frame
        // loop (that pinned ~200 VGPRs and capped occupancy at 1 wave/SIMD).
        int t = t0;
        asm volatile("" : "+v"(t));
        // Two workgroups share a CU for the whole launch and the SIMD arbiter
        // favours the older one (issue priority, then age): it ran ahead and
        // left the younger one alone for the last third (phase stamps: loop
        // times 917 vs 1357 us per 100 frames).  Alternating the priority
        // every frame between the first-dispatched half of the grid and the
        // second keeps a pair in step (1082..1305 us).
        // Block 0 (the packed group's extra exchanges: the kernel's critical
        // path, phase stamps) keeps the highest priority throughout (same-call
        // A/B: ≈ 1 % over alternating it too, and over raising the packed group only).
        if (blk0) __builtin_amdgcn_s_setprio(3);
        else if ((fr ^ ((int)blockIdx.x >= nb_prio / 2 ? 1 : 0)) & 1) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
#ifdef MM_K2_NOGAHEAD
        load_g(fr < nframes ? fr : nframes - 1, t);
#else
        // (Gprev: issued before the prologue; later frames' loads mid-iteration)
#endif
        K2_STAMP(0);
        __builtin_amdgcn_sched_barrier(0);   // keep the stores behind the loads
        {
            float4 sv[NST];
#pragma unroll
            for (int i = 0; i < NST; ++i) sv[i] = rd_base[i * GPW * T];   // (slots past the staging: unused)
            // (aliased staging) staging read before this frame's FFT rewrites the buffers
            if (!stg_ded) __syncthreads();
            const int qfr = __builtin_amdgcn_readfirstlane(fr > 0 ? fr - 1 : 0);   // uniform
            const auto qrs = __builtin_amdgcn_make_buffer_rsrc(
                Q + (size_t)qfr * q_stride, 0, staged ? (int)(q_stride * sizeof(c2)) : 0, 0x00020000);
            unsigned so[NST];
#pragma unroll
            for (int i = 0; i < NST; ++i) {
                if constexpr (HOIST) {
                    so[i] = so_st[i];
                } else {   // per frame from the opaque t (registers)
                    const int e = grp * T + t + i * GPW * T;
                    const int kt = e / BLK, r = e - kt * BLK;
                    const bool ok = e < nq && (GPW <= N / 2 || fb + (2 * r) / TK < N / 2);
                    so[i] = ok ? (unsigned)((kt * g.Qs + fb) * TK + 2 * r) * 8u : 0x80000000u;
                }
            }
#pragma unroll
            for (int i = 0; i < NST; ++i) {
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                u32x4 d = {__float_as_uint(sv[i].x), __float_as_uint(sv[i].y), __float_as_uint(sv[i].z),
                           __float_as_uint(sv[i].w)};
                if constexpr (blk0) {
                    // a piece of the packed group (column 0: group 0 of block 0)
                    // holds (Q0, QN) per row: column 0 gets the real parts, column
                    // N/2 (same rows, N/2 bins further in the tile row) the rest
                    const int e = grp * T + t + i * GPW * T;
                    if ((2 * (e % BLK)) / TK == 0) {
                        const u32x4 dn = {d.y, 0u, d.w, 0u};
                        d.y = 0u;
                        d.w = 0u;
                        __builtin_amdgcn_raw_buffer_store_b128(dn, qrs, so[i] + (unsigned)((N / 2) * TK * 8), 0, 0);
                    }
                }
                __builtin_amdgcn_raw_buffer_store_b128(d, qrs, so[i], 0, 0);
            }
        }
        K2_STAMP(1);
        if (fr == nframes) return false;
        c2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)   // G[0][r], G[N/2][r] are real (exact zero imaginary parts)
            v[j] = packed ? mk(ga[j].x, gb[j]) : ga[j];
        const bool pass_frame = fr < 0;   // the prime (fr = -1)
#ifndef MM_K2_NOGAHEAD
        // the prime's successor (frame 0) loads now, under the prime's transform
        // (the prime has no op, so its "after the op" slot below came one
        // transform later; a one-frame call waits on these loads next)
        if (pass_frame) load_g(nframes > 0 ? 0 : -1, t);
#endif
        // opaque per-iteration copy of the twiddle bases (same reason as t: the
        // products of their powers must not be hoisted into live registers)
        c2 wt[kTwSlots];
#pragma unroll
        for (int i = 0; i < kTwSlots; ++i) {
            wt[i] = wtw[i];
            if (tw_slot_used_wl(LOG2N, i) && !(TT && i < 12)) asm volatile("" : "+v"(wt[i]));
        }
        K2_STAMP(2);
        MM_MARK("M1_fwd_start");
        fft_dif<LOG2N, -1, TT>(v, t, lds, wt, ttab);
        MM_MARK("M2_fwd_end");
        K2_STAMP(3);
        // the spectral op of a regular group (all groups but the packed one)
        auto regular_op = [&]() {
            if (pass_frame) {
#pragma unroll
                for (int j = 0; j < 8; ++j) prev[j] = v[j];
            } else if (k2_one_band_op<MODE>() && (OPK == 1 || (OPK < 0 && !wave_two_band))) {
                // no bin of this wave has two middle bands: branch-free op, bins
                // interleaved MM_K2_OPG at a time
                // bin j: fy = fy0 + j N/8 (fy0 = fft_bin(t, 0)), table entry fy
                // for j < 4, N - fy for j >= 4 (fy <= N/2 exactly for j < 4).
                // N/8 is a multiple of C, so both are slots of two per-frame
                // bases plus immediates (k2_tix): entry fy0 + m C at slot
                // k2_tix(fy0) + m, entry M - fy0 (M a multiple of C) at slot
                // k2_tix(C - w) - 1 - fy0 / C + M / C for w = fy0 mod C > 0.
                constexpr int C = fft_c_v(LOG2N);
                const int fy0 = fft_bin<LOG2N>(HOIST ? t0 : t, 0);   // frame-invariant (hoisted: t0)
                const int w = fy0 % C;
                const float2 *tlo = HOIST ? tlo0 : tab0 + k2_tix<LOG2N>(fy0);
                const float2 *thi = HOIST ? thi0 : tab0 + (w ? k2_tix<LOG2N>(C - w) - 1 : 0) - fy0 / C;
#ifndef MM_K2_OPX1
#pragma unroll
#ifndef MM_K2_OPX2G
#define MM_K2_OPX2G 8   // bins per scheduling group of the two-bin op (2, 4: K2 +3 %, +1 %)
#endif
                for (int j = 0; j < 8; j += 2) {   // two bins per packed op
                    if (j % MM_K2_OPX2G == 0) __builtin_amdgcn_sched_barrier(0);
                    const float2 mt0 = tab_ld(j < 4 ? tlo + j * (N / 8) / C : thi + (N - j * (N / 8)) / C);
                    const float2 mt1 = tab_ld(j + 1 < 4 ? tlo + (j + 1) * (N / 8) / C : thi + (N - (j + 1) * (N / 8)) / C);
                    if constexpr (SP > 0)
                        pyramid_op_pow_x2<SP, false>(v[j], prev[j], mt0, 0.0f, v[j + 1], prev[j + 1], mt1, 0.0f, sp);
                    else
                        pyramid_op_1band_x2(v[j], prev[j], mt0, v[j + 1], prev[j + 1], mt1, sp);
                }
#else
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (j % MM_K2_OPG == 0) __builtin_amdgcn_sched_barrier(0);
                    const float2 mt = j < 4 ? tlo[j * (N / 8) / C] : thi[(N - j * (N / 8)) / C];
                    const c2 a = pyramid_op_1band(v[j], prev[j], sp, mt);
                    prev[j] = v[j];
                    v[j] = a;
                }
#endif
                __builtin_amdgcn_sched_barrier(0);
            } else if (MODE == MM_K2_PYR_TAB2) {
                // a bin of this wave has two middle bands (L = 6 layouts): the
                // branch-free two-band op, same table addressing + mask sums
                constexpr int C = fft_c_v(LOG2N);
                const int fy0 = fft_bin<LOG2N>(HOIST ? t0 : t, 0);
                const int w = fy0 % C;
                const float2 *tlo = HOIST ? tlo0 : tab0 + k2_tix<LOG2N>(fy0);
                const float2 *thi = HOIST ? thi0 : tab0 + (w ? k2_tix<LOG2N>(C - w) - 1 : 0) - fy0 / C;
                const float *mlo = ms0 + (tlo - tab0), *mhi = ms0 + (thi - tab0);
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    if (j % MM_K2_OPX2G == 0) __builtin_amdgcn_sched_barrier(0);
                    const int i0 = j < 4 ? j * (N / 8) / C : (N - j * (N / 8)) / C;
                    const int i1 = j + 1 < 4 ? (j + 1) * (N / 8) / C : (N - (j + 1) * (N / 8)) / C;
                    const float2 mt0 = tab_ld(j < 4 ? tlo + i0 : thi + i0), mt1 = tab_ld(j + 1 < 4 ? tlo + i1 : thi + i1);
                    const float s0 = j < 4 ? mlo[i0] : mhi[i0], s1 = j + 1 < 4 ? mlo[i1] : mhi[i1];
                    if constexpr (SP > 0)
                        pyramid_op_pow_x2<SP, true>(v[j], prev[j], mt0, s0, v[j + 1], prev[j + 1], mt1, s1, sp);
                    else
                        pyramid_op_2band_x2(v[j], prev[j], mt0, s0, v[j + 1], prev[j + 1], mt1, s1, sp);
                }
                __builtin_amdgcn_sched_barrier(0);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    // one bin at a time: keeps the 8 op instances from being interleaved
                    __builtin_amdgcn_sched_barrier(0);
                    const c2 a = k2_op<LOG2N, MODE>(v[j], prev[j], f, fft_bin<LOG2N>(t, j), sp, tab0);
                    prev[j] = v[j];
                    v[j] = a;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        if constexpr (blk0) {
            // packed group (see above the kernel).  First every wave leaves its
            // fft_dif region; then Z of every bin to LDS for the partner reads.
            __syncthreads();
            if (packed) {
#pragma unroll
                for (int j = 0; j < 8; ++j) lds[zslot<LOG2N>(fft_bin<LOG2N>(t, j))] = v[j];
            }
            __syncthreads();
            // v[j] becomes A0(fy) (j < 4) / AN(N - fy) (j >= 4)
            if (packed) {
                // unpack every bin (partner Z(N - fy) from LDS), then the ops
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int fy = fft_bin<LOG2N>(t, j);
                    const c2 z = v[j], m = lds[zslot<LOG2N>((N - fy) & (N - 1))];
                    const c2 f0 = mk(0.5f * (z.x + m.x), 0.5f * (z.y - m.y));    // F0(fy)
                    const c2 fn = mk(0.5f * (z.y + m.y), -0.5f * (z.x - m.x));   // FN(fy)
                    v[j] = pk_col0(j, fy) ? f0 : mk(fn.x, -fn.y);                // or FN(N - fy)
                }
                if (!pass_frame) {
                    if (k2_one_band_op<MODE>() && !wave_two_band) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            __builtin_amdgcn_sched_barrier(0);   // one bin at a time: registers
                            const int fy = fft_bin<LOG2N>(t, j);
                            const c2 c = v[j];
                            const float2 mt = pk_col0(j, fy) ? tab0[k2_tix<LOG2N>(fy)] : tabN[k2_tix<LOG2N>(N - fy)];
                            if constexpr (SP > 0)
                                v[j] = pyramid_op_pow1<SP, false>(c, prev[j], sp, mt, 0.0f);
                            else
                                v[j] = pyramid_op_1band(c, prev[j], sp, mt);
                            prev[j] = c;
                        }
                    } else if (MODE == MM_K2_PYR_TAB2) {   // two-band waves
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            __builtin_amdgcn_sched_barrier(0);
                            const int fy = fft_bin<LOG2N>(t, j);
                            const bool c0 = pk_col0(j, fy);
                            const int ix = k2_tix<LOG2N>(c0 ? fy : N - fy);
                            const c2 c = v[j];
                            if constexpr (SP > 0)
                                v[j] = pyramid_op_pow1<SP, true>(c, prev[j], sp, c0 ? tab0[ix] : tabN[ix],
                                                                 c0 ? ms0[ix] : msN[ix]);
                            else
                                v[j] = pyramid_op_2band(c, prev[j], sp, c0 ? tab0[ix] : tabN[ix],
                                                        c0 ? ms0[ix] : msN[ix]);
                            prev[j] = c;
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            __builtin_amdgcn_sched_barrier(0);
                            const int fy = fft_bin<LOG2N>(t, j);
                            const c2 c = v[j];
                            v[j] = pk_col0(j, fy) ? k2_op<LOG2N, MODE>(c, prev[j], 0, fy, sp, tab0)
                                                  : k2_op<LOG2N, MODE>(c, prev[j], N / 2, N - fy, sp, tabN);
                            prev[j] = c;
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) prev[j] = v[j];
                }
                // column N/2's real bins 0 and N/2: FN = Im Z there (Z(0) and
                // Z(N/2) are their own partners, still in LDS), op against
                // F_{t-1} in ldsX[0..1]; AN to ldsX[2..3] for thread 0's
                // recombine.  Threads T/4 and 3T/4 (waves 1 and 3 at N = 2048,
                // not wave 0, which holds fy = 0 and N/2 in the recombine).
#pragma unroll
                for (int x = 0; x < 2; ++x) {
                    if (t == (x ? 3 * T / 4 : T / 4)) {
                        const int fyx = x ? N / 2 : 0;
                        const c2 z = lds[zslot<LOG2N>(fyx)];
                        const c2 fn = mk(0.5f * (z.y + z.y), -0.5f * (z.x - z.x));
                        if (!pass_frame) ldsX[2 + x] = k2_op<LOG2N, MODE>(fn, ldsX[x], N / 2, fyx, sp, tabN);
                        ldsX[x] = fn;
                    }
                }
            } else {
                regular_op();   // the block's other group, between the same barriers
            }
            __syncthreads();   // partner reads of Z done: the buffer takes the ops
            // A0 at zslot_h(fy), AN at ZH + zslot_h(fy) (fy <= N/2): each
            // wave's writes and reads are consecutive slots (tools/lds_banks.py)
            constexpr int ZH = zslot_h_size<LOG2N>();
            static_assert(2 * ZH <= lds_complex<N>(), "recombine exchange fits the buffer");
            if (packed && !pass_frame) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int fy = fft_bin<LOG2N>(t, j);
                    if (pk_col0(j, fy)) lds[zslot_h<LOG2N>(fy)] = v[j];
                    else lds[ZH + zslot_h<LOG2N>(N - fy)] = v[j];
                }
            }
            __syncthreads();
            if (packed && !pass_frame) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int fy = fft_bin<LOG2N>(t, j);
                    c2 a0, an;
                    if (pk_col0(j, fy)) {   // A(fy) = A0(fy) + i AN(fy)
                        a0 = v[j];
                        an = fy == 0 ? ldsX[2] : (fy == N / 2 ? ldsX[3] : lds[ZH + zslot_h<LOG2N>(fy)]);
                    } else {                // A(fy) = conj A0(N-fy) + i conj AN(N-fy)
                        const c2 b = lds[zslot_h<LOG2N>(N - fy)];
                        a0 = mk(b.x, -b.y);
                        an = mk(v[j].x, -v[j].y);
                    }
                    v[j] = mk(a0.x - an.y, a0.y + an.x);
                }
            }
            __syncthreads();   // the inverse FFT rewrites the buffer
        }
        if constexpr (!blk0) regular_op();
#ifndef MM_K2_NOGAHEAD
        // next frame's G loads now: they land during this frame's inverse
        // transform, staging and Q stores instead of stalling the next frame
        // at its top (same-call K2 8.94 -> 8.33 us/frame, profiles/r03_abv.txt;
        // the op's registers are free again here: no spill at 123 VGPRs)
        if (!pass_frame) load_g(fr + 1 < nframes ? fr + 1 : nframes - 1, t);
#endif
        staged = !pass_frame;
        if (!pass_frame) {
        K2_STAMP(4);
        MM_MARK("M3_inv_start");
        fft_dit<LOG2N, +1, TT>(v, t, lds, wt, ttab);   // natural row order again
        MM_MARK("M4_inv_end");
        K2_STAMP(5);
        if (!stg_ded) __syncthreads();   // (aliased) every wave past its exchange reads: the staging overwrites them
        // Q is stored by row pairs (q_index) so that K3 reads each of its two
        // rows' values as one 16-B piece per bin, contiguous across the wave (a
        // column-major Q made K3's 16-B gathers cost it 4 of its 7 us/frame at
        // 1080p).  The GPW columns of the workgroup are transposed through LDS
        // (over the exchange buffers) and leave as one contiguous GPW*16-byte piece
        // per row pair; same-XCD workgroups complete the 128-B lines.
        // Rows that never wrap (rb >= 0, rb + Hq <= N, every geometry but H
        // close to N): list row k = t + jT - rb, staging slot s(k) = s(k0) + jT GPW
        // (T a multiple of TK): one base and immediate offsets.
        if (cstage) {
            const int s0 = ((t >> 1) * GPW + grp) * TK + (t & 1);   // T even: (t + jT)/2 = t/2 + jT/2
            if (valid) {
#pragma unroll
                for (int j = 0; j < 8; ++j) stg[k2_stg_swz(s0) + j * (T / 2) * GPW * TK] = v[j];   // packed: (Q0, QN)
            }
        } else if (T % TK == 0 && g.rb >= 0 && g.rb + g.Hq <= N) {
            const int k0 = t - g.rb;   // may be negative: floor division below
            const int s0 = ((k0 >> ilog2c(TK)) * GPW) * TK + (k0 & (TK - 1));
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (valid && (unsigned)(k0 + j * T) < (unsigned)g.Hq)
                    stg[k2_stg_swz(s0 + j * T * GPW + TK * grp)] = v[j];   // packed (grp 0): (Q0, QN)
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = (t + j * T - g.rb + 2 * N) & (N - 1);
                if (valid && k < g.Hq) stg[k2_stg_swz(((k / TK) * GPW) * TK + (k % TK) + TK * grp)] = v[j];
            }
        }
        }   // !pass_frame
        __syncthreads();   // staged pieces complete (stored at the top of the next iteration)
        K2_STAMP(6);
        return true;
    };
#ifndef MM_K2_UNROLL
#define MM_K2_UNROLL 1
#endif
    auto run_frames = [&](auto opk_c) __attribute__((always_inline)) {
        {
            int fr_prime = -1;   // opaque: the prime instance keeps the runtime passthrough test
            asm volatile("" : "+s"(fr_prime));
            frame_iter(fr_prime, opk_c);
        }
#if MM_K2_UNROLL == 2
        // two frames per trip: F_{t-1} alternates between the two bodies'
        // registers instead of being copied back at the loop's end
        for (int fr = 0;; fr += 2) {
            if (!frame_iter(fr, opk_c)) break;
            if (!frame_iter(fr + 1, opk_c)) break;
        }
#else
        for (int fr = 0;; ++fr)
            if (!frame_iter(fr, opk_c)) break;   // (fr >= 0 here: no passthrough branch)
#endif
    };
    if constexpr (blk0 || !k2_one_band_op<MODE>()) run_frames(std::integral_constant<int, -1>());
    else if (!wave_two_band) run_frames(std::integral_constant<int, 1>());
    else run_frames(std::integral_constant<int, 0>());
#ifdef MM_K2_STAMPS
    st_acc[7] = (__builtin_amdgcn_s_memrealtime() - st_acc[7]) << 32 | (st_acc[7] & 0xffffffffull);
    __builtin_amdgcn_s_waitcnt(0);   // every load and store of the wave completed
    const unsigned long long st_exit = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x % 64 == 0) {
        // k_cols_tail's workgroups (one per frame) after k_cols's 4096 waves
        const int w = (blk0 && nframes == 1 && gridDim.x < 512 ? 4096 : 0) +
                      blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        for (int i = 0; i < 8; ++i) mm_k2_stamps[w * 8 + i] = st_acc[i];
        mm_k2_entry[w] = st_entry;
        mm_k2_exit[w] = st_exit;
    }
#endif
}

#ifndef MM_K2_WAVES
#define MM_K2_WAVES 4
#endif

template <int LOG2N, int MODE, int SP = 0>
__global__ __launch_bounds__(k2_threads<LOG2N>()) __attribute__((amdgpu_waves_per_eu(MM_K2_WAVES)))
void k_cols(const c2 *G, size_t g_stride, const c2 *Gprev, c2 *Q, size_t q_stride,   // not restrict: G loads must stay ahead of Q stores
            int nframes, Geo g, Spec sp, const c2 *__restrict__ tw, const float2 *__restrict__ ktab,
            const float *__restrict__ kmsum, int stg_c2, int nframes_blk0, int tail_blocks, int ktail,
            int pk_off)
{
    // Blocks nb .. nb + tail_blocks - 1 (tail_blocks <= nb / 2) are tails: the
    // last ktail frames of the columns of second-half block nb/2 + i, which
    // stops that many frames early.  A CU's second workgroup (the younger,
    // second half of the dispatch) runs behind its first all launch long
    // (phase stamps: first half done at ~825 us, second at ~1,045 us per 100
    // frames); its tail starts in the slot the first one frees, primed with the
    // frame before its first (the state is a pure function of that frame).
    // pk_off = 1: block 0 (the packed group) is not in this launch (all its
    // frames run in k_cols_tail): the column blocks are 1 .. nb
    const int nb = gridDim.x - tail_blocks;
    const bool tail = (int)blockIdx.x >= nb;
    const int p = tail ? nb / 2 + ((int)blockIdx.x - nb) : (int)blockIdx.x;
    // same-XCD blocks own consecutive columns, so the pieces of one 128-B Q line
    // are merged in one L2 (split over XCDs they left as partial-line writes)
    const int blk = xcd_remap(p, nb) + pk_off;
    if (blk == 0) {   // the packed block stops nframes_blk0 frames in (k_cols_tail)
        k_cols_body<LOG2N, MODE, true, SP>(G, g_stride, Gprev, Q, q_stride, nframes_blk0, g, sp, tw, ktab, kmsum, stg_c2,
                                       blk, nb);
    } else {
        const int f0 = tail ? nframes - ktail : 0;
        const int nf = tail ? ktail : (p >= nb / 2 && p - nb / 2 < tail_blocks ? nframes - ktail : nframes);
        k_cols_body<LOG2N, MODE, false, SP>(G + (size_t)f0 * g_stride, g_stride,
                                        tail ? G + (size_t)(f0 - 1) * g_stride : Gprev,
                                        Q + (size_t)f0 * q_stride, q_stride, nf, g, sp, tw, ktab, kmsum, stg_c2,
                                        blk, nb);
    }
}

// The packed block's last frames, one workgroup per frame, after k_cols.
// Block 0 carries the packed group's extra exchanges and is k_cols's critical
// path, so the other blocks would idle at the end of the launch (rocprofv3:
// k_cols 1,016 us per 100 frames alone; 939 us + 24.5 us of k_cols_tail with
// the last 30 frames moved, 940 + 24.6 with 45: the 30 % default is past the
// point where block 0 stops being the critical path).  The state is a pure
// function of the previous input frame (.cs:142), so workgroup i primes with
// frame f0 + i - 1 (its passthrough frame sets F_{t-1} exactly as the frame
// loop would: bitwise the same outputs) and then runs frame f0 + i.
template <int LOG2N, int MODE, int SP = 0>
__global__ __launch_bounds__(k2_threads<LOG2N>()) __attribute__((amdgpu_waves_per_eu(MM_K2_WAVES)))
void k_cols_tail(const c2 *G, size_t g_stride, const c2 *Gprev, c2 *Q, size_t q_stride, int f0, Geo g, Spec sp,
                 const c2 *__restrict__ tw, const float2 *__restrict__ ktab, const float *__restrict__ kmsum,
                 int stg_c2)
{
    const int fr = f0 + (int)blockIdx.x;   // frame 0 primes with the state slot
    k_cols_body<LOG2N, MODE, true, SP>(G + (size_t)fr * g_stride, g_stride,
                                       fr > 0 ? G + (size_t)(fr - 1) * g_stride : Gprev,
                                       Q + (size_t)fr * q_stride, q_stride, 1, g, sp, tw, ktab, kmsum, stg_c2, 0);
}

// K2's per-bin tables of every column in LDS slot order ([N/2+1][k2_tab_slots]):
// the frame-invariant bin_static values (pyramid masks pre-scaled by inv_nn, a
// power of two: exact), evaluated once per parameter set on the launch stream
// (mm_api.hip launch_k2) instead of in every k_cols workgroup's prologue.
template <int LOG2N, int MODE>
__global__ __launch_bounds__(256) void k_k2_table(float2 *__restrict__ ktab, float *__restrict__ kmsum, Spec sp)
{
    constexpr int N = 1 << LOG2N, TE = k2_tab_entries<LOG2N>(), TS = k2_tab_slots<LOG2N>();
    constexpr int C = fft_c_v(LOG2N), QN = k2_tab_q<LOG2N>();
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= (N / 2 + 1) * TS) return;
    const int f = id / TS, slot = id - f * TS;
    const int e = C == 1 ? slot : (slot % QN) * C + slot / QN;   // k2_tix(e) == slot
    float2 v = make_float2(0.0f, 0.0f);
    float ms = 0.0f;
    if (e < TE) {
        const float ks = k2_tabled<MODE>() ? sp.inv_nn : 1.0f;
        const float2 b = bin_static<LOG2N, MODE>(f, e, sp);
        v = make_float2(b.x * ks, b.y * ks);
        if constexpr (k2_tabled<MODE>()) ms = bin_mask_sum<LOG2N>(f, e, sp) * ks;   // (read by MM_K2_PYR_TAB2)
    }
    ktab[id] = v;
    if constexpr (k2_tabled<MODE>()) kmsum[id] = ms;
}

// =========================================================================
// K3a: row C2R IFFT -> |z| -> horizontal blur -> Yh rows (fp32, global)
// =========================================================================
// One FFT group per pair of Q list rows (ka, ka+1); list row k is canvas row
// (rb + k) mod N.  PerformIFFT (.cs:563-620) ends in |z| (FFT.compute:143-150);
// the horizontal half of ApplyAntiAliasing (.cs:428-429) follows.
// One workgroup per Q tile (TK rows = GPW row pairs; pairs_per_frame = Hq/2
// counts the tile padding, pairs at or past Hn/2 compute but store nothing).
template <int LOG2N>
__global__ __launch_bounds__(k3_threads<LOG2N>())
void k_rows_inv(const c2 *__restrict__ Q, size_t q_stride, float *__restrict__ Yh,
                size_t yh_stride, int frame0, int pairs_per_frame, int total_pairs, Geo g,
                Blur5 bw, const c2 *__restrict__ tw)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), GPW = k3_groups<LOG2N>(), TK = q_tile<LOG2N>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = GPW == 1 ? 0 : (T % 64 == 0 ? __builtin_amdgcn_readfirstlane(threadIdx.x / T)
                                               : threadIdx.x / T);
    const int t = GPW == 1 ? threadIdx.x : threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const int logical = xcd_remap(blockIdx.x, gridDim.x) * GPW + grp;
    const int pair = logical % pairs_per_frame;
    const bool valid = logical < total_pairs && 2 * pair < g.Hn;
    const int frame = frame0 + (logical < total_pairs ? logical / pairs_per_frame : 0);
    const int ka = 2 * pair;
    // rows (ka, ka+1) of tile ka / TK: one 16-B piece per bin, TK*8 bytes apart
    // across the wave; the workgroup's groups read the whole TK*8-byte blocks
    const float4 *Qp = reinterpret_cast<const float4 *>(
        Q + (size_t)frame * q_stride + (size_t)(ka / TK) * g.Qs * TK + (ka % TK));
    float4 qv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {   // all 8 loads in flight (addresses always valid)
        const int fq = t + j * T;
        const int ff = fq > N / 2 ? N - fq : fq;
        qv[j] = Qp[(size_t)ff * (TK / 2)];
    }
    c2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int fq = t + j * T;
        const bool mirror = fq > N / 2;
        const int ff = mirror ? N - fq : fq;
        float4 q = qv[j];
        if (ff == 0 || ff == N / 2) { q.y = 0.0f; q.w = 0.0f; }   // C2R: DC/Nyquist real
        if (mirror) { q.y = -q.y; q.w = -q.w; }                   // X[N-f] = conj X[f]
        v[j] = valid ? mk(q.x - q.w, q.y + q.z) : mk(0.0f, 0.0f); // Z = Qa + i Qb
    }
    fft_regs<LOG2N, +1>(v, t, lds, tw);
    // the four-wide path reads the |z| rows kZShift floats in (taps c-2 .. c+5
    // as two aligned ds_read_b128, see k_rows_inv_compose)
    const bool wide = g.x0 >= 4 && g.x0 % 4 == 0 && g.Wy % 4 == 0 && g.x0 + g.Wy + 4 <= N;
    float *raw = reinterpret_cast<float *>(lds) + (wide ? kZShift : 0);   // [2][N] |z| of rows a, b
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        raw[t + j * T] = fabsf(v[j].x);
        raw[N + t + j * T] = fabsf(v[j].y);
    }
    __syncthreads();
    if (!valid) return;
    float *out = Yh + (size_t)frame * yh_stride + (size_t)ka * g.Wy;
    if (wide) {
        // four outputs per thread, one 16-B store; same expression and order
        // as the scalar form below
        const int W4 = g.Wy / 4;
        const float4 *raw4 = reinterpret_cast<const float4 *>(lds);
        for (int e = t; e < 2 * W4; e += T) {
            const int r = e >= W4 ? 1 : 0, X = 4 * (e - r * W4);
            const float4 *rw = raw4 + ((r * N + g.x0 + X) >> 2);
            const float4 P = rw[0], Z = rw[1];   // z[c-2 .. c+1], z[c+2 .. c+5]
            float4 o;
            o.x = bw.w0 * P.z + bw.w1 * (P.y + P.w) + bw.w2 * (P.x + Z.x);
            o.y = bw.w0 * P.w + bw.w1 * (P.z + Z.x) + bw.w2 * (P.y + Z.y);
            o.z = bw.w0 * Z.x + bw.w1 * (P.w + Z.y) + bw.w2 * (P.z + Z.z);
            o.w = bw.w0 * Z.y + bw.w1 * (Z.x + Z.z) + bw.w2 * (P.w + Z.w);
            st_stream<float4>(out, (unsigned)((r * g.Wy + X) * 4), o);
        }
        return;
    }
    // Wy = W columns (W + 1 for odd W: the crop's second texel)
    const bool interior = g.x0 >= 2 && g.x0 + g.Wy + 2 <= N;
    for (int e = t; e < 2 * g.Wy; e += T) {
        const int r = e >= g.Wy ? 1 : 0, X = e - r * g.Wy;
        const float *rw = raw + r * N;
        const int c = g.x0 + X;
        float acc;
        if (interior) {
            acc = bw.w0 * rw[c] + bw.w1 * (rw[c - 1] + rw[c + 1]) + bw.w2 * (rw[c - 2] + rw[c + 2]);
        } else {
            acc = bw.w0 * rw[wrap_idx(c, N, g.edge)];
            acc += bw.w1 * (rw[wrap_idx(c - 1, N, g.edge)] + rw[wrap_idx(c + 1, N, g.edge)]);
            acc += bw.w2 * (rw[wrap_idx(c - 2, N, g.edge)] + rw[wrap_idx(c + 2, N, g.edge)]);
        }
        out[(size_t)r * g.Wy + X] = acc;
    }
}

// =========================================================================
// K4: vertical blur -> YIQ recombine -> YIQ->RGB -> saturate -> crop
// =========================================================================
// One work-group per tile of kTileRows output rows x kTileCols columns, one
// column per thread: the vertical half of ApplyAntiAliasing (.cs:430-431) on
// Yh, CombineYIQChannels (.cs:437-442; I/Q of the windowed, padded current frame
// re-derived from the input through the same composite resample as K1), the
// YIQ->RGB blit (.cs:200-204) and CropTexture (.cs:386-410).
// The composite taps of image row/column i lie in {i-1, i, i+1} (checked on the
// host), so they are merged into 3 weights (w3 tables) and a tile needs source
// rows [i0-1, i0+TR] x columns [c0-1, c0+TC]: their I/Q are staged once in LDS;
// the horizontal 3-tap combine of every staged row and the TR+4 Yh values of the
// thread's column then live in registers.  One barrier per tile.
#ifndef MM_K4_ROWS
#define MM_K4_ROWS 6   // one-frame calls at 1080p: 8 -> 6 rows per tile 48.4-48.9 -> 47.6-47.8 us per call (4: 49.0-49.2, 16: 49.1-49.8; profiles/r03k_k4_rows_ab.txt)
#endif
#ifndef MM_K4_COLS
#define MM_K4_COLS 256
#endif
constexpr int kTileRows = MM_K4_ROWS, kTileCols = MM_K4_COLS;

template <int FMT>
__global__ __launch_bounds__(kTileCols)
void k_compose(const float *__restrict__ Yh, size_t yh_stride, const uint8_t *__restrict__ frames_in,
               uint8_t *__restrict__ frames_out, size_t frame_bytes, int frame0, int row_tiles,
               int col_tiles, Geo g, Blur5 bw, const float4 *__restrict__ colW3,
               const float4 *__restrict__ rowW3)
{
    constexpr int TR = kTileRows, TC = kTileCols, WC = TC + 2;
    __shared__ c2 iq[(TR + 2) * WC];         // I/Q of the staged source pixels
    const int tid = threadIdx.x;
    int b = blockIdx.x;
    const int ct = b % col_tiles;
    b /= col_tiles;
    const int rt = b % row_tiles;
    const int frame = frame0 + b / row_tiles;
    const int i0 = rt * TR, c0 = ct * TC;
    const uint8_t *img = frames_in + (size_t)frame * frame_bytes;

    // Staged entry (sr, j) is source pixel (row i0-1+sr, column c0-1+j), wrapped
    // or clamped like the resample's sampler.  Rows are workgroup-uniform (scalar
    // base pointers); thread tid stages column j = tid of every row, and threads
    // 0, 1 also the halo columns j = TC, TC+1.
    using raw_t = typename Pix<FMT>::raw_t;
    // 32-bit offsets from workgroup-uniform row pointers: scalar base + vector
    // offset addressing, no 64-bit address math per access
    const unsigned colA = (unsigned)wrap_near(min(c0 - 1 + tid, g.W), g.W, g.edge);
    raw_t pa[TR + 2];
#pragma unroll
    for (int sr = 0; sr < TR + 2; ++sr) {   // all staging loads in flight, then convert
        const int row = wrap_near(min(i0 - 1 + sr, g.H), g.H, g.edge);
        pa[sr] = ld_off<raw_t>(img, (unsigned)(row * g.W + colA) * Pix<FMT>::bpp);
    }
    const int X = c0 + tid;
    const bool vx = X < g.W;
    const float4 wc = colW3[min(X, g.W - 1)];
    // Yh of this column for the TR+4 canvas rows y0+i0-2 .. y0+i0+TR+1 (wrapped
    // or clamped like the blur's sampler, then mapped to Yh list rows), issued
    // before the I/Q conversions so that all loads share one memory round trip
    const float *Yf = Yh + (size_t)frame * yh_stride;
    const unsigned Xc = (unsigned)min(X, g.W - 1);
    float yv[TR + 4];
#pragma unroll
    for (int v = 0; v < TR + 4; ++v) {   // unconditional loads at clamped addresses
        const int cy = wrap_near(g.y0 + i0 - 2 + v, g.N, g.edge);
        const int k = (cy - g.rb + 2 * g.N) & (g.N - 1);
        const float y = ld_off<float>(Yf, (unsigned)(min(k, g.Hn - 1) * g.Wy + Xc) * 4u);
        yv[v] = k < g.Hn ? y : 0.0f;
    }
    // halo columns j = TC, TC + 1 of the TR + 2 rows: one entry for each of
    // threads 0 .. 2(TR+2)-1, loaded with the others (unconditional, clamped)
    constexpr int NH = 2 * (TR + 2);
    const int hs = min(tid, NH - 1);
    const int hrow = wrap_near(min(i0 - 1 + (hs >> 1), g.H), g.H, g.edge);
    const int hcol = wrap_near(min(c0 - 1 + TC + (hs & 1), g.W), g.W, g.edge);
    const raw_t ph = ld_off<raw_t>(img, (unsigned)(hrow * g.W + hcol) * Pix<FMT>::bpp);
    if (tid < NH) iq[(hs >> 1) * WC + TC + (hs & 1)] = chroma_iq2<FMT>(ph);
#pragma unroll
    for (int sr = 0; sr < TR + 2; ++sr) iq[sr * WC + tid] = chroma_iq2<FMT>(pa[sr]);
    __syncthreads();
    if (!vx) return;
    c2 hc[TR + 2];   // horizontally combined (I, Q) of each staged row
#pragma unroll
    for (int sr = 0; sr < TR + 2; ++sr) {
        const c2 a = iq[sr * WC + tid], m = iq[sr * WC + tid + 1], c = iq[sr * WC + tid + 2];
        hc[sr] = wc.x * a + wc.y * m + wc.z * c;
    }
    uint8_t *outp = frames_out + (size_t)frame * frame_bytes;
    const Blur5 bv = vblur_w<FMT>(bw);
#pragma unroll
    for (int r = 0; r < TR; ++r) {
        const int i = i0 + r;
        if (i < g.H) {
            const float4 wr = rowW3[i];                        // source rows i-1, i, i+1
            const c2 cc = wr.x * hc[r] + wr.y * hc[r + 1] + wr.z * hc[r + 2];   // (ci, cq)
            const float yb = bv.w0 * yv[r + 2] + bv.w1 * (yv[r + 1] + yv[r + 3]) +
                             bv.w2 * (yv[r] + yv[r + 4]);
            float rr, gg, bb;
            yiq_rgb<FMT>(yb, cc, rr, gg, bb);
            out_store<FMT>(outp + (unsigned)(i * g.W * Pix<FMT>::bpp), (unsigned)X, rr, gg, bb);
        }
    }
}

// =========================================================================
// K34: K3 + K4 fused (even W, H with W % 8 == 0, N - W >= 8, N - H >= 4)
// =========================================================================
// One workgroup of two FFT groups (2T = N/4 threads >= W/4 column quads) walks
// a strip of R = 4 (steps - 1) output rows of one frame top to bottom.  Step s
// inverse-transforms the Q list-row pairs i0/2 + 2s + {0, 1} (list rows
// i0+4s .. i0+4s+3) exactly as k_rows_inv does, blurs them horizontally from
// LDS, and thread q keeps the blurred values of its quad X = 4q .. 4q+3 in
// registers.  Output row i reads list rows i .. i+4 (rb = y0 - 2 and no row of
// the vertical blur wraps when N - H >= 4), so from step 1 on the 8 list rows
// in registers are the taps of output rows i0+4s-4 .. i0+4s-1, composed as
// k_compose does (same expressions).  Yh never goes through HBM: the frame
// saves its write and re-read (2 x 4 Hn W bytes); a strip re-transforms 4
// halo rows (4 / R more Q reads and FFT work).
#ifdef MM_K34_STAMPS
// Diagnostic build only: per-wave cycle totals of the strip-step phases
// (s_memtime deltas), written by lane 0 with a vector store after the walk.
__device__ unsigned long long mm_k34_stamps[65536 * 8];
#define K34_STAMP(i)                                                     \
    do {                                                                 \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();      \
        st_acc[i] += n_ - st_prev;                                       \
        st_prev = n_;                                                    \
    } while (0)
#else
#define K34_STAMP(i) do { } while (0)
#endif
template <int LOG2N, int FMT>
__global__ __launch_bounds__(2 * fft_T<LOG2N>()) __attribute__((amdgpu_waves_per_eu(4)))
void k_rows_inv_compose(const c2 *__restrict__ Q, size_t q_stride,
                        const uint8_t *__restrict__ frames_in, uint8_t *__restrict__ frames_out,
                        size_t frame_bytes, int frame0, int strips, int steps, Geo g, Blur5 bw,
                        const float4 *__restrict__ colW3, const float4 *__restrict__ rowW3,
                        const c2 *__restrict__ tw)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), TK = q_tile<LOG2N>();
    using raw_t = typename Pix<FMT>::raw_t;
    constexpr unsigned bpp = Pix<FMT>::bpp;
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = T % 64 == 0 ? __builtin_amdgcn_readfirstlane(threadIdx.x / T) : threadIdx.x / T;
    const int t = threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const float *raw_all = reinterpret_cast<const float *>(lds_all);
    constexpr int GROUP_FLOATS = 2 * lds_complex<N>();
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int frame = frame0 + b / strips;
    const int i0 = (b % strips) * 4 * (steps - 1);
    const c2 *Qf = Q + (size_t)frame * q_stride;
    const uint8_t *img = frames_in + (size_t)frame * frame_bytes;
    uint8_t *outp = frames_out + (size_t)frame * frame_bytes;

    const int q = threadIdx.x;
    const bool vq = 4 * q < g.W;
    const int X = vq ? 4 * q : g.W - 4;     // clamped quad (loads stay in the image)
    const unsigned cl = (unsigned)wrap_near(X - 1, g.W, g.edge);
    const unsigned cr = (unsigned)wrap_near(X + 4, g.W, g.edge);
    // horizontally combined I/Q of one source row for the quad (k_compose's
    // staged 3-tap combine over columns X-1 .. X+4)
    const Blur5 bv = vblur_w<FMT>(bw);   // the compose's vertical blur
    auto chroma_row = [&](int i, c2 (&hc)[4]) {
        const int row = wrap_near(min(i, g.H), g.H, g.edge);
        const unsigned base = (unsigned)(row * g.W);
        raw_t p[6];
        p[0] = ld_off<raw_t>(img, (base + cl) * bpp);
        if constexpr (bpp == 4) {
            const uint4 m = ld_off<uint4>(img, (base + (unsigned)X) * bpp);
            p[1] = m.x; p[2] = m.y; p[3] = m.z; p[4] = m.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) p[1 + k] = ld_off<raw_t>(img, (base + (unsigned)X + k) * bpp);
        }
        p[5] = ld_off<raw_t>(img, (base + cr) * bpp);
        c2 a[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) a[k] = chroma_iq2<FMT>(p[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 wc = colW3[X + k];
            hc[k] = wc.x * a[k] + wc.y * a[k + 1] + wc.z * a[k + 2];
        }
    };

    float yw[8][4];            // list rows i0+4s-4 .. i0+4s+3 of the quad (blurred horizontally)
                               // (as column pairs for a packed vertical blur: +3 spills, not kept)
    c2 hc[6][4];               // combined (I, Q) of source rows i0+4s-5 .. i0+4s
    chroma_row(i0 - 1, hc[4]);
    chroma_row(i0, hc[5]);
#ifdef MM_K34_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
    st_acc[7] = __builtin_amdgcn_s_memrealtime();
#endif
    // Q rows of step s: list-row pair i0/2 + 2s + grp (zero beyond Hn).
    // MM_K34_QPF=1 (diagnostic) issues step s+1's Q loads after step s's blur,
    // to land under its compose: +32 live VGPRs, 120 B of spills at the
    // 128-VGPR bound (4 waves per SIMD) even with the compose two rows at a
    // time (MM_K34_ROWS2), so off by default.
    float4 qv[8];
    auto load_q = [&](int s_) {
        const int ka_ = i0 + 4 * s_ + 2 * grp;
        const int kl = ka_ < g.Hn ? ka_ : 0;
        const float4 *Qp = reinterpret_cast<const float4 *>(Qf + (size_t)(kl / TK) * g.Qs * TK + (kl % TK));
        // column ff = t + jT (j < 4) or N - t - jT (j >= 4; = N/2 at t = 0,
        // j = 4): a workgroup-uniform base per j plus one of two per-thread
        // offsets, not eight loop-invariant VGPR offsets
        const unsigned up = (unsigned)t * (TK / 2), dn = (unsigned)(T - 1 - t) * (TK / 2);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < 4) qv[j] = (Qp + (size_t)(j * T) * (TK / 2))[up];
            else qv[j] = (Qp + (size_t)(N - j * T - (T - 1)) * (TK / 2))[dn];
        }
    };
#ifndef MM_K34_QPF
#define MM_K34_QPF 0
#endif
    if (MM_K34_QPF) load_q(0);
    for (int s = 0; s < steps; ++s) {
        const int ka = i0 + 4 * s + 2 * grp;
        const bool valid = ka < g.Hn;
        if (!MM_K34_QPF) load_q(s);
        c2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int fq = t + j * T;
            const bool mirror = fq > N / 2;
            const int ff = mirror ? N - fq : fq;
            float4 qq = qv[j];
            if (ff == 0 || ff == N / 2) { qq.y = 0.0f; qq.w = 0.0f; }
            if (mirror) { qq.y = -qq.y; qq.w = -qq.w; }
            v[j] = valid ? mk(qq.x - qq.w, qq.y + qq.z) : mk(0.0f, 0.0f);
        }
        K34_STAMP(0);
        fft_regs<LOG2N, +1>(v, t, lds, tw);
        K34_STAMP(1);
#ifndef MM_K34_BLUR_R3
        float *raw = reinterpret_cast<float *>(lds) + kZShift;   // [2][N] |z| of rows ka, ka+1
#else
        float *raw = reinterpret_cast<float *>(lds);
#endif
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            raw[t + j * T] = fabsf(v[j].x);
            raw[N + t + j * T] = fabsf(v[j].y);
        }
        __syncthreads();
        K34_STAMP(2);
        // ---- horizontal blur of the 4 new list rows ----
        // |z| rows sit 2 floats into their LDS rows (zshift), so the taps
        // c-2 .. c+5 of the quad are TWO 16-B aligned ds_read_b128 (conflict-
        // free: consecutive 16 B per lane) instead of the compiler's two
        // ds_read2_b64 of 8-B aligned halves (2-way conflicts on every one,
        // tools/lds_banks.py "k34"); same expressions and order as k_rows_inv
        // one base address; the rows are immediate offsets
#ifndef MM_K34_BLUR_R3
        const float4 *b4 = reinterpret_cast<const float4 *>(raw_all) + ((g.x0 + X) >> 2);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 *r4 = b4 + ((r >> 1) * GROUP_FLOATS + (r & 1) * N) / 4;
            const float4 P = r4[0], Z = r4[1];   // z[c-2 .. c+1], z[c+2 .. c+5]
#else   // diagnostic: round 3's unshifted rows (taps read by the compiler's ds_read2_b64)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 *r4 = reinterpret_cast<const float4 *>(raw_all + (r >> 1) * GROUP_FLOATS + (r & 1) * N + g.x0 + X);
            const float4 A = r4[-1], B = r4[0], C = r4[1];
            const float4 P = make_float4(A.z, A.w, B.x, B.y), Z = make_float4(B.z, B.w, C.x, C.y);
#endif
            yw[4 + r][0] = bw.w0 * P.z + bw.w1 * (P.y + P.w) + bw.w2 * (P.x + Z.x);
            yw[4 + r][1] = bw.w0 * P.w + bw.w1 * (P.z + Z.x) + bw.w2 * (P.y + Z.y);
            yw[4 + r][2] = bw.w0 * Z.x + bw.w1 * (P.w + Z.y) + bw.w2 * (P.z + Z.z);
            yw[4 + r][3] = bw.w0 * Z.y + bw.w1 * (Z.x + Z.z) + bw.w2 * (P.w + Z.w);
        }
        __syncthreads();   // LDS free for the next step's FFT
        K34_STAMP(3);
        if (MM_K34_QPF && s + 1 < steps) load_q(s + 1);
        if (s > 0) {
            // ---- K4 on output rows i0+4s-4 .. i0+4s-1, two at a time ----
#pragma unroll
#ifndef MM_K34_ROWS2   // the 4 chroma rows' loads first (one memory round trip)
            for (int r = 0; r < 4; ++r) chroma_row(i0 + 4 * s - 3 + r, hc[2 + r]);
#endif
            for (int r = 0; r < 4; ++r) {
#ifdef MM_K34_ROWS2   // diagnostic: two rows at a time (120 VGPRs; same-call K34 +8 %, r04d)
                if (r % 2 == 0) {
                    chroma_row(i0 + 4 * s - 3 + r, hc[2 + r]);
                    chroma_row(i0 + 4 * s - 2 + r, hc[3 + r]);
                }
#endif
                K34_STAMP(4);
                const int i = i0 + 4 * s - 4 + r;
                if (vq && i < g.H) {
                    const float4 wr = rowW3[i];
                    float rr[4], gg[4], bb[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const c2 cc = wr.x * hc[r][k] + wr.y * hc[r + 1][k] + wr.z * hc[r + 2][k];
                        const float yb = bv.w0 * yw[r + 2][k] + bv.w1 * (yw[r + 1][k] + yw[r + 3][k]) +
                                         bv.w2 * (yw[r][k] + yw[r + 4][k]);
                        yiq_rgb<FMT>(yb, cc, rr[k], gg[k], bb[k]);
                    }
                    const unsigned o = (unsigned)(i * g.W + X);
                    if constexpr (bpp == 4) {
                        uint4 px;
                        px.x = out_pack<FMT>(rr[0], gg[0], bb[0]);
                        px.y = out_pack<FMT>(rr[1], gg[1], bb[1]);
                        px.z = out_pack<FMT>(rr[2], gg[2], bb[2]);
                        px.w = out_pack<FMT>(rr[3], gg[3], bb[3]);
                        // scalar row base + the thread's column offset: one
                        // live VGPR, not a hoisted offset per row
                        st_stream<uint4>(outp + (size_t)(unsigned)(i * g.W) * 4u, (unsigned)X * 4u, px);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) out_store<FMT>(outp, o + k, rr[k], gg[k], bb[k]);
                    }
                }
            }
        }
        K34_STAMP(5);
        // ---- slide: keep list rows i0+4s .. +3 and source rows i0+4s-1, i0+4s
        // (after step 0: the primed rows i0-1, i0) ----
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k) yw[r][k] = yw[4 + r][k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            hc[0][k] = hc[4][k];
            hc[1][k] = hc[5][k];
        }
    }
#ifdef MM_K34_STAMPS
    st_acc[6] = (unsigned long long)steps;
    st_acc[7] = (__builtin_amdgcn_s_memrealtime() - st_acc[7]) << 32 | (st_acc[7] & 0xffffffffull);
    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if (threadIdx.x % 64 == 0 && w < 65536)
        for (int i = 0; i < 8; ++i) mm_k34_stamps[w * 8 + i] = st_acc[i];
#endif
}

// K34 in one shot, for short launches (the one-frame drop-in call): a strip of
// 4 output rows needs list rows i0 .. i0+7, so a workgroup of FOUR FFT groups
// transforms all of them at once (group g: list-row pair i0/2 + g, exactly
// k_rows_inv_compose's step code), and then its two halves compose output
// rows i0 + 2hh and i0 + 2hh + 1 (hh = 0, 1) from the 6 list rows and 4 source
// rows they read: no sequential walk.  Twice the FFTs of the walking form
// (every list row is transformed by two strips), but one workgroup round, one
// launch instead of K3 + K4, and no Yh round trip.  Same expressions in the
// same order as K3 + K4: bitwise equal (tests/test_k34.py).  N <= 2048 (4T
// threads <= 1024).
template <int LOG2N, int FMT>
__global__ __launch_bounds__(4 * fft_T<LOG2N>())
void k_rows_inv_compose4(const c2 *__restrict__ Q, size_t q_stride,
                         const uint8_t *__restrict__ frames_in, uint8_t *__restrict__ frames_out,
                         size_t frame_bytes, int frame0, int strips, Geo g, Blur5 bw,
                         const float4 *__restrict__ colW3, const float4 *__restrict__ rowW3,
                         const c2 *__restrict__ tw)
{
    constexpr int N = 1 << LOG2N, T = fft_T<LOG2N>(), TK = q_tile<LOG2N>();
    using raw_t = typename Pix<FMT>::raw_t;
    constexpr unsigned bpp = Pix<FMT>::bpp;
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = T % 64 == 0 ? __builtin_amdgcn_readfirstlane(threadIdx.x / T) : threadIdx.x / T;
    const int t = threadIdx.x % T;
    c2 *lds = lds_all + grp * lds_complex<N>();
    const float *raw_all = reinterpret_cast<const float *>(lds_all);
    constexpr int GROUP_FLOATS = 2 * lds_complex<N>();
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int frame = frame0 + b / strips;
    const int i0 = (b % strips) * 4;
    const c2 *Qf = Q + (size_t)frame * q_stride;
    const uint8_t *img = frames_in + (size_t)frame * frame_bytes;
    uint8_t *outp = frames_out + (size_t)frame * frame_bytes;

    // ---- K3 on list-row pair i0/2 + grp (zero beyond Hn) ----
    {
        const int ka = i0 + 2 * grp;
        const bool valid = ka < g.Hn;
        const int kl = valid ? ka : 0;
        const float4 *Qp = reinterpret_cast<const float4 *>(Qf + (size_t)(kl / TK) * g.Qs * TK + (kl % TK));
        float4 qv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int fq = t + j * T;
            const int ff = fq > N / 2 ? N - fq : fq;
            qv[j] = Qp[(size_t)ff * (TK / 2)];
        }
        c2 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int fq = t + j * T;
            const bool mirror = fq > N / 2;
            const int ff = mirror ? N - fq : fq;
            float4 qq = qv[j];
            if (ff == 0 || ff == N / 2) { qq.y = 0.0f; qq.w = 0.0f; }
            if (mirror) { qq.y = -qq.y; qq.w = -qq.w; }
            v[j] = valid ? mk(qq.x - qq.w, qq.y + qq.z) : mk(0.0f, 0.0f);
        }
        fft_regs<LOG2N, +1>(v, t, lds, tw);
        float *raw = reinterpret_cast<float *>(lds) + kZShift;   // [2][N] |z| of rows ka, ka+1
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            raw[t + j * T] = fabsf(v[j].x);
            raw[N + t + j * T] = fabsf(v[j].y);
        }
    }
    __syncthreads();

    // ---- compose: half hh of the workgroup, output rows i0 + 2hh, i0 + 2hh + 1 ----
    const int q = threadIdx.x % (2 * T), hh = threadIdx.x / (2 * T);
    const bool vq = 4 * q < g.W;
    const int X = vq ? 4 * q : g.W - 4;
    const unsigned cl = (unsigned)wrap_near(X - 1, g.W, g.edge);
    const unsigned cr = (unsigned)wrap_near(X + 4, g.W, g.edge);
    const Blur5 bv = vblur_w<FMT>(bw);   // the compose's vertical blur
    auto chroma_row = [&](int i, c2 (&hc)[4]) {   // k_rows_inv_compose's
        const int row = wrap_near(min(i, g.H), g.H, g.edge);
        const unsigned base = (unsigned)(row * g.W);
        raw_t p[6];
        p[0] = ld_off<raw_t>(img, (base + cl) * bpp);
        if constexpr (bpp == 4) {
            const uint4 m = ld_off<uint4>(img, (base + (unsigned)X) * bpp);
            p[1] = m.x; p[2] = m.y; p[3] = m.z; p[4] = m.w;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) p[1 + k] = ld_off<raw_t>(img, (base + (unsigned)X + k) * bpp);
        }
        p[5] = ld_off<raw_t>(img, (base + cr) * bpp);
        c2 a[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) a[k] = chroma_iq2<FMT>(p[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 wc = colW3[X + k];
            hc[k] = wc.x * a[k] + wc.y * a[k + 1] + wc.z * a[k + 2];
        }
    };
    const int r0 = i0 + 2 * hh;   // first output row of this half
    c2 hc[4][4];                  // combined (I, Q) of source rows r0-1 .. r0+2
#pragma unroll
    for (int k = 0; k < 4; ++k) chroma_row(r0 - 1 + k, hc[k]);
    float yw[6][4];               // list rows r0 .. r0+5 of the quad, blurred horizontally
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int r = 2 * hh + k;   // list row i0 + r: group r/2, row r%2 (zshift: k_rows_inv_compose)
        const float4 *r4 = reinterpret_cast<const float4 *>(raw_all) + ((g.x0 + X) >> 2) +
                           ((r >> 1) * GROUP_FLOATS + (r & 1) * N) / 4;
        const float4 P = r4[0], Z = r4[1];   // z[c-2 .. c+1], z[c+2 .. c+5]
        yw[k][0] = bw.w0 * P.z + bw.w1 * (P.y + P.w) + bw.w2 * (P.x + Z.x);
        yw[k][1] = bw.w0 * P.w + bw.w1 * (P.z + Z.x) + bw.w2 * (P.y + Z.y);
        yw[k][2] = bw.w0 * Z.x + bw.w1 * (P.w + Z.y) + bw.w2 * (P.z + Z.z);
        yw[k][3] = bw.w0 * Z.y + bw.w1 * (Z.x + Z.z) + bw.w2 * (P.w + Z.w);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int i = r0 + r;
        if (vq && i < g.H) {
            const float4 wr = rowW3[i];
            float rr[4], gg[4], bb[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const c2 cc = wr.x * hc[r][k] + wr.y * hc[r + 1][k] + wr.z * hc[r + 2][k];
                const float yb = bv.w0 * yw[r + 2][k] + bv.w1 * (yw[r + 1][k] + yw[r + 3][k]) +
                                 bv.w2 * (yw[r][k] + yw[r + 4][k]);
                yiq_rgb<FMT>(yb, cc, rr[k], gg[k], bb[k]);
            }
            const unsigned o = (unsigned)(i * g.W + X);
            if constexpr (bpp == 4) {
                uint4 px;
                px.x = out_pack<FMT>(rr[0], gg[0], bb[0]);
                px.y = out_pack<FMT>(rr[1], gg[1], bb[1]);
                px.z = out_pack<FMT>(rr[2], gg[2], bb[2]);
                px.w = out_pack<FMT>(rr[3], gg[3], bb[3]);
                st_stream<uint4>(outp, o * 4u, px);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) out_store<FMT>(outp, o + k, rr[k], gg[k], bb[k]);
            }
        }
    }
}

// K4 for odd W and/or H: the quad's edge then sits half a texel off the
// texel grid (x0 + 0.5), and CropTexture (.cs:386-410) samples the final
// texture between two texels (four when both are odd) with weights 1/2: output
// pixel (X, Y) = mean of saturate(YIQ->RGB) at canvas texels x0 + X (+1),
// y0 + Y (+1) (oracle mm_ref.c crop).  A texel outside the quad has I = Q = 0
// (the cleared canvas) and the blurred Y' of that position.  One thread per
// output pixel; the I/Q of a texel is the composite resample from the unmerged
// Tap4 tables (taps on i-2 .. i+1 for odd sizes).
template <int FMT>
__global__ __launch_bounds__(256)
void k_compose_odd(const float *__restrict__ Yh, size_t yh_stride, const uint8_t *__restrict__ frames_in,
                   uint8_t *__restrict__ frames_out, size_t frame_bytes, int frame0, int nframes, Geo g,
                   Blur5 bw, const Tap4 *__restrict__ colT, const Tap4 *__restrict__ rowT)
{
    const size_t npx = (size_t)g.W * g.H;
    const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (e >= npx * nframes) return;
    const int k = (int)(e / npx);
    const int p = (int)(e - (size_t)k * npx);
    const int Y = p / g.W, X = p - Y * g.W;
    const int frame = frame0 + k;
    const uint8_t *img = frames_in + (size_t)frame * frame_bytes;
    const float *Yf = Yh + (size_t)frame * yh_stride;
    const float wt = (g.ox ? 0.5f : 1.0f) * (g.oy ? 0.5f : 1.0f);
    float acc[3] = {0.0f, 0.0f, 0.0f};
    for (int dy = 0; dy <= g.oy; ++dy)
        for (int dx = 0; dx <= g.ox; ++dx) {
            const int tx = X + dx, ty = Y + dy;   // texel's image column / row (may be W / H)
            // Y': vertical 5-tap blur of Yh (list row of canvas row y0+ty+d is ty+2+d)
            float yv[5];
            for (int d = 0; d < 5; ++d) {
                const int cy = wrap_near(g.y0 + ty - 2 + d, g.N, g.edge);
                const int kk = (cy - g.rb + 2 * g.N) & (g.N - 1);
                yv[d] = kk < g.Hn ? Yf[(size_t)kk * g.Wy + tx] : 0.0f;
            }
            const float yb = bw.w0 * yv[2] + bw.w1 * (yv[1] + yv[3]) + bw.w2 * (yv[0] + yv[4]);
            float ci = 0.0f, cq = 0.0f;
            if (tx < g.W && ty < g.H) {
                const Tap4 tc = colT[tx], tr = rowT[ty];
                for (int a = 0; a < 4; ++a) {
                    if (tr.w[a] == 0.0f) continue;
                    const int sr = wrap_near(tr.idx[a], g.H, g.edge);
                    float hi = 0.0f, hq = 0.0f;
                    for (int b = 0; b < 4; ++b) {
                        const int sc = wrap_near(tc.idx[b], g.W, g.edge);
                        const float2 iq = chroma_iq<FMT>(Pix<FMT>::raw(img, (size_t)sr * g.W + sc));
                        hi += tc.w[b] * iq.x;
                        hq += tc.w[b] * iq.y;
                    }
                    ci += tr.w[a] * hi;
                    cq += tr.w[a] * hq;
                }
            }
            acc[0] += wt * sat(1.0f * yb + 0.956f * ci + 0.621f * cq);
            acc[1] += wt * sat(1.0f * yb + -0.272f * ci + -0.647f * cq);
            acc[2] += wt * sat(1.0f * yb + -1.106f * ci + 1.703f * cq);
        }
    Pix<FMT>::store(frames_out + (size_t)frame * frame_bytes, (unsigned)p, acc[0], acc[1], acc[2]);
}

// =========================================================================
// f3 debug views: ProcessDebugView (.cs:234-257)
// =========================================================================
// The reference shows complexBuffer1 after PerformFFT, which its ping-pong
// (.cs:517-549) leaves one radix-2 column stage short of the spectrum: with
// R[r][kx] = (-1)^r Frow[r][(kx + N/2) mod N] (centred, row-transformed), rows
// [0, N/2) hold the N/2-point column DFT of the even rows r = 2m and rows
// [N/2, N) that of the odd rows (oracle mm_ref_fft_buffer1, tests/np_twin.py).
// One WG per (frame, column kx): group 0 transforms the even rows, group 1 the
// odd rows (T/2 threads each, N/2-point FFT).  Frow comes from K1's half
// spectra G (Hermitian: Frow[r][f] = conj G[N-f][r] for f > N/2; rows outside
// the image are zero).  Chunk frame fr = frame0 + blockIdx / N reads G[fr] and
// writes view texture fr - frame0.  Writes the log-magnitude view
// (ConvertComplexMagToTexScaled, FFT.compute:152-161) and/or the phase view
// (ConvertComplexPhaseToTex, :164-172) as N x N float textures.
template <int LOG2N>
__global__ __launch_bounds__(2 * fft_T<LOG2N - 1>())
void k_dbg_cols(const c2 *__restrict__ G, size_t g_stride, float *__restrict__ tex,
                size_t tex_stride, int frame0, int want_mag, int want_phase, Geo g,
                const c2 *__restrict__ tw_half)
{
    constexpr int N = 1 << LOG2N, M = N / 2, T = fft_T<LOG2N - 1>();
    extern __shared__ __attribute__((aligned(16))) c2 lds_all[];
    const int grp = threadIdx.x / T, t = threadIdx.x % T;   // 0: even rows, 1: odd rows
    c2 *lds = lds_all + grp * lds_complex<M>();
    const int kx = blockIdx.x % N, fr = frame0 + blockIdx.x / N;
    const int f = (kx + N / 2) & (N - 1);
    const bool mirror = f > N / 2;
    const c2 *Gc = G + (size_t)fr * g_stride + (size_t)(mirror ? N - f : f) * g.Hg;
    const float sgn = grp ? -1.0f : 1.0f;                     // (-1)^r
    c2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int r = 2 * (t + j * T) + grp;                   // canvas row
        const int rr = r - g.y0;
        const c2 a = Gc[min(max(rr, 0), g.H - 1)];
        const bool in = rr >= 0 && rr < g.H;
        v[j] = in ? mk(sgn * a.x, sgn * (mirror ? -a.y : a.y)) : mk(0.0f, 0.0f);
    }
    fft_regs<LOG2N - 1, -1>(v, t, lds, tw_half);
    float *mag = tex + (size_t)(fr - frame0) * tex_stride;
    float *pha = mag + (size_t)N * N;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int row = grp * M + t + j * T;
        const float m2 = v[j].x * v[j].x + v[j].y * v[j].y;
        if (want_mag) mag[(size_t)row * N + kx] = __log10f(__builtin_amdgcn_sqrtf(m2) * 10.0f + 1.0f) * 0.25f;
        if (want_phase) pha[(size_t)row * N + kx] = fabsf(atan2f(v[j].y, v[j].x)) * (1.0f / 1.57079632679f);
    }
}

// CropTexture (.cs:386-410) of one view, or ShowSplitScreen (.cs:458-487) of
// both (each N x N texture drawn bilinearly into one half).  RFloat textures
// sample as (v, 0, 0, 1).
template <int FMT>
__global__ __launch_bounds__(256)
void k_dbg_out(const float *__restrict__ tex, size_t tex_stride, uint8_t *__restrict__ frames_out,
               size_t frame_bytes, int frame0, int nframes, int show_mag, int show_phase, Geo g)
{
    const size_t npx = (size_t)g.W * g.H;
    const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (e >= npx * nframes) return;
    const int k = (int)(e / npx);
    const int p = (int)(e - (size_t)k * npx);
    const int Y = p / g.W, X = p - Y * g.W;
    const float *mag = tex + (size_t)k * tex_stride, *pha = mag + (size_t)g.N * g.N;
    float v;
    if (show_mag && show_phase) {
        const bool right = 2 * X + 1 >= g.W;
        const float u = (float)(2 * X + 1 - (right ? g.W : 0)) / (float)g.W;
        const float vv = (float)(2 * Y + 1) / (float)(2 * g.H);
        const float *tx = right ? pha : mag;
        // bilinear at texel (u N - 0.5, v N - 0.5), sampler wrap = edge mode
        const float sx = u * (float)g.N - 0.5f, sy = vv * (float)g.N - 0.5f;
        const float fx0 = floorf(sx), fy0 = floorf(sy);
        const float ax = sx - fx0, ay = sy - fy0;
        const int ix = (int)fx0, iy = (int)fy0;
        const int xa = wrap_idx(ix, g.N, g.edge), xb = wrap_idx(ix + 1, g.N, g.edge);
        const int ya = wrap_idx(iy, g.N, g.edge), yb = wrap_idx(iy + 1, g.N, g.edge);
        const float a = (1.0f - ax) * tx[(size_t)ya * g.N + xa] + ax * tx[(size_t)ya * g.N + xb];
        const float b = (1.0f - ax) * tx[(size_t)yb * g.N + xa] + ax * tx[(size_t)yb * g.N + xb];
        v = (1.0f - ay) * a + ay * b;
    } else {
        v = (show_mag ? mag : pha)[(size_t)(g.y0 + Y) * g.N + g.x0 + X];
    }
    if (kUnorm<FMT>) v = sat(v);   // UNORM destination
    Pix<FMT>::store(frames_out + (size_t)(frame0 + k) * frame_bytes, (unsigned)p, v, 0.0f, 0.0f);
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

static __global__ void k_synth(uint8_t *out, int W, int H, int t0, int count, uint64_t seed, int gray)
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
