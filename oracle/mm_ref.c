/*
 * mm_ref.c — CPU ORACLE (test infrastructure only; see mm_ref.h header).
 *
 * A literal fp32 restatement of the reference Unity pipeline, pyramid mode:
 *   OnRenderImage                 Assets/Scripts/MotionMagnificationProcessor.cs:101-143
 *   ProcessFrameWithPyramid...    .cs:145-206
 *   PadTexture / CropTexture      .cs:358-410 (+ BlitCopy.shader:42-46)
 *   ApplyWindowingFunction        .cs:412-421 (+ WindowingFunction.shader:47-70)
 *   ApplyAntiAliasing             .cs:423-433 (+ GaussianBlur.shader:47-60)
 *   ExtractY / CombineYIQ         .cs:435-442 (+ ExtractYChannel.shader:42-50,
 *                                   CombineYIQChannels.shader:44-57)
 *   RGB<->YIQ                     RGBToYIQ.shader:46-61, YIQToRGB.shader:51-79
 *   PerformFFT / PerformIFFT      .cs:508-620 (+ FFT.compute:79-276)
 *   GeneratePyramidFilters        .cs:694-708 (+ PyramidOperations.compute:25-87)
 *   Apply/Accumulate pyramid      PyramidOperations.compute:90-138
 *   ProcessPyramidPhaseDifference PyramidPhaseDifference.compute:47-101
 *
 * Engine-side semantics the reference does not pin (SURVEY.md §8c decisions):
 *   - bilinear filtering with exact fp32 weights, texel t = u*size - 0.5;
 *   - sampler wrap for the resamples and the blur: REPEAT (default) or CLAMP;
 *   - GL quad coverage: pixel X covered iff x0 <= X+0.5 < x0+W, u=(X+.5-x0)/W.
 * Build with -ffp-contract=off: every product/sum is rounded like the shader.
 */
#include "mm_ref.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI_F 3.14159265359f          /* FFT.compute:21, PyramidOperations.compute:5 */

typedef struct { float x, y; } cplx;

struct mm_ref {
    int W, H, N;
    int levels;
    float min_freq, max_freq, phase_scale, tau;
    int edge_mode;
    int apply;
    int first;               /* isFirstFrame, .cs:75 */
    float *prev;             /* previousSourceTexture, W*H*4, .cs:307 */
    float *masks;            /* pyramidFilters, levels*N*N, .cs:680 */
    int masks_levels;
    float mask_min, mask_max;
    /* standard (non-pyramid) mode, .cs:33-43 */
    int standard, bp_apply;
    float bp_low, bp_high, bp_steep, bp_sens, bp_edge;
    /* debug views showMagnitude / showPhase, .cs:13-14 */
    int show_mag, show_phase;
};

/* ------------------------------------------------------------------ */
/* small helpers                                                      */
/* ------------------------------------------------------------------ */
static int next_pow2(int v)                      /* Mathf.NextPowerOfTwo, .cs:301 */
{
    int n = 1;
    while (n < v) n <<= 1;
    return n;
}

static inline int wrap_index(int i, int n, int edge_mode)
{
    if (edge_mode == MMREF_EDGE_CLAMP) return i < 0 ? 0 : (i >= n ? n - 1 : i);
    int r = i % n;
    return r < 0 ? r + n : r;
}

static inline float saturatef(float v) { return v < 0.f ? 0.f : (v > 1.f ? 1.f : v); }

/* HLSL smoothstep(a,b,x) */
static inline float smoothstepf(float a, float b, float x)
{
    float t = saturatef((x - a) / (b - a));
    return t * t * (3.0f - 2.0f * t);
}

static inline cplx cmul(cplx a, cplx b)          /* FFT.compute:58-61 */
{
    cplx r;
    r.x = a.x * b.x - a.y * b.y;
    r.y = a.x * b.y + a.y * b.x;
    return r;
}

/* tex2D with bilinear filtering on a (w x h) texture of `ch` floats per texel,
 * sampled at normalized uv; result written to out[ch]. */
static void sample_bilinear(const float *tex, int w, int h, int ch, float u, float v,
                            int edge_mode, float *out)
{
    float tx = u * (float)w - 0.5f;
    float ty = v * (float)h - 0.5f;
    float fx0 = floorf(tx), fy0 = floorf(ty);
    int ix = (int)fx0, iy = (int)fy0;
    float fx = tx - fx0, fy = ty - fy0;
    int x0 = wrap_index(ix, w, edge_mode), x1 = wrap_index(ix + 1, w, edge_mode);
    int y0 = wrap_index(iy, h, edge_mode), y1 = wrap_index(iy + 1, h, edge_mode);
    const float *p00 = tex + ((size_t)y0 * w + x0) * ch;
    const float *p10 = tex + ((size_t)y0 * w + x1) * ch;
    const float *p01 = tex + ((size_t)y1 * w + x0) * ch;
    const float *p11 = tex + ((size_t)y1 * w + x1) * ch;
    for (int c = 0; c < ch; ++c) {
        float a = (1.0f - fx) * p00[c] + fx * p10[c];
        float b = (1.0f - fx) * p01[c] + fx * p11[c];
        out[c] = (1.0f - fy) * a + fy * b;
    }
}

/* ------------------------------------------------------------------ */
/* colour                                                             */
/* ------------------------------------------------------------------ */
void mm_ref_rgb_to_yiq(const float *rgb, float *yiq)   /* RGBToYIQ.shader:46-58 */
{
    yiq[0] = 0.299f * rgb[0] + 0.587f * rgb[1] + 0.114f * rgb[2];
    yiq[1] = 0.596f * rgb[0] + -0.274f * rgb[1] + -0.322f * rgb[2];
    yiq[2] = 0.211f * rgb[0] + -0.523f * rgb[1] + 0.312f * rgb[2];
}

void mm_ref_yiq_to_rgb(const float *yiq, float *rgb)   /* YIQToRGB.shader:51-76 */
{
    rgb[0] = saturatef(1.0f * yiq[0] + 0.956f * yiq[1] + 0.621f * yiq[2]);
    rgb[1] = saturatef(1.0f * yiq[0] + -0.272f * yiq[1] + -0.647f * yiq[2]);
    rgb[2] = saturatef(1.0f * yiq[0] + -1.106f * yiq[1] + 1.703f * yiq[2]);
}

/* ------------------------------------------------------------------ */
/* FFT.compute restatement                                             */
/* ------------------------------------------------------------------ */
static void bitrev_indices(int n, unsigned *rev)        /* FFT.compute:79-96 */
{
    int bits = 0;
    while ((1 << (bits + 1)) <= n) ++bits;              /* firstbithigh(N) */
    for (int i = 0; i < n; ++i) {
        unsigned r = 0, o = (unsigned)i;
        for (int j = 0; j < bits; ++j) { r = (r << 1) | (o & 1u); o >>= 1; }
        rev[i] = r;
    }
}

static void twiddles(int n, cplx *tw)                   /* FFT.compute:99-110 */
{
    for (int k = 0; k < n / 2; ++k) {
        float phase = -(float)k * (2.0f * PI_F) / (float)n;
        tw[k].x = cosf(phase);
        tw[k].y = sinf(phase);
    }
}

/* Row then column radix-2 DIT passes over src (in place via ping-pong);
 * returns the buffer holding the result.  .cs:517-549 / FFT.compute:213-276 */
static cplx *fft2d_passes(int n, cplx *b1, cplx *b2)
{
    unsigned *rev = (unsigned *)malloc(sizeof(unsigned) * n);
    cplx *tw = (cplx *)malloc(sizeof(cplx) * (n / 2 > 0 ? n / 2 : 1));
    bitrev_indices(n, rev);
    twiddles(n, tw);

    /* BitRevByRow: b2 -> b1 */
    #pragma omp parallel for schedule(static)
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x)
            b1[(size_t)y * n + x] = b2[(size_t)y * n + rev[x]];
    cplx *src = b1, *dst = b2;
    for (int s = 2; s <= n; s *= 2) {                     /* ButterflyByRow */
        const int half = s / 2;
        #pragma omp parallel for schedule(static)
        for (int y = 0; y < n; ++y) {
            const cplx *row = src + (size_t)y * n;
            cplx *out = dst + (size_t)y * n;
            for (int x = 0; x < n; ++x) {
                int grp = x / s, gi = x % s, off = grp * s, hi = gi % half;
                cplx a = row[off + hi];
                cplx b = row[off + half + hi];
                cplx w = tw[(size_t)hi * (unsigned)n / (unsigned)s];
                cplx bw = cmul(b, w);
                cplx r;
                if (gi < half) { r.x = a.x + bw.x; r.y = a.y + bw.y; }
                else           { r.x = a.x - bw.x; r.y = a.y - bw.y; }
                out[x] = r;
            }
        }
        cplx *t = src; src = dst; dst = t;
    }
    /* (reference recomputes bitrev/twiddles for N=height here; square => same) */
    #pragma omp parallel for schedule(static)
    for (int y = 0; y < n; ++y)                           /* BitRevByCol */
        for (int x = 0; x < n; ++x)
            dst[(size_t)y * n + x] = src[(size_t)rev[y] * n + x];
    { cplx *t = src; src = dst; dst = t; }
    for (int s = 2; s <= n; s *= 2) {                     /* ButterflyByCol */
        const int half = s / 2;
        #pragma omp parallel for schedule(static)
        for (int y = 0; y < n; ++y) {
            int grp = y / s, gi = y % s, off = grp * s, hi = gi % half;
            const cplx *ra = src + (size_t)(off + hi) * n;
            const cplx *rb = src + (size_t)(off + half + hi) * n;
            cplx w = tw[(size_t)hi * (unsigned)n / (unsigned)s];
            cplx *out = dst + (size_t)y * n;
            for (int x = 0; x < n; ++x) {
                cplx bw = cmul(rb[x], w);
                cplx r;
                if (gi < half) { r.x = ra[x].x + bw.x; r.y = ra[x].y + bw.y; }
                else           { r.x = ra[x].x - bw.x; r.y = ra[x].y - bw.y; }
                out[x] = r;
            }
        }
        cplx *t = src; src = dst; dst = t;
    }
    free(rev);
    free(tw);
    return src;
}

/* PerformFFT (.cs:508-553): ConvertTexToComplex (FFT.compute:113-120),
 * CenterComplex (:175-189), row/col passes, ConvertComplexToTexRG (:133-140). */
void mm_ref_fft_centered(int n, const float *y, float *out_cplx)
{
    size_t nn = (size_t)n * n;
    cplx *b1 = (cplx *)malloc(sizeof(cplx) * nn);
    cplx *b2 = (cplx *)malloc(sizeof(cplx) * nn);
    #pragma omp parallel for schedule(static)
    for (int yy = 0; yy < n; ++yy)
        for (int x = 0; x < n; ++x) {
            size_t p = (size_t)yy * n + x;
            float v = y[p];
            b1[p].x = v; b1[p].y = 0.0f;
            if (((x + yy) & 1) != 0) { b2[p].x = -b1[p].x; b2[p].y = -b1[p].y; }
            else b2[p] = b1[p];
        }
    cplx *res = fft2d_passes(n, b1, b2);
    memcpy(out_cplx, res, sizeof(cplx) * nn);
    free(b1);
    free(b2);
}

/* complexBuffer1 after PerformFFT (.cs:508-553), the buffer ProcessDebugView
 * reads (.cs:243-255).  The ping-pong of .cs:517-549 always ends with the
 * spectrum in complexBuffer2, so complexBuffer1 holds the state after the
 * PENULTIMATE column butterfly stage: rows [0,N/2) the N/2-point column DFTs of
 * the even (centred) rows, rows [N/2,N) those of the odd rows, each row already
 * fully transformed.  Restated literally (fft2d_passes' b1). */
void mm_ref_fft_buffer1(int n, const float *y, float *out_cplx)
{
    size_t nn = (size_t)n * n;
    cplx *b1 = (cplx *)malloc(sizeof(cplx) * nn);
    cplx *b2 = (cplx *)malloc(sizeof(cplx) * nn);
    #pragma omp parallel for schedule(static)
    for (int yy = 0; yy < n; ++yy)
        for (int x = 0; x < n; ++x) {
            size_t p = (size_t)yy * n + x;
            float v = y[p];
            b1[p].x = v; b1[p].y = 0.0f;
            if (((x + yy) & 1) != 0) { b2[p].x = -b1[p].x; b2[p].y = -b1[p].y; }
            else b2[p] = b1[p];
        }
    cplx *res = fft2d_passes(n, b1, b2);
    (void)res;   /* == b2 for every n (even + odd stage counts), see above */
    memcpy(out_cplx, b1, sizeof(cplx) * nn);
    free(b1);
    free(b2);
}

/* PerformIFFT (.cs:563-620): ConvertTextureToComplex, Conjugate, passes,
 * Conjugate, DivideComplexByDimensions (FFT.compute:202-210), CenterComplex,
 * ConvertComplexMagToTex (FFT.compute:143-150). */
void mm_ref_ifft_mag(int n, const float *in_cplx, float *out_mag)
{
    size_t nn = (size_t)n * n;
    cplx *b1 = (cplx *)malloc(sizeof(cplx) * nn);
    cplx *b2 = (cplx *)malloc(sizeof(cplx) * nn);
    const cplx *in = (const cplx *)in_cplx;
    #pragma omp parallel for schedule(static)
    for (size_t p = 0; p < nn; ++p) { b2[p].x = in[p].x; b2[p].y = -in[p].y; }
    cplx *res = fft2d_passes(n, b1, b2);
    float dim = (float)n * (float)n;
    #pragma omp parallel for schedule(static)
    for (int yy = 0; yy < n; ++yy)
        for (int x = 0; x < n; ++x) {
            size_t p = (size_t)yy * n + x;
            cplx v = res[p];
            v.y = -v.y;                                    /* ConjugateComplex */
            v.x = v.x / dim; v.y = v.y / dim;              /* Divide */
            if (((x + yy) & 1) != 0) { v.x = -v.x; v.y = -v.y; } /* Center */
            out_mag[p] = sqrtf(v.x * v.x + v.y * v.y);     /* ComplexMagnitude */
        }
    free(b1);
    free(b2);
}

/* ------------------------------------------------------------------ */
/* PyramidOperations.compute:25-87                                     */
/* ------------------------------------------------------------------ */
void mm_ref_mask(int n, int levels, int index, float min_freq, float max_freq,
                 float *out)
{
    #pragma omp parallel for schedule(static)
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) {
            float fx = ((float)x / (float)n) - 0.5f;
            float fy = ((float)y / (float)n) - 0.5f;
            float freq = sqrtf(fx * fx + fy * fy);
            float v = 0.0f;
            if (index == 0) {
                if (freq > max_freq) v = 1.0f;
                else if (freq > max_freq * 0.8f) {
                    float t = (freq - max_freq * 0.8f) / (max_freq * 0.2f);
                    v = smoothstepf(0.0f, 1.0f, t);
                }
            } else if (index == levels - 1) {
                if (freq < min_freq) v = 1.0f;
                else if (freq < min_freq * 1.2f) {
                    float t = (freq - min_freq) / (min_freq * 0.2f);
                    v = 1.0f - smoothstepf(0.0f, 1.0f, t);
                }
            } else {
                float ratio = (float)(index - 1) / (float)(levels - 3); /* L=3: NaN */
                float center = min_freq * powf(max_freq / min_freq, 1.0f - ratio);
                float bw = center * 0.5f;
                float lo = center - bw, hi = center + bw;
                if (freq >= lo && freq <= hi) {
                    float nrm = (freq - lo) / (hi - lo);
                    v = 0.5f * (1.0f + cosf(2.0f * PI_F * (nrm - 0.5f)));
                }
            }
            out[(size_t)y * n + x] = v;
        }
}

/* PhaseDifferenceComputeShader.compute:74-85 */
static float spatial_frequency(int x, int y, int n)
{
    float fx = ((float)x / (float)n) - 0.5f;
    float fy = ((float)y / (float)n) - 0.5f;
    float freq = sqrtf(fx * fx + fy * fy);
    float r = freq / 0.707f;
    return r < 1.0f ? r : 1.0f;
}

/* PhaseDifferenceComputeShader.compute:88-122 */
static float bandpass_weight(float sf, int apply, float low, float high, float steep,
                             float sens, float edge)
{
    if (apply == 0) return 1.0f;
    float weight = 1.0f;
    if (sf < low) {
        float ratio = sf / fmaxf(low, 0.001f);
        weight *= powf(ratio, steep);
    }
    if (sf > high) {
        float ratio = (1.0f - sf) / fmaxf(1.0f - high, 0.001f);
        weight *= powf(ratio, steep);
    }
    weight *= sens;
    if (sf > low && sf < high) {
        float edge_factor = 1.0f + edge * sinf(PI_F * (sf - low) / (high - low));
        weight *= edge_factor;
    }
    return fmaxf(weight, 0.0f);
}

void mm_ref_bandpass_weights(int n, int apply, float low, float high, float steep,
                             float sens, float edge, float *out)
{
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x)
            out[(size_t)y * n + x] =
                bandpass_weight(spatial_frequency(x, y, n), apply, low, high, steep, sens, edge);
}

/* PyramidPhaseDifference.compute:47-54 */
float mm_ref_normalize_phase(float phase)
{
    while (phase > PI_F) phase -= 2.0f * PI_F;
    while (phase < -PI_F) phase += 2.0f * PI_F;
    return phase;
}

/* ------------------------------------------------------------------ */
/* raster passes                                                        */
/* ------------------------------------------------------------------ */
/* Graphics.Blit(src W*H -> yiq N*N, RGBToYIQ) (.cs:147), PadTexture (.cs:358-384)
 * with BlitCopy quad sampling, then ApplyWindowingFunction (.cs:412-421). */
void mm_ref_pad_window(mm_ref *ctx, const float *in_rgba, float *out_canvas)
{
    const int W = ctx->W, H = ctx->H, N = ctx->N;
    size_t nn = (size_t)N * N;
    float *yiq = (float *)malloc(sizeof(float) * nn * 4);
    /* stretch blit with the RGB->YIQ material: full-screen, uv at texel centres */
    #pragma omp parallel for schedule(static)
    for (int Y = 0; Y < N; ++Y)
        for (int X = 0; X < N; ++X) {
            float uv_x = ((float)X + 0.5f) / (float)N;
            float uv_y = ((float)Y + 0.5f) / (float)N;
            float c[4];
            sample_bilinear(in_rgba, W, H, 4, uv_x, uv_y, ctx->edge_mode, c);
            float *o = yiq + ((size_t)Y * N + X) * 4;
            mm_ref_rgb_to_yiq(c, o);
            o[3] = c[3];
        }
    /* GL.Clear(black) then the quad over [x0,x0+W) x [y0,y0+H) */
    #pragma omp parallel for schedule(static)
    for (int Y = 0; Y < N; ++Y)
        for (int X = 0; X < N; ++X) {
            float *o = out_canvas + ((size_t)Y * N + X) * 4;
            int nx = 2 * X + 1 - (N - W), ny = 2 * Y + 1 - (N - H);
            if (nx < 0 || nx >= 2 * W || ny < 0 || ny >= 2 * H) {
                o[0] = o[1] = o[2] = o[3] = 0.0f;
            } else {
                float u = (float)nx / (float)(2 * W);
                float v = (float)ny / (float)(2 * H);
                sample_bilinear(yiq, N, N, 4, u, v, ctx->edge_mode, o);
            }
            /* WindowingFunction.shader:47-70 (rgb only; alpha kept) */
            float wu = ((float)X + 0.5f) / (float)N;
            float wv = ((float)Y + 0.5f) / (float)N;
            float wx = 0.5f * (1.0f - cosf(2.0f * PI_F * wu));
            float wy = 0.5f * (1.0f - cosf(2.0f * PI_F * wv));
            float w = wx * wy;
            o[0] *= w; o[1] *= w; o[2] *= w;
        }
    free(yiq);
}

/* ApplyAntiAliasing (.cs:423-433) with GaussianBlur.shader:47-60, in place. */
static void blur_pass(int n, int edge_mode, const float *src, float *dst, int dirx)
{
    const float texel = (1.0f / (float)n) * 0.5f;    /* _MainTex_TexelSize * _BlurSize */
    const float o1 = texel * 1.3846153846f, o2 = texel * 3.2307692308f;
    #pragma omp parallel for schedule(static)
    for (int Y = 0; Y < n; ++Y)
        for (int X = 0; X < n; ++X) {
            float u = ((float)X + 0.5f) / (float)n;
            float v = ((float)Y + 0.5f) / (float)n;
            float du1 = dirx ? o1 : 0.0f, dv1 = dirx ? 0.0f : o1;
            float du2 = dirx ? o2 : 0.0f, dv2 = dirx ? 0.0f : o2;
            float s;
            float col;
            sample_bilinear(src, n, n, 1, u, v, edge_mode, &s);
            col = s * 0.2270270270f;
            sample_bilinear(src, n, n, 1, u + du1, v + dv1, edge_mode, &s);
            col += s * 0.3162162162f;
            sample_bilinear(src, n, n, 1, u - du1, v - dv1, edge_mode, &s);
            col += s * 0.3162162162f;
            sample_bilinear(src, n, n, 1, u + du2, v + dv2, edge_mode, &s);
            col += s * 0.0702702703f;
            sample_bilinear(src, n, n, 1, u - du2, v - dv2, edge_mode, &s);
            col += s * 0.0702702703f;
            dst[(size_t)Y * n + X] = col;
        }
}

void mm_ref_blur(int n, int edge_mode, float *img)
{
    float *tmp = (float *)malloc(sizeof(float) * (size_t)n * n);
    blur_pass(n, edge_mode, img, tmp, 1);
    blur_pass(n, edge_mode, tmp, img, 0);
    free(tmp);
}

/* ------------------------------------------------------------------ */
/* operator                                                             */
/* ------------------------------------------------------------------ */
static void regen_masks(mm_ref *c)                    /* GeneratePyramidFilters .cs:694-708 */
{
    size_t nn = (size_t)c->N * c->N;
    free(c->masks);
    c->masks = (float *)malloc(sizeof(float) * nn * (c->levels > 0 ? c->levels : 1));
    for (int i = 0; i < c->levels; ++i)
        mm_ref_mask(c->N, c->levels, i, c->min_freq, c->max_freq, c->masks + nn * i);
    c->masks_levels = c->levels;
    c->mask_min = c->min_freq;
    c->mask_max = c->max_freq;
}

mm_ref *mm_ref_create(int width, int height, int levels, float min_freq,
                      float max_freq, float phase_scale, float mag_threshold,
                      int edge_mode)
{
    if (width <= 0 || height <= 0 || levels < 1) return NULL;
    mm_ref *c = (mm_ref *)calloc(1, sizeof(mm_ref));
    c->W = width;
    c->H = height;
    c->N = next_pow2(width > height ? width : height);  /* .cs:298-302 */
    c->apply = 1;
    c->first = 1;
    mm_ref_set_standard(c, 0, 1, 0.05f, 0.4f, 3.0f, 1.5f, 0.8f);   /* .cs:35-43 */
    c->prev = (float *)calloc((size_t)width * height * 4, sizeof(float));
    mm_ref_set_params(c, levels, min_freq, max_freq, phase_scale, mag_threshold,
                      edge_mode);
    return c;
}

void mm_ref_destroy(mm_ref *c)
{
    if (!c) return;
    free(c->prev);
    free(c->masks);
    free(c);
}

int mm_ref_padded_size(const mm_ref *c) { return c->N; }

void mm_ref_set_params(mm_ref *c, int levels, float min_freq, float max_freq,
                       float phase_scale, float mag_threshold, int edge_mode)
{
    c->levels = levels;
    c->min_freq = min_freq;
    c->max_freq = max_freq;
    c->phase_scale = phase_scale;
    c->tau = mag_threshold;
    c->edge_mode = edge_mode;
    if (!c->masks || c->masks_levels != levels || c->mask_min != min_freq ||
        c->mask_max != max_freq)
        regen_masks(c);
}

void mm_ref_set_apply(mm_ref *c, int apply) { c->apply = apply; }

void mm_ref_set_standard(mm_ref *c, int use_standard, int apply_bandpass, float low,
                         float high, float steep, float sens, float edge)
{
    c->standard = use_standard;
    c->bp_apply = apply_bandpass;
    c->bp_low = low;
    c->bp_high = high;
    c->bp_steep = steep;
    c->bp_sens = sens;
    c->bp_edge = edge;
}
void mm_ref_reset(mm_ref *c) { c->first = 1; }

size_t mm_ref_state_size(const mm_ref *c)
{
    return 16 + sizeof(float) * (size_t)c->W * c->H * 4;
}

void mm_ref_get_state(const mm_ref *c, void *buf)
{
    int32_t hdr[4] = {0x4d4d5246, c->first, c->W, c->H};
    memcpy(buf, hdr, 16);
    memcpy((char *)buf + 16, c->prev, sizeof(float) * (size_t)c->W * c->H * 4);
}

void mm_ref_set_state(mm_ref *c, const void *buf)
{
    int32_t hdr[4];
    memcpy(hdr, buf, 16);
    c->first = hdr[1];
    memcpy(c->prev, (const char *)buf + 16, sizeof(float) * (size_t)c->W * c->H * 4);
}

void mm_ref_set_debug(mm_ref *c, int show_magnitude, int show_phase)
{
    c->show_mag = show_magnitude ? 1 : 0;
    c->show_phase = show_phase ? 1 : 0;
}

/* ConvertComplexMagToTexScaled (FFT.compute:152-161): log10(|z| 10 + 1) / 4 */
static float debug_mag(cplx z) { return log10f(sqrtf(z.x * z.x + z.y * z.y) * 10.0f + 1.0f) / 4.0f; }
/* ConvertComplexPhaseToTex (FFT.compute:164-172): |atan2| / PI_2, PI_2 = 1.57079632679 */
static float debug_phase(cplx z) { return fabsf(atan2f(z.y, z.x)) / 1.57079632679f; }

/* ProcessDebugView (.cs:234-257).  The view textures are RFloat (.cs:321-322):
 * DstTex.rgb writes keep R only and sampling them yields (v, 0, 0, 1).  One
 * view: CropTexture (.cs:386-410, texel-exact).  Both: ShowSplitScreen
 * (.cs:458-487), each N x N texture drawn bilinearly into one half. */
static void debug_view(mm_ref *c, const float *in, float *out)
{
    const int W = c->W, H = c->H, N = c->N;
    const size_t nn = (size_t)N * N;
    float *pad = (float *)malloc(sizeof(float) * nn * 4);
    float *ybuf = (float *)malloc(sizeof(float) * nn);
    cplx *B = (cplx *)malloc(sizeof(cplx) * nn);
    float *mag = (float *)malloc(sizeof(float) * nn);
    float *pha = (float *)malloc(sizeof(float) * nn);
    mm_ref_pad_window(c, in, pad);                            /* :236-237 */
    for (size_t p = 0; p < nn; ++p) ybuf[p] = pad[p * 4];     /* :238 */
    mm_ref_fft_buffer1(N, ybuf, (float *)B);                  /* :239 */
    #pragma omp parallel for schedule(static)
    for (long p = 0; p < (long)nn; ++p) {
        mag[p] = debug_mag(B[p]);
        pha[p] = debug_phase(B[p]);
    }
    const int x0 = (N - W) / 2, y0 = (N - H) / 2;
    #pragma omp parallel for schedule(static)
    for (int Y = 0; Y < H; ++Y)
        for (int X = 0; X < W; ++X) {
            float v;
            if (c->show_mag && c->show_phase) {
                const int right = 2 * X + 1 >= W;
                const float u = (float)(2 * X + 1 - (right ? W : 0)) / (float)W;
                const float vv = (float)(2 * Y + 1) / (float)(2 * H);
                sample_bilinear(right ? pha : mag, N, N, 1, u, vv, c->edge_mode, &v);
            } else {
                v = (c->show_mag ? mag : pha)[(size_t)(y0 + Y) * N + x0 + X];
            }
            float *o = out + ((size_t)Y * W + X) * 4;
            o[0] = v; o[1] = 0.0f; o[2] = 0.0f; o[3] = 1.0f;
        }
    free(pad); free(ybuf); free(B); free(mag); free(pha);
}

/* ProcessFrameWithPyramidDecomposition (.cs:145-206); with c->standard the
 * spectral step is ProcessFrameWithStandardMagnification's (.cs:208-232) */
static void process_pyramid(mm_ref *c, const float *in, float *out, mm_ref_dbg *dbg)
{
    const int W = c->W, H = c->H, N = c->N, L = c->levels;
    const size_t nn = (size_t)N * N;
    float *pad_cur = (float *)malloc(sizeof(float) * nn * 4);
    float *pad_prev = (float *)malloc(sizeof(float) * nn * 4);
    float *ybuf = (float *)malloc(sizeof(float) * nn);
    cplx *Fc = (cplx *)malloc(sizeof(cplx) * nn);
    cplx *Fp = (cplx *)malloc(sizeof(cplx) * nn);
    cplx *acc = (cplx *)malloc(sizeof(cplx) * nn);
    float *ymag = (float *)malloc(sizeof(float) * nn);

    mm_ref_pad_window(c, in, pad_cur);                    /* :147-149 */
    mm_ref_pad_window(c, c->prev, pad_prev);              /* :151-153 */
    for (size_t p = 0; p < nn; ++p) ybuf[p] = pad_cur[p * 4];
    if (dbg && dbg->y_cur) memcpy(dbg->y_cur, ybuf, sizeof(float) * nn);
    mm_ref_fft_centered(N, ybuf, (float *)Fc);             /* :155 */
    for (size_t p = 0; p < nn; ++p) ybuf[p] = pad_prev[p * 4];
    mm_ref_fft_centered(N, ybuf, (float *)Fp);             /* :156 */

    const float S = c->phase_scale, tau = c->tau;
    if (c->standard) {
        /* ProcessPhaseDifferenceWithComputeShader (.cs:489-506) ->
         * ProcessPhaseDifference (PhaseDifferenceComputeShader.compute:124-179) */
        #pragma omp parallel for schedule(static)
        for (int y = 0; y < N; ++y)
            for (int x = 0; x < N; ++x) {
                size_t p = (size_t)y * N + x;
                cplx cur = Fc[p], prv = Fp[p];
                float cm = sqrtf(cur.x * cur.x + cur.y * cur.y);
                float pm = sqrtf(prv.x * prv.x + prv.y * prv.y);
                if (cm < tau || pm < tau) { acc[p] = cur; continue; }      /* :140-146 */
                float d = mm_ref_normalize_phase(atan2f(prv.y, prv.x) - atan2f(cur.y, cur.x));
                float w = bandpass_weight(spatial_frequency(x, y, N), c->bp_apply, c->bp_low,
                                          c->bp_high, c->bp_steep, c->bp_sens, c->bp_edge);
                float md = (d * w) * S;                                      /* :158-165 */
                cplx e = {cosf(md), sinf(md)};
                acc[p] = cmul(cur, e);                                       /* :171-174 */
            }
    } else {
    /* :158-194 — ApplyPyramidFilter x2, phase difference, accumulate (per level,
     * in level order, accumulator initialised to 0: PyramidOperations:131-138) */
    #pragma omp parallel for schedule(static)
    for (size_t p = 0; p < nn; ++p) {
        cplx a = {0.0f, 0.0f};
        for (int i = 0; i < L; ++i) {
            float m = c->masks[nn * i + p];
            cplx cur = {Fc[p].x * m, Fc[p].y * m};         /* :90-108 */
            cplx prv = {Fp[p].x * m, Fp[p].y * m};
            cplx o;
            if (i == 0 || i == L - 1) {                    /* :73-77 */
                o = cur;
            } else {
                float cm = sqrtf(cur.x * cur.x + cur.y * cur.y);
                float pm = sqrtf(prv.x * prv.x + prv.y * prv.y);
                if (cm < tau || pm < tau) {                /* :82-86 */
                    o = cur;
                } else {
                    float cph = atan2f(cur.y, cur.x);
                    float pph = atan2f(prv.y, prv.x);
                    float d = mm_ref_normalize_phase(pph - cph);   /* :92 */
                    float md = d * S;
                    cplx e = {cosf(md), sinf(md)};
                    o = cmul(cur, e);
                }
            }
            a.x += o.x;                                    /* :111-128 */
            a.y += o.y;
        }
        acc[p] = a;
    }
    }
    if (dbg && dbg->F_cur) memcpy(dbg->F_cur, Fc, sizeof(cplx) * nn);
    if (dbg && dbg->F_prev) memcpy(dbg->F_prev, Fp, sizeof(cplx) * nn);
    if (dbg && dbg->A) memcpy(dbg->A, acc, sizeof(cplx) * nn);

    mm_ref_ifft_mag(N, (const float *)acc, ymag);          /* :196 */
    if (dbg && dbg->y_mag) memcpy(dbg->y_mag, ymag, sizeof(float) * nn);
    mm_ref_blur(N, c->edge_mode, ymag);                    /* :197 */
    if (dbg && dbg->y_blur) memcpy(dbg->y_blur, ymag, sizeof(float) * nn);

    /* CombineYIQChannels (:198) + YIQ->RGB blit (:200-204) + CropTexture (:205) */
    #pragma omp parallel for schedule(static)
    for (int j = 0; j < H; ++j)
        for (int i = 0; i < W; ++i) {
            /* crop samples the final texture at texel x0+i, y0+j (bilinear) */
            float tx = (float)((N - W) + 2 * i) / 2.0f;
            float ty = (float)((N - H) + 2 * j) / 2.0f;
            float fx0 = floorf(tx), fy0 = floorf(ty);
            float fx = tx - fx0, fy = ty - fy0;
            int ix = (int)fx0, iy = (int)fy0;
            float res[3] = {0, 0, 0};
            for (int dy = 0; dy < 2; ++dy)
                for (int dx = 0; dx < 2; ++dx) {
                    float w = (dx ? fx : 1.0f - fx) * (dy ? fy : 1.0f - fy);
                    if (w == 0.0f) continue;
                    int X = wrap_index(ix + dx, N, c->edge_mode);
                    int Y = wrap_index(iy + dy, N, c->edge_mode);
                    size_t p = (size_t)Y * N + X;
                    float yiq[3] = {ymag[p], pad_cur[p * 4 + 1], pad_cur[p * 4 + 2]};
                    float rgb[3];
                    mm_ref_yiq_to_rgb(yiq, rgb);
                    res[0] += w * rgb[0]; res[1] += w * rgb[1]; res[2] += w * rgb[2];
                }
            float *o = out + ((size_t)j * W + i) * 4;
            o[0] = res[0]; o[1] = res[1]; o[2] = res[2];
            o[3] = 1.0f;                                   /* combine alpha = 1 */
        }

    free(pad_cur); free(pad_prev); free(ybuf); free(Fc); free(Fp); free(acc); free(ymag);
}

/* OnRenderImage (.cs:101-143) */
void mm_ref_process(mm_ref *c, const float *in, float *out, mm_ref_dbg *dbg)
{
    const size_t px = (size_t)c->W * c->H * 4;
    if (c->first) {                                        /* :111-117 */
        memcpy(c->prev, in, sizeof(float) * px);
        memcpy(out, in, sizeof(float) * px);
        c->first = 0;
        return;
    }
    if (c->show_mag || c->show_phase) {                    /* :119-123 */
        debug_view(c, in, out);
        memcpy(c->prev, in, sizeof(float) * px);
        return;
    }
    if (c->apply) process_pyramid(c, in, out, dbg);        /* :126-136 (both modes) */
    else memcpy(out, in, sizeof(float) * px);              /* :139 */
    memcpy(c->prev, in, sizeof(float) * px);               /* :142 */
}

void mm_ref_process_u8(mm_ref *c, const uint8_t *in, uint8_t *out)
{
    const size_t px = (size_t)c->W * c->H * 4;
    float *fi = (float *)malloc(sizeof(float) * px);
    float *fo = (float *)malloc(sizeof(float) * px);
    if (!fi || !fo) { free(fi); free(fo); return; }
    int passthrough = c->first || (!c->apply && !c->show_mag && !c->show_phase);
    for (size_t i = 0; i < px; ++i) fi[i] = (float)in[i] / 255.0f;
    mm_ref_process(c, fi, fo, NULL);
    if (passthrough) memcpy(out, in, px);                  /* bitwise copy */
    else
        for (size_t i = 0; i < px; ++i)
            out[i] = (uint8_t)(saturatef(fo[i]) * 255.0f + 0.5f);
    free(fi);
    free(fo);
}

/* ------------------------------------------------------------------ */
/* the engine's other frame formats (include/mm.h MM_RGBA16F, MM_RGBA8_SRGB) */
/* ------------------------------------------------------------------ */
/* The reference camera renders HDR (SampleScene.unity:663, m_HDR: 1) in Linear
 * colour space (ProjectSettings.asset:50): OnRenderImage's source (.cs:101) is
 * a linear half-float target that .cs:109 blits into ARGBFloat, i.e. the
 * float pipeline above sees the half values exactly; the destination write
 * rounds to half.  An 8-bit target in Linear colour space is sRGB: sampled as
 * linear light (IEC 61966-2-1 decode), encoded on write. */
float mm_ref_half_to_float(uint16_t h)
{
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    uint32_t b;
    if (e == 0) {                                          /* zero / subnormal: m 2^-24 */
        float v = ldexpf((float)m, -24);
        return s ? -v : v;
    }
    if (e == 31) b = s | 0x7f800000u | (m << 13);          /* inf / NaN */
    else b = s | ((e - 15 + 127) << 23) | (m << 13);
    float f;
    memcpy(&f, &b, 4);
    return f;
}

/* IEEE binary16, round to nearest even (what the destination write does) */
uint16_t mm_ref_float_to_half(float f)
{
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);   /* >= 65520: inf */
    if (ax < 0x38800000u) {                                      /* below 2^-14: subnormal */
        float a;
        memcpy(&a, &ax, 4);
        return (uint16_t)(sign | (uint32_t)rintf(a * 16777216.0f));   /* exact scale, RNE */
    }
    uint32_t h = ((((ax >> 23) - 127 + 15) << 10) | ((ax & 0x7fffffu) >> 13));
    const uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
}

static double srgb_lin(double c)
{
    return c <= 0.04045 ? c / 12.92 : pow((c + 0.055) / 1.055, 2.4);
}

/* dec[b] = lin(b/255); thr[b] = lin((b - 0.5)/255) (b = 1..255), thr[0] = -inf,
 * thr[256] = +inf: double formula rounded to fp32 (tools/gen_srgb.py states
 * the same tables for the kernels) */
void mm_ref_srgb_tables(float *dec, float *thr)
{
    for (int b = 0; b < 256; ++b) dec[b] = (float)srgb_lin(b / 255.0);
    thr[0] = -HUGE_VALF;
    for (int b = 1; b < 256; ++b) thr[b] = (float)srgb_lin((b - 0.5) / 255.0);
    thr[256] = HUGE_VALF;
}

/* the byte whose sRGB interval holds v (largest b with v >= thr[b]) */
static uint8_t srgb_encode(const float *thr, float v)
{
    int lo = 0, hi = 255;                                   /* thr[lo] <= v always */
    while (lo < hi) {
        int mid = (lo + hi + 1) / 2;
        if (v >= thr[mid]) lo = mid;
        else hi = mid - 1;
    }
    return (uint8_t)lo;
}

void mm_ref_process_f16(mm_ref *c, const uint16_t *in, uint16_t *out)
{
    const size_t px = (size_t)c->W * c->H * 4;
    float *fi = (float *)malloc(sizeof(float) * px);
    float *fo = (float *)malloc(sizeof(float) * px);
    if (!fi || !fo) { free(fi); free(fo); return; }
    int passthrough = c->first || (!c->apply && !c->show_mag && !c->show_phase);
    for (size_t i = 0; i < px; ++i) fi[i] = mm_ref_half_to_float(in[i]);
    mm_ref_process(c, fi, fo, NULL);
    if (passthrough) memcpy(out, in, sizeof(uint16_t) * px);   /* bitwise copy */
    else
        for (size_t i = 0; i < px; ++i) out[i] = mm_ref_float_to_half(fo[i]);
    free(fi);
    free(fo);
}

void mm_ref_process_srgb8(mm_ref *c, const uint8_t *in, uint8_t *out)
{
    const size_t px = (size_t)c->W * c->H * 4;
    float dec[256], thr[257];
    mm_ref_srgb_tables(dec, thr);
    float *fi = (float *)malloc(sizeof(float) * px);
    float *fo = (float *)malloc(sizeof(float) * px);
    if (!fi || !fo) { free(fi); free(fo); return; }
    int passthrough = c->first || (!c->apply && !c->show_mag && !c->show_phase);
    for (size_t i = 0; i < px; ++i)                        /* alpha is linear in sRGB targets */
        fi[i] = (i & 3) == 3 ? (float)in[i] / 255.0f : dec[in[i]];
    mm_ref_process(c, fi, fo, NULL);
    if (passthrough) memcpy(out, in, px);                  /* bitwise copy */
    else
        for (size_t i = 0; i < px; ++i)
            out[i] = (i & 3) == 3 ? (uint8_t)(saturatef(fo[i]) * 255.0f + 0.5f)
                                  : srgb_encode(thr, saturatef(fo[i]));
    free(fi);
    free(fo);
}

/* ------------------------------------------------------------------ */
/* synthetic stream                                      */
/* ------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void mm_ref_synth_frame(int W, int H, int t, uint64_t seed, int gray, uint8_t *out)
{
    const double two_pi = 6.283185307179586;
    const double g[3] = {1.0, 0.8, 0.6};
    double d = 0.5 * sin(two_pi * 0.05 * t);
    #pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint8_t *o = out + ((size_t)y * W + x) * 4;
            double sx = sin(two_pi * (x + d) / 37.0), cy = cos(two_pi * y / 53.0);
            for (int ch = 0; ch < 3; ++ch) {
                int cc = gray ? 0 : ch;
                uint64_t h = splitmix64(seed ^ ((uint64_t)((size_t)y * W + x) * 3u + cc));
                double u = (double)(h >> 40) * (1.0 / 16777216.0);
                double v = 0.4 + 0.3 * sx * cy * g[cc] + 0.15 * u;
                v = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
                o[ch] = (uint8_t)floor(v * 255.0 + 0.5);
            }
            o[3] = 255;
        }
}

int mm_ref_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}
