/*
 * mm_ref.h — CPU ORACLE for the MotionMagnificationProcessor pyramid-mode frame
 * operator.  TEST INFRASTRUCTURE ONLY: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker /
 * CPU baseline.  The product path (libmm355.so) never links or calls it.
 *
 * This is a literal fp32 restatement of the reference's per-frame pipeline
 * (Assets/Scripts/MotionMagnificationProcessor.cs:101-206 and the shaders it
 * drives).  Each function in mm_ref.c cites the reference file:line it follows.
 *
 * Parity status: the reference is a Unity C#/HLSL project; neither C#/Unity nor
 * an HLSL compiler exists in this image and the reference ships no tests or
 * golden vectors.  This oracle is therefore "parity
 * unpinned" by reference fixtures; it is cross-checked against an independent
 * float64 numpy restatement (tests/np_twin.py) and analytic known-answer tests.
 */
#ifndef MM_REF_H
#define MM_REF_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { MMREF_EDGE_REPEAT = 0, MMREF_EDGE_CLAMP = 1 };

typedef struct mm_ref mm_ref;

/* Intermediate dumps of one processed frame (all optional; NULL = skip).
 * Canvas arrays are N*N, row-major [y][x], index y*N+x, in the reference's
 * CENTERED spectral layout (FFT.compute:175-189). */
typedef struct {
    float *y_cur;      /* windowed padded luma of the current frame (N*N)        */
    float *F_cur;      /* centered spectrum of y_cur, interleaved re,im (2*N*N)   */
    float *F_prev;     /* centered spectrum of the previous frame (2*N*N)         */
    float *A;          /* accumulated modified spectrum (2*N*N)                   */
    float *y_mag;      /* |IFFT(A)| before the blur (N*N)                         */
    float *y_blur;     /* after the H+V Gaussian (N*N)                            */
} mm_ref_dbg;

mm_ref *mm_ref_create(int width, int height, int levels, float min_freq,
                      float max_freq, float phase_scale, float mag_threshold,
                      int edge_mode);
void    mm_ref_destroy(mm_ref *ctx);
int     mm_ref_padded_size(const mm_ref *ctx);
/* OnValidate analog: new parameters take effect on the next frame. */
void    mm_ref_set_params(mm_ref *ctx, int levels, float min_freq, float max_freq,
                          float phase_scale, float mag_threshold, int edge_mode);
void    mm_ref_set_apply(mm_ref *ctx, int apply_magnification);
/* usePyramidDecomposition = false (.cs:18, :128-135): standard mode with the
 * phase-delta band-pass of PhaseDifferenceComputeShader.compute (.cs:33-43,
 * :489-506).  `edge_enhancement` is the value the component passes:
 * enhanceEdges ? edgeEnhancement : 0 (.cs:504). */
void    mm_ref_set_standard(mm_ref *ctx, int use_standard, int apply_bandpass,
                            float low_cutoff, float high_cutoff, float steepness,
                            float motion_sensitivity, float edge_enhancement);
/* calculate_spatial_frequency + calculate_bandpass_weight
 * (PhaseDifferenceComputeShader.compute:74-122) on the centred N*N grid. */
void    mm_ref_bandpass_weights(int n, int apply_bandpass, float low_cutoff,
                                float high_cutoff, float steepness,
                                float motion_sensitivity, float edge_enhancement,
                                float *out);
void    mm_ref_reset(mm_ref *ctx);                 /* isFirstFrame = true */
/* State = previousSourceTexture (W*H*4 floats) + first-frame flag. */
size_t  mm_ref_state_size(const mm_ref *ctx);
void    mm_ref_get_state(const mm_ref *ctx, void *buf);
void    mm_ref_set_state(mm_ref *ctx, const void *buf);

/* One OnRenderImage call on RGBA float frames (H rows of W pixels). */
void    mm_ref_process(mm_ref *ctx, const float *in_rgba, float *out_rgba,
                       mm_ref_dbg *dbg);
/* Same on RGBA8 frames: in = u8/255 (UNORM), out = round(saturate(v)*255). */
void    mm_ref_process_u8(mm_ref *ctx, const uint8_t *in_rgba, uint8_t *out_rgba);

/* Linear half frames (MM_RGBA16F, IEEE binary16 bits): in decoded exactly,
 * out rounded to nearest even; first frame bitwise.                         */
void    mm_ref_process_f16(mm_ref *ctx, const uint16_t *in_rgba, uint16_t *out_rgba);
/* 8-bit sRGB frames (MM_RGBA8_SRGB): in = dec[byte] (alpha byte/255), out =
 * the byte whose sRGB interval holds saturate(v) (alpha 255).              */
void    mm_ref_process_srgb8(mm_ref *ctx, const uint8_t *in_rgba, uint8_t *out_rgba);
void    mm_ref_srgb_tables(float *dec256, float *thr257);
float   mm_ref_half_to_float(uint16_t h);
uint16_t mm_ref_float_to_half(float f);

/* showMagnitude / showPhase (.cs:13-14): ProcessDebugView (.cs:234-257)
 * replaces the magnified output while either is set (state still follows
 * the input, .cs:122).                                                      */
void    mm_ref_set_debug(mm_ref *ctx, int show_magnitude, int show_phase);

/* ---- stage-level entry points for known-answer tests ---- */
/* PerformFFT (.cs:508-553): centered forward 2D FFT of a real N*N image.   */
void    mm_ref_fft_centered(int n, const float *y, float *out_cplx);
/* complexBuffer1 after PerformFFT: what ProcessDebugView reads (.cs:239-255);
 * the state after the penultimate column stage (see mm_ref.c).              */
void    mm_ref_fft_buffer1(int n, const float *y, float *out_cplx);
/* PerformIFFT (.cs:563-620): |ifft| of a centered N*N spectrum.            */
void    mm_ref_ifft_mag(int n, const float *in_cplx, float *out_mag);
/* GeneratePyramidFilters (PyramidOperations.compute:25-87) for one level.   */
void    mm_ref_mask(int n, int levels, int index, float min_freq, float max_freq,
                    float *out);
/* normalize_phase (PyramidPhaseDifference.compute:47-54).                   */
float   mm_ref_normalize_phase(float phase);
/* RGBToYIQ.shader:46-61 / YIQToRGB.shader:51-79 on one pixel.              */
void    mm_ref_rgb_to_yiq(const float *rgb, float *yiq);
void    mm_ref_yiq_to_rgb(const float *yiq, float *rgb);
/* Stretch(RGB->YIQ) + PadTexture + window for one frame: out N*N*4.        */
void    mm_ref_pad_window(mm_ref *ctx, const float *in_rgba, float *out_canvas);
/* ApplyAntiAliasing (.cs:423-433): H then V blur of an N*N image in place.  */
void    mm_ref_blur(int n, int edge_mode, float *img);

/* Synthetic stream frame; RGBA8, gray != 0 gives R=G=B=v0. */
void    mm_ref_synth_frame(int width, int height, int t, uint64_t seed, int gray,
                           uint8_t *out_rgba);
int     mm_ref_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
