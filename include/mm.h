/*
 * mm.h — C-ABI of the MI355X-native MotionMagnificationProcessor frame operator.
 *
 * Drop-in boundary for the reference Unity component
 *   [RequireComponent(typeof(Camera))] public class MotionMagnificationProcessor
 *   (Assets/Scripts/MotionMagnificationProcessor.cs:4-5)
 * whose per-frame entry point is the image-effect callback
 *   void OnRenderImage(RenderTexture source, RenderTexture destination)  (.cs:101)
 * An RGBA frame goes in, the PhaseScale-amplified frame comes out.
 *
 * Conventions
 *   - Every function returns MM_OK (0) or a negative MM_ERR_* code; nothing
 *     throws or aborts across the ABI.  mm_strerror() names a code.
 *   - Frames are caller-owned, row-major, H rows of W RGBA pixels, tightly
 *     packed (pitch = W * bytes-per-pixel, mm_frame_bytes).  RGBA8 is UNORM
 *     (v = byte/255); RGBA32F and RGBA16F are linear float; RGBA8_SRGB is an
 *     8-bit sRGB target as Unity's Linear colour space sees it (decoded to
 *     linear light on read, encoded on write).  The handle owns all device
 *     scratch and the one-frame temporal state.
 *   - A handle is not thread-safe: one handle per video stream, calls in frame
 *     order (Unity calls OnRenderImage serially on its render thread).
 *   - The first frame after mm_create/mm_reset is passed through bitwise
 *     (alpha included) and becomes the temporal state (.cs:111-117); after
 *     that output alpha is 1 (CombineYIQChannels.shader:56).
 *   - Geometry: the padded square is N = nextpow2(max(W, H)) (.cs:298-302);
 *     this build covers 16 <= N <= 8192, i.e. 9 <= max(W, H) <= 8192 (other
 *     sizes: MM_ERR_UNSUPPORTED from mm_create); MM_MODE_STEERABLE stops at
 *     N = 4096.  Odd W or H are supported in every mode (and the debug
 *     views).  The fused K3+K4 kernel runs for
 *     even sizes with W % 8 == 0 and margins N - W >= 8, N - H >= 4; every
 *     other geometry takes the unfused pair (same results).
 *   - Every entry point that takes a handle runs on the handle's device and
 *     restores the caller's current HIP device before it returns.
 */
#ifndef MM_H
#define MM_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MM_ABI_VERSION 10  /* 8: the state is G_{t-1} (row spectra), see mm_state_size;
                              9: handle-scoped teardown and batch changes (mm_destroy,
                                 mm_set_batch), no device-wide synchronisation;
                             10: MM_RGBA16F and MM_RGBA8_SRGB frames, mm_frame_bytes */

/* error codes */
#define MM_OK               0
#define MM_ERR_INVALID     -1  /* bad argument / handle */
#define MM_ERR_UNSUPPORTED -2  /* geometry or mode not supported by this build */
#define MM_ERR_HIP         -3  /* HIP runtime error (launch, copy, ...) */
#define MM_ERR_NO_DEVICE   -4  /* no usable gfx950 device */
#define MM_ERR_OOM         -5  /* device allocation failed */
#define MM_ERR_NO_STATE    -6  /* mm_get_state before any frame was seen */

/* frame formats (every entry point that takes frames takes each of them) */
#define MM_RGBA8   0       /* 4 B/px, UNORM: v = byte / 255; out round(saturate(v) * 255) */
#define MM_RGBA32F 1       /* 16 B/px, linear float                                       */
/* The frames the reference actually receives (since ABI 10): its camera
 * renders HDR (Assets/Scenes/SampleScene.unity:663, m_HDR: 1) in Linear colour
 * space (ProjectSettings/ProjectSettings.asset:50, m_ActiveColorSpace: 1), so
 * OnRenderImage's source (.cs:101) is a linear half-float target (values may
 * exceed 1) that .cs:109 blits into ARGBFloat; an LDR camera's 8-bit target is
 * sRGB, sampled as linear light and encoded on write. */
#define MM_RGBA16F    2    /* 8 B/px, linear IEEE half; values above 1 pass until the
                              reference's saturate (YIQToRGB); out rounded to nearest
                              even half, alpha 1.0                                   */
#define MM_RGBA8_SRGB 3    /* 4 B/px, sRGB-encoded bytes: in = the exact IEC 61966-2-1
                              decode of each byte (a 256-entry fp32 table), the whole
                              pipeline in linear light, out = the byte whose sRGB
                              interval holds saturate(v) (halfway points in linear
                              light; tools/gen_srgb.py); alpha byte / 255, out 255    */

/* mm_params.mode */
#define MM_MODE_PYRAMID   0   /* usePyramidDecomposition = true (.cs:18, :128-131) */
#define MM_MODE_STANDARD  1   /* usePyramidDecomposition = false (.cs:132-135, :208-232) */
#define MM_MODE_STEERABLE 2  /* extension f2: oriented local-phase subbands + temporal filter */
#define MM_FILTER_DIFF 0      /* steerable: the reference's 2-tap phase difference per coefficient */
#define MM_FILTER_IIR  1      /* steerable: band-pass IIR of the unwrapped local phase */
/* mm_params.edge_mode: sampler wrap of the engine resamples and the blur
 * (unpinned by the reference) */
#define MM_EDGE_REPEAT 0
#define MM_EDGE_CLAMP  1

/* mm_process flags */
#define MM_FRAMES_ON_DEVICE 1  /* in/out are device pointers (else host memory) */

typedef struct mm_handle mm_handle;

/* Inspector fields of the reference component (.cs:12-43). */
typedef struct {
    int   levels;              /* pyramidLevels            .cs:19  (1..16)      */
    float min_freq;            /* minFrequency             .cs:20               */
    float max_freq;            /* maxFrequency             .cs:21               */
    float phase_scale;         /* phaseScale (PhaseScale)  .cs:29               */
    float magnitude_threshold; /* magnitudeThreshold=0.01  .cs:30               */
    int   orientations;        /* 1 (reference semantics); 4, 6, 8 with MM_MODE_STEERABLE */
    int   mode;                /* MM_MODE_PYRAMID | MM_MODE_STANDARD | MM_MODE_STEERABLE */
    int   edge_mode;           /* MM_EDGE_REPEAT | MM_EDGE_CLAMP                */
    int   apply_magnification; /* applyMotionMagnification .cs:12 (0: passthrough) */
    /* standard mode's phase-delta band-pass (PhaseDifferenceComputeShader.compute:88-122) */
    int   apply_bandpass_filter;  /* applyBandpassFilter  .cs:35 */
    float low_frequency_cutoff;   /* lowFrequencyCutoff   .cs:36 */
    float high_frequency_cutoff;  /* highFrequencyCutoff  .cs:37 */
    float filter_steepness;       /* filterSteepness      .cs:38 */
    float motion_sensitivity;     /* motionSensitivity    .cs:41 */
    int   enhance_edges;          /* enhanceEdges         .cs:42 */
    float edge_enhancement;       /* edgeEnhancement      .cs:43 (used iff enhance_edges, .cs:504) */
    /* debug views (ProcessDebugView .cs:234-257): while either is set the output
     * is the |spectrum| (log-scaled) and/or |phase| view, R channel only (RFloat
     * textures), cropped (one view) or split screen (both); the state still
     * follows the input (.cs:122).  Since ABI 3. */
    int   show_magnitude;         /* showMagnitude        .cs:13 */
    int   show_phase;             /* showPhase            .cs:14 */
    /* MM_MODE_STEERABLE (extension; spec oracle/steerable_ref.py;
     * no reference counterpart): `orientations` in {4, 6, 8} oriented cos^4
     * subbands per middle level, local phase filtered per coefficient by
     * `temporal_filter` (MM_FILTER_DIFF | MM_FILTER_IIR with first-order
     * low-pass coefficients iir_low < iir_high in (0, 1]), amplified by
     * phase_scale; magnitude_threshold gates |subband| < tau.  Since ABI 4. */
    int   temporal_filter;
    float iir_low;
    float iir_high;
} mm_params;

/* Reference defaults (.cs:12-43): levels 5, 0.05/0.45, phaseScale 10, threshold
 * 0.01, pyramid mode; band-pass on, 0.05/0.4, steepness 3, sensitivity 1.5,
 * edges on at 0.8. */
int mm_params_default(mm_params *p);

/* Start()/InitializeProcessor (.cs:90-94, :289-342): geometry frozen here. */
int mm_create(int width, int height, const mm_params *p, int hip_device,
              mm_handle **out);

/* OnValidate (.cs:78-88): new parameters apply from the next frame.  Does not
 * synchronise the device: a change of edge_mode (which rewrites the resample
 * tables) waits only for this handle's own latest work.
 * edge_mode mid-stream: the state is the previous frame's RESAMPLED rows
 * (G_{t-1}, built with the tables of the call that processed that frame), so
 * the first frame after an edge_mode change pairs an old-edge G_{t-1} with a
 * new-edge G_t; from the frame after it both use the new tables.  The
 * reference re-resamples previousSourceTexture with the current sampler every
 * frame (.cs:151); its sampler wrap is an unpinned engine choice (SURVEY.md
 * §8c).  A caller that needs the reference's behaviour exactly calls
 * mm_reset with the change (that frame then passes through). */
int mm_set_params(mm_handle *h, const mm_params *p);
int mm_get_params(const mm_handle *h, mm_params *p);

/* Padded FFT size N (.cs:300-302). */
int mm_padded_size(const mm_handle *h, int *n);

/* Bytes of one W x H frame of `format` (MM_ERR_INVALID for an unknown format
 * or size).  Since ABI 10. */
int mm_frame_bytes(int width, int height, int format, size_t *bytes);

/* OnRenderImage (.cs:101-143): one frame in, one frame out.
 * flags & MM_FRAMES_ON_DEVICE: in/out are device pointers and the call is
 * asynchronous on `hip_stream` (NULL = the default stream, as everywhere in
 * HIP; mm_stream(h) is a non-blocking stream owned by the handle); otherwise
 * in/out are host pointers and the call returns when out is written.
 * Every device-pointer entry point below orders its work on `hip_stream` the
 * same way: a caller that produced the input on another stream synchronises.
 * A call on a different stream than the handle's previous call first makes
 * that stream wait for the previous call's work (since ABI 9: calls of one
 * handle never overlap, whatever streams they use). */
int mm_process(mm_handle *h, const void *in, void *out, int format, int flags,
               void *hip_stream);

/* Consecutive frames of one stream in a single call (device pointers;
 * frame k at in + k*W*H*bpp).  Equivalent, frame for frame, to `count`
 * mm_process calls; batches the launches. Asynchronous on hip_stream. */
int mm_process_stream(mm_handle *h, const void *in, void *out, int count,
                      int format, void *hip_stream);

/* isFirstFrame = true (.cs:75): the next frame is passed through.  The same
 * happens after a MM_MODE_STEERABLE mm_set_state followed by a switch to
 * another mode (that state holds local phases, not G_{t-1}). */
int mm_reset(mm_handle *h);

/* The temporal state carried between frames (previousSourceTexture, .cs:142):
 * the previous input frame's row half-spectra G_{t-1} (K1's output: complex
 * fp32 [N/2 + 1][H rounded up to even], rows of the windowed luma after the
 * stretch+pad resample; 8.86 MB at 1920x1080), from which the next call
 * recomputes the previous frame's 2D spectrum.  `dev_buf` is device memory of
 * mm_state_size() bytes.  Ordered on hip_stream (NULL = default stream).
 * MM_MODE_STEERABLE: the per-coefficient local phases (one float plane per
 * band; MM_FILTER_IIR adds the two filter planes), so the size follows the
 * mode, levels, orientations and filter of the current parameters. */
int mm_state_size(const mm_handle *h, size_t *bytes);
int mm_get_state(mm_handle *h, void *dev_buf, size_t bytes, void *hip_stream);
int mm_set_state(mm_handle *h, const void *dev_buf, size_t bytes, void *hip_stream);
/* Compute the state that frame `in` would leave behind (its row spectra) into
 * dev_buf without touching the handle's own state (used by the multi-GPU ring
 * to hand the chunk-boundary state to the next rank). */
int mm_compute_state(mm_handle *h, const void *in_dev, int format, void *dev_buf,
                     size_t bytes, void *hip_stream);

/* The handle's HIP stream (hipStream_t). */
void *mm_stream(mm_handle *h);

/* Frames per internal batch of mm_process_stream: the launches of one batch
 * cover `frames` frames, and the column kernel keeps the previous spectrum on
 * chip across them (each launch first re-transforms the state G_{t-1}).
 * Larger batches amortise that and the launch gaps; the hand-off buffers take
 * about 17.8 MB per 1080p frame (4x at 2160p).  Default: min(64, 2 GiB of
 * buffers).  Results do not depend on the batch size.  MM_MODE_STEERABLE
 * holds, besides, the band rows of one column chunk independent of the batch
 * (O = 8: 231 MB per 1080p frame x 8 frames, 1.2 GB per 2160p frame x 2; the
 * MM_SB_CF environment variable, 2..16, sets the 1080p chunk) and the state
 * planes (100 MB DIFF / 300 MB IIR at 1080p).  Reallocates: the
 * old buffers retire behind this handle's latest work and the call waits for
 * that work only (not for the device, since ABI 9); call between frames.
 * Failure-atomic: on MM_ERR_OOM the handle keeps its previous batch size,
 * buffers and state.  Since ABI 5. */
int mm_set_batch(mm_handle *h, int frames);
int mm_get_batch(const mm_handle *h, int *frames);

/* Zero-copy frames (f4): device memory owned by another API — an engine's
 * render target exported as an opaque POSIX fd (Vulkan VK_KHR_external_memory_fd,
 * or a HIP VMM allocation via hipMemExportToShareableHandle) — imported into the
 * handle's device (hipImportExternalMemory) and mapped as a device pointer that
 * mm_process / mm_process_stream take with MM_FRAMES_ON_DEVICE, in place: no
 * staging copy, no PCIe transfer (the reference's OnRenderImage works on the
 * engine's RenderTextures, .cs:101).  `bytes` = the exported allocation's
 * size, `offset` = where the frames start in it.  On success the fd belongs to
 * the import (do not close it).  Release before the exporter frees the memory.
 * Since ABI 6. */
typedef struct mm_ext_frames mm_ext_frames;
int mm_import_frames(mm_handle *h, int fd, size_t bytes, size_t offset, mm_ext_frames **out);
void *mm_ext_frames_ptr(const mm_ext_frames *x);
int mm_release_frames(mm_ext_frames *x);

/* OnDestroy/ReleaseResources (.cs:96-99, :344-356).  Returns the handle's
 * device memory to the device's stream-ordered pool behind the handle's own
 * latest work (every call that queued work records an event) and waits for
 * that work only, never for the whole device: other handles and streams on
 * the GPU keep running.  Work the CALLER queued on its streams that reads
 * handle-owned memory (none through this API: frames are caller-owned) is the
 * caller's to finish first.  Since ABI 9.
 * Hardware-queue caveat (this and mm_set_params / mm_set_batch): the HIP
 * runtime maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4)
 * round-robin, and streams that share a hardware queue execute in one order.
 * With more live streams than queues, this handle's stream can sit behind
 * another stream's blocked work on the same queue, and the wait for "this
 * handle's own work" then also waits for that work.  The entry point itself
 * never synchronises the device; a process that must not couple streams that
 * way raises GPU_MAX_HW_QUEUES (tests/test_handle.py runs its no-stall tests
 * with 16). */
void mm_destroy(mm_handle *h);

const char *mm_strerror(int code);
int mm_abi_version(void);

/* ---- utilities (not on the reference surface) ---- */
/* Per-kernel device time, measured with HIP events recorded on the launch
 * stream around every launch between mm_profile_begin and mm_profile_end.
 * Kernel ids: */
#define MM_K_ROWS_FWD 0   /* K1: resample + window + row real FFT      */
#define MM_K_COLS     1   /* K2: column FFT + pyramid phase op + IFFT  */
#define MM_K_ROWS_INV 2   /* K3: row C2R IFFT + |z| + horizontal blur    */
#define MM_K_COMPOSE  3   /* K4: vertical blur + YIQ recombine + RGB + crop */
#define MM_K_ROWS_INV_COMPOSE 4   /* K3 + K4 fused (even sizes, N - H >= 4)  */
#define MM_K_COUNT    5
int mm_profile_begin(mm_handle *h);
/* Waits for the recorded events; ms[k] = summed device ms, launches[k],
 * frames[k] = frames processed by kernel k, k < MM_K_COUNT (arrays of
 * MM_K_COUNT entries; any pointer may be NULL). */
int mm_profile_end(mm_handle *h, double *ms, int *launches, int *frames);

/* Synthetic stream frames generated on the device:
 * frames t0..t0+count-1 into dev_out (RGBA8). */
int mm_synth_frames(void *dev_out, int width, int height, int t0, int count,
                    uint64_t seed, int gray, void *hip_stream);

/* Host-side geometry tables (no GPU needed), exposed for tests:
 * per image column (row) the 4 source indices and 4 weights of the composite
 * stretch+pad bilinear resample, including the Hann window factor. */
int mm_resample_table(int width, int height, int axis, int edge_mode,
                      int32_t *idx4, float *w4);

#ifdef __cplusplus
}
#endif
#endif
