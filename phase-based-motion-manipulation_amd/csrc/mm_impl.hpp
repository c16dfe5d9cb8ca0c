// mm_impl.hpp — the handle and the per-padded-size host drivers of the C-ABI
// (include/mm.h), shared by the translation units: mm_api.hip (the entry
// points and the size dispatch) and mm_n<L>.hip (one per log2 of the padded
// size N: the kernels of that size are instantiated there, so that a build
// compiles the sizes in parallel).
#pragma once
#if (defined(MM_K2_STAMPS) || defined(MM_K34_STAMPS)) && !defined(MM_ONLY_LOG2N)
#error "stamp builds are one-size builds: compile csrc/mm_api.hip alone with -DMM_ONLY_LOG2N=<log2 N>"
#endif
// C-ABI implementation (include/mm.h) of the MI355X-native
// MotionMagnificationProcessor frame operator.
//
// Reference surface (Assets/Scripts/MotionMagnificationProcessor.cs):
//   Start/InitializeProcessor :90-94,:289-342 -> mm_create
//   OnValidate                :78-88          -> mm_set_params
//   OnRenderImage             :101-143        -> mm_process / mm_process_stream
//   OnDestroy/ReleaseResources:96-99,:344-356 -> mm_destroy
// There is no CPU fallback: every frame is computed by the HIP kernels of
// mm_kernels.hpp; without a gfx950 device mm_create fails with MM_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/mm.h"
#include "mm_steer.hpp"

using namespace mm;

#define HIPCHK(x)                                                             \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            if (getenv("MM_DEBUG"))                                           \
                fprintf(stderr, "mm355: %s failed: %s (%s:%d)\n", #x,         \
                        hipGetErrorString(e_), __FILE__, __LINE__);           \
            return MM_ERR_HIP;                                                \
        }                                                                     \
    } while (0)

struct mm_handle {
    int W, H, N, log2n, device;
    mm_params p;
    hipStream_t stream;
    Geo geo;
    Spec spec;
    Blur5 blur;
    Tap4 *d_col, *d_row;
    float4 *d_col3, *d_row3;    // the same taps merged onto offsets -1, 0, +1
    c2 *d_tw;
    float2 *d_ktab;             // K2's per-bin tables of every column (k_k2_table)
    float *d_kmsum;             // ... and the bins' whole mask sums (pyramid tables)
    int ktab_mode;              // table kind d_ktab holds (-1: stale, refilled before the next K2)
    c2 *d_tw_half;              // W_{N/2} table (debug views, lazily)
    float *d_dbg;               // debug view textures [dbg_frames][mag, phase][N][N] (lazily)
    // MM_MODE_STEERABLE (lazily, for the current levels/orientations):
    c2 *d_Fb;                   // per batch frame half spectrum [fb_frames][N/2+1][N] (lazily)
    c2 *d_T;                    // band rows [nb+1][t_rows(Hn)][N] (row groups, MM_SB_RROWS; k_sb_cols -> k_sb_rows)
    float *d_sst;               // temporal-filter state: phi, u_h, u_l planes [nb][Hn][W+4]
    int steer_nb;               // bands the steerable buffers were sized for (-1: none)
    int steer_planes;           // state planes allocated (1: DIFF, 3: IIR)
    int sb_nf;                  // frames per k_sb_rows launch (MM_SB_NF; 2: pairs)
    int sb_cf;                  // frames per k_sb_cols launch at N <= 2048 (MM_SB_CF)
    int sb_cf4k;                // frames per column chunk at N = 4096 (MM_SB_CF4K; launches stay per frame)
    int sb_rg;                  // k_sb_rows: a chunk's frame groups in one launch (MM_SB_RG)
    bool sb_stg_own;            // k_sb_cols stages in its own LDS area where it fits (MM_SB_STG)
    bool steer_valid;           // d_sst holds the state after the previous frame
    // G: chunk + 1 slots of K1's row spectra.  Slot gs holds G_{t-1}, the row
    // spectra of the previous input frame: the temporal state
    // (previousSourceTexture, .cs:142), valid while has_state.  A batch's
    // frames go to slots that avoid gs (place_batch).
    c2 *d_G, *d_Q;
    float *d_Yh;                // unfused K3 -> K4 / steerable rows (lazily, yh_frames)
    size_t g_stride, q_stride, yh_stride;  // elements per frame
    int chunk;                  // frames per K1/K2/K3 batch (mm_set_batch)
    int gs;                     // G slot of the state
    int yh_frames, fb_frames, dbg_frames;  // frames the lazy buffers hold
    hipEvent_t last_ev;         // recorded after this handle's latest work (mm_set_params)
    hipEvent_t retire_ev;       // orders a buffer's return to the pool behind a call's stream
    bool last_ev_set;
    hipStream_t last_s;         // the stream last_ev was recorded on
    bool k2_tab;                // pyramid masks from the per-bin LDS table (<= 2 bands/bin)
    int k2_sp;                  // ... and the phase factor as z^S, |S| == k2_sp (k_cols SP; 0: atan2)
    bool k2_tab2;               // ... with overlapping middle bands (MM_K2_PYR_TAB2)
    bool k2_stg_ded;            // k_cols stages Q in its own LDS area where it fits (MM_K2_STGD=1)
    uint8_t *d_stage_in, *d_stage_out;
    size_t stage_bytes;
    bool has_state;
    bool g_valid;               // the G slot gs holds G_{t-1} (K1 or a non-steerable mm_set_state
                                // wrote it; a steerable mm_set_state sets only the local phases)
    int k2_tail_pct;            // share of a batch's frames of k_cols's packed block run by k_cols_tail
    bool k2_pk_all;             // ... all of them (batches >= 24 frames): block 0 leaves k_cols
    int k2_tail2_pct;           // share of the second-half blocks' frames run by k_cols's tail blocks
    int k34_rows;               // output rows per k_rows_inv_compose strip (0: K3 + K4 unfused;
                                // -1: by the launch's frame count, k34_strip_rows)
    int k34_oneshot;            // short launches: k_rows_inv_compose4 when its strips fit one
                                // workgroup round (MM_K34_ONESHOT: 0 never: K3 -> K4, 2 always)
    int num_cu;                 // compute units of the device
    // mm_profile_begin/end: HIP events around each launch on its stream
    struct ProfRec { hipEvent_t a, b; int kernel, frames; };
    bool prof;
    std::vector<ProfRec> prof_recs;
};

// Makes the handle's device current for the scope of an entry point and gives
// the caller's current device back on the way out (a multi-GPU host or an
// engine plugin keeps its own device selection across mm_* calls).
struct DeviceScope {
    int prev = -1;
    hipError_t err;
    explicit DeviceScope(int dev)
    {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
        else if (err == hipSuccess) prev = -1;   // already current: nothing to restore
    }
    ~DeviceScope()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
#define DEVICE_SCOPE(h)                                  \
    DeviceScope dev_scope_((h)->device);                 \
    if (dev_scope_.err != hipSuccess) return MM_ERR_HIP

// Device memory of a handle comes from the device's stream-ordered pool
// (hipMallocAsync on the handle's own stream) and goes back with hipFreeAsync
// ordered behind the handle's own work: hipFree would synchronise the whole
// device (hip_runtime_api.h: "implicit hipDeviceSynchronize"), stalling every
// other handle and stream on the GPU at a teardown or a batch change
// (VERDICT r3 #6).  An allocation is made usable on every stream by waiting
// for the handle's stream (nothing else is queued there).
// A failed allocation leaves no error behind: the next launch check
// (hipGetLastError) would otherwise report it as that launch's failure (an
// OOM from mm_set_batch must leave the handle usable).
template <class T>
static hipError_t h_alloc(mm_handle *h, T **p, size_t bytes)
{
    hipError_t e = hipMallocAsync(reinterpret_cast<void **>(p), bytes, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        if (*p && e != hipErrorOutOfMemory) (void)hipFreeAsync(*p, h->stream);
        *p = nullptr;
        (void)hipGetLastError();
    }
    return e;
}

// Returns a buffer to the pool once this handle's work that may read it is
// done: the handle's last call (last_ev) and, when given, what the current
// call has queued on its stream s so far.  No host wait.
static void h_retire(mm_handle *h, void *p, hipStream_t s = nullptr, bool have_s = false)
{
    if (!p) return;
    if (h->last_ev_set) (void)hipStreamWaitEvent(h->stream, h->last_ev, 0);
    if (have_s && s != h->stream && hipEventRecord(h->retire_ev, s) == hipSuccess)
        (void)hipStreamWaitEvent(h->stream, h->retire_ev, 0);
    (void)hipFreeAsync(p, h->stream);
}

// Marks the end of this handle's latest work on stream s (mm_set_params waits
// for it before rewriting the tables that work may read).
static int note_work(mm_handle *h, hipStream_t s)
{
    HIPCHK(hipEventRecord(h->last_ev, s));
    h->last_ev_set = true;
    h->last_s = s;
    return MM_OK;
}

// A call on another stream than the handle's previous call first waits for
// that call's work (last_ev), so last_ev always covers every earlier call and
// the buffers h_retire returns behind it are not still read on the old stream.
// Same stream (the one-frame drop-in pattern): nothing to do.
static int order_after_last(mm_handle *h, hipStream_t s)
{
    if (h->last_ev_set && s != h->last_s) HIPCHK(hipStreamWaitEvent(s, h->last_ev, 0));
    return MM_OK;
}

// Brackets one kernel launch with events when profiling is on.
struct ProfScope {
    mm_handle *h;
    hipStream_t s;
    mm_handle::ProfRec r;
    bool on;
    ProfScope(mm_handle *h_, hipStream_t s_, int kernel, int frames) : h(h_), s(s_), on(h_->prof)
    {
        if (!on) return;
        r.kernel = kernel;
        r.frames = frames;
        // timing only: a device-scope release (no system-scope cache write-back
        // between the kernels being timed)
        on = hipEventCreateWithFlags(&r.a, hipEventDisableSystemFence) == hipSuccess &&
             hipEventCreateWithFlags(&r.b, hipEventDisableSystemFence) == hipSuccess &&
             hipEventRecord(r.a, s) == hipSuccess;
    }
    ~ProfScope()
    {
        if (on && hipEventRecord(r.b, s) == hipSuccess) h->prof_recs.push_back(r);
    }
};

// Bytes per pixel of a frame format (include/mm.h); the kernels' FMT template
// argument is the format code itself (Pix<FMT>, mm_kernels.hpp).
static inline size_t fmt_bpp(int fmt)
{
    return fmt == MM_RGBA32F ? 16 : fmt == MM_RGBA16F ? 8 : 4;
}
static inline bool fmt_valid(int fmt)
{
    return fmt == MM_RGBA8 || fmt == MM_RGBA32F || fmt == MM_RGBA16F || fmt == MM_RGBA8_SRGB;
}
// Runs the statement with the compile-time format FMT_ of the runtime `fmt`.
#define MM_FMT_SWITCH(fmt, ...)                                                \
    switch (fmt) {                                                             \
    case MM_RGBA8: { constexpr int FMT_ = MM_RGBA8; __VA_ARGS__; } break;      \
    case MM_RGBA32F: { constexpr int FMT_ = MM_RGBA32F; __VA_ARGS__; } break;  \
    case MM_RGBA16F: { constexpr int FMT_ = MM_RGBA16F; __VA_ARGS__; } break;  \
    default: { constexpr int FMT_ = MM_RGBA8_SRGB; __VA_ARGS__; } break;       \
    }

// ------------------------------------------------------------------------
// host tables
// ------------------------------------------------------------------------
static int wrap_host(int i, int n, int edge)
{
    if (edge) return i < 0 ? 0 : (i >= n ? n - 1 : i);
    int r = i % n;
    return r < 0 ? r + n : r;
}

static int next_pow2(int v)
{
    int n = 1;
    while (n < v) n <<= 1;
    return n;
}

// Composite of the stretch blit (src S texels -> N, RGBToYIQ pass, .cs:147) and
// the PadTexture quad resample (N -> S texels placed at (N-S)/2, .cs:358-381),
// both bilinear at texel t = u*size - 0.5, times the Hann window of the canvas
// position (WindowingFunction.shader:47-70).  fp32 formulas as the oracle.
static void build_tab(int S, int N, int edge, std::vector<Tap4> &tab)
{
    tab.resize(S);
    const int off = (N - S) / 2;
    for (int i = 0; i < S; ++i) {
        const int X = off + i;
        const float u = (float)(2 * X + 1 - (N - S)) / (float)(2 * S);
        const float tp = u * (float)N - 0.5f;
        const float af = floorf(tp);
        const int a = (int)af;
        const float gfr = tp - af;
        Tap4 e;
        for (int k = 0; k < 2; ++k) {
            const int aa = wrap_host(a + k, N, edge);
            const float us = ((float)aa + 0.5f) / (float)N;
            const float ts = us * (float)S - 0.5f;
            const float bf = floorf(ts);
            const int b = (int)bf;
            const float fr = ts - bf;
            const float wk = k ? gfr : 1.0f - gfr;
            // source indices stay UNWRAPPED (always in {i-1, i, i+1}); kernels wrap
            // them with the edge mode on use (wrap_near)
            e.idx[2 * k] = b;
            e.w[2 * k] = wk * (1.0f - fr);
            e.idx[2 * k + 1] = b + 1;
            e.w[2 * k + 1] = wk * fr;
        }
        const float wu = ((float)X + 0.5f) / (float)N;
        const float hann = 0.5f * (1.0f - cosf(2.0f * kPi * wu));
        for (int m = 0; m < 4; ++m) {
            e.w[m] *= hann;
            if (e.w[m] == 0.0f) e.idx[m] = i;   // zero taps (e.g. W == N) stay local
        }
        tab[i] = e;
    }
}

static void build_spec(const mm_params &p, int N, Spec &sp)
{
    memset(&sp, 0, sizeof(sp));
    sp.mode = p.mode;
    // standard mode: ProcessPhaseDifferenceWithComputeShader uniforms (.cs:489-506)
    sp.bp_apply = p.apply_bandpass_filter ? 1 : 0;
    sp.bp_low = p.low_frequency_cutoff;
    sp.bp_high = p.high_frequency_cutoff;
    sp.bp_steep = p.filter_steepness;
    sp.bp_sens = p.motion_sensitivity;
    sp.bp_edge = p.enhance_edges ? p.edge_enhancement : 0.0f;      // .cs:504
    sp.bp_inv_low = 1.0f / fmaxf(p.low_frequency_cutoff, 0.001f);
    sp.bp_inv_1mhigh = 1.0f / fmaxf(1.0f - p.high_frequency_cutoff, 0.001f);
    sp.bp_inv_band = 1.0f / (p.high_frequency_cutoff - p.low_frequency_cutoff);
    sp.L = p.levels;
    sp.minF = p.min_freq;
    sp.maxF = p.max_freq;
    sp.S = p.phase_scale;
    sp.tau2 = p.magnitude_threshold * p.magnitude_threshold;
    sp.inv_nn = 1.0f / ((float)N * (float)N);
    sp.S_rev = (float)((double)p.phase_scale / (2.0 * 3.14159265358979323846));
    // integer phase scale (the reference default 10, BASELINE's 25): the power form
    const float aS = fabsf(p.phase_scale);
    sp.S_pow = (aS == floorf(aS) && aS <= 4096.0f) ? (int)aS : -1;
    sp.S_sgn = p.phase_scale < 0.0f ? -1.0f : 1.0f;
    sp.tau2_nn = sp.tau2 * sp.inv_nn * sp.inv_nn;   // exact: inv_nn is a power of two
    sp.hp_lo = p.max_freq * 0.8f;             // PyramidOperations.compute:36-41
    sp.hp_inv = 1.0f / (p.max_freq * 0.2f);
    sp.lp_hi = p.min_freq * 1.2f;             // PyramidOperations.compute:48-53
    sp.lp_inv = 1.0f / (p.min_freq * 0.2f);
    // steerable extension (mm_steer.hpp)
    sp.O = p.mode == MM_MODE_STEERABLE ? p.orientations : 1;
    sp.filt = p.temporal_filter;
    sp.r_low = p.iir_low;
    sp.r_high = p.iir_high;
    for (int k = 0; k < 8; ++k) {
        const double a = k < sp.O ? 2.0 * M_PI * k / sp.O : 0.0;
        sp.ang_c[k] = (float)cos(a);
        sp.ang_s[k] = (float)sin(a);
    }
    for (int i = 1; i < p.levels - 1; ++i) {
        // PyramidOperations.compute:59-64 (L=3: 0/0 = NaN -> empty band)
        volatile float num = (float)(i - 1), den = (float)(p.levels - 3);
        const float ratio = num / den;
        const float center = p.min_freq * powf(p.max_freq / p.min_freq, 1.0f - ratio);
        const float bwid = center * 0.5f;
        sp.lo[i] = center - bwid;
        sp.hi[i] = center + bwid;
        sp.inv_w[i] = 1.0f / (sp.hi[i] - sp.lo[i]);
    }
}

// k_cols' pyramid table holds <= 2 middle-band masks per bin: true unless some
// three bands share an open interval (ratio maxF/minF spread over few levels).
static bool bands_fit_table(const Spec &sp)
{
    for (int a = 1; a < sp.L - 1; ++a)
        for (int b = a + 1; b < sp.L - 1; ++b)
            for (int c = b + 1; c < sp.L - 1; ++c) {
                const float lo = fmaxf(sp.lo[a], fmaxf(sp.lo[b], sp.lo[c]));
                const float hi = fminf(sp.hi[a], fminf(sp.hi[b], sp.hi[c]));
                if (lo < hi) return false;   // NaN bands (L = 3) compare false
            }
    return true;
}

// Two middle bands overlap on an interval of positive width (relative 1e-5:
// bands that only touch at a mask zero, L <= 5 at the default 0.05 / 0.45,
// can share a bin by a rounding ulp, which the kernel's per-wave check still
// routes to the generic op): k_cols runs MM_K2_PYR_TAB2.
static bool bands_overlap(const Spec &sp)
{
    for (int a = 1; a < sp.L - 1; ++a)
        for (int b = a + 1; b < sp.L - 1; ++b) {
            const float lo = fmaxf(sp.lo[a], sp.lo[b]), hi = fminf(sp.hi[a], sp.hi[b]);
            if (hi - lo > 1e-5f * hi) return true;   // NaN bands (L = 3) compare false
        }
    return false;
}

// k_cols' power-form instance for this handle (mm_kernels.hpp cpow_x2), opt-in
// with MM_K2_POW=1 (measured slower than the atan2 form): |S| for an integer
// phase scale with a compiled instance (|S| 25 and 10, the configurations'
// values, at N >= 2048), else 0 (the atan2 form).
static int k2_power_exponent(const Spec &sp, int N)
{
    if (!getenv("MM_K2_POW") || atoi(getenv("MM_K2_POW")) == 0) return 0;
    return N >= 2048 && (sp.S_pow == 25 || sp.S_pow == 10) ? sp.S_pow : 0;
}

// GaussianBlur.shader:47-60 at _BlurSize 0.5 (.cs:427): bilinear taps at
// +-0.6923 and +-1.6154 texels == a 5-tap FIR.
static Blur5 build_blur()
{
    const double c0 = 0.2270270270, c1 = 0.3162162162, c2w = 0.0702702703;
    const double f1 = 0.5 * 1.3846153846, f2 = 0.5 * 3.2307692308 - 1.0;
    Blur5 b;
    b.w0 = (float)(c0 + 2.0 * c1 * (1.0 - f1));
    b.w1 = (float)(c1 * f1 + c2w * (1.0 - f2));
    b.w2 = (float)(c2w * f2);
    return b;
}

static int validate_params(const mm_params *p)
{
    if (!p) return MM_ERR_INVALID;
    if (p->levels < 1 || p->levels > kMaxLevels) return MM_ERR_UNSUPPORTED;
    if (p->mode == MM_MODE_STEERABLE) {
        // cos^4 lobes cover every direction from 4 orientations up; even O pairs
        // each lobe with its conjugate mirror (oracle/steerable_ref.py)
        if (p->orientations != 4 && p->orientations != 6 && p->orientations != 8)
            return MM_ERR_UNSUPPORTED;
        if (p->temporal_filter != MM_FILTER_DIFF && p->temporal_filter != MM_FILTER_IIR)
            return MM_ERR_INVALID;
        if (p->temporal_filter == MM_FILTER_IIR &&
            !(p->iir_low > 0.0f && p->iir_low < p->iir_high && p->iir_high <= 1.0f))
            return MM_ERR_INVALID;
    } else {
        if (p->orientations != 1) return MM_ERR_UNSUPPORTED;
        if (p->mode != MM_MODE_PYRAMID && p->mode != MM_MODE_STANDARD) return MM_ERR_UNSUPPORTED;
    }
    if (p->edge_mode != MM_EDGE_REPEAT && p->edge_mode != MM_EDGE_CLAMP) return MM_ERR_INVALID;
    if (!(p->min_freq > 0.0f) || !(p->max_freq > 0.0f)) return MM_ERR_INVALID;
    return MM_OK;
}

// ------------------------------------------------------------------------
// launches
// ------------------------------------------------------------------------
// slots of one column of K2's per-bin table (k2_tab_slots)
static constexpr int ktab_slots(int log2n)
{
    const int C = fft_c_v(log2n), te = (1 << log2n) / 2 + 1;
    return (te + C - 1) / C * C;
}

static int ilog2(int n)
{
    int l = 0;
    while ((1 << l) < n) ++l;
    return l;
}

template <int LOG2N> static size_t lds_fft_bytes()
{
    return sizeof(c2) * (size_t)groups_per_wg<LOG2N>() * lds_complex<(1 << LOG2N)>();
}
template <int LOG2N>
static int set_attrs(int W)
{
    (void)W;   // every other kernel stays within the default 64 KiB dynamic LDS
    if constexpr (LOG2N == 12) {   // k_rows_inv_compose: two 4096-point groups, 73.7 KB
        const int lds = (int)(sizeof(c2) * 2 * lds_complex<4096>());
        for (int f = 0; f < 4; ++f)
            MM_FMT_SWITCH(f, HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rows_inv_compose<12, FMT_>),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds)))
        // k_sb_cols: exchange buffers (73.7 KB) + its own staging (run_steer)
        HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sb_cols<12>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        // k_sb_rows: sb_rows_groups<12>() 4096-point transforms (73.7 KB at two)
        if constexpr (sb_rows_groups<12>() > 1) {
            const int rl = (int)(sizeof(c2) * sb_rows_groups<12>() * lds_complex<4096>());
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sb_rows<12, false, 1>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, rl));
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sb_rows<12, false, 2>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, rl));
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sb_rows<12, false, 4>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, rl));
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sb_rows<12, true, 1>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, rl));
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sb_rows<12, true, 2>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, rl));
        }
    }
    if constexpr (LOG2N == 13) {   // N = 8192: one 8192-point transform per workgroup, 73.7 KB and more
        auto set = [](const void *f, size_t b) {
            return b > 65536 ? hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b)
                             : hipSuccess;
        };
        const size_t x = sizeof(c2) * lds_complex<8192>();
        HIPCHK(set(reinterpret_cast<const void *>(&k_rows_inv<13>), sizeof(c2) * k3_groups<13>() * lds_complex<8192>()));
        HIPCHK(set(reinterpret_cast<const void *>(&k_dbg_cols<13>), 2 * sizeof(c2) * lds_complex<4096>()));
        (void)x;
#define MM_SET_K2(MODE, SP)                                                                                       \
        HIPCHK(set(reinterpret_cast<const void *>(&k_cols<13, MODE, SP>), k2_lds_bytes<13, MODE>()));            \
        HIPCHK(set(reinterpret_cast<const void *>(&k_cols_tail<13, MODE, SP>), k2_lds_bytes<13, MODE>()))
        MM_SET_K2(MM_MODE_PYRAMID, 0);
        MM_SET_K2(MM_MODE_STANDARD, 0);
        MM_SET_K2(MM_K2_PYR_TAB, 0);
        MM_SET_K2(MM_K2_PYR_TAB, 25);
        MM_SET_K2(MM_K2_PYR_TAB, 10);
        // (no two-band instance: its mask-sum arrays would take K2 past 160 KB
        // of LDS at N = 8192; overlapping bands run the generic op there)
#undef MM_SET_K2
    }
    if constexpr (LOG2N == 11) {   // k_rows_inv_compose4: four 2048-point groups, 73.7 KB
        const int lds = (int)(sizeof(c2) * 4 * lds_complex<2048>());
        for (int f = 0; f < 4; ++f)
            MM_FMT_SWITCH(f, HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rows_inv_compose4<11, FMT_>),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, lds)))
        // k_sb_cols with four columns per workgroup (MM_SB_MIN_GROUPS = 4):
        // exchange buffers (73.7 KB) + its own staging
        if constexpr (sb_groups<11>() == 4)
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_sb_cols<11>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    return MM_OK;
}

template <int LOG2N>
static int launch_k1(mm_handle *h, const uint8_t *in, int nframes, int fmt, hipStream_t s, c2 *G)
{
    const int ppf = (h->H + 1) / 2;   // odd H: the last pair's second row is zero
    const int total = ppf * nframes;
    // fewer than 2 workgroups per CU at the batch form: the one-pair form
    const bool lat = (total + k1_groups<LOG2N>() - 1) / k1_groups<LOG2N>() < 512;
    const size_t fb = (size_t)h->W * h->H * fmt_bpp(fmt);
    ProfScope ps(h, s, MM_K_ROWS_FWD, nframes);
#define MM_K1_LAUNCH(F, GEN, LAT)                                                                  \
    do {                                                                                           \
        constexpr int gpw = k1_gpw<LOG2N, LAT>();                                                  \
        const size_t lds = sizeof(c2) * (size_t)gpw * lds_complex<(1 << LOG2N)>();                \
        if (lds > 65536)                                                                           \
            HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_rows_fwd<LOG2N, F, GEN, LAT>), \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));     \
        hipLaunchKernelGGL((k_rows_fwd<LOG2N, F, GEN, LAT>), dim3((total + gpw - 1) / gpw),         \
                           dim3(gpw * fft_T<LOG2N>()), lds, s, in, fb, ppf, total, h->geo,         \
                           h->d_col3, h->d_row3, h->d_col, h->d_row, h->d_tw, G, h->g_stride);     \
    } while (0)
    const bool gen = h->geo.ox || h->geo.oy;   // odd W/H: taps span i-2 .. i+1
    MM_FMT_SWITCH(fmt, if (gen) MM_K1_LAUNCH(FMT_, true, false);
                       else if (lat) MM_K1_LAUNCH(FMT_, false, true);
                       else MM_K1_LAUNCH(FMT_, false, false))
#undef MM_K1_LAUNCH
    HIPCHK(hipGetLastError());
    return MM_OK;
}

// K2 over frames G[0 .. nframes) (K1's row spectra), primed with Gprev = G_{t-1}
// (the state slot, or frame 0 itself for a stream's first batch, whose frame 0
// passes through): Q of frame fr to d_Q + fr * q_stride.
template <int LOG2N>
static int launch_k2(mm_handle *h, int nframes, const c2 *Gprev, const c2 *G, hipStream_t s)
{
    const int gpw = k2_groups<LOG2N>();
    const int cols = (1 << LOG2N) / 2;   // f = 0 and f = N/2 share group 0 (k_cols)
    const int blocks = (cols + gpw - 1) / gpw;
    // the per-bin tables, stream-ordered before this launch after a parameter change
    static_assert(ktab_slots(LOG2N) == k2_tab_slots<LOG2N>(), "d_ktab column stride");
    const int tab_mode = h->spec.mode == MM_MODE_STANDARD ? MM_MODE_STANDARD : h->k2_tab ? MM_K2_PYR_TAB : -1;
    if (tab_mode >= 0 && h->ktab_mode != tab_mode) {
        const int n = (cols + 1) * k2_tab_slots<LOG2N>();
        if (tab_mode == MM_MODE_STANDARD)
            hipLaunchKernelGGL((k_k2_table<LOG2N, MM_MODE_STANDARD>), dim3((n + 255) / 256), dim3(256), 0, s,
                               h->d_ktab, h->d_kmsum, h->spec);
        else
            hipLaunchKernelGGL((k_k2_table<LOG2N, MM_K2_PYR_TAB>), dim3((n + 255) / 256), dim3(256), 0, s,
                               h->d_ktab, h->d_kmsum, h->spec);
        HIPCHK(hipGetLastError());
        h->ktab_mode = tab_mode;
    }
    ProfScope ps(h, s, MM_K_COLS, nframes);
    // the packed block's last k frames go to k_cols_tail (k_cols's critical
    // path); all of them (k = nframes, block 0 not in k_cols) where
    // k2_pk_all is set: k_cols's LDS then omits the packed group's arrays
    const bool pk_all = h->k2_pk_all && nframes >= 24 && blocks >= 2;
    int k = nframes >= 24 ? nframes * h->k2_tail_pct / 100 : 0;
    k = pk_all ? nframes : std::max(0, std::min(k, nframes - 2));
    const int pk_off = pk_all ? 1 : 0, cb = blocks - pk_off;   // column blocks of k_cols
    // second-half tails (k_cols): the last k2 frames of each second-half block's
    // columns in extra blocks (MM_K2_TAIL2 percent)
    const int k2t = nframes >= 24 && cb >= 2 ? std::min(nframes * h->k2_tail2_pct / 100, nframes - 2) : 0;
    const int tb = k2t > 0 ? cb / 2 : 0;
#define MM_K2_LAUNCH(MODE, SP)                                                                       \
    do {                                                                                             \
        const int sc2 = h->k2_stg_ded ? k2_stg_c2<LOG2N, MODE>(h->geo.Hq, !pk_all) : 0; /* dedicated staging */ \
        /* (dedicated staging +) exchange buffers + per-bin tables (+ the packed group's) */       \
        const size_t lds = k2_lds_bytes<LOG2N, MODE>(!pk_all) + sizeof(c2) * (size_t)sc2;           \
        hipLaunchKernelGGL((k_cols<LOG2N, MODE, SP>), dim3(cb + tb), dim3(k2_threads<LOG2N>()), lds, s, G, \
                           h->g_stride, Gprev, h->d_Q, h->q_stride, nframes, h->geo, h->spec, h->d_tw, h->d_ktab, \
                           h->d_kmsum, sc2, nframes - k, tb, k2t, pk_off);                           \
        if (k) {                                                                                     \
            const int sct = h->k2_stg_ded ? k2_stg_c2<LOG2N, MODE>(h->geo.Hq) : 0;                  \
            const size_t ldt = k2_lds_bytes<LOG2N, MODE>() + sizeof(c2) * (size_t)sct;              \
            hipLaunchKernelGGL((k_cols_tail<LOG2N, MODE, SP>), dim3(k), dim3(k2_threads<LOG2N>()),  \
                               ldt, s, G, h->g_stride, Gprev,                                       \
                               h->d_Q, h->q_stride, nframes - k, h->geo, h->spec, h->d_tw, h->d_ktab,   \
                               h->d_kmsum, sct);                                                     \
        }                                                                                            \
    } while (0)
    // the power-form instances (k2_power_exponent): 1080p and 2160p, |S| 25, 10
    constexpr bool pow_ok = LOG2N >= 11;
    if (h->spec.mode == MM_MODE_STANDARD) MM_K2_LAUNCH(MM_MODE_STANDARD, 0);
    else if (pow_ok && h->k2_tab2 && h->k2_sp == 25) MM_K2_LAUNCH(MM_K2_PYR_TAB2, (pow_ok ? 25 : 0));
    else if (pow_ok && h->k2_tab2 && h->k2_sp == 10) MM_K2_LAUNCH(MM_K2_PYR_TAB2, (pow_ok ? 10 : 0));
    else if (h->k2_tab2) MM_K2_LAUNCH(MM_K2_PYR_TAB2, 0);
    else if (pow_ok && h->k2_tab && h->k2_sp == 25) MM_K2_LAUNCH(MM_K2_PYR_TAB, (pow_ok ? 25 : 0));
    else if (pow_ok && h->k2_tab && h->k2_sp == 10) MM_K2_LAUNCH(MM_K2_PYR_TAB, (pow_ok ? 10 : 0));
    else if (h->k2_tab) MM_K2_LAUNCH(MM_K2_PYR_TAB, 0);
    else MM_K2_LAUNCH(MM_MODE_PYRAMID, 0);
#undef MM_K2_LAUNCH
    HIPCHK(hipGetLastError());
    return MM_OK;
}

// Grows a per-batch buffer that only some paths use to `frames` frames of
// `per_frame` bytes.  The old buffer is retired behind this handle's work
// (its previous calls and what this call queued on s), not behind the
// device's; a failed allocation leaves the old one in place.
static int ensure_frames(mm_handle *h, void **buf, int *have, int frames, size_t per_frame, hipStream_t s)
{
    if (*buf && *have >= frames) return MM_OK;
    void *p = nullptr;
    if (h_alloc(h, &p, per_frame * (size_t)frames) != hipSuccess) return MM_ERR_OOM;
    h_retire(h, *buf, s, true);
    *buf = p;
    *have = frames;
    return MM_OK;
}
static int ensure_yh(mm_handle *h, hipStream_t s)
{
    return ensure_frames(h, reinterpret_cast<void **>(&h->d_Yh), &h->yh_frames, h->chunk,
                         sizeof(float) * h->yh_stride, s);
}

// G slot of the first frame of an n-frame batch: the batch must not
// overwrite the state slot gs (read by the batch's K2 as G_{t-1}).  With
// chunk + 1 slots the state moves (one slot copy) only when neither the slots
// after gs nor those before it hold the batch: once per full batch at most,
// never in the one-frame-per-call pattern (it alternates slots 0 and 1).
static int place_batch(mm_handle *h, int n, hipStream_t s, int *base)
{
    *base = 0;
    if (!h->g_valid) return MM_OK;   // no state slot to keep
    if (h->gs + 1 + n <= h->chunk + 1) {
        *base = h->gs + 1;
        return MM_OK;
    }
    if (n > h->gs) {
        HIPCHK(hipMemcpyAsync(h->d_G + h->g_stride * h->chunk, h->d_G + h->g_stride * h->gs,
                              sizeof(c2) * h->g_stride, hipMemcpyDeviceToDevice, s));
        h->gs = h->chunk;
    }
    return MM_OK;
}

static int launch_k4(mm_handle *h, const uint8_t *in, uint8_t *out, int frame0, int nframes,
                     int fmt, hipStream_t s);

// k_rows_inv_compose's geometry: even sizes whose quads tile the rows (W % 8 == 0
// puts x0 on a multiple of 4), the horizontal blur's float4 taps inside the
// canvas, and no vertical blur tap wrapping (list row of output row i + v is i + v)
static bool k34_fits(const mm_handle *h)
{
    const Geo &g = h->geo;
    return g.N <= 4096 &&   // two transforms per workgroup: 2 N / 8 <= 1024 threads
           !g.ox && !g.oy && g.W % 8 == 0 && g.x0 >= 4 && g.x0 % 4 == 0 &&
           g.x0 + g.W + 4 <= g.N && g.N - g.H >= 4 && g.Hn == g.H + 4 && g.rb == g.y0 - 2 &&
           2 * (g.N / 8) >= g.W / 4;
}

// Strip height of one k_rows_inv_compose launch over nout frames.  A strip is
// one workgroup walking its rows in sequence, so a launch needs many strips:
// about 4 workgroups per CU (H nout / R >= 1024) with R <= 64, and the unfused
// pair (0) when that would take strips under 16 rows (the one-frame drop-in
// call: K3 + K4 spread one frame over thousands of workgroups).  MM_K34_ROWS
// forces a strip height (0: unfused).
#ifndef MM_K34_ROWS_4K
#define MM_K34_ROWS_4K 128
#endif
static int k34_strip_rows(const mm_handle *h, int nout)
{
    if (h->k34_rows >= 0) return h->k34_rows;
    // at N = 4096 a K34 workgroup (1,024 threads, 125 VGPRs) is alone on its
    // CU, so a longer strip halves the halo rows at no cost in concurrency
    // (C3 same-call: R 64 -> 128, K34 26.4-26.8 -> 25.7-25.8 us per frame;
    // at 1080p 96 and 128 were slower than 64)
    const int cap = h->N >= 4096 ? MM_K34_ROWS_4K : 64;
    const int R = std::min(cap, (int)((long long)h->H * nout / 1024) / 4 * 4);
    return R >= 16 ? R : 0;
}

template <int LOG2N>
static int launch_k3(mm_handle *h, const uint8_t *in, uint8_t *out, int frame0, int nframes,
                     int fmt, hipStream_t s)
{
    const int nout = nframes - frame0;
    if (nout <= 0) return MM_OK;
    const size_t fb = (size_t)h->W * h->H * fmt_bpp(fmt);
    const int R = k34_strip_rows(h, nout);
    // Short launches (the one-frame call) at N <= 1024 whose strips fit one
    // workgroup round (4 waves per SIMD at <= 128 VGPRs: 1024 / 4T workgroups
    // per CU): K3 + K4 fused in one shot, four FFT groups per 4-row strip, no
    // walk (k_rows_inv_compose4).  One-frame calls, same call
    // (profiles/r03k_k34_oneshot.txt): 960x540 33.0 -> 29.8 us, 640x480
    // 30.4 -> 28.3 us, 1024x768 equal; at N = 2048 (16-wave workgroups, one
    // per CU) it lost even in one round (1280x720 42.0 -> 42.6 us) and 1080p's
    // 270 strips take two rounds (48.0 -> 54.4 us): K3 -> K4 there
    // (MM_K34_ONESHOT=2 forces it, 0 disables it).
    constexpr int k34o_per_cu = 4 * fft_T<LOG2N>() <= 1024 ? 1024 / (4 * fft_T<LOG2N>()) : 0;
    if constexpr (LOG2N <= 11) if (R == 0 && h->k34_rows < 0 && h->k34_oneshot && k34_fits(h) &&
                                   ((LOG2N <= 10 && (h->H + 3) / 4 * nout <= k34o_per_cu * h->num_cu) ||
                                    h->k34_oneshot == 2)) {
        const int strips = (h->H + 3) / 4;
        const size_t lds = sizeof(c2) * 4 * lds_complex<(1 << LOG2N)>();
        const dim3 grid((unsigned)(strips * nout)), block(4 * fft_T<LOG2N>());
        ProfScope ps(h, s, MM_K_ROWS_INV_COMPOSE, nout);
        MM_FMT_SWITCH(fmt, hipLaunchKernelGGL((k_rows_inv_compose4<LOG2N, FMT_>), grid, block, lds, s, h->d_Q,
                                              h->q_stride, in, out, fb, frame0, strips, h->geo, h->blur,
                                              h->d_col3, h->d_row3, h->d_tw))
        HIPCHK(hipGetLastError());
        return MM_OK;
    }
    if (R >= 4 && k34_fits(h)) {   // K3 + K4 fused: Yh stays on chip
        const int strips = (h->H + R - 1) / R, steps = R / 4 + 1;
        const size_t lds = sizeof(c2) * 2 * lds_complex<(1 << LOG2N)>();
        const dim3 grid((unsigned)(strips * nout)), block(2 * fft_T<LOG2N>());
        ProfScope ps(h, s, MM_K_ROWS_INV_COMPOSE, nout);
        MM_FMT_SWITCH(fmt, hipLaunchKernelGGL((k_rows_inv_compose<LOG2N, FMT_>), grid, block, lds, s, h->d_Q,
                                              h->q_stride, in, out, fb, frame0, strips, steps, h->geo,
                                              h->blur, h->d_col3, h->d_row3, h->d_tw))
        HIPCHK(hipGetLastError());
        return MM_OK;
    }
    const int ppf = h->geo.Hq / 2;   // whole Q tiles (k_rows_inv)
    const int total = ppf * nout;
    const int gpw = k3_groups<LOG2N>();
    int rc = ensure_yh(h, s);
    if (rc) return rc;
    {
        ProfScope ps(h, s, MM_K_ROWS_INV, nout);
        hipLaunchKernelGGL((k_rows_inv<LOG2N>), dim3((total + gpw - 1) / gpw),
                           dim3(k3_threads<LOG2N>()), sizeof(c2) * (size_t)gpw * lds_complex<(1 << LOG2N)>(),
                           s, h->d_Q,
                           h->q_stride, h->d_Yh, h->yh_stride, frame0, ppf, total, h->geo,
                           h->blur, h->d_tw);
        HIPCHK(hipGetLastError());
    }
    return launch_k4(h, in, out, frame0, nframes, fmt, s);
}

// K4 k_compose over chunk frames [frame0, nframes) (Yh of those frames ready)
static int launch_k4(mm_handle *h, const uint8_t *in, uint8_t *out, int frame0, int nframes,
                     int fmt, hipStream_t s)
{
    const int nout = nframes - frame0;
    if (nout <= 0) return MM_OK;
    const size_t fb = (size_t)h->W * h->H * fmt_bpp(fmt);
    if (h->geo.ox || h->geo.oy) {   // odd W/H: the crop samples between texels
        const size_t tot = (size_t)nout * h->W * h->H;
        ProfScope ps(h, s, MM_K_COMPOSE, nout);
        const dim3 grid((unsigned)((tot + 255) / 256));
        MM_FMT_SWITCH(fmt, hipLaunchKernelGGL((k_compose_odd<FMT_>), grid, dim3(256), 0, s, h->d_Yh,
                                              h->yh_stride, in, out, fb, frame0, nout, h->geo, h->blur,
                                              h->d_col, h->d_row))
        HIPCHK(hipGetLastError());
        return MM_OK;
    }
    const int rt = (h->H + kTileRows - 1) / kTileRows, ct = (h->W + kTileCols - 1) / kTileCols;
    const dim3 grid(rt * ct * nout);
    ProfScope ps(h, s, MM_K_COMPOSE, nout);
    MM_FMT_SWITCH(fmt, hipLaunchKernelGGL((k_compose<FMT_>), grid, dim3(kTileCols), 0, s, h->d_Yh,
                                          h->yh_stride, in, out, fb, frame0, rt, ct, h->geo, h->blur,
                                          h->d_col3, h->d_row3))
    HIPCHK(hipGetLastError());
    return MM_OK;
}

// ---- MM_MODE_STEERABLE (mm_steer.hpp) -----------------------------------
static int steer_bands(const mm_handle *h)
{
    const int nmid = h->spec.L >= 3 ? h->spec.L - 2 : 0;
    return nmid * (h->spec.O / 2);
}
// state planes: phi (DIFF reads only the previous local phase), + u_h, u_l (IIR)
static int steer_planes(const mm_handle *h) { return h->spec.filt == MM_FILTER_IIR ? 3 : 1; }
static size_t steer_plane_floats(const mm_handle *h)
{
    return (size_t)steer_bands(h) * h->geo.Hn * (h->geo.Wy + 4);
}
static size_t steer_state_bytes(const mm_handle *h)
{
    return sizeof(float) * steer_planes(h) * steer_plane_floats(h);
}
// Band buffers and the temporal state planes for the current levels and
// orientations.  Reallocated (state invalid) only when those change, never
// by mm_set_batch: the per-batch spectra Fb grow separately (ensure_frames).
// frames of one k_sb_cols launch chunk (MM_SB_CF, 2 .. 16: k_sb_rows' write
// mask holds a bit per frame of its launch; per-frame launches at N = 4096)
static int sb_cols_frames(const mm_handle *h)
{
    return std::min(16, std::max(2, h->N >= 4096 ? h->sb_cf4k : h->sb_cf));
}
static int steer_alloc(mm_handle *h, hipStream_t s)
{
    const int nb = steer_bands(h);
    const size_t fstride = (size_t)(h->N / 2 + 1) * h->N;
    int rc = ensure_frames(h, reinterpret_cast<void **>(&h->d_Fb), &h->fb_frames, h->chunk,
                           sizeof(c2) * fstride, s);
    if (rc) return rc;
    if ((rc = ensure_yh(h, s))) return rc;
    if (h->steer_nb == nb && h->steer_planes >= steer_planes(h)) return MM_OK;
    // in-flight work of this handle may still use the old planes
    h_retire(h, h->d_T, s, true);
    h_retire(h, h->d_sst, s, true);
    h->d_T = nullptr;
    h->d_sst = nullptr;
    h->steer_nb = -1;
    h->steer_valid = false;
    // band rows of the frames one k_sb_cols launch chunk covers (sb_cols_frames;
    // at least the k_sb_rows group: pairs, MM_SB_NF=4: DIFF in fours)
    const int tfr = std::max(sb_cols_frames(h), h->sb_nf >= 4 ? 4 : 2);
    if (h_alloc(h, &h->d_T, sizeof(c2) * tfr * (size_t)(nb + 1) * h->N * t_rows(h->geo.Hn)) != hipSuccess ||
        h_alloc(h, &h->d_sst, steer_state_bytes(h) + sizeof(float)) != hipSuccess)
        return MM_ERR_OOM;
    h->steer_nb = nb;
    h->steer_planes = steer_planes(h);
    return MM_OK;
}

// Batch frames [0, n) with K1's row spectra in G: k_cols_fwd -> per frame
// k_sb_cols, k_sb_rows (the temporal filter runs frame by frame) -> K4.
// `sst`: state planes (nullptr: the handle's own, whose first frame passes
// through and seeds them when they hold no valid state; a caller's buffer
// (mm_compute_state) is always seeded).  write == false: outputs pass through,
// the state keeps following the input.
template <int LOG2N>
static int run_steer(mm_handle *h, const uint8_t *in, uint8_t *out, int n, int fmt, float *sst,
                     bool write, hipStream_t s, const c2 *G)
{
    constexpr int N = 1 << LOG2N;
    int rc;
    if ((rc = steer_alloc(h, s))) return rc;   // may invalidate the handle's planes
    const int seed = sst ? 1 : (h->steer_valid ? 0 : 1);
    if (!sst) sst = h->d_sst;
    const size_t fstride = (size_t)(N / 2 + 1) * N;
    const int gpw = groups_per_wg<LOG2N>();
    const size_t lds = lds_fft_bytes<LOG2N>();
    {
        const int total = n * (N / 2 + 1);
        ProfScope ps(h, s, MM_K_COLS, n);
        hipLaunchKernelGGL((k_cols_fwd<LOG2N>), dim3((total + gpw - 1) / gpw),
                           dim3(wg_threads<LOG2N>()), lds, s, G, h->g_stride, h->d_Fb,
                           fstride, total, h->geo, h->d_tw);
        HIPCHK(hipGetLastError());
    }
    const size_t band_stride = (size_t)N * t_rows(h->geo.Hn);
    // DIFF reads and writes only the phi plane (a caller's DIFF state buffer
    // holds just that plane); IIR the three
    const size_t plane = steer_planes(h) == 3 ? steer_plane_floats(h) : 0;
    // frames in pairs: both frames' band columns, then one k_sb_rows launch
    // whose workgroups carry the first frame's new state to the second in
    // registers (MM_SB_NF=1: one frame per launch)
    const size_t t_stride = band_stride * (size_t)(steer_bands(h) + 1);
    // frames of this k_sb_rows launch: 4 (MM_SB_NF=4, DIFF; opt-in: C3
    // k_sb_rows -1.3 % but k_sb_cols +2.3 %, 1080p k_sb_rows +16 % at 4
    // waves per SIMD, profiles/r06h_sb_rows_layout_ab.txt), 2 or 1
    const int nfm = h->sb_nf >= 4 && h->spec.filt != MM_FILTER_IIR ? 4 : h->sb_nf >= 2 ? 2 : 1;
    // k_sb_cols runs the band columns of sb_cf (MM_SB_CF, default 8) frames per
    // launch at N <= 2048 (blockIdx.y: frame), then the chunk's k_sb_rows
    // groups: the kernel boundaries are what it saves (1080p O = 8 DIFF, same
    // call: 1 / 2 / 4 / 8 frames per launch 5.33k / 5.54k / 5.64k / 5.67k
    // frames/s; 1.85 GB of band rows at 8); per frame at N = 4096, whose
    // 2,048-workgroup launches gain nothing from it (C3 k_sb_cols 424 -> 430
    // us at 2; profiles/r06h_sb_rows_layout_ab.txt)
    const int cf = std::max(sb_cols_frames(h), nfm);
    for (int c0 = 0; c0 < n; c0 += cf) {
        const int cn = std::min(cf, n - c0);
        {
            ProfScope ps(h, s, MM_K_COLS, 0);
            const int g2 = sb_groups<LOG2N>();
            // the staging [Hn][GPW] gets its own LDS area where it costs no
            // residency: two workgroups per CU at N <= 2048 (1080p: 54 KB
            // each), and at N = 4096, whose 1,024-thread workgroups are alone
            // on their CU anyway (126 VGPRs: 4 waves per SIMD), within the
            // CU's 160 KB (2160p: 73.7 + 34.6 KB); else it aliases the
            // exchange buffers (one more barrier per band, and a band's
            // stores cannot overlap the next band's transform)
            // (one column per workgroup, sb_direct: two exchange buffers, no staging)
            const size_t lx = sizeof(c2) * (size_t)(sb_direct<LOG2N>() ? 2 : g2) * lds_complex<N>(),
                         ls = sizeof(c2) * (size_t)g2 * sb_stg_stride(h->geo.Hn, N);   // (whole row groups)
            const size_t own_cap = sb_threads<LOG2N>() >= 1024 ? 160 * 1024 : 81920;
            const int own = !sb_direct<LOG2N>() && h->sb_stg_own && lx + ls <= own_cap ? 1 : 0;
            const int per = LOG2N >= 12 ? 1 : cn;
            for (int f = 0; f < cn; f += per) {
                hipLaunchKernelGGL((k_sb_cols<LOG2N>), dim3((N + g2 - 1) / g2, per), dim3(sb_threads<LOG2N>()),
                                   lx + (own ? ls : 0), s, h->d_Fb + fstride * (c0 + f), h->d_T + t_stride * f,
                                   band_stride, h->geo, h->spec, h->d_tw, own, fstride, t_stride);
                HIPCHK(hipGetLastError());
            }
        }
        for (int k = c0; k < c0 + cn;) {
            const int left = c0 + cn - k;
            const int nf = left >= nfm ? nfm : (nfm >= 2 && left >= 2 ? 2 : 1);
            // the chunk's whole groups of nf frames in one launch, each
            // workgroup running them one after the other (MM_SB_RG=0: a launch
            // per group)
            const int ng = h->sb_rg && h->spec.filt != MM_FILTER_IIR ? left / nf : 1;
            const int reset = k < seed;
            // bit f: frame k + f's Yh (the stream's first frame passes through)
            const int wmask = write ? (((1 << (ng * nf)) - 1) & ~(reset ? 1 : 0)) : 0;
            ProfScope ps(h, s, MM_K_ROWS_INV, __builtin_popcount(wmask));
            constexpr int rg = sb_rows_groups<LOG2N>();
            const dim3 grid((h->geo.Hn + rg - 1) / rg), block(sb_rows_threads<LOG2N>());
            const size_t rlds = sizeof(c2) * (size_t)rg * lds_complex<N>();
            float *yh = h->d_Yh + h->yh_stride * k;
            c2 *tk = h->d_T + t_stride * (k - c0);
#define MM_SB_ROWS(IIRV, NFV)                                                                              \
            hipLaunchKernelGGL((k_sb_rows<LOG2N, IIRV, NFV>), grid, block, rlds, s, tk, band_stride, t_stride, \
                               yh, h->yh_stride, sst, sst + plane, sst + 2 * plane, reset, wmask, h->geo,   \
                               h->spec, h->blur, h->d_tw, ng)
            if (h->spec.filt == MM_FILTER_IIR) {
                if (nf == 2) MM_SB_ROWS(true, 2);
                else MM_SB_ROWS(true, 1);
            } else {
                if (nf == 4) MM_SB_ROWS(false, 4);
                else if (nf == 2) MM_SB_ROWS(false, 2);
                else MM_SB_ROWS(false, 1);
            }
#undef MM_SB_ROWS
            HIPCHK(hipGetLastError());
            k += ng * nf;
        }
    }
    if (sst == h->d_sst) h->steer_valid = true;
    const size_t fb = (size_t)h->W * h->H * fmt_bpp(fmt);
    if (!write) {
        if (out) HIPCHK(hipMemcpyAsync(out, in, fb * n, hipMemcpyDeviceToDevice, s));
        return MM_OK;
    }
    if (seed) HIPCHK(hipMemcpyAsync(out, in, fb, hipMemcpyDeviceToDevice, s));
    return launch_k4(h, in, out, seed, n, fmt, s);
}

// ProcessDebugView (.cs:119-123, :234-257) for batch frames [first, n) whose
// row spectra are in G: k_dbg_cols (view textures) -> k_dbg_out (crop or split
// screen).  The state follows the input (.cs:122): the caller's slot update.
template <int LOG2N>
static int run_debug(mm_handle *h, uint8_t *out, int n, int first, int fmt, hipStream_t s,
                     const c2 *G)
{
    constexpr int N = 1 << LOG2N;
    if (n <= first) return MM_OK;
    const size_t tex_stride = (size_t)2 * N * N;
    // lazily (only handles that show a debug view pay for it), sized for the batch
    int rc = ensure_frames(h, reinterpret_cast<void **>(&h->d_dbg), &h->dbg_frames, h->chunk,
                           sizeof(float) * tex_stride, s);
    if (rc) return rc;
    if (!h->d_tw_half) {
        std::vector<c2> twh(N / 2);
        for (int k = 0; k < N / 2; ++k) {
            const double a = -2.0 * M_PI * (double)k / (double)(N / 2);
            twh[k] = mk((float)cos(a), (float)sin(a));
        }
        HIPCHK(h_alloc(h, &h->d_tw_half, sizeof(c2) * (N / 2)));
        HIPCHK(hipMemcpyAsync(h->d_tw_half, twh.data(), sizeof(c2) * (N / 2), hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    }
    const int m = n - first;
    constexpr int T = fft_T<LOG2N - 1>();
    hipLaunchKernelGGL((k_dbg_cols<LOG2N>), dim3(m * N), dim3(2 * T),
                       2 * sizeof(c2) * lds_complex<N / 2>(), s, G, h->g_stride, h->d_dbg,
                       tex_stride, first, h->p.show_magnitude, h->p.show_phase, h->geo,
                       h->d_tw_half);
    HIPCHK(hipGetLastError());
    const size_t fb = (size_t)h->W * h->H * fmt_bpp(fmt);
    const size_t tot = (size_t)m * h->W * h->H;
    const dim3 grid((unsigned)((tot + 255) / 256));
    MM_FMT_SWITCH(fmt, hipLaunchKernelGGL((k_dbg_out<FMT_>), grid, dim3(256), 0, s, h->d_dbg, tex_stride,
                                          out, fb, first, m, h->p.show_magnitude, h->p.show_phase, h->geo))
    HIPCHK(hipGetLastError());
    return MM_OK;
}

// One batch of `n` consecutive frames (n <= chunk), all on the device.
template <int LOG2N>
static int run_chunk(mm_handle *h, const uint8_t *in, uint8_t *out, int n, int fmt,
                     hipStream_t s)
{
    const size_t fb = (size_t)h->W * h->H * fmt_bpp(fmt);
    const bool mag = h->p.apply_magnification != 0;
    const bool dbg = h->p.show_magnitude || h->p.show_phase;
    // the steerable path's state is its local-phase planes; every other path
    // needs G_{t-1} in the G slot (a steerable mm_set_state leaves it unset:
    // the next pyramid frame then passes through, as after a reset)
    const bool steer = !dbg && h->p.mode == MM_MODE_STEERABLE;
    const bool have = h->has_state && (steer || h->g_valid);
    const int first = have ? 0 : 1;
    int rc, base;
    if (first) HIPCHK(hipMemcpyAsync(out, in, fb, hipMemcpyDeviceToDevice, s));
    if ((rc = place_batch(h, n, s, &base))) return rc;
    c2 *G = h->d_G + h->g_stride * base;
    // G_{t-1}: the state slot; a stream's first frame primes with itself (its
    // Q is computed and not used: it passes through)
    const c2 *Gprev = have ? h->d_G + h->g_stride * h->gs : G;
    if (!dbg && h->p.mode != MM_MODE_STEERABLE && !mag) {
        // applyMotionMagnification == false: Blit(source, destination) (.cs:139),
        // but previousSourceTexture still follows the input (.cs:142): K1 of
        // the batch's last frame only.
        const int from = first ? 1 : 0;
        if (n > from)
            HIPCHK(hipMemcpyAsync(out + fb * from, in + fb * from, fb * (n - from),
                                  hipMemcpyDeviceToDevice, s));
        if ((rc = launch_k1<LOG2N>(h, in + fb * (n - 1), 1, fmt, s, G))) return rc;
        h->gs = base;
        h->has_state = h->g_valid = true;
        return MM_OK;
    }
    if ((rc = launch_k1<LOG2N>(h, in, n, fmt, s, G))) return rc;
    if (dbg) {
        h->steer_valid = false;   // the debug path does not advance the local-phase state
        rc = run_debug<LOG2N>(h, out, n, first, fmt, s, G);
    } else if (h->p.mode == MM_MODE_STEERABLE) {
        if (first) h->steer_valid = false;
        // two transforms per band workgroup: N <= 4096 (mm_create refuses more)
        if constexpr (LOG2N <= 12) rc = run_steer<LOG2N>(h, in, out, n, fmt, nullptr, mag, s, G);
        else rc = MM_ERR_UNSUPPORTED;
    } else {
        if ((rc = launch_k2<LOG2N>(h, n, Gprev, G, s))) return rc;
        rc = launch_k3<LOG2N>(h, in, out, first, n, fmt, s);
    }
    if (rc) return rc;
    h->gs = base + n - 1;   // the state follows the input in every mode (.cs:142)
    h->has_state = h->g_valid = true;
    return MM_OK;
}

template <int LOG2N>
static int run_stream(mm_handle *h, const uint8_t *in, uint8_t *out, int count, int fmt,
                      hipStream_t s)
{
    const size_t fb = (size_t)h->W * h->H * fmt_bpp(fmt);
    for (int f0 = 0; f0 < count; f0 += h->chunk) {
        const int n = std::min(h->chunk, count - f0);
        int rc = run_chunk<LOG2N>(h, in + fb * f0, out + fb * f0, n, fmt, s);
        if (rc) return rc;
    }
    return MM_OK;
}

// The state frame `in` leaves behind: its row spectra (K1) straight into dst;
// steerable DIFF: its local phases (K1 to a free G slot, then the band path).
template <int LOG2N>
static int compute_state(mm_handle *h, const uint8_t *in, int fmt, void *dst, hipStream_t s)
{
    int rc;
    if (h->p.mode == MM_MODE_STEERABLE) {
        int base;
        if ((rc = place_batch(h, 1, s, &base))) return rc;
        c2 *G = h->d_G + h->g_stride * base;
        if ((rc = launch_k1<LOG2N>(h, in, 1, fmt, s, G))) return rc;
        if constexpr (LOG2N <= 12)
            return run_steer<LOG2N>(h, in, nullptr, 1, fmt, reinterpret_cast<float *>(dst), false, s, G);
        else
            return MM_ERR_UNSUPPORTED;
    }
    return launch_k1<LOG2N>(h, in, 1, fmt, s, reinterpret_cast<c2 *>(dst));
}

// MM_ONLY_LOG2N=n (experiment builds only): instantiate one padded size, so an
// A/B variant compiles in a fraction of the full build's time

// The per-size entry points (defined in mm_n<L>.hip by MM_SIZE_ENTRIES(L),
// or in mm_api.hip itself for a one-size experiment build, MM_ONLY_LOG2N)
#define MM_SIZE_DECLS(L)                                                                            \
    int mm_size_set_attrs_##L(mm_handle *h);                                                        \
    int mm_size_stream_##L(mm_handle *h, const uint8_t *in, uint8_t *out, int count, int fmt,       \
                           hipStream_t s);                                                          \
    int mm_size_compute_state_##L(mm_handle *h, const uint8_t *in, int fmt, void *dst, hipStream_t s);
#define MM_SIZE_ENTRIES(L) MM_SIZE_ENTRIES_(L)
#define MM_SIZE_ENTRIES_(L)                                                                         \
    int mm_size_set_attrs_##L(mm_handle *h) { return set_attrs<L>(h->W); }                          \
    int mm_size_stream_##L(mm_handle *h, const uint8_t *in, uint8_t *out, int count, int fmt,       \
                           hipStream_t s)                                                           \
    {                                                                                               \
        return run_stream<L>(h, in, out, count, fmt, s);                                            \
    }                                                                                               \
    int mm_size_compute_state_##L(mm_handle *h, const uint8_t *in, int fmt, void *dst, hipStream_t s) \
    {                                                                                               \
        return compute_state<L>(h, in, fmt, dst, s);                                                \
    }
MM_SIZE_DECLS(4)
MM_SIZE_DECLS(5)
MM_SIZE_DECLS(6)
MM_SIZE_DECLS(7)
MM_SIZE_DECLS(8)
MM_SIZE_DECLS(9)
MM_SIZE_DECLS(10)
MM_SIZE_DECLS(11)
MM_SIZE_DECLS(12)
MM_SIZE_DECLS(13)
