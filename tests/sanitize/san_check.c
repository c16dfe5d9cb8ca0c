/*
 * san_check.c — the CPU-side C code under AddressSanitizer + UndefinedBehavior
 * Sanitizer: the oracle (oracle/mm_ref.c) and the C driver's
 * YUV4MPEG2 module (phase-based-motion-manipulation_amd/host/y4m.c), compiled
 * together with -fsanitize=address,undefined -fno-sanitize-recover by
 * tests/test_sanitize.py.  Test infrastructure; exits non-zero on any finding.
 *
 * Exercised: the oracle's frame operator in pyramid, standard and debug-view
 * modes over several geometries (odd sizes and CLAMP included), state
 * get/set/reset, the stage entry points; the Y4M writer and reader round trip
 * for 4:4:4, 4:2:0 and mono streams, and malformed headers and truncated frames.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mm_ref.h"
#include "y4m.h"

static int oracle_stream(int W, int H, int L, float S, int edge, int mode)
{
    mm_ref *c = mm_ref_create(W, H, L, 0.05f, 0.45f, S, 0.01f, edge);
    if (!c) return 1;
    if (mode == 1) mm_ref_set_standard(c, 1, 1, 0.05f, 0.4f, 3.0f, 1.5f, 0.8f);
    if (mode == 2) mm_ref_set_debug(c, 1, 1);
    const size_t px = (size_t)W * H * 4;
    uint8_t *in = malloc(px), *out = malloc(px);
    float *fin = malloc(px * sizeof(float)), *fout = malloc(px * sizeof(float));
    void *st = malloc(mm_ref_state_size(c));
    if (!in || !out || !fin || !fout || !st) return 1;
    for (int t = 0; t < 4; ++t) {
        mm_ref_synth_frame(W, H, t, 0x5EED0000ull, 0, in);
        if (t == 2) {   /* state round trip mid-stream */
            mm_ref_get_state(c, st);
            mm_ref_set_state(c, st);
        }
        mm_ref_process_u8(c, in, out);
        for (size_t i = 0; i < px; ++i) fin[i] = in[i] / 255.0f;
    }
    mm_ref_process(c, fin, fout, NULL);
    mm_ref_reset(c);
    mm_ref_process(c, fin, fout, NULL);
    free(in);
    free(out);
    free(fin);
    free(fout);
    free(st);
    mm_ref_destroy(c);
    return 0;
}

static int stage_points(void)
{
    const int n = 64;
    float *y = calloc((size_t)n * n, sizeof(float)), *cx = calloc((size_t)2 * n * n, sizeof(float));
    float *m = calloc((size_t)n * n, sizeof(float));
    if (!y || !cx || !m) return 1;
    y[n * 3 + 5] = 1.0f;
    mm_ref_fft_centered(n, y, cx);
    mm_ref_fft_buffer1(n, y, cx);
    mm_ref_ifft_mag(n, cx, y);
    for (int i = 0; i < 5; ++i) mm_ref_mask(n, 5, i, 0.05f, 0.45f, m);
    mm_ref_mask(n, 3, 1, 0.05f, 0.45f, m);   /* the L=3 NaN band */
    mm_ref_bandpass_weights(n, 1, 0.05f, 0.4f, 3.0f, 1.5f, 0.8f, m);
    mm_ref_blur(n, 0, y);
    mm_ref_blur(n, 1, y);
    (void)mm_ref_normalize_phase(7.5f);
    free(y);
    free(cx);
    free(m);
    return 0;
}

static int y4m_roundtrip(int chroma, int W, int H)
{
    FILE *f = tmpfile();
    if (!f) return 1;
    const int cw = chroma == Y4M_420 ? (W + 1) / 2 : W, ch = chroma == Y4M_420 ? (H + 1) / 2 : H;
    fprintf(f, "YUV4MPEG2 W%d H%d F30000:1001 Ip A1:1%s\n", W, H,
            chroma == Y4M_420 ? " C420jpeg" : chroma == Y4M_444 ? " C444" : " Cmono");
    const size_t plane = (size_t)W * H, cplane = chroma == Y4M_MONO ? 0 : (size_t)cw * ch;
    uint8_t *buf = malloc(plane + 2 * cplane);
    for (int k = 0; k < 3; ++k) {
        fputs("FRAME\n", f);
        for (size_t i = 0; i < plane + 2 * cplane; ++i) buf[i] = (uint8_t)(i * 7 + k);
        fwrite(buf, 1, plane + 2 * cplane, f);
    }
    fputs("FRAME\n", f);          /* truncated last frame */
    fwrite(buf, 1, plane / 2, f);
    rewind(f);
    y4m_info info;
    if (y4m_read_header(f, &info)) return 1;
    uint8_t *planes = malloc(y4m_frame_bytes(&info) > 3 * plane ? y4m_frame_bytes(&info) : 3 * plane);
    uint8_t *rgba = malloc(plane * 4);
    int frames = 0, r;
    while ((r = y4m_read_frame(f, &info, planes)) == 1) {
        y4m_to_rgba(&info, planes, rgba, 0);
        y4m_to_rgba(&info, planes, rgba, 1);
        y4m_from_rgba(W, H, rgba, planes, 0);
        ++frames;
    }
    fclose(f);
    FILE *o = tmpfile();
    if (!o || y4m_write_header(o, W, H, 25, 1) || y4m_write_frame(o, W, H, planes)) return 1;
    fclose(o);
    free(buf);
    free(planes);
    free(rgba);
    return frames == 3 && r < 0 ? 0 : 1;   /* 3 frames, then the truncated one is malformed */
}

static int y4m_malformed(void)
{
    const char *bad[] = {"", "YUV4MPEG2\n", "YUV4MPEG2 W0 H0\n", "YUV4MPEG2 W-5 H7\n",
                         "YUV4MPEG2 W16 H16 C411\n", "YUV4MPEG2 W99999999 H99999999\n",
                         "NOTY4M W16 H16\n", "YUV4MPEG2 W16 H16 F0:0 A0:0 Xfoo=bar\n"};
    for (size_t i = 0; i < sizeof bad / sizeof bad[0]; ++i) {
        FILE *f = tmpfile();
        if (!f) return 1;
        fputs(bad[i], f);
        rewind(f);
        y4m_info info;
        if (y4m_read_header(f, &info) == 0) {   /* accepted: a frame read must still be safe */
            const size_t n = y4m_frame_bytes(&info);
            uint8_t *p = n && n < (1u << 28) ? malloc(n) : NULL;
            if (p) (void)y4m_read_frame(f, &info, p);
            free(p);
        }
        fclose(f);
    }
    return 0;
}

int main(void)
{
    mm_ref_set_threads(2);
    int fail = 0;
    fail |= oracle_stream(64, 48, 5, 25.0f, 0, 0);
    fail |= oracle_stream(64, 48, 4, 9.7f, 1, 0);
    fail |= oracle_stream(63, 47, 5, 10.0f, 0, 0);   /* odd: fractional pad offsets */
    fail |= oracle_stream(40, 72, 3, 10.0f, 0, 0);
    fail |= oracle_stream(64, 48, 5, 25.0f, 0, 1);   /* standard mode */
    fail |= oracle_stream(64, 48, 5, 25.0f, 1, 2);   /* debug views */
    fail |= stage_points();
    fail |= y4m_roundtrip(Y4M_444, 32, 24);
    fail |= y4m_roundtrip(Y4M_420, 33, 25);
    fail |= y4m_roundtrip(Y4M_MONO, 16, 16);
    fail |= y4m_malformed();
    printf(fail ? "san_check: FAILED\n" : "san_check: ok\n");
    return fail;
}
