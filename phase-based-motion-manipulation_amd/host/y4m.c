/* y4m.c — see y4m.h. */
#include "y4m.h"

#include <stdlib.h>
#include <string.h>

static int clamp255(float v)
{
    int i = (int)(v + 0.5f);
    return i < 0 ? 0 : (i > 255 ? 255 : i);
}

/* "A:B" -> a, b */
static int parse_ratio(const char *s, int *a, int *b)
{
    return sscanf(s, "%d:%d", a, b) == 2 ? 0 : -1;
}

int y4m_read_header(FILE *f, y4m_info *info)
{
    char line[512];
    size_t n = 0;
    int c;
    while ((c = fgetc(f)) != EOF && c != '\n')
        if (n + 1 < sizeof(line)) line[n++] = (char)c;
    if (c != '\n') return -1;
    line[n] = 0;
    if (strncmp(line, "YUV4MPEG2", 9) != 0) return -1;
    memset(info, 0, sizeof(*info));
    info->fps_num = 25;
    info->fps_den = 1;
    info->aspect_num = info->aspect_den = 1;
    info->chroma = Y4M_420;
    info->interlace = 'p';
    char *save = NULL;
    for (char *tok = strtok_r(line + 9, " ", &save); tok; tok = strtok_r(NULL, " ", &save)) {
        const char *v = tok + 1;
        switch (tok[0]) {
        case 'W': info->width = atoi(v); break;
        case 'H': info->height = atoi(v); break;
        case 'F': if (parse_ratio(v, &info->fps_num, &info->fps_den)) return -1; break;
        case 'A': if (parse_ratio(v, &info->aspect_num, &info->aspect_den)) return -1; break;
        case 'I': info->interlace = v[0]; break;
        case 'C':
            if (!strcmp(v, "420") || !strcmp(v, "420jpeg") || !strcmp(v, "420paldv") ||
                !strcmp(v, "420mpeg2"))
                info->chroma = Y4M_420;
            else if (!strcmp(v, "444")) info->chroma = Y4M_444;
            else if (!strcmp(v, "mono")) info->chroma = Y4M_MONO;
            else return -1;   /* 422, 411, high bit depth, alpha: unsupported */
            break;
        default: break;       /* X (comments) and unknown tags */
        }
    }
    if (info->width <= 0 || info->height <= 0) return -1;
    return 0;
}

size_t y4m_frame_bytes(const y4m_info *info)
{
    const size_t w = (size_t)info->width, h = (size_t)info->height;
    if (info->chroma == Y4M_MONO) return w * h;
    if (info->chroma == Y4M_444) return 3 * w * h;
    const size_t cw = (w + 1) / 2, ch = (h + 1) / 2;
    return w * h + 2 * cw * ch;
}

int y4m_read_frame(FILE *f, const y4m_info *info, uint8_t *planes)
{
    char tag[6];
    if (fread(tag, 1, 5, f) != 5) return 0;
    tag[5] = 0;
    if (strcmp(tag, "FRAME") != 0) return -1;
    int c;
    while ((c = fgetc(f)) != EOF && c != '\n') {}   /* frame parameters: ignored */
    if (c != '\n') return -1;
    const size_t nb = y4m_frame_bytes(info);
    return fread(planes, 1, nb, f) == nb ? 1 : -1;
}

void y4m_to_rgba(const y4m_info *info, const uint8_t *planes, uint8_t *rgba, int full_range)
{
    const int W = info->width, H = info->height;
    const int cw = info->chroma == Y4M_420 ? (W + 1) / 2 : W;
    const uint8_t *Yp = planes;
    const uint8_t *Cb = planes + (size_t)W * H;
    const uint8_t *Cr = Cb + (size_t)cw * (info->chroma == Y4M_420 ? (H + 1) / 2 : H);
    /* BT.601: limited range scales Y by 255/219 and C by 255/224 */
    const float ky = full_range ? 1.0f : 255.0f / 219.0f, y0 = full_range ? 0.0f : 16.0f;
    const float kc = full_range ? 1.0f : 255.0f / 224.0f;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const float Y = ((float)Yp[(size_t)y * W + x] - y0) * ky;
            float cb = 0.0f, cr = 0.0f;
            if (info->chroma != Y4M_MONO) {
                const size_t ci = info->chroma == Y4M_420 ? (size_t)(y / 2) * cw + x / 2
                                                          : (size_t)y * W + x;
                cb = ((float)Cb[ci] - 128.0f) * kc;
                cr = ((float)Cr[ci] - 128.0f) * kc;
            }
            uint8_t *o = rgba + ((size_t)y * W + x) * 4;
            o[0] = (uint8_t)clamp255(Y + 1.402f * cr);
            o[1] = (uint8_t)clamp255(Y - 0.344136f * cb - 0.714136f * cr);
            o[2] = (uint8_t)clamp255(Y + 1.772f * cb);
            o[3] = 255;
        }
}

void y4m_from_rgba(int W, int H, const uint8_t *rgba, uint8_t *planes444, int full_range)
{
    const float ky = full_range ? 1.0f : 219.0f / 255.0f, y0 = full_range ? 0.0f : 16.0f;
    const float kc = full_range ? 1.0f : 224.0f / 255.0f;
    uint8_t *Yp = planes444, *Cb = planes444 + (size_t)W * H, *Cr = Cb + (size_t)W * H;
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        const float r = rgba[4 * i], g = rgba[4 * i + 1], b = rgba[4 * i + 2];
        const float Y = 0.299f * r + 0.587f * g + 0.114f * b;
        Yp[i] = (uint8_t)clamp255(Y * ky + y0);
        Cb[i] = (uint8_t)clamp255((b - Y) * (0.5f / 0.886f) * kc + 128.0f);
        Cr[i] = (uint8_t)clamp255((r - Y) * (0.5f / 0.701f) * kc + 128.0f);
    }
}

int y4m_write_header(FILE *f, int W, int H, int fps_num, int fps_den)
{
    return fprintf(f, "YUV4MPEG2 W%d H%d F%d:%d Ip A1:1 C444\n", W, H, fps_num, fps_den) > 0 ? 0 : -1;
}

int y4m_write_frame(FILE *f, int W, int H, const uint8_t *planes444)
{
    if (fputs("FRAME\n", f) < 0) return -1;
    const size_t nb = (size_t)3 * W * H;
    return fwrite(planes444, 1, nb, f) == nb ? 0 : -1;
}
