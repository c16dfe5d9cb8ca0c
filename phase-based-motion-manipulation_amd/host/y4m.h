/*
 * y4m.h — YUV4MPEG2 (.y4m) stream I/O and BT.601 colour conversion for the C
 * host driver (real clips instead of synthetic streams).
 *
 * Reads 8-bit 4:2:0 (C420, C420jpeg, C420paldv, C420mpeg2), 4:4:4 (C444) and
 * mono (Cmono) streams; writes 4:4:4.  Chroma is upsampled by sample
 * replication (each 4:2:0 sample covers its 2x2 block).  Colour matrix BT.601,
 * limited range (Y 16..235, C 16..240) unless `full_range` (JPEG-style 0..255).
 * Host-side only: the frames then go through mm_process_stream as RGBA8.
 */
#ifndef MM355_Y4M_H
#define MM355_Y4M_H

#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { Y4M_420 = 0, Y4M_444 = 1, Y4M_MONO = 2 };

typedef struct {
    int width, height;
    int fps_num, fps_den;   /* F tag (default 25:1) */
    int aspect_num, aspect_den;
    int chroma;             /* Y4M_420 | Y4M_444 | Y4M_MONO */
    char interlace;         /* I tag, 'p' if absent */
} y4m_info;

/* Parse the stream header.  Returns 0, or -1 (not Y4M / unsupported chroma or
 * bit depth / malformed). */
int y4m_read_header(FILE *f, y4m_info *info);

/* Bytes of one frame's planes for `info`. */
size_t y4m_frame_bytes(const y4m_info *info);

/* Read one frame ("FRAME..." line + planes) into `planes`
 * (y4m_frame_bytes bytes).  Returns 1 on a frame, 0 at end of stream, -1 on
 * a malformed frame. */
int y4m_read_frame(FILE *f, const y4m_info *info, uint8_t *planes);

/* planes -> RGBA8 (alpha 255), and RGBA8 -> 4:4:4 planes (Y, Cb, Cr). */
void y4m_to_rgba(const y4m_info *info, const uint8_t *planes, uint8_t *rgba, int full_range);
void y4m_from_rgba(int width, int height, const uint8_t *rgba, uint8_t *planes444, int full_range);

/* Write a C444 header / one C444 frame. */
int y4m_write_header(FILE *f, int width, int height, int fps_num, int fps_den);
int y4m_write_frame(FILE *f, int width, int height, const uint8_t *planes444);

#ifdef __cplusplus
}
#endif
#endif
