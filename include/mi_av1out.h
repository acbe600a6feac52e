/*
 * mi_av1out.h — the output side of the decode path: displayed pictures from the device to the
 * host (film grain fused with the copy) and the reference's output muxers.
 *
 * Two libraries implement it:
 *   - librav1d_amd.so (gfx950): mi_host_picture_alloc / _free, mi_output_picture;
 *   - libmi_av1dec.so (host C++): the muxers mi_muxer_* (no GPU code).
 *
 * Reference: the CLI's output stage (tools/output/output.rs), its muxers md5
 * (tools/output/md5.rs:541-637), yuv (tools/output/yuv.rs) and y4m2 (tools/output/y4m2.rs),
 * and the film-grain application rav1d runs on the picture it returns to the caller
 * (rav1d_apply_grain, src/fg_apply.rs:272-284; src/lib.rs output_picture_ready).
 *
 * Errors: 0 or a negative errno, as in mi_av1dsp.h.
 */
#ifndef MI_AV1OUT_H
#define MI_AV1OUT_H

#include <stddef.h>
#include <stdint.h>

#include "mi_av1dsp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- device -> host (librav1d_amd.so) ---------------------------------------------------- */

/* A picture in pinned, device-mapped host memory with the default-allocator geometry of the
 * device pictures (src/picture.rs:98-115: 128-aligned planes, +64 B on strides that are a
 * multiple of 1024), so a kernel can write it directly over PCIe. */
int  mi_host_picture_alloc(int w, int h, int layout, int bpc, MiPicture *pic);
void mi_host_picture_free(MiPicture *pic);

/* Enqueue the output of one displayed picture on `stream`: `out` (from mi_host_picture_alloc,
 * same geometry as `in`) receives `in` with film grain applied when `fg` is non-NULL — the
 * grain kernel stores its output straight into the host picture, so the grain pass and the
 * device-to-host copy are one pass over the picture — or a plain copy of the visible w x h
 * area otherwise. The host may read `out` once the stream is synchronised. */
int mi_output_picture(MiCtx *ctx, const MiPicture *in, const MiPicture *out,
                      const MiFilmGrainData *fg, int mtrx_identity, void *stream);

/* ---- muxers (libmi_av1dec.so) ----------------------------------------------------------- */

/* What a muxer's header needs (Dav1dPictureParameters + the sequence / frame header fields
 * y4m2 reads: seq_hdr.chr, frame_hdr.render_width / render_height). */
typedef struct MiOutParams {
    int32_t w, h, bpc, layout;
    int32_t chr;                  /* Dav1dChromaSamplePosition: 0 unknown, 1 vertical, 2 colocated */
    int32_t render_w, render_h;
} MiOutParams;

typedef struct MiMuxer MiMuxer;

/* name: "md5", "yuv", "y4m2" or "null" (tools/output/output.rs muxer table). file: a path, or
 * "-" for stdout, or NULL (md5 only: keep the digest for mi_muxer_digest / mi_muxer_verify).
 * fps: numerator, denominator (y4m2 header). -EINVAL on an unknown muxer, -EIO if the file
 * cannot be opened. */
int  mi_muxer_open(MiMuxer **out, const char *name, const char *file, const MiOutParams *p,
                   const unsigned fps[2]);
/* Write one displayed picture (host memory; rows of w << (bpc > 8) bytes per plane, the
 * visible area only, little-endian pixels). */
int  mi_muxer_write(MiMuxer *m, const MiPicture *pic);
/* md5: finish the hash and compare with a 32-hex-digit string (md5_verify): 0 equal, 1
 * different, -1 string too short; other muxers -EINVAL. */
int  mi_muxer_verify(MiMuxer *m, const char *md5_str);
/* md5: finish the hash and write the 32 hex digits + NUL to out (what md5_close prints). */
int  mi_muxer_digest(MiMuxer *m, char out[33]);
/* Write the trailer (md5: the digest line), close the file, free the muxer. */
void mi_muxer_close(MiMuxer *m);

#ifdef __cplusplus
}
#endif
#endif /* MI_AV1OUT_H */
