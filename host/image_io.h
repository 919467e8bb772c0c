/* image_io.h -- OpenEXR / PNG file I/O for the BMFR host.
 *
 * Replaces the reference's OpenImageIO calls: read_image_file()
 * (bmfr.cpp:145-163, ImageInput::open + read_image(TypeDesc::FLOAT), 3
 * channels) and the PNG output of bmfr.cpp:519-553 (ImageOutput, FLOAT ->
 * 8 bit).  Self-contained over zlib: OpenEXR 2.x single-part files, scanline
 * or tiled (one-level; the full-resolution level of mip / rip maps), with
 * HALF / FLOAT / UINT channels and NONE, RLE, ZIPS, ZIP, PIZ, PXR24, B44,
 * B44A, DWAA or DWAB compression (the formats of the BMFR dataset and of
 * common renderers; B44 channels with the pLinear flag and deep / multi-part
 * files are rejected with an error); writer: FLOAT RGB, NONE or ZIP.  No
 * OpenEXR library or reference file exists here: parity is unpinned (the
 * tests check against independent encoders of the published schemes).
 */
#ifndef BMFR_IMAGE_IO_H
#define BMFR_IMAGE_IO_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum bmfr_exr_compression {
    BMFR_EXR_NONE = 0,
    BMFR_EXR_RLE = 1,
    BMFR_EXR_ZIPS = 2,
    BMFR_EXR_ZIP = 3,
    BMFR_EXR_PIZ = 4,   /* read only */
    BMFR_EXR_PXR24 = 5, /* read only (lossy: FLOAT samples keep 24 bits) */
    BMFR_EXR_B44 = 6,   /* read only (lossy for HALF samples: 4x4 blocks in 14 bytes) */
    BMFR_EXR_B44A = 7,  /* read only (B44, flat blocks in 3 bytes) */
    BMFR_EXR_DWAA = 8,  /* read only (lossy DCT of HALF colour channels, 32 lines per chunk) */
    BMFR_EXR_DWAB = 9   /* read only (DWAA with 256 lines per chunk) */
} bmfr_exr_compression;

/* Size of an EXR file's data window.  0 on success, else -1 (message via
 * bmfr_io_error()). */
int bmfr_exr_info(const char *path, int *width, int *height, int *channels);

/* Read the R, G, B channels (exactly three channels named R, G, B, or any
 * three channels in file order when there are exactly three) into an
 * interleaved float RGB buffer of width*height*3, rows top to bottom --
 * what read_image(TypeDesc::FLOAT) returns for the dataset's files.
 * Half and uint samples are converted to float. */
int bmfr_exr_read_rgb(const char *path, int width, int height, float *rgb);

/* Write interleaved float RGB (row stride `stride` floats, >= width*3) as a
 * FLOAT scanline EXR with the given compression (NONE or ZIP). */
int bmfr_exr_write_rgb(const char *path, int width, int height, const float *rgb, size_t stride,
                       bmfr_exr_compression compression);

/* Write interleaved float RGB as an 8-bit RGB PNG: each sample clamped to
 * [0, 1] and quantised to round(255 v) (OpenImageIO's FLOAT -> UINT8). */
int bmfr_png_write_rgb(const char *path, int width, int height, const float *rgb, size_t stride);

/* Last error message of this thread. */
const char *bmfr_io_error(void);

#ifdef __cplusplus
}
#endif
#endif /* BMFR_IMAGE_IO_H */
