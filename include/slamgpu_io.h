/* slamgpu_io.h -- the ingest step before the hot path: the KITTI
 * sequence listing of examples/main_stereo.cpp:16-49 (LoadKittiImages) and the image read of
 * :105-106 (cv::imread(path, CV_LOAD_IMAGE_UNCHANGED)) for 8-bit PNG files, on the host (zlib).
 * The decoded image goes to slamgpu_gray / slamgpu_gray_device (slamgpu_bow.h), the tracker's
 * cvtColor (tracker.cpp:110-127), then to the frame calls of slamgpu.h.
 *
 * C ABI: plain pointers and sizes, int status (0 ok, SLAMGPU_E* < 0), slamgpu_io_last_error()
 * for the message of the calling thread's last failure. */
#ifndef SLAMGPU_IO_H_
#define SLAMGPU_IO_H_

#include <stddef.h>
#include <stdint.h>

#include "slamgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

const char* slamgpu_io_last_error(void);

/* Replaces: LoadKittiImages(kitti_path, left_paths, right_paths, timestamps)
 * main_stereo.cpp:16-49. Reads kitti_path/times.txt: one timestamp per non-empty line (std::stod);
 * up to `cap` of them go to timestamps[] (may be NULL), *n_frames gets the count. Frame i's
 * images are slamgpu_kitti_image_path(kitti_path, 2 or 3, i). A missing times.txt is an error
 * (the reference prints it and continues with no frames). */
int slamgpu_kitti_load_images(const char* kitti_path, double* timestamps, int cap, int* n_frames);

/* "<kitti_path>/image_<camera>/<index as %06d>.png" into out (cap bytes, NUL-terminated);
 * camera 2 = left, 3 = right as the reference's stereo example uses them. */
int slamgpu_kitti_image_path(const char* kitti_path, int camera, int index, char* out, size_t cap);

/* PNG header of an in-memory file: width, height and the channel count cv::imread(...,
 * IMREAD_UNCHANGED) returns for it (1 gray, 3 colour or palette, 4 colour+alpha, gray+alpha or
 * palette+tRNS).
 * Only 8-bit samples (and palettes of 1/2/4/8-bit indices, gray of 1/2/4/8 bits) are supported:
 * 16-bit files give SLAMGPU_EINVAL. */
int slamgpu_png_info(const uint8_t* data, size_t size, int* width, int* height, int* channels);

/* Decodes an in-memory PNG (any of the five row filters, Adam7 or not) into out: height rows of
 * width * channels bytes, out_pitch bytes apart, channels in cv::imread order (BGR / BGRA for
 * colour, palettes expanded to BGR(A)); out_cap = bytes available at out. */
int slamgpu_png_decode(const uint8_t* data, size_t size, uint8_t* out, size_t out_pitch,
                       size_t out_cap, int* width, int* height, int* channels);

/* cv::imread(path, CV_LOAD_IMAGE_UNCHANGED) of a PNG file: slamgpu_png_decode of its bytes. With
 * out == NULL only the size and channels are returned. */
int slamgpu_imread_png(const char* path, uint8_t* out, size_t out_pitch, size_t out_cap,
                       int* width, int* height, int* channels);

#ifdef __cplusplus
}
#endif
#endif /* SLAMGPU_IO_H_ */
