/* multimot_track_amd/cli/mmt_io.h -- sequence input decoding for the rgbd_mmt drop-in
 * (SURVEY §8b "Drop-in CLI", §8f-2 input formats).  No OpenCV: PNG through zlib, Middlebury .flo,
 * and the semantic text masks, with the semantics of the reference's loader
 * (Examples/RGB-D/rgbd_tum.cc:122-131 main loop, LoadData :213-312, LoadMask :316-513).
 * Buffers returned through `void**` are malloc'd; release them with mmt_io_free. */
#ifndef MMT_IO_H
#define MMT_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cv::imread(path, IMREAD_UNCHANGED) for non-interlaced PNGs: gray / gray+alpha / RGB / RGBA,
 * 8 or 16 bits per sample.  Colour comes back in OpenCV order (BGR / BGRA); 16-bit samples in
 * host byte order.  *channels and *depth_bytes (1 or 2) describe the buffer (w*h*channels
 * samples, row-major, no padding).  0 on success, <0 on error (unsupported or corrupt file). */
int mmt_io_read_png(const char* path, int* w, int* h, int* channels, int* depth_bytes,
                    void** data);

/* cv::optflow::readOpticalFlow: Middlebury .flo (float tag 202021.25, int32 width, height, then
 * h*w*2 float32 u,v row-major).  0 on success. */
int mmt_io_read_flo(const char* path, int* w, int* h, float** data);

/* LoadMask (rgbd_tum.cc:316-513): one text line per image row with `cols` integers; labels
 * with tmp != 0 && tmp < 4 are kept, everything else becomes 0.  Rows missing from the file are
 * left untouched (the reference leaves the cv::Mat uninitialised there; the CLI zero-fills).
 * Returns the number of rows read, <0 on error. */
int mmt_io_read_mask(const char* path, int rows, int cols, int32_t* out);

/* LoadData's text files (rgbd_tum.cc:217-312).  times: one double per non-empty line.
 * poses: "id r00 ... r33" per line -> 16 floats each.  objects: 10 floats per line. */
int mmt_io_read_times(const char* path, double** out, int* n);
int mmt_io_read_poses(const char* path, float** out, int* n);
int mmt_io_read_object_poses(const char* path, float** out, int* n);

/* The `Key: value` scalars of an OpenCV FileStorage YAML settings file (kitti03.yaml). */
int mmt_io_yaml_float(const char* path, const char* key, double* value);

/* cv::imwrite(path, img) for an 8-bit BGR image (w*h*3, row-major, no padding): a PNG with RGB
 * samples, filter 0, zlib deflate.  0 on success. */
int mmt_io_write_png_bgr(const char* path, const uint8_t* bgr, int w, int h);

void mmt_io_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
