// image_io.cpp -- the ingest step before the hot path (include/slamgpu_io.h): KITTI's sequence
// listing (examples/main_stereo.cpp:16-49 LoadKittiImages) and an 8-bit PNG reader standing in
// for the reference's cv::imread(path, CV_LOAD_IMAGE_UNCHANGED) (:105-106), on zlib's inflate.
//
// PNG (ISO/IEC 15948): IHDR, optional PLTE / tRNS, IDAT chunks concatenated into one zlib
// stream, IEND. Each scanline starts with a filter byte (0 none, 1 sub, 2 up, 3 average,
// 4 Paeth) applied per byte with bpp = bytes per complete pixel (>= 1); Adam7 interlacing stores
// seven reduced images, each filtered on its own. cv::imread's channel order is BGR(A): colour
// samples are swapped on output; palette images expand to BGR (BGRA when tRNS is present) and
// gray + alpha to BGRA, as OpenCV 3.x's PNG decoder (grfmt_png.cpp) types them; gray images with
// fewer than 8 bits scale to 0..255 by bit replication (1-bit: 0 / 255), as libpng's
// png_set_expand_gray_1_2_4_to_8 does. Parity for the colour types KITTI does not use (palette,
// alpha, < 8 bits) rests on this recollection of OpenCV / libpng and is unpinned.
#include <zlib.h>

#include <algorithm>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/slamgpu_io.h"

namespace {

thread_local std::string t_err;

int fail(int rc, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  return rc;
}

// A chunk type for messages: its four letters, or hex when they are not printable ASCII.
std::string chunk_name(const uint8_t* t) {
  char buf[16];
  const bool letters = std::all_of(t, t + 4, [](uint8_t c) { return c >= 32 && c < 127; });
  if (letters) std::snprintf(buf, sizeof(buf), "%c%c%c%c", t[0], t[1], t[2], t[3]);
  else std::snprintf(buf, sizeof(buf), "0x%02x%02x%02x%02x", t[0], t[1], t[2], t[3]);
  return buf;
}

uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

struct Png {
  uint32_t w = 0, h = 0;
  int depth = 0, color = 0, interlace = 0;
  int out_channels = 0;  // cv::imread(UNCHANGED) channels
  int samples = 0;       // samples per pixel in the file
  std::vector<uint8_t> plte;   // RGB triples
  std::vector<uint8_t> trns;   // palette alpha
  std::vector<uint8_t> idat;
};

// Chunks of the file; with headers_only the IDAT data are not collected.
int parse(const uint8_t* d, size_t n, Png* p, bool headers_only) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (!d || n < 8 + 25 || std::memcmp(d, sig, 8) != 0)
    return fail(SLAMGPU_EINVAL, "not a PNG file");
  size_t off = 8;
  bool have_ihdr = false, have_iend = false;
  while (off + 12 <= n) {
    const uint32_t len = be32(d + off);
    const uint8_t* type = d + off + 4;
    const uint8_t* body = d + off + 8;
    if (len > n - off - 12) return fail(SLAMGPU_EINVAL, "PNG chunk overruns the file");
    const uint32_t crc = be32(body + len);
    if ((uint32_t)crc32(crc32(0L, Z_NULL, 0), type, len + 4) != crc)
      return fail(SLAMGPU_EINVAL, "PNG chunk %s: CRC mismatch", chunk_name(type).c_str());
    if (!have_ihdr) {
      if (std::memcmp(type, "IHDR", 4) != 0 || len != 13)
        return fail(SLAMGPU_EINVAL, "PNG: IHDR is not the first chunk");
      p->w = be32(body);
      p->h = be32(body + 4);
      p->depth = body[8];
      p->color = body[9];
      p->interlace = body[12];
      if (body[10] != 0 || body[11] != 0 || p->interlace > 1)
        return fail(SLAMGPU_EINVAL, "PNG: unknown compression / filter / interlace method");
      if (p->w == 0 || p->h == 0 || p->w > (1u << 24) || p->h > (1u << 24))
        return fail(SLAMGPU_EINVAL, "PNG: bad size %ux%u", p->w, p->h);
      switch (p->color) {
        case 0: p->samples = 1; p->out_channels = 1; break;  // gray
        case 2: p->samples = 3; p->out_channels = 3; break;  // RGB
        case 3: p->samples = 1; p->out_channels = 3; break;  // palette
        case 4: p->samples = 2; p->out_channels = 4; break;  // gray + alpha -> BGRA
        case 6: p->samples = 4; p->out_channels = 4; break;  // RGBA
        default: return fail(SLAMGPU_EINVAL, "PNG: colour type %d", p->color);
      }
      const bool ok_depth = p->depth == 8 || ((p->color == 0 || p->color == 3) &&
                                              (p->depth == 1 || p->depth == 2 || p->depth == 4));
      if (!ok_depth)
        return fail(SLAMGPU_EINVAL, "PNG: %d-bit samples of colour type %d are not supported "
                    "(8-bit images only)", p->depth, p->color);
      have_ihdr = true;
    } else if (std::memcmp(type, "PLTE", 4) == 0) {
      if (len % 3 || len > 768) return fail(SLAMGPU_EINVAL, "PNG: bad PLTE");
      p->plte.assign(body, body + len);
    } else if (std::memcmp(type, "tRNS", 4) == 0) {
      if (p->color == 3) p->trns.assign(body, body + len);
    } else if (std::memcmp(type, "IDAT", 4) == 0) {
      if (!headers_only) p->idat.insert(p->idat.end(), body, body + len);
    } else if (std::memcmp(type, "IEND", 4) == 0) {
      have_iend = true;
      break;
    } else if (!(type[0] & 0x20)) {
      return fail(SLAMGPU_EINVAL, "PNG: unknown critical chunk %s", chunk_name(type).c_str());
    }
    off += 12 + (size_t)len;
  }
  if (!have_ihdr) return fail(SLAMGPU_EINVAL, "PNG: no IHDR");
  if (p->color == 3) {
    if (p->plte.empty()) return fail(SLAMGPU_EINVAL, "PNG: palette image without PLTE");
    if (!p->trns.empty()) p->out_channels = 4;
  }
  if (!headers_only && !have_iend) return fail(SLAMGPU_EINVAL, "PNG: truncated (no IEND)");
  return 0;
}

uint8_t paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return (uint8_t)a;
  if (pb <= pc) return (uint8_t)b;
  return (uint8_t)c;
}

// Undoes the row filters of one (sub)image of `rows` scanlines of `rowbytes` bytes (+ 1 filter
// byte each) in place; out receives the unfiltered rows back to back.
int unfilter(const uint8_t* in, size_t rows, size_t rowbytes, int bpp, std::vector<uint8_t>* out) {
  out->assign(rows * rowbytes, 0);
  std::vector<uint8_t> zero(rowbytes, 0);
  for (size_t y = 0; y < rows; y++) {
    const uint8_t f = in[y * (rowbytes + 1)];
    const uint8_t* src = in + y * (rowbytes + 1) + 1;
    uint8_t* cur = out->data() + y * rowbytes;
    const uint8_t* prev = y ? out->data() + (y - 1) * rowbytes : zero.data();
    for (size_t x = 0; x < rowbytes; x++) {
      const int a = x >= (size_t)bpp ? cur[x - bpp] : 0, b = prev[x],
                c = x >= (size_t)bpp ? prev[x - bpp] : 0;
      int v = src[x];
      switch (f) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: return fail(SLAMGPU_EINVAL, "PNG: row filter %d", f);
      }
      cur[x] = (uint8_t)v;
    }
  }
  return 0;
}

// Sample k (0-based) of an unfiltered scanline with `depth`-bit samples.
inline int sample(const uint8_t* row, size_t k, int depth) {
  if (depth == 8) return row[k];
  const size_t bit = k * depth;
  return (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
}

// Writes pixel x of an unfiltered scanline to dst (cv::imread channel order).
inline void put_pixel(const Png& p, const uint8_t* row, size_t x, uint8_t* dst) {
  const int s = p.samples;
  switch (p.color) {
    case 0: {
      int v = sample(row, x, p.depth);
      if (p.depth < 8) v = v * 255 / ((1 << p.depth) - 1);  // bit replication == this scaling
      dst[0] = (uint8_t)v;
      break;
    }
    case 2:
      dst[0] = row[x * s + 2];
      dst[1] = row[x * s + 1];
      dst[2] = row[x * s];
      break;
    case 3: {
      const int i = sample(row, x, p.depth);
      const size_t n = p.plte.size() / 3;
      const uint8_t* c = (size_t)i < n ? &p.plte[3 * (size_t)i] : nullptr;
      dst[0] = c ? c[2] : 0;
      dst[1] = c ? c[1] : 0;
      dst[2] = c ? c[0] : 0;
      if (p.out_channels == 4) dst[3] = (size_t)i < p.trns.size() ? p.trns[i] : 255;
      break;
    }
    case 4:
      dst[0] = dst[1] = dst[2] = row[x * s];
      dst[3] = row[x * s + 1];
      break;
    case 6:
      dst[0] = row[x * s + 2];
      dst[1] = row[x * s + 1];
      dst[2] = row[x * s];
      dst[3] = row[x * s + 3];
      break;
  }
}

int decode(const uint8_t* data, size_t size, uint8_t* out, size_t pitch, size_t cap, int* wo,
           int* ho, int* co) {
  Png p;
  if (int r = parse(data, size, &p, false)) return r;
  if (wo) *wo = (int)p.w;
  if (ho) *ho = (int)p.h;
  if (co) *co = p.out_channels;
  const size_t row_out = (size_t)p.w * p.out_channels;
  if (!out) return 0;
  if (pitch < row_out || cap < pitch * (p.h - 1) + row_out)
    return fail(SLAMGPU_ECAP, "PNG %ux%ux%d: output buffer too small", p.w, p.h,
                p.out_channels);
  const int bits_pp = p.samples * p.depth, bpp = bits_pp >= 8 ? bits_pp / 8 : 1;
  // Adam7 passes (x0, y0, dx, dy); a single full pass when not interlaced
  static const int passes[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                   {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
  const int np = p.interlace ? 7 : 1;
  size_t raw_size = 0;
  std::vector<size_t> pw(np), ph(np);
  for (int k = 0; k < np; k++) {
    const int x0 = p.interlace ? passes[k][0] : 0, y0 = p.interlace ? passes[k][1] : 0;
    const int dx = p.interlace ? passes[k][2] : 1, dy = p.interlace ? passes[k][3] : 1;
    pw[k] = p.w > (uint32_t)x0 ? (p.w - x0 + dx - 1) / dx : 0;
    ph[k] = p.h > (uint32_t)y0 ? (p.h - y0 + dy - 1) / dy : 0;
    if (pw[k] && ph[k]) raw_size += ph[k] * (1 + (pw[k] * bits_pp + 7) / 8);
  }
  std::vector<uint8_t> raw(raw_size);
  uLongf got = (uLongf)raw_size;
  const int zr = uncompress(raw.data(), &got, p.idat.data(), (uLong)p.idat.size());
  if (zr != Z_OK || got != raw_size)
    return fail(SLAMGPU_EINVAL, "PNG: image data does not inflate to %zu bytes (zlib %d)",
                raw_size, zr);
  size_t off = 0;
  std::vector<uint8_t> rows;
  for (int k = 0; k < np; k++) {
    if (!pw[k] || !ph[k]) continue;
    const size_t rb = (pw[k] * bits_pp + 7) / 8;
    if (int r = unfilter(raw.data() + off, ph[k], rb, bpp, &rows)) return r;
    off += ph[k] * (rb + 1);
    const int x0 = p.interlace ? passes[k][0] : 0, y0 = p.interlace ? passes[k][1] : 0;
    const int dx = p.interlace ? passes[k][2] : 1, dy = p.interlace ? passes[k][3] : 1;
    for (size_t y = 0; y < ph[k]; y++) {
      uint8_t* dst_row = out + (y0 + y * dy) * pitch;
      const uint8_t* src = rows.data() + y * rb;
      for (size_t x = 0; x < pw[k]; x++)
        put_pixel(p, src, x, dst_row + (x0 + x * dx) * p.out_channels);
    }
  }
  return 0;
}

bool read_file(const char* path, std::vector<uint8_t>* buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  uint8_t tmp[1 << 16];
  size_t n;
  while ((n = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf->insert(buf->end(), tmp, tmp + n);
  const bool ok = !std::ferror(f);
  std::fclose(f);
  return ok;
}

}  // namespace

extern "C" {

const char* slamgpu_io_last_error(void) { return t_err.c_str(); }

int slamgpu_kitti_load_images(const char* kitti_path, double* timestamps, int cap,
                              int* n_frames) {
  if (!kitti_path || !n_frames || cap < 0) return fail(SLAMGPU_EINVAL, "bad arguments");
  *n_frames = 0;
  const std::string file = std::string(kitti_path) + "/times.txt";
  FILE* f = std::fopen(file.c_str(), "r");
  if (!f) return fail(SLAMGPU_EINVAL, "Error opening %s", file.c_str());
  char line[256];
  int n = 0;
  while (std::fgets(line, sizeof(line), f)) {
    // getline + `if (!s.empty()) stod(s)` (:24-31): a non-empty line that does not parse is an
    // error (std::stod throws), an empty one is skipped
    size_t len = std::strlen(line);
    while (len && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
    if (!len) continue;
    errno = 0;
    char* end = nullptr;
    const double t = std::strtod(line, &end);
    if (end == line || errno == ERANGE) {
      std::fclose(f);
      return fail(SLAMGPU_EINVAL, "%s: line %d is not a number", file.c_str(), n + 1);
    }
    if (timestamps && n < cap) timestamps[n] = t;
    n++;
  }
  std::fclose(f);
  *n_frames = n;
  return 0;
}

int slamgpu_kitti_image_path(const char* kitti_path, int camera, int index, char* out,
                             size_t cap) {
  if (!kitti_path || !out || index < 0 || camera < 0 || camera > 9)
    return fail(SLAMGPU_EINVAL, "bad arguments");
  const int n = std::snprintf(out, cap, "%s/image_%d/%06d.png", kitti_path, camera, index);
  if (n < 0 || (size_t)n >= cap) return fail(SLAMGPU_ECAP, "path needs %d bytes", n + 1);
  return 0;
}

int slamgpu_png_info(const uint8_t* data, size_t size, int* width, int* height, int* channels) {
  Png p;
  if (int r = parse(data, size, &p, true)) return r;
  if (width) *width = (int)p.w;
  if (height) *height = (int)p.h;
  if (channels) *channels = p.out_channels;
  return 0;
}

int slamgpu_png_decode(const uint8_t* data, size_t size, uint8_t* out, size_t out_pitch,
                       size_t out_cap, int* width, int* height, int* channels) {
  if (!out) return fail(SLAMGPU_EINVAL, "png_decode: no output buffer");
  return decode(data, size, out, out_pitch, out_cap, width, height, channels);
}

int slamgpu_imread_png(const char* path, uint8_t* out, size_t out_pitch, size_t out_cap,
                       int* width, int* height, int* channels) {
  std::vector<uint8_t> buf;
  if (!path || !read_file(path, &buf)) return fail(SLAMGPU_EINVAL, "cannot read %s", path ? path : "");
  if (!out) return slamgpu_png_info(buf.data(), buf.size(), width, height, channels);
  return decode(buf.data(), buf.size(), out, out_pitch, out_cap, width, height, channels);
}

}  // extern "C"
