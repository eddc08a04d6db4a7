/*
 * oracle/cv_semantics.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Restatement of the third-party primitives the reference hot path calls. None of these
 * dependencies is under /root/reference and none is installed in this image:
 *   - OpenCV 3.x (find_package(OpenCV 3.0 REQUIRED), CMakeLists.txt:44; ROS Kinetic => 3.3.1):
 *     cvRound, fastAtan2, resize(INTER_LINEAR, CV_8U), GaussianBlur(7x7, sigma 2, CV_8U),
 *     FAST(TYPE_9_16, nonmax). We restate the published 3.3.1 non-IPP C/SSE2 algorithms
 *     (SURVEY.md Appendix A); the SSE2 paths are bit-identical to the scalar ones except the
 *     GaussianBlur column rounding, which is reproduced per column range.
 *   - glibc 2.35 sinf/cosf, x86-64 FMA ifunc variant (called via std::cos(float)/std::sin(float)
 *     at orb_extractor.cpp:54). Algorithm and constants: the optimized-routines sincosf used by
 *     glibc >= 2.28; constants read from this host's libm rodata and verified bit-exactly over
 *     every float in [0, 2pi) by oracle/check_sincosf.c.
 * Compiled with -ffp-contract=off; every fused multiply-add is an explicit fma()/fmaf().
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

/* cvRound(float) on x86-64 = cvtss2si under the default MXCSR: round half to even. */
int oc_cv_round(float v) { return (int)lrintf(v); }

/* cv::fastAtan2 (OpenCV 3.3.1 core/src/mathfuncs_core.cpp atan_f32). Compiled at the SSE
 * baseline: no FMA. Coefficients are float products of the double constants with
 * (float)(180/CV_PI). */
float oc_fast_atan2(float y, float x) {
  const float k180pi = (float)(180.0 / 3.14159265358979323846);
  const float p1 = 0.9997878412794807f * k180pi;
  const float p3 = -0.3258083974640975f * k180pi;
  const float p5 = 0.1555786518463281f * k180pi;
  const float p7 = -0.04432655554792128f * k180pi;
  const float eps = (float)2.2204460492503131e-16; /* (float)DBL_EPSILON */
  float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

/* ---- glibc 2.35 sincosf (FMA variant) --------------------------------------------------- */
/* Table layout as in libm's __sincosf_table (two 14-double records, the second for
 * quadrants with n & 2): sign[4], hpi_inv (2/pi * 2^24), hpi, c0, c1, s1, c2, s2, c3, s3, c4. */
typedef struct {
  double sign[4];
  double hpi_inv, hpi;
  double c0, c1, s1, c2, s2, c3, s3, c4;
} sc_table;

static const sc_table kSinCos[2] = {
    {{1.0, -1.0, -1.0, 1.0},
     0x1.45f306dc9c883p+23,
     0x1.921fb54442d18p+0,
     0x1p+0,
     -0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3,
     0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7,
     -0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13,
     0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0},
     0x1.45f306dc9c883p+23,
     0x1.921fb54442d18p+0,
     -0x1p+0,
     0x1.ffffffd0c621cp-2,
     -0x1.555545995a603p-3,
     -0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7,
     0x1.6c087e89a359dp-10,
     -0x1.994eb3774cf24p-13,
     -0x1.99343027bf8c3p-16},
};

static inline uint32_t abstop12(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  return (u >> 20) & 0x7ff;
}

/* sinf_poly, odd branch: x already carries the quadrant sign. */
static inline float sc_sin_poly(double x, double x2, const sc_table* p) {
  double s1 = fma(x2, p->s3, p->s2);
  double x3 = x2 * x;
  double x7 = x2 * x3;
  double s = fma(x3, p->s1, x);
  return (float)fma(s1, x7, s);
}

static inline float sc_cos_poly(double x2, const sc_table* p) {
  double x4 = x2 * x2;
  double c1 = fma(x2, p->c1, p->c0);
  double c2 = fma(x2, p->c4, p->c3);
  double x6 = x2 * x4;
  double c = fma(x4, p->c2, c1);
  return (float)fma(c2, x6, c);
}

/* reduce_fast without TOINT intrinsics: n = ((int)(x * 2^24 * 2/pi) + 2^23) >> 24. */
static inline double sc_reduce(double x, int* np) {
  double r = x * kSinCos[0].hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fma(-(double)n, kSinCos[0].hpi, x);
}

float oc_sinf(float y) {
  double x = y;
  uint32_t top = abstop12(y);
  if (top < 0x3f4) { /* |y| < pi/4 */
    if (top < 0x398) return y;
    return sc_sin_poly(x, x * x, &kSinCos[0]);
  }
  if (top < 0x42f) { /* |y| < 120 */
    int n;
    double r = sc_reduce(x, &n);
    const sc_table* p = (n & 2) ? &kSinCos[1] : &kSinCos[0];
    if ((n & 1) == 0) return sc_sin_poly(r * kSinCos[0].sign[n & 3], r * r, p);
    return sc_cos_poly(r * r, p);
  }
  /* Large arguments never occur on the hot path (angles are in [0, 2pi)). */
  return (float)sin(x);
}

float oc_cosf(float y) {
  double x = y;
  uint32_t top = abstop12(y);
  if (top < 0x3f4) {
    if (top < 0x398) return 1.0f;
    return sc_cos_poly(x * x, &kSinCos[0]);
  }
  if (top < 0x42f) {
    int n;
    double r = sc_reduce(x, &n);
    const sc_table* p = (n & 2) ? &kSinCos[1] : &kSinCos[0];
    if (n & 1) return sc_sin_poly(r * kSinCos[0].sign[n & 3], r * r, p);
    return sc_cos_poly(r * r, p);
  }
  return (float)cos(x);
}

/* ---- resize INTER_LINEAR, CV_8U (OpenCV 3.3.1 imgproc/src/resize.cpp resizeGeneric_ with
 * HResizeLinear<uchar,int,short,2048> / VResizeLinear<...,FixedPtCast<int,uchar,22>>) ---- */
static inline short sat_short(float v) {
  int i = (int)lrintf(v);
  return (short)(i < -32768 ? -32768 : (i > 32767 ? 32767 : i));
}

void oc_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t sstep, uint8_t* dst, int dw,
                         int dh, size_t dstep) {
  const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
  const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
  int* xofs = (int*)malloc(sizeof(int) * dw);
  short* ialpha = (short*)malloc(sizeof(short) * 2 * dw);
  int xmax = dw;
  for (int dx = 0; dx < dw; dx++) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx); /* cvFloor */
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= sw) {
      if (dx < xmax) xmax = dx;
      if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
    }
    xofs[dx] = sx;
    ialpha[2 * dx] = sat_short((1.f - fx) * 2048);
    ialpha[2 * dx + 1] = sat_short(fx * 2048);
  }
  int* row0 = (int*)malloc(sizeof(int) * dw);
  int* row1 = (int*)malloc(sizeof(int) * dw);
  for (int dy = 0; dy < dh; dy++) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = (int)floorf(fy);
    fy -= sy;
    short b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
    /* clip(sy0 - ksize2 + 1 + k, 0, sh) for k = 0, 1 */
    int y0 = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);
    int y1 = sy + 1 < 0 ? 0 : (sy + 1 >= sh ? sh - 1 : sy + 1);
    const uint8_t* S0 = src + (size_t)y0 * sstep;
    const uint8_t* S1 = src + (size_t)y1 * sstep;
    for (int dx = 0; dx < dw; dx++) {
      int sx = xofs[dx];
      if (dx < xmax) {
        row0[dx] = S0[sx] * ialpha[2 * dx] + S0[sx + 1] * ialpha[2 * dx + 1];
        row1[dx] = S1[sx] * ialpha[2 * dx] + S1[sx + 1] * ialpha[2 * dx + 1];
      } else {
        row0[dx] = S0[sx] * 2048;
        row1[dx] = S1[sx] * 2048;
      }
    }
    uint8_t* D = dst + (size_t)dy * dstep;
    for (int x = 0; x < dw; x++)
      D[x] = (uint8_t)((((b0 * (row0[x] >> 4)) >> 16) + ((b1 * (row1[x] >> 4)) >> 16) + 2) >> 2);
  }
  free(row0);
  free(row1);
  free(xofs);
  free(ialpha);
}

/* ---- GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101), CV_8U -------------------------------
 * getGaussianKernel(7, 2, CV_32F) -> int kernel cvRound(k * 256) = {18,34,49,55,49,34,18}
 * (sum 257, not renormalised); row pass RowFilter<uchar,int> (exact ints); column pass
 * SymmColumnFilter<FixedPtCastEx<int,uchar>(16), SymmColumnVec_32s8u>: the SSE2 vector op
 * covers x < w - w%4 and rounds V/65536 half-to-even (float, exact here); the scalar tail
 * computes (V + 32768) >> 16. Both saturate to [0, 255]. */
static void gauss_kernel_int(int k[7]) {
  float cf[7];
  double sum = 0;
  const double sigma = 2.0, scale2X = -0.5 / (sigma * sigma);
  for (int i = 0; i < 7; i++) {
    double x = i - 3.0;
    cf[i] = (float)exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) {
    cf[i] = (float)(cf[i] * sum);
    k[i] = (int)lrint((double)cf[i] * 256.0);
  }
}

static inline int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

void oc_gaussian_blur7_u8(const uint8_t* src, int w, int h, size_t sstep, uint8_t* dst,
                          size_t dstep) {
  int k[7];
  gauss_kernel_int(k);
  int* H = (int*)malloc(sizeof(int) * (size_t)w * h);
  for (int y = 0; y < h; y++) {
    const uint8_t* S = src + (size_t)y * sstep;
    for (int x = 0; x < w; x++) {
      int s = 0;
      for (int i = 0; i < 7; i++) s += k[i] * S[reflect101(x + i - 3, w)];
      H[(size_t)y * w + x] = s;
    }
  }
  const int xvec = w - (w % 4);
  for (int y = 0; y < h; y++) {
    uint8_t* D = dst + (size_t)y * dstep;
    for (int x = 0; x < w; x++) {
      int v = k[3] * H[(size_t)y * w + x];
      for (int i = 1; i <= 3; i++)
        v += k[3 + i] * (H[(size_t)reflect101(y + i, h) * w + x] +
                         H[(size_t)reflect101(y - i, h) * w + x]);
      int r;
      if (x < xvec)
        r = (int)lrintf((float)v * (1.0f / 65536.0f));
      else
        r = (v + 32768) >> 16;
      D[x] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
  }
  free(H);
}

/* ---- FAST TYPE_9_16 (OpenCV 3.3.1 features2d/src/fast.cpp FAST_t<16>, cornerScore<16>) --- */
static void make_offsets16(int pixel[25], int step) {
  static const int off[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},   {3, -1},
                                 {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                 {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};
  int k = 0;
  for (; k < 16; k++) pixel[k] = off[k][0] + off[k][1] * step;
  for (; k < 25; k++) pixel[k] = pixel[k - 16];
}

static int corner_score16(const uint8_t* ptr, const int pixel[], int threshold) {
  const int K = 8, N = K * 3 + 1;
  int k, v = ptr[0];
  short d[25];
  for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
  int a0 = threshold;
  for (k = 0; k < 16; k += 2) {
    int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
    a = a < d[k + 3] ? a : d[k + 3];
    if (a <= a0) continue;
    for (int m = 4; m <= 8; m++) a = a < d[k + m] ? a : d[k + m];
    int t = a < d[k] ? a : d[k];
    a0 = a0 > t ? a0 : t;
    t = a < d[k + 9] ? a : d[k + 9];
    a0 = a0 > t ? a0 : t;
  }
  int b0 = -a0;
  for (k = 0; k < 16; k += 2) {
    int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
    for (int m = 3; m <= 5; m++) b = b > d[k + m] ? b : d[k + m];
    if (b >= b0) continue;
    for (int m = 6; m <= 8; m++) b = b > d[k + m] ? b : d[k + m];
    int t = b > d[k] ? b : d[k];
    b0 = b0 < t ? b0 : t;
    t = b > d[k + 9] ? b : d[k + 9];
    b0 = b0 < t ? b0 : t;
  }
  return -b0 - 1;
}

int oc_fast16(const uint8_t* img, int w, int h, size_t step, int threshold, int nonmax,
              oc_keypoint* out, int cap) {
  const int K = 8, N = 16 + K + 1;
  int pixel[25];
  make_offsets16(pixel, (int)step);
  threshold = threshold < 0 ? 0 : (threshold > 255 ? 255 : threshold);
  uint8_t tab[512];
  for (int i = -255; i <= 255; i++)
    tab[i + 255] = (uint8_t)(i < -threshold ? 1 : (i > threshold ? 2 : 0));
  uint8_t* buf[3];
  int* cpbuf[3];
  uint8_t* bufmem = (uint8_t*)calloc((size_t)3 * (w + 1), 1);
  int* cpmem = (int*)calloc((size_t)3 * (w + 2), sizeof(int));
  for (int i = 0; i < 3; i++) {
    buf[i] = bufmem + (size_t)i * (w + 1);
    cpbuf[i] = cpmem + (size_t)i * (w + 2) + 1;
  }
  int nout = 0;
  for (int i = 3; i < h - 2; i++) {
    const uint8_t* ptr = img + (size_t)i * step + 3;
    uint8_t* curr = buf[(i - 3) % 3];
    int* cornerpos = cpbuf[(i - 3) % 3];
    memset(curr, 0, w);
    int ncorners = 0;
    if (i < h - 3) {
      for (int j = 3; j < w - 3; j++, ptr++) {
        int v = ptr[0];
        const uint8_t* tb = &tab[0] - v + 255;
        int d = tb[ptr[pixel[0]]] | tb[ptr[pixel[8]]];
        if (d == 0) continue;
        d &= tb[ptr[pixel[2]]] | tb[ptr[pixel[10]]];
        d &= tb[ptr[pixel[4]]] | tb[ptr[pixel[12]]];
        d &= tb[ptr[pixel[6]]] | tb[ptr[pixel[14]]];
        if (d == 0) continue;
        d &= tb[ptr[pixel[1]]] | tb[ptr[pixel[9]]];
        d &= tb[ptr[pixel[3]]] | tb[ptr[pixel[11]]];
        d &= tb[ptr[pixel[5]]] | tb[ptr[pixel[13]]];
        d &= tb[ptr[pixel[7]]] | tb[ptr[pixel[15]]];
        if (d & 1) {
          int vt = v - threshold, count = 0;
          for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x < vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                if (nonmax) curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else
              count = 0;
          }
        }
        if (d & 2) {
          int vt = v + threshold, count = 0;
          for (int k = 0; k < N; k++) {
            int x = ptr[pixel[k]];
            if (x > vt) {
              if (++count > K) {
                cornerpos[ncorners++] = j;
                if (nonmax) curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                break;
              }
            } else
              count = 0;
          }
        }
      }
    }
    cornerpos[-1] = ncorners;
    if (i == 3) continue;
    const uint8_t* prev = buf[(i - 4 + 3) % 3];
    const uint8_t* pprev = buf[(i - 5 + 3) % 3];
    cornerpos = cpbuf[(i - 4 + 3) % 3];
    ncorners = cornerpos[-1];
    for (int k = 0; k < ncorners; k++) {
      int j = cornerpos[k];
      int score = prev[j];
      if (!nonmax || (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                      score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                      score > curr[j] && score > curr[j + 1])) {
        if (nout < cap) {
          oc_keypoint* kp = &out[nout];
          kp->x = (float)j;
          kp->y = (float)(i - 1);
          kp->size = 7.f;
          kp->angle = -1.f;
          kp->response = (float)score;
          kp->octave = 0;
          kp->class_id = -1;
        }
        nout++;
      }
    }
  }
  free(bufmem);
  free(cpmem);
  return nout;
}

/* ---- glibc 2.35 logf, x86-64 FMA ifunc variant (__logf_fma: sysdeps/ieee754/flt-32/e_logf.c
 * compiled with -mfma -mavx2). MapPoint::PredictScale calls std::log(float) (map_point.cpp:372).
 * Table and polynomial = __logf_data of this host's libm (16 {invc, logc} records, ln2, poly).
 * Pinned bit-exactly against host logf on every positive float (oracle/check_logf.c). */
static const double kLogfTab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
static const double kLogfLn2 = 0x1.62e42fefa39efp-1;
static const double kLogfPoly[3] = {-0x1.00ea348b88334p-2, 0x1.5575b0be00b6ap-2,
                                    -0x1.ffffef20a4123p-2};

float oc_logf(float x) {
  uint32_t ix;
  memcpy(&ix, &x, 4);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    /* x < 0x1p-126 or inf or nan */
    if (ix * 2 == 0) return -INFINITY;
    if (ix == 0x7f800000u) return x;
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return (x - x) / (x - x);
    const float xs = x * 0x1p23f; /* subnormal: normalise */
    memcpy(&ix, &xs, 4);
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> (23 - 4)) % 16);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  float zf;
  memcpy(&zf, &iz, 4);
  const double invc = kLogfTab[i][0], logc = kLogfTab[i][1], z = (double)zf;
  const double r = fma(z, invc, -1.0);
  const double y0 = fma((double)k, kLogfLn2, logc);
  const double r2 = r * r;
  double y = fma(kLogfPoly[1], r, kLogfPoly[2]);
  y = fma(kLogfPoly[0], r2, y);
  y = fma(y, r2, y0 + r);
  return (float)y;
}
