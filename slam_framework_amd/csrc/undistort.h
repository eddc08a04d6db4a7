// undistort.h -- cv::undistortPoints(src, dst, K, D, noArray(), K) on CV_32FC2 points, the call
// of Frame::UndistortKeyPoints (frame.cpp:614-641) and Frame::ComputeImageBounds (:644-675).
//
// OpenCV 3.3.1 cvUndistortPoints (imgproc/src/undistort.cpp), for the reference's arguments:
//   * K (CV_32F) and D (CV_32F, 4 or 5 coefficients k1 k2 p1 p2 [k3]) converted to double; every
//     further coefficient (k4..k6, s1..s4, tau) is 0;
//   * x = (u - cx) / fx as (u - cx) * (1./fx), same for y;
//   * the tilt compensation with tau = 0 is an exact identity (invMatTilt = I, 1/w = 1);
//   * 5 fixed-point iterations (iters = 5 whenever D is given):
//       r2 = x*x + y*y
//       icdist = (1 + ((k6*r2 + k5)*r2 + k4)*r2) / (1 + ((k3*r2 + k2)*r2 + k1)*r2)
//       deltaX = 2*p1*x*y + p2*(r2 + 2*x*x) + s1*r2 + s2*r2*r2
//       deltaY = p1*(r2 + 2*y*y) + 2*p2*x*y + s3*r2 + s4*r2*r2
//       x = (x0 - deltaX)*icdist;  y = (y0 - deltaY)*icdist
//   * RR = P * I = K: xx = fx*x + 0*y + cx, yy = 0*x + fy*y + cy, ww = 1./(0*x + 0*y + 1);
//   * the result rounded to float.
// All in IEEE double, no contraction (the library is built -ffp-contract=off, as the scalar
// OpenCV build of this loop has no FMA). Shared by the device kernel and the host entry point.
#pragma once
#include <hip/hip_runtime.h>

namespace slamgpu {

struct Distortion {
  float k[5];  // k1, k2, p1, p2, k3 (k3 = 0 for a 4-coefficient DistCoef)
};

__host__ __device__ inline void undistort_point(float fxf, float fyf, float cxf, float cyf,
                                                const Distortion& dc, float u, float v,
                                                float* uo, float* vo) {
  const double fx = fxf, fy = fyf, cx = cxf, cy = cyf;
  const double ifx = 1. / fx, ify = 1. / fy;
  const double k0 = dc.k[0], k1 = dc.k[1], k2 = dc.k[2], k3 = dc.k[3], k4 = dc.k[4];
  const double k5 = 0, k6 = 0, k7 = 0, k8 = 0, k9 = 0, k10 = 0, k11 = 0;
  double x = ((double)u - cx) * ifx;
  double y = ((double)v - cy) * ify;
  const double x0 = x, y0 = y;
  for (int j = 0; j < 5; j++) {
    const double r2 = x * x + y * y;
    const double icdist = (1 + ((k7 * r2 + k6) * r2 + k5) * r2) / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
    const double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x) + k8 * r2 + k9 * r2 * r2;
    const double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y + k10 * r2 + k11 * r2 * r2;
    x = (x0 - deltaX) * icdist;
    y = (y0 - deltaY) * icdist;
  }
  const double xx = fx * x + 0. * y + cx;
  const double yy = 0. * x + fy * y + cy;
  const double ww = 1. / (0. * x + 0. * y + 1.);
  *uo = (float)(xx * ww);
  *vo = (float)(yy * ww);
}

}  // namespace slamgpu
