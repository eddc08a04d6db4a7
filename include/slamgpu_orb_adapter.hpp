// slamgpu_orb_adapter.hpp -- reference-side drop-in for the ORB hot path (header only).
//
// Keeps the reference's class surfaces so src/slam_system.cpp and src/core/* stay untouched:
//   ORBextractor (src/orb_features/orb_extractor.h:25-93) and the per-frame parts of
//   OrbMatcher / Frame. Every call forwards to the C ABI in slamgpu.h. This header needs OpenCV
//   (cv::Mat, cv::KeyPoint) and is compiled only inside the reference's build; it is not part of
//   this repository's own build (OpenCV is absent from this image).
#pragma once
#include <opencv2/core/core.hpp>

#include <stdexcept>
#include <string>
#include <vector>

#include "slamgpu.h"

namespace slamgpu_adapter {

static_assert(sizeof(cv::KeyPoint) == sizeof(slamgpu_keypoint), "cv::KeyPoint layout");

class ORBextractor {
 public:
  // Same ctor as orb_extractor.h:35-39; the device context is sized lazily per image size.
  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
               int device = 0)
      : params_{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST}, device_(device) {}
  ~ORBextractor() { slamgpu_destroy(ctx_); }
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // orb_extractor.cpp:985-1049: empty image -> outputs untouched; kps cleared and refilled;
  // desc N x 32 CV_8U, released when N == 0; mask ignored.
  void Compute(cv::InputArray _image, cv::InputArray /*mask*/, std::vector<cv::KeyPoint>& kps,
               cv::OutputArray _desc) {
    if (_image.empty()) return;
    cv::Mat image = _image.getMat();
    CV_Assert(image.type() == CV_8UC1);
    ensure(image.cols, image.rows);
    const int cap = slamgpu_kp_capacity(ctx_);
    kps.resize(cap);
    cv::Mat desc(cap, 32, CV_8U);
    int n = 0;
    check(slamgpu_extract(ctx_, image.data, image.step,
                          reinterpret_cast<slamgpu_keypoint*>(kps.data()), desc.data, cap, &n));
    kps.resize(n);
    if (n == 0) {
      _desc.release();
    } else {
      _desc.create(n, 32, CV_8U);
      desc.rowRange(0, n).copyTo(_desc.getMat());
    }
    pyramid_valid_ = false;
  }

  int GetLevels() const { return params_.nlevels; }
  float GetScaleFactor() const { return params_.scale_factor; }
  std::vector<float> GetScaleFactors() const { return table(0); }
  std::vector<float> GetInverseScaleFactors() const { return table(1); }
  std::vector<float> GetScaleSigmaSquares() const { return table(2); }
  std::vector<float> GetInverseScaleSigmaSquares() const { return table(3); }

  // orb_extractor.h:62 -- downloaded lazily, only when a caller (stereo matching on the CPU)
  // asks for it; slamgpu_frame_stereo keeps the whole stereo step on the device instead.
  const std::vector<cv::Mat>& GetImagePyramid() {
    if (!pyramid_valid_) {
      pyramid_.resize(params_.nlevels);
      for (int l = 0; l < params_.nlevels; l++) {
        int w = 0, h = 0;
        check(slamgpu_get_pyramid_level(ctx_, 0, l, nullptr, 0, &w, &h));
        pyramid_[l].create(h, w, CV_8U);
        check(slamgpu_get_pyramid_level(ctx_, 0, l, pyramid_[l].data, pyramid_[l].step, &w, &h));
      }
      pyramid_valid_ = true;
    }
    return pyramid_;
  }

  slamgpu_ctx* context() { return ctx_; }

 private:
  void ensure(int cols, int rows) {
    if (ctx_ && cols == cols_ && rows == rows_) return;
    slamgpu_destroy(ctx_);
    ctx_ = nullptr;
    check(slamgpu_create(device_, &params_, cols, rows, 1, &ctx_));
    cols_ = cols;
    rows_ = rows;
  }
  // the ctor tables do not depend on the image size: computed host-side, no device context
  std::vector<float> table(int which) const {
    std::vector<float> t(params_.nlevels);
    float* ptrs[4] = {nullptr, nullptr, nullptr, nullptr};
    ptrs[which] = t.data();
    check(slamgpu_orb_scale_tables(&params_, ptrs[0], ptrs[1], ptrs[2], ptrs[3], nullptr));
    return t;
  }
  void check(int rc) const {
    if (rc != SLAMGPU_OK)
      throw std::runtime_error(std::string("slamgpu: ") +
                               (ctx_ ? slamgpu_last_error(ctx_) : "invalid ORB parameters"));
  }

  slamgpu_orb_params params_;
  int device_;
  slamgpu_ctx* ctx_ = nullptr;
  int cols_ = 0, rows_ = 0;
  bool pyramid_valid_ = false;
  std::vector<cv::Mat> pyramid_;
};

// OrbMatcher::DescriptorDistance (orb_matcher.cpp:1630-1646).
inline int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return slamgpu_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

}  // namespace slamgpu_adapter
