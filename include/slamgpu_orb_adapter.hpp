// slamgpu_orb_adapter.hpp -- reference-side drop-in for ORBextractor (header only, OpenCV shell).
//
// Keeps the reference's class surface (src/orb_features/orb_extractor.h:25-93) so Frame,
// Tracker and src/core/* stay untouched. Everything that is not an OpenCV type conversion lives
// in slamgpu_adapter::OrbExtractorCore (slamgpu_adapters.hpp), which this repository compiles and
// tests without OpenCV (tests/adapter_check.cpp, tests/capi_check.cpp); this file only wraps
// cv::Mat / cv::KeyPoint around it and is compiled inside the reference's build (OpenCV is absent
// from this image).
#pragma once
#include <opencv2/core/core.hpp>

#include <vector>

#include "slamgpu_adapters.hpp"

namespace slamgpu_adapter {

static_assert(sizeof(cv::KeyPoint) == sizeof(slamgpu_keypoint), "cv::KeyPoint layout");

class ORBextractor {
 public:
  // Same ctor as orb_extractor.h:35-39; the device context is sized lazily per image size.
  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
               int device = 0)
      : core_(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device) {}

  // orb_extractor.cpp:985-1049: empty image -> outputs untouched; kps cleared and refilled;
  // desc N x 32 CV_8U, released when N == 0; mask ignored.
  void Compute(cv::InputArray _image, cv::InputArray /*mask*/, std::vector<cv::KeyPoint>& kps,
               cv::OutputArray _desc) {
    if (_image.empty()) return;
    cv::Mat image = _image.getMat();
    CV_Assert(image.type() == CV_8UC1);
    const int n = core_.Compute(image.data, image.rows, image.cols, image.step, kps_, desc_);
    kps.resize(n);
    if (n > 0) std::memcpy(kps.data(), kps_.data(), sizeof(slamgpu_keypoint) * n);
    if (n == 0) {
      _desc.release();
    } else {
      _desc.create(n, 32, CV_8U);
      std::memcpy(_desc.getMat().data, desc_.data(), (size_t)n * 32);
    }
    pyramid_valid_ = false;
  }

  int GetLevels() const { return core_.GetLevels(); }
  float GetScaleFactor() const { return core_.GetScaleFactor(); }
  std::vector<float> GetScaleFactors() const { return core_.GetScaleFactors(); }
  std::vector<float> GetInverseScaleFactors() const { return core_.GetInverseScaleFactors(); }
  std::vector<float> GetScaleSigmaSquares() const { return core_.GetScaleSigmaSquares(); }
  std::vector<float> GetInverseScaleSigmaSquares() const {
    return core_.GetInverseScaleSigmaSquares();
  }

  // orb_extractor.h:62 -- downloaded lazily, only when a caller (stereo matching on the CPU)
  // asks for it; slamgpu_frame_stereo keeps the whole stereo step on the device instead.
  const std::vector<cv::Mat>& GetImagePyramid() {
    if (!pyramid_valid_) {
      const std::vector<std::vector<uint8_t>>& levels = core_.GetImagePyramid();
      pyramid_.resize(levels.size());
      for (size_t l = 0; l < levels.size(); l++) {
        const std::pair<int, int> wh = core_.pyramid_size((int)l);
        pyramid_[l].create(wh.second, wh.first, CV_8U);
        std::memcpy(pyramid_[l].data, levels[l].data(), levels[l].size());
      }
      pyramid_valid_ = true;
    }
    return pyramid_;
  }

  slamgpu_ctx* context() { return core_.context(); }

 private:
  OrbExtractorCore core_;
  std::vector<slamgpu_keypoint> kps_;
  std::vector<uint8_t> desc_;
  bool pyramid_valid_ = false;
  std::vector<cv::Mat> pyramid_;
};

// OrbMatcher::DescriptorDistance (orb_matcher.cpp:1630-1646).
inline int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return slamgpu_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

}  // namespace slamgpu_adapter
