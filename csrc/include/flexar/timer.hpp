// Timers (reference cost_model/timer.h:1-134: a std::chrono stopwatch in ms/us/ns/s).
// HostTimer: steady_clock stopwatch. DeviceTimer (HIP translation units only): hipEvent pair
// timing the work enqueued on a stream between start() and stop().
#pragma once

#include <chrono>

namespace flexar {

class HostTimer {
 public:
  HostTimer() { start(); }
  void start() { t0_ = std::chrono::steady_clock::now(); }
  double seconds() const { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count(); }
  double ms() const { return seconds() * 1e3; }
  double us() const { return seconds() * 1e6; }
  double ns() const { return seconds() * 1e9; }

 private:
  std::chrono::steady_clock::time_point t0_;
};

#if defined(__HIP_PLATFORM_AMD__) || defined(__HIPCC__)
}  // namespace flexar
#include <hip/hip_runtime.h>
namespace flexar {
class DeviceTimer {
 public:
  DeviceTimer() {
    (void)hipEventCreate(&a_);
    (void)hipEventCreate(&b_);
  }
  ~DeviceTimer() {
    (void)hipEventDestroy(a_);
    (void)hipEventDestroy(b_);
  }
  void start(hipStream_t s = nullptr) { (void)hipEventRecord(a_, s); }
  void stop(hipStream_t s = nullptr) { (void)hipEventRecord(b_, s); }
  double ms() {  // synchronises on the stop event
    float m = 0;
    (void)hipEventSynchronize(b_);
    (void)hipEventElapsedTime(&m, a_, b_);
    return m;
  }

 private:
  hipEvent_t a_, b_;
};
#endif

}  // namespace flexar
