// Timers (reference cost_model/timer.h:1-134: a std::chrono stopwatch in ms/us/ns/s).
// HostTimer: steady_clock stopwatch (bench/flexar_bench.cpp host-path timing). DeviceTimer: a hipEvent
// pair timing the work enqueued on a stream between start() and stop(); the FLEXAR_PROFILE per-call
// records of the communicator (comm.hip ProfRec) are DeviceTimers resolved by flexar_comm_stats.
#pragma once

#include <hip/hip_runtime_api.h>

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

class DeviceTimer {
 public:
  DeviceTimer() {
    if (hipEventCreate(&a_) != hipSuccess || hipEventCreate(&b_) != hipSuccess) ok_ = false;
  }
  ~DeviceTimer() {
    if (a_) (void)hipEventDestroy(a_);
    if (b_) (void)hipEventDestroy(b_);
  }
  DeviceTimer(const DeviceTimer&) = delete;
  DeviceTimer& operator=(const DeviceTimer&) = delete;
  bool ok() const { return ok_; }
  void start(hipStream_t s = nullptr) { ok_ = ok_ && hipEventRecord(a_, s) == hipSuccess; }
  void stop(hipStream_t s = nullptr) { ok_ = ok_ && hipEventRecord(b_, s) == hipSuccess; }
  // synchronises on the stop event; < 0 if an event could not be created / recorded
  double ms() {
    float m = 0;
    if (!ok_ || hipEventSynchronize(b_) != hipSuccess || hipEventElapsedTime(&m, a_, b_) != hipSuccess) return -1.0;
    return m;
  }

 private:
  hipEvent_t a_ = nullptr, b_ = nullptr;
  bool ok_ = true;
};

}  // namespace flexar
