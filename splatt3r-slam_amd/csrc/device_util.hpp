// Host helpers for entry points that take a caller's stream: the stream's
// device, and a scope that makes it current (allocations and events belong
// to the stream's device even when the caller's current device differs).
#pragma once
#include <hip/hip_runtime.h>

namespace s3 {

// The device a stream belongs to (the null stream: the current device).
inline hipError_t stream_device(hipStream_t st, int* dev) {
  if (!st) return hipGetDevice(dev);
  hipDevice_t d = 0;
  const hipError_t e = hipStreamGetDevice(st, &d);
  *dev = (int)d;
  return e;
}

// Makes `dev` current for its scope and restores the previous device.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace s3
