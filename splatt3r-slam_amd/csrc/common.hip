// ABI bookkeeping: last-error buffer, version and arch queries.
#include "common.hpp"
#include "device_util.hpp"
#include "host_wait.hpp"

#include <chrono>
#include <cstdlib>
#include <cstring>

namespace s3 {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

hipError_t wait_event_spin(hipEvent_t ev) {
  // the budget of the Python side's waits (splatt3r_amd/_lib.py wait_event)
  static const double budget_us = [] {
    const char* v = std::getenv("S3_SPIN_US");
    return v ? std::atof(v) : 1000.0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
    const double us =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (us > budget_us) return hipEventSynchronize(ev);
  }
}

}  // namespace s3

extern "C" const char* s3_last_error(void) { return s3::g_err; }
extern "C" int s3_abi_version(void) { return 1; }
extern "C" const char* s3_arch(void) { return "gfx950"; }

extern "C" int s3_stream_create(int device, int priority, void** out) {
  S3_REQUIRE(out, "s3_stream_create: null out");
  s3::DeviceGuard guard(device);
  int least = 0, greatest = 0;
  S3_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  const int pr = priority < greatest ? greatest : (priority > least ? least : priority);
  hipStream_t s = nullptr;
  S3_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, pr));
  *out = reinterpret_cast<void*>(s);
  return S3_OK;
}

extern "C" int s3_stream_destroy(void* stream) {
  if (stream) S3_HIP(hipStreamDestroy(s3::as_stream(stream)));
  return S3_OK;
}
