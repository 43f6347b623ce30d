// Host-side waits shared by the C-ABI entry points (definition in common.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace s3 {
// Host wait for a recorded event: polled (no blocking wake-up latency) for
// up to S3_SPIN_US microseconds (default 1000), then a blocking synchronize.
hipError_t wait_event_spin(hipEvent_t ev);
}  // namespace s3
