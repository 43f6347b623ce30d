// Internal helpers shared by every translation unit of libsplatt3r_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include "s3_common.h"

namespace s3 {

// Thread-local last-error buffer behind s3_last_error().
void set_error(const char* fmt, ...);
void clear_error();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace s3

// Validate an argument; on failure record the message and return S3_ERR_INVALID.
#define S3_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      ::s3::set_error(__VA_ARGS__);           \
      return S3_ERR_INVALID;                  \
    }                                         \
  } while (0)

// Check a HIP runtime call.
#define S3_HIP(call)                                                        \
  do {                                                                      \
    hipError_t _e = (call);                                                 \
    if (_e != hipSuccess) {                                                 \
      ::s3::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,          \
                      hipGetErrorString(_e));                               \
      return S3_ERR_HIP;                                                    \
    }                                                                       \
  } while (0)

// Check the launch that was just issued.
#define S3_LAUNCH_CHECK() S3_HIP(hipGetLastError())
