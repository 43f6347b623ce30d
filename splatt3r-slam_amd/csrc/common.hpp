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

// Wave reduce-scatter of N <= 64 per-lane sums (padded to 64 slots): at
// offset o each lane keeps the half of its slots selected by lane bit o and
// adds its partner's copy of that half (63 shuffles in all, against N x 6
// for N separate butterflies).  Returns, in lane k < N, the wave total of
// acc[k] (the other lanes return 0 or a padding slot).
template <int N>
__device__ __forceinline__ float wave_reduce_scatter(const float (&acc)[N]) {
  static_assert(N <= 64, "at most 64 sums");
  const int lane = threadIdx.x & 63;
  float v[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) v[k] = k < N ? acc[k] : 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int j = 0; j < o; ++j) {
      const float keep = hi ? v[j + o] : v[j];
      const float send = hi ? v[j] : v[j + o];
      v[j] = keep + __shfl_xor(send, o, 64);
    }
  }
  return v[0];
}

// The barrier of an LDS-DMA ring (buffer_load ... lds into stages the waves
// read with ds_read).  s_barrier alone does not wait for this wave's LDS
// reads: one still in flight at the barrier could be overtaken by another
// wave's DMA refill of the same stage issued just after it (a rare, timing-
// dependent corruption of a few operands).  Drain them first.  One asm
// statement with a memory clobber also keeps the compiler from moving LDS
// reads across the barrier either way (__builtin_amdgcn_s_barrier is
// modelled as touching no memory).
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

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
