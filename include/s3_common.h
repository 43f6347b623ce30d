/*
 * s3_common.h — shared conventions of the splatt3r-slam_amd C ABI.
 *
 * Every entry point of libsplatt3r_hip.so is `extern "C"`, takes plain
 * pointers + sizes (no torch types), runs asynchronously on the HIP stream
 * passed as `void* stream` (NULL = legacy default stream) and returns an
 * s3_status.  Device pointers are caller-owned; the library keeps no global
 * device state, so it is re-entrant per stream.  A non-zero status leaves a
 * human-readable message retrievable with s3_last_error() (thread-local).
 *
 * Reference boundary this ABI replaces: the pybind modules
 * `mast3r_slam_backends` (splatt3r_slam/backend/src/gn.cpp:116-122),
 * `diff_gaussian_rasterization` (external submodule, call sites
 * splatt3r_core/src/pixelsplat_src/cuda_splatting.py:100-125) and
 * `lietorch` (external submodule, call sites listed in SURVEY.md §8 A8).
 */
#ifndef S3_COMMON_H
#define S3_COMMON_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  S3_OK = 0,
  S3_ERR_INVALID = 1,   /* bad shape / argument (reference: TORCH_CHECK -> RuntimeError) */
  S3_ERR_HIP = 2,       /* HIP runtime error (launch failure, bad stream, ...) */
  S3_ERR_WORKSPACE = 3  /* caller workspace too small */
} s3_status;

/* Message of the last failing call on this thread ("" if none). */
const char* s3_last_error(void);

/* ABI version: bump on any signature change. */
int s3_abi_version(void);

/* Name of the offload architecture the library was built for ("gfx950"). */
const char* s3_arch(void);

/* A non-blocking HIP stream of the given priority (HIP numbering: 0 =
 * normal, negative = higher) on `device`, for the frame loop's dedicated
 * streams (splatt3r_amd/_lib.py frame_stream): the runtime hands every new
 * stream a hardware queue when it is created (GPU_MAX_HW_QUEUES per
 * priority, then shared), so streams created first, in a fixed order, get
 * queues of their own.  *out receives the hipStream_t. */
int s3_stream_create(int device, int priority, void** out);
int s3_stream_destroy(void* stream);

#ifdef __cplusplus
}
#endif
#endif /* S3_COMMON_H */
