"""splatt3r_amd — MI355X-native runtime for the Splatt3R-SLAM per-frame
inference-and-render path (HIP kernels in libsplatt3r_hip.so, C ABI in
include/*.h).  Drop-in modules live beside this package:
`diff_gaussian_rasterization`, `mast3r_slam_backends`, `lietorch`."""
