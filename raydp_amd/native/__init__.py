"""In-tree native libraries (C++ runtime/executor kernels, gfx950 HIP kernels)."""
