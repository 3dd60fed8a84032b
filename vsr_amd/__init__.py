"""vsr_amd — MI355X-native (gfx950) cardiac cine-MRI super-resolution train step.

The generators' forward/backward run as hand-written HIP kernels behind the C
ABI in include/vsrk.h (library: vsr_amd/_lib/libvsrk.so).
"""
__version__ = "0.1.0"
