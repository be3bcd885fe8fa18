"""GPU operator library: Python wrappers over the gfx950 kernels in csrc/kernels."""
