"""ptmi — MI355X (gfx950) path-tracing integrator.

Drop-in replacement for the hot loop of fakhirsh/path-tracer-python's Taichi
renderer (src/render_server/taichi_renderer): host surface in Python on
PyTorch-ROCm tensors, hot path in hand-written HIP behind the C-ABI of
include/ptmi.h (libptmi.so, built in-tree under ptmi/_lib/).
"""
__version__ = '0.1.0'
