"""Callbacks with the reference's interface (src/callbacks): the checkpoint
Monitor.  The TensorBoard loggers stay the reference's (rank 0 only)."""
from .monitor import Monitor

__all__ = ["Monitor"]
