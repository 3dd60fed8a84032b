"""Callbacks with the reference's interface (src/callbacks): the checkpoint
Monitor and the per-epoch loggers (TensorBoard when importable, else plain
files; rank 0 only)."""
from . import loggers
from .loggers import (AcdcMISRLogger, AcdcSISRLogger, AcdcSISRSRFBLogger, AcdcVSRLogger, BaseLogger, Dsb15MISRLogger,
                      Dsb15SISRLogger, Dsb15SISRSRFBLogger, Dsb15VSRLogger)
from .monitor import Monitor

__all__ = ["Monitor", "loggers", "BaseLogger", "AcdcSISRLogger", "AcdcSISRSRFBLogger", "AcdcMISRLogger",
           "AcdcVSRLogger", "Dsb15SISRLogger", "Dsb15SISRSRFBLogger", "Dsb15MISRLogger", "Dsb15VSRLogger"]
