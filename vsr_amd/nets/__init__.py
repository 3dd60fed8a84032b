"""Generators resolvable by name, as src.model.nets is in the reference
(main.py:56 `_get_instance(src.model.nets, config.net)`)."""
from .base_net import BaseNet
from .drf_net import DRFNet, DRFSISRNet
from .duf_net import DUFNet
from .edsr_net import EDSRNet

__all__ = ["BaseNet", "EDSRNet", "DUFNet", "DRFNet", "DRFSISRNet"]
