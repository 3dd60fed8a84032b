"""TEST INFRASTRUCTURE ONLY — import the reference's net files by path.

Runs only in the build container (where /root/reference exists).  The
reference package `src` cannot be imported whole (src/__init__.py:1-4 pulls
nibabel, SimpleITK, tensorboard and the unbuilt DCN extension), so stub
parent packages are registered and each hot-path module is loaded from its
file.  Nothing from the reference is copied into the repository.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

REF = os.environ.get("VSR_REFERENCE", "/root/reference")

_FILES = {
    "src.model.nets.base_net": "src/model/nets/base_net.py",
    "src.model.nets.edsr_net": "src/model/nets/edsr_net.py",
    "src.model.nets.duf_net": "src/model/nets/duf_net.py",
    "src.model.nets.drf_net": "src/model/nets/drf_net.py",
    "src.model.nets.drf_sisr_net": "src/model/nets/drf_sisr_net.py",
    "src.model.losses": "src/model/losses.py",
    "src.model.metrics": "src/model/metrics.py",
    "src.utils": "src/utils.py",
}


def available() -> bool:
    return os.path.isdir(os.path.join(REF, "src", "model", "nets"))


def load(name: str):
    """Load reference module `name` (a key of _FILES) without executing src/__init__.py."""
    sys.dont_write_bytecode = True  # the reference tree is read-only
    for pkg in ("src", "src.model", "src.model.nets"):
        if pkg not in sys.modules:
            m = types.ModuleType(pkg)
            m.__path__ = []
            sys.modules[pkg] = m
    if name in sys.modules and getattr(sys.modules[name], "__file__", None):
        return sys.modules[name]
    if name != "src.model.nets.base_net" and name.startswith("src.model.nets."):
        load("src.model.nets.base_net")
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, _FILES[name]))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod
