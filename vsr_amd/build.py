"""Builds the HIP kernels (gfx950) into the in-tree C-ABI library
``vsr_amd/_lib/libvsrk.so`` with plain ``hipcc`` (no torch headers involved:
the boundary is the C ABI declared in ``include/vsrk.h``)."""
from __future__ import annotations

import hashlib
import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
LIBDIR = ROOT / "_lib"
LIB = LIBDIR / "libvsrk.so"
INCLUDE = ROOT.parent / "include"
ARCH = os.environ.get("VSRK_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]
# Per-source extra flags.  The rolling convs: no SLP vectorisation -- it
# packed the BN prologue / epilogue into v_pk_fma_f32 with a v_mov per
# operand pair to marshal the packed registers (76 -> 28 v_mov per weight-
# gradient stage), and packed f32 VALU beside MFMAs costs more issue than the
# scalar form (MI355X_MICROARCH.md, cycle constants).
SRC_FLAGS = {"conv_roll.hip": ["-fno-slp-vectorize"], "conv_roll_fold.hip": ["-fno-slp-vectorize"],
             "conv_wgrad_roll.hip": ["-fno-slp-vectorize"]}


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _digest() -> str:
    h = hashlib.sha256()
    for p in sources() + sorted(CSRC.glob("*.h")) + sorted(INCLUDE.glob("*.h")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(FLAGS).encode())
    h.update(repr(sorted(SRC_FLAGS.items())).encode())
    return h.hexdigest()[:16]


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _includes(src: Path) -> list[Path]:
    """Local headers `src` includes, transitively, in a stable order."""
    seen: dict[Path, None] = {}
    todo = [src]
    while todo:
        cur = todo.pop()
        for name in _INC.findall(cur.read_text()):
            p = (cur.parent / name).resolve()
            if p.exists() and p not in seen:
                seen[p] = None
                todo.append(p)
    return sorted(seen)


def is_current() -> bool:
    """Whether libvsrk.so was built from the current sources and flags."""
    stamp = LIBDIR / "libvsrk.stamp"
    return LIB.exists() and stamp.exists() and stamp.read_text() == _digest()


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile every ``csrc/*.hip`` and link ``libvsrk.so``; skipped when the
    sources are unchanged since the last build (digest stamp)."""
    LIBDIR.mkdir(exist_ok=True)
    stamp = LIBDIR / "libvsrk.stamp"
    digest = _digest()
    if not force and LIB.exists() and stamp.exists() and stamp.read_text() == digest:
        return LIB
    objdir = LIBDIR / "obj"
    objdir.mkdir(exist_ok=True)

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        # per-object stamp: recompile only when this source, a header it
        # includes (transitively) or the flags changed
        deps = b"".join(p.read_bytes() for p in _includes(src))
        flags = FLAGS + SRC_FLAGS.get(src.name, [])
        key = hashlib.sha256(src.read_bytes() + deps + " ".join(flags).encode()).hexdigest()[:16]
        ostamp = objdir / (src.stem + ".stamp")
        if not force and obj.exists() and ostamp.exists() and ostamp.read_text() == key:
            return obj
        cmd = [HIPCC, *flags, "-I", str(INCLUDE), "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
        ostamp.write_text(key)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(sources()))) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", *[str(o) for o in objs], "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, LIB)
    stamp.write_text(digest)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
