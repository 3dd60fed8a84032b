"""Thin Python layer over the vsrk C ABI (include/vsrk.h).

Activations are channels-last tensors shaped (N, D, H, W, C) — 2-D feature
maps use D = 1 — in the compute dtype (bfloat16 or float32).  Every function
launches native HIP kernels on torch's current stream; none of them has a
CPU or PyTorch fallback.
"""
from __future__ import annotations

import os

import ctypes as C

import torch

from . import _native as N
from ._native import ACT_NONE, ACT_PRELU, ACT_RELU, PRO_AFFINE, PRO_AFFINE_RELU, PRO_NONE, PRO_RELU  # noqa: F401

__all__ = [
    "pack_weight", "conv", "conv_wgrad", "to_view", "from_view", "relu_bwd", "add",
    "loss_fwd", "loss_bwd", "psnr", "ssim", "workspace", "LOSS_KINDS",
    "bn_stats", "bn_finalize", "bn_fold_running", "bn_apply", "bn_relu_bwd_reduce", "bn_relu_bwd_apply",
    "duf_dynfilter_fwd", "duf_dynfilter_bwd",
    "subpixel_conv_weight", "subpixel_wgrad_fold", "prelu_wgrad", "prelu_bwd", "slope_slot_doubles",
    "slope_final_sum",
]

LOSS_KINDS = {"L1Loss": 0, "MSELoss": 1, "HuberLoss": 2, "CharbonnierLoss": 3}

_ws: dict[tuple[int, int], torch.Tensor] = {}


class KernelTimer:
    """Brackets selected native launches with HIP events on the launch stream
    (torch's current stream, where every vsrk kernel runs).  ``match(kind, xv,
    yv)`` sees the launch kind (("conv_fwd" | "conv_wgrad", (kd, kh, kw))) and
    its logical views (vsrk_tensor5: for a weight gradient the input and the
    output gradient) and returns the launch's algorithmic FLOP, or 0 to skip
    it.  Each timed launch is labelled by direction: "wgrad" for a weight
    gradient, else "fwd" or "dgrad" by ``phase``, which the caller sets to
    "fwd" before the forward and "bwd" before the backward.  Every conv entry point that can run
    a roofline kernel goes through ``wrap`` -- the plain conv, the fused conv +
    reduction (conv_reduce) and the fused conv + PReLU backward
    (conv_prelu_bwd) -- so a fused data gradient is timed like the unfused one.
    bench.py uses it for the roofline of the dominant conv.  Each launch also
    carries its algorithmic HBM bytes (``view_bytes`` of the operands it reads
    and writes once: x and y, plus the residual / mask / accumulate / BN-input
    operands the caller passes as ``extra``), so the roofline can price a
    launch at max(FLOP / MFMA peak, bytes / HBM peak) (``bound_seconds``)."""

    def __init__(self, match):
        self.match = match
        self.events: list[tuple[torch.cuda.Event, torch.cuda.Event, float, str, float, str]] = []
        self.enabled = True
        self.phase = "fwd"

    def wrap(self, kind, xv, yv, launch, launched=lambda rc: True, extra: float = 0.0):
        """launch() -> status; ``launched(status)`` False means nothing ran
        (a fused entry point reporting "not eligible"): the events are dropped."""
        flop = self.match(kind, xv, yv) if self.enabled else 0
        if not flop:
            return launch()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = launch()
        e.record()
        if launched(out):
            label = "wgrad" if kind[0] == "conv_wgrad" else ("dgrad" if self.phase == "bwd" else "fwd")
            self.events.append((s, e, float(flop), label, view_bytes(xv) + view_bytes(yv) + float(extra),
                                _launch_desc(kind, xv, yv)))
        return out

    def totals(self, label: str | None = None) -> tuple[float, float, int]:
        """(total FLOP, total seconds, launches) of the matched launches [of one direction]."""
        torch.cuda.synchronize()
        ev = [x for x in self.events if label is None or x[3] == label]
        t = sum(x[0].elapsed_time(x[1]) for x in ev) * 1e-3
        return sum(x[2] for x in ev), t, len(ev)

    def bound_seconds(self, mfma_peak: float, hbm_peak: float, label: str | None = None) -> tuple[float, float, float]:
        """(sum over launches of max(FLOP / mfma_peak, bytes / hbm_peak), the
        MFMA part of that sum, total bytes) -- the roofline time of the
        matched launches [of one direction]."""
        ev = [x for x in self.events if label is None or x[3] == label]
        tb = sum(max(x[2] / mfma_peak, x[4] / hbm_peak) for x in ev)
        tm = sum(x[2] / mfma_peak for x in ev if x[2] / mfma_peak >= x[4] / hbm_peak)
        return tb, tm, sum(x[4] for x in ev)

    def per_launch(self, steps: int, mfma_peak: float, hbm_peak: float) -> list[dict]:
        """The matched launches by position within a step (the step's launch
        order is fixed): mean time, FLOP, bytes, MFMA and bound fractions --
        the per-unit table of the roofline kernel.  [] if the launch count is
        not a multiple of ``steps``."""
        torch.cuda.synchronize()
        n = len(self.events)
        if steps <= 0 or n % steps:
            return []
        per = n // steps
        rows = []
        for i in range(per):
            ev = self.events[i::per]
            t = sum(x[0].elapsed_time(x[1]) for x in ev) * 1e-3 / len(ev)
            f, b = ev[0][2], ev[0][4]
            tb = max(f / mfma_peak, b / hbm_peak)
            rows.append({"pos": i, "dir": ev[0][3], "shape": ev[0][5], "us": t * 1e6, "gflop": f / 1e9,
                         "mb": b / 1e6, "frac": f / t / mfma_peak if t > 0 else None,
                         "hbm_frac": b / t / hbm_peak if t > 0 else None,
                         "bound_frac": tb / t if t > 0 else None})
        return rows

    def labels(self) -> list[str]:
        return [d for d in ("fwd", "dgrad", "wgrad") if any(x[3] == d for x in self.events)]

    def mean_ms(self) -> float:
        flop, t, n = self.totals()
        return t / n * 1e3 if n else float("nan")


timer: KernelTimer | None = None


def _launch_desc(kind, xv, yv) -> str:
    """Launch shape for the per-unit table: kernel taps, channels x depth of
    the input (weight gradient: the input and the output gradient) and output."""
    k = "x".join(str(i) for i in kind[1])
    return f"{k} {xv.c}x{xv.d}->{yv.c}x{yv.d} @{xv.n}x{xv.h}x{xv.w}"


def view_bytes(v) -> float:
    """Bytes of a logical view (vsrk_tensor5): voxels x channels x element size."""
    return float(v.n) * v.d * v.h * v.w * v.c * (4 if v.dtype == N.VSRK_F32 else 2)


_ws_kept: list = []


def workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    """A scratch buffer per (device, current stream): grown on demand, reused in
    stream order (the nets run weight gradients on a second stream, which
    gets its own)."""
    dev = device.index if device.index is not None else torch.cuda.current_device()
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        if buf is not None and torch.cuda.is_current_stream_capturing():
            # inside a graph capture a freed block can go to the next captured
            # allocation on another stream while this stream's kernels still
            # use it: the outgrown buffer is kept
            _ws_kept.append(buf)
        buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf


def _lib():
    return N.load()


def _kdims(w: torch.Tensor) -> tuple[int, int, int]:
    if w.dim() == 5:
        return tuple(w.shape[2:])
    if w.dim() == 4:
        return (1, w.shape[2], w.shape[3])
    raise ValueError(f"conv weight must be 4-D or 5-D, got {tuple(w.shape)}")


def pack_weight(w: torch.Tensor, mode: int, dtype: torch.dtype, perm_r: int = 1) -> torch.Tensor:
    """Repack an fp32 torch conv weight (cout, cin, [kd,] kh, kw) for the kernel.
    mode 0 = forward, mode 1 = data-gradient (transposed, flipped taps)."""
    lib = _lib()
    cout, cin = w.shape[:2]
    kd, kh, kw = _kdims(w)
    n = lib.vsrk_conv_packed_elems(cout, cin, kd, kh, kw, mode)
    out = torch.empty(n, dtype=dtype, device=w.device)
    wc = w.detach()
    if wc.dtype != torch.float32 or not wc.is_contiguous():
        wc = wc.float().contiguous()
    N.check(lib.vsrk_conv_pack_weight(N.dtype_code(dtype), wc.data_ptr(), cout, cin, kd, kh, kw, mode, perm_r,
                                      out.data_ptr(), N.stream_ptr(w.device)), "conv_pack_weight")
    return out


class WeightPacker:
    """All the packed conv weights of a step in one launch
    (vsrk_conv_pack_weights).  specs: [(weight, mode, perm_r), ...] of fp32
    torch conv weights; the packed buffers and the device descriptor table
    are allocated once and reused every step (the optimizer updates the
    weights in place; a moved weight rebuilds the table).  run() returns
    {(id(weight), mode, perm_r): packed tensor}."""

    def __init__(self, specs, dtype: torch.dtype):
        self.specs = [(w, int(m), int(r)) for w, m, r in specs]
        self.dtype = dtype
        self._ptrs = None

    def _build(self):
        lib = _lib()
        dev = self.specs[0][0].device
        descs = (N.PackDesc * len(self.specs))()
        self.out, self.max_elems = {}, 0
        for i, (w, m, r) in enumerate(self.specs):
            if w.dtype != torch.float32 or not w.is_contiguous():
                raise ValueError("WeightPacker needs contiguous fp32 weights")
            cout, cin = w.shape[:2]
            kd, kh, kw = _kdims(w)
            n = lib.vsrk_conv_packed_elems(cout, cin, kd, kh, kw, m)
            buf = torch.empty(n, dtype=self.dtype, device=dev)
            self.out[(id(w), m, r)] = buf
            self.max_elems = max(self.max_elems, n)
            descs[i] = N.PackDesc(w.data_ptr(), buf.data_ptr(), cout, cin, kd, kh, kw, m, r, 0)
        raw = torch.frombuffer(bytearray(C.string_at(C.addressof(descs), C.sizeof(descs))), dtype=torch.uint8)
        self.table = raw.to(dev)
        self._ptrs = tuple(w.data_ptr() for w, _, _ in self.specs)

    def run(self) -> dict:
        if self._ptrs != tuple(w.data_ptr() for w, _, _ in self.specs):
            self._build()
        N.check(_lib().vsrk_conv_pack_weights(N.dtype_code(self.dtype), len(self.specs), self.table.data_ptr(),
                                              self.max_elems, N.stream_ptr(self.table.device)), "conv_pack_weights")
        return self.out


def subpixel_code(k: int, s: int, p: int, transposed: bool, flipped: bool) -> int:
    """VSRK_SUBPIXEL (include/vsrk.h): the sub-pixel structure of a
    subpixel_conv_weight image packed with mode `flipped` (1 = data gradient)."""
    return k | (s << 8) | (p << 16) | ((1 << 24) if transposed else 0) | ((1 << 25) if flipped else 0)


def _desc(k, pad, prologue=PRO_NONE, act=ACT_NONE, out_scale=1.0, accumulate=False, bias_r=1,
          act_param=None, mask_slope=None, subpixel=0) -> N.ConvDesc:
    kd, kh, kw = k
    pd, ph, pw = pad
    return N.ConvDesc(kd, kh, kw, pd, ph, pw, prologue, act, float(out_scale), 1 if accumulate else 0, bias_r,
                      N.ptr(act_param), N.ptr(mask_slope), int(subpixel))


def conv(x: torch.Tensor, wp: torch.Tensor, y: torch.Tensor, k, pad, *, bias: torch.Tensor | None = None,
         prologue: int = PRO_NONE, pro_scale: torch.Tensor | None = None, pro_shift: torch.Tensor | None = None,
         act: int = ACT_NONE, out_scale: float = 1.0, accumulate: bool = False,
         residual: torch.Tensor | None = None, mask: torch.Tensor | None = None,
         x_shuffle: int = 1, y_shuffle: int = 1, act_param: torch.Tensor | None = None,
         mask_slope: torch.Tensor | None = None, bias_r: int | None = None, subpixel: int = 0) -> torch.Tensor:
    """y[...] = epilogue(conv(prologue(x), W) + bias); writes into the given y view.

    residual/mask are views with y's logical shape (and y_shuffle addressing).
    act=ACT_PRELU reads its slope from the device scalar act_param; with
    mask_slope the mask keeps mask_slope * value where mask <= 0 (PReLU
    backward) instead of zero (ReLU backward).  bias_r overrides the bias
    order (default: torch pixel-shuffle order of a y_shuffle output).
    subpixel: subpixel_code(...) of a subpixel_conv_weight image (its zero
    taps per phase may be skipped)."""
    lib = _lib()
    br = bias_r if bias_r is not None else (y_shuffle if bias is not None else 1)
    d = _desc(k, pad, prologue, act, out_scale, accumulate, br, act_param, mask_slope, subpixel)
    xv = N.t5(x, x_shuffle)
    yv = N.t5(y, y_shuffle)
    rv = N.t5(residual, y_shuffle) if residual is not None else None
    mv = N.t5(mask, y_shuffle) if mask is not None else None
    def launch():
        return lib.vsrk_conv_fwd(C.byref(d), C.byref(xv), wp.data_ptr(), N.ptr(bias), N.ptr(pro_scale),
                                 N.ptr(pro_shift), C.byref(rv) if rv is not None else None,
                                 C.byref(mv) if mv is not None else None, C.byref(yv), N.stream_ptr(x.device))

    if timer is not None:
        extra = (view_bytes(rv) if rv is not None else 0.0) + (view_bytes(mv) if mv is not None else 0.0) + (
            view_bytes(yv) if accumulate else 0.0)
        rc = timer.wrap(("conv_fwd", tuple(k)), xv, yv, launch, extra=extra)
    else:
        rc = launch()
    N.check(rc, "conv_fwd")
    return y


# A/B knob: VSRK_FUSE=0 makes the fused conv + reduction / PReLU-backward
# entry points report "not eligible", so the nets run the separate kernels
FUSE = os.environ.get("VSRK_FUSE", "1") != "0"


def _launched(rc) -> bool:
    return rc != 2  # VSRK_ERR_UNSUPPORTED: the fused entry point launched nothing


def conv_prelu_bwd(x: torch.Tensor, wp: torch.Tensor, y: torch.Tensor, k, pad, y_fwd: torch.Tensor,
                   a: torch.Tensor, da: torch.Tensor, accumulate_da: bool, *, x_shuffle: int = 1, y_shuffle: int = 1,
                   subpixel: int = 0, accumulate: bool = False, c_lo: int = 0,
                   slot: torch.Tensor | None = None) -> bool:
    """y = (conv(x) [+ y]) * (y_fwd > 0 ? 1 : a) on channels >= c_lo and da
    [+]= the PReLU slope gradient (vsrk_conv_fwd_prelu_bwd): conv [accumulate]
    followed by prelu_bwd(y_fwd, y, a, y, da) on y[..., c_lo:] in one kernel.
    False when the shape is not eligible (nothing launched).  slot: keep the
    slope partials there instead (see prelu_bwd; da unused)."""
    if not FUSE:
        return False
    lib = _lib()
    d = _desc(k, pad, accumulate=accumulate, mask_slope=a, subpixel=subpixel)
    xv, yv, mv = N.t5(x, x_shuffle), N.t5(y, y_shuffle), N.t5(y_fwd, y_shuffle)
    ws = slot if slot is not None else workspace(lib.vsrk_conv_prelu_bwd_workspace(), y.device)
    nbytes = ws.numel() * ws.element_size()

    def launch():
        return lib.vsrk_conv_fwd_prelu_bwd(C.byref(d), C.byref(xv), wp.data_ptr(), None, C.byref(mv), C.byref(yv),
                                           int(c_lo), None if slot is not None else da.data_ptr(),
                                           1 if accumulate_da else 0, ws.data_ptr(), nbytes, N.stream_ptr(y.device))

    rc = (timer.wrap(("conv_fwd", tuple(k)), xv, yv, launch, _launched,
                     extra=view_bytes(mv) + (view_bytes(yv) if accumulate else 0.0)) if timer is not None else launch())
    if rc == 2:  # VSRK_ERR_UNSUPPORTED
        return False
    N.check(rc, "conv_fwd_prelu_bwd")
    return True


def conv_reduce(x: torch.Tensor, wp: torch.Tensor, y: torch.Tensor, *, bias: torch.Tensor | None = None,
                prologue: int = PRO_NONE, pro_scale: torch.Tensor | None = None,
                pro_shift: torch.Tensor | None = None, bnx: torch.Tensor | None = None,
                st: torch.Tensor | None = None, k=(1, 1, 1), pad=(0, 0, 0)) -> torch.Tensor | None:
    """A 1x1x1 conv into y with a per-channel reduction of y fused into its
    store pass (vsrk_conv_fwd_reduce; k = (3, 3, 3): the data gradient of a
    Conv3d 3x3x3 on the rolling kernel, bnx form only): with a prologue (bnx None) the
    (sum, sumsq) statistics of y, as bn_stats(y); without, given the BN
    input bnx and its bn_finalize constants st, (sum dy', sum dy' xhat) of
    the BN+ReLU backward with dz = y, as bn_relu_bwd_reduce(bnx, y, st).
    -> (2, C) fp32, or None when the shape is not eligible (nothing was
    launched: the caller runs conv + the separate reduction)."""
    if not FUSE:
        return None
    lib = _lib()
    mode = 2 if bnx is not None else 1
    d = _desc(tuple(k), tuple(pad), prologue)
    c = y.shape[-1]
    out = torch.empty((2, c), dtype=torch.float32, device=y.device)
    xv, yv = N.t5(x), N.t5(y)
    ws = workspace(lib.vsrk_conv_fwd_reduce_workspace(C.byref(d), C.byref(yv)), y.device)
    bv = N.t5(bnx) if bnx is not None else None

    def launch():
        return lib.vsrk_conv_fwd_reduce(C.byref(d), C.byref(xv), wp.data_ptr(), N.ptr(bias), N.ptr(pro_scale),
                                        N.ptr(pro_shift), C.byref(yv), mode, C.byref(bv) if bv is not None else None,
                                        *(st[i].data_ptr() if st is not None else None for i in range(4)),
                                        out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(), ws.numel(),
                                        N.stream_ptr(y.device))

    rc = (timer.wrap(("conv_fwd", tuple(k)), xv, yv, launch, _launched,
                     extra=view_bytes(bv) if bv is not None else 0.0) if timer is not None else launch())
    if rc == 2:  # VSRK_ERR_UNSUPPORTED
        return None
    N.check(rc, "conv_fwd_reduce")
    return out


def conv_reduce_bnb(bn_x: torch.Tensor, dz: torch.Tensor, pst: torch.Tensor, gamma, pred: torch.Tensor,
                    count: float, x_out: torch.Tensor, wp: torch.Tensor, y: torch.Tensor, *, bnx: torch.Tensor,
                    st: torch.Tensor) -> torch.Tensor | None:
    """conv_reduce's BN+ReLU backward form (a square 1x1x1 data gradient into
    y, bnx / st the next BatchNorm's) whose input is the BN+ReLU backward
    apply of the previous BatchNorm, computed in the operand load
    (vsrk_conv_fwd_reduce_bnb): x_out receives
    bn_relu_bwd_apply(bn_x, dz, pst, gamma, pred, count) -- bitwise -- for
    the weight gradient.  y may be dz's storage.  -> (2, C) fp32 sums of y,
    or None when not eligible (nothing launched: apply + conv_reduce)."""
    if not FUSE:
        return None
    lib = _lib()
    d = _desc((1, 1, 1), (0, 0, 0), PRO_NONE)
    c = y.shape[-1]
    out = torch.empty((2, c), dtype=torch.float32, device=y.device)
    qv, ov, yv, bv = N.t5(bn_x), N.t5(x_out), N.t5(y), N.t5(bnx)
    pst, pred = pst.contiguous(), pred.contiguous()
    g = gamma.contiguous() if gamma is not None else None
    pre = N.BnContrib(N.t5(dz), 0, pst[0].data_ptr(), pst[1].data_ptr(), pst[2].data_ptr(), pst[3].data_ptr(),
                      N.ptr(g), pred[0].data_ptr(), pred[1].data_ptr(), float(count))
    ws = workspace(lib.vsrk_conv_fwd_reduce_workspace(C.byref(d), C.byref(yv)), y.device)

    def launch():
        return lib.vsrk_conv_fwd_reduce_bnb(C.byref(d), C.byref(qv), C.byref(pre), C.byref(ov), wp.data_ptr(),
                                            C.byref(yv), C.byref(bv), *(st[i].data_ptr() for i in range(4)),
                                            out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(), ws.numel(),
                                            N.stream_ptr(y.device))

    rc = (timer.wrap(("conv_fwd", (1, 1, 1)), N.t5(dz), yv, launch, _launched) if timer is not None else launch())
    if rc == 2:  # VSRK_ERR_UNSUPPORTED
        return None
    N.check(rc, "conv_fwd_reduce_bnb")
    return out


def conv_wgrad(x: torch.Tensor, dy: torch.Tensor, k, pad, dw: torch.Tensor, dbias: torch.Tensor | None = None, *,
               prologue: int = PRO_NONE, pro_scale: torch.Tensor | None = None,
               pro_shift: torch.Tensor | None = None, dy_scale: float = 1.0, perm_r: int = 1,
               accumulate: bool = False, x_shuffle: int = 1, dy_shuffle: int = 1, subpixel: int = 0) -> None:
    """dw (fp32, torch layout) [+]= dy_scale * dL/dW; dbias likewise.
    subpixel: subpixel_code(...) of the forward weight; only the taps that
    weight carries per phase are computed (the others come out zero)."""
    lib = _lib()
    d = _desc(k, pad, prologue, subpixel=subpixel)
    xv = N.t5(x, x_shuffle)
    gv = N.t5(dy, dy_shuffle)
    assert dw.dtype == torch.float32 and dw.is_contiguous()
    nbytes = lib.vsrk_conv_wgrad_workspace_size(C.byref(d), C.byref(xv), C.byref(gv))
    ws = workspace(nbytes, x.device)
    def launch():
        return lib.vsrk_conv_wgrad(C.byref(d), C.byref(xv), C.byref(gv), N.ptr(pro_scale), N.ptr(pro_shift),
                                   float(dy_scale), perm_r, dw.data_ptr(), N.ptr(dbias), 1 if accumulate else 0,
                                   ws.data_ptr(), ws.numel(), N.stream_ptr(x.device))

    rc = timer.wrap(("conv_wgrad", tuple(k)), xv, gv, launch) if timer is not None else launch()
    N.check(rc, "conv_wgrad")


def set_conv_path(path: str, mode: int) -> None:
    """Select a conv kernel family ("fast", "pw", "pw_wide", "roll", "roll_wr", "roll_fold", "thin", "wgrad_pipe",
    "wgrad_roll", "wgrad_row"):
    -1 default, 0 off, 1 on
    (for "roll" / "wgrad_roll": 1 forces the rolling kernel on every eligible
    shape, the default also skips shallow output depths where it is slower;
    "wgrad_row": 2 also takes the sub-pixel tap-skip views; "roll_wr": the
    rolling conv's resident weights, 2 also with the prefetched residual / mask
    epilogue, where they are slower)."""
    N.check(_lib().vsrk_conv_set_path(path.encode(), int(mode)), "conv_set_path")


def set_roll_depth(depths: int) -> None:
    """Test knob: output depths per tile of the rolling-depth Conv3d 3x3x3
    kernels, forward/dgrad and weight gradient (0 = automatic)."""
    N.check(_lib().vsrk_conv_set_roll_depth(int(depths)), "conv_set_roll_depth")


def set_grid_cap(max_workgroups: int) -> None:
    """Cap the persistent conv grids / wgrad split (0 = default); tests use it to
    run many tiles per workgroup at small shapes."""
    N.check(_lib().vsrk_conv_set_grid_cap(int(max_workgroups)), "conv_set_grid_cap")


def to_view(src: torch.Tensor, dtype: torch.dtype, cpad: int | None = None) -> torch.Tensor:
    """(N, C, [D,] H, W) fp32 -> channels-last (N, D, H, W, cpad) in dtype (zero padded).
    Slice [..., :C] of a padded result for a C-channel view the kernels can
    still read in whole 16-byte chunks."""
    lib = _lib()
    if src.dim() == 4:
        n, c, h, w = src.shape
        d = 1
    else:
        n, c, d, h, w = src.shape
    cp = cpad or c
    out = torch.empty((n, d, h, w, cp), dtype=dtype, device=src.device)
    s = src if (src.dtype == torch.float32 and src.is_contiguous()) else src.float().contiguous()
    v = N.t5(out)
    N.check(lib.vsrk_ncdhw_to_view(s.data_ptr(), n, c, d, h, w, C.byref(v), N.stream_ptr(src.device)),
            "ncdhw_to_view")
    return out


def from_view(v: torch.Tensor, c: int | None = None, two_d: bool = True) -> torch.Tensor:
    """channels-last (N, D, H, W, C) -> fp32 (N, C, H, W) (D must be 1 when two_d) or (N, C, D, H, W)."""
    lib = _lib()
    n, d, h, w, cc = v.shape
    c = c or cc
    shape = (n, c, h, w) if (two_d and d == 1) else (n, c, d, h, w)
    out = torch.empty(shape, dtype=torch.float32, device=v.device)
    tv = N.t5(v)
    N.check(lib.vsrk_view_to_ncdhw(C.byref(tv), out.data_ptr(), c, N.stream_ptr(v.device)), "view_to_ncdhw")
    return out


def relu_bwd(y: torch.Tensor, dy: torch.Tensor, dx: torch.Tensor) -> torch.Tensor:
    lib = _lib()
    a, b, c = N.t5(y), N.t5(dy), N.t5(dx)
    N.check(lib.vsrk_relu_bwd(C.byref(a), C.byref(b), C.byref(c), N.stream_ptr(y.device)), "relu_bwd")
    return dx


def add(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    lib = _lib()
    x, y, z = N.t5(a), N.t5(b), N.t5(out)
    N.check(lib.vsrk_add(C.byref(x), C.byref(y), C.byref(z), N.stream_ptr(a.device)), "add")
    return out


def loss_fwd(kind: int, param: float, out: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean-reduced loss of two fp32 tensors -> device scalar."""
    lib = _lib()
    assert out.dtype == torch.float32 and target.dtype == torch.float32
    o, t = out.contiguous(), target.contiguous()
    res = torch.empty((), dtype=torch.float32, device=out.device)
    nb = lib.vsrk_loss_workspace_size(o.numel())
    ws = torch.empty(nb, dtype=torch.uint8, device=out.device)
    N.check(lib.vsrk_loss_fwd(kind, float(param), o.data_ptr(), t.data_ptr(), o.numel(), res.data_ptr(),
                              ws.data_ptr(), nb, N.stream_ptr(out.device)), "loss_fwd")
    return res


def loss_bwd(kind: int, param: float, out: torch.Tensor, target: torch.Tensor, gscale: torch.Tensor | None,
             dtype: torch.dtype = torch.float32) -> torch.Tensor:
    lib = _lib()
    o, t = out.contiguous(), target.contiguous()
    g = torch.empty(o.shape, dtype=dtype, device=out.device)
    gs = gscale.float().contiguous() if gscale is not None else None
    N.check(lib.vsrk_loss_bwd(kind, float(param), o.data_ptr(), t.data_ptr(), o.numel(), N.ptr(gs), g.data_ptr(),
                              N.dtype_code(dtype), N.stream_ptr(out.device)), "loss_bwd")
    return g


def psnr(out: torch.Tensor, target: torch.Tensor, mean: float = 0.0, std: float = 1.0, max_value: float = 255.0,
         denormalize: bool = True):
    """[Denormalize (x*std+mean, round, clamp [0,255]) both,] per-sample PSNR;
    returns (batch mean, per-sample) as device tensors."""
    lib = _lib()
    o = out.float().contiguous()
    t = target.float().contiguous()
    b = o.shape[0]
    per = o.numel() // b
    ps = torch.empty(b, dtype=torch.float32, device=o.device)
    m = torch.empty((), dtype=torch.float32, device=o.device)
    nb = lib.vsrk_psnr_workspace_size(b, per)
    ws = torch.empty(nb, dtype=torch.uint8, device=o.device)
    N.check(lib.vsrk_psnr(o.data_ptr(), t.data_ptr(), b, per, 1 if denormalize else 0, float(mean), float(std),
                          float(max_value),
                          ps.data_ptr(), m.data_ptr(), ws.data_ptr(), nb, N.stream_ptr(o.device)), "psnr")
    return m, ps


def ssim(out: torch.Tensor, target: torch.Tensor, mean: float = 0.0, std: float = 1.0, value_range: float = 255.0,
         denormalize: bool = False):
    """SSIM of (N, C, H, W) images (2-D window) or (N, C, D, H, W) volumes
    (3-D window) ([denormalized] in the kernel); returns (batch mean,
    per-sample) as device tensors."""
    lib = _lib()
    if out.dim() == 5:
        o = out.float().contiguous()
        t = target.float().contiguous()
        b, c, d, h, w = o.shape
        ps = torch.empty(b, dtype=torch.float32, device=o.device)
        m = torch.empty((), dtype=torch.float32, device=o.device)
        nb = lib.vsrk_ssim3d_workspace_size(b, c, d, h, w)
        ws = torch.empty(nb, dtype=torch.uint8, device=o.device)
        N.check(lib.vsrk_ssim3d(o.data_ptr(), t.data_ptr(), b, c, d, h, w, 1 if denormalize else 0, float(mean),
                                float(std), float(value_range), ps.data_ptr(), m.data_ptr(), ws.data_ptr(), nb,
                                N.stream_ptr(o.device)), "ssim3d")
        return m, ps
    if out.dim() != 4:
        raise ValueError(f"ssim: expected (N, C, H, W) images or (N, C, D, H, W) volumes, got {tuple(out.shape)}")
    o = out.float().contiguous()
    t = target.float().contiguous()
    b, c, h, w = o.shape
    ps = torch.empty(b, dtype=torch.float32, device=o.device)
    m = torch.empty((), dtype=torch.float32, device=o.device)
    nb = lib.vsrk_ssim_workspace_size(b, c, h, w)
    ws = torch.empty(nb, dtype=torch.uint8, device=o.device)
    N.check(lib.vsrk_ssim(o.data_ptr(), t.data_ptr(), b, c, h, w, 1 if denormalize else 0, float(mean), float(std),
                          float(value_range), ps.data_ptr(), m.data_ptr(), ws.data_ptr(), nb,
                          N.stream_ptr(o.device)), "ssim")
    return m, ps


# ---------------------------------------------------------------- BatchNorm --
def _bn_ws(c: int, device) -> torch.Tensor:
    return workspace(_lib().vsrk_bn_workspace_size(c), device)


def bn_stats(x: torch.Tensor):
    """Per-channel (sum, sumsq) fp32 over every voxel of a channels-last view."""
    lib = _lib()
    c = x.shape[-1]
    out = torch.empty((2, c), dtype=torch.float32, device=x.device)
    xv = N.t5(x)
    ws = _bn_ws(c, x.device)
    N.check(lib.vsrk_bn_stats(C.byref(xv), out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(), ws.numel(),
                              N.stream_ptr(x.device)), "bn_stats")
    return out


def bn_stats_depth(x: torch.Tensor) -> torch.Tensor:
    """Per-depth per-channel (sum, sumsq) of a channels-last (N, D, H, W, C)
    view -> (D, 2, C) fp32.  One launch: rows are walked depth-major and each
    depth's partials are reduced on their own (vsrk_bn_stats_grouped)."""
    lib = _lib()
    d, c = x.shape[1], x.shape[-1]
    out = torch.empty((2, d, c), dtype=torch.float32, device=x.device)
    xv = N.t5(x.transpose(0, 1))  # n := depth, so depth d owns one contiguous run of rows
    ws = _bn_ws(c, x.device)
    N.check(lib.vsrk_bn_stats_grouped(C.byref(xv), d, out[0].data_ptr(), out[1].data_ptr(), ws.data_ptr(),
                                      ws.numel(), N.stream_ptr(x.device)), "bn_stats_grouped")
    return out.transpose(0, 1)


BN_MULTI_MAX = 8  # VSRK_BN_MULTI_MAX (more than 3: blocks of <= 256 channels)


def bn_relu_bwd_apply_multi(x: torch.Tensor, dx: torch.Tensor, accumulate: bool, contribs) -> torch.Tensor:
    """dx [+]= sum of up to BN_MULTI_MAX BN+ReLU backward applies over one block
    x (N, D, H, W, C): contribs = [(dz, d0, st, gamma, red, count), ...] with dz
    covering the block's depths [d0, d0 + dz.shape[1]), st / gamma / red already
    sliced to the block's channels (bn_finalize rows, BN weight, reduce sums)."""
    lib = _lib()
    if not 1 <= len(contribs) <= BN_MULTI_MAX:
        raise ValueError(f"1..{BN_MULTI_MAX} contributors")
    arr = (N.BnContrib * len(contribs))()
    keep = []
    for i, (dz, d0, st, gamma, red, count) in enumerate(contribs):
        st = st.contiguous()
        red = red.contiguous()
        keep += [st, red]
        arr[i] = N.BnContrib(N.t5(dz), int(d0), st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(),
                             st[3].data_ptr(), N.ptr(gamma.contiguous() if gamma is not None else None),
                             red[0].data_ptr(), red[1].data_ptr(), float(count))
        if gamma is not None:
            keep.append(gamma.contiguous())
            arr[i].gamma = keep[-1].data_ptr()
    xv, ov = N.t5(x), N.t5(dx)
    N.check(lib.vsrk_bn_relu_bwd_apply_multi(C.byref(xv), C.byref(ov), 1 if accumulate else 0, len(contribs), arr,
                                             N.stream_ptr(x.device)), "bn_relu_bwd_apply_multi")
    return dx


def bn_finalize(sums: torch.Tensor, count: float, gamma, beta, eps: float, momentum: float,
                running_mean=None, running_var=None, count_dev: torch.Tensor | None = None) -> torch.Tensor:
    """-> (4, C) fp32: scale, shift, mean, invstd (running stats updated in place).
    count_dev: a float64 device scalar; the voxel count is then count *
    count_dev, read by the kernel (no host synchronisation)."""
    lib = _lib()
    c = sums.shape[1]
    out = torch.empty((4, c), dtype=torch.float32, device=sums.device)
    if count_dev is not None:
        assert count_dev.dtype == torch.float64 and count_dev.device == sums.device
        N.check(lib.vsrk_bn_finalize_dcount(sums[0].data_ptr(), sums[1].data_ptr(), count_dev.data_ptr(),
                                            float(count), N.ptr(gamma), N.ptr(beta), float(eps), float(momentum),
                                            N.ptr(running_mean), N.ptr(running_var), out[0].data_ptr(),
                                            out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(), c,
                                            N.stream_ptr(sums.device)), "bn_finalize_dcount")
        return out
    N.check(lib.vsrk_bn_finalize(sums[0].data_ptr(), sums[1].data_ptr(), float(count), N.ptr(gamma), N.ptr(beta),
                                 float(eps), float(momentum), N.ptr(running_mean), N.ptr(running_var),
                                 out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(), out[3].data_ptr(), c,
                                 N.stream_ptr(sums.device)), "bn_finalize")
    return out


def bn_fold_running(gamma, beta, running_mean, running_var, eps: float) -> torch.Tensor:
    """eval mode -> (4, C): scale, shift, running mean, 1/sqrt(running var + eps)."""
    lib = _lib()
    c = running_mean.shape[0]
    out = torch.empty((4, c), dtype=torch.float32, device=running_mean.device)
    N.check(lib.vsrk_bn_fold_running(N.ptr(gamma), N.ptr(beta), running_mean.data_ptr(), running_var.data_ptr(),
                                     float(eps), out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr(),
                                     out[3].data_ptr(), c, N.stream_ptr(running_mean.device)), "bn_fold_running")
    return out


def bn_apply(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, relu: bool, y: torch.Tensor) -> torch.Tensor:
    """y = x * scale + shift [relu], per channel of channels-last views."""
    lib = _lib()
    xv, yv = N.t5(x), N.t5(y)
    N.check(lib.vsrk_bn_apply(C.byref(xv), scale.data_ptr(), shift.data_ptr(), 1 if relu else 0, C.byref(yv),
                              N.stream_ptr(x.device)), "bn_apply")
    return y


def bn_relu_bwd_reduce(x: torch.Tensor, dz: torch.Tensor, st: torch.Tensor) -> torch.Tensor:
    """-> (2, C): sum_dy (= dbeta), sum_dy_xhat (= dgamma); st from bn_finalize."""
    lib = _lib()
    c = x.shape[-1]
    out = torch.empty((2, c), dtype=torch.float32, device=x.device)
    xv, gv = N.t5(x), N.t5(dz)
    ws = _bn_ws(c, x.device)
    N.check(lib.vsrk_bn_relu_bwd_reduce(C.byref(xv), C.byref(gv), st[0].data_ptr(), st[1].data_ptr(),
                                        st[2].data_ptr(), st[3].data_ptr(), out[0].data_ptr(), out[1].data_ptr(),
                                        ws.data_ptr(), ws.numel(), N.stream_ptr(x.device)), "bn_relu_bwd_reduce")
    return out


def bn_relu_bwd_apply(x: torch.Tensor, dz: torch.Tensor, st: torch.Tensor, gamma, red: torch.Tensor,
                      count: float, dx: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    lib = _lib()
    xv, gv, ov = N.t5(x), N.t5(dz), N.t5(dx)
    N.check(lib.vsrk_bn_relu_bwd_apply(C.byref(xv), C.byref(gv), st[0].data_ptr(), st[1].data_ptr(),
                                       st[2].data_ptr(), st[3].data_ptr(), N.ptr(gamma), red[0].data_ptr(),
                                       red[1].data_ptr(), float(count), C.byref(ov), 1 if accumulate else 0,
                                       N.stream_ptr(x.device)), "bn_relu_bwd_apply")
    return dx


# ---------------------------------------------------------- DUF upsampling --
def duf_dynfilter_fwd(x: torch.Tensor, logits: torch.Tensor, residual: torch.Tensor, k: int, r: int) -> torch.Tensor:
    """x (n,h,w) fp32; logits (n,h,w,k*k*r*r) fp32; residual (n,h,w,r*r) fp32 -> (n,1,r*h,r*w) fp32."""
    lib = _lib()
    n, h, w = x.shape
    out = torch.empty((n, 1, h * r, w * r), dtype=torch.float32, device=x.device)
    N.check(lib.vsrk_duf_dynfilter_fwd(x.data_ptr(), logits.data_ptr(), residual.data_ptr(), n, h, w, k, r,
                                       out.data_ptr(), N.stream_ptr(x.device)), "duf_dynfilter_fwd")
    return out


def duf_dynfilter_bwd(x: torch.Tensor, logits: torch.Tensor, gout: torch.Tensor, k: int, r: int,
                      dtype: torch.dtype):
    """-> (d logits (n,h,w,k*k*r*r), d residual (n,h,w,r*r)) in dtype."""
    lib = _lib()
    n, h, w = x.shape
    dl = torch.empty((n, h, w, k * k * r * r), dtype=dtype, device=x.device)
    dr = torch.empty((n, h, w, r * r), dtype=dtype, device=x.device)
    g = gout.float().contiguous()
    N.check(lib.vsrk_duf_dynfilter_bwd(x.data_ptr(), logits.data_ptr(), g.data_ptr(), n, h, w, k, r, dl.data_ptr(),
                                       dr.data_ptr(), N.dtype_code(dtype), N.stream_ptr(x.device)),
            "duf_dynfilter_bwd")
    return dl, dr


# ------------------------------------------------------- DRF (sub-pixel, PReLU) --
def subpixel_conv_weight(w: torch.Tensor, bias: torch.Tensor | None, k: int, s: int, p: int, transposed: bool):
    """Equivalent 3x3 conv weight/bias (fp32, torch layout, view channel order)
    of nn.Conv2d / nn.ConvTranspose2d(k, stride s, padding p) on the sub-pixel grid."""
    lib = _lib()
    if transposed:
        cin, cout = w.shape[:2]
        weq = torch.empty((s * s * cout, cin, 3, 3), dtype=torch.float32, device=w.device)
        beq = torch.empty(s * s * cout, dtype=torch.float32, device=w.device)
    else:
        cout, cin = w.shape[:2]
        weq = torch.empty((cout, s * s * cin, 3, 3), dtype=torch.float32, device=w.device)
        beq = torch.empty(cout, dtype=torch.float32, device=w.device)
    wc = w.detach().float().contiguous()
    bc = bias.detach().float().contiguous() if bias is not None else None
    N.check(lib.vsrk_subpixel_conv_weight(wc.data_ptr(), N.ptr(bc), cin, cout, k, s, p, 1 if transposed else 0,
                                          weq.data_ptr(), beq.data_ptr(), N.stream_ptr(w.device)),
            "subpixel_conv_weight")
    return weq, beq


def subpixel_wgrad_fold(dweq: torch.Tensor, dbeq: torch.Tensor | None, dw: torch.Tensor, db: torch.Tensor | None,
                        k: int, s: int, p: int, transposed: bool, accumulate: bool = False) -> None:
    lib = _lib()
    if transposed:
        cin, cout = dw.shape[:2]
    else:
        cout, cin = dw.shape[:2]
    assert dw.dtype == torch.float32 and dw.is_contiguous()
    N.check(lib.vsrk_subpixel_wgrad_fold(dweq.data_ptr(), N.ptr(dbeq), cin, cout, k, s, p, 1 if transposed else 0,
                                         dw.data_ptr(), N.ptr(db), 1 if accumulate else 0, N.stream_ptr(dw.device)),
            "subpixel_wgrad_fold")


def prelu_wgrad(y: torch.Tensor, dx: torch.Tensor, a: torch.Tensor, da: torch.Tensor, accumulate: bool) -> None:
    """da [+]= sum_{y<0} dx * y / a^2 (nn.PReLU slope gradient from output and input gradient)."""
    lib = _lib()
    nb = lib.vsrk_prelu_workspace_size()
    ws = workspace(nb, y.device)
    yv, dv = N.t5(y), N.t5(dx)
    N.check(lib.vsrk_prelu_wgrad(C.byref(yv), C.byref(dv), a.data_ptr(), da.data_ptr(), 1 if accumulate else 0,
                                 ws.data_ptr(), ws.numel(), N.stream_ptr(y.device)), "prelu_wgrad")


def prelu_bwd(y: torch.Tensor, dy: torch.Tensor, a: torch.Tensor, dx: torch.Tensor, da: torch.Tensor | None,
              accumulate_da: bool, dy2: torch.Tensor | None = None, pre: bool = False,
              slot: torch.Tensor | None = None) -> torch.Tensor:
    """dx = (dy [+ dy2]) * (y > 0 ? 1 : a); da [+]= sum_{y<0} dx*y/a^2 (one
    pass) for the PReLU output y (exact while a > 0).  pre=True: y is the
    pre-activation x (vsrk_prelu_bwd_pre, any slope): dx = g (x > 0 ? 1 : a),
    da [+]= sum_{x<0} g x with g = dy [+ dy2].  slot: a zero-filled float64
    tensor of slope_slot_doubles() elements that keeps this call's slope
    partials instead (da unused; slope_final_sum later)."""
    lib = _lib()
    ws = slot if slot is not None else workspace(lib.vsrk_prelu_workspace_size(), y.device)
    nbytes = ws.numel() * ws.element_size()
    yv, gv, ov = N.t5(y), N.t5(dy), N.t5(dx)
    g2 = N.t5(dy2) if dy2 is not None else None
    fn = lib.vsrk_prelu_bwd_pre if pre else lib.vsrk_prelu_bwd
    N.check(fn(C.byref(yv), C.byref(gv), C.byref(g2) if g2 is not None else None, a.data_ptr(),
               C.byref(ov), None if slot is not None else da.data_ptr(), 1 if accumulate_da else 0, ws.data_ptr(),
               nbytes, N.stream_ptr(y.device)), "prelu_bwd_pre" if pre else "prelu_bwd")
    return dx


def slope_slot_doubles() -> int:
    """float64 elements of one deferred PReLU slope-partial slot."""
    return int(_lib().vsrk_slope_slot_doubles())


def slope_final_sum(part: torch.Tensor, a: torch.Tensor, da: torch.Tensor, accumulate: bool, pre: bool) -> None:
    """da [+]= the slope gradient of every deferred call whose slot lies in
    part (float64, zero-filled before the calls), summed in slot order."""
    N.check(_lib().vsrk_slope_final_sum(part.data_ptr(), part.numel(), a.data_ptr(), da.data_ptr(),
                                        1 if accumulate else 0, 1 if pre else 0, N.stream_ptr(part.device)),
            "slope_final_sum")


# ------------------------------------------------------------ device peaks --
def measured_peaks(device, mfma_iters: int = 20000, copy_bytes: int = 1 << 31, reps: int = 10) -> dict:
    """Measured ceilings of this device (vsrk_peak_mfma / vsrk_peak_copy):
    dense bf16 MFMA TFLOP/s on register operands and HBM copy TB/s (read +
    write bytes), each the best of `reps` timed launches after a warm-up."""
    lib = _lib()
    blocks = lib.vsrk_peak_mfma_blocks()
    out = torch.empty(blocks * 256, dtype=torch.float32, device=device)
    src = torch.empty(copy_bytes // 4, dtype=torch.float32, device=device).uniform_()
    dst = torch.empty_like(src)
    sp = N.stream_ptr(device)

    def best(fn):
        fn()
        t = []
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            t.append(s.elapsed_time(e) * 1e-3)
        return min(t)

    t_mfma = best(lambda: N.check(lib.vsrk_peak_mfma(mfma_iters, out.data_ptr(), sp), "peak_mfma"))
    t_copy = best(lambda: N.check(lib.vsrk_peak_copy(src.data_ptr(), dst.data_ptr(), copy_bytes, sp), "peak_copy"))
    flop = blocks * 4 * mfma_iters * 4 * 32768.0
    return {"mfma_bf16_tflops": flop / t_mfma / 1e12, "hbm_copy_tbs": 2.0 * copy_bytes / t_copy / 1e12,
            "method": f"v_mfma_f32_32x32x16_bf16 x{mfma_iters * 4} per wave, {blocks} x 4 waves; "
                      f"{copy_bytes >> 20} MiB device copy (read+write); best of {reps}"}
