"""Minimal NIfTI-1 reader / writer for the reference's on-disk format.

The reference reads its preprocessed volumes with nibabel
(``nib.load(path).get_data()``, src/data/datasets/acdc_*_dataset.py;
written by acdc_preprocess.py:55-85 as ``*_2d+1d_sequenceSS.nii.gz``, (H, W, 1, T)
float32).  nibabel is not installed here, so this module restates the part of
the NIfTI-1 format those files use: a 348-byte little- or big-endian header
(dim[8] int16 at byte 40, datatype int16 at 70, bitpix at 72, vox_offset
float32 at 108, scl_slope / scl_inter float32 at 112 / 116), the voxels from
vox_offset in Fortran (column-major) order, optional gzip.  ``get_data``
semantics: a nonzero scl_slope other than (1, 0) scales the data to float.
"""
from __future__ import annotations

import gzip
import struct
from pathlib import Path

import numpy as np

# NIfTI-1 datatype codes -> numpy dtypes (the ones medical volumes use)
_DTYPES = {2: np.uint8, 4: np.int16, 8: np.int32, 16: np.float32, 64: np.float64, 256: np.int8, 512: np.uint16,
           768: np.uint32, 1024: np.int64, 1280: np.uint64}
_CODES = {np.dtype(v): k for k, v in _DTYPES.items()}


def _open(path: Path, mode: str):
    return gzip.open(path, mode) if str(path).endswith(".gz") else open(path, mode)


class NiftiImage:
    """What the datasets use of nibabel's image: ``header.get_data_shape()``
    and ``get_data()`` (nib.load(...).get_data() in the reference)."""

    def __init__(self, path):
        self.path = Path(path)
        with _open(self.path, "rb") as f:
            raw = f.read()
        if len(raw) < 348:
            raise ValueError(f"{path}: not a NIfTI-1 file (short header)")
        endian = "<" if struct.unpack("<i", raw[:4])[0] == 348 else ">"
        if struct.unpack(endian + "i", raw[:4])[0] != 348:
            raise ValueError(f"{path}: not a NIfTI-1 file (sizeof_hdr != 348)")
        dim = struct.unpack(endian + "8h", raw[40:56])
        ndim = dim[0]
        if not 1 <= ndim <= 7:
            raise ValueError(f"{path}: bad dim[0] = {ndim}")
        self.shape = tuple(int(d) for d in dim[1:1 + ndim])
        code = struct.unpack(endian + "h", raw[70:72])[0]
        if code not in _DTYPES:
            raise ValueError(f"{path}: unsupported NIfTI datatype {code}")
        self.dtype = np.dtype(_DTYPES[code]).newbyteorder(endian)
        self.vox_offset = int(struct.unpack(endian + "f", raw[108:112])[0])
        self.scl_slope, self.scl_inter = struct.unpack(endian + "2f", raw[112:120])
        self._raw = raw

    class _Header:
        def __init__(self, shape):
            self._shape = shape

        def get_data_shape(self):
            return self._shape

    @property
    def header(self):
        return NiftiImage._Header(self.shape)

    def get_data(self) -> np.ndarray:
        n = int(np.prod(self.shape))
        data = np.frombuffer(self._raw, dtype=self.dtype, count=n, offset=self.vox_offset)
        data = data.reshape(self.shape, order="F").astype(self.dtype.newbyteorder("="))
        if self.scl_slope not in (0.0, 1.0) or (self.scl_slope == 1.0 and self.scl_inter != 0.0):
            data = data.astype(np.float64) * self.scl_slope + self.scl_inter
        return data

    get_fdata = get_data


def load(path) -> NiftiImage:
    """nib.load for NIfTI-1 single files (.nii / .nii.gz)."""
    return NiftiImage(path)


def save(arr: np.ndarray, path, pixdim=None) -> None:
    """Write arr as a single-file NIfTI-1 (.nii or .nii.gz), Fortran order,
    identity scaling -- the layout acdc_preprocess.py writes with
    nib.save(nib.Nifti1Image(img, affine), path)."""
    arr = np.asarray(arr)
    if arr.dtype not in _CODES:
        raise ValueError(f"unsupported dtype {arr.dtype}")
    if not 1 <= arr.ndim <= 7:
        raise ValueError("1 to 7 dimensions")
    hdr = bytearray(352)  # 348-byte header + 4-byte extension flag
    struct.pack_into("<i", hdr, 0, 348)
    dim = [arr.ndim] + list(arr.shape) + [1] * (7 - arr.ndim)
    struct.pack_into("<8h", hdr, 40, *dim)
    struct.pack_into("<h", hdr, 70, _CODES[arr.dtype])
    struct.pack_into("<h", hdr, 72, arr.dtype.itemsize * 8)
    pd = [1.0] + list(pixdim or [1.0] * arr.ndim) + [1.0] * (7 - arr.ndim)
    struct.pack_into("<8f", hdr, 76, *pd[:8])
    struct.pack_into("<f", hdr, 108, 352.0)  # vox_offset
    struct.pack_into("<2f", hdr, 112, 1.0, 0.0)  # scl_slope, scl_inter
    struct.pack_into("<4s", hdr, 344, b"n+1\x00")  # magic: single file
    body = np.asfortranarray(arr).astype(arr.dtype.newbyteorder("<")).tobytes(order="F")
    with _open(Path(path), "wb") as f:
        f.write(bytes(hdr) + body)
