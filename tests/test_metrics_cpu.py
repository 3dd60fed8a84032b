"""Host-side metric plumbing: the Cardiac coordinates loader reads the
reference's pickle format without executing anything from the file."""
import json
import pickle

import pytest

from vsr_amd.metrics import _load_coordinates


class _Evil:
    def __reduce__(self):
        return (print, ("executed",))


def test_coordinates_plain_pickle_and_json(tmp_path):
    coords = {"patient001": (2, 17, 3, 20), "p2": [0, 5, 1, 9]}
    p = tmp_path / "c.pkl"
    p.write_bytes(pickle.dumps(coords))
    assert _load_coordinates(str(p)) == {"patient001": (2, 17, 3, 20), "p2": (0, 5, 1, 9)}
    j = tmp_path / "c.json"
    j.write_text(json.dumps({k: list(v) for k, v in coords.items()}))
    assert _load_coordinates(str(j)) == {"patient001": (2, 17, 3, 20), "p2": (0, 5, 1, 9)}


def test_coordinates_pickle_with_globals_is_refused(tmp_path):
    p = tmp_path / "evil.pkl"
    p.write_bytes(pickle.dumps({"x": _Evil()}))
    with pytest.raises(pickle.UnpicklingError):
        _load_coordinates(str(p))
