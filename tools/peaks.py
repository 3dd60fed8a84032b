"""Print this device's measured MFMA / HBM copy peaks (vsrk_peak_mfma /
vsrk_peak_copy via functional.measured_peaks); VSRK_LIB selects a build."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from vsr_amd import functional as F  # noqa: E402

print(json.dumps(F.measured_peaks(torch.device("cuda"))))
