"""Average duration of the dominant conv launches in a rocprofv3 kernel trace,
to cross-check bench.py's HIP-event `roofline.kernel_ms`.

A template instantiation (e.g. conv_fwd_kernel<bf16, NT=64, MS=2, KK=3, XM=0>)
serves several layer shapes.  For EDSR the dominant population is the 66
64->64 3x3 launches per step (33 forward, 33 data-gradient), 140-300 us each;
the same template's 64->256 up-convs (>= 600 us) and the 1-channel head
(~110 us) fall outside that band.

    python tools/trace_dominant.py run_kernel_trace.csv conv_fwd_kernelIDF16bLi64ELi2ELi3ELi0EDF16b 130 300 4
"""
import csv
import statistics
import sys

path, pat = sys.argv[1], sys.argv[2]
lo, hi = float(sys.argv[3]), float(sys.argv[4])
steps = float(sys.argv[5]) if len(sys.argv) > 5 else 1.0
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
     for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
sel = [x for x in d if lo <= x <= hi]
print(f"{len(d)} launches of *{pat}*; {len(sel)} in [{lo:g}, {hi:g}] us "
      f"({len(sel) / steps:.1f}/step): mean {statistics.mean(sel):.1f} us")
