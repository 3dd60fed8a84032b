"""Summarise tools/ab.sh output (stdin or files): best-of-passes us per
(case, what) for each library, and the change of every library against the
first one listed."""
import collections
import re
import sys

rows = collections.defaultdict(list)
libs = []
src = [open(f) for f in sys.argv[1:]] or [sys.stdin]
for fh in src:
    for line in fh:
        m = re.match(r"\[(\S+)\]\s+(\S+)\s+(\S+)\s+([\d.]+) us", line)
        if m:
            lib, case, what, us = m.group(1), m.group(2), m.group(3), float(m.group(4))
            if lib not in libs:
                libs.append(lib)
            rows[(case, what, lib)].append(us)
for case, what in sorted({(c, w) for c, w, _ in rows}):
    base = rows.get((case, what, libs[0]))
    out = f"{case:10s} {what:9s}"
    for lib in libs:
        v = rows.get((case, what, lib))
        if not v:
            continue
        out += f"  {lib.split('/')[-2] if '/' in lib else lib}: {min(v):8.1f}"
        if lib != libs[0] and base:
            out += f" ({100 * (min(v) / min(base) - 1):+.1f}%)"
    print(out)
