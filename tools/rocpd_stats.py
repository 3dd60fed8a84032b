"""Summarise a rocprofv3 rocpd database (run_results.db): top kernels in ms per
step, like tools/kstats.py does for kernel_stats.csv.

    python tools/rocpd_stats.py DB STEPS [TOP] [--split N]

--split N cuts the dispatch timeline at its N-1 largest idle gaps (bench.py
runs its models one after another, with host-side set-up in between) and
prints one table per segment."""
import argparse
import re
import sqlite3
from collections import defaultdict


def table(rows, steps, top):
    tot = sum(r[2] - r[1] for r in rows)
    agg = defaultdict(lambda: [0, 0])
    for name, s, e in rows:
        agg[name][0] += e - s
        agg[name][1] += 1
    out = []
    for name, (ns, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        nm = re.sub(r"\(anonymous namespace\)::", "", name)
        out.append(f"{ns / 1e6 / steps:8.2f} ms/step {100 * ns / tot:6.2f}% n={n / steps:6.1f}/step "
                   f"avg={ns / n / 1e3:8.1f}us  {nm[:110]}")
    out.append(f"total {tot / 1e6 / steps:.2f} ms/step over {steps} steps")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("steps", type=float)
    ap.add_argument("top", type=int, nargs="?", default=25)
    ap.add_argument("--split", type=int, default=1)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])
    cuts = []
    if a.split > 1:
        gaps = sorted(((rows[i + 1][1] - rows[i][2], i + 1) for i in range(len(rows) - 1)), reverse=True)
        cuts = sorted(i for _, i in gaps[:a.split - 1])
    lo = 0
    for k, hi in enumerate(cuts + [len(rows)]):
        if a.split > 1:
            print(f"# segment {k + 1}: {hi - lo} dispatches")
        print(table(rows[lo:hi], a.steps, a.top))
        lo = hi


if __name__ == "__main__":
    main()
