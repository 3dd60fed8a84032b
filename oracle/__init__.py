"""TEST INFRASTRUCTURE ONLY — the parity oracle.

CPU fp32 restatement of the reference's hot path (yangsenwxy/VSR) in stock
torch.nn, with the reference's module names so state_dicts interchange.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package; the product path (vsr_amd) never does.

Parity pinning: the reference has no golden vectors of its own,
so the restatement is pinned against the reference itself — oracle/make_golden.py
imports the reference net files by path in the build container, checks the
restatement bit-for-bit on fp32 CPU and writes small fixtures to tests/golden/.
"""
