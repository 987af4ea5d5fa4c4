"""Kernel timeline of a rocprofv3 rocpd database (--kernel-trace): per kernel name the count
and mean duration, and the mean gap before each kernel (end of the previous dispatch on the
same queue to this one's start) -- the launch boundaries of a step.
Usage: python tools/trace_gaps.py <results.db> [name-substring ...]"""
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
rows = db.execute("select * from kernels").fetchall()
ix = {c: i for i, c in enumerate(cols)}
name_col = "kernel_name" if "kernel_name" in ix else "name"
rows.sort(key=lambda r: r[ix["start"]])
dur = defaultdict(list)
gap = defaultdict(list)
prev_end = None
for r in rows:
    nm = r[ix[name_col]].split("(")[0][:60]
    st, en = r[ix["start"]], r[ix["end"]]
    dur[nm].append(en - st)
    if prev_end is not None and 0 <= st - prev_end < 50_000:
        gap[nm].append(st - prev_end)
    prev_end = en
flt = sys.argv[2:]
for nm, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    if flt and not any(f in nm for f in flt):
        continue
    g = gap.get(nm, [])
    print("%-60s n=%6d  dur %8.2f us  gap-before %6.2f us (n=%d)" % (
        nm, len(d), sum(d) / len(d) / 1e3, (sum(g) / len(g) / 1e3) if g else float("nan"), len(g)))
