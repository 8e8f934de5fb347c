"""Summarise rocprofv3 run_results.db files: per kernel name, calls and
min/median duration (ms).   python scripts/kdb.py gpurun_out/kp_*/run_results.db"""
import sqlite3
import statistics
import sys

for f in sys.argv[1:]:
    c = sqlite3.connect(f)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        rows.setdefault(name.replace("(anonymous namespace)::", "").split("(")[0][-60:], []).append(dur / 1e6)
    print(f)
    for k, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:60s} n={len(v):4d} min={min(v):8.3f} med={statistics.median(v):8.3f}")
