"""Per-case device ms (summed over a compress call's segment launches, averaged
over reps) of the kernels whose name contains PATTERN, for a kbench run of
NCASE cases x REPS reps.   python scripts/kdb_cases.py DB NCASE REPS PATTERN..."""
import collections
import sqlite3
import sys

db, ncase, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
pats = sys.argv[4:]
rows = sqlite3.connect(db).execute("select name, duration from kernels order by start").fetchall()
for pat in pats:
    ds = [d / 1e6 for n, d in rows if pat in n]
    per = len(ds) // (ncase * reps)
    out = []
    for c in range(ncase):
        seg = ds[c * reps * per:(c + 1) * reps * per]
        out.append(round(sum(seg) / reps, 2))
    print(pat, out)
