"""Per-kernel stats (calls, total / average ms) from a rocprofv3 SQLite database
(rocprofv3 -d DIR writes run_results.db when no CSV output is requested)."""
import sqlite3
import sys


def stats(path, top=20):
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                      f"group by {name} order by sum(end - start) desc limit {top}").fetchall()
    return [(n, c, t / 1e6, a / 1e6) for n, c, t, a in rows]


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p)
        for n, c, t, a in stats(p):
            print(f"  {t:10.3f} ms  {c:6d} x {a:9.4f} ms  {n[:110]}")
