"""Print the kernel timeline of one compress step from a rocprofv3 kernel trace.

    python scripts/trace_step.py gpurun_out/prof_q/run_kernel_trace.csv [step_from_end]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
enc = [i for i, r in enumerate(rows) if "k_encode" in r["Kernel_Name"]]
first = enc[-4 * back]
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first:first + 40]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if s > 40:
        break
    print(f"{r['Kernel_Name'][:44]:46s} q{r['Queue_Id']:3s} {s:8.3f} {e:8.3f} {e - s:7.3f}")
