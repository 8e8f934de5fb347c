"""Print gpurun_out/ab.log (scripts/ab_kbench.sh) as per-library, per-input encode times."""
import collections
import json
import sys

lib, r = None, collections.defaultdict(list)
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    if line.startswith("=="):
        lib = line.split()[-1]
    elif line.startswith("{"):
        d = json.loads(line)
        r[(d["input"], lib)].append(d["encode_ms"])
for k, v in sorted(r.items()):
    print(f"{k[0]:7s} {k[1]:22s} {v}")
