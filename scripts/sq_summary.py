"""Merge two rocprofv3 --pmc SQ passes of the same command into per-dispatch
records (per kernel, in dispatch order) with per-wave figures.

    python scripts/sq_summary.py PASS1_DIR PASS2_DIR [--kernels k_encode,k_dict] [--group N --labels a,b,c]

--group N: average every N consecutive dispatches of a kernel (e.g. the 4
pipelined segments of one ambc_compress_device call) and label the groups."""
import argparse
import collections
import csv
import json
import os


def load(d):
    per = collections.OrderedDict()
    for f in sorted(os.listdir(d)):
        if not f.endswith("counter_collection.csv"):
            continue
        with open(os.path.join(d, f)) as fh:
            for r in csv.DictReader(fh):
                key = (r["Kernel_Name"], int(r["Dispatch_Id"]))
                per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    out = collections.defaultdict(list)
    for (name, _), ctr in sorted(per.items(), key=lambda kv: kv[0][1]):
        out[name].append(ctr)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("p1")
    ap.add_argument("p2")
    ap.add_argument("--kernels", default="k_encode")
    ap.add_argument("--group", type=int, default=1)
    ap.add_argument("--labels", default="")
    a = ap.parse_args()
    d1, d2 = load(a.p1), load(a.p2)
    labels = a.labels.split(",") if a.labels else []
    res = {}
    for name in d1:
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("ambc::", "")
        if not any(k in short for k in a.kernels.split(",")):
            continue
        recs = [dict(x, **y) for x, y in zip(d1[name], d2.get(name, []))]
        groups = []
        for g in range(0, len(recs), a.group):
            part = recs[g:g + a.group]
            tot = {k: sum(r.get(k, 0.0) for r in part) for k in part[0]}
            w = max(tot.get("SQ_WAVES", 1.0), 1.0)
            per_wave = {k.replace("SQ_", "").lower(): round(v / w, 1) for k, v in tot.items() if k != "SQ_WAVES"}
            lab = labels[len(groups)] if len(groups) < len(labels) else str(len(groups))
            groups.append({"label": lab, "dispatches": len(part), "waves": int(w), "per_wave": per_wave})
        res[short] = groups
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
