"""Summarise rocprofv3 runs of bench.py into profiles/ (per round).

    python scripts/pmc_summary.py --round r1 --stats DIR --fetch DIR --write DIR --bench JSON

* kernel stats: copies <stats>/run_kernel_stats.csv to profiles/<round>_kernel_stats.csv
* HBM traffic of k_encode per launch from the two PMC passes (FETCH_SIZE and
  WRITE_SIZE cannot share a pass on gfx950), with the MI355X_MICROARCH.md
  correction: FETCH_SIZE counts half the bytes of 16-B-per-lane streaming
  reads, so it is doubled.  Round 5 calibrated the other widths the encoder
  uses (profiles/r5_pmc_calibration.json, scripts/pmc_calib.hip): every read
  reaches EA as 128-B requests, which FETCH_SIZE's expression counts as 64 B
  (its TCC_BUBBLE term stays 0 on gfx950), so the doubling holds for dword,
  byte and unaligned reads too; WRITE_SIZE is exact (+2 % for byte stores)
  and taken as is.  Both counters are in KiB.
  -> profiles/pmc_<round>.json (read by bench.py for roofline.traffic)
"""
import argparse
import csv
import json
import os
import shutil
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(d, name, kernel="k_encode"):
    vals = []
    for f in os.listdir(d):
        if f.endswith("counter_collection.csv"):
            with open(os.path.join(d, f)) as fh:
                for r in csv.DictReader(fh):
                    if r["Counter_Name"] == name and kernel + "<" in r["Kernel_Name"]:
                        vals.append(float(r["Counter_Value"]))
    return vals


def kernel_totals(d, name):
    """sum of a counter per kernel name over every dispatch of the run"""
    tot = {}
    for f in os.listdir(d):
        if f.endswith("counter_collection.csv"):
            with open(os.path.join(d, f)) as fh:
                for r in csv.DictReader(fh):
                    if r["Counter_Name"] == name:
                        tot[r["Kernel_Name"]] = tot.get(r["Kernel_Name"], 0.0) + float(r["Counter_Value"])
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench")
    ap.add_argument("--req", help="pass with TCC_EA0_RDREQ_{32B,64B,128B}_sum: EA read bytes per request size")
    args = ap.parse_args()
    out = os.path.join(REPO, "profiles")
    os.makedirs(out, exist_ok=True)
    if args.stats:
        src = os.path.join(args.stats, "run_kernel_stats.csv")
        shutil.copy(src, os.path.join(out, f"{args.round}_kernel_stats.csv"))
    if args.fetch and args.write:
        fetch = counter(args.fetch, "FETCH_SIZE")
        write = counter(args.write, "WRITE_SIZE")
        f_kib, w_kib = statistics.median(fetch), statistics.median(write)
        rec = {"round": args.round, "kernel": "k_encode",
               "fetch_size_kib_raw": f_kib, "write_size_kib": w_kib,
               "fetch_bytes_corrected": f_kib * 1024 * 2, "write_bytes": w_kib * 1024,
               "hbm_bytes_per_launch": int(f_kib * 1024 * 2 + w_kib * 1024),
               "note": "FETCH_SIZE x2 (gfx950: 128-B read requests count half, every width; profiles/r5_pmc_calibration.json), "
                       "separate --pmc passes, median over launches"}
        # whole compress call: every kernel of the call (encode, scan, segment
        # bases, compaction, stats, end chunk, fills/copies), per call
        fk, wk = kernel_totals(args.fetch, "FETCH_SIZE"), kernel_totals(args.write, "WRITE_SIZE")
        calls = max(1, len(fetch) // 4)
        skip = ("k_synth", "k_equal")
        step_f = sum(v for k, v in fk.items() if not any(x in k for x in skip)) * 1024 * 2 / calls
        step_w = sum(v for k, v in wk.items() if not any(x in k for x in skip)) * 1024 / calls
        rec["whole_call"] = {"calls": calls, "fetch_bytes_corrected": int(step_f), "write_bytes": int(step_w),
                             "hbm_bytes": int(step_f + step_w),
                             "per_kernel_kib": {k.split("(")[0][-40:]: [round(fk.get(k, 0) / calls),
                                                                         round(wk.get(k, 0) / calls)]
                                                for k in sorted(set(fk) | set(wk))
                                                if not any(x in k for x in skip)}}
        if args.req:
            # the same traffic from the read requests by size (no FETCH_SIZE correction)
            q = {n: counter(args.req, n) for n in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                                                   "TCC_EA0_RDREQ_128B_sum")}
            per = [32 * a + 64 * b + 128 * c for a, b, c in zip(q["TCC_EA0_RDREQ_32B_sum"], q["TCC_EA0_RDREQ_64B_sum"],
                                                                 q["TCC_EA0_RDREQ_128B_sum"])]
            rec["fetch_bytes_from_requests"] = int(statistics.median(per))
            rec["fetch_check"] = "k_encode EA read bytes from TCC_EA0_RDREQ_{32B,64B,128B} x size, median over launches"
        if args.bench:
            with open(args.bench) as fh:
                b = json.loads(fh.read().strip().splitlines()[-1])
            rec["workload"] = b["config"]["workload"]
            rec["algorithmic_bytes_per_launch"] = b["roofline"]["algorithmic_bytes_per_launch"]
        with open(os.path.join(out, f"pmc_{args.round}.json"), "w") as fh:
            json.dump(rec, fh, indent=1)
        print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
