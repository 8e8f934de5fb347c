"""Print a same-box A/B's kbench + bench lines: python scripts/ab_summary.py DIR lib1 lib2 ..."""
import json
import os
import sys

d = sys.argv[1]
for lib in sys.argv[2:]:
    for rep in (1, 2, 3):
        kf, bf = os.path.join(d, f"kbench_{lib}_{rep}.log"), os.path.join(d, f"bench_{lib}_{rep}.json")
        if not os.path.exists(kf):
            continue
        ks = [json.loads(l) for l in open(kf) if l.startswith("{")]
        line = " ".join("%s%s:%.3f" % (k["input"][:3], "".join(map(str, k["methods"])), k["encode_ms"]) for k in ks)
        if os.path.exists(bf) and os.path.getsize(bf):
            b = json.loads(open(bf).read().strip().splitlines()[-1])
            line += " bench %s k_enc %s" % (b["value"], b["roofline"]["achieved"])
        print(lib, rep, line)
