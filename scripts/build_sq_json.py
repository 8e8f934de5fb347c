"""Assemble profiles/r2_pmc_sq.json from the SQ passes of scripts/profile_r2.sh
(gpurun_out/r2/*): per kernel and input class, SQ counters per wave.

    python scripts/build_sq_json.py [DIR] [OUT]"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def summ(d, p1, p2, kernels, group, labels=""):
    cmd = [sys.executable, os.path.join(HERE, "sq_summary.py"), os.path.join(d, p1), os.path.join(d, p2),
           "--kernels", kernels, "--group", str(group)]
    if labels:
        cmd += ["--labels", labels]
    return json.loads(subprocess.check_output(cmd))


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r2"
    out = sys.argv[2] if len(sys.argv) > 2 else "profiles/r2_pmc_sq.json"
    res = {
        "note": "rocprofv3 --pmc SQ counters (two passes per command, scripts/profile_r2.sh), per wave; "
                "k_encode / k_deflate / k_decode*: one wave per chunk or job; k_dict<4096>: 8 waves per "
                "chunk (multiply per_wave by 8 for per chunk); SQ_WAVE_CYCLES/WAIT/ACTIVE in quad-cycles. "
                "Built by scripts/build_sq_json.py from scripts/sq_summary.py.",
        "k_encode_1349_per_class": summ(d, "sq_enc1", "sq_enc2", "k_encode", 4, "random,ascii,mixed"),
        "k_deflate_k_dict_alt_sets": dict(
            labels="per kernel: ascii 256 MiB, then mixed 256 MiB (4 pipelined segments each)",
            **summ(d, "sq_alt1", "sq_alt2", "k_deflate,k_dict", 4, "ascii,mixed")),
        "k_decode_inflate_1345": dict(
            labels="dbench 64 MiB per class, dispatch order: zero, ascii, mixed",
            **summ(d, "sq_dec1", "sq_dec2", "k_decode_inflate", 1, "zero,ascii,mixed")),
        "k_decode_1234": dict(
            labels="Dictionary / Huffman packages, dbench 64 MiB, dispatch order",
            **summ(d, "sq_decd1", "sq_decd2", "k_decode_light,k_decode,k_decode_dict", 1)),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
