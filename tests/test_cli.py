"""CLI + history compatibility: main.py compress /
decompress / analyze (main.py:91-249) and the CompressionAnalyzer record format
(compression_analyzer.py:30-215), pinned by records of the reference's own
compression_results/compression_history.json (tests/golden/history_sample.json)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, PKG_DIR


def _sample():
    with open(os.path.join(GOLDEN, "history_sample.json")) as f:
        return json.load(f)


def test_size_labels_match_reference_records():
    from ambc.analyzer import format_file_size
    for r in _sample():
        assert format_file_size(r["original_size"]) == r["size_label"]
    assert format_file_size(0) == "0 B"


def test_add_result_produces_reference_record_keys(tmp_path):
    from ambc.analyzer import CompressionAnalyzer
    ref = _sample()[0]
    stats = {k: v for k, v in ref.items()
             if k not in ("filename", "extension", "filename_no_ext", "timestamp", "size_label")}
    a = CompressionAnalyzer()
    a.add_result("/some/dir/" + ref["filename"], stats)
    rec = a.results[0]
    assert set(rec) == set(ref)
    for k in ("filename", "extension", "filename_no_ext", "size_label"):
        assert rec[k] == ref[k]
    out = tmp_path / "h.json"
    a.save_results(str(out))
    b = CompressionAnalyzer()
    assert b.load_results(str(out)) == 1
    assert b.results[0]["filename"] == ref["filename"]


def test_history_dedup_and_summary(tmp_path):
    from ambc.analyzer import CompressionAnalyzer
    recs = _sample()
    dup = dict(recs[0])
    dup["timestamp"] = recs[0]["timestamp"] + 10
    dup["compressed_size"] = 1
    p = tmp_path / "h.json"
    p.write_text(json.dumps(recs + [dup]))
    a = CompressionAnalyzer()
    assert a.load_results(str(p)) == len(recs)
    assert a.results[a.filename_map[recs[0]["filename"]]]["compressed_size"] == 1
    s = a.get_summary_stats()
    tot_o = sum(r["original_size"] for r in a.results)
    tot_c = sum(r["compressed_size"] for r in a.results)
    assert s["total_files"] == len(recs)
    assert s["overall_ratio"] == pytest.approx(tot_c / tot_o)
    assert s["average_ratio"] == pytest.approx(sum(r["ratio"] for r in a.results) / len(recs))
    m = a.get_method_usage_stats()
    assert m["total_chunks"] == sum(sum(r["chunk_stats"]["method_usage"].values()) for r in a.results)


def test_analyze_command_writes_summary(tmp_path):
    p = tmp_path / "h.json"
    p.write_text(json.dumps(_sample()))
    out = tmp_path / "analysis"
    r = subprocess.run([sys.executable, os.path.join(PKG_DIR, "main.py"), "analyze", "--results-file", str(p),
                        "--output-dir", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Summary Statistics:" in r.stdout and "Analysis completed successfully." in r.stdout
    assert json.loads((out / "summary.json").read_text())["total_files"] == len(_sample())


@pytest.mark.gpu
def test_cli_compress_decompress_round_trip(tmp_path, hip_lib):
    from oracle import oracle as orc
    data = orc.synth(300000, 5)
    src, dst, back = tmp_path / "in.bin", tmp_path / "out.ambc", tmp_path / "back.bin"
    src.write_bytes(data)
    hist = tmp_path / "compression_results" / "compression_history.json"
    main = os.path.join(PKG_DIR, "main.py")
    r = subprocess.run([sys.executable, main, "compress", str(src), str(dst), "--history", str(hist)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    for line in ("Compression Statistics:", "Compression ratio:", "Chunk Statistics:",
                 "Compression completed successfully."):
        assert line in r.stdout
    r = subprocess.run([sys.executable, main, "decompress", str(dst), str(back)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert back.read_bytes() == data
    rec = json.loads(hist.read_text())
    assert len(rec) == 1 and set(rec[0]) == set(_sample()[0])
    assert rec[0]["compressed_size"] == os.path.getsize(dst)
