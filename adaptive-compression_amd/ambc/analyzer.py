"""Compression history, record-compatible with the reference's
``CompressionAnalyzer`` (compression_analyzer.py:9-258): the JSON list that
``main.py compress`` appends to ``compression_results/compression_history.json``
and ``main.py analyze`` summarises.

Each record is the ``compress()`` stats dict plus ``filename``, ``extension``,
``filename_no_ext``, ``timestamp`` and ``size_label`` (add_result, :30-62);
one record per base filename, the newest wins (:46-62, :74-137).  The plots
(:295-856) are the reference's reporting UI and are not rebuilt here.
"""
import json
import os
import time
from collections import defaultdict

METHOD_LABELS = {
    "1": "RLE", "2": "Dictionary", "3": "Huffman", "4": "Delta", "5": "DEFLATE", "6": "BZIP2",
    "7": "LZMA", "8": "ZStd", "9": "LZ4", "10": "Brotli", "11": "LZHAM", "255": "No Compression",
}


def format_file_size(size_bytes):
    """'39.1 KB' style labels (compression_analyzer.py:857-876)."""
    if size_bytes == 0:
        return "0 B"
    units = ["B", "KB", "MB", "GB", "TB"]
    v, i = float(size_bytes), 0
    while v >= 1024 and i < len(units) - 1:
        v /= 1024.0
        i += 1
    return f"{v:.1f} {units[i]}"


def _newest_per_file(records):
    latest = {}
    for r in records:
        name = r.get("filename", "unknown")
        if name not in latest or r.get("timestamp", 0) > latest[name].get("timestamp", 0):
            latest[name] = r
    return list(latest.values())


class CompressionAnalyzer:
    def __init__(self):
        self.results = []
        self.filename_map = {}
        self.method_names = dict(METHOD_LABELS)

    def _reindex(self):
        self.filename_map = {r.get("filename", f"file_{i}"): i for i, r in enumerate(self.results)}

    def add_result(self, filename, stats):
        base = os.path.basename(filename)
        stem, ext = os.path.splitext(base)
        stats["filename"] = base
        stats["extension"] = ext.lower() or "unknown"
        stats["filename_no_ext"] = stem
        stats["timestamp"] = time.time()
        stats["size_label"] = format_file_size(stats.get("original_size", 0))
        if base in self.filename_map:
            i = self.filename_map[base]
            if stats["timestamp"] > self.results[i].get("timestamp", 0):
                print(f"Replacing previous result for '{base}'")
                self.results[i] = stats
        else:
            self.results.append(stats)
            self.filename_map[base] = len(self.results) - 1

    def save_results(self, filename):
        with open(filename, "w") as f:
            json.dump(self.results, f, indent=2)

    def load_results(self, filename):
        try:
            with open(filename) as f:
                records = json.load(f)
        except (OSError, ValueError) as e:
            print(f"Error loading results: {e}")
            self.results, self.filename_map = [], {}
            return 0
        before = len(records)
        self.results = _newest_per_file(records)
        for i, r in enumerate(self.results):
            name = r.get("filename", f"file_{i}")
            stem, ext = os.path.splitext(name)
            r.setdefault("extension", ext.lower() or "unknown")
            r.setdefault("filename_no_ext", stem)
            r.setdefault("size_label", format_file_size(r.get("original_size", 0)))
        self._reindex()
        dropped = before - len(self.results)
        if dropped > 0:
            print(f"Loaded {len(self.results)} unique results (removed {dropped} duplicates)")
        else:
            print(f"Loaded {len(self.results)} results (no duplicates found)")
        return len(self.results)

    def clear_results(self):
        self.results, self.filename_map = [], {}

    def remove_duplicates(self):
        before = len(self.results)
        self.results = _newest_per_file(self.results)
        self._reindex()
        if before - len(self.results) > 0:
            print(f"Removed {before - len(self.results)} duplicate entries")
        return before - len(self.results)

    def get_summary_stats(self):
        """compression_analyzer.py:146-215."""
        if not self.results:
            return {"total_files": 0, "total_original_size": 0, "total_compressed_size": 0,
                    "average_ratio": 0, "average_percent_reduction": 0, "average_throughput": 0,
                    "file_types": {}}
        count = defaultdict(int)
        reductions = defaultdict(list)
        osz = defaultdict(int)
        csz = defaultdict(int)
        for r in self.results:
            ext = r.get("extension", "unknown").lower()
            count[ext] += 1
            reductions[ext].append(r.get("percent_reduction", 0))
            osz[ext] += r.get("original_size", 0)
            csz[ext] += r.get("compressed_size", 0)
        tot_o = sum(r.get("original_size", 0) for r in self.results)
        tot_c = sum(r.get("compressed_size", 0) for r in self.results)
        k = len(self.results)
        s = {
            "total_files": k, "total_original_size": tot_o, "total_compressed_size": tot_c,
            "average_ratio": sum(r.get("ratio", 0) for r in self.results) / k,
            "average_percent_reduction": sum(r.get("percent_reduction", 0) for r in self.results) / k,
            "average_throughput": sum(r.get("throughput_mb_per_sec", 0) for r in self.results) / k,
            "file_types": dict(count),
            "type_avg_compression": {e: sum(v) / len(v) if v else 0 for e, v in reductions.items()},
            "type_ratio": {e: csz[e] / osz[e] if osz[e] > 0 else 1.0 for e in count},
            "type_original_size": dict(osz), "type_compressed_size": dict(csz),
        }
        s["overall_ratio"] = tot_c / tot_o if tot_o > 0 else 1.0
        s["overall_percent_reduction"] = (1 - s["overall_ratio"]) * 100 if tot_o > 0 else 0.0
        s["total_original_size_formatted"] = format_file_size(tot_o)
        s["total_compressed_size_formatted"] = format_file_size(tot_c)
        return s

    def get_method_usage_stats(self):
        """compression_analyzer.py:259-293."""
        if not self.results:
            return {}
        counts = defaultdict(int)
        per_type = defaultdict(lambda: defaultdict(int))
        for r in self.results:
            ext = r.get("extension", "unknown")
            for mid, c in r.get("chunk_stats", {}).get("method_usage", {}).items():
                counts[mid] += c
                per_type[ext][mid] += c
        total = sum(counts.values())
        return {"method_counts": dict(counts),
                "method_percentages": {m: (c / total * 100) if total > 0 else 0 for m, c in counts.items()},
                "total_chunks": total,
                "file_type_method_usage": {e: dict(m) for e, m in per_type.items()}}
