"""Command line of the reference (main.py:91-163) for the MI355X engine:

    python main.py compress   INPUT OUTPUT   [--chunk-size C] [--mode native|reference]
                                             [--methods 1,3,4,9] [--reference-candidates]
    python main.py decompress INPUT OUTPUT
    python main.py analyze    [--results-file F] [--output-dir D]

Same printouts as the reference's compress_file / decompress_file /
analyze_results (main.py:166-249); compress appends its stats to the
CompressionAnalyzer history (main.py:184-194, compression_analyzer.py:30-72).
The Gradio GUI (``gui``, the reference's default) is not part of this engine.
"""
import argparse
import json
import os
import sys

from .analyzer import CompressionAnalyzer
from .registry import METHOD_NAMES, REFERENCE_CHUNK_SIZE_CANDIDATES

LONG_NAMES = {1: "Run-Length Encoding (RLE)", 2: "Dictionary-Based", 3: "Huffman Coding",
              4: "Delta Encoding", 5: "DEFLATE", 6: "BZIP2", 7: "LZMA", 8: "ZStandard", 9: "LZ4",
              10: "Brotli", 11: "LZHAM", 255: "No Compression"}
HISTORY = os.path.join("compression_results", "compression_history.json")


def get_method_name(method_id):
    try:
        method_id = int(method_id)
    except (TypeError, ValueError):
        return f"Method {method_id}"
    return LONG_NAMES.get(method_id, METHOD_NAMES.get(method_id, f"Method {method_id}"))


def _compressor(args):
    from .compressor import AdaptiveCompressor
    methods = tuple(int(x) for x in args.methods.split(",")) if args.methods else None
    comp = AdaptiveCompressor(chunk_size=args.chunk_size, mode=args.mode, methods=methods)
    if args.reference_candidates:
        comp.CHUNK_SIZE_CANDIDATES = list(REFERENCE_CHUNK_SIZE_CANDIDATES)
    return comp


def compress_file(input_path, output_path, args, history=HISTORY):
    print(f"Compressing {input_path} to {output_path}...")
    try:
        stats = _compressor(args).compress(input_path, output_path)
        print("\nCompression Statistics:")
        print(f"  Original size: {stats['original_size']} bytes")
        print(f"  Compressed size: {stats['compressed_size']} bytes")
        print(f"  Compression ratio: {stats['ratio']:.4f}")
        print(f"  Space saving: {stats['percent_reduction']:.2f}%")
        print(f"  Elapsed time: {stats['elapsed_time']:.4f} seconds")
        print(f"  Throughput: {stats['throughput_mb_per_sec']:.2f} MB/s")
        print("\nChunk Statistics:")
        print(f"  Total chunks: {stats['chunk_stats']['total_chunks']}")
        for mid, count in stats["chunk_stats"]["method_usage"].items():
            if count > 0:
                print(f"    {get_method_name(mid)}: {count} chunks")
        if history:
            os.makedirs(os.path.dirname(history) or ".", exist_ok=True)
            analyzer = CompressionAnalyzer()
            if os.path.exists(history):
                analyzer.load_results(history)
            analyzer.add_result(input_path, stats)
            analyzer.save_results(history)
        print("\nCompression completed successfully.")
        return stats
    except Exception as e:  # noqa: BLE001 -- the reference reports and exits 1 (main.py:197-199)
        print(f"Error during compression: {e}")
        sys.exit(1)


def decompress_file(input_path, output_path, args=None):
    print(f"Decompressing {input_path} to {output_path}...")
    try:
        from .compressor import AdaptiveCompressor
        stats = AdaptiveCompressor().decompress(input_path, output_path)
        print("\nDecompression Statistics:")
        print(f"  Compressed size: {stats['compressed_size']} bytes")
        print(f"  Decompressed size: {stats['decompressed_size']} bytes")
        print(f"  Elapsed time: {stats['elapsed_time']:.4f} seconds")
        print(f"  Throughput: {stats['throughput_mb_per_sec']:.2f} MB/s")
        print("\nDecompression completed successfully.")
        return stats
    except Exception as e:  # noqa: BLE001 -- main.py:214-216
        print(f"Error during decompression: {e}")
        sys.exit(1)


def analyze_results(results_file, output_dir):
    print(f"Analyzing compression results from {results_file}...")
    try:
        analyzer = CompressionAnalyzer()
        analyzer.load_results(results_file)
        os.makedirs(output_dir, exist_ok=True)
        summary = analyzer.get_summary_stats()
        print("\nSummary Statistics:")
        for key, value in summary.items():
            print(f"  {key}: {value}")
        with open(os.path.join(output_dir, "summary.json"), "w") as f:
            json.dump(summary, f, indent=2)
        with open(os.path.join(output_dir, "method_usage.json"), "w") as f:
            json.dump(analyzer.get_method_usage_stats(), f, indent=2)
        print("\nAnalysis completed successfully.")
        return summary
    except Exception as e:  # noqa: BLE001 -- main.py:246-248
        print(f"Error during analysis: {e}")
        sys.exit(1)


def build_parser():
    ap = argparse.ArgumentParser(description="Adaptive Marker-Based Compression Algorithm (MI355X engine)")
    sub = ap.add_subparsers(dest="command", help="Command to execute")
    c = sub.add_parser("compress", help="Compress a file")
    c.add_argument("input")
    c.add_argument("output")
    c.add_argument("--chunk-size", type=int, default=None, help="CHUNK_SIZE_CANDIDATES=[C] (default 4096)")
    c.add_argument("--mode", choices=["native", "reference"], default="native")
    c.add_argument("--methods", default=None, help="GPU method ids, e.g. 1,3,4,9 (default) or 1,2,3,4")
    c.add_argument("--reference-candidates", action="store_true",
                   help="the reference's 8-size CHUNK_SIZE_CANDIDATES walk (adaptive_compressor.py:61-62)")
    c.add_argument("--history", default=HISTORY, help="history JSON ('' to skip)")
    d = sub.add_parser("decompress", help="Decompress a file")
    d.add_argument("input")
    d.add_argument("output")
    a = sub.add_parser("analyze", help="Analyze compression results")
    a.add_argument("--results-file", default=HISTORY)
    a.add_argument("--output-dir", default="analysis_output")
    sub.add_parser("gui", help="(not available: the reference's Gradio GUI is not part of this engine)")
    return ap


def main(argv=None):
    args = build_parser().parse_args(argv)
    if args.command == "compress":
        compress_file(args.input, args.output, args, history=args.history)
    elif args.command == "decompress":
        decompress_file(args.input, args.output, args)
    elif args.command == "analyze":
        analyze_results(args.results_file, args.output_dir)
    else:
        print("The Gradio GUI is not part of the MI355X engine; use compress / decompress / analyze.")
        return 2
    return 0
