"""One rank of the multi-process RCCL shard test (tests/test_gpu_distributed.py:
test_rccl_multi_rank_shards).  Launched once per GPU with RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT in the environment; rank r drives GPU r through
ambc_comm_init_rank (a real RCCL communicator over every GPU, no host
transport) and runs ambc_compress_shard / ambc_decompress_shard / the gather in
native and reference mode.  Rank 0 checks the gathered body against the CPU
oracle and the decoded bytes against the input; every rank prints one JSON
line and exits non-zero on a mismatch."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adaptive-compression_amd")]


def main():
    from ambc import AdaptiveCompressor, _lib
    from ambc.comm import GpuGroup
    from ambc.distributed import compress_shard, decompress_shard, shard_range
    from oracle import oracle as orc
    g = GpuGroup()
    rank, world = g.rank, g.world
    res = {"rank": rank, "world": world, "checks": []}
    ok = True
    cases = [("native", 4096, (1, 3, 4, 9), (8 << 20) + 12345, None),
             ("native", 8192, (1, 3, 4, 9), (6 << 20) + 8192 * 3, None),     # C4's chunk
             ("reference", 1024, (1, 3, 4), 0, 37)]                          # the remainder in shard ~1
    for mode, chunk, methods, n, raw_at in cases:
        if mode == "reference":
            parts = [orc.random_bytes(chunk, 2000 + k) if k == raw_at else bytes([k % 5]) * chunk
                     for k in range(24 * world)]
            data = b"".join(parts) + b"\x01" * 333
            n = len(data)
        else:
            data = orc.synth(n, 41 + chunk)
        ref, _ = orc.compress_body(data, orc.make_params(chunk, mode, tuple(methods) + (255,), n_total=n))
        b0, b1 = shard_range(n, chunk, world, rank)
        p, keep = AdaptiveCompressor(chunk_size=chunk, mode=mode, methods=methods)._params(n)
        d_in = _lib.DeviceBuffer(g.ctx, max(b1 - b0, 1) + 64)
        if b1 > b0:
            d_in.upload(data[b0:b1])
        cap = g.lib.ambc_compress_bound(n, chunk)
        d_out = _lib.DeviceBuffer(g.ctx, cap + 64)
        info, st = compress_shard(g, d_in, n, p, d_out, cap, root=0)
        c = {"mode": mode, "chunk": chunk, "n": n, "total": info.total, "local": info.local_len,
             "offset": info.offset, "chunks": st.total_chunks}
        if rank == 0:
            c["body_equals_oracle"] = bytes(d_out.download(info.total)) == ref
            ok &= c["body_equals_oracle"]
        ok &= info.total == len(ref)
        d_dec = _lib.DeviceBuffer(g.ctx, n + 64)
        dinfo, _ = decompress_shard(g, ref, n, d_dec, n + 64, root=0)
        if rank == 0:
            c["decode_equals_input"] = bytes(d_dec.download(n)) == data
            ok &= c["decode_equals_input"]
        res["checks"].append(c)
        for b in (d_in, d_out, d_dec):
            b.free()
        g.barrier()
    res["ok"] = bool(ok)
    print(json.dumps(res), flush=True)
    g.close()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
