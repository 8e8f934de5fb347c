"""GPU coverage of the sharded decode (SURVEY §8(e), config C5 at N GPUs):
the body split at package boundaries (ambc_split_body), every range decoded on
the GPU into device memory (ambc_decompress_device) and gathered in file order
must equal the input; the same through torch.distributed with two ranks on the
one GPU of the test box (gloo carries the exchange there; RCCL on a node)."""
import os
import socket

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _body(n, chunk, methods, seed):
    data = orc.synth(n, seed)
    body, _ = orc.compress_body(data, orc.make_params(chunk, "native", methods, n_total=n))
    return data, body


@pytest.mark.parametrize("n,chunk,methods,parts", [
    ((1 << 22) + 123, 4096, (1, 3, 4, 9), 8),
    (1 << 21, 1024, (1, 3, 4, 9), 3),
    ((1 << 21) + 77, 4096, (1, 3, 5), 8),        # C5 method set (zlib-9 DEFLATE chunks)
])
def test_split_ranges_decode_on_device(hip_lib, n, chunk, methods, parts):
    from ambc.distributed import hip_decode_fn, split_body
    data, body = _body(n, chunk, methods, 11)
    fn = hip_decode_fn()
    sp = split_body(body, n, parts)
    got = bytearray()
    for b0, b1, o0, o1 in sp:
        if b1 == b0:
            continue
        out, produced = fn(memoryview(body)[b0:b1], o1 - o0)
        assert produced == o1 - o0
        got += out.cpu().numpy().tobytes()
    assert bytes(got) == data


def test_device_decode_rejects_host_codec_packages(hip_lib):
    """ids 6/7 (bz2 / lzma) are host codecs: the device-output call says so."""
    import bz2
    import struct
    from ambc import _lib
    from ambc.distributed import hip_decode_fn
    payload = bz2.compress(b"q" * 500)
    body = b"\xff\xff\x00\x00" + bytes([6, 0]) + struct.pack("<III", 500, 500, len(payload)) + \
        payload + b"\xff\xff\x00\x00" + bytes(12)
    with pytest.raises(_lib.AmbcError) as e:
        hip_decode_fn()(body, 500)
    assert e.value.code == _lib.AMBC_E_HOSTCODEC


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, body, n, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "adaptive-compression_amd")]
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ambc.distributed import decompress_sharded, hip_decode_fn
    fn = hip_decode_fn()

    def cpu_fn(sub, m):                      # gloo moves host tensors
        out, produced = fn(sub, m)
        return out.cpu(), produced

    out = decompress_sharded(body, n, cpu_fn)
    if rank == 0:
        q.put(out.numpy().tobytes())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_decode_two_ranks(hip_lib):
    import torch.multiprocessing as mp
    n = (1 << 21) + 5
    data, body = _body(n, 4096, (1, 3, 4, 9), 5)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, body, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == data
