"""Process groups for the multi-GPU path, without PyTorch.

One process per GPU, launched by ``torch.distributed.run`` / ``torchrun`` (the
driver's launcher) or by ``bench.py --gpus N`` itself: the environment gives
``RANK``, ``WORLD_SIZE``, ``LOCAL_RANK``, ``MASTER_ADDR`` and ``MASTER_PORT``.

* ``HostGroup`` -- a TCP star on ``MASTER_ADDR:MASTER_PORT + 1`` (or
  ``AMBC_RDZV_PORT``): rank 0 listens, the others connect.  It carries the
  control plane only: the 128-byte RCCL unique id, and small all-gathers
  (timings, flags) -- a few bytes per call.
* ``GpuGroup`` -- a one-device ``Context`` on GPU ``LOCAL_RANK`` whose RCCL
  communicator (``ambc_comm_init_rank``) carries every device-side exchange
  of ``ambc.distributed`` (AllGather of body sizes, AllReduce of statistics,
  the gather of bodies over xGMI).

The reference has no process groups at all (it is single-threaded,
adaptive_compressor.py:363-394); this is the build's own plumbing for
SURVEY.md §8(e).
"""
import ctypes as C
import os
import socket
import struct
import time

from . import _lib


def env_ranks():
    """(rank, world, local_rank) from the launcher's environment (1 rank if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def rendezvous_address():
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = os.environ.get("AMBC_RDZV_PORT")
    if port is None:
        port = int(os.environ.get("MASTER_PORT", "29500")) + 1
    return addr, int(port)


def _send(sock, payload):
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        part = sock.recv(n - len(buf))
        if not part:
            raise ConnectionError("peer closed the rendezvous connection")
        buf += part
    return bytes(buf)


def _recv(sock):
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class HostGroup:
    """Small control messages between the ranks of one job (TCP star)."""

    def __init__(self, rank, world, addr=None, port=None, timeout=300.0):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world = rank, world
        self.peers = {}
        self.sock = None
        if world == 1:
            return
        if addr is None or port is None:
            a, p = rendezvous_address()
            addr = a if addr is None else addr
            port = p if port is None else port
        deadline = time.time() + timeout
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(max(1.0, deadline - time.time()))
            try:
                while len(self.peers) < world - 1:
                    conn, _ = srv.accept()
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    conn.settimeout(timeout)
                    (r,) = struct.unpack("<I", _recv_exact(conn, 4))
                    if r in self.peers or not 0 < r < world:
                        conn.close()
                        raise ConnectionError(f"bad or duplicate rank {r} at the rendezvous")
                    self.peers[r] = conn
            finally:
                srv.close()
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(timeout)
            s.sendall(struct.pack("<I", rank))
            self.sock = s

    def allgather(self, payload):
        """Every rank's bytes, in rank order, on every rank."""
        payload = bytes(payload)
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            parts = [payload] + [_recv(self.peers[r]) for r in range(1, self.world)]
            packed = b"".join(struct.pack("<Q", len(p)) + p for p in parts)
            for r in range(1, self.world):
                _send(self.peers[r], packed)
            return parts
        _send(self.sock, payload)
        packed, parts, o = _recv(self.sock), [], 0
        while o < len(packed):
            (n,) = struct.unpack_from("<Q", packed, o)
            parts.append(packed[o + 8:o + 8 + n])
            o += 8 + n
        return parts

    def broadcast(self, payload, src=0):
        return self.allgather(payload if self.rank == src else b"")[src]

    def barrier(self):
        self.allgather(b"")

    def allgather_obj(self, values):
        """A tuple of floats / ints from every rank (struct-packed doubles)."""
        vals = [float(v) for v in values]
        parts = self.allgather(struct.pack(f"<{len(vals)}d", *vals))
        return [struct.unpack(f"<{len(p) // 8}d", p) for p in parts]

    def close(self):
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None


class GpuGroup:
    """This process's rank: a one-device Context on GPU ``local_rank`` with an
    RCCL communicator over all ``world`` ranks (none when world == 1)."""

    def __init__(self, rank=None, world=None, local_rank=None, host=None, rccl=None):
        r, w, lr = env_ranks()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self.local_rank = lr if local_rank is None else local_rank
        self.host = host or HostGroup(self.rank, self.world)
        self.ctx = _lib.Context([self.local_rank])
        self.lib = self.ctx.lib
        if self.world > 1 or rccl:          # rccl=True: a communicator even for one rank
            uid = (C.c_uint8 * _lib.COMM_ID_BYTES)()
            if self.rank == 0:
                _lib.check(self.lib.ambc_comm_unique_id(uid), self.lib)
            got = self.host.broadcast(bytes(uid) if self.rank == 0 else b"")
            if len(got) != _lib.COMM_ID_BYTES:
                raise ConnectionError("RCCL unique id did not arrive whole")
            uid = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(got)
            _lib.check(self.lib.ambc_comm_init_rank(self.ctx.h, self.world, self.rank, uid), self.lib)

    def barrier(self):
        """Device-level barrier (RCCL AllReduce + device synchronize)."""
        _lib.check(self.lib.ambc_comm_barrier(self.ctx.h), self.lib)

    def close(self):
        self.ctx.close()
        self.host.close()
