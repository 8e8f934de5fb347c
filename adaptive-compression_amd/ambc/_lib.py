"""ctypes binding of libambc_hip.so (include/ambc.h).

This is the only way the product reaches its codecs: there is no CPU codec
path.  ``load()`` raises ``AmbcUnavailable`` when the in-tree library is
missing or cannot be loaded, and ``Context`` raises when no gfx950 device is
present -- the product fails loudly instead of silently falling back.
"""
import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libambc_hip.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)

AMBC_OK = 0
AMBC_E_INVAL = -1
AMBC_E_DEVICE = -2
AMBC_E_NOMEM = -3
AMBC_E_RANGE = -4
AMBC_E_MARKER = -5
AMBC_E_CAPACITY = -6
AMBC_E_HOSTCODEC = -7
AMBC_E_CODEC = -8
AMBC_E_COMM = -9

OP_SUM, OP_MIN, OP_MAX = 0, 1, 2
COMM_ID_BYTES = 128

MODE_NATIVE = 0
MODE_REFERENCE = 1
FLAG_NO_END_CHUNK = 1
FLAG_ZLIB9 = 2          # id 5 = zlib.compress(data, 9)'s bytes (chunk_size <= 65536)
FLAG_INPUT_PADDED = 4   # device inputs: 64 readable bytes after n (large chunks read in place)
MAX_CHUNK = 65536

EXPORTS = (
    "ambc_abi_version", "ambc_last_error", "ambc_device_count", "ambc_init", "ambc_destroy",
    "ambc_compress_bound", "ambc_compress_batch", "ambc_decompress_batch", "ambc_decompress_ex",
    "ambc_compress_device", "ambc_encode_method", "ambc_analyze", "ambc_dict_encode", "ambc_encode_any", "ambc_analyze_any", "ambc_host_alloc",
    "ambc_host_free", "ambc_device_alloc", "ambc_device_free", "ambc_memcpy_h2d",
    "ambc_memcpy_d2h", "ambc_synchronize", "ambc_synth_fill", "ambc_synth_device",
    "ambc_last_kernel_times", "ambc_split_body", "ambc_decompress_device",
    "ambc_last_encode_launches", "ambc_memcpy_d2d", "ambc_memset_device",
    "ambc_comm_unique_id", "ambc_comm_init_rank", "ambc_comm_size", "ambc_comm_barrier",
    "ambc_comm_allreduce_u64", "ambc_comm_allgather_u64", "ambc_comm_gather", "ambc_shard_range",
    "ambc_compress_shard", "ambc_decompress_shard", "ambc_decompress_multi",
    "ambc_synth_device_range", "ambc_device_equal", "ambc_compress_multisize",
    "ambc_last_multisize_info", "ambc_fetch_body", "ambc_compress_multisize_ex", "ambc_debug_walk",
    "ambc_test_inject_failure",
)


class AmbcUnavailable(RuntimeError):
    """libambc_hip.so or a gfx950 device is missing (no CPU fallback exists)."""


class AmbcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ambc error {code}: {msg}")
        self.code = code
        self.msg = msg


class Params(C.Structure):
    _fields_ = [("chunk_size", C.c_uint32), ("mode", C.c_uint32), ("method_mask", C.c_uint32),
                ("flags", C.c_uint32), ("pref_min", C.c_uint32 * 16),
                ("pref_max", C.c_uint32 * 16), ("ent_full", C.c_void_p),
                ("ent_tail", C.c_void_p)]


class Stats(C.Structure):
    _fields_ = [("method_usage", C.c_uint64 * 256), ("total_chunks", C.c_uint64),
                ("compressed_chunks", C.c_uint64), ("raw_chunks", C.c_uint64),
                ("bytes_saved", C.c_uint64), ("payload_bytes", C.c_uint64),
                ("overhead_bytes", C.c_uint64), ("kernel_ns", C.c_uint64),
                ("h2d_ns", C.c_uint64), ("d2h_ns", C.c_uint64), ("walk_ns", C.c_uint64),
                ("total_ns", C.c_uint64), ("host_codec_ns", C.c_uint64)]


class HostChunk(C.Structure):
    _fields_ = [("body_off", C.c_uint64), ("out_off", C.c_uint64), ("clen", C.c_uint32),
                ("orig", C.c_uint32), ("type", C.c_uint32), ("reserved", C.c_uint32)]


class ShardInfo(C.Structure):
    _fields_ = [("local_len", C.c_uint64), ("offset", C.c_uint64), ("total", C.c_uint64),
                ("shard_begin", C.c_uint64), ("shard_end", C.c_uint64)]


_lib = None
_lock = threading.RLock()


def _declare(lib):
    vp, u8p, u32, u64, i32 = C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    sig = {
        "ambc_abi_version": ([], i32),
        "ambc_last_error": ([], C.c_char_p),
        "ambc_device_count": ([C.POINTER(i32)], i32),
        "ambc_init": ([C.POINTER(i32), i32, C.POINTER(vp)], i32),
        "ambc_destroy": ([vp], None),
        "ambc_compress_bound": ([u64, u32], u64),
        "ambc_compress_batch": ([vp, u8p, u64, C.POINTER(Params), u8p, u64, C.POINTER(u64),
                                 C.POINTER(Stats)], i32),
        "ambc_decompress_batch": ([vp, u8p, u64, u64, u8p, C.POINTER(Stats)], i32),
        "ambc_decompress_ex": ([vp, u8p, u64, u64, C.POINTER(u64), u8p, C.POINTER(HostChunk), u32,
                                C.POINTER(u32), C.POINTER(Stats)], i32),
        "ambc_compress_device": ([vp, i32, vp, u64, C.POINTER(Params), vp, u64, C.POINTER(u64),
                                  C.POINTER(Stats), vp], i32),
        "ambc_encode_method": ([vp, i32, u8p, u32, u8p, u32, C.POINTER(u32)], i32),
        "ambc_analyze": ([vp, u8p, u64, C.POINTER(Params), u8p, u8p, u8p], i32),
        "ambc_dict_encode": ([vp, u8p, u64, C.c_int64, C.c_int64, u8p, u64, C.POINTER(u64)], i32),
        "ambc_encode_any": ([vp, i32, u8p, u64, u8p, u64, C.POINTER(u64)], i32),
        "ambc_analyze_any": ([vp, u8p, u64, u64, C.POINTER(u32)], i32),
        "ambc_host_alloc": ([u64], vp),
        "ambc_host_free": ([vp], None),
        "ambc_device_alloc": ([vp, i32, u64], vp),
        "ambc_device_free": ([vp, i32, vp], None),
        "ambc_memcpy_h2d": ([vp, i32, vp, vp, u64], i32),
        "ambc_memcpy_d2h": ([vp, i32, vp, vp, u64], i32),
        "ambc_synchronize": ([vp, i32], i32),
        "ambc_synth_fill": ([u8p, u64, u64], None),
        "ambc_synth_device": ([vp, i32, vp, u64, u64], i32),
        "ambc_last_kernel_times": ([vp, i32, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)], i32),
        "ambc_last_encode_launches": ([vp, i32, C.POINTER(C.c_uint32)], i32),
        "ambc_split_body": ([u8p, u64, u64, C.POINTER(u64), u32, C.POINTER(u64), C.POINTER(u64)], i32),
        "ambc_decompress_device": ([vp, i32, u8p, u64, u64, C.POINTER(u64), vp, C.POINTER(Stats)], i32),
        "ambc_memcpy_d2d": ([vp, i32, vp, vp, u64], i32),
        "ambc_memset_device": ([vp, i32, vp, i32, u64], i32),
        "ambc_comm_unique_id": ([vp], i32),
        "ambc_comm_init_rank": ([vp, i32, i32, vp], i32),
        "ambc_comm_size": ([vp, C.POINTER(i32), C.POINTER(i32)], i32),
        "ambc_comm_barrier": ([vp], i32),
        "ambc_comm_allreduce_u64": ([vp, C.POINTER(u64), u32, i32], i32),
        "ambc_comm_allgather_u64": ([vp, C.POINTER(u64), u32, C.POINTER(u64)], i32),
        "ambc_comm_gather": ([vp, vp, u64, vp, u64, C.POINTER(u64), C.POINTER(u64)], i32),
        "ambc_shard_range": ([u64, u32, i32, i32, C.POINTER(u64), C.POINTER(u64)], i32),
        "ambc_compress_shard": ([vp, vp, u64, C.POINTER(Params), vp, u64, i32, C.POINTER(ShardInfo),
                                 C.POINTER(Stats)], i32),
        "ambc_decompress_shard": ([vp, u8p, u64, u64, C.POINTER(u64), vp, u64, i32,
                                   C.POINTER(ShardInfo), C.POINTER(Stats)], i32),
        "ambc_decompress_multi": ([vp, u8p, u64, u64, C.POINTER(u64), u8p, C.POINTER(Stats)], i32),
        "ambc_synth_device_range": ([vp, i32, vp, u64, u64, u64, u64], i32),
        "ambc_device_equal": ([vp, i32, vp, vp, u64, C.POINTER(i32)], i32),
        "ambc_compress_multisize": ([vp, u8p, u64, C.POINTER(Params), C.POINTER(u32), u32, C.POINTER(u32),
                                     C.POINTER(C.c_void_p), u32, u8p, u64, C.POINTER(u64),
                                     C.POINTER(Stats)], i32),
        "ambc_last_multisize_info": ([vp, C.POINTER(u32), C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)], i32),
        "ambc_fetch_body": ([vp, u8p, u64], i32),
        "ambc_compress_multisize_ex": ([vp, u8p, u64, C.POINTER(Params), C.POINTER(u32), u32, C.POINTER(u32),
                                        C.POINTER(C.c_void_p), u32, vp, u8p, u64, C.POINTER(u64),
                                        C.POINTER(Stats)], i32),
        "ambc_debug_walk": ([u8p, u64, u64, u32, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)], i32),
        "ambc_test_inject_failure": ([i32], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def load(path=None):
    """Load the in-tree libambc_hip.so (raises AmbcUnavailable if absent)."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("AMBC_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise AmbcUnavailable(
                f"{p} not found: build it with `make -C adaptive-compression_amd/csrc` "
                "(hipcc --offload-arch=gfx950); the product has no CPU fallback")
        try:
            lib = C.CDLL(p)
        except OSError as e:
            raise AmbcUnavailable(f"cannot load {p}: {e}") from e
        missing = [s for s in EXPORTS if not hasattr(lib, s)]
        if missing:
            raise AmbcUnavailable(f"{p} lacks exports {missing}")
        _declare(lib)
        if path is None:
            _lib = lib
        return lib


def last_error(lib=None):
    lib = lib or load()
    m = lib.ambc_last_error()
    return m.decode(errors="replace") if m else ""


def check(rc, lib=None):
    if rc != AMBC_OK:
        raise AmbcError(rc, last_error(lib))
    return rc


def addr(buf):
    """Address of a writable/readonly bytes-like object without copying."""
    if buf is None:
        return None
    if isinstance(buf, int):
        return buf
    mv = memoryview(buf)
    if mv.readonly:
        # ctypes cannot take a pointer to read-only memory: numpy's view of the
        # caller's own buffer gives its address without a copy (valid while the
        # caller holds the object)
        import numpy as np
        return np.frombuffer(mv, dtype=np.uint8).ctypes.data if mv.nbytes else None
    return C.addressof(C.c_char.from_buffer(mv))


class Context:
    """One ambc_ctx (streams + device workspaces) on one or more GPUs."""

    def __init__(self, devices=None):
        self.lib = load()
        n = C.c_int(0)
        rc = self.lib.ambc_device_count(C.byref(n))
        if rc != AMBC_OK or n.value == 0:
            raise AmbcUnavailable("no HIP device visible: libambc_hip has no CPU fallback")
        devs = list(devices) if devices else [0]
        arr = (C.c_int * len(devs))(*devs)
        h = C.c_void_p()
        rc = self.lib.ambc_init(arr, len(devs), C.byref(h))
        if rc != AMBC_OK:
            raise AmbcUnavailable(last_error(self.lib))
        self.h = h
        self.devices = devs
        # one call at a time per context: its device workspaces (and a body that
        # ambc_compress_multisize(out=NULL) leaves for ambc_fetch_body) are shared.
        # Every libambc call on the context's workspaces takes it (compressor.py,
        # methods.py, distributed.py)
        self.lock = threading.RLock()

    def close(self):
        if getattr(self, "h", None):
            self.lib.ambc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class DeviceBuffer:
    """nbytes of device memory on one device of a Context (ambc_device_alloc):
    the Python layer's HBM buffers, no PyTorch."""

    def __init__(self, ctx, nbytes, dev=0):
        self.ctx, self.dev, self.nbytes = ctx, dev, int(nbytes)
        p = ctx.lib.ambc_device_alloc(ctx.h, dev, max(self.nbytes, 1))
        if not p:
            raise MemoryError(f"ambc_device_alloc({self.nbytes}) failed: {last_error(ctx.lib)}")
        self.ptr = p

    def __int__(self):
        return self.ptr

    def free(self):
        if getattr(self, "ptr", None) and self.ctx.h:
            self.ctx.lib.ambc_device_free(self.ctx.h, self.dev, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    def upload(self, data, offset=0):
        n = len(memoryview(data).cast("B"))
        if offset + n > self.nbytes:
            raise ValueError("upload past the end of the device buffer")
        if n:
            check(self.ctx.lib.ambc_memcpy_h2d(self.ctx.h, self.dev, self.ptr + offset, addr(data), n),
                  self.ctx.lib)

    def download(self, n=None, offset=0, out=None):
        """n bytes from offset into a new bytearray (or the writable buffer out)."""
        n = self.nbytes - offset if n is None else int(n)
        if offset + n > self.nbytes:
            raise ValueError("download past the end of the device buffer")
        buf = bytearray(n) if out is None else out
        if n:
            check(self.ctx.lib.ambc_memcpy_d2h(self.ctx.h, self.dev, addr(buf), self.ptr + offset, n),
                  self.ctx.lib)
        return buf


_ctx = None
_plugin_ctx = {}   # device list -> the per-chunk plugins' context on those devices


def default_context(devices=None):
    global _ctx
    with _lock:
        if _ctx is None or (devices and list(devices) != _ctx.devices):
            _ctx = Context(devices)
        return _ctx


def plugin_context(devices=None):
    """The per-chunk plugins' own context (methods.py): a plugin called from a
    host-codec callback while a walk holds the default context's lock (the
    reference-side binding scores the instance's own method objects on host
    threads) must not wait for that lock.  It lives on the devices given, else
    on those of the active default context (a rank process on GPU LOCAL_RANK
    keeps its plugins there), else on device 0 -- one context per device list."""
    with _lock:
        if devices is None:
            devices = _ctx.devices if _ctx is not None else [0]
        key = tuple(devices)
        if key not in _plugin_ctx:
            _plugin_ctx[key] = Context(list(key))
        return _plugin_ctx[key]
