"""CPU-side checks of the C-ABI library (no compute calls without a GPU)."""
import ctypes as C
import os
import re

import pytest

from conftest import REPO, gpu_present


def header_functions():
    with open(os.path.join(REPO, "include", "ambc.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ambc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from ambc import _lib
    lib = _lib.load()
    decl = header_functions()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(lib, name), name
    assert set(decl) == set(_lib.EXPORTS)


def test_abi_version_and_bound():
    from ambc import _lib
    lib = _lib.load()
    assert lib.ambc_abi_version() == 3
    assert lib.ambc_compress_bound(0, 4096) == 16
    assert lib.ambc_compress_bound(4096, 4096) == 4096 + 18 + 16
    assert lib.ambc_compress_bound(4097, 4096) == 4097 + 36 + 16
    assert lib.ambc_compress_bound(1 << 32, 4096) == (1 << 32) + 18 * (1 << 20) + 16


def test_library_is_gfx950_code_object():
    path = os.path.join(REPO, "adaptive-compression_amd", "ambc", "libambc_hip.so")
    with open(path, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


@pytest.mark.skipif(gpu_present(), reason="checks the no-device failure path")
def test_no_device_fails_loudly():
    from ambc import _lib
    with pytest.raises(_lib.AmbcUnavailable):
        _lib.Context()
    lib = _lib.load()
    h = C.c_void_p()
    assert lib.ambc_init(None, 1, C.byref(h)) != 0
    assert "no" in _lib.last_error(lib).lower() or _lib.last_error(lib)


def test_missing_library_raises(tmp_path):
    from ambc import _lib
    with pytest.raises(_lib.AmbcUnavailable):
        _lib.load(str(tmp_path / "nope.so"))


def test_library_links_rccl():
    """The multi-GPU exchanges are RCCL inside the library (no PyTorch)."""
    import subprocess
    path = os.path.join(REPO, "adaptive-compression_amd", "ambc", "libambc_hip.so")
    out = subprocess.run(["ldd", path], capture_output=True, text=True).stdout
    assert "librccl" in out


def test_shard_range_host_only():
    from ambc import _lib
    lib = _lib.load()
    b, e = C.c_uint64(), C.c_uint64()
    assert lib.ambc_shard_range(32 << 30, 8192, 8, 7, C.byref(b), C.byref(e)) == 0
    assert (b.value, e.value) == (28 << 30, 32 << 30)
    assert lib.ambc_shard_range(100, 16, 0, 0, C.byref(b), C.byref(e)) == _lib.AMBC_E_INVAL


def test_binding_module_mirrors_the_abi():
    """integration/ambc_binding.py (the reference-side binding INTEGRATION.md
    quotes) declares the same struct layouts as include/ambc.h / ambc._lib, loads
    the library and, without a device, fails loudly at bind time."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "integration"))
    import ambc_binding as B
    from ambc import _lib
    for a, b in ((B.Params, _lib.Params), (B.Stats, _lib.Stats), (B.HostChunk, _lib.HostChunk)):
        assert C.sizeof(a) == C.sizeof(b)
        assert [f[0] for f in a._fields_] == [f[0] for f in b._fields_]
    from ambc.hostcodecs import HostCodecs
    assert C.sizeof(B.HostCodecs) == C.sizeof(HostCodecs)
    lib = B.load_library()
    assert lib.ambc_compress_bound(4096, 4096) == 4096 + 18 + 16
    with open(os.path.join(REPO, "INTEGRATION.md")) as f:
        doc = f.read()
    assert "integration/ambc_binding.py" in doc
    if not gpu_present():
        class K:
            def _adaptive_compress(self, d):
                return d

            def _adaptive_decompress(self, d, n):
                return d
        with pytest.raises(RuntimeError):
            B.bind(K)
        assert K._adaptive_compress(None, b"x") == b"x"


def test_integration_doc_quotes_the_binding_verbatim():
    with open(os.path.join(REPO, "INTEGRATION.md")) as f:
        doc = f.read()
    with open(os.path.join(REPO, "integration", "ambc_binding.py")) as f:
        src = f.read()
    assert "```python\n" + src + "```" in doc


def test_library_never_registers_caller_memory():
    """DESIGN §9 (round 6): caller buffers move through the library's own pinned
    staging only; the shipped library imports no host-registration entry point,
    so no caller page is ever mapped into the GPU."""
    with open(os.path.join(REPO, "adaptive-compression_amd", "ambc", "libambc_hip.so"), "rb") as f:
        blob = f.read()
    for sym in (b"hipHostRegister", b"hipHostUnregister", b"hsa_amd_memory_lock"):
        assert sym not in blob, sym
