"""Test-only stand-in for the third-party ``bitarray`` package.

Used ONLY by ``tests/golden/make_golden.py`` so that the read-only reference at
/root/reference can be imported in the build container to produce golden
vectors.  ``bitarray`` is not installed in this image and nothing here is part
of the product.  Only the handful of operations the reference's hot path uses
are provided (``adaptive_compressor.py:196-219,303-310``): the str/empty
constructors, ``frombytes``, slicing, ``to01``, ``append``, ``+``, ``len`` and
``tobytes`` (big-endian bit order, zero-padded to a whole byte).
"""


class bitarray:
    def __init__(self, init=None):
        if init is None:
            self._b = []
        elif isinstance(init, str):
            self._b = [1 if c == "1" else 0 for c in init if c in "01"]
        elif isinstance(init, (list, tuple)):
            self._b = [1 if x else 0 for x in init]
        else:
            raise TypeError("unsupported initialiser for bitarray stand-in")

    def frombytes(self, data):
        for byte in bytes(data):
            for k in range(7, -1, -1):
                self._b.append((byte >> k) & 1)

    def __getitem__(self, item):
        if isinstance(item, slice):
            return bitarray(self._b[item])
        return self._b[item]

    def __len__(self):
        return len(self._b)

    def __add__(self, other):
        return bitarray(self._b + list(other._b))

    def append(self, bit):
        self._b.append(1 if bit else 0)

    def to01(self):
        return "".join("1" if b else "0" for b in self._b)

    def tobytes(self):
        out = bytearray()
        for i in range(0, len(self._b), 8):
            chunk = self._b[i:i + 8]
            chunk = chunk + [0] * (8 - len(chunk))
            v = 0
            for b in chunk:
                v = (v << 1) | b
            out.append(v)
        return bytes(out)

    def search(self, other, limit=None):  # used only by marker_finder (off-path)
        pat = other._b
        res = []
        for i in range(len(self._b) - len(pat) + 1):
            if self._b[i:i + len(pat)] == pat:
                res.append(i)
                if limit is not None and len(res) >= limit:
                    break
        return res
