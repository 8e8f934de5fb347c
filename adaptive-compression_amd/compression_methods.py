"""Drop-in module name of the reference's plugin module (GPU-backed)."""
from ambc.methods import (CompressionMethod, DeltaCompression,  # noqa: F401
                          DictionaryCompression, HuffmanCompression, NoCompression,
                          RLECompression)
