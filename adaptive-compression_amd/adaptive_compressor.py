"""Drop-in module name of the reference (``from adaptive_compressor import
AdaptiveCompressor``) backed by the MI355X engine in ``ambc``."""
from ambc.compressor import AdaptiveCompressor  # noqa: F401
