"""Drop-in module name of the reference's history analyzer (records only)."""
from ambc.analyzer import CompressionAnalyzer  # noqa: F401
