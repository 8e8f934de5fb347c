"""Drop-in for the reference's ``main.py`` CLI (compress / decompress / analyze)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ambc.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
