"""Import helpers for the test-suite (test infrastructure)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "okvis2-x_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
