"""Test-side loader for the product package (reed-solomon-cc_amd/reedsol_amd)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "reed-solomon-cc_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import reedsol_amd  # noqa: E402

HEADER = os.path.join(ROOT, "include", "reedsol.h")
