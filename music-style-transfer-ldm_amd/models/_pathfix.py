"""Make `ldm_amd` importable whichever way the drop-in modules are imported:
`import models.model` (package root on sys.path) or `from model import LDM` (models/ on sys.path,
as the reference does at model.py:7-8)."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
