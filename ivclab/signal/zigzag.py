"""ivclab.signal.zigzag (reference ivclab/signal/zigzag.py:3-26)."""
from ivclab_amd.signal.zigzag import zigzag_scan

__all__ = ["zigzag_scan"]
