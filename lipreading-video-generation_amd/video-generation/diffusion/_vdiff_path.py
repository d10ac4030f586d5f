"""Puts the vdiff package (lipreading-video-generation_amd/) on sys.path so the flat
reference module names (unet, utils, ...) resolve to the MI355X implementation."""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)
