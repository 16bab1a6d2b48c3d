"""multimodal-financial-analysis-tool-using-paligemma_amd -- MI355X-native PaliGemma inference.

Put this directory on sys.path to use it as a drop-in for the reference's modules:
``import modeling_gemma, modeling_siglip, processing_paligemma, utils`` resolve to the
MI355X-native implementations here.
"""
import os as _os
import sys as _sys

_HERE = _os.path.dirname(_os.path.abspath(__file__))
if _HERE not in _sys.path:
    _sys.path.insert(0, _HERE)
