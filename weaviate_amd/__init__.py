"""weaviate_amd -- MI355X-native (gfx950) backend for Weaviate's vector-scoring
hot path: flat fp32 scan, BQ Hamming scan, PQ ADC scan and the top-k that
feeds rescoring.  The product is the C-ABI library ``libwvgpu.so``
(include/wvgpu.h, sources in weaviate_amd/csrc); the Python modules are thin
mirrors of the reference's Go interfaces used by the tests and the bench.
"""
from ._lib import LIB_PATH, WvgError, load  # noqa: F401

__all__ = ["LIB_PATH", "WvgError", "load"]
