#!/usr/bin/env python3
"""bench.py with K1 workgroups per CU forced (tuning key 1): python tools/bench_gpc.py G [bench args]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# A/B knobs (wvgx_set_tuning) exist only in the tools build: make -C weaviate_amd/csrc tools
os.environ.setdefault("WVG_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libwvgpu_tools.so"))
g = int(sys.argv[1])
sys.argv = ["bench.py"] + sys.argv[2:]
import torch  # noqa: E402

torch.cuda.init()  # torch's HIP context first (as bench.py does before the library's)
from weaviate_amd import _lib  # noqa: E402

lib = _lib.load()
lib.wvgx_set_tuning.restype = ctypes.c_int
lib.wvgx_set_tuning.argtypes = [ctypes.c_int, ctypes.c_int]
lib.wvgx_set_tuning(1, g)
import bench  # noqa: E402

bench.main()
