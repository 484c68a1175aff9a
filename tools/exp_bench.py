"""bench.py against an alternative build of the library (A/B experiments of
compile-time kernel parameters: `make exp EXP=name EXPFLAGS=-D...`).  GPU only.

    python tools/exp_bench.py tools/exp/libmsckf_<name>.so [bench.py args]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
from msckf_amd import _lib  # noqa: E402

lib = os.path.abspath(sys.argv[1])
_lib.load_library(lib)   # cached: every Context of this process uses it
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
