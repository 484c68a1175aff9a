"""Any repo script against an alternative build of the library (A/B
experiments of compile-time kernel parameters: `make exp EXP=name
EXPFLAGS=-D...`).  GPU only.

    python tools/exp_run.py tools/exp/libmsckf_<name>.so tools/prop_sweep.py [script args]
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import msckf_pkg  # noqa: E402,F401
from msckf_amd import _lib  # noqa: E402

_lib.load_library(os.path.abspath(sys.argv[1]))   # cached: every Context of this process uses it
script = os.path.abspath(sys.argv[2])
sys.argv = [script] + sys.argv[3:]
sys.path.insert(0, os.path.dirname(script))
runpy.run_path(script, run_name="__main__")
