"""tools/profile_frame.py against an alternative build of the library (A/B of
the per-frame path on one box).  GPU only.

    python tools/exp_frame.py tools/exp/libmsckf_<name>.so [profile_frame.py args]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import msckf_pkg  # noqa: E402,F401
from msckf_amd import _lib  # noqa: E402

_lib.load_library(os.path.abspath(sys.argv[1]))   # cached: every Context of this process uses it
sys.argv = [os.path.join(ROOT, "tools", "profile_frame.py")] + sys.argv[2:]
import profile_frame  # noqa: E402

profile_frame.main()
