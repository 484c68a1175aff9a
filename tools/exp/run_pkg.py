"""Runs a tool against an alternative copy of the Python package (A/B of host
code): python tools/exp/run_pkg.py PKG_DIR tools/bench_sequences.py [args]"""
import importlib.util
import os
import runpy
import sys

pkg = os.path.abspath(sys.argv[1])
spec = importlib.util.spec_from_file_location("msckf_amd", os.path.join(pkg, "__init__.py"),
                                              submodule_search_locations=[pkg])
mod = importlib.util.module_from_spec(spec)
sys.modules["msckf_amd"] = mod
spec.loader.exec_module(mod)
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
