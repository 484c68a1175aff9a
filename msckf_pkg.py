"""Import shim for the product package.

The package directory is ``visual-inertial-odometry-msckf-stereo_amd/`` (the
name the build contract fixes), which is not a valid Python identifier.  This
module registers it in ``sys.modules`` as ``msckf_amd`` so that tests, the
bench and ``__graft_entry__`` can ``import msckf_amd``.
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "visual-inertial-odometry-msckf-stereo_amd")
NAME = "msckf_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod


load()
