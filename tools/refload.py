"""Load the reference MSCKF (read-only, /root/reference/MSCKF) as the golden
oracle IN THE BUILD CONTAINER ONLY.

numba and cv2 are not installed here; both are replaced by in-memory stub
modules (no files are written anywhere): ``numba.jit`` becomes the identity
decorator (the jitted bodies are plain numpy, so semantics are unchanged up to
LAPACK rounding), and ``cv2`` only provides the three integer constants that
config.py:37-44 reads.  Bytecode writing is disabled so nothing lands in the
read-only reference tree.  Nothing from the reference is copied into this repo.
"""
import sys
import types

REF_DIR = "/root/reference/MSCKF"


def load_reference():
    sys.dont_write_bytecode = True
    if "numba" not in sys.modules:
        nb = types.ModuleType("numba")
        nb.jit = lambda *a, **k: (lambda f: f)
        sys.modules["numba"] = nb
    if "cv2" not in sys.modules:
        cv = types.ModuleType("cv2")
        cv.TERM_CRITERIA_EPS, cv.TERM_CRITERIA_COUNT, cv.OPTFLOW_USE_INITIAL_FLOW = 2, 1, 4
        sys.modules["cv2"] = cv
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import config, msckf, feature, utils, jit_utils  # noqa: E401
    return types.SimpleNamespace(config=config, msckf=msckf, feature=feature,
                                 utils=utils, jit_utils=jit_utils)


def fresh_filter(ref):
    """A new reference MSCKF with its class-level globals reset (quirk Q7)."""
    ref.msckf.IMUState._vio_next_id__ = 0
    ref.feature.Feature._vio_next_id__ = 0
    cfg = ref.config.ConfigEuRoC()
    return ref.msckf.MSCKF(cfg), cfg
