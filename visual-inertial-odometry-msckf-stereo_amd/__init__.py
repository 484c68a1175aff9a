"""msckf_amd -- MI355X-native MSCKF stereo-VIO EKF update path.

Host side (this package, Python) mirrors the reference filter API
``MSCKF.imu_callback`` / ``MSCKF.feature_callback`` (MSCKF/msckf.py:166-233);
all filter arithmetic runs in hand-written HIP kernels for gfx950 behind the
C-ABI declared in ``include/msckf_hip.h`` (``csrc/msckf_hip.hip``), loaded with
ctypes.  There is no CPU fallback: if ``libmsckf_hip.so`` is missing or no GPU
is present, the filter raises.
"""
from .config import FilterConfig, OptimizationConfig, CHI2_05, chi2_threshold  # noqa: F401
from .msckf import MSCKF, VioResult  # noqa: F401
from ._lib import Context, MsckfError, load_library  # noqa: F401

__all__ = ["FilterConfig", "OptimizationConfig", "CHI2_05", "chi2_threshold", "MSCKF",
           "VioResult", "Context", "MsckfError", "load_library"]
