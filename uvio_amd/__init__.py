"""uvio_amd — MI355X-native implementation of the uvio/OpenVINS per-frame hot path
(track -> propagate -> MSCKF/SLAM/UWB update -> EKF update) behind a C ABI (include/uvio_hp.h).

The estimator runs in ``libuvio_hp.so`` (host C++ orchestration + gfx950 HIP kernels).  This package
only binds it: ``VioManager`` mirrors ov_msckf::VioManager / uvio::UVioManager.
"""
from . import _native  # noqa: F401
from .manager import VioManager, apply_overrides, compress, ekf_update, load_options, undistort  # noqa: F401

__all__ = ["VioManager", "load_options", "apply_overrides", "ekf_update", "compress", "undistort"]
