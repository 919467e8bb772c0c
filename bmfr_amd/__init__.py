"""bmfr_amd -- MI355X-native BMFR (blockwise multi-order feature regression)
denoiser.  Hot path: libbmfr.so (HIP kernels for gfx950 behind the C ABI of
include/bmfr.h); this package is the host-side mirror of the reference's
frame driver (/root/reference/opencl/bmfr.cpp)."""
from ._lib import BmfrError, StaleLibraryError, build_id, load  # noqa: F401
from .pipeline import (BmfrConfig, Denoiser, StagePipeline, SCALED_DEFAULT,  # noqa: F401
                       SCALED_THIRD_ORDER, NOT_SCALED_DEFAULT, synth_camera, synth_frame_device, synth_region_device,
                       synth_frame_host, hip_memcpy_d2d)

__all__ = ["BmfrConfig", "Denoiser", "StagePipeline", "BmfrError", "StaleLibraryError", "build_id", "load", "synth_camera",
           "synth_frame_device", "synth_frame_host", "synth_region_device"]
