"""ctypes binding of libbmfr.so (include/bmfr.h).

torch is imported first on purpose: torch ships its own libamdhip64.so
(soname libamdhip64.so.7).  Loaded in this order, libbmfr's NEEDED entry
resolves to torch's copy, so device pointers and streams are shared with
torch; loading libbmfr first would map a second HIP runtime.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# BMFR_LIB=NAME selects libbmfr_NAME.so: the diagnostic build (diag, in-kernel
# timestamps) or an A/B variant build (bmfr_amd/_build.py --variant).
_variant = os.environ.get("BMFR_LIB", "")
LIB_PATH = os.path.join(HERE, f"libbmfr_{_variant}.so" if _variant else "libbmfr.so")

MAX_FEATURES = 16

# bmfr_feature
FEATURE_ONE, NORMAL_X, NORMAL_Y, NORMAL_Z = 0, 1, 2, 3
POSITION_X, POSITION_Y, POSITION_Z = 4, 5, 6
POSITION_X2, POSITION_Y2, POSITION_Z2 = 7, 8, 9
POSITION_X3, POSITION_Y3, POSITION_Z3 = 10, 11, 12

STATUS = {0: "ok", 1: "invalid argument", 2: "unsupported configuration",
          3: "out of device memory", 4: "HIP runtime error", 5: "no HIP device",
          6: "reprojection reached past the tile halo",
          7: "a kernel's bounded wait for another work-group gave up"}
HALO_EXCEEDED = 6
SYNC_TIMEOUT = 7


class BmfrError(RuntimeError):
    def __init__(self, status: int, what: str):
        super().__init__(f"{what}: {STATUS.get(status, status)} (status {status})")
        self.status = status


class Config(C.Structure):
    _fields_ = [
        ("image_width", C.c_int), ("image_height", C.c_int),
        ("features_not_scaled", C.c_int), ("features_scaled", C.c_int),
        ("feature_buffers", C.c_int * MAX_FEATURES),
        ("noise_amount", C.c_double),
        ("blend_alpha", C.c_float), ("second_blend_alpha", C.c_float),
        ("taa_blend_alpha", C.c_float),
        ("position_limit_squared", C.c_double), ("normal_limit_squared", C.c_double),
        ("use_half_precision_in_tmp_data", C.c_int),
        ("tile_x", C.c_int), ("tile_y", C.c_int), ("tile_width", C.c_int), ("tile_height", C.c_int),
        ("tile_halo", C.c_int),
        ("input_half", C.c_int),
        ("library_powr", C.c_int),
        ("fast_fit", C.c_int),
    ]


class Sizes(C.Structure):
    _fields_ = [
        ("buffer_count", C.c_int), ("r_edge", C.c_int),
        ("workset_width", C.c_int), ("workset_height", C.c_int),
        ("workset_with_margins_width", C.c_int), ("workset_with_margins_height", C.c_int),
        ("blocks", C.c_int),
        ("tmp_data_bytes", C.c_size_t), ("weights_bytes", C.c_size_t),
        ("mins_maxs_bytes", C.c_size_t), ("image_bytes", C.c_size_t),
        ("region_x", C.c_int), ("region_y", C.c_int), ("region_width", C.c_int), ("region_height", C.c_int),
        ("region_bytes", C.c_size_t),
        ("frame_launches", C.c_int),
    ]


class FrameInputs(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("noisy", "normals", "positions", "albedo", "prev_normals", "prev_positions")]


class StateView(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("noisy_accumulated", "spp", "filtered_accumulated", "tone_mapped",
                 "prev_frame_pixel", "accept", "result")]


class FrameProfile(C.Structure):
    _fields_ = [("frame_number", C.c_int), ("fused_block_ms", C.c_float), ("taa_ms", C.c_float),
                ("total_ms", C.c_float)]


# name -> (restype, argtypes); the full exported surface of include/bmfr.h.
_P, _I, _F16, _F2 = C.c_void_p, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)
SIGNATURES = {
    "bmfr_config_default": (None, [C.POINTER(Config), _I, _I]),
    "bmfr_config_sizes": (_I, [C.POINTER(Config), C.POINTER(Sizes)]),
    "bmfr_status_string": (C.c_char_p, [_I]),
    "bmfr_last_hip_error": (_I, []),
    "bmfr_build_id": (C.c_char_p, []),
    "bmfr_create": (_I, [C.POINTER(Config), _I, C.POINTER(_P)]),
    "bmfr_destroy": (_I, [_P]),
    "bmfr_get_sizes": (_I, [_P, C.POINTER(Sizes)]),
    "bmfr_accumulate_noisy_data": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                        _F16, _F2, _I]),
    "bmfr_fitter": (_I, [_P, _P, _P, _P, _P, _I]),
    "bmfr_weighted_sum": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I]),
    "bmfr_accumulate_filtered_data": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I]),
    "bmfr_taa": (_I, [_P, _P, _P, _P, _P, _P, _I]),
    "bmfr_process_frame": (_I, [_P, _P, C.POINTER(FrameInputs), _F16, _F2, _I]),
    "bmfr_process_frame_interior": (_I, [_P, _P, C.POINTER(FrameInputs), _F16, _F2, _I]),
    "bmfr_halo_copy": (_I, [_P, _P, C.POINTER(C.c_int), _I, _P, _I, C.POINTER(C.c_size_t)]),
    "bmfr_halo_need": (_I, [C.POINTER(Config), _I, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "bmfr_process_sequence": (_I, [_P, _P, _I, C.POINTER(FrameInputs), _F16, _F2, _I, C.POINTER(_P)]),
    "bmfr_process_frame_border": (_I, [_P, _P, C.POINTER(FrameInputs), _F16, _F2, _I]),
    "bmfr_output": (_P, [_P]),
    "bmfr_halo_status": (_I, [_P, C.POINTER(C.c_uint)]),
    "bmfr_frame_status": (_I, [_P]),
    "bmfr_state": (_I, [_P, _I, C.POINTER(StateView)]),
    "bmfr_set_profiling": (_I, [_P, _I, _I]),
    "bmfr_set_profiling_stride": (_I, [_P, _I]),
    "bmfr_get_profile": (_I, [_P, C.POINTER(FrameProfile), _I, C.POINTER(_I)]),
    "bmfr_halo_plan": (_I, [C.POINTER(Config), C.POINTER(_I), _I, _I, _I, C.POINTER(_I), C.POINTER(_I),
                            C.POINTER(_I), C.POINTER(_I), _I, C.POINTER(_I)]),
    "bmfr_comm_unique_id": (_I, [C.c_char_p]),
    "bmfr_comm_create": (_I, [C.c_char_p, _I, _I, _I, C.POINTER(_P)]),
    "bmfr_comm_create_all": (_I, [_I, C.POINTER(_I), C.POINTER(_P)]),
    "bmfr_comm_destroy": (_I, [_P]),
    "bmfr_exchange_create": (_I, [_P, C.POINTER(Config), C.POINTER(_I), _I, _I, _P, C.POINTER(_P)]),
    "bmfr_exchange_run": (_I, [_P, _P, _I]),
    "bmfr_exchange_run_all": (_I, [C.POINTER(_P), _I, C.POINTER(_P), _I]),
    "bmfr_exchange_bytes": (_I, [_P, _I, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "bmfr_exchange_destroy": (_I, [_P]),
    "bmfr_synth_camera": (None, [_I, _I, _I, _F16, _F2]),
    "bmfr_debug_stamps": (_I, [_P, _P, C.c_size_t]),  # include/bmfr_debug.h
    "bmfr_debug_sync": (_I, [_P, _I, _I]),  # include/bmfr_debug.h
    "bmfr_debug_frame_launches": (_I, [_P, _I]),
    "bmfr_synth_frame_host": (_I, [_I, _I, _I, C.c_uint32, _P, _P, _P, _P, _P]),
    "bmfr_synth_frame_device": (_I, [_I, _I, _I, C.c_uint32, _P, _P, _P, _P, _P, _P]),
    "bmfr_synth_region_device": (_I, [_I, _I, _I, _I, _I, _I, _I, C.c_uint32, _P, _P, _P, _P, _P, _P]),
}

_lib = None


class StaleLibraryError(ImportError):
    """The library on disk was not built from the sources in this tree."""


def check_build_id(lib: C.CDLL, path: str) -> str:
    """Refuse a library built from other sources than this tree's (the id is
    the SHA-256 of csrc/ + include/, _build.source_hash) or a probe build
    (BMFR_PROBE_* flags: timing experiments with knowingly wrong results)
    unless BMFR_ALLOW_PROBE=1.  Never rebuilds: on the GPU box the library
    that runs must be the one shipped with the tree."""
    from . import _build
    if not hasattr(lib, "bmfr_build_id"):
        raise StaleLibraryError(f"{path} predates bmfr_build_id(): rebuild it (__graft_entry__.build())")
    lib.bmfr_build_id.restype = C.c_char_p
    got = lib.bmfr_build_id().decode()
    want = _build.source_hash()
    # BMFR_ALLOW_FOREIGN_BUILD=1: A/B timing of a library built from another
    # revision's sources (tools/ab.py build-rev); never set by tests or bench.py
    if got.split("+")[0] != want and os.environ.get("BMFR_ALLOW_FOREIGN_BUILD") != "1":
        raise StaleLibraryError(f"{path} was built from other sources (build id {got[:16]}..., tree "
                                f"{want[:16]}...): rebuild it (__graft_entry__.build())")
    if "BMFR_PROBE" in got and os.environ.get("BMFR_ALLOW_PROBE") != "1":
        raise StaleLibraryError(f"{path} is a probe build ({got.split('+', 1)[1]}): its results are not "
                                f"guaranteed; set BMFR_ALLOW_PROBE=1 to time it anyway")
    return got


def build_id() -> str:
    return load().bmfr_build_id().decode()


def load() -> C.CDLL:
    """Load libbmfr.so; raises if it has not been built, or was built from
    other sources (no silent fallback, no rebuild)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = C.CDLL(LIB_PATH)
        check_build_id(lib, LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if _variant and not hasattr(lib, name):
                continue  # an A/B build of older sources may predate a symbol
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        raise BmfrError(status, what)


def floats(values, n: int):
    arr = (C.c_float * n)(*[float(v) for v in values])
    return arr
