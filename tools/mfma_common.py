"""Shared by tools/mfma_experiment.py and tests/test_gpu_mfma_wy.py: the
compact-WY fitter library and a stage pipeline run with a replaceable fitter."""
import ctypes as C

import torch

from bmfr_amd._lib import check, floats
from bmfr_amd.pipeline import _ptr


def load_wy(path):
    wy = C.CDLL(path)
    wy.wy_fitter.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.c_void_p, C.c_int,
                             C.c_int]
    return wy


def run_stages(sp, vp, jit, f, fitter):
    """StagePipeline.run_stages with the fitter stage replaced by `fitter(sp, f)`."""
    lib, h, st = sp.lib, sp.handle, torch.cuda.current_stream().cuda_stream
    check(lib.bmfr_accumulate_noisy_data(
        h, st, _ptr(sp.prev_pixels), _ptr(sp.accept), _ptr(sp.cur(sp.normals)), _ptr(sp.prev(sp.normals)),
        _ptr(sp.cur(sp.positions)), _ptr(sp.prev(sp.positions)), _ptr(sp.cur(sp.noisy)), _ptr(sp.prev(sp.noisy)),
        _ptr(sp.prev(sp.spp)), _ptr(sp.cur(sp.spp)), _ptr(sp.tmp_data), floats(vp, 16), floats(jit, 2), f), "acc")
    fitter(sp, f)
    check(lib.bmfr_weighted_sum(h, st, _ptr(sp.weights), _ptr(sp.mins_maxs), _ptr(sp.filtered),
                                _ptr(sp.cur(sp.normals)), _ptr(sp.cur(sp.positions)), _ptr(sp.cur(sp.noisy)), f), "ws")
    check(lib.bmfr_accumulate_filtered_data(
        h, st, _ptr(sp.filtered), _ptr(sp.prev_pixels), _ptr(sp.accept), _ptr(sp.albedo), _ptr(sp.tone_mapped),
        _ptr(sp.cur(sp.spp)), _ptr(sp.prev(sp.out)), _ptr(sp.cur(sp.out)), f), "af")
    check(lib.bmfr_taa(h, st, _ptr(sp.prev_pixels), _ptr(sp.tone_mapped), _ptr(sp.cur(sp.result)),
                       _ptr(sp.prev(sp.result)), f), "taa")
