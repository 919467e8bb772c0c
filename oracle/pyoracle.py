"""ctypes driver of the CPU oracle (liboracle.so).  TEST INFRASTRUCTURE ONLY.

`OracleLoop` replays the reference frame loop (bmfr.cpp:417-485) with numpy
buffers laid out like the reference's (bmfr.cpp:315-347) and records every
inter-stage buffer of every frame.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class OracleCfg(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int),
        ("n_not_scaled", C.c_int), ("n_scaled", C.c_int),
        ("codes", C.c_int * 16),
        ("noise_amount", C.c_double),
        ("blend_alpha", C.c_float), ("second_blend_alpha", C.c_float), ("taa_blend_alpha", C.c_float),
        ("position_limit_sq", C.c_float), ("normal_limit_sq", C.c_float),
        ("half_tmp", C.c_int),
    ]


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = C.CDLL(LIB_PATH)
        P = C.c_void_p
        lib.oracle_num_blocks.restype = C.c_int
        lib.oracle_num_blocks.argtypes = [C.POINTER(OracleCfg)]
        lib.oracle_accumulate_noisy_data.argtypes = [C.POINTER(OracleCfg)] + [P] * 11 + [P, P, C.c_int]
        lib.oracle_fitter.argtypes = [C.POINTER(OracleCfg), P, P, P, C.c_int]
        lib.oracle_weighted_sum.argtypes = [C.POINTER(OracleCfg), P, P, P, P, P, C.c_int]
        lib.oracle_accumulate_filtered_data.argtypes = [C.POINTER(OracleCfg)] + [P] * 8 + [C.c_int]
        lib.oracle_taa.argtypes = [C.POINTER(OracleCfg), P, P, P, P, C.c_int]
        lib.oracle_f32_to_f16.restype = C.c_uint16
        lib.oracle_f32_to_f16.argtypes = [C.c_float]
        lib.oracle_f16_to_f32.restype = C.c_float
        lib.oracle_f16_to_f32.argtypes = [C.c_uint16]
        lib.oracle_threads.restype = C.c_int
        _lib = lib
    return _lib


def make_cfg(width, height, not_scaled, scaled, half_tmp, noise_amount=1e-2, blend_alpha=0.2,
             second_blend_alpha=0.1, taa_blend_alpha=0.2, position_limit_squared=0.01,
             normal_limit_squared=0.1) -> OracleCfg:
    c = OracleCfg()
    c.width, c.height = width, height
    c.n_not_scaled, c.n_scaled = len(not_scaled), len(scaled)
    codes = tuple(not_scaled) + tuple(scaled)
    for i, v in enumerate(codes):
        c.codes[i] = v
    c.noise_amount = noise_amount
    c.blend_alpha, c.second_blend_alpha, c.taa_blend_alpha = blend_alpha, second_blend_alpha, taa_blend_alpha
    # float(%g text) exactly as the kernel sees the -D value (bmfr.cpp:226-227).
    c.position_limit_sq = float(np.float32(float("%g" % position_limit_squared)))
    c.normal_limit_sq = float(np.float32(float("%g" % normal_limit_squared)))
    c.half_tmp = int(half_tmp)
    return c


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


class OracleLoop:
    """The reference frame loop on the CPU oracle."""

    def __init__(self, cfg: OracleCfg):
        self.lib = load()
        self.cfg = cfg
        W, H = cfg.width, cfg.height
        B = cfg.n_not_scaled + cfg.n_scaled + 3
        self.B = B
        G = self.lib.oracle_num_blocks(C.byref(cfg))
        self.G = G
        mw = 32 * ((W + 31) // 32) + 32
        mh = 32 * ((H + 31) // 32) + 32
        img = lambda: np.zeros(W * H * 3, np.float32)  # noqa: E731
        self.normals, self.positions, self.noisy = [img(), img()], [img(), img()], [img(), img()]
        self.out, self.result = [img(), img()], [img(), img()]
        self.spp = [np.zeros(W * H, np.uint8), np.zeros(W * H, np.uint8)]
        self.albedo, self.filtered, self.tone = img(), img(), img()
        self.prev_pixels = np.zeros(W * H * 2, np.float32)
        self.accept = np.zeros(W * H, np.uint8)
        self.tmp = np.zeros(mw * mh * B, np.uint16 if cfg.half_tmp else np.float32)
        self.weights = np.zeros(G * (B - 3) * 3, np.float32)
        self.mins_maxs = np.zeros(G * cfg.n_scaled * 2, np.float32)
        self.swapped = False

    def cur(self, pair):
        return pair[0] if self.swapped else pair[1]

    def prev(self, pair):
        return pair[1] if self.swapped else pair[0]

    def upload(self, noisy, normals, positions, albedo) -> None:
        self.cur(self.noisy)[:] = np.asarray(noisy, np.float32).reshape(-1)
        self.cur(self.normals)[:] = np.asarray(normals, np.float32).reshape(-1)
        self.cur(self.positions)[:] = np.asarray(positions, np.float32).reshape(-1)
        self.albedo[:] = np.asarray(albedo, np.float32).reshape(-1)

    def run_stages(self, prev_vp, jitter, frame: int, record=None) -> None:
        lib, c = self.lib, C.byref(self.cfg)
        vp = np.asarray(prev_vp, np.float32)
        jt = np.asarray(jitter, np.float32)
        lib.oracle_accumulate_noisy_data(
            c, _p(self.prev_pixels), _p(self.accept), _p(self.cur(self.normals)), _p(self.prev(self.normals)),
            _p(self.cur(self.positions)), _p(self.prev(self.positions)), _p(self.cur(self.noisy)),
            _p(self.prev(self.noisy)), _p(self.prev(self.spp)), _p(self.cur(self.spp)), _p(self.tmp),
            _p(vp), _p(jt), frame)
        if record is not None:
            record["tmp_noisy"] = self.tmp.copy()
        lib.oracle_fitter(c, _p(self.weights), _p(self.mins_maxs), _p(self.tmp), frame)
        lib.oracle_weighted_sum(c, _p(self.weights), _p(self.mins_maxs), _p(self.filtered),
                                _p(self.cur(self.normals)), _p(self.cur(self.positions)), frame)
        lib.oracle_accumulate_filtered_data(
            c, _p(self.filtered), _p(self.prev_pixels), _p(self.accept), _p(self.albedo), _p(self.tone),
            _p(self.cur(self.spp)), _p(self.prev(self.out)), _p(self.cur(self.out)), frame)
        lib.oracle_taa(c, _p(self.prev_pixels), _p(self.tone), _p(self.cur(self.result)),
                       _p(self.prev(self.result)), frame)
        if record is not None:
            record.update(
                tmp_fit=self.tmp.copy(), weights=self.weights.copy(), mins_maxs=self.mins_maxs.copy(),
                filtered=self.filtered.copy(), acc=self.cur(self.out).copy(), tone=self.tone.copy(),
                result=self.cur(self.result).copy(), spp=self.cur(self.spp).copy(),
                accept=self.accept.copy(), prev_pixel=self.prev_pixels.copy(),
                noisy=self.cur(self.noisy).copy())

    def swap(self) -> None:
        self.swapped = not self.swapped
