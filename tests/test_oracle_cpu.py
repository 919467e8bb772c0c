"""CPU-side checks of the oracle (no GPU): binary16 conversion, and the oracle
against the golden vectors produced by the reference kernels themselves
(tests/golden/*.npz, made by tests/golden/make_golden.py on an MI355X)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import pyoracle
from ref_configs import REF_CONFIGS
from seq_util import EXACT_KEYS, POWR_KEYS, digest, frame_inputs, input_digest, run_loop, sample_idx

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_half_to_float_exhaustive():
    lib = pyoracle.load()
    h = np.arange(65536, dtype=np.uint16)
    want = h.view(np.float16).astype(np.float32)
    got = np.array([lib.oracle_f16_to_f32(int(x)) for x in h], np.float32)
    ok = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    assert ok.all()


def test_float_to_half_round_to_nearest_even():
    lib = pyoracle.load()
    rng = np.random.default_rng(1)
    bits = np.concatenate([
        rng.integers(0, 2 ** 32, 200000, dtype=np.uint64).astype(np.uint32),
        # values around every half rounding boundary and the overflow edge
        (np.arange(0, 65536, dtype=np.uint32).view(np.float32) if False else np.array([], np.uint32)),
    ])
    f = bits.view(np.float32)
    edge = np.array([65504, 65519.99, 65520, 65536, 6.1e-5, 5.96e-8, 2.98e-8, 2.99e-8, 1e-9, -65520,
                     0.0, -0.0, np.inf, -np.inf], np.float32)
    f = np.concatenate([f, edge, (np.arange(-70000, 70000, 0.37)).astype(np.float32)])
    want = f.astype(np.float16).view(np.uint16)
    got = np.array([lib.oracle_f32_to_f16(float(x)) for x in f], np.uint16)
    nan = np.isnan(f)
    assert (got[~nan] == want[~nan]).all(), f[~nan][got[~nan] != want[~nan]][:10]
    assert ((got[nan] & 0x7c00) == 0x7c00).all() and ((got[nan] & 0x3ff) != 0).all()


def golden_names():
    return sorted(n[:-4] for n in os.listdir(GOLDEN) if n.endswith(".npz")) if os.path.isdir(GOLDEN) else []


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference_golden_vectors(name):
    rc = REF_CONFIGS[name]
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    frames = meta["frames"]
    for f in range(frames):
        assert input_digest(frame_inputs(rc, f)) == meta["inputs"][f], \
            f"synthetic inputs of frame {f} changed: regenerate tests/golden with make_golden.py"
    cfg = pyoracle.make_cfg(rc.width, rc.height, rc.not_scaled, rc.scaled, rc.half_tmp)
    got = run_loop(pyoracle.OracleLoop(cfg), rc, frames)
    for f, g in enumerate(got):
        np.testing.assert_array_equal(g["weights"], z[f"weights_{f}"], err_msg=f"frame {f} weights")
        np.testing.assert_array_equal(g["mins_maxs"], z[f"mins_maxs_{f}"], err_msg=f"frame {f} mins_maxs")
        bad = [k for k in EXACT_KEYS if digest(g[k]) != meta["digests"][f][k]]
        assert not bad, f"frame {f}: oracle differs from the reference in {bad}"
        for k in POWR_KEYS:
            ref = z[f"{k}_sample_{f}"].astype(np.float64)
            mine = g[k][sample_idx(g[k].size)].astype(np.float64)
            assert np.abs(mine - ref).max() <= 4e-7, (f, k, np.abs(mine - ref).max())
            st = meta["stats"][f][k]
            a = g[k].astype(np.float64)
            assert abs(a.sum() - st["sum"]) <= 1e-6 * a.size, (f, k)
