#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the reference's own
kernels.  TEST INFRASTRUCTURE; runs on an MI355X (the reference .cl compiled
by oracle/build_ref.py in strict mode, driven by oracle/ref_run.py).

Inputs are the deterministic synthetic frames of libbmfr's host generator;
their SHA-256 is stored so a changed generator is detected instead of
silently compared.  Per frame the fixture keeps
  * SHA-256 of every bit-exact buffer (seq_util.EXACT_KEYS),
  * weights and mins_maxs in full,
  * tone / result (powr-dependent) as float64 sums and an 8192-element
    strided sample (compared with a tolerance on the CPU side).

Usage (GPU box): python tests/golden/make_golden.py [--out DIR] [config ...]
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ref_run  # noqa: E402
from ref_configs import REF_CONFIGS  # noqa: E402
from seq_util import EXACT_KEYS, POWR_KEYS, digest, frame_inputs, input_digest, run_loop, sample_idx  # noqa: E402


def make(name: str, out_dir: str = HERE) -> str:
    rc = REF_CONFIGS[name]
    frames = run_loop(ref_run.RefLoop(rc, "strict"), rc, rc.frames,
                      to_device=lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda(),
                      sync=torch.cuda.synchronize)
    meta = {"config": name, "frames": rc.frames, "mode": "strict", "seed": rc.seed,
            "inputs": [input_digest(frame_inputs(rc, f)) for f in range(rc.frames)],
            "digests": [{k: digest(fr[k]) for k in EXACT_KEYS} for fr in frames],
            "stats": []}
    arrays = {}
    for f, fr in enumerate(frames):
        arrays[f"weights_{f}"] = fr["weights"]
        arrays[f"mins_maxs_{f}"] = fr["mins_maxs"]
        st = {}
        for k in POWR_KEYS:
            a = fr[k].astype(np.float64)
            st[k] = {"sum": float(a.sum()), "sumsq": float((a * a).sum())}
            arrays[f"{k}_sample_{f}"] = fr[k][sample_idx(fr[k].size)]
        meta["stats"].append(st)
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"{name}.npz")
    np.savez_compressed(path, meta=np.frombuffer(json.dumps(meta).encode(), np.uint8), **arrays)
    return path


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*")
    ap.add_argument("--out", default=HERE, help="output directory (default: tests/golden)")
    a = ap.parse_args()
    for n in a.configs or list(REF_CONFIGS):
        print(make(n, a.out), flush=True)
