#!/usr/bin/env python3
"""SHA-256 digests of the reference kernels' outputs at BASELINE.json's sizes
(oracle/ref_configs.py FULL_REF_CONFIGS), for tests/test_gpu_reference_fullsize.py.
TEST INFRASTRUCTURE; runs on an MI355X with the reference compiled by
oracle/build_ref.py (strict build).  Inputs are libbmfr's GPU renderer of the
synthetic sequence, exactly as the test renders them.

Usage (GPU box): python tests/golden/make_fullsize_digests.py [--out FILE] [case ...]
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import ref_run  # noqa: E402
from ref_configs import FULL_REF_CONFIGS  # noqa: E402
from test_gpu_reference_fullsize import CASES, DIGESTS, cameras, frame_planes, sha  # noqa: E402


def make(case: str, build: str, half_in: int) -> dict:
    rc = FULL_REF_CONFIGS[build]
    ref = ref_run.RefLoop(rc, "strict")
    out = []
    for f in range(rc.frames):
        _, wide = frame_planes(rc, f, half_in)
        rec = {}
        ref.upload(wide["noisy"], wide["normals"], wide["positions"], wide["albedo"])
        ref.run_stages(*cameras(rc, f), f, record=rec)
        ref.swap()
        out.append({"result": sha(rec["result"]), "spp": sha(rec["spp"])})
    return {"build": build, "half_inputs": half_in, "mode": "strict", "seed": rc.seed, "frames": out}


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*")
    ap.add_argument("--out", default=DIGESTS)
    a = ap.parse_args()
    want = set(a.cases)
    d = {}
    if os.path.exists(a.out):
        with open(a.out) as fh:
            d = json.load(fh)
    for case, build, half_in in CASES:
        if want and case not in want:
            continue
        d[case] = make(case, build, half_in)
        print(case, "done", flush=True)
    with open(a.out, "w") as fh:
        json.dump(d, fh, indent=1)
