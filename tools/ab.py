#!/usr/bin/env python3
"""A/B timing of libbmfr builds on the GPU.

  build (here):   python tools/ab.py build NAME="-DFLAG=1 ..." ...   -> bmfr_amd/libbmfr_NAME.so
                  python tools/ab.py build-rev NAME=GITREV ...         (the library of another revision)
  time (GPU box): python tools/ab.py time [W H] NAME ...             ("base" = libbmfr.so)

Each timing runs in its own process (BMFR_LIB selects the library): frames
0..44 of the synthetic sequence per frame, K1 / K2 means over frames 5..44
from libbmfr's profiling events, rounds interleaved to even out drift."""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(specs):
    from bmfr_amd import _build as b
    b.build()

    def one(spec):
        name, flags = spec.split("=", 1)
        return b.build(force=True, variant=name, extra_flags=flags.split())

    with cf.ThreadPoolExecutor(max_workers=2) as ex:
        for lib in ex.map(one, specs):
            print(lib)


def build_rev(specs):
    """NAME=REV: libbmfr_NAME.so from the library sources of git revision REV
    (csrc/ + include/, the build id of that tree), for A/B timing against
    the working tree (timed with BMFR_ALLOW_FOREIGN_BUILD=1)."""
    import shutil
    import tempfile
    from bmfr_amd import _build as b
    for spec in specs:
        name, rev = spec.split("=", 1)
        with tempfile.TemporaryDirectory() as d:
            subprocess.run(f"git -C {ROOT} archive {rev} bmfr_amd/csrc include | tar -x -C {d}", shell=True,
                           check=True)
            objdir = os.path.join(d, "obj")
            os.makedirs(objdir)
            csrc = os.path.join(d, "bmfr_amd", "csrc")
            srcs = sorted(f for f in os.listdir(csrc) if f.endswith(".hip"))
            with open(os.path.join(objdir, "bmfr_build_id.h"), "w") as f:
                f.write(f'#define BMFR_BUILD_ID "rev-{rev}"\n')

            def one(src):
                obj = os.path.join(objdir, src.replace(".hip", ".o"))
                subprocess.run([b.HIPCC, *b.FLAGS, "-I", objdir, "-c", os.path.join(csrc, src), "-o", obj],
                               check=True)
                return obj
            with cf.ThreadPoolExecutor(max_workers=len(srcs)) as ex:
                objs = list(ex.map(one, srcs))
            out = os.path.join(ROOT, "bmfr_amd", f"libbmfr_{name}.so")
            subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp", *objs, "-ldl"],
                           check=True)
            shutil.move(out + ".tmp", out)
            print(out)


def time_one(W, H, frames=45, first=5):
    import numpy as np
    import torch

    import bmfr_amd
    # AB_FAST_FIT=1: time the fast_fit configuration; AB_F32TMP=1: f32 tmp_data;
    # AB_CFG5=1: BASELINE config 5 (third-order features, half input planes)
    cfg5 = os.environ.get("AB_CFG5") == "1"
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H,
                                                fast_fit=int(os.environ.get("AB_FAST_FIT", "0")),
                                                use_half_precision_in_tmp_data=0 if os.environ.get("AB_F32TMP") == "1"
                                                else 1,
                                                scaled=bmfr_amd.SCALED_THIRD_ORDER if cfg5 else bmfr_amd.SCALED_DEFAULT,
                                                input_half=int(cfg5)))
    fr = [bmfr_amd.synth_frame_device(W, H, f) for f in range(frames)]
    if cfg5:
        fr = [{k: (v.half() if k in ("noisy", "normals", "positions", "albedo") else v) for k, v in x.items()}
              for x in fr]
    den.set_profiling(True, capacity=frames, stride=1)
    for f in range(frames):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        den.process_frame(fr[f]["noisy"], fr[f]["normals"], fr[f]["positions"], fr[f]["albedo"], vp, jit, f)
    torch.cuda.synchronize()
    p = den.profile()[first:]
    print(f"RESULT {np.mean([x[1] for x in p]):.4f} {np.mean([x[2] for x in p]):.4f}", flush=True)


def time_all(W, H, names, rounds=2):
    res = {n: [] for n in names}
    for _ in range(rounds):
        for n in names:
            env = dict(os.environ, BMFR_LIB="" if n == "base" else n, BMFR_ALLOW_FOREIGN_BUILD="1",
                       BMFR_ALLOW_PROBE="1")
            out = subprocess.run([sys.executable, __file__, "one", str(W), str(H)], env=env, capture_output=True,
                                 text=True, timeout=300)
            line = [x for x in out.stdout.splitlines() if x.startswith("RESULT")]
            if not line:
                print(n, "FAILED", out.stderr[-2000:], flush=True)
                continue
            k1, k2 = map(float, line[0].split()[1:])
            res[n].append((k1, k2))
            print(f"{n:20s} K1 {k1:.4f} ms  K2 {k2:.4f} ms", flush=True)
    print("--- means")
    for n, v in res.items():
        if v:
            print(f"{n:20s} K1 {sum(x[0] for x in v) / len(v):.4f}  K2 {sum(x[1] for x in v) / len(v):.4f}")


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "build":
        build(sys.argv[2:])
    elif cmd == "build-rev":
        build_rev(sys.argv[2:])
    elif cmd == "one":
        time_one(int(sys.argv[2]), int(sys.argv[3]))
    else:
        args = sys.argv[2:]
        W, H = (int(args[0]), int(args[1])) if args and args[0].isdigit() else (3840, 2160)
        names = [a for a in args if not a.isdigit()]
        time_all(W, H, names)
