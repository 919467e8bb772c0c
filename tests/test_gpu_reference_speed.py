"""The reference's own kernels and libbmfr timed on the same MI355X, on the
same synthetic frames (informative: BASELINE.md §5 quotes the figures).

REF  /root/reference/opencl/bmfr.cl compiled by oracle/build_ref.py with the
     reference's own options (the "default" build: bmfr.cpp's -D set, no
     extra flags), launched as tasks() launches it (bmfr.cpp:417-476):
     accumulate_noisy_data over the margin grid in 8x8 work-groups, the
     fitter one 256-item work-group per block, weighted_sum /
     accumulate_filtered_data / taa over the workset in 8x8 work-groups.
OURS libbmfr's bmfr_process_frame: the library default (exact fit) and the
     bench's fast_fit, on the same feature set (B = 13, or config 5's
     third-order B = 16; f32 input planes, as the reference reads them).

Both are timed per frame the way the reference times itself (bmfr.cpp:
495-502: START of accumulate_noisy_data to END of taa, device time, host
copies excluded): a HIP event before the frame's first launch and after its
last, on the stream they run on, frames WARM..N-1 averaged.  The reference's
input upload (its enqueueWriteBuffer, untimed there too) happens before the
first event.  Inputs are the GPU-rendered synthetic sequence, resident in HBM.
Results go to the parity log under speed/<case>.
"""
from __future__ import annotations

import pytest
import torch

import bmfr_amd
import ref_run
from ref_configs import FULL_REF_CONFIGS

pytestmark = pytest.mark.gpu

# (reference build, frames run, warm-up frames not averaged)
CASES = [("f1920x1080_h13", 24, 4), ("f3840x2160_h13", 14, 4), ("f3840x2160_h16", 14, 4),
         ("f7680x4320_h13", 10, 3)]


def _frames(rc, n):
    return [bmfr_amd.synth_frame_device(rc.width, rc.height, f, seed=rc.seed) for f in range(n)]


def _cams(rc, n):
    out = []
    for f in range(n):
        vp, _ = bmfr_amd.synth_camera(rc.width, rc.height, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(rc.width, rc.height, f)
        out.append((vp, jit))
    return out


def _time(step, n, warm):
    """step(f) issues frame f; returns mean device ms over frames warm..n-1."""
    evs = []
    for f in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        step(f, a, b)
        evs.append((a, b))
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in evs[warm:]]
    return sum(ms) / len(ms)


@pytest.mark.parametrize("build,nframes,warm", CASES, ids=[c[0] for c in CASES])
def test_reference_kernels_vs_libbmfr_same_gpu(build, nframes, warm, gpu, parity_log):
    rc = FULL_REF_CONFIGS[build]
    if not ref_run.available(build, "default"):
        pytest.skip(f"reference build {build}_default missing (oracle/build_ref.py)")
    frames, cams = _frames(rc, nframes), _cams(rc, nframes)
    ref = ref_run.RefLoop(rc, "default")
    marks = []

    def ref_step(f, a, b):
        fr = frames[f]
        ref.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        a.record()
        mk = []
        ref.run_stages(*cams[f], f, upstream_launch=True, marks=mk)
        b.record()
        marks.append([a] + mk)
        ref.swap()

    ref_ms = _time(ref_step, nframes, warm)
    names = ("accumulate_noisy_data", "fitter", "weighted_sum", "accumulate_filtered_data", "taa")
    ref_split = {n: sum(m[i].elapsed_time(m[i + 1]) for m in marks[warm:]) / (nframes - warm)
                 for i, n in enumerate(names)}
    del ref
    torch.cuda.empty_cache()
    ours = {}
    for name, fast in (("exact", 0), ("fast_fit", 1)):
        den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=rc.width, image_height=rc.height,
                                                    scaled=tuple(rc.scaled), fast_fit=fast))

        def step(f, a, b, den=den):
            fr = frames[f]
            a.record()
            den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], *cams[f], f)
            b.record()

        ours[name] = _time(step, nframes, warm)
        # the K1 / K2 split: a second pass with libbmfr's per-kernel events
        den.set_profiling(True, capacity=nframes, stride=1)
        for f in range(nframes):
            step(f, torch.cuda.Event(), torch.cuda.Event())
        torch.cuda.synchronize()
        prof = den.profile()[warm:]
        ours[name + "_k1"] = sum(p[1] for p in prof) / len(prof)
        ours[name + "_k2"] = sum(p[2] for p in prof) / len(prof)
        den.close()
    print(f"{build}: reference kernels {ref_ms:.4f} ms/frame; libbmfr exact {ours['exact']:.4f} "
          f"({ref_ms / ours['exact']:.2f}x), fast_fit {ours['fast_fit']:.4f} ({ref_ms / ours['fast_fit']:.2f}x)")
    parity_log(f"speed/{build}", {
        "image": f"{rc.width}x{rc.height}", "frames_averaged": nframes - warm,
        "reference_default_build_ms_per_frame": ref_ms,
        "reference_kernels_ms": {k: round(v, 4) for k, v in ref_split.items()},
        "libbmfr_kernels_ms": {f"{k}_{j}": round(ours[f"{k}_{j}"], 4) for k in ("exact", "fast_fit")
                               for j in ("k1", "k2")},
        "libbmfr_exact_ms_per_frame": ours["exact"], "libbmfr_fast_fit_ms_per_frame": ours["fast_fit"],
        "speedup_exact": ref_ms / ours["exact"], "speedup_fast_fit": ref_ms / ours["fast_fit"],
        "timing": "HIP events around each frame (bmfr.cpp:495-502's START accumulate_noisy_data .. END taa)"})
    # the library must not be slower than the reference's own kernels on the
    # same GPU (measured: several times faster)
    assert ours["exact"] < ref_ms and ours["fast_fit"] < ref_ms
