"""bmfr_process_frame's one-launch frame (k_fused_cols_taa<..., SAME = true>:
the TAA tiles of a frame wait on completion flags of the K1 blocks under
them and read their outputs device-coherent) against the same frames run as
two launches (K1, then K2: what a profiled frame does), bit for bit on the
output and every temporal-state plane, at the BASELINE sizes and a small
odd size.  Frames of 4096 K1 blocks or more (4K) run as two launches
unprofiled too (bmfr_sizes.frame_launches): there the per-frame path is
checked against the profiled one, and the one-launch kernel is forced
(include/bmfr_debug.h bmfr_debug_frame_launches) and checked as well.  The
full-size reference tests (test_gpu_reference_fullsize.py) pin the default
paths to the reference kernels."""
import pytest
import torch

import bmfr_amd

pytestmark = pytest.mark.gpu


def run(W, H, frames, profiled, launches=0):
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    den.debug_frame_launches(launches)
    if profiled:  # per-kernel events on every frame: K1 and K2 as two launches
        den.set_profiling(True, capacity=frames, stride=1)
    n = W * H
    out = []
    for f in range(frames):
        fr = bmfr_amd.synth_frame_device(W, H, f)
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        out.append({
            "result": den.copy_output(torch.empty(3 * n, device="cuda")),
            "acc": den.copy_state("filtered_accumulated", torch.empty(3 * n, device="cuda")),
            "noisy": den.copy_state("noisy_accumulated", torch.empty(3 * n, device="cuda")),
            "spp": den.copy_state("spp", torch.empty(n, dtype=torch.uint8, device="cuda")),
            "prev_pixel": den.copy_state("prev_frame_pixel", torch.empty(2 * n, device="cuda")),
        })
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("W,H,frames", [(3840, 2160, 5), (1920, 1080, 8), (200, 136, 20)])
def test_one_launch_frame_equals_two_launches(W, H, frames, gpu):
    launches = bmfr_amd.BmfrConfig(image_width=W, image_height=H).sizes().frame_launches
    assert launches == (2 if W >= 3840 else 1)
    two = run(W, H, frames, True)
    runs = {"default": run(W, H, frames, False)}
    if launches == 2:  # the one-launch kernel at this size too
        runs["one launch"] = run(W, H, frames, False, launches=1)
    for name, one in runs.items():
        for f in range(frames):
            for k in one[f]:
                a, b = one[f][k], two[f][k]
                if a.dtype == torch.float32:
                    a, b = a.view(torch.int32), b.view(torch.int32)
                assert torch.equal(a, b), f"{name}: frame {f} {k}: {int((a != b).sum())} of {a.numel()} differ"
