"""Child process of tests/test_gpu_fast_fit.py: run W x H synthetic frames
through the library variant BMFR_LIB names and save the frame outputs
(float32, frames x W*H*3) to the .npy path given; an optional sixth
argument "cfg5" selects BASELINE config 5 (third-order features, half input
planes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402


def main(W, H, n, fast_fit, out, cfg5=False):
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, fast_fit=fast_fit, input_half=int(cfg5),
                              scaled=bmfr_amd.SCALED_THIRD_ORDER if cfg5 else bmfr_amd.SCALED_DEFAULT)
    den = bmfr_amd.Denoiser(cfg)
    res = np.empty((n, W * H * 3), np.float32)
    for f in range(n):
        fr = bmfr_amd.synth_frame_device(W, H, f)
        if cfg5:
            fr = {k: (v.half() if k in ("noisy", "normals", "positions", "albedo") else v) for k, v in fr.items()}
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        res[f] = den.copy_output(torch.empty(W * H * 3, device="cuda")).cpu().numpy()
    np.save(out, res)
    print("build", bmfr_amd.build_id())


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5],
         len(sys.argv) > 6 and sys.argv[6] == "cfg5")
