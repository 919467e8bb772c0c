"""Shared command line of the profiling tools (k1_frames.py, frame_times.py,
k1_phases.py): W H FRAMES [PASSES] and the configuration flags of bench.py
(--third-order: B = 16; --input-half: half3 input planes; --f32-tmp: f32
tmp_data; --fast-fit: bmfr_config.fast_fit)."""
import argparse

import bmfr_amd


def parse(default_passes=1, argv=None, default_frames=100):
    ap = argparse.ArgumentParser()
    ap.add_argument("W", type=int, nargs="?", default=3840)
    ap.add_argument("H", type=int, nargs="?", default=2160)
    ap.add_argument("frames", type=int, nargs="?", default=default_frames)
    ap.add_argument("passes", type=int, nargs="?", default=default_passes)
    ap.add_argument("--third-order", action="store_true")
    ap.add_argument("--input-half", action="store_true")
    ap.add_argument("--f32-tmp", action="store_true")
    ap.add_argument("--fast-fit", action="store_true")
    a = ap.parse_args(argv)
    cfg = bmfr_amd.BmfrConfig(image_width=a.W, image_height=a.H,
                              scaled=bmfr_amd.SCALED_THIRD_ORDER if a.third_order else bmfr_amd.SCALED_DEFAULT,
                              use_half_precision_in_tmp_data=0 if a.f32_tmp else 1, input_half=int(a.input_half),
                              fast_fit=int(a.fast_fit))

    def render(f):
        fr = bmfr_amd.synth_frame_device(a.W, a.H, f)
        if a.input_half:
            fr = {k: v.half() for k, v in fr.items()}
        return fr
    a.render = render
    return a, cfg
