"""Test configurations shared by the oracle, the reference build and the tests.

TEST INFRASTRUCTURE ONLY.  A configuration is the reference's `#define`
surface (bmfr.cpp:32-118) for one image size / feature set / tmp precision.
`ref_build_options()` reproduces the JIT `-D` string of bmfr.cpp:205-232.
"""
from __future__ import annotations

import dataclasses

# Feature codes (same numbering as include/bmfr.h and oracle/bmfr_oracle.h)
# and the OpenCL expression text the reference pastes into FEATURE_BUFFERS.
FEATURE_TEXT = {
    0: "1.f",
    1: "normal.x", 2: "normal.y", 3: "normal.z",
    4: "world_position.x", 5: "world_position.y", 6: "world_position.z",
    7: "world_position.x*world_position.x",
    8: "world_position.y*world_position.y",
    9: "world_position.z*world_position.z",
    10: "world_position.x*world_position.x*world_position.x",
    11: "world_position.y*world_position.y*world_position.y",
    12: "world_position.z*world_position.z*world_position.z",
}

NOT_SCALED_DEFAULT = (0, 1, 2, 3)                 # bmfr.cpp:65-69
SCALED_DEFAULT = (4, 5, 6, 7, 8, 9)               # bmfr.cpp:71-77
SCALED_THIRD_ORDER = SCALED_DEFAULT + (10, 11, 12)  # BASELINE config 5


def fmt_g(x: float) -> str:
    """`std::ostream << double` with default flags: %g, 6 significant digits
    (bmfr.cpp:226-227 stream the dataset limits this way)."""
    return "%g" % x


@dataclasses.dataclass(frozen=True)
class RefConfig:
    name: str
    width: int
    height: int
    not_scaled: tuple = NOT_SCALED_DEFAULT
    scaled: tuple = SCALED_DEFAULT
    half_tmp: int = 1
    frames: int = 4
    noise_amount: str = "1e-2"          # NOISE_AMOUNT text, bmfr.cpp:58
    blend_alpha: str = "0.2f"           # bmfr.cpp:60
    second_blend_alpha: str = "0.1f"    # bmfr.cpp:61
    taa_blend_alpha: str = "0.2f"       # bmfr.cpp:62
    position_limit_squared: float = 0.01
    normal_limit_squared: float = 0.1
    seed: int = 0x424D4652

    @property
    def buffer_count(self) -> int:
        return len(self.not_scaled) + len(self.scaled) + 3

    @property
    def workset(self):
        return (32 * ((self.width + 31) // 32), 32 * ((self.height + 31) // 32))

    @property
    def margins(self):
        ww, wh = self.workset
        return ww + 32, wh + 32

    @property
    def blocks(self) -> int:
        mw, mh = self.margins
        return (mw // 32) * (mh // 32)

    def feature_text(self) -> str:
        return ",".join(FEATURE_TEXT[c] for c in self.not_scaled + self.scaled)

    def ref_build_options(self) -> list:
        ww, wh = self.workset
        mw, mh = self.margins
        b = self.buffer_count
        d = {
            "BUFFER_COUNT": b,
            "FEATURES_NOT_SCALED": len(self.not_scaled),
            "FEATURES_SCALED": len(self.scaled),
            "IMAGE_WIDTH": self.width,
            "IMAGE_HEIGHT": self.height,
            "WORKSET_WIDTH": ww,
            "WORKSET_HEIGHT": wh,
            "FEATURE_BUFFERS": self.feature_text(),
            "LOCAL_WIDTH": 8,
            "LOCAL_HEIGHT": 8,
            "WORKSET_WITH_MARGINS_WIDTH": mw,
            "WORKSET_WITH_MARGINS_HEIGHT": mh,
            "BLOCK_EDGE_LENGTH": 32,
            "BLOCK_PIXELS": 1024,
            "R_EDGE": b - 2,
            "NOISE_AMOUNT": self.noise_amount,
            "BLEND_ALPHA": self.blend_alpha,
            "SECOND_BLEND_ALPHA": self.second_blend_alpha,
            "TAA_BLEND_ALPHA": self.taa_blend_alpha,
            "POSITION_LIMIT_SQUARED": fmt_g(self.position_limit_squared),
            "NORMAL_LIMIT_SQUARED": fmt_g(self.normal_limit_squared),
            "COMPRESSED_R": 1,
            "CACHE_TMP_DATA": 1,
            "ADD_REQD_WG_SIZE": 1,
            "LOCAL_SIZE": 256,
            "USE_HALF_PRECISION_IN_TMP_DATA": self.half_tmp,
        }
        return [f"-D{k}={v}" for k, v in d.items()]


# Golden-vector configurations: small enough for the
# pure-CPU oracle to run in seconds, covering height padding (80 -> 96),
# width padding (100 -> 128), all 16 block offsets over 16 frames, both tmp
# precisions, the 3rd-order feature set (B = 16) and non-default feature
# lists (B = 7, 10, 12; no scaled features).
REF_CONFIGS = {
    c.name: c
    for c in (
        RefConfig("s128x80_h13", 128, 80, frames=17),
        RefConfig("s128x80_f13", 128, 80, half_tmp=0, frames=6),
        RefConfig("s100x72_h16", 100, 72, scaled=SCALED_THIRD_ORDER, frames=6),
        RefConfig("s96x64_f16", 96, 64, scaled=SCALED_THIRD_ORDER, half_tmp=0, frames=4),
        RefConfig("s48x48_h13", 48, 48, frames=4),
        RefConfig("s1280x720_h13", 1280, 720, frames=2),
        # other feature lists (bmfr.cpp:65-77): generic-count kernels
        RefConfig("s96x64_h7", 96, 64, not_scaled=(0,), scaled=(4, 5, 6), frames=4),
        RefConfig("s96x64_f10", 96, 64, scaled=(4, 5, 6), half_tmp=0, frames=4),
        RefConfig("s80x64_h12", 80, 64, not_scaled=(0, 3), scaled=(10, 11, 12, 7, 8, 9, 4), frames=4),
        RefConfig("s64x64_h7", 64, 64, scaled=(), frames=3),
    )
}

# BASELINE.json's configurations at their own sizes (GPU tests only: the CPU
# oracle is too slow there, so no golden .npz; tests/golden/fullsize_digests.json
# keeps SHA-256 digests of the reference's outputs).  frames: how many frames
# tests/test_gpu_reference_fullsize.py compares.
FULL_REF_CONFIGS = {
    c.name: c
    for c in (
        RefConfig("f1920x1080_h13", 1920, 1080, frames=17),              # config 2
        # 4K: 17 frames, so every one of the 16 block-grid offsets (bmfr.cl:267-285) is hit
        RefConfig("f3840x2160_h13", 3840, 2160, frames=17),              # config 3 (reference default build)
        RefConfig("f3840x2160_f13", 3840, 2160, half_tmp=0, frames=17),  # config 3, fp32 tmp_data
        RefConfig("f3840x2160_h16", 3840, 2160, scaled=SCALED_THIRD_ORDER, frames=17),  # config 5 (3rd order)
        RefConfig("f7680x4320_h13", 7680, 4320, frames=3),               # config 4's frame, untiled
        # B = 16 with f32 tmp_data: the MFMA experiment's tolerance reference (tools/mfma_experiment.py)
        RefConfig("f3840x2160_f16", 3840, 2160, scaled=SCALED_THIRD_ORDER, half_tmp=0, frames=4),
        RefConfig("f1280x720_h13", 1280, 720, frames=60),                # a whole 60-frame sequence
    )
}

# Build modes of the reference: "strict" fixes the arithmetic OpenCL leaves to
# the implementation (no contraction, correctly rounded / and sqrt) and is the
# one the oracle is pinned to bit-for-bit; "default" is what bmfr.cpp's
# options alone give (contraction on, 2.5-ulp divide) and is compared with a
# tolerance.
REF_MODES = {
    "strict": ["-ffp-contract=off", "-cl-fp32-correctly-rounded-divide-sqrt"],
    "default": [],
}
