"""The built gfx950 code carries every software wait state the hardware needs
(tools/isa_hazards.py): DOT -> VALU (3), transcendental -> VALU (1),
VALU -> DPP / permlane swap (2), sub-dword write -> VALU (1).  The compiler
inserts them for the instructions it generates; this catches an inline-asm
reader it cannot see -- the round-3 fast_fit bug (the pivot row's asm FMA two
instructions after a v_dot2) -- in the product library and in the build
without the fast update's scheduling barrier."""
from __future__ import annotations

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_hazards  # noqa: E402


@pytest.mark.parametrize("name", ["libbmfr.so", "libbmfr_fastnosb.so"])
def test_no_unguarded_hazards(name):
    lib = os.path.join(ROOT, "bmfr_amd", name)
    if not os.path.exists(lib):
        pytest.fail(f"{lib} missing (__graft_entry__.build())")
    res = isa_hazards.scan_library(lib)
    n = res.pop("__functions_scanned__")
    assert n > 100, n
    assert not res, {k: v[:3] for k, v in res.items()}


def test_scanner_finds_a_dot_hazard():
    """The scanner itself: a v_dot2 result read by another VALU two
    instruction later is reported; with s_nop 1 also in between (three wait
    states) it is not."""
    bad = ["v_dot2c_f32_f16_e32 v35, v6, v26", "v_mov_b32_e32 v1, 0",
           "v_fma_mix_f32 v35, v1, v2, v35 op_sel_hi:[1,0,0]"]
    hits = isa_hazards.scan_function(bad)
    assert [h[0] for h in hits] == ["dot->valu"]
    good = bad[:2] + ["s_nop 1"] + bad[2:]
    assert isa_hazards.scan_function(good) == []
    # the same DOT accumulating into its own destination needs no wait
    assert isa_hazards.scan_function(["v_dot2c_f32_f16_e32 v35, v6, v26",
                                      "v_dot2c_f32_f16_e32 v35, v7, v27"]) == []
    perm = ["v_add_f32_e32 v22, v22, v35", "v_mov_b32_e32 v35, v22", "v_permlane16_swap_b32_e32 v22, v35"]
    assert {h[0] for h in isa_hazards.scan_function(perm)} == {"valu->permlane_swap"}
    assert isa_hazards.scan_function(perm[:2] + ["s_nop 1"] + perm[2:]) == []
