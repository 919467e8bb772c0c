#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths of
K1/K2 (16-B, 12-B float3 and 1-B per lane).  Run under
`rocprofv3 --pmc FETCH_SIZE` (and separately WRITE_SIZE); each dispatch
touches exactly BYTES bytes of a 1 GiB buffer (larger than the 256 MiB
Infinity Cache, so nothing is served on-die), then
`prof_summary.py calib <dir> <counter>` prints counter KB / true KB.

  python tools/pmc_calibrate.py build   # here: compile tools/_pmc_calib.so
  python tools/pmc_calibrate.py run     # on the GPU box, under rocprofv3
"""
import ctypes as C
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_pmc_calib.so")
BYTES = 3 * (1 << 30) // 4 // 48 * 48  # 768 MiB, divisible by 16, 12 and 1
KINDS = ["read_16B", "read_12B", "read_1B", "write_12B", "write_1B"]


def build():
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           os.path.join(HERE, "pmc_calib.hip"), "-o", SO])


def run():
    import torch  # binds torch's HIP runtime first (as bmfr_amd/_lib.py)
    lib = C.CDLL(SO)
    lib.calib_run.argtypes = [C.c_int, C.c_void_p, C.c_long, C.c_void_p]
    buf = torch.ones(BYTES // 4, dtype=torch.float32, device="cuda")
    sink = torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    for k, name in enumerate(KINDS):
        for _ in range(3):
            rc = lib.calib_run(k, buf.data_ptr(), BYTES, sink.data_ptr())
            assert rc == 0, (name, rc)
        print(f"{name}: 3 dispatches x {BYTES} bytes", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
