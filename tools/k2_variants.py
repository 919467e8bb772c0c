"""Build A/B variants of libbmfr that differ only in one source's
compile-time knobs (VARIANT_SRC, default bmfr_kernels.hip) (the other objects are reused from the main build):
python tools/k2_variants.py NAME="-DFLAG ..." ...  -> bmfr_amd/libbmfr_NAME.so
(select at run time with BMFR_LIB=NAME)."""
import concurrent.futures as cf
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bmfr_amd import _build as b  # noqa: E402


SRC = os.environ.get("VARIANT_SRC", "bmfr_kernels.hip")  # the one source the flags apply to


def one(spec):
    name, flags = spec.split("=", 1)
    objdir = os.path.join(b.HERE, "_obj")
    obj = os.path.join("/tmp", f"k2v_{name}.o")
    subprocess.run([b.HIPCC, *b.FLAGS, *flags.split(), "-c", os.path.join(b.CSRC, SRC), "-o", obj],
                   check=True)
    objs = [obj if s == SRC else os.path.join(objdir, s.replace(".hip", ".o")) for s in b.SOURCES]
    lib = os.path.join(b.HERE, f"libbmfr_{name}.so")
    subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    return lib


if __name__ == "__main__":
    b.build()
    with cf.ThreadPoolExecutor(max_workers=6) as ex:
        for lib in ex.map(one, sys.argv[1:]):
            print(lib)
