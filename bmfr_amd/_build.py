"""Build libbmfr.so in-tree with hipcc for gfx950.

The library is plain HIP C++ behind the C ABI of include/bmfr.h; it is built
with `-ffp-contract=off` because the kernels promise the reference's
per-operation rounding (see csrc/bmfr_device.h).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libbmfr.so")
DIAG_LIB = os.path.join(HERE, "libbmfr_diag.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["bmfr_kernels.hip", "bmfr_fused.hip", "bmfr_fused_cols.hip", "bmfr_fused_cols_f32.hip", "bmfr_capi.hip",
           "bmfr_exchange.hip",
           "bmfr_synth.hip",
           "bmfr_generic_ns1.hip", "bmfr_generic_ns2.hip", "bmfr_generic_ns3.hip", "bmfr_generic_ns4.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
         "-Wall", "-Wno-unused-function"]
LINK_FLAGS = ["--offload-arch=gfx950", "-shared", "-fPIC"]
LINK_LIBS = ["-ldl"]  # after the objects on the link line


INCLUDE = os.path.join(HERE, "..", "include")
ID_MARK = b"bmfr-build-id:"


def source_files() -> list:
    """Every file libbmfr.so is compiled from: csrc/ and the public headers."""
    files = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".hip", ".h"))]
    files += [os.path.join(INCLUDE, f) for f in sorted(os.listdir(INCLUDE)) if f.endswith(".h")]
    return files


def source_hash() -> str:
    """SHA-256 over the library's sources (names and contents) and the compile
    and link flags (bit-exactness depends on -ffp-contract=off and
    -fno-slp-vectorize): the build id libbmfr.so carries (bmfr_build_id())
    and the loader checks (_lib.load)."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode() + b"\0" + " ".join(LINK_FLAGS + LINK_LIBS).encode() + b"\0")
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def build_id(diag: bool = False, extra_flags=()) -> str:
    """The id a build of the current sources with these options carries:
    the source hash, then '+' and the extra compile flags of a variant."""
    flags = (["-DBMFR_STAMPS"] if diag else []) + [f for f in extra_flags if f]
    return source_hash() + ("+" + ",".join(flags) if flags else "")


def embedded_id(lib: str) -> str | None:
    """The build id stored in a built library (read from the file: no dlopen)."""
    if not os.path.exists(lib):
        return None
    with open(lib, "rb") as f:
        data = f.read()
    i = data.find(ID_MARK)
    if i < 0:
        return None
    j = data.index(b"\0", i)
    return data[i + len(ID_MARK):j].decode()


class _BuildLock:
    """One build at a time across processes (pytest-xdist workers may all
    find a library stale at once and would race on the same object files)."""

    def __enter__(self):
        import fcntl
        self.f = open(os.path.join(HERE, ".build.lock"), "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def _on_gpu_box() -> bool:
    """gpurun's GPU box (it exports GRAFT_REPO_ROOT): libraries are built in
    this container and travel with the tree -- never rebuilt there, even when
    file times make them look older than a source."""
    return bool(os.environ.get("GRAFT_REPO_ROOT"))


def build(force: bool = False, verbose: bool = False, diag: bool = False, variant: str = "",
          extra_flags=()) -> str:
    lib = DIAG_LIB if diag else (os.path.join(HERE, f"libbmfr_{variant}.so") if variant else LIB)
    if _on_gpu_box() and os.path.exists(lib) and not force:
        return lib
    with _BuildLock():
        return _build(force, verbose, diag, variant, extra_flags)


def _build(force, verbose, diag, variant, extra_flags) -> str:
    """Build libbmfr.so (or, diag=True, libbmfr_diag.so: same library with
    in-kernel phase timestamps compiled in, for profiling only; or, with
    variant=NAME, libbmfr_NAME.so built with extra_flags, for A/B timing --
    selected at run time by BMFR_LIB=NAME)."""
    lib = DIAG_LIB if diag else (os.path.join(HERE, f"libbmfr_{variant}.so") if variant else LIB)
    want = build_id(diag, extra_flags)
    if not force and embedded_id(lib) == want:
        return lib
    objdir = os.path.join(HERE, "_obj_diag" if diag else (f"_obj_{variant}" if variant else "_obj"))
    os.makedirs(objdir, exist_ok=True)
    # the id, as a generated header only bmfr_capi.hip includes (bmfr_build_id())
    with open(os.path.join(objdir, "bmfr_build_id.h"), "w") as f:
        f.write(f'#define BMFR_BUILD_ID "{want}"\n')

    def compile_one(src: str) -> str:
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        cmd = [HIPCC, *FLAGS, *(["-DBMFR_STAMPS"] if diag else []), *extra_flags, "-I", objdir, "-c",
               os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        return obj

    with cf.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + ".tmp"
    subprocess.run([HIPCC, *LINK_FLAGS, "-o", tmp, *objs, *LINK_LIBS], check=True)
    os.replace(tmp, lib)
    return lib


TOOLS = os.path.join(HERE, "..", "tools")


def build_tool(src: str, out: str) -> str:
    """A stand-alone HIP experiment library under tools/ (e.g. libwy.so), with
    the same build lock and the same never-rebuild-on-the-GPU-box rule."""
    src, out = os.path.join(TOOLS, src), os.path.join(TOOLS, out)
    if os.path.exists(out) and (_on_gpu_box() or os.path.getmtime(out) >= os.path.getmtime(src)):
        return out
    with _BuildLock():
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", src, "-o",
                        out + ".tmp"], check=True)
        os.replace(out + ".tmp", out)
    return out


HOST_DIR = os.path.join(HERE, "..", "host")
IO_LIB = os.path.join(HERE, "libbmfr_io.so")
HOST_EXE = os.path.join(HERE, "bmfr_host")


def build_host(force: bool = False, verbose: bool = False) -> str:
    """Build the host side: libbmfr_io.so (EXR / PNG I/O, host/image_io.cpp)
    and the bmfr_host program (host/bmfr_host.cpp, the reference's bmfr.cpp
    on libbmfr), next to libbmfr.so (rpath $ORIGIN)."""
    build(verbose=verbose)
    if _on_gpu_box() and os.path.exists(IO_LIB) and os.path.exists(HOST_EXE) and not force:
        return HOST_EXE
    with _BuildLock():
        return _build_host(force, verbose)


def _build_host(force, verbose) -> str:
    srcs = [os.path.join(HOST_DIR, f) for f in os.listdir(HOST_DIR)]
    newest = max(os.path.getmtime(f) for f in srcs + [LIB])
    steps = [
        (IO_LIB, ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", os.path.join(HOST_DIR, "image_io.cpp"),
                  "-o", IO_LIB + ".tmp", "-lz"]),
        (HOST_EXE, [HIPCC, "-O2", "-std=c++17", "-Wall", "-fopenmp", "-I", os.path.join(HERE, "..", "include"),
                    "-I", HOST_DIR, os.path.join(HOST_DIR, "bmfr_host.cpp"), os.path.join(HOST_DIR, "image_io.cpp"),
                    "-L", HERE, "-lbmfr", "-lz", "-Wl,-rpath,$ORIGIN", "-o", HOST_EXE + ".tmp"]),
    ]
    for out, cmd in steps:
        if not force and os.path.exists(out) and os.path.getmtime(out) >= newest:
            continue
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return HOST_EXE


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--diag", action="store_true")
    ap.add_argument("--variant", default="")
    ap.add_argument("--flags", default="", help="extra hipcc flags for a variant build")
    ap.add_argument("--host", action="store_true", help="also build libbmfr_io.so and bmfr_host")
    a = ap.parse_args()
    print(build(force=True, verbose=True, diag=a.diag, variant=a.variant, extra_flags=a.flags.split()))
    if a.host:
        print(build_host(force=True, verbose=True))
