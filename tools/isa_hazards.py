"""Scan the gfx950 machine code of a built library for VALU hazards that
need software wait states.

Why (round 4): the `fast_fit` column update gave wrong results (5.6e-3
rel-L2 at 200x136) once its `sched_barrier` was removed.  Cause: gfx950
needs three wait states between a DOT instruction (`v_dot2*`) writing a VGPR
and a different VALU instruction reading it.  LLVM's hazard recognizer
inserts them when the reader is a VALU instruction it knows, but not when the
reader is an inline-asm statement -- and the pivot row's fused mixed-precision
FMA (`fma_h`) was inline asm reading the dot-product chain's sum.  With the
barrier the scheduler happened to keep them three instructions apart; without
it they were two.  `fma_h` is now a plain `fmaf` on the widened half (the
compiler selects the same `v_fma_mix_f32` and sees the hazard), and this
scanner runs over the final code as a test (tests/test_isa_hazards.py), so
the class of bug cannot come back unnoticed.

Checked on the final instruction stream of every kernel (wait states: one per
instruction, N + 1 per `s_nop N`), within a basic block:
  * DOT write -> read by any other opcode, or as src A/B of the same DOT: 3;
  * transcendental (v_rcp / v_sqrt / v_rsq / v_exp / v_log / v_sin / v_cos)
    write -> non-transcendental VALU read: 1;
  * VALU write -> DPP read: 2;
  * VALU write -> v_permlane16/32_swap read: 2;
  * VALU write with a sub-dword destination (SDWA dst_sel != DWORD or VOP3
    op_sel[3]) -> VALU read: 1.

Usage: python tools/isa_hazards.py [lib.so ...]  (default bmfr_amd/libbmfr.so)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
TRANS = ("v_rcp_", "v_sqrt_", "v_rsq_", "v_exp_", "v_log_", "v_sin_", "v_cos_")

_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def _regs(text: str) -> set:
    out = set()
    for m in _VREG.finditer(text):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def code_objects(lib: str, workdir: str) -> list:
    """The gfx950 code objects of every offload bundle in lib's .hip_fatbin."""
    fat = os.path.join(workdir, "fatbin.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(workdir, "x.so")],
                   check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    cos = []
    for i, s in enumerate(starts):
        end = starts[i + 1] if i + 1 < len(starts) else len(data)
        b = os.path.join(workdir, f"b{i}.bin")
        with open(b, "wb") as f:
            f.write(data[s:end])
        co = os.path.join(workdir, f"co{i}.o")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--targets={TARGET}",
                            f"--input={b}", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            cos.append(co)
    return cos


def disassemble(co: str) -> dict:
    """{kernel symbol: [instruction text, ...]} with '' entries at labels / branch targets."""
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--no-show-raw-insn", co],
                         check=True, capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for ln in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is None:
            continue
        s = ln.split("//")[0].strip()
        if not s:
            continue
        if s.endswith(">:"):  # local label
            cur.append("")
            continue
        cur.append(s)
    return funcs


def _parse(s: str):
    parts = s.split(None, 1)
    op = parts[0]
    rest = parts[1] if len(parts) > 1 else ""
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", rest)]
    return op, ops


def _defs_uses(op: str, ops: list):
    if op.startswith("v_") and not op.startswith(("v_readlane", "v_readfirstlane", "v_cmp")) and ops and ops[0]:
        d = _regs(ops[0])
        u = set()
        for o in ops[1:]:
            u |= _regs(o)
        # read-modify-write destinations: DPP old value, dot2c / mac / fmac accumulators, permlane swaps
        if "_dpp" in op or "dot2c" in op or "mac_" in op or "permlane" in op:
            u |= d
        return d, u
    u = set()
    for o in ops:
        u |= _regs(o)
    return set(), u


def _is_branch(op: str) -> bool:
    return op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc", "s_endpgm"))


def scan_function(insts: list) -> list:
    """Hazards in one kernel: (kind, wait states found, producer, consumer)."""
    parsed = []
    for s in insts:
        if not s:
            parsed.append(None)
            continue
        op, ops = _parse(s)
        d, u = _defs_uses(op, ops)
        parsed.append((op, ops, d, u, s))
    hits = []
    for i, x in enumerate(parsed):
        if x is None:
            continue
        op, ops, d, u, s = x
        if not op.startswith("v_") or not u:
            continue
        is_dpp = "_dpp" in op or "quad_perm" in s or "row_" in s
        is_perm = op.startswith(("v_permlane16_swap", "v_permlane32_swap"))
        ws = 0
        for j in range(i - 1, max(i - 16, -1), -1):
            p = parsed[j]
            if p is None:
                break
            pop, pops, pd, pu, ps = p
            if _is_branch(pop):
                break
            if pop.startswith("s_nop"):
                ws += int(pops[0], 0) + 1 if pops and pops[0] else 1
                continue
            hit = pd & u
            if hit and pop.startswith("v_"):
                if pop.startswith("v_dot") and ws < 3:
                    reads_ab = any(pd & _regs(o) for o in ops[1:3])
                    if op != pop or reads_ab:
                        hits.append(("dot->valu", ws, ps, s))
                if pop.startswith(TRANS) and not op.startswith(TRANS) and ws < 1:
                    hits.append(("trans->valu", ws, ps, s))
                if is_dpp and ws < 2:
                    hits.append(("valu->dpp", ws, ps, s))
                if is_perm and ws < 2:
                    hits.append(("valu->permlane_swap", ws, ps, s))
                subdword = ("dst_sel:WORD" in ps or "dst_sel:BYTE" in ps
                            or re.search(r"op_sel:\[[01],[01],[01],1\]", ps) is not None)
                if subdword and ws < 1:
                    hits.append(("subdword->valu", ws, ps, s))
            ws += 1
            if ws >= 3:
                break
    return hits


def scan_library(lib: str) -> dict:
    """{kernel: [hazards]} for every kernel of lib (kernels without hazards omitted);
    raises if no gfx950 code is found."""
    with tempfile.TemporaryDirectory() as wd:
        cos = code_objects(lib, wd)
        if not cos:
            raise RuntimeError(f"no {TARGET} code object in {lib}")
        res, nfun = {}, 0
        for co in cos:
            for name, insts in disassemble(co).items():
                nfun += 1
                h = scan_function(insts)
                if h:
                    res[name] = h
    res["__functions_scanned__"] = nfun
    return res


def main(argv):
    libs = argv or [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bmfr_amd", "libbmfr.so")]
    bad = 0
    for lib in libs:
        res = scan_library(lib)
        n = res.pop("__functions_scanned__")
        print(f"{lib}: {n} functions scanned, {len(res)} with hazards")
        for k, hs in res.items():
            bad += len(hs)
            print(f"  {k}")
            for h in hs[:8]:
                print(f"    {h[0]} (wait states {h[1]}): {h[2]}  ->  {h[3]}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
