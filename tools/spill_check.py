#!/usr/bin/env python3
"""Scratch (spill) accesses inside the traversal loop of the timed kernels.

The bounce launches lost 9% when the 7-wave wf_kernel's allocator started
spilling inside the walk (2-3 scratch loads per DDA/triangle trip; DESIGN.md
§5).  This reads the gfx950 code object out of build/obj/render.o
(clang-offload-bundler), disassembles it (llvm-objdump) and, per kernel,
counts scratch loads/stores inside every loop (backward branch) that issues
triangle loads (global_load_dwordx3/x4) and spans < 1000 instructions: the
cell walk.  Usage: spill_check.py [render.o] [kernel-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUNDLE = "hipv4-amdgcn-amd-amdhsa--gfx950"


def timed():
    """The timed kernel instantiations, as libzrt reports them
    (zrt_timed_kernels: built from the same constants render.hip launches)."""
    sys.path.insert(0, ROOT)
    from zig_raytracing_contest_amd import native
    return native.timed_kernels()


def has_gfx950(obj):
    """True if the object's offload bundle holds a gfx950 code object."""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        if subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                           os.path.join(d, "x.o")], capture_output=True).returncode != 0:
            return False
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={fb}"],
                           capture_output=True, text=True)
        return r.returncode == 0 and BUNDLE in r.stdout


def disassemble(obj):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fatbin"), os.path.join(d, "gfx950.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                        os.path.join(d, "x.o")], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--targets={BUNDLE}", f"--input={fb}",
                        f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True,
                              capture_output=True, text=True).stdout


def kernels(dis):
    """{symbol: [(address, text)]}"""
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:$", line)
        if m:
            cur = out.setdefault(m.group(1), [])
            continue
        m = re.search(r"//\s*([0-9A-Fa-f]+):", line)
        if cur is not None and m:
            cur.append((int(m.group(1), 16), line))
    return out


def walk_spills(ins):
    """[(loop first addr, last addr, scratch ops)] for the walk-like loops."""
    if not ins:
        return []
    base = ins[0][0]
    res = []
    for k, (addr, text) in enumerate(ins):
        m = re.search(r"s_c?branch\w*\s.*<[^+>]+\+0x([0-9a-f]+)>", text)
        if not m:
            continue
        tgt = base + int(m.group(1), 16)
        if tgt >= addr:
            continue
        body = [t for a, t in ins if tgt <= a <= addr]
        if len(body) >= 1000 or not any(re.search(r"global_load_dwordx[34]\b", t) for t in body):
            continue
        res.append((tgt, addr, sum(1 for t in body if "scratch_load" in t or "scratch_store" in t)))
    return res


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "obj", "render.o")
    want = sys.argv[2:] or timed()
    ks = kernels(disassemble(obj))
    bad = 0
    for w in want:
        names = [n for n in ks if w in n]
        if not names:
            print(f"{w}: not found")
            bad += 1
            continue
        for n in names:
            loops = walk_spills(ks[n])
            worst = max((s for _, _, s in loops), default=0)
            print(f"{n}: {len(loops)} walk loops, max scratch ops in one: {worst}")
            bad += worst > 0
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
