"""Codegen guard for the timed kernels (CPU; reads the gfx950 code object).

The timed wf_kernel instantiations must not touch scratch memory inside the
cell walk: when the 7-wave bounce kernel did (2-3 spill reloads per trip), the
bounce launches ran 9% slower with bit-identical output, which no parity test
can see.  tools/spill_check.py does the disassembly; the
8-wave instantiation (64 VGPRs against a ~100-VGPR working set) is the control
that shows the check finds walk spills when they are there.
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
OBJ = os.path.join(ROOT, "build", "obj", "render.o")


@pytest.fixture(scope="module")
def code():
    import spill_check
    if not os.path.exists(OBJ):
        pytest.skip("build/obj/render.o not built (make)")
    if not shutil.which(os.path.join(spill_check.LLVM, "llvm-objdump")):
        pytest.skip("ROCm llvm tools absent")
    return spill_check, spill_check.kernels(spill_check.disassemble(OBJ))


def _walk_scratch(sc, ks, sub):
    names = [n for n in ks if sub in n]
    assert names, sub
    loops = sc.walk_spills(ks[names[0]])
    assert loops, f"no walk loop found in {names[0]}"
    return max(s for _, _, s in loops)


@pytest.mark.parametrize("sub", ["wf_kernelILi2ELi7ELb1ELb0EE", "wf_kernelILi2ELi6ELb0ELb0EE"])
def test_timed_kernels_do_not_spill_in_the_walk(code, sub):
    sc, ks = code
    assert sub in sc.TIMED
    assert _walk_scratch(sc, ks, sub) == 0


def test_spill_check_sees_walk_spills(code):
    sc, ks = code
    assert _walk_scratch(sc, ks, "wf_kernelILi2ELi8ELb0ELb0EE") > 0
