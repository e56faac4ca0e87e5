"""Codegen guard for the timed kernels (CPU; reads the gfx950 code object).

The timed kernel instantiations must not touch scratch memory inside the
cell walk: when the 7-wave bounce kernel did (2-3 spill reloads per trip), the
bounce launches ran 9% slower with bit-identical output, which no parity test
can see.  tools/spill_check.py does the disassembly; which
instantiations are timed comes from libzrt itself (zrt_timed_kernels), so a
change of the launch constants cannot leave the check on a stale kernel.  A
synthetic disassembly is the control that the loop scan finds walk spills.
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
    if not spill_check.has_gfx950(OBJ):
        pytest.skip("render.o holds no gfx950 code object (ARCH= build)")
    return spill_check, spill_check.kernels(spill_check.disassemble(OBJ))


def _kernel(ks, sub):
    names = [n for n in ks if sub in n]
    assert names, sub
    return ks[names[0]]


def test_timed_kernel_names_come_from_the_library():
    import spill_check
    t = spill_check.timed()
    assert t[0].startswith("wf_kernel") and any(n.startswith("wf_park_kernel") for n in t)
    assert any(n.startswith("wf_shade_kernel") for n in t)


def test_timed_kernels_do_not_spill_in_the_walk(code):
    sc, ks = code
    for sub in sc.timed():
        ins = _kernel(ks, sub)
        loops = sc.walk_spills(ins)
        if sub.startswith(("wf_kernel", "wf_park_kernel")):
            assert loops, f"no walk loop found in {sub}"
        assert max((s for _, _, s in loops), default=0) == 0, sub


def test_park_and_shade_kernels_use_no_scratch(code):
    """The park and shade kernels touch no scratch at all (not only in the
    walk): their whole state lives in VGPRs and LDS."""
    sc, ks = code
    for sub in sc.timed():
        if sub.startswith(("wf_park_kernel", "wf_shade_kernel")):
            assert not any("scratch_" in t for _, t in _kernel(ks, sub)), sub


def test_spill_check_sees_walk_spills():
    import spill_check as sc
    base = 0x1000
    lines = [
        (base + 0x00, "  s_mov_b32 s0, 0  // 000000001000:"),
        (base + 0x04, "  global_load_dwordx4 v[0:3], v[4:5], off  // 000000001004:"),
        (base + 0x0c, "  scratch_load_dword v7, off, s0 offset:16  // 00000000100C:"),
        (base + 0x14, "  v_add_f32 v1, v1, v2  // 000000001014:"),
        (base + 0x18, "  s_cbranch_vccnz 65532 <_Zkern+0x4>  // 000000001018:"),
    ]
    loops = sc.walk_spills(lines)
    assert loops and max(s for _, _, s in loops) == 1
    clean = [l for l in lines if "scratch" not in l[1]]
    assert max(s for _, _, s in sc.walk_spills(clean)) == 0


def test_park_kernel_m0_only_feeds_the_range_dma(code):
    """park_load_range sets M0 in inline asm, which cannot declare M0
    clobbered (reserved): the park kernels must not use M0 for anything else,
    and every LDS-DMA must follow its own M0 write."""
    sc, ks = code
    import re
    names = [n for n in ks if "wf_park_kernel" in n]
    assert names
    for n in names:
        ins = [re.sub(r"\s*//.*", "", t).strip() for _, t in ks[n]]
        for i, t in enumerate(ins):
            if re.search(r"\bm0\b", t):
                assert t.startswith(("s_mov_b32 m0,", "s_add_u32 m0, m0, 0x100")), (n, t)
            if t.startswith("global_load_lds"):
                assert any(re.search(r"\bm0\b", x) for x in ins[max(0, i - 3):i]), (n, i, ins[i - 3:i + 1])


def _loops(ins):
    """(first index, last index) of every backward-branch loop body."""
    import re
    idx = {a: k for k, (a, _) in enumerate(ins)}
    out = []
    for k, (a, t) in enumerate(ins):
        m = re.search(r"\bs_(?:cbranch_\w+|branch) (\d+)", t)
        if not m:
            continue
        off = int(m.group(1))
        off = off - 65536 if off > 32767 else off
        tgt = a + 4 + 4 * off
        if tgt <= a and tgt in idx:
            out.append((idx[tgt], k))
    return out


def _walk_steps():
    """DDA steps per park walk trip with / without the escape table (the
    render.hip defaults of ZRT_WALK_STEPS / ZRT_WALK_STEPS_NOESC)."""
    import re
    with open(os.path.join(ROOT, "zig_raytracing_contest_amd", "csrc", "render.hip")) as fh:
        src = fh.read()
    return (int(re.search(r"#define ZRT_WALK_STEPS (\d+)", src).group(1)),
            int(re.search(r"#define ZRT_WALK_STEPS_NOESC (\d+)", src).group(1)))


def _walk_trip(ins, steps=4):
    trips = []
    for b, e in _loops(ins):
        body = [t.strip() for _, t in ins[b:e + 1]]
        # (the trip's OccX lookups are two ds_read_b64 per step; besides them
        # the escape slot and the parked lanes' range slots are read, and a
        # parking lane writes its slots' not-landed marks)
        if sum(t.startswith("ds_read_b64") for t in body) == 2 * steps \
                and any(t.startswith("global_load_lds") for t in body + ins_after(ins, e)):
            trips.append(body)
    assert trips, "walk loop not found"
    body = min(trips, key=len)
    return {"valu": sum(t.startswith("v_") for t in body), "movs": sum(t.startswith("v_mov") for t in body),
            # the trip's selects are v_cndmask on lane masks (DDAV_STEPM): no
            # execz branch around a select inside the trip (round 3's per-lane
            # booleans put four there, each with its own exec save/restore)
            "execz": sum(t.startswith("s_cbranch_execz") for t in body[:-1])}


def test_park_walk_trip_is_not_a_register_shuffle(code):
    """The walk trip (ZRT_WALK_STEPS = 4 DDA steps, four OccX lookups = 8 LDS
    reads, one range DMA issue point) stays ~179 VALU (202 before its
    booleans became lane masks; round 2's two-step trip was 115, round 3's 76
    before the trip grew to four steps).  Its old branchy
    form let the compiler copy the whole walk state through every join: a
    one-line change elsewhere in the kernel took it from 160 to 232 VALU (96
    v_mov) and cfg3 lost 2-3% with identical images.
    The plain kernel (wf_park_kernel<false>) keeps round 3's limits; the
    escape-table kernel (<true>) may exceed them only by the escape block
    (the slot read, the set-bit check and one LDS-DMA issue per brick:
    ~30 VALU and one execz branch), so a regression in the shared trip still
    fails here."""
    sc, ks = code
    # (field words, then brick-major words, dda.h: 165 VALU per trip since
    # r05ag, the brick and in-brick indices taken straight from the word; 157
    # since r05ak, the step's gap fill one v_bitop3)
    # (round 6: the plain kernel walks ZRT_WALK_STEPS_NOESC = 5 steps per trip;
    # its limits scale per step, and the escape kernel's trip is compared with
    # the plain one's per-step VALU times its own step count)
    se, sp = _walk_steps()
    for bm, limit in (("ELb0E", 200), ("ELb1E", 165)):
        plain = _walk_trip(_kernel(ks, "wf_park_kernelILb0" + bm), sp)
        esc = _walk_trip(_kernel(ks, "wf_park_kernelILb1" + bm), se)
        assert plain["valu"] <= limit * sp / 4 and plain["movs"] <= 10 and plain["execz"] <= 2, (bm, plain)
        assert esc["valu"] - plain["valu"] * se / sp <= 40 and esc["movs"] - plain["movs"] <= 6, (bm, esc, plain)
        assert esc["execz"] <= plain["execz"] + 1, (bm, esc, plain)


_WRITES01 = None


def _s01_source(lines, k, loop=None):
    """What s[0:1] holds at line k: 'spill' if the latest write to s0 or s1
    before it in program order is a v_readlane_b32 (an SGPR spill reload),
    'other' for any other write, 'entry' if nothing writes it first (the
    kernel-argument pointer).  With loop = (b, e) holding k, a write to s0/s1
    later in the loop body that is not a spill reload also makes it 'other'
    (the back edge carries it to the use)."""
    import re
    w = re.compile(r"^\s*(\S+)\s+(s\[0:1\]|s0|s1)\s*,")
    if loop is not None:
        for j in range(k + 1, loop[1] + 1):
            m = w.search(lines[j])
            if m and m.group(1) != "v_readlane_b32":
                return "other"
    for j in range(k - 1, -1, -1):
        m = w.search(lines[j])
        if m:
            return "spill" if m.group(1) == "v_readlane_b32" else "other"
    return "entry"


def test_walk_loops_load_nothing_from_the_kernel_arguments(code):
    """A select between kernel-argument fields (the packed walk's field masks
    f0/f1/f2) became, in round 3's primary lane walk, a vector load from the
    kernel-argument segment at a selected offset, waited on by a vmcnt(0) in
    every DDA step; the fields are laundered into registers now.  No timed
    kernel may form a vector address from s[0:1] inside a loop unless the
    latest write to s0/s1 before that use is an SGPR spill reload
    (v_readlane, a spilled pointer such as the cell records' base): the
    kernel-argument pointer itself (s[0:1] at entry, nothing written since)
    and any other scalar write -- a scalar load may reload the kernarg
    pointer -- are refused.  (Since r05ay the primary reloads
    its cell-record base before the walk loop instead of in it.)"""
    import re
    sc, ks = code
    use = re.compile(r"v_lshl_add_u64 v\[\d+:\d+\], s\[0:1\]")
    for sub in sc.timed():
        ins = _kernel(ks, sub)
        lines = [t.split("//")[0] for _, t in ins]
        loops = _loops(ins)
        for k in range(len(lines)):
            if not use.search(lines[k]):
                continue
            inner = [(b, e) for b, e in loops if b <= k <= e]
            if not inner:
                continue
            # (the innermost loop's back edge; an outer loop re-enters it
            # through the code in front of its header, which the backward
            # scan covers)
            b, e = min(inner, key=lambda x: x[1] - x[0])
            assert _s01_source(lines, k, (b, e)) == "spill", (sub, k, lines[k].strip())


def test_kernel_argument_check_sees_a_kernarg_address():
    """Control for the check above: an address formed from the entry s[0:1]
    or from s[0:1] written by a scalar load is caught; one after a spill
    reload is not, nor is one whose loop rewrites s0/s1 only by reloads."""
    use = "v_lshl_add_u64 v[0:1], s[0:1], 0, v[0:1]"
    assert _s01_source(["v_add_f32 v1, v1, v2", use], 1) == "entry"
    assert _s01_source(["v_readlane_b32 s0, v70, 31", "v_readlane_b32 s1, v70, 32", use], 2) == "spill"
    assert _s01_source(["s_load_dwordx2 s[0:1], s[4:5], 0x10", use], 1) == "other"
    assert _s01_source(["v_readlane_b32 s0, v70, 31", "v_readlane_b32 s1, v70, 32", use,
                        "s_mov_b32 s0, 0x3ffffe"], 2, (0, 3)) == "other"
    assert _s01_source(["v_readlane_b32 s0, v70, 31", "v_readlane_b32 s1, v70, 32", use,
                        "v_readlane_b32 s0, v70, 31"], 2, (0, 3)) == "spill"


def ins_after(ins, e, n=40):
    return [t.strip() for _, t in ins[e + 1:e + 1 + n]]
