"""Instruction counts of the park kernel's walk trip in a render.o (the loop
test_codegen.py guards): python tools/trip_isa.py [render.o] [--dump out.s]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import spill_check as sc  # noqa: E402
from test_codegen import _loops  # noqa: E402


def trips(obj):
    ks = sc.kernels(sc.disassemble(obj))
    ins = ks[[k for k in ks if "wf_park_kernel" in k][0]]
    out = []
    for b, e in _loops(ins):
        body = [t.strip() for _, t in ins[b:e + 1]]
        if sum(t.startswith("ds_read") for t in body) == 8 and not any(t.startswith("ds_write") for t in body):
            out.append(body)
    return out


if __name__ == "__main__":
    obj = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else os.path.join(
        ROOT, "build", "obj", "render.o")
    for body in trips(obj):
        print({"insts": len(body), "valu": sum(t.startswith("v_") for t in body),
               "salu": sum(t.startswith("s_") for t in body),
               "v_mov": sum(t.startswith("v_mov") for t in body),
               "v_cndmask": sum(t.startswith("v_cndmask") for t in body)})
    if "--dump" in sys.argv:
        body = min(trips(obj), key=len)
        open(sys.argv[sys.argv.index("--dump") + 1], "w").write("\n".join(body) + "\n")
