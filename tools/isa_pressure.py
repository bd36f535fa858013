"""Approximate VGPR liveness over one kernel's ISA (build/wgaead-gfx950.s): backward
dataflow on the basic-block CFG, first VGPR operand = def for loads/VALU, all operands
= uses for stores/ds_write. Prints the program points with the highest live-VGPR count.
Usage: python tools/isa_pressure.py <mangled-name> [top]"""
import re
import sys

name = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
s = open("build/wgaead-gfx950.s").read()
a = s.index(name + ":")
b = s.index(".Lfunc_end", a)
lines = s[a:b].splitlines()[1:]

REG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")


def vregs(txt):
    out = set()
    for m in REG.finditer(txt):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


insts = []  # (label_or_None, text)
for l in lines:
    t = l.split(";")[0].rstrip()
    if re.match(r"^\.LBB\S+:", t):
        insts.append(("L", t[:-1]))
    elif l.startswith("\t") and t.strip() and not t.strip().startswith("."):
        insts.append(("I", t.strip()))

blocks, cur = [], {"name": "entry", "ins": []}
for k, t in insts:
    if k == "L":
        blocks.append(cur)
        cur = {"name": t, "ins": []}
    else:
        cur["ins"].append(t)
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append(cur)
            cur = {"name": cur["name"] + "+", "ins": []}
blocks.append(cur)
blocks = [b for b in blocks if b["ins"] or b["name"]]
idx = {b["name"]: i for i, b in enumerate(blocks)}
for i, bl in enumerate(blocks):
    succ = []
    last = bl["ins"][-1] if bl["ins"] else ""
    op = last.split()[0] if last else ""
    if op.startswith(("s_branch", "s_cbranch")):
        tgt = last.split()[1]
        if tgt in idx:
            succ.append(idx[tgt])
    if op not in ("s_branch", "s_endpgm", "s_setpc_b64") and i + 1 < len(blocks):
        succ.append(i + 1)
    bl["succ"] = succ


def defs_uses(t):
    op, _, rest = t.partition(" ")
    ops = [x.strip() for x in rest.split(",")] if rest else []
    if not ops:
        return set(), set()
    if op.startswith(("global_store", "buffer_store", "ds_write", "flat_store", "scratch_store")) or op.startswith("ds_bpermute") is False and op.startswith("ds_write"):
        return set(), vregs(rest)
    if op.startswith("v_cmp") or op.startswith("v_readfirstlane") or op.startswith("v_readlane") or op.startswith("s_"):
        return set(), vregs(rest) if not op.startswith("s_") else set()
    d = vregs(ops[0])
    u = vregs(",".join(ops[1:]))
    return d, u


live_in = [set() for _ in blocks]
changed = True
while changed:
    changed = False
    for i in range(len(blocks) - 1, -1, -1):
        bl = blocks[i]
        out = set().union(*[live_in[j] for j in bl["succ"]]) if bl["succ"] else set()
        live = set(out)
        for t in reversed(bl["ins"]):
            d, u = defs_uses(t)
            live = (live - d) | u
        if live != live_in[i]:
            live_in[i] = live
            changed = True

points = []
for i, bl in enumerate(blocks):
    out = set().union(*[live_in[j] for j in bl["succ"]]) if bl["succ"] else set()
    live = set(out)
    for t in reversed(bl["ins"]):
        d, u = defs_uses(t)
        live = (live - d) | u
        points.append((len(live), bl["name"], t))
points.sort(key=lambda x: -x[0])
for n, bn, t in points[:top]:
    print(f"{n:3d}  {bn:14s} {t[:80]}")

if len(sys.argv) > 3:  # dump live set at the first instruction of block argv[3] with last defs
    want = sys.argv[3]
    i = idx[want]
    live = sorted(live_in[i])
    print("live-in", want, len(live), live)
    flat = [(bl["name"], t) for bl in blocks for t in bl["ins"]]
    start = [k for k, (bn, _) in enumerate(flat) if bn == want][0]
    for r in live:
        for k in range(start - 1, -1, -1):
            d, _ = defs_uses(flat[k][1])
            if r in d:
                print(f"  v{r:<3d} <- {flat[k][0]:12s} {flat[k][1][:70]}")
                break
