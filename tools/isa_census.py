"""Instruction census of one kernel in build/wgaead-gfx950.s (make -C wireguard-java_amd/csrc asm).
Usage: python tools/isa_census.py <mangled-name> [top]; prints static counts per opcode and per
basic block (label) so loop bodies can be weighed by their trip counts."""
import collections
import re
import sys

name = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
s = open("build/wgaead-gfx950.s").read()
a = s.index(name + ":")
b = s.index(".Lfunc_end", a)
lines = s[a:b].splitlines()
ops = collections.Counter()
blocks = collections.OrderedDict()
cur = "entry"
for l in lines:
    if re.match(r"^\.LBB\S+:", l):
        cur = l.split(":")[0]
        blocks[cur] = collections.Counter()
        continue
    t = l.strip()
    if not l.startswith("\t") or t.startswith((".", ";")) or not t:
        continue
    op = t.split()[0]
    ops[op] += 1
    blocks.setdefault(cur, collections.Counter())[op] += 1
print("total", sum(ops.values()), "valu", sum(v for k, v in ops.items() if k.startswith("v_")))
for k, v in ops.most_common(top):
    print(f"  {k:30s}{v}")
print("blocks (valu count):")
for k, c in blocks.items():
    nv = sum(v for o, v in c.items() if o.startswith("v_"))
    if nv:
        print(f"  {k:16s} valu {nv:5d}  total {sum(c.values()):5d}")
