"""Static instruction counts per phase of k_transport between the WG_MARKS asm comments
(hipcc -S -DWG_MARKS ...; see wg_transport.hip). Counts every instruction of every block in
the region, so branches that a given packet skips are included; loops are not multiplied.
Usage: python tools/isa_phases.py build/marks.s <kernel-symbol>"""
import collections
import re
import sys

path, name = sys.argv[1], sys.argv[2]
s = open(path).read()
a = s.index(name + ":")
b = s.index(".Lfunc_end", a)
region = "prologue"
cnt = collections.OrderedDict()
for line in s[a:b].splitlines():
    m = re.search(r";; WGMARK (\d+)", line)
    if m:
        region = "after mark " + m.group(1)
        continue
    t = line.strip()
    if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
        continue
    op = t.split()[0]
    c = cnt.setdefault(region, collections.Counter())
    kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(("s_load", "s_buffer", "s_waitcnt", "s_cbranch", "s_branch", "s_nop")) else
            "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else
            "branch" if op.startswith(("s_cbranch", "s_branch")) else "other")
    c[kind] += 1
    c["op:" + op] += 1
for r, c in cnt.items():
    print(f"{r:16s} valu {c['valu']:5d} salu {c['salu']:4d} lds {c['lds']:3d} vmem {c['vmem']:3d} branch {c['branch']:3d}")
    top = sorted(((v, k[3:]) for k, v in c.items() if k.startswith("op:v_")), reverse=True)[:8]
    print("                 " + ", ".join(f"{k} {v}" for v, k in top))
