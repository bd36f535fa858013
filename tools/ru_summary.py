"""Per-kernel register / scratch / occupancy summary of the transport kernels from the
-Rpass-analysis=kernel-resource-usage remarks (make -C wireguard-java_amd/csrc asm)."""
import re
import subprocess
import sys

KEYS = [("V", r"VGPRs: (\d+)"), ("S", r"TotalSGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
        ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("sgpr_spill", r"SGPRs Spill: (\d+)"),
        ("vgpr_spill", r"VGPRs Spill: (\d+)")]
pat = sys.argv[2] if len(sys.argv) > 2 else r"k_step|k_transport<|k_transport_mixed"
for blk in open(sys.argv[1]).read().split("Function Name: ")[1:]:
    name = blk.split()[0]
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if not re.search(pat, dem):
        continue
    vals = []
    for k, rx in KEYS:
        m = re.search(rx, blk)
        vals.append(f"{k}={m.group(1) if m else '?'}")
    print(f"{dem[:72]:72s} " + " ".join(vals))
