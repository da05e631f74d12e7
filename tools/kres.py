"""Per-kernel VGPRs / scratch / occupancy from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"\s(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0] + ("Spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for name, r in rows.items():
    if pat in name:
        short = re.sub(r"_ZN3hrs12_GLOBAL__N_1\d+", "", name)[:90]
        print(f"{short:92s} vgpr={r.get('VGPRs')} spill={r.get('VGPRsSpill')} scratch={r.get('ScratchSize')} occ={r.get('Occupancy')}")
