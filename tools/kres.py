"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin) as a table."""
import re, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\S+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat in r["name"]:
        print(f'{r["name"][:60]:60s} vgpr={r.get("VGPRs")} agpr={r.get("AGPRs")} sgpr={r.get("TotalSGPRs")} '
              f'occ={r.get("Occupancy [waves/SIMD]")} scratch={r.get("ScratchSize [bytes/lane]")} lds={r.get("LDS Size [bytes/block]")}')
