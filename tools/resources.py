#!/usr/bin/env python
"""Per-kernel register / scratch / spill summary of libnestmc (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys
import os

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mcmc-for-nested-data_amd",
                    "csrc")
out = subprocess.run(["make", "-s", "-B", "asm"], cwd=CSRC, capture_output=True, text=True).stderr
pat = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if pat in r["name"]:
        print("%-62s sgpr=%-4s vgpr=%-4s scratch=%-3s occ=%-2s sspill=%-4s vspill=%s" % (
            r["name"][:62], r.get("TotalSGPRs"), r.get("VGPRs"), r.get("ScratchSize [bytes/lane]"),
            r.get("Occupancy [waves/SIMD]"), r.get("SGPRs Spill"), r.get("VGPRs Spill")))
