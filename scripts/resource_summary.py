"""Condense hipcc -Rpass-analysis=kernel-resource-usage remarks to one line per kernel."""
import re
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(.+?): (\S+) \[-Rpass", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
keys = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("TotalSGPRs", "sgpr"), ("VGPRs Spill", "vspill"),
        ("SGPRs Spill", "sspill"), ("ScratchSize [bytes/lane]", "scratch"), ("Occupancy [waves/SIMD]", "occ")]
for r in rows:
    if "step_kernel" not in r["name"]:
        continue
    import subprocess
    try:
        name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    except OSError:
        name = r["name"]
    print(f"{name:70s} " + " ".join(f"{short}={r.get(k, '?')}" for k, short in keys))
