"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin)."""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                       capture_output=True, text=True).stdout.splitlines()
for r, n in zip(rows, names):
    n = n.replace("dpf_amd::", "")
    n = n[:70]
    print("%-70s vgpr=%-4s agpr=%-4s scratch=%-4s occ=%s lds=%s" % (
        n, r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize [bytes/lane]"),
        r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))
