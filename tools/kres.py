"""Print per-kernel VGPR/SGPR/LDS/occupancy from hipcc -Rpass-analysis output.

usage: python tools/kres.py <file.hip> [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast",
       "-I", "orange3_spark_amd/ops/csrc", "-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, stderr=subprocess.PIPE, stdout=subprocess.PIPE, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([\w \[\]/]+?): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if flt in k:
        print(f"{v.get('VGPRs','?'):>4} vgpr {v.get('AGPRs','?'):>3} agpr {v.get('TotalSGPRs','?'):>4} sgpr "
              f"occ {v.get('Occupancy [waves/SIMD]','?'):>2} lds {v.get('LDS Size [bytes/block]','?'):>6} "
              f"scratch {v.get('ScratchSize [bytes/lane]','?')}  {k[:110]}")
