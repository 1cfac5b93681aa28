"""Kernel resource table (VGPRs, SGPR / VGPR spills, occupancy) of one HIP source, from
hipcc -Rpass-analysis=kernel-resource-usage.  usage: kres.py file.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
p = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                    "-ffp-contract=off", "-c", "-o", "/tmp/_kres.o", src,
                    "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:],
                   capture_output=True, text=True)
cur, rows = None, {}
for line in p.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: ([A-Za-z \[\]/]+): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{v.get('VGPRs', 0):4d} vgpr {v.get('SGPRs', 0):4d} sgpr "
              f"{v.get('SGPRs Spill', 0):3d} sspill {v.get('VGPRs Spill', 0):3d} vspill "
              f"occ {v.get('Occupancy [waves/SIMD]', 0)}  {k[:90]}")
