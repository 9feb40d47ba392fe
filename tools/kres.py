"""Per-kernel resource usage (VGPRs, SGPRs, spills, scratch, occupancy, LDS)
of csrc/kernels.hip from the compiler's kernel-resource-usage remarks.
    python tools/kres.py [extra hipcc flags...]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
CSRC = ROOT + "/madrona-mp-env_amd/csrc"
cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-c",
       CSRC + "/kernels.hip", "-o", "/tmp/kres.o", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
       "-I" + CSRC, "-I" + ROOT + "/include", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(-?\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for f, r in rows.items():
    name = re.sub(r"_ZN5mpenv\d+(\w+?)E.*", r"\1", f)
    if not name.startswith("k_"):
        continue
    print(f"{name:16s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', 0):>3} SGPR {r.get('SGPRs', '?'):>4} "
          f"VGPRspill {r.get('VGPRs Spill', 0):>4} SGPRspill {r.get('SGPRs Spill', 0):>4} "
          f"scratch {r.get('ScratchSize [bytes/lane]', 0):>4} occ {r.get('Occupancy [waves/SIMD]', '?'):>2} "
          f"LDS {r.get('LDS Size [bytes/block]', 0)}")
