"""Register / LDS / scratch usage of the kernels of one translation unit (hipcc -Rpass-analysis remarks).
Usage: python tools/regs.py qoc_run_tchain [regex]"""
import re
import subprocess
import sys

tu = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
src = f"quantumoptimalcontrol.jl_amd/csrc/{tu}.hip"
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-o", "/dev/null",
                      "-Wno-unused-value", "-Wno-unused-result", "-Rpass-analysis=kernel-resource-usage", src],
                     capture_output=True, text=True).stderr
cur, res = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        res[cur] = {}
        continue
    m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
    if m and cur:
        res[cur][m.group(1).split()[0]] = int(m.group(2))
names = subprocess.run(["c++filt"], input="\n".join(res), capture_output=True, text=True).stdout.splitlines()
for (k, v), d in zip(res.items(), names):
    if pat.search(d):
        print(f"{d[:100]:100s} V{v.get('VGPRs')} A{v.get('AGPRs')} S{v.get('ScratchSize')} occ{v.get('Occupancy')}")
