"""Per-kernel VGPRs / occupancy / scratch of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage),
optionally against the same file at a git revision: python scripts/reg_usage.py csrc/x.hip [rev]"""
import os
import re
import subprocess
import sys

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gemma.ggml_amd")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
         "-I../include", "-Icsrc", "-c", "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]


def usage(path):
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, path], cwd=PKG, capture_output=True, text=True)
    out, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]|VGPRs Spill): (\d+)", line)
        if m and cur:
            key = {"VGPRs": "vgpr", "VGPRs Spill": "vspill", "ScratchSize [bytes/lane]": "scratch"}.get(m.group(1), "occ")
            out[cur][key] = int(m.group(2))
    return out


if __name__ == "__main__":
    src = sys.argv[1]
    new = usage(src)
    old = None
    if len(sys.argv) > 2:
        txt = subprocess.run(["git", "show", f"{sys.argv[2]}:gemma.ggml_amd/{src}"], cwd=PKG, capture_output=True, text=True).stdout
        tmp = os.path.join(PKG, os.path.dirname(src), "_ru_old_" + os.path.basename(src))
        open(tmp, "w").write(txt)
        try:
            old = usage(os.path.relpath(tmp, PKG))
        finally:
            os.remove(tmp)
    for k, v in sorted(new.items()):
        o = old.get(k) if old else None
        if old is not None and o == v:
            continue
        print(f"{k[:90]:90s} {v}" + (f"   was {o}" if old is not None else ""))
