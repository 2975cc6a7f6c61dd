"""Register / LDS / occupancy table of every kernel in a HIP source, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (compile only, no GPU).
usage: python tools/kernel_resources.py inferd_amd/csrc/gemm.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = ["-fno-honor-nans", "-fno-slp-vectorize"] if src.endswith("attention.hip") else []
p = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-c", src, "-o", "/dev/null",
                    "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"] + extra,
                   capture_output=True, text=True)
rows, cur = [], None
for line in p.stderr.splitlines():
    m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
try:
    import subprocess as sp
    dem = sp.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(r["name"] for r in rows),
                 capture_output=True, text=True).stdout.splitlines()
    for r, d in zip(rows, dem):
        r["name"] = d
except Exception:
    pass
for r in rows:
    if flt in r["name"]:
        print(f'{r.get("VGPRs","?"):>4} v {r.get("AGPRs","?"):>3} a  spill {r.get("VGPRs Spill","?")}/'
              f'{r.get("SGPRs Spill","?")}  occ {r.get("Occupancy [waves/SIMD]","?")}  '
              f'lds {r.get("LDS Size [bytes/block]","?"):>6}  {r["name"][:150]}')
