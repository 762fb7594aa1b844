"""Per-kernel VGPRs / scratch / occupancy of kernels.hip from the compiler's
resource-usage remarks (run from smallpt-enoki-optix_amd/):
    python ../tools/kres.py [extra hipcc flags]"""
import re
import subprocess
import sys

# the Makefile's device flags (COMMON + HIPFLAGS): without -ffp-contract=off the
# compiler forms FMAs the product does not, and the register counts differ
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I../include",
       "-Icsrc", "-x", "hip", "-fhip-fp32-correctly-rounded-divide-sqrt",
       "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
       "-Rpass-analysis=kernel-resource-usage",
       "-c", "csrc/kernels.hip", "-o", "/dev/null"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
name = None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        rec = {}
        continue
    for k in ("VGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(k + r": (\d+)", line)
        if m and name:
            rec[k.split()[0]] = int(m.group(1))
            if k.startswith("Occupancy"):
                short = re.sub(r"_ZN3spt\d+", "", name)[:70]
                print(f"{short:72s} vgpr {rec.get('VGPRs')} scratch {rec.get('ScratchSize')} waves {rec['Occupancy']}")
