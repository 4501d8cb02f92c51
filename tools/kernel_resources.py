"""Per-kernel register / scratch / occupancy report of libgsr's HIP sources (CPU only: hipcc's
kernel-resource-usage remarks).  A render kernel that spills at its waves-per-SIMD bound pays
scratch round trips in its batch loop.  Usage: python tools/kernel_resources.py [regex]"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splatam_amd import build  # noqa: E402


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else "render_|gauss_bwd|preprocess|duplicate")
    for src in build.SOURCES:
        cmd = [build.hipcc(), *build.flags(), "--cuda-device-only", "-c", "-o", os.devnull,
               os.path.join(build.CSRC, src), "-Rpass-analysis=kernel-resource-usage"]
        out = subprocess.run(cmd, capture_output=True, text=True).stderr
        cur = None
        rows = []
        for line in out.splitlines():
            m = re.search(r"remark: (.*?) \[-Rpass", line)
            if not m:
                continue
            body = m.group(1).strip()
            if body.startswith("Function Name:"):
                cur = {"name": body.split(":", 1)[1].strip()}
                rows.append(cur)
            elif cur is not None and ":" in body:
                k, v = body.split(":", 1)
                cur[k.strip()] = v.strip()
        for r in rows:
            if not pat.search(r["name"]):
                continue
            name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
            name = re.sub(r"\(.*", "", name).replace("gsr::", "")
            print(f"{name:60s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} "
                  f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4s} occ {r.get('Occupancy [waves/SIMD]', '?'):>2s} "
                  f"lds {r.get('LDS Size [bytes/block]', '?')}")


if __name__ == "__main__":
    main()
