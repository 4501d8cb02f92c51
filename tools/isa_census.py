"""ISA census of a kernel's innermost loops (CPU only: hipcc -S for gfx950).

usage: python tools/isa_census.py SOURCE.hip KERNEL_SUBSTRING [EXTRA_HIPCC_FLAGS...]

Compiles SOURCE for gfx950 (same flags as splatam_amd/build.py), finds the first kernel whose
mangled name contains KERNEL_SUBSTRING and prints, for every loop of depth >= 2 (the render walks),
its VALU / SALU / LDS / VMEM instruction counts, plus the kernel's VGPR / SGPR / LDS / occupancy
metadata.  A loop's count is static (one pass through its body)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, name = sys.argv[1], sys.argv[2]
    extra = sys.argv[3:]
    out = os.path.join(tempfile.gettempdir(), "gsr_census.s")
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950", *([] if os.environ.get("CENSUS_SLP") else ["-fno-slp-vectorize"]),
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "splatam_amd", "csrc"),
           "--cuda-device-only", "-S", "-o", out, src, *extra]
    subprocess.run(cmd, check=True, capture_output=True)
    lines = open(out).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(name) + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    # loops: '; =>This Inner Loop Header: Depth=N' labels up to the back-edge branching to them
    headers = []  # (line of the loop's label, depth, label)
    for i, l in enumerate(body):
        m = re.search(r"Loop Header: Depth=(\d+)", l)
        if m:
            j = i if l.startswith(".LBB") else i - 1
            headers.append((j, int(m.group(1)), body[j].split(":")[0]))

    def classify(seg):
        c = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "trans": 0, "dpp": 0}
        for x in seg:
            t = x.strip().split()
            if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
                continue
            op = t[0]
            if op.startswith("v_"):
                c["valu"] += 1
                if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_", op):
                    c["trans"] += 1
                if "dpp" in op or "row_" in x or "quad_perm" in x:
                    c["dpp"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith(("global_", "buffer_", "flat_")):
                c["vmem"] += 1
        return c

    def block_starts():
        return [j for j, l in enumerate(body) if l.startswith(".LBB") or l.startswith("; %bb.")]

    starts = block_starts()
    for i, depth, lab in headers:
        key = "Header=" + lab[2:]  # (".LBB5_94" -> "Header=BB5_94")
        mine = [j for j in starts if j == i or key in body[j]] or [i]  # the loop's blocks (nested loops' blocks
        first = min(mine)                                              # name their own header, so are excluded:
        last_start = max(mine)                                         # fine for innermost loops)
        nxt = [j for j in starts if j > last_start]
        end_ = (nxt[0] - 1) if nxt else len(body) - 1
        if depth >= 2:
            print(f"loop {lab} depth {depth}: lines {first}-{end_}", classify(body[first:end_ + 1]))
    print("kernel total (static)", classify(body))
    for l in lines[end:end + 40]:
        if any(k in l for k in ("NumVgprs", "ScratchSize", "Occupancy", "LDSByteSize")):
            print(l.strip())


if __name__ == "__main__":
    main()
