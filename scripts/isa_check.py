#!/usr/bin/env python3
"""Register-pressure check of the closest-point traversal kernel (CPU only, no GPU needed).

Compiles mesh_amd/csrc/nearest.hip to gfx950 assembly (optionally with extra -D flags) and reports, for
k_knn<MODE, false, LIST, PF>, the VGPR count, the spill count and how many scratch (spill) instructions sit inside
the tile's traversal loop (LLVM's block annotations "in Loop: ... Depth=N", N >= 2).  A spill reload
inside that loop costs a memory round trip per iteration: A/B runs showed -13 % for two such reloads, so a
variant with loop spills is not worth a GPU session.

    python scripts/isa_check.py [-DMSH_LEAF_Q=4 ...]
"""
import os
import re
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(R, "mesh_amd", "csrc", "nearest.hip")


def compile_asm(flags):
    out = tempfile.NamedTemporaryFile(suffix=".s", delete=False).name
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950",
           "--cuda-device-only", "-S", SRC, "-o", out] + flags
    subprocess.run(cmd, check=True, cwd=os.path.dirname(SRC), stderr=subprocess.DEVNULL)
    with open(out) as f:
        s = f.read()
    os.unlink(out)
    return s


def report(s, mode):
    name = f"_ZN3msh5k_knnILi{mode}ELb0ELb{int(LIST)}ELb{int(PF)}EEEvNS_7KnnArgsE"
    meta = s[re.search(r"\.name:\s+" + name + r"\n", s).start():][:1500]
    vgpr = int(re.search(r"\.vgpr_count:\s+(\d+)", meta).group(1))
    spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", meta).group(1))
    a = s.index(name + ":")
    b = s.index(".end_amdhsa_kernel", a)
    depth = 0
    total = in_loop = 0
    for line in s[a:b].split("\n"):
        m = re.search(r"Depth=(\d+)", line)
        if line.startswith(".LBB") or line.startswith("; %bb"):
            depth = int(m.group(1)) if m else 0
        if "scratch_" in line:
            total += 1
            if depth >= 2:
                in_loop += 1
    lds = int(re.search(r"amdhsa_group_segment_fixed_size (\d+)", s[a:b + 400]).group(1))
    return dict(mode=mode, vgpr=vgpr, vgpr_spill=spill, scratch_ops=total, scratch_in_loop=in_loop, lds=lds)


LIST = True  # the wave-leaf-list instantiation k_knn<MODE, false, true, PF> (the closest-point path)
PF = True    # with LDS node prefetch and 4-B stack entries (trees of <= 2^20 leaves)


def main():
    global LIST, PF
    flags = sys.argv[1:]
    s = compile_asm(flags)
    for LIST, PF in ((True, True), (True, False), (False, False)):
        for mode in (0, 3):
            print(dict(report(s, mode), list=LIST, prefetch=PF))


if __name__ == "__main__":
    main()
