#!/usr/bin/env python3
"""Per-kernel register / spill / scratch figures of the gfx950 code objects in build/obj/*.o (the objects
libkoordgpu.so is linked from): the AMDGPU metadata notes (.vgpr_count, .agpr_count, .sgpr_count, .vgpr_spill_count,
.sgpr_spill_count, .private_segment_fixed_size, .group_segment_fixed_size).

usage: python tools/kernel_resources.py [substring ...]   (default: every kernel)"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
        ".private_segment_fixed_size", ".group_segment_fixed_size")


def code_object(obj: str, tmp: str) -> str:
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, "co.elf")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(tmp, "x.o")])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                           f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"])
    return co


def kernels(co: str):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*(\.[a-z_]+):\s*(.*)$", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == ".agpr_count" and cur is None:
            cur = {}
        if cur is None:
            continue
        if k in KEYS:
            cur[k] = int(v)
        elif k == ".name":
            cur[".name"] = v
        elif k == ".wavefront_size":
            out.append(cur)
            cur = None
    return out


def main():
    subs = sys.argv[1:]
    rows = {}
    with tempfile.TemporaryDirectory() as tmp:
        for obj in sorted(glob.glob(os.path.join(ROOT, "build", "obj", "*.o"))):
            try:
                co = code_object(obj, tmp)
            except subprocess.CalledProcessError:
                continue
            for k in kernels(co):
                name = k.get(".name", "?")
                if subs and not any(s in name for s in subs):
                    continue
                rows[name] = k
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'lds':>6}  kernel")
    for name, k in sorted(rows.items()):
        print(f"{k.get('.vgpr_count', 0):5d} {k.get('.agpr_count', 0):5d} {k.get('.sgpr_count', 0):5d} "
              f"{k.get('.vgpr_spill_count', 0):6d} {k.get('.sgpr_spill_count', 0):6d} "
              f"{k.get('.private_segment_fixed_size', 0):7d} {k.get('.group_segment_fixed_size', 0):6d}  {name}")


if __name__ == "__main__":
    main()
