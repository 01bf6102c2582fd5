#!/usr/bin/env python3
"""Per-kernel resource table of a built library, read from its gfx950 code objects: VGPRs, AGPRs,
SGPRs, scratch bytes per lane, VGPR / SGPR spill counts (SGPRs spill to VGPR lanes, not memory), static
LDS bytes, workgroup size limit.  No GPU needed (the code objects
sit in the .so's offload bundles; llvm-readelf prints their AMDGPU metadata notes).

    python scripts/kernel_resources.py [sclmd_amd/_lib/libhipgle.so] [--json]

tests/test_kernel_resources.py fails the CPU suite when a kernel of the release library uses scratch
(a register spill or a runtime-indexed register array: both turn into per-lane memory traffic)."""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_FIELDS = {".name": str, ".symbol": str, ".vgpr_count": int, ".agpr_count": int, ".sgpr_count": int,
           ".private_segment_fixed_size": int, ".group_segment_fixed_size": int, ".vgpr_spill_count": int,
           ".sgpr_spill_count": int, ".max_flat_workgroup_size": int, ".wavefront_size": int}


def code_objects(lib, arch="gfx950"):
    """The device ELF images of `arch` in every offload bundle of `lib` (one bundle per source file)."""
    d = open(lib, "rb").read()
    i = d.find(_MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", d, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", d, p)
            triple = d[p + 24:p + 24 + tl]
            p += 24 + tl
            if arch.encode() in triple and size:
                yield d[i + off:i + off + size]
        i = d.find(_MAGIC, i + 1)


def _kernels(notes):
    """Parse the amdhsa.kernels list of one metadata note (YAML as printed by llvm-readelf): one dict
    per kernel, keyed by the top-level kernel fields only (argument entries are nested deeper)."""
    out, cur, kind = [], None, None
    for line in notes.splitlines():
        m = re.match(r"^  - (\.\w+):\s*(.*)$", line)
        if m:  # a new kernel entry starts
            cur = {}
            out.append(cur)
            line = "    %s: %s" % (m.group(1), m.group(2))
        m = re.match(r"^    (\.\w+):\s*(.*)$", line)
        if m and cur is not None and m.group(1) in _FIELDS:
            kind = _FIELDS[m.group(1)]
            try:
                cur[m.group(1)[1:]] = kind(m.group(2).strip())
            except ValueError:
                pass
        if line.startswith("amdhsa.target") or line.startswith("amdhsa.version"):
            cur = None
    return out


def kernel_resources(lib, arch="gfx950"):
    rows = []
    for img in code_objects(lib, arch):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(img)
            f.flush()
            notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True, check=True).stdout
        rows += [k for k in _kernels(notes) if "name" in k]
    return rows


def _demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(ROOT, "sclmd_amd", "_lib", "libhipgle.so")
    rows = kernel_resources(lib)
    if "--json" in sys.argv:
        print(json.dumps(rows))
        return
    names = _demangle([r["name"] for r in rows])
    print("%-6s %-5s %-5s %-8s %-7s %-7s %-7s %-5s  %s" % ("vgpr", "agpr", "sgpr", "scratch", "vspill", "sspill", "lds",
                                                      "wg", "kernel"))
    for r, nm in sorted(zip(rows, names), key=lambda x: x[1]):
        print("%-6d %-5d %-5d %-8d %-7d %-7d %-7d %-5d  %s" % (
            r.get("vgpr_count", 0), r.get("agpr_count", 0), r.get("sgpr_count", 0),
            r.get("private_segment_fixed_size", 0), r.get("vgpr_spill_count", 0), r.get("sgpr_spill_count", 0),
            r.get("group_segment_fixed_size", 0), r.get("max_flat_workgroup_size", 0), nm[:150]))


if __name__ == "__main__":
    main()
