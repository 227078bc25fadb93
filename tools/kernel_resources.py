"""Per-kernel resource usage (VGPRs, SGPRs, LDS, scratch) of the gfx950 code object inside a hipcc -c object.

The object's .hip_fatbin section is a clang offload bundle ("__CLANG_OFFLOAD_BUNDLE__", entry count, then
per entry: offset, size, triple length, triple); the gfx950 entry is an AMDGPU ELF whose note holds the
kernel metadata that `llvm-readelf --notes` prints.  Used by tests/test_kernel_resources.py to keep the
occupancy budgets DESIGN.md depends on (K2R: two 8-wave workgroups per CU).

usage: python3 tools/kernel_resources.py semi-direct-visual-odometry_amd/build/align_ref.o
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size",
          "vgpr_spill_count", "sgpr_spill_count")


def code_object(obj_path, arch="gfx950"):
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj_path, os.path.join(td, "o")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    if not data.startswith(magic):
        raise ValueError(f"{obj_path}: .hip_fatbin is not an uncompressed offload bundle")
    pos = len(magic)
    (n,) = struct.unpack_from("<Q", data, pos)
    pos += 8
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", data, pos)
        pos += 24
        triple = data[pos:pos + tlen].decode()
        pos += tlen
        if triple.endswith(arch) or f"--{arch}" in triple:
            return data[off:off + size]
    raise ValueError(f"{obj_path}: no {arch} entry in the bundle")


def resources(obj_path, arch="gfx950"):
    """{kernel symbol: {field: int}} from the code object's metadata note."""
    co = code_object(obj_path, arch)
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        text = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], check=True, capture_output=True,
                              text=True).stdout
    out, cur = {}, {}
    # each kernel's map lists its fields alphabetically, .vgpr_spill_count last
    for line in text.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if key in FIELDS:
            cur[key] = int(val)
        elif key == "name" and val.startswith("_Z"):
            cur["_name"] = val
        if key == "vgpr_spill_count":
            if "_name" in cur:
                out[cur.pop("_name")] = {k: v for k, v in cur.items() if k in FIELDS}
            cur = {}
    return out


def main():
    for name, r in sorted(resources(sys.argv[1]).items()):
        print(name, " ".join(f"{k}={r.get(k)}" for k in FIELDS))


if __name__ == "__main__":
    main()
