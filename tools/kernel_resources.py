"""Per-kernel register / scratch usage of the gfx950 code objects inside libu3d.so (test + diagnostics).

Reads the .hip_fatbin section of the shared library (llvm-objcopy), splits its clang offload bundles, and parses the
AMDGPU metadata notes of every gfx950 code object (llvm-readelf --notes): name, .vgpr_count, .agpr_count,
.vgpr_spill_count, .sgpr_spill_count, .private_segment_fixed_size, .group_segment_fixed_size.
Usage: python tools/kernel_resources.py [lib.so] [--spills]"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "multimodal-pl_amd", "u3d", "libu3d.so")
KEYS = (".vgpr_count", ".agpr_count", ".vgpr_spill_count", ".sgpr_spill_count", ".private_segment_fixed_size",
        ".group_segment_fixed_size")


def code_objects(lib):
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fb, lib, os.devnull],
                       check=True, capture_output=True)
        b = open(fb, "rb").read()
    i = 0
    while True:
        j = b.find(b"__CLANG_OFFLOAD_BUNDLE__", i)
        if j < 0:
            return
        n = struct.unpack_from("<Q", b, j + 24)[0]
        p = j + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, p)
            triple = b[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                yield b[j + off:j + off + size]
        i = j + 1


def kernels(lib=LIB):
    """{kernel symbol: {key: int}} over every gfx950 code object of the library."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for k, co in enumerate(code_objects(lib)):
            f = os.path.join(d, f"co{k}.elf")
            with open(f, "wb") as fh:
                fh.write(co)
            txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f], check=True,
                                 capture_output=True, text=True).stdout
            for block in re.split(r"\n\s+- \.agpr_count:", txt)[1:]:
                block = ".agpr_count:" + block
                name = re.search(r"\.name:\s+(\S+)", block)
                if not name:
                    continue
                vals = {}
                for key in KEYS:
                    m = re.search(re.escape(key) + r":\s+(\d+)", block)
                    vals[key] = int(m.group(1)) if m else 0
                out[name.group(1)] = vals
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
        return r.stdout.splitlines() if r.returncode == 0 else list(names)
    except OSError:
        return list(names)


if __name__ == "__main__":
    lib = next((a for a in sys.argv[1:] if a.endswith(".so")), LIB)
    ks = kernels(lib)
    rows = sorted(ks.items(), key=lambda kv: (-kv[1][".vgpr_spill_count"], -kv[1][".private_segment_fixed_size"]))
    if "--spills" in sys.argv:
        rows = [r for r in rows if r[1][".vgpr_spill_count"] or r[1][".private_segment_fixed_size"]]
    for (name, v), dn in zip(rows, demangle([r[0] for r in rows])):
        print(f"vgpr {v['.vgpr_count']:3d} agpr {v['.agpr_count']:3d} spill {v['.vgpr_spill_count']:3d} "
              f"scratch {v['.private_segment_fixed_size']:4d} lds {v['.group_segment_fixed_size']:6d}  {dn}")
    print(f"{len(ks)} kernels")
