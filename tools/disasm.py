"""Disassemble the gfx950 code of the kernels of libu3d.so whose (mangled) symbol matches a regex, and count their
instruction classes. Usage: python tools/disasm.py REGEX [lib.so] [--full]"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_resources as KR  # noqa: E402


def disasm(rx, lib=KR.LIB):
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for k, co in enumerate(KR.code_objects(lib)):
            f = os.path.join(d, f"co{k}.elf")
            open(f, "wb").write(co)
            txt = subprocess.run([os.path.join(KR.LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", f],
                                 check=True, capture_output=True, text=True).stdout
            for m in re.finditer(r"\n([0-9a-f]+) <([^>]+)>:\n(.*?)(?=\n[0-9a-f]+ <|\Z)", txt, re.S):
                if re.search(rx, m.group(2)):
                    out[m.group(2)] = [ln.strip() for ln in m.group(3).splitlines() if ln.strip()]
    return out


if __name__ == "__main__":
    rx = sys.argv[1]
    lib = next((a for a in sys.argv[2:] if a.endswith(".so")), KR.LIB)
    for name, lines in disasm(rx, lib).items():
        ops = Counter(ln.split()[0] for ln in lines if not ln.startswith(";"))
        cls = Counter()
        for op, c in ops.items():
            key = ("mfma" if "mfma" in op else "ds_read" if op.startswith("ds_read") else
                   "ds_write" if op.startswith("ds_write") else "vmem_load" if re.match(r"(buffer|global)_load", op) else
                   "vmem_store" if re.match(r"(buffer|global)_store", op) else "s_waitcnt" if op == "s_waitcnt" else
                   "s_barrier" if op == "s_barrier" else "smem_store" if re.match(r"s_(store|buffer_store|atomic)", op)
                   else "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else "other")
            cls[key] += c
        print(KR.demangle([name])[0], dict(cls))
        if "--full" in sys.argv:
            print("\n".join(lines))
