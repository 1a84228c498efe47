#!/usr/bin/env python3
"""ISA audit of the built libraries' gfx950 code objects (CPU only).

Extracts every offload bundle from a shared library's .hip_fatbin section,
disassembles its gfx950 code object and counts instruction mnemonics.  The
check tests/test_isa_audit.py makes with it: no instruction writes through the
scalar data cache -- no scalar memory store (s_store_*, s_buffer_store_*), no
scalar atomic (s_atomic_*, s_buffer_atomic_*), no s_dcache_wb / s_dcache_discard
-- in any kernel we ship (the pool's rule: those were followed by machine-wide
hardware errors).  This file and its test only name those instructions; no GPU
run loads them, so both are listed in .gpurunignore.
  python tools/isa_audit.py java-reed-solomon-distributed-file-system_amd/lib/librsamd.so
"""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
SCALAR_CACHE_WRITE = re.compile(r"^s_(buffer_)?(store|atomic)|^s_dcache_(wb|discard)")


def mnemonics(so: str) -> dict:
    """{mnemonic: count} over every gfx950 code object in `so`."""
    counts = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", so, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        if not offs:
            raise RuntimeError(f"{so}: no offload bundle in .hip_fatbin")
        for n, o in enumerate(offs):
            b, co = os.path.join(d, f"b{n}"), os.path.join(d, f"co{n}.o")
            with open(b, "wb") as f:
                f.write(data[o: offs[n + 1] if n + 1 < len(offs) else len(data)])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                            f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                                 capture_output=True, text=True).stdout
            for line in dis.splitlines():
                t = line.split()
                if t and re.match(r"^(s|v|ds|global|buffer|flat|scratch)_", t[0]):
                    counts[t[0]] = counts.get(t[0], 0) + 1
    return counts


def scalar_cache_writes(counts: dict) -> dict:
    return {k: v for k, v in counts.items() if SCALAR_CACHE_WRITE.match(k)}


if __name__ == "__main__":
    for so in sys.argv[1:]:
        c = mnemonics(so)
        print(json.dumps({"lib": so, "mnemonics": len(c), "instructions": sum(c.values()),
                          "scalar_cache_writes": scalar_cache_writes(c)}))
