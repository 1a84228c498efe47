"""No kernel we ship writes through the scalar data cache (tools/isa_audit.py):
the product and bounds-checking builds' gfx950 code objects are disassembled
and searched.  CPU only (hipcc's LLVM tools); listed in .gpurunignore."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIBS = [os.path.join(ROOT, "java-reed-solomon-distributed-file-system_amd", "lib", p)
        for p in ("librsamd.so", os.path.join("bounds", "librsamd.so"))]


@pytest.mark.parametrize("so", LIBS, ids=["product", "bounds"])
def test_no_scalar_cache_writes(so):
    import isa_audit
    if not os.path.exists(so) or not os.path.exists(os.path.join(isa_audit.LLVM, "llvm-objdump")):
        pytest.skip("library or LLVM tools absent")
    counts = isa_audit.mnemonics(so)
    assert sum(counts.values()) > 1000 and "v_perm_b32" in counts and "v_bitop3_b32" in counts
    assert isa_audit.scalar_cache_writes(counts) == {}
