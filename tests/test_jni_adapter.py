"""jni/rs_jni.c -- the JNIEnv adapter, the one product file no JDK-less build
compiles -- compiled against a declarations-only jni.h written from the JNI
specification (tests/jni_spec/jni.h), with -Wall -Wextra -Werror and every
symbol resolved (-Wl,--no-undefined against librsamd.so).  Then the natives
it exports are checked against the `native` methods of the Java classes
(jni/java/edu/cmu/reedsolomon/*.java): every declared native has exactly one
implementation under its JNI name and nothing else is exported as a native.

This checks names, argument and return types; it does not claim ABI parity
with a real JDK's jni.h (the subset's function table omits unused entries).
"""
import os
import re
import subprocess

import pytest

from conftest import PKG_DIR, ROOT

JNI = os.path.join(PKG_DIR, "jni")
JAVA = os.path.join(JNI, "java", "edu", "cmu", "reedsolomon")


def java_natives():
    """JNI names of every `native` method of the Java facade classes."""
    out = set()
    for cls in ("NativeReedSolomon", "GpuCodingLoop"):
        text = open(os.path.join(JAVA, cls + ".java")).read()
        for name in re.findall(r"\bnative\s+[\w\[\]<>.]+\s+(\w+)\s*\(", text):
            assert "_" not in name  # (JNI would escape it as _1)
            out.add(f"Java_edu_cmu_reedsolomon_{cls}_{name}")
    return out


def test_adapter_compiles_and_exports_every_native(tmp_path):
    from rsamd import _lib
    _lib.load()  # the library is built (build()); the link resolves against it
    so = str(tmp_path / "librsamd_jni.so")
    libdir = os.path.join(PKG_DIR, "lib")
    cmd = ["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "tests", "jni_spec"), "-I" + os.path.join(ROOT, "include"), "-I" + JNI,
           os.path.join(JNI, "rs_jni.c"), os.path.join(JNI, "rs_jni_core.c"), "-L" + libdir, "-lrsamd",
           "-Wl,--no-undefined", "-o", so]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert p.returncode == 0, p.stdout
    nm = subprocess.run(["nm", "-D", "--defined-only", so], stdout=subprocess.PIPE, text=True, check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if " T Java_" in line}
    want = java_natives()
    assert len(want) >= 20
    assert exported == want, (sorted(want - exported), sorted(exported - want))


def test_spec_subset_is_not_a_jdk_header():
    """The subset header says what it is and that nothing built on it may run."""
    text = open(os.path.join(ROOT, "tests", "jni_spec", "jni.h")).read()
    assert "declarations-only" in text and "nothing built against" in text
    if os.path.exists("/usr/lib/jvm"):
        pytest.skip("a JDK is present: build against its own jni.h too (INTEGRATION.md)")
