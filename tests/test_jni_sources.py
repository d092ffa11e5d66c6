"""CPU: the JVM drop-in sources agree with the C-ABI.

There is no JDK in this image, so src/main/native/sux_jni.c, SuxNative.java and the Scala plugin
classes cannot be compiled here.  What can be checked statically, is:
  - every `native` method of SuxNative.java has its JNI function in sux_jni.c and back, with the
    same number of arguments (JNIEnv* and jclass aside);
  - every sux_* function sux_jni.c calls is declared in include/sparkucx_amd.h and exported by
    the built library;
  - every SuxNative.x the Java/Scala sources call is declared;
  - SuxNative's constants equal the header's #defines (status codes, partitioner kinds, ABI).
"""
import os
import re

import pytest

from sparkucx_amd import native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "src", "main", "native", "sux_jni.c")
JAVA = os.path.join(ROOT, "src", "main", "java", "org", "apache", "spark", "shuffle", "ucx", "gpu",
                    "SuxNative.java")
HEADER = os.path.join(ROOT, "include", "sparkucx_amd.h")


def _read(p):
    with open(p) as f:
        return f.read()


def _java_natives():
    text = _read(JAVA)
    out = {}
    for m in re.finditer(r"public static native [\w\[\]]+ (\w+)\(([^)]*)\);", text, re.S):
        params = [p for p in m.group(2).split(",") if p.strip()]
        out[m.group(1)] = len(params)
    return out


def _jni_functions():
    text = _read(JNI)
    out = {}
    for m in re.finditer(r"JNIEXPORT [\w\s]+ JNICALL FN\((\w+)\)\(([^)]*)\)", text, re.S):
        params = [p for p in m.group(2).split(",") if p.strip()]
        out[m.group(1)] = len(params) - 2  # JNIEnv*, jclass
    return out


def test_every_native_method_has_its_jni_function():
    java, c = _java_natives(), _jni_functions()
    assert len(java) >= 25
    assert set(java) == set(c), set(java) ^ set(c)
    for name, n in java.items():
        assert c[name] == n, (name, n, c[name])


def test_jni_calls_only_declared_and_exported_c_abi():
    called = set(re.findall(r"\b(sux_[a-z_0-9]+)\(", _read(JNI)))
    declared = set(N.header_symbols())
    assert called <= declared, called - declared
    lib = N.load()
    assert all(hasattr(lib, s) for s in called)


def test_plugin_sources_call_declared_natives():
    java = _java_natives()
    used = set()
    for d, _, files in os.walk(os.path.join(ROOT, "src", "main")):
        for f in files:
            if f.endswith((".scala", ".java")):
                used |= set(re.findall(r"SuxNative\.(\w+)\(", _read(os.path.join(d, f))))
    assert used, "the plugin classes call the native layer"
    assert used <= set(java), used - set(java)


@pytest.mark.parametrize("java_name,define", [
    ("OK", "SUX_OK"), ("EINVAL", "SUX_EINVAL"), ("ENOMEM", "SUX_ENOMEM"), ("EHIP", "SUX_EHIP"),
    ("ECOMM", "SUX_ECOMM"), ("ENOENT", "SUX_ENOENT"), ("ESTATE", "SUX_ESTATE"),
    ("ERANGE", "SUX_ERANGE"), ("EIO", "SUX_EIO"), ("ABI_VERSION", "SUX_ABI_VERSION"),
    ("PART_RANGE_BYTES", "SUX_PART_RANGE_BYTES"), ("PART_MURMUR3_LONG", "SUX_PART_MURMUR3_LONG"),
    ("PART_MURMUR3_INT", "SUX_PART_MURMUR3_INT"), ("PART_MURMUR3_BYTES", "SUX_PART_MURMUR3_BYTES"),
    ("PART_HASH_LONG", "SUX_PART_HASH_LONG"), ("PART_HASH_INT", "SUX_PART_HASH_INT"),
])
def test_constants_match_header(java_name, define):
    h = re.search(rf"#define {define} (-?\d+)", _read(HEADER))
    j = re.search(rf"\b{java_name} = (-?\d+)", _read(JAVA))
    assert h and j and int(h.group(1)) == int(j.group(1)), (java_name, define)


def test_jni_binding_compiles_warning_free():
    """sux_jni.c compiles with -Wall -Wextra -Werror against the JNI test double (no JDK here):
    every JNI call it makes names a JNI function with the specification's signature."""
    import subprocess
    src = os.path.join(ROOT, "src", "main", "native", "sux_jni.c")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", os.path.join(ROOT, "tests", "jni"), src],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
