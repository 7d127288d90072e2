"""C ABI: libpqgpu.so loads, exports every function include/pqgpu.h declares, the ctypes
mirror matches the C struct layouts, and without a GPU every entry point fails loudly
(no CPU fallback). No compute calls here."""
import ctypes as C
import os
import re
import subprocess

import pytest

from pqgpu import abi, native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "pqgpu.h")
HEADERS = [os.path.join(REPO, "include", h) for h in sorted(os.listdir(os.path.join(REPO, "include"))) if h.endswith(".h")]


def declared_functions():
    text = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*\s]+?\b(pqg_\w+)\s*\(", text, re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ["pqg_decode", "pqg_decode_host", "pqg_plan_create", "pqg_plan_launch", "pqg_sync",
              "pqg_unpack_runs", "pqg_router_read", "pqg_ctx_create", "pqg_ctx_destroy"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = native.lib()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(native.EXPORTS) <= set(declared_functions())
    assert lib.pqg_abi_version() == abi.ABI_VERSION


def test_exports_via_nm():
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True).stdout
    syms = set(re.findall(r"\bT (pqg_\w+)", out))
    assert set(declared_functions()) <= syms


LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "pqgpu.h"
#define O(s, f) printf("%s.%s %zu\n", #s, #f, offsetof(s, f))
int main(void) {
  printf("pqg_page_desc %zu\npqg_column_desc %zu\npqg_status %zu\n", sizeof(pqg_page_desc), sizeof(pqg_column_desc), sizeof(pqg_status));
  O(pqg_page_desc, offset); O(pqg_page_desc, num_values); O(pqg_page_desc, dl_byte_length);
  O(pqg_page_desc, flags); O(pqg_page_desc, num_nulls);
  O(pqg_column_desc, dict_offset); O(pqg_column_desc, values); O(pqg_column_desc, def_levels);
  O(pqg_column_desc, binary_data); O(pqg_column_desc, values_written);
  O(pqg_status, value_index); O(pqg_status, message);
  return 0;
}
"""


def test_ctypes_layout_matches_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    assert int(got["pqg_page_desc"]) == C.sizeof(abi.PageDesc)
    assert int(got["pqg_column_desc"]) == C.sizeof(abi.ColumnDesc)
    assert int(got["pqg_status"]) == C.sizeof(abi.Status)
    for k, v in got.items():
        if "." in k:
            s, f = k.split(".")
            cls = {"pqg_page_desc": abi.PageDesc, "pqg_column_desc": abi.ColumnDesc, "pqg_status": abi.Status}[s]
            assert getattr(cls, f).offset == int(v), k
    assert abi.PAGE_DTYPE.itemsize == int(got["pqg_page_desc"])


def test_error_names_match():
    lib = native.lib()
    for code, name in abi.ERROR_NAMES.items():
        assert lib.pqg_error_name(code).decode() == name


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-device behaviour")
def test_no_device_fails_loudly():
    lib = native.lib()
    assert lib.pqg_device_count() == 0
    h = C.c_void_p()
    assert lib.pqg_ctx_create(0, None, C.byref(h)) == abi.ERR_NO_DEVICE
    from pqgpu import decoder
    with pytest.raises(native.PqgError):
        decoder.Decoder(0)


# ---- the JNI glue (shim/) against the C ABI: no JDK in the image, so a compile check and a name check --------

SHIM = os.path.join(REPO, "shim")


def test_jni_glue_compiles_against_the_abi():
    """shim/jni/pqgpu_jni.c compiles warning-free against include/ and a declaration-only jni.h
    (tests/c/jni_stub/jni.h: the JNI functions the glue calls, with the specification's signatures)."""
    subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I",
                    os.path.join(REPO, "tests", "c", "jni_stub"), "-I", os.path.join(REPO, "include"),
                    os.path.join(SHIM, "jni", "pqgpu_jni.c")], check=True)


def test_every_java_native_has_its_jni_symbol():
    """Each `native` method of PqGpu.java has the JNIEXPORT function the JVM binds it to
    (Java_<package>_<class>_<method>), and the glue exports nothing else."""
    java = open(os.path.join(SHIM, "java", "org", "apache", "parquet", "column", "values", "gpu", "PqGpu.java")).read()
    natives = set(re.findall(r"\bstatic\s+native\s+[\w\[\]]+\s+(\w+)\s*\(", java))
    glue = open(os.path.join(SHIM, "jni", "pqgpu_jni.c")).read()
    exported = set(re.findall(r"Java_org_apache_parquet_column_values_gpu_PqGpu_(\w+)\s*\(", glue))
    assert natives and natives == exported, (natives ^ exported)


def test_java_readers_use_only_declared_batch_members():
    """The readers call GpuPageBatch members that exist (a name check of the Java sources, which cannot be
    compiled here)."""
    d = os.path.join(SHIM, "java", "org", "apache", "parquet", "column", "values", "gpu")
    batch = open(os.path.join(d, "GpuPageBatch.java")).read()
    for f in ("GpuValuesReader.java", "GpuLevelsReader.java"):
        src = open(os.path.join(d, f)).read()
        for m in set(re.findall(r"\bbatch\.(\w+)", src)):
            assert re.search(r"\b" + m + r"\b\s*[;(=\[]", batch), (f, m)
