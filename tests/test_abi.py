"""The C-ABI boundary (include/skm.h) on the CPU: libskm.so loads, exports every declared entry
point, and the host-only entry points behave (no GPU compute is issued here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "skm.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(skm_\w+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("skm_build_create", "skm_build_add_batch", "skm_build_finish", "skm_db_open",
                 "skm_db_lookup", "skm_annotate", "skm_mph_build", "skm_find_best_call", "skm_last_error"):
        assert must in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol(skm):
    lib = skm.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and they are real dynamic exports (extern "C", default visibility)
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT\s+(\w+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def test_python_bindings_cover_the_header(skm):
    assert set(declared_functions()) <= set(skm._SIGS)


def test_struct_layouts(skm):
    assert skm.STORED_DTYPE.itemsize == 10      # StoredKmerData, kmer_data.h:114-128
    assert skm.CALL_DTYPE.itemsize == 24        # KmerCall, call_functions.h:23-48
    assert C.sizeof(skm._AnnotOpts) == 24


def test_version_and_errors(skm):
    lib = skm.lib()
    assert "gfx950" in lib.skm_version().decode()
    # argument errors are reported, not thrown, and set skm_last_error
    rc = lib.skm_build_create(None, None, 0, None)
    assert rc == -1
    assert len(lib.skm_last_error()) > 0


def test_device_count_without_gpu_is_graceful(skm):
    n = C.c_int(-1)
    rc = skm.lib().skm_device_count(C.byref(n))
    assert rc == 0 and n.value >= 0


def test_build_on_cpu_only_host_fails_loudly(skm):
    if skm.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(skm.SkmError):
        skm.SignatureBuilder(4, device=0)


def test_comm_stub_reports_comm_error(skm):
    buf = (C.c_uint8 * 128)()
    rc = skm.lib().skm_comm_unique_id(buf)
    assert rc in (0, -5)
