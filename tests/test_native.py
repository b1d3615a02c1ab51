"""libttga.so boundary tests that need no GPU: the library loads, exports every
symbol include/ttga.h declares, and fails loudly (never silently on the CPU)."""
import ctypes
import pathlib
import re

import numpy as np
import pytest

from ttga import native

REPO = pathlib.Path(__file__).resolve().parent.parent
HEADER = REPO / "include" / "ttga.h"


def header_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(tt_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_exports():
    assert set(header_symbols()) == set(native.EXPORTS)


def test_library_exports_every_header_symbol():
    lib = native.load()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert lib.tt_version() >= 1


def test_null_arguments_rejected_without_device():
    lib = native.load()
    out = ctypes.c_void_p()
    assert lib.tt_problem_create(0, 1, 0, 0, None, None, None, None, 0, ctypes.byref(out)) == native.TT_ERR_INVALID
    assert b"dimensions" in lib.tt_last_error()
    assert lib.tt_eval(None, None, None, 1, None, None, None, None, None) == native.TT_ERR_INVALID
    assert lib.tt_problem_destroy(None) == native.TT_OK


def test_non_binary_matrix_rejected():
    lib = native.load()
    rs = np.array([10], np.int32)
    A = np.array([[2, 0]], np.int32)
    out = ctypes.c_void_p()
    rc = lib.tt_problem_create(2, 1, 0, 1, rs.ctypes.data, A.ctypes.data, None, None, 0, ctypes.byref(out))
    assert rc == native.TT_ERR_INVALID


def test_too_many_rooms_is_a_limit_error():
    lib = native.load()
    rs = np.full(65, 10, np.int32)
    A = np.zeros((1, 2), np.int32)
    out = ctypes.c_void_p()
    rc = lib.tt_problem_create(2, 65, 0, 1, rs.ctypes.data, A.ctypes.data, None, None, 0, ctypes.byref(out))
    assert rc == native.TT_ERR_LIMIT


def test_native_driver_cli_errors_without_device():
    """ttga-ga parses its command line as Control::Control (Control.cpp:7-39)
    before touching a device: odd argument counts and a missing -i exit 1."""
    import subprocess
    exe = REPO / "timetabling-ga-mpi-openmp_amd" / "ttga-ga"
    assert exe.exists(), "ttga-ga not built (make -C timetabling-ga-mpi-openmp_amd)"
    r = subprocess.run([str(exe), "-s"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Parse error: Number of command line parameters incorrect" in r.stderr
    r = subprocess.run([str(exe), "-s", "5", "-c", "4"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Error: No input file given, exiting" in r.stderr
    assert "Max number of threads 4" in r.stdout
