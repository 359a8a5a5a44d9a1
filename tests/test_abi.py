"""The drop-in boundary: the C-ABI library loads on a machine without a GPU and exports every
entry point include/*.h declares (no compute calls here — those are the -m gpu tests)."""
import ctypes
import os
import re
import subprocess

import pytest

from tests.conftest import ROOT
from tigerbeetle_amd import _lib, types


def declared_functions():
    names = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names |= set(re.findall(r"\b(tbgpu_\w+)\s*\(", text))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    from tigerbeetle_amd import build
    build.build(verbose=False)
    return _lib.load()


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("tbgpu_init", "tbgpu_deinit", "tbgpu_reset", "tbgpu_commit", "tbgpu_commit_many",
                     "tbgpu_commit_device_async", "tbgpu_sync", "tbgpu_commit_timestamp",
                     "tbgpu_test_set_balances", "tbgpu_export_accounts", "tbgpu_export_transfers"):
        assert required in names


def test_library_exports_every_declared_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name
    # ... and the ctypes signature table covers them all.
    assert {n for n, _, _ in _lib.SIGNATURES} == set(declared_functions())


def test_exports_are_plain_c_symbols(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\b(tbgpu_\w+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported  # unmangled extern "C"


def test_home_function_is_host_side(lib):
    # tbgpu_home needs no device: the router and the tests compute homes on the host.
    homes = [lib.tbgpu_home(i, 0, 8) for i in range(1, 2001)]
    assert set(homes) == set(range(8))
    assert all(lib.tbgpu_home(i, 0, 1) == 0 for i in range(1, 100))
    ids = (ctypes.c_uint64 * 4000)(*[v for i in range(1, 2001) for v in (i, 0)])
    out = (ctypes.c_uint32 * 2000)()
    lib.tbgpu_homes(ids, 2000, 8, out)
    assert list(out) == homes


def test_struct_layouts_match_reference():
    # src/tigerbeetle.zig:7-104 offsets.
    T = types.TRANSFER_DTYPE
    assert T.fields["amount_lo"][1] == 48 and T.fields["pending_id_lo"][1] == 64
    assert T.fields["timeout"][1] == 108 and T.fields["ledger"][1] == 112
    assert T.fields["code"][1] == 116 and T.fields["flags"][1] == 118 and T.fields["timestamp"][1] == 120
    A = types.ACCOUNT_DTYPE
    assert A.fields["credits_posted_lo"][1] == 64 and A.fields["reserved"][1] == 108
    assert A.fields["flags"][1] == 118 and A.fields["timestamp"][1] == 120


def test_init_without_gpu_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    cfg = _lib.tbgpu_config(1024, 1024, 8192, 16, 0, 0)
    h = ctypes.c_void_p()
    st = lib.tbgpu_init(ctypes.byref(cfg), ctypes.byref(h))
    assert st != _lib.STATUS_OK and not h.value
    assert lib.tbgpu_last_error()


def test_init_refuses_capacities_past_the_engine_limits(lib):
    """Capacity contract: a device holds at most 2^31 accounts and 2^31 transfer-log
    positions (31-bit positions in the 8-B index entries).  init refuses more with INVALID before it
    touches any device, so this runs without a GPU."""
    h = ctypes.c_void_p()
    for accounts, transfers in (((1 << 31) + 1, 1024), (1024, (1 << 31) + 1), (0, 1024), (1024, 0)):
        cfg = _lib.tbgpu_config(accounts, transfers, 8192, 1, 0, 0)
        assert lib.tbgpu_init(ctypes.byref(cfg), ctypes.byref(h)) == _lib.STATUS_INVALID
        assert not h.value
        if accounts and transfers:
            assert b"2^31" in lib.tbgpu_last_error()
