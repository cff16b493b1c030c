"""The C-ABI library (CPU-side checks; no GPU compute).

* it loads and exports every function declared in include/*.h;
* the per-call drop-ins (leveldb::crc32c::Extend, Google crc32c_*) are
  bit-exact against the reference KATs and the oracle;
* without a device, the batch API reports LVKV_ERR_NO_DEVICE (no silent CPU
  fallback).
"""
from __future__ import annotations

import ctypes
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO


def _declared_functions():
    names = set()
    for h in sorted((REPO / "include").glob("*.h")):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*;", text):
            names.add(m.group(1))
    return names


def test_library_is_in_tree(lvkv):
    assert lvkv.LIB_PATH.parent == REPO / "leveldb-kv-separation_amd"
    assert lvkv.LIB_PATH.exists()


def test_exports_every_declared_symbol(lvkv):
    declared = _declared_functions()
    assert {"lvkv_crc32c_batch_device", "lvkv_crc32c_uniform_device", "lvkv_sst_verify_device",
            "lvkv_log_verify_device", "lvkv_crc32c_batch_host", "lvkv_crc32c_extend",
            "crc32c_extend", "crc32c_value", "lvkv_debug_tables"} <= declared
    out = subprocess.run(["nm", "-D", "--defined-only", str(lvkv.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = declared - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    # The C++ drop-ins: leveldb::crc32c::Extend (util/crc32c.h:17) and the
    # Google ::crc32c::Extend bound by port::AcceleratedCRC32C.
    assert "_ZN7leveldb6crc32c6ExtendEjPKcm" in exported
    assert "_ZN6crc32c6ExtendEjPKhm" in exported


def test_per_call_known_answers(lvkv, golden):
    for v in golden("kat.json")["vectors"]:
        data = bytes.fromhex(v["hex"])
        assert lvkv.Extend(v["init"], data) == v["crc"], v["name"]
        assert lvkv.Mask(v["crc"]) == v["masked"]
        assert lvkv.Unmask(v["masked"]) == v["crc"]
    assert lvkv.Value(b"TestCRCBuffer") == 0xDCBC59FA
    assert lvkv.kMaskDelta == golden("kat.json")["mask_delta"]


def test_per_call_matches_oracle_every_alignment(lvkv, oracle):
    rng = np.random.default_rng(3)
    buf = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
    for n in list(range(0, 70)) + [255, 256, 4095, 4096, 4105, 32762]:
        for a in range(8):
            init = int(rng.integers(0, 2**32))
            assert lvkv.Extend(init, buf[a:a + n]) == oracle.extend(init, buf[a:a + n])


def test_google_abi_and_cpp_symbol(lvkv):
    L = lvkv.lib
    assert L.crc32c_value(b"123456789", 9) == 0xE3069283
    assert L.crc32c_extend(L.crc32c_value(b"hello ", 6), b"world", 5) == lvkv.Value(b"hello world")
    f = getattr(L, "_ZN7leveldb6crc32c6ExtendEjPKcm")
    f.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    f.restype = ctypes.c_uint32
    assert f(0, b"TestCRCBuffer", 13) == 0xDCBC59FA


def test_portable_and_hw_paths_agree(lvkv, oracle, golden):
    # Both per-call implementations: the one picked for this CPU (the public
    # entry points) and the portable slicing-by-8 (debug export), against the
    # reference KATs and the oracle on every length 0..300 and alignment.
    assert lvkv.cpu_impl() in ("sse4.2", "portable-slice8")
    f = lvkv.lib.lvkv_debug_extend_portable
    f.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    f.restype = ctypes.c_uint32
    for v in golden("kat.json")["vectors"]:
        data = bytes.fromhex(v["hex"])
        assert f(v["init"], data, len(data)) == v["crc"], v["name"]
    rng = np.random.default_rng(8)
    buf = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    for n in list(range(0, 300)) + [4095, 4096, 4097, 32762, 65536]:
        for a in (0, 1, 3, 5):
            init = int(rng.integers(0, 2**32))
            want = oracle.extend(init, buf[a:a + n])
            assert f(init, buf[a:], n) == want
            assert lvkv.Extend(init, buf[a:a + n]) == want


def test_no_device_is_an_error_not_a_fallback(lvkv):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    out = np.zeros(4, dtype=np.uint32)
    buf = np.zeros(64, dtype=np.uint8)
    rc = lvkv.lib.lvkv_crc32c_uniform_device(ctypes.c_void_p(buf.ctypes.data), 16, 16, 0,
                                             ctypes.c_void_p(out.ctypes.data), 4, 0, None)
    assert rc == -2
    with pytest.raises(lvkv.LvkvError):
        lvkv.crc32c_batch_host(buf, np.array([0], np.uint64), np.array([16], np.uint32))


def test_empty_batch_is_ok_without_device(lvkv):
    rc = lvkv.lib.lvkv_crc32c_uniform_device(None, 0, 0, 0, None, 0, 0, None)
    assert rc == 0
    assert lvkv.lib.lvkv_crc32c_batch_device(None, None, None, None, 0, None, 0, 0, None) == 0


def test_invalid_arguments(lvkv):
    buf = np.zeros(16, np.uint8)
    rc = lvkv.lib.lvkv_crc32c_uniform_device(ctypes.c_void_p(buf.ctypes.data), 16, 16, 0,
                                             None, 1, 0, None)
    assert rc == -1


def test_package_calls_pass_every_declared_argument(lvkv):
    """ctypes does not count arguments (extra ones pass as varargs): every
    `_lib.<fn>(...)` call in the package passes exactly len(argtypes)."""
    import ast
    src = (REPO / "leveldb-kv-separation_amd" / "__init__.py").read_text()
    bad = []
    for node in ast.walk(ast.parse(src)):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute) and \
                isinstance(node.func.value, ast.Name) and node.func.value.id == "_lib":
            fn = getattr(lvkv.lib, node.func.attr)
            if fn.argtypes is not None and any(isinstance(a, ast.Starred) for a in node.args):
                continue
            if fn.argtypes is not None and len(node.args) != len(fn.argtypes):
                bad.append((node.func.attr, node.lineno, len(node.args), len(fn.argtypes)))
    assert not bad, bad
