"""In-tree build of liblvkv_crc32c.so (gfx950) and of the oracle checker.

Used by __graft_entry__.build() and tests/conftest.py. Plain subprocess calls
to hipcc / g++ / make — no cmake, no JIT cache outside the repo — so the built
.so files travel with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = REPO / "include"
BUILD = REPO / "build" / "lvkv"
LIB = PKG / "liblvkv_crc32c.so"
# The probe build: the same sources with -DLVKV_PROBE_BUILD (schedule
# variants, timestamp builds, read-bandwidth kernel; tools/probe/lvkv_probe.h).
PROBE_BUILD = REPO / "build" / "lvkv_probe"
PROBE_LIB = REPO / "tools" / "probe" / "liblvkv_probe.so"
ORACLE_DIR = REPO / "oracle"
ORACLE_LIB = ORACLE_DIR / "liboracle_crc32c.so"
REF_LIB = ORACLE_DIR / "_ref" / "libref_crc32c.so"
REFERENCE = Path("/root/reference")
# HBM read-ceiling kernels (bench.py roofline.ceiling; measurement only, not in
# the library): an unbundled code object the engine loads as a probe.
CEILING_SRC = REPO / "tools" / "probe" / "ceiling_kernels.hip"
CEILING_CO = REPO / "tools" / "probe" / "ceiling_kernels.co"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("LVKV_OFFLOAD_ARCH", "gfx950")

# Host-only C++ (no device code): built with g++.
HOST_SOURCES = ["lvkv_tables.cpp", "lvkv_cpu_crc32c.cpp", "leveldb_crc32c_shim.cc"]
# HIP sources: kernels and the runtime-facing C-ABI.
HIP_SOURCES = ["crc32c_kernel.hip", "crc32c_uniform.hip", "crc32c_compact.hip",
               "crc32c_ragged.hip", "lvkv_sst_table.hip", "lvkv_log_blocks.hip",
               "lvkv_log_assemble.hip", "lvkv_snappy.hip", "lvkv_zstd.hip",
               "lvkv_zstd_compress.hip", "lvkv_capi.cpp", "lvkv_engine.cpp"]
# Kernels of the AQL engine: compiled alone into a gfx950 code object that is
# embedded in the library (.incbin) and loaded through the HSA loader.
ENGINE_KERNELS = "lvkv_engine_kernels.hip"
HEADERS = ["lvkv_kernel_args.h", "lvkv_tables.h", "crc32c_device_common.h",
           "crc32c_uniform_common.h", "crc32c_compact_common.h", "crc32c_burst.h",
           "crc32c_ragged_body.h", "lvkv_log_events.h", "lvkv_zstd_tables.h"]


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True)


def _newer(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return False
    t = target.stat().st_mtime
    return all(d.stat().st_mtime <= t for d in deps)


def build_lib(verbose: bool = False, force: bool = False, probe: bool = False) -> Path:
    lib = PROBE_LIB if probe else LIB
    build = PROBE_BUILD if probe else BUILD
    deps = [CSRC / s for s in HOST_SOURCES + HIP_SOURCES + HEADERS + [ENGINE_KERNELS]]
    deps += sorted(INCLUDE.glob("*.h")) + [Path(__file__)]
    if not force and _newer(lib, deps):
        return lib
    build.mkdir(parents=True, exist_ok=True)
    objs, cmds = [], []
    common = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-I", INCLUDE, "-I", CSRC]
    if probe:
        common.append("-DLVKV_PROBE_BUILD")
    for src in HOST_SOURCES:
        obj = build / (Path(src).stem + ".o")
        cmds.append(["g++", *common, "-c", CSRC / src, "-o", obj])
        objs.append(obj)
    for src in HIP_SOURCES:
        obj = build / (Path(src).stem + ".hip.o")
        cmds.append([HIPCC, f"--offload-arch={ARCH}", *common, "-c", CSRC / src, "-o", obj])
        objs.append(obj)
    co = build / "lvkv_engine.co"
    cmds.append([HIPCC, f"--offload-arch={ARCH}", *common, "--cuda-device-only",
                 "--no-gpu-bundle-output", "-c", CSRC / ENGINE_KERNELS, "-o", co])
    # translation units are independent: compile them concurrently
    with ThreadPoolExecutor(max_workers=min(len(cmds), os.cpu_count() or 1, 8)) as ex:
        list(ex.map(lambda c: _run(c, verbose), cmds))
    asm = build / "lvkv_engine_co.S"
    asm.write_text(
        "\t.section .rodata\n\t.balign 4096\n\t.globl lvkv_engine_co\n"
        "\t.type lvkv_engine_co, @object\nlvkv_engine_co:\n"
        f"\t.incbin \"{co}\"\n\t.globl lvkv_engine_co_end\nlvkv_engine_co_end:\n"
        "\t.section .note.GNU-stack,\"\",@progbits\n")
    co_obj = build / "lvkv_engine_co.o"
    _run(["gcc", "-c", asm, "-o", co_obj], verbose)
    objs.append(co_obj)
    tmp = lib.with_suffix(".so.tmp")
    # the probe library binds its own symbols (it may be loaded next to the
    # product library in one process)
    extra = ["-Wl,-Bsymbolic"] if probe else []
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp, "-lpthread",
          "-L/opt/rocm/lib", "-lhsa-runtime64", *extra], verbose)
    os.replace(tmp, lib)
    return lib


def build_ceiling(verbose: bool = False, force: bool = False) -> Path:
    deps = [CEILING_SRC, Path(__file__)] + [CSRC / h for h in HEADERS]
    if not force and _newer(CEILING_CO, deps):
        return CEILING_CO
    tmp = CEILING_CO.with_suffix(".co.tmp")
    _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "--cuda-device-only",
          "--no-gpu-bundle-output", "-I", INCLUDE, "-I", CSRC, "-c", CEILING_SRC, "-o", tmp],
         verbose)
    os.replace(tmp, CEILING_CO)
    return CEILING_CO


def build_oracle(verbose: bool = False) -> Path:
    """Build the C restatement (always) and the reference-backed checker
    oracle/_ref (only where /root/reference exists, i.e. this container)."""
    _run(["make", "-s", "-C", ORACLE_DIR, "all"], verbose)
    if REFERENCE.is_dir() and shutil.which("g++"):
        _run(["make", "-s", "-C", ORACLE_DIR, "ref", f"REF={REFERENCE}"], verbose)
    return ORACLE_LIB


def build_all(verbose: bool = False, force: bool = False) -> None:
    build_lib(verbose=verbose, force=force)
    build_lib(verbose=verbose, force=force, probe=True)
    build_ceiling(verbose=verbose, force=force)
    build_oracle(verbose=verbose)


if __name__ == "__main__":
    import sys

    build_all(verbose=True, force="--force" in sys.argv)
