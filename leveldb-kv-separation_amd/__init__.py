"""MI355X batched CRC32C engine for ArcueidType/LevelDB-KV-Separation.

Host-side mirror of the reference's checksum interface (util/crc32c.h:17-38)
over the C-ABI in include/lvkv_crc32c.h, plus the batched device API that the
SST writer/reader (table/table_builder.cc:199-203, table/format.cc:92-99) and
WAL writer/reader (db/log_writer.cc:94-95, db/log_reader.cc:243-257) checksum
paths map onto.

The package directory name contains dashes, so import it through
``load()`` (or ``importlib``); it registers itself as
``leveldb_kv_separation_amd``. Every call goes to the native library
``liblvkv_crc32c.so``; if it is missing, importing fails loudly — there is no
Python or CPU fallback for the batch (GPU) path.
"""
from __future__ import annotations

import ctypes
from pathlib import Path
from typing import Optional, Tuple

__all__ = [
    "Extend", "Value", "Mask", "Unmask", "kMaskDelta",
    "crc32c_batch", "crc32c_uniform", "sst_verify", "log_verify",
    "crc32c_batch_host", "LvkvError", "lib", "LIB_PATH", "device_groups", "Engine",
]

LIB_PATH = Path(__file__).resolve().parent / "liblvkv_crc32c.so"
kMaskDelta = 0xA282EAD8  # util/crc32c.h:22

LVKV_OK = 0
LVKV_ERR_INVALID = -1
LVKV_FLAG_MASK = 1
LVKV_FLAG_ORDERED = 2
LVKV_FLAG_SYSTEM_ACQUIRE = 4
LVKV_FLAG_FINAL = 8
LVKV_FLAG_SMALL_BLOCKS = 16


class LvkvError(RuntimeError):
    """A C-ABI call returned a negative code (see lvkv_strerror)."""

    def __init__(self, fn: str, code: int):
        msg = _lib.lvkv_strerror(code).decode()
        if code in (-2, -3):
            msg += f" (hipError_t {_lib.lvkv_last_hip_error()})"
        super().__init__(f"{fn}: {msg} [{code}]")
        self.code = code


def _load() -> ctypes.CDLL:
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7.
    # Loading torch FIRST makes this library's NEEDED libamdhip64.so.7 bind to
    # that same (already loaded) runtime, so device pointers and streams are
    # shared. Loading this library first would map /opt/rocm's runtime and
    # torch would then map a second one (device enumeration then fails).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the GPU path has no fallback)")
    L = ctypes.CDLL(str(LIB_PATH))
    u32, u64, sz, vp, i32 = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t,
                             ctypes.c_void_p, ctypes.c_int)
    L.lvkv_crc32c_extend.argtypes = [u32, ctypes.c_char_p, sz]
    L.lvkv_crc32c_extend.restype = u32
    L.lvkv_crc32c_value.argtypes = [ctypes.c_char_p, sz]
    L.lvkv_crc32c_value.restype = u32
    L.lvkv_crc32c_mask.argtypes = [u32]
    L.lvkv_crc32c_mask.restype = u32
    L.lvkv_crc32c_unmask.argtypes = [u32]
    L.lvkv_crc32c_unmask.restype = u32
    L.lvkv_crc32c_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, sz, u32, vp]
    L.lvkv_crc32c_batch_device.restype = i32
    L.lvkv_crc32c_uniform_device.argtypes = [vp, u64, u32, u32, vp, sz, u32, vp]
    L.lvkv_crc32c_uniform_device.restype = i32
    L.lvkv_sst_verify_device.argtypes = [vp, vp, vp, vp, vp, sz, vp]
    L.lvkv_sst_verify_device.restype = i32
    L.lvkv_sst_verify_table_device.argtypes = [vp, u64, vp, vp, vp, vp, sz, ctypes.c_char_p,
                                               vp, vp]
    L.lvkv_sst_verify_table_device.restype = i32
    L.lvkv_sst_verify_tables_device.argtypes = [vp, vp, vp, sz, vp, vp, vp, vp, sz,
                                                ctypes.c_char_p, vp, vp]
    L.lvkv_sst_verify_tables_device.restype = i32
    L.lvkv_sst_fill_trailers_device.argtypes = [vp, vp, vp, vp, sz, vp]
    L.lvkv_sst_fill_trailers_device.restype = i32
    L.lvkv_log_fill_headers_device.argtypes = [vp, vp, vp, sz, vp]
    L.lvkv_log_fill_headers_device.restype = i32
    L.lvkv_log_verify_blocks_device.argtypes = [vp, u64, vp, vp, vp, sz, vp, vp, vp, vp]
    L.lvkv_log_verify_blocks_device.restype = i32
    L.lvkv_log_read_device.argtypes = [vp, u64, vp, vp, vp, sz, vp, vp, vp, vp, sz, vp, sz, u64,
                                       vp, vp]
    L.lvkv_log_read_device.restype = i32
    L.lvkv_log_gather_device.argtypes = [vp, vp, sz, vp, vp, sz, vp, vp, u64, vp, vp]
    L.lvkv_log_gather_device.restype = i32
    L.lvkv_debug_set_sst_form.argtypes = [i32]
    L.lvkv_debug_set_sst_form.restype = i32
    L.lvkv_log_verify_device.argtypes = [vp, vp, vp, vp, sz, vp]
    L.lvkv_log_verify_device.restype = i32
    L.lvkv_crc32c_batch_host.argtypes = [vp, vp, vp, vp, u32, vp, sz, u32]
    L.lvkv_crc32c_batch_host.restype = i32
    L.lvkv_engine_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.lvkv_engine_create.restype = i32
    L.lvkv_engine_destroy.argtypes = [vp]
    L.lvkv_engine_destroy.restype = None
    L.lvkv_engine_crc32c_uniform.argtypes = [vp, vp, u64, u32, u32, vp, sz, u32]
    L.lvkv_engine_crc32c_uniform.restype = i32
    L.lvkv_engine_crc32c_batch.argtypes = [vp, vp, vp, vp, vp, u32, vp, sz, u32]
    L.lvkv_engine_crc32c_batch.restype = i32
    L.lvkv_engine_sst_verify.argtypes = [vp, vp, vp, vp, vp, vp, sz, u32]
    L.lvkv_engine_sst_verify.restype = i32
    L.lvkv_engine_log_verify.argtypes = [vp, vp, vp, vp, vp, sz, u32]
    L.lvkv_engine_log_verify.restype = i32
    L.lvkv_engine_sst_fill_trailers.argtypes = [vp, vp, vp, vp, vp, sz, u32]
    L.lvkv_engine_sst_fill_trailers.restype = i32
    L.lvkv_engine_log_fill_headers.argtypes = [vp, vp, vp, vp, sz, u32]
    L.lvkv_engine_log_fill_headers.restype = i32
    L.lvkv_engine_wait.argtypes = [vp]
    L.lvkv_engine_wait.restype = i32
    L.lvkv_engine_queues.argtypes = [vp, i32]
    L.lvkv_engine_queues.restype = i32
    L.lvkv_engine_shape.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32),
                                    ctypes.POINTER(u32)]
    L.lvkv_engine_shape.restype = i32
    L.lvkv_debug_engine_kernarg_cache.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.lvkv_debug_engine_kernarg_cache.restype = i32
    L.lvkv_engine_profile.argtypes = [vp, i32]
    L.lvkv_engine_profile.restype = i32
    L.lvkv_engine_profile_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double), sz]
    L.lvkv_engine_profile_read.restype = ctypes.c_long
    L.lvkv_engine_load_probe.argtypes = [vp, ctypes.c_char_p, sz, ctypes.c_char_p, u32, u32,
                                         u32, i32]
    L.lvkv_engine_load_probe.restype = i32
    L.lvkv_debug_engine_stall.argtypes = [vp, i32, ctypes.c_double]
    L.lvkv_debug_engine_stall.restype = i32
    L.lvkv_snappy_max_compressed_length.argtypes = [sz]
    L.lvkv_snappy_max_compressed_length.restype = sz
    L.lvkv_snappy_compress_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, sz, u32, vp]
    L.lvkv_snappy_compress_device.restype = i32
    L.lvkv_snappy_uncompressed_length_device.argtypes = [vp, vp, vp, vp, vp, sz, vp]
    L.lvkv_snappy_uncompressed_length_device.restype = i32
    L.lvkv_snappy_uncompress_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, sz, u32, vp]
    L.lvkv_snappy_uncompress_device.restype = i32
    L.lvkv_zstd_uncompressed_length_device.argtypes = [vp, vp, vp, vp, vp, sz, vp]
    L.lvkv_zstd_uncompressed_length_device.restype = i32
    L.lvkv_zstd_uncompress_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, sz, u32, vp]
    L.lvkv_zstd_uncompress_device.restype = i32
    L.lvkv_debug_zstd_uncompress_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, u32,
                                                    vp]
    L.lvkv_debug_zstd_uncompress_device.restype = i32
    L.lvkv_sst_write_scratch_bytes.argtypes = [sz, u32]
    L.lvkv_sst_write_scratch_bytes.restype = sz
    L.lvkv_sst_write_blocks_device.argtypes = [vp, vp, vp, sz, i32, u32, vp, vp, u64, vp, vp, vp,
                                               vp, vp]
    L.lvkv_sst_write_blocks_device.restype = i32
    L.lvkv_sst_write_blocks_level_device.argtypes = [vp, vp, vp, sz, i32, i32, u32, vp, vp, u64,
                                                     vp, vp, vp, vp, vp]
    L.lvkv_sst_write_blocks_level_device.restype = i32
    L.lvkv_zstd_compress_bound.argtypes = [sz]
    L.lvkv_zstd_compress_bound.restype = sz
    L.lvkv_zstd_compress_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, sz, u32, i32, vp]
    L.lvkv_zstd_compress_device.restype = i32
    L.lvkv_sst_read_blocks_device.argtypes = [vp, vp, vp, sz, i32, vp, vp, vp, vp, vp, u32, vp]
    L.lvkv_sst_read_blocks_device.restype = i32
    L.lvkv_strerror.argtypes = [i32]
    L.lvkv_strerror.restype = ctypes.c_char_p
    L.lvkv_last_hip_error.argtypes = []
    L.lvkv_last_hip_error.restype = i32
    L.lvkv_cpu_impl.argtypes = []
    L.lvkv_cpu_impl.restype = ctypes.c_char_p
    L.lvkv_device_groups.argtypes = []
    L.lvkv_device_groups.restype = i32
    # Link-level drop-ins (C++ / Google ABI) — resolved to check they exist.
    L.crc32c_extend.argtypes = [u32, ctypes.c_char_p, sz]
    L.crc32c_extend.restype = u32
    L.crc32c_value.argtypes = [ctypes.c_char_p, sz]
    L.crc32c_value.restype = u32
    return L


_lib = _load()
lib = _lib


def _check(fn: str, rc: int) -> None:
    if rc != LVKV_OK:
        raise LvkvError(fn, rc)


# --------------------------------------------------------------------------
# util/crc32c.h mirror (per call, host)


def _as_bytes(data) -> bytes:
    if isinstance(data, (bytes, bytearray)):
        return bytes(data)
    if isinstance(data, str):
        return data.encode()
    return memoryview(data).tobytes()


def Extend(init_crc: int, data, n: Optional[int] = None) -> int:
    """leveldb::crc32c::Extend (util/crc32c.h:17): crc32c of A||data given
    init_crc = crc32c(A)."""
    b = _as_bytes(data)
    if n is None:
        n = len(b)
    if n > len(b):
        raise ValueError("n exceeds data length")
    return int(_lib.lvkv_crc32c_extend(init_crc & 0xFFFFFFFF, b, n))


def Value(data, n: Optional[int] = None) -> int:
    """leveldb::crc32c::Value (util/crc32c.h:20)."""
    return Extend(0, data, n)


def Mask(crc: int) -> int:
    """leveldb::crc32c::Mask (util/crc32c.h:29-32)."""
    return int(_lib.lvkv_crc32c_mask(crc & 0xFFFFFFFF))


def Unmask(masked_crc: int) -> int:
    """leveldb::crc32c::Unmask (util/crc32c.h:35-38)."""
    return int(_lib.lvkv_crc32c_unmask(masked_crc & 0xFFFFFFFF))


def cpu_impl() -> str:
    return _lib.lvkv_cpu_impl().decode()


def device_groups() -> int:
    g = int(_lib.lvkv_device_groups())
    _check("lvkv_device_groups", g if g < 0 else 0)
    return g


# --------------------------------------------------------------------------
# batched device API (torch tensors are only device-memory plumbing)


def _torch():
    import torch
    return torch


def _dev_ptr(t, name: str, dtype=None, numel: Optional[int] = None):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise TypeError(f"{name} must be a CUDA (HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype not in dtype:
        raise TypeError(f"{name} must have dtype in {dtype}, got {t.dtype}")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name} has {t.numel()} elements, need {numel}")
    return ctypes.c_void_p(t.data_ptr())


def _stream_handle(stream, device):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def _u32_out(torch, n, device, out):
    if out is None:
        return torch.empty(n, dtype=torch.int32, device=device)
    return out


def crc32c_batch(buf, offsets, lengths, *, init: int = 0, inits=None,
                 mask: bool = False, out=None, stream=None):
    """Batched Extend over block i = buf[offsets[i] : offsets[i]+lengths[i]].

    buf: uint8/int8 CUDA tensor; offsets: int64 CUDA tensor; lengths, inits:
    int32 CUDA tensors (bit patterns of u32). Returns an int32 tensor of CRC
    bit patterns (Mask()ed if mask=True)."""
    torch = _torch()
    n = offsets.numel()
    if lengths.numel() != n:
        raise ValueError("offsets and lengths differ in length")
    out = _u32_out(torch, n, buf.device, out)
    with torch.cuda.device(buf.device):
        rc = _lib.lvkv_crc32c_batch_device(
            _dev_ptr(buf, "buf", (torch.uint8, torch.int8)),
            _dev_ptr(offsets, "offsets", (torch.int64,)),
            _dev_ptr(lengths, "lengths", (torch.int32,)),
            _dev_ptr(inits, "inits", (torch.int32,), n) if inits is not None else None,
            init & 0xFFFFFFFF,
            _dev_ptr(out, "out", (torch.int32,), n), n,
            LVKV_FLAG_MASK if mask else 0, _stream_handle(stream, buf.device))
    _check("lvkv_crc32c_batch_device", rc)
    return out


def crc32c_uniform(buf, nblocks: int, length: int, stride: Optional[int] = None, *,
                   init: int = 0, mask: bool = False, out=None, stream=None):
    """Batched Extend over nblocks blocks of `length` bytes at buf + i*stride."""
    torch = _torch()
    stride = length if stride is None else stride
    if nblocks and (nblocks - 1) * stride + length > buf.numel():
        raise ValueError("blocks exceed the buffer")
    out = _u32_out(torch, nblocks, buf.device, out)
    with torch.cuda.device(buf.device):
        rc = _lib.lvkv_crc32c_uniform_device(
            _dev_ptr(buf, "buf", (torch.uint8, torch.int8)), stride, length,
            init & 0xFFFFFFFF, _dev_ptr(out, "out", (torch.int32,), nblocks),
            nblocks, LVKV_FLAG_MASK if mask else 0,
            _stream_handle(stream, buf.device))
    _check("lvkv_crc32c_uniform_device", rc)
    return out


def sst_verify(file_buf, offsets, sizes, *, stream=None) -> Tuple["object", "object"]:
    """Batched ReadBlock checksum test (table/format.cc:92-99) over the
    BlockHandles {offsets[i], sizes[i]} of an SST image. Returns (actual crc
    int32 tensor, status uint8 tensor: 0 ok / 1 'block checksum mismatch')."""
    torch = _torch()
    n = offsets.numel()
    actual = torch.empty(n, dtype=torch.int32, device=file_buf.device)
    status = torch.empty(n, dtype=torch.uint8, device=file_buf.device)
    with torch.cuda.device(file_buf.device):
        rc = _lib.lvkv_sst_verify_device(
            _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(offsets, "offsets", (torch.int64,)),
            _dev_ptr(sizes, "sizes", (torch.int32,), n),
            _dev_ptr(actual, "actual"), _dev_ptr(status, "status"), n,
            _stream_handle(stream, file_buf.device))
    _check("lvkv_sst_verify_device", rc)
    return actual, status


class SstReport(ctypes.Structure):
    """lvkv_sst_report (include/lvkv_crc32c.h)."""
    _fields_ = [("status", ctypes.c_int32), ("nblocks", ctypes.c_uint32),
                ("ndata", ctypes.c_uint32), ("has_filter", ctypes.c_uint32),
                ("nbad", ctypes.c_uint32), ("first_bad", ctypes.c_uint32),
                ("index_crc", ctypes.c_uint32), ("meta_crc", ctypes.c_uint32),
                ("index_status", ctypes.c_uint8), ("meta_status", ctypes.c_uint8),
                ("reserved0_", ctypes.c_uint8 * 2), ("first", ctypes.c_uint32),
                ("index_offset", ctypes.c_uint64), ("index_size", ctypes.c_uint64),
                ("meta_offset", ctypes.c_uint64), ("meta_size", ctypes.c_uint64),
                ("link_", ctypes.c_uint64), ("total_", ctypes.c_uint32),
                ("done_", ctypes.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_
                if not k.endswith("_")}


SST_STATUS = {0: "OK", 1: "file is too short to be an sstable",
              2: "not an sstable (bad magic number)", 3: "bad block handle",
              4: "truncated block read (index)", 5: "block checksum mismatch (index)",
              6: "index block type not readable here", 7: "bad index block contents",
              8: "capacity too small"}
BLOCK_STATUS = {0: "OK", 1: "block checksum mismatch", 2: "truncated block read",
                3: "bad block type", 4: "bad block handle", 5: "bad entry in block",
                6: "compressed block (no codec as built)", 7: "not read"}
# FilterPolicy::Name() of leveldb::NewBloomFilterPolicy (util/bloom.cc)
BLOOM_POLICY = "leveldb.BuiltinBloomFilter2"


def _policy(filter_policy):
    return None if filter_policy is None else filter_policy.encode()


def sst_verify_table(file_buf, *, capacity: Optional[int] = None,
                     filter_policy: Optional[str] = BLOOM_POLICY, stream=None):
    """Whole-SSTable verify on the device (lvkv_sst_verify_table_device):
    footer, index, metaindex, filter and every data block of the SST image
    in `file_buf` (uint8 CUDA tensor). filter_policy: the reader's
    FilterPolicy::Name() (None: no policy, no filter block). Returns (report
    dict, offsets int64, sizes int32, actual int32, status uint8) — the
    per-block tensors cut to report['nblocks'] entries (data blocks in index
    order, then the filter). With capacity=None a first guess is retried once
    at the index's size."""
    torch = _torch()
    dev = file_buf.device
    size = file_buf.numel()
    cap = capacity if capacity is not None else max(64, size // 2048 + 2)
    for attempt in range(2):
        off = torch.empty(cap, dtype=torch.int64, device=dev)
        sizes = torch.empty(cap, dtype=torch.int32, device=dev)
        actual = torch.empty(cap, dtype=torch.int32, device=dev)
        status = torch.empty(cap, dtype=torch.uint8, device=dev)
        rep = torch.zeros(ctypes.sizeof(SstReport), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            rc = _lib.lvkv_sst_verify_table_device(
                _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)), size,
                _dev_ptr(off, "offsets"), _dev_ptr(sizes, "sizes"), _dev_ptr(actual, "actual"),
                _dev_ptr(status, "status"), cap, _policy(filter_policy), _dev_ptr(rep, "report"),
                _stream_handle(stream, dev))
        _check("lvkv_sst_verify_table_device", rc)
        r = SstReport.from_buffer_copy(bytes(rep.cpu().numpy()))
        if r.status == 8 and capacity is None and attempt == 0:
            cap = r.ndata + 1
            continue
        break
    n = r.nblocks
    return r.as_dict(), off[:n], sizes[:n], actual[:n], status[:n]


def sst_verify_tables(file_buf, table_offsets, table_sizes, *, capacity=None,
                      filter_policy: Optional[str] = BLOOM_POLICY, stream=None):
    """Many SST images in one device buffer (lvkv_sst_verify_tables_device):
    two launches for all of them. Returns one (report dict, offsets, sizes,
    actual, status) per table as sst_verify_table would for that image alone,
    except that offsets are into file_buf. capacity (shared by all tables)
    defaults to file_buf.numel() // 2048 + 64 per table; a table that does
    not fit reports LVKV_SST_CAPACITY (8)."""
    torch = _torch()
    dev = file_buf.device
    T = len(table_offsets)
    toff = torch.tensor([int(x) for x in table_offsets], dtype=torch.int64, device=dev)
    tsz = torch.tensor([int(x) for x in table_sizes], dtype=torch.int64, device=dev)
    cap = capacity if capacity is not None else file_buf.numel() // 2048 + 64 * T
    o = torch.empty(cap, dtype=torch.int64, device=dev)
    sz = torch.empty(cap, dtype=torch.int32, device=dev)
    act = torch.empty(cap, dtype=torch.int32, device=dev)
    st = torch.empty(cap, dtype=torch.uint8, device=dev)
    rsz = ctypes.sizeof(SstReport)
    reps = torch.zeros(T * rsz, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.lvkv_sst_verify_tables_device(
            _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)), _dev_ptr(toff, "toff"),
            _dev_ptr(tsz, "tsize"), T, _dev_ptr(o, "offsets"), _dev_ptr(sz, "sizes"),
            _dev_ptr(act, "actual"), _dev_ptr(st, "status"), cap, _policy(filter_policy),
            _dev_ptr(reps, "reports"), _stream_handle(stream, dev))
    _check("lvkv_sst_verify_tables_device", rc)
    host = bytes(reps.cpu().numpy())
    out = []
    for t in range(T):
        r = SstReport.from_buffer_copy(host[t * rsz:(t + 1) * rsz])
        f, n = r.first, r.nblocks
        out.append((r.as_dict(), o[f:f + n], sz[f:f + n], act[f:f + n], st[f:f + n]))
    return out


def log_verify(file_buf, hdr_offsets, *, stream=None):
    """Batched ReadPhysicalRecord checksum test (db/log_reader.cc:243-257)
    over physical records whose 7-byte headers start at hdr_offsets[i]."""
    torch = _torch()
    n = hdr_offsets.numel()
    actual = torch.empty(n, dtype=torch.int32, device=file_buf.device)
    status = torch.empty(n, dtype=torch.uint8, device=file_buf.device)
    with torch.cuda.device(file_buf.device):
        rc = _lib.lvkv_log_verify_device(
            _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(hdr_offsets, "hdr_offsets", (torch.int64,)),
            _dev_ptr(actual, "actual"), _dev_ptr(status, "status"), n,
            _stream_handle(stream, file_buf.device))
    _check("lvkv_log_verify_device", rc)
    return actual, status


def sst_fill_trailers(file_buf, offsets, sizes, *, stream=None):
    """Batched TableBuilder::WriteRawBlock checksum (table_builder.cc:192-209):
    for each block handle (offsets int64, sizes int32 CUDA tensors) whose type
    byte is already in file_buf, writes Mask(CRC32C(contents + type)) into
    the trailer in place. Returns the unmasked CRCs (int32 tensor)."""
    torch = _torch()
    n = offsets.numel()
    crc = torch.empty(n, dtype=torch.int32, device=file_buf.device)
    with torch.cuda.device(file_buf.device):
        rc = _lib.lvkv_sst_fill_trailers_device(
            _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(offsets, "offsets", (torch.int64,)),
            _dev_ptr(sizes, "sizes", (torch.int32,), n), _dev_ptr(crc, "crc"), n,
            _stream_handle(stream, file_buf.device))
    _check("lvkv_sst_fill_trailers_device", rc)
    return crc


def log_fill_headers(file_buf, hdr_offsets, *, stream=None):
    """Batched log::Writer::EmitPhysicalRecord checksum (log_writer.cc:82-108):
    fills header bytes 0..3 of every record in place. Returns the unmasked
    CRCs (int32 tensor)."""
    torch = _torch()
    n = hdr_offsets.numel()
    crc = torch.empty(n, dtype=torch.int32, device=file_buf.device)
    with torch.cuda.device(file_buf.device):
        rc = _lib.lvkv_log_fill_headers_device(
            _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(hdr_offsets, "hdr_offsets", (torch.int64,)), _dev_ptr(crc, "crc"), n,
            _stream_handle(stream, file_buf.device))
    _check("lvkv_log_fill_headers_device", rc)
    return crc


# --------------------------------------------------------------------------
# Snappy block codec (include/lvkv_snappy.h; port/port_stdcxx.h:90-133)

SNAPPY_OK, SNAPPY_BAD_LENGTH, SNAPPY_BAD_CONTENTS, SNAPPY_CAPACITY, SNAPPY_TOO_LARGE = range(5)
SNAPPY_MAX_BLOCK = 49152


def snappy_max_compressed_length(n: int) -> int:
    """snappy::MaxCompressedLength (32 + n + n/6)."""
    return int(_lib.lvkv_snappy_max_compressed_length(n))


def _packed_offsets(torch, sizes, device):
    """Exclusive prefix sum of sizes (int64, on device)."""
    off = torch.zeros(sizes.numel(), dtype=torch.int64, device=device)
    if sizes.numel() > 1:
        off[1:] = torch.cumsum(sizes[:-1].to(torch.int64), 0)
    return off


def snappy_compress(src, offsets, lengths, *, max_len: Optional[int] = None, dst=None,
                    dst_offsets=None, stream=None):
    """Batched port::Snappy_Compress (port/port_stdcxx.h:90-106) of block
    i = src[offsets[i] : offsets[i] + lengths[i]]: snappy 1.1.8's bytes.

    Without dst, every block gets MaxCompressedLength bytes, packed. Returns
    (dst uint8, dst_offsets int64, compressed lengths int32, status uint8:
    SNAPPY_OK or SNAPPY_TOO_LARGE for a block longer than max_len)."""
    torch = _torch()
    n = offsets.numel()
    dev = src.device
    if lengths.numel() != n:
        raise ValueError("offsets and lengths differ in length")
    if max_len is None:
        max_len = int(lengths.max().item()) if n else 0
    if dst is None:
        lens = lengths.to(torch.int64)
        room = 32 + lens + lens // 6
        dst_offsets = _packed_offsets(torch, room, dev)
        dst = torch.empty(int(room.sum().item()) if n else 0, dtype=torch.uint8, device=dev)
    elif dst_offsets is None:
        raise ValueError("dst needs dst_offsets")
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    if n:
        with torch.cuda.device(dev):
            rc = _lib.lvkv_snappy_compress_device(
                _dev_ptr(src, "src", (torch.uint8, torch.int8)),
                _dev_ptr(offsets, "offsets", (torch.int64,)),
                _dev_ptr(lengths, "lengths", (torch.int32,)),
                _dev_ptr(dst, "dst", (torch.uint8, torch.int8)),
                _dev_ptr(dst_offsets, "dst_offsets", (torch.int64,), n),
                _dev_ptr(out_len, "out_len"), _dev_ptr(status, "status"), n,
                max(0, min(int(max_len), 0xFFFFFFFF)), _stream_handle(stream, dev))
        _check("lvkv_snappy_compress_device", rc)
    return dst, dst_offsets, out_len, status


def snappy_uncompressed_length(src, offsets, lengths, *, stream=None):
    """Batched port::Snappy_GetUncompressedLength (port/port_stdcxx.h:108-119).
    Returns (lengths int32 as u32 bit patterns, status uint8: SNAPPY_OK /
    SNAPPY_BAD_LENGTH)."""
    torch = _torch()
    n = offsets.numel()
    dev = src.device
    ulen = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    if n:
        with torch.cuda.device(dev):
            rc = _lib.lvkv_snappy_uncompressed_length_device(
                _dev_ptr(src, "src", (torch.uint8, torch.int8)),
                _dev_ptr(offsets, "offsets", (torch.int64,)),
                _dev_ptr(lengths, "lengths", (torch.int32,), n),
                _dev_ptr(ulen, "ulen"), _dev_ptr(status, "status"), n,
                _stream_handle(stream, dev))
        _check("lvkv_snappy_uncompressed_length_device", rc)
    return ulen, status


def snappy_uncompress(src, offsets, lengths, *, max_ulen: int, dst=None, dst_offsets=None,
                      dst_caps=None, stream=None):
    """Batched port::Snappy_Uncompress (port/port_stdcxx.h:121-133) as
    ReadBlock runs it (table/format.cc:120-135). Without dst, every stream
    gets max_ulen bytes. max_ulen sizes the LDS staging; a longer stream is
    decoded from HBM by the call's second kernel. Returns (dst uint8,
    dst_offsets int64, uncompressed lengths int32, status uint8: SNAPPY_OK /
    BAD_LENGTH / BAD_CONTENTS / CAPACITY)."""
    torch = _torch()
    n = offsets.numel()
    dev = src.device
    if not 0 <= max_ulen <= SNAPPY_MAX_BLOCK:
        raise ValueError(f"max_ulen must be in [0, {SNAPPY_MAX_BLOCK}]")
    if dst is None:
        dst_caps = torch.full((n,), max_ulen, dtype=torch.int32, device=dev)
        dst_offsets = torch.arange(n, dtype=torch.int64, device=dev) * max_ulen
        dst = torch.empty(max(1, n * max_ulen), dtype=torch.uint8, device=dev)
    elif dst_offsets is None or dst_caps is None:
        raise ValueError("dst needs dst_offsets and dst_caps")
    out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    if n:
        with torch.cuda.device(dev):
            rc = _lib.lvkv_snappy_uncompress_device(
                _dev_ptr(src, "src", (torch.uint8, torch.int8)),
                _dev_ptr(offsets, "offsets", (torch.int64,)),
                _dev_ptr(lengths, "lengths", (torch.int32,), n),
                _dev_ptr(dst, "dst", (torch.uint8, torch.int8)),
                _dev_ptr(dst_offsets, "dst_offsets", (torch.int64,), n),
                _dev_ptr(dst_caps, "dst_caps", (torch.int32,), n),
                _dev_ptr(out_len, "out_len"), _dev_ptr(status, "status"), n, max_ulen,
                _stream_handle(stream, dev))
        _check("lvkv_snappy_uncompress_device", rc)
    return dst, dst_offsets, out_len, status


ZSTD_OK, ZSTD_BAD_LENGTH, ZSTD_BAD_CONTENTS, ZSTD_CAPACITY, ZSTD_TOO_LARGE, \
    ZSTD_UNSUPPORTED = range(6)
ZSTD_MAX_BLOCK = 49152
ZSTD_COMPRESS_MAX_BLOCK = 20480


def zstd_compress_bound(n: int) -> int:
    """ZSTD_compressBound (libzstd 1.4.9)."""
    return int(_lib.lvkv_zstd_compress_bound(n))


def zstd_compress(src, offsets, lengths, *, level: int = 1, max_len: Optional[int] = None,
                  dst=None, dst_offsets=None, stream=None):
    """Batched port::Zstd_Compress(level, block) (port/port_stdcxx.h:133-161) of
    block i = src[offsets[i] : offsets[i] + lengths[i]]: libzstd 1.4.9's frame
    as ZSTD_compress2 writes it after getCParams(level, max(n, 1)) +
    setCParams. Without dst, every block gets ZSTD_compressBound bytes,
    packed. Returns (dst uint8, dst_offsets int64, frame lengths int32,
    status uint8: ZSTD_OK / ZSTD_TOO_LARGE / ZSTD_UNSUPPORTED)."""
    torch = _torch()
    n = offsets.numel()
    dev = src.device
    if lengths.numel() != n:
        raise ValueError("offsets and lengths differ in length")
    if max_len is None:
        max_len = int(lengths.max().item()) if n else 0
    # (max_len past ZSTD_COMPRESS_MAX_BLOCK: the C-ABI's LVKV_ERR_INVALID)
    if dst is None:
        lens = lengths.to(torch.int64)
        room = lens + (lens >> 8) + torch.clamp((131072 - lens) >> 11, min=0)
        dst_offsets = _packed_offsets(torch, room, dev)
        dst = torch.empty(max(1, int(room.sum().item())) if n else 1, dtype=torch.uint8,
                          device=dev)
    elif dst_offsets is None:
        raise ValueError("dst needs dst_offsets")
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    if n:
        with torch.cuda.device(dev):
            rc = _lib.lvkv_zstd_compress_device(
                _dev_ptr(src, "src", (torch.uint8, torch.int8)),
                _dev_ptr(offsets, "offsets", (torch.int64,)),
                _dev_ptr(lengths, "lengths", (torch.int32,)),
                _dev_ptr(dst, "dst", (torch.uint8, torch.int8)),
                _dev_ptr(dst_offsets, "dst_offsets", (torch.int64,), n),
                _dev_ptr(out_len, "out_len"), _dev_ptr(status, "status"), n, int(max_len),
                int(level), _stream_handle(stream, dev))
        _check("lvkv_zstd_compress_device", rc)
    return dst, dst_offsets, out_len, status


READ_OK, READ_CHECKSUM, READ_BAD_TYPE, READ_SNAPPY_LENGTH, READ_SNAPPY_CONTENTS, \
    READ_ZSTD_LENGTH, READ_CAPACITY, READ_TOO_LARGE, READ_ZSTD_CONTENTS = range(9)


def zstd_uncompressed_length(src, offsets, lengths, *, stream=None):
    """Batched port::Zstd_GetUncompressedLength (port/port_stdcxx.h:163-177):
    (lengths int32 as u32, status uint8: SNAPPY_OK / SNAPPY_BAD_LENGTH (0) /
    SNAPPY_TOO_LARGE (unknown, malformed, > 32 bits))."""
    torch = _torch()
    n = offsets.numel()
    dev = src.device
    ulen = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    if n:
        with torch.cuda.device(dev):
            rc = _lib.lvkv_zstd_uncompressed_length_device(
                _dev_ptr(src, "src", (torch.uint8, torch.int8)),
                _dev_ptr(offsets, "offsets", (torch.int64,)),
                _dev_ptr(lengths, "lengths", (torch.int32,), n),
                _dev_ptr(ulen, "ulen"), _dev_ptr(status, "status"), n,
                _stream_handle(stream, dev))
        _check("lvkv_zstd_uncompressed_length_device", rc)
    return ulen, status


def zstd_uncompress(src, offsets, lengths, *, max_ulen: int, dst=None, dst_offsets=None,
                    dst_caps=None, detail: bool = False, stream=None):
    """Batched port::Zstd_Uncompress (port/port_stdcxx.h:179-199) as ReadBlock
    runs it (table/format.cc:138-155). Statuses as snappy_uncompress. With
    detail=True also returns the failure site per stream (a debug hook)."""
    torch = _torch()
    n = offsets.numel()
    dev = src.device
    if not 0 <= max_ulen <= SNAPPY_MAX_BLOCK:
        raise ValueError(f"max_ulen must be in [0, {SNAPPY_MAX_BLOCK}]")
    if dst is None:
        dst_caps = torch.full((n,), max_ulen, dtype=torch.int32, device=dev)
        dst_offsets = torch.arange(n, dtype=torch.int64, device=dev) * max_ulen
        dst = torch.empty(max(1, n * max_ulen), dtype=torch.uint8, device=dev)
    elif dst_offsets is None or dst_caps is None:
        raise ValueError("dst needs dst_offsets and dst_caps")
    out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    why = torch.zeros(max(1, n), dtype=torch.int32, device=dev)
    if n:
        args = [_dev_ptr(src, "src", (torch.uint8, torch.int8)),
                _dev_ptr(offsets, "offsets", (torch.int64,)),
                _dev_ptr(lengths, "lengths", (torch.int32,), n),
                _dev_ptr(dst, "dst", (torch.uint8, torch.int8)),
                _dev_ptr(dst_offsets, "dst_offsets", (torch.int64,), n),
                _dev_ptr(dst_caps, "dst_caps", (torch.int32,), n),
                _dev_ptr(out_len, "out_len"), _dev_ptr(status, "status")]
        with torch.cuda.device(dev):
            if detail:
                rc = _lib.lvkv_debug_zstd_uncompress_device(*args, _dev_ptr(why, "detail"), n,
                                                            max_ulen, _stream_handle(stream, dev))
            else:
                rc = _lib.lvkv_zstd_uncompress_device(*args, n, max_ulen,
                                                      _stream_handle(stream, dev))
        _check("lvkv_zstd_uncompress_device", rc)
    if detail:
        return dst, dst_offsets, out_len, status, why
    return dst, dst_offsets, out_len, status


def sst_write_blocks(raw, offsets, lengths, *, compression: int = 1, max_len: Optional[int] = None,
                     file=None, file_offset: int = 0, zstd_level: int = 1, stream=None):
    """Batched TableBuilder::WriteBlock + WriteRawBlock (table/table_builder.cc:
    141-209): blocks raw[offsets[i] : offsets[i] + lengths[i]] written in order
    from file_offset of the file image `file` (allocated when None: file_offset
    + sum(lengths + 5) bytes). Returns (file, handle offsets int64, handle
    sizes int32, types uint8, end offset int64 tensor of one)."""
    torch = _torch()
    n = offsets.numel()
    dev = raw.device
    if max_len is None:
        max_len = int(lengths.max().item()) if n else 0
    if file is None:
        total = file_offset + (int(lengths.to(torch.int64).sum().item()) if n else 0) + 5 * n
        file = torch.zeros(max(1, total), dtype=torch.uint8, device=dev)
    hoff = torch.empty(n, dtype=torch.int64, device=dev)
    hsize = torch.empty(n, dtype=torch.int32, device=dev)
    typ = torch.empty(n, dtype=torch.uint8, device=dev)
    end = torch.empty(1, dtype=torch.int64, device=dev)
    scratch = None
    if compression in (1, 2) and n:
        scratch = torch.empty(int(_lib.lvkv_sst_write_scratch_bytes(n, max_len)),
                              dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.lvkv_sst_write_blocks_level_device(
            _dev_ptr(raw, "raw", (torch.uint8, torch.int8)) if n else None,
            _dev_ptr(offsets, "offsets", (torch.int64,)) if n else None,
            _dev_ptr(lengths, "lengths", (torch.int32,), n) if n else None, n, compression,
            int(zstd_level), max_len, _dev_ptr(scratch, "scratch") if scratch is not None else None,
            _dev_ptr(file, "file", (torch.uint8, torch.int8)), file_offset,
            _dev_ptr(hoff, "hoff") if n else None, _dev_ptr(hsize, "hsize") if n else None,
            _dev_ptr(typ, "type") if n else None, _dev_ptr(end, "end"),
            _stream_handle(stream, dev))
    _check("lvkv_sst_write_blocks_level_device", rc)
    return file, hoff, hsize, typ, end


def sst_read_blocks(file, handle_off, handle_size, *, max_ulen: int, verify: bool = True,
                    out=None, out_offsets=None, out_caps=None, stream=None):
    """Batched ReadBlock (table/format.cc:69-162): checksum, then contents by
    type (raw copied, snappy decoded). Without out, each block gets max_ulen
    bytes. Returns (out uint8, out_offsets int64, lengths int32, status uint8
    READ_*)."""
    torch = _torch()
    n = handle_off.numel()
    dev = file.device
    if not 0 <= max_ulen <= SNAPPY_MAX_BLOCK:
        raise ValueError(f"max_ulen must be in [0, {SNAPPY_MAX_BLOCK}]")
    if out is None:
        out_caps = torch.full((n,), max_ulen, dtype=torch.int32, device=dev)
        out_offsets = torch.arange(n, dtype=torch.int64, device=dev) * max_ulen
        out = torch.empty(max(1, n * max_ulen), dtype=torch.uint8, device=dev)
    elif out_offsets is None or out_caps is None:
        raise ValueError("out needs out_offsets and out_caps")
    out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    if n:
        with torch.cuda.device(dev):
            rc = _lib.lvkv_sst_read_blocks_device(
                _dev_ptr(file, "file", (torch.uint8, torch.int8)),
                _dev_ptr(handle_off, "handle_off", (torch.int64,)),
                _dev_ptr(handle_size, "handle_size", (torch.int32,), n), n, 1 if verify else 0,
                _dev_ptr(out, "out", (torch.uint8, torch.int8)),
                _dev_ptr(out_offsets, "out_offsets", (torch.int64,), n),
                _dev_ptr(out_caps, "out_caps", (torch.int32,), n),
                _dev_ptr(out_len, "out_len"), _dev_ptr(status, "status"), max_ulen,
                _stream_handle(stream, dev))
        _check("lvkv_sst_read_blocks_device", rc)
    return out, out_offsets, out_len, status


class LogReport(ctypes.Structure):
    """lvkv_log_report (include/lvkv_crc32c.h)."""
    _fields_ = [("status", ctypes.c_int32), ("nblocks", ctypes.c_uint32),
                ("nrecords", ctypes.c_uint32), ("ngood", ctypes.c_uint32),
                ("ncorrupt", ctypes.c_uint32), ("first_bad_block", ctypes.c_uint32),
                ("dropped_bytes", ctypes.c_uint64), ("count_", ctypes.c_uint32),
                ("reserved_", ctypes.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.endswith("_")}


def log_verify_blocks(file_buf, *, capacity: Optional[int] = None, stream=None):
    """Every physical record of the log image in `file_buf` (uint8 CUDA
    tensor), walked and verified on the device (lvkv_log_verify_blocks_device).
    Returns (report dict, hdr_offsets int64, actual int32, rec_status uint8 —
    cut to report['nrecords'] — block_status uint8, block_drop int32)."""
    torch = _torch()
    dev = file_buf.device
    size = file_buf.numel()
    nblocks = (size + 32767) // 32768
    cap = capacity if capacity is not None else max(64, size // 256)
    for attempt in range(2):
        hdr = torch.empty(cap, dtype=torch.int64, device=dev)
        actual = torch.empty(cap, dtype=torch.int32, device=dev)
        rst = torch.empty(cap, dtype=torch.uint8, device=dev)
        bst = torch.empty(max(1, nblocks), dtype=torch.uint8, device=dev)
        bdrop = torch.empty(max(1, nblocks), dtype=torch.int32, device=dev)
        rep = torch.zeros(ctypes.sizeof(LogReport), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            rc = _lib.lvkv_log_verify_blocks_device(
                _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)), size,
                _dev_ptr(hdr, "hdr"), _dev_ptr(actual, "actual"), _dev_ptr(rst, "rec_status"),
                cap, _dev_ptr(bst, "block_status"), _dev_ptr(bdrop, "block_drop"),
                _dev_ptr(rep, "report"), _stream_handle(stream, dev))
        _check("lvkv_log_verify_blocks_device", rc)
        r = LogReport.from_buffer_copy(bytes(rep.cpu().numpy()))
        if r.status == 1 and capacity is None and attempt == 0:
            cap = r.nrecords
            continue
        break
    n = r.nrecords if r.status == 0 else 0
    return r.as_dict(), hdr[:n], actual[:n], rst[:n], bst[:nblocks], bdrop[:nblocks]


class LogReadReport(ctypes.Structure):
    """lvkv_log_read_report (include/lvkv_crc32c.h)."""
    _fields_ = [("status", ctypes.c_int32), ("nrecords", ctypes.c_uint32),
                ("nreports", ctypes.c_uint32), ("stopped", ctypes.c_uint32),
                ("bytes", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


# Reporter::Corruption reasons (LVKV_LOGR_*) as the reference words them
# (db/log_reader.cc); an unknown type carries its number.
LOG_REASONS = {1: "checksum mismatch", 2: "bad record length",
               3: "partial record without end(1)", 4: "partial record without end(2)",
               5: "missing start of fragmented record(1)",
               6: "missing start of fragmented record(2)", 7: "error in middle of record",
               8: "unknown record type {}"}


def log_read(file_buf, *, initial_offset: int = 0, capacity: Optional[int] = None,
             record_capacity: Optional[int] = None, report_capacity: Optional[int] = None,
             gather: bool = False, stream=None):
    """log::Reader(reporter, checksum=True, initial_offset) over the log image
    in `file_buf` (uint8 CUDA tensor), all on the device
    (lvkv_log_read_device): ReadRecord until it returns false.

    Returns (read report dict, records, reports, physical):
      records  list of (LastRecordOffset, length, first fragment, fragments)
      reports  list of (bytes, reason text) — every Reporter::Corruption call
      physical the log_verify_blocks tuple of the same call
    With gather=True a fifth element: (payload, positions), the records'
    bytes as lvkv_log_gather_device lays them end to end on the device
    (uint8 tensor) and each record's offset in it (int64 tensor).
    Capacities default to sizes that always fit; a LVKV_LOG_CAPACITY result
    from smaller ones is returned as is."""
    import numpy as np
    if initial_offset < 0:
        raise ValueError("initial_offset must be >= 0")
    torch = _torch()
    dev = file_buf.device
    size = file_buf.numel()
    nblocks = (size + 32767) // 32768
    cap = capacity if capacity is not None else max(64, size // 7 + nblocks)
    rcap = record_capacity if record_capacity is not None else cap
    pcap = report_capacity if report_capacity is not None else cap + nblocks
    hdr = torch.empty(cap, dtype=torch.int64, device=dev)
    actual = torch.empty(cap, dtype=torch.int32, device=dev)
    rst = torch.empty(cap, dtype=torch.uint8, device=dev)
    bst = torch.empty(max(1, nblocks), dtype=torch.uint8, device=dev)
    bdrop = torch.empty(max(1, nblocks), dtype=torch.int32, device=dev)
    rep = torch.zeros(ctypes.sizeof(LogReport), dtype=torch.uint8, device=dev)
    recs = torch.zeros(max(1, rcap) * 24, dtype=torch.uint8, device=dev)
    reps = torch.zeros(max(1, pcap) * 16, dtype=torch.uint8, device=dev)
    rd = torch.zeros(ctypes.sizeof(LogReadReport), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.lvkv_log_read_device(
            _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)), size,
            _dev_ptr(hdr, "hdr"), _dev_ptr(actual, "actual"), _dev_ptr(rst, "rec_status"), cap,
            _dev_ptr(bst, "block_status"), _dev_ptr(bdrop, "block_drop"), _dev_ptr(rep, "report"),
            _dev_ptr(recs, "records"), rcap, _dev_ptr(reps, "reports"), pcap,
            int(initial_offset), _dev_ptr(rd, "read"), _stream_handle(stream, dev))
    _check("lvkv_log_read_device", rc)
    if gather:
        payload = torch.empty(max(1, size), dtype=torch.uint8, device=dev)
        pos = torch.zeros(max(1, rcap), dtype=torch.int64, device=dev)
        with torch.cuda.device(dev):
            rc = _lib.lvkv_log_gather_device(
                _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)), _dev_ptr(hdr, "hdr"),
                cap, _dev_ptr(rep, "report"), _dev_ptr(recs, "records"), rcap,
                _dev_ptr(rd, "read"), _dev_ptr(payload, "payload"), payload.numel(),
                _dev_ptr(pos, "positions"), _stream_handle(stream, dev))
        _check("lvkv_log_gather_device", rc)
    r = LogReport.from_buffer_copy(bytes(rep.cpu().numpy()))
    o = LogReadReport.from_buffer_copy(bytes(rd.cpu().numpy()))
    nrec = min(o.nrecords, rcap)
    nrep = min(o.nreports, pcap)
    rv = recs.cpu().numpy()[: nrec * 24].view(np.uint64).reshape(-1, 3)
    records = [(int(x[0]), int(x[1]), int(x[2]) & 0xFFFFFFFF, int(x[2]) >> 32) for x in rv]
    pv = reps.cpu().numpy()[: nrep * 16].view(np.uint64).reshape(-1, 2)
    reports = []
    for x in pv:
        reason, typ = int(x[1]) & 0xFFFFFFFF, int(x[1]) >> 32
        text = LOG_REASONS.get(reason, "?")
        reports.append((int(x[0]), text.format(typ) if reason == 8 else text))
    n = r.nrecords if r.status == 0 else 0
    physical = (r.as_dict(), hdr[:n], actual[:n], rst[:n], bst[:nblocks], bdrop[:nblocks])
    if gather:
        return o.as_dict(), records, reports, physical, (payload, pos[:nrec])
    return o.as_dict(), records, reports, physical


def crc32c_batch_host(data, offsets, lengths, *, init: int = 0, inits=None,
                      mask: bool = False):
    """Host-resident batch: numpy uint8 buffer + numpy offsets/lengths; the
    library stages through pinned memory to the current device and back.
    Returns a numpy uint32 array."""
    import numpy as np
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = offsets.size
    if lengths.size != n:
        raise ValueError("offsets and lengths differ in length")
    if n and int((offsets + lengths).max()) > data.size:
        raise ValueError("blocks exceed the buffer")
    out = np.empty(n, dtype=np.uint32)
    ip = None
    if inits is not None:
        inits = np.ascontiguousarray(inits, dtype=np.uint32)
        ip = ctypes.c_void_p(inits.ctypes.data)
    rc = _lib.lvkv_crc32c_batch_host(
        ctypes.c_void_p(data.ctypes.data), ctypes.c_void_p(offsets.ctypes.data),
        ctypes.c_void_p(lengths.ctypes.data), ip, init & 0xFFFFFFFF,
        ctypes.c_void_p(out.ctypes.data), n, LVKV_FLAG_MASK if mask else 0)
    _check("lvkv_crc32c_batch_host", rc)
    return out


# --------------------------------------------------------------------------
# the AQL engine (lvkv_engine_*): batches dispatched into hardware queues


class Engine:
    """Per-device batch engine (include/lvkv_crc32c.h, lvkv_engine_*): a
    submit writes AQL dispatch packets into the engine's own hardware queues
    (no HIP launch), consecutive batches overlap on the device, ``wait()``
    fences every queue. Inputs must be complete before a submit (synchronize
    the stream that produced them); results are valid after ``wait()``.

    Same results as ``crc32c_uniform`` / ``crc32c_batch`` / ``sst_verify``
    / ``log_verify`` / the fill calls, for any block layout."""

    def __init__(self, device=None):
        torch = _torch()
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else
                           (device.index if isinstance(device, torch.device) else int(device)))
        h = ctypes.c_void_p()
        _check("lvkv_engine_create", _lib.lvkv_engine_create(dev.index, ctypes.byref(h)))
        self.device = dev
        self.handle = h
        # the raw entry, for callers that pass pointers themselves (bench.py)
        self.submit_ptr = _lib.lvkv_engine_crc32c_uniform
        # inputs and outputs of submitted batches, held until the wait() that
        # covers them: the engine reads and writes them outside any torch
        # stream, so the caching allocator must not hand their memory out
        self._inflight = []

    def crc32c_uniform(self, buf, nblocks: int, length: int, stride: Optional[int] = None, *,
                       init: int = 0, mask: bool = False, ordered: bool = False,
                       fresh: bool = True, final: bool = False, out=None):
        """fresh: the input may have been written by a copy engine or the host
        (LVKV_FLAG_SYSTEM_ACQUIRE); False when a kernel on this device wrote it.
        final: a wait follows (LVKV_FLAG_FINAL)."""
        torch = _torch()
        stride = length if stride is None else stride
        if nblocks and (nblocks - 1) * stride + length > buf.numel():
            raise ValueError("blocks exceed the buffer")
        out = _u32_out(torch, nblocks, buf.device, out)
        flags = self._flags(mask, ordered, fresh, final)
        # the engine does not follow HIP streams: the inputs must be complete
        torch.cuda.current_stream(buf.device).synchronize()
        rc = _lib.lvkv_engine_crc32c_uniform(
            self.handle, _dev_ptr(buf, "buf", (torch.uint8, torch.int8)), stride, length,
            init & 0xFFFFFFFF, _dev_ptr(out, "out", (torch.int32,), nblocks), nblocks, flags)
        _check("lvkv_engine_crc32c_uniform", rc)
        self._inflight.append((buf, out))
        return out

    def _flags(self, mask=False, ordered=False, fresh=True, final=False):
        return ((LVKV_FLAG_MASK if mask else 0) | (LVKV_FLAG_ORDERED if ordered else 0) |
                (LVKV_FLAG_SYSTEM_ACQUIRE if fresh else 0) | (LVKV_FLAG_FINAL if final else 0))

    def crc32c_batch(self, buf, offsets, lengths, *, init: int = 0, inits=None,
                     mask: bool = False, ordered: bool = False, fresh: bool = True,
                     final: bool = False, small: bool = False, out=None):
        """lvkv_engine_crc32c_batch: crc32c_batch's contract on the engine.
        small: the blocks are mostly under ~2 KiB (LVKV_FLAG_SMALL_BLOCKS)."""
        torch = _torch()
        n = offsets.numel()
        if lengths.numel() != n:
            raise ValueError("offsets and lengths differ in length")
        out = _u32_out(torch, n, buf.device, out)
        torch.cuda.current_stream(buf.device).synchronize()
        rc = _lib.lvkv_engine_crc32c_batch(
            self.handle, _dev_ptr(buf, "buf", (torch.uint8, torch.int8)),
            _dev_ptr(offsets, "offsets", (torch.int64,)),
            _dev_ptr(lengths, "lengths", (torch.int32,)),
            _dev_ptr(inits, "inits", (torch.int32,), n) if inits is not None else None,
            init & 0xFFFFFFFF, _dev_ptr(out, "out", (torch.int32,), n), n,
            self._flags(mask, ordered, fresh, final) | (LVKV_FLAG_SMALL_BLOCKS if small else 0))
        _check("lvkv_engine_crc32c_batch", rc)
        self._inflight.append((buf, offsets, lengths, inits, out))
        return out

    def sst_verify(self, file_buf, offsets, sizes, *, ordered=False, fresh=True, final=False):
        """lvkv_engine_sst_verify: (actual int32, status uint8) as sst_verify."""
        torch = _torch()
        n = offsets.numel()
        actual = torch.empty(n, dtype=torch.int32, device=file_buf.device)
        status = torch.empty(n, dtype=torch.uint8, device=file_buf.device)
        torch.cuda.current_stream(file_buf.device).synchronize()
        rc = _lib.lvkv_engine_sst_verify(
            self.handle, _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(offsets, "offsets", (torch.int64,)), _dev_ptr(sizes, "sizes", (torch.int32,), n),
            _dev_ptr(actual, "actual"), _dev_ptr(status, "status"), n,
            self._flags(False, ordered, fresh, final))
        _check("lvkv_engine_sst_verify", rc)
        self._inflight.append((file_buf, offsets, sizes, actual, status))
        return actual, status

    def log_verify(self, file_buf, hdr_offsets, *, ordered=False, fresh=True, final=False):
        """lvkv_engine_log_verify: (actual int32, status uint8) as log_verify."""
        torch = _torch()
        n = hdr_offsets.numel()
        actual = torch.empty(n, dtype=torch.int32, device=file_buf.device)
        status = torch.empty(n, dtype=torch.uint8, device=file_buf.device)
        torch.cuda.current_stream(file_buf.device).synchronize()
        rc = _lib.lvkv_engine_log_verify(
            self.handle, _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(hdr_offsets, "hdr_offsets", (torch.int64,)), _dev_ptr(actual, "actual"),
            _dev_ptr(status, "status"), n, self._flags(False, ordered, fresh, final))
        _check("lvkv_engine_log_verify", rc)
        self._inflight.append((file_buf, hdr_offsets, actual, status))
        return actual, status

    def sst_fill_trailers(self, file_buf, offsets, sizes, *, ordered=False, fresh=True, final=False):
        """lvkv_engine_sst_fill_trailers: sst_fill_trailers on the engine."""
        torch = _torch()
        n = offsets.numel()
        crc = torch.empty(n, dtype=torch.int32, device=file_buf.device)
        torch.cuda.current_stream(file_buf.device).synchronize()
        rc = _lib.lvkv_engine_sst_fill_trailers(
            self.handle, _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(offsets, "offsets", (torch.int64,)), _dev_ptr(sizes, "sizes", (torch.int32,), n),
            _dev_ptr(crc, "crc"), n, self._flags(False, ordered, fresh, final))
        _check("lvkv_engine_sst_fill_trailers", rc)
        self._inflight.append((file_buf, offsets, sizes, crc))
        return crc

    def log_fill_headers(self, file_buf, hdr_offsets, *, ordered=False, fresh=True, final=False):
        """lvkv_engine_log_fill_headers: log_fill_headers on the engine."""
        torch = _torch()
        n = hdr_offsets.numel()
        crc = torch.empty(n, dtype=torch.int32, device=file_buf.device)
        torch.cuda.current_stream(file_buf.device).synchronize()
        rc = _lib.lvkv_engine_log_fill_headers(
            self.handle, _dev_ptr(file_buf, "file_buf", (torch.uint8, torch.int8)),
            _dev_ptr(hdr_offsets, "hdr_offsets", (torch.int64,)), _dev_ptr(crc, "crc"), n,
            self._flags(False, ordered, fresh, final))
        _check("lvkv_engine_log_fill_headers", rc)
        self._inflight.append((file_buf, hdr_offsets, crc))
        return crc

    def wait(self) -> None:
        _check("lvkv_engine_wait", _lib.lvkv_engine_wait(self.handle))
        self._inflight.clear()

    def kernarg_cache(self) -> Tuple[int, int]:
        """(hits, misses) of the engine's kernel-argument cache."""
        h, m = ctypes.c_uint64(), ctypes.c_uint64()
        _check("lvkv_debug_engine_kernarg_cache",
               _lib.lvkv_debug_engine_kernarg_cache(self.handle, ctypes.byref(h), ctypes.byref(m)))
        return int(h.value), int(m.value)

    def queues(self, n: int = 0) -> int:
        r = int(_lib.lvkv_engine_queues(self.handle, n))
        _check("lvkv_engine_queues", r if r < 0 else 0)
        return r

    def shape(self):
        w, c, g = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check("lvkv_engine_shape", _lib.lvkv_engine_shape(self.handle, ctypes.byref(w),
                                                            ctypes.byref(c), ctypes.byref(g)))
        return w.value, c.value, g.value

    def profile(self, enable: bool) -> None:
        _check("lvkv_engine_profile", _lib.lvkv_engine_profile(self.handle, int(enable)))

    def profile_read(self, n: int = 4096):
        """[(start_us, end_us)] of the most recent profiled dispatches, in
        submission order (HSA system clock)."""
        t0, t1 = (ctypes.c_double * n)(), (ctypes.c_double * n)()
        k = int(_lib.lvkv_engine_profile_read(self.handle, t0, t1, n))
        _check("lvkv_engine_profile_read", k if k < 0 else 0)
        return list(zip(t0[:k], t1[:k]))

    def load_probe(self, code_object: Optional[bytes], kernel: str = "", waves: int = 8,
                   chains: int = 5, per_cu: int = 1, overlapped: bool = True) -> None:
        """Measurement only (lvkv_engine_load_probe): overlapped (or ordered)
        uniform submits dispatch `kernel` from a separate gfx950 code object
        instead of the engine's own; None restores them."""
        if code_object is None:
            rc = _lib.lvkv_engine_load_probe(self.handle, None, 0, None, 0, 0, 0, 0)
        else:
            rc = _lib.lvkv_engine_load_probe(self.handle, code_object, len(code_object),
                                             (kernel + ".kd").encode(), waves, chains, per_cu,
                                             int(overlapped))
        _check("lvkv_engine_load_probe", rc)

    def close(self) -> None:
        if self.handle:
            _lib.lvkv_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass
