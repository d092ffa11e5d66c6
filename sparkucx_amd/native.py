"""ctypes binding of libsparkucx_amd.so (include/sparkucx_amd.h).

This is plumbing for tests and bench.py: every call goes straight through the C-ABI into the
gfx950 kernels.  There is no CPU fallback — if the shared library is missing, importing
`load()` raises and the caller fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsparkucx_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "sparkucx_amd.h")

# status codes / constants (mirrors include/sparkucx_amd.h)
SUX_OK, SUX_EINVAL, SUX_ENOMEM, SUX_EHIP, SUX_ECOMM, SUX_ENOENT, SUX_ESTATE, SUX_ERANGE = (
    0, -1, -2, -3, -4, -5, -6, -7)
PART_RANGE_BYTES, PART_MURMUR3_LONG, PART_MURMUR3_INT, PART_MURMUR3_BYTES = 1, 2, 3, 4
PART_HASH_LONG, PART_HASH_INT = 5, 6
GEN_TERASORT, GEN_SMALL, GEN_ZIPF = 1, 2, 3
SORT_BYTES, SORT_LONG, SORT_INT = 1, 2, 3
SUX_EIO = -8
SUX_CODEC_NONE, SUX_CODEC_LZ4 = 0, 1
KERNELS = ("hist", "scan", "scatter", "copy")


class SuxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class Conf(C.Structure):
    _fields_ = [("device", C.c_int32), ("rank", C.c_int32), ("world_size", C.c_int32),
                ("num_streams", C.c_int32), ("comm_id", C.c_uint8 * 128),
                ("min_buffer_size", C.c_uint64), ("min_allocation_size", C.c_uint64),
                ("metadata_block_size", C.c_uint64), ("num_prealloc", C.c_uint32),
                ("pool_limit_mib", C.c_uint32), ("prealloc_size", C.c_uint64 * 16),
                ("prealloc_count", C.c_uint64 * 16)]


TUNING_FIELDS = ("hist_kernel", "scatter_kernel", "coresident", "scatter_chunk", "scatter_depth",
                 "hist_stage", "s6_chunk", "tiles_per_item", "small_groups", "tile_records",
                 "onepass", "varlen_kernel", "varlen_tile", "sort_max_digit_bits", "sort_gather",
                 "sort_all_passes", "hist_wgs_per_cu", "small_kernel", "small_waves", "scatter_order",
                 "small_wgs_per_cu", "sort_msd", "exchange_self", "hist_nt", "counts_layout",
                 "scatter_counters", "lz4_queue", "scatter_nt", "gather_kernel", "split_cus",
                 "msd_direct")


class Tuning(C.Structure):
    _fields_ = [(f, C.c_int32) for f in TUNING_FIELDS] + [("reserved", C.c_int32 * 1)]


# int (*sux_allgather_fn)(void* ctx, uint64_t tag, const void* send, uint64_t bytes, void* recv)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p)


class PartitionerDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("num_partitions", C.c_int32), ("key_offset", C.c_int32),
                ("key_len", C.c_int32), ("seed", C.c_int32), ("ascending", C.c_int32),
                ("range_bounds", C.c_void_p)]


class HandleDesc(C.Structure):
    _fields_ = [("shuffle_id", C.c_int32), ("num_maps", C.c_int32),
                ("num_partitions", C.c_int32), ("record_size", C.c_int32),
                ("directory_bytes", C.c_uint64)]


class XPlanEntry(C.Structure):
    _fields_ = [("map", C.c_int32), ("owner", C.c_int32), ("batch", C.c_int32),
                ("reserved", C.c_int32)]


class BlockId(C.Structure):
    _fields_ = [("map_index", C.c_int32), ("start_reduce", C.c_int32),
                ("end_reduce", C.c_int32), ("reserved", C.c_int32)]


P, I32, I64, U64, U32, SZ = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_uint32, C.c_size_t
_SIGS = {
    "sux_conf_init": (None, [C.POINTER(Conf)]),
    "sux_conf_set_prealloc": (C.c_int, [C.POINTER(Conf), C.c_char_p]),
    "sux_node_set_bootstrap": (C.c_int, [P, ALLGATHER_FN, P]),
    "sux_node_connect": (C.c_int, [P]),
    "sux_exchange_group_post": (C.c_int, [P, P, I32, I32, P, P, C.POINTER(P)]),
    "sux_exchange_group_issue": (C.c_int, [P, P, P, P, U64, P, P]),
    "sux_exchange_group_discard": (C.c_int, [P, P]),
    "sux_group_create": (C.c_int, [C.c_int32, C.POINTER(P)]),
    "sux_group_destroy": (C.c_int, [P]),
    "sux_group_join": (C.c_int, [P, C.c_char_p, C.c_char_p, C.POINTER(C.c_int32),
                                 C.POINTER(C.c_int32)]),
    "sux_group_size": (C.c_int, [P, C.POINTER(C.c_int32)]),
    "sux_node_set_tuning": (C.c_int, [P, C.POINTER(Tuning)]),
    "sux_node_get_tuning": (C.c_int, [P, C.POINTER(Tuning)]),
    "sux_node_check": (C.c_int, [P]),
    "sux_partition_maps_pipelined": (C.c_int, [P, P, P, U32, U64, U64, U64, P, P, P, P]),
    "sux_pool_stats": (C.c_int, [P, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64),
                                 C.POINTER(U64)]),
    "sux_write_map_outputs": (C.c_int, [P, I32, I32, P, P, U64, U64, P]),
    "sux_wait_map_outputs": (C.c_int, [P, I32]),
    "sux_abi_version": (C.c_int, []),
    "sux_last_error": (C.c_int, [C.c_char_p, SZ]),
    "sux_comm_unique_id": (C.c_int, [P]),
    "sux_node_create": (C.c_int, [C.POINTER(Conf), C.c_int, C.POINTER(P)]),
    "sux_node_destroy": (C.c_int, [P]),
    "sux_partitioner_create": (C.c_int, [P, C.POINTER(PartitionerDesc), C.POINTER(P)]),
    "sux_partitioner_destroy": (C.c_int, [P]),
    "sux_partition_workspace_size": (C.c_int, [P, U32, U64, U64, C.POINTER(U64)]),
    "sux_partition_maps": (C.c_int, [P, P, P, U32, U64, U64, P, P, P, P, P, U64, P]),
    "sux_partition_maps_peer_major": (C.c_int, [P, P, P, U32, U64, U64, I32, P, P, P, P, P, U64,
                                                P]),
    "sux_plan_group": (C.c_int, [I32, I32, I32, I32, P, P, P, P, P]),
    "sux_plan_block_offset": (I64, [I32, I32, I32, I32, P, I32, I32, I32]),
    "sux_plan_group_owned": (C.c_int, [I32, I32, I32, I32, P, P, P, P, P, P]),
    "sux_plan_block_offset_owned": (I64, [I32, I32, I32, I32, P, P, I32, I32, I32]),
    "sux_plan_ownership": (C.c_int, [I32, I32, P, P]),
    "sux_node_set_ownership": (C.c_int, [P, I32, I32, P]),
    "sux_exchange_group": (C.c_int, [P, P, P, I32, I32, P, P, U64, P, P]),
    "sux_partition_ids": (C.c_int, [P, P, P, U32, U64, P, P]),
    "sux_partition_varlen_workspace_size": (C.c_int, [P, U64, U64, C.POINTER(U64)]),
    "sux_partition_varlen": (C.c_int, [P, P, P, P, U64, U64, P, P, P, P, P, P, U64, P]),
    "sux_index_file_commit": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, P, I32, P, P]),
    "sux_write_map_files": (C.c_int, [P, P, P, I32, I32, P, P, P, P]),
    "sux_read_file_blocks": (C.c_int, [P, C.c_char_p, C.c_char_p, I32, I32, I32, P, U64,
                                       C.POINTER(U64), P]),
    "sux_compress_bound": (C.c_int, [U64, I32, I32, I32, C.POINTER(U64)]),
    "sux_compress_workspace_size": (C.c_int, [U64, I32, I32, I32, C.POINTER(U64)]),
    "sux_compress_map_outputs": (C.c_int, [P, P, U64, P, I32, I32, I32, P, U64, P, P, P, P, U64,
                                           P]),
    "sux_decompress_workspace_size": (C.c_int, [U64, I32, I32, C.POINTER(U64)]),
    "sux_decompress_blocks": (C.c_int, [P, P, U64, P, I32, I32, P, U64, P, P, U64, P]),
    "sux_register_shuffle": (C.c_int, [P, I32, I32, I32, I32, C.POINTER(HandleDesc)]),
    "sux_unregister_shuffle": (C.c_int, [P, I32]),
    "sux_write_map_output": (C.c_int, [P, I32, I32, P, P, U64, P]),
    "sux_commit_map_output": (C.c_int, [P, I32, I32, P, U64, P, P]),
    "sux_map_output_index": (C.c_int, [P, I32, I32, P, U64]),
    "sux_exchange": (C.c_int, [P, I32, P]),
    "sux_exchange_maps": (C.c_int, [P, I32, I32, I32, P]),
    "sux_exchange_wait": (C.c_int, [P, I32]),
    "sux_plan_exchange": (C.c_int, [I32, I32, I32, I32, P, P, P, I32, C.POINTER(I32), P, P, P, P]),
    "sux_adopt_map_outputs": (C.c_int, [P, I32, I32, P, U64, U64, P, P]),
    "sux_node_set_spill_dir": (C.c_int, [P, C.c_char_p]),
    "sux_node_spills": (C.c_int, [P, C.POINTER(U64)]),
    "sux_owned_partitions": (C.c_int, [P, I32, I32, C.POINTER(I32), C.POINTER(I32)]),
    "sux_fetch_blocks": (C.c_int, [P, I32, P, I32, P, C.POINTER(P), P]),
    "sux_resolve_blocks": (C.c_int, [P, I32, P, I32, P, P]),
    "sux_buffer_info": (C.c_int, [P, C.POINTER(P), C.POINTER(U64), C.POINTER(U64)]),
    "sux_buffer_alloc": (C.c_int, [P, U64, C.POINTER(P)]),
    "sux_buffer_retain": (C.c_int, [P, I32]),
    "sux_buffer_read": (C.c_int, [P, U64, P, U64, P]),
    "sux_write_map_output_host": (C.c_int, [P, I32, I32, P, P, U64, P]),
    "sux_buffer_release": (C.c_int, [P]),
    "sux_buffer_decompress": (C.c_int, [P, P, U64, P, I32, I32, C.POINTER(P), P, P]),
    "sux_shuffle_set_codec": (C.c_int, [P, I32, I32, I32]),
    "sux_set_kernel_timing": (C.c_int, [P, C.c_int]),
    "sux_kernel_times": (C.c_int, [P, P, P, I32]),
    "sux_kernel_variant": (C.c_int, [P, I32, C.c_char_p, SZ]),
    "sux_generate": (C.c_int, [P, I32, U64, U64, U64, C.c_double, U64, P, P]),
    "sux_ipc_export": (C.c_int, [P, P, P]),
    "sux_ipc_open": (C.c_int, [P, P, C.POINTER(P)]),
    "sux_ipc_close": (C.c_int, [P, P]),
    "sux_pull_group": (C.c_int, [P, I32, I32, P, P, I32, I32, P, U64, P, P]),
    "sux_stream_create": (C.c_int, [P, I32, I32, C.POINTER(P)]),
    "sux_stream_destroy": (C.c_int, [P, P]),
    "sux_sort_workspace_size": (C.c_int, [U64, U32, C.POINTER(U64)]),
    "sux_sort_records": (C.c_int, [P, I32, P, U64, U32, I32, I32, P, P, U64, P]),
    "sux_sort_segments": (C.c_int, [P, I32, P, U64, U32, I32, I32, P, I32, P, P, U64, P]),
}

_lib = None


def header_symbols() -> list[str]:
    """Every function the public header declares."""
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|void|int64_t)\s+(sux_\w+)\s*\(", text, re.M)))


def _init_torch_hip_first() -> None:
    """In a torch process, torch must initialise the shared HIP runtime before this library's
    load-time code-object registration runs; otherwise the runtime reports no device to torch
    (and to us).  Without a GPU (the CPU test job) this is a no-op."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C sparkucx_amd/csrc` "
                          "(there is no CPU fallback for the shuffle path)")
    _init_torch_hip_first()
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    buf = C.create_string_buffer(4096)
    load().sux_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    if rc != SUX_OK:
        raise SuxError(rc, f"{what}: {last_error()}")


def default_conf(device=0, rank=0, world_size=1, comm_id: bytes | None = None,
                 prealloc: str | None = None, **kw) -> Conf:
    """sux_conf with the reference's defaults; `prealloc` is Spark's
    spark.shuffle.ucx.memory.preAllocateBuffers string ("4k:1000,16k:500")."""
    c = Conf()
    load().sux_conf_init(C.byref(c))
    c.device, c.rank, c.world_size = device, rank, world_size
    if comm_id is not None:
        C.memmove(c.comm_id, comm_id, 128)
    if prealloc is not None:
        check(load().sux_conf_set_prealloc(C.byref(c), prealloc.encode()), "sux_conf_set_prealloc")
    for k, v in kw.items():
        setattr(c, k, v)
    return c


HIP_H2D, HIP_D2H, HIP_D2D = 1, 2, 3
_hip = None


def hip_memcpy(dst: int, src: int, nbytes: int, kind: int) -> None:
    """Synchronous hipMemcpy through the HIP runtime already loaded in this process."""
    global _hip
    if _hip is None:
        load()
        _hip = C.CDLL("libamdhip64.so.7")
        _hip.hipMemcpy.restype = C.c_int
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    rc = _hip.hipMemcpy(dst, src, nbytes, kind)
    if rc != 0:
        raise SuxError(SUX_EHIP, f"hipMemcpy failed ({rc})")


def plan_ownership(world: int, partition_bytes) -> "np.ndarray":
    """sux_plan_ownership: the contiguous split of R partitions into `world` non-empty owner
    ranges whose largest holds the fewest bytes; returns the world + 1 int32 bounds."""
    import numpy as np
    b = np.ascontiguousarray(np.asarray(partition_bytes, dtype=np.int64))
    own = np.zeros(world + 1, dtype=np.int32)
    check(load().sux_plan_ownership(world, b.size, b.ctypes.data, own.ctypes.data),
          "sux_plan_ownership")
    return own


def unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    check(load().sux_comm_unique_id(buf), "sux_comm_unique_id")
    return bytes(buf)
