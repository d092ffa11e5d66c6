"""Thin torch-facing wrappers over the C-ABI (device tensors in, device tensors out).

Used by tests/ and bench.py.  torch is only plumbing here: it allocates HBM and provides the
stream; every byte of the shuffle path is moved by the library's gfx950 kernels.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch

from . import native as N


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(stream) -> int | None:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else stream


class Partitioner:
    def __init__(self, node: "Node", kind: int, num_partitions: int, key_offset: int = 0,
                 key_len: int = 8, seed: int = 42, ascending: bool = True,
                 bounds: bytes | None = None):
        self.node, self.kind, self.R = node, kind, num_partitions
        self.key_offset, self.key_len = key_offset, key_len
        self._bounds = None if bounds is None else C.create_string_buffer(bytes(bounds), len(bounds))
        d = N.PartitionerDesc(kind, num_partitions, key_offset, key_len, seed, int(ascending),
                              C.cast(self._bounds, C.c_void_p) if self._bounds is not None else None)
        h = C.c_void_p()
        N.check(N.load().sux_partitioner_create(node.h, C.byref(d), C.byref(h)),
                "sux_partitioner_create")
        self.h = h

    def close(self):
        if self.h:
            N.check(N.load().sux_partitioner_destroy(self.h), "sux_partitioner_destroy")
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Node:
    """One executor's shuffle node on one GPU (UcxNode analog)."""

    def __init__(self, device: int = 0, rank: int = 0, world_size: int = 1,
                 comm_id: bytes | None = None, is_driver: bool = False, **conf):
        self.lib = N.load()
        self.device = device
        # torch must bring up its HIP context first: its lazy init refuses the device once another
        # user of the (shared) HIP runtime in this process has initialised it
        torch.cuda.init()
        c = N.default_conf(device, rank, world_size, comm_id, **conf)
        h = C.c_void_p()
        N.check(self.lib.sux_node_create(C.byref(c), int(is_driver), C.byref(h)), "sux_node_create")
        self.h = h
        self.rank, self.world_size = rank, world_size
        self.dev = torch.device("cuda", device)
        self._streams: list[int] = []

    def close(self):
        if self.h:
            for st in list(self._streams):
                self.destroy_stream(st)
            N.check(self.lib.sux_node_destroy(self.h), "sux_node_destroy")
            self.h = None

    def set_bootstrap(self, allgather):
        """Control plane for the exchange without RCCL: `allgather(b: bytes) -> list[bytes]` (one
        entry per rank, rank order), e.g. torch.distributed.all_gather_object over gloo."""
        def fn(_ctx, _tag, send, nbytes, recv):
            # (torch.distributed collectives are matched by issue order, so the tag is unused)
            try:
                parts = allgather(C.string_at(send, nbytes))
                if len(parts) != self.world_size or any(len(p) != nbytes for p in parts):
                    return -1  # a contribution of another size: the ranks are out of step
                C.memmove(recv, b"".join(parts), nbytes * len(parts))
                return 0
            except Exception:  # pragma: no cover - reported as SUX_ECOMM by the library
                return -1
        self._boot = N.ALLGATHER_FN(fn)  # kept alive as long as the node
        N.check(self.lib.sux_node_set_bootstrap(self.h, self._boot, None), "sux_node_set_bootstrap")

    def connect(self):
        """sux_node_connect: join the group's RCCL communicator through the bootstrap (rank 0's
        unique id all-gathered, then ncclCommInitRank) — a collective over the group."""
        N.check(self.lib.sux_node_connect(self.h), "sux_node_connect")

    def tuning(self) -> dict:
        t = N.Tuning()
        N.check(self.lib.sux_node_get_tuning(self.h, C.byref(t)), "sux_node_get_tuning")
        return {f: getattr(t, f) for f in N.TUNING_FIELDS}

    def set_tuning(self, **fields) -> dict:
        """Update fields of the node's kernel tuning table (sux_tuning; 0 = default); returns
        the previous table so a caller can restore it."""
        old = self.tuning()
        t = N.Tuning()
        for f, v in {**old, **fields}.items():
            setattr(t, f, int(v))
        N.check(self.lib.sux_node_set_tuning(self.h, C.byref(t)), "sux_node_set_tuning")
        return old

    def check(self):
        """sux_node_check: raise if a kernel recorded a failure in the device error word."""
        N.check(self.lib.sux_node_check(self.h), "sux_node_check")

    def pool_stats(self) -> dict:
        v = [C.c_uint64() for _ in range(4)]
        N.check(self.lib.sux_pool_stats(self.h, *[C.byref(x) for x in v]), "sux_pool_stats")
        return dict(zip(("allocated_bytes", "requests", "allocs", "preallocs"), [x.value for x in v]))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- partitioners ----------------------------------------------------------------------
    def partitioner(self, kind, num_partitions, **kw) -> Partitioner:
        return Partitioner(self, kind, num_partitions, **kw)

    # ---- inputs ------------------------------------------------------------------------------
    def generate(self, kind: int, seed: int, first: int, n: int, record_size: int,
                 zipf_s: float = 1.1, zipf_n: int = 1 << 24, out: torch.Tensor | None = None,
                 stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty(n * record_size, dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_generate(self.h, kind, seed, first, n, zipf_s, zipf_n, _ptr(out),
                                      _stream(stream)), "sux_generate")
        return out

    # ---- stateless map side ------------------------------------------------------------------
    def workspace_size(self, part: Partitioner, record_size: int, records_per_map: int,
                       num_records: int) -> int:
        v = C.c_uint64()
        N.check(self.lib.sux_partition_workspace_size(part.h, record_size, records_per_map,
                                                      num_records, C.byref(v)),
                "sux_partition_workspace_size")
        return v.value

    def partition_maps(self, part: Partitioner, records: torch.Tensor, record_size: int,
                       records_per_map: int, num_records: int | None = None,
                       out: torch.Tensor | None = None, index: torch.Tensor | None = None,
                       index_be: torch.Tensor | None = None, pids: torch.Tensor | None = None,
                       workspace: torch.Tensor | None = None, want_be: bool = True,
                       stream=None):
        n = records.numel() // record_size if num_records is None else num_records
        maps = max(1, -(-n // records_per_map))
        R = part.R
        if out is None:
            out = torch.empty(max(1, n * record_size), dtype=torch.uint8, device=self.dev)
        if index is None:
            index = torch.empty(maps * (R + 1), dtype=torch.int64, device=self.dev)
        if index_be is None and want_be:
            index_be = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=self.dev)
        if workspace is None:
            workspace = torch.empty(max(1, self.workspace_size(part, record_size, records_per_map,
                                                               n)),
                                    dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_partition_maps(self.h, part.h, _ptr(records), record_size,
                                            records_per_map, n, _ptr(out), _ptr(index),
                                            _ptr(index_be), _ptr(pids), _ptr(workspace),
                                            workspace.numel(), _stream(stream)),
                "sux_partition_maps")
        return out, index, index_be

    def partition_maps_pipelined(self, part: Partitioner, records: torch.Tensor,
                                 record_size: int, records_per_map: int,
                                 num_records: int | None = None, group_records: int = 0,
                                 out: torch.Tensor | None = None,
                                 index: torch.Tensor | None = None,
                                 index_be: torch.Tensor | None = None, want_be: bool = True,
                                 stream=None):
        """sux_partition_maps_pipelined: launch groups of whole maps on the node's two map
        streams (node-owned workspaces), joined back into `stream`."""
        n = records.numel() // record_size if num_records is None else num_records
        maps = max(1, -(-n // records_per_map))
        R = part.R
        if out is None:
            out = torch.empty(max(1, n * record_size), dtype=torch.uint8, device=self.dev)
        if index is None:
            index = torch.empty(maps * (R + 1), dtype=torch.int64, device=self.dev)
        if index_be is None and want_be:
            index_be = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_partition_maps_pipelined(
            self.h, part.h, _ptr(records), record_size, records_per_map, n, group_records,
            _ptr(out), _ptr(index), _ptr(index_be), _stream(stream)),
            "sux_partition_maps_pipelined")
        return out, index, index_be

    def partition_maps_peer_major(self, part: Partitioner, records: torch.Tensor,
                                  record_size: int, records_per_map: int, world: int,
                                  num_records: int | None = None, out=None, index=None,
                                  index_be=None, peer_bytes=None, workspace=None, stream=None):
        n = records.numel() // record_size if num_records is None else num_records
        maps = max(1, -(-n // records_per_map))
        R = part.R
        if out is None:
            out = torch.empty(max(1, n * record_size), dtype=torch.uint8, device=self.dev)
        if index is None:
            index = torch.empty(maps * (R + 1), dtype=torch.int64, device=self.dev)
        if peer_bytes is None:
            peer_bytes = torch.zeros(world, dtype=torch.int64, device=self.dev)
        if workspace is None:
            workspace = torch.empty(max(1, self.workspace_size(part, record_size, records_per_map,
                                                               n)),
                                    dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_partition_maps_peer_major(
            self.h, part.h, _ptr(records), record_size, records_per_map, n, world, _ptr(out),
            _ptr(index), _ptr(index_be), _ptr(peer_bytes), _ptr(workspace), workspace.numel(),
            _stream(stream)), "sux_partition_maps_peer_major")
        return out, index, peer_bytes

    def partition_ids(self, part: Partitioner, records: torch.Tensor, record_size: int,
                      stream=None) -> torch.Tensor:
        n = records.numel() // record_size
        pids = torch.empty(max(1, n), dtype=torch.int16, device=self.dev)
        N.check(self.lib.sux_partition_ids(self.h, part.h, _ptr(records), record_size, n,
                                           _ptr(pids), _stream(stream)), "sux_partition_ids")
        return pids[:n]

    def varlen_workspace_size(self, part: Partitioner, records_per_map: int,
                              num_records: int) -> int:
        b = C.c_uint64()
        N.check(self.lib.sux_partition_varlen_workspace_size(part.h, records_per_map, num_records,
                                                             C.byref(b)),
                "sux_partition_varlen_workspace_size")
        return b.value

    def partition_varlen(self, part: Partitioner, data: torch.Tensor, offsets: torch.Tensor,
                         records_per_map: int, pids_in: torch.Tensor | None = None,
                         out: torch.Tensor | None = None, index: torch.Tensor | None = None,
                         index_be: torch.Tensor | None = None, pids: torch.Tensor | None = None,
                         workspace: torch.Tensor | None = None, want_be: bool = True,
                         stream=None):
        """Variable-length rows (Spark SQL UnsafeRowSerializer framing): row i is
        data[offsets[i] - offsets[0] : offsets[i+1] - offsets[0]] (offsets: int64, n + 1, device).
        Returns (out, index, index_be); map m's data file is out[offsets[m*rpm] - offsets[0] :
        offsets[min((m+1)*rpm, n)] - offsets[0]] and its index holds byte offsets."""
        n = offsets.numel() - 1
        maps = max(1, -(-n // records_per_map))
        R = part.R
        if out is None:
            out = torch.empty(max(4, data.numel()), dtype=torch.uint8, device=self.dev)
        if index is None:
            index = torch.empty(maps * (R + 1), dtype=torch.int64, device=self.dev)
        if index_be is None and want_be:
            index_be = torch.empty(maps * (R + 1) * 8, dtype=torch.uint8, device=self.dev)
        if workspace is None:
            workspace = torch.empty(max(1, self.varlen_workspace_size(part, records_per_map,
                                                                      max(n, 0))),
                                    dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_partition_varlen(self.h, part.h, _ptr(data), _ptr(offsets),
                                              records_per_map, max(n, 0), _ptr(pids_in),
                                              _ptr(out), _ptr(index), _ptr(index_be), _ptr(pids),
                                              _ptr(workspace), workspace.numel(),
                                              _stream(stream)),
                "sux_partition_varlen")
        return out, index, index_be

    # ---- Spark's on-disk files ---------------------------------------------------------------
    def write_map_files(self, data: torch.Tensor, index: torch.Tensor, num_maps: int, R: int,
                        data_paths: list[str], index_paths: list[str], stream=None) -> np.ndarray:
        """Consecutive device map outputs -> one committed data + index file pair per map
        (IndexShuffleBlockResolver.writeIndexFileAndCommit semantics).  Returns the committed
        lengths, int64[num_maps, R] (an already committed pair's lengths win)."""
        dp = (C.c_char_p * num_maps)(*[p.encode() for p in data_paths])
        ip = (C.c_char_p * num_maps)(*[p.encode() for p in index_paths])
        out = np.zeros(num_maps * R, np.int64)
        N.check(self.lib.sux_write_map_files(self.h, _ptr(data), _ptr(index), num_maps, R, dp, ip,
                                             out.ctypes.data, _stream(stream)),
                "sux_write_map_files")
        return out.reshape(num_maps, R)

    def read_file_blocks(self, data_path: str, index_path: str, R: int, start: int, end: int,
                         out: torch.Tensor | None = None, capacity: int | None = None,
                         stream=None) -> torch.Tensor:
        """Partitions [start, end) of one map's files into device memory."""
        if out is None:
            cap = capacity if capacity is not None else os.path.getsize(data_path)
            out = torch.empty(max(1, cap), dtype=torch.uint8, device=self.dev)
        n = C.c_uint64()
        N.check(self.lib.sux_read_file_blocks(self.h, data_path.encode(), index_path.encode(), R,
                                              start, end, _ptr(out), out.numel(), C.byref(n),
                                              _stream(stream)), "sux_read_file_blocks")
        return out[:n.value]

    def compress_bound(self, data_bytes: int, num_maps: int, R: int, block_size: int = 32768) -> int:
        b = C.c_uint64()
        N.check(self.lib.sux_compress_bound(data_bytes, num_maps, R, block_size, C.byref(b)),
                "sux_compress_bound")
        return b.value

    def compress_workspace_size(self, data_bytes: int, num_maps: int, R: int,
                                block_size: int = 32768) -> int:
        b = C.c_uint64()
        N.check(self.lib.sux_compress_workspace_size(data_bytes, num_maps, R, block_size,
                                                     C.byref(b)), "sux_compress_workspace_size")
        return b.value

    def compress_map_outputs(self, data: torch.Tensor, index: torch.Tensor, num_maps: int, R: int,
                             block_size: int = 32768, data_bytes: int | None = None,
                             out: torch.Tensor | None = None, out_index=None, out_index_be=None,
                             out_bytes: torch.Tensor | None = None,
                             workspace: torch.Tensor | None = None, want_be: bool = True,
                             stream=None):
        """spark.shuffle.compress=true (lz4): every (map, partition) run of the consecutive map
        outputs in `data` -> its own LZ4BlockOutputStream stream.  Returns (out, out_index,
        out_index_be, out_bytes) with out_bytes a 1-element device int64 tensor (the total)."""
        nb = data.numel() if data_bytes is None else data_bytes
        if out is None:
            out = torch.empty(max(16, self.compress_bound(nb, num_maps, R, block_size)),
                              dtype=torch.uint8, device=self.dev)
        if out_index is None:
            out_index = torch.empty(num_maps * (R + 1), dtype=torch.int64, device=self.dev)
        if out_index_be is None and want_be:
            out_index_be = torch.empty(num_maps * (R + 1) * 8, dtype=torch.uint8, device=self.dev)
        if out_bytes is None:
            out_bytes = torch.zeros(1, dtype=torch.int64, device=self.dev)
        if workspace is None:
            workspace = torch.empty(self.compress_workspace_size(nb, num_maps, R, block_size),
                                    dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_compress_map_outputs(self.h, _ptr(data), nb, _ptr(index), num_maps, R,
                                                  block_size, _ptr(out), out.numel(),
                                                  _ptr(out_index), _ptr(out_index_be),
                                                  _ptr(out_bytes), _ptr(workspace),
                                                  workspace.numel(), _stream(stream)),
                "sux_compress_map_outputs")
        return out, out_index, out_index_be, out_bytes

    def decompress_workspace_size(self, in_bytes: int, num_blocks: int,
                                  max_block_size: int = 32768) -> int:
        b = C.c_uint64()
        N.check(self.lib.sux_decompress_workspace_size(in_bytes, num_blocks, max_block_size,
                                                       C.byref(b)),
                "sux_decompress_workspace_size")
        return b.value

    def decompress_blocks(self, data: torch.Tensor, offsets: torch.Tensor,
                          max_block_size: int = 32768, out: torch.Tensor | None = None,
                          out_offsets: torch.Tensor | None = None,
                          workspace: torch.Tensor | None = None, in_bytes: int | None = None,
                          stream=None):
        """The reader's side of spark.shuffle.compress=true: the LZ4Block streams of the fetched
        blocks [offsets[k], offsets[k + 1]) of `data` (device int64 offsets) decoded, blocks
        consecutive.  Returns (out, out_offsets).  With out=None the decoded size is read first
        (one host wait: sux_decompress_blocks without an output, then with one).  Corruption or a
        too-small `out` sets the node's error word: call check()."""
        nb = offsets.numel() - 1
        ib = data.numel() if in_bytes is None else in_bytes
        if out_offsets is None:
            out_offsets = torch.empty(nb + 1, dtype=torch.int64, device=self.dev)
        if workspace is None:
            workspace = torch.empty(self.decompress_workspace_size(ib, nb, max_block_size),
                                    dtype=torch.uint8, device=self.dev)
        if out is None:
            N.check(self.lib.sux_decompress_blocks(self.h, _ptr(data), ib, _ptr(offsets), nb,
                                                   max_block_size, None, 0, _ptr(out_offsets),
                                                   _ptr(workspace), workspace.numel(),
                                                   _stream(stream)),
                    "sux_decompress_blocks (sizes)")
            torch.cuda.synchronize(self.dev)
            total = int(out_offsets[nb].item())
            out = torch.empty(max(16, total), dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_decompress_blocks(self.h, _ptr(data), ib, _ptr(offsets), nb,
                                               max_block_size, _ptr(out), out.numel(),
                                               _ptr(out_offsets), _ptr(workspace),
                                               workspace.numel(), _stream(stream)),
                "sux_decompress_blocks")
        return out, out_offsets

    def exchange_group(self, send: torch.Tensor, index: torch.Tensor, num_maps: int, R: int,
                       gathered: torch.Tensor, recv: torch.Tensor, stream=None) -> np.ndarray:
        rb = (C.c_uint64 * self.world_size)()
        N.check(self.lib.sux_exchange_group(self.h, _ptr(send), _ptr(index), num_maps, R,
                                            _ptr(gathered), _ptr(recv), recv.numel(), rb,
                                            _stream(stream)), "sux_exchange_group")
        return np.frombuffer(rb, dtype=np.uint64).copy()

    def exchange_group_post(self, index: torch.Tensor, num_maps: int, R: int,
                            gathered: torch.Tensor, stream=None):
        """First half of exchange_group: the all-gather of the index tables + their async
        read-back; returns the ticket exchange_group_issue consumes."""
        t = C.c_void_p()
        N.check(self.lib.sux_exchange_group_post(self.h, _ptr(index), num_maps, R, _ptr(gathered),
                                                 _stream(stream), C.byref(t)),
                "sux_exchange_group_post")
        return t

    def exchange_group_issue(self, ticket, send: torch.Tensor, recv: torch.Tensor,
                             stream=None) -> np.ndarray:
        """Second half: plan from the read-back (host wait) and enqueue the all-to-all."""
        rb = (C.c_uint64 * self.world_size)()
        N.check(self.lib.sux_exchange_group_issue(self.h, ticket, _ptr(send), _ptr(recv),
                                                  recv.numel(), rb, _stream(stream)),
                "sux_exchange_group_issue")
        return np.frombuffer(rb, dtype=np.uint64).copy()

    def set_ownership(self, world: int, R: int, bounds=None):
        """sux_node_set_ownership: peer h owns partitions [bounds[h], bounds[h + 1]) in the
        stateless group calls; None restores the equal split."""
        if bounds is None:
            N.check(self.lib.sux_node_set_ownership(self.h, world, R, None),
                    "sux_node_set_ownership")
            return
        b = np.ascontiguousarray(np.asarray(bounds, dtype=np.int32))
        N.check(self.lib.sux_node_set_ownership(self.h, world, R, b.ctypes.data),
                "sux_node_set_ownership")

    def exchange_group_discard(self, ticket):
        """A posted ticket that will not be issued: wait for its read-back and free it."""
        N.check(self.lib.sux_exchange_group_discard(self.h, ticket), "sux_exchange_group_discard")

    # ---- one-sided exchange over HIP IPC ----------------------------------------------------
    def ipc_handle(self, t: torch.Tensor) -> bytes:
        """72-byte descriptor: IPC handle of t's allocation + t's offset in it."""
        buf = (C.c_uint8 * 72)()
        N.check(self.lib.sux_ipc_export(self.h, _ptr(t), buf), "sux_ipc_export")
        return bytes(buf)

    def ipc_open(self, handle: bytes) -> int:
        hb = (C.c_uint8 * 72).from_buffer_copy(handle)
        p = C.c_void_p()
        N.check(self.lib.sux_ipc_open(self.h, hb, C.byref(p)), "sux_ipc_open")
        return p.value

    def ipc_close(self, ptr: int):
        N.check(self.lib.sux_ipc_close(self.h, ptr), "sux_ipc_close")

    def pull_group(self, world: int, rank: int, src_ptrs: torch.Tensor, gathered: torch.Tensor,
                   num_maps: int, R: int, recv: torch.Tensor, recv_bytes: torch.Tensor | None = None,
                   stream=None):
        N.check(self.lib.sux_pull_group(self.h, world, rank, _ptr(src_ptrs), _ptr(gathered),
                                        num_maps, R, _ptr(recv), recv.numel(), _ptr(recv_bytes),
                                        _stream(stream)), "sux_pull_group")

    # ---- shuffle lifecycle / plugin surface -----------------------------------------------------
    def register_shuffle(self, shuffle_id: int, num_maps: int, num_partitions: int,
                         record_size: int) -> N.HandleDesc:
        d = N.HandleDesc()
        N.check(self.lib.sux_register_shuffle(self.h, shuffle_id, num_maps, num_partitions,
                                              record_size, C.byref(d)), "sux_register_shuffle")
        return d

    def set_shuffle_codec(self, shuffle_id: int, codec: int, block_size: int = 32768):
        """spark.shuffle.compress for the maps this node writes: N.SUX_CODEC_LZ4 or _NONE."""
        N.check(self.lib.sux_shuffle_set_codec(self.h, shuffle_id, codec, block_size),
                "sux_shuffle_set_codec")

    def unregister_shuffle(self, shuffle_id: int):
        N.check(self.lib.sux_unregister_shuffle(self.h, shuffle_id), "sux_unregister_shuffle")

    def write_map_output(self, shuffle_id: int, map_index: int, part: Partitioner,
                         records: torch.Tensor, num_records: int, stream=None):
        N.check(self.lib.sux_write_map_output(self.h, shuffle_id, map_index, part.h,
                                              _ptr(records), num_records, _stream(stream)),
                "sux_write_map_output")

    def write_map_output_host(self, shuffle_id: int, map_index: int, part: Partitioner,
                              host_records: torch.Tensor, num_records: int, stream=None):
        """The JVM writer's entry (GpuShuffleWriter -> SuxNative.writeMapOutputHostAddr): rows in
        host memory (pinned or pageable) staged to HBM, partitioned and published; waits."""
        assert host_records.device.type == "cpu", "host rows"
        N.check(self.lib.sux_write_map_output_host(self.h, shuffle_id, map_index, part.h,
                                                   _ptr(host_records), num_records,
                                                   _stream(stream)),
                "sux_write_map_output_host")

    def write_map_outputs(self, shuffle_id: int, first_map: int, part: Partitioner,
                          records: torch.Tensor, records_per_map: int, num_records: int,
                          stream=None):
        """Consecutive map tasks first_map.. in one launch group; published lazily (no wait)."""
        N.check(self.lib.sux_write_map_outputs(self.h, shuffle_id, first_map, part.h,
                                               _ptr(records), records_per_map, num_records,
                                               _stream(stream)), "sux_write_map_outputs")

    def wait_map_outputs(self, shuffle_id: int):
        N.check(self.lib.sux_wait_map_outputs(self.h, shuffle_id), "sux_wait_map_outputs")

    def commit_map_output(self, shuffle_id: int, map_index: int, data: torch.Tensor | None,
                          lengths, stream=None):
        arr = np.ascontiguousarray(np.asarray(lengths, dtype=np.int64))
        nbytes = 0 if data is None else data.numel()
        N.check(self.lib.sux_commit_map_output(self.h, shuffle_id, map_index, _ptr(data), nbytes,
                                               arr.ctypes.data, _stream(stream)),
                "sux_commit_map_output")

    def map_output_index(self, shuffle_id: int, map_index: int, R: int) -> bytes:
        buf = (C.c_uint8 * (8 * (R + 1)))()
        N.check(self.lib.sux_map_output_index(self.h, shuffle_id, map_index, buf, len(buf)),
                "sux_map_output_index")
        return bytes(buf)

    def exchange(self, shuffle_id: int, stream=None):
        N.check(self.lib.sux_exchange(self.h, shuffle_id, _stream(stream)), "sux_exchange")

    def exchange_maps(self, shuffle_id: int, first_map: int, num_maps: int, stream=None):
        """Asynchronous exchange of the map window [first_map, first_map + num_maps) (collective)."""
        N.check(self.lib.sux_exchange_maps(self.h, shuffle_id, first_map, num_maps,
                                           _stream(stream)), "sux_exchange_maps")

    def exchange_wait(self, shuffle_id: int):
        N.check(self.lib.sux_exchange_wait(self.h, shuffle_id), "sux_exchange_wait")

    def adopt_map_outputs(self, shuffle_id: int, first_map: int, out: torch.Tensor,
                          records_per_map: int, num_records: int, index: torch.Tensor,
                          stream=None):
        """Commit map outputs a stateless partition call wrote (no copy; published lazily)."""
        N.check(self.lib.sux_adopt_map_outputs(self.h, shuffle_id, first_map, _ptr(out),
                                               records_per_map, num_records, _ptr(index),
                                               _stream(stream)), "sux_adopt_map_outputs")

    def set_spill_dir(self, path: str | None):
        N.check(self.lib.sux_node_set_spill_dir(self.h, None if path is None else path.encode()),
                "sux_node_set_spill_dir")

    def spills(self) -> int:
        v = C.c_uint64()
        N.check(self.lib.sux_node_spills(self.h, C.byref(v)), "sux_node_spills")
        return v.value

    def owned_partitions(self, shuffle_id: int, rank: int | None = None) -> tuple[int, int]:
        a, b = C.c_int32(), C.c_int32()
        N.check(self.lib.sux_owned_partitions(self.h, shuffle_id, self.rank if rank is None else rank,
                                              C.byref(a), C.byref(b)), "sux_owned_partitions")
        return a.value, b.value

    @staticmethod
    def _blocks(blocks) -> np.ndarray:
        """sux_block_id rows (map, start, end, 0) as one C-contiguous int32 (n, 4) array, from
        (map, start[, end]) tuples or an int (n, 2|3|4) numpy array.  An int32 (n, 4) array is
        used as it is (no copy: a reducer that keeps its block list resolves without converting)."""
        if isinstance(blocks, np.ndarray):
            if (blocks.dtype == np.int32 and blocks.ndim == 2 and blocks.shape[1] == 4
                    and blocks.flags.c_contiguous and len(blocks)):
                return blocks
            b = np.zeros((max(1, len(blocks)), 4), np.int32)
            if len(blocks):
                b[:len(blocks), :2] = blocks[:, :2]
                b[:len(blocks), 2] = blocks[:, 2] if blocks.shape[1] > 2 else blocks[:, 1] + 1
            return b
        if len(blocks) and len({len(b) for b in blocks}) == 1 and len(blocks[0]) in (2, 3):
            try:  # uniform tuples: one numpy conversion
                return Node._blocks(np.asarray(blocks, dtype=np.int64))
            except (TypeError, ValueError, OverflowError):
                pass
        b = np.zeros((max(1, len(blocks)), 4), np.int32)
        for i, t in enumerate(blocks):
            b[i, 0], b[i, 1] = t[0], t[1]
            b[i, 2] = t[2] if len(t) > 2 else t[1] + 1
        return b

    def fetch_blocks(self, shuffle_id: int, blocks, stream=None):
        """Returns (FetchedBuffer, sizes[list])."""
        arr = self._blocks(blocks)
        k = len(blocks)
        sizes = np.empty(max(1, k), np.int64)
        h = C.c_void_p()
        N.check(self.lib.sux_fetch_blocks(self.h, shuffle_id, arr.ctypes.data, k,
                                          sizes.ctypes.data, C.byref(h), _stream(stream)),
                "sux_fetch_blocks")
        return FetchedBuffer(self, h, k), sizes[:k].tolist()

    def resolve_blocks(self, shuffle_id: int, blocks):
        """(device addresses uint64[n], sizes int64[n]) of the blocks (zero-copy)."""
        arr = self._blocks(blocks)
        k = len(blocks)
        addrs = np.empty(max(1, k), np.uint64)
        sizes = np.empty(max(1, k), np.int64)
        N.check(self.lib.sux_resolve_blocks(self.h, shuffle_id, arr.ctypes.data, k,
                                            addrs.ctypes.data, sizes.ctypes.data),
                "sux_resolve_blocks")
        return addrs[:k], sizes[:k]

    # ---- measurement -------------------------------------------------------------------------
    def sort_records(self, records: torch.Tensor, record_size: int, key_kind: int,
                     key_offset: int, key_len: int, num_records: int | None = None,
                     out: torch.Tensor | None = None, workspace: torch.Tensor | None = None,
                     stream=None) -> torch.Tensor:
        """Stable GPU sort of fixed-size records by key (reduce side, UcxShuffleReader's
        ExternalSorter step).  Returns `out` (records in ascending key order)."""
        n = records.numel() // record_size if num_records is None else num_records
        if out is None:
            out = torch.empty(max(1, n * record_size), dtype=torch.uint8, device=self.dev)
        if workspace is None:
            workspace = torch.empty(max(1, self.sort_workspace_size(n, record_size)),
                                    dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_sort_records(self.h, key_kind, _ptr(records), n, record_size,
                                          key_offset, key_len, _ptr(out), _ptr(workspace),
                                          workspace.numel(), _stream(stream)), "sux_sort_records")
        return out

    def sort_segments(self, records: torch.Tensor, record_size: int, key_kind: int,
                      key_offset: int, key_len: int, segment_offsets: torch.Tensor,
                      num_records: int | None = None, out: torch.Tensor | None = None,
                      workspace: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        """Sort every run [segment_offsets[k], segment_offsets[k+1]) of records by key, stably,
        in one call (a reducer's partitions).  segment_offsets: device int64, num_segments + 1."""
        n = records.numel() // record_size if num_records is None else num_records
        if out is None:
            out = torch.empty(max(1, n * record_size), dtype=torch.uint8, device=self.dev)
        if workspace is None:
            workspace = torch.empty(max(1, self.sort_workspace_size(n, record_size)),
                                    dtype=torch.uint8, device=self.dev)
        N.check(self.lib.sux_sort_segments(self.h, key_kind, _ptr(records), n, record_size,
                                           key_offset, key_len, _ptr(segment_offsets),
                                           segment_offsets.numel() - 1, _ptr(out),
                                           _ptr(workspace), workspace.numel(), _stream(stream)),
                "sux_sort_segments")
        return out

    def sort_workspace_size(self, n: int, record_size: int) -> int:
        b = C.c_uint64()
        N.check(self.lib.sux_sort_workspace_size(n, record_size, C.byref(b)),
                "sux_sort_workspace_size")
        return b.value

    def cu_stream(self, num_cus: int, complement: bool = False) -> int:
        """hipStream_t (as int) running on `num_cus` CUs spread over the XCDs, or on the other CUs
        (complement).  Wrap with torch.cuda.ExternalStream; destroy with destroy_stream()."""
        out = C.c_void_p()
        N.check(self.lib.sux_stream_create(self.h, int(num_cus), int(bool(complement)),
                                           C.byref(out)), "sux_stream_create")
        self._streams.append(out.value)
        return out.value

    def destroy_stream(self, stream: int):
        if stream in self._streams:
            self._streams.remove(stream)
            N.check(self.lib.sux_stream_destroy(self.h, C.c_void_p(stream)), "sux_stream_destroy")

    def set_kernel_timing(self, on: bool):
        N.check(self.lib.sux_set_kernel_timing(self.h, int(on)), "sux_set_kernel_timing")

    def kernel_times(self) -> dict:
        n = len(N.KERNELS)
        launches, ms = (C.c_int64 * n)(), (C.c_double * n)()
        N.check(self.lib.sux_kernel_times(self.h, launches, ms, n), "sux_kernel_times")
        return {k: (launches[i], ms[i]) for i, k in enumerate(N.KERNELS)}

    def kernel_variant(self, slot: int) -> str:
        """Kernel last launched for slot 0=hist 1=scan 2=scatter 3=copy (e.g. 'k_scatter7')."""
        buf = C.create_string_buffer(64)
        N.check(self.lib.sux_kernel_variant(self.h, slot, buf, len(buf)), "sux_kernel_variant")
        return buf.value.decode()


def plan_exchange(world: int, rank: int, entries, seg, length, loopback: bool = False,
                  max_rounds: int = 4096) -> dict:
    """sux_plan_exchange (host arithmetic): entries = [(map, owner, batch)], seg/length =
    int arrays [n, world].  Returns the per-round all-to-all arguments of `rank`."""
    n = len(entries)
    ents = (N.XPlanEntry * max(1, n))(*[N.XPlanEntry(int(m), int(o), int(b), 0)
                                        for m, o, b in entries])
    sg = np.ascontiguousarray(np.asarray(seg, dtype=np.uint64).reshape(-1))
    ln = np.ascontiguousarray(np.asarray(length, dtype=np.uint64).reshape(-1))
    rounds = C.c_int32()
    counts = np.zeros((max_rounds, 4, world), np.uint64)
    piece = np.full((max_rounds, world), -1, np.int32)
    base = np.zeros(max_rounds + 1, np.uint64)
    roff = np.zeros(max(1, n), np.uint64)
    N.check(N.load().sux_plan_exchange(world, rank, int(loopback), n, ents,
                                       sg.ctypes.data if n else None,
                                       ln.ctypes.data if n else None, max_rounds,
                                       C.byref(rounds), counts.ctypes.data, piece.ctypes.data,
                                       base.ctypes.data, roff.ctypes.data), "sux_plan_exchange")
    k = rounds.value
    return {"rounds": k, "sendcounts": counts[:k, 0], "sdispls": counts[:k, 1],
            "recvcounts": counts[:k, 2], "rdispls": counts[:k, 3], "piece": piece[:k],
            "round_base": base[:k + 1], "recv_off": roff[:n]}


class FetchedBuffer:
    """Pooled device buffer of a fetch (refcounted; one reference per block)."""

    def __init__(self, node: Node, h, refs: int):
        self.node, self.h, self.refs = node, h, max(1, refs)

    def info(self):
        p, size, cap = C.c_void_p(), C.c_uint64(), C.c_uint64()
        N.check(self.node.lib.sux_buffer_info(self.h, C.byref(p), C.byref(size), C.byref(cap)),
                "sux_buffer_info")
        return p.value, size.value, cap.value

    def to_bytes(self) -> bytes:
        p, size, _ = self.info()
        if size == 0:
            return b""
        host = (C.c_uint8 * size)()
        torch.cuda.synchronize(self.node.dev)
        N.hip_memcpy(C.addressof(host), p, size, N.HIP_D2H)
        return bytes(host)

    def release(self, count: int = 1):
        for _ in range(count):
            N.check(self.node.lib.sux_buffer_release(self.h), "sux_buffer_release")
        self.refs -= count

    def decompress(self, sizes, max_block_size: int = 32768, offset: int = 0, stream=None):
        """The blocks' LZ4Block streams (sizes[k] bytes each, consecutive from offset) decoded on
        the device (sux_buffer_decompress).  Returns (FetchedBuffer with one reference, decoded
        sizes[list])."""
        sz = np.ascontiguousarray(np.asarray(sizes, dtype=np.int64).reshape(-1))
        k = sz.size
        out_sizes = np.zeros(max(1, k), np.int64)
        h = C.c_void_p()
        N.check(self.node.lib.sux_buffer_decompress(self.node.h, self.h, offset,
                                                    sz.ctypes.data if k else None, k,
                                                    max_block_size, C.byref(h),
                                                    out_sizes.ctypes.data, _stream(stream)),
                "sux_buffer_decompress")
        return FetchedBuffer(self.node, h, 1), out_sizes[:k].tolist()


def index_file_commit(index_path: str, data_path: str, data_tmp: str | None,
                      lengths) -> tuple[np.ndarray, bool]:
    """IndexShuffleBlockResolver.writeIndexFileAndCommit (host only, no device).  Returns
    (committed lengths, reused an existing consistent pair)."""
    ln = np.ascontiguousarray(lengths, np.int64)
    out = np.zeros(ln.size, np.int64)
    reused = C.c_int32()
    N.check(N.load().sux_index_file_commit(index_path.encode(), data_path.encode(),
                                           None if data_tmp is None else data_tmp.encode(),
                                           ln.ctypes.data if ln.size else None, ln.size,
                                           out.ctypes.data if ln.size else None,
                                           C.byref(reused)), "sux_index_file_commit")
    return out, bool(reused.value)
