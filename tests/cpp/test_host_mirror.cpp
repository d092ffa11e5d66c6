// test_host_mirror.cpp — the C++ plugin mirror (include/sparkucx_amd/ucx_shuffle.hpp) end to end
// on one GPU, checked against the CPU oracle (oracle/oracle.c, test infrastructure).
// Reads like the reference's own flow: registerShuffle -> getWriter(...).write -> index commit ->
// getReader(...).read / UcxShuffleClient.fetchBlocks -> listener callbacks -> release.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/sparkucx_amd/ucx_shuffle.hpp"
#include "../../oracle/oracle.h"

using namespace sparkucx;

static int failures = 0;
#define EXPECT(cond, ...)                                      \
  do {                                                         \
    if (!(cond)) {                                             \
      ++failures;                                              \
      fprintf(stderr, "FAIL %s:%d: %s  ", __FILE__, __LINE__, #cond); \
      fprintf(stderr, __VA_ARGS__);                            \
      fprintf(stderr, "\n");                                   \
    }                                                          \
  } while (0)

#define HIP_OK(x)                                  \
  do {                                             \
    if ((x) != hipSuccess) {                       \
      fprintf(stderr, "%s failed\n", #x);          \
      exit(2);                                     \
    }                                              \
  } while (0)

static std::vector<uint8_t> d2h(const void* p, uint64_t n) {
  std::vector<uint8_t> h(n);
  if (n && hipMemcpy(h.data(), p, n, hipMemcpyDeviceToHost) != hipSuccess) {
    fprintf(stderr, "hipMemcpy failed\n");
    exit(2);
  }
  return h;
}

int main() {
  const int R = 50, S = 100, M = 4, per = 3000;
  const int counts[M] = {per, per, per, 1700};
  std::vector<uint8_t> bounds((R - 1) * 10);
  o_range_bounds_uniform(R, 10, bounds.data());
  sux_partitioner_desc pdesc{SUX_PART_RANGE_BYTES, R, 0, 10, 42, 1, bounds.data()};
  o_part opart{1, R, 0, 10, 42, 1, bounds.data()};

  // the executor components refuse a map-output writer before initializeExecutor
  // (UcxLocalDiskShuffleExecutorComponents.scala:31-33, IllegalStateException analog)
  {
    UcxShuffleManager m(UcxShuffleConf(std::map<std::string, std::string>{{"spark.shuffle.ucx.gpu.device", "0"},
                                                                     {"spark.shuffle.compress", "false"}}), false);
    UcxLocalDiskShuffleExecutorComponents c(m);
    bool threw = false;
    try {
      c.createMapOutputWriter(1, 1, R);
    } catch (const UcxException& e) {
      threw = e.code() == SUX_ESTATE &&
              std::string(e.what()).find("must be initialized before getting writers") != std::string::npos;
    }
    EXPECT(threw, "a writer before initializeExecutor must throw IllegalStateException-like");
    c.initializeExecutor("app-1", "1");
    EXPECT(c.initialized(), "initializeExecutor starts the node");
    c.createMapOutputWriter(1, 1, R);  // now fine
  }

  // the raw-file half of the contract (spark.shuffle.compress=false); the compressed half, Spark's
  // default, follows below
  UcxShuffleConf conf(std::map<std::string, std::string>{{"spark.shuffle.ucx.memory.minBufferSize", "1k"},
                       {"spark.shuffle.ucx.memory.minAllocationSize", "4"},
                       {"spark.shuffle.ucx.rkeySize", "150"},
                       {"spark.shuffle.compress", "false"}});
  EXPECT(conf.minRegistrationSize() == (4u << 20), "minAllocationSize bare number is MiB");
  EXPECT(conf.metadataBlockSize() == 300, "metadata block = 2 * rkeySize");
  UcxShuffleManager manager(conf, /*isDriver=*/true);
  UcxShuffleHandle h = manager.registerShuffle(7, M, pdesc, S);
  EXPECT(h.desc.directory_bytes == (uint64_t)M * 300, "directory sized by maps (Q1 fix)");

  // map side: inputs on the device, one writer per map task (attempt id 100+i, partition i)
  std::vector<std::vector<uint8_t>> in(M), want_data(M), want_be(M);
  std::vector<std::vector<int64_t>> want_len(M), want_idx(M);
  std::map<int64_t, int> mapIdToBlockIndex;
  uint64_t first = 0;
  for (int i = 0; i < M; ++i) {
    in[i].resize((size_t)counts[i] * S);
    o_gen_terasort(9, first, counts[i], in[i].data());
    void* dev = nullptr;
    HIP_OK(hipMalloc(&dev, in[i].size()));
    HIP_OK(hipMemcpy(dev, in[i].data(), in[i].size(), hipMemcpyHostToDevice));
    UcxShuffleWriter w = manager.getWriter(h, 100 + i, i);
    w.write(dev, counts[i]);
    HIP_OK(hipFree(dev));
    want_data[i].resize(in[i].size());
    want_len[i].resize(R);
    want_idx[i].resize(R + 1);
    want_be[i].resize(8 * (R + 1));
    o_write_map(&opart, in[i].data(), counts[i], S, want_data[i].data(), want_len[i].data(),
                want_idx[i].data(), want_be[i].data());
    EXPECT(w.getPartitionLengths() == want_len[i], "map %d lengths", i);
    EXPECT(manager.shuffleBlockResolver().getIndexFile(7, i, R) == want_be[i], "map %d index", i);
    mapIdToBlockIndex[100 + i] = i;
    first += counts[i];
  }

  // getWriter on a FRESH executor-side manager, with no manual start: the
  // reference's getWriter forces its lazy executor components, whose initializeExecutor starts
  // the node (compat/spark_3_0/UcxShuffleManager.scala:21,46,49,63-72).  The handle comes from
  // the driver; the executor registers the shuffle and builds the partitioner on its own node.
  {
    UcxShuffleManager exec(UcxShuffleConf(std::map<std::string, std::string>{
                               {"spark.shuffle.ucx.gpu.device", "0"},
                               {"spark.shuffle.compress", "false"}}),
                           /*isDriver=*/false);
    void* dev = nullptr;
    HIP_OK(hipMalloc(&dev, in[2].size()));
    HIP_OK(hipMemcpy(dev, in[2].data(), in[2].size(), hipMemcpyHostToDevice));
    UcxShuffleWriter w = exec.getWriter(h, 102, 2);  // the executor's first call of any kind
    w.write(dev, counts[2]);
    HIP_OK(hipFree(dev));
    EXPECT(w.getPartitionLengths() == want_len[2], "fresh executor: map lengths");
    EXPECT(exec.shuffleBlockResolver().getIndexFile(7, 2, R) == want_be[2], "fresh executor: index");
    auto got = exec.getReader(h, 0, R, {{102, 2}}).read();
    EXPECT(got.failures.empty() && got.blocks.size() == 1, "fresh executor: read back");
    if (!got.blocks.empty()) {
      EXPECT(d2h(got.blocks[0].second.devicePtr(), got.blocks[0].second.size()) == want_data[2],
             "fresh executor: map output bytes");
      got.blocks[0].second.release();
    }
    EXPECT(exec.shuffleExecutorComponents().initialized(), "components initialised by getWriter");
    EXPECT(exec.unregisterShuffle(7), "the executor unregisters its copy");
  }

  // reduce side: batch fetch of [10, 23) from every map, through the reader
  {
    UcxShuffleReader reader = manager.getReader(h, 10, 23, mapIdToBlockIndex);
    auto got = reader.read();
    EXPECT(got.failures.empty(), "reader failures: %zu", got.failures.size());
    EXPECT(got.blocks.size() == (size_t)M, "blocks: %zu", got.blocks.size());
    for (auto& kv : got.blocks) {
      ShuffleBlockId b = ShuffleBlockId::parse(kv.first);
      int m = mapIdToBlockIndex[b.mapId];
      int64_t s = want_idx[m][10], e = want_idx[m][23];
      auto bytes = d2h(kv.second.devicePtr(), kv.second.size());
      EXPECT((int64_t)bytes.size() == e - s, "block %s size", kv.first.c_str());
      EXPECT(std::memcmp(bytes.data(), want_data[m].data() + s, bytes.size()) == 0,
             "block %s bytes", kv.first.c_str());
      kv.second.release();
    }
  }

  // single blocks through the client, including failures the reference never reports
  {
    struct Collect : BlockFetchingListener {
      std::map<std::string, std::vector<uint8_t>> ok;
      std::vector<std::string> failed;
      void onBlockFetchSuccess(const std::string& id, ManagedBuffer b) override {
        ok[id] = d2h(b.devicePtr(), b.size());
        b.release();
      }
      void onBlockFetchFailure(const std::string& id, const std::exception&) override {
        failed.push_back(id);
      }
    } l;
    UcxShuffleClient client(7, manager.ucxNode(), mapIdToBlockIndex);
    std::vector<std::string> ids = {"shuffle_7_102_0",  "shuffle_7_100_49", "shuffle_7_103_5_9",
                                    "shuffle_7_999_1",  "bogus_block",      "shuffle_7_101_3"};
    client.fetchBlocks("localhost", 0, "exec-1", ids, l);
    EXPECT(l.failed.size() == 2, "two failures expected, got %zu", l.failed.size());
    auto check_block = [&](const std::string& id, int m, int s, int e) {
      auto it = l.ok.find(id);
      EXPECT(it != l.ok.end(), "missing %s", id.c_str());
      if (it == l.ok.end()) return;
      int64_t a = want_idx[m][s], b = want_idx[m][e];
      EXPECT((int64_t)it->second.size() == b - a &&
                 std::memcmp(it->second.data(), want_data[m].data() + a, b - a) == 0,
             "bytes of %s", id.c_str());
    };
    check_block("shuffle_7_102_0", 2, 0, 1);
    check_block("shuffle_7_100_49", 0, 49, 50);
    check_block("shuffle_7_103_5_9", 3, 5, 9);
    check_block("shuffle_7_101_3", 1, 3, 4);
  }

  // writeIndexFileAndCommit of an externally produced map output (second shuffle)
  {
    UcxShuffleHandle h2 = manager.registerShuffle(8, 2, pdesc, S);
    void* dev = nullptr;
    HIP_OK(hipMalloc(&dev, want_data[1].size()));
    HIP_OK(hipMemcpy(dev, want_data[1].data(), want_data[1].size(), hipMemcpyHostToDevice));
    manager.shuffleBlockResolver().writeIndexFileAndCommit(8, 555, want_len[1], dev,
                                                           want_data[1].size(), 1);
    HIP_OK(hipFree(dev));
    EXPECT(manager.shuffleBlockResolver().getIndexFile(8, 1, R) == want_be[1], "committed index");
    // a mismatching length table is refused
    bool threw = false;
    std::vector<int64_t> bad = want_len[1];
    bad[0] += 100;
    try {
      manager.shuffleBlockResolver().writeIndexFileAndCommit(8, 556, bad, nullptr, 0, 0);
    } catch (const UcxException& e) {
      threw = e.code() == SUX_EINVAL;
    }
    EXPECT(threw, "bad lengths must be refused");
    UcxShuffleReader reader = manager.getReader(h2, 0, R, {{555, 1}});
    auto got = reader.read();
    EXPECT(got.blocks.size() == 1 && got.failures.empty(), "whole-map batch");
    if (!got.blocks.empty()) {
      auto bytes = d2h(got.blocks[0].second.devicePtr(), got.blocks[0].second.size());
      EXPECT(bytes == want_data[1], "whole-map bytes");
      got.blocks[0].second.release();
    }
    // map 0 of shuffle 8 was never committed: its block fails
    UcxShuffleReader r0 = manager.getReader(h2, 0, 1, {{554, 0}});
    EXPECT(r0.read().failures.size() == 1, "uncommitted map must fail");
    EXPECT(manager.unregisterShuffle(8), "unregister");
    EXPECT(!manager.unregisterShuffle(8), "second unregister is false");
  }

  // the JVM flow of a GPU shuffle: the handle carries the row layout (100-byte rows, 10-byte key)
  // and an unsigned-bytes key ordering; map tasks write -> the coordinator's exchange window +
  // completion -> the reader decodes rows and sorts them on the GPU (ExternalSorter's step)
  {
    UcxShuffleHandle h3 = manager.registerShuffle(9, M, pdesc, GpuRowLayout{S, 0, 10}, SUX_SORT_BYTES,
                                                  /*aggregator=*/false);
    std::map<int64_t, int> ids3;
    uint64_t f3 = 0;
    for (int i = 0; i < M; ++i) {
      void* dev = nullptr;
      HIP_OK(hipMalloc(&dev, in[i].size()));
      HIP_OK(hipMemcpy(dev, in[i].data(), in[i].size(), hipMemcpyHostToDevice));
      manager.getWriter(h3, 300 + i, i).write(dev, counts[i]);
      HIP_OK(hipFree(dev));
      ids3[300 + i] = i;
      f3 += counts[i];
    }
    manager.exchangeWindow(9, 0, M);
    manager.exchangeDone(9);
    for (auto range : {std::make_pair(10, 23), std::make_pair(0, R), std::make_pair(49, 50)}) {
      bool gpu = false;
      auto rows = manager.getReader(h3, range.first, range.second, ids3).readRows(nullptr, &gpu);
      // expected: the canonical map-ordered concatenation of the blocks, stably sorted by key
      std::vector<uint8_t> cat;
      for (int m = 0; m < M; ++m)
        cat.insert(cat.end(), want_data[m].begin() + want_idx[m][range.first],
                   want_data[m].begin() + want_idx[m][range.second]);
      std::vector<uint32_t> order(cat.size() / S);
      for (uint32_t k = 0; k < order.size(); ++k) order[k] = k;
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return std::memcmp(&cat[(size_t)a * S], &cat[(size_t)b * S], 10) < 0;
      });
      std::vector<uint8_t> want(cat.size());
      for (size_t k = 0; k < order.size(); ++k)
        std::memcpy(&want[k * S], &cat[(size_t)order[k] * S], S);
      EXPECT(gpu, "rows of [%d, %d) sorted on the GPU", range.first, range.second);
      EXPECT(rows == want, "GPU-sorted rows of [%d, %d) equal the stable key sort",
             range.first, range.second);
    }
    // an aggregating dependency keeps Spark's path: the rows come back in fetch order
    UcxShuffleHandle h4 = h3;
    h4.aggregator = true;
    bool gpu = true;
    auto rows = manager.getReader(h4, 5, 6, ids3).readRows(nullptr, &gpu);
    std::vector<uint8_t> cat;
    for (int m = 0; m < M; ++m)
      cat.insert(cat.end(), want_data[m].begin() + want_idx[m][5], want_data[m].begin() + want_idx[m][6]);
    EXPECT(!gpu && rows == cat, "aggregating reader: fetch-order rows");
    EXPECT(manager.unregisterShuffle(9), "unregister 9");
  }

  // the batch-fetch guard (compat/spark_3_0/UcxShuffleReader.scala:165-187): a non-relocatable
  // serializer gets one ShuffleBlockId per non-empty (map, partition), and the rows are the same
  {
    UcxShuffleHandle h5 = manager.registerShuffle(10, M, pdesc, GpuRowLayout{S, 0, 10}, 0,
                                                  /*aggregator=*/true);
    std::map<int64_t, int> ids5;
    for (int i = 0; i < M; ++i) {
      void* dev = nullptr;
      HIP_OK(hipMalloc(&dev, in[i].size()));
      HIP_OK(hipMemcpy(dev, in[i].data(), in[i].size(), hipMemcpyHostToDevice));
      manager.getWriter(h5, 500 + i, i).write(dev, counts[i]);
      HIP_OK(hipFree(dev));
      ids5[500 + i] = i;
    }
    std::vector<uint8_t> cat;
    for (int m = 0; m < M; ++m)
      cat.insert(cat.end(), want_data[m].begin() + want_idx[m][7], want_data[m].begin() + want_idx[m][31]);
    UcxShuffleReader batch = manager.getReader(h5, 7, 31, ids5);
    EXPECT(batch.fetchContinuousBlocksInBatch() && batch.blockIds().size() == (size_t)M,
           "relocatable serializer: one ShuffleBlockBatchId per map (%zu ids)", batch.blockIds().size());
    EXPECT(batch.blockIds()[0] == "shuffle_10_500_7_31", "batch id %s", batch.blockIds()[0].c_str());
    EXPECT(batch.readRows() == cat, "batch rows");
    UcxShuffleHandle h6 = h5;
    h6.serializerRelocatable = false;  // Java serialization: per-stream headers
    UcxShuffleReader single(manager.ucxNode(), h6, 7, 31, ids5, conf, true);
    size_t nonEmpty = 0;
    for (int m = 0; m < M; ++m)
      for (int r = 7; r < 31; ++r) nonEmpty += want_len[m][r] != 0;
    const auto sids = single.blockIds();
    EXPECT(!single.fetchContinuousBlocksInBatch() && sids.size() == nonEmpty,
           "non-relocatable serializer: %zu per-partition ids, want %zu", sids.size(), nonEmpty);
    bool allSingle = true;
    for (const auto& id : sids) allSingle = allSingle && !ShuffleBlockId::parse(id).batch;
    EXPECT(allSingle, "no ShuffleBlockBatchId without a relocatable serializer");
    EXPECT(single.readRows() == cat, "per-partition rows equal the batch rows");
    // the old fetch protocol, and shouldBatchFetch = false, also fetch per partition
    std::map<std::string, std::string> old = {{"spark.shuffle.compress", "false"},
                                              {"spark.shuffle.useOldFetchProtocol", "true"}};
    EXPECT(!UcxShuffleReader(manager.ucxNode(), h5, 7, 31, ids5, UcxShuffleConf(old), true)
                .fetchContinuousBlocksInBatch(),
           "old fetch protocol: no batch");
    EXPECT(!UcxShuffleReader(manager.ucxNode(), h5, 7, 31, ids5, conf, false)
                .fetchContinuousBlocksInBatch(),
           "shouldBatchFetch false: no batch");
    // bounded delivery: whole rows, chunks of at most 1000 bytes, the same bytes in order
    std::vector<uint8_t> chunked;
    size_t chunks = 0;
    bool whole = true;
    batch.readRowsChunked([&](const uint8_t* p, size_t n) {
      whole = whole && n % S == 0 && n <= 1000;
      chunked.insert(chunked.end(), p, p + n);
      ++chunks;
    }, 1000);
    EXPECT(whole && chunks == (cat.size() + 999) / 1000 && chunked == cat,
           "chunked rows: %zu chunks", chunks);
    EXPECT(manager.unregisterShuffle(10), "unregister 10");
  }

  manager.stop();

  // ---- Spark's default: spark.shuffle.compress=true with the lz4 codec --------
  // The GPU writer commits LZ4Block streams byte-equal to Spark's writers' (so the reader's
  // wrapStream decodes GPU- and Spark-written shuffles alike); the GPU sort decodes before sorting.
  {
    const int BS = 32768;
    auto compress_map = [&](int m, std::vector<uint8_t>& out, std::vector<int64_t>& cix) {
      const size_t runs = R;
      out.resize(want_data[m].size() + (want_data[m].size() / BS + runs + 1) * 21 + runs * 21 + 64);
      cix.resize(R + 1);
      const uint64_t nb = o_lz4_map_outputs(want_data[m].data(), want_idx[m].data(), 1, R, BS,
                                            out.data(), cix.data());
      out.resize(nb);
    };
    std::vector<std::vector<uint8_t>> cdata(M);
    std::vector<std::vector<int64_t>> cidx(M);
    for (int m = 0; m < M; ++m) compress_map(m, cdata[m], cidx[m]);
    UcxShuffleConf zconf;  // every key at Spark's default
    int32_t codec = -1, bs = 0;
    EXPECT(zconf.shuffleCompress() && zconf.compressionCodec() == "lz4" && zconf.gpuCodec(&codec, &bs) &&
               codec == SUX_CODEC_LZ4 && bs == BS,
           "Spark's defaults: lz4, 32k blocks");
    UcxShuffleManager zm(zconf, /*isDriver=*/true);
    UcxShuffleHandle hz = zm.registerShuffle(20, M, pdesc, GpuRowLayout{S, 0, 10}, SUX_SORT_BYTES, false);
    std::map<int64_t, int> idz;
    for (int i = 0; i < M; ++i) {
      void* dev = nullptr;
      HIP_OK(hipMalloc(&dev, in[i].size()));
      HIP_OK(hipMemcpy(dev, in[i].data(), in[i].size(), hipMemcpyHostToDevice));
      UcxShuffleWriter w = zm.getWriter(hz, 700 + i, i);
      w.write(dev, counts[i]);
      HIP_OK(hipFree(dev));
      std::vector<int64_t> clen(R);
      for (int r = 0; r < R; ++r) clen[r] = cidx[i][r + 1] - cidx[i][r];
      EXPECT(w.getPartitionLengths() == clen, "compressed: map %d lengths are the LZ4 streams'", i);
      idz[700 + i] = i;
    }
    // the fetched blocks are the streams Spark's writer would have written
    {
      auto got = zm.getReader(hz, 3, 40, idz).read();
      EXPECT(got.failures.empty() && got.blocks.size() == (size_t)M, "compressed batch fetch");
      for (auto& kv : got.blocks) {
        const int m = idz[ShuffleBlockId::parse(kv.first).mapId];
        auto bytes = d2h(kv.second.devicePtr(), kv.second.size());
        EXPECT(bytes.size() == (size_t)(cidx[m][40] - cidx[m][3]) &&
                   std::memcmp(bytes.data(), cdata[m].data() + cidx[m][3], bytes.size()) == 0,
               "compressed block %s equals lz4-java's stream bytes", kv.first.c_str());
        kv.second.release();
      }
    }
    auto sorted_cat = [&](int lo, int hi) {
      std::vector<uint8_t> cat;
      for (int m = 0; m < M; ++m)
        cat.insert(cat.end(), want_data[m].begin() + want_idx[m][lo], want_data[m].begin() + want_idx[m][hi]);
      std::vector<uint32_t> order(cat.size() / S);
      for (uint32_t k = 0; k < order.size(); ++k) order[k] = k;
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return std::memcmp(&cat[(size_t)a * S], &cat[(size_t)b * S], 10) < 0;
      });
      std::vector<uint8_t> want(cat.size());
      for (size_t k = 0; k < order.size(); ++k) std::memcpy(&want[k * S], &cat[(size_t)order[k] * S], S);
      return std::make_pair(cat, want);
    };
    for (auto range : {std::make_pair(0, R), std::make_pair(12, 13), std::make_pair(20, 37)}) {
      bool gpu = false;
      auto rows = zm.getReader(hz, range.first, range.second, idz).readRows(nullptr, &gpu);
      EXPECT(gpu && rows == sorted_cat(range.first, range.second).second,
             "compressed GPU-written [%d, %d): decoded, then sorted on the GPU", range.first, range.second);
    }
    // non-sorting reader (an aggregator keeps Spark's path): decoded rows in fetch order
    UcxShuffleHandle hza = hz;
    hza.aggregator = true;
    bool gpu = true;
    auto rows = zm.getReader(hza, 5, 30, idz).readRows(nullptr, &gpu);
    EXPECT(!gpu && rows == sorted_cat(5, 30).first, "compressed, unsorted: raw rows in fetch order");
    // a Spark-written compressed shuffle adopted by the resolver, then GPU-sorted (VERDICT r05 weak
    // #2b: the compressed bytes used to be sorted as rows)
    UcxShuffleHandle hs = zm.registerShuffle(21, M, pdesc, GpuRowLayout{S, 0, 10}, SUX_SORT_BYTES, false);
    for (int m = 0; m < M; ++m) {
      void* dev = nullptr;
      HIP_OK(hipMalloc(&dev, cdata[m].size()));
      HIP_OK(hipMemcpy(dev, cdata[m].data(), cdata[m].size(), hipMemcpyHostToDevice));
      std::vector<int64_t> clen(R);
      for (int r = 0; r < R; ++r) clen[r] = cidx[m][r + 1] - cidx[m][r];
      zm.shuffleBlockResolver().writeIndexFileAndCommit(21, 900 + m, clen, dev, cdata[m].size(), m);
      HIP_OK(hipFree(dev));
    }
    std::map<int64_t, int> ids;
    for (int m = 0; m < M; ++m) ids[900 + m] = m;
    for (auto range : {std::make_pair(0, R), std::make_pair(33, 34)}) {
      bool g = false;
      auto r2 = zm.getReader(hs, range.first, range.second, ids).readRows(nullptr, &g);
      EXPECT(g && r2 == sorted_cat(range.first, range.second).second,
             "adopted Spark LZ4 files [%d, %d): decoded, then sorted", range.first, range.second);
    }
    // per-partition blocks of a non-relocatable serializer decode one stream each, same rows
    UcxShuffleHandle hn = hs;
    hn.serializerRelocatable = false;
    hn.aggregator = true;
    UcxShuffleReader rn(zm.ucxNode(), hn, 0, R, ids, zconf, true);
    EXPECT(!rn.fetchContinuousBlocksInBatch() && rn.readRows() == sorted_cat(0, R).first,
           "compressed per-partition blocks");
    // another codec: Spark's writer (the GPU cannot restate it); its streams concatenate
    UcxShuffleConf snappy(std::map<std::string, std::string>{
        {"spark.io.compression.codec", "org.apache.spark.io.SnappyCompressionCodec"}});
    EXPECT(snappy.compressionCodec() == "snappy" && snappy.codecConcatenation() &&
               !snappy.gpuCodec(&codec, &bs),
           "snappy: no GPU writer, concatenation supported");
    bool threw = false;
    try {
      UcxShuffleManager sm(snappy, true);
      UcxShuffleHandle hh = sm.registerShuffle(22, 1, pdesc, S);
      sm.getWriter(hh, 1, 0);
    } catch (const UcxException& e) {
      threw = e.code() == SUX_EINVAL;
    }
    EXPECT(threw, "getWriter under snappy is Spark's writer (EINVAL here)");
    UcxShuffleConf enc(std::map<std::string, std::string>{{"spark.io.encryption.enabled", "true"}});
    EXPECT(!enc.gpuCodec(&codec, &bs), "encrypted shuffle streams: Spark's writer");
    zm.stop();
  }

  // spark.shuffle.ucx.gpu.tuning.<field> reaches the node's tuning table; a value outside a
  // field's set is rejected when the node starts
  {
    UcxShuffleConf tc(std::map<std::string, std::string>{
        {"spark.shuffle.ucx.gpu.tuning.scatter_kernel", "7"},
        {"spark.shuffle.ucx.gpu.tuning.small_kernel", "2"}});
    UcxNode node(tc, /*isDriver=*/false);
    sux_tuning t;
    EXPECT(sux_node_get_tuning(node.native(), &t) == SUX_OK && t.scatter_kernel == 7 &&
               t.small_kernel == 2 && t.hist_kernel == 0,
           "tuning keys reach the node");
    node.check();  // nothing ran: the device error word is clear
    bool threw = false;
    try {
      UcxNode bad(UcxShuffleConf(std::map<std::string, std::string>{
                      {"spark.shuffle.ucx.gpu.tuning.scatter_chunk", "333"}}),
                  false);
    } catch (const UcxException& e) {
      threw = e.code() == SUX_EINVAL;
    }
    EXPECT(threw, "an out-of-set tuning value is EINVAL");
  }
  if (failures) {
    fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  printf("host mirror ok\n");
  return 0;
}
