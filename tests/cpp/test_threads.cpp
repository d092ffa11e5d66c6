// test_threads.cpp — the plugin's threading model under load: Spark runs
// one task per executor core (config C1 is local[8]) and SparkUCX gives every task thread its own
// UCX worker (UcxNode.java:85-95, getThreadLocalWorker :147-176) whose completions run inside
// that thread's progress() (UcxWorkerWrapper.scala:100-120).  Here 8 host threads, each with its
// own HIP stream (the thread-local worker's analog), drive one node at once:
//   phase 1: every thread runs getWriter(...).write for its own map tasks (the blocking
//            single-map sux_write_map_output) and right away fetches single and batch blocks of
//            them while the other threads are still writing theirs;
//   phase 2: every thread enqueues a batch of map tasks with sux_write_map_outputs (no wait);
//            once all are enqueued every thread fetches its own and another thread's maps — the
//            fetch makes the pending maps of ALL threads progress (publish on completion);
//   phase 3: two threads race to commit the same maps; the first commit wins, bytes unchanged.
// Every fetched block is compared with the CPU oracle (oracle/oracle.c, test infrastructure).
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sparkucx_amd/ucx_shuffle.hpp"
#include "../../oracle/oracle.h"

using namespace sparkucx;

static std::atomic<int> failures{0};
static std::mutex log_mu;
#define EXPECT(cond, ...)                                              \
  do {                                                                 \
    if (!(cond)) {                                                     \
      ++failures;                                                      \
      std::lock_guard<std::mutex> lk(log_mu);                          \
      fprintf(stderr, "FAIL %s:%d: %s  ", __FILE__, __LINE__, #cond);  \
      fprintf(stderr, __VA_ARGS__);                                    \
      fprintf(stderr, "\n");                                           \
    }                                                                  \
  } while (0)

#define HIP_OK(x)                                  \
  do {                                             \
    if ((x) != hipSuccess) {                       \
      fprintf(stderr, "%s failed\n", #x);          \
      exit(2);                                     \
    }                                              \
  } while (0)

namespace {
constexpr int kThreads = 8, kMapsPerThread = 4, R = 64, S = 100, kRpm = 6000;
constexpr int M = kThreads * kMapsPerThread;

struct Want {
  std::vector<uint8_t> data;
  std::vector<int64_t> idx;
};

std::vector<uint8_t> d2h(const void* p, uint64_t n, hipStream_t s) {
  std::vector<uint8_t> h(n);
  if (n) {
    HIP_OK(hipMemcpyAsync(h.data(), p, n, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  return h;
}

// records of map m of shuffle `sid`: single-map writers (shuffle 1) get maps of varying size;
// a batch (shuffle 2) holds kRpm-row maps, only its last map is shorter
uint64_t rows_of(int sid, int m) {
  const uint64_t ragged = kRpm - (uint64_t)((m * 37 + sid * 11) % 900);
  if (sid == 1) return ragged;
  return m % kMapsPerThread == kMapsPerThread - 1 ? ragged : kRpm;
}

Want oracle_map(const o_part& op, int sid, int m, std::vector<uint8_t>* recs_out) {
  const uint64_t n = rows_of(sid, m);
  std::vector<uint8_t> recs(n * S);
  o_gen_terasort(1000 + sid, (uint64_t)m * kRpm, n, recs.data());
  Want w;
  w.data.resize(recs.size());
  w.idx.resize(R + 1);
  std::vector<int64_t> len(R);
  std::vector<uint8_t> be(8 * (R + 1));
  o_write_map(&op, recs.data(), n, S, w.data.data(), len.data(), w.idx.data(), be.data());
  if (recs_out) *recs_out = std::move(recs);
  return w;
}

// fetch (map, [s, e)) through the client on this thread's stream, compare with the oracle
void fetch_and_check(UcxShuffleManager& mgr, int sid, const std::map<int64_t, int>& ids,
                     const std::vector<Want>& want, const std::vector<std::pair<int, std::pair<int, int>>>& blocks,
                     hipStream_t s, int t) {
  struct Collect : BlockFetchingListener {
    std::map<std::string, ManagedBuffer> ok;
    std::vector<std::string> failed;
    void onBlockFetchSuccess(const std::string& id, ManagedBuffer b) override { ok[id] = b; }
    void onBlockFetchFailure(const std::string& id, const std::exception& e) override {
      failed.push_back(id + ": " + e.what());
    }
  } l;
  std::vector<std::string> names;
  for (auto& b : blocks) {
    ShuffleBlockId id{sid, 7000 + b.first, b.second.first, b.second.second,
                      b.second.second - b.second.first > 1};
    names.push_back(id.name());
  }
  UcxShuffleClient client(sid, mgr.ucxNode(), ids);
  client.fetchBlocks("localhost", 0, "exec", names, l, s);
  EXPECT(l.failed.empty(), "thread %d: %zu failures, first %s", t, l.failed.size(),
         l.failed.empty() ? "" : l.failed[0].c_str());
  for (size_t i = 0; i < blocks.size(); ++i) {
    auto it = l.ok.find(names[i]);
    if (it == l.ok.end()) continue;
    const int m = blocks[i].first, a = blocks[i].second.first, e = blocks[i].second.second;
    auto bytes = d2h(it->second.devicePtr(), it->second.size(), s);
    const int64_t lo = want[m].idx[a], hi = want[m].idx[e];
    EXPECT((int64_t)bytes.size() == hi - lo &&
               std::memcmp(bytes.data(), want[m].data.data() + lo, bytes.size()) == 0,
           "thread %d block %s bytes", t, names[i].c_str());
    it->second.release();
  }
}
}  // namespace

int main() {
  std::vector<uint8_t> bounds((R - 1) * 10);
  o_range_bounds_uniform(R, 10, bounds.data());
  sux_partitioner_desc pdesc{SUX_PART_RANGE_BYTES, R, 0, 10, 42, 1, bounds.data()};
  o_part op{1, R, 0, 10, 42, 1, bounds.data()};
  // raw data files (the bytes are checked against the oracle's; the compressed contract has its
  // own test in test_host_mirror.cpp)
  UcxShuffleConf conf(std::map<std::string, std::string>{
      {"spark.shuffle.ucx.memory.preAllocateBuffers", "4k:64,1m:8"},
      {"spark.shuffle.compress", "false"}});
  UcxShuffleManager mgr(conf, /*isDriver=*/false);
  mgr.startUcxNodeIfMissing();
  uint64_t pre = 0;
  check(sux_pool_stats(mgr.ucxNode().native(), nullptr, nullptr, nullptr, &pre), "pool stats");
  EXPECT(pre == 2, "executor preallocated %llu stacks, want 2", (unsigned long long)pre);

  for (int sid : {1, 2}) {
    UcxShuffleHandle h = mgr.registerShuffle(sid, M, pdesc, S);
    std::vector<Want> want(M);
    std::vector<std::vector<uint8_t>> recs(M);
    for (int m = 0; m < M; ++m) want[m] = oracle_map(op, sid, m, &recs[m]);
    std::map<int64_t, int> ids;
    for (int m = 0; m < M; ++m) ids[7000 + m] = m;

    std::atomic<int> enqueued{0};
    std::vector<std::thread> th;
    for (int t = 0; t < kThreads; ++t)
      th.emplace_back([&, t] {
        hipStream_t s;
        HIP_OK(hipSetDevice(0));
        HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const int m0 = t * kMapsPerThread;
        // one device buffer with this thread's maps back to back (kRpm rows apart)
        void* dev = nullptr;
        HIP_OK(hipMalloc(&dev, (size_t)kMapsPerThread * kRpm * S));
        for (int k = 0; k < kMapsPerThread; ++k)
          HIP_OK(hipMemcpyAsync(static_cast<uint8_t*>(dev) + (size_t)k * kRpm * S,
                                recs[m0 + k].data(), recs[m0 + k].size(), hipMemcpyHostToDevice, s));
        if (sid == 1) {
          // phase 1: blocking single-map writers, then fetch own + other threads' maps
          for (int k = 0; k < kMapsPerThread; ++k) {
            UcxShuffleWriter w = mgr.getWriter(h, 7000 + m0 + k, m0 + k);
            w.write(static_cast<uint8_t*>(dev) + (size_t)k * kRpm * S, rows_of(sid, m0 + k), s);
            std::vector<int64_t> len = w.getPartitionLengths();
            for (int p = 0; p < R; ++p)
              EXPECT(len[p] == want[m0 + k].idx[p + 1] - want[m0 + k].idx[p], "map %d len", m0 + k);
          }
          std::vector<std::pair<int, std::pair<int, int>>> bl;
          for (int k = 0; k < kMapsPerThread; ++k) {
            bl.push_back({m0 + k, {t, t + 1}});
            bl.push_back({m0 + k, {3, 3 + 2 * t + 1}});
          }
          fetch_and_check(mgr, sid, ids, want, bl, s, t);
        } else {
          // phase 2: enqueue the whole batch without a wait; the fetch below publishes the
          // maps of every thread that completed (progress on the calling thread)
          const uint64_t n = (uint64_t)(kMapsPerThread - 1) * kRpm +
                             rows_of(sid, m0 + kMapsPerThread - 1);
          check(sux_write_map_outputs(mgr.ucxNode().native(), sid, m0, h.partitioner.get(), dev,
                                      kRpm, n, s),
                "sux_write_map_outputs");
          ++enqueued;
          while (enqueued.load() < kThreads) std::this_thread::yield();
          std::vector<std::pair<int, std::pair<int, int>>> bl;
          for (int k = 0; k < kMapsPerThread; ++k) {
            bl.push_back({m0 + k, {0, R}});
            bl.push_back({(m0 + k + kMapsPerThread) % M, {t, t + 3}});  // another thread's map
          }
          fetch_and_check(mgr, sid, ids, want, bl, s, t);
        }
        HIP_OK(hipStreamSynchronize(s));
        HIP_OK(hipFree(dev));
        HIP_OK(hipStreamDestroy(s));
      });
    for (auto& x : th) x.join();
    // phase 3: two threads race to commit the same maps of a fresh shuffle
    if (sid == 1) {
      UcxShuffleHandle h3 = mgr.registerShuffle(3, 4, pdesc, S);
      std::vector<std::thread> race;
      for (int t = 0; t < 2; ++t)
        race.emplace_back([&, t] {
          hipStream_t s;
          HIP_OK(hipSetDevice(0));
          HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
          for (int m = 0; m < 4; ++m) {
            void* dev = nullptr;
            HIP_OK(hipMalloc(&dev, recs[m].size()));
            HIP_OK(hipMemcpyAsync(dev, recs[m].data(), recs[m].size(), hipMemcpyHostToDevice, s));
            UcxShuffleWriter w = mgr.getWriter(h3, 9000 + m, m);
            w.write(dev, rows_of(sid, m), s);
            HIP_OK(hipStreamSynchronize(s));
            HIP_OK(hipFree(dev));
          }
          HIP_OK(hipStreamDestroy(s));
        });
      for (auto& x : race) x.join();
      std::map<int64_t, int> ids3;
      for (int m = 0; m < 4; ++m) ids3[7000 + m] = m;
      hipStream_t s;
      HIP_OK(hipStreamCreate(&s));
      fetch_and_check(mgr, 3, ids3, want, {{0, {0, R}}, {1, {0, R}}, {2, {5, 9}}, {3, {0, R}}}, s, -1);
      HIP_OK(hipStreamDestroy(s));
      EXPECT(mgr.unregisterShuffle(3), "unregister 3");
    }
    EXPECT(mgr.unregisterShuffle(sid), "unregister %d", sid);
  }
  mgr.stop();
  if (failures) {
    fprintf(stderr, "%d failure(s)\n", failures.load());
    return 1;
  }
  printf("threads ok: %d threads x %d maps, blocking + batched writers, concurrent fetches\n",
         kThreads, kMapsPerThread);
  return 0;
}
