// sux_api.cpp — C-ABI of libsparkucx_amd.so (include/sparkucx_amd.h).
//
// Host runtime around the gfx950 kernels: node lifecycle (UcxNode), device memory pool
// (MemoryPool/RegisteredMemory), per-shuffle directory (driver metadata table), map commit
// (CommonUcxShuffleBlockResolver), fetch (UcxShuffleClient + callbacks) and the RCCL exchange.
// No C++ exception crosses the boundary: every entry point is wrapped in guard().
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <dirent.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <atomic>
#include <climits>
#include <initializer_list>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/sparkucx_amd.h"
#include "sux_internal.h"

// ============================================================================================
// errors
// ============================================================================================
namespace {
thread_local std::string g_err;

struct SuxError {
  int code;
  std::string msg;
};

[[noreturn]] void raise(int code, const std::string& msg) { throw SuxError{code, msg}; }

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) raise(SUX_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) raise(SUX_ECOMM, std::string(what) + ": " + ncclGetErrorString(r));
  // RCCL's internal HIP calls can leave a stale error in the thread's last-error slot (seen
  // after a communicator's init/teardown: "invalid device ordinal"); our kernel launches check
  // hipGetLastError(), so it must not survive a successful RCCL call
  (void)hipGetLastError();
}
// The all-to-all of every exchange: per peer, the byte range [sd[h], sd[h] + sc[h]) of `send` goes
// to peer h and [rd[h], rd[h] + rc[h]) of `recv` arrives from it, as grouped ncclSend/ncclRecv
// pieces of at most kA2aPiece bytes.  ncclAllToAllv itself is not used: the RCCL that torch
// ships (2.26.6) delivers only the first half of a 1.68 GB per-peer count (torch's own
// all_to_all_single shows it too; 0.84 GB arrives whole — tools/a2a_probe.py,
// profiles/r04_f/a2a_probe.txt).  Both sides of a pair cut the same count the same way, so the
// pieces pair up in order without any agreement between ranks.
constexpr size_t kA2aPiece = size_t(256) << 20;
void all_to_all_pieces(const uint8_t* send, const uint64_t* sc, const uint64_t* sd, uint8_t* recv,
                       const uint64_t* rc, const uint64_t* rd, int W, ncclComm_t comm,
                       hipStream_t s) {
  nccl_check(ncclGroupStart(), "ncclGroupStart");
  ncclResult_t r = ncclSuccess;
  for (int h = 0; h < W && r == ncclSuccess; ++h) {
    for (uint64_t o = 0; o < sc[h] && r == ncclSuccess; o += kA2aPiece)
      r = ncclSend(send + sd[h] + o, std::min<uint64_t>(kA2aPiece, sc[h] - o), ncclUint8, h, comm, s);
    for (uint64_t o = 0; o < rc[h] && r == ncclSuccess; o += kA2aPiece)
      r = ncclRecv(recv + rd[h] + o, std::min<uint64_t>(kA2aPiece, rc[h] - o), ncclUint8, h, comm, s);
  }
  const ncclResult_t e = ncclGroupEnd();
  nccl_check(r, "ncclSend/ncclRecv");
  nccl_check(e, "ncclGroupEnd(all-to-all)");
}

// A failed check throws SuxError; the message expression is evaluated only then (some checks run
// once per block of a fetch).
#define require(ok, code, ...)                    \
  do {                                            \
    if (!(ok)) raise((code), (__VA_ARGS__));      \
  } while (0)

template <class F>
int guard(F&& f) {
  // the HIP runtime's per-thread last error is shared with every other library in the process
  // (RCCL, torch): a stale one would be taken for a failed launch of ours (hipGetLastError after
  // each launch), so every entry point starts clean
  (void)hipGetLastError();
  try {
    f();
    return SUX_OK;
  } catch (const SuxError& e) {
    g_err = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "host allocation failed";
    return SUX_ENOMEM;
  } catch (const std::exception& e) {
    g_err = e.what();
    return SUX_EINVAL;
  } catch (...) {
    g_err = "unknown error";
    return SUX_EINVAL;
  }
}
}  // namespace

// ============================================================================================
// kernel timing (sux_set_kernel_timing / sux_kernel_times)
// ============================================================================================
namespace sux {
struct Timer {
  std::mutex mu;
  bool enabled = false;
  struct Rec {
    int slot;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> spare;
  hipEvent_t open[kNumSlots] = {};
  const char* variant[kNumSlots] = {};

  hipEvent_t get() {
    if (!spare.empty()) {
      hipEvent_t e = spare.back();
      spare.pop_back();
      return e;
    }
    hipEvent_t e;
    hip_check(hipEventCreate(&e), "hipEventCreate");
    return e;
  }
  ~Timer() {
    for (auto& r : recs) {
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
    for (auto e : spare) (void)hipEventDestroy(e);
  }
};

void timer_begin(Timer* t, int slot, hipStream_t s) {
  if (!t || !t->enabled) return;
  std::lock_guard<std::mutex> lk(t->mu);
  hipEvent_t e = t->get();
  (void)hipEventRecord(e, s);
  t->open[slot] = e;
}

void timer_note(Timer* t, int slot, const char* kernel) {
  if (!t || slot < 0 || slot >= kNumSlots) return;
  std::lock_guard<std::mutex> lk(t->mu);
  t->variant[slot] = kernel;
}

void timer_end(Timer* t, int slot, hipStream_t s) {
  if (!t || !t->enabled) return;
  std::lock_guard<std::mutex> lk(t->mu);
  if (!t->open[slot]) return;
  hipEvent_t e = t->get();
  (void)hipEventRecord(e, s);
  t->recs.push_back({slot, t->open[slot], e});
  t->open[slot] = nullptr;
}
}  // namespace sux

// ============================================================================================
// device memory pool — MemoryPool.java semantics on HBM
// ============================================================================================
namespace {
struct PoolBuf {
  uint8_t* ptr = nullptr;
  uint64_t cap = 0;  // size class
};

class DevicePool {
 public:
  DevicePool(uint64_t min_buf, uint64_t min_alloc) : min_buf_(min_buf), min_alloc_(min_alloc) {}
  ~DevicePool() {
    for (void* p : allocations_) (void)hipFree(p);
  }

  // MemoryPool.roundUpToTheNextPowerOf2 (:137-151) up to minAllocationSize.  Above it the class
  // is the next multiple of minAllocationSize (deliberate divergence: map outputs and receive
  // buffers run to GBs, where power-of-two classes would leave up to half of the HBM idle).
  uint64_t size_class(uint64_t n) const {
    if (n < min_buf_) return min_buf_;
    if (n > min_alloc_) return (n + min_alloc_ - 1) / min_alloc_ * min_alloc_;
    uint64_t c = 1;
    while (c < n) c <<= 1;
    return c;
  }

  // Cap on the bytes the pool may hold in device allocations (sux_conf.pool_limit_mib; 0 = none).
  // Past it get() fails with SUX_ENOMEM exactly like a failed hipMalloc, so the HBM-capacity
  // fallback (spill to Spark's files) can be exercised without filling 288 GB.
  void set_limit(uint64_t bytes) { limit_ = bytes; }

  // Returns every free buffer that is a whole allocation of its own (classes >= minAllocationSize)
  // to the device: after a spill, the memory can serve a different size class.  Slab-allocated
  // small classes stay (their allocation is shared).  Returns the bytes freed.
  uint64_t trim() {
    std::lock_guard<std::mutex> lk(mu_);
    uint64_t freed = 0;
    for (auto& kv : stacks_) {
      if (kv.first < min_alloc_) continue;
      for (const PoolBuf& b : kv.second.free) {
        auto it = std::find(allocations_.begin(), allocations_.end(), (void*)b.ptr);
        if (it == allocations_.end()) continue;  // part of a preallocated slab
        (void)hipFree(b.ptr);
        allocations_.erase(it);
        allocated_ -= b.cap;
        freed += b.cap;
      }
      kv.second.free.erase(std::remove_if(kv.second.free.begin(), kv.second.free.end(),
                                          [&](const PoolBuf& b) {
                                            return std::find(allocations_.begin(), allocations_.end(),
                                                             (void*)b.ptr) == allocations_.end();
                                          }),
                           kv.second.free.end());
    }
    return freed;
  }

  // MemoryPool.get (:153-162) + AllocatorStack.get (:52-82): LIFO reuse, slab-allocate classes
  // below minAllocationSize in one registration (preallocate :89-114).
  PoolBuf get(uint64_t n) {
    uint64_t cls = size_class(n ? n : 1);
    std::lock_guard<std::mutex> lk(mu_);
    auto& st = stacks_[cls];
    st.requests++;
    requests_++;
    if (st.free.empty()) {
      if (cls < min_alloc_) {
        uint64_t count = min_alloc_ / cls;
        uint8_t* p = alloc(count * cls);
        for (uint64_t i = 0; i < count; ++i) st.free.push_back(PoolBuf{p + i * cls, cls});
        st.preallocs++;
      } else {
        st.free.push_back(PoolBuf{alloc(cls), cls});
      }
      st.allocs++;
    }
    PoolBuf b = st.free.back();
    st.free.pop_back();
    return b;
  }

  // MemoryPool.put (:164-168)
  void put(const PoolBuf& b) {
    if (!b.ptr) return;
    std::lock_guard<std::mutex> lk(mu_);
    stacks_[b.cap].free.push_back(b);
  }

  // AllocatorStack.preallocate (:89-114): `count` buffers of one class in ONE allocation, the
  // total capped below 2^31 bytes like the reference's direct-buffer limit.  The class is the
  // size rounded as get() rounds it (the reference keys the stack by the raw size, so a size
  // that is not a power of two is never handed out again; here it is).
  void preallocate(uint64_t size, uint64_t count) {
    const uint64_t cls = size_class(size ? size : 1);
    if (cls * count > (uint64_t)INT32_MAX) count = (uint64_t)INT32_MAX / cls;
    if (count == 0) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto& st = stacks_[cls];
    uint8_t* p = alloc(cls * count);
    for (uint64_t i = 0; i < count; ++i) st.free.push_back(PoolBuf{p + i * cls, cls});
    st.preallocs++;
    st.allocs++;
    preallocs_++;
  }

  void stats(uint64_t* bytes, uint64_t* requests, uint64_t* allocs, uint64_t* preallocs) {
    std::lock_guard<std::mutex> lk(mu_);
    if (bytes) *bytes = allocated_;
    if (requests) *requests = requests_;
    if (allocs) *allocs = allocations_.size();
    if (preallocs) *preallocs = preallocs_;
  }

 private:
  uint8_t* alloc(uint64_t bytes) {  // caller holds mu_
    void* p = nullptr;
    if (limit_ && allocated_ + bytes > limit_)
      raise(SUX_ENOMEM, "device pool limit: " + std::to_string(allocated_) + " + " +
                            std::to_string(bytes) + " bytes > " + std::to_string(limit_));
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) raise(SUX_ENOMEM, "hipMalloc(" + std::to_string(bytes) + ") failed");
    allocations_.push_back(p);
    allocated_ += bytes;
    return static_cast<uint8_t*>(p);
  }
  struct Stack {
    std::vector<PoolBuf> free;
    uint64_t requests = 0, allocs = 0, preallocs = 0;
  };
  uint64_t min_buf_, min_alloc_, limit_ = 0;
  std::mutex mu_;
  std::map<uint64_t, Stack> stacks_;
  std::vector<void*> allocations_;
  uint64_t allocated_ = 0, requests_ = 0, preallocs_ = 0;
};

// Pinned host staging for index read-backs (reused; freed with the node).
class HostPool {
 public:
  ~HostPool() {
    for (auto& kv : free_)
      for (void* p : kv.second) (void)hipHostFree(p);
  }
  std::pair<void*, uint64_t> get(uint64_t n) {
    uint64_t cls = 4096;
    while (cls < n) cls <<= 1;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto& v = free_[cls];
      if (!v.empty()) {
        void* p = v.back();
        v.pop_back();
        return {p, cls};
      }
    }
    void* p = nullptr;
    hip_check(hipHostMalloc(&p, cls, hipHostMallocDefault), "hipHostMalloc(index staging)");
    return {p, cls};
  }
  void put(std::pair<void*, uint64_t> b) {
    if (!b.first) return;
    std::lock_guard<std::mutex> lk(mu_);
    free_[b.second].push_back(b.first);
  }

 private:
  std::mutex mu_;
  std::map<uint64_t, std::vector<void*>> free_;
};

// A HostPool block, returned on every exit path (callers sync the stream that reads it first).
struct HostLease {
  HostPool& hp;
  std::pair<void*, uint64_t> b;
  HostLease(HostPool& p, uint64_t n) : hp(p), b(p.get(n)) {}
  ~HostLease() { hp.put(b); }
  HostLease(const HostLease&) = delete;
  HostLease& operator=(const HostLease&) = delete;
};

struct Event {  // one completion event, shared by a write job and a thread that waits on it
  hipEvent_t e = nullptr;
  Event() { hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate"); }
  ~Event() { (void)hipEventDestroy(e); }
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
};

// A device buffer shared by several map slots (one batch of map outputs, or one exchange's
// receive buffer); the last reference returns it to the pool.  A slab without a pool wraps
// memory the caller owns (sux_adopt_map_outputs) and frees nothing.  `ready` (receive buffers)
// fires when the exchange that fills it has completed on its stream.
struct Slab {
  DevicePool* pool = nullptr;
  PoolBuf buf;
  PoolBuf aux;  // the device index tables of the slab's maps (world-1 writes), freed with it
  std::shared_ptr<Event> ready;
  Slab(DevicePool* p, PoolBuf b) : pool(p), buf(b) {}
  ~Slab() {
    if (pool) {
      pool->put(buf);
      pool->put(aux);
    }
  }
  Slab(const Slab&) = delete;
  Slab& operator=(const Slab&) = delete;
};

// per-map directory slot: the analog of the 300-byte driver descriptor (DriverMetadata,
// UcxWorkerWrapper.scala:27-65) plus the index file it points at.  Where the map's bytes live:
//   - own maps, map-major (world 1, adopted or committed outputs): Spark's data file at
//     slab + off;
//   - own maps written at world > 1: the batch slab is peer-major [peer h][map][h's partitions],
//     so the map's range for peer h starts at slab + seg[h] (seg has world entries);
//   - own maps spilled to Spark's files (HBM fallback): spill_data / spill_index;
//   - after an exchange: this rank's owned range of the map at rslab + recv_off (remote maps,
//     and own maps when the exchange loops back through the transport).
struct MapSlot {
  bool present = false;
  bool pending = false;  // enqueued by a write job that has not completed yet
  bool sent = false;     // own map: its ranges went out in an exchange
  int32_t owner = -1;
  int32_t batch = -1;    // own maps: the batch (exchange piece) the map belongs to
  std::shared_ptr<Slab> slab;  // local maps: the device buffer holding the data file
  uint64_t off = 0;            // byte offset of this map's data file in the slab (map-major)
  std::vector<uint64_t> seg;   // per peer: offset of the map's range for that peer in the slab
  uint64_t bytes = 0;
  std::vector<int64_t> index;  // R+1 cumulative offsets (the index file, native order)
  // adopted map outputs (world 1): the caller's device index table; the host copy above is made
  // on first use (host_index) — resolves read only the entries they need, on the device
  const int64_t* d_index = nullptr;
  std::shared_ptr<Slab> rslab; // receive buffer holding this rank's owned range of the map
  uint64_t recv_off = 0;       // offset of that range in rslab
  // after an exchange, per rank h: where h serves its owned range of this map — an index into
  // Shuffle::serve_desc (h's batch slab or receive buffer) and the range's offset there; lets
  // any rank read any block (a peer read over xGMI, the reference's one-sided GET)
  std::vector<std::pair<int32_t, uint64_t>> serve;
  std::string spill_data, spill_index;  // spilled: Spark's data + index files
  uint8_t* data() const { return slab ? slab->buf.ptr + off : nullptr; }
  bool spilled() const { return !spill_data.empty(); }
};

// The map's index table on the host: an adopted map's is read back from the device on first use.
const std::vector<int64_t>& host_index(MapSlot& sl, int R) {
  if (sl.index.empty() && sl.d_index) {
    sl.index.resize((size_t)R + 1);
    hip_check(hipMemcpy(sl.index.data(), sl.d_index, 8 * ((size_t)R + 1), hipMemcpyDeviceToHost),
              "index read-back");
  }
  return sl.index;
}

// One sux_write_map_outputs / sux_adopt_map_outputs call in flight: published by progress()
// once `done` has fired.
struct WriteJob {
  int32_t first = 0;
  uint32_t maps = 0;
  uint64_t rpm = 0, n = 0;
  int32_t world = 1;             // > 1: the slab is peer-major over this many peers
  int32_t batch = -1;            // batch id of its maps (map-major at world > 1: one per map)
  std::vector<uint8_t> claimed;  // maps of the batch this job publishes
  std::shared_ptr<Slab> slab;
  PoolBuf ws;
  std::pair<void*, uint64_t> hidx{nullptr, 0};  // pinned copy of the batch's index tables
  const int64_t* dindex = nullptr;  // adopted at world 1: the index tables stay on the device
  uint32_t rs = 0;                  // (and the maps' sizes come from their record counts)
  // compressed shuffle (sux_shuffle_set_codec): the maps are packed back to back in the slab,
  // map k starting where map k - 1's compressed data file ends
  bool packed = false;
  std::shared_ptr<Event> done;
};

struct Shuffle {
  int32_t id = 0, num_maps = 0, R = 0, rec_size = 0;
  // spark.shuffle.compress with the lz4 codec (sux_shuffle_set_codec): the maps the node writes
  // are committed as lz4-java LZ4BlockOutputStream streams of codec_block-byte chunks
  int32_t codec = SUX_CODEC_NONE, codec_block = 0;
  std::vector<MapSlot> maps;
  std::vector<uint8_t> directory;  // num_maps * metadata_block_size bytes (big-endian fields)
  std::vector<std::unique_ptr<WriteJob>> jobs;
  int busy = 0;        // jobs taken out of `jobs` by a thread that is waiting on them
  int submitting = 0;  // writes that claimed slots and have not queued their job yet
  bool exchanging = false;
  // sux_resolve_blocks handed out raw device addresses of this shuffle's map outputs: callers
  // read them without holding a reference, so its slabs are never spilled (spill_some) until
  // the shuffle is unregistered
  bool zero_copy = false;
  int32_t next_batch = 0;
  // exchanges enqueued and not yet waited for (sux_exchange_wait): their completion events and,
  // with the IPC transport, whether the closing all-gather (every peer finished its pulls) is due
  std::vector<std::shared_ptr<Event>> xfers;
  std::vector<PoolBuf> xfer_aux;                      // their copy descriptors (IPC pulls)
  std::vector<std::pair<void*, uint64_t>> xfer_host;  // and the descriptors' pinned staging
  bool ack_due = false;
  // collective host all-gathers of this shuffle so far: with the shuffle id they tag each one
  // (every rank issues them in the same order), so a control plane can match contributions
  uint32_t gathers = 0;
  std::map<std::string, void*> ipc_bases;  // opened peer allocations (64-byte handle -> base)
  std::vector<std::string> serve_desc;     // IPC descriptors of the buffers peers serve from
  std::map<std::string, int32_t> serve_idx;
};

int32_t owner_lo(int32_t h, int32_t R, int32_t G) { return (int32_t)(((int64_t)h * R) / G); }
// First partition of peer h under an ownership table (nullptr = the equal split).
int32_t own_lo(const int32_t* own, int32_t h, int32_t R, int32_t G) {
  return own ? own[h] : owner_lo(h, R, G);
}
// An ownership table is W + 1 rising bounds from 0 to R.
void check_ownership(int32_t W, int32_t R, const int32_t* own) {
  require(own[0] == 0 && own[W] == R, SUX_EINVAL, "ownership must run from 0 to R");
  for (int h = 0; h < W; ++h)
    require(own[h] <= own[h + 1], SUX_EINVAL, "ownership bounds must not fall");
}
}  // namespace

struct sux_node {
  sux_conf conf{};
  bool is_driver = false;
  ncclComm_t comm = nullptr;
  // the all-to-alls' own communicator (ncclCommSplit of `comm`, made on first use by
  // sux_exchange_group_post): the index all-gather of launch group k and the all-to-all of group
  // k - 1 then run on two streams at once without sharing one communicator's ordering
  ncclComm_t comm_x = nullptr;
  std::unique_ptr<DevicePool> pool;
  HostPool hpool;
  sux::Timer timer;
  std::mutex mu;
  std::condition_variable cv;  // a write job was published (Shuffle::jobs/busy/submitting moved)
  std::map<int32_t, std::unique_ptr<Shuffle>> shuffles;
  std::map<void*, std::pair<void*, std::string>> ipc_bases;  // sux_ipc_open: pointer -> (base, handle)
  // every peer allocation this process has mapped (the exchange, the serve path, sux_ipc_open):
  // mapped base -> (64-byte handle, references taken) — see ipc_open_fresh
  std::mutex ipc_mu;
  std::map<void*, std::pair<std::string, int>> ipc_maps;
  // allocations this process exported (export_ipc): base -> (the allocation's buffer id, size,
  // handle).  ONE handle per live allocation: the runtime may hand out a new handle per
  // hipIpcGetMemHandle call (hsa_amd_ipc_memory_create: "repeated calls for the same allocation
  // may ... return unique handles"), and an importer that opens two handles of one allocation
  // gets one mapping under two keys — which ipc_open_fresh must be able to read as "the exporter
  // freed the old allocation" (the IPC open failure of round 3)
  struct IpcExport {
    unsigned long long id;
    size_t size;
    uint8_t handle[64];
  };
  std::mutex export_mu;
  std::map<void*, IpcExport> ipc_exports;
  // sux_exchange_group_post tickets not yet issued or discarded (freed by sux_node_destroy)
  std::set<sux_xticket*> tickets;
  // live partitioners and pooled buffers of this node: sux_node_destroy orphans them (their
  // node pointer cleared), so a handle released after its node — a garbage-collected wrapper,
  // a JVM finalizer — never dereferences the freed node (a partitioner destroyed late used to
  // bind the freed node's device: hipSetDevice(garbage) left "invalid device ordinal" behind)
  std::mutex live_mu;
  std::set<sux_partitioner*> live_parts;
  std::set<sux_buffer*> live_bufs;
  // sux_node_set_ownership: which contiguous partition range each peer owns in the stateless
  // group calls (peer-major partition, exchange_group / post / issue, pull) for groups of
  // own_R partitions among own_W peers; empty = the equal split
  int32_t own_W = 0, own_R = 0;
  std::vector<int32_t> own;
  int32_t* d_own = nullptr;  // device copy (own_W + 1 int32)
  const int32_t* own_host(int W, int R) const {
    return (!own.empty() && own_W == W && own_R == R) ? own.data() : nullptr;
  }
  const int32_t* own_dev(int W, int R) const {
    return (!own.empty() && own_W == W && own_R == R) ? d_own : nullptr;
  }
  sux_allgather_fn boot = nullptr;   // host all-gather of the embedding runtime
  void* boot_ctx = nullptr;
  sux_tuning tuning{};               // all zero = measured defaults (resolve_tuning)
  std::string spill_dir;             // spark.local.dir analog: HBM-capacity fallback (sux_node_set_spill_dir)
  uint64_t spills = 0;               // map outputs spilled so far
  uint32_t* d_err = nullptr;         // device error word (sux::kErr* bits), sux_node_check
  // sux_partition_maps_pipelined: two map streams, their group workspaces, fork/join events
  hipStream_t pipe[2] = {nullptr, nullptr};
  PoolBuf pipe_ws[2];
  hipEvent_t pipe_ev[3] = {nullptr, nullptr, nullptr};
  uint32_t pipe_next = 0;            // round robin of sux_write_map_outputs batches
  std::mutex pipe_mu;                // guards the above and every fork/join on them

  void make_pipe() {  // pipe_mu held
    for (hipStream_t& p : pipe)
      if (!p) hip_check(hipStreamCreateWithFlags(&p, hipStreamNonBlocking), "map stream");
    for (hipEvent_t& e : pipe_ev)
      if (!e) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "map event");
  }
  // split mode of sux_partition_maps_pipelined: [0] K1 on `cus` CUs, [1] K2 + K3 on the rest;
  // split_ev [0, 1] K1 done per workspace slot, [2, 3] K3 done per slot.  pipe_mu held.
  hipStream_t pipe_split[2] = {nullptr, nullptr};
  int pipe_split_cus = 0;
  hipEvent_t split_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  void make_split(int cus);
  // sux_sort_records: the side stream of the large-bucket launches and its fork / join events;
  // sort_mu held while a sort enqueues on them
  hipStream_t sort_side = nullptr;
  hipEvent_t sort_ev[2] = {nullptr, nullptr};
  std::mutex sort_mu;
  int cus = 0;  // the device's CU count (device_cus)
  int device_cus();

  void bind() { hip_check(hipSetDevice(conf.device), "hipSetDevice"); }

  // NULL = the HIP null stream (torch's default stream).  Per-task-thread streams, the analog
  // of UcxNode.getThreadLocalWorker (UcxNode.java:147-176), are passed in by the caller
  // (e.g. hipStreamPerThread from a JNI task thread).
  hipStream_t stream(void* s) { return static_cast<hipStream_t>(s); }

  Shuffle& shuffle(int32_t id) {
    auto it = shuffles.find(id);
    require(it != shuffles.end(), SUX_ENOENT, "unknown shuffle " + std::to_string(id));
    return *it->second;
  }
};

struct sux_partitioner {
  sux_node* node = nullptr;  // nullptr once the node is destroyed (sux_node_destroy orphans it)
  int device = 0;            // the node's device: a partitioner destroyed after its node frees here
  sux_partitioner_desc desc{};
  sux::PartDev pd{};
  void* d_bounds = nullptr;
  void* d_lut = nullptr;
};

struct sux_buffer {
  sux_node* node = nullptr;  // nullptr once the node is destroyed (its pool freed the memory)
  PoolBuf buf;
  PoolBuf aux;  // copy descriptors
  uint64_t size = 0;
  std::atomic<int32_t> refs{1};
};

// ============================================================================================
// helpers
// ============================================================================================
namespace {
void check_record_size(uint32_t rs) {
  require(rs >= 4 && rs <= (uint32_t)sux::kMaxRecordSize && rs % 4 == 0, SUX_EINVAL,
          "record_size must be a multiple of 4 in [4, 4096], got " + std::to_string(rs));
}

void check_key_fits(const sux_partitioner* p, uint32_t rs) {
  require(p->desc.key_offset >= 0 && (uint64_t)p->desc.key_offset + p->desc.key_len <= rs,
          SUX_EINVAL, "key [" + std::to_string(p->desc.key_offset) + ", +" +
                          std::to_string(p->desc.key_len) + ") does not fit a " +
                          std::to_string(rs) + "-byte record");
}

void store_be64(uint8_t* p, uint64_t v) {
  for (int k = 0; k < 8; ++k) p[k] = (uint8_t)(v >> (56 - 8 * k));
}
void store_be32(uint8_t* p, uint32_t v) {
  for (int k = 0; k < 4; ++k) p[k] = (uint8_t)(v >> (24 - 8 * k));
}

// Descriptor of one committed map, written into its directory slot (big-endian like the
// reference's putLong/putInt, CommonUcxShuffleBlockResolver.scala:80-87):
// |u64 index dev addr|u64 data dev addr|i32 owner rank|i32 R|u64 data bytes| = 32 bytes

void publish_slot(sux_node* n, Shuffle& sh, int32_t m, uint64_t index_addr) {
  MapSlot& s = sh.maps[m];
  const uint64_t blk = n->conf.metadata_block_size;  // >= kSlotBytes (checked at node create)
  uint8_t* d = sh.directory.data() + (uint64_t)m * blk;
  store_be64(d, index_addr);
  store_be64(d + 8, (uint64_t)(uintptr_t)s.data());
  store_be32(d + 16, (uint32_t)s.owner);
  store_be32(d + 20, (uint32_t)sh.R);
  store_be64(d + 24, s.bytes);
}

// The device error word after a job's kernels completed: a bounded in-kernel wait that timed out
// (the turn-taking small-record scatter, sux::kErrTurnTimeout) stopped without writing all of its
// records.  Returns the word and clears it.
uint32_t take_device_err(sux_node* node) {
  uint32_t w = 0;
  hip_check(hipMemcpy(&w, node->d_err, sizeof w, hipMemcpyDeviceToHost), "read error word");
  if (w) hip_check(hipMemset(node->d_err, 0, sizeof w), "clear error word");
  return w;
}

// Jobs whose kernels reported a device error: their maps are not published (the writes may be
// retried, as after a failed launch); the pool buffers go back.  Called with the node lock held.
[[noreturn]] void reject_jobs(sux_node* node, Shuffle& sh, std::vector<std::unique_ptr<WriteJob>>& jobs,
                              uint32_t w) {
  std::string maps;
  for (auto& j : jobs) {
    if (!j) continue;
    for (uint32_t k = 0; k < j->maps; ++k)
      if (j->claimed[k]) sh.maps[j->first + k].pending = false;
    maps += " [" + std::to_string(j->first) + ", " + std::to_string(j->first + (int32_t)j->maps) + ")";
    node->pool->put(j->ws);
    node->hpool.put(j->hidx);
    j.reset();
  }
  node->cv.notify_all();
  char b[16];
  std::snprintf(b, sizeof b, "%x", w);
  raise(SUX_EHIP, std::string("device error word 0x") + b +
                      ": a kernel stopped before writing all records; map outputs of maps" + maps +
                      " were not published");
}

// A completed write job's maps get their slots: index tables from the pinned read-back, the
// data location (map-major offset, or per-peer segments of a peer-major slab) and the batch.
void publish_job(sux_node* node, Shuffle& sh, WriteJob& j) {
  const int R = sh.R, W = j.world;
  if (j.dindex) {  // adopted at world 1: no host copy of the index tables
    for (uint32_t k = 0; k < j.maps; ++k) {
      if (!j.claimed[k]) continue;
      MapSlot& slot = sh.maps[j.first + k];
      slot.pending = false;
      slot.present = true;
      slot.sent = false;
      slot.owner = node->conf.rank;
      slot.slab = j.slab;
      slot.batch = j.batch;
      slot.off = (uint64_t)k * j.rpm * (uint64_t)j.rs;
      const uint64_t recs = std::min<uint64_t>(j.rpm, j.n - (uint64_t)k * j.rpm);
      slot.bytes = recs * j.rs;
      slot.index.clear();
      slot.d_index = j.dindex + (uint64_t)k * (R + 1);
      slot.rslab.reset();
      slot.seg.assign(1, slot.off);  // world 1: the one peer's range starts at the data file
      publish_slot(node, sh, j.first + (int32_t)k, (uint64_t)(uintptr_t)slot.d_index);
    }
    node->pool->put(j.ws);
    j.ws = PoolBuf{};
    return;
  }
  const int64_t* hx = static_cast<const int64_t*>(j.hidx.first);
  auto ix = [&](uint32_t k, int p) { return hx[(uint64_t)k * (R + 1) + p]; };
  // peer-major: sections [h] of the whole job (every map the kernels wrote, claimed or not)
  std::vector<uint64_t> run((size_t)W, 0);
  uint64_t packed_off = 0;  // packed (compressed) maps: where map k starts in the slab
  if (W > 1) {
    uint64_t acc = 0;
    for (int h = 0; h < W; ++h) {
      run[h] = acc;
      const int lo = owner_lo(h, R, W), hi = owner_lo(h + 1, R, W);
      for (uint32_t k = 0; k < j.maps; ++k) acc += (uint64_t)(ix(k, hi) - ix(k, lo));
    }
  }
  for (uint32_t k = 0; k < j.maps; ++k) {
    if (j.claimed[k]) {
      MapSlot& slot = sh.maps[j.first + k];
      slot.pending = false;
      slot.present = true;
      slot.sent = false;
      slot.owner = node->conf.rank;
      slot.slab = j.slab;
      slot.batch = j.batch >= 0 ? j.batch : sh.next_batch++;  // map-major at W > 1: own piece
      slot.off = j.packed ? packed_off : (uint64_t)k * j.rpm * (uint64_t)sh.rec_size;
      slot.bytes = (uint64_t)ix(k, R);
      slot.index.assign(hx + (uint64_t)k * (R + 1), hx + (uint64_t)(k + 1) * (R + 1));
      slot.d_index = nullptr;
      slot.rslab.reset();
      if (W > 1) {
        slot.seg = run;
      } else {  // map-major: peer h's range of the map is a sub-range of its data file
        const int NW = node->conf.world_size;
        slot.seg.resize((size_t)NW);
        for (int h = 0; h < NW; ++h) slot.seg[h] = slot.off + (uint64_t)ix(k, owner_lo(h, R, NW));
      }
      publish_slot(node, sh, j.first + (int32_t)k, 0);
    }
    packed_off += (uint64_t)ix(k, R);
    if (W > 1)
      for (int h = 0; h < W; ++h)
        run[h] += (uint64_t)(ix(k, owner_lo(h + 1, R, W)) - ix(k, owner_lo(h, R, W)));
  }
  node->pool->put(j.ws);
  node->hpool.put(j.hidx);
  j.ws = PoolBuf{};
  j.hidx = {nullptr, 0};
}

// Publish every write job of `sh` whose kernels have completed (wait = block for all of them):
// the directory slots of its maps get their index tables.  The analog of the reference's
// completion callbacks, which run inside worker.progress() on the calling thread
// (UcxWorkerWrapper.scala:100-120).  Called with `lk` held; waits with it released.
void progress(sux_node* node, Shuffle& sh, std::unique_lock<std::mutex>& lk, bool wait) {
  while (!sh.jobs.empty()) {
    std::vector<std::unique_ptr<WriteJob>> jobs;
    jobs.swap(sh.jobs);
    sh.busy += (int)jobs.size();
    std::vector<char> done(jobs.size(), 0);
    hipError_t err = hipSuccess;
    lk.unlock();
    for (size_t i = 0; i < jobs.size() && err == hipSuccess; ++i) {
      hipError_t e = wait ? hipEventSynchronize(jobs[i]->done->e) : hipEventQuery(jobs[i]->done->e);
      if (e == hipSuccess) done[i] = 1;
      else if (e != hipErrorNotReady) err = e;
    }
    uint32_t derr = 0;
    if (err == hipSuccess && std::find(done.begin(), done.end(), 1) != done.end())
      derr = take_device_err(node);
    lk.lock();
    sh.busy -= (int)jobs.size();
    if (derr) {
      std::vector<std::unique_ptr<WriteJob>> bad;
      for (size_t i = 0; i < jobs.size(); ++i) {
        if (done[i]) bad.push_back(std::move(jobs[i]));
        else sh.jobs.push_back(std::move(jobs[i]));
      }
      reject_jobs(node, sh, bad, derr);
    }
    for (size_t i = 0; i < jobs.size(); ++i) {
      if (!done[i]) {
        sh.jobs.push_back(std::move(jobs[i]));
        continue;
      }
      publish_job(node, sh, *jobs[i]);
      jobs[i].reset();
    }
    node->cv.notify_all();
    hip_check(err, "map output completion");
    if (!wait) return;
  }
}

// Wait for (and publish) only the jobs that write maps of [lo, hi), and for writes that claimed a
// slot there and are still submitting.  Jobs of later map batches keep running: an exchange of
// batch k does not wait for batch k+1's kernels (the overlap of sux_exchange_maps).
void drain_range(sux_node* node, Shuffle& sh, std::unique_lock<std::mutex>& lk, int32_t lo,
                 int32_t hi) {
  while (true) {
    std::vector<std::unique_ptr<WriteJob>> mine;
    for (auto& j : sh.jobs)
      if (j && j->first < hi && j->first + (int32_t)j->maps > lo) mine.push_back(std::move(j));
    sh.jobs.erase(std::remove(sh.jobs.begin(), sh.jobs.end(), nullptr), sh.jobs.end());
    if (!mine.empty()) {
      sh.busy += (int)mine.size();
      hipError_t err = hipSuccess;
      lk.unlock();
      for (auto& j : mine) {
        const hipError_t e = hipEventSynchronize(j->done->e);
        if (e != hipSuccess && err == hipSuccess) err = e;
      }
      const uint32_t derr = err == hipSuccess ? take_device_err(node) : 0u;
      lk.lock();
      sh.busy -= (int)mine.size();
      if (derr) reject_jobs(node, sh, mine, derr);
      for (auto& j : mine) publish_job(node, sh, *j);
      node->cv.notify_all();
      hip_check(err, "map output completion");
      continue;
    }
    bool pending = false;
    for (int32_t m = lo; m < hi && !pending; ++m) pending = sh.maps[m].pending;
    if (!pending) return;
    node->cv.wait(lk);  // another thread is waiting on, or still submitting, one of those jobs
  }
}

// Block until no write of `sh` is queued, being waited on by another thread, or being submitted
// (every claimed slot is published).  Called with `lk` held.
void drain(sux_node* node, Shuffle& sh, std::unique_lock<std::mutex>& lk) {
  while (!sh.jobs.empty() || sh.busy > 0 || sh.submitting > 0) {
    if (!sh.jobs.empty()) progress(node, sh, lk, true);
    else node->cv.wait(lk);
  }
}

}  // namespace
void export_ipc(sux_node* node, const void* p, uint8_t out[SUX_IPC_DESC_BYTES]);
void free_ticket(sux_xticket* t);
namespace {

// Map a peer allocation by its 64-byte IPC handle.  The HIP runtime keys the mappings it hands
// out by the exporter's address: when a peer frees an allocation this process still maps and its
// allocator gives the address to a new allocation, opening the NEW handle returns the old mapping
// — the freed memory, not the new bytes (tests/test_gpu_ipc_reuse.py).  A returned base this
// process already holds under another handle is that stale mapping: every reference to it is
// dropped (its allocation is gone; whoever still held it held freed memory) and the handle is
// opened again.
//
// The open itself is bounded: it runs on a helper thread and a caller that waits
// longer than SUX_IPC_OPEN_TIMEOUT_S seconds (default 120) gets SUX_ECOMM naming the exporter
// instead of a hang.  Measured on the box (profiles/r06_ipc/): hipIpcOpenMemHandle of a peer's
// torch-allocated 2048 or 3072 MiB buffer never returns when the importing process holds a torch
// buffer of its own of that size (1024, 1536 and 4096 MiB open in < 1 ms; raw hipMalloc buffers
// of every size from 256 MiB to 8 GiB open in < 1 ms) — it reproduces with no call of this
// library in either process, so it is the runtime's; a stuck helper thread is abandoned.
hipError_t ipc_open_bounded(sux_node* node, void** base, const hipIpcMemHandle_t& h,
                            double* waited_s) {
  static const double limit_s = [] {
    const char* v = std::getenv("SUX_IPC_OPEN_TIMEOUT_S");
    const double t = v ? std::atof(v) : 120.0;
    return t > 0 ? t : 120.0;
  }();
  struct Call {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    bool abandoned = false;  // the caller stopped waiting: a late mapping is closed, not leaked
    hipError_t e = hipErrorUnknown;
    void* base = nullptr;
  };
  auto c = std::make_shared<Call>();
  const int device = node->conf.device;
  std::thread([c, h, device] {
    void* b = nullptr;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess);
    bool late = false;
    {
      std::lock_guard<std::mutex> lk(c->mu);
      c->e = e;
      c->base = b;
      c->done = true;
      late = c->abandoned;
      c->cv.notify_all();
    }
    if (late && e == hipSuccess) (void)hipIpcCloseMemHandle(b);
  }).detach();
  const auto t0 = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lk(c->mu);
  const bool done = c->cv.wait_for(lk, std::chrono::duration<double>(limit_s), [&] { return c->done; });
  *waited_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (!done) {  // the helper keeps running; a mapping it still gets is closed by the helper
    c->abandoned = true;
    return hipErrorNotReady;
  }
  *base = c->base;
  return c->e;
}

void* ipc_open_fresh(sux_node* node, const uint8_t* handle) {
  std::lock_guard<std::mutex> lk(node->ipc_mu);
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, 64);
  const std::string key(reinterpret_cast<const char*>(handle), 64);
  for (int attempt = 0; attempt < 2; ++attempt) {
    void* base = nullptr;
    double waited = 0;
    const hipError_t e = ipc_open_bounded(node, &base, h, &waited);
    if (e == hipErrorNotReady) {
      uint64_t va = 0;
      uint32_t pid = 0;
      std::memcpy(&va, handle, 8);
      std::memcpy(&pid, handle + 8, 4);
      char msg[320];
      std::snprintf(msg, sizeof msg,
                    "hipIpcOpenMemHandle of the allocation at 0x%llx exported by pid %u did not "
                    "return in %.0f s (the import is abandoned; SUX_IPC_OPEN_TIMEOUT_S sets the "
                    "bound)",
                    (unsigned long long)va, pid, waited);
      raise(SUX_ECOMM, msg);
    }
    if (e != hipSuccess) {
      // reported at once, with what a diagnosis needs (the round-3 failure): the
      // exporter's address and pid as ROCm 7.2 lays them in the handle, and this process's open
      // descriptors against its limit (an import opens one)
      uint64_t va = 0;
      uint32_t pid = 0;
      std::memcpy(&va, handle, 8);
      std::memcpy(&pid, handle + 8, 4);
      struct rlimit rl {};
      (void)getrlimit(RLIMIT_NOFILE, &rl);
      long fds = 0;
      if (DIR* d = opendir("/proc/self/fd")) {
        while (readdir(d)) ++fds;
        closedir(d);
      }
      char msg[256];
      std::snprintf(msg, sizeof msg,
                    "hipIpcOpenMemHandle: %s (handle of exporter pid %u, address 0x%llx; "
                    "%ld open descriptors, limit %llu)",
                    hipGetErrorString(e), pid, (unsigned long long)va, fds - 2,
                    (unsigned long long)rl.rlim_cur);
      raise(SUX_EHIP, msg);
    }
    auto it = node->ipc_maps.find(base);
    if (it == node->ipc_maps.end()) {
      node->ipc_maps[base] = {key, 1};
      return base;
    }
    if (it->second.first == key) {
      it->second.second++;
      return base;
    }
    (void)hipIpcCloseMemHandle(base);  // the reference just taken
    for (int r = 0; r < it->second.second; ++r) (void)hipIpcCloseMemHandle(base);
    node->ipc_maps.erase(it);
  }
  raise(SUX_EHIP, "hipIpcOpenMemHandle keeps returning the mapping of a freed allocation");
  return nullptr;
}

// Drop one reference taken by ipc_open_fresh (none if the mapping was already dropped as stale).
void ipc_close_ref(sux_node* node, void* base, const std::string& key) {
  std::lock_guard<std::mutex> lk(node->ipc_mu);
  auto it = node->ipc_maps.find(base);
  if (it == node->ipc_maps.end() || it->second.first != key) return;
  (void)hipIpcCloseMemHandle(base);
  if (--it->second.second == 0) node->ipc_maps.erase(it);
}

// Everything a shuffle holds on the device: slabs and receive buffers (via the slots), IPC
// mappings, spill files.
void release_shuffle(sux_node* node, Shuffle& sh) {
  for (auto& kv : sh.ipc_bases) ipc_close_ref(node, kv.second, kv.first);
  sh.ipc_bases.clear();
  for (auto& m : sh.maps) {
    m.slab.reset();
    m.rslab.reset();
    if (m.spilled()) {  // CommonUcxShuffleBlockResolver.removeShuffle deletes the files too
      ::unlink(m.spill_data.c_str());
      ::unlink(m.spill_index.c_str());
    }
  }
}

struct Group {
  sux::MapGroup g{};
  sux::Workspace ws{};
};

// The node's tuning table with every default filled in.  `pipelined`: the call keeps two launch
// groups in flight (sux_partition_maps_pipelined, sux_write_map_outputs); the co-resident K1/K3
// shapes are then possible, but measured slower (profiles/r02_sw_b: 1331 vs 1437 GB/s on
// TeraSort 100 GB: a K1 beside K3 takes K3's HBM share), so they are opt-in.
constexpr int kDefaultSmallKernel = 4;  // two-level MSD passes (profiles/r02_sweeps/msd: 752 -> 800 GB/s)

sux::Tuning resolve_tuning(const sux_tuning& t, bool pipelined) {
  sux::Tuning r;
  if (t.hist_kernel) r.hist_kernel = t.hist_kernel;
  if (t.scatter_kernel) r.scatter_kernel = t.scatter_kernel;
  r.coresident = t.coresident > 0 && pipelined;
  r.scatter_chunk = t.scatter_chunk ? t.scatter_chunk : r.coresident ? 768 : 1024;
  if (t.scatter_depth) r.scatter_depth = t.scatter_depth;
  if (t.hist_stage) r.hist_stage = t.hist_stage;
  r.hist_wgs_per_cu = t.hist_wgs_per_cu;
  if (t.s6_chunk) r.s6_chunk = t.s6_chunk;
  r.tiles_per_item = t.tiles_per_item;
  if (t.small_groups) r.small_groups = t.small_groups;
  r.tile_records = t.tile_records;
  r.onepass = t.onepass == 1;
  if (t.varlen_kernel) r.varlen_kernel = t.varlen_kernel;
  r.varlen_tile = t.varlen_tile;
  r.small_kernel = t.small_kernel ? t.small_kernel : kDefaultSmallKernel;
  r.small_auto = t.small_kernel == 0;
  r.scatter_order = t.scatter_order;
  if (t.small_wgs_per_cu) r.small_wgs_per_cu = t.small_wgs_per_cu;
  r.hist_nt = t.hist_nt >= 0;  // 0: non-temporal (round 3 A/B: 1639 vs 1596 GB/s), -1: plain
  r.counts_tm = t.counts_layout != 1;
  if (t.scatter_counters) r.scatter_counters = t.scatter_counters;
  r.lz4_queue = t.lz4_queue != 2;  // the work queue: 46.6 -> 53.0 GB/s (profiles/r03)
  r.scatter_nt = t.scatter_nt > 0 ? t.scatter_nt : 0;
  r.split_cus = t.split_cus > 0 ? t.split_cus : 0;
  r.gather_kernel = t.gather_kernel ? t.gather_kernel : 3;
  // 0: 32-partition buckets + pass B's element -> run map (bits 3 + 4; round 5, C5 965 -> 993
  // GB/s, profiles/r05_h) + pass A's tag match (bit 7; round 6: pass A alone 1.57-1.59 ->
  // 1.49-1.52 ms, the C5 leg +0.4 %, profiles/r06_msd16a/tag_*); -1: round 4's shape
  // (16-partition buckets, run-table search)
  r.msd_direct = t.msd_direct > 0 ? t.msd_direct : t.msd_direct == 0 ? 152 : 0;
  r.gather16 = r.gather_kernel != 2;
  return r;
}

Group make_group(const sux_partitioner* part, const void* recs, uint32_t rs, uint64_t rpm,
                 uint64_t n) {
  check_record_size(rs);
  check_key_fits(part, rs);
  require(rpm > 0, SUX_EINVAL, "records_per_map must be > 0");
  uint64_t maps = (n + rpm - 1) / rpm;
  require(maps <= 0xFFFFFFFFull, SUX_EINVAL, "too many maps in one group");
  require(n < (1ull << 32), SUX_ERANGE, "a launch group holds < 2^32 records");
  require(((uintptr_t)recs & 3) == 0, SUX_EINVAL, "records must be 4-byte aligned");
  Group G;
  uint32_t R = (uint32_t)part->desc.num_partitions;
  require(part->node != nullptr, SUX_ESTATE, "the partitioner's node was destroyed");
  uint32_t tile = sux::choose_tile_recs(R, rs, rpm, resolve_tuning(part->node->tuning, false));
  G.g.recs = static_cast<const uint8_t*>(recs);
  G.g.records_per_map = rpm;
  G.g.num_records = n;
  G.g.num_maps = (uint32_t)maps;
  G.g.rec_size = rs;
  G.g.tile_recs = tile;
  G.g.tiles_per_map = (uint32_t)((rpm + tile - 1) / tile);
  G.g.err = part->node->d_err;
  G.ws = sux::workspace_layout(R, rs, rpm, n, tile, true, sux::small_two_pass_shape(R, rs));
  return G;
}

void run_group(sux_node* node, const sux_partitioner* part, const Group& G, int32_t world,
               void* d_out, int64_t* d_index, uint8_t* d_index_be, uint16_t* d_pids,
               uint64_t* d_peer_bytes, void* d_ws, uint64_t ws_bytes, hipStream_t s,
               bool pipelined = false, hipStream_t s_k1 = nullptr, hipEvent_t k1_done = nullptr,
               const int32_t* d_own = nullptr) {
  require(d_ws || G.ws.total == 0, SUX_EINVAL, "workspace is NULL");
  require(ws_bytes >= G.ws.total, SUX_EINVAL,
          "workspace too small: need " + std::to_string(G.ws.total) + " bytes");
  require(d_out && d_index, SUX_EINVAL, "output or index pointer is NULL");
  require(((uintptr_t)d_out & 3) == 0 && ((uintptr_t)d_index & 7) == 0 &&
              ((uintptr_t)d_index_be & 7) == 0 && ((uintptr_t)d_ws & 255) == 0,
          SUX_EINVAL, "output (4 B), index (8 B) and workspace (256 B) must be aligned");
  if (G.g.num_records == 0) return;
  sux::LayoutDesc lay{world, G.g.rec_size, d_own};
  hip_check(sux::launch_partition_group(part->pd, G.g, lay, static_cast<uint8_t*>(d_out), d_index,
                                        d_index_be, d_pids, static_cast<uint8_t*>(d_ws), G.ws,
                                        d_peer_bytes, resolve_tuning(node->tuning, pipelined),
                                        &node->timer, s, s_k1, k1_done),
            "partition launch");
}
}  // namespace

// ============================================================================================
// C-ABI
// ============================================================================================
extern "C" {

void sux_conf_init(sux_conf* c) {
  if (!c) return;
  std::memset(c, 0, sizeof *c);
  c->world_size = 1;
  c->min_buffer_size = 1024;                 // spark.shuffle.ucx.memory.minBufferSize
  c->min_allocation_size = 4ull << 20;       // spark.shuffle.ucx.memory.minAllocationSize
  c->metadata_block_size = 2 * 150;          // 2 * spark.shuffle.ucx.rkeySize
}

// UcxShuffleConf.preallocateBuffersMap (:56-64): "size:count" pairs, comma separated, sizes in
// Utils.byteStringAsBytes notation (binary multiples), empty entries skipped.
int sux_conf_set_prealloc(sux_conf* c, const char* spec) {
  return guard([&] {
    require(c && spec, SUX_EINVAL, "NULL argument");
    std::vector<std::pair<uint64_t, uint64_t>> out;
    std::string all(spec);
    size_t b = 0;
    while (b <= all.size()) {
      size_t e = all.find(',', b);
      if (e == std::string::npos) e = all.size();
      std::string ent = all.substr(b, e - b);
      b = e + 1;
      auto trim = [](std::string x) {
        size_t i = x.find_first_not_of(" \t"), j = x.find_last_not_of(" \t");
        return i == std::string::npos ? std::string() : x.substr(i, j - i + 1);
      };
      ent = trim(ent);
      if (ent.empty()) continue;
      const size_t colon = ent.find(':');
      require(colon != std::string::npos && ent.find(':', colon + 1) == std::string::npos,
              SUX_EINVAL, "preAllocateBuffers entry '" + ent + "' is not size:count");
      std::string sz = trim(ent.substr(0, colon)), ct = trim(ent.substr(colon + 1));
      size_t i = 0;
      while (i < sz.size() && std::isdigit((unsigned char)sz[i])) ++i;
      require(i > 0, SUX_EINVAL, "bad buffer size '" + sz + "'");
      uint64_t v = std::stoull(sz.substr(0, i));
      std::string suf = sz.substr(i);
      for (auto& ch : suf) ch = (char)std::tolower((unsigned char)ch);
      int sh = -1;
      if (suf.empty() || suf == "b") sh = 0;
      else if (suf == "k" || suf == "kb") sh = 10;
      else if (suf == "m" || suf == "mb") sh = 20;
      else if (suf == "g" || suf == "gb") sh = 30;
      else if (suf == "t" || suf == "tb") sh = 40;
      require(sh >= 0, SUX_EINVAL, "bad buffer size '" + sz + "'");
      require(!ct.empty() && ct.find_first_not_of("0123456789") == std::string::npos, SUX_EINVAL,
              "bad buffer count '" + ct + "'");
      out.emplace_back(v << sh, std::stoull(ct));
    }
    require(out.size() <= SUX_MAX_PREALLOC, SUX_EINVAL,
            "at most " + std::to_string(SUX_MAX_PREALLOC) + " preAllocateBuffers entries");
    c->num_prealloc = (uint32_t)out.size();
    for (size_t k = 0; k < out.size(); ++k) {
      c->prealloc_size[k] = out[k].first;
      c->prealloc_count[k] = out[k].second;
    }
  });
}

int sux_abi_version(void) { return SUX_ABI_VERSION; }

int sux_last_error(char* buf, size_t len) {
  if (buf && len) {
    size_t k = std::min(len - 1, g_err.size());
    std::memcpy(buf, g_err.data(), k);
    buf[k] = 0;
  }
  return (int)g_err.size();
}

int sux_comm_unique_id(uint8_t out[128]) {
  return guard([&] {
    require(out != nullptr, SUX_EINVAL, "out is NULL");
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out, &id, 128);
  });
}

int sux_node_create(const sux_conf* conf, int is_driver, sux_node** out) {
  return guard([&] {
    require(conf && out, SUX_EINVAL, "conf/out is NULL");
    require(conf->world_size >= 1 && conf->rank >= 0 && conf->rank < conf->world_size, SUX_EINVAL,
            "rank/world_size out of range");
    require(conf->min_buffer_size > 0 && conf->min_allocation_size > 0, SUX_EINVAL,
            "pool sizes must be positive");
    require(conf->num_prealloc <= SUX_MAX_PREALLOC, SUX_EINVAL, "num_prealloc out of range");
    // every directory slot holds one 32-byte descriptor (publish_slot); the reference throws
    // the same way when its descriptor outgrows the slot (CommonUcxShuffleBlockResolver.scala:72-76)
    require(conf->metadata_block_size >= 32, SUX_ERANGE,
            "Metadata block size 32 is greater then configured (" +
                std::to_string(conf->metadata_block_size) + ")");
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    require(conf->device >= 0 && conf->device < ndev, SUX_EINVAL,
            "device " + std::to_string(conf->device) + " not present (" + std::to_string(ndev) +
                " devices)");
    auto n = std::make_unique<sux_node>();
    n->conf = *conf;
    n->is_driver = is_driver != 0;
    n->bind();
    n->pool = std::make_unique<DevicePool>(conf->min_buffer_size, conf->min_allocation_size);
    n->pool->set_limit((uint64_t)conf->pool_limit_mib << 20);
    hip_check(hipMalloc(&n->d_err, sizeof(uint32_t)), "hipMalloc(error word)");
    hip_check(hipMemset(n->d_err, 0, sizeof(uint32_t)), "hipMemset(error word)");
    // UcxNode.java:81-83: executors preallocate the configured buffers
    if (!n->is_driver)
      for (uint32_t k = 0; k < conf->num_prealloc; ++k)
        n->pool->preallocate(conf->prealloc_size[k], conf->prealloc_count[k]);
    // a communicator for world_size > 1, or at world_size 1 when a unique id is supplied (the
    // exchange then runs through RCCL with one rank: the single-GPU rehearsal of the N > 1 path)
    bool have_id = false;
    for (int i = 0; i < 128; ++i) have_id |= conf->comm_id[i] != 0;
    if (have_id) {
      ncclUniqueId id;
      std::memcpy(&id, conf->comm_id, 128);
      nccl_check(ncclCommInitRank(&n->comm, conf->world_size, id, conf->rank), "ncclCommInitRank");
    }
    *out = n.release();
  });
}

int sux_node_set_bootstrap(sux_node* node, sux_allgather_fn fn, void* ctx) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    std::lock_guard<std::mutex> lk(node->mu);
    node->boot = fn;
    node->boot_ctx = ctx;
  });
}

int sux_node_connect(sux_node* node) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    {
      std::lock_guard<std::mutex> lk(node->mu);
      if (node->comm) return;
      require(node->boot != nullptr, SUX_ESTATE,
              "sux_node_connect needs the group's bootstrap (sux_node_set_bootstrap)");
    }
    node->bind();
    const int W = node->conf.world_size, r = node->conf.rank;
    ncclUniqueId mine;
    std::memset(&mine, 0, sizeof mine);
    if (r == 0) nccl_check(ncclGetUniqueId(&mine), "ncclGetUniqueId");
    std::vector<uint8_t> all((size_t)W * sizeof mine);
    const int rc = node->boot(node->boot_ctx, SUX_TAG_COMM_ID, &mine, sizeof mine, all.data());
    require(rc == 0, SUX_ECOMM, "bootstrap all-gather of the RCCL unique id failed (" +
                                    std::to_string(rc) + ")");
    ncclUniqueId id;
    std::memcpy(&id, all.data(), sizeof id);  // rank 0's
    ncclComm_t comm = nullptr;
    nccl_check(ncclCommInitRank(&comm, W, id, r), "ncclCommInitRank");
    std::lock_guard<std::mutex> lk(node->mu);
    node->comm = comm;
  });
}

// ---- executor group membership (driver side; host-only: no HIP call, so a driver without a
// GPU, or a parent process that forks its executors, never initialises the runtime) ----------
}  // extern "C"
struct sux_group {
  int32_t world = 0;
  std::mutex mu;
  std::map<std::string, std::pair<int32_t, int32_t>> members;  // executor id -> (rank, local)
  std::map<std::string, int32_t> per_host;                     // host -> executors joined
};

namespace {
template <class F>
int host_guard(F&& f) {
  try {
    f();
    return SUX_OK;
  } catch (const SuxError& e) {
    g_err = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    g_err = "host allocation failed";
    return SUX_ENOMEM;
  } catch (...) {
    g_err = "unknown error";
    return SUX_EINVAL;
  }
}
}  // namespace

extern "C" {
int sux_group_create(int32_t world_size, sux_group** out) {
  return host_guard([&] {
    require(out, SUX_EINVAL, "NULL argument");
    require(world_size >= 1, SUX_EINVAL, "world size must be >= 1");
    auto g = std::make_unique<sux_group>();
    g->world = world_size;
    *out = g.release();
  });
}

int sux_group_destroy(sux_group* group) {
  return host_guard([&] { delete group; });
}

int sux_group_join(sux_group* group, const char* executor_id, const char* host, int32_t* rank,
                   int32_t* local_index) {
  return host_guard([&] {
    require(group && executor_id && host && rank && local_index, SUX_EINVAL, "NULL argument");
    const std::string id(executor_id);
    require(!id.empty(), SUX_EINVAL, "empty executor id");
    std::lock_guard<std::mutex> lk(group->mu);
    auto it = group->members.find(id);
    if (it == group->members.end()) {
      require((int32_t)group->members.size() < group->world, SUX_ERANGE,
              "executor " + id + " joins a GPU group of " + std::to_string(group->world) +
                  " that is already complete");
      const int32_t r = (int32_t)group->members.size();
      const int32_t l = group->per_host[host]++;
      it = group->members.emplace(id, std::make_pair(r, l)).first;
    }
    *rank = it->second.first;
    *local_index = it->second.second;
  });
}

int sux_group_size(sux_group* group, int32_t* joined) {
  return host_guard([&] {
    require(group && joined, SUX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(group->mu);
    *joined = (int32_t)group->members.size();
  });
}

int sux_node_set_spill_dir(sux_node* node, const char* dir) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    std::string d = dir ? dir : "";
    if (!d.empty()) {
      struct stat st;
      require(::stat(d.c_str(), &st) == 0 && S_ISDIR(st.st_mode), SUX_EIO,
              "spill directory " + d + " does not exist");
    }
    std::lock_guard<std::mutex> lk(node->mu);
    node->spill_dir = d;
  });
}

int sux_node_spills(sux_node* node, uint64_t* spilled_maps) {
  return guard([&] {
    require(node && spilled_maps, SUX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(node->mu);
    *spilled_maps = node->spills;
  });
}

int sux_pool_stats(sux_node* node, uint64_t* bytes, uint64_t* requests, uint64_t* allocs,
                   uint64_t* preallocs) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    node->pool->stats(bytes, requests, allocs, preallocs);
  });
}

int sux_node_set_tuning(sux_node* node, const sux_tuning* t) {
  return guard([&] {
    require(t, SUX_EINVAL, "NULL tuning");
    auto in = [](int32_t v, std::initializer_list<int32_t> ok) {
      if (v == 0) return true;
      for (int32_t o : ok)
        if (v == o) return true;
      return false;
    };
    require(in(t->hist_kernel, {1, 3, 4}), SUX_EINVAL, "hist_kernel must be 1, 3 or 4");
    require(in(t->scatter_kernel, {1, 6, 7, 8}), SUX_EINVAL, "scatter_kernel must be 1, 6, 7 or 8");
    require(t->coresident >= -1 && t->coresident <= 1, SUX_EINVAL, "coresident must be -1, 0 or 1");
    require(in(t->scatter_chunk, {512, 768, 1024}), SUX_EINVAL,
            "scatter_chunk must be 512, 768 or 1024");
    require(in(t->scatter_depth, {1, 2}), SUX_EINVAL, "scatter_depth must be 1 or 2");
    require(t->scatter_depth != 2 || t->scatter_chunk == 768, SUX_EINVAL,
            "scatter_depth 2 needs scatter_chunk 768");
    require(in(t->hist_stage, {64, 128}), SUX_EINVAL, "hist_stage must be 64 or 128");
    require(t->hist_wgs_per_cu >= 0 && t->hist_wgs_per_cu <= 8, SUX_EINVAL,
            "hist_wgs_per_cu must be 0..8");
    require(in(t->small_kernel, {1, 2, 4}), SUX_EINVAL, "small_kernel must be 1, 2 or 4");
    require(in(t->small_waves, {8, 16}), SUX_EINVAL, "small_waves must be 8 or 16");
    require(in(t->scatter_order, {1, 2}), SUX_EINVAL, "scatter_order must be 1 or 2");
    require(in(t->small_wgs_per_cu, {1, 2}), SUX_EINVAL, "small_wgs_per_cu must be 1 or 2");
    require(in(t->sort_msd, {1, 2, 3}), SUX_EINVAL, "sort_msd must be 1, 2 or 3");
    require(in(t->s6_chunk, {256, 384, 512, 1024}), SUX_EINVAL, "s6_chunk must be 256..1024");
    require(t->tiles_per_item >= 0 && t->tiles_per_item <= 4096, SUX_EINVAL,
            "tiles_per_item must be 0..4096");
    require(in(t->small_groups, {1, 2, 4}), SUX_EINVAL, "small_groups must be 1, 2 or 4");
    require(t->tile_records == 0 || (t->tile_records >= 64 && t->tile_records <= (1 << 22) &&
                                     (t->tile_records & (t->tile_records - 1)) == 0),
            SUX_EINVAL, "tile_records must be a power of two in [64, 2^22]");
    require(t->onepass == 0 || t->onepass == 1, SUX_EINVAL, "onepass must be 0 or 1");
    require(in(t->varlen_kernel, {1, 2, 3}), SUX_EINVAL, "varlen_kernel must be 1, 2 or 3");
    require(t->varlen_tile == 0 || (t->varlen_tile >= 64 && t->varlen_tile <= 65536 &&
                                    t->varlen_tile % 64 == 0),
            SUX_EINVAL, "varlen_tile must be a multiple of 64 in [64, 65536]");
    require(t->sort_max_digit_bits == 0 ||
                (t->sort_max_digit_bits >= 8 && t->sort_max_digit_bits <= 16),
            SUX_EINVAL, "sort_max_digit_bits must be 8..16");
    require(t->sort_gather == 0 || t->sort_gather == 1, SUX_EINVAL, "sort_gather must be 0 or 1");
    require(t->sort_all_passes == 0 || t->sort_all_passes == 1, SUX_EINVAL,
            "sort_all_passes must be 0 or 1");
    require(t->exchange_self >= -1 && t->exchange_self <= 1, SUX_EINVAL,
            "exchange_self must be -1, 0 or 1");
    require(t->hist_nt >= -1 && t->hist_nt <= 1, SUX_EINVAL, "hist_nt must be -1, 0 or 1");
    require(in(t->counts_layout, {1, 2}), SUX_EINVAL, "counts_layout must be 1 or 2");
    require(in(t->scatter_counters, {1, 2}), SUX_EINVAL, "scatter_counters must be 1 or 2");
    require(in(t->lz4_queue, {1, 2}), SUX_EINVAL, "lz4_queue must be 1 or 2");
    require(t->scatter_nt >= -1 && t->scatter_nt <= 3, SUX_EINVAL, "scatter_nt must be -1 .. 3");
    require(in(t->gather_kernel, {1, 2, 3}), SUX_EINVAL, "gather_kernel must be 1, 2 or 3");
    require(t->split_cus == -1 || (t->split_cus >= 0 && t->split_cus <= 224 && t->split_cus % 32 == 0),
            SUX_EINVAL, "split_cus must be -1, 0 or a multiple of 32 up to 224");
    require(t->msd_direct >= -1 && t->msd_direct <= 255, SUX_EINVAL, "msd_direct must be -1 .. 255");
    for (int32_t r : t->reserved) require(r == 0, SUX_EINVAL, "reserved tuning fields must be 0");
    require(node, SUX_EINVAL, "NULL node");
    std::lock_guard<std::mutex> lk(node->mu);
    node->tuning = *t;
  });
}

int sux_node_check(sux_node* node) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    node->bind();
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    uint32_t w = 0;
    hip_check(hipMemcpy(&w, node->d_err, sizeof w, hipMemcpyDeviceToHost), "read error word");
    if (w == 0) return;
    hip_check(hipMemset(node->d_err, 0, sizeof w), "clear error word");
    std::string what;
    if (w & sux::kErrTurnTimeout)
      what += "a small-record scatter wave timed out waiting for its turn (the launch stopped "
              "without writing its remaining records); ";
    if (w & sux::kErrLz4Stream) what += "a compressed block is corrupted (sux_decompress_blocks: header, lengths "
                        "or LZ4 sequence); ";
    if (w & sux::kErrLz4Capacity) what += "decompressed bytes exceed the output capacity (nothing decoded); ";
    if (w & sux::kErrLz4Checksum) what += "a decompressed chunk's XXH32 differs from its header (stream corrupted); ";
    raise(SUX_EHIP, "device error word 0x" + [&] {
      char b[16];
      std::snprintf(b, sizeof b, "%x", w);
      return std::string(b);
    }() + ": " + what);
  });
}

int sux_node_get_tuning(sux_node* node, sux_tuning* t) {
  return guard([&] {
    require(node && t, SUX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(node->mu);
    *t = node->tuning;
  });
}

int sux_node_destroy(sux_node* node) {
  return guard([&] {
    if (!node) return;
    node->bind();
    {
      std::unique_lock<std::mutex> lk(node->mu);
      for (auto& kv : node->shuffles) drain(node, *kv.second, lk);
    }
    (void)hipDeviceSynchronize();
    for (sux_xticket* t : node->tickets) free_ticket(t);  // posted, never issued: leases return
    node->tickets.clear();
    {
      std::lock_guard<std::mutex> lk(node->live_mu);
      for (sux_partitioner* p : node->live_parts) p->node = nullptr;
      for (sux_buffer* b : node->live_bufs) b->node = nullptr;
      node->live_parts.clear();
      node->live_bufs.clear();
    }
    for (int i = 0; i < 2; ++i) {
      if (node->pipe[i]) (void)hipStreamDestroy(node->pipe[i]);
      node->pool->put(node->pipe_ws[i]);
    }
    for (hipEvent_t e : node->pipe_ev)
      if (e) (void)hipEventDestroy(e);
    for (hipStream_t p : node->pipe_split)
      if (p) (void)hipStreamDestroy(p);
    for (hipEvent_t e : node->split_ev)
      if (e) (void)hipEventDestroy(e);
    if (node->sort_side) (void)hipStreamDestroy(node->sort_side);
    for (hipEvent_t e : node->sort_ev)
      if (e) (void)hipEventDestroy(e);
    if (node->d_err) (void)hipFree(node->d_err);
    if (node->d_own) (void)hipFree(node->d_own);
    for (auto& kv : node->shuffles) release_shuffle(node, *kv.second);
    node->shuffles.clear();
    for (auto& kv : node->ipc_bases) ipc_close_ref(node, kv.second.first, kv.second.second);
    node->ipc_bases.clear();
    if (node->comm_x) (void)ncclCommDestroy(node->comm_x);
    if (node->comm) (void)ncclCommDestroy(node->comm);
    (void)hipGetLastError();  // see nccl_check
    delete node;
  });
}

// ---- partitioner ----------------------------------------------------------------------------
int sux_partitioner_create(sux_node* node, const sux_partitioner_desc* d, sux_partitioner** out) {
  return guard([&] {
    require(node && d && out, SUX_EINVAL, "NULL argument");
    const int R = d->num_partitions;
    require(R >= 1 && R <= sux::kMaxPartitions, SUX_EINVAL,
            "num_partitions must be in [1, 32768], got " + std::to_string(R));
    require(d->key_offset >= 0, SUX_EINVAL, "key_offset < 0");
    switch (d->kind) {
      case SUX_PART_RANGE_BYTES:
        require(d->key_len >= 1 && d->key_len <= 16, SUX_EINVAL, "range key_len must be 1..16");
        require(R == 1 || d->range_bounds, SUX_EINVAL, "range partitioner needs R-1 bounds");
        break;
      case SUX_PART_MURMUR3_LONG:
      case SUX_PART_HASH_LONG:
        require(d->key_len == 8, SUX_EINVAL, "long key needs key_len 8");
        break;
      case SUX_PART_MURMUR3_INT:
      case SUX_PART_HASH_INT:
        require(d->key_len == 4, SUX_EINVAL, "int key needs key_len 4");
        break;
      case SUX_PART_MURMUR3_BYTES:
        require(d->key_len >= 1 && d->key_len <= 4096, SUX_EINVAL, "binary key_len must be >= 1");
        break;
      default:
        raise(SUX_EINVAL, "unknown partitioner kind " + std::to_string(d->kind));
    }
    node->bind();
    auto p = std::make_unique<sux_partitioner>();
    p->node = node;
    p->device = node->conf.device;
    p->desc = *d;
    p->desc.range_bounds = nullptr;
    p->pd.kind = d->kind;
    p->pd.R = R;
    p->pd.key_offset = d->key_offset;
    p->pd.key_len = d->key_len;
    p->pd.seed = d->seed;
    p->pd.ascending = d->ascending;
    p->pd.rmagic = sux::part_magic(R);
    if (d->kind == SUX_PART_RANGE_BYTES && R > 1) {
      const int L = d->key_len;
      // strictly rising bounds (RangePartitioner.determineBounds guarantees it)
      for (int i = 1; i + 1 < R; ++i)
        require(std::memcmp(d->range_bounds + (size_t)(i - 1) * L, d->range_bounds + (size_t)i * L,
                            (size_t)L) < 0,
                SUX_EINVAL, "range bounds must be strictly increasing (bound " +
                                std::to_string(i) + ")");
      std::vector<uint64_t> packed(2 * (size_t)(R - 1));
      for (int i = 0; i + 1 < R; ++i) {
        uint8_t k[16] = {0};
        std::memcpy(k, d->range_bounds + (size_t)i * L, (size_t)L);
        uint64_t hi = 0, lo = 0;
        for (int b = 0; b < 8; ++b) hi = (hi << 8) | k[b];
        for (int b = 8; b < 16; ++b) lo = (lo << 8) | k[b];
        packed[2 * i] = hi;
        packed[2 * i + 1] = lo;
      }
      // top-10-bit lookup (4 KiB, LDS-resident in the v3 kernels): candidate answer interval
      // per key prefix
      const int bits = sux::kLutBits;
      std::vector<uint32_t> lut((size_t)1 << bits);
      auto count_less = [&](uint64_t hi, uint64_t lo) {  // #{bounds < (hi, lo)}
        int a = 0, b = R - 1;
        while (a < b) {
          int mid = (a + b) / 2;
          bool less = packed[2 * mid] < hi || (packed[2 * mid] == hi && packed[2 * mid + 1] < lo);
          if (less) a = mid + 1; else b = mid;
        }
        return a;
      };
      for (uint64_t v = 0; v < lut.size(); ++v) {
        uint64_t kmin = v << (64 - bits), kmax = kmin | (~0ull >> bits);
        uint32_t a = (uint32_t)count_less(kmin, 0), b = (uint32_t)count_less(kmax, ~0ull);
        lut[v] = a | (b << 16);
      }
      hip_check(hipMalloc(&p->d_bounds, packed.size() * 8), "hipMalloc(bounds)");
      hip_check(hipMemcpy(p->d_bounds, packed.data(), packed.size() * 8, hipMemcpyHostToDevice),
                "hipMemcpy(bounds)");
      hip_check(hipMalloc(&p->d_lut, lut.size() * 4), "hipMalloc(lut)");
      hip_check(hipMemcpy(p->d_lut, lut.data(), lut.size() * 4, hipMemcpyHostToDevice),
                "hipMemcpy(lut)");
      p->pd.bounds = static_cast<const uint64_t*>(p->d_bounds);
      p->pd.lut = static_cast<const uint32_t*>(p->d_lut);
      p->pd.lut_bits = bits;
    }
    {
      std::lock_guard<std::mutex> lk(node->live_mu);
      node->live_parts.insert(p.get());
    }
    *out = p.release();
  });
}

int sux_partitioner_destroy(sux_partitioner* p) {
  return guard([&] {
    if (!p) return;
    if (p->node) {
      std::lock_guard<std::mutex> lk(p->node->live_mu);
      p->node->live_parts.erase(p);
    }
    hip_check(hipSetDevice(p->device), "hipSetDevice");
    if (p->d_bounds) (void)hipFree(p->d_bounds);
    if (p->d_lut) (void)hipFree(p->d_lut);
    delete p;
  });
}

// ---- stateless map side ----------------------------------------------------------------------
int sux_partition_workspace_size(const sux_partitioner* part, uint32_t rs, uint64_t rpm,
                                 uint64_t n, uint64_t* bytes) {
  return guard([&] {
    require(part && bytes, SUX_EINVAL, "NULL argument");
    Group G = make_group(part, nullptr, rs, rpm, n);
    *bytes = G.ws.total;
  });
}

int sux_partition_maps(sux_node* node, const sux_partitioner* part, const void* d_records,
                       uint32_t rs, uint64_t rpm, uint64_t n, void* d_out, int64_t* d_index,
                       uint8_t* d_index_be, uint16_t* d_pids, void* d_ws, uint64_t ws_bytes,
                       void* stream) {
  return guard([&] {
    require(node && part, SUX_EINVAL, "NULL node/partitioner");
    require(d_records || n == 0, SUX_EINVAL, "records pointer is NULL");
    node->bind();
    Group G = make_group(part, d_records, rs, rpm, n);
    run_group(node, part, G, 1, d_out, d_index, d_index_be, d_pids, nullptr, d_ws, ws_bytes,
              node->stream(stream));
  });
}

int sux_partition_maps_pipelined(sux_node* node, const sux_partitioner* part,
                                 const void* d_records, uint32_t rs, uint64_t rpm, uint64_t n,
                                 uint64_t group_records, void* d_out, int64_t* d_index,
                                 uint8_t* d_index_be, void* stream) {
  return guard([&] {
    require(node && part, SUX_EINVAL, "NULL node/partitioner");
    require(d_records || n == 0, SUX_EINVAL, "records pointer is NULL");
    require(rpm > 0, SUX_EINVAL, "records_per_map must be > 0");
    if (group_records == 0) group_records = std::max<uint64_t>(1, (1ull << 27) / rpm) * rpm;
    require(group_records % rpm == 0, SUX_EINVAL, "group_records must be whole maps");
    require(group_records < (1ull << 32), SUX_ERANGE, "a launch group holds < 2^32 records");
    node->bind();
    if (n == 0) return;
    const uint64_t R = (uint64_t)part->desc.num_partitions;
    const uint64_t first = std::min(n, group_records);
    // every group's workspace fits in the first (largest) group's
    const Group G0 = make_group(part, d_records, rs, rpm, first);
    std::lock_guard<std::mutex> lk(node->pipe_mu);
    node->make_pipe();
    for (int i = 0; i < 2; ++i) {
      if (node->pipe_ws[i].cap < G0.ws.total) {
        hip_check(hipStreamSynchronize(node->pipe[i]), "map stream drain");
        node->pool->put(node->pipe_ws[i]);
        node->pipe_ws[i] = node->pool->get(G0.ws.total);
      }
    }
    hipStream_t s = node->stream(stream);
    const uint8_t* recs = static_cast<const uint8_t*>(d_records);
    uint8_t* out = static_cast<uint8_t*>(d_out);
    const int split = resolve_tuning(node->tuning, true).split_cus;
    if (split > 0 && sux::stream_cus(s) == node->device_cus()) {
      // split mode: K1 of group g on `split` CUs (pipe_split[0]) beside K2 + K3 of group g - 1
      // on the other CUs (pipe_split[1]) — K1 streams at nearly its full rate on a quarter of
      // the CUs while K3, which scales with its CUs, keeps the rest (tools/cu_split_probe.py).
      // A group's workspace slot is reused by group g + 2: its K1 waits for K3 of group g.
      node->make_split(split);
      hipStream_t h = node->pipe_split[0], k = node->pipe_split[1];
      hip_check(hipEventRecord(node->pipe_ev[0], s), "fork");
      hip_check(hipStreamWaitEvent(h, node->pipe_ev[0], 0), "fork");
      hip_check(hipStreamWaitEvent(k, node->pipe_ev[0], 0), "fork");
      for (uint64_t r0 = 0, g = 0; r0 < n; r0 += group_records, ++g) {
        const uint64_t r1 = std::min(n, r0 + group_records), m0 = r0 / rpm;
        const Group G = make_group(part, recs + r0 * rs, rs, rpm, r1 - r0);
        if (g >= 2) hip_check(hipStreamWaitEvent(h, node->split_ev[2 + g % 2], 0), "slot free");
        run_group(node, part, G, 1, out + r0 * rs, d_index + m0 * (R + 1),
                  d_index_be ? d_index_be + m0 * (R + 1) * 8 : nullptr, nullptr, nullptr,
                  node->pipe_ws[g % 2].ptr, node->pipe_ws[g % 2].cap, k, true, h,
                  node->split_ev[g % 2]);
        hip_check(hipEventRecord(node->split_ev[2 + g % 2], k), "slot done");
      }
      hip_check(hipEventRecord(node->pipe_ev[1], k), "join");
      hip_check(hipStreamWaitEvent(s, node->pipe_ev[1], 0), "join");
      hip_check(hipEventRecord(node->pipe_ev[2], h), "join");
      hip_check(hipStreamWaitEvent(s, node->pipe_ev[2], 0), "join");
      return;
    }
    hip_check(hipEventRecord(node->pipe_ev[0], s), "fork");
    for (hipStream_t p : node->pipe) hip_check(hipStreamWaitEvent(p, node->pipe_ev[0], 0), "fork");
    for (uint64_t r0 = 0, g = 0; r0 < n; r0 += group_records, ++g) {
      const uint64_t r1 = std::min(n, r0 + group_records), m0 = r0 / rpm;
      const Group G = make_group(part, recs + r0 * rs, rs, rpm, r1 - r0);
      run_group(node, part, G, 1, out + r0 * rs, d_index + m0 * (R + 1),
                d_index_be ? d_index_be + m0 * (R + 1) * 8 : nullptr, nullptr, nullptr,
                node->pipe_ws[g % 2].ptr, node->pipe_ws[g % 2].cap, node->pipe[g % 2], true);
    }
    for (int i = 0; i < 2; ++i) {
      hip_check(hipEventRecord(node->pipe_ev[1 + i], node->pipe[i]), "join");
      hip_check(hipStreamWaitEvent(s, node->pipe_ev[1 + i], 0), "join");
    }
  });
}

int sux_partition_maps_peer_major(sux_node* node, const sux_partitioner* part,
                                  const void* d_records, uint32_t rs, uint64_t rpm, uint64_t n,
                                  int32_t world, void* d_send, int64_t* d_index,
                                  uint8_t* d_index_be, uint64_t* d_peer_bytes, void* d_ws,
                                  uint64_t ws_bytes, void* stream) {
  return guard([&] {
    require(node && part, SUX_EINVAL, "NULL node/partitioner");
    require(world >= 1 && world <= part->desc.num_partitions && world <= 1024, SUX_EINVAL,
            "world must be in [1, min(R, 1024)]");
    require(d_records || n == 0, SUX_EINVAL, "records pointer is NULL");
    node->bind();
    Group G = make_group(part, d_records, rs, rpm, n);
    run_group(node, part, G, world, d_send, d_index, d_index_be, nullptr, d_peer_bytes, d_ws,
              ws_bytes, node->stream(stream), false, nullptr, nullptr,
              node->own_dev(world, part->desc.num_partitions));
  });
}

int sux_partition_ids(sux_node* node, const sux_partitioner* part, const void* d_records,
                      uint32_t rs, uint64_t n, uint16_t* d_pids, void* stream) {
  return guard([&] {
    require(node && part && (d_records || n == 0) && (d_pids || n == 0), SUX_EINVAL,
            "NULL argument");
    check_record_size(rs);
    check_key_fits(part, rs);
    node->bind();
    hip_check(sux::launch_partition_ids(part->pd, static_cast<const uint8_t*>(d_records), rs, n,
                                        d_pids, node->stream(stream)),
              "pid launch");
  });
}

// ---- variable-length records (Spark SQL UnsafeRowSerializer framing) ---------------------------
}  // extern "C"

namespace {
struct VGroup {
  sux::VarGroup g;
  sux::VarWorkspace ws;
};
VGroup make_vgroup(const sux_partitioner* part, const void* data, const uint64_t* offs,
                   uint64_t rpm, uint64_t n) {
  require(rpm > 0, SUX_EINVAL, "records_per_map must be > 0");
  const uint64_t maps = (n + rpm - 1) / rpm;
  require(maps <= 0xFFFFFFFFull, SUX_EINVAL, "too many maps in one group");
  require(n < (1ull << 32), SUX_ERANGE, "a launch group holds < 2^32 records");
  const int R = part->desc.num_partitions;
  require(R <= sux::kMaxVarPartitions, SUX_EINVAL,
          "variable-length records support num_partitions <= " +
              std::to_string(sux::kMaxVarPartitions));
  require(((uintptr_t)data & 3) == 0 && ((uintptr_t)offs & 7) == 0, SUX_EINVAL,
          "data must be 4-byte and offsets 8-byte aligned");
  VGroup G;
  require(part->node != nullptr, SUX_ESTATE, "the partitioner's node was destroyed");
  const uint32_t tile =
      sux::choose_varlen_tile((uint32_t)R, n, resolve_tuning(part->node->tuning, false));
  G.g.data = static_cast<const uint8_t*>(data);
  G.g.offs = offs;
  G.g.records_per_map = rpm;
  G.g.num_records = n;
  G.g.num_maps = (uint32_t)maps;
  G.g.tile_recs = tile;
  G.g.tiles_per_map = (uint32_t)((rpm + tile - 1) / tile);
  G.g.pad = 0;
  G.ws = sux::varlen_workspace_layout((uint32_t)R, rpm, n, tile);
  return G;
}
}  // namespace

extern "C" {

int sux_partition_varlen_workspace_size(const sux_partitioner* part, uint64_t rpm, uint64_t n,
                                        uint64_t* bytes) {
  return guard([&] {
    require(part && bytes, SUX_EINVAL, "NULL argument");
    *bytes = make_vgroup(part, nullptr, nullptr, rpm, n).ws.total;
  });
}

int sux_partition_varlen(sux_node* node, const sux_partitioner* part, const void* d_data,
                         const uint64_t* d_offsets, uint64_t rpm, uint64_t n,
                         const uint16_t* d_pids_in, void* d_out, int64_t* d_index,
                         uint8_t* d_index_be, uint16_t* d_pids, void* d_ws, uint64_t ws_bytes,
                         void* stream) {
  return guard([&] {
    require(node && part, SUX_EINVAL, "NULL node/partitioner");
    require(d_offsets || n == 0, SUX_EINVAL, "offsets pointer is NULL");
    node->bind();
    VGroup G = make_vgroup(part, d_data, d_offsets, rpm, n);
    require(d_ws || G.ws.total == 0, SUX_EINVAL, "workspace is NULL");
    require(ws_bytes >= G.ws.total, SUX_EINVAL,
            "workspace too small: need " + std::to_string(G.ws.total) + " bytes");
    require(d_out && d_index, SUX_EINVAL, "output or index pointer is NULL");
    require(((uintptr_t)d_out & 3) == 0 && ((uintptr_t)d_index & 7) == 0 &&
                ((uintptr_t)d_index_be & 7) == 0 && ((uintptr_t)d_ws & 255) == 0,
            SUX_EINVAL, "output (4 B), index (8 B) and workspace (256 B) must be aligned");
    if (n == 0) return;
    hip_check(sux::launch_varlen_group(part->pd, G.g, static_cast<uint8_t*>(d_out), d_index,
                                       d_index_be, d_pids_in, d_pids,
                                       static_cast<uint8_t*>(d_ws), G.ws,
                                       resolve_tuning(node->tuning, false), &node->timer,
                                       node->stream(stream)),
              "variable-length partition launch");
  });
}

// ---- compressed map outputs (spark.shuffle.compress with the lz4 codec) ------------------------
}  // extern "C"

namespace {
void check_lz4_args(uint64_t data_bytes, int32_t maps, int32_t R, int32_t bs) {
  require(maps >= 1 && R >= 1 && R <= sux::kMaxPartitions, SUX_EINVAL,
          "num_maps must be >= 1 and num_partitions in [1, 32768]");
  require(bs >= 64 && bs <= 65536 && bs % 4 == 0, SUX_EINVAL,
          "block_size must be a multiple of 4 in [64, 65536], got " + std::to_string(bs));
  require((uint64_t)maps * R < (1ull << 31), SUX_ERANGE, "too many (map, partition) runs");
  require(sux::lz4_chunk_bound(data_bytes, (uint64_t)maps * R, (uint32_t)bs) < (1ull << 32),
          SUX_ERANGE, "too many compression chunks in one call");
}
}  // namespace

extern "C" {

int sux_compress_bound(uint64_t data_bytes, int32_t num_maps, int32_t R, int32_t block_size,
                       uint64_t* bytes) {
  return guard([&] {
    require(bytes, SUX_EINVAL, "NULL argument");
    check_lz4_args(data_bytes, num_maps, R, block_size);
    *bytes = sux::lz4_output_bound(data_bytes, (uint64_t)num_maps * R, (uint32_t)block_size);
  });
}

int sux_compress_workspace_size(uint64_t data_bytes, int32_t num_maps, int32_t R,
                                int32_t block_size, uint64_t* bytes) {
  return guard([&] {
    require(bytes, SUX_EINVAL, "NULL argument");
    check_lz4_args(data_bytes, num_maps, R, block_size);
    *bytes = sux::lz4_workspace_layout(data_bytes, (uint32_t)num_maps, (uint32_t)R,
                                       (uint32_t)block_size).total;
  });
}

int sux_compress_map_outputs(sux_node* node, const void* d_data, uint64_t data_bytes,
                             const int64_t* d_index, int32_t num_maps, int32_t R,
                             int32_t block_size, void* d_out, uint64_t out_capacity,
                             int64_t* d_out_index, uint8_t* d_out_index_be,
                             uint64_t* d_out_bytes, void* d_ws, uint64_t ws_bytes, void* stream) {
  return guard([&] {
    require(node && d_index && d_out && d_out_index, SUX_EINVAL, "NULL argument");
    require(d_data || data_bytes == 0, SUX_EINVAL, "data pointer is NULL");
    check_lz4_args(data_bytes, num_maps, R, block_size);
    const sux::Lz4Workspace w = sux::lz4_workspace_layout(data_bytes, (uint32_t)num_maps,
                                                          (uint32_t)R, (uint32_t)block_size);
    require(d_ws && ws_bytes >= w.total, SUX_EINVAL,
            "workspace too small: need " + std::to_string(w.total) + " bytes");
    require(((uintptr_t)d_ws & 255) == 0 && ((uintptr_t)d_out_index & 7) == 0 &&
                ((uintptr_t)d_out_index_be & 7) == 0 && ((uintptr_t)d_index & 7) == 0,
            SUX_EINVAL, "index (8 B) and workspace (256 B) must be aligned");
    const uint64_t need =
        sux::lz4_output_bound(data_bytes, (uint64_t)num_maps * R, (uint32_t)block_size);
    require(out_capacity >= need, SUX_EINVAL,
            "output capacity too small: need sux_compress_bound = " + std::to_string(need));
    node->bind();
    hip_check(sux::launch_lz4_compress(static_cast<const uint8_t*>(d_data), d_index,
                                       (uint32_t)num_maps, (uint32_t)R, (uint32_t)block_size,
                                       static_cast<uint8_t*>(d_out), d_out_index, d_out_index_be,
                                       d_out_bytes, static_cast<uint8_t*>(d_ws), w,
                                       resolve_tuning(node->tuning, false).lz4_queue,
                                       node->stream(stream)),
              "compress launch");
  });
}

}  // extern "C"
namespace {
void check_lz4d_args(uint64_t in_bytes, int32_t nb, int32_t max_bs) {
  require(nb >= 0 && nb < (1 << 30), SUX_EINVAL, "num_blocks must be in [0, 2^30)");
  require(max_bs >= 64 && max_bs <= 65536, SUX_EINVAL,
          "max_block_size must be in [64, 65536], got " + std::to_string(max_bs));
  require(sux::lz4d_chunk_bound(in_bytes) < (1ull << 32), SUX_ERANGE,
          "too many compressed chunks in one call");
}
}  // namespace
extern "C" {

int sux_decompress_workspace_size(uint64_t in_bytes, int32_t num_blocks, int32_t max_block_size,
                                  uint64_t* bytes) {
  return guard([&] {
    require(bytes, SUX_EINVAL, "NULL argument");
    check_lz4d_args(in_bytes, num_blocks, max_block_size);
    *bytes = sux::lz4d_workspace_layout(in_bytes, (uint32_t)num_blocks).total;
  });
}

int sux_decompress_blocks(sux_node* node, const void* d_in, uint64_t in_bytes,
                          const int64_t* d_in_offsets, int32_t num_blocks, int32_t max_block_size,
                          void* d_out, uint64_t out_capacity, int64_t* d_out_offsets, void* d_ws,
                          uint64_t ws_bytes, void* stream) {
  return guard([&] {
    require(node && d_in_offsets && d_out_offsets, SUX_EINVAL, "NULL argument");
    require(d_in || in_bytes == 0, SUX_EINVAL, "input pointer is NULL");
    check_lz4d_args(in_bytes, num_blocks, max_block_size);
    const sux::Lz4DWorkspace w = sux::lz4d_workspace_layout(in_bytes, (uint32_t)num_blocks);
    require(d_ws && ws_bytes >= w.total, SUX_EINVAL,
            "workspace too small: need " + std::to_string(w.total) + " bytes");
    require(((uintptr_t)d_ws & 255) == 0 && ((uintptr_t)d_in_offsets & 7) == 0 &&
                ((uintptr_t)d_out_offsets & 7) == 0,
            SUX_EINVAL, "offsets (8 B) and workspace (256 B) must be aligned");
    node->bind();
    hip_check(sux::launch_lz4_decompress(static_cast<const uint8_t*>(d_in), in_bytes, d_in_offsets,
                                         (uint32_t)num_blocks, (uint32_t)max_block_size,
                                         static_cast<uint8_t*>(d_out), out_capacity,
                                         d_out_offsets, static_cast<uint8_t*>(d_ws), w,
                                         node->d_err, node->stream(stream)),
              "decompress launch");
  });
}

// ---- local-disk shuffle files (Spark's on-disk format) -------------------------------------------
// The reference keeps Spark's files (it mmaps the committed data file,
// CommonUcxShuffleBlockResolver.scala:45-58) and commits through
// IndexShuffleBlockResolver.writeIndexFileAndCommit [ext] (super call at
// compat/spark_3_0/UcxShuffleBlockResolver.scala:35).  These entry points write / read that format
// from device-resident map outputs, so Spark's local-disk fallback and external shuffle service
// can serve the GPU's outputs.
}  // extern "C"

namespace {
std::mutex g_commit_mu;  // the `synchronized` around Spark's check-and-commit

int64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int k = 0; k < 8; ++k) v = (v << 8) | p[k];
  return (int64_t)v;
}

bool file_size(const std::string& path, int64_t& size) {
  struct stat st;
  if (stat(path.c_str(), &st) != 0) return false;
  size = (int64_t)st.st_size;
  return true;
}

// IndexShuffleBlockResolver.checkIndexAndDataFile [ext]: the committed lengths, or false.
// A missing file has length 0 (java.io.File.length()).
bool check_index_and_data(const std::string& index, const std::string& data, int R,
                          std::vector<int64_t>& lengths) {
  int64_t isz = 0, dsz = 0;
  if (!file_size(index, isz)) isz = 0;
  if (isz != (int64_t)(R + 1) * 8) return false;
  std::vector<uint8_t> buf((size_t)(R + 1) * 8);
  FILE* f = fopen(index.c_str(), "rb");
  if (!f) return false;
  const size_t got = fread(buf.data(), 1, buf.size(), f);
  fclose(f);
  if (got != buf.size() || be64(buf.data()) != 0) return false;
  lengths.assign(R, 0);
  int64_t sum = 0;
  for (int i = 0; i < R; ++i) {
    lengths[i] = be64(buf.data() + 8 * (i + 1)) - be64(buf.data() + 8 * i);
    sum += lengths[i];
  }
  if (!file_size(data, dsz)) dsz = 0;
  return dsz == sum;
}

void write_all(int fd, const uint8_t* p, size_t n, const std::string& what) {
  while (n) {
    const ssize_t w = ::write(fd, p, n);
    if (w < 0 && errno == EINTR) continue;
    require(w > 0, SUX_EIO, "write " + what + ": " + std::strerror(errno));
    p += w;
    n -= (size_t)w;
  }
}

std::string tmp_name(const std::string& path) {
  static std::atomic<uint64_t> ctr{0};
  return path + "." + std::to_string((long)getpid()) + "." + std::to_string(ctr++) + ".tmp";
}

// writeIndexFileAndCommit's body: keep an already committed, consistent pair (another attempt
// of the same map won); otherwise write the index, replace both files by rename.
bool commit_pair(const std::string& index, const std::string& data, const std::string& data_tmp,
                 const int64_t* lengths, int R, int64_t* lengths_out) {
  const std::string itmp = tmp_name(index);
  std::lock_guard<std::mutex> lk(g_commit_mu);
  std::vector<int64_t> existing;
  bool reused = false;
  if (check_index_and_data(index, data, R, existing)) {
    if (lengths_out) std::memcpy(lengths_out, existing.data(), (size_t)R * 8);
    if (!data_tmp.empty()) ::unlink(data_tmp.c_str());
    reused = true;
  } else {
    std::vector<uint8_t> buf((size_t)(R + 1) * 8);
    int64_t off = 0;
    for (int i = 0; i <= R; ++i) {
      store_be64(buf.data() + 8 * i, (uint64_t)off);
      if (i < R) off += lengths[i];
    }
    const int fd = ::open(itmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    require(fd >= 0, SUX_EIO, "open " + itmp + ": " + std::strerror(errno));
    try {
      write_all(fd, buf.data(), buf.size(), itmp);
    } catch (...) {
      ::close(fd);
      ::unlink(itmp.c_str());
      throw;
    }
    ::close(fd);
    ::unlink(index.c_str());
    ::unlink(data.c_str());
    if (::rename(itmp.c_str(), index.c_str()) != 0) {
      ::unlink(itmp.c_str());
      raise(SUX_EIO, "fail to rename file " + itmp + " to " + index);
    }
    if (!data_tmp.empty() && ::access(data_tmp.c_str(), F_OK) == 0 &&
        ::rename(data_tmp.c_str(), data.c_str()) != 0)
      raise(SUX_EIO, "fail to rename file " + data_tmp + " to " + data);
    if (lengths_out) std::memcpy(lengths_out, lengths, (size_t)R * 8);
  }
  ::unlink(itmp.c_str());  // the finally block
  return reused;
}

// Two pinned staging buffers: the D2H copy of chunk k+1 runs while chunk k is written.
struct Staging {
  static constexpr size_t kChunk = 32u << 20;
  uint8_t* h[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  Staging() {
    for (int i = 0; i < 2; ++i) {
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&h[i]), kChunk, hipHostMallocDefault),
                "hipHostMalloc(staging)");
      hip_check(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming), "hipEventCreate");
    }
  }
  ~Staging() {
    for (int i = 0; i < 2; ++i) {
      if (h[i]) (void)hipHostFree(h[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
    }
  }
};

// One map output (n device bytes at src, Spark's lengths[R]) -> a committed data + index file
// pair: D2H of chunk k+1 overlaps the write() of chunk k; temp file, then commit_pair.
void write_map_file(const uint8_t* src, uint64_t n, const int64_t* lengths, int R,
                    const std::string& data, const std::string& index, hipStream_t s,
                    Staging& st, int64_t* lengths_out) {
  const std::string tmp = tmp_name(data);
  const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  require(fd >= 0, SUX_EIO, "open " + tmp + ": " + std::strerror(errno));
  try {
    const uint64_t nch = (n + Staging::kChunk - 1) / Staging::kChunk;
    auto issue = [&](uint64_t k) {
      const uint64_t a = k * Staging::kChunk, len = std::min<uint64_t>(Staging::kChunk, n - a);
      hip_check(hipMemcpyAsync(st.h[k & 1], src + a, len, hipMemcpyDeviceToHost, s),
                "hipMemcpy(data)");
      hip_check(hipEventRecord(st.ev[k & 1], s), "hipEventRecord");
    };
    if (nch) issue(0);
    for (uint64_t k = 0; k < nch; ++k) {
      hip_check(hipEventSynchronize(st.ev[k & 1]), "hipEventSynchronize");
      if (k + 1 < nch) issue(k + 1);
      const uint64_t a = k * Staging::kChunk, len = std::min<uint64_t>(Staging::kChunk, n - a);
      write_all(fd, st.h[k & 1], len, tmp);
    }
  } catch (...) {
    ::close(fd);
    ::unlink(tmp.c_str());
    throw;
  }
  require(::close(fd) == 0, SUX_EIO, "close " + tmp);
  commit_pair(index, data, tmp, lengths, R, lengths_out);
}

// Bytes [off, off + n) of a file -> device memory (pinned double buffer: the pread of chunk k+1
// overlaps the H2D copy of chunk k).  Waits for the copies.
void read_file_range(const std::string& path, uint64_t off, uint64_t n, uint8_t* dst,
                     hipStream_t s, Staging& st) {
  if (n == 0) return;
  const int fd = ::open(path.c_str(), O_RDONLY);
  require(fd >= 0, SUX_EIO, "open " + path + ": " + std::strerror(errno));
  try {
    const uint64_t nch = (n + Staging::kChunk - 1) / Staging::kChunk;
    for (uint64_t k = 0; k < nch; ++k) {
      const uint64_t o = k * Staging::kChunk, len = std::min<uint64_t>(Staging::kChunk, n - o);
      if (k >= 2) hip_check(hipEventSynchronize(st.ev[k & 1]), "hipEventSynchronize");
      uint64_t done = 0;
      while (done < len) {
        const ssize_t r = ::pread(fd, st.h[k & 1] + done, len - done, (off_t)(off + o + done));
        if (r < 0 && errno == EINTR) continue;
        require(r > 0, SUX_EIO, "read " + path + ": short file");
        done += (uint64_t)r;
      }
      hip_check(hipMemcpyAsync(dst + o, st.h[k & 1], len, hipMemcpyHostToDevice, s),
                "hipMemcpy(blocks)");
      hip_check(hipEventRecord(st.ev[k & 1], s), "hipEventRecord");
    }
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
}

// HBM-capacity fallback: spill whole slabs of committed, device-resident map outputs (world 1:
// Spark's data files as they stand) to Spark's files under the spill directory until `need`
// bytes of pool memory were returned, then free the pool's idle allocations.  Returns false
// when nothing could be spilled.  The reference's map outputs live in such files from the start
// (CommonUcxShuffleBlockResolver.scala:45-58 mmaps them).
bool spill_some(sux_node* node, uint64_t need) {
  std::unique_lock<std::mutex> lk(node->mu);
  if (node->spill_dir.empty() || node->conf.world_size != 1) return false;
  // candidate slabs: pool-owned, every map on them published and device-resident; oldest
  // shuffle and lowest map first (the reducers of early maps run first)
  std::vector<std::pair<Slab*, std::vector<std::pair<Shuffle*, int32_t>>>> victims;
  std::map<Slab*, size_t> at;
  for (auto& kv : node->shuffles) {
    Shuffle& sh = *kv.second;
    if (sh.zero_copy) continue;  // resolved addresses may still be read
    for (int32_t m = 0; m < sh.num_maps; ++m) {
      MapSlot& sl = sh.maps[m];
      if (!(sl.present && !sl.spilled() && sl.slab && sl.slab->pool && sl.owner == node->conf.rank))
        continue;
      auto f = at.find(sl.slab.get());
      if (f == at.end()) {
        f = at.emplace(sl.slab.get(), victims.size()).first;
        victims.push_back({sl.slab.get(), {}});
      }
      victims[f->second].second.push_back({&sh, m});
    }
  }
  if (victims.empty()) return false;
  // in-flight readers of these buffers (fetch copies, exchanges) finish first
  hip_check(hipDeviceSynchronize(), "sync before spill");
  hipStream_t s = nullptr;
  hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "spill stream");
  uint64_t freed = 0;
  try {
    Staging st;
    for (auto& v : victims) {
      if (freed >= need) break;
      // a slab some reader still holds (a fetch's copy, an exchange) would stay allocated:
      // spilling its maps frees nothing now
      const auto& s0 = v.second.front();
      if ((size_t)s0.first->maps[s0.second].slab.use_count() > v.second.size()) continue;
      const uint64_t cap = v.first->buf.cap;
      for (auto& sm : v.second) {
        Shuffle& sh = *sm.first;
        MapSlot& sl = sh.maps[sm.second];
        const std::string base = node->spill_dir + "/shuffle_" + std::to_string(sh.id) + "_" +
                                 std::to_string(sm.second) + "_0";
        std::vector<int64_t> lengths((size_t)sh.R);
        const std::vector<int64_t>& ix = host_index(sl, sh.R);
        for (int p = 0; p < sh.R; ++p) lengths[p] = ix[p + 1] - ix[p];
        write_map_file(sl.data(), sl.bytes, lengths.data(), sh.R, base + ".data", base + ".index",
                       s, st, nullptr);
        sl.spill_data = base + ".data";
        sl.spill_index = base + ".index";
        sl.d_index = nullptr;  // (host_index above made the host copy)
        sl.slab.reset();
        node->spills++;
      }
      freed += cap;
    }
  } catch (...) {
    (void)hipStreamDestroy(s);
    throw;
  }
  (void)hipStreamDestroy(s);
  lk.unlock();
  node->pool->trim();
  return freed > 0;
}

// A pool buffer; on SUX_ENOMEM spill map outputs (if configured) and retry.
// Idle cached allocations go back first (a fetch after the writes spilled everything they could
// finds the pool full of the writers' freed workspaces and slabs, not of map outputs).
PoolBuf pool_get_or_spill(sux_node* node, uint64_t bytes) {
  for (int attempt = 0;; ++attempt) {
    try {
      return node->pool->get(bytes);
    } catch (const SuxError& e) {
      if (e.code != SUX_ENOMEM || attempt >= 64) throw;
      if (node->pool->trim() > 0) continue;
      if (!spill_some(node, bytes)) throw;
    }
  }
}
}  // namespace

extern "C" {

int sux_index_file_commit(const char* index_path, const char* data_path, const char* data_tmp,
                          const int64_t* lengths, int32_t R, int64_t* lengths_out,
                          int32_t* reused) {
  return guard([&] {
    require(index_path && data_path && (lengths || R == 0), SUX_EINVAL, "NULL argument");
    require(R >= 0, SUX_EINVAL, "num_partitions < 0");
    const bool r = commit_pair(index_path, data_path, data_tmp ? data_tmp : "", lengths, R,
                               lengths_out);
    if (reused) *reused = r ? 1 : 0;
  });
}

int sux_write_map_files(sux_node* node, const void* d_data, const int64_t* d_index,
                        int32_t num_maps, int32_t R, const char* const* data_paths,
                        const char* const* index_paths, int64_t* lengths_out, void* stream) {
  return guard([&] {
    require(node && d_index && data_paths && index_paths, SUX_EINVAL, "NULL argument");
    require(num_maps >= 1 && R >= 1, SUX_EINVAL, "num_maps and num_partitions must be >= 1");
    node->bind();
    hipStream_t s = node->stream(stream);
    std::vector<int64_t> ix((size_t)num_maps * (R + 1));
    hip_check(hipMemcpyAsync(ix.data(), d_index, ix.size() * 8, hipMemcpyDeviceToHost, s),
              "hipMemcpy(index)");
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    Staging st;
    uint64_t base = 0;
    for (int32_t m = 0; m < num_maps; ++m) {
      const int64_t* im = ix.data() + (size_t)m * (R + 1);
      require(im[0] == 0, SUX_EINVAL, "index table of map " + std::to_string(m) + " does not start at 0");
      std::vector<int64_t> lengths(R);
      for (int p = 0; p < R; ++p) lengths[p] = im[p + 1] - im[p];
      const uint64_t n = (uint64_t)im[R];
      require(d_data || n == 0, SUX_EINVAL, "data pointer is NULL");
      write_map_file(static_cast<const uint8_t*>(d_data) + base, n, lengths.data(), R,
                     data_paths[m], index_paths[m], s, st,
                     lengths_out ? lengths_out + (size_t)m * R : nullptr);
      base += n;
    }
  });
}

int sux_read_file_blocks(sux_node* node, const char* data_path, const char* index_path, int32_t R,
                         int32_t start_partition, int32_t end_partition, void* d_dst,
                         uint64_t capacity, uint64_t* bytes, void* stream) {
  return guard([&] {
    require(node && data_path && index_path && bytes, SUX_EINVAL, "NULL argument");
    require(0 <= start_partition && start_partition <= end_partition && end_partition <= R,
            SUX_EINVAL, "partition range must satisfy 0 <= start <= end <= R");
    std::vector<int64_t> lengths;
    {
      int64_t isz = 0;
      require(file_size(index_path, isz) && isz == (int64_t)(R + 1) * 8, SUX_EIO,
              std::string("index file ") + index_path + " is not " + std::to_string(R + 1) +
                  " offsets");
    }
    std::vector<uint8_t> ib((size_t)(R + 1) * 8);
    FILE* f = fopen(index_path, "rb");
    require(f != nullptr, SUX_EIO, std::string("open ") + index_path);
    const size_t got = fread(ib.data(), 1, ib.size(), f);
    fclose(f);
    require(got == ib.size(), SUX_EIO, std::string("read ") + index_path);
    const int64_t a = be64(ib.data() + 8 * start_partition), e = be64(ib.data() + 8 * end_partition);
    require(0 <= a && a <= e, SUX_EIO, "index offsets decrease");
    const uint64_t n = (uint64_t)(e - a);
    require(n <= capacity && (d_dst || n == 0), SUX_ERANGE,
            "blocks need " + std::to_string(n) + " bytes, capacity " + std::to_string(capacity));
    *bytes = n;
    if (n == 0) return;
    node->bind();
    Staging st;
    read_file_range(data_path, (uint64_t)a, n, static_cast<uint8_t*>(d_dst), node->stream(stream),
                    st);
  });
}

// ---- exchange plan (host arithmetic) -----------------------------------------------------------
int sux_plan_ownership(int32_t W, int32_t R, const int64_t* bytes, int32_t* own) {
  return host_guard([&] {
    require(W >= 1 && R >= W && bytes && own, SUX_EINVAL, "bad ownership shape");
    // min over contiguous splits into W non-empty ranges of the largest range's bytes: binary
    // search on that cap; a cap is feasible when greedy ranges — each as long as the cap allows,
    // leaving one partition for every owner after it — cover all R partitions
    int64_t total = 0, most = 0;
    for (int p = 0; p < R; ++p) {
      require(bytes[p] >= 0, SUX_EINVAL, "negative partition size");
      total += bytes[p];
      most = std::max(most, bytes[p]);
    }
    auto fill = [&](int64_t cap, int32_t* out) {
      int p = 0;
      for (int h = 0; h < W; ++h) {
        if (out) out[h] = p;
        if (h == W - 1) {
          int64_t rest = 0;
          for (int q = p; q < R; ++q) rest += bytes[q];
          p = R;
          if (rest > cap) return false;
          break;
        }
        int64_t sum = bytes[p++];  // every owner takes at least one partition
        if (sum > cap) return false;
        while (p < R - (W - 1 - h) && sum + bytes[p] <= cap) sum += bytes[p++];
      }
      if (out) out[W] = R;
      return p == R;
    };
    int64_t lo = most, hi = total;  // fill(hi) always succeeds
    while (lo < hi) {
      const int64_t mid = lo + (hi - lo) / 2;
      if (fill(mid, nullptr)) hi = mid; else lo = mid + 1;
    }
    const bool ok = fill(lo, own);
    require(ok, SUX_EINVAL, "ownership plan failed");
  });
}

int sux_node_set_ownership(sux_node* node, int32_t W, int32_t R, const int32_t* own) {
  return guard([&] {
    require(node && W >= 1 && R >= W, SUX_EINVAL, "bad ownership shape");
    if (own) check_ownership(W, R, own);
    node->bind();
    std::lock_guard<std::mutex> lk(node->mu);
    // a posted exchange keeps the table it was posted with (its ticket's snapshot), but a table
    // changed between post and issue would no longer match the send buffer's layout: refuse it
    // 
    require(node->tickets.empty(), SUX_ESTATE,
            "exchange groups are posted and not yet issued: set the ownership between shuffles");
    if (!own) {
      node->own.clear();
      return;
    }
    // the node's streams are non-blocking (a null-stream copy does not order against them): every
    // partition or pull launch still reading the old table completes first
    hip_check(hipDeviceSynchronize(), "sync before the ownership update");
    if (!node->d_own || node->own_W < W) {
      if (node->d_own) (void)hipFree(node->d_own);
      node->d_own = nullptr;
      hip_check(hipMalloc(&node->d_own, sizeof(int32_t) * (W + 1)), "hipMalloc(ownership)");
    }
    hip_check(hipMemcpy(node->d_own, own, sizeof(int32_t) * (W + 1), hipMemcpyHostToDevice),
              "ownership upload");
    node->own.assign(own, own + W + 1);
    node->own_W = W;
    node->own_R = R;
  });
}

int sux_plan_group(int32_t W, int32_t rank, int32_t M, int32_t R, const int64_t* gi,
                   uint64_t* sendcounts, uint64_t* sdispls, uint64_t* recvcounts,
                   uint64_t* rdispls) {
  return sux_plan_group_owned(W, rank, M, R, gi, nullptr, sendcounts, sdispls, recvcounts,
                              rdispls);
}

int sux_plan_group_owned(int32_t W, int32_t rank, int32_t M, int32_t R, const int64_t* gi,
                         const int32_t* own, uint64_t* sendcounts, uint64_t* sdispls,
                         uint64_t* recvcounts, uint64_t* rdispls) {
  return guard([&] {
    require(W >= 1 && rank >= 0 && rank < W && M >= 0 && R >= W, SUX_EINVAL, "bad plan shape");
    require(gi || M == 0, SUX_EINVAL, "gathered index is NULL");
    if (own) check_ownership(W, R, own);
    const int64_t stride = (int64_t)R + 1;
    auto idx = [&](int g, int m, int p) { return gi[((int64_t)g * M + m) * stride + p]; };
    uint64_t sacc = 0, racc = 0;
    for (int h = 0; h < W; ++h) {
      int lo = own_lo(own, h, R, W), hi = own_lo(own, h + 1, R, W);
      uint64_t s = 0;
      for (int m = 0; m < M; ++m) s += (uint64_t)(idx(rank, m, hi) - idx(rank, m, lo));
      if (sendcounts) sendcounts[h] = s;
      if (sdispls) sdispls[h] = sacc;
      sacc += s;
    }
    int lo = own_lo(own, rank, R, W), hi = own_lo(own, rank + 1, R, W);
    for (int g = 0; g < W; ++g) {
      uint64_t r = 0;
      for (int m = 0; m < M; ++m) r += (uint64_t)(idx(g, m, hi) - idx(g, m, lo));
      if (recvcounts) recvcounts[g] = r;
      if (rdispls) rdispls[g] = racc;
      racc += r;
    }
  });
}

int64_t sux_plan_block_offset(int32_t W, int32_t rank, int32_t M, int32_t R, const int64_t* gi,
                              int32_t g, int32_t m, int32_t p) {
  return sux_plan_block_offset_owned(W, rank, M, R, gi, nullptr, g, m, p);
}

int64_t sux_plan_block_offset_owned(int32_t W, int32_t rank, int32_t M, int32_t R,
                                    const int64_t* gi, const int32_t* own, int32_t g, int32_t m,
                                    int32_t p) {
  if (!gi || W < 1 || rank < 0 || rank >= W || g < 0 || g >= W || m < 0 || m >= M || R < W)
    return -1;
  int lo = own_lo(own, rank, R, W), hi = own_lo(own, rank + 1, R, W);
  if (p < lo || p >= hi) return -1;
  const int64_t stride = (int64_t)R + 1;
  auto idx = [&](int gg, int mm, int pp) { return gi[((int64_t)gg * M + mm) * stride + pp]; };
  int64_t off = 0;
  for (int gg = 0; gg < g; ++gg)
    for (int mm = 0; mm < M; ++mm) off += idx(gg, mm, hi) - idx(gg, mm, lo);
  for (int mm = 0; mm < m; ++mm) off += idx(g, mm, hi) - idx(g, mm, lo);
  return off + idx(g, m, p) - idx(g, m, lo);
}

int sux_exchange_group(sux_node* node, const void* d_send, const int64_t* d_index, int32_t M,
                       int32_t R, int64_t* d_gathered, void* d_recv, uint64_t recv_capacity,
                       uint64_t* recv_bytes, void* stream) {
  return guard([&] {
    require(node && d_index && d_gathered, SUX_EINVAL, "NULL argument");
    const int W = node->conf.world_size, rank = node->conf.rank;
    require(R >= W && M >= 1, SUX_EINVAL, "need R >= world and >= 1 map");
    node->bind();
    hipStream_t s = node->stream(stream);
    const size_t per_rank = (size_t)M * (R + 1);
    // pinned staging (node->hpool): the read-back is a true async copy, not a pageable bounce
    HostLease hb(node->hpool, per_rank * W * 8);
    int64_t* host = static_cast<int64_t*>(hb.b.first);
    if (!node->comm) {
      hip_check(hipMemcpyAsync(d_gathered, d_index, per_rank * 8, hipMemcpyDeviceToDevice, s),
                "copy index");
    } else {
      nccl_check(ncclAllGather(d_index, d_gathered, per_rank, ncclInt64, node->comm, s),
                 "ncclAllGather(index)");
    }
    hip_check(hipMemcpyAsync(host, d_gathered, per_rank * W * 8, hipMemcpyDeviceToHost, s),
              "D2H gathered index");
    hip_check(hipStreamSynchronize(s), "sync gathered index");
    std::vector<uint64_t> sc(W), sd(W), rc(W), rd(W);
    int rc_plan = sux_plan_group_owned(W, rank, M, R, host, node->own_host(W, R), sc.data(),
                                       sd.data(), rc.data(), rd.data());
    require(rc_plan == SUX_OK, rc_plan, g_err);
    uint64_t total = rd[W - 1] + rc[W - 1];
    require(total <= recv_capacity, SUX_ERANGE,
            "receive buffer too small: need " + std::to_string(total) + " bytes");
    if (recv_bytes)
      for (int g = 0; g < W; ++g) recv_bytes[g] = rc[g];
    if (!node->comm) {
      if (total)
        hip_check(hipMemcpyAsync(d_recv, d_send, total, hipMemcpyDeviceToDevice, s), "self copy");
      return;
    }
    require(d_send && d_recv, SUX_EINVAL, "send/recv buffer is NULL");
    all_to_all_pieces(static_cast<const uint8_t*>(d_send), sc.data(), sd.data(),
                      static_cast<uint8_t*>(d_recv), rc.data(), rd.data(), W, node->comm, s);
  });
}

// ---- the same exchange in two halves (no host wait in front of an all-to-all) -------------------
}  // extern "C"
struct sux_xticket {
  int32_t M = 0, R = 0;
  std::vector<int32_t> own;  // the ownership table at post time (empty: the equal split)
  int64_t* d_gathered = nullptr;
  std::unique_ptr<HostLease> host;  // the gathered index tables, read back asynchronously
  Event done;                       // after the read-back
};
void free_ticket(sux_xticket* t) {
  (void)hipEventSynchronize(t->done.e);
  delete t;
}
extern "C" {

int sux_exchange_group_post(sux_node* node, const int64_t* d_index, int32_t M, int32_t R,
                            int64_t* d_gathered, void* stream, sux_xticket** out) {
  return guard([&] {
    require(node && d_index && d_gathered && out, SUX_EINVAL, "NULL argument");
    const int W = node->conf.world_size;
    require(R >= W && M >= 1, SUX_EINVAL, "need R >= world and >= 1 map");
    node->bind();
    hipStream_t s = node->stream(stream);
    if (node->comm && !node->comm_x)  // collective: every rank's first post makes it
      nccl_check(ncclCommSplit(node->comm, 0, node->conf.rank, &node->comm_x, nullptr),
                 "ncclCommSplit");
    const size_t per_rank = (size_t)M * (R + 1);
    auto t = std::make_unique<sux_xticket>();
    t->M = M;
    t->R = R;
    t->d_gathered = d_gathered;
    {
      std::lock_guard<std::mutex> lk(node->mu);
      if (const int32_t* o = node->own_host(W, R)) t->own.assign(o, o + W + 1);
    }
    t->host = std::make_unique<HostLease>(node->hpool, per_rank * W * 8);
    if (!node->comm)
      hip_check(hipMemcpyAsync(d_gathered, d_index, per_rank * 8, hipMemcpyDeviceToDevice, s),
                "copy index");
    else
      nccl_check(ncclAllGather(d_index, d_gathered, per_rank, ncclInt64, node->comm, s),
                 "ncclAllGather(index)");
    hip_check(hipMemcpyAsync(t->host->b.first, d_gathered, per_rank * W * 8,
                             hipMemcpyDeviceToHost, s),
              "D2H gathered index");
    hip_check(hipEventRecord(t->done.e, s), "hipEventRecord(gathered index)");
    std::lock_guard<std::mutex> lk(node->mu);
    node->tickets.insert(t.get());
    *out = t.release();
  });
}

int sux_exchange_group_discard(sux_node* node, sux_xticket* ticket) {
  std::unique_ptr<sux_xticket> t(ticket);
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    if (!t) return;
    {
      std::lock_guard<std::mutex> lk(node->mu);
      node->tickets.erase(t.get());
    }
    node->bind();
    // the read-back into the pinned lease must land before the lease goes back to the pool
    (void)hipEventSynchronize(t->done.e);
  });
}

int sux_exchange_group_issue(sux_node* node, sux_xticket* ticket, const void* d_send,
                             void* d_recv, uint64_t recv_capacity, uint64_t* recv_bytes,
                             void* stream) {
  std::unique_ptr<sux_xticket> t(ticket);  // consumed, whatever happens
  if (node && ticket) {
    std::lock_guard<std::mutex> lk(node->mu);
    node->tickets.erase(ticket);
  }
  return guard([&] {
    require(node && t, SUX_EINVAL, "NULL argument");
    const int W = node->conf.world_size, rank = node->conf.rank;
    node->bind();
    hipStream_t s = node->stream(stream);
    // the host waits here for the read-back posted a launch group earlier (long done when the
    // caller issues group k - 1 after posting group k); `stream` itself never waits on the host
    hip_check(hipEventSynchronize(t->done.e), "sync gathered index");
    std::vector<uint64_t> sc(W), sd(W), rc(W), rd(W);
    int rc_plan = sux_plan_group_owned(W, rank, t->M, t->R,
                                       static_cast<const int64_t*>(t->host->b.first),
                                       t->own.empty() ? nullptr : t->own.data(), sc.data(),
                                       sd.data(), rc.data(), rd.data());
    require(rc_plan == SUX_OK, rc_plan, g_err);
    const uint64_t total = rd[W - 1] + rc[W - 1];
    require(total <= recv_capacity, SUX_ERANGE,
            "receive buffer too small: need " + std::to_string(total) + " bytes");
    if (recv_bytes)
      for (int g = 0; g < W; ++g) recv_bytes[g] = rc[g];
    if (!node->comm) {
      if (total)
        hip_check(hipMemcpyAsync(d_recv, d_send, total, hipMemcpyDeviceToDevice, s), "self copy");
      return;
    }
    require(d_send && d_recv, SUX_EINVAL, "send/recv buffer is NULL");
    all_to_all_pieces(static_cast<const uint8_t*>(d_send), sc.data(), sd.data(),
                      static_cast<uint8_t*>(d_recv), rc.data(), rd.data(), W,
                      node->comm_x ? node->comm_x : node->comm, s);
  });
}

// ---- one-sided exchange over HIP IPC ----------------------------------------------------------
int sux_ipc_export(sux_node* node, const void* d_ptr, uint8_t out[SUX_IPC_DESC_BYTES]) {
  return guard([&] {
    require(node && d_ptr && out, SUX_EINVAL, "NULL argument");
    node->bind();
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "hipIpcMemHandle_t is 64 bytes");
    export_ipc(node, d_ptr, out);
  });
}

int sux_ipc_open(sux_node* node, const uint8_t desc[SUX_IPC_DESC_BYTES], void** d_ptr) {
  return guard([&] {
    require(node && desc && d_ptr, SUX_EINVAL, "NULL argument");
    node->bind();
    uint64_t off;
    std::memcpy(&off, desc + 64, 8);
    void* base = ipc_open_fresh(node, desc);
    *d_ptr = static_cast<uint8_t*>(base) + off;
    std::lock_guard<std::mutex> lk(node->mu);
    auto& slot = node->ipc_bases[*d_ptr];
    if (slot.first) ipc_close_ref(node, slot.first, slot.second);  // opened twice: one reference
    slot = {base, std::string(reinterpret_cast<const char*>(desc), 64)};
  });
}

int sux_ipc_close(sux_node* node, void* d_ptr) {
  return guard([&] {
    require(node && d_ptr, SUX_EINVAL, "NULL argument");
    node->bind();
    std::pair<void*, std::string> m;
    {
      std::lock_guard<std::mutex> lk(node->mu);
      auto it = node->ipc_bases.find(d_ptr);
      require(it != node->ipc_bases.end(), SUX_ENOENT, "pointer was not opened by sux_ipc_open");
      m = it->second;
      node->ipc_bases.erase(it);
    }
    ipc_close_ref(node, m.first, m.second);
  });
}

int sux_pull_group(sux_node* node, int32_t W, int32_t rank, const uint64_t* d_src_ptrs,
                   const int64_t* d_gathered, int32_t M, int32_t R, void* d_recv, uint64_t cap,
                   uint64_t* d_recv_bytes, void* stream) {
  return guard([&] {
    require(node && d_src_ptrs && d_gathered && d_recv, SUX_EINVAL, "NULL argument");
    require(W >= 1 && rank >= 0 && rank < W && M >= 1 && R >= W, SUX_EINVAL, "bad pull shape");
    node->bind();
    hip_check(sux::launch_pull(W, rank, d_src_ptrs, d_gathered, M, R,
                               static_cast<uint8_t*>(d_recv), cap, d_recv_bytes,
                               node->stream(stream), node->own_dev(W, R)),
              "pull launch");
  });
}

// ---- shuffle lifecycle ---------------------------------------------------------------------
int sux_register_shuffle(sux_node* node, int32_t shuffle_id, int32_t num_maps, int32_t R,
                         int32_t rec_size, sux_handle_desc* out) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    require(num_maps >= 0 && R >= 1 && R <= sux::kMaxPartitions, SUX_EINVAL,
            "bad num_maps/num_partitions");
    check_record_size((uint32_t)rec_size);
    std::lock_guard<std::mutex> lk(node->mu);
    require(!node->shuffles.count(shuffle_id), SUX_ESTATE,
            "shuffle " + std::to_string(shuffle_id) + " already registered");
    auto sh = std::make_unique<Shuffle>();
    sh->id = shuffle_id;
    sh->num_maps = num_maps;
    sh->R = R;
    sh->rec_size = rec_size;
    sh->maps.resize((size_t)num_maps);
    sh->directory.assign((size_t)num_maps * node->conf.metadata_block_size, 0);
    if (out) {
      out->shuffle_id = shuffle_id;
      out->num_maps = num_maps;
      out->num_partitions = R;
      out->record_size = rec_size;
      out->directory_bytes = sh->directory.size();
    }
    node->shuffles[shuffle_id] = std::move(sh);
  });
}

int sux_shuffle_set_codec(sux_node* node, int32_t shuffle_id, int32_t codec, int32_t block_size) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    require(codec == SUX_CODEC_NONE || codec == SUX_CODEC_LZ4, SUX_EINVAL,
            "codec must be SUX_CODEC_NONE or SUX_CODEC_LZ4, got " + std::to_string(codec));
    if (codec == SUX_CODEC_LZ4)
      require(block_size >= 64 && block_size <= 65536 && block_size % 4 == 0, SUX_EINVAL,
              "spark.io.compression.lz4.blockSize must be a multiple of 4 in [64, 65536], got " +
                  std::to_string(block_size));
    std::lock_guard<std::mutex> lk(node->mu);
    Shuffle& sh = node->shuffle(shuffle_id);
    bool written = !sh.jobs.empty() || sh.submitting > 0 || sh.busy > 0;
    for (const MapSlot& m : sh.maps) written = written || m.present || m.pending;
    require(!written, SUX_ESTATE,
            "shuffle " + std::to_string(shuffle_id) + " already has map outputs: set its codec first");
    sh.codec = codec;
    sh.codec_block = codec == SUX_CODEC_LZ4 ? block_size : 0;
  });
}

int sux_unregister_shuffle(sux_node* node, int32_t shuffle_id) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    node->bind();
    std::unique_ptr<Shuffle> gone;
    {
      std::unique_lock<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      require(!sh.exchanging, SUX_ESTATE, "shuffle " + std::to_string(shuffle_id) + " is exchanging");
      // IPC pulls: peers may still read this rank's slabs until the closing all-gather
      require(!sh.ack_due, SUX_ESTATE,
              "shuffle " + std::to_string(shuffle_id) +
                  " has an exchange not yet completed by sux_exchange_wait");
      drain(node, sh, lk);  // writes in flight finish before their slabs go back
      gone = std::move(node->shuffles[shuffle_id]);
      node->shuffles.erase(shuffle_id);
    }
    // no lock held: readers of this shuffle's buffers are ordered before this call by the
    // caller (CommonUcxShuffleBlockResolver.removeShuffle runs after the stage)
    hip_check(hipDeviceSynchronize(), "sync before unregister");
    release_shuffle(node, *gone);
  });
}

int sux_write_map_outputs(sux_node* node, int32_t shuffle_id, int32_t first,
                          const sux_partitioner* part, const void* d_records, uint64_t rpm,
                          uint64_t n, void* stream) {
  return guard([&] {
    require(node && part, SUX_EINVAL, "NULL node/partitioner");
    require(d_records || n == 0, SUX_EINVAL, "records pointer is NULL");
    require(rpm > 0, SUX_EINVAL, "records_per_map must be > 0");
    node->bind();
    hipStream_t s = node->stream(stream);
    const uint64_t maps = (n + rpm - 1) / rpm;
    auto job = std::make_unique<WriteJob>();
    int R = 0;
    uint32_t rs = 0;
    int32_t codec = SUX_CODEC_NONE, cblock = 0;
    {
      std::unique_lock<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      codec = sh.codec;
      cblock = sh.codec_block;
      require(first >= 0 && (uint64_t)first + maps <= (uint64_t)sh.num_maps, SUX_EINVAL,
              "maps [" + std::to_string(first) + ", " + std::to_string((uint64_t)first + maps) +
                  ") out of [0, " + std::to_string(sh.num_maps) + ")");
      require(part->desc.num_partitions == sh.R, SUX_EINVAL,
              "partitioner has " + std::to_string(part->desc.num_partitions) +
                  " partitions, shuffle has " + std::to_string(sh.R));
      require(sh.R >= node->conf.world_size, SUX_EINVAL, "need at least one partition per rank");
      progress(node, sh, lk, false);
      R = sh.R;
      rs = (uint32_t)sh.rec_size;
      // UcxShuffleBlockResolver.scala:42-45: an empty data file publishes nothing;
      // IndexShuffleBlockResolver [ext]: a map another attempt committed (or is writing) keeps
      // the first commit
      job->claimed.assign((size_t)maps, 0);
      bool any = false;
      for (uint64_t k = 0; k < maps; ++k) {
        MapSlot& sl = sh.maps[first + k];
        if (sl.present || sl.pending) continue;
        sl.pending = true;
        job->claimed[k] = 1;
        any = true;
      }
      if (!any) return;
      sh.submitting++;
    }
    job->first = first;
    job->maps = (uint32_t)maps;
    job->rpm = rpm;
    job->n = n;
    auto unclaim = [&] {  // a failed launch leaves the maps writable again
      std::lock_guard<std::mutex> lk(node->mu);
      auto it = node->shuffles.find(shuffle_id);
      if (it != node->shuffles.end()) {
        for (uint64_t k = 0; k < maps; ++k)
          if (job->claimed[k]) it->second->maps[first + k].pending = false;
        it->second->submitting--;
      }
      node->cv.notify_all();
    };
    // Map tasks run several at a time in Spark (one per executor core): consecutive batches go
    // round robin to the node's two map streams, so that one batch's K1 runs beside the other's
    // K3 (the co-resident shapes of sux_partition_maps_pipelined).  Forked from the caller's
    // stream (its input is ready there) and joined back into it (the caller may reuse the
    // input buffer after its own stream's later work, as with a launch on `stream` itself).
    hipStream_t ms = s;
    // at world > 1 the batch is written peer-major: every peer's share of it is one contiguous
    // range, so the exchange sends the slab as it stands (one all-to-all per batch, no repack)
    const int32_t W = node->conf.world_size;
    job->world = W;
    const bool lz4 = codec == SUX_CODEC_LZ4;
    try {
      Group G = make_group(part, d_records, rs, rpm, n);
      auto up = [](uint64_t v) { return (v + 255) / 256 * 256; };
      const uint64_t ix_bytes = 8 * maps * (uint64_t)(R + 1);
      // compressed shuffle: the maps are partitioned map-major into scratch (`plain`), then every
      // non-empty (map, partition) run is compressed into the slab as its own LZ4Block stream —
      // the per-partition wrapStream of Spark's writers under spark.shuffle.compress — and the
      // committed index is the compressed one (the MapStatus lengths are compressed lengths)
      sux::Lz4Workspace lw{};
      uint64_t plain_off = 0, lws_off = 0, cix_off = 0, cbytes_off = 0, ws_total = 0;
      uint64_t slab_bytes = n * rs;
      if (lz4) {
        check_lz4_args(n * rs, (int32_t)maps, R, cblock);
        lw = sux::lz4_workspace_layout(n * rs, (uint32_t)maps, (uint32_t)R, (uint32_t)cblock);
        slab_bytes = sux::lz4_output_bound(n * rs, maps * (uint64_t)R, (uint32_t)cblock);
        plain_off = up(G.ws.total) + up(ix_bytes);
        lws_off = plain_off + up(n * rs);
        cix_off = lws_off + up(lw.total);
        cbytes_off = cix_off + up(ix_bytes);
        ws_total = cbytes_off + 256;
      } else {
        ws_total = G.ws.total + ix_bytes + 256;
      }
      job->slab = std::make_shared<Slab>(node->pool.get(), pool_get_or_spill(node, slab_bytes));
      job->ws = pool_get_or_spill(node, ws_total);
      int64_t* d_idx = reinterpret_cast<int64_t*>(job->ws.ptr + (G.ws.total + 255) / 256 * 256);
      if (lz4) {
        // packed map-major outputs at any world (each map its own exchange piece at W > 1, like
        // a committed data file); the compressed index tables come back to the host
        job->world = 1;
        job->packed = true;
        job->hidx = node->hpool.get(ix_bytes);
      } else if (W == 1) {
        // world 1: the index tables stay on the device with the slab (no maps x (R + 1) read-back
        // per batch; resolves gather the entries they need, host_index the rest on demand)
        job->slab->aux = pool_get_or_spill(node, 8 * maps * (uint64_t)(R + 1));
        d_idx = reinterpret_cast<int64_t*>(job->slab->aux.ptr);
        job->dindex = d_idx;
        job->rs = (uint32_t)rs;
      } else {
        job->hidx = node->hpool.get(8 * maps * (uint64_t)(R + 1));
      }
      {
        std::lock_guard<std::mutex> lk(node->mu);
        // packed at W > 1: one exchange piece per map, assigned when published
        job->batch = lz4 && W > 1 ? -1 : node->shuffle(shuffle_id).next_batch++;
      }
      std::lock_guard<std::mutex> plk(node->pipe_mu);
      node->make_pipe();
      ms = node->pipe[node->pipe_next++ & 1];
      hip_check(hipEventRecord(node->pipe_ev[0], s), "fork");
      hip_check(hipStreamWaitEvent(ms, node->pipe_ev[0], 0), "fork");
      if (lz4) {
        uint8_t* plain = job->ws.ptr + plain_off;
        int64_t* d_cix = reinterpret_cast<int64_t*>(job->ws.ptr + cix_off);
        run_group(node, part, G, 1, plain, d_idx, nullptr, nullptr, nullptr, job->ws.ptr,
                  G.ws.total, ms, true);
        hip_check(sux::launch_lz4_compress(plain, d_idx, (uint32_t)maps, (uint32_t)R,
                                           (uint32_t)cblock, job->slab->buf.ptr, d_cix, nullptr,
                                           reinterpret_cast<uint64_t*>(job->ws.ptr + cbytes_off),
                                           job->ws.ptr + lws_off, lw,
                                           resolve_tuning(node->tuning, false).lz4_queue, ms),
                  "compress launch");
        hip_check(hipMemcpyAsync(job->hidx.first, d_cix, ix_bytes, hipMemcpyDeviceToHost, ms),
                  "D2H compressed index");
      } else {
        run_group(node, part, G, W, job->slab->buf.ptr, d_idx, nullptr, nullptr, nullptr,
                  job->ws.ptr, G.ws.total, ms, true);
        if (W != 1)
          hip_check(hipMemcpyAsync(job->hidx.first, d_idx, ix_bytes, hipMemcpyDeviceToHost, ms),
                    "D2H index");
      }
      job->done = std::make_shared<Event>();
      hip_check(hipEventRecord(job->done->e, ms), "hipEventRecord");
      hip_check(hipStreamWaitEvent(s, job->done->e, 0), "join");
    } catch (...) {
      unclaim();
      (void)hipStreamSynchronize(ms);  // nothing on the stream may still use the buffers
      node->pool->put(job->ws);
      node->hpool.put(job->hidx);
      throw;
    }
    std::lock_guard<std::mutex> lk(node->mu);
    auto it = node->shuffles.find(shuffle_id);
    require(it != node->shuffles.end(), SUX_ENOENT, "shuffle unregistered during the write");
    it->second->jobs.push_back(std::move(job));
    it->second->submitting--;
    node->cv.notify_all();
  });
}

int sux_wait_map_outputs(sux_node* node, int32_t shuffle_id) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    node->bind();
    std::unique_lock<std::mutex> lk(node->mu);
    drain(node, node->shuffle(shuffle_id), lk);
  });
}

int sux_write_map_output(sux_node* node, int32_t shuffle_id, int32_t map_index,
                         const sux_partitioner* part, const void* d_records, uint64_t n,
                         void* stream) {
  int rc = SUX_OK;
  if (n == 0) {  // UcxShuffleBlockResolver.scala:42-45; still validates the arguments
    return guard([&] {
      require(node && part, SUX_EINVAL, "NULL node/partitioner");
      std::lock_guard<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      require(map_index >= 0 && map_index < sh.num_maps, SUX_EINVAL,
              "map index " + std::to_string(map_index) + " out of [0, " +
                  std::to_string(sh.num_maps) + ")");
    });
  }
  rc = sux_write_map_outputs(node, shuffle_id, map_index, part, d_records, n, n, stream);
  if (rc != SUX_OK) return rc;
  // CommonUcxShuffleBlockResolver.scala:101-103: block until the map output is published
  return guard([&] {
    std::unique_lock<std::mutex> lk(node->mu);
    Shuffle& sh = node->shuffle(shuffle_id);
    while (sh.maps[map_index].pending) {
      if (!sh.jobs.empty()) progress(node, sh, lk, true);
      else node->cv.wait(lk);
    }
  });
}

int sux_write_map_output_host(sux_node* node, int32_t shuffle_id, int32_t map_index,
                              const sux_partitioner* part, const void* host_records, uint64_t n,
                              void* stream) {
  int rs = 0;
  int rc = guard([&] {
    require(node && part && (host_records || n == 0), SUX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(node->mu);
    rs = node->shuffle(shuffle_id).rec_size;
  });
  if (rc != SUX_OK || n == 0)
    return rc != SUX_OK ? rc : sux_write_map_output(node, shuffle_id, map_index, part, nullptr, 0, stream);
  PoolBuf stage;
  rc = guard([&] {
    node->bind();
    stage = pool_get_or_spill(node, n * (uint64_t)rs);
    hip_check(hipMemcpyAsync(stage.ptr, host_records, n * (uint64_t)rs, hipMemcpyHostToDevice,
                             node->stream(stream)),
              "H2D records");
  });
  if (rc == SUX_OK) rc = sux_write_map_output(node, shuffle_id, map_index, part, stage.ptr, n, stream);
  // the write waited for its map (or failed before launching): the staging buffer is free
  (void)hipStreamSynchronize(node->stream(stream));
  node->pool->put(stage);
  return rc;
}

int sux_commit_map_output(sux_node* node, int32_t shuffle_id, int32_t map_index,
                          const void* d_data, uint64_t bytes, const int64_t* lengths,
                          void* stream) {
  return guard([&] {
    require(node && lengths, SUX_EINVAL, "NULL argument");
    node->bind();
    hipStream_t s = node->stream(stream);
    std::vector<int64_t> index;
    {
      std::unique_lock<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      require(map_index >= 0 && map_index < sh.num_maps, SUX_EINVAL, "map index out of range");
      index.resize((size_t)sh.R + 1);
      int64_t acc = 0;
      for (int r = 0; r < sh.R; ++r) {
        require(lengths[r] >= 0, SUX_EINVAL, "negative partition length");
        index[r] = acc;
        acc += lengths[r];
      }
      index[sh.R] = acc;
      require((uint64_t)acc == bytes, SUX_EINVAL,
              "sum(lengths) = " + std::to_string(acc) + " != data bytes " + std::to_string(bytes));
      progress(node, sh, lk, false);
      if (bytes == 0 || sh.maps[map_index].present || sh.maps[map_index].pending) return;
      require(d_data, SUX_EINVAL, "data pointer is NULL");
      sh.maps[map_index].pending = true;
      sh.submitting++;
    }
    std::shared_ptr<Slab> slab;
    try {
      slab = std::make_shared<Slab>(node->pool.get(), pool_get_or_spill(node, bytes));
      hip_check(hipMemcpyAsync(slab->buf.ptr, d_data, bytes, hipMemcpyDefault, s), "adopt data");
      hip_check(hipStreamSynchronize(s), "sync commit");
    } catch (...) {
      std::lock_guard<std::mutex> lk(node->mu);
      auto it = node->shuffles.find(shuffle_id);
      if (it != node->shuffles.end()) {
        it->second->maps[map_index].pending = false;
        it->second->submitting--;
      }
      node->cv.notify_all();
      throw;
    }
    std::lock_guard<std::mutex> lk(node->mu);
    Shuffle& sh = node->shuffle(shuffle_id);
    sh.submitting--;
    node->cv.notify_all();
    MapSlot& slot = sh.maps[map_index];
    slot.pending = false;
    slot.present = true;
    slot.sent = false;
    slot.owner = node->conf.rank;
    slot.batch = sh.next_batch++;  // a committed data file is its own exchange piece
    slot.slab = slab;
    slot.off = 0;
    slot.bytes = bytes;
    slot.index = std::move(index);
    slot.d_index = nullptr;
    slot.rslab.reset();
    const int NW = node->conf.world_size;
    slot.seg.resize((size_t)NW);
    for (int h = 0; h < NW; ++h) slot.seg[h] = (uint64_t)slot.index[owner_lo(h, sh.R, NW)];
    publish_slot(node, sh, map_index, 0);
  });
}

int sux_adopt_map_outputs(sux_node* node, int32_t shuffle_id, int32_t first,
                          const void* d_out, uint64_t rpm, uint64_t n, const int64_t* d_index,
                          void* stream) {
  return guard([&] {
    require(node && d_index && (d_out || n == 0), SUX_EINVAL, "NULL argument");
    require(rpm > 0, SUX_EINVAL, "records_per_map must be > 0");
    if (n == 0) return;
    node->bind();
    hipStream_t s = node->stream(stream);
    const uint64_t maps = (n + rpm - 1) / rpm;
    auto job = std::make_unique<WriteJob>();
    int R = 0, rs = 0;
    {
      std::unique_lock<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      require(first >= 0 && (uint64_t)first + maps <= (uint64_t)sh.num_maps, SUX_EINVAL,
              "maps [" + std::to_string(first) + ", " + std::to_string((uint64_t)first + maps) +
                  ") out of [0, " + std::to_string(sh.num_maps) + ")");
      progress(node, sh, lk, false);
      R = sh.R;
      rs = sh.rec_size;
      job->claimed.assign((size_t)maps, 0);
      bool any = false;
      for (uint64_t k = 0; k < maps; ++k) {
        MapSlot& sl = sh.maps[first + k];
        if (sl.present || sl.pending) continue;  // first commit wins
        sl.pending = true;
        job->claimed[k] = 1;
        any = true;
      }
      if (!any) return;
      sh.submitting++;
      // map-major outputs: one exchange piece per map at world > 1, the whole batch at world 1
      job->batch = node->conf.world_size == 1 ? sh.next_batch++ : -1;
    }
    job->first = first;
    job->maps = (uint32_t)maps;
    job->rpm = rpm;
    job->n = n;
    job->world = 1;
    PoolBuf borrowed;
    borrowed.ptr = static_cast<uint8_t*>(const_cast<void*>(d_out));
    borrowed.cap = 0;
    job->slab = std::make_shared<Slab>(nullptr, borrowed);  // not the node's: nothing to free
    try {
      if (node->conf.world_size == 1) {
        // the index tables stay where the caller keeps them (like the data): no read-back of
        // maps x (R + 1) entries — 82 MB a step at C5's R = 10 000 — blocks resolve from them on
        // the device
        job->dindex = d_index;
        job->rs = (uint32_t)rs;
      } else {
        job->hidx = node->hpool.get(8 * maps * (uint64_t)(R + 1));
        hip_check(hipMemcpyAsync(job->hidx.first, d_index, 8 * maps * (uint64_t)(R + 1),
                                 hipMemcpyDeviceToHost, s),
                  "D2H index");
      }
      job->done = std::make_shared<Event>();
      hip_check(hipEventRecord(job->done->e, s), "hipEventRecord");
    } catch (...) {
      (void)hipStreamSynchronize(s);
      node->hpool.put(job->hidx);
      std::lock_guard<std::mutex> lk(node->mu);
      auto it = node->shuffles.find(shuffle_id);
      if (it != node->shuffles.end()) {
        for (uint64_t k = 0; k < maps; ++k)
          if (job->claimed[k]) it->second->maps[first + k].pending = false;
        it->second->submitting--;
      }
      node->cv.notify_all();
      throw;
    }
    std::lock_guard<std::mutex> lk(node->mu);
    auto it = node->shuffles.find(shuffle_id);
    require(it != node->shuffles.end(), SUX_ENOENT, "shuffle unregistered during the commit");
    it->second->jobs.push_back(std::move(job));
    it->second->submitting--;
    node->cv.notify_all();
  });
}

int sux_map_output_index(sux_node* node, int32_t shuffle_id, int32_t map_index, uint8_t* out,
                         uint64_t out_len) {
  return guard([&] {
    require(node && out, SUX_EINVAL, "NULL argument");
    std::unique_lock<std::mutex> lk(node->mu);
    Shuffle& sh = node->shuffle(shuffle_id);
    require(map_index >= 0 && map_index < sh.num_maps, SUX_EINVAL, "map index out of range");
    progress(node, sh, lk, false);
    MapSlot& slot = sh.maps[map_index];
    require(slot.present, SUX_ENOENT, "map " + std::to_string(map_index) + " has no output");
    require(out_len >= 8 * (uint64_t)(sh.R + 1), SUX_EINVAL, "index buffer too small");
    const std::vector<int64_t>& ix = host_index(slot, sh.R);
    for (int r = 0; r <= sh.R; ++r) store_be64(out + 8 * (size_t)r, (uint64_t)ix[r]);
  });
}

int sux_owned_partitions(sux_node* node, int32_t shuffle_id, int32_t rank, int32_t* start,
                         int32_t* end) {
  return guard([&] {
    require(node && start && end, SUX_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(node->mu);
    Shuffle& sh = node->shuffle(shuffle_id);
    const int W = node->conf.world_size;
    require(rank >= 0 && rank < W, SUX_EINVAL, "rank out of range");
    *start = owner_lo(rank, sh.R, W);
    *end = owner_lo(rank + 1, sh.R, W);
  });
}

// ---- shuffle-level exchange -------------------------------------------------------------------
}  // extern "C"

namespace {
// One committed map as every rank sees it after the directory all-gather: the DriverMetadata
// slot (UcxWorkerWrapper.scala:27-65) plus what the all-to-all needs — the batch (exchange
// piece) it belongs to and, per peer h, the offset of its range for h in the batch's slab.
struct DirEntry {
  int32_t map = -1, owner = -1, batch = -1;
  std::vector<int64_t> index;  // R + 1
  std::vector<uint64_t> seg;   // world
  uint8_t ipc[SUX_IPC_DESC_BYTES] = {};  // the batch slab (IPC transport only)
};

// Host all-gather of `bytes` per rank: the embedding runtime's bootstrap, or RCCL through a
// device bounce buffer.  The caller holds no node lock.
void host_allgather(sux_node* node, uint64_t tag, const void* send, uint64_t bytes, void* recv,
                    hipStream_t s) {
  const int W = node->conf.world_size;
  if (W == 1 && !node->boot && !node->comm) {  // one rank, no transport: nothing to gather
    if (bytes) std::memcpy(recv, send, bytes);
    return;
  }
  if (node->boot) {
    const int rc = node->boot(node->boot_ctx, tag, send, bytes, recv);
    require(rc == 0, SUX_ECOMM, "bootstrap all-gather failed (" + std::to_string(rc) + ")");
    return;
  }
  require(node->comm != nullptr, SUX_ESTATE,
          "world_size > 1 needs an RCCL communicator (comm_id) or a bootstrap "
          "(sux_node_set_bootstrap)");
  const uint64_t pad = (bytes + 255) / 256 * 256;
  PoolBuf tmp = pool_get_or_spill(node, pad * (W + 1));
  try {
    hip_check(hipMemcpyAsync(tmp.ptr, send, bytes, hipMemcpyHostToDevice, s), "H2D all-gather");
    nccl_check(ncclAllGather(tmp.ptr, tmp.ptr + pad, pad, ncclUint8, node->comm, s),
               "ncclAllGather(directory)");
    for (int r = 0; r < W; ++r)
      hip_check(hipMemcpyAsync(static_cast<uint8_t*>(recv) + (uint64_t)r * bytes,
                               tmp.ptr + pad + (uint64_t)r * pad, bytes, hipMemcpyDeviceToHost, s),
                "D2H all-gather");
    hip_check(hipStreamSynchronize(s), "sync all-gather");
  } catch (...) {
    node->pool->put(tmp);
    throw;
  }
  node->pool->put(tmp);
}

// DriverMetadata analog (UcxWorkerWrapper.scala:27-65): every rank contributes one entry per
// map of the window it committed — |i32 map|i32 owner|i32 batch|i32 0|(R+1) x i64 index|
// W x u64 seg|72-byte IPC descriptor| — padded to the largest contribution; the merged table
// replaces the per-map driver slots fetched by fetchDriverMetadataBuffer (:176-196) and the
// phase-1 offset GETs (UcxShuffleClient.java:50-92).
std::vector<DirEntry> gather_directory(sux_node* node, uint64_t tag, int R,
                                       const std::vector<DirEntry>& mine, hipStream_t s) {
  const int W = node->conf.world_size;
  const uint64_t E = 16 + 8 * (uint64_t)(R + 1) + 8 * (uint64_t)W + SUX_IPC_DESC_BYTES;
  int64_t cnt = (int64_t)mine.size();
  std::vector<int64_t> cnts((size_t)W);
  host_allgather(node, tag, &cnt, 8, cnts.data(), s);
  int64_t most = 0;
  for (int64_t c : cnts) {
    require(c >= 0, SUX_ECOMM, "malformed directory count");
    most = std::max(most, c);
  }
  std::vector<DirEntry> all;
  if (most == 0) return all;
  std::vector<uint8_t> send((size_t)(most * E), 0), recv((size_t)(most * E * W));
  for (size_t k = 0; k < mine.size(); ++k) {
    uint8_t* e = send.data() + k * E;
    std::memcpy(e, &mine[k].map, 4);
    std::memcpy(e + 4, &mine[k].owner, 4);
    std::memcpy(e + 8, &mine[k].batch, 4);
    std::memcpy(e + 16, mine[k].index.data(), 8 * (size_t)(R + 1));
    std::memcpy(e + 16 + 8 * (size_t)(R + 1), mine[k].seg.data(), 8 * (size_t)W);
    std::memcpy(e + 16 + 8 * (size_t)(R + 1) + 8 * (size_t)W, mine[k].ipc, SUX_IPC_DESC_BYTES);
  }
  host_allgather(node, tag + 1, send.data(), send.size(), recv.data(), s);
  for (int r = 0; r < W; ++r)
    for (int64_t k = 0; k < cnts[r]; ++k) {
      const uint8_t* e = recv.data() + ((uint64_t)r * most + k) * E;
      DirEntry d;
      std::memcpy(&d.map, e, 4);
      std::memcpy(&d.owner, e + 4, 4);
      std::memcpy(&d.batch, e + 8, 4);
      d.index.resize((size_t)R + 1);
      std::memcpy(d.index.data(), e + 16, 8 * (size_t)(R + 1));
      d.seg.resize((size_t)W);
      std::memcpy(d.seg.data(), e + 16 + 8 * (size_t)(R + 1), 8 * (size_t)W);
      std::memcpy(d.ipc, e + 16 + 8 * (size_t)(R + 1) + 8 * (size_t)W, SUX_IPC_DESC_BYTES);
      all.push_back(std::move(d));
    }
  return all;
}

}  // namespace

// The 72-byte descriptor of device pointer p: the 64-byte IPC handle of the allocation holding
// it (allocators sub-allocate: the handle names the whole allocation) + p's offset in it.  An
// allocation is exported once while it lives: later calls return the cached handle, recognised
// by the allocation's base, size and buffer id (HIP_POINTER_ATTRIBUTE_BUFFER_ID: unique per
// allocation, so a new allocation at a freed one's address is exported afresh).
void export_ipc(sux_node* node, const void* p, uint8_t out[SUX_IPC_DESC_BYTES]) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hip_check(hipMemGetAddressRange(&base, &size, const_cast<void*>(p)), "hipMemGetAddressRange");
  unsigned long long id = 0;
  hip_check(hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, base),
            "hipPointerGetAttribute(BUFFER_ID)");
  const uint64_t off = (uint64_t)(static_cast<const uint8_t*>(p) - static_cast<const uint8_t*>(base));
  std::lock_guard<std::mutex> lk(node->export_mu);
  auto it = node->ipc_exports.find(base);
  if (it == node->ipc_exports.end() || it->second.id != id || it->second.size != size) {
    // a new export: first drop the entries of allocations that were freed since (their base no
    // longer resolves to the same buffer id), so the cache holds live allocations only (ADVICE
    // r04: it used to keep one entry per base for the node's whole life)
    for (auto e = node->ipc_exports.begin(); e != node->ipc_exports.end();) {
      unsigned long long eid = 0;
      const bool live = e->first != base &&
                        hipPointerGetAttribute(&eid, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                               e->first) == hipSuccess &&
                        eid == e->second.id;
      e = live ? std::next(e) : node->ipc_exports.erase(e);
    }
    (void)hipGetLastError();  // a freed base's failed query must not linger as the last error
    hipIpcMemHandle_t h;
    hip_check(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
    sux_node::IpcExport e{id, size, {}};
    std::memcpy(e.handle, &h, 64);
    it = node->ipc_exports.insert_or_assign(base, e).first;
  }
  std::memcpy(out, it->second.handle, 64);
  std::memcpy(out + 64, &off, 8);
}
namespace {

// Copy descriptors -> one gather-copy launch (64 KiB chunks, block i to its own destination).
// `aux` (device tables) and `hostblk` (their pinned staging) stay with the caller until the
// stream has run the launch.
void launch_copies(sux_node* node, const std::vector<sux::CopyDesc>& desc, PoolBuf& aux,
                   std::pair<void*, uint64_t>& hostblk, hipStream_t s) {
  if (desc.empty()) return;
  std::vector<uint32_t> first(desc.size());
  uint64_t chunks = 0;
  const uint64_t kChunk = 64 * 1024;
  for (size_t i = 0; i < desc.size(); ++i) {
    first[i] = (uint32_t)chunks;
    chunks += desc[i].bytes ? (desc[i].bytes + kChunk - 1) / kChunk : 1;
  }
  require(chunks < (1ull << 31), SUX_ERANGE, "copy request too large");
  const uint64_t dbytes = desc.size() * sizeof(sux::CopyDesc), fbytes = first.size() * 4;
  const uint64_t dpad = ((dbytes + 255) / 256) * 256;
  aux = pool_get_or_spill(node, dpad + fbytes);
  hostblk = node->hpool.get(dpad + fbytes);
  uint8_t* h = static_cast<uint8_t*>(hostblk.first);
  std::memcpy(h, desc.data(), dbytes);
  std::memcpy(h + dpad, first.data(), fbytes);
  hip_check(hipMemcpyAsync(aux.ptr, h, dpad + fbytes, hipMemcpyHostToDevice, s), "H2D desc");
  hip_check(sux::launch_gather_copy(reinterpret_cast<const sux::CopyDesc*>(aux.ptr),
                                    (uint32_t)desc.size(), (uint32_t)chunks,
                                    reinterpret_cast<const uint32_t*>(aux.ptr + dpad),
                                    &node->timer, s),
            "gather copy");
}

// The exchange plan of one window (host arithmetic; every rank computes it from the same
// gathered directory, so the counts of the collective agree).  A piece = the maps of one batch of
// one owner; owner g's pieces, in batch order, are its rounds 0, 1, ...; round k is one
// partition-aligned all-to-all of every owner's k-th piece.  In a piece the maps' ranges for
// peer h are consecutive in the batch slab (peer-major [h][map][h's partitions]), so h's share of
// the piece is ONE range [a_h, e_h): sendcounts/sdispls come straight from the index tables,
// like ncclAllToAllv's counts in SURVEY.md §8(e), and the slab is the send buffer as it stands.
struct XPlan {
  int rounds = 0;
  std::vector<uint64_t> sc, sd, rc, rd;  // [round][peer]
  std::vector<int32_t> piece;            // [round][owner]: the piece's first (lowest-map) entry
  std::vector<uint64_t> base;            // [round + 1]: receive-buffer offset of each round
  std::vector<uint64_t> recv_off;        // [entry]: offset of its owned range (UINT64_MAX: none)
};

XPlan plan_exchange(int W, int me, bool loopback, int n, const int32_t* map, const int32_t* owner,
                    const int32_t* batch, const uint64_t* seg, const uint64_t* len) {
  XPlan P;
  // pieces per owner, ordered by batch; entries of a piece ordered by map
  std::vector<std::map<int32_t, std::vector<int32_t>>> pieces((size_t)W);
  for (int i = 0; i < n; ++i) {
    require(owner[i] >= 0 && owner[i] < W, SUX_ESTATE, "directory entry with a bad owner");
    pieces[owner[i]][batch[i]].push_back(i);
  }
  for (auto& pg : pieces)
    for (auto& kv : pg)
      std::sort(kv.second.begin(), kv.second.end(),
                [&](int32_t a, int32_t b) { return map[a] < map[b]; });
  for (auto& pg : pieces) P.rounds = std::max(P.rounds, (int)pg.size());
  const size_t RW = (size_t)P.rounds * W;
  P.sc.assign(RW, 0);
  P.sd.assign(RW, 0);
  P.rc.assign(RW, 0);
  P.rd.assign(RW, 0);
  P.piece.assign(RW, -1);
  P.base.assign((size_t)P.rounds + 1, 0);
  P.recv_off.assign((size_t)n, UINT64_MAX);
  // [a_h, e_h) of a piece for peer h
  auto span = [&](const std::vector<int32_t>& ents, int h, uint64_t& a, uint64_t& e) {
    a = UINT64_MAX;
    e = 0;
    for (int32_t i : ents) {
      a = std::min(a, seg[(size_t)i * W + h]);
      e = std::max(e, seg[(size_t)i * W + h] + len[(size_t)i * W + h]);
    }
    if (e < a) e = a;
  };
  std::vector<std::map<int32_t, std::vector<int32_t>>::const_iterator> it((size_t)W);
  for (int g = 0; g < W; ++g) it[g] = pieces[g].begin();
  uint64_t base = 0;
  for (int k = 0; k < P.rounds; ++k) {
    P.base[k] = base;
    uint64_t racc = 0;
    for (int g = 0; g < W; ++g) {
      const size_t kg = (size_t)k * W + g;
      P.rd[kg] = racc;
      if (it[g] == pieces[g].end()) continue;
      const std::vector<int32_t>& ents = it[g]->second;
      P.piece[kg] = ents.front();
      if (g == me) {  // this rank's send side of the round
        for (int h = 0; h < W; ++h) {
          uint64_t a, e;
          span(ents, h, a, e);
          P.sd[(size_t)k * W + h] = a;
          P.sc[(size_t)k * W + h] = (h == me && !loopback) ? 0 : e - a;
        }
      }
      if (g != me || loopback) {
        uint64_t a, e;
        span(ents, me, a, e);
        P.rc[kg] = e - a;
        for (int32_t i : ents) P.recv_off[i] = base + racc + (seg[(size_t)i * W + me] - a);
        racc += e - a;
      }
    }
    for (int g = 0; g < W; ++g)
      if (it[g] != pieces[g].end()) ++it[g];
    base += racc;
  }
  P.base[P.rounds] = base;
  return P;
}

struct ExchangingFlag {  // clears Shuffle::exchanging on every exit path
  sux_node* node;
  int32_t id;
  ~ExchangingFlag() {
    std::lock_guard<std::mutex> lk(node->mu);
    auto it = node->shuffles.find(id);
    if (it != node->shuffles.end()) it->second->exchanging = false;
  }
};
}  // namespace

extern "C" {

int sux_plan_exchange(int32_t world, int32_t rank, int32_t loopback, int32_t n,
                      const sux_xplan_entry* entries, const uint64_t* seg, const uint64_t* len,
                      int32_t max_rounds, int32_t* rounds, uint64_t* counts, int32_t* piece_entry,
                      uint64_t* round_base, uint64_t* recv_off) {
  return guard([&] {
    require(world >= 1 && rank >= 0 && rank < world && n >= 0 && rounds, SUX_EINVAL, "bad plan shape");
    require(n == 0 || (entries && seg && len), SUX_EINVAL, "NULL argument");
    std::vector<int32_t> m((size_t)n), o((size_t)n), b((size_t)n);
    for (int i = 0; i < n; ++i) {
      m[i] = entries[i].map;
      o[i] = entries[i].owner;
      b[i] = entries[i].batch;
    }
    const XPlan P = plan_exchange(world, rank, loopback != 0, n, m.data(), o.data(), b.data(), seg, len);
    *rounds = P.rounds;
    require(P.rounds <= max_rounds, SUX_ERANGE, "plan has " + std::to_string(P.rounds) + " rounds");
    for (int k = 0; k < P.rounds; ++k)
      for (int h = 0; h < world; ++h) {
        const size_t kh = (size_t)k * world + h;
        if (counts) {
          counts[(size_t)k * 4 * world + h] = P.sc[kh];
          counts[(size_t)k * 4 * world + world + h] = P.sd[kh];
          counts[(size_t)k * 4 * world + 2 * world + h] = P.rc[kh];
          counts[(size_t)k * 4 * world + 3 * world + h] = P.rd[kh];
        }
        if (piece_entry) piece_entry[kh] = P.piece[kh];
      }
    if (round_base)
      for (int k = 0; k <= P.rounds; ++k) round_base[k] = P.base[k];
    if (recv_off)
      for (int i = 0; i < n; ++i) recv_off[i] = P.recv_off[i];
  });
}

// Asynchronous exchange of one window of maps (see the header): directory all-gather, then one
// partition-aligned ncclAllToAllv per round of batches, or the same plan as one gather-copy of
// one-sided pulls from the owners' IPC-mapped slabs (bootstrap transport).
int sux_exchange_maps(sux_node* node, int32_t shuffle_id, int32_t first, int32_t count,
                      void* stream) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    node->bind();
    hipStream_t s = node->stream(stream);
    const int W = node->conf.world_size, me = node->conf.rank;
    bool loopback = false;
    int R = 0;
    uint64_t tag = 0;
    std::vector<DirEntry> mine;
    std::vector<std::shared_ptr<Slab>> mine_slab;
    {
      std::unique_lock<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      require(first >= 0 && count >= 0 && (int64_t)first + count <= sh.num_maps, SUX_EINVAL,
              "window [" + std::to_string(first) + ", +" + std::to_string(count) +
                  ") out of the shuffle's maps");
      require(!sh.exchanging, SUX_ESTATE,
              "shuffle " + std::to_string(shuffle_id) + " is already exchanging");
      loopback = node->tuning.exchange_self > 0;
      drain_range(node, sh, lk, first, first + count);
      if (W == 1 && !loopback) return;  // every block is local: resolve reads it in place
      R = sh.R;
      require(R >= W, SUX_EINVAL, "need at least one partition per rank");
      sh.exchanging = true;
      tag = ((uint64_t)(uint32_t)shuffle_id << 32) | sh.gathers;
      sh.gathers += 3;
      for (int m = first; m < first + count; ++m) {
        MapSlot& sl = sh.maps[m];
        if (!sl.present || sl.owner != me || sl.sent || !sl.slab || sl.spilled()) continue;
        DirEntry d;
        d.map = m;
        d.owner = me;
        d.batch = sl.batch;
        d.index = host_index(sl, sh.R);
        d.seg = sl.seg;
        mine.push_back(std::move(d));
        mine_slab.push_back(sl.slab);
      }
    }
    ExchangingFlag flag{node, shuffle_id};
    const bool ipc = node->comm == nullptr;
    // every batch slab is exported (the IPC transport pulls from it; with either transport any
    // rank may later read a block its owner serves from it)
    for (size_t k = 0; k < mine.size(); ++k) export_ipc(node, mine_slab[k]->buf.ptr, mine[k].ipc);
    // 1. directory of the window (replaces the driver table + the phase-1 offset GETs)
    std::vector<DirEntry> all = gather_directory(node, tag, R, mine, s);
    const int n = (int)all.size();
    std::vector<int32_t> em((size_t)n), eo((size_t)n), eb((size_t)n);
    std::vector<uint64_t> seg((size_t)n * W), len((size_t)n * W);
    std::vector<int32_t> seen((size_t)first + count, -1);
    for (int i = 0; i < n; ++i) {
      const DirEntry& d = all[i];
      require(d.map >= first && d.map < first + count && d.owner >= 0 && d.owner < W,
              SUX_ESTATE, "malformed directory entry");
      require(seen[d.map] < 0, SUX_ESTATE,
              "map " + std::to_string(d.map) + " committed by more than one rank");
      seen[d.map] = d.owner;
      em[i] = d.map;
      eo[i] = d.owner;
      eb[i] = d.batch;
      for (int h = 0; h < W; ++h) {
        seg[(size_t)i * W + h] = d.seg[h];
        len[(size_t)i * W + h] =
            (uint64_t)(d.index[owner_lo(h + 1, R, W)] - d.index[owner_lo(h, R, W)]);
      }
    }
    // 2. the plan: rounds of partition-aligned all-to-alls, receive layout [round][source]
    const XPlan P = plan_exchange(W, me, loopback, n, em.data(), eo.data(), eb.data(), seg.data(),
                                  len.data());
    const uint64_t total = P.base[P.rounds];
    auto recv = std::make_shared<Slab>(node->pool.get(), total ? pool_get_or_spill(node, total)
                                                               : PoolBuf{});
    // this rank's batch slabs by batch id (the send buffers)
    std::map<int32_t, uint8_t*> my_slab;
    for (size_t k = 0; k < mine.size(); ++k) my_slab[mine[k].batch] = mine_slab[k]->buf.ptr;
    PoolBuf aux;
    std::pair<void*, uint64_t> hostblk{nullptr, 0};
    try {
      if (!ipc) {
        // 3a. RCCL: one all-to-all per round (grouped send/recv pieces over xGMI)
        for (int k = 0; k < P.rounds; ++k) {
          const int32_t pe = P.piece[(size_t)k * W + me];
          uint8_t* sendbuf = pe >= 0 ? my_slab.at(all[pe].batch) : nullptr;
          uint8_t* recvbuf = recv->buf.ptr ? recv->buf.ptr + P.base[k] : nullptr;
          const size_t kw = (size_t)k * W;
          all_to_all_pieces(sendbuf, &P.sc[kw], &P.sd[kw], recvbuf, &P.rc[kw], &P.rd[kw], W,
                            node->comm, s);
        }
      } else {
        // 3b. bootstrap: the same plan as one-sided pulls (OnOffsetsFetchCallback.java:80-87's
        //     GETs, one per (round, source) instead of one per block)
        std::vector<sux::CopyDesc> desc;
        for (int k = 0; k < P.rounds; ++k)
          for (int g = 0; g < W; ++g) {
            const size_t kg = (size_t)k * W + g;
            const int32_t pe = P.piece[kg];
            if (pe < 0 || P.rc[kg] == 0) continue;
            const uint8_t* src = nullptr;
            if (g == me) {
              src = my_slab.at(all[pe].batch);
            } else {
              // one mapping per exported allocation per process (the serve path shares it)
              std::string key(reinterpret_cast<const char*>(all[pe].ipc), 64);
              void* base = nullptr;
              {
                std::lock_guard<std::mutex> lk(node->mu);
                auto& ib = node->shuffle(shuffle_id).ipc_bases;
                auto f = ib.find(key);
                if (f != ib.end()) base = f->second;
              }
              if (!base) {
                base = ipc_open_fresh(node, all[pe].ipc);
                std::lock_guard<std::mutex> lk(node->mu);
                void*& slot = node->shuffle(shuffle_id).ipc_bases[key];
                if (slot) ipc_close_ref(node, base, key);  // another thread mapped it meanwhile
                else slot = base;
                base = slot;
              }
              uint64_t off;
              std::memcpy(&off, all[pe].ipc + 64, 8);
              src = static_cast<const uint8_t*>(base) + off;
            }
            desc.push_back({src + seg[(size_t)pe * W + me], recv->buf.ptr + P.base[k] + P.rd[kg],
                            P.rc[kg]});
          }
        launch_copies(node, desc, aux, hostblk, s);
      }
    } catch (...) {
      (void)hipStreamSynchronize(s);
      node->pool->put(aux);
      node->hpool.put(hostblk);
      throw;
    }
    auto ev = std::make_shared<Event>();
    hip_check(hipEventRecord(ev->e, s), "hipEventRecord(exchange)");
    recv->ready = ev;
    // 4a. where every rank serves its owned ranges of the window's maps: its receive buffer
    //     (descriptors all-gathered) at its own plan's offsets, or its own batch slab
    std::vector<uint8_t> rdesc((size_t)W * SUX_IPC_DESC_BYTES, 0);
    {
      std::vector<uint8_t> mine_desc(SUX_IPC_DESC_BYTES, 0);
      if (recv->buf.ptr) export_ipc(node, recv->buf.ptr, mine_desc.data());
      host_allgather(node, tag + 2, mine_desc.data(), SUX_IPC_DESC_BYTES, rdesc.data(), s);
    }
    std::vector<std::vector<uint64_t>> peer_off((size_t)W);
    for (int h = 0; h < W; ++h)
      peer_off[h] = h == me ? P.recv_off
                            : plan_exchange(W, h, loopback, n, em.data(), eo.data(), eb.data(),
                                            seg.data(), len.data()).recv_off;
    // 4. adopt: remote maps (and, looped back, own maps) now live in the receive buffer
    std::lock_guard<std::mutex> lk(node->mu);
    Shuffle& sh = node->shuffle(shuffle_id);
    sh.xfers.push_back(ev);
    if (aux.ptr) sh.xfer_aux.push_back(aux);
    if (hostblk.first) sh.xfer_host.push_back(hostblk);
    // W > 1: the closing all-gather of sux_exchange_wait is due — with IPC pulls the owners'
    // slabs are read until then, and with either transport a peer read of a block another rank
    // received needs that rank's exchange complete
    if (W > 1) sh.ack_due = true;
    auto serve_id = [&](const uint8_t* d) {
      std::string k(reinterpret_cast<const char*>(d), SUX_IPC_DESC_BYTES);
      auto f = sh.serve_idx.find(k);
      if (f != sh.serve_idx.end()) return f->second;
      const int32_t id = (int32_t)sh.serve_desc.size();
      sh.serve_desc.push_back(k);
      sh.serve_idx[k] = id;
      return id;
    };
    for (int i = 0; i < n; ++i) {
      MapSlot& sl = sh.maps[em[i]];
      sl.serve.assign((size_t)W, {-1, 0});
      for (int h = 0; h < W; ++h) {
        if (peer_off[h][i] == UINT64_MAX)  // h's own map, not looped back: its batch slab
          sl.serve[h] = {serve_id(all[i].ipc), seg[(size_t)i * W + h]};
        else
          sl.serve[h] = {serve_id(rdesc.data() + (size_t)h * SUX_IPC_DESC_BYTES), peer_off[h][i]};
      }
      if (eo[i] == me) sl.sent = true;
      if (P.recv_off[i] == UINT64_MAX) continue;
      if (eo[i] != me) {
        sl.present = true;
        sl.owner = eo[i];
        sl.batch = eb[i];
        sl.slab.reset();
        sl.off = 0;
        sl.seg.clear();
        sl.index = all[i].index;
        sl.bytes = (uint64_t)sl.index[R];
      }
      sl.rslab = recv;
      sl.recv_off = P.recv_off[i];
    }
  });
}

int sux_exchange_wait(sux_node* node, int32_t shuffle_id) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    node->bind();
    std::vector<std::shared_ptr<Event>> evs;
    std::vector<PoolBuf> aux;
    std::vector<std::pair<void*, uint64_t>> host;
    bool ack = false;
    uint64_t tag = 0;
    {
      std::lock_guard<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      require(!sh.exchanging, SUX_ESTATE, "shuffle " + std::to_string(shuffle_id) + " is exchanging");
      evs.swap(sh.xfers);
      aux.swap(sh.xfer_aux);
      host.swap(sh.xfer_host);
      ack = sh.ack_due;
      sh.ack_due = false;
      if (ack) tag = ((uint64_t)(uint32_t)shuffle_id << 32) | sh.gathers++;
    }
    hipError_t err = hipSuccess;
    for (auto& e : evs) {
      const hipError_t r = hipEventSynchronize(e->e);
      if (r != hipSuccess && err == hipSuccess) err = r;
    }
    for (PoolBuf& b : aux) node->pool->put(b);
    for (auto& b : host) node->hpool.put(b);
    hip_check(err, "exchange completion");
    if (ack) {  // every rank has finished its pulls before anyone may free what was pulled
      int64_t one = 1;
      std::vector<int64_t> acks((size_t)node->conf.world_size);
      host_allgather(node, tag, &one, 8, acks.data(), nullptr);
    }
  });
}

// The whole shuffle's exchange, synchronous: every committed map not yet exchanged, then the wait.
int sux_exchange(sux_node* node, int32_t shuffle_id, void* stream) {
  int32_t maps = 0;
  int rc = guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    std::lock_guard<std::mutex> lk(node->mu);
    maps = node->shuffle(shuffle_id).num_maps;
  });
  if (rc != SUX_OK) return rc;
  rc = sux_exchange_maps(node, shuffle_id, 0, maps, stream);
  if (rc != SUX_OK) return rc;
  return sux_exchange_wait(node, shuffle_id);
}

// ---- fetch -----------------------------------------------------------------------------------
}  // extern "C"

namespace {
// Where one block's bytes are: device memory (addr; `ready` = the exchange that fills it, if
// any) or, for a spilled map, a byte range of Spark's data file.
struct BlockLoc {
  uint64_t addr = 0;
  int64_t size = 0;
  std::shared_ptr<Slab> hold;  // keeps the device bytes allocated while a copy may read them
  const Slab* rslab = nullptr;
  const std::string* file = nullptr;
  uint64_t file_off = 0;
};

// Resolve one block; throws SUX_ENOENT for a block not readable here.  At world > 1 a rank
// reads its owned partitions of every map (after the exchange) and any partitions of its own
// maps (within one peer's range: an own peer-major slab holds each peer's share separately).
// ae: the block's two index entries when the caller already gathered them (adopted maps, whose
// index tables stay on the device); hold = false: no reference on the buffer (a zero-copy
// resolve that returns bare addresses).
BlockLoc resolve(sux_node* node, Shuffle& sh, const sux_block_id& b, const int64_t* ae = nullptr,
                 bool hold = true) {
  const int R = sh.R;
  auto name = [&] {
    return "shuffle_" + std::to_string(sh.id) + "_" + std::to_string(b.map_index) + "_" +
           std::to_string(b.start_reduce) +
           (b.end_reduce != b.start_reduce + 1 ? "_" + std::to_string(b.end_reduce) : "");
  };
  // (messages are built only on failure: this runs once per block of every fetch)
  if (!(b.map_index >= 0 && b.map_index < sh.num_maps && b.start_reduce >= 0 &&
        b.end_reduce > b.start_reduce && b.end_reduce <= R))
    raise(SUX_EINVAL, "malformed block " + name());
  MapSlot& sl = sh.maps[b.map_index];
  if (!sl.present) raise(SUX_ENOENT, "Unknown block " + name() + ": map output not committed");
  BlockLoc L;
  const int64_t a = ae ? ae[0] : host_index(sl, R)[b.start_reduce];
  const int64_t e = ae ? ae[1] : host_index(sl, R)[b.end_reduce];
  L.size = e - a;
  const int W = node->conf.world_size, me = node->conf.rank;
  const int lo = owner_lo(me, R, W), hi = owner_lo(me + 1, R, W);
  const bool owned = b.start_reduce >= lo && b.end_reduce <= hi;
  if (sl.rslab && owned) {  // received (or looped back) by an exchange
    L.addr = (uint64_t)(uintptr_t)(sl.rslab->buf.ptr + sl.recv_off + (a - host_index(sl, R)[lo]));
    L.rslab = sl.rslab.get();
    if (hold) L.hold = sl.rslab;
    return L;
  }
  if (sl.owner == me) {
    if (sl.spilled()) {
      L.file = &sl.spill_data;
      L.file_off = (uint64_t)a;
      return L;
    }
    if (hold) L.hold = sl.slab;
    if (W == 1 || sl.seg.empty()) {
      L.addr = (uint64_t)(uintptr_t)(sl.data() + a);
      return L;
    }
    // peer h's range of the map: one contiguous piece of its batch slab
    int h = 0;
    while (owner_lo(h + 1, R, W) <= b.start_reduce) ++h;
    if (b.end_reduce > owner_lo(h + 1, R, W))
      raise(SUX_EINVAL, "block " + name() + " spans the partition ranges of two ranks; split it");
    L.addr = (uint64_t)(uintptr_t)(sl.slab->buf.ptr + sl.seg[h] +
                                   (uint64_t)(a - host_index(sl, R)[owner_lo(h, R, W)]));
    return L;
  }
  if (sl.serve.empty())
    raise(SUX_ESTATE, "block " + name() + " is remote and its map has not been exchanged");
  // another rank's partitions: read where their owner serves them, through the owner's
  // IPC-mapped HBM (a peer read over xGMI — the one-sided GET of OnOffsetsFetchCallback.java:80-87)
  int h = 0;
  while (owner_lo(h + 1, R, W) <= b.start_reduce) ++h;
  if (b.end_reduce > owner_lo(h + 1, R, W))
    raise(SUX_EINVAL, "block " + name() + " spans the partition ranges of two ranks; split it");
  const auto& sv = sl.serve[h];
  if (sv.first < 0) raise(SUX_ENOENT, "block " + name() + " has no serving rank");
  const std::string& desc = sh.serve_desc[sv.first];
  const std::string key = desc.substr(0, 64);  // the allocation's handle (see the pull path)
  void* base = nullptr;
  auto f = sh.ipc_bases.find(key);
  if (f != sh.ipc_bases.end()) {
    base = f->second;
  } else {
    base = ipc_open_fresh(node, reinterpret_cast<const uint8_t*>(desc.data()));
    sh.ipc_bases[key] = base;
  }
  uint64_t doff;
  std::memcpy(&doff, desc.data() + 64, 8);
  L.addr = (uint64_t)(uintptr_t)(static_cast<uint8_t*>(base) + doff + sv.second +
                                 (uint64_t)(a - host_index(sl, R)[owner_lo(h, R, W)]));
  return L;
}

// The (start, end) index entries of every block whose map keeps its index table on the device
// (adopted outputs), gathered in one device pass: ae[2i], ae[2i+1]; has[i] = 1 for those blocks.
// Called with the node lock held (no pool spill from here: the device buffer is a plain get).
// A dense request (a whole stage's reducers: about as many entries per map as the map's table
// has) reads the referenced maps' whole tables back — fewer bytes than two pointers and two
// entries per block — in one copy per run of maps whose tables are adjacent in device memory (one
// adopt call's tables are), and keeps them as the maps' host copies, so later resolves of those
// maps are host arithmetic.  Returns true when every referenced map has its host copy afterwards.
bool dense_index_readback(sux_node* node, Shuffle& sh, const sux_block_id* blocks, int32_t n) {
  std::vector<uint8_t> seen((size_t)sh.num_maps, 0);
  uint64_t entries = 0;
  for (int i = 0; i < n; ++i) {
    const sux_block_id& b = blocks[i];
    if (b.map_index < 0 || b.map_index >= sh.num_maps) continue;
    const MapSlot& sl = sh.maps[b.map_index];
    if (!sl.present || !sl.index.empty() || !sl.d_index) continue;
    seen[(size_t)b.map_index] = 1;
    entries += 2;
  }
  if (!entries) return true;
  std::vector<int32_t> mm;  // the distinct maps, ascending
  for (int32_t m = 0; m < sh.num_maps; ++m)
    if (seen[(size_t)m]) mm.push_back(m);
  const uint64_t row = (uint64_t)sh.R + 1;
  if (entries < mm.size() * row) return false;
  node->bind();
  hipStream_t s = node->stream(nullptr);
  HostLease hp(node->hpool, 8 * row * mm.size());
  int64_t* h = static_cast<int64_t*>(hp.b.first);
  for (size_t j = 0; j < mm.size();) {  // one copy per run of adjacent tables
    size_t k = j + 1;
    while (k < mm.size() && mm[k] == mm[k - 1] + 1 &&
           sh.maps[mm[k]].d_index == sh.maps[mm[k - 1]].d_index + row)
      ++k;
    hip_check(hipMemcpyAsync(h + j * row, sh.maps[mm[j]].d_index, 8 * row * (k - j),
                             hipMemcpyDeviceToHost, s),
              "index tables read-back");
    j = k;
  }
  hip_check(hipStreamSynchronize(s), "index tables read-back");
  for (size_t j = 0; j < mm.size(); ++j) sh.maps[mm[j]].index.assign(h + j * row, h + (j + 1) * row);
  return true;
}

void gather_device_entries(sux_node* node, Shuffle& sh, const sux_block_id* blocks, int32_t n,
                           std::vector<int64_t>& ae, std::vector<uint8_t>& has) {
  has.assign((size_t)n, 0);
  if (dense_index_readback(node, sh, blocks, n)) return;  // every block's map has its host copy
  std::vector<const int64_t*> ptrs;
  std::vector<int32_t> at;
  for (int i = 0; i < n; ++i) {
    const sux_block_id& b = blocks[i];
    if (b.map_index < 0 || b.map_index >= sh.num_maps || b.start_reduce < 0 ||
        b.end_reduce <= b.start_reduce || b.end_reduce > sh.R)
      continue;  // resolve() reports it
    const MapSlot& sl = sh.maps[b.map_index];
    if (!sl.present || !sl.index.empty() || !sl.d_index) continue;
    ptrs.push_back(sl.d_index + b.start_reduce);
    ptrs.push_back(sl.d_index + b.end_reduce);
    at.push_back(i);
  }
  if (at.empty()) return;
  const uint64_t k = ptrs.size(), pbytes = 8 * k, pad = (pbytes + 255) / 256 * 256;
  node->bind();
  hipStream_t s = node->stream(nullptr);
  PoolBuf dev = node->pool->get(pad + 8 * k);
  HostLease hp(node->hpool, pad + 8 * k);
  uint8_t* h = static_cast<uint8_t*>(hp.b.first);
  try {
    std::memcpy(h, ptrs.data(), pbytes);
    hip_check(hipMemcpyAsync(dev.ptr, h, pbytes, hipMemcpyHostToDevice, s), "H2D entry pointers");
    hip_check(sux::launch_gather_i64(reinterpret_cast<const int64_t* const*>(dev.ptr), (uint32_t)k,
                                     reinterpret_cast<int64_t*>(dev.ptr + pad), s),
              "gather index entries");
    hip_check(hipMemcpyAsync(h + pad, dev.ptr + pad, 8 * k, hipMemcpyDeviceToHost, s),
              "D2H index entries");
    hip_check(hipStreamSynchronize(s), "sync index entries");
  } catch (...) {
    (void)hipStreamSynchronize(s);
    node->pool->put(dev);
    throw;
  }
  node->pool->put(dev);
  ae.resize(2 * (size_t)n);
  const int64_t* r = reinterpret_cast<const int64_t*>(h + pad);
  for (size_t j = 0; j < at.size(); ++j) {
    ae[2 * (size_t)at[j]] = r[2 * j];
    ae[2 * (size_t)at[j] + 1] = r[2 * j + 1];
    has[(size_t)at[j]] = 1;
  }
}
}  // namespace

extern "C" {

int sux_resolve_blocks(sux_node* node, int32_t shuffle_id, const sux_block_id* blocks, int32_t n,
                       uint64_t* addrs, int64_t* sizes) {
  return guard([&] {
    require(node && (blocks || n == 0) && (addrs || n == 0) && (sizes || n == 0) && n >= 0,
            SUX_EINVAL, "NULL argument");
    std::unique_lock<std::mutex> lk(node->mu);
    Shuffle& sh = node->shuffle(shuffle_id);
    drain(node, sh, lk);
    const int R = sh.R;
    // the addresses returned are read with no reference held: a successful resolve pins the
    // shuffle's slabs against spilling until it is unregistered (set under mu, which spill_some
    // takes too, before the call returns; a failed resolve returns no address and pins nothing)
    if (node->conf.world_size == 1 && n > 0 && !dense_index_readback(node, sh, blocks, n)) {
      // a sparse request over maps whose index tables live on the device: the whole resolve
      // runs there (block ids up, addresses and sizes down, no per-block host work); blocks the
      // kernel cannot place (another owner's range, a received or spilled map, a malformed id)
      // come back with size -1 and are resolved on the host below, which reports their errors
      std::vector<sux::ResolveMap> tab((size_t)sh.num_maps, sux::ResolveMap{nullptr, 0});
      for (int32_t m = 0; m < sh.num_maps; ++m) {
        const MapSlot& sl = sh.maps[m];
        if (sl.present && sl.d_index && sl.slab && !sl.rslab && !sl.spilled() &&
            sl.owner == node->conf.rank)
          tab[m] = sux::ResolveMap{sl.d_index, (uint64_t)(uintptr_t)sl.data()};
      }
      node->bind();
      hipStream_t s = node->stream(nullptr);
      auto up = [](uint64_t v) { return (v + 255) / 256 * 256; };
      const uint64_t bb = up(16ull * n), tb = up(sizeof(sux::ResolveMap) * tab.size()),
                     ab = up(8ull * n);
      PoolBuf dev = node->pool->get(bb + tb + 2 * ab);
      try {
        hip_check(hipMemcpyAsync(dev.ptr, blocks, 16ull * n, hipMemcpyHostToDevice, s),
                  "H2D block ids");
        hip_check(hipMemcpyAsync(dev.ptr + bb, tab.data(), sizeof(sux::ResolveMap) * tab.size(),
                                 hipMemcpyHostToDevice, s),
                  "H2D map table");
        hip_check(sux::launch_resolve_blocks(
                      dev.ptr, (uint32_t)n, reinterpret_cast<const sux::ResolveMap*>(dev.ptr + bb),
                      sh.num_maps, R, reinterpret_cast<uint64_t*>(dev.ptr + bb + tb),
                      reinterpret_cast<int64_t*>(dev.ptr + bb + tb + ab), s),
                  "resolve blocks");
        hip_check(hipMemcpyAsync(addrs, dev.ptr + bb + tb, 8ull * n, hipMemcpyDeviceToHost, s),
                  "D2H addresses");
        hip_check(hipMemcpyAsync(sizes, dev.ptr + bb + tb + ab, 8ull * n, hipMemcpyDeviceToHost, s),
                  "D2H sizes");
        hip_check(hipStreamSynchronize(s), "resolve blocks");
      } catch (...) {
        (void)hipStreamSynchronize(s);
        node->pool->put(dev);
        throw;
      }
      node->pool->put(dev);
      for (int i = 0; i < n; ++i) {
        if (sizes[i] >= 0) continue;
        const BlockLoc L = resolve(node, sh, blocks[i], nullptr, false);
        if (L.file)
          raise(SUX_ESTATE, "map " + std::to_string(blocks[i].map_index) +
                                " was spilled to " + *L.file + ": fetch its blocks");
        addrs[i] = L.addr;
        sizes[i] = L.size;
      }
      sh.zero_copy = true;
      return;
    }
    std::vector<int64_t> ae;
    std::vector<uint8_t> has;
    gather_device_entries(node, sh, blocks, n, ae, has);
    // the common case first — this rank's own committed maps at world 1 with host copies of
    // their index tables (the zero-copy local read): address and size are two table reads;
    // anything else (a block of another owner, a received range, a spilled map, a malformed id)
    // takes resolve() below
    int i0 = 0;
    if (node->conf.world_size == 1) {
      for (; i0 < n; ++i0) {
        const sux_block_id& b = blocks[i0];
        if (b.map_index < 0 || b.map_index >= sh.num_maps || b.start_reduce < 0 ||
            b.end_reduce <= b.start_reduce || b.end_reduce > R)
          break;
        const MapSlot& sl = sh.maps[b.map_index];
        if (!sl.present || sl.rslab || !sl.slab || sl.spilled() || sl.owner != node->conf.rank)
          break;
        int64_t a, e;
        if (has[(size_t)i0]) {
          a = ae[2 * (size_t)i0];
          e = ae[2 * (size_t)i0 + 1];
        } else if (!sl.index.empty()) {
          a = sl.index[b.start_reduce];
          e = sl.index[b.end_reduce];
        } else {
          break;
        }
        addrs[i0] = (uint64_t)(uintptr_t)(sl.data() + a);
        sizes[i0] = e - a;
      }
    }
    for (int i = i0; i < n; ++i) {
      const BlockLoc L = resolve(node, sh, blocks[i], has[i] ? &ae[2 * (size_t)i] : nullptr, false);
      if (L.file)
        raise(SUX_ESTATE, "map " + std::to_string(blocks[i].map_index) +
                              " was spilled to " + *L.file + ": fetch its blocks");
      addrs[i] = L.addr;
      sizes[i] = L.size;
    }
    if (n > 0) sh.zero_copy = true;
  });
}

int sux_fetch_blocks(sux_node* node, int32_t shuffle_id, const sux_block_id* blocks, int32_t n,
                     int64_t* sizes, sux_buffer** out, void* stream) {
  return guard([&] {
    require(node && out && (blocks || n == 0) && (sizes || n == 0) && n >= 0, SUX_EINVAL,
            "NULL argument");
    node->bind();
    hipStream_t s = node->stream(stream);
    std::vector<BlockLoc> loc((size_t)n);
    std::vector<std::string> files((size_t)n);  // copies: the slot may be spilled/freed later
    std::vector<std::shared_ptr<Event>> waits;
    uint64_t total = 0;
    auto resolve_all = [&] {
      std::unique_lock<std::mutex> lk(node->mu);
      Shuffle& sh = node->shuffle(shuffle_id);
      drain(node, sh, lk);  // maps written without a wait are published first
      // phase 1 (UcxShuffleClient.submitFetchOffsets :50-92 / OnOffsetsFetchCallback :53-72):
      // sizes from the index tables of the directory
      total = 0;
      waits.clear();
      std::vector<int64_t> ae;
      std::vector<uint8_t> has;
      gather_device_entries(node, sh, blocks, n, ae, has);
      const Slab* last = nullptr;
      for (int i = 0; i < n; ++i) {
        loc[i] = resolve(node, sh, blocks[i], has[i] ? &ae[2 * (size_t)i] : nullptr);
        sizes[i] = loc[i].size;
        total += (uint64_t)loc[i].size;
        files[i] = loc[i].file ? *loc[i].file : std::string();
        // blocks received by an exchange still in flight: the copy waits for it
        if (loc[i].rslab && loc[i].rslab != last && loc[i].rslab->ready) {
          waits.push_back(loc[i].rslab->ready);
          last = loc[i].rslab;
        }
      }
    };
    resolve_all();
    auto buf = std::make_unique<sux_buffer>();
    buf->node = node;
    buf->size = total;
    buf->refs = n > 0 ? n : 1;  // one reference per block slice (OnBlocksFetchCallback :35)
    // OnOffsetsFetchCallback :75-76: one pooled buffer for the whole request.  Taken with the
    // blocks' device buffers released: when the pool is full, the allocation spills map outputs
    // (which then must be free to go), and the blocks are resolved again afterwards — a spilled
    // map's blocks come from its file (same sizes, so the layout of the buffer holds)
    loc.assign((size_t)n, BlockLoc{});
    buf->buf = pool_get_or_spill(node, total ? total : 1);
    resolve_all();
    for (auto& w : waits) hip_check(hipStreamWaitEvent(s, w->e, 0), "wait for the exchange");
    try {
      if (total) {
        // phase 2 (:80-87): block i -> contiguous destination at a running offset; device blocks
        // in one gather-copy launch, spilled blocks read from their files
        std::vector<sux::CopyDesc> desc;
        std::vector<uint32_t> first;
        uint64_t pos = 0, chunks = 0;
        const uint64_t kChunk = 64 * 1024;
        std::vector<std::pair<int, uint64_t>> from_file;
        for (int i = 0; i < n; ++i) {
          const uint64_t sz = (uint64_t)loc[i].size;
          if (loc[i].file) {
            from_file.push_back({i, pos});
          } else if (sz) {
            desc.push_back({reinterpret_cast<const uint8_t*>(loc[i].addr), buf->buf.ptr + pos, sz});
            first.push_back((uint32_t)chunks);
            chunks += (sz + kChunk - 1) / kChunk;
          }
          pos += sz;
        }
        require(chunks < (1ull << 31), SUX_ERANGE, "fetch request too large");
        if (!desc.empty()) {
          const uint64_t dbytes = desc.size() * sizeof(sux::CopyDesc), fbytes = first.size() * 4;
          const uint64_t dpad = ((dbytes + 255) / 256) * 256;
          buf->aux = pool_get_or_spill(node, dpad + fbytes);
          uint8_t* d_desc = buf->aux.ptr;
          uint8_t* d_first = buf->aux.ptr + dpad;
          // both tables through one pinned staging block: one true async upload instead of two
          // pageable bounces (the staging returns to node->hpool after the sync below)
          HostLease hb(node->hpool, dpad + fbytes);
          uint8_t* h = static_cast<uint8_t*>(hb.b.first);
          std::memcpy(h, desc.data(), dbytes);
          std::memcpy(h + dpad, first.data(), fbytes);
          hip_check(hipMemcpyAsync(d_desc, h, dpad + fbytes, hipMemcpyHostToDevice, s), "H2D desc");
          hip_check(sux::launch_gather_copy(reinterpret_cast<const sux::CopyDesc*>(d_desc),
                                            (uint32_t)desc.size(), (uint32_t)chunks,
                                            reinterpret_cast<const uint32_t*>(d_first),
                                            &node->timer, s),
                    "gather copy");
          // completion is delivered to the caller like OnBlocksFetchCallback.onSuccess: the
          // blocks are in place when this call returns
          hip_check(hipStreamSynchronize(s), "sync fetch");
        }
        if (!from_file.empty()) {
          Staging st;
          for (auto& f : from_file)
            read_file_range(files[f.first], loc[f.first].file_off, (uint64_t)loc[f.first].size,
                            buf->buf.ptr + f.second, s, st);
        }
      }
    } catch (...) {
      (void)hipStreamSynchronize(s);
      node->pool->put(buf->buf);
      node->pool->put(buf->aux);
      throw;
    }
    {
      std::lock_guard<std::mutex> lk(node->live_mu);
      node->live_bufs.insert(buf.get());
    }
    *out = buf.release();
  });
}

int sux_buffer_alloc(sux_node* node, uint64_t bytes, sux_buffer** out) {
  return guard([&] {
    require(node && out, SUX_EINVAL, "NULL argument");
    node->bind();
    auto buf = std::make_unique<sux_buffer>();
    buf->node = node;
    buf->size = bytes;
    buf->refs = 1;
    buf->buf = pool_get_or_spill(node, bytes ? bytes : 1);
    {
      std::lock_guard<std::mutex> lk(node->live_mu);
      node->live_bufs.insert(buf.get());
    }
    *out = buf.release();
  });
}

int sux_buffer_info(sux_buffer* b, void** ptr, uint64_t* size, uint64_t* cap) {
  return guard([&] {
    require(b, SUX_EINVAL, "NULL buffer");
    if (ptr) *ptr = b->buf.ptr;
    if (size) *size = b->size;
    if (cap) *cap = b->buf.cap;
  });
}

int sux_buffer_read(sux_buffer* b, uint64_t offset, void* dst, uint64_t len, void* stream) {
  return guard([&] {
    require(b && (dst || len == 0), SUX_EINVAL, "NULL argument");
    require(b->node, SUX_ESTATE, "the buffer's node was destroyed");
    require(offset <= b->size && len <= b->size - offset, SUX_ERANGE,
            "read of [" + std::to_string(offset) + ", +" + std::to_string(len) +
                ") past a buffer of " + std::to_string(b->size) + " bytes");
    if (len == 0) return;
    b->node->bind();
    hipStream_t s = b->node->stream(stream);
    hip_check(hipMemcpyAsync(dst, b->buf.ptr + offset, len, hipMemcpyDeviceToHost, s), "D2H block");
    hip_check(hipStreamSynchronize(s), "sync block read");
  });
}

int sux_buffer_retain(sux_buffer* b, int32_t count) {
  return guard([&] {
    require(b && count > 0, SUX_EINVAL, "bad retain");
    b->refs += count;
  });
}

// NioManagedBuffer.release override (OnBlocksFetchCallback.java:45-53): the last release
// returns the pooled buffer.
int sux_buffer_release(sux_buffer* b) {
  return guard([&] {
    require(b, SUX_EINVAL, "NULL buffer");
    int32_t left = --b->refs;
    require(left >= 0, SUX_ESTATE, "buffer released more often than referenced");
    if (left == 0) {
      if (b->node) {  // else the node is gone and its pool freed the memory
        {
          std::lock_guard<std::mutex> lk(b->node->live_mu);
          b->node->live_bufs.erase(b);
        }
        b->node->pool->put(b->buf);
        b->node->pool->put(b->aux);
      }
      delete b;
    }
  });
}

// The reader's side of spark.shuffle.compress (the GPU-sort path of the JVM reader, which must
// decode the LZ4Block streams it fetched before sorting rows): blocks k of `in`, consecutive from
// in_offset, decoded into a new pooled buffer.  One host wait (the decoded sizes), one at the end
// (the device error word: a corrupted stream is SUX_EIO, Spark's "Stream is corrupted").
int sux_buffer_decompress(sux_node* node, sux_buffer* in, uint64_t in_offset,
                          const int64_t* block_sizes, int32_t num_blocks, int32_t max_block_size,
                          sux_buffer** out, int64_t* out_sizes, void* stream) {
  return guard([&] {
    require(node && in && out && (block_sizes || num_blocks == 0), SUX_EINVAL, "NULL argument");
    require(in->node == node, SUX_EINVAL, "the buffer belongs to another node");
    require(num_blocks >= 0, SUX_EINVAL, "negative block count");
    std::vector<int64_t> ioff((size_t)num_blocks + 1);
    uint64_t total = 0;
    for (int32_t k = 0; k < num_blocks; ++k) {
      require(block_sizes[k] >= 0, SUX_EINVAL, "negative block size");
      ioff[k] = (int64_t)(in_offset + total);
      total += (uint64_t)block_sizes[k];
    }
    ioff[num_blocks] = (int64_t)(in_offset + total);
    require(in_offset <= in->size && total <= in->size - in_offset, SUX_ERANGE,
            "blocks [" + std::to_string(in_offset) + ", +" + std::to_string(total) +
                ") past a buffer of " + std::to_string(in->size) + " bytes");
    check_lz4d_args(in_offset + total, num_blocks, max_block_size);
    node->bind();
    hipStream_t s = node->stream(stream);
    const uint64_t ws_bytes =
        sux::lz4d_workspace_layout(in_offset + total, (uint32_t)num_blocks).total;
    const uint64_t tab = (uint64_t)(num_blocks + 1) * 8;
    const uint64_t tab_up = (tab + 255) / 256 * 256;
    PoolBuf aux = pool_get_or_spill(node, ws_bytes + 2 * tab_up);
    PoolBuf dst{};
    auto give_back = [&] {
      (void)hipStreamSynchronize(s);
      node->pool->put(aux);
      if (dst.ptr) node->pool->put(dst);
    };
    try {
      int64_t* d_ioff = reinterpret_cast<int64_t*>(aux.ptr + ws_bytes);
      int64_t* d_ooff = reinterpret_cast<int64_t*>(aux.ptr + ws_bytes + tab_up);
      std::vector<int64_t> ooff((size_t)num_blocks + 1, 0);
      hip_check(hipMemcpyAsync(d_ioff, ioff.data(), tab, hipMemcpyHostToDevice, s), "H2D offsets");
      auto device_error = [&] {
        hip_check(hipStreamSynchronize(s), "sync decompress");
        const uint32_t w = take_device_err(node);
        if (w & (sux::kErrLz4Stream | sux::kErrLz4Checksum))
          raise(SUX_EIO, "Stream is corrupted: a fetched block is not a valid LZ4Block stream "
                         "(header, lengths, LZ4 sequence or checksum)");
        if (w) raise(SUX_EHIP, "device error word set while decompressing");
      };
      // pass 1: the decoded sizes
      hip_check(sux::launch_lz4_decompress(in->buf.ptr, in_offset + total, d_ioff,
                                           (uint32_t)num_blocks, (uint32_t)max_block_size, nullptr,
                                           0, d_ooff, aux.ptr,
                                           sux::lz4d_workspace_layout(in_offset + total,
                                                                      (uint32_t)num_blocks),
                                           node->d_err, s),
                "decompress sizes");
      hip_check(hipMemcpyAsync(ooff.data(), d_ooff, tab, hipMemcpyDeviceToHost, s), "D2H sizes");
      device_error();
      const uint64_t decoded = (uint64_t)ooff[num_blocks];
      dst = pool_get_or_spill(node, decoded ? decoded : 1);
      if (decoded) {
        hip_check(sux::launch_lz4_decompress(in->buf.ptr, in_offset + total, d_ioff,
                                             (uint32_t)num_blocks, (uint32_t)max_block_size,
                                             dst.ptr, decoded, d_ooff, aux.ptr,
                                             sux::lz4d_workspace_layout(in_offset + total,
                                                                        (uint32_t)num_blocks),
                                             node->d_err, s),
                  "decompress");
        device_error();
      }
      auto buf = std::make_unique<sux_buffer>();
      buf->node = node;
      buf->size = decoded;
      buf->refs = 1;
      buf->buf = dst;
      if (out_sizes)
        for (int32_t k = 0; k < num_blocks; ++k) out_sizes[k] = ooff[k + 1] - ooff[k];
      node->pool->put(aux);
      {
        std::lock_guard<std::mutex> lk(node->live_mu);
        node->live_bufs.insert(buf.get());
      }
      *out = buf.release();
    } catch (...) {
      give_back();
      throw;
    }
  });
}

// ---- reduce-side sort ----------------------------------------------------
namespace {
struct SortPlan {
  uint64_t n;
  uint32_t rs;
  sux::MapGroup g{};
  sux::Workspace ws{};
  uint64_t pairs_bytes, part_off, index_off, span_off, total;
};

// Digit widths a sort may use: kSortMinDigitBits .. kSortMaxDigitBits; the workspace is sized for
// the widest so that the caller's buffer fits whichever width the key length selects.
constexpr int kSortMinDigitBits = 8;
constexpr int kSortMaxDigitBits = 15;
constexpr int kSortDefaultMaxDigitBits = 12;

void sort_plan(uint64_t n, uint32_t rs, SortPlan& P, int digit_bits) {
  check_record_size(rs);
  require(n < (1ull << 32), SUX_ERANGE, "sort: fewer than 2^32 records per call");
  P.n = n;
  P.rs = rs;
  const uint32_t R = 1u << digit_bits;
  const uint64_t rpm = n ? n : 1;
  uint32_t tile = sux::choose_tile_recs(R, 16, rpm, sux::Tuning{});
  // long sorts: longer tiles while >= 256 of them remain (fewer counters for k_tile_scan_tm to
  // scan; profiles/r01_v13/sort_tile_sweep.txt: 32 Mi pairs 6.04 -> 5.73 ms at 65536, while 5 M
  // pairs lose 55 % there, hence the tile-count floor)
  while (tile < 65536 && rpm / (2ull * tile) >= 256) tile *= 2;
  P.g.records_per_map = rpm;
  P.g.num_records = n;
  P.g.num_maps = 1;
  P.g.rec_size = 16;
  P.g.tile_recs = tile;
  P.g.tiles_per_map = (uint32_t)((rpm + tile - 1) / tile);
  P.ws = sux::workspace_layout(R, 16, rpm, n, tile, true);
  auto up = [](uint64_t v) { return (v + 255) / 256 * 256; };
  P.pairs_bytes = up(16 * (n ? n : 1));
  P.part_off = 2 * P.pairs_bytes;
  P.index_off = P.part_off + up(P.ws.total);
  P.span_off = P.index_off + up(8ull * (R + 1));
  P.total = P.span_off + up(sux::kSortSpanBytes);
}

// True when bits [lo, hi) of the big-endian 128-bit pair differ between some records.  `span` is
// the AND of key words 0..2 then their OR (pair bytes 0..11 = the 96 high bits, byte 0 first).
bool span_varies(const uint32_t* span, int lo, int hi) {
  for (int b = std::max(lo, 32); b < std::min(hi, 128); ++b) {
    const int byte = 15 - b / 8;  // memory byte of the pair holding bit b
    const uint32_t diff = span[byte / 4] ^ span[3 + byte / 4];
    if ((diff >> (8 * (byte % 4) + b % 8)) & 1u) return true;
  }
  return false;
}

// The device plan's slot (SortPlanDev): past every digit width's layout, so no pass of any width
// writes over it.
uint64_t sort_plan_offset(uint64_t n, uint32_t record_size) {
  uint64_t most = 0;
  for (int d = kSortMinDigitBits; d <= kSortMaxDigitBits; ++d) {
    SortPlan P;
    sort_plan(n, record_size, P, d);
    most = std::max(most, P.total);
  }
  return most;
}

// The chunked top pass's workspace, after the plan slot: the chunked pairs, the chunks' bucket
// starts (sized for 2^kTopMaxBits buckets), the bucket totals.  0: n takes the one-pass top pass
// (more than kTopMaxChunks chunks).
uint64_t top_chunked_bytes(uint64_t n) {
  const uint64_t nch = (n + sux::kTopChunk - 1) / sux::kTopChunk;
  if (n == 0 || nch > sux::kTopMaxChunks) return 0;
  auto up = [](uint64_t v) { return (v + 255) / 256 * 256; };
  const uint64_t R = 1ull << sux::kTopMaxBits;
  return up(16 * n) + up(nch * (R + 1) * 2) + up(R * 4);
}

int sort_key_bits(int32_t kind, int32_t key_len) {
  switch (kind) {
    case SUX_SORT_BYTES:
      require(key_len >= 1 && key_len <= 12, SUX_EINVAL, "sort: byte keys of 1..12 bytes");
      return 8 * key_len;
    case SUX_SORT_LONG:
      require(key_len == 8, SUX_EINVAL, "sort: a long key is 8 bytes");
      return 64;
    case SUX_SORT_INT:
      require(key_len == 4, SUX_EINVAL, "sort: an int key is 4 bytes");
      return 32;
  }
  raise(SUX_EINVAL, "sort: unknown key kind " + std::to_string(kind));
  return 0;
}
}  // namespace

int sux_sort_workspace_size(uint64_t n, uint32_t record_size, uint64_t* bytes) {
  return guard([&] {
    require(bytes, SUX_EINVAL, "NULL argument");
    *bytes = sort_plan_offset(n, record_size) + sux::kSortPlanBytes + top_chunked_bytes(n);
  });
}

namespace {
void sort_impl(sux_node* node, int32_t key_kind, const void* d_in, uint64_t n,
               uint32_t record_size, int32_t key_offset, int32_t key_len, const int64_t* d_seg,
               int32_t nseg, void* d_out, void* d_ws, uint64_t ws_bytes, void* stream) {
  require(node, SUX_EINVAL, "NULL node");
  int bits = sort_key_bits(key_kind, key_len);
  int sbytes = 0;
  if (d_seg) {
    require(nseg >= 1, SUX_EINVAL, "sort: num_segments must be >= 1");
    // the segment id rides above the key in at most 3 bytes: more segments would alias segment
    // k with k mod 2^24 and interleave their records
    require(nseg <= (1 << 24), SUX_ERANGE,
            "sort: at most 2^24 segments per call, got " + std::to_string(nseg));
    sbytes = nseg <= 1 ? 0 : nseg <= 256 ? 1 : nseg <= 65536 ? 2 : 3;
    require(bits / 8 + sbytes <= 12, SUX_EINVAL,
            "sort: key bytes + segment-id bytes (" + std::to_string(sbytes) + ") exceed 12");
    bits += 8 * sbytes;
  }
  require(key_offset >= 0 && (uint64_t)key_offset + key_len <= record_size, SUX_EINVAL,
          "sort: the key does not fit the record");
  // fewest passes at <= max_digit bits each, then the narrowest digit giving that pass count
  // (80-bit TeraSort keys: 6 passes of 14 bits instead of 7 of 12)
  const int max_digit = std::min(
      std::max(node->tuning.sort_max_digit_bits ? node->tuning.sort_max_digit_bits
                                                : kSortDefaultMaxDigitBits,
               kSortMinDigitBits),
      kSortMaxDigitBits);
  const int passes = (bits + max_digit - 1) / max_digit;
  const int digit = std::max(kSortMinDigitBits, (bits + passes - 1) / passes);
  SortPlan P;
  sort_plan(n, record_size, P, digit);
  if (n == 0) return;
  require(d_in && d_out && d_ws, SUX_EINVAL, "NULL buffer");
  const uint64_t plan_off = sort_plan_offset(n, record_size);
  require(ws_bytes >= plan_off + sux::kSortPlanBytes, SUX_EINVAL,
          "sort workspace too small: need sux_sort_workspace_size = " +
              std::to_string(plan_off + sux::kSortPlanBytes) + " bytes");
  require(((uintptr_t)d_in & 3) == 0 && ((uintptr_t)d_out & 3) == 0 &&
              ((uintptr_t)d_ws & 255) == 0,
          SUX_EINVAL, "records (4 B) and workspace (256 B) must be aligned");
  require(d_in != d_out, SUX_EINVAL, "sort is out of place");
  node->bind();
  hipStream_t s = node->stream(stream);
  uint8_t* ws = static_cast<uint8_t*>(d_ws);
  uint8_t* const a = ws;                  // pair buffers (both plans lay them out alike)
  uint8_t* const b = ws + P.pairs_bytes;
  int64_t* index = reinterpret_cast<int64_t*>(ws + P.index_off);
  // records of <= 16 bytes (with the segment id) travel inside the pairs: no gather at the end
  const bool inline_rec = node->tuning.sort_gather != 1 && record_size + (uint32_t)sbytes <= 16;
  sux::PartDev pd{};
  pd.kind = sux::kPartRadix;
  pd.R = 1 << digit;
  pd.key_offset = 0;
  pd.key_len = 16;
  pd.ascending = 1;
  sux::LayoutDesc lay{1, 16};
  // the digit passes use the turn-free sorted-chunk small-record scatter: the turn-taking one can
  // time out into the device error word, and the sort returns before its kernels run
  sux::Tuning sort_tn = resolve_tuning(node->tuning, false);
  if (node->tuning.small_kernel == 0 || node->tuning.small_kernel == 4) sort_tn.small_kernel = 2;
  const bool all_passes = node->tuning.sort_all_passes == 1;

  // ---- the default: MSD planned on the device, no host wait (graph-capturable).  One stable
  // digit pass over the top tb varying key bits (the span reduction finds them in the key span), then
  // every bucket sorted by the lower varying 8-bit digits — in LDS (k_sort_local, <= 4096 pairs)
  // or, for a skewed key set's larger buckets, through global memory by one workgroup each
  // (k_sort_bucket_global).  Each pair crosses HBM twice after the top pass instead of twice per
  // digit, and nothing is decided on the host.
  int tb = kSortMinDigitBits;  // ~<= 1536 pairs per bucket on average, at most 2^14 buckets
#ifndef SUX_SORT_BUCKET_TARGET
#define SUX_SORT_BUCKET_TARGET 1536
#endif
#ifndef SUX_SORT_BUCKET_MSD_MAX
#define SUX_SORT_BUCKET_MSD_MAX (sux::kSortLocalCap / 2)
#endif
  while (tb < 14 && (n >> tb) > SUX_SORT_BUCKET_TARGET) ++tb;
  // the chunked top digit (sort_msd 0 / 1): up to kTopMaxChunks chunks and 12 bits.  Aiming it
  // at ~768-pair buckets (13 bits at 5 M pairs) measured slower: 0.69 vs 0.58 ms
  const uint64_t top_bytes = top_chunked_bytes(n);
  const bool chunked = node->tuning.sort_msd != 3 && node->tuning.sort_msd != 2 && !all_passes &&
                       tb <= sux::kTopMaxBits && top_bytes &&
                       ws_bytes >= plan_off + sux::kSortPlanBytes + top_bytes;
  if (node->tuning.sort_msd != 2 && !all_passes && (n >> tb) <= SUX_SORT_BUCKET_MSD_MAX) {
    SortPlan P1;
    sort_plan(n, record_size, P1, tb);
    sux::SortPlanDev* plan = reinterpret_cast<sux::SortPlanDev*>(ws + plan_off);
    // the fused sort (sorted buckets gather their own records by index) may rebase its buckets'
    // keys: the pairs' key bits are not read after the LDS sort
    const bool fused = !inline_rec && resolve_tuning(node->tuning, false).gather_kernel == 3 &&
                       sux::sort_gather_fusable(record_size);
    hip_check(sux::launch_sort_pairs(static_cast<const uint8_t*>(d_in), n, record_size, key_kind,
                                     key_offset, key_len, d_seg, nseg, sbytes, a,
                                     ws + P1.span_off, inline_rec, s, bits, tb, plan,
                                     chunked ? (fused ? 2 : 1) : 0),
              "sort pairs + plan");
    int64_t* index1 = reinterpret_cast<int64_t*>(ws + P1.index_off);
    sux::PartDev pd1 = pd;
    pd1.R = 1 << tb;
    pd1.dseed = &plan->top_lo;
    // the top digit: chunked (each chunk sorted in place, buckets read as runs; sort_msd 0 / 1)
    // or one stable partition pass (sort_msd 3, or more pairs than kTopMaxChunks chunks)
    sux::SortRuns runs;
    if (chunked) {
      auto up = [](uint64_t v) { return (v + 255) / 256 * 256; };
      const uint64_t nch = (n + sux::kTopChunk - 1) / sux::kTopChunk;
      uint8_t* top = ws + plan_off + sux::kSortPlanBytes;
      uint16_t* offs = reinterpret_cast<uint16_t*>(top + up(16 * n));
      uint32_t* tot = reinterpret_cast<uint32_t*>(
          top + up(16 * n) + up(nch * ((1ull << sux::kTopMaxBits) + 1) * 2));
      hip_check(sux::launch_top_chunks(a, n, tb, plan, top, offs, tot, index1, s),
                "sort top digit (chunked)");
      runs.pairs = top;
      runs.offs = offs;
      runs.nch = (uint32_t)nch;
    } else {
      P1.g.recs = a;
      P1.g.err = node->d_err;
      hip_check(sux::launch_partition_group(pd1, P1.g, lay, b, index1, nullptr, nullptr,
                                            ws + P1.part_off, P1.ws, nullptr, sort_tn,
                                            &node->timer, s),
                "sort top digit pass");
    }
    const sux::Tuning gt = resolve_tuning(node->tuning, false);
    // the large-bucket launches on the node's side stream, unless `s` is being captured into a
    // graph (the side stream is shared by the node's sorts)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    hip_check(hipStreamIsCapturing(s, &cap), "hipStreamIsCapturing");
    std::unique_lock<std::mutex> side_lk(node->sort_mu, std::defer_lock);
    sux::SortSide side;
    if (cap == hipStreamCaptureStatusNone) {
      side_lk.lock();
      if (!node->sort_side)
        hip_check(hipStreamCreateWithFlags(&node->sort_side, hipStreamNonBlocking), "sort stream");
      for (hipEvent_t& e : node->sort_ev)
        if (!e) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "sort event");
      side.s = node->sort_side;
      side.fork = node->sort_ev[0];
      side.join = node->sort_ev[1];
    }
    if (!inline_rec && gt.gather_kernel == 3 && sux::sort_gather_fusable(record_size)) {
      // the fused sort: sorted buckets gather their records themselves, the rest after them
      hip_check(sux::launch_sort_local_planned(b, a, index1, (uint32_t)pd1.R, plan, s, d_in,
                                               d_out, record_size, runs, side, n >> tb),
                "sort buckets");
      hip_check(sux::launch_gather_rest(d_in, a, b, index1, (uint32_t)pd1.R, n, plan, record_size,
                                        d_out, s),
                "sort gather rest");
      return;
    }
    hip_check(sux::launch_sort_local_planned(b, a, index1, (uint32_t)pd1.R, plan, s, nullptr,
                                             nullptr, 0, runs, side, n >> tb),
              "sort buckets");
    if (inline_rec)
      hip_check(sux::launch_unpair_records_sel(a, b, &plan->final_b, n, record_size, key_kind,
                                               key_offset, key_len, sbytes, d_out, s),
                "sort unpair");
    else
      hip_check(sux::launch_gather_records_sel(d_in, a, b, &plan->final_b, n, record_size, d_out,
                                               s, gt.gather16),
                "sort gather");
    return;
  }

  // ---- LSD digit passes (sort_msd = 2, sort_all_passes = 1, or more than 2^14 x 2048 pairs).
  // Passes whose digit never varies are skipped — which needs the key span on the host (one
  // 24-byte read-back); a stream being captured into a HIP graph cannot be waited on, so there
  // every pass runs (a skipped pass is an identity permutation: the bytes are the same).
  uint8_t* pa = a;
  uint8_t* pb = b;
  hip_check(sux::launch_sort_pairs(static_cast<const uint8_t*>(d_in), n, record_size, key_kind,
                                   key_offset, key_len, d_seg, nseg, sbytes, pa, ws + P.span_off,
                                   inline_rec, s),
            "sort pairs");
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  hip_check(hipStreamIsCapturing(s, &cap), "hipStreamIsCapturing");
  const bool run_all = all_passes || cap != hipStreamCaptureStatusNone;
  uint32_t span[6] = {0, 0, 0, ~0u, ~0u, ~0u};  // AND = 0, OR = ~0: every bit varies
  if (!run_all) {
    // pinned staging (a true async copy, not a pageable bounce); taken only when reading back:
    // under graph capture a cold pool would hipHostMalloc mid-capture
    HostLease hrb(node->hpool, 64);
    uint8_t* hrd = static_cast<uint8_t*>(hrb.b.first);
    hip_check(hipMemcpyAsync(hrd, ws + P.span_off, sizeof span, hipMemcpyDeviceToHost, s),
              "sort key span");
    hip_check(hipStreamSynchronize(s), "sort key span");
    std::memcpy(span, hrd, sizeof span);
  }
  // the key occupies bits [128 - bits, 128) of the big-endian pair; least significant digit first
  for (int sh = 128 - bits; sh < 128; sh += digit) {
    if (!run_all && !span_varies(span, sh, sh + digit)) continue;  // identity pass
    pd.seed = sh;
    P.g.recs = pa;
    P.g.err = node->d_err;
    hip_check(sux::launch_partition_group(pd, P.g, lay, pb, index, nullptr, nullptr,
                                          ws + P.part_off, P.ws, nullptr, sort_tn, &node->timer, s),
              "sort digit pass");
    std::swap(pa, pb);
  }
  if (inline_rec)
    hip_check(sux::launch_unpair_records(pa, n, record_size, key_kind, key_offset, key_len, sbytes,
                                         d_out, s),
              "sort unpair");
  else
    hip_check(sux::launch_gather_records(d_in, pa, n, record_size, d_out, s), "sort gather");
}
}  // namespace

int sux_sort_records(sux_node* node, int32_t key_kind, const void* d_in, uint64_t n,
                     uint32_t record_size, int32_t key_offset, int32_t key_len, void* d_out,
                     void* d_ws, uint64_t ws_bytes, void* stream) {
  return guard([&] {
    sort_impl(node, key_kind, d_in, n, record_size, key_offset, key_len, nullptr, 0, d_out, d_ws,
              ws_bytes, stream);
  });
}

int sux_sort_segments(sux_node* node, int32_t key_kind, const void* d_in, uint64_t n,
                      uint32_t record_size, int32_t key_offset, int32_t key_len,
                      const int64_t* d_segment_offsets, int32_t num_segments, void* d_out,
                      void* d_ws, uint64_t ws_bytes, void* stream) {
  return guard([&] {
    require(d_segment_offsets, SUX_EINVAL, "NULL segment offsets");
    sort_impl(node, key_kind, d_in, n, record_size, key_offset, key_len, d_segment_offsets,
              num_segments, d_out, d_ws, ws_bytes, stream);
  });
}

// ---- CU-partitioned streams -------------------------------------------------------------------
// CU-mask bit of the k-th reserved CU.  Measured (tools/cu_probe: HW_REG_XCC_ID + HW_REG_HW_ID
// of the workgroups of masked streams, profiles/r01_cu_probe_*.txt): the driver maps the mask
// symmetrically, bit b -> XCD b % 8, shader engine (b / 8) % 4, CU slot b / 32, and ignores a
// mask that leaves an XCD without CUs.  A kernel's workgroups are dealt evenly over the XCDs and,
// inside one, over its 4 SEs, so an SE that lost more CUs than the others is the launch's
// straggler (4 of SE0's 8 CUs reserved on every XCD ran the scatter 1.5x slower).  Bits 0..C-1
// take the reserved CUs round-robin over all 32 (XCD, SE) pairs: keep C a multiple of 32.
static uint32_t reserved_cu(uint32_t k) { return k; }

// A stream on num_cus CUs picked round robin over the (XCD, SE) pairs, or on the other CUs.
static hipStream_t create_cu_stream(sux_node* node, int32_t num_cus, int32_t complement) {
  const uint32_t P = (uint32_t)node->device_cus();
  require(num_cus >= 0 && (uint32_t)num_cus <= P, SUX_EINVAL,
          "num_cus must be in [0, " + std::to_string(P) + "]");
  hipStream_t st = nullptr;
  if (num_cus == 0 || (uint32_t)num_cus == P) {
    // nothing to partition: an ordinary stream (all CUs, or all CUs for the complement of 0)
    require(!(num_cus == (int32_t)P && complement), SUX_EINVAL, "empty CU set");
    require(!(num_cus == 0 && !complement), SUX_EINVAL, "empty CU set");
    hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
  } else {
    std::vector<uint32_t> mask((P + 31) / 32, 0u);
    std::vector<uint8_t> pick(P, 0);
    for (uint32_t k = 0; k < (uint32_t)num_cus; ++k) {
      uint32_t i = reserved_cu(k);
      pick[i] = 1;
    }
    for (uint32_t i = 0; i < P; ++i)
      if (pick[i] != (complement ? 1 : 0)) mask[i / 32] |= 1u << (i % 32);
    hip_check(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()),
              "hipExtStreamCreateWithCUMask");
  }
  return st;
}

int sux_node::device_cus() {
  if (!cus) {
    hipDeviceProp_t prop;
    hip_check(hipGetDeviceProperties(&prop, conf.device), "hipGetDeviceProperties");
    cus = prop.multiProcessorCount;
  }
  return cus;
}

void sux_node::make_split(int n) {  // pipe_mu held
  if (pipe_split_cus != n) {
    for (hipStream_t& p : pipe_split) {
      if (p) {
        hip_check(hipStreamSynchronize(p), "split stream drain");
        (void)hipStreamDestroy(p);
        p = nullptr;
      }
    }
    pipe_split[0] = create_cu_stream(this, n, 0);
    pipe_split[1] = create_cu_stream(this, n, 1);
    pipe_split_cus = n;
  }
  for (hipEvent_t& e : split_ev)
    if (!e) hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "split event");
}

int sux_stream_create(sux_node* node, int32_t num_cus, int32_t complement, void** out) {
  return guard([&] {
    require(node && out, SUX_EINVAL, "NULL argument");
    node->bind();
    *out = create_cu_stream(node, num_cus, complement);
  });
}

int sux_stream_destroy(sux_node* node, void* stream) {
  return guard([&] {
    require(node && stream, SUX_EINVAL, "NULL argument");
    node->bind();
    hip_check(hipStreamDestroy(static_cast<hipStream_t>(stream)), "hipStreamDestroy");
  });
}

// ---- measurement -----------------------------------------------------------------------------
int sux_set_kernel_timing(sux_node* node, int enable) {
  return guard([&] {
    require(node, SUX_EINVAL, "NULL node");
    std::lock_guard<std::mutex> lk(node->timer.mu);
    node->timer.enabled = enable != 0;
  });
}

int sux_kernel_times(sux_node* node, int64_t* launches, double* total_ms, int32_t nk) {
  return guard([&] {
    require(node && launches && total_ms && nk >= 0, SUX_EINVAL, "NULL argument");
    node->bind();
    std::lock_guard<std::mutex> lk(node->timer.mu);
    for (int k = 0; k < nk; ++k) {
      launches[k] = 0;
      total_ms[k] = 0;
    }
    for (auto& r : node->timer.recs) {
      hip_check(hipEventSynchronize(r.b), "hipEventSynchronize");
      float ms = 0;
      hip_check(hipEventElapsedTime(&ms, r.a, r.b), "hipEventElapsedTime");
      if (r.slot < nk) {
        launches[r.slot]++;
        total_ms[r.slot] += ms;
      }
      node->timer.spare.push_back(r.a);
      node->timer.spare.push_back(r.b);
    }
    node->timer.recs.clear();
  });
}

int sux_kernel_variant(sux_node* node, int32_t slot, char* buf, size_t len) {
  return guard([&] {
    require(node && buf && len > 0, SUX_EINVAL, "NULL argument");
    require(slot >= 0 && slot < sux::kNumSlots, SUX_EINVAL, "slot out of range");
    std::lock_guard<std::mutex> lk(node->timer.mu);
    const char* v = node->timer.variant[slot] ? node->timer.variant[slot] : "";
    std::snprintf(buf, len, "%s", v);
  });
}

// ---- generators --------------------------------------------------------------------------------
int sux_generate(sux_node* node, int32_t kind, uint64_t seed, uint64_t first, uint64_t n,
                 double zipf_s, uint64_t zipf_n, void* d_out, void* stream) {
  return guard([&] {
    require(node && (d_out || n == 0), SUX_EINVAL, "NULL argument");
    require(kind == SUX_GEN_TERASORT || kind == SUX_GEN_SMALL || kind == SUX_GEN_ZIPF, SUX_EINVAL,
            "unknown generator");
    node->bind();
    hipStream_t s = node->stream(stream);
    void* zb = nullptr;
    void* zt = nullptr;
    int nb = 0;
    if (kind == SUX_GEN_ZIPF) {
      require(zipf_n >= 1 && zipf_s > 0, SUX_EINVAL, "zipf needs n >= 1 and s > 0");
      nb = sux::zipf_table_size(zipf_n);
      std::vector<uint64_t> b((size_t)nb + 1), t((size_t)nb + 1);
      sux::zipf_table(zipf_s, zipf_n, b.data(), t.data());
      hip_check(hipMalloc(&zb, b.size() * 8), "hipMalloc(zipf)");
      hip_check(hipMalloc(&zt, t.size() * 8), "hipMalloc(zipf)");
      hip_check(hipMemcpy(zb, b.data(), b.size() * 8, hipMemcpyHostToDevice), "H2D zipf");
      hip_check(hipMemcpy(zt, t.data(), t.size() * 8, hipMemcpyHostToDevice), "H2D zipf");
    }
    hipError_t e = sux::launch_generate(kind, seed, first, n, static_cast<const uint64_t*>(zb),
                                        static_cast<const uint64_t*>(zt), nb,
                                        static_cast<uint8_t*>(d_out), s);
    if (zb) {
      (void)hipStreamSynchronize(s);
      (void)hipFree(zb);
      (void)hipFree(zt);
    }
    hip_check(e, "generate launch");
  });
}

}  // extern "C"
