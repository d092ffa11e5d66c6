// loopback_rccl.cpp — TEST INFRASTRUCTURE, never product code: a stand-in for the RCCL calls the
// library makes (ncclGetUniqueId, ncclCommInitRank / Split / Destroy, ncclGroupStart / End,
// ncclSend / ncclRecv, ncclAllGather), linked into a separate build of the library
// (libsparkucx_amd_loop.so: sux_api.cpp compiled with every nccl* call renamed sux_loop_nccl*,
// csrc/Makefile).  Why: RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), and the
// test boxes have one GPU, so the exchange's RCCL code path — the all-gather of the index tables,
// the split communicator of post/issue, the grouped send/recv pieces of <= 256 MiB and their
// pairing between ranks — could only ever run with one rank.  Here W processes on the one GPU
// each hold a communicator whose messages travel through files under /dev/shm:
//   send #k from rank a to rank b  ->  <dir>/<a>-<b>-<k> (written whole, then renamed into place)
//   recv #k on rank b from rank a  <-  the same file (polled), its byte count checked against the
//                                      receive's, copied into the device buffer, unlinked
// k counts the messages of the ordered pair on that communicator — RCCL's own pairing rule (a
// pair's sends and receives match in the order both sides post them).  A receive whose size
// differs from the matching send fails with ncclInvalidUsage and says which message: real RCCL
// would hang or corrupt.  Semantics kept: a group's sends are all posted before its receives (so
// a group never deadlocks on itself); every operation is ordered after the work already on its
// stream (hipStreamSynchronize) and complete when the call returns (stronger than RCCL, which is
// only stream-ordered — a test of the call pattern and the bytes, not of overlap or speed).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

struct ncclComm {
  int W = 0, rank = 0;
  std::string dir;
  int splits = 0;
  std::vector<uint64_t> sseq, rseq;  // messages sent to / received from each peer
};

namespace {
struct Op {
  bool send;
  void* buf;
  size_t bytes;
  int peer;
  ncclComm* comm;
  hipStream_t s;
};
std::mutex g_mu;  // one op at a time per process (the comm counters, the staging buffer)
thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;
constexpr size_t kStage = size_t(64) << 20;

size_t dsize(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;  // ncclInt64, ncclUint64, ncclFloat64
  }
}
double timeout_s() {
  const char* e = getenv("SUX_LOOPBACK_TIMEOUT");
  return e ? atof(e) : 120.0;
}
std::string msg_path(const ncclComm* c, int from, int to, uint64_t k) {
  return c->dir + "/" + std::to_string(from) + "-" + std::to_string(to) + "-" + std::to_string(k);
}
bool write_all(int fd, const void* p, size_t n) {
  const char* b = static_cast<const char*>(p);
  while (n) {
    const ssize_t w = ::write(fd, b, n);
    if (w <= 0) return false;
    b += w;
    n -= (size_t)w;
  }
  return true;
}
bool read_all(int fd, void* p, size_t n) {
  char* b = static_cast<char*>(p);
  while (n) {
    const ssize_t r = ::read(fd, b, n);
    if (r <= 0) return false;
    b += r;
    n -= (size_t)r;
  }
  return true;
}
void* stage() {
  static void* h = nullptr;
  if (!h && hipHostMalloc(&h, kStage, hipHostMallocDefault) != hipSuccess) h = nullptr;
  return h;
}

ncclResult_t do_send(const Op& o) {
  std::lock_guard<std::mutex> lk(g_mu);
  ncclComm* c = o.comm;
  const uint64_t k = c->sseq[o.peer]++;
  const std::string path = msg_path(c, c->rank, o.peer, k), part = path + ".part";
  if (hipStreamSynchronize(o.s) != hipSuccess) return ncclUnhandledCudaError;
  void* h = stage();
  const int fd = ::open(part.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0600);
  if (fd < 0 || !h) return ncclSystemError;
  const uint64_t n = o.bytes;
  bool ok = write_all(fd, &n, sizeof n);
  for (size_t off = 0; ok && off < n; off += kStage) {
    const size_t m = std::min(kStage, n - off);
    ok = hipMemcpy(h, static_cast<const char*>(o.buf) + off, m, hipMemcpyDefault) == hipSuccess &&
         write_all(fd, h, m);
  }
  ok = (::close(fd) == 0) && ok;
  if (!ok || ::rename(part.c_str(), path.c_str()) != 0) return ncclSystemError;
  if (getenv("SUX_LOOPBACK_LOG"))  // the tests read the message sizes (the <= 256 MiB pieces)
    fprintf(stderr, "loopback rccl: %s rank %d -> %d #%llu %llu bytes\n",
            c->dir.substr(c->dir.rfind('/') + 1).c_str(), c->rank, o.peer, (unsigned long long)k,
            (unsigned long long)n);
  return ncclSuccess;
}

ncclResult_t do_recv(const Op& o) {
  ncclComm* c;
  uint64_t k;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    c = o.comm;
    k = c->rseq[o.peer]++;
  }
  const std::string path = msg_path(c, o.peer, c->rank, k);
  const auto t0 = std::chrono::steady_clock::now();
  int fd;
  while ((fd = ::open(path.c_str(), O_RDONLY)) < 0) {
    const double w = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (w > timeout_s()) {
      fprintf(stderr, "loopback rccl: rank %d waited %.0f s for message #%llu from rank %d (%s)\n",
              c->rank, w, (unsigned long long)k, o.peer, path.c_str());
      return ncclSystemError;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  std::lock_guard<std::mutex> lk(g_mu);
  uint64_t n = 0;
  if (!read_all(fd, &n, sizeof n)) {
    ::close(fd);
    return ncclSystemError;
  }
  if (n != o.bytes) {
    fprintf(stderr, "loopback rccl: rank %d receive #%llu from rank %d expects %zu bytes, the "
            "matching send carried %llu\n", c->rank, (unsigned long long)k, o.peer, o.bytes,
            (unsigned long long)n);
    ::close(fd);
    return ncclInvalidUsage;
  }
  if (hipStreamSynchronize(o.s) != hipSuccess) {
    ::close(fd);
    return ncclUnhandledCudaError;
  }
  void* h = stage();
  bool ok = h != nullptr;
  for (size_t off = 0; ok && off < n; off += kStage) {
    const size_t m = std::min(kStage, (size_t)n - off);
    ok = read_all(fd, h, m) &&
         hipMemcpy(static_cast<char*>(o.buf) + off, h, m, hipMemcpyDefault) == hipSuccess;
  }
  ::close(fd);
  ::unlink(path.c_str());
  return ok ? ncclSuccess : ncclSystemError;
}

ncclResult_t run_ops(std::vector<Op>& ops) {
  ncclResult_t r = ncclSuccess;
  for (const Op& o : ops)
    if (o.send && r == ncclSuccess) r = do_send(o);
  for (const Op& o : ops)
    if (!o.send && r == ncclSuccess) r = do_recv(o);
  ops.clear();
  return r;
}

ncclResult_t post(const Op& o) {
  if (!o.comm || o.peer < 0 || o.peer >= o.comm->W) return ncclInvalidArgument;
  if (g_depth > 0) {
    g_ops.push_back(o);
    return ncclSuccess;
  }
  std::vector<Op> one{o};
  return run_ops(one);
}
}  // namespace

extern "C" {

const char* sux_loop_ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (loopback rccl)";
    case ncclUnhandledCudaError: return "HIP call failed (loopback rccl)";
    case ncclSystemError: return "file or timeout error (loopback rccl)";
    case ncclInvalidArgument: return "invalid argument (loopback rccl)";
    case ncclInvalidUsage: return "send/recv sizes do not pair up (loopback rccl)";
    default: return "error (loopback rccl)";
  }
}

ncclResult_t sux_loop_ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::memset(id, 0, sizeof *id);
  unsigned long long r = 0;
  const int fd = ::open("/dev/urandom", O_RDONLY);
  if (fd >= 0) {
    (void)read_all(fd, &r, sizeof r);
    ::close(fd);
  }
  snprintf(id->internal, sizeof id->internal, "suxloop-%d-%016llx", (int)getpid(), r);
  return ncclSuccess;
}

ncclResult_t sux_loop_ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks || strncmp(id.internal, "suxloop-", 8))
    return ncclInvalidArgument;
  const char* root = getenv("SUX_LOOPBACK_DIR");
  auto* c = new ncclComm;
  c->W = nranks;
  c->rank = rank;
  c->dir = std::string(root ? root : "/dev/shm") + "/" + id.internal;
  c->sseq.assign(nranks, 0);
  c->rseq.assign(nranks, 0);
  if (::mkdir(c->dir.c_str(), 0700) != 0 && errno != EEXIST) {
    delete c;
    return ncclSystemError;
  }
  *comm = c;
  return ncclSuccess;
}

// The library splits only with one color for every rank and key = rank (its exchange
// communicator); anything else is refused rather than guessed.
ncclResult_t sux_loop_ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm,
                                    ncclConfig_t*) {
  if (!comm || !newcomm) return ncclInvalidArgument;
  if (color == NCCL_SPLIT_NOCOLOR) {
    *newcomm = nullptr;
    return ncclSuccess;
  }
  if (color != 0 || key != comm->rank) return ncclInvalidUsage;
  auto* c = new ncclComm;
  c->W = comm->W;
  c->rank = comm->rank;
  c->dir = comm->dir + "-split" + std::to_string(comm->splits++);
  c->sseq.assign(c->W, 0);
  c->rseq.assign(c->W, 0);
  if (::mkdir(c->dir.c_str(), 0700) != 0 && errno != EEXIST) {
    delete c;
    return ncclSystemError;
  }
  *newcomm = c;
  return ncclSuccess;
}

ncclResult_t sux_loop_ncclCommDestroy(ncclComm_t comm) {
  if (comm) {
    (void)::rmdir(comm->dir.c_str());  // the last rank out removes it (fails while non-empty)
    delete comm;
  }
  return ncclSuccess;
}

ncclResult_t sux_loop_ncclGroupStart() {
  ++g_depth;
  return ncclSuccess;
}

ncclResult_t sux_loop_ncclGroupEnd() {
  if (g_depth <= 0) return ncclInvalidUsage;
  if (--g_depth > 0) return ncclSuccess;
  return run_ops(g_ops);
}

ncclResult_t sux_loop_ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer,
                               ncclComm_t comm, hipStream_t s) {
  return post(Op{true, const_cast<void*>(buf), count * dsize(t), peer, comm, s});
}

ncclResult_t sux_loop_ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer,
                               ncclComm_t comm, hipStream_t s) {
  return post(Op{false, buf, count * dsize(t), peer, comm, s});
}

ncclResult_t sux_loop_ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t t,
                                    ncclComm_t comm, hipStream_t s) {
  if (!comm) return ncclInvalidArgument;
  const size_t b = count * dsize(t);
  ncclResult_t r = sux_loop_ncclGroupStart();
  for (int h = 0; h < comm->W && r == ncclSuccess; ++h)
    r = sux_loop_ncclSend(send, count, t, h, comm, s);
  for (int h = 0; h < comm->W && r == ncclSuccess; ++h)
    r = sux_loop_ncclRecv(static_cast<char*>(recv) + (size_t)h * b, count, t, h, comm, s);
  const ncclResult_t e = sux_loop_ncclGroupEnd();
  return r != ncclSuccess ? r : e;
}

}  // extern "C"
