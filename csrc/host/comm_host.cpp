// Host-staged communicator backend (KMLS_COMM=host): the miner's in-loop collectives without
// RCCL, for running the transaction-DP protocol as several processes on ONE GPU (the GPU boxes
// here have one MI355X) and for CPU-side multi-process tests.
//
// The ranks of one node share a POSIX shared-memory segment: a header (barrier, attach count,
// abort flag) and one slot per rank.  all_reduce / all_gather move device buffers through
// pinned staging memory (D2H, stream sync), combine the slots on the host, and copy back (H2D).
// Every wait is bounded (KMLS_COMM_TIMEOUT_S, default 300 s); any rank can raise the shared
// abort flag, which makes every other rank's next wait throw instead of hanging: the
// abort-on-rank-failure path of SURVEY §5.3 for this backend.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>

#include "kmls/comm_host.hpp"

namespace kmls {

namespace {

struct alignas(64) ShmHeader {
  std::atomic<uint32_t> ready;     // rank 0 finished initialising the segment
  std::atomic<uint32_t> attached;  // ranks that mapped it
  std::atomic<uint32_t> arrived;   // barrier arrivals in the current phase
  std::atomic<uint32_t> phase;     // barrier generation
  std::atomic<uint32_t> aborted;   // any rank gave up: everyone's next wait throws
  uint32_t world;
  uint64_t slot_bytes;
};
static_assert(sizeof(ShmHeader) <= 4096, "header must fit its page");
constexpr size_t kHeaderBytes = 4096;

double timeout_seconds() {
  if (const char* e = std::getenv("KMLS_COMM_TIMEOUT_S")) {
    const double v = std::atof(e);
    if (v > 0) return v;
  }
  return 300.0;
}

template <typename T>
void reduce_into(T* dst, const T* src, size_t n, bool max_op) {
  if (max_op)
    for (size_t i = 0; i < n; ++i) dst[i] = src[i] > dst[i] ? src[i] : dst[i];
  else
    for (size_t i = 0; i < n; ++i) dst[i] += src[i];
}

}  // namespace

std::string host_comm_unique_id() {
  std::random_device rd;
  char name[64];
  std::snprintf(name, sizeof name, "/kmls_comm_%08x%08x%08x", rd(), rd(), (unsigned)getpid());
  std::string id(kHostCommIdBytes, '\0');
  std::memcpy(&id[0], name, std::strlen(name));
  return id;
}

ShmComm::ShmComm(int rank, int world, const std::string& uid)
    : rank_(rank), world_(world), timeout_s_(timeout_seconds()) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("kmls shm comm: bad rank/world");
  name_ = std::string(uid.c_str());  // NUL-terminated inside the 128-byte id
  if (name_.size() < 2 || name_[0] != '/') throw std::runtime_error("kmls shm comm: bad unique id");
  size_t slot = 8u << 20;
  if (const char* e = std::getenv("KMLS_SHM_SLOT_MB")) slot = (size_t)std::max(1, std::atoi(e)) << 20;
  bytes_ = kHeaderBytes + slot * (size_t)world;
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::milliseconds((int64_t)(timeout_s_ * 1000));
  int fd = -1;
  if (rank == 0) {
    fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("kmls shm comm: shm_open(create) failed for " + name_);
    if (ftruncate(fd, (off_t)bytes_) != 0) {
      close(fd);
      shm_unlink(name_.c_str());
      throw std::runtime_error("kmls shm comm: ftruncate failed");
    }
  } else {
    while ((fd = shm_open(name_.c_str(), O_RDWR, 0600)) < 0) {
      if (std::chrono::steady_clock::now() > deadline)
        throw std::runtime_error("kmls shm comm: timed out waiting for rank 0's segment " + name_);
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    // rank 0 may not have sized it yet
    struct stat st;
    while (fstat(fd, &st) == 0 && (size_t)st.st_size < bytes_) {
      if (std::chrono::steady_clock::now() > deadline) {
        close(fd);
        throw std::runtime_error("kmls shm comm: segment never reached its size");
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    if (rank == 0) shm_unlink(name_.c_str());
    throw std::runtime_error("kmls shm comm: mmap failed");
  }
  auto* h = reinterpret_cast<ShmHeader*>(base_);
  if (rank == 0) {
    new (h) ShmHeader();
    h->world = (uint32_t)world;
    h->slot_bytes = slot;
    h->ready.store(1, std::memory_order_release);
  } else {
    while (h->ready.load(std::memory_order_acquire) != 1) {
      if (std::chrono::steady_clock::now() > deadline)
        throw std::runtime_error("kmls shm comm: rank 0 never initialised the segment");
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if ((int)h->world != world) throw std::runtime_error("kmls shm comm: world size mismatch");
  }
  slot_bytes_ = h->slot_bytes;
  h->attached.fetch_add(1);
  barrier();
  if (rank == 0) shm_unlink(name_.c_str());  // every rank is mapped: the name can go
}

ShmComm::~ShmComm() {
  if (base_) munmap(base_, bytes_);
}

void ShmComm::abort() {
  if (base_) reinterpret_cast<ShmHeader*>(base_)->aborted.store(1);
}

bool ShmComm::aborted() const {
  return base_ && reinterpret_cast<ShmHeader*>(base_)->aborted.load() != 0;
}

void ShmComm::barrier() {
  auto* h = reinterpret_cast<ShmHeader*>(base_);
  const uint32_t ph = h->phase.load(std::memory_order_acquire);
  if (h->arrived.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)world_ - 1) {
    h->arrived.store(0, std::memory_order_relaxed);
    h->phase.store(ph + 1, std::memory_order_release);
    return;
  }
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::milliseconds((int64_t)(timeout_s_ * 1000));
  int spins = 0;
  while (h->phase.load(std::memory_order_acquire) == ph) {
    if (h->aborted.load()) throw std::runtime_error("kmls shm comm: aborted by another rank");
    if (++spins > 256) {
      spins = 0;
      if (std::chrono::steady_clock::now() > deadline) {
        h->aborted.store(1);
        throw std::runtime_error("kmls shm comm: barrier timed out (a rank died or hung); "
                                 "all ranks aborted");
      }
      sched_yield();
    }
  }
}

char* ShmComm::slot(int r) const { return (char*)base_ + kHeaderBytes + (size_t)r * slot_bytes_; }

void ShmComm::all_reduce(void* buf, size_t count, size_t elem, int kind, bool max_op) {
  char* p = (char*)buf;
  const size_t per = slot_bytes_ / elem;
  for (size_t off = 0; off < count; off += per) {
    const size_t n = std::min(per, count - off);
    std::memcpy(slot(rank_), p + off * elem, n * elem);
    barrier();
    // every rank reduces the whole chunk in rank order: identical results on every rank
    std::memcpy(p + off * elem, slot(0), n * elem);
    for (int r = 1; r < world_; ++r) {
      void* d = p + off * elem;
      const void* s = slot(r);
      switch (kind) {
        case 0: reduce_into((uint32_t*)d, (const uint32_t*)s, n, max_op); break;
        case 1: reduce_into((int64_t*)d, (const int64_t*)s, n, max_op); break;
        case 2: reduce_into((uint64_t*)d, (const uint64_t*)s, n, max_op); break;
        case 3: reduce_into((double*)d, (const double*)s, n, max_op); break;
        default: throw std::runtime_error("kmls shm comm: bad dtype");
      }
    }
    barrier();  // slots may be overwritten by the next chunk
  }
}

void ShmComm::all_gather(const void* send, void* recv, size_t bytes) {
  const char* s = (const char*)send;
  char* d = (char*)recv;
  for (size_t off = 0; off < bytes; off += slot_bytes_) {
    const size_t n = std::min(slot_bytes_, bytes - off);
    std::memcpy(slot(rank_), s + off, n);
    barrier();
    for (int r = 0; r < world_; ++r) std::memcpy(d + (size_t)r * bytes + off, slot(r), n);
    barrier();
  }
}


void ShmComm::reduce_scatter(const void* send, void* recv, size_t count, size_t elem, int kind,
                             bool max_op) {
  const char* src = (const char*)send;
  char* dst = (char*)recv;
  const size_t per = slot_bytes_ / elem;
  for (size_t off = 0; off < count; off += per) {
    const size_t n = std::min(per, count - off);
    // every destination block in turn: each rank publishes its chunk of block d, rank d sums
    for (int d = 0; d < world_; ++d) {
      std::memcpy(slot(rank_), src + ((size_t)d * count + off) * elem, n * elem);
      barrier();
      if (d == rank_) {
        void* o = dst + off * elem;
        std::memcpy(o, slot(0), n * elem);
        for (int r = 1; r < world_; ++r) {
          const void* sl = slot(r);
          switch (kind) {
            case 0: reduce_into((uint32_t*)o, (const uint32_t*)sl, n, max_op); break;
            case 1: reduce_into((int64_t*)o, (const int64_t*)sl, n, max_op); break;
            case 2: reduce_into((uint64_t*)o, (const uint64_t*)sl, n, max_op); break;
            case 3: reduce_into((double*)o, (const double*)sl, n, max_op); break;
            default: throw std::runtime_error("kmls shm comm: bad dtype");
          }
        }
      }
      barrier();
    }
  }
}

void ShmComm::all_to_all(const void* send, void* recv, size_t bytes) {
  const char* s = (const char*)send;
  char* d = (char*)recv;
  const size_t per = slot_bytes_ / (size_t)world_;  // a slot holds one chunk of every block
  if (per == 0) throw std::runtime_error("kmls shm comm: slot smaller than world");
  for (size_t off = 0; off < bytes; off += per) {
    const size_t n = std::min(per, bytes - off);
    for (int b = 0; b < world_; ++b) std::memcpy(slot(rank_) + (size_t)b * per, s + (size_t)b * bytes + off, n);
    barrier();
    for (int r = 0; r < world_; ++r) std::memcpy(d + (size_t)r * bytes + off, slot(r) + (size_t)rank_ * per, n);
    barrier();
  }
}

void ShmComm::sendrecv(const void* send, size_t send_bytes, int send_peer, void* recv,
                       size_t recv_bytes, int recv_peer) {
  (void)send_peer;  // the slot of this rank is read by whoever names it as recv_peer
  const char* s = (const char*)send;
  char* d = (char*)recv;
  const size_t total = std::max(send_bytes, recv_bytes);
  // every rank runs the same number of rounds: the longest message of any rank is unknown
  // here, so the rounds follow max(send, recv) of this pair and the callers keep sizes equal
  // within a call (ring shifts of equal-size blocks)
  for (size_t off = 0; off < total; off += slot_bytes_) {
    const size_t n = std::min(slot_bytes_, total - off);
    if (off < send_bytes) std::memcpy(slot(rank_), s + off, std::min(n, send_bytes - off));
    barrier();
    if (off < recv_bytes) std::memcpy(d + off, slot(recv_peer), std::min(n, recv_bytes - off));
    barrier();
  }
}

}  // namespace kmls
