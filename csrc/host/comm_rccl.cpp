// Native communicators for the miner's in-loop collectives (SURVEY §7.1 "comm/", §5.3, §5.8).
//
// backend "rccl": Python's torch.distributed (backend "nccl" = RCCL) bootstraps the process
// group; this layer opens a second, native communicator over the SAME librccl that torch loaded
// (looked up with dlopen(RTLD_NOLOAD) — linking /opt/rocm's copy would drag in a second HIP
// runtime), so the C++ mining loop can all-reduce per-level candidate counts on its own HIP
// stream without a Python round trip per level.  The unique id travels through
// torch.distributed (broadcast of 128 bytes).  The communicator is created NON-blocking and its
// initialisation polled against a deadline (KMLS_COMM_TIMEOUT_S, default 300 s): a rank that
// never joins makes the others abort (ncclCommAbort) and raise instead of hanging; host waits of
// the mining loop are bounded the same way (wait_stream).
//
// backend "host" (comm_host.cpp): device buffers staged through pinned memory and combined in a
// POSIX shared-memory segment — the same protocol as several processes on one GPU (the test
// boxes have one MI355X) or without RCCL at all.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "kmls/comm_host.hpp"
#include "kmls/gpu.hpp"

namespace kmls {
namespace gpu {

namespace {

constexpr int kIdBytes = 128;
static_assert(sizeof(ncclUniqueId) == kIdBytes, "RCCL unique id size");

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t,
                                ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static bool init = false;
  if (init) return r;
  const char* names[] = {"librccl.so.1", "librccl.so"};
  for (const char* n : names) {
    r.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);  // torch's copy, already mapped
    if (r.h) break;
  }
  if (!r.h) {
    const char* p = std::getenv("KMLS_RCCL_PATH");
    if (p) r.h = dlopen(p, RTLD_NOW | RTLD_GLOBAL);
  }
  if (!r.h)
    throw std::runtime_error("kmls comm: librccl is not loaded (import torch and initialise "
                             "torch.distributed with the nccl backend first)");
  auto sym = [&](const char* s) {
    void* f = dlsym(r.h, s);
    if (!f) throw std::runtime_error(std::string("kmls comm: missing RCCL symbol ") + s);
    return f;
  };
  r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
  r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
  r.CommInitRankConfig = (decltype(r.CommInitRankConfig))sym("ncclCommInitRankConfig");
  r.CommGetAsyncError = (decltype(r.CommGetAsyncError))sym("ncclCommGetAsyncError");
  r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
  r.CommAbort = (decltype(r.CommAbort))sym("ncclCommAbort");
  r.AllReduce = (decltype(r.AllReduce))sym("ncclAllReduce");
  r.AllGather = (decltype(r.AllGather))sym("ncclAllGather");
  r.ReduceScatter = (decltype(r.ReduceScatter))sym("ncclReduceScatter");
  r.Send = (decltype(r.Send))sym("ncclSend");
  r.Recv = (decltype(r.Recv))sym("ncclRecv");
  r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
  r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
  r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
  init = true;
  return r;
}

void check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + rccl().GetErrorString(e));
}

ncclDataType_t dtype_of(CommDtype t) {
  switch (t) {
    case CommDtype::U32: return ncclUint32;
    case CommDtype::I64: return ncclInt64;
    case CommDtype::U64: return ncclUint64;
    case CommDtype::F64: return ncclFloat64;
  }
  return ncclUint32;
}

double comm_timeout_s() {
  if (const char* e = std::getenv("KMLS_COMM_TIMEOUT_S")) {
    const double v = std::atof(e);
    if (v > 0) return v;
  }
  return 300.0;
}

int kind_of(CommDtype t) {
  switch (t) {
    case CommDtype::U32: return 0;
    case CommDtype::I64: return 1;
    case CommDtype::U64: return 2;
    case CommDtype::F64: return 3;
  }
  return 0;
}

}  // namespace

std::string comm_unique_id() {
  ncclUniqueId id;
  std::memset(id.internal, 0, kIdBytes);
  check(rccl().GetUniqueId(&id), "GetUniqueId");
  return std::string(id.internal, kIdBytes);
}

Comm::Comm(int rank, int world, const std::string& uid, int device, const std::string& backend)
    : rank_(rank), world_(world), timeout_s_(comm_timeout_s()), backend_(backend) {
  if ((int)uid.size() != kIdBytes) throw std::runtime_error("kmls comm: unique id must be 128 bytes");
  if (backend != "rccl" && backend != "host")
    throw std::runtime_error("kmls comm: backend must be 'rccl' or 'host'");
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("kmls comm: hipSetDevice");
  // one rank: collectives degenerate to copies and no communicator is needed — unless
  // KMLS_COMM_FORCE=1 asks for a real one-rank RCCL communicator (tests the RCCL path: loading,
  // non-blocking init, the collectives and teardown, on a one-GPU box)
  const char* fe = std::getenv("KMLS_COMM_FORCE");
  const bool force = fe && fe[0] == '1' && backend == "rccl";
  if (world == 1 && !force) {
    direct_ = true;
    return;
  }
  if (backend == "host") {
    host_ = std::make_unique<ShmComm>(rank, world, uid);
    return;
  }
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), kIdBytes);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;  // poll the initialisation against a deadline instead of hanging in it
  ncclComm_t c = nullptr;
  const ncclResult_t r0 = rccl().CommInitRankConfig(&c, world, id, rank, &cfg);
  if (r0 != ncclSuccess && r0 != ncclInProgress) check(r0, "CommInitRankConfig");
  comm_ = c;
  progress("CommInitRank");
}

Comm::~Comm() {
  if (comm_) (void)rccl().CommDestroy((ncclComm_t)comm_);
  if (staging_) (void)hipHostFree(staging_);
}

// Wait until the communicator has no operation in progress (non-blocking communicators may
// return ncclInProgress from any call); abort and throw past the deadline.
void Comm::progress(const char* what) {
  if (!comm_) return;
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::milliseconds((int64_t)(timeout_s_ * 1000));
  for (;;) {
    ncclResult_t st = ncclSuccess;
    check(rccl().CommGetAsyncError((ncclComm_t)comm_, &st), "CommGetAsyncError");
    if (st == ncclSuccess) return;
    if (st != ncclInProgress) {
      abort();
      throw std::runtime_error(std::string("RCCL ") + what + " failed: " +
                               rccl().GetErrorString(st) + " (communicator aborted)");
    }
    if (std::chrono::steady_clock::now() > deadline) {
      abort();
      throw std::runtime_error(std::string("RCCL ") + what + " timed out after " +
                               std::to_string((int)timeout_s_) +
                               " s (a rank never joined or died); communicator aborted");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

void Comm::abort() {
  if (comm_) (void)rccl().CommAbort((ncclComm_t)comm_);
  comm_ = nullptr;
  if (host_) host_->abort();
}

// Host wait for a stream that has collectives on it: bounded, so a dead peer (whose collective
// never completes) aborts the communicator and raises instead of hanging the job.
void Comm::wait_stream(void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (direct_) {
    if (hipStreamSynchronize(s) != hipSuccess) throw std::runtime_error("kmls comm: stream sync failed");
    return;
  }
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::milliseconds((int64_t)(timeout_s_ * 1000));
  for (int spins = 0;; ++spins) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) throw std::runtime_error(std::string("kmls comm: stream error ") + hipGetErrorString(e));
    if (host_ && host_->aborted()) throw std::runtime_error("kmls comm: aborted by another rank");
    if (std::chrono::steady_clock::now() > deadline) {
      abort();
      throw std::runtime_error("kmls comm: collective did not complete within " +
                               std::to_string((int)timeout_s_) + " s; communicator aborted");
    }
    if (spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void* Comm::stage(size_t bytes) {
  if (bytes > staging_bytes_) {
    if (staging_) (void)hipHostFree(staging_);
    staging_ = nullptr;
    staging_bytes_ = std::max(bytes, staging_bytes_ * 2);
    if (hipHostMalloc(&staging_, staging_bytes_) != hipSuccess)
      throw std::runtime_error("kmls comm: pinned staging allocation failed");
  }
  return staging_;
}

void Comm::all_reduce(const void* send, void* recv, size_t count, CommDtype t, bool max_op,
                      void* stream) {
  const size_t bytes = count * comm_dtype_bytes(t);
  if (direct_) {
    if (send != recv)
      (void)hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    return;
  }
  if (host_) {  // stream-ordered by construction: D2H, sync, combine, H2D, sync
    if (!count) return;
    hipStream_t s = (hipStream_t)stream;
    void* h = stage(bytes);
    if (hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    host_->all_reduce(h, count, comm_dtype_bytes(t), kind_of(t), max_op);
    if (hipMemcpyAsync(recv, h, bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    return;
  }
  const ncclResult_t r = rccl().AllReduce(send, recv, count, dtype_of(t), max_op ? ncclMax : ncclSum,
                                          (ncclComm_t)comm_, (hipStream_t)stream);
  if (r == ncclInProgress) progress("AllReduce");
  else check(r, "AllReduce");
}

void Comm::all_gather(const void* send, void* recv, size_t count, CommDtype t, void* stream) {
  const size_t bytes = count * comm_dtype_bytes(t);
  if (direct_) {
    if (send != recv)
      (void)hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    return;
  }
  if (host_) {
    if (!count) return;
    hipStream_t s = (hipStream_t)stream;
    char* h = (char*)stage(bytes * (size_t)(world_ + 1));
    if (hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    host_->all_gather(h, h + bytes, bytes);
    if (hipMemcpyAsync(recv, h + bytes, bytes * (size_t)world_, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    return;
  }
  const ncclResult_t r = rccl().AllGather(send, recv, count, dtype_of(t), (ncclComm_t)comm_,
                                          (hipStream_t)stream);
  if (r == ncclInProgress) progress("AllGather");
  else check(r, "AllGather");
}

void Comm::reduce_scatter(const void* send, void* recv, size_t recv_count, CommDtype t,
                          bool max_op, void* stream) {
  const size_t eb = comm_dtype_bytes(t), bytes = recv_count * eb;
  hipStream_t s = (hipStream_t)stream;
  if (direct_) {
    if (send != recv) (void)hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s);
    return;
  }
  if (host_) {
    if (!recv_count) return;
    char* h = (char*)stage(bytes * (size_t)(world_ + 1));
    if (hipMemcpyAsync(h, send, bytes * (size_t)world_, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    host_->reduce_scatter(h, h + bytes * (size_t)world_, recv_count, eb, kind_of(t), max_op);
    if (hipMemcpyAsync(recv, h + bytes * (size_t)world_, bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    return;
  }
  const ncclResult_t r = rccl().ReduceScatter(send, recv, recv_count, dtype_of(t),
                                              max_op ? ncclMax : ncclSum, (ncclComm_t)comm_, s);
  if (r == ncclInProgress) progress("ReduceScatter");
  else check(r, "ReduceScatter");
}

void Comm::all_to_all(const void* send, void* recv, size_t count, CommDtype t, void* stream) {
  const size_t eb = comm_dtype_bytes(t), bytes = count * eb;
  hipStream_t s = (hipStream_t)stream;
  if (direct_) {
    if (send != recv) (void)hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s);
    return;
  }
  if (host_) {
    if (!count) return;
    char* h = (char*)stage(2 * bytes * (size_t)world_);
    if (hipMemcpyAsync(h, send, bytes * (size_t)world_, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    host_->all_to_all(h, h + bytes * (size_t)world_, bytes);
    if (hipMemcpyAsync(recv, h + bytes * (size_t)world_, bytes * (size_t)world_,
                       hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    return;
  }
  // grouped point-to-point: one send and one receive per peer, every xGMI link busy at once
  check(rccl().GroupStart(), "GroupStart");
  for (int p = 0; p < world_; ++p) {
    const ncclResult_t a = rccl().Send((const char*)send + (size_t)p * bytes, count, dtype_of(t), p,
                                       (ncclComm_t)comm_, s);
    if (a != ncclSuccess && a != ncclInProgress) check(a, "Send");
    const ncclResult_t b = rccl().Recv((char*)recv + (size_t)p * bytes, count, dtype_of(t), p,
                                       (ncclComm_t)comm_, s);
    if (b != ncclSuccess && b != ncclInProgress) check(b, "Recv");
  }
  const ncclResult_t e = rccl().GroupEnd();
  if (e == ncclInProgress) progress("AllToAll");
  else check(e, "GroupEnd");
}

void Comm::sendrecv(const void* send, int send_peer, void* recv, int recv_peer, size_t count,
                    CommDtype t, void* stream) {
  const size_t bytes = count * comm_dtype_bytes(t);
  hipStream_t s = (hipStream_t)stream;
  if (direct_) {
    if (send != recv) (void)hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s);
    return;
  }
  if (host_) {
    char* h = (char*)stage(2 * bytes);
    if (hipMemcpyAsync(h, send, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    host_->sendrecv(h, bytes, send_peer, h + bytes, bytes, recv_peer);
    if (hipMemcpyAsync(recv, h + bytes, bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      throw std::runtime_error("kmls comm: staging copy failed");
    return;
  }
  check(rccl().GroupStart(), "GroupStart");
  const ncclResult_t a = rccl().Send(send, count, dtype_of(t), send_peer, (ncclComm_t)comm_, s);
  if (a != ncclSuccess && a != ncclInProgress) check(a, "Send");
  const ncclResult_t b = rccl().Recv(recv, count, dtype_of(t), recv_peer, (ncclComm_t)comm_, s);
  if (b != ncclSuccess && b != ncclInProgress) check(b, "Recv");
  const ncclResult_t e = rccl().GroupEnd();
  if (e == ncclInProgress) progress("SendRecv");
  else check(e, "GroupEnd");
}

size_t comm_dtype_bytes(CommDtype t) {
  switch (t) {
    case CommDtype::U32: return 4;
    case CommDtype::I64:
    case CommDtype::U64:
    case CommDtype::F64: return 8;
  }
  return 4;
}

}  // namespace gpu
}  // namespace kmls
