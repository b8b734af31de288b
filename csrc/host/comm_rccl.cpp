// Native RCCL communicator for the miner's in-loop collectives (SURVEY §7.1 "comm/").
//
// Python's torch.distributed (backend "nccl" = RCCL) bootstraps the process group; this layer
// opens a second, native communicator over the SAME librccl that torch loaded (looked up with
// dlopen(RTLD_NOLOAD) — linking /opt/rocm's copy would drag in a second HIP runtime), so the C++
// mining loop can all-reduce per-level candidate counts on its own HIP stream without a Python
// round trip per level.  The unique id travels through torch.distributed (broadcast of 128
// bytes).  Collectives used: all-reduce (supports, pair counts, candidate counts), all-gather.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "kmls/gpu.hpp"

namespace kmls {
namespace gpu {

namespace {

using ncclResult_t = int;
struct ncclComm;
using ncclComm_t = ncclComm*;
constexpr int kIdBytes = 128;
struct ncclUniqueId { char internal[kIdBytes]; };
// rccl.h enums (ncclDataType_t / ncclRedOp_t)
constexpr int kUint32 = 3, kInt64 = 4, kUint64 = 5, kFloat64 = 8;
constexpr int kSum = 0, kMax = 2;

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
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
  r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
  r.CommAbort = (decltype(r.CommAbort))sym("ncclCommAbort");
  r.AllReduce = (decltype(r.AllReduce))sym("ncclAllReduce");
  r.AllGather = (decltype(r.AllGather))sym("ncclAllGather");
  r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
  init = true;
  return r;
}

void check(ncclResult_t e, const char* what) {
  if (e != 0)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + rccl().GetErrorString(e));
}

int dtype_of(CommDtype t) {
  switch (t) {
    case CommDtype::U32: return kUint32;
    case CommDtype::I64: return kInt64;
    case CommDtype::U64: return kUint64;
    case CommDtype::F64: return kFloat64;
  }
  return kUint32;
}

}  // namespace

std::string comm_unique_id() {
  ncclUniqueId id;
  std::memset(id.internal, 0, kIdBytes);
  check(rccl().GetUniqueId(&id), "GetUniqueId");
  return std::string(id.internal, kIdBytes);
}

Comm::Comm(int rank, int world, const std::string& uid, int device) : rank_(rank), world_(world) {
  if ((int)uid.size() != kIdBytes) throw std::runtime_error("kmls comm: unique id must be 128 bytes");
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("kmls comm: hipSetDevice");
  if (world == 1) return;  // collectives degenerate to copies; no communicator needed
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), kIdBytes);
  ncclComm_t c = nullptr;
  check(rccl().CommInitRank(&c, world, id, rank), "CommInitRank");
  comm_ = c;
}

Comm::~Comm() {
  if (comm_) (void)rccl().CommDestroy((ncclComm_t)comm_);
}

void Comm::abort() {
  if (comm_) (void)rccl().CommAbort((ncclComm_t)comm_);
  comm_ = nullptr;
}

void Comm::all_reduce(const void* send, void* recv, size_t count, CommDtype t, bool max_op,
                      void* stream) {
  if (world_ == 1) {
    if (send != recv)
      (void)hipMemcpyAsync(recv, send, count * comm_dtype_bytes(t), hipMemcpyDeviceToDevice,
                           (hipStream_t)stream);
    return;
  }
  check(rccl().AllReduce(send, recv, count, dtype_of(t), max_op ? kMax : kSum, (ncclComm_t)comm_,
                         (hipStream_t)stream), "AllReduce");
}

void Comm::all_gather(const void* send, void* recv, size_t count, CommDtype t, void* stream) {
  if (world_ == 1) {
    if (send != recv)
      (void)hipMemcpyAsync(recv, send, count * comm_dtype_bytes(t), hipMemcpyDeviceToDevice,
                           (hipStream_t)stream);
    return;
  }
  check(rccl().AllGather(send, recv, count, dtype_of(t), (ncclComm_t)comm_, (hipStream_t)stream),
        "AllGather");
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
