// Host shared-memory communicator (comm_host.cpp): the backend behind KMLS_COMM=host.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace kmls {

constexpr int kHostCommIdBytes = 128;   // same size as an RCCL unique id
std::string host_comm_unique_id();     // "/kmls_comm_<random>" padded to 128 bytes

// One segment per communicator, one slot per rank; every wait is bounded by
// KMLS_COMM_TIMEOUT_S and observes the shared abort flag.
class ShmComm {
 public:
  ShmComm(int rank, int world, const std::string& uid);
  ~ShmComm();
  ShmComm(const ShmComm&) = delete;
  ShmComm& operator=(const ShmComm&) = delete;
  // in place over host memory; kind: 0 u32, 1 i64, 2 u64, 3 f64
  void all_reduce(void* buf, size_t count, size_t elem, int kind, bool max_op);
  // recv = world x bytes (rank order)
  void all_gather(const void* send, void* recv, size_t bytes);
  // send = world blocks of `count` elements; recv = the sum (max) of every rank's block `rank`
  void reduce_scatter(const void* send, void* recv, size_t count, size_t elem, int kind,
                      bool max_op);
  // send = world blocks of `bytes`; recv block r = rank r's block `rank`
  void all_to_all(const void* send, void* recv, size_t bytes);
  // every rank calls it together: this rank's `send` goes to `send_peer`, `recv` gets what
  // `recv_peer` sent (ring shifts, pairwise exchanges)
  void sendrecv(const void* send, size_t send_bytes, int send_peer, void* recv, size_t recv_bytes,
                int recv_peer);
  void barrier();
  void abort();
  bool aborted() const;
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  char* slot(int r) const;
  int rank_, world_;
  double timeout_s_;
  std::string name_;
  void* base_ = nullptr;
  size_t bytes_ = 0, slot_bytes_ = 0;
};

}  // namespace kmls
