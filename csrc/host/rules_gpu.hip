// Host side of the GPU rule engine (kernels: csrc/kernels/rules.hip; CPU twin: rules_cpu.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/kernels.hpp"
#include "kmls/gpu.hpp"
#include "kmls/trace.hpp"

#define KMLS_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));     \
  } while (0)

namespace kmls {
namespace gpu {

namespace {
struct DevBuf {  // RAII hipMalloc
  void* p = nullptr;
  explicit DevBuf(size_t bytes) { KMLS_HIP(hipMalloc(&p, std::max<size_t>(bytes, 256))); }
  ~DevBuf() { if (p) (void)hipFree(p); }
  template <class T> T* as() const { return (T*)p; }
};
}  // namespace

RuleSet association_rules_gpu(int device, const int64_t* parent, const int32_t* item,
                              const uint32_t* count, const uint8_t* depth, int64_t n, int64_t n_tx,
                              RuleMetric metric, double min_threshold, int max_antecedent,
                              double* kernel_ms) {
  trace::Range rg_("kmls.rules_gpu");
  RuleSet out;
  if (n == 0 || n_tx == 0) return out;
  KMLS_CHECK(n < (1ll << 31) - 1, "GPU rules: trie larger than 2^31 nodes");
  KMLS_HIP(hipSetDevice(device));
  hipStream_t s;
  KMLS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{s};
  int kmax = 0;
  for (int64_t i = 0; i < n; ++i) kmax = std::max<int>(kmax, depth[i]);
  DevBuf d_par(n * 8), d_item(n * 4), d_cnt(n * 4), d_dep(n);
  KMLS_HIP(hipMemcpyAsync(d_par.p, parent, n * 8, hipMemcpyHostToDevice, s));
  KMLS_HIP(hipMemcpyAsync(d_item.p, item, n * 4, hipMemcpyHostToDevice, s));
  KMLS_HIP(hipMemcpyAsync(d_cnt.p, count, n * 4, hipMemcpyHostToDevice, s));
  KMLS_HIP(hipMemcpyAsync(d_dep.p, depth, n, hipMemcpyHostToDevice, s));
  uint64_t cap = 1;
  while (cap < (uint64_t)n * 2) cap <<= 1;
  DevBuf d_keys(cap * 8), d_vals(cap * 4);
  KMLS_HIP(hipMemsetAsync(d_keys.p, 0xFF, cap * 8, s));
  hipEvent_t e0, e1;
  KMLS_HIP(hipEventCreate(&e0));
  KMLS_HIP(hipEventCreate(&e1));
  KMLS_HIP(hipEventRecord(e0, s));
  kern::rules_hash_build(d_par.as<int64_t>(), d_item.as<int32_t>(), n, d_keys.as<unsigned long long>(),
                         d_vals.as<int32_t>(), cap - 1, s);
  hipDeviceProp_t prop;
  KMLS_HIP(hipGetDeviceProperties(&prop, device));
  const int grid = kern::rules_grid(std::max(1, prop.multiProcessorCount));
  const int64_t waves = (int64_t)grid * kern::rules_waves_per_block();
  int smax = 18;  // per-wave global tables up to 2^18 entries; deeper itemsets walk
  if (const char* e = std::getenv("KMLS_RULES_SCRATCH_BITS")) smax = std::atoi(e);
  int sbits = 0;
  if (kmax > 12 && smax > 12) sbits = std::min(kmax, smax);
  DevBuf d_scr(sbits ? (size_t)waves * ((size_t)1 << sbits) * 4 : 0);
  DevBuf d_ctl(64);
  KMLS_HIP(hipMemsetAsync(d_ctl.p, 0, 64, s));
  DevBuf d_nr((n + 1) * 8), d_off((n + 1) * 8);
  KMLS_HIP(hipMemsetAsync(d_nr.as<int64_t>() + n, 0, 8, s));
  kern::RuleArgs a{};
  a.parent = d_par.as<int64_t>();
  a.item = d_item.as<int32_t>();
  a.count = d_cnt.as<uint32_t>();
  a.depth = d_dep.as<uint8_t>();
  a.n = n;
  a.T = (double)n_tx;
  a.metric = (int)metric;
  a.thr = min_threshold;
  a.max_ante = max_antecedent;
  a.keys = d_keys.as<unsigned long long>();
  a.vals = d_vals.as<int32_t>();
  a.mask = cap - 1;
  a.scratch = sbits ? d_scr.as<int32_t>() : nullptr;
  a.scratch_bits = sbits;
  a.ticket = (unsigned long long*)d_ctl.p;
  a.error = (unsigned int*)((char*)d_ctl.p + 16);
  a.pass = 0;
  a.nrules = d_nr.as<int64_t>();
  kern::rules_pass(a, grid, s);
  const size_t tb = kern::rules_scan_temp_bytes(n);
  DevBuf d_tmp(tb);
  kern::rules_scan(d_nr.as<int64_t>(), d_off.as<int64_t>(), n, d_tmp.p, tb, s);
  int64_t total = 0;
  unsigned int err = 0;
  KMLS_HIP(hipMemcpyAsync(&total, d_off.as<int64_t>() + n, 8, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipMemcpyAsync(&err, a.error, 4, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  KMLS_CHECK(err == 0, "GPU rules: a subset of a frequent itemset is missing from the trie "
                       "(trie not closed under subsets, or itemset longer than 30)");
  DevBuf o_is(total * 8), o_a(total * 8), o_c(total * 8), o_conf(total * 8), o_lift(total * 8);
  KMLS_HIP(hipMemsetAsync(d_ctl.p, 0, 8, s));  // ticket
  a.pass = 1;
  a.off = d_off.as<int64_t>();
  a.o_itemset = o_is.as<int64_t>();
  a.o_ante = o_a.as<int64_t>();
  a.o_cons = o_c.as<int64_t>();
  a.o_conf = o_conf.as<double>();
  a.o_lift = o_lift.as<double>();
  kern::rules_pass(a, grid, s);
  KMLS_HIP(hipEventRecord(e1, s));
  out.itemset.resize((size_t)total);
  out.antecedent.resize((size_t)total);
  out.consequent.resize((size_t)total);
  out.confidence.resize((size_t)total);
  out.lift.resize((size_t)total);
  if (total) {
    KMLS_HIP(hipMemcpyAsync(out.itemset.data(), o_is.p, total * 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(out.antecedent.data(), o_a.p, total * 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(out.consequent.data(), o_c.p, total * 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(out.confidence.data(), o_conf.p, total * 8, hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(out.lift.data(), o_lift.p, total * 8, hipMemcpyDeviceToHost, s));
  }
  KMLS_HIP(hipStreamSynchronize(s));
  float ms = 0.f;
  KMLS_HIP(hipEventElapsedTime(&ms, e0, e1));
  if (kernel_ms) *kernel_ms = ms;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return out;
}

CSR group_to_csr_gpu(int device, const int32_t* keys, const int32_t* vals, int64_t n,
                     int32_t n_keys, bool dedup) {
  trace::Range rg_("kmls.groupby_gpu");
  KMLS_CHECK(n < (1ll << 31), "GPU group-by: more than 2^31 rows per call");
  KMLS_HIP(hipSetDevice(device));
  hipStream_t s;
  KMLS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{s};
  DevBuf d_k(n * 4), d_v(n * 4), d_ptr((size_t)(n_keys + 1) * 8), d_idx(n * 4);
  const size_t tb = kern::groupby_csr_temp_bytes(n, n_keys);
  DevBuf d_tmp(tb);
  KMLS_HIP(hipMemcpyAsync(d_k.p, keys, n * 4, hipMemcpyHostToDevice, s));
  KMLS_HIP(hipMemcpyAsync(d_v.p, vals, n * 4, hipMemcpyHostToDevice, s));
  const int64_t nnz = kern::groupby_csr(d_k.as<int32_t>(), d_v.as<int32_t>(), n, n_keys, dedup,
                                        d_ptr.as<int64_t>(), d_idx.as<int32_t>(), d_tmp.p, tb, s);
  CSR out;
  out.ptr.resize((size_t)n_keys + 1);
  out.idx.resize((size_t)nnz);
  KMLS_HIP(hipMemcpyAsync(out.ptr.data(), d_ptr.p, out.ptr.size() * 8, hipMemcpyDeviceToHost, s));
  if (nnz) KMLS_HIP(hipMemcpyAsync(out.idx.data(), d_idx.p, (size_t)nnz * 4, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  return out;
}

}  // namespace gpu
}  // namespace kmls
