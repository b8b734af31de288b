// pybind11 bindings of the HIP runtime objects (GpuMiner, GpuRuleIndex).
#include <cstring>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../kernels/kernels.hpp"
#include "kmls/gpu.hpp"
#include "kmls/trace.hpp"

namespace py = pybind11;

namespace kmls {

namespace {
template <typename T>
py::array_t<T> to_array(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>({(py::ssize_t)heap->size()}, {(py::ssize_t)sizeof(T)}, heap->data(), owner);
}

template <typename T>
py::array_t<T> pinned_array(const std::shared_ptr<void>& buf, int64_t n) {
  if (!buf) return py::array_t<T>(0);
  auto* keep = new std::shared_ptr<void>(buf);
  py::capsule owner(keep, [](void* p) { delete reinterpret_cast<std::shared_ptr<void>*>(p); });
  return py::array_t<T>({(py::ssize_t)n}, {(py::ssize_t)sizeof(T)}, (T*)buf.get(), owner);
}

py::dict result_to_dict(gpu::GpuMineResult&& r) {
  py::dict d;
  // element widths follow the download format (compact on the device-resident path)
  if (r.par_w == 4) d["parent"] = pinned_array<int32_t>(r.h_parent, r.n_nodes);
  else d["parent"] = pinned_array<int64_t>(r.h_parent, r.n_nodes);
  if (r.item_w == 2) d["item"] = pinned_array<uint16_t>(r.h_item, r.n_nodes);
  else d["item"] = pinned_array<int32_t>(r.h_item, r.n_nodes);
  if (r.cnt_w == 2) d["count"] = pinned_array<uint16_t>(r.h_count, r.n_nodes);
  else d["count"] = pinned_array<uint32_t>(r.h_count, r.n_nodes);
  d["depth"] = pinned_array<uint8_t>(r.h_depth, r.n_nodes);
  py::dict s;
  s["n_frequent_items"] = r.stats.n_frequent_items;
  s["n_itemsets"] = r.stats.n_itemsets;
  s["n_candidates"] = r.stats.n_candidates;
  s["max_depth"] = r.stats.max_depth;
  s["seconds"] = r.stats.seconds;
  s["arena_high_water"] = r.arena_high_water;
  s["levels_path"] = r.levels_path;
  s["level2_method"] = r.level2_method;
  s["cooc_pairs"] = r.cooc_pairs;
  s["level2_comm"] = r.level2_comm;
  if (r.hl_tx_kept >= 0) {
    py::dict h;
    h["tx_kept"] = r.hl_tx_kept;
    h["nnz_kept"] = r.hl_nnz_kept;
    h["per_level"] = r.hl_per_level;
    h["hits"] = r.hl_hits;
    s["horizontal"] = h;
  }
  py::dict ph;
  for (auto& p : r.phases) ph[py::str(p.name)] = p.ms;
  s["phases_ms"] = ph;
  d["stats"] = s;
  if (r.idx_nnz >= 0) {  // rule map built on the device (cfg.rule_index)
    py::dict ix;
    ix["nnz"] = r.idx_nnz;
    ix["row_ptr"] = pinned_array<int64_t>(r.h_idx_row_ptr, r.n_items_idx);
    ix["cons"] = pinned_array<int32_t>(r.h_idx_cons, r.idx_nnz);
    ix["count"] = pinned_array<uint32_t>(r.h_idx_cnt, r.idx_nnz);
    d["index"] = ix;
  }
  return d;
}

MineConfig make_cfg(double ms, int max_len, bool pairs_only, bool gram, bool mfma,
                    bool rule_index = false) {
  MineConfig c;
  c.rule_index = rule_index;
  c.min_support = ms;
  c.max_len = max_len;
  c.pairs_only = pairs_only;
  c.level2_gram = gram;
  c.level2_mfma = mfma;
  return c;
}

using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
using U32 = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>;
using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;
}  // namespace

static gpu::CommDtype comm_dtype(const std::string& s) {
  if (s == "u32") return gpu::CommDtype::U32;
  if (s == "u64") return gpu::CommDtype::U64;
  if (s == "i64") return gpu::CommDtype::I64;
  if (s == "f64") return gpu::CommDtype::F64;
  throw std::invalid_argument("comm dtype must be u32, u64, i64 or f64");
}

static int shm_kind(const py::array& buf) {
  const auto k = buf.dtype().kind();
  const size_t e = (size_t)buf.itemsize();
  if (k == 'u' && e == 4) return 0;
  if (k == 'i' && e == 8) return 1;
  if (k == 'u' && e == 8) return 2;
  if (k == 'f' && e == 8) return 3;
  throw std::invalid_argument("dtype must be uint32, int64, uint64 or float64");
}

void register_gpu_bindings(py::module_& m) {
  m.def("gpu_available", &gpu::available);
  m.def("roctx_enabled", &trace::enabled);
  m.def("roctx_push", [](const std::string& n) { trace::push(n.c_str()); });
  m.def("roctx_pop", &trace::pop);
  m.def("gpu_device_count", &gpu::device_count);
  m.def("extend_split_launches", &kern::extend_split_launches);
  m.def("gpu_device_name", &gpu::device_name);

  m.def("association_rules_gpu", [](I64 parent, I32 item, U32 count, U8 depth, int64_t n_tx,
                                    int metric, double min_threshold, int max_antecedent,
                                    int device) {
    const int64_t n = item.size();
    KMLS_CHECK(parent.size() == n && count.size() == n && depth.size() == n, "trie arrays differ in size");
    RuleSet r;
    double ms = 0;
    {
      py::gil_scoped_release nogil;
      r = gpu::association_rules_gpu(device, parent.data(), item.data(), count.data(), depth.data(),
                                     n, n_tx, (RuleMetric)metric, min_threshold, max_antecedent, &ms);
    }
    py::dict d;
    d["itemset"] = to_array(std::move(r.itemset));
    d["antecedent"] = to_array(std::move(r.antecedent));
    d["consequent"] = to_array(std::move(r.consequent));
    d["confidence"] = to_array(std::move(r.confidence));
    d["lift"] = to_array(std::move(r.lift));
    d["kernel_ms"] = ms;
    return d;
  }, py::arg("parent"), py::arg("item"), py::arg("count"), py::arg("depth"), py::arg("n_tx"),
     py::arg("metric") = 0, py::arg("min_threshold") = 0.8, py::arg("max_antecedent") = 0,
     py::arg("device") = 0);

  m.def("group_to_csr_gpu", [](I32 keys, I32 vals, int32_t n_keys, bool dedup, int device) {
    KMLS_CHECK(keys.size() == vals.size(), "keys/vals differ in size");
    CSR g;
    {
      py::gil_scoped_release nogil;
      g = gpu::group_to_csr_gpu(device, keys.data(), vals.data(), keys.size(), n_keys, dedup);
    }
    return py::make_tuple(to_array(std::move(g.ptr)), to_array(std::move(g.idx)));
  }, py::arg("keys"), py::arg("vals"), py::arg("n_keys"), py::arg("dedup") = true,
     py::arg("device") = 0);

  m.def("comm_unique_id", []() { return py::bytes(gpu::comm_unique_id()); });
  m.def("host_comm_unique_id", []() { return py::bytes(host_comm_unique_id()); });
  py::class_<gpu::Comm>(m, "Comm")
      .def(py::init([](int rank, int world, py::bytes uid, int device, const std::string& backend) {
             std::string u = uid;
             py::gil_scoped_release nogil;
             return new gpu::Comm(rank, world, u, device, backend);
           }), py::arg("rank"), py::arg("world"), py::arg("uid"), py::arg("device"),
           py::arg("backend") = "rccl")
      .def_property_readonly("rank", &gpu::Comm::rank)
      .def_property_readonly("world", &gpu::Comm::world)
      .def_property_readonly("backend", &gpu::Comm::backend)
      .def("all_reduce_u32", [](gpu::Comm& c, uintptr_t buf, size_t n, uintptr_t stream) {
        py::gil_scoped_release nogil;
        c.all_reduce((void*)buf, (void*)buf, n, gpu::CommDtype::U32, false, (void*)stream);
      })
      .def("wait_stream", [](gpu::Comm& c, uintptr_t stream) {
        py::gil_scoped_release nogil;
        c.wait_stream((void*)stream);
      })
      // device-pointer collectives (u32/u64/i64/f64 by name), ordered on `stream`
      .def("all_reduce", [](gpu::Comm& c, uintptr_t send, uintptr_t recv, size_t n,
                            const std::string& dt, bool max_op, uintptr_t stream) {
        const gpu::CommDtype t = comm_dtype(dt);
        py::gil_scoped_release nogil;
        c.all_reduce((void*)send, (void*)recv, n, t, max_op, (void*)stream);
      }, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
         py::arg("max_op") = false, py::arg("stream") = 0)
      .def("all_gather", [](gpu::Comm& c, uintptr_t send, uintptr_t recv, size_t n,
                            const std::string& dt, uintptr_t stream) {
        const gpu::CommDtype t = comm_dtype(dt);
        py::gil_scoped_release nogil;
        c.all_gather((void*)send, (void*)recv, n, t, (void*)stream);
      }, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
         py::arg("stream") = 0)
      .def("reduce_scatter", [](gpu::Comm& c, uintptr_t send, uintptr_t recv, size_t n,
                                const std::string& dt, bool max_op, uintptr_t stream) {
        const gpu::CommDtype t = comm_dtype(dt);
        py::gil_scoped_release nogil;
        c.reduce_scatter((void*)send, (void*)recv, n, t, max_op, (void*)stream);
      }, py::arg("send"), py::arg("recv"), py::arg("recv_count"), py::arg("dtype"),
         py::arg("max_op") = false, py::arg("stream") = 0)
      .def("all_to_all", [](gpu::Comm& c, uintptr_t send, uintptr_t recv, size_t n,
                            const std::string& dt, uintptr_t stream) {
        const gpu::CommDtype t = comm_dtype(dt);
        py::gil_scoped_release nogil;
        c.all_to_all((void*)send, (void*)recv, n, t, (void*)stream);
      }, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
         py::arg("stream") = 0)
      .def("sendrecv", [](gpu::Comm& c, uintptr_t send, int send_peer, uintptr_t recv,
                          int recv_peer, size_t n, const std::string& dt, uintptr_t stream) {
        const gpu::CommDtype t = comm_dtype(dt);
        py::gil_scoped_release nogil;
        c.sendrecv((void*)send, send_peer, (void*)recv, recv_peer, n, t, (void*)stream);
      }, py::arg("send"), py::arg("send_peer"), py::arg("recv"), py::arg("recv_peer"),
         py::arg("count"), py::arg("dtype"), py::arg("stream") = 0)
      .def("abort", &gpu::Comm::abort);

  // host shared-memory communicator on its own (CPU multi-process tests of the backend)
  py::class_<ShmComm>(m, "ShmComm")
      .def(py::init([](int rank, int world, py::bytes uid) {
             std::string u = uid;
             py::gil_scoped_release nogil;
             return new ShmComm(rank, world, u);
           }), py::arg("rank"), py::arg("world"), py::arg("uid"))
      .def("all_reduce", [](ShmComm& c, py::array buf, bool max_op) {
        KMLS_CHECK(buf.flags() & py::array::c_style, "buffer must be C-contiguous");
        KMLS_CHECK(buf.writeable(), "buffer must be writeable");
        const auto k = buf.dtype().kind();
        const size_t e = (size_t)buf.itemsize();
        int kind = -1;
        if (k == 'u' && e == 4) kind = 0;
        else if (k == 'i' && e == 8) kind = 1;
        else if (k == 'u' && e == 8) kind = 2;
        else if (k == 'f' && e == 8) kind = 3;
        KMLS_CHECK(kind >= 0, "dtype must be uint32, int64, uint64 or float64");
        void* p = buf.mutable_data();
        const size_t n = (size_t)buf.size();
        py::gil_scoped_release nogil;
        c.all_reduce(p, n, e, kind, max_op);
      }, py::arg("buf"), py::arg("max_op") = false)
      .def("reduce_scatter", [](ShmComm& c, py::array send, bool max_op) {
        KMLS_CHECK(send.flags() & py::array::c_style, "buffer must be C-contiguous");
        const int kind = shm_kind(send);
        const size_t e = (size_t)send.itemsize(), n = (size_t)send.size();
        KMLS_CHECK(n % (size_t)c.world() == 0, "send size must be a multiple of world");
        py::array out(send.dtype(), std::vector<py::ssize_t>{(py::ssize_t)(n / c.world())});
        const void* sp = send.data();
        void* op = out.mutable_data();
        {
          py::gil_scoped_release nogil;
          c.reduce_scatter(sp, op, n / c.world(), e, kind, max_op);
        }
        return out;
      }, py::arg("send"), py::arg("max_op") = false)
      .def("all_to_all", [](ShmComm& c, py::array send) {
        KMLS_CHECK(send.flags() & py::array::c_style, "buffer must be C-contiguous");
        const size_t bytes = (size_t)send.nbytes();
        KMLS_CHECK(bytes % (size_t)c.world() == 0, "send size must be a multiple of world");
        py::array out(send.dtype(), std::vector<py::ssize_t>{(py::ssize_t)send.size()});
        const void* sp = send.data();
        void* op = out.mutable_data();
        {
          py::gil_scoped_release nogil;
          c.all_to_all(sp, op, bytes / c.world());
        }
        return out;
      })
      .def("sendrecv", [](ShmComm& c, py::array send, int send_peer, int recv_peer) {
        KMLS_CHECK(send.flags() & py::array::c_style, "buffer must be C-contiguous");
        py::array out(send.dtype(), std::vector<py::ssize_t>{(py::ssize_t)send.size()});
        const void* sp = send.data();
        void* op = out.mutable_data();
        const size_t bytes = (size_t)send.nbytes();
        {
          py::gil_scoped_release nogil;
          c.sendrecv(sp, bytes, send_peer, op, bytes, recv_peer);
        }
        return out;
      })
      .def("barrier", &ShmComm::barrier, py::call_guard<py::gil_scoped_release>())
      .def("abort", &ShmComm::abort);

  py::class_<gpu::GpuMiner>(m, "GpuMiner")
      .def(py::init<int, size_t, uintptr_t>(), py::arg("device") = 0, py::arg("arena_bytes") = 0,
           py::arg("stream") = 0)
      .def("load_csr", [](gpu::GpuMiner& g, I64 tx_ptr, I32 items, int64_t n_items) {
        KMLS_CHECK(tx_ptr.size() >= 1, "tx_ptr must have T+1 entries");
        py::gil_scoped_release nogil;
        g.load_csr(tx_ptr.data(), items.data(), tx_ptr.size() - 1, n_items);
      })
      .def_property_readonly("n_tx", &gpu::GpuMiner::n_tx)
      .def_property_readonly("n_items", &gpu::GpuMiner::n_items)
      .def_property_readonly("stream", &gpu::GpuMiner::stream)
      .def_property_readonly("arena_capacity", &gpu::GpuMiner::arena_capacity)
      .def("item_support", &gpu::GpuMiner::item_support, py::call_guard<py::gil_scoped_release>())
      .def("select", [](gpu::GpuMiner& g, U32 counts, int64_t n_tx, double ms) {
        KMLS_CHECK(counts.size() == g.n_items(), "counts size != n_items");
        py::gil_scoped_release nogil;
        return g.select(counts.data(), n_tx, ms);
      })
      .def("select_device", [](gpu::GpuMiner& g, uintptr_t d_counts, int64_t n_tx, double ms) {
        // the selection from supports already on the device (an all-reduced histogram): no
        // copies of the vocabulary's counts either way
        py::gil_scoped_release nogil;
        return g.select_device((const uint32_t*)d_counts, n_tx, ms, nullptr);
      }, py::arg("counts"), py::arg("n_tx"), py::arg("min_support"))
      .def("use_frequent_subset", [](gpu::GpuMiner& g, I64 keep) {
        py::gil_scoped_release nogil;
        g.use_frequent_subset(keep.data(), (int64_t)keep.size());
      }, py::arg("keep"))
      .def("frequent", [](const gpu::GpuMiner& g) {
        auto& f = g.frequent();
        return py::make_tuple(to_array(std::vector<int32_t>(f.ids)),
                              to_array(std::vector<uint32_t>(f.counts)), f.minsup2);
      })
      .def("words_local", &gpu::GpuMiner::words_local)
      .def("encode_bitmaps", &gpu::GpuMiner::encode_bitmaps, py::call_guard<py::gil_scoped_release>())
      .def("pair_counts", &gpu::GpuMiner::pair_counts, py::call_guard<py::gil_scoped_release>())
      .def("pair_counts_csr", &gpu::GpuMiner::pair_counts_csr, py::arg("out"), py::arg("ld"),
           py::call_guard<py::gil_scoped_release>())
      .def("cooc_check", &gpu::GpuMiner::cooc_check, py::call_guard<py::gil_scoped_release>())
      .def("cooc_likely", &gpu::GpuMiner::cooc_likely)
      .def("pair_counts_csr_direct", &gpu::GpuMiner::pair_counts_csr_direct, py::arg("out"),
           py::arg("ld"), py::call_guard<py::gil_scoped_release>())
      .def("subset_active", &gpu::GpuMiner::subset_active)
      .def("cooc_preferred", &gpu::GpuMiner::cooc_preferred,
           py::call_guard<py::gil_scoped_release>())
      .def("cooc_stats", [](gpu::GpuMiner& g) {
        gpu::GpuMiner::CoocStats st;
        {
          py::gil_scoped_release nogil;
          st = g.cooc_stats();
        }
        py::dict d;
        d["pairs"] = st.pairs;
        d["max_k"] = st.max_k;
        return d;
      })
      .def("rule_map_from_gram",
           [](gpu::GpuMiner& g, uintptr_t gram, int64_t ld, uint32_t minsup) {
             gpu::GpuMiner::RuleMap m;
             {
               py::gil_scoped_release nogil;
               m = g.rule_map_from_gram(gram, ld, minsup);
             }
             py::dict d;
             d["nnz"] = m.nnz;
             d["status"] = m.status;
             d["row_ptr"] = py::array_t<int64_t>((py::ssize_t)m.row_ptr.size(), m.row_ptr.data());
             d["cons"] = py::array_t<int32_t>((py::ssize_t)m.cons.size(), m.cons.data());
             d["count"] = py::array_t<uint32_t>((py::ssize_t)m.cnt.size(), m.cnt.data());
             return d;
           },
           py::arg("gram"), py::arg("ld"), py::arg("minsup"))
      .def("gram_mirror", &gpu::GpuMiner::gram_mirror, py::arg("gram"), py::arg("ld"), py::arg("F"),
           py::call_guard<py::gil_scoped_release>())
      .def("rows_union", &gpu::GpuMiner::rows_union, py::arg("rows"), py::arg("Wp"), py::arg("idx"),
           py::arg("n"), py::arg("W"), py::arg("mask"), py::call_guard<py::gil_scoped_release>())
      .def("word_popc", &gpu::GpuMiner::word_popc, py::arg("mask"), py::arg("W"), py::arg("cnt"),
           py::call_guard<py::gil_scoped_release>())
      .def("compact_rows", &gpu::GpuMiner::compact_rows, py::arg("rows"), py::arg("R"),
           py::arg("Wp_in"), py::arg("mask"), py::arg("nzw"), py::arg("off"), py::arg("n_nz"),
           py::arg("out"), py::arg("Wp_out"), py::call_guard<py::gil_scoped_release>())
      .def("rule_map_rows",
           [](gpu::GpuMiner& g, uintptr_t rows, int64_t ld, int64_t r0, int64_t nrows,
              uint32_t minsup) {
             gpu::GpuMiner::RuleMap m;
             {
               py::gil_scoped_release nogil;
               m = g.rule_map_rows(rows, ld, r0, nrows, minsup);
             }
             py::dict d;
             d["nnz"] = m.nnz;
             d["status"] = m.status;
             d["row_ptr"] = py::array_t<int64_t>((py::ssize_t)m.row_ptr.size(), m.row_ptr.data());
             d["cons"] = py::array_t<int32_t>((py::ssize_t)m.cons.size(), m.cons.data());
             d["count"] = py::array_t<uint32_t>((py::ssize_t)m.cnt.size(), m.cnt.data());
             return d;
           },
           py::arg("rows"), py::arg("ld"), py::arg("r0"), py::arg("nrows"), py::arg("minsup"))
      .def("bitgemm_rect", &gpu::GpuMiner::bitgemm_rect, py::call_guard<py::gil_scoped_release>())
      .def("ring_pair_rows", &gpu::GpuMiner::ring_pair_rows, py::arg("comm"), py::arg("X"),
           py::arg("F"), py::arg("Ws"), py::arg("out"), py::arg("ldo"),
           py::call_guard<py::gil_scoped_release>())
      .def("mine_bitmaps", [](gpu::GpuMiner& g, uintptr_t bm, int64_t Wp, double ms, int max_len,
                              bool pairs_only, py::object owned, bool emit_level1, bool download,
                              bool gram, bool mfma) {
        MineConfig c = make_cfg(ms, max_len, pairs_only, gram, mfma);
        std::vector<uint8_t> own;
        const uint8_t* po = nullptr;
        if (!owned.is_none()) {
          U8 o = owned.cast<U8>();
          own.assign(o.data(), o.data() + o.size());
          KMLS_CHECK((int64_t)own.size() == (int64_t)g.frequent().ids.size(), "owned mask size != F");
          po = own.data();
        }
        gpu::GpuMineResult r;
        {
          py::gil_scoped_release nogil;
          r = g.mine_bitmaps(bm, Wp, c, po, emit_level1, download);
        }
        return result_to_dict(std::move(r));
      }, py::arg("bm"), py::arg("Wp"), py::arg("min_support"), py::arg("max_len") = 0,
         py::arg("pairs_only") = false, py::arg("owned") = py::none(), py::arg("emit_level1") = true,
         py::arg("download") = true, py::arg("gram") = true, py::arg("mfma") = false)
      .def("set_tie_rank", [](gpu::GpuMiner& g, I32 tie) {
        py::gil_scoped_release nogil;
        g.set_tie_rank(tie.data(), tie.size());
      }, py::arg("tie"))
      .def("mine", [](gpu::GpuMiner& g, double ms, int max_len, bool pairs_only, bool download,
                      bool gram, bool mfma, bool prefetch, bool rule_index) {
        MineConfig c = make_cfg(ms, max_len, pairs_only, gram, mfma, rule_index);
        gpu::GpuMineResult r;
        {
          py::gil_scoped_release nogil;
          r = g.mine(c, download, prefetch);
        }
        return result_to_dict(std::move(r));
      }, py::arg("min_support"), py::arg("max_len") = 0, py::arg("pairs_only") = false,
         py::arg("download") = true, py::arg("gram") = true, py::arg("mfma") = false,
         py::arg("prefetch") = false, py::arg("rule_index") = false)
      .def("mine_partition", [](gpu::GpuMiner& g, double ms, int max_len, bool download, int rank,
                                int world, bool prefetch, bool rule_index) {
        gpu::GpuMineResult r;
        {
          py::gil_scoped_release nogil;
          r = g.mine_partition(make_cfg(ms, max_len, false, true, false, rule_index),
                               download, rank, world, prefetch);
        }
        return result_to_dict(std::move(r));
      }, py::arg("min_support"), py::arg("max_len") = 0, py::arg("download") = true,
         py::arg("rank") = 0, py::arg("world") = 1, py::arg("prefetch") = false,
         py::arg("rule_index") = false)
      .def("mine_txdp", [](gpu::GpuMiner& g, gpu::Comm* comm, int64_t global_n_tx, double ms,
                           int max_len, bool download, bool mfma, int support_tiles) {
        gpu::GpuMineResult r;
        {
          py::gil_scoped_release nogil;
          r = g.mine_txdp(comm, global_n_tx, make_cfg(ms, max_len, false, true, mfma), download,
                          support_tiles);
        }
        return result_to_dict(std::move(r));
      }, py::arg("comm"), py::arg("global_n_tx"), py::arg("min_support"), py::arg("max_len") = 0,
         py::arg("download") = true, py::arg("mfma") = false, py::arg("support_tiles") = 4)
      .def("mine_shard", [](gpu::GpuMiner& g, gpu::Comm* comm, int64_t global_n_tx, double ms,
                            int max_len, bool download, int support_tiles) -> py::object {
        gpu::GpuMineResult r;
        bool declined = false;
        {
          py::gil_scoped_release nogil;
          r = g.mine_shard(comm, global_n_tx, make_cfg(ms, max_len, false, true, false), download,
                           support_tiles, &declined);
        }
        if (declined) return py::none();
        return result_to_dict(std::move(r));
      }, py::arg("comm"), py::arg("global_n_tx"), py::arg("min_support"), py::arg("max_len") = 0,
         py::arg("download") = true, py::arg("support_tiles") = 4)
      .def("mine_deep", [](gpu::GpuMiner& g, double ms, int max_len, int rank, int world,
                           py::object comm, unsigned long long budget0, unsigned long long budget,
                           unsigned split_min, int blocks_per_cu, int stack_mb, bool steal,
                           unsigned steal_idle, int assign, bool trace, unsigned presplit_cost,
                           unsigned long long presplit_budget, bool emit, int deal_key) {
        gpu::DeepOpts o;
        o.emit = emit;
        o.deal_key = deal_key;
        o.assign = assign;
        o.trace = trace;
        o.presplit_cost = presplit_cost;
        o.presplit_budget = presplit_budget;
        o.steal = steal;
        o.steal_idle = steal_idle;
        o.budget0 = budget0;
        o.budget = budget;
        o.split_min = split_min;
        o.blocks_per_cu = blocks_per_cu;
        o.stack_mb = stack_mb;
        gpu::Comm* c = comm.is_none() ? nullptr : comm.cast<gpu::Comm*>();
        gpu::DeepResult r;
        {
          py::gil_scoped_release nogil;
          r = g.mine_deep(ms, max_len, rank, world, c, o);
        }
        py::dict d;
        d["per_level"] = r.per_level;
        d["n_itemsets"] = r.n_itemsets;
        d["n_frequent_items"] = r.n_frequent_items;
        d["max_depth"] = r.max_depth;
        d["candidates"] = r.candidates;
        d["chunks"] = r.chunks;
        d["level2_tasks"] = r.level2_tasks;
        char buf[64];
        std::snprintf(buf, sizeof buf, "%016llx%016llx", (unsigned long long)r.digest_sum,
                      (unsigned long long)r.digest_xor);
        d["digest"] = std::string(buf);
        d["round_tasks"] = r.round_tasks;
        d["spilled_tasks"] = r.spilled_tasks;
        d["handoffs"] = r.handoffs;
        d["round_ms"] = r.round_ms;
        py::dict ph;
        ph["prologue"] = r.ms_prologue;
        ph["level2_classes"] = r.ms_root;
        ph["rounds"] = r.ms_rounds;
        ph["combine"] = r.ms_combine;
        ph["total"] = r.ms_total;
        ph["assign"] = r.ms_assign;
        ph["presplit"] = r.ms_presplit;
        d["presplit"] = py::make_tuple(r.presplit_in, r.presplit_out);
        if (emit) {
          d["arena_nodes"] = r.arena_nodes;
          d["arena_cap"] = r.arena_cap;
        }
        d["phases_ms"] = ph;
        if (trace) {
          const size_t nw = r.trace.size() / kern::kDeepTraceWords;
          py::array_t<uint64_t> tr({(py::ssize_t)nw, (py::ssize_t)kern::kDeepTraceWords});
          if (!r.trace.empty()) std::memcpy(tr.mutable_data(), r.trace.data(), r.trace.size() * 8);
          d["trace"] = tr;
          d["task_ticks"] = py::array_t<uint64_t>((py::ssize_t)r.task_ticks.size(), r.task_ticks.data());
          d["task_ids"] = py::array_t<int64_t>((py::ssize_t)r.task_ids.size(), r.task_ids.data());
          d["task_cost"] = py::array_t<uint32_t>((py::ssize_t)r.task_cost.size(), r.task_cost.data());
          d["clock_khz"] = r.clock_khz;
          d["t_drain"] = r.t_drain;
          d["trace_bucket"] = r.trace_bucket;
        }
        return d;
      }, py::arg("min_support"), py::arg("max_len") = 0, py::arg("rank") = 0, py::arg("world") = 1,
         py::arg("comm") = py::none(), py::arg("budget0") = 1024ull, py::arg("budget") = 16ull,
         py::arg("split_min") = 8u, py::arg("blocks_per_cu") = 0, py::arg("stack_mb") = 0,
         py::arg("steal") = true, py::arg("steal_idle") = 1u, py::arg("assign") = 1,
         py::arg("trace") = false, py::arg("presplit_cost") = 16u,
         py::arg("presplit_budget") = 1ull, py::arg("emit") = false, py::arg("deal_key") = -1)
      .def("deep_arena_digest", [](gpu::GpuMiner& g, int min_depth) {
        gpu::GpuMiner::ArenaDigest r;
        {
          py::gil_scoped_release nogil;
          r = g.deep_arena_digest(min_depth);
        }
        char buf[64];
        std::snprintf(buf, sizeof buf, "%016llx%016llx", (unsigned long long)r.sum,
                      (unsigned long long)r.xr);
        py::dict d;
        d["digest"] = std::string(buf);
        d["sum"] = r.sum;
        d["xor"] = r.xr;
        d["n"] = r.n;
        d["per_depth"] = r.per_depth;
        return d;
      }, py::arg("min_depth") = 1)
      .def("deep_arena_download", [](gpu::GpuMiner& g, int64_t n) {
        py::array_t<int64_t> parent((py::ssize_t)n);
        py::array_t<int32_t> item((py::ssize_t)n);
        py::array_t<uint32_t> count((py::ssize_t)n);
        py::array_t<uint8_t> depth((py::ssize_t)n);
        int64_t* pp = parent.mutable_data();
        int32_t* pi = item.mutable_data();
        uint32_t* pc = count.mutable_data();
        uint8_t* pd = depth.mutable_data();
        {
          py::gil_scoped_release nogil;
          g.deep_arena_download(n, pp, pi, pc, pd);
        }
        py::dict d;
        d["parent"] = parent;
        d["item"] = item;
        d["count"] = count;
        d["depth"] = depth;
        return d;
      }, py::arg("n"))
      .def("deep_arena_trie", [](gpu::GpuMiner& g, int min_depth, int64_t base) {
        bool item16 = true;
        int64_t n = 0;
        {
          py::gil_scoped_release nogil;
          n = g.deep_arena_trie(min_depth, base, &item16);
        }
        py::array_t<int32_t> parent((py::ssize_t)n);
        py::array item = item16 ? (py::array)py::array_t<uint16_t>((py::ssize_t)n)
                                : (py::array)py::array_t<int32_t>((py::ssize_t)n);
        py::array_t<uint16_t> count((py::ssize_t)n);
        py::array_t<uint8_t> depth((py::ssize_t)n);
        int32_t* pp = parent.mutable_data();
        void* pi = item.mutable_data();
        uint16_t* pc = count.mutable_data();
        uint8_t* pd = depth.mutable_data();
        {
          py::gil_scoped_release nogil;
          g.deep_trie_download(pp, pi, pc, pd);
        }
        py::dict d;
        d["parent"] = parent;
        d["item"] = item;
        d["count"] = count;
        d["depth"] = depth;
        d["n"] = n;
        return d;
      }, py::arg("min_depth") = 1, py::arg("base") = 0)
      .def("synchronize", &gpu::GpuMiner::synchronize, py::call_guard<py::gil_scoped_release>());

  py::class_<gpu::GpuRuleIndex, std::shared_ptr<gpu::GpuRuleIndex>>(m, "GpuRuleIndex")
      .def(py::init<int, const RuleIndex&, uintptr_t>(), py::arg("device"), py::arg("index"),
           py::arg("stream") = 0)
      .def_property_readonly("nnz", &gpu::GpuRuleIndex::nnz)
      .def_property_readonly("max_row", &gpu::GpuRuleIndex::max_row)
      .def("query_batch", [](gpu::GpuRuleIndex& ix, I64 q_ptr, I32 seeds, int k) {
        const int64_t B = q_ptr.size() - 1;
        py::array_t<int32_t> ids({(py::ssize_t)B, (py::ssize_t)k});
        py::array_t<int32_t> ns({(py::ssize_t)B});
        int32_t* po = ids.mutable_data();
        int32_t* pn = ns.mutable_data();
        {
          py::gil_scoped_release nogil;
          ix.query_batch(q_ptr.data(), B, seeds.data(), k, po, pn);
        }
        return py::make_tuple(ids, ns);
      })
      .def("query_loop", [](gpu::GpuRuleIndex& ix, I64 q_ptr, I32 seeds, int k) {
        const int64_t B = q_ptr.size() - 1;
        py::array_t<int32_t> ids({(py::ssize_t)B, (py::ssize_t)k});
        py::array_t<int32_t> ns({(py::ssize_t)B});
        int32_t* po = ids.mutable_data();
        int32_t* pn = ns.mutable_data();
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = ix.query_loop(q_ptr.data(), B, seeds.data(), k, po, pn);
        }
        return py::make_tuple(ids, ns, ok);
      })
      .def("merged_size", [](const gpu::GpuRuleIndex& ix, I32 seeds) {
        return ix.merged_size(seeds.data(), (int64_t)seeds.size());
      });
  m.def("serve_loop_stats", [](int device) {
    const gpu::ServeLoopStats st = gpu::GpuServeLoop::for_device(device).stats();
    py::dict d;
    d["requests"] = st.requests;
    d["queries"] = st.queries;
    d["launches"] = st.launches;
    d["refused"] = st.refused;
    d["last_us"] = st.last_us;
    d["mean_us"] = st.requests ? st.sum_us / (double)st.requests : 0.0;
    d["kernel_mean_us"] = st.requests ? st.kernel_us / (double)st.requests : 0.0;
    d["stage_mean_us"] = st.requests ? st.stage_us / (double)st.requests : 0.0;
    d["compute_mean_us"] = st.requests ? st.compute_us / (double)st.requests : 0.0;
    py::list ph;
    for (int i = 0; i < 4; ++i) ph.append(st.requests ? st.phase_us[i] / (double)st.requests : 0.0);
    d["phase_mean_us"] = ph;
    return d;
  }, py::arg("device") = 0);
  m.def("serve_loop_pause", [](int device, bool pause) {
    if (pause) gpu::GpuServeLoop::for_device(device).pause();
    else gpu::GpuServeLoop::for_device(device).resume();
  }, py::arg("device") = 0, py::arg("pause") = true, py::call_guard<py::gil_scoped_release>());
}

}  // namespace kmls
