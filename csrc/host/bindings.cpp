// pybind11 bindings of the kmls native runtime (module `_native`).
//
// All heavy calls release the GIL.  GPU entry points take raw device pointers / stream
// handles (ints) so Python can hand in torch-allocated HBM buffers and torch's current HIP
// stream; the native code never links libtorch.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "kmls/comm_host.hpp"
#include "kmls/gpu.hpp"
#include "kmls/host.hpp"

namespace py = pybind11;
using namespace kmls;

template <typename T>
static py::array_t<T> to_array(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>({(py::ssize_t)heap->size()}, {(py::ssize_t)sizeof(T)}, heap->data(), owner);
}

static py::dict trie_to_dict(ItemsetTrie&& t) {
  py::dict d;
  d["parent"] = to_array(std::move(t.parent));
  d["item"] = to_array(std::move(t.item));
  d["count"] = to_array(std::move(t.count));
  d["depth"] = to_array(std::move(t.depth));
  return d;
}

using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
using F64 = py::array_t<double, py::array::c_style | py::array::forcecast>;
using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

// KMLS_SEGV_TRACE=1: a SIGSEGV/SIGBUS prints the faulting address and the native backtrace
// (addresses resolve with addr2line against the .so) before the default action.
static void segv_trace(int sig, siginfo_t* si, void*) {
  char buf[96];
  const int n = std::snprintf(buf, sizeof buf, "kmls: signal %d at address %p\n", sig, si->si_addr);
  (void)!write(2, buf, (size_t)n);
  void* frames[64];
  const int k = backtrace(frames, 64);
  backtrace_symbols_fd(frames, k, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static void install_segv_trace() {
  const char* e = std::getenv("KMLS_SEGV_TRACE");
  if (!e || e[0] != '1') return;
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = segv_trace;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
}

PYBIND11_MODULE(_native, m) {
  install_segv_trace();
  m.def("install_segv_trace", &install_segv_trace);
  m.doc() = "kmls native runtime: CSV ingest, CPU/HIP FP-Growth miners, rule-index matchers";

  // ---------------- ingest ----------------
  m.def("read_csv_encoded", [](const std::string& path, const std::vector<std::string>& cols) {
    EncodedTable t;
    {
      py::gil_scoped_release nogil;
      t = read_csv_encoded(path, cols);
    }
    py::dict out;
    out["n_rows"] = t.n_rows;
    out["header"] = t.header;
    py::dict cd;
    for (size_t w = 0; w < t.columns.size(); ++w) {
      py::list u;
      for (auto& s : t.uniques[w]) u.append(py::str(s));
      cd[py::str(t.columns[w])] = py::make_tuple(to_array(std::move(t.codes[w])), u);
    }
    out["columns"] = cd;
    return out;
  }, py::arg("path"), py::arg("columns"));

  m.def("group_to_csr", [](I32 keys, I32 vals, int32_t n_keys, bool dedup, bool sort_rows) {
    KMLS_CHECK(keys.size() == vals.size(), "keys/vals size mismatch");
    CSR g;
    {
      py::gil_scoped_release nogil;
      g = group_to_csr(keys.data(), vals.data(), keys.size(), n_keys, dedup, sort_rows);
    }
    return py::make_tuple(to_array(std::move(g.ptr)), to_array(std::move(g.idx)));
  }, py::arg("keys"), py::arg("vals"), py::arg("n_keys"), py::arg("dedup") = true,
     py::arg("sort_rows") = true);

  // ---------------- thresholds ----------------
  m.def("level1_threshold", &level1_threshold);
  m.def("level2_threshold", &level2_threshold);

  // ---------------- CPU miner ----------------
  m.def("mine_cpu", [](I64 tx_ptr, I32 items, int64_t n_items, double min_support, int max_len,
                       int threads, bool pairs_only) {
    KMLS_CHECK(tx_ptr.size() >= 1, "tx_ptr must have T+1 entries");
    MineConfig cfg;
    cfg.min_support = min_support; cfg.max_len = max_len; cfg.threads = threads;
    cfg.pairs_only = pairs_only;
    MineStats st;
    ItemsetTrie t;
    {
      py::gil_scoped_release nogil;
      t = mine_cpu(tx_ptr.data(), items.data(), tx_ptr.size() - 1, n_items, cfg, &st);
    }
    py::dict d = trie_to_dict(std::move(t));
    py::dict s;
    s["n_frequent_items"] = st.n_frequent_items; s["n_itemsets"] = st.n_itemsets;
    s["n_candidates"] = st.n_candidates; s["max_depth"] = st.max_depth; s["seconds"] = st.seconds;
    d["stats"] = s;
    return d;
  }, py::arg("tx_ptr"), py::arg("items"), py::arg("n_items"), py::arg("min_support"),
     py::arg("max_len") = 0, py::arg("threads") = 0, py::arg("pairs_only") = false);

  m.def("mine_cpu_txdp", [](I64 tx_ptr, I32 items, int64_t n_items, int64_t n_tx_global,
                            double min_support, int max_len, py::object comm) {
    KMLS_CHECK(tx_ptr.size() >= 1, "tx_ptr must have T+1 entries");
    ShmComm* c = comm.is_none() ? nullptr : comm.cast<ShmComm*>();
    MineStats st;
    ItemsetTrie t;
    {
      py::gil_scoped_release nogil;
      t = mine_cpu_txdp(tx_ptr.data(), items.data(), tx_ptr.size() - 1, n_items, n_tx_global,
                        min_support, max_len, c, &st);
    }
    py::dict d = trie_to_dict(std::move(t));
    py::dict s;
    s["n_frequent_items"] = st.n_frequent_items; s["n_itemsets"] = st.n_itemsets;
    s["n_candidates"] = st.n_candidates; s["max_depth"] = st.max_depth;
    d["stats"] = s;
    return d;
  }, py::arg("tx_ptr"), py::arg("items"), py::arg("n_items"), py::arg("n_tx_global"),
     py::arg("min_support"), py::arg("max_len") = 0, py::arg("comm") = py::none());

  m.def("mine_cpu_count", [](I64 tx_ptr, I32 items, int64_t n_items, double min_support,
                             int max_len, int64_t cap, int threads, int rank, int world) {
    KMLS_CHECK(tx_ptr.size() >= 1, "tx_ptr must have T+1 entries");
    CountResult r;
    {
      py::gil_scoped_release nogil;
      r = mine_cpu_count(tx_ptr.data(), items.data(), tx_ptr.size() - 1, n_items, min_support,
                         max_len, cap, threads, rank, world);
    }
    py::dict s;
    s["n_frequent_items"] = r.n_frequent_items; s["n_itemsets"] = r.n_itemsets;
    s["max_depth"] = r.max_depth; s["capped"] = r.capped; s["seconds"] = r.seconds;
    s["per_level"] = r.per_level;
    char buf[64];
    std::snprintf(buf, sizeof buf, "%016llx%016llx", (unsigned long long)r.digest_sum,
                  (unsigned long long)r.digest_xor);
    s["digest"] = std::string(buf);
    return s;
  }, py::arg("tx_ptr"), py::arg("items"), py::arg("n_items"), py::arg("min_support"),
     py::arg("max_len") = 0, py::arg("cap") = (int64_t)1 << 62, py::arg("threads") = 0,
     py::arg("rank") = 0, py::arg("world") = 1);

  m.def("trie_digest", [](py::array parent, py::array item, py::array count, py::object depth,
                          int min_depth) {
    const int64_t n = (int64_t)item.size();
    KMLS_CHECK((int64_t)parent.size() == n && (int64_t)count.size() == n, "trie arrays differ in size");
    auto cont = [](const py::array& a) {
      KMLS_CHECK(a.flags() & py::array::c_style, "trie_digest: arrays must be C-contiguous");
      return a.data();
    };
    const uint8_t* dp = nullptr;
    U8 d8;
    if (!depth.is_none()) {
      d8 = depth.cast<U8>();
      KMLS_CHECK((int64_t)d8.size() == n, "depth size differs");
      dp = d8.data();
    }
    install_segv_trace();
    const void *pp = cont(parent), *ip = cont(item), *cp = cont(count);
    const int pw = (int)parent.itemsize(), iw = (int)item.itemsize(), cw = (int)count.itemsize();
    TrieDigest r;
    {
      py::gil_scoped_release nogil;
      r = trie_digest(pp, pw, ip, iw, cp, cw, dp, n, min_depth);
    }
    char buf[64];
    std::snprintf(buf, sizeof buf, "%016llx%016llx", (unsigned long long)r.sum,
                  (unsigned long long)r.xr);
    py::dict out;
    out["n"] = r.n;
    out["digest"] = std::string(buf);
    out["sum"] = r.sum;
    out["xor"] = r.xr;
    out["per_depth"] = r.per_depth;
    return out;
  }, py::arg("parent"), py::arg("item"), py::arg("count"), py::arg("depth") = py::none(),
     py::arg("min_depth") = 0);

  m.def("synth_transactions", [](int64_t n_tx, int64_t n_items, double mean_len, int n_genres,
                                 double affinity, double zipf_s, uint64_t seed, int threads,
                                 int64_t tx_begin, int64_t tx_end) {
    std::vector<int64_t> ptr;
    std::vector<int32_t> items;
    {
      py::gil_scoped_release nogil;
      synth_transactions(n_tx, n_items, mean_len, n_genres, affinity, zipf_s, seed, threads, ptr,
                         items, tx_begin, tx_end);
    }
    return py::make_tuple(to_array(std::move(ptr)), to_array(std::move(items)));
  }, py::arg("n_tx"), py::arg("n_items"), py::arg("mean_len"), py::arg("n_genres"),
     py::arg("affinity"), py::arg("zipf_s") = 0.85, py::arg("seed") = 0, py::arg("threads") = 0,
     py::arg("tx_begin") = 0, py::arg("tx_end") = -1);

  m.def("select_frequent", [](py::array_t<uint32_t, py::array::c_style | py::array::forcecast> counts,
                              int64_t n_tx, double ms) {
    FrequentItems f = select_frequent(counts.data(), counts.size(), (uint64_t)n_tx, ms);
    return py::make_tuple(to_array(std::move(f.ids)), to_array(std::move(f.counts)),
                          to_array(std::move(f.rank_of)), f.minsup2);
  });
  m.def("encode_bitmaps_cpu", [](I64 tx_ptr, I32 items, I32 rank_of, int64_t F, int64_t W) {
    py::array_t<uint64_t> bm({(py::ssize_t)F, (py::ssize_t)W});
    uint64_t* p = bm.mutable_data();
    {
      py::gil_scoped_release nogil;
      std::fill(p, p + F * W, 0ull);
      encode_bitmaps_cpu(tx_ptr.data(), items.data(), tx_ptr.size() - 1, rank_of.data(), p, W);
    }
    return bm;
  });
  m.def("mine_cpu_bitmaps", [](py::array_t<uint64_t, py::array::c_style | py::array::forcecast> bm,
                               I32 ids, py::array_t<uint32_t, py::array::c_style | py::array::forcecast> counts,
                               uint32_t minsup, int max_len, py::object owned, int threads) {
    KMLS_CHECK(bm.ndim() == 2 && bm.shape(0) == ids.size(), "bm must be [F][W]");
    FrequentItems fi;
    fi.ids.assign(ids.data(), ids.data() + ids.size());
    fi.counts.assign(counts.data(), counts.data() + counts.size());
    fi.minsup2 = minsup;
    std::vector<uint8_t> own;
    if (!owned.is_none()) {
      U8 o = owned.cast<U8>();
      own.assign(o.data(), o.data() + o.size());
      KMLS_CHECK(own.size() == fi.ids.size(), "owned mask size != F");
    }
    MineStats st;
    ItemsetTrie t;
    {
      py::gil_scoped_release nogil;
      t = mine_cpu_bitmaps(bm.data(), bm.shape(0), bm.shape(1), fi, max_len, threads,
                           own.empty() ? nullptr : own.data(), &st);
    }
    py::dict d = trie_to_dict(std::move(t));
    py::dict s;
    s["n_frequent_items"] = st.n_frequent_items; s["n_itemsets"] = st.n_itemsets;
    s["n_candidates"] = st.n_candidates; s["max_depth"] = st.max_depth; s["seconds"] = st.seconds;
    d["stats"] = s;
    return d;
  }, py::arg("bm"), py::arg("ids"), py::arg("counts"), py::arg("minsup"), py::arg("max_len") = 0,
     py::arg("owned") = py::none(), py::arg("threads") = 0);

  // ---------------- association rules ----------------
  m.def("association_rules", [](I64 parent, I32 item, py::array_t<uint32_t, py::array::c_style | py::array::forcecast> count,
                                U8 depth, int64_t n_tx, int metric, double min_threshold,
                                int max_antecedent, int threads) {
    const int64_t n = item.size();
    KMLS_CHECK(parent.size() == n && count.size() == n && depth.size() == n, "trie arrays differ in size");
    RuleSet r;
    {
      py::gil_scoped_release nogil;
      r = association_rules_cpu(parent.data(), item.data(), count.data(), depth.data(), n, n_tx,
                                (RuleMetric)metric, min_threshold, max_antecedent, threads);
    }
    py::dict d;
    d["itemset"] = to_array(std::move(r.itemset));
    d["antecedent"] = to_array(std::move(r.antecedent));
    d["consequent"] = to_array(std::move(r.consequent));
    d["confidence"] = to_array(std::move(r.confidence));
    d["lift"] = to_array(std::move(r.lift));
    return d;
  }, py::arg("parent"), py::arg("item"), py::arg("count"), py::arg("depth"), py::arg("n_tx"),
     py::arg("metric") = 0, py::arg("min_threshold") = 0.8, py::arg("max_antecedent") = 0,
     py::arg("threads") = 0);

  // ---------------- CPU matcher ----------------
  py::class_<RuleIndex, std::shared_ptr<RuleIndex>>(m, "RuleIndex")
      .def(py::init([](int64_t n_items, I64 row_ptr, I32 cons, F64 score, U8 is_key) {
        return std::make_shared<RuleIndex>(
            n_items, std::vector<int64_t>(row_ptr.data(), row_ptr.data() + row_ptr.size()),
            std::vector<int32_t>(cons.data(), cons.data() + cons.size()),
            std::vector<double>(score.data(), score.data() + score.size()),
            std::vector<uint8_t>(is_key.data(), is_key.data() + is_key.size()));
      }))
      .def_property_readonly("n_items", &RuleIndex::n_items)
      .def_property_readonly("nnz", &RuleIndex::nnz)
      .def("query", [](const RuleIndex& ix, I32 seeds, int k) -> py::object {
        std::vector<int32_t> ids((size_t)std::max(k, 0));
        int n;
        {
          py::gil_scoped_release nogil;
          n = ix.query(seeds.data(), (int)seeds.size(), k, ids.data(), nullptr);
        }
        if (n < 0) return py::none();
        ids.resize((size_t)n);
        return to_array(std::move(ids));
      })
      .def("query_batch", [](const RuleIndex& ix, I64 q_ptr, I32 seeds, int k) {
        // returns (ids int32[B,k], n int32[B]) ; n = -1 means "no seed known"
        const int64_t B = q_ptr.size() - 1;
        py::array_t<int32_t> ids({(py::ssize_t)B, (py::ssize_t)k});
        py::array_t<int32_t> ns({(py::ssize_t)B});
        int32_t* po = ids.mutable_data();
        int32_t* pn = ns.mutable_data();
        const int64_t* qp = q_ptr.data();
        const int32_t* sd = seeds.data();
        {
          py::gil_scoped_release nogil;
          std::fill(po, po + B * k, -1);
          for (int64_t b = 0; b < B; ++b)
            pn[b] = ix.query(sd + qp[b], (int)(qp[b + 1] - qp[b]), k, po + b * k, nullptr);
        }
        return py::make_tuple(ids, ns);
      });

  // ---------------- HIP runtime ----------------
  register_gpu_bindings(m);
  register_front_bindings(m);
}
