// pybind11 bindings of the native HTTP serving front (http_front.cpp) and of its fallback
// sampler (so tests can pin it against CPython's random.Random.sample).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "kmls/gpu.hpp"
#include "kmls/http_front.hpp"
#include "kmls/loadgen.hpp"
#include <pybind11/numpy.h>

namespace py = pybind11;

namespace kmls {

void register_front_bindings(py::module_& m) {
  py::class_<HttpFront>(m, "HttpFront")
      .def(py::init<const std::string&, int, int, int, const std::string&, int, int>(),
           py::arg("host"), py::arg("port"), py::arg("threads"), py::arg("k"),
           py::arg("version"), py::arg("batch_max") = 256, py::arg("batch_wait_us") = 100)
      .def("start", &HttpFront::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &HttpFront::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &HttpFront::port)
      .def_property_readonly("slow_fd", &HttpFront::slow_fd)
      .def("set_model", [](HttpFront& f, std::shared_ptr<RuleIndex> index,
                           const std::vector<std::string>& names,
                           const std::vector<std::string>& best, py::object marker,
                           std::shared_ptr<gpu::GpuRuleIndex> gpu, int gpu_min_batch,
                           int gpu_min_merge) {
        std::string mk;
        const std::string* mp = nullptr;
        if (!marker.is_none()) {
          mk = marker.cast<std::string>();
          mp = &mk;
        }
        py::gil_scoped_release nogil;
        f.set_model(std::move(index), names, best, mp, std::move(gpu), gpu_min_batch,
                    gpu_min_merge);
      }, py::arg("index"), py::arg("names"), py::arg("best_names"), py::arg("marker"),
         py::arg("gpu") = nullptr, py::arg("gpu_min_batch") = 0, py::arg("gpu_min_merge") = -1)
      .def("clear_model", &HttpFront::clear_model)
      .def("next_slow", [](HttpFront& f) -> py::object {
        SlowRequest r;
        if (!f.next_slow(r)) return py::none();
        py::list headers;
        for (auto& h : r.headers) headers.append(py::make_tuple(py::bytes(h.first), py::bytes(h.second)));
        return py::make_tuple(r.token, r.method, py::bytes(r.path), py::bytes(r.query),
                              r.http_version, headers, py::bytes(r.body), r.client_host,
                              r.client_port);
      })
      .def("respond", [](HttpFront& f, uint64_t token, int status, py::list headers,
                         py::bytes body) {
        std::vector<std::pair<std::string, std::string>> hs;
        for (auto h : headers) {
          auto t = h.cast<py::tuple>();
          hs.emplace_back(t[0].cast<std::string>(), t[1].cast<std::string>());
        }
        std::string b = body;
        py::gil_scoped_release nogil;
        f.respond(token, status, hs, b);
      })
      .def("stats", [](HttpFront& f) {
        const FrontStats s = f.stats();
        py::dict d;
        d["requests"] = s.requests;
        d["native"] = s.native_ok;
        d["fallback"] = s.fallback;
        d["slow"] = s.slow;
        d["gpu_batches"] = s.gpu_batches;
        d["gpu_queries"] = s.gpu_queries;
        d["gpu_loop_batches"] = s.gpu_loop_batches;
        d["gpu_loop_refused"] = s.gpu_loop_refused;
        d["connections"] = s.connections;
        d["bytes_in"] = s.bytes_in;
        d["bytes_out"] = s.bytes_out;
        return d;
      });
  m.def("loadgen", [](const std::string& host, int port, std::vector<py::bytes> reqs, double qps,
                      double duration, int connections, int threads, double drain) {
    std::vector<std::string> r;
    for (auto& b : reqs) r.push_back(std::string(b));
    LoadResult res;
    {
      py::gil_scoped_release nogil;
      res = run_loadgen(host, port, r, qps, duration, connections, threads, drain);
    }
    py::dict d;
    d["lat_ns"] = py::array_t<int64_t>((py::ssize_t)res.lat_ns.size(), res.lat_ns.data());
    d["lag_ns"] = py::array_t<int64_t>((py::ssize_t)res.lag_ns.size(), res.lag_ns.data());
    d["at_ns"] = py::array_t<int64_t>((py::ssize_t)res.at_ns.size(), res.at_ns.data());
    d["offered"] = res.offered;
    d["sent"] = res.sent;
    d["completed"] = res.completed;
    d["errors"] = res.errors;
    return d;
  }, py::arg("host"), py::arg("port"), py::arg("requests"), py::arg("qps"), py::arg("duration"),
     py::arg("connections") = 64, py::arg("threads") = 2, py::arg("drain") = 5.0);
  m.def("python_random_sample", &python_random_sample, py::arg("seed"), py::arg("n"), py::arg("k"));
  m.def("fallback_seed", [](std::vector<std::string> seeds) { return fallback_seed(std::move(seeds)); });
  m.def("json_escape", [](const std::string& s) {
    std::string out;
    json_escape_append(out, s);
    return py::bytes(out);
  });
}

}  // namespace kmls
