// pybind11 bindings of the host runtime: module `_ragk_rt` (built in-tree by rag_llm_k8s_amd/_build.py).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"
#include "tokenizer.h"

namespace py = pybind11;
using namespace ragk_rt;

static py::dtype np_dtype(const std::string& dt) {
  if (dt == "F32") return py::dtype("float32");
  if (dt == "F64") return py::dtype("float64");
  if (dt == "F16") return py::dtype("float16");
  if (dt == "BF16" || dt == "U16" || dt == "I16") return py::dtype(dt == "I16" ? "int16" : "uint16");
  if (dt == "I64") return py::dtype("int64");
  if (dt == "I32") return py::dtype("int32");
  if (dt == "U32") return py::dtype("uint32");
  if (dt == "I8") return py::dtype("int8");
  if (dt == "BOOL") return py::dtype("bool");
  return py::dtype("uint8");
}

PYBIND11_MODULE(_ragk_rt, m) {
  m.doc() = "rag_llm_k8s_amd native host runtime (safetensors mmap, faiss I/O, KV blocks, tokenizers)";
#ifndef RAGK_RT_STAMP
#define RAGK_RT_STAMP "unstamped"
#endif
  // content hash of csrc/runtime at build time (_build.runtime_source_hash), checked at import
  m.def("build_stamp", []() { return std::string(RAGK_RT_STAMP); });

  py::class_<SafeTensors, std::shared_ptr<SafeTensors>>(m, "SafeTensors")
      .def(py::init<const std::string&>())
      .def("keys", &SafeTensors::keys)
      .def("metadata", &SafeTensors::metadata)
      .def("info",
           [](const SafeTensors& s, const std::string& n) {
             const TensorInfo& t = s.info(n);
             return py::make_tuple(t.dtype, t.shape, t.begin, t.end);
           })
      // zero-copy read-only numpy view over the mmap (keeps the file object alive)
      .def("view",
           [](std::shared_ptr<SafeTensors> s, const std::string& n) {
             const TensorInfo& t = s->info(n);
             std::vector<py::ssize_t> shape(t.shape.begin(), t.shape.end());
             py::capsule owner(new std::shared_ptr<SafeTensors>(s),
                               [](void* p) { delete reinterpret_cast<std::shared_ptr<SafeTensors>*>(p); });
             py::array a(np_dtype(t.dtype), shape, {}, s->data(n), owner);
             py::detail::array_proxy(a.ptr())->flags &= ~py::detail::npy_api::NPY_ARRAY_WRITEABLE_;
             return a;
           })
      // copy of rows [r0,r1) (and cols [c0,c1) if c0 >= 0): TP shard extraction without touching other bytes
      .def("slice",
           [](const SafeTensors& s, const std::string& n, int64_t r0, int64_t r1, int64_t c0, int64_t c1) {
             const TensorInfo& t = s.info(n);
             std::vector<py::ssize_t> shape(t.shape.begin(), t.shape.end());
             if (!shape.empty()) {
               if (r0 >= 0) shape[0] = r1 - r0;
               if (c0 >= 0) shape[1] = c1 - c0;
             }
             py::array a(np_dtype(t.dtype), shape);
             {
               py::gil_scoped_release nogil;
               s.copy_slice(n, r0, r1, c0, c1, (char*)a.mutable_data());
             }
             return a;
           },
           py::arg("name"), py::arg("r0") = -1, py::arg("r1") = -1, py::arg("c0") = -1, py::arg("c1") = -1);

  m.def("read_flat_index", [](const std::string& path) {
    FlatIndexData r = read_flat_index(path);
    py::array_t<float> xb({(py::ssize_t)r.ntotal, (py::ssize_t)r.d});
    if (!r.xb.empty()) std::memcpy(xb.mutable_data(), r.xb.data(), r.xb.size() * 4);
    return py::make_tuple(r.d, r.ntotal, r.metric, xb);
  });
  m.def("write_flat_index", [](const std::string& path, py::array_t<float, py::array::c_style | py::array::forcecast> x) {
    if (x.ndim() != 2) throw std::invalid_argument("xb must be [n, d]");
    write_flat_index(path, x.data(), x.shape(0), (int32_t)x.shape(1));
  });

  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, bool>(), py::arg("num_blocks"), py::arg("reserve_scratch") = true)
      .def("free_blocks", &BlockManager::free_blocks)
      .def("blocks_needed", &BlockManager::blocks_needed)
      .def("can_allocate", &BlockManager::can_allocate)
      .def("ensure", &BlockManager::ensure, py::return_value_policy::copy)
      .def("table", &BlockManager::table, py::return_value_policy::copy)
      .def("slot", &BlockManager::slot)
      .def("free", &BlockManager::free)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks);

  py::class_<Tokenizer>(m, "Tokenizer")
      .def(py::init<const std::string&>())
      .def("encode",
           [](const Tokenizer& t, const std::string& s, bool add_special, int max_tokens) {
             std::vector<int> ids;
             {
               py::gil_scoped_release nogil;
               ids = t.encode(s, add_special, max_tokens);
             }
             return ids;
           },
           py::arg("text"), py::arg("add_special_tokens") = true, py::arg("max_tokens") = -1)
      .def("encode_batch",
           [](const Tokenizer& t, const std::vector<std::string>& texts, bool add_special, int threads,
              int max_tokens) {
             std::vector<std::vector<int>> ids;
             {
               py::gil_scoped_release nogil;
               ids = t.encode_batch(texts, add_special, threads, max_tokens);
             }
             return ids;
           },
           py::arg("texts"), py::arg("add_special_tokens") = true, py::arg("threads") = 8,
           py::arg("max_tokens") = -1)
      // ingest path: (ids int32 [sum lens], lens int32 [n]) with right truncation to max_length that
      // keeps a trailing special token -- no per-token Python objects on the way to the encoder
      .def("encode_batch_flat",
           [](const Tokenizer& t, const std::vector<std::string>& texts, bool add_special, int threads,
              int max_length) {
             std::vector<int32_t> flat, lens(texts.size());
             {
               py::gil_scoped_release nogil;
               std::vector<std::vector<int>> ids = t.encode_batch(texts, add_special, threads, max_length);
               size_t tot = 0;
               for (size_t i = 0; i < ids.size(); ++i) {
                 std::vector<int>& v = ids[i];
                 if (max_length > 0 && (int)v.size() > max_length) {
                   const int last = v.back();
                   if (add_special && t.is_special(last)) {
                     v.resize(max_length - 1);
                     v.push_back(last);
                   } else {
                     v.resize(max_length);
                   }
                 }
                 lens[i] = (int32_t)v.size();
                 tot += v.size();
               }
               flat.reserve(tot);
               for (const auto& v : ids) flat.insert(flat.end(), v.begin(), v.end());
             }
             return py::make_tuple(py::array_t<int32_t>(flat.size(), flat.data()),
                                   py::array_t<int32_t>(lens.size(), lens.data()));
           },
           py::arg("texts"), py::arg("add_special_tokens") = true, py::arg("threads") = 8,
           py::arg("max_length") = -1)
      .def("decode", &Tokenizer::decode, py::arg("ids"), py::arg("skip_special_tokens") = true)
      .def("vocab_size", &Tokenizer::vocab_size)
      .def("token_to_id",
           [](const Tokenizer& t, const std::string& s) -> py::object {
             const int id = t.token_to_id(s);
             if (id < 0) return py::none();
             return py::int_(id);
           })
      .def("model_type", &Tokenizer::model_type);
}
